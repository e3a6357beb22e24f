// lachain_amd/csrc/k_ts.hip — gfx950 kernels: threshold-signature share verification.
#include "kcommon.hpp"

LCB_ASM_LIBRARY(k_ts)
LCB_TU_CONFIG(k_ts)

// ================================================================================= threshold signatures
// k_ts_msg_prepare (hash to G2 + the message's line set) lives in k_prep.hip at 256 registers (round 5)
// two-pair Miller loop of a signature check: the message's line set (normalised, or its point's lines on the fly
// when it could not be normalised) and the share's lines on the fly
DN void miller2_ts_fallback(fp12 &f, const u32 *lsH, const g1a &PK, const g2a &S, const g1a &G) {
    g2a Q;
    lineset_point(Q, lsH);
    LinesOnTheFly sH, sS;
    sH.init(Q);
    sS.init(S);
    miller2(f, sH, PK, sS, G);
}
DI void miller2_ts(fp12 &f, const u32 *lsH, const g1a &PK, const g2a &S, const g1a &G) {
    if (lineset_normalised(lsH)) {
        LinesNorm sH{lsH};
        LinesOnTheFly sS;
        sS.init(S);
        miller2(f, sH, PK, sS, G);
    } else {
        miller2_ts_fallback(f, lsH, PK, S, G);
    }
}

// ValidateSignature: e(PK, H) == e(G, sig) <=> e(PK, H) e(-G, sig) == 1
// Exact per-share check, two kernels: the 2-pair Miller loop parks f in HBM (word-major SoA) and k_final_exp_check
// (k_tpke.hip) finishes, so each half gets its own register budget.
extern "C" __global__ void LCB_PAIR_BOUNDS k_ts_miller(const u32 *lines, const uint8_t *msg_ok, u32 n_msgs, const g1a_st *pks,
                                                 u32 n_pks, const uint8_t *sigs, const u32 *msg_idx,
                                                 const u32 *pk_idx, u32 n, u32 *f_soa, uint8_t *accept) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u32 m = msg_idx[i], k = pk_idx[i];
    g2a S;
    g1a PK, G;
    bool ok = k < n_pks && m < n_msgs;   // an out-of-range index rejects the share (and is clamped)
    m = m < n_msgs ? m : 0;
    ok = ok && msg_ok[m];
    ok = g2_decompress(S, sigs + 96 * (size_t)i) && ok;
    g1a_st ps = pks[k < n_pks ? k : 0];
    ok = ok && ps.ok;
    st_to_g1a(PK, ps);
    g1_generator(G);
    fp_neg(G.y, G.y);
    fp12 f;
    miller2_ts(f, lines + (size_t)m * LCB_LINESET_WORDS, PK, S, G);
    fp12_store_soa(f_soa, n, i, f);
    accept[i] = ok;
}

// Share selection for Lagrange assembly, one lane per group (a CommonCoin round, or a TPKE ciphertext):
//   ThresholdSigner.AddShare -> PublicKeySet.AssembleSignature (ThresholdSigner.cs:62-75, PublicKeySet.cs:34-42)
//   TPKE.PublicKey.FullDecrypt (TPKE/PublicKey.cs:55-86; shares ordered by DecryptorId)
// takes the first k shares (in index order) that passed verification, x = index + 1.  A group with fewer than k
// valid shares gets x = 0 entries, which the Lagrange stage reports as status 0 (the reference keeps waiting
// for shares / FullDecrypt throws).  pbytes = 48 (G1) or 96 (G2).
// order (nullable): the caller's arrival order per group — order[r * per_group + j] = the position (DecryptorId /
// signer index) of the j-th share to arrive; entries >= per_group are absent arrivals.  Null: index order.
extern "C" __global__ void LCB_BOUNDS k_select_first_valid(const uint8_t *accept, const uint8_t *pts, u32 pbytes,
                                                          u32 per_group, u32 k, u32 n_groups, uint8_t *xs,
                                                          uint8_t *ys, u32 *off, const u32 *order, u32 *src_out) {
    u32 r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_groups) return;
    off[r] = r * k;
    if (r == n_groups - 1) off[n_groups] = n_groups * k;
    const u32 pw = pbytes / 4;
    u32 cnt = 0;
    for (u32 j = 0; j < per_group && cnt < k; j++) {
        const u32 i = order ? order[(size_t)r * per_group + j] : j;
        if (i >= per_group) continue;
        size_t src = (size_t)r * per_group + i;
        if (!accept[src]) continue;
        size_t dst = (size_t)r * k + cnt;
        u32 *xw = (u32 *)(xs + 32 * dst);
        xw[0] = i + 1;
        for (int q = 1; q < 8; q++) xw[q] = 0;
        const u32 *sw = (const u32 *)(pts + (size_t)pbytes * src);
        u32 *yw = (u32 *)(ys + (size_t)pbytes * dst);
        for (u32 q = 0; q < pw; q++) yw[q] = sw[q];
        if (src_out) src_out[dst] = (u32)src;           // the share's index in pts (its ts_share_st record)
        cnt++;
    }
    for (; cnt < k; cnt++) {
        size_t dst = (size_t)r * k + cnt;
        u32 *xw = (u32 *)(xs + 32 * dst);
        u32 *yw = (u32 *)(ys + (size_t)pbytes * dst);
        for (int q = 0; q < 8; q++) xw[q] = 0;
        for (u32 q = 0; q < pw; q++) yw[q] = 0;
        if (src_out) src_out[dst] = 0xffffffffu;
    }
}

// CommonCoin consumers of the combined signature bytes (one lane per coin):
//   CoinResult.Parity  = popcount(XOR of all 96 bytes) odd        (src/Lachain.Consensus/CommonCoin/CoinResult.cs:16-20)
//   GetNonceFromCoin   = 8-byte XOR fold of the 96 bytes, LE u64  (src/Lachain.Consensus/RootProtocol/RootProtocol.cs:316-322)
extern "C" __global__ void LCB_BOUNDS k_coin_fold(const uint8_t *sigs, u32 n, uint8_t *parity, uint64_t *nonce) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint2 *w = (const uint2 *)(sigs + 96 * (size_t)i);
    uint2 acc = make_uint2(0, 0);
#pragma unroll
    for (int q = 0; q < 12; q++) { uint2 v = w[q]; acc.x ^= v.x; acc.y ^= v.y; }
    u32 b = acc.x ^ acc.y;
    b ^= b >> 16;
    b ^= b >> 8;                     // XOR of all 96 bytes in the low byte
    if (parity) parity[i] = __popc(b & 0xffu) & 1;
    if (nonce) nonce[i] = (uint64_t)acc.x | ((uint64_t)acc.y << 32);
}

// ---------------------------------------------------------------- host launch wrappers
extern "C" void lcbk_ts_miller(dim3 grid, hipStream_t s, const u32 *lines, const uint8_t *msg_ok, u32 n_msgs, const void *pks, u32 n_pks, const uint8_t *sigs, const u32 *msg_idx, const u32 *pk_idx, u32 n, u32 *f_soa, uint8_t *accept) {
    LCB_LAUNCH(k_ts_miller, lines, msg_ok, n_msgs, (const g1a_st *)pks, n_pks, sigs, msg_idx, pk_idx, n, f_soa, accept);
}
extern "C" void lcbk_select_first_valid(dim3 grid, hipStream_t s, const uint8_t *accept, const uint8_t *pts, u32 pbytes, u32 per_group, u32 k, u32 n_groups, uint8_t *xs, uint8_t *ys, u32 *off, const u32 *order, u32 *src) {
    LCB_LAUNCH(k_select_first_valid, accept, pts, pbytes, per_group, k, n_groups, xs, ys, off, order, src);
}
extern "C" void lcbk_coin_fold(dim3 grid, hipStream_t s, const uint8_t *sigs, u32 n, uint8_t *parity, uint64_t *nonce) {
    LCB_LAUNCH(k_coin_fold, sigs, n, parity, nonce);
}
