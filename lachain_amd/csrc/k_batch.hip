// lachain_amd/csrc/k_batch.hip — gfx950 kernels: randomized batch verification of TPKE decryption shares
// (small-exponent test, Bellare–Garay–Rabin 1998) over the per-share check of TPKE/PublicKey.cs:88-92.
//
// The reference decides every share on its own: e(U_i, H) == e(Y_i, W) (two pairings per share).  Every value
// e(., .) is a reduced pairing, so the ratio g_i = e(U_i, H) / e(Y_i, W) lies in mu_r (order r, prime) whatever
// U_i is: for a G2 point Q the (ate) pairing is linear in its G1 argument on all of E(Fp) (Weil reciprocity; the
// error term is an r-th power, killed by the final exponentiation) and kills the cofactor-torsion part, so off-
// subgroup U_i / Y_i are covered.  H is in G2 by construction; W is checked (k_lineset_fill, lineset_in_g2) and a ciphertext with
// W outside G2 gets exact per-share checks.  For secret random exponents s_i (2^64 values, none 0 mod r; rlc_scalar):
// prod_i g_i^(s_i) == 1  <=>  e(sum s_i U_i, H) e(-sum s_i Y_i, W) == 1, and if some g_i != 1 the product is 1 with
// probability <= 2^-64.  So one Miller pair + final exponentiation decides a whole group of shares of one ciphertext;
// a group that fails is split and re-checked, down to single shares, where g_i^(s_i) == 1 <=> g_i == 1 (gcd(s_i, r)
// = 1): every rejected share is rejected by an exact check of its own, every accepted share by a group check (false
// accept <= 2^-64 per group, over the secret exponents).
//
// Level 2 (one bad share per group, the usual failure): the first level also forms W = sum (j+1) s_j U_j etc. (j = the
// share's position in its group, so the weights c_j = j+1 are distinct and public).  A failed group's gamma =
// prod g_i^(s_i) (its final-exponentiation output) and gamma' = prod g_i^(c_i s_i) (one more group check) satisfy
// gamma' = gamma^(c_j) exactly when j is the only bad share: k_rlc_search tries c = 1..len (len Fp12 products) and
// rejects share j; with two or more bad shares no c matches except with probability <= len 2^-64 (the exponents
// s_i are secret), and the group's shares get single checks at the next level.  So at most three levels.
//
// Pipeline (host side in lcb_host.cpp: rlc_points_enqueue + rlc_levels):
//   k_tpke_rlc_points   one lane per share: validity as k_tpke_miller, (a_i, b_i) = ChaCha20(key, i), s_i U_i and
//                       s_i Y_i with s_i = a_i + b_i lambda (32-bit GLV form, rlc_scalar) -> quad-major SoA Jacobian
//                       records (invalid share: infinity)
//   k_rlc_groups        one lane per 256 consecutive shares: runs of equal ciphertext index (<= 32) -> level-1 groups
//   k_lineset_fill      (k_tpke.hip) W's line set also decides W in G2 (else its shares get exact per-share checks)
//   k_tpke_rlc_sum      one lane per group: ciphertext validity, the two sums, to affine with one shared inversion,
//                       -sum s_i Y_i (or an exact single share's own U_i, -Y_i)
//   k_tpke_rlc_miller   one lane per group: the two-pair Miller loop over the ciphertext's line sets
//   k_final_exp_check   (k_tpke.hip) group decision
//   k_rlc_resolve       one lane per group: failed single share -> reject; failed group -> sub-groups of the next level
#include "kcommon.hpp"

LCB_ASM_LIBRARY(k_batch)

struct rlc_key { u32 k[8]; u32 nonce[2]; };   // ChaCha20 key (256 bit, from getrandom) and a per-call nonce

#define LCB_RLC_SINGLES 8       // a failed group this short (below level 1) splits into single shares

// ---------------------------------------------------------------- suspect keys (Byzantine validators)
// A faulty validator corrupts its share in EVERY ciphertext / coin (HoneyBadgerMalicious.cs:17-23 reverses each
// share it sends; HoneyBadgerSmartMalicious.cs:28-48 sends valid off-subgroup points), so with F of them every group
// carries F bad shares and every group check fails.  The census (exact single checks of a prefix of the batch, before
// the groups are formed) marks a key suspect when at least half of its sampled shares that decoded failed their exact
// check; every share of a suspect key is then checked on its own and the groups are summed over the other keys only.
// The bitmap only changes the cost: every decision is still an exact single check or a group check.
DI bool key_suspect(const u32 *susp, u32 k, u32 n_keys) {
    return susp && k < n_keys && ((susp[k >> 5] >> (k & 31)) & 1u);
}
// the same read while the census may still be writing the bitmap (k_*_rlc_points runs beside it on the other
// stream): a stale 0 only costs a randomisation that is not used
DI bool key_suspect_live(const u32 *susp, u32 k, u32 n_keys) {
    if (!susp || k >= n_keys) return false;
    return (__atomic_load_n(susp + (k >> 5), __ATOMIC_RELAXED) >> (k & 31)) & 1u;
}

// ---------------------------------------------------------------- ChaCha20 (RFC 8439 block function)
DI u32 rotl32(u32 x, int r) { return (x << r) | (x >> (32 - r)); }
#define CHACHA_QR(a, b, c, d)                  \
    a += b; d ^= a; d = rotl32(d, 16);         \
    c += d; b ^= c; b = rotl32(b, 12);         \
    a += b; d ^= a; d = rotl32(d, 8);          \
    c += d; b ^= c; b = rotl32(b, 7);
// share exponent s_i = a_i + b_i lambda (lambda = z^2 - 1, phi(x, y) = (beta x, y)) from the 32-bit words a_i, b_i of
// ChaCha20 block i: a_i P + b_i phi(P) takes 32 shared doublings.  phi acts as lambda on the r-torsion and the reduced
// pairing kills every other component of an E(Fp) point, so e(a P + b phi(P), Q) = e(P, Q)^(a + b lambda) for ANY
// P on the curve; the 2^64 pairs (a, b) give 2^64 distinct exponents mod r (a + b lambda < 2^160 < r), none zero
// ((0, 0) -> (1, 0)): the soundness of a uniform 64-bit exponent.
DI void rlc_scalar(const rlc_key &key, u32 i, u32 &a, u32 &b) {
    u32 x[16], s[16];
    s[0] = 0x61707865u; s[1] = 0x3320646eu; s[2] = 0x79622d32u; s[3] = 0x6b206574u;
#pragma unroll
    for (int j = 0; j < 8; j++) s[4 + j] = key.k[j];
    s[12] = i; s[13] = 0; s[14] = key.nonce[0]; s[15] = key.nonce[1];
#pragma unroll
    for (int j = 0; j < 16; j++) x[j] = s[j];
#pragma unroll 1
    for (int r = 0; r < 10; r++) {
        CHACHA_QR(x[0], x[4], x[8], x[12]);
        CHACHA_QR(x[1], x[5], x[9], x[13]);
        CHACHA_QR(x[2], x[6], x[10], x[14]);
        CHACHA_QR(x[3], x[7], x[11], x[15]);
        CHACHA_QR(x[0], x[5], x[10], x[15]);
        CHACHA_QR(x[1], x[6], x[11], x[12]);
        CHACHA_QR(x[2], x[7], x[8], x[13]);
        CHACHA_QR(x[3], x[4], x[9], x[14]);
    }
    a = x[0] + s[0];
    b = x[1] + s[1];
    if ((a | b) == 0) a = 1;
}

// ---------------------------------------------------------------- quad-major SoA records (NW words, NW % 4 == 0)
template <int NW> DI void soa_store(u32 *base, size_t n, size_t i, const void *v) {
    const u32 *s = (const u32 *)v;
#pragma unroll
    for (int q = 0; q < NW / 4; q++)
        *(uint4 *)(base + ((size_t)q * n + i) * 4) = make_uint4(s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]);
}
template <int NW> DI void soa_load(void *v, const u32 *base, size_t n, size_t i) {
    u32 *d = (u32 *)v;
#pragma unroll
    for (int q = 0; q < NW / 4; q++) {
        uint4 x = *(const uint4 *)(base + ((size_t)q * n + i) * 4);
        d[4 * q] = x.x; d[4 * q + 1] = x.y; d[4 * q + 2] = x.z; d[4 * q + 3] = x.w;
    }
}
DI void g1_store_soa(u32 *base, size_t n, size_t i, const g1 &p) { soa_store<36>(base, n, i, &p); }
DI void g1_load_soa(g1 &p, const u32 *base, size_t n, size_t i) { soa_load<36>(&p, base, n, i); }
DI void g2_store_soa(u32 *base, size_t n, size_t i, const g2 &p) { soa_store<72>(base, n, i, &p); }
DI void g2_load_soa(g2 &p, const u32 *base, size_t n, size_t i) { soa_load<72>(&p, base, n, i); }

// a P + b phi(P) for an affine P, phi(x, y) = (beta x, y).  Joint bits: the addend is P (1, 0), phi(P) (0, 1) or
// P + phi(P) = (beta^2 x, -y) (1, 1; the chord through two points of equal y has slope 0 and 1 + beta + beta^2 = 0),
// so each bit costs one mixed addition, and a wave (whose lanes' bits differ) executes 32 of them instead of 64.
DI void g1_ab_addends(fp &bx, fp &b2x, fp &ny, const g1a &P) {
    fp beta;
    fp_load_const(beta, LCB_G1_BETA);
    fp_mul(bx, P.x, beta);
    fp_mul(b2x, bx, beta);
    fp_neg(ny, P.y);
}
DN void g1_mul_ab_n(g1 &r, const g1a &P, u32 a, u32 b) {
    g1 acc;
    jac_set_inf(acc);
    if (!P.inf) {
        fp bx, b2x, ny;
        g1_ab_addends(bx, b2x, ny, P);
        for (int k = 31; k >= 0; k--) {
            grp_dbl(acc, acc);
            u32 da = (a >> k) & 1, db = (b >> k) & 1;
            if (da | db) grp_madd(acc, acc, da ? (db ? b2x : P.x) : bx, (da & db) ? ny : P.y);
        }
    }
    r = acc;
}
// (a + b lambda) S for S in G2: psi^2(x, y) = (beta x, -y) acts on G2 as z^2 (mod r) and psi^4(x, y) = (beta^2 x, y)
// as z^4 = z^2 - 1 = lambda, so (a + b lambda) S = a S + b psi^4(S); the joint addend S + psi^4(S) = psi^2(S) (equal
// y again): one mixed addition per bit as in G1
DI void g2_ab_addends(fp2 &x4, fp2 &x2, fp2 &ny, const g2a &S) {
    fp beta, b2;
    fp_load_const(beta, LCB_G1_BETA);
    fp_sqr(b2, beta);
    fp2_mul_fp(x4, S.x, b2);
    fp2_mul_fp(x2, S.x, beta);
    fp2_neg(ny, S.y);
}
// the same with the point arithmetic inlined (no call frames: the DN form passes the accumulator through scratch at
// every doubling / addition)
DI void g1_mul_ab_inl(g1 &r, const g1a &P, u32 a, u32 b) {
    jac_set_inf(r);
    if (P.inf) return;
    fp bx, b2x, ny;
    g1_ab_addends(bx, b2x, ny, P);
#pragma unroll 1
    for (int k = 31; k >= 0; k--) {
        jac_dbl(r, r);
        u32 da = (a >> k) & 1, db = (b >> k) & 1;
        if (da | db) jac_add_aff(r, r, da ? (db ? b2x : P.x) : bx, (da & db) ? ny : P.y);
    }
}
// G2 form of g1_mul_ab_inl: a S + b psi^4(S) with the point arithmetic inlined
DI void g2_mul_ab_inl(g2 &r, const g2a &S, u32 a, u32 b) {
    jac_set_inf(r);
    if (S.inf) return;
    fp2 x4, x2, ny;
    g2_ab_addends(x4, x2, ny, S);
#pragma unroll 1
    for (int k = 31; k >= 0; k--) {
        jac_dbl(r, r);
        u32 da = (a >> k) & 1, db = (b >> k) & 1;
        if (da | db) jac_add_aff(r, r, da ? (db ? x2 : S.x) : x4, (da & db) ? ny : S.y);
    }
}
// affine records of Jacobian points (inf = 1 for the point at infinity), optionally negated
DI void g1_to_st(g1a_st &o, const g1 &p, bool neg) {
    g1a a;
    jac_to_aff(a, p);
    o.ok = 1; o.pad[0] = o.pad[1] = 0;
    o.inf = a.inf;
    o.x = a.x;
    if (neg && !a.inf) fp_neg(o.y, a.y);
    else o.y = a.y;
}
DI void g2_to_st(g2a_st &o, const g2 &p) {
    g2a a;
    jac_to_aff(a, p);
    o.ok = 1; o.pad[0] = o.pad[1] = 0;
    o.inf = a.inf;
    o.x = a.x;
    o.y = a.y;
}
DI void g1_inf_st(g1a_st &o) { o.ok = 1; o.pad[0] = o.pad[1] = 0; o.inf = 1; o.x = fp_zero(); o.y = fp_zero(); }
DI void g2_inf_st(g2a_st &o) { o.ok = 1; o.pad[0] = o.pad[1] = 0; o.inf = 1; o.x = fp2_zero(); o.y = fp2_zero(); }

// ---------------------------------------------------------------- fixed-base tables of the validators' keys
// The keys (TPKE verification keys Y_d, threshold-signature public keys PK_k) are the same for every ciphertext /
// coin of a batch: per key, table[w][d - 1] = d 2^(8w) K (affine x, y and beta x, d = 1..255, w = 0..3) turns
// a K + b phi(K) for 32-bit a, b into at most 8 mixed additions (4 byte digits of a, 4 of b on the phi entries) instead
// of 32 doublings + ~32 mixed additions.  One lane per (key, window): 8w doublings, 254 additions into a
// Jacobian scratch, then one batched inversion (Montgomery's trick) to affine.  A key whose chain meets the point at
// infinity (a key with no r-torsion part) or that did not decompress gets ktab_ok = 0: its shares use the ladder.
#define LCB_KTAB_ENTRIES (4 * 255)
#define LCB_KTAB_CHUNK 32                              // entries per lane: 8 lanes per (key, window)
#define LCB_KTAB_LANES 32                              // lanes (and flags) per key
extern "C" __global__ void LCB_BOUNDS k_rlc_key_tables(const g1a_st *keys, u32 n_keys, u32 *jtab, u32 *pre, u32 *tab,
                                                      uint8_t *ktab_ok) {
    u32 t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= LCB_KTAB_LANES * n_keys) return;
    u32 k = t / LCB_KTAB_LANES, w = (t / 8) & 3, ch = t & 7;
    u32 d0 = ch * LCB_KTAB_CHUNK + 1, d1 = min(255u, d0 + LCB_KTAB_CHUNK - 1);   // entries d0 .. d1
    g1a K;
    g1a_st ks = keys[k];
    st_to_g1a(K, ks);
    const size_t stride = (size_t)n_keys * LCB_KTAB_ENTRIES;      // SoA over every (key, entry)
    const size_t e0 = (size_t)k * LCB_KTAB_ENTRIES + (size_t)w * 255;
    bool ok = ks.ok && !K.inf;
    g1 B, acc;
    jac_from_aff(B, K);
#pragma unroll 1
    for (u32 j = 0; ok && j < 8 * w; j++) jac_dbl(B, B);            // B = 2^(8w) K
    jac_mul_u64_inl(acc, B, d0);                                   // d0 B
    fp run = fp_one();
#pragma unroll 1
    for (u32 d = d0; ok && d <= d1; d++) {            // Jacobian entries and the running product of their z
        if (jac_is_inf(acc)) { ok = false; break; }
        g1_store_soa(jtab, stride, e0 + d - 1, acc);
        fp_mul(run, run, acc.z);
        soa_store<12>(pre, stride, e0 + d - 1, &run);
        jac_add(acc, acc, B);
    }
    ktab_ok[t] = ok;
    if (!ok) return;
    fp inv, beta;
    fp_inv(inv, run);                                  // 1 / (z_d0 ... z_d1)
    fp_load_const(beta, LCB_G1_BETA);
#pragma unroll 1
    for (u32 d = d1; d >= d0; d--) {
        g1 p;
        g1_load_soa(p, jtab, stride, e0 + d - 1);
        fp zi, zi2, pd;
        if (d > d0) {
            soa_load<12>(&pd, pre, stride, e0 + d - 2);
            fp_mul(zi, inv, pd);                       // 1 / z_d
            fp_mul(inv, inv, p.z);
        } else {
            zi = inv;
        }
        fp_sqr(zi2, zi);
        fp xyb[3];                                     // x, y, beta x (phi(x, y) = (beta x, y))
        fp_mul(xyb[0], p.x, zi2);
        fp_mul(zi2, zi2, zi);
        fp_mul(xyb[1], p.y, zi2);
        fp_mul(xyb[2], xyb[0], beta);
        soa_store<36>(tab, stride, e0 + d - 1, xyb);
    }
}
// a K + b phi(K) from key k's affine table (phi(x, y) = (beta x, y) also acts on Jacobian coordinates)
DN void g1_mul_ab_tab(g1 &r, const u32 *tab, u32 n_keys, u32 k, u32 a, u32 b) {
    const size_t stride = (size_t)n_keys * LCB_KTAB_ENTRIES, e0 = (size_t)k * LCB_KTAB_ENTRIES;
    g1 acc;
    jac_set_inf(acc);
    fp xyb[3];
    // one digit at a time (the loads are not hoisted: eight live table points would cost 192 registers); the b digits
    // add phi(entry) = (beta x, y), stored beside the entry
#pragma unroll 1
    for (u32 j = 0; j < 8; j++) {
        u32 w = j & 3, dg = ((j < 4 ? b : a) >> (8 * w)) & 255;
        if (!dg) continue;
        asm volatile("" ::: "memory");
        soa_load<36>(xyb, tab, stride, e0 + w * 255 + dg - 1);
        grp_madd(acc, acc, j < 4 ? xyb[2] : xyb[0], xyb[1]);
    }
    r = acc;
}
DI bool ktab_usable(const uint8_t *ktab_ok, u32 k) {      // all 32 lanes of the key's table succeeded
    if (!ktab_ok) return false;
    const uint4 *f = (const uint4 *)(ktab_ok + (size_t)LCB_KTAB_LANES * k);
    uint4 x = f[0], y = f[1];
    return (x.x & x.y & x.z & x.w & y.x & y.y & y.z & y.w) == 0x01010101u;
}

// ---------------------------------------------------------------- TPKE: per-share randomisation
// validity as k_tpke_miller except the ciphertext's (applied per group by k_tpke_rlc_sum, so this kernel needs only
// the decompressed keys and may run beside the ciphertext preparation)
// Shares [i0, n) (the census decides [0, i0) exactly); a share of a key the census has already marked suspect only
// gets its validity (it is checked on its own).
extern "C" __global__ void __launch_bounds__(LCB_BLOCK) __attribute__((amdgpu_waves_per_eu(1)))
k_tpke_rlc_points(u32 n_cts, const g1a_st *keys, u32 n_keys, const u32 *ct_idx,
                                                       const u32 *dec_idx, const uint8_t *ui, u32 i0, u32 n,
                                                       rlc_key key, u32 *rU, u32 *rY, uint8_t *accept,
                                                       const u32 *ktab, const uint8_t *ktab_ok, const u32 *susp) {
    u32 i = i0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u32 c = ct_idx[i], d = dec_idx[i];
    bool ok = d < n_keys && c < n_cts;
    g1a Ui, Y;
    ok = g1_decompress(Ui, ui + 48 * (size_t)i) && ok;
    g1a_st ks = keys[d < n_keys ? d : 0];
    ok = ok && ks.ok;
    st_to_g1a(Y, ks);
    g1 p, q;
    if (ok && !key_suspect_live(susp, d, n_keys)) {
        u32 a, b;
        rlc_scalar(key, i, a, b);
        // share side inlined (measured 144.7 vs 148.8 ms per 1M-share step with the call), key side from the key's
        // fixed-base table (148.8 vs 159.8 ms without)
        g1_mul_ab_inl(p, Ui, a, b);
        if (ktab_usable(ktab_ok, d)) g1_mul_ab_tab(q, ktab, n_keys, d, a, b);
        else g1_mul_ab_n(q, Y, a, b);
    } else {                             // an invalid (or suspect) share contributes nothing to its group
        jac_set_inf(p);
        jac_set_inf(q);
    }
    g1_store_soa(rU, n, i, p);
    g1_store_soa(rY, n, i, q);
    accept[i] = ok;
}

// ---------------------------------------------------------------- level-1 groups: runs of one ciphertext / message
// one lane per share; the first share of a run emits the run as groups of at most `cap` shares.
// desc = {first share, length, ciphertext / message, 0}; order of the records is irrelevant
extern "C" __global__ void LCB_BOUNDS k_rlc_groups(const u32 *key_idx, u32 i0, u32 n, u32 n_keys, u32 cap,
                                                  uint4 *desc, u32 *count) {
    u32 i = i0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u32 c = key_idx[i];
    c = c < n_keys ? c : 0;
    if (i > i0) {
        u32 p = key_idx[i - 1];
        p = p < n_keys ? p : 0;
        if (p == c) return;
    }
    u32 j = i + 1;
    while (j < n) {
        u32 q = key_idx[j];
        q = q < n_keys ? q : 0;
        if (q != c) break;
        j++;
    }
    for (u32 st = i; st < j; st += cap) {
        u32 len = min(cap, j - st);
        u32 slot = atomicAdd(count, 1u);
        desc[slot] = make_uint4(st, len, c, 0);
    }
}

// ---------------------------------------------------------------- TPKE group sums -> two affine points per group
// gpts[2g] = sum s_i U_i, gpts[2g + 1] = -sum s_i Y_i (g1a_st records; inf = 1 for the point at infinity).
// desc.w = 0: a randomized group.  A group of an invalid ciphertext rejects its shares; a group whose ciphertext's W
// is outside G2 (the pairing is linear in its G1 argument only for a G2 point: W comes from the wire unchecked) is
// handed to exact checks (gexact = 1: resolve re-emits its shares as desc.w = 1 singles).  Both check two points at
// infinity (they pass).  desc.w = 1: the exact single check of share desc.x, e(U_i, H) e(-Y_i, W) == 1 as
// k_tpke_miller does it (a share already rejected checks infinity).
// Shares of suspect keys are skipped (they have singles of their own).  A single re-derives the share's whole
// validity (census singles have had none yet): a share that is not live is rejected, and cval (census only) records
// which shares were live.
extern "C" __global__ void LCB_BOUNDS k_tpke_rlc_sum(const uint4 *desc, u32 n_groups, u32 lanes, const uint8_t *ct_ok,
                                                    const uint8_t *ct_g2, const g1a_st *keys, u32 n_keys,
                                                    const u32 *dec_idx, const uint8_t *ui, const u32 *rU,
                                                    const u32 *rY, u32 n, g1a_st *gpts, uint8_t *accept,
                                                    uint8_t *gexact, u32 *wsum, const u32 *susp, uint8_t *cval) {
    // lanes = 4 (latency-bound levels): four lanes per group, t = 4g + 2 half + side — side 0 sums the U records,
    // side 1 the Y records, each half half of the group's shares; half 1's partial sum reaches half 0 through LDS (one
    // addition), so the serial chain is ~len/2 additions + one inversion.  lanes = 1 (levels of many entries, e.g.
    // every share a single when every key is suspect): one lane per group does both sides.  Singles and invalid
    // ciphertexts are handled by the group's first lane.  (wsum: unused — TPKE forms its weighted sums at level 2.)
    __shared__ g1 part[LCB_BLOCK];
    const u32 t = blockIdx.x * blockDim.x + threadIdx.x;
    const bool four = lanes == 4;
    const bool in = t < (four ? 4 * n_groups : n_groups);
    const u32 g = four ? t >> 2 : t, side = four ? t & 1 : 0, half = four ? (t >> 1) & 1 : 0;
    const bool lead = in && !side && !half;
    bool work = false;
    g1 su[2];
    jac_set_inf(su[0]);
    jac_set_inf(su[1]);
    if (in) {
        const uint4 dsc = desc[g];
        g1a_st o;
        g1_inf_st(o);
        if (dsc.w == 1) {                // exact single of share dsc.x of ciphertext dsc.z
            if (lead) {
                gexact[g] = 0;
                g1a U, Y;
                U.inf = Y.inf = true;
                u32 d = dec_idx[dsc.x];
                bool live = accept[dsc.x] != 0 && d < n_keys && ct_ok[dsc.z];
                if (live) {
                    g1a_st ks = keys[d];
                    live = ks.ok && g1_decompress(U, ui + 48 * (size_t)dsc.x);
                    st_to_g1a(Y, ks);
                }
                if (!live) accept[dsc.x] = 0;
                if (cval) cval[dsc.x] = live;
                if (live && !U.inf) { o.x = U.x; o.y = U.y; o.inf = 0; }
                gpts[2 * (size_t)g] = o;
                g1_inf_st(o);
                if (live && !Y.inf) { o.x = Y.x; fp_neg(o.y, Y.y); o.inf = 0; }
                gpts[2 * (size_t)g + 1] = o;
            }
        } else {
            const bool cok = ct_ok[dsc.z];
            if (!cok || !ct_g2[dsc.z]) {
                if (!half) {
                    gpts[2 * (size_t)g + side] = o;
                    if (!four) gpts[2 * (size_t)g + 1] = o;
                }
                if (lead) {
                    gexact[g] = cok ? 1 : 0;
                    if (!cok)
                        for (u32 j = 0; j < dsc.y; j++) accept[dsc.x + j] = 0;
                }
            } else {
                if (lead) gexact[g] = 0;
                work = true;
                const u32 mid = four ? dsc.y / 2 : 0, j0 = half ? mid : 0, j1 = (four && !half) ? mid : dsc.y;
                g1 tp;
                for (u32 j = j0; j < j1; j++) {
                    if (key_suspect(susp, dec_idx[dsc.x + j], n_keys)) continue;
                    g1_load_soa(tp, side ? rY : rU, n, dsc.x + j);
                    grp_add(su[0], su[0], tp);
                    if (!four) {
                        g1_load_soa(tp, rY, n, dsc.x + j);
                        grp_add(su[1], su[1], tp);
                    }
                }
            }
        }
    }
    if (four) {
        if (half) part[threadIdx.x] = su[0];
        __syncthreads();
        if (half) work = false;
        else {
            g1 other = part[threadIdx.x + 2];
            if (work) grp_add(su[0], su[0], other);
        }
    }
    if (work) {
        g1a_st o;
        g1_to_st(o, su[0], side != 0);
        gpts[2 * (size_t)g + side] = o;
        if (!four) {
            g1_to_st(o, su[1], true);
            gpts[2 * (size_t)g + 1] = o;
        }
    }
}

// the weighted sums of the level-1 groups listed in sdesc (.w = level-1 group index) as affine records
extern "C" __global__ void LCB_BOUNDS k_tpke_rlc_wsum(const uint4 *sdesc, u32 n_s, const u32 *wsum, u32 n_l1,
                                                     g1a_st *gpts) {
    u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_s) return;
    u32 l = sdesc[g].w;
    g1 p;
    g1a_st o;
    g1_load_soa(p, wsum, 2 * (size_t)n_l1, 2 * (size_t)l);
    g1_to_st(o, p, false);
    gpts[2 * (size_t)g] = o;
    g1_load_soa(p, wsum, 2 * (size_t)n_l1, 2 * (size_t)l + 1);
    g1_to_st(o, p, true);
    gpts[2 * (size_t)g + 1] = o;
}

// Level 2 of TPKE (two-error location, see k_tpke_rlc_search2): the weighted sums of the failed level-1 groups listed
// in sdesc, formed from the shares' randomised records: four lanes per group ((U, Y) side x (w, v) output), last share to first,
// s = suffix sum, w = sum of the s (weights c_j = j + 1), v = sum of the w (weights t_j = c_j (c_j + 1) / 2).  Shares of
// suspect keys keep their positions and add nothing.  gpts[2g + side] = w, gpts[2 (ns + g) + side] = v (Y side
// negated), so checks g and ns + g give gamma_c = prod g_i^(c_i s_i) and gamma_t = prod g_i^(t_i s_i).
extern "C" __global__ void LCB_BOUNDS k_tpke_rlc_wsum2(const uint4 *sdesc, u32 ns, const u32 *rU, const u32 *rY, u32 n,
                                                      const u32 *dec_idx, u32 n_keys, const u32 *susp, g1a_st *gpts) {
    // four lanes per group: (side, which) — each lane one output record, so one inversion (to affine) per lane
    u32 t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 4 * ns) return;
    const u32 g = t >> 2, side = t & 1, which = (t >> 1) & 1;
    const uint4 d = sdesc[g];
    const u32 *rec = side ? rY : rU;
    g1 sa, wa, va, p;
    jac_set_inf(sa);
    jac_set_inf(wa);
    jac_set_inf(va);
    for (u32 j = d.y; j-- > 0;) {
        if (!key_suspect(susp, dec_idx[d.x + j], n_keys)) {
            g1_load_soa(p, rec, n, d.x + j);
            grp_add(sa, sa, p);
        }
        grp_add(wa, wa, sa);
        if (which) grp_add(va, va, wa);
    }
    g1a_st o;
    g1_to_st(o, which ? va : wa, side != 0);
    gpts[2 * ((size_t)(which ? ns : 0) + g) + side] = o;
}

// ---------------------------------------------------------------- TPKE group Miller loops (k_tpke_miller's loop)
extern "C" __global__ void LCB_PAIR_BOUNDS k_tpke_rlc_miller(const u32 *lines, const uint4 *desc, const g1a_st *gpts,
                                                            u32 n_groups, u32 *f_soa, uint8_t *gacc) {
    __shared__ uint4 lds_pts[12 * LCB_BLOCK];
    u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_groups) return;
    u32 c = desc[g].z;
    g1a P, Q;
    st_to_g1a(P, gpts[2 * (size_t)g]);
    st_to_g1a(Q, gpts[2 * (size_t)g + 1]);
    fp12 f;
    const u32 *lsH = lines + (size_t)(2 * c) * LCB_LINESET_WORDS, *lsW = lines + (size_t)(2 * c + 1) * LCB_LINESET_WORDS;
    if (lineset_normalised(lsH) && lineset_normalised(lsW)) {
        uint4 *pt = lds_pts + threadIdx.x;
        g1_park_lds(pt, P);
        g1_park_lds(pt + 6 * LCB_BLOCK_PTS, Q);
        miller2_norm_lds(f, lsH, pt, P.inf, lsW, pt + 6 * LCB_BLOCK_PTS, Q.inf);
    } else {
        miller2_sets_fallback(f, lsH, P, lsW, Q);
    }
    fp12_store_soa(f_soa, n_groups, g, f);
    gacc[g] = 1;
}

// ---------------------------------------------------------------- threshold signatures (ValidateSignature)
// e(PK_i, H(m)) == e(G, sig_i) <=> e(PK_i, H) e(-G, sig_i) == 1.  The randomisation of sig_i uses linearity of the
// pairing in its G2 argument, which holds on G2: a share whose sig_i is outside G2 (G2.FromBytes does not check) is
// emitted straight away as an exact single (desc.w = 1) and contributes nothing to its group.
// TS group record: g1a_st P (sum s_i PK_i) then g2a_st S (sum s_i sig_i), 320 B
struct ts_grp { g1a_st p; g2a_st s; };
extern "C" __global__ void LCB_BOUNDS k_ts_rlc_points(u32 n_msgs, const g1a_st *pks, u32 n_pks, const u32 *msg_idx,
                                                     const u32 *pk_idx, const uint8_t *sigs, u32 i0, u32 n,
                                                     rlc_key key, u32 *rP, u32 *rS, uint8_t *accept, uint4 *desc,
                                                     u32 *count, const u32 *ktab, const uint8_t *ktab_ok,
                                                     const u32 *susp) {
    u32 i = i0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u32 m = msg_idx[i], k = pk_idx[i];
    bool ok = k < n_pks && m < n_msgs;
    g2a S;
    g1a PK;
    ok = g2_decompress(S, sigs + 96 * (size_t)i) && ok;
    g1a_st ps = pks[k < n_pks ? k : 0];
    ok = ok && ps.ok;
    st_to_g1a(PK, ps);
    g1 p;
    g2 q;
    jac_set_inf(p);
    jac_set_inf(q);
    if (ok && !key_suspect_live(susp, k, n_pks)) {      // (a suspect key's shares get their singles from the split)
        if (g2_in_subgroup_inl(S)) {    // inline: measured faster than the call (CommonCoin batch)
            u32 a, b;
            rlc_scalar(key, i, a, b);
            if (ktab_usable(ktab_ok, k)) g1_mul_ab_tab(p, ktab, n_pks, k, a, b);
            else g1_mul_ab_n(p, PK, a, b);
            g2_mul_ab_inl(q, S, a, b);  // inline: 937 vs 1015 ms per 6.55M-share CommonCoin batch with the call
        } else {
            u32 slot = atomicAdd(count, 1u);
            desc[slot] = make_uint4(i, 1, m < n_msgs ? m : 0, 1);
        }
    }
    g1_store_soa(rP, n, i, p);
    g2_store_soa(rS, n, i, q);
    accept[i] = ok;
}
extern "C" __global__ void LCB_BOUNDS k_ts_rlc_sum(const uint4 *desc, u32 n_groups, u32 first, const uint8_t *msg_ok,
                                                  const g1a_st *pks, u32 n_pks, const u32 *pk_idx, const uint8_t *sigs,
                                                  const u32 *rP, const u32 *rS, u32 n, ts_grp *gpts, uint8_t *accept,
                                                  uint8_t *gexact, u32 *wsum, const u32 *susp, uint8_t *cval) {
    u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_groups) return;
    uint4 dsc = desc[g];
    ts_grp o;
    g1_inf_st(o.p);
    g2_inf_st(o.s);
    gexact[g] = 0;
    if (dsc.w == 1) {                    // exact single: the share's own PK and sig (whole validity re-derived)
        u32 k = pk_idx[dsc.x];
        bool live = accept[dsc.x] && msg_ok[dsc.z] && k < n_pks;
        if (live) {
            g2a S;
            live = pks[k].ok && g2_decompress(S, sigs + 96 * (size_t)dsc.x);
            if (live) {
                o.p = pks[k];
                o.s.x = S.x; o.s.y = S.y; o.s.inf = S.inf;
            }
        }
        if (!live) accept[dsc.x] = 0;
        if (cval) cval[dsc.x] = live;
        gpts[g] = o;
        return;
    }
    if (!msg_ok[dsc.z]) {
        for (u32 j = 0; j < dsc.y; j++) accept[dsc.x + j] = 0;
        gpts[g] = o;
        return;
    }
    g1 sp, t, wp;
    g2 ss, u, ws;
    jac_set_inf(sp);
    jac_set_inf(wp);
    jac_set_inf(ss);
    jac_set_inf(ws);
    for (u32 j = dsc.y; j-- > 0;) {
        if (!key_suspect(susp, pk_idx[dsc.x + j], n_pks)) {
            g1_load_soa(t, rP, n, dsc.x + j);
            grp_add(sp, sp, t);
            g2_load_soa(u, rS, n, dsc.x + j);
            grp_add(ss, ss, u);
        }
        if (first) {
            grp_add(wp, wp, sp);
            grp_add(ws, ws, ss);
        }
    }
    if (first) {
        g1_store_soa(wsum, n_groups, g, wp);
        g2_store_soa(wsum + (size_t)36 * n_groups, n_groups, g, ws);
    }
    g1_to_st(o.p, sp, false);
    g2_to_st(o.s, ss);
    gpts[g] = o;
}
extern "C" __global__ void LCB_BOUNDS k_ts_rlc_wsum(const uint4 *sdesc, u32 n_s, const u32 *wsum, u32 n_l1,
                                                   ts_grp *gpts) {
    u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_s) return;
    u32 l = sdesc[g].w;
    g1 p;
    g2 q;
    ts_grp o;
    g1_load_soa(p, wsum, n_l1, l);
    g2_load_soa(q, wsum + (size_t)36 * n_l1, n_l1, l);
    g1_to_st(o.p, p, false);
    g2_to_st(o.s, q);
    gpts[g] = o;
}
// miller2_ts (k_ts.hip): the message's line set with sum s_i PK_i, the group signature's lines on the fly with -G
DN void miller2_ts_grp(fp12 &f, const u32 *lsH, const g1a &PK, const g2a &S, const g1a &G) {
    g2a Q;
    LinesOnTheFly sS;
    sS.init(S);
    if (lineset_normalised(lsH)) {
        LinesNorm sH{lsH};
        miller2(f, sH, PK, sS, G);
    } else {
        lineset_point(Q, lsH);
        LinesOnTheFly sH;
        sH.init(Q);
        miller2(f, sH, PK, sS, G);
    }
}
extern "C" __global__ void LCB_PAIR_BOUNDS k_ts_rlc_miller(const u32 *lines, const uint4 *desc, const ts_grp *gpts,
                                                          u32 n_groups, u32 *f_soa, uint8_t *gacc) {
    u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_groups) return;
    u32 m = desc[g].z;
    g1a P, G;
    g2a S;
    st_to_g1a(P, gpts[g].p);
    st_to_g2a(S, gpts[g].s);
    g1_generator(G);
    fp_neg(G.y, G.y);
    fp12 f;
    miller2_ts_grp(f, lines + (size_t)m * LCB_LINESET_WORDS, P, S, G);
    fp12_store_soa(f_soa, n_groups, g, f);
    gacc[g] = 1;
}

// ---------------------------------------------------------------- resolve a level (TPKE and TS)
// The shares of group d that still need a check of their own, as singles of kind w (0: a group of one randomized
// share, 1: an exact single): not those already rejected, nor those of suspect keys (they have exact singles since
// level 1).
DI void emit_singles(const uint4 &d, u32 w, const uint8_t *accept, const u32 *key_idx, u32 n_keys, const u32 *susp,
                     uint4 *next, u32 *next_count) {
    u32 cnt = 0;
    for (u32 k = 0; k < d.y; k++)
        cnt += accept[d.x + k] && !key_suspect(susp, key_idx[d.x + k], n_keys);
    if (!cnt) return;
    u32 slot = atomicAdd(next_count, cnt);
    for (u32 k = 0; k < d.y; k++)
        if (accept[d.x + k] && !key_suspect(susp, key_idx[d.x + k], n_keys))
            next[slot++] = make_uint4(d.x + k, 1, d.z, w);
}
// Groups [o, o + m) of this level, decided by the final-exponentiation chunk park (stride m).  A failed group of one
// share rejects it.  At level 1 (first) a failed group of len > 1 goes to the search list (its gamma copied out of the
// park); below level 1 it becomes ceil(len / s) sub-groups of s = ceil(len / ceil(sqrt(len))) shares, or single
// shares when len <= LCB_RLC_SINGLES.  gexact (TPKE: W outside G2): every share of the group gets an exact single.
extern "C" __global__ void LCB_BOUNDS k_rlc_resolve(const uint4 *desc, u32 o, u32 m, const uint8_t *gacc,
                                                   const uint8_t *gexact, const u32 *park, u32 first, uint8_t *accept,
                                                   uint4 *next, u32 *next_count, uint4 *search, u32 *search_count,
                                                   u32 *gamma, const u32 *key_idx, u32 n_keys, const u32 *susp) {
    u32 gl = blockIdx.x * blockDim.x + threadIdx.x;
    if (gl >= m) return;
    u32 g = o + gl;
    uint4 d = desc[g];
    if (gexact && gexact[g]) {           // W outside G2: every share of the group gets its exact check
        emit_singles(d, 1, accept, key_idx, n_keys, susp, next, next_count);
        return;
    }
    if (gacc[g]) return;
    if (d.y == 1) { accept[d.x] = 0; return; }        // (exact singles always have d.y == 1)
    if (first) {
        u32 slot = atomicAdd(search_count, 1u);
        search[slot] = make_uint4(d.x, d.y, d.z, g);
        fp12 f;
        fp12_load_soa(f, park, m, gl);
        const u32 *w = (const u32 *)&f;
        uint4 *dst = (uint4 *)(gamma + (size_t)slot * 144);
#pragma unroll
        for (int q = 0; q < 36; q++) dst[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
        return;
    }
    if (d.y <= LCB_RLC_SINGLES) {
        emit_singles(d, 0, accept, key_idx, n_keys, susp, next, next_count);
        return;
    }
    u32 parts = 1;
    while (parts * parts < d.y) parts++;
    u32 s = (d.y + parts - 1) / parts;
    u32 cnt = (d.y + s - 1) / s;
    u32 slot = atomicAdd(next_count, cnt);
    for (u32 k = 0; k < cnt; k++) {
        u32 st = d.x + k * s, len = min(s, d.y - k * s);
        next[slot + k] = make_uint4(st, len, d.z, 0);
    }
}
// Level 2: search entries [o, o + m): gamma' (the weighted group check's final-exponentiation output, park stride m)
// against gamma^c, c = 1..len.  A match rejects share c - 1 of the group (the only bad one, see the header); no match
// sends every share of the group to a single check at the next level.
extern "C" __global__ void LCB_BOUNDS k_rlc_search(const uint4 *search, u32 o, u32 m, const u32 *gamma, const u32 *park,
                                                  uint8_t *accept, uint4 *next, u32 *next_count, const u32 *key_idx,
                                                  u32 n_keys, const u32 *susp) {
    u32 gl = blockIdx.x * blockDim.x + threadIdx.x;
    if (gl >= m) return;
    u32 g = o + gl;
    uint4 d = search[g];
    fp12 gm, gp, acc;
    u32 *w = (u32 *)&gm;
    const uint4 *src = (const uint4 *)(gamma + (size_t)g * 144);
#pragma unroll
    for (int q = 0; q < 36; q++) {
        uint4 v = src[q];
        w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
    fp12_load_soa(gp, park, m, gl);
    acc = gm;
    u32 found = 0;
    for (u32 c = 1; c <= d.y; c++) {
        const u32 *a = (const u32 *)&acc, *b = (const u32 *)&gp;
        u32 x = 0;
#pragma unroll
        for (int q = 0; q < 144; q++) x |= a[q] ^ b[q];
        if (x == 0) { found = c; break; }
        fp12_mul_n(acc, acc, gm);
    }
    if (found) {
        accept[d.x + found - 1] = 0;
        return;
    }
    emit_singles(d, 0, accept, key_idx, n_keys, susp, next, next_count);
}

// the final-exponentiation outputs of checks [o, o + m) (park stride m) -> rows o.. of dst (576 B each)
extern "C" __global__ void LCB_BOUNDS k_rlc_park_copy(const u32 *park, u32 o, u32 m, u32 *dst) {
    u32 gl = blockIdx.x * blockDim.x + threadIdx.x;
    if (gl >= m) return;
    fp12 f;
    fp12_load_soa(f, park, m, gl);
    const u32 *w = (const u32 *)&f;
    uint4 *d = (uint4 *)(dst + (size_t)(o + gl) * 144);
#pragma unroll
    for (int q = 0; q < 36; q++) d[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}
DI void fp12_load_row(fp12 &f, const u32 *row) {
    u32 *w = (u32 *)&f;
    const uint4 *src = (const uint4 *)row;
#pragma unroll
    for (int q = 0; q < 36; q++) {
        uint4 v = src[q];
        w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
}
DI bool fp12_words_eq(const fp12 &a, const fp12 &b) {
    const u32 *x = (const u32 *)&a, *y = (const u32 *)&b;
    u32 d = 0;
#pragma unroll
    for (int q = 0; q < 144; q++) d |= x[q] ^ y[q];
    return d == 0;
}
// r = a^e for a in the cyclotomic subgroup (GT), 1 <= e < 2^8
DN void gt_pow_small(fp12 &r, const fp12 &a, u32 e) {
    fp12 t = a;
    int top = 7;
    while (top > 0 && !((e >> top) & 1)) top--;
    for (int b = top - 1; b >= 0; b--) {
        fp12_cyc_sqr_n(t, t);
        if ((e >> b) & 1) fp12_mul_n(t, t, a);
    }
    r = t;
}
DI u32 fp12_fingerprint(const fp12 &a) {
    const u32 *w = (const u32 *)&a;
    u32 h = 0;
#pragma unroll
    for (int q = 0; q < 144; q++) h = ((h << 5) | (h >> 27)) ^ w[q];
    return h;
}
DI u32 half_ballot(bool p) {
    const unsigned long long m = __ballot(p);
    return (u32)(m >> (32 * ((threadIdx.x >> 5) & 1)));
}
// Level 2 of TPKE: locate up to TWO bad shares per failed group.  With e_i = s_i log g_i (nonzero exactly for the bad
// shares) the three group values are gamma_0 (level 1) ~ sum e_i, gamma_c ~ sum e_i c_i and gamma_t ~ sum e_i t_i, so
// gamma_2 = gamma_t^2 / gamma_c ~ sum e_i c_i^2 (c^2 = 2t - c).
//   one error at j:      gamma_c = gamma_0^(c_j)  (k_tpke_rlc_search2a: one lane per group, c = 1..len as k_rlc_search);
//   two errors at j, k:  for lane j of the group's half-wave (k_tpke_rlc_search2b, only the groups 2a left open),
//                        D_j = gamma_c / gamma_0^(c_j) ~ e_k (c_k - c_j) and E_j = gamma_2 / gamma_c^(c_j) ~
//                        e_k c_k (c_k - c_j), so E_j = D_j^(c_k): exactly two lanes whose searches name each other
//                        reject both shares.
// Any other outcome (three or more bad shares) sends the group's shares to single checks.  A false location needs a
// relation among the e_i, whose factors s_i are secret: probability <= len^2 2^-64 per group.
extern "C" __global__ void LCB_BOUNDS k_tpke_rlc_search2a(const uint4 *search, u32 ns, const u32 *gamma0,
                                                         const u32 *gamma12, uint8_t *accept, u32 *open,
                                                         u32 *open_count) {
    u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= ns) return;
    const uint4 d = search[g];
    fp12 gm, gc, acc;
    fp12_load_row(gm, gamma0 + (size_t)g * 144);
    fp12_load_row(gc, gamma12 + (size_t)g * 144);
    acc = gm;
    u32 found = 0;
    for (u32 c = 1; c <= d.y; c++) {
        if (fp12_words_eq(acc, gc)) { found = c; break; }
        if (c < d.y) fp12_mul_n(acc, acc, gm);
    }
    if (found) accept[d.x + found - 1] = 0;
    else open[atomicAdd(open_count, 1u)] = g;
}
extern "C" __global__ void __launch_bounds__(64) k_tpke_rlc_search2b(const uint4 *search, u32 ns, const u32 *gamma0,
                                                                    const u32 *gamma12, const u32 *open,
                                                                    const u32 *open_count, uint8_t *accept, uint4 *next,
                                                                    u32 *next_count, const u32 *key_idx, u32 n_keys,
                                                                    const u32 *susp) {
    const u32 j = threadIdx.x & 31, k = blockIdx.x * 2 + (threadIdx.x >> 5);
    if (blockIdx.x * 2 >= *open_count) return;          // (uniform per block)
    const bool live = k < *open_count;
    const u32 g = live ? open[k] : 0;
    const uint4 d = live ? search[g] : make_uint4(0, 0, 0, 0);
    const bool cand = live && j < d.y && accept[d.x + j] && !key_suspect(susp, key_idx[d.x + j], n_keys);
    const u32 cj = j + 1;
    fp12 a, b, D;
    fp12_load_row(a, gamma0 + (size_t)g * 144);
    gt_pow_small(b, a, cj);
    fp12_conj(b, b);
    fp12_load_row(a, gamma12 + (size_t)g * 144);           // gamma_c
    fp12_mul_n(D, a, b);                                   // D_j = gamma_c / gamma_0^(c_j)
    gt_pow_small(b, a, cj + 1);                            // gamma_c^(c_j + 1)
    fp12_conj(b, b);
    fp12_load_row(a, gamma12 + ((size_t)ns + g) * 144);    // gamma_t
    fp12_cyc_sqr_n(a, a);
    fp12_mul_n(a, a, b);                                   // E_j = gamma_t^2 / gamma_c^(c_j + 1) = gamma_2 / gamma_c^(c_j)
    // E_j = D_j^c for some c in [1, len] (len <= 32): baby-step giant-step with m = 6 — 32-bit fingerprints of the
    // baby values D^k (k = 1..6), giant steps Y_i = E D^(-6 i) (D is unitary: D^-6 = conj(D^6)), a fingerprint match
    // confirmed by the full comparison E == D^c: 10 products instead of up to len
    u32 found = 0;
    if (cand) {
        u32 fpb[6];
        fpb[0] = fp12_fingerprint(D);
        b = D;
#pragma unroll
        for (int k = 1; k < 6; k++) {
            fp12_mul_n(b, b, D);
            fpb[k] = fp12_fingerprint(b);
        }
        fp12_conj(b, b);                                   // D^-6
        fp12 E = a;                                        // Y_0
        for (int i = 0; i < 6 && !found; i++) {
            const u32 h = fp12_fingerprint(a);
#pragma unroll
            for (int k = 0; k < 6; k++) {
                const u32 c = 6 * i + k + 1;
                if (!found && h == fpb[k] && c <= d.y && c != cj) {
                    fp12 chk;
                    gt_pow_small(chk, D, c);
                    if (fp12_words_eq(chk, E)) found = c;
                }
            }
            if (i < 5) fp12_mul_n(a, a, b);
        }
    }
    const u32 m2 = half_ballot(found != 0);
    const u32 m3 = half_ballot(found != 0 && !((m2 >> (found - 1)) & 1u));
    if (__popc(m2) == 2 && !m3) {
        if (found) accept[d.x + j] = 0;
    } else if (live && j == 0) {
        emit_singles(d, 0, accept, key_idx, n_keys, susp, next, next_count);
    }
}

// ---------------------------------------------------------------- census (suspect keys) and the level-1 split
// exact singles of shares [0, m): desc = {i, 1, group index (ciphertext / message), 1}; an out-of-range index rejects
extern "C" __global__ void LCB_BOUNDS k_rlc_census_desc(const u32 *grp_idx, const u32 *key_idx, u32 m, u32 n_grp,
                                                       u32 n_keys, uint4 *desc, uint8_t *accept) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    u32 c = grp_idx[i];
    bool ok = c < n_grp && key_idx[i] < n_keys;
    accept[i] = ok;
    desc[i] = make_uint4(i, 1, ok ? c : 0, 1);
}
// one lane per key: over the census shares that were live (cval), the key is suspect when at least two were sampled
// and at least half of them failed their exact check.  count[0] += suspect keys.
extern "C" __global__ void LCB_BOUNDS k_rlc_census_stats(const u32 *key_idx, u32 m, u32 n_keys, const uint8_t *cval,
                                                        const uint8_t *accept, u32 *susp, u32 *count) {
    u32 k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_keys) return;
    u32 live = 0, bad = 0;
    for (u32 i = 0; i < m; i++) {
        if (key_idx[i] != k || !cval[i]) continue;
        live++;
        bad += accept[i] == 0;
    }
    if (live >= 2 && 2 * bad >= live) {
        atomicOr(susp + (k >> 5), 1u << (k & 31));
        atomicAdd(count, 1u);
    }
}
// level 1 with suspect keys: every group keeps its place (its sum skips the suspect keys' shares) unless it has no
// live share of another key (then it is dropped), and each live share of a suspect key becomes an exact single.  count: [0] entries out
extern "C" __global__ void LCB_BOUNDS k_rlc_suspect_split(const uint4 *desc, u32 n_groups, const u32 *key_idx,
                                                         u32 n_keys, const u32 *susp, const uint8_t *accept,
                                                         uint4 *out, u32 *count) {
    u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_groups) return;
    uint4 d = desc[g];
    u32 ns = 0, nc = 0;
    for (u32 k = 0; k < d.y; k++) {
        if (!accept[d.x + k]) continue;
        if (key_suspect(susp, key_idx[d.x + k], n_keys)) ns++;
        else nc++;
    }
    if (!nc && !ns) return;              // nothing live: every share of the group is already rejected
    u32 slot = atomicAdd(count, ns + (nc ? 1u : 0u));
    if (nc) out[slot++] = d;
    for (u32 k = 0; k < d.y; k++)
        if (accept[d.x + k] && key_suspect(susp, key_idx[d.x + k], n_keys))
            out[slot++] = make_uint4(d.x + k, 1, d.z, 1);
}

// ---------------------------------------------------------------- host launch wrappers
// table workspace per key: Jacobian scratch 144 B + prefix products 48 B + table 144 B per entry + 32 flags
extern "C" size_t lcbk_key_table_bytes(u32 n_keys) {
    return (size_t)n_keys * (LCB_KTAB_ENTRIES * 336 + LCB_KTAB_LANES) + 16;
}
extern "C" void lcbk_rlc_key_tables(dim3 grid, hipStream_t s, const void *keys, u32 n_keys, u32 *ws, u32 **tab,
                                    uint8_t **ktab_ok) {
    const size_t ne = (size_t)n_keys * LCB_KTAB_ENTRIES;
    u32 *jtab = ws, *pre = ws + 36 * ne, *t = ws + 48 * ne;
    uint8_t *okv = (uint8_t *)(ws + 84 * ne);
    *tab = t;
    *ktab_ok = okv;
    grid = dim3((LCB_KTAB_LANES * n_keys + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_rlc_key_tables, (const g1a_st *)keys, n_keys, jtab, pre, t, okv);
}
extern "C" void lcbk_tpke_rlc_points(hipStream_t s, u32 n_cts, const void *keys, u32 n_keys, const u32 *ct_idx,
                                     const u32 *dec_idx, const uint8_t *ui, u32 i0, u32 n, const u32 key[10], u32 *rU,
                                     u32 *rY, uint8_t *accept, const u32 *ktab, const uint8_t *ktab_ok,
                                     const u32 *susp) {
    rlc_key k;
    for (int j = 0; j < 8; j++) k.k[j] = key[j];
    k.nonce[0] = key[8];
    k.nonce[1] = key[9];
    dim3 grid((n - i0 + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_tpke_rlc_points, n_cts, (const g1a_st *)keys, n_keys, ct_idx, dec_idx, ui, i0, n, k, rU, rY, accept,
               ktab, ktab_ok, susp);
}
extern "C" void lcbk_ts_rlc_points(hipStream_t s, u32 n_msgs, const void *pks, u32 n_pks, const u32 *msg_idx,
                                   const u32 *pk_idx, const uint8_t *sigs, u32 i0, u32 n, const u32 key[10], u32 *rP,
                                   u32 *rS, uint8_t *accept, void *desc, u32 *count, const u32 *ktab,
                                   const uint8_t *ktab_ok, const u32 *susp) {
    rlc_key k;
    for (int j = 0; j < 8; j++) k.k[j] = key[j];
    k.nonce[0] = key[8];
    k.nonce[1] = key[9];
    dim3 grid((n - i0 + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_ts_rlc_points, n_msgs, (const g1a_st *)pks, n_pks, msg_idx, pk_idx, sigs, i0, n, k, rP, rS, accept,
               (uint4 *)desc, count, ktab, ktab_ok, susp);
}
extern "C" void lcbk_rlc_groups(hipStream_t s, const u32 *key_idx, u32 i0, u32 n, u32 n_keys, u32 cap, void *desc,
                                u32 *count) {
    dim3 grid((n - i0 + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_rlc_groups, key_idx, i0, n, n_keys, cap, (uint4 *)desc, count);
}
extern "C" void lcbk_tpke_rlc_sum(dim3 grid, hipStream_t s, const void *desc, u32 n_groups, u32 lanes,
                                  const uint8_t *ct_ok, const uint8_t *ct_g2, const void *keys, u32 n_keys,
                                  const u32 *dec_idx, const uint8_t *ui, const u32 *rU, const u32 *rY, u32 n,
                                  void *gpts, uint8_t *accept, uint8_t *gexact, u32 *wsum, const u32 *susp,
                                  uint8_t *cval) {
    LCB_LAUNCH(k_tpke_rlc_sum, (const uint4 *)desc, n_groups, lanes, ct_ok, ct_g2, (const g1a_st *)keys, n_keys,
               dec_idx, ui, rU, rY, n, (g1a_st *)gpts, accept, gexact, wsum, susp, cval);
}
extern "C" void lcbk_tpke_rlc_wsum(dim3 grid, hipStream_t s, const void *sdesc, u32 n_s, const u32 *wsum, u32 n_l1,
                                   void *gpts) {
    LCB_LAUNCH(k_tpke_rlc_wsum, (const uint4 *)sdesc, n_s, wsum, n_l1, (g1a_st *)gpts);
}
extern "C" void lcbk_tpke_rlc_miller(dim3 grid, hipStream_t s, const u32 *lines, const void *desc, const void *gpts,
                                     u32 n_groups, u32 *f_soa, uint8_t *gacc) {
    LCB_LAUNCH(k_tpke_rlc_miller, lines, (const uint4 *)desc, (const g1a_st *)gpts, n_groups, f_soa, gacc);
}
extern "C" void lcbk_ts_rlc_sum(dim3 grid, hipStream_t s, const void *desc, u32 n_groups, u32 first,
                                const uint8_t *msg_ok, const void *pks, u32 n_pks, const u32 *pk_idx,
                                const uint8_t *sigs, const u32 *rP, const u32 *rS, u32 n, void *gpts, uint8_t *accept,
                                uint8_t *gexact, u32 *wsum, const u32 *susp, uint8_t *cval) {
    LCB_LAUNCH(k_ts_rlc_sum, (const uint4 *)desc, n_groups, first, msg_ok, (const g1a_st *)pks, n_pks, pk_idx, sigs,
               rP, rS, n, (ts_grp *)gpts, accept, gexact, wsum, susp, cval);
}
extern "C" void lcbk_ts_rlc_wsum(dim3 grid, hipStream_t s, const void *sdesc, u32 n_s, const u32 *wsum, u32 n_l1,
                                 void *gpts) {
    LCB_LAUNCH(k_ts_rlc_wsum, (const uint4 *)sdesc, n_s, wsum, n_l1, (ts_grp *)gpts);
}
extern "C" void lcbk_ts_rlc_miller(dim3 grid, hipStream_t s, const u32 *lines, const void *desc, const void *gpts,
                                   u32 n_groups, u32 *f_soa, uint8_t *gacc) {
    LCB_LAUNCH(k_ts_rlc_miller, lines, (const uint4 *)desc, (const ts_grp *)gpts, n_groups, f_soa, gacc);
}
extern "C" void lcbk_rlc_resolve(dim3 grid, hipStream_t s, const void *desc, u32 o, u32 m, const uint8_t *gacc,
                                 const uint8_t *gexact, const u32 *park, u32 first, uint8_t *accept, void *next,
                                 u32 *next_count, void *search, u32 *search_count, u32 *gamma, const u32 *key_idx,
                                 u32 n_keys, const u32 *susp) {
    LCB_LAUNCH(k_rlc_resolve, (const uint4 *)desc, o, m, gacc, gexact, park, first, accept, (uint4 *)next, next_count,
               (uint4 *)search, search_count, gamma, key_idx, n_keys, susp);
}
extern "C" void lcbk_rlc_search(dim3 grid, hipStream_t s, const void *search, u32 o, u32 m, const u32 *gamma,
                                const u32 *park, uint8_t *accept, void *next, u32 *next_count, const u32 *key_idx,
                                u32 n_keys, const u32 *susp) {
    LCB_LAUNCH(k_rlc_search, (const uint4 *)search, o, m, gamma, park, accept, (uint4 *)next, next_count, key_idx,
               n_keys, susp);
}
extern "C" void lcbk_tpke_rlc_wsum2(hipStream_t s, const void *sdesc, u32 ns, const u32 *rU, const u32 *rY, u32 n,
                                    const u32 *dec_idx, u32 n_keys, const u32 *susp, void *gpts) {
    dim3 grid((4 * (size_t)ns + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_tpke_rlc_wsum2, (const uint4 *)sdesc, ns, rU, rY, n, dec_idx, n_keys, susp, (g1a_st *)gpts);
}
extern "C" void lcbk_rlc_park_copy(hipStream_t s, const u32 *park, u32 o, u32 m, u32 *dst) {
    dim3 grid((m + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_rlc_park_copy, park, o, m, dst);
}
extern "C" void lcbk_tpke_rlc_search2(hipStream_t s, const void *search, u32 ns, const u32 *gamma0, const u32 *gamma12,
                                      uint8_t *accept, void *next, u32 *next_count, const u32 *key_idx, u32 n_keys,
                                      const u32 *susp, u32 *open, u32 *open_count) {
    (void)hipMemsetAsync(open_count, 0, 4, s);
    dim3 grid((ns + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_tpke_rlc_search2a, (const uint4 *)search, ns, gamma0, gamma12, accept, open, open_count);
    hipLaunchKernelGGL(k_tpke_rlc_search2b, dim3((ns + 1) / 2), dim3(64), 0, s, (const uint4 *)search, ns, gamma0,
                       gamma12, open, open_count, accept, (uint4 *)next, next_count, key_idx, n_keys, susp);
}
extern "C" void lcbk_rlc_census_desc(hipStream_t s, const u32 *grp_idx, const u32 *key_idx, u32 m, u32 n_grp,
                                     u32 n_keys, void *desc, uint8_t *accept) {
    dim3 grid((m + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_rlc_census_desc, grp_idx, key_idx, m, n_grp, n_keys, (uint4 *)desc, accept);
}
extern "C" void lcbk_rlc_census_stats(hipStream_t s, const u32 *key_idx, u32 m, u32 n_keys, const uint8_t *cval,
                                      const uint8_t *accept, u32 *susp, u32 *count) {
    dim3 grid((n_keys + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_rlc_census_stats, key_idx, m, n_keys, cval, accept, susp, count);
}
extern "C" void lcbk_rlc_suspect_split(hipStream_t s, const void *desc, u32 n_groups, const u32 *key_idx, u32 n_keys,
                                       const u32 *susp, const uint8_t *accept, void *out, u32 *count) {
    dim3 grid((n_groups + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_rlc_suspect_split, (const uint4 *)desc, n_groups, key_idx, n_keys, susp, accept, (uint4 *)out, count);
}
extern "C" size_t lcbk_ts_grp_bytes() { return sizeof(ts_grp); }
