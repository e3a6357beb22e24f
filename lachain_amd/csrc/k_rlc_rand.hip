// lachain_amd/csrc/k_rlc_rand.hip — gfx950 kernels of the randomized batch check's first phase (TPKE): the
// validators' fixed-base tables, the per-share randomisation and the group sums (levels 1 and 2).  A translation unit
// of its own so that it builds without VGPR-to-AGPR spilling (Makefile): these kernels then fit 256 registers and run
// two waves per SIMD (measured 98.5 vs 102.0 ms per 1M-share step, profiles/r03/abf); the pairing kernels of
// k_batch.hip keep the AGPR spills (scratch spills measured slower there).  The algorithm is described in k_batch.hip.
#include "kcommon.hpp"
#include "rlc_common.hpp"

LCB_ASM_LIBRARY(k_rlc_rand)
LCB_TU_CONFIG(k_rlc_rand)

extern "C" __global__ void LCB_BOUNDS k_rlc_key_tables(const g1a_st *keys, u32 n_keys, u32 *jtab, u32 *pre, u32 *tab,
                                                      uint8_t *ktab_ok) {
    LCB_LATENCY_PRIO();          // a short serial chain ahead of the randomisation, beside the preparation's waves
    u32 t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= LCB_KTAB_LANES * n_keys) return;
    u32 k = t / LCB_KTAB_LANES, w = (t / LCB_KTAB_CHUNKS) & 3, ch = t % LCB_KTAB_CHUNKS;
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
    fp_inv_gcd(inv, run);                              // 1 / (z_d0 ... z_d1)
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
    if (ok && !key_suspect_live(susp, d, n_keys)) {
        u32 a, b;
        rlc_scalar(key, i, a, b);
        // share side inlined (measured 144.7 vs 148.8 ms per 1M-share step with the call), key side from the key's
        // fixed-base table (148.8 vs 159.8 ms without).  Each record is stored as soon as it is formed (round 6): the
        // share side's point is then not live across the key side's call (its 36 words were the kernel's spills)
        {
            g1 p;
            g1_mul_ab_inl(p, Ui, a, b);
            g1_store_soa(rU, n, i, p);
        }
        g1 q;
        if (ktab_usable(ktab_ok, d)) g1_mul_ab_tab(q, ktab, n_keys, d, a, b);
        else g1_mul_ab_n(q, Y, a, b);
        g1_store_soa(rY, n, i, q);
    } else {                             // an invalid (or suspect) share contributes nothing to its group
        g1 p;
        jac_set_inf(p);
        g1_store_soa(rU, n, i, p);
        g1_store_soa(rY, n, i, p);
    }
    accept[i] = ok;
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
    LCB_LATENCY_PRIO();
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
        g1_to_st_gcd(o, su[0], side != 0);
        gpts[2 * (size_t)g + side] = o;
        if (!four) {
            g1_to_st_gcd(o, su[1], true);
            gpts[2 * (size_t)g + 1] = o;
        }
    }
}

// Level 2 of TPKE (two-error location, see k_tpke_rlc_search2a/2b): the weighted sums of failed level-1 groups,
// formed from the shares' randomised records, last share to first: s = suffix sum, w = sum of the s (weights c_j =
// j + 1), v = sum of the w (weights t_j = c_j (c_j + 1) / 2).  Shares of suspect keys keep their positions and add
// nothing.  Two lanes per group ((U, Y) side), the Y side negated, so a check gives gamma_c = prod g_i^(c_i s_i) (w) or
// gamma_t = prod g_i^(t_i s_i) (v):
//   open == nullptr: the w sums of the ns groups of sdesc -> gpts[2 g + side]
//   open != nullptr: the v sums of the ns groups open[k] the one-error search left open -> gpts[2 k + side], and
//                    their descriptors -> sdesc_out[k] (gamma_t is needed for those alone)
extern "C" __global__ void LCB_BOUNDS k_tpke_rlc_wsum2(const uint4 *sdesc, u32 ns, const u32 *open, const u32 *rU,
                                                      const u32 *rY, u32 n, const u32 *dec_idx, u32 n_keys,
                                                      const u32 *susp, g1a_st *gpts, uint4 *sdesc_out) {
    LCB_LATENCY_PRIO();
    const u32 t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 2 * ns) return;
    const u32 k = t >> 1, side = t & 1, g = open ? open[k] : k;
    const bool which = open != nullptr;
    const uint4 d = sdesc[g];
    if (which && !side) sdesc_out[k] = d;
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
    g1_to_st_gcd(o, which ? va : wa, side != 0);
    gpts[2 * (size_t)k + side] = o;
}

// ---------------------------------------------------------------- threshold signatures: per-share randomisation
// (k_batch.hip describes the check).  Built here, without VGPR-to-AGPR spilling and for two waves per SIMD (256
// registers, the rest spilled to scratch), like k_tpke_rlc_points: in k_batch.hip it took 512 registers, one wave
// per SIMD.
extern "C" __global__ void __launch_bounds__(LCB_BLOCK) __attribute__((amdgpu_waves_per_eu(2))) k_ts_rlc_points(u32 n_msgs, const g1a_st *pks, u32 n_pks, const u32 *msg_idx,
                                                     const u32 *pk_idx, const uint8_t *sigs, u32 i0, u32 n,
                                                     rlc_key key, u32 *rP, u32 *rS, uint8_t *accept, uint4 *desc,
                                                     u32 *count, const u32 *ktab, const uint8_t *ktab_ok,
                                                     const u32 *susp, ts_share_st *dec) {
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
        const bool in_g2 = g2_in_subgroup_inl(S);       // inline: measured faster than the call (CommonCoin batch)
        if (dec) {                                      // the decoded share for the assembly (ts_share_st)
            ts_share_st *e = dec + i;
            const uint4 *src = (const uint4 *)(sigs + 96 * (size_t)i);
#pragma unroll
            for (int q = 0; q < 6; q++) ((uint4 *)e->raw)[q] = src[q];
            g2a_st o;
            o.x = S.x; o.y = S.y; o.inf = 0; o.ok = 1; o.pad[0] = in_g2 ? 1u : 0u; o.pad[1] = 0;
            e->p = o;
        }
        if (in_g2) {
            u32 a, b;
            rlc_scalar(key, i, a, b);
            if (ktab_usable(ktab_ok, k)) g1_mul_ab_tab(p, ktab, n_pks, k, a, b);
            else g1_mul_ab_n(p, PK, a, b);
#if LCB_G2AB_MEM
            g2_mul_ab_rec(q, S, a, b, rS, n, i);         // (its addends in the output record; rS is written below)
#else
            g2_mul_ab_inl(q, S, a, b);  // inline: 937 vs 1015 ms per 6.55M-share CommonCoin batch with the call
#endif
        } else {
            u32 slot = atomicAdd(count, 1u);
            desc[slot] = make_uint4(i, 1, m < n_msgs ? m : 0, 1);
        }
    }
    g1_store_soa(rP, n, i, p);
    g2_store_soa(rS, n, i, q);
    accept[i] = ok;
}

// ---------------------------------------------------------------- host launch wrappers
extern "C" void lcbk_ts_rlc_points(hipStream_t s, u32 n_msgs, const void *pks, u32 n_pks, const u32 *msg_idx,
                                   const u32 *pk_idx, const uint8_t *sigs, u32 i0, u32 n, const u32 key[10], u32 *rP,
                                   u32 *rS, uint8_t *accept, void *desc, u32 *count, const u32 *ktab,
                                   const uint8_t *ktab_ok, const u32 *susp, void *dec) {
    rlc_key k;
    for (int j = 0; j < 8; j++) k.k[j] = key[j];
    k.nonce[0] = key[8];
    k.nonce[1] = key[9];
    dim3 grid((n - i0 + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_ts_rlc_points, n_msgs, (const g1a_st *)pks, n_pks, msg_idx, pk_idx, sigs, i0, n, k, rP, rS, accept,
               (uint4 *)desc, count, ktab, ktab_ok, susp, (ts_share_st *)dec);
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
extern "C" void lcbk_tpke_rlc_sum(dim3 grid, hipStream_t s, const void *desc, u32 n_groups, u32 lanes,
                                  const uint8_t *ct_ok, const uint8_t *ct_g2, const void *keys, u32 n_keys,
                                  const u32 *dec_idx, const uint8_t *ui, const u32 *rU, const u32 *rY, u32 n,
                                  void *gpts, uint8_t *accept, uint8_t *gexact, u32 *wsum, const u32 *susp,
                                  uint8_t *cval) {
    LCB_LAUNCH(k_tpke_rlc_sum, (const uint4 *)desc, n_groups, lanes, ct_ok, ct_g2, (const g1a_st *)keys, n_keys,
               dec_idx, ui, rU, rY, n, (g1a_st *)gpts, accept, gexact, wsum, susp, cval);
}
extern "C" void lcbk_tpke_rlc_wsum2(hipStream_t s, const void *sdesc, u32 ns, const u32 *open, const u32 *rU,
                                    const u32 *rY, u32 n, const u32 *dec_idx, u32 n_keys, const u32 *susp, void *gpts,
                                    void *sdesc_out) {
    if (!ns) return;
    dim3 grid((2 * (size_t)ns + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_tpke_rlc_wsum2, (const uint4 *)sdesc, ns, open, rU, rY, n, dec_idx, n_keys, susp, (g1a_st *)gpts,
               (uint4 *)sdesc_out);
}
