// lachain_amd/csrc/k_coop.hip — gfx950 kernels of the cooperative pairing check (coop.hpp: nine lanes per check,
// seven checks per wave): the randomized batch check's group Miller loops and final exponentiations at the small
// levels, and the single pairings of the mcl surface.  Same Fp12 values as the one-lane kernels (k_batch.hip,
// k_tpke.hip), which they replace where a launch would be below one wave per SIMD.
#include "coop.hpp"

LCB_ASM_LIBRARY(k_coop)
LCB_TU_CONFIG(k_coop)

// TPKE group check Miller pair (k_tpke_rlc_miller's function): f = f_{|z|,H}(sum s_i U_i) f_{|z|,W}(-sum s_i Y_i)
// conjugated, from the ciphertext's two normalised line sets.  Lanes 3..6 evaluate the line coefficients
// (B'_1 x_1, C'_1 y_1, B'_2 x_2, C'_2 y_2).  A group whose line sets are not normalised (some A_k == 0, only for
// adversarial W) is flagged in fb and left to k_rlc_miller_fallback.
// npairs = 1: only the first pair (mclBn_pairing: the second set is the point at infinity's, whose lines are 1 — the
// skipped products are exact multiplications by 1, so the value is the same)
extern "C" __global__ void __launch_bounds__(CP_BLOCK) k_coop_tpke_miller(const u32 *lines, const uint4 *desc,
                                                                         const g1a_st *gpts, u32 n_groups,
                                                                         u32 *f_soa, uint8_t *gacc, uint8_t *fb,
                                                                         u32 npairs) {
    LCB_LATENCY_PRIO();
    __shared__ uint4 lds[CP_LDS_QUADS];
    const Cp c = cp_init(lds);
    const u32 item = blockIdx.x * CP_G + c.g;
    const bool live = c.g < CP_G && item < n_groups;
    const u32 it = live ? item : 0;
    if (cpj(c) == 0) cp_put(c, S_Z, fp2_zero());
    const u32 ct = desc[it].z;
    const u32 *ls1 = lines + (size_t)(2 * ct) * LCB_LINESET_WORDS, *ls2 = ls1 + LCB_LINESET_WORDS;
    const bool norm = lineset_normalised(ls1) && lineset_normalised(ls2);
    const int e = cpj(c) - 3;
    const bool evl = e >= 0 && e < 4;
    const int ee = evl ? e : 0, pr = ee >> 1, cf = ee & 1;
    const u32 *lse = (pr ? ls2 : ls1) + 24 * cf;
    CpEval ev;
    ev.on = evl;
    {
        const g1a_st *P = gpts + 2 * (size_t)it + pr;
        ev.yinf = P->inf != 0;                               // a point at infinity: every line evaluates to 1
        ev.yp = (const u32 *)(cf ? &P->y : &P->x);
    }
    cp_sync();
    fp2 R;
    cp_one(R, c);
    int k = 0;
#pragma unroll 1
    for (int i = 62; i >= 0; i--) {
        ev.xp = lse + (size_t)k * LCB_NLINE_WORDS;
        if (i == 62) cp_eval_round(c, ev);
        else cp_sqr12(R, c, ev);
        cp_line(R, c, S_LE, S_LE + 1);
        if (npairs > 1) cp_line(R, c, S_LE + 2, S_LE + 3);
        k++;
        if ((LCB_Z_ABS >> i) & 1) {
            ev.xp = lse + (size_t)k * LCB_NLINE_WORDS;
            cp_eval_round(c, ev);
            cp_line(R, c, S_LE, S_LE + 1);
            if (npairs > 1) cp_line(R, c, S_LE + 2, S_LE + 3);
            k++;
        }
    }
    cp_conj(R, c);
    park_put(f_soa, n_groups, it, cpj(c), live && norm, R);
    if (live && cpj(c) == 0) {
        gacc[item] = 1;
        fb[item] = !norm;
    }
}
// the groups k_coop_tpke_miller flagged: one lane each, the one-lane fallback (lines of the un-normalised set computed
// on the fly).  (Built for two waves per SIMD, its waves could be placed beside the randomisation's, but the doubled
// resident-wave count doubled the scratch each HIP queue reserves for it — 4.5 KB per lane — and two bench ranks on
// one GPU then failed a dispatch with HSA_STATUS_ERROR_OUT_OF_RESOURCES: reverted, profiles/r04/r04f.)
extern "C" __global__ void LCB_PAIR_BOUNDS k_rlc_miller_fallback(const u32 *lines, const uint4 *desc, const g1a_st *gpts,
                                                                u32 n_groups, u32 *f_soa, const uint8_t *fb) {
    LCB_LATENCY_PRIO();
    u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_groups || !fb[g]) return;
    u32 c = desc[g].z;
    g1a P, Q;
    st_to_g1a(P, gpts[2 * (size_t)g]);
    st_to_g1a(Q, gpts[2 * (size_t)g + 1]);
    fp12 f;
    miller2_sets_fallback(f, lines + (size_t)(2 * c) * LCB_LINESET_WORDS, P, lines + (size_t)(2 * c + 1) * LCB_LINESET_WORDS, Q);
    fp12_store_soa(f_soa, n_groups, g, f);
}

// accept[i] &= (final_exp(f_i) == 1) for f_i in park slot 0 (slots 0..4 as working space); slot 0 <- the final
// exponentiation (the GT value: the level-2 search of k_batch.hip compares these), as k_final_exp_check leaves it
extern "C" __global__ void __launch_bounds__(CP_BLOCK) k_coop_final_exp_check(u32 *park, u32 n, uint8_t *accept) {
    LCB_LATENCY_PRIO();
    __shared__ uint4 lds[CP_LDS_QUADS];
    cp_final_exp_check_run(lds, park, n, accept);
}

// The exact per-share check (k_tpke_miller's inputs) in the cooperative kernels' form, for small batches: share i
// becomes check i with points (U_i, -Y_i) on ciphertext c's two line sets.  accept[i] = the share's validity
// (index range, decompression, key, ciphertext), ANDed with the pairing result by k_coop_final_exp_check.
extern "C" __global__ void LCB_BOUNDS k_tpke_exact_points(const uint8_t *ct_ok, u32 n_cts, const g1a_st *keys,
                                                         u32 n_keys, const u32 *ct_idx, const u32 *dec_idx,
                                                         const uint8_t *ui, u32 n, g1a_st *gpts, uint4 *desc,
                                                         uint8_t *accept) {
    LCB_LATENCY_PRIO();
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u32 c = ct_idx[i], d = dec_idx[i];
    bool ok = d < n_keys && c < n_cts;
    c = c < n_cts ? c : 0;
    ok = ok && ct_ok[c];
    g1a U;
    ok = g1_decompress(U, ui + 48 * (size_t)i) && ok;
    g1a_st ks = keys[d < n_keys ? d : 0];
    ok = ok && ks.ok;
    g1a_st o;
    o.ok = 1; o.pad[0] = o.pad[1] = 0;
    o.inf = U.inf ? 1 : 0; o.x = U.x; o.y = U.y;
    gpts[2 * (size_t)i] = o;
    o.inf = ks.inf; o.x = ks.x; fp_neg(o.y, ks.y);
    gpts[2 * (size_t)i + 1] = o;
    desc[i] = make_uint4(i, 1, c, 0);
    accept[i] = ok;
}

// ---------------------------------------------------------------- test hook: one cooperative operation vs field.hpp
// op: 0 sqr12, 1 cyc_sqr, 2 mul12, 3 mul12 (conj a), 4..6 frob1..3, 7 inverse, 8 conj, 9 line (b, c = coefficients 0, 1
// of b), 10 final exponentiation.  a in park slot 0 of ws (6 slots), b in b_soa; out = cooperative result, ref = the
// one-lane field.hpp / pairing.hpp result (computed by lane 0 of each group)
extern "C" __global__ void __launch_bounds__(CP_BLOCK) k_coop_debug(int op, u32 *ws, const u32 *b_soa, u32 n, u32 *out,
                                                                   u32 *ref) {
    __shared__ uint4 lds[CP_LDS_QUADS];
    const Cp c = cp_init(lds);
    const u32 item = blockIdx.x * CP_G + c.g;
    const bool live = c.g < CP_G && item < n;
    const size_t it = live ? item : 0;
    if (cpj(c) == 0) cp_put(c, S_Z, fp2_zero());
    cp_sync();
    fp12 fa, fb, fr;
    if (cpj(c) == 0) {
        fp12_load_soa(fa, ws, n, it);
        fp12_load_soa(fb, b_soa, n, it);
    }
    fp2 R;
    park_get(R, ws, n, it, cpj(c));
    if (op == 0) { CpEval ev; ev.on = false; ev.yinf = true; ev.xp = ev.yp = ws; cp_sqr12(R, c, ev); }
    else if (op == 1) cp_cyc_sqr(R, c);
    else if (op == 2 || op == 3) cp_mul12(R, c, op == 3, b_soa, n, it);
    else if (op >= 4 && op <= 6) cp_frob(R, c, op - 3);
    else if (op == 7) cp_inv(R, c);
    else if (op == 8) cp_conj(R, c);
    else if (op == 9) {
        fp2 b, cc;
        park_get(b, b_soa, n, it, 0);
        park_get(cc, b_soa, n, it, 1);
        if (cpj(c) == 0) { cp_put(c, S_LE, b); cp_put(c, S_LE + 1, cc); }
        cp_sync();
        cp_line(R, c, S_LE, S_LE + 1);
    } else {
        cp_final_exp(R, c, ws, n, it, live);
    }
    park_put(out, n, it, cpj(c), live, R);
    if (live && cpj(c) == 0) {
        if (op == 0) fp12_sqr_n(fr, fa);
        else if (op == 1) fp12_cyc_sqr_n(fr, fa);
        else if (op == 2) fp12_mul_n(fr, fa, fb);
        else if (op == 3) { fp12_conj(fa, fa); fp12_mul_n(fr, fa, fb); }
        else if (op == 4) fp12_frob1_n(fr, fa);
        else if (op == 5) fp12_frob2_n(fr, fa);
        else if (op == 6) fp12_frob3_n(fr, fa);
        else if (op == 7) fp12_inv_n(fr, fa);
        else if (op == 8) fp12_conj(fr, fa);
        else if (op == 9) { fr = fa; fp12_mul_line_n(fr, fb.c0.c0, fb.c0.c1); }
        else final_exp(fr, fa);
        fp12_store_soa(ref, n, it, fr);
    }
}

// ---------------------------------------------------------------- host launch wrappers
// fallback = 0: the caller knows every line set the groups use is normalised (no group can be flagged), so the one-lane
// fallback kernel is not dispatched
extern "C" void lcbk_coop_tpke_miller(hipStream_t s, const u32 *lines, const void *desc, const void *gpts, u32 n_groups,
                                      u32 *f_soa, uint8_t *gacc, uint8_t *fb, u32 npairs, int fallback) {
    dim3 grid((n_groups + CP_G - 1) / CP_G);
    LCB_LAUNCH_GATED(k_coop_tpke_miller, grid, dim3(CP_BLOCK), 0, s, lines, (const uint4 *)desc, (const g1a_st *)gpts,
                       n_groups, f_soa, gacc, fb, npairs);
    if (!fallback) return;
    grid = dim3((n_groups + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_rlc_miller_fallback, lines, (const uint4 *)desc, (const g1a_st *)gpts, n_groups, f_soa, fb);
}
extern "C" void lcbk_coop_final_exp_check(hipStream_t s, u32 *park, u32 n, uint8_t *accept) {
    dim3 grid((n + CP_G - 1) / CP_G);
    LCB_LAUNCH_GATED(k_coop_final_exp_check, grid, dim3(CP_BLOCK), 0, s, park, n, accept);
}
extern "C" void lcbk_tpke_exact_points(hipStream_t s, const uint8_t *ct_ok, u32 n_cts, const void *keys, u32 n_keys,
                                       const u32 *ct_idx, const u32 *dec_idx, const uint8_t *ui, u32 n, void *gpts,
                                       void *desc, uint8_t *accept) {
    dim3 grid((n + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_tpke_exact_points, ct_ok, n_cts, (const g1a_st *)keys, n_keys, ct_idx, dec_idx, ui, n, (g1a_st *)gpts,
               (uint4 *)desc, accept);
}
extern "C" void lcbk_coop_debug(hipStream_t s, int op, u32 *ws, const u32 *b_soa, u32 n, u32 *out, u32 *ref) {
    dim3 grid((n + CP_G - 1) / CP_G);
    LCB_LAUNCH_GATED(k_coop_debug, grid, dim3(CP_BLOCK), 0, s, op, ws, b_soa, n, out, ref);
}
