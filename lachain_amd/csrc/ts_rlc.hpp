// lachain_amd/csrc/ts_rlc.hpp — the CommonCoin group checks of the randomized batch verification (k_batch.hip
// header): the group sums and the two-pair Miller loop, shared by k_batch.hip (every level) and k_prep.hip (the
// census copies at 256 registers, which run beside the randomisation instead of after it).
#pragma once
#include "rlc_common.hpp"

// ---------------------------------------------------------------- threshold signatures (ValidateSignature)
// e(PK_i, H(m)) == e(G, sig_i) <=> e(PK_i, H) e(-G, sig_i) == 1.  The randomisation of sig_i uses linearity of the
// pairing in its G2 argument, which holds on G2: a share whose sig_i is outside G2 (G2.FromBytes does not check) is
// emitted straight away as an exact single (desc.w = 1) and contributes nothing to its group.
// TS group record: g1a_st P (sum s_i PK_i) then g2a_st S (sum s_i sig_i), 320 B
struct ts_grp { g1a_st p; g2a_st s; };
DI void ts_rlc_sum_run(const uint4 *desc, u32 n_groups, u32 first, const uint8_t *msg_ok, const g1a_st *pks, u32 n_pks,
                       const u32 *pk_idx, const uint8_t *sigs, const u32 *rP, const u32 *rS, u32 n, ts_grp *gpts,
                       uint8_t *accept, uint8_t *gexact, u32 *wsum, const u32 *susp, uint8_t *cval) {
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
    g1_to_st_gcd(o.p, sp, false);
    g2_to_st_gcd(o.s, ss);
    gpts[g] = o;
}
// The same sums with TWO lanes per group (k_prep.hip k_ts_rlc_sum2, 256 registers: the 2,048 waves of configs[2]'s
// level 1 run two per SIMD where one lane per group left one 294-register wave per SIMD issue-starved).  Lane h sums
// shares [a_h, b_h) (a_0 = 0, a_1 = L = ceil(len / 2)) into sp_h, ss_h and the locally weighted wp_h = sum (j - a_h + 1)
// P_j; lane 1 adds L sp_1 (so its weights become the global j + 1), the pair exchanges its four partial sums by
// shuffles and both lanes add them; lane 0 converts and stores the G1 side, lane 1 the G2 side.  The group law makes
// the affine records the same field elements as the one-lane sums' (the Jacobian wsum rows are converted before use).
template <class J> DI void jac_shfl_pair(J &r, const J &x) {      // r = partner lane's x (lanes 2g, 2g + 1)
    u32 *rw = (u32 *)&r;
    const u32 *xw = (const u32 *)&x;
#pragma unroll
    for (int q = 0; q < (int)(sizeof(J) / 4); q++) rw[q] = (u32)__shfl_xor((int)xw[q], 1);
}
DI void ts_rlc_sum2_run(const uint4 *desc, u32 n_groups, u32 first, const uint8_t *msg_ok, const g1a_st *pks,
                        u32 n_pks, const u32 *pk_idx, const uint8_t *sigs, const u32 *rP, const u32 *rS, u32 n,
                        ts_grp *gpts, uint8_t *accept, uint8_t *gexact, u32 *wsum, const u32 *susp, uint8_t *cval) {
    const u32 t = blockIdx.x * blockDim.x + threadIdx.x, g = t >> 1, h = t & 1;
    if (g >= n_groups) return;                         // (both lanes of a pair)
    const uint4 dsc = desc[g];
    if (dsc.w == 1 || !msg_ok[dsc.z]) {                // an exact single / an undecodable message: lane 0 alone
        if (h) return;
        ts_grp o;
        g1_inf_st(o.p);
        g2_inf_st(o.s);
        gexact[g] = 0;
        if (dsc.w == 1) {
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
        } else {
            for (u32 j = 0; j < dsc.y; j++) accept[dsc.x + j] = 0;
        }
        gpts[g] = o;
        return;
    }
    const u32 L = (dsc.y + 1) >> 1, a = h ? L : 0, b = h ? dsc.y : L;
    g1 sp, t1, wp;
    g2 ss, u, ws;
    jac_set_inf(sp);
    jac_set_inf(wp);
    jac_set_inf(ss);
    jac_set_inf(ws);
    for (u32 j = b; j-- > a;) {
        if (!key_suspect(susp, pk_idx[dsc.x + j], n_pks)) {
            g1_load_soa(t1, rP, n, dsc.x + j);
            grp_add(sp, sp, t1);
            g2_load_soa(u, rS, n, dsc.x + j);
            grp_add(ss, ss, u);
        }
        if (first) {
            grp_add(wp, wp, sp);
            grp_add(ws, ws, ss);
        }
    }
    if (first && h) {                                  // weights j - L + 1 -> j + 1
        jac_mul_u64(t1, sp, L);
        grp_add(wp, wp, t1);
        jac_mul_u64(u, ss, L);
        grp_add(ws, ws, u);
    }
    jac_shfl_pair(t1, sp);
    grp_add(sp, sp, t1);
    jac_shfl_pair(u, ss);
    grp_add(ss, ss, u);
    if (first) {
        jac_shfl_pair(t1, wp);
        jac_shfl_pair(u, ws);
        if (h) {
            grp_add(ws, ws, u);
            g2_store_soa(wsum + (size_t)36 * n_groups, n_groups, g, ws);
        } else {
            grp_add(wp, wp, t1);
            g1_store_soa(wsum, n_groups, g, wp);
        }
    }
    if (h) {
        g2_to_st_gcd(gpts[g].s, ss);
    } else {
        gexact[g] = 0;
        g1_to_st_gcd(gpts[g].p, sp, false);
    }
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
DI void ts_rlc_miller_run(const u32 *lines, const uint4 *desc, const ts_grp *gpts, u32 n_groups, u32 *f_soa,
                          uint8_t *gacc) {
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
