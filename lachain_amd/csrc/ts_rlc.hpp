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
