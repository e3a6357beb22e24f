// lachain_amd/csrc/k_ptmul.hip — latency kernel of the mcl single-element scalar multiplications (mclBnG1_mul,
// mclBnG2_mul: TPKE/PublicKey.cs:25-37, TPKE/PrivateKey.cs:21-31, ThresholdSignature/PrivateKeyShare.cs:21-27 call them
// one element at a time).
//
// A one-lane ladder is ~2,500-3,500 serial Fp products at ~1.1 us each (the issue time of one wave), whatever else
// the GPU does.  Here one wave runs up to 16 LADDERS side by side, each on a GROUP of four lanes:
//   * every group runs the SAME program — a signed 4-bit window table T[1..8] of its base point, then for each window
//     four doublings and one addition of +-T[|digit|] (digits in [-7, 8]: 6 table additions instead of 13) — on its
//     own base point and digit string, so the wave never diverges between groups (a skipped addition for a zero
//     digit is the only data-dependent branch);
//   * inside a group the four lanes share each point operation: every lane holds the group's values (X, Y, Z, the
//     temporaries) and a ROUND is one Fp (G1) or Fp2 (G2) product per lane on operands it selects by its role, then the
//     four products are exchanged through LDS.  dbl-2009-l takes 3 rounds instead of 7 serial products, add-2007-bl 5
//     instead of 16 (the formulas, special cases and results of curve.hpp's jac_dbl / jac_add exactly).
// The host splits the scalar (lcb_host.cpp): G1 by GLV (k P = k1 P + k2 phi(P), 129-bit halves), each half cut at
// bit 65 over P and [2^65] P (four groups of 18 windows); G2 by GLS (four 64-bit digits over +-psi^i(Q)), each digit
// cut at bit 32 over +-psi^i(Q) and +-psi^i([2^32] Q) (eight groups of 9 windows).  The host computes the [2^65] /
// [2^32] multiples and the membership test the split needs ([z^2] P == (beta^2 x, -y), psi(Q) == -[|z|] Q) with its
// own field code, and adds the groups' results; a base point outside the subgroup takes the exact one-lane ladder
// instead (k_op), so every input gets k P exactly.  The multi-term calls (mulVec, Lagrange, EvaluatePolynomial) keep
// the ladders' own membership group (three / five groups per term, k_ptmul_g1_multi / _g2_multi).
#include "coop_pt.hpp"

LCB_ASM_LIBRARY(k_ptmul)
LCB_TU_CONFIG(k_ptmul)

#define PT_MAX_GROUPS 8               // G1 uses 4, G2 8 (LDS: 9 areas, 22 / 45 KB)
#define PT_MAX_WIN 33              // signed 4-bit windows (129-bit GLV halves; 17 for the 64-bit GLS digits)

// one group's job: affine base point (inf = 1: the point at infinity) and nwin signed digits, most significant
// first, one byte each: |digit| (<= 8) in bits 0-3, bit 7 set for a negative digit (lcb_host.cpp put_digits)
template <class F> struct PtJob {
    F x, y;
    u32 inf, nwin, pad[2];
    uint8_t nib[36];
};
// one wave, groups g = lane / 4 (< n_groups <= PT_MAX_GROUPS); out[g] = [digits] base_g (Jacobian, mcl layout).  Every
// group runs nwin windows (the host pads the digit strings to one length), so the loop is wave-uniform.
template <class F, int MAXG = PT_MAX_GROUPS> DI void pt_ladder(const PtJob<F> *jobs, u32 n_groups, jac<F> *out,
                                                           PtLds<F> *lds) {
    const u32 g = threadIdx.x / PT_LANES;
    const bool live = g < n_groups;
    const u32 gj = live ? g : 0;                 // idle lanes shadow group 0 (same control flow, no stores)
    PtLds<F> *L = lds + (live ? g : MAXG);
    const PtJob<F> &J = jobs[gj];
    jac<F> P, acc;
    if (J.inf) jac_set_inf(P);
    else { P.x = J.x; P.y = J.y; f_one(P.z); }
    // table T[1..8] = d P; a negative digit adds -T[|d|] = (X, -Y, Z)
    if (pt_role() == 0) L->tab[1] = P;
    jac<F> cur;
    pt_dbl(L, cur, P);
    if (pt_role() == 0) L->tab[2] = cur;
#pragma unroll 1
    for (int d = 3; d <= PT_TAB_MAX; d++) {
        pt_add(L, cur, cur, P);
        if (pt_role() == 0) L->tab[d] = cur;
    }
    __syncthreads();
    jac_set_inf(acc);
    const u32 nwin = jobs[0].nwin;               // one window count for every group: a wave-uniform loop
#pragma unroll 1
    for (u32 w = 0; w < nwin; w++) {
        if (w) {
            pt_dbl(L, acc, acc);
            pt_dbl(L, acc, acc);
            pt_dbl(L, acc, acc);
            pt_dbl(L, acc, acc);
        }
        const u32 dig = J.nib[w], mag = dig & 15u;
        if (__any(mag != 0)) {                       // wave-uniform; a group with a zero digit adds infinity
            jac<F> T = L->tab[(mag && mag <= PT_TAB_MAX) ? mag : 1];
            if (dig & 0x80u) f_neg(T.y, T.y);
            if (!mag) jac_set_inf(T);
            pt_add(L, acc, acc, T);
        }
    }
    if (live && pt_role() == 0) out[g] = acc;
}

extern "C" __global__ void __launch_bounds__(64, 1) k_ptmul_g1(const PtJob<fp> *jobs, u32 n_groups, g1 *out) {
    __shared__ PtLds<fp> lds[PT_MAX_GROUPS + 1];
    pt_ladder(jobs, n_groups, out, lds);
}
extern "C" __global__ void __launch_bounds__(64, 1) k_ptmul_g2(const PtJob<fp2> *jobs, u32 n_groups, g2 *out) {
    __shared__ PtLds<fp2> lds[PT_MAX_GROUPS + 1];
    pt_ladder(jobs, n_groups, out, lds);
}
// many G1 ladders at once (mclBnG1_mulVec, mclBn_G1LagrangeInterpolation: three groups per term, lcb_host.cpp
// g1_mulvec_coop): block b runs groups [16 b, 16 b + 16), every group of a wave with its own LDS area
#define PT_MULTI_GROUPS 16
extern "C" __global__ void __launch_bounds__(64, 1) k_ptmul_g1_multi(const PtJob<fp> *jobs, u32 n_groups, g1 *out) {
    __shared__ PtLds<fp> lds[PT_MULTI_GROUPS + 1];
    const u32 base = blockIdx.x * PT_MULTI_GROUPS;
    if (base >= n_groups) return;                // uniform
    const u32 n = min(n_groups - base, (u32)PT_MULTI_GROUPS);
    pt_ladder<fp, PT_MULTI_GROUPS>(jobs + base, n, out + base, lds);
}
// the same for G2 (five groups per term: the four GLS digits' ladders and [|z|] Q for the membership test)
extern "C" __global__ void __launch_bounds__(64, 1) k_ptmul_g2_multi(const PtJob<fp2> *jobs, u32 n_groups, g2 *out) {
    __shared__ PtLds<fp2> lds[PT_MULTI_GROUPS + 1];
    const u32 base = blockIdx.x * PT_MULTI_GROUPS;
    if (base >= n_groups) return;                // uniform
    const u32 n = min(n_groups - base, (u32)PT_MULTI_GROUPS);
    pt_ladder<fp2, PT_MULTI_GROUPS>(jobs + base, n, out + base, lds);
}
static_assert(sizeof(PtJob<fp>) == 96 + 16 + 36, "PtJob<fp> layout (launch.h LCB_PTJOB_G1_BYTES)");
static_assert(sizeof(PtJob<fp2>) == 192 + 16 + 36, "PtJob<fp2> layout (launch.h LCB_PTJOB_G2_BYTES)");

// mclBnG2_hashAndMapTo (G2.SetHashOf: TPKE/Utils.cs:21-27, ThresholdSignature/PrivateKeyShare.cs:23-25) on one lane
// in a kernel of its own: k_op's single-operation switch carries every operation's state (3,038 spilled registers).
// io as k_op's OP_G2_HASH: io[250] = message length, the message at io + 256; out: the Jacobian point at io[0..72),
// io[248] = 1 on success (0: no point, infinity written)
// The map (SHA-512, calcBN) runs on lane 0; the Budroni-Pintore cofactor clearing's two 64-bit ladders and its
// additions run on groups of four lanes (coop_pt.hpp: a G2 doubling in 3 Fp2-product rounds instead of 7 serial
// products) — the same point as h2g2.hpp g2_clear_cofactor_bp (its Jacobian coordinates may differ: general instead
// of mixed additions).  The original-cofactor mode (one 508-bit ladder, a tuning option) stays on lane 0.
#ifndef LCB_MCL_HASH_COOP
#define LCB_MCL_HASH_COOP 1
#endif
template <class LT> DI void pt_mul_u64(LT *L, g2 &r, const g2 &p, u64 k) {   // k uniform: a wave-uniform ladder
    const int top = 63 - __clzll(k);
    g2 acc = p;
#pragma unroll 1
    for (int i = top - 1; i >= 0; i--) {
        pt_dbl(L, acc, acc);
        if ((k >> i) & 1) pt_add(L, acc, acc, p);
    }
    r = acc;
}
template <class LT> DI void pt_clear_cofactor_bp(LT *L, g2 &Q, const g2 &P) {   // h2g2.hpp g2_clear_cofactor_bp
    // with A = (z - 1) P = -[|z| + 1] P: Q = -[|z|] A + (psi^2(2P) - P) + psi(A); three points live at a time
    g2 V, A, W;
    pt_dbl(L, V, P);
    g2_psi2(V, V);
    jac_neg(W, P);
    pt_add(L, V, V, W);                          // psi^2(2P) - P
    pt_mul_u64(L, A, P, LCB_Z_ABS + 1);
    jac_neg(A, A);                               // A = (z - 1) P
    g2_psi(W, A);
    pt_add(L, V, V, W);                          // psi^2(2P) - P + psi(A)
    pt_mul_u64(L, W, A, LCB_Z_ABS);
    jac_neg(W, W);                               // z A
    pt_add(L, Q, W, V);
}
extern "C" __global__ void __launch_bounds__(64, 1) k_mcl_g2_hash(u32 *io, int orig_cof) {
    if (threadIdx.x) return;
    uint8_t d[64];
    sha512_2(d, (const uint8_t *)(io + 256), io[250], (const uint8_t *)(io + 256), 0);
#if LCB_MCL_HASH_COOP
    fp2 t;                                       // the map only; k_mcl_g2_clear clears the cofactor (io[249] = 1)
    fp_set_hash_digest(t.a, d);
    t.b = fp_zero();
    g2 P;
    const bool ok = g2_calc_bn(P, t);
    if (ok && orig_cof) { g2 H; g2_clear_cofactor_h2(H, P); P = H; }
    if (!ok) jac_set_inf(P);
    *(g2 *)io = P;
    io[248] = ok ? 1u : 0u;
    io[249] = ok && !orig_cof ? 1u : 0u;
#else
    g2 H;
    const bool ok = g2_hash_digest(H, d, orig_cof != 0);
    if (!ok) jac_set_inf(H);
    *(g2 *)io = H;
    io[248] = ok ? 1u : 0u;
#endif
}
// io[0..72) = the clearing of the mapped point io[0..72) when io[249] is set (every lane group computes it; lane 0
// stores)
extern "C" __global__ void __launch_bounds__(64, 1) k_mcl_g2_clear(u32 *io) {
    __shared__ PtProd<fp2> lds[64 / PT_LANES];
    if (io[249] == 0u) return;                   // uniform
    const g2 P = *(const g2 *)io;
    g2 H;
    pt_clear_cofactor_bp(lds + threadIdx.x / PT_LANES, H, P);
    __syncthreads();
    if (threadIdx.x == 0) *(g2 *)io = H;
}
extern "C" void lcbk_mcl_g2_hash(hipStream_t s, u32 *io, int orig_cof) {
    LCB_LAUNCH_GATED(k_mcl_g2_hash, dim3(1), dim3(64), 0, s, io, orig_cof);
#if LCB_MCL_HASH_COOP
    LCB_LAUNCH_GATED(k_mcl_g2_clear, dim3(1), dim3(64), 0, s, io);
#endif
}
extern "C" void lcbk_ptmul_g1(hipStream_t s, const void *jobs, u32 n_groups, void *out) {
    LCB_LAUNCH_GATED(k_ptmul_g1, dim3(1), dim3(64), 0, s, (const PtJob<fp> *)jobs, n_groups, (g1 *)out);
}
extern "C" void lcbk_ptmul_g1_multi(hipStream_t s, const void *jobs, u32 n_groups, void *out) {
    const dim3 grid((n_groups + PT_MULTI_GROUPS - 1) / PT_MULTI_GROUPS);
    LCB_LAUNCH_GATED(k_ptmul_g1_multi, grid, dim3(64), 0, s, (const PtJob<fp> *)jobs, n_groups, (g1 *)out);
}
extern "C" void lcbk_ptmul_g2_multi(hipStream_t s, const void *jobs, u32 n_groups, void *out) {
    const dim3 grid((n_groups + PT_MULTI_GROUPS - 1) / PT_MULTI_GROUPS);
    LCB_LAUNCH_GATED(k_ptmul_g2_multi, grid, dim3(64), 0, s, (const PtJob<fp2> *)jobs, n_groups, (g2 *)out);
}
extern "C" void lcbk_ptmul_g2(hipStream_t s, const void *jobs, u32 n_groups, void *out) {
    LCB_LAUNCH_GATED(k_ptmul_g2, dim3(1), dim3(64), 0, s, (const PtJob<fp2> *)jobs, n_groups, (g2 *)out);
}
