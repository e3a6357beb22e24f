// lachain_amd/csrc/k_ptmul.hip — latency kernel of the mcl single-element scalar multiplications (mclBnG1_mul,
// mclBnG2_mul: TPKE/PublicKey.cs:25-37, TPKE/PrivateKey.cs:21-31, ThresholdSignature/PrivateKeyShare.cs:21-27 call them
// one element at a time).
//
// A one-lane ladder is ~2,500-3,500 serial Fp products at ~1.1 us each (the issue time of one wave), whatever else
// the GPU does.  Here one wave runs up to 16 LADDERS side by side, each on a GROUP of four lanes:
//   * every group runs the SAME program — a 4-bit window table T[1..15] of its base point, then for each window four
//     doublings and one addition of T[nibble] — on its own base point and digit string, so the wave never diverges
//     between groups (a skipped addition for a zero nibble is the only data-dependent branch);
//   * inside a group the four lanes share each point operation: every lane holds the group's values (X, Y, Z, the
//     temporaries) and a ROUND is one Fp (G1) or Fp2 (G2) product per lane on operands it selects by its role, then the
//     four products are exchanged through LDS.  dbl-2009-l takes 3 rounds instead of 7 serial products, add-2007-bl 5
//     instead of 16 (the formulas, special cases and results of curve.hpp's jac_dbl / jac_add exactly).
// The host splits the scalar (lcb_host.cpp): G1 by GLV (k P = k1 P + k2 phi(P), 129-bit halves) with a third group
// computing [z^2] P, the G1 membership test the split needs; G2 by GLS (four 64-bit digits over +-psi^i(Q)) with a
// fifth group computing [|z|] Q for psi(Q) == -[|z|] Q.  The host adds the groups' results and checks membership; a
// base point outside the subgroup takes the exact one-lane ladder instead (k_op), so every input gets k P exactly.
#include "kcommon.hpp"

LCB_ASM_LIBRARY(k_ptmul)
LCB_TU_CONFIG(k_ptmul)

#define PT_LANES 4                 // lanes per group
#define PT_MAX_GROUPS 8               // G1 uses 3, G2 5 (LDS: 9 areas, 22 / 45 KB)
#define PT_MAX_WIN 33              // 4-bit windows (129-bit GLV halves)

// one group's job: affine base point (inf = 1: the point at infinity) and nwin nibbles, most significant first
template <class F> struct PtJob {
    F x, y;
    u32 inf, nwin, pad[2];
    uint8_t nib[36];
};
template <class F> struct PtLds {
    F prod[PT_LANES];
    jac<F> tab[16];
};

DI int pt_role() {
    int r = (int)(threadIdx.x & (PT_LANES - 1));
    asm volatile("" : "+v"(r));
    return r;
}
template <class F> DI void f_sel(F &r, bool c, const F &a, const F &b) {
    u32 *rw = (u32 *)&r;
    const u32 *aw = (const u32 *)&a, *bw = (const u32 *)&b;
#pragma unroll
    for (int q = 0; q < (int)(sizeof(F) / 4); q++) rw[q] = c ? aw[q] : bw[q];
}
// operand of this lane's role among four candidates
template <class F> DI void f_sel4(F &r, int role, const F &a, const F &b, const F &c, const F &d) {
    f_sel(r, role == 0, a, d);
    f_sel(r, role == 1, b, r);
    f_sel(r, role == 2, c, r);
}
// one round: lane `role` computes x_role * y_role; returns with every lane holding the four products
template <class F> DI void pt_round(PtLds<F> *L, F (&p)[PT_LANES], const F &x0, const F &y0, const F &x1,
                                    const F &y1, const F &x2, const F &y2, const F &x3, const F &y3) {
    const int role = pt_role();
    F x, y, m;
    f_sel4(x, role, x0, x1, x2, x3);
    f_sel4(y, role, y0, y1, y2, y3);
    f_mul(m, x, y);
    L->prod[role] = m;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT_LANES; k++) p[k] = L->prod[k];
    __syncthreads();
}
template <class F> DI void f_dbl(F &r, const F &a) { f_add(r, a, a); }

// dbl-2009-l (curve.hpp jac_dbl): rounds {A = X^2, B = Y^2, YZ}, {C = B^2, (X + B)^2, F = E^2}, {E (D - X3)}
template <class F> DI void pt_dbl(PtLds<F> *L, jac<F> &r, const jac<F> &q) {
    F p[PT_LANES], A, B, C, D, E, Fv, t, x3, y3, z3;
    pt_round(L, p, q.x, q.x, q.y, q.y, q.y, q.z, q.x, q.x);
    A = p[0];
    B = p[1];
    z3 = p[2];
    f_add(t, q.x, B);
    f_add(E, A, A);
    f_add(E, E, A);
    pt_round(L, p, B, B, t, t, E, E, B, B);
    C = p[0];
    Fv = p[2];
    f_sub(D, p[1], A);
    f_sub(D, D, C);
    f_dbl(D, D);
    f_dbl(t, D);
    f_sub(x3, Fv, t);
    f_sub(t, D, x3);
    pt_round(L, p, E, t, E, t, E, t, E, t);
    f_dbl(t, C);
    f_dbl(t, t);
    f_dbl(t, t);
    f_sub(y3, p[0], t);
    f_dbl(z3, z3);
    r.x = x3;
    r.y = y3;
    r.z = z3;
}
// add-2007-bl with jac_add's special cases (either input at infinity, P == Q -> doubling, P == -Q -> infinity)
template <class F> DI void pt_add(PtLds<F> *L, jac<F> &r, const jac<F> &a, const jac<F> &b) {
    const bool ai = f_is_zero(a.z), bi = f_is_zero(b.z);
    F p[PT_LANES], z1z1, z2z2, u1, u2, s1, s2, h, i, rr, j, v, t, x3, y3, z3;
    pt_round(L, p, a.z, a.z, b.z, b.z, a.y, b.z, b.y, a.z);
    z1z1 = p[0];
    z2z2 = p[1];
    pt_round(L, p, a.x, z2z2, b.x, z1z1, p[2], z2z2, p[3], z1z1);
    u1 = p[0];
    u2 = p[1];
    s1 = p[2];
    s2 = p[3];
    f_sub(h, u2, u1);
    f_sub(rr, s2, s1);
    f_dbl(rr, rr);
    f_dbl(i, h);
    f_add(t, a.z, b.z);
    pt_round(L, p, i, i, rr, rr, t, t, i, i);
    i = p[0];
    F r2 = p[1], zz = p[2];
    f_sub(zz, zz, z1z1);
    f_sub(zz, zz, z2z2);
    pt_round(L, p, h, i, u1, i, zz, h, h, i);
    j = p[0];
    v = p[1];
    z3 = p[2];
    f_sub(x3, r2, j);
    f_sub(x3, x3, v);
    f_sub(x3, x3, v);
    f_sub(t, v, x3);
    pt_round(L, p, rr, t, s1, j, rr, t, rr, t);
    f_dbl(t, p[1]);
    f_sub(y3, p[0], t);
    jac<F> o;
    o.x = x3;
    o.y = y3;
    o.z = z3;
    const bool same_x = !ai && !bi && f_eq(u1, u2);  // uniform within the group (every lane holds u1, u2, s1, s2)
    const bool need_dbl = same_x && f_eq(s1, s2);
    if (__any(need_dbl)) {                           // wave-uniform branch: the rounds' LDS exchange stays convergent
        jac<F> d;
        pt_dbl(L, d, a);
        if (need_dbl) o = d;
    }
    if (same_x && !need_dbl) jac_set_inf(o);
    if (bi) o = a;
    if (ai) o = b;
    r = o;
}

// one wave, groups g = lane / 4 (< n_groups <= PT_MAX_GROUPS); out[g] = [digits] base_g (Jacobian, mcl layout).  Every
// group runs nwin windows (the host pads the digit strings to one length), so the loop is wave-uniform.
template <class F> DI void pt_ladder(const PtJob<F> *jobs, u32 n_groups, jac<F> *out, PtLds<F> *lds) {
    const u32 g = threadIdx.x / PT_LANES;
    const bool live = g < n_groups;
    const u32 gj = live ? g : 0;                 // idle lanes shadow group 0 (same control flow, no stores)
    PtLds<F> *L = lds + (live ? g : PT_MAX_GROUPS);
    const PtJob<F> &J = jobs[gj];
    jac<F> P, acc;
    if (J.inf) jac_set_inf(P);
    else { P.x = J.x; P.y = J.y; f_one(P.z); }
    // table T[1..15] = d P
    if (pt_role() == 0) L->tab[1] = P;
    jac<F> cur;
    pt_dbl(L, cur, P);
    if (pt_role() == 0) L->tab[2] = cur;
#pragma unroll 1
    for (int d = 3; d < 16; d++) {
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
        const u32 nib = J.nib[w];
        if (__any(nib != 0)) {                       // wave-uniform; a group with a zero nibble adds infinity
            jac<F> T = L->tab[nib ? nib : 1];
            if (!nib) jac_set_inf(T);
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
static_assert(sizeof(PtJob<fp>) == 96 + 16 + 36, "PtJob<fp> layout (launch.h LCB_PTJOB_G1_BYTES)");
static_assert(sizeof(PtJob<fp2>) == 192 + 16 + 36, "PtJob<fp2> layout (launch.h LCB_PTJOB_G2_BYTES)");

extern "C" void lcbk_ptmul_g1(hipStream_t s, const void *jobs, u32 n_groups, void *out) {
    hipLaunchKernelGGL(k_ptmul_g1, dim3(1), dim3(64), 0, s, (const PtJob<fp> *)jobs, n_groups, (g1 *)out);
}
extern "C" void lcbk_ptmul_g2(hipStream_t s, const void *jobs, u32 n_groups, void *out) {
    hipLaunchKernelGGL(k_ptmul_g2, dim3(1), dim3(64), 0, s, (const PtJob<fp2> *)jobs, n_groups, (g2 *)out);
}
