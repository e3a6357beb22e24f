// lachain_amd/csrc/coop_pt.hpp — point operations shared by a group of four lanes (k_ptmul.hip, k_msm.hip's window
// combination): every lane of the group holds the group's values, a ROUND is one Fp (G1) or Fp2 (G2) product per lane
// on operands it selects by its role, and the four products are exchanged through the group's LDS area.
// dbl-2009-l takes 3 rounds instead of 7 serial products, add-2007-bl 5 instead of 16, with curve.hpp's formulas and
// special cases (the results are the same Jacobian coordinates as jac_dbl / jac_add).  The rounds synchronise the
// workgroup: callers keep the control flow around them wave-uniform (one wave per workgroup).
#pragma once
#include "kcommon.hpp"

#define PT_LANES 4                 // lanes per group
#define PT_TAB_MAX 8               // k_ptmul.hip's signed-digit table T[1..8]

template <class F> struct PtLds {
    F prod[PT_LANES];
    jac<F> tab[PT_TAB_MAX + 1];
};
template <class F> struct PtProd {   // a group's product exchange alone (k_msm.hip's block reductions: 64 groups)
    F prod[PT_LANES];
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
template <class LT, class F> DI void pt_round(LT *L, F (&p)[PT_LANES], const F &x0, const F &y0, const F &x1,
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
template <class LT, class F> DI void pt_dbl(LT *L, jac<F> &r, const jac<F> &q) {
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
// add-2007-bl with jac_add's special cases (either input at infinity, P == Q -> doubling, P == -Q -> infinity).
// BLK: several waves share the workgroup's barriers, so the doubling branch is taken block-wide (__syncthreads_or)
template <bool BLK = false, class LT, class F> DI void pt_add(LT *L, jac<F> &r, const jac<F> &a, const jac<F> &b) {
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
    if (BLK ? __syncthreads_or(need_dbl) : __any(need_dbl)) {   // uniform branch: the rounds' exchange stays convergent
        jac<F> d;
        pt_dbl(L, d, a);
        if (need_dbl) o = d;
    }
    if (same_x && !need_dbl) jac_set_inf(o);
    if (bi) o = a;
    if (ai) o = b;
    r = o;
}

