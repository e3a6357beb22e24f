// lachain_amd/csrc/curve.hpp — G1 (E: y^2 = x^3 + 4 over Fp) and G2 (E': y^2 = x^3 + 4(1+i) over Fp2,
// M-type twist) in Jacobian coordinates, MCL-format (de)serialization, the psi endomorphism and
// scalar multiplication.  One point per lane.
//
// Wire formats (pinned by test/Lachain.CryptoTest/SerializationTest.cs:31-57):
//   G1 48 B = x (LE) with bit 7 of byte 47 = parity(y); G2 96 B = x.a (LE) || x.b (LE), bit 7 of byte 95
//   = parity(y.a) (mcl Fp2::isOdd looks at the `a` coordinate); all-zero = point at infinity.
// Deserialization is mcl's default (lax): reject x >= p and points not on the curve, no subgroup check
// (evidence: test/Lachain.ConsensusTest/HoneyBadgerSmartMalicious.cs:57-73).
#pragma once
#include "field.hpp"

// ---------------------------------------------------------------- overload set used by the templates
DI void f_add(fp &r, const fp &a, const fp &b) { fp_add(r, a, b); }
DI void f_sub(fp &r, const fp &a, const fp &b) { fp_sub(r, a, b); }
DI void f_mul(fp &r, const fp &a, const fp &b) { fp_mul(r, a, b); }
DI void f_sqr(fp &r, const fp &a) { fp_sqr(r, a); }
DI void f_neg(fp &r, const fp &a) { fp_neg(r, a); }
DI void f_inv(fp &r, const fp &a) { fp_inv(r, a); }
DI bool f_is_zero(const fp &a) { return fp_is_zero(a); }
DI bool f_eq(const fp &a, const fp &b) { return fp_eq(a, b); }
DI void f_one(fp &r) { r = fp_one(); }
DI void f_zero(fp &r) { r = fp_zero(); }
DI void f_add(fp2 &r, const fp2 &a, const fp2 &b) { fp2_add(r, a, b); }
DI void f_sub(fp2 &r, const fp2 &a, const fp2 &b) { fp2_sub(r, a, b); }
DI void f_mul(fp2 &r, const fp2 &a, const fp2 &b) { fp2_mul(r, a, b); }
DI void f_sqr(fp2 &r, const fp2 &a) { fp2_sqr(r, a); }
DI void f_neg(fp2 &r, const fp2 &a) { fp2_neg(r, a); }
DI void f_inv(fp2 &r, const fp2 &a) { fp2_inv_n(r, a); }
DI bool f_is_zero(const fp2 &a) { return fp2_is_zero(a); }
DI bool f_eq(const fp2 &a, const fp2 &b) { return fp2_eq(a, b); }
DI void f_one(fp2 &r) { r = fp2_one(); }
DI void f_zero(fp2 &r) { r = fp2_zero(); }

template <class F> struct jac { F x, y, z; };
typedef jac<fp> g1;
typedef jac<fp2> g2;
template <class F> struct aff { F x, y; bool inf; };
typedef aff<fp> g1a;
typedef aff<fp2> g2a;

template <class F> DI bool jac_is_inf(const jac<F> &p) { return f_is_zero(p.z); }
template <class F> DI void jac_set_inf(jac<F> &p) { f_one(p.x); f_one(p.y); f_zero(p.z); }
template <class F> DI void jac_from_aff(jac<F> &r, const aff<F> &a) {
    if (a.inf) { jac_set_inf(r); return; }
    r.x = a.x; r.y = a.y; f_one(r.z);
}
// Round 6 (LCB_LEAN_FORMULAS, default): the same formulas with their operations ordered so that fewer values are live
// at once — Z3 first (Y, Z dead after B), (Z1 + H)^2 right after HH (Z1, Z1Z1 dead) — for the kernels at a register
// cap (the two-waves-per-SIMD randomisation lanes, the G2 ladders): dbl 7 -> 5 live values, madd 9 -> 7.
#ifndef LCB_LEAN_FORMULAS
#define LCB_LEAN_FORMULAS 1
#endif
#if LCB_LEAN_FORMULAS
// dbl-2009-l (a = 0)
template <class F> DI void jac_dbl(jac<F> &r, const jac<F> &p) {
    F A, B, C, D, E, t, z3;
    f_mul(z3, p.y, p.z);
    f_add(z3, z3, z3);                  // Z3 = 2 Y Z
    f_sqr(B, p.y);                      // B = Y^2           (Y, Z dead)
    f_add(D, p.x, B);
    f_sqr(D, D);                        // (X + B)^2
    f_sqr(A, p.x);                      // A = X^2           (X dead)
    f_sqr(C, B);                        // C = B^2           (B dead)
    f_sub(D, D, A);
    f_sub(D, D, C);
    f_add(D, D, D);                     // D = 2((X + B)^2 - A - C)
    f_add(E, A, A);
    f_add(E, E, A);                     // E = 3A            (A dead)
    f_sqr(A, E);                        // F = E^2
    f_add(t, D, D);
    f_sub(r.x, A, t);                   // X3 = F - 2D
    f_sub(t, D, r.x);
    f_mul(r.y, E, t);
    f_add(t, C, C);
    f_add(t, t, t);
    f_add(t, t, t);
    f_sub(r.y, r.y, t);                 // Y3 = E (D - X3) - 8C
    r.z = z3;
}
#else
// dbl-2009-l (a = 0)
template <class F> DI void jac_dbl(jac<F> &r, const jac<F> &p) {
    F A, B, C, D, E, Fv, t, x3, y3, z3;
    f_sqr(A, p.x);
    f_sqr(B, p.y);
    f_sqr(C, B);
    f_add(D, p.x, B);
    f_sqr(D, D);
    f_sub(D, D, A);
    f_sub(D, D, C);
    f_add(D, D, D);
    f_add(E, A, A);
    f_add(E, E, A);
    f_sqr(Fv, E);
    f_add(t, D, D);
    f_sub(x3, Fv, t);
    f_sub(t, D, x3);
    f_mul(y3, E, t);
    f_add(t, C, C);
    f_add(t, t, t);
    f_add(t, t, t);
    f_sub(y3, y3, t);
    f_mul(z3, p.y, p.z);
    f_add(z3, z3, z3);
    r.x = x3; r.y = y3; r.z = z3;
}
#endif
// add-2007-bl, complete for the doubling / inverse / infinity special cases
template <class F> DI void jac_add(jac<F> &r, const jac<F> &p, const jac<F> &q) {
    if (jac_is_inf(p)) { r = q; return; }
    if (jac_is_inf(q)) { r = p; return; }
    F z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t, x3, y3, z3;
    f_sqr(z1z1, p.z);
    f_sqr(z2z2, q.z);
    f_mul(u1, p.x, z2z2);
    f_mul(u2, q.x, z1z1);
    f_mul(s1, p.y, q.z);
    f_mul(s1, s1, z2z2);
    f_mul(s2, q.y, p.z);
    f_mul(s2, s2, z1z1);
    if (f_eq(u1, u2)) {
        if (f_eq(s1, s2)) { jac_dbl(r, p); return; }
        jac_set_inf(r);
        return;
    }
    f_sub(h, u2, u1);
    f_add(i, h, h);
    f_sqr(i, i);
    f_mul(j, h, i);
    f_sub(rr, s2, s1);
    f_add(rr, rr, rr);
    f_mul(v, u1, i);
    f_sqr(x3, rr);
    f_sub(x3, x3, j);
    f_sub(x3, x3, v);
    f_sub(x3, x3, v);
    f_sub(t, v, x3);
    f_mul(y3, rr, t);
    f_mul(t, s1, j);
    f_add(t, t, t);
    f_sub(y3, y3, t);
    f_add(z3, p.z, q.z);
    f_sqr(z3, z3);
    f_sub(z3, z3, z1z1);
    f_sub(z3, z3, z2z2);
    f_mul(z3, z3, h);
    r.x = x3; r.y = y3; r.z = z3;
}
// madd-2007-bl: p + q with q affine (q finite)
#if LCB_LEAN_FORMULAS
template <class F> DI void jac_add_aff(jac<F> &r, const jac<F> &p, const F &qx, const F &qy) {
    if (jac_is_inf(p)) { r.x = qx; r.y = qy; f_one(r.z); return; }
    F z1z1, u2, s2, h, hh, rr, z3;
    f_sqr(z1z1, p.z);
    f_mul(u2, qx, z1z1);
    f_mul(s2, qy, p.z);
    f_mul(s2, s2, z1z1);
    if (f_eq(u2, p.x)) {
        if (f_eq(s2, p.y)) { jac_dbl(r, p); return; }
        jac_set_inf(r);
        return;
    }
    f_sub(h, u2, p.x);                  // H = U2 - X1
    f_sub(rr, s2, p.y);
    f_add(rr, rr, rr);                  // r = 2 (S2 - Y1)
    f_sqr(hh, h);                       // HH = H^2
    f_add(z3, p.z, h);
    f_sqr(z3, z3);
    f_sub(z3, z3, z1z1);
    f_sub(z3, z3, hh);                  // Z3 = (Z1 + H)^2 - Z1Z1 - HH   (Z1, Z1Z1 dead)
    f_add(hh, hh, hh);
    f_add(hh, hh, hh);                  // I = 4 HH
    f_mul(u2, h, hh);                   // J = H I                      (H dead)
    f_mul(s2, p.x, hh);                 // V = X1 I                     (X1, I dead)
    f_mul(h, p.y, u2);                  // Y1 J                         (Y1 dead)
    f_sqr(hh, rr);
    f_sub(hh, hh, u2);
    f_sub(hh, hh, s2);
    f_sub(r.x, hh, s2);                 // X3 = r^2 - J - 2V
    f_sub(hh, s2, r.x);
    f_mul(r.y, rr, hh);
    f_add(h, h, h);
    f_sub(r.y, r.y, h);                 // Y3 = r (V - X3) - 2 Y1 J
    r.z = z3;
}
#else
template <class F> DI void jac_add_aff(jac<F> &r, const jac<F> &p, const F &qx, const F &qy) {
    if (jac_is_inf(p)) { r.x = qx; r.y = qy; f_one(r.z); return; }
    F z1z1, u2, s2, h, hh, i, j, rr, v, t, x3, y3, z3;
    f_sqr(z1z1, p.z);
    f_mul(u2, qx, z1z1);
    f_mul(s2, qy, p.z);
    f_mul(s2, s2, z1z1);
    if (f_eq(u2, p.x)) {
        if (f_eq(s2, p.y)) { jac_dbl(r, p); return; }
        jac_set_inf(r);
        return;
    }
    f_sub(h, u2, p.x);
    f_sqr(hh, h);
    f_add(i, hh, hh);
    f_add(i, i, i);
    f_mul(j, h, i);
    f_sub(rr, s2, p.y);
    f_add(rr, rr, rr);
    f_mul(v, p.x, i);
    f_sqr(x3, rr);
    f_sub(x3, x3, j);
    f_sub(x3, x3, v);
    f_sub(x3, x3, v);
    f_sub(t, v, x3);
    f_mul(y3, rr, t);
    f_mul(t, p.y, j);
    f_add(t, t, t);
    f_sub(y3, y3, t);
    f_add(z3, p.z, h);
    f_sqr(z3, z3);
    f_sub(z3, z3, z1z1);
    f_sub(z3, z3, hh);
    r.x = x3; r.y = y3; r.z = z3;
}
#endif
template <class F> DI void jac_neg(jac<F> &r, const jac<F> &p) { r.x = p.x; f_neg(r.y, p.y); r.z = p.z; }
template <class F> DI void jac_to_aff(aff<F> &a, const jac<F> &p) {
    if (jac_is_inf(p)) { a.inf = true; f_zero(a.x); f_zero(a.y); return; }
    F zi, zi2;
    f_inv(zi, p.z);
    f_sqr(zi2, zi);
    f_mul(a.x, p.x, zi2);
    f_mul(zi2, zi2, zi);
    f_mul(a.y, p.y, zi2);
    a.inf = false;
}
// the same for G2 with the binary-GCD Fp inversion (field.hpp fp2_inv_gn: ~40 K instructions against the
// exponentiation's 263 K; the same canonical result), for the one-lane hash lanes where the call is cheap
DI void g2_jac_to_aff_g(g2a &a, const g2 &p) {
    if (jac_is_inf(p)) { a.inf = true; f_zero(a.x); f_zero(a.y); return; }
    fp2 zi, zi2;
    fp2_inv_gn(zi, p.z);
    f_sqr(zi2, zi);
    f_mul(a.x, p.x, zi2);
    f_mul(zi2, zi2, zi);
    f_mul(a.y, p.y, zi2);
    a.inf = false;
}
// G1 with the binary-GCD inversion (fp_inv_gcd), for the serialisations below
DI void g1_jac_to_aff_g(g1a &a, const g1 &p) {
    if (jac_is_inf(p)) { a.inf = true; f_zero(a.x); f_zero(a.y); return; }
    fp zi, zi2;
    fp_inv_gcd(zi, p.z);
    f_sqr(zi2, zi);
    f_mul(a.x, p.x, zi2);
    f_mul(zi2, zi2, zi);
    f_mul(a.y, p.y, zi2);
    a.inf = false;
}
DN void g1_dbl_n(g1 &r, const g1 &p) { g1 t; jac_dbl(t, p); r = t; }
DN void g1_add_n(g1 &r, const g1 &p, const g1 &q) { g1 t; jac_add(t, p, q); r = t; }
DN void g2_dbl_n(g2 &r, const g2 &p) { g2 t; jac_dbl(t, p); r = t; }
DN void g2_add_n(g2 &r, const g2 &p, const g2 &q) { g2 t; jac_add(t, p, q); r = t; }
DI void grp_dbl(g1 &r, const g1 &p) { g1_dbl_n(r, p); }
DI void grp_add(g1 &r, const g1 &p, const g1 &q) { g1_add_n(r, p, q); }
DI void grp_dbl(g2 &r, const g2 &p) { g2_dbl_n(r, p); }
DI void grp_add(g2 &r, const g2 &p, const g2 &q) { g2_add_n(r, p, q); }
// scalar multiplication by a canonical little-endian integer of nbits bits (left-to-right
// double-and-add over the scalar's own bits; scalars differ per lane, so the add is predicated)
template <class F> DI void jac_mul_bits(jac<F> &r, const jac<F> &p, const u32 *k, int nbits) {
    jac<F> acc;
    jac_set_inf(acc);
    for (int i = nbits - 1; i >= 0; i--) {
        grp_dbl(acc, acc);
        if ((k[i >> 5] >> (i & 31)) & 1) grp_add(acc, acc, p);
    }
    r = acc;
}
DN void g1_madd_n(g1 &r, const g1 &p, const fp &qx, const fp &qy) { g1 t; jac_add_aff(t, p, qx, qy); r = t; }
DN void g2_madd_n(g2 &r, const g2 &p, const fp2 &qx, const fp2 &qy) { g2 t; jac_add_aff(t, p, qx, qy); r = t; }
DI void grp_madd(g1 &r, const g1 &p, const fp &qx, const fp &qy) { g1_madd_n(r, p, qx, qy); }
DI void grp_madd(g2 &r, const g2 &p, const fp2 &qx, const fp2 &qy) { g2_madd_n(r, p, qx, qy); }
// same for an affine base point: mixed additions (G1 7M+4S, G2 the same in Fp2) instead of full Jacobian ones
// (11M+5S) — the base of every var-base multiplication on the path arrives affine (decompressed)
template <class F> DI void jac_mul_aff(jac<F> &r, const aff<F> &p, const u32 *k, int nbits) {
    jac<F> acc;
    jac_set_inf(acc);
    if (!p.inf) {
        for (int i = nbits - 1; i >= 0; i--) {
            grp_dbl(acc, acc);
            if ((k[i >> 5] >> (i & 31)) & 1) grp_madd(acc, acc, p.x, p.y);
        }
    }
    r = acc;
}
// Affine tables for the windowed ladders: Jacobian entries t[1..n-1] turned affine with one batched inversion (Montgomery's
// trick); false when an entry is the point at infinity (small-order inputs), and the caller takes its plain ladder.
template <class F, int N> DI bool jac_table_to_aff(aff<F> (&ta)[N], jac<F> (&t)[N]) {
    F pre[N];
    f_one(pre[0]);
#pragma unroll 1
    for (int i = 1; i < N; i++) f_mul(pre[i], pre[i - 1], t[i].z);
    if (f_is_zero(pre[N - 1])) return false;
    F inv;
    f_inv(inv, pre[N - 1]);
#pragma unroll 1
    for (int i = N - 1; i >= 1; i--) {
        F zi, zi2;
        f_mul(zi, inv, pre[i - 1]);        // 1 / z_i
        f_mul(inv, inv, t[i].z);
        f_sqr(zi2, zi);
        f_mul(ta[i].x, t[i].x, zi2);
        f_mul(zi2, zi2, zi);
        f_mul(ta[i].y, t[i].y, zi2);
        ta[i].inf = false;
    }
    return true;
}
// k P (k: 8 LE words) for any on-curve P with a fixed 4-bit window: 256 doublings and 64 mixed additions of table
// entries (1..15) P, instead of 256 doublings and 256 additions per wave (some lane of a wave has every bit set).
// Integer scalar multiplication throughout, so exact outside the r-torsion too (G1.FromBytes accepts such points);
// a table entry at infinity (a point of order <= 15) falls back to the binary ladder.
template <class F> DI void jac_mul_win4(jac<F> &r, const aff<F> &P, const u32 k[8]) {
    jac_set_inf(r);
    if (P.inf) return;
    jac<F> t[16];
    jac_from_aff(t[1], P);
    jac_dbl(t[2], t[1]);
#pragma unroll 1
    for (int i = 3; i < 16; i++) jac_add_aff(t[i], t[i - 1], P.x, P.y);
    aff<F> ta[16];
    if (!jac_table_to_aff(ta, t)) { jac_mul_aff(r, P, k, 256); return; }
#pragma unroll 1
    for (int w = 63; w >= 0; w--) {
        jac_dbl(r, r); jac_dbl(r, r); jac_dbl(r, r); jac_dbl(r, r);
        u32 nib = (k[w >> 3] >> (4 * (w & 7))) & 15;
        if (nib) jac_add_aff(r, r, ta[nib].x, ta[nib].y);
    }
}
// k p for a small public k: doublings only from k's top bit (the bucket-reduce offsets are < 2^c)
template <class F> DI void jac_mul_u64(jac<F> &r, const jac<F> &p, u64 k) {
    if (k == 0) { jac_set_inf(r); return; }
    int top = 63 - __clzll(k);
    jac<F> acc = p;
    for (int i = top - 1; i >= 0; i--) {
        grp_dbl(acc, acc);
        if ((k >> i) & 1) grp_add(acc, acc, p);
    }
    r = acc;
}

// jac_mul_u64 with the group operations inlined (the latency chains of hash-to-G2's cofactor clearing)
template <class F> DI void jac_mul_u64_inl(jac<F> &r, const jac<F> &p, u64 k) {
    if (k == 0) { jac_set_inf(r); return; }
    int top = 63 - __clzll(k);
    jac<F> acc = p;
#pragma unroll 1
    for (int i = top - 1; i >= 0; i--) {
        jac_dbl(acc, acc);
        if ((k >> i) & 1) jac_add(acc, acc, p);
    }
    r = acc;
}

// ---------------------------------------------------------------- G2 endomorphism psi (M-type twist)
// psi(x, y) = (conj(x) xi^-(p-1)/3, conj(y) xi^-(p-1)/2); Jacobian-compatible since conj commutes
DI void g2_psi(g2 &r, const g2 &p) {
    fp2 cx, cy;
    fp2_load_const(cx, LCB_PSI_X);
    fp2_load_const(cy, LCB_PSI_Y);
    fp2 x, y, z;
    fp2_conj(x, p.x);
    fp2_conj(y, p.y);
    fp2_conj(z, p.z);
    fp2_mul(r.x, x, cx);
    fp2_mul(r.y, y, cy);
    r.z = z;
}
DI void g2_psi2(g2 &r, const g2 &p) {
    fp cx, cy;
    fp_load_const(cx, LCB_PSI2_X);
    fp_load_const(cy, LCB_PSI2_Y);
    fp2_mul_fp(r.x, p.x, cx);
    fp2_mul_fp(r.y, p.y, cy);
    r.z = p.z;
}

// ---------------------------------------------------------------- GLS scalar multiplication in G2
// psi acts on G2 as multiplication by p = z (mod r), and r = z^4 - z^2 + 1 < u^4 with u = |z|, so a canonical
// scalar k < r splits into four base-u digits k = d0 + d1 u + d2 u^2 + d3 u^3 (d_i < u < 2^64) and
// k Q = d0 Q + d1 (-psi Q) + d2 psi^2 Q + d3 (-psi^3 Q): 64 shared doublings instead of 255, same additions.
DI void u256_divmod_u(u32 q[8], u64 &rem) {   // q <- q / u, rem <- q mod u (binary long division)
    const u64 u = LCB_Z_ABS;
    u32 out[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    u64 r = 0;
    for (int w = 7; w >= 0; w--) {
        u32 word = q[w], qw = 0;
        for (int b = 31; b >= 0; b--) {
            u64 hi = r >> 63;
            r = (r << 1) | ((word >> b) & 1);
            u32 take = (hi || r >= u) ? 1u : 0u;
            if (take) r -= u;
            qw = (qw << 1) | take;
        }
        out[w] = qw;
    }
#pragma unroll
    for (int j = 0; j < 8; j++) q[j] = out[j];
    rem = r;
}
DN void g2_mul_gls(g2 &r, const g2a &A, const u32 k[8]) {
    g2 acc;
    jac_set_inf(acc);
    if (A.inf) { r = acc; return; }
    u32 q[8];
#pragma unroll
    for (int j = 0; j < 8; j++) q[j] = k[j];
    u64 d[4];
    u256_divmod_u(q, d[0]);
    u256_divmod_u(q, d[1]);
    u256_divmod_u(q, d[2]);
    d[3] = (u64)q[0] | ((u64)q[1] << 32);   // k < u^4: the last quotient fits in 64 bits
    g2 P, T;
    jac_from_aff(P, A);
    g2a Q[4];
    Q[0] = A;
    g2_psi(T, P);                                   // psi Q   (z = 1 stays 1: conj(1) = 1)
    Q[1].x = T.x; fp2_neg(Q[1].y, T.y); Q[1].inf = false;
    g2_psi2(T, P);                                  // psi^2 Q
    Q[2].x = T.x; Q[2].y = T.y; Q[2].inf = false;
    g2_psi(T, T);                                   // psi^3 Q
    Q[3].x = T.x; fp2_neg(Q[3].y, T.y); Q[3].inf = false;
    for (int b = 63; b >= 0; b--) {
        grp_dbl(acc, acc);
#pragma unroll
        for (int i = 0; i < 4; i++)
            if ((d[i] >> b) & 1) grp_madd(acc, acc, Q[i].x, Q[i].y);
    }
    r = acc;
}

// G2 membership (Scott, "A note on group membership tests for G1, G2 and GT on BLS pairing-friendly curves"):
// an on-curve point P of E' lies in G2 iff psi(P) == [z]P = -[|z|]P.  One 64-bit ladder (63 doublings, 5 mixed
// additions) decides whether the GLS decomposition (valid only on G2) may be used.
DN bool g2_in_subgroup(const g2a &A) {
    if (A.inf) return true;
    g2 P, T, S;
    jac_from_aff(P, A);
    const u32 u[2] = {(u32)LCB_Z_ABS, (u32)(LCB_Z_ABS >> 32)};
    jac_mul_aff(T, A, u, 64);     // [|z|] P
    if (jac_is_inf(T)) return false;
    g2_psi(S, P);                 // psi(P), affine (Z stays 1)
    fp2 z2, z3, t, ny;
    fp2_sqr(z2, T.z);
    fp2_mul(z3, z2, T.z);
    fp2_mul(t, S.x, z2);
    bool okx = fp2_eq(t, T.x);
    fp2_mul(t, S.y, z3);
    fp2_neg(ny, T.y);
    return okx && fp2_eq(t, ny);
}

// g2_in_subgroup with the 64-bit ladder inlined (no call frames: for kernels where the test is a hot step)
DI bool g2_in_subgroup_inl(const g2a &A) {
    if (A.inf) return true;
    g2 T, S, P;
    jac_set_inf(T);
#pragma unroll 1
    for (int i = 63; i >= 0; i--) {
        jac_dbl(T, T);
        if ((LCB_Z_ABS >> i) & 1) jac_add_aff(T, T, A.x, A.y);
    }
    if (jac_is_inf(T)) return false;
    jac_from_aff(P, A);
    g2_psi(S, P);
    fp2 z2, z3, t, ny;
    fp2_sqr(z2, T.z);
    fp2_mul(z3, z2, T.z);
    fp2_mul(t, S.x, z2);
    bool okx = fp2_eq(t, T.x);
    fp2_mul(t, S.y, z3);
    fp2_neg(ny, T.y);
    return okx && fp2_eq(t, ny);
}
// ---------------------------------------------------------------- GLV scalar multiplication in G1
// phi(x, y) = (beta x, y) acts on the r-torsion as lambda = z^2 - 1 = u^2 - 1.  Two base-u digits and the
// quotient give k = d0 + d1 u + a1 u^2 = (a0 + a1) + a1 lambda with a0 = d0 + d1 u, so
// k P = (a0 + a1) P + a1 phi(P): 129 shared doublings instead of 255, the same number of additions.  Valid for
// points of order r (the Lagrange inputs are verified shares); a non-canonical scalar (>= 2^128 u^2) falls back
// to the plain ladder.
DN void g1_mul_glv(g1 &r, const g1a &A, const u32 k[8]) {
    u32 q[8];
#pragma unroll
    for (int j = 0; j < 8; j++) q[j] = k[j];
    u64 d0, d1;
    u256_divmod_u(q, d0);
    u256_divmod_u(q, d1);
    if (A.inf || (q[4] | q[5] | q[6] | q[7])) {
        jac_mul_aff(r, A, k, 256);
        return;
    }
    const u64 u = LCB_Z_ABS;
    u64 m_lo = u * d1, m_hi = __umul64hi(u, d1);
    u64 a0_lo = m_lo + d0, a0_hi = m_hi + (a0_lo < d0 ? 1 : 0);
    u64 a1_lo = (u64)q[0] | ((u64)q[1] << 32), a1_hi = (u64)q[2] | ((u64)q[3] << 32);
    u64 s_lo = a0_lo + a1_lo;
    u64 c = s_lo < a0_lo ? 1 : 0;
    u64 s_hi = a0_hi + a1_hi + c;
    u64 s_top = (s_hi < a0_hi || (c && s_hi == a0_hi)) ? 1 : 0;
    u32 sv[5] = {(u32)s_lo, (u32)(s_lo >> 32), (u32)s_hi, (u32)(s_hi >> 32), (u32)s_top};
    u32 av[4] = {(u32)a1_lo, (u32)(a1_lo >> 32), (u32)a1_hi, (u32)(a1_hi >> 32)};
    fp beta, phx;
    fp_load_const(beta, LCB_G1_BETA);
    fp_mul(phx, A.x, beta);
    g1 acc;
    jac_set_inf(acc);
    for (int b = 128; b >= 0; b--) {
        grp_dbl(acc, acc);
        if ((sv[b >> 5] >> (b & 31)) & 1) grp_madd(acc, acc, A.x, A.y);
        if (b < 128 && ((av[b >> 5] >> (b & 31)) & 1)) grp_madd(acc, acc, phx, A.y);
    }
    r = acc;
}

// ---------------------------------------------------------------- serialization
// Which coordinate's parity the G2 wire flag carries (unpinned mcl convention): 0 = y.a (default),
// 1 = y.b.  One copy per translation unit, set by every unit's lcbk_cfg_<unit> (kcommon.hpp LCB_TU_CONFIG) through
// lcb_set_g2_sign_from_b; read once per (de)compression.
static __device__ u32 lcb_g2_sign_b = 0;
// 1 = the latency-bound kernels of the batched checks (preparation chain, every level) raise their waves' issue
// priority (s_setprio) over the bulk randomisation waves that share their SIMDs (lcb_set_wave_priority)
static __device__ u32 lcb_wave_prio = 1;
#define LCB_LATENCY_PRIO()                                                                                         \
    do {                                                                                                          \
        if (lcb_wave_prio) __builtin_amdgcn_s_setprio(3);                                                         \
    } while (0)
DI const fp &g2_sign_coord(const fp2 &y) { return lcb_g2_sign_b ? y.b : y.a; }
DI void bytes48_to_raw(fp &raw, const uint8_t *b) { // 4-byte aligned source
    const u32 *w = (const u32 *)b;
#pragma unroll
    for (int j = 0; j < 12; j++) raw.v[j] = w[j];
}
DI void raw_to_bytes48(uint8_t *b, const fp &raw) {
    u32 *w = (u32 *)b;
#pragma unroll
    for (int j = 0; j < 12; j++) w[j] = raw.v[j];
}
// G1.FromBytes: returns false on a malformed encoding
DN bool g1_decompress(g1a &out, const uint8_t *b) {
    fp raw;
    bytes48_to_raw(raw, b);
    u32 any = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) any |= raw.v[j];
    if (any == 0) { out.inf = true; out.x = fp_zero(); out.y = fp_zero(); return true; }
    bool odd = raw.v[11] >> 31;
    raw.v[11] &= 0x7fffffffu;
    if (!fp_raw_lt_p(raw)) return false;
    fp x, t, y, b1;
    fp_from_raw(x, raw);
    fp_sqr(t, x);
    fp_mul(t, t, x);
    fp_load_const(b1, LCB_B1);
    fp_add(t, t, b1);
    if (!fp_sqrt(y, t)) return false;
    if (fp_is_odd(y) != odd) fp_neg(y, y);
    out.x = x; out.y = y; out.inf = false;
    return true;
}
DI void g1_compress(uint8_t *b, const g1a &a) {
    if (a.inf) { fp z = fp_zero(); raw_to_bytes48(b, z); return; }
    fp rx, ry;
    fp_to_raw(rx, a.x);
    fp_to_raw(ry, a.y);
    if (ry.v[0] & 1) rx.v[11] |= 0x80000000u;
    raw_to_bytes48(b, rx);
}
DN bool g2_decompress(g2a &out, const uint8_t *b) {
    fp ra, rb;
    bytes48_to_raw(ra, b);
    bytes48_to_raw(rb, b + 48);
    u32 any = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) any |= ra.v[j] | rb.v[j];
    if (any == 0) { out.inf = true; out.x = fp2_zero(); out.y = fp2_zero(); return true; }
    bool odd = rb.v[11] >> 31;
    rb.v[11] &= 0x7fffffffu;
    if (!fp_raw_lt_p(ra) || !fp_raw_lt_p(rb)) return false;
    fp2 x, t, y, b2;
    fp_from_raw(x.a, ra);
    fp_from_raw(x.b, rb);
    fp2_sqr(t, x);
    fp2_mul(t, t, x);
    fp2_load_const(b2, LCB_B2);
    fp2_add(t, t, b2);
    if (!fp2_sqrt_any(y, t)) return false;            // the sign is fixed below, so any root serves
    if (fp_is_odd(g2_sign_coord(y)) != odd) fp2_neg(y, y);
    out.x = x; out.y = y; out.inf = false;
    return true;
}
DI void g2_compress(uint8_t *b, const g2a &a) {
    if (a.inf) {
        fp z = fp_zero();
        raw_to_bytes48(b, z);
        raw_to_bytes48(b + 48, z);
        return;
    }
    fp xa, xb, ya;
    fp_to_raw(xa, a.x.a);
    fp_to_raw(xb, a.x.b);
    fp_to_raw(ya, g2_sign_coord(a.y));
    if (ya.v[0] & 1) xb.v[11] |= 0x80000000u;
    raw_to_bytes48(b, xa);
    raw_to_bytes48(b + 48, xb);
}
// serialisation of a Jacobian point: the affine conversion by the binary-GCD inversion (the same canonical inverse as
// the exponentiation's, ~40 K instructions against 263 K — the whole latency of the one-lane serialisations that end an
// MSM, a Lagrange sum or an mcl call; calls, so a caller's registers do not add to the inversion's)
DN void g1_compress_jac(uint8_t *b, const g1 &p) { g1a a; g1_jac_to_aff_g(a, p); g1_compress(b, a); }
DN void g2_compress_jac(uint8_t *b, const g2 &p) { g2a a; g2_jac_to_aff_g(a, p); g2_compress(b, a); }
DI void g1_generator(g1a &g) {
    fp_load_const(g.x, LCB_G1_GEN);
    fp_load_const(g.y, LCB_G1_GEN + 12);
    g.inf = false;
}
DI void g2_generator(g2a &g) {
    fp_load_const(g.x.a, LCB_G2_GEN);
    fp_load_const(g.x.b, LCB_G2_GEN + 12);
    fp_load_const(g.y.a, LCB_G2_GEN + 24);
    fp_load_const(g.y.b, LCB_G2_GEN + 36);
    g.inf = false;
}
