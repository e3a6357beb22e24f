// lachain_amd/csrc/lean.hpp — register-frugal forms of the pairing hot loops (one pairing per lane).
//
// Why: the Fp2 leaf routines (asm_routines.hpp) clobber v0..v131 at every call, so anything live across a call
// must sit in v132..v255 or in AGPRs: ~380 words per lane.  The round-1 tower code kept up to ~480 words live
// in the Miller loop (f, its Karatsuba temporaries and the line) and passed Fp12 values by reference to
// non-inlined helpers in the final exponentiation — both forced per-lane scratch (1.5 KB and 6.3 KB per lane,
// ~1 MB of HBM traffic per share).  Here every hot-loop value stays in registers:
//   * an Fp12 squaring / line multiplication parks ONE Fp6 temporary in LDS (72 words per lane, word-major,
//     bank-conflict free: lane t's word w at lds[w * LCB_BLOCK + t]) and updates f in place;
//   * Fp6 products are computed in place with 7 Fp2 temporaries instead of 8 + an output;
//   * the final exponentiation works on explicit SoA slots in HBM (word w of slot s of item i at
//     park[(s * 144 + w) * n + i], coalesced) through a few non-inlined slot operations whose arguments are
//     scalars, and pow-by-|z| keeps its base in LDS (144 words per lane = 144 KiB per 256-lane block) so only
//     the running value (144 words) and the squaring temporaries are live in its 63-step loop.
// The arithmetic is exactly the round-1 tower's (same formulas, same order of field operations up to
// commutativity), so every output is bit-identical.
//
// MEASURED SLOWER, so opt-in only (LCB_LEAN_MILLER / LCB_LEAN_FE): on one MI355X, 262,144 shares, k_tpke_miller
// 58.0 -> 78.1 ms and k_final_exp_check 63.4 -> 83.3 ms (tools/ab_bench.sh, profiles/r02/ab_lean.txt).  The
// compiler still spills around the fixed-register leaf calls, and the parking adds LDS/VMEM waits that one wave
// per SIMD cannot hide; the pairing kernels are bound by their instruction count, not by scratch traffic.
#pragma once
#include "pairing.hpp"

#ifndef LCB_BLOCK
#define LCB_BLOCK 256
#endif

// one lane's column of a word-major LDS array
// Accesses are volatile on purpose: they are loop-invariant inside pow-by-|z|, and letting the compiler hoist
// them back into registers would recreate exactly the register pressure the parking removes.
struct LdsCol {
    u32 *p;   // &lds[threadIdx.x]
    DI void put(int w, u32 v) const { ((volatile u32 *)p)[w * LCB_BLOCK] = v; }
    DI u32 get(int w) const { return ((volatile const u32 *)p)[w * LCB_BLOCK]; }
    DI void put2(int k, const fp2 &x) const {
        const u32 *s = (const u32 *)&x;
#pragma unroll
        for (int w = 0; w < 24; w++) ((volatile u32 *)p)[(24 * k + w) * LCB_BLOCK] = s[w];
    }
    DI fp2 get2(int k) const {
        fp2 r;
        u32 *d = (u32 *)&r;
#pragma unroll
        for (int w = 0; w < 24; w++) d[w] = ((volatile const u32 *)p)[(24 * k + w) * LCB_BLOCK];
        return r;
    }
};

// ------------------------------------------------------------------ Fp6 in place
// x <- x * b for b given by a functor b(j) -> fp2 (j = 0..2); same formulas as fp6_mul
template <class B> DI void fp6_mul_inplace(fp6 &x, const B &b) {
    fp2 t0, t1, t2, u;
    fp2_mul(t0, x.c0, b(0));
    fp2_mul(t1, x.c1, b(1));
    fp2_mul(t2, x.c2, b(2));
    fp2 s01, s02;
    fp2_add(s01, x.c0, x.c1);
    fp2_add(s02, x.c0, x.c2);
    fp2_add(x.c0, x.c1, x.c2);        // s12 (x.c1, x.c2 no longer needed below)
    fp2_add(u, b(1), b(2));
    fp2_mul(x.c0, x.c0, u);
    fp2_sub(x.c0, x.c0, t1);
    fp2_sub(x.c0, x.c0, t2);
    fp2_mul_xi(x.c0, x.c0);
    fp2_add(x.c0, x.c0, t0);
    fp2_add(u, b(0), b(1));
    fp2_mul(x.c1, s01, u);
    fp2_sub(x.c1, x.c1, t0);
    fp2_sub(x.c1, x.c1, t1);
    fp2_mul_xi(u, t2);
    fp2_add(x.c1, x.c1, u);
    fp2_add(u, b(0), b(2));
    fp2_mul(x.c2, s02, u);
    fp2_sub(x.c2, x.c2, t0);
    fp2_sub(x.c2, x.c2, t2);
    fp2_add(x.c2, x.c2, t1);
}
// x <- x * (b0, b1, 0) in place (same formulas as fp6_mul_01)
DI void fp6_mul_01_inplace(fp6 &x, const fp2 &b0, const fp2 &b1) {
    fp2 t0, t1, s, u;
    fp2_mul(t0, x.c0, b0);
    fp2_mul(t1, x.c1, b1);
    fp2_add(s, x.c0, x.c1);
    fp2_add(u, b0, b1);
    fp2_mul(x.c1, s, u);
    fp2_sub(x.c1, x.c1, t0);
    fp2_sub(x.c1, x.c1, t1);
    fp2_mul(x.c0, x.c2, b1);
    fp2_mul_xi(x.c0, x.c0);
    fp2_add(x.c0, x.c0, t0);
    fp2_mul(x.c2, x.c2, b0);
    fp2_add(x.c2, x.c2, t1);
}

// ------------------------------------------------------------------ Fp12 in place with one LDS Fp6
// f <- f^2 (complex squaring as fp12_sqr); t (72 words) holds c0 c1
DI void fp12_sqr_lean(fp12 &f, const LdsCol &t) {
    {
        // t = c0 * c1 written coefficient by coefficient (fp6_mul's formulas)
        fp2 t0, t1, t2, s, u, c;
        fp2_mul(t0, f.c0.c0, f.c1.c0);
        fp2_mul(t1, f.c0.c1, f.c1.c1);
        fp2_mul(t2, f.c0.c2, f.c1.c2);
        fp2_add(s, f.c0.c1, f.c0.c2);
        fp2_add(u, f.c1.c1, f.c1.c2);
        fp2_mul(c, s, u);
        fp2_sub(c, c, t1);
        fp2_sub(c, c, t2);
        fp2_mul_xi(c, c);
        fp2_add(c, c, t0);
        t.put2(0, c);
        fp2_add(s, f.c0.c0, f.c0.c1);
        fp2_add(u, f.c1.c0, f.c1.c1);
        fp2_mul(c, s, u);
        fp2_sub(c, c, t0);
        fp2_sub(c, c, t1);
        fp2_mul_xi(s, t2);
        fp2_add(c, c, s);
        t.put2(1, c);
        fp2_add(s, f.c0.c0, f.c0.c2);
        fp2_add(u, f.c1.c0, f.c1.c2);
        fp2_mul(c, s, u);
        fp2_sub(c, c, t0);
        fp2_sub(c, c, t2);
        fp2_add(c, c, t1);
        t.put2(2, c);
    }
    // s1 = v c1 + c0 (into c1), c0 <- (c0 + c1_old)(v c1_old + c0): c0 + c1 first, kept in c0
    {
        fp2 x;
        fp2_mul_xi(x, f.c1.c2);           // (v c1).c0 = xi c1.c2
        fp6 s;
        fp6_add(s, f.c0, f.c1);           // c0 + c1
        fp2 n0, n1, n2;
        fp2_add(n0, f.c0.c0, x);
        fp2_add(n1, f.c0.c1, f.c1.c0);
        fp2_add(n2, f.c0.c2, f.c1.c1);
        f.c1.c0 = n0; f.c1.c1 = n1; f.c1.c2 = n2;   // c1 <- c0 + v c1
        f.c0 = s;
    }
    fp6_mul_inplace(f.c0, [&](int j) -> fp2 { return j == 0 ? f.c1.c0 : (j == 1 ? f.c1.c1 : f.c1.c2); });
    // c0 <- c0 - t - v t ; c1 <- 2 t
    {
        fp2 a0 = t.get2(0), a1 = t.get2(1), a2 = t.get2(2), x;
        fp2_sub(f.c0.c0, f.c0.c0, a0);
        fp2_sub(f.c0.c1, f.c0.c1, a1);
        fp2_sub(f.c0.c2, f.c0.c2, a2);
        fp2_mul_xi(x, a2);
        fp2_sub(f.c0.c0, f.c0.c0, x);
        fp2_sub(f.c0.c1, f.c0.c1, a0);
        fp2_sub(f.c0.c2, f.c0.c2, a1);
        fp2_add(f.c1.c0, a0, a0);
        fp2_add(f.c1.c1, a1, a1);
        fp2_add(f.c1.c2, a2, a2);
    }
}

// f <- f * ((A + B v) + (C v) w) (the sparse line; same formulas as fp12_mul_line); t1 = f1 * (0, C, 0) in LDS
DI void fp12_mul_line_lean(fp12 &f, const fp2 &A, const fp2 &B, const fp2 &C, const LdsCol &t) {
    {
        fp2 x;
        fp2_mul(x, f.c1.c2, C);
        fp2_mul_xi(x, x);
        t.put2(0, x);
        fp2_mul(x, f.c1.c0, C);
        t.put2(1, x);
        fp2_mul(x, f.c1.c1, C);
        t.put2(2, x);
    }
    fp6_add(f.c1, f.c0, f.c1);
    fp6_mul_01_inplace(f.c0, A, B);
    fp2 bc;
    fp2_add(bc, B, C);
    fp6_mul_01_inplace(f.c1, A, bc);
    fp6_sub(f.c1, f.c1, f.c0);
    fp2 a0 = t.get2(0), a1 = t.get2(1), a2 = t.get2(2), x;
    fp2_sub(f.c1.c0, f.c1.c0, a0);
    fp2_sub(f.c1.c1, f.c1.c1, a1);
    fp2_sub(f.c1.c2, f.c1.c2, a2);
    fp2_mul_xi(x, a2);                    // v t1 = (xi t1.c2, t1.c0, t1.c1)
    fp2_add(f.c0.c0, f.c0.c0, x);
    fp2_add(f.c0.c1, f.c0.c1, a0);
    fp2_add(f.c0.c2, f.c0.c2, a1);
}
DI void fp12_mul_line_at_lean(fp12 &f, line &l, const fp &xP, const fp &yP, const LdsCol &t) {
    fp2_mul_fp(l.Bc, l.Bc, xP);
    fp2_mul_fp(l.Cc, l.Cc, yP);
    fp12_mul_line_lean(f, l.A, l.Bc, l.Cc, t);
}

// two-pair Miller loop (miller2) with the lean Fp12 operations
template <class S1, class S2>
DI void miller2_lean(fp12 &f, S1 &s1, const g1a &P1, S2 &s2, const g1a &P2, const LdsCol &t) {
    f = fp12_one();
    line l;
    bool first = true;
    for (int i = 62; i >= 0; i--) {
        if (!first) fp12_sqr_lean(f, t);
        first = false;
        s1.next(l, false);
        if (!P1.inf) fp12_mul_line_at_lean(f, l, P1.x, P1.y, t);
        s2.next(l, false);
        if (!P2.inf) fp12_mul_line_at_lean(f, l, P2.x, P2.y, t);
        if ((LCB_Z_ABS >> i) & 1) {
            s1.next(l, true);
            if (!P1.inf) fp12_mul_line_at_lean(f, l, P1.x, P1.y, t);
            s2.next(l, true);
            if (!P2.inf) fp12_mul_line_at_lean(f, l, P2.x, P2.y, t);
        }
    }
    fp12_conj(f, f);
}

// ------------------------------------------------------------------ final exponentiation on SoA slots
// Granger-Scott cyclotomic squaring in place (fp12_cyc_sqr's formulas)
DI void fp12_cyc_sqr_inplace(fp12 &f) {
    fp2 &z0 = f.c0.c0, &z4 = f.c0.c1, &z3 = f.c0.c2, &z2 = f.c1.c0, &z1 = f.c1.c1, &z5 = f.c1.c2;
    fp2 t0, t1, t2, t3;
    fp4_sqr(t0, t1, z0, z1);
    fp2_sub(z0, t0, z0); fp2_dbl(z0, z0); fp2_add(z0, z0, t0);
    fp2_add(z1, t1, z1); fp2_dbl(z1, z1); fp2_add(z1, z1, t1);
    fp4_sqr(t0, t1, z2, z3);
    fp4_sqr(t2, t3, z4, z5);
    fp2_sub(z4, t0, z4); fp2_dbl(z4, z4); fp2_add(z4, z4, t0);
    fp2_add(z5, t1, z5); fp2_dbl(z5, z5); fp2_add(z5, z5, t1);
    fp2_mul_xi(t0, t3);
    fp2_add(z2, t0, z2); fp2_dbl(z2, z2); fp2_add(z2, z2, t0);
    fp2_sub(z3, t2, z3); fp2_dbl(z3, z3); fp2_add(z3, z3, t2);
}

struct FeSlots {
    u32 *base;
    size_t n, i;
    DI u32 *at(int s, int w) const { return base + (size_t)s * 144 * n + soa_at(n, i, w); }
    DI void store(int s, const fp12 &f) const {
        const u32 *w = (const u32 *)&f;
#pragma unroll
        for (int k = 0; k < 144; k++) *at(s, k) = w[k];
    }
    DI void load(fp12 &f, int s) const {
        u32 *w = (u32 *)&f;
#pragma unroll
        for (int k = 0; k < 144; k++) w[k] = *at(s, k);
    }
    // coefficient k (0..5, struct order c0.c0 .. c1.c2) of slot s, negated for k >= 3 when conj (conj = (c0, -c1))
    DI fp2 get2(int s, int k, bool conj) const {
        fp2 r;
        u32 *d = (u32 *)&r;
#pragma unroll
        for (int w = 0; w < 24; w++) d[w] = *(volatile const u32 *)at(s, 24 * k + w);  // not hoisted: see LdsCol
        if (conj && k >= 3) fp2_neg(r, r);
        return r;
    }
};

// a <- a * b with b's coefficients from a functor b(k), k = 0..5 (fp12_mul's Karatsuba, in place)
template <class B> DI void fp12_mul_src(fp12 &a, const B &b) {
    fp6 t1 = a.c1;
    fp6_mul_inplace(t1, [&](int j) -> fp2 { return b(3 + j); });      // t1 = a1 b1
    fp6_add(a.c1, a.c1, a.c0);
    fp6_mul_inplace(a.c0, [&](int j) -> fp2 { return b(j); });        // t0 = a0 b0 (in a.c0)
    fp6_mul_inplace(a.c1, [&](int j) -> fp2 { fp2 x = b(j), y = b(3 + j); fp2_add(x, x, y); return x; });
    fp6_sub(a.c1, a.c1, a.c0);
    fp6_sub(a.c1, a.c1, t1);
    fp6_mul_v(t1, t1);
    fp6_add(a.c0, a.c0, t1);
}

// slot operations (non-inlined, scalar arguments only: no aggregate crosses a call boundary)
DN void fe_slot_mul(u32 *park, size_t n, size_t i, int dst, int a, int b, int conj_b) {
    FeSlots S{park, n, i};
    fp12 x;
    S.load(x, a);
    fp12_mul_src(x, [&](int k) -> fp2 { return S.get2(b, k, conj_b != 0); });
    S.store(dst, x);
}
DN void fe_slot_frob(u32 *park, size_t n, size_t i, int dst, int src, int k) {
    FeSlots S{park, n, i};
    fp12 x, y;
    S.load(x, src);
    if (k == 1) fp12_frob1(y, x);
    else if (k == 2) fp12_frob2(y, x);
    else fp12_frob3(y, x);
    S.store(dst, y);
}
DN void fe_slot_cyc_sqr(u32 *park, size_t n, size_t i, int dst, int src, int conj) {
    FeSlots S{park, n, i};
    fp12 x;
    S.load(x, src);
    if (conj) fp12_conj(x, x);
    fp12_cyc_sqr_inplace(x);
    S.store(dst, x);
}
// dst <- src^z (z = -|z|) for unitary src: the base lives in this lane's LDS column, the running value in registers
DN void fe_slot_pow_z(u32 *park, size_t n, size_t i, int dst, int src, u32 *lds_col) {
    FeSlots S{park, n, i};
    LdsCol L{lds_col};
    fp12 acc;
    S.load(acc, src);
    {
        const u32 *w = (const u32 *)&acc;
#pragma unroll
        for (int k = 0; k < 144; k++) L.put(k, w[k]);
    }
    for (int b = 62; b >= 0; b--) {
        fp12_cyc_sqr_inplace(acc);
        if ((LCB_Z_ABS >> b) & 1) fp12_mul_src(acc, [&](int k) -> fp2 { return L.get2(k); });
    }
    fp12_conj(acc, acc);
    S.store(dst, acc);
}
// easy part f^((p^6 - 1)(p^2 + 1)) of the value in slot 0, in place (fe_easy's operations)
DN void fe_slot_easy(u32 *park, size_t n, size_t i) {
    FeSlots S{park, n, i};
    fp12 f, t;
    S.load(f, 0);
    fp12_inv(t, f);
    fp12_conj(f, f);
    fp12_mul(f, f, t);          // f^(p^6 - 1)
    fp12_frob2(t, f);
    fp12_mul(f, t, f);          // ^(p^2 + 1)
    S.store(0, f);
}

// Final exponentiation of the Fp12 in slot 0 (6 slots per item), result in slot 4; the same exponent and product
// as fe_hard (mcl expHardPartBLS12 shape): slots X=0 T=1 U=2 V=3 A=4 W=5
DI void final_exp_slots(u32 *park, size_t n, size_t i, u32 *lds_col) {
    enum { X = 0, T = 1, U = 2, V = 3, A = 4, W = 5 };
    fe_slot_easy(park, n, i);
    fe_slot_pow_z(park, n, i, T, X, lds_col);          // t = x^z
    fe_slot_cyc_sqr(park, n, i, U, X, 1);              // x^-2
    fe_slot_mul(park, n, i, U, U, T, 0);               // u = x^(z-2)
    fe_slot_pow_z(park, n, i, V, U, lds_col);          // v = x^(z^2-2z)
    fe_slot_mul(park, n, i, A, V, X, 0);               // x^c3
    fe_slot_frob(park, n, i, A, A, 3);
    fe_slot_pow_z(park, n, i, V, V, lds_col);          // v = x^(z^3-2z^2)
    fe_slot_mul(park, n, i, W, V, T, 0);               // x^c2
    fe_slot_frob(park, n, i, W, W, 2);
    fe_slot_mul(park, n, i, A, A, W, 0);
    fe_slot_pow_z(park, n, i, V, V, lds_col);          // v = x^(z^4-2z^3)
    fe_slot_cyc_sqr(park, n, i, T, T, 0);              // t = x^2z
    fe_slot_mul(park, n, i, V, V, T, 0);               // v = x^(z^4-2z^3+2z)
    fe_slot_mul(park, n, i, W, V, X, 1);               // x^c1 = conj(x) v
    fe_slot_frob(park, n, i, W, W, 1);
    fe_slot_mul(park, n, i, A, A, W, 0);
    fe_slot_pow_z(park, n, i, V, V, lds_col);          // v = x^(z^5-2z^4+2z^2)
    fe_slot_mul(park, n, i, U, V, U, 1);               // x^(2-z) v
    fe_slot_mul(park, n, i, U, U, X, 0);               // x^c0
    fe_slot_mul(park, n, i, A, A, U, 0);               // y
}
DN bool fe_slot_is_one(u32 *park, size_t n, size_t i, int s) {
    FeSlots S{park, n, i};
    fp12 y;
    S.load(y, s);
    return fp12_is_one(y);
}
