// lachain_amd/csrc/coop.hpp — cooperative pairing check: NINE lanes of a wave share one Miller loop and one final
// exponentiation (seven checks per wave), for the launches that are too small to fill the GPU one check per lane.
//
// Why: a one-lane pairing check (k_tpke_miller + k_final_exp_check) is ~15 K serial Fp products, ~20-25 ms at one wave
// per SIMD whatever the launch size below 65,536 lanes — the latency floor of the randomized batch check's splitting
// levels, its census, the queue flushes and every mcl single-element pairing.  Every Fp12 operation of the pairing is
// one round of <= 9 (or 18) INDEPENDENT Fp2 products (Karatsuba over Fp6 / Fp12, Granger-Scott squaring, the sparse
// line product), so nine lanes each compute one Fp2 product per round and the whole check takes ~650 rounds.
//
// Data flow, per group of nine lanes (role j = lane % 9):
//   * the Fp12 accumulator is DISTRIBUTED: lane j < 6 holds coefficient j in a register (R), in field.hpp's layout
//     c0 = (F0, F1, F2), c1 = (F3, F4, F5);
//   * an operation publishes R to the group's LDS slots, each lane gathers its two operands (sums of <= 2 slots,
//     optionally times xi) and computes one Fp2 product (the asm leaf routines of field.hpp), publishes it (and xi * it),
//     and lanes 0..5 recombine their new coefficient from <= 4 published values;
//   * every per-lane difference is DATA (slot indices packed 6 bits per lane in a 64-bit constant, selected by j), never
//     control flow: the wave executes each phase once for all seven groups (a divergent branch would be executed once
//     per distinct role);
//   * Fp12 values the final exponentiation keeps (x, t, u, v, acc, w) are parked in HBM in the SoA park layout of the
//     one-lane kernels (kcommon.hpp), which the Miller kernels also write f into: the kernels interoperate.
// The results are the same field elements as the one-lane code (same formulas, same order of the products), so every
// GT value, Miller value and decision is bit-identical (tests/test_gpu_coop.py compares them).
#pragma once
#include "kcommon.hpp"

#define CP_L 9                 // lanes per pairing check
#define CP_G 7                 // checks per wave (lanes 0..62; lane 63 is a dummy group of its own)
#define CP_AREAS 7             // one LDS area per live group (the dummy lane 63 reads area 0 and never writes)
#define CP_BLOCK 64            // one wave per workgroup (__syncthreads is the wave's LDS ordering point)
// Fp2 slots of a group's LDS area (96 B each)
#define S_F 0                  // 6: the published accumulator
#define S_Z 6                  // the constant 0
#define S_P 7                  // 18: products (a reader applies xi itself: cp_lin4's flags)
#define S_AUX 25               // 9: pre-sums / recombination outputs
#define S_JUNK (-1)            // "nothing to publish": the store is skipped (exec-masked)
#define S_LE (S_P + 14)        // 4 evaluated line coefficients (Miller loop only; overlays P[14..17])
#define CP_NS 34               // 7 areas x 34 x 96 B = 22,848 B per wave: seven waves per CU
#define CP_LDS_QUADS (CP_AREAS * CP_NS * 6)

typedef unsigned long long u64c;
#define PK9(a0, a1, a2, a3, a4, a5, a6, a7, a8)                                                                        \
    ((u64c)(a0) | (u64c)(a1) << 6 | (u64c)(a2) << 12 | (u64c)(a3) << 18 | (u64c)(a4) << 24 | (u64c)(a5) << 30 |       \
     (u64c)(a6) << 36 | (u64c)(a7) << 42 | (u64c)(a8) << 48)
DI int sel9(u64c t, int j) {
    asm volatile("" : "+v"(j));       // per use: the per-lane slot indices are not hoisted into long-lived registers
    return (int)((t >> (6 * j)) & 63);
}
DI bool bit9(unsigned m, int j) {      // this lane's flag of a 9-bit per-role mask
    asm volatile("" : "+v"(j));
    return (m >> j) & 1u;
}
// aliases for the tables
#define Z_ S_Z
#define P_(k) (S_P + (k))
#define A_(k) (S_AUX + (k))

struct Cp {
    uint4 *s;          // the group's LDS area
    int j;             // role 0..8
    int g;             // group in the wave (7 = the dummy lane)
};
// the lane's role, re-read at every use: the per-lane slot indices, LDS and park addresses derived from it are then
// recomputed where they are used (a few instructions each) instead of being hoisted out of the program loops into
// ~100 long-lived registers (the final exponentiation kernel held 391 registers with them, 230 without)
DI int cpj(const Cp &c) {
    int j = c.j;
    asm volatile("" : "+v"(j));
    return j;
}
DI Cp cp_init(uint4 *lds) {
    Cp c;
    const int l = threadIdx.x & 63;
    c.g = l / CP_L;
    c.j = l - CP_L * c.g;
    c.s = lds + (c.g < CP_G ? c.g : 0) * (CP_NS * 6);
    return c;
}
DI void cp_sync() { __syncthreads(); }
DI void cp_put(const Cp &c, int slot, const fp2 &x) {
    if (slot < 0 || c.g >= CP_G) return;
    uint4 *p = c.s + slot * 6;
    const u32 *w = (const u32 *)&x;
#pragma unroll
    for (int q = 0; q < 6; q++) p[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}
DI void cp_get(fp2 &x, const Cp &c, int slot) {
    const uint4 *p = c.s + slot * 6;
    u32 *w = (u32 *)&x;
#pragma unroll
    for (int q = 0; q < 6; q++) {
        uint4 v = p[q];
        w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
}
DI void fp2_sel(fp2 &r, bool c, const fp2 &a, const fp2 &b) {       // r = c ? a : b, word by word
    u32 *rw = (u32 *)&r;
    const u32 *aw = (const u32 *)&a, *bw = (const u32 *)&b;
#pragma unroll
    for (int q = 0; q < 24; q++) rw[q] = c ? aw[q] : bw[q];
}
DI void fp2_cxi(fp2 &r, const fp2 &x, bool c) { fp2 t; fp2_mul_xi(t, x); fp2_sel(r, c, t, x); }
DI void fp2_cneg(fp2 &r, const fp2 &x, bool c) { fp2 t; fp2_neg(t, x); fp2_sel(r, c, t, x); }
// the publish of R (lanes 0..5) and the zero slot
DI void cp_publish(const Cp &c, const fp2 &R) { cp_put(c, cpj(c) < 6 ? S_F + cpj(c) : S_JUNK, R); }
// out = xi^fa (L[a] - L[b] - L[cc]) + xi^fd L[d]: the recombinations of the Karatsuba / Granger-Scott products
// (every lane's formula is a difference of three values and a fourth, each group with one power of xi)
DI void cp_lin4(fp2 &o, const Cp &c, int a, int b, int cc, int d, bool fa, bool fd) {
    fp2 x;
    cp_get(o, c, a);
    cp_get(x, c, b);
    fp2_sub(o, o, x);
    cp_get(x, c, cc);
    fp2_sub(o, o, x);
    fp2_cxi(o, o, fa);
    cp_get(x, c, d);
    fp2_cxi(x, x, fd);
    fp2_add(o, o, x);
}
// cp_lin4 without the fourth value's xi (no lane of the call site applies it): the wave skips one xi product and one
// select per recombination (round 6; the squarings, line products and Fp12 products' last stage)
DI void cp_lin3(fp2 &o, const Cp &c, int a, int b, int cc, int d, bool fa) {
    fp2 x;
    cp_get(o, c, a);
    cp_get(x, c, b);
    fp2_sub(o, o, x);
    cp_get(x, c, cc);
    fp2_sub(o, o, x);
    fp2_cxi(o, o, fa);
    cp_get(x, c, d);
    fp2_add(o, o, x);
}
// one product per lane: (L[xa] + L[xb]) * xi^yx (L[ya] + L[yb]) -> P[pk] (pk = -1: nothing published); XI = false:
// no lane applies xi (the wave skips the xi product and its select)
template <bool XI = true> DI void cp_prod(const Cp &c, int xa, int xb, int ya, int yb, bool yx, int pk) {
    fp2 x, y, t;
    cp_get(x, c, xa);
    cp_get(t, c, xb);
    fp2_add(x, x, t);
    cp_get(y, c, ya);
    cp_get(t, c, yb);
    fp2_add(y, y, t);
    if (XI) fp2_cxi(y, y, yx);
    fp2_mul(x, x, y);
    cp_put(c, pk >= 0 ? S_P + pk : S_JUNK, x);
}

// ---------------------------------------------------------------- park (HBM) access: lane j < 6 owns coefficient j
// SoA quad-major slots of n items (kcommon.hpp fp12_store_soa): coefficient j = words 24j..24j+23 = quads 6j..6j+5
DI void park_get(fp2 &x, const u32 *slot, size_t n, size_t i, int j) {
    const int k = j < 6 ? j : 0;
    u32 *w = (u32 *)&x;
    const char *b = (const char *)slot;
#pragma unroll
    for (int q = 0; q < 6; q++) {
        uint4 v = *(const uint4 *)(b + ((size_t)(6 * k + q) * n + i) * 16);
        w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
}
DI void park_put(u32 *slot, size_t n, size_t i, int j, bool live, const fp2 &x) {
    if (!live || j >= 6) return;
    const u32 *w = (const u32 *)&x;
    char *b = (char *)slot;
#pragma unroll
    for (int q = 0; q < 6; q++)
        *(uint4 *)(b + ((size_t)(6 * j + q) * n + i) * 16) = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}
// coefficient k of a parked value (k == 6: zero)
DI void park_coef(fp2 &x, const u32 *slot, size_t n, size_t i, int k) {
    park_get(x, slot, n, i, k < 6 ? k : 0);
    fp2 z = fp2_zero();
    fp2_sel(x, k >= 6, z, x);
}

// ---------------------------------------------------------------- the Fp12 operations (all lanes call them)
// R <- R^2 (any Fp12): T = c0 c1 and Q = (c0 + c1)(c0 + v c1) as two Karatsuba Fp6 products (12 products), then
// c0' = Q - T - v T, c1' = 2 T (field.hpp fp12_sqr).  Round B's idle lanes 3..6 evaluate the next line's coefficients
// (ev: a product whose operands come from HBM: a line coefficient and a point coordinate).
struct CpEval {                // a product lane's HBM operands: line coefficient x point coordinate (as (c, 0)),
    bool on;                   // read where they are used (not held across the loop)
    bool yinf;                 // the point is at infinity: coordinate 0, so every line evaluates to 1
    const u32 *xp, *yp;
};
DI void cp_ev_get(fp2 &x, fp2 &y, const CpEval &ev) {
    fp2_load_w(x, ev.xp);
    const uint4 *q = (const uint4 *)ev.yp;
    u32 *w = (u32 *)&y.a;
#pragma unroll
    for (int g = 0; g < 3; g++) {
        uint4 v = q[g];
        w[4 * g] = v.x; w[4 * g + 1] = v.y; w[4 * g + 2] = v.z; w[4 * g + 3] = v.w;
    }
    if (ev.yinf) y.a = fp_zero();
    y.b = fp_zero();
}
DI void cp_sqr12(fp2 &R, const Cp &c, const CpEval &ev) {
    const int j = cpj(c);
    cp_publish(c, R);
    cp_sync();
    {   // S_k = a_k + b_k (lanes 0..2), U = (a0 + xi b2, a1 + b0, a2 + b1) (lanes 3..5) -> AUX0..5
        fp2 x, y;
        cp_get(x, c, sel9(PK9(0, 1, 2, 0, 1, 2, Z_, Z_, Z_), j));
        cp_get(y, c, sel9(PK9(3, 4, 5, 5, 3, 4, Z_, Z_, Z_), j));
        fp2_cxi(y, y, j == 3);
        fp2_add(x, x, y);
        cp_put(c, j < 6 ? S_AUX + j : S_JUNK, x);
    }
    cp_sync();
    // round A: T's six products, Q's first three
    cp_prod<false>(c, sel9(PK9(0, 1, 2, 1, 0, 0, A_(0), A_(1), A_(2)), j), sel9(PK9(Z_, Z_, Z_, 2, 1, 2, Z_, Z_, Z_), j),
            sel9(PK9(3, 4, 5, 4, 3, 3, A_(3), A_(4), A_(5)), j), sel9(PK9(Z_, Z_, Z_, 5, 4, 5, Z_, Z_, Z_), j), false, j);
    {   // round B: Q's cross products (lanes 0..2) + the line evaluations (lanes 3..6)
        fp2 x, y, t;
        cp_get(x, c, sel9(PK9(A_(1), A_(0), A_(0), Z_, Z_, Z_, Z_, Z_, Z_), j));
        cp_get(t, c, sel9(PK9(A_(2), A_(1), A_(2), Z_, Z_, Z_, Z_, Z_, Z_), j));
        fp2_add(x, x, t);
        cp_get(y, c, sel9(PK9(A_(4), A_(3), A_(3), Z_, Z_, Z_, Z_, Z_, Z_), j));
        cp_get(t, c, sel9(PK9(A_(5), A_(4), A_(5), Z_, Z_, Z_, Z_, Z_, Z_), j));
        fp2_add(y, y, t);
        {
            fp2 ex, ey;
            cp_ev_get(ex, ey, ev);
            fp2_sel(x, ev.on, ex, x);
            fp2_sel(y, ev.on, ey, y);
        }
        fp2_mul(x, x, y);
        const int slot = j < 3 ? S_P + 9 + j : (ev.on ? S_LE + j - 3 : S_JUNK);
        cp_put(c, slot, x);
    }
    cp_sync();
    {   // T_k = fp6 recombination of P0..5 (lanes 0..2), Q_k of P6..11 (lanes 3..5) -> AUX0..5
        fp2 o;
        cp_lin4(o, c, sel9(PK9(P_(3), P_(4), P_(1), P_(9), P_(10), P_(7), Z_, Z_, Z_), j),
                sel9(PK9(P_(1), P_(0), P_(0), P_(7), P_(6), P_(6), Z_, Z_, Z_), j),
                sel9(PK9(P_(2), P_(1), P_(2), P_(8), P_(7), P_(8), Z_, Z_, Z_), j),
                sel9(PK9(P_(0), P_(2), P_(5), P_(6), P_(8), P_(11), Z_, Z_, Z_), j), bit9(0x009u, j), bit9(0x012u, j));
        cp_put(c, j < 6 ? S_AUX + j : S_JUNK, o);
    }
    cp_sync();
    {   // c0'_k = Q_k - T_k - (v T)_k (lanes 0..2), c1'_k = 2 T_k (lanes 3..5); (v T) = (xi T2, T0, T1)
        fp2 o, x;
        cp_get(o, c, sel9(PK9(A_(3), A_(4), A_(5), A_(0), A_(1), A_(2), Z_, Z_, Z_), j));
        cp_get(x, c, sel9(PK9(A_(0), A_(1), A_(2), Z_, Z_, Z_, Z_, Z_, Z_), j));
        fp2_sub(o, o, x);
        cp_get(x, c, sel9(PK9(A_(2), A_(0), A_(1), Z_, Z_, Z_, Z_, Z_, Z_), j));
        fp2_cxi(x, x, j == 0);
        fp2_sub(o, o, x);
        cp_get(x, c, sel9(PK9(Z_, Z_, Z_, A_(0), A_(1), A_(2), Z_, Z_, Z_), j));
        fp2_add(o, o, x);
        if (j < 6) R = o;
    }
}
// R <- R * (1 + b v + c v w) for the normalised line evaluated into slots sb, sc (field.hpp fp12_mul_line_n):
// X = v f0, Y = v f1; t0_k = b X_k, t1_k = c Y_k, s_k = (b + c)(X_k + Y_k);
// f0_k += t0_k + (v t1)_k, f1_k += s_k - t0_k - t1_k
DI void cp_line(fp2 &R, const Cp &c, int sb, int sc) {
    const int j = cpj(c);
    cp_publish(c, R);
    cp_sync();
    const int xa = j < 3 ? sb : (j < 6 ? sc : sb), xb = j < 6 ? S_Z : sc;
    cp_prod(c, xa, xb, sel9(PK9(2, 0, 1, 5, 3, 4, 2, 0, 1), j), sel9(PK9(Z_, Z_, Z_, Z_, Z_, Z_, 5, 3, 4), j),
            j == 0 || j == 3 || j == 6, j);
    cp_sync();
    fp2 o;
    cp_lin3(o, c, sel9(PK9(P_(5), P_(3), P_(4), P_(6), P_(7), P_(8), Z_, Z_, Z_), j),
            sel9(PK9(Z_, Z_, Z_, P_(0), P_(1), P_(2), Z_, Z_, Z_), j),
            sel9(PK9(Z_, Z_, Z_, P_(3), P_(4), P_(5), Z_, Z_, Z_), j),
            sel9(PK9(P_(0), P_(1), P_(2), Z_, Z_, Z_, Z_, Z_, Z_), j), bit9(0x001u, j));
    fp2_add(o, o, R);
    if (j < 6) R = o;
}
// a round of products whose operands come from HBM only (the line evaluations of a step without squaring)
// (the evaluating lanes are 3..6, as in cp_sqr12's round B)
DI void cp_eval_round(const Cp &c, const CpEval &ev) {
    fp2 x, y;
    cp_ev_get(x, y, ev);
    fp2_mul(x, x, y);
    cp_put(c, ev.on ? S_LE + cpj(c) - 3 : S_JUNK, x);
}
// R <- R^2 for R in the cyclotomic subgroup (Granger-Scott, field.hpp fp12_cyc_sqr): per pair (a, b) of
// (z0, z1) = (F0, F4), (z2, z3) = (F3, F2), (z4, z5) = (F1, F5): a^2, b^2, (a + b)^2; c0 = a^2 + xi b^2,
// c1 = (a + b)^2 - a^2 - b^2; z' = 3 c -/+ 2 z
DI void cp_cyc_sqr(fp2 &R, const Cp &c) {
    const int j = cpj(c);
    cp_publish(c, R);
    cp_sync();
    {
        fp2 x, t;
        cp_get(x, c, sel9(PK9(0, 4, 0, 3, 2, 3, 1, 5, 1), j));
        cp_get(t, c, sel9(PK9(Z_, Z_, 4, Z_, Z_, 2, Z_, Z_, 5), j));
        fp2_add(x, x, t);
        fp2_sqr(x, x);
        cp_put(c, S_P + j, x);
    }
    cp_sync();
    fp2 y, u;
    // F0: c0(0) = P0 + xi P1, F1: c0(1) = P3 + xi P4, F2: c0(2) = P6 + xi P7, F3: xi c1(2), F4: c1(0), F5: c1(1)
    cp_lin3(y, c, sel9(PK9(P_(1), P_(4), P_(7), P_(8), P_(2), P_(5), Z_, Z_, Z_), j),
            sel9(PK9(Z_, Z_, Z_, P_(6), P_(0), P_(3), Z_, Z_, Z_), j),
            sel9(PK9(Z_, Z_, Z_, P_(7), P_(1), P_(4), Z_, Z_, Z_), j),
            sel9(PK9(P_(0), P_(3), P_(6), Z_, Z_, Z_, Z_, Z_, Z_), j), bit9(0x00fu, j));
    fp2_cneg(u, R, j < 3);          // 3y - 2z (c0 outputs) or 3y + 2z (c1 outputs) = y + 2 (y -/+ z)
    fp2_add(u, u, y);
    fp2_add(u, u, u);
    fp2_add(u, u, y);
    if (j < 6) R = u;
}
// R <- (conj_a ? conj(R) : R) * B with B parked at bslot (Karatsuba over Fp6: T = a0 b0, U = a1 b1,
// M = (a0 + a1)(b0 + b1): 18 products in two rounds; c0 = T + v U, c1 = M - T - U)
DI void cp_mul12(fp2 &R, const Cp &c, bool conj_a, const u32 *bslot, size_t n, size_t i) {
    const int j = cpj(c);
    fp2 a;
    fp2_cneg(a, R, conj_a && j >= 3);
    cp_publish(c, a);
    cp_sync();
    {   // SA_k = a0_k + a1_k (lanes 0..2) -> AUX0..2
        fp2 x, y;
        cp_get(x, c, j < 3 ? j : S_Z);
        cp_get(y, c, j < 3 ? j + 3 : S_Z);
        fp2_add(x, x, y);
        cp_put(c, j < 3 ? S_AUX + j : S_JUNK, x);
    }
    cp_sync();
#pragma unroll
    for (int r = 0; r < 2; r++) {
        // x = L[xa] + L[xb], y = B[y0] + B[y1] + B[y2] + B[y3] (B coefficients from the park, 6 = zero)
        const u64c XA = r == 0 ? PK9(0, 1, 2, 1, 0, 0, 3, 4, 5) : PK9(4, 3, 3, A_(0), A_(1), A_(2), A_(1), A_(0), A_(0));
        const u64c XB = r == 0 ? PK9(Z_, Z_, Z_, 2, 1, 2, Z_, Z_, Z_) : PK9(5, 4, 5, Z_, Z_, Z_, A_(2), A_(1), A_(2));
        const u64c Y0 = r == 0 ? PK9(0, 1, 2, 1, 0, 0, 3, 4, 5) : PK9(4, 3, 3, 0, 1, 2, 1, 0, 0);
        const u64c Y1 = r == 0 ? PK9(6, 6, 6, 2, 1, 2, 6, 6, 6) : PK9(5, 4, 5, 3, 4, 5, 4, 3, 3);
        const u64c Y2 = r == 0 ? PK9(6, 6, 6, 6, 6, 6, 6, 6, 6) : PK9(6, 6, 6, 6, 6, 6, 2, 1, 2);
        const u64c Y3 = r == 0 ? PK9(6, 6, 6, 6, 6, 6, 6, 6, 6) : PK9(6, 6, 6, 6, 6, 6, 5, 4, 5);
        fp2 x, y, t;
        cp_get(x, c, sel9(XA, j));
        cp_get(t, c, sel9(XB, j));
        fp2_add(x, x, t);
        park_coef(y, bslot, n, i, sel9(Y0, j));
        park_coef(t, bslot, n, i, sel9(Y1, j));
        fp2_add(y, y, t);
        if (r == 1) {                 // (round 0's third and fourth terms are zero for every role)
            park_coef(t, bslot, n, i, sel9(Y2, j));
            fp2_add(y, y, t);
            park_coef(t, bslot, n, i, sel9(Y3, j));
            fp2_add(y, y, t);
        }
        fp2_mul(x, x, y);
        cp_put(c, S_P + 9 * r + j, x);
    }
    cp_sync();
    {   // T_k (lanes 0..2), U_k (3..5), M_k (6..8): fp6 recombination of P0..5, P6..11, P12..17 -> AUX0..8
        fp2 o;
        cp_lin4(o, c, sel9(PK9(P_(3), P_(4), P_(1), P_(9), P_(10), P_(7), P_(15), P_(16), P_(13)), j),
                sel9(PK9(P_(1), P_(0), P_(0), P_(7), P_(6), P_(6), P_(13), P_(12), P_(12)), j),
                sel9(PK9(P_(2), P_(1), P_(2), P_(8), P_(7), P_(8), P_(14), P_(13), P_(14)), j),
                sel9(PK9(P_(0), P_(2), P_(5), P_(6), P_(8), P_(11), P_(12), P_(14), P_(17)), j), bit9(0x049u, j),
                bit9(0x092u, j));
        cp_put(c, S_AUX + j, o);
    }
    cp_sync();
    {   // c0 = (T0 + xi U2, T1 + U0, T2 + U1) (lanes 0..2), c1_k = M_k - T_k - U_k (lanes 3..5)
        fp2 o;
        cp_lin3(o, c, sel9(PK9(A_(5), A_(3), A_(4), A_(6), A_(7), A_(8), Z_, Z_, Z_), j),
                sel9(PK9(Z_, Z_, Z_, A_(0), A_(1), A_(2), Z_, Z_, Z_), j),
                sel9(PK9(Z_, Z_, Z_, A_(3), A_(4), A_(5), Z_, Z_, Z_), j),
                sel9(PK9(A_(0), A_(1), A_(2), Z_, Z_, Z_, Z_, Z_, Z_), j), bit9(0x001u, j));
        if (j < 6) R = o;
    }
}
// Frobenius maps (field.hpp fp12_frob1/2/3): coefficient g_m (m = (0, 2, 4, 1, 3, 5)[j]) times gamma_k[m], conjugated
// for k = 1, 3
DI void cp_frob(fp2 &R, const Cp &c, int k) {
    const int j = cpj(c) < 6 ? cpj(c) : 0;
    const int m = (int)((0x531420u >> (4 * j)) & 15);
    fp2 g, cst;
    if (k != 2) fp2_conj(g, R);
    else g = R;
    if (k == 1) fp2_load_const(cst, LCB_GAMMA1 + 24 * m);
    else if (k == 3) fp2_load_const(cst, LCB_GAMMA3 + 24 * m);
    else { fp_load_const(cst.a, LCB_GAMMA2 + 12 * m); cst.b = fp_zero(); }
    fp2_mul(g, g, cst);
    if (cpj(c) < 6) R = g;
}
DI void cp_conj(fp2 &R, const Cp &c) { fp2_cneg(R, R, cpj(c) >= 3 && cpj(c) < 6); }
DI void cp_one(fp2 &R, const Cp &c) { R = cpj(c) == 0 ? fp2_one() : fp2_zero(); }
// fp6 products of two Fp6 operands held in slots, two per call: (a0 (slots xa..xa+2) x b0 (ya..)) -> P0..5 and
// (a1 (xb..) x b1 (yb..)) -> P6..11, Karatsuba (t_k = a_k b_k, (a1+a2)(b1+b2), (a0+a1)(b0+b1), (a0+a2)(b0+b2)) in two
// rounds of nine lanes
DI void cp_fp6_pair(const Cp &c, int xa, int ya, int xb, int yb) {
    const int j = cpj(c);
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const int pk = 9 * r + j;                      // product 0..11 (12..17: idle)
        const int m = pk < 6 ? pk : pk - 6;            // index within its fp6 product
        const int bx = pk < 6 ? xa : xb, by = pk < 6 ? ya : yb;
        const int i0 = (int)((0x001210u >> (4 * m)) & 15), i1 = (int)((0x212000u >> (4 * m)) & 15);
        const bool two = m >= 3;
        const bool on = pk < 12;
        cp_prod<false>(c, bx + i0, two ? bx + i1 : S_Z, by + i0, two ? by + i1 : S_Z, false, on ? pk : -1);
    }
}
// R <- R^-1 (field.hpp fp12_inv / fp6_inv / fp2_inv): c0^2 and c1^2, d = c0^2 - v c1^2, d^-1 by the fp6 adjugate and
// one Fp inversion (role-0 lanes only), then (c0 d^-1, -c1 d^-1)
DI void cp_inv(fp2 &R, const Cp &c) {
    const int j = cpj(c);
    cp_publish(c, R);
    cp_sync();
    cp_fp6_pair(c, 0, 0, 3, 3);                        // c0^2 -> P0..5, c1^2 -> P6..11
    cp_sync();
    {   // T = c0^2 (lanes 0..2), U = c1^2 (lanes 3..5) -> AUX0..5 (fp6 recombination, as cp_sqr12 stage 1)
        fp2 o;
        cp_lin4(o, c, sel9(PK9(P_(3), P_(4), P_(1), P_(9), P_(10), P_(7), Z_, Z_, Z_), j),
                sel9(PK9(P_(1), P_(0), P_(0), P_(7), P_(6), P_(6), Z_, Z_, Z_), j),
                sel9(PK9(P_(2), P_(1), P_(2), P_(8), P_(7), P_(8), Z_, Z_, Z_), j),
                sel9(PK9(P_(0), P_(2), P_(5), P_(6), P_(8), P_(11), Z_, Z_, Z_), j), bit9(0x009u, j), bit9(0x012u, j));
        cp_put(c, j < 6 ? S_AUX + j : S_JUNK, o);
    }
    cp_sync();
    {   // d = T - v U = (T0 - xi U2, T1 - U0, T2 - U1) (lanes 0..2) -> AUX6..8
        fp2 o, x;
        cp_get(o, c, j < 3 ? S_AUX + j : S_Z);
        cp_get(x, c, sel9(PK9(A_(5), A_(3), A_(4), Z_, Z_, Z_, Z_, Z_, Z_), j));
        fp2_cxi(x, x, j == 0);
        fp2_sub(o, o, x);
        cp_put(c, j < 3 ? S_AUX + 6 + j : S_JUNK, o);
    }
    cp_sync();
    // adjugate products: d0^2, d1 d2, d2^2, d0 d1, d1^2, d0 d2 -> P0..5
    cp_prod<false>(c, sel9(PK9(A_(6), A_(7), A_(8), A_(6), A_(7), A_(6), Z_, Z_, Z_), j), S_Z,
            sel9(PK9(A_(6), A_(8), A_(8), A_(7), A_(7), A_(8), Z_, Z_, Z_), j), S_Z, false, j < 6 ? j : -1);
    cp_sync();
    {   // A = d0^2 - xi d1 d2, B = xi d2^2 - d0 d1, C = d1^2 - d0 d2 (lanes 0..2) -> AUX0..2
        fp2 o;
        cp_lin4(o, c, sel9(PK9(Z_, Z_, P_(4), Z_, Z_, Z_, Z_, Z_, Z_), j),
                sel9(PK9(P_(1), P_(3), P_(5), Z_, Z_, Z_, Z_, Z_, Z_), j), S_Z,
                sel9(PK9(P_(0), P_(2), Z_, Z_, Z_, Z_, Z_, Z_, Z_), j), bit9(0x001u, j), bit9(0x002u, j));
        cp_put(c, j < 3 ? S_AUX + j : S_JUNK, o);
    }
    cp_sync();
    // N = d0 A + xi (d2 B + d1 C): products d0 A, d2 B, d1 C -> P0..2
    cp_prod<false>(c, sel9(PK9(A_(6), A_(8), A_(7), Z_, Z_, Z_, Z_, Z_, Z_), j), S_Z,
            sel9(PK9(A_(0), A_(1), A_(2), Z_, Z_, Z_, Z_, Z_, Z_), j), S_Z, false, j < 3 ? j : -1);
    cp_sync();
    if (j == 0) {      // N^-1 = conj(N) / (a^2 + b^2): the one Fp inversion of the check (role-0 lanes only)
        fp2 nv, t;
        cp_get(nv, c, S_P + 1);
        cp_get(t, c, S_P + 2);
        fp2_add(nv, nv, t);
        fp2_mul_xi(nv, nv);
        cp_get(t, c, S_P + 0);
        fp2_add(nv, nv, t);
        fp a2, b2, nrm;
        fp_mul2(a2, nv.a, nv.a, b2, nv.b, nv.b);
        fp_add(nrm, a2, b2);
        fp_inv_gcd(nrm, nrm);          // binary GCD: ~40 K instructions against the exponentiation's 263 K
        fp2_mul_fp(nv, nv, nrm);
        fp_neg(nv.b, nv.b);
        cp_put(c, S_AUX + 3, nv);
    }
    cp_sync();
    // d^-1 = (A, B, C) N^-1 -> AUX6..8 (lanes 0..2)
    cp_prod<false>(c, j < 3 ? S_AUX + j : S_Z, S_Z, S_AUX + 3, S_Z, false, j < 3 ? j : -1);
    cp_sync();
    {
        fp2 o;
        cp_get(o, c, j < 3 ? S_P + j : S_Z);
        cp_put(c, j < 3 ? S_AUX + 6 + j : S_JUNK, o);
    }
    cp_sync();
    cp_fp6_pair(c, S_F + 0, S_AUX + 6, S_F + 3, S_AUX + 6);   // c0 d^-1 -> P0..5, c1 d^-1 -> P6..11
    cp_sync();
    fp2 o;
    cp_lin4(o, c, sel9(PK9(P_(3), P_(4), P_(1), P_(9), P_(10), P_(7), Z_, Z_, Z_), j),
            sel9(PK9(P_(1), P_(0), P_(0), P_(7), P_(6), P_(6), Z_, Z_, Z_), j),
            sel9(PK9(P_(2), P_(1), P_(2), P_(8), P_(7), P_(8), Z_, Z_, Z_), j),
            sel9(PK9(P_(0), P_(2), P_(5), P_(6), P_(8), P_(11), Z_, Z_, Z_), j), bit9(0x009u, j), bit9(0x012u, j));
    fp2_cneg(o, o, j >= 3);                            // r1 = -(c1 d^-1)
    if (j < 6) R = o;
}
// all six coefficients equal those of 1 (wave ballot over the group's lanes 0..5)
DI bool cp_is_one(const fp2 &R, const Cp &c) {
    fp2 e = cpj(c) == 0 ? fp2_one() : fp2_zero();
    const bool bad = cpj(c) < 6 && !fp2_eq(R, e);
    const u64c m = __ballot(bad);
    return ((m >> (CP_L * c.g)) & 0x3f) == 0;
}

// ---------------------------------------------------------------- final exponentiation (pairing.hpp fe_easy + fe_hard)
// A program of Fp12 operations on R and the park slots X 0, T 1, U 2, V 3, ACC 4 (slot 0 holds f on entry), run by one
// loop so each operation's code exists once (the inlined sequence took 512 registers and spilled).  Same exponent,
// products and order as fe_easy + fe_hard.
enum { FE_LD = 0, FE_ST, FE_CJ, FE_CS, FE_MU, FE_MC, FE_FR, FE_IV };
struct FeProg {
    unsigned char op[512];
    int n;
};
constexpr FeProg fe_program() {
    FeProg p{};
    int n = 0;
    auto e = [&](int kind, int s) { p.op[n++] = (unsigned char)(kind | s << 4); };
    auto pow_z = [&](int base) {               // R <- R^z, R unitary and parked at base
        for (int b = 62; b >= 0; b--) {
            e(FE_CS, 0);
            if ((LCB_Z_ABS >> b) & 1) e(FE_MU, base);
        }
        e(FE_CJ, 0);
    };
    // easy part: m = (conj(f) f^-1)^(p^2 + 1)
    e(FE_LD, 0); e(FE_IV, 0); e(FE_ST, 1); e(FE_LD, 0); e(FE_MC, 1); e(FE_ST, 2); e(FE_FR, 2); e(FE_MU, 2);
    // hard part
    e(FE_ST, 0);                                // x
    pow_z(0); e(FE_ST, 1);                      // t = x^z
    e(FE_LD, 0); e(FE_CJ, 0); e(FE_CS, 0); e(FE_MU, 1); e(FE_ST, 2);      // u = x^(z-2)
    pow_z(2); e(FE_ST, 3);                      // v = x^(z^2-2z)
    e(FE_MU, 0); e(FE_FR, 3); e(FE_ST, 4);      // acc = (v x)^(p^3)
    e(FE_LD, 3); pow_z(3); e(FE_ST, 3);         // v = x^(z^3-2z^2)
    e(FE_MU, 1); e(FE_FR, 2); e(FE_MU, 4); e(FE_ST, 4);                   // acc *= (v t)^(p^2)
    e(FE_LD, 3); pow_z(3); e(FE_ST, 3);         // v = x^(z^4-2z^3)
    e(FE_LD, 1); e(FE_CS, 0); e(FE_ST, 1);      // t = x^2z
    e(FE_LD, 3); e(FE_MU, 1); e(FE_ST, 3);      // v = x^(z^4-2z^3+2z)
    e(FE_LD, 0); e(FE_MC, 3); e(FE_FR, 1); e(FE_MU, 4); e(FE_ST, 4);      // acc *= (x^-1 v)^p
    e(FE_LD, 3); pow_z(3); e(FE_ST, 3);         // v = x^(z^5-2z^4+2z^2)
    e(FE_LD, 2); e(FE_MC, 3); e(FE_MU, 0); e(FE_MU, 4);                   // y = acc x^(2-z) v x
    p.n = n;
    return p;
}
__constant__ FeProg LCB_FE_PROG = fe_program();
DI u32 *fe_slot(u32 *park, size_t n, int s) { return park + (size_t)144 * n * s; }
// R <- f^((p^12 - 1) / r) (x3, mcl's normalisation) for f in park slot 0 of item i; live = the item exists.  A parked
// value is read by other lanes only inside a later cp_mul12, after its first __syncthreads.
DI void cp_final_exp(fp2 &R, const Cp &c, u32 *park, size_t n, size_t i, bool live) {
    const int np = LCB_FE_PROG.n;
#pragma unroll 1
    for (int pc = 0; pc < np; pc++) {
        const int op = LCB_FE_PROG.op[pc], kind = op & 15, s = op >> 4;
        u32 *slot = fe_slot(park, n, s);
        if (kind == FE_LD) park_get(R, slot, n, i, cpj(c));
        else if (kind == FE_ST) park_put(slot, n, i, cpj(c), live, R);
        else if (kind == FE_CJ) cp_conj(R, c);
        else if (kind == FE_CS) cp_cyc_sqr(R, c);
        else if (kind == FE_MU || kind == FE_MC) cp_mul12(R, c, kind == FE_MC, slot, n, i);
        else if (kind == FE_FR) cp_frob(R, c, s);
        else cp_inv(R, c);
    }
}
// accept[i] &= (final_exp(f_i) == 1) for f_i in park slot 0, slot 0 <- the GT value (k_coop_final_exp_check, and the
// census copy in k_prep.hip at 256 registers); lds = the wave's CP_LDS_QUADS
DI void cp_final_exp_check_run(uint4 *lds, u32 *park, u32 n, uint8_t *accept) {
    const Cp c = cp_init(lds);
    const u32 item = blockIdx.x * CP_G + c.g;
    const bool live = c.g < CP_G && item < n;
    const size_t it = live ? item : 0;
    if (cpj(c) == 0) cp_put(c, S_Z, fp2_zero());
    cp_sync();
    fp2 R;
    cp_final_exp(R, c, park, n, it, live);
    const bool one = cp_is_one(R, c);
    park_put(park, n, it, cpj(c), live, R);
    if (live && cpj(c) == 0 && accept) accept[item] = accept[item] && one;
}
