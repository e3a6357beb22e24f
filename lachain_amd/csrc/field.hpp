// lachain_amd/csrc/field.hpp — BLS12-381 field tower on gfx950 (device code).
//
// Fp : 12 x 32-bit limbs, Montgomery form (R = 2^384), always fully reduced to [0, p).
// Fr : 8 x 32-bit limbs, Montgomery form (R = 2^256), fully reduced.
// Fp2 = Fp[i]/(i^2 + 1), Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v), xi = 1 + i: the herumi mcl
// tower that Lachain reaches through MCL.BLS12_381.Native.
//
// Register / code-size strategy: one field element per lane, all state in VGPRs.
// The Montgomery multiply is the only non-inlined leaf (`lcb_fp_mul_v`): it takes/returns vector
// types so the AMDGPU calling convention keeps operands in v0..v23 (aggregates >16 registers would be
// passed through scratch), and it needs < 40 VGPRs, so it clobbers no callee-saved registers.  Every
// Fp2/Fp6/Fp12 routine is inlined around those calls, which keeps the hot loops' code in the I-cache.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bls_constants.hpp"
#include "asm_routines.hpp"

typedef uint32_t u32;
typedef uint64_t u64;
typedef u32 u32x12 __attribute__((ext_vector_type(12)));
typedef u32 u32x8 __attribute__((ext_vector_type(8)));

#define DI __device__ __forceinline__
#define DN __device__ __noinline__

struct fp { u32 v[12]; };
struct fp2 { fp a, b; };
struct fp6 { fp2 c0, c1, c2; };
struct fp12 { fp6 c0, c1; };
struct fr { u32 v[8]; };

// ------------------------------------------------------------------------------------------------ Fp
DI void fp_load_const(fp &r, const u32 *c) {
#pragma unroll
    for (int j = 0; j < 12; j++) r.v[j] = c[j];
}
DI fp fp_zero() { fp r; for (int j = 0; j < 12; j++) r.v[j] = 0; return r; }
DI fp fp_one() { fp r; fp_load_const(r, LCB_ONE); return r; }
DI bool fp_is_zero(const fp &a) {
    u32 x = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) x |= a.v[j];
    return x == 0;
}
DI bool fp_eq(const fp &a, const fp &b) {
    u32 x = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) x |= a.v[j] ^ b.v[j];
    return x == 0;
}
// r = (t >= p) ? t - p : t, for t < 2p
DI void fp_reduce_once(fp &r, const fp &t) {
    u32 d[12];
    u32 br = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
        u64 x = (u64)t.v[j] - LCB_P[j] - br;
        d[j] = (u32)x;
        br = (u32)(x >> 32) & 1;
    }
#pragma unroll
    for (int j = 0; j < 12; j++) r.v[j] = br ? t.v[j] : d[j];
}
DI void fp_add_c(fp &r, const fp &a, const fp &b) {
    fp t;
    u32 c = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
        u64 s = (u64)a.v[j] + b.v[j] + c;
        t.v[j] = (u32)s;
        c = (u32)(s >> 32);
    }
    fp_reduce_once(r, t); // a + b < 2p < 2^382: no carry out of limb 11
}
DI void fp_sub_c(fp &r, const fp &a, const fp &b) {
    fp t;
    u32 br = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
        u64 x = (u64)a.v[j] - b.v[j] - br;
        t.v[j] = (u32)x;
        br = (u32)(x >> 32) & 1;
    }
    fp d;
    u32 c = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
        u64 s = (u64)t.v[j] + LCB_P[j] + c;
        d.v[j] = (u32)s;
        c = (u32)(s >> 32);
    }
#pragma unroll
    for (int j = 0; j < 12; j++) r.v[j] = br ? d.v[j] : t.v[j];
}
DI void fp_neg_c(fp &r, const fp &a) {
    fp z = fp_zero();
    fp_sub_c(r, z, a);
}
DI void fp_add(fp &r, const fp &a, const fp &b) { lcb_fp_add_asm(r.v, a.v, b.v); }  // 36-instruction VCC chain
// r = a + b without reduction (< 2p): only as a Montgomery multiplicand (R > 4p)
DI void fp_add_nr(fp &r, const fp &a, const fp &b) { lcb_fp_add_nr_asm(r.v, a.v, b.v); }
DI void fp_dbl(fp &r, const fp &a) { fp_add(r, a, a); }
DI void fp_sub(fp &r, const fp &a, const fp &b) { lcb_fp_sub_asm(r.v, a.v, b.v); }
DI void fp_neg(fp &r, const fp &a) { lcb_fp_neg_asm(r.v, a.v); }

DI u32x12 fp_to_v(const fp &a) {
    u32x12 v;
#pragma unroll
    for (int j = 0; j < 12; j++) v[j] = a.v[j];
    return v;
}
DI fp fp_from_v(const u32x12 &v) {
    fp a;
#pragma unroll
    for (int j = 0; j < 12; j++) a.v[j] = v[j];
    return a;
}
DI void fp_mul(fp &r, const fp &a, const fp &b) { r = fp_from_v(lcb_asm_fp_mul(fp_to_v(a), fp_to_v(b))); }
// dedicated Montgomery square (tools/gen_asm.py lcb_r_fp_sqr: 78 + 144 products, 551 instructions against 662)
DI void fp_sqr(fp &r, const fp &a) { r = fp_from_v(lcb_asm_fp_sqr(fp_to_v(a))); }
#define LCB_POW_SQR(x) lcb_asm_fp_sqr(x)

// conversions between canonical integers (12 LE limbs) and Montgomery form
DI void fp_from_raw(fp &r, const fp &raw) {
    fp r2;
    fp_load_const(r2, LCB_R2);
    fp_mul(r, raw, r2);
}
DI void fp_to_raw(fp &r, const fp &a) {
    fp one = fp_zero();
    one.v[0] = 1;
    fp_mul(r, a, one);
}
DI bool fp_raw_lt_p(const fp &raw) {
    u32 br = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
        u64 x = (u64)raw.v[j] - LCB_P[j] - br;
        br = (u32)(x >> 32) & 1;
    }
    return br != 0;
}
DI bool fp_is_odd(const fp &a) {
    fp t;
    fp_to_raw(t, a);
    return t.v[0] & 1;
}
// a^e for an exponent given as 12 LE limbs in constant memory.  The exponent bits are wave-uniform, so no
// branch diverges.  Non-inlined, operands in VGPRs.
// left-to-right sliding window of width 4 over the odd powers a, a^3, ..., a^15 (8 precomputation products):
// ~381 squarings + ~76 window products instead of ~190 for p - 2, (p + 1)/4 and (p - 1)/2.  The table is
// selected by a uniform switch over named registers, never by a dynamic register index (that would go to scratch).
DI u32x12 lcb_fp_pow_sel(int k, const u32x12 &t1, const u32x12 &t3, const u32x12 &t5, const u32x12 &t7,
                         const u32x12 &t9, const u32x12 &t11, const u32x12 &t13, const u32x12 &t15) {
    switch (k) {
    case 1: return t1;
    case 3: return t3;
    case 5: return t5;
    case 7: return t7;
    case 9: return t9;
    case 11: return t11;
    case 13: return t13;
    default: return t15;
    }
}
// which: 0 = p - 2, 1 = (p + 1)/4, 2 = (p - 1)/2, 3 = (p - 3)/4, made wave-uniform (readfirstlane).
// Round 6: the generated routine lcb_r_fp_pow (tools/gen_asm.py) runs the same windows with the table t1..t15 in
// VGPRs above the leaf routines' clobbers.  The compiled loop below (LCB_FP_POW_COMPILED=1) kept the table in scratch
// and reloaded 48 B per window, ~4.6 KB of scratch reads per exponentiation: most of the HBM traffic of every
// decompression lane.  A call (not inlined): the routine clobbers only the ABI's caller-saved registers beyond the
// leaf routines' own, so its callers see an ordinary call.
#ifndef LCB_FP_POW_COMPILED
#define LCB_FP_POW_COMPILED 0
#endif
#if !LCB_FP_POW_COMPILED
DN u32x12 lcb_fp_pow_v(u32x12 av, int which) {
    return lcb_asm_fp_pow(av, __builtin_amdgcn_readfirstlane(which));
}
#else
// the compiled form: the exponent words come through the scalar cache and every bit test is a scalar branch
DN u32x12 lcb_fp_pow_v(u32x12 av, int which) {
    which = __builtin_amdgcn_readfirstlane(which);
    const u32 *e = which == 0 ? LCB_P_MINUS_2 : which == 1 ? LCB_P_PLUS1_DIV4 : which == 2 ? LCB_P_MINUS1_DIV2
                                                                                          : LCB_P_MINUS3_DIV4;
    int top = 383;
    while (top > 0 && !((e[top >> 5] >> (top & 31)) & 1)) top--;
    u32x12 a2 = lcb_asm_fp_mul(av, av);
    u32x12 t1 = av;
    u32x12 t3 = lcb_asm_fp_mul(t1, a2);
    u32x12 t5 = lcb_asm_fp_mul(t3, a2);
    u32x12 t7 = lcb_asm_fp_mul(t5, a2);
    u32x12 t9 = lcb_asm_fp_mul(t7, a2);
    u32x12 t11 = lcb_asm_fp_mul(t9, a2);
    u32x12 t13 = lcb_asm_fp_mul(t11, a2);
    u32x12 t15 = lcb_asm_fp_mul(t13, a2);
    u32x12 acc = av;
    bool first = true;
    int i = top;
    while (i >= 0) {
        if (!((e[i >> 5] >> (i & 31)) & 1)) {
            acc = LCB_POW_SQR(acc);
            i--;
            continue;
        }
        int j = i - 3 > 0 ? i - 3 : 0;
        while (!((e[j >> 5] >> (j & 31)) & 1)) j++;  // the window i..j ends in a set bit
        int w = 0;
        for (int b = i; b >= j; b--) w = (w << 1) | (int)((e[b >> 5] >> (b & 31)) & 1);
        if (first) {
            acc = lcb_fp_pow_sel(w, t1, t3, t5, t7, t9, t11, t13, t15);
            first = false;
        } else {
            for (int b = i; b >= j; b--) acc = LCB_POW_SQR(acc);
            acc = lcb_asm_fp_mul(acc, lcb_fp_pow_sel(w, t1, t3, t5, t7, t9, t11, t13, t15));
        }
        i = j - 1;
    }
    return acc;
}
#endif
DI void fp_pow_const(fp &r, const fp &a, int which) { r = fp_from_v(lcb_fp_pow_v(fp_to_v(a), which)); }
DI void fp_inv(fp &r, const fp &a) { fp_pow_const(r, a, 0); }   // a^(p-2): 463 products

// ---- inversion by binary GCD (Pornin, "Optimized Binary GCD for Modular Inversion", eprint 2020/972): 26 outer
// iterations; each runs 30 divsteps on 62-bit approximations of a, b (the low 30 bits and the top 32 bits of the
// longer one) to get a 2 x 2 matrix of signed coefficients (|f|, |g| <= 2^30), then applies it to the full a, b
// (exact: the low 30 bits of the combinations are zero) and to the coefficients u, v with one 32-bit Montgomery
// reduction modulo p.  From a = X, b = p, u = 1, v = 0 the loop ends with b = 1 and v = X^-1 2^(26 (30 - 32)), so one
// Montgomery product by LCB_BINV_C = 2^52 R^3 gives the Montgomery form of x^-1 for X = x R (0 -> 0, as a^(p-2)).
// About 40 K instructions against the exponentiation's 263 K; the same canonical result.  A call (not inlined): its
// ~150 live registers would otherwise add to the caller's.  Used where the caller's state around the call is small —
// every Fp2 / Fp6 / Fp12 inversion (line-set normalisation, hash-to-G2, the final exponentiation's easy part) and the
// key tables; the G1 affine conversions of the group sums and the nine-lane kernels keep fp_inv (the exponentiation
// routine's narrow calling convention), where the call measured spills.
DI void fpi_mul32(u32 (&r)[13], const u32 (&x)[12], u32 m) {           // r = x m (13 limbs)
    u64 c = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
        u64 t = (u64)x[j] * m + c;
        r[j] = (u32)t;
        c = t >> 32;
    }
    r[12] = (u32)c;
}
DI void fpi_cneg13(u32 (&r)[13], bool neg) {                           // two's complement negation if neg
    const u32 m = neg ? 0xffffffffu : 0u;
    u64 c = neg ? 1u : 0u;
#pragma unroll
    for (int j = 0; j < 13; j++) {
        u64 t = (u64)(r[j] ^ m) + c;
        r[j] = (u32)t;
        c = t >> 32;
    }
}
DI void fpi_add13(u32 (&r)[13], const u32 (&x)[13]) {
    u64 c = 0;
#pragma unroll
    for (int j = 0; j < 13; j++) {
        u64 t = (u64)r[j] + x[j] + c;
        r[j] = (u32)t;
        c = t >> 32;
    }
}
// t = x f + y g as 13-limb two's complement (x, y < 2^384 unsigned, |f|, |g| <= 2^30)
DI void fpi_lin(u32 (&t)[13], const u32 (&x)[12], const u32 (&y)[12], int f, int g) {
    u32 t2[13];
    fpi_mul32(t, x, (u32)(f < 0 ? -f : f));
    fpi_cneg13(t, f < 0);
    fpi_mul32(t2, y, (u32)(g < 0 ? -g : g));
    fpi_cneg13(t2, g < 0);
    fpi_add13(t, t2);
}
// r = |x f + y g| >> 30; returns true when x f + y g < 0
DI bool fpi_lin_shift(u32 (&r)[12], const u32 (&x)[12], const u32 (&y)[12], int f, int g) {
    u32 t[13];
    fpi_lin(t, x, y, f, g);
#pragma unroll
    for (int j = 0; j < 12; j++) t[j] = (t[j] >> 30) | (t[j + 1] << 2);
    t[12] = (u32)((int)t[12] >> 30);
    const bool neg = (int)t[12] < 0;
    fpi_cneg13(t, neg);
#pragma unroll
    for (int j = 0; j < 12; j++) r[j] = t[j];
    return neg;
}
// r = (x f + y g) 2^-32 mod p in [0, p) (x, y in [0, p))
DI void fpi_mont_lin(u32 (&r)[12], const u32 (&x)[12], const u32 (&y)[12], int f, int g) {
    u32 t[13], qp[13];
    fpi_lin(t, x, y, f, g);
    const u32 q = t[0] * LCB_P_INV;                   // t + q p = 0 mod 2^32
    u32 pl[12];
#pragma unroll
    for (int j = 0; j < 12; j++) pl[j] = LCB_P[j];
    fpi_mul32(qp, pl, q);
    fpi_add13(t, qp);                                 // |t| < 2^33 p < 2^415: no overflow of 13 signed limbs
    // t / 2^32 (t[0] == 0): limbs 1..12, sign in t[12]; the value lies in (-p/2, 3p/2)
    u32 s[12], d[12];
    const bool neg = (int)t[12] < 0;
#pragma unroll
    for (int j = 0; j < 12; j++) s[j] = t[j + 1];     // two's complement low 384 bits of t / 2^32
    // neg: s + p (the true value + p is in [0, p)); else s - p if s >= p
    u64 c = 0;
    u32 br = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
        if (neg) {
            u64 x2 = (u64)s[j] + LCB_P[j] + c;
            d[j] = (u32)x2;
            c = x2 >> 32;
        } else {
            u64 x2 = (u64)s[j] - LCB_P[j] - br;
            d[j] = (u32)x2;
            br = (u32)(x2 >> 32) & 1;
        }
    }
    const bool take = neg || !br;                      // s + p, or s - p when s >= p
#pragma unroll
    for (int j = 0; j < 12; j++) r[j] = take ? d[j] : s[j];
}
// the top 32 bits of x below bit position s + 32 (x < 2^384, 30 <= s <= 352), i.e. bits s .. s + 31
DI u32 fpi_bits32(const u32 (&x)[12], u32 li, u32 o) {
    u32 lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
        lo = (u32)j == li ? x[j] : lo;
        hi = (u32)j == li + 1 ? x[j] : hi;
    }
    return o ? (lo >> o) | (hi << (32 - o)) : lo;
}
DN void fp_inv_gcd(fp &r, const fp &x) {
    u32 a[12], b[12], u[12], v[12];
#pragma unroll
    for (int j = 0; j < 12; j++) {
        a[j] = x.v[j];
        b[j] = LCB_P[j];
        u[j] = j == 0 ? 1u : 0u;
        v[j] = 0u;
    }
#pragma unroll 1
    for (int it = 0; it < 26; it++) {
        // approximations: the low 30 bits and bits n - 32 .. n - 1 of a, b, n = max(bit length of a | b, 62)
        u32 hiw = 0, top = 0;
#pragma unroll
        for (int j = 0; j < 12; j++) {
            const u32 w = a[j] | b[j];
            hiw = w ? (u32)j : hiw;
            top = w ? w : top;
        }
        u32 n = 32 * hiw + (32 - (u32)__clz(top | 1));
        n = n < 62 ? 62 : n;
        const u32 s = n - 32, li = s >> 5, o = s & 31;
        u64 ab = ((u64)fpi_bits32(a, li, o) << 30) | (a[0] & 0x3fffffffu);
        u64 bb = ((u64)fpi_bits32(b, li, o) << 30) | (b[0] & 0x3fffffffu);
        int f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#pragma unroll 2
        for (int i = 0; i < 30; i++) {
            const bool odd = ab & 1;
            const bool sw = odd && ab < bb;
            const u64 ta = sw ? bb : ab, tb = sw ? ab : bb;
            const int tf0 = sw ? f1 : f0, tg0 = sw ? g1 : g0, tf1 = sw ? f0 : f1, tg1 = sw ? g0 : g1;
            ab = (odd ? ta - tb : ta) >> 1;
            bb = tb;
            f0 = odd ? tf0 - tf1 : tf0;
            g0 = odd ? tg0 - tg1 : tg0;
            f1 = tf1 * 2;
            g1 = tg1 * 2;
        }
        u32 na[12], nb[12], nu[12], nv[12];
        if (fpi_lin_shift(na, a, b, f0, g0)) { f0 = -f0; g0 = -g0; }
        if (fpi_lin_shift(nb, a, b, f1, g1)) { f1 = -f1; g1 = -g1; }
        fpi_mont_lin(nu, u, v, f0, g0);
        fpi_mont_lin(nv, u, v, f1, g1);
#pragma unroll
        for (int j = 0; j < 12; j++) {
            a[j] = na[j];
            b[j] = nb[j];
            u[j] = nu[j];
            v[j] = nv[j];
        }
    }
    fp vv, c;
#pragma unroll
    for (int j = 0; j < 12; j++) vv.v[j] = v[j];
    fp_load_const(c, LCB_BINV_C);
    fp_mul(r, vv, c);
    if (fp_is_zero(x)) r = fp_zero();
}
// Legendre symbol (x / p) by the binary Jacobi-symbol algorithm, on the Montgomery words (x R / p = x / p: R = 2^384 is
// a square): a = xR, b = p; strip factors 2 from a ((2 / b) = -1 for b = 3, 5 mod 8), swap when a < b (reciprocity: -1
// when both are 3 mod 4), a -= b; at a = 0, b = gcd = 1 unless x = 0.  About 500 subtract-and-shift steps of ~120
// instructions against the exponentiation's 263 K (fp_legendre below); the step count depends on x (a wave runs its
// lanes' longest), which is public here: the candidates of hash-to-G2.  Returns 1, -1, or 0 for x = 0.
DN int fp_jacobi(const fp &x) {
    u32 a[12], b[12];
#pragma unroll
    for (int j = 0; j < 12; j++) {
        a[j] = x.v[j];
        b[j] = LCB_P[j];
    }
    u32 neg = 0;
#pragma unroll 1
    for (;;) {
        u32 any = 0;
#pragma unroll
        for (int j = 0; j < 12; j++) any |= a[j];
        if (!any) break;
#pragma unroll 1
        while (a[0] == 0) {                            // a zero word: 2^32 is a square, the sign stays
#pragma unroll
            for (int j = 0; j < 11; j++) a[j] = a[j + 1];
            a[11] = 0;
        }
        const u32 t = (u32)__builtin_ctz(a[0]);
        if (t) {
#pragma unroll
            for (int j = 0; j < 11; j++) a[j] = __builtin_amdgcn_alignbit(a[j + 1], a[j], t);
            a[11] >>= t;
            const u32 b8 = b[0] & 7u;
            if ((t & 1u) && (b8 == 3u || b8 == 5u)) neg ^= 1u;
        }
        u32 d[12], br = 0;                             // a odd: d = a - b
#pragma unroll
        for (int j = 0; j < 12; j++) {
            const u64 w = (u64)a[j] - b[j] - br;
            d[j] = (u32)w;
            br = (u32)(w >> 32) & 1u;
        }
        if (br) {                                      // a < b: (a, b) <- (b - a, a)
            if ((a[0] & 3u) == 3u && (b[0] & 3u) == 3u) neg ^= 1u;
            u32 c = 1;
#pragma unroll
            for (int j = 0; j < 12; j++) {
                const u64 w = (u64)(~d[j]) + c;
                b[j] = a[j];
                a[j] = (u32)w;
                c = (u32)(w >> 32);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 12; j++) a[j] = d[j];
        }
    }
    u32 one = b[0] == 1u;
#pragma unroll
    for (int j = 1; j < 12; j++) one &= b[j] == 0u;
    return one ? (neg ? -1 : 1) : 0;
}
// mcl Fp::squareRoot for p = 3 mod 4: y = a^((p+1)/4), valid iff y^2 == a
DI bool fp_sqrt(fp &r, const fp &a) {
    fp y, t;
    fp_pow_const(y, a, 1);
    fp_sqr(t, y);
    bool ok = fp_eq(t, a); // compare before writing r: callers pass r aliasing a
    r = y;
    return ok;
}
#ifndef LCB_JACOBI
#define LCB_JACOBI 1
#endif
DI int fp_legendre(const fp &a) {
#if LCB_JACOBI
    return fp_jacobi(a);
#else
    if (fp_is_zero(a)) return 0;
    fp t;
    fp_pow_const(t, a, 2);
    return fp_eq(t, fp_one()) ? 1 : -1;
#endif
}

// ------------------------------------------------------------------------------------------------ Fp2
// both components in one interleaved pair of carry chains (asm_routines.hpp, tools/gen_asm.py)
DI void fp2_add(fp2 &r, const fp2 &x, const fp2 &y) { lcb_fp2_add_asm(r.a.v, r.b.v, x.a.v, x.b.v, y.a.v, y.b.v); }
DI void fp2_sub(fp2 &r, const fp2 &x, const fp2 &y) { lcb_fp2_sub_asm(r.a.v, r.b.v, x.a.v, x.b.v, y.a.v, y.b.v); }
DI void fp2_dbl(fp2 &r, const fp2 &x) { lcb_fp2_add_asm(r.a.v, r.b.v, x.a.v, x.b.v, x.a.v, x.b.v); }
DI void fp2_neg(fp2 &r, const fp2 &x) { lcb_fp2_neg_asm(r.a.v, r.b.v, x.a.v, x.b.v); }
DI void fp2_conj(fp2 &r, const fp2 &x) { r.a = x.a; fp_neg(r.b, x.b); }
DI bool fp2_is_zero(const fp2 &x) { return fp_is_zero(x.a) && fp_is_zero(x.b); }
DI bool fp2_eq(const fp2 &x, const fp2 &y) { return fp_eq(x.a, y.a) && fp_eq(x.b, y.b); }
DI fp2 fp2_zero() { fp2 r; r.a = fp_zero(); r.b = fp_zero(); return r; }
DI fp2 fp2_one() { fp2 r; r.a = fp_one(); r.b = fp_zero(); return r; }
DI void fp2_load_const(fp2 &r, const u32 *c) { fp_load_const(r.a, c); fp_load_const(r.b, c + 12); }
// Fp2 products go to the hand-scheduled assembly routines (tools/gen_asm.py): 3 (mul) or 2 (sqr, mul_fp)
// independent Montgomery chains interleaved in one call.
DI void fp2_mul(fp2 &r, const fp2 &x, const fp2 &y) {
    u32x12 xa = fp_to_v(x.a), xb = fp_to_v(x.b);
    lcb_asm_fp2_mul(xa, xb, fp_to_v(y.a), fp_to_v(y.b));
    r.a = fp_from_v(xa);
    r.b = fp_from_v(xb);
}
DI void fp2_sqr(fp2 &r, const fp2 &x) {
    u32x12 xa = fp_to_v(x.a), xb = fp_to_v(x.b);
    lcb_asm_fp2_sqr(xa, xb);
    r.a = fp_from_v(xa);
    r.b = fp_from_v(xb);
}
DI void fp2_mul_fp(fp2 &r, const fp2 &x, const fp &s) {
    u32x12 xa = fp_to_v(x.a), xb = fp_to_v(x.b);
    lcb_asm_fp2_mul_fp(xa, xb, fp_to_v(s));
    r.a = fp_from_v(xa);
    r.b = fp_from_v(xb);
}
// two independent Fp products in one call
DI void fp_mul2(fp &r0, const fp &a0, const fp &b0, fp &r1, const fp &a1, const fp &b1) {
    u32x12 x0 = fp_to_v(a0), x1 = fp_to_v(a1);
    lcb_asm_fp_mul2(x0, fp_to_v(b0), x1, fp_to_v(b1));
    r0 = fp_from_v(x0);
    r1 = fp_from_v(x1);
}
DI void fp2_mul_xi(fp2 &r, const fp2 &x) { // (a + b i)(1 + i) = (a - b) + (a + b) i
    lcb_fp2_mul_xi_asm(r.a.v, r.b.v, x.a.v, x.b.v);
}
DI void fp2_norm(fp &r, const fp2 &x) {
    fp t, u;
    fp_mul2(u, x.a, x.a, t, x.b, x.b);
    fp_add(r, u, t);
}
DI void fp2_inv(fp2 &r, const fp2 &x) {
    fp n;
    fp2_norm(n, x);
    fp_inv(n, n);
    fp2 t;
    fp2_mul_fp(t, x, n);
    r.a = t.a;
    fp_neg(r.b, t.b);
}
// the same with the binary-GCD Fp inversion (fp_inv_gcd: its call is cheap where few values are live around it)
DI void fp2_inv_g(fp2 &r, const fp2 &x) {
    fp n;
    fp2_norm(n, x);
    fp_inv_gcd(n, n);
    fp2 t;
    fp2_mul_fp(t, x, n);
    r.a = t.a;
    fp_neg(r.b, t.b);
}
// mcl Fp2T::squareRoot (norm method; root choice reproduced exactly): t = sqrt(a^2 + b^2), then the
// root of c = (a + t)/2, else of (a - t)/2, as y.a, and y.b = b / (2 y.a).  mcl takes that root and inverts it with two
// exponentiations; here one gives both: s = c^((p-3)/4), c s = c^((p+1)/4) (mcl's root) and, when c is a square
// (c s^2 = c^((p-1)/2) = 1, Euler's criterion — mcl's check y.a^2 == c), 1/(c s) = s.  For b != 0, c != 0 (c = 0 would
// need t = -a, so b = 0), so the two tests agree and every output is the same field element.
DI bool fp2_sqrt(fp2 &y, const fp2 &x) {
    fp t1, t2, inv2;
    fp_load_const(inv2, LCB_INV2);
    if (fp_is_zero(x.b)) {
        if (fp_sqrt(t1, x.a)) {
            y.a = t1;
            y.b = fp_zero();
        } else {
            fp na;
            fp_neg(na, x.a);
            if (!fp_sqrt(t1, na)) return false;
            y.a = fp_zero();
            y.b = t1;
        }
        return true;
    }
    fp_sqr(t1, x.a);
    fp_sqr(t2, x.b);
    fp_add(t1, t1, t2);
    if (!fp_sqrt(t1, t1)) return false;
#pragma unroll 1
    for (int k = 0; k < 2; k++) {
        fp c, s, cs, e;
        if (k == 0) fp_add(c, x.a, t1);
        else fp_sub(c, x.a, t1);
        fp_mul(c, c, inv2);
        fp_pow_const(s, c, 3);
        fp_mul(cs, c, s);                              // c^((p+1)/4)
        fp_mul(e, cs, s);                              // c^((p-1)/2)
        if (fp_eq(e, fp_one())) {
            y.a = cs;
            fp_mul(t2, x.b, s);
            fp_mul(y.b, t2, inv2);                     // b / (2 c^((p+1)/4)) = b s / 2
            return true;
        }
    }
    return false;
}
// fp2_sqrt for an x whose norm N(x) = a^2 + b^2 the caller has already found square, with nr = N(x)^((p+1)/4) (fp_sqrt's
// root of the norm): the same root as fp2_sqrt(x) (its x.b == 0 branch included)
DI void fp2_sqrt_normed(fp2 &y, const fp2 &x, const fp &nr) {
    if (fp_is_zero(x.b)) { (void)fp2_sqrt(y, x); return; }
    fp inv2;
    fp_load_const(inv2, LCB_INV2);
#if LCB_JACOBI
    {   // fp2_sqrt's two tries, c = (a + nr)/2 first: the first one that is a nonzero square, chosen by its Legendre
        // symbol, then ONE exponentiation (the loop below ran the second for the wave whenever one lane needed it)
        fp c, s, cs, e, t2;
        fp_add(c, x.a, nr);
        fp_mul(c, c, inv2);
        if (fp_jacobi(c) != 1) {
            fp_sub(c, x.a, nr);
            fp_mul(c, c, inv2);
        }
        fp_pow_const(s, c, 3);
        fp_mul(cs, c, s);                              // c^((p+1)/4)
        fp_mul(e, cs, s);                              // c^((p-1)/2)
        if (fp_eq(e, fp_one())) {
            y.a = cs;
            fp_mul(t2, x.b, s);
            fp_mul(y.b, t2, inv2);                     // b / (2 c^((p+1)/4)) = b s / 2
        }
        return;
    }
#endif
#pragma unroll 1
    for (int k = 0; k < 2; k++) {
        fp c, s, cs, e, t2;
        if (k == 0) fp_add(c, x.a, nr);
        else fp_sub(c, x.a, nr);
        fp_mul(c, c, inv2);
        fp_pow_const(s, c, 3);
        fp_mul(cs, c, s);                              // c^((p+1)/4)
        fp_mul(e, cs, s);                              // c^((p-1)/2)
        if (fp_eq(e, fp_one())) {
            y.a = cs;
            fp_mul(t2, x.b, s);
            fp_mul(y.b, t2, inv2);                     // b / (2 c^((p+1)/4)) = b s / 2
            return;
        }
    }
}
// A square root of x in Fp2 when the caller fixes the sign itself (G2 decompression): two exponentiations instead
// of fp2_sqrt's four per wave (its second Fp root runs whenever one lane needs it, and it ends in an inversion).
// With t = sqrt(a^2 + b^2), c = (a + t)/2 and s = c^((p-3)/4): if c is a square, y = (c s, b s / 2) (c s = c^((p+1)/4)
// and 1/(c s) = s since c s^2 = 1); otherwise d = (a - t)/2 = -b^2/(4c) is one, s^2 = -1/c and y = (b s / 2, -c s).
// The root may differ in sign from fp2_sqrt's; the result is checked (y^2 == x) before it is returned.
DI bool fp2_sqrt_any(fp2 &y, const fp2 &x) {
    if (fp_is_zero(x.b)) return fp2_sqrt(y, x);
    fp t, c, s, u, inv2, bs;
    fp_load_const(inv2, LCB_INV2);
    fp_sqr(t, x.a);
    fp_sqr(u, x.b);
    fp_add(t, t, u);
    if (!fp_sqrt(t, t)) return false;                  // N(x) is a square iff x is
    fp_add(c, x.a, t);
    fp_mul(c, c, inv2);
    fp_pow_const(s, c, 3);
    fp_sqr(u, s);
    fp_mul(u, u, c);                                   // c^((p-1)/2) = +-1
    fp_mul(bs, x.b, s);
    fp_mul(bs, bs, inv2);                              // b s / 2
    fp cs;
    fp_mul(cs, c, s);
    fp2 r;
    if (fp_eq(u, fp_one())) {
        r.a = cs;
        r.b = bs;
    } else {
        r.a = bs;
        fp_neg(r.b, cs);
    }
    fp2 chk;
    fp2_sqr(chk, r);
    if (!(fp_eq(chk.a, x.a) && fp_eq(chk.b, x.b))) return false;
    y = r;
    return true;
}

// ------------------------------------------------------------------------------------------------ Fp6
// (three interleaved carry chains per Fp6 addition measured 2 % slower in k_tpke_miller: more spills)
DI void fp6_add(fp6 &r, const fp6 &x, const fp6 &y) { fp2_add(r.c0, x.c0, y.c0); fp2_add(r.c1, x.c1, y.c1); fp2_add(r.c2, x.c2, y.c2); }
DI void fp6_sub(fp6 &r, const fp6 &x, const fp6 &y) { fp2_sub(r.c0, x.c0, y.c0); fp2_sub(r.c1, x.c1, y.c1); fp2_sub(r.c2, x.c2, y.c2); }
DI void fp6_neg(fp6 &r, const fp6 &x) { fp2_neg(r.c0, x.c0); fp2_neg(r.c1, x.c1); fp2_neg(r.c2, x.c2); }
DI void fp6_mul(fp6 &r, const fp6 &a, const fp6 &b) {
    fp2 t0, t1, t2, s0, s1, c0, c1, c2;
    fp2_mul(t0, a.c0, b.c0);
    fp2_mul(t1, a.c1, b.c1);
    fp2_mul(t2, a.c2, b.c2);
    fp2_add(s0, a.c1, a.c2);
    fp2_add(s1, b.c1, b.c2);
    fp2_mul(c0, s0, s1);
    fp2_sub(c0, c0, t1);
    fp2_sub(c0, c0, t2);
    fp2_mul_xi(c0, c0);
    fp2_add(c0, c0, t0);
    fp2_add(s0, a.c0, a.c1);
    fp2_add(s1, b.c0, b.c1);
    fp2_mul(c1, s0, s1);
    fp2_sub(c1, c1, t0);
    fp2_sub(c1, c1, t1);
    fp2_mul_xi(s0, t2);
    fp2_add(c1, c1, s0);
    fp2_add(s0, a.c0, a.c2);
    fp2_add(s1, b.c0, b.c2);
    fp2_mul(c2, s0, s1);
    fp2_sub(c2, c2, t0);
    fp2_sub(c2, c2, t2);
    fp2_add(c2, c2, t1);
    r.c0 = c0; r.c1 = c1; r.c2 = c2;
}
DI void fp6_mul_v(fp6 &r, const fp6 &a) { // a * v = (xi c2, c0, c1)
    fp2 t;
    fp2_mul_xi(t, a.c2);
    r.c2 = a.c1;
    r.c1 = a.c0;
    r.c0 = t;
}
DI void fp6_mul_01(fp6 &r, const fp6 &a, const fp2 &b0, const fp2 &b1) { // a * (b0, b1, 0)
    fp2 t0, t1, c0, c1, c2, s, u;
    fp2_mul(t0, a.c0, b0);
    fp2_mul(t1, a.c1, b1);
    fp2_mul(c0, a.c2, b1);
    fp2_mul_xi(c0, c0);
    fp2_add(c0, c0, t0);
    fp2_add(s, a.c0, a.c1);
    fp2_add(u, b0, b1);
    fp2_mul(c1, s, u);
    fp2_sub(c1, c1, t0);
    fp2_sub(c1, c1, t1);
    fp2_mul(c2, a.c2, b0);
    fp2_add(c2, c2, t1);
    r.c0 = c0; r.c1 = c1; r.c2 = c2;
}
DI void fp6_mul_1(fp6 &r, const fp6 &a, const fp2 &b1) { // a * (0, b1, 0) = b1 (xi a2, a0, a1)
    fp2 c0, c1, c2;
    fp2_mul(c0, a.c2, b1);
    fp2_mul_xi(c0, c0);
    fp2_mul(c1, a.c0, b1);
    fp2_mul(c2, a.c1, b1);
    r.c0 = c0; r.c1 = c1; r.c2 = c2;
}
DI void fp6_inv(fp6 &r, const fp6 &a) {
    fp2 c0, c1, c2, t, s;
    fp2_sqr(c0, a.c0);
    fp2_mul(t, a.c1, a.c2);
    fp2_mul_xi(t, t);
    fp2_sub(c0, c0, t);
    fp2_sqr(c1, a.c2);
    fp2_mul_xi(c1, c1);
    fp2_mul(t, a.c0, a.c1);
    fp2_sub(c1, c1, t);
    fp2_sqr(c2, a.c1);
    fp2_mul(t, a.c0, a.c2);
    fp2_sub(c2, c2, t);
    fp2_mul(t, a.c2, c1);
    fp2_mul(s, a.c1, c2);
    fp2_add(t, t, s);
    fp2_mul_xi(t, t);
    fp2_mul(s, a.c0, c0);
    fp2_add(t, t, s);
    fp2_inv_g(t, t);     // (reached only from fp12_inv_n / the single-op switch: calls)
    fp2_mul(r.c0, c0, t);
    fp2_mul(r.c1, c1, t);
    fp2_mul(r.c2, c2, t);
}

// ------------------------------------------------------------------------------------------------ Fp12
DI fp12 fp12_one() {
    fp12 r;
    r.c0.c0 = fp2_one(); r.c0.c1 = fp2_zero(); r.c0.c2 = fp2_zero();
    r.c1.c0 = fp2_zero(); r.c1.c1 = fp2_zero(); r.c1.c2 = fp2_zero();
    return r;
}
DI bool fp12_is_one(const fp12 &a) {
    fp12 o = fp12_one();
    const fp *x = &a.c0.c0.a, *y = &o.c0.c0.a;
    bool eq = true;
#pragma unroll
    for (int i = 0; i < 12; i++) eq = eq && fp_eq(x[i], y[i]);
    return eq;
}
DI void fp12_mul(fp12 &r, const fp12 &a, const fp12 &b) {
    fp6 t0, t1, s0, s1;
    fp6_mul(t0, a.c0, b.c0);
    fp6_mul(t1, a.c1, b.c1);
    fp6_add(s0, a.c0, a.c1);
    fp6_add(s1, b.c0, b.c1);
    fp6_mul(s0, s0, s1);
    fp6_sub(s0, s0, t0);
    fp6_sub(r.c1, s0, t1);
    fp6_mul_v(t1, t1);
    fp6_add(r.c0, t0, t1);
}
// (c0 + c1 w)^2 = (c0^2 + v c1^2) + 2 c0 c1 w, computed as c0' = (c0 + c1)(c0 + v c1) - t - v t, c1' = 2t
// (t = c0 c1), updating r in place so only t and s1 are live beside it (register pressure: one Fp12 per lane)
DI void fp12_sqr(fp12 &r, const fp12 &a) {
    fp6 t, s1;
    if (&r != &a) r = a;
    fp6_mul(t, r.c0, r.c1);
    fp6_mul_v(s1, r.c1);
    fp6_add(s1, s1, r.c0);
    fp6_add(r.c0, r.c0, r.c1);
    fp6_mul(r.c0, r.c0, s1);
    fp6_sub(r.c0, r.c0, t);
    fp6_mul_v(s1, t);
    fp6_sub(r.c0, r.c0, s1);
    fp6_add(r.c1, t, t);
}
DI void fp12_conj(fp12 &r, const fp12 &a) { r.c0 = a.c0; fp6_neg(r.c1, a.c1); }
DI void fp12_inv(fp12 &r, const fp12 &a) {
    fp6 t0, t1;
    fp6_mul(t0, a.c0, a.c0);
    fp6_mul(t1, a.c1, a.c1);
    fp6_mul_v(t1, t1);
    fp6_sub(t0, t0, t1);
    fp6_inv(t0, t0);
    fp6_mul(r.c0, a.c0, t0);
    fp6_mul(r.c1, a.c1, t0);
    fp6_neg(r.c1, r.c1);
}
// f *= (A + B v) + (C v) w  — the sparse shape of a Miller-loop line (13 Fp2 muls)
DI void fp12_mul_line(fp12 &f, const fp2 &A, const fp2 &B, const fp2 &C) {
    // f0' = f0 l0 + v f1 l1, f1' = (f0 + f1)(l0 + l1) - f0 l0 - f1 l1 with l0 = A + B v, l1 = C v;
    // f is overwritten in place so only t1 = f1 l1 is live beside it
    fp6 t1;
    fp2 bc;
    fp6_mul_1(t1, f.c1, C);
    fp6_add(f.c1, f.c0, f.c1);
    fp6_mul_01(f.c0, f.c0, A, B);
    fp2_add(bc, B, C);
    fp6_mul_01(f.c1, f.c1, A, bc);
    fp6_sub(f.c1, f.c1, f.c0);
    fp6_sub(f.c1, f.c1, t1);
    fp6_mul_v(t1, t1);
    fp6_add(f.c0, f.c0, t1);
}
// Frobenius maps: element = sum g_k w^k, (g w^k)^p = conj(g) gamma1_k w^k; layout c0 = (g0, g2, g4),
// c1 = (g1, g3, g5)
DI void fp12_frob1(fp12 &r, const fp12 &a) {
    const fp2 *in[6] = {&a.c0.c0, &a.c1.c0, &a.c0.c1, &a.c1.c1, &a.c0.c2, &a.c1.c2};
    fp12 t;
    fp2 *tt[6] = {&t.c0.c0, &t.c1.c0, &t.c0.c1, &t.c1.c1, &t.c0.c2, &t.c1.c2};
#pragma unroll
    for (int k = 0; k < 6; k++) {
        fp2 g, c;
        fp2_conj(g, *in[k]);
        if (k == 0) {
            *tt[k] = g;
        } else {
            fp2_load_const(c, LCB_GAMMA1 + 24 * k);
            fp2_mul(*tt[k], g, c);
        }
    }
    r = t;
}
DI void fp12_frob2(fp12 &r, const fp12 &a) {
    fp12 t;
    const fp2 *in[6] = {&a.c0.c0, &a.c1.c0, &a.c0.c1, &a.c1.c1, &a.c0.c2, &a.c1.c2};
    fp2 *tt[6] = {&t.c0.c0, &t.c1.c0, &t.c0.c1, &t.c1.c1, &t.c0.c2, &t.c1.c2};
#pragma unroll
    for (int k = 0; k < 6; k++) {
        if (k == 0) {
            *tt[k] = *in[k];
        } else {
            fp c;
            fp_load_const(c, LCB_GAMMA2 + 12 * k);
            fp2_mul_fp(*tt[k], *in[k], c);
        }
    }
    r = t;
}
DI void fp12_frob3(fp12 &r, const fp12 &a) {
    fp12 t;
    const fp2 *in[6] = {&a.c0.c0, &a.c1.c0, &a.c0.c1, &a.c1.c1, &a.c0.c2, &a.c1.c2};
    fp2 *tt[6] = {&t.c0.c0, &t.c1.c0, &t.c0.c1, &t.c1.c1, &t.c0.c2, &t.c1.c2};
#pragma unroll
    for (int k = 0; k < 6; k++) {
        fp2 g, c;
        fp2_conj(g, *in[k]);
        if (k == 0) {
            *tt[k] = g;
        } else {
            fp2_load_const(c, LCB_GAMMA3 + 24 * k);
            fp2_mul(*tt[k], g, c);
        }
    }
    r = t;
}
// Granger-Scott cyclotomic squaring (valid for elements of the cyclotomic subgroup)
DI void fp4_sqr(fp2 &c0, fp2 &c1, const fp2 &a, const fp2 &b) {
    fp2 t0, t1, t2;
    fp2_sqr(t0, a);
    fp2_sqr(t1, b);
    fp2_mul_xi(t2, t1);
    fp2_add(c0, t2, t0);
    fp2_add(t2, a, b);
    fp2_sqr(t2, t2);
    fp2_sub(t2, t2, t0);
    fp2_sub(c1, t2, t1);
}
DI void fp12_cyc_sqr(fp12 &r, const fp12 &f) {
    fp2 z0 = f.c0.c0, z4 = f.c0.c1, z3 = f.c0.c2, z2 = f.c1.c0, z1 = f.c1.c1, z5 = f.c1.c2;
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
    r.c0.c0 = z0; r.c0.c1 = z4; r.c0.c2 = z3;
    r.c1.c0 = z2; r.c1.c1 = z1; r.c1.c2 = z5;
}

// ------------------------------------------------------------------------------------------------ Fr
// Montgomery arithmetic mod r (8 x 32-bit limbs, R = 2^256), CIOS; used for Lagrange coefficients.
DI void fr_reduce_once(fr &r, const u32 *t, u32 top) {
    u32 d[8];
    u32 br = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        u64 x = (u64)t[j] - LCB_R[j] - br;
        d[j] = (u32)x;
        br = (u32)(x >> 32) & 1;
    }
    bool ge = top || !br;
#pragma unroll
    for (int j = 0; j < 8; j++) r.v[j] = ge ? d[j] : t[j];
}
DI void fr_mul(fr &r, const fr &a, const fr &b) {
    u32 t[10];
#pragma unroll
    for (int j = 0; j < 10; j++) t[j] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        u64 c = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            u64 s = (u64)a.v[j] * b.v[i] + t[j] + c;
            t[j] = (u32)s;
            c = s >> 32;
        }
        u64 s = (u64)t[8] + c;
        t[8] = (u32)s;
        t[9] = (u32)(s >> 32);
        u32 m = t[0] * LCB_R_INV;
        s = (u64)m * LCB_R[0] + t[0];
        c = s >> 32;
#pragma unroll
        for (int j = 1; j < 8; j++) {
            s = (u64)m * LCB_R[j] + t[j] + c;
            t[j - 1] = (u32)s;
            c = s >> 32;
        }
        s = (u64)t[8] + c;
        t[7] = (u32)s;
        t[8] = t[9] + (u32)(s >> 32);
    }
    fr_reduce_once(r, t, t[8]);
}
DI void fr_add(fr &r, const fr &a, const fr &b) {
    u32 t[8];
    u32 c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        u64 s = (u64)a.v[j] + b.v[j] + c;
        t[j] = (u32)s;
        c = (u32)(s >> 32);
    }
    fr_reduce_once(r, t, c);
}
DI void fr_sub(fr &r, const fr &a, const fr &b) {
    u32 t[8];
    u32 br = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        u64 x = (u64)a.v[j] - b.v[j] - br;
        t[j] = (u32)x;
        br = (u32)(x >> 32) & 1;
    }
    u32 c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        u64 s = (u64)t[j] + (br ? LCB_R[j] : 0u) + c;
        r.v[j] = (u32)s;
        c = (u32)(s >> 32);
    }
}
DI bool fr_is_zero(const fr &a) {
    u32 x = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) x |= a.v[j];
    return x == 0;
}
DI fr fr_one() { fr r; for (int j = 0; j < 8; j++) r.v[j] = LCB_R_ONE[j]; return r; }
DI void fr_from_raw(fr &r, const fr &raw) {
    fr r2;
    for (int j = 0; j < 8; j++) r2.v[j] = LCB_R_R2[j];
    fr_mul(r, raw, r2);
}
DI void fr_to_raw(fr &r, const fr &a) {
    fr one;
    for (int j = 0; j < 8; j++) one.v[j] = j == 0;
    fr_mul(r, a, one);
}
DI bool fr_raw_lt_r(const fr &raw) {
    u32 br = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        u64 x = (u64)raw.v[j] - LCB_R[j] - br;
        br = (u32)(x >> 32) & 1;
    }
    return br != 0;
}
DI void fr_inv(fr &r, const fr &a) {
    fr acc = fr_one();
    for (int i = 254; i >= 0; i--) {
        fr_mul(acc, acc, acc);
        if ((LCB_R_MINUS_2[i >> 5] >> (i & 31)) & 1) fr_mul(acc, acc, a);
    }
    r = acc;
}

// ------------------------------------------------------------------------------------------------ cold
// Non-inlined Fp12 routines for the final exponentiation and other coarse uses: each call does >= 50
// Fp multiplications, so passing operands through the private stack costs little, and it keeps one copy
// of the code per translation unit (compile time and I-cache).
DN void fp12_mul_n(fp12 &r, const fp12 &a, const fp12 &b) { fp12 t; fp12_mul(t, a, b); r = t; }
DN void fp12_sqr_n(fp12 &r, const fp12 &a) { fp12 t; fp12_sqr(t, a); r = t; }
DN void fp12_cyc_sqr_n(fp12 &r, const fp12 &a) { fp12 t; fp12_cyc_sqr(t, a); r = t; }
DN void fp12_inv_n(fp12 &r, const fp12 &a) { fp12 t; fp12_inv(t, a); r = t; }
DN void fp12_frob1_n(fp12 &r, const fp12 &a) { fp12 t; fp12_frob1(t, a); r = t; }
DN void fp12_frob2_n(fp12 &r, const fp12 &a) { fp12 t; fp12_frob2(t, a); r = t; }
DN void fp12_frob3_n(fp12 &r, const fp12 &a) { fp12 t; fp12_frob3(t, a); r = t; }
DN void fp2_inv_n(fp2 &r, const fp2 &a) { fp2 t; fp2_inv(t, a); r = t; }
DN void fp2_inv_gn(fp2 &r, const fp2 &a) { fp2 t; fp2_inv_g(t, a); r = t; }   // line-set normalisation
DN bool fp2_sqrt_n(fp2 &r, const fp2 &a) { fp2 t; bool ok = fp2_sqrt(t, a); r = t; return ok; }
