// lachain_amd/csrc/fe_asm.hpp — final exponentiation over the Fp12-level assembly routines (asm_tower.hpp).
//
// Same exponent, products and order as fe_hard (pairing.hpp: mcl's expHardPartBLS12 shape), but
//  * every run of squarings in an exponentiation by z is ONE call of lcb_r_cyc_sqr_n, which loads the Fp12 into
//    AGPRs a[0:143], squares it there (lazy-reduced Granger-Scott, tools/gen_tower_asm.py) and stores it back, so
//    the 63 squarings neither spill nor shuffle the accumulator around Fp2 leaf calls;
//  * the other Fp12 values of the hard part (x, t, u, v, acc) are parked in per-share SoA slots in HBM (word w of
//    share i at w * n + i: a wave reads 256 contiguous bytes per word) instead of being live across the loops —
//    at most two Fp12 are live outside the loops, and the exponentiation base is re-read at the 5 multiply steps.
// The park buffer holds LCB_FE_ASM_SLOTS slots of 144 words per share; slot 0 is f from the Miller kernel.
// Every slot access, C++ or assembly, is wave-coalesced 16-byte quads (kcommon.hpp soa_at).
#pragma once
#include "kcommon.hpp"
#include "asm_tower.hpp"

#define LCB_FE_ASM_SLOTS 6

// ---- slot operations: Fp12 values live in the park slots between them (noinline: arguments are pointers)
DN void fx_easy(u32 *x, size_t n, size_t i) {
    fp12 f;
    fp12_load_soa(f, x, n, i);
    fe_easy(f, f);
    fp12_store_soa(x, n, i, f);
}
// one lane's column of the block's LDS scratch: 36 quads (t0 = quads 0..17, t1 = quads 18..35), quad g at
// p[g * LCB_BLOCK] (a wave's 64 lanes touch 1 KB contiguous per quad access)
struct FxLds { uint4 *p; };
DI void fp6_load_half(fp6 &x, const u32 *slot, int half, size_t n, size_t i) {
    u32 *d = (u32 *)&x;
    u32 off = (u32)(i * 16);
    asm volatile("" : "+v"(off));
    const char *b = (const char *)slot;
#pragma unroll
    for (int g = 0; g < 18; g++) {
        uint4 v = *(const uint4 *)(b + (size_t)(18 * half + g) * n * 16 + off);
        d[4 * g] = v.x; d[4 * g + 1] = v.y; d[4 * g + 2] = v.z; d[4 * g + 3] = v.w;
    }
}
DI void fp6_store_half(u32 *slot, int half, size_t n, size_t i, const fp6 &x) {
    const u32 *s = (const u32 *)&x;
    u32 off = (u32)(i * 16);
    asm volatile("" : "+v"(off));
    char *b = (char *)slot;
#pragma unroll
    for (int g = 0; g < 18; g++)
        *(uint4 *)(b + (size_t)(18 * half + g) * n * 16 + off) = make_uint4(s[4 * g], s[4 * g + 1], s[4 * g + 2], s[4 * g + 3]);
}
DI void fp6_lds_store(FxLds t, int which, const fp6 &x) {
    const u32 *s = (const u32 *)&x;
#pragma unroll
    for (int g = 0; g < 18; g++)
        t.p[(18 * which + g) * LCB_BLOCK] = make_uint4(s[4 * g], s[4 * g + 1], s[4 * g + 2], s[4 * g + 3]);
}
DI void fp6_lds_load(fp6 &x, FxLds t, int which) {
    u32 *d = (u32 *)&x;
#pragma unroll
    for (int g = 0; g < 18; g++) {
        uint4 v = t.p[(18 * which + g) * LCB_BLOCK];
        d[4 * g] = v.x; d[4 * g + 1] = v.y; d[4 * g + 2] = v.z; d[4 * g + 3] = v.w;
    }
}
// dst = (conj_a ? conj(a) : a) * b  (dst may alias a or b).  Karatsuba over Fp6 in phases that each hold at
// most two Fp6 operands + one product: t1 = a1 b1 and t0 = a0 b0 are parked in LDS, the operands re-read from
// their slots, so the compiler-built Fp6 products run without scratch spills.
DN void fx_mul(u32 *dst, const u32 *a, const u32 *b, int conj_a, size_t n, size_t i, FxLds t) {
    {
        fp6 x, y, r;
        fp6_load_half(x, a, 1, n, i);
        if (conj_a) fp6_neg(x, x);
        fp6_load_half(y, b, 1, n, i);
        fp6_mul(r, x, y);
        fp6_lds_store(t, 1, r);                            // t1 = a1 b1
    }
    asm volatile("" ::: "memory");
    {
        fp6 x, y, r;
        fp6_load_half(x, a, 0, n, i);
        fp6_load_half(y, b, 0, n, i);
        fp6_mul(r, x, y);
        fp6_lds_store(t, 0, r);                            // t0 = a0 b0
    }
    asm volatile("" ::: "memory");
    fp6 s;
    {
        fp6 x, y, u;
        fp6_load_half(x, a, 0, n, i);
        fp6_load_half(u, a, 1, n, i);
        if (conj_a) fp6_sub(x, x, u);
        else fp6_add(x, x, u);
        fp6_load_half(y, b, 0, n, i);
        fp6_load_half(u, b, 1, n, i);
        fp6_add(y, y, u);
        fp6_mul(s, x, y);                                  // (a0 + a1)(b0 + b1)
    }
    asm volatile("" ::: "memory");
    {
        fp6 t0, t1;
        fp6_lds_load(t0, t, 0);
        fp6_lds_load(t1, t, 1);
        fp6_sub(s, s, t0);
        fp6_sub(s, s, t1);
        fp6_store_half(dst, 1, n, i, s);                   // r1 = s - t0 - t1
        fp6_mul_v(t1, t1);
        fp6_add(t0, t0, t1);
        fp6_store_half(dst, 0, n, i, t0);                  // r0 = t0 + v t1
    }
}
// dst = frob_k(a), k = 1, 2, 3
DN void fx_frob(u32 *dst, const u32 *a, int k, size_t n, size_t i) {
    fp12 x, r;
    fp12_load_soa(x, a, n, i);
    if (k == 1) fp12_frob1(r, x);
    else if (k == 2) fp12_frob2(r, x);
    else fp12_frob3(r, x);
    fp12_store_soa(dst, n, i, r);
}
DN void fx_conj(u32 *dst, const u32 *a, size_t n, size_t i) {
    fp12 x;
    fp12_load_soa(x, a, n, i);
    fp12_conj(x, x);
    fp12_store_soa(dst, n, i, x);
}

// dst = x^z (z = -|z| < 0, x unitary in slot `base`), slot `acc` as the accumulator: each run of squarings
// between the set bits of |z| (1, 2, 3, 9, 32, 16) is ONE call of the assembly routine, the five products by x
// are slot products; dst may alias base
DI void fx_pow_z(u32 *dst, const u32 *base, u32 *acc, size_t n, size_t i, FxLds t) {
    const u32 n16 = (u32)(n * 16), off = (u32)(i * 16);
    bool first = true;
    int b = 62;
    while (b >= 0) {
        u32 cnt = 0;
        int bb = b;
        while (bb >= 0) {
            cnt++;
            if ((LCB_Z_ABS >> bb) & 1) break;
            bb--;
        }
        lcb_asm_cyc_sqr_n(first ? base : acc, acc, n16, off, cnt);
        first = false;
        if (bb >= 0) fx_mul(acc, acc, base, 0, n, i, t);   // bit bb of |z| is set
        b = bb - 1;
    }
    fx_conj(dst, acc, n, i);
}

// f^((p^12 - 1)/r) (x3, mcl's normalisation) of the Fp12 in slot 0 -> slot 0; slots 1..5 as working space.
// Stage structure and products: fe_hard (pairing.hpp).
DI void final_exp_asm(u32 *park, size_t n, size_t i, FxLds t) {
    u32 *X = park, *T = park + (size_t)144 * n, *U = park + (size_t)288 * n, *V = park + (size_t)432 * n,
        *A = park + (size_t)576 * n, *W = park + (size_t)720 * n;
    fx_easy(X, n, i);
    fx_pow_z(T, X, W, n, i, t);                          // t = x^z
    lcb_asm_cyc_sqr_n(X, U, (u32)(n * 16), (u32)(i * 16), 1);
    fx_mul(U, U, T, 1, n, i, t);                         // u = conj(x^2) t = x^(z-2)
    fx_pow_z(V, U, W, n, i, t);                          // v = x^(z^2-2z)
    fx_mul(A, V, X, 0, n, i, t);
    fx_frob(A, A, 3, n, i);                           // acc = (v x)^(p^3)
    fx_pow_z(V, V, W, n, i, t);                          // v = x^(z^3-2z^2)
    fx_mul(W, V, T, 0, n, i, t);
    fx_frob(W, W, 2, n, i);
    fx_mul(A, A, W, 0, n, i, t);                         // acc *= (v t)^(p^2)
    fx_pow_z(V, V, W, n, i, t);                          // v = x^(z^4-2z^3)
    lcb_asm_cyc_sqr_n(T, T, (u32)(n * 16), (u32)(i * 16), 1);
    fx_mul(V, V, T, 0, n, i, t);                         // v = x^(z^4-2z^3+2z)
    fx_mul(W, X, V, 1, n, i, t);
    fx_frob(W, W, 1, n, i);
    fx_mul(A, A, W, 0, n, i, t);                         // acc *= (x^-1 v)^p
    fx_pow_z(V, V, W, n, i, t);                          // v = x^(z^5-2z^4+2z^2)
    fx_mul(U, U, V, 1, n, i, t);                         // x^(2-z) v
    fx_mul(U, U, X, 0, n, i, t);                         //   ... x
    fx_mul(X, A, U, 0, n, i, t);
}
