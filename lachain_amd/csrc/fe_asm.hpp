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
// dst = (conj_a ? conj(a) : a) * b  (dst may alias a or b)
DN void fx_mul(u32 *dst, const u32 *a, const u32 *b, int conj_a, size_t n, size_t i) {
    fp12 x, y, r;
    fp12_load_soa(x, a, n, i);
    if (conj_a) fp12_conj(x, x);
    fp12_load_soa(y, b, n, i);
    fp12_mul(r, x, y);
    fp12_store_soa(dst, n, i, r);
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
DI void fx_pow_z(u32 *dst, const u32 *base, u32 *acc, size_t n, size_t i) {
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
        if (bb >= 0) fx_mul(acc, acc, base, 0, n, i);   // bit bb of |z| is set
        b = bb - 1;
    }
    fx_conj(dst, acc, n, i);
}

// f^((p^12 - 1)/r) (x3, mcl's normalisation) of the Fp12 in slot 0 -> slot 0; slots 1..5 as working space.
// Stage structure and products: fe_hard (pairing.hpp).
DI void final_exp_asm(u32 *park, size_t n, size_t i) {
    u32 *X = park, *T = park + (size_t)144 * n, *U = park + (size_t)288 * n, *V = park + (size_t)432 * n,
        *A = park + (size_t)576 * n, *W = park + (size_t)720 * n;
    fx_easy(X, n, i);
    fx_pow_z(T, X, W, n, i);                          // t = x^z
    lcb_asm_cyc_sqr_n(X, U, (u32)(n * 16), (u32)(i * 16), 1);
    fx_mul(U, U, T, 1, n, i);                         // u = conj(x^2) t = x^(z-2)
    fx_pow_z(V, U, W, n, i);                          // v = x^(z^2-2z)
    fx_mul(A, V, X, 0, n, i);
    fx_frob(A, A, 3, n, i);                           // acc = (v x)^(p^3)
    fx_pow_z(V, V, W, n, i);                          // v = x^(z^3-2z^2)
    fx_mul(W, V, T, 0, n, i);
    fx_frob(W, W, 2, n, i);
    fx_mul(A, A, W, 0, n, i);                         // acc *= (v t)^(p^2)
    fx_pow_z(V, V, W, n, i);                          // v = x^(z^4-2z^3)
    lcb_asm_cyc_sqr_n(T, T, (u32)(n * 16), (u32)(i * 16), 1);
    fx_mul(V, V, T, 0, n, i);                         // v = x^(z^4-2z^3+2z)
    fx_mul(W, X, V, 1, n, i);
    fx_frob(W, W, 1, n, i);
    fx_mul(A, A, W, 0, n, i);                         // acc *= (x^-1 v)^p
    fx_pow_z(V, V, W, n, i);                          // v = x^(z^5-2z^4+2z^2)
    fx_mul(U, U, V, 1, n, i);                         // x^(2-z) v
    fx_mul(U, U, X, 0, n, i);                         //   ... x
    fx_mul(X, A, U, 0, n, i);
}
