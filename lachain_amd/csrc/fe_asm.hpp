// lachain_amd/csrc/fe_asm.hpp — final exponentiation over the Fp12-level assembly routines (asm_tower.hpp).
//
// Same exponent, products and order as fe_hard (pairing.hpp: mcl's expHardPartBLS12 shape), but
//  * every run of squarings in an exponentiation by z is ONE call of lcb_r_cyc_sqr_n, which loads the Fp12 into
//    AGPRs a[0:143], squares it there (lazy-reduced Granger-Scott, tools/gen_tower_asm.py) and stores it back, so
//    the 63 squarings neither spill nor shuffle the accumulator around Fp2 leaf calls;
//  * round 5: the five products by x inside an exponentiation by z run in the same assembly call (lcb_r_pow_z), so
//    the accumulator stays in AGPRs for all 63 squarings and 5 products, and every other slot product is one call
//    of lcb_r_fp12_mul_n (lazily reduced Fp6 products: 18 Montgomery reductions per Fp12 product instead of 36);
//  * the other Fp12 values of the hard part (x, t, u, v, acc) are parked in per-share SoA slots in HBM (word w of
//    share i at w * n + i: a wave reads 256 contiguous bytes per word) instead of being live across the loops.
// The park buffer holds LCB_FE_ASM_SLOTS slots of 144 words per share; slot 0 is f from the Miller kernel.
// Every slot access, C++ or assembly, is wave-coalesced 16-byte quads (kcommon.hpp soa_at).
#pragma once
#include "kcommon.hpp"
#include "asm_tower.hpp"
#include "pairing.hpp"

#define LCB_FE_ASM_SLOTS 6

// ---- slot operations: Fp12 values live in the park slots between them (noinline: arguments are pointers)
DN void fx_easy(u32 *x, size_t n, size_t i) {
    fp12 f;
    fp12_load_soa(f, x, n, i);
    fe_easy(f, f);
    fp12_store_soa(x, n, i, f);
}
// dst = (conj_a ? conj(a) : a) * b over slots: lcb_r_fp12_mul_n (asm_tower.hpp — Karatsuba over lazily reduced Fp6
// products with the accumulator in AGPRs; the double-width Fp2 products of each Fp6 product pass through the lane's
// 36 LDS quads at `lds`, the t0 / t1 halves through dst, which is never b).  dst may alias a.
DI void fx_mul(u32 *dst, const u32 *a, const u32 *b, int conj_a, size_t n, size_t i, u32 lds) {
    lcb_asm_fp12_mul_n(a, (u32)conj_a, b, dst, dst, (u32)(n * 16), (u32)(i * 16), lds);
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

// dst = x^z (z = -|z| < 0, x unitary in slot `base`): lcb_r_pow_z keeps the accumulator in AGPRs from the first
// squaring to the last — the runs of squarings between the set bits of |z| (1, 2, 3, 9, 32, 16) and the five products
// by x (read from `base` each time); `tmp` holds the products' t0 / t1 halves.  dst may alias base, tmp may not.
DI void fx_pow_z(u32 *dst, const u32 *base, u32 *tmp, size_t n, size_t i, u32 lds) {
    lcb_asm_pow_z(base, tmp, dst, (u32)(n * 16), (u32)(i * 16), lds);
}

// f^((p^12 - 1)/r) (x3, mcl's normalisation) of the Fp12 in slot 0 -> slot 0; slots 1..5 as working space.
// Stage structure and products: fe_hard (pairing.hpp).
DI void final_exp_asm(u32 *park, size_t n, size_t i, u32 t) {
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

// ---- the two-pair Miller loop in assembly (asm_tower.hpp lcb_r_miller2, round 5): f = conj(prod_k l1_k(P1) l2_k(P2))
// over two normalised line sets with the accumulator in AGPRs from the first line to the last — the same residues as
// miller2_norm_lds (pairing.hpp).  Park buffer slots (of n items): P1 / P2 at quads 0..5 / 6..11 of slot 3 ((0, 0)
// for a point at infinity: its lines evaluate to 1), slots 1 and 2 the squarings' operands, f -> slot 0.
DI void g1_park_slot(u32 *slot, u32 q0, size_t n, size_t i, const g1a &P) {
    const fp x = P.inf ? fp_zero() : P.x, y = P.inf ? fp_zero() : P.y;
    char *b = (char *)slot;
    u32 off = (u32)(i * 16);
    asm volatile("" : "+v"(off));
#pragma unroll
    for (int q = 0; q < 3; q++) {
        *(uint4 *)(b + (size_t)(q0 + q) * n * 16 + off) = make_uint4(x.v[4 * q], x.v[4 * q + 1], x.v[4 * q + 2], x.v[4 * q + 3]);
        *(uint4 *)(b + (size_t)(q0 + 3 + q) * n * 16 + off) = make_uint4(y.v[4 * q], y.v[4 * q + 1], y.v[4 * q + 2], y.v[4 * q + 3]);
    }
}
DI void miller2_asm(u32 *park, size_t n, size_t i, u32 lds, const u32 *ls1, const g1a &P1, const u32 *ls2,
                    const g1a &P2) {
    u32 *pslot = park + (size_t)3 * 144 * n;
    g1_park_slot(pslot, 0, n, i, P1);
    g1_park_slot(pslot, 6, n, i, P2);
    lcb_asm_miller2(ls1, ls2, pslot, park + (size_t)144 * n, park + (size_t)288 * n, park, (u32)(n * 16), (u32)(i * 16),
                    lds);
}
// this lane's 36 LDS quads (quad g at + g * 1024) in a block's 36 x LCB_BLOCK quads: wave w's 36 KB, lane l at l * 16
DI u32 lane_lds36(uint4 *base) {
    typedef __attribute__((address_space(3))) uint4 lds_quad_t;
    return (u32)(uintptr_t)(lds_quad_t *)base + (threadIdx.x >> 6) * (36u * 1024u) + (threadIdx.x & 63u) * 16u;
}
