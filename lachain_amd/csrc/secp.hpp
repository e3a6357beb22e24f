// lachain_amd/csrc/secp.hpp — secp256k1 arithmetic on gfx950 (device code) for the root protocol's ECDSA header-signature
// checks (RootProtocol.cs:91-105 -> DefaultCrypto.VerifySignatureHashed, DefaultCrypto.cs:79-101).
//
// Field: p = 2^256 - C, C = 2^32 + 977.  Elements are 8 x 32-bit little-endian limbs holding any value in [0, 2^256)
// ("weakly reduced": congruent mod p, at most one p too large); fe_canon gives the canonical value.  The special form
// makes reduction two folds of the high half by C (no Montgomery constants), so a product is 64 + 16 MADs.
// Scalars mod n (only for s^-1, u1, u2): Montgomery form, CIOS.
// Points: Jacobian (X, Y, Z) on y^2 = x^3 + 7; additions take an affine second operand (madd-2007-bl, 7M + 4S) and
// handle the exceptional cases (infinity, P == Q, P == -Q) exactly, so adversarial scalars cannot change a decision.
#pragma once
#ifndef SECP_HOST_EMULATION          // tools/secp_emul.cpp compiles this file for the CPU to debug the kernels
#include <hip/hip_runtime.h>
#endif
#include <stdint.h>

typedef uint32_t u32;
typedef uint64_t u64;
#define SDI __device__ __forceinline__

struct fe { u32 v[8]; };
struct sc { u32 v[8]; };
struct secp_aff { fe x, y; };                 // 64 B table entry (canonical coordinates)
struct secp_jac { fe x, y, z; bool inf; };

__constant__ static const u32 SECP_P[8] = {0xfffffc2fu, 0xfffffffeu, 0xffffffffu, 0xffffffffu,
                                           0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
__constant__ static const u32 SECP_N[8] = {0xd0364141u, 0xbfd25e8cu, 0xaf48a03bu, 0xbaaedce6u,
                                           0xfffffffeu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
__constant__ static const u32 SECP_NH[8] = {0x681b20a0u, 0xdfe92f46u, 0x57a4501du, 0x5d576e73u,
                                            0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu};   // (n - 1) / 2
__constant__ static const u32 SECP_R2N[8] = {0x67d7d140u, 0x896cf214u, 0x0e7cf878u, 0x741496c2u,
                                             0x5bcd07c6u, 0xe697f5e4u, 0x81c69bc5u, 0x9d671cd5u};  // 2^512 mod n
__constant__ static const u32 SECP_PMN[8] = {0x2fc9baeeu, 0x402da172u, 0x50b75fc4u, 0x45512319u, 1u, 0u, 0u, 0u}; // p - n
__constant__ static const u32 SECP_GX[8] = {0x16f81798u, 0x59f2815bu, 0x2dce28d9u, 0x029bfcdbu,
                                            0xce870b07u, 0x55a06295u, 0xf9dcbbacu, 0x79be667eu};
__constant__ static const u32 SECP_GY[8] = {0xfb10d4b8u, 0x9c47d08fu, 0xa6855419u, 0xfd17b448u,
                                            0x0e1108a8u, 0x5da4fbfcu, 0x26a3c465u, 0x483ada77u};
#define SECP_NINV 0x5588b13fu          // -n^-1 mod 2^32
#define SECP_C977 977u

// ------------------------------------------------------------------------------------------------ 256-bit helpers
SDI bool u256_lt(const u32 *a, const u32 *b) {     // a < b
    u32 br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        u64 d = (u64)a[i] - b[i] - br;
        br = (u32)(d >> 32) & 1;
    }
    return br != 0;
}
SDI bool u256_is_zero(const u32 *a) {
    u32 x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x |= a[i];
    return x == 0;
}
// 32 big-endian bytes -> little-endian limbs
SDI void u256_from_be(u32 *r, const uint8_t *b) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint8_t *q = b + 28 - 4 * i;
        r[i] = ((u32)q[0] << 24) | ((u32)q[1] << 16) | ((u32)q[2] << 8) | (u32)q[3];
    }
}

// ------------------------------------------------------------------------------------------------ Fp
SDI fe fe_from(const u32 *c) { fe r; for (int i = 0; i < 8; i++) r.v[i] = c[i]; return r; }
SDI fe fe_zero() { fe r; for (int i = 0; i < 8; i++) r.v[i] = 0; return r; }
SDI fe fe_small(u32 a) { fe r = fe_zero(); r.v[0] = a; return r; }

// r = t + k * C for a small k (0..2^34) carried in from above 2^256: r < 2^256 afterwards (the input is < 2^256 and
// the sum wraps at most once more, leaving a value far below 2^256 - C)
SDI void fe_fold(fe &r, const u32 *t, u64 k) {
    u64 k977 = k * SECP_C977;
    u64 c = (u64)t[0] + (u32)k977;
    r.v[0] = (u32)c; c >>= 32;
    c += (u64)t[1] + (k977 >> 32) + (u32)k;
    r.v[1] = (u32)c; c >>= 32;
    c += (u64)t[2] + (k >> 32);
    r.v[2] = (u32)c; c >>= 32;
#pragma unroll
    for (int i = 3; i < 8; i++) { c += t[i]; r.v[i] = (u32)c; c >>= 32; }
    // wrapped once more (c = 1): add C again; the value is now < 2^35 * C, so this cannot carry out of limb 7
    u32 w = (u32)c;
    c = (u64)r.v[0] + w * SECP_C977;
    r.v[0] = (u32)c; c >>= 32;
    c += (u64)r.v[1] + w;
    r.v[1] = (u32)c; c >>= 32;
#pragma unroll
    for (int i = 2; i < 8; i++) { c += r.v[i]; r.v[i] = (u32)c; c >>= 32; }
}
// 512-bit product t[0..15] -> weakly reduced element: lo + hi * C = lo + hi * 977 + (hi << 32), then fold the top
SDI void fe_reduce_wide(fe &r, const u32 *t) {
    u32 w[8];
    u64 c = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        c += (u64)t[k] + (u64)t[8 + k] * SECP_C977 + (k ? t[7 + k] : 0u);
        w[k] = (u32)c;
        c >>= 32;
    }
    c += t[15];                     // (hi << 32) contributes hi[7] at limb 8
    fe_fold(r, w, c);
}
#if !defined(SECP_HOST_EMULATION) && !defined(SECP_C_FIELD)
#include "secp_asm.hpp"
// gfx950: generated inline-assembly product / square (tools/gen_secp_asm.py); SECP_C_FIELD selects the C++ below
SDI u32x8 fe_to_v(const fe &a) { u32x8 v; for (int i = 0; i < 8; i++) v[i] = a.v[i]; return v; }
SDI fe fe_from_v(const u32x8 &v) { fe a; for (int i = 0; i < 8; i++) a.v[i] = v[i]; return a; }
SDI void fe_mul(fe &r, const fe &a, const fe &b) { r = fe_from_v(secp_asm_mul(fe_to_v(a), fe_to_v(b))); }
SDI void fe_sqr(fe &r, const fe &a) { r = fe_from_v(secp_asm_sqr(fe_to_v(a))); }
#else
SDI void fe_mul(fe &r, const fe &a, const fe &b) {
    u32 t[16];
#pragma unroll
    for (int i = 0; i < 16; i++) t[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        u64 c = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            c += (u64)a.v[j] * b.v[i] + t[i + j];
            t[i + j] = (u32)c;
            c >>= 32;
        }
        t[i + 8] = (u32)c;
    }
    fe_reduce_wide(r, t);
}
SDI void fe_sqr(fe &r, const fe &a) {
    // off-diagonal products once, doubled, plus the squares
    u32 t[16];
#pragma unroll
    for (int i = 0; i < 16; i++) t[i] = 0;
#pragma unroll
    for (int i = 0; i < 7; i++) {
        u64 c = 0;
#pragma unroll
        for (int j = i + 1; j < 8; j++) {
            c += (u64)a.v[j] * a.v[i] + t[i + j];
            t[i + j] = (u32)c;
            c >>= 32;
        }
        t[i + 8] = (u32)c;
    }
    u32 top = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) {      // t <<= 1
        u32 nt = t[i] >> 31;
        t[i] = (t[i] << 1) | top;
        top = nt;
    }
    u64 c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        u64 sq = (u64)a.v[i] * a.v[i];
        c += (u64)t[2 * i] + (u32)sq;
        t[2 * i] = (u32)c; c >>= 32;
        c += (u64)t[2 * i + 1] + (u32)(sq >> 32);
        t[2 * i + 1] = (u32)c; c >>= 32;
    }
    fe_reduce_wide(r, t);
}
#endif
#if !defined(SECP_HOST_EMULATION) && !defined(SECP_C_FIELD)
SDI void fe_add(fe &r, const fe &a, const fe &b) { secp_asm_add(r, a, b); }
SDI void fe_sub(fe &r, const fe &a, const fe &b) { secp_asm_sub(r, a, b); }
#else
SDI void fe_add(fe &r, const fe &a, const fe &b) {
    u32 t[8];
    u64 c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) { c += (u64)a.v[i] + b.v[i]; t[i] = (u32)c; c >>= 32; }
    fe_fold(r, t, c);
}
// r = a - b: on borrow add p (= subtract C mod 2^256), twice if the first correction borrows again
SDI void fe_sub(fe &r, const fe &a, const fe &b) {
    u32 t[8];
    u32 br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        u64 d = (u64)a.v[i] - b.v[i] - br;
        t[i] = (u32)d;
        br = (u32)(d >> 32) & 1;
    }
#pragma unroll
    for (int pass = 0; pass < 2; pass++) {
        u32 k = br;
        br = 0;
        u64 d = (u64)t[0] - k * SECP_C977;
        t[0] = (u32)d; br = (u32)(d >> 32) ? 1u : 0u;
        d = (u64)t[1] - k - br;
        t[1] = (u32)d; br = (u32)(d >> 32) & 1;
#pragma unroll
        for (int i = 2; i < 8; i++) {
            d = (u64)t[i] - br;
            t[i] = (u32)d;
            br = (u32)(d >> 32) & 1;
        }
    }
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = t[i];
}
#endif
SDI void fe_neg(fe &r, const fe &a) { fe_sub(r, fe_zero(), a); }
SDI void fe_dbl(fe &r, const fe &a) { fe_add(r, a, a); }
// canonical representative in [0, p)
SDI fe fe_canon(const fe &a) {
    u32 t[8];
    u64 c = (u64)a.v[0] + SECP_C977;
    t[0] = (u32)c; c >>= 32;
    c += (u64)a.v[1] + 1u;
    t[1] = (u32)c; c >>= 32;
#pragma unroll
    for (int i = 2; i < 8; i++) { c += a.v[i]; t[i] = (u32)c; c >>= 32; }
    fe r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = c ? t[i] : a.v[i];   // a + C >= 2^256  <=>  a >= p
    return r;
}
SDI bool fe_is_zero(const fe &a) { fe c = fe_canon(a); return u256_is_zero(c.v); }
SDI bool fe_eq(const fe &a, const fe &b) { fe d; fe_sub(d, a, b); return fe_is_zero(d); }
SDI bool fe_is_odd(const fe &a) { return fe_canon(a).v[0] & 1; }
SDI void fe_sqr_n(fe &r, const fe &a, int n) {
    r = a;
    for (int i = 0; i < n; i++) fe_sqr(r, r);
}
// a^(2^k - 1) blocks shared by the inversion and square-root chains (libsecp256k1's published addition chain)
SDI void fe_chain223(fe &x223, fe &x22, fe &x2, const fe &a) {
    fe x3, x6, x9, x11, x44, x88, x176, x220, t;
    fe_sqr(t, a); fe_mul(x2, t, a);
    fe_sqr(t, x2); fe_mul(x3, t, a);
    fe_sqr_n(t, x3, 3); fe_mul(x6, t, x3);
    fe_sqr_n(t, x6, 3); fe_mul(x9, t, x3);
    fe_sqr_n(t, x9, 2); fe_mul(x11, t, x2);
    fe_sqr_n(t, x11, 11); fe_mul(x22, t, x11);
    fe_sqr_n(t, x22, 22); fe_mul(x44, t, x22);
    fe_sqr_n(t, x44, 44); fe_mul(x88, t, x44);
    fe_sqr_n(t, x88, 88); fe_mul(x176, t, x88);
    fe_sqr_n(t, x176, 44); fe_mul(x220, t, x44);
    fe_sqr_n(t, x220, 3); fe_mul(x223, t, x3);
}
// a^(p-2) = a^-1 (0 -> 0)
SDI void fe_inv(fe &r, const fe &a) {
    fe x223, x22, x2, t;
    fe_chain223(x223, x22, x2, a);
    fe_sqr_n(t, x223, 23); fe_mul(t, t, x22);
    fe_sqr_n(t, t, 5); fe_mul(t, t, a);
    fe_sqr_n(t, t, 3); fe_mul(t, t, x2);
    fe_sqr_n(t, t, 2); fe_mul(r, t, a);
}
// a^((p+1)/4): a square root when one exists (the caller checks r^2 == a)
SDI void fe_sqrt(fe &r, const fe &a) {
    fe x223, x22, x2, t;
    fe_chain223(x223, x22, x2, a);
    fe_sqr_n(t, x223, 23); fe_mul(t, t, x22);
    fe_sqr_n(t, t, 6); fe_mul(t, t, x2);
    fe_sqr_n(r, t, 2);
}

// ------------------------------------------------------------------------------------------------ scalars mod n
SDI void sc_mont_mul(sc &r, const sc &a, const sc &b) {
    u32 t[10];
#pragma unroll
    for (int i = 0; i < 10; i++) t[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        u64 c = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) { c += (u64)a.v[j] * b.v[i] + t[j]; t[j] = (u32)c; c >>= 32; }
        c += t[8]; t[8] = (u32)c; t[9] = (u32)(c >> 32);
        u32 m = t[0] * SECP_NINV;
        c = ((u64)m * SECP_N[0] + t[0]) >> 32;
#pragma unroll
        for (int j = 1; j < 8; j++) { c += (u64)m * SECP_N[j] + t[j]; t[j - 1] = (u32)c; c >>= 32; }
        c += t[8]; t[7] = (u32)c; t[8] = t[9] + (u32)(c >> 32);
    }
    u32 d[8], br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) { u64 x = (u64)t[i] - SECP_N[i] - br; d[i] = (u32)x; br = (u32)(x >> 32) & 1; }
    bool sub = t[8] || !br;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = sub ? d[i] : t[i];
}
SDI sc sc_from(const u32 *c) { sc r; for (int i = 0; i < 8; i++) r.v[i] = c[i]; return r; }
// Montgomery-domain inverse: a R -> a^-1 R (a^(n-2) by square-and-multiply over the public exponent n - 2)
SDI void sc_mont_inv(sc &r, const sc &a) {
    sc acc = a;                       // the top bit of n - 2 is bit 255
    for (int i = 254; i >= 0; i--) {
        sc_mont_mul(acc, acc, acc);
        u32 e = SECP_N[i >> 5] - (i < 32 ? 2u : 0u);   // n - 2 differs from n only in limb 0 (no borrow: n0 > 1)
        if ((e >> (i & 31)) & 1) sc_mont_mul(acc, acc, a);
    }
    r = acc;
}

// ------------------------------------------------------------------------------------------------ points
SDI void jac_set_aff(secp_jac &r, const fe &x, const fe &y) { r.x = x; r.y = y; r.z = fe_small(1); r.inf = false; }
// dbl-2009-l (a = 0): 2M + 5S
SDI void jac_dbl(secp_jac &r, const secp_jac &p) {
    if (p.inf) { r.inf = true; return; }
    fe a, b, c, d, e, f, t, x3, y3, z3;
    fe_sqr(a, p.x);
    fe_sqr(b, p.y);
    fe_sqr(c, b);
    fe_add(t, p.x, b); fe_sqr(d, t); fe_sub(d, d, a); fe_sub(d, d, c); fe_dbl(d, d);
    fe_dbl(e, a); fe_add(e, e, a);
    fe_sqr(f, e);
    fe_sub(x3, f, d); fe_sub(x3, x3, d);
    fe_sub(t, d, x3); fe_mul(y3, e, t);
    fe_dbl(c, c); fe_dbl(c, c); fe_dbl(c, c); fe_sub(y3, y3, c);
    fe_mul(z3, p.y, p.z); fe_dbl(z3, z3);
    r.x = x3; r.y = y3; r.z = z3;
    r.inf = fe_is_zero(z3);          // y = 0 has no point on this curve (order n is odd); kept for safety
}
// r = p + (x2, y2) affine: madd-2007-bl, with the exceptional cases
SDI void jac_add_aff(secp_jac &r, const secp_jac &p, const fe &x2, const fe &y2) {
    if (p.inf) { jac_set_aff(r, x2, y2); return; }
    fe z1z1, u2, s2, h, hh, i4, j, rr, v, t, x3, y3, z3;
    fe_sqr(z1z1, p.z);
    fe_mul(u2, x2, z1z1);
    fe_mul(t, p.z, z1z1); fe_mul(s2, y2, t);
    fe_sub(h, u2, p.x);
    fe_sub(rr, s2, p.y);
    if (fe_is_zero(h)) {
        if (fe_is_zero(rr)) {            // p == q: double the affine point
            secp_jac q;
            jac_set_aff(q, x2, y2);
            jac_dbl(r, q);
        } else {
            r.inf = true;                // p == -q
        }
        return;
    }
    fe_dbl(rr, rr);
    fe_sqr(hh, h);
    fe_dbl(i4, hh); fe_dbl(i4, i4);
    fe_mul(j, h, i4);
    fe_mul(v, p.x, i4);
    fe_sqr(x3, rr); fe_sub(x3, x3, j); fe_sub(x3, x3, v); fe_sub(x3, x3, v);
    fe_sub(t, v, x3); fe_mul(y3, rr, t);
    fe_mul(t, p.y, j); fe_dbl(t, t); fe_sub(y3, y3, t);
    fe_add(t, p.z, h); fe_sqr(z3, t); fe_sub(z3, z3, z1z1); fe_sub(z3, z3, hh);
    r.x = x3; r.y = y3; r.z = z3; r.inf = false;
}
// general Jacobian addition (add-2007-bl, 11M + 5S) with the exceptional cases; used by the table builder
SDI void jac_add(secp_jac &r, const secp_jac &p, const secp_jac &q) {
    if (p.inf) { r = q; return; }
    if (q.inf) { r = p; return; }
    fe z1z1, z2z2, u1, u2, s1, s2, t, h, rr;
    fe_sqr(z1z1, p.z);
    fe_sqr(z2z2, q.z);
    fe_mul(u1, p.x, z2z2);
    fe_mul(u2, q.x, z1z1);
    fe_mul(t, q.z, z2z2); fe_mul(s1, p.y, t);
    fe_mul(t, p.z, z1z1); fe_mul(s2, q.y, t);
    fe_sub(h, u2, u1);
    fe_sub(rr, s2, s1);
    if (fe_is_zero(h)) {
        if (fe_is_zero(rr)) jac_dbl(r, p);
        else r.inf = true;
        return;
    }
    fe i, j, v, x3, y3, z3;
    fe_dbl(i, h); fe_sqr(i, i);
    fe_mul(j, h, i);
    fe_dbl(rr, rr);
    fe_mul(v, u1, i);
    fe_sqr(x3, rr); fe_sub(x3, x3, j); fe_sub(x3, x3, v); fe_sub(x3, x3, v);
    fe_sub(t, v, x3); fe_mul(y3, rr, t);
    fe_mul(t, s1, j); fe_dbl(t, t); fe_sub(y3, y3, t);
    fe_add(t, p.z, q.z); fe_sqr(z3, t); fe_sub(z3, z3, z1z1); fe_sub(z3, z3, z2z2); fe_mul(z3, z3, h);
    r.x = x3; r.y = y3; r.z = z3; r.inf = false;
}

// ------------------------------------------------------------------------------------------------ Keccak-f[1600]
__constant__ static const u64 SECP_KRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
SDI u64 rotl64(u64 v, int r) { return r ? (v << r) | (v >> (64 - r)) : v; }
SDI void keccak_f1600(u64 *s) {
    const int rot[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
    for (int round = 0; round < 24; round++) {
        u64 C[5], D[5], B[25];
#pragma unroll
        for (int x = 0; x < 5; x++) C[x] = s[x] ^ s[x + 5] ^ s[x + 10] ^ s[x + 15] ^ s[x + 20];
#pragma unroll
        for (int x = 0; x < 5; x++) D[x] = C[(x + 4) % 5] ^ rotl64(C[(x + 1) % 5], 1);
#pragma unroll
        for (int i = 0; i < 25; i++) s[i] ^= D[i % 5];
#pragma unroll
        for (int x = 0; x < 5; x++)
#pragma unroll
            for (int y = 0; y < 5; y++) B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(s[x + 5 * y], rot[x + 5 * y]);
#pragma unroll
        for (int x = 0; x < 5; x++)
#pragma unroll
            for (int y = 0; y < 5; y++) s[x + 5 * y] = B[x + 5 * y] ^ ((~B[(x + 1) % 5 + 5 * y]) & B[(x + 2) % 5 + 5 * y]);
        s[0] ^= SECP_KRC[round];
    }
}
