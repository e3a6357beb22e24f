/*
 * oracle/bls.c — TEST INFRASTRUCTURE ONLY (see bls_oracle.h for the contract).
 *
 * Plain-C restatement of the BLS12-381 arithmetic Lachain reaches through herumi mcl
 * (MCL.BLS12_381.Native 0.0.5, un-vendored NuGet dependency; call sites listed in SURVEY.md §8a):
 *   Fp  : 6x64-bit Montgomery (R = 2^384)            Fr : 4x64-bit Montgomery (R = 2^256)
 *   Fp2 = Fp[i]/(i^2+1), Fp6 = Fp2[v]/(v^3-xi), Fp12 = Fp6[w]/(w^2-v), xi = 1+i (mcl default tower)
 *   G1 : y^2 = x^3 + 4 over Fp; G2 : y^2 = x^3 + 4(1+i) over Fp2 (M-type twist); Jacobian coordinates
 *   pairing: optimal ate, loop on |z| = 0xd201000000010000, z < 0 (conjugate at the end),
 *            final exponentiation f^((p^12-1)/r * 3) — the "3x hard part" normalisation mcl uses
 *            (GT is only compared for equality in Lachain, never serialized: DESIGN.md §Parity).
 * Two independent pairing paths exist for self-checking: affine Miller loop + direct exponentiation
 * by the big integer 3(p^4-p^2+1)/r (orc_pairing_slow), and projective lines + addition-chain hard
 * part (orc_pairing, the one used by the protocol functions and the CPU baseline).
 */
#include <stdint.h>
#include <omp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "bls_oracle.h"

typedef uint64_t u64;
typedef unsigned __int128 u128;

void orc_drg_bytes(uint8_t *out, size_t len, const uint8_t *seed, size_t seedlen);

/* ================================================================== big integers */
static int bn_cmp(const u64 *a, const u64 *b, int n) {
    for (int i = n - 1; i >= 0; i--) {
        if (a[i] > b[i]) return 1;
        if (a[i] < b[i]) return -1;
    }
    return 0;
}
static u64 bn_add(u64 *r, const u64 *a, const u64 *b, int n) {
    u64 c = 0;
    for (int i = 0; i < n; i++) {
        u128 s = (u128)a[i] + b[i] + c;
        r[i] = (u64)s;
        c = (u64)(s >> 64);
    }
    return c;
}
static u64 bn_sub(u64 *r, const u64 *a, const u64 *b, int n) {
    u64 br = 0;
    for (int i = 0; i < n; i++) {
        u128 d = (u128)a[i] - b[i] - br;
        r[i] = (u64)d;
        br = (u64)(d >> 64) & 1;
    }
    return br;
}
static int bn_is_zero(const u64 *a, int n) {
    u64 x = 0;
    for (int i = 0; i < n; i++) x |= a[i];
    return x == 0;
}
static void bn_from_hex(u64 *r, int n, const char *hex) {
    memset(r, 0, sizeof(u64) * n);
    if (hex[0] == '0' && (hex[1] == 'x' || hex[1] == 'X')) hex += 2;
    int len = (int)strlen(hex);
    for (int i = 0; i < len; i++) {
        char ch = hex[len - 1 - i];
        int v = (ch >= '0' && ch <= '9') ? ch - '0' : (ch >= 'a' && ch <= 'f') ? ch - 'a' + 10 : ch - 'A' + 10;
        r[i / 16] |= (u64)v << (4 * (i % 16));
    }
}
static int bn_bit(const u64 *a, int i) { return (int)((a[i / 64] >> (i % 64)) & 1); }
static int bn_bitlen(const u64 *a, int n) {
    for (int i = n - 1; i >= 0; i--)
        if (a[i]) return 64 * i + 64 - __builtin_clzll(a[i]);
    return 0;
}
static void bn_shr(u64 *a, int n, int s) { /* s < 64 */
    for (int i = 0; i < n; i++) a[i] = (a[i] >> s) | (i + 1 < n && s ? a[i + 1] << (64 - s) : 0);
}
static void bn_from_le(u64 *r, int n, const uint8_t *b, int nbytes) {
    memset(r, 0, sizeof(u64) * n);
    for (int i = 0; i < nbytes; i++) r[i / 8] |= (u64)b[i] << (8 * (i % 8));
}
static void bn_to_le(uint8_t *b, int nbytes, const u64 *a) {
    for (int i = 0; i < nbytes; i++) b[i] = (uint8_t)(a[i / 8] >> (8 * (i % 8)));
}
/* r = a*b (na x nb limbs) into r[na+nb] */
static void bn_mul(u64 *r, const u64 *a, int na, const u64 *b, int nb) {
    memset(r, 0, sizeof(u64) * (na + nb));
    for (int i = 0; i < na; i++) {
        u64 c = 0;
        for (int j = 0; j < nb; j++) {
            u128 s = (u128)a[i] * b[j] + r[i + j] + c;
            r[i + j] = (u64)s;
            c = (u64)(s >> 64);
        }
        r[i + nb] = c;
    }
}
/* schoolbook long division by a small multi-limb divisor using bit-serial restoring division */
static void bn_divmod(u64 *q, u64 *rem, const u64 *a, int na, const u64 *d, int nd) {
    u64 R[16] = {0};
    memset(q, 0, sizeof(u64) * na);
    for (int i = 64 * na - 1; i >= 0; i--) {
        /* R = R*2 + bit */
        u64 carry = bn_bit(a, i);
        for (int k = 0; k < nd + 1; k++) {
            u64 nc = R[k] >> 63;
            R[k] = (R[k] << 1) | carry;
            carry = nc;
        }
        u64 dd[16] = {0};
        memcpy(dd, d, sizeof(u64) * nd);
        if (bn_cmp(R, dd, nd + 1) >= 0) {
            bn_sub(R, R, dd, nd + 1);
            q[i / 64] |= 1ULL << (i % 64);
        }
    }
    if (rem) memcpy(rem, R, sizeof(u64) * nd);
}

/* ================================================================== Montgomery fields */
#define NP 6
#define NR 4
static u64 P[NP], P_INV, P_R2[NP], P_ONE[NP];
static u64 R_[NR], R_INV, R_R2[NR], R_ONE[NR];
static u64 g_count = 0;
static int g_counting = 0;
void orc_count_reset(void) { g_count = 0; g_counting = 1; }
uint64_t orc_count_get(void) { return g_count; }
/* 1 when this build's Fp product is the MULX / ADX assembly (timing build), 0 for the portable C product */
int orc_fp_impl(void) {
#if defined(ORC_FAST) && defined(__x86_64__) && defined(__ADX__) && defined(__BMI2__)
    return 1;
#else
    return 0;
#endif
}

static u64 neg_inv64(u64 m0) { /* -m0^{-1} mod 2^64 */
    u64 x = 1;
    for (int i = 0; i < 7; i++) x *= 2 - m0 * x;
    return (u64)0 - x;
}

#define DEF_MONT_MUL(NAME, N)                                                       \
    static void NAME(u64 *res, const u64 *a, const u64 *b, const u64 *m, u64 inv) { \
        u64 t[N + 2];                                                               \
        memset(t, 0, sizeof t);                                                     \
        for (int i = 0; i < N; i++) {                                               \
            u64 c = 0;                                                              \
            for (int j = 0; j < N; j++) {                                           \
                u128 s = (u128)a[j] * b[i] + t[j] + c;                              \
                t[j] = (u64)s;                                                      \
                c = (u64)(s >> 64);                                                 \
            }                                                                       \
            u128 s = (u128)t[N] + c;                                                \
            t[N] = (u64)s;                                                          \
            t[N + 1] = (u64)(s >> 64);                                              \
            u64 mm = t[0] * inv;                                                    \
            s = (u128)mm * m[0] + t[0];                                             \
            c = (u64)(s >> 64);                                                     \
            for (int j = 1; j < N; j++) {                                           \
                s = (u128)mm * m[j] + t[j] + c;                                     \
                t[j - 1] = (u64)s;                                                  \
                c = (u64)(s >> 64);                                                 \
            }                                                                       \
            s = (u128)t[N] + c;                                                     \
            t[N - 1] = (u64)s;                                                      \
            t[N] = t[N + 1] + (u64)(s >> 64);                                       \
        }                                                                           \
        if (t[N] || bn_cmp(t, m, N) >= 0) bn_sub(t, t, m, N);                       \
        memcpy(res, t, sizeof(u64) * N);                                            \
    }
DEF_MONT_MUL(mont_mul6, 6)
DEF_MONT_MUL(mont_mul4, 4)

/* ---------------------------------------------------------------- Fp */
typedef struct { u64 l[NP]; } fp;
static fp FP_ZERO, FP_ONE_M;

#if defined(ORC_FAST) && defined(__x86_64__) && defined(__ADX__) && defined(__BMI2__)
/* timing build (bench CPU baseline, `make native`): MULX / ADCX / ADOX product, no operation counting */
#include "mont_adx.h"
static u64 PX[NP + 1];
static inline void fp_mul(fp *r, const fp *a, const fp *b) { mont_mul6_adx(r->l, a->l, b->l, PX); }
#define ORC_FP_ADX 1
#else
static inline void fp_mul(fp *r, const fp *a, const fp *b) {
    if (g_counting) g_count++;
    mont_mul6(r->l, a->l, b->l, P, P_INV);
}
#endif
static inline void fp_sqr(fp *r, const fp *a) { fp_mul(r, a, a); }
static inline void fp_add(fp *r, const fp *a, const fp *b) {
    u64 c = bn_add(r->l, a->l, b->l, NP);
    if (c || bn_cmp(r->l, P, NP) >= 0) bn_sub(r->l, r->l, P, NP);
}
static inline void fp_sub(fp *r, const fp *a, const fp *b) {
    if (bn_sub(r->l, a->l, b->l, NP)) bn_add(r->l, r->l, P, NP);
}
static inline void fp_neg(fp *r, const fp *a) {
    if (bn_is_zero(a->l, NP)) *r = *a;
    else bn_sub(r->l, P, a->l, NP);
}
static inline int fp_is_zero(const fp *a) { return bn_is_zero(a->l, NP); }
static inline int fp_eq(const fp *a, const fp *b) { return memcmp(a->l, b->l, sizeof a->l) == 0; }
static void fp_from_int(fp *r, const u64 *v) { mont_mul6(r->l, v, P_R2, P, P_INV); } /* v < p */
static void fp_to_int(u64 *v, const fp *a) {
    u64 one[NP] = {1, 0, 0, 0, 0, 0};
    mont_mul6(v, a->l, one, P, P_INV);
}
static void fp_set_u64(fp *r, u64 x) {
    u64 v[NP] = {x, 0, 0, 0, 0, 0};
    fp_from_int(r, v);
}
static void fp_pow(fp *r, const fp *a, const u64 *e, int ne) {
    fp acc = FP_ONE_M;
    int nb = bn_bitlen(e, ne);
    for (int i = nb - 1; i >= 0; i--) {
        fp_sqr(&acc, &acc);
        if (bn_bit(e, i)) fp_mul(&acc, &acc, a);
    }
    *r = acc;
}
static u64 P_MINUS_2[NP], P_PLUS1_DIV4[NP], P_MINUS1_DIV2[NP];
static fp FP_INV2; /* 1/2 */
static void fp_inv(fp *r, const fp *a) { fp_pow(r, a, P_MINUS_2, NP); }
static int fp_is_odd(const fp *a) {
    u64 v[NP];
    fp_to_int(v, a);
    return (int)(v[0] & 1);
}
/* mcl Fp::squareRoot for p = 3 mod 4: y = a^((p+1)/4), succeed iff y^2 == a */
static int fp_sqrt(fp *r, const fp *a) {
    fp y, t;
    fp_pow(&y, a, P_PLUS1_DIV4, NP);
    fp_sqr(&t, &y);
    if (!fp_eq(&t, a)) return 0;
    *r = y;
    return 1;
}
static int fp_legendre(const fp *a) { /* 0, 1, -1 */
    if (fp_is_zero(a)) return 0;
    fp t;
    fp_pow(&t, a, P_MINUS1_DIV2, NP);
    return fp_eq(&t, &FP_ONE_M) ? 1 : -1;
}

/* ---------------------------------------------------------------- Fr */
typedef struct { u64 l[NR]; } fr;
static fr FR_ONE_M;
static u64 R_MINUS_2[NR];
static void fr_mul(fr *r, const fr *a, const fr *b) { mont_mul4(r->l, a->l, b->l, R_, R_INV); }
static void fr_add(fr *r, const fr *a, const fr *b) {
    u64 c = bn_add(r->l, a->l, b->l, NR);
    if (c || bn_cmp(r->l, R_, NR) >= 0) bn_sub(r->l, r->l, R_, NR);
}
static void fr_sub(fr *r, const fr *a, const fr *b) {
    if (bn_sub(r->l, a->l, b->l, NR)) bn_add(r->l, r->l, R_, NR);
}
static int fr_is_zero(const fr *a) { return bn_is_zero(a->l, NR); }
static void fr_from_int(fr *r, const u64 *v) { mont_mul4(r->l, v, R_R2, R_, R_INV); }
static void fr_to_int(u64 *v, const fr *a) {
    u64 one[NR] = {1, 0, 0, 0};
    mont_mul4(v, a->l, one, R_, R_INV);
}
static void fr_inv(fr *r, const fr *a) {
    fr acc = FR_ONE_M;
    int nb = bn_bitlen(R_MINUS_2, NR);
    for (int i = nb - 1; i >= 0; i--) {
        fr_mul(&acc, &acc, &acc);
        if (bn_bit(R_MINUS_2, i)) fr_mul(&acc, &acc, a);
    }
    *r = acc;
}
static int fr_from_bytes(fr *r, const uint8_t b[32]) {
    u64 v[NR];
    bn_from_le(v, NR, b, 32);
    if (bn_cmp(v, R_, NR) >= 0) return 0;
    fr_from_int(r, v);
    return 1;
}
static void fr_to_bytes(uint8_t b[32], const fr *a) {
    u64 v[NR];
    fr_to_int(v, a);
    bn_to_le(b, 32, v);
}

/* ---------------------------------------------------------------- Fp2 */
typedef struct { fp a, b; } fp2;
static inline void fp2_add(fp2 *r, const fp2 *x, const fp2 *y) { fp_add(&r->a, &x->a, &y->a); fp_add(&r->b, &x->b, &y->b); }
static inline void fp2_sub(fp2 *r, const fp2 *x, const fp2 *y) { fp_sub(&r->a, &x->a, &y->a); fp_sub(&r->b, &x->b, &y->b); }
static inline void fp2_neg(fp2 *r, const fp2 *x) { fp_neg(&r->a, &x->a); fp_neg(&r->b, &x->b); }
static inline void fp2_conj(fp2 *r, const fp2 *x) { r->a = x->a; fp_neg(&r->b, &x->b); }
static inline int fp2_is_zero(const fp2 *x) { return fp_is_zero(&x->a) && fp_is_zero(&x->b); }
static inline int fp2_eq(const fp2 *x, const fp2 *y) { return fp_eq(&x->a, &y->a) && fp_eq(&x->b, &y->b); }
static void fp2_mul(fp2 *r, const fp2 *x, const fp2 *y) {
    fp t0, t1, t2, t3;
    fp_mul(&t0, &x->a, &y->a);
    fp_mul(&t1, &x->b, &y->b);
    fp_add(&t2, &x->a, &x->b);
    fp_add(&t3, &y->a, &y->b);
    fp_mul(&t2, &t2, &t3);
    fp_sub(&r->a, &t0, &t1);
    fp_sub(&t2, &t2, &t0);
    fp_sub(&r->b, &t2, &t1);
}
static void fp2_sqr(fp2 *r, const fp2 *x) {
    fp t0, t1, t2;
    fp_add(&t0, &x->a, &x->b);
    fp_sub(&t1, &x->a, &x->b);
    fp_mul(&t2, &x->a, &x->b);
    fp_mul(&r->a, &t0, &t1);
    fp_add(&r->b, &t2, &t2);
}
static void fp2_mul_fp(fp2 *r, const fp2 *x, const fp *s) { fp_mul(&r->a, &x->a, s); fp_mul(&r->b, &x->b, s); }
static void fp2_mul_xi(fp2 *r, const fp2 *x) { /* (a+bi)(1+i) = (a-b) + (a+b)i */
    fp t;
    fp_sub(&t, &x->a, &x->b);
    fp_add(&r->b, &x->a, &x->b);
    r->a = t;
}
static void fp2_norm(fp *r, const fp2 *x) {
    fp t;
    fp_sqr(r, &x->a);
    fp_sqr(&t, &x->b);
    fp_add(r, r, &t);
}
static void fp2_inv(fp2 *r, const fp2 *x) {
    fp n;
    fp2_norm(&n, x);
    fp_inv(&n, &n);
    fp_mul(&r->a, &x->a, &n);
    fp_mul(&r->b, &x->b, &n);
    fp_neg(&r->b, &r->b);
}
static void fp2_pow(fp2 *r, const fp2 *a, const u64 *e, int ne) {
    fp2 acc;
    acc.a = FP_ONE_M;
    acc.b = FP_ZERO;
    int nb = bn_bitlen(e, ne);
    for (int i = nb - 1; i >= 0; i--) {
        fp2_sqr(&acc, &acc);
        if (bn_bit(e, i)) fp2_mul(&acc, &acc, a);
    }
    *r = acc;
}
/* mcl Fp2T::squareRoot (norm-based; see DESIGN.md §Parity for the root choice) */
static int fp2_sqrt(fp2 *y, const fp2 *x) {
    fp t1, t2;
    if (fp_is_zero(&x->b)) {
        if (fp_sqrt(&t1, &x->a)) {
            y->a = t1;
            y->b = FP_ZERO;
        } else {
            fp na;
            fp_neg(&na, &x->a);
            if (!fp_sqrt(&t1, &na)) return 0; /* cannot happen for p = 3 mod 4 */
            y->a = FP_ZERO;
            y->b = t1;
        }
        return 1;
    }
    fp_sqr(&t1, &x->a);
    fp_sqr(&t2, &x->b);
    fp_add(&t1, &t1, &t2);
    if (!fp_sqrt(&t1, &t1)) return 0;
    fp_add(&t2, &x->a, &t1);
    fp_mul(&t2, &t2, &FP_INV2);
    if (!fp_sqrt(&t2, &t2)) {
        fp_sub(&t2, &x->a, &t1);
        fp_mul(&t2, &t2, &FP_INV2);
        if (!fp_sqrt(&t2, &t2)) return 0;
    }
    fp inv2c;
    y->a = t2;
    fp_add(&t2, &t2, &t2);
    fp_inv(&inv2c, &t2);
    fp_mul(&y->b, &x->b, &inv2c);
    return 1;
}

/* ---------------------------------------------------------------- Fp6, Fp12 */
typedef struct { fp2 c0, c1, c2; } fp6;
typedef struct { fp6 c0, c1; } fp12;
static void fp6_add(fp6 *r, const fp6 *x, const fp6 *y) { fp2_add(&r->c0, &x->c0, &y->c0); fp2_add(&r->c1, &x->c1, &y->c1); fp2_add(&r->c2, &x->c2, &y->c2); }
static void fp6_sub(fp6 *r, const fp6 *x, const fp6 *y) { fp2_sub(&r->c0, &x->c0, &y->c0); fp2_sub(&r->c1, &x->c1, &y->c1); fp2_sub(&r->c2, &x->c2, &y->c2); }
static void fp6_neg(fp6 *r, const fp6 *x) { fp2_neg(&r->c0, &x->c0); fp2_neg(&r->c1, &x->c1); fp2_neg(&r->c2, &x->c2); }
static void fp6_mul(fp6 *r, const fp6 *a, const fp6 *b) {
    fp2 t0, t1, t2, s0, s1, c0, c1, c2;
    fp2_mul(&t0, &a->c0, &b->c0);
    fp2_mul(&t1, &a->c1, &b->c1);
    fp2_mul(&t2, &a->c2, &b->c2);
    fp2_add(&s0, &a->c1, &a->c2);
    fp2_add(&s1, &b->c1, &b->c2);
    fp2_mul(&c0, &s0, &s1);
    fp2_sub(&c0, &c0, &t1);
    fp2_sub(&c0, &c0, &t2);
    fp2_mul_xi(&c0, &c0);
    fp2_add(&c0, &c0, &t0);
    fp2_add(&s0, &a->c0, &a->c1);
    fp2_add(&s1, &b->c0, &b->c1);
    fp2_mul(&c1, &s0, &s1);
    fp2_sub(&c1, &c1, &t0);
    fp2_sub(&c1, &c1, &t1);
    fp2_mul_xi(&s0, &t2);
    fp2_add(&c1, &c1, &s0);
    fp2_add(&s0, &a->c0, &a->c2);
    fp2_add(&s1, &b->c0, &b->c2);
    fp2_mul(&c2, &s0, &s1);
    fp2_sub(&c2, &c2, &t0);
    fp2_sub(&c2, &c2, &t2);
    fp2_add(&c2, &c2, &t1);
    r->c0 = c0; r->c1 = c1; r->c2 = c2;
}
static void fp6_mul_v(fp6 *r, const fp6 *a) { /* a*v = (xi*c2, c0, c1) */
    fp2 t;
    fp2_mul_xi(&t, &a->c2);
    r->c2 = a->c1;
    r->c1 = a->c0;
    r->c0 = t;
}
static void fp6_inv(fp6 *r, const fp6 *a) {
    fp2 c0, c1, c2, t, s;
    fp2_sqr(&c0, &a->c0);
    fp2_mul(&t, &a->c1, &a->c2);
    fp2_mul_xi(&t, &t);
    fp2_sub(&c0, &c0, &t);
    fp2_sqr(&c1, &a->c2);
    fp2_mul_xi(&c1, &c1);
    fp2_mul(&t, &a->c0, &a->c1);
    fp2_sub(&c1, &c1, &t);
    fp2_sqr(&c2, &a->c1);
    fp2_mul(&t, &a->c0, &a->c2);
    fp2_sub(&c2, &c2, &t);
    fp2_mul(&t, &a->c2, &c1);
    fp2_mul(&s, &a->c1, &c2);
    fp2_add(&t, &t, &s);
    fp2_mul_xi(&t, &t);
    fp2_mul(&s, &a->c0, &c0);
    fp2_add(&t, &t, &s);
    fp2_inv(&t, &t);
    fp2_mul(&r->c0, &c0, &t);
    fp2_mul(&r->c1, &c1, &t);
    fp2_mul(&r->c2, &c2, &t);
}
static fp12 FP12_ONE;
static void fp12_mul(fp12 *r, const fp12 *a, const fp12 *b) {
    fp6 t0, t1, s0, s1;
    fp6_mul(&t0, &a->c0, &b->c0);
    fp6_mul(&t1, &a->c1, &b->c1);
    fp6_add(&s0, &a->c0, &a->c1);
    fp6_add(&s1, &b->c0, &b->c1);
    fp6_mul(&s0, &s0, &s1);
    fp6_sub(&s0, &s0, &t0);
    fp6_sub(&r->c1, &s0, &t1);
    fp6_mul_v(&t1, &t1);
    fp6_add(&r->c0, &t0, &t1);
}
static void fp12_sqr(fp12 *r, const fp12 *a) {
    fp6 t, s0, s1, tv;
    fp6_mul(&t, &a->c0, &a->c1);
    fp6_add(&s0, &a->c0, &a->c1);
    fp6_mul_v(&s1, &a->c1);
    fp6_add(&s1, &s1, &a->c0);
    fp6_mul(&s0, &s0, &s1);
    fp6_sub(&s0, &s0, &t);
    fp6_mul_v(&tv, &t);
    fp6_sub(&r->c0, &s0, &tv);
    fp6_add(&r->c1, &t, &t);
}
static void fp12_conj(fp12 *r, const fp12 *a) { r->c0 = a->c0; fp6_neg(&r->c1, &a->c1); }
static void fp12_inv(fp12 *r, const fp12 *a) {
    fp6 t0, t1;
    fp6_mul(&t0, &a->c0, &a->c0);
    fp6_mul(&t1, &a->c1, &a->c1);
    fp6_mul_v(&t1, &t1);
    fp6_sub(&t0, &t0, &t1);
    fp6_inv(&t0, &t0);
    fp6_mul(&r->c0, &a->c0, &t0);
    fp6_mul(&r->c1, &a->c1, &t0);
    fp6_neg(&r->c1, &r->c1);
}
static int fp12_eq(const fp12 *a, const fp12 *b) { return memcmp(a, b, sizeof *a) == 0; }
/* Frobenius: element = sum g_k w^k (k=0..5), g_k in Fp2; (g w^k)^p = conj(g) * gamma_k * w^k,
   gamma_k = xi^(k(p-1)/6). Layout: c0 = (g0, g2, g4), c1 = (g1, g3, g5). */
static fp2 GAMMA1[6];
static void fp12_frob(fp12 *r, const fp12 *a) {
    fp2 g[6];
    g[0] = a->c0.c0; g[2] = a->c0.c1; g[4] = a->c0.c2;
    g[1] = a->c1.c0; g[3] = a->c1.c1; g[5] = a->c1.c2;
    for (int k = 0; k < 6; k++) {
        fp2_conj(&g[k], &g[k]);
        fp2_mul(&g[k], &g[k], &GAMMA1[k]);
    }
    r->c0.c0 = g[0]; r->c0.c1 = g[2]; r->c0.c2 = g[4];
    r->c1.c0 = g[1]; r->c1.c1 = g[3]; r->c1.c2 = g[5];
}
static void fp12_pow(fp12 *r, const fp12 *a, const u64 *e, int ne) {
    fp12 acc = FP12_ONE;
    int nb = bn_bitlen(e, ne);
    for (int i = nb - 1; i >= 0; i--) {
        fp12_sqr(&acc, &acc);
        if (bn_bit(e, i)) fp12_mul(&acc, &acc, a);
    }
    *r = acc;
}

/* ================================================================== curves */
static const u64 Z_ABS = 0xd201000000010000ULL; /* z = -Z_ABS */
typedef struct { fp x, y, z; } g1;  /* Jacobian, z == 0 <=> infinity */
typedef struct { fp2 x, y, z; } g2;
static fp B1;            /* 4 */
static fp2 B2;           /* 4(1+i) */
static g1 G1_GEN;
static g2 G2_GEN;
static fp2 PSI_X, PSI_Y; /* xi^(-(p-1)/3), xi^(-(p-1)/2) */
static int g_sign_from_b = 0;
static int g_orig_cofactor = 0;
static u64 H2_COFACTOR[8];
static int H2_NLIMBS = 8;
void orc_set_g2_sign_from_b(int v) { g_sign_from_b = v; }
void orc_set_g2_original_cofactor(int v) { g_orig_cofactor = v; }

#define DEF_CURVE(G, F, FADD, FSUB, FMUL, FSQR, FNEG, FISZERO, FEQ, FINV, ONE)                  \
    static int G##_is_inf(const G *p) { return FISZERO(&p->z); }                                 \
    static void G##_set_inf(G *p) { memset(p, 0, sizeof *p); }                                   \
    static void G##_dbl(G *r, const G *p) {                                                      \
        if (G##_is_inf(p)) { *r = *p; return; }                                                  \
        F A, Bv, C, D, E, Fv, t;                                                                 \
        FSQR(&A, &p->x);                                                                         \
        FSQR(&Bv, &p->y);                                                                        \
        FSQR(&C, &Bv);                                                                           \
        FADD(&D, &p->x, &Bv);                                                                    \
        FSQR(&D, &D);                                                                            \
        FSUB(&D, &D, &A);                                                                        \
        FSUB(&D, &D, &C);                                                                        \
        FADD(&D, &D, &D);                                                                        \
        FADD(&E, &A, &A);                                                                        \
        FADD(&E, &E, &A);                                                                        \
        FSQR(&Fv, &E);                                                                           \
        F x3, y3, z3;                                                                            \
        FADD(&t, &D, &D);                                                                        \
        FSUB(&x3, &Fv, &t);                                                                      \
        FSUB(&t, &D, &x3);                                                                       \
        FMUL(&y3, &E, &t);                                                                       \
        FADD(&t, &C, &C);                                                                        \
        FADD(&t, &t, &t);                                                                        \
        FADD(&t, &t, &t);                                                                        \
        FSUB(&y3, &y3, &t);                                                                      \
        FMUL(&z3, &p->y, &p->z);                                                                 \
        FADD(&z3, &z3, &z3);                                                                     \
        r->x = x3; r->y = y3; r->z = z3;                                                         \
    }                                                                                            \
    static void G##_add(G *r, const G *p, const G *q) {                                          \
        if (G##_is_inf(p)) { *r = *q; return; }                                                  \
        if (G##_is_inf(q)) { *r = *p; return; }                                                  \
        F z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;                                         \
        FSQR(&z1z1, &p->z);                                                                      \
        FSQR(&z2z2, &q->z);                                                                      \
        FMUL(&u1, &p->x, &z2z2);                                                                 \
        FMUL(&u2, &q->x, &z1z1);                                                                 \
        FMUL(&s1, &p->y, &q->z);                                                                 \
        FMUL(&s1, &s1, &z2z2);                                                                   \
        FMUL(&s2, &q->y, &p->z);                                                                 \
        FMUL(&s2, &s2, &z1z1);                                                                   \
        if (FEQ(&u1, &u2)) {                                                                     \
            if (FEQ(&s1, &s2)) { G##_dbl(r, p); return; }                                        \
            G##_set_inf(r); return;                                                              \
        }                                                                                        \
        FSUB(&h, &u2, &u1);                                                                      \
        FADD(&i, &h, &h);                                                                        \
        FSQR(&i, &i);                                                                            \
        FMUL(&j, &h, &i);                                                                        \
        FSUB(&rr, &s2, &s1);                                                                     \
        FADD(&rr, &rr, &rr);                                                                     \
        FMUL(&v, &u1, &i);                                                                       \
        F x3, y3, z3;                                                                            \
        FSQR(&x3, &rr);                                                                          \
        FSUB(&x3, &x3, &j);                                                                      \
        FSUB(&x3, &x3, &v);                                                                      \
        FSUB(&x3, &x3, &v);                                                                      \
        FSUB(&t, &v, &x3);                                                                       \
        FMUL(&y3, &rr, &t);                                                                      \
        FMUL(&t, &s1, &j);                                                                       \
        FADD(&t, &t, &t);                                                                        \
        FSUB(&y3, &y3, &t);                                                                      \
        FADD(&z3, &p->z, &q->z);                                                                 \
        FSQR(&z3, &z3);                                                                          \
        FSUB(&z3, &z3, &z1z1);                                                                   \
        FSUB(&z3, &z3, &z2z2);                                                                   \
        FMUL(&z3, &z3, &h);                                                                      \
        r->x = x3; r->y = y3; r->z = z3;                                                         \
    }                                                                                            \
    static void G##_neg(G *r, const G *p) { *r = *p; FNEG(&r->y, &p->y); }                       \
    static void G##_to_affine(F *x, F *y, const G *p) { /* p finite */                           \
        if (FEQ(&p->z, &ONE)) { *x = p->x; *y = p->y; return; }                                  \
        F zi, zi2;                                                                               \
        FINV(&zi, &p->z);                                                                        \
        FSQR(&zi2, &zi);                                                                         \
        FMUL(x, &p->x, &zi2);                                                                    \
        FMUL(&zi2, &zi2, &zi);                                                                   \
        FMUL(y, &p->y, &zi2);                                                                    \
    }                                                                                            \
    static void G##_normalize(G *p) {                                                            \
        if (G##_is_inf(p)) { G##_set_inf(p); return; }                                           \
        G##_to_affine(&p->x, &p->y, p);                                                          \
        p->z = ONE;                                                                              \
    }                                                                                            \
    static int G##_eq(const G *p, const G *q) {                                                  \
        G a = *p, b = *q;                                                                        \
        G##_normalize(&a);                                                                       \
        G##_normalize(&b);                                                                       \
        if (G##_is_inf(&a) || G##_is_inf(&b)) return G##_is_inf(&a) && G##_is_inf(&b);          \
        return FEQ(&a.x, &b.x) && FEQ(&a.y, &b.y);                                               \
    }                                                                                            \
    /* scalar multiplication by a non-negative multi-limb integer, 4-bit fixed window */         \
    static void G##_mul_int(G *r, const G *p, const u64 *e, int ne) {                            \
        G tab[16];                                                                               \
        G##_set_inf(&tab[0]);                                                                    \
        tab[1] = *p;                                                                             \
        for (int k = 2; k < 16; k++) G##_add(&tab[k], &tab[k - 1], p);                           \
        G acc;                                                                                   \
        G##_set_inf(&acc);                                                                       \
        int nb = bn_bitlen(e, ne);                                                               \
        int top = (nb + 3) / 4;                                                                  \
        for (int w = top - 1; w >= 0; w--) {                                                     \
            for (int k = 0; k < 4; k++) G##_dbl(&acc, &acc);                                     \
            int d = 0;                                                                           \
            for (int k = 3; k >= 0; k--) d = (d << 1) | (4 * w + k < 64 * ne ? bn_bit(e, 4 * w + k) : 0); \
            if (d) G##_add(&acc, &acc, &tab[d]);                                                 \
        }                                                                                        \
        *r = acc;                                                                                \
    }

static void fp_sqr_(fp *r, const fp *a) { fp_sqr(r, a); }
DEF_CURVE(g1, fp, fp_add, fp_sub, fp_mul, fp_sqr_, fp_neg, fp_is_zero, fp_eq, fp_inv, FP_ONE_M)
static fp2 FP2_ONE;
DEF_CURVE(g2, fp2, fp2_add, fp2_sub, fp2_mul, fp2_sqr, fp2_neg, fp2_is_zero, fp2_eq, fp2_inv, FP2_ONE)

static int g1_on_curve_affine(const fp *x, const fp *y) {
    fp l, r;
    fp_sqr(&l, y);
    fp_sqr(&r, x);
    fp_mul(&r, &r, x);
    fp_add(&r, &r, &B1);
    return fp_eq(&l, &r);
}
static int g2_on_curve_affine(const fp2 *x, const fp2 *y) {
    fp2 l, r;
    fp2_sqr(&l, y);
    fp2_sqr(&r, x);
    fp2_mul(&r, &r, x);
    fp2_add(&r, &r, &B2);
    return fp2_eq(&l, &r);
}
static void g1_mul_fr(g1 *r, const g1 *p, const fr *s) {
    u64 v[NR];
    fr_to_int(v, s);
    g1_mul_int(r, p, v, NR);
}
static void g2_mul_fr(g2 *r, const g2 *p, const fr *s) {
    u64 v[NR];
    fr_to_int(v, s);
    g2_mul_int(r, p, v, NR);
}
/* psi = untwist o Frobenius o twist on E' (M-type): (x,y) -> (conj(x) xi^{-(p-1)/3}, conj(y) xi^{-(p-1)/2}) */
static void g2_psi(g2 *r, const g2 *p) {
    /* Jacobian is compatible: x = X/Z^2, y = Y/Z^3 and conj commutes with the scaling */
    fp2_conj(&r->x, &p->x);
    fp2_conj(&r->y, &p->y);
    fp2_conj(&r->z, &p->z);
    fp2_mul(&r->x, &r->x, &PSI_X);
    fp2_mul(&r->y, &r->y, &PSI_Y);
}
static void g1_mul_u64(g1 *r, const g1 *p, u64 k) { g1_mul_int(r, p, &k, 1); }
static void g2_mul_u64(g2 *r, const g2 *p, u64 k) { g2_mul_int(r, p, &k, 1); }

/* ------------------------------------------------------------------ serialization */
static void fp_to_bytes(uint8_t b[48], const fp *a) {
    u64 v[NP];
    fp_to_int(v, a);
    bn_to_le(b, 48, v);
}
static int fp_from_bytes_canon(fp *a, const uint8_t b[48]) {
    u64 v[NP];
    bn_from_le(v, NP, b, 48);
    if (bn_cmp(v, P, NP) >= 0) return 0;
    fp_from_int(a, v);
    return 1;
}
static int g2_y_odd(const fp2 *y) { return g_sign_from_b ? fp_is_odd(&y->b) : fp_is_odd(&y->a); }

static void g1_ser(uint8_t out[48], const g1 *p) {
    if (g1_is_inf(p)) { memset(out, 0, 48); return; }
    fp x, y;
    g1_to_affine(&x, &y, p);
    fp_to_bytes(out, &x);
    if (fp_is_odd(&y)) out[47] |= 0x80;
}
static int g1_deser(g1 *p, const uint8_t in[48]) {
    int allz = 1;
    for (int i = 0; i < 48; i++) allz &= in[i] == 0;
    if (allz) { g1_set_inf(p); return 1; }
    uint8_t b[48];
    memcpy(b, in, 48);
    int odd = b[47] >> 7;
    b[47] &= 0x7f;
    fp x, y, t;
    if (!fp_from_bytes_canon(&x, b)) return 0;
    fp_sqr(&t, &x);
    fp_mul(&t, &t, &x);
    fp_add(&t, &t, &B1);
    if (!fp_sqrt(&y, &t)) return 0;
    if (fp_is_odd(&y) != odd) fp_neg(&y, &y);
    p->x = x; p->y = y; p->z = FP_ONE_M;
    return 1;
}
static void g2_ser(uint8_t out[96], const g2 *p) {
    if (g2_is_inf(p)) { memset(out, 0, 96); return; }
    fp2 x, y;
    g2_to_affine(&x, &y, p);
    fp_to_bytes(out, &x.a);
    fp_to_bytes(out + 48, &x.b);
    if (g2_y_odd(&y)) out[95] |= 0x80;
}
static int g2_deser(g2 *p, const uint8_t in[96]) {
    int allz = 1;
    for (int i = 0; i < 96; i++) allz &= in[i] == 0;
    if (allz) { g2_set_inf(p); return 1; }
    uint8_t b[96];
    memcpy(b, in, 96);
    int odd = b[95] >> 7;
    b[95] &= 0x7f;
    fp2 x, y, t;
    if (!fp_from_bytes_canon(&x.a, b)) return 0;
    if (!fp_from_bytes_canon(&x.b, b + 48)) return 0;
    fp2_sqr(&t, &x);
    fp2_mul(&t, &t, &x);
    fp2_add(&t, &t, &B2);
    if (!fp2_sqrt(&y, &t)) return 0;
    if (g2_y_odd(&y) != odd) fp2_neg(&y, &y);
    p->x = x; p->y = y; p->z = FP2_ONE;
    return 1;
}

/* ------------------------------------------------------------------ hash-to-G2 (mcl ORIGINAL) */
static fp C1_SQRT_M3, C2_HALF; /* sqrt(-3) via (p+1)/4 power, (-1 + sqrt(-3))/2 */
/* Fp::setHashOf: SHA-512, first 48 bytes LE, mask to 381 bits, if >= p mask to 380 bits */
static void fp_set_hash_of(fp *r, const uint8_t *msg, size_t len) {
    uint8_t d[64];
    orc_sha512(d, msg, len);
    u64 v[NP];
    bn_from_le(v, NP, d, 48);
    v[5] &= (1ULL << (381 - 320)) - 1;
    if (bn_cmp(v, P, NP) >= 0) v[5] &= (1ULL << (380 - 320)) - 1;
    fp_from_int(r, v);
}
/* Fouque-Tibouchi / SW "calcBN" map (mcl MapTo::calcBN<G2,Fp2>) */
static int g2_calc_bn(g2 *P_, const fp2 *t) {
    fp nrm;
    fp2_norm(&nrm, t);
    int leg = fp_legendre(&nrm);
    if (leg == 0) return 0; /* t == 0 */
    int negative = leg < 0;
    fp2 w, x, y, tmp;
    fp2_sqr(&w, t);
    fp2_add(&w, &w, &B2);
    fp_add(&w.a, &w.a, &FP_ONE_M);
    if (fp2_is_zero(&w)) return 0;
    fp2_inv(&w, &w);
    fp2_mul_fp(&w, &w, &C1_SQRT_M3);
    fp2_mul(&w, &w, t);
    for (int i = 0; i < 3; i++) {
        switch (i) {
        case 0:
            fp2_mul(&x, t, &w);
            fp2_neg(&x, &x);
            fp_add(&x.a, &x.a, &C2_HALF);
            break;
        case 1:
            fp2_neg(&x, &x);
            fp_sub(&x.a, &x.a, &FP_ONE_M);
            break;
        case 2:
            fp2_sqr(&x, &w);
            fp2_inv(&x, &x);
            fp_add(&x.a, &x.a, &FP_ONE_M);
            break;
        }
        fp2_sqr(&tmp, &x);
        fp2_mul(&tmp, &tmp, &x);
        fp2_add(&tmp, &tmp, &B2);
        if (fp2_sqrt(&y, &tmp)) {
            if (negative) fp2_neg(&y, &y);
            P_->x = x; P_->y = y; P_->z = FP2_ONE;
            return 1;
        }
    }
    return 0;
}
/* Budroni-Pintore: (z^2 - z - 1) P + psi((z - 1) P) + psi^2(2P) */
static void g2_clear_cofactor(g2 *Q, const g2 *P_) {
    if (g_orig_cofactor) {
        g2_mul_int(Q, P_, H2_COFACTOR, H2_NLIMBS);
        return;
    }
    g2 T0, T1, T2;
    g2_mul_u64(&T0, P_, Z_ABS + 1); /* |z-1| P */
    g2_neg(&T0, &T0);               /* (z-1) P */
    g2_mul_u64(&T1, &T0, Z_ABS);
    g2_neg(&T1, &T1);               /* z(z-1) P */
    g2_neg(&T2, P_);
    g2_add(&T1, &T1, &T2);          /* (z^2 - z - 1) P */
    g2_psi(&T0, &T0);
    g2_add(&T0, &T0, &T1);
    g2_dbl(&T1, P_);
    g2_psi(&T1, &T1);
    g2_psi(&T1, &T1);
    g2_add(Q, &T0, &T1);
}
static int g2_hash(g2 *out, const uint8_t *msg, size_t len) {
    fp2 t;
    fp_set_hash_of(&t.a, msg, len);
    t.b = FP_ZERO;
    g2 P_;
    if (!g2_calc_bn(&P_, &t)) return 0;
    g2_clear_cofactor(out, &P_);
    return 1;
}

/* ================================================================== pairing */
/* line value l = A + B v + C v w (sparse Fp12), A, B, C in Fp2 */
static void fp12_mul_line_generic(fp12 *f, const fp2 *A, const fp2 *Bc, const fp2 *C) {
    fp12 l;
    memset(&l, 0, sizeof l);
    l.c0.c0 = *A;
    l.c0.c1 = *Bc;
    l.c1.c1 = *C;
    fp12_mul(f, f, &l);
}
/* (a0,a1,a2) * (b0,b1,0) in Fp6: 5 Fp2 muls */
static void fp6_mul_01(fp6 *r, const fp6 *a, const fp2 *b0, const fp2 *b1) {
    fp2 t0, t1, c0, c1, c2, s, u;
    fp2_mul(&t0, &a->c0, b0);
    fp2_mul(&t1, &a->c1, b1);
    fp2_mul(&c0, &a->c2, b1);
    fp2_mul_xi(&c0, &c0);
    fp2_add(&c0, &c0, &t0);
    fp2_add(&s, &a->c0, &a->c1);
    fp2_add(&u, b0, b1);
    fp2_mul(&c1, &s, &u);
    fp2_sub(&c1, &c1, &t0);
    fp2_sub(&c1, &c1, &t1);
    fp2_mul(&c2, &a->c2, b0);
    fp2_add(&c2, &c2, &t1);
    r->c0 = c0; r->c1 = c1; r->c2 = c2;
}
/* (a0,a1,a2) * (0,b1,0) = b1 * (xi a2, a0, a1): 3 Fp2 muls */
static void fp6_mul_1(fp6 *r, const fp6 *a, const fp2 *b1) {
    fp2 c0, c1, c2;
    fp2_mul(&c0, &a->c2, b1);
    fp2_mul_xi(&c0, &c0);
    fp2_mul(&c1, &a->c0, b1);
    fp2_mul(&c2, &a->c1, b1);
    r->c0 = c0; r->c1 = c1; r->c2 = c2;
}
/* f *= (A + B v) + (C v) w : 13 Fp2 muls */
static void fp12_mul_line(fp12 *f, const fp2 *A, const fp2 *Bc, const fp2 *C) {
    fp6 t0, t1, s;
    fp2 bc;
    fp6_mul_01(&t0, &f->c0, A, Bc);
    fp6_mul_1(&t1, &f->c1, C);
    fp6_add(&s, &f->c0, &f->c1);
    fp2_add(&bc, Bc, C);
    fp6_mul_01(&s, &s, A, &bc);
    fp6_sub(&s, &s, &t0);
    fp6_sub(&f->c1, &s, &t1);
    fp6_mul_v(&t1, &t1);
    fp6_add(&f->c0, &t0, &t1);
}
/* --- slow reference Miller loop: affine T, explicit slopes, untwisted line ---
   l(P) scaled by w^3:  (lambda x_T - y_T) + (-lambda x_P) v + (y_P) v w */
static void miller_affine(fp12 *f, const g1 *Pp, const g2 *Qp) {
    *f = FP12_ONE;
    if (g1_is_inf(Pp) || g2_is_inf(Qp)) return;
    fp xP, yP;
    g1_to_affine(&xP, &yP, Pp);
    fp2 xQ, yQ, xT, yT;
    g2_to_affine(&xQ, &yQ, Qp);
    xT = xQ; yT = yQ;
    int nb = 64 - __builtin_clzll(Z_ABS);
    for (int i = nb - 2; i >= 0; i--) {
        fp2 lam, num, den, A, Bc, C, t;
        /* doubling */
        fp2_sqr(&num, &xT);
        fp2_add(&t, &num, &num);
        fp2_add(&num, &num, &t);
        fp2_add(&den, &yT, &yT);
        fp2_inv(&den, &den);
        fp2_mul(&lam, &num, &den);
        fp2_mul(&A, &lam, &xT);
        fp2_sub(&A, &A, &yT);
        fp2_mul_fp(&Bc, &lam, &xP);
        fp2_neg(&Bc, &Bc);
        C.a = yP; C.b = FP_ZERO;
        fp12_sqr(f, f);
        fp12_mul_line(f, &A, &Bc, &C);
        fp2 x3, y3;
        fp2_sqr(&x3, &lam);
        fp2_sub(&x3, &x3, &xT);
        fp2_sub(&x3, &x3, &xT);
        fp2_sub(&t, &xT, &x3);
        fp2_mul(&y3, &lam, &t);
        fp2_sub(&y3, &y3, &yT);
        xT = x3; yT = y3;
        if ((Z_ABS >> i) & 1) {
            fp2_sub(&num, &yT, &yQ);
            fp2_sub(&den, &xT, &xQ);
            fp2_inv(&den, &den);
            fp2_mul(&lam, &num, &den);
            fp2_mul(&A, &lam, &xQ);
            fp2_sub(&A, &A, &yQ);
            fp2_mul_fp(&Bc, &lam, &xP);
            fp2_neg(&Bc, &Bc);
            fp12_mul_line(f, &A, &Bc, &C);
            fp2_sqr(&x3, &lam);
            fp2_sub(&x3, &x3, &xT);
            fp2_sub(&x3, &x3, &xQ);
            fp2_sub(&t, &xT, &x3);
            fp2_mul(&y3, &lam, &t);
            fp2_sub(&y3, &y3, &yT);
            xT = x3; yT = y3;
        }
    }
    fp12_conj(f, f); /* z < 0 */
}
/* --- fast Miller loop: homogeneous projective T = (X, Y, Z), lines scaled by Fp2 factors ---
   doubling: l = (Y^2 - 3b'Z^2) + (-3X^2 xP) v + (2YZ yP) v w
   addition with affine Q: theta = Y - yQ Z, lambda = X - xQ Z,
           l = (theta xQ - lambda yQ) + (-theta xP) v + (lambda yP) v w */
static fp2 B2_3; /* 3b' */
static void dbl_step(fp2 *X, fp2 *Y, fp2 *Z, fp2 *A, fp2 *Bc, fp2 *C, const fp *xP, const fp *yP) {
    fp2 XX, YY, ZZ, bZZ, t, YZ;
    fp2_sqr(&XX, X);
    fp2_sqr(&YY, Y);
    fp2_sqr(&ZZ, Z);
    fp2_mul(&bZZ, &ZZ, &B2_3); /* 3b'Z^2 */
    fp2_mul(&YZ, Y, Z);
    /* line */
    fp2_sub(A, &YY, &bZZ);
    fp2_add(&t, &XX, &XX);
    fp2_add(&t, &t, &XX);
    fp2_mul_fp(Bc, &t, xP);
    fp2_neg(Bc, Bc);
    fp2_add(&t, &YZ, &YZ);
    fp2_mul_fp(C, &t, yP);
    /* point: X3 = XY/2 (Y^2 - 9b'Z^2), Y3 = ((Y^2 + 9b'Z^2)/2)^2 - 27 b'^2 Z^4, Z3 = 2 Y^3 Z */
    fp2 b9, X3, Y3, Z3, s;
    fp2_add(&b9, &bZZ, &bZZ);
    fp2_add(&b9, &b9, &bZZ); /* 9b'Z^2 */
    fp2_mul(&X3, X, Y);
    fp2_mul_fp(&X3, &X3, &FP_INV2);
    fp2_sub(&s, &YY, &b9);
    fp2_mul(&X3, &X3, &s);
    fp2_add(&s, &YY, &b9);
    fp2_mul_fp(&s, &s, &FP_INV2);
    fp2_sqr(&Y3, &s);
    fp2_sqr(&t, &bZZ);        /* 9 b'^2 Z^4 */
    fp2_add(&s, &t, &t);
    fp2_add(&s, &s, &t);      /* 27 b'^2 Z^4 */
    fp2_sub(&Y3, &Y3, &s);
    fp2_mul(&Z3, &YY, &YZ);
    fp2_add(&Z3, &Z3, &Z3);
    *X = X3; *Y = Y3; *Z = Z3;
}
static void add_step(fp2 *X, fp2 *Y, fp2 *Z, fp2 *A, fp2 *Bc, fp2 *C, const fp2 *xQ, const fp2 *yQ,
                     const fp *xP, const fp *yP) {
    fp2 th, la, t, s;
    fp2_mul(&t, yQ, Z);
    fp2_sub(&th, Y, &t);
    fp2_mul(&t, xQ, Z);
    fp2_sub(&la, X, &t);
    fp2_mul(A, &th, xQ);
    fp2_mul(&t, &la, yQ);
    fp2_sub(A, A, &t);
    fp2_mul_fp(Bc, &th, xP);
    fp2_neg(Bc, Bc);
    fp2_mul_fp(C, &la, yP);
    fp2 Cc, D, E, F, G, H;
    fp2_sqr(&Cc, &th);
    fp2_sqr(&D, &la);
    fp2_mul(&E, &la, &D);
    fp2_mul(&F, Z, &Cc);
    fp2_mul(&G, X, &D);
    fp2_add(&H, &E, &F);
    fp2_sub(&H, &H, &G);
    fp2_sub(&H, &H, &G);
    fp2_mul(X, &la, &H);
    fp2_sub(&t, &G, &H);
    fp2_mul(&s, &th, &t);
    fp2_mul(&t, Y, &E);
    fp2_sub(Y, &s, &t);
    fp2_mul(Z, Z, &E);
}
/* multi-Miller loop over n pairs, shared squaring */
static uint64_t g_line_count = 0; /* Fp-mul spent generating lines (dbl_step / add_step), instrumentation only */
static void miller_multi(fp12 *f, const g1 *Ps, const g2 *Qs, int n) {
    fp xP[4], yP[4];
    fp2 xQ[4], yQ[4], X[4], Y[4], Z[4];
    int act[4];
    for (int k = 0; k < n; k++) {
        act[k] = !(g1_is_inf(&Ps[k]) || g2_is_inf(&Qs[k]));
        if (!act[k]) continue;
        g1_to_affine(&xP[k], &yP[k], &Ps[k]);
        g2_to_affine(&xQ[k], &yQ[k], &Qs[k]);
        X[k] = xQ[k]; Y[k] = yQ[k]; Z[k] = FP2_ONE;
    }
    *f = FP12_ONE;
    int nb = 64 - __builtin_clzll(Z_ABS);
    for (int i = nb - 2; i >= 0; i--) {
        fp12_sqr(f, f);
        for (int k = 0; k < n; k++) {
            if (!act[k]) continue;
            fp2 A, Bc, C;
            uint64_t c0 = g_count;
            dbl_step(&X[k], &Y[k], &Z[k], &A, &Bc, &C, &xP[k], &yP[k]);
            g_line_count += g_count - c0 - 4; /* the 4 evaluation muls (Bc xP, C yP) stay with the loop */
            fp12_mul_line(f, &A, &Bc, &C);
        }
        if ((Z_ABS >> i) & 1) {
            for (int k = 0; k < n; k++) {
                if (!act[k]) continue;
                fp2 A, Bc, C;
                uint64_t c0 = g_count;
                add_step(&X[k], &Y[k], &Z[k], &A, &Bc, &C, &xQ[k], &yQ[k], &xP[k], &yP[k]);
                g_line_count += g_count - c0 - 4;
                fp12_mul_line(f, &A, &Bc, &C);
            }
        }
    }
    fp12_conj(f, f);
}
static u64 HARD3[24]; /* 3(p^4 - p^2 + 1)/r */
static int HARD3_N = 24;
static void fe_easy(fp12 *r, const fp12 *f) {
    fp12 t0, t1;
    fp12_conj(&t0, f);
    fp12_inv(&t1, f);
    fp12_mul(&t0, &t0, &t1);      /* f^(p^6 - 1) */
    fp12_frob(&t1, &t0);
    fp12_frob(&t1, &t1);          /* ^(p^2) */
    fp12_mul(r, &t1, &t0);        /* ^(p^2 + 1) */
}
static void final_exp_direct(fp12 *r, const fp12 *f) {
    fp12 t;
    fe_easy(&t, f);
    fp12_pow(r, &t, HARD3, HARD3_N);
}
/* x^|z| then conjugate (x unitary), i.e. x^z */
/* Granger-Scott cyclotomic squaring (valid after the easy part): 9 Fp2 squarings */
static void fp4_sqr(fp2 *c0, fp2 *c1, const fp2 *a, const fp2 *b) {
    fp2 t0, t1, t2;
    fp2_sqr(&t0, a);
    fp2_sqr(&t1, b);
    fp2_mul_xi(&t2, &t1);
    fp2_add(c0, &t2, &t0);
    fp2_add(&t2, a, b);
    fp2_sqr(&t2, &t2);
    fp2_sub(&t2, &t2, &t0);
    fp2_sub(c1, &t2, &t1);
}
static void fp12_cyc_sqr(fp12 *r, const fp12 *f) {
    fp2 z0 = f->c0.c0, z4 = f->c0.c1, z3 = f->c0.c2, z2 = f->c1.c0, z1 = f->c1.c1, z5 = f->c1.c2;
    fp2 t0, t1, t2, t3;
    fp4_sqr(&t0, &t1, &z0, &z1);
    fp2_sub(&z0, &t0, &z0); fp2_add(&z0, &z0, &z0); fp2_add(&z0, &z0, &t0);
    fp2_add(&z1, &t1, &z1); fp2_add(&z1, &z1, &z1); fp2_add(&z1, &z1, &t1);
    fp4_sqr(&t0, &t1, &z2, &z3);
    fp4_sqr(&t2, &t3, &z4, &z5);
    fp2_sub(&z4, &t0, &z4); fp2_add(&z4, &z4, &z4); fp2_add(&z4, &z4, &t0);
    fp2_add(&z5, &t1, &z5); fp2_add(&z5, &z5, &z5); fp2_add(&z5, &z5, &t1);
    fp2_mul_xi(&t0, &t3);
    fp2_add(&z2, &t0, &z2); fp2_add(&z2, &z2, &z2); fp2_add(&z2, &z2, &t0);
    fp2_sub(&z3, &t2, &z3); fp2_add(&z3, &z3, &z3); fp2_add(&z3, &z3, &t2);
    r->c0.c0 = z0; r->c0.c1 = z4; r->c0.c2 = z3;
    r->c1.c0 = z2; r->c1.c1 = z1; r->c1.c2 = z5;
}
static void pow_z(fp12 *r, const fp12 *x) {
    fp12 acc = *x;
    for (int i = 62; i >= 0; i--) {
        fp12_cyc_sqr(&acc, &acc);
        if ((Z_ABS >> i) & 1) fp12_mul(&acc, &acc, x);
    }
    fp12_conj(r, &acc);
}
/* hard part via 3(p^4-p^2+1)/r = (z-1)^2 (z+p)(z^2+p^2-1) + 3 = c0 + c1 p + c2 p^2 + c3 p^3 with
   c3 = z^2-2z+1, c2 = z^3-2z^2+z, c1 = z^4-2z^3+2z-1, c0 = z^5-2z^4+2z^2-z+3 (mcl expHardPartBLS12 shape) */
static void fe_hard_chain(fp12 *y, const fp12 *x) {
    fp12 a0, a1, a2, a3, a4, a5, a6, a7;
    fp12_conj(&a0, x);           /* x^-1 */
    fp12_sqr(&a1, &a0);          /* x^-2 */
    pow_z(&a2, x);               /* x^z */
    fp12_sqr(&a3, &a2);          /* x^2z */
    fp12_mul(&a1, &a1, &a2);     /* x^(z-2) */
    pow_z(&a7, &a1);             /* x^(z^2-2z) */
    pow_z(&a4, &a7);             /* x^(z^3-2z^2) */
    pow_z(&a5, &a4);             /* x^(z^4-2z^3) */
    fp12_mul(&a3, &a3, &a5);     /* x^(z^4-2z^3+2z) */
    pow_z(&a6, &a3);             /* x^(z^5-2z^4+2z^2) */
    fp12_conj(&a1, &a1);         /* x^(2-z) */
    fp12_mul(&a1, &a1, &a6);     /* x^(z^5-2z^4+2z^2-z+2) */
    fp12_mul(&a1, &a1, x);       /* x^c0 */
    fp12_mul(&a3, &a3, &a0);     /* x^(z^4-2z^3+2z-1) = x^c1 */
    fp12_frob(&a3, &a3);
    fp12_mul(&a1, &a1, &a3);
    fp12_mul(&a4, &a4, &a2);     /* x^(z^3-2z^2+z) = x^c2 */
    fp12_frob(&a4, &a4);
    fp12_frob(&a4, &a4);
    fp12_mul(&a1, &a1, &a4);
    fp12_mul(&a7, &a7, x);       /* x^(z^2-2z+1) = x^c3 */
    fp12_frob(y, &a7);
    fp12_frob(y, y);
    fp12_frob(y, y);
    fp12_mul(y, y, &a1);
}
static void final_exp(fp12 *r, const fp12 *f) {
    fp12 t;
    fe_easy(&t, f);
    fe_hard_chain(r, &t);
}

/* ================================================================== init */
static int g_inited = 0;
static const char *P_HEX = "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab";
static const char *R_HEX = "73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001";
static void set_fp_hex(fp *r, const char *h) {
    u64 v[NP];
    bn_from_hex(v, NP, h);
    fp_from_int(r, v);
}
void orc_init(void) {
    if (g_inited) return;
    bn_from_hex(P, NP, P_HEX);
    bn_from_hex(R_, NR, R_HEX);
    P_INV = neg_inv64(P[0]);
#ifdef ORC_FP_ADX
    memcpy(PX, P, sizeof P);
    PX[NP] = P_INV;
#endif
    R_INV = neg_inv64(R_[0]);
    /* R2 = 2^(2*64*N) mod m by repeated doubling of 1 */
    {
        u64 x[NP] = {1, 0, 0, 0, 0, 0};
        for (int i = 0; i < 2 * 64 * NP; i++) {
            u64 c = bn_add(x, x, x, NP);
            if (c || bn_cmp(x, P, NP) >= 0) bn_sub(x, x, P, NP);
        }
        memcpy(P_R2, x, sizeof x);
        u64 y[NR] = {1, 0, 0, 0};
        for (int i = 0; i < 2 * 64 * NR; i++) {
            u64 c = bn_add(y, y, y, NR);
            if (c || bn_cmp(y, R_, NR) >= 0) bn_sub(y, y, R_, NR);
        }
        memcpy(R_R2, y, sizeof y);
    }
    {
        u64 one[NP] = {1, 0, 0, 0, 0, 0};
        fp_from_int(&FP_ONE_M, one);
        memcpy(P_ONE, FP_ONE_M.l, sizeof P_ONE);
        memset(&FP_ZERO, 0, sizeof FP_ZERO);
        u64 o4[NR] = {1, 0, 0, 0};
        fr_from_int(&FR_ONE_M, o4);
        memcpy(R_ONE, FR_ONE_M.l, sizeof R_ONE);
    }
    {
        u64 two[NP] = {2, 0, 0, 0, 0, 0}, one[NP] = {1, 0, 0, 0, 0, 0};
        bn_sub(P_MINUS_2, P, two, NP);
        bn_add(P_PLUS1_DIV4, P, one, NP);
        bn_shr(P_PLUS1_DIV4, NP, 2);
        bn_sub(P_MINUS1_DIV2, P, one, NP);
        bn_shr(P_MINUS1_DIV2, NP, 1);
        u64 t2[NR] = {2, 0, 0, 0};
        bn_sub(R_MINUS_2, R_, t2, NR);
        fp two_m;
        fp_set_u64(&two_m, 2);
        fp_inv(&FP_INV2, &two_m);
    }
    fp_set_u64(&B1, 4);
    B2.a = B1; B2.b = B1;
    FP2_ONE.a = FP_ONE_M; FP2_ONE.b = FP_ZERO;
    fp2_add(&B2_3, &B2, &B2);
    fp2_add(&B2_3, &B2_3, &B2);
    memset(&FP12_ONE, 0, sizeof FP12_ONE);
    FP12_ONE.c0.c0.a = FP_ONE_M;
    /* Frobenius constants gamma_k = xi^(k(p-1)/6) */
    {
        u64 e[NP], one[NP] = {1, 0, 0, 0, 0, 0}, six[NP] = {6, 0, 0, 0, 0, 0}, q[NP];
        bn_sub(e, P, one, NP);
        bn_divmod(q, NULL, e, NP, six, 1);
        fp2 xi;
        xi.a = FP_ONE_M; xi.b = FP_ONE_M;
        fp2 g;
        fp2_pow(&g, &xi, q, NP);
        GAMMA1[0] = FP2_ONE;
        for (int k = 1; k < 6; k++) fp2_mul(&GAMMA1[k], &GAMMA1[k - 1], &g);
        /* psi constants: xi^{-(p-1)/3} = gamma_2^{-1}, xi^{-(p-1)/2} = gamma_3^{-1} */
        fp2_inv(&PSI_X, &GAMMA1[2]);
        fp2_inv(&PSI_Y, &GAMMA1[3]);
    }
    /* generators (decoded from SerializationTest.cs:36,51) */
    set_fp_hex(&G1_GEN.x, "0e5454a6c4f973127bd5d51c7bbf19d16dd7b5d9817ca7272cbd2d5b2b7bd95862f641bff2da2af2415318b88e8f32e9");
    set_fp_hex(&G1_GEN.y, "18e171756d9e54a7b29f1aa051ef55eaff3d711383326e366c9235c5f6aa5c190e77c650dee524f15af0ab82a1d9fbae");
    G1_GEN.z = FP_ONE_M;
    set_fp_hex(&G2_GEN.x.a, "0a1759ba7c80bb84b99e847e84fc90072e223cfe0923d95185d891a2a8bf2a3bbddb347450690df000b037f3067643f1");
    set_fp_hex(&G2_GEN.x.b, "1949e450c5ae6143726578cffef88943a2bd815594308673ebfe24b2ddec17e711a724a2aba25e7075a357940e48630a");
    set_fp_hex(&G2_GEN.y.a, "18145ab7c5e672b450b3460a520444257aa855987b0c41a9187697ccfeebec39f6eacbbfa7446b26111ccbfc9367de9e");
    set_fp_hex(&G2_GEN.y.b, "0473958a234fbb325505d1d0ce3d508d803f95040888045d77022b9afa6173e854c9aa413fb91dc7240c16ee68606262");
    G2_GEN.z = FP2_ONE;
    /* sqrt(-3) and (-1 + sqrt(-3)) / 2 */
    {
        fp m3;
        fp_set_u64(&m3, 3);
        fp_neg(&m3, &m3);
        fp_sqrt(&C1_SQRT_M3, &m3);
        fp_sub(&C2_HALF, &C1_SQRT_M3, &FP_ONE_M);
        fp_mul(&C2_HALF, &C2_HALF, &FP_INV2);
    }
    /* 3(p^4 - p^2 + 1)/r */
    {
        u64 p2[12], p4[24], num[24], q[24];
        bn_mul(p2, P, NP, P, NP);
        bn_mul(p4, p2, 12, p2, 12);
        u64 p2e[24] = {0};
        memcpy(p2e, p2, sizeof p2);
        bn_sub(num, p4, p2e, 24);
        u64 one[24] = {1};
        bn_add(num, num, one, 24);
        u64 three[24] = {3};
        u64 n3[48];
        bn_mul(n3, num, 24, three, 1);
        bn_divmod(q, NULL, n3, 24, R_, NR);
        memcpy(HARD3, q, sizeof q);
    }
    /* original G2 cofactor h2 = (z^8 - 4z^7 + 5z^6 - 4z^4 + 6z^3 - 4z^2 - 4z + 13)/9 (as hex constant) */
    bn_from_hex(H2_COFACTOR, 8,
                "5d543a95414e7f1091d50792876a202cd91de4547085abaa68a205b2e5a7ddfa628f1cb4d9e82ef21537e293a6691ae1616ec6e786f0c70cf1c38e31c7238e5");
    g_inited = 1;
}

/* ================================================================== public API */
static int g1_load(g1 *p, const uint8_t b[48]) { return g1_deser(p, b); }
static int g2_load(g2 *p, const uint8_t b[96]) { return g2_deser(p, b); }

int orc_fr_from_int(uint8_t out[32], int64_t v) {
    orc_init();
    fr a;
    u64 x[NR] = {(u64)(v < 0 ? -v : v), 0, 0, 0};
    fr_from_int(&a, x);
    if (v < 0) {
        fr z;
        memset(&z, 0, sizeof z);
        fr_sub(&a, &z, &a);
    }
    fr_to_bytes(out, &a);
    return 0;
}
int orc_fr_is_canonical(const uint8_t a[32]) {
    orc_init();
    fr t;
    return fr_from_bytes(&t, a);
}
int orc_fr_add(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]) {
    orc_init();
    fr x, y;
    if (!fr_from_bytes(&x, a) || !fr_from_bytes(&y, b)) return -1;
    fr_add(&x, &x, &y);
    fr_to_bytes(out, &x);
    return 0;
}
int orc_fr_sub(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]) {
    orc_init();
    fr x, y;
    if (!fr_from_bytes(&x, a) || !fr_from_bytes(&y, b)) return -1;
    fr_sub(&x, &x, &y);
    fr_to_bytes(out, &x);
    return 0;
}
int orc_fr_mul(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]) {
    orc_init();
    fr x, y;
    if (!fr_from_bytes(&x, a) || !fr_from_bytes(&y, b)) return -1;
    fr_mul(&x, &x, &y);
    fr_to_bytes(out, &x);
    return 0;
}
int orc_fr_inv(uint8_t out[32], const uint8_t a[32]) {
    orc_init();
    fr x;
    if (!fr_from_bytes(&x, a) || fr_is_zero(&x)) return -1;
    fr_inv(&x, &x);
    fr_to_bytes(out, &x);
    return 0;
}
void orc_fr_from_wide(uint8_t out[32], const uint8_t in[64]) {
    orc_init();
    u64 v[8], q[8], rem[NR];
    bn_from_le(v, 8, in, 64);
    bn_divmod(q, rem, v, 8, R_, NR);
    bn_to_le(out, 32, rem);
}
void orc_g1_generator(uint8_t out[48]) { orc_init(); g1_ser(out, &G1_GEN); }
void orc_g2_generator(uint8_t out[96]) { orc_init(); g2_ser(out, &G2_GEN); }
int orc_g1_is_valid_encoding(const uint8_t a[48]) { orc_init(); g1 p; return g1_load(&p, a); }
int orc_g2_is_valid_encoding(const uint8_t a[96]) { orc_init(); g2 p; return g2_load(&p, a); }
int orc_g1_in_subgroup(const uint8_t a[48]) {
    orc_init();
    g1 p, q;
    if (!g1_load(&p, a)) return 0;
    g1_mul_int(&q, &p, R_, NR);
    return g1_is_inf(&q);
}
int orc_g2_in_subgroup(const uint8_t a[96]) {
    orc_init();
    g2 p, q;
    if (!g2_load(&p, a)) return 0;
    g2_mul_int(&q, &p, R_, NR);
    return g2_is_inf(&q);
}
int orc_g1_add(uint8_t out[48], const uint8_t a[48], const uint8_t b[48]) {
    orc_init();
    g1 x, y;
    if (!g1_load(&x, a) || !g1_load(&y, b)) return -1;
    g1_add(&x, &x, &y);
    g1_ser(out, &x);
    return 0;
}
int orc_g2_add(uint8_t out[96], const uint8_t a[96], const uint8_t b[96]) {
    orc_init();
    g2 x, y;
    if (!g2_load(&x, a) || !g2_load(&y, b)) return -1;
    g2_add(&x, &x, &y);
    g2_ser(out, &x);
    return 0;
}
int orc_g1_neg(uint8_t out[48], const uint8_t a[48]) {
    orc_init();
    g1 x;
    if (!g1_load(&x, a)) return -1;
    g1_neg(&x, &x);
    g1_ser(out, &x);
    return 0;
}
int orc_g2_neg(uint8_t out[96], const uint8_t a[96]) {
    orc_init();
    g2 x;
    if (!g2_load(&x, a)) return -1;
    g2_neg(&x, &x);
    g2_ser(out, &x);
    return 0;
}
int orc_g1_mul(uint8_t out[48], const uint8_t a[48], const uint8_t s[32]) {
    orc_init();
    g1 x;
    fr k;
    if (!g1_load(&x, a) || !fr_from_bytes(&k, s)) return -1;
    g1_mul_fr(&x, &x, &k);
    g1_ser(out, &x);
    return 0;
}
int orc_g2_mul(uint8_t out[96], const uint8_t a[96], const uint8_t s[32]) {
    orc_init();
    g2 x;
    fr k;
    if (!g2_load(&x, a) || !fr_from_bytes(&k, s)) return -1;
    g2_mul_fr(&x, &x, &k);
    g2_ser(out, &x);
    return 0;
}
int orc_g2_hash(uint8_t out[96], const uint8_t *msg, size_t len) {
    orc_init();
    g2 h;
    if (!g2_hash(&h, msg, len)) return -1;
    g2_ser(out, &h);
    return 0;
}

/* Lagrange coefficients at 0: lambda_i = prod_{j!=i} x_j / (x_j - x_i); fail on k==0, zero or dup x */
static int lagrange_coeffs(fr *lam, const fr *xs, size_t k) {
    if (k == 0) return -1;
    for (size_t i = 0; i < k; i++) {
        if (fr_is_zero(&xs[i])) return -1;
        for (size_t j = 0; j < i; j++)
            if (memcmp(&xs[i], &xs[j], sizeof(fr)) == 0) return -1;
    }
    fr a = FR_ONE_M;
    for (size_t i = 0; i < k; i++) fr_mul(&a, &a, &xs[i]);
    for (size_t i = 0; i < k; i++) {
        fr b = xs[i], d;
        for (size_t j = 0; j < k; j++) {
            if (j == i) continue;
            fr_sub(&d, &xs[j], &xs[i]);
            fr_mul(&b, &b, &d);
        }
        fr_inv(&b, &b);
        fr_mul(&lam[i], &a, &b);
    }
    return 0;
}
static int load_xs(fr *xs, const uint8_t *b, size_t k) {
    for (size_t i = 0; i < k; i++)
        if (!fr_from_bytes(&xs[i], b + 32 * i)) return 0;
    return 1;
}
int orc_g1_lagrange(uint8_t out[48], const uint8_t *xb, const uint8_t *yb, size_t k) {
    orc_init();
    fr *xs = malloc(sizeof(fr) * (k ? k : 1)), *lam = malloc(sizeof(fr) * (k ? k : 1));
    int rc = -1;
    if (!load_xs(xs, xb, k) || lagrange_coeffs(lam, xs, k)) goto done;
    g1 acc, t;
    g1_set_inf(&acc);
    for (size_t i = 0; i < k; i++) {
        if (!g1_load(&t, yb + 48 * i)) goto done;
        g1_mul_fr(&t, &t, &lam[i]);
        g1_add(&acc, &acc, &t);
    }
    g1_ser(out, &acc);
    rc = 0;
done:
    free(xs); free(lam);
    return rc;
}
int orc_g2_lagrange(uint8_t out[96], const uint8_t *xb, const uint8_t *yb, size_t k) {
    orc_init();
    fr *xs = malloc(sizeof(fr) * (k ? k : 1)), *lam = malloc(sizeof(fr) * (k ? k : 1));
    int rc = -1;
    if (!load_xs(xs, xb, k) || lagrange_coeffs(lam, xs, k)) goto done;
    g2 acc, t;
    g2_set_inf(&acc);
    for (size_t i = 0; i < k; i++) {
        if (!g2_load(&t, yb + 96 * i)) goto done;
        g2_mul_fr(&t, &t, &lam[i]);
        g2_add(&acc, &acc, &t);
    }
    g2_ser(out, &acc);
    rc = 0;
done:
    free(xs); free(lam);
    return rc;
}
int orc_fr_lagrange(uint8_t out[32], const uint8_t *xb, const uint8_t *yb, size_t k) {
    orc_init();
    fr *xs = malloc(sizeof(fr) * (k ? k : 1)), *lam = malloc(sizeof(fr) * (k ? k : 1));
    int rc = -1;
    if (!load_xs(xs, xb, k) || lagrange_coeffs(lam, xs, k)) goto done;
    fr acc, t;
    memset(&acc, 0, sizeof acc);
    for (size_t i = 0; i < k; i++) {
        if (!fr_from_bytes(&t, yb + 32 * i)) goto done;
        fr_mul(&t, &t, &lam[i]);
        fr_add(&acc, &acc, &t);
    }
    fr_to_bytes(out, &acc);
    rc = 0;
done:
    free(xs); free(lam);
    return rc;
}
int orc_fr_eval_poly(uint8_t out[32], const uint8_t *cb, size_t n, const uint8_t xb[32]) {
    orc_init();
    if (n == 0) return -1;
    fr x, acc, c;
    if (!fr_from_bytes(&x, xb)) return -1;
    if (!fr_from_bytes(&acc, cb + 32 * (n - 1))) return -1;
    for (size_t i = n - 1; i-- > 0;) { /* Horner */
        if (!fr_from_bytes(&c, cb + 32 * i)) return -1;
        fr_mul(&acc, &acc, &x);
        fr_add(&acc, &acc, &c);
    }
    fr_to_bytes(out, &acc);
    return 0;
}
int orc_g1_msm(uint8_t out[48], const uint8_t *pts, const uint8_t *scalars, size_t n) {
    orc_init();
    g1 acc, t;
    fr s;
    g1_set_inf(&acc);
    for (size_t i = 0; i < n; i++) {
        if (!g1_load(&t, pts + 48 * i) || !fr_from_bytes(&s, scalars + 32 * i)) return -1;
        g1_mul_fr(&t, &t, &s);
        g1_add(&acc, &acc, &t);
    }
    g1_ser(out, &acc);
    return 0;
}

/* Same result as orc_g1_msm with the n independent scalar multiplications spread over `nthreads` OpenMP threads
   (per-thread partial sums, added in thread order): the CPU baseline of the MSM bench line.  Like MCL's
   LagrangeInterpolation it does one var-base multiplication per point (no bucket method). */
int orc_g1_msm_mt(uint8_t out[48], const uint8_t *pts, const uint8_t *scalars, size_t n, int nthreads) {
    orc_init();
    if (nthreads < 1) nthreads = 1;
    g1 part[256];
    int bad = 0;
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; t++) g1_set_inf(&part[t]);
#pragma omp parallel num_threads(nthreads) reduction(| : bad)
    {
        int t = omp_get_thread_num();
        g1 acc, p;
        fr s;
        g1_set_inf(&acc);
#pragma omp for schedule(static)
        for (size_t i = 0; i < n; i++) {
            if (!g1_load(&p, pts + 48 * i) || !fr_from_bytes(&s, scalars + 32 * i)) { bad = 1; continue; }
            g1_mul_fr(&p, &p, &s);
            g1_add(&acc, &acc, &p);
        }
        part[t] = acc;
    }
    if (bad) return -1;
    g1 acc;
    g1_set_inf(&acc);
    for (int t = 0; t < nthreads; t++) g1_add(&acc, &acc, &part[t]);
    g1_ser(out, &acc);
    return 0;
}

/* GT encoding: 12 canonical Fp, 48 B LE each, order c0.c0.a, c0.c0.b, c0.c1.a, ..., c1.c2.b */
static void gt_ser(uint8_t out[576], const fp12 *f) {
    const fp *e = (const fp *)f;
    for (int i = 0; i < 12; i++) fp_to_bytes(out + 48 * i, &e[i]);
}
static int gt_deser(fp12 *f, const uint8_t in[576]) {
    fp *e = (fp *)f;
    for (int i = 0; i < 12; i++)
        if (!fp_from_bytes_canon(&e[i], in + 48 * i)) return 0;
    return 1;
}
int orc_miller_loop(uint8_t out[576], const uint8_t pb[48], const uint8_t qb[96]) {
    orc_init();
    g1 p; g2 q;
    if (!g1_load(&p, pb) || !g2_load(&q, qb)) return -1;
    fp12 f;
    miller_multi(&f, &p, &q, 1);
    gt_ser(out, &f);
    return 0;
}
int orc_final_exp(uint8_t out[576], const uint8_t fb[576]) {
    orc_init();
    fp12 f, r;
    if (!gt_deser(&f, fb)) return -1;
    final_exp(&r, &f);
    gt_ser(out, &r);
    return 0;
}
int orc_final_exp_direct(uint8_t out[576], const uint8_t fb[576]) {
    orc_init();
    fp12 f, r;
    if (!gt_deser(&f, fb)) return -1;
    final_exp_direct(&r, &f);
    gt_ser(out, &r);
    return 0;
}
static void pairing(fp12 *r, const g1 *p, const g2 *q) {
    fp12 f;
    miller_multi(&f, p, q, 1);
    final_exp(r, &f);
}
int orc_pairing(uint8_t out[576], const uint8_t pb[48], const uint8_t qb[96]) {
    orc_init();
    g1 p; g2 q;
    if (!g1_load(&p, pb) || !g2_load(&q, qb)) return -1;
    fp12 r;
    pairing(&r, &p, &q);
    gt_ser(out, &r);
    return 0;
}
int orc_pairing_slow(uint8_t out[576], const uint8_t pb[48], const uint8_t qb[96]) {
    orc_init();
    g1 p; g2 q;
    if (!g1_load(&p, pb) || !g2_load(&q, qb)) return -1;
    fp12 f, r;
    miller_affine(&f, &p, &q);
    final_exp_direct(&r, &f);
    gt_ser(out, &r);
    return 0;
}
int orc_gt_pow(uint8_t out[576], const uint8_t ab[576], const uint8_t sb[32]) {
    orc_init();
    fp12 a, r;
    fr s;
    if (!gt_deser(&a, ab) || !fr_from_bytes(&s, sb)) return -1;
    u64 v[NR];
    fr_to_int(v, &s);
    fp12_pow(&r, &a, v, NR);
    gt_ser(out, &r);
    return 0;
}
int orc_gt_mul(uint8_t out[576], const uint8_t ab[576], const uint8_t bb[576]) {
    orc_init();
    fp12 a, b;
    if (!gt_deser(&a, ab) || !gt_deser(&b, bb)) return -1;
    fp12_mul(&a, &a, &b);
    gt_ser(out, &a);
    return 0;
}
int orc_gt_is_one(const uint8_t ab[576]) {
    orc_init();
    fp12 a;
    if (!gt_deser(&a, ab)) return 0;
    return fp12_eq(&a, &FP12_ONE);
}

/* ================================================================== Lachain protocol restatements */
static int hash_to_g2_tpke(g2 *h, const g1 *u, const uint8_t *v, size_t vlen) {
    /* TPKE/Utils.cs:21-27: G2.SetHashOf(U.ToBytes() || V) */
    uint8_t stackbuf[256];
    uint8_t *buf = vlen + 48 <= sizeof stackbuf ? stackbuf : malloc(vlen + 48);
    g1_ser(buf, u);
    memcpy(buf + 48, v, vlen);
    int ok = g2_hash(h, buf, vlen + 48);
    if (buf != stackbuf) free(buf);
    return ok;
}
int orc_tpke_encrypt(uint8_t ub[48], uint8_t *v, uint8_t wb[96], const uint8_t yb[48], const uint8_t *data,
                     size_t len, const uint8_t rb[32]) {
    orc_init();
    g1 y, u, t;
    fr r;
    if (!g1_load(&y, yb) || !fr_from_bytes(&r, rb)) return -1;
    g1_mul_fr(&u, &G1_GEN, &r);
    g1_mul_fr(&t, &y, &r);
    uint8_t tb[48];
    g1_ser(tb, &t);
    orc_xor_with_hash(v, tb, data, len);
    g2 h, w;
    if (!hash_to_g2_tpke(&h, &u, v, len)) return -1;
    g2_mul_fr(&w, &h, &r);
    g1_ser(ub, &u);
    g2_ser(wb, &w);
    return 0;
}
int orc_tpke_decrypt(uint8_t uib[48], const uint8_t ub[48], const uint8_t *v, size_t vlen, const uint8_t wb[96],
                     const uint8_t xb[32]) {
    orc_init();
    g1 u, ui;
    g2 w, h;
    fr x;
    if (!g1_load(&u, ub) || !g2_load(&w, wb) || !fr_from_bytes(&x, xb)) return -2;
    if (!hash_to_g2_tpke(&h, &u, v, vlen)) return -2;
    fp12 e1, e2;
    pairing(&e1, &G1_GEN, &w);
    pairing(&e2, &u, &h);
    if (!fp12_eq(&e1, &e2)) return -1; /* "Invalid share!" */
    g1_mul_fr(&ui, &u, &x);
    g1_ser(uib, &ui);
    return 0;
}
static int tpke_verify_loaded(const g1 *yi, const g1 *u, const uint8_t *v, size_t vlen, const g2 *w, const g1 *ui) {
    g2 h;
    if (!hash_to_g2_tpke(&h, u, v, vlen)) return -1;
    fp12 e1, e2;
    pairing(&e1, ui, &h);
    pairing(&e2, yi, w);
    return fp12_eq(&e1, &e2);
}
int orc_tpke_verify_share(const uint8_t yb[48], const uint8_t ub[48], const uint8_t *v, size_t vlen,
                          const uint8_t wb[96], const uint8_t uib[48]) {
    orc_init();
    g1 yi, u, ui;
    g2 w;
    if (!g1_load(&yi, yb) || !g1_load(&u, ub) || !g2_load(&w, wb) || !g1_load(&ui, uib)) return -1;
    return tpke_verify_loaded(&yi, &u, v, vlen, &w, &ui);
}
int orc_tpke_full_decrypt(uint8_t *out, const uint8_t *v, size_t vlen, const int32_t *ids, const uint8_t *uis,
                          size_t k) {
    orc_init();
    uint8_t *xs = malloc(32 * (k ? k : 1));
    for (size_t i = 0; i < k; i++) orc_fr_from_int(xs + 32 * i, (int64_t)ids[i] + 1);
    uint8_t u[48];
    int rc = orc_g1_lagrange(u, xs, uis, k);
    free(xs);
    if (rc) return rc;
    orc_xor_with_hash(out, u, v, vlen);
    return 0;
}
int orc_ts_validate(const uint8_t pkb[48], const uint8_t sigb[96], const uint8_t *msg, size_t len) {
    orc_init();
    g1 pk;
    g2 sig, h;
    if (!g1_load(&pk, pkb) || !g2_load(&sig, sigb)) return -1;
    if (!g2_hash(&h, msg, len)) return -1;
    fp12 e1, e2;
    pairing(&e1, &pk, &h);
    pairing(&e2, &G1_GEN, &sig);
    return fp12_eq(&e1, &e2);
}
int orc_ts_sign(uint8_t sigb[96], const uint8_t skb[32], const uint8_t *msg, size_t len) {
    orc_init();
    fr sk;
    g2 h;
    if (!fr_from_bytes(&sk, skb) || !g2_hash(&h, msg, len)) return -1;
    g2_mul_fr(&h, &h, &sk);
    g2_ser(sigb, &h);
    return 0;
}

/* ================================================================== trustless DKG (Commitment) restatement */
static void fr_from_i32(fr *r, int32_t v) { uint8_t b[32]; orc_fr_from_int(b, v); fr_from_bytes(r, b); }
static int dkg_index(int i, int j) { if (i > j) { int t = i; i = j; j = t; } return i * (i + 1) / 2 + j; } /* Commitment.cs:55-59 */
/* Commitment.Evaluate(x, y) exactly as written (src/Lachain.Consensus/ThresholdKeygen/Data/Commitment.cs:23-37):
   powX = Powers(Fr(x), D+1), powY = Powers(Fr(y), D+1); result += C[Index(i,j)] * powX[i] * powY[j], i.e. two
   successive G1 x Fr multiplications per term, (D+1)^2 terms. */
int orc_dkg_commitment_eval(uint8_t out[48], const uint8_t *coeffs, int D, int32_t x, int32_t y) {
    orc_init();
    int n = (D + 1) * (D + 2) / 2;
    g1 *C = malloc(sizeof(g1) * n);
    fr *px = malloc(sizeof(fr) * (D + 1)), *py = malloc(sizeof(fr) * (D + 1));
    int ok = C && px && py;
    for (int k = 0; ok && k < n; k++) ok = g1_load(&C[k], coeffs + 48 * (size_t)k);
    if (ok) {
        fr fx, fy;
        fr_from_i32(&fx, x);
        fr_from_i32(&fy, y);
        fr_from_i32(&px[0], 1);
        fr_from_i32(&py[0], 1);
        for (int k = 1; k <= D; k++) { fr_mul(&px[k], &px[k - 1], &fx); fr_mul(&py[k], &py[k - 1], &fy); }
        g1 acc, t;
        memset(&acc, 0, sizeof acc);
        for (int i = 0; i <= D; i++)
            for (int j = 0; j <= D; j++) {
                g1_mul_fr(&t, &C[dkg_index(i, j)], &px[i]);
                g1_mul_fr(&t, &t, &py[j]);
                g1_add(&acc, &acc, &t);
            }
        g1_ser(out, &acc);
    }
    free(C); free(px); free(py);
    return ok ? 0 : -1;
}
/* Commitment.Evaluate(x) (Commitment.cs:39-53): row[i] = sum_j C[Index(i,j)] * x^j, D+1 points */
int orc_dkg_commitment_row(uint8_t *out, const uint8_t *coeffs, int D, int32_t x) {
    orc_init();
    int n = (D + 1) * (D + 2) / 2;
    g1 *C = malloc(sizeof(g1) * n);
    int ok = C != NULL;
    for (int k = 0; ok && k < n; k++) ok = g1_load(&C[k], coeffs + 48 * (size_t)k);
    if (ok) {
        fr fx;
        fr_from_i32(&fx, x);
        for (int i = 0; i <= D; i++) {
            g1 acc, t;
            memset(&acc, 0, sizeof acc);
            fr xp;
            fr_from_i32(&xp, 1);
            for (int j = 0; j <= D; j++) {
                g1_mul_fr(&t, &C[dkg_index(i, j)], &xp);
                g1_add(&acc, &acc, &t);
                fr_mul(&xp, &xp, &fx);
            }
            g1_ser(out + 48 * (size_t)i, &acc);
        }
    }
    free(C);
    return ok ? 0 : -1;
}
/* MclBls12381.EvaluatePolynomial over G1 (TrustlessKeygen.cs:172-174): sum_k c_k x^k by Horner with Fr x */
int orc_g1_eval_poly(uint8_t out[48], const uint8_t *coeffs, size_t n, const uint8_t xb[32]) {
    orc_init();
    fr x;
    if (!n || !fr_from_bytes(&x, xb)) return -1;
    g1 acc, c;
    if (!g1_load(&acc, coeffs + 48 * (n - 1))) return -1;
    for (size_t k = n - 1; k-- > 0;) {
        if (!g1_load(&c, coeffs + 48 * k)) return -1;
        g1_mul_fr(&acc, &acc, &x);
        g1_add(&acc, &acc, &c);
    }
    g1_ser(out, &acc);
    return 0;
}

/* ================================================================== CPU baseline batch */
/* ThresholdSignature.PublicKey.ValidateSignature for a batch (ThresholdSignature/PublicKey.cs:16-21), as the
   reference calls it: hash-to-G2 of the message and two pairings per share, OpenMP over shares.  The CPU
   baseline of the CommonCoin bench line (test infrastructure). */
int orc_ts_validate_batch(uint8_t *accept, size_t n, const uint8_t *pks, const uint8_t *sigs, const uint8_t *msgs,
                          const uint32_t *msg_off, const uint32_t *msg_idx, const uint32_t *pk_idx, int nthreads) {
    orc_init();
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthreads)
    for (size_t i = 0; i < n; i++) {
        uint32_t m = msg_idx[i];
        int rc = orc_ts_validate(pks + 48 * (size_t)pk_idx[i], sigs + 96 * i, msgs + msg_off[m],
                                 msg_off[m + 1] - msg_off[m]);
        accept[i] = (uint8_t)(rc == 1);
    }
    return 0;
}

int orc_tpke_verify_batch(uint8_t *accept, size_t n, const uint8_t *y_keys, const uint8_t *cts_u,
                          const uint8_t *cts_v, size_t vlen, const uint8_t *cts_w, const uint32_t *ct_idx,
                          const uint32_t *dec_idx, const uint8_t *uis, int nthreads) {
    orc_init();
    int bad = 0;
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthreads) reduction(+ : bad)
    for (size_t i = 0; i < n; i++) {
        uint32_t c = ct_idx[i], d = dec_idx[i];
        /* as-reference: Decode (G1.FromBytes) then VerifyShare (hash + 2 pairings + Equals) */
        g1 yi, u, ui;
        g2 w;
        int rc;
        if (!g1_load(&yi, y_keys + 48 * (size_t)d) || !g1_load(&u, cts_u + 48 * (size_t)c) ||
            !g2_load(&w, cts_w + 96 * (size_t)c) || !g1_load(&ui, uis + 48 * i))
            rc = 0;
        else
            rc = tpke_verify_loaded(&yi, &u, cts_v + vlen * (size_t)c, vlen, &w, &ui);
        if (rc < 0) { bad++; rc = 0; }
        accept[i] = (uint8_t)rc;
    }
    return bad ? -1 : 0;
}

/* ================================================================== CPU baseline, amortized
   The same algorithm the GPU runs, on host cores, so the GPU/CPU ratio compares like with like:
   H(U||V) and the Miller lines of H and W are computed once per ciphertext (once per message for threshold
   signatures), and each share costs one two-pair Miller loop against those lines plus ONE final exponentiation
   of e(Ui, H) e(-Yi, W) (decision identical to the reference's two separate pairings + Equals,
   TPKE/PublicKey.cs:88-92).  TEST INFRASTRUCTURE (bench.py cpu_baseline leg) only. */
typedef struct { fp2 A, Bc, C; } oline;   /* unevaluated line: A + (Bc xP) v + (C yP) v w */
#define OLINES 68
static void lines_precompute(oline *L, const g2 *Qp) {
    if (g2_is_inf(Qp)) {
        for (int k = 0; k < OLINES; k++) { L[k].A = FP2_ONE; memset(&L[k].Bc, 0, sizeof(fp2)); memset(&L[k].C, 0, sizeof(fp2)); }
        return;
    }
    fp2 xQ, yQ, X, Y, Z;
    g2_to_affine(&xQ, &yQ, Qp);
    X = xQ; Y = yQ; Z = FP2_ONE;
    int nb = 64 - __builtin_clzll(Z_ABS), k = 0;
    for (int i = nb - 2; i >= 0; i--) {
        dbl_step(&X, &Y, &Z, &L[k].A, &L[k].Bc, &L[k].C, &FP_ONE_M, &FP_ONE_M); k++;
        if ((Z_ABS >> i) & 1) { add_step(&X, &Y, &Z, &L[k].A, &L[k].Bc, &L[k].C, &xQ, &yQ, &FP_ONE_M, &FP_ONE_M); k++; }
    }
}
/* Round 2 (as the GPU, lachain_amd/csrc/pairing.hpp lineset_compute): normalise a line set to A = 1 with one
   Fp2 inversion (Montgomery's batch trick); the Fp2 factors A^-1 change the Miller value by an Fp6 element, which
   the final exponentiation maps to 1.  Returns 0 (set left as is) when some A == 0. */
static int lines_normalise(oline *L) {
    fp2 pre[OLINES], acc = FP2_ONE, inv;
    for (int k = 0; k < OLINES; k++) {
        fp2_mul(&acc, &acc, &L[k].A);
        pre[k] = acc;
    }
    if (fp2_is_zero(&acc)) return 0;
    fp2_inv(&inv, &acc);
    for (int k = OLINES - 1; k >= 0; k--) {
        fp2 ai;
        if (k > 0) fp2_mul(&ai, &inv, &pre[k - 1]);
        else ai = inv;
        fp2_mul(&inv, &inv, &L[k].A);
        fp2_mul(&L[k].Bc, &L[k].Bc, &ai);
        fp2_mul(&L[k].C, &L[k].C, &ai);
        L[k].A = FP2_ONE;
    }
    return 1;
}
/* f *= 1 + b v + c v w: Karatsuba over Fp6 with X = v f0, Y = v f1 — 9 Fp2 muls (pairing.hpp fp12_mul_line_n) */
static void fp12_mul_line_n(fp12 *f, const fp2 *b, const fp2 *c) {
    fp6 X, Y, t0, t1, s, u;
    fp2 bc;
    fp6_mul_v(&X, &f->c0);
    fp6_mul_v(&Y, &f->c1);
    fp2_mul(&t0.c0, b, &X.c0); fp2_mul(&t0.c1, b, &X.c1); fp2_mul(&t0.c2, b, &X.c2);
    fp2_mul(&t1.c0, c, &Y.c0); fp2_mul(&t1.c1, c, &Y.c1); fp2_mul(&t1.c2, c, &Y.c2);
    fp2_add(&bc, b, c);
    fp6_add(&u, &X, &Y);
    fp2_mul(&s.c0, &bc, &u.c0); fp2_mul(&s.c1, &bc, &u.c1); fp2_mul(&s.c2, &bc, &u.c2);
    fp6_sub(&s, &s, &t0);
    fp6_sub(&s, &s, &t1);
    fp6_add(&f->c1, &f->c1, &s);                  /* f1 + b Y + c X */
    fp6_mul_v(&t1, &t1);
    fp6_add(&f->c0, &f->c0, &t0);
    fp6_add(&f->c0, &f->c0, &t1);                 /* f0 + b X + v c Y */
}
/* f = f_{|z|,Q1}(P1) f_{|z|,Q2}(P2), conjugated (z < 0); a pair whose G1 point is infinity contributes 1 */
static void miller2_lines(fp12 *f, const oline *L1, const g1 *P1, const oline *L2, const g1 *P2) {
    const oline *L[2] = {L1, L2};
    const g1 *P[2] = {P1, P2};
    fp xP[2], yP[2];
    int act[2];
    for (int j = 0; j < 2; j++) {
        act[j] = !g1_is_inf(P[j]);
        if (act[j]) g1_to_affine(&xP[j], &yP[j], P[j]);
    }
    *f = FP12_ONE;
    int nb = 64 - __builtin_clzll(Z_ABS), k = 0;
    for (int i = nb - 2; i >= 0; i--) {
        fp12_sqr(f, f);
        int steps = ((Z_ABS >> i) & 1) ? 2 : 1;
        for (int s_ = 0; s_ < steps; s_++, k++)
            for (int j = 0; j < 2; j++) {
                if (!act[j]) continue;
                fp2 B, C;
                fp2_mul_fp(&B, &L[j][k].Bc, &xP[j]);
                fp2_mul_fp(&C, &L[j][k].C, &yP[j]);
                if (fp2_eq(&L[j][k].A, &FP2_ONE)) fp12_mul_line_n(f, &B, &C);   /* normalised set */
                else fp12_mul_line(f, &L[j][k].A, &B, &C);
            }
    }
    fp12_conj(f, f);
}
static int check_pair_product(const oline *L1, const g1 *P1, const oline *L2, const g1 *P2) {
    fp12 f, e;
    miller2_lines(&f, L1, P1, L2, P2);
    final_exp(&e, &f);
    return fp12_eq(&e, &FP12_ONE);
}
int orc_tpke_verify_batch_amortized(uint8_t *accept, size_t n, const uint8_t *y_keys, size_t n_keys,
                                    const uint8_t *cts_u, const uint8_t *cts_v, size_t vlen, const uint8_t *cts_w,
                                    size_t n_cts, const uint32_t *ct_idx, const uint32_t *dec_idx, const uint8_t *uis,
                                    int nthreads) {
    orc_init();
    oline *LH = malloc(sizeof(oline) * OLINES * (n_cts ? n_cts : 1));
    oline *LW = malloc(sizeof(oline) * OLINES * (n_cts ? n_cts : 1));
    uint8_t *ctok = malloc(n_cts ? n_cts : 1);
    g1 *Y = malloc(sizeof(g1) * (n_keys ? n_keys : 1));
    uint8_t *kok = malloc(n_keys ? n_keys : 1);
    if (!LH || !LW || !ctok || !Y || !kok) { free(LH); free(LW); free(ctok); free(Y); free(kok); return -1; }
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
    for (size_t c = 0; c < n_cts; c++) {
        g1 u; g2 w, h;
        int ok = g1_load(&u, cts_u + 48 * c) && g2_load(&w, cts_w + 96 * c);
        ok = ok && hash_to_g2_tpke(&h, &u, cts_v + vlen * c, vlen);
        ctok[c] = (uint8_t)ok;
        if (!ok) { memset(&h, 0, sizeof h); memset(&w, 0, sizeof w); }
        lines_precompute(LH + OLINES * c, &h);
        lines_precompute(LW + OLINES * c, &w);
        lines_normalise(LH + OLINES * c);
        lines_normalise(LW + OLINES * c);
    }
#pragma omp parallel for schedule(static) num_threads(nthreads)
    for (size_t d = 0; d < n_keys; d++) {
        kok[d] = (uint8_t)g1_load(&Y[d], y_keys + 48 * d);
        if (kok[d]) g1_neg(&Y[d], &Y[d]);   /* -Y: e(Ui, H) e(-Yi, W) == 1 */
    }
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthreads)
    for (size_t i = 0; i < n; i++) {
        uint32_t c = ct_idx[i], d = dec_idx[i];
        g1 ui;
        int ok = c < n_cts && d < n_keys && ctok[c] && kok[d] && g1_load(&ui, uis + 48 * i);
        accept[i] = (uint8_t)(ok && check_pair_product(LH + OLINES * c, &ui, LW + OLINES * c, &Y[d]));
    }
    free(LH); free(LW); free(ctok); free(Y); free(kok);
    return 0;
}
int orc_ts_validate_batch_amortized(uint8_t *accept, size_t n, const uint8_t *pks, size_t n_pks, const uint8_t *sigs,
                                    const uint8_t *msgs, const uint32_t *msg_off, size_t n_msgs,
                                    const uint32_t *msg_idx, const uint32_t *pk_idx, int nthreads) {
    orc_init();
    oline *LH = malloc(sizeof(oline) * OLINES * (n_msgs ? n_msgs : 1));
    uint8_t *mok = malloc(n_msgs ? n_msgs : 1);
    if (!LH || !mok) { free(LH); free(mok); return -1; }
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
    for (size_t m = 0; m < n_msgs; m++) {
        g2 h;
        int ok = g2_hash(&h, msgs + msg_off[m], msg_off[m + 1] - msg_off[m]);
        mok[m] = (uint8_t)ok;
        if (!ok) memset(&h, 0, sizeof h);
        lines_precompute(LH + OLINES * m, &h);
        lines_normalise(LH + OLINES * m);
    }
    g1 ngen;
    g1_neg(&ngen, &G1_GEN);
#pragma omp parallel for schedule(dynamic, 4) num_threads(nthreads)
    for (size_t i = 0; i < n; i++) {
        uint32_t m = msg_idx[i], k = pk_idx[i];
        g1 pk; g2 sig;
        oline LS[OLINES];
        int ok = m < n_msgs && k < n_pks && mok[m] && g1_load(&pk, pks + 48 * (size_t)k) && g2_load(&sig, sigs + 96 * i);
        if (ok) lines_precompute(LS, &sig);   /* the signature side's lines, once per share (on the fly on the GPU) */
        accept[i] = (uint8_t)(ok && check_pair_product(LH + OLINES * m, &pk, LS, &ngen));
    }
    free(LH); free(mok);
    return 0;
}

/* ================================================================== CPU baseline, randomized batch (k_batch.hip)
   The GPU's batched algorithm restated for the host cores: groups = runs of one ciphertext (<= 32 shares), exponents
   s_i = a_i + b_i lambda from 32-bit a_i, b_i (splitmix64 from `seed`: the cost of the GPU's ChaCha20 is negligible
   beside the curve arithmetic; this leg is timing and parity, not a randomness source), one two-pair Miller loop +
   final exponentiation per group, for a failed group the weighted re-check and the level-2 search, single checks when
   the search names no share.  Decisions equal orc_tpke_verify_batch's (tests/test_oracle.py). */
static fp G1_BETA_O;
static int g1_beta_ready = 0;
static void g1_beta_init(void) {
    if (g1_beta_ready) return;
    /* the cube root of unity beta with (beta x, y) = lambda (x, y) on the r-torsion, lambda = z^2 - 1 */
    u64 e[NP];
    u128 rem = 0;
    for (int j = NP - 1; j >= 0; j--) {   /* (p - 1) / 3 */
        u128 cur = (rem << 64) | (j == 0 ? P[0] - 1 : P[j]);
        e[j] = (u64)(cur / 3);
        rem = cur % 3;
    }
    fp two, c, c2;
    fp_set_u64(&two, 2);
    fp_pow(&c, &two, e, NP);
    fp_mul(&c2, &c, &c);
    u64 lam[2];
    u128 z2 = (u128)Z_ABS * Z_ABS - 1;
    lam[0] = (u64)z2;
    lam[1] = (u64)(z2 >> 64);
    g1 t;
    g1_mul_int(&t, &G1_GEN, lam, 2);
    fp tx, ty, gx, gy, bx;
    g1_to_affine(&tx, &ty, &t);
    g1_to_affine(&gx, &gy, &G1_GEN);
    fp_mul(&bx, &gx, &c);
    G1_BETA_O = fp_eq(&bx, &tx) ? c : c2;
    g1_beta_ready = 1;
}
/* p + (qx, qy), q affine and finite (madd-2007-bl; the doubling / inverse cases through the full addition) */
static void g1_madd(g1 *r, const g1 *p, const fp *qx, const fp *qy) {
    g1 q;
    q.x = *qx; q.y = *qy; q.z = FP_ONE_M;
    if (g1_is_inf(p)) { *r = q; return; }
    fp z1z1, u2, s2, h, hh, i4, j, rr, v, t;
    fp_sqr(&z1z1, &p->z);
    fp_mul(&u2, qx, &z1z1);
    fp_mul(&s2, qy, &p->z);
    fp_mul(&s2, &s2, &z1z1);
    if (fp_eq(&u2, &p->x)) { g1_add(r, p, &q); return; }
    fp_sub(&h, &u2, &p->x);
    fp_sqr(&hh, &h);
    fp_add(&i4, &hh, &hh);
    fp_add(&i4, &i4, &i4);
    fp_mul(&j, &h, &i4);
    fp_sub(&rr, &s2, &p->y);
    fp_add(&rr, &rr, &rr);
    fp_mul(&v, &p->x, &i4);
    g1 o;
    fp_sqr(&o.x, &rr);
    fp_sub(&o.x, &o.x, &j);
    fp_sub(&o.x, &o.x, &v);
    fp_sub(&o.x, &o.x, &v);
    fp_sub(&t, &v, &o.x);
    fp_mul(&o.y, &rr, &t);
    fp_mul(&t, &p->y, &j);
    fp_add(&t, &t, &t);
    fp_sub(&o.y, &o.y, &t);
    fp_add(&o.z, &p->z, &h);
    fp_sqr(&o.z, &o.z);
    fp_sub(&o.z, &o.z, &z1z1);
    fp_sub(&o.z, &o.z, &hh);
    *r = o;
}
/* a P + b phi(P): 32 shared doublings */
static void g1_mul_ab(g1 *r, const g1 *P_, uint32_t a, uint32_t b) {
    g1_set_inf(r);
    if (g1_is_inf(P_)) return;
    fp x, y, px;
    g1_to_affine(&x, &y, P_);
    fp_mul(&px, &x, &G1_BETA_O);
    for (int k = 31; k >= 0; k--) {
        g1_dbl(r, r);
        if ((a >> k) & 1) g1_madd(r, r, &x, &y);
        if ((b >> k) & 1) g1_madd(r, r, &px, &y);
    }
}
static u64 splitmix64(u64 *st) {
    u64 z = (*st += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
/* e = final_exp(Miller(P1 on L1) Miller(P2 on L2)) */
static void pair_product_gt(fp12 *e, const oline *L1, const g1 *P1, const oline *L2, const g1 *P2) {
    fp12 f;
    miller2_lines(&f, L1, P1, L2, P2);
    final_exp(e, &f);
}
/* Level 2 search (k_rlc_search): gamma' == gamma^c for c = 1..len names the group's only bad share (index c - 1) */
static int rlc_search(const fp12 *gm, const fp12 *gp, size_t len) {
    fp12 acc = *gm;
    for (size_t c = 1; c <= len; c++) {
        if (fp12_eq(&acc, gp)) return (int)c;
        fp12_mul(&acc, &acc, gm);
    }
    return 0;
}
/* a^e for a small exponent e >= 1 */
static void fp12_pow_small(fp12 *r, const fp12 *a, unsigned e) {
    fp12 t = *a;
    int top = 31;
    while (top > 0 && !((e >> top) & 1)) top--;
    for (int b = top - 1; b >= 0; b--) {
        fp12_sqr(&t, &t);
        if ((e >> b) & 1) fp12_mul(&t, &t, a);
    }
    *r = t;
}
/* Level 2, two-error location (k_tpke_rlc_search2b): with gamma_0 = gm, gamma_c = gp (weights c_j = j + 1) and
   gamma_t = gt (weights t_j = c_j (c_j + 1) / 2), D_j = gamma_c / gamma_0^(c_j) and E_j = gamma_t^2 / gamma_c^(c_j + 1);
   E_j = D_j^(c_k) (c_k != c_j) names the partner k of bad share j.  Returns 1 and the two shares when exactly two
   shares name each other. */
static int rlc_search2(const fp12 *gm, const fp12 *gp, const fp12 *gt, size_t len, size_t *j0, size_t *j1) {
    unsigned found[32] = {0};
    fp12 t2;
    fp12_sqr(&t2, gt);
    size_t nf = 0;
    for (size_t j = 0; j < len && j < 32; j++) {
        fp12 b, D, E, acc;
        fp12_pow_small(&b, gm, (unsigned)j + 1);
        fp12_conj(&b, &b);
        fp12_mul(&D, gp, &b);
        fp12_pow_small(&b, gp, (unsigned)j + 2);
        fp12_conj(&b, &b);
        fp12_mul(&E, &t2, &b);
        acc = D;
        for (size_t c = 1; c <= len; c++) {
            if (c != j + 1 && fp12_eq(&acc, &E)) { found[j] = (unsigned)c; break; }
            fp12_mul(&acc, &acc, &D);
        }
        if (found[j]) { if (nf == 0) *j0 = j; else *j1 = j; nf++; }
    }
    return nf == 2 && found[*j0] == *j1 + 1 && found[*j1] == *j0 + 1;
}
/* the GPU's level structure on one group (k_batch.hip): the group check; if it fails, the weighted re-checks with
   weights c_j = j+1 and t_j = c_j (c_j + 1) / 2, the one-error search, then the two-error location; if that names no
   pair, single checks of every share */
static void rlc_check_group(uint8_t *accept, const g1 *sU, const g1 *sY, size_t st, size_t len, const oline *LH,
                            const oline *LW) {
    g1 a, b, wa, wb, va, vb;
    g1_set_inf(&a); g1_set_inf(&b); g1_set_inf(&wa); g1_set_inf(&wb); g1_set_inf(&va); g1_set_inf(&vb);
    for (size_t j = st + len; j-- > st;) {       /* suffix sums: wa = sum c_j sU_j, va = sum t_j sU_j */
        g1_add(&a, &a, &sU[j]);
        g1_add(&b, &b, &sY[j]);
        g1_add(&wa, &wa, &a);
        g1_add(&wb, &wb, &b);
        g1_add(&va, &va, &wa);
        g1_add(&vb, &vb, &wb);
    }
    fp12 gm, gp, gt;
    pair_product_gt(&gm, LH, &a, LW, &b);
    if (fp12_eq(&gm, &FP12_ONE)) return;                 /* every (valid) share of the group accepted */
    if (len == 1) { accept[st] = 0; return; }
    pair_product_gt(&gp, LH, &wa, LW, &wb);
    pair_product_gt(&gt, LH, &va, LW, &vb);
    int c = rlc_search(&gm, &gp, len);
    if (c) { accept[st + c - 1] = 0; return; }
    size_t j0 = 0, j1 = 0;
    if (rlc_search2(&gm, &gp, &gt, len, &j0, &j1)) { accept[st + j0] = 0; accept[st + j1] = 0; return; }
    for (size_t j = st; j < st + len; j++)
        if (!check_pair_product(LH, &sU[j], LW, &sY[j])) accept[j] = 0;
}
int orc_tpke_verify_batch_rlc(uint8_t *accept, size_t n, const uint8_t *y_keys, size_t n_keys, const uint8_t *cts_u,
                              const uint8_t *cts_v, size_t vlen, const uint8_t *cts_w, size_t n_cts,
                              const uint32_t *ct_idx, const uint32_t *dec_idx, const uint8_t *uis, uint64_t seed,
                              int nthreads) {
    orc_init();
    g1_beta_init();
    oline *LH = malloc(sizeof(oline) * OLINES * (n_cts ? n_cts : 1));
    oline *LW = malloc(sizeof(oline) * OLINES * (n_cts ? n_cts : 1));
    uint8_t *ctok = malloc(n_cts ? n_cts : 1);
    g1 *Y = malloc(sizeof(g1) * (n_keys ? n_keys : 1));
    uint8_t *kok = malloc(n_keys ? n_keys : 1);
    g1 *sU = malloc(sizeof(g1) * (n ? n : 1)), *sY = malloc(sizeof(g1) * (n ? n : 1));
    size_t *gst = malloc(sizeof(size_t) * (n + 1));
    if (!LH || !LW || !ctok || !Y || !kok || !sU || !sY || !gst) {
        free(LH); free(LW); free(ctok); free(Y); free(kok); free(sU); free(sY); free(gst);
        return -1;
    }
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
    for (size_t c = 0; c < n_cts; c++) {
        g1 u; g2 w, h;
        int ok = g1_load(&u, cts_u + 48 * c) && g2_load(&w, cts_w + 96 * c);
        ok = ok && hash_to_g2_tpke(&h, &u, cts_v + vlen * c, vlen);
        ctok[c] = (uint8_t)ok;
        if (!ok) { memset(&h, 0, sizeof h); memset(&w, 0, sizeof w); }
        lines_precompute(LH + OLINES * c, &h);
        lines_precompute(LW + OLINES * c, &w);
        lines_normalise(LH + OLINES * c);
        lines_normalise(LW + OLINES * c);
    }
#pragma omp parallel for schedule(static) num_threads(nthreads)
    for (size_t d = 0; d < n_keys; d++) {
        kok[d] = (uint8_t)g1_load(&Y[d], y_keys + 48 * d);
        if (kok[d]) g1_neg(&Y[d], &Y[d]);   /* -Y: e(sum s U, H) e(-sum s Y, W) == 1 */
    }
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads)
    for (size_t i = 0; i < n; i++) {
        uint32_t c = ct_idx[i], d = dec_idx[i];
        g1 ui;
        int ok = c < n_cts && d < n_keys && ctok[c] && kok[d] && g1_load(&ui, uis + 48 * i);
        accept[i] = (uint8_t)ok;
        if (!ok) { g1_set_inf(&sU[i]); g1_set_inf(&sY[i]); continue; }
        u64 st = seed ^ (0x9E3779B97F4A7C15ULL * (i + 1));
        u64 r = splitmix64(&st);
        uint32_t a = (uint32_t)r, b = (uint32_t)(r >> 32);
        if ((a | b) == 0) a = 1;
        g1_mul_ab(&sU[i], &ui, a, b);
        g1_mul_ab(&sY[i], &Y[d], a, b);
    }
    size_t ng = 0;                                    /* runs of one ciphertext, at most 32 shares */
    for (size_t i = 0; i < n;) {
        size_t j = i + 1;
        while (j < n && j - i < 32 && ct_idx[j] == ct_idx[i]) j++;
        gst[ng++] = i;
        i = j;
    }
    gst[ng] = n;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
    for (size_t g = 0; g < ng; g++) {
        size_t c = ct_idx[gst[g]];
        if (c >= n_cts) continue;                     /* its shares are already rejected */
        rlc_check_group(accept, sU, sY, gst[g], gst[g + 1] - gst[g], LH + OLINES * c, LW + OLINES * c);
    }
    free(LH); free(LW); free(ctok); free(Y); free(kok); free(sU); free(sY); free(gst);
    return 0;
}

/* G2 membership as the GPU tests it (Scott: psi(P) == [z] P = -[|z|] P on G2), for the batched CPU legs */
static int g2_in_subgroup_psi(const g2 *P_) {
    if (g2_is_inf(P_)) return 1;
    g2 t, ps;
    g2_mul_u64(&t, P_, Z_ABS);
    g2_neg(&t, &t);
    g2_psi(&ps, P_);
    return g2_eq(&ps, &t);
}
int orc_g2_in_subgroup_psi(const uint8_t a[96]) {
    orc_init();
    g2 p;
    if (!g2_load(&p, a)) return 0;
    return g2_in_subgroup_psi(&p);
}
/* (a + b lambda) S = (a - b) S + b psi^2(S) on G2 */
static void g2_mul_ab(g2 *r, const g2 *S, uint32_t a, uint32_t b) {
    g2_set_inf(r);
    if (g2_is_inf(S)) return;
    g2 s2, p1;
    g2_psi(&s2, S);
    g2_psi(&s2, &s2);
    p1 = *S;
    uint32_t d = a - b;
    if (a < b) { d = b - a; g2_neg(&p1, &p1); }
    for (int k = 31; k >= 0; k--) {
        g2_dbl(r, r);
        if ((d >> k) & 1) g2_add(r, r, &p1);
        if ((b >> k) & 1) g2_add(r, r, &s2);
    }
}
static void ts_rlc_check_group(uint8_t *accept, const g1 *sP, const g2 *sS, const uint8_t *exact, size_t st,
                               size_t len, const oline *LH, const g1 *ngen, const g1 *pkv, const g2 *sigv) {
    g1 a, wa;
    g2 b, wb;
    g1_set_inf(&a); g1_set_inf(&wa); g2_set_inf(&b); g2_set_inf(&wb);
    for (size_t j = st + len; j-- > st;) {
        if (!exact[j]) {
            g1_add(&a, &a, &sP[j]);
            g2_add(&b, &b, &sS[j]);
        }
        g1_add(&wa, &wa, &a);
        g2_add(&wb, &wb, &b);
    }
    oline LS[OLINES];
    fp12 gm, gp;
    lines_precompute(LS, &b);
    pair_product_gt(&gm, LH, &a, LS, ngen);
    if (fp12_eq(&gm, &FP12_ONE)) return;
    int c = 0;
    if (len > 1) {
        lines_precompute(LS, &wb);
        pair_product_gt(&gp, LH, &wa, LS, ngen);
        c = rlc_search(&gm, &gp, len);
    }
    if (c) { accept[st + c - 1] = 0; return; }
    for (size_t j = st; j < st + len; j++) {
        if (!accept[j] || exact[j]) continue;
        lines_precompute(LS, &sigv[j]);
        if (!check_pair_product(LH, &pkv[j], LS, ngen)) accept[j] = 0;
    }
}
/* CPU baseline with the GPU's batched threshold-signature algorithm (k_batch.hip): groups = runs of one message
   (<= 128 shares), s_i = a_i + b_i lambda (splitmix64, see orc_tpke_verify_batch_rlc), signatures outside G2 checked
   exactly, the level-2 search, single checks when it names no share */
int orc_ts_validate_batch_rlc(uint8_t *accept, size_t n, const uint8_t *pks, size_t n_pks, const uint8_t *sigs,
                              const uint8_t *msgs, const uint32_t *msg_off, size_t n_msgs, const uint32_t *msg_idx,
                              const uint32_t *pk_idx, uint64_t seed, int nthreads) {
    orc_init();
    g1_beta_init();
    oline *LH = malloc(sizeof(oline) * OLINES * (n_msgs ? n_msgs : 1));
    uint8_t *mok = malloc(n_msgs ? n_msgs : 1), *exact = malloc(n ? n : 1);
    g1 *sP = malloc(sizeof(g1) * (n ? n : 1)), *pkv = malloc(sizeof(g1) * (n ? n : 1));
    g2 *sS = malloc(sizeof(g2) * (n ? n : 1)), *sigv = malloc(sizeof(g2) * (n ? n : 1));
    size_t *gst = malloc(sizeof(size_t) * (n + 1));
    if (!LH || !mok || !exact || !sP || !pkv || !sS || !sigv || !gst) {
        free(LH); free(mok); free(exact); free(sP); free(pkv); free(sS); free(sigv); free(gst);
        return -1;
    }
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
    for (size_t m = 0; m < n_msgs; m++) {
        g2 h;
        int ok = g2_hash(&h, msgs + msg_off[m], msg_off[m + 1] - msg_off[m]);
        mok[m] = (uint8_t)ok;
        if (!ok) memset(&h, 0, sizeof h);
        lines_precompute(LH + OLINES * m, &h);
        lines_normalise(LH + OLINES * m);
    }
    g1 ngen;
    g1_neg(&ngen, &G1_GEN);
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads)
    for (size_t i = 0; i < n; i++) {
        uint32_t m = msg_idx[i], k = pk_idx[i];
        int ok = m < n_msgs && k < n_pks && mok[m] && g1_load(&pkv[i], pks + 48 * (size_t)k) &&
                 g2_load(&sigv[i], sigs + 96 * i);
        accept[i] = (uint8_t)ok;
        exact[i] = 0;
        g1_set_inf(&sP[i]);
        g2_set_inf(&sS[i]);
        if (!ok) continue;
        if (!g2_in_subgroup_psi(&sigv[i])) {      /* exact check, as the GPU's desc.w = 1 singles */
            oline LS[OLINES];
            exact[i] = 1;
            lines_precompute(LS, &sigv[i]);
            accept[i] = (uint8_t)check_pair_product(LH + OLINES * m, &pkv[i], LS, &ngen);
            continue;
        }
        u64 st = seed ^ (0x9E3779B97F4A7C15ULL * (i + 1));
        u64 r = splitmix64(&st);
        uint32_t a = (uint32_t)r, b = (uint32_t)(r >> 32);
        if ((a | b) == 0) a = 1;
        g1_mul_ab(&sP[i], &pkv[i], a, b);
        g2_mul_ab(&sS[i], &sigv[i], a, b);
    }
    size_t ng = 0;
    for (size_t i = 0; i < n;) {
        size_t j = i + 1;
        while (j < n && j - i < 128 && msg_idx[j] == msg_idx[i]) j++;
        gst[ng++] = i;
        i = j;
    }
    gst[ng] = n;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
    for (size_t g = 0; g < ng; g++) {
        size_t m = msg_idx[gst[g]];
        if (m >= n_msgs || !mok[m]) continue;          /* its shares are already rejected */
        ts_rlc_check_group(accept, sP, sS, exact, gst[g], gst[g + 1] - gst[g], LH + OLINES * m, &ngen, pkv, sigv);
    }
    free(LH); free(mok); free(exact); free(sP); free(pkv); free(sS); free(sigv); free(gst);
    return 0;
}

/* ---- test hooks (oracle self-checks) ---- */
int orc_test_cyc_sqr(uint8_t out[576], const uint8_t fb[576]) {
    orc_init();
    fp12 f, t;
    if (!gt_deser(&f, fb)) return -1;
    fe_easy(&t, &f);
    fp12 a, b;
    fp12_cyc_sqr(&a, &t);
    fp12_sqr(&b, &t);
    gt_ser(out, &a);
    return fp12_eq(&a, &b) ? 0 : 1;
}
int orc_test_sparse_line(const uint8_t fb[576], const uint8_t abc[288]) {
    orc_init();
    fp12 f, g;
    if (!gt_deser(&f, fb)) return -1;
    fp2 A, Bc, C;
    fp_from_bytes_canon(&A.a, abc); fp_from_bytes_canon(&A.b, abc + 48);
    fp_from_bytes_canon(&Bc.a, abc + 96); fp_from_bytes_canon(&Bc.b, abc + 144);
    fp_from_bytes_canon(&C.a, abc + 192); fp_from_bytes_canon(&C.b, abc + 240);
    g = f;
    fp12_mul_line(&f, &A, &Bc, &C);
    fp12_mul_line_generic(&g, &A, &Bc, &C);
    return fp12_eq(&f, &g) ? 0 : 1;
}
/* Fp-mul counts of the canonical work units, measured on this restatement:
   out[0] C_ML1_EVAL  one-pair Miller loop, evaluation side only (lines precomputed)
   out[1] C_ML2_EVAL  two-pair Miller loop with shared squarings, evaluation side only
   out[2] C_LINES     line generation for one G2 point (63 doubling + 5 addition steps)
   out[3] C_FE        final exponentiation (easy part incl. one Fp inversion + hard part)
   out[4] C_H2G2      hash-and-map to G2 (SHA-512 not counted)
   out[5] C_DEC1      G1 decompression from 48 bytes
   out[6] C_DEC2      G2 decompression from 96 bytes
   out[7] C_MUL1      255-bit G1 variable-base scalar multiplication (4-bit window, Jacobian)
   out[8] C_MUL2      255-bit G2 variable-base scalar multiplication
   out[9] C_AFF2      Jacobian -> affine conversion of a G2 point (one Fp2 inversion) */
int orc_count_units(uint64_t out[10]) {
    orc_init();
    g1 P1 = G1_GEN, P2; g2 Q1 = G2_GEN, Q2;
    g1_dbl(&P2, &P1); g1_normalize(&P2);
    g2_dbl(&Q2, &Q1); g2_normalize(&Q2);
    g1 Ps[2] = {P1, P2}; g2 Qs[2] = {Q1, Q2};
    fp12 f, r;
    orc_count_reset(); g_line_count = 0; miller_multi(&f, Ps, Qs, 1);
    out[2] = g_line_count; out[0] = orc_count_get() - g_line_count;
    orc_count_reset(); g_line_count = 0; miller_multi(&f, Ps, Qs, 2);
    out[1] = orc_count_get() - g_line_count;
    orc_count_reset(); final_exp(&r, &f); out[3] = orc_count_get();
    g2 h; orc_count_reset(); g2_hash(&h, (const uint8_t *)"lachain", 7); out[4] = orc_count_get();
    uint8_t b1[48], b2[96]; g1_ser(b1, &P2); g2_ser(b2, &Q2);
    g1 d1; g2 d2;
    orc_count_reset(); g1_deser(&d1, b1); out[5] = orc_count_get();
    orc_count_reset(); g2_deser(&d2, b2); out[6] = orc_count_get();
    fr s; u64 sv[NR] = {0x0123456789abcdefULL, 0xfedcba9876543210ULL, 0x0f0f0f0f0f0f0f0fULL, 0x3333333333333333ULL};
    fr_from_int(&s, sv);
    orc_count_reset(); g1_mul_fr(&d1, &P2, &s); out[7] = orc_count_get();
    orc_count_reset(); g2_mul_fr(&d2, &Q2, &s); out[8] = orc_count_get();
    fp2 ax, ay; orc_count_reset(); g2_to_affine(&ax, &ay, &d2); out[9] = orc_count_get();
    g_counting = 0;
    return 0;
}

/* ================================================================== CPU Pippenger MSM (bench CPU leg)
   The bucket method the GPU runs (k_msm.hip), on the host cores: signed c-bit digits of the 255-bit scalars, per
   (window, slice of the points) task 2^(c-1) Jacobian buckets filled with mixed additions, a running-sum bucket
   reduction per task, the task sums added per window and the windows combined by Horner (c doublings each).  The
   points are decompressed beforehand (orc_g1_affine_batch; the GPU's points are resident affine records too), so the
   timed part is the same algorithm as the GPU's plain form.  Result equals orc_g1_msm (tests/test_oracle.py). */
typedef struct { fp x, y; } g1aff_o;
int orc_g1_affine_batch(uint8_t *aff, const uint8_t *pts, size_t n, int nthreads) {
    orc_init();
    if (nthreads < 1) nthreads = 1;
    g1aff_o *a = (g1aff_o *)aff;
    int bad = 0;
#pragma omp parallel for num_threads(nthreads) schedule(static) reduction(| : bad)
    for (size_t i = 0; i < n; i++) {
        g1 p;
        if (!g1_load(&p, pts + 48 * i)) { bad = 1; continue; }
        if (g1_is_inf(&p)) { memset(&a[i], 0, sizeof a[i]); continue; }   /* (0, 0) is not on the curve: infinity */
        g1_to_affine(&a[i].x, &a[i].y, &p);
    }
    return bad ? -1 : 0;
}
size_t orc_g1_affine_bytes(void) { return sizeof(g1aff_o); }
static int aff_is_inf(const g1aff_o *p) { return fp_is_zero(&p->x) && fp_is_zero(&p->y); }
int orc_g1_msm_pippenger(uint8_t out[48], const uint8_t *aff, const uint8_t *scalars, size_t n, int c, int nthreads) {
    orc_init();
    if (nthreads < 1) nthreads = 1;
    if (c < 2 || c > 20) return -1;
    const g1aff_o *a = (const g1aff_o *)aff;
    const int nwin = (256 + c - 1) / c + 1;                 /* one more window for the last signed carry */
    const size_t nb = (size_t)1 << (c - 1);
    /* signed digits, window-major: d[w * n + i] in [-2^(c-1), 2^(c-1)] */
    int32_t *dg = malloc(sizeof(int32_t) * (size_t)nwin * (n ? n : 1));
    if (!dg) return -1;
    int bad = 0;
#pragma omp parallel for num_threads(nthreads) schedule(static) reduction(| : bad)
    for (size_t i = 0; i < n; i++) {
        u64 s[4];
        memcpy(s, scalars + 32 * i, 32);
        if (bn_cmp(s, R_, NR) >= 0) { bad = 1; continue; }
        int carry = 0;
        for (int w = 0; w < nwin; w++) {
            int v = carry;
            for (int k = 0; k < c; k++) {
                int bit = w * c + k;
                if (bit < 256) v += (int)((s[bit >> 6] >> (bit & 63)) & 1) << k;
            }
            carry = v > (1 << (c - 1));
            if (carry) v -= 1 << c;
            dg[(size_t)w * n + i] = v;
        }
    }
    if (bad) { free(dg); return -1; }
    int splits = (2 * nthreads + nwin - 1) / nwin;
    if ((size_t)splits > n / 1024 + 1) splits = (int)(n / 1024 + 1);
    const int ntask = nwin * splits;
    g1 *tsum = malloc(sizeof(g1) * ntask);
    if (!tsum) { free(dg); return -1; }
#pragma omp parallel num_threads(nthreads)
    {
        g1 *bk = malloc(sizeof(g1) * nb);
#pragma omp for schedule(dynamic, 1)
        for (int t = 0; t < ntask; t++) {
            const int w = t / splits, sp = t % splits;
            const size_t lo = n * (size_t)sp / splits, hi = n * (size_t)(sp + 1) / splits;
            for (size_t b = 0; b < nb; b++) g1_set_inf(&bk[b]);
            const int32_t *d = dg + (size_t)w * n;
            for (size_t i = lo; i < hi; i++) {
                int v = d[i];
                if (!v || aff_is_inf(&a[i])) continue;
                if (v > 0) g1_madd(&bk[v - 1], &bk[v - 1], &a[i].x, &a[i].y);
                else {
                    fp ny;
                    fp_neg(&ny, &a[i].y);
                    g1_madd(&bk[-v - 1], &bk[-v - 1], &a[i].x, &ny);
                }
            }
            g1 run, acc;                                    /* sum_b (b + 1) bk[b] by running sums */
            g1_set_inf(&run);
            g1_set_inf(&acc);
            for (size_t b = nb; b-- > 0;) {
                g1_add(&run, &run, &bk[b]);
                g1_add(&acc, &acc, &run);
            }
            tsum[t] = acc;
        }
        free(bk);
    }
    g1 res;
    g1_set_inf(&res);
    for (int w = nwin - 1; w >= 0; w--) {
        for (int k = 0; k < c; k++) g1_dbl(&res, &res);
        for (int sp = 0; sp < splits; sp++) g1_add(&res, &res, &tsum[w * splits + sp]);
    }
    free(tsum);
    free(dg);
    g1_ser(out, &res);
    return 0;
}
