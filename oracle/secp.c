/* oracle/secp.c — TEST INFRASTRUCTURE ONLY: CPU restatement of the secp256k1 ECDSA header-signature check of
 * Lachain's root protocol.
 *
 * Reference path: RootProtocol verifies every SignedHeaderMessage with
 *   _crypto.VerifySignatureHashed(header.Keccak(), signature.Encode(), EcdsaPublicKeySet[idx].EncodeCompressed(),
 *                                 _useNewChainId)            (src/Lachain.Consensus/RootProtocol/RootProtocol.cs:91-105)
 * DefaultCrypto.VerifySignatureHashed (src/Lachain.Crypto/DefaultCrypto.cs:79-101):
 *   - hash must be 32 bytes and the signature SignatureSize(useNewChainId) = 65 / 66 bytes (DefaultCrypto.cs:26-29);
 *   - Secp256K1.PublicKeyParse(publicKey) must succeed;
 *   - recId = (RestoreEncodedRecIdFromSignatureBuffer(sig) - 36) / 2 / ChainId(useNewChainId) in C# int arithmetic
 *     (truncating division; chain id 0 throws), must be in [0, 3] (an exception, caught by RootProtocol.cs:103 as
 *     "not verified"); the encoded id is sig[64] (65 B) or sig[64] * 256 + sig[65] (66 B) (DefaultCrypto.cs:31-44);
 *   - RecoverableSignatureParseCompact(sig[0..64), recId), then Secp256K1.Verify(sig[0..64), hash, pk).
 * The secp256k1 calls go to the Secp256k1.Net 0.1.55 / Secp256k1.Native 0.1.20 NuGet packages
 * (src/Lachain.Crypto/Lachain.Crypto.csproj:21-22), i.e. bitcoin-core libsecp256k1, which is NOT in the reference
 * tree.  Restated from its published algorithm:
 *   - pubkey parse: 33 B 0x02/0x03 || x (x < p, x^3 + 7 must be a square; y of the given parity) or 65 B
 *     0x04/0x06/0x07 || x || y (x, y < p, on the curve; for 0x06/0x07 the parity of y must match the tag);
 *   - compact signature parse: r, s 32 B big-endian each, rejected when >= n (zero is accepted at parse);
 *   - verify: reject high s (s > n/2, lower-S rule), r = 0 or s = 0; m = hash (big-endian) mod n;
 *     R = (m/s) G + (r/s) Q; reject R = infinity; accept iff x(R) mod n == r.
 * Pinned by the reference's own known answers (tests/golden/secp256k1_kats.json, made by
 * tests/golden/make_secp256k1_kats.py from test/Lachain.CryptoTest/CryptographyTest.cs): the private key -> address
 * pair (:176-178, :238-256), four reference-produced EIP-155 signatures of known transactions (Test_TxHash2 :251-271
 * and Test_External_Signature :334-380) that must verify, the Keccak-256 vector (:68-73) and the header hash of
 * Test_HeaderKeccak (:115-128).
 *
 * Arithmetic: 4 x 64-bit limbs, Montgomery form (one generic CIOS routine for p and for n), __int128 products.
 * Scalar multiplication for the timing leg: Straus-Shamir joint double-and-add with 4-bit windows over G and Q.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t u64;
typedef unsigned __int128 u128;

typedef struct { u64 m[4]; u64 inv; u64 r2[4]; u64 one[4]; } mod_t;   /* inv = -m^-1 mod 2^64 */
static mod_t MP, MN;
static int g_init = 0;

static const u64 P_[4] = {0xFFFFFFFEFFFFFC2FULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL};
static const u64 N_[4] = {0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL};
static const u64 NH_[4] = {0xDFE92F46681B20A0ULL, 0x5D576E7357A4501DULL, 0xFFFFFFFFFFFFFFFFULL, 0x7FFFFFFFFFFFFFFFULL}; /* n/2 */
static const u64 GX_[4] = {0x59F2815B16F81798ULL, 0x029BFCDB2DCE28D9ULL, 0x55A06295CE870B07ULL, 0x79BE667EF9DCBBACULL};
static const u64 GY_[4] = {0x9C47D08FFB10D4B8ULL, 0xFD17B448A6855419ULL, 0x5DA4FBFC0E1108A8ULL, 0x483ADA7726A3C465ULL};

/* ---------------------------------------------------------------- 256-bit integers */
static int cmp4(const u64 *a, const u64 *b) {
    for (int i = 3; i >= 0; i--) {
        if (a[i] > b[i]) return 1;
        if (a[i] < b[i]) return -1;
    }
    return 0;
}
static int is_zero4(const u64 *a) { return !(a[0] | a[1] | a[2] | a[3]); }
static u64 add4(u64 *r, const u64 *a, const u64 *b) {
    u128 c = 0;
    for (int i = 0; i < 4; i++) { c += (u128)a[i] + b[i]; r[i] = (u64)c; c >>= 64; }
    return (u64)c;
}
static u64 sub4(u64 *r, const u64 *a, const u64 *b) {
    u64 br = 0;
    for (int i = 0; i < 4; i++) {
        u128 d = (u128)a[i] - b[i] - br;
        r[i] = (u64)d;
        br = (u64)(d >> 64) & 1;
    }
    return br;
}
static void from_be32(u64 *r, const uint8_t *b) {
    for (int i = 0; i < 4; i++) {
        u64 v = 0;
        for (int j = 0; j < 8; j++) v = (v << 8) | b[(3 - i) * 8 + j];
        r[i] = v;
    }
}
static void to_be32(uint8_t *b, const u64 *r) {
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) b[(3 - i) * 8 + j] = (uint8_t)(r[i] >> (56 - 8 * j));
}

/* ---------------------------------------------------------------- Montgomery arithmetic mod m (m < 2^256, odd) */
static void mmul(const mod_t *M, u64 *r, const u64 *a, const u64 *b) {
    u64 t[6] = {0};
    for (int i = 0; i < 4; i++) {
        u128 c = 0;
        for (int j = 0; j < 4; j++) { c += (u128)a[j] * b[i] + t[j]; t[j] = (u64)c; c >>= 64; }
        c += t[4]; t[4] = (u64)c; t[5] = (u64)(c >> 64);
        u64 q = t[0] * M->inv;
        c = ((u128)q * M->m[0] + t[0]) >> 64;
        for (int j = 1; j < 4; j++) { c += (u128)q * M->m[j] + t[j]; t[j - 1] = (u64)c; c >>= 64; }
        c += t[4]; t[3] = (u64)c; t[4] = t[5] + (u64)(c >> 64);
    }
    u64 s[4];
    u64 br = sub4(s, t, M->m);
    if (t[4] || !br) memcpy(r, s, 32); else memcpy(r, t, 32);
}
static void madd(const mod_t *M, u64 *r, const u64 *a, const u64 *b) {
    u64 s[4], c = add4(r, a, b);
    if (c || cmp4(r, M->m) >= 0) { sub4(s, r, M->m); memcpy(r, s, 32); }
}
static void msub(const mod_t *M, u64 *r, const u64 *a, const u64 *b) {
    if (sub4(r, a, b)) add4(r, r, M->m);
}
static void mto(const mod_t *M, u64 *r, const u64 *a) { mmul(M, r, a, M->r2); }          /* a < m */
static void mfrom(const mod_t *M, u64 *r, const u64 *a) { u64 one[4] = {1, 0, 0, 0}; mmul(M, r, a, one); }
static void mpow(const mod_t *M, u64 *r, const u64 *a, const u64 *e) {   /* Montgomery in/out, plain exponent */
    u64 acc[4];
    memcpy(acc, M->one, 32);
    for (int i = 255; i >= 0; i--) {
        mmul(M, acc, acc, acc);
        if ((e[i / 64] >> (i % 64)) & 1) mmul(M, acc, acc, a);
    }
    memcpy(r, acc, 32);
}
static void minv(const mod_t *M, u64 *r, const u64 *a) {
    u64 e[4], two[4] = {2, 0, 0, 0};
    sub4(e, M->m, two);
    mpow(M, r, a, e);
}
static void mod_setup(mod_t *M, const u64 *m) {
    memcpy(M->m, m, 32);
    u64 x = 1;                                   /* Newton: x = m^-1 mod 2^64 */
    for (int i = 0; i < 6; i++) x *= 2 - m[0] * x;
    M->inv = (u64)0 - x;
    u64 r[4] = {0, 0, 0, 0};                     /* R mod m by doubling 1 256 times, then R^2 by 256 more */
    r[0] = 1;
    for (int i = 0; i < 512; i++) madd(M, r, r, r);
    memcpy(M->r2, r, 32);
    u64 one[4] = {1, 0, 0, 0};
    mto(M, M->one, one);
}
static void init(void) {
    if (g_init) return;
    mod_setup(&MP, P_);
    mod_setup(&MN, N_);
    g_init = 1;
}

/* ---------------------------------------------------------------- field helpers (Montgomery form mod p) */
#define FMUL(r, a, b) mmul(&MP, r, a, b)
#define FADD(r, a, b) madd(&MP, r, a, b)
#define FSUB(r, a, b) msub(&MP, r, a, b)
static void fsqrt(u64 *r, const u64 *a) {      /* a^((p+1)/4), p = 3 mod 4 */
    u64 e[4], one[4] = {1, 0, 0, 0};
    add4(e, P_, one);
    for (int i = 0; i < 4; i++) e[i] = (e[i] >> 2) | (i < 3 ? e[i + 1] << 62 : 0);
    mpow(&MP, r, a, e);
}
static void fseven(u64 *r) { u64 s[4] = {7, 0, 0, 0}; mto(&MP, r, s); }
static int fodd(const u64 *a) { u64 t[4]; mfrom(&MP, t, a); return (int)(t[0] & 1); }

/* ---------------------------------------------------------------- Jacobian points, y^2 = x^3 + 7 */
typedef struct { u64 x[4], y[4], z[4]; int inf; } jac_t;

static void jdbl(jac_t *r, const jac_t *p) {
    if (p->inf || is_zero4(p->y)) { r->inf = 1; return; }
    u64 a[4], b[4], c[4], d[4], e[4], f[4], t[4];
    FMUL(a, p->x, p->x);
    FMUL(b, p->y, p->y);
    FMUL(c, b, b);
    FADD(t, p->x, b); FMUL(d, t, t); FSUB(d, d, a); FSUB(d, d, c); FADD(d, d, d);   /* D = 2((X+B)^2 - A - C) */
    FADD(e, a, a); FADD(e, e, a);                                                     /* E = 3A */
    FMUL(f, e, e);                                                                    /* F = E^2 */
    u64 x3[4], y3[4], z3[4];
    FSUB(x3, f, d); FSUB(x3, x3, d);
    FSUB(t, d, x3); FMUL(y3, e, t);
    FADD(c, c, c); FADD(c, c, c); FADD(c, c, c); FSUB(y3, y3, c);
    FMUL(z3, p->y, p->z); FADD(z3, z3, z3);
    memcpy(r->x, x3, 32); memcpy(r->y, y3, 32); memcpy(r->z, z3, 32);
    r->inf = 0;
}
static void jadd(jac_t *r, const jac_t *p, const jac_t *q) {
    if (p->inf) { *r = *q; return; }
    if (q->inf) { *r = *p; return; }
    u64 z1z1[4], z2z2[4], u1[4], u2[4], s1[4], s2[4], t[4];
    FMUL(z1z1, p->z, p->z);
    FMUL(z2z2, q->z, q->z);
    FMUL(u1, p->x, z2z2);
    FMUL(u2, q->x, z1z1);
    FMUL(t, q->z, z2z2); FMUL(s1, p->y, t);
    FMUL(t, p->z, z1z1); FMUL(s2, q->y, t);
    u64 h[4], rr[4];
    FSUB(h, u2, u1);
    FSUB(rr, s2, s1);
    if (is_zero4(h)) {
        if (is_zero4(rr)) { jdbl(r, p); return; }
        r->inf = 1;
        return;
    }
    u64 hh[4], hhh[4], v[4], x3[4], y3[4], z3[4];
    FMUL(hh, h, h);
    FMUL(hhh, hh, h);
    FMUL(v, u1, hh);
    FMUL(x3, rr, rr); FSUB(x3, x3, hhh); FSUB(x3, x3, v); FSUB(x3, x3, v);
    FSUB(t, v, x3); FMUL(y3, rr, t); FMUL(t, s1, hhh); FSUB(y3, y3, t);
    FMUL(t, p->z, q->z); FMUL(z3, t, h);
    memcpy(r->x, x3, 32); memcpy(r->y, y3, 32); memcpy(r->z, z3, 32);
    r->inf = 0;
}
static void jneg(jac_t *r, const jac_t *p) {
    *r = *p;
    u64 zero[4] = {0, 0, 0, 0};
    FSUB(r->y, zero, p->y);
}
static void jaff(u64 *x, u64 *y, const jac_t *p) {    /* Montgomery-form affine coordinates; p not infinity */
    u64 zi[4], zi2[4], zi3[4];
    minv(&MP, zi, p->z);
    FMUL(zi2, zi, zi);
    FMUL(zi3, zi2, zi);
    FMUL(x, p->x, zi2);
    FMUL(y, p->y, zi3);
}
static void gen(jac_t *g) {
    mto(&MP, g->x, GX_);
    mto(&MP, g->y, GY_);
    memcpy(g->z, MP.one, 32);
    g->inf = 0;
}
/* r = a*P + b*Q (plain scalars, Straus-Shamir with 4-bit windows) */
static void jmul2(jac_t *r, const u64 *a, const jac_t *P, const u64 *b, const jac_t *Q) {
    jac_t tp[16], tq[16];
    tp[0].inf = 1; tq[0].inf = 1;
    tp[1] = *P; tq[1] = *Q;
    for (int i = 2; i < 16; i++) { jadd(&tp[i], &tp[i - 1], P); jadd(&tq[i], &tq[i - 1], Q); }
    jac_t acc;
    acc.inf = 1;
    for (int w = 63; w >= 0; w--) {
        for (int k = 0; k < 4; k++) jdbl(&acc, &acc);
        int da = (int)((a[w / 16] >> (4 * (w % 16))) & 15), db = (int)((b[w / 16] >> (4 * (w % 16))) & 15);
        if (da) jadd(&acc, &acc, &tp[da]);
        if (db) jadd(&acc, &acc, &tq[db]);
    }
    *r = acc;
}

/* ---------------------------------------------------------------- libsecp256k1 semantics */
/* secp256k1_ec_pubkey_parse: 33- or 65-byte encodings; out x, y Montgomery form */
static int pk_parse(u64 *x, u64 *y, const uint8_t *pk, size_t len) {
    u64 xi[4], yi[4], x3[4], t[4], sev[4];
    if (len == 33 && (pk[0] == 2 || pk[0] == 3)) {
        from_be32(xi, pk + 1);
        if (cmp4(xi, P_) >= 0) return 0;
        mto(&MP, x, xi);
        FMUL(t, x, x); FMUL(x3, t, x); fseven(sev); FADD(x3, x3, sev);
        fsqrt(y, x3);
        FMUL(t, y, y);
        if (cmp4(t, x3) != 0) return 0;
        if (fodd(y) != (pk[0] == 3)) { u64 zero[4] = {0}; FSUB(y, zero, y); }
        return 1;
    }
    if (len == 65 && (pk[0] == 4 || pk[0] == 6 || pk[0] == 7)) {
        from_be32(xi, pk + 1);
        from_be32(yi, pk + 33);
        if (cmp4(xi, P_) >= 0 || cmp4(yi, P_) >= 0) return 0;
        if ((pk[0] == 6 || pk[0] == 7) && (int)(yi[0] & 1) != (pk[0] == 7)) return 0;
        mto(&MP, x, xi); mto(&MP, y, yi);
        FMUL(t, x, x); FMUL(x3, t, x); fseven(sev); FADD(x3, x3, sev);
        FMUL(t, y, y);
        return cmp4(t, x3) == 0;
    }
    return 0;
}

/* DefaultCrypto.RestoreEncodedRecIdFromSignatureBuffer + the recId arithmetic of VerifySignatureHashed; returns 1
   when recId lands in [0, 3] (C and C# int division both truncate toward zero) */
int orc_ecdsa_recid_ok(const uint8_t *sig, size_t sig_len, int32_t chain_id) {
    int32_t enc;
    if (sig_len == 66) enc = (int32_t)sig[64] * 256 + sig[65];
    else if (sig_len == 65) enc = sig[64];
    else return 0;
    if (chain_id == 0) return 0;                 /* DivideByZeroException in the reference: not verified */
    int32_t rec = (enc - 36) / 2 / chain_id;
    return rec >= 0 && rec <= 3;
}

/* secp256k1_ecdsa_verify over the compact (r || s) form; hash = 32 bytes */
int orc_ecdsa_verify_compact(const uint8_t *hash32, const uint8_t *sig64, const uint8_t *pk, size_t pk_len) {
    init();
    u64 r[4], s[4], m[4], qx[4], qy[4];
    from_be32(r, sig64);
    from_be32(s, sig64 + 32);
    if (cmp4(r, N_) >= 0 || cmp4(s, N_) >= 0) return 0;           /* compact parse overflow */
    if (!pk_parse(qx, qy, pk, pk_len)) return 0;
    if (cmp4(s, NH_) > 0) return 0;                                 /* high s */
    if (is_zero4(r) || is_zero4(s)) return 0;
    from_be32(m, hash32);
    if (cmp4(m, N_) >= 0) sub4(m, m, N_);
    u64 sm[4], w[4], u1[4], u2[4], t[4];
    mto(&MN, sm, s);
    minv(&MN, w, sm);
    mto(&MN, t, m); mmul(&MN, t, t, w); mfrom(&MN, u1, t);
    mto(&MN, t, r); mmul(&MN, t, t, w); mfrom(&MN, u2, t);
    jac_t G, Q, R;
    gen(&G);
    memcpy(Q.x, qx, 32); memcpy(Q.y, qy, 32); memcpy(Q.z, MP.one, 32); Q.inf = 0;
    jmul2(&R, u1, &G, u2, &Q);
    if (R.inf) return 0;
    /* x(R) mod n == r  <=>  X == r Z^2  or (r + n < p and X == (r + n) Z^2) */
    u64 z2[4], xr[4], rx[4];
    FMUL(z2, R.z, R.z);
    mto(&MP, xr, r);
    FMUL(rx, xr, z2);
    if (cmp4(rx, R.x) == 0) return 1;
    u64 rn[4];
    if (add4(rn, r, N_)) return 0;
    if (cmp4(rn, P_) >= 0) return 0;
    mto(&MP, xr, rn);
    FMUL(rx, xr, z2);
    return cmp4(rx, R.x) == 0;
}

/* DefaultCrypto.VerifySignatureHashed (DefaultCrypto.cs:79-101) with TransactionUtils.ChainId(useNewChainId) given */
int orc_ecdsa_verify_hashed(const uint8_t *hash32, size_t hash_len, const uint8_t *sig, size_t sig_len,
                            const uint8_t *pk, size_t pk_len, int use_new_chain_id, int32_t chain_id) {
    if (hash_len != 32 || sig_len != (size_t)(use_new_chain_id ? 66 : 65)) return 0;
    init();
    u64 x[4], y[4];
    if (!pk_parse(x, y, pk, pk_len)) return 0;
    if (!orc_ecdsa_recid_ok(sig, sig_len, chain_id)) return 0;
    return orc_ecdsa_verify_compact(hash32, sig, pk, pk_len);
}

/* batch of the above over a key table (the C leg of the CPU baseline); out[i] in {0, 1} */
void orc_ecdsa_verify_batch_mt(uint8_t *out, const uint8_t *hashes, const uint8_t *sigs, size_t sig_len,
                               const uint8_t *pks, size_t pk_len, const int32_t *pk_idx, size_t n_pks, size_t n,
                               int use_new_chain_id, int32_t chain_id, int threads) {
    init();
    if (threads <= 0) threads = 1;
#pragma omp parallel for schedule(dynamic, 16) num_threads(threads)
    for (long i = 0; i < (long)n; i++) {
        int32_t k = pk_idx[i];
        out[i] = (k >= 0 && (size_t)k < n_pks)
                     ? (uint8_t)orc_ecdsa_verify_hashed(hashes + 32 * (size_t)i, 32, sigs + sig_len * (size_t)i, sig_len,
                                                         pks + pk_len * (size_t)k, pk_len, use_new_chain_id, chain_id)
                     : 0;
    }
}

void orc_ecdsa_verify_batch(uint8_t *out, const uint8_t *hashes, const uint8_t *sigs, size_t sig_len,
                            const uint8_t *pks, size_t pk_len, const int32_t *pk_idx, size_t n_pks, size_t n,
                            int use_new_chain_id, int32_t chain_id) {
    orc_ecdsa_verify_batch_mt(out, hashes, sigs, sig_len, pks, pk_len, pk_idx, n_pks, n, use_new_chain_id, chain_id, 8);
}

/* ---------------------------------------------------------------- test-vector helpers (signing side) */
/* compressed (33 B) and uncompressed (65 B) public key of a private key (big-endian, 0 < d < n) */
int orc_ecdsa_pubkey(uint8_t *out33, uint8_t *out65, const uint8_t *priv32) {
    init();
    u64 d[4], zero[4] = {0};
    from_be32(d, priv32);
    if (is_zero4(d) || cmp4(d, N_) >= 0) return -1;
    jac_t G, P;
    gen(&G);
    jmul2(&P, d, &G, zero, &G);
    u64 x[4], y[4], xi[4], yi[4];
    jaff(x, y, &P);
    mfrom(&MP, xi, x); mfrom(&MP, yi, y);
    if (out33) { out33[0] = (uint8_t)(2 + (yi[0] & 1)); to_be32(out33 + 1, xi); }
    if (out65) { out65[0] = 4; to_be32(out65 + 1, xi); to_be32(out65 + 33, yi); }
    return 0;
}
/* r || s (low-s normalised, as libsecp256k1 signs) and the recovery id, for nonce k; -1 if k or the result is bad */
int orc_ecdsa_sign_k(uint8_t *sig64, int *recid, const uint8_t *hash32, const uint8_t *priv32, const uint8_t *k32) {
    init();
    u64 d[4], k[4], m[4], zero[4] = {0};
    from_be32(d, priv32);
    from_be32(k, k32);
    from_be32(m, hash32);
    if (cmp4(m, N_) >= 0) sub4(m, m, N_);
    if (is_zero4(d) || cmp4(d, N_) >= 0 || is_zero4(k) || cmp4(k, N_) >= 0) return -1;
    jac_t G, R;
    gen(&G);
    jmul2(&R, k, &G, zero, &G);
    u64 x[4], y[4], xi[4], yi[4];
    jaff(x, y, &R);
    mfrom(&MP, xi, x); mfrom(&MP, yi, y);
    int rid = (int)(yi[0] & 1);
    u64 r[4];
    memcpy(r, xi, 32);
    if (cmp4(r, N_) >= 0) { sub4(r, r, N_); rid |= 2; }
    if (is_zero4(r)) return -1;
    u64 km[4], ki[4], rm[4], dm[4], mm[4], t[4], s[4];
    mto(&MN, km, k); minv(&MN, ki, km);
    mto(&MN, rm, r); mto(&MN, dm, d); mto(&MN, mm, m);
    mmul(&MN, t, rm, dm);
    madd(&MN, t, t, mm);
    mmul(&MN, t, t, ki);
    mfrom(&MN, s, t);
    if (is_zero4(s)) return -1;
    if (cmp4(s, NH_) > 0) { sub4(s, N_, s); rid ^= 1; }
    to_be32(sig64, r);
    to_be32(sig64 + 32, s);
    if (recid) *recid = rid;
    return 0;
}

/* secp256k1_ecdsa_recover (the reference's RecoverSignatureHashed, DefaultCrypto.cs:148-172): public key (33 B
   compressed) from hash, r || s and recovery id; -1 when there is none.  Used to pin the oracle against the
   reference's recover-to-address known answers and to build signatures whose x(R) lies in [n, p). */
int orc_ecdsa_recover(uint8_t *out33, const uint8_t *hash32, const uint8_t *sig64, int recid) {
    init();
    u64 r[4], s[4], m[4], fx[4];
    if (recid < 0 || recid > 3) return -1;
    from_be32(r, sig64);
    from_be32(s, sig64 + 32);
    if (cmp4(r, N_) >= 0 || cmp4(s, N_) >= 0 || is_zero4(r) || is_zero4(s)) return -1;
    from_be32(m, hash32);
    if (cmp4(m, N_) >= 0) sub4(m, m, N_);
    memcpy(fx, r, 32);
    if (recid & 2) {
        if (add4(fx, r, N_) || cmp4(fx, P_) >= 0) return -1;
    }
    uint8_t enc[33];
    enc[0] = (uint8_t)(2 + (recid & 1));
    to_be32(enc + 1, fx);
    jac_t R, G, Q;
    if (!pk_parse(R.x, R.y, enc, 33)) return -1;
    memcpy(R.z, MP.one, 32);
    R.inf = 0;
    gen(&G);
    u64 rm[4], ri[4], mm[4], sm[4], t[4], u1[4], u2[4], zero[4] = {0};
    mto(&MN, rm, r); minv(&MN, ri, rm);
    mto(&MN, mm, m); mmul(&MN, t, mm, ri); msub(&MN, t, zero, t); mfrom(&MN, u1, t);
    mto(&MN, sm, s); mmul(&MN, t, sm, ri); mfrom(&MN, u2, t);
    jmul2(&Q, u1, &G, u2, &R);
    if (Q.inf) return -1;
    u64 x[4], y[4], xi[4], yi[4];
    jaff(x, y, &Q);
    mfrom(&MP, xi, x); mfrom(&MP, yi, y);
    out33[0] = (uint8_t)(2 + (yi[0] & 1));
    to_be32(out33 + 1, xi);
    return 0;
}
