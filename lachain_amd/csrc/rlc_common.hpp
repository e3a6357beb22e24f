// lachain_amd/csrc/rlc_common.hpp — device helpers shared by the randomized batch check's kernels (k_batch.hip,
// k_rlc_rand.hip): batch-exponent key and ChaCha20 scalars, suspect-key bitmap, quad-major SoA records, the joint
// (a + b lambda) ladders and the validators' fixed-base tables.
#pragma once
#include "kcommon.hpp"

struct rlc_key { u32 k[8]; u32 nonce[2]; };   // ChaCha20 key (256 bit, from getrandom) and a per-call nonce

#define LCB_RLC_SINGLES 8       // a failed group this short (below level 1) splits into single shares

// ---------------------------------------------------------------- suspect keys (Byzantine validators)
// A faulty validator corrupts its share in EVERY ciphertext / coin (HoneyBadgerMalicious.cs:17-23 reverses each
// share it sends; HoneyBadgerSmartMalicious.cs:28-48 sends valid off-subgroup points), so with F of them every group
// carries F bad shares and every group check fails.  The census (exact single checks of a prefix of the batch, before
// the groups are formed) marks a key suspect when at least half of its sampled shares that decoded failed their exact
// check; every share of a suspect key is then checked on its own and the groups are summed over the other keys only.
// The bitmap only changes the cost: every decision is still an exact single check or a group check.
DI bool key_suspect(const u32 *susp, u32 k, u32 n_keys) {
    return susp && k < n_keys && ((susp[k >> 5] >> (k & 31)) & 1u);
}
// the same read while the census may still be writing the bitmap (k_*_rlc_points runs beside it on the other
// stream): a stale 0 only costs a randomisation that is not used
DI bool key_suspect_live(const u32 *susp, u32 k, u32 n_keys) {
    if (!susp || k >= n_keys) return false;
    return (__atomic_load_n(susp + (k >> 5), __ATOMIC_RELAXED) >> (k & 31)) & 1u;
}

// ---------------------------------------------------------------- ChaCha20 (RFC 8439 block function)
DI u32 rotl32(u32 x, int r) { return (x << r) | (x >> (32 - r)); }
#define CHACHA_QR(a, b, c, d)                  \
    a += b; d ^= a; d = rotl32(d, 16);         \
    c += d; b ^= c; b = rotl32(b, 12);         \
    a += b; d ^= a; d = rotl32(d, 8);          \
    c += d; b ^= c; b = rotl32(b, 7);
// share exponent s_i = a_i + b_i lambda (lambda = z^2 - 1, phi(x, y) = (beta x, y)) from the 32-bit words a_i, b_i of
// ChaCha20 block i: a_i P + b_i phi(P) takes 32 shared doublings.  phi acts as lambda on the r-torsion and the reduced
// pairing kills every other component of an E(Fp) point, so e(a P + b phi(P), Q) = e(P, Q)^(a + b lambda) for ANY
// P on the curve; the 2^64 pairs (a, b) give 2^64 distinct exponents mod r (a + b lambda < 2^160 < r), none zero
// ((0, 0) -> (1, 0)): the soundness of a uniform 64-bit exponent.
DI void rlc_scalar(const rlc_key &key, u32 i, u32 &a, u32 &b) {
    u32 x[16], s[16];
    s[0] = 0x61707865u; s[1] = 0x3320646eu; s[2] = 0x79622d32u; s[3] = 0x6b206574u;
#pragma unroll
    for (int j = 0; j < 8; j++) s[4 + j] = key.k[j];
    s[12] = i; s[13] = 0; s[14] = key.nonce[0]; s[15] = key.nonce[1];
#pragma unroll
    for (int j = 0; j < 16; j++) x[j] = s[j];
#pragma unroll 1
    for (int r = 0; r < 10; r++) {
        CHACHA_QR(x[0], x[4], x[8], x[12]);
        CHACHA_QR(x[1], x[5], x[9], x[13]);
        CHACHA_QR(x[2], x[6], x[10], x[14]);
        CHACHA_QR(x[3], x[7], x[11], x[15]);
        CHACHA_QR(x[0], x[5], x[10], x[15]);
        CHACHA_QR(x[1], x[6], x[11], x[12]);
        CHACHA_QR(x[2], x[7], x[8], x[13]);
        CHACHA_QR(x[3], x[4], x[9], x[14]);
    }
    a = x[0] + s[0];
    b = x[1] + s[1];
    if ((a | b) == 0) a = 1;
}

// ---------------------------------------------------------------- quad-major SoA records (NW words, NW % 4 == 0)
template <int NW> DI void soa_store(u32 *base, size_t n, size_t i, const void *v) {
    const u32 *s = (const u32 *)v;
#pragma unroll
    for (int q = 0; q < NW / 4; q++)
        *(uint4 *)(base + ((size_t)q * n + i) * 4) = make_uint4(s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]);
}
template <int NW> DI void soa_load(void *v, const u32 *base, size_t n, size_t i) {
    u32 *d = (u32 *)v;
#pragma unroll
    for (int q = 0; q < NW / 4; q++) {
        uint4 x = *(const uint4 *)(base + ((size_t)q * n + i) * 4);
        d[4 * q] = x.x; d[4 * q + 1] = x.y; d[4 * q + 2] = x.z; d[4 * q + 3] = x.w;
    }
}
DI void g1_store_soa(u32 *base, size_t n, size_t i, const g1 &p) { soa_store<36>(base, n, i, &p); }
DI void g1_load_soa(g1 &p, const u32 *base, size_t n, size_t i) { soa_load<36>(&p, base, n, i); }
DI void g2_store_soa(u32 *base, size_t n, size_t i, const g2 &p) { soa_store<72>(base, n, i, &p); }
DI void g2_load_soa(g2 &p, const u32 *base, size_t n, size_t i) { soa_load<72>(&p, base, n, i); }

// a P + b phi(P) for an affine P, phi(x, y) = (beta x, y).  Joint bits: the addend is P (1, 0), phi(P) (0, 1) or
// P + phi(P) = (beta^2 x, -y) (1, 1; the chord through two points of equal y has slope 0 and 1 + beta + beta^2 = 0),
// so each bit costs one mixed addition, and a wave (whose lanes' bits differ) executes 32 of them instead of 64.
DI void g1_ab_addends(fp &bx, fp &b2x, fp &ny, const g1a &P) {
    fp beta;
    fp_load_const(beta, LCB_G1_BETA);
    fp_mul(bx, P.x, beta);
    fp_mul(b2x, bx, beta);
    fp_neg(ny, P.y);
}
DN void g1_mul_ab_n(g1 &r, const g1a &P, u32 a, u32 b) {
    g1 acc;
    jac_set_inf(acc);
    if (!P.inf) {
        fp bx, b2x, ny;
        g1_ab_addends(bx, b2x, ny, P);
        for (int k = 31; k >= 0; k--) {
            grp_dbl(acc, acc);
            u32 da = (a >> k) & 1, db = (b >> k) & 1;
            if (da | db) grp_madd(acc, acc, da ? (db ? b2x : P.x) : bx, (da & db) ? ny : P.y);
        }
    }
    r = acc;
}
// (a + b lambda) S for S in G2: psi^2(x, y) = (beta x, -y) acts on G2 as z^2 (mod r) and psi^4(x, y) = (beta^2 x, y)
// as z^4 = z^2 - 1 = lambda, so (a + b lambda) S = a S + b psi^4(S); the joint addend S + psi^4(S) = psi^2(S) (equal
// y again): one mixed addition per bit as in G1
DI void g2_ab_addends(fp2 &x4, fp2 &x2, fp2 &ny, const g2a &S) {
    fp beta, b2;
    fp_load_const(beta, LCB_G1_BETA);
    fp_sqr(b2, beta);
    fp2_mul_fp(x4, S.x, b2);
    fp2_mul_fp(x2, S.x, beta);
    fp2_neg(ny, S.y);
}
// the same with the point arithmetic inlined (no call frames: the DN form passes the accumulator through scratch at
// every doubling / addition).  Round 6 (LCB_AB_LEAN, default): only x, y and beta x stay live across the ladder — the
// joint addend's beta^2 x = -(x + beta x) (1 + beta + beta^2 = 0) and -y are formed per column from them, 24 fewer
// registers live across every product (k_tpke_rlc_points runs at 248 registers, two waves per SIMD)
#ifndef LCB_AB_LEAN
#define LCB_AB_LEAN 1
#endif
DI void g1_mul_ab_inl(g1 &r, const g1a &P, u32 a, u32 b) {
    jac_set_inf(r);
    if (P.inf) return;
#if LCB_AB_LEAN
    fp bx, beta;
    fp_load_const(beta, LCB_G1_BETA);
    fp_mul(bx, P.x, beta);
#pragma unroll 1
    for (int k = 31; k >= 0; k--) {
        jac_dbl(r, r);
        u32 da = (a >> k) & 1, db = (b >> k) & 1;
        if (da | db) {
            fp ax, ay;
            if (da & db) {                       // P + phi(P) = (beta^2 x, -y)
                fp_add(ax, P.x, bx);
                fp_neg(ax, ax);
                fp_neg(ay, P.y);
            } else {
                ax = da ? P.x : bx;
                ay = P.y;
            }
            jac_add_aff(r, r, ax, ay);
        }
    }
#else
    fp bx, b2x, ny;
    g1_ab_addends(bx, b2x, ny, P);
#pragma unroll 1
    for (int k = 31; k >= 0; k--) {
        jac_dbl(r, r);
        u32 da = (a >> k) & 1, db = (b >> k) & 1;
        if (da | db) jac_add_aff(r, r, da ? (db ? b2x : P.x) : bx, (da & db) ? ny : P.y);
    }
#endif
}
// G2 form of g1_mul_ab_inl: a S + b psi^4(S) with the point arithmetic inlined; lean form: x, y and beta x live, the
// psi^4 addend's beta^2 x = -(x + beta x) and the joint addend psi^2(S) = (beta x, -y) formed per column
DI void g2_mul_ab_inl(g2 &r, const g2a &S, u32 a, u32 b) {
    jac_set_inf(r);
    if (S.inf) return;
#if LCB_AB_LEAN
    fp2 x2;
    {
        fp beta;
        fp_load_const(beta, LCB_G1_BETA);
        fp2_mul_fp(x2, S.x, beta);
    }
#pragma unroll 1
    for (int k = 31; k >= 0; k--) {
        jac_dbl(r, r);
        u32 da = (a >> k) & 1, db = (b >> k) & 1;
        if (da | db) {
            fp2 ax, ay;
            if (da & db) {                       // S + psi^4(S) = psi^2(S) = (beta x, -y)
                ax = x2;
                fp2_neg(ay, S.y);
            } else if (da) {
                ax = S.x;
                ay = S.y;
            } else {                             // psi^4(S) = (beta^2 x, y)
                fp2_add(ax, S.x, x2);
                fp2_neg(ax, ax);
                ay = S.y;
            }
            jac_add_aff(r, r, ax, ay);
        }
    }
#else
    fp2 x4, x2, ny;
    g2_ab_addends(x4, x2, ny, S);
#pragma unroll 1
    for (int k = 31; k >= 0; k--) {
        jac_dbl(r, r);
        u32 da = (a >> k) & 1, db = (b >> k) & 1;
        if (da | db) jac_add_aff(r, r, da ? (db ? x2 : S.x) : x4, (da & db) ? ny : S.y);
    }
#endif
}
// The same G2 ladder with its addends read from a record slot instead of held in registers (round 6, LCB_G2AB_MEM): x,
// y and beta x of S are stored in the output record's x, y, z words (g2_store_soa layout, wave-coalesced), read back at
// every column (L1 / L2), and the record is overwritten with the result after the last column — 72 registers fewer live
// across the ladder of the 256-register CommonCoin randomisation lanes
#ifndef LCB_G2AB_MEM
#define LCB_G2AB_MEM 1
#endif
DI void g2_mul_ab_rec(g2 &r, const g2a &S, u32 a, u32 b, u32 *rec, size_t n, size_t i) {
    jac_set_inf(r);
    if (S.inf) return;
    {
        g2 st;
        st.x = S.x;
        st.y = S.y;
        fp beta;
        fp_load_const(beta, LCB_G1_BETA);
        fp2_mul_fp(st.z, S.x, beta);                     // beta x in the z words
        g2_store_soa(rec, n, i, st);
    }
#pragma unroll 1
    for (int k = 31; k >= 0; k--) {
        jac_dbl(r, r);
        u32 da = (a >> k) & 1, db = (b >> k) & 1;
        if (da | db) {
            fp2 ax, ay, x2;
            asm volatile("" ::: "memory");
            soa_load<24>(&ax, rec, n, i);
            soa_load<24>(&ay, rec + (size_t)24 * n, n, i);
            soa_load<24>(&x2, rec + (size_t)48 * n, n, i);
            if (da & db) {                               // S + psi^4(S) = psi^2(S) = (beta x, -y)
                ax = x2;
                fp2_neg(ay, ay);
            } else if (!da) {                            // psi^4(S) = (beta^2 x, y)
                fp2_add(ax, ax, x2);
                fp2_neg(ax, ax);
            }
            jac_add_aff(r, r, ax, ay);
        }
    }
}
// affine records of Jacobian points (inf = 1 for the point at infinity), optionally negated
DI void g1_to_st(g1a_st &o, const g1 &p, bool neg) {
    g1a a;
    jac_to_aff(a, p);
    o.ok = 1; o.pad[0] = o.pad[1] = 0;
    o.inf = a.inf;
    o.x = a.x;
    if (neg && !a.inf) fp_neg(o.y, a.y);
    else o.y = a.y;
}
// the same record with the binary-GCD inversion (field.hpp fp_inv_gcd): the group sums' chains are a few additions,
// so the inversion is most of their work
DI void g1_to_st_gcd(g1a_st &o, const g1 &p, bool neg) {
    o.ok = 1; o.pad[0] = o.pad[1] = 0;
    if (jac_is_inf(p)) { o.inf = 1; o.x = fp_zero(); o.y = fp_zero(); return; }
    fp zi, zi2, y;
    fp_inv_gcd(zi, p.z);
    fp_sqr(zi2, zi);
    fp_mul(o.x, p.x, zi2);
    fp_mul(zi2, zi2, zi);
    fp_mul(y, p.y, zi2);
    o.inf = 0;
    if (neg) fp_neg(o.y, y);
    else o.y = y;
}
DI void g2_to_st(g2a_st &o, const g2 &p) {
    g2a a;
    jac_to_aff(a, p);
    o.ok = 1; o.pad[0] = o.pad[1] = 0;
    o.inf = a.inf;
    o.x = a.x;
    o.y = a.y;
}
DI void g2_to_st_gcd(g2a_st &o, const g2 &p) {      // (curve.hpp g2_jac_to_aff_g: the binary-GCD inversion)
    g2a a;
    g2_jac_to_aff_g(a, p);
    o.ok = 1; o.pad[0] = o.pad[1] = 0;
    o.inf = a.inf;
    o.x = a.x;
    o.y = a.y;
}
DI void g1_inf_st(g1a_st &o) { o.ok = 1; o.pad[0] = o.pad[1] = 0; o.inf = 1; o.x = fp_zero(); o.y = fp_zero(); }
DI void g2_inf_st(g2a_st &o) { o.ok = 1; o.pad[0] = o.pad[1] = 0; o.inf = 1; o.x = fp2_zero(); o.y = fp2_zero(); }

// ---------------------------------------------------------------- fixed-base tables of the validators' keys
// The keys (TPKE verification keys Y_d, threshold-signature public keys PK_k) are the same for every ciphertext /
// coin of a batch: per key, table[w][d - 1] = d 2^(8w) K (affine x, y and beta x, d = 1..255, w = 0..3) turns
// a K + b phi(K) for 32-bit a, b into at most 8 mixed additions (4 byte digits of a, 4 of b on the phi entries) instead
// of 32 doublings + ~32 mixed additions.  LCB_KTAB_CHUNKS lanes per (key, window), each 8w doublings, a start multiple and
// LCB_KTAB_CHUNK - 1 additions into a Jacobian scratch, then one batched inversion (Montgomery's trick) to affine.  A key whose chain meets the point at
// infinity (a key with no r-torsion part) or that did not decompress gets ktab_ok = 0: its shares use the ladder.
#define LCB_KTAB_ENTRIES (4 * 255)
#define LCB_KTAB_CHUNK 16                              // entries per lane: 16 lanes per (key, window)
#define LCB_KTAB_CHUNKS 16                             // (255 + LCB_KTAB_CHUNK - 1) / LCB_KTAB_CHUNK
#define LCB_KTAB_LANES 64                              // lanes (and flags) per key: 4 windows x LCB_KTAB_CHUNKS
DN void g1_mul_ab_tab(g1 &r, const u32 *tab, u32 n_keys, u32 k, u32 a, u32 b) {
    const size_t stride = (size_t)n_keys * LCB_KTAB_ENTRIES, e0 = (size_t)k * LCB_KTAB_ENTRIES;
    g1 acc;
    jac_set_inf(acc);
    fp xyb[3];
    // one digit at a time (the loads are not hoisted: eight live table points would cost 192 registers); the b digits
    // add phi(entry) = (beta x, y), stored beside the entry
#pragma unroll 1
    for (u32 j = 0; j < 8; j++) {
        u32 w = j & 3, dg = ((j < 4 ? b : a) >> (8 * w)) & 255;
        if (!dg) continue;
        asm volatile("" ::: "memory");
        soa_load<36>(xyb, tab, stride, e0 + w * 255 + dg - 1);
        grp_madd(acc, acc, j < 4 ? xyb[2] : xyb[0], xyb[1]);
    }
    r = acc;
}
DI bool ktab_usable(const uint8_t *ktab_ok, u32 k) {      // all LCB_KTAB_LANES lanes of the key's table succeeded
    if (!ktab_ok) return false;
    const uint4 *f = (const uint4 *)(ktab_ok + (size_t)LCB_KTAB_LANES * k);
    u32 a = 0x01010101u;
#pragma unroll
    for (int q = 0; q < LCB_KTAB_LANES / 16; q++) {
        const uint4 x = f[q];
        a &= x.x & x.y & x.z & x.w;
    }
    return a == 0x01010101u;
}
static_assert(LCB_KTAB_CHUNK * LCB_KTAB_CHUNKS >= 255 && LCB_KTAB_CHUNK * (LCB_KTAB_CHUNKS - 1) < 255, "key-table chunks");
static_assert(LCB_KTAB_LANES == 4 * LCB_KTAB_CHUNKS && LCB_KTAB_LANES % 16 == 0, "key-table lanes");

// ---------------------------------------------------------------- level helpers shared by k_batch.hip and k_tpke.hip
// The shares of group d that still need a check of their own, as singles of kind w (0: a group of one randomized
// share, 1: an exact single): not those already rejected, nor those of suspect keys (they have exact singles since
// level 1).
DI void emit_singles(const uint4 &d, u32 w, const uint8_t *accept, const u32 *key_idx, u32 n_keys, const u32 *susp,
                     uint4 *next, u32 *next_count) {
    u32 cnt = 0;
    for (u32 k = 0; k < d.y; k++)
        cnt += accept[d.x + k] && !key_suspect(susp, key_idx[d.x + k], n_keys);
    if (!cnt) return;
    u32 slot = atomicAdd(next_count, cnt);
    for (u32 k = 0; k < d.y; k++)
        if (accept[d.x + k] && !key_suspect(susp, key_idx[d.x + k], n_keys))
            next[slot++] = make_uint4(d.x + k, 1, d.z, w);
}
DI void fp12_load_row(fp12 &f, const u32 *row) {
    u32 *w = (u32 *)&f;
    const uint4 *src = (const uint4 *)row;
#pragma unroll
    for (int q = 0; q < 36; q++) {
        uint4 v = src[q];
        w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
}
DI bool fp12_words_eq(const fp12 &a, const fp12 &b) {
    const u32 *x = (const u32 *)&a, *y = (const u32 *)&b;
    u32 d = 0;
#pragma unroll
    for (int q = 0; q < 144; q++) d |= x[q] ^ y[q];
    return d == 0;
}
DI u32 fp12_fingerprint(const fp12 &a) {
    const u32 *w = (const u32 *)&a;
    u32 h = 0;
#pragma unroll
    for (int q = 0; q < 144; q++) h = ((h << 5) | (h >> 27)) ^ w[q];
    return h;
}
DI u32 half_ballot(bool p) {
    const unsigned long long m = __ballot(p);
    return (u32)(m >> (32 * ((threadIdx.x >> 5) & 1)));
}
