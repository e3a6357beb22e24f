// lachain_amd/csrc/h2g2.hpp — SHA-512 and mcl "ORIGINAL"-mode hash-and-map to G2 on the device.
//
// G2.SetHashOf(msg) (used by /root/reference/src/Lachain.Crypto/TPKE/Utils.cs:21-27 and
// ThresholdSignature/PublicKey.cs:18-19, PrivateKeyShare.cs:23-25) = mclBnG2_hashAndMapTo:
//   t.a = Fp::setHashOf(msg): SHA-512(msg), first 48 bytes little-endian, masked to 381 bits, and to
//         380 bits if still >= p;  t.b = 0
//   P   = MapTo::calcBN<G2, Fp2>(t)  (Fouque-Tibouchi / Shallue-van de Woestijne, mcl root choices)
//   H   = Budroni-Pintore cofactor clearing (z^2 - z - 1)P + psi((z - 1)P) + psi^2(2P)
// The algorithm is restated from mcl and is UNPINNED by any reference vector; the
// oracle (oracle/bls.c:g2_hash) implements the same steps independently.
#pragma once
#include "curve.hpp"

__constant__ u64 LCB_K512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

DI u64 rotr64(u64 x, int n) { return (x >> n) | (x << (64 - n)); }

// SHA-512 of the concatenation part1[0..n1) || part2[0..n2) (either may be empty); byte-wise reads
DN void sha512_2(uint8_t out[64], const uint8_t *p1, u32 n1, const uint8_t *p2, u32 n2) {
    u64 h[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
    u32 n = n1 + n2;
    u32 nblocks = (n + 17 + 127) / 128;
    for (u32 blk = 0; blk < nblocks; blk++) {
        // the message schedule in a ring of 16 words, every index a compile-time constant (registers, not the 640-byte
        // scratch array of the textbook 80-word schedule): rounds r + i, i = 0..15, with W_t (t >= 16) formed in place
        u64 w[16];
#pragma unroll
        for (int i = 0; i < 16; i++) {
            u64 v = 0;
            for (int k = 0; k < 8; k++) {
                u32 idx = blk * 128 + i * 8 + k;
                u32 byte;
                if (idx < n1) byte = p1[idx];
                else if (idx < n) byte = p2[idx - n1];
                else if (idx == n) byte = 0x80;
                else byte = 0;
                v = (v << 8) | byte;
            }
            if (blk == nblocks - 1 && i == 15) v = (u64)n * 8;
            w[i] = v;
        }
        u64 a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll 1
        for (int r = 0; r < 80; r += 16) {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                if (r) {
                    const u64 x15 = w[(i + 1) & 15], x2 = w[(i + 14) & 15];
                    const u64 s0 = rotr64(x15, 1) ^ rotr64(x15, 8) ^ (x15 >> 7);
                    const u64 s1 = rotr64(x2, 19) ^ rotr64(x2, 61) ^ (x2 >> 6);
                    w[i] = w[i] + s0 + w[(i + 9) & 15] + s1;
                }
                u64 S1 = rotr64(e, 14) ^ rotr64(e, 18) ^ rotr64(e, 41);
                u64 ch = (e & f) ^ (~e & g);
                u64 t1 = hh + S1 + ch + LCB_K512[r + i] + w[i];
                u64 S0 = rotr64(a, 28) ^ rotr64(a, 34) ^ rotr64(a, 39);
                u64 mj = (a & b) ^ (a & c) ^ (b & c);
                u64 t2 = S0 + mj;
                hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
            }
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
    }
    for (int k = 0; k < 8; k++)
        for (int j = 0; j < 8; j++) out[8 * k + j] = (uint8_t)(h[k] >> (56 - 8 * j));
}

// Fp::setHashOf on a 64-byte SHA-512 digest
DI void fp_set_hash_digest(fp &r, const uint8_t d[64]) {
    fp raw;
#pragma unroll
    for (int j = 0; j < 12; j++)
        raw.v[j] = (u32)d[4 * j] | ((u32)d[4 * j + 1] << 8) | ((u32)d[4 * j + 2] << 16) | ((u32)d[4 * j + 3] << 24);
    raw.v[11] &= (1u << (381 - 352)) - 1;
    if (!fp_raw_lt_p(raw)) raw.v[11] &= (1u << (380 - 352)) - 1;
    fp_from_raw(r, raw);
}

// MapTo::calcBN<G2, Fp2>
#ifndef LCB_SVDW_UNIFORM
#define LCB_SVDW_UNIFORM 1
#endif
DI bool g2_calc_bn(g2 &P, const fp2 &t) {
    // mcl's sign: the Legendre symbol of N(t).  For the hash's t = (t.a, 0), N(t) = t.a^2 is a square, so the symbol
    // is 1 unless t = 0 — no exponentiation needed
    int leg;
    if (fp_is_zero(t.b)) {
        leg = fp_is_zero(t.a) ? 0 : 1;
    } else {
        fp nrm;
        fp2_norm(nrm, t);
        leg = fp_legendre(nrm);
    }
    if (leg == 0) return false;
    bool negative = leg < 0;
    fp2 w, x, y, tmp, b2;
    fp c1, c2, one = fp_one();
    fp_load_const(c1, LCB_C1_SQRT_M3);
    fp_load_const(c2, LCB_C2_HALF);
    fp2_load_const(b2, LCB_B2);
    fp2_sqr(w, t);
    fp2_add(w, w, b2);
    fp_add(w.a, w.a, one);
    if (fp2_is_zero(w)) return false;
    fp2_inv_g(w, w);
    fp2_mul_fp(w, w, c1);
    fp2_mul(w, w, t);
#if LCB_SVDW_UNIFORM
    // Round 6: the first candidate whose g(x) = x^3 + b is a square, all three tested for every lane by the Legendre
    // symbol of the norm N(g(x)) (fp_jacobi, binary; g(x) is a square iff its norm is), then the chosen norm's root
    // and one fp2_sqrt of the chosen value from it (fp2_sqrt_normed: the same root as fp2_sqrt).  The loop with an
    // early exit ran up to three exponentiations per candidate for the wave whenever any lane needed them: 9 per wave,
    // then 5 with one exponentiation (the norm's root) per candidate, now 2; the selected x, and so H, is the same.
    fp2 xs, ts;
    fp ns;
    bool found = false;
#pragma unroll 1
    for (int i = 0; i < 3; i++) {
        if (i == 0) {
            fp2_mul(x, t, w);
            fp2_neg(x, x);
            fp_add(x.a, x.a, c2);
        } else if (i == 1) {
            fp2_neg(x, x);
            fp_sub(x.a, x.a, one);
        } else {
            fp2_sqr(x, w);
            fp2_inv_g(x, x);
            fp_add(x.a, x.a, one);
        }
        fp2_sqr(tmp, x);
        fp2_mul(tmp, tmp, x);
        fp2_add(tmp, tmp, b2);
        fp n, nr;
        {
            fp u;
            fp_sqr(n, tmp.a);
            fp_sqr(u, tmp.b);
            fp_add(n, n, u);                      // N(g(x)): a square iff g(x) is one
        }
#if LCB_JACOBI
        const bool sq = fp_jacobi(n) >= 0;        // the Legendre symbol only; the chosen norm's root below
        nr = n;
#else
        const bool sq = fp_sqrt(nr, n);
#endif
        if (!found && sq) {
            found = true;
            xs = x;
            ts = tmp;
            ns = nr;
        }
    }
    if (!found) return false;
#if LCB_JACOBI
    (void)fp_sqrt(ns, ns);                        // a square: fp_sqrt's root, as before
#endif
    fp2_sqrt_normed(y, ts, ns);
    if (negative) fp2_neg(y, y);
    P.x = xs; P.y = y; P.z = fp2_one();
    return true;
#else
    for (int i = 0; i < 3; i++) {
        if (i == 0) {
            fp2_mul(x, t, w);
            fp2_neg(x, x);
            fp_add(x.a, x.a, c2);
        } else if (i == 1) {
            fp2_neg(x, x);
            fp_sub(x.a, x.a, one);
        } else {
            fp2_sqr(x, w);
            fp2_inv_g(x, x);
            fp_add(x.a, x.a, one);
        }
        fp2_sqr(tmp, x);
        fp2_mul(tmp, tmp, x);
        fp2_add(tmp, tmp, b2);
        if (fp2_sqrt(y, tmp)) {
            if (negative) fp2_neg(y, y);
            P.x = x; P.y = y; P.z = fp2_one();
            return true;
        }
    }
    return false;
#endif
}
// Budroni-Pintore: (z^2 - z - 1) P + psi((z - 1) P) + psi^2(2P), z = -|z|
// the cofactor clearing's two 64-bit ladders with the group operations inlined (measured faster than the calls)
#define H2G2_MUL_U64(r, p, k) jac_mul_u64_inl(r, p, k)
// [k] P for P with Z = 1 (the map's output): mixed additions (7M + 4S over Fp2 instead of 11M + 5S); the same point
DI void g2_mul_u64_z1_inl(g2 &r, const g2 &p, u64 k) {
    int top = 63 - __clzll(k);
    g2 acc = p;
#pragma unroll 1
    for (int i = top - 1; i >= 0; i--) {
        jac_dbl(acc, acc);
        if ((k >> i) & 1) jac_add_aff(acc, acc, p.x, p.y);
    }
    r = acc;
}
DI void g2_clear_cofactor_bp(g2 &Q, const g2 &P) {
    g2 T0, T1, T2;
    g2_mul_u64_z1_inl(T0, P, LCB_Z_ABS + 1);   // |z - 1| P   (P.z = 1: g2_calc_bn)
    jac_neg(T0, T0);                     // (z - 1) P
    H2G2_MUL_U64(T1, T0, LCB_Z_ABS);
    jac_neg(T1, T1);                     // z (z - 1) P
    jac_neg(T2, P);
    g2_add_n(T1, T1, T2);                // (z^2 - z - 1) P
    g2_psi(T0, T0);
    g2_add_n(T0, T0, T1);
    g2_dbl_n(T1, P);
    g2_psi2(T1, T1);
    g2_add_n(Q, T0, T1);
}
DI void g2_clear_cofactor_h2(g2 &Q, const g2 &P) { jac_mul_bits(Q, P, LCB_H2_COFACTOR, LCB_H2_BITS); }

// hash a message already digested with SHA-512
DN bool g2_hash_digest(g2 &H, const uint8_t d[64], bool original_cofactor) {
    fp2 t;
    fp_set_hash_digest(t.a, d);
    t.b = fp_zero();
    g2 P;
    if (!g2_calc_bn(P, t)) return false;
    if (original_cofactor) g2_clear_cofactor_h2(H, P);
    else g2_clear_cofactor_bp(H, P);
    return true;
}
