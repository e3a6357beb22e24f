// lachain_amd/csrc/k_batch.hip — gfx950 kernels: randomized batch verification of TPKE decryption shares
// (small-exponent test, Bellare–Garay–Rabin 1998) over the per-share check of TPKE/PublicKey.cs:88-92.
//
// The reference decides every share on its own: e(U_i, H) == e(Y_i, W) (two pairings per share).  Every value
// e(., .) is a reduced pairing, so the ratio g_i = e(U_i, H) / e(Y_i, W) lies in mu_r (order r, prime) whatever
// U_i is: for a G2 point Q the (ate) pairing is linear in its G1 argument on all of E(Fp) (Weil reciprocity; the
// error term is an r-th power, killed by the final exponentiation) and kills the cofactor-torsion part, so off-
// subgroup U_i / Y_i are covered.  H is in G2 by construction; W is checked (k_tpke_ct_g2check) and a ciphertext with
// W outside G2 gets exact per-share checks.  For secret random exponents s_i (2^64 values, none 0 mod r; rlc_scalar):
// prod_i g_i^(s_i) == 1  <=>  e(sum s_i U_i, H) e(-sum s_i Y_i, W) == 1, and if some g_i != 1 the product is 1 with
// probability <= 2^-64.  So one Miller pair + final exponentiation decides a whole group of shares of one ciphertext;
// a group that fails is split and re-checked, down to single shares, where g_i^(s_i) == 1 <=> g_i == 1 (gcd(s_i, r)
// = 1): every rejected share is rejected by an exact check of its own, every accepted share by a group check (false
// accept <= 2^-64 per group, over the secret exponents).
//
// Pipeline (host side in lcb_host.cpp: rlc_points_enqueue + rlc_levels):
//   k_tpke_rlc_points   one lane per share: validity as k_tpke_miller, (a_i, b_i) = ChaCha20(key, i), s_i U_i and
//                       s_i Y_i with s_i = a_i + b_i lambda (32-bit GLV form, rlc_scalar) -> quad-major SoA Jacobian
//                       records (invalid share: infinity)
//   k_rlc_groups        one lane per 256 consecutive shares: runs of equal ciphertext index (<= 32) -> level-1 groups
//   k_tpke_ct_g2check   one lane per ciphertext: W in G2 (else its shares get exact per-share checks)
//   k_tpke_rlc_sum      one lane per group: ciphertext validity, the two sums, to affine with one shared inversion,
//                       -sum s_i Y_i (or an exact single share's own U_i, -Y_i)
//   k_tpke_rlc_miller   one lane per group: the two-pair Miller loop over the ciphertext's line sets
//   k_final_exp_check   (k_tpke.hip) group decision
//   k_rlc_resolve       one lane per group: failed single share -> reject; failed group -> sub-groups of the next level
#include "kcommon.hpp"

LCB_ASM_LIBRARY(k_batch)

struct rlc_key { u32 k[8]; u32 nonce[2]; };   // ChaCha20 key (256 bit, from getrandom) and a per-call nonce

#define LCB_RLC_RUN 32          // longest level-1 group
#define LCB_RLC_SPAN 256        // shares scanned by one k_rlc_groups lane
#define LCB_RLC_SINGLES 8       // a failed group this short splits into single shares

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

// ---------------------------------------------------------------- quad-major SoA Jacobian G1 records (36 words)
DI void g1_store_soa(u32 *base, size_t n, size_t i, const g1 &p) {
    const u32 *s = (const u32 *)&p;
#pragma unroll
    for (int q = 0; q < 9; q++)
        *(uint4 *)(base + ((size_t)q * n + i) * 4) = make_uint4(s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]);
}
DI void g1_load_soa(g1 &p, const u32 *base, size_t n, size_t i) {
    u32 *d = (u32 *)&p;
#pragma unroll
    for (int q = 0; q < 9; q++) {
        uint4 v = *(const uint4 *)(base + ((size_t)q * n + i) * 4);
        d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
    }
}
// a P + b phi(P) for an affine P: 32 doublings, mixed additions of P and phi(P)
DN void g1_mul_ab_n(g1 &r, const g1a &P, u32 a, u32 b) {
    g1 acc;
    jac_set_inf(acc);
    if (!P.inf) {
        fp beta, phx;
        fp_load_const(beta, LCB_G1_BETA);
        fp_mul(phx, P.x, beta);
        for (int k = 31; k >= 0; k--) {
            grp_dbl(acc, acc);
            if ((a >> k) & 1) grp_madd(acc, acc, P.x, P.y);
            if ((b >> k) & 1) grp_madd(acc, acc, phx, P.y);
        }
    }
    r = acc;
}

// both multiplications in one loop with the point arithmetic inlined (two independent dependency chains per lane, no
// call frames): a U + b phi(U) and a Y + b phi(Y).  Opt-in (LCB_RLC_JOINT): measured slower than the two calls to
// g1_mul_ab_n (randomisation 77.7 vs 63.5 ms per 1M shares): 290 VGPRs allow one wave per SIMD instead of two.
DI void g1_mul_ab2(g1 &ru, g1 &ry, const g1a &U, const g1a &Y, u32 a, u32 b) {
    fp beta, pux, pyx;
    fp_load_const(beta, LCB_G1_BETA);
    fp_mul(pux, U.x, beta);
    fp_mul(pyx, Y.x, beta);
    jac_set_inf(ru);
    jac_set_inf(ry);
#pragma unroll 1
    for (int k = 31; k >= 0; k--) {
        jac_dbl(ru, ru);
        jac_dbl(ry, ry);
        if ((a >> k) & 1) {
            jac_add_aff(ru, ru, U.x, U.y);
            jac_add_aff(ry, ry, Y.x, Y.y);
        }
        if ((b >> k) & 1) {
            jac_add_aff(ru, ru, pux, U.y);
            jac_add_aff(ry, ry, pyx, Y.y);
        }
    }
    if (U.inf) jac_set_inf(ru);
    if (Y.inf) jac_set_inf(ry);
}

// ---------------------------------------------------------------- per-share randomisation
// validity as k_tpke_miller except the ciphertext's (applied per group by k_tpke_rlc_sum, so this kernel needs only
// the decompressed keys and may run beside the ciphertext preparation)
extern "C" __global__ void LCB_BOUNDS k_tpke_rlc_points(u32 n_cts, const g1a_st *keys, u32 n_keys, const u32 *ct_idx,
                                                       const u32 *dec_idx, const uint8_t *ui, u32 n, rlc_key key,
                                                       u32 *rU, u32 *rY, uint8_t *accept) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u32 c = ct_idx[i], d = dec_idx[i];
    bool ok = d < n_keys && c < n_cts;
    g1a Ui, Y;
    ok = g1_decompress(Ui, ui + 48 * (size_t)i) && ok;
    g1a_st ks = keys[d < n_keys ? d : 0];
    ok = ok && ks.ok;
    st_to_g1a(Y, ks);
    g1 p, q;
    if (ok) {
        u32 a, b;
        rlc_scalar(key, i, a, b);
#ifdef LCB_RLC_JOINT
        g1_mul_ab2(p, q, Ui, Y, a, b);
#else
        g1_mul_ab_n(p, Ui, a, b);
        g1_mul_ab_n(q, Y, a, b);
#endif
    } else {                             // an invalid share is rejected and contributes nothing to its group
        jac_set_inf(p);
        jac_set_inf(q);
    }
    g1_store_soa(rU, n, i, p);
    g1_store_soa(rY, n, i, q);
    accept[i] = ok;
}

// ---------------------------------------------------------------- level-1 groups: runs of one ciphertext
// desc = {first share, length, ciphertext, 0}; order of the records is irrelevant
extern "C" __global__ void LCB_BOUNDS k_rlc_groups(const u32 *ct_idx, u32 n, u32 n_cts, uint4 *desc, u32 *count) {
    u32 b = blockIdx.x * blockDim.x + threadIdx.x;
    size_t lo = (size_t)b * LCB_RLC_SPAN;
    if (lo >= n) return;
    u32 hi = (u32)min((size_t)n, lo + LCB_RLC_SPAN);
    u32 start = (u32)lo, cur = ct_idx[lo];
    cur = cur < n_cts ? cur : 0;
    for (u32 j = (u32)lo + 1; j <= hi; j++) {
        u32 c = 0;
        if (j < hi) { c = ct_idx[j]; c = c < n_cts ? c : 0; }
        if (j == hi || c != cur || j - start == LCB_RLC_RUN) {
            u32 slot = atomicAdd(count, 1u);
            desc[slot] = make_uint4(start, j - start, cur, 0);
            start = j;
            cur = c;
        }
    }
}

// ---------------------------------------------------------------- group sums -> two affine points per group
// gpts[2g] = sum s_i U_i, gpts[2g + 1] = -sum s_i Y_i (g1a_st records; inf = 1 for the point at infinity).
// desc.w = 0: a randomized group.  A group of an invalid ciphertext rejects its shares; a group whose ciphertext's W
// is outside G2 (the pairing is linear in its G1 argument only for a G2 point: W comes from the wire unchecked) is
// handed to exact checks (gexact = 1: resolve re-emits its shares as desc.w = 1 singles).  Both check two points at
// infinity (they pass).  desc.w = 1: the exact single check of share desc.x, e(U_i, H) e(-Y_i, W) == 1 as
// k_tpke_miller does it (a share already rejected checks infinity).
extern "C" __global__ void LCB_BOUNDS k_tpke_rlc_sum(const uint4 *desc, u32 n_groups, const uint8_t *ct_ok,
                                                    const uint8_t *ct_g2, const g1a_st *keys, u32 n_keys,
                                                    const u32 *dec_idx, const uint8_t *ui, const u32 *rU,
                                                    const u32 *rY, u32 n, g1a_st *gpts, uint8_t *accept,
                                                    uint8_t *gexact) {
    u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_groups) return;
    uint4 dsc = desc[g];
    g1a_st o;
    o.ok = 1; o.pad[0] = o.pad[1] = 0;
    o.inf = 1; o.x = fp_zero(); o.y = fp_zero();
    gexact[g] = 0;
    if (dsc.w == 1) {                    // exact single
        g1a U, Y;
        bool live = accept[dsc.x] != 0;
        if (live) {
            u32 d = dec_idx[dsc.x];
            live = g1_decompress(U, ui + 48 * (size_t)dsc.x) && d < n_keys;
            st_to_g1a(Y, keys[d < n_keys ? d : 0]);
        }
        if (live && !U.inf) { o.x = U.x; o.y = U.y; o.inf = 0; }
        gpts[2 * (size_t)g] = o;
        o.inf = 1; o.x = fp_zero(); o.y = fp_zero();
        if (live && !Y.inf) { o.x = Y.x; fp_neg(o.y, Y.y); o.inf = 0; }
        gpts[2 * (size_t)g + 1] = o;
        return;
    }
    const bool cok = ct_ok[dsc.z];
    if (!cok || !ct_g2[dsc.z]) {
        if (!cok)
            for (u32 j = 0; j < dsc.y; j++) accept[dsc.x + j] = 0;
        else
            gexact[g] = 1;
        gpts[2 * (size_t)g] = o;
        gpts[2 * (size_t)g + 1] = o;
        return;
    }
    g1 su, sy, t;
    jac_set_inf(su);
    jac_set_inf(sy);
    for (u32 j = 0; j < dsc.y; j++) {
        g1_load_soa(t, rU, n, dsc.x + j);
        grp_add(su, su, t);
        g1_load_soa(t, rY, n, dsc.x + j);
        grp_add(sy, sy, t);
    }
    // one inversion for both: 1 / (z_u z_y), an infinite sum's z replaced by 1
    bool iu = jac_is_inf(su), iy = jac_is_inf(sy);
    fp zu = iu ? fp_one() : su.z, zy = iy ? fp_one() : sy.z, zz, inv, zi, zi2;
    fp_mul(zz, zu, zy);
    fp_inv(inv, zz);
    fp_mul(zi, inv, zy);                 // 1 / z_u
    fp_sqr(zi2, zi);
    fp_mul(o.x, su.x, zi2);
    fp_mul(zi2, zi2, zi);
    fp_mul(o.y, su.y, zi2);
    o.inf = iu;
    if (iu) { o.x = fp_zero(); o.y = fp_zero(); }
    gpts[2 * (size_t)g] = o;
    fp_mul(zi, inv, zu);                 // 1 / z_y
    fp_sqr(zi2, zi);
    fp_mul(o.x, sy.x, zi2);
    fp_mul(zi2, zi2, zi);
    fp_mul(o.y, sy.y, zi2);
    fp_neg(o.y, o.y);
    o.inf = iy;
    if (iy) { o.x = fp_zero(); o.y = fp_zero(); }
    gpts[2 * (size_t)g + 1] = o;
}

// W of every ciphertext in G2 (Scott's psi test, curve.hpp g2_in_subgroup); H = hash-to-G2 output is in G2 by
// construction
extern "C" __global__ void LCB_BOUNDS k_tpke_ct_g2check(const u32 *lines, const uint8_t *ct_ok, u32 n_cts,
                                                       uint8_t *ct_g2) {
    u32 c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_cts) return;
    g2a W;
    lineset_point(W, lines + (size_t)(2 * c + 1) * LCB_LINESET_WORDS);
    ct_g2[c] = ct_ok[c] ? g2_in_subgroup(W) : 0;
}

// ---------------------------------------------------------------- group Miller loops (k_tpke_miller's loop)
extern "C" __global__ void LCB_PAIR_BOUNDS k_tpke_rlc_miller(const u32 *lines, const uint4 *desc, const g1a_st *gpts,
                                                            u32 n_groups, u32 *f_soa, uint8_t *gacc) {
    __shared__ uint4 lds_pts[12 * LCB_BLOCK];
    u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_groups) return;
    u32 c = desc[g].z;
    g1a P, Q;
    st_to_g1a(P, gpts[2 * (size_t)g]);
    st_to_g1a(Q, gpts[2 * (size_t)g + 1]);
    fp12 f;
    const u32 *lsH = lines + (size_t)(2 * c) * LCB_LINESET_WORDS, *lsW = lines + (size_t)(2 * c + 1) * LCB_LINESET_WORDS;
    if (lineset_normalised(lsH) && lineset_normalised(lsW)) {
        uint4 *pt = lds_pts + threadIdx.x;
        g1_park_lds(pt, P);
        g1_park_lds(pt + 6 * LCB_BLOCK_PTS, Q);
        miller2_norm_lds(f, lsH, pt, P.inf, lsW, pt + 6 * LCB_BLOCK_PTS, Q.inf);
    } else {
        miller2_sets_fallback(f, lsH, P, lsW, Q);
    }
    fp12_store_soa(f_soa, n_groups, g, f);
    gacc[g] = 1;
}

// ---------------------------------------------------------------- resolve a level
// a failed group of one share rejects it; a failed group of len > 1 becomes ceil(len / s) sub-groups of s =
// ceil(len / ceil(sqrt(len))) shares (one bad share among len then costs about 2 sqrt(len) group checks), or single
// shares when len <= LCB_RLC_SINGLES: every level is one latency-bound launch (~one serial pairing check per lane), so
// fewer levels beat fewer checks there
extern "C" __global__ void LCB_BOUNDS k_rlc_resolve(const uint4 *desc, u32 n_groups, const uint8_t *gacc,
                                                   const uint8_t *gexact, uint8_t *accept, uint4 *next,
                                                   u32 *next_count) {
    u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_groups) return;
    uint4 d = desc[g];
    if (gexact[g]) {                     // W outside G2: every share of the group gets its exact check
        u32 slot = atomicAdd(next_count, d.y);
        for (u32 k = 0; k < d.y; k++) next[slot + k] = make_uint4(d.x + k, 1, d.z, 1);
        return;
    }
    if (gacc[g]) return;
    if (d.y == 1) { accept[d.x] = 0; return; }
    u32 parts = 1;
    while (parts * parts < d.y) parts++;
    u32 s = d.y <= LCB_RLC_SINGLES ? 1u : (d.y + parts - 1) / parts;
    u32 m = (d.y + s - 1) / s;
    u32 slot = atomicAdd(next_count, m);
    for (u32 k = 0; k < m; k++) {
        u32 st = d.x + k * s, len = min(s, d.y - k * s);
        next[slot + k] = make_uint4(st, len, d.z, 0);     // (a failed exact single has d.y == 1: rejected above)
    }
}

// ---------------------------------------------------------------- host launch wrappers
extern "C" void lcbk_tpke_rlc_points(dim3 grid, hipStream_t s, u32 n_cts, const void *keys, u32 n_keys,
                                     const u32 *ct_idx, const u32 *dec_idx, const uint8_t *ui, u32 n,
                                     const u32 key[10], u32 *rU, u32 *rY, uint8_t *accept) {
    rlc_key k;
    for (int j = 0; j < 8; j++) k.k[j] = key[j];
    k.nonce[0] = key[8];
    k.nonce[1] = key[9];
    LCB_LAUNCH(k_tpke_rlc_points, n_cts, (const g1a_st *)keys, n_keys, ct_idx, dec_idx, ui, n, k, rU, rY, accept);
}
extern "C" u32 lcbk_rlc_span() { return LCB_RLC_SPAN; }
extern "C" void lcbk_rlc_groups(dim3 grid, hipStream_t s, const u32 *ct_idx, u32 n, u32 n_cts, void *desc, u32 *count) {
    LCB_LAUNCH(k_rlc_groups, ct_idx, n, n_cts, (uint4 *)desc, count);
}
extern "C" void lcbk_tpke_rlc_sum(dim3 grid, hipStream_t s, const void *desc, u32 n_groups, const uint8_t *ct_ok,
                                  const uint8_t *ct_g2, const void *keys, u32 n_keys, const u32 *dec_idx,
                                  const uint8_t *ui, const u32 *rU, const u32 *rY, u32 n, void *gpts,
                                  uint8_t *accept, uint8_t *gexact) {
    LCB_LAUNCH(k_tpke_rlc_sum, (const uint4 *)desc, n_groups, ct_ok, ct_g2, (const g1a_st *)keys, n_keys, dec_idx, ui,
               rU, rY, n, (g1a_st *)gpts, accept, gexact);
}
extern "C" void lcbk_tpke_ct_g2check(dim3 grid, hipStream_t s, const u32 *lines, const uint8_t *ct_ok, u32 n_cts,
                                     uint8_t *ct_g2) {
    LCB_LAUNCH(k_tpke_ct_g2check, lines, ct_ok, n_cts, ct_g2);
}
extern "C" void lcbk_tpke_rlc_miller(dim3 grid, hipStream_t s, const u32 *lines, const void *desc, const void *gpts,
                                     u32 n_groups, u32 *f_soa, uint8_t *gacc) {
    LCB_LAUNCH(k_tpke_rlc_miller, lines, (const uint4 *)desc, (const g1a_st *)gpts, n_groups, f_soa, gacc);
}
extern "C" void lcbk_rlc_resolve(dim3 grid, hipStream_t s, const void *desc, u32 n_groups, const uint8_t *gacc,
                                 const uint8_t *gexact, uint8_t *accept, void *next, u32 *next_count) {
    LCB_LAUNCH(k_rlc_resolve, (const uint4 *)desc, n_groups, gacc, gexact, accept, (uint4 *)next, next_count);
}
