// lachain_amd/csrc/k_batch.hip — gfx950 kernels: randomized batch verification of TPKE decryption shares
// (small-exponent test, Bellare–Garay–Rabin 1998) over the per-share check of TPKE/PublicKey.cs:88-92.
//
// The reference decides every share on its own: e(U_i, H) == e(Y_i, W) (two pairings per share).  Every value
// e(., .) is a reduced pairing, so the ratio g_i = e(U_i, H) / e(Y_i, W) lies in mu_r (order r, prime) whatever
// U_i is: for a G2 point Q the (ate) pairing is linear in its G1 argument on all of E(Fp) (Weil reciprocity; the
// error term is an r-th power, killed by the final exponentiation) and kills the cofactor-torsion part, so off-
// subgroup U_i / Y_i are covered.  H is in G2 by construction; W is checked (k_lineset_fill, lineset_in_g2) and a ciphertext with
// W outside G2 gets exact per-share checks.  For secret random exponents s_i (2^64 values, none 0 mod r; rlc_scalar):
// prod_i g_i^(s_i) == 1  <=>  e(sum s_i U_i, H) e(-sum s_i Y_i, W) == 1, and if some g_i != 1 the product is 1 with
// probability <= 2^-64.  So one Miller pair + final exponentiation decides a whole group of shares of one ciphertext;
// a group that fails is split and re-checked, down to single shares, where g_i^(s_i) == 1 <=> g_i == 1 (gcd(s_i, r)
// = 1): every rejected share is rejected by an exact check of its own, every accepted share by a group check (false
// accept <= 2^-64 per group, over the secret exponents).
//
// Level 2 (one bad share per group, the usual failure): the first level also forms W = sum (j+1) s_j U_j etc. (j = the
// share's position in its group, so the weights c_j = j+1 are distinct and public).  A failed group's gamma =
// prod g_i^(s_i) (its final-exponentiation output) and gamma' = prod g_i^(c_i s_i) (one more group check) satisfy
// gamma' = gamma^(c_j) exactly when j is the only bad share: k_rlc_search tries c = 1..len (len Fp12 products) and
// rejects share j; with two or more bad shares no c matches except with probability <= len 2^-64 (the exponents
// s_i are secret), and the group's shares get single checks at the next level.  So at most three levels.
//
// Pipeline (host side in lcb_host.cpp: rlc_points_enqueue + rlc_levels):
//   k_tpke_rlc_points   one lane per share: validity as k_tpke_miller, (a_i, b_i) = ChaCha20(key, i), s_i U_i and
//                       s_i Y_i with s_i = a_i + b_i lambda (32-bit GLV form, rlc_scalar) -> quad-major SoA Jacobian
//                       records (invalid share: infinity)
//   k_rlc_groups        one lane per 256 consecutive shares: runs of equal ciphertext index (<= 32) -> level-1 groups
//   k_lineset_fill      (k_tpke.hip) W's line set also decides W in G2 (else its shares get exact per-share checks)
//   k_tpke_rlc_sum      one lane per group: ciphertext validity, the two sums, to affine with one shared inversion,
//                       -sum s_i Y_i (or an exact single share's own U_i, -Y_i)
//   k_tpke_rlc_miller   one lane per group: the two-pair Miller loop over the ciphertext's line sets
//   k_final_exp_check   (k_tpke.hip) group decision
//   k_rlc_resolve       one lane per group: failed single share -> reject; failed group -> sub-groups of the next level
#include "kcommon.hpp"
#include "rlc_common.hpp"
#include "ts_rlc.hpp"

LCB_ASM_LIBRARY(k_batch)
LCB_TU_CONFIG(k_batch)
#ifndef LCB_SEARCH2B_BY_POSITION
#define LCB_SEARCH2B_BY_POSITION 0
#endif
#ifndef LCB_SEARCH2B_DEBUG
#define LCB_SEARCH2B_DEBUG 0
#endif
#if LCB_SEARCH2B_DEBUG
// diagnostic builds only: per (open check, lane) fingerprints of D, E, gamma_c^-(c_j + 1), the group, found, cand
__device__ u32 *lcb_s2b_dbg = nullptr;
#endif

// ---------------------------------------------------------------- level-1 groups: runs of one ciphertext / message
// one lane per share; the first share of a run emits the run as groups of at most `cap` shares.
// desc = {first share, length, ciphertext / message, 0}; order of the records is irrelevant
extern "C" __global__ void LCB_BOUNDS k_rlc_groups(const u32 *key_idx, u32 i0, u32 n, u32 n_keys, u32 cap,
                                                  uint4 *desc, u32 *count) {
    LCB_LATENCY_PRIO();
    u32 i = i0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u32 c = key_idx[i];
    c = c < n_keys ? c : 0;
    if (i > i0) {
        u32 p = key_idx[i - 1];
        p = p < n_keys ? p : 0;
        if (p == c) return;
    }
    u32 j = i + 1;
    while (j < n) {
        u32 q = key_idx[j];
        q = q < n_keys ? q : 0;
        if (q != c) break;
        j++;
    }
    for (u32 st = i; st < j; st += cap) {
        u32 len = min(cap, j - st);
        u32 slot = atomicAdd(count, 1u);
        desc[slot] = make_uint4(st, len, c, 0);
    }
}

// the weighted sums of the level-1 groups listed in sdesc (.w = level-1 group index) as affine records
extern "C" __global__ void LCB_BOUNDS k_tpke_rlc_wsum(const uint4 *sdesc, u32 n_s, const u32 *wsum, u32 n_l1,
                                                     g1a_st *gpts) {
    LCB_LATENCY_PRIO();
    u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_s) return;
    u32 l = sdesc[g].w;
    g1 p;
    g1a_st o;
    g1_load_soa(p, wsum, 2 * (size_t)n_l1, 2 * (size_t)l);
    g1_to_st_gcd(o, p, false);
    gpts[2 * (size_t)g] = o;
    g1_load_soa(p, wsum, 2 * (size_t)n_l1, 2 * (size_t)l + 1);
    g1_to_st_gcd(o, p, true);
    gpts[2 * (size_t)g + 1] = o;
}

// ---------------------------------------------------------------- threshold signatures: the group sums and Miller
// loops (ts_rlc.hpp)
extern "C" __global__ void LCB_BOUNDS k_ts_rlc_sum(const uint4 *desc, u32 n_groups, u32 first, const uint8_t *msg_ok,
                                                  const g1a_st *pks, u32 n_pks, const u32 *pk_idx, const uint8_t *sigs,
                                                  const u32 *rP, const u32 *rS, u32 n, ts_grp *gpts, uint8_t *accept,
                                                  uint8_t *gexact, u32 *wsum, const u32 *susp, uint8_t *cval) {
    LCB_LATENCY_PRIO();
    ts_rlc_sum_run(desc, n_groups, first, msg_ok, pks, n_pks, pk_idx, sigs, rP, rS, n, gpts, accept, gexact, wsum, susp,
                   cval);
}
extern "C" __global__ void LCB_BOUNDS k_ts_rlc_wsum(const uint4 *sdesc, u32 n_s, const u32 *wsum, u32 n_l1,
                                                   ts_grp *gpts) {
    LCB_LATENCY_PRIO();
    u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_s) return;
    u32 l = sdesc[g].w;
    g1 p;
    g2 q;
    ts_grp o;
    g1_load_soa(p, wsum, n_l1, l);
    g2_load_soa(q, wsum + (size_t)36 * n_l1, n_l1, l);
    g1_to_st_gcd(o.p, p, false);
    g2_to_st_gcd(o.s, q);
    gpts[g] = o;
}
extern "C" __global__ void LCB_PAIR_BOUNDS k_ts_rlc_miller(const u32 *lines, const uint4 *desc, const ts_grp *gpts,
                                                          u32 n_groups, u32 *f_soa, uint8_t *gacc) {
    LCB_LATENCY_PRIO();
    ts_rlc_miller_run(lines, desc, gpts, n_groups, f_soa, gacc);
}

// ---------------------------------------------------------------- resolve a level (TPKE and TS)
// Groups [o, o + m) of this level, decided by the final-exponentiation chunk park (stride m).  A failed group of one
// share rejects it.  At level 1 (first) a failed group of len > 1 goes to the search list (its gamma copied out of the
// park); below level 1 it becomes ceil(len / s) sub-groups of s = ceil(len / ceil(sqrt(len))) shares, or single
// shares when len <= LCB_RLC_SINGLES.  gexact (TPKE: W outside G2): every share of the group gets an exact single.
extern "C" __global__ void LCB_BOUNDS k_rlc_resolve(const uint4 *desc, u32 o, u32 m, const uint8_t *gacc,
                                                   const uint8_t *gexact, const u32 *park, u32 first, uint8_t *accept,
                                                   uint4 *next, u32 *next_count, uint4 *search, u32 *search_count,
                                                   u32 *gamma, const u32 *key_idx, u32 n_keys, const u32 *susp) {
    LCB_LATENCY_PRIO();
    u32 gl = blockIdx.x * blockDim.x + threadIdx.x;
    if (gl >= m) return;
    u32 g = o + gl;
    uint4 d = desc[g];
    if (gexact && gexact[g]) {           // W outside G2: every share of the group gets its exact check
        emit_singles(d, 1, accept, key_idx, n_keys, susp, next, next_count);
        return;
    }
    if (gacc[g]) return;
    if (d.y == 1) { accept[d.x] = 0; return; }        // (exact singles always have d.y == 1)
    if (first) {
        u32 slot = atomicAdd(search_count, 1u);
        search[slot] = make_uint4(d.x, d.y, d.z, g);
        fp12 f;
        fp12_load_soa(f, park, m, gl);
        const u32 *w = (const u32 *)&f;
        uint4 *dst = (uint4 *)(gamma + (size_t)slot * 144);
#pragma unroll
        for (int q = 0; q < 36; q++) dst[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
        return;
    }
    if (d.y <= LCB_RLC_SINGLES) {
        emit_singles(d, 0, accept, key_idx, n_keys, susp, next, next_count);
        return;
    }
    u32 parts = 1;
    while (parts * parts < d.y) parts++;
    u32 s = (d.y + parts - 1) / parts;
    u32 cnt = (d.y + s - 1) / s;
    u32 slot = atomicAdd(next_count, cnt);
    for (u32 k = 0; k < cnt; k++) {
        u32 st = d.x + k * s, len = min(s, d.y - k * s);
        next[slot + k] = make_uint4(st, len, d.z, 0);
    }
}
// the final-exponentiation outputs of checks [o, o + m) (park stride m) -> rows o.. of dst (576 B each)
// *flag |= 1 when a line set of ciphertexts [c0, c1) is not normalised (the Miller fallback will be needed)
extern "C" __global__ void LCB_BOUNDS k_lines_unnormalised(const u32 *lines, u32 c0, u32 c1, u32 *flag) {
    LCB_LATENCY_PRIO();
    const u32 k = 2 * c0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= 2 * c1) return;
    if (!lineset_normalised(lines + (size_t)k * LCB_LINESET_WORDS)) atomicOr(flag, 1u);
}
extern "C" __global__ void LCB_BOUNDS k_rlc_park_copy(const u32 *park, u32 o, u32 m, u32 *dst, const u32 *map) {
    LCB_LATENCY_PRIO();
    u32 gl = blockIdx.x * blockDim.x + threadIdx.x;
    if (gl >= m) return;
    fp12 f;
    fp12_load_soa(f, park, m, gl);
    const u32 *w = (const u32 *)&f;
    uint4 *d = (uint4 *)(dst + (size_t)(map ? map[o + gl] : o + gl) * 144);   // (map: row of check o + gl)
#pragma unroll
    for (int q = 0; q < 36; q++) d[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}
// r = a^e for a in the cyclotomic subgroup (GT), e >= 1
DN void gt_pow_small(fp12 &r, const fp12 &a, u32 e) {
    fp12 t = a;
    int top = 31;
    while (top > 0 && !((e >> top) & 1)) top--;
    for (int b = top - 1; b >= 0; b--) {
        fp12_cyc_sqr_n(t, t);
        if ((e >> b) & 1) fp12_mul_n(t, t, a);
    }
    r = t;
}
// x <- x_0 x_1 ... x_j over lane j's half-wave (inclusive product scan; Hillis-Steele, five shuffle rounds).  Every
// lane of the wave must be active.
DN void gt_half_scan(fp12 &x) {
    const u32 j = threadIdx.x & 31;
#pragma unroll 1
    for (u32 off = 1; off < 32; off <<= 1) {
        fp12 y;
        u32 *yw = (u32 *)&y;
        const u32 *xw = (const u32 *)&x;
#pragma unroll
        for (int q = 0; q < 144; q++) yw[q] = (u32)__shfl_up((int)xw[q], off, 32);
        if (j >= off) fp12_mul_n(x, x, y);
    }
}
// Level 2: search entries [o, o + m): gamma' (the weighted group check's final-exponentiation output, park stride m)
// against gamma^c, c = 1..len.  A match rejects share c - 1 of the group (the only bad one, see the header); no match
// sends every share of the group to a single check at the next level.  gamma != 1 (the group failed) has order r, so at
// most one c in [1, len] matches.  Baby-step giant-step (round 5; the linear scan took len / 2 products on average,
// 13.5 ms for configs[2]'s 100-share rounds): 32-bit fingerprints of gamma^1 .. gamma^M, giant steps
// Y_i = gamma' gamma^(-M i) (gamma is unitary: gamma^-M = conj(gamma^M)); the first fingerprint match Y_i ~ gamma^(k+1)
// names the candidate c = M i + k + 1, confirmed by the full comparison gamma^c == gamma' — M + len / (2M) + ~10
// products.  A fingerprint collision that is not a match (probability ~ len 2^-32) falls back to the linear scan, so
// the decision is the linear scan's in every case.
#define RLC_BS_M 12
DN u32 rlc_search_linear(const fp12 &gm, const fp12 &gp, u32 len) {
    fp12 acc = gm;
    for (u32 c = 1; c <= len; c++) {
        if (fp12_words_eq(acc, gp)) return c;
        fp12_mul_n(acc, acc, gm);
    }
    return 0;
}
extern "C" __global__ void LCB_BOUNDS k_rlc_search(const uint4 *search, u32 o, u32 m, const u32 *gamma, const u32 *park,
                                                  uint8_t *accept, uint4 *next, u32 *next_count, const u32 *key_idx,
                                                  u32 n_keys, const u32 *susp) {
    LCB_LATENCY_PRIO();
    u32 gl = blockIdx.x * blockDim.x + threadIdx.x;
    if (gl >= m) return;
    u32 g = o + gl;
    uint4 d = search[g];
    const u32 *grow = gamma + (size_t)g * 144;
    fp12 y, t;
    u32 fpb[RLC_BS_M];
    fp12_load_row(t, grow);
    fpb[0] = fp12_fingerprint(t);
    if (d.y > 1) {
        fp12 gm;
        fp12_load_row(gm, grow);
#pragma unroll
        for (int k = 1; k < RLC_BS_M; k++) {
            fp12_mul_n(t, t, gm);
            fpb[k] = fp12_fingerprint(t);
        }
    }
    fp12_conj(t, t);                                       // gamma^-M
    fp12_load_soa(y, park, m, gl);                         // Y_0 = gamma'
    u32 cand = 0;
    for (u32 base = 0; base < d.y && !cand; base += RLC_BS_M) {
        const u32 fy = fp12_fingerprint(y);
#pragma unroll
        for (int k = 0; k < RLC_BS_M; k++)
            if (!cand && base + k + 1 <= d.y && fpb[k] == fy) cand = base + k + 1;
        if (!cand && base + RLC_BS_M < d.y) fp12_mul_n(y, y, t);
    }
    u32 found = 0;
    if (cand) {
        fp12 gm, gp;
        fp12_load_row(gm, grow);
        fp12_load_soa(gp, park, m, gl);
        gt_pow_small(t, gm, cand);
        found = fp12_words_eq(t, gp) ? cand : rlc_search_linear(gm, gp, d.y);
    }
    if (found) {
        accept[d.x + found - 1] = 0;
        return;
    }
    emit_singles(d, 0, accept, key_idx, n_keys, susp, next, next_count);
}
// Level 2 of TPKE: locate up to TWO bad shares per failed group.  With e_i = s_i log g_i (nonzero exactly for the bad
// shares) the three group values are gamma_0 (level 1) ~ sum e_i, gamma_c ~ sum e_i c_i and gamma_t ~ sum e_i t_i, so
// gamma_2 = gamma_t^2 / gamma_c ~ sum e_i c_i^2 (c^2 = 2t - c).
//   one error at j:      gamma_c = gamma_0^(c_j)  (k_tpke_rlc_search2a: four lanes per group, c = 1..len);
//   two errors at j, k:  for lane j of the group's half-wave (k_tpke_rlc_search2b, only the groups 2a left open),
//                        D_j = gamma_c / gamma_0^(c_j) ~ e_k (c_k - c_j) and E_j = gamma_2 / gamma_c^(c_j) ~
//                        e_k c_k (c_k - c_j), so E_j = D_j^(c_k): exactly two lanes whose searches name each other
//                        reject both shares.
// Any other outcome (three or more bad shares) sends the group's shares to single checks.  A false location needs a
// relation among the e_i, whose factors s_i are secret: probability <= len^2 2^-64 per group.
extern "C" __global__ void LCB_BOUNDS k_tpke_rlc_search2a(const uint4 *search, u32 ns, const u32 *gamma0,
                                                         const u32 *gamma12, uint8_t *accept, u32 *open,
                                                         u32 *open_count) {
    LCB_LATENCY_PRIO();
    // four lanes per group (a latency-bound launch of ~1 % of the groups): lane r tries c = r + 1, r + 5, ... from
    // gamma_0^(r+1) in steps of gamma_0^4, so the serial chain is ~len/4 products instead of len.  The smallest c that
    // matches wins, as in the one-lane scan.  No lane returns early: the shuffles below need the whole wave.
    const u32 t = blockIdx.x * blockDim.x + threadIdx.x, g = t >> 2, r = t & 3;
    const bool live = g < ns;
    const uint4 d = live ? search[g] : make_uint4(0, 0, 0, 0);
    u32 found = 0xffffffffu;
    if (live) {
        fp12 gm, gc, acc, st;
        fp12_load_row(gm, gamma0 + (size_t)g * 144);
        fp12_load_row(gc, gamma12 + (size_t)g * 144);
        gt_pow_small(acc, gm, r + 1);
        fp12_cyc_sqr_n(st, gm);
        fp12_cyc_sqr_n(st, st);
        for (u32 c = r + 1; c <= d.y; c += 4) {
            if (fp12_words_eq(acc, gc)) { found = c; break; }
            if (c + 4 <= d.y) fp12_mul_n(acc, acc, st);
        }
    }
    found = min(found, (u32)__shfl_xor((int)found, 1));
    found = min(found, (u32)__shfl_xor((int)found, 2));
    if (live && r == 0) {
        if (found != 0xffffffffu) accept[d.x + found - 1] = 0;
        else open[atomicAdd(open_count, 1u)] = g;
    }
}
extern "C" __global__ void __launch_bounds__(64) k_tpke_rlc_search2b(const uint4 *search, u32 ns, const u32 *gamma0,
                                                                    const u32 *gamma12, const u32 *open,
                                                                    const u32 *open_count, uint8_t *accept, uint4 *next,
                                                                    u32 *next_count, const u32 *key_idx, u32 n_keys,
                                                                    const u32 *susp) {
    LCB_LATENCY_PRIO();
    const u32 j = threadIdx.x & 31, k = blockIdx.x * 2 + (threadIdx.x >> 5);
    if (blockIdx.x * 2 >= *open_count) return;          // (uniform per block)
    const bool live = k < *open_count;
    const u32 g = live ? open[k] : 0;
    const uint4 d = live ? search[g] : make_uint4(0, 0, 0, 0);
    const bool cand = live && j < d.y && accept[d.x + j] && !key_suspect(susp, key_idx[d.x + j], n_keys);
    const u32 cj = j + 1;
    fp12 a, b, D;
    // gamma_0^(c_j) and gamma_c^(c_j + 1) for every lane j of the half-wave from product scans over its 32 lanes
    // (5 products each) instead of one square-and-multiply per lane
    fp12_load_row(b, gamma0 + (size_t)g * 144);
    gt_half_scan(b);                                       // gamma_0^(c_j)
    fp12_conj(b, b);
    fp12_load_row(a, gamma12 + (size_t)g * 144);           // gamma_c
    fp12_mul_n(D, a, b);                                   // D_j = gamma_c / gamma_0^(c_j)
    gt_half_scan(a);                                       // gamma_c^(c_j)
    fp12_load_row(b, gamma12 + (size_t)g * 144);
    fp12_mul_n(b, a, b);                                   // gamma_c^(c_j + 1)
    fp12_conj(b, b);
#if LCB_SEARCH2B_BY_POSITION
    fp12_load_row(a, gamma12 + ((size_t)ns + k) * 144);    // gamma_t of open check k (diagnostic variant)
#else
    fp12_load_row(a, gamma12 + ((size_t)ns + g) * 144);    // gamma_t
#endif
    fp12_cyc_sqr_n(a, a);
    fp12_mul_n(a, a, b);                                   // E_j = gamma_t^2 / gamma_c^(c_j + 1) = gamma_2 / gamma_c^(c_j)
#if LCB_SEARCH2B_DEBUG
    if (lcb_s2b_dbg && live) {
        u32 *o = lcb_s2b_dbg + ((size_t)k * 32 + j) * 8;
        o[0] = fp12_fingerprint(D);
        o[1] = fp12_fingerprint(a);
        o[2] = fp12_fingerprint(b);
        o[3] = g;
    }
#endif
    // E_j = D_j^c for some c in [1, len] (len <= 32): baby-step giant-step with m = 6 — 32-bit fingerprints of the
    // baby values D^k (k = 1..6), giant steps Y_i = E D^(-6 i) (D is unitary: D^-6 = conj(D^6)), a fingerprint match
    // Y_i ~ D^(k+1) confirmed by the full comparison Y_i == D^(k+1) (<=> E == D^c, c = 6 i + k + 1): 10 products
    // instead of up to len
    u32 found = 0;
    if (cand) {
        u32 fpb[6];
        fpb[0] = fp12_fingerprint(D);
        b = D;
#pragma unroll
        for (int k = 1; k < 6; k++) {
            fp12_mul_n(b, b, D);
            fpb[k] = fp12_fingerprint(b);
        }
        fp12_conj(b, b);                                   // D^-6
        for (int i = 0; i < 6 && !found; i++) {
            const u32 h = fp12_fingerprint(a);
#pragma unroll 1
            for (int k = 0; k < 6; k++) {
                const u32 c = 6 * i + k + 1;
                if (!found && h == fpb[k] && c <= d.y && c != cj) {
                    fp12 chk = D;
#pragma unroll 1
                    for (int q = 0; q < k; q++) fp12_mul_n(chk, chk, D);
                    if (fp12_words_eq(chk, a)) found = c;
                }
            }
            if (i < 5) fp12_mul_n(a, a, b);
        }
    }
#if LCB_SEARCH2B_DEBUG
    if (lcb_s2b_dbg && live) {
        u32 *o = lcb_s2b_dbg + ((size_t)k * 32 + j) * 8;
        o[4] = found;
        o[5] = cand;
    }
#endif
    const u32 m2 = half_ballot(found != 0);
    const u32 m3 = half_ballot(found != 0 && !((m2 >> ((found - 1) & 31u)) & 1u));
    if (__popc(m2) == 2 && !m3) {
        if (found) accept[d.x + j] = 0;
    } else if (live && j == 0) {
        emit_singles(d, 0, accept, key_idx, n_keys, susp, next, next_count);
    }
}

// ---------------------------------------------------------------- census (suspect keys) and the level-1 split
// exact singles of shares [0, m): desc = {i, 1, group index (ciphertext / message), 1}; an out-of-range index rejects
extern "C" __global__ void LCB_BOUNDS k_rlc_census_desc(const u32 *grp_idx, const u32 *key_idx, u32 m, u32 n_grp,
                                                       u32 n_keys, uint4 *desc, uint8_t *accept) {
    LCB_LATENCY_PRIO();
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    u32 c = grp_idx[i];
    bool ok = c < n_grp && key_idx[i] < n_keys;
    accept[i] = ok;
    desc[i] = make_uint4(i, 1, ok ? c : 0, 1);
}
// one lane per key: over the census shares that were live (cval), the key is suspect when at least two were sampled
// and at least half of them failed their exact check.  count[0] += suspect keys.
extern "C" __global__ void LCB_BOUNDS k_rlc_census_stats(const u32 *key_idx, u32 m, u32 n_keys, const uint8_t *cval,
                                                        const uint8_t *accept, u32 *susp, u32 *count) {
    LCB_LATENCY_PRIO();
    u32 k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_keys) return;
    u32 live = 0, bad = 0;
    for (u32 i = 0; i < m; i++) {
        if (key_idx[i] != k || !cval[i]) continue;
        live++;
        bad += accept[i] == 0;
    }
    if (live >= 2 && 2 * bad >= live) {
        atomicOr(susp + (k >> 5), 1u << (k & 31));
        atomicAdd(count, 1u);
    }
}
// level 1 with suspect keys: every group keeps its place (its sum skips the suspect keys' shares) unless it has no
// live share of another key (then it is dropped), and each live share of a suspect key becomes an exact single.  count: [0] entries out
extern "C" __global__ void LCB_BOUNDS k_rlc_suspect_split(const uint4 *desc, u32 n_groups, const u32 *key_idx,
                                                         u32 n_keys, const u32 *susp, const uint8_t *accept,
                                                         uint4 *out, u32 *count) {
    LCB_LATENCY_PRIO();
    u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_groups) return;
    uint4 d = desc[g];
    u32 ns = 0, nc = 0;
    for (u32 k = 0; k < d.y; k++) {
        if (!accept[d.x + k]) continue;
        if (key_suspect(susp, key_idx[d.x + k], n_keys)) ns++;
        else nc++;
    }
    if (!nc && !ns) return;              // nothing live: every share of the group is already rejected
    u32 slot = atomicAdd(count, ns + (nc ? 1u : 0u));
    if (nc) out[slot++] = d;
    for (u32 k = 0; k < d.y; k++)
        if (accept[d.x + k] && key_suspect(susp, key_idx[d.x + k], n_keys))
            out[slot++] = make_uint4(d.x + k, 1, d.z, 1);
}

// ---------------------------------------------------------------- host launch wrappers
// table workspace per key: Jacobian scratch 144 B + prefix products 48 B + table 144 B per entry + 32 flags
extern "C" size_t lcbk_key_table_bytes(u32 n_keys) {
    return (size_t)n_keys * (LCB_KTAB_ENTRIES * 336 + LCB_KTAB_LANES) + 16;
}
extern "C" void lcbk_rlc_groups(hipStream_t s, const u32 *key_idx, u32 i0, u32 n, u32 n_keys, u32 cap, void *desc,
                                u32 *count) {
    dim3 grid((n - i0 + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_rlc_groups, key_idx, i0, n, n_keys, cap, (uint4 *)desc, count);
}
extern "C" void lcbk_tpke_rlc_wsum(dim3 grid, hipStream_t s, const void *sdesc, u32 n_s, const u32 *wsum, u32 n_l1,
                                   void *gpts) {
    LCB_LAUNCH(k_tpke_rlc_wsum, (const uint4 *)sdesc, n_s, wsum, n_l1, (g1a_st *)gpts);
}
extern "C" void lcbk_ts_rlc_sum(dim3 grid, hipStream_t s, const void *desc, u32 n_groups, u32 first,
                                const uint8_t *msg_ok, const void *pks, u32 n_pks, const u32 *pk_idx,
                                const uint8_t *sigs, const u32 *rP, const u32 *rS, u32 n, void *gpts, uint8_t *accept,
                                uint8_t *gexact, u32 *wsum, const u32 *susp, uint8_t *cval) {
    LCB_LAUNCH(k_ts_rlc_sum, (const uint4 *)desc, n_groups, first, msg_ok, (const g1a_st *)pks, n_pks, pk_idx, sigs,
               rP, rS, n, (ts_grp *)gpts, accept, gexact, wsum, susp, cval);
}
extern "C" void lcbk_ts_rlc_wsum(dim3 grid, hipStream_t s, const void *sdesc, u32 n_s, const u32 *wsum, u32 n_l1,
                                 void *gpts) {
    LCB_LAUNCH(k_ts_rlc_wsum, (const uint4 *)sdesc, n_s, wsum, n_l1, (ts_grp *)gpts);
}
extern "C" void lcbk_ts_rlc_miller(dim3 grid, hipStream_t s, const u32 *lines, const void *desc, const void *gpts,
                                   u32 n_groups, u32 *f_soa, uint8_t *gacc) {
    LCB_LAUNCH(k_ts_rlc_miller, lines, (const uint4 *)desc, (const ts_grp *)gpts, n_groups, f_soa, gacc);
}
extern "C" void lcbk_rlc_resolve(dim3 grid, hipStream_t s, const void *desc, u32 o, u32 m, const uint8_t *gacc,
                                 const uint8_t *gexact, const u32 *park, u32 first, uint8_t *accept, void *next,
                                 u32 *next_count, void *search, u32 *search_count, u32 *gamma, const u32 *key_idx,
                                 u32 n_keys, const u32 *susp) {
    LCB_LAUNCH(k_rlc_resolve, (const uint4 *)desc, o, m, gacc, gexact, park, first, accept, (uint4 *)next, next_count,
               (uint4 *)search, search_count, gamma, key_idx, n_keys, susp);
}
extern "C" void lcbk_rlc_search(dim3 grid, hipStream_t s, const void *search, u32 o, u32 m, const u32 *gamma,
                                const u32 *park, uint8_t *accept, void *next, u32 *next_count, const u32 *key_idx,
                                u32 n_keys, const u32 *susp) {
    LCB_LAUNCH(k_rlc_search, (const uint4 *)search, o, m, gamma, park, accept, (uint4 *)next, next_count, key_idx,
               n_keys, susp);
}
extern "C" void lcbk_lines_unnormalised(hipStream_t s, const u32 *lines, u32 c0, u32 c1, u32 *flag) {
    if (c1 <= c0) return;
    dim3 grid((2 * (c1 - c0) + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_lines_unnormalised, lines, c0, c1, flag);
}
extern "C" void lcbk_rlc_park_copy(hipStream_t s, const u32 *park, u32 o, u32 m, u32 *dst, const u32 *map) {
    dim3 grid((m + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_rlc_park_copy, park, o, m, dst, map);
}
extern "C" void lcbk_tpke_rlc_search2a(hipStream_t s, const void *search, u32 ns, const u32 *gamma0,
                                       const u32 *gamma12, uint8_t *accept, u32 *open, u32 *open_count) {
    (void)hipMemsetAsync(open_count, 0, 4, s);
    dim3 grid((4 * ns + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_tpke_rlc_search2a, (const uint4 *)search, ns, gamma0, gamma12, accept, open, open_count);
}
// 1: the diagnostic variant that reads gamma_t of open check k at row ns + k (the copy then writes rows by check)
extern "C" int lcbk_search2b_by_position(void) { return LCB_SEARCH2B_BY_POSITION; }
// diagnostic builds (-DLCB_SEARCH2B_DEBUG=1): point the kernel's record buffer at p (nullptr: off); -1 in other builds
extern "C" int lcbk_search2b_debug(void *p) {
#if LCB_SEARCH2B_DEBUG
    return hipMemcpyToSymbol(HIP_SYMBOL(lcb_s2b_dbg), &p, sizeof p) == hipSuccess ? 0 : -1;
#else
    (void)p;
    return -1;
#endif
}
// n_open = *open_count (read by the host after search2a); gamma12 + 144 (ns + g) holds gamma_t of the open group g
extern "C" void lcbk_tpke_rlc_search2b(hipStream_t s, const void *search, u32 ns, u32 n_open, const u32 *gamma0,
                                       const u32 *gamma12, const u32 *open, const u32 *open_count, uint8_t *accept,
                                       void *next, u32 *next_count, const u32 *key_idx, u32 n_keys, const u32 *susp) {
    if (!n_open) return;
    LCB_LAUNCH_GATED(k_tpke_rlc_search2b, dim3((n_open + 1) / 2), dim3(64), 0, s, (const uint4 *)search, ns, gamma0,
                       gamma12, open, open_count, accept, (uint4 *)next, next_count, key_idx, n_keys, susp);
}
extern "C" void lcbk_rlc_census_desc(hipStream_t s, const u32 *grp_idx, const u32 *key_idx, u32 m, u32 n_grp,
                                     u32 n_keys, void *desc, uint8_t *accept) {
    dim3 grid((m + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_rlc_census_desc, grp_idx, key_idx, m, n_grp, n_keys, (uint4 *)desc, accept);
}
extern "C" void lcbk_rlc_census_stats(hipStream_t s, const u32 *key_idx, u32 m, u32 n_keys, const uint8_t *cval,
                                      const uint8_t *accept, u32 *susp, u32 *count) {
    dim3 grid((n_keys + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_rlc_census_stats, key_idx, m, n_keys, cval, accept, susp, count);
}
extern "C" void lcbk_rlc_suspect_split(hipStream_t s, const void *desc, u32 n_groups, const u32 *key_idx, u32 n_keys,
                                       const u32 *susp, const uint8_t *accept, void *out, u32 *count) {
    dim3 grid((n_groups + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_rlc_suspect_split, (const uint4 *)desc, n_groups, key_idx, n_keys, susp, accept, (uint4 *)out, count);
}
extern "C" size_t lcbk_ts_grp_bytes() { return sizeof(ts_grp); }
