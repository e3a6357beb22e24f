// lachain_amd/csrc/k_msm.hip — gfx950 Pippenger multi-scalar multiplication over G1 (SURVEY.md §8a row a4 at
// scale, BASELINE configs[3]).  Lagrange-in-the-exponent for large k reduces to sum_i s_i P_i
// (MclBls12381.LagrangeInterpolate, called from TPKE/PublicKey.cs:83 and ThresholdSignature/PublicKeySet.cs:31).
//
// Pipeline (one stream, no host round trip):
//   1. k_msm_digits      one lane per point: signed c-bit digits of s_i (s_i mod r), one (key, value) record per
//                        window; key = window * 2^(c-1) + |digit| - 1 (or a sentinel for digit 0), value = point
//                        index | sign << 31.  Window-major so a wave writes 256 contiguous bytes per window.
//   2. radix sort        hipCUB DeviceRadixSort on the (key, value) pairs, only the key bits that are used.
//   3. k_msm_bounds      start/end of every bucket in the sorted order.
//   4. k_msm_bucket_acc  one lane per bucket: Jacobian += affine (mixed add, 11 Fp-mul) over its points.  This is
//                        the HBM phase: each record gathers a 96-byte affine point.
//   5. k_msm_bucket_reduce  one lane per segment of L buckets: running-sum trick sum_j (j+1) B_j, plus a*T to
//                        place the segment at its offset a inside the window.
//   6. k_g1_jac_reduce_block (LDS tree, until one sum per window) + k_msm_horner: sum_w 2^(c w) W_w by doubling.
// Points are affine, Montgomery form, 12 x u32 limbs per coordinate (= the x,y words of mcl's mclBnG1 with
// z = 1); (0, 0) encodes the point at infinity.
#include "coop_pt.hpp"
#include <hipcub/hipcub.hpp>

LCB_ASM_LIBRARY(k_msm)
LCB_TU_CONFIG(k_msm)

// s mod r for any 256-bit s (2^256 < 3r: at most two subtractions)
DI void fr_raw_reduce(fr &s) {
#pragma unroll
    for (int k = 0; k < 2; k++) {
        if (fr_raw_lt_r(s)) return;
        u32 br = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            u64 x = (u64)s.v[j] - LCB_R[j] - br;
            s.v[j] = (u32)x;
            br = (u32)(x >> 32) & 1;
        }
    }
}
DI u32 word_sel(const fr &s, u32 k) {  // s.v[k] without dynamic register indexing (0 past the top)
    u32 r = 0;
#pragma unroll
    for (u32 j = 0; j < 8; j++) r = (j == k) ? s.v[j] : r;
    return r;
}

extern "C" __global__ void LCB_BOUNDS k_msm_digits(const uint8_t *scalars, u32 n, u32 c, u32 nwin, u32 *keys,
                                                  u32 *vals) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fr s;
    const uint4 *sw = (const uint4 *)(scalars + 32 * (size_t)i);
    uint4 a = sw[0], b = sw[1];
    s.v[0] = a.x; s.v[1] = a.y; s.v[2] = a.z; s.v[3] = a.w;
    s.v[4] = b.x; s.v[5] = b.y; s.v[6] = b.z; s.v[7] = b.w;
    fr_raw_reduce(s);
    const u32 half = 1u << (c - 1), mask = (1u << c) - 1, sentinel = nwin << (c - 1);
    u32 carry = 0;
    for (u32 w = 0; w < nwin; w++) {
        u32 bit = w * c, lo = bit >> 5, sh = bit & 31;
        u64 word = (u64)word_sel(s, lo) | ((u64)word_sel(s, lo + 1) << 32);
        u32 d = ((u32)(word >> sh) & mask) + carry;
        u32 v = i;
        if (d > half) { d = (1u << c) - d; carry = 1; v |= 0x80000000u; }
        else carry = 0;
        keys[(size_t)w * n + i] = d ? (w << (c - 1)) | (d - 1) : sentinel;
        vals[(size_t)w * n + i] = v;
    }
}

// GLV form (points of order r only): s = s1 + s2 lambda with lambda = u^2 - 1 = z^2 - 1 (u = |z|).  From two base-u
// digits and the quotient, s = a1 u^2 + a0 = a1 lambda + (a0 + a1); s1 = (a0 + a1) mod lambda (at most two
// subtractions), s2 = a1 + (number subtracted): both < lambda + 2 < 2^128.  Point i carries s1 and point n + i
// (= phi(P_i) = (beta x, y) = lambda P_i) carries s2; records are window-major over the 2n points.  The scalars
// are 128-bit, so windows 0 .. nwin-2 use signed digits and the top window takes its value plus the incoming carry
// unsigned (no carry out of bit 128): its digits reach 2^tw (tw <= c), i.e. up to 2 half buckets, keyed as key
// windows nwin - 1 and nwin (the reduction adds half to the latter's offsets and the combination folds them).
DI void push_digits_glv(const u32 *sv, u32 idx, u32 c, u32 nwin, size_t stride, u32 *keys, u32 *vals) {
    const u32 half = 1u << (c - 1), mask = (1u << c) - 1, sentinel = (nwin + 1) << (c - 1);
    u32 carry = 0;
    for (u32 w = 0; w < nwin; w++) {
        u32 bit = w * c, lo = bit >> 5, sh = bit & 31;
        u32 w0 = 0, w1 = 0;
#pragma unroll
        for (u32 j = 0; j < 4; j++) {
            w0 = (j == lo) ? sv[j] : w0;
            w1 = (j == lo + 1) ? sv[j] : w1;
        }
        u64 word = (u64)w0 | ((u64)w1 << 32);
        u32 d = ((u32)(word >> sh) & mask) + carry;
        u32 v = idx;
        if (w + 1 < nwin && d > half) { d = (1u << c) - d; carry = 1; v |= 0x80000000u; }
        else carry = 0;
        keys[(size_t)w * stride + idx] = d ? (w << (c - 1)) + (d - 1) : sentinel;
        vals[(size_t)w * stride + idx] = v;
    }
}
extern "C" __global__ void LCB_BOUNDS k_msm_digits_glv(const uint8_t *scalars, u32 n, u32 c, u32 nwin, u32 *keys,
                                                      u32 *vals) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fr s;
    const uint4 *sw = (const uint4 *)(scalars + 32 * (size_t)i);
    uint4 a = sw[0], b = sw[1];
    s.v[0] = a.x; s.v[1] = a.y; s.v[2] = a.z; s.v[3] = a.w;
    s.v[4] = b.x; s.v[5] = b.y; s.v[6] = b.z; s.v[7] = b.w;
    fr_raw_reduce(s);
    u32 q[8];
#pragma unroll
    for (int j = 0; j < 8; j++) q[j] = s.v[j];
    u64 d0, d1;
    u256_divmod_u(q, d0);
    u256_divmod_u(q, d1);                                  // q = a1 < r / u^2 < 2^128
    const u64 u = LCB_Z_ABS;
    u64 m_lo = u * d1, m_hi = __umul64hi(u, d1);
    u64 a0_lo = m_lo + d0, a0_hi = m_hi + (a0_lo < d0 ? 1 : 0);
    u64 a1_lo = (u64)q[0] | ((u64)q[1] << 32), a1_hi = (u64)q[2] | ((u64)q[3] << 32);
    u64 t_lo = a0_lo + a1_lo;
    u64 cy = t_lo < a0_lo ? 1 : 0;
    u64 t_hi = a0_hi + a1_hi + cy;
    u64 t_top = (t_hi < a0_hi || (cy && t_hi == a0_hi)) ? 1 : 0;
    // lambda = u^2 - 1 as a 128-bit value
    const u64 l_lo = u * u - 1, l_hi = __umul64hi(u, u) - ((u * u) == 0 ? 1 : 0);
#pragma unroll
    for (int k = 0; k < 2; k++) {                          // t >= lambda: t -= lambda, a1 += 1
        bool ge = t_top || t_hi > l_hi || (t_hi == l_hi && t_lo >= l_lo);
        u64 nlo = t_lo - l_lo, b0 = t_lo < l_lo ? 1 : 0;
        u64 nhi = t_hi - l_hi - b0;
        u64 ntop = t_top - ((t_hi < l_hi || (t_hi == l_hi && b0)) ? 1 : 0);
        if (ge) {
            t_lo = nlo; t_hi = nhi; t_top = ntop;
            a1_lo += 1;
            if (a1_lo == 0) a1_hi += 1;
        }
    }
    u32 s1[4] = {(u32)t_lo, (u32)(t_lo >> 32), (u32)t_hi, (u32)(t_hi >> 32)};
    u32 s2[4] = {(u32)a1_lo, (u32)(a1_lo >> 32), (u32)a1_hi, (u32)(a1_hi >> 32)};
    push_digits_glv(s1, i, c, nwin, 2 * (size_t)n, keys, vals);
    push_digits_glv(s2, n + i, c, nwin, 2 * (size_t)n, keys, vals);
}
// phi(P) = (beta x, y) for the GLV form ((0, 0), the point at infinity, maps to itself)
extern "C" __global__ void LCB_BOUNDS k_msm_phi(const fp *pts, u32 n, fp *out) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fp beta, x = pts[2 * (size_t)i], y = pts[2 * (size_t)i + 1];
    fp_load_const(beta, LCB_G1_BETA);
    fp_mul(x, x, beta);
    out[2 * (size_t)i] = x;
    out[2 * (size_t)i + 1] = y;
}

extern "C" __global__ void LCB_BOUNDS k_msm_bounds(const u32 *keys, u32 m, u32 sentinel, u32 *start, u32 *end) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    u32 k = keys[i];
    if (k >= sentinel) return;
    if (i == 0 || keys[i - 1] != k) start[k] = i;
    if (i == m - 1 || keys[i + 1] != k) end[k] = i + 1;
}

DI void load_aff(fp &x, fp &y, const fp *pts, u32 idx) {
    const uint4 *p = (const uint4 *)(pts + 2 * (size_t)idx);
    uint4 q[6];
#pragma unroll
    for (int j = 0; j < 6; j++) q[j] = p[j];
    const u32 *w = (const u32 *)q;
#pragma unroll
    for (int j = 0; j < 12; j++) { x.v[j] = w[j]; y.v[j] = w[12 + j]; }
}

// Bucket layout: bucket k = (segment s = k / L, position j = k % L) of the reduction (k_msm_bucket_reduce) is stored at
// j * n_seg + s, so the reduction's lanes (one segment each, all at the same position j per step) read 64 consecutive
// buckets per wave instruction instead of 64 buckets L apart.
DI size_t bidx(u32 k, u32 L, u32 n_seg) { return (size_t)(k % L) * n_seg + k / L; }

// point index v < n_pts reads pts, v >= n_pts reads pts2 (the phi(P) half of the GLV form).  The next record's
// point is loaded while the current addition runs (one gather in flight per lane).
extern "C" __global__ void LCB_BOUNDS k_msm_bucket_acc(const fp *pts, const fp *pts2, u32 n_pts, const u32 *vals,
                                                      const u32 *start, const u32 *end, u32 nb, g1 *buckets, u32 L,
                                                      u32 n_seg) {
    u32 b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    g1 acc;
    jac_set_inf(acc);
    u32 e = start[b], e1 = end[b];
    fp nx, ny;
    u32 nv = 0;
    if (e < e1) {
        nv = vals[e];
        u32 idx = nv & 0x7fffffffu;
        load_aff(nx, ny, idx < n_pts ? pts : pts2, idx < n_pts ? idx : idx - n_pts);
    }
    for (; e < e1; e++) {
        fp x = nx, y = ny;
        u32 v = nv;
        if (e + 1 < e1) {
            nv = vals[e + 1];
            u32 idx = nv & 0x7fffffffu;
            load_aff(nx, ny, idx < n_pts ? pts : pts2, idx < n_pts ? idx : idx - n_pts);
        }
        if (fp_is_zero(x) && fp_is_zero(y)) continue;  // point at infinity
        if (v >> 31) fp_neg(y, y);
        jac_add_aff(acc, acc, x, y);
    }
    buckets[bidx(b, L, n_seg)] = acc;
}

#define MSM_ADD(r, p, q) grp_add(r, p, q)
#define MSM_DBL(r, p) grp_dbl(r, p)
// Record-balanced form of k_msm_bucket_acc: lane j adds exactly the K sorted records [jK, (j + 1)K) (the digit
// distribution is uneven — Poisson bucket sizes, and a short top window piles its records into few buckets — so one
// lane per bucket waits for the wave's largest bucket).  A bucket wholly inside the chunk is written to buckets[k]
// directly; the chunk's first bucket when it started in an earlier chunk goes to headp[j], its last bucket when it
// continues into a later chunk to tailp[j] (both always written, infinity when unused), and k_msm_bucket_fix adds the
// pieces of the buckets that span chunks.  The sentinel records (digit 0) sort last and end a chunk.
DI void msm_flush(const g1 &acc, u32 k, u32 e0, u32 e1, const u32 *start, const u32 *end, g1 *buckets, g1 *head,
                  g1 *tail, u32 L, u32 n_seg) {
    const u32 s = start[k], en = end[k];
    if (s >= e0 && en <= e1) buckets[bidx(k, L, n_seg)] = acc;
    else if (s < e0) *head = acc;
    else *tail = acc;
}
extern "C" __global__ void LCB_BOUNDS k_msm_chunk_acc(const fp *pts, const fp *pts2, u32 n_pts, const u32 *keys,
                                                     const u32 *vals, u32 m, u32 K, u32 sentinel, const u32 *start,
                                                     const u32 *end, g1 *buckets, g1 *headp, g1 *tailp, u32 L,
                                                     u32 n_seg) {
    const u32 j = blockIdx.x * blockDim.x + threadIdx.x;
    const size_t e0s = (size_t)j * K;
    if (e0s >= m) return;
    const u32 e0 = (u32)e0s, e1 = (u32)min((size_t)m, e0s + K);
    g1 acc, inf;
    jac_set_inf(inf);
    headp[j] = inf;
    tailp[j] = inf;
    acc = inf;
    u32 cur = keys[e0];
    if (cur >= sentinel) return;
    fp nx, ny;
    u32 nv = vals[e0];
    {
        const u32 idx = nv & 0x7fffffffu;
        load_aff(nx, ny, idx < n_pts ? pts : pts2, idx < n_pts ? idx : idx - n_pts);
    }
#pragma unroll 1
    for (u32 e = e0; e < e1; e++) {
        const u32 k = keys[e];
        if (k >= sentinel) break;
        fp x = nx, y = ny;
        const u32 v = nv;
        if (e + 1 < e1) {                                   // the next record's point, loaded during this addition
            nv = vals[e + 1];
            const u32 idx = nv & 0x7fffffffu;
            load_aff(nx, ny, idx < n_pts ? pts : pts2, idx < n_pts ? idx : idx - n_pts);
        }
        if (k != cur) {
            msm_flush(acc, cur, e0, e1, start, end, buckets, headp + j, tailp + j, L, n_seg);
            acc = inf;
            cur = k;
        }
        if (fp_is_zero(x) && fp_is_zero(y)) continue;      // point at infinity
        if (v >> 31) fp_neg(y, y);
        jac_add_aff(acc, acc, x, y);
    }
    msm_flush(acc, cur, e0, e1, start, end, buckets, headp + j, tailp + j, L, n_seg);
}
// buckets spanning chunks: tail of the first chunk + heads of the later ones; empty buckets: infinity
extern "C" __global__ void LCB_BOUNDS k_msm_bucket_fix(const u32 *start, const u32 *end, u32 K, const g1 *headp,
                                                      const g1 *tailp, u32 nb, g1 *buckets, u32 L, u32 n_seg) {
    const u32 k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nb) return;
    const u32 s = start[k], en = end[k];
    if (s == en) {
        g1 inf;
        jac_set_inf(inf);
        buckets[bidx(k, L, n_seg)] = inf;
        return;
    }
    const u32 j0 = s / K, j1 = (en - 1) / K;
    if (j0 == j1) return;
    g1 acc = tailp[j0];
#pragma unroll 1
    for (u32 j = j0 + 1; j <= j1; j++) MSM_ADD(acc, acc, headp[j]);
    buckets[bidx(k, L, n_seg)] = acc;
}

// The reduction / combination kernels are latency chains (one lane's serial additions and doublings); their group
// operations are the call forms (inlining them measured mixed: 2^20 bucket reduce 1.21 vs 1.06 ms, combine 2.17 vs
// 1.98 ms; 2^24 combine 3.26 vs 3.59 ms).
#ifndef MSM_ADD
#define MSM_ADD(r, p, q) grp_add(r, p, q)
#define MSM_DBL(r, p) grp_dbl(r, p)
#endif
// segment q of window w covers buckets a = q*L .. a+L-1 (digit values a+1 .. a+L)
// hi_win: the key window that holds the upper half of the GLV top window's digits (digit = half + a + j + 1), or
// ~0u when there is none
extern "C" __global__ void LCB_BOUNDS k_msm_bucket_reduce(const g1 *buckets, u32 half, u32 L, u32 n_seg, u32 hi_win,
                                                         g1 *seg_out) {
    u32 s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_seg) return;
    u32 per_win = half / L, w = s / per_win, a = (s % per_win) * L;
    const g1 *B = buckets + s;                      // position j of segment s at j * n_seg + s (bidx)
    if (w == hi_win) a += half;
    g1 run, acc;
    jac_set_inf(run);
    jac_set_inf(acc);
    g1 nb = B[(size_t)(L - 1) * n_seg];
#pragma unroll 1
    for (u32 j = L; j-- > 0;) {
        const g1 cb = nb;
        if (j) nb = B[(size_t)(j - 1) * n_seg];      // the next bucket, loaded during these additions
        MSM_ADD(run, run, cb);
        MSM_ADD(acc, acc, run);
    }
    if (a) {
        g1 t;
        jac_mul_u64(t, run, a);
        MSM_ADD(acc, acc, t);
    }
    seg_out[s] = acc;
}

extern "C" __global__ void LCB_BOUNDS k_g1_jac_reduce_groups(const g1 *in, u32 n_in, u32 group, g1 *out) {
    u32 j = blockIdx.x * blockDim.x + threadIdx.x;
    u32 n_out = (n_in + group - 1) / group;
    if (j >= n_out) return;
    g1 acc;
    jac_set_inf(acc);
    u32 e = min(n_in, (j + 1) * group);
    for (u32 i = j * group; i < e; i++) MSM_ADD(acc, acc, in[i]);
    out[j] = acc;
}

// out[b] = sum of in[b*group .. (b+1)*group) (clipped to n_in): lanes add strided inputs, then a log2(256)-deep
// tree in LDS, so the dependent chain is group/256 + 8 additions instead of group
extern "C" __global__ void LCB_BOUNDS k_g1_jac_reduce_block(const g1 *in, u32 n_in, u32 group, g1 *out) {
    __shared__ g1 sh[LCB_BLOCK];
    u32 t = threadIdx.x, b = blockIdx.x;
    size_t lo = (size_t)b * group, hi = min((size_t)n_in, lo + group);
    g1 acc;
    jac_set_inf(acc);
    for (size_t i = lo + t; i < hi; i += LCB_BLOCK) MSM_ADD(acc, acc, in[i]);
    sh[t] = acc;
    __syncthreads();
    for (u32 s = LCB_BLOCK / 2; s > 0; s >>= 1) {
        if (t < s) {
            g1 x = sh[t], y = sh[t + s];
            MSM_ADD(x, x, y);
            sh[t] = x;
        }
        __syncthreads();
    }
    if (t == 0) out[b] = sh[0];
}

// the same sums with the tree's additions on groups of four lanes (coop_pt.hpp: 5 product latencies per addition
// instead of 16; 64 groups per block, the first level in two passes) — the same pairs in the same order, so the same
// Jacobian coordinates as k_g1_jac_reduce_block
extern "C" __global__ void LCB_BOUNDS k_g1_jac_reduce_block_coop(const g1 *in, u32 n_in, u32 group, g1 *out) {
    __shared__ g1 sh[LCB_BLOCK];
    __shared__ PtProd<fp> lds[LCB_BLOCK / PT_LANES];
    const u32 t = threadIdx.x, b = blockIdx.x, gi = t / PT_LANES;
    size_t lo = (size_t)b * group, hi = min((size_t)n_in, lo + group);
    g1 acc;
    jac_set_inf(acc);
    for (size_t i = lo + t; i < hi; i += LCB_BLOCK) MSM_ADD(acc, acc, in[i]);
    sh[t] = acc;
    __syncthreads();
#pragma unroll 1
    for (u32 s = LCB_BLOCK / 2; s > 0; s >>= 1) {
#pragma unroll 1
        for (u32 base = 0; base < s; base += LCB_BLOCK / PT_LANES) {
            const u32 p = base + gi;
            const bool live = p < s;
            g1 x, y;
            if (live) { x = sh[p]; y = sh[p + s]; }
            else { jac_set_inf(x); jac_set_inf(y); }
            pt_add<true>(lds + gi, x, x, y);              // every lane of the block: the rounds' barriers
            if (live && pt_role() == 0) sh[p] = x;          // pt_add's last round ended with a barrier after the reads
            __syncthreads();
        }
    }
    if (t == 0) out[b] = sh[0];
}

// fold_top: win[nwin] has the same weight as win[nwin - 1] (the GLV top window's upper digit half)
extern "C" __global__ void LCB_BOUNDS k_msm_horner(const g1 *win, u32 nwin, u32 c, u32 fold_top, g1 *out) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    g1 acc = win[nwin - 1];
    if (fold_top) MSM_ADD(acc, acc, win[nwin]);
    for (u32 w = nwin - 1; w-- > 0;) {
#pragma unroll 1
        for (u32 t = 0; t < c; t++) MSM_DBL(acc, acc);
        MSM_ADD(acc, acc, win[w]);
    }
    out[0] = acc;
}

// the same combination on one group of four lanes (coop_pt.hpp: a doubling in 3 product latencies instead of 7, an
// addition in 5 instead of 16) — the serial tail of every MSM
extern "C" __global__ void __launch_bounds__(64, 1) k_msm_horner_coop(const g1 *win, u32 nwin, u32 c, u32 fold_top,
                                                                     g1 *out) {
    __shared__ PtLds<fp> lds;
    g1 acc = win[nwin - 1];
    if (fold_top) { g1 t = win[nwin]; pt_add(&lds, acc, acc, t); }
#pragma unroll 1
    for (u32 w = nwin - 1; w-- > 0;) {
#pragma unroll 1
        for (u32 t = 0; t < c; t++) pt_dbl(&lds, acc, acc);
        g1 t = win[w];
        pt_add(&lds, acc, acc, t);
    }
    if (threadIdx.x == 0) out[0] = acc;
}

extern "C" __global__ void LCB_BOUNDS k_g1_jac_compress(const g1 *in, u32 n, uint8_t *out) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    g1_compress_jac(out + 48 * (size_t)i, in[i]);
}

// 48-byte serialized G1 -> 96-byte affine Montgomery (MSM input layout); ok[i] = 0 on a malformed encoding
extern "C" __global__ void LCB_BOUNDS k_g1_to_affine(const uint8_t *in, u32 n, fp *out, uint8_t *ok) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    g1a A;
    bool good = g1_decompress(A, in + 48 * (size_t)i);
    if (!good || A.inf) { A.x = fp_zero(); A.y = fp_zero(); }
    out[2 * (size_t)i] = A.x;
    out[2 * (size_t)i + 1] = A.y;
    if (ok) ok[i] = good;
}

// ---------------------------------------------------------------- host launch wrappers
extern "C" void lcbk_msm_digits(dim3 grid, hipStream_t s, const uint8_t *scalars, u32 n, u32 c, u32 nwin, u32 *keys, u32 *vals) {
    LCB_LAUNCH(k_msm_digits, scalars, n, c, nwin, keys, vals);
}
extern "C" void lcbk_msm_bounds(dim3 grid, hipStream_t s, const u32 *keys, u32 m, u32 sentinel, u32 *start, u32 *end) {
    LCB_LAUNCH(k_msm_bounds, keys, m, sentinel, start, end);
}
extern "C" void lcbk_msm_bucket_acc(dim3 grid, hipStream_t s, const void *pts, const void *pts2, u32 n_pts, const u32 *vals, const u32 *start, const u32 *end, u32 nb, void *buckets, u32 L, u32 n_seg) {
    LCB_LAUNCH(k_msm_bucket_acc, (const fp *)pts, (const fp *)pts2, n_pts, vals, start, end, nb, (g1 *)buckets, L, n_seg);
}
extern "C" void lcbk_msm_chunk_acc(hipStream_t s, const void *pts, const void *pts2, u32 n_pts, const u32 *keys, const u32 *vals, u32 m, u32 K, u32 sentinel, const u32 *start, const u32 *end, void *buckets, void *headp, void *tailp, u32 L, u32 n_seg) {
    const u32 n_chunks = (u32)(((size_t)m + K - 1) / K);
    dim3 grid((n_chunks + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_msm_chunk_acc, (const fp *)pts, (const fp *)pts2, n_pts, keys, vals, m, K, sentinel, start, end, (g1 *)buckets, (g1 *)headp, (g1 *)tailp, L, n_seg);
}
extern "C" void lcbk_msm_bucket_fix(hipStream_t s, const u32 *start, const u32 *end, u32 K, const void *headp, const void *tailp, u32 nb, void *buckets, u32 L, u32 n_seg) {
    dim3 grid((nb + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_msm_bucket_fix, start, end, K, (const g1 *)headp, (const g1 *)tailp, nb, (g1 *)buckets, L, n_seg);
}
extern "C" void lcbk_msm_digits_glv(dim3 grid, hipStream_t s, const uint8_t *scalars, u32 n, u32 c, u32 nwin, u32 *keys, u32 *vals) {
    LCB_LAUNCH(k_msm_digits_glv, scalars, n, c, nwin, keys, vals);
}
extern "C" void lcbk_msm_phi(dim3 grid, hipStream_t s, const void *pts, u32 n, void *out) {
    LCB_LAUNCH(k_msm_phi, (const fp *)pts, n, (fp *)out);
}
extern "C" void lcbk_msm_bucket_reduce(dim3 grid, hipStream_t s, const void *buckets, u32 half, u32 L, u32 n_seg, u32 hi_win, void *seg_out) {
    LCB_LAUNCH(k_msm_bucket_reduce, (const g1 *)buckets, half, L, n_seg, hi_win, (g1 *)seg_out);
}
extern "C" void lcbk_g1_jac_reduce_groups(dim3 grid, hipStream_t s, const void *in, u32 n_in, u32 group, void *out) {
    LCB_LAUNCH(k_g1_jac_reduce_groups, (const g1 *)in, n_in, group, (g1 *)out);
}
#ifndef LCB_TREE_COOP
#define LCB_TREE_COOP 1
#endif
extern "C" void lcbk_g1_jac_reduce_block(hipStream_t s, const void *in, u32 n_in, u32 group, void *out) {
    dim3 grid((n_in + group - 1) / group);
#if LCB_TREE_COOP
    LCB_LAUNCH(k_g1_jac_reduce_block_coop, (const g1 *)in, n_in, group, (g1 *)out);
#else
    LCB_LAUNCH(k_g1_jac_reduce_block, (const g1 *)in, n_in, group, (g1 *)out);
#endif
}
extern "C" void lcbk_msm_horner(hipStream_t s, const void *win, u32 nwin, u32 c, u32 fold_top, void *out) {
    LCB_LAUNCH_GATED(k_msm_horner_coop, dim3(1), dim3(PT_LANES), 0, s, (const g1 *)win, nwin, c, fold_top, (g1 *)out);
}
extern "C" void lcbk_g1_jac_compress(dim3 grid, hipStream_t s, const void *in, u32 n, uint8_t *out) {
    LCB_LAUNCH(k_g1_jac_compress, (const g1 *)in, n, out);
}
extern "C" void lcbk_g1_to_affine(dim3 grid, hipStream_t s, const uint8_t *in, u32 n, void *out, uint8_t *ok) {
    LCB_LAUNCH(k_g1_to_affine, in, n, (fp *)out, ok);
}
// stable radix sort of (key, value) pairs on key bits [0, end_bit); temp == nullptr queries *temp_bytes.
// Returns 1 when the sorted data ended in the alternate buffers (keys_alt / vals_alt).
extern "C" int lcbk_sort_pairs(void *temp, size_t *temp_bytes, u32 *keys, u32 *keys_alt, u32 *vals, u32 *vals_alt,
                               u32 m, int end_bit, hipStream_t s) {
    hipcub::DoubleBuffer<u32> dk(keys, keys_alt), dv(vals, vals_alt);
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(temp, *temp_bytes, dk, dv, (int)m, 0, end_bit, s);
    if (e != hipSuccess) return -1;
    return dk.Current() == keys_alt ? 1 : 0;
}
