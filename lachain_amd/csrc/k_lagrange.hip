// lachain_amd/csrc/k_lagrange.hip — gfx950 kernels: Lagrange interpolation at 0 and MSM.
#include "kcommon.hpp"

LCB_ASM_LIBRARY(k_lagrange)
LCB_TU_CONFIG(k_lagrange)

// ================================================================================= Lagrange at 0
// lambda_i = prod_{j != i} x_j / (x_j - x_i) (mcl: a = prod x_j, b_i = x_i prod_{j!=i}(x_j - x_i),
// lambda_i = a / b_i); one lane per problem; writes canonical raw lambdas and a status byte.
extern "C" __global__ void LCB_BOUNDS k_lagrange_coeffs(const uint8_t *xs, const u32 *off, u32 n_problems,
                                                       fr *lam_raw, uint8_t *status) {
    u32 j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_problems) return;
    u32 o0 = off[j], k = off[j + 1] - o0;
    bool ok = k > 0;
    // a = prod x
    fr a = fr_one();
    for (u32 i = 0; i < k && ok; i++) {
        fr xr, x;
        const u32 *w = (const u32 *)(xs + 32 * (size_t)(o0 + i));
        for (int q = 0; q < 8; q++) xr.v[q] = w[q];
        if (!fr_raw_lt_r(xr) || fr_is_zero(xr)) { ok = false; break; }
        fr_from_raw(x, xr);
        fr_mul(a, a, x);
    }
    // b_i and prefix products for one batch inversion (stored in lam_raw as scratch)
    fr acc = fr_one();
    for (u32 i = 0; i < k && ok; i++) {
        fr xi_r, xi;
        const u32 *w = (const u32 *)(xs + 32 * (size_t)(o0 + i));
        for (int q = 0; q < 8; q++) xi_r.v[q] = w[q];
        fr_from_raw(xi, xi_r);
        fr b = xi;
        for (u32 t = 0; t < k; t++) {
            if (t == i) continue;
            fr xt_r, xt, d;
            const u32 *wt = (const u32 *)(xs + 32 * (size_t)(o0 + t));
            for (int q = 0; q < 8; q++) xt_r.v[q] = wt[q];
            fr_from_raw(xt, xt_r);
            fr_sub(d, xt, xi);
            if (fr_is_zero(d)) { ok = false; break; }
            fr_mul(b, b, d);
        }
        if (!ok) break;
        lam_raw[o0 + i] = b;      // b_i (Montgomery) for now
    }
    if (ok) {
        // batch inversion of b_i: prefix products, one inversion, back-substitution
        for (u32 i = 0; i < k; i++) {
            fr b = lam_raw[o0 + i];
            fr_mul(acc, acc, b);
        }
        fr inv;
        fr_inv(inv, acc);
        for (u32 i = k; i-- > 0;) {
            // inv = 1/(b_0..b_i); prefix up to i-1 recomputed (k is small: O(k^2) Fr muls overall)
            fr pre = fr_one();
            for (u32 t = 0; t < i; t++) fr_mul(pre, pre, lam_raw[o0 + t]);
            fr bi_inv, l, lr;
            fr_mul(bi_inv, inv, pre);
            fr_mul(inv, inv, lam_raw[o0 + i]);
            fr_mul(l, a, bi_inv);
            fr_to_raw(lr, l);
            lam_raw[o0 + i] = lr;
        }
    }
    status[j] = ok;
}
// Inlined ladders for the lanes below (no call frames: the DN group operations pass the accumulator through scratch
// at every step).  LCB_LAG_CALLS restores the call form.
template <class F> DI void jac_mul_aff_inl(jac<F> &r, const aff<F> &p, const u32 *k, int nbits) {
    jac_set_inf(r);
    if (p.inf) return;
#pragma unroll 1
    for (int i = nbits - 1; i >= 0; i--) {
        jac_dbl(r, r);
        if ((k[i >> 5] >> (i & 31)) & 1) jac_add_aff(r, r, p.x, p.y);
    }
}
// g2_mul_gls (curve.hpp) with the loop inlined
DI void g2_mul_gls_inl(g2 &r, const g2a &A, const u32 k[8]) {
    jac_set_inf(r);
    if (A.inf) return;
    u32 q[8];
#pragma unroll
    for (int j = 0; j < 8; j++) q[j] = k[j];
    u64 d[4];
    u256_divmod_u(q, d[0]);
    u256_divmod_u(q, d[1]);
    u256_divmod_u(q, d[2]);
    d[3] = (u64)q[0] | ((u64)q[1] << 32);
    g2 P, T;
    jac_from_aff(P, A);
    g2a Q[4];
    Q[0] = A;
    g2_psi(T, P);
    Q[1].x = T.x; fp2_neg(Q[1].y, T.y); Q[1].inf = false;
    g2_psi2(T, P);
    Q[2].x = T.x; Q[2].y = T.y; Q[2].inf = false;
    g2_psi(T, T);
    Q[3].x = T.x; fp2_neg(Q[3].y, T.y); Q[3].inf = false;
#pragma unroll 1
    for (int b = 63; b >= 0; b--) {
        jac_dbl(r, r);
#pragma unroll 1
        for (int i = 0; i < 4; i++)
            if ((d[i] >> b) & 1) jac_add_aff(r, r, Q[i].x, Q[i].y);
    }
}
// GLS in G2 with one addition per digit column: the 15 non-empty sums of Q = {A, -psi A, psi^2 A, -psi^3 A} (index
// bit i <-> Q_i) in an affine table — Q_2, Q_3 = psi^2(Q_0, Q_1), so 1 + 9 additions and one batched inversion —
// then 64 doublings and 64 mixed additions instead of 64 doublings and 256 additions per wave.  For A in G2 no entry
// is infinity (|i0 - i1 z + i2 z^2 - i3 z^3| < r); the plain GLS loop stays as a guard.
DI void g2_mul_gls_tab(g2 &r, const g2a &A, const u32 k[8]) {
    jac_set_inf(r);
    if (A.inf) return;
    u32 q[8];
#pragma unroll
    for (int j = 0; j < 8; j++) q[j] = k[j];
    u64 d[4];
    u256_divmod_u(q, d[0]);
    u256_divmod_u(q, d[1]);
    u256_divmod_u(q, d[2]);
    d[3] = (u64)q[0] | ((u64)q[1] << 32);
    g2 t[16];
    jac_from_aff(t[1], A);
    g2_psi(t[2], t[1]);
    fp2_neg(t[2].y, t[2].y);                         // -psi(A), z = 1
    jac_add_aff(t[3], t[1], t[2].x, t[2].y);
#pragma unroll 1
    for (int j = 1; j < 4; j++) g2_psi2(t[4 * j], t[j]);
#pragma unroll 1
    for (int j = 4; j < 16; j += 4)
#pragma unroll 1
        for (int i = 1; i < 4; i++) jac_add(t[j + i], t[i], t[j]);
    g2a ta[16];
    if (!jac_table_to_aff(ta, t)) { g2_mul_gls_inl(r, A, k); return; }
#pragma unroll 1
    for (int b = 63; b >= 0; b--) {
        jac_dbl(r, r);
        u32 idx = (u32)((d[0] >> b) & 1) | (u32)((d[1] >> b) & 1) << 1 | (u32)((d[2] >> b) & 1) << 2 |
                  (u32)((d[3] >> b) & 1) << 3;
        if (idx) jac_add_aff(r, r, ta[idx].x, ta[idx].y);
    }
}
// GLS digits of k (< r): k = d0 + d1 u + d2 u^2 + d3 u^3, u = |z| (curve.hpp u256_divmod_u)
DI void g2_gls_digits(u64 d[4], const u32 k[8]) {
    u32 q[8];
#pragma unroll
    for (int j = 0; j < 8; j++) q[j] = k[j];
    u256_divmod_u(q, d[0]);
    u256_divmod_u(q, d[1]);
    u256_divmod_u(q, d[2]);
    d[3] = (u64)q[0] | ((u64)q[1] << 32);
}
// g2_mul_gls_tab's 15 sums of {A, -psi A, psi^2 A, -psi^3 A} (index bit i <-> Q_i) into t[1..15], Jacobian
DI void g2_gls_sums(g2 *t, const g2a &A) {
    jac_from_aff(t[1], A);
    g2_psi(t[2], t[1]);
    fp2_neg(t[2].y, t[2].y);
    jac_add_aff(t[3], t[1], t[2].x, t[2].y);
#pragma unroll 1
    for (int j = 1; j < 4; j++) g2_psi2(t[4 * j], t[j]);
#pragma unroll 1
    for (int j = 4; j < 16; j += 4)
#pragma unroll 1
        for (int i = 1; i < 4; i++) jac_add(t[j + i], t[i], t[j]);
}
// lambda_a A + lambda_b B for two points of G2 with one shared run of 64 doublings (Straus) and one batched inversion
// for both tables (entries 1..15: A's sums, 16..30: B's); false when a table entry is infinity (never in G2, as for
// g2_mul_gls_tab) — the caller then multiplies the points one by one
DI bool g2_mul2_gls_tab(g2 &r, const g2a &A, const u32 ka[8], const g2a &B, const u32 kb[8]) {
    u64 da[4], db[4];
    g2_gls_digits(da, ka);
    g2_gls_digits(db, kb);
    g2 t[31];
    g2_gls_sums(t, A);
    g2_gls_sums(t + 15, B);
    g2a ta[31];
    if (!jac_table_to_aff(ta, t)) return false;
    jac_set_inf(r);
#pragma unroll 1
    for (int b = 63; b >= 0; b--) {
        jac_dbl(r, r);
        u32 ia = (u32)((da[0] >> b) & 1) | (u32)((da[1] >> b) & 1) << 1 | (u32)((da[2] >> b) & 1) << 2 |
                 (u32)((da[3] >> b) & 1) << 3;
        u32 ib = (u32)((db[0] >> b) & 1) | (u32)((db[1] >> b) & 1) << 1 | (u32)((db[2] >> b) & 1) << 2 |
                 (u32)((db[3] >> b) & 1) << 3;
        if (ia) jac_add_aff(r, r, ta[ia].x, ta[ia].y);
        if (ib) jac_add_aff(r, r, ta[15 + ib].x, ta[15 + ib].y);
    }
    return true;
}
// a G2 entry's point: the ts_share_st record when it holds exactly the entry's bytes, else decoded and psi-tested here
DI void g2_entry_point(g2a &A, bool &ok, bool &in_g2, const uint8_t *y, const ts_share_st *dec, u32 n_dec, u32 si) {
    bool hit = false;
    if (dec && si < n_dec && dec[si].p.ok) {
        const uint4 *r = (const uint4 *)dec[si].raw, *w = (const uint4 *)y;
        hit = true;
#pragma unroll
        for (int q = 0; q < 6; q++) {
            const uint4 a = r[q], b = w[q];
            hit = hit && a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w;
        }
    }
    if (hit) {
        const g2a_st e = dec[si].p;
        st_to_g2a(A, e);
        ok = true;
        in_g2 = e.pad[0] != 0;
    } else {
        ok = g2_decompress(A, y);
        in_g2 = g2_in_subgroup_inl(A);
    }
}

// partial products lambda_i * Y_i for every entry (one lane per entry)
extern "C" __global__ void LCB_BOUNDS k_g1_mul_lanes(const uint8_t *ys, const fr *lam_raw, u32 n_entries, g1 *out,
                                                    uint8_t *ok_out) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_entries) return;
    g1a A;
    bool ok = g1_decompress(A, ys + 48 * (size_t)i);
    // plain double-and-add on the canonical integer lambda: exact for every on-curve input, including points
    // outside the r-torsion that G1.FromBytes accepts (GLV would be wrong for their cofactor component)
    g1 R;
    fr k = lam_raw[i];
    jac_mul_win4(R, A, k.v);      // 4-bit window, affine table (measured faster than the plain ladder)
    out[i] = R;
    ok_out[i] = ok;
}
// dec / src (nullable): the decoded shares of the context's last batched CommonCoin check (ts_share_st) and each
// entry's index among them; an entry whose record holds exactly its input bytes takes the record's point and G2 flag
extern "C" __global__ void LCB_BOUNDS k_g2_mul_lanes(const uint8_t *ys, const fr *lam_raw, u32 n_entries, g2 *out,
                                                    uint8_t *ok_out, const ts_share_st *dec, u32 n_dec,
                                                    const u32 *src) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_entries) return;
    g2a A;
    bool ok, in_g2;
    g2_entry_point(A, ok, in_g2, ys + 96 * (size_t)i, dec, n_dec, src ? src[i] : 0xffffffffu);
    // GLS (64 shared doublings) only for points proven to lie in G2 (psi(P) == [z]P, 64 doublings); any other
    // on-curve input takes the plain ladder, so the result equals the oracle's for every input
    g2 R;
    fr k = lam_raw[i];
    if (in_g2) g2_mul_gls_tab(R, A, k.v);
    else jac_mul_aff_inl(R, A, k.v, 256);
    out[i] = R;
    ok_out[i] = ok;
}
// two entries per lane (entries 2p, 2p + 1 of one problem: the caller guarantees even problem offsets): both in G2 ->
// lambda_a A + lambda_b B by g2_mul2_gls_tab into out[2p] (out[2p + 1] = infinity), else each on its own as
// k_g2_mul_lanes does; the problem sums (k_g2_sum) are the same points
extern "C" __global__ void LCB_BOUNDS k_g2_mul2_lanes(const uint8_t *ys, const fr *lam_raw, u32 n_pairs, g2 *out,
                                                     uint8_t *ok_out, const ts_share_st *dec, u32 n_dec,
                                                     const u32 *src) {
    u32 p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_pairs) return;
    const u32 i0 = 2 * p, i1 = 2 * p + 1;
    g2a A, B;
    bool oka, okb, ga, gb;
    g2_entry_point(A, oka, ga, ys + 96 * (size_t)i0, dec, n_dec, src ? src[i0] : 0xffffffffu);
    g2_entry_point(B, okb, gb, ys + 96 * (size_t)i1, dec, n_dec, src ? src[i1] : 0xffffffffu);
    fr ka = lam_raw[i0], kb = lam_raw[i1];
    g2 R0, R1;
    jac_set_inf(R1);
    if (!(ga && gb && !A.inf && !B.inf && g2_mul2_gls_tab(R0, A, ka.v, B, kb.v))) {
        // inline (measured 199 ms per 65,536-round assembly vs 205 ms with one shared call, despite more spills)
        if (ga) g2_mul_gls_tab(R0, A, ka.v);
        else jac_mul_aff_inl(R0, A, ka.v, 256);
        if (gb) g2_mul_gls_tab(R1, B, kb.v);
        else jac_mul_aff_inl(R1, B, kb.v, 256);
    }
    out[i0] = R0;
    out[i1] = R1;
    ok_out[i0] = oka;
    ok_out[i1] = okb;
}
extern "C" __global__ void LCB_BOUNDS k_g1_sum(const g1 *parts, const uint8_t *ok_in, const u32 *off, u32 n_problems,
                                              uint8_t *status, uint8_t *out) {
    u32 j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_problems) return;
    g1 acc;
    jac_set_inf(acc);
    bool ok = status[j];
    for (u32 i = off[j]; i < off[j + 1]; i++) {
        ok = ok && ok_in[i];
        jac_add(acc, acc, parts[i]);
    }
    if (!ok) jac_set_inf(acc);
    g1_compress_jac(out + 48 * (size_t)j, acc);
    status[j] = ok;
}
extern "C" __global__ void LCB_BOUNDS k_g2_sum(const g2 *parts, const uint8_t *ok_in, const u32 *off, u32 n_problems,
                                              uint8_t *status, uint8_t *out) {
    u32 j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_problems) return;
    g2 acc;
    jac_set_inf(acc);
    bool ok = status[j];
    for (u32 i = off[j]; i < off[j + 1]; i++) {
        ok = ok && ok_in[i];
        jac_add(acc, acc, parts[i]);
    }
    if (!ok) jac_set_inf(acc);
    g2_compress_jac(out + 96 * (size_t)j, acc);
    status[j] = ok;
}

// ---------------------------------------------------------------- host launch wrappers
extern "C" void lcbk_lagrange_coeffs(dim3 grid, hipStream_t s, const uint8_t *xs, const u32 *off, u32 n_problems, void *lam_raw, uint8_t *status) {
    LCB_LAUNCH(k_lagrange_coeffs, xs, off, n_problems, (fr *)lam_raw, status);
}
extern "C" void lcbk_g1_mul_lanes(dim3 grid, hipStream_t s, const uint8_t *ys, const void *lam_raw, u32 n_entries, void *out, uint8_t *ok_out) {
    LCB_LAUNCH(k_g1_mul_lanes, ys, (const fr *)lam_raw, n_entries, (g1 *)out, ok_out);
}
extern "C" void lcbk_g2_mul_lanes(dim3 grid, hipStream_t s, const uint8_t *ys, const void *lam_raw, u32 n_entries, void *out, uint8_t *ok_out, const void *dec, u32 n_dec, const u32 *src) {
    LCB_LAUNCH(k_g2_mul_lanes, ys, (const fr *)lam_raw, n_entries, (g2 *)out, ok_out, (const ts_share_st *)dec, n_dec, src);
}
extern "C" void lcbk_g2_mul2_lanes(hipStream_t s, const uint8_t *ys, const void *lam_raw, u32 n_entries, void *out, uint8_t *ok_out, const void *dec, u32 n_dec, const u32 *src) {
    const u32 n_pairs = n_entries / 2;
    dim3 grid((n_pairs + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_g2_mul2_lanes, ys, (const fr *)lam_raw, n_pairs, (g2 *)out, ok_out, (const ts_share_st *)dec, n_dec, src);
}
extern "C" void lcbk_g1_sum(dim3 grid, hipStream_t s, const void *parts, const uint8_t *ok_in, const u32 *off, u32 n_problems, uint8_t *status, uint8_t *out) {
    LCB_LAUNCH(k_g1_sum, (const g1 *)parts, ok_in, off, n_problems, status, out);
}
extern "C" void lcbk_g2_sum(dim3 grid, hipStream_t s, const void *parts, const uint8_t *ok_in, const u32 *off, u32 n_problems, uint8_t *status, uint8_t *out) {
    LCB_LAUNCH(k_g2_sum, (const g2 *)parts, ok_in, off, n_problems, status, out);
}
