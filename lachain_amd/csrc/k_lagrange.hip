// lachain_amd/csrc/k_lagrange.hip — gfx950 kernels: Lagrange interpolation at 0 and MSM.
#include "kcommon.hpp"
#include "lanetab.hpp"

LCB_ASM_LIBRARY(k_lagrange)
LCB_TU_CONFIG(k_lagrange)

// ================================================================================= Lagrange at 0
// lambda_i = prod_{j != i} x_j / (x_j - x_i) (mcl: a = prod x_j, b_i = x_i prod_{j!=i}(x_j - x_i),
// lambda_i = a / b_i); one lane per problem; writes canonical raw lambdas and a status byte.  Every x is used as its
// raw integer read as a Montgomery representation (the value x R^-1): a and every b_i are products of k such factors,
// so both carry R^-k and lambda_i = a / b_i is exact without converting any x (round 5: the conversions were one
// product per (i, j) pair).  The batch inversion keeps its prefix products in pre (one slot per entry).
extern "C" __global__ void LCB_BOUNDS k_lagrange_coeffs(const uint8_t *xs, const u32 *off, u32 n_problems,
                                                       fr *lam_raw, fr *pre, uint8_t *status) {
    u32 j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_problems) return;
    u32 o0 = off[j], k = off[j + 1] - o0;
    bool ok = k > 0;
    // a = prod x
    fr a = fr_one();
    for (u32 i = 0; i < k && ok; i++) {
        fr xr;
        const u32 *w = (const u32 *)(xs + 32 * (size_t)(o0 + i));
        for (int q = 0; q < 8; q++) xr.v[q] = w[q];
        if (!fr_raw_lt_r(xr) || fr_is_zero(xr)) { ok = false; break; }
        fr_mul(a, a, xr);
    }
    // b_i, and the prefix products b_0 .. b_(i-1) for one batch inversion
    fr acc = fr_one();
    for (u32 i = 0; i < k && ok; i++) {
        fr xi;
        const u32 *w = (const u32 *)(xs + 32 * (size_t)(o0 + i));
        for (int q = 0; q < 8; q++) xi.v[q] = w[q];
        fr b = xi;
        for (u32 t = 0; t < k; t++) {
            if (t == i) continue;
            fr xt, d;
            const u32 *wt = (const u32 *)(xs + 32 * (size_t)(o0 + t));
            for (int q = 0; q < 8; q++) xt.v[q] = wt[q];
            fr_sub(d, xt, xi);
            if (fr_is_zero(d)) { ok = false; break; }
            fr_mul(b, b, d);
        }
        if (!ok) break;
        lam_raw[o0 + i] = b;      // b_i for now
        pre[o0 + i] = acc;        // b_0 .. b_(i-1)
        fr_mul(acc, acc, b);
    }
    if (ok) {
        fr inv;
        fr_inv(inv, acc);         // 1 / (b_0 .. b_(k-1))
        for (u32 i = k; i-- > 0;) {
            const fr bi = lam_raw[o0 + i];
            fr bi_inv, l, lr;
            fr_mul(bi_inv, inv, pre[o0 + i]);   // 1 / b_i
            fr_mul(inv, inv, bi);               // 1 / (b_0 .. b_(i-1))
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

// Lagrange lanes with their tables in a workspace slot (lanetab.hpp): persistent grids of as many blocks as are resident
// at once, each lane walking the entries gid, gid + grid, ... with its own slot, so the workspace is sized by the grid
// and the kernels need no scratch for their tables (round 5; the register-resident tables spilled 5.4 / 10.3 / 22.7 KB
// of scratch per lane for the G1 / G2 / paired G2 lanes).
//
// partial products lambda_i * Y_i for every entry (one lane per entry)
extern "C" __global__ void LCB_BOUNDS k_g1_mul_lanes(const uint8_t *ys, const fr *lam_raw, u32 n_entries, g1 *out,
                                                    uint8_t *ok_out, u32 *ws) {
    const u32 gid = blockIdx.x * blockDim.x + threadIdx.x, gsz = gridDim.x * blockDim.x;
    char *slot = lw_slot(ws, LW_WIN4_QUADS(fp), gid);
#pragma unroll 1
    for (u32 i = gid; i < n_entries; i += gsz) {
        g1a A;
        bool ok = g1_decompress(A, ys + 48 * (size_t)i);
        // the canonical integer lambda with a 4-bit window: exact for every on-curve input, including points outside
        // the r-torsion that G1.FromBytes accepts (GLV would be wrong for their cofactor component)
        g1 R;
        fr k = lam_raw[i];
        lw_mul_win4(R, slot, A, k.v);
        out[i] = R;
        ok_out[i] = ok;
    }
}
// k A for one G2 entry: GLS over the slot's table (entries 1..15) for a point proven to lie in G2, else the plain
// ladder, so the result equals the oracle's for every on-curve input
DI void lw_g2_mul_entry(g2 &R, char *slot, const g2a &A, bool in_g2, const fr &k) {
    if (A.inf) { jac_set_inf(R); return; }
    if (in_g2) {
        u64 d[4];
        lw_gls_digits(d, k.v);
        lw_g2_gls_sums(slot, 0, A);
        if (lw_table_to_aff<fp2>(slot, 15)) { lw_g2_gls_ladder(R, slot, d); return; }
    }
    jac_mul_aff_inl(R, A, k.v, 256);
}
// dec / src (nullable): the decoded shares of the context's last batched CommonCoin check (ts_share_st) and each
// entry's index among them; an entry whose record holds exactly its input bytes takes the record's point and G2 flag
extern "C" __global__ void LCB_BOUNDS k_g2_mul_lanes(const uint8_t *ys, const fr *lam_raw, u32 n_entries, g2 *out,
                                                    uint8_t *ok_out, const ts_share_st *dec, u32 n_dec,
                                                    const u32 *src, u32 *ws) {
    const u32 gid = blockIdx.x * blockDim.x + threadIdx.x, gsz = gridDim.x * blockDim.x;
    char *slot = lw_slot(ws, LW_G2_TAB_QUADS, gid);
#pragma unroll 1
    for (u32 i = gid; i < n_entries; i += gsz) {
        g2a A;
        bool ok, in_g2;
        g2_entry_point(A, ok, in_g2, ys + 96 * (size_t)i, dec, n_dec, src ? src[i] : 0xffffffffu);
        g2 R;
        lw_g2_mul_entry(R, slot, A, in_g2, lam_raw[i]);
        out[i] = R;
        ok_out[i] = ok;
    }
}
// two entries per lane (entries 2p, 2p + 1 of one problem: the caller guarantees even problem offsets): both in G2 ->
// lambda_a A + lambda_b B with one shared run of 64 doublings over both tables (Straus) and one batched inversion for
// the 30 entries, into out[2p] (out[2p + 1] = infinity), else each on its own as k_g2_mul_lanes does; the problem sums
// (k_g2_sum) are the same points
extern "C" __global__ void LCB_BOUNDS k_g2_mul2_lanes(const uint8_t *ys, const fr *lam_raw, u32 n_pairs, g2 *out,
                                                     uint8_t *ok_out, const ts_share_st *dec, u32 n_dec,
                                                     const u32 *src, u32 *ws) {
    const u32 gid = blockIdx.x * blockDim.x + threadIdx.x, gsz = gridDim.x * blockDim.x;
    char *slot = lw_slot(ws, 2 * LW_G2_TAB_QUADS, gid);
#pragma unroll 1
    for (u32 p = gid; p < n_pairs; p += gsz) {
        const u32 i0 = 2 * p, i1 = 2 * p + 1;
        g2a A, B;
        bool oka, okb, ga, gb;
        g2_entry_point(A, oka, ga, ys + 96 * (size_t)i0, dec, n_dec, src ? src[i0] : 0xffffffffu);
        g2_entry_point(B, okb, gb, ys + 96 * (size_t)i1, dec, n_dec, src ? src[i1] : 0xffffffffu);
        const fr ka = lam_raw[i0], kb = lam_raw[i1];
        g2 R0, R1;
        jac_set_inf(R1);
        bool done = false;
        if (ga && gb && !A.inf && !B.inf) {
            lw_g2_gls_sums(slot, 0, A);
            lw_g2_gls_sums(slot, 15, B);
            if (lw_table_to_aff<fp2>(slot, 30)) {
                u64 da[4], db[4];
                lw_gls_digits(da, ka.v);
                lw_gls_digits(db, kb.v);
                lw_g2_gls_ladder2(R0, slot, da, db);
                done = true;
            }
        }
        if (!done) {
            lw_g2_mul_entry(R0, slot, A, ga, ka);
            lw_g2_mul_entry(R1, slot, B, gb, kb);
        }
        out[i0] = R0;
        out[i1] = R1;
        ok_out[i0] = oka;
        ok_out[i1] = okb;
    }
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
extern "C" void lcbk_lagrange_coeffs(dim3 grid, hipStream_t s, const uint8_t *xs, const u32 *off, u32 n_problems, void *lam_raw, void *pre, uint8_t *status) {
    LCB_LAUNCH(k_lagrange_coeffs, xs, off, n_problems, (fr *)lam_raw, (fr *)pre, status);
}
static u32 g_rb_g1, g_rb_g2, g_rb_g2p;
static u32 lanes_blocks(int which, u32 n) {
    const void *k = which == 1 ? (const void *)k_g1_mul_lanes : which == 2 ? (const void *)k_g2_mul_lanes : (const void *)k_g2_mul2_lanes;
    u32 *cache = which == 1 ? &g_rb_g1 : which == 2 ? &g_rb_g2 : &g_rb_g2p;
    return lcb_persist_blocks(k, cache, which == 3 ? n / 2 : n);
}
static u32 lanes_quads(int which) { return which == 1 ? LW_WIN4_QUADS(fp) : which == 2 ? LW_G2_TAB_QUADS : 2 * LW_G2_TAB_QUADS; }
// workspace bytes of the Lagrange lanes over n entries: 1 = G1, 2 = G2, 3 = paired G2
extern "C" size_t lcbk_lanes_ws_bytes(int which, u32 n) {
    return LCB_WS_BYTES(lanes_blocks(which, n), lanes_quads(which));
}
extern "C" void lcbk_g1_mul_lanes(hipStream_t s, const uint8_t *ys, const void *lam_raw, u32 n_entries, void *out, uint8_t *ok_out, u32 *ws) {
    dim3 grid(lanes_blocks(1, n_entries));
    LCB_LAUNCH(k_g1_mul_lanes, ys, (const fr *)lam_raw, n_entries, (g1 *)out, ok_out, ws);
}
extern "C" void lcbk_g2_mul_lanes(hipStream_t s, const uint8_t *ys, const void *lam_raw, u32 n_entries, void *out, uint8_t *ok_out, const void *dec, u32 n_dec, const u32 *src, u32 *ws) {
    dim3 grid(lanes_blocks(2, n_entries));
    LCB_LAUNCH(k_g2_mul_lanes, ys, (const fr *)lam_raw, n_entries, (g2 *)out, ok_out, (const ts_share_st *)dec, n_dec, src, ws);
}
extern "C" void lcbk_g2_mul2_lanes(hipStream_t s, const uint8_t *ys, const void *lam_raw, u32 n_entries, void *out, uint8_t *ok_out, const void *dec, u32 n_dec, const u32 *src, u32 *ws) {
    const u32 n_pairs = n_entries / 2;
    dim3 grid(lanes_blocks(3, n_entries));
    LCB_LAUNCH(k_g2_mul2_lanes, ys, (const fr *)lam_raw, n_pairs, (g2 *)out, ok_out, (const ts_share_st *)dec, n_dec, src, ws);
}
extern "C" void lcbk_g1_sum(dim3 grid, hipStream_t s, const void *parts, const uint8_t *ok_in, const u32 *off, u32 n_problems, uint8_t *status, uint8_t *out) {
    LCB_LAUNCH(k_g1_sum, (const g1 *)parts, ok_in, off, n_problems, status, out);
}
extern "C" void lcbk_g2_sum(dim3 grid, hipStream_t s, const void *parts, const uint8_t *ok_in, const u32 *off, u32 n_problems, uint8_t *status, uint8_t *out) {
    LCB_LAUNCH(k_g2_sum, (const g2 *)parts, ok_in, off, n_problems, status, out);
}
