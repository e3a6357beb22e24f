// lachain_amd/csrc/k_tpke.hip — gfx950 kernels: TPKE decryption-share pipeline (decompression, per-ciphertext preparation, per-share verification, partial decryption).
#include "kcommon.hpp"
#include "fe_asm.hpp"
#include "rlc_common.hpp"

LCB_ASM_LIBRARY(k_tpke)
LCB_TU_CONFIG(k_tpke)
LCB_ASM_TOWER_LIBRARY(k_tpke)

// ================================================================================= decompression
extern "C" __global__ void LCB_BOUNDS k_g1_decompress(const uint8_t *in, u32 n, g1a_st *out) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    g1a a;
    bool ok = g1_decompress(a, in + 48 * (size_t)i);
    g1a_st s;
    s.x = a.x; s.y = a.y; s.inf = ok ? (u32)a.inf : 1u; s.ok = ok; s.pad[0] = s.pad[1] = 0;
    out[i] = s;
}
extern "C" __global__ void LCB_BOUNDS k_g2_decompress(const uint8_t *in, u32 n, g2a_st *out) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    g2a a;
    bool ok = g2_decompress(a, in + 96 * (size_t)i);
    g2a_st s;
    s.x = a.x; s.y = a.y; s.inf = ok ? (u32)a.inf : 1u; s.ok = ok; s.pad[0] = s.pad[1] = 0;
    out[i] = s;
}

// ================================================================================= TPKE
// lines layout: lines[(2*c + 0) * LINESET] = H lines, lines[(2*c + 1) * LINESET] = W lines
// slot (nullable): ciphertext c's line sets and validity go to slot[c] instead of c (the prepared-ciphertext cache)
extern "C" __global__ void LCB_BOUNDS k_tpke_ct_prepare(const uint8_t *cts_u, const uint8_t *cts_w,
                                                       const uint8_t *v_data, const u32 *v_off, u32 n_cts,
                                                       u32 *lines, uint8_t *ct_ok, int flags, const u32 *slot) {
    // flags: bit 0 = mcl's original G2 cofactor clearing in hash-to-G2, bit 1 = mark the line sets un-normalised
    LCB_LATENCY_PRIO();
    u32 c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_cts) return;
    const u32 o = slot ? slot[c] : c;
    const uint8_t *ub = cts_u + 48 * (size_t)c;
    g1a U;
    g2a W, Ha;
    bool ok = g1_decompress(U, ub);
    ok = g2_decompress(W, cts_w + 96 * (size_t)c) && ok;
    // H = G2.SetHashOf(U.ToBytes() || V): for a valid U the wire bytes are its canonical encoding
    uint8_t d[64];
    u32 v0 = v_off[c], v1 = v_off[c + 1];
    sha512_2(d, ub, 48, v_data + v0, v1 - v0);
    g2 H;
    bool hok = g2_hash_digest(H, d, (flags & 1) != 0);
    ok = ok && hok;
    if (hok) g2_jac_to_aff_g(Ha, H);                       // binary-GCD inversion (as k_prep.hip)
    else { Ha.inf = true; Ha.x = fp2_zero(); Ha.y = fp2_zero(); }
    if (!ok) { W.inf = true; Ha.inf = true; }
    // the two points go to their line sets' point slots; k_lineset_fill computes the 2 * n_cts line sets one lane
    // each (the per-ciphertext serial path is hash + one line set instead of hash + two)
    u32 *lsH = lines + (size_t)(2 * o) * LCB_LINESET_WORDS, *lsW = lines + (size_t)(2 * o + 1) * LCB_LINESET_WORDS;
    lineset_put_point(lsH, Ha);
    lineset_put_point(lsW, W);
    lsH[LCB_LS_FLAG + 2] = lsW[LCB_LS_FLAG + 2] = (flags & 2) ? 1 : 0;
    ct_ok[o] = ok;
}

extern "C" __global__ void LCB_BOUNDS k_ct_ok_merge(uint8_t *ct_ok, const uint8_t *h_ok, u32 c0, u32 n_cts) {
    LCB_LATENCY_PRIO();
    u32 c = c0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (c < n_cts) ct_ok[c] = ct_ok[c] && h_ok[c];
}

// line sets of points stored by a prepare kernel (lineset_put_point): one lane per set; sets (nullable) lists the
// set indices to fill (the prepared-ciphertext cache fills scattered slots).  w_g2 (nullable, with sets == nullptr):
// the batched check's W-in-G2 flags, w_g2[c] for set 2c + 1 (W of ciphertext c) from the loop's last point
// (lineset_in_g2): the membership test costs no ladder of its own.
extern "C" __global__ void LCB_BOUNDS k_lineset_fill(u32 *lines, u32 n_sets, const u32 *sets, uint8_t *w_g2) {
    LCB_LATENCY_PRIO();
    u32 k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_sets) return;
    u32 *ls = lines + (size_t)(sets ? sets[k] : k) * LCB_LINESET_WORDS;
    g2a Q;
    lineset_get_point(Q, ls);
    u32 force_general = ls[LCB_LS_FLAG + 2];
    u32 r = lineset_compute(ls, Q);
    if (force_general) ls[LCB_LS_FLAG] = 0;
    if (w_g2 && (k & 1)) w_g2[k >> 1] = (r & LCB_LS_IN_G2) ? 1 : 0;
}

// Exact per-share check, two kernels: the Miller loop parks f in HBM (SoA, 576 B/share) and k_final_exp_check finishes;
// each kernel gets its own register budget (a single fused kernel spilled more and measured slower).  accept[i] carries the
// decompression / key / ciphertext validity from the first kernel to the second.
extern "C" __global__ void LCB_PAIR_BOUNDS k_tpke_miller(const u32 *lines, const uint8_t *ct_ok, u32 n_cts,
                                                         const g1a_st *keys, u32 n_keys, const u32 *ct_idx,
                                                         const u32 *dec_idx, const uint8_t *ui, u32 n, u32 *f_soa,
                                                         uint8_t *accept) {
    __shared__ uint4 ml_lds[36 * LCB_BLOCK];    // the assembly Miller loop's double-width products (lcb_r_miller2)
    const u32 lds = lane_lds36(ml_lds);
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u32 c = ct_idx[i], d = dec_idx[i];
    g1a Ui, Y;
    bool ok = d < n_keys && c < n_cts;   // an out-of-range index rejects the share (and is clamped)
    c = c < n_cts ? c : 0;
    ok = ok && ct_ok[c];
    ok = g1_decompress(Ui, ui + 48 * (size_t)i) && ok;
    g1a_st ks = keys[d < n_keys ? d : 0];
    ok = ok && ks.ok;
    st_to_g1a(Y, ks);
    fp_neg(Y.y, Y.y);
    const u32 *lsH = lines + (size_t)(2 * c) * LCB_LINESET_WORDS, *lsW = lines + (size_t)(2 * c + 1) * LCB_LINESET_WORDS;
    if (lineset_normalised(lsH) && lineset_normalised(lsW)) {
        miller2_asm(f_soa, n, i, lds, lsH, Ui, lsW, Y);  // f -> slot 0 (slots 1..3 as its scratch)
    } else {
        fp12 f;
        miller2_sets_fallback(f, lsH, Ui, lsW, Y);
        fp12_store_soa(f_soa, n, i, f);
    }
    accept[i] = ok;
}
// accept[i] &= (final_exp(f_i) == 1).  park: SoA Fp12 slots per item (lcbk_fe_slots()), slot 0 = f from the Miller
// kernel, left holding the final exponentiation (the level-2 search reads it): fe_asm.hpp (exponentiations by z over
// the AGPR-resident Fp12 assembly squaring, the hard part's other values in slots 0..5).  Measured alternatives, removed:
// the compiler-built __noinline__ Fp12 functions 62.5 ms, the exp-by-z loop inlined in the kernel 69.1 ms per 262,144
// shares, Fp12 state parked in LDS 30 % slower than the former.
extern "C" int lcbk_fe_slots() { return LCB_FE_ASM_SLOTS; }
extern "C" __global__ void LCB_PAIR_BOUNDS k_final_exp_check(u32 *park, u32 n, uint8_t *accept) {
    LCB_LATENCY_PRIO();
    __shared__ uint4 fx_lds[36 * LCB_BLOCK];      // per lane: the double-width Fp2 products of an Fp6 product
    typedef __attribute__((address_space(3))) uint4 lds_quad_t;
    // wave w's 36 KB: quad g of lane l at g * 1024 + l * 16 (a wave's access is 1 KB contiguous per quad)
    const u32 lds = (u32)(uintptr_t)(lds_quad_t *)fx_lds + (threadIdx.x >> 6) * (36u * 1024u) + (threadIdx.x & 63u) * 16u;
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    final_exp_asm(park, n, i, lds);
    fp12 f;
    fp12_load_soa(f, park, n, i);
    accept[i] = accept[i] && fp12_is_one(f);
}

// TPKE.PrivateKey.Decrypt (TPKE/PrivateKey.cs:21-31): validity e(G, W) == e(U, H) <=> e(-G, W) e(U, H) == 1, then
// Ui = x U.  Three launches over ciphertexts c0 + [0, m) (round 5; one fused kernel spilled 7.7 KB of scratch per lane):
// the Miller loop parks f (SoA, as k_tpke_miller), k_final_exp_check ANDs f^((p^12-1)/r) == 1 into status, and the
// ladder writes x U for the valid ones (zero bytes otherwise).
extern "C" __global__ void LCB_PAIR_BOUNDS k_tpke_pd_miller(const u32 *lines, const uint8_t *ct_ok, const uint8_t *cts_u,
                                                            u32 c0, u32 m, u32 *f_soa, uint8_t *status) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const u32 c = c0 + i;
    g1a U, G;
    bool ok = g1_decompress(U, cts_u + 48 * (size_t)c) && ct_ok[c];
    g1_generator(G);
    fp_neg(G.y, G.y);
    fp12 f;
    miller2_sets(f, lines + (size_t)(2 * c) * LCB_LINESET_WORDS, U, lines + (size_t)(2 * c + 1) * LCB_LINESET_WORDS, G);
    fp12_store_soa(f_soa, m, i, f);
    status[c] = ok;
}
extern "C" __global__ void LCB_BOUNDS k_tpke_pd_mul(const uint8_t *cts_u, const fr *x_raw, u32 x_stride, u32 c0, u32 m,
                                                   const uint8_t *status, uint8_t *ui_out) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const u32 c = c0 + i;
    uint8_t *o = ui_out + 48 * (size_t)c;
    g1a U;
    if (!status[c] || !g1_decompress(U, cts_u + 48 * (size_t)c)) {
        fp z = fp_zero();
        raw_to_bytes48(o, z);
        return;
    }
    g1 R;
    fr k = x_raw[(size_t)c * x_stride];
    jac_mul_aff(R, U, k.v, 256);
    g1_compress_jac(o, R);
}


// ---------------------------------------------------------------- host launch wrappers
extern "C" void lcbk_g1_decompress(dim3 grid, hipStream_t s, const uint8_t *in, u32 n, void *out) {
    LCB_LAUNCH(k_g1_decompress, in, n, (g1a_st *)out);
}
extern "C" void lcbk_g2_decompress(dim3 grid, hipStream_t s, const uint8_t *in, u32 n, void *out) {
    LCB_LAUNCH(k_g2_decompress, in, n, (g2a_st *)out);
}
extern "C" void lcbk_tpke_ct_prepare(dim3 grid, hipStream_t s, const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data, const u32 *v_off, u32 n_cts, u32 *lines, uint8_t *ct_ok, int orig_cof, const u32 *slot) {
    LCB_LAUNCH(k_tpke_ct_prepare, cts_u, cts_w, v_data, v_off, n_cts, lines, ct_ok, orig_cof, slot);
}
// the same kernel in one-wave workgroups, for the few census ciphertexts of the batched check: a wave at 346 registers
// needs one SIMD with that many free, where a 256-lane workgroup needs four on one CU (round 5: behind the
// randomisation's two waves per SIMD the census's single workgroup waited 34 ms for a whole CU in about half the steps)
extern "C" void lcbk_tpke_ct_prepare_w64(hipStream_t s, const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data, const u32 *v_off, u32 n_cts, u32 *lines, uint8_t *ct_ok, int orig_cof) {
    LCB_LAUNCH_GATED(k_tpke_ct_prepare, dim3((n_cts + 63) / 64), dim3(64), 0, s, cts_u, cts_w, v_data, v_off, n_cts,
                     lines, ct_ok, orig_cof, (const u32 *)nullptr);
}
extern "C" void lcbk_ct_ok_merge(hipStream_t s, uint8_t *ct_ok, const uint8_t *h_ok, u32 c0, u32 c1) {
    dim3 grid((c1 - c0 + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_ct_ok_merge, ct_ok, h_ok, c0, c1);
}
extern "C" void lcbk_lineset_fill(dim3 grid, hipStream_t s, u32 *lines, u32 n_sets, const u32 *sets, uint8_t *w_g2) {
    LCB_LAUNCH(k_lineset_fill, lines, n_sets, sets, w_g2);
}
// ---------------------------------------------------------------- TPKE group Miller loops of the batched check
// (k_batch.hip describes the levels): one lane per group, the two-pair loop of k_tpke_miller over the group's two
// points (sum s_i U_i, -sum s_i Y_i) — here, beside the assembly library the loop calls
extern "C" __global__ void LCB_PAIR_BOUNDS k_tpke_rlc_miller(const u32 *lines, const uint4 *desc, const g1a_st *gpts,
                                                            u32 n_groups, u32 *f_soa, uint8_t *gacc) {
    LCB_LATENCY_PRIO();
    __shared__ uint4 ml_lds[36 * LCB_BLOCK];
    const u32 lds = lane_lds36(ml_lds);
    u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_groups) return;
    u32 c = desc[g].z;
    g1a P, Q;
    st_to_g1a(P, gpts[2 * (size_t)g]);
    st_to_g1a(Q, gpts[2 * (size_t)g + 1]);
    const u32 *lsH = lines + (size_t)(2 * c) * LCB_LINESET_WORDS, *lsW = lines + (size_t)(2 * c + 1) * LCB_LINESET_WORDS;
    if (lineset_normalised(lsH) && lineset_normalised(lsW)) {
        miller2_asm(f_soa, n_groups, g, lds, lsH, P, lsW, Q);
    } else {
        fp12 f;
        miller2_sets_fallback(f, lsH, P, lsW, Q);
        fp12_store_soa(f_soa, n_groups, g, f);
    }
    gacc[g] = 1;
}
extern "C" void lcbk_tpke_rlc_miller(dim3 grid, hipStream_t s, const u32 *lines, const void *desc, const void *gpts,
                                     u32 n_groups, u32 *f_soa, uint8_t *gacc) {
    LCB_LAUNCH(k_tpke_rlc_miller, lines, (const uint4 *)desc, (const g1a_st *)gpts, n_groups, f_soa, gacc);
}
extern "C" void lcbk_tpke_miller(dim3 grid, hipStream_t s, const u32 *lines, const uint8_t *ct_ok, u32 n_cts, const void *keys, u32 n_keys, const u32 *ct_idx, const u32 *dec_idx, const uint8_t *ui, u32 n, u32 *f_soa, uint8_t *accept) {
    LCB_LAUNCH(k_tpke_miller, lines, ct_ok, n_cts, (const g1a_st *)keys, n_keys, ct_idx, dec_idx, ui, n, f_soa, accept);
}
extern "C" void lcbk_final_exp_check(dim3 grid, hipStream_t s, u32 *park, u32 n, uint8_t *accept) {
    LCB_LAUNCH(k_final_exp_check, park, n, accept);
}
extern "C" void lcbk_tpke_pd_miller(hipStream_t s, const u32 *lines, const uint8_t *ct_ok, const uint8_t *cts_u, u32 c0, u32 m, u32 *f_soa, uint8_t *status) {
    dim3 grid((m + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_tpke_pd_miller, lines, ct_ok, cts_u, c0, m, f_soa, status);
}
extern "C" void lcbk_tpke_pd_mul(hipStream_t s, const uint8_t *cts_u, const void *x_raw, u32 x_stride, u32 c0, u32 m, const uint8_t *status, uint8_t *ui_out) {
    dim3 grid((m + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_tpke_pd_mul, cts_u, (const fr *)x_raw, x_stride, c0, m, status, ui_out);
}

// ================================================================================= level-2 two-error search (TPKE)
// k_tpke_rlc_search2b (k_batch.hip: the algorithm and its proof) with every Fp12 product and squaring on the assembly
// routines (asm_tower.hpp lcb_r_fp12_mul_n / lcb_r_cyc_sqr_n) over per-lane park slots, instead of the compiled
// products that passed three Fp12 values through the lane's stack each (round 6: 133 KB of HBM traffic per lane, and
// the level's longest kernel on the single batch's critical path).  The same products in the same order on canonical
// values, so the same words, fingerprints and decisions.  Slots (n = the launch's lanes, 144 words each): X, Y (the
// scans), D, E0 / E1 (the giant steps), the baby powers D^1 .. D^6.
#define S2B_SLOTS 11
DI void s2b_half_scan(u32 *SX, u32 *SY, size_t n, size_t i, u32 n16, u32 i16, u32 la) {
    const u32 j = threadIdx.x & 31;
#pragma unroll 1
    for (u32 off = 1; off < 32; off <<= 1) {          // x <- x_0 x_1 ... x_j (the lanes below off multiply by 1)
        fp12 x, y;
        fp12_load_soa_fresh(x, SX, n, i);
        u32 *yw = (u32 *)&y;
        const u32 *xw = (const u32 *)&x;
#pragma unroll
        for (int q = 0; q < 144; q++) yw[q] = (u32)__shfl_up((int)xw[q], off, 32);
        if (j < off) y = fp12_one();
        fp12_store_soa(SY, n, i, y);
        lcb_asm_fp12_mul_n(SX, 0, SY, SX, SX, n16, i16, la);
    }
}
extern "C" __global__ void __launch_bounds__(64) k_tpke_rlc_search2b_asm(const uint4 *search, u32 ns, const u32 *gamma0,
                                                                        const u32 *gamma12, const u32 *open,
                                                                        const u32 *open_count, uint8_t *accept,
                                                                        uint4 *next, u32 *next_count,
                                                                        const u32 *key_idx, u32 n_keys,
                                                                        const u32 *susp, u32 *park) {
    __shared__ uint4 lds[36 * 64];
    LCB_LATENCY_PRIO();
    const u32 j = threadIdx.x & 31, k = blockIdx.x * 2 + (threadIdx.x >> 5);
    if (blockIdx.x * 2 >= *open_count) return;          // (uniform per block)
    const bool live = k < *open_count;
    const u32 g = live ? open[k] : 0;
    const uint4 d = live ? search[g] : make_uint4(0, 0, 0, 0);
    const bool cand = live && j < d.y && accept[d.x + j] && !key_suspect(susp, key_idx[d.x + j], n_keys);
    const u32 cj = j + 1;
    const size_t n = (size_t)gridDim.x * 64, i = (size_t)blockIdx.x * 64 + threadIdx.x;
    const u32 n16 = (u32)(n * 16), i16 = (u32)(i * 16), la = lane_lds36(lds);
    u32 *SX = park, *SY = park + 144 * n, *SD = park + 288 * n, *SE0 = park + 432 * n, *SE1 = park + 576 * n;
    u32 *BP = park + 720 * n;                           // D^(k + 1) at BP + 144 n k
    fp12 t;
    fp12_load_row(t, gamma0 + (size_t)g * 144);
    fp12_store_soa(SX, n, i, t);
    s2b_half_scan(SX, SY, n, i, n16, i16, la);          // gamma_0^(c_j)
    fp12_load_row(t, gamma12 + (size_t)g * 144);
    fp12_store_soa(SE0, n, i, t);                       // gamma_c
    lcb_asm_fp12_mul_n(SX, 1, SE0, SD, SD, n16, i16, la);        // D_j = gamma_c / gamma_0^(c_j)
    s2b_half_scan(SE0, SY, n, i, n16, i16, la);         // gamma_c^(c_j)
    fp12_load_row(t, gamma12 + (size_t)g * 144);
    fp12_store_soa(SE1, n, i, t);
    lcb_asm_fp12_mul_n(SE0, 0, SE1, SX, SX, n16, i16, la);       // gamma_c^(c_j + 1)
    fp12_load_row(t, gamma12 + ((size_t)ns + g) * 144); // gamma_t
    fp12_store_soa(SE1, n, i, t);
    lcb_asm_cyc_sqr_n(SE1, SE1, n16, i16, 1);
    lcb_asm_fp12_mul_n(SX, 1, SE1, SE0, SE0, n16, i16, la);      // E_j = gamma_t^2 / gamma_c^(c_j + 1)
    // baby steps: fingerprints of D^1 .. D^6 (every lane: the products stay uniform across the wave)
    u32 fpb[6];
    fp12_load_soa_fresh(t, SD, n, i);
    fpb[0] = fp12_fingerprint(t);
    fp12_store_soa(BP, n, i, t);
#pragma unroll 1
    for (int kk = 1; kk < 6; kk++) {
        u32 *dst = BP + 144 * n * (size_t)kk;
        lcb_asm_fp12_mul_n(BP + 144 * n * (size_t)(kk - 1), 0, SD, dst, dst, n16, i16, la);
        fp12_load_soa_fresh(t, dst, n, i);
        fpb[kk] = fp12_fingerprint(t);
    }
    // giant steps Y_i = E D^(-6 i): a fingerprint match Y_i ~ D^(k+1) confirmed against the stored baby power
    u32 found = 0;
    u32 *Y = SE0, *Yn = SE1;
#pragma unroll 1
    for (int gi = 0; gi < 6; gi++) {
        fp12_load_soa_fresh(t, Y, n, i);
        const u32 h = fp12_fingerprint(t);
#pragma unroll 1
        for (int kk = 0; kk < 6; kk++) {
            const u32 c = 6 * gi + kk + 1;
            if (cand && !found && h == fpb[kk] && c <= d.y && c != cj) {
                fp12 chk;
                fp12_load_soa_fresh(chk, BP + 144 * n * (size_t)kk, n, i);
                if (fp12_words_eq(chk, t)) found = c;
            }
        }
        if (gi < 5) {
            lcb_asm_fp12_mul_n(BP + 144 * n * 5, 1, Y, Yn, Yn, n16, i16, la);   // Y D^-6 (D unitary)
            u32 *sw = Y;
            Y = Yn;
            Yn = sw;
        }
    }
    const u32 m2 = half_ballot(found != 0);
    const u32 m3 = half_ballot(found != 0 && !((m2 >> ((found - 1) & 31u)) & 1u));
    if (__popc(m2) == 2 && !m3) {
        if (found) accept[d.x + j] = 0;
    } else if (live && j == 0) {
        emit_singles(d, 0, accept, key_idx, n_keys, susp, next, next_count);
    }
}
extern "C" size_t lcbk_tpke_rlc_search2b_asm_park_bytes(u32 n_open) {
    return (size_t)((n_open + 1) / 2) * 64 * S2B_SLOTS * 576;
}
extern "C" void lcbk_tpke_rlc_search2b_asm(hipStream_t s, const void *search, u32 ns, u32 n_open, const u32 *gamma0,
                                           const u32 *gamma12, const u32 *open, const u32 *open_count, uint8_t *accept,
                                           void *next, u32 *next_count, const u32 *key_idx, u32 n_keys,
                                           const u32 *susp, u32 *park) {
    if (!n_open) return;
    LCB_LAUNCH_GATED(k_tpke_rlc_search2b_asm, dim3((n_open + 1) / 2), dim3(64), 0, s, (const uint4 *)search, ns, gamma0,
                     gamma12, open, open_count, accept, (uint4 *)next, next_count, key_idx, n_keys, susp, park);
}
