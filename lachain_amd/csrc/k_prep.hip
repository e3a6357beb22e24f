// lachain_amd/csrc/k_prep.hip — gfx950 kernels: the split TPKE preparation of the fused batched verify (hash lane and
// point lane, each through its line set).  A translation unit of its own, built like k_rlc_rand.hip without
// VGPR-to-AGPR spilling and with every kernel at two waves per SIMD, so the attribute reaches the non-inlined callees
// (line sets, hash to G2, decompression) and the lanes fit in 256 registers: one preparation wave (256) then shares a
// SIMD with one randomisation wave (248) instead of holding it to itself with 346 (round 5, VERDICT r4 #4: the
// randomisation started 14-16 ms into the step, when the preparation waves retired).
#include "kcommon.hpp"
#include "lines_coop.hpp"
#include "coop.hpp"
#include "ts_rlc.hpp"

LCB_ASM_LIBRARY(k_prep)
LCB_TU_CONFIG(k_prep)

#define LCB_PREP_BOUNDS __launch_bounds__(LCB_BLOCK) __attribute__((amdgpu_waves_per_eu(2)))

// k_tpke_ct_prepare split in two lane kinds that run side by side (fused batched verify, fork mode 3), each through
// its line set: the hash lane (H = G2.SetHashOf(U || V), then H's line set; h_ok = the hash succeeded) and the point
// lane (U and W decode, then W's line set with its G2 flag; ct_ok = both decode).  k_ct_ok_merge then ANDs h_ok into
// ct_ok.  An undecodable ciphertext keeps H's real line set (ct_ok = 0 gates every use) and gets W = infinity.
DI void ct_prepare_h_run(u32 c, const uint8_t *cts_u, const uint8_t *v_data, const u32 *v_off, u32 *lines, uint8_t *h_ok,
                        int flags) {
    uint8_t d[64];
    u32 v0 = v_off[c], v1 = v_off[c + 1];
    sha512_2(d, cts_u + 48 * (size_t)c, 48, v_data + v0, v1 - v0);
    g2 H;
    g2a Ha;
    bool hok = g2_hash_digest(H, d, (flags & 1) != 0);
    if (hok) g2_jac_to_aff_g(Ha, H);
    else { Ha.inf = true; Ha.x = fp2_zero(); Ha.y = fp2_zero(); }
    u32 *ls = lines + (size_t)(2 * c) * LCB_LINESET_WORDS;
    lineset_compute(ls, Ha);
    if (flags & 2) ls[LCB_LS_FLAG] = 0;
    h_ok[c] = hok;
}
DI void ct_prepare_w_run(u32 c, const uint8_t *cts_u, const uint8_t *cts_w, u32 *lines, uint8_t *ct_ok, uint8_t *w_g2,
                        int flags) {
    g1a U;
    g2a W;
    bool ok = g1_decompress(U, cts_u + 48 * (size_t)c);
    ok = g2_decompress(W, cts_w + 96 * (size_t)c) && ok;
    if (!ok) { W.inf = true; W.x = fp2_zero(); W.y = fp2_zero(); }
    u32 *ls = lines + (size_t)(2 * c + 1) * LCB_LINESET_WORDS;
    u32 r = lineset_compute(ls, W);
    if (flags & 2) ls[LCB_LS_FLAG] = 0;
    ct_ok[c] = ok;
    w_g2[c] = (r & LCB_LS_IN_G2) ? 1 : 0;
}
extern "C" __global__ void LCB_PREP_BOUNDS k_tpke_ct_prepare_h(const uint8_t *cts_u, const uint8_t *v_data, const u32 *v_off,
                                                         u32 c0, u32 n_cts, u32 *lines, uint8_t *h_ok, int flags) {
    LCB_LATENCY_PRIO();
    u32 c = c0 + blockIdx.x * blockDim.x + threadIdx.x;     // ciphertexts [c0, n_cts)
    if (c >= n_cts) return;
    ct_prepare_h_run(c, cts_u, v_data, v_off, lines, h_ok, flags);
}
extern "C" __global__ void LCB_PREP_BOUNDS k_tpke_ct_prepare_w(const uint8_t *cts_u, const uint8_t *cts_w, u32 c0,
                                                         u32 n_cts, u32 *lines, uint8_t *ct_ok, uint8_t *w_g2,
                                                         int flags) {
    LCB_LATENCY_PRIO();
    u32 c = c0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_cts) return;
    ct_prepare_w_run(c, cts_u, cts_w, lines, ct_ok, w_g2, flags);
}
// Both lane kinds in one dispatch (fork mode 4: one high-priority stream per context): blocks [0, nb_h) are hash
// lanes, the rest point lanes, over ciphertexts [0, n_cts).  At the box's GPU_MAX_HW_QUEUES = 4 a context's two
// preparation streams of fork mode 3 shared hardware queues with the other batches in flight.
extern "C" __global__ void LCB_PREP_BOUNDS k_tpke_ct_prepare_hw(const uint8_t *cts_u, const uint8_t *cts_w,
                                                          const uint8_t *v_data, const u32 *v_off, u32 n_cts, u32 nb_h,
                                                          u32 *lines, uint8_t *h_ok, uint8_t *ct_ok, uint8_t *w_g2,
                                                          int flags) {
    LCB_LATENCY_PRIO();
    const bool hash = blockIdx.x < nb_h;
    u32 c = (hash ? blockIdx.x : blockIdx.x - nb_h) * blockDim.x + threadIdx.x;
    if (c >= n_cts) return;
    if (hash) ct_prepare_h_run(c, cts_u, v_data, v_off, lines, h_ok, flags);
    else ct_prepare_w_run(c, cts_u, cts_w, lines, ct_ok, w_g2, flags);
}

// H(m) and its line set per message (the CommonCoin preparation, ThresholdSigner.cs:44-87 hashes each coin's message):
// here at 256 registers, so the 1,024 waves of configs[2] share their SIMDs with the randomisation's instead of
// waiting for whole SIMDs to drain (at 346 registers the kernel ran 462 ms beside k_ts_rlc_points against 16 ms
// ahead of it, round-5 trace)
extern "C" __global__ void LCB_PREP_BOUNDS k_ts_msg_prepare(const uint8_t *msg_data, const u32 *msg_off, u32 n_msgs,
                                                           u32 *lines, uint8_t *msg_ok, int flags) {
    LCB_LATENCY_PRIO();
    u32 m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= n_msgs) return;
    uint8_t d[64];
    u32 o0 = msg_off[m], o1 = msg_off[m + 1];
    sha512_2(d, msg_data + o0, o1 - o0, msg_data, 0);
    g2 H;
    g2a Ha;
    bool ok = g2_hash_digest(H, d, (flags & 1) != 0);
    if (ok) g2_jac_to_aff_g(Ha, H);
    else { Ha.inf = true; Ha.x = fp2_zero(); Ha.y = fp2_zero(); }
    lineset_compute(lines + (size_t)m * LCB_LINESET_WORDS, Ha);
    if (flags & 2) lines[(size_t)m * LCB_LINESET_WORDS + LCB_LS_FLAG] = 0;
    msg_ok[m] = ok;
}

// k_lineset_coop (k_lines.hip) at two waves per SIMD: the census ciphertexts' line sets, which run while the
// randomisation and the preparation hold the SIMDs (at 417 registers a wave of k_lineset_coop found room only as
// those waves retired: 4 -> 24 ms in the round-5 A/B)
extern "C" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) k_lineset_coop_2w(
        u32 *lines, u32 n_sets, const u32 *sets, uint8_t *w_g2) {
    __shared__ LsLds lds[LS_GROUPS + 1];
    lineset_coop_run(lds, lines, n_sets, sets, w_g2);
}

// The CommonCoin census chain (lcb_host.cpp rlc_census: the census shares' exact singles, their two-pair Miller loops,
// the nine-lane final exponentiation) at 256 registers: k_ts_rlc_points holds two 256-register waves per SIMD for
// ~450 ms, and the 294 / 360 / 284-register copies of k_batch.hip / k_coop.hip found no SIMD with room until it
// retired, so the census ran after the randomisation, on the step's critical path (round-5 trace: 20 ms).  At 256 a
// census wave takes the slot of the first randomisation wave that retires (its stream has the higher priority).  The
// nine-lane final exponentiation's copy (248 registers, the same spills) serves every batched level (rlc_checks): with
// three TPKE batches in flight its waves share SIMDs with the other batches' randomisation waves.
extern "C" __global__ void LCB_PREP_BOUNDS k_ts_rlc_sum_census(const uint4 *desc, u32 n_groups, u32 first,
                                                              const uint8_t *msg_ok, const g1a_st *pks, u32 n_pks,
                                                              const u32 *pk_idx, const uint8_t *sigs, const u32 *rP,
                                                              const u32 *rS, u32 n, ts_grp *gpts, uint8_t *accept,
                                                              uint8_t *gexact, u32 *wsum, const u32 *susp,
                                                              uint8_t *cval) {
    LCB_LATENCY_PRIO();
    ts_rlc_sum_run(desc, n_groups, first, msg_ok, pks, n_pks, pk_idx, sigs, rP, rS, n, gpts, accept, gexact, wsum, susp,
                   cval);
}
// the CommonCoin group sums of every level with two lanes per group (ts_rlc.hpp ts_rlc_sum2_run)
extern "C" __global__ void LCB_PREP_BOUNDS k_ts_rlc_sum2(const uint4 *desc, u32 n_groups, u32 first,
                                                        const uint8_t *msg_ok, const g1a_st *pks, u32 n_pks,
                                                        const u32 *pk_idx, const uint8_t *sigs, const u32 *rP,
                                                        const u32 *rS, u32 n, ts_grp *gpts, uint8_t *accept,
                                                        uint8_t *gexact, u32 *wsum, const u32 *susp, uint8_t *cval) {
    LCB_LATENCY_PRIO();
    ts_rlc_sum2_run(desc, n_groups, first, msg_ok, pks, n_pks, pk_idx, sigs, rP, rS, n, gpts, accept, gexact, wsum, susp,
                    cval);
}
extern "C" __global__ void LCB_PREP_BOUNDS k_ts_rlc_miller_census(const u32 *lines, const uint4 *desc,
                                                                 const ts_grp *gpts, u32 n_groups, u32 *f_soa,
                                                                 uint8_t *gacc) {
    LCB_LATENCY_PRIO();
    ts_rlc_miller_run(lines, desc, gpts, n_groups, f_soa, gacc);
}
extern "C" __global__ void __launch_bounds__(CP_BLOCK) __attribute__((amdgpu_waves_per_eu(2)))
k_coop_final_exp_check_2w(u32 *park, u32 n, uint8_t *accept) {
    LCB_LATENCY_PRIO();
    __shared__ uint4 lds[CP_LDS_QUADS];
    cp_final_exp_check_run(lds, park, n, accept);
}

// ---------------------------------------------------------------- host launch wrappers
extern "C" void lcbk_ts_rlc_sum_census(dim3 grid, hipStream_t s, const void *desc, u32 n_groups, u32 first,
                                       const uint8_t *msg_ok, const void *pks, u32 n_pks, const u32 *pk_idx,
                                       const uint8_t *sigs, const u32 *rP, const u32 *rS, u32 n, void *gpts,
                                       uint8_t *accept, uint8_t *gexact, u32 *wsum, const u32 *susp, uint8_t *cval) {
    LCB_LAUNCH(k_ts_rlc_sum_census, (const uint4 *)desc, n_groups, first, msg_ok, (const g1a_st *)pks, n_pks, pk_idx,
               sigs, rP, rS, n, (ts_grp *)gpts, accept, gexact, wsum, susp, cval);
}
extern "C" void lcbk_ts_rlc_sum2(hipStream_t s, const void *desc, u32 n_groups, u32 first, const uint8_t *msg_ok,
                                 const void *pks, u32 n_pks, const u32 *pk_idx, const uint8_t *sigs, const u32 *rP,
                                 const u32 *rS, u32 n, void *gpts, uint8_t *accept, uint8_t *gexact, u32 *wsum,
                                 const u32 *susp, uint8_t *cval) {
    dim3 grid((2 * (size_t)n_groups + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_ts_rlc_sum2, (const uint4 *)desc, n_groups, first, msg_ok, (const g1a_st *)pks, n_pks, pk_idx, sigs,
               rP, rS, n, (ts_grp *)gpts, accept, gexact, wsum, susp, cval);
}
extern "C" void lcbk_ts_rlc_miller_census(dim3 grid, hipStream_t s, const u32 *lines, const void *desc,
                                          const void *gpts, u32 n_groups, u32 *f_soa, uint8_t *gacc) {
    LCB_LAUNCH(k_ts_rlc_miller_census, lines, (const uint4 *)desc, (const ts_grp *)gpts, n_groups, f_soa, gacc);
}
extern "C" void lcbk_coop_final_exp_check_2w(hipStream_t s, u32 *park, u32 n, uint8_t *accept) {
    dim3 grid((n + CP_G - 1) / CP_G);
    LCB_LAUNCH_GATED(k_coop_final_exp_check_2w, grid, dim3(CP_BLOCK), 0, s, park, n, accept);
}
extern "C" void lcbk_lineset_coop_2w(hipStream_t s, u32 *lines, u32 n_sets, const u32 *sets, uint8_t *w_g2) {
    if (!n_sets) return;
    LCB_LAUNCH_GATED(k_lineset_coop_2w, dim3((n_sets + LS_GROUPS - 1) / LS_GROUPS), dim3(64), 0, s, lines, n_sets,
                       sets, w_g2);
}
extern "C" void lcbk_ts_msg_prepare(dim3 grid, hipStream_t s, const uint8_t *msg_data, const u32 *msg_off, u32 n_msgs,
                                    u32 *lines, uint8_t *msg_ok, int orig_cof) {
    LCB_LAUNCH(k_ts_msg_prepare, msg_data, msg_off, n_msgs, lines, msg_ok, orig_cof);
}
// ciphertexts [c0, c1)
extern "C" void lcbk_tpke_ct_prepare_h(hipStream_t s, const uint8_t *cts_u, const uint8_t *v_data, const u32 *v_off, u32 c0, u32 c1, u32 *lines, uint8_t *h_ok, int flags) {
    dim3 grid((c1 - c0 + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_tpke_ct_prepare_h, cts_u, v_data, v_off, c0, c1, lines, h_ok, flags);
}
extern "C" void lcbk_tpke_ct_prepare_w(hipStream_t s, const uint8_t *cts_u, const uint8_t *cts_w, u32 c0, u32 c1, u32 *lines, uint8_t *ct_ok, uint8_t *w_g2, int flags) {
    dim3 grid((c1 - c0 + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_tpke_ct_prepare_w, cts_u, cts_w, c0, c1, lines, ct_ok, w_g2, flags);
}
extern "C" void lcbk_tpke_ct_prepare_hw(hipStream_t s, const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data,
                                        const u32 *v_off, u32 n_cts, u32 *lines, uint8_t *h_ok, uint8_t *ct_ok,
                                        uint8_t *w_g2, int flags) {
    if (!n_cts) return;
    const u32 nb = (n_cts + LCB_BLOCK - 1) / LCB_BLOCK;
    dim3 grid(2 * nb);
    LCB_LAUNCH(k_tpke_ct_prepare_hw, cts_u, cts_w, v_data, v_off, n_cts, nb, lines, h_ok, ct_ok, w_g2, flags);
}
