// lachain_amd/csrc/launch.h — host-side launch wrappers exported by the kernel translation units
// (device-internal record types are passed as opaque pointers).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "ops.h"
typedef uint32_t u32;
#define LCB_TS_SHARE_REC_BYTES 304     // ts_share_st (kcommon.hpp): a decoded CommonCoin share
extern "C" void lcbk_g1_decompress(dim3 grid, hipStream_t s, const uint8_t *in, u32 n, void *out);
extern "C" void lcbk_g2_decompress(dim3 grid, hipStream_t s, const uint8_t *in, u32 n, void *out);
extern "C" void lcbk_tpke_ct_prepare(dim3 grid, hipStream_t s, const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data, const u32 *v_off, u32 n_cts, u32 *lines, uint8_t *ct_ok, int orig_cof, const u32 *slot);
extern "C" void lcbk_tpke_ct_prepare_w64(hipStream_t s, const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data, const u32 *v_off, u32 n_cts, u32 *lines, uint8_t *ct_ok, int orig_cof);
extern "C" void lcbk_tpke_ct_prepare_h(hipStream_t s, const uint8_t *cts_u, const uint8_t *v_data, const u32 *v_off, u32 c0, u32 c1, u32 *lines, uint8_t *h_ok, int flags);
extern "C" void lcbk_tpke_ct_prepare_w(hipStream_t s, const uint8_t *cts_u, const uint8_t *cts_w, u32 c0, u32 c1, u32 *lines, uint8_t *ct_ok, uint8_t *w_g2, int flags);
extern "C" void lcbk_tpke_ct_prepare_hw(hipStream_t s, const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data, const u32 *v_off, u32 n_cts, u32 *lines, uint8_t *h_ok, uint8_t *ct_ok, uint8_t *w_g2, int flags);
extern "C" void lcbk_ct_ok_merge(hipStream_t s, uint8_t *ct_ok, const uint8_t *h_ok, u32 c0, u32 c1);
extern "C" void lcbk_lineset_fill(dim3 grid, hipStream_t s, u32 *lines, u32 n_sets, const u32 *sets, uint8_t *w_g2);
extern "C" void lcbk_mcl_g2_hash(hipStream_t s, u32 *io, int orig_cof);
extern "C" void lcbk_lineset_coop(hipStream_t s, u32 *lines, u32 n_sets, const u32 *sets, uint8_t *w_g2);
// the same at two waves per SIMD (k_prep.hip): the census ciphertexts of the fused batched verify
extern "C" void lcbk_lineset_coop_2w(hipStream_t s, u32 *lines, u32 n_sets, const u32 *sets, uint8_t *w_g2);
extern "C" void lcbk_tpke_miller(dim3 grid, hipStream_t s, const u32 *lines, const uint8_t *ct_ok, u32 n_cts, const void *keys, u32 n_keys, const u32 *ct_idx, const u32 *dec_idx, const uint8_t *ui, u32 n, u32 *f_soa, uint8_t *accept);
extern "C" int lcbk_fe_slots();
extern "C" void lcbk_final_exp_check(dim3 grid, hipStream_t s, u32 *park, u32 n, uint8_t *accept);
// TPKE partial decryption over ciphertexts c0 + [0, m): Miller loop into f_soa (m x 576 B x lcbk_fe_slots()), then
// lcbk_final_exp_check(f_soa, m, status + c0), then the ladder
extern "C" void lcbk_tpke_pd_miller(hipStream_t s, const u32 *lines, const uint8_t *ct_ok, const uint8_t *cts_u, u32 c0, u32 m, u32 *f_soa, uint8_t *status);
extern "C" void lcbk_tpke_pd_mul(hipStream_t s, const uint8_t *cts_u, const void *x_raw, u32 x_stride, u32 c0, u32 m, const uint8_t *status, uint8_t *ui_out);
extern "C" void lcbk_ts_rlc_sum_census(dim3 grid, hipStream_t s, const void *desc, u32 n_groups, u32 first, const uint8_t *msg_ok, const void *pks, u32 n_pks, const u32 *pk_idx, const uint8_t *sigs, const u32 *rP, const u32 *rS, u32 n, void *gpts, uint8_t *accept, uint8_t *gexact, u32 *wsum, const u32 *susp, uint8_t *cval);
extern "C" void lcbk_ts_rlc_sum2(hipStream_t s, const void *desc, u32 n_groups, u32 first, const uint8_t *msg_ok, const void *pks, u32 n_pks, const u32 *pk_idx, const uint8_t *sigs, const u32 *rP, const u32 *rS, u32 n, void *gpts, uint8_t *accept, uint8_t *gexact, u32 *wsum, const u32 *susp, uint8_t *cval);
extern "C" void lcbk_ts_rlc_miller_census(dim3 grid, hipStream_t s, const u32 *lines, const void *desc, const void *gpts, u32 n_groups, u32 *f_soa, uint8_t *gacc);
extern "C" void lcbk_coop_final_exp_check_2w(hipStream_t s, u32 *park, u32 n, uint8_t *accept);
extern "C" void lcbk_ts_msg_prepare(dim3 grid, hipStream_t s, const uint8_t *msg_data, const u32 *msg_off, u32 n_msgs, u32 *lines, uint8_t *msg_ok, int orig_cof);
extern "C" void lcbk_ts_miller(dim3 grid, hipStream_t s, const u32 *lines, const uint8_t *msg_ok, u32 n_msgs, const void *pks, u32 n_pks, const uint8_t *sigs, const u32 *msg_idx, const u32 *pk_idx, u32 n, u32 *f_soa, uint8_t *accept);
extern "C" void lcbk_coin_fold(dim3 grid, hipStream_t s, const uint8_t *sigs, u32 n, uint8_t *parity, uint64_t *nonce);
extern "C" void lcbk_select_first_valid(dim3 grid, hipStream_t s, const uint8_t *accept, const uint8_t *pts, u32 pbytes, u32 per_group, u32 k, u32 n_groups, uint8_t *xs, uint8_t *ys, u32 *off, const u32 *order, u32 *src);
// scalar-multiplication lanes (persistent grids, window tables in the workspace of lcbk_scalar_ws_bytes: 1 = G1, 2 = G2,
// 3 = TPKE encrypt phase 1)
extern "C" size_t lcbk_scalar_ws_bytes(int which, u32 n);
extern "C" void lcbk_g1_mul(hipStream_t s, const uint8_t *pts, int use_gen, const uint8_t *scalars, u32 n, uint8_t *out, uint8_t *ok_out, u32 *ws);
extern "C" void lcbk_g2_mul(hipStream_t s, const uint8_t *pts, int use_gen, const uint8_t *scalars, u32 n, uint8_t *out, uint8_t *ok_out, u32 *ws);
extern "C" void lcbk_g2_hash(dim3 grid, hipStream_t s, const uint8_t *msg_data, const u32 *msg_off, u32 n, uint8_t *out, uint8_t *ok_out, int orig_cof);
extern "C" void lcbk_tpke_encrypt1(hipStream_t s, const uint8_t *ybytes, const uint8_t *rs, u32 n, uint8_t *u_out, uint8_t *t_out, uint8_t *ok_out, u32 *ws);
extern "C" void lcbk_tpke_encrypt2(dim3 grid, hipStream_t s, const uint8_t *u, const uint8_t *rs, const uint8_t *v_data, const u32 *v_off, u32 n, uint8_t *w_out, uint8_t *ok_out, int orig_cof);
extern "C" void lcbk_ts_sign(dim3 grid, hipStream_t s, const uint8_t *sks, const uint8_t *msg_data, const u32 *msg_off, const u32 *msg_idx, u32 n, uint8_t *out, uint8_t *ok_out, int orig_cof);
extern "C" void lcbk_lagrange_coeffs(dim3 grid, hipStream_t s, const uint8_t *xs, const u32 *off, u32 n_problems, void *lam_raw, void *pre, uint8_t *status);
// Lagrange lanes (persistent grids, tables in the workspace `ws` of lcbk_lanes_ws_bytes: 1 = G1, 2 = G2, 3 = paired G2)
extern "C" size_t lcbk_lanes_ws_bytes(int which, u32 n_entries);
extern "C" void lcbk_g1_mul_lanes(hipStream_t s, const uint8_t *ys, const void *lam_raw, u32 n_entries, void *out, uint8_t *ok_out, u32 *ws);
extern "C" void lcbk_g2_mul_lanes(hipStream_t s, const uint8_t *ys, const void *lam_raw, u32 n_entries, void *out, uint8_t *ok_out, const void *dec, u32 n_dec, const u32 *src, u32 *ws);
// two entries per lane (n_entries even, problems at even offsets): shared doublings for two points of G2
extern "C" void lcbk_g2_mul2_lanes(hipStream_t s, const uint8_t *ys, const void *lam_raw, u32 n_entries, void *out, uint8_t *ok_out, const void *dec, u32 n_dec, const u32 *src, u32 *ws);
extern "C" void lcbk_g1_sum(dim3 grid, hipStream_t s, const void *parts, const uint8_t *ok_in, const u32 *off, u32 n_problems, uint8_t *status, uint8_t *out);
extern "C" void lcbk_g2_sum(dim3 grid, hipStream_t s, const void *parts, const uint8_t *ok_in, const u32 *off, u32 n_problems, uint8_t *status, uint8_t *out);
extern "C" void lcbk_msm_digits(dim3 grid, hipStream_t s, const uint8_t *scalars, u32 n, u32 c, u32 nwin, u32 *keys, u32 *vals);
extern "C" void lcbk_msm_bounds(dim3 grid, hipStream_t s, const u32 *keys, u32 m, u32 sentinel, u32 *start, u32 *end);
extern "C" void lcbk_msm_bucket_acc(dim3 grid, hipStream_t s, const void *pts, const void *pts2, u32 n_pts, const u32 *vals, const u32 *start, const u32 *end, u32 nb, void *buckets, u32 L, u32 n_seg);
// record-balanced bucket accumulation (K records per lane) and the fix-up of buckets spanning chunks
extern "C" void lcbk_msm_chunk_acc(hipStream_t s, const void *pts, const void *pts2, u32 n_pts, const u32 *keys, const u32 *vals, u32 m, u32 K, u32 sentinel, const u32 *start, const u32 *end, void *buckets, void *headp, void *tailp, u32 L, u32 n_seg);
extern "C" void lcbk_msm_bucket_fix(hipStream_t s, const u32 *start, const u32 *end, u32 K, const void *headp, const void *tailp, u32 nb, void *buckets, u32 L, u32 n_seg);
extern "C" void lcbk_msm_digits_glv(dim3 grid, hipStream_t s, const uint8_t *scalars, u32 n, u32 c, u32 nwin, u32 *keys, u32 *vals);
extern "C" void lcbk_msm_phi(dim3 grid, hipStream_t s, const void *pts, u32 n, void *out);
extern "C" void lcbk_msm_bucket_reduce(dim3 grid, hipStream_t s, const void *buckets, u32 half, u32 L, u32 n_seg, u32 hi_win, void *seg_out);
extern "C" void lcbk_g1_jac_reduce_groups(dim3 grid, hipStream_t s, const void *in, u32 n_in, u32 group, void *out);
extern "C" void lcbk_g1_jac_reduce_block(hipStream_t s, const void *in, u32 n_in, u32 group, void *out);
extern "C" void lcbk_msm_horner(hipStream_t s, const void *win, u32 nwin, u32 c, u32 fold_top, void *out);
extern "C" void lcbk_g1_jac_compress(dim3 grid, hipStream_t s, const void *in, u32 n, uint8_t *out);
extern "C" void lcbk_g1_to_affine(dim3 grid, hipStream_t s, const uint8_t *in, u32 n, void *out, uint8_t *ok);
extern "C" int lcbk_sort_pairs(void *temp, size_t *temp_bytes, u32 *keys, u32 *keys_alt, u32 *vals, u32 *vals_alt, u32 m, int end_bit, hipStream_t s);
extern "C" void lcbk_dkg_rows(dim3 grid, hipStream_t s, const void *coef, u32 n_coef, u32 n_comm, u32 D, const u32 *comm, const int *xs, u32 n_q, void *rows, uint8_t *ok_out);
extern "C" void lcbk_dkg_horner(dim3 grid, hipStream_t s, const void *rows, const uint8_t *row_ok, u32 D, const u32 *row, const int *ys, u32 n_q, uint8_t *out48, uint8_t *status, u32 neg_exact);
extern "C" void lcbk_and_groups(hipStream_t s, const uint8_t *in, u32 n_out, u32 group, uint8_t *out);
extern "C" void lcbk_g1_subgroup_any(hipStream_t s, const void *pts, u32 n, u32 *any);
extern "C" void lcbk_dkg_exact_terms(hipStream_t s, const void *coef, u32 n_coef, u32 n_comm, u32 D, const u32 *comm, const int *xs, u32 n_q, void *terms, uint8_t *ok_out);
extern "C" void lcbk_dkg_exact_combine(hipStream_t s, const void *rows, u32 D, const u32 *row, const int *ys, u32 n_q, void *terms);
extern "C" void lcbk_g1a_to_jac(dim3 grid, hipStream_t s, const void *in, u32 n, void *out, uint8_t *ok);
extern "C" const void *lcbk_rs_matrix_kernel();
extern "C" void lcbk_rs_matrix(hipStream_t s, const int *pe, int m, const int *pk, int k, int n, uint8_t *M, uint8_t *ok);
extern "C" void lcbk_rs_apply(hipStream_t s, const uint8_t *M, const uint8_t *ok, int m, int k, const uint8_t *src, size_t S, const int *pe, uint8_t *dst);
extern "C" size_t lcbk_secp_job_bytes(void);
extern "C" size_t lcbk_secp_table_bytes(void);
extern "C" size_t lcbk_secp_aff_bytes(void);
extern "C" void lcbk_secp_key_parse(hipStream_t s, const uint8_t *pks, u32 pk_len, u32 n_keys, void *out, u32 *ok);
extern "C" void lcbk_secp_comb_build(hipStream_t s, const void *base, const u32 *base_ok, u32 n_tables, void *tables, void *tmp);
extern "C" void lcbk_secp_header_hash(hipStream_t s, const uint8_t *hdr, u32 n, uint64_t era, uint8_t *hash, uint8_t *pre_ok);
extern "C" void lcbk_secp_scalars(hipStream_t s, const uint8_t *hashes, const uint8_t *sigs, u32 sig_len, u32 want_len, int chain_id, const int32_t *key_idx, u32 n_keys, const u32 *key_ok, const uint8_t *pre_ok, u32 n, void *jobs);
extern "C" void lcbk_secp_verify(hipStream_t s, const void *jobs, u32 n, const void *g_table, const void *key_tables, uint8_t *out);
extern "C" void lcbk_secp_gen(hipStream_t s, void *out, u32 *ok);
extern "C" void lcbk_secp_pubkey(hipStream_t s, const uint8_t *privs, u32 n, const void *g_table, uint8_t *out33, uint8_t *ok);
extern "C" void lcbk_secp_sign(hipStream_t s, const uint8_t *hashes, const uint8_t *privs, const uint8_t *nonces, u32 n, const void *g_table, int chain_id, int use_new, uint8_t *out, uint8_t *ok);
extern "C" size_t lcbk_key_table_bytes(u32 n_keys);
extern "C" void lcbk_rlc_key_tables(dim3 grid, hipStream_t s, const void *keys, u32 n_keys, u32 *ws, u32 **tab, uint8_t **ktab_ok);
extern "C" void lcbk_tpke_rlc_points(hipStream_t s, u32 n_cts, const void *keys, u32 n_keys, const u32 *ct_idx, const u32 *dec_idx, const uint8_t *ui, u32 i0, u32 n, const u32 key[10], u32 *rU, u32 *rY, uint8_t *accept, const u32 *ktab, const uint8_t *ktab_ok, const u32 *susp);
extern "C" void lcbk_ts_rlc_points(hipStream_t s, u32 n_msgs, const void *pks, u32 n_pks, const u32 *msg_idx, const u32 *pk_idx, const uint8_t *sigs, u32 i0, u32 n, const u32 key[10], u32 *rP, u32 *rS, uint8_t *accept, void *desc, u32 *count, const u32 *ktab, const uint8_t *ktab_ok, const u32 *susp, void *dec);
extern "C" void lcbk_rlc_groups(hipStream_t s, const u32 *key_idx, u32 i0, u32 n, u32 n_keys, u32 cap, void *desc, u32 *count);
extern "C" void lcbk_tpke_rlc_sum(dim3 grid, hipStream_t s, const void *desc, u32 n_groups, u32 lanes, const uint8_t *ct_ok, const uint8_t *ct_g2, const void *keys, u32 n_keys, const u32 *dec_idx, const uint8_t *ui, const u32 *rU, const u32 *rY, u32 n, void *gpts, uint8_t *accept, uint8_t *gexact, u32 *wsum, const u32 *susp, uint8_t *cval);
extern "C" void lcbk_tpke_rlc_wsum(dim3 grid, hipStream_t s, const void *sdesc, u32 n_s, const u32 *wsum, u32 n_l1, void *gpts);
extern "C" void lcbk_tpke_rlc_miller(dim3 grid, hipStream_t s, const u32 *lines, const void *desc, const void *gpts, u32 n_groups, u32 *f_soa, uint8_t *gacc);
extern "C" void lcbk_ts_rlc_sum(dim3 grid, hipStream_t s, const void *desc, u32 n_groups, u32 first, const uint8_t *msg_ok, const void *pks, u32 n_pks, const u32 *pk_idx, const uint8_t *sigs, const u32 *rP, const u32 *rS, u32 n, void *gpts, uint8_t *accept, uint8_t *gexact, u32 *wsum, const u32 *susp, uint8_t *cval);
extern "C" void lcbk_ts_rlc_wsum(dim3 grid, hipStream_t s, const void *sdesc, u32 n_s, const u32 *wsum, u32 n_l1, void *gpts);
extern "C" void lcbk_ts_rlc_miller(dim3 grid, hipStream_t s, const u32 *lines, const void *desc, const void *gpts, u32 n_groups, u32 *f_soa, uint8_t *gacc);
extern "C" void lcbk_rlc_resolve(dim3 grid, hipStream_t s, const void *desc, u32 o, u32 m, const uint8_t *gacc, const uint8_t *gexact, const u32 *park, u32 first, uint8_t *accept, void *next, u32 *next_count, void *search, u32 *search_count, u32 *gamma, const u32 *key_idx, u32 n_keys, const u32 *susp);
extern "C" void lcbk_tpke_rlc_wsum2(hipStream_t s, const void *sdesc, u32 ns, const u32 *open, const u32 *rU, const u32 *rY, u32 n, const u32 *dec_idx, u32 n_keys, const u32 *susp, void *gpts, void *sdesc_out);
extern "C" void lcbk_rlc_park_copy(hipStream_t s, const u32 *park, u32 o, u32 m, u32 *dst, const u32 *map);
extern "C" void lcbk_tpke_rlc_search2a(hipStream_t s, const void *search, u32 ns, const u32 *gamma0, const u32 *gamma12, uint8_t *accept, u32 *open, u32 *open_count);
extern "C" int lcbk_search2b_by_position(void);
extern "C" int lcbk_search2b_debug(void *p);
extern "C" void lcbk_tpke_rlc_search2b(hipStream_t s, const void *search, u32 ns, u32 n_open, const u32 *gamma0, const u32 *gamma12, const u32 *open, const u32 *open_count, uint8_t *accept, void *next, u32 *next_count, const u32 *key_idx, u32 n_keys, const u32 *susp);
extern "C" void lcbk_tpke_rlc_search2b_asm(hipStream_t s, const void *search, u32 ns, u32 n_open, const u32 *gamma0, const u32 *gamma12, const u32 *open, const u32 *open_count, uint8_t *accept, void *next, u32 *next_count, const u32 *key_idx, u32 n_keys, const u32 *susp, u32 *park);
extern "C" size_t lcbk_tpke_rlc_search2b_asm_park_bytes(u32 n_open);
extern "C" void lcbk_rlc_search(dim3 grid, hipStream_t s, const void *search, u32 o, u32 m, const u32 *gamma, const u32 *park, uint8_t *accept, void *next, u32 *next_count, const u32 *key_idx, u32 n_keys, const u32 *susp);
extern "C" void lcbk_rlc_census_desc(hipStream_t s, const u32 *grp_idx, const u32 *key_idx, u32 m, u32 n_grp, u32 n_keys, void *desc, uint8_t *accept);
extern "C" void lcbk_rlc_census_stats(hipStream_t s, const u32 *key_idx, u32 m, u32 n_keys, const uint8_t *cval, const uint8_t *accept, u32 *susp, u32 *count);
extern "C" void lcbk_rlc_suspect_split(hipStream_t s, const void *desc, u32 n_groups, const u32 *key_idx, u32 n_keys, const u32 *susp, const uint8_t *accept, void *out, u32 *count);
extern "C" size_t lcbk_ts_grp_bytes();
extern "C" void lcbk_coop_tpke_miller(hipStream_t s, const u32 *lines, const void *desc, const void *gpts, u32 n_groups, u32 *f_soa, uint8_t *gacc, uint8_t *fb, u32 npairs, int fallback);
// *flag |= 1 when a line set of ciphertexts [c0, c1) is not normalised
extern "C" void lcbk_lines_unnormalised(hipStream_t s, const u32 *lines, u32 c0, u32 c1, u32 *flag);
extern "C" size_t lcbk_mcl_terms_ws_bytes(u32 n);
extern "C" void lcbk_mcl_g1_terms(hipStream_t s, const void *pts, const void *scal, u32 n, void *terms, u32 *ws);
extern "C" size_t lcbk_mcl_terms_wide_ws_bytes(u32 n);
extern "C" void lcbk_mcl_g1_terms_wide(hipStream_t s, const void *pts, const u32 *scal, u32 n, void *terms, u32 *ws);
extern "C" void lcbk_mcl_horner(hipStream_t s, int g, const u32 *coef, u32 n, const void *x_raw, u32 *out);
extern "C" void lcbk_mcl_g1_sum(hipStream_t s, const void *in, u32 n, void *out);
extern "C" void lcbk_mcl_from_bytes(hipStream_t s, int g, const uint8_t *in, u32 n, u32 *out, uint8_t *ok);
extern "C" void lcbk_mcl_to_bytes(hipStream_t s, int g, const u32 *in, u32 n, uint8_t *out);
extern "C" void lcbk_tpke_exact_points(hipStream_t s, const uint8_t *ct_ok, u32 n_cts, const void *keys, u32 n_keys, const u32 *ct_idx, const u32 *dec_idx, const uint8_t *ui, u32 n, void *gpts, void *desc, uint8_t *accept);
extern "C" void lcbk_coop_debug(hipStream_t s, int op, u32 *ws, const u32 *b_soa, u32 n, u32 *out, u32 *ref);
extern "C" void lcbk_coop_final_exp_check(hipStream_t s, u32 *park, u32 n, uint8_t *accept);
extern "C" void lcbk_op(dim3 grid, hipStream_t s, int op, u32 *io, int orig_cof);

// sizes of the device records the host allocates
#define LCB_G1A_ST_BYTES 112
#define LCB_G2A_ST_BYTES 208
#define LCB_FR_BYTES 32
#define LCB_G1_JAC_BYTES 144
#define LCB_G2_JAC_BYTES 288
#define LCB_LINESET_BYTES 26368   /* pairing.hpp LCB_LINESET_WORDS * 4 */
#define LCB_LS_POINT_WORD 6528    /* pairing.hpp LCB_LS_POINT: the set's affine point (48 words), then LCB_LS_FLAG */
extern "C" int lcbk_cfg_k_batch(u32 sign_b);
extern "C" int lcbk_cfg_k_coop(u32 sign_b);
extern "C" int lcbk_cfg_k_dkg(u32 sign_b);
extern "C" int lcbk_cfg_k_lagrange(u32 sign_b);
extern "C" int lcbk_cfg_k_mcl(u32 sign_b);
extern "C" int lcbk_cfg_k_msm(u32 sign_b);
extern "C" int lcbk_cfg_k_ops(u32 sign_b);
extern "C" int lcbk_cfg_k_rlc_rand(u32 sign_b);
extern "C" int lcbk_cfg_k_scalar(u32 sign_b);
extern "C" int lcbk_cfg_k_tpke(u32 sign_b);
extern "C" int lcbk_cfg_k_ts(u32 sign_b);
extern "C" int lcbk_cfg_k_ptmul(u32 sign_b);
extern "C" int lcbk_cfg_k_prep(u32 sign_b);
// cooperative single scalar multiplications (k_ptmul.hip): n_groups ladders of one wave
extern "C" void lcbk_ptmul_g1(hipStream_t s, const void *jobs, u32 n_groups, void *out);
extern "C" void lcbk_ptmul_g1_multi(hipStream_t s, const void *jobs, u32 n_groups, void *out);
extern "C" void lcbk_ptmul_g2_multi(hipStream_t s, const void *jobs, u32 n_groups, void *out);
extern "C" void lcbk_ptmul_g2(hipStream_t s, const void *jobs, u32 n_groups, void *out);
extern "C" int lcbk_prio_k_batch(u32 on);
extern "C" int lcbk_prio_k_coop(u32 on);
extern "C" int lcbk_prio_k_dkg(u32 on);
extern "C" int lcbk_prio_k_lagrange(u32 on);
extern "C" int lcbk_prio_k_mcl(u32 on);
extern "C" int lcbk_prio_k_msm(u32 on);
extern "C" int lcbk_prio_k_ops(u32 on);
extern "C" int lcbk_prio_k_rlc_rand(u32 on);
extern "C" int lcbk_prio_k_scalar(u32 on);
extern "C" int lcbk_prio_k_tpke(u32 on);
extern "C" int lcbk_prio_k_ts(u32 on);
extern "C" int lcbk_prio_k_ptmul(u32 on);
extern "C" int lcbk_prio_k_prep(u32 on);
static inline int lcbk_set_wave_prio(int on) {
    int rc = 0;
    rc |= lcbk_prio_k_batch((u32)on);
    rc |= lcbk_prio_k_coop((u32)on);
    rc |= lcbk_prio_k_dkg((u32)on);
    rc |= lcbk_prio_k_lagrange((u32)on);
    rc |= lcbk_prio_k_mcl((u32)on);
    rc |= lcbk_prio_k_msm((u32)on);
    rc |= lcbk_prio_k_ops((u32)on);
    rc |= lcbk_prio_k_rlc_rand((u32)on);
    rc |= lcbk_prio_k_scalar((u32)on);
    rc |= lcbk_prio_k_tpke((u32)on);
    rc |= lcbk_prio_k_ts((u32)on);
    rc |= lcbk_prio_k_ptmul((u32)on);
    rc |= lcbk_prio_k_prep((u32)on);
    return rc;
}
// every kernel unit's G2 sign-flag convention (curve.hpp lcb_g2_sign_b)
static inline int lcbk_set_g2_sign_b(int sign_b) {
    int rc = 0;
    rc |= lcbk_cfg_k_batch((u32)sign_b);
    rc |= lcbk_cfg_k_coop((u32)sign_b);
    rc |= lcbk_cfg_k_dkg((u32)sign_b);
    rc |= lcbk_cfg_k_lagrange((u32)sign_b);
    rc |= lcbk_cfg_k_mcl((u32)sign_b);
    rc |= lcbk_cfg_k_msm((u32)sign_b);
    rc |= lcbk_cfg_k_ops((u32)sign_b);
    rc |= lcbk_cfg_k_rlc_rand((u32)sign_b);
    rc |= lcbk_cfg_k_scalar((u32)sign_b);
    rc |= lcbk_cfg_k_tpke((u32)sign_b);
    rc |= lcbk_cfg_k_ts((u32)sign_b);
    rc |= lcbk_cfg_k_ptmul((u32)sign_b);
    rc |= lcbk_cfg_k_prep((u32)sign_b);
    return rc;
}
