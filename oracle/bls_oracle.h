/*
 * oracle/bls_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the BLS12-381 arithmetic that Lachain's hot path reaches through
 * MCL.BLS12_381.Net 0.0.4 / MCL.BLS12_381.Native 0.0.5 (herumi mcl; third-party, not vendored in
 * /root/reference, see /root/reference/src/Lachain.Crypto/Lachain.Crypto.csproj:18-19), plus the
 * Lachain.Crypto protocol functions that orchestrate it (TPKE/ and ThresholdSignature/ sources).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and only
 * as the checker / the timed CPU baseline — never as the product path (lachain_amd/ is the product).
 *
 * Parity pinning: serialization, generators and G1/G2 doubling are pinned by
 * test/Lachain.CryptoTest/SerializationTest.cs:20-57; the TPKE KDF by CryptographyTest.cs:103-113.
 * hash-to-G2 (mcl "ORIGINAL" map), the G2 compressed sign bit and GT normalisation are restated from
 * the mcl algorithm and are UNPINNED by any reference vector.
 *
 * All multi-byte encodings are MCL serialize format: Fr 32 B LE, G1 48 B, G2 96 B (x.a || x.b),
 * bit 7 of the last byte = "y is odd" flag, all-zero = point at infinity.
 */
#ifndef LACHAIN_BLS_ORACLE_H
#define LACHAIN_BLS_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define ORC_FR_BYTES 32
#define ORC_G1_BYTES 48
#define ORC_G2_BYTES 96
#define ORC_GT_BYTES 576

void orc_init(void);

/* configuration switches for the unpinned mcl choices (defaults = best-known mcl behaviour) */
void orc_set_g2_sign_from_b(int use_b);        /* 0: flag = parity(y.a) (default), 1: parity(y.b) */
void orc_set_g2_original_cofactor(int enable); /* 0: Budroni-Pintore h_eff (default), 1: h2       */

/* Fp-mul instrumentation (counts fp_mul + fp_sqr calls, single-threaded use only) */
void orc_count_reset(void);
uint64_t orc_count_get(void);

/* ---- Fr ---- */
int orc_fr_from_int(uint8_t out[32], int64_t v);
int orc_fr_is_canonical(const uint8_t a[32]);
int orc_fr_add(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]);
int orc_fr_sub(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]);
int orc_fr_mul(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]);
int orc_fr_inv(uint8_t out[32], const uint8_t a[32]);
/* 64-byte wide reduction mod r (used by the synthetic-input DRBG) */
void orc_fr_from_wide(uint8_t out[32], const uint8_t in[64]);

/* ---- G1 / G2 (serialized in / out) ---- */
void orc_g1_generator(uint8_t out[48]);
void orc_g2_generator(uint8_t out[96]);
int orc_g1_is_valid_encoding(const uint8_t a[48]); /* 1 ok, 0 rejected */
int orc_g2_is_valid_encoding(const uint8_t a[96]);
int orc_g1_in_subgroup(const uint8_t a[48]);
int orc_g2_in_subgroup(const uint8_t a[96]);
int orc_g1_add(uint8_t out[48], const uint8_t a[48], const uint8_t b[48]);
int orc_g2_add(uint8_t out[96], const uint8_t a[96], const uint8_t b[96]);
int orc_g1_neg(uint8_t out[48], const uint8_t a[48]);
int orc_g2_neg(uint8_t out[96], const uint8_t a[96]);
int orc_g1_mul(uint8_t out[48], const uint8_t a[48], const uint8_t s[32]);
int orc_g2_mul(uint8_t out[96], const uint8_t a[96], const uint8_t s[32]);
int orc_g2_hash(uint8_t out[96], const uint8_t *msg, size_t len);      /* G2.SetHashOf */
int orc_g1_lagrange(uint8_t out[48], const uint8_t *xs, const uint8_t *ys, size_t k);
int orc_g2_lagrange(uint8_t out[96], const uint8_t *xs, const uint8_t *ys, size_t k);
int orc_fr_lagrange(uint8_t out[32], const uint8_t *xs, const uint8_t *ys, size_t k);
int orc_fr_eval_poly(uint8_t out[32], const uint8_t *coeffs, size_t n, const uint8_t x[32]);
int orc_ts_validate_batch(uint8_t *accept, size_t n, const uint8_t *pks, const uint8_t *sigs, const uint8_t *msgs,
                          const uint32_t *msg_off, const uint32_t *msg_idx, const uint32_t *pk_idx, int nthreads);
int orc_g1_msm_mt(uint8_t out[48], const uint8_t *pts, const uint8_t *scalars, size_t n, int nthreads);
int orc_g1_msm(uint8_t out[48], const uint8_t *pts, const uint8_t *scalars, size_t n);

/* ---- GT / pairing (GT = 12 Fp, canonical big-endian-free LE layout) ---- */
int orc_pairing(uint8_t out[576], const uint8_t p[48], const uint8_t q[96]);
int orc_pairing_slow(uint8_t out[576], const uint8_t p[48], const uint8_t q[96]); /* affine + direct FE */
int orc_gt_pow(uint8_t out[576], const uint8_t a[576], const uint8_t s[32]);
int orc_gt_mul(uint8_t out[576], const uint8_t a[576], const uint8_t b[576]);
int orc_gt_is_one(const uint8_t a[576]);
int orc_miller_loop(uint8_t out[576], const uint8_t p[48], const uint8_t q[96]);
int orc_final_exp(uint8_t out[576], const uint8_t f[576]);
int orc_final_exp_direct(uint8_t out[576], const uint8_t f[576]);

/* ---- hashing / KDF ---- */
void orc_sha512(uint8_t out[64], const uint8_t *m, size_t n);
void orc_sha256(uint8_t out[32], const uint8_t *m, size_t n);
void orc_sha3_256(uint8_t out[32], const uint8_t *m, size_t n);
/* TPKE Utils.XorWithHash: BouncyCastle DigestRandomGenerator(Sha3Digest) keystream XOR */
void orc_xor_with_hash(uint8_t *out, const uint8_t g1[48], const uint8_t *data, size_t len);
/* CoinResult.Parity / RootProtocol.GetNonceFromCoin over serialized signature bytes */
int orc_coin_parity(const uint8_t *bytes, size_t len);
uint64_t orc_coin_nonce(const uint8_t *bytes, size_t len);

/* ---- Lachain.Crypto protocol restatements ---- */
/* TPKE.PublicKey.Encrypt with caller-supplied r (TPKE/PublicKey.cs:25-37) */
int orc_tpke_encrypt(uint8_t u[48], uint8_t *v, uint8_t w[96], const uint8_t y[48],
                     const uint8_t *data, size_t len, const uint8_t r[32]);
/* TPKE.PrivateKey.Decrypt (TPKE/PrivateKey.cs:21-31): 0 ok, -1 "Invalid share!" */
int orc_tpke_decrypt(uint8_t ui[48], const uint8_t u[48], const uint8_t *v, size_t vlen,
                     const uint8_t w[96], const uint8_t x[32]);
/* TPKE.PublicKey.VerifyShare (TPKE/PublicKey.cs:88-92): 1 accept, 0 reject, -1 decode error */
int orc_tpke_verify_share(const uint8_t y_i[48], const uint8_t u[48], const uint8_t *v, size_t vlen,
                          const uint8_t w[96], const uint8_t ui[48]);
/* TPKE.PublicKey.FullDecrypt Lagrange + KDF part (TPKE/PublicKey.cs:74-84) */
int orc_tpke_full_decrypt(uint8_t *out, const uint8_t *v, size_t vlen, const int32_t *decryptor_ids,
                          const uint8_t *uis, size_t k);
/* ThresholdSignature.PublicKey.ValidateSignature (ThresholdSignature/PublicKey.cs:16-21) */
int orc_ts_validate(const uint8_t pk[48], const uint8_t sig[96], const uint8_t *msg, size_t len);
/* PrivateKeyShare.HashAndSign (ThresholdSignature/PrivateKeyShare.cs:21-27) */
int orc_ts_sign(uint8_t sig[96], const uint8_t sk[32], const uint8_t *msg, size_t len);

/* ---- batch (CPU-baseline) entry points, OpenMP over items ---- */
/* per share i: ct index ct_idx[i], decryptor dec_idx[i]; as-reference semantics
   (hash recomputed per share, two separate pairings compared) */
/* reliable-broadcast Reed-Solomon erasure coding (rs.c) */
int orc_rs_encode_codeword(int *cw, int n, int ecc);
int orc_rs_decode_erasures(int *cw, int n, int ecc, const int *pos, int m);
int orc_rs_encode_shards(uint8_t *out, const uint8_t *input, size_t len, int shards, int erasures);
int orc_rs_decode_shards(uint8_t *out, const uint8_t *echo_data, const int32_t *from, int n_echos, size_t S, int shards,
                         int erasures);
/* trustless DKG: Commitment.Evaluate(x, y) / Evaluate(x) as the reference writes them, G1 polynomial evaluation */
int orc_dkg_commitment_eval(uint8_t out[48], const uint8_t *coeffs, int D, int32_t x, int32_t y);
int orc_dkg_commitment_row(uint8_t *out, const uint8_t *coeffs, int D, int32_t x);
int orc_g1_eval_poly(uint8_t out[48], const uint8_t *coeffs, size_t n, const uint8_t x[32]);
/* CPU baseline with the GPU's algorithm (per-ciphertext / per-message H and Miller lines, one final exp per
   share): bench.py's "amortized" cpu_baseline legs */
int orc_tpke_verify_batch_amortized(uint8_t *accept, size_t n, const uint8_t *y_keys, size_t n_keys,
                                    const uint8_t *cts_u, const uint8_t *cts_v, size_t vlen, const uint8_t *cts_w,
                                    size_t n_cts, const uint32_t *ct_idx, const uint32_t *dec_idx, const uint8_t *uis,
                                    int nthreads);
int orc_ts_validate_batch_amortized(uint8_t *accept, size_t n, const uint8_t *pks, size_t n_pks, const uint8_t *sigs,
                                    const uint8_t *msgs, const uint32_t *msg_off, size_t n_msgs,
                                    const uint32_t *msg_idx, const uint32_t *pk_idx, int nthreads);
/* CPU baseline with the GPU's randomized batch algorithm (k_batch.hip): bench.py's batched cpu_baseline leg */
int orc_tpke_verify_batch_rlc(uint8_t *accept, size_t n, const uint8_t *y_keys, size_t n_keys, const uint8_t *cts_u,
                              const uint8_t *cts_v, size_t vlen, const uint8_t *cts_w, size_t n_cts,
                              const uint32_t *ct_idx, const uint32_t *dec_idx, const uint8_t *uis, uint64_t seed,
                              int nthreads);
int orc_ts_validate_batch_rlc(uint8_t *accept, size_t n, const uint8_t *pks, size_t n_pks, const uint8_t *sigs,
                              const uint8_t *msgs, const uint32_t *msg_off, size_t n_msgs, const uint32_t *msg_idx,
                              const uint32_t *pk_idx, uint64_t seed, int nthreads);
int orc_g2_in_subgroup_psi(const uint8_t a[96]);
int orc_tpke_verify_batch(uint8_t *accept, size_t n_shares, const uint8_t *y_keys,
                          const uint8_t *cts_u, const uint8_t *cts_v, size_t vlen, const uint8_t *cts_w,
                          const uint32_t *ct_idx, const uint32_t *dec_idx, const uint8_t *uis,
                          int nthreads);

#ifdef __cplusplus
}
#endif
#endif
