/*
 * include/lachain_bls.h — C ABI of liblachain_bls.so, the MI355X (gfx950) replacement for the native
 * BLS12-381 library behind Lachain's threshold-crypto hot path.
 *
 * Boundary being replaced: Lachain.Crypto (C#) P/Invokes herumi mcl through the NuGet packages
 * MCL.BLS12_381.Net 0.0.4 / MCL.BLS12_381.Native 0.0.5
 * (/root/reference/src/Lachain.Crypto/Lachain.Crypto.csproj:18-19).  That wrapper's sources are not in
 * the reference tree; the export set below is mcl's public C API (mcl/bn.h, mclbn384_256 build) as
 * inferred from the managed call sites (census in SURVEY.md §8b), so the managed wrapper can be
 * re-pointed at this library by changing its DllImport name.  Every function cites the Lachain call
 * site(s) it serves.  The lcb_* functions are the batch entry points the consensus layer (or a shim,
 * INTEGRATION.md) calls with whole batches of shares.
 *
 * Data layouts: the in-memory structs are byte-compatible with mcl's: Montgomery form, 64-bit limbs
 * little-endian (Fr: R = 2^256, Fp: R = 2^384), G1/G2 Jacobian (x, y, z), GT = Fp12 as 12 Fp.
 * All-zero bytes = zero / point at infinity.  Serialized sizes: Fr 32 B, G1 48 B, G2 96 B, GT 576 B
 * (mcl serialize format; pinned by test/Lachain.CryptoTest/SerializationTest.cs).
 *
 * Errors never cross the ABI as exceptions: int functions return 0 on success and -1 on failure,
 * (de)serializers return the number of bytes written/read or 0.  All arithmetic runs on the GPU; if no
 * gfx950 device can be opened, mclBn_init returns -1 and every other call fails loudly (there is no
 * CPU fallback).
 *
 * Threading (callers: one thread per consensus protocol, src/Lachain.Consensus/AbstractProtocol.cs:46-47):
 * every entry point may be called concurrently from any number of threads.  Single-element mcl operations are
 * synchronous and serialized by an internal lock.  Batch calls run in an execution context (lcb_ctx) that owns
 * their device workspaces: the lcb_ctx_* forms take one explicitly, the other forms use the calling thread's
 * own implicit context (one for the *_dev entry points, another for the synchronous host-pointer ones).  Work
 * of one context runs in the order it was enqueued whatever stream it is enqueued on, TPKE and threshold-
 * signature workspaces are separate, and a *_prepared call fails unless its batch shape is the one prepared
 * in the same context.  lcb_set_device applies to every calling thread.
 */
#ifndef LACHAIN_BLS_H
#define LACHAIN_BLS_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define MCL_BLS12_381 5
#define MCLBN_COMPILED_TIME_VAR 46 /* mclbn384_256: (MCLBN_FP_UNIT_SIZE * 10 + MCLBN_FR_UNIT_SIZE) */

typedef int64_t mclInt;
typedef size_t mclSize;
typedef struct { uint64_t d[4]; } mclBnFr;
typedef struct { uint64_t d[6]; } mclBnFp;
typedef struct { mclBnFp d[2]; } mclBnFp2;
typedef struct { mclBnFp x, y, z; } mclBnG1;
typedef struct { mclBnFp2 x, y, z; } mclBnG2;
typedef struct { mclBnFp d[12]; } mclBnGT;

/* ------------------------------------------------------------------ init / sizes
   Mcl.Init / static constructor of the managed wrapper (dead test/ToolsTest.cs:18 shows `Mcl.Init()`) */
int mclBn_init(int curve, int compiledTimeVar);
int mclBn_getOpUnitSize(void);
int mclBn_getG1ByteSize(void); /* G1.ByteSize = 48 (src/Lachain.Utility/Serialization/SerialiaztionUtils.cs:24-26) */
int mclBn_getFrByteSize(void); /* Fr.ByteSize = 32 */
int mclBn_getFpByteSize(void);

/* ------------------------------------------------------------------ Fr
   Fr.FromInt (23 call sites, e.g. TPKE/PublicKey.cs:79), Fr.GetRandom (TPKE/PublicKey.cs:29),
   Fr.FromBytes / ToBytes (ThresholdSignature/PrivateKeyShare.cs:31), operators + * (MclTests.cs:57) */
int mclBnFr_setInt(mclBnFr *y, mclInt x);
int mclBnFr_setInt32(mclBnFr *y, int x);
int mclBnFr_setByCSPRNG(mclBnFr *x);
int mclBnFr_setLittleEndian(mclBnFr *x, const void *buf, mclSize bufSize);
mclSize mclBnFr_serialize(void *buf, mclSize maxBufSize, const mclBnFr *x);
mclSize mclBnFr_deserialize(mclBnFr *x, const void *buf, mclSize bufSize);
void mclBnFr_clear(mclBnFr *x);
int mclBnFr_isValid(const mclBnFr *x);
int mclBnFr_isEqual(const mclBnFr *x, const mclBnFr *y);
int mclBnFr_isZero(const mclBnFr *x);
int mclBnFr_isOne(const mclBnFr *x);
void mclBnFr_neg(mclBnFr *y, const mclBnFr *x);
void mclBnFr_inv(mclBnFr *y, const mclBnFr *x);
void mclBnFr_sqr(mclBnFr *y, const mclBnFr *x);
void mclBnFr_add(mclBnFr *z, const mclBnFr *x, const mclBnFr *y);
void mclBnFr_sub(mclBnFr *z, const mclBnFr *x, const mclBnFr *y);
void mclBnFr_mul(mclBnFr *z, const mclBnFr *x, const mclBnFr *y);
void mclBnFr_div(mclBnFr *z, const mclBnFr *x, const mclBnFr *y);

/* ------------------------------------------------------------------ G1
   G1.Generator (24 sites), G1.FromBytes (HoneyBadger decode, TPKE/PublicKey.cs:41), G1 * Fr
   (TPKE/PublicKey.cs:30-32, TPKE/PrivateKey.cs:28), G1 + G1 (MclTests.cs:59), IsValid
   (ThresholdKeygen/Data/Commitment.cs:78) */
mclSize mclBnG1_serialize(void *buf, mclSize maxBufSize, const mclBnG1 *x);
mclSize mclBnG1_deserialize(mclBnG1 *x, const void *buf, mclSize bufSize);
int mclBnG1_isValid(const mclBnG1 *x);
int mclBnG1_isEqual(const mclBnG1 *x, const mclBnG1 *y);
int mclBnG1_isZero(const mclBnG1 *x);
void mclBnG1_clear(mclBnG1 *x);
void mclBnG1_neg(mclBnG1 *y, const mclBnG1 *x);
void mclBnG1_dbl(mclBnG1 *y, const mclBnG1 *x);
void mclBnG1_normalize(mclBnG1 *y, const mclBnG1 *x);
void mclBnG1_add(mclBnG1 *z, const mclBnG1 *x, const mclBnG1 *y);
void mclBnG1_sub(mclBnG1 *z, const mclBnG1 *x, const mclBnG1 *y);
void mclBnG1_mul(mclBnG1 *z, const mclBnG1 *x, const mclBnFr *y);
void mclBnG1_mulVec(mclBnG1 *z, const mclBnG1 *x, const mclBnFr *y, mclSize n);
/* convenience (not in mcl): the Lachain G1 generator (SerializationTest.cs:36) */
void lcb_g1_generator(mclBnG1 *g);

/* ------------------------------------------------------------------ G2
   G2.Generator, G2.FromBytes (ThresholdSignature/Signature.cs:38), G2.SetHashOf
   (TPKE/Utils.cs:24-25, ThresholdSignature/PublicKey.cs:19, PrivateKeyShare.cs:24), G2 * Fr
   (TPKE/PublicKey.cs:34, PrivateKeyShare.cs:25) */
mclSize mclBnG2_serialize(void *buf, mclSize maxBufSize, const mclBnG2 *x);
mclSize mclBnG2_deserialize(mclBnG2 *x, const void *buf, mclSize bufSize);
int mclBnG2_isValid(const mclBnG2 *x);
int mclBnG2_isEqual(const mclBnG2 *x, const mclBnG2 *y);
int mclBnG2_isZero(const mclBnG2 *x);
void mclBnG2_clear(mclBnG2 *x);
int mclBnG2_hashAndMapTo(mclBnG2 *x, const void *buf, mclSize bufSize);
void mclBnG2_neg(mclBnG2 *y, const mclBnG2 *x);
void mclBnG2_dbl(mclBnG2 *y, const mclBnG2 *x);
void mclBnG2_normalize(mclBnG2 *y, const mclBnG2 *x);
void mclBnG2_add(mclBnG2 *z, const mclBnG2 *x, const mclBnG2 *y);
void mclBnG2_sub(mclBnG2 *z, const mclBnG2 *x, const mclBnG2 *y);
void mclBnG2_mul(mclBnG2 *z, const mclBnG2 *x, const mclBnFr *y);
void lcb_g2_generator(mclBnG2 *g);

/* ------------------------------------------------------------------ GT / pairing
   GT.Pairing (8 sites: TPKE/PrivateKey.cs:26, TPKE/PublicKey.cs:91, ThresholdSignature/PublicKey.cs:20),
   GT.Equals, GT.Pow (MclTests.cs:73) */
void mclBn_pairing(mclBnGT *z, const mclBnG1 *x, const mclBnG2 *y);
void mclBn_millerLoop(mclBnGT *z, const mclBnG1 *x, const mclBnG2 *y);
void mclBn_millerLoopVec(mclBnGT *z, const mclBnG1 *x, const mclBnG2 *y, mclSize n);
void mclBn_finalExp(mclBnGT *y, const mclBnGT *x);
int mclBnGT_isEqual(const mclBnGT *x, const mclBnGT *y);
int mclBnGT_isOne(const mclBnGT *x);
int mclBnGT_isZero(const mclBnGT *x);
void mclBnGT_clear(mclBnGT *x);
void mclBnGT_mul(mclBnGT *z, const mclBnGT *x, const mclBnGT *y);
void mclBnGT_pow(mclBnGT *z, const mclBnGT *x, const mclBnFr *y);
mclSize mclBnGT_serialize(void *buf, mclSize maxBufSize, const mclBnGT *x);
mclSize mclBnGT_deserialize(mclBnGT *x, const void *buf, mclSize bufSize);

/* ------------------------------------------------------------------ polynomials / Lagrange
   MclBls12381.LagrangeInterpolate (TPKE/PublicKey.cs:83, ThresholdSignature/PublicKeySet.cs:31,41,
   ThresholdKeygen/Data/State.cs:43), MclBls12381.EvaluatePolynomial (TPKE/TrustedKeyGen.cs:23-33) */
int mclBn_FrLagrangeInterpolation(mclBnFr *out, const mclBnFr *xVec, const mclBnFr *yVec, mclSize k);
int mclBn_G1LagrangeInterpolation(mclBnG1 *out, const mclBnFr *xVec, const mclBnG1 *yVec, mclSize k);
int mclBn_G2LagrangeInterpolation(mclBnG2 *out, const mclBnFr *xVec, const mclBnG2 *yVec, mclSize k);
int mclBn_FrEvaluatePolynomial(mclBnFr *out, const mclBnFr *cVec, mclSize cSize, const mclBnFr *x);
int mclBn_G1EvaluatePolynomial(mclBnG1 *out, const mclBnG1 *cVec, mclSize cSize, const mclBnFr *x);
int mclBn_G2EvaluatePolynomial(mclBnG2 *out, const mclBnG2 *cVec, mclSize cSize, const mclBnFr *x);

/* ================================================================== batch entry points (new)
   Host-pointer forms copy to/from the GPU; *_dev forms take device pointers and a hipStream_t (as void*)
   and enqueue without synchronizing.  All serialized inputs use the 48/96-byte wire formats. */

/* library configuration */
int lcb_set_device(int device_id);                 /* before mclBn_init; default: HIP device 0 */
int lcb_get_device(void);
void lcb_set_original_g2_cofactor(int enable);     /* unpinned mcl choice, DESIGN.md §Parity */
/* unpinned mcl convention: the G2 wire flag (bit 7 of byte 95) is the parity of y.a (use_b = 0, the
   default) or of y.b (use_b = 1), for every G2 (de)serialization — the mcl surface and every batch kernel alike.
   Mirrors the oracle's orc_set_g2_sign_from_b (oracle/bls.c:517-521,691).  Call before batch work, not during it.
   Returns -1 without a device. */
int lcb_set_g2_sign_from_b(int use_b);
/* Line sets prepared for TPKE ciphertexts / signed messages are normalised (A = 1) unless a line has A == 0, in
   which case the Miller loop computes that point's lines on the fly.  general = 1 makes every later prepare take
   the on-the-fly path (test hook: the fallback must give the same decisions); 0 restores the default.
   Tuning hook: returns -1 (and changes nothing) unless the environment has LCB_ALLOW_TUNING=1. */
int lcb_set_line_mode(int general);
const char *lcb_last_error(void);
/* number of failures recorded on the calling thread so far (each sets lcb_last_error).  The mcl entry points that
   return void (mclBnG1_mul, mclBn_pairing, ...) have no return code: a caller detects their failure by this counter
   changing across the call.  A failed void call also writes a random, non-canonical value to its output (the top limb
   of the first coordinate is all ones), so two failed calls never compare equal. */
uint64_t lcb_error_count(void);
/* test hook: the next `count` passes through fault site `site` fail (1: the single-operation staging's pinned host
   buffer, 2: the prepared-ciphertext cache's uploads after its slots were assigned, 3: mclBn_pairing, 4: a
   single-operation round trip); 0 disables.  Returns -1 unless the environment has LCB_ALLOW_TEST_HOOKS=1. */
int lcb_test_inject_failure(int site, int count);
/* test hook: the line sets of n G2 wire points (96-byte encodings; an undecodable one is the point at infinity), on the
   five-lane kernel (coop = 1) or the one-lane kernel, force[k] = 1 forcing set k's flag to the on-the-fly path.
   out: n sets of 26,368 bytes (pairing.hpp layout); w_g2[k] = 1 iff point 2k + 1 lies in G2.  Returns -1 unless the
   environment has LCB_ALLOW_TEST_HOOKS=1. */
int lcb_test_linesets(int coop, const uint8_t *g2_wire, const uint8_t *force, size_t n, uint32_t *out, uint8_t *w_g2);

/* TPKE.PublicKey.VerifyShare for a batch (TPKE/PublicKey.cs:88-92, called per share from
   HoneyBadger.cs:211-212).  Ciphertext c = (U_c, V_c, W_c) with V_c = v_data[v_off[c] .. v_off[c+1]);
   share i pairs ciphertext ct_idx[i] with decryptor dec_idx[i] (verification key y_keys[dec_idx[i]]) and
   partial decryption ui[i].  accept[i] = 1 iff e(Ui, H(U||V)) == e(Y_i, W) (malformed encodings -> 0). */
int lcb_tpke_verify_shares(uint8_t *accept, size_t n_shares, const uint8_t *y_keys, size_t n_keys,
                           const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data,
                           const uint32_t *v_off, size_t n_cts, const uint32_t *ct_idx,
                           const uint32_t *dec_idx, const uint8_t *ui);
int lcb_tpke_verify_shares_dev(uint8_t *accept, size_t n_shares, const uint8_t *y_keys, size_t n_keys,
                               const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data,
                               const uint32_t *v_off, size_t n_cts, const uint32_t *ct_idx,
                               const uint32_t *dec_idx, const uint8_t *ui, void *stream);

/* The two stages of lcb_tpke_verify_shares_dev, for callers that pipeline or time them separately:
   prepare = verification-key decompression + per-ciphertext H(U||V) and Miller-line precomputation into
   the calling thread's TPKE workspace; verify = the per-share pairing-product check against that workspace
   (n_keys and n_cts must be the prepared ones).  The workspace stays valid until the next TPKE prepare in the
   same context (lcb_ctx_* forms below for explicit contexts). */
int lcb_tpke_prepare_dev(const uint8_t *y_keys, size_t n_keys, const uint8_t *cts_u, const uint8_t *cts_w,
                         const uint8_t *v_data, const uint32_t *v_off, size_t n_cts, void *stream);
int lcb_tpke_verify_prepared_dev(uint8_t *accept, size_t n_shares, size_t n_keys, size_t n_cts,
                                 const uint32_t *ct_idx, const uint32_t *dec_idx, const uint8_t *ui, void *stream);

/* TPKE.PrivateKey.Decrypt for a batch (TPKE/PrivateKey.cs:21-31): status[c] = 1 and ui[c] = x*U_c when
   e(G, W_c) == e(U_c, H(U_c||V_c)), status[c] = 0 ("Invalid share!") otherwise. */
int lcb_tpke_partial_decrypt(uint8_t *ui_out, uint8_t *status, const uint8_t x[32], const uint8_t *cts_u,
                             const uint8_t *cts_w, const uint8_t *v_data, const uint32_t *v_off, size_t n_cts);

/* TPKE.PublicKey.Encrypt for a batch with caller-supplied randomness r (TPKE/PublicKey.cs:25-37):
   U = rG, T = rY (serialized, for the XorWithHash KDF done by the caller), W = r H(U||V). Two-phase
   because V = data XOR KDF(T) is computed between the phases (TPKE/Utils.cs:12-19). */
int lcb_tpke_encrypt_phase1(uint8_t *u_out, uint8_t *t_out, const uint8_t y[48], const uint8_t *r, size_t n);
int lcb_tpke_encrypt_phase2(uint8_t *w_out, const uint8_t *u, const uint8_t *r, const uint8_t *v_data,
                            const uint32_t *v_off, size_t n);

/* ThresholdSignature.PublicKey.ValidateSignature for a batch (ThresholdSignature/PublicKey.cs:16-21,
   ThresholdSigner.cs:62,89-92): share i is checked against message msg_idx[i] (messages concatenated in
   msg_data with offsets msg_off) and public key pks[pk_idx[i]].  accept[i] = e(PK, H(m)) == e(G, sig). */
int lcb_ts_verify_shares(uint8_t *accept, size_t n, const uint8_t *pks, size_t n_pks, const uint8_t *sigs,
                         const uint8_t *msg_data, const uint32_t *msg_off, size_t n_msgs,
                         const uint32_t *msg_idx, const uint32_t *pk_idx);
int lcb_ts_verify_shares_dev(uint8_t *accept, size_t n, const uint8_t *pks, size_t n_pks, const uint8_t *sigs,
                             const uint8_t *msg_data, const uint32_t *msg_off, size_t n_msgs,
                             const uint32_t *msg_idx, const uint32_t *pk_idx, void *stream);

/* Split form of lcb_ts_verify_shares_dev for callers that verify several batches against the same messages and
   keys (e.g. the shares of a coin, then the combined signature): prepare decompresses the keys and hashes every
   message to G2 with its Miller lines; verify_prepared checks items against that workspace. */
int lcb_ts_prepare_dev(const uint8_t *pks, size_t n_pks, const uint8_t *msg_data, const uint32_t *msg_off,
                       size_t n_msgs, void *stream);
int lcb_ts_verify_prepared_dev(uint8_t *accept, size_t n, size_t n_pks, size_t n_msgs, const uint8_t *sigs,
                               const uint32_t *msg_idx, const uint32_t *pk_idx, void *stream);
/* ThresholdSigner.AddShare assembly for whole batches of rounds (ThresholdSigner.cs:62-75, PublicKeySet.cs:34-42):
   round r owns shares [r*per_round, (r+1)*per_round) with verification bits in accept (device); the first k
   accepted shares in index order (x = index + 1) are Lagrange-combined in G2.  sig_out: n_rounds x 96 B,
   status[r] = 0 when round r has fewer than k valid shares.  All pointers are device pointers. */
int lcb_ts_assemble_dev(uint8_t *sig_out, uint8_t *status, const uint8_t *accept, const uint8_t *sigs,
                        size_t per_round, size_t k, size_t n_rounds, void *stream);

/* TPKE.PrivateKey.Decrypt (TPKE/PrivateKey.cs:21-31) against the workspace of lcb_tpke_prepare_dev (same
   ciphertexts): ciphertext validity e(G, W) == e(U, H), then U_i = x U.  x_raw: 32-byte LE secrets (device),
   x_stride = 0 uses one secret for every ciphertext, 1 gives ciphertext c its own secret x_raw[c] (one
   decrypting node per ciphertext, as in an epoch replay).  ui_out: 48 B per ciphertext (zero when invalid),
   status[c] = validity.  Device pointers. */
int lcb_tpke_partial_decrypt_prepared_dev(uint8_t *ui_out, uint8_t *status, const uint8_t *x_raw, size_t x_stride,
                                          const uint8_t *cts_u, size_t n_cts, void *stream);
/* TPKE.PublicKey.FullDecrypt's combination step (TPKE/PublicKey.cs:74-84) for whole batches: ciphertext c owns
   shares [c*per_ct, (c+1)*per_ct) ordered by DecryptorId, with verification bits in accept; the first k
   accepted shares (x = DecryptorId + 1) are Lagrange-combined in G1: u_out[c] = sum lambda_i U_i (48 B),
   status[c] = 0 with fewer than k valid shares.  The plaintext is then lcb_xor_with_hash(u, V) on the host. */
int lcb_tpke_combine_dev(uint8_t *u_out, uint8_t *status, const uint8_t *accept, const uint8_t *shares,
                         size_t per_ct, size_t k, size_t n_cts, void *stream);
/* Arrival-order forms of the two combinations: HoneyBadger.cs:237-247 / ThresholdSigner.cs:62-75 combine the first
   F+1 valid shares to ARRIVE.  order (device, per_group u32 per group): order[g * per_group + j] = the position
   (DecryptorId / signer index) of the j-th share to arrive in group g; entries >= per_group mark arrivals that did
   not happen.  A position listed twice makes the group fail (status 0: repeated abscissa).  The selection then
   walks this order instead of index order; everything else is as lcb_tpke_combine_dev / lcb_ts_assemble_dev. */
int lcb_tpke_combine_ordered_dev(uint8_t *u_out, uint8_t *status, const uint8_t *accept, const uint8_t *shares,
                                 const uint32_t *order, size_t per_ct, size_t k, size_t n_cts, void *stream);
int lcb_ts_assemble_ordered_dev(uint8_t *sig_out, uint8_t *status, const uint8_t *accept, const uint8_t *sigs,
                                const uint32_t *order, size_t per_round, size_t k, size_t n_rounds, void *stream);

/* device time (ms) of k_tpke_miller and k_final_exp_check in the last split TPKE verify (waits for it) */
int lcb_tpke_verify_phase_ms(float ms[2]);
/* Line sets of up to max_sets points per preparation on the five-lane kernel (latency), larger preparations one lane
   per set (throughput); -1 restores the default (8,192).  Tuning hook: -1 unless LCB_ALLOW_TUNING=1. */
int lcb_set_lines_coop_max(int max_sets);
/* 1 (default): the fused batched calls build the validators' fixed-base tables before forking the preparation streams;
   0: on the randomisation stream beside them.  Tuning hook: -1 unless LCB_ALLOW_TUNING=1. */
int lcb_set_keys_first(int on);

/* Randomized batch form of lcb_tpke_verify_prepared_dev (same arguments, same workspace, same validity rules;
   replaces the per-share loop over TPKE/PublicKey.cs:88-92 driven from HoneyBadger.cs:211-212).  Shares are grouped
   into runs of one ciphertext (pass ciphertext-major batches); a group is accepted when
   e(sum r_i U_i, H) == e(sum r_i Y_i, W) for secret 64-bit r_i (getrandom per call), a failed group is split and
   re-checked down to single shares.  Every rejection is exact; a false acceptance has probability <= 2^-64 per group.
   Returns when the decisions are final (one small device-to-host read per splitting level). */
int lcb_tpke_verify_prepared_batched_dev(uint8_t *accept, size_t n_shares, size_t n_keys, size_t n_cts,
                                         const uint32_t *ct_idx, const uint32_t *dec_idx, const uint8_t *ui,
                                         void *stream);
/* prepare + batched verify in one call (arguments of lcb_tpke_verify_shares_dev): the per-share randomisation runs on
   a second stream of the context beside the per-ciphertext hashing and line sets; the prepared workspace is left as
   lcb_tpke_prepare_dev leaves it */
int lcb_tpke_verify_shares_batched_dev(uint8_t *accept, size_t n_shares, const uint8_t *y_keys, size_t n_keys,
                                       const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data,
                                       const uint32_t *v_off, size_t n_cts, const uint32_t *ct_idx,
                                       const uint32_t *dec_idx, const uint8_t *ui, void *stream);
/* lcb_tpke_verify_shares with a per-context cache of prepared ciphertexts (2048 slots: the line sets of H and W and
   the ciphertext's validity, keyed by its bytes U || W || V, least recently used replaced) and of decompressed
   verification keys (4096 slots).  For callers that verify a ciphertext's shares over several calls
   (HoneyBadger.cs:211-212 verifies one share per call): each ciphertext is hashed to G2 and its Miller lines computed
   once.  A call with more than 1024 ciphertexts or more than 4096 keys runs uncached.  Same decisions as
   lcb_tpke_verify_shares for any input. */
int lcb_tpke_verify_shares_cached(uint8_t *accept, size_t n, const uint8_t *y_keys, size_t n_keys,
                                  const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data,
                                  const uint32_t *v_off, size_t n_cts, const uint32_t *ct_idx, const uint32_t *dec_idx,
                                  const uint8_t *ui);
/* host-pointer form of the batched verify (arguments of lcb_tpke_verify_shares) */
int lcb_tpke_verify_shares_batched(uint8_t *accept, size_t n_shares, const uint8_t *y_keys, size_t n_keys,
                                   const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data,
                                   const uint32_t *v_off, size_t n_cts, const uint32_t *ct_idx,
                                   const uint32_t *dec_idx, const uint8_t *ui);
/* Randomized batch forms of the threshold-signature share check (ThresholdSignature/PublicKey.cs:16-21, called per
   share from ThresholdSigner.cs:62): groups = runs of shares of one message (pass message-major batches), checked as
   e(sum s_i PK_i, H(m)) == e(G, sum s_i sig_i); a share whose signature is outside G2 gets its exact check.  Same
   arguments as lcb_ts_verify_prepared_dev / lcb_ts_verify_shares_dev / lcb_ts_verify_shares. */
int lcb_ts_verify_prepared_batched_dev(uint8_t *accept, size_t n, size_t n_pks, size_t n_msgs, const uint8_t *sigs,
                                       const uint32_t *msg_idx, const uint32_t *pk_idx, void *stream);
int lcb_ts_verify_shares_batched_dev(uint8_t *accept, size_t n, const uint8_t *pks, size_t n_pks, const uint8_t *sigs,
                                     const uint8_t *msg_data, const uint32_t *msg_off, size_t n_msgs,
                                     const uint32_t *msg_idx, const uint32_t *pk_idx, void *stream);
int lcb_ts_verify_shares_batched(uint8_t *accept, size_t n, const uint8_t *pks, size_t n_pks, const uint8_t *sigs,
                                 const uint8_t *msg_data, const uint32_t *msg_off, size_t n_msgs,
                                 const uint32_t *msg_idx, const uint32_t *pk_idx);
/* the last batched verify (TPKE or threshold signatures) completed by the calling thread (any context; the
   lcb_ctx_ form: the last one of that context): groups checked per level
   (levels[0] = level 1, levels[1] = the level-2 weighted re-checks of failed groups, then single checks) and device
   ms of [randomisation + grouping, all levels, then summed over the levels: group sums, group Miller loops, final
   exponentiations (+ resolve / search), the fused call's preparation chain (hashing, line sets and census on the
   preparation stream, beside the randomisation; 0 for other calls)]; returns the number of levels (waits for the call) */
int lcb_tpke_batched_stats(uint32_t levels[8], float ms[6]);
/* test hook: fixed 32-byte ChaCha20 key for the batch exponents (NULL restores getrandom).  Honoured only when the
   environment has LCB_ALLOW_FIXED_BATCH_SEED=1 (a fixed key makes the exponents predictable); ignored otherwise. */
void lcb_set_batch_seed(const uint8_t *seed32);
/* Byzantine validators (HoneyBadgerMalicious.cs:17-23 corrupts the share a faulty validator sends in EVERY
   ciphertext): batched calls of at least min_shares shares (default 16384; 0 = never) first check a prefix of the
   batch (512..2048 shares, at most a quarter) share by share — the census — and mark a key suspect when at least half
   of its sampled, decodable shares failed; every share of a suspect key is then checked on its own and the groups are
   summed over the other keys.  Decisions are unchanged; only the cost changes. */
void lcb_set_batch_census(size_t min_shares);
/* census of the last batched verify: {census shares, suspect keys, level-1 groups, level-1 entries after moving the
   suspect keys' shares to single checks} (lcb_ctx_ form: that context's last one) */
int lcb_batched_census(uint32_t out[4]);
/* levels of at most max_checks group checks run on the cooperative kernels (k_coop.hip: nine lanes per pairing check,
   lower latency below one wave per SIMD); 0 = always one check per lane.  Default 32768.  This and the next two are
   tuning hooks: each returns -1 (and changes nothing) unless the environment has LCB_ALLOW_TUNING=1. */
int lcb_set_coop_max(uint32_t max_checks);
/* the cooperative threshold of the group Miller loops alone (default 65536; the final exponentiations keep
   lcb_set_coop_max's) */
int lcb_set_coop_miller_max(uint32_t max_checks);
/* shares / group checks per Miller + final-exponentiation launch pair (default and maximum 2^21): a test hook that
   makes small batches run several chunks (chunk offsets in the copies and searches).  Set it only while no batch call
   is in flight.  Tuning hook (LCB_ALLOW_TUNING=1). */
int lcb_set_verify_chunk(size_t checks);
/* stream layout of the fused batched verifies (lcb_tpke_verify_shares_batched_dev, lcb_ts_verify_shares_batched_dev):
   0 = randomisation on the context's second stream beside the preparation on the caller's; 1 = the
   latency-bound preparation chain (hash-to-G2, line sets, census) on a high-priority stream and the randomisation on
   the caller's; 2 = as 1 with the preparation's first kernel enqueued ahead of the randomisation; 3 = as 2 with the
   TPKE preparation split into hash + H's line set and U / W decoding + W's line set, on two more high-priority
   streams; 4 (default, round 6) = the split preparation's two lane kinds in one dispatch on the one high-priority
   stream, the census behind it, so a context uses one hardware queue per priority (threshold signatures: modes 2-4
   act as 1).  Decisions are unchanged. */
int lcb_set_fork_mode(int mode);
/* the scratch gate (round 6 model): the HSA runtime binds a dispatch's FULL-device scratch
   (private segment per lane rounded to 16 B x 64 lanes x CUs x 32 wave slots) to its hardware queue whenever that is
   below the agent's bind limit (24 GiB on the box), and all queues share one pool (32 GiB); a request the pool cannot
   serve aborts the process.  A launch whose full-device size exceeds the per-queue share T = (pool - 4.5 GiB) / Q
   (Q = 2 x GPU_MAX_HW_QUEUES: the library uses two stream priorities) runs on one process-wide stream per device,
   ordered with the caller's stream by events, so the queues' bound scratch stays within the pool.  `bytes` replaces T
   (environment LCB_SCRATCH_GATE_MB); -1 = off, 0 = every launch with scratch, < -1 = back to the model.  Tuning hook
   (LCB_ALLOW_TUNING=1). */
int lcb_set_scratch_gate(long long bytes);
/* the calling thread's device's scratch model: out[0] pool bytes (HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX, 0 unknown),
   [1] bind limit (..._SCRATCH_LIMIT_CURRENT), [2] wave slots (CUs x waves per CU), [3] Q, [4] the per-queue share T,
   [5] the threshold in force (UINT64_MAX: gate off).  0 on success. */
int lcb_scratch_info(uint64_t out[6]);
/* launches routed through the gate / launches checked, since the process started */
void lcb_scratch_gate_stats(uint64_t *routed, uint64_t *seen);
/* the persistent grids of the table-walking kernels (Lagrange lanes, scalar-multiplication batches) use at most this
   many blocks of 256 lanes (0 = as many as are resident): a test hook that makes small batches walk several items per
   lane.  Tuning hook (LCB_ALLOW_TUNING=1). */
int lcb_set_persist_blocks(uint32_t max_blocks);
/* tuning hook (LCB_ALLOW_TUNING=1): records per lane of the MSM bucket accumulation (k_msm_chunk_acc, default 64);
   0 = one lane per bucket (k_msm_bucket_acc).  Results are unchanged. */
int lcb_set_msm_chunk(int records_per_lane);
/* tuning hook (LCB_ALLOW_TUNING=1): the MSM bucket reduction uses the fewest serial segments up to max_segments lanes
   (0 = by form: the GLV form the fewest segments up to 65,536, the plain form the most of at least 65,536).
   Results are unchanged. */
int lcb_set_msm_segments(int max_segments);
/* tuning hook (LCB_ALLOW_TUNING=1): 1 (default) = the latency-bound kernels of the batched checks (preparation chain,
   every level) raise their waves' issue priority over the bulk randomisation waves sharing their SIMDs; 0 = off */
int lcb_set_wave_priority(int on);
/* test hook: final exponentiation of n Fp12 values (144 x u32 each, Montgomery form, field.hpp layout) by the one-lane
   (coop = 0) or the cooperative (coop = 1) kernel */
int lcb_debug_final_exp(const uint32_t *in, size_t n, uint32_t *out, int coop);
/* test hook: one cooperative Fp12 operation (op: 0 square, 1 cyclotomic square, 2 product, 3 product by the conjugate,
   4..6 Frobenius 1..3, 7 inverse, 8 conjugate, 9 sparse line product, 10 final exponentiation) on n values a (and b),
   with the one-lane field.hpp result beside it in ref */
int lcb_debug_coop_op(int op, const uint32_t *a, const uint32_t *b, size_t n, uint32_t *out, uint32_t *ref);

/* ------------------------------------------------------------------ explicit execution contexts
   A context owns the device workspaces of the prepare/verify, assembly, Lagrange and MSM calls below
   (the context-less forms above use the calling thread's implicit context).  ctx == NULL selects that implicit
   context.  A context may be shared by threads (calls on it are serialized) and its work executes in enqueue
   order across streams; lcb_ctx_synchronize waits for all of it. */
typedef struct lcb_ctx lcb_ctx;
lcb_ctx *lcb_ctx_create(void);
void lcb_ctx_destroy(lcb_ctx *ctx);
int lcb_ctx_synchronize(lcb_ctx *ctx);
int lcb_ctx_tpke_prepare_dev(lcb_ctx *ctx, const uint8_t *y_keys, size_t n_keys, const uint8_t *cts_u,
                             const uint8_t *cts_w, const uint8_t *v_data, const uint32_t *v_off, size_t n_cts,
                             void *stream);
int lcb_ctx_tpke_verify_prepared_dev(lcb_ctx *ctx, uint8_t *accept, size_t n_shares, size_t n_keys, size_t n_cts,
                                     const uint32_t *ct_idx, const uint32_t *dec_idx, const uint8_t *ui, void *stream);
int lcb_ctx_tpke_partial_decrypt_prepared_dev(lcb_ctx *ctx, uint8_t *ui_out, uint8_t *status, const uint8_t *x_raw,
                                              size_t x_stride, const uint8_t *cts_u, size_t n_cts, void *stream);
int lcb_ctx_tpke_combine_dev(lcb_ctx *ctx, uint8_t *u_out, uint8_t *status, const uint8_t *accept,
                             const uint8_t *shares, size_t per_ct, size_t k, size_t n_cts, void *stream);
int lcb_ctx_tpke_combine_ordered_dev(lcb_ctx *ctx, uint8_t *u_out, uint8_t *status, const uint8_t *accept,
                                     const uint8_t *shares, const uint32_t *order, size_t per_ct, size_t k,
                                     size_t n_cts, void *stream);
int lcb_ctx_ts_assemble_ordered_dev(lcb_ctx *ctx, uint8_t *sig_out, uint8_t *status, const uint8_t *accept,
                                    const uint8_t *sigs, const uint32_t *order, size_t per_round, size_t k,
                                    size_t n_rounds, void *stream);
int lcb_ctx_tpke_verify_phase_ms(lcb_ctx *ctx, float ms[2]);
int lcb_ctx_tpke_verify_prepared_batched_dev(lcb_ctx *ctx, uint8_t *accept, size_t n_shares, size_t n_keys,
                                             size_t n_cts, const uint32_t *ct_idx, const uint32_t *dec_idx,
                                             const uint8_t *ui, void *stream);
int lcb_ctx_tpke_verify_shares_batched_dev(lcb_ctx *ctx, uint8_t *accept, size_t n_shares, const uint8_t *y_keys,
                                           size_t n_keys, const uint8_t *cts_u, const uint8_t *cts_w,
                                           const uint8_t *v_data, const uint32_t *v_off, size_t n_cts,
                                           const uint32_t *ct_idx, const uint32_t *dec_idx, const uint8_t *ui,
                                           void *stream);
int lcb_ctx_tpke_batched_stats(lcb_ctx *ctx, uint32_t levels[8], float ms[6]);
int lcb_ctx_batched_census(lcb_ctx *ctx, uint32_t out[4]);
int lcb_ctx_ts_verify_prepared_batched_dev(lcb_ctx *ctx, uint8_t *accept, size_t n, size_t n_pks, size_t n_msgs,
                                           const uint8_t *sigs, const uint32_t *msg_idx, const uint32_t *pk_idx,
                                           void *stream);
int lcb_ctx_ts_verify_shares_batched_dev(lcb_ctx *ctx, uint8_t *accept, size_t n, const uint8_t *pks, size_t n_pks,
                                         const uint8_t *sigs, const uint8_t *msg_data, const uint32_t *msg_off,
                                         size_t n_msgs, const uint32_t *msg_idx, const uint32_t *pk_idx,
                                         void *stream);
int lcb_ctx_ts_prepare_dev(lcb_ctx *ctx, const uint8_t *pks, size_t n_pks, const uint8_t *msg_data,
                           const uint32_t *msg_off, size_t n_msgs, void *stream);
int lcb_ctx_ts_verify_prepared_dev(lcb_ctx *ctx, uint8_t *accept, size_t n, size_t n_pks, size_t n_msgs,
                                   const uint8_t *sigs, const uint32_t *msg_idx, const uint32_t *pk_idx, void *stream);
int lcb_ctx_ts_assemble_dev(lcb_ctx *ctx, uint8_t *sig_out, uint8_t *status, const uint8_t *accept,
                            const uint8_t *sigs, size_t per_round, size_t k, size_t n_rounds, void *stream);
int lcb_ctx_g1_lagrange_dev(lcb_ctx *ctx, uint8_t *out, uint8_t *status, const uint8_t *xs, const uint8_t *ys,
                            const uint32_t *off, size_t n_problems, size_t n_entries, void *stream);
int lcb_ctx_g2_lagrange_dev(lcb_ctx *ctx, uint8_t *out, uint8_t *status, const uint8_t *xs, const uint8_t *ys,
                            const uint32_t *off, size_t n_problems, size_t n_entries, void *stream);
int lcb_ctx_g1_msm_dev(lcb_ctx *ctx, void *out_jac, const void *points_aff, const uint8_t *scalars, size_t n,
                       int window_bits, void *stream);
int lcb_ctx_g1_msm_phase_ms(lcb_ctx *ctx, float *ms, int n_phases);

/* ------------------------------------------------------------------ trustless DKG G1 work
   coeffs: n_comm commitments x (degree+1)(degree+2)/2 serialized G1 coefficients each, in Commitment's symmetric
   Index(i, j) order (src/Lachain.Consensus/ThresholdKeygen/Data/Commitment.cs:14-21,55-59).
   lcb_dkg_commitment_eval: out[q] = Commitment.Evaluate(xs[q], ys[q]) of commitment comm_idx[q] (Commitment.cs:23-37,
     the per-value check of TrustlessKeygen.HandleSendValue, TrustlessKeygen.cs:150-152).
   lcb_dkg_commitment_rows: rows_out[q] = Commitment.Evaluate(xs[q]) = degree+1 points (Commitment.cs:39-53; the
     commit check of HandleCommit, TrustlessKeygen.cs:90-94, and TryGetKeys' Evaluate(0), :166).
   lcb_g1_eval_poly_batch: MclBls12381.EvaluatePolynomial over G1 at many small x (TryGetKeys, TrustlessKeygen.cs:172-174).
   x, y are the reference's int arguments (player indices); status[q] = 0 for a malformed coefficient or a
   comm_idx >= n_comm.  Results equal the reference's Fr-power sums for coefficients in G1. */
int lcb_dkg_commitment_eval(uint8_t *out, uint8_t *status, const uint8_t *coeffs, size_t n_comm, int degree,
                            const uint32_t *comm_idx, const int32_t *xs, const int32_t *ys, size_t n_queries);
int lcb_dkg_commitment_rows(uint8_t *rows_out, uint8_t *status, const uint8_t *coeffs, size_t n_comm, int degree,
                            const uint32_t *comm_idx, const int32_t *xs, size_t n_queries);
int lcb_g1_eval_poly_batch(uint8_t *out, uint8_t *status, const uint8_t *coeffs, size_t n_coeffs, const int32_t *xs,
                           size_t n_points);

/* ------------------------------------------------------------------ reliable broadcast: Reed-Solomon
   The EncryptedShare bytes travel as N shards of a GF(2^8) Reed-Solomon code (polynomial 0x11D, alpha = 2, generator
   roots alpha^0..alpha^(erasures-1): ErasureCoding.cs:13), erasures = 2F.
   lcb_rs_encode = ReliableBroadcast.ErasureCodingShards(input, n_shards, erasures) (ReliableBroadcast.cs:393-419):
     input_len must be a multiple of n_shards - erasures (AugmentInput pads it); shards_out = n_shards x shard bytes.
   lcb_rs_decode = DecodeFromEchos (ReliableBroadcast.cs:421-446): exactly n_shards - erasures echoes, echo e is shard
     from[e]; out = all n_shards shards.  -1 on bad arguments or an unsolvable erasure set (only with > 255 shards). */
int lcb_rs_encode(uint8_t *shards_out, const uint8_t *input, size_t input_len, int n_shards, int erasures);
int lcb_rs_decode(uint8_t *out, const uint8_t *echo_data, const int32_t *from, int n_echos, size_t shard_size,
                  int n_shards, int erasures);

/* ------------------------------------------------------------------ secp256k1 ECDSA header signatures
   RootProtocol checks every SignedHeaderMessage with
     DefaultCrypto.VerifySignatureHashed(header.Keccak(), signature, EcdsaPublicKeySet[idx].EncodeCompressed(),
                                         useNewChainId)            (RootProtocol.cs:91-105, DefaultCrypto.cs:79-101)
   accept[i] = 1 exactly when the reference returns true: signature i is sig_len bytes (must equal 65 for the old
   chain id, 66 for the new one, DefaultCrypto.cs:26-29), its recovery id (sig[64], or sig[64] * 256 + sig[65]) gives
   (enc - 36) / 2 / chain_id in [0, 3] (C# int arithmetic; chain_id 0 rejects everything), r || s (big-endian) parse
   below n, s <= (n - 1) / 2, and x(u1 G + u2 Q) mod n == r with u1 = z / s, u2 = r / s, z = hash mod n (libsecp256k1
   semantics; Secp256k1.Net 0.1.55 / Secp256k1.Native 0.1.20, Lachain.Crypto.csproj:21-22).  key_idx[i] selects the
   key; an index out of range or a key that fails secp256k1_ec_pubkey_parse (33-byte 02/03 or 65-byte 04/06/07
   encodings) rejects.  `chain_id` is TransactionUtils.ChainId(use_new_chain_id) (TransactionUtils.cs:25-28).
   A key set keeps the validators' keys resident on the device with a 270 KB fixed-base table per key, built once;
   the host-pointer calls cache the last key list they saw in the calling thread's context. */
typedef struct lcb_ecdsa_keyset lcb_ecdsa_keyset;
/* BlockHeader (block.proto:7-15) as raw bytes; hashed as HashUtils.Keccak(BlockHeader) (HashUtils.cs:40-53) */
typedef struct {
    uint64_t index;
    uint8_t prev_block_hash[32];
    uint8_t merkle_root[32];
    uint8_t state_hash[32];
    uint64_t nonce;
} lcb_block_header;
lcb_ecdsa_keyset *lcb_ecdsa_keyset_create(const uint8_t *pubkeys, size_t pk_len, size_t n_keys);
void lcb_ecdsa_keyset_destroy(lcb_ecdsa_keyset *ks);
size_t lcb_ecdsa_keyset_size(const lcb_ecdsa_keyset *ks);
int lcb_ecdsa_keyset_valid(const lcb_ecdsa_keyset *ks, uint8_t *ok_out);   /* per key: parsed (1) or not (0) */
/* host pointers; hashes: n x 32 bytes (the reference's messageHash) */
int lcb_ecdsa_verify_hashed_batch(uint8_t *accept, const uint8_t *hashes, const uint8_t *sigs, size_t sig_len,
                                  const uint8_t *pubkeys, size_t pk_len, size_t n_keys, const int32_t *key_idx,
                                  size_t n, int use_new_chain_id, int32_t chain_id);
/* RootProtocol's whole check: header.Index == era (RootProtocol.cs:94-96), Keccak of the header, then the above */
int lcb_root_header_verify_batch(uint8_t *accept, const lcb_block_header *headers, uint64_t era, const uint8_t *sigs,
                                 size_t sig_len, const uint8_t *pubkeys, size_t pk_len, size_t n_keys,
                                 const int32_t *key_idx, size_t n, int use_new_chain_id, int32_t chain_id);
int lcb_header_keccak_batch(uint8_t *hashes, const lcb_block_header *headers, size_t n);
/* device pointers, enqueued on `stream` in a context (NULL = the calling thread's default context) */
int lcb_ctx_ecdsa_verify_hashed_dev(lcb_ctx *ctx, uint8_t *accept, const uint8_t *hashes, const uint8_t *sigs,
                                    size_t sig_len, const int32_t *key_idx, size_t n, const lcb_ecdsa_keyset *ks,
                                    int use_new_chain_id, int32_t chain_id, void *stream);
int lcb_ctx_root_header_verify_dev(lcb_ctx *ctx, uint8_t *accept, const uint8_t *headers, uint64_t era,
                                   const uint8_t *sigs, size_t sig_len, const int32_t *key_idx, size_t n,
                                   const lcb_ecdsa_keyset *ks, int use_new_chain_id, int32_t chain_id, void *stream);
/* signing side (EcdsaKeyPair / DefaultCrypto.SignHashed, DefaultCrypto.cs:107-137) with caller-given nonces (not
   RFC 6979, so signature bytes differ from libsecp256k1's for the same key and hash; every one verifies): key
   derivation out33 = compressed d G, and r || s (low s) || v encoded as SignHashed encodes it.  ok[i] = 0 for a
   private key or nonce outside [1, n) or a zero r / s.  Used for synthetic inputs and the node's own header. */
int lcb_ecdsa_pubkey_batch(uint8_t *out33, uint8_t *ok, const uint8_t *privs, size_t n);
int lcb_ecdsa_sign_hashed_batch(uint8_t *sigs_out, uint8_t *ok, const uint8_t *hashes, const uint8_t *privs,
                                const uint8_t *nonces, size_t n, int use_new_chain_id, int32_t chain_id);
int lcb_ctx_ecdsa_pubkey_dev(lcb_ctx *ctx, uint8_t *out33, uint8_t *ok, const uint8_t *privs, size_t n, void *stream);
int lcb_ctx_ecdsa_sign_hashed_dev(lcb_ctx *ctx, uint8_t *sigs_out, uint8_t *ok, const uint8_t *hashes,
                                  const uint8_t *privs, const uint8_t *nonces, size_t n, int use_new_chain_id,
                                  int32_t chain_id, void *stream);
int lcb_ecdsa_pubkey_dev(uint8_t *out33, uint8_t *ok, const uint8_t *privs, size_t n, void *stream);
int lcb_ecdsa_sign_hashed_dev(uint8_t *sigs_out, uint8_t *ok, const uint8_t *hashes, const uint8_t *privs,
                              const uint8_t *nonces, size_t n, int use_new_chain_id, int32_t chain_id, void *stream);
/* kernel milliseconds of the last verification in the context: header hash (0 if hashes were given), scalars, verify */
int lcb_ctx_ecdsa_phase_ms(lcb_ctx *ctx, float ms[3]);
int lcb_ecdsa_phase_ms(float ms[3]);
int lcb_ecdsa_verify_hashed_dev(uint8_t *accept, const uint8_t *hashes, const uint8_t *sigs, size_t sig_len,
                                const int32_t *key_idx, size_t n, const lcb_ecdsa_keyset *ks, int use_new_chain_id,
                                int32_t chain_id, void *stream);
int lcb_root_header_verify_dev(uint8_t *accept, const uint8_t *headers, uint64_t era, const uint8_t *sigs,
                               size_t sig_len, const int32_t *key_idx, size_t n, const lcb_ecdsa_keyset *ks,
                               int use_new_chain_id, int32_t chain_id, void *stream);

/* ------------------------------------------------------------------ aggregation queue (one share per call)
   The consensus code verifies one share per call from many protocol threads (HoneyBadger.cs:156-158,211-212,
   ThresholdSigner.cs:62, AbstractProtocol.cs:46-47).  A queue aggregates such calls into GPU batches: submit
   returns a ticket (> 0, or -1 on bad arguments), a worker thread runs the pending shares as one batch when
   max_batch are pending or the oldest has waited max_delay_us, and lcb_queue_wait returns the share's decision
   (1 accept, 0 reject, -1 batch error / unknown or already-waited ticket).  Decisions equal the batch entry
   points' (PublicKey.VerifyShare, TPKE/PublicKey.cs:88-92; ValidateSignature, ThresholdSignature/PublicKey.cs:16-21).
   destroy flushes and runs everything still pending; stats: {batches, shares, largest batch}. */
typedef struct lcb_queue lcb_queue;
lcb_queue *lcb_queue_create(size_t max_batch, uint32_t max_delay_us);
void lcb_queue_destroy(lcb_queue *q);
int64_t lcb_queue_tpke_verify(lcb_queue *q, const uint8_t y48[48], const uint8_t u48[48], const uint8_t *v,
                              size_t v_len, const uint8_t w96[96], const uint8_t ui48[48]);
int64_t lcb_queue_ts_verify(lcb_queue *q, const uint8_t pk48[48], const uint8_t *msg, size_t msg_len,
                            const uint8_t sig96[96]);
/* prepare a TPKE ciphertext (U || V || W: hash-to-G2 of U || V and both line sets) on the worker its shares go to,
   ahead of them — the reference decrypts every ciphertext of the common subset (HoneyBadger.cs:144-146) before it
   handles the other validators' shares for it (HoneyBadger.cs:190-213).  Asynchronous; 0 or -1 (bad arguments). */
int lcb_queue_tpke_prepare(lcb_queue *q, const uint8_t u48[48], const uint8_t *v, size_t v_len, const uint8_t w96[96]);
int lcb_queue_wait(lcb_queue *q, int64_t ticket);
int lcb_queue_flush(lcb_queue *q);
int lcb_queue_stats(lcb_queue *q, uint64_t out[3]);
const char *lcb_queue_last_error(lcb_queue *q);
/* flushes of at least min_shares shares use the randomized batch checks (lcb_tpke_verify_shares_batched /
   lcb_ts_verify_shares_batched, shares reordered by ciphertext / message inside the flush); 0 = exact checks only
   (the default) */
int lcb_queue_set_batched(lcb_queue *q, size_t min_shares);

/* ------------------------------------------------------------------ CommonCoin consumers (row a13)
   The combined signature's serialized bytes feed two consensus decisions:
   CoinResult.Parity = popcount(XOR of all bytes) is odd   (src/Lachain.Consensus/CommonCoin/CoinResult.cs:16-20)
   block nonce = little-endian u64 of the 8-byte XOR fold   (src/Lachain.Consensus/RootProtocol/RootProtocol.cs:316-322)
   Host forms take any byte length; the device form folds n 96-byte signatures (8-byte aligned) in one launch,
   either output nullable. */
int lcb_coin_parity(const uint8_t *sig_bytes, size_t len);
uint64_t lcb_coin_nonce(const uint8_t *sig_bytes, size_t len);
int lcb_coin_fold_dev(uint8_t *parity, uint64_t *nonce, const uint8_t *sigs96, size_t n, void *stream);

/* PrivateKeyShare.HashAndSign for a batch of (key, message) pairs (ThresholdSignature/PrivateKeyShare.cs:21-27) */
int lcb_ts_sign(uint8_t *sigs_out, const uint8_t *sks, const uint8_t *msg_data, const uint32_t *msg_off,
                const uint32_t *msg_idx, size_t n);

/* Batched Lagrange interpolation at 0 (MclBls12381.LagrangeInterpolate; PublicKeySet.AssembleSignature,
   ThresholdSignature/PublicKeySet.cs:34-42, and TPKE FullDecrypt, TPKE/PublicKey.cs:74-84).
   Problem j uses k = off[j+1]-off[j] entries starting at off[j]: x values as 32-byte Fr, y values serialized.
   status[j] = 1 ok, 0 on k == 0, zero x or duplicate x (mcl returns -1). */
int lcb_g1_lagrange_batch(uint8_t *out, uint8_t *status, const uint8_t *xs, const uint8_t *ys,
                          const uint32_t *off, size_t n_problems);
int lcb_g2_lagrange_batch(uint8_t *out, uint8_t *status, const uint8_t *xs, const uint8_t *ys,
                          const uint32_t *off, size_t n_problems);

/* Device-pointer forms of the batched Lagrange interpolation above (n_entries = off[n_problems]). */
int lcb_g1_lagrange_dev(uint8_t *out, uint8_t *status, const uint8_t *xs, const uint8_t *ys, const uint32_t *off,
                        size_t n_problems, size_t n_entries, void *stream);
int lcb_g2_lagrange_dev(uint8_t *out, uint8_t *status, const uint8_t *xs, const uint8_t *ys, const uint32_t *off,
                        size_t n_problems, size_t n_entries, void *stream);

/* G1 multi-scalar multiplication sum_i s_i P_i (serialized points, 32-byte LE scalars < r): the large-k form of
   MclBls12381.LagrangeInterpolate / mclBnG1_mulVec (TPKE/PublicKey.cs:83, ThresholdSignature/PublicKeySet.cs:31).
   Pippenger bucket method on the GPU (k_msm.hip).  Returns -1 on a malformed point or a scalar >= r. */
int lcb_g1_msm(uint8_t out[48], const uint8_t *points, const uint8_t *scalars, size_t n);

/* Device-resident MSM (BASELINE configs[3]).  points_aff: n x 96 B affine points in mcl's in-memory Fp layout
   (x then y, Montgomery form, 6 x u64 LE each = the x,y words of a normalized mclBnG1; (0,0) = infinity);
   scalars: n x 32 B LE, reduced mod r on the device.  out_jac: 144 B Jacobian result (mclBnG1 layout) in device
   memory.  window_bits = 0 picks the Pippenger window width from n (lcb_g1_msm_window).  Enqueued on `stream`
   (a hipStream_t); nothing is synchronised. */
int lcb_g1_msm_dev(void *out_jac, const void *points_aff, const uint8_t *scalars, size_t n, int window_bits,
                   void *stream);
int lcb_g1_msm_window(size_t n);
/* GLV form of the same MSM for points of order r (e.g. generated as a_i G, or checked with a subgroup test):
   s_i = s1 + s2 lambda (lambda = z^2 - 1, s1 < 2^129, s2 < 2^128) over the 2n points P_i, phi(P_i) = (beta x, y):
   half the windows, so half the serial window combination and bucket reduction.  For a point with a component
   outside the r-subgroup phi(P) != lambda P and the result differs from lcb_g1_msm_dev's (which is exact for any
   point), so wire-supplied points (e.g. LagrangeInterpolate over shares) must use lcb_g1_msm_dev. */
int lcb_g1_msm_glv_dev(void *out_jac, const void *points_aff, const uint8_t *scalars, size_t n, int window_bits,
                       void *stream);
int lcb_ctx_g1_msm_glv_dev(lcb_ctx *ctx, void *out_jac, const void *points_aff, const uint8_t *scalars, size_t n,
                           int window_bits, void *stream);
int lcb_g1_msm_glv_window(size_t n);
/* per-phase device time (ms) of the last MSM: digits, sort, bucket bounds, bucket accumulation, bucket
   reduction, window combination (waits for the last MSM to finish) */
int lcb_g1_msm_phase_ms(float *ms, int n_phases);
/* 48-byte serialized G1 -> 96-byte affine device layout above; ok[i] = 0 for a malformed encoding (nullable) */
int lcb_g1_to_affine_dev(void *out_aff, uint8_t *ok, const uint8_t *points, size_t n, void *stream);
/* sum of k Jacobian G1 points (device, 144 B each, e.g. the per-GPU MSM partials after an RCCL all-gather);
   writes the serialized sum to out48 and/or the Jacobian sum to out_jac (device pointers, either nullable) */
int lcb_g1_jac_sum_dev(uint8_t *out48, void *out_jac, const void *parts, size_t k, void *stream);
int lcb_ctx_g1_jac_sum_dev(lcb_ctx *ctx, uint8_t *out48, void *out_jac, const void *parts, size_t k, void *stream);

/* batched scalar multiplication of the G1 / G2 generator or of given points (key generation, synthetic inputs) */
int lcb_g1_mul_batch(uint8_t *out, const uint8_t *points, int points_is_generator, const uint8_t *scalars, size_t n);
int lcb_g2_mul_batch(uint8_t *out, const uint8_t *points, int points_is_generator, const uint8_t *scalars, size_t n);
int lcb_g2_hash_batch(uint8_t *out, const uint8_t *msg_data, const uint32_t *msg_off, size_t n);

/* TPKE Utils.XorWithHash (BouncyCastle DigestRandomGenerator(Sha3Digest) keystream, TPKE/Utils.cs:12-19):
   host-side byte work, provided so a non-.NET host can finish FullDecrypt/Encrypt. */
void lcb_xor_with_hash(uint8_t *out, const uint8_t g1[48], const uint8_t *data, size_t len);

#ifdef __cplusplus
}
#endif
#endif
