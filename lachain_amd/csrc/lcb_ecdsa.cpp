// lachain_amd/csrc/lcb_ecdsa.cpp — host side of the batched secp256k1 ECDSA header-signature checks
// (include/lachain_bls.h "secp256k1 ECDSA").
//
// Reference call: RootProtocol.cs:91-105 ->
//   DefaultCrypto.VerifySignatureHashed(header.Keccak(), sig, EcdsaPublicKeySet[idx].EncodeCompressed(), useNewChainId)
// (DefaultCrypto.cs:79-101).  A key set (lcb_ecdsa_keyset) holds the validators' keys on one device, each with its
// fixed-base comb table (k_secp.hip); the generator's table is built once per device.  The host-pointer entry points
// keep the last key list they were given in the calling thread's context, so a caller that passes the same
// EcdsaPublicKeySet every era builds the tables once.  No CPU fallback: every check runs in k_secp.hip.
#include <hip/hip_runtime.h>
#include <string.h>
#include <mutex>
#include <vector>

#include "launch.h"
#include "lcb_internal.hpp"
#include "../../include/lachain_bls.h"

using namespace lcb_int;

struct lcb_ecdsa_keyset {
    int device = 0;
    size_t n_keys = 0;
    void *aff = nullptr;        // n_keys affine points (64 B)
    u32 *ok = nullptr;          // n_keys validity words
    void *tables = nullptr;     // n_keys comb tables
    std::vector<uint8_t> ok_host;
};

namespace {

std::mutex g_gen_mu;
void *g_gen_table[64] = {};   // per device: the generator's comb table

void keyset_free(lcb_ecdsa_keyset *ks) {
    if (!ks) return;
    if (ks->aff) (void)hipFree(ks->aff);
    if (ks->ok) (void)hipFree(ks->ok);
    if (ks->tables) (void)hipFree(ks->tables);
    delete ks;
}

// comb tables of n points already parsed into aff / ok (device), on stream s; temporary space is freed before return
bool build_tables(hipStream_t s, const void *aff, const u32 *ok, size_t n, void *tables) {
    size_t tmp_bytes = 2 * 128 * 33 * n * 32;
    void *tmp = nullptr;
    hipError_t e = hipMalloc(&tmp, tmp_bytes);
    if (e != hipSuccess) { set_error("comb table workspace", e); return false; }
    lcbk_secp_comb_build(s, aff, ok, (u32)n, tables, tmp);
    bool good = launch_ok("comb table build");
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) { set_error("comb table build", e); good = false; }
    (void)hipFree(tmp);
    return good;
}

const void *gen_table(hipStream_t s) {
    int dev = device();
    if (dev < 0 || dev >= 64) { set_error("device index out of range"); return nullptr; }
    std::lock_guard<std::mutex> lk(g_gen_mu);
    if (g_gen_table[dev]) return g_gen_table[dev];
    void *aff = nullptr, *tab = nullptr;
    u32 *ok = nullptr;
    hipError_t e = hipMalloc(&aff, lcbk_secp_aff_bytes());
    if (e == hipSuccess) e = hipMalloc(&ok, 4);
    if (e == hipSuccess) e = hipMalloc(&tab, lcbk_secp_table_bytes());
    if (e != hipSuccess) {
        set_error("generator table allocation", e);
        if (aff) (void)hipFree(aff);
        if (ok) (void)hipFree(ok);
        if (tab) (void)hipFree(tab);
        return nullptr;
    }
    lcbk_secp_gen(s, aff, ok);
    bool good = build_tables(s, aff, ok, 1, tab);
    (void)hipFree(aff);
    (void)hipFree(ok);
    if (!good) { (void)hipFree(tab); return nullptr; }
    g_gen_table[dev] = tab;
    return tab;
}

lcb_ecdsa_keyset *keyset_new(lcb_ctx *c, const uint8_t *pubkeys, size_t pk_len, size_t n_keys) {
    if (pk_len != 33 && pk_len != 65) { set_error("ecdsa key set: keys must be 33 (compressed) or 65 bytes"); return nullptr; }
    if (n_keys == 0 || n_keys > (1u << 20)) { set_error("ecdsa key set: 1 .. 2^20 keys"); return nullptr; }
    Enq q(c, c->stream);
    if (!gen_table(c->stream)) return nullptr;
    lcb_ecdsa_keyset *ks = new lcb_ecdsa_keyset;
    ks->device = c->device;
    ks->n_keys = n_keys;
    uint8_t *dpk = nullptr;
    hipError_t e = hipMalloc(&ks->aff, lcbk_secp_aff_bytes() * n_keys);
    if (e == hipSuccess) e = hipMalloc(&ks->ok, 4 * n_keys);
    if (e == hipSuccess) e = hipMalloc(&ks->tables, lcbk_secp_table_bytes() * n_keys);
    if (e == hipSuccess) e = hipMalloc(&dpk, pk_len * n_keys);
    if (e != hipSuccess) {
        set_error("ecdsa key set allocation", e);
        if (dpk) (void)hipFree(dpk);
        keyset_free(ks);
        return nullptr;
    }
    hipMemcpyAsync(dpk, pubkeys, pk_len * n_keys, hipMemcpyHostToDevice, c->stream);
    lcbk_secp_key_parse(c->stream, dpk, (u32)pk_len, (u32)n_keys, ks->aff, ks->ok);
    bool good = launch_ok("ecdsa key parse") && build_tables(c->stream, ks->aff, ks->ok, n_keys, ks->tables);
    (void)hipFree(dpk);
    if (good) {
        std::vector<u32> okw(n_keys);
        e = hipMemcpy(okw.data(), ks->ok, 4 * n_keys, hipMemcpyDeviceToHost);
        if (e != hipSuccess) { set_error("ecdsa key set", e); good = false; }
        ks->ok_host.resize(n_keys);
        for (size_t i = 0; i < n_keys; i++) ks->ok_host[i] = okw[i] != 0;
    }
    if (!good) { keyset_free(ks); return nullptr; }
    return ks;
}

// the verification pipeline on device pointers; hashes == nullptr means "hash the headers first"
int verify_enqueue(lcb_ctx *c, hipStream_t s, uint8_t *accept, const uint8_t *hashes, const uint8_t *headers,
                   uint64_t era, const uint8_t *sigs, size_t sig_len, const int32_t *key_idx, size_t n,
                   const lcb_ecdsa_keyset *ks, int use_new_chain_id, int32_t chain_id) {
    if (!n) return 0;
    if (!ks) { set_error("ecdsa: null key set"); return -1; }
    if (ks->device != c->device) { set_error("ecdsa: key set belongs to another device"); return -1; }
    if (n > 0xffffffffu / 2) { set_error("ecdsa: batch too large"); return -1; }
    if (sig_len == 0 || sig_len > 4096) { set_error("ecdsa: bad signature stride"); return -1; }
    const void *gt = gen_table(s);
    if (!gt) return -1;
    void *jobs = c->ec[0].get(lcbk_secp_job_bytes() * n);
    if (!jobs) { set_error("device allocation failed"); return -1; }
    if (!c->ec_ev_ready) {
        for (auto &e : c->ec_ev)
            if (hipEventCreate(&e) != hipSuccess) { set_error("event creation"); return -1; }
        c->ec_ev_ready = true;
    }
    const uint8_t *pre_ok = nullptr;
    (void)hipEventRecord(c->ec_ev[0], s);
    c->ec_hashed = hashes == nullptr;
    if (!hashes) {
        uint8_t *h = (uint8_t *)c->ec[1].get(32 * n), *po = (uint8_t *)c->ec[2].get(n);
        if (!h || !po) { set_error("device allocation failed"); return -1; }
        lcbk_secp_header_hash(s, headers, (u32)n, era, h, po);
        hashes = h;
        pre_ok = po;
    }
    (void)hipEventRecord(c->ec_ev[1], s);
    u32 want = use_new_chain_id ? 66u : 65u;      // DefaultCrypto.SignatureSize (DefaultCrypto.cs:26-29)
    lcbk_secp_scalars(s, hashes, sigs, (u32)sig_len, want, chain_id, key_idx, (u32)ks->n_keys, ks->ok, pre_ok, (u32)n,
                      jobs);
    (void)hipEventRecord(c->ec_ev[2], s);
    lcbk_secp_verify(s, jobs, (u32)n, gt, ks->tables, accept);
    (void)hipEventRecord(c->ec_ev[3], s);
    c->ec_ran = true;
    return launch_ok("ecdsa verify launch") ? 0 : -1;
}

// the host API's key set: reuse the context's cached one when the key list is byte-identical
const lcb_ecdsa_keyset *cached_keyset(lcb_ctx *c, const uint8_t *pubkeys, size_t pk_len, size_t n_keys) {
    size_t bytes = pk_len * n_keys;
    if (c->ec_cache && c->ec_cache_pk_len == pk_len && c->ec_cache_keys.size() == bytes &&
        memcmp(c->ec_cache_keys.data(), pubkeys, bytes) == 0)
        return c->ec_cache;
    keyset_free(c->ec_cache);
    c->ec_cache = nullptr;
    c->ec_cache_keys.clear();
    lcb_ecdsa_keyset *ks = keyset_new(c, pubkeys, pk_len, n_keys);
    if (!ks) return nullptr;
    c->ec_cache = ks;
    c->ec_cache_keys.assign(pubkeys, pubkeys + bytes);
    c->ec_cache_pk_len = pk_len;
    return ks;
}

int verify_host(uint8_t *accept, const uint8_t *hashes, const uint8_t *headers, uint64_t era, const uint8_t *sigs,
                size_t sig_len, const uint8_t *pubkeys, size_t pk_len, size_t n_keys, const int32_t *key_idx, size_t n,
                int use_new_chain_id, int32_t chain_id) {
    lcb_ctx *c = ctx_sync();
    if (!c) return -1;
    if (!n) return 0;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    const lcb_ecdsa_keyset *ks = cached_keyset(c, pubkeys, pk_len, n_keys);
    if (!ks) return -1;
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    size_t in_bytes = headers ? 112 * n : 32 * n;
    uint8_t *din = (uint8_t *)c->ec[3].get(in_bytes), *dsig = (uint8_t *)c->ec[4].get(sig_len * n);
    int32_t *didx = (int32_t *)c->ec[5].get(4 * n);
    uint8_t *dout = (uint8_t *)c->out[0].get(n);
    if (!din || !dsig || !didx || !dout) { set_error("device allocation failed"); return -1; }
    hipMemcpyAsync(din, headers ? headers : hashes, in_bytes, hipMemcpyHostToDevice, s);
    hipMemcpyAsync(dsig, sigs, sig_len * n, hipMemcpyHostToDevice, s);
    hipMemcpyAsync(didx, key_idx, 4 * n, hipMemcpyHostToDevice, s);
    if (verify_enqueue(c, s, dout, headers ? nullptr : din, headers ? din : nullptr, era, dsig, sig_len, didx, n, ks,
                       use_new_chain_id, chain_id))
        return -1;
    hipMemcpyAsync(accept, dout, n, hipMemcpyDeviceToHost, s);
    return sync_ok(c, "ecdsa verify") ? 0 : -1;
}

}  // namespace

namespace lcb_int {
void ecdsa_ctx_release(lcb_ctx *c) {
    if (c->ec_ev_ready) for (auto &e : c->ec_ev) (void)hipEventDestroy(e);
    c->ec_ev_ready = false;
    keyset_free(c->ec_cache);
    c->ec_cache = nullptr;
    c->ec_cache_keys.clear();
    for (auto &b : c->ec) b.release();
}
}  // namespace lcb_int

// ------------------------------------------------------------------ exported
extern "C" lcb_ecdsa_keyset *lcb_ecdsa_keyset_create(const uint8_t *pubkeys, size_t pk_len, size_t n_keys) {
    lcb_ctx *c = ctx_sync();
    if (!c) return nullptr;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    return keyset_new(c, pubkeys, pk_len, n_keys);
}
extern "C" void lcb_ecdsa_keyset_destroy(lcb_ecdsa_keyset *ks) {
    if (ks) (void)hipDeviceSynchronize();   // a verification enqueued by another thread may still read the tables
    keyset_free(ks);
}
extern "C" size_t lcb_ecdsa_keyset_size(const lcb_ecdsa_keyset *ks) { return ks ? ks->n_keys : 0; }
extern "C" int lcb_ecdsa_keyset_valid(const lcb_ecdsa_keyset *ks, uint8_t *ok_out) {
    if (!ks) { set_error("ecdsa: null key set"); return -1; }
    memcpy(ok_out, ks->ok_host.data(), ks->n_keys);
    return 0;
}
extern "C" int lcb_ctx_ecdsa_verify_hashed_dev(lcb_ctx *ctx, uint8_t *accept, const uint8_t *hashes, const uint8_t *sigs,
                                               size_t sig_len, const int32_t *key_idx, size_t n,
                                               const lcb_ecdsa_keyset *ks, int use_new_chain_id, int32_t chain_id,
                                               void *stream) {
    lcb_ctx *c = ctx_resolve(ctx);
    if (!c) return -1;
    Enq q(c, (hipStream_t)stream);
    return verify_enqueue(c, q.s, accept, hashes, nullptr, 0, sigs, sig_len, key_idx, n, ks, use_new_chain_id, chain_id);
}
extern "C" int lcb_ctx_root_header_verify_dev(lcb_ctx *ctx, uint8_t *accept, const uint8_t *headers, uint64_t era,
                                              const uint8_t *sigs, size_t sig_len, const int32_t *key_idx, size_t n,
                                              const lcb_ecdsa_keyset *ks, int use_new_chain_id, int32_t chain_id,
                                              void *stream) {
    lcb_ctx *c = ctx_resolve(ctx);
    if (!c) return -1;
    Enq q(c, (hipStream_t)stream);
    return verify_enqueue(c, q.s, accept, nullptr, headers, era, sigs, sig_len, key_idx, n, ks, use_new_chain_id, chain_id);
}
// kernel milliseconds of the context's last verification: header hash (0 when hashes were given), scalars, verify
extern "C" int lcb_ctx_ecdsa_phase_ms(lcb_ctx *ctx, float ms[3]) {
    lcb_ctx *c = ctx_resolve(ctx);
    if (!c) return -1;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    if (!c->ec_ran) { set_error("no ECDSA verification has run in this context"); return -1; }
    for (int k = 0; k < 3; k++) {
        hipError_t e = hipEventSynchronize(c->ec_ev[k + 1]);
        if (e == hipSuccess) e = hipEventElapsedTime(&ms[k], c->ec_ev[k], c->ec_ev[k + 1]);
        if (e != hipSuccess) { set_error("ecdsa phase timing", e); return -1; }
    }
    if (!c->ec_hashed) ms[0] = 0.f;
    return 0;
}
extern "C" int lcb_ecdsa_phase_ms(float ms[3]) { return lcb_ctx_ecdsa_phase_ms(nullptr, ms); }
extern "C" int lcb_ecdsa_verify_hashed_dev(uint8_t *accept, const uint8_t *hashes, const uint8_t *sigs, size_t sig_len,
                                           const int32_t *key_idx, size_t n, const lcb_ecdsa_keyset *ks,
                                           int use_new_chain_id, int32_t chain_id, void *stream) {
    return lcb_ctx_ecdsa_verify_hashed_dev(nullptr, accept, hashes, sigs, sig_len, key_idx, n, ks, use_new_chain_id,
                                           chain_id, stream);
}
extern "C" int lcb_root_header_verify_dev(uint8_t *accept, const uint8_t *headers, uint64_t era, const uint8_t *sigs,
                                          size_t sig_len, const int32_t *key_idx, size_t n, const lcb_ecdsa_keyset *ks,
                                          int use_new_chain_id, int32_t chain_id, void *stream) {
    return lcb_ctx_root_header_verify_dev(nullptr, accept, headers, era, sigs, sig_len, key_idx, n, ks, use_new_chain_id,
                                          chain_id, stream);
}
extern "C" int lcb_ecdsa_verify_hashed_batch(uint8_t *accept, const uint8_t *hashes, const uint8_t *sigs, size_t sig_len,
                                             const uint8_t *pubkeys, size_t pk_len, size_t n_keys,
                                             const int32_t *key_idx, size_t n, int use_new_chain_id, int32_t chain_id) {
    return verify_host(accept, hashes, nullptr, 0, sigs, sig_len, pubkeys, pk_len, n_keys, key_idx, n, use_new_chain_id,
                       chain_id);
}
extern "C" int lcb_root_header_verify_batch(uint8_t *accept, const lcb_block_header *headers, uint64_t era,
                                            const uint8_t *sigs, size_t sig_len, const uint8_t *pubkeys, size_t pk_len,
                                            size_t n_keys, const int32_t *key_idx, size_t n, int use_new_chain_id,
                                            int32_t chain_id) {
    return verify_host(accept, nullptr, (const uint8_t *)headers, era, sigs, sig_len, pubkeys, pk_len, n_keys, key_idx,
                       n, use_new_chain_id, chain_id);
}
extern "C" int lcb_header_keccak_batch(uint8_t *hashes, const lcb_block_header *headers, size_t n) {
    lcb_ctx *c = ctx_sync();
    if (!c) return -1;
    if (!n) return 0;
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    uint8_t *dh = (uint8_t *)c->ec[3].get(112 * n), *dout = (uint8_t *)c->ec[1].get(32 * n), *po = (uint8_t *)c->ec[2].get(n);
    if (!dh || !dout || !po) { set_error("device allocation failed"); return -1; }
    hipMemcpyAsync(dh, headers, 112 * n, hipMemcpyHostToDevice, s);
    lcbk_secp_header_hash(s, dh, (u32)n, 0, dout, po);
    if (!launch_ok("header hash launch")) return -1;
    hipMemcpyAsync(hashes, dout, 32 * n, hipMemcpyDeviceToHost, s);
    return sync_ok(c, "header hash") ? 0 : -1;
}

// ------------------------------------------------------------------ signing side (key derivation, SignHashed with given
// nonces): input generation for tests and benches, and the root protocol's own header signature
extern "C" int lcb_ctx_ecdsa_pubkey_dev(lcb_ctx *ctx, uint8_t *out33, uint8_t *ok, const uint8_t *privs, size_t n,
                                        void *stream) {
    lcb_ctx *c = ctx_resolve(ctx);
    if (!c) return -1;
    Enq q(c, (hipStream_t)stream);
    if (!n) return 0;
    const void *gt = gen_table(q.s);
    if (!gt) return -1;
    lcbk_secp_pubkey(q.s, privs, (u32)n, gt, out33, ok);
    return launch_ok("ecdsa pubkey launch") ? 0 : -1;
}
extern "C" int lcb_ctx_ecdsa_sign_hashed_dev(lcb_ctx *ctx, uint8_t *sigs_out, uint8_t *ok, const uint8_t *hashes,
                                             const uint8_t *privs, const uint8_t *nonces, size_t n,
                                             int use_new_chain_id, int32_t chain_id, void *stream) {
    lcb_ctx *c = ctx_resolve(ctx);
    if (!c) return -1;
    Enq q(c, (hipStream_t)stream);
    if (!n) return 0;
    const void *gt = gen_table(q.s);
    if (!gt) return -1;
    lcbk_secp_sign(q.s, hashes, privs, nonces, (u32)n, gt, chain_id, use_new_chain_id, sigs_out, ok);
    return launch_ok("ecdsa sign launch") ? 0 : -1;
}
extern "C" int lcb_ecdsa_pubkey_dev(uint8_t *out33, uint8_t *ok, const uint8_t *privs, size_t n, void *stream) {
    return lcb_ctx_ecdsa_pubkey_dev(nullptr, out33, ok, privs, n, stream);
}
extern "C" int lcb_ecdsa_sign_hashed_dev(uint8_t *sigs_out, uint8_t *ok, const uint8_t *hashes, const uint8_t *privs,
                                         const uint8_t *nonces, size_t n, int use_new_chain_id, int32_t chain_id,
                                         void *stream) {
    return lcb_ctx_ecdsa_sign_hashed_dev(nullptr, sigs_out, ok, hashes, privs, nonces, n, use_new_chain_id, chain_id,
                                         stream);
}
// host-pointer forms
extern "C" int lcb_ecdsa_pubkey_batch(uint8_t *out33, uint8_t *ok, const uint8_t *privs, size_t n) {
    lcb_ctx *c = ctx_sync();
    if (!c) return -1;
    if (!n) return 0;
    Enq q(c, c->stream);
    uint8_t *dp = (uint8_t *)c->ec[3].get(32 * n), *dout = (uint8_t *)c->ec[4].get(34 * n);
    if (!dp || !dout) { set_error("device allocation failed"); return -1; }
    hipMemcpyAsync(dp, privs, 32 * n, hipMemcpyHostToDevice, c->stream);
    if (lcb_ctx_ecdsa_pubkey_dev(c, dout, dout + 33 * n, dp, n, c->stream)) return -1;
    hipMemcpyAsync(out33, dout, 33 * n, hipMemcpyDeviceToHost, c->stream);
    hipMemcpyAsync(ok, dout + 33 * n, n, hipMemcpyDeviceToHost, c->stream);
    return sync_ok(c, "ecdsa pubkey") ? 0 : -1;
}
extern "C" int lcb_ecdsa_sign_hashed_batch(uint8_t *sigs_out, uint8_t *ok, const uint8_t *hashes, const uint8_t *privs,
                                           const uint8_t *nonces, size_t n, int use_new_chain_id, int32_t chain_id) {
    lcb_ctx *c = ctx_sync();
    if (!c) return -1;
    if (!n) return 0;
    Enq q(c, c->stream);
    size_t L = use_new_chain_id ? 66 : 65;
    uint8_t *din = (uint8_t *)c->ec[3].get(96 * n), *dout = (uint8_t *)c->ec[4].get((L + 1) * n);
    if (!din || !dout) { set_error("device allocation failed"); return -1; }
    hipMemcpyAsync(din, hashes, 32 * n, hipMemcpyHostToDevice, c->stream);
    hipMemcpyAsync(din + 32 * n, privs, 32 * n, hipMemcpyHostToDevice, c->stream);
    hipMemcpyAsync(din + 64 * n, nonces, 32 * n, hipMemcpyHostToDevice, c->stream);
    if (lcb_ctx_ecdsa_sign_hashed_dev(c, dout, dout + L * n, din, din + 32 * n, din + 64 * n, n, use_new_chain_id,
                                      chain_id, c->stream))
        return -1;
    hipMemcpyAsync(sigs_out, dout, L * n, hipMemcpyDeviceToHost, c->stream);
    hipMemcpyAsync(ok, dout + L * n, n, hipMemcpyDeviceToHost, c->stream);
    return sync_ok(c, "ecdsa sign") ? 0 : -1;
}
