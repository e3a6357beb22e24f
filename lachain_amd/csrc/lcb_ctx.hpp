// lachain_amd/csrc/lcb_ctx.hpp — the library's per-caller execution context (host side, internal).
//
// An lcb_ctx owns every device workspace a batch call needs, so concurrent callers never share one: the TPKE
// and threshold-signature line sets are separate, and a *_prepared call checks the exact shape (keys,
// ciphertexts / messages) and generation its prepare recorded instead of a buffer capacity.  Work of one
// context is ordered by an event chain: every enqueue waits on the context's previous work and records a new
// event, so a workspace is never rewritten while a kernel on another stream still reads it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <mutex>
#include <vector>
#include <string>
#include <unordered_map>

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    void *get(size_t n) {
        if (n == 0) n = 16;
        if (n > cap) {
            if (p) (void)hipFree(p);
            p = nullptr;
            if (hipMalloc(&p, n) != hipSuccess) { cap = 0; p = nullptr; return nullptr; }
            cap = n;
        }
        return p;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct lcb_ctx {
    std::recursive_mutex mu;        // one enqueue at a time per context (contexts may be shared by threads)
    int device = 0;
    hipStream_t stream = nullptr;   // for the synchronous host-pointer entry points
    hipEvent_t order = nullptr;     // completion of the last work enqueued in this context
    bool order_valid = false;
    int enq_depth = 0;              // nesting of Enq scopes held by the owning thread
    size_t chunk = (size_t)1 << 21; // lcb_set_verify_chunk's value, read once per outermost enqueue (LCB_VERIFY_CHUNK)
    // TPKE workspace (lcb_*tpke_prepare_dev): line sets of H and W per ciphertext, validity, decompressed keys
    DevBuf t_lines, t_ctok, t_keys, t_f;
    DevBuf t_coop[3];                 // small exact batches on the cooperative kernels: point records, checks, flags
    // prepared-ciphertext cache of lcb_tpke_verify_shares_cached (line sets + validity per slot, keyed by the bytes)
    DevBuf cc_lines, cc_ok;
    std::unordered_map<std::string, uint32_t> cc_map;
    std::vector<std::string> cc_keys;
    std::vector<uint64_t> cc_used;
    uint64_t cc_tick = 0;
    int cc_flags = -1;
    // decompressed-key cache of the same entry point (an epoch's verification keys recur in every flush): one slot per
    // 48-byte key, filled in order; a call that would overflow it starts it afresh
    DevBuf kc_pts;
    std::unordered_map<std::string, uint32_t> kc_map;
    uint32_t kc_n = 0;
    size_t t_n_cts = 0, t_n_keys = 0;
    uint64_t t_gen = 0;
    bool t_ready = false;
    // threshold-signature workspace (lcb_*ts_prepare_dev): line sets of H(m) per message, keys
    DevBuf s_lines, s_mok, s_keys, s_f;
    DevBuf s_dec;                     // decoded shares of the batched CommonCoin checks (ts_share_st), for the assembly
    size_t s_dec_n = 0;
    size_t s_n_msgs = 0, s_n_pks = 0;
    uint64_t s_gen = 0;
    bool s_ready = false;
    // Lagrange / assembly / MSM / staging
    DevBuf lag[5], sel[4], msm[15], in[8], out[4], dkg[9];
    DevBuf lws;                       // lanetab.hpp workspaces of the persistent scalar-multiplication grids
    DevBuf mcl[10];                   // the mcl surface's pairing / multi-scalar / Horner / Lagrange staging
    // mclBn_pairing's cache of G2 line sets (pc_lines: slot k = Q_k's set and the infinity set), least recently used
    // slot replaced: the protocol pairs every share of a ciphertext / coin with the same H, W (TPKE/PublicKey.cs:91).
    // A buffer of its own: the other mcl calls' staging (mcl[]) must not overwrite cached sets between pairings
    DevBuf pc_lines;
    std::vector<uint32_t> pc_keys;    // 72 words (the mclBnG2 record) per slot
    std::vector<uint64_t> pc_used;    // last use (0: empty)
    uint64_t pc_tick = 0;
    hipEvent_t ver_ev[3] = {};
    bool ver_ev_ready = false, ver_ran = false;
    // randomized batch verification (k_batch.hip): r_i U_i / r_i Y_i records, group lists, group points, counts
    DevBuf rlc[20];                   // [12]: the keys' fixed-base tables, [13] suspect-key bitmap, [14] census validity,
                                      // [15] coop Miller fallback flags, [16] TPKE level-2 gamma_c / gamma_t rows, [17] its open groups,
                                      // [18] H's hash validity (split preparation, fork mode 3)
    hipEvent_t rlc_ev[3] = {};
    hipEvent_t rlc_lev_ev[4] = {};    // per level: before sum / Miller / final exp / resolve
    float rlc_ms[4] = {};             // accumulated over the levels of the last call: sums, Miller, final exp (+ resolve
                                      // / search), the fused call's preparation chain (0 for other calls)
    bool rlc_ev_ready = false, rlc_ran = false;
    uint32_t rlc_levels[8] = {};
    uint32_t rlc_census[4] = {};      // census shares, suspect keys, level-1 groups before / entries after the split
    int rlc_nlev = 0;
    uint64_t rlc_calls = 0;
    // which prepared line sets are not normalised (adversarial W): [0] the census's ciphertexts, [1] all; the one-lane
    // Miller fallback is dispatched only when the flag is set (round 5: an idle fallback dispatch waited ~15 ms for a
    // SIMD with 360 free registers behind the randomisation).  Device words, pinned copies, events after the copies.
    DevBuf unn;
    uint32_t *unn_pin = nullptr;
    hipEvent_t unn_ev[2] = {};
    bool unn_set[2] = {false, false};
    int unn_census = 1;               // the flag the census reads: 0 when its ciphertexts were prepared first (split)
    hipStream_t aux = nullptr;        // second stream of the fused batched verify (randomisation beside preparation)
    hipStream_t hi = nullptr;         // high-priority stream: the latency-bound preparation chain (lcb_set_fork_mode 1)
    hipStream_t hi2 = nullptr;        // second high-priority stream: U / W decompression + W's line sets (fork mode 3)
    hipStream_t hi3 = nullptr;        // third: the bulk of the split preparation when the census ciphertexts go first
    hipEvent_t fork_ev[5] = {};
    hipEvent_t prep_ev[3] = {};       // timed: the fused call's preparation chain (stats ms[5]); [2] after the hashing
    bool prep_timed = false;
    bool fork_ready = false;
    hipEvent_t msm_ev[7] = {};
    bool msm_ev_ready = false, msm_ran = false;
    // secp256k1 ECDSA (lcb_ecdsa.cpp): job records / header hashes / staging, and the host API's cached key set
    DevBuf ec[6];
    hipEvent_t ec_ev[4] = {};         // around header hash / scalars / verify of the last verification
    bool ec_ev_ready = false, ec_ran = false, ec_hashed = false;
    struct lcb_ecdsa_keyset *ec_cache = nullptr;
    std::vector<uint8_t> ec_cache_keys;
    size_t ec_cache_pk_len = 0;
};

// Enqueue scope: exclusive use of the context, stream ordered after the context's previous work, and the
// context's order event recorded after this call's work.  The outermost scope snapshots the verify chunk, so a call
// sizes its park buffers and steps its chunk loops with one value even if lcb_set_verify_chunk runs meanwhile.
size_t lcb_verify_chunk_now();
struct Enq {
    lcb_ctx *c;
    hipStream_t s;
    std::unique_lock<std::recursive_mutex> lk;
    Enq(lcb_ctx *c_, hipStream_t s_) : c(c_), s(s_), lk(c_->mu) {
        if (c->enq_depth++ == 0) c->chunk = lcb_verify_chunk_now();
        if (c->order_valid) (void)hipStreamWaitEvent(s, c->order, 0);
    }
    ~Enq() {
        if (hipEventRecord(c->order, s) == hipSuccess) c->order_valid = true;
        --c->enq_depth;
    }
};
