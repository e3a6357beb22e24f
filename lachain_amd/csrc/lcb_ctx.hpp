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
    // TPKE workspace (lcb_*tpke_prepare_dev): line sets of H and W per ciphertext, validity, decompressed keys
    DevBuf t_lines, t_ctok, t_keys, t_f;
    size_t t_n_cts = 0, t_n_keys = 0;
    uint64_t t_gen = 0;
    bool t_ready = false;
    // threshold-signature workspace (lcb_*ts_prepare_dev): line sets of H(m) per message, keys
    DevBuf s_lines, s_mok, s_keys, s_f;
    size_t s_n_msgs = 0, s_n_pks = 0;
    uint64_t s_gen = 0;
    bool s_ready = false;
    // Lagrange / assembly / MSM / staging
    DevBuf lag[3], sel[3], msm[12], in[8], out[4], dkg[6];
    hipEvent_t ver_ev[3] = {};
    bool ver_ev_ready = false, ver_ran = false;
    hipEvent_t msm_ev[7] = {};
    bool msm_ev_ready = false, msm_ran = false;
};
