// lachain_amd/csrc/lcb_host.cpp — host implementation of include/lachain_bls.h (liblachain_bls.so).
//
// Batch work (share verification, Lagrange combination, MSM, scalar multiplications, pairings, hashing to G2) runs
// on gfx950 kernels (k_*.hip).  The mcl single-element calls that are O(1) field work — Fr arithmetic (fr_host.hpp)
// and G1 / G2 add, sub, neg, dbl, normalize, compare, validity, (de)serialization, GT products (fp_host.hpp) — run on
// the calling thread, word for word the kernels' formulas, because a GPU round trip costs 50-100x the operation.
// There is deliberately no CPU fallback for the GPU work: without a gfx950 device mclBn_init returns -1 and every
// entry point fails (returns -1 / 0 bytes / leaves outputs zeroed) with lcb_last_error() describing why.
//
// Concurrency model (the reference calls mcl from one thread per consensus protocol,
// /root/reference/src/Lachain.Consensus/AbstractProtocol.cs:46-47):
//   * scalar Fr arithmetic runs on the host (fr_host.hpp); every other single-element mcl operation is a GPU round trip
//     on the calling thread's own staging buffers and stream (no process-wide lock), and the pairing, multi-scalar
//     products, Lagrange interpolation and polynomial evaluation go to batch / cooperative kernels;
//   * every batch entry point runs in an lcb_ctx — explicit (lcb_ctx_*) or the calling thread's own default
//     context — which owns all device workspaces the call needs (TPKE and TS line sets separately, Lagrange,
//     MSM, staging).  A context's work executes in the order it was enqueued whatever stream it is enqueued on
//     (each call waits on the context's last event and records a new one), and a *_prepared call checks the
//     exact batch shape its prepare recorded, so no two callers can read or overwrite each other's workspace.
//   * the HIP device is bound per calling thread (lcb_set_device applies to every thread that enters).
#include <hip/hip_runtime.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include <mutex>
#include <atomic>
#include <vector>
#include <string>
#include <algorithm>
#include <sys/random.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include "launch.h"
#include "bls_constants_host.h"
#include "../../include/lachain_bls.h"
#include "host_sha3.hpp"
#include "lcb_ctx.hpp"
#include "lcb_internal.hpp"
#include "fr_host.hpp"
#include "fp_host.hpp"

#define LCB_BLOCK 256

namespace {

std::mutex g_mu;               // device initialisation
int g_device = 0;
bool g_ready = false;
int g_orig_cofactor = 0;
const size_t IO_WORDS = 4096; // 16 KB staging per thread
thread_local std::string g_err;
thread_local uint64_t g_err_count = 0;   // failures on this thread (lcb_error_count): the void mcl entry points have no
                                         // return code, so a caller detects their failure by this counter changing
thread_local int t_bound_device = -1;

void set_err(const char *what, hipError_t e = hipSuccess) {
    char buf[256];
    if (e != hipSuccess) snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    else snprintf(buf, sizeof buf, "%s", what);
    g_err = buf;
    g_err_count++;
}

// opt-in switches read from the environment at call time: the tuning hooks (lcb_set_coop_max, ...) change the kernel
// families a batch runs on and the fault-injection hooks make calls fail; neither belongs in a production process
bool env_on(const char *name) {
    const char *e = getenv(name);
    return e && e[0] == '1';
}
bool tuning_allowed(const char *what) {
    if (env_on("LCB_ALLOW_TUNING")) return true;
    set_err((std::string(what) + ": tuning hooks need LCB_ALLOW_TUNING=1").c_str());
    return false;
}
// fault injection (lcb_test_inject_failure, LCB_ALLOW_TEST_HOOKS=1): the next `count` passes through site `site` fail
std::atomic<int> g_inject_site{0}, g_inject_count{0};
bool injected(int site) {
    if (g_inject_site.load(std::memory_order_relaxed) != site) return false;
    int c = g_inject_count.load();
    while (c > 0)
        if (g_inject_count.compare_exchange_weak(c, c - 1)) return true;
    return false;
}
enum { INJ_STAGE_HOST_ALLOC = 1, INJ_CT_CACHE_ALLOC = 2, INJ_PAIRING_ALLOC = 3, INJ_STAGE_OP = 4 };
bool inject_armed(int site) {             // a pending failure at `site` (not consumed)
    return g_inject_site.load(std::memory_order_relaxed) == site && g_inject_count.load() > 0;
}

// the output of a failed void mcl call (mclBnG1_mul, mclBn_pairing, ...): random words with the top limb of the first
// coordinate set to all ones, so it is not a canonical field element (isValid / serialize reject it), and two failed
// calls never compare equal (an equality check between two failed pairings cannot pass)
void fail_out(void *out, size_t bytes) {
    uint8_t *b = (uint8_t *)out;
    size_t got = 0;
    while (got < bytes) {
        ssize_t r = getrandom(b + got, bytes - got, 0);
        if (r <= 0) break;
        got += (size_t)r;
    }
    for (size_t i = got; i < bytes; i++) b[i] = (uint8_t)(0x5a ^ i);
    if (bytes >= 48) memset(b + 44, 0xff, 4);
}

// HIP's current device is per thread: bind every thread that enters the library to the configured device
bool bind_thread() {
    if (t_bound_device == g_device) return true;
    hipError_t e = hipSetDevice(g_device);
    if (e != hipSuccess) { set_err("hipSetDevice", e); return false; }
    t_bound_device = g_device;
    return true;
}

bool init_locked() {
    if (g_ready) return bind_thread();
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= g_device) { set_err("no HIP device", e); return false; }
    if (!bind_thread()) return false;
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, g_device)) != hipSuccess) { set_err("hipGetDeviceProperties", e); return false; }
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) { set_err("device is not gfx950"); return false; }
    g_ready = true;
    return true;
}

// the library is usable from this thread (device opened once per process, bound once per thread)
bool ready() {
    if (g_ready && t_bound_device == g_device) return true;
    std::lock_guard<std::mutex> lk(g_mu);
    return init_locked();
}

// single-element operations: every calling thread owns its staging (device and pinned host buffers, a stream), so the
// protocol threads (AbstractProtocol.cs:46-47) never queue behind each other's round trips
// A thread's staging and implicit contexts are NOT released when it exits: HIP calls from thread-local destructors
// race the runtime's (and a profiler's) own per-thread teardown (an abort under rocprofv3 in round 4).  They are
// retired to process-wide free lists instead and handed to the next thread that needs one, so their number stays
// bounded by the peak number of calling threads.  The lists are leaked on purpose (no static-destruction order issue).
struct StageRes {
    u32 *dev = nullptr, *host = nullptr;
    hipStream_t s = nullptr;
};
std::mutex &retired_mu() {
    static std::mutex *m = new std::mutex;
    return *m;
}
std::vector<StageRes> &retired_stages() {
    static std::vector<StageRes> *v = new std::vector<StageRes>;
    return *v;
}
struct OpStage : StageRes {
    ~OpStage() {
        if (!(s && dev && host)) return;             // a half-built stage never survives stage_ready
        std::lock_guard<std::mutex> lk(retired_mu());
        retired_stages().push_back(*this);
    }
};
thread_local OpStage t_stage;
bool stage_ready() {
    if (!ready()) return false;
    if (t_stage.s && t_stage.dev && t_stage.host) return true;
    {
        std::lock_guard<std::mutex> lk(retired_mu());
        auto &v = retired_stages();
        // (a pending staging-allocation failure builds a new stage, so the test hook reaches the allocation)
        if (!v.empty() && !t_stage.s && !t_stage.dev && !t_stage.host && !inject_armed(INJ_STAGE_HOST_ALLOC)) {
            static_cast<StageRes &>(t_stage) = v.back();
            v.pop_back();
            return true;
        }
    }
    // all three or none: a partial failure releases what was created, so the next call retries from scratch instead
    // of passing a half-built stage (a set stream with a null host buffer would be written through)
    hipError_t e = t_stage.s ? hipSuccess : hipStreamCreateWithFlags(&t_stage.s, hipStreamNonBlocking);
    if (e == hipSuccess && !t_stage.dev) e = hipMalloc(&t_stage.dev, IO_WORDS * 4);
    if (e == hipSuccess && !t_stage.host) {
        if (injected(INJ_STAGE_HOST_ALLOC)) e = hipErrorOutOfMemory;
        else e = hipHostMalloc(&t_stage.host, IO_WORDS * 4, hipHostMallocDefault);
    }
    if (e != hipSuccess) {
        set_err("single-operation staging", e);
        if (t_stage.host) (void)hipHostFree(t_stage.host);
        if (t_stage.dev) (void)hipFree(t_stage.dev);
        if (t_stage.s) (void)hipStreamDestroy(t_stage.s);
        t_stage.host = nullptr;
        t_stage.dev = nullptr;
        t_stage.s = nullptr;
        return false;
    }
    return true;
}
#define IOH (t_stage.host)

// run one k_op on the thread's staging buffer: copy `in_words` words to the device, launch, copy `out_words` back
bool run_op(int op, size_t in_words, size_t out_words) {
    hipError_t e;
    if (injected(INJ_STAGE_OP)) { set_err("injected failure (single operation)"); return false; }
    if ((e = hipMemcpyAsync(t_stage.dev, t_stage.host, in_words * 4, hipMemcpyHostToDevice, t_stage.s)) != hipSuccess) { set_err("H2D", e); return false; }
    lcbk_op(dim3(1), t_stage.s, op, t_stage.dev, g_orig_cofactor);
    if ((e = hipGetLastError()) != hipSuccess) { set_err("k_op launch", e); return false; }
    if ((e = hipMemcpyAsync(t_stage.host, t_stage.dev, out_words * 4, hipMemcpyDeviceToHost, t_stage.s)) != hipSuccess) { set_err("D2H", e); return false; }
    if ((e = hipStreamSynchronize(t_stage.s)) != hipSuccess) { set_err("k_op", e); return false; }
    return true;
}

// mclBnG2_hashAndMapTo's round trip: as run_op, on the dedicated one-lane hash kernel (k_ptmul.hip)
bool run_hash(size_t in_words, size_t out_words) {
    hipError_t e;
    if (injected(INJ_STAGE_OP)) { set_err("injected failure (single operation)"); return false; }
    if ((e = hipMemcpyAsync(t_stage.dev, t_stage.host, in_words * 4, hipMemcpyHostToDevice, t_stage.s)) != hipSuccess) { set_err("H2D", e); return false; }
    lcbk_mcl_g2_hash(t_stage.s, t_stage.dev, g_orig_cofactor);
    if ((e = hipGetLastError()) != hipSuccess) { set_err("k_mcl_g2_hash launch", e); return false; }
    if ((e = hipMemcpyAsync(t_stage.host, t_stage.dev, out_words * 4, hipMemcpyDeviceToHost, t_stage.s)) != hipSuccess) { set_err("D2H", e); return false; }
    if ((e = hipStreamSynchronize(t_stage.s)) != hipSuccess) { set_err("k_mcl_g2_hash", e); return false; }
    return true;
}

#define LOCKED_OR(ret)                        \
    if (!stage_ready()) return ret;

inline u32 nblk(size_t n) { return (u32)((n + LCB_BLOCK - 1) / LCB_BLOCK); }

// canonical Fr bytes (32-byte LE < r)
bool fr_bytes_lt_r(const uint8_t *b) {
    for (int j = 7; j >= 0; j--) {
        uint32_t w = (uint32_t)b[4 * j] | (uint32_t)b[4 * j + 1] << 8 | (uint32_t)b[4 * j + 2] << 16 | (uint32_t)b[4 * j + 3] << 24;
        if (w != LCB_R_HOST[j]) return w < LCB_R_HOST[j];
    }
    return false;
}

} // namespace

// ================================================================== init / config
extern "C" int lcb_set_device(int id) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ready) return id == g_device ? 0 : -1;
    g_device = id;
    return 0;
}
extern "C" int lcb_get_device(void) { return g_device; }
extern "C" void lcb_set_original_g2_cofactor(int enable) { g_orig_cofactor = enable != 0; }
int g_line_mode = 0;   // 1: prepare marks every line set un-normalised (test hook for the on-the-fly fallback)
extern "C" int lcb_set_line_mode(int general) {
    if (!tuning_allowed("lcb_set_line_mode")) return -1;
    g_line_mode = general != 0;
    return 0;
}
extern "C" const char *lcb_last_error(void) { return g_err.c_str(); }

// ================================================================== the scratch gate (gate.hpp LCB_LAUNCH_GATED)
// What the runtime does with a dispatch's private segment (ROCr's queue scratch handler; hsa_ext_amd.h:686-703 for the
// two agent limits, measured on the box in profiles/r06/scratch_limits.txt): the per-lane size S is rounded up to 16 B
// (a wave's 1 KB granule) and the FULL-device size  full(S) = S x 64 lanes x CUs x wave slots per CU  is requested for
// the dispatch's hardware queue.  When full(S) <= the agent's async scratch limit (HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_
// CURRENT) the memory stays BOUND to that queue after the dispatch and serves its later dispatches; above it, it is a
// use-once allocation of the dispatch's own size, released when the dispatch retires.  All queues share one pool
// (SCRATCH_LIMIT_MAX).  A use-once request that does not fit waits while another use-once allocation is outstanding;
// a request that finds the pool held by bound reservations of busy queues aborts the process with
// HSA_STATUS_ERROR_OUT_OF_RESOURCES (the round-5 aborts: DESIGN.md §14.1).
// Measured on the box (profiles/r06/scratch_limits.txt): pool 32 GiB, bind limit 24 GiB, 256 CUs x 32 slots — every
// kernel of this library binds (the largest, k_op_gt at 8,148 B per lane, binds 4.27 GB), so the sum of the
// hardware queues' bound reservations is what must stay within the pool.  HIP keeps GPU_MAX_HW_QUEUES queues per stream
// priority and the library uses two priorities (the preparation chains run on high-priority streams), so a process
// holds up to Q = 2 x GPU_MAX_HW_QUEUES queues: 8 at the box's default 4, 16 when a caller raises it to 8 (the round-5
// bench did: 16 queues x up to 2.5 GB bound by the preparation lanes exceed the 32 GiB pool — the aborts).
// The gate therefore bounds the bound reservations: a launch whose full(S) exceeds the per-queue share
// T = (pool - LCB_GATE_RESERVE) / Q runs on one process-wide stream per device, ordered with the caller's stream by
// events, so every other queue binds <= T and the gate's queue at most LCB_GATE_RESERVE (>= every kernel's full(S):
// tests/test_kernel_resources.py), and  Q x T + reserve <= pool.  At Q = 8: T = 3.44 GiB, and only the single-lane
// mcl-surface / debug kernels (> 6.7 KB per lane) are routed; at Q = 16 the pairing kernels above ~3.5 KB are too.
// Launches whose scratch is use-once (full(S) above the bind limit) are left on the caller's stream.
#define LCB_GATE_RESERVE (9ull << 29)                 // 4.5 GiB: the gate queue's bound reservation, >= every kernel's full(S)
namespace {
struct GateDev {
    std::mutex mu, init_mu;
    hipStream_t s = nullptr;
    hipEvent_t in = nullptr, out = nullptr;
    std::atomic<int> ready{0};
    uint64_t slots = 0;           // CUs x wave slots per CU
    uint64_t pool = 0;            // HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX (0: unknown)
    uint64_t bind_limit = 0;      // HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_CURRENT (0: unknown: every full(S) binds)
    uint64_t per_queue = 0;       // T
    int hwq = 8;                  // hardware queues the process may hold (both priorities)
};
GateDev g_gate[64];
std::atomic<long long> g_gate_bytes{-2};            // -2: not read from LCB_SCRATCH_GATE_MB yet; -3: the model's T
std::atomic<unsigned long long> g_gate_routed{0}, g_gate_seen{0};
thread_local int t_gate_dev = -1;                   // device whose gate mutex this thread holds (-1: none)
long long gate_override() {
    long long v = g_gate_bytes.load(std::memory_order_relaxed);
    if (v != -2) return v;
    const char *e = getenv("LCB_SCRATCH_GATE_MB");
    v = e && *e ? atoll(e) * (1ll << 20) : -3;
    long long expect = -2;
    g_gate_bytes.compare_exchange_strong(expect, v);
    return g_gate_bytes.load();
}
struct HsaFind { int want, seen; hsa_agent_t agent; bool found; };
hsa_status_t hsa_find_gpu(hsa_agent_t a, void *d) {
    HsaFind *f = (HsaFind *)d;
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
        return HSA_STATUS_SUCCESS;
    if (f->seen++ == f->want) { f->agent = a; f->found = true; return HSA_STATUS_INFO_BREAK; }
    return HSA_STATUS_SUCCESS;
}
// the device's scratch model, read once (HIP device ordinal i = the i-th GPU agent of the runtime)
void gate_model(GateDev &g, int dev) {
    if (g.ready.load(std::memory_order_acquire)) return;
    std::lock_guard<std::mutex> lk(g.init_mu);
    if (g.ready.load()) return;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    uint32_t wpc = 0;
    HsaFind f{dev, 0, {0}, false};
    if (hsa_init() == HSA_STATUS_SUCCESS) {
        hsa_iterate_agents(hsa_find_gpu, &f);
        if (f.found) {
            uint64_t v = 0;
            if (hsa_agent_get_info(f.agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX, &v) == HSA_STATUS_SUCCESS) g.pool = v;
            v = 0;
            if (hsa_agent_get_info(f.agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_CURRENT, &v) == HSA_STATUS_SUCCESS) g.bind_limit = v;
            if (hsa_agent_get_info(f.agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_MAX_WAVES_PER_CU, &wpc) != HSA_STATUS_SUCCESS) wpc = 0;
        }
        hsa_shut_down();
    }
    g.slots = (uint64_t)cus * (wpc ? wpc : 32);
    const char *q = getenv("GPU_MAX_HW_QUEUES");
    g.hwq = 2 * (q && atoi(q) > 0 ? atoi(q) : 4);      // queues per priority x the two priorities the library uses
    // unknown pool: assume the measured 32 GiB rather than none
    const uint64_t pool = g.pool ? g.pool : (32ull << 30);
    g.per_queue = pool > LCB_GATE_RESERVE ? (pool - LCB_GATE_RESERVE) / (uint64_t)g.hwq : 0;
    g.ready.store(1, std::memory_order_release);
}
}  // namespace
extern "C" hipStream_t lcb_gate_enter(const void *kern, long long *scratch_cache, size_t lanes, hipStream_t s) {
    long long sc = __atomic_load_n(scratch_cache, __ATOMIC_RELAXED);
    if (sc < 0) {
        hipFuncAttributes a;
        sc = hipFuncGetAttributes(&a, kern) == hipSuccess ? (long long)a.localSizeBytes : 0;
        __atomic_store_n(scratch_cache, sc, __ATOMIC_RELAXED);
    }
    g_gate_seen.fetch_add(1, std::memory_order_relaxed);
    const long long ovr = gate_override();
    if (sc == 0 || ovr == -1 || lanes == 0) return s;
    int dev = -1;
    if (hipStreamGetDevice(s, &dev) != hipSuccess || dev < 0) {          // (the caller's stream decides the device)
        if (hipGetDevice(&dev) != hipSuccess) return s;
    }
    if (dev < 0 || dev >= 64) return s;
    GateDev &g = g_gate[dev];
    gate_model(g, dev);
    const uint64_t per_lane = ((uint64_t)sc + 15) & ~(uint64_t)15;
    const uint64_t full = per_lane * 64 * g.slots;
    const bool binds = g.bind_limit == 0 || full <= g.bind_limit;
    const uint64_t thr = ovr >= 0 ? (uint64_t)ovr : g.per_queue;
    if (ovr != 0 && !(binds && full > thr)) return s;   // (override 0: every launch with scratch is routed)
    g.mu.lock();
    if (!g.s) {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (cur != dev) (void)hipSetDevice(dev);
        if (hipStreamCreateWithFlags(&g.s, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&g.in, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&g.out, hipEventDisableTiming) != hipSuccess)
            g.s = nullptr;
        if (cur >= 0 && cur != dev) (void)hipSetDevice(cur);
        if (!g.s) {                   // (the launch stays on the caller's stream)
            g.mu.unlock();
            return s;
        }
    }
    t_gate_dev = dev;
    g_gate_routed.fetch_add(1, std::memory_order_relaxed);
    (void)hipEventRecord(g.in, s);
    (void)hipStreamWaitEvent(g.s, g.in, 0);
    return g.s;
}
extern "C" void lcb_gate_exit(hipStream_t s, hipStream_t used) {
    if (used == s || t_gate_dev < 0) return;
    GateDev &g = g_gate[t_gate_dev];
    (void)hipEventRecord(g.out, used);
    (void)hipStreamWaitEvent(s, g.out, 0);
    t_gate_dev = -1;
    g.mu.unlock();
}
// the scratch model of the calling thread's device: out[0] pool, [1] bind limit, [2] wave slots, [3] hardware queues,
// [4] the per-queue share T, [5] the gate threshold in force (-1 off)
extern "C" int lcb_scratch_info(uint64_t out[6]) {
    int dev = 0;
    if (!out || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
    GateDev &g = g_gate[dev];
    gate_model(g, dev);
    const long long ovr = gate_override();
    out[0] = g.pool;
    out[1] = g.bind_limit;
    out[2] = g.slots;
    out[3] = (uint64_t)g.hwq;
    out[4] = g.per_queue;
    out[5] = ovr == -1 ? ~0ull : ovr >= 0 ? (uint64_t)ovr : g.per_queue;
    return 0;
}
// tuning / test hook: the gate's threshold in bytes of reservation (-1: off, 0: every launch with scratch is routed)
extern "C" int lcb_set_scratch_gate(long long bytes) {
    if (!tuning_allowed("lcb_set_scratch_gate")) return -1;
    gate_override();
    g_gate_bytes.store(bytes < -1 ? -3 : bytes);    // < -1: back to the model's per-queue share
    return 0;
}
// test hook: at most this many blocks in the persistent grids (lanetab.hpp workspaces), so a small batch walks several
// items per lane; 0 = as many as are resident
std::atomic<uint32_t> g_persist_cap{0};
extern "C" uint32_t lcb_persist_cap(void) { return g_persist_cap.load(std::memory_order_relaxed); }
extern "C" int lcb_set_persist_blocks(uint32_t max_blocks) {
    if (!tuning_allowed("lcb_set_persist_blocks")) return -1;
    g_persist_cap.store(max_blocks);
    return 0;
}
extern "C" void lcb_scratch_gate_stats(uint64_t *routed, uint64_t *seen) {
    if (routed) *routed = g_gate_routed.load();
    if (seen) *seen = g_gate_seen.load();
}

extern "C" int mclBn_init(int curve, int compiledTimeVar) {
    if (curve != MCL_BLS12_381 || compiledTimeVar != MCLBN_COMPILED_TIME_VAR) {
        set_err("unsupported curve / compiledTimeVar");
        return -1;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    return init_locked() ? 0 : -1;
}
extern "C" int mclBn_getOpUnitSize(void) { return 6; }
extern "C" int mclBn_getG1ByteSize(void) { return 48; }
extern "C" int mclBn_getFrByteSize(void) { return 32; }
extern "C" int mclBn_getFpByteSize(void) { return 48; }

// ================================================================== Fr (host arithmetic, fr_host.hpp)
static inline const uint64_t *FRV(const mclBnFr *x) { return (const uint64_t *)x; }
static inline uint64_t *FRW(mclBnFr *x) { return (uint64_t *)x; }
static int fr_set_raw(mclBnFr *y, const u32 raw[8]) {
    uint64_t r[4];
    memcpy(r, raw, 32);
    if (!frh::lt_r(r)) { memset(y, 0, 32); return -1; }
    frh::from_raw(FRW(y), r);
    return 0;
}
static int fr_get_raw(u32 raw[8], const mclBnFr *x) {
    uint64_t r[4];
    frh::to_raw(r, FRV(x));
    memcpy(raw, r, 32);
    return 0;
}
extern "C" int mclBnFr_setInt(mclBnFr *y, mclInt x) {
    u32 raw[8] = {0};
    uint64_t ax = x < 0 ? (uint64_t)(-(x + 1)) + 1 : (uint64_t)x;
    raw[0] = (u32)ax; raw[1] = (u32)(ax >> 32);
    if (fr_set_raw(y, raw)) return -1;
    if (x < 0) mclBnFr_neg(y, y);
    return 0;
}
extern "C" int mclBnFr_setInt32(mclBnFr *y, int x) { return mclBnFr_setInt(y, x); }
extern "C" int mclBnFr_setByCSPRNG(mclBnFr *x) {
    // rejection sampling of a uniform 255-bit value < r
    for (int tries = 0; tries < 64; tries++) {
        u32 raw[8];
        if (getrandom(raw, sizeof raw, 0) != (ssize_t)sizeof raw) return -1;
        raw[7] &= 0x7fffffffu;
        if (fr_set_raw(x, raw) == 0) return 0;
    }
    return -1;
}
extern "C" int mclBnFr_setLittleEndian(mclBnFr *x, const void *buf, mclSize n) {
    // mcl setArrayMask: take at most 32 bytes, mask to 255 bits, and to 254 if still >= r
    u32 raw[8] = {0};
    memcpy(raw, buf, n < 32 ? n : 32);
    raw[7] &= 0x7fffffffu;
    uint64_t r[4];
    memcpy(r, raw, 32);
    if (!frh::lt_r(r)) raw[7] &= 0x3fffffffu;
    return fr_set_raw(x, raw);
}
extern "C" mclSize mclBnFr_serialize(void *buf, mclSize max, const mclBnFr *x) {
    if (max < 32) return 0;
    u32 raw[8];
    fr_get_raw(raw, x);
    memcpy(buf, raw, 32);
    return 32;
}
extern "C" mclSize mclBnFr_deserialize(mclBnFr *x, const void *buf, mclSize n) {
    if (n < 32) return 0;
    u32 raw[8];
    memcpy(raw, buf, 32);
    return fr_set_raw(x, raw) == 0 ? 32 : 0;
}
extern "C" void mclBnFr_clear(mclBnFr *x) { memset(x, 0, sizeof *x); }
extern "C" int mclBnFr_isValid(const mclBnFr *x) { return frh::lt_r(FRV(x)); }
extern "C" int mclBnFr_isEqual(const mclBnFr *x, const mclBnFr *y) { return memcmp(x, y, 32) == 0; }
extern "C" int mclBnFr_isZero(const mclBnFr *x) { return frh::is_zero(FRV(x)); }
extern "C" int mclBnFr_isOne(const mclBnFr *x) { return memcmp(x, frh::ONE, 32) == 0; }
extern "C" void mclBnFr_neg(mclBnFr *y, const mclBnFr *x) { frh::neg(FRW(y), FRV(x)); }
extern "C" void mclBnFr_inv(mclBnFr *y, const mclBnFr *x) { frh::inv(FRW(y), FRV(x)); }
extern "C" void mclBnFr_sqr(mclBnFr *y, const mclBnFr *x) { frh::mul(FRW(y), FRV(x), FRV(x)); }
extern "C" void mclBnFr_add(mclBnFr *z, const mclBnFr *x, const mclBnFr *y) { frh::add(FRW(z), FRV(x), FRV(y)); }
extern "C" void mclBnFr_sub(mclBnFr *z, const mclBnFr *x, const mclBnFr *y) { frh::sub(FRW(z), FRV(x), FRV(y)); }
extern "C" void mclBnFr_mul(mclBnFr *z, const mclBnFr *x, const mclBnFr *y) { frh::mul(FRW(z), FRV(x), FRV(y)); }
extern "C" void mclBnFr_div(mclBnFr *z, const mclBnFr *x, const mclBnFr *y) {
    mclBnFr t;
    mclBnFr_inv(&t, y);
    mclBnFr_mul(z, x, &t);
}

// ================================================================== G1 / G2 (host field work, fp_host.hpp)
// O(1) field work runs on the host like Fr (fp_host.hpp header); G1 / G2 multiplication, the hash to G2 and the
// pairing below stay on the GPU.  Bit-identical to the kernels' results (same formulas, fully reduced residues).
static void g1_op(int op, mclBnG1 *z, const mclBnG1 *x, const mclBnG1 *y, const mclBnFr *k) {
    if (!stage_ready()) { fail_out(z, 144); return; }
    memcpy(IOH + 36, x, 144);
    if (y) memcpy(IOH + 72, y, 144);
    if (k) memcpy(IOH + 108, k, 32);
    if (run_op(op, 116, 36)) memcpy(z, IOH, 144);
    else fail_out(z, 144);
}
std::atomic<int> g_g2_sign_b{0};      // lcb_set_g2_sign_from_b: the G2 wire flag is parity(y.b) instead of parity(y.a)
static inline fph::g1 *G1W(mclBnG1 *x) { return (fph::g1 *)x; }
static inline const fph::g1 *G1R(const mclBnG1 *x) { return (const fph::g1 *)x; }
static inline fph::g2 *G2W(mclBnG2 *x) { return (fph::g2 *)x; }
static inline const fph::g2 *G2R(const mclBnG2 *x) { return (const fph::g2 *)x; }
extern "C" mclSize mclBnG1_serialize(void *buf, mclSize max, const mclBnG1 *x) {
    if (max < 48) return 0;
    fph::g1_compress((uint8_t *)buf, *G1R(x));
    return 48;
}
extern "C" mclSize mclBnG1_deserialize(mclBnG1 *x, const void *buf, mclSize n) {
    if (n < 48) return 0;
    fph::g1a a;
    if (!fph::g1_decompress(a, (const uint8_t *)buf)) return 0;
    fph::jac_from_aff(*G1W(x), a);
    return 48;
}
extern "C" int mclBnG1_isValid(const mclBnG1 *x) { return fph::jac_valid(*G1R(x)); }
extern "C" int mclBnG1_isEqual(const mclBnG1 *x, const mclBnG1 *y) { return fph::jac_eq(*G1R(x), *G1R(y)); }
extern "C" int mclBnG1_isZero(const mclBnG1 *x) {
    static const u32 z[12] = {0};
    return memcmp(&x->z, z, 48) == 0;
}
extern "C" void mclBnG1_clear(mclBnG1 *x) { memset(x, 0, sizeof *x); }
extern "C" void mclBnG1_neg(mclBnG1 *y, const mclBnG1 *x) { fph::jac_neg(*G1W(y), *G1R(x)); }
extern "C" void mclBnG1_dbl(mclBnG1 *y, const mclBnG1 *x) { fph::g1 t; fph::jac_dbl(t, *G1R(x)); *G1W(y) = t; }
extern "C" void mclBnG1_normalize(mclBnG1 *y, const mclBnG1 *x) { fph::jac_normalize(*G1W(y), *G1R(x)); }
extern "C" void mclBnG1_add(mclBnG1 *z, const mclBnG1 *x, const mclBnG1 *y) {
    fph::g1 t;
    fph::jac_add(t, *G1R(x), *G1R(y));
    *G1W(z) = t;
}
extern "C" void mclBnG1_sub(mclBnG1 *z, const mclBnG1 *x, const mclBnG1 *y) {
    fph::g1 ny, t;
    fph::jac_neg(ny, *G1R(y));
    fph::jac_add(t, *G1R(x), ny);
    *G1W(z) = t;
}
// ---- mclBnG1_mul / mclBnG2_mul: the cooperative ladders of k_ptmul.hip (four lanes per ladder, several ladders per
// wave) on the scalar split below, the result assembled here; a base point outside the subgroup (the split is only
// valid on it) takes the exact one-lane ladder of k_op
struct PtJobG1 { u32 x[12], y[12], inf, nwin, pad[2]; uint8_t nib[36]; };
struct PtJobG2 { u32 x[24], y[24], inf, nwin, pad[2]; uint8_t nib[36]; };
static_assert(sizeof(PtJobG1) == 148 && sizeof(PtJobG2) == 244, "k_ptmul.hip PtJob layouts");
typedef unsigned __int128 u128h;
static const uint64_t Z_ABS_H = 0xd201000000010000ull;
// q <- q / u (256-bit), returns q mod u
static uint64_t divmod_u(uint64_t q[4]) {
    u128h rem = 0;
    for (int i = 3; i >= 0; i--) {
        u128h cur = rem << 64 | q[i];
        q[i] = (uint64_t)(cur / Z_ABS_H);
        rem = cur % Z_ABS_H;
    }
    return (uint64_t)rem;
}
// nwin signed 4-bit digits of the little-endian words v (nw 64-bit words), most significant first: each window's
// nibble plus the carry, minus 16 (carry 1) when above 8, so every digit is in [-7, 8] and k_ptmul.hip's table holds
// T[1..8].  A byte is |digit| with bit 7 set for a negative digit.  False if a carry leaves the top window (the
// callers size nwin so that it cannot: 33 windows for < 2^129, 17 for one 64-bit word).
template <class J> static bool put_digits(J &job, const uint64_t *v, int nw, u32 nwin) {
    job.nwin = nwin;
    int carry = 0;
    for (u32 i = 0; i < nwin; i++) {              // i: window index from the least significant
        const u32 bit = 4 * i, word = bit / 64;
        int d = (word < (u32)nw ? (int)((v[word] >> (bit % 64)) & 15) : 0) + carry;
        carry = d > 8;
        if (carry) d -= 16;
        job.nib[nwin - 1 - i] = d < 0 ? (uint8_t)(0x80 | -d) : (uint8_t)d;
    }
    return carry == 0;
}
template <class J, class A> static void put_point(J &job, const A &a) {
    job.inf = a.inf ? 1u : 0u;
    memcpy(job.x, &a.x, sizeof a.x);
    memcpy(job.y, &a.y, sizeof a.y);
}
// run n_jobs ladders (k_ptmul_g1 / _g2) on the thread's staging; outputs the groups' Jacobian results
static bool ptmul_run(int g, const void *jobs, size_t job_bytes, u32 n_jobs, void *out, size_t out_bytes) {
    if (!stage_ready()) return false;
    if (injected(INJ_STAGE_OP)) { set_err("injected failure (single operation)"); return false; }
    memcpy(IOH, jobs, job_bytes * n_jobs);
    const size_t out_w = 1024;                    // results at word 1024 of the 16 KB staging
    hipError_t e;
    if ((e = hipMemcpyAsync(t_stage.dev, t_stage.host, job_bytes * n_jobs, hipMemcpyHostToDevice, t_stage.s)) != hipSuccess) { set_err("H2D", e); return false; }
    if (g == 1) lcbk_ptmul_g1(t_stage.s, t_stage.dev, n_jobs, t_stage.dev + out_w);
    else lcbk_ptmul_g2(t_stage.s, t_stage.dev, n_jobs, t_stage.dev + out_w);
    if ((e = hipGetLastError()) != hipSuccess) { set_err("k_ptmul launch", e); return false; }
    if ((e = hipMemcpyAsync(t_stage.host + out_w, t_stage.dev + out_w, out_bytes * n_jobs, hipMemcpyDeviceToHost, t_stage.s)) != hipSuccess) { set_err("D2H", e); return false; }
    if ((e = hipStreamSynchronize(t_stage.s)) != hipSuccess) { set_err("k_ptmul", e); return false; }
    memcpy(out, IOH + out_w, out_bytes * n_jobs);
    return true;
}
extern "C" void mclBnG1_mul(mclBnG1 *z, const mclBnG1 *x, const mclBnFr *y) {
    uint64_t k[4];
    frh::to_raw(k, FRV(y));                       // canonical scalar < r
    fph::g1a P;
    fph::jac_to_aff(P, *G1R(x));
    if (P.inf || (k[0] | k[1] | k[2] | k[3]) == 0 || !fph::jac_on_curve(*G1R(x))) {
        if (P.inf || (k[0] | k[1] | k[2] | k[3]) == 0) { fph::jac_set_inf(*G1W(z)); return; }
        g1_op(OP_G1_MUL, z, x, nullptr, y);       // not a curve point: mcl's generic ladder semantics
        return;
    }
    // GLV (curve.hpp g1_mul_glv): k = d0 + d1 u + a1 u^2 = (a0 + a1) + a1 lambda, a0 = d0 + d1 u
    uint64_t q[4] = {k[0], k[1], k[2], k[3]};
    const uint64_t d0 = divmod_u(q), d1 = divmod_u(q);   // q = a1 < 2^128
    u128h a0 = (u128h)d1 * Z_ABS_H + d0, a1 = (u128h)q[1] << 64 | q[0];
    u128h s = a0 + a1;
    const uint64_t s_top = s < a0 ? 1 : 0;
    const uint64_t k1[3] = {(uint64_t)s, (uint64_t)(s >> 64), s_top}, k2[2] = {(uint64_t)a1, (uint64_t)(a1 >> 64)};
    const u128h zz = (u128h)Z_ABS_H * Z_ABS_H;
    fph::g1a phiP;
    fph::g1_phi(phiP, P);
    {   // membership on the host: [z^2] P == P + phi(P) = (beta^2 x, -y) (128 doublings of host field code)
        fph::g1 m, PJ;
        fph::jac_from_aff(PJ, P);
        fph::jac_set_inf(m);
        for (int b = 127; b >= 0; b--) {
            fph::jac_dbl(m, m);
            if ((zz >> b) & 1) fph::jac_add(m, m, PJ);
        }
        fph::g1a chk;
        fph::g1_phi(chk, phiP);                   // (beta^2 x, y)
        fph::neg(chk.y, chk.y);
        if (!fph::jac_eq_aff(m, chk)) {           // outside G1: the split does not apply
            g1_op(OP_G1_MUL, z, x, nullptr, y);
            return;
        }
    }
    // four ladders of <= 65 bits: k1 = k1_lo + 2^65 k1_hi over P and [2^65] P, k2 likewise over phi(P) and
    // [2^65] phi(P) = phi([2^65] P) (the doublings on the host): half the serial rounds of two 129-bit ladders
    fph::g1a P65, phiP65;
    {
        fph::g1 t;
        fph::jac_from_aff(t, P);
        for (int i = 0; i < 65; i++) fph::jac_dbl(t, t);
        fph::jac_to_aff(P65, t);
        fph::g1_phi(phiP65, P65);
    }
    if (P65.inf) { g1_op(OP_G1_MUL, z, x, nullptr, y); return; }    // unreachable in G1 (2^65 < r)
    const uint64_t k1lo[2] = {k1[0], k1[1] & 1}, k1hi[2] = {(k1[1] >> 1) | (k1[2] << 63), k1[2] >> 1};
    const uint64_t k2lo[2] = {k2[0], k2[1] & 1}, k2hi[2] = {k2[1] >> 1, 0};
    PtJobG1 jobs[4];
    memset(jobs, 0, sizeof jobs);
    put_point(jobs[0], P);
    put_point(jobs[1], P65);
    put_point(jobs[2], phiP);
    put_point(jobs[3], phiP65);
    if (!put_digits(jobs[0], k1lo, 2, 18) || !put_digits(jobs[1], k1hi, 2, 18) || !put_digits(jobs[2], k2lo, 2, 18) ||
        !put_digits(jobs[3], k2hi, 2, 18)) {
        g1_op(OP_G1_MUL, z, x, nullptr, y);       // unreachable (< 2^66 in 18 signed windows): the exact ladder
        return;
    }
    fph::g1 acc[4];
    if (!ptmul_run(1, jobs, sizeof(PtJobG1), 4, acc, sizeof(fph::g1))) { fail_out(z, 144); return; }
    fph::g1 r;
    fph::jac_add(r, acc[0], acc[1]);
    fph::jac_add(r, r, acc[2]);
    fph::jac_add(r, r, acc[3]);
    *G1W(z) = r;
}
extern "C" void lcb_g1_generator(mclBnG1 *g) { fph::g1_generator(*G1W(g)); }

extern "C" mclSize mclBnG2_serialize(void *buf, mclSize max, const mclBnG2 *x) {
    if (max < 96) return 0;
    fph::g2_compress((uint8_t *)buf, *G2R(x), g_g2_sign_b.load() != 0);
    return 96;
}
extern "C" mclSize mclBnG2_deserialize(mclBnG2 *x, const void *buf, mclSize n) {
    if (n < 96) return 0;
    fph::g2a a;
    if (!fph::g2_decompress(a, (const uint8_t *)buf, g_g2_sign_b.load() != 0)) return 0;
    fph::jac_from_aff(*G2W(x), a);
    return 96;
}
extern "C" int mclBnG2_isValid(const mclBnG2 *x) { return fph::jac_valid(*G2R(x)); }
extern "C" int mclBnG2_isEqual(const mclBnG2 *x, const mclBnG2 *y) { return fph::jac_eq(*G2R(x), *G2R(y)); }
extern "C" int mclBnG2_isZero(const mclBnG2 *x) {
    static const u32 z[24] = {0};
    return memcmp(&x->z, z, 96) == 0;
}
extern "C" void mclBnG2_clear(mclBnG2 *x) { memset(x, 0, sizeof *x); }
extern "C" int mclBnG2_hashAndMapTo(mclBnG2 *x, const void *buf, mclSize n) {
    if (n > (IO_WORDS - 256) * 4) { set_err("message too long"); return -1; }
    LOCKED_OR(-1)
    IOH[250] = (u32)n;
    memcpy(IOH + 256, buf, n);
    if (!run_hash(256 + (n + 3) / 4, 249) || !IOH[248]) return -1;
    memcpy(x, IOH, 288);
    return 0;
}
static void g2_op(int op, mclBnG2 *z, const mclBnG2 *x, const mclBnG2 *y, const mclBnFr *k) {
    if (!stage_ready()) { fail_out(z, 288); return; }
    memcpy(IOH + 72, x, 288);
    if (y) memcpy(IOH + 144, y, 288);
    if (k) memcpy(IOH + 216, k, 32);
    if (run_op(op, 224, 72)) memcpy(z, IOH, 288);
    else fail_out(z, 288);
}
extern "C" void mclBnG2_neg(mclBnG2 *y, const mclBnG2 *x) { fph::jac_neg(*G2W(y), *G2R(x)); }
extern "C" void mclBnG2_dbl(mclBnG2 *y, const mclBnG2 *x) { fph::g2 t; fph::jac_dbl(t, *G2R(x)); *G2W(y) = t; }
extern "C" void mclBnG2_normalize(mclBnG2 *y, const mclBnG2 *x) { fph::jac_normalize(*G2W(y), *G2R(x)); }
extern "C" void mclBnG2_add(mclBnG2 *z, const mclBnG2 *x, const mclBnG2 *y) {
    fph::g2 t;
    fph::jac_add(t, *G2R(x), *G2R(y));
    *G2W(z) = t;
}
extern "C" void mclBnG2_sub(mclBnG2 *z, const mclBnG2 *x, const mclBnG2 *y) {
    fph::g2 ny, t;
    fph::jac_neg(ny, *G2R(y));
    fph::jac_add(t, *G2R(x), ny);
    *G2W(z) = t;
}
extern "C" void mclBnG2_mul(mclBnG2 *z, const mclBnG2 *x, const mclBnFr *y) {
    uint64_t k[4];
    frh::to_raw(k, FRV(y));
    fph::g2a Q;
    fph::jac_to_aff(Q, *G2R(x));
    if (Q.inf || (k[0] | k[1] | k[2] | k[3]) == 0 || !fph::jac_on_curve(*G2R(x))) {
        if (Q.inf || (k[0] | k[1] | k[2] | k[3]) == 0) { fph::jac_set_inf(*G2W(z)); return; }
        g2_op(OP_G2_MUL, z, x, nullptr, y);
        return;
    }
    // GLS (curve.hpp g2_mul_gls): k = d0 + d1 u + d2 u^2 + d3 u^3 over Q, -psi Q, psi^2 Q, -psi^3 Q
    uint64_t q[4] = {k[0], k[1], k[2], k[3]}, d[4];
    d[0] = divmod_u(q);
    d[1] = divmod_u(q);
    d[2] = divmod_u(q);
    d[3] = q[0];                                  // k < r < u^4
    fph::g2a B[4];
    B[0] = Q;
    fph::g2_psi(B[1], Q);
    fph::g2_psi(B[2], B[1]);
    fph::g2_psi(B[3], B[2]);
    fph::g2a psiQ = B[1];
    {   // membership on the host: psi(Q) == -[|z|] Q (64 doublings of host field code)
        fph::g2 m, QJ;
        fph::jac_from_aff(QJ, Q);
        fph::jac_set_inf(m);
        for (int b = 63; b >= 0; b--) {
            fph::jac_dbl(m, m);
            if ((Z_ABS_H >> b) & 1) fph::jac_add(m, m, QJ);
        }
        fph::g2a chk = psiQ;
        fph::neg(chk.y, chk.y);
        if (!fph::jac_eq_aff(m, chk)) {           // outside G2: the split does not apply
            g2_op(OP_G2_MUL, z, x, nullptr, y);
            return;
        }
    }
    // eight ladders of 32 bits: each digit d_i = lo + 2^32 hi over B_i and [2^32] B_i (= +-psi^i([2^32] Q), the
    // doublings on the host): half the serial rounds of four 64-bit ladders
    fph::g2a Q32, C[4];
    {
        fph::g2 t;
        fph::jac_from_aff(t, Q);
        for (int i = 0; i < 32; i++) fph::jac_dbl(t, t);
        fph::jac_to_aff(Q32, t);
    }
    if (Q32.inf) { g2_op(OP_G2_MUL, z, x, nullptr, y); return; }    // unreachable in G2 (2^32 < r)
    C[0] = Q32;
    fph::g2_psi(C[1], Q32);
    fph::g2_psi(C[2], C[1]);
    fph::g2_psi(C[3], C[2]);
    fph::neg(C[1].y, C[1].y);
    fph::neg(C[3].y, C[3].y);
    fph::neg(B[1].y, B[1].y);
    fph::neg(B[3].y, B[3].y);
    PtJobG2 jobs[8];
    memset(jobs, 0, sizeof jobs);
    bool dig_ok = true;
    for (int i = 0; i < 4; i++) {
        const uint64_t lo = d[i] & 0xffffffffull, hi = d[i] >> 32;
        put_point(jobs[2 * i], B[i]);
        put_point(jobs[2 * i + 1], C[i]);
        dig_ok &= put_digits(jobs[2 * i], &lo, 1, 9);
        dig_ok &= put_digits(jobs[2 * i + 1], &hi, 1, 9);
    }
    if (!dig_ok) { g2_op(OP_G2_MUL, z, x, nullptr, y); return; }   // unreachable (32-bit digits): the exact ladder
    fph::g2 acc[8];
    if (!ptmul_run(2, jobs, sizeof(PtJobG2), 8, acc, sizeof(fph::g2))) { fail_out(z, 288); return; }
    fph::g2 r = acc[0];
    for (int i = 1; i < 8; i++) fph::jac_add(r, r, acc[i]);
    *G2W(z) = r;
}
extern "C" void lcb_g2_generator(mclBnG2 *g) { fph::g2_generator(*G2W(g)); }

// ================================================================== GT / pairing
static void pair_op(int op, mclBnGT *z, const mclBnG1 *x, const mclBnG2 *y) {
    if (!stage_ready()) { fail_out(z, 576); return; }
    memcpy(IOH + 144, x, 144);
    memcpy(IOH + 180, y, 288);
    if (run_op(op, 252, 144)) memcpy(z, IOH, 576);
    else fail_out(z, 576);
}
extern "C" void mclBn_millerLoop(mclBnGT *z, const mclBnG1 *x, const mclBnG2 *y) { pair_op(OP_MILLER, z, x, y); }
static void gt_op(int op, mclBnGT *z, const mclBnGT *a, const mclBnGT *b, const mclBnFr *k) {
    if (!stage_ready()) { fail_out(z, 576); return; }
    memcpy(IOH + 252, a, 576);
    if (b) memcpy(IOH + 396, b, 576);
    if (k) memcpy(IOH + 540, k, 32);
    if (run_op(op, 548, 144)) memcpy(z, IOH, 576);
    else fail_out(z, 576);
}
extern "C" void mclBn_millerLoopVec(mclBnGT *z, const mclBnG1 *x, const mclBnG2 *y, mclSize n) {
    mclBnGT acc, t;
    memset(&acc, 0, sizeof acc);
    const uint64_t errs = g_err_count;
    for (mclSize i = 0; i < n && g_err_count == errs; i++) {
        mclBn_millerLoop(&t, &x[i], &y[i]);
        if (i == 0) acc = t;
        else mclBnGT_mul(&acc, &acc, &t);
    }
    if (g_err_count != errs) fail_out(&acc, 576);
    *z = acc;
}
// debug-only (not in include/lachain_bls.h): apply tower routine `which` (k_ops.hip OP_DEBUG_FP12) to raw GT words
extern "C" int lcb_debug_fp12(int which, const uint32_t in[144], uint32_t out[144]) {
    LOCKED_OR(-1)
    memcpy(IOH + 252, in, 576);
    IOH[548] = (u32)which;
    if (!run_op(OP_DEBUG_FP12, 549, 144)) return -1;
    memcpy(out, IOH, 576);
    return 0;
}
extern "C" void mclBnGT_mul(mclBnGT *z, const mclBnGT *x, const mclBnGT *y) {
    fph::fp12 t;
    fph::mul(t, *(const fph::fp12 *)x, *(const fph::fp12 *)y);
    memcpy(z, &t, 576);
}
extern "C" void mclBnGT_pow(mclBnGT *z, const mclBnGT *x, const mclBnFr *y) { gt_op(OP_GT_POW, z, x, nullptr, y); }
extern "C" int mclBnGT_isEqual(const mclBnGT *x, const mclBnGT *y) { return memcmp(x, y, 576) == 0; }
extern "C" int mclBnGT_isOne(const mclBnGT *x) {
    // Montgomery one of Fp in the first coordinate, zero elsewhere
    const u32 *w = (const u32 *)x;
    if (memcmp(w, LCB_ONE_HOST, 48) != 0) return 0;
    for (int i = 12; i < 144; i++) if (w[i]) return 0;
    return 1;
}
extern "C" int mclBnGT_isZero(const mclBnGT *x) {
    const u32 *w = (const u32 *)x;
    for (int i = 0; i < 144; i++) if (w[i]) return 0;
    return 1;
}
extern "C" void mclBnGT_clear(mclBnGT *x) { memset(x, 0, sizeof *x); }
extern "C" mclSize mclBnGT_serialize(void *buf, mclSize max, const mclBnGT *x) {
    if (max < 576) return 0;
    const fph::fp *a = (const fph::fp *)x;
    uint8_t *b = (uint8_t *)buf;
    for (int i = 0; i < 12; i++) {
        fph::fp r;
        fph::to_raw(r, a[i]);
        memcpy(b + 48 * i, r.v, 48);
    }
    return 576;
}
extern "C" mclSize mclBnGT_deserialize(mclBnGT *x, const void *buf, mclSize n) {
    if (n < 576) return 0;
    fph::fp m[12];
    for (int i = 0; i < 12; i++) {
        fph::fp raw;
        memcpy(raw.v, (const uint8_t *)buf + 48 * i, 48);
        if (!fph::raw_lt_p(raw)) return 0;
        fph::from_raw(m[i], raw);
    }
    memcpy(x, m, 576);
    return 576;
}
extern "C" int lcb_set_g2_sign_from_b(int use_b) {
    // unpinned mcl convention: which coordinate's parity the G2 wire flag carries.  Applies to every
    // later call, host (de)serialization and every kernel that (de)compresses G2 points alike; call it before any
    // batch work, not while one is running.
    if (!ready()) return -1;
    g_g2_sign_b.store(use_b != 0);
    if (lcbk_set_g2_sign_b(use_b != 0)) { set_err("lcb_set_g2_sign_from_b: device configuration failed"); return -1; }
    return 0;
}

// ================================================================== Fr Lagrange / polynomials (host, fr_host.hpp)
extern "C" int mclBn_FrLagrangeInterpolation(mclBnFr *out, const mclBnFr *xVec, const mclBnFr *yVec, mclSize k) {
    // mcl LagrangeInterpolation: sum_i y_i prod_{j != i} x_j / (x_j - x_i); zero or repeated x is an error
    if (k == 0) return -1;
    for (mclSize i = 0; i < k; i++) {
        if (mclBnFr_isZero(&xVec[i])) return -1;
        for (mclSize j = 0; j < i; j++)
            if (mclBnFr_isEqual(&xVec[i], &xVec[j])) return -1;
    }
    if (k == 1) { *out = yVec[0]; return 0; }
    mclBnFr a, acc, t, d;
    memcpy(&a, &xVec[0], 32);
    for (mclSize i = 1; i < k; i++) mclBnFr_mul(&a, &a, &xVec[i]);
    mclBnFr_clear(&acc);
    for (mclSize i = 0; i < k; i++) {
        mclBnFr b = xVec[i];
        for (mclSize j = 0; j < k; j++) {
            if (j == i) continue;
            mclBnFr_sub(&d, &xVec[j], &xVec[i]);
            mclBnFr_mul(&b, &b, &d);
        }
        mclBnFr_div(&t, &a, &b);
        mclBnFr_mul(&t, &t, &yVec[i]);
        mclBnFr_add(&acc, &acc, &t);
    }
    *out = acc;
    return 0;
}
extern "C" int mclBn_FrEvaluatePolynomial(mclBnFr *out, const mclBnFr *c, mclSize n, const mclBnFr *x) {
    if (n == 0) return -1;
    mclBnFr acc = c[n - 1];
    for (mclSize i = n - 1; i-- > 0;) {
        mclBnFr_mul(&acc, &acc, x);
        mclBnFr_add(&acc, &acc, &c[i]);
    }
    *out = acc;
    return 0;
}

// line sets of n points a prepare kernel (or the host) stored in their sets: the five-lane kernel (k_lines.hip, ~1.5 ms
// of latency) for the small preparations the single calls and the aggregation queue make, one lane per set (~4 ms of
// latency, but about half the work per set) for large batches
#define LCB_LINES_COOP_MAX 8192
std::atomic<int> g_lines_coop_max{LCB_LINES_COOP_MAX};
void lines_fill(hipStream_t s, u32 *lines, size_t n, const u32 *sets, uint8_t *w_g2) {
    if (!n) return;
    if (n <= (size_t)g_lines_coop_max.load()) lcbk_lineset_coop(s, lines, (u32)n, sets, w_g2);
    else lcbk_lineset_fill(dim3(nblk(n)), s, lines, (u32)n, sets, w_g2);
}
// Un-normalised line sets (only an adversarial W, or the line-mode test hook, makes one): after a preparation the flag
// `which` (0 = the census's ciphertexts, 1 = all) is reduced on the device and copied to pinned memory; the host reads
// it (lines_unnormalised) before it enqueues the checks that use those sets and dispatches the one-lane Miller
// fallback only when it is set.  Any failure reads as "set" (the fallback then runs, as before round 5).
void lines_flag_enqueue(lcb_ctx *c, int which, const u32 *lines, u32 c0, u32 c1, hipStream_t s) {
    c->unn_set[which] = false;
    if (!c->unn_pin && hipHostMalloc((void **)&c->unn_pin, 16, hipHostMallocDefault) != hipSuccess) {
        c->unn_pin = nullptr;
        return;
    }
    for (auto &e : c->unn_ev)
        if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return;
    u32 *d = (u32 *)c->unn.get(16);
    if (!d) return;
    if (hipMemsetAsync(d + which, 0, 4, s) != hipSuccess) return;
    lcbk_lines_unnormalised(s, lines, c0, c1, d + which);
    if (hipMemcpyAsync(c->unn_pin + which, d + which, 4, hipMemcpyDeviceToHost, s) != hipSuccess) return;
    if (hipEventRecord(c->unn_ev[which], s) != hipSuccess) return;
    c->unn_set[which] = true;
}
bool lines_unnormalised(lcb_ctx *c, int which) {
    if (!c->unn_set[which] || hipEventSynchronize(c->unn_ev[which]) != hipSuccess) return true;
    return __atomic_load_n(c->unn_pin + which, __ATOMIC_ACQUIRE) != 0;
}

// ================================================================== execution contexts
namespace {

void ctx_free(lcb_ctx *c) {
    if (!c) return;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->order_valid) (void)hipEventSynchronize(c->order);
    for (DevBuf *b : {&c->t_lines, &c->t_ctok, &c->t_keys, &c->t_f, &c->s_lines, &c->s_mok, &c->s_keys, &c->s_f})
        b->release();
    for (auto &b : c->lag) b.release();
    c->lws.release();
    for (auto &b : c->sel) b.release();
    for (auto &b : c->msm) b.release();
    for (auto &b : c->in) b.release();
    for (auto &b : c->out) b.release();
    for (auto &b : c->dkg) b.release();
    for (auto &b : c->mcl) b.release();
    c->pc_lines.release();
    for (auto &b : c->t_coop) b.release();
    c->cc_lines.release();
    c->cc_ok.release();
    for (auto &b : c->rlc) b.release();
    c->unn.release();
    if (c->unn_pin) (void)hipHostFree(c->unn_pin);
    for (auto &e : c->unn_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->rlc_ev_ready) {
        for (auto &e : c->rlc_ev) (void)hipEventDestroy(e);
        for (auto &e : c->rlc_lev_ev) (void)hipEventDestroy(e);
    }
    if (c->fork_ready) {
        for (hipStream_t x : {c->aux, c->hi, c->hi2, c->hi3})
            if (x) {
                (void)hipStreamSynchronize(x);
                (void)hipStreamDestroy(x);
            }
        for (auto &e : c->fork_ev) (void)hipEventDestroy(e);
        for (auto &e : c->prep_ev) (void)hipEventDestroy(e);
    }
    lcb_int::ecdsa_ctx_release(c);
    if (c->ver_ev_ready) for (auto &e : c->ver_ev) (void)hipEventDestroy(e);
    if (c->msm_ev_ready) for (auto &e : c->msm_ev) (void)hipEventDestroy(e);
    if (c->order) (void)hipEventDestroy(c->order);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}
lcb_ctx *ctx_new() {
    if (!ready()) return nullptr;
    lcb_ctx *c = new lcb_ctx;
    c->device = g_device;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->order, hipEventDisableTiming);
    if (e != hipSuccess) { set_err("context creation", e); ctx_free(c); return nullptr; }
    return c;
}
// each thread owns two implicit contexts: one for the *_dev entry points without a context argument, one for the
// synchronous host-pointer entry points (so a host-pointer call never touches a workspace a *_dev caller prepared)
std::vector<lcb_ctx *> &retired_ctxs() {
    static std::vector<lcb_ctx *> *v = new std::vector<lcb_ctx *>;
    return *v;
}
struct ThreadCtx {
    lcb_ctx *c = nullptr;
    ~ThreadCtx() {                                   // retired, not freed (see OpStage)
        if (!c) return;
        std::lock_guard<std::mutex> lk(retired_mu());
        retired_ctxs().push_back(c);
    }
};
thread_local ThreadCtx t_dev_ctx, t_sync_ctx;
// an implicit context for this thread: a retired one of the current device (its prepared state dropped, its
// buffers, caches keyed by content and event chain kept), else a new one
lcb_ctx *implicit_ctx_new() {
    {
        std::lock_guard<std::mutex> lk(retired_mu());
        auto &v = retired_ctxs();
        for (size_t k = v.size(); k-- > 0;) {
            lcb_ctx *c = v[k];
            if (c->device != g_device) continue;
            v.erase(v.begin() + (long)k);
            std::lock_guard<std::recursive_mutex> cl(c->mu);
            c->t_ready = c->s_ready = false;
            c->t_gen++;
            c->s_gen++;
            return c;
        }
    }
    return ctx_new();
}
lcb_ctx *resolve(lcb_ctx *c) {
    if (!ready()) return nullptr;
    if (c) {
        if (c->device != g_device) { set_err("context belongs to another device"); return nullptr; }
        return c;
    }
    if (!t_dev_ctx.c) t_dev_ctx.c = implicit_ctx_new();
    return t_dev_ctx.c;
}
lcb_ctx *sync_ctx() {
    if (!ready()) return nullptr;
    if (!t_sync_ctx.c) t_sync_ctx.c = implicit_ctx_new();
    return t_sync_ctx.c;
}

#define CTX_OR(var, ctxarg, ret)                 \
    lcb_ctx *var = resolve(ctxarg);              \
    if (!var) return ret;
#define SYNC_CTX_OR(var, ret)                    \
    lcb_ctx *var = sync_ctx();                   \
    if (!var) return ret;

template <class T> T *up(DevBuf &b, const T *src, size_t count, hipStream_t s) {
    T *d = (T *)b.get(count * sizeof(T));
    if (d && count) hipMemcpyAsync(d, src, count * sizeof(T), hipMemcpyHostToDevice, s);
    return d;
}
bool launched(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) { set_err(what, e); return false; }
    return true;
}
bool sync_check(lcb_ctx *c, const char *what) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) { set_err(what, e); return false; }
    return true;
}

// ------------------------------------------------------------------ TPKE
// shares / checks per Miller + final-exponentiation launch pair (bounds the park buffers); lcb_set_verify_chunk (test
// hook) lowers it so small batches run several chunks.  A call reads it once, when it takes its context (lcb_ctx.hpp
// Enq), and uses that value for its buffer sizes and its chunk loops alike.
std::atomic<size_t> g_verify_chunk{(size_t)1 << 21};
#define LCB_VERIFY_CHUNK (c->chunk)
#define LCB_CT_CACHE 2048                       // prepared-ciphertext cache slots per context (52.7 KB of lines each)
#define LCB_KEY_CACHE 4096                      // decompressed verification keys per context (LCB_G1A_ST_BYTES each)

int tpke_prepare(lcb_ctx *c, const uint8_t *d_y, size_t n_keys, const uint8_t *d_u, const uint8_t *d_w,
                 const uint8_t *d_v, const uint32_t *d_voff, size_t n_cts, hipStream_t s) {
    if (n_cts > 0xffffffffu || n_keys > 0xffffffffu) { set_err("tpke prepare: batch too large"); return -1; }
    c->t_ready = false;
    c->unn_set[0] = c->unn_set[1] = false;     // the fallback flags describe the line sets prepared below
    u32 *lines = (u32 *)c->t_lines.get((size_t)n_cts * 2 * LCB_LINESET_BYTES);
    uint8_t *ctok = (uint8_t *)c->t_ctok.get(n_cts);
    void *keys = c->t_keys.get(n_keys * LCB_G1A_ST_BYTES);
    uint8_t *ctg2 = (uint8_t *)c->rlc[8].get(n_cts);     // W in G2 (the batched check's flags), from the line sets
    if (!lines || !ctok || !keys || !ctg2) { set_err("device allocation failed"); return -1; }
    if (n_keys) lcbk_g1_decompress(dim3(nblk(n_keys)), s, d_y, (u32)n_keys, keys);
    if (n_cts) {
        lcbk_tpke_ct_prepare(dim3(nblk(n_cts)), s, d_u, d_w, d_v, d_voff, (u32)n_cts, lines, ctok,
                             g_orig_cofactor | (g_line_mode << 1), nullptr);
        lines_fill(s, lines, 2 * n_cts, nullptr, ctg2);
    }
    c->unn_census = 1;
    lines_flag_enqueue(c, 1, lines, 0, (u32)n_cts, s);
    if (!launched("tpke prepare launch")) return -1;
    c->t_n_cts = n_cts;
    c->t_n_keys = n_keys;
    c->t_gen++;
    c->t_ready = true;
    return 0;
}
bool tpke_shape_ok(lcb_ctx *c, size_t n_keys, size_t n_cts, const char *what) {
    if (!c->t_ready) { set_err((std::string(what) + ": no TPKE batch prepared in this context").c_str()); return false; }
    if (c->t_n_cts != n_cts || c->t_n_keys != n_keys) {
        set_err((std::string(what) + ": batch shape differs from the one prepared in this context").c_str());
        return false;
    }
    return true;
}
// level-2 two-error search on the assembly Fp12 products (k_tpke.hip k_tpke_rlc_search2b_asm, round 6)
#ifndef LCB_SEARCH2B_ASM
#define LCB_SEARCH2B_ASM 1
#endif
std::atomic<int> g_fork_mode{4};            // lcb_set_fork_mode: stream layout of the fused batched verify (1: measured
                                            // 104.8 vs 117.8 ms per 1M-share TPKE step, profiles/r03/ab1; 3, the split
                                            // preparation: 99.6 vs 103.2 ms, profiles/r03/ab8; 4, the split preparation
                                            // in one dispatch on one high-priority stream: DESIGN.md §14.2)
std::atomic<uint32_t> g_coop_max{32768};    // lcb_set_coop_max: batches / levels of <= this many checks use the 9-lane kernels
std::atomic<uint32_t> g_coop_miller_max{65536};   // lcb_set_coop_miller_max: the same for the group Miller loops only
                                                  // (65536: level 1 too, 105.5 vs 106.1 ms, profiles/r03/ab2)
// the exact check of n shares against prepared line sets (lines, ctok: n_cts ciphertexts) and decompressed keys
int tpke_verify_core(lcb_ctx *c, const u32 *lines, const uint8_t *ctok, size_t n_cts, const void *keys, size_t n_keys,
                     uint8_t *d_accept, size_t n, const uint32_t *d_ct, const uint32_t *d_dec, const uint8_t *d_ui,
                     hipStream_t s) {
    if (n > 0xffffffffu) { set_err("tpke verify: batch too large"); return -1; }
    if (n) {
        // chunks of at most LCB_VERIFY_CHUNK shares: bounded park buffer (slots x 576 B per share) whatever n is;
        // the phase events time the first chunk
        const size_t nf = n < LCB_VERIFY_CHUNK ? n : LCB_VERIFY_CHUNK;
        u32 *f = (u32 *)c->t_f.get(nf * 576 * (size_t)lcbk_fe_slots())   /* SoA Fp12 slots: Miller output (+ final-exp parking) */;
        if (!f) { set_err("device allocation failed"); return -1; }
        if (!c->ver_ev_ready) {
            for (auto &e : c->ver_ev) hipEventCreate(&e);
            c->ver_ev_ready = true;
        }
        // small batches (the protocol's one-share-per-call shape, the queue's flushes): nine lanes per check
        // (k_coop.hip) instead of one, below the size where the one-lane kernels fill the GPU
        // (never above one chunk: the cooperative buffers below are sized for n)
        const bool coop = n <= g_coop_max.load() && n <= LCB_VERIFY_CHUNK;
        void *gpts = coop ? c->t_coop[0].get(n * 2 * LCB_G1A_ST_BYTES) : nullptr;
        void *desc = coop ? c->t_coop[1].get(n * 16) : nullptr;
        uint8_t *fl = coop ? (uint8_t *)c->t_coop[2].get(2 * n) : nullptr;
        if (coop && (!gpts || !desc || !fl)) { set_err("device allocation failed"); return -1; }
        for (size_t o = 0; o < n; o += LCB_VERIFY_CHUNK) {
            const size_t m = n - o < LCB_VERIFY_CHUNK ? n - o : LCB_VERIFY_CHUNK;
            if (o == 0) hipEventRecord(c->ver_ev[0], s);
            if (coop) {
                lcbk_tpke_exact_points(s, ctok, (u32)n_cts, keys, (u32)n_keys, d_ct + o, d_dec + o,
                                       d_ui + 48 * o, (u32)m, gpts, desc, d_accept + o);
                lcbk_coop_tpke_miller(s, lines, desc, gpts, (u32)m, f, fl, fl + m, 2, 1);
            } else {
                lcbk_tpke_miller(dim3(nblk(m)), s, lines, ctok, (u32)n_cts, keys, (u32)n_keys, d_ct + o,
                                 d_dec + o, d_ui + 48 * o, (u32)m, f, d_accept + o);
            }
            if (o == 0) hipEventRecord(c->ver_ev[1], s);
            if (coop) lcbk_coop_final_exp_check(s, f, (u32)m, d_accept + o);
            else lcbk_final_exp_check(dim3(nblk(m)), s, f, (u32)m, d_accept + o);
            if (o == 0) hipEventRecord(c->ver_ev[2], s);
        }
        c->ver_ran = true;
    }
    return launched("tpke verify launch") ? 0 : -1;
}
int tpke_verify_prepared(lcb_ctx *c, uint8_t *d_accept, size_t n, size_t n_keys, size_t n_cts, const uint32_t *d_ct,
                         const uint32_t *d_dec, const uint8_t *d_ui, hipStream_t s) {
    if (!tpke_shape_ok(c, n_keys, n_cts, "tpke verify")) return -1;
    return tpke_verify_core(c, (const u32 *)c->t_lines.p, (const uint8_t *)c->t_ctok.p, n_cts, c->t_keys.p, n_keys,
                            d_accept, n, d_ct, d_dec, d_ui, s);
}
int tpke_partial_decrypt_prepared(lcb_ctx *c, uint8_t *ui_out, uint8_t *status, const uint8_t *x_raw, size_t x_stride,
                                  const uint8_t *cts_u, size_t n_cts, hipStream_t s) {
    if (!tpke_shape_ok(c, c->t_n_keys, n_cts, "tpke partial decrypt")) return -1;
    for (size_t o = 0; o < n_cts; o += LCB_VERIFY_CHUNK) {
        const size_t m = std::min(LCB_VERIFY_CHUNK, n_cts - o);
        u32 *f = (u32 *)c->t_f.get(m * 576 * (size_t)lcbk_fe_slots());
        if (!f) { set_err("device allocation failed"); return -1; }
        lcbk_tpke_pd_miller(s, (const u32 *)c->t_lines.p, (const uint8_t *)c->t_ctok.p, cts_u, (u32)o, (u32)m, f, status);
        lcbk_final_exp_check(dim3(nblk(m)), s, f, (u32)m, status + o);
        lcbk_tpke_pd_mul(s, cts_u, x_raw, (u32)x_stride, (u32)o, (u32)m, status, ui_out);
    }
    return launched("tpke partial decrypt launch") ? 0 : -1;
}

// Randomized batch verification (k_batch.hip header): the same accept / reject decisions as the exact per-share
// checks, except with probability <= 2^-64 per group decision (the exponents are secret).  Groups are runs of shares
// of one ciphertext (TPKE) / message (threshold signatures) in the caller's order: ciphertext- / message-major batches
// give one group per ciphertext / message.  A level's group count comes back to the host (one 8-byte read per level).
std::mutex g_seed_mu;                       // lcb_set_batch_seed (test hook) vs. the callers' key fills
uint8_t g_rlc_seed[32];
bool g_rlc_seed_set = false;
std::atomic<size_t> g_census_min{16384};    // lcb_set_batch_census: batches of at least this many shares get a census
enum RlcKind { RLC_TPKE = 0, RLC_TS = 1 };
struct RlcStats {
    bool valid = false;
    int nlev = 0;
    uint32_t levels[8] = {};
    float ms[6] = {};
    uint32_t census[4] = {};
};
thread_local RlcStats t_rlc_stats;
// cnt: [0] current level's groups, [1] next level's, [2] search entries, [3] suspect keys, [4] level-1 entries after
// the suspect split; susp: the suspect-key bitmap; m: census shares [0, m)
struct RlcWs {
    u32 *rA, *rB;
    uint8_t *dA, *dB;
    u32 *cnt;
    u32 *susp;
    u32 m;
    u32 *ktab = nullptr;               // the keys' fixed-base tables when built ahead of the fork (keys_first_tables)
    uint8_t *kok = nullptr;
    bool ktab_pre = false;
};
// the fused batched calls build the keys' fixed-base tables on the caller's stream BEFORE forking the preparation: a
// key-table wave (277 registers) cannot be placed beside a preparation wave (346), so launched beside them the tables
// (and the randomisation behind them) waited up to ~20 ms for the preparation to drain (profiles/r04/ab1)
std::atomic<int> g_keys_first{1};
u32 *rlc_key_tables(lcb_ctx *c, const void *keys, size_t n_keys, hipStream_t s, uint8_t **ktab_ok);
void keys_first_tables(lcb_ctx *c, RlcWs &w, const void *keys, size_t n_keys, size_t n, hipStream_t s) {
    if (!g_keys_first.load() || w.m >= n) return;
    w.ktab = rlc_key_tables(c, keys, n_keys, s, &w.kok);
    w.ktab_pre = true;
}
bool rlc_key_fill(lcb_ctx *c, u32 key[10]) {
    bool fixed;
    {
        std::lock_guard<std::mutex> lk(g_seed_mu);
        fixed = g_rlc_seed_set;
        if (fixed) memcpy(key, g_rlc_seed, 32);
    }
    if (!fixed && getrandom(key, 32, 0) != 32) { set_err("batched verify: getrandom failed"); return false; }
    c->rlc_calls++;
    key[8] = (u32)c->rlc_calls;
    key[9] = (u32)(c->rlc_calls >> 32);
    return true;
}
// census size: a prefix of the batch large enough to sample every key a few times (>= 8 shares per key on average,
// 512 .. 2048 shares), at most a quarter of the batch; 0 = no census (small batches, or disabled)
u32 census_size(size_t n, size_t n_keys) {
    const size_t min_n = g_census_min.load();
    if (!min_n || n < min_n || n_keys < 2 || n_keys > 4096) return 0;
    size_t m = std::min<size_t>(std::max<size_t>(512, 8 * n_keys), 2048);
    m = std::min(m, n / 4);
    return m < 16 ? 0 : (u32)m;
}
bool rlc_ws(lcb_ctx *c, RlcWs &w, size_t n, size_t rec_a, size_t rec_b, size_t n_keys, u32 m, hipStream_t s) {
    w.rA = (u32 *)c->rlc[0].get(n * rec_a);
    w.rB = (u32 *)c->rlc[1].get(n * rec_b);
    w.dA = (uint8_t *)c->rlc[2].get(n * 16);
    w.dB = (uint8_t *)c->rlc[3].get(n * 16);
    w.cnt = (u32 *)c->rlc[4].get(32);
    const size_t sw = (n_keys + 31) / 32;
    w.susp = m ? (u32 *)c->rlc[13].get(4 * sw) : nullptr;
    w.m = m;
    if (!w.rA || !w.rB || !w.dA || !w.dB || !w.cnt || (m && !w.susp)) { set_err("device allocation failed"); return false; }
    if (!c->rlc_ev_ready) {
        for (auto &e : c->rlc_ev) hipEventCreate(&e);
        for (auto &e : c->rlc_lev_ev) hipEventCreate(&e);
        c->rlc_ev_ready = true;
    }
    // zeroed on the calling stream before any kernel of the call (the randomisation on the second stream reads
    // the bitmap while the census writes it)
    hipMemsetAsync(w.cnt, 0, 32, s);
    if (m) hipMemsetAsync(w.susp, 0, 4 * sw, s);
    c->rlc_census[0] = m;
    c->prep_timed = false;
    c->rlc_census[1] = c->rlc_census[2] = c->rlc_census[3] = 0;
    return true;
}
// fixed-base tables of the batch's keys (k_rlc_key_tables), when the batch is large enough to repay them
// (4 x 255 points per key, 64 lanes per key, ~24 additions of latency); nullptr: the points kernel multiplies the keys directly
u32 *rlc_key_tables(lcb_ctx *c, const void *keys, size_t n_keys, hipStream_t s, uint8_t **ktab_ok) {
    *ktab_ok = nullptr;
    if (!n_keys || n_keys > 4096) return nullptr;
    u32 *ws = (u32 *)c->rlc[12].get(lcbk_key_table_bytes((u32)n_keys));
    if (!ws) return nullptr;
    u32 *tab = nullptr;
    lcbk_rlc_key_tables(dim3(1), s, keys, (u32)n_keys, ws, &tab, ktab_ok);
    return tab;
}
// phase 1 (needs the decompressed keys only): per-share exponent multiples of shares [m, n) + level-1 groups (count
// left on device in cnt[0])
int rlc_points_enqueue(lcb_ctx *c, RlcWs &w, uint8_t *d_accept, size_t n, size_t n_keys, size_t n_cts,
                       const uint32_t *d_ct, const uint32_t *d_dec, const uint8_t *d_ui, hipStream_t s) {
    u32 key[10];
    if (!rlc_key_fill(c, key)) return -1;
    hipEventRecord(c->rlc_ev[0], s);
    if (w.m < n) {
        uint8_t *kok = w.kok;
        u32 *ktab = w.ktab_pre ? w.ktab : rlc_key_tables(c, c->t_keys.p, n_keys, s, &kok);
        lcbk_tpke_rlc_points(s, (u32)n_cts, c->t_keys.p, (u32)n_keys, d_ct, d_dec, d_ui, w.m, (u32)n, key, w.rA, w.rB,
                             d_accept, ktab, kok, w.susp);
        lcbk_rlc_groups(s, d_ct, w.m, (u32)n, (u32)n_cts, 32, w.dA, w.cnt);
    }
    hipEventRecord(c->rlc_ev[1], s);
    return launched("tpke batched verify launch") ? 0 : -1;
}
int ts_rlc_points_enqueue(lcb_ctx *c, RlcWs &w, uint8_t *d_accept, size_t n, size_t n_pks, size_t n_msgs,
                          const uint8_t *d_sigs, const uint32_t *d_midx, const uint32_t *d_pidx, hipStream_t s) {
    u32 key[10];
    if (!rlc_key_fill(c, key)) return -1;
    hipEventRecord(c->rlc_ev[0], s);
    if (w.m < n) {
        uint8_t *kok = w.kok;
        u32 *ktab = w.ktab_pre ? w.ktab : rlc_key_tables(c, c->s_keys.p, n_pks, s, &kok);
        // decoded-share records for the assembly (optional: without the buffer the assembly decodes the shares)
        const size_t rec = n * (size_t)LCB_TS_SHARE_REC_BYTES;
        const bool grow = c->s_dec.cap < rec;
        void *dec = c->s_dec.get(rec);
        if (dec && grow) hipMemsetAsync(dec, 0, c->s_dec.cap, s);   // no record is valid until written
        c->s_dec_n = dec ? c->s_dec.cap / LCB_TS_SHARE_REC_BYTES : 0;
        lcbk_ts_rlc_points(s, (u32)n_msgs, c->s_keys.p, (u32)n_pks, d_midx, d_pidx, d_sigs, w.m, (u32)n, key, w.rA,
                           w.rB, d_accept, w.dA, w.cnt, ktab, kok, w.susp, dec);
        lcbk_rlc_groups(s, d_midx, w.m, (u32)n, (u32)n_msgs, 128, w.dA, w.cnt);
    }
    hipEventRecord(c->rlc_ev[1], s);
    return launched("ts batched verify launch") ? 0 : -1;
}
bool read_counts(u32 *v, const u32 *d, int k, hipStream_t s) {
    if (hipMemcpyAsync(v, d, 4 * k, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
        set_err("batched verify: group count");
        return false;
    }
    return true;
}
struct RlcIo {                     // the per-share inputs the exact singles re-read
    const uint32_t *d_key;         // dec_idx (TPKE) / pk_idx (TS)
    const uint8_t *d_pts;          // ui (TPKE) / sigs (TS)
    const uint32_t *d_grp;         // ct_idx (TPKE) / msg_idx (TS): the census singles' groups
};
struct RlcKindInfo {
    bool ts;
    bool fb = true;                   // TPKE: some line set the checks use may be un-normalised (dispatch the fallback)
    const u32 *lines;
    const uint8_t *okv, *ctg2;
    const void *keys;
    size_t n_keys, n_grp, rec, wrec;
};
RlcKindInfo rlc_kind(lcb_ctx *c, RlcKind kind) {
    RlcKindInfo k;
    k.ts = kind == RLC_TS;
    k.lines = (const u32 *)(k.ts ? c->s_lines.p : c->t_lines.p);
    k.okv = (const uint8_t *)(k.ts ? c->s_mok.p : c->t_ctok.p);
    k.ctg2 = (const uint8_t *)c->rlc[8].p;
    k.keys = k.ts ? c->s_keys.p : c->t_keys.p;
    k.n_keys = k.ts ? c->s_n_pks : c->t_n_keys;
    k.n_grp = k.ts ? c->s_n_msgs : c->t_n_cts;
    k.rec = k.ts ? lcbk_ts_grp_bytes() : 2 * LCB_G1A_ST_BYTES;
    k.wrec = k.ts ? LCB_G1_JAC_BYTES + LCB_G2_JAC_BYTES : 2 * LCB_G1_JAC_BYTES;
    return k;
}
// the group sums / singles of a level's desc list -> gpts (k_*_rlc_sum)
// the CommonCoin level sums on two lanes per group (1) or one (0: k_batch.hip); LCB_TS_SUM2 (with LCB_ALLOW_TUNING=1)
// overrides it for A/B runs
std::atomic<int> g_ts_sum2{[] {
    const char *e = getenv("LCB_TS_SUM2");
    return (e && env_on("LCB_ALLOW_TUNING")) ? atoi(e) : 1;
}()};
// (census: the CommonCoin census's 256-register copies, k_prep.hip)
void rlc_sum_enqueue(const RlcKindInfo &K, RlcWs &w, const uint8_t *desc, u32 groups, bool first, uint8_t *d_accept,
                     size_t n, RlcIo io, void *gpts, uint8_t *gex, u32 *wsum, uint8_t *cval, hipStream_t s,
                     bool census = false) {
    const u32 *susp = w.susp;
    if (K.ts && census)
        lcbk_ts_rlc_sum_census(dim3(nblk(groups)), s, desc, groups, first, K.okv, K.keys, (u32)K.n_keys, io.d_key,
                               io.d_pts, w.rA, w.rB, (u32)n, gpts, d_accept, gex, wsum, susp, cval);
    else if (K.ts && g_ts_sum2.load())          // two lanes per group (k_prep.hip)
        lcbk_ts_rlc_sum2(s, desc, groups, first, K.okv, K.keys, (u32)K.n_keys, io.d_key, io.d_pts, w.rA, w.rB, (u32)n,
                         gpts, d_accept, gex, wsum, susp, cval);
    else if (K.ts)
        lcbk_ts_rlc_sum(dim3(nblk(groups)), s, desc, groups, first, K.okv, K.keys, (u32)K.n_keys, io.d_key, io.d_pts,
                        w.rA, w.rB, (u32)n, gpts, d_accept, gex, wsum, susp, cval);
    else
        // four lanes per group while the level is latency-bound, one when it is large (e.g. all singles)
        lcbk_tpke_rlc_sum(dim3(nblk((groups <= 262144 ? 4 : 1) * (size_t)groups)), s, desc, groups,
                          groups <= 262144 ? 4u : 1u, K.okv, K.ctg2, K.keys, (u32)K.n_keys, io.d_key,
                          io.d_pts, w.rA, w.rB, (u32)n, gpts, d_accept, gex, wsum, susp, cval);
}
// Stage dump of the TPKE two-error search (test hook, LCB_ALLOW_TEST_HOOKS=1 and LCB_DUMP_SEARCH2B=<path prefix>):
// before ("in") and after ("out") k_tpke_rlc_search2b, the open list, gamma_0 rows, gamma_c / gamma_t rows and the accept
// bytes go to <prefix>.<stage>.<call>.bin — the header {ns, n_open, n, by_position} then the four arrays
std::atomic<int> g_dump_calls{0};
// Diagnostic builds (-DLCB_SEARCH2B_DEBUG=1) also record per (open check, lane) fingerprints inside the kernel: the
// "in" stage returns the record buffer (set on the kernel), the "out" stage appends it to its file and frees it.
void *search2b_dump(hipStream_t s, const char *stage, u32 ns, u32 no, const u32 *gamma, const u32 *g12, const u32 *open,
                    const uint8_t *d_accept, size_t n, void *dbg = nullptr) {
    const char *pre = getenv("LCB_DUMP_SEARCH2B");
    if (!pre || !*pre || !env_on("LCB_ALLOW_TEST_HOOKS")) return nullptr;
    if (hipStreamSynchronize(s) != hipSuccess) return nullptr;
    std::vector<u32> rec;
    if (stage[0] == 'o' && dbg) {
        rec.resize((size_t)no * 32 * 8);
        hipMemcpy(rec.data(), dbg, 4 * rec.size(), hipMemcpyDeviceToHost);
        lcbk_search2b_debug(nullptr);
        hipFree(dbg);
    }
    std::vector<u32> op(no + 4), g0((size_t)ns * 144), gg(2 * (size_t)ns * 144);
    std::vector<uint8_t> acc(n);
    hipMemcpy(op.data(), open, 4 * (no + 4), hipMemcpyDeviceToHost);
    hipMemcpy(g0.data(), gamma, 4 * g0.size(), hipMemcpyDeviceToHost);
    hipMemcpy(gg.data(), g12, 4 * gg.size(), hipMemcpyDeviceToHost);
    hipMemcpy(acc.data(), d_accept, n, hipMemcpyDeviceToHost);
    const int call = stage[0] == 'i' ? g_dump_calls.fetch_add(1) : g_dump_calls.load() - 1;
    char path[512];
    snprintf(path, sizeof path, "%s.%s.%d.bin", pre, stage, call);
    FILE *fh = fopen(path, "wb");
    if (!fh) return nullptr;
    const u32 hdr[4] = {ns, no, (u32)n, (u32)lcbk_search2b_by_position()};
    fwrite(hdr, 4, 4, fh);
    fwrite(op.data(), 4, op.size(), fh);
    fwrite(g0.data(), 4, g0.size(), fh);
    fwrite(gg.data(), 4, gg.size(), fh);
    fwrite(acc.data(), 1, acc.size(), fh);
    if (!rec.empty()) fwrite(rec.data(), 4, rec.size(), fh);
    fclose(fh);
    void *buf = nullptr;
    if (stage[0] == 'i' && hipMalloc(&buf, (size_t)no * 32 * 8 * 4) == hipSuccess) {
        hipMemset(buf, 0xff, (size_t)no * 32 * 8 * 4);
        if (lcbk_search2b_debug(buf) != 0) { hipFree(buf); buf = nullptr; }
    }
    return buf;
}
// Miller + final exponentiation (+ resolve / search) over the groups of desc in chunks; gpts holds the points
enum RlcStage { RLC_RESOLVE = 0, RLC_SEARCH = 1, RLC_COPY = 2 };   // after a chunk's checks: resolve / search / copy out
void rlc_checks(lcb_ctx *c, const RlcKindInfo &K, RlcWs &w, const uint8_t *desc, u32 count, void *gpts, uint8_t *gacc,
                u32 *f, RlcStage stage, bool first, uint8_t *gex, uint4 *sdesc, u32 *gamma, uint8_t *d_accept,
                RlcIo io, hipStream_t s, const u32 *copy_map = nullptr, bool census = false) {
    hipEvent_t *ev = c->rlc_lev_ev;
    const bool tsc = census && K.ts;      // the CommonCoin census: the 256-register copies (k_prep.hip)
    float t;
    for (size_t o = 0; o < count; o += LCB_VERIFY_CHUNK) {
        const size_t m = count - o < LCB_VERIFY_CHUNK ? count - o : LCB_VERIFY_CHUNK;
        hipEventRecord(ev[1], s);
        // small levels (below one wave per SIMD as one check per lane): nine lanes per check (k_coop.hip)
        const bool coop = m <= g_coop_max.load(), coop_ml = m <= g_coop_miller_max.load();
        if (tsc)
            lcbk_ts_rlc_miller_census(dim3(nblk(m)), s, K.lines, desc + 16 * o, (const uint8_t *)gpts + K.rec * o,
                                      (u32)m, f, gacc + o);
        else if (K.ts)
            lcbk_ts_rlc_miller(dim3(nblk(m)), s, K.lines, desc + 16 * o, (const uint8_t *)gpts + K.rec * o, (u32)m, f,
                               gacc + o);
        else if (coop_ml)
            lcbk_coop_tpke_miller(s, K.lines, desc + 16 * o, (const uint8_t *)gpts + K.rec * o, (u32)m, f, gacc + o,
                                  (uint8_t *)c->rlc[15].get(m), 2, K.fb ? 1 : 0);
        else
            lcbk_tpke_rlc_miller(dim3(nblk(m)), s, K.lines, desc + 16 * o, (const uint8_t *)gpts + K.rec * o, (u32)m, f,
                                 gacc + o);
        hipEventRecord(ev[2], s);
        // the nine-lane final exponentiation at 248 registers (k_prep.hip): it shares a SIMD with a randomisation wave
        // of the batches in flight (three TPKE batches: 15.50-15.78 vs 15.26-15.46 M/s, profiles/r05/abfe2w)
        if (coop) lcbk_coop_final_exp_check_2w(s, f, (u32)m, gacc + o);
        else lcbk_final_exp_check(dim3(nblk(m)), s, f, (u32)m, gacc + o);
        hipEventRecord(ev[3], s);
        if (stage == RLC_COPY)
            lcbk_rlc_park_copy(s, f, (u32)o, (u32)m, gamma, copy_map);
        else if (stage == RLC_SEARCH)
            lcbk_rlc_search(dim3(nblk(m)), s, sdesc, (u32)o, (u32)m, gamma, f, d_accept, w.dB, w.cnt + 1, io.d_key,
                            (u32)K.n_keys, w.susp);
        else
            lcbk_rlc_resolve(dim3(nblk(m)), s, desc, (u32)o, (u32)m, gacc, gex, f, first ? 1u : 0u, d_accept, w.dB,
                             w.cnt + 1, sdesc, w.cnt + 2, gamma, io.d_key, (u32)K.n_keys, w.susp);
        if (hipEventSynchronize(ev[3]) == hipSuccess) {
            if (hipEventElapsedTime(&t, ev[1], ev[2]) == hipSuccess) c->rlc_ms[1] += t;
            if (hipEventElapsedTime(&t, ev[2], ev[3]) == hipSuccess) c->rlc_ms[2] += t;
        }
    }
}
// the census (SURVEY-style Byzantine validators, k_batch.hip "suspect keys"): exact single checks of shares [0, m),
// then the suspect-key bitmap and its count (cnt[3]); everything stays on the device (no host read)
int rlc_census(lcb_ctx *c, RlcKind kind, RlcWs &w, uint8_t *d_accept, RlcIo io, hipStream_t s) {
    if (!w.m) return 0;
    RlcKindInfo K = rlc_kind(c, kind);
    if (!K.ts) K.fb = lines_unnormalised(c, c->unn_census);    // waits for the census ciphertexts' line sets
    const u32 m = w.m;
    // the census uses dB as its desc list (dA is the level-1 list being built on the second stream)
    void *gpts = c->rlc[5].get((size_t)m * K.rec);
    uint8_t *gacc = (uint8_t *)c->rlc[6].get(m), *gex = (uint8_t *)c->rlc[7].get(m);
    uint8_t *cval = (uint8_t *)c->rlc[14].get(m);
    u32 *f = (u32 *)c->t_f.get((size_t)m * 576 * (size_t)lcbk_fe_slots());
    if (!gpts || !gacc || !gex || !cval || !f) { set_err("device allocation failed"); return -1; }
    lcbk_rlc_census_desc(s, io.d_grp, io.d_key, m, (u32)K.n_grp, (u32)K.n_keys, w.dB, d_accept);
    RlcWs cw = w;
    cw.susp = nullptr;                  // the census singles are exact checks whatever the bitmap says
    rlc_sum_enqueue(K, cw, w.dB, m, false, d_accept, m, io, gpts, gex, nullptr, cval, s, true);
    rlc_checks(c, K, cw, w.dB, m, gpts, gacc, f, RLC_RESOLVE, false, gex, nullptr, nullptr, d_accept, io, s, nullptr,
               true);
    lcbk_rlc_census_stats(s, io.d_key, m, (u32)K.n_keys, cval, d_accept, w.susp, w.cnt + 3);
    return launched("batched verify census launch") ? 0 : -1;
}
// phase 2 (after the preparation and the randomisation): level 1 group checks (with suspect keys: the groups summed
// over the other keys, every share of a suspect key as an exact single); level 2: weighted re-check + search of the
// failed groups; then single checks
int rlc_levels(lcb_ctx *c, RlcKind kind, RlcWs &w, uint8_t *d_accept, size_t n, RlcIo io, hipStream_t s) {
    RlcKindInfo K = rlc_kind(c, kind);
    u32 cnt[5] = {0, 0, 0, 0, 0};
    for (auto &m : c->rlc_ms) m = 0.0f;
    if (!read_counts(cnt, w.cnt, 4, s)) return -1;
    if (!K.ts) K.fb = lines_unnormalised(c, 1) || (c->unn_census == 0 && lines_unnormalised(c, 0));
    u32 groups = cnt[0];
    c->rlc_census[1] = cnt[3];
    c->rlc_census[2] = c->rlc_census[3] = groups;
    hipEvent_t *ev = c->rlc_lev_ev;
    float t;
    if (cnt[3] && groups) {             // suspect keys: split their shares out of the level-1 groups
        lcbk_rlc_suspect_split(s, w.dA, groups, io.d_key, (u32)K.n_keys, w.susp, d_accept, w.dB, w.cnt + 4);
        if (!launched("batched verify launch") || !read_counts(cnt + 4, w.cnt + 4, 1, s)) return -1;
        groups = cnt[4];
        c->rlc_census[3] = groups;
        std::swap(w.dA, w.dB);
    } else {
        w.susp = nullptr;               // no suspect key: the sums need not test the bitmap
    }
    for (int lev = 0; groups; lev++) {
        if (lev > 40) { set_err("batched verify: group splitting did not terminate"); return -1; }
        if (lev < 8) c->rlc_levels[lev] = groups;
        c->rlc_nlev = lev + 1;
        const bool first = lev == 0;
        void *gpts = c->rlc[5].get((size_t)groups * K.rec);
        uint8_t *gacc = (uint8_t *)c->rlc[6].get(groups), *gex = (uint8_t *)c->rlc[7].get(groups);
        const size_t nf = groups < LCB_VERIFY_CHUNK ? groups : LCB_VERIFY_CHUNK;
        u32 *f = (u32 *)c->t_f.get(nf * 576 * (size_t)lcbk_fe_slots());
        uint4 *sdesc = nullptr;
        u32 *gamma = nullptr, *wsum = nullptr;
        if (first) {
            sdesc = (uint4 *)c->rlc[9].get((size_t)groups * 16 * (K.ts ? 1 : 2));
            gamma = (u32 *)c->rlc[10].get((size_t)groups * 576);
            if (K.ts) wsum = (u32 *)c->rlc[11].get((size_t)groups * K.wrec);   // (TPKE: formed at level 2)
        }
        if (!gpts || !gacc || !gex || !f || (first && (!sdesc || !gamma || (K.ts && !wsum)))) {
            set_err("device allocation failed");
            return -1;
        }
        hipMemsetAsync(w.cnt + 1, 0, 8, s);
        hipEventRecord(ev[0], s);
        rlc_sum_enqueue(K, w, w.dA, groups, first, d_accept, n, io, gpts, gex, wsum, nullptr, s);
        hipEventRecord(ev[1], s);
        if (hipEventSynchronize(ev[1]) == hipSuccess && hipEventElapsedTime(&t, ev[0], ev[1]) == hipSuccess)
            c->rlc_ms[0] += t;
        rlc_checks(c, K, w, w.dA, groups, gpts, gacc, f, RLC_RESOLVE, first, gex, sdesc, gamma, d_accept, io, s);
        if (!launched("batched verify launch")) return -1;
        if (!read_counts(cnt, w.cnt, 3, s)) return -1;
        if (first && cnt[2] && !K.ts) {  // TPKE level 2: weighted re-check per failed group, one-error search, then
            // for the groups it leaves open a second weighted check and the two-error location
            const u32 ns = cnt[2];
            if (lev + 1 < 8) c->rlc_levels[lev + 1] = ns;
            c->rlc_nlev = ++lev + 1;
            const size_t nf2 = ns < LCB_VERIFY_CHUNK ? ns : LCB_VERIFY_CHUNK;
            void *gp2 = c->rlc[5].get((size_t)ns * K.rec);
            uint8_t *gacc2 = (uint8_t *)c->rlc[6].get(ns);
            u32 *g12 = (u32 *)c->rlc[16].get(2 * (size_t)ns * 576);     // gamma_c rows, then gamma_t rows
            u32 *f2 = (u32 *)c->t_f.get(nf2 * 576 * (size_t)lcbk_fe_slots());
            u32 *open = (u32 *)c->rlc[17].get((size_t)ns * 4 + 16);    // unresolved groups + their count
            if (!gp2 || !gacc2 || !g12 || !f2 || !open) { set_err("device allocation failed"); return -1; }
            hipEventRecord(ev[0], s);
            lcbk_tpke_rlc_wsum2(s, sdesc, ns, nullptr, w.rA, w.rB, (u32)n, io.d_key, (u32)K.n_keys, w.susp, gp2, nullptr);
            hipEventRecord(ev[1], s);
            if (hipEventSynchronize(ev[1]) == hipSuccess && hipEventElapsedTime(&t, ev[0], ev[1]) == hipSuccess)
                c->rlc_ms[0] += t;
            rlc_checks(c, K, w, (const uint8_t *)sdesc, ns, gp2, gacc2, f2, RLC_COPY, false, nullptr, sdesc, g12,
                       d_accept, io, s);
            lcbk_tpke_rlc_search2a(s, sdesc, ns, gamma, g12, d_accept, open + 4, open);
            u32 no = 0;
            if (!launched("batched verify launch") || !read_counts(&no, open, 1, s)) return -1;
            if (no) {
                if (lev + 1 < 8) c->rlc_levels[lev + 1] = no;
                c->rlc_nlev = ++lev + 1;
                hipEventRecord(ev[0], s);
                // sdesc[ns, 2 ns) is free (sized for two entries per level-1 group): the open groups' descriptors
                lcbk_tpke_rlc_wsum2(s, sdesc, no, open + 4, w.rA, w.rB, (u32)n, io.d_key, (u32)K.n_keys, w.susp, gp2,
                                    sdesc + ns);
                hipEventRecord(ev[1], s);
                if (hipEventSynchronize(ev[1]) == hipSuccess && hipEventElapsedTime(&t, ev[0], ev[1]) == hipSuccess)
                    c->rlc_ms[0] += t;
                // gamma_t of open group g -> row ns + g
                rlc_checks(c, K, w, (const uint8_t *)(sdesc + ns), no, gp2, gacc2, f2, RLC_COPY, false, nullptr,
                           sdesc + ns, g12 + (size_t)ns * 144, d_accept, io, s,
                           lcbk_search2b_by_position() ? nullptr : open + 4);
                void *dbg = search2b_dump(s, "in", ns, no, gamma, g12, open, d_accept, n);
#if LCB_SEARCH2B_ASM
                u32 *s2b_park = (u32 *)c->rlc[19].get(lcbk_tpke_rlc_search2b_asm_park_bytes(no));
                if (!s2b_park) { set_err("device allocation failed (level-2 search slots)"); return -1; }
                lcbk_tpke_rlc_search2b_asm(s, sdesc, ns, no, gamma, g12, open + 4, open, d_accept, w.dB, w.cnt + 1,
                                           io.d_key, (u32)K.n_keys, w.susp, s2b_park);
#else
                lcbk_tpke_rlc_search2b(s, sdesc, ns, no, gamma, g12, open + 4, open, d_accept, w.dB, w.cnt + 1,
                                       io.d_key, (u32)K.n_keys, w.susp);
#endif
                search2b_dump(s, "out", ns, no, gamma, g12, open, d_accept, n, dbg);
            }
            if (!launched("batched verify launch")) return -1;
            if (!read_counts(cnt + 1, w.cnt + 1, 1, s)) return -1;
        } else if (first && cnt[2]) {    // level 2: weighted re-check of the failed groups, then the search
            const u32 ns = cnt[2];
            if (lev + 1 < 8) c->rlc_levels[lev + 1] = ns;
            c->rlc_nlev = ++lev + 1;
            void *gp2 = c->rlc[5].get((size_t)ns * K.rec);   // (ns <= groups: the level-1 buffers are large enough)
            hipEventRecord(ev[0], s);
            if (K.ts) lcbk_ts_rlc_wsum(dim3(nblk(ns)), s, sdesc, ns, wsum, groups, gp2);
            else lcbk_tpke_rlc_wsum(dim3(nblk(ns)), s, sdesc, ns, wsum, groups, gp2);
            hipEventRecord(ev[1], s);
            if (hipEventSynchronize(ev[1]) == hipSuccess && hipEventElapsedTime(&t, ev[0], ev[1]) == hipSuccess)
                c->rlc_ms[0] += t;
            rlc_checks(c, K, w, (const uint8_t *)sdesc, ns, gp2, gacc, f, RLC_SEARCH, false, nullptr, sdesc, gamma,
                       d_accept, io, s);
            if (!launched("batched verify launch")) return -1;
            if (!read_counts(cnt + 1, w.cnt + 1, 1, s)) return -1;
        }
        groups = cnt[1];
        std::swap(w.dA, w.dB);            // the next level's groups
    }
    hipEventRecord(c->rlc_ev[2], s);
    c->rlc_ran = true;
    // the calling thread's copy of the statistics (lcb_tpke_batched_stats without a context)
    RlcStats &st = t_rlc_stats;
    st.valid = hipEventSynchronize(c->rlc_ev[2]) == hipSuccess;
    if (st.valid && c->prep_timed && hipEventElapsedTime(&c->rlc_ms[3], c->prep_ev[0], c->prep_ev[1]) != hipSuccess)
        c->rlc_ms[3] = -1.0f;
    if (st.valid && c->prep_timed && getenv("LCB_PREP_TRACE")) {       // diagnostics: hashing / line sets + census
        float a = -1.0f, b = -1.0f;
        hipEventElapsedTime(&a, c->prep_ev[0], c->prep_ev[2]);
        hipEventElapsedTime(&b, c->prep_ev[2], c->prep_ev[1]);
        fprintf(stderr, "prep_trace hash %.2f lines+census %.2f ms\n", a, b);
    }
    st.nlev = c->rlc_nlev;
    for (int i = 0; i < 8; i++) st.levels[i] = i < c->rlc_nlev ? c->rlc_levels[i] : 0;
    for (int i = 0; i < 2; i++)
        if (!st.valid || hipEventElapsedTime(&st.ms[i], c->rlc_ev[i], c->rlc_ev[i + 1]) != hipSuccess) st.ms[i] = -1.0f;
    for (int i = 0; i < 4; i++) st.ms[2 + i] = c->rlc_ms[i];
    for (int i = 0; i < 4; i++) st.census[i] = c->rlc_census[i];
    return launched("batched verify launch") ? 0 : -1;
}
int tpke_verify_prepared_rlc(lcb_ctx *c, uint8_t *d_accept, size_t n, size_t n_keys, size_t n_cts, const uint32_t *d_ct,
                             const uint32_t *d_dec, const uint8_t *d_ui, hipStream_t s) {
    if (!tpke_shape_ok(c, n_keys, n_cts, "tpke batched verify")) return -1;
    if (n > 0xffffffffu) { set_err("tpke batched verify: batch too large"); return -1; }
    c->rlc_nlev = 0;
    if (!n) return 0;
    RlcWs w;
    const RlcIo io{d_dec, d_ui, d_ct};
    if (!rlc_ws(c, w, n, LCB_G1_JAC_BYTES, LCB_G1_JAC_BYTES, n_keys, census_size(n, n_keys), s)) return -1;
    if (rlc_census(c, RLC_TPKE, w, d_accept, io, s)) return -1;   // before the randomisation: suspects skip it
    if (rlc_points_enqueue(c, w, d_accept, n, n_keys, n_cts, d_ct, d_dec, d_ui, s)) return -1;
    return rlc_levels(c, RLC_TPKE, w, d_accept, n, io, s);
}
bool fork_ready(lcb_ctx *c) {
    if (c->fork_ready) return true;
    int least = 0, greatest = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->hi, hipStreamNonBlocking, greatest);
    for (auto &ev : c->fork_ev)
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    for (auto &ev : c->prep_ev)
        if (e == hipSuccess) e = hipEventCreate(&ev);
    if (e != hipSuccess) { set_err("batched verify: stream creation", e); return false; }
    c->fork_ready = true;
    return true;
}
// fork mode 0's second normal-priority stream, created on first use
bool aux_ready(lcb_ctx *c) {
    if (c->aux) return true;
    hipError_t e = hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking);
    if (e != hipSuccess) { c->aux = nullptr; set_err("batched verify: stream creation", e); return false; }
    return true;
}
// fork mode 3's two more preparation streams, created on first use: HIP hands every stream a hardware queue when it
// is created (GPU_MAX_HW_QUEUES per priority, shared round-robin beyond that), so streams a context never uses would
// still crowd the other contexts' queues
bool split_ready(lcb_ctx *c) {
    if (c->hi2) return true;
    int least = 0, greatest = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->hi2, hipStreamNonBlocking, greatest);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->hi3, hipStreamNonBlocking, greatest);
    if (e != hipSuccess) { set_err("batched verify: stream creation", e); return false; }
    return true;
}
// prepare + batched verify in one call: the randomisation (needs only the keys) runs on the context's second
// stream beside the per-ciphertext hashing / line sets and the census (latency-bound: < 1 wave per SIMD for 50 K
// ciphertexts); a key the census marks suspect before the randomisation reaches its shares skips them
int tpke_verify_shares_rlc_fused(lcb_ctx *c, uint8_t *d_accept, size_t n, const uint8_t *d_y, size_t n_keys,
                                 const uint8_t *d_u, const uint8_t *d_w, const uint8_t *d_v, const uint32_t *d_voff,
                                 size_t n_cts, const uint32_t *d_ct, const uint32_t *d_dec, const uint8_t *d_ui,
                                 hipStream_t s) {
    if (n_cts > 0xffffffffu || n_keys > 0xffffffffu || n > 0xffffffffu) { set_err("tpke batched verify: batch too large"); return -1; }
    c->t_ready = false;
    c->unn_set[0] = c->unn_set[1] = false;     // the fallback flags describe the line sets prepared below
    c->rlc_nlev = 0;
    u32 *lines = (u32 *)c->t_lines.get((size_t)n_cts * 2 * LCB_LINESET_BYTES);
    uint8_t *ctok = (uint8_t *)c->t_ctok.get(n_cts);
    void *keys = c->t_keys.get(n_keys * LCB_G1A_ST_BYTES);
    uint8_t *ctg2 = (uint8_t *)c->rlc[8].get(n_cts);     // W in G2, from the line sets (k_lineset_fill)
    if (!lines || !ctok || !keys || !ctg2) { set_err("device allocation failed"); return -1; }
    if (!fork_ready(c)) return -1;
    const int fm = g_fork_mode.load();
    const bool hp = fm >= 1, prep_first = fm >= 2 && n_cts, split = fm >= 3, one_hi = fm == 4;
    // split mode with a census: the ciphertexts of the census shares [0, m) (indices read to the host before this call
    // launches anything; used when they all lie below a small bound c_early) are prepared first, on the preparation
    // stream, so the census runs while the bulk is prepared
    u32 c_early = 0;
    const u32 m_census = n ? census_size(n, n_keys) : 0;
    if (n_cts && split && !one_hi && m_census) {
        std::vector<uint32_t> ci(m_census);
        if (hipMemcpyAsync(ci.data(), d_ct, 4 * (size_t)m_census, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) { set_err("tpke batched verify: census index read"); return -1; }
        u32 mx = 0;
        for (uint32_t x : ci) mx = std::max(mx, x);
        if ((size_t)mx + 1 < n_cts && mx < 4096u) c_early = mx + 1;
    }
    const int fl = g_orig_cofactor | (g_line_mode << 1);
    // the census ciphertexts' decode + hash needs no key: it starts before the keys' decompression and tables (≈ 2 ms
    // on an otherwise idle device in a single batch), ordered after the context's earlier work like the caller's stream
    // (c_early is set in split mode only, whose preparation stream is c->hi)
    const bool early = c_early != 0;
    if (early) {
        hipEventRecord(c->fork_ev[4], s);
        hipStreamWaitEvent(c->hi, c->fork_ev[4], 0);
        hipEventRecord(c->prep_ev[0], c->hi);
        lcbk_tpke_ct_prepare_w64(c->hi, d_u, d_w, d_v, d_voff, c_early, lines, ctok, fl);
    }
    if (n_keys) lcbk_g1_decompress(dim3(nblk(n_keys)), s, d_y, (u32)n_keys, keys);
    RlcWs w;
    const RlcIo io{d_dec, d_ui, d_ct};
    // mode 0: randomisation on the second stream, preparation + census on the caller's; mode 1: the latency-bound
    // preparation chain (one lane per ciphertext / line set, < 1.5 waves per SIMD) on a high-priority stream, so
    // its waves are dispatched ahead of the randomisation's 16 K waves, which run on the caller's stream
    if (!hp && !aux_ready(c)) return -1;
    hipStream_t sr = hp ? s : c->aux, sp = hp ? c->hi : s;
    if (n) {
        if (!rlc_ws(c, w, n, LCB_G1_JAC_BYTES, LCB_G1_JAC_BYTES, n_keys, m_census, s)) return -1;
        keys_first_tables(c, w, keys, n_keys, n, s);
        hipEventRecord(c->fork_ev[0], s);
        hipStreamWaitEvent(hp ? sp : sr, c->fork_ev[0], 0);
        if (hp && !early) hipEventRecord(c->prep_ev[0], sp);
        if (!prep_first && rlc_points_enqueue(c, w, d_accept, n, n_keys, n_cts, d_ct, d_dec, d_ui, sr)) return -1;
        if (!hp) hipEventRecord(c->fork_ev[1], sr);
    } else if (hp) {
        hipEventRecord(c->fork_ev[0], s);
        hipStreamWaitEvent(sp, c->fork_ev[0], 0);
        hipEventRecord(c->prep_ev[0], sp);
    }
    if (n_cts && split) {
        // split preparation: hash + H's line set per lane, U / W decompression + W's line set (and its G2 flag) per
        // lane, on separate high-priority streams; each lane keeps its SIMD from the hash to the last line, so no
        // second dispatch waits behind the randomisation's waves.  With c_early: ciphertexts [0, c_early) first
        // (one decode + hash lane each, then their line sets on the five-lane kernel, then the census, all on the
        // preparation stream), the rest [c_early, n_cts) beside them on the second and third streams.
        uint8_t *hok = (uint8_t *)c->rlc[18].get(n_cts);
        if (!hok) { set_err("device allocation failed"); return -1; }
        const u32 nc = (u32)n_cts;
        if (one_hi) {
            // fork mode 4: both lane kinds in one dispatch on the context's one high-priority stream, then the census
            // behind it on the same stream; a context holds one queue per priority, so three batches in flight fit
            // the box's GPU_MAX_HW_QUEUES = 4
            lcbk_tpke_ct_prepare_hw(sp, d_u, d_w, d_v, d_voff, nc, lines, hok, ctok, ctg2, fl);
            hipEventRecord(c->prep_ev[2], sp);
            if (n && rlc_points_enqueue(c, w, d_accept, n, n_keys, n_cts, d_ct, d_dec, d_ui, sr)) return -1;
            lcbk_ct_ok_merge(sp, ctok, hok, 0, nc);
            lines_flag_enqueue(c, 1, lines, 0, nc, sp);
            c->unn_census = 1;
        } else {
        if (!split_ready(c)) return -1;
        hipStreamWaitEvent(c->hi2, c->fork_ev[0], 0);
        hipStreamWaitEvent(c->hi3, c->fork_ev[0], 0);
        const u32 ce = c_early;
        c->unn_census = ce ? 0 : 1;
        if (ce) {                    // the census's ciphertexts (decode + hash per lane launched above): their
                                     // line sets on the five-lane kernel
            lcbk_lineset_coop_2w(sp, lines, 2 * ce, nullptr, ctg2);   // (2 ce <= 8192 sets: lines_fill's coop range)
            lines_flag_enqueue(c, 0, lines, 0, ce, sp);
        }
        lcbk_tpke_ct_prepare_h(c->hi2, d_u, d_v, d_voff, ce, nc, lines, hok, fl);
        lcbk_tpke_ct_prepare_w(c->hi3, d_u, d_w, ce, nc, lines, ctok, ctg2, fl);
        hipEventRecord(c->prep_ev[2], c->hi2);
        if (n && rlc_points_enqueue(c, w, d_accept, n, n_keys, n_cts, d_ct, d_dec, d_ui, sr)) return -1;
        hipEventRecord(c->fork_ev[2], c->hi2);
        hipStreamWaitEvent(c->hi3, c->fork_ev[2], 0);
        lcbk_ct_ok_merge(c->hi3, ctok, hok, ce, nc);
        lines_flag_enqueue(c, 1, lines, ce, nc, c->hi3);
        hipEventRecord(c->fork_ev[3], c->hi3);
        if (!ce) hipStreamWaitEvent(sp, c->fork_ev[3], 0);     // the census (below) needs every ciphertext
        }
    } else if (n_cts) {
        lcbk_tpke_ct_prepare(dim3(nblk(n_cts)), sp, d_u, d_w, d_v, d_voff, (u32)n_cts, lines, ctok,
                             g_orig_cofactor | (g_line_mode << 1), nullptr);
        if (hp) hipEventRecord(c->prep_ev[2], sp);
        if (prep_first && n && rlc_points_enqueue(c, w, d_accept, n, n_keys, n_cts, d_ct, d_dec, d_ui, sr)) return -1;
        lines_fill(sp, lines, 2 * n_cts, nullptr, ctg2);
        c->unn_census = 1;
        lines_flag_enqueue(c, 1, lines, 0, (u32)n_cts, sp);
    }
    if (!launched("tpke prepare launch")) return -1;
    c->t_n_cts = n_cts;
    c->t_n_keys = n_keys;
    c->t_gen++;
    c->t_ready = true;
    if (n && rlc_census(c, RLC_TPKE, w, d_accept, io, sp)) return -1;
    if (n_cts && split && c_early) hipStreamWaitEvent(sp, c->fork_ev[3], 0);   // the bulk's preparation
    if (hp) {
        hipEventRecord(c->prep_ev[1], sp);
        c->prep_timed = true;
        hipEventRecord(c->fork_ev[1], sp);
        hipStreamWaitEvent(s, c->fork_ev[1], 0);
    } else if (n) {
        hipStreamWaitEvent(s, c->fork_ev[1], 0);
    }
    if (!n) return 0;
    return rlc_levels(c, RLC_TPKE, w, d_accept, n, io, s);
}

// ------------------------------------------------------------------ threshold signatures
int ts_prepare(lcb_ctx *c, const uint8_t *d_pks, size_t n_pks, const uint8_t *d_msg, const uint32_t *d_moff,
               size_t n_msgs, hipStream_t s) {
    if (n_msgs > 0xffffffffu || n_pks > 0xffffffffu) { set_err("ts prepare: batch too large"); return -1; }
    c->s_ready = false;
    u32 *lines = (u32 *)c->s_lines.get((size_t)n_msgs * LCB_LINESET_BYTES);
    uint8_t *mok = (uint8_t *)c->s_mok.get(n_msgs);
    void *keys = c->s_keys.get(n_pks * LCB_G1A_ST_BYTES);
    if (!lines || !mok || !keys) { set_err("device allocation failed"); return -1; }
    if (n_pks) lcbk_g1_decompress(dim3(nblk(n_pks)), s, d_pks, (u32)n_pks, keys);
    if (n_msgs) lcbk_ts_msg_prepare(dim3(nblk(n_msgs)), s, d_msg, d_moff, (u32)n_msgs, lines, mok,
                                      g_orig_cofactor | (g_line_mode << 1));
    if (!launched("ts prepare launch")) return -1;
    c->s_n_msgs = n_msgs;
    c->s_n_pks = n_pks;
    c->s_gen++;
    c->s_ready = true;
    return 0;
}
int ts_verify_prepared(lcb_ctx *c, uint8_t *d_accept, size_t n, size_t n_pks, size_t n_msgs, const uint8_t *d_sigs,
                       const uint32_t *d_midx, const uint32_t *d_pidx, hipStream_t s) {
    if (!c->s_ready) { set_err("ts verify: no threshold-signature batch prepared in this context"); return -1; }
    if (c->s_n_msgs != n_msgs || c->s_n_pks != n_pks) {
        set_err("ts verify: batch shape differs from the one prepared in this context");
        return -1;
    }
    if (n > 0xffffffffu) { set_err("ts verify: batch too large"); return -1; }
    const u32 *lines = (const u32 *)c->s_lines.p;
    const uint8_t *mok = (const uint8_t *)c->s_mok.p;
    if (n) {
        const size_t nf = n < LCB_VERIFY_CHUNK ? n : LCB_VERIFY_CHUNK;
        u32 *f = (u32 *)c->s_f.get(nf * 576 * (size_t)lcbk_fe_slots())   /* SoA Fp12 slots: Miller output (+ final-exp parking) */;
        if (!f) { set_err("device allocation failed"); return -1; }
        for (size_t o = 0; o < n; o += LCB_VERIFY_CHUNK) {
            const size_t m = n - o < LCB_VERIFY_CHUNK ? n - o : LCB_VERIFY_CHUNK;
            lcbk_ts_miller(dim3(nblk(m)), s, lines, mok, (u32)n_msgs, c->s_keys.p, (u32)n_pks, d_sigs + 96 * o,
                           d_midx + o, d_pidx + o, (u32)m, f, d_accept + o);
            lcbk_final_exp_check(dim3(nblk(m)), s, f, (u32)m, d_accept + o);
        }
    }
    return launched("ts verify launch") ? 0 : -1;
}

bool ts_shape_ok(lcb_ctx *c, size_t n_pks, size_t n_msgs, const char *what) {
    if (!c->s_ready) { set_err((std::string(what) + ": no threshold-signature batch prepared in this context").c_str()); return false; }
    if (c->s_n_msgs != n_msgs || c->s_n_pks != n_pks) {
        set_err((std::string(what) + ": batch shape differs from the one prepared in this context").c_str());
        return false;
    }
    return true;
}
// randomized batch form of ts_verify_prepared (k_batch.hip): groups = runs of one message (<= 128 shares)
int ts_verify_prepared_rlc(lcb_ctx *c, uint8_t *d_accept, size_t n, size_t n_pks, size_t n_msgs, const uint8_t *d_sigs,
                           const uint32_t *d_midx, const uint32_t *d_pidx, hipStream_t s) {
    if (!ts_shape_ok(c, n_pks, n_msgs, "ts batched verify")) return -1;
    if (n > 0xffffffffu) { set_err("ts batched verify: batch too large"); return -1; }
    c->rlc_nlev = 0;
    if (!n) return 0;
    RlcWs w;
    const RlcIo io{d_pidx, d_sigs, d_midx};
    if (!rlc_ws(c, w, n, LCB_G1_JAC_BYTES, LCB_G2_JAC_BYTES, n_pks, census_size(n, n_pks), s)) return -1;
    if (rlc_census(c, RLC_TS, w, d_accept, io, s)) return -1;
    if (ts_rlc_points_enqueue(c, w, d_accept, n, n_pks, n_msgs, d_sigs, d_midx, d_pidx, s)) return -1;
    return rlc_levels(c, RLC_TS, w, d_accept, n, io, s);
}
// prepare + batched verify: the randomisation (keys only) beside the message hashing and the census on the second
// stream
int ts_verify_shares_rlc_fused(lcb_ctx *c, uint8_t *d_accept, size_t n, const uint8_t *d_pks, size_t n_pks,
                               const uint8_t *d_sigs, const uint8_t *d_msg, const uint32_t *d_moff, size_t n_msgs,
                               const uint32_t *d_midx, const uint32_t *d_pidx, hipStream_t s) {
    if (n_msgs > 0xffffffffu || n_pks > 0xffffffffu || n > 0xffffffffu) { set_err("ts batched verify: batch too large"); return -1; }
    c->s_ready = false;
    c->rlc_nlev = 0;
    u32 *lines = (u32 *)c->s_lines.get((size_t)n_msgs * LCB_LINESET_BYTES);
    uint8_t *mok = (uint8_t *)c->s_mok.get(n_msgs);
    void *keys = c->s_keys.get(n_pks * LCB_G1A_ST_BYTES);
    if (!lines || !mok || !keys) { set_err("device allocation failed"); return -1; }
    if (!fork_ready(c)) return -1;
    if (n_pks) lcbk_g1_decompress(dim3(nblk(n_pks)), s, d_pks, (u32)n_pks, keys);
    RlcWs w;
    const RlcIo io{d_pidx, d_sigs, d_midx};
    // stream layout as in tpke_verify_shares_rlc_fused (lcb_set_fork_mode; 2 acts as 1 here)
    const bool hp = g_fork_mode.load() >= 1;
    if (!hp && !aux_ready(c)) return -1;
    hipStream_t sr = hp ? s : c->aux, sp = hp ? c->hi : s;
    if (n) {
        if (!rlc_ws(c, w, n, LCB_G1_JAC_BYTES, LCB_G2_JAC_BYTES, n_pks, census_size(n, n_pks), s)) return -1;
        keys_first_tables(c, w, keys, n_pks, n, s);
        hipEventRecord(c->fork_ev[0], s);
        hipStreamWaitEvent(hp ? sp : sr, c->fork_ev[0], 0);
        if (hp) hipEventRecord(c->prep_ev[0], sp);
    } else if (hp) {
        hipEventRecord(c->fork_ev[0], s);
        hipStreamWaitEvent(sp, c->fork_ev[0], 0);
        hipEventRecord(c->prep_ev[0], sp);
    }
    // the message preparation (latency-bound, one lane per message) is enqueued ahead of the randomisation, so its
    // waves take their SIMD slots before the randomisation's fill the device (round 5: enqueued after it, the
    // preparation ran 462 ms beside a 447 ms randomisation and the census chain waited for it)
    if (n_msgs) lcbk_ts_msg_prepare(dim3(nblk(n_msgs)), sp, d_msg, d_moff, (u32)n_msgs, lines, mok,
                                    g_orig_cofactor | (g_line_mode << 1));
    if (n) {
        if (ts_rlc_points_enqueue(c, w, d_accept, n, n_pks, n_msgs, d_sigs, d_midx, d_pidx, sr)) return -1;
        if (!hp) hipEventRecord(c->fork_ev[1], sr);
    }
    if (!launched("ts prepare launch")) return -1;
    c->s_n_msgs = n_msgs;
    c->s_n_pks = n_pks;
    c->s_gen++;
    c->s_ready = true;
    if (n && rlc_census(c, RLC_TS, w, d_accept, io, sp)) return -1;
    if (hp) {
        hipEventRecord(c->prep_ev[1], sp);
        c->prep_timed = true;
        hipEventRecord(c->fork_ev[1], sp);
        hipStreamWaitEvent(s, c->fork_ev[1], 0);
    } else if (n) {
        hipStreamWaitEvent(s, c->fork_ev[1], 0);
    }
    if (!n) return 0;
    return rlc_levels(c, RLC_TS, w, d_accept, n, io, s);
}

// ------------------------------------------------------------------ Lagrange / assembly
// device-side Lagrange at 0 for np problems (entries off[j]..off[j+1]); dout = serialized results, dst = status
int lagrange_enqueue(lcb_ctx *c, int g, uint8_t *dout, uint8_t *dst, const uint8_t *dx, const uint8_t *dy,
                     const uint32_t *doff, size_t np, size_t ne, hipStream_t s, const u32 *src = nullptr,
                     bool pairs = false) {
    if (np > 0xffffffffu || ne > 0xffffffffu) { set_err("lagrange: batch too large"); return -1; }
    void *lam = c->lag[0].get(LCB_FR_BYTES * (ne ? ne : 1));
    void *pre = c->lag[4].get(LCB_FR_BYTES * (ne ? ne : 1));      // the batch inversion's prefix products
    void *parts = c->lag[1].get((g == 1 ? LCB_G1_JAC_BYTES : LCB_G2_JAC_BYTES) * (ne ? ne : 1));
    uint8_t *pok = (uint8_t *)c->lag[2].get(ne ? ne : 1);
    if (!lam || !pre || !parts || !pok) { set_err("device allocation failed"); return -1; }
    lcbk_lagrange_coeffs(dim3(nblk(np)), s, dx, doff, (u32)np, lam, pre, dst);
    if (ne) {
        const int which = g == 1 ? 1 : pairs ? 3 : 2;   // pairs: even problem offsets (assembly with even k)
        u32 *ws = (u32 *)c->lag[3].get(lcbk_lanes_ws_bytes(which, (u32)ne));
        if (!ws) { set_err("device allocation failed (Lagrange lanes workspace)"); return -1; }
        if (g == 1) lcbk_g1_mul_lanes(s, dy, lam, (u32)ne, parts, pok, ws);
        else if (pairs)   // two entries per lane, shared doublings
            lcbk_g2_mul2_lanes(s, dy, lam, (u32)ne, parts, pok, src ? c->s_dec.p : nullptr,
                               (u32)std::min<size_t>(c->s_dec_n, 0xffffffffu), src, ws);
        else lcbk_g2_mul_lanes(s, dy, lam, (u32)ne, parts, pok, src ? c->s_dec.p : nullptr,
                               (u32)std::min<size_t>(c->s_dec_n, 0xffffffffu), src, ws);
    }
    if (g == 1) lcbk_g1_sum(dim3(nblk(np)), s, parts, pok, doff, (u32)np, dst, dout);
    else lcbk_g2_sum(dim3(nblk(np)), s, parts, pok, doff, (u32)np, dst, dout);
    return launched("lagrange launch") ? 0 : -1;
}
int assemble_enqueue(lcb_ctx *c, int g, uint8_t *out, uint8_t *status, const uint8_t *accept, const uint8_t *pts,
                     size_t per_group, size_t k, size_t n_groups, hipStream_t s, const uint32_t *order = nullptr) {
    if (!n_groups) return 0;
    if (k == 0 || k > per_group) { set_err("assemble: need 0 < k <= shares per group"); return -1; }
    size_t pb = g == 1 ? 48 : 96, ne = n_groups * k;
    if (ne > 0xffffffffu || (size_t)n_groups * per_group > 0xffffffffu) { set_err("assemble: batch too large"); return -1; }
    uint8_t *xs = (uint8_t *)c->sel[0].get(32 * ne), *ys = (uint8_t *)c->sel[1].get(pb * ne);
    u32 *off = (u32 *)c->sel[2].get(4 * (n_groups + 1));
    // G2 (signature shares): each entry's share index, so the lanes can reuse the batched check's decoded shares
    u32 *src = g == 2 && c->s_dec_n ? (u32 *)c->sel[3].get(4 * ne) : nullptr;
    if (!xs || !ys || !off) { set_err("device allocation failed"); return -1; }
    lcbk_select_first_valid(dim3(nblk(n_groups)), s, accept, pts, (u32)pb, (u32)per_group, (u32)k, (u32)n_groups, xs,
                            ys, off, order, src);
    return lagrange_enqueue(c, g, out, status, xs, ys, off, n_groups, ne, s, src, g == 2 && k % 2 == 0);
}

// ------------------------------------------------------------------ Pippenger MSM (k_msm.hip)
// window width minimising ceil-windows * (n mixed adds * 11 + 2^(c-1) buckets * 2 Jacobian adds * 16) Fp-mul
// GLV form: 2n points with 128-bit scalars, windows ceil(128 / c); only widths whose top window is nearly full
// (a short top window concentrates 2n records in few buckets, one lane each)
std::atomic<int> g_msm_segs{0};     // lcb_set_msm_segments: bucket-reduction lanes rule (0: by form, see msm_enqueue)
std::atomic<int> g_msm_chunk{64};   // records per lane of k_msm_chunk_acc (0: one lane per bucket, k_msm_bucket_acc)
u32 msm_window(size_t n, bool glv = false) {
    u32 best = 4;
    double best_cost = 1e300;
    if (glv) {
        for (u32 c : {8u, 10u, 13u, 16u}) {
            double w = (128 + c - 1) / c;
            double cost = w * (2.0 * (double)n * 11.0) + (w + 1) * (double)(1u << (c - 1)) * 32.0;
            if (cost < best_cost) { best_cost = cost; best = c; }
        }
        return best;
    }
    for (u32 c = 4; c <= 20; c++) {
        double w = 255 / c + 1;
        double cost = w * ((double)n * 11.0 + (double)(1u << (c - 1)) * 32.0);
        if (cost < best_cost) { best_cost = cost; best = c; }
    }
    return best;
}
// the GLV form halves the serial window combination and the bucket reduction, but at the window widths it can use
// (<= 16) it needs more additions than the plain form's wider windows once n is large
bool msm_use_glv(size_t n) { return n <= ((size_t)1 << 22); }
int msm_enqueue(lcb_ctx *cx, void *out_jac, const void *pts, const uint8_t *scalars, size_t n, int window_bits,
                hipStream_t s, bool glv = false) {
    if (n > (glv ? 0x3fffffffu : 0x7fffffffu)) { set_err("msm: too many points"); return -1; }
    u32 c = window_bits > 0 ? (u32)window_bits : msm_window(n, glv);
    if (c < 2 || c > 24) { set_err("msm: window bits out of range"); return -1; }
    // GLV: nwin windows of the 128-bit halves, plus one key window for the top window's upper digit half
    u32 nwin = glv ? (128 + c - 1) / c : 255 / c + 1, half = 1u << (c - 1);
    u32 nb = (glv ? nwin + 1 : nwin) * half, sentinel = nb;
    size_t np = glv ? 2 * n : n;                 // points the digit records refer to
    size_t m = np * nwin;
    if (m > 0xffffffffu) { set_err("msm: n * windows exceeds 2^32"); return -1; }
    int end_bit = 1;
    while ((1ull << end_bit) <= sentinel) end_bit++;
    u32 L = 1;
    // GLV form (n <= 2^22): the fewest segments up to 65,536 (2^20: 0.87 vs 1.05 ms of reduction); the plain form at
    // 2^24 keeps the most segments of at least 65,536 (6.3 vs 7.7 ms) — profiles/r04/q2
    const int seg_rule = g_msm_segs.load() ? g_msm_segs.load() : (glv ? 65536 : 0);
    if (seg_rule > 0) {                          // the fewest segments (serial lanes) up to seg_rule of them
        while ((size_t)nb / L > (size_t)seg_rule && L * 2 <= half) L *= 2;
    } else {                                     // the most segments of at least 65,536
        while ((size_t)nb / (L * 2) >= 65536 && L * 2 <= half) L *= 2;
    }
    u32 n_seg = nb / L, per_win = half / L, n_l1 = n_seg / (per_win < 256 ? per_win : 256);
    u32 kwin = nb / half;                        // key windows (nwin, or nwin + 1 in the GLV form)
    if (!cx->msm_ev_ready) {
        for (auto &e : cx->msm_ev) hipEventCreate(&e);
        cx->msm_ev_ready = true;
    }
    DevBuf *b = cx->msm;
    u32 *keys = (u32 *)b[0].get(m * 4), *keys2 = (u32 *)b[1].get(m * 4);
    u32 *vals = (u32 *)b[2].get(m * 4), *vals2 = (u32 *)b[3].get(m * 4);
    u32 *st = (u32 *)b[4].get((size_t)nb * 4), *en = (u32 *)b[5].get((size_t)nb * 4);
    void *buckets = b[6].get((size_t)nb * LCB_G1_JAC_BYTES);
    void *segs = b[7].get((size_t)n_seg * LCB_G1_JAC_BYTES);
    void *l1 = b[8].get((size_t)n_l1 * LCB_G1_JAC_BYTES);
    void *wins = b[9].get((size_t)kwin * LCB_G1_JAC_BYTES);
    size_t tb = 0;
    if (n && lcbk_sort_pairs(nullptr, &tb, keys, keys2, vals, vals2, (u32)m, end_bit, s) < 0) { set_err("msm: sort query"); return -1; }
    void *temp = b[10].get(tb);
    if (!keys || !keys2 || !vals || !vals2 || !st || !en || !buckets || !segs || !l1 || !wins || !temp) {
        set_err("msm: device allocation failed");
        return -1;
    }
    void *phi = glv ? b[11].get(n * 96) : nullptr;
    if (glv && !phi) { set_err("msm: device allocation failed"); return -1; }
    hipEventRecord(cx->msm_ev[0], s);
    if (n && glv) {
        lcbk_msm_phi(dim3(nblk(n)), s, pts, (u32)n, phi);
        lcbk_msm_digits_glv(dim3(nblk(n)), s, scalars, (u32)n, c, nwin, keys, vals);
    } else if (n) {
        lcbk_msm_digits(dim3(nblk(n)), s, scalars, (u32)n, c, nwin, keys, vals);
    }
    hipEventRecord(cx->msm_ev[1], s);
    int alt = n ? lcbk_sort_pairs(temp, &tb, keys, keys2, vals, vals2, (u32)m, end_bit, s) : 0;
    if (alt < 0) { set_err("msm: radix sort"); return -1; }
    if (alt) { keys = keys2; vals = vals2; }
    hipEventRecord(cx->msm_ev[2], s);
    hipMemsetAsync(st, 0, (size_t)nb * 4, s);
    hipMemsetAsync(en, 0, (size_t)nb * 4, s);
    if (m) lcbk_msm_bounds(dim3(nblk(m)), s, keys, (u32)m, sentinel, st, en);
    hipEventRecord(cx->msm_ev[3], s);
    if (g_msm_chunk > 0) {                       // record-balanced accumulation (k_msm_chunk_acc)
        const u32 K = (u32)g_msm_chunk.load();
        const size_t nch = (m + K - 1) / K;
        void *hp = b[12].get((nch ? nch : 1) * LCB_G1_JAC_BYTES), *tp = b[13].get((nch ? nch : 1) * LCB_G1_JAC_BYTES);
        if (!hp || !tp) { set_err("msm: device allocation failed"); return -1; }
        if (m) lcbk_msm_chunk_acc(s, pts, phi, (u32)n, keys, vals, (u32)m, K, sentinel, st, en, buckets, hp, tp, L, n_seg);
        lcbk_msm_bucket_fix(s, st, en, K, hp, tp, nb, buckets, L, n_seg);
    } else {
        lcbk_msm_bucket_acc(dim3(nblk(nb)), s, pts, phi, (u32)n, vals, st, en, nb, buckets, L, n_seg);
    }
    hipEventRecord(cx->msm_ev[4], s);
    lcbk_msm_bucket_reduce(dim3(nblk(n_seg)), s, buckets, half, L, n_seg, glv ? nwin : 0xffffffffu, segs);
    hipEventRecord(cx->msm_ev[5], s);
    // per-window sums: LDS tree reductions of up to 256 segment sums per block, ping-ponging segs <-> l1
    void *cur = segs, *nxt = l1;
    for (u32 cnt = per_win, total = n_seg; cnt > 1;) {
        u32 g = cnt < 256 ? cnt : 256;
        void *dst = (cnt == g) ? wins : nxt;
        lcbk_g1_jac_reduce_block(s, cur, total, g, dst);
        cnt /= g;
        total /= g;
        cur = dst;
        nxt = (dst == l1) ? segs : l1;
    }
    if (per_win == 1) hipMemcpyAsync(wins, segs, (size_t)kwin * LCB_G1_JAC_BYTES, hipMemcpyDeviceToDevice, s);
    lcbk_msm_horner(s, wins, nwin, c, glv ? 1u : 0u, out_jac);
    hipEventRecord(cx->msm_ev[6], s);
    cx->msm_ran = true;
    return launched("msm launch") ? 0 : -1;
}

} // namespace
size_t lcb_verify_chunk_now() { return g_verify_chunk.load(std::memory_order_relaxed); }

extern "C" lcb_ctx *lcb_ctx_create(void) { return ctx_new(); }
extern "C" void lcb_ctx_destroy(lcb_ctx *ctx) {
    if (!ctx) return;
    { std::lock_guard<std::recursive_mutex> lk(ctx->mu); }
    ctx_free(ctx);
}
extern "C" int lcb_ctx_synchronize(lcb_ctx *ctx) {
    CTX_OR(c, ctx, -1)
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    if (!c->order_valid) return 0;
    hipError_t e = hipEventSynchronize(c->order);
    if (e != hipSuccess) { set_err("context synchronize", e); return -1; }
    return 0;
}

// ================================================================== batch: TPKE
extern "C" int lcb_ctx_tpke_prepare_dev(lcb_ctx *ctx, const uint8_t *y_keys, size_t n_keys, const uint8_t *cts_u,
                                        const uint8_t *cts_w, const uint8_t *v_data, const uint32_t *v_off,
                                        size_t n_cts, void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    return tpke_prepare(c, y_keys, n_keys, cts_u, cts_w, v_data, v_off, n_cts, q.s);
}
extern "C" int lcb_ctx_tpke_verify_prepared_dev(lcb_ctx *ctx, uint8_t *accept, size_t n, size_t n_keys, size_t n_cts,
                                                const uint32_t *ct_idx, const uint32_t *dec_idx, const uint8_t *ui,
                                                void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    return tpke_verify_prepared(c, accept, n, n_keys, n_cts, ct_idx, dec_idx, ui, q.s);
}
extern "C" int lcb_ctx_tpke_partial_decrypt_prepared_dev(lcb_ctx *ctx, uint8_t *ui_out, uint8_t *status,
                                                         const uint8_t *x_raw, size_t x_stride, const uint8_t *cts_u,
                                                         size_t n_cts, void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    return tpke_partial_decrypt_prepared(c, ui_out, status, x_raw, x_stride, cts_u, n_cts, q.s);
}
extern "C" int lcb_ctx_tpke_combine_dev(lcb_ctx *ctx, uint8_t *u_out, uint8_t *status, const uint8_t *accept,
                                        const uint8_t *shares, size_t per_ct, size_t k, size_t n_cts, void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    return assemble_enqueue(c, 1, u_out, status, accept, shares, per_ct, k, n_cts, q.s);
}
extern "C" int lcb_ctx_tpke_combine_ordered_dev(lcb_ctx *ctx, uint8_t *u_out, uint8_t *status, const uint8_t *accept,
                                                const uint8_t *shares, const uint32_t *order, size_t per_ct, size_t k,
                                                size_t n_cts, void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    return assemble_enqueue(c, 1, u_out, status, accept, shares, per_ct, k, n_cts, q.s, order);
}
extern "C" int lcb_tpke_combine_ordered_dev(uint8_t *u_out, uint8_t *status, const uint8_t *accept,
                                           const uint8_t *shares, const uint32_t *order, size_t per_ct, size_t k,
                                           size_t n_cts, void *stream) {
    return lcb_ctx_tpke_combine_ordered_dev(nullptr, u_out, status, accept, shares, order, per_ct, k, n_cts, stream);
}
extern "C" int lcb_ctx_tpke_verify_phase_ms(lcb_ctx *ctx, float ms[2]) {
    CTX_OR(c, ctx, -1)
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    if (!c->ver_ran) { set_err("tpke verify: no split verify has run in this context"); return -1; }
    if (hipEventSynchronize(c->ver_ev[2]) != hipSuccess) { set_err("tpke verify: event sync"); return -1; }
    for (int i = 0; i < 2; i++)
        if (hipEventElapsedTime(&ms[i], c->ver_ev[i], c->ver_ev[i + 1]) != hipSuccess) ms[i] = -1.0f;
    return 0;
}

extern "C" int lcb_ctx_tpke_verify_prepared_batched_dev(lcb_ctx *ctx, uint8_t *accept, size_t n, size_t n_keys,
                                                        size_t n_cts, const uint32_t *ct_idx, const uint32_t *dec_idx,
                                                        const uint8_t *ui, void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    return tpke_verify_prepared_rlc(c, accept, n, n_keys, n_cts, ct_idx, dec_idx, ui, q.s);
}
extern "C" int lcb_ctx_tpke_verify_shares_batched_dev(lcb_ctx *ctx, uint8_t *accept, size_t n, const uint8_t *y_keys,
                                                      size_t n_keys, const uint8_t *cts_u, const uint8_t *cts_w,
                                                      const uint8_t *v_data, const uint32_t *v_off, size_t n_cts,
                                                      const uint32_t *ct_idx, const uint32_t *dec_idx,
                                                      const uint8_t *ui, void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    return tpke_verify_shares_rlc_fused(c, accept, n, y_keys, n_keys, cts_u, cts_w, v_data, v_off, n_cts, ct_idx,
                                        dec_idx, ui, q.s);
}
extern "C" int lcb_tpke_verify_shares_batched_dev(uint8_t *accept, size_t n, const uint8_t *y_keys, size_t n_keys,
                                                  const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data,
                                                  const uint32_t *v_off, size_t n_cts, const uint32_t *ct_idx,
                                                  const uint32_t *dec_idx, const uint8_t *ui, void *stream) {
    return lcb_ctx_tpke_verify_shares_batched_dev(nullptr, accept, n, y_keys, n_keys, cts_u, cts_w, v_data, v_off,
                                                  n_cts, ct_idx, dec_idx, ui, stream);
}
extern "C" int lcb_tpke_verify_prepared_batched_dev(uint8_t *accept, size_t n, size_t n_keys, size_t n_cts,
                                                    const uint32_t *ct_idx, const uint32_t *dec_idx, const uint8_t *ui,
                                                    void *stream) {
    return lcb_ctx_tpke_verify_prepared_batched_dev(nullptr, accept, n, n_keys, n_cts, ct_idx, dec_idx, ui, stream);
}
extern "C" int lcb_ctx_tpke_batched_stats(lcb_ctx *ctx, uint32_t levels[8], float ms[6]) {
    CTX_OR(c, ctx, -1)
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    if (!c->rlc_ran) { set_err("tpke batched verify: none has run in this context"); return -1; }
    if (hipEventSynchronize(c->rlc_ev[2]) != hipSuccess) { set_err("tpke batched verify: event sync"); return -1; }
    for (int i = 0; i < 8; i++) levels[i] = i < c->rlc_nlev ? c->rlc_levels[i] : 0;
    for (int i = 0; i < 2; i++)
        if (hipEventElapsedTime(&ms[i], c->rlc_ev[i], c->rlc_ev[i + 1]) != hipSuccess) ms[i] = -1.0f;
    for (int i = 0; i < 4; i++) ms[2 + i] = c->rlc_ms[i];
    return c->rlc_nlev;
}
extern "C" int lcb_tpke_batched_stats(uint32_t levels[8], float ms[6]) {
    const RlcStats &st = t_rlc_stats;
    if (!st.valid) { set_err("batched verify: none has completed on this thread"); return -1; }
    for (int i = 0; i < 8; i++) levels[i] = st.levels[i];
    for (int i = 0; i < 6; i++) ms[i] = st.ms[i];
    return st.nlev;
}
extern "C" void lcb_set_batch_seed(const uint8_t *seed32) {
    // test hook: a fixed ChaCha key makes the batch exponents predictable, so it is honoured only when the process
    // opted in (LCB_ALLOW_FIXED_BATCH_SEED=1); otherwise the call is ignored and the exponents stay secret
    const char *e = getenv("LCB_ALLOW_FIXED_BATCH_SEED");
    std::lock_guard<std::mutex> lk(g_seed_mu);
    if (seed32 && e && e[0] == '1') { memcpy(g_rlc_seed, seed32, 32); g_rlc_seed_set = true; }
    else g_rlc_seed_set = false;
}
extern "C" void lcb_set_batch_census(size_t min_shares) { g_census_min.store(min_shares); }
extern "C" int lcb_set_coop_max(uint32_t max_checks) {
    if (!tuning_allowed("lcb_set_coop_max")) return -1;
    g_coop_max.store(max_checks);
    g_coop_miller_max.store(max_checks);
    return 0;
}
extern "C" int lcb_set_verify_chunk(size_t checks) {
    if (!tuning_allowed("lcb_set_verify_chunk")) return -1;
    if (checks == 0 || checks > ((size_t)1 << 21)) { set_err("lcb_set_verify_chunk: 1 .. 2^21"); return -1; }
    g_verify_chunk.store(checks);
    return 0;
}
extern "C" int lcb_set_coop_miller_max(uint32_t max_checks) {
    if (!tuning_allowed("lcb_set_coop_miller_max")) return -1;
    g_coop_miller_max.store(max_checks);
    return 0;
}
extern "C" int lcb_set_fork_mode(int mode) {
    if (!tuning_allowed("lcb_set_fork_mode")) return -1;
    g_fork_mode.store(mode >= 1 && mode <= 4 ? mode : 0);
    return 0;
}
extern "C" int lcb_set_wave_priority(int on) {
    if (!tuning_allowed("lcb_set_wave_priority")) return -1;
    if (!ready()) return -1;
    if (lcbk_set_wave_prio(on != 0)) { set_err("lcb_set_wave_priority: device configuration failed"); return -1; }
    return 0;
}
extern "C" int lcb_set_msm_segments(int max_segments) {
    if (!tuning_allowed("lcb_set_msm_segments")) return -1;
    g_msm_segs.store(max_segments > 0 ? max_segments : 0);
    return 0;
}
extern "C" int lcb_set_keys_first(int on) {
    if (!tuning_allowed("lcb_set_keys_first")) return -1;
    g_keys_first.store(on ? 1 : 0);
    return 0;
}
extern "C" int lcb_set_lines_coop_max(int max_sets) {
    if (!tuning_allowed("lcb_set_lines_coop_max")) return -1;
    g_lines_coop_max.store(max_sets < 0 ? LCB_LINES_COOP_MAX : max_sets);
    return 0;
}
extern "C" int lcb_set_msm_chunk(int records_per_lane) {
    if (!tuning_allowed("lcb_set_msm_chunk")) return -1;
    if (records_per_lane < 0 || records_per_lane > 65536) { set_err("lcb_set_msm_chunk: 0..65536"); return -1; }
    g_msm_chunk.store(records_per_lane);
    return 0;
}
extern "C" int lcb_test_inject_failure(int site, int count) {
    if (!env_on("LCB_ALLOW_TEST_HOOKS")) { set_err("lcb_test_inject_failure: needs LCB_ALLOW_TEST_HOOKS=1"); return -1; }
    g_inject_count.store(0);
    g_inject_site.store(site);
    g_inject_count.store(count);
    return 0;
}
extern "C" uint64_t lcb_error_count(void) { return g_err_count; }
// test hook: the line sets of n G2 wire points (an undecodable encoding -> the point at infinity) on the five-lane
// (coop = 1) or the one-lane kernel, force[k] = the set's force-general flag; out: n sets of LCB_LINESET_BYTES,
// w_g2[k] = the G2 flag of set 2k + 1 (k_lineset_fill's contract)
extern "C" int lcb_test_linesets(int coop, const uint8_t *g2_wire, const uint8_t *force, size_t n, uint32_t *out,
                                 uint8_t *w_g2) {
    if (!env_on("LCB_ALLOW_TEST_HOOKS")) { set_err("lcb_test_linesets: needs LCB_ALLOW_TEST_HOOKS=1"); return -1; }
    if (!n || n > 4096) { set_err("lcb_test_linesets: 1..4096 points"); return -1; }
    SYNC_CTX_OR(c, -1)
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const size_t W = LCB_LINESET_BYTES / 4;
    u32 *lines = (u32 *)c->in[0].get(n * LCB_LINESET_BYTES);
    uint8_t *dg = (uint8_t *)c->in[1].get(n / 2 + 1);
    if (!lines || !dg) { set_err("device allocation failed"); return -1; }
    std::vector<u32> host(n * W, 0u);
    for (size_t k = 0; k < n; k++) {
        fph::g2a a;
        const bool ok = fph::g2_decompress(a, g2_wire + 96 * k, g_g2_sign_b.load() != 0);
        u32 *pt = &host[k * W + LCB_LS_POINT_WORD];
        if (ok && !a.inf) {
            memcpy(pt, &a.x, 96);
            memcpy(pt + 24, &a.y, 96);
        }
        pt[49] = (ok && !a.inf) ? 0u : 1u;
        pt[50] = force[k] ? 1u : 0u;
    }
    if (hipMemcpyAsync(lines, host.data(), n * LCB_LINESET_BYTES, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemsetAsync(dg, 0, n / 2 + 1, s) != hipSuccess) { set_err("lcb_test_linesets: upload"); return -1; }
    if (coop == 2) lcbk_lineset_coop_2w(s, lines, (u32)n, nullptr, dg);     // the fused census's instance (k_prep.hip)
    else if (coop) lcbk_lineset_coop(s, lines, (u32)n, nullptr, dg);
    else lcbk_lineset_fill(dim3(nblk(n)), s, lines, (u32)n, nullptr, dg);
    hipMemcpyAsync(out, lines, n * LCB_LINESET_BYTES, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(w_g2, dg, n / 2, hipMemcpyDeviceToHost, s);
    return sync_check(c, "lcb_test_linesets") ? 0 : -1;
}
// one cooperative Fp12 operation (k_coop_debug) on n values a (and b) vs the one-lane field.hpp routine: AoS in / out
extern "C" int lcb_debug_coop_op(int op, const uint32_t *a, const uint32_t *b, size_t n, uint32_t *out, uint32_t *ref) {
    SYNC_CTX_OR(c, -1)
    Enq q(c, c->stream);
    if (!n || n > 65536) { set_err("debug coop op: 1..65536 values"); return -1; }
    const size_t W = (size_t)144 * n;
    std::vector<u32> sa(W * 6, 0), sb(W), so(W), sr(W);
    for (size_t i = 0; i < n; i++)
        for (int w = 0; w < 144; w++) {
            sa[((size_t)(w >> 2) * n + i) * 4 + (w & 3)] = a[144 * i + w];
            sb[((size_t)(w >> 2) * n + i) * 4 + (w & 3)] = b[144 * i + w];
        }
    u32 *da = (u32 *)c->out[0].get(W * 24), *db = (u32 *)c->out[1].get(W * 4), *dout = (u32 *)c->out[2].get(W * 4),
        *dref = (u32 *)c->out[3].get(W * 4);
    if (!da || !db || !dout || !dref) { set_err("device allocation failed"); return -1; }
    hipMemcpyAsync(da, sa.data(), W * 24, hipMemcpyHostToDevice, q.s);
    hipMemcpyAsync(db, sb.data(), W * 4, hipMemcpyHostToDevice, q.s);
    lcbk_coop_debug(q.s, op, da, db, (u32)n, dout, dref);
    hipMemcpyAsync(so.data(), dout, W * 4, hipMemcpyDeviceToHost, q.s);
    hipMemcpyAsync(sr.data(), dref, W * 4, hipMemcpyDeviceToHost, q.s);
    if (!sync_check(c, "debug coop op")) return -1;
    for (size_t i = 0; i < n; i++)
        for (int w = 0; w < 144; w++) {
            out[144 * i + w] = so[((size_t)(w >> 2) * n + i) * 4 + (w & 3)];
            ref[144 * i + w] = sr[((size_t)(w >> 2) * n + i) * 4 + (w & 3)];
        }
    return 0;
}
// the final exponentiation of n Fp12 values (144 words each, Montgomery form, AoS) by the one-lane kernel (coop = 0) or
// the nine-lane kernel (coop = 1): tests compare the two bit for bit
extern "C" int lcb_debug_final_exp(const uint32_t *in, size_t n, uint32_t *out, int coop) {
    SYNC_CTX_OR(c, -1)
    Enq q(c, c->stream);
    if (!n || n > 65536) { set_err("debug final exp: 1..65536 values"); return -1; }
    std::vector<u32> soa((size_t)144 * n * lcbk_fe_slots(), 0);
    for (size_t i = 0; i < n; i++)
        for (int w = 0; w < 144; w++) soa[((size_t)(w >> 2) * n + i) * 4 + (w & 3)] = in[144 * i + w];
    u32 *d = (u32 *)c->out[0].get(soa.size() * 4);
    uint8_t *acc = (uint8_t *)c->out[1].get(n);
    if (!d || !acc) { set_err("device allocation failed"); return -1; }
    hipMemcpyAsync(d, soa.data(), soa.size() * 4, hipMemcpyHostToDevice, q.s);
    hipMemsetAsync(acc, 1, n, q.s);
    if (coop) lcbk_coop_final_exp_check(q.s, d, (u32)n, acc);
    else lcbk_final_exp_check(dim3(nblk(n)), q.s, d, (u32)n, acc);
    hipMemcpyAsync(soa.data(), d, (size_t)144 * n * 4, hipMemcpyDeviceToHost, q.s);
    if (!sync_check(c, "debug final exp")) return -1;
    for (size_t i = 0; i < n; i++)
        for (int w = 0; w < 144; w++) out[144 * i + w] = soa[((size_t)(w >> 2) * n + i) * 4 + (w & 3)];
    return 0;
}
extern "C" int lcb_ctx_batched_census(lcb_ctx *ctx, uint32_t out[4]) {
    CTX_OR(c, ctx, -1)
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    if (!c->rlc_ran) { set_err("batched verify: none has run in this context"); return -1; }
    for (int i = 0; i < 4; i++) out[i] = c->rlc_census[i];
    return 0;
}
extern "C" int lcb_batched_census(uint32_t out[4]) {
    const RlcStats &st = t_rlc_stats;
    if (!st.valid) { set_err("batched verify: none has completed on this thread"); return -1; }
    for (int i = 0; i < 4; i++) out[i] = st.census[i];
    return 0;
}

extern "C" int lcb_tpke_prepare_dev(const uint8_t *y_keys, size_t n_keys, const uint8_t *cts_u, const uint8_t *cts_w,
                                    const uint8_t *v_data, const uint32_t *v_off, size_t n_cts, void *stream) {
    return lcb_ctx_tpke_prepare_dev(nullptr, y_keys, n_keys, cts_u, cts_w, v_data, v_off, n_cts, stream);
}
extern "C" int lcb_tpke_verify_prepared_dev(uint8_t *accept, size_t n, size_t n_keys, size_t n_cts, const uint32_t *ct_idx,
                                            const uint32_t *dec_idx, const uint8_t *ui, void *stream) {
    return lcb_ctx_tpke_verify_prepared_dev(nullptr, accept, n, n_keys, n_cts, ct_idx, dec_idx, ui, stream);
}
extern "C" int lcb_tpke_partial_decrypt_prepared_dev(uint8_t *ui_out, uint8_t *status, const uint8_t *x_raw,
                                                     size_t x_stride, const uint8_t *cts_u, size_t n_cts, void *stream) {
    return lcb_ctx_tpke_partial_decrypt_prepared_dev(nullptr, ui_out, status, x_raw, x_stride, cts_u, n_cts, stream);
}
extern "C" int lcb_tpke_combine_dev(uint8_t *u_out, uint8_t *status, const uint8_t *accept, const uint8_t *shares,
                                    size_t per_ct, size_t k, size_t n_cts, void *stream) {
    return lcb_ctx_tpke_combine_dev(nullptr, u_out, status, accept, shares, per_ct, k, n_cts, stream);
}
extern "C" int lcb_tpke_verify_phase_ms(float ms[2]) { return lcb_ctx_tpke_verify_phase_ms(nullptr, ms); }
extern "C" int lcb_tpke_verify_shares_dev(uint8_t *accept, size_t n, const uint8_t *y_keys, size_t n_keys,
                                          const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data,
                                          const uint32_t *v_off, size_t n_cts, const uint32_t *ct_idx,
                                          const uint32_t *dec_idx, const uint8_t *ui, void *stream) {
    CTX_OR(c, nullptr, -1)
    Enq q(c, (hipStream_t)stream);
    if (tpke_prepare(c, y_keys, n_keys, cts_u, cts_w, v_data, v_off, n_cts, q.s)) return -1;
    return tpke_verify_prepared(c, accept, n, n_keys, n_cts, ct_idx, dec_idx, ui, q.s);
}
static int tpke_verify_shares_host(uint8_t *accept, size_t n, const uint8_t *y_keys, size_t n_keys,
                                   const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data,
                                   const uint32_t *v_off, size_t n_cts, const uint32_t *ct_idx,
                                   const uint32_t *dec_idx, const uint8_t *ui, bool batched) {
    SYNC_CTX_OR(c, -1)
    for (size_t i = 0; i < n; i++) {
        if (ct_idx[i] >= n_cts) { set_err("ct_idx out of range"); return -1; }
        if (dec_idx[i] >= n_keys) { set_err("dec_idx out of range"); return -1; }
    }
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    size_t vbytes = n_cts ? v_off[n_cts] : 0;
    const uint8_t *dy = up(c->in[0], y_keys, 48 * n_keys, s);
    const uint8_t *du = up(c->in[1], cts_u, 48 * n_cts, s);
    const uint8_t *dw = up(c->in[2], cts_w, 96 * n_cts, s);
    const uint8_t *dv = up(c->in[3], v_data, vbytes, s);
    const uint32_t *dvo = up(c->in[4], v_off, n_cts + 1, s);
    const uint32_t *dct = up(c->in[5], ct_idx, n, s);
    const uint32_t *ddec = up(c->in[6], dec_idx, n, s);
    const uint8_t *dui = up(c->in[7], ui, 48 * n, s);
    uint8_t *dacc = (uint8_t *)c->out[0].get(n);
    if (!dy || !du || !dw || !dv || !dvo || !dct || !ddec || !dui || !dacc) { set_err("device allocation failed"); return -1; }
    if (batched) {
        if (tpke_verify_shares_rlc_fused(c, dacc, n, dy, n_keys, du, dw, dv, dvo, n_cts, dct, ddec, dui, s)) return -1;
    } else {
        if (tpke_prepare(c, dy, n_keys, du, dw, dv, dvo, n_cts, s)) return -1;
        if (tpke_verify_prepared(c, dacc, n, n_keys, n_cts, dct, ddec, dui, s)) return -1;
    }
    if (n) hipMemcpyAsync(accept, dacc, n, hipMemcpyDeviceToHost, s);
    return sync_check(c, "tpke verify") ? 0 : -1;
}
// lcb_tpke_verify_shares with a per-context cache of prepared ciphertexts (the line sets of H and W and the
// validity, keyed by the ciphertext's bytes, least recently used slot replaced): the protocol verifies the N shares of
// a ciphertext in separate calls (HoneyBadger.cs:211-212), so each ciphertext is hashed to G2 and its lines computed
// once, not once per call.  Same decisions as lcb_tpke_verify_shares (a cache entry is the prepare output for the
// same bytes under the same prepare flags).
extern "C" int lcb_tpke_verify_shares_cached(uint8_t *accept, size_t n, const uint8_t *y_keys, size_t n_keys,
                                             const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data,
                                             const uint32_t *v_off, size_t n_cts, const uint32_t *ct_idx,
                                             const uint32_t *dec_idx, const uint8_t *ui) {
    SYNC_CTX_OR(c, -1)
    // a batch this wide gains nothing from the caches (and more keys than the key cache holds cannot use it): the
    // uncached call gives the same decisions
    if (n_cts > LCB_CT_CACHE / 2 || n_keys > LCB_KEY_CACHE)
        return tpke_verify_shares_host(accept, n, y_keys, n_keys, cts_u, cts_w, v_data, v_off, n_cts, ct_idx, dec_idx,
                                       ui, false);
    for (size_t i = 0; i < n; i++) {
        if (ct_idx[i] >= n_cts) { set_err("ct_idx out of range"); return -1; }
        if (dec_idx[i] >= n_keys) { set_err("dec_idx out of range"); return -1; }
    }
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const int flags = g_orig_cofactor | (g_line_mode << 1);
    if (c->cc_used.empty() || c->cc_flags != flags) {           // first use, or prepare flags changed: empty cache
        c->cc_map.clear();
        c->cc_keys.assign(LCB_CT_CACHE, std::string());
        c->cc_used.assign(LCB_CT_CACHE, 0);
        c->cc_flags = flags;
    }
    u32 *lines = (u32 *)c->cc_lines.get((size_t)LCB_CT_CACHE * 2 * LCB_LINESET_BYTES);
    uint8_t *ctok = (uint8_t *)c->cc_ok.get(LCB_CT_CACHE);
    void *keys = c->kc_pts.get((size_t)LCB_KEY_CACHE * LCB_G1A_ST_BYTES);
    if (!lines || !ctok || !keys) { set_err("device allocation failed"); return -1; }
    const uint64_t tick = ++c->cc_tick;
    // the maps below name slots before their line sets / points exist: any failure from here on empties both caches
    // (the next call starts from first use), so no later call can take a slot this call left unfilled
    auto cache_fail = [c]() {
        c->cc_used.clear();
        c->kc_map.clear();
        c->kc_n = 0;
        return -1;
    };
    // verification keys -> key-cache slots; the misses are decompressed into consecutive slots [kc_n, kc_n + misses)
    std::vector<u32> kslot(n_keys);
    u32 kfirst = c->kc_n;
    for (int pass = 0; pass < 2; pass++) {
        kfirst = c->kc_n;
        u32 next = kfirst;
        bool full = false;
        for (size_t k = 0; k < n_keys && !full; k++) {
            std::string key((const char *)y_keys + 48 * k, 48);
            auto it = c->kc_map.find(key);
            if (it != c->kc_map.end()) { kslot[k] = it->second; continue; }
            if (next == LCB_KEY_CACHE) { full = true; break; }
            kslot[k] = next;
            c->kc_map.emplace(std::move(key), next++);
        }
        if (!full) { c->kc_n = next; break; }
        c->kc_map.clear();                               // this call's keys do not fit beside the old ones: start afresh
        c->kc_n = 0;
    }
    std::vector<uint8_t> kmiss;
    for (size_t k = 0; k < n_keys; k++)
        if (kslot[k] >= kfirst) {                        // first sight, in slot order (a repeated key maps to one slot)
            if (kmiss.size() / 48 == kslot[k] - kfirst) kmiss.insert(kmiss.end(), y_keys + 48 * k, y_keys + 48 * k + 48);
        }
    std::vector<u32> slot_of(n_cts), miss;
    for (size_t k = 0; k < n_cts; k++) {
        const u32 v0 = v_off[k], v1 = v_off[k + 1];
        std::string key((const char *)cts_u + 48 * k, 48);
        key.append((const char *)cts_w + 96 * k, 96);
        key.append((const char *)v_data + v0, v1 - v0);
        auto it = c->cc_map.find(key);
        if (it != c->cc_map.end()) {
            slot_of[k] = it->second;
            c->cc_used[it->second] = tick;
            continue;
        }
        u32 victim = 0;                  // least recently used slot not taken by this batch
        for (u32 j = 1; j < LCB_CT_CACHE; j++)
            if (c->cc_used[j] < c->cc_used[victim]) victim = j;
        if (!c->cc_keys[victim].empty()) c->cc_map.erase(c->cc_keys[victim]);
        c->cc_keys[victim] = key;
        c->cc_map.emplace(std::move(key), victim);
        c->cc_used[victim] = tick;
        slot_of[k] = victim;
        miss.push_back((u32)k);
    }
    // prepare the misses straight into their slots
    if (!kmiss.empty()) {
        const size_t km = kmiss.size() / 48;
        const uint8_t *dy = up(c->in[0], kmiss.data(), kmiss.size(), s);
        if (!dy) { set_err("device allocation failed"); return cache_fail(); }
        lcbk_g1_decompress(dim3(nblk(km)), s, dy, (u32)km, (uint8_t *)keys + (size_t)kfirst * LCB_G1A_ST_BYTES);
    }
    if (!miss.empty()) {
        const size_t m = miss.size();
        std::vector<uint8_t> mu(48 * m), mw(96 * m), mv;
        std::vector<u32> mvo(1, 0), mslot(m), msets(2 * m);
        for (size_t j = 0; j < m; j++) {
            const u32 k = miss[j];
            memcpy(&mu[48 * j], cts_u + 48 * (size_t)k, 48);
            memcpy(&mw[96 * j], cts_w + 96 * (size_t)k, 96);
            mv.insert(mv.end(), v_data + v_off[k], v_data + v_off[k + 1]);
            mvo.push_back((u32)mv.size());
            mslot[j] = slot_of[k];
            msets[2 * j] = 2 * slot_of[k];
            msets[2 * j + 1] = 2 * slot_of[k] + 1;
        }
        if (mv.empty()) mv.push_back(0);
        const uint8_t *du = up(c->in[1], mu.data(), mu.size(), s);
        const uint8_t *dw = up(c->in[2], mw.data(), mw.size(), s);
        const uint8_t *dv = up(c->in[3], mv.data(), mv.size(), s);
        const uint32_t *dvo = up(c->in[4], mvo.data(), mvo.size(), s);
        const uint32_t *dsl = up(c->sel[0], mslot.data(), m, s);
        const uint32_t *dse = up(c->sel[1], msets.data(), 2 * m, s);
        if (!du || !dw || !dv || !dvo || !dsl || !dse || injected(INJ_CT_CACHE_ALLOC)) {
            set_err("device allocation failed");
            return cache_fail();
        }
        lcbk_tpke_ct_prepare(dim3(nblk(m)), s, du, dw, dv, dvo, (u32)m, lines, ctok, flags, dsl);
        lines_fill(s, lines, 2 * m, dse, nullptr);
    }
    std::vector<u32> cslot(n);
    for (size_t i = 0; i < n; i++) cslot[i] = slot_of[ct_idx[i]];
    const uint32_t *dct = up(c->in[5], cslot.data(), n, s);
    std::vector<u32> kdec(n);
    for (size_t i = 0; i < n; i++) kdec[i] = kslot[dec_idx[i]];
    const uint32_t *ddec = up(c->in[6], kdec.data(), n, s);
    const uint8_t *dui = up(c->in[7], ui, 48 * n, s);
    uint8_t *dacc = (uint8_t *)c->out[0].get(n);
    if (!dct || !ddec || !dui || !dacc) { set_err("device allocation failed"); return cache_fail(); }
    if (tpke_verify_core(c, lines, ctok, LCB_CT_CACHE, keys, c->kc_n, dacc, n, dct, ddec, dui, s)) return cache_fail();
    if (n) hipMemcpyAsync(accept, dacc, n, hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "tpke verify (cached)")) return cache_fail();
    return 0;
}
extern "C" int lcb_tpke_verify_shares(uint8_t *accept, size_t n, const uint8_t *y_keys, size_t n_keys,
                                      const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data,
                                      const uint32_t *v_off, size_t n_cts, const uint32_t *ct_idx,
                                      const uint32_t *dec_idx, const uint8_t *ui) {
    return tpke_verify_shares_host(accept, n, y_keys, n_keys, cts_u, cts_w, v_data, v_off, n_cts, ct_idx, dec_idx, ui,
                                   false);
}
extern "C" int lcb_tpke_verify_shares_batched(uint8_t *accept, size_t n, const uint8_t *y_keys, size_t n_keys,
                                              const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data,
                                              const uint32_t *v_off, size_t n_cts, const uint32_t *ct_idx,
                                              const uint32_t *dec_idx, const uint8_t *ui) {
    return tpke_verify_shares_host(accept, n, y_keys, n_keys, cts_u, cts_w, v_data, v_off, n_cts, ct_idx, dec_idx, ui,
                                   true);
}

extern "C" int lcb_tpke_partial_decrypt(uint8_t *ui_out, uint8_t *status, const uint8_t x[32], const uint8_t *cts_u,
                                        const uint8_t *cts_w, const uint8_t *v_data, const uint32_t *v_off,
                                        size_t n_cts) {
    SYNC_CTX_OR(c, -1)
    if (!n_cts) return 0;
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    size_t vbytes = v_off[n_cts];
    const uint8_t *du = up(c->in[1], cts_u, 48 * n_cts, s);
    const uint8_t *dw = up(c->in[2], cts_w, 96 * n_cts, s);
    const uint8_t *dv = up(c->in[3], v_data, vbytes, s);
    const uint32_t *dvo = up(c->in[4], v_off, n_cts + 1, s);
    const uint8_t *dx = up(c->in[0], x, 32, s);
    uint8_t *dui = (uint8_t *)c->out[0].get(48 * n_cts);
    uint8_t *dst = (uint8_t *)c->out[1].get(n_cts);
    if (!du || !dw || !dv || !dvo || !dx || !dui || !dst) { set_err("device allocation failed"); return -1; }
    if (tpke_prepare(c, nullptr, 0, du, dw, dv, dvo, n_cts, s)) return -1;
    if (tpke_partial_decrypt_prepared(c, dui, dst, dx, 0, du, n_cts, s)) return -1;
    hipMemcpyAsync(ui_out, dui, 48 * n_cts, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(status, dst, n_cts, hipMemcpyDeviceToHost, s);
    return sync_check(c, "tpke partial decrypt") ? 0 : -1;
}

extern "C" int lcb_tpke_encrypt_phase1(uint8_t *u_out, uint8_t *t_out, const uint8_t y[48], const uint8_t *r, size_t n) {
    SYNC_CTX_OR(c, -1)
    if (!n) return 0;
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const uint8_t *dy = up(c->in[0], y, 48, s);
    const uint8_t *dr = up(c->in[1], r, 32 * n, s);
    uint8_t *du = (uint8_t *)c->out[0].get(48 * n), *dt = (uint8_t *)c->out[1].get(48 * n), *dok = (uint8_t *)c->out[2].get(n);
    u32 *ws = (u32 *)c->lws.get(lcbk_scalar_ws_bytes(3, (u32)n));
    if (!dy || !dr || !du || !dt || !dok || !ws) { set_err("device allocation failed"); return -1; }
    lcbk_tpke_encrypt1(s, dy, dr, (u32)n, du, dt, dok, ws);
    std::vector<uint8_t> ok(n);
    hipMemcpyAsync(u_out, du, 48 * n, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(t_out, dt, 48 * n, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(ok.data(), dok, n, hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "tpke encrypt1")) return -1;
    for (size_t i = 0; i < n; i++) if (!ok[i]) { set_err("invalid public key or scalar"); return -1; }
    return 0;
}
extern "C" int lcb_tpke_encrypt_phase2(uint8_t *w_out, const uint8_t *u, const uint8_t *r, const uint8_t *v_data,
                                       const uint32_t *v_off, size_t n) {
    SYNC_CTX_OR(c, -1)
    if (!n) return 0;
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const uint8_t *du = up(c->in[0], u, 48 * n, s);
    const uint8_t *dr = up(c->in[1], r, 32 * n, s);
    const uint8_t *dv = up(c->in[2], v_data, v_off[n], s);
    const uint32_t *dvo = up(c->in[3], v_off, n + 1, s);
    uint8_t *dw = (uint8_t *)c->out[0].get(96 * n), *dok = (uint8_t *)c->out[1].get(n);
    if (!du || !dr || !dv || !dvo || !dw || !dok) { set_err("device allocation failed"); return -1; }
    lcbk_tpke_encrypt2(dim3(nblk(n)), s, du, dr, dv, dvo, (u32)n, dw, dok, g_orig_cofactor);
    std::vector<uint8_t> ok(n);
    hipMemcpyAsync(w_out, dw, 96 * n, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(ok.data(), dok, n, hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "tpke encrypt2")) return -1;
    for (size_t i = 0; i < n; i++) if (!ok[i]) { set_err("hash-to-G2 failed"); return -1; }
    return 0;
}

// ================================================================== batch: threshold signatures
extern "C" int lcb_ctx_ts_prepare_dev(lcb_ctx *ctx, const uint8_t *pks, size_t n_pks, const uint8_t *msg_data,
                                      const uint32_t *msg_off, size_t n_msgs, void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    return ts_prepare(c, pks, n_pks, msg_data, msg_off, n_msgs, q.s);
}
extern "C" int lcb_ctx_ts_verify_prepared_dev(lcb_ctx *ctx, uint8_t *accept, size_t n, size_t n_pks, size_t n_msgs,
                                              const uint8_t *sigs, const uint32_t *msg_idx, const uint32_t *pk_idx,
                                              void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    return ts_verify_prepared(c, accept, n, n_pks, n_msgs, sigs, msg_idx, pk_idx, q.s);
}
extern "C" int lcb_ctx_ts_assemble_dev(lcb_ctx *ctx, uint8_t *sig_out, uint8_t *status, const uint8_t *accept,
                                       const uint8_t *sigs, size_t per_round, size_t k, size_t n_rounds, void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    return assemble_enqueue(c, 2, sig_out, status, accept, sigs, per_round, k, n_rounds, q.s);
}
extern "C" int lcb_ctx_ts_assemble_ordered_dev(lcb_ctx *ctx, uint8_t *sig_out, uint8_t *status, const uint8_t *accept,
                                               const uint8_t *sigs, const uint32_t *order, size_t per_round, size_t k,
                                               size_t n_rounds, void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    return assemble_enqueue(c, 2, sig_out, status, accept, sigs, per_round, k, n_rounds, q.s, order);
}
extern "C" int lcb_ts_assemble_ordered_dev(uint8_t *sig_out, uint8_t *status, const uint8_t *accept, const uint8_t *sigs,
                                          const uint32_t *order, size_t per_round, size_t k, size_t n_rounds,
                                          void *stream) {
    return lcb_ctx_ts_assemble_ordered_dev(nullptr, sig_out, status, accept, sigs, order, per_round, k, n_rounds, stream);
}
extern "C" int lcb_ts_prepare_dev(const uint8_t *pks, size_t n_pks, const uint8_t *msg_data, const uint32_t *msg_off,
                                  size_t n_msgs, void *stream) {
    return lcb_ctx_ts_prepare_dev(nullptr, pks, n_pks, msg_data, msg_off, n_msgs, stream);
}
extern "C" int lcb_ts_verify_prepared_dev(uint8_t *accept, size_t n, size_t n_pks, size_t n_msgs, const uint8_t *sigs,
                                          const uint32_t *msg_idx, const uint32_t *pk_idx, void *stream) {
    return lcb_ctx_ts_verify_prepared_dev(nullptr, accept, n, n_pks, n_msgs, sigs, msg_idx, pk_idx, stream);
}
extern "C" int lcb_ts_assemble_dev(uint8_t *sig_out, uint8_t *status, const uint8_t *accept, const uint8_t *sigs,
                                   size_t per_round, size_t k, size_t n_rounds, void *stream) {
    return lcb_ctx_ts_assemble_dev(nullptr, sig_out, status, accept, sigs, per_round, k, n_rounds, stream);
}
extern "C" int lcb_ts_verify_shares_dev(uint8_t *accept, size_t n, const uint8_t *pks, size_t n_pks, const uint8_t *sigs,
                                        const uint8_t *msg_data, const uint32_t *msg_off, size_t n_msgs,
                                        const uint32_t *msg_idx, const uint32_t *pk_idx, void *stream) {
    CTX_OR(c, nullptr, -1)
    Enq q(c, (hipStream_t)stream);
    if (ts_prepare(c, pks, n_pks, msg_data, msg_off, n_msgs, q.s)) return -1;
    return ts_verify_prepared(c, accept, n, n_pks, n_msgs, sigs, msg_idx, pk_idx, q.s);
}
extern "C" int lcb_ctx_ts_verify_prepared_batched_dev(lcb_ctx *ctx, uint8_t *accept, size_t n, size_t n_pks,
                                                      size_t n_msgs, const uint8_t *sigs, const uint32_t *msg_idx,
                                                      const uint32_t *pk_idx, void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    return ts_verify_prepared_rlc(c, accept, n, n_pks, n_msgs, sigs, msg_idx, pk_idx, q.s);
}
extern "C" int lcb_ts_verify_prepared_batched_dev(uint8_t *accept, size_t n, size_t n_pks, size_t n_msgs,
                                                  const uint8_t *sigs, const uint32_t *msg_idx, const uint32_t *pk_idx,
                                                  void *stream) {
    return lcb_ctx_ts_verify_prepared_batched_dev(nullptr, accept, n, n_pks, n_msgs, sigs, msg_idx, pk_idx, stream);
}
extern "C" int lcb_ctx_ts_verify_shares_batched_dev(lcb_ctx *ctx, uint8_t *accept, size_t n, const uint8_t *pks,
                                                    size_t n_pks, const uint8_t *sigs, const uint8_t *msg_data,
                                                    const uint32_t *msg_off, size_t n_msgs, const uint32_t *msg_idx,
                                                    const uint32_t *pk_idx, void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    return ts_verify_shares_rlc_fused(c, accept, n, pks, n_pks, sigs, msg_data, msg_off, n_msgs, msg_idx, pk_idx, q.s);
}
extern "C" int lcb_ts_verify_shares_batched_dev(uint8_t *accept, size_t n, const uint8_t *pks, size_t n_pks,
                                                const uint8_t *sigs, const uint8_t *msg_data, const uint32_t *msg_off,
                                                size_t n_msgs, const uint32_t *msg_idx, const uint32_t *pk_idx,
                                                void *stream) {
    return lcb_ctx_ts_verify_shares_batched_dev(nullptr, accept, n, pks, n_pks, sigs, msg_data, msg_off, n_msgs,
                                                msg_idx, pk_idx, stream);
}
static int ts_verify_shares_host(uint8_t *accept, size_t n, const uint8_t *pks, size_t n_pks, const uint8_t *sigs,
                                 const uint8_t *msg_data, const uint32_t *msg_off, size_t n_msgs,
                                 const uint32_t *msg_idx, const uint32_t *pk_idx, bool batched) {
    SYNC_CTX_OR(c, -1)
    for (size_t i = 0; i < n; i++) {
        if (msg_idx[i] >= n_msgs) { set_err("msg_idx out of range"); return -1; }
        if (pk_idx[i] >= n_pks) { set_err("pk_idx out of range"); return -1; }
    }
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    size_t mbytes = n_msgs ? msg_off[n_msgs] : 0;
    const uint8_t *dpk = up(c->in[0], pks, 48 * n_pks, s);
    const uint8_t *dsig = up(c->in[1], sigs, 96 * n, s);
    const uint8_t *dm = up(c->in[2], msg_data, mbytes, s);
    const uint32_t *dmo = up(c->in[3], msg_off, n_msgs + 1, s);
    const uint32_t *dmi = up(c->in[4], msg_idx, n, s);
    const uint32_t *dpi = up(c->in[5], pk_idx, n, s);
    uint8_t *dacc = (uint8_t *)c->out[0].get(n);
    if (!dpk || !dsig || !dm || !dmo || !dmi || !dpi || !dacc) { set_err("device allocation failed"); return -1; }
    if (batched) {
        if (ts_verify_shares_rlc_fused(c, dacc, n, dpk, n_pks, dsig, dm, dmo, n_msgs, dmi, dpi, s)) return -1;
    } else {
        if (ts_prepare(c, dpk, n_pks, dm, dmo, n_msgs, s)) return -1;
        if (ts_verify_prepared(c, dacc, n, n_pks, n_msgs, dsig, dmi, dpi, s)) return -1;
    }
    if (n) hipMemcpyAsync(accept, dacc, n, hipMemcpyDeviceToHost, s);
    return sync_check(c, "ts verify") ? 0 : -1;
}
extern "C" int lcb_ts_verify_shares(uint8_t *accept, size_t n, const uint8_t *pks, size_t n_pks, const uint8_t *sigs,
                                    const uint8_t *msg_data, const uint32_t *msg_off, size_t n_msgs,
                                    const uint32_t *msg_idx, const uint32_t *pk_idx) {
    return ts_verify_shares_host(accept, n, pks, n_pks, sigs, msg_data, msg_off, n_msgs, msg_idx, pk_idx, false);
}
extern "C" int lcb_ts_verify_shares_batched(uint8_t *accept, size_t n, const uint8_t *pks, size_t n_pks,
                                            const uint8_t *sigs, const uint8_t *msg_data, const uint32_t *msg_off,
                                            size_t n_msgs, const uint32_t *msg_idx, const uint32_t *pk_idx) {
    return ts_verify_shares_host(accept, n, pks, n_pks, sigs, msg_data, msg_off, n_msgs, msg_idx, pk_idx, true);
}
extern "C" int lcb_ts_sign(uint8_t *sigs_out, const uint8_t *sks, const uint8_t *msg_data, const uint32_t *msg_off,
                           const uint32_t *msg_idx, size_t n) {
    SYNC_CTX_OR(c, -1)
    if (!n) return 0;
    u32 nm = 0;
    for (size_t i = 0; i < n; i++) nm = msg_idx[i] + 1 > nm ? msg_idx[i] + 1 : nm;
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const uint8_t *dsk = up(c->in[0], sks, 32 * n, s);
    const uint8_t *dm = up(c->in[1], msg_data, msg_off[nm], s);
    const uint32_t *dmo = up(c->in[2], msg_off, nm + 1, s);
    const uint32_t *dmi = up(c->in[3], msg_idx, n, s);
    uint8_t *dsig = (uint8_t *)c->out[0].get(96 * n), *dok = (uint8_t *)c->out[1].get(n);
    if (!dsk || !dm || !dmo || !dmi || !dsig || !dok) { set_err("device allocation failed"); return -1; }
    lcbk_ts_sign(dim3(nblk(n)), s, dsk, dm, dmo, dmi, (u32)n, dsig, dok, g_orig_cofactor);
    std::vector<uint8_t> ok(n);
    hipMemcpyAsync(sigs_out, dsig, 96 * n, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(ok.data(), dok, n, hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "ts sign")) return -1;
    for (size_t i = 0; i < n; i++) if (!ok[i]) { set_err("invalid key share"); return -1; }
    return 0;
}

// ================================================================== coin consumers (CoinResult.Parity, block nonce)
extern "C" int lcb_coin_parity(const uint8_t *sig_bytes, size_t len) {
    uint32_t acc = 0;
    for (size_t i = 0; i < len; i++) acc ^= sig_bytes[i];
    return __builtin_popcount(acc) & 1;
}
extern "C" uint64_t lcb_coin_nonce(const uint8_t *sig_bytes, size_t len) {
    uint8_t r[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (size_t i = 0; i < len; i++) r[i % 8] ^= sig_bytes[i];
    uint64_t v = 0;
    for (int j = 7; j >= 0; j--) v = (v << 8) | r[j];
    return v;
}
extern "C" int lcb_coin_fold_dev(uint8_t *parity, uint64_t *nonce, const uint8_t *sigs, size_t n, void *stream) {
    if (!ready()) return -1;
    if (n > 0xffffffffu) { set_err("coin fold: batch too large"); return -1; }
    if (n) lcbk_coin_fold(dim3(nblk(n)), (hipStream_t)stream, sigs, (u32)n, parity, nonce);
    return launched("coin fold launch") ? 0 : -1;
}

// ================================================================== trustless DKG G1 work (k_dkg.hip)
// Commitment.Evaluate(x, y) / Evaluate(x) (src/Lachain.Consensus/ThresholdKeygen/Data/Commitment.cs:23-53) for whole
// batches: rows of every distinct (commitment, x) once, then Horner in y per query.
namespace {
// any decodable point of d_aff (n records) outside G1 (k_g1_subgroup_any; one 4-byte read)
int g1_any_off_subgroup(lcb_ctx *c, const void *d_aff, size_t n, hipStream_t s, bool *any) {
    u32 *d = (u32 *)c->dkg[8].get(4);
    if (!d) { set_err("device allocation failed"); return -1; }
    hipMemsetAsync(d, 0, 4, s);
    if (n) lcbk_g1_subgroup_any(s, d_aff, (u32)n, d);
    u32 h = 0;
    if (!launched("subgroup test launch") || !read_counts(&h, d, 1, s)) return -1;
    *any = h != 0;
    return 0;
}
// Commitment.Evaluate(x) rows of n_rows (commitment, x) pairs.  Honest commitments (every coefficient in G1): Horner in
// the small x (k_dkg_rows).  A batch with a coefficient outside G1: the reference's own terms [x^j mod r] C (exact).
int dkg_rows_enqueue(lcb_ctx *c, const uint8_t *d_coeffs, size_t n_comm, size_t n_coef, int degree,
                     const uint32_t *d_comm, const int32_t *d_xs, size_t n_rows, hipStream_t s, void **rows_out,
                     uint8_t **rows_ok, bool *exact) {
    size_t total = n_comm * n_coef, lanes = n_rows * (size_t)(degree + 1);
    if (total > 0xffffffffu || lanes > 0xffffffffu) { set_err("dkg: batch too large"); return -1; }
    void *aff = c->dkg[0].get(total * LCB_G1A_ST_BYTES);
    void *rows = c->dkg[1].get(lanes * LCB_G1_JAC_BYTES);
    uint8_t *rok = (uint8_t *)c->dkg[2].get(lanes);
    if (!aff || !rows || !rok) { set_err("device allocation failed"); return -1; }
    if (total) lcbk_g1_decompress(dim3(nblk(total)), s, d_coeffs, (u32)total, aff);
    if (g1_any_off_subgroup(c, aff, total, s, exact)) return -1;
    if (lanes && !*exact) {
        lcbk_dkg_rows(dim3(nblk(lanes)), s, aff, (u32)n_coef, (u32)n_comm, (u32)degree, d_comm, d_xs, (u32)n_rows, rows,
                      rok);
    } else if (lanes) {
        const size_t nt = lanes * (size_t)(degree + 1);
        if (nt > 0xffffffffu) { set_err("dkg: batch too large for the exact form"); return -1; }
        void *terms = c->dkg[6].get(nt * LCB_G1_JAC_BYTES);
        uint8_t *tok = (uint8_t *)c->dkg[7].get(nt);
        if (!terms || !tok) { set_err("device allocation failed"); return -1; }
        lcbk_dkg_exact_terms(s, aff, (u32)n_coef, (u32)n_comm, (u32)degree, d_comm, d_xs, (u32)n_rows, terms, tok);
        lcbk_g1_jac_reduce_groups(dim3(nblk(lanes)), s, terms, (u32)nt, (u32)(degree + 1), rows);
        lcbk_and_groups(s, tok, (u32)lanes, (u32)(degree + 1), rok);
    }
    *rows_out = rows;
    *rows_ok = rok;
    return launched("dkg rows launch") ? 0 : -1;
}
bool dkg_shape(size_t n_comm, int degree, size_t *n_coef) {
    if (degree < 0 || degree > 4096) { set_err("dkg: degree out of range"); return false; }
    *n_coef = (size_t)(degree + 1) * (size_t)(degree + 2) / 2;
    (void)n_comm;
    return true;
}
}  // namespace
extern "C" int lcb_dkg_commitment_rows(uint8_t *rows_out, uint8_t *status, const uint8_t *coeffs, size_t n_comm,
                                       int degree, const uint32_t *comm_idx, const int32_t *xs, size_t n_queries) {
    SYNC_CTX_OR(c, -1)
    size_t n_coef;
    if (!dkg_shape(n_comm, degree, &n_coef)) return -1;
    if (!n_queries) return 0;
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    size_t lanes = n_queries * (size_t)(degree + 1);
    const uint8_t *dco = up(c->in[0], coeffs, 48 * n_comm * n_coef, s);
    const uint32_t *dci = up(c->in[1], comm_idx, n_queries, s);
    const int32_t *dx = up(c->in[2], xs, n_queries, s);
    uint8_t *dout = (uint8_t *)c->out[0].get(48 * lanes);
    if (!dco || !dci || !dx || !dout) { set_err("device allocation failed"); return -1; }
    void *rows;
    uint8_t *rok;
    bool exact = false;
    if (dkg_rows_enqueue(c, dco, n_comm, n_coef, degree, dci, dx, n_queries, s, &rows, &rok, &exact)) return -1;
    lcbk_g1_jac_compress(dim3(nblk(lanes)), s, rows, (u32)lanes, dout);
    std::vector<uint8_t> ok(lanes);
    hipMemcpyAsync(rows_out, dout, 48 * lanes, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(ok.data(), rok, lanes, hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "dkg rows")) return -1;
    for (size_t qi = 0; qi < n_queries; qi++) {
        uint8_t st = 1;
        for (int i = 0; i <= degree; i++) st &= ok[qi * (degree + 1) + i];
        status[qi] = st;
    }
    return 0;
}
extern "C" int lcb_dkg_commitment_eval(uint8_t *out, uint8_t *status, const uint8_t *coeffs, size_t n_comm, int degree,
                                       const uint32_t *comm_idx, const int32_t *xs, const int32_t *ys,
                                       size_t n_queries) {
    SYNC_CTX_OR(c, -1)
    size_t n_coef;
    if (!dkg_shape(n_comm, degree, &n_coef)) return -1;
    if (!n_queries) return 0;
    // distinct (commitment, x) pairs -> rows; every query evaluates its row at y
    std::vector<uint32_t> row_comm, row_of(n_queries);
    std::vector<int32_t> row_x;
    {
        std::vector<std::pair<uint64_t, uint32_t>> keys(n_queries);
        for (size_t i = 0; i < n_queries; i++) keys[i] = {((uint64_t)comm_idx[i] << 32) | (uint32_t)xs[i], (uint32_t)i};
        std::sort(keys.begin(), keys.end());
        for (size_t i = 0; i < n_queries; i++) {
            if (i == 0 || keys[i].first != keys[i - 1].first) {
                row_comm.push_back((uint32_t)(keys[i].first >> 32));
                row_x.push_back((int32_t)(uint32_t)keys[i].first);
            }
            row_of[keys[i].second] = (uint32_t)(row_comm.size() - 1);
        }
    }
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const uint8_t *dco = up(c->in[0], coeffs, 48 * n_comm * n_coef, s);
    const uint32_t *drc = up(c->in[1], row_comm.data(), row_comm.size(), s);
    const int32_t *drx = up(c->in[2], row_x.data(), row_x.size(), s);
    const uint32_t *drow = up(c->in[3], row_of.data(), n_queries, s);
    const int32_t *dy = up(c->in[4], ys, n_queries, s);
    uint8_t *dout = (uint8_t *)c->out[0].get(48 * n_queries), *dst = (uint8_t *)c->out[1].get(n_queries);
    if (!dco || !drc || !drx || !drow || !dy || !dout || !dst) { set_err("device allocation failed"); return -1; }
    void *rows;
    uint8_t *rok;
    bool exact = false;
    if (dkg_rows_enqueue(c, dco, n_comm, n_coef, degree, drc, drx, row_comm.size(), s, &rows, &rok, &exact)) return -1;
    if (!exact) {
        lcbk_dkg_horner(dim3(nblk(n_queries)), s, rows, rok, (u32)degree, drow, dy, (u32)n_queries, dout, dst, 0);
        hipMemcpyAsync(out, dout, 48 * n_queries, hipMemcpyDeviceToHost, s);
        hipMemcpyAsync(status, dst, n_queries, hipMemcpyDeviceToHost, s);
        return sync_check(c, "dkg eval") ? 0 : -1;
    }
    // a coefficient outside G1: sum_j [y^j mod r] row_j(x) (Commitment.cs:23-37 as written)
    const size_t D1 = (size_t)degree + 1, nt = n_queries * D1;
    void *terms = c->dkg[6].get(nt * LCB_G1_JAC_BYTES), *sums = c->dkg[3].get(n_queries * LCB_G1_JAC_BYTES);
    if (!terms || !sums) { set_err("device allocation failed"); return -1; }
    lcbk_dkg_exact_combine(s, rows, (u32)degree, drow, dy, (u32)n_queries, terms);
    lcbk_g1_jac_reduce_groups(dim3(nblk(n_queries)), s, terms, (u32)nt, (u32)D1, sums);
    lcbk_g1_jac_compress(dim3(nblk(n_queries)), s, sums, (u32)n_queries, dout);
    std::vector<uint8_t> rk(row_comm.size() * D1);
    hipMemcpyAsync(out, dout, 48 * n_queries, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(rk.data(), rok, rk.size(), hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "dkg eval")) return -1;
    for (size_t qi = 0; qi < n_queries; qi++) {
        uint8_t st = 1;
        for (size_t j = 0; j < D1; j++) st &= rk[row_of[qi] * D1 + j];
        status[qi] = st;
        if (!st) memset(out + 48 * qi, 0, 48);
    }
    return 0;
}
extern "C" int lcb_g1_eval_poly_batch(uint8_t *out, uint8_t *status, const uint8_t *coeffs, size_t n_coeffs,
                                      const int32_t *xs, size_t n_points) {
    SYNC_CTX_OR(c, -1)
    if (!n_coeffs) { set_err("eval poly: no coefficients"); return -1; }
    if (!n_points) return 0;
    if (n_coeffs > 0xffffffffu || n_points > 0xffffffffu) { set_err("eval poly: batch too large"); return -1; }
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const uint8_t *dco = up(c->in[0], coeffs, 48 * n_coeffs, s);
    const int32_t *dx = up(c->in[1], xs, n_points, s);
    void *aff = c->dkg[0].get(n_coeffs * LCB_G1A_ST_BYTES), *rows = c->dkg[1].get(n_coeffs * LCB_G1_JAC_BYTES);
    uint8_t *rok = (uint8_t *)c->dkg[2].get(n_coeffs);
    uint32_t *drow = (uint32_t *)c->dkg[3].get(4 * n_points);
    uint8_t *dout = (uint8_t *)c->out[0].get(48 * n_points), *dst = (uint8_t *)c->out[1].get(n_points);
    if (!dco || !dx || !aff || !rows || !rok || !drow || !dout || !dst) { set_err("device allocation failed"); return -1; }
    hipMemsetAsync(drow, 0, 4 * n_points, s);    // every point evaluates row 0 (the coefficient vector)
    lcbk_g1_decompress(dim3(nblk(n_coeffs)), s, dco, (u32)n_coeffs, aff);
    bool off = false;                            // a coefficient outside G1: negative x multiply by Fr.FromInt(x)
    bool neg = false;
    for (size_t i = 0; i < n_points; i++) neg |= xs[i] < 0;
    if (neg && g1_any_off_subgroup(c, aff, n_coeffs, s, &off)) return -1;
    lcbk_g1a_to_jac(dim3(nblk(n_coeffs)), s, aff, (u32)n_coeffs, rows, rok);
    lcbk_dkg_horner(dim3(nblk(n_points)), s, rows, rok, (u32)(n_coeffs - 1), drow, dx, (u32)n_points, dout, dst,
                    off ? 1u : 0u);
    hipMemcpyAsync(out, dout, 48 * n_points, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(status, dst, n_points, hipMemcpyDeviceToHost, s);
    return sync_check(c, "eval poly") ? 0 : -1;
}

// ================================================================== reliable-broadcast Reed-Solomon (k_rs.hip)
// ReliableBroadcast.ErasureCodingShards / DecodeFromEchos (src/Lachain.Consensus/ReliableBroadcast/ReliableBroadcast.cs:
// 393-446): the erased / parity shards are M times the known shards, M = H_E^-1 H_K built on the GPU.
namespace {
int rs_enqueue(lcb_ctx *c, uint8_t *d_out, const uint8_t *d_known, const std::vector<int> &pe,
               const std::vector<int> &pk, int n, size_t S, hipStream_t s, uint8_t **d_ok) {
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute((const void *)lcbk_rs_matrix_kernel(), hipFuncAttributeMaxDynamicSharedMemorySize, 65536 * 2);
        attr = true;
    }
    int m = (int)pe.size(), k = (int)pk.size();
    int *dpe = (int *)c->dkg[4].get(4 * (pe.size() + pk.size()));
    uint8_t *M = (uint8_t *)c->dkg[5].get((size_t)m * k + 16);
    if (!dpe || !M) { set_err("device allocation failed"); return -1; }
    std::vector<int> both(pe);
    both.insert(both.end(), pk.begin(), pk.end());
    hipMemcpyAsync(dpe, both.data(), 4 * both.size(), hipMemcpyHostToDevice, s);
    uint8_t *ok = M + (size_t)m * k;
    lcbk_rs_matrix(s, dpe, m, dpe + m, k, n, M, ok);
    lcbk_rs_apply(s, M, ok, m, k, d_known, S, dpe, d_out);
    *d_ok = ok;
    return launched("rs launch") ? 0 : -1;
}
}  // namespace
extern "C" int lcb_rs_encode(uint8_t *shards_out, const uint8_t *input, size_t input_len, int n_shards, int erasures) {
    SYNC_CTX_OR(c, -1)
    int k = n_shards - erasures;
    if (n_shards <= 0 || erasures < 0 || k <= 0 || input_len % (size_t)k) {
        set_err("rs encode: need 0 <= erasures < shards and input length divisible by the data shards");
        return -1;
    }
    size_t S = input_len / (size_t)k;
    if (erasures == 0 || S == 0) { memcpy(shards_out, input, input_len); return 0; }
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    uint8_t *dout = (uint8_t *)c->out[0].get(S * n_shards);
    if (!dout) { set_err("device allocation failed"); return -1; }
    hipMemcpyAsync(dout, input, input_len, hipMemcpyHostToDevice, s);   // data shards stay in place (systematic)
    std::vector<int> pe, pk;
    for (int j = k; j < n_shards; j++) pe.push_back(j);
    for (int j = 0; j < k; j++) pk.push_back(j);
    uint8_t *dok;
    if (rs_enqueue(c, dout, dout, pe, pk, n_shards, S, s, &dok)) return -1;
    uint8_t ok = 0;
    hipMemcpyAsync(shards_out, dout, S * n_shards, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(&ok, dok, 1, hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "rs encode")) return -1;
    if (!ok) { set_err("rs encode: parity positions are not independent (more than 255 shards)"); return -1; }
    return 0;
}
extern "C" int lcb_rs_decode(uint8_t *out, const uint8_t *echo_data, const int32_t *from, int n_echos, size_t shard_size,
                             int n_shards, int erasures) {
    SYNC_CTX_OR(c, -1)
    int k = n_shards - erasures;
    if (n_shards <= 0 || erasures < 0 || k <= 0 || n_echos != k) {
        set_err("rs decode: need exactly shards - erasures echoes (DecodeFromEchos asserts N - 2F)");
        return -1;
    }
    std::vector<char> have(n_shards, 0);
    std::vector<int> pe, pk;
    for (int e = 0; e < n_echos; e++) {
        if (from[e] < 0 || from[e] >= n_shards || have[from[e]]) { set_err("rs decode: bad or duplicate echo index"); return -1; }
        have[from[e]] = 1;
        pk.push_back(from[e]);
    }
    for (int j = 0; j < n_shards; j++) if (!have[j]) pe.push_back(j);
    size_t S = shard_size;
    if (S == 0) return 0;
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    uint8_t *dout = (uint8_t *)c->out[0].get(S * n_shards);
    const uint8_t *decho = up(c->in[0], echo_data, S * (size_t)n_echos, s);
    if (!dout || !decho) { set_err("device allocation failed"); return -1; }
    for (int e = 0; e < n_echos; e++)
        hipMemcpyAsync(dout + (size_t)from[e] * S, decho + (size_t)e * S, S, hipMemcpyDeviceToDevice, s);
    uint8_t ok = 1;
    if (!pe.empty()) {
        uint8_t *dok;
        if (rs_enqueue(c, dout, decho, pe, pk, n_shards, S, s, &dok)) return -1;
        hipMemcpyAsync(&ok, dok, 1, hipMemcpyDeviceToHost, s);
    }
    hipMemcpyAsync(out, dout, S * n_shards, hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "rs decode")) return -1;
    if (!ok) { set_err("rs decode: erased positions share an evaluation point (more than 255 shards)"); return -1; }
    return 0;
}

// ================================================================== batch: Lagrange, scalar mul, hash, MSM
static int lagrange_batch(int g, uint8_t *out, uint8_t *status, const uint8_t *xs, const uint8_t *ys, const uint32_t *off,
                          size_t np) {
    SYNC_CTX_OR(c, -1)
    if (!np) return 0;
    Enq q(c, c->stream);
    size_t ne = off[np];
    size_t pb = g == 1 ? 48 : 96;
    hipStream_t s = c->stream;
    const uint8_t *dx = up(c->in[0], xs, 32 * ne, s);
    const uint8_t *dy = up(c->in[1], ys, pb * ne, s);
    const uint32_t *doff = up(c->in[2], off, np + 1, s);
    uint8_t *dst = (uint8_t *)c->out[0].get(np), *dout = (uint8_t *)c->out[1].get(pb * np);
    if (!dx || !dy || !doff || !dst || !dout) { set_err("device allocation failed"); return -1; }
    if (lagrange_enqueue(c, g, dout, dst, dx, dy, doff, np, ne, s)) return -1;
    hipMemcpyAsync(out, dout, pb * np, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(status, dst, np, hipMemcpyDeviceToHost, s);
    return sync_check(c, "lagrange") ? 0 : -1;
}
extern "C" int lcb_ctx_g1_lagrange_dev(lcb_ctx *ctx, uint8_t *out, uint8_t *status, const uint8_t *xs, const uint8_t *ys,
                                       const uint32_t *off, size_t n_problems, size_t n_entries, void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    return n_problems ? lagrange_enqueue(c, 1, out, status, xs, ys, off, n_problems, n_entries, q.s) : 0;
}
extern "C" int lcb_ctx_g2_lagrange_dev(lcb_ctx *ctx, uint8_t *out, uint8_t *status, const uint8_t *xs, const uint8_t *ys,
                                       const uint32_t *off, size_t n_problems, size_t n_entries, void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    return n_problems ? lagrange_enqueue(c, 2, out, status, xs, ys, off, n_problems, n_entries, q.s) : 0;
}
extern "C" int lcb_g1_lagrange_dev(uint8_t *out, uint8_t *status, const uint8_t *xs, const uint8_t *ys,
                                   const uint32_t *off, size_t n_problems, size_t n_entries, void *stream) {
    return lcb_ctx_g1_lagrange_dev(nullptr, out, status, xs, ys, off, n_problems, n_entries, stream);
}
extern "C" int lcb_g2_lagrange_dev(uint8_t *out, uint8_t *status, const uint8_t *xs, const uint8_t *ys,
                                   const uint32_t *off, size_t n_problems, size_t n_entries, void *stream) {
    return lcb_ctx_g2_lagrange_dev(nullptr, out, status, xs, ys, off, n_problems, n_entries, stream);
}
extern "C" int lcb_g1_lagrange_batch(uint8_t *out, uint8_t *status, const uint8_t *xs, const uint8_t *ys,
                                     const uint32_t *off, size_t n) { return lagrange_batch(1, out, status, xs, ys, off, n); }
extern "C" int lcb_g2_lagrange_batch(uint8_t *out, uint8_t *status, const uint8_t *xs, const uint8_t *ys,
                                     const uint32_t *off, size_t n) { return lagrange_batch(2, out, status, xs, ys, off, n); }

// ================================================================== mcl surface on the batch / cooperative kernels
// (k_mcl.hip, k_coop.hip) — each a single synchronous call on the calling thread's own context

#define LCB_PAIR_CACHE 32    // line-set slots per context (2 x 26 KB each)
// mclBn_pairing (GT.Pairing: TPKE/PrivateKey.cs:26, TPKE/PublicKey.cs:91, ThresholdSignature/PublicKey.cs:20) as a
// one-group cooperative check: P and the point at infinity, Q's normalised line set and the set of infinity, then
// the nine-lane final exponentiation.  The lines are normalised (divided by their Fp2 leading coefficient), which
// changes the Miller value by a factor the final exponentiation removes: the GT value is mcl's.
// The line set of one G2 point on the host (pairing.hpp lineset_compute: the same 68 steps and formulas with the host
// field code, which gives the kernels' canonical residues; the normalised lines B' = Bc / A, C' = Cc / A depend only on
// the affine points, so they are the words k_lineset_coop writes).  False when some A_k == 0 (a point outside G2: the
// caller then takes the kernel, whose Miller loop computes such a set's lines on the fly).
static const bool g_pair_host_lines = !(getenv("LCB_PAIR_HOST_LINES") && atoi(getenv("LCB_PAIR_HOST_LINES")) == 0);
static bool lineset_host(uint32_t *dst, const fph::g2a &Q) {
    const int PT = LCB_LS_POINT_WORD, FLAG = PT + 48, NL = 68, NLW = 48;
    memset(dst, 0, LCB_LINESET_BYTES);
    memcpy(dst + PT, &Q.x, 96);
    memcpy(dst + PT + 24, &Q.y, 96);
    dst[FLAG + 1] = Q.inf ? 1u : 0u;
    if (Q.inf) { dst[FLAG] = 1u; return true; }   // every line is the constant 1: B' = C' = 0
    fph::fp twelve, raw12 = fph::zero();
    raw12.v[0] = 12;
    fph::from_raw(twelve, raw12);
    fph::fp2 b3;                                  // 3 b' = 12 (1 + u)
    b3.a = twelve;
    b3.b = twelve;
    fph::fp2 Tx = Q.x, Ty = Q.y, Tz = fph::one2();
    std::vector<fph::fp2> A(NL), B(NL), C(NL);
    int k = 0;
    for (int i = 62; i >= 0; i--) {
        {   // doubling step (ls_dbl_store): A = Y^2 - 3b'Z^2, Bc = -3X^2, Cc = 2YZ; T <- 2T
            fph::fp2 YZ, XY, ZZ, YY, t, u;
            fph::mul(YZ, Ty, Tz);
            fph::mul(XY, Tx, Ty);
            fph::sqr(ZZ, Tz);
            fph::sqr(YY, Ty);
            fph::sqr(t, Tx);
            fph::add(u, t, t);
            fph::add(u, u, t);
            fph::neg(B[k], u);
            fph::add(C[k], YZ, YZ);
            fph::mul(Tz, YY, YZ);
            fph::add(Tz, Tz, Tz);
            fph::mul(ZZ, ZZ, b3);
            fph::sub(A[k], YY, ZZ);
            k++;
            fph::add(t, ZZ, ZZ);
            fph::add(t, t, ZZ);
            fph::mul_fp(XY, XY, fph::INV2);
            fph::sub(u, YY, t);
            fph::mul(Tx, XY, u);
            fph::add(u, YY, t);
            fph::mul_fp(u, u, fph::INV2);
            fph::sqr(Ty, u);
            fph::sqr(t, ZZ);
            fph::add(u, t, t);
            fph::add(u, u, t);
            fph::sub(Ty, Ty, u);
        }
        if ((Z_ABS_H >> i) & 1) {   // addition step (ls_add_store): A = th xQ - la yQ, Bc = -th, Cc = la; T <- T + Q
            fph::fp2 th, la, t, D, E, G;
            fph::mul(t, Q.y, Tz);
            fph::sub(th, Ty, t);
            fph::mul(t, Q.x, Tz);
            fph::sub(la, Tx, t);
            fph::mul(A[k], th, Q.x);
            fph::mul(t, la, Q.y);
            fph::sub(A[k], A[k], t);
            fph::neg(B[k], th);
            C[k] = la;
            k++;
            fph::sqr(D, la);
            fph::mul(E, la, D);
            fph::mul(G, Tx, D);
            fph::sqr(t, th);
            fph::mul(D, Tz, t);
            fph::mul(Tz, Tz, E);
            fph::add(D, E, D);
            fph::sub(D, D, G);
            fph::sub(D, D, G);
            fph::mul(Tx, la, D);
            fph::sub(t, G, D);
            fph::mul(G, th, t);
            fph::mul(t, Ty, E);
            fph::sub(Ty, G, t);
        }
    }
    if (k != NL) return false;
    std::vector<fph::fp2> pre(NL);                // A_0 ... A_k, then one inversion (Montgomery's trick)
    pre[0] = A[0];
    for (int j = 1; j < NL; j++) fph::mul(pre[j], pre[j - 1], A[j]);
    if (fph::is_zero(pre[NL - 1])) return false;
    fph::fp2 inv;
    fph::inv(inv, pre[NL - 1]);
    for (int j = NL - 1; j >= 0; j--) {
        fph::fp2 ai, b, c;
        if (j > 0) fph::mul(ai, inv, pre[j - 1]);
        else ai = inv;
        fph::mul(inv, inv, A[j]);
        fph::mul(b, B[j], ai);
        fph::mul(c, C[j], ai);
        memcpy(dst + j * NLW, &b, 96);
        memcpy(dst + j * NLW + 24, &c, 96);
    }
    dst[FLAG] = 1u;
    return true;
}
extern "C" void mclBn_pairing(mclBnGT *z, const mclBnG1 *x, const mclBnG2 *y) {
    fail_out(z, 576);                  // overwritten on success; a failed call leaves a value no other call produces
    if (injected(INJ_PAIRING_ALLOC)) { set_err("injected failure (pairing)"); return; }
    SYNC_CTX_OR(c, )
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const size_t slots = lcbk_fe_slots() > 6 ? (size_t)lcbk_fe_slots() : 6;
    // the group record (P and infinity, then the check's descriptor), staged in one copy
    struct PairIn {
        uint32_t g[2][LCB_G1A_ST_BYTES / 4];
        uint32_t desc[4];
    };
    static_assert(sizeof(PairIn) == 2 * LCB_G1A_ST_BYTES + 16, "PairIn layout");
    uint8_t *gin = (uint8_t *)c->mcl[1].get(sizeof(PairIn));
    u32 *lines = (u32 *)c->pc_lines.get((size_t)2 * LCB_PAIR_CACHE * LCB_LINESET_BYTES);
    u32 *park = (u32 *)c->mcl[4].get(576 * slots);
    uint8_t *fl = (uint8_t *)c->mcl[5].get(64);
    if (!gin || !lines || !park || !fl) { set_err("device allocation failed"); return; }
    void *gpts = gin, *desc = gin + 2 * LCB_G1A_ST_BYTES;
    if (c->pc_used.empty()) {
        c->pc_keys.assign((size_t)72 * LCB_PAIR_CACHE, 0);
        c->pc_used.assign(LCB_PAIR_CACHE, 0);
    }
    u32 slot = 0;
    bool hit = false;
    for (u32 k = 0; k < LCB_PAIR_CACHE; k++) {
        if (c->pc_used[k] && memcmp(&c->pc_keys[72 * (size_t)k], y, 288) == 0) { slot = k; hit = true; break; }
        if (c->pc_used[k] < c->pc_used[slot]) slot = k;
    }
    c->pc_used[slot] = ++c->pc_tick;
    if (!hit) memcpy(&c->pc_keys[72 * (size_t)slot], y, 288);
    // P and Q to affine on the calling thread (host inversions, tens of us) rather than in a one-lane kernel (~0.5 ms
    // per inversion): the same canonical residues the device's jac_to_aff gives
    PairIn pin;
    memset(&pin, 0, sizeof pin);
    {
        fph::g1 P;
        fph::g1a pa;
        memcpy(&P, x, sizeof P);
        fph::jac_to_aff(pa, P);
        memcpy(&pin.g[0][0], &pa.x, 48);
        memcpy(&pin.g[0][12], &pa.y, 48);
        pin.g[0][24] = pa.inf ? 1u : 0u;
        pin.g[0][25] = 1u;                           // ok
        pin.g[1][24] = 1u;                           // the point at infinity
        pin.g[1][25] = 1u;
        pin.desc[0] = 0u;                            // check 0: points 0 and 1, line-set pair `slot`
        pin.desc[1] = 1u;
        pin.desc[2] = slot;
    }
    hipMemcpyAsync(gin, &pin, sizeof pin, hipMemcpyHostToDevice, s);
    std::vector<uint32_t> hsets;                     // the host line sets (alive until the call's synchronisation)
    bool host_sets = false;
    if (!hit && g_pair_host_lines) {                 // Q's set and the infinity set computed here, one upload
        fph::g2 Q;
        fph::g2a qa, ia;
        memcpy(&Q, y, sizeof Q);
        fph::jac_to_aff(qa, Q);
        memset(&ia, 0, sizeof ia);
        ia.inf = true;
        hsets.assign((size_t)2 * LCB_LINESET_BYTES / 4, 0u);
        if (lineset_host(hsets.data(), qa) && lineset_host(hsets.data() + LCB_LINESET_BYTES / 4, ia)) {
            hipMemcpyAsync(lines + (size_t)2 * slot * (LCB_LINESET_BYTES / 4), hsets.data(), 2 * (size_t)LCB_LINESET_BYTES,
                           hipMemcpyHostToDevice, s);
            host_sets = true;
        }
    }
    if (!hit && !host_sets) {                        // the two sets' points for k_lineset_fill: Q, then infinity
        fph::g2 Q;
        fph::g2a qa;
        memcpy(&Q, y, sizeof Q);
        fph::jac_to_aff(qa, Q);
        uint32_t pt[2][51];                          // x, y (48 words), LCB_LS_FLAG, + 1 (infinity), + 2 (force general)
        memset(pt, 0, sizeof pt);
        memcpy(&pt[0][0], &qa.x, 96);
        memcpy(&pt[0][24], &qa.y, 96);
        pt[0][49] = qa.inf ? 1u : 0u;
        pt[1][49] = 1u;
        for (int k = 0; k < 2; k++)
            hipMemcpyAsync(lines + (size_t)(2 * slot + k) * (LCB_LINESET_BYTES / 4) + LCB_LS_POINT_WORD, pt[k],
                           sizeof pt[k], hipMemcpyHostToDevice, s);
    }
    if (!hit && !host_sets) lcbk_lineset_coop(s, lines + (size_t)2 * slot * (LCB_LINESET_BYTES / 4), 2, nullptr, nullptr);
    lcbk_coop_tpke_miller(s, lines, desc, gpts, 1, park, fl, fl + 32, 1, 1);
    lcbk_coop_final_exp_check(s, park, 1, nullptr);
    u32 r[144];
    hipMemcpyAsync(r, park, 576, hipMemcpyDeviceToHost, s);
    if (sync_check(c, "pairing")) memcpy(z, r, 576);
    else c->pc_used[slot] = 0;                    // the slot's lines may be incomplete
}
// mclBn_finalExp on the nine-lane kernel (park slot 0 of a one-value workspace)
extern "C" void mclBn_finalExp(mclBnGT *y, const mclBnGT *x) {
    mclBnGT xin = *x;                  // y may alias x
    x = &xin;
    fail_out(y, 576);
    SYNC_CTX_OR(c, )
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const size_t slots = lcbk_fe_slots() > 6 ? (size_t)lcbk_fe_slots() : 6;
    u32 *park = (u32 *)c->mcl[4].get(576 * slots);
    if (!park) { set_err("device allocation failed"); return; }
    hipMemcpyAsync(park, x, 576, hipMemcpyHostToDevice, s);
    lcbk_coop_final_exp_check(s, park, 1, nullptr);
    u32 r[144];
    hipMemcpyAsync(r, park, 576, hipMemcpyDeviceToHost, s);
    if (sync_check(c, "final exp")) memcpy(y, r, 576);
}
// sum_i [k_i] x_i (canonical scalars k_i < r, raw words) on the cooperative ladders of mclBnG1_mul: three groups per
// term (GLV halves over P and phi(P), and [z^2] P for the membership the split needs), k_ptmul_g1_multi, the terms
// added on the host.  Returns 1 with *z set, 0 when a term is not on the curve or outside G1 (the caller then takes
// its exact path, so every input keeps that path's value), -1 on a device error.
static const size_t MULVEC_COOP_MAX = 512;
static const bool g_mulvec_coop = !(getenv("LCB_MULVEC_COOP") && atoi(getenv("LCB_MULVEC_COOP")) == 0);
static int g1_mulvec_coop(lcb_ctx *c, mclBnG1 *z, const mclBnG1 *x, const uint64_t (*kraw)[4], size_t n) {
    std::vector<PtJobG1> jobs(3 * n);
    memset(jobs.data(), 0, jobs.size() * sizeof(PtJobG1));
    std::vector<fph::g1a> phis(n);
    std::vector<uint8_t> live(n, 0);
    const u128h zz = (u128h)Z_ABS_H * Z_ABS_H;
    const uint64_t z2[2] = {(uint64_t)zz, (uint64_t)(zz >> 64)}, zero[1] = {0};
    for (size_t i = 0; i < n; i++) {
        PtJobG1 *J = &jobs[3 * i];
        const uint64_t *k = kraw[i];
        fph::g1a P;
        fph::jac_to_aff(P, *G1R(&x[i]));
        if (!P.inf && !fph::jac_on_curve(*G1R(&x[i]))) return 0;
        if (P.inf || (k[0] | k[1] | k[2] | k[3]) == 0) {          // a zero term: three idle ladders
            for (int j = 0; j < 3; j++) { J[j].inf = 1; put_digits(J[j], zero, 1, 33); }
            continue;
        }
        uint64_t q[4] = {k[0], k[1], k[2], k[3]};
        const uint64_t d0 = divmod_u(q), d1 = divmod_u(q);
        const u128h a0 = (u128h)d1 * Z_ABS_H + d0, a1 = (u128h)q[1] << 64 | q[0];
        const u128h sum = a0 + a1;
        const uint64_t k1[3] = {(uint64_t)sum, (uint64_t)(sum >> 64), sum < a0 ? 1ull : 0ull};
        const uint64_t k2[2] = {(uint64_t)a1, (uint64_t)(a1 >> 64)};
        fph::g1_phi(phis[i], P);
        put_point(J[0], P);
        put_point(J[1], phis[i]);
        put_point(J[2], P);
        if (!put_digits(J[0], k1, 3, 33) || !put_digits(J[1], k2, 2, 33) || !put_digits(J[2], z2, 2, 33)) return 0;
        live[i] = 1;
    }
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const void *dj = up(c->mcl[8], (const u32 *)jobs.data(), jobs.size() * sizeof(PtJobG1) / 4, s);
    void *dout = c->mcl[9].get(3 * n * sizeof(fph::g1));
    if (!dj || !dout) { set_err("device allocation failed"); return -1; }
    lcbk_ptmul_g1_multi(s, dj, (u32)(3 * n), dout);
    std::vector<fph::g1> acc(3 * n);
    hipMemcpyAsync(acc.data(), dout, 3 * n * sizeof(fph::g1), hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "mulVec")) return -1;
    fph::g1 r;
    fph::jac_set_inf(r);
    for (size_t i = 0; i < n; i++) {
        if (!live[i]) continue;
        fph::g1a chk;
        fph::g1_phi(chk, phis[i]);                // (beta^2 x, y) -> membership: [z^2] P == (beta^2 x, -y)
        fph::neg(chk.y, chk.y);
        if (!fph::jac_eq_aff(acc[3 * i + 2], chk)) return 0;
        fph::g1 t;
        fph::jac_add(t, acc[3 * i], acc[3 * i + 1]);
        fph::jac_add(r, r, t);
    }
    *G1W(z) = r;
    return 1;
}
// the G2 counterpart: sum_i [k_i] x_i on mclBnG2_mul's GLS ladders (five groups per term, k_ptmul_g2_multi); the
// same return convention (0: a term off the curve or outside G2 — the caller's exact path)
static int g2_terms_coop(lcb_ctx *c, mclBnG2 *z, const mclBnG2 *x, const uint64_t (*kraw)[4], size_t n) {
    std::vector<PtJobG2> jobs(5 * n);
    memset(jobs.data(), 0, jobs.size() * sizeof(PtJobG2));
    std::vector<fph::g2a> psis(n);
    std::vector<uint8_t> live(n, 0);
    const uint64_t zero[1] = {0};
    for (size_t i = 0; i < n; i++) {
        PtJobG2 *J = &jobs[5 * i];
        const uint64_t *k = kraw[i];
        fph::g2a Q;
        fph::jac_to_aff(Q, *G2R(&x[i]));
        if (!Q.inf && !fph::jac_on_curve(*G2R(&x[i]))) return 0;
        if (Q.inf || (k[0] | k[1] | k[2] | k[3]) == 0) {
            for (int j = 0; j < 5; j++) { J[j].inf = 1; put_digits(J[j], zero, 1, 17); }
            continue;
        }
        uint64_t q[4] = {k[0], k[1], k[2], k[3]}, d[4];
        d[0] = divmod_u(q);
        d[1] = divmod_u(q);
        d[2] = divmod_u(q);
        d[3] = q[0];
        fph::g2a B[4];
        B[0] = Q;
        fph::g2_psi(B[1], Q);
        fph::g2_psi(B[2], B[1]);
        fph::g2_psi(B[3], B[2]);
        psis[i] = B[1];
        fph::neg(B[1].y, B[1].y);
        fph::neg(B[3].y, B[3].y);
        bool ok = true;
        for (int j = 0; j < 4; j++) {
            put_point(J[j], B[j]);
            ok &= put_digits(J[j], &d[j], 1, 17);
        }
        put_point(J[4], Q);
        ok &= put_digits(J[4], &Z_ABS_H, 1, 17);
        if (!ok) return 0;
        live[i] = 1;
    }
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const void *dj = up(c->mcl[8], (const u32 *)jobs.data(), jobs.size() * sizeof(PtJobG2) / 4, s);
    void *dout = c->mcl[9].get(5 * n * sizeof(fph::g2));
    if (!dj || !dout) { set_err("device allocation failed"); return -1; }
    lcbk_ptmul_g2_multi(s, dj, (u32)(5 * n), dout);
    std::vector<fph::g2> acc(5 * n);
    hipMemcpyAsync(acc.data(), dout, 5 * n * sizeof(fph::g2), hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "G2 terms")) return -1;
    fph::g2 r;
    fph::jac_set_inf(r);
    for (size_t i = 0; i < n; i++) {
        if (!live[i]) continue;
        fph::g2a chk = psis[i];                   // membership: psi(Q) == -[|z|] Q
        fph::neg(chk.y, chk.y);
        if (!fph::jac_eq_aff(acc[5 * i + 4], chk)) return 0;
        for (int j = 0; j < 4; j++) fph::jac_add(r, r, acc[5 * i + j]);
    }
    *G2W(z) = r;
    return 1;
}
// Lagrange coefficients lambda_i = prod_{j != i} x_j / (x_j - x_i) as canonical raw words; false on a zero or
// repeated x (the error of k_lagrange_coeffs)
static bool lagrange_lambdas(std::vector<uint64_t> &raw, const mclBnFr *xVec, size_t k) {
    raw.assign(4 * k, 0);
    static const uint64_t one_raw[4] = {1, 0, 0, 0};
    for (size_t i = 0; i < k; i++) {
        const uint64_t *xi = FRV(&xVec[i]);
        if (frh::is_zero(xi)) { set_err("lagrange: zero x"); return false; }
        uint64_t num[4], den[4], t[4];
        frh::from_raw(num, one_raw);
        memcpy(den, num, 32);
        for (size_t j = 0; j < k; j++) {
            if (j == i) continue;
            const uint64_t *xj = FRV(&xVec[j]);
            frh::sub(t, xj, xi);
            if (frh::is_zero(t)) { set_err("lagrange: repeated x"); return false; }
            frh::mul(num, num, xj);
            frh::mul(den, den, t);
        }
        frh::inv(den, den);
        frh::mul(t, num, den);
        frh::to_raw(&raw[4 * i], t);
    }
    return true;
}
// mclBnG1_mulVec: sum_i [y_i] x_i with the canonical scalars (mcl's per-term product, exact for any on-curve x_i):
// up to MULVEC_COOP_MAX terms on the cooperative ladders above; otherwise (or for a term outside G1) one lane per term
// (windowed ladder), then block reductions and a one-lane sum
static bool g1_mulvec(mclBnG1 *z, const mclBnG1 *x, const mclBnFr *y, mclSize n) {
    SYNC_CTX_OR(c, false)
    if (n > 0xffffffffu) { set_err("mulVec: too large"); return false; }
    std::vector<uint64_t> raw(4 * n);
    for (size_t i = 0; i < n; i++) frh::to_raw(&raw[4 * i], FRV(&y[i]));
    if (n <= MULVEC_COOP_MAX && g_mulvec_coop) {
        const int rc = g1_mulvec_coop(c, z, x, (const uint64_t (*)[4])raw.data(), n);
        if (rc != 0) return rc > 0;
    }
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const u32 *pts = up(c->mcl[0], (const u32 *)x, 36 * n, s);
    const uint64_t *sc = up(c->mcl[1], raw.data(), 4 * n, s);
    uint8_t *terms = (uint8_t *)c->mcl[2].get(LCB_G1_JAC_BYTES * n);
    uint8_t *tmp = (uint8_t *)c->mcl[3].get(LCB_G1_JAC_BYTES * ((n + 255) / 256));
    uint8_t *dz = (uint8_t *)c->mcl[5].get(LCB_G1_JAC_BYTES);
    u32 *ws = (u32 *)c->lws.get(lcbk_mcl_terms_ws_bytes((u32)n));
    if (!pts || !sc || !terms || !tmp || !dz || !ws) { set_err("device allocation failed"); return false; }
    lcbk_mcl_g1_terms(s, pts, sc, (u32)n, terms, ws);
    uint8_t *cur = terms;
    size_t cnt = n;
    while (cnt > 256) {
        uint8_t *dst = cur == terms ? tmp : terms;
        lcbk_g1_jac_reduce_block(s, cur, (u32)cnt, 256, dst);
        cnt = (cnt + 255) / 256;
        cur = dst;
    }
    lcbk_mcl_g1_sum(s, cur, (u32)cnt, dz);
    mclBnG1 r;
    hipMemcpyAsync(&r, dz, 144, hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "mulVec")) return false;
    *z = r;
    return true;
}
extern "C" void mclBnG1_mulVec(mclBnG1 *z, const mclBnG1 *x, const mclBnFr *y, mclSize n) {
    if (n == 0) { mclBnG1_clear(z); return; }
    if (!g1_mulvec(z, x, y, n)) fail_out(z, 144);
}
// G1 / G2 Lagrange interpolation of one problem on the batch kernels: mcl records -> wire bytes on the device, the
// k_lagrange.hip coefficient + product kernels, the result decoded back into an mcl record (one round trip)
static int lagrange_points(int g, void *out, const mclBnFr *xVec, const void *yVec, mclSize k) {
    if (k == 0) return -1;
    SYNC_CTX_OR(c, -1)
    if (k > 0xffffffffu) { set_err("lagrange: too large"); return -1; }
    const size_t pb = g == 1 ? 48 : 96, words = g == 1 ? 36 : 72;
    std::vector<uint64_t> xs(4 * k);
    for (size_t i = 0; i < k; i++) frh::to_raw(&xs[4 * i], FRV(&xVec[i]));
    const uint32_t off[2] = {0, (uint32_t)k};
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const uint8_t *dx = (const uint8_t *)up(c->mcl[0], xs.data(), 4 * k, s);
    const u32 *dyr = up(c->mcl[1], (const u32 *)yVec, words * k, s);
    const uint32_t *doff = up(c->mcl[2], off, 2, s);
    uint8_t *dy = (uint8_t *)c->mcl[3].get(pb * k);
    uint8_t *dst = (uint8_t *)c->mcl[4].get(16), *dout = (uint8_t *)c->mcl[5].get(pb);
    u32 *rec = (u32 *)c->mcl[6].get(words * 4);
    uint8_t *dok = (uint8_t *)c->mcl[7].get(16);
    if (!dx || !dyr || !doff || !dy || !dst || !dout || !rec || !dok) { set_err("device allocation failed"); return -1; }
    lcbk_mcl_to_bytes(s, g, dyr, (u32)k, dy);
    if (lagrange_enqueue(c, g, dout, dst, dx, dy, doff, 1, k, s)) return -1;
    lcbk_mcl_from_bytes(s, g, dout, 1, rec, dok);
    u32 r[72];
    uint8_t st = 0, ok = 0;
    hipMemcpyAsync(r, rec, words * 4, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(&st, dst, 1, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(&ok, dok, 1, hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "lagrange") || !st || !ok) return -1;
    memcpy(out, r, words * 4);
    return 0;
}
// G1 Lagrange interpolation of up to 64 points: the coefficients lambda_i = prod_{j != i} x_j / (x_j - x_i) on the host
// (-1 on a zero or repeated x, as k_lagrange_coeffs), the products on the cooperative ladders (g1_mulvec_coop); 1 done,
// 0 for the batch kernels' path (a point outside G1, or more points)
static int g1_lagrange_coop(mclBnG1 *out, const mclBnFr *xVec, const mclBnG1 *yVec, size_t k) {
    if (k > 64 || !g_mulvec_coop) return 0;
    SYNC_CTX_OR(c, -1)
    std::vector<uint64_t> raw;
    if (!lagrange_lambdas(raw, xVec, k)) return -1;
    const int rc = g1_mulvec_coop(c, out, yVec, (const uint64_t (*)[4])raw.data(), k);
    return rc < 0 ? -1 : rc;
}
// the same in G2 (AssembleSignature's interpolation, ThresholdSignature/PublicKeySet.cs:34-42)
static int g2_lagrange_coop(mclBnG2 *out, const mclBnFr *xVec, const mclBnG2 *yVec, size_t k) {
    if (k > 64 || !g_mulvec_coop) return 0;
    SYNC_CTX_OR(c, -1)
    std::vector<uint64_t> raw;
    if (!lagrange_lambdas(raw, xVec, k)) return -1;
    const int rc = g2_terms_coop(c, out, yVec, (const uint64_t (*)[4])raw.data(), k);
    return rc < 0 ? -1 : rc;
}
extern "C" int mclBn_G1LagrangeInterpolation(mclBnG1 *out, const mclBnFr *xVec, const mclBnG1 *yVec, mclSize k) {
    if (k == 1) { *out = yVec[0]; return mclBnFr_isZero(&xVec[0]) ? -1 : 0; }
    if (k == 0) return -1;
    const int rc = g1_lagrange_coop(out, xVec, yVec, k);
    if (rc != 0) return rc > 0 ? 0 : -1;
    return lagrange_points(1, out, xVec, yVec, k);
}
extern "C" int mclBn_G2LagrangeInterpolation(mclBnG2 *out, const mclBnFr *xVec, const mclBnG2 *yVec, mclSize k) {
    if (k == 1) { *out = yVec[0]; return mclBnFr_isZero(&xVec[0]) ? -1 : 0; }
    if (k == 0) return -1;
    const int rc = g2_lagrange_coop(out, xVec, yVec, k);
    if (rc != 0) return rc > 0 ? 0 : -1;
    return lagrange_points(2, out, xVec, yVec, k);
}
// out = a x mod #E(Fp) for G1 (a < #E, x < 2^256): #E(Fp) = p - z = h r (z = -0xd201000000010000), so [k] P depends
// only on k mod #E for every point P of E(Fp), in the subgroup or not
static void ne_mulmod(uint64_t out[6], const uint64_t a[6], const uint64_t x[4]) {
    static const uint64_t NE[6] = {0x8c0000000000aaabull, 0x1eabfffeb1540000ull, 0x6730d2a0f6b0f624ull,
                                   0x64774b84f38512bfull, 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};
    typedef unsigned __int128 u128;
    uint64_t prod[10] = {0};
    for (int i = 0; i < 6; i++) {
        uint64_t carry = 0;
        for (int j = 0; j < 4; j++) {
            const u128 t = (u128)a[i] * x[j] + prod[i + j] + carry;
            prod[i + j] = (uint64_t)t;
            carry = (uint64_t)(t >> 64);
        }
        prod[i + 4] = carry;
    }
    uint64_t rem[6] = {0};                       // long division by bits: rem < NE < 2^381, so 2 rem + 1 fits
    for (int b = 639; b >= 0; b--) {
        for (int k = 5; k > 0; k--) rem[k] = (rem[k] << 1) | (rem[k - 1] >> 63);
        rem[0] = (rem[0] << 1) | ((prod[b >> 6] >> (b & 63)) & 1);
        int ge = 1;
        for (int k = 5; k >= 0; k--) {
            if (rem[k] != NE[k]) { ge = rem[k] > NE[k]; break; }
        }
        if (ge) {
            uint64_t br = 0;
            for (int k = 0; k < 6; k++) {
                const u128 t = (u128)rem[k] - NE[k] - br;
                rem[k] = (uint64_t)t;
                br = (uint64_t)(t >> 64) & 1;
            }
        }
    }
    memcpy(out, rem, 48);
}
// G1 EvaluatePolynomial as a sum of independent terms: sum_i [x^i mod #E] c_i (k_mcl_g1_terms_wide, one lane per term,
// then the mulVec sums) — the value of mcl's Horner rule for every on-curve coefficient, with the products side by
// side instead of n - 1 dependent ones
static int eval_poly_g1_terms(lcb_ctx *c, mclBnG1 *out, const mclBnG1 *coef, size_t n, const uint64_t xr[4]) {
    std::vector<uint32_t> sc(12 * n);
    uint64_t e[6] = {1, 0, 0, 0, 0, 0};
    for (size_t i = 0; i < n; i++) {
        if (i) ne_mulmod(e, e, xr);
        memcpy(&sc[12 * i], e, 48);
    }
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const u32 *pts = up(c->mcl[0], (const u32 *)coef, 36 * n, s);
    const u32 *dsc = up(c->mcl[1], sc.data(), 12 * n, s);
    uint8_t *terms = (uint8_t *)c->mcl[2].get(LCB_G1_JAC_BYTES * n);
    uint8_t *tmp = (uint8_t *)c->mcl[3].get(LCB_G1_JAC_BYTES * ((n + 255) / 256));
    uint8_t *dz = (uint8_t *)c->mcl[5].get(LCB_G1_JAC_BYTES);
    u32 *ws = (u32 *)c->lws.get(lcbk_mcl_terms_wide_ws_bytes((u32)n));
    if (!pts || !dsc || !terms || !tmp || !dz || !ws) { set_err("device allocation failed"); return -1; }
    lcbk_mcl_g1_terms_wide(s, pts, dsc, (u32)n, terms, ws);
    uint8_t *cur = terms;
    size_t cnt = n;
    while (cnt > 256) {
        uint8_t *dst = cur == terms ? tmp : terms;
        lcbk_g1_jac_reduce_block(s, cur, (u32)cnt, 256, dst);
        cnt = (cnt + 255) / 256;
        cur = dst;
    }
    lcbk_mcl_g1_sum(s, cur, (u32)cnt, dz);
    mclBnG1 r;
    hipMemcpyAsync(&r, dz, 144, hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "evaluate polynomial")) return -1;
    *out = r;
    return 0;
}
// G1 / G2 EvaluatePolynomial: mcl's Horner rule (y = c[n-1]; y = y x + c[i]) — the products are by the integer x, as
// mcl's, so off-subgroup coefficients give mcl's value too.  G1 (n >= 2): the same value as independent terms (above);
// G2 and LCB_EVAL_HORNER=1: the Horner chain in one kernel launch
static int eval_poly(int g, void *out, const void *coef, mclSize n, const mclBnFr *x) {
    if (n == 0) return -1;
    SYNC_CTX_OR(c, -1)
    if (n > 0xffffffffu) { set_err("evaluate polynomial: too large"); return -1; }
    const size_t words = g == 1 ? 36 : 72;
    uint64_t xr[4];
    frh::to_raw(xr, FRV(x));
    static const bool horner = getenv("LCB_EVAL_HORNER") && atoi(getenv("LCB_EVAL_HORNER")) == 1;
    if (g == 1 && n >= 2 && n <= MULVEC_COOP_MAX && !horner && g_mulvec_coop) {
        // coefficients in G1: [x^i mod r] c_i on the cooperative ladders (a coefficient outside G1 returns 0 here
        // and takes the terms below, whose powers are reduced mod #E(Fp) instead)
        std::vector<uint64_t> raw(4 * n);
        uint64_t pw[4], one_raw[4] = {1, 0, 0, 0};
        frh::from_raw(pw, one_raw);
        for (size_t i = 0; i < n; i++) {
            frh::to_raw(&raw[4 * i], pw);
            frh::mul(pw, pw, FRV(x));
        }
        const int rc = g1_mulvec_coop(c, (mclBnG1 *)out, (const mclBnG1 *)coef, (const uint64_t (*)[4])raw.data(), n);
        if (rc != 0) return rc > 0 ? 0 : -1;
    }
    if (g == 1 && n >= 2 && !horner) return eval_poly_g1_terms(c, (mclBnG1 *)out, (const mclBnG1 *)coef, n, xr);
    if (g == 2 && n >= 2 && n <= 64 && !horner && g_mulvec_coop) {   // coefficients in G2: [x^i mod r] c_i, GLS
        std::vector<uint64_t> raw(4 * n);
        uint64_t pw[4], one_raw[4] = {1, 0, 0, 0};
        frh::from_raw(pw, one_raw);
        for (size_t i = 0; i < n; i++) {
            frh::to_raw(&raw[4 * i], pw);
            frh::mul(pw, pw, FRV(x));
        }
        const int rc = g2_terms_coop(c, (mclBnG2 *)out, (const mclBnG2 *)coef, (const uint64_t (*)[4])raw.data(), n);
        if (rc != 0) return rc > 0 ? 0 : -1;
    }
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const u32 *dc = up(c->mcl[0], (const u32 *)coef, words * n, s);
    const uint64_t *dx = up(c->mcl[1], xr, 4, s);
    u32 *dout = (u32 *)c->mcl[2].get(words * 4);
    if (!dc || !dx || !dout) { set_err("device allocation failed"); return -1; }
    lcbk_mcl_horner(s, g, dc, (u32)n, dx, dout);
    u32 r[72];
    hipMemcpyAsync(r, dout, words * 4, hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "evaluate polynomial")) return -1;
    memcpy(out, r, words * 4);
    return 0;
}
extern "C" int mclBn_G1EvaluatePolynomial(mclBnG1 *out, const mclBnG1 *c, mclSize n, const mclBnFr *x) {
    return eval_poly(1, out, c, n, x);
}
extern "C" int mclBn_G2EvaluatePolynomial(mclBnG2 *out, const mclBnG2 *c, mclSize n, const mclBnFr *x) {
    return eval_poly(2, out, c, n, x);
}

static int mul_batch(int g, uint8_t *out, const uint8_t *points, int use_gen, const uint8_t *scalars, size_t n) {
    SYNC_CTX_OR(c, -1)
    if (!n) return 0;
    if (n > 0xffffffffu) { set_err("mul batch: too large"); return -1; }
    Enq q(c, c->stream);
    size_t pb = g == 1 ? 48 : 96;
    hipStream_t s = c->stream;
    const uint8_t *dp = use_gen ? (const uint8_t *)c->in[0].get(16) : up(c->in[0], points, pb * n, s);
    const uint8_t *dsc = up(c->in[1], scalars, 32 * n, s);
    uint8_t *dout = (uint8_t *)c->out[0].get(pb * n), *dok = (uint8_t *)c->out[1].get(n);
    u32 *ws = (u32 *)c->lws.get(lcbk_scalar_ws_bytes(g, (u32)n));
    if (!dp || !dsc || !dout || !dok || !ws) { set_err("device allocation failed"); return -1; }
    if (g == 1) lcbk_g1_mul(s, dp, use_gen, dsc, (u32)n, dout, dok, ws);
    else lcbk_g2_mul(s, dp, use_gen, dsc, (u32)n, dout, dok, ws);
    std::vector<uint8_t> ok(n);
    hipMemcpyAsync(out, dout, pb * n, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(ok.data(), dok, n, hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "mul batch")) return -1;
    for (size_t i = 0; i < n; i++) if (!ok[i]) { set_err("invalid point or scalar"); return -1; }
    return 0;
}
extern "C" int lcb_g1_mul_batch(uint8_t *out, const uint8_t *points, int gen, const uint8_t *scalars, size_t n) {
    return mul_batch(1, out, points, gen, scalars, n);
}
extern "C" int lcb_g2_mul_batch(uint8_t *out, const uint8_t *points, int gen, const uint8_t *scalars, size_t n) {
    return mul_batch(2, out, points, gen, scalars, n);
}
extern "C" int lcb_g2_hash_batch(uint8_t *out, const uint8_t *msg_data, const uint32_t *msg_off, size_t n) {
    SYNC_CTX_OR(c, -1)
    if (!n) return 0;
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const uint8_t *dm = up(c->in[0], msg_data, msg_off[n], s);
    const uint32_t *dmo = up(c->in[1], msg_off, n + 1, s);
    uint8_t *dout = (uint8_t *)c->out[0].get(96 * n), *dok = (uint8_t *)c->out[1].get(n);
    if (!dm || !dmo || !dout || !dok) { set_err("device allocation failed"); return -1; }
    lcbk_g2_hash(dim3(nblk(n)), s, dm, dmo, (u32)n, dout, dok, g_orig_cofactor);
    std::vector<uint8_t> ok(n);
    hipMemcpyAsync(out, dout, 96 * n, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(ok.data(), dok, n, hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "hash batch")) return -1;
    for (size_t i = 0; i < n; i++) if (!ok[i]) { set_err("hash-to-G2 failed"); return -1; }
    return 0;
}

extern "C" int lcb_g1_msm_window(size_t n) { return (int)msm_window(n); }
extern "C" int lcb_g1_msm_glv_window(size_t n) { return msm_use_glv(n) ? (int)msm_window(n, true) : -(int)msm_window(n); }
// GLV form: every point must have order r (generated as a G or checked); see include/lachain_bls.h
extern "C" int lcb_ctx_g1_msm_glv_dev(lcb_ctx *ctx, void *out_jac, const void *points_aff, const uint8_t *scalars,
                                      size_t n, int window_bits, void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    bool glv = window_bits > 0 || msm_use_glv(n);   // an explicit width selects the GLV form
    return msm_enqueue(c, out_jac, points_aff, scalars, n, window_bits, q.s, glv);
}
extern "C" int lcb_g1_msm_glv_dev(void *out_jac, const void *points_aff, const uint8_t *scalars, size_t n,
                                  int window_bits, void *stream) {
    return lcb_ctx_g1_msm_glv_dev(nullptr, out_jac, points_aff, scalars, n, window_bits, stream);
}
extern "C" int lcb_ctx_g1_msm_dev(lcb_ctx *ctx, void *out_jac, const void *points_aff, const uint8_t *scalars, size_t n,
                                  int window_bits, void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    return msm_enqueue(c, out_jac, points_aff, scalars, n, window_bits, q.s);
}
extern "C" int lcb_g1_msm_dev(void *out_jac, const void *points_aff, const uint8_t *scalars, size_t n, int window_bits,
                              void *stream) {
    return lcb_ctx_g1_msm_dev(nullptr, out_jac, points_aff, scalars, n, window_bits, stream);
}
extern "C" int lcb_ctx_g1_msm_phase_ms(lcb_ctx *ctx, float *ms, int n_phases) {
    CTX_OR(c, ctx, -1)
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    if (!c->msm_ran) { set_err("msm: no MSM has run in this context"); return -1; }
    if (hipEventSynchronize(c->msm_ev[6]) != hipSuccess) { set_err("msm: event sync"); return -1; }
    for (int i = 0; i < n_phases && i < 6; i++)
        if (hipEventElapsedTime(&ms[i], c->msm_ev[i], c->msm_ev[i + 1]) != hipSuccess) ms[i] = -1.0f;
    return 0;
}
extern "C" int lcb_g1_msm_phase_ms(float *ms, int n_phases) { return lcb_ctx_g1_msm_phase_ms(nullptr, ms, n_phases); }
extern "C" int lcb_g1_to_affine_dev(void *out_aff, uint8_t *ok, const uint8_t *points, size_t n, void *stream) {
    if (!ready()) return -1;
    if (n > 0xffffffffu) { set_err("to_affine: batch too large"); return -1; }
    if (n) lcbk_g1_to_affine(dim3(nblk(n)), (hipStream_t)stream, points, (u32)n, out_aff, ok);
    return launched("to_affine launch") ? 0 : -1;
}
extern "C" int lcb_ctx_g1_jac_sum_dev(lcb_ctx *ctx, uint8_t *out48, void *out_jac, const void *parts, size_t k,
                                      void *stream) {
    CTX_OR(c, ctx, -1)
    Enq q(c, (hipStream_t)stream);
    if (k == 1 && !out_jac && out48) {          // one partial (a single rank): serialise it as it is
        lcbk_g1_jac_compress(dim3(1), q.s, parts, 1, out48);
        return launched("jac sum launch") ? 0 : -1;
    }
    void *acc = out_jac ? out_jac : c->msm[14].get(LCB_G1_JAC_BYTES);
    if (!acc) { set_err("device allocation failed"); return -1; }
    lcbk_g1_jac_reduce_groups(dim3(1), q.s, parts, (u32)k, k ? (u32)k : 1u, acc);
    if (out48) lcbk_g1_jac_compress(dim3(1), q.s, acc, 1, out48);
    return launched("jac sum launch") ? 0 : -1;
}
extern "C" int lcb_g1_jac_sum_dev(uint8_t *out48, void *out_jac, const void *parts, size_t k, void *stream) {
    return lcb_ctx_g1_jac_sum_dev(nullptr, out48, out_jac, parts, k, stream);
}
extern "C" int lcb_g1_msm(uint8_t out[48], const uint8_t *points, const uint8_t *scalars, size_t n) {
    SYNC_CTX_OR(c, -1)
    if (n == 0) { memset(out, 0, 48); return 0; }
    for (size_t i = 0; i < n; i++) {   // mclBnFr values are canonical (< r); reject what mcl would not hold
        const uint8_t *sc = scalars + 32 * i;
        if (!fr_bytes_lt_r(sc)) { set_err("invalid point or scalar"); return -1; }
    }
    Enq q(c, c->stream);
    hipStream_t s = c->stream;
    const uint8_t *dp = up(c->in[0], points, 48 * n, s);
    const uint8_t *dsc = up(c->in[1], scalars, 32 * n, s);
    void *aff = c->in[2].get(96 * n);
    uint8_t *dok = (uint8_t *)c->out[0].get(n), *dout = (uint8_t *)c->out[1].get(48);
    void *jac = c->out[2].get(LCB_G1_JAC_BYTES);
    if (!dp || !dsc || !aff || !dok || !dout || !jac) { set_err("device allocation failed"); return -1; }
    lcbk_g1_to_affine(dim3(nblk(n)), s, dp, (u32)n, aff, dok);
    if (msm_enqueue(c, jac, aff, dsc, n, 0, s)) return -1;
    lcbk_g1_jac_compress(dim3(1), s, jac, 1, dout);
    std::vector<uint8_t> ok(n);
    hipMemcpyAsync(out, dout, 48, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(ok.data(), dok, n, hipMemcpyDeviceToHost, s);
    if (!sync_check(c, "msm")) return -1;
    for (size_t i = 0; i < n; i++) if (!ok[i]) { set_err("invalid point or scalar"); return -1; }
    return 0;
}

// ================================================================== KDF (host byte work)
extern "C" void lcb_xor_with_hash(uint8_t *out, const uint8_t g1b[48], const uint8_t *data, size_t len) {
    lcb_host::xor_with_hash(out, g1b, data, len);
}

// ================================================================== internal interface for the other host files
namespace lcb_int {
void set_error(const char *what, hipError_t e) { set_err(what, e); }
lcb_ctx *ctx_resolve(lcb_ctx *c) { return resolve(c); }
lcb_ctx *ctx_sync() { return sync_ctx(); }
bool launch_ok(const char *what) { return launched(what); }
bool sync_ok(lcb_ctx *c, const char *what) { return sync_check(c, what); }
int device() { return g_device; }
}  // namespace lcb_int
