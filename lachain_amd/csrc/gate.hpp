// lachain_amd/csrc/gate.hpp — the scratch gate's launch macro, shared by every kernel translation unit.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

// The scratch gate (lcb_host.cpp lcb_gate_enter, round 5): the HIP runtime reserves a dispatch's scratch on its
// hardware queue for min(waves, device wave slots) waves, so a large-grid launch of a kernel with kilobytes of private
// segment per lane reserves gigabytes on that queue.  Launches whose reservation would reach the gate's threshold run on
// one process-wide stream per device (ordered with the caller's stream by events), so at most one queue per process holds
// such a reservation and concurrent callers cannot exhaust the scratch resources (which the runtime reports by aborting
// the process).  The kernel's private segment size is read once per launch site (hipFuncGetAttributes).
extern "C" hipStream_t lcb_gate_enter(const void *kern, long long *scratch_cache, size_t lanes, hipStream_t s);
extern "C" void lcb_gate_exit(hipStream_t s, hipStream_t used);
#define LCB_LAUNCH_GATED(name, grd, blk, shm, strm, ...)                                                            \
    do {                                                                                                          \
        static long long lcb_sc_ = -1;                                                                            \
        const dim3 lcb_g_ = (grd), lcb_b_ = (blk);                                                                \
        hipStream_t lcb_s_ = lcb_gate_enter((const void *)name, &lcb_sc_,                                         \
                                            (size_t)lcb_g_.x * lcb_g_.y * lcb_g_.z * lcb_b_.x * lcb_b_.y * lcb_b_.z, \
                                            (strm));                                                              \
        hipLaunchKernelGGL(name, lcb_g_, lcb_b_, (shm), lcb_s_, __VA_ARGS__);                                     \
        lcb_gate_exit((strm), lcb_s_);                                                                            \
    } while (0)
