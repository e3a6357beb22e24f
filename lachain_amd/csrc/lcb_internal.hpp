// lachain_amd/csrc/lcb_internal.hpp — the few host internals lcb_host.cpp shares with the other host files
// (error slot, context resolution, launch / synchronisation checks).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include "lcb_ctx.hpp"

namespace lcb_int {
void set_error(const char *what, hipError_t e = hipSuccess);
lcb_ctx *ctx_resolve(lcb_ctx *c);     // explicit context, or the calling thread's default *_dev context
lcb_ctx *ctx_sync();                  // the calling thread's context for host-pointer entry points
bool launch_ok(const char *what);     // hipGetLastError after launches
bool sync_ok(lcb_ctx *c, const char *what);
int device();
void ecdsa_ctx_release(lcb_ctx *c);   // lcb_ecdsa.cpp: the context's cached key set
}  // namespace lcb_int
