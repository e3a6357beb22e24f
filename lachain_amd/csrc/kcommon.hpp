// lachain_amd/csrc/kcommon.hpp — shared definitions of the kernel translation units.
#pragma once
#include "h2g2.hpp"
#include "pairing.hpp"
#include "ops.h"

#define LCB_BLOCK 256
#define LCB_BOUNDS __launch_bounds__(LCB_BLOCK, 1)
// the one-lane pairing kernels run one wave per SIMD (512 registers per lane; two waves measured slower: more spills)
#define LCB_PAIR_BOUNDS __launch_bounds__(LCB_BLOCK, 1)

// affine point records in device memory
struct g1a_st { fp x, y; u32 inf, ok, pad[2]; };   // 112 B
struct g2a_st { fp2 x, y; u32 inf, ok, pad[2]; };  // 208 B
// a signature share as the batched CommonCoin check decoded it (k_ts_rlc_points): its 96 wire bytes, the affine point,
// ok = 1 for a written record and pad[0] = 1 when the point is in G2; the assembly's Lagrange lanes reuse a record
// whose bytes equal their input (k_g2_mul_lanes) instead of decompressing and testing the share again
struct ts_share_st { u32 raw[24]; g2a_st p; };        // 304 B
static_assert(sizeof(ts_share_st) == 304, "ts_share_st layout (launch.h LCB_TS_SHARE_REC_BYTES)");
DI void st_to_g1a(g1a &a, const g1a_st &s) { a.x = s.x; a.y = s.y; a.inf = s.inf != 0; }
DI void st_to_g2a(g2a &a, const g2a_st &s) { a.x = s.x; a.y = s.y; a.inf = s.inf != 0; }

// Fp12 values parked in HBM between the Miller-loop and final-exponentiation kernels: quad-major SoA (words
// 4g..4g+3 of item i at u32 index (g * n + i) * 4), so a wave's 64 lanes read / write 1 KB contiguous per
// 16-byte access and the assembly routines (asm_tower.hpp) move an Fp12 with 36 global_load/store_dwordx4.
// Addresses: a wave-uniform 64-bit base per quad (SGPRs, advanced by n * 16 bytes per quad) plus a 32-bit per-lane
// byte offset (i * 16) that is made opaque first, so the compiler cannot hoist 36 per-lane 64-bit addresses per slot
// out of the callers' loops (it did, and spilled them).  Valid for any n < 2^28 (the lane offset stays 32-bit).
DI void fp12_store_soa(u32 *base, size_t n, size_t i, const fp12 &f) {
    const u32 *s = (const u32 *)&f;
    u32 off = (u32)(i * 16);
    asm volatile("" : "+v"(off));
    char *b = (char *)base;
#pragma unroll
    for (int g = 0; g < 36; g++)
        *(uint4 *)(b + (size_t)g * n * 16 + off) = make_uint4(s[4 * g], s[4 * g + 1], s[4 * g + 2], s[4 * g + 3]);
}
DI void fp12_load_soa(fp12 &f, const u32 *base, size_t n, size_t i) {
    u32 *d = (u32 *)&f;
    u32 off = (u32)(i * 16);
    asm volatile("" : "+v"(off));
    const char *b = (const char *)base;
#pragma unroll
    for (int g = 0; g < 36; g++) {
        uint4 v = *(const uint4 *)(b + (size_t)g * n * 16 + off);
        d[4 * g] = v.x; d[4 * g + 1] = v.y; d[4 * g + 2] = v.z; d[4 * g + 3] = v.w;
    }
}
// the same load, never hoisted out of a loop
DI void fp12_load_soa_fresh(fp12 &f, const u32 *base, size_t n, size_t i) {
    asm volatile("" ::: "memory");
    fp12_load_soa(f, base, n, i);
}

// per-unit configuration setter (curve.hpp lcb_g2_sign_b): one per kernel translation unit, called by
// lcbk_set_g2_sign_b (lcb_host.cpp) for every unit
#define LCB_TU_CONFIG(tag)                                                                                        \
    extern "C" int lcbk_cfg_##tag(u32 sign_b) {                                                                 \
        return hipMemcpyToSymbol(HIP_SYMBOL(lcb_g2_sign_b), &sign_b, sizeof sign_b) == hipSuccess ? 0 : -1;     \
    }                                                                                                             \
    extern "C" int lcbk_prio_##tag(u32 on) {                                                                    \
        return hipMemcpyToSymbol(HIP_SYMBOL(lcb_wave_prio), &on, sizeof on) == hipSuccess ? 0 : -1;             \
    }
#include "gate.hpp"
#define LCB_LAUNCH(name, ...) LCB_LAUNCH_GATED(name, grid, dim3(LCB_BLOCK), 0, s, __VA_ARGS__)
// Persistent grids (the kernels with a lanetab.hpp workspace): as many blocks as are resident at once on the calling
// thread's device (occupancy x CUs, cached per kernel), at most one block per LCB_BLOCK work items; the workspace holds
// one slot per lane of that grid (LCB_WS_BYTES)
static inline u32 lcb_resident_blocks(const void *kern, u32 *cache) {
    u32 v = __atomic_load_n(cache, __ATOMIC_RELAXED);
    if (v) return v;
    int nb = 0, dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, LCB_BLOCK, 0) != hipSuccess || nb < 1 || cus < 1) {
        nb = 1;
        cus = 256;
    }
    v = (u32)nb * (u32)cus;
    __atomic_store_n(cache, v, __ATOMIC_RELAXED);
    return v;
}
extern "C" u32 lcb_persist_cap(void);      // lcb_set_persist_blocks (test hook): 0 = no cap
static inline u32 lcb_persist_blocks(const void *kern, u32 *cache, u32 items) {
    u32 r = lcb_resident_blocks(kern, cache);
    const u32 cap = lcb_persist_cap(), b = (u32)(((size_t)items + LCB_BLOCK - 1) / LCB_BLOCK);
    if (cap && cap < r) r = cap;
    return b < 1 ? 1 : b < r ? b : r;
}
#define LCB_WS_BYTES(blocks, quads) ((size_t)(blocks) * (LCB_BLOCK / 64) * (size_t)(quads) * 1024)
static_assert(sizeof(g1a_st) == 112 && sizeof(g2a_st) == 208, "record sizes");
static_assert(sizeof(g1) == 144 && sizeof(g2) == 288 && sizeof(fr) == 32, "struct sizes");
