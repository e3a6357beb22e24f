// lachain_amd/csrc/kcommon.hpp — shared definitions of the kernel translation units.
#pragma once
#include "h2g2.hpp"
#include "pairing.hpp"
#include "lean.hpp"
#include "ops.h"

#define LCB_BLOCK 256
#define LCB_BOUNDS __launch_bounds__(LCB_BLOCK, 1)
// the pairing kernels are issue-latency bound at one wave per SIMD; LCB_PAIR_WAVES=2 trades spills for a second
// wave per SIMD (256 registers per lane)
#ifndef LCB_PAIR_WAVES
#define LCB_PAIR_WAVES 1
#endif
#define LCB_PAIR_BOUNDS __launch_bounds__(LCB_BLOCK, LCB_PAIR_WAVES)

// affine point records in device memory
struct g1a_st { fp x, y; u32 inf, ok, pad[2]; };   // 112 B
struct g2a_st { fp2 x, y; u32 inf, ok, pad[2]; };  // 208 B
DI void st_to_g1a(g1a &a, const g1a_st &s) { a.x = s.x; a.y = s.y; a.inf = s.inf != 0; }
DI void st_to_g2a(g2a &a, const g2a_st &s) { a.x = s.x; a.y = s.y; a.inf = s.inf != 0; }

// Fp12 values parked in HBM between the Miller-loop and final-exponentiation kernels: word-major SoA
// (word w of item i at w * n + i) so a wave's 64 lanes touch 256 contiguous bytes per word.
DI void fp12_store_soa(u32 *base, size_t n, size_t i, const fp12 &f) {
    const u32 *s = (const u32 *)&f;
#pragma unroll
    for (int w = 0; w < 144; w++) base[(size_t)w * n + i] = s[w];
}
DI void fp12_load_soa(fp12 &f, const u32 *base, size_t n, size_t i) {
    u32 *d = (u32 *)&f;
#pragma unroll
    for (int w = 0; w < 144; w++) d[w] = base[(size_t)w * n + i];
}

#define LCB_LAUNCH(name, ...) hipLaunchKernelGGL(name, grid, dim3(LCB_BLOCK), 0, s, __VA_ARGS__)
static_assert(sizeof(g1a_st) == 112 && sizeof(g2a_st) == 208, "record sizes");
static_assert(sizeof(g1) == 144 && sizeof(g2) == 288 && sizeof(fr) == 32, "struct sizes");
