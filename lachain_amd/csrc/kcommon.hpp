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

// Final exponentiation with its five exponentiations by z run by ONE inline loop in the calling kernel.  In the
// noinline form (pairing.hpp: fe_hard -> cyc_pow_z) the loop lives in a called function, which gets at most 256
// VGPRs and no AGPR spill space, so its accumulator + base (288 registers) spill to scratch on every iteration
// (most of the kernel's 683 KB/share of HBM traffic).  Here the loop runs in the kernel (AGPRs available), and the
// exponentiation base, needed at only 5 of 63 steps, is parked in its own SoA slot (park slot 1) and re-read there.
// The stage structure is fe_hard's (same exponent and products, pairing.hpp).
DI void final_exp_staged(fp12 &f, u32 *park, size_t n, size_t i) {
    u32 *base_slot = park + (size_t)144 * n;
    fe_easy(f, f);
    fp12 x = f, t, u, v, acc, w;
    for (int st = 0; st < 5; st++) {
        fp12 a;
        if (st == 0) a = x;
        else if (st == 1) a = u;
        else a = v;
        fp12_store_soa(base_slot, n, i, a);
        for (int b = 62; b >= 0; b--) {
            fp12_cyc_sqr(a, a);
            if ((LCB_Z_ABS >> b) & 1) {
                fp12 bs;
                fp12_load_soa_fresh(bs, base_slot, n, i);
                fp12_mul(a, a, bs);
            }
        }
        fp12_conj(a, a);                                  // x^z (z < 0, x unitary)
        if (st == 0) {                                    // t = x^z, u = x^(z-2)
            t = a;
            fp12_conj(u, x);
            fp12_cyc_sqr_n(u, u);
            fp12_mul_n(u, u, t);
        } else if (st == 1) {                             // v = x^(z^2-2z); acc = (v x)^(p^3)
            v = a;
            fp12_mul_n(acc, v, x);
            fp12_frob3_n(acc, acc);
        } else if (st == 2) {                             // v = x^(z^3-2z^2); acc *= (v t)^(p^2)
            v = a;
            fp12_mul_n(w, v, t);
            fp12_frob2_n(w, w);
            fp12_mul_n(acc, acc, w);
        } else if (st == 3) {                             // v = x^(z^4-2z^3+2z); acc *= (x^-1 v)^p
            v = a;
            fp12_cyc_sqr_n(t, t);
            fp12_mul_n(v, v, t);
            fp12_conj(w, x);
            fp12_mul_n(w, w, v);
            fp12_frob1_n(w, w);
            fp12_mul_n(acc, acc, w);
        } else {                                          // v = x^(z^5-2z^4+2z^2); y = acc x^(2-z) v x
            v = a;
            fp12_conj(u, u);
            fp12_mul_n(u, u, v);
            fp12_mul_n(u, u, x);
            fp12_mul_n(f, acc, u);
        }
    }
}

#define LCB_LAUNCH(name, ...) hipLaunchKernelGGL(name, grid, dim3(LCB_BLOCK), 0, s, __VA_ARGS__)
static_assert(sizeof(g1a_st) == 112 && sizeof(g2a_st) == 208, "record sizes");
static_assert(sizeof(g1) == 144 && sizeof(g2) == 288 && sizeof(fr) == 32, "struct sizes");
