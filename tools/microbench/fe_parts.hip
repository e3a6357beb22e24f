// tools/microbench/fe_parts.hip — times the parts of the final exponentiation on gfx950, one share per lane,
// 1 wave per SIMD (LCB_PAIR_BOUNDS), so the kernels that matter can be tuned separately:
//   sqr_asm    63 Granger-Scott squarings through lcb_asm_cyc_sqr_n (AGPR accumulator, asm_tower.hpp)
//   sqr_c      63 compiler-built squarings (fp12_cyc_sqr inline, Fp2 leaf routines)
//   mul_slot   5 slot products (fe_asm.hpp fx_mul, compiler-built fp12_mul)
//   easy       the easy part (fx_easy)
//   fe_asm     the whole final exponentiation, fe_asm.hpp
//   fe_funcs   the whole final exponentiation, round-2 form (pairing.hpp final_exp_inplace)
// Output: JSON lines {"part": ..., "ms": ..., "us_per_op_per_lane_batch": ...}.  Inputs are arbitrary values
// < 2^352 (timing only: the arithmetic is data-independent).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I lachain_amd/csrc -o tools/microbench/fe_parts tools/microbench/fe_parts.hip
#include "fe_asm.hpp"
#include <stdio.h>

LCB_ASM_LIBRARY(mb)
LCB_ASM_TOWER_LIBRARY(mb)

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("{\"error\": \"%s\", \"line\": %d}\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

extern "C" __global__ void LCB_PAIR_BOUNDS k_sqr_asm(u32 *park, u32 n) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    lcb_asm_cyc_sqr_n(park, park, n * 16, i * 16, 63);
}
extern "C" __global__ void LCB_PAIR_BOUNDS k_sqr_c(u32 *park, u32 n) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fp12 f;
    fp12_load_soa(f, park, n, i);
    for (int k = 0; k < 63; k++) fp12_cyc_sqr(f, f);
    fp12_store_soa(park, n, i, f);
}
extern "C" __global__ void LCB_PAIR_BOUNDS k_mul_slot(u32 *park, u32 n) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    __shared__ uint4 lds[36 * LCB_BLOCK];
    for (int k = 0; k < 5; k++) fx_mul(park, park, park + (size_t)144 * n, 0, n, i, FxLds{lds + threadIdx.x});
}
extern "C" __global__ void LCB_PAIR_BOUNDS k_easy(u32 *park, u32 n) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fx_easy(park, n, i);
}
extern "C" __global__ void LCB_PAIR_BOUNDS k_fe_asm(u32 *park, u32 n) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    __shared__ uint4 lds[36 * LCB_BLOCK];
    final_exp_asm(park, n, i, FxLds{lds + threadIdx.x});
}
extern "C" __global__ void LCB_PAIR_BOUNDS k_fe_funcs(u32 *park, u32 n) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fp12 f;
    fp12_load_soa(f, park, n, i);
    final_exp_inplace(f);
    fp12_store_soa(park, n, i, f);
}

// occupancy probe: a chain of 200 Fp2 products (lazy leaf routine) per lane with few live registers, at 1 and 2
// waves per SIMD (not 4: the leaf routine writes v0..v131, beyond a 4-wave budget of 128 VGPRs)
template <int W>
__device__ __forceinline__ void fp2_chain(u32 *park, u32 n) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fp2 x, y;
    for (int j = 0; j < 12; j++) { x.a.v[j] = park[j * n + i]; x.b.v[j] = park[(12 + j) * n + i]; y.a.v[j] = park[(24 + j) * n + i]; y.b.v[j] = park[(36 + j) * n + i]; }
    for (int k = 0; k < 200; k++) fp2_mul(x, x, y);
    for (int j = 0; j < 12; j++) { park[j * n + i] = x.a.v[j]; park[(12 + j) * n + i] = x.b.v[j]; }
}
extern "C" __global__ void __launch_bounds__(256, 1) k_fp2_w1(u32 *park, u32 n) { fp2_chain<1>(park, n); }
extern "C" __global__ void __launch_bounds__(256, 2) k_fp2_w2(u32 *park, u32 n) { fp2_chain<2>(park, n); }
extern "C" __global__ void __launch_bounds__(256, 2) k_sqr_c_w2(u32 *park, u32 n) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    fp12 f;
    fp12_load_soa(f, park, n, i);
    for (int k = 0; k < 63; k++) fp12_cyc_sqr(f, f);
    fp12_store_soa(park, n, i, f);
}

typedef void (*kfn)(u32 *, u32);
int main(int argc, char **argv) {
    u32 n = argc > 1 ? (u32)atoi(argv[1]) : 262144;
    size_t words = (size_t)n * 144 * LCB_FE_ASM_SLOTS;
    u32 *h = (u32 *)malloc(words * 4);
    for (size_t k = 0; k < words; k++) h[k] = (u32)(k * 2654435761u) & ((k % 48) >= 44 ? 0 : 0xffffffffu);
    u32 *d;
    CK(hipMalloc(&d, words * 4));
    CK(hipMemcpy(d, h, words * 4, hipMemcpyHostToDevice));
    struct { const char *name; kfn f; int ops; } parts[] = {
        {"sqr_asm", k_sqr_asm, 63}, {"sqr_c", k_sqr_c, 63}, {"mul_slot", k_mul_slot, 5}, {"easy", k_easy, 1},
        {"fe_asm", k_fe_asm, 1}, {"fe_funcs", k_fe_funcs, 1},
        {"fp2x200_w1", k_fp2_w1, 200}, {"fp2x200_w2", k_fp2_w2, 200},
        {"sqr_c_w2", k_sqr_c_w2, 63}};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (auto &p : parts) {
        dim3 grid((n + LCB_BLOCK - 1) / LCB_BLOCK);
        hipLaunchKernelGGL(p.f, grid, dim3(LCB_BLOCK), 0, 0, d, n);   // warm-up
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(p.f, grid, dim3(LCB_BLOCK), 0, 0, d, n);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("{\"part\": \"%s\", \"n\": %u, \"ms\": %.3f, \"ms_per_op\": %.4f}\n", p.name, n, ms, ms / p.ops);
        fflush(stdout);
    }
    return 0;
}
