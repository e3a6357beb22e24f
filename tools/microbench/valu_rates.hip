// tools/microbench/valu_rates.hip — measures gfx950 VALU throughput of the integer instructions the
// Fp (381-bit, 12x32-bit limb) Montgomery multiply is built from.  Prints one JSON line per test.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t u32; typedef uint64_t u64;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("{\"error\": \"%s\"}\n", hipGetErrorString(e)); return 1; } } while (0)

// 8 independent v_mad_u64_u32 accumulation chains per lane (acc = a*b + acc, in-place pair)
extern "C" __global__ void __launch_bounds__(256) k_mad64(u64 *out, u32 seed, int iters) {
    u32 tid = blockIdx.x * blockDim.x + threadIdx.x;
    u64 acc[8]; u32 b[8];
    for (int k = 0; k < 8; k++) { acc[k] = tid + k; b[k] = seed * (k + 3) + tid; }
    u32 a = seed ^ tid;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) acc[k] = (u64)a * b[k] + acc[k];
        a += 0x9e3779b9u;
    }
    u64 s = 0;
    for (int k = 0; k < 8; k++) s ^= acc[k];
    out[tid] = s;
}
// v_mul_lo_u32 + v_mul_hi_u32 pair chains
extern "C" __global__ void __launch_bounds__(256) k_mul32(u32 *out, u32 seed, int iters) {
    u32 tid = blockIdx.x * blockDim.x + threadIdx.x;
    u32 x[8];
    for (int k = 0; k < 8; k++) x[k] = tid * (k + 7) + seed;
    u32 m = seed | 1;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = x[k] * m + k;
    }
    u32 s = 0;
    for (int k = 0; k < 8; k++) s ^= x[k];
    out[tid] = s;
}
// full-rate reference: v_add3_u32 chains
extern "C" __global__ void __launch_bounds__(256) k_add32(u32 *out, u32 seed, int iters) {
    u32 tid = blockIdx.x * blockDim.x + threadIdx.x;
    u32 x[8];
    for (int k = 0; k < 8; k++) x[k] = tid * (k + 7) + seed;
    u32 m = seed | 1;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = (x[k] ^ m) + (x[(k + 1) & 7]);
        m += 0x3c6ef372u;
    }
    u32 s = 0;
    for (int k = 0; k < 8; k++) s ^= x[k];
    out[tid] = s;
}

static float run(const char *name, void (*launch)(void *, u32, int, int), void *buf, int blocks, int iters, double ops_per_iter_lane, hipEvent_t e0, hipEvent_t e1) {
    launch(buf, 1, 16, blocks);
    hipDeviceSynchronize();
    hipEventRecord(e0, 0);
    launch(buf, 1, iters, blocks);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double lanes = (double)blocks * 256;
    double ops = lanes * iters * ops_per_iter_lane;
    printf("{\"test\": \"%s\", \"ms\": %.3f, \"lane_ops_per_s\": %.4e, \"blocks\": %d, \"iters\": %d}\n", name, ms, ops / (ms * 1e-3), blocks, iters);
    return ms;
}
static void L_mad(void *b, u32 s, int it, int bl) { hipLaunchKernelGGL(k_mad64, dim3(bl), dim3(256), 0, 0, (u64 *)b, s, it); }
static void L_mul(void *b, u32 s, int it, int bl) { hipLaunchKernelGGL(k_mul32, dim3(bl), dim3(256), 0, 0, (u32 *)b, s, it); }
static void L_add(void *b, u32 s, int it, int bl) { hipLaunchKernelGGL(k_add32, dim3(bl), dim3(256), 0, 0, (u32 *)b, s, it); }

int main() {
    hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
    printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
    int blocks = prop.multiProcessorCount * 8;
    void *buf; CK(hipMalloc(&buf, (size_t)blocks * 256 * 8));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    run("v_mad_u64_u32", L_mad, buf, blocks, 20000, 8, e0, e1);
    run("v_mul_lo_u32+add", L_mul, buf, blocks, 20000, 8, e0, e1);
    run("xor+add (2 ops)", L_add, buf, blocks, 20000, 16, e0, e1);
    return 0;
}
