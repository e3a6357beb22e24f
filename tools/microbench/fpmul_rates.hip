// tools/microbench/fpmul_rates.hip — correctness + throughput of candidate 381-bit Montgomery multiplies
// (12 x 32-bit limbs) on gfx950, plus raw v_mad_u64_u32 throughput / latency.  JSON lines on stdout.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
typedef uint32_t u32; typedef uint64_t u64;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("{\"error\": \"%s\", \"line\": %d}\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
static const u32 P_H[12] = {0xffffaaab,0xb9feffff,0xb153ffff,0x1eabfffe,0xf6b0f624,0x6730d2a0,0xf38512bf,0x64774b84,0x434bacd7,0x4b1ba7b6,0x397fe69a,0x1a0111ea};
__constant__ u32 PM[12] = {0xffffaaab,0xb9feffff,0xb153ffff,0x1eabfffe,0xf6b0f624,0x6730d2a0,0xf38512bf,0x64774b84,0x434bacd7,0x4b1ba7b6,0x397fe69a,0x1a0111ea};
#define PINV 0xfffcfffdu

// ---------------- style A: CIOS no-carry in plain C (compiler-generated)
__device__ __forceinline__ void mulA(u32 *r, const u32 *a, const u32 *b) {
    u32 t[12];
#pragma unroll
    for (int j = 0; j < 12; j++) t[j] = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
        u64 s = (u64)a[0] * b[i] + t[0];
        u32 A = s >> 32; t[0] = (u32)s;
        u32 m = t[0] * PINV;
        s = (u64)m * PM[0] + t[0];
        u32 C = s >> 32;
#pragma unroll
        for (int j = 1; j < 12; j++) {
            s = (u64)a[j] * b[i] + t[j] + A; A = s >> 32; t[j] = (u32)s;
            s = (u64)m * PM[j] + t[j] + C; C = s >> 32; t[j - 1] = (u32)s;
        }
        t[11] = C + A;
    }
    u32 d[12]; u32 br = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) { u64 x = (u64)t[j] - PM[j] - br; d[j] = (u32)x; br = (x >> 32) & 1; }
#pragma unroll
    for (int j = 0; j < 12; j++) r[j] = br ? t[j] : d[j];
}

// ---------------- style B: product scanning (FIPS) Montgomery, asm MAC with carry-out into a 3rd word
__device__ __forceinline__ void mac(u64 &acc, u32 &hi, u32 a, u32 b) {
    asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc"
        : "+v"(acc), "+v"(hi) : "v"(a), "v"(b) : "vcc");
}
template <int NACC>
__device__ __forceinline__ void mulB(u32 *r, const u32 *a, const u32 *b) {
    u32 m[12];
    u64 acc[NACC]; u32 hi[NACC];
    u64 carry = 0; u32 carry_hi = 0;   // running column value (beyond the low word): 96-bit (carry_hi:carry)
#pragma unroll
    for (int k = 0; k < 23; k++) {
#pragma unroll
        for (int q = 0; q < NACC; q++) { acc[q] = 0; hi[q] = 0; }
        acc[0] = carry; hi[0] = carry_hi;
        int n = 0;
        int lo = k < 12 ? 0 : k - 11, up = k < 12 ? k : 11;
#pragma unroll
        for (int i = lo; i <= up; i++) {
            mac(acc[n % NACC], hi[n % NACC], a[i], b[k - i]); n++;
            if (i < k && i < 12 && k - i < 12 && i <= 11 && i < k) {
                if (i < 12 && (k < 12 ? i < k : true)) { mac(acc[n % NACC], hi[n % NACC], m[i], PM[k - i]); n++; }
            }
        }
        // merge accumulators
#pragma unroll
        for (int q = 1; q < NACC; q++) {
            u64 s = acc[0] + acc[q];
            hi[0] += hi[q] + (s < acc[0]);
            acc[0] = s;
        }
        if (k < 12) {
            m[k] = (u32)acc[0] * PINV;
            mac(acc[0], hi[0], m[k], PM[0]);
        } else {
            r[k - 12] = (u32)acc[0];
        }
        carry = (acc[0] >> 32) | ((u64)hi[0] << 32);
        carry_hi = 0;
    }
    r[11] = (u32)carry;
    u32 d[12]; u32 br = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) { u64 x = (u64)r[j] - PM[j] - br; d[j] = (u32)x; br = (x >> 32) & 1; }
#pragma unroll
    for (int j = 0; j < 12; j++) r[j] = br ? r[j] : d[j];
}

template <int STYLE, int CHAINS>
__global__ void __launch_bounds__(256) k_fpmul(u32 *out, const u32 *in, int n, int iters) {
    int gid = blockIdx.x * blockDim.x + threadIdx.x;
    int src = gid % n;
    u32 a[CHAINS][12], b[12];
#pragma unroll
    for (int j = 0; j < 12; j++) { b[j] = in[j * n + src]; }
#pragma unroll
    for (int c = 0; c < CHAINS; c++)
#pragma unroll
        for (int j = 0; j < 12; j++) a[c][j] = in[(12 + j) * n + (src + c) % n];
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) {
            if (STYLE == 0) mulA(a[c], a[c], b);
            else if (STYLE == 1) mulB<1>(a[c], a[c], b);
            else mulB<2>(a[c], a[c], b);
        }
    }
    int total = gridDim.x * blockDim.x;
#pragma unroll
    for (int j = 0; j < 12; j++) { u32 x = 0; for (int c = 0; c < CHAINS; c++) x ^= a[c][j]; out[j * total + gid] = x; }
}

__global__ void __launch_bounds__(256) k_mad_lat(u64 *out, u32 seed, int iters) {
    u32 tid = blockIdx.x * blockDim.x + threadIdx.x;
    u64 acc = tid; u32 a = seed ^ tid, b = seed + 7;
    for (int it = 0; it < iters; it++) {
#pragma unroll 16
        for (int k = 0; k < 16; k++) acc = (u64)((u32)acc ^ a) * b + acc;
    }
    out[tid] = acc;
}
__global__ void __launch_bounds__(256) k_mad_tp(u64 *out, u32 seed, int iters) {
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

// ---------------- host reference (CIOS, 64-bit intermediate)
static void host_mul(u32 *r, const u32 *a, const u32 *b) {
    u32 t[14] = {0};
    for (int i = 0; i < 12; i++) {
        u64 c = 0;
        for (int j = 0; j < 12; j++) { u64 s = (u64)a[j] * b[i] + t[j] + c; t[j] = (u32)s; c = s >> 32; }
        u64 s = (u64)t[12] + c; t[12] = (u32)s; t[13] = (u32)(s >> 32);
        u32 m = t[0] * PINV;
        s = (u64)m * P_H[0] + t[0]; c = s >> 32;
        for (int j = 1; j < 12; j++) { s = (u64)m * P_H[j] + t[j] + c; t[j - 1] = (u32)s; c = s >> 32; }
        s = (u64)t[12] + c; t[11] = (u32)s; t[12] = t[13] + (u32)(s >> 32);
    }
    u32 d[12]; u32 br = 0;
    for (int j = 0; j < 12; j++) { u64 x = (u64)t[j] - P_H[j] - br; d[j] = (u32)x; br = (x >> 32) & 1; }
    int ge = !br || t[12];
    for (int j = 0; j < 12; j++) r[j] = ge ? d[j] : t[j];
}
static u64 rng = 0x243f6a8885a308d3ULL;
static u32 rnd() { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return (u32)rng; }

template <int STYLE, int CHAINS>
static int bench(const char *name, u32 *d_in, u32 *h_in, int n, u32 *d_out, int blocks, hipEvent_t e0, hipEvent_t e1) {
    int total = blocks * 256;
    // correctness: iters = 3, compare lanes < n (chain 0 only when CHAINS == 1)
    hipLaunchKernelGGL((k_fpmul<STYLE, 1>), dim3(n / 256), dim3(256), 0, 0, d_out, d_in, n, 3);
    CK(hipDeviceSynchronize());
    u32 *h_out = (u32 *)malloc((size_t)n * 12 * 4);
    CK(hipMemcpy(h_out, d_out, (size_t)n * 12 * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int l = 0; l < n; l++) {
        u32 a[12], b[12];
        for (int j = 0; j < 12; j++) { b[j] = h_in[j * n + l]; a[j] = h_in[(12 + j) * n + l]; }
        for (int it = 0; it < 3; it++) host_mul(a, a, b);
        for (int j = 0; j < 12; j++) if (a[j] != h_out[j * (n / 256) * 256 + l]) { bad++; break; }
    }
    free(h_out);
    hipLaunchKernelGGL((k_fpmul<STYLE, CHAINS>), dim3(blocks), dim3(256), 0, 0, d_out, d_in, n, 8);
    CK(hipDeviceSynchronize());
    int iters = 2000;
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL((k_fpmul<STYLE, CHAINS>), dim3(blocks), dim3(256), 0, 0, d_out, d_in, n, iters);
    hipEventRecord(e1, 0);
    CK(hipEventSynchronize(e1));
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double muls = (double)total * iters * CHAINS;
    printf("{\"test\": \"%s\", \"chains\": %d, \"mismatch\": %d, \"ms\": %.3f, \"fpmul_per_s\": %.4e, \"mac32_per_s\": %.4e}\n",
           name, CHAINS, bad, ms, muls / (ms * 1e-3), 300.0 * muls / (ms * 1e-3));
    return 0;
}

int main() {
    hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
    printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
    int blocks = prop.multiProcessorCount * 8;
    int n = 4096;
    u32 *h_in = (u32 *)malloc((size_t)n * 24 * 4);
    for (int j = 0; j < 24; j++)
        for (int l = 0; l < n; l++) h_in[j * n + l] = rnd();
    for (int l = 0; l < n; l++) { h_in[11 * n + l] &= 0x0fffffff; h_in[23 * n + l] &= 0x0fffffff; }  // < p
    u32 *d_in, *d_out; u64 *d_o64;
    CK(hipMalloc(&d_in, (size_t)n * 24 * 4));
    CK(hipMalloc(&d_out, (size_t)blocks * 256 * 12 * 4));
    CK(hipMalloc(&d_o64, (size_t)blocks * 256 * 8));
    CK(hipMemcpy(d_in, h_in, (size_t)n * 24 * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    // raw mad throughput and latency
    {
        int iters = 20000;
        hipLaunchKernelGGL(k_mad_tp, dim3(blocks), dim3(256), 0, 0, d_o64, 1u, 16);
        CK(hipDeviceSynchronize());
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_mad_tp, dim3(blocks), dim3(256), 0, 0, d_o64, 1u, iters);
        hipEventRecord(e1, 0); CK(hipEventSynchronize(e1));
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("{\"test\": \"v_mad_u64_u32 throughput\", \"ms\": %.3f, \"lane_mad_per_s\": %.4e}\n", ms, (double)blocks * 256 * iters * 8 / (ms * 1e-3));
        int lb = prop.multiProcessorCount * 4 / 4;  // one wave per SIMD: 256 CUs x 4 SIMDs = blocks of 64? use 256-thread blocks, 1 per CU
        hipLaunchKernelGGL(k_mad_lat, dim3(prop.multiProcessorCount), dim3(256), 0, 0, d_o64, 1u, 16);
        CK(hipDeviceSynchronize());
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_mad_lat, dim3(prop.multiProcessorCount), dim3(256), 0, 0, d_o64, 1u, 2000);
        hipEventRecord(e1, 0); CK(hipEventSynchronize(e1));
        hipEventElapsedTime(&ms, e0, e1);
        printf("{\"test\": \"dependent (xor+mad) chain, 1 wave/SIMD\", \"ms\": %.3f, \"ns_per_link\": %.3f}\n", ms, ms * 1e6 / (2000.0 * 16));
        (void)lb;
    }
    bench<0, 1>("A cios-C", d_in, h_in, n, d_out, blocks, e0, e1);
    bench<0, 2>("A cios-C", d_in, h_in, n, d_out, blocks, e0, e1);
    bench<1, 1>("B comba-asm 1acc", d_in, h_in, n, d_out, blocks, e0, e1);
    bench<1, 2>("B comba-asm 1acc", d_in, h_in, n, d_out, blocks, e0, e1);
    bench<2, 1>("B comba-asm 2acc", d_in, h_in, n, d_out, blocks, e0, e1);
    bench<2, 2>("B comba-asm 2acc", d_in, h_in, n, d_out, blocks, e0, e1);
    return 0;
}
