// tools/microbench/occupancy.hip — Fp2 multiplications per second of the production asm leaf routine
// (lcb_asm_fp2_mul, lachain_amd/csrc/asm_routines.hpp) at 1, 2 and 3 waves per SIMD: tells whether the pairing
// kernels (one wave per SIMD) are bound by per-wave latency or by the VALU pipe.  JSON lines on stdout.
#include "../../lachain_amd/csrc/kcommon.hpp"
#include <stdio.h>

LCB_ASM_LIBRARY(occ)

extern "C" __global__ void __launch_bounds__(256) k_fp2mul_loop(u32 *out, int iters) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    fp2 x, y;
    for (int j = 0; j < 12; j++) { x.a.v[j] = i * 7 + j; x.b.v[j] = i * 13 + j; y.a.v[j] = i + 3 * j; y.b.v[j] = j; }
    x.a.v[11] &= 0x0fffffff; x.b.v[11] &= 0x0fffffff; y.a.v[11] &= 0x0fffffff; y.b.v[11] &= 0x0fffffff;
    for (int k = 0; k < iters; k++) fp2_mul(x, x, y);
    u32 acc = 0;
    for (int j = 0; j < 12; j++) acc ^= x.a.v[j] ^ x.b.v[j];
    out[i] = acc;
}
// two independent chains per lane (what a second share per lane would give)
extern "C" __global__ void __launch_bounds__(256) k_fp2mul_loop2(u32 *out, int iters) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    fp2 x, y, z;
    for (int j = 0; j < 12; j++) { x.a.v[j] = i * 7 + j; x.b.v[j] = i * 13 + j; y.a.v[j] = i + 3 * j; y.b.v[j] = j; z.a.v[j] = i ^ j; z.b.v[j] = 5 * j; }
    x.a.v[11] &= 0x0fffffff; x.b.v[11] &= 0x0fffffff; y.a.v[11] &= 0x0fffffff; y.b.v[11] &= 0x0fffffff;
    z.a.v[11] &= 0x0fffffff; z.b.v[11] &= 0x0fffffff;
    for (int k = 0; k < iters; k++) { fp2_mul(x, x, y); fp2_mul(z, z, y); }
    u32 acc = 0;
    for (int j = 0; j < 12; j++) acc ^= x.a.v[j] ^ x.b.v[j] ^ z.a.v[j] ^ z.b.v[j];
    out[i] = acc;
}

// the Miller-loop arithmetic without memory: 63 x (fp12 square + two sparse line products) per lane, lines held
// in registers — compared with k_tpke_miller's per-iteration time it separates arithmetic from line loads / spills
extern "C" __global__ void LCB_BOUNDS k_miller_arith(u32 *out, int iters) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    fp12 f;
    u32 *fw = (u32 *)&f;
    for (int j = 0; j < 144; j++) fw[j] = (i * 2654435761u + j * 40503u) & (j % 12 == 11 ? 0x0fffffffu : 0xffffffffu);
    line l;
    u32 *lw = (u32 *)&l;
    for (int j = 0; j < 72; j++) lw[j] = (i + j * 977u) & (j % 12 == 11 ? 0x0fffffffu : 0xffffffffu);
    fp x1 = f.c0.c0.a, y1 = f.c0.c1.b, x2 = f.c1.c2.a, y2 = f.c1.c0.b;
    for (int k = 0; k < iters; k++) {
        fp12_sqr(f, f);
        fp12_mul_line_at(f, l, x1, y1);
        fp12_mul_line_at(f, l, x2, y2);
    }
    u32 acc = 0;
    for (int j = 0; j < 144; j++) acc ^= fw[j];
    out[i] = acc;
}

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    int cus = prop.multiProcessorCount;
    u32 *d;
    hipMalloc(&d, (size_t)cus * 256 * 16 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 2000;
    for (int chains = 1; chains <= 2; chains++) {
        for (int wps = 1; wps <= 4; wps++) {          // waves per SIMD = blocks per CU (4 waves per block)
            int blocks = cus * wps;
            auto k = chains == 1 ? k_fp2mul_loop : k_fp2mul_loop2;
            hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 10);
            hipDeviceSynchronize();
            hipEventRecord(e0);
            hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            double fp2 = (double)blocks * 256 * iters * chains;
            printf("{\"test\": \"fp2_mul asm\", \"chains_per_lane\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, "
                   "\"fp2mul_per_s\": %.4e, \"fpmul_equiv_per_s\": %.4e, \"cycles_per_fp2mul_per_wave\": %.0f}\n",
                   chains, wps, ms, fp2 / (ms * 1e-3), 3 * fp2 / (ms * 1e-3),
                   ms * 1e-3 * 2.4e9 / (iters * chains));
        }
    }
    {
        int blocks = cus;   // one 256-thread block per CU = one wave per SIMD, as k_tpke_miller runs
        hipLaunchKernelGGL(k_miller_arith, dim3(blocks), dim3(256), 0, 0, d, 2);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_miller_arith, dim3(blocks), dim3(256), 0, 0, d, 63);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("{\"test\": \"miller arithmetic, lines in registers\", \"waves_per_simd\": 1, \"iters\": 63, \"ms\": %.3f, "
               "\"cycles_per_iter_per_wave\": %.0f}\n", ms, ms * 1e-3 * 2.4e9 / 63);
    }
    return 0;
}
