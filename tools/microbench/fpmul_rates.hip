// tools/microbench/fpmul_rates.hip — correctness + throughput of candidate 381-bit Montgomery multiplies
// (12 x 32-bit limbs) on gfx950, plus raw v_mad_u64_u32 throughput / latency.  JSON lines on stdout.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <fenv.h>
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

// ---------------- style F: FP64-FMA product on 8 x 52-bit limbs (Emmart, Zheng, Weems, "Faster modular exponentiation
// using double precision floating point arithmetic on the GPU", ARITH 2018).  A 52 x 52-bit product is split exactly by
// two round-toward-zero FMAs: hi = fma(a, b, 2^104) keeps floor(ab / 2^52) in its mantissa, lo = fma(a, b, 2^104 + 2^52
// - hi) = 2^52 + (ab mod 2^52).  Column sums are kept as the integer bit patterns of hi / lo (biases folded by the
// compiler), Montgomery reduction with R = 2^416 (> 4p, so inputs and outputs stay lazily below 2p).  The kernel sets
// the f64 rounding mode (MODE.FP_ROUND[3:2]) to round-toward-zero at entry.
#define M52 0xfffffffffffffull
#define B104 0x4670000000000000ull
#define B52 0x4330000000000000ull
#define PINV52 0x3fffcfffcfffdull
static const u64 P52_H[8] = {0xeffffffffaaabull, 0xfeb153ffffb9full, 0x6b0f6241eabffull, 0x12bf6730d2a0full,
                             0x764774b84f385ull, 0x1ba7b6434bacdull, 0x1ea397fe69a4bull, 0x1a011ull};
#define HD __host__ __device__ __forceinline__
HD u64 dbits(double x) { u64 r; memcpy(&r, &x, 8); return r; }
HD double bitsd(u64 x) { double r; memcpy(&r, &x, 8); return r; }
HD void fsplit(u64 &lo_col, u64 &hi_col, double a, double b) {
    double hi = __builtin_fma(a, b, 0x1p104);
    double lo = __builtin_fma(a, b, (0x1p104 + 0x1p52) - hi);
    hi_col += dbits(hi) - B104;
    lo_col += dbits(lo) - B52;
}
HD void mul52(double *r, const double *a, const double *b) {
    const double P52D[8] = {(double)0xeffffffffaaabull, (double)0xfeb153ffffb9full, (double)0x6b0f6241eabffull,
                            (double)0x12bf6730d2a0full, (double)0x764774b84f385ull, (double)0x1ba7b6434bacdull,
                            (double)0x1ea397fe69a4bull, (double)0x1a011ull};
    u64 col[17];
#pragma unroll
    for (int k = 0; k < 17; k++) col[k] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 8; j++) fsplit(col[i + j], col[i + j + 1], a[i], b[j]);
#pragma unroll
    for (int i = 0; i < 8; i++) {
        double t = bitsd(B52 | (col[i] & M52)) - 0x1p52;
        double mh = __builtin_fma(t, (double)PINV52, 0x1p104);
        double ml = __builtin_fma(t, (double)PINV52, (0x1p104 + 0x1p52) - mh);
        double m = ml - 0x1p52;
#pragma unroll
        for (int j = 0; j < 8; j++) fsplit(col[i + j], col[i + j + 1], m, P52D[j]);
        col[i + 1] += col[i] >> 52;
    }
#pragma unroll
    for (int k = 8; k < 16; k++) {
        col[k + 1] += col[k] >> 52;
        r[k - 8] = bitsd(B52 | (col[k] & M52)) - 0x1p52;
    }
}
__device__ __forceinline__ void set_f64_round_toward_zero() {
    asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 3" ::: "memory");
}

template <int CHAINS>
__global__ void __launch_bounds__(256) k_fpmul52(u64 *out, const u64 *in, int n, int iters) {
    set_f64_round_toward_zero();
    int gid = blockIdx.x * blockDim.x + threadIdx.x;
    int src = gid % n;
    double a[CHAINS][8], b[8];
#pragma unroll
    for (int j = 0; j < 8; j++) b[j] = bitsd(B52 | in[j * n + src]) - 0x1p52;
#pragma unroll
    for (int c = 0; c < CHAINS; c++)
#pragma unroll
        for (int j = 0; j < 8; j++) a[c][j] = bitsd(B52 | in[(8 + j) * n + (src + c) % n]) - 0x1p52;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) mul52(a[c], a[c], b);
    }
    int total = gridDim.x * blockDim.x;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        u64 x = 0;
        for (int c = 0; c < CHAINS; c++) x ^= dbits(a[c][j] + 0x1p52) & M52;
        out[j * total + gid] = x;
    }
}

// raw issue rates of the two instruction kinds the FP64 product is made of
__global__ void __launch_bounds__(256) k_fma64_tp(double *out, double seed, int iters) {
    u32 tid = blockIdx.x * blockDim.x + threadIdx.x;
    double acc[8], x = seed + tid, y = seed * 0.5;
    for (int k = 0; k < 8; k++) acc[k] = tid + k;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) acc[k] = __builtin_fma(acc[k], x, y);
    }
    double s = 0;
    for (int k = 0; k < 8; k++) s += acc[k];
    out[tid] = s;
}
__global__ void __launch_bounds__(256) k_add64_tp(u64 *out, u64 seed, int iters) {
    u32 tid = blockIdx.x * blockDim.x + threadIdx.x;
    u64 acc[8], b[8];
    for (int k = 0; k < 8; k++) { acc[k] = tid + k; b[k] = seed * (k + 3) + tid; }
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) { acc[k] += b[k]; b[k] ^= acc[k]; }
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

// x < 2p in 52-bit limbs -> 12 x 32-bit words reduced below p
static void from52(u32 *w, const u64 *l) {
    memset(w, 0, 48);
    for (int i = 0; i < 8; i++)
        for (int b = 0; b < 52; b++)
            if ((l[i] >> b) & 1) { int pos = 52 * i + b; if (pos < 384) w[pos / 32] |= 1u << (pos % 32); }
    u32 d[12]; u32 br = 0;
    for (int j = 0; j < 12; j++) { u64 x = (u64)w[j] - P_H[j] - br; d[j] = (u32)x; br = (x >> 32) & 1; }
    if (!br) memcpy(w, d, 48);
}
static void to52(u64 *l, const u32 *w) {
    memset(l, 0, 64);
    for (int pos = 0; pos < 384; pos++)
        if ((w[pos / 32] >> (pos % 32)) & 1) l[pos / 52] |= 1ull << (pos % 52);
}
static void pow2_mod_p(u32 *w, int e) {   // 2^e mod p by doubling
    memset(w, 0, 48); w[0] = 1;
    for (int k = 0; k < e; k++) {
        u32 c = 0;
        for (int j = 0; j < 12; j++) { u32 nc = w[j] >> 31; w[j] = (w[j] << 1) | c; c = nc; }
        u32 d[12]; u32 br = 0;
        for (int j = 0; j < 12; j++) { u64 x = (u64)w[j] - P_H[j] - br; d[j] = (u32)x; br = (x >> 32) & 1; }
        if (!br) memcpy(w, d, 48);
    }
}

template <int CHAINS>
static int bench52(u32 *h_in, int n, int blocks, hipEvent_t e0, hipEvent_t e1) {
    const int ITER_CHECK = 3;
    int total = blocks * 256;
    u64 *h52 = (u64 *)malloc((size_t)n * 16 * 8);
    for (int l = 0; l < n; l++) {
        u32 a[12], b[12]; u64 la[8], lb[8];
        for (int j = 0; j < 12; j++) { b[j] = h_in[j * n + l]; a[j] = h_in[(12 + j) * n + l]; }
        to52(lb, b); to52(la, a);
        for (int j = 0; j < 8; j++) { h52[j * n + l] = lb[j]; h52[(8 + j) * n + l] = la[j]; }
    }
    u64 *d_in, *d_out;
    CK(hipMalloc(&d_in, (size_t)n * 16 * 8));
    CK(hipMalloc(&d_out, (size_t)total * 8 * 8));
    CK(hipMemcpy(d_in, h52, (size_t)n * 16 * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL((k_fpmul52<1>), dim3(n / 256), dim3(256), 0, 0, d_out, d_in, n, ITER_CHECK);
    CK(hipDeviceSynchronize());
    u64 *h_out = (u64 *)malloc((size_t)n * 8 * 8);
    CK(hipMemcpy(h_out, d_out, (size_t)n * 8 * 8, hipMemcpyDeviceToHost));
    // kernel: a b^3 2^(-3*416); 32-bit CIOS: a b^3 2^(-3*384); the latter = host_mul(former, 2^(96+384) mod p)
    u32 c480[12]; pow2_mod_p(c480, 480);
    int bad = 0, over = 0;
    for (int l = 0; l < n; l++) {
        u32 a[12], b[12], x[12]; u64 lx[8];
        for (int j = 0; j < 12; j++) { b[j] = h_in[j * n + l]; a[j] = h_in[(12 + j) * n + l]; }
        for (int it = 0; it < ITER_CHECK; it++) host_mul(a, a, b);
        for (int j = 0; j < 8; j++) { lx[j] = h_out[j * (n / 256) * 256 + l]; if (lx[j] >> 52) over++; }
        from52(x, lx);
        host_mul(x, x, c480);
        if (memcmp(x, a, 48)) bad++;
    }
    free(h_out); free(h52);
    hipLaunchKernelGGL((k_fpmul52<CHAINS>), dim3(blocks), dim3(256), 0, 0, d_out, d_in, n, 8);
    CK(hipDeviceSynchronize());
    int iters = 2000;
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL((k_fpmul52<CHAINS>), dim3(blocks), dim3(256), 0, 0, d_out, d_in, n, iters);
    hipEventRecord(e1, 0);
    CK(hipEventSynchronize(e1));
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double muls = (double)total * iters * CHAINS;
    printf("{\"test\": \"F fp64-fma 52-bit\", \"chains\": %d, \"mismatch\": %d, \"limb_overflow\": %d, \"checked\": %d, "
           "\"ms\": %.3f, \"fpmul_per_s\": %.4e, \"vs_5.69e10\": %.3f}\n",
           CHAINS, bad, over, n, ms, muls / (ms * 1e-3), muls / (ms * 1e-3) / 5.69e10);
    CK(hipFree(d_in)); CK(hipFree(d_out));
    return 0;
}

// the FP64 product on the host FPU under round-toward-zero: same check as the GPU one (`fpmul_rates --host-only`)
static int host_check52(int n) {
    fesetround(FE_TOWARDZERO);
    u32 c480[12]; pow2_mod_p(c480, 480);
    int bad = 0, over = 0;
    for (int l = 0; l < n; l++) {
        u32 a[12], b[12], x[12]; u64 la[8], lb[8], lx[8]; double da[8], db[8];
        for (int j = 0; j < 12; j++) { a[j] = rnd(); b[j] = rnd(); }
        a[11] &= 0x0fffffff; b[11] &= 0x0fffffff;
        if (l == 0) { memcpy(a, P_H, 48); a[0] -= 1; memcpy(b, a, 48); }   // p - 1 squared
        to52(la, a); to52(lb, b);
        for (int j = 0; j < 8; j++) { da[j] = (double)la[j]; db[j] = (double)lb[j]; }
        for (int it = 0; it < 3; it++) { mul52(da, da, db); host_mul(a, a, b); }
        for (int j = 0; j < 8; j++) { lx[j] = (u64)da[j]; if (lx[j] >> 52) over++; }
        from52(x, lx);
        host_mul(x, x, c480);
        if (memcmp(x, a, 48)) bad++;
    }
    fesetround(FE_TONEAREST);
    printf("{\"test\": \"F fp64-fma 52-bit host (RZ)\", \"checked\": %d, \"mismatch\": %d, \"limb_overflow\": %d}\n", n, bad, over);
    return bad || over;
}

int main(int argc, char **argv) {
    if (argc > 1 && !strcmp(argv[1], "--host-only")) return host_check52(20000);
    if (host_check52(2000)) return 1;
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
    {
        double *d_f; CK(hipMalloc(&d_f, (size_t)blocks * 256 * 8));
        int iters = 20000;
        hipLaunchKernelGGL(k_fma64_tp, dim3(blocks), dim3(256), 0, 0, d_f, 1.0000001, 16);
        CK(hipDeviceSynchronize());
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_fma64_tp, dim3(blocks), dim3(256), 0, 0, d_f, 1.0000001, iters);
        hipEventRecord(e1, 0); CK(hipEventSynchronize(e1));
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("{\"test\": \"v_fma_f64 throughput\", \"ms\": %.3f, \"lane_fma_per_s\": %.4e}\n", ms, (double)blocks * 256 * iters * 8 / (ms * 1e-3));
        hipLaunchKernelGGL(k_add64_tp, dim3(blocks), dim3(256), 0, 0, d_o64, 3ull, 16);
        CK(hipDeviceSynchronize());
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k_add64_tp, dim3(blocks), dim3(256), 0, 0, d_o64, 3ull, iters);
        hipEventRecord(e1, 0); CK(hipEventSynchronize(e1));
        hipEventElapsedTime(&ms, e0, e1);
        printf("{\"test\": \"u64 add+xor throughput\", \"ms\": %.3f, \"lane_add64_xor64_per_s\": %.4e}\n", ms, (double)blocks * 256 * iters * 8 / (ms * 1e-3));
        CK(hipFree(d_f));
    }
    bench<0, 1>("A cios-C", d_in, h_in, n, d_out, blocks, e0, e1);
    bench<0, 2>("A cios-C", d_in, h_in, n, d_out, blocks, e0, e1);
    bench<1, 1>("B comba-asm 1acc", d_in, h_in, n, d_out, blocks, e0, e1);
    bench<1, 2>("B comba-asm 1acc", d_in, h_in, n, d_out, blocks, e0, e1);
    bench<2, 1>("B comba-asm 2acc", d_in, h_in, n, d_out, blocks, e0, e1);
    bench<2, 2>("B comba-asm 2acc", d_in, h_in, n, d_out, blocks, e0, e1);
    bench52<1>(h_in, n, blocks, e0, e1);
    bench52<2>(h_in, n, blocks, e0, e1);
    return 0;
}
