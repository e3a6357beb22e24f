// lachain_amd/csrc/k_rs.hip — gfx950 kernels: Reed–Solomon erasure coding of the reliable-broadcast payloads
// (ReliableBroadcast.ErasureCodingShards / DecodeFromEchos,
// /root/reference/src/Lachain.Consensus/ReliableBroadcast/ReliableBroadcast.cs:393-446).
//
// Code: GF(2^8) with polynomial 0x11D, alpha = 2, codeword C(x) = sum_j c_j x^(n-1-j) vanishing at alpha^0..alpha^(ecc-1)
// (ErasureCoding.cs:13, GenericGF(285, 256, 0)).  Both directions are one linear map per shard pattern: the unknown
// symbols c_E (parity positions when encoding, the missing shards when decoding) satisfy H_E c_E = H_K c_K with
// H[i][j] = alpha^(i (n-1-j)), so c_E = M c_K with M = H_E^-1 H_K.  One workgroup builds M by Gauss-Jordan
// elimination in LDS (k_rs_matrix); then every byte column of the shards is an independent GF(2^8) matrix-vector
// product (k_rs_apply, byte work: log/exp tables in LDS, 4 bytes per lane, coalesced across the shard).  With as
// many unknowns as parity symbols the solution is the unique codeword through the known symbols, so the bytes equal
// any correct RS encoder/erasure decoder's, the reference's included.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gate.hpp"

typedef uint32_t u32;
#define RS_THREADS 256

__device__ __forceinline__ void gf_tables(uint8_t *ex, uint8_t *lg) {
    if (threadIdx.x == 0) {
        u32 x = 1;
        for (int i = 0; i < 255; i++) {
            ex[i] = (uint8_t)x;
            lg[x] = (uint8_t)i;
            x <<= 1;
            if (x & 0x100) x ^= 0x11D;
        }
        for (int i = 255; i < 512; i++) ex[i] = ex[i - 255];
        lg[0] = 0;
    }
    __syncthreads();
}
__device__ __forceinline__ uint8_t gmul(const uint8_t *ex, const uint8_t *lg, uint8_t a, uint8_t b) {
    return (a && b) ? ex[lg[a] + lg[b]] : 0;
}

// M (m x k, row-major) = H_E^-1 H_K for unknown positions pe[0..m) and known positions pk[0..k) of an n-symbol
// codeword; ok[0] = 0 when H_E is singular (two unknown positions with the same evaluation point, n > 255)
extern "C" __global__ void __launch_bounds__(RS_THREADS) k_rs_matrix(const int *pe, int m, const int *pk, int k, int n,
                                                                    uint8_t *M, uint8_t *ok) {
    __shared__ uint8_t ex[512], lg[256];
    extern __shared__ uint8_t A[];       // m x (m + k) augmented matrix [H_E | H_K]
    __shared__ int piv;
    gf_tables(ex, lg);
    const int w = m + k;
    for (int t = threadIdx.x; t < m * w; t += blockDim.x) {
        int i = t / w, c = t % w;
        int pos = c < m ? pe[c] : pk[c - m];
        int e = (i * (n - 1 - pos)) % 255;
        A[t] = ex[e < 0 ? e + 255 : e];
    }
    __syncthreads();
    bool good = true;
    for (int c = 0; c < m; c++) {
        if (threadIdx.x == 0) {
            int p = -1;
            for (int r = c; r < m; r++)
                if (A[r * w + c]) { p = r; break; }
            piv = p;
        }
        __syncthreads();
        int p = piv;
        if (p < 0) { good = false; break; }
        if (p != c)
            for (int t = threadIdx.x; t < w; t += blockDim.x) {
                uint8_t a = A[p * w + t];
                A[p * w + t] = A[c * w + t];
                A[c * w + t] = a;
            }
        __syncthreads();
        uint8_t inv = ex[(255 - lg[A[c * w + c]]) % 255];
        __syncthreads();
        for (int t = threadIdx.x; t < w; t += blockDim.x) A[c * w + t] = gmul(ex, lg, A[c * w + t], inv);
        __syncthreads();
        for (int t = threadIdx.x; t < m * w; t += blockDim.x) {
            int r = t / w, cc = t % w;
            if (r == c) continue;
            uint8_t f = A[r * w + c];
            if (f && cc != c) A[t] ^= gmul(ex, lg, f, A[c * w + cc]);
        }
        __syncthreads();
        for (int r = threadIdx.x; r < m; r += blockDim.x)
            if (r != c) A[r * w + c] = 0;
        __syncthreads();
    }
    for (int t = threadIdx.x; t < m * k; t += blockDim.x) M[t] = good ? A[(t / k) * w + m + (t % k)] : 0;
    if (threadIdx.x == 0) ok[0] = good;
}

// out shard pe[r] (row r of M) = sum_j M[r][j] * (known shard j); known shard j at src + j * S, output shard at
// dst + pe[r] * S.  One lane per (r, 4-byte column group).
extern "C" __global__ void __launch_bounds__(RS_THREADS) k_rs_apply(const uint8_t *M, const uint8_t *ok, int m, int k,
                                                                   const uint8_t *src, size_t S, const int *pe,
                                                                   uint8_t *dst) {
    __shared__ uint8_t ex[512], lg[256];
    gf_tables(ex, lg);
    size_t groups = (S + 3) / 4;
    size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)m * groups) return;
    int r = (int)(t / groups);
    size_t i0 = (t % groups) * 4;
    int nb = (int)((S - i0) < 4 ? (S - i0) : 4);
    u32 acc = 0;
    if (ok[0]) {
        const uint8_t *Mr = M + (size_t)r * k;
        for (int j = 0; j < k; j++) {
            uint8_t c = Mr[j];
            if (!c) continue;
            int lc = lg[c];
            const uint8_t *s = src + (size_t)j * S + i0;
            u32 v = 0;
            if (nb == 4 && ((((uintptr_t)s) & 3) == 0)) v = *(const u32 *)s;
            else for (int b = 0; b < nb; b++) v |= (u32)s[b] << (8 * b);
#pragma unroll
            for (int b = 0; b < 4; b++) {
                u32 x = (v >> (8 * b)) & 0xffu;
                if (x) acc ^= (u32)ex[lc + lg[x]] << (8 * b);
            }
        }
    }
    uint8_t *d = dst + (size_t)pe[r] * S + i0;
    if (nb == 4 && ((((uintptr_t)d) & 3) == 0)) *(u32 *)d = acc;
    else for (int b = 0; b < nb; b++) d[b] = (uint8_t)(acc >> (8 * b));
}

// ---------------------------------------------------------------- host launch wrappers
extern "C" const void *lcbk_rs_matrix_kernel() { return (const void *)k_rs_matrix; }
extern "C" void lcbk_rs_matrix(hipStream_t s, const int *pe, int m, const int *pk, int k, int n, uint8_t *M, uint8_t *ok) {
    LCB_LAUNCH_GATED(k_rs_matrix, dim3(1), dim3(RS_THREADS), (size_t)m * (m + k), s, pe, m, pk, k, n, M, ok);
}
extern "C" void lcbk_rs_apply(hipStream_t s, const uint8_t *M, const uint8_t *ok, int m, int k, const uint8_t *src, size_t S,
                              const int *pe, uint8_t *dst) {
    size_t lanes = (size_t)m * ((S + 3) / 4);
    if (!lanes) return;
    LCB_LAUNCH_GATED(k_rs_apply, dim3((unsigned)((lanes + RS_THREADS - 1) / RS_THREADS)), dim3(RS_THREADS), 0, s, M, ok, m,
                       k, src, S, pe, dst);
}
