// lachain_amd/csrc/fr_host.hpp — scalar field Fr (mod r) on the host for the mcl single-element surface.
//
// mclBnFr values are four 64-bit limbs in Montgomery form (R = 2^256), the layout the device kernels use (k_scalar.hip,
// 8 x u32).  Scalar arithmetic on one element is nanoseconds on a CPU core and microseconds as a GPU round trip, and the
// reference's Fr-heavy code (TPKE/TrustedKeyGen.cs:23-33, ThresholdKeygen/Data/Commitment.cs:23-55, the Lagrange
// coefficients) calls it element by element, so the library keeps it on the host; every group / pairing operation stays
// on the GPU.  CIOS Montgomery product over unsigned __int128 (the compiler emits MULX / ADC on x86-64).
#pragma once
#include <stdint.h>
#include <string.h>

namespace frh {
typedef unsigned __int128 u128;
static const uint64_t R_[4] = {0xffffffff00000001ull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull,
                               0x73eda753299d7d48ull};
static const uint64_t RINV = 0xfffffffeffffffffull;              // -r^-1 mod 2^64
static const uint64_t R2[4] = {0xc999e990f3f29c6dull, 0x2b6cedcb87925c23ull, 0x05d314967254398full,
                               0x0748d9d99f59ff11ull};            // 2^512 mod r
static const uint64_t ONE[4] = {0x00000001fffffffeull, 0x5884b7fa00034802ull, 0x998c4fefecbc4ff5ull,
                                0x1824b159acc5056full};            // 2^256 mod r

inline bool geq(const uint64_t a[4], const uint64_t b[4]) {
    for (int i = 3; i >= 0; i--)
        if (a[i] != b[i]) return a[i] > b[i];
    return true;
}
inline void sub_r(uint64_t a[4]) {
    uint64_t br = 0;
    for (int i = 0; i < 4; i++) {
        u128 d = (u128)a[i] - R_[i] - br;
        a[i] = (uint64_t)d;
        br = (uint64_t)(d >> 64) & 1;
    }
}
inline bool lt_r(const uint64_t a[4]) { return !geq(a, R_); }
inline void add(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) {
    uint64_t t[4], c = 0;
    for (int i = 0; i < 4; i++) {
        u128 s = (u128)a[i] + b[i] + c;
        t[i] = (uint64_t)s;
        c = (uint64_t)(s >> 64);
    }
    if (c || geq(t, R_)) sub_r(t);
    memcpy(r, t, 32);
}
inline void sub(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) {
    uint64_t t[4], br = 0;
    for (int i = 0; i < 4; i++) {
        u128 d = (u128)a[i] - b[i] - br;
        t[i] = (uint64_t)d;
        br = (uint64_t)(d >> 64) & 1;
    }
    if (br) {
        uint64_t c = 0;
        for (int i = 0; i < 4; i++) {
            u128 s = (u128)t[i] + R_[i] + c;
            t[i] = (uint64_t)s;
            c = (uint64_t)(s >> 64);
        }
    }
    memcpy(r, t, 32);
}
inline void neg(uint64_t r[4], const uint64_t a[4]) {
    static const uint64_t z[4] = {0, 0, 0, 0};
    sub(r, z, a);
}
// Montgomery product a b R^-1 mod r (CIOS)
inline void mul(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) {
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; i++) {
        uint64_t c = 0;
        for (int j = 0; j < 4; j++) {
            u128 s = (u128)a[j] * b[i] + t[j] + c;
            t[j] = (uint64_t)s;
            c = (uint64_t)(s >> 64);
        }
        u128 s = (u128)t[4] + c;
        t[4] = (uint64_t)s;
        t[5] = (uint64_t)(s >> 64);
        uint64_t m = t[0] * RINV;
        s = (u128)m * R_[0] + t[0];
        c = (uint64_t)(s >> 64);
        for (int j = 1; j < 4; j++) {
            s = (u128)m * R_[j] + t[j] + c;
            t[j - 1] = (uint64_t)s;
            c = (uint64_t)(s >> 64);
        }
        s = (u128)t[4] + c;
        t[3] = (uint64_t)s;
        t[4] = t[5] + (uint64_t)(s >> 64);
    }
    if (t[4] || geq(t, R_)) sub_r(t);
    memcpy(r, t, 32);
}
inline void from_raw(uint64_t r[4], const uint64_t raw[4]) { mul(r, raw, R2); }   // raw < r
inline void to_raw(uint64_t r[4], const uint64_t a[4]) {
    static const uint64_t one[4] = {1, 0, 0, 0};
    mul(r, a, one);
}
// a^(r-2) (Fermat; 0 -> 0, as mcl's inverse of zero)
inline void inv(uint64_t r[4], const uint64_t a[4]) {
    static const uint64_t E[4] = {0xfffffffeffffffffull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull,
                                  0x73eda753299d7d48ull};       // r - 2
    uint64_t acc[4];
    memcpy(acc, ONE, 32);
    for (int i = 255; i >= 0; i--) {
        mul(acc, acc, acc);
        if ((E[i >> 6] >> (i & 63)) & 1) mul(acc, acc, a);
    }
    memcpy(r, acc, 32);
}
inline bool is_zero(const uint64_t a[4]) { return (a[0] | a[1] | a[2] | a[3]) == 0; }
}  // namespace frh
