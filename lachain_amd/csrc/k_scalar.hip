// lachain_amd/csrc/k_scalar.hip — gfx950 kernels: scalar multiplication, hash-to-G2, TPKE encrypt, HashAndSign.
#include "kcommon.hpp"
#include "lanetab.hpp"

LCB_ASM_LIBRARY(k_scalar)
LCB_TU_CONFIG(k_scalar)

// ================================================================================= scalar multiplication
// out[i] = s_i * P_i (or s_i * generator), serialized; scalars are canonical 32-byte LE (< r checked).  Persistent grids
// with the 4-bit window tables in a workspace slot per lane (lanetab.hpp; round 5: 5.6 / 10.6 KB of scratch before)
template <class F>
DI void scalar_mul_lanes(const uint8_t *pts, int use_gen, const uint8_t *scalars, u32 n, uint8_t *out, uint8_t *ok_out,
                         u32 *ws) {
    constexpr u32 PB = sizeof(F);               // wire bytes: 48 (G1) / 96 (G2), one coordinate
    const u32 gid = blockIdx.x * blockDim.x + threadIdx.x, gsz = gridDim.x * blockDim.x;
    char *slot = lw_slot(ws, LW_WIN4_QUADS(F), gid);
#pragma unroll 1
    for (u32 i = gid; i < n; i += gsz) {
        aff<F> A;
        bool ok = true;
        if constexpr (sizeof(F) == sizeof(fp)) {
            if (use_gen) g1_generator(A);
            else ok = g1_decompress(A, pts + PB * (size_t)i);
        } else {
            if (use_gen) g2_generator(A);
            else ok = g2_decompress(A, pts + PB * (size_t)i);
        }
        fr k;
        const u32 *sw = (const u32 *)(scalars + 32 * (size_t)i);
        for (int j = 0; j < 8; j++) k.v[j] = sw[j];
        ok = ok && fr_raw_lt_r(k);
        jac<F> R;
        k.v[7] &= 0x7fffffffu;                  // 255-bit scalars (k < r is checked above)
        lw_mul_win4(R, slot, A, k.v);
        if constexpr (sizeof(F) == sizeof(fp)) g1_compress_jac(out + PB * (size_t)i, R);
        else g2_compress_jac(out + PB * (size_t)i, R);
        if (ok_out) ok_out[i] = ok;
    }
}
extern "C" __global__ void LCB_BOUNDS k_g1_mul(const uint8_t *pts, int use_gen, const uint8_t *scalars, u32 n,
                                              uint8_t *out, uint8_t *ok_out, u32 *ws) {
    scalar_mul_lanes<fp>(pts, use_gen, scalars, n, out, ok_out, ws);
}
extern "C" __global__ void LCB_BOUNDS k_g2_mul(const uint8_t *pts, int use_gen, const uint8_t *scalars, u32 n,
                                              uint8_t *out, uint8_t *ok_out, u32 *ws) {
    scalar_mul_lanes<fp2>(pts, use_gen, scalars, n, out, ok_out, ws);
}
// H(m_i) for a batch of messages
extern "C" __global__ void LCB_BOUNDS k_g2_hash(const uint8_t *msg_data, const u32 *msg_off, u32 n, uint8_t *out,
                                               uint8_t *ok_out, int orig_cof) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t d[64];
    sha512_2(d, msg_data + msg_off[i], msg_off[i + 1] - msg_off[i], msg_data, 0);
    g2 H;
    bool ok = g2_hash_digest(H, d, orig_cof != 0);
    if (!ok) jac_set_inf(H);
    g2_compress_jac(out + 96 * (size_t)i, H);
    ok_out[i] = ok;
}
// TPKE Encrypt phase 1: U = rG, T = rY; phase 2: W = r H(U || V)
extern "C" __global__ void LCB_BOUNDS k_tpke_encrypt1(const uint8_t *ybytes, const uint8_t *rs, u32 n, uint8_t *u_out,
                                                     uint8_t *t_out, uint8_t *ok_out, u32 *ws) {
    const u32 gid = blockIdx.x * blockDim.x + threadIdx.x, gsz = gridDim.x * blockDim.x;
    char *slot = lw_slot(ws, LW_WIN4_QUADS(fp), gid);
#pragma unroll 1
    for (u32 i = gid; i < n; i += gsz) {
        g1a G, Y;
        g1_generator(G);
        bool ok = g1_decompress(Y, ybytes);
        fr k;
        const u32 *sw = (const u32 *)(rs + 32 * (size_t)i);
        for (int j = 0; j < 8; j++) k.v[j] = sw[j];
        ok = ok && fr_raw_lt_r(k);
        g1 R;
        k.v[7] &= 0x7fffffffu;                  // 255-bit scalars (k < r is checked above)
        lw_mul_win4(R, slot, G, k.v);
        g1_compress_jac(u_out + 48 * (size_t)i, R);
        lw_mul_win4(R, slot, Y, k.v);
        g1_compress_jac(t_out + 48 * (size_t)i, R);
        ok_out[i] = ok;
    }
}
extern "C" __global__ void LCB_BOUNDS k_tpke_encrypt2(const uint8_t *u, const uint8_t *rs, const uint8_t *v_data,
                                                     const u32 *v_off, u32 n, uint8_t *w_out, uint8_t *ok_out,
                                                     int orig_cof) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t d[64];
    sha512_2(d, u + 48 * (size_t)i, 48, v_data + v_off[i], v_off[i + 1] - v_off[i]);
    g2 H, W;
    bool ok = g2_hash_digest(H, d, orig_cof != 0);
    fr k;
    const u32 *sw = (const u32 *)(rs + 32 * (size_t)i);
    for (int j = 0; j < 8; j++) k.v[j] = sw[j];
    jac_mul_bits(W, H, k.v, 255);
    g2_compress_jac(w_out + 96 * (size_t)i, W);
    ok_out[i] = ok;
}
// HashAndSign: sig_i = sk_i * H(m_{msg_idx[i]})
extern "C" __global__ void LCB_BOUNDS k_ts_sign(const uint8_t *sks, const uint8_t *msg_data, const u32 *msg_off,
                                               const u32 *msg_idx, u32 n, uint8_t *out, uint8_t *ok_out,
                                               int orig_cof) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u32 m = msg_idx[i];
    uint8_t d[64];
    sha512_2(d, msg_data + msg_off[m], msg_off[m + 1] - msg_off[m], msg_data, 0);
    g2 H, S;
    bool ok = g2_hash_digest(H, d, orig_cof != 0);
    fr k;
    const u32 *sw = (const u32 *)(sks + 32 * (size_t)i);
    for (int j = 0; j < 8; j++) k.v[j] = sw[j];
    ok = ok && fr_raw_lt_r(k);
    jac_mul_bits(S, H, k.v, 255);
    g2_compress_jac(out + 96 * (size_t)i, S);
    ok_out[i] = ok;
}


// ---------------------------------------------------------------- host launch wrappers
static u32 g_rb_scalar[3];
static u32 scalar_blocks(int which, u32 n) {
    const void *k = which == 1 ? (const void *)k_g1_mul : which == 2 ? (const void *)k_g2_mul : (const void *)k_tpke_encrypt1;
    return lcb_persist_blocks(k, &g_rb_scalar[which - 1], n);
}
// workspace bytes of the scalar-multiplication lanes over n items: 1 = k_g1_mul, 2 = k_g2_mul, 3 = k_tpke_encrypt1
extern "C" size_t lcbk_scalar_ws_bytes(int which, u32 n) {
    return LCB_WS_BYTES(scalar_blocks(which, n), which == 2 ? LW_WIN4_QUADS(fp2) : LW_WIN4_QUADS(fp));
}
extern "C" void lcbk_g1_mul(hipStream_t s, const uint8_t *pts, int use_gen, const uint8_t *scalars, u32 n, uint8_t *out, uint8_t *ok_out, u32 *ws) {
    dim3 grid(scalar_blocks(1, n));
    LCB_LAUNCH(k_g1_mul, pts, use_gen, scalars, n, out, ok_out, ws);
}
extern "C" void lcbk_g2_mul(hipStream_t s, const uint8_t *pts, int use_gen, const uint8_t *scalars, u32 n, uint8_t *out, uint8_t *ok_out, u32 *ws) {
    dim3 grid(scalar_blocks(2, n));
    LCB_LAUNCH(k_g2_mul, pts, use_gen, scalars, n, out, ok_out, ws);
}
extern "C" void lcbk_g2_hash(dim3 grid, hipStream_t s, const uint8_t *msg_data, const u32 *msg_off, u32 n, uint8_t *out, uint8_t *ok_out, int orig_cof) {
    LCB_LAUNCH(k_g2_hash, msg_data, msg_off, n, out, ok_out, orig_cof);
}
extern "C" void lcbk_tpke_encrypt1(hipStream_t s, const uint8_t *ybytes, const uint8_t *rs, u32 n, uint8_t *u_out, uint8_t *t_out, uint8_t *ok_out, u32 *ws) {
    dim3 grid(scalar_blocks(3, n));
    LCB_LAUNCH(k_tpke_encrypt1, ybytes, rs, n, u_out, t_out, ok_out, ws);
}
extern "C" void lcbk_tpke_encrypt2(dim3 grid, hipStream_t s, const uint8_t *u, const uint8_t *rs, const uint8_t *v_data, const u32 *v_off, u32 n, uint8_t *w_out, uint8_t *ok_out, int orig_cof) {
    LCB_LAUNCH(k_tpke_encrypt2, u, rs, v_data, v_off, n, w_out, ok_out, orig_cof);
}
extern "C" void lcbk_ts_sign(dim3 grid, hipStream_t s, const uint8_t *sks, const uint8_t *msg_data, const u32 *msg_off, const u32 *msg_idx, u32 n, uint8_t *out, uint8_t *ok_out, int orig_cof) {
    LCB_LAUNCH(k_ts_sign, sks, msg_data, msg_off, msg_idx, n, out, ok_out, orig_cof);
}
