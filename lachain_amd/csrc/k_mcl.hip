// lachain_amd/csrc/k_mcl.hip — gfx950 kernels behind the mcl single-element surface (include/lachain_bls.h, SURVEY.md
// §8b): the pairing on the cooperative kernels, G1 multi-scalar products, Horner evaluation with an Fr point and the
// conversion of mcl's Jacobian records to wire bytes for the batched Lagrange path.  mcl's G1 / G2 records are the
// device's own Jacobian layout (x, y, z in Montgomery form, 12 x u32 per Fp), scalars arrive as canonical integers.
#include "coop.hpp"
#include "lanetab.hpp"

LCB_ASM_LIBRARY(k_mcl)
LCB_TU_CONFIG(k_mcl)

// the line-set layout the host stages for mclBn_pairing (launch.h LCB_LS_POINT_WORD, LCB_LINESET_BYTES)
static_assert(LCB_LS_POINT == 6528 && LCB_LS_FLAG == 6528 + 48 && LCB_LINESET_WORDS * 4 == 26368, "line-set layout");

// terms[i] = [k_i] P_i for n G1 points (Jacobian) and canonical 256-bit scalars: the 4-bit windowed ladder over the
// point's affine table, exact for every on-curve input (persistent grid, the table in a workspace slot: lanetab.hpp)
extern "C" __global__ void LCB_BOUNDS k_mcl_g1_terms(const g1 *pts, const fr *scal, u32 n, g1 *terms, u32 *ws) {
    const u32 gid = blockIdx.x * blockDim.x + threadIdx.x, gsz = gridDim.x * blockDim.x;
    char *slot = lw_slot(ws, LW_WIN4_QUADS(fp), gid);
#pragma unroll 1
    for (u32 i = gid; i < n; i += gsz) {
        g1a a;
        g1_jac_to_aff_g(a, pts[i]);                    // binary-GCD inversion
        fr k = scal[i];
        g1 r;
        lw_mul_win4(r, slot, a, k.v);
        terms[i] = r;
    }
}

// terms[i] = [e_i] P_i with 384-bit scalars (12 words each): mclBn_G1EvaluatePolynomial's e_i = x^i mod #E(Fp), so
// sum_i [e_i] c_i is the Horner value sum_i [x^i] c_i for every on-curve coefficient (lcb_host.cpp eval_poly)
extern "C" __global__ void LCB_BOUNDS k_mcl_g1_terms_wide(const g1 *pts, const u32 *scal, u32 n, g1 *terms, u32 *ws) {
    const u32 gid = blockIdx.x * blockDim.x + threadIdx.x, gsz = gridDim.x * blockDim.x;
    char *slot = lw_slot(ws, LW_WIN4_QUADS(fp), gid);
#pragma unroll 1
    for (u32 i = gid; i < n; i += gsz) {
        g1a a;
        g1_jac_to_aff_g(a, pts[i]);
        u32 k[12];
#pragma unroll
        for (int j = 0; j < 12; j++) k[j] = scal[12 * (size_t)i + j];
        g1 r;
        lw_mul_win4<fp, 12>(r, slot, a, k);
        terms[i] = r;
    }
}

// Horner with an Fr point x (mcl evaluatePolynomial: y = c[n-1]; y = y x + c[i]), one lane; g = 1 (G1) or 2 (G2)
extern "C" __global__ void LCB_BOUNDS k_mcl_horner(int g, const u32 *coef, u32 n, const fr *x_raw, u32 *out) {
    if (blockIdx.x || threadIdx.x) return;
    const fr x = *x_raw;
    if (g == 1) {
        const g1 *c = (const g1 *)coef;
        g1 acc = c[n - 1];
        for (u32 i = n - 1; i-- > 0;) {
            jac_mul_bits(acc, acc, x.v, 255);
            grp_add(acc, acc, c[i]);
        }
        *(g1 *)out = acc;
    } else {
        const g2 *c = (const g2 *)coef;
        g2 acc = c[n - 1];
        for (u32 i = n - 1; i-- > 0;) {
            jac_mul_bits(acc, acc, x.v, 255);
            grp_add(acc, acc, c[i]);
        }
        *(g2 *)out = acc;
    }
}

// out = sum of n G1 Jacobian records, one lane (mulVec's final sum for n <= one block; larger n reduce by blocks first)
extern "C" __global__ void LCB_BOUNDS k_mcl_g1_sum(const g1 *in, u32 n, g1 *out) {
    if (blockIdx.x || threadIdx.x) return;
    g1 acc;
    jac_set_inf(acc);
    for (u32 i = 0; i < n; i++) grp_add(acc, acc, in[i]);
    *out = acc;
}

// wire encodings -> mcl Jacobian records (z = 1, or the point at infinity), ok[i] = the encoding decoded
extern "C" __global__ void LCB_BOUNDS k_mcl_from_bytes(int g, const uint8_t *in, u32 n, u32 *out, uint8_t *ok) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (g == 1) {
        g1a a;
        ok[i] = g1_decompress(a, in + 48 * (size_t)i);
        jac_from_aff(((g1 *)out)[i], a);
    } else {
        g2a a;
        ok[i] = g2_decompress(a, in + 96 * (size_t)i);
        jac_from_aff(((g2 *)out)[i], a);
    }
}

// mcl Jacobian records -> 48 / 96-byte wire encodings (g = 1 / 2)
extern "C" __global__ void LCB_BOUNDS k_mcl_to_bytes(int g, const u32 *in, u32 n, uint8_t *out) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (g == 1) g1_compress_jac(out + 48 * (size_t)i, ((const g1 *)in)[i]);
    else g2_compress_jac(out + 96 * (size_t)i, ((const g2 *)in)[i]);
}

// ---------------------------------------------------------------- host launch wrappers
static u32 g_rb_terms;
extern "C" size_t lcbk_mcl_terms_ws_bytes(u32 n) {
    return LCB_WS_BYTES(lcb_persist_blocks((const void *)k_mcl_g1_terms, &g_rb_terms, n), LW_WIN4_QUADS(fp));
}
extern "C" void lcbk_mcl_g1_terms(hipStream_t s, const void *pts, const void *scal, u32 n, void *terms, u32 *ws) {
    dim3 grid(lcb_persist_blocks((const void *)k_mcl_g1_terms, &g_rb_terms, n));
    LCB_LAUNCH(k_mcl_g1_terms, (const g1 *)pts, (const fr *)scal, n, (g1 *)terms, ws);
}
static u32 g_rb_terms_wide;
extern "C" size_t lcbk_mcl_terms_wide_ws_bytes(u32 n) {
    return LCB_WS_BYTES(lcb_persist_blocks((const void *)k_mcl_g1_terms_wide, &g_rb_terms_wide, n), LW_WIN4_QUADS(fp));
}
extern "C" void lcbk_mcl_g1_terms_wide(hipStream_t s, const void *pts, const u32 *scal, u32 n, void *terms, u32 *ws) {
    dim3 grid(lcb_persist_blocks((const void *)k_mcl_g1_terms_wide, &g_rb_terms_wide, n));
    LCB_LAUNCH(k_mcl_g1_terms_wide, (const g1 *)pts, scal, n, (g1 *)terms, ws);
}
extern "C" void lcbk_mcl_horner(hipStream_t s, int g, const u32 *coef, u32 n, const void *x_raw, u32 *out) {
    dim3 grid(1);
    LCB_LAUNCH(k_mcl_horner, g, coef, n, (const fr *)x_raw, out);
}
extern "C" void lcbk_mcl_g1_sum(hipStream_t s, const void *in, u32 n, void *out) {
    dim3 grid(1);
    LCB_LAUNCH(k_mcl_g1_sum, (const g1 *)in, n, (g1 *)out);
}
extern "C" void lcbk_mcl_from_bytes(hipStream_t s, int g, const uint8_t *in, u32 n, u32 *out, uint8_t *ok) {
    dim3 grid((n + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_mcl_from_bytes, g, in, n, out, ok);
}
extern "C" void lcbk_mcl_to_bytes(hipStream_t s, int g, const u32 *in, u32 n, uint8_t *out) {
    dim3 grid((n + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_mcl_to_bytes, g, in, n, out);
}
