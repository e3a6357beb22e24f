// lachain_amd/csrc/k_ops.hip — gfx950 kernels: single mcl-shaped operations.
#include "kcommon.hpp"

LCB_ASM_LIBRARY(k_ops)
LCB_TU_CONFIG(k_ops)

// ================================================================================= single operations
DI bool g1_on_curve(const g1 &p) { // Jacobian: Y^2 = X^3 + 4 Z^6
    if (jac_is_inf(p)) return true;
    fp l, r, z2, z6, b;
    fp_sqr(l, p.y);
    fp_sqr(r, p.x);
    fp_mul(r, r, p.x);
    fp_sqr(z2, p.z);
    fp_mul(z6, z2, z2);
    fp_mul(z6, z6, z2);
    fp_load_const(b, LCB_B1);
    fp_mul(z6, z6, b);
    fp_add(r, r, z6);
    return fp_eq(l, r);
}
DI bool g2_on_curve(const g2 &p) {
    if (jac_is_inf(p)) return true;
    fp2 l, r, z2, z6, b;
    fp2_sqr(l, p.y);
    fp2_sqr(r, p.x);
    fp2_mul(r, r, p.x);
    fp2_sqr(z2, p.z);
    fp2_mul(z6, z2, z2);
    fp2_mul(z6, z6, z2);
    fp2_load_const(b, LCB_B2);
    fp2_mul(z6, z6, b);
    fp2_add(r, r, z6);
    return fp2_eq(l, r);
}
DI bool fp_words_lt_p(const fp &a) { return fp_raw_lt_p(a); }
template <class G> DI bool jac_eq(const G &p, const G &q) {
    bool pi = jac_is_inf(p), qi = jac_is_inf(q);
    if (pi || qi) return pi && qi;
    // X1 Z2^2 == X2 Z1^2 and Y1 Z2^3 == Y2 Z1^3
    decltype(p.x) z1z1, z2z2, u1, u2, s1, s2;
    f_sqr(z1z1, p.z);
    f_sqr(z2z2, q.z);
    f_mul(u1, p.x, z2z2);
    f_mul(u2, q.x, z1z1);
    f_mul(s1, p.y, q.z);
    f_mul(s1, s1, z2z2);
    f_mul(s2, q.y, p.z);
    f_mul(s2, s2, z1z1);
    return f_eq(u1, u2) && f_eq(s1, s2);
}
// One lane executes one mcl-shaped operation on mcl-layout structs held in `io` (u32 words).  One kernel per operation
// family (round 5: the single switch kernel inlined every family into one 512-register frame with 8.4 KB of scratch per
// lane); lcbk_op picks the family.
//
// Fr, G1, G2 (group operations, (de)serialization, hash to G2, generators)
extern "C" __global__ void LCB_BOUNDS k_op_grp(int op, u32 *io, int orig_cof) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    switch (op) {
    // ---- Fr: io[0..8) = out, io[8..16) = x, io[16..24) = y (mclBnFr layout = 8 u32 Montgomery)
    case OP_FR_FROM_RAW: { fr x = *(fr *)(io + 8); if (!fr_raw_lt_r(x)) { io[24] = 0; break; } fr_from_raw(*(fr *)io, x); io[24] = 1; break; }
    case OP_FR_TO_RAW: { fr x = *(fr *)(io + 8); fr_to_raw(*(fr *)io, x); break; }
    case OP_FR_ADD: { fr x = *(fr *)(io + 8), y = *(fr *)(io + 16); fr_add(*(fr *)io, x, y); break; }
    case OP_FR_SUB: { fr x = *(fr *)(io + 8), y = *(fr *)(io + 16); fr_sub(*(fr *)io, x, y); break; }
    case OP_FR_MUL: { fr x = *(fr *)(io + 8), y = *(fr *)(io + 16); fr_mul(*(fr *)io, x, y); break; }
    case OP_FR_INV: { fr x = *(fr *)(io + 8); fr_inv(*(fr *)io, x); break; }
    case OP_FR_NEG: { fr x = *(fr *)(io + 8), z; for (int j = 0; j < 8; j++) z.v[j] = 0; fr_sub(*(fr *)io, z, x); break; }
    // ---- G1: io[0..36) out (Jacobian), io[36..72) x, io[72..108) y, io[108..116) Fr, io[116..128) bytes, io[128] flag
    case OP_G1_DESER: {
        g1a a; bool ok = g1_decompress(a, (const uint8_t *)(io + 116));
        g1 p; jac_from_aff(p, a); *(g1 *)io = p; io[128] = ok; break;
    }
    case OP_G1_SER: { g1 p = *(g1 *)(io + 36); g1_compress_jac((uint8_t *)(io + 116), p); break; }
    case OP_G1_ADD: { g1 p = *(g1 *)(io + 36), q = *(g1 *)(io + 72); jac_add(*(g1 *)io, p, q); break; }
    case OP_G1_DBL: { g1 p = *(g1 *)(io + 36); jac_dbl(*(g1 *)io, p); break; }
    case OP_G1_NEG: { g1 p = *(g1 *)(io + 36); jac_neg(*(g1 *)io, p); break; }
    case OP_G1_MUL: {
        g1 p = *(g1 *)(io + 36); fr k = *(fr *)(io + 108), kr; fr_to_raw(kr, k);
        jac_mul_bits(*(g1 *)io, p, kr.v, 255); break;
    }
    case OP_G1_EQ: { g1 p = *(g1 *)(io + 36), q = *(g1 *)(io + 72); io[128] = jac_eq(p, q); break; }
    case OP_G1_VALID: {
        g1 p = *(g1 *)(io + 36);
        io[128] = fp_words_lt_p(p.x) && fp_words_lt_p(p.y) && fp_words_lt_p(p.z) && g1_on_curve(p); break;
    }
    case OP_G1_NORM: {
        g1 p = *(g1 *)(io + 36); g1a a; g1_jac_to_aff_g(a, p); g1 q; jac_from_aff(q, a);
        if (a.inf) jac_set_inf(q); *(g1 *)io = q; break;
    }
    // ---- G2: io[0..72) out, io[72..144) x, io[144..216) y, io[216..224) Fr, io[224..248) bytes, io[248] flag
    case OP_G2_DESER: {
        g2a a; bool ok = g2_decompress(a, (const uint8_t *)(io + 224));
        g2 p; jac_from_aff(p, a); *(g2 *)io = p; io[248] = ok; break;
    }
    case OP_G2_SER: { g2 p = *(g2 *)(io + 72); g2_compress_jac((uint8_t *)(io + 224), p); break; }
    case OP_G2_ADD: { g2 p = *(g2 *)(io + 72), q = *(g2 *)(io + 144); jac_add(*(g2 *)io, p, q); break; }
    case OP_G2_DBL: { g2 p = *(g2 *)(io + 72); jac_dbl(*(g2 *)io, p); break; }
    case OP_G2_NEG: { g2 p = *(g2 *)(io + 72); jac_neg(*(g2 *)io, p); break; }
    case OP_G2_MUL: {
        g2 p = *(g2 *)(io + 72); fr k = *(fr *)(io + 216), kr; fr_to_raw(kr, k);
        jac_mul_bits(*(g2 *)io, p, kr.v, 255); break;
    }
    case OP_G2_EQ: { g2 p = *(g2 *)(io + 72), q = *(g2 *)(io + 144); io[248] = jac_eq(p, q); break; }
    case OP_G2_VALID: {
        g2 p = *(g2 *)(io + 72);
        io[248] = fp_words_lt_p(p.x.a) && fp_words_lt_p(p.x.b) && fp_words_lt_p(p.y.a) && fp_words_lt_p(p.y.b) &&
                  fp_words_lt_p(p.z.a) && fp_words_lt_p(p.z.b) && g2_on_curve(p); break;
    }
    case OP_G2_NORM: {
        g2 p = *(g2 *)(io + 72); g2a a; g2_jac_to_aff_g(a, p); g2 q; jac_from_aff(q, a);
        if (a.inf) jac_set_inf(q); *(g2 *)io = q; break;
    }
    case OP_G2_HASH: {
        // io[250] = message length, message bytes at io + 256 (digest computed here)
        uint8_t d[64];
        sha512_2(d, (const uint8_t *)(io + 256), io[250], (const uint8_t *)(io + 256), 0);
        g2 H; bool ok = g2_hash_digest(H, d, orig_cof != 0);
        if (!ok) jac_set_inf(H); *(g2 *)io = H; io[248] = ok; break;
    }
    case OP_G1_GEN: { g1a a; g1_generator(a); jac_from_aff(*(g1 *)io, a); break; }
    case OP_G2_GEN: { g2a a; g2_generator(a); jac_from_aff(*(g2 *)io, a); break; }
    default: break;
    }
}
// the Miller loop (and the pairing) of one pair
extern "C" __global__ void LCB_BOUNDS k_op_pair(int op, u32 *io, int orig_cof) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    switch (op) {
    // ---- pairing / GT: io[0..144) out GT, io[144..180) G1, io[180..252) G2, io[252..396) GT a, io[396..540) GT b,
    //      io[540..548) Fr, io[548] flag
    case OP_PAIRING:
    case OP_MILLER: {
        g1 p = *(g1 *)(io + 144); g2 q = *(g2 *)(io + 180);
        g1a pa; g2a qa; jac_to_aff(pa, p); jac_to_aff(qa, q);
        LinesOnTheFly s; s.init(qa);
        fp12 f; miller1(f, s, pa);
        if (op == OP_PAIRING) { fp12 e; final_exp(e, f); *(fp12 *)io = e; }
        else *(fp12 *)io = f;
        break;
    }
    default: break;
    }
}
// GT: final exponentiation, product, power, comparison, (de)serialization
extern "C" __global__ void LCB_BOUNDS k_op_gt(int op, u32 *io, int orig_cof) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    switch (op) {
    case OP_FINAL_EXP: { fp12 a = *(fp12 *)(io + 252); fp12 e; final_exp(e, a); *(fp12 *)io = e; break; }
    case OP_GT_MUL: { fp12 a = *(fp12 *)(io + 252), b = *(fp12 *)(io + 396); fp12_mul(*(fp12 *)io, a, b); break; }
    case OP_GT_POW: {
        fp12 a = *(fp12 *)(io + 252); fr k = *(fr *)(io + 540), kr; fr_to_raw(kr, k);
        fp12 acc = fp12_one();
        for (int i = 254; i >= 0; i--) {
            fp12_sqr(acc, acc);
            if ((kr.v[i >> 5] >> (i & 31)) & 1) fp12_mul(acc, acc, a);
        }
        *(fp12 *)io = acc; break;
    }
    case OP_GT_EQ: {
        fp12 a = *(fp12 *)(io + 252), b = *(fp12 *)(io + 396);
        const fp *x = &a.c0.c0.a, *y = &b.c0.c0.a; bool eq = true;
        for (int i = 0; i < 12; i++) eq = eq && fp_eq(x[i], y[i]);
        io[548] = eq; break;
    }
    case OP_GT_SER: { // canonical raw limbs of the 12 Fp into io[0..144)
        fp12 a = *(fp12 *)(io + 252); fp *x = &a.c0.c0.a;
        for (int i = 0; i < 12; i++) { fp r; fp_to_raw(r, x[i]); *(fp *)(io + 12 * i) = r; }
        break;
    }
    case OP_GT_DESER: { // raw limbs io[252..396) -> Montgomery io[0..144), flag = all < p
        fp *x = (fp *)(io + 252); bool ok = true;
        for (int i = 0; i < 12; i++) { ok = ok && fp_raw_lt_p(x[i]); fp m; fp_from_raw(m, x[i]); *(fp *)(io + 12 * i) = m; }
        io[548] = ok; break;
    }
    default: break;
    }
}
// tower routines on raw GT words (tools/debug)
extern "C" __global__ void LCB_BOUNDS k_op_debug(int op, u32 *io, int orig_cof) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    switch (op) {
    case OP_DEBUG_FP12: {
        fp12 a = *(fp12 *)(io + 252), r = a;
        switch (io[548]) {
        case 0: fp12_inv_n(r, a); break;
        case 1: fp12_cyc_sqr_n(r, a); break;
        case 2: fp12_frob1_n(r, a); break;
        case 3: fp12_frob2_n(r, a); break;
        case 4: fp12_frob3_n(r, a); break;
        case 5: fe_easy(r, a); break;
        case 6: cyc_pow_z(r, a); break;
        case 7: fp12_sqr_n(r, a); break;
        case 8: fp6_inv(r.c0, a.c0); break;
        case 9: fp2_inv_n(r.c0.c0, a.c0.c0); break;
        case 10: fp12_conj(r, a); break;
        case 11: fe_hard(r, a); break;
        case 12: {                                 // Legendre symbols of the 12 Fp words: binary (fp_jacobi), exponent
            u32 *w = (u32 *)&r;
            const fp *xs = (const fp *)&a;
#pragma unroll 1
            for (int k = 0; k < 12; k++) {
                fp t;
                fp_pow_const(t, xs[k], 2);
                w[2 * k] = (u32)fp_jacobi(xs[k]);
                w[2 * k + 1] = fp_is_zero(xs[k]) ? 0u : (fp_eq(t, fp_one()) ? 1u : 0xffffffffu);
            }
            break;
        }
        default: break;
        }
        *(fp12 *)io = r;
        break;
    }
    default: break;
    }
}

// ---------------------------------------------------------------- host launch wrappers
extern "C" void lcbk_op(dim3 grid, hipStream_t s, int op, u32 *io, int orig_cof) {
    if (op == OP_PAIRING || op == OP_MILLER) LCB_LAUNCH(k_op_pair, op, io, orig_cof);
    else if (op >= OP_FINAL_EXP && op <= OP_GT_DESER) LCB_LAUNCH(k_op_gt, op, io, orig_cof);
    else if (op == OP_DEBUG_FP12) LCB_LAUNCH(k_op_debug, op, io, orig_cof);
    else LCB_LAUNCH(k_op_grp, op, io, orig_cof);
}
