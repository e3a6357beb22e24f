// lachain_amd/csrc/k_dkg.hip — gfx950 kernels for the trustless-DKG G1 work.
//
// Reference: Commitment of a symmetric bivariate polynomial f(x, y) = sum_{i,j<=D} c_{Index(i,j)} x^i y^j as G1 points
// C_k = c_k G (src/Lachain.Consensus/ThresholdKeygen/Data/Commitment.cs:14-21, Index :55-59), evaluated per received
// value  Evaluate(x, y) = sum_{i,j} C_{Index(i,j)} x^i y^j        (Commitment.cs:23-37, TrustlessKeygen.cs:150-152)
// and per commit  Evaluate(x) = row_i = sum_j C_{Index(i,j)} x^j   (Commitment.cs:39-53, TrustlessKeygen.cs:90-94)
// and TryGetKeys' EvaluatePolynomial over G1 at i = 0..N            (TrustlessKeygen.cs:172-174).
// The reference multiplies every coefficient by full Fr powers of x and y ((D+1)^2 255-bit scalar multiplications per
// Evaluate(x, y)); x and y are small protocol indices (player index + 1), so Horner's rule in x then y computes the
// same G1 element with (D+1) small-integer multiplications per output: for coefficients in G1 (every honest
// commitment: C_k = c_k G), sum_i C x^i y^j with the powers reduced mod r equals the Horner value exactly.
// G1.FromBytes accepts on-curve points outside G1 and TrustlessKeygen never calls Commitment.IsValid,
// so a Byzantine dealer can add a cofactor-torsion component, for which the reduction mod r matters: every
// coefficient is tested for G1 membership (k_g1_subgroup_any) and a batch with one outside G1 is evaluated in the
// reference's own form, [y^j mod r]([x^i mod r] C_Index(i,j)) (k_dkg_exact_terms / k_dkg_exact_combine).
#include "kcommon.hpp"

LCB_ASM_LIBRARY(k_dkg)
LCB_TU_CONFIG(k_dkg)

DI u32 dkg_index(u32 i, u32 j) {   // Commitment.Index: symmetric, i <= j
    if (i > j) { u32 t = i; i = j; j = t; }
    return i * (i + 1) / 2 + j;
}

// G1 membership: phi(P) = [z^2 - 1] P (phi(x, y) = (beta x, y), the endomorphism k_batch.hip uses), i.e.
// [z^2] P == P + phi(P) = (beta^2 x, -y).  Detects a component of every prime factor of the G1 cofactor
// (tests/test_gpu_dkg.py checks it against the oracle's [r] P == O).
DI bool g1_in_subgroup(const g1a &P) {
    if (P.inf) return true;
    g1 Q;
    jac_from_aff(Q, P);
    jac_mul_u64_inl(Q, Q, LCB_Z_ABS);
    jac_mul_u64_inl(Q, Q, LCB_Z_ABS);                  // [z^2] P (z^2 = |z|^2)
    if (jac_is_inf(Q)) return false;
    fp beta, b2x, ny, z2, z3, t;
    fp_load_const(beta, LCB_G1_BETA);
    fp_sqr(b2x, beta);
    fp_mul(b2x, b2x, P.x);
    fp_neg(ny, P.y);
    fp_sqr(z2, Q.z);
    fp_mul(z3, z2, Q.z);
    fp_mul(t, b2x, z2);
    if (!fp_eq(t, Q.x)) return false;
    fp_mul(t, ny, z3);
    return fp_eq(t, Q.y);
}
// any decodable point of pts outside G1 -> *any = 1
extern "C" __global__ void LCB_BOUNDS k_g1_subgroup_any(const g1a_st *pts, u32 n, u32 *any) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    g1a_st s = pts[i];
    g1a a;
    st_to_g1a(a, s);
    if (s.ok && !g1_in_subgroup(a)) atomicOr(any, 1u);
}
// Fr.FromInt(x)^e as a canonical 256-bit integer (Fr.FromInt of a negative x is r - |x|)
DI void fr_int_pow(u32 out[8], int x, u32 e) {
    fr b, acc;
    u32 a = x < 0 ? (u32)(-(long long)x) : (u32)x;
    for (int k = 0; k < 8; k++) b.v[k] = k == 0 ? a : 0u;
    if (x < 0) {                                       // r - |x|
        u32 br = 0;
        for (int k = 0; k < 8; k++) {
            u64 d = (u64)LCB_R[k] - b.v[k] - br;
            b.v[k] = (u32)d;
            br = (u32)(d >> 32) & 1;
        }
    }
    fr_from_raw(b, b);
    acc = fr_one();
    for (int k = 31; k >= 0; k--) {
        fr_mul(acc, acc, acc);
        if ((e >> k) & 1) fr_mul(acc, acc, b);
    }
    fr_to_raw(acc, acc);
    for (int k = 0; k < 8; k++) out[k] = acc.v[k];
}
// the reference's terms for commitments with coefficients outside G1: term (q, i, j) = [x_q^j mod r] C_Index(i,j)
// (Commitment.Evaluate(x), Commitment.cs:39-53); a reduction over j gives the rows
extern "C" __global__ void LCB_BOUNDS k_dkg_exact_terms(const g1a_st *coef, u32 n_coef, u32 n_comm, u32 D,
                                                       const u32 *comm, const int *xs, u32 n_q, g1 *terms,
                                                       uint8_t *ok_out) {
    const size_t D1 = (size_t)D + 1;
    size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)n_q * D1 * D1) return;
    u32 q = (u32)(t / (D1 * D1)), rem = (u32)(t % (D1 * D1)), i = rem / (u32)D1, j = rem % (u32)D1, c = comm[q];
    bool ok = c < n_comm;
    g1a_st s = coef[(size_t)(ok ? c : 0) * n_coef + dkg_index(i, j)];
    ok = ok && s.ok;
    u32 k[8];
    fr_int_pow(k, xs[q], j);
    g1a a;
    st_to_g1a(a, s);
    g1 r;
    jac_mul_aff(r, a, k, 256);
    terms[t] = r;
    ok_out[t] = ok;
}
// out[g] = AND of in[g * group .. (g + 1) * group)
extern "C" __global__ void LCB_BOUNDS k_and_groups(const uint8_t *in, u32 n_out, u32 group, uint8_t *out) {
    u32 g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_out) return;
    uint8_t a = 1;
    for (u32 k = 0; k < group; k++) a &= in[(size_t)g * group + k] != 0;
    out[g] = a;
}
// Evaluate(x, y) = sum_j [y^j mod r] row_j(x) (Commitment.cs:23-37 with Index symmetric): term (q, j)
extern "C" __global__ void LCB_BOUNDS k_dkg_exact_combine(const g1 *rows, u32 D, const u32 *row, const int *ys, u32 n_q,
                                                         g1 *terms) {
    const u32 D1 = D + 1;
    size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)n_q * D1) return;
    u32 q = (u32)(t / D1), j = (u32)(t % D1);
    u32 k[8];
    fr_int_pow(k, ys[q], j);
    g1 r;
    jac_mul_bits(r, rows[(size_t)row[q] * D1 + j], k, 256);
    terms[t] = r;
}

// acc <- k * acc for a 32-bit signed integer k (double-and-add over |k|, negated for k < 0)
DI void g1_mul_small(g1 &acc, int k) {
    u32 a = k < 0 ? (u32)(-(long long)k) : (u32)k;
    g1 r;
    jac_set_inf(r);
    if (a != 0) {
        int top = 31 - __clz(a);
        r = acc;
        for (int b = top - 1; b >= 0; b--) {
            grp_dbl(r, r);
            if ((a >> b) & 1) grp_add(r, r, acc);
        }
    }
    if (k < 0) jac_neg(r, r);
    acc = r;
}

// rows[t] for t = q * (D+1) + i: Evaluate(x_q) row i of commitment comm[q] = sum_j C_{Index(i,j)} x^j (Horner in x)
extern "C" __global__ void LCB_BOUNDS k_dkg_rows(const g1a_st *coef, u32 n_coef, u32 n_comm, u32 D, const u32 *comm,
                                                const int *xs, u32 n_q, g1 *rows, uint8_t *ok_out) {
    u32 t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_q * (D + 1)) return;
    u32 q = t / (D + 1), i = t % (D + 1), c = comm[q];
    bool ok = c < n_comm;
    const g1a_st *C = coef + (size_t)(ok ? c : 0) * n_coef;
    int x = xs[q];
    g1 acc;
    jac_set_inf(acc);
    for (int j = (int)D; j >= 0; j--) {
        g1_mul_small(acc, x);
        g1a_st s = C[dkg_index(i, (u32)j)];
        ok = ok && s.ok;
        if (!s.inf) grp_madd(acc, acc, s.x, s.y);
    }
    rows[t] = acc;
    if (ok_out) ok_out[t] = ok;
}

// out[q] = sum_j R_j y_q^j over the (D+1)-point row rows[row[q] * (D+1) ..] (Horner in y); status from the row's lanes
// (neg_exact: a negative y multiplies by r - |y| — Fr.FromInt's value — instead of -|y|, which differs for points
// outside G1; mcl's EvaluatePolynomial is this Horner rule with an Fr x)
extern "C" __global__ void LCB_BOUNDS k_dkg_horner(const g1 *rows, const uint8_t *row_ok, u32 D, const u32 *row,
                                                  const int *ys, u32 n_q, uint8_t *out48, uint8_t *status,
                                                  u32 neg_exact) {
    u32 q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n_q) return;
    const g1 *R = rows + (size_t)row[q] * (D + 1);
    const uint8_t *rok = row_ok + (size_t)row[q] * (D + 1);
    int y = ys[q];
    bool ok = true;
    g1 acc;
    jac_set_inf(acc);
    u32 ky[8];
    const bool full = neg_exact && y < 0;
    if (full) fr_int_pow(ky, y, 1);
    for (int j = (int)D; j >= 0; j--) {
        if (full) jac_mul_bits(acc, acc, ky, 256);
        else g1_mul_small(acc, y);
        grp_add(acc, acc, R[j]);
        ok = ok && rok[j];
    }
    if (!ok) jac_set_inf(acc);
    g1_compress_jac(out48 + 48 * (size_t)q, acc);
    status[q] = ok;
}

// affine records -> Jacobian (one row of polynomial coefficients for k_dkg_horner)
extern "C" __global__ void LCB_BOUNDS k_g1a_to_jac(const g1a_st *in, u32 n, g1 *out, uint8_t *ok) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    g1a_st s = in[i];
    g1a a;
    st_to_g1a(a, s);
    g1 r;
    jac_from_aff(r, a);
    out[i] = r;
    ok[i] = s.ok;
}

// ---------------------------------------------------------------- host launch wrappers
extern "C" void lcbk_dkg_rows(dim3 grid, hipStream_t s, const void *coef, u32 n_coef, u32 n_comm, u32 D, const u32 *comm,
                              const int *xs, u32 n_q, void *rows, uint8_t *ok_out) {
    LCB_LAUNCH(k_dkg_rows, (const g1a_st *)coef, n_coef, n_comm, D, comm, xs, n_q, (g1 *)rows, ok_out);
}
extern "C" void lcbk_dkg_horner(dim3 grid, hipStream_t s, const void *rows, const uint8_t *row_ok, u32 D, const u32 *row,
                                const int *ys, u32 n_q, uint8_t *out48, uint8_t *status, u32 neg_exact) {
    LCB_LAUNCH(k_dkg_horner, (const g1 *)rows, row_ok, D, row, ys, n_q, out48, status, neg_exact);
}
extern "C" void lcbk_and_groups(hipStream_t s, const uint8_t *in, u32 n_out, u32 group, uint8_t *out) {
    dim3 grid((n_out + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_and_groups, in, n_out, group, out);
}
extern "C" void lcbk_g1_subgroup_any(hipStream_t s, const void *pts, u32 n, u32 *any) {
    dim3 grid((n + LCB_BLOCK - 1) / LCB_BLOCK);
    LCB_LAUNCH(k_g1_subgroup_any, (const g1a_st *)pts, n, any);
}
extern "C" void lcbk_dkg_exact_terms(hipStream_t s, const void *coef, u32 n_coef, u32 n_comm, u32 D, const u32 *comm,
                                     const int *xs, u32 n_q, void *terms, uint8_t *ok_out) {
    const size_t n = (size_t)n_q * (D + 1) * (D + 1);
    dim3 grid((u32)((n + LCB_BLOCK - 1) / LCB_BLOCK));
    LCB_LAUNCH(k_dkg_exact_terms, (const g1a_st *)coef, n_coef, n_comm, D, comm, xs, n_q, (g1 *)terms, ok_out);
}
extern "C" void lcbk_dkg_exact_combine(hipStream_t s, const void *rows, u32 D, const u32 *row, const int *ys, u32 n_q,
                                       void *terms) {
    const size_t n = (size_t)n_q * (D + 1);
    dim3 grid((u32)((n + LCB_BLOCK - 1) / LCB_BLOCK));
    LCB_LAUNCH(k_dkg_exact_combine, (const g1 *)rows, D, row, ys, n_q, (g1 *)terms);
}
extern "C" void lcbk_g1a_to_jac(dim3 grid, hipStream_t s, const void *in, u32 n, void *out, uint8_t *ok) {
    LCB_LAUNCH(k_g1a_to_jac, (const g1a_st *)in, n, (g1 *)out, ok);
}
