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
#include "kcommon.hpp"

LCB_ASM_LIBRARY(k_dkg)

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
DI u32 dkg_index(u32 i, u32 j) {   // Commitment.Index: symmetric, i <= j
    if (i > j) { u32 t = i; i = j; j = t; }
    return i * (i + 1) / 2 + j;
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
extern "C" __global__ void LCB_BOUNDS k_dkg_horner(const g1 *rows, const uint8_t *row_ok, u32 D, const u32 *row,
                                                  const int *ys, u32 n_q, uint8_t *out48, uint8_t *status) {
    u32 q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n_q) return;
    const g1 *R = rows + (size_t)row[q] * (D + 1);
    const uint8_t *rok = row_ok + (size_t)row[q] * (D + 1);
    int y = ys[q];
    bool ok = true;
    g1 acc;
    jac_set_inf(acc);
    for (int j = (int)D; j >= 0; j--) {
        g1_mul_small(acc, y);
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
                                const int *ys, u32 n_q, uint8_t *out48, uint8_t *status) {
    LCB_LAUNCH(k_dkg_horner, (const g1 *)rows, row_ok, D, row, ys, n_q, out48, status);
}
extern "C" void lcbk_g1a_to_jac(dim3 grid, hipStream_t s, const void *in, u32 n, void *out, uint8_t *ok) {
    LCB_LAUNCH(k_g1a_to_jac, (const g1a_st *)in, n, (g1 *)out, ok);
}
