// lachain_amd/csrc/k_lines.hip — the line set of a G2 point on FIVE lanes (latency path of the small preparations:
// mclBn_pairing with a G2 argument it has not seen, the cached / queued verification's first-sight ciphertexts).
//
// lineset_compute (pairing.hpp) is one lane's serial chain of ~3,700 Fp products (~4 ms).  Here a group of five lanes
// shares every step, coop_pt.hpp's idea with one Fp2 product per lane and ROUND:
//   doubling  {Y^2, Z^2, XY, YZ, X^2} then {XY s, s'^2, (3b'Z^2)^2, Y^2 YZ, acc A}   2 rounds instead of 11 products
//   addition  {yQ Z, xQ Z}, {th xQ, la yQ, th^2, la^2}, {la D, Z C, X D, acc A}, {la H, th (G - H), Y E, Z E}   4 rounds
// (3b' Z^2 = 12 (1 + u) Z^2 and the halvings are additions: the same field elements as line_dbl_step's products by the
// constants), then the normalisation's backward pass one round per line: {inv pre_(k-1), inv A_k, Bc_(k+1) a_(k+1),
// Cc_(k+1) a_(k+1)}, each lane loading its own operand.  Every value is the fully reduced residue, so the set is
// word-for-word lineset_compute's (tests/test_gpu_lines.py compares the two kernels' sets).
// One wave holds 12 groups (lanes 60..63 shadow group 0 without storing); the rounds synchronise the workgroup, so the
// control flow around them is wave-uniform.
#include "lines_coop.hpp"

LCB_ASM_LIBRARY(k_lines)
LCB_TU_CONFIG(k_lines)

// k_lineset_fill's contract (line sets of points a prepare kernel stored, sets / w_g2 as there), 12 sets per block
extern "C" __global__ void __launch_bounds__(64, 1) k_lineset_coop(u32 *lines, u32 n_sets, const u32 *sets,
                                                                   uint8_t *w_g2) {
    __shared__ LsLds lds[LS_GROUPS + 1];
    lineset_coop_run(lds, lines, n_sets, sets, w_g2);
}

extern "C" void lcbk_lineset_coop(hipStream_t s, u32 *lines, u32 n_sets, const u32 *sets, uint8_t *w_g2) {
    if (!n_sets) return;
    LCB_LAUNCH_GATED(k_lineset_coop, dim3((n_sets + LS_GROUPS - 1) / LS_GROUPS), dim3(64), 0, s, lines, n_sets, sets,
                       w_g2);
}
