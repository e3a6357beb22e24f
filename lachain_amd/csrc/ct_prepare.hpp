// lachain_amd/csrc/ct_prepare.hpp — one ciphertext's preparation for the exact and census paths (k_tpke.hip
// k_tpke_ct_prepare; k_prep.hip's 256-register copy for the batched check's census ciphertexts): U and W decoded,
// H = G2.SetHashOf(U || V) (TPKE/Utils.cs:21-27, PublicKey.cs:88-92), both points put in their line sets' point slots
// for a line-set kernel to fill.
#pragma once
#include "kcommon.hpp"

// lines layout: lines[(2*c + 0) * LINESET] = H lines, lines[(2*c + 1) * LINESET] = W lines
// slot (nullable): ciphertext c's line sets and validity go to slot[c] instead of c (the prepared-ciphertext cache)
// flags: bit 0 = mcl's original G2 cofactor clearing in hash-to-G2, bit 1 = mark the line sets un-normalised
DI void tpke_ct_prepare_run(const uint8_t *cts_u, const uint8_t *cts_w, const uint8_t *v_data, const u32 *v_off,
                            u32 n_cts, u32 *lines, uint8_t *ct_ok, int flags, const u32 *slot) {
    u32 c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_cts) return;
    const u32 o = slot ? slot[c] : c;
    const uint8_t *ub = cts_u + 48 * (size_t)c;
    g1a U;
    g2a W, Ha;
    bool ok = g1_decompress(U, ub);
    ok = g2_decompress(W, cts_w + 96 * (size_t)c) && ok;
    // H = G2.SetHashOf(U.ToBytes() || V): for a valid U the wire bytes are its canonical encoding
    uint8_t d[64];
    u32 v0 = v_off[c], v1 = v_off[c + 1];
    sha512_2(d, ub, 48, v_data + v0, v1 - v0);
    g2 H;
    bool hok = g2_hash_digest(H, d, (flags & 1) != 0);
    ok = ok && hok;
    if (hok) g2_jac_to_aff_g(Ha, H);
    else { Ha.inf = true; Ha.x = fp2_zero(); Ha.y = fp2_zero(); }
    if (!ok) { W.inf = true; Ha.inf = true; }
    // the two points go to their line sets' point slots; k_lineset_fill computes the 2 * n_cts line sets one lane
    // each (the per-ciphertext serial path is hash + one line set instead of hash + two)
    u32 *lsH = lines + (size_t)(2 * o) * LCB_LINESET_WORDS, *lsW = lines + (size_t)(2 * o + 1) * LCB_LINESET_WORDS;
    lineset_put_point(lsH, Ha);
    lineset_put_point(lsW, W);
    lsH[LCB_LS_FLAG + 2] = lsW[LCB_LS_FLAG + 2] = (flags & 2) ? 1 : 0;
    ct_ok[o] = ok;
}
