// lachain_amd/csrc/k_secp.hip — gfx950 kernels for batched secp256k1 ECDSA header-signature checks.
//
// Reference: RootProtocol checks every SignedHeaderMessage with
//   _crypto.VerifySignatureHashed(header.Keccak(), signature, EcdsaPublicKeySet[idx].EncodeCompressed(), useNewChainId)
// (src/Lachain.Consensus/RootProtocol/RootProtocol.cs:91-105; DefaultCrypto.cs:79-101 over libsecp256k1's verify).
//
// MI355X design: the validators' keys are fixed for a whole cycle, so each key gets a resident fixed-base comb table in
// HBM (33 windows x 128 affine multiples d 2^(8w) Q, 270 KB per key; the generator has one too).  A verification is
// then u1 G + u2 Q = sum of at most 66 table entries selected by signed 8-bit digits of u1, u2: 66 mixed additions and
// no doublings.  The scalar work (s^-1 mod n) is batched per thread with Montgomery's trick (one inversion per 16
// signatures).  Kernels:
//   k_secp_key_parse   33/65-byte public keys -> affine points + validity (libsecp256k1 pubkey_parse rules)
//   k_secp_comb_build  one lane per (key, window): the window's 128 multiples, batch-normalised to affine
//   k_secp_header_hash HashUtils.Keccak(BlockHeader): Keccak-256 of the RLP list, plus the Index == era check
//   k_secp_scalars     signature parsing / recId / low-s checks, s^-1, u1 = z/s, u2 = r/s -> signed digits (job records)
//   k_secp_verify      sum of the table entries, then x(R) mod n == r on Jacobian coordinates (no inversion)
#include "secp.hpp"
#ifndef SECP_HOST_EMULATION
#include "gate.hpp"
#endif

#define SECP_BLOCK 256
#define SECP_WIN 33                  // signed 8-bit digits of a scalar < n: 32 bytes + the final carry
#define SECP_TAB 128                 // multiples 1..128 per window
#define SECP_BATCH 16                // signatures per thread in the batched inversion

struct secp_job {                    // 112 B, written by k_secp_scalars, read by k_secp_verify
    int8_t d1[36], d2[36];           // digits of u1 (generator) and u2 (key), windows 0..32
    u32 r[8];
    u32 key;
    u32 flags;                       // bit 0: all checks passed; bit 1: r < p - n (x(R) may be r + n)
};
static_assert(sizeof(secp_job) == 112, "job record");

// ------------------------------------------------------------------------------------------------ keys
// secp256k1_ec_pubkey_parse: 0x02/0x03 || x (x < p, on the curve) or 0x04/0x06/0x07 || x || y (hybrid tag = y parity)
extern "C" __global__ void __launch_bounds__(SECP_BLOCK) k_secp_key_parse(const uint8_t *pks, u32 pk_len, u32 n_keys,
                                                                         secp_aff *out, u32 *ok_out) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_keys) return;
    const uint8_t *pk = pks + (size_t)i * pk_len;
    u32 tag = pk[0];
    bool ok = false;
    fe x, y;
    if (pk_len == 33 && (tag == 2 || tag == 3)) {
        u256_from_be(x.v, pk + 1);
        ok = u256_lt(x.v, SECP_P);
        fe x3, t;
        fe_sqr(t, x); fe_mul(x3, t, x); fe_add(x3, x3, fe_small(7));
        fe_sqrt(y, x3);
        fe_sqr(t, y);
        ok = ok && fe_eq(t, x3);
        y = fe_canon(y);
        if ((y.v[0] & 1) != (tag & 1)) fe_neg(y, y);
    } else if (pk_len == 65 && (tag == 4 || tag == 6 || tag == 7)) {
        u256_from_be(x.v, pk + 1);
        u256_from_be(y.v, pk + 33);
        ok = u256_lt(x.v, SECP_P) && u256_lt(y.v, SECP_P);
        if (tag != 4) ok = ok && ((y.v[0] & 1) == (tag & 1));
        fe x3, t;
        fe_sqr(t, x); fe_mul(x3, t, x); fe_add(x3, x3, fe_small(7));
        fe_sqr(t, y);
        ok = ok && fe_eq(t, x3);
    } else {
        x = fe_zero(); y = fe_zero();
    }
    out[i].x = fe_canon(x);
    out[i].y = fe_canon(y);
    ok_out[i] = ok;
}

// ------------------------------------------------------------------------------------------------ comb tables
// lane (t, w): tables[(t * 33 + w) * 128 + d - 1] = d 2^(8w) base[t] for d = 1..128 (affine, canonical).  tmp_z and
// tmp_pre hold 128 field elements per lane (word-major: element d of lane L at d * lanes + L).
extern "C" __global__ void __launch_bounds__(SECP_BLOCK) k_secp_comb_build(const secp_aff *base, const u32 *base_ok,
                                                                          u32 n_tables, secp_aff *tables, fe *tmp_z,
                                                                          fe *tmp_pre) {
    u32 lanes = n_tables * SECP_WIN;
    u32 L = blockIdx.x * blockDim.x + threadIdx.x;
    if (L >= lanes) return;
    u32 t = L / SECP_WIN, w = L % SECP_WIN;
    secp_aff *T = tables + (size_t)L * SECP_TAB;
    if (!base_ok[t]) return;                          // never read: the verify kernel rejects invalid keys first
    secp_jac B;
    jac_set_aff(B, base[t].x, base[t].y);
    for (u32 k = 0; k < 8 * w; k++) jac_dbl(B, B);
    fe zi, zi2, bx, by;
    fe_inv(zi, B.z);
    fe_sqr(zi2, zi);
    fe_mul(bx, B.x, zi2);
    fe_mul(zi2, zi2, zi);
    fe_mul(by, B.y, zi2);
    secp_jac P;
    jac_set_aff(P, bx, by);
    fe acc;
    for (int d = 0; d < SECP_TAB; d++) {
        T[d].x = P.x;
        T[d].y = P.y;
        tmp_z[(size_t)d * lanes + L] = P.z;
        if (d == 0) acc = P.z; else fe_mul(acc, acc, P.z);
        tmp_pre[(size_t)d * lanes + L] = acc;
        if (d + 1 < SECP_TAB) jac_add_aff(P, P, bx, by);
    }
    fe inv;
    fe_inv(inv, acc);
    for (int d = SECP_TAB - 1; d >= 0; d--) {
        fe z = tmp_z[(size_t)d * lanes + L];
        fe zd;
        if (d > 0) fe_mul(zd, inv, tmp_pre[(size_t)(d - 1) * lanes + L]); else zd = inv;
        fe_mul(inv, inv, z);
        fe zd2, x, y;
        fe_sqr(zd2, zd);
        fe_mul(x, T[d].x, zd2);
        fe_mul(zd2, zd2, zd);
        fe_mul(y, T[d].y, zd2);
        T[d].x = fe_canon(x);
        T[d].y = fe_canon(y);
    }
}

// ------------------------------------------------------------------------------------------------ header hash
// lcb_block_header (112 B): u64 index | prev_block_hash[32] | merkle_root[32] | state_hash[32] | u64 nonce.
// HashUtils.Keccak(BlockHeader) (HashUtils.cs:40-53): Keccak-256 of RLP [prev, state, merkle, index LE8, nonce LE8]
// = 0xf8 0x75 | 0xa0 prev | 0xa0 state | 0xa0 merkle | 0x88 index | 0x88 nonce  (119 bytes: one 136-byte block)
extern "C" __global__ void __launch_bounds__(SECP_BLOCK) k_secp_header_hash(const uint8_t *hdr, u32 n, u64 era,
                                                                           uint8_t *hash_out, uint8_t *pre_ok) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t *h = hdr + (size_t)i * 112;
    uint8_t m[136];
#pragma unroll
    for (int k = 0; k < 136; k++) m[k] = 0;
    m[0] = 0xf8; m[1] = 0x75;
    const int src[3] = {8, 72, 40};                     // prev, state, merkle offsets inside the record
#pragma unroll
    for (int f = 0; f < 3; f++) {
        m[2 + 33 * f] = 0xa0;
#pragma unroll
        for (int k = 0; k < 32; k++) m[3 + 33 * f + k] = h[src[f] + k];
    }
    m[101] = 0x88;
#pragma unroll
    for (int k = 0; k < 8; k++) m[102 + k] = h[k];        // index, little-endian
    m[110] = 0x88;
#pragma unroll
    for (int k = 0; k < 8; k++) m[111 + k] = h[104 + k];  // nonce
    m[119] ^= 0x01;                                       // Keccak padding (original domain byte)
    m[135] ^= 0x80;
    u64 s[25];
#pragma unroll
    for (int k = 0; k < 25; k++) s[k] = 0;
#pragma unroll
    for (int k = 0; k < 17; k++) {
        u64 v = 0;
#pragma unroll
        for (int b = 0; b < 8; b++) v |= (u64)m[8 * k + b] << (8 * b);
        s[k] = v;
    }
    keccak_f1600(s);
#pragma unroll
    for (int k = 0; k < 32; k++) hash_out[32 * (size_t)i + k] = (uint8_t)(s[k / 8] >> (8 * (k % 8)));
    u64 index = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) index |= (u64)h[k] << (8 * k);
    pre_ok[i] = index == era;                              // RootProtocol.cs:94-96
}

// ------------------------------------------------------------------------------------------------ scalars
struct sig_in {
    u32 r[8], s[8], z[8];
    u32 key;
    bool ok;
};
// DefaultCrypto.VerifySignatureHashed's checks before the curve arithmetic; z = hash mod n
__device__ __forceinline__ void load_sig(sig_in &q, size_t i, const uint8_t *hashes, const uint8_t *sigs, u32 sig_len,
                                         u32 want_len, int chain_id, const int32_t *key_idx, u32 n_keys,
                                         const u32 *key_ok, const uint8_t *pre_ok) {
    const uint8_t *sg = sigs + i * sig_len;
    u256_from_be(q.r, sg);
    u256_from_be(q.s, sg + 32);
    u256_from_be(q.z, hashes + 32 * i);
    if (!u256_lt(q.z, SECP_N)) {                           // z < 2^256 < 2n: one subtraction
        u32 br = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) { u64 d = (u64)q.z[k] - SECP_N[k] - br; q.z[k] = (u32)d; br = (u32)(d >> 32) & 1; }
    }
    // RestoreEncodedRecIdFromSignatureBuffer (DefaultCrypto.cs:31-44) and recId = (enc - 36) / 2 / chainId in
    // [0, 3]; C and C# both truncate toward zero; chain id 0 is a DivideByZeroException (not verified)
    int enc = sig_len == 66 ? (int)sg[64] * 256 + (int)sg[65] : (int)sg[64];
    bool rec_ok = false;
    if (chain_id != 0) {
        int rec = (enc - 36) / 2 / chain_id;
        rec_ok = rec >= 0 && rec <= 3;
    }
    int32_t k = key_idx[i];
    bool key_in = k >= 0 && (u32)k < n_keys;
    q.key = key_in ? (u32)k : 0u;
    bool ok = sig_len == want_len && rec_ok && key_in && key_ok[q.key] != 0;
    ok = ok && u256_lt(q.r, SECP_N) && u256_lt(q.s, SECP_N);          // compact parse: overflow
    ok = ok && !u256_lt(SECP_NH, q.s);                                  // low-s rule: s <= (n - 1) / 2
    ok = ok && !u256_is_zero(q.r) && !u256_is_zero(q.s);
    if (pre_ok) ok = ok && pre_ok[i] != 0;
    q.ok = ok;
}
__device__ __forceinline__ void recode(int8_t *d, const sc &u) {
    u32 carry = 0;
#pragma unroll
    for (int w = 0; w < 32; w++) {
        u32 v = ((u.v[w >> 2] >> (8 * (w & 3))) & 0xffu) + carry;
        carry = v >= 128u;                                 // digits in [-128, 127]: int8 range
        d[w] = (int8_t)(int)(carry ? (int)v - 256 : (int)v);
    }
    d[32] = (int8_t)carry;
#pragma unroll
    for (int w = 33; w < 36; w++) d[w] = 0;
}
extern "C" __global__ void __launch_bounds__(SECP_BLOCK) k_secp_scalars(const uint8_t *hashes, const uint8_t *sigs,
                                                                       u32 sig_len, u32 want_len, int chain_id,
                                                                       const int32_t *key_idx, u32 n_keys,
                                                                       const u32 *key_ok, const uint8_t *pre_ok,
                                                                       u32 n, secp_job *jobs) {
    const size_t T = (size_t)gridDim.x * blockDim.x;
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    sc one = {{1, 0, 0, 0, 0, 0, 0, 0}}, r2 = sc_from(SECP_R2N);
    sc pre[SECP_BATCH];
#pragma unroll
    for (int k = 0; k < SECP_BATCH; k++) {
        size_t i = tid + k * T;
        sc sM = one;
        if (i < n) {
            sig_in q;
            load_sig(q, i, hashes, sigs, sig_len, want_len, chain_id, key_idx, n_keys, key_ok, pre_ok);
            if (q.ok) sM = sc_from(q.s);
        }
        sc_mont_mul(sM, sM, r2);
        if (k == 0) pre[k] = sM; else sc_mont_mul(pre[k], pre[k - 1], sM);
    }
    sc inv;
    sc_mont_inv(inv, pre[SECP_BATCH - 1]);
#pragma unroll
    for (int k = SECP_BATCH - 1; k >= 0; k--) {
        size_t i = tid + k * T;
        sc sM = one;
        sig_in q;
        q.ok = false;
        if (i < n) {
            load_sig(q, i, hashes, sigs, sig_len, want_len, chain_id, key_idx, n_keys, key_ok, pre_ok);
            if (q.ok) sM = sc_from(q.s);
        }
        sc_mont_mul(sM, sM, r2);
        sc wM;
        if (k > 0) sc_mont_mul(wM, inv, pre[k - 1]); else wM = inv;
        sc_mont_mul(inv, inv, sM);
        if (i < n) {
            secp_job j;
            sc u1, u2;
            sc_mont_mul(u1, sc_from(q.z), wM);             // z s^-1 (plain: the Montgomery factors cancel)
            sc_mont_mul(u2, sc_from(q.r), wM);
            recode(j.d1, u1);
            recode(j.d2, u2);
#pragma unroll
            for (int l = 0; l < 8; l++) j.r[l] = q.r[l];
            j.key = q.key;
            j.flags = (q.ok ? 1u : 0u) | (u256_lt(q.r, SECP_PMN) ? 2u : 0u);
            jobs[i] = j;
        }
    }
}

// ------------------------------------------------------------------------------------------------ verify
__device__ __forceinline__ void comb_add_entry(secp_jac &acc, const secp_aff &e, int d) {
    if (d == 0) return;
    fe y = e.y;
    if (d < 0) fe_neg(y, y);
    jac_add_aff(acc, acc, e.x, y);
}
__device__ __forceinline__ void comb_add(secp_jac &acc, const secp_aff *tab, int w, int d) {
    if (d == 0) return;
    const secp_aff e = tab[w * SECP_TAB + (d < 0 ? -d : d) - 1];
    fe y = e.y;
    if (d < 0) fe_neg(y, y);
    jac_add_aff(acc, acc, e.x, y);
}
extern "C" __global__ void __launch_bounds__(SECP_BLOCK) k_secp_verify(const secp_job *jobs, u32 n,
                                                                      const secp_aff *g_table,
                                                                      const secp_aff *key_tables, uint8_t *out) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const secp_job *jp = jobs + i;
    const secp_job j = *jp;
    if (!(j.flags & 1u)) { out[i] = 0; return; }
    const secp_aff *KT = key_tables + (size_t)j.key * SECP_WIN * SECP_TAB;
    secp_jac acc;
    acc.inf = true;
    acc.x = acc.y = acc.z = fe_zero();
    // digits re-read from the (cached) record (no indexed registers); the next window's two table entries are
    // loaded while the current window's additions run
    int dg = jp->d1[0], dk = jp->d2[0];
    secp_aff eg = g_table[dg ? (dg < 0 ? -dg : dg) - 1 : 0], ek = KT[dk ? (dk < 0 ? -dk : dk) - 1 : 0];
    for (int w = 0; w < SECP_WIN; w++) {
        const int cg = dg, ck = dk;
        const secp_aff xg = eg, xk = ek;
        if (w + 1 < SECP_WIN) {
            dg = jp->d1[w + 1];
            dk = jp->d2[w + 1];
            eg = g_table[(w + 1) * SECP_TAB + (dg ? (dg < 0 ? -dg : dg) - 1 : 0)];
            ek = KT[(w + 1) * SECP_TAB + (dk ? (dk < 0 ? -dk : dk) - 1 : 0)];
        }
        comb_add_entry(acc, xg, cg);
        comb_add_entry(acc, xk, ck);
    }
    bool good = false;
    if (!acc.inf) {
        // x(R) mod n == r  <=>  X == r Z^2, or (r < p - n and X == (r + n) Z^2)   (libsecp256k1 ecdsa_sig_verify)
        fe z2, rx, r = fe_from(j.r);
        fe_sqr(z2, acc.z);
        fe_mul(rx, r, z2);
        good = fe_eq(rx, acc.x);
        if (!good && (j.flags & 2u)) {
            fe rn;
            u64 c = 0;
#pragma unroll
            for (int l = 0; l < 8; l++) { c += (u64)j.r[l] + SECP_N[l]; rn.v[l] = (u32)c; c >>= 32; }
            fe_mul(rx, rn, z2);
            good = fe_eq(rx, acc.x);
        }
    }
    out[i] = good;
}

// ------------------------------------------------------------------------------------------------ signing side
// k G through the generator's comb table, as an affine point (k < n, k != 0)
__device__ __forceinline__ void gen_mul_aff(fe &x, fe &y, const sc &k, const secp_aff *g_table) {
    int8_t d[36];
    recode(d, k);
    secp_jac acc;
    acc.inf = true;
    acc.x = acc.y = acc.z = fe_zero();
    for (int w = 0; w < SECP_WIN; w++) comb_add(acc, g_table, w, d[w]);
    fe zi, zi2;
    fe_inv(zi, acc.z);
    fe_sqr(zi2, zi);
    fe_mul(x, acc.x, zi2);
    fe_mul(zi2, zi2, zi);
    fe_mul(y, acc.y, zi2);
    x = fe_canon(x);
    y = fe_canon(y);
}
// compressed public keys d G (DefaultCrypto / EcdsaKeyPair key derivation); ok = 0 for d = 0 or d >= n
extern "C" __global__ void __launch_bounds__(SECP_BLOCK) k_secp_pubkey(const uint8_t *privs, u32 n,
                                                                      const secp_aff *g_table, uint8_t *out33,
                                                                      uint8_t *ok_out) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    sc d;
    u256_from_be(d.v, privs + 32 * (size_t)i);
    bool ok = !u256_is_zero(d.v) && u256_lt(d.v, SECP_N);
    if (!ok) d = sc_from(SECP_GX);                 // any scalar: the output is discarded
    fe x, y;
    gen_mul_aff(x, y, d, g_table);
    uint8_t *o = out33 + 33 * (size_t)i;
    o[0] = ok ? (uint8_t)(2 + (y.v[0] & 1)) : 0;
#pragma unroll
    for (int k = 0; k < 32; k++) o[1 + k] = ok ? (uint8_t)(x.v[7 - k / 4] >> (8 * (3 - k % 4))) : 0;
    ok_out[i] = ok;
}
// ECDSA signatures with caller-given nonces: r = x(k G) mod n, s = k^-1 (z + r d) mod n normalised to low s, recovery
// id = parity of y(k G) | 2 (x(k G) >= n), flipped with s (libsecp256k1 ecdsa_sig_sign).  out: r || s (BE) || v with
// DefaultCrypto.SignHashed's encoding (DefaultCrypto.cs:114-136): v = chainId * 2 + 35 + recId as 1 byte (the int's
// low byte, old chain id) or 2 bytes big-endian (new chain id)
extern "C" __global__ void __launch_bounds__(SECP_BLOCK) k_secp_sign(const uint8_t *hashes, const uint8_t *privs,
                                                                    const uint8_t *nonces, u32 n,
                                                                    const secp_aff *g_table, int chain_id, int use_new,
                                                                    uint8_t *out, uint8_t *ok_out) {
    u32 i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    sc d, k, z;
    u256_from_be(d.v, privs + 32 * (size_t)i);
    u256_from_be(k.v, nonces + 32 * (size_t)i);
    u256_from_be(z.v, hashes + 32 * (size_t)i);
    bool ok = !u256_is_zero(d.v) && u256_lt(d.v, SECP_N) && !u256_is_zero(k.v) && u256_lt(k.v, SECP_N);
    if (!ok) k = sc_from(SECP_GX);
    if (!u256_lt(z.v, SECP_N)) {
        u32 br = 0;
#pragma unroll
        for (int l = 0; l < 8; l++) { u64 t = (u64)z.v[l] - SECP_N[l] - br; z.v[l] = (u32)t; br = (u32)(t >> 32) & 1; }
    }
    fe x, y;
    gen_mul_aff(x, y, k, g_table);
    u32 recid = y.v[0] & 1;
    sc r = sc_from(x.v);
    if (!u256_lt(r.v, SECP_N)) {
        u32 br = 0;
#pragma unroll
        for (int l = 0; l < 8; l++) { u64 t = (u64)r.v[l] - SECP_N[l] - br; r.v[l] = (u32)t; br = (u32)(t >> 32) & 1; }
        recid |= 2;
    }
    sc r2 = sc_from(SECP_R2N), kM, kiM, rM, dM, zM, t, s;
    sc_mont_mul(kM, k, r2);
    sc_mont_inv(kiM, kM);
    sc_mont_mul(rM, r, r2);
    sc_mont_mul(dM, d, r2);
    sc_mont_mul(zM, z, r2);
    sc_mont_mul(t, rM, dM);
    {   // t = t + zM mod n
        u64 c = 0;
        u32 sum[8], dd[8], br = 0;
#pragma unroll
        for (int l = 0; l < 8; l++) { c += (u64)t.v[l] + zM.v[l]; sum[l] = (u32)c; c >>= 32; }
#pragma unroll
        for (int l = 0; l < 8; l++) { u64 q = (u64)sum[l] - SECP_N[l] - br; dd[l] = (u32)q; br = (u32)(q >> 32) & 1; }
        bool sub = c || !br;
#pragma unroll
        for (int l = 0; l < 8; l++) t.v[l] = sub ? dd[l] : sum[l];
    }
    sc_mont_mul(t, t, kiM);
    sc one = {{1, 0, 0, 0, 0, 0, 0, 0}};
    sc_mont_mul(s, t, one);                                  // out of Montgomery form
    if (u256_lt(SECP_NH, s.v)) {                             // s > (n - 1) / 2: s = n - s
        u32 br = 0;
#pragma unroll
        for (int l = 0; l < 8; l++) { u64 q = (u64)SECP_N[l] - s.v[l] - br; s.v[l] = (u32)q; br = (u32)(q >> 32) & 1; }
        recid ^= 1;
    }
    ok = ok && !u256_is_zero(r.v) && !u256_is_zero(s.v);
    uint8_t *o = out + (use_new ? 66 : 65) * (size_t)i;
#pragma unroll
    for (int b = 0; b < 32; b++) {
        o[b] = (uint8_t)(r.v[7 - b / 4] >> (8 * (3 - b % 4)));
        o[32 + b] = (uint8_t)(s.v[7 - b / 4] >> (8 * (3 - b % 4)));
    }
    u32 v = (u32)(chain_id * 2 + 35 + (int)recid);
    if (use_new) { o[64] = (uint8_t)(v >> 8); o[65] = (uint8_t)v; }
    else o[64] = (uint8_t)v;
    ok_out[i] = ok;
}

// generator as a one-entry key list (affine, canonical) for the generator's comb table
extern "C" __global__ void k_secp_gen(secp_aff *out, u32 *ok) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        out->x = fe_from(SECP_GX);
        out->y = fe_from(SECP_GY);
        *ok = 1;
    }
}

#ifndef SECP_HOST_EMULATION
// ---------------------------------------------------------------- host launch wrappers
static unsigned blocks_for(size_t n) { return (unsigned)((n + SECP_BLOCK - 1) / SECP_BLOCK); }
extern "C" size_t lcbk_secp_job_bytes(void) { return sizeof(secp_job); }
extern "C" size_t lcbk_secp_table_bytes(void) { return (size_t)SECP_WIN * SECP_TAB * sizeof(secp_aff); }
extern "C" size_t lcbk_secp_aff_bytes(void) { return sizeof(secp_aff); }
extern "C" void lcbk_secp_key_parse(hipStream_t s, const uint8_t *pks, u32 pk_len, u32 n_keys, void *out, u32 *ok) {
    if (!n_keys) return;
    LCB_LAUNCH_GATED(k_secp_key_parse, dim3(blocks_for(n_keys)), dim3(SECP_BLOCK), 0, s, pks, pk_len, n_keys,
                       (secp_aff *)out, ok);
}
// tmp must hold 2 * 128 * n_tables * 33 field elements (32 B each)
extern "C" void lcbk_secp_comb_build(hipStream_t s, const void *base, const u32 *base_ok, u32 n_tables, void *tables,
                                     void *tmp) {
    if (!n_tables) return;
    size_t lanes = (size_t)n_tables * SECP_WIN;
    fe *tz = (fe *)tmp, *tp = tz + lanes * SECP_TAB;
    LCB_LAUNCH_GATED(k_secp_comb_build, dim3(blocks_for(lanes)), dim3(SECP_BLOCK), 0, s, (const secp_aff *)base,
                       base_ok, n_tables, (secp_aff *)tables, tz, tp);
}
extern "C" void lcbk_secp_header_hash(hipStream_t s, const uint8_t *hdr, u32 n, u64 era, uint8_t *hash, uint8_t *pre_ok) {
    if (!n) return;
    LCB_LAUNCH_GATED(k_secp_header_hash, dim3(blocks_for(n)), dim3(SECP_BLOCK), 0, s, hdr, n, era, hash, pre_ok);
}
extern "C" void lcbk_secp_scalars(hipStream_t s, const uint8_t *hashes, const uint8_t *sigs, u32 sig_len, u32 want_len,
                                  int chain_id, const int32_t *key_idx, u32 n_keys, const u32 *key_ok,
                                  const uint8_t *pre_ok, u32 n, void *jobs) {
    if (!n) return;
    size_t threads = (n + SECP_BATCH - 1) / SECP_BATCH;
    LCB_LAUNCH_GATED(k_secp_scalars, dim3(blocks_for(threads)), dim3(SECP_BLOCK), 0, s, hashes, sigs, sig_len,
                       want_len, chain_id, key_idx, n_keys, key_ok, pre_ok, n, (secp_job *)jobs);
}
extern "C" void lcbk_secp_verify(hipStream_t s, const void *jobs, u32 n, const void *g_table, const void *key_tables,
                                 uint8_t *out) {
    if (!n) return;
    LCB_LAUNCH_GATED(k_secp_verify, dim3(blocks_for(n)), dim3(SECP_BLOCK), 0, s, (const secp_job *)jobs, n,
                       (const secp_aff *)g_table, (const secp_aff *)key_tables, out);
}
extern "C" void lcbk_secp_pubkey(hipStream_t s, const uint8_t *privs, u32 n, const void *g_table, uint8_t *out33,
                                 uint8_t *ok) {
    if (!n) return;
    LCB_LAUNCH_GATED(k_secp_pubkey, dim3(blocks_for(n)), dim3(SECP_BLOCK), 0, s, privs, n, (const secp_aff *)g_table,
                       out33, ok);
}
extern "C" void lcbk_secp_sign(hipStream_t s, const uint8_t *hashes, const uint8_t *privs, const uint8_t *nonces, u32 n,
                               const void *g_table, int chain_id, int use_new, uint8_t *out, uint8_t *ok) {
    if (!n) return;
    LCB_LAUNCH_GATED(k_secp_sign, dim3(blocks_for(n)), dim3(SECP_BLOCK), 0, s, hashes, privs, nonces, n,
                       (const secp_aff *)g_table, chain_id, use_new, out, ok);
}
extern "C" void lcbk_secp_gen(hipStream_t s, void *out, u32 *ok) {
    LCB_LAUNCH_GATED(k_secp_gen, dim3(1), dim3(64), 0, s, (secp_aff *)out, ok);
}
#endif  // SECP_HOST_EMULATION
