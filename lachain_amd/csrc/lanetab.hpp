// lachain_amd/csrc/lanetab.hpp — per-lane point tables in a device workspace the library allocates, instead of in
// registers that spill to scratch (round 5).
//
// Why: a kernel's scratch (private segment) is reserved by the HIP runtime per hardware queue for every wave slot of
// the device, whatever the launch's occupancy — 22.7 KB per lane (k_g2_mul2_lanes' two GLS tables in scratch) came to
// ~12 GB per queue, and two contexts (or two processes) running CommonCoin assemblies on different queues aborted the
// process with HSA_STATUS_ERROR_OUT_OF_RESOURCES.  A workspace is sized by the launch (its persistent grid), owned
// by the caller's context and freed with it, and a failed allocation is an error code, not a queue abort.
//
// Layout: the slot of lane l of wave w holds Q 16-byte quads; quad q of that lane is at byte
//   ws + ((w * Q + q) * 64 + l) * 16,
// so when a wave's lanes write the same entry (the table builds) every access is 1 KB contiguous, and a lane's gather
// of its own entry touches the same lines as the scratch it replaces.  The byte offset is made opaque where used so the
// compiler cannot hoist one 64-bit address per quad out of the ladders (kcommon.hpp fp12_store_soa does the same).
#pragma once
#include "curve.hpp"

// the slot of global lane `gid` in a workspace of `quads` quads per lane
DI char *lw_slot(u32 *ws, u32 quads, u32 gid) {
    return (char *)ws + ((size_t)(gid >> 6) * quads * 64 + (gid & 63)) * 16;
}
template <class F> DI void lw_put(char *p, u32 q, const F &v) {
    static_assert(sizeof(F) % 16 == 0, "quad-sized values");
    const u32 *s = (const u32 *)&v;
    u32 off = q * 1024u;
    asm volatile("" : "+v"(off));
#pragma unroll
    for (int g = 0; g < (int)(sizeof(F) / 16); g++)
        *(uint4 *)(p + off + g * 1024) = make_uint4(s[4 * g], s[4 * g + 1], s[4 * g + 2], s[4 * g + 3]);
}
template <class F> DI void lw_get(F &v, const char *p, u32 q) {
    static_assert(sizeof(F) % 16 == 0, "quad-sized values");
    u32 *d = (u32 *)&v;
    u32 off = q * 1024u;
    asm volatile("" : "+v"(off));
#pragma unroll
    for (int g = 0; g < (int)(sizeof(F) / 16); g++) {
        const uint4 x = *(const uint4 *)(p + off + g * 1024);
        d[4 * g] = x.x; d[4 * g + 1] = x.y; d[4 * g + 2] = x.z; d[4 * g + 3] = x.w;
    }
}

// Table entries e = 1..n of a lane, each x | y | z | prefix product (4 field elements): while building, (x, y, z) is the
// Jacobian entry; lw_table_to_aff turns (x, y) into the affine entry in place.
template <class F> struct LwTab {
    static constexpr u32 FQ = sizeof(F) / 16;     // quads per field element (fp 3, fp2 6)
    static constexpr u32 EQ = 4 * FQ;             // quads per entry
    DI static u32 base(u32 e) { return (e - 1) * EQ; }
    DI static void put_jac(char *p, u32 e, const jac<F> &t) {
        lw_put(p, base(e), t.x);
        lw_put(p, base(e) + FQ, t.y);
        lw_put(p, base(e) + 2 * FQ, t.z);
    }
    DI static void get_jac(jac<F> &t, const char *p, u32 e) {
        lw_get(t.x, p, base(e));
        lw_get(t.y, p, base(e) + FQ);
        lw_get(t.z, p, base(e) + 2 * FQ);
    }
    DI static void get_aff(F &x, F &y, const char *p, u32 e) {
        lw_get(x, p, base(e));
        lw_get(y, p, base(e) + FQ);
    }
};
DI void lw_inv(fp &r, const fp &a) { fp_inv_gcd(r, a); }
DI void lw_inv(fp2 &r, const fp2 &a) { fp2_inv_gn(r, a); }

// jac_table_to_aff (curve.hpp) over entries 1..n of the slot: one batched inversion (Montgomery's trick; binary-GCD
// inversion, the same residue as the exponentiation); false when an entry is the point at infinity
template <class F> DI bool lw_table_to_aff(char *p, u32 n) {
    typedef LwTab<F> T;
    F acc, z;
    f_one(acc);
#pragma unroll 1
    for (u32 i = 1; i <= n; i++) {
        lw_get(z, p, T::base(i) + 2 * T::FQ);
        f_mul(acc, acc, z);
        lw_put(p, T::base(i) + 3 * T::FQ, acc);
    }
    if (f_is_zero(acc)) return false;
    F inv;
    lw_inv(inv, acc);
#pragma unroll 1
    for (u32 i = n; i >= 1; i--) {
        F zi, zi2, pre, x, y;
        if (i > 1) lw_get(pre, p, T::base(i - 1) + 3 * T::FQ);
        else f_one(pre);
        lw_get(z, p, T::base(i) + 2 * T::FQ);
        f_mul(zi, inv, pre);                 // 1 / z_i
        f_mul(inv, inv, z);
        f_sqr(zi2, zi);
        T::get_aff(x, y, p, i);
        f_mul(x, x, zi2);
        f_mul(zi2, zi2, zi);
        f_mul(y, y, zi2);
        lw_put(p, T::base(i), x);
        lw_put(p, T::base(i) + T::FQ, y);
    }
    return true;
}

// ------------------------------------------------------------------ G2: GLS with the 15 sums of the psi-images
// entries e0 + 1 .. e0 + 15: the non-empty sums of Q = {A, -psi A, psi^2 A, -psi^3 A} (index bit i <-> Q_i); for A in
// G2 no sum is infinity (|i0 - i1 z + i2 z^2 - i3 z^3| < r).  Q_2, Q_3 = psi^2(Q_0, Q_1), so 1 + 9 additions
#define LW_G2_TAB_QUADS (15 * 24)
DI void lw_g2_gls_sums(char *p, u32 e0, const g2a &A) {
    typedef LwTab<fp2> T;
    {
        g2 t1, t2, t3;
        jac_from_aff(t1, A);
        g2_psi(t2, t1);
        fp2_neg(t2.y, t2.y);                         // -psi(A), z = 1
        jac_add_aff(t3, t1, t2.x, t2.y);
        T::put_jac(p, e0 + 1, t1);
        T::put_jac(p, e0 + 2, t2);
        T::put_jac(p, e0 + 3, t3);
    }
#pragma unroll 1
    for (u32 j = 1; j < 4; j++) {
        g2 t;
        T::get_jac(t, p, e0 + j);
        g2_psi2(t, t);
        T::put_jac(p, e0 + 4 * j, t);
    }
#pragma unroll 1
    for (u32 j = 4; j < 16; j += 4)
#pragma unroll 1
        for (u32 i = 1; i < 4; i++) {
            g2 a, b, t;
            T::get_jac(a, p, e0 + i);
            T::get_jac(b, p, e0 + j);
            jac_add(t, a, b);
            T::put_jac(p, e0 + j + i, t);
        }
}
// the digit column of bit b of the four GLS digits
DI u32 lw_gls_col(const u64 d[4], int b) {
    return (u32)((d[0] >> b) & 1) | (u32)((d[1] >> b) & 1) << 1 | (u32)((d[2] >> b) & 1) << 2 |
           (u32)((d[3] >> b) & 1) << 3;
}
// GLS digits of k (< r): k = d0 + d1 u + d2 u^2 + d3 u^3, u = |z| (curve.hpp u256_divmod_u)
DI void lw_gls_digits(u64 d[4], const u32 k[8]) {
    u32 q[8];
#pragma unroll
    for (int j = 0; j < 8; j++) q[j] = k[j];
    u256_divmod_u(q, d[0]);
    u256_divmod_u(q, d[1]);
    u256_divmod_u(q, d[2]);
    d[3] = (u64)q[0] | ((u64)q[1] << 32);
}
// k A for A in G2 (k < r) from the slot's table at entries 1..15 (built and made affine); 64 doublings, <= 64 mixed adds
DI void lw_g2_gls_ladder(g2 &r, const char *p, const u64 d[4]) {
    jac_set_inf(r);
#pragma unroll 1
    for (int b = 63; b >= 0; b--) {
        jac_dbl(r, r);
        const u32 idx = lw_gls_col(d, b);
        if (idx) {
            fp2 x, y;
            LwTab<fp2>::get_aff(x, y, p, idx);
            jac_add_aff(r, r, x, y);
        }
    }
}
// ka A + kb B for A, B in G2: one run of 64 doublings over both tables (Straus), entries 1..15 and 16..30
DI void lw_g2_gls_ladder2(g2 &r, const char *p, const u64 da[4], const u64 db[4]) {
    jac_set_inf(r);
#pragma unroll 1
    for (int b = 63; b >= 0; b--) {
        jac_dbl(r, r);
        const u32 ia = lw_gls_col(da, b), ib = lw_gls_col(db, b);
#pragma unroll 1
        for (int s = 0; s < 2; s++) {
            const u32 idx = s ? (ib ? ib + 15 : 0) : ia;
            if (idx) {
                fp2 x, y;
                LwTab<fp2>::get_aff(x, y, p, idx);
                jac_add_aff(r, r, x, y);
            }
        }
    }
}

// ------------------------------------------------------------------ 4-bit fixed window over any on-curve point
// jac_mul_win4 (curve.hpp) with its table in the slot (entries 1..15 = 1P..15P): integer scalar multiplication, exact
// outside the r-torsion; a table entry at infinity (order <= 15) takes the binary ladder
#define LW_WIN4_QUADS(F) (15 * LwTab<F>::EQ)
// (NW words of scalar: 8 for Fr, 12 for mclBn_G1EvaluatePolynomial's powers reduced mod the curve order)
template <class F, int NW = 8> DI void lw_mul_win4(jac<F> &r, char *p, const aff<F> &P, const u32 *k) {
    typedef LwTab<F> T;
    jac_set_inf(r);
    if (P.inf) return;
    {
        jac<F> t;
        jac_from_aff(t, P);
        T::put_jac(p, 1, t);
        jac_dbl(t, t);
        T::put_jac(p, 2, t);
#pragma unroll 1
        for (u32 i = 3; i < 16; i++) {
            jac_add_aff(t, t, P.x, P.y);
            T::put_jac(p, i, t);
        }
    }
    if (!lw_table_to_aff<F>(p, 15)) { jac_mul_aff(r, P, k, 32 * NW); return; }
#pragma unroll 1
    for (int w = 8 * NW - 1; w >= 0; w--) {
        jac_dbl(r, r); jac_dbl(r, r); jac_dbl(r, r); jac_dbl(r, r);
        const u32 nib = (k[w >> 3] >> (4 * (w & 7))) & 15;
        if (nib) {
            F x, y;
            T::get_aff(x, y, p, nib);
            jac_add_aff(r, r, x, y);
        }
    }
}
