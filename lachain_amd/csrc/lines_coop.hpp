// lachain_amd/csrc/lines_coop.hpp — the five-lane line-set computation of k_lineset_coop (k_lines.hip header), shared
// by its two instantiations: k_lineset_coop (k_lines.hip, the single-call latency path) and k_lineset_coop_2w
// (k_prep.hip, two waves per SIMD: the census ciphertexts of the fused batched verify, whose waves must find room
// beside the randomisation).
#pragma once
#include "coop_pt.hpp"

#define LS_LANES 5
#define LS_GROUPS 12

struct LsLds { fp2 prod[LS_LANES]; };

DI int ls_role() {
    int r = (int)(threadIdx.x % LS_LANES);
    asm volatile("" : "+v"(r));
    return r;
}
DI void f_sel5(fp2 &r, int role, const fp2 &a, const fp2 &b, const fp2 &c, const fp2 &d, const fp2 &e) {
    f_sel(r, role == 0, a, e);
    f_sel(r, role == 1, b, r);
    f_sel(r, role == 2, c, r);
    f_sel(r, role == 3, d, r);
}
// every lane of the group gets the five lanes' products
DI void ls_xchg(LsLds *L, fp2 (&p)[LS_LANES], const fp2 &m, int role) {
    L->prod[role] = m;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < LS_LANES; k++) p[k] = L->prod[k];
    __syncthreads();
}
DI void ls_round(LsLds *L, fp2 (&p)[LS_LANES], int role, const fp2 &x0, const fp2 &y0, const fp2 &x1, const fp2 &y1,
                 const fp2 &x2, const fp2 &y2, const fp2 &x3, const fp2 &y3, const fp2 &x4, const fp2 &y4) {
    fp2 x, y, m;
    f_sel5(x, role, x0, x1, x2, x3, x4);
    f_sel5(y, role, y0, y1, y2, y3, y4);
    fp2_mul(m, x, y);
    ls_xchg(L, p, m, role);
}
// r = a / 2 (a < p: a even -> a >> 1, odd -> (a + p) >> 1; a + p < 2^382, no carry out)
DI void fp_half(fp &r, const fp &a) {
    const bool odd = a.v[0] & 1u;
    u32 t[12], c = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
        u64 s = (u64)a.v[j] + (odd ? LCB_P[j] : 0u) + c;
        t[j] = (u32)s;
        c = (u32)(s >> 32);
    }
#pragma unroll
    for (int j = 0; j < 11; j++) r.v[j] = (t[j] >> 1) | (t[j + 1] << 31);
    r.v[11] = t[11] >> 1;
}
DI void fp2_half(fp2 &r, const fp2 &a) { fp_half(r.a, a.a); fp_half(r.b, a.b); }
// r = 3 b' x = 12 (1 + u) x (LCB_B2_3): (a + b u)(1 + u) = (a - b) + (a + b) u, times 12 by additions
DI void fp2_mul_b3(fp2 &r, const fp2 &x) {
    fp2 t, t4, t8;
    fp_sub(t.a, x.a, x.b);
    fp_add(t.b, x.a, x.b);
    fp2_add(t4, t, t);
    fp2_add(t4, t4, t4);
    fp2_add(t8, t4, t4);
    fp2_add(r, t8, t4);
}
// line k's un-normalised Bc, Cc, its A and the prefix product acc, one value per lane (roles 0..3)
DI void ls_store_line(u32 *ls, int k, int role, bool st, const fp2 &Bc, const fp2 &Cc, const fp2 &A, const fp2 &acc) {
    if (!st || role > 3) return;
    fp2 v;
    f_sel4(v, role, Bc, Cc, A, acc);
    const u32 off = role == 0 ? k * LCB_NLINE_WORDS
                  : role == 1 ? k * LCB_NLINE_WORDS + 24
                  : role == 2 ? LCB_LS_A + 24 * k : LCB_LS_PRE + 24 * k;
    fp2_store_w(ls + off, v);
}

// k_lineset_fill's contract (line sets of points a prepare kernel stored, sets / w_g2 as there), 12 sets per block
// lds: LS_GROUPS + 1 slots of the calling kernel
DI void lineset_coop_run(LsLds *lds, u32 *lines, u32 n_sets, const u32 *sets, uint8_t *w_g2) {
    LCB_LATENCY_PRIO();
    const u32 g = threadIdx.x / LS_LANES;                // 12 for the shadow lanes 60..63
    const int role = ls_role();
    const u32 k0 = blockIdx.x * LS_GROUPS, kg = k0 + g;
    const bool live = g < LS_GROUPS && kg < n_sets;
    const u32 k = live ? kg : k0;                        // a dead group shadows the block's first set (read only)
    LsLds *L = lds + g;
    u32 *ls = lines + (size_t)(sets ? sets[k] : k) * LCB_LINESET_WORDS;
    g2a Q;
    lineset_get_point(Q, ls);
    const u32 force_general = ls[LCB_LS_FLAG + 2];
    const bool st = live && !Q.inf;                      // this group writes the computed lines
    g2 T;
    T.x = Q.x;
    T.y = Q.y;
    T.z = fp2_one();
    fp2 acc = fp2_one(), p[LS_LANES];
    int kl = 0;
#pragma unroll 1
    for (int i = 62; i >= 0; i--) {
        {   // doubling step: line from T, T <- 2T
            ls_round(L, p, role, T.y, T.y, T.z, T.z, T.x, T.y, T.y, T.z, T.x, T.x);
            fp2 YY = p[0], XY = p[2], YZ = p[3], bZZ, A, Bc, Cc, b9, s, s2, t;
            fp2_mul_b3(bZZ, p[1]);
            fp2_sub(A, YY, bZZ);
            fp2_add(t, p[4], p[4]);
            fp2_add(t, t, p[4]);
            fp2_neg(Bc, t);
            fp2_add(Cc, YZ, YZ);
            fp2_add(b9, bZZ, bZZ);
            fp2_add(b9, b9, bZZ);
            fp2_sub(s, YY, b9);
            fp2_add(s2, YY, b9);
            fp2_half(s2, s2);
            ls_round(L, p, role, XY, s, s2, s2, bZZ, bZZ, YY, YZ, acc, A);
            fp2_half(T.x, p[0]);                         // XY/2 (Y^2 - 9b'Z^2)
            fp2_add(t, p[2], p[2]);
            fp2_add(t, t, p[2]);
            fp2_sub(T.y, p[1], t);                       // ((Y^2 + 9b'Z^2)/2)^2 - 27 b'^2 Z^4
            fp2_add(T.z, p[3], p[3]);                    // 2 Y^3 Z
            acc = p[4];
            ls_store_line(ls, kl, role, st, Bc, Cc, A, acc);
            kl++;
        }
        if ((LCB_Z_ABS >> i) & 1) {                      // addition step: line through T and Q, T <- T + Q
            ls_round(L, p, role, Q.y, T.z, Q.x, T.z, Q.y, T.z, Q.y, T.z, Q.y, T.z);
            fp2 th, la, A, Bc, C, D, H, GH;
            fp2_sub(th, T.y, p[0]);
            fp2_sub(la, T.x, p[1]);
            ls_round(L, p, role, th, Q.x, la, Q.y, th, th, la, la, th, th);
            fp2_sub(A, p[0], p[1]);
            fp2_neg(Bc, th);
            C = p[2];
            D = p[3];
            ls_round(L, p, role, la, D, T.z, C, T.x, D, acc, A, la, D);
            const fp2 E = p[0], G = p[2];
            acc = p[3];
            fp2_add(H, E, p[1]);
            fp2_sub(H, H, G);
            fp2_sub(H, H, G);
            fp2_sub(GH, G, H);
            ls_round(L, p, role, la, H, th, GH, T.y, E, T.z, E, la, H);
            T.x = p[0];
            fp2_sub(T.y, p[1], p[2]);
            T.z = p[3];
            ls_store_line(ls, kl, role, st, Bc, la, A, acc);
            kl++;
        }
    }
    const bool g2m = Q.inf || lineset_in_g2(T, Q);
    const bool ok = Q.inf || !fp2_is_zero(acc);
    fp2 inv;
    fp2_inv_gn(inv, acc);                                // (A_0 ... A_67)^-1 (0 when some A_k = 0: not stored)
    __syncthreads();                                     // the group's line stores are visible to its five lanes
    // backward pass: round j = 67 .. -1 gives a_j (lane 0) and the new inv (lane 1), lanes 2 and 3 normalise line j + 1
    const bool nst = st && ok;
    fp2 a_next = fp2_zero();
#pragma unroll 1
    for (int j = LCB_NLINES - 1; j >= -1; j--) {
        fp2 y = fp2_one();
        const int jn = j + 1;
        if (role == 0 && j > 0) fp2_load_w(y, ls + LCB_LS_PRE + 24 * (j - 1));
        else if (role == 1 && j >= 0) fp2_load_w(y, ls + LCB_LS_A + 24 * j);
        else if (role == 2 && jn < LCB_NLINES) fp2_load_w(y, ls + jn * LCB_NLINE_WORDS);
        else if (role == 3 && jn < LCB_NLINES) fp2_load_w(y, ls + jn * LCB_NLINE_WORDS + 24);
        fp2 x, m;
        f_sel(x, role < 2, inv, a_next);
        fp2_mul(m, x, y);
        if (nst && (role == 2 || role == 3) && jn < LCB_NLINES)
            fp2_store_w(ls + jn * LCB_NLINE_WORDS + (role == 3 ? 24 : 0), m);
        ls_xchg(L, p, m, role);
        a_next = p[0];                                   // a_j = (A_0 ... A_(j-1)) inv... = A_j^-1 (j = 0: inv)
        inv = p[1];                                      // (A_0 ... A_(j-1))^-1
    }
    if (live) {
        if (Q.inf) {                                     // every line the constant 1: B' = C' = 0
            const fp2 z = fp2_zero();
#pragma unroll 1
            for (int q = role; q < LCB_NLINES; q += LS_LANES) {
                fp2_store_w(ls + q * LCB_NLINE_WORDS, z);
                fp2_store_w(ls + q * LCB_NLINE_WORDS + 24, z);
            }
        }
        if (role == 0) {
            ls[LCB_LS_FLAG] = force_general ? 0u : (ok ? 1u : 0u);
            if (w_g2 && (kg & 1)) w_g2[kg >> 1] = g2m ? 1 : 0;
        }
    }
}
