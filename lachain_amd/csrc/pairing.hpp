// lachain_amd/csrc/pairing.hpp — optimal-ate pairing on BLS12-381 for batched share verification.
//
// Miller loop over |z| = 0xd201000000010000 (63 doubling steps, 5 addition steps = 68 lines), z < 0
// handled by a final conjugation.  Lines are computed in homogeneous projective coordinates on the
// twist and written in the sparse shape  l = A + (Bc * xP) v + (Cc * yP) v w, so that everything that
// depends only on the G2 point (A, Bc, Cc) can be PRECOMPUTED ONCE per G2 point and shared by all
// G1 points paired with it (every decryption share of a ciphertext pairs with the same H and W:
// /root/reference/src/Lachain.Crypto/TPKE/PublicKey.cs:88-92).  Line scalings by Fp2 constants are
// killed by the final exponentiation, so the result equals the reference's e(P, Q) exactly.
//   doubling : A = Y^2 - 3b'Z^2, Bc = -3X^2, Cc = 2YZ;  T <- 2T
//   addition : theta = Y - yQ Z, lambda = X - xQ Z, A = theta xQ - lambda yQ, Bc = -theta, Cc = lambda
// Final exponentiation: easy part f^((p^6-1)(p^2+1)), hard part via the decomposition
// 3(p^4-p^2+1)/r = c0 + c1 p + c2 p^2 + c3 p^3 (mcl expHardPartBLS12 shape), cyclotomic squarings.
// GT values therefore equal e(P, Q)^3 of the textbook reduced pairing — the normalisation mcl uses;
// accept/reject decisions are unaffected by it (x -> x^3 is a bijection on mu_r).
#pragma once
#include "curve.hpp"

// word w of parked Fp12 item i (of n) in the quad-major SoA layout (kcommon.hpp)
DI size_t soa_at(size_t n, size_t i, int w) { return ((size_t)(w >> 2) * n + i) * 4 + (w & 3); }

#define LCB_NLINES 68
#define LCB_LINE_WORDS (6 * 12)                      // A, Bc, Cc : three Fp2 (general lines)
// Precomputed line set of one G2 point (device memory, words):
//   [0, 3264)     68 normalised lines (B', C') = (Bc / A, Cc / A), 48 words each: l = 1 + (B' xP) v + (C' yP) v w
//   [3264, 4896)  A_k of each line        (prepare-time scratch for the batched inversion)
//   [4896, 6528)  prefix products A_0..A_k (prepare-time scratch)
//   [6528, 6576)  the affine point (x, y), [6576] flag: 1 = normalised lines valid, 0 = some A_k == 0 (the
//                 Miller loop then computes this point's lines on the fly)
// Scaling a line by the Fp2 constant 1/A multiplies the Miller value by an Fp6 element, which the final
// exponentiation maps to 1 (x^(p^6 - 1) = 1 on Fp6*): decisions and GT values are unchanged, and the sparse
// product by a normalised line costs 9 Fp2 products instead of 13.
#define LCB_NLINE_WORDS 48
#define LCB_LS_A (LCB_NLINES * LCB_NLINE_WORDS)
#define LCB_LS_PRE (LCB_LS_A + LCB_NLINES * 24)
#define LCB_LS_POINT (LCB_LS_PRE + LCB_NLINES * 24)
#define LCB_LS_FLAG (LCB_LS_POINT + 48)
#define LCB_LINESET_WORDS (LCB_LS_FLAG + 16)          // 6592 u32 = 26368 B per G2 point

struct line { fp2 A, Bc, Cc; };

DI void line_dbl_step(g2 &T, line &l) {
    fp2 XX, YY, ZZ, bZZ, t, YZ, b3;
    fp2_load_const(b3, LCB_B2_3);
    fp2_sqr(XX, T.x);
    fp2_sqr(YY, T.y);
    fp2_sqr(ZZ, T.z);
    fp2_mul(bZZ, ZZ, b3);       // 3b'Z^2
    fp2_mul(YZ, T.y, T.z);
    fp2_sub(l.A, YY, bZZ);
    fp2_add(t, XX, XX);
    fp2_add(t, t, XX);
    fp2_neg(l.Bc, t);
    fp2_add(l.Cc, YZ, YZ);
    // X3 = XY/2 (Y^2 - 9b'Z^2), Y3 = ((Y^2 + 9b'Z^2)/2)^2 - 27 b'^2 Z^4, Z3 = 2 Y^3 Z
    fp2 b9, X3, Y3, Z3, s;
    fp inv2;
    fp_load_const(inv2, LCB_INV2);
    fp2_add(b9, bZZ, bZZ);
    fp2_add(b9, b9, bZZ);
    fp2_mul(X3, T.x, T.y);
    fp2_mul_fp(X3, X3, inv2);
    fp2_sub(s, YY, b9);
    fp2_mul(X3, X3, s);
    fp2_add(s, YY, b9);
    fp2_mul_fp(s, s, inv2);
    fp2_sqr(Y3, s);
    fp2_sqr(t, bZZ);
    fp2_add(s, t, t);
    fp2_add(s, s, t);
    fp2_sub(Y3, Y3, s);
    fp2_mul(Z3, YY, YZ);
    fp2_add(Z3, Z3, Z3);
    T.x = X3; T.y = Y3; T.z = Z3;
}
DI void line_add_step(g2 &T, const fp2 &xQ, const fp2 &yQ, line &l) {
    fp2 th, la, t, s;
    fp2_mul(t, yQ, T.z);
    fp2_sub(th, T.y, t);
    fp2_mul(t, xQ, T.z);
    fp2_sub(la, T.x, t);
    fp2_mul(l.A, th, xQ);
    fp2_mul(t, la, yQ);
    fp2_sub(l.A, l.A, t);
    fp2_neg(l.Bc, th);
    l.Cc = la;
    fp2 C, D, E, F, G, H;
    fp2_sqr(C, th);
    fp2_sqr(D, la);
    fp2_mul(E, la, D);
    fp2_mul(F, T.z, C);
    fp2_mul(G, T.x, D);
    fp2_add(H, E, F);
    fp2_sub(H, H, G);
    fp2_sub(H, H, G);
    fp2_mul(T.x, la, H);
    fp2_sub(t, G, H);
    fp2_mul(s, th, t);
    fp2_mul(t, T.y, E);
    fp2_sub(T.y, s, t);
    fp2_mul(T.z, T.z, E);
}
// "one" line (for a point at infinity on either side): A = 1, Bc = Cc = 0
DI void line_one(line &l) { l.A = fp2_one(); l.Bc = fp2_zero(); l.Cc = fp2_zero(); }

DI void line_store(u32 *dst, const line &l) {
    const u32 *s = (const u32 *)&l;
#pragma unroll
    for (int q = 0; q < LCB_LINE_WORDS / 4; q++)
        ((uint4 *)dst)[q] = make_uint4(s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]);
}
DI void line_load(line &l, const u32 *src) {
    u32 *d = (u32 *)&l;
#pragma unroll
    for (int q = 0; q < LCB_LINE_WORDS / 4; q++) {
        uint4 v = ((const uint4 *)src)[q];
        d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
    }
}

DI void fp2_store_w(u32 *dst, const fp2 &x) {
    const u32 *s = (const u32 *)&x;
#pragma unroll
    for (int q = 0; q < 6; q++) ((uint4 *)dst)[q] = make_uint4(s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]);
}
DI void fp2_load_w(fp2 &x, const u32 *src) {
    u32 *d = (u32 *)&x;
#pragma unroll
    for (int q = 0; q < 6; q++) {
        uint4 v = ((const uint4 *)src)[q];
        d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
    }
}

// G2 membership of Q from the Miller loop's last point: the line steps run T from Q through the bits of |z| (top bit
// first), so T = [|z|]Q in homogeneous coordinates (x = X/Z, y = Y/Z), and Q is in G2 iff psi(Q) == [z]Q = -T
// (Scott's test, curve.hpp g2_in_subgroup).  On a point of G2 no step is exceptional (T = +-Q or Y = 0 would need
// (k -+ 1)Q = 0 for some k < r); off G2 an exceptional addition or doubling leaves Z = 0 for every later step, and Z = 0
// is rejected, so the answer is g2_in_subgroup's for every on-curve Q.
DI bool lineset_in_g2(const g2 &T, const g2a &Q) {
    if (fp2_is_zero(T.z)) return false;
    g2 P, S;
    jac_from_aff(P, Q);
    g2_psi(S, P);                                     // psi(Q), affine (Z stays 1)
    fp2 t, ny;
    fp2_mul(t, S.x, T.z);
    bool okx = fp2_eq(t, T.x);
    fp2_mul(t, S.y, T.z);
    fp2_neg(ny, T.y);
    return okx && fp2_eq(t, ny);
}

#define LCB_LS_NORMALISED 1u                          // lineset_compute result bits
#define LCB_LS_IN_G2 2u
// Round 6 (LCB_LEAN_LINES, default): the line steps of lineset_compute with every coefficient stored to the set as soon
// as it is formed (no `line` struct live across the step), the operations ordered so that fewer values are live at once
// (X Y and Y Z first, then the squares; Z3 before the coefficient A), and Q re-read from the set's point slot in the
// five addition steps instead of held across the 68 steps: the loop carries T and the prefix product only.  The same
// operations on the same operands as line_dbl_step / line_add_step, so the same words.
#ifndef LCB_LEAN_LINES
#define LCB_LEAN_LINES 1
#endif
DI void ls_put_line(u32 *dst, int k, const fp2 &A, const fp2 &Bc, const fp2 &Cc, fp2 &acc) {
    fp2_store_w(dst + k * LCB_NLINE_WORDS, Bc);          // not yet normalised
    fp2_store_w(dst + k * LCB_NLINE_WORDS + 24, Cc);
    fp2_store_w(dst + LCB_LS_A + 24 * k, A);
    fp2_mul(acc, acc, A);
    fp2_store_w(dst + LCB_LS_PRE + 24 * k, acc);         // A_0 ... A_k
}
DI void ls_dbl_store(g2 &T, u32 *dst, int k, fp2 &acc) {
    fp2 YZ, XY, ZZ, YY, t, u;
    fp2_mul(YZ, T.y, T.z);
    fp2_mul(XY, T.x, T.y);
    fp2_sqr(ZZ, T.z);                                     // (Z dead)
    fp2_sqr(YY, T.y);                                     // (Y dead)
    fp2_sqr(t, T.x);                                      // XX (X dead)
    fp2_add(u, t, t);
    fp2_add(u, u, t);
    fp2_neg(t, u);                                        // Bc = -3 X^2
    fp2_add(u, YZ, YZ);                                   // Cc = 2 Y Z
    fp2_mul(T.z, YY, YZ);
    fp2_add(T.z, T.z, T.z);                               // Z3 = 2 Y^3 Z  (YZ dead)
    {
        fp2 b3;
        fp2_load_const(b3, LCB_B2_3);
        fp2_mul(ZZ, ZZ, b3);                              // bZZ = 3 b' Z^2
    }
    {
        fp2 A;
        fp2_sub(A, YY, ZZ);                               // A = Y^2 - 3 b' Z^2
        ls_put_line(dst, k, A, t, u, acc);
    }
    fp inv2;
    fp_load_const(inv2, LCB_INV2);
    fp2_add(t, ZZ, ZZ);
    fp2_add(t, t, ZZ);                                    // b9 = 9 b' Z^2
    fp2_mul_fp(XY, XY, inv2);
    fp2_sub(u, YY, t);
    fp2_mul(T.x, XY, u);                                  // X3 = X Y / 2 (Y^2 - 9 b' Z^2)
    fp2_add(u, YY, t);
    fp2_mul_fp(u, u, inv2);
    fp2_sqr(T.y, u);
    fp2_sqr(t, ZZ);
    fp2_add(u, t, t);
    fp2_add(u, u, t);
    fp2_sub(T.y, T.y, u);                                 // Y3 = ((Y^2 + 9 b' Z^2) / 2)^2 - 27 b'^2 Z^4
}
DI void ls_add_store(g2 &T, u32 *dst, int k, fp2 &acc) {
    fp2 xQ, yQ, th, la, t;
    fp2_load_w(xQ, dst + LCB_LS_POINT);
    fp2_load_w(yQ, dst + LCB_LS_POINT + 24);
    fp2_mul(t, yQ, T.z);
    fp2_sub(th, T.y, t);
    fp2_mul(t, xQ, T.z);
    fp2_sub(la, T.x, t);
    {
        fp2 A, nth;
        fp2_mul(A, th, xQ);
        fp2_mul(t, la, yQ);
        fp2_sub(A, A, t);
        fp2_neg(nth, th);
        ls_put_line(dst, k, A, nth, la, acc);
    }
    fp2 D, E, G;
    fp2_sqr(D, la);
    fp2_mul(E, la, D);
    fp2_mul(G, T.x, D);                                   // (X, D dead)
    fp2_sqr(t, th);
    fp2_mul(D, T.z, t);                                   // F = Z C
    fp2_mul(T.z, T.z, E);                                 // Z3 = Z E
    fp2_add(D, E, D);
    fp2_sub(D, D, G);
    fp2_sub(D, D, G);                                     // H = E + F - 2 G
    fp2_mul(T.x, la, D);                                  // X3 = la H
    fp2_sub(t, G, D);
    fp2_mul(G, th, t);
    fp2_mul(t, T.y, E);
    fp2_sub(T.y, G, t);                                   // Y3 = th (G - H) - Y E
}

// the 68 lines of a G2 point (affine, possibly infinity) into dst[LCB_LINESET_WORDS], normalised to A = 1 with
// one Fp2 inversion (Montgomery's batch trick over the 68 A's).  Returns LCB_LS_NORMALISED unless some A_k == 0
// (flag 0), | LCB_LS_IN_G2 when Q lies in G2 (lineset_in_g2; infinity does).
#if LCB_LEAN_LINES
DN u32 lineset_compute(u32 *dst, const g2a &Q) {
    fp2_store_w(dst + LCB_LS_POINT, Q.x);
    fp2_store_w(dst + LCB_LS_POINT + 24, Q.y);
    dst[LCB_LS_FLAG + 1] = Q.inf ? 1 : 0;
    if (Q.inf) {                                      // every line is the constant 1: B' = C' = 0
        fp2 z = fp2_zero();
        for (int k = 0; k < LCB_NLINES; k++) {
            fp2_store_w(dst + k * LCB_NLINE_WORDS, z);
            fp2_store_w(dst + k * LCB_NLINE_WORDS + 24, z);
        }
        dst[LCB_LS_FLAG] = 1;
        return LCB_LS_NORMALISED | LCB_LS_IN_G2;
    }
    g2 T;
    T.x = Q.x; T.y = Q.y; T.z = fp2_one();
    fp2 acc = fp2_one();
    int k = 0;
#pragma unroll 1
    for (int i = 62; i >= 0; i--) {
        ls_dbl_store(T, dst, k++, acc);
        if ((LCB_Z_ABS >> i) & 1) ls_add_store(T, dst, k++, acc);
    }
    u32 g2m;
    {
        g2a Qr;
        fp2_load_w(Qr.x, dst + LCB_LS_POINT);
        fp2_load_w(Qr.y, dst + LCB_LS_POINT + 24);
        Qr.inf = false;
        g2m = lineset_in_g2(T, Qr) ? LCB_LS_IN_G2 : 0u;
    }
    bool ok = !fp2_is_zero(acc);
    dst[LCB_LS_FLAG] = ok;
    if (!ok) return g2m;
    fp2 inv;
    fp2_inv_gn(inv, acc);                              // (A_0 ... A_67)^-1
#pragma unroll 1
    for (k = LCB_NLINES - 1; k >= 0; k--) {
        fp2 ai, a, b, c;
        if (k > 0) {
            fp2 pre;
            fp2_load_w(pre, dst + LCB_LS_PRE + 24 * (k - 1));
            fp2_mul(ai, inv, pre);                     // A_k^-1
        } else {
            ai = inv;
        }
        fp2_load_w(a, dst + LCB_LS_A + 24 * k);
        fp2_mul(inv, inv, a);                          // (A_0 ... A_{k-1})^-1
        fp2_load_w(b, dst + k * LCB_NLINE_WORDS);
        fp2_load_w(c, dst + k * LCB_NLINE_WORDS + 24);
        fp2_mul(b, b, ai);
        fp2_mul(c, c, ai);
        fp2_store_w(dst + k * LCB_NLINE_WORDS, b);
        fp2_store_w(dst + k * LCB_NLINE_WORDS + 24, c);
    }
    return LCB_LS_NORMALISED | g2m;
}
#else
DN u32 lineset_compute(u32 *dst, const g2a &Q) {
    fp2_store_w(dst + LCB_LS_POINT, Q.x);
    fp2_store_w(dst + LCB_LS_POINT + 24, Q.y);
    dst[LCB_LS_FLAG + 1] = Q.inf ? 1 : 0;
    if (Q.inf) {                                      // every line is the constant 1: B' = C' = 0
        fp2 z = fp2_zero();
        for (int k = 0; k < LCB_NLINES; k++) {
            fp2_store_w(dst + k * LCB_NLINE_WORDS, z);
            fp2_store_w(dst + k * LCB_NLINE_WORDS + 24, z);
        }
        dst[LCB_LS_FLAG] = 1;
        return LCB_LS_NORMALISED | LCB_LS_IN_G2;
    }
    g2 T;
    T.x = Q.x; T.y = Q.y; T.z = fp2_one();
    line l;
    fp2 acc = fp2_one();
    int k = 0;
    for (int i = 62; i >= 0; i--) {
        for (int step = 0; step < 2; step++) {
            if (step == 0) line_dbl_step(T, l);
            else if ((LCB_Z_ABS >> i) & 1) line_add_step(T, Q.x, Q.y, l);
            else break;
            fp2_store_w(dst + k * LCB_NLINE_WORDS, l.Bc);      // not yet normalised
            fp2_store_w(dst + k * LCB_NLINE_WORDS + 24, l.Cc);
            fp2_store_w(dst + LCB_LS_A + 24 * k, l.A);
            fp2_mul(acc, acc, l.A);
            fp2_store_w(dst + LCB_LS_PRE + 24 * k, acc);        // A_0 ... A_k
            k++;
        }
    }
    const u32 g2m = lineset_in_g2(T, Q) ? LCB_LS_IN_G2 : 0u;
    bool ok = !fp2_is_zero(acc);
    dst[LCB_LS_FLAG] = ok;
    if (!ok) return g2m;
    fp2 inv;
    fp2_inv_gn(inv, acc);                              // (A_0 ... A_67)^-1
    for (k = LCB_NLINES - 1; k >= 0; k--) {
        fp2 ai, a, b, c;
        if (k > 0) {
            fp2 pre;
            fp2_load_w(pre, dst + LCB_LS_PRE + 24 * (k - 1));
            fp2_mul(ai, inv, pre);                     // A_k^-1
        } else {
            ai = inv;
        }
        fp2_load_w(a, dst + LCB_LS_A + 24 * k);
        fp2_mul(inv, inv, a);                          // (A_0 ... A_{k-1})^-1
        fp2_load_w(b, dst + k * LCB_NLINE_WORDS);
        fp2_load_w(c, dst + k * LCB_NLINE_WORDS + 24);
        fp2_mul(b, b, ai);
        fp2_mul(c, c, ai);
        fp2_store_w(dst + k * LCB_NLINE_WORDS, b);
        fp2_store_w(dst + k * LCB_NLINE_WORDS + 24, c);
    }
    return LCB_LS_NORMALISED | g2m;
}
#endif

// f *= l evaluated at P = (xP, yP)
DI void fp12_mul_line_at(fp12 &f, const line &l, const fp &xP, const fp &yP) {
    fp2 B, C;
    fp2_mul_fp(B, l.Bc, xP);
    fp2_mul_fp(C, l.Cc, yP);
    fp12_mul_line(f, l.A, B, C);
}

// line evaluated at P: (A, Bc xP, Cc yP), or the constant 1 when P is the point at infinity
DI void line_eval(fp2 &A, fp2 &B, fp2 &C, const line &l, const g1a &P) {
    if (P.inf) { A = fp2_one(); B = fp2_zero(); C = fp2_zero(); return; }
    A = l.A;
    fp2_mul_fp(B, l.Bc, P.x);
    fp2_mul_fp(C, l.Cc, P.y);
}
// f *= l1 l2 for two evaluated lines of the same Miller step: the product of the two sparse lines
// (6 Fp2 products, Karatsuba) is L0 + (x v + y v^2) w, and f * L costs 17 Fp2 products — 23 in total instead of
// 2 x 13 for two separate sparse multiplications.  Exact field arithmetic: the same f as line by line.
DI void fp12_mul_line_pair(fp12 &f, const fp2 &A1, const fp2 &B1, const fp2 &C1, const fp2 &A2, const fp2 &B2,
                           const fp2 &C2) {
    fp6 L0, t0, t1;
    fp2 x, y, aa, bb, cc, s, u;
    fp2_mul(aa, A1, A2);
    fp2_mul(bb, B1, B2);
    fp2_mul(cc, C1, C2);
    fp2_mul_xi(s, cc);
    fp2_add(L0.c0, aa, s);
    fp2_add(s, A1, B1);
    fp2_add(u, A2, B2);
    fp2_mul(L0.c1, s, u);
    fp2_sub(L0.c1, L0.c1, aa);
    fp2_sub(L0.c1, L0.c1, bb);
    L0.c2 = bb;
    fp2_add(s, A1, C1);
    fp2_add(u, A2, C2);
    fp2_mul(x, s, u);
    fp2_sub(x, x, aa);
    fp2_sub(x, x, cc);
    fp2_add(s, B1, C1);
    fp2_add(u, B2, C2);
    fp2_mul(y, s, u);
    fp2_sub(y, y, bb);
    fp2_sub(y, y, cc);
    // t1 = f1 * (x v + y v^2): c0 = xi((a1 + a2)(x + y) - a1 x - a2 y), c1 = a0 x + xi a2 y, c2 = a0 y + a1 x
    {
        fp2 a0x, a0y, a1x, a2y;
        fp2_mul(a0x, f.c1.c0, x);
        fp2_mul(a0y, f.c1.c0, y);
        fp2_mul(a1x, f.c1.c1, x);
        fp2_mul(a2y, f.c1.c2, y);
        fp2_add(s, f.c1.c1, f.c1.c2);
        fp2_add(u, x, y);
        fp2_mul(s, s, u);
        fp2_sub(s, s, a1x);
        fp2_sub(s, s, a2y);
        fp2_mul_xi(t1.c0, s);
        fp2_mul_xi(s, a2y);
        fp2_add(t1.c1, a0x, s);
        fp2_add(t1.c2, a0y, a1x);
    }
    // f1' = (f0 + f1)(L0 + L1) - t0 - t1, f0' = t0 + v t1 (f updated in place)
    fp6_mul(t0, f.c0, L0);
    fp6_add(f.c1, f.c0, f.c1);
    fp2_add(L0.c1, L0.c1, x);
    fp2_add(L0.c2, L0.c2, y);
    fp6_mul(f.c1, f.c1, L0);
    fp6_sub(f.c1, f.c1, t0);
    fp6_sub(f.c1, f.c1, t1);
    fp6_mul_v(t1, t1);
    fp6_add(f.c0, t0, t1);
}

// f *= 1 + b v + c v w  (a normalised line evaluated at P: b = B' xP, c = C' yP), Karatsuba over Fp6 with
// X = v f0, Y = v f1:  f0' = f0 + b X + v (c Y),  f1' = f1 + (b + c)(X + Y) - b X - c Y  — 9 Fp2 products.
// The three coefficient positions are processed in the order 2, 1, 0 so f is updated in place: position k reads
// X_k = f0_{k-1}, Y_k = f1_{k-1} (X_0 = xi f0_2, Y_0 = xi f1_2, taken first).
DI void fp12_mul_line_n(fp12 &f, const fp2 &b, const fp2 &c) {
    fp2 bc, X0, Y0, t12;
    fp2_add(bc, b, c);
    fp2_mul_xi(X0, f.c0.c2);
    fp2_mul_xi(Y0, f.c1.c2);
    fp2 *f0[3] = {&f.c0.c0, &f.c0.c1, &f.c0.c2};
    fp2 *f1[3] = {&f.c1.c0, &f.c1.c1, &f.c1.c2};
    // v (c Y) = (xi t1_2, t1_0, t1_1) is folded in as soon as each t1_k exists: t1_1 into f0_2 (no longer read),
    // t1_0 into f0_1 (read as X_2 before), only t1_2 waits for the end (f0_0 is X_1)
#pragma unroll
    for (int k = 2; k >= 0; k--) {
        const fp2 &X = k == 0 ? X0 : *f0[k - 1];
        const fp2 &Y = k == 0 ? Y0 : *f1[k - 1];
        fp2 t0, t1, s, u;
        fp2_mul(t0, b, X);
        fp2_mul(t1, c, Y);
        fp2_add(u, X, Y);
        fp2_mul(s, bc, u);
        fp2_sub(s, s, t0);
        fp2_sub(s, s, t1);
        fp2_add(*f1[k], *f1[k], s);                    // f1_k is not read after position k
        fp2_add(*f0[k], *f0[k], t0);                   // f0_k was last read as X_{k+1}
        if (k == 2) t12 = t1;
        else fp2_add(*f0[k + 1], *f0[k + 1], t1);      // f0_2 += t1_1, f0_1 += t1_0
    }
    fp2 w;
    fp2_mul_xi(w, t12);
    fp2_add(f.c0.c0, f.c0.c0, w);
}

// Line sources for the two-pair Miller loop: apply(f, P, is_add) multiplies f by the source's next line
// evaluated at P (a point at infinity contributes 1)
struct LinesFromMemory {   // general (A, Bc, Cc) lines, LCB_LINE_WORDS each
    const u32 *p;
    DI void next(line &l, bool) { line_load(l, p); p += LCB_LINE_WORDS; }
    DI void apply(fp12 &f, const g1a &P, bool is_add) {
        line l;
        next(l, is_add);
        if (!P.inf) fp12_mul_line_at(f, l, P.x, P.y);
    }
};
struct LinesOnTheFly {
    g2 T; fp2 xQ, yQ; bool inf;
    DI void init(const g2a &Q) { inf = Q.inf; xQ = Q.x; yQ = Q.y; T.x = Q.x; T.y = Q.y; T.z = fp2_one(); }
    DI void next(line &l, bool is_add) {
        if (inf) { line_one(l); return; }
        if (is_add) line_add_step(T, xQ, yQ, l);
        else line_dbl_step(T, l);
    }
    DI void apply(fp12 &f, const g1a &P, bool is_add) {
        line l;
        next(l, is_add);
        if (!P.inf) fp12_mul_line_at(f, l, P.x, P.y);
    }
};
struct LinesNorm {          // normalised lines of a line set (lineset_compute)
    const u32 *p;
    DI void apply(fp12 &f, const g1a &P, bool) {
        fp2 b, c;
        fp2_load_w(b, p);
        fp2_load_w(c, p + 24);
        p += LCB_NLINE_WORDS;
        if (P.inf) return;
        fp2_mul_fp(b, b, P.x);
        fp2_mul_fp(c, c, P.y);
        fp12_mul_line_n(f, b, c);
    }
};
// the same, with its G1 point parked in LDS (6 quads per lane, quad q at pt[q * LCB_BLOCK_PTS]) and re-read at
// every line: keeps the point's 24 words out of the Miller loop's live registers (the loop otherwise spills)
#define LCB_BLOCK_PTS 256
struct LinesNormLds {
    const u32 *p;
    const uint4 *pt;
    bool inf;
    DI void apply(fp12 &f, const g1a &, bool) {
        fp2 b, c;
        fp2_load_w(b, p);
        fp2_load_w(c, p + 24);
        p += LCB_NLINE_WORDS;
        if (inf) return;
        asm volatile("" ::: "memory");                // re-read the point: not kept live across the loop
        fp x, y;
        u32 *xw = x.v, *yw = y.v;
#pragma unroll
        for (int q = 0; q < 3; q++) {
            uint4 vx = pt[q * LCB_BLOCK_PTS], vy = pt[(3 + q) * LCB_BLOCK_PTS];
            xw[4 * q] = vx.x; xw[4 * q + 1] = vx.y; xw[4 * q + 2] = vx.z; xw[4 * q + 3] = vx.w;
            yw[4 * q] = vy.x; yw[4 * q + 1] = vy.y; yw[4 * q + 2] = vy.z; yw[4 * q + 3] = vy.w;
        }
        fp2_mul_fp(b, b, x);
        fp2_mul_fp(c, c, y);
        fp12_mul_line_n(f, b, c);
    }
};
// f *= the normalised line at lp evaluated at the point parked at pt (nothing for a point at infinity)
DI void apply_norm_lds(fp12 &f, const u32 *lp, const uint4 *pt, bool inf) {
    fp2 b, c;
    fp2_load_w(b, lp);
    fp2_load_w(c, lp + 24);
    if (inf) return;
    asm volatile("" ::: "memory");
    fp x, y;
    u32 *xw = x.v, *yw = y.v;
#pragma unroll
    for (int q = 0; q < 3; q++) {
        uint4 vx = pt[q * LCB_BLOCK_PTS], vy = pt[(3 + q) * LCB_BLOCK_PTS];
        xw[4 * q] = vx.x; xw[4 * q + 1] = vx.y; xw[4 * q + 2] = vx.z; xw[4 * q + 3] = vx.w;
        yw[4 * q] = vy.x; yw[4 * q + 1] = vy.y; yw[4 * q + 2] = vy.z; yw[4 * q + 3] = vy.w;
    }
    fp2_mul_fp(b, b, x);
    fp2_mul_fp(c, c, y);
    fp12_mul_line_n(f, b, c);
}
// miller2 over two normalised line sets with LDS-parked points, written as a loop over the 68 lines so the
// squaring and the line product each appear ONCE in the code (the bit-driven form inlines the line product
// four times: ~150 KB of loop body, beyond the instruction cache)
DI void miller2_norm_lds(fp12 &f, const u32 *ls1, const uint4 *pt1, bool inf1, const u32 *ls2, const uint4 *pt2,
                         bool inf2) {
    f = fp12_one();
    int i = 62;
    bool add_next = false;
#pragma unroll 1
    for (int k = 0; k < LCB_NLINES; k++) {
        if (add_next) {
            add_next = false;
        } else {
            if (k > 0) fp12_sqr(f, f);
            add_next = (LCB_Z_ABS >> i) & 1;
            i--;
        }
#pragma unroll 1
        for (int s = 0; s < 2; s++) {
            const u32 *lp = (s == 0 ? ls1 : ls2) + (size_t)k * LCB_NLINE_WORDS;
            apply_norm_lds(f, lp, s == 0 ? pt1 : pt2, s == 0 ? inf1 : inf2);
        }
    }
    fp12_conj(f, f);
}
DI void g1_park_lds(uint4 *pt, const g1a &P) {
    const u32 *x = P.x.v, *y = P.y.v;
#pragma unroll
    for (int q = 0; q < 3; q++) {
        pt[q * LCB_BLOCK_PTS] = make_uint4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
        pt[(3 + q) * LCB_BLOCK_PTS] = make_uint4(y[4 * q], y[4 * q + 1], y[4 * q + 2], y[4 * q + 3]);
    }
}
DI bool lineset_normalised(const u32 *ls) { return ls[LCB_LS_FLAG] != 0; }
DI void lineset_point(g2a &Q, const u32 *ls) {
    fp2_load_w(Q.x, ls + LCB_LS_POINT);
    fp2_load_w(Q.y, ls + LCB_LS_POINT + 24);
    Q.inf = ls[LCB_LS_FLAG + 1] != 0;
}
// a prepare kernel stores the point; k_lineset_fill computes its lines
DI void lineset_put_point(u32 *ls, const g2a &Q) {
    fp2_store_w(ls + LCB_LS_POINT, Q.x);
    fp2_store_w(ls + LCB_LS_POINT + 24, Q.y);
    ls[LCB_LS_FLAG + 1] = Q.inf ? 1 : 0;
}
DI void lineset_get_point(g2a &Q, const u32 *ls) { lineset_point(Q, ls); }

// f = prod_k f_{|z|, Q_k}(P_k), conjugated (z < 0).  A pair whose G1 point is infinity contributes 1.  (Multiplying the
// two lines of a step together first, 23 instead of 26 Fp2 products, measured slower: k_tpke_miller 227 -> 232 ms per
// 1M shares, the six live evaluated Fp2 values doubled the spill traffic.)
template <class S1, class S2>
DI void miller2(fp12 &f, S1 &s1, const g1a &P1, S2 &s2, const g1a &P2) {
    f = fp12_one();
    bool first = true;
    for (int i = 62; i >= 0; i--) {
        if (!first) fp12_sqr(f, f);
        first = false;
        s1.apply(f, P1, false);
        s2.apply(f, P2, false);
        if ((LCB_Z_ABS >> i) & 1) {
            s1.apply(f, P1, true);
            s2.apply(f, P2, true);
        }
    }
    fp12_conj(f, f);
}
template <class S1>
DI void miller1(fp12 &f, S1 &s1, const g1a &P1) {
    f = fp12_one();
    bool first = true;
    for (int i = 62; i >= 0; i--) {
        if (!first) fp12_sqr(f, f);
        first = false;
        s1.apply(f, P1, false);
        if ((LCB_Z_ABS >> i) & 1) s1.apply(f, P1, true);
    }
    fp12_conj(f, f);
}
// two-pair Miller loop over two line sets: normalised lines where the set has them, otherwise the set's point's
// lines on the fly (only for a point with some A_k == 0: never for the outputs of hashing or honest ciphertexts)
DN void miller2_sets_fallback(fp12 &f, const u32 *ls1, const g1a &P1, const u32 *ls2, const g1a &P2) {
    g2a Q;
    if (lineset_normalised(ls1)) {
        LinesNorm s1{ls1};
        lineset_point(Q, ls2);
        LinesOnTheFly s2;
        s2.init(Q);
        miller2(f, s1, P1, s2, P2);
    } else if (lineset_normalised(ls2)) {
        lineset_point(Q, ls1);
        LinesOnTheFly s1;
        s1.init(Q);
        LinesNorm s2{ls2};
        miller2(f, s1, P1, s2, P2);
    } else {
        lineset_point(Q, ls1);
        LinesOnTheFly s1;
        s1.init(Q);
        lineset_point(Q, ls2);
        LinesOnTheFly s2;
        s2.init(Q);
        miller2(f, s1, P1, s2, P2);
    }
}
DI void miller2_sets(fp12 &f, const u32 *ls1, const g1a &P1, const u32 *ls2, const g1a &P2) {
    if (lineset_normalised(ls1) && lineset_normalised(ls2)) {
        LinesNorm s1{ls1}, s2{ls2};
        miller2(f, s1, P1, s2, P2);
    } else {
        miller2_sets_fallback(f, ls1, P1, ls2, P2);
    }
}

// ---------------------------------------------------------------- final exponentiation
DN void fe_easy(fp12 &r, const fp12 &f) {
    fp12 t0, t1;
    fp12_conj(t0, f);
    fp12_inv_n(t1, f);
    fp12_mul_n(t0, t0, t1);  // f^(p^6 - 1)
    fp12_frob2_n(t1, t0);
    fp12_mul_n(r, t1, t0);   // ^(p^2 + 1)
}
// x^z for unitary x (z = -|z|): cyclotomic square-and-multiply over |z|, then conjugate
DN void cyc_pow_z(fp12 &r, const fp12 &x) {
    fp12 acc = x;
    fp12 base = x; // kept in registers for the whole loop (the squaring chain never touches memory)
    for (int i = 62; i >= 0; i--) {
        fp12_cyc_sqr(acc, acc);
        if ((LCB_Z_ABS >> i) & 1) fp12_mul(acc, acc, base);
    }
    fp12_conj(r, acc);
}
// Same exponent and product as mcl's expHardPartBLS12 (y = x^c0 (x^c1)^p (x^c2)^p^2 (x^c3)^p^3), evaluated
// in an order that folds each Frobenius term into the accumulator as soon as its power is available, so at
// most five Fp12 values (x, t, u, v, acc) are live at once instead of nine: every live Fp12 beyond the
// register file is 576 B of per-lane scratch, and scratch traffic is what bounds this kernel.
DN void fe_hard(fp12 &y, const fp12 &x) {
    fp12 t, u, v, acc, w;
    cyc_pow_z(t, x);              // t = x^z
    fp12_conj(u, x);
    fp12_cyc_sqr_n(u, u);         // x^-2
    fp12_mul_n(u, u, t);          // u = x^(z-2)
    cyc_pow_z(v, u);              // v = x^(z^2-2z)
    fp12_mul_n(acc, v, x);        // x^c3
    fp12_frob3_n(acc, acc);
    cyc_pow_z(v, v);              // v = x^(z^3-2z^2)
    fp12_mul_n(w, v, t);          // x^c2
    fp12_frob2_n(w, w);
    fp12_mul_n(acc, acc, w);
    cyc_pow_z(v, v);              // v = x^(z^4-2z^3)
    fp12_cyc_sqr_n(t, t);         // t = x^2z
    fp12_mul_n(v, v, t);          // v = x^(z^4-2z^3+2z)
    fp12_conj(w, x);
    fp12_mul_n(w, w, v);          // x^c1
    fp12_frob1_n(w, w);
    fp12_mul_n(acc, acc, w);
    cyc_pow_z(v, v);              // v = x^(z^5-2z^4+2z^2)
    fp12_conj(u, u);              // x^(2-z)
    fp12_mul_n(u, u, v);
    fp12_mul_n(u, u, x);          // x^c0
    fp12_mul_n(y, acc, u);
}
// in place: fe_easy and fe_hard read their input before writing their output, so no third Fp12 frame
DN void final_exp_inplace(fp12 &f) {
    fe_easy(f, f);
    fe_hard(f, f);
}
DN void final_exp(fp12 &r, const fp12 &f) {
    r = f;
    final_exp_inplace(r);
}
