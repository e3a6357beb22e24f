#!/usr/bin/env python3
"""tools/gen_asm.py — emits lachain_amd/csrc/asm_routines.hpp: hand-scheduled gfx950 assembly leaf
routines for the hot field arithmetic, with a custom register calling convention, plus the HIP wrappers
that call them.

Why: the pairing runs one lane per share with ~400 live VGPRs (one wave per SIMD).  A compiler-built
Montgomery multiply is a single dependent MAC chain (each v_mad_u64_u32 waits ~12 cycles for the previous
one: profiles/r01_valu_rates.jsonl), and passing Fp2 operands to a non-inlined function goes through
scratch (the AMDGPU ABI passes aggregates >16 registers in memory).  These routines instead take their
operands in fixed VGPRs (v0..), interleave 2-3 independent Montgomery products column by column
(product-scanning / FIPS Montgomery, 12x32-bit limbs, R = 2^384) so consecutive MACs are independent,
and give each product chain its own SGPR carry pair.  Callers reach them with `s_swappc_b64` from inline
asm whose register-tuple constraints and clobber list tell the compiler exactly which registers move.

Per MAC: `v_mad_u64_u32 acc, s[c], x, y, acc` (half rate) + `v_addc_co_u32 hi, s[c], 0, hi, s[c]`.
Modulus limbs live in VGPRs inside a routine (GFX9 VOP3 reads at most one SGPR per instruction).
All routine outputs are fully reduced (< p); unreduced Karatsuba sums (< 2p) are valid multiplicands
because R > 4p.

Routines (label: inputs -> outputs, all 12-limb little-endian Montgomery):
  lcb_r_fp_mul      v[0:11]=a, v[12:23]=b                 -> v[0:11]=a*b
  lcb_r_fp_sqr      v[0:11]=a                             -> v[0:11]=a^2   (78 products for a*a)
  lcb_r_fp_mul2     v[0:11]=a0, v[12:23]=b0, v[24:35]=a1, v[36:47]=b1 -> v[0:11]=a0*b0, v[24:35]=a1*b1
  lcb_r_fp2_mul     v[0:23]=x, v[24:47]=y                 -> v[0:23]=x*y   (Karatsuba, 3 chains)
  lcb_r_fp2_sqr     v[0:23]=x                             -> v[0:23]=x^2   ((a+b)(a-b), 2ab: 2 chains)
  lcb_r_fp2_mul_fp  v[0:23]=x, v[24:35]=s                 -> v[0:23]=x*s   (2 chains)
"""
import os

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
N = 12
PINV = (-pow(P, -1, 1 << 32)) % (1 << 32)
PL = [(P >> (32 * i)) & 0xFFFFFFFF for i in range(N)]

S_PINV = 88
CARRY = [90, 92, 94]          # per-chain carry SGPR pairs
S_TMP = 96                    # scratch carry pair for add/sub chains (s[96:97])
S_TMP2 = 98                   # second scratch pair (s[98:99])
CLOBBER_SGPRS = [30, 31, S_PINV] + [c + d for c in CARRY for d in (0, 1)] + [S_TMP, S_TMP + 1, S_TMP2, S_TMP2 + 1]


def v(i):
    return f"v{i}"


def vr(base):
    return [base + j for j in range(N)]


class Asm:
    def __init__(self):
        self.lines = []

    def __call__(self, s):
        self.lines.append("  " + s)

    def label(self, name):
        self.lines.append(f"{name}:")

    def text(self):
        return "\n".join(self.lines)


def load_p(a, pbase):
    for j in range(N):
        a(f"v_mov_b32 v{pbase + j}, 0x{PL[j]:08x}")
    a(f"s_mov_b32 s{S_PINV}, 0x{PINV:08x}")


def products(a, chains, pbase):
    """chains: list of dict(a=[12 regs], b=[12 regs], m=[12 regs], acc=reg base (4 regs, even), out=[12 regs]).
    out[j] may alias a[j] (written after a[j]'s last use).  Results are in [0, 2p) (not yet reduced).

    Column accumulator = an even-aligned 64-bit pair (v_mad_u64_u32 needs aligned pairs on gfx950) plus a
    carry word, rotated through a 4-register ring so the 32-bit shift between columns is one v_mov:
    even columns use pair (R0,R1) + carry R3, odd columns pair (R2,R3) + carry R1.  The first carry add of
    a column writes the fresh carry word (0 + 0 + carry), so it needs no zeroing."""
    def ring(c, k):
        r = c["acc"]
        return (r, r + 1, r + 3) if k % 2 == 0 else (r + 2, r + 3, r + 1)

    for c in chains:
        acc = c["acc"]
        a(f"v_mov_b32 v{acc}, 0")
        a(f"v_mov_b32 v{acc + 1}, 0")
    for k in range(2 * N - 1):
        lo = 0 if k < N else k - (N - 1)
        up = k if k < N else N - 1
        terms = []
        for i in range(lo, up + 1):
            terms.append(("ab", i, k - i))
            if i < k:
                terms.append(("mp", i, k - i))
        if k < N:
            terms.append(("m", k, 0))
        for n_t, (kind, i, j) in enumerate(terms):
            if kind == "m":
                for t, c in enumerate(chains):
                    a(f"v_mul_lo_u32 v{c['m'][k]}, v{ring(c, k)[0]}, s{S_PINV}")
            for t, c in enumerate(chains):
                L, H, C = ring(c, k)
                if kind == "ab":
                    x, y = c["a"][i], c["b"][j]
                elif kind == "mp":
                    x, y = c["m"][i], pbase + j
                else:
                    x, y = c["m"][k], pbase
                a(f"v_mad_u64_u32 v[{L}:{H}], s[{CARRY[t]}:{CARRY[t] + 1}], v{x}, v{y}, v[{L}:{H}]")
            for t, c in enumerate(chains):
                L, H, C = ring(c, k)
                sc = f"s[{CARRY[t]}:{CARRY[t] + 1}]"
                if n_t == 0:
                    a(f"v_addc_co_u32_e64 v{C}, {sc}, 0, 0, {sc}")
                else:
                    a(f"v_addc_co_u32_e64 v{C}, {sc}, 0, v{C}, {sc}")
        for c in chains:
            L, H, C = ring(c, k)
            if k >= N:
                a(f"v_mov_b32 v{c['out'][k - N]}, v{L}")
            if k == 2 * N - 2:
                a(f"v_mov_b32 v{c['out'][N - 1]}, v{H}")   # top carry word is 0: result < 2p < 2^384
            else:
                L2, H2, C2 = ring(c, k + 1)
                assert H2 == C
                a(f"v_mov_b32 v{L2}, v{H}")


def reduce_once(a, r, tmp, pbase, sc=S_TMP):
    """r <- r - p if r >= p (r < 2p).  tmp: 12 scratch VGPRs."""
    a(f"v_sub_co_u32_e64 v{tmp[0]}, s[{sc}:{sc + 1}], v{r[0]}, v{pbase}")
    for j in range(1, N):
        a(f"v_subb_co_u32_e64 v{tmp[j]}, s[{sc}:{sc + 1}], v{r[j]}, v{pbase + j}, s[{sc}:{sc + 1}]")
    for j in range(N):
        a(f"v_cndmask_b32_e64 v{r[j]}, v{tmp[j]}, v{r[j]}, s[{sc}:{sc + 1}]")


def add_unreduced(a, r, x, y, sc=S_TMP):
    """r <- x + y (no reduction; x, y < p so r < 2p < 2^382)."""
    a(f"v_add_co_u32_e64 v{r[0]}, s[{sc}:{sc + 1}], v{x[0]}, v{y[0]}")
    for j in range(1, N):
        a(f"v_addc_co_u32_e64 v{r[j]}, s[{sc}:{sc + 1}], v{x[j]}, v{y[j]}, s[{sc}:{sc + 1}]")


def sub_plus_p(a, r, x, y, pbase, sc=S_TMP):
    """r <- x - y + p (no reduction; in (0, 2p) for x, y < p)."""
    a(f"v_sub_co_u32_e64 v{r[0]}, s[{sc}:{sc + 1}], v{x[0]}, v{y[0]}")
    for j in range(1, N):
        a(f"v_subb_co_u32_e64 v{r[j]}, s[{sc}:{sc + 1}], v{x[j]}, v{y[j]}, s[{sc}:{sc + 1}]")
    a(f"v_add_co_u32_e64 v{r[0]}, s[{sc}:{sc + 1}], v{r[0]}, v{pbase}")
    for j in range(1, N):
        a(f"v_addc_co_u32_e64 v{r[j]}, s[{sc}:{sc + 1}], v{r[j]}, v{pbase + j}, s[{sc}:{sc + 1}]")


def sub_mod(a, r, x, y, tmp, pbase):
    """r <- x - y mod p (x, y < p); r may alias x or y."""
    sc, sc2 = S_TMP, S_TMP2
    a(f"v_sub_co_u32_e64 v{tmp[0]}, s[{sc}:{sc + 1}], v{x[0]}, v{y[0]}")
    for j in range(1, N):
        a(f"v_subb_co_u32_e64 v{tmp[j]}, s[{sc}:{sc + 1}], v{x[j]}, v{y[j]}, s[{sc}:{sc + 1}]")
    # r = borrow ? tmp + p : tmp
    a(f"v_add_co_u32_e64 v{r[0]}, s[{sc2}:{sc2 + 1}], v{tmp[0]}, v{pbase}")
    for j in range(1, N):
        a(f"v_addc_co_u32_e64 v{r[j]}, s[{sc2}:{sc2 + 1}], v{tmp[j]}, v{pbase + j}, s[{sc2}:{sc2 + 1}]")
    for j in range(N):
        a(f"v_cndmask_b32_e64 v{r[j]}, v{tmp[j]}, v{r[j]}, s[{sc}:{sc + 1}]")


def add_mod(a, r, x, y, tmp, pbase):
    """r <- x + y mod p (x, y < p)."""
    add_unreduced(a, r, x, y)
    reduce_once(a, r, tmp, pbase)


def mov(a, dst, src):
    for j in range(N):
        a(f"v_mov_b32 v{dst[j]}, v{src[j]}")


# ------------------------------------------------------------------ routines
def r_fp_mul():
    a = Asm()
    a.label("lcb_r_fp_mul")
    P_ = 40
    load_p(a, P_)
    A, B, M = vr(0), vr(12), vr(24)
    products(a, [dict(a=A, b=B, m=M, acc=36, out=A)], P_)
    reduce_once(a, A, M, P_)
    a("s_setpc_b64 s[30:31]")
    return a.text(), 52


def r_fp_mul2():
    a = Asm()
    a.label("lcb_r_fp_mul2")
    P_ = 80
    load_p(a, P_)
    A0, B0, A1, B1, M0, M1 = vr(0), vr(12), vr(24), vr(36), vr(48), vr(60)
    products(a, [dict(a=A0, b=B0, m=M0, acc=72, out=A0), dict(a=A1, b=B1, m=M1, acc=76, out=A1)], P_)
    reduce_once(a, A0, M0, P_)
    reduce_once(a, A1, M1, P_)
    a("s_setpc_b64 s[30:31]")
    return a.text(), 92


def products_sqr(a, A, F, E, M, acc, pbase):
    """Montgomery square of A (FIPS as products(), one chain): a^2 = sum_i a_i 2^(32i) W_i with
    W_i = a_i 2^(32i) + 2 sum_{j>i} a_j 2^(32j), whose limbs are a_i (j = i), F[j] = a_j << 1 (j = i + 1) and
    E[j] = limb j of 2a = (a_j << 1) | (a_{j-1} >> 31) (j > i + 1; a_11 < 2^29, so no limb 12): 78 products
    instead of 144 for the a*a half.  F, E are indexed by limb (dicts); the result (< 2p) is written over A."""
    def ring(k):
        return (acc, acc + 1, acc + 3) if k % 2 == 0 else (acc + 2, acc + 3, acc + 1)

    a(f"v_mov_b32 v{acc}, 0")
    a(f"v_mov_b32 v{acc + 1}, 0")
    sc = f"s[{CARRY[0]}:{CARRY[0] + 1}]"
    for k in range(2 * N - 1):
        terms = []
        for i in range(max(0, k - (N - 1)), k // 2 + 1):
            j = k - i
            terms.append(("sq", A[i], A[i] if j == i else (F[j] if j == i + 1 else E[j])))
        lo = 0 if k < N else k - (N - 1)
        up = k if k < N else N - 1
        for i in range(lo, up + 1):
            if i < k:
                terms.append(("mp", M[i], pbase + k - i))
        if k < N:
            terms.append(("m", M[k], pbase))
        L, H, C = ring(k)
        for n_t, (kind, x, y) in enumerate(terms):
            if kind == "m":
                a(f"v_mul_lo_u32 v{M[k]}, v{L}, s{S_PINV}")
            a(f"v_mad_u64_u32 v[{L}:{H}], {sc}, v{x}, v{y}, v[{L}:{H}]")
            if n_t == 0:
                a(f"v_addc_co_u32_e64 v{C}, {sc}, 0, 0, {sc}")
            else:
                a(f"v_addc_co_u32_e64 v{C}, {sc}, 0, v{C}, {sc}")
        if k >= N:
            a(f"v_mov_b32 v{A[k - N]}, v{L}")      # A[k-N]'s last use (as a_i, i <= k - 12 ... ) was column k - 1
        if k == 2 * N - 2:
            a(f"v_mov_b32 v{A[N - 1]}, v{H}")
        else:
            L2, H2, C2 = ring(k + 1)
            assert H2 == C
            a(f"v_mov_b32 v{L2}, v{H}")


def r_fp_sqr():
    a = Asm()
    a.label("lcb_r_fp_sqr")
    P_ = 50
    load_p(a, P_)
    A = vr(0)
    F = {j: 11 + j for j in range(1, N)}          # v12..v22
    E = {j: 21 + j for j in range(2, N)}          # v23..v32
    M = [33 + j for j in range(N)]                # v33..v44
    for j in range(1, N):
        a(f"v_lshlrev_b32 v{F[j]}, 1, v{A[j]}")
    for j in range(2, N):
        a(f"v_alignbit_b32 v{E[j]}, v{A[j]}, v{A[j - 1]}, 31")
    products_sqr(a, A, F, E, M, 46, P_)
    reduce_once(a, A, M, P_)
    a("s_setpc_b64 s[30:31]")
    return a.text(), 62


def r_fp2_sqr():
    a = Asm()
    a.label("lcb_r_fp2_sqr")
    P_ = 80
    load_p(a, P_)
    XA, XB, S, D, M0, M1 = vr(0), vr(12), vr(24), vr(36), vr(48), vr(60)
    add_unreduced(a, S, XA, XB)       # a + b   (< 2p)
    sub_plus_p(a, D, XA, XB, P_)      # a - b + p (< 2p)
    products(a, [dict(a=S, b=D, m=M0, acc=72, out=S),
                 dict(a=XA, b=XB, m=M1, acc=76, out=XA)], P_)
    reduce_once(a, S, M0, P_)         # r.a = a^2 - b^2
    reduce_once(a, XA, M1, P_)        # ab
    add_mod(a, XB, XA, XA, M1, P_)    # r.b = 2ab
    mov(a, XA, S)
    a("s_setpc_b64 s[30:31]")
    return a.text(), 92


def r_fp2_mul_fp():
    a = Asm()
    a.label("lcb_r_fp2_mul_fp")
    P_ = 80
    load_p(a, P_)
    XA, XB, S, M0, M1 = vr(0), vr(12), vr(24), vr(36), vr(48)
    products(a, [dict(a=XA, b=S, m=M0, acc=72, out=XA), dict(a=XB, b=S, m=M1, acc=76, out=XB)], P_)
    reduce_once(a, XA, M0, P_)
    reduce_once(a, XB, M1, P_)
    a("s_setpc_b64 s[30:31]")
    return a.text(), 92


# ------------------------------------------------------------------ lazy (double-width) reduction
P2X4 = 4 * P * P          # 4p^2 < 2^764: keeps T0 - T1 + 4p^2 positive for multiplicands < 2p
P2X4L = [(P2X4 >> (32 * i)) & 0xFFFFFFFF for i in range(2 * N)]


def products_plain(a, chains):
    """Comba products T = a*b (24 words) for interleaved chains: dict(a=[12], b=[12], acc=base (4 regs, even),
    out=[24 regs]).  out[k] is written at the end of column k and may alias a[k-11] (k >= 11: a[k-11]'s last
    use is column k) — that is how the 24-word products fit in the registers the operands free."""
    def ring(c, k):
        r = c["acc"]
        return (r, r + 1, r + 3) if k % 2 == 0 else (r + 2, r + 3, r + 1)

    for c in chains:
        a(f"v_mov_b32 v{c['acc']}, 0")
        a(f"v_mov_b32 v{c['acc'] + 1}, 0")
    for k in range(2 * N - 1):
        terms = [(i, k - i) for i in range(max(0, k - (N - 1)), min(k, N - 1) + 1)]
        for n_t, (i, j) in enumerate(terms):
            for t, c in enumerate(chains):
                L, H, C = ring(c, k)
                a(f"v_mad_u64_u32 v[{L}:{H}], s[{CARRY[t]}:{CARRY[t] + 1}], v{c['a'][i]}, v{c['b'][j]}, v[{L}:{H}]")
            for t, c in enumerate(chains):
                L, H, C = ring(c, k)
                sc = f"s[{CARRY[t]}:{CARRY[t] + 1}]"
                a(f"v_addc_co_u32_e64 v{C}, {sc}, 0, {0 if n_t == 0 else 'v%d' % C}, {sc}")
        for c in chains:
            L, H, C = ring(c, k)
            a(f"v_mov_b32 v{c['out'][k]}, v{L}")
            if k == 2 * N - 2:
                a(f"v_mov_b32 v{c['out'][2 * N - 1]}, v{H}")   # top word; the carry word is 0 (T < 2^768)
            else:
                L2, H2, C2 = ring(c, k + 1)
                assert H2 == C
                a(f"v_mov_b32 v{L2}, v{H}")


def redc(a, chains, pbase):
    """Montgomery reduction (U + m p) / 2^384 of 24-word U, product scanning, interleaved chains:
    dict(u=[24 regs], m=[12 regs], acc=base, out=[12 regs]); out[j] may alias u[j + 12] (consumed at the start
    of column j + 12).  For U < 8p^2 the result is < 2p (not yet reduced)."""
    def ring(c, k):
        r = c["acc"]
        return (r, r + 1, r + 3) if k % 2 == 0 else (r + 2, r + 3, r + 1)

    for c in chains:
        a(f"v_mov_b32 v{c['acc']}, 0")
        a(f"v_mov_b32 v{c['acc'] + 1}, 0")
    for k in range(2 * N):
        # acc += U_k (the column's carry word starts fresh here)
        for t, c in enumerate(chains):
            L, H, C = ring(c, k)
            a(f"v_add_co_u32_e64 v{L}, s[{CARRY[t]}:{CARRY[t] + 1}], v{L}, v{c['u'][k]}")
        for t, c in enumerate(chains):
            L, H, C = ring(c, k)
            sc = f"s[{CARRY[t]}:{CARRY[t] + 1}]"
            a(f"v_addc_co_u32_e64 v{H}, {sc}, v{H}, 0, {sc}")
        for t, c in enumerate(chains):
            L, H, C = ring(c, k)
            sc = f"s[{CARRY[t]}:{CARRY[t] + 1}]"
            a(f"v_addc_co_u32_e64 v{C}, {sc}, 0, 0, {sc}")
        terms = [(i, k - i) for i in range(max(0, k - (N - 1)), min(k - 1, N - 1) + 1)]
        if k < N:
            terms.append(("m", k))
        for kind in terms:
            if kind[0] == "m":
                for c in chains:
                    L, H, C = ring(c, k)
                    a(f"v_mul_lo_u32 v{c['m'][k]}, v{L}, s{S_PINV}")
                x = lambda c: c["m"][k]
                y = pbase
            else:
                i, j = kind
                x = lambda c, i=i: c["m"][i]
                y = pbase + j
            for t, c in enumerate(chains):
                L, H, C = ring(c, k)
                a(f"v_mad_u64_u32 v[{L}:{H}], s[{CARRY[t]}:{CARRY[t] + 1}], v{x(c)}, v{y}, v[{L}:{H}]")
            for t, c in enumerate(chains):
                L, H, C = ring(c, k)
                sc = f"s[{CARRY[t]}:{CARRY[t] + 1}]"
                a(f"v_addc_co_u32_e64 v{C}, {sc}, 0, v{C}, {sc}")
        for c in chains:
            L, H, C = ring(c, k)
            if k >= N:
                a(f"v_mov_b32 v{c['out'][k - N]}, v{L}")
            if k < 2 * N - 1:
                L2, H2, C2 = ring(c, k + 1)
                assert H2 == C
                a(f"v_mov_b32 v{L2}, v{H}")


def wide_sub(a, r, x, y, sc):
    """r <- x - y over len(r) words (borrow chain in SGPR pair sc)"""
    a(f"v_sub_co_u32_e64 v{r[0]}, s[{sc}:{sc + 1}], v{x[0]}, v{y[0]}")
    for j in range(1, len(r)):
        a(f"v_subb_co_u32_e64 v{r[j]}, s[{sc}:{sc + 1}], v{x[j]}, v{y[j]}, s[{sc}:{sc + 1}]")


def wide_add(a, r, x, y, sc):
    a(f"v_add_co_u32_e64 v{r[0]}, s[{sc}:{sc + 1}], v{x[0]}, v{y[0]}")
    for j in range(1, len(r)):
        a(f"v_addc_co_u32_e64 v{r[j]}, s[{sc}:{sc + 1}], v{x[j]}, v{y[j]}, s[{sc}:{sc + 1}]")


def interleave2(a, emit0, emit1):
    """emit two independent chains alternately (each emit_k(asm) appends its instructions)"""
    s0, s1 = Asm(), Asm()
    emit0(s0)
    emit1(s1)
    l0, l1 = s0.lines, s1.lines
    for k in range(max(len(l0), len(l1))):
        if k < len(l0):
            a.lines.append(l0[k])
        if k < len(l1):
            a.lines.append(l1[k])


def reduce_to(a, dst, src, tmp, pbase, sc):
    """dst <- src - p if src >= p else src (src < 2p); tmp: 12 scratch VGPRs"""
    a(f"v_sub_co_u32_e64 v{tmp[0]}, s[{sc}:{sc + 1}], v{src[0]}, v{pbase}")
    for j in range(1, N):
        a(f"v_subb_co_u32_e64 v{tmp[j]}, s[{sc}:{sc + 1}], v{src[j]}, v{pbase + j}, s[{sc}:{sc + 1}]")
    for j in range(N):
        a(f"v_cndmask_b32_e64 v{dst[j]}, v{tmp[j]}, v{src[j]}, s[{sc}:{sc + 1}]")


def r_fp2_mul_lazy():
    """x*y in Fp2 with one Montgomery reduction per output coefficient (Karatsuba over double-width products):
    T0 = xa ya, T1 = xb yb, T2 = (xa + xb)(ya + yb) as 768-bit comba products (3 interleaved chains),
    U1 = T2 - T0 - T1, U0 = T0 - T1 + 4p^2, then REDC(U0), REDC(U1) (2 chains) and one conditional subtraction
    each: 3 x 144 + 2 x 156 = 744 MADs instead of 3 x 300 = 900, and no modular add/sub chains.
    Same contract as the eager routine: v[0:23] = x, v[24:47] = y in; v[0:23] = x*y out (fully reduced)."""
    a = Asm()
    a.label("lcb_r_fp2_mul")
    P_ = 120
    XA, XB, YA, YB, SA, SB = vr(0), vr(12), vr(24), vr(36), vr(48), vr(60)
    F0, F1, F2 = vr(72), vr(84), vr(96)
    T0 = F0[:11] + XA + [F0[11]]
    T1 = F1[:11] + XB + [F1[11]]
    T2 = F2[:11] + SA + [F2[11]]
    D = YA + YB                                   # b operands are dead after the products
    load_p(a, P_)
    interleave2(a, lambda q: add_unreduced(q, SA, XA, XB, sc=S_TMP),
                lambda q: add_unreduced(q, SB, YA, YB, sc=S_TMP2))
    products_plain(a, [dict(a=XA, b=YA, acc=108, out=T0),
                       dict(a=XB, b=YB, acc=112, out=T1),
                       dict(a=SA, b=SB, acc=116, out=T2)])
    interleave2(a, lambda q: wide_sub(q, T2, T2, T0, S_TMP), lambda q: wide_sub(q, D, T0, T1, S_TMP2))
    wide_sub(a, T2, T2, T1, S_TMP)                # U1 = T2 - T0 - T1  (>= 0)
    for j in range(2 * N):                        # 4p^2 into T1's registers
        a(f"v_mov_b32 v{T1[j]}, 0x{P2X4L[j]:08x}")
    wide_add(a, D, D, T1, S_TMP2)                 # U0 = T0 - T1 + 4p^2  (> 0, mod 2^768)
    redc(a, [dict(u=D, m=F0, acc=108, out=D[N:]), dict(u=T2, m=F1, acc=112, out=T2[N:])], P_)
    interleave2(a, lambda q: reduce_to(q, XA, D[N:], SB, P_, S_TMP),
                lambda q: reduce_to(q, XB, T2[N:], F0, P_, S_TMP2))
    a("s_setpc_b64 s[30:31]")
    return a.text(), 132


# ------------------------------------------------------------------ exponentiation by the field's constants
# lcb_r_fp_pow: v[0:11] = a, s84 = which (wave-uniform: 0 = p - 2, 1 = (p + 1)/4, 2 = (p - 1)/2, 3 = (p - 3)/4)
# -> v[0:11] = a^e.  The same sliding 4-bit windows as the compiled lcb_fp_pow_v (field.hpp), but the window table
# t1, t3, ..., t15 stays in VGPRs across the product calls: 12 caller-saved 8-register islands of the AMDGPU ABI from
# v64 (v64-71, v80-87, ..., v240-247), above every leaf routine's clobbers (<= v61), so neither this routine nor its
# callers save or reload it.  The compiled form kept the table in scratch (48 B reloaded per window, ~4.6 KB per
# exponentiation: most of the HBM traffic of every decompression lane, round 6).  The windows are known here, so
# each exponent is a straight-line program of steps `s_mov_b32 s82, cnt | idx << 16` + a call of lcb_r_fp_pow_step
# (cnt squarings, then one product by table entry idx; idx = 0xff: none).  Return addresses: s[80:81] (the
# routine), s[86:87] (the step); s83 counts.
POW_ISLANDS = [64 + 16 * k + j for k in range(12) for j in range(8)]           # v64-71, v80-87, ..., v240-247
POW_T = [POW_ISLANDS[12 * e:12 * e + 12] for e in range(8)]                     # t_(2e+1)
POW_EXPS = [P - 2, (P + 1) // 4, (P - 1) // 2, (P - 3) // 4]


def pow_program(e):
    """the sliding windows of field.hpp lcb_fp_pow_v for exponent e: (first table index, [(squarings, idx)])"""
    bit = lambda i: (e >> i) & 1
    i = e.bit_length() - 1
    first, steps, pend = None, [], 0
    while i >= 0:
        if not bit(i):
            pend += 1
            i -= 1
            continue
        j = max(i - 3, 0)
        while not bit(j):
            j += 1
        w = 0
        for b in range(i, j - 1, -1):
            w = (w << 1) | bit(b)
        if first is None:
            first = (w - 1) // 2
        else:
            steps.append((pend + i - j + 1, (w - 1) // 2))
        pend = 0
        i = j - 1
    if pend:
        steps.append((pend, 0xff))
    return first, steps


def pow_eval(a, e):
    """the program's value in plain integers (generator self-check)"""
    first, steps = pow_program(e)
    T = [pow(a, 2 * k + 1, P) for k in range(8)]
    acc = T[first]
    for cnt, idx in steps:
        for _ in range(cnt):
            acc = acc * acc % P
        if idx != 0xff:
            acc = acc * T[idx] % P
    return acc


def r_fp_pow():
    a = Asm()
    for ex in POW_EXPS:                         # generation-time check of the window programs
        assert pow_eval(7, ex) == pow(7, ex, P) and pow_eval(P - 3, ex) == pow(P - 3, ex, P)
    a.label("lcb_r_fp_pow")
    a("s_mov_b64 s[80:81], s[30:31]")
    mov(a, POW_T[0], vr(0))                     # t1 = a
    a(call_seq_asm("lcb_r_fp_sqr"))
    mov(a, POW_T[7], vr(0))                     # a^2, parked in t15's slot until t15 is formed
    for k in range(1, 8):
        mov(a, vr(0), POW_T[k - 1])
        mov(a, vr(12), POW_T[7])
        a(call_seq_asm("lcb_r_fp_mul"))
        mov(a, POW_T[k], vr(0))
    for w, ex in enumerate(POW_EXPS):
        a(f"s_cmp_eq_u32 s84, {w}")
        a(f"s_cbranch_scc1 lcb_r_fp_pow_e{w}")
    a("s_branch lcb_r_fp_pow_e0")
    for w, ex in enumerate(POW_EXPS):
        first, steps = pow_program(ex)
        a.label(f"lcb_r_fp_pow_e{w}")
        mov(a, vr(0), POW_T[first])
        for cnt, idx in steps:
            a(f"s_mov_b32 s82, {cnt | (idx << 16)}")
            a(call_seq_asm("lcb_r_fp_pow_step"))
        a("s_setpc_b64 s[80:81]")
    # the step: s82 = cnt | idx << 16
    a.label("lcb_r_fp_pow_step")
    a("s_mov_b64 s[86:87], s[30:31]")
    a("s_and_b32 s83, s82, 0xffff")
    a.label("lcb_r_fp_pow_sq")
    a("s_cmp_eq_u32 s83, 0")
    a("s_cbranch_scc1 lcb_r_fp_pow_sel")
    a(call_seq_asm("lcb_r_fp_sqr"))
    a("s_sub_u32 s83, s83, 1")
    a("s_branch lcb_r_fp_pow_sq")
    a.label("lcb_r_fp_pow_sel")
    a("s_lshr_b32 s83, s82, 16")
    for k in range(8):
        a(f"s_cmp_eq_u32 s83, {k}")
        a(f"s_cbranch_scc1 lcb_r_fp_pow_t{k}")
    a("s_setpc_b64 s[86:87]")                   # idx 0xff: squarings only
    for k in range(8):
        a.label(f"lcb_r_fp_pow_t{k}")
        mov(a, vr(12), POW_T[k])
        a("s_branch lcb_r_fp_pow_mul")
    a.label("lcb_r_fp_pow_mul")
    a(call_seq_asm("lcb_r_fp_mul"))
    a("s_setpc_b64 s[86:87]")
    return a.text(), 64


def call_seq_asm(label):
    """the call sequence of call_seq() as plain assembly lines (a routine calling a leaf routine)"""
    return (f"s_getpc_b64 s[{S_TMP}:{S_TMP + 1}]\n  s_add_u32 s{S_TMP}, s{S_TMP}, {label}@rel32@lo+4\n"
            f"  s_addc_u32 s{S_TMP + 1}, s{S_TMP + 1}, {label}@rel32@hi+12\n  s_swappc_b64 s[30:31], s[{S_TMP}:{S_TMP + 1}]")


ROUTINES = [r_fp_mul, r_fp_sqr, r_fp_mul2, r_fp2_mul_lazy, r_fp2_sqr, r_fp2_mul_fp, r_fp_pow]


def clobber_list(nvgpr, keep):
    regs = [f'"v{i}"' for i in range(nvgpr) if i not in keep]
    regs += [f'"s{s}"' for s in CLOBBER_SGPRS]
    regs += ['"scc"']  # the call sequence's s_add_u32/s_addc_u32 write SCC; a compare the compiler hoisted
    return ", ".join(regs)  # above the call would otherwise feed a stale SCC to the branch after it


def pow_clobbers():
    regs = [f'"v{i}"' for i in list(range(12, 64)) + POW_ISLANDS]
    regs += [f'"s{x}"' for x in [30, 31, 80, 81, 82, 83, 86, 87] + CLOBBER_SGPRS[2:]]
    regs += ['"scc"']
    return ", ".join(regs)


def call_seq(label):
    return (f'"s_getpc_b64 s[{S_TMP}:{S_TMP + 1}]\\n\\t"\n'
            f'        "s_add_u32 s{S_TMP}, s{S_TMP}, {label}@rel32@lo+4\\n\\t"\n'
            f'        "s_addc_u32 s{S_TMP + 1}, s{S_TMP + 1}, {label}@rel32@hi+12\\n\\t"\n'
            f'        "s_swappc_b64 s[30:31], s[{S_TMP}:{S_TMP + 1}]"')


def emit():
    bodies = []
    nv = {}
    for fn in ROUTINES:
        txt, n = fn()
        bodies.append(txt)
        nv[fn.__name__] = n
    lib = "\n".join(["  .p2align 8\n" + b for b in bodies])
    out = []
    out.append("// GENERATED by tools/gen_asm.py — do not edit.\n")
    out.append("// gfx950 assembly leaf routines with a register calling convention (see the generator's docstring).\n")
    out.append("#pragma once\n#include <hip/hip_runtime.h>\n#include <stdint.h>\n\n")
    out.append("typedef uint32_t u32;\ntypedef u32 u32x12 __attribute__((ext_vector_type(12)));\n\n")
    # library kernel (one per translation unit; never launched, it only hosts the routines' code)
    out.append("#define LCB_ASM_LIBRARY(tag) \\\n")
    out.append("extern \"C\" __global__ void __launch_bounds__(64) lcb_asm_library_##tag() { \\\n")
    out.append("    asm volatile(LCB_ASM_LIBRARY_TEXT); \\\n}\n\n")
    esc = lib.replace("\\", "\\\\").replace('"', '\\"')
    out.append("#define LCB_ASM_LIBRARY_TEXT \\\n    \"  s_endpgm\\n\" \\\n")
    for line in esc.split("\n"):
        out.append(f'    "{line}\\n" \\\n')
    out.append('    ""\n\n')
    # wrappers
    out.append(f"""// r = a*b
__device__ __forceinline__ u32x12 lcb_asm_fp_mul(u32x12 a, u32x12 b) {{
    asm({call_seq("lcb_r_fp_mul")}
        : "+{{v[0:11]}}"(a), "+{{v[12:23]}}"(b)
        :
        : {clobber_list(nv['r_fp_mul'], set(range(24)))});
    return a;
}}
// r = a^2 (78 + 144 products instead of 288)
__device__ __forceinline__ u32x12 lcb_asm_fp_sqr(u32x12 a) {{
    asm({call_seq("lcb_r_fp_sqr")}
        : "+{{v[0:11]}}"(a)
        :
        : {clobber_list(nv['r_fp_sqr'], set(range(12)))});
    return a;
}}
// (a0*b0, a1*b1)
__device__ __forceinline__ void lcb_asm_fp_mul2(u32x12 &a0, u32x12 b0, u32x12 &a1, u32x12 b1) {{
    asm({call_seq("lcb_r_fp_mul2")}
        : "+{{v[0:11]}}"(a0), "+{{v[12:23]}}"(b0), "+{{v[24:35]}}"(a1), "+{{v[36:47]}}"(b1)
        :
        : {clobber_list(nv['r_fp_mul2'], set(range(48)))});
}}
// x*y in Fp2: (xa, xb) <- (xa, xb) * (ya, yb); lazy reduction (one REDC per coefficient)
__device__ __forceinline__ void lcb_asm_fp2_mul(u32x12 &xa, u32x12 &xb, u32x12 ya, u32x12 yb) {{
    asm({call_seq("lcb_r_fp2_mul")}
        : "+{{v[0:11]}}"(xa), "+{{v[12:23]}}"(xb), "+{{v[24:35]}}"(ya), "+{{v[36:47]}}"(yb)
        :
        : {clobber_list(nv['r_fp2_mul_lazy'], set(range(48)))});
}}
// x^2 in Fp2
__device__ __forceinline__ void lcb_asm_fp2_sqr(u32x12 &xa, u32x12 &xb) {{
    asm({call_seq("lcb_r_fp2_sqr")}
        : "+{{v[0:11]}}"(xa), "+{{v[12:23]}}"(xb)
        :
        : {clobber_list(nv['r_fp2_sqr'], set(range(24)))});
}}
// a^e for e = p - 2, (p + 1)/4, (p - 1)/2, (p - 3)/4 (which = 0..3, wave-uniform): the window table in VGPR islands
__device__ __forceinline__ u32x12 lcb_asm_fp_pow(u32x12 a, int which) {{
    asm({call_seq("lcb_r_fp_pow")}
        : "+{{v[0:11]}}"(a)
        : "{{s84}}"(which)
        : {pow_clobbers()});
    return a;
}}
// x*s for x in Fp2, s in Fp
__device__ __forceinline__ void lcb_asm_fp2_mul_fp(u32x12 &xa, u32x12 &xb, u32x12 s) {{
    asm({call_seq("lcb_r_fp2_mul_fp")}
        : "+{{v[0:11]}}"(xa), "+{{v[12:23]}}"(xb), "+{{v[24:35]}}"(s)
        :
        : {clobber_list(nv['r_fp2_mul_fp'], set(range(36)))});
}}
""")
    return "".join(out)


# ------------------------------------------------------------------ inline add / sub (no call)
# Compiler-built 12-limb add/sub with C carries costs ~160 VALU instructions (64-bit adds + shifts); these
# are the 36-37 instruction carry chains.  Carries ride in VCC through VOP2 (e32) forms only: gfx940+ has a
# 2-wait-state hazard for an explicit SGPR read right after a VALU SGPR write, the implicit VCC read of
# VOP2 does not.  Operands are 12 separate u32 (r, temps, a, b) so the register allocator places them.
def inline_fn(name, comment, body, n_tmp, n_in, reduced_doc, r_early=False, with_p=False):
    outs = [f'"=&v"(t[{j}])' for j in range(n_tmp)]
    r_ops = [f'"=&v"(r[{j}])' if r_early else f'"=v"(r[{j}])' for j in range(N)]
    ins = []
    for k in range(n_in):
        ins += [f'"v"({"ab"[k]}[{j}])' for j in range(N)]
    if with_p:
        ins += [f'"v"(0x{PL[j]:08x}u)' for j in range(N)]
    # gfx940+ hazard: a VALU write of VCC needs 2 wait states before a VALU reads it as carry-in
    # (LLVM emits `s_nop 1` between the links of its own carry chains on gfx942/gfx950).
    hz = []
    for line in body:
        if line.rstrip().endswith(", vcc") and hz and "vcc," in hz[-1]:
            hz.append("s_nop 1")
        hz.append(line)
    txt = "\\n\\t".join(hz)
    args = ", ".join(["u32 *r"] + [f"const u32 *{'ab'[k]}" for k in range(n_in)])
    tmp_decl = f"    u32 t[{n_tmp}];\n" if n_tmp else ""
    return (f"// {comment} ({reduced_doc})\n"
            f"__device__ __forceinline__ void {name}({args}) {{\n{tmp_decl}"
            f"    asm volatile(\"{txt}\"\n        : {', '.join(r_ops + outs)}\n        : {', '.join(ins)}\n        : \"vcc\");\n}}\n")


def op_index(n_tmp):
    """operand numbering: r = 0..11, t = 12..12+n_tmp-1, a = next 12, b = next 12"""
    r = list(range(N))
    t = list(range(N, N + n_tmp))
    a = list(range(N + n_tmp, 2 * N + n_tmp))
    b = list(range(2 * N + n_tmp, 3 * N + n_tmp))
    return r, t, a, b


def gen_add_mod():
    # the compare-subtract chain needs p in VGPRs: a VOP2 with carry-in already uses the constant bus (VCC)
    r, t, a, b = op_index(N)
    pv = list(range(3 * N + N, 4 * N + N))
    s = [f"v_add_co_u32_e32 %{t[0]}, vcc, %{a[0]}, %{b[0]}"]
    s += [f"v_addc_co_u32_e32 %{t[j]}, vcc, %{a[j]}, %{b[j]}, vcc" for j in range(1, N)]
    s += [f"v_sub_co_u32_e32 %{r[0]}, vcc, %{t[0]}, %{pv[0]}"]
    s += [f"v_subb_co_u32_e32 %{r[j]}, vcc, %{t[j]}, %{pv[j]}, vcc" for j in range(1, N)]
    s += [f"v_cndmask_b32_e32 %{r[j]}, %{r[j]}, %{t[j]}, vcc" for j in range(N)]  # borrow -> keep t
    return inline_fn("lcb_fp_add_asm", "r = a + b mod p", s, N, 2, "a, b < p -> r < p", r_early=True, with_p=True)


def gen_sub_mod():
    r, t, a, b = op_index(N + 1)
    mw = t[N]
    s = [f"v_sub_co_u32_e32 %{t[0]}, vcc, %{a[0]}, %{b[0]}"]
    s += [f"v_subb_co_u32_e32 %{t[j]}, vcc, %{a[j]}, %{b[j]}, vcc" for j in range(1, N)]
    # mw = t0 - t0 - borrow = all-ones iff a < b
    s += [f"v_subb_co_u32_e32 %{mw}, vcc, %{t[0]}, %{t[0]}, vcc"]
    s += [f"v_and_b32_e32 %{r[j]}, 0x{PL[j]:08x}, %{mw}" for j in range(N)]
    s += [f"v_add_co_u32_e32 %{r[0]}, vcc, %{t[0]}, %{r[0]}"]
    s += [f"v_addc_co_u32_e32 %{r[j]}, vcc, %{t[j]}, %{r[j]}, vcc" for j in range(1, N)]
    return inline_fn("lcb_fp_sub_asm", "r = a - b mod p", s, N + 1, 2, "a, b < p -> r < p")


def gen_add_nr():
    r, t, a, b = op_index(0)
    s = [f"v_add_co_u32_e32 %{r[0]}, vcc, %{a[0]}, %{b[0]}"]
    s += [f"v_addc_co_u32_e32 %{r[j]}, vcc, %{a[j]}, %{b[j]}, vcc" for j in range(1, N)]
    return inline_fn("lcb_fp_add_nr_asm", "r = a + b, not reduced", s, 0, 2, "a, b < p -> r < 2p: multiplicand only",
                     r_early=True)


def gen_neg():
    r, t, a, b = op_index(N + 1)
    mw = t[N]
    # t = 0 - a; borrow iff a != 0; r = t + (p & -borrow)
    s = [f"v_sub_co_u32_e32 %{t[0]}, vcc, 0, %{a[0]}"]
    s += [f"v_subb_co_u32_e32 %{t[j]}, vcc, 0, %{a[j]}, vcc" for j in range(1, N)]
    s += [f"v_subb_co_u32_e32 %{mw}, vcc, %{t[0]}, %{t[0]}, vcc"]
    s += [f"v_and_b32_e32 %{r[j]}, 0x{PL[j]:08x}, %{mw}" for j in range(N)]
    s += [f"v_add_co_u32_e32 %{r[0]}, vcc, %{t[0]}, %{r[0]}"]
    s += [f"v_addc_co_u32_e32 %{r[j]}, vcc, %{t[j]}, %{r[j]}, vcc" for j in range(1, N)]
    return inline_fn("lcb_fp_neg_asm", "r = -a mod p", s, N + 1, 1, "a < p -> r < p")


# ------------------------------------------------------------------ two-chain (Fp2) add / sub / neg
# The single-chain forms above pay `s_nop 1` on every carry link: one wave per SIMD has nothing else to issue in
# the hazard slots.  An Fp2 operation has two independent 12-limb chains; interleaving them (chain A carries in
# VCC through VOP2, chain B in a compiler-chosen SGPR pair through VOP3) puts the other chain's instruction in
# the slot and needs only `s_nop 0` per link pair.
def _chain_add(r, t, a, b, pv, c):
    e = "e32" if c == "vcc" else "e64"
    s = [f"v_add_co_u32_{e} %{t[0]}, {c}, %{a[0]}, %{b[0]}"]
    s += [f"v_addc_co_u32_{e} %{t[j]}, {c}, %{a[j]}, %{b[j]}, {c}" for j in range(1, N)]
    s += [f"v_sub_co_u32_{e} %{r[0]}, {c}, %{t[0]}, %{pv[0]}"]
    s += [f"v_subb_co_u32_{e} %{r[j]}, {c}, %{t[j]}, %{pv[j]}, {c}" for j in range(1, N)]
    if c == "vcc":
        s += [f"v_cndmask_b32_e32 %{r[j]}, %{r[j]}, %{t[j]}, vcc" for j in range(N)]
    else:
        s += [f"v_cndmask_b32_e64 %{r[j]}, %{r[j]}, %{t[j]}, {c}" for j in range(N)]
    return s


def _chain_sub(r, t, a, b, c, neg=False):
    e = "e32" if c == "vcc" else "e64"
    mw = t[N]
    if neg:
        s = [f"v_sub_co_u32_{e} %{t[0]}, {c}, 0, %{a[0]}"]
        s += [f"v_subb_co_u32_{e} %{t[j]}, {c}, 0, %{a[j]}, {c}" for j in range(1, N)]
    else:
        s = [f"v_sub_co_u32_{e} %{t[0]}, {c}, %{a[0]}, %{b[0]}"]
        s += [f"v_subb_co_u32_{e} %{t[j]}, {c}, %{a[j]}, %{b[j]}, {c}" for j in range(1, N)]
    s += [f"v_subb_co_u32_{e} %{mw}, {c}, %{t[0]}, %{t[0]}, {c}"]
    s += [f"v_and_b32_e32 %{r[j]}, 0x{PL[j]:08x}, %{mw}" for j in range(N)]
    s += [f"v_add_co_u32_{e} %{r[0]}, {c}, %{t[0]}, %{r[0]}"]
    s += [f"v_addc_co_u32_{e} %{r[j]}, {c}, %{t[j]}, %{r[j]}, {c}" for j in range(1, N)]
    return s


def _reads_carry(line):
    return line.rstrip().endswith(", vcc") or line.rstrip().endswith(", %S")


_CARRY_OPS = ("v_add_co_u32", "v_addc_co_u32", "v_sub_co_u32", "v_subb_co_u32")


def _interleave(la, lb, sop):
    """Alternate the two chains' instructions; before an instruction that reads its chain's carry, pad with
    s_nop so that at least 2 wait states separate it from that chain's last carry write (chains of unequal
    length finish alone with `s_nop 1` links)."""
    out, last_w = [], {0: None, 1: None}
    seqs = [list(la), list(lb)]
    idx = [0, 0]
    turn = 0
    while idx[0] < len(seqs[0]) or idx[1] < len(seqs[1]):
        if idx[turn] >= len(seqs[turn]):
            turn ^= 1
        line = seqs[turn][idx[turn]]
        idx[turn] += 1
        if _reads_carry(line) and last_w[turn] is not None:
            gap = len(out) - last_w[turn] - 1          # instructions issued since the carry write
            if gap < 2:
                out.append(f"s_nop {1 - gap}")
        if line.split()[0].startswith(_CARRY_OPS):
            last_w[turn] = len(out)
        out.append(line)
        turn ^= 1
    return [l.replace("%S", f"%{sop}") for l in out]


def _interleave_k(seqs, sops):
    """Round-robin over K chains (chain 0 carries in VCC, chain c > 0 in the SGPR pair operand sops[c-1]),
    padding with s_nop where a chain's carry read would come < 2 wait states after its carry write."""
    out, last_w = [], [None] * len(seqs)
    idx = [0] * len(seqs)
    c = 0
    while any(idx[k] < len(seqs[k]) for k in range(len(seqs))):
        while idx[c] >= len(seqs[c]):
            c = (c + 1) % len(seqs)
        line = seqs[c][idx[c]]
        idx[c] += 1
        if _reads_carry(line) and last_w[c] is not None:
            gap = len(out) - last_w[c] - 1
            if gap < 2:
                out.append(f"s_nop {1 - gap}")
        if line.split()[0].startswith(_CARRY_OPS):
            last_w[c] = len(out)
        out.append(line if c == 0 else line.replace("%S", f"%{sops[c - 1]}"))
        c = (c + 1) % len(seqs)
    return out


def inline_fnk(name, comment, K, n_tmp, n_in, with_p, build):
    """K independent 12-limb chains in one asm block: r_k = op(x_k[, y_k])."""
    r = [list(range(k * N, (k + 1) * N)) for k in range(K)]
    base = K * N
    t = [list(range(base + k * n_tmp, base + (k + 1) * n_tmp)) for k in range(K)]
    base += K * n_tmp
    sops = list(range(base, base + K - 1))
    base += K - 1
    x = [list(range(base + k * N, base + (k + 1) * N)) for k in range(K)]
    base += K * N
    y = [list(range(base + k * N, base + (k + 1) * N)) for k in range(K)] if n_in == 2 else [None] * K
    base += K * N if n_in == 2 else 0
    pv = list(range(base, base + N)) if with_p else None
    body = _interleave_k([build(r[k], t[k], x[k], y[k], pv, "vcc" if k == 0 else "%S") for k in range(K)], sops)
    outs = [f'"=&v"(r{k}[{j}])' for k in range(K) for j in range(N)]
    outs += [f'"=&v"(t{k}[{j}])' for k in range(K) for j in range(n_tmp)]
    outs += [f'"=&s"(sc{k})' for k in range(1, K)]
    ins = [f'"v"(x{k}[{j}])' for k in range(K) for j in range(N)]
    if n_in == 2:
        ins += [f'"v"(y{k}[{j}])' for k in range(K) for j in range(N)]
    if with_p:
        ins += [f'"v"(0x{PL[j]:08x}u)' for j in range(N)]
    args = ", ".join([f"u32 *r{k}" for k in range(K)] + [f"const u32 *x{k}" for k in range(K)] +
                     ([f"const u32 *y{k}" for k in range(K)] if n_in == 2 else []))
    decl = "".join(f"    u32 t{k}[{n_tmp}];\n" for k in range(K))
    decl += "    unsigned long long " + ", ".join(f"sc{k}" for k in range(1, K)) + ";\n"
    txt = "\\n\\t".join(body)
    return (f"// {comment}: {K} independent carry chains interleaved in one block\n"
            f"__device__ __forceinline__ void {name}({args}) {{\n{decl}"
            f"    asm volatile(\"{txt}\"\n        : {', '.join(outs)}\n        : {', '.join(ins)}\n        : \"vcc\");\n}}\n")


def gen_fp3_add():
    return inline_fnk("lcb_fp3_add_asm", "r_k = x_k + y_k mod p, k = 0..2", 3, N, 2, True,
                      lambda r, t, a, b, pv, c: _chain_add(r, t, a, b, pv, c))


def gen_fp3_sub():
    return inline_fnk("lcb_fp3_sub_asm", "r_k = x_k - y_k mod p, k = 0..2", 3, N + 1, 2, False,
                      lambda r, t, a, b, pv, c: _chain_sub(r, t, a, b, c))


def inline_fn2(name, comment, n_tmp, n_in, with_p, build, second_operands_swap=False):
    # operands: rA 0..11, rB 12..23, tA, tB, S; inputs aA, aB, [bA, bB], [p]
    rA, rB = list(range(N)), list(range(N, 2 * N))
    tA = list(range(2 * N, 2 * N + n_tmp))
    tB = list(range(2 * N + n_tmp, 2 * N + 2 * n_tmp))
    sop = 2 * N + 2 * n_tmp
    k = sop + 1
    aA, aB = list(range(k, k + N)), list(range(k + N, k + 2 * N))
    k += 2 * N
    bA, bB = (list(range(k, k + N)), list(range(k + N, k + 2 * N))) if n_in == 2 else (None, None)
    k += 2 * N if n_in == 2 else 0
    pv = list(range(k, k + N)) if with_p else None
    if second_operands_swap:   # both chains combine the two inputs: chain A (aA, aB), chain B (aA, aB)
        body = _interleave(build(rA, tA, aA, aB, pv, "vcc"), build(rB, tB, aA, aB, pv, "%S"), sop)
    else:
        body = _interleave(build(rA, tA, aA, bA, pv, "vcc"), build(rB, tB, aB, bB, pv, "%S"), sop)
    outs = [f'"=&v"(ra[{j}])' for j in range(N)] + [f'"=&v"(rb[{j}])' for j in range(N)]
    outs += [f'"=&v"(ta[{j}])' for j in range(n_tmp)] + [f'"=&v"(tb[{j}])' for j in range(n_tmp)]
    outs += ['"=&s"(sc)']
    ins = [f'"v"(xa[{j}])' for j in range(N)] + [f'"v"(xb[{j}])' for j in range(N)]
    if n_in == 2:
        ins += [f'"v"(ya[{j}])' for j in range(N)] + [f'"v"(yb[{j}])' for j in range(N)]
    if with_p:
        ins += [f'"v"(0x{PL[j]:08x}u)' for j in range(N)]
    args = "u32 *ra, u32 *rb, const u32 *xa, const u32 *xb" + (", const u32 *ya, const u32 *yb" if n_in == 2 else "")
    txt = "\\n\\t".join(body)
    return (f"// {comment}: both Fp components in one interleaved pair of carry chains\n"
            f"__device__ __forceinline__ void {name}({args}) {{\n"
            f"    u32 ta[{n_tmp}], tb[{n_tmp}];\n    unsigned long long sc;\n"
            f"    asm volatile(\"{txt}\"\n        : {', '.join(outs)}\n        : {', '.join(ins)}\n        : \"vcc\");\n}}\n")


def gen_fp2_mul_xi():
    # (a + b i)(1 + i) = (a - b) + (a + b) i: a subtraction chain and an addition chain side by side
    def build(r, t, a, b, pv, c):
        return _chain_sub(r, t, a, b, c) if c == "vcc" else _chain_add(r, t, a, b, pv, c)
    return inline_fn2("lcb_fp2_mul_xi_asm", "(ra, rb) = (xa - xb, xa + xb) mod p", N + 1, 1, True, build,
                      second_operands_swap=True)


def gen_fp2_add():
    return inline_fn2("lcb_fp2_add_asm", "(ra, rb) = (xa + ya, xb + yb) mod p", N, 2, True,
                      lambda r, t, a, b, pv, c: _chain_add(r, t, a, b, pv, c))


def gen_fp2_sub():
    return inline_fn2("lcb_fp2_sub_asm", "(ra, rb) = (xa - ya, xb - yb) mod p", N + 1, 2, False,
                      lambda r, t, a, b, pv, c: _chain_sub(r, t, a, b, c))


def gen_fp2_neg():
    return inline_fn2("lcb_fp2_neg_asm", "(ra, rb) = (-xa, -xb) mod p", N + 1, 1, False,
                      lambda r, t, a, b, pv, c: _chain_sub(r, t, a, None, c, neg=True))


INLINE = [gen_add_mod, gen_sub_mod, gen_add_nr, gen_neg, gen_fp2_add, gen_fp2_sub, gen_fp2_neg, gen_fp2_mul_xi, gen_fp3_add, gen_fp3_sub]


def main():
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lachain_amd", "csrc", "asm_routines.hpp")
    with open(dst, "w") as f:
        f.write(emit())
        f.write("\n// ------------------------------------------------------------------ inline carry chains\n")
        for g in INLINE:
            f.write(g())
    print("wrote", os.path.normpath(dst))


if __name__ == "__main__":
    main()
