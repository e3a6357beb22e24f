#!/usr/bin/env python3
"""tools/gen_secp_asm.py — generates lachain_amd/csrc/secp_asm.hpp: gfx950 inline-assembly bodies of the secp256k1
field product and square (p = 2^256 - 2^32 - 977) used by k_secp.hip.

Each function is one asm block whose operands are pinned to v0..v15 (inputs / output); its temporaries are listed
as clobbers, so the compiler moves values in and out but never splits the carry chains.  Product: column (product)
scanning with a 64-bit accumulator pair and a carry-count word rotating through a 4-register ring (one
v_mad_u64_u32 + one v_addc per partial product, no zeroing: the first carry add of a column writes 0 + 0 + carry),
as in tools/gen_asm.py for BLS12-381.  Square: the 28 cross products once, doubled by a 1-bit shift, plus the 8
squares.  Reduction: t = lo + hi * 977 + (hi << 32) column by column, then the top word (< 2^34) folded once more by
C = 2^32 + 977, and a final conditional + C if that wraps (the result is < 2^256, congruent mod p: "weakly reduced",
the representation secp.hpp uses).  Carries ride in VCC and are only read through VOP2 (e32) forms: on gfx940+ an
explicit SGPR read right after a VALU writes that SGPR needs two wait states that inline assembly does not get, the
implicit VCC read of VOP2 does not (tools/gen_asm.py uses the same rule).  977 and 0 live in VGPRs (gfx9 VOP3 takes
no literal operands, VOP2 needs a VGPR second source).

Verified by tests/test_secp_emul.py on the CPU only through the C++ path; the asm is checked on the GPU by
tests/test_gpu_ecdsa.py (every decision against the oracle) and by tools/emul/secp_stage_dump.hip diffs.
"""
import os

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lachain_amd", "csrc", "secp_asm.hpp")


class Asm:
    def __init__(self):
        self.lines = []

    def __call__(self, s):
        self.lines.append(s)


ZERO = 41


def product(a, A, B, T, ring):
    """T[0..15] <- A[0..7] * B[0..7] (A, B, T register numbers); ring: 4 registers, ring[0] even"""
    def rk(k):
        r = ring
        return (r[0], r[1], r[3]) if k % 2 == 0 else (r[2], r[3], r[1])
    a(f"v_mov_b32 v{ring[0]}, 0")
    a(f"v_mov_b32 v{ring[1]}, 0")
    for k in range(15):
        L, H, C = rk(k)
        terms = [(i, k - i) for i in range(8) if 0 <= k - i <= 7]
        for n, (i, j) in enumerate(terms):
            a(f"v_mad_u64_u32 v[{L}:{H}], vcc, v{A[i]}, v{B[j]}, v[{L}:{H}]")
            a(f"v_addc_co_u32_e32 v{C}, vcc, 0, v{C if n else ZERO}, vcc")
        a(f"v_mov_b32 v{T[k]}, v{L}")
        L2, H2, C2 = rk(k + 1)
        assert H2 == C
        a(f"v_mov_b32 v{L2}, v{H}")
    L, H, C = rk(15)
    a(f"v_mov_b32 v{T[15]}, v{L}")


def square(a, A, T, ring):
    """T <- A^2: cross products once (columns 1..13), doubled, plus the squares"""
    def rk(k):
        r = ring
        return (r[0], r[1], r[3]) if k % 2 == 0 else (r[2], r[3], r[1])
    a(f"v_mov_b32 v{T[0]}, 0")
    a(f"v_mov_b32 v{ring[2]}, 0")
    a(f"v_mov_b32 v{ring[3]}, 0")
    for k in range(1, 14):
        L, H, C = rk(k)
        terms = [(i, k - i) for i in range(8) if i < k - i <= 7]
        for n, (i, j) in enumerate(terms):
            a(f"v_mad_u64_u32 v[{L}:{H}], vcc, v{A[i]}, v{A[j]}, v[{L}:{H}]")
            a(f"v_addc_co_u32_e32 v{C}, vcc, 0, v{C if n else ZERO}, vcc")
        a(f"v_mov_b32 v{T[k]}, v{L}")
        L2, H2, C2 = rk(k + 1)
        a(f"v_mov_b32 v{L2}, v{H}")
    L, H, C = rk(14)
    a(f"v_mov_b32 v{T[14]}, v{L}")
    a(f"v_mov_b32 v{T[15]}, v{H}")                         # column 13's carry count: bits 480..511
    # double: T <<= 1 (top bit of T[14] goes to T[15])
    for k in range(15, 0, -1):
        a(f"v_alignbit_b32 v{T[k]}, v{T[k]}, v{T[k - 1]}, 31")
    a(f"v_lshlrev_b32 v{T[0]}, 1, v{T[0]}")
    # + squares: a_i^2 at columns 2i, 2i+1, carry chained through the whole 512 bits
    sq = ring  # two pairs
    for i in range(8):
        p0, p1 = (sq[0], sq[1]) if i % 2 == 0 else (sq[2], sq[3])
        a(f"v_mul_lo_u32 v{p0}, v{A[i]}, v{A[i]}")
        a(f"v_mul_hi_u32 v{p1}, v{A[i]}, v{A[i]}")
        if i == 0:
            a(f"v_add_co_u32_e32 v{T[0]}, vcc, v{T[0]}, v{p0}")
        else:
            a(f"v_addc_co_u32_e32 v{T[2 * i]}, vcc, v{T[2 * i]}, v{p0}, vcc")
        a(f"v_addc_co_u32_e32 v{T[2 * i + 1]}, vcc, v{T[2 * i + 1]}, v{p1}, vcc")


def reduce(a, T, R, X, K977):
    """R[0..7] <- T[0..15] mod p, weakly reduced.  X: 4 scratch registers (X[0] even); K977 holds 977."""
    L, H = X[0], X[1]
    # column k: t_k + 977 t_(8+k) + t_(7+k) (k >= 1) + carry; (L, H) = 64-bit column sum
    a(f"v_mov_b32 v{L}, v{T[0]}")
    a(f"v_mov_b32 v{H}, 0")
    for k in range(8):
        a(f"v_mad_u64_u32 v[{L}:{H}], vcc, v{T[8 + k]}, v{K977}, v[{L}:{H}]")   # < 2^64: no carry out
        if k >= 1:
            a(f"v_add_co_u32_e32 v{L}, vcc, v{L}, v{T[7 + k]}")
            a(f"v_addc_co_u32_e32 v{H}, vcc, 0, v{H}, vcc")
        a(f"v_mov_b32 v{R[k]}, v{L}")
        if k < 7:
            a(f"v_add_co_u32_e32 v{L}, vcc, v{H}, v{T[k + 1]}")
            a(f"v_addc_co_u32_e32 v{H}, vcc, 0, v{ZERO}, vcc")
    # k8 = carry + t_15 (the (hi << 32) term at limb 8), as (L, H) with H <= 1
    a(f"v_add_co_u32_e32 v{L}, vcc, v{H}, v{T[15]}")
    a(f"v_addc_co_u32_e32 v{H}, vcc, 0, v{ZERO}, vcc")
    # R += k8 C = k8 977 + (k8 << 32): limb 0 lo(L 977), limb 1 hi(L 977) + H 977 + L, limb 2 H
    P0, P1 = X[2], X[3]
    a(f"v_mul_lo_u32 v{P0}, v{L}, v{K977}")
    a(f"v_mul_hi_u32 v{P1}, v{L}, v{K977}")
    a(f"v_mad_u32_u24 v{P1}, v{H}, v{K977}, v{P1}")        # < 2^11: no overflow
    a(f"v_add_co_u32_e32 v{R[0]}, vcc, v{R[0]}, v{P0}")
    a(f"v_addc_co_u32_e32 v{R[1]}, vcc, v{R[1]}, v{P1}, vcc")
    a(f"v_addc_co_u32_e32 v{R[2]}, vcc, v{R[2]}, v{H}, vcc")
    for k in range(3, 8):
        a(f"v_addc_co_u32_e32 v{R[k]}, vcc, 0, v{R[k]}, vcc")
    a(f"v_addc_co_u32_e32 v{P0}, vcc, 0, v{ZERO}, vcc")      # wrap of the first chain (0 / 1)
    a(f"v_add_co_u32_e32 v{R[1]}, vcc, v{R[1]}, v{L}")
    for k in range(2, 8):
        a(f"v_addc_co_u32_e32 v{R[k]}, vcc, 0, v{R[k]}, vcc")
    a(f"v_addc_co_u32_e32 v{P0}, vcc, v{P0}, v{ZERO}, vcc")  # total wraps w (at most one: the sum added is < 2^67)
    # R += w C (the value is < 2^67 after a wrap: no further carry out)
    a(f"v_mul_u32_u24 v{P1}, v{P0}, v{K977}")
    a(f"v_add_co_u32_e32 v{R[0]}, vcc, v{R[0]}, v{P1}")
    a(f"v_addc_co_u32_e32 v{R[1]}, vcc, v{R[1]}, v{P0}, vcc")
    for k in range(2, 8):
        a(f"v_addc_co_u32_e32 v{R[k]}, vcc, 0, v{R[k]}, vcc")


def addsub_lines(sub):
    """inline asm with compiler-allocated operands: %0..%7 r (early clobber), %8 t, %9 u, %10 z (temps),
    %11..%18 a, %19..%26 b.  add: r = a + b, then + C per carry out (twice at most); sub: r = a - b, then - C
    (= + p mod 2^256) per borrow (twice at most) — the same values as secp.hpp's C++ fe_add / fe_sub."""
    R = [f"%{i}" for i in range(8)]
    T, U, Z = "%8", "%9", "%10"
    A = [f"%{11 + i}" for i in range(8)]
    B = [f"%{19 + i}" for i in range(8)]
    op0, opc = ("v_sub_co_u32_e32", "v_subb_co_u32_e32") if sub else ("v_add_co_u32_e32", "v_addc_co_u32_e32")
    L = [f"v_mov_b32 {Z}, 0", f"{op0} {R[0]}, vcc, {A[0]}, {B[0]}"]
    for k in range(1, 8):
        L.append(f"{opc} {R[k]}, vcc, {A[k]}, {B[k]}, vcc")
    for _ in range(2):
        L.append(f"v_addc_co_u32_e32 {T}, vcc, 0, {Z}, vcc")       # t = carry / borrow (0 / 1)
        L.append(f"v_mul_u32_u24_e32 {U}, 977, {T}")
        L.append(f"{op0} {R[0]}, vcc, {R[0]}, {U}")
        L.append(f"{opc} {R[1]}, vcc, {R[1]}, {T}, vcc")
        for k in range(2, 8):
            L.append(f"{opc} {R[k]}, vcc, {R[k]}, {Z}, vcc")
    return L


def addsub_fn(name, sub, comment):
    body = "\n".join(f'        "{l}\\n\\t"' for l in addsub_lines(sub))
    outs = ", ".join(f'"=&v"(r.v[{i}])' for i in range(8)) + ', "=&v"(t), "=&v"(u), "=&v"(z)'
    ins = ", ".join(f'"v"(a.v[{i}])' for i in range(8)) + ", " + ", ".join(f'"v"(b.v[{i}])' for i in range(8))
    return "\n".join([
        f"// {comment}",
        f"__device__ __forceinline__ void {name}(fe &r, const fe &a, const fe &b) {{",
        "    u32 t, u, z;",
        "    asm volatile(",
        body,
        f"        : {outs}",
        f"        : {ins}",
        '        : "vcc");',
        "}",
    ])


def block(lines):
    return "\n".join(f'        "{l}\\n\\t"' for l in lines)


def gen():
    A = list(range(0, 8))
    B = list(range(8, 16))
    T = list(range(16, 32))
    ring = [32, 33, 34, 35]
    X = [36, 37, 38, 39]
    K = 40
    m = Asm()
    m(f"v_mov_b32 v{K}, 977")
    m(f"v_mov_b32 v{ZERO}, 0")
    product(m, A, B, T, ring)
    reduce(m, T, A, X, K)
    s = Asm()
    s(f"v_mov_b32 v{K}, 977")
    s(f"v_mov_b32 v{ZERO}, 0")
    square(s, A, T, ring)
    reduce(s, T, A, X, K)
    clob = ", ".join(f'"v{i}"' for i in range(16, 42)) + ', "vcc"'
    clob_sq = ", ".join(f'"v{i}"' for i in range(8, 42)) + ', "vcc"'
    out = [
        "// GENERATED by tools/gen_secp_asm.py — do not edit.",
        "// secp256k1 field product / square (p = 2^256 - 2^32 - 977) as gfx950 inline assembly; see the generator.",
        "#pragma once",
        "#include <stdint.h>",
        "typedef uint32_t u32;",
        "typedef u32 u32x8 __attribute__((ext_vector_type(8)));",
        "",
        "// a * b, weakly reduced (< 2^256, congruent mod p)",
        "__device__ __forceinline__ u32x8 secp_asm_mul(u32x8 a, u32x8 b) {",
        "    asm volatile(",
        block(m.lines),
        '        : "+{v[0:7]}"(a), "+{v[8:15]}"(b)',
        "        :",
        f"        : {clob});",
        "    return a;",
        "}",
        addsub_fn("secp_asm_add", False, "r = a + b, weakly reduced (fe_add)"),
        addsub_fn("secp_asm_sub", True, "r = a - b mod p, weakly reduced (fe_sub)"),
        "// a^2, weakly reduced",
        "__device__ __forceinline__ u32x8 secp_asm_sqr(u32x8 a) {",
        "    asm volatile(",
        block(s.lines),
        '        : "+{v[0:7]}"(a)',
        "        :",
        f"        : {clob_sq});",
        "    return a;",
        "}",
        "",
    ]
    with open(OUT, "w") as f:
        f.write("\n".join(out))
    print("wrote", OUT, len(m.lines), "/", len(s.lines), "instructions")


if __name__ == "__main__":
    gen()
