"""CPU check of the round-5 Fp12 assembly routines (lachain_amd/csrc/asm_tower.hpp, tools/gen_tower_asm.py):
lcb_r_fp2dw (double-width Fp2 product), lcb_r_fp12_mul_n (slot x slot Fp12 product over lazily reduced Fp6
products, optional conjugate of the first operand) and lcb_r_pow_z (conj(B^|z|) with the accumulator in AGPRs).

tools/asm_sim.py runs the library for one lane: registers, SALU, branches, calls, the slots in a simulated global
memory and the lane's LDS quads.  Results are compared with the oracle's Fp12 arithmetic (oracle.gt_mul /
gt_pow on canonical bytes, converted from the kernels' Montgomery words), and every register a routine writes must
be in the clobber set its HIP wrapper declares.  No GPU needed.
"""
import os
import random
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import asm_sim  # noqa: E402
import oracle as o  # noqa: E402

P = o.P
R = 1 << 384
RINV = pow(R, -1, P)
Z_ABS = 0xd201000000010000
BASE_A, BASE_M, BASE_T, BASE_D = 0x100000, 0x200000, 0x300000, 0x400000


@pytest.fixture(scope="module")
def prog():
    return asm_sim.load_program()


def words_of(vals):                 # 12 Fp values (Montgomery residues) -> 144 words
    return [(v >> (32 * j)) & 0xffffffff for v in vals for j in range(12)]


def to_bytes(vals):                 # Montgomery residues -> canonical GT bytes (oracle layout)
    return b"".join((v * RINV % P).to_bytes(48, "little") for v in vals)


def from_bytes(b):
    return [int.from_bytes(b[48 * i:48 * i + 48], "little") * R % P for i in range(12)]


def put_slot(lane, base, vals, n=2, i=1):
    """item i of an n-item quad-major slot (quad g of item i at base + (g * n + i) * 16)"""
    w = words_of(vals)
    for g in range(36):
        lane.store(base + (g * n + i) * 16, sum(w[4 * g + k] << (32 * k) for k in range(4)), 4)


def get_slot(lane, base, n=2, i=1):
    w = []
    for g in range(36):
        q = lane.load(base + (g * n + i) * 16, 4)
        w += [(q >> (32 * k)) & 0xffffffff for k in range(4)]
    return [sum(w[12 * c + j] << (32 * j) for j in range(12)) for c in range(12)]


def new_lane(n=2, i=1):
    lane = asm_sim.ProgLane()
    lane.v[248] = i * 16
    lane.v[249] = 64 + i * 16                     # LDS lane address (quad g at + g * 1024)
    lane.s[19] = n * 16
    for r in (30, 31):
        lane.s[r] = 0
    return lane


def set_pair(lane, s, addr):
    lane.s[s], lane.s[s + 1] = addr & 0xffffffff, addr >> 32


def contract(label):
    src = open(asm_sim.TOWER_HPP).read()
    i = src.index(f"{label}@rel32@lo", src.index("__device__ __forceinline__ void lcb_asm_fp12_mul_n"))
    blk = src[i:src.index("\n}", i)]
    return ({int(x) for x in re.findall(r'"v(\d+)"', blk)}, {int(x) for x in re.findall(r'"a(\d+)"', blk)},
            {int(x) for x in re.findall(r'"s(\d+)"', blk)})


def check_contract(label, lane, inputs_s):
    vs, as_, ss = contract(label)
    assert lane.written_v <= vs, sorted(lane.written_v - vs)
    assert lane.written_a <= as_, sorted(lane.written_a - as_)
    assert lane.written_s <= ss | inputs_s, sorted(lane.written_s - ss - inputs_s)
    assert not (lane.written_s & inputs_s - {30, 31}), "an input SGPR was overwritten"


def rand_fp12(rng, edge=False):
    if edge:
        return [rng.choice([0, 1, P - 1, P - 2, rng.randrange(P)]) for _ in range(12)]
    return [rng.randrange(P) for _ in range(12)]


def conj(vals):
    return vals[:6] + [(P - v) % P for v in vals[6:]]


def test_fp2dw(prog):
    """RE = xa ya - xb yb, IM = (xa + xb)(ya + yb) - xa ya - xb yb, mod 2^768, for inputs < p"""
    prg, labels = prog
    rng = random.Random(5)
    for t in range(12):
        x = [rng.choice([0, P - 1, rng.randrange(P)]) for _ in range(4)]
        lane = new_lane()
        for k, val in enumerate(x):
            for j in range(12):
                lane.v[12 * k + j] = (val >> (32 * j)) & 0xffffffff
        lane.s[28] = lane.s[29] = 0
        asm_sim.run_program(prg, labels, "lcb_r_fp2dw", lane)
        rd = lambda base: sum(lane.v[base + j] << (32 * j) for j in range(24))      # noqa: E731
        xa, xb, ya, yb = x
        assert rd(72) == (xa * ya - xb * yb) % (1 << 768)
        assert rd(120) == (xa * yb + xb * ya)
        assert max(lane.written_v) < 160


@pytest.mark.parametrize("conj_a", [0, 1])
def test_fp12_mul_n(prog, conj_a):
    prg, labels = prog
    rng = random.Random(11 + conj_a)
    for t in range(3):
        a, m = rand_fp12(rng, edge=(t == 0)), rand_fp12(rng, edge=(t == 1))
        lane = new_lane()
        put_slot(lane, BASE_A, a)
        put_slot(lane, BASE_M, m)
        set_pair(lane, 56, BASE_A)
        set_pair(lane, 20, BASE_M)
        set_pair(lane, 22, BASE_D)                # tmp = the destination (fe_asm.hpp's choice)
        set_pair(lane, 60, BASE_D)
        lane.s[65] = conj_a
        asm_sim.run_program(prg, labels, "lcb_r_fp12_mul_n", lane)
        got = get_slot(lane, BASE_D)
        want = from_bytes(o.gt_mul(to_bytes(conj(a) if conj_a else a), to_bytes(m)))
        assert got == want, t
        check_contract("lcb_r_fp12_mul_n", lane, {19, 20, 21, 22, 23, 56, 57, 60, 61, 65, 30, 31})
    if conj_a == 0:
        print("lcb_r_fp12_mul_n dynamic instructions:", sum(v for k, v in lane.counts.items() if not
                                                            k.startswith("s_nop")), "s_nop", lane.counts.get("s_nop"))


def test_fp12_mul_n_dst_is_a(prog):
    """fx_mul(U, U, T, ...): the destination is the first operand (loaded before anything is written)"""
    prg, labels = prog
    rng = random.Random(3)
    a, m = rand_fp12(rng), rand_fp12(rng)
    lane = new_lane()
    put_slot(lane, BASE_A, a)
    put_slot(lane, BASE_M, m)
    for s, v in ((56, BASE_A), (20, BASE_M), (22, BASE_A), (60, BASE_A)):
        set_pair(lane, s, v)
    lane.s[65] = 1
    asm_sim.run_program(prg, labels, "lcb_r_fp12_mul_n", lane)
    assert get_slot(lane, BASE_A) == from_bytes(o.gt_mul(to_bytes(conj(a)), to_bytes(m)))


@pytest.mark.parametrize("same", [False, True])
def test_pow_z(prog, same):
    """conj(B^|z|) = B^(r - |z|) for B in GT (a pairing value); the destination may be the base slot"""
    prg, labels = prog
    gt = o.pairing(o.g1_mul(o.g1_gen(), o.fr(7 + same)), o.g2_gen())
    b = from_bytes(gt)
    lane = new_lane()
    put_slot(lane, BASE_M, b)
    set_pair(lane, 20, BASE_M)
    set_pair(lane, 22, BASE_T)
    set_pair(lane, 60, BASE_M if same else BASE_D)
    asm_sim.run_program(prg, labels, "lcb_r_pow_z", lane)
    got = get_slot(lane, BASE_M if same else BASE_D)
    assert got == from_bytes(o.gt_pow(gt, o.fr(o.R - Z_ABS)))
    check_contract("lcb_r_pow_z", lane, {19, 20, 21, 22, 23, 60, 61, 30, 31})


# ---------------------------------------------------------------- the Miller loop routines (lcb_r_fp12sq, lcb_r_line,
# lcb_r_miller2)
sys.path.insert(0, os.path.join(ROOT, "tests", "pyref"))
import bls12_381 as pr  # noqa: E402

BASE_S2, BASE_P, BASE_LS1, BASE_LS2 = 0x500000, 0x600000, 0x700000, 0x800000
B3 = (12, 12)                                     # 3 b', b' = 4 (1 + u)
INV2 = pow(2, -1, P)


def mont(x):
    return x * R % P


def f2w(x):                                       # Fp2 (canonical) -> 24 Montgomery words
    return words_of([mont(x[0]), mont(x[1])])[:24]


def line_set(Q):
    """pairing.hpp lineset_compute in canonical arithmetic: 68 normalised lines (B', C') of the affine G2 point Q"""
    f2 = pr
    xq, yq = Q
    T = [xq, yq, (1, 0)]
    raw = []

    def dbl(T):
        x, y, z = T
        XX, YY, ZZ = f2.f2mul(x, x), f2.f2mul(y, y), f2.f2mul(z, z)
        bZZ = f2.f2mul(ZZ, B3)
        YZ = f2.f2mul(y, z)
        A = f2.f2sub(YY, bZZ)
        Bc = f2.f2neg(f2.f2add(f2.f2add(XX, XX), XX))
        Cc = f2.f2add(YZ, YZ)
        b9 = f2.f2add(f2.f2add(bZZ, bZZ), bZZ)
        X3 = f2.f2mul(f2.f2mul(f2.f2mul(x, y), (INV2, 0)), f2.f2sub(YY, b9))
        s = f2.f2mul(f2.f2add(YY, b9), (INV2, 0))
        t = f2.f2mul(bZZ, bZZ)
        Y3 = f2.f2sub(f2.f2mul(s, s), f2.f2add(f2.f2add(t, t), t))
        Z3 = f2.f2mul(YY, YZ)
        Z3 = f2.f2add(Z3, Z3)
        return (A, Bc, Cc), [X3, Y3, Z3]

    def add(T):
        x, y, z = T
        th = f2.f2sub(y, f2.f2mul(yq, z))
        la = f2.f2sub(x, f2.f2mul(xq, z))
        A = f2.f2sub(f2.f2mul(th, xq), f2.f2mul(la, yq))
        C, D = f2.f2mul(th, th), f2.f2mul(la, la)
        E, F, G = f2.f2mul(la, D), f2.f2mul(z, C), f2.f2mul(x, D)
        H = f2.f2sub(f2.f2sub(f2.f2add(E, F), G), G)
        return (A, f2.f2neg(th), la), [f2.f2mul(la, H), f2.f2sub(f2.f2mul(th, f2.f2sub(G, H)), f2.f2mul(y, E)),
                                       f2.f2mul(z, E)]

    for i in range(62, -1, -1):
        ln, T = dbl(T)
        raw.append(ln)
        if (Z_ABS >> i) & 1:
            ln, T = add(T)
            raw.append(ln)
    assert len(raw) == 68
    out = []
    for A, Bc, Cc in raw:
        ai = pr.f2inv(A)
        out.append((pr.f2mul(Bc, ai), pr.f2mul(Cc, ai)))
    return out


def put_lines(lane, base, lines):
    w = []
    for b_, c_ in lines:
        w += f2w(b_) + f2w(c_)
    for j in range(0, len(w), 4):
        lane.store(base + 4 * j, sum(w[j + k] << (32 * k) for k in range(4)), 4)


def put_points(lane, pts, n=2, i=1):
    """P1 at quads 0..5, P2 at quads 6..11 of the P slot; infinity -> (0, 0)"""
    w = []
    for pt in pts:
        x, y = (0, 0) if pt is None else (mont(pt[0]), mont(pt[1]))
        w += words_of([x, y])[:24]
    for g in range(12):
        lane.store(BASE_P + (g * n + i) * 16, sum(w[4 * g + k] << (32 * k) for k in range(4)), 4)


def set_p(lane):                                  # PR = p in v160..171 and PINV in s88 (set by lcb_r_miller2)
    for r_, v in zip(range(160, 172), [(P >> (32 * j)) & 0xffffffff for j in range(12)]):
        lane.v[r_] = v
    lane.s[88] = (-pow(P, -1, 1 << 32)) % (1 << 32)


def test_fp12sq(prog):
    prg, labels = prog
    rng = random.Random(21)
    for t in range(2):
        a = rand_fp12(rng, edge=(t == 0))
        lane = new_lane()
        set_p(lane)
        for j, v in enumerate(words_of(a)):
            lane.a[j] = v
        for s_, base in ((22, BASE_T), (58, BASE_S2)):
            set_pair(lane, s_, base)
        asm_sim.run_program(prg, labels, "lcb_r_fp12sq", lane)
        got = [sum(lane.a[12 * c + j] << (32 * j) for j in range(12)) for c in range(12)]
        assert got == from_bytes(o.gt_mul(to_bytes(a), to_bytes(a))), t


def test_line(prog):
    """f * (1 + b v + c v w), b = B' xP, c = C' yP: against the full Fp12 product by the line's element"""
    prg, labels = prog
    rng = random.Random(22)
    for t, inf in enumerate((False, True)):
        f = rand_fp12(rng, edge=(t == 1))
        Bp = (rng.randrange(P), rng.randrange(P))
        Cp = (rng.randrange(P), rng.randrange(P))
        pt = None if inf else (rng.randrange(P), rng.randrange(P))
        lane = new_lane()
        for j, v in enumerate(words_of(f)):
            lane.a[j] = v
        put_lines(lane, BASE_LS1, [(Bp, Cp)])
        put_points(lane, [pt, None])
        set_pair(lane, 56, BASE_P)
        lane.v[244], lane.v[245] = BASE_LS1 & 0xffffffff, BASE_LS1 >> 32
        lane.v[246], lane.v[247] = 0, 0
        set_p(lane)
        lane.s[62], lane.s[63] = 0, 0
        asm_sim.run_program(prg, labels, "lcb_r_line", lane)
        got = [sum(lane.a[12 * c + j] << (32 * j) for j in range(12)) for c in range(12)]
        b_ = (0, 0) if inf else pr.f2mul(Bp, (pt[0], 0))
        c_ = (0, 0) if inf else pr.f2mul(Cp, (pt[1], 0))
        L = [mont(1), 0, mont(b_[0]), mont(b_[1]), 0, 0, 0, 0, mont(c_[0]), mont(c_[1]), 0, 0]
        assert got == from_bytes(o.gt_mul(to_bytes(f), to_bytes(L))), t


@pytest.mark.parametrize("p2_inf", [False, True])
def test_miller2(prog, p2_inf):
    """final_exp(lcb_r_miller2) == e(P1, Q1) e(P2, Q2) (the normalised lines differ from the oracle's Miller value by
    factors the final exponentiation removes); P2 at infinity contributes 1"""
    prg, labels = prog
    s1, s2, t1, t2 = 11, 29, 5, 13 + p2_inf
    Q1b, Q2b = o.g2_mul(o.g2_gen(), o.fr(s1)), o.g2_mul(o.g2_gen(), o.fr(s2))
    P1b, P2b = o.g1_mul(o.g1_gen(), o.fr(t1)), o.g1_mul(o.g1_gen(), o.fr(t2))
    Q1, Q2, P1, P2 = pr.g2_from_bytes(Q1b), pr.g2_from_bytes(Q2b), pr.g1_from_bytes(P1b), pr.g1_from_bytes(P2b)
    lane = new_lane()
    put_lines(lane, BASE_LS1, line_set(Q1))
    put_lines(lane, BASE_LS2, line_set(Q2))
    put_points(lane, [P1, None if p2_inf else P2])
    set_pair(lane, 56, BASE_P)
    set_pair(lane, 22, BASE_T)
    set_pair(lane, 58, BASE_S2)
    set_pair(lane, 60, BASE_D)
    lane.v[250], lane.v[251] = BASE_LS1 & 0xffffffff, BASE_LS1 >> 32
    lane.v[252], lane.v[253] = BASE_LS2 & 0xffffffff, BASE_LS2 >> 32
    asm_sim.run_program(prg, labels, "lcb_r_miller2", lane)
    f = get_slot(lane, BASE_D)
    want = o.pairing(P1b, Q1b)
    if not p2_inf:
        want = o.gt_mul(want, o.pairing(P2b, Q2b))
    assert o.final_exp(to_bytes(f)) == want
    vs, as_, ss = contract("lcb_r_miller2")
    assert lane.written_v <= vs and lane.written_a <= as_, (sorted(lane.written_v - vs), sorted(lane.written_a - as_))
    inputs = {19, 22, 23, 56, 57, 58, 59, 60, 61, 30, 31}
    assert lane.written_s <= ss | inputs and not (lane.written_s & inputs - {30, 31})
