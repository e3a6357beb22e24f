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
