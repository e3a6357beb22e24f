"""CPU check of the generated gfx950 leaf routines (lachain_amd/csrc/asm_routines.hpp, tools/gen_asm.py).

tools/asm_sim.py interprets each routine for one lane; results are compared with Python big-integer
Montgomery arithmetic (R = 2^384), and every register a routine writes must be inside the clobber/output
set its HIP wrapper declares (a routine writing an undeclared register would corrupt compiler-allocated
values on the GPU).  No GPU needed.
"""
import os
import random
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import asm_sim  # noqa: E402

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 1 << 384
RINV = pow(R, -1, P)


def mont(a, b):
    return a * b * RINV % P


@pytest.fixture(scope="module")
def lib():
    return asm_sim.load_library()


def wrapper_contract(label):
    """(VGPRs, SGPRs) the HIP wrapper of `label` lets the routine write (outputs + clobbers)."""
    src = open(asm_sim.HPP).read()
    body_end = src.index('    ""\n', src.index("#define LCB_ASM_LIBRARY_TEXT"))   # past the routines' own calls
    i = src.index(f"{label}@rel32@lo", body_end)
    blk = src[i:src.index("\n}", i)]
    vs = {int(x) for x in re.findall(r'"v(\d+)"', blk)}
    for lo, hi in re.findall(r'\{v\[(\d+):(\d+)\]\}', blk):
        vs |= set(range(int(lo), int(hi) + 1))
    ss = {int(x) for x in re.findall(r'"s(\d+)"', blk)}
    return vs, ss


def check_contract(label, lane):
    vs, ss = wrapper_contract(label)
    assert lane.written_v <= vs, f"{label} writes undeclared VGPRs {sorted(lane.written_v - vs)}"
    assert lane.written_s <= ss, f"{label} writes undeclared SGPRs {sorted(lane.written_s - ss)}"


def cases(rng, n):
    edge = [0, 1, P - 1, P - 2, (P - 1) // 2]
    out = [(rng.choice(edge), rng.choice(edge)) for _ in range(4)]
    out += [(rng.randrange(P), rng.randrange(P)) for _ in range(n)]
    return out


def test_fp_mul(lib):
    rng = random.Random(1)
    for a, b in cases(rng, 30):
        lane, rd = asm_sim.call(lib, "lcb_r_fp_mul", {0: a, 12: b})
        assert rd(0) == mont(a, b)
    check_contract("lcb_r_fp_mul", lane)


def test_fp_sqr(lib):
    rng = random.Random(11)
    for a, _ in cases(rng, 40):
        lane, rd = asm_sim.call(lib, "lcb_r_fp_sqr", {0: a})
        assert rd(0) == mont(a, a)
    check_contract("lcb_r_fp_sqr", lane)


def test_fp_mul_unreduced_multiplicands(lib):
    # Karatsuba sums reach the multiplier unreduced (< 2p); outputs must still be fully reduced
    rng = random.Random(2)
    for _ in range(30):
        a, b = rng.randrange(2 * P), rng.randrange(2 * P)
        lane, rd = asm_sim.call(lib, "lcb_r_fp_mul", {0: a, 12: b})
        assert rd(0) == mont(a, b)


def test_fp_mul2(lib):
    rng = random.Random(3)
    for (a0, b0), (a1, b1) in zip(cases(rng, 20), cases(rng, 20)):
        lane, rd = asm_sim.call(lib, "lcb_r_fp_mul2", {0: a0, 12: b0, 24: a1, 36: b1})
        assert rd(0) == mont(a0, b0) and rd(24) == mont(a1, b1)
    check_contract("lcb_r_fp_mul2", lane)


def test_fp2_mul(lib):
    rng = random.Random(4)
    for (xa, xb), (ya, yb) in zip(cases(rng, 20), cases(rng, 20)):
        lane, rd = asm_sim.call(lib, "lcb_r_fp2_mul", {0: xa, 12: xb, 24: ya, 36: yb})
        assert rd(0) == (mont(xa, ya) - mont(xb, yb)) % P
        assert rd(12) == (mont(xa, yb) + mont(xb, ya)) % P
    check_contract("lcb_r_fp2_mul", lane)


def test_fp2_sqr(lib):
    rng = random.Random(5)
    for xa, xb in cases(rng, 30):
        lane, rd = asm_sim.call(lib, "lcb_r_fp2_sqr", {0: xa, 12: xb})
        assert rd(0) == (mont(xa, xa) - mont(xb, xb)) % P
        assert rd(12) == 2 * mont(xa, xb) % P
    check_contract("lcb_r_fp2_sqr", lane)


def test_fp2_mul_fp(lib):
    rng = random.Random(6)
    for (xa, xb), (s, _) in zip(cases(rng, 20), cases(rng, 20)):
        lane, rd = asm_sim.call(lib, "lcb_r_fp2_mul_fp", {0: xa, 12: xb, 24: s})
        assert rd(0) == mont(xa, s) and rd(12) == mont(xb, s)
    check_contract("lcb_r_fp2_mul_fp", lane)


@pytest.mark.parametrize("which", [0, 1, 2, 3])
def test_fp_pow(which):
    """lcb_r_fp_pow (round 6): a^e for the four field exponents with the window table in VGPR islands, run as a
    program (labels, branches, nested calls) in the simulator; every register it writes is declared by its wrapper"""
    prog, labels = asm_sim.load_program(asm_sim.HPP, "LCB_ASM_LIBRARY_TEXT")
    e = [P - 2, (P + 1) // 4, (P - 1) // 2, (P - 3) // 4][which]
    vs, ss = wrapper_contract("lcb_r_fp_pow")
    rng = random.Random(which)
    for a in (rng.randrange(P), 1, P - 1):
        lane = asm_sim.ProgLane()
        am = a * R % P
        for j in range(12):
            lane.v[j] = (am >> (32 * j)) & 0xFFFFFFFF
        lane.s[84] = which
        lane.s[30] = lane.s[31] = 0
        asm_sim.run_program(prog, labels, "lcb_r_fp_pow", lane)
        got = sum(lane.v[j] << (32 * j) for j in range(12))
        assert got == pow(a, e, P) * R % P
        assert lane.written_v <= vs, sorted(lane.written_v - vs)
        assert lane.written_s <= ss | {84}, sorted(lane.written_s - ss)
