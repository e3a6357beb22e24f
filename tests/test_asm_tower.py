"""CPU check of the generated Fp12-level gfx950 routines (lachain_amd/csrc/asm_tower.hpp, tools/gen_tower_asm.py).

tools/asm_sim.py interprets the routines for one lane (AGPR file included, nested calls followed); results are
compared with a plain big-integer restatement of mcl's tower (Fp2 = Fp[i]/(i^2+1), Fp6 = Fp2[v]/(v^3-(1+i)),
Fp12 = Fp6[w]/(w^2-v)) in Montgomery form (R = 2^384), and every register a routine writes must be declared by
its HIP wrapper.  No GPU needed.
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


# ---- mcl tower over plain integers (elements as nested tuples; Fp12 flattened to 12 Fp in struct order)
def f2mul(x, y):
    return ((x[0] * y[0] - x[1] * y[1]) % P, (x[0] * y[1] + x[1] * y[0]) % P)


def f2add(x, y):
    return ((x[0] + y[0]) % P, (x[1] + y[1]) % P)


def f2xi(x):  # (a + b i)(1 + i)
    return ((x[0] - x[1]) % P, (x[0] + x[1]) % P)


def f6mul(a, b):
    c = [(0, 0)] * 5
    for i in range(3):
        for j in range(3):
            c[i + j] = f2add(c[i + j], f2mul(a[i], b[j]))
    return (f2add(c[0], f2xi(c[3])), f2add(c[1], f2xi(c[4])), c[2])


def f6add(a, b):
    return tuple(f2add(x, y) for x, y in zip(a, b))


def f6v(a):  # a * v
    return (f2xi(a[2]), a[0], a[1])


def f12mul(a, b):
    t0, t1 = f6mul(a[0], b[0]), f6mul(a[1], b[1])
    c1 = f6add(f6mul(a[0], b[1]), f6mul(a[1], b[0]))
    return (f6add(t0, f6v(t1)), c1)


def f12pow(a, e):
    acc = ((((1, 0), (0, 0), (0, 0)), ((0, 0), (0, 0), (0, 0))))
    for bit in bin(e)[2:]:
        acc = f12mul(acc, acc)
        if bit == "1":
            acc = f12mul(acc, a)
    return acc


def flat(a):
    return [a[d][c][k] for d in range(2) for c in range(3) for k in range(2)]


def unflat(v):
    return tuple(tuple((v[6 * d + 2 * c], v[6 * d + 2 * c + 1]) for c in range(3)) for d in range(2))


def cyclotomic(rng):
    h = unflat([rng.randrange(P) for _ in range(12)])
    return f12pow(h, (P ** 6 - 1) * (P ** 2 + 1))


@pytest.fixture(scope="module")
def lib():
    return asm_sim.load_library(asm_sim.TOWER_HPP, "LCB_ASM_TOWER_LIBRARY_TEXT")


@pytest.fixture(scope="module")
def cyc_elems():
    rng = random.Random(7)
    return [cyclotomic(rng) for _ in range(3)]


def wrapper_contract(label):
    src = open(asm_sim.TOWER_HPP).read()
    i = src.index(f"{label}@rel32@lo")
    blk = src[i:src.index("\n}", i)]
    vs = {int(x) for x in re.findall(r'"v(\d+)"', blk)}
    ags = {int(x) for x in re.findall(r'"a(\d+)"', blk)}
    for lo, hi in re.findall(r'\{a\[(\d+):(\d+)\]\}', blk):
        ags |= set(range(int(lo), int(hi) + 1))
    ss = {int(x) for x in re.findall(r'"s(\d+)"', blk)}
    return vs, ags, ss


def run_cyc_sqr(lib, f):
    mont = [x * R % P for x in flat(f)]
    lane, _ = asm_sim.call(lib, "lcb_r_cyc_sqr", {}, {12 * k: mont[k] for k in range(12)})
    out = [sum(lane.a[12 * k + j] << (32 * j) for j in range(12)) for k in range(12)]
    return lane, out


def test_cyc_sqr_matches_tower_square(lib, cyc_elems):
    rinv = pow(R, -1, P)
    for f in cyc_elems:
        lane, out = run_cyc_sqr(lib, f)
        assert all(o < P for o in out), "outputs must be fully reduced"
        assert [o * rinv % P for o in out] == flat(f12mul(f, f))
    vs, ags, ss = wrapper_contract("lcb_r_cyc_sqr")
    assert lane.written_v <= vs, sorted(lane.written_v - vs)
    assert lane.written_a <= ags, sorted(lane.written_a - ags)
    assert lane.written_s <= ss, sorted(lane.written_s - ss)


def test_cyc_sqr_chain(lib, cyc_elems):
    """three squarings in a row (outputs feed inputs, as in the exponentiation loop)"""
    rinv = pow(R, -1, P)
    f = cyc_elems[0]
    x = f
    for _ in range(3):
        _, out = run_cyc_sqr(lib, x)
        x = unflat([o * rinv % P for o in out])
    assert flat(x) == flat(f12pow(f, 8))


def test_cyc_sqr_edge_values(lib):
    """the identity and its conjugate-free edge: 1^2 = 1; p - 1 limbs exercise the 3p/8p ranges"""
    one = unflat([1] + [0] * 11)
    rinv = pow(R, -1, P)
    _, out = run_cyc_sqr(lib, one)
    assert [o * rinv % P for o in out] == flat(one)
