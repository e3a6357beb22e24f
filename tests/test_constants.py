"""CPU test: the GLV constant of G1 emitted by tools/gen_constants.py into lachain_amd/csrc/bls_constants.hpp
(LCB_G1_BETA, used by g1_mul_glv in curve.hpp) is the cube root of unity whose map (x, y) -> (beta x, y) is
multiplication by lambda = z^2 - 1, checked against the oracle's own scalar multiplication of the generator.
"""
import os
import re

import oracle as o

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
Z_ABS = 0xD201000000010000


def _const(name):
    text = open(os.path.join(ROOT, "lachain_amd", "csrc", "bls_constants.hpp")).read()
    m = re.search(name + r"\[\d+\] = \{([^}]*)\}", text)
    assert m, name
    limbs = [int(v.strip().rstrip("u"), 16) for v in m.group(1).split(",")]
    return sum(v << (32 * i) for i, v in enumerate(limbs))


def _x(enc48):
    b = bytearray(enc48)
    b[47] &= 0x1F  # flag bits
    return int.from_bytes(bytes(b), "little")


def test_g1_glv_beta_matches_lambda():
    beta = _const("LCB_G1_BETA") * pow(1 << 384, -1, P) % P  # out of Montgomery form
    assert beta != 1 and pow(beta, 3, P) == 1
    lam = Z_ABS * Z_ABS - 1
    assert (lam * lam + lam + 1) % R == 0
    g = o.g1_gen()
    lg = o.g1_mul(g, lam.to_bytes(32, "little"))
    assert _x(lg) == beta * _x(g) % P
    # phi keeps y: lambda G and G share the y-parity flag
    assert (lg[47] & 0xE0) == (g[47] & 0xE0)
