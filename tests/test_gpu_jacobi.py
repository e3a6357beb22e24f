"""The binary Legendre-symbol routine (field.hpp fp_jacobi) that picks hash-to-G2's SvdW candidate and fp2_sqrt's
branch (h2g2.hpp g2_calc_bn, field.hpp fp2_sqrt_normed; the choice mcl's calcBN makes by square roots, reached from
TPKE/Utils.cs:21-27) against the exponent form a^((p-1)/2) on the same device and against Python's pow: random field
words, 0, 1, p - 1, small values, words with long runs of zero bits (the routine's whole-word shifts) and values next to
powers of two.  Run through the debug tower op (k_ops.hip OP_DEBUG_FP12, routine 12: twelve symbols per call)."""
import ctypes

import pytest

from helpers import Drbg, gpu_native

pytestmark = pytest.mark.gpu
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


def _legendre(v):
    v %= P
    if v == 0:
        return 0
    return 1 if pow(v, (P - 1) // 2, P) == 1 else -1


def _values(d):
    vs = [0, 1, 2, 3, 4, 5, P - 1, P - 2, P - 4, (P - 1) // 2, (P + 1) // 2, 1 << 32, 1 << 64, (1 << 96) + 1,
          (1 << 380) - 1, 1 << 380, 3 << 300, 0xFFFFFFFF, (1 << 352) | 1, 7 << 200]
    vs += [int.from_bytes(d.fr() + d.fr(), "little") % P for _ in range(100)]
    vs += [(int.from_bytes(d.fr(), "little") << (32 * k)) % P for k in range(6)]   # low words zero
    vs += [k * k % P for k in range(2, 14)] + [(k * k * 2) % P for k in range(2, 14)]   # squares, 2 * squares
    while len(vs) % 12:
        vs.append(int.from_bytes(d.fr(), "little"))
    return vs


def test_fp_jacobi_matches_the_exponent_and_python():
    nat = gpu_native()
    lib = nat.lib()
    d = Drbg(b"gpu-jacobi")
    vs = _values(d)
    for i in range(0, len(vs), 12):
        chunk = vs[i:i + 12]
        words = b"".join(v.to_bytes(48, "little") for v in chunk)
        out = ctypes.create_string_buffer(576)
        assert lib.lcb_debug_fp12(12, words, out) == 0
        w = [int.from_bytes(out.raw[4 * j:4 * j + 4], "little", signed=True) for j in range(24)]
        for k, v in enumerate(chunk):
            want = _legendre(v)
            assert w[2 * k] == want, (hex(v), w[2 * k], want)
            assert w[2 * k + 1] == want, (hex(v), w[2 * k + 1], want)
