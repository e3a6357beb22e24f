"""The oracle's timing build (bench CPU baseline: gcc -O3 -march=native -DORC_FAST, the MULX/ADCX/ADOX Fp product of
oracle/mont_adx.h) against the portable test build: same bytes for every routine the baselines time.  CPU test."""
import ctypes
import os
import shutil
import subprocess

import pytest

import oracle as o
from helpers import Drbg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORC = os.path.join(ROOT, "oracle")


@pytest.fixture(scope="module")
def fast(tmp_path_factory):
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    out = str(tmp_path_factory.mktemp("orc") / "liborc_fast.so")
    src = [os.path.join(ORC, f) for f in ("bls.c", "hash.c", "rs.c", "secp.c")]
    subprocess.run(["gcc", "-O3", "-march=native", "-DORC_FAST", "-fPIC", "-fopenmp", "-shared", "-o", out] + src,
                   check=True, capture_output=True, timeout=300)
    lib = ctypes.CDLL(out)
    lib.orc_init()
    if lib.orc_fp_impl() != 1:
        pytest.skip("host without BMI2/ADX: the timing build keeps the C product")
    return lib


def _call(lib, name, size, *args):
    buf = ctypes.create_string_buffer(size)
    assert getattr(lib, name)(buf, *args) == 0
    return buf.raw


def test_timing_build_matches_portable(fast):
    ref = o.lib()
    assert ref.orc_fp_impl() == 0
    d = Drbg(b"orc-adx")
    g1, g2 = o.g1_gen(), o.g2_gen()
    for _ in range(6):
        a, b = d.fr(), d.fr()
        P = _call(ref, "orc_g1_mul", 48, g1, a)
        Q = _call(ref, "orc_g2_mul", 96, g2, b)
        assert _call(fast, "orc_g1_mul", 48, g1, a) == P
        assert _call(fast, "orc_g2_mul", 96, g2, b) == Q
        assert _call(fast, "orc_pairing", 576, P, Q) == _call(ref, "orc_pairing", 576, P, Q)
        m = d.bytes(40)
        assert _call(fast, "orc_g2_hash", 96, m, ctypes.c_size_t(len(m))) == \
            _call(ref, "orc_g2_hash", 96, m, ctypes.c_size_t(len(m)))
        assert _call(fast, "orc_fr_mul", 32, a, b) == _call(ref, "orc_fr_mul", 32, a, b)
    # TPKE share check, both outcomes
    x, r = d.fr(), d.fr()
    Y = _call(ref, "orc_g1_mul", 48, g1, x)
    msg = d.bytes(32)
    U, V, W = o.tpke_encrypt(Y, msg, r)
    Ui = _call(ref, "orc_g1_mul", 48, U, x)
    for lib in (fast, ref):
        assert lib.orc_tpke_verify_share(Y, U, V, ctypes.c_size_t(len(V)), W, Ui) == 1
        assert lib.orc_tpke_verify_share(Y, U, V, ctypes.c_size_t(len(V)), W, Y) == 0
