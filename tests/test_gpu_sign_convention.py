"""lcb_set_g2_sign_from_b: the G2 wire flag carries the parity of y.b instead of y.a (an unpinned mcl convention,
DESIGN.md §4), switched at run time for the host (de)serialization and for every kernel that (de)compresses G2 points,
mirroring the oracle's orc_set_g2_sign_from_b (oracle/bls.c:517-521,691).  Checked in both settings against the
oracle: host round trips, the device hash-to-G2 output (device compression), a G2 Lagrange batch (device decompression
and compression) and the G2 scalar multiplication's output."""
import pytest

import oracle as o
from helpers import Drbg, gpu_native

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nat():
    n = gpu_native()
    yield n
    n.set_g2_sign_from_b(False)
    o.set_g2_sign_from_b(0)


@pytest.mark.parametrize("use_b", [True, False])
def test_g2_sign_flag_both_conventions(nat, use_b):
    from lachain_amd import mcl
    nat.set_g2_sign_from_b(use_b)
    o.set_g2_sign_from_b(1 if use_b else 0)
    try:
        d = Drbg(b"g2-sign-%d" % use_b)
        scal = [d.fr() for _ in range(6)]
        pts = [o.g2_mul(o.g2_gen(), s) for s in scal]
        for s, p in zip(scal, pts):
            P = mcl.G2.FromBytes(p)
            assert P.ToBytes() == p
            assert (mcl.G2.Generator() * mcl.Fr.FromBytes(s)).ToBytes() == p      # device mul, host serialize
        msgs = [d.bytes(n) for n in (0, 7, 32, 100)]
        assert nat.g2_hash_batch(msgs) == [o.g2_hash(m) for m in msgs]
        xs = [o.fr(i + 1) for i in range(4)]
        got = nat.lagrange_batch(2, [(xs, pts[:4])])
        assert got == [o.g2_lagrange(xs, pts[:4])]
    finally:
        nat.set_g2_sign_from_b(False)
        o.set_g2_sign_from_b(0)


def test_default_convention_restored(nat):
    from lachain_amd import mcl
    from helpers import kats
    assert mcl.G2.Generator().ToBytes().hex() == kats()["g2_generator"]["hex"]
