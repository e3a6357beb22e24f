"""mclBnG1_mul / mclBnG2_mul on the cooperative ladders (k_ptmul.hip: GLV / GLS split on the host, four lanes per
ladder, the subgroup test as a ladder of its own) against the oracle's plain ladder (TPKE/PublicKey.cs:25-37,
TPKE/PrivateKey.cs:21-31 call them one element at a time).  Covers random points and scalars, the scalar edge cases
(0, 1, 2, r - 1, scalars with zero windows, the GLV half's carry bit), points outside the subgroup (the exact one-lane
fallback), the point at infinity, and Jacobian inputs with z != 1."""
import pytest

import oracle as o
from helpers import Drbg, gpu_native
from test_gpu_batched import off_subgroup_g1, off_subgroup_g2

pytestmark = pytest.mark.gpu
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


@pytest.fixture(scope="module")
def mcl():
    gpu_native()
    from lachain_amd import mcl as m
    return m


def _scalars(d):
    ks = [0, 1, 2, 3, 15, 16, R - 1, R - 2, (1 << 128) - 1, 1 << 128, (1 << 64) + 1, 0xd201000000010000 ** 2]
    ks += [d.fr_int() for _ in range(8)]
    return [k % R for k in ks]


@pytest.mark.parametrize("g", [1, 2])
def test_mul_matches_oracle(mcl, g):
    d = Drbg(b"gpu-ptmul-%d" % g)
    G = mcl.G1 if g == 1 else mcl.G2
    omul = o.g1_mul if g == 1 else o.g2_mul
    gen = o.g1_gen() if g == 1 else o.g2_gen()
    base = omul(gen, d.fr())
    B = G.FromBytes(base)
    J = B + G.FromBytes(gen)                                   # a Jacobian input with z != 1
    jb = J.ToBytes()
    for k in _scalars(d):
        kb = k.to_bytes(32, "little")
        assert (B * mcl.Fr.FromBytes(kb)).ToBytes() == omul(base, kb), k
        assert (J * mcl.Fr.FromBytes(kb)).ToBytes() == omul(jb, kb), k
    assert (G.Zero() * mcl.Fr.FromInt(5)).IsZero()


@pytest.mark.parametrize("g", [1, 2])
def test_mul_split_boundaries(mcl, g):
    """Round 6 cuts the GLV halves at bit 65 (G1) and the GLS digits at bit 32 (G2) over host-computed [2^65] P /
    [2^32] Q: scalars whose parts sit at those cuts (below lambda ~ 2^128 the G1 split is k1 = k, below |z| ~ 2^64 the G2
    digit d0 = k) and the parts' extremes, plus sums over the second half / digits."""
    d = Drbg(b"gpu-ptmul-split-%d" % g)
    G = mcl.G1 if g == 1 else mcl.G2
    omul = o.g1_mul if g == 1 else o.g2_mul
    gen = o.g1_gen() if g == 1 else o.g2_gen()
    base = omul(gen, d.fr())
    B = G.FromBytes(base)
    u = 0xD201000000010000
    if g == 1:
        ks = [1 << 64, (1 << 65) - 1, 1 << 65, (1 << 65) + 1, (1 << 66) - 1, (1 << 128) - 1, (1 << 127) + (1 << 65),
              u * u - 2, u * u - 1, u * u, (u * u - 1) * ((1 << 65) + 3) % R, (1 << 65) * (u * u - 1) % R]
    else:
        ks = [(1 << 32) - 1, 1 << 32, (1 << 32) + 1, (1 << 33) - 1, u - 1, (1 << 32) * u, ((1 << 32) - 1) * u + (1 << 32),
              u ** 3 + (1 << 32) * u ** 2 + 1, ((1 << 32) - 1) * (1 + u + u * u + u ** 3) % R]
    for k in ks:
        kb = (k % R).to_bytes(32, "little")
        assert (B * mcl.Fr.FromBytes(kb)).ToBytes() == omul(base, kb), hex(k)


@pytest.mark.parametrize("g", [1, 2])
def test_mul_outside_subgroup(mcl, g):
    """points with a cofactor-torsion component: the split's membership ladder rejects them and the exact one-lane
    ladder gives k P (G1.FromBytes / G2.FromBytes accept such points: HoneyBadgerSmartMalicious.cs:57-73)"""
    d = Drbg(b"gpu-ptmul-off-%d" % g)
    G = mcl.G1 if g == 1 else mcl.G2
    omul = o.g1_mul if g == 1 else o.g2_mul
    for _ in range(2):
        q = off_subgroup_g1(d) if g == 1 else off_subgroup_g2(d)
        Q = G.FromBytes(q)
        for k in (d.fr_int(), 7, R - 1):
            kb = k.to_bytes(32, "little")
            assert (Q * mcl.Fr.FromBytes(kb)).ToBytes() == omul(q, kb)


def test_mul_from_threads(mcl):
    import threading
    d = Drbg(b"gpu-ptmul-threads")
    base = o.g2_mul(o.g2_gen(), d.fr())
    ks = [d.fr() for _ in range(8)]
    want = [o.g2_mul(base, k) for k in ks]
    out, errs = [None] * 8, []

    def work(i):
        try:
            out[i] = (mcl.G2.FromBytes(base) * mcl.Fr.FromBytes(ks[i])).ToBytes()
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=work, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs and out == want
