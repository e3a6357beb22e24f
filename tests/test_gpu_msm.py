"""GPU parity of the Pippenger G1 MSM (k_msm.hip) against the oracle (oracle/bls.c orc_g1_msm, the
restatement of mclBnG1_mulVec / MclBls12381.LagrangeInterpolate in G1 — TPKE/PublicKey.cs:83,
ThresholdSignature/PublicKeySet.cs:31).  Bit-exact: serialized 48-byte G1 results.

Edge cases: n = 0/1/2, zero and r-1 scalars, duplicated points (doubling inside a bucket), P and -P
(cancellation), points at infinity, every window width the digit decomposition has a special case for
(255 mod c == 0 adds a carry window), raw scalars >= r on the device path (reduced mod r), and the
per-GPU-partial sum used after the RCCL all-gather.
"""
import pytest

import oracle as o
from helpers import Drbg, R, gpu_native

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nat():
    return gpu_native()


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    return torch, torch.device("cuda", 0)


def _expected(points, scalars):
    acc = bytes(48)
    for p, s in zip(points, scalars):
        acc = o.g1_add(acc, o.g1_mul(p, o.fr(s % R)))
    return acc


def _dev_msm(nat, torch, dev, points48, scalars_raw, window_bits=0, glv=False):
    """points48: serialized G1; scalars_raw: 32-byte LE (any 256-bit value) -> serialized MSM via the _dev ABI"""
    n = len(points48)
    lib = nat.lib()
    s = torch.cuda.current_stream(dev).cuda_stream
    d_in = torch.frombuffer(bytearray(b"".join(points48) or b"\0"), dtype=torch.uint8).to(dev)
    d_sc = torch.frombuffer(bytearray(b"".join(scalars_raw) or b"\0"), dtype=torch.uint8).to(dev)
    d_aff = torch.zeros(max(1, 96 * n), dtype=torch.uint8, device=dev)
    d_ok = torch.zeros(max(1, n), dtype=torch.uint8, device=dev)
    d_jac = torch.zeros(144, dtype=torch.uint8, device=dev)
    d_out = torch.zeros(48, dtype=torch.uint8, device=dev)
    assert lib.lcb_g1_to_affine_dev(d_aff.data_ptr(), d_ok.data_ptr(), d_in.data_ptr(), n, s) == 0
    fn = lib.lcb_g1_msm_glv_dev if glv else lib.lcb_g1_msm_dev
    assert fn(d_jac.data_ptr(), d_aff.data_ptr(), d_sc.data_ptr(), n, window_bits, s) == 0, nat.last_error()
    assert lib.lcb_g1_jac_sum_dev(d_out.data_ptr(), None, d_jac.data_ptr(), 1, s) == 0
    torch.cuda.synchronize(dev)
    if n:
        assert bool(d_ok.cpu().all())
    return bytes(d_out.cpu().numpy().tobytes()), d_jac


def test_msm_known_answer_sizes(nat):
    d = Drbg(b"gpu-msm-sizes")
    for n in (1, 2, 3, 64, 1000):
        a = [d.fr_int() for _ in range(n)]
        s = [d.fr_int() for _ in range(n)]
        pts = nat.mul_batch(1, None, [o.fr(v) for v in a], generator=True)
        got = nat.g1_msm(pts, [o.fr(v) for v in s])
        assert got == o.g1_mul(o.g1_gen(), o.fr(sum(x * y for x, y in zip(a, s)) % R)), n


def test_msm_matches_oracle_mulvec(nat):
    d = Drbg(b"gpu-msm-mulvec")
    n = 40
    pts = nat.mul_batch(1, None, [d.fr() for _ in range(n)], generator=True)
    sc = [d.fr() for _ in range(n)]
    assert nat.g1_msm(pts, sc) == o.g1_msm(pts, sc)


def test_msm_edge_scalars_and_points(nat):
    d = Drbg(b"gpu-msm-edges")
    G = o.g1_gen()
    P = o.g1_mul(G, d.fr())
    Q = o.g1_mul(G, d.fr())
    zero = bytes(48)
    points = [P, P, P, o.g1_neg(P), Q, zero, Q, G, G]
    scal = [5, 5, 0, 5, R - 1, 123, 1, 1, (1 << 200) + 7]
    assert nat.g1_msm(points, [o.fr(v) for v in scal]) == _expected(points, scal)
    # all-zero scalars and a sum that cancels to infinity
    assert nat.g1_msm([P, Q], [o.fr(0), o.fr(0)]) == zero
    assert nat.g1_msm([P, o.g1_neg(P)], [o.fr(9), o.fr(9)]) == zero
    assert nat.g1_msm([], []) == zero


def test_msm_rejects_noncanonical_scalar_and_bad_point(nat):
    G = o.g1_gen()
    with pytest.raises(RuntimeError):
        nat.g1_msm([G], [R.to_bytes(32, "little")])
    bad = bytearray(G)
    bad[0] ^= 1  # x no longer on the curve (with overwhelming probability)
    if not o.g1_valid(bytes(bad)):
        with pytest.raises(RuntimeError):
            nat.g1_msm([bytes(bad)], [o.fr(1)])


@pytest.mark.parametrize("c", [2, 4, 5, 7, 8, 12, 13, 15, 16, 17, 20])
def test_msm_window_widths(nat, torch_dev, c):
    torch, dev = torch_dev
    d = Drbg(b"gpu-msm-window-%d" % c)
    n = 300
    a = [d.fr_int() for _ in range(n)]
    s = [d.fr_int() for _ in range(n)]
    s[0], s[1], s[2] = 0, R - 1, (1 << 255) - 1 - ((1 << 255) - 1) % R  # a multiple of r: contributes 0
    pts = nat.mul_batch(1, None, [o.fr(v) for v in a], generator=True)
    got, _ = _dev_msm(nat, torch, dev, pts, [v.to_bytes(32, "little") for v in s], c)
    assert got == o.g1_mul(o.g1_gen(), o.fr(sum(x * y for x, y in zip(a, s)) % R)), c


def test_msm_dev_reduces_raw_scalars(nat, torch_dev):
    torch, dev = torch_dev
    d = Drbg(b"gpu-msm-raw")
    n = 50
    a = [d.fr_int() for _ in range(n)]
    s = [int.from_bytes(d.bytes(32), "little") for _ in range(n)]   # uniform 256-bit, mostly >= r
    s[0] = (1 << 256) - 1
    pts = nat.mul_batch(1, None, [o.fr(v) for v in a], generator=True)
    got, _ = _dev_msm(nat, torch, dev, pts, [v.to_bytes(32, "little") for v in s])
    assert got == o.g1_mul(o.g1_gen(), o.fr(sum(x * y for x, y in zip(a, s)) % R))


def test_msm_partials_sum(nat, torch_dev):
    # the multi-GPU path: per-rank Jacobian partials, all-gathered, summed by lcb_g1_jac_sum_dev
    torch, dev = torch_dev
    d = Drbg(b"gpu-msm-partials")
    parts, total = [], 0
    for k in range(4):
        n = 100 + 37 * k
        a = [d.fr_int() for _ in range(n)]
        s = [d.fr_int() for _ in range(n)]
        total += sum(x * y for x, y in zip(a, s))
        pts = nat.mul_batch(1, None, [o.fr(v) for v in a], generator=True)
        _, jac = _dev_msm(nat, torch, dev, pts, [o.fr(v) for v in s])
        parts.append(jac.clone())
    cat = torch.cat(parts)
    out = torch.zeros(48, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    assert nat.lib().lcb_g1_jac_sum_dev(out.data_ptr(), None, cat.data_ptr(), 4, st) == 0
    torch.cuda.synchronize(dev)
    assert bytes(out.cpu().numpy().tobytes()) == o.g1_mul(o.g1_gen(), o.fr(total % R))


def test_glv_msm_vs_oracle(nat, torch_dev):
    """lcb_g1_msm_glv_dev (points of order r): s = s1 + s2 lambda over P and phi(P); edge scalars 0, 1, r - 1,
    lambda, lambda + 1, u^2 multiples, raw values >= r, duplicated / opposite points, infinity; every window width
    with a special case in the 129-bit digit split"""
    torch, dev = torch_dev
    d = Drbg(b"gpu-msm-glv")
    G = o.g1_gen()
    lam = 0xD201000000010000 ** 2 - 1
    u2 = 0xD201000000010000 ** 2
    edge = [0, 1, R - 1, lam, lam + 1, u2, u2 - 1, 2 * u2 + 5, (R - 1) // u2 * u2, 2 ** 256 - 1, R, R + 7]
    for n in (1, 2, 13, 300):
        pts = [o.g1_mul(G, d.fr()) for _ in range(n)]
        if n >= 13:
            pts[3] = pts[2]
            pts[4] = o.g1_neg(pts[2])
            pts[5] = bytes(48)
        raw = [d.fr_int() for _ in range(n)]
        for k, e in enumerate(edge[: n]):
            raw[k] = e
        sc = [(v % 2 ** 256).to_bytes(32, "little") for v in raw]
        want = o.g1_msm(pts, [o.fr(v % R) for v in raw])
        for c in (0, 4, 5, 7, 8, 13, 16, 17):
            got, _ = _dev_msm(nat, torch, dev, pts, sc, c, glv=True)
            assert got == want, (n, c)


def test_glv_msm_known_answer_1m(nat, torch_dev):
    torch, dev = torch_dev
    d = Drbg(b"gpu-msm-glv-1m")
    n = 1 << 20
    a = [d.fr_int() for _ in range(n)]
    s = [d.fr_int() for _ in range(n)]
    pts = nat.mul_batch_raw(1, None, b"".join(o.fr(v) for v in a), n, generator=True)
    got, _ = _dev_msm(nat, torch, dev, [pts[48 * i:48 * i + 48] for i in range(n)], [o.fr(v) for v in s], 0, glv=True)
    assert got == o.g1_mul(o.g1_gen(), o.fr(sum(x * y for x, y in zip(a, s)) % R))


@pytest.mark.parametrize("chunk", [0, 1, 3, 64, 4096])
@pytest.mark.parametrize("glv", [False, True])
def test_msm_record_chunks(nat, torch_dev, chunk, glv):
    """record-balanced bucket accumulation (k_msm_chunk_acc + k_msm_bucket_fix) at several chunk sizes, on a skewed
    digit distribution: one scalar repeated (every record of a window in one bucket, spanning many chunks), duplicated
    points, P and -P, zero scalars, and random ones; the result equals the oracle's and the one-lane-per-bucket form's
    (chunk 0)"""
    torch, dev = torch_dev
    d = Drbg(b"gpu-msm-chunks")
    n = 700
    base = [o.g1_mul(o.g1_gen(), d.fr()) for _ in range(n // 2)]
    pts = base + base[: n - len(base)]
    pts[5] = o.g1_neg(pts[4])
    sc = [d.fr_int() for _ in range(n)]
    for i in range(0, n, 3):
        sc[i] = 0x1234567890ABCDEF1234567890ABCDEF12345678
    for i in range(1, n, 17):
        sc[i] = 0
    want = _expected(pts, sc)
    nat.set_msm_chunk(chunk)
    try:
        got, _ = _dev_msm(nat, torch, dev, pts, [s.to_bytes(32, "little") for s in sc], 8 if glv else 6, glv)
    finally:
        nat.set_msm_chunk(64)
    assert got == want
