"""GPU parity of the batched share checks under the reference's Byzantine patterns, where a faulty validator corrupts
its share in EVERY ciphertext / coin (HoneyBadgerMalicious.cs:17-23 reverses the bytes of each decryption share it
sends, HoneyBadgerTest.cs:75-94 makes validator 0 that node; HoneyBadgerSmartMalicious.cs:28-48 sends valid points that
are not the share).  With F such validators every group of a ciphertext carries F bad shares, every group check fails,
and the census (k_batch.hip "suspect keys": exact single checks of a prefix of the batch) must route the faulty keys'
shares to single checks.  Every decision is compared with the oracle's per-share check (TPKE/PublicKey.cs:88-92,
ThresholdSignature/PublicKey.cs:16-21) and with the product's exact path; the census statistics are checked where the
pattern determines them (wrong valid points: every sampled share of a faulty key fails)."""
import numpy as np
import pytest

import oracle as o
from test_gpu_batched import Batch, off_subgroup_g1, run_dev
from test_gpu_batched_ts import Rounds

pytestmark = pytest.mark.gpu

N, F, C = 22, 7, 48                     # configs[1]'s validator set; 48 ciphertexts = 1,056 shares


@pytest.fixture(scope="module")
def nat():
    from helpers import gpu_native
    return gpu_native()


@pytest.fixture(scope="module")
def tdev():
    import torch
    return torch, torch.device("cuda", 0)


@pytest.fixture(scope="module")
def batch():
    return Batch(b"gpu-byzantine-tpke", N, F, C)


@pytest.fixture
def census_on(nat):
    nat.set_batch_census(1)             # small test batches get the census (default: >= 16,384 shares)
    yield
    nat.set_batch_census(16384)


TPKE_PATTERNS = {                       # faulty decryptors, what they send
    "one_reversed": ([0], "reversed"),
    "f_reversed": (list(range(F)), "reversed"),
    "one_wrong": ([0], "wrong"),
    "f_wrong": (list(range(F)), "wrong"),
    "f_off_subgroup": ([3, 5, 8, 11, 13, 17, 21], "off"),
    "all_wrong": (list(range(N)), "wrong"),
}


def tpke_pattern(b, pattern):
    faulty, kind = TPKE_PATTERNS[pattern]
    shares, expect = [], []
    for c in range(C):
        for j in range(N):
            s = b.good[c][j]
            if j in faulty:
                s = {"reversed": s[::-1], "wrong": b.bad[c][j], "off": None}[kind]
                if s is None:
                    s = off_subgroup_g1(b.d)
            shares.append(s)
            expect.append(1 if j not in faulty else int(b.expect(c, j, s)))
    return faulty, kind, shares, np.array(expect, dtype=np.uint8)


@pytest.mark.parametrize("pattern", list(TPKE_PATTERNS))
def test_tpke_byzantine_validators(nat, tdev, batch, census_on, pattern):
    faulty, kind, shares, expect = tpke_pattern(batch, pattern)
    assert expect[[c * N + j for c in range(C) for j in faulty]].sum() == 0     # every faulty share is rejected
    ct = np.repeat(np.arange(C, dtype=np.uint32), N)
    dec = np.tile(np.arange(N, dtype=np.uint32), C)
    exact = nat.tpke_verify_shares(batch.yi, batch.cts, [(int(c), int(j), s) for c, j, s in zip(ct, dec, shares)])
    assert np.array_equal(np.array(exact, dtype=np.uint8), expect)
    for fused in (False, True):
        got = run_dev(nat, tdev, batch, ct, dec, shares, fused=fused)
        assert np.array_equal(got, expect), (pattern, fused)
        m, n_susp, groups, entries = nat.batched_census()
        assert m == C * N // 4
        if kind in ("wrong", "off"):    # every decodable share of a faulty key fails its check
            assert n_susp == len(faulty)
            # each remaining ciphertext: its group (unless every key is faulty) + one single per faulty key
            n_ct = groups
            assert entries == n_ct * len(faulty) + (n_ct if len(faulty) < N else 0)


def test_tpke_byzantine_census_off_below_threshold(nat, tdev, batch):
    """below the census threshold the F-validator pattern is still decided exactly (by group splitting)"""
    _, _, shares, expect = tpke_pattern(batch, "f_wrong")
    ct = np.repeat(np.arange(C, dtype=np.uint32), N)
    dec = np.tile(np.arange(N, dtype=np.uint32), C)
    got = run_dev(nat, tdev, batch, ct, dec, shares, fused=True)
    assert np.array_equal(got, expect)
    assert nat.batched_census()[0] == 0


@pytest.fixture(scope="module")
def rounds():
    return Rounds(b"gpu-byzantine-ts", 100, 12)


@pytest.mark.parametrize("n_bad", [1, 33])
def test_ts_byzantine_signers(nat, rounds, census_on, n_bad):
    """CommonCoin rounds of N=100 (configs[2]) where 1 or F=33 signers send a wrong share in every round"""
    r = rounds
    faulty = set(range(0, 3 * n_bad, 3))
    items, expect = [], []
    for m in range(r.m):
        for i in range(r.n):
            sig = r.bad[m][i] if i in faulty else r.good[m][i]
            items.append((m, i, sig))
            expect.append(i not in faulty)
    exact = nat.ts_verify_shares(r.pks, r.msgs, items)
    assert exact == expect
    got = nat.ts_verify_shares(r.pks, r.msgs, items, batched=True)
    assert got == expect
    m, n_susp, groups, entries = nat.batched_census()
    assert m == r.m * r.n // 4 and n_susp == n_bad
    assert entries == groups * (n_bad + 1)
