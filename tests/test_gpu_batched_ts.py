"""GPU parity of the randomized batch verification of threshold-signature shares (lcb_ts_verify_shares_batched[_dev],
lcb_ts_verify_prepared_batched_dev; k_batch.hip) against the oracle's per-share ValidateSignature
(ThresholdSignature/PublicKey.cs:16-21), and of the level-2 search (one bad share per group found from gamma' =
gamma^c) for both TPKE and threshold signatures.

Covered: the committed N=7 / N=100 transcripts (wrong-signer, reversed, off-subgroup, infinity shares; both line-set
modes), signature shares outside G2 (a cofactor-torsion component, which the reference's check may accept, and a
random off-subgroup point) that must get their exact decision, corruption densities 0 %, 1 %, 30 % and 100 %, the
bench's one-bad-share-per-round pattern (resolved in two levels, no single checks) and two bad shares per group (the
search fails, single checks follow)."""
import json
import os

import numpy as np
import pytest

import oracle as o
from helpers import Drbg, R, gpu_native

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
T = json.load(open(os.path.join(HERE, "golden", "transcripts.json")))
H = bytes.fromhex


@pytest.fixture(scope="module")
def nat():
    return gpu_native()


@pytest.fixture(scope="module")
def tdev():
    import torch
    return torch, torch.device("cuda", 0)


@pytest.fixture(params=["normalised", "on_the_fly"])
def line_mode(nat, request):
    nat.set_line_mode(request.param == "on_the_fly")
    yield request.param
    nat.set_line_mode(False)


def up(torch, dev, b):
    if isinstance(b, np.ndarray):
        b = b.tobytes()
    return torch.frombuffer(bytearray(b if len(b) else b"\0"), dtype=torch.uint8).to(dev)


def off_subgroup_g2(d):
    while True:
        xa = int.from_bytes(d.bytes(48), "little") % o.P
        xb = int.from_bytes(d.bytes(48), "little") % o.P
        enc = bytearray(xa.to_bytes(48, "little") + xb.to_bytes(48, "little"))
        enc[95] |= 0x80 * (d.bytes(1)[0] & 1)
        enc = bytes(enc)
        if o.g2_valid(enc) and not o.g2_in_subgroup(enc):
            return enc


class Rounds:
    """n signers (keys sk_i), m messages; good[r][i] = sk_i H(m_r), bad[r][i] = signer i+1's share (valid point, wrong
    key)"""

    def __init__(self, seed, n, m):
        d = Drbg(seed)
        self.d = d
        self.sks = [d.fr_int() for _ in range(n)]
        self.pks = [o.g1_mul(o.g1_gen(), o.fr(x)) for x in self.sks]
        self.msgs = [d.bytes(24) for _ in range(m)]
        self.good = [[o.ts_sign(o.fr(x), msg) for x in self.sks] for msg in self.msgs]
        self.bad = [[row[(i + 1) % n] for i in range(n)] for row in self.good]
        self.n, self.m = n, m

    def expect(self, r, i, sig):
        return o.g2_valid(sig) and o.ts_validate(self.pks[i], sig, self.msgs[r]) == 1


@pytest.mark.parametrize("key", ["ts_n7", "ts_n100"])
def test_ts_batched_transcript(nat, key, line_mode):
    t = T[key]
    msgs = [H(r["msg"]) for r in t["rounds"]]
    items = [(ri, i, H(s)) for ri, r in enumerate(t["rounds"]) for i, s in enumerate(r["sigs"])]
    got = nat.ts_verify_shares([H(p) for p in t["pk_i"]], msgs, items, batched=True)
    assert got == [a for r in t["rounds"] for a in r["accept"]]


def test_ts_batched_outside_g2(nat):
    """signature shares with a G2 cofactor-torsion component or off the subgroup altogether get their exact decisions
    (equal to the oracle's and to the exact GPU path); the rest of their rounds are decided by the group check"""
    b = Rounds(b"gpu-ts-batched-g2", 9, 3)
    d = b.d
    q = off_subgroup_g2(d)
    t2 = o.g2_add(o.g2_mul(q, o.fr(R - 1)), q)
    items = []
    for r in range(3):
        for i in range(9):
            items.append([r, i, b.good[r][i]])
    items[4][2] = o.g2_add(b.good[0][4], t2)         # torsion component
    items[9 + 2][2] = off_subgroup_g2(d)             # off the subgroup
    items[9 + 6][2] = b.bad[1][6]
    items[18 + 8][2] = o.g2_add(b.bad[2][8], t2)
    expect = [b.expect(r, i, s) for r, i, s in items]
    exact = nat.ts_verify_shares(b.pks, b.msgs, [tuple(x) for x in items])
    assert exact == expect
    assert nat.ts_verify_shares(b.pks, b.msgs, [tuple(x) for x in items], batched=True) == expect


def run_dev(nat, tdev, b, midx, pidx, sigs, fused):
    torch, dev = tdev
    lib = nat.lib()
    sh = torch.cuda.current_stream(dev).cuda_stream
    n = len(sigs)
    d_pk = up(torch, dev, b"".join(b.pks))
    d_m = up(torch, dev, b"".join(b.msgs))
    d_mo = up(torch, dev, np.arange(0, 24 * (b.m + 1), 24, dtype=np.uint32))
    d_mi = up(torch, dev, np.asarray(midx, dtype=np.uint32))
    d_pi = up(torch, dev, np.asarray(pidx, dtype=np.uint32))
    d_s = up(torch, dev, b"".join(sigs))
    d_acc = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    if fused:
        rc = lib.lcb_ts_verify_shares_batched_dev(d_acc.data_ptr(), n, d_pk.data_ptr(), b.n, d_s.data_ptr(),
                                                  d_m.data_ptr(), d_mo.data_ptr(), b.m, d_mi.data_ptr(),
                                                  d_pi.data_ptr(), sh)
    else:
        assert lib.lcb_ts_prepare_dev(d_pk.data_ptr(), b.n, d_m.data_ptr(), d_mo.data_ptr(), b.m, sh) == 0
        rc = lib.lcb_ts_verify_prepared_batched_dev(d_acc.data_ptr(), n, b.n, b.m, d_s.data_ptr(), d_mi.data_ptr(),
                                                    d_pi.data_ptr(), sh)
    assert rc == 0, nat.last_error()
    torch.cuda.synchronize(dev)
    return d_acc.cpu().numpy()


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("density", [0.0, 0.01, 0.3, 1.0])
def test_ts_batched_density(nat, tdev, density, fused):
    """20 signers, 6 messages tiled to 3,840 shares (192 rounds of 20, message-major); each share independently
    replaced by a wrong one with the given probability"""
    b = Rounds(b"gpu-ts-batched-density", 20, 6)
    rng = np.random.default_rng(int(density * 1000) + 17)
    reps = 32
    n = 6 * 20 * reps
    bad = rng.random(n) < density
    midx = np.tile(np.repeat(np.arange(6, dtype=np.uint32), 20), reps)
    pidx = np.tile(np.arange(20, dtype=np.uint32), 6 * reps)
    sigs = [(b.bad if bad[i] else b.good)[midx[i]][pidx[i]] for i in range(n)]
    got = run_dev(nat, tdev, b, midx, pidx, sigs, fused)
    assert np.array_equal(got, (~bad).astype(np.uint8))
    levels, _ = nat.tpke_batched_stats()
    assert levels[0] == 6 * reps
    if density == 0.0:
        assert len(levels) == 1


def test_ts_one_bad_per_round_two_levels(nat, tdev):
    """the bench's corruption pattern: exactly one wrong share per round, at a different position each round — every
    group fails level 1 and the level-2 search names the bad share (two levels, no single checks)"""
    b = Rounds(b"gpu-ts-one-bad", 30, 4)
    reps = 16
    rounds = 4 * reps
    midx = np.repeat(np.arange(4, dtype=np.uint32), 30)
    midx = np.tile(midx, reps)
    pidx = np.tile(np.arange(30, dtype=np.uint32), rounds)
    sigs, expect = [], []
    for r in range(rounds):
        j = (7 * r) % 30
        for i in range(30):
            sigs.append(b.bad[r % 4][i] if i == j else b.good[r % 4][i])
            expect.append(i != j)
    # consecutive rounds of the same message index would merge into one run: interleave so runs are single rounds
    got = run_dev(nat, tdev, b, midx, pidx, sigs, True)
    assert got.tolist() == [int(e) for e in expect]
    levels, _ = nat.tpke_batched_stats()
    assert levels == [rounds, rounds]


@pytest.mark.parametrize("kind", ["ts", "tpke"])
def test_two_bad_per_group_search_fails(nat, tdev, kind):
    """two wrong shares in a group: gamma' is no power gamma^c (c <= len), so for TS the group's shares get single checks
    (three levels) and for TPKE the two-error location names them (two levels); one wrong share: found by the one-error
    search"""
    if kind == "ts":
        b = Rounds(b"gpu-ts-two-bad", 12, 2)
        items = [[r, i, b.good[r][i]] for r in range(2) for i in range(12)]
        items[3][2] = b.bad[0][3]
        items[7][2] = b.bad[0][7]
        items[12 + 5][2] = b.bad[1][5]
        got = nat.ts_verify_shares(b.pks, b.msgs, [tuple(x) for x in items], batched=True)
        expect = [b.expect(r, i, s) for r, i, s in items]
    else:
        from test_gpu_batched import Batch
        b = Batch(b"gpu-tpke-two-bad", 12, 3, 2)
        items = [[c, j, b.good[c][j]] for c in range(2) for j in range(12)]
        items[3][2] = b.bad[0][3]
        items[7][2] = b.bad[0][7]
        items[12 + 5][2] = b.bad[1][5]
        got = nat.tpke_verify_shares(b.yi, b.cts, [tuple(x) for x in items], batched=True)
        expect = [b.expect(c, j, s) for c, j, s in items]
    assert got == expect and expect.count(False) == 3
    levels, _ = nat.tpke_batched_stats()
    # TS: the one-error search fails on the two-bad group, whose shares get single checks; TPKE: level 2 re-checks each
    # failed group with weights c (the one-error search names the single bad share), the open group with weights t, and
    # the two-error location names both bad shares
    assert levels == ([2, 2, 12] if kind == "ts" else [2, 2, 1])


@pytest.mark.parametrize("k", [3, 4])
def test_ts_assembly_reuses_decoded_shares(nat, tdev, k):
    """the assembly after a batched CommonCoin check takes each selected share's decoded point and G2 flag from the
    check's records (ts_share_st) when the record holds the same 96 bytes, and decodes the share itself otherwise:
    AddShare's Lagrange combination (ThresholdSigner.cs:62-75) equals the oracle's for a share with a G2
    cofactor-torsion component (ladder, not GLS), for shares the check decoded, and for an input whose bytes differ
    from the checked share"""
    torch, dev = tdev
    n, rounds = 7, 4                                        # k = 4: two entries per lane (k_g2_mul2_lanes)
    b = Rounds(b"gpu-ts-assembly-records", n, rounds)
    q = off_subgroup_g2(b.d)
    t2 = o.g2_add(o.g2_mul(q, o.fr(R - 1)), q)
    sigs = [list(row) for row in b.good]
    sigs[0][0] = o.g2_add(sigs[0][0], t2)                  # torsion component
    sigs[2][1] = b.bad[2][1]
    items = [(r, i, sigs[r][i]) for r in range(rounds) for i in range(n)]
    acc = nat.ts_verify_shares(b.pks, b.msgs, items, batched=True)
    assert acc == [b.expect(r, i, s) for r, i, s in items]
    assert not acc[0]                                       # the torsion share fails the check ...
    flat = [s for row in sigs for s in row]
    changed = list(flat)
    changed[7 + 1] = o.g2_add(b.good[1][1], b.good[1][1])   # bytes the check never saw (accept bit kept)
    forced = list(acc)
    forced[0] = True                                        # ... a caller may still hand it to the assembly
    for v, a in ((flat, acc), (changed, acc), (flat, forced)):
        d_acc = up(torch, dev, bytes(int(x) for x in a))
        d_sig = up(torch, dev, b"".join(v))
        d_out = torch.zeros(96 * rounds, dtype=torch.uint8, device=dev)
        d_st = torch.zeros(rounds, dtype=torch.uint8, device=dev)
        sh = torch.cuda.current_stream(dev).cuda_stream
        assert nat.lib().lcb_ts_assemble_dev(d_out.data_ptr(), d_st.data_ptr(), d_acc.data_ptr(), d_sig.data_ptr(),
                                             n, k, rounds, sh) == 0
        torch.cuda.synchronize(dev)
        out = d_out.cpu().numpy().tobytes()
        assert d_st.cpu().numpy().tolist() == [1] * rounds
        for r in range(rounds):
            valid = [i for i in range(n) if a[r * n + i]][:k]
            want = o.g2_lagrange([o.fr(i + 1) for i in valid], [v[r * n + i] for i in valid])
            assert out[96 * r:96 * r + 96] == want, (r, valid)
