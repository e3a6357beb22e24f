"""Round 5: the table-walking kernels keep their tables in a workspace the context owns (lanetab.hpp)
instead of 5-23 KB of scratch per lane, on persistent grids, and launches with a large scratch reservation are gated onto
one stream per device (lcb_set_scratch_gate).  Checked against the oracle:

* persistent grids capped to one block (lcb_set_persist_blocks) so every lane walks several items: G1 / G2 scalar
  multiplication batches (generator and variable base, off-subgroup G1 points), the G2 Lagrange lanes and the
  CommonCoin assembly's paired lanes (even k) and single lanes (odd k), with an off-subgroup share in a pair;
* the gate forced on for every launch with scratch (threshold 0): the same results, and the launches were routed;
* two protocol threads, each with its own context and stream, assembling coins concurrently with large grids
  (the reference's threading model, src/Lachain.Consensus/AbstractProtocol.cs:46-47; ThresholdSigner.cs:78-80).
"""
import threading

import numpy as np
import pytest

import oracle as o
from helpers import Drbg, R, gpu_native

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nat():
    return gpu_native()


@pytest.fixture(scope="module")
def tdev():
    import torch
    return torch, torch.device("cuda", 0)


def _up(torch, dev, b):
    b = b if isinstance(b, (bytes, bytearray)) else b.tobytes()
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)


def _off_subgroup_g2(d):
    while True:
        xa = int.from_bytes(d.bytes(48), "little") % o.P
        xb = int.from_bytes(d.bytes(48), "little") % o.P
        enc = bytearray(xa.to_bytes(48, "little") + xb.to_bytes(48, "little"))
        enc[95] |= 0x80 * (d.bytes(1)[0] & 1)
        enc = bytes(enc)
        if o.g2_valid(enc) and not o.g2_in_subgroup(enc):
            return enc


def _off_subgroup_g1(d):
    while True:
        x = int.from_bytes(d.bytes(48), "little") % o.P
        enc = bytearray(x.to_bytes(48, "little"))
        enc[47] |= 0x80 * (d.bytes(1)[0] & 1)
        enc = bytes(enc)
        if o.g1_valid(enc) and enc != bytes(48) and not o.g1_in_subgroup(enc):
            return enc


@pytest.fixture
def one_block(nat):
    nat.set_persist_blocks(1)
    yield
    nat.set_persist_blocks(0)


def test_scalar_batches_walk_items(nat, one_block):
    d = Drbg(b"gpu-persist-mul")
    n = 700                                           # 256 lanes: up to three items per lane
    ks = [d.fr() for _ in range(n)]
    ks[0], ks[1] = o.fr(0), o.fr(1)
    g1s = nat.mul_batch(1, None, ks, generator=True)
    for i in list(range(0, n, 37)) + [n - 1]:
        assert g1s[i] == o.g1_mul(o.g1_gen(), ks[i]), i
    pts = list(g1s[:n])
    pts[5] = _off_subgroup_g1(d)                      # the window ladder is exact off the subgroup
    pts[300] = bytes(48)                              # infinity
    ks2 = [d.fr() for _ in range(n)]
    out = nat.mul_batch(1, pts, ks2)
    for i in [5, 300] + list(range(0, n, 41)) + [n - 1]:
        assert out[i] == o.g1_mul(pts[i], ks2[i]), i
    m = 300
    g2s = nat.mul_batch(2, None, ks[:m], generator=True)
    for i in list(range(0, m, 29)) + [m - 1]:
        assert g2s[i] == o.g2_mul(o.g2_gen(), ks[i]), i
    q = list(g2s)
    q[7] = _off_subgroup_g2(d)
    out2 = nat.mul_batch(2, q, ks2[:m])
    for i in [7] + list(range(0, m, 31)) + [m - 1]:
        assert out2[i] == o.g2_mul(q[i], ks2[i]), i


def test_g2_lagrange_lanes_walk_items(nat, one_block):
    d = Drbg(b"gpu-persist-lag")
    pool = nat.mul_batch(2, None, [d.fr() for _ in range(16)], generator=True)
    probs = []
    for j in range(120):                              # 120 x 3 = 360 entries on 256 lanes
        k = 3
        xs = [o.fr(1 + (7 * j + t) % 90 + 100 * t) for t in range(k)]
        ys = [pool[(j + 5 * t) % 16] for t in range(k)]
        probs.append((xs, ys))
    probs[3] = (probs[3][0], [_off_subgroup_g2(d)] + probs[3][1][1:])
    got = nat.lagrange_batch(2, probs)
    for j in list(range(0, 120, 11)) + [3, 119]:
        assert got[j] == o.g2_lagrange(*probs[j]), j


def _coin_inputs(torch, dev, nat, d, rounds, per_round, tile=1):
    """rounds x per_round signature shares (G2 points from a small pool, one off-subgroup share in round 2) with
    validator indices 1..per_round; accept all; expected coins by the oracle for the first `rounds` rounds, repeated
    `tile` times"""
    pool = nat.mul_batch(2, None, [d.fr() for _ in range(24)], generator=True)
    sigs = [[pool[(7 * r + 3 * i) % 24] for i in range(per_round)] for r in range(rounds)]
    sigs[2][1] = _off_subgroup_g2(d)
    flat = b"".join(s for row in sigs for s in row) * tile
    return sigs, _up(torch, dev, flat)


def _expected(sigs, k):
    xs = [o.fr(i + 1) for i in range(k)]
    return [o.g2_lagrange(xs, row[:k]) for row in sigs]


@pytest.mark.parametrize("k", [3, 4])
def test_assembly_lanes_walk_items(nat, tdev, one_block, k):
    torch, dev = tdev
    d = Drbg(b"gpu-persist-coin-%d" % k)
    rounds, per = 300, 7                               # k = 4: 600 pairs on 256 lanes; k = 3: 900 single entries
    sigs, d_sigs = _coin_inputs(torch, dev, nat, d, rounds, per)
    expect = _expected(sigs, k)
    lib = nat.lib()
    sh = torch.cuda.current_stream(dev).cuda_stream
    d_acc = torch.ones(rounds * per, dtype=torch.uint8, device=dev)
    d_comb = torch.zeros(96 * rounds, dtype=torch.uint8, device=dev)
    d_cst = torch.zeros(rounds, dtype=torch.uint8, device=dev)
    assert lib.lcb_ts_assemble_dev(d_comb.data_ptr(), d_cst.data_ptr(), d_acc.data_ptr(), d_sigs.data_ptr(), per, k,
                                   rounds, sh) == 0, nat.last_error()
    torch.cuda.synchronize(dev)
    comb = d_comb.cpu().numpy().tobytes()
    assert d_cst.cpu().numpy().tolist() == [1] * rounds
    for r in range(rounds):
        assert comb[96 * r:96 * r + 96] == expect[r], r


def test_gate_forced_on_gives_identical_results(nat, tdev):
    torch, dev = tdev
    d = Drbg(b"gpu-gate")
    rounds, per, k = 64, 7, 4
    sigs, d_sigs = _coin_inputs(torch, dev, nat, d, rounds, per)
    expect = _expected(sigs, k)
    lib = nat.lib()
    sh = torch.cuda.current_stream(dev).cuda_stream
    routed0, seen0 = nat.scratch_gate_stats()
    nat.set_scratch_gate(0)
    try:
        d_acc = torch.ones(rounds * per, dtype=torch.uint8, device=dev)
        d_comb = torch.zeros(96 * rounds, dtype=torch.uint8, device=dev)
        d_cst = torch.zeros(rounds, dtype=torch.uint8, device=dev)
        assert lib.lcb_ts_assemble_dev(d_comb.data_ptr(), d_cst.data_ptr(), d_acc.data_ptr(), d_sigs.data_ptr(), per,
                                       k, rounds, sh) == 0, nat.last_error()
        # a TPKE batch through both verification paths while every launch with scratch crosses to the gate stream
        n, f = 4, 1
        coeffs = [o.fr(17), o.fr(23)]
        x = [o.fr_eval_poly(coeffs, o.fr(i + 1)) for i in range(n)]
        y = o.g1_mul(o.g1_gen(), o.fr_eval_poly(coeffs, o.fr(0)))
        yi = [o.g1_mul(o.g1_gen(), xi) for xi in x]
        U, V, W = o.tpke_encrypt(y, b"gate test payload", o.fr(5))
        shares = [(0, i, o.tpke_decrypt(U, V, W, x[i])) for i in range(n)]
        shares.append((0, 1, o.g1_add(shares[1][2], o.g1_gen())))
        want = [True] * n + [False]
        assert nat.tpke_verify_shares(yi, [(U, V, W)], shares) == want
        assert nat.tpke_verify_shares(yi, [(U, V, W)], shares, batched=True) == want
        torch.cuda.synchronize(dev)
    finally:
        nat.set_scratch_gate(-3)                     # back to the model's per-queue share
    routed1, seen1 = nat.scratch_gate_stats()
    assert routed1 > routed0 and seen1 > seen0
    comb = d_comb.cpu().numpy().tobytes()
    for r in range(rounds):
        assert comb[96 * r:96 * r + 96] == expect[r], r


def test_concurrent_assemblies_two_threads(nat, tdev):
    """two protocol threads, each with its own context and stream, assembling 16,384 coins at once (paired lanes at
    full occupancy), three times each: no queue abort, every coin equal to the oracle's"""
    torch, dev = tdev
    d = Drbg(b"gpu-gate-threads")
    base, tile, per, k = 64, 256, 7, 4
    rounds = base * tile
    sigs, d_sigs = _coin_inputs(torch, dev, nat, d, base, per, tile)
    expect = b"".join(_expected(sigs, k))
    lib = nat.lib()
    errs, outs = [], {}

    def worker(t):
        try:
            ctx = nat.Context()
            st = torch.cuda.Stream(dev)
            with torch.cuda.stream(st):     # the fills are ordered before the library's kernels on st
                d_acc = torch.ones(rounds * per, dtype=torch.uint8, device=dev)
                d_comb = torch.zeros(96 * rounds, dtype=torch.uint8, device=dev)
                d_cst = torch.zeros(rounds, dtype=torch.uint8, device=dev)
            for _ in range(3):
                rc = lib.lcb_ctx_ts_assemble_dev(ctx.ptr, d_comb.data_ptr(), d_cst.data_ptr(), d_acc.data_ptr(),
                                                 d_sigs.data_ptr(), per, k, rounds, st.cuda_stream)
                if rc != 0:
                    raise RuntimeError(nat.last_error())
                st.synchronize()
                outs.setdefault(t, []).append((d_comb.cpu().numpy().tobytes(), d_cst.cpu().numpy().copy()))
            ctx.close()
        except Exception as e:          # noqa: BLE001 — reported below
            errs.append(repr(e))

    torch.cuda.synchronize(dev)             # the shared inputs, written on the default stream
    ths = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errs, errs
    import numpy as np
    want = np.frombuffer(expect * tile, dtype=np.uint8).reshape(rounds, 96)
    for t in range(2):
        assert len(outs[t]) == 3
        for rep, (comb, cst) in enumerate(outs[t]):
            bad_st = np.nonzero(cst != 1)[0]
            got = np.frombuffer(comb, dtype=np.uint8).reshape(rounds, 96)
            bad_sig = np.nonzero((got != want).any(axis=1))[0]
            # (counts and first indices only: a list diff of 16,384 statuses outlives the test's time limit)
            assert bad_st.size == 0 and bad_sig.size == 0, (t, rep, bad_st.size, bad_st[:16].tolist(),
                                                           bad_sig.size, bad_sig[:16].tolist())


def test_scratch_model_bounds_the_bound_reservations(nat, tdev):
    """round 6: the runtime binds a kernel's full-device scratch to its hardware queue; the gate's
    per-queue share T keeps Q x T + the gate queue's 4.5 GiB within the pool, a batched TPKE verify at the default share
    routes nothing (its largest kernel binds 2.5 GB), and a GT power (k_op_gt, 8,148 B per lane: 4.27 GB full-device)
    is routed"""
    import lachain_amd.mcl as mcl
    torch, dev = tdev
    info = nat.scratch_info()
    assert info["slots"] >= 64 and info["queues"] >= 2 and info["threshold"] == info["per_queue"]
    if info["pool"]:
        assert info["queues"] * info["per_queue"] + (9 << 29) <= info["pool"]
    full = lambda per_lane: ((per_lane + 15) // 16 * 16) * 64 * info["slots"]
    if info["per_queue"] < full(5000):
        pytest.skip("the environment's queue count makes the preparation kernels gated too")
    n, f = 4, 1
    coeffs = [o.fr(3), o.fr(9)]
    x = [o.fr_eval_poly(coeffs, o.fr(i + 1)) for i in range(n)]
    y = o.g1_mul(o.g1_gen(), o.fr_eval_poly(coeffs, o.fr(0)))
    yi = [o.g1_mul(o.g1_gen(), xi) for xi in x]
    U, V, W = o.tpke_encrypt(y, b"model test", o.fr(11))
    shares = [(0, i, o.tpke_decrypt(U, V, W, x[i])) for i in range(n)]
    r0, s0 = nat.scratch_gate_stats()
    assert nat.tpke_verify_shares(yi, [(U, V, W)], shares, batched=True) == [True] * n
    r1, s1 = nat.scratch_gate_stats()
    assert s1 > s0 and r1 == r0
    g = mcl.GT.Pairing(mcl.G1.Generator(), mcl.G2.Generator())
    r1, _ = nat.scratch_gate_stats()
    h = mcl.GT.Pow(g, mcl.Fr.FromInt(2))             # k_op_gt on the device
    r2, _ = nat.scratch_gate_stats()
    assert r2 > r1
    assert h == g * g                                # (the product runs on the host)
