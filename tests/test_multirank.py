"""The N > 1 path on CPU: world_size-2 gloo process groups running the same shard/gather code the bench runs
over RCCL (lachain_amd/shard.py), with the oracle standing in for the per-rank GPU work (it is the checker
here, not the product).  Checks: ciphertext-block partition covers every share exactly once and keeps the
shares of one ciphertext together; per-rank bitmaps gathered in rank order equal the single-rank bitmap; the
MSM exchange (per-rank partials, all-gather, sum) equals the single-rank MSM.
"""
import os
import socket

import numpy as np
import pytest

from helpers import Drbg, R

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tpke_case():
    import oracle as o
    n, f = 4, 1
    d = Drbg(b"multirank-tpke")
    coeffs = [d.fr_int() for _ in range(f + 1)]
    poly = lambda x: sum(c * pow(x, i, R) for i, c in enumerate(coeffs)) % R
    xs = [poly(i + 1) for i in range(n)]
    y = o.g1_mul(o.g1_gen(), o.fr(poly(0)))
    yi = [o.g1_mul(o.g1_gen(), o.fr(x)) for x in xs]
    cts = [o.tpke_encrypt(y, b"payload %d" % c, o.fr(d.fr_int())) for c in range(3)]
    shares, ct_idx = [], []
    for c, (U, V, W) in enumerate(cts):
        for j in range(n):
            ui = o.tpke_decrypt(U, V, W, o.fr(xs[j]))
            if (c, j) in ((0, 1), (2, 3)):
                ui = o.g1_add(ui, o.g1_gen())          # corrupted share (rejected)
            shares.append((j, ui))
            ct_idx.append(c)
    return yi, cts, shares, np.array(ct_idx, dtype=np.uint32)


def _verify(yi, cts, shares, ct_idx, sel):
    import oracle as o
    out = []
    for i in sel:
        j, ui = shares[i]
        U, V, W = cts[ct_idx[i]]
        out.append(1 if o.tpke_verify_share(yi[j], U, V, W, ui) == 1 else 0)
    return np.array(out, dtype=np.uint8)


def _msm_case():
    import oracle as o
    d = Drbg(b"multirank-msm")
    n = 21
    pts = [o.g1_mul(o.g1_gen(), o.fr(d.fr_int())) for _ in range(n)]
    sc = [o.fr(d.fr_int()) for _ in range(n)]
    return pts, sc


def _worker(rank, port, q):
    import torch
    import torch.distributed as dist
    import oracle as o
    from lachain_amd import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        yi, cts, shares, ct_idx = _tpke_case()
        lo, hi, sel = shard.tpke_shard(ct_idx, len(cts), rank, WORLD)
        bits = torch.from_numpy(_verify(yi, cts, shares, ct_idx, sel))
        parts = shard.gather_bitmaps(dist, bits, WORLD)
        pts, sc = _msm_case()
        plo, phi = shard.block_range(len(pts), rank, WORLD)
        local = torch.frombuffer(bytearray(o.g1_msm(pts[plo:phi], sc[plo:phi])), dtype=torch.uint8)

        def sum_partials(allp, w):
            acc = bytes(48)
            raw = allp.numpy().tobytes()
            for k in range(w):
                acc = o.g1_add(acc, raw[48 * k:48 * k + 48])
            return acc

        total = shard.msm_combine(dist, local, WORLD, sum_partials)
        # the bench's timing reduction (bench.py: every timed section): max of the elapsed times, sum of the counts
        mt = shard.max_time_sum(dist, torch, "cpu", 1.5 + rank, rank, 10)
        q.put((rank, lo, hi, sel.tolist(), [p.tolist() for p in parts], total, mt))
    finally:
        dist.destroy_process_group()


def test_block_range_partitions():
    from lachain_amd import shard
    for n in (0, 1, 7, 47663, 1 << 20):
        for w in (1, 2, 3, 8):
            rs = [shard.block_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[k][1] == rs[k + 1][0] for k in range(w - 1))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def test_two_rank_gloo_shard_and_gather():
    import torch.multiprocessing as mp
    import oracle as o
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    yi, cts, shares, ct_idx = _tpke_case()
    full = _verify(yi, cts, shares, ct_idx, range(len(shares))).tolist()
    # every share exactly once, ciphertexts not split across ranks
    sels = [r[3] for r in res]
    assert sorted(sels[0] + sels[1]) == list(range(len(shares)))
    assert not set(ct_idx[sels[0]]) & set(ct_idx[sels[1]])
    # gathered bitmaps (identical on both ranks) in rank order == single-rank bitmap
    for r in res:
        assert r[4][0] + r[4][1] == full
    assert full.count(0) == 2
    pts, sc = _msm_case()
    expect = o.g1_msm(pts, sc)
    assert res[0][5] == expect and res[1][5] == expect
    assert res[0][6] == res[1][6] == [2.5, 1.0, 20.0]
