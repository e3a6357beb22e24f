"""The N > 1 path with the product as the per-rank worker: two processes on the one GPU of the test box, a gloo
process group for the exchange (RCCL needs one GPU per rank; the shard / gather / combine code is the same
lachain_amd/shard.py the bench runs over RCCL, with the partials staged through host tensors here).  Each rank
verifies its ciphertext block of TPKE shares through liblachain_bls.so, runs the Pippenger MSM of its point slice on
the GPU (lcb_g1_msm_dev), all-gathers the 144-byte Jacobian partials and sums them on the GPU (lcb_g1_jac_sum_dev),
and verifies its block of header signatures (lcb_root_header_verify_batch).  Everything is compared with the oracle's
single-rank answers.
"""
import os
import random
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, q):
    import torch
    torch.zeros(1, device="cuda:0")                     # torch's HIP runtime first (tests/conftest.py)
    import torch.distributed as dist
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "oracle"))
    sys.path.insert(0, os.path.dirname(here))
    from test_multirank import _tpke_case, _msm_case
    from lachain_amd import native, shard
    native.load()
    lib = native.lib()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        dev = torch.device("cuda", 0)
        # TPKE shares of this rank's ciphertext block, verified by the product
        yi, cts, shares, ct_idx = _tpke_case()
        lo, hi, sel = shard.tpke_shard(ct_idx, len(cts), rank, WORLD)
        items = [(int(ct_idx[i]), shares[i][0], shares[i][1]) for i in sel]
        bits = native.tpke_verify_shares(yi, cts, items)
        parts = shard.gather_bitmaps(dist, torch.tensor(bits, dtype=torch.uint8), WORLD)
        # MSM slice on the GPU, partials exchanged and summed on the GPU
        pts, sc = _msm_case()
        plo, phi = shard.block_range(len(pts), rank, WORLD)
        n = phi - plo
        st = torch.cuda.current_stream(dev).cuda_stream
        d_in = torch.frombuffer(bytearray(b"".join(pts[plo:phi])), dtype=torch.uint8).to(dev)
        d_sc = torch.frombuffer(bytearray(b"".join(sc[plo:phi])), dtype=torch.uint8).to(dev)
        d_aff = torch.zeros(96 * n, dtype=torch.uint8, device=dev)
        d_ok = torch.zeros(n, dtype=torch.uint8, device=dev)
        d_jac = torch.zeros(144, dtype=torch.uint8, device=dev)
        assert lib.lcb_g1_to_affine_dev(d_aff.data_ptr(), d_ok.data_ptr(), d_in.data_ptr(), n, st) == 0
        assert lib.lcb_g1_msm_dev(d_jac.data_ptr(), d_aff.data_ptr(), d_sc.data_ptr(), n, 0, st) == 0

        def sum_partials(allp, w):
            d_all = allp.to(dev)
            d_out = torch.zeros(48, dtype=torch.uint8, device=dev)
            assert lib.lcb_g1_jac_sum_dev(d_out.data_ptr(), None, d_all.data_ptr(), w, st) == 0
            torch.cuda.synchronize(dev)
            return bytes(d_out.cpu().numpy().tobytes())

        torch.cuda.synchronize(dev)
        total = shard.msm_combine(dist, d_jac.cpu(), WORLD, sum_partials)
        # header signatures: eras block-partitioned over the ranks, each rank checks its own
        import oracle as o
        rng = random.Random(77)
        privs = [rng.randrange(1, o.SECP_N) for _ in range(5)]
        keys = b"".join(o.ecdsa_pubkey(p.to_bytes(32, "big"))[0] for p in privs)
        eras = list(range(10, 16))
        elo, ehi = shard.block_range(len(eras), rank, WORLD)
        acc_all = []
        for era in eras[elo:ehi]:
            recs, sigs, idx = [], [], []
            for v in range(5):
                f = [rng.randbytes(32) for _ in range(3)]
                recs.append(native.header_bytes(era, f[0], f[1], f[2], era * 7 + v))
                h = o.header_keccak(f[0], f[2], f[1], era, era * 7 + v)
                c, rid = o.ecdsa_sign_compact(h, privs[v].to_bytes(32, "big"), rng.randrange(1, o.SECP_N).to_bytes(32, "big"))
                sig = o.ecdsa_encode(c, rid, 225, True)
                if v == era % 5:
                    sig = sig[:40] + bytes([sig[40] ^ 1]) + sig[41:]
                sigs.append(sig)
                idx.append(v)
            acc_all.append(list(native.root_header_verify_batch(b"".join(recs), era, b"".join(sigs), 66, keys, 33, idx,
                                                                True, 225)))
        q.put((rank, sel.tolist(), [p.tolist() for p in parts], total, (elo, ehi, acc_all)))
    finally:
        dist.destroy_process_group()


def test_two_rank_product_workers():
    import torch.multiprocessing as mp
    import oracle as o
    from test_multirank import _tpke_case, _msm_case, _verify
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    yi, cts, shares, ct_idx = _tpke_case()
    full = _verify(yi, cts, shares, ct_idx, range(len(shares))).tolist()
    assert sorted(res[0][1] + res[1][1]) == list(range(len(shares)))
    for r in res:
        assert r[2][0] + r[2][1] == full
    pts, sc = _msm_case()
    expect = o.g1_msm(pts, sc)
    assert res[0][3] == expect and res[1][3] == expect
    # every era checked once; exactly the tampered signature of each era rejected
    eras = sorted(sum((list(range(10 + r[4][0], 10 + r[4][1])) for r in res), []))
    assert eras == list(range(10, 16))
    for r in res:
        for k, acc in enumerate(r[4][2]):
            era = 10 + r[4][0] + k
            assert acc == [0 if v == era % 5 else 1 for v in range(5)]
