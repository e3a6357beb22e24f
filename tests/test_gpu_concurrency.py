"""Re-entrancy of the batch boundary under the reference's threading model: many consensus protocol threads call
the crypto library concurrently (src/Lachain.Consensus/AbstractProtocol.cs:46-47, one thread per HoneyBadger /
CommonCoin instance).  TPKE and threshold-signature prepare/verify are interleaved on several streams and threads
— in one thread, in two threads with their implicit contexts, and in two threads sharing one explicit lcb_ctx —
and every accept bitmap must equal the oracle's.  No sleeps: ordering comes from the library alone.
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


def _keys(d, n, f):
    coeffs = [d.fr_int() for _ in range(f + 1)]
    poly = lambda x: sum(c * pow(x, i, R) for i, c in enumerate(coeffs)) % R
    return [poly(i + 1) for i in range(n)], poly(0)


@pytest.fixture(scope="module")
def batches(tdev):
    torch, dev = tdev
    d = Drbg(b"gpu-concurrency")
    up = lambda b: torch.frombuffer(bytearray(b if isinstance(b, (bytes, bytearray)) else b.tobytes()),
                                    dtype=torch.uint8).to(dev)
    # TPKE: N=4 F=1, 5 ciphertexts x 4 shares, two corrupted
    n, f, nc = 4, 1, 5
    xs, ys = _keys(d, n, f)
    yi = [o.g1_mul(o.g1_gen(), o.fr(x)) for x in xs]
    cts = [o.tpke_encrypt(o.g1_mul(o.g1_gen(), o.fr(ys)), d.bytes(32), o.fr(d.fr_int())) for _ in range(nc)]
    shares = [o.g1_mul(cts[c][0], o.fr(xs[j])) for c in range(nc) for j in range(n)]
    shares[3] = o.g1_add(shares[3], o.g1_gen())
    shares[9] = shares[10]
    t_exp = [o.tpke_verify_share(yi[i % n], *cts[i // n], shares[i]) == 1 for i in range(nc * n)]
    tp = dict(n_keys=n, n_cts=nc, n=nc * n, y=up(b"".join(yi)), u=up(b"".join(c[0] for c in cts)),
              w=up(b"".join(c[2] for c in cts)), v=up(b"".join(c[1] for c in cts)),
              voff=up(np.arange(0, 32 * (nc + 1), 32, dtype=np.uint32)),
              ct=up(np.repeat(np.arange(nc, dtype=np.uint32), n)), dec=up(np.tile(np.arange(n, dtype=np.uint32), nc)),
              ui=up(b"".join(shares)), expect=t_exp)
    # TS: N=7 F=2, 3 messages x 7 shares, two corrupted — a different batch shape from the TPKE one
    n2, f2, nm = 7, 2, 3
    sks, _ = _keys(d, n2, f2)
    pks = [o.g1_mul(o.g1_gen(), o.fr(x)) for x in sks]
    msgs = [b"coin %d ........................" % m for m in range(nm)]
    sigs = [o.ts_sign(o.fr(sks[j]), msgs[m]) for m in range(nm) for j in range(n2)]
    sigs[2] = sigs[3]
    sigs[15] = o.g2_add(sigs[15], sigs[15])
    s_exp = [o.ts_validate(pks[i % n2], sigs[i], msgs[i // n2]) == 1 for i in range(nm * n2)]
    ts = dict(n_pks=n2, n_msgs=nm, n=nm * n2, pks=up(b"".join(pks)), msg=up(b"".join(msgs)),
              moff=up(np.cumsum([0] + [len(m) for m in msgs]).astype(np.uint32)),
              sigs=up(b"".join(sigs)), midx=up(np.repeat(np.arange(nm, dtype=np.uint32), n2)),
              pidx=up(np.tile(np.arange(n2, dtype=np.uint32), nm)), expect=s_exp)
    assert not all(t_exp) and not all(s_exp)
    return tp, ts


def _tpke_prepare(lib, tp, s, ctx=None):
    args = (tp["y"].data_ptr(), tp["n_keys"], tp["u"].data_ptr(), tp["w"].data_ptr(), tp["v"].data_ptr(),
            tp["voff"].data_ptr(), tp["n_cts"], s)
    return lib.lcb_ctx_tpke_prepare_dev(ctx, *args) if ctx else lib.lcb_tpke_prepare_dev(*args)


def _tpke_verify(lib, tp, acc, s, ctx=None):
    args = (acc.data_ptr(), tp["n"], tp["n_keys"], tp["n_cts"], tp["ct"].data_ptr(), tp["dec"].data_ptr(),
            tp["ui"].data_ptr(), s)
    return lib.lcb_ctx_tpke_verify_prepared_dev(ctx, *args) if ctx else lib.lcb_tpke_verify_prepared_dev(*args)


def _ts_prepare(lib, ts, s, ctx=None):
    args = (ts["pks"].data_ptr(), ts["n_pks"], ts["msg"].data_ptr(), ts["moff"].data_ptr(), ts["n_msgs"], s)
    return lib.lcb_ctx_ts_prepare_dev(ctx, *args) if ctx else lib.lcb_ts_prepare_dev(*args)


def _ts_verify(lib, ts, acc, s, ctx=None):
    args = (acc.data_ptr(), ts["n"], ts["n_pks"], ts["n_msgs"], ts["sigs"].data_ptr(), ts["midx"].data_ptr(),
            ts["pidx"].data_ptr(), s)
    return lib.lcb_ctx_ts_verify_prepared_dev(ctx, *args) if ctx else lib.lcb_ts_verify_prepared_dev(*args)


def _bits(acc):
    return [bool(x) for x in acc.cpu().numpy()]


def test_interleaved_in_one_thread(nat, tdev, batches):
    """prepare TPKE, prepare TS, then verify both: each verify must see its own workspace (round-1 defect)."""
    torch, dev = tdev
    tp, ts = batches
    lib = nat.lib()
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    a1 = torch.zeros(tp["n"], dtype=torch.uint8, device=dev)
    a2 = torch.zeros(ts["n"], dtype=torch.uint8, device=dev)
    for _ in range(3):
        a1.zero_(); a2.zero_()
        torch.cuda.synchronize(dev)
        assert _tpke_prepare(lib, tp, s1.cuda_stream) == 0
        assert _ts_prepare(lib, ts, s2.cuda_stream) == 0
        assert _tpke_verify(lib, tp, a1, s1.cuda_stream) == 0, nat.last_error()
        assert _ts_verify(lib, ts, a2, s2.cuda_stream) == 0, nat.last_error()
        torch.cuda.synchronize(dev)
        assert _bits(a1) == tp["expect"]
        assert _bits(a2) == ts["expect"]


def test_shape_mismatch_and_unprepared_fail(nat, tdev, batches):
    torch, dev = tdev
    tp, ts = batches
    lib = nat.lib()
    s = torch.cuda.current_stream(dev).cuda_stream
    a = torch.zeros(tp["n"], dtype=torch.uint8, device=dev)
    with nat.Context() as ctx:
        assert _tpke_verify(lib, tp, a, s, ctx.ptr) == -1            # nothing prepared in this context
        assert "no TPKE batch prepared" in nat.last_error()
        assert _tpke_prepare(lib, tp, s, ctx.ptr) == 0
        bad = dict(tp, n_cts=tp["n_cts"] - 1)
        assert _tpke_verify(lib, bad, a, s, ctx.ptr) == -1            # shape differs from the prepared one
        assert _ts_verify(lib, ts, torch.zeros(ts["n"], dtype=torch.uint8, device=dev), s, ctx.ptr) == -1
        assert _tpke_verify(lib, tp, a, s, ctx.ptr) == 0
        ctx.synchronize()
        assert _bits(a) == tp["expect"]


def _worker(lib, torch, dev, fn_pairs, iters, errors):
    try:
        st = torch.cuda.Stream(dev)
        for it in range(iters):
            for prep, ver, b, n in fn_pairs:
                with torch.cuda.stream(st):   # the output's zero fill is ordered before the library's kernels
                    acc = torch.zeros(n, dtype=torch.uint8, device=dev)
                if prep(st.cuda_stream) != 0 or ver(acc, st.cuda_stream) != 0:
                    errors.append("call failed: " + lib.lcb_last_error().decode())
                    return
                st.synchronize()
                if _bits(acc) != b:
                    errors.append(f"iteration {it}: bitmap differs from the oracle")
                    return
    except Exception as e:  # noqa: BLE001 — surfaced through the errors list
        errors.append(repr(e))


def test_two_threads_implicit_contexts(nat, tdev, batches):
    """two protocol threads, each alternating TPKE and TS batches on its own stream"""
    torch, dev = tdev
    tp, ts = batches
    lib = nat.lib()
    pairs = [(lambda s: _tpke_prepare(lib, tp, s), lambda a, s: _tpke_verify(lib, tp, a, s), tp["expect"], tp["n"]),
             (lambda s: _ts_prepare(lib, ts, s), lambda a, s: _ts_verify(lib, ts, a, s), ts["expect"], ts["n"])]
    errors = []
    th = [threading.Thread(target=_worker, args=(lib, torch, dev, pairs if k == 0 else pairs[::-1], 6, errors))
          for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in th)
    assert not errors, errors


def test_two_threads_shared_explicit_context(nat, tdev, batches):
    """one lcb_ctx shared by a TPKE thread and a TS thread on different streams: the context serializes the
    calls and orders the work, and the TPKE / TS workspaces stay separate"""
    torch, dev = tdev
    tp, ts = batches
    lib = nat.lib()
    with nat.Context() as ctx:
        c = ctx.ptr
        p_t = [(lambda s: _tpke_prepare(lib, tp, s, c), lambda a, s: _tpke_verify(lib, tp, a, s, c), tp["expect"],
                tp["n"])]
        p_s = [(lambda s: _ts_prepare(lib, ts, s, c), lambda a, s: _ts_verify(lib, ts, a, s, c), ts["expect"],
                ts["n"])]
        errors = []
        th = [threading.Thread(target=_worker, args=(lib, torch, dev, p, 6, errors)) for p in (p_t, p_s)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=100)
        assert not any(t.is_alive() for t in th)
        assert not errors, errors
