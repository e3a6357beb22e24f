"""The aggregation queue (lcb_queue) under the reference's call pattern: many protocol threads
each verifying ONE share per call (HoneyBadger.cs:211-212 VerifyShare, ThresholdSigner.cs:62 ValidateSignature,
threads per AbstractProtocol.cs:46-47).  16 threads submit single TPKE and threshold-signature shares; every
decision must equal the oracle's, and the shares must have run in fewer, larger GPU batches.
"""
import threading

import pytest

import oracle as o
from helpers import Drbg, R, gpu_native

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nat():
    return gpu_native()


def _keys(d, n, f):
    coeffs = [d.fr_int() for _ in range(f + 1)]
    poly = lambda x: sum(c * pow(x, i, R) for i, c in enumerate(coeffs)) % R
    return [poly(i + 1) for i in range(n)], poly(0)


@pytest.fixture(scope="module")
def items():
    d = Drbg(b"gpu-queue")
    out = []
    n, f = 4, 1
    xs, ys = _keys(d, n, f)
    yi = [o.g1_mul(o.g1_gen(), o.fr(x)) for x in xs]
    y = o.g1_mul(o.g1_gen(), o.fr(ys))
    for c in range(6):
        U, V, W = o.tpke_encrypt(y, d.bytes(20 + c), o.fr(d.fr_int()))
        for j in range(n):
            ui = o.g1_mul(U, o.fr(xs[j]))
            if (c + j) % 5 == 0:
                ui = o.g1_add(ui, o.g1_gen())      # wrong share
            out.append(("tpke", (yi[j], U, V, W, ui), o.tpke_verify_share(yi[j], U, V, W, ui) == 1))
    n2, f2 = 7, 2
    sks, _ = _keys(d, n2, f2)
    pks = [o.g1_mul(o.g1_gen(), o.fr(x)) for x in sks]
    for m in range(4):
        msg = b"CoinId" + bytes([m]) * 18
        for j in range(n2):
            sig = o.ts_sign(o.fr(sks[j]), msg)
            if (m * n2 + j) % 6 == 1:
                sig = o.ts_sign(o.fr(sks[(j + 1) % n2]), msg)   # another validator's signature
            out.append(("ts", (pks[j], msg, sig), o.ts_validate(pks[j], sig, msg) == 1))
    assert any(e for _, _, e in out) and not all(e for _, _, e in out)
    return out


@pytest.mark.parametrize("batched_min", [0, 8])
def test_queue_sixteen_threads_single_shares(nat, items, batched_min):
    """batched_min = 8: flushes of >= 8 shares go through the randomized batch checks (lcb_queue_set_batched), the
    shares of a flush reordered by ciphertext / message inside the library; decisions still equal the oracle's"""
    errors = []
    with nat.BatchQueue(max_batch=64, max_delay_ms=3.0, batched_min=batched_min) as q:
        def worker(k):
            try:
                for rep in range(3):
                    for idx in range(k, len(items), 16):
                        kind, args, expect = items[idx]
                        got = q.verify_tpke(*args) if kind == "tpke" else q.verify_ts(*args)
                        if got != expect:
                            errors.append((k, rep, idx, got, expect))
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))
        th = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=100)
        assert not any(t.is_alive() for t in th)
        st = q.stats()
    assert not errors, errors[:5]
    assert st["shares"] == 3 * len(items)
    assert st["batches"] < st["shares"] and st["largest_batch"] > 1, st


def test_queue_deadline_flush_and_tickets(nat, items):
    # one share, a batch size it never reaches: the deadline alone must flush it
    kind, args, expect = next(it for it in items if it[0] == "tpke")
    with nat.BatchQueue(max_batch=1 << 20, max_delay_ms=2.0) as q:
        t = q.submit_tpke(*args)
        assert q.wait(t) == expect
        with pytest.raises(RuntimeError):
            q.wait(t)                       # a ticket is consumed by its wait
        # submit many, wait in reverse order
        tickets = [(q.submit_ts(*a) if k == "ts" else q.submit_tpke(*a), e) for k, a, e in items]
        for tk, e in reversed(tickets):
            assert q.wait(tk) == e


def test_queue_prepare_ahead(nat, items):
    """lcb_queue_tpke_prepare: the ciphertexts prepared on their workers before any share (HoneyBadger.cs:144-146
    decrypts the common subset's ciphertexts first), an undecodable ciphertext and a repeated prepare among them; the
    shares then submitted from 16 threads get the oracle's decisions, TS shares beside them"""
    cts = []
    for kind, args, _ in items:
        if kind == "tpke" and (args[1], args[2], args[3]) not in cts:
            cts.append((args[1], args[2], args[3]))
    errors = []
    with nat.BatchQueue(max_batch=64, max_delay_ms=2.0) as q:
        for u, v, w in cts + cts[:2]:
            q.prepare_tpke(u, v, w)
        q.prepare_tpke(b"\xff" * 48, b"x", b"\xff" * 96)       # not a ciphertext: prepared as invalid, harmless
        with pytest.raises(ValueError):
            q.prepare_tpke(b"", b"", b"")

        def worker(k):
            try:
                for idx in range(k, len(items), 16):
                    kind, args, expect = items[idx]
                    got = q.verify_tpke(*args) if kind == "tpke" else q.verify_ts(*args)
                    if got != expect:
                        errors.append((k, idx, got, expect))
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))
        th = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=100)
        assert not any(t.is_alive() for t in th)
    assert not errors, errors[:5]


@pytest.mark.parametrize("workers", ["1", "4"])
def test_queue_worker_counts(nat, items, workers, monkeypatch):
    """LCB_QUEUE_WORKERS (read when the queue is created): one worker (every flush serial) and four (flushes side by
    side, two of the workers' streams sharing a hardware queue at the default GPU_MAX_HW_QUEUES) give the same decisions,
    with ciphertexts prepared ahead on every worker and some not"""
    monkeypatch.setenv("LCB_QUEUE_WORKERS", workers)
    errors = []
    cts = []
    for kind, args, _ in items:
        if kind == "tpke" and (args[1], args[2], args[3]) not in cts:
            cts.append((args[1], args[2], args[3]))
    with nat.BatchQueue(max_batch=16, max_delay_ms=1.0) as q:
        for u, v, w in cts[::2]:                        # half prepared ahead, half met first in a flush
            q.prepare_tpke(u, v, w)

        def worker(k):
            try:
                for rep in range(2):
                    for idx in range(k, len(items), 8):
                        kind, args, expect = items[idx]
                        got = q.verify_tpke(*args) if kind == "tpke" else q.verify_ts(*args)
                        if got != expect:
                            errors.append((k, rep, idx, got, expect))
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))
        th = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=100)
        assert not any(t.is_alive() for t in th)
        st = q.stats()
    assert not errors, errors[:5]
    assert st["shares"] == 2 * len(items)

