#!/usr/bin/env python3
"""tools/queue_bench.py — latency / throughput of the aggregation queue (lcb_queue).

T caller threads each verify ONE TPKE decryption share per call (submit + wait), as HoneyBadger's protocol threads
do (HoneyBadger.cs:211-212, AbstractProtocol.cs:46-47), for a fixed wall time per setting.  Reported per batch
deadline (1, 5, 20 ms) and caller count: shares/s, mean batch size, and submit->decision latency percentiles.
Inputs: N=22 F=7 shares of 1,024 ciphertexts generated with the product's batch kernels (1 % corrupted); every
decision is checked against the construction.  Callers are Python threads (ctypes releases the GIL in the call),
so at high rates the Python side, not the GPU, bounds throughput; the numbers are the floor a native host gets.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shares", type=int, default=22 * 1024)
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--deadlines", default="1,5,20")
    ap.add_argument("--threads", default="16,64")
    ap.add_argument("--max-batch", type=int, default=65536)
    ap.add_argument("--prepare-ahead", type=int, default=1,
                    help="1: every ciphertext is prepared (lcb_queue_tpke_prepare) before its shares are submitted, as "
                         "HoneyBadger decrypts the common subset's ciphertexts (HoneyBadger.cs:144-146) before it "
                         "handles the other validators' shares (HoneyBadger.cs:190-213); 0: first sight in a flush")
    ap.add_argument("--prepare-stream", type=float, default=0.0,
                    help="ciphertexts per second prepared CONTINUOUSLY by a producer thread while the callers run "
                         "(ADVICE r5: the queue's latency with prepares arriving); callers verify shares of the "
                         "ciphertexts prepared so far.  0: off (--prepare-ahead decides)")
    ap.add_argument("--burst", type=int, default=1,
                    help="shares a caller submits before waiting for them (1 = strict one-share-per-call)")
    args = ap.parse_args()
    from lachain_amd import native as nat
    import bench
    nat.lib()
    inp = bench.make_inputs(nat, 0, args.shares, 22, 7, 32)
    vlen = 32
    recs = []
    for i in range(args.shares):
        c, j = int(inp["ct_idx"][i]), int(inp["dec_idx"][i])
        u, v, w = inp["cts_list"][c]
        recs.append((inp["keys_list"][j], u, v, w, inp["ui"][48 * i:48 * i + 48], bool(inp["expect"][i])))
    rows = []
    for dl in [float(x) for x in args.deadlines.split(",")]:
        for nt in [int(x) for x in args.threads.split(",")]:
            lat, bad, count = [], [0], [0]
            stop = time.perf_counter() + args.seconds
            n_cts = len(inp["cts_list"])
            ready = [n_cts]                             # ciphertexts whose shares may be submitted
            with nat.BatchQueue(max_batch=args.max_batch, max_delay_ms=dl) as q:
                stream = args.prepare_stream > 0
                if stream:                              # prepares arrive while the callers run
                    ready[0] = 0
                    n_prep = [0]

                    def producer():
                        t0 = time.perf_counter()
                        while ready[0] < n_cts and time.perf_counter() < stop:
                            u, v, w = inp["cts_list"][ready[0]]
                            q.prepare_tpke(u, v, w)
                            ready[0] += 1
                            n_prep[0] += 1
                            nxt = t0 + ready[0] / args.prepare_stream
                            while time.perf_counter() < nxt:
                                time.sleep(0.0002)
                    prod = threading.Thread(target=producer)
                    prod.start()
                    while ready[0] == 0:
                        time.sleep(0.0005)
                elif args.prepare_ahead:                # the epoch's ciphertexts, decrypted before shares arrive
                    for u, v, w in inp["cts_list"]:
                        q.prepare_tpke(u, v, w)
                    q.flush()
                    y, u, v, w, ui, e = recs[0]
                    assert q.verify_tpke(y, u, v, w, ui) == e   # the prepares ran (one worker queue is FIFO)
                    time.sleep(0.5)
                def caller(k):
                    idx, my = k, []
                    while time.perf_counter() < stop:
                        t0 = time.perf_counter()
                        pend = []
                        for _ in range(args.burst):
                            # shares of the ciphertexts prepared so far (ciphertext-major: 22 shares per ciphertext)
                            lim = max(1, min(len(recs), 22 * ready[0]))
                            y, u, v, w, ui, e = recs[idx % lim]
                            pend.append((q.submit_tpke(y, u, v, w, ui), e))
                            idx += nt
                        for tk, e in pend:
                            if q.wait(tk) != e:
                                bad[0] += 1
                        dt = time.perf_counter() - t0
                        my.extend([dt] * len(pend))
                    lat.extend(my)
                    count[0] += len(my)
                t_start = time.perf_counter()
                th = [threading.Thread(target=caller, args=(k,)) for k in range(nt)]
                for t in th:
                    t.start()
                for t in th:
                    t.join()
                elapsed = time.perf_counter() - t_start
                if stream:
                    prod.join()
                st = q.stats()
            ms = np.array(lat) * 1e3
            rows.append(dict(deadline_ms=dl, callers=nt, burst=args.burst, prepare_ahead=args.prepare_ahead,
                             prepare_stream_cts_per_s=args.prepare_stream, shares_per_s=count[0] / elapsed,
                             mean_batch=st["shares"] / max(1, st["batches"]), batches=st["batches"],
                             latency_ms={"p50": float(np.percentile(ms, 50)), "p90": float(np.percentile(ms, 90)),
                                         "p99": float(np.percentile(ms, 99))},
                             decision_mismatches=bad[0]))
            print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
