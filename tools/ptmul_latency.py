"""Median latency of mclBnG1_mul / mclBnG2_mul (k_ptmul.hip's cooperative ladders) through the mcl surface, the same
measurement as bench.py's mcl_latency leg, without the rest of the bench.  Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lachain_amd import mcl  # noqa: E402


def med(fn, reps=400):
    for _ in range(20):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return 1e3 * ts[len(ts) // 2]


a, b = mcl.Fr.GetRandom(), mcl.Fr.GetRandom()
P, Q = mcl.G1.Generator() * a, mcl.G2.Generator() * b
k = mcl.Fr.GetRandom()
print(json.dumps({"G1_mul_ms": round(med(lambda: P * k), 4), "G2_mul_ms": round(med(lambda: Q * k), 4)}))
