"""Stress of the mcl binding from many threads starting at once (the first call of every function races to create
it; lachain_amd/mcl.py _f): 16 threads x 4 rounds of G1 / G2 multiplications and a pairing, results checked against
the first thread's.  Usage: python tools/mcl_thread_stress.py"""
import os
import sys
import threading

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402,F401  (HIP runtime first, as bench.py / conftest do)

if torch.cuda.is_available():
    torch.zeros(1, device="cuda:0")
from lachain_amd import mcl  # noqa: E402

start = threading.Barrier(16)
out, errs = [None] * 16, []


def work(i):
    try:
        start.wait()
        for _ in range(4):
            a = mcl.G1.Generator() * mcl.Fr.FromInt(7 + i % 3)
            b = mcl.G2.Generator() * mcl.Fr.FromInt(11)
            out[i] = (i % 3, mcl.GT.Pairing(a, b).ToBytes(), (a + a).ToBytes(), (-b).ToBytes())
    except Exception as e:  # noqa: BLE001
        errs.append(e)


ts = [threading.Thread(target=work, args=(i,)) for i in range(16)]
for t in ts:
    t.start()
for t in ts:
    t.join()
assert not errs, errs
ref = {}
for r in out:
    ref.setdefault(r[0], r)
    assert ref[r[0]] == r
print("mcl thread stress ok")
