"""GPU debug probe: Miller loop, final exponentiation and GT mul of the product vs the oracle, op by op."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle as o
from helpers import Drbg
from lachain_amd import native as _nat
if os.environ.get("LCB_SO"): _nat.LIB_PATH = os.environ["LCB_SO"]
from lachain_amd import mcl
from lachain_amd.mcl import _f, P
from lachain_amd.native import mclBnGT, mclBnG1, mclBnG2

Fr, G1, G2, GT = mcl.Fr, mcl.G1, mcl.G2, mcl.GT
d = Drbg(b"gpu-pairing")
a, b = d.fr(), d.fr()
A = G1.Generator() * Fr.FromBytes(a)
B = G2.Generator() * Fr.FromBytes(b)
f = GT()
_f("mclBn_millerLoop", None, [P(mclBnGT), P(mclBnG1), P(mclBnG2)])(ctypes.byref(f.v), ctypes.byref(A.v), ctypes.byref(B.v))
fo = o.miller_loop(A.ToBytes(), B.ToBytes())
print("miller equal:", f.ToBytes() == fo)
e = GT()
_f("mclBn_finalExp", None, [P(mclBnGT), P(mclBnGT)])(ctypes.byref(e.v), ctypes.byref(f.v))
print("final_exp(gpu f) equal oracle final_exp(gpu f):", e.ToBytes() == o.final_exp(f.ToBytes()))
m = f * f
print("gt_mul equal:", m.ToBytes() == o.gt_mul(f.ToBytes(), f.ToBytes()))
