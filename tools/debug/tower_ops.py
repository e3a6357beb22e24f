"""GPU debug probe: run each tower routine (OP_DEBUG_FP12) of two builds of liblachain_bls.so on the same
input and report which outputs differ."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from lachain_amd import native as nat
from lachain_amd import mcl
from lachain_amd.mcl import _f, P
from lachain_amd.native import mclBnGT, mclBnG1, mclBnG2
from helpers import Drbg

Fr, G1, G2, GT = mcl.Fr, mcl.G1, mcl.G2, mcl.GT
d = Drbg(b"gpu-pairing")
A = G1.Generator() * Fr.FromBytes(d.fr())
B = G2.Generator() * Fr.FromBytes(d.fr())
f = GT()
_f("mclBn_millerLoop", None, [P(mclBnGT), P(mclBnG1), P(mclBnG2)])(ctypes.byref(f.v), ctypes.byref(A.v), ctypes.byref(B.v))
fin = bytes(f.v)
# a unitary input for the cyclotomic routines: f^(p^6-1)(p^2+1) computed by the primary build
libs = [ctypes.CDLL(p) for p in sys.argv[1:]]
def run(lib, which, x):
    out = ctypes.create_string_buffer(576)
    assert lib.lcb_debug_fp12(which, x, out) == 0
    return out.raw
uni = run(libs[0], 5, fin)
names = ["inv", "cyc_sqr", "frob1", "frob2", "frob3", "fe_easy", "cyc_pow_z", "sqr", "fp6_inv", "fp2_inv", "conj", "fe_hard"]
for w, n in enumerate(names):
    x = uni if n in ("cyc_sqr", "cyc_pow_z", "fe_hard") else fin
    outs = [run(l, w, x) for l in libs]
    print(f"{n:10s}", "same" if all(o == outs[0] for o in outs) else "DIFF")
