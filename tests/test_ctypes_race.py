"""Hypothesis (a) of the round-3 many-thread segfault (VERDICT r3 What's weak #2): the round-3 binding set `restype` /
`argtypes` on a ctypes function object that other threads were calling through.  Reproduced here on the CPU with the
host-only Fr exports (fr_host.hpp: no GPU needed), in the most adversarial form — EVERY call re-configures the shared
function object (the old `_f` did it only on a name's first use) — from 16 threads at once, in a child process so a
crash cannot take the test runner with it.  Every result is checked against Python integers mod r.

Finding: ctypes reads the converters and restype under the GIL before it releases the GIL for the foreign call and
does not use them after the call, and the types involved (c_int, c_size_t, POINTER(...) types, None) are never
freed, so the re-configuration is harmless — the process survives and every product is exact.  The round-3 crash
therefore did not come from the binding; the library-side cause (a half-built per-thread staging area written
through a null pinned buffer, lcb_host.cpp stage_ready) is fixed and tested in tests/test_gpu_failures.py."""
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "lachain_amd", "liblachain_bls.so")

CHILD = textwrap.dedent(r"""
    import ctypes, random, sys, threading
    R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    lib = ctypes.CDLL(sys.argv[1])
    class Fr(ctypes.Structure):
        _fields_ = [("d", ctypes.c_uint64 * 4)]
    P = ctypes.POINTER
    def old_f(name, res, args):            # the round-3 pattern, made worse: re-configure on every call
        fn = getattr(lib, name)             # CDLL attribute access returns one cached object per name
        fn.restype = res
        fn.argtypes = args
        return fn
    N_THREADS, N_CALLS = 16, int(sys.argv[2])
    start = threading.Barrier(N_THREADS)
    bad = []
    def to_fr(x):
        v = Fr()
        rc = old_f("mclBnFr_setLittleEndian", ctypes.c_int, [P(Fr), ctypes.c_char_p, ctypes.c_size_t])(
            ctypes.byref(v), x.to_bytes(32, "little"), 32)
        assert rc == 0
        return v
    def from_fr(v):
        buf = ctypes.create_string_buffer(32)
        n = old_f("mclBnFr_serialize", ctypes.c_size_t, [ctypes.c_char_p, ctypes.c_size_t, P(Fr)])(
            buf, 32, ctypes.byref(v))
        assert n == 32
        return int.from_bytes(buf.raw, "little")
    def work(seed):
        rng = random.Random(seed)
        start.wait()
        try:
            for _ in range(N_CALLS):
                a, b = rng.randrange(R >> 2), rng.randrange(R >> 2)
                x, y, z = to_fr(a), to_fr(b), Fr()
                op = rng.randrange(3)
                name = ("mclBnFr_mul", "mclBnFr_add", "mclBnFr_sub")[op]
                old_f(name, None, [P(Fr), P(Fr), P(Fr)])(ctypes.byref(z), ctypes.byref(x), ctypes.byref(y))
                want = (a * b, a + b, a - b)[op] % R
                if from_fr(z) != want:
                    bad.append((name, a, b))
        except Exception as e:
            bad.append(repr(e))
    ts = [threading.Thread(target=work, args=(i,)) for i in range(N_THREADS)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    print("bad", len(bad), bad[:3], "calls", N_THREADS * N_CALLS)
    sys.exit(1 if bad else 0)
""")


def test_reconfigured_function_objects_from_16_threads():
    r = subprocess.run([sys.executable, "-X", "faulthandler", "-c", CHILD, LIB, "4000"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "bad 0" in r.stdout


def test_current_binding_from_16_threads():
    """the binding as shipped (lachain_amd/mcl.py: one function object per name, configured once under a lock)"""
    code = textwrap.dedent(r"""
        import sys, threading, random
        sys.path.insert(0, sys.argv[1])
        from lachain_amd import native, mcl
        native.load(False)._inited = True     # no GPU here: the Fr surface is host code and needs no mclBn_init
        R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
        start = threading.Barrier(16)
        bad, done = [], []
        def work(seed):
            rng = random.Random(seed)
            start.wait()
            for _ in range(2000):
                a, b = rng.randrange(1 << 62), rng.randrange(1 << 62)
                x, y = mcl.Fr.FromInt(a), mcl.Fr.FromInt(b)
                if int.from_bytes((x * y - x).ToBytes(), "little") != (a * b - a) % R:
                    bad.append((a, b))
            done.append(seed)
        ts = [threading.Thread(target=work, args=(i,)) for i in range(16)]
        for t in ts: t.start()
        for t in ts: t.join()
        print("bad", len(bad), "done", len(done))
        sys.exit(1 if bad or len(done) != 16 else 0)
    """)
    r = subprocess.run([sys.executable, "-X", "faulthandler", "-c", code, ROOT], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
