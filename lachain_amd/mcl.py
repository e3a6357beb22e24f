"""lachain_amd/mcl.py — Python mirror of the managed MCL.BLS12_381.Net types Lachain uses
(Fr, G1, G2, GT, MclBls12381), backed by liblachain_bls.so's mcl-shaped C ABI (GPU kernels).

Method names follow the C# API census in SURVEY.md §8b (Fr.FromInt, Fr.GetRandom, G1.Generator,
G1.FromBytes, G2.SetHashOf, GT.Pairing, GT.Pow, MclBls12381.LagrangeInterpolate,
MclBls12381.EvaluatePolynomial, ...) so the parity tests read like test/Lachain.CryptoTest/MclTests.cs.
Failures raise (the reference's wrapper throws on a failed FromBytes / interpolation), including those of the
void GPU-backed calls (detected through lcb_error_count).
"""
import ctypes
import threading

from . import native
from .native import mclBnFr, mclBnG1, mclBnG2, mclBnGT

_FN = {}
_FN_LOCK = threading.Lock()


def _f(name, res, args):
    # a function object of its own per name (CDLL.__getitem__ does not cache; attribute access returns the object
    # native.py configured), configured once under a lock: setting restype / argtypes on an object another thread is
    # calling through frees the converters that call is using (a segfault with many calling threads)
    fn = _FN.get(name)
    if fn is None:
        with _FN_LOCK:
            fn = _FN.get(name)
            if fn is None:
                fn = native.lib()[name]
                fn.restype = res
                fn.argtypes = args
                _FN[name] = fn
    return fn


P = ctypes.POINTER
_sz = ctypes.c_size_t


def _void(name, args, *call):
    """call a void mcl entry point that runs on the GPU and raise if it failed: the C ABI has no return code for these
    (mcl's own signatures), so the library counts failures per thread (lcb_error_count) and a failed call also writes
    a random non-canonical value to its output (include/lachain_bls.h)"""
    cnt = _f("lcb_error_count", ctypes.c_uint64, [])
    before = cnt()
    _f(name, None, args)(*call)
    if cnt() != before:
        raise RuntimeError(f"{name} failed: {native.last_error()}")


class Fr:
    ByteSize = 32
    __slots__ = ("v",)

    def __init__(self, v=None):
        self.v = v if v is not None else mclBnFr()

    @staticmethod
    def FromInt(x):
        r = Fr()
        if _f("mclBnFr_setInt", ctypes.c_int, [P(mclBnFr), ctypes.c_int64])(ctypes.byref(r.v), int(x)) != 0:
            raise ValueError("Fr.FromInt failed")
        return r

    @staticmethod
    def GetRandom():
        r = Fr()
        if _f("mclBnFr_setByCSPRNG", ctypes.c_int, [P(mclBnFr)])(ctypes.byref(r.v)) != 0:
            raise RuntimeError("Fr.GetRandom failed")
        return r

    @staticmethod
    def FromBytes(b):
        r = Fr()
        b = bytes(b)
        if _f("mclBnFr_deserialize", _sz, [P(mclBnFr), ctypes.c_char_p, _sz])(ctypes.byref(r.v), b, len(b)) != 32:
            raise ValueError("Fr.FromBytes: invalid encoding")
        return r

    def ToBytes(self):
        buf = ctypes.create_string_buffer(32)
        if _f("mclBnFr_serialize", _sz, [ctypes.c_char_p, _sz, P(mclBnFr)])(buf, 32, ctypes.byref(self.v)) != 32:
            raise RuntimeError("Fr.ToBytes failed")
        return buf.raw

    @staticmethod
    def Zero():
        return Fr()

    @staticmethod
    def One():
        return Fr.FromInt(1)

    def _bin(self, name, other):
        r = Fr()
        _f(name, None, [P(mclBnFr), P(mclBnFr), P(mclBnFr)])(ctypes.byref(r.v), ctypes.byref(self.v),
                                                            ctypes.byref(other.v))
        return r

    def __add__(self, o):
        return self._bin("mclBnFr_add", o)

    def __sub__(self, o):
        return self._bin("mclBnFr_sub", o)

    def __mul__(self, o):
        return self._bin("mclBnFr_mul", o)

    def __truediv__(self, o):
        return self._bin("mclBnFr_div", o)

    def __neg__(self):
        r = Fr()
        _f("mclBnFr_neg", None, [P(mclBnFr), P(mclBnFr)])(ctypes.byref(r.v), ctypes.byref(self.v))
        return r

    def Inverse(self):
        r = Fr()
        _f("mclBnFr_inv", None, [P(mclBnFr), P(mclBnFr)])(ctypes.byref(r.v), ctypes.byref(self.v))
        return r

    def IsZero(self):
        return bool(_f("mclBnFr_isZero", ctypes.c_int, [P(mclBnFr)])(ctypes.byref(self.v)))

    def __eq__(self, o):
        return isinstance(o, Fr) and bytes(self.v) == bytes(o.v)

    def __hash__(self):
        return hash(bytes(self.v))

    def __repr__(self):
        return "Fr(0x" + self.ToBytes()[::-1].hex() + ")"


class _Point:
    _T = None
    _P = ""
    ByteSize = 0

    def __init__(self, v=None):
        self.v = v if v is not None else self._T()

    @classmethod
    def FromBytes(cls, b):
        r = cls()
        b = bytes(b)
        fn = _f(f"mclBn{cls._P}_deserialize", _sz, [P(cls._T), ctypes.c_char_p, _sz])
        if fn(ctypes.byref(r.v), b, len(b)) != cls.ByteSize:
            raise ValueError(f"{cls._P}.FromBytes: invalid encoding")
        return r

    def ToBytes(self):
        buf = ctypes.create_string_buffer(self.ByteSize)
        fn = _f(f"mclBn{self._P}_serialize", _sz, [ctypes.c_char_p, _sz, P(self._T)])
        if fn(buf, self.ByteSize, ctypes.byref(self.v)) != self.ByteSize:
            raise RuntimeError("ToBytes failed")
        return buf.raw

    @classmethod
    def Zero(cls):
        return cls()

    def _bin(self, op, other):
        r = type(self)()
        _void(f"mclBn{self._P}_{op}", [P(self._T), P(self._T), P(self._T)],
              ctypes.byref(r.v), ctypes.byref(self.v), ctypes.byref(other.v))
        return r

    def __add__(self, o):
        return self._bin("add", o)

    def __sub__(self, o):
        return self._bin("sub", o)

    def __neg__(self):
        r = type(self)()
        _void(f"mclBn{self._P}_neg", [P(self._T), P(self._T)], ctypes.byref(r.v), ctypes.byref(self.v))
        return r

    def __mul__(self, k):
        if not isinstance(k, Fr):
            return NotImplemented
        r = type(self)()
        _void(f"mclBn{self._P}_mul", [P(self._T), P(self._T), P(mclBnFr)],
              ctypes.byref(r.v), ctypes.byref(self.v), ctypes.byref(k.v))
        return r

    def IsValid(self):
        return bool(_f(f"mclBn{self._P}_isValid", ctypes.c_int, [P(self._T)])(ctypes.byref(self.v)))

    def IsZero(self):
        return bool(_f(f"mclBn{self._P}_isZero", ctypes.c_int, [P(self._T)])(ctypes.byref(self.v)))

    def __eq__(self, o):
        if type(o) is not type(self):
            return False
        return bool(_f(f"mclBn{self._P}_isEqual", ctypes.c_int, [P(self._T), P(self._T)])(
            ctypes.byref(self.v), ctypes.byref(o.v)))

    def __hash__(self):
        return hash(self.ToBytes())

    def __repr__(self):
        return f"{self._P}(0x{self.ToBytes().hex()})"


class G1(_Point):
    _T = mclBnG1
    _P = "G1"
    ByteSize = 48

    @staticmethod
    def Generator():
        r = G1()
        _void("lcb_g1_generator", [P(mclBnG1)], ctypes.byref(r.v))
        return r


class G2(_Point):
    _T = mclBnG2
    _P = "G2"
    ByteSize = 96

    @staticmethod
    def Generator():
        r = G2()
        _void("lcb_g2_generator", [P(mclBnG2)], ctypes.byref(r.v))
        return r

    def SetHashOf(self, msg):
        msg = bytes(msg)
        if _f("mclBnG2_hashAndMapTo", ctypes.c_int, [P(mclBnG2), ctypes.c_char_p, _sz])(
                ctypes.byref(self.v), msg, len(msg)) != 0:
            raise RuntimeError("G2.SetHashOf failed")
        return self


class GT:
    __slots__ = ("v",)

    def __init__(self, v=None):
        self.v = v if v is not None else mclBnGT()

    @staticmethod
    def Pairing(a, b):
        r = GT()
        _void("mclBn_pairing", [P(mclBnGT), P(mclBnG1), P(mclBnG2)], ctypes.byref(r.v), ctypes.byref(a.v),
              ctypes.byref(b.v))
        return r

    @staticmethod
    def Pow(a, k):
        r = GT()
        _void("mclBnGT_pow", [P(mclBnGT), P(mclBnGT), P(mclBnFr)], ctypes.byref(r.v), ctypes.byref(a.v),
              ctypes.byref(k.v))
        return r

    def __mul__(self, o):
        r = GT()
        _void("mclBnGT_mul", [P(mclBnGT), P(mclBnGT), P(mclBnGT)], ctypes.byref(r.v), ctypes.byref(self.v),
              ctypes.byref(o.v))
        return r

    def ToBytes(self):
        buf = ctypes.create_string_buffer(576)
        if _f("mclBnGT_serialize", _sz, [ctypes.c_char_p, _sz, P(mclBnGT)])(buf, 576, ctypes.byref(self.v)) != 576:
            raise RuntimeError("GT.ToBytes failed")
        return buf.raw

    def IsOne(self):
        return bool(_f("mclBnGT_isOne", ctypes.c_int, [P(mclBnGT)])(ctypes.byref(self.v)))

    def __eq__(self, o):
        return isinstance(o, GT) and bytes(self.v) == bytes(o.v)

    def __hash__(self):
        return hash(bytes(self.v))


class MclBls12381:
    @staticmethod
    def LagrangeInterpolate(xs, ys):
        k = len(xs)
        if k == 0 or len(ys) != k:
            raise ValueError("LagrangeInterpolate: bad sizes")
        xa = (mclBnFr * k)(*[x.v for x in xs])
        t = type(ys[0])
        if t is Fr:
            ya = (mclBnFr * k)(*[y.v for y in ys])
            out = Fr()
            fn = _f("mclBn_FrLagrangeInterpolation", ctypes.c_int, [P(mclBnFr), P(mclBnFr), P(mclBnFr), _sz])
        elif t is G1:
            ya = (mclBnG1 * k)(*[y.v for y in ys])
            out = G1()
            fn = _f("mclBn_G1LagrangeInterpolation", ctypes.c_int, [P(mclBnG1), P(mclBnFr), P(mclBnG1), _sz])
        else:
            ya = (mclBnG2 * k)(*[y.v for y in ys])
            out = G2()
            fn = _f("mclBn_G2LagrangeInterpolation", ctypes.c_int, [P(mclBnG2), P(mclBnFr), P(mclBnG2), _sz])
        if fn(ctypes.byref(out.v), xa, ya, k) != 0:
            raise ValueError("LagrangeInterpolate failed (zero or duplicate x)")
        return out

    @staticmethod
    def EvaluatePolynomial(coeffs, x):
        n = len(coeffs)
        if n == 0:
            raise ValueError("EvaluatePolynomial: empty")
        t = type(coeffs[0])
        if t is Fr:
            ca = (mclBnFr * n)(*[c.v for c in coeffs])
            out = Fr()
            fn = _f("mclBn_FrEvaluatePolynomial", ctypes.c_int, [P(mclBnFr), P(mclBnFr), _sz, P(mclBnFr)])
        elif t is G1:
            ca = (mclBnG1 * n)(*[c.v for c in coeffs])
            out = G1()
            fn = _f("mclBn_G1EvaluatePolynomial", ctypes.c_int, [P(mclBnG1), P(mclBnG1), _sz, P(mclBnFr)])
        else:
            ca = (mclBnG2 * n)(*[c.v for c in coeffs])
            out = G2()
            fn = _f("mclBn_G2EvaluatePolynomial", ctypes.c_int, [P(mclBnG2), P(mclBnG2), _sz, P(mclBnFr)])
        if fn(ctypes.byref(out.v), ca, n, ctypes.byref(x.v)) != 0:
            raise ValueError("EvaluatePolynomial failed")
        return out
