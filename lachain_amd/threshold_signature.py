"""lachain_amd/threshold_signature.py — Python mirror of Lachain.Crypto.ThresholdSignature on
liblachain_bls.so (BLS threshold signatures: signatures in G2, keys in G1).

  PublicKey.ValidateSignature     /root/reference/src/Lachain.Crypto/ThresholdSignature/PublicKey.cs:16-21
  PrivateKeyShare.HashAndSign     ThresholdSignature/PrivateKeyShare.cs:21-27
  PublicKeySet (AssemblePublicKey, AssembleSignature)   ThresholdSignature/PublicKeySet.cs:19-42
  Signature (Parity, wire form)   ThresholdSignature/Signature.cs:9-39
  ThresholdSigner (Sign, AddShare state machine)        ThresholdSignature/ThresholdSigner.cs:24-92
  TrustedKeyGen (degree f, f+1 coefficients)            ThresholdSignature/TrustedKeyGen.cs:14-31
"""
from . import native
from .mcl import Fr, G1, G2, MclBls12381


class Signature:
    def __init__(self, raw: bytes):
        self.RawSignature = bytes(raw)  # serialized G2

    def Parity(self):
        p = 0
        for b in self.RawSignature:
            p ^= b
        return bin(p).count("1") % 2 == 1

    def ToBytes(self):
        return self.RawSignature

    @staticmethod
    def FromBytes(b):
        G2.FromBytes(b)  # throws on malformed input
        return Signature(bytes(b))

    def __eq__(self, o):
        return isinstance(o, Signature) and o.RawSignature == self.RawSignature

    def __hash__(self):
        return hash(self.RawSignature)


class PublicKey:
    def __init__(self, raw_key: bytes):
        self.RawKey = bytes(raw_key)

    def ValidateSignature(self, signature: Signature, message: bytes) -> bool:
        return native.ts_verify_shares([self.RawKey], [bytes(message)], [(0, 0, signature.RawSignature)])[0]

    def __eq__(self, o):
        return isinstance(o, PublicKey) and o.RawKey == self.RawKey

    def __hash__(self):
        return hash(self.RawKey)


class PrivateKeyShare:
    def __init__(self, sk: Fr):
        self._sk = sk

    def GetPublicKeyShare(self) -> PublicKey:
        return PublicKey((G1.Generator() * self._sk).ToBytes())

    def HashAndSign(self, message: bytes) -> Signature:
        return Signature(native.ts_sign([self._sk.ToBytes()], [bytes(message)], [0])[0])

    def ToBytes(self):
        return self._sk.ToBytes()


def validate_batch(pks, messages, items):
    """Batch ValidateSignature: items = (message index, public-key index, Signature)."""
    return native.ts_verify_shares([pk.RawKey for pk in pks], [bytes(m) for m in messages],
                                   [(mi, ki, s.RawSignature) for mi, ki, s in items])


class PublicKeySet:
    def __init__(self, pub_key_shares, faulty: int):
        self._keys = list(pub_key_shares)
        n = len(self._keys)
        xs = [Fr.FromInt(i).ToBytes() for i in range(1, n + 1)]
        shared = native.lagrange_batch(1, [(xs, [k.RawKey for k in self._keys])])[0]
        if shared is None:
            raise ValueError("AssemblePublicKey failed")
        self.SharedPublicKey = PublicKey(shared)
        self.Threshold = faulty

    @property
    def Keys(self):
        return self._keys

    @property
    def Count(self):
        return len(self._keys)

    def __getitem__(self, i):
        return self._keys[i]

    def AssembleSignature(self, shares):
        """shares: iterable of (index, Signature); uses the first Threshold+1 in iteration order."""
        pairs = list(shares)[: self.Threshold + 1]
        if len(pairs) <= self.Threshold:
            raise ValueError("not enough shares for signature")
        xs = [Fr.FromInt(k + 1).ToBytes() for k, _ in pairs]
        sig = native.lagrange_batch(2, [(xs, [s.RawSignature for _, s in pairs])])[0]
        if sig is None:
            raise ValueError("LagrangeInterpolate failed")
        return Signature(sig)


class ThresholdSigner:
    def __init__(self, data_to_sign: bytes, private_key_share: PrivateKeyShare, public_key_set: PublicKeySet):
        if private_key_share.GetPublicKeyShare() not in public_key_set.Keys:
            raise ValueError("Invalid private key share for threshold signature: "
                             "corresponding public key is not in keyring")
        self._data = bytes(data_to_sign)
        self._sk = private_key_share
        self._pks = public_key_set
        self._collected = [None] * public_key_set.Count
        self._n_collected = 0
        self._signature = None

    def Sign(self) -> Signature:
        return self._sk.HashAndSign(self._data)

    def AddShare(self, idx: int, sig_share: Signature):
        """Returns (accepted: bool, result Signature | None) — ThresholdSigner.cs:44-87."""
        if idx < 0 or idx >= self._pks.Count:
            return False, None
        pub = self._pks[idx]
        if self._collected[idx] is not None:
            if sig_share != self._collected[idx]:
                return False, None
            self._n_collected -= 1
        if not pub.ValidateSignature(sig_share, self._data):
            return False, None
        if self._n_collected > self._pks.Threshold:
            return True, self._signature
        self._collected[idx] = sig_share
        self._n_collected += 1
        if self._n_collected <= self._pks.Threshold:
            return True, None
        signature = self._pks.AssembleSignature((i, s) for i, s in enumerate(self._collected) if s is not None)
        if not self._pks.SharedPublicKey.ValidateSignature(signature, self._data):
            raise RuntimeError("Fatal error: all shares are valid but combined signature is not")
        self._signature = signature
        return True, signature


class TrustedKeyGen:
    def __init__(self, n: int, f: int, coeffs=None):
        if n <= 3 * f:
            raise ValueError(f"n should be greater than 3*f, but {n} <= 3 * {f} = {3 * f}")
        self._degree = f
        self._parties = n
        self._coeffs = list(coeffs) if coeffs is not None else [Fr.GetRandom() for _ in range(f + 1)]

    def GetPrivateShares(self):
        return [PrivateKeyShare(MclBls12381.EvaluatePolynomial(self._coeffs, Fr.FromInt(i + 1)))
                for i in range(self._parties)]
