"""lachain_amd/tpke.py — Python mirror of Lachain.Crypto.TPKE (threshold public-key encryption) on
liblachain_bls.so.  Class / method names and error behaviour follow the reference:

  EncryptedShare            /root/reference/src/Lachain.Crypto/TPKE/EncryptedShare.cs:9-34
  PartiallyDecryptedShare   TPKE/PartiallyDecryptedShare.cs:5-18
  PrivateKey.Decrypt        TPKE/PrivateKey.cs:21-31   (throws "Invalid share!")
  PublicKey.Encrypt         TPKE/PublicKey.cs:25-37
  PublicKey.FullDecrypt     TPKE/PublicKey.cs:55-86    (count / duplicate-id / share-id checks)
  PublicKey.VerifyShare     TPKE/PublicKey.cs:88-92
  TrustedKeyGen             TPKE/TrustedKeyGen.cs:11-34 (degree-(f-1) polynomial, f coefficients)
  Utils.XorWithHash / HashToG2  TPKE/Utils.cs:12-27

Batch entry points (`VerifyShares`, `DecryptBatch`) hand whole batches to the GPU in one call — the
shape HoneyBadger's loops can use (HoneyBadger.cs:141-175, 200-247).
"""
import struct

from . import native
from .mcl import Fr, G1, MclBls12381


class RawShare:
    def __init__(self, data: bytes, id_: int):
        self.Data = bytes(data)
        self.Id = id_

    def ToBytes(self):
        return self.Data

    def __eq__(self, o):
        return isinstance(o, RawShare) and o.Id == self.Id and o.Data == self.Data


class EncryptedShare:
    """U (G1 48 B), V (bytes), W (G2 96 B), Id (int32); wire = Id LE || U || W || V (EncryptedShare.cs:25-28)."""

    def __init__(self, u: bytes, v: bytes, w: bytes, id_: int):
        self.U, self.V, self.W, self.Id = bytes(u), bytes(v), bytes(w), id_

    def ToBytes(self):
        return struct.pack("<i", self.Id) + self.U + self.W + self.V

    @staticmethod
    def FromBytes(b: bytes):
        (id_,) = struct.unpack_from("<i", b, 0)
        u = b[4:52]
        w = b[52:148]
        G1.FromBytes(u)  # FixedWithSerializer.Deserialize decodes U and W (throws on malformed input)
        from .mcl import G2
        G2.FromBytes(w)
        return EncryptedShare(u, b[148:], w, id_)

    def __eq__(self, o):
        return isinstance(o, EncryptedShare) and (self.U, self.V, self.W, self.Id) == (o.U, o.V, o.W, o.Id)


class PartiallyDecryptedShare:
    def __init__(self, ui: bytes, decryptor_id: int, share_id: int):
        self.Ui, self.DecryptorId, self.ShareId = bytes(ui), decryptor_id, share_id


class Utils:
    @staticmethod
    def XorWithHash(g1_bytes: bytes, data: bytes) -> bytes:
        return native.xor_with_hash(g1_bytes, data)

    @staticmethod
    def HashToG2(u_bytes: bytes, v: bytes) -> bytes:
        return native.g2_hash_batch([bytes(u_bytes) + bytes(v)])[0]


class PrivateKey:
    def __init__(self, x: Fr, id_: int):
        self._x = x
        self._id = id_

    def Decrypt(self, share: EncryptedShare) -> PartiallyDecryptedShare:
        ok, ui = native.tpke_partial_decrypt(self._x.ToBytes(), [(share.U, share.V, share.W)])[0]
        if not ok:
            raise ValueError("Invalid share!")
        return PartiallyDecryptedShare(ui, self._id, share.Id)

    def DecryptBatch(self, shares):
        """Decrypt for a batch; returns PartiallyDecryptedShare or None ("Invalid share!") per item."""
        res = native.tpke_partial_decrypt(self._x.ToBytes(), [(s.U, s.V, s.W) for s in shares])
        return [PartiallyDecryptedShare(ui, self._id, s.Id) if ok else None for (ok, ui), s in zip(res, shares)]


class PublicKey:
    def __init__(self, y: bytes, t: int):
        self._y = bytes(y)
        self._t = t

    @property
    def Y(self):
        return self._y

    def Encrypt(self, raw_share: RawShare, r: Fr = None) -> EncryptedShare:
        r = r if r is not None else Fr.GetRandom()
        rb = r.ToBytes()
        (u,), (t,) = native.tpke_encrypt_phase1(self._y, [rb])
        v = Utils.XorWithHash(t, raw_share.ToBytes())
        (w,) = native.tpke_encrypt_phase2([u], [rb], [v])
        return EncryptedShare(u, v, w, raw_share.Id)

    def VerifyShare(self, share: EncryptedShare, ps: PartiallyDecryptedShare) -> bool:
        # the reference calls this once per (ciphertext, validator) (HoneyBadger.cs:211-212): the thread context's
        # prepared-ciphertext and key caches (lcb_tpke_verify_shares_cached) keep H(U, V), the line sets and Y_i
        # across the N calls of one ciphertext; the decision is the same exact check
        return native.tpke_verify_shares([self._y], [(share.U, share.V, share.W)], [(0, 0, ps.Ui)], cached=True)[0]

    @staticmethod
    def VerifyShares(verification_keys, shares, partials):
        """Batch of VerifyShare calls: partials[i] = (ciphertext index into `shares`,
        PartiallyDecryptedShare); the verification key is verification_keys[DecryptorId]."""
        keys = [vk.Y if isinstance(vk, PublicKey) else bytes(vk) for vk in verification_keys]
        return native.tpke_verify_shares(keys, [(s.U, s.V, s.W) for s in shares],
                                         [(ci, ps.DecryptorId, ps.Ui) for ci, ps in partials])

    def FullDecrypt(self, share: EncryptedShare, us):
        if len(us) < self._t:
            raise ValueError("Insufficient number of shares!")
        ids = set()
        for part in us:
            if part.DecryptorId in ids:
                raise ValueError(f"Id {part.DecryptorId} was provided more than once!")
            if part.ShareId != share.Id:
                raise ValueError(f"Share id mismatch for decryptor {part.DecryptorId}")
            ids.add(part.DecryptorId)
        xs = [Fr.FromInt(p.DecryptorId + 1).ToBytes() for p in us]
        u = native.lagrange_batch(1, [(xs, [p.Ui for p in us])])[0]
        if u is None:
            raise ValueError("LagrangeInterpolate failed")
        return RawShare(Utils.XorWithHash(u, share.V), share.Id)

    def ToBytes(self):
        return struct.pack("<i", self._t) + self._y

    @staticmethod
    def FromBytes(b):
        (t,) = struct.unpack_from("<i", b, 0)
        y = b[4:52]
        G1.FromBytes(y)
        return PublicKey(y, t)

    def __eq__(self, o):
        return isinstance(o, PublicKey) and o._y == self._y and o._t == self._t


class TrustedKeyGen:
    """TPKE trusted dealer: f random coefficients (degree f-1), TrustedKeyGen.cs:11-34."""

    def __init__(self, n: int, f: int, coeffs=None):
        if n <= 3 * f:
            raise ValueError(f"n should be greater than 3*f, but {n} <= 3 * {f} = {3 * f}")
        self._degree = f
        self._coeffs = list(coeffs) if coeffs is not None else [Fr.GetRandom() for _ in range(f)]

    def _eval(self, x: int) -> Fr:
        return MclBls12381.EvaluatePolynomial(self._coeffs, Fr.FromInt(x))

    def GetPubKey(self):
        return PublicKey((G1.Generator() * self._eval(0)).ToBytes(), self._degree)

    def GetPrivKey(self, i: int):
        return PrivateKey(self._eval(i + 1), i)

    def GetVerificationPubKey(self, i: int):
        return PublicKey((G1.Generator() * self._eval(i + 1)).ToBytes(), self._degree)
