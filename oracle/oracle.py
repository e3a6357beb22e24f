"""oracle/oracle.py — TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/liborc.so, the plain-C restatement of the MCL BLS12-381 path Lachain uses
(see bls_oracle.h).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liborc.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle/liborc.so not built (run `make -C oracle`)")
        _LIB = ctypes.CDLL(path)
        _LIB.orc_init()
        _LIB.orc_count_get.restype = ctypes.c_uint64
    return _LIB


def _buf(n):
    return ctypes.create_string_buffer(n)


def _ck(rc, what):
    if rc != 0:
        raise ValueError(f"oracle {what} failed ({rc})")


# ---------------------------------------------------------------- Fr
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


def fr(v: int) -> bytes:
    return (v % R).to_bytes(32, "little")


def fr_from_int(v: int) -> bytes:
    o = _buf(32); lib().orc_fr_from_int(o, ctypes.c_int64(v)); return o.raw


def fr_mul(a, b):
    o = _buf(32); _ck(lib().orc_fr_mul(o, a, b), "fr_mul"); return o.raw


def fr_add(a, b):
    o = _buf(32); _ck(lib().orc_fr_add(o, a, b), "fr_add"); return o.raw


def fr_from_wide(b64: bytes) -> bytes:
    o = _buf(32); lib().orc_fr_from_wide(o, b64); return o.raw


# ---------------------------------------------------------------- groups
def g1_gen():
    o = _buf(48); lib().orc_g1_generator(o); return o.raw


def g2_gen():
    o = _buf(96); lib().orc_g2_generator(o); return o.raw


def g1_mul(p, s):
    o = _buf(48); _ck(lib().orc_g1_mul(o, p, s), "g1_mul"); return o.raw


def g2_mul(p, s):
    o = _buf(96); _ck(lib().orc_g2_mul(o, p, s), "g2_mul"); return o.raw


def g1_add(a, b):
    o = _buf(48); _ck(lib().orc_g1_add(o, a, b), "g1_add"); return o.raw


def g2_add(a, b):
    o = _buf(96); _ck(lib().orc_g2_add(o, a, b), "g2_add"); return o.raw


def g1_neg(a):
    o = _buf(48); _ck(lib().orc_g1_neg(o, a), "g1_neg"); return o.raw


def g2_neg(a):
    o = _buf(96); _ck(lib().orc_g2_neg(o, a), "g2_neg"); return o.raw


def g1_valid(a):
    return bool(lib().orc_g1_is_valid_encoding(a))


def g2_valid(a):
    return bool(lib().orc_g2_is_valid_encoding(a))


def g1_in_subgroup(a):
    return bool(lib().orc_g1_in_subgroup(a))


def g2_in_subgroup(a):
    return bool(lib().orc_g2_in_subgroup(a))


def g2_hash(msg: bytes):
    o = _buf(96); _ck(lib().orc_g2_hash(o, msg, ctypes.c_size_t(len(msg))), "g2_hash"); return o.raw


def _lagr(fn, size, xs, ys):
    o = _buf(size)
    rc = fn(o, b"".join(xs), b"".join(ys), ctypes.c_size_t(len(xs)))
    if rc != 0:
        return None
    return o.raw


def g1_lagrange(xs, ys):
    return _lagr(lib().orc_g1_lagrange, 48, xs, ys)


def g2_lagrange(xs, ys):
    return _lagr(lib().orc_g2_lagrange, 96, xs, ys)


def fr_lagrange(xs, ys):
    return _lagr(lib().orc_fr_lagrange, 32, xs, ys)


def fr_eval_poly(coeffs, x):
    o = _buf(32)
    _ck(lib().orc_fr_eval_poly(o, b"".join(coeffs), ctypes.c_size_t(len(coeffs)), x), "eval_poly")
    return o.raw


def g1_msm(points, scalars):
    o = _buf(48)
    _ck(lib().orc_g1_msm(o, b"".join(points), b"".join(scalars), ctypes.c_size_t(len(points))), "msm")
    return o.raw


def dkg_commitment_eval(coeffs, degree, x, y):
    o = _buf(48)
    _ck(lib().orc_dkg_commitment_eval(o, b"".join(coeffs), degree, ctypes.c_int32(x), ctypes.c_int32(y)), "dkg eval")
    return o.raw


def dkg_commitment_row(coeffs, degree, x):
    o = _buf(48 * (degree + 1))
    _ck(lib().orc_dkg_commitment_row(o, b"".join(coeffs), degree, ctypes.c_int32(x)), "dkg row")
    return [o.raw[48 * i:48 * i + 48] for i in range(degree + 1)]


def g1_eval_poly(coeffs, x):
    o = _buf(48)
    _ck(lib().orc_g1_eval_poly(o, b"".join(coeffs), ctypes.c_size_t(len(coeffs)), x), "g1 eval poly")
    return o.raw


def rs_encode_codeword(data, ecc):
    n = len(data) + ecc
    arr = (ctypes.c_int * n)(*(list(data) + [0] * ecc))
    _ck(lib().orc_rs_encode_codeword(arr, n, ecc), "rs encode")
    return list(arr)


def rs_encode_shards(data: bytes, shards, erasures):
    out = _buf(len(data) // (shards - erasures) * shards)
    _ck(lib().orc_rs_encode_shards(out, data, ctypes.c_size_t(len(data)), shards, erasures), "rs encode shards")
    return out.raw


def rs_decode_shards(echos, shard_size, shards, erasures):
    """echos: list of (from, shard bytes) -> all shards concatenated, or None if unsolvable"""
    out = _buf(shard_size * shards)
    frm = (ctypes.c_int32 * max(1, len(echos)))(*[e[0] for e in echos])
    rc = lib().orc_rs_decode_shards(out, b"".join(e[1] for e in echos), frm, len(echos), ctypes.c_size_t(shard_size),
                                    shards, erasures)
    return out.raw if rc == 0 else None


# ---------------------------------------------------------------- pairing
def pairing(p, q):
    o = _buf(576); _ck(lib().orc_pairing(o, p, q), "pairing"); return o.raw


def pairing_slow(p, q):
    o = _buf(576); _ck(lib().orc_pairing_slow(o, p, q), "pairing_slow"); return o.raw


def miller_loop(p, q):
    o = _buf(576); _ck(lib().orc_miller_loop(o, p, q), "miller"); return o.raw


def final_exp(f):
    o = _buf(576); _ck(lib().orc_final_exp(o, f), "fe"); return o.raw


def final_exp_direct(f):
    o = _buf(576); _ck(lib().orc_final_exp_direct(o, f), "fe_direct"); return o.raw


def gt_pow(a, s):
    o = _buf(576); _ck(lib().orc_gt_pow(o, a, s), "gt_pow"); return o.raw


def gt_mul(a, b):
    o = _buf(576); _ck(lib().orc_gt_mul(o, a, b), "gt_mul"); return o.raw


# ---------------------------------------------------------------- hashing / KDF
def sha3_256(m):
    o = _buf(32); lib().orc_sha3_256(o, m, ctypes.c_size_t(len(m))); return o.raw


def sha512(m):
    o = _buf(64); lib().orc_sha512(o, m, ctypes.c_size_t(len(m))); return o.raw


def sha256(m):
    o = _buf(32); lib().orc_sha256(o, m, ctypes.c_size_t(len(m))); return o.raw


def drg_bytes(seed: bytes, n: int) -> bytes:
    o = _buf(n); lib().orc_drg_bytes(o, ctypes.c_size_t(n), seed, ctypes.c_size_t(len(seed))); return o.raw


def xor_with_hash(g1b: bytes, data: bytes) -> bytes:
    o = _buf(max(1, len(data))); lib().orc_xor_with_hash(o, g1b, data, ctypes.c_size_t(len(data)))
    return o.raw[: len(data)]


def coin_parity(sig: bytes) -> bool:
    return bool(lib().orc_coin_parity(sig, ctypes.c_size_t(len(sig))))


def coin_nonce(sig: bytes) -> int:
    f = lib().orc_coin_nonce
    f.restype = ctypes.c_uint64
    return int(f(sig, ctypes.c_size_t(len(sig))))


# ---------------------------------------------------------------- protocol
def tpke_encrypt(y, data, r):
    u, v, w = _buf(48), _buf(max(1, len(data))), _buf(96)
    _ck(lib().orc_tpke_encrypt(u, v, w, y, data, ctypes.c_size_t(len(data)), r), "encrypt")
    return u.raw, v.raw[: len(data)], w.raw


def tpke_decrypt(u, v, w, x):
    ui = _buf(48)
    rc = lib().orc_tpke_decrypt(ui, u, v, ctypes.c_size_t(len(v)), w, x)
    if rc == -1:
        raise ValueError("Invalid share!")
    _ck(rc, "decrypt")
    return ui.raw


def tpke_verify_share(y_i, u, v, w, ui):
    return lib().orc_tpke_verify_share(y_i, u, v, ctypes.c_size_t(len(v)), w, ui)


def tpke_full_decrypt(v, ids, uis):
    o = _buf(max(1, len(v)))
    ids_arr = (ctypes.c_int32 * max(1, len(ids)))(*ids)
    _ck(lib().orc_tpke_full_decrypt(o, v, ctypes.c_size_t(len(v)), ids_arr, b"".join(uis),
                                    ctypes.c_size_t(len(uis))), "full_decrypt")
    return o.raw[: len(v)]


def ts_sign(sk, msg):
    o = _buf(96); _ck(lib().orc_ts_sign(o, sk, msg, ctypes.c_size_t(len(msg))), "sign"); return o.raw


def ts_validate(pk, sig, msg):
    return lib().orc_ts_validate(pk, sig, msg, ctypes.c_size_t(len(msg)))


def set_g2_sign_from_b(v):
    lib().orc_set_g2_sign_from_b(int(v))


def set_g2_original_cofactor(v):
    lib().orc_set_g2_original_cofactor(int(v))


def count_reset():
    lib().orc_count_reset()


def count_get():
    return lib().orc_count_get()


# ---------------------------------------------------------------- secp256k1 ECDSA / Keccak (oracle/secp.c, §8f row 4)
SECP_N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
SECP_P = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F


def keccak256(m: bytes) -> bytes:
    o = _buf(32); lib().orc_keccak256(o, m, ctypes.c_size_t(len(m))); return o.raw


def header_keccak(prev: bytes, state: bytes, merkle: bytes, index: int, nonce: int) -> bytes:
    o = _buf(32)
    lib().orc_header_keccak(o, prev, state, merkle, ctypes.c_uint64(index), ctypes.c_uint64(nonce))
    return o.raw


def ecdsa_pubkey(priv: bytes):
    """(compressed 33 B, uncompressed 65 B) public key of a 32-byte big-endian private key"""
    c33, c65 = _buf(33), _buf(65)
    _ck(lib().orc_ecdsa_pubkey(c33, c65, priv), "ecdsa_pubkey")
    return c33.raw, c65.raw


def ecdsa_sign_compact(hash32: bytes, priv: bytes, k: bytes):
    """(r || s low-s, recovery id) with nonce k"""
    sig, rid = _buf(64), ctypes.c_int(0)
    _ck(lib().orc_ecdsa_sign_k(sig, ctypes.byref(rid), hash32, priv, k), "ecdsa_sign")
    return sig.raw, rid.value


def ecdsa_encode(sig64: bytes, recid: int, chain_id: int, use_new_chain_id: bool) -> bytes:
    """DefaultCrypto.SignHashed's trailer (DefaultCrypto.cs:114-136): v = chainId * 2 + 35 + recId, 1 byte (low
    byte of the int) for the old chain id, 2 bytes big-endian for the new one"""
    v = chain_id * 2 + 35 + recid
    return sig64 + ((v & 0xffff).to_bytes(2, "big") if use_new_chain_id else bytes([v & 0xff]))


def ecdsa_verify_hashed(hash32: bytes, sig: bytes, pk: bytes, use_new_chain_id: bool, chain_id: int) -> bool:
    f = lib().orc_ecdsa_verify_hashed
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                  ctypes.c_int, ctypes.c_int32]
    return bool(f(hash32, len(hash32), sig, len(sig), pk, len(pk), int(bool(use_new_chain_id)), chain_id))


def ecdsa_verify_batch(hashes: bytes, sigs: bytes, sig_len: int, pks: bytes, pk_len: int, pk_idx, n: int,
                       use_new_chain_id: bool, chain_id: int, lib_=None) -> bytes:
    import numpy as np
    L = lib_ or lib()
    idx = np.ascontiguousarray(np.asarray(pk_idx, dtype=np.int32))
    o = _buf(max(1, n))
    f = L.orc_ecdsa_verify_batch
    f.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                  ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.c_int32]
    f(o, hashes, sigs, sig_len, pks, pk_len, idx.ctypes.data, len(pks) // max(1, pk_len), n, int(bool(use_new_chain_id)),
      chain_id)
    return o.raw[:n]


def ecdsa_recover(hash32: bytes, sig64: bytes, recid: int):
    """compressed public key recovered from (hash, r || s, recid), or None"""
    o = _buf(33)
    return o.raw if lib().orc_ecdsa_recover(o, hash32, sig64, int(recid)) == 0 else None
