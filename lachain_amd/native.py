"""lachain_amd/native.py — ctypes binding of liblachain_bls.so (include/lachain_bls.h).

This is the product path: every call lands in gfx950 kernels.  There is no CPU fallback — if the
library is missing or no gfx950 device can be opened, `lib()` raises.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# LCB_LIB_PATH selects another build of the same library (A/B timing of kernel variants)
LIB_PATH = os.environ.get("LCB_LIB_PATH") or os.path.join(_HERE, "liblachain_bls.so")
MCL_BLS12_381 = 5
MCLBN_COMPILED_TIME_VAR = 46

_lib = None
_lock = threading.Lock()

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_size = ctypes.c_size_t


class mclBnFr(ctypes.Structure):
    _fields_ = [("d", ctypes.c_uint64 * 4)]


class mclBnFp(ctypes.Structure):
    _fields_ = [("d", ctypes.c_uint64 * 6)]


class mclBnFp2(ctypes.Structure):
    _fields_ = [("d", mclBnFp * 2)]


class mclBnG1(ctypes.Structure):
    _fields_ = [("x", mclBnFp), ("y", mclBnFp), ("z", mclBnFp)]


class mclBnG2(ctypes.Structure):
    _fields_ = [("x", mclBnFp2), ("y", mclBnFp2), ("z", mclBnFp2)]


class mclBnGT(ctypes.Structure):
    _fields_ = [("d", mclBnFp * 12)]


# exported symbols (also checked by tests/test_abi_exports.py against include/lachain_bls.h)
_SIGS = {
    "mclBn_init": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "lcb_set_device": (ctypes.c_int, [ctypes.c_int]),
    "lcb_get_device": (ctypes.c_int, []),
    "lcb_set_original_g2_cofactor": (None, [ctypes.c_int]),
    "lcb_set_line_mode": (ctypes.c_int, [ctypes.c_int]),
    "lcb_set_g2_sign_from_b": (ctypes.c_int, [ctypes.c_int]),
    "lcb_set_msm_chunk": (ctypes.c_int, [ctypes.c_int]),
    "lcb_set_msm_segments": (ctypes.c_int, [ctypes.c_int]),
    "lcb_set_wave_priority": (ctypes.c_int, [ctypes.c_int]),
    "lcb_last_error": (ctypes.c_char_p, []),
    "lcb_error_count": (ctypes.c_uint64, []),
    "lcb_test_inject_failure": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "lcb_set_lines_coop_max": (ctypes.c_int, [ctypes.c_int]),
    "lcb_set_keys_first": (ctypes.c_int, [ctypes.c_int]),
    "lcb_test_linesets": (ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t,
                                          ctypes.c_void_p, ctypes.c_void_p]),
    "lcb_tpke_verify_shares": (ctypes.c_int, [c_u8p, c_size, c_u8p, c_size, c_u8p, c_u8p, c_u8p, c_u32p, c_size,
                                              c_u32p, c_u32p, c_u8p]),
    "lcb_tpke_verify_shares_cached": (ctypes.c_int, [c_u8p, c_size, c_u8p, c_size, c_u8p, c_u8p, c_u8p, c_u32p, c_size,
                                                     c_u32p, c_u32p, c_u8p]),
    "lcb_tpke_verify_shares_dev": (ctypes.c_int, [ctypes.c_void_p, c_size, ctypes.c_void_p, c_size, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_size,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "lcb_tpke_prepare_dev": (ctypes.c_int, [ctypes.c_void_p, c_size, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, c_size, ctypes.c_void_p]),
    "lcb_tpke_verify_prepared_dev": (ctypes.c_int, [ctypes.c_void_p, c_size, c_size, c_size, ctypes.c_void_p,
                                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "lcb_tpke_verify_shares_batched": (ctypes.c_int, [c_u8p, c_size, c_u8p, c_size, c_u8p, c_u8p, c_u8p, c_u32p,
                                                      c_size, c_u32p, c_u32p, c_u8p]),
    "lcb_tpke_verify_shares_batched_dev": (ctypes.c_int, [ctypes.c_void_p, c_size, ctypes.c_void_p, c_size,
                                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                          ctypes.c_void_p, c_size, ctypes.c_void_p, ctypes.c_void_p,
                                                          ctypes.c_void_p, ctypes.c_void_p]),
    "lcb_tpke_verify_prepared_batched_dev": (ctypes.c_int, [ctypes.c_void_p, c_size, c_size, c_size, ctypes.c_void_p,
                                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "lcb_ts_verify_shares_batched": (ctypes.c_int, [c_u8p, c_size, c_u8p, c_size, c_u8p, c_u8p, c_u32p, c_size,
                                                    c_u32p, c_u32p]),
    "lcb_ts_verify_prepared_batched_dev": (ctypes.c_int, [ctypes.c_void_p, c_size, c_size, c_size, ctypes.c_void_p,
                                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "lcb_ts_verify_shares_batched_dev": (ctypes.c_int, [ctypes.c_void_p, c_size, ctypes.c_void_p, c_size,
                                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_size,
                                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "lcb_tpke_batched_stats": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_float)]),
    "lcb_set_batch_seed": (None, [ctypes.c_char_p]),
    "lcb_set_batch_census": (None, [c_size]),
    "lcb_set_coop_max": (ctypes.c_int, [ctypes.c_uint32]),
    "lcb_set_scratch_gate": (ctypes.c_int, [ctypes.c_longlong]),
    "lcb_scratch_gate_stats": (None, [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "lcb_scratch_info": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64)]),
    "lcb_set_persist_blocks": (ctypes.c_int, [ctypes.c_uint32]),
    "lcb_set_verify_chunk": (ctypes.c_int, [c_size]),
    "lcb_set_fork_mode": (ctypes.c_int, [ctypes.c_int]),
    "lcb_set_coop_miller_max": (ctypes.c_int, [ctypes.c_uint32]),
    "lcb_debug_coop_op": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                         c_size, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
    "lcb_debug_final_exp": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint32), c_size, ctypes.POINTER(ctypes.c_uint32),
                                           ctypes.c_int]),
    "lcb_batched_census": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint32)]),
    "lcb_tpke_partial_decrypt": (ctypes.c_int, [c_u8p, c_u8p, c_u8p, c_u8p, c_u8p, c_u8p, c_u32p, c_size]),
    "lcb_tpke_encrypt_phase1": (ctypes.c_int, [c_u8p, c_u8p, c_u8p, c_u8p, c_size]),
    "lcb_tpke_encrypt_phase2": (ctypes.c_int, [c_u8p, c_u8p, c_u8p, c_u8p, c_u32p, c_size]),
    "lcb_ts_verify_shares": (ctypes.c_int, [c_u8p, c_size, c_u8p, c_size, c_u8p, c_u8p, c_u32p, c_size, c_u32p,
                                            c_u32p]),
    "lcb_ts_verify_shares_dev": (ctypes.c_int, [ctypes.c_void_p, c_size, ctypes.c_void_p, c_size, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_void_p, c_size, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_void_p]),
    "lcb_ts_prepare_dev": (ctypes.c_int, [ctypes.c_void_p, c_size, ctypes.c_void_p, ctypes.c_void_p, c_size,
                                          ctypes.c_void_p]),
    "lcb_ts_verify_prepared_dev": (ctypes.c_int, [ctypes.c_void_p, c_size, c_size, c_size, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "lcb_ts_assemble_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           c_size, c_size, c_size, ctypes.c_void_p]),
    "lcb_g1_lagrange_dev": (ctypes.c_int, [ctypes.c_void_p] * 5 + [c_size, c_size, ctypes.c_void_p]),
    "lcb_g2_lagrange_dev": (ctypes.c_int, [ctypes.c_void_p] * 5 + [c_size, c_size, ctypes.c_void_p]),
    "lcb_tpke_partial_decrypt_prepared_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_size,
                                                             ctypes.c_void_p, c_size, ctypes.c_void_p]),
    "lcb_tpke_combine_dev": (ctypes.c_int, [ctypes.c_void_p] * 4 + [c_size, c_size, c_size, ctypes.c_void_p]),
    "lcb_tpke_combine_ordered_dev": (ctypes.c_int, [ctypes.c_void_p] * 5 + [c_size, c_size, c_size, ctypes.c_void_p]),
    "lcb_ts_assemble_ordered_dev": (ctypes.c_int, [ctypes.c_void_p] * 5 + [c_size, c_size, c_size, ctypes.c_void_p]),
    "lcb_tpke_verify_phase_ms": (ctypes.c_int, [ctypes.POINTER(ctypes.c_float)]),
    "lcb_ts_sign": (ctypes.c_int, [c_u8p, c_u8p, c_u8p, c_u32p, c_u32p, c_size]),
    "lcb_g1_lagrange_batch": (ctypes.c_int, [c_u8p, c_u8p, c_u8p, c_u8p, c_u32p, c_size]),
    "lcb_g2_lagrange_batch": (ctypes.c_int, [c_u8p, c_u8p, c_u8p, c_u8p, c_u32p, c_size]),
    "lcb_g1_msm": (ctypes.c_int, [c_u8p, c_u8p, c_u8p, c_size]),
    "lcb_g1_msm_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_size, ctypes.c_int,
                                      ctypes.c_void_p]),
    "lcb_g1_msm_window": (ctypes.c_int, [c_size]),
    "lcb_g1_msm_glv_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_size, ctypes.c_int,
                                          ctypes.c_void_p]),
    "lcb_g1_msm_glv_window": (ctypes.c_int, [c_size]),
    "lcb_g1_msm_phase_ms": (ctypes.c_int, [ctypes.POINTER(ctypes.c_float), ctypes.c_int]),
    "lcb_g1_to_affine_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_size,
                                            ctypes.c_void_p]),
    "lcb_g1_jac_sum_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_size,
                                          ctypes.c_void_p]),
    "lcb_g1_mul_batch": (ctypes.c_int, [c_u8p, c_u8p, ctypes.c_int, c_u8p, c_size]),
    "lcb_g2_mul_batch": (ctypes.c_int, [c_u8p, c_u8p, ctypes.c_int, c_u8p, c_size]),
    "lcb_g2_hash_batch": (ctypes.c_int, [c_u8p, c_u8p, c_u32p, c_size]),
    "lcb_xor_with_hash": (None, [c_u8p, c_u8p, c_u8p, c_size]),
    "lcb_coin_parity": (ctypes.c_int, [c_u8p, c_size]),
    "lcb_coin_nonce": (ctypes.c_uint64, [c_u8p, c_size]),
    "lcb_coin_fold_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_size, ctypes.c_void_p]),
    "lcb_dkg_commitment_eval": (ctypes.c_int, [c_u8p, c_u8p, c_u8p, c_size, ctypes.c_int, c_u32p,
                                               ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32), c_size]),
    "lcb_dkg_commitment_rows": (ctypes.c_int, [c_u8p, c_u8p, c_u8p, c_size, ctypes.c_int, c_u32p,
                                               ctypes.POINTER(ctypes.c_int32), c_size]),
    "lcb_g1_eval_poly_batch": (ctypes.c_int, [c_u8p, c_u8p, c_u8p, c_size, ctypes.POINTER(ctypes.c_int32), c_size]),
    "lcb_rs_encode": (ctypes.c_int, [c_u8p, c_u8p, c_size, ctypes.c_int, ctypes.c_int]),
    "lcb_rs_decode": (ctypes.c_int, [c_u8p, c_u8p, ctypes.POINTER(ctypes.c_int32), ctypes.c_int, c_size, ctypes.c_int,
                                     ctypes.c_int]),
    "lcb_queue_create": (ctypes.c_void_p, [c_size, ctypes.c_uint32]),
    "lcb_queue_destroy": (None, [ctypes.c_void_p]),
    "lcb_queue_tpke_verify": (ctypes.c_int64, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                               c_size, ctypes.c_char_p, ctypes.c_char_p]),
    "lcb_queue_ts_verify": (ctypes.c_int64, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, c_size,
                                             ctypes.c_char_p]),
    "lcb_queue_tpke_prepare": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, c_size,
                                              ctypes.c_char_p]),
    "lcb_queue_wait": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    "lcb_queue_flush": (ctypes.c_int, [ctypes.c_void_p]),
    "lcb_queue_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    "lcb_queue_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "lcb_queue_set_batched": (ctypes.c_int, [ctypes.c_void_p, c_size]),
    "lcb_ecdsa_keyset_create": (ctypes.c_void_p, [c_u8p, c_size, c_size]),
    "lcb_ecdsa_keyset_destroy": (None, [ctypes.c_void_p]),
    "lcb_ecdsa_keyset_size": (c_size, [ctypes.c_void_p]),
    "lcb_ecdsa_keyset_valid": (ctypes.c_int, [ctypes.c_void_p, c_u8p]),
    "lcb_ecdsa_verify_hashed_batch": (ctypes.c_int, [c_u8p, c_u8p, c_u8p, c_size, c_u8p, c_size, c_size,
                                                     ctypes.POINTER(ctypes.c_int32), c_size, ctypes.c_int,
                                                     ctypes.c_int32]),
    "lcb_root_header_verify_batch": (ctypes.c_int, [c_u8p, c_u8p, ctypes.c_uint64, c_u8p, c_size, c_u8p, c_size,
                                                    c_size, ctypes.POINTER(ctypes.c_int32), c_size, ctypes.c_int,
                                                    ctypes.c_int32]),
    "lcb_header_keccak_batch": (ctypes.c_int, [c_u8p, c_u8p, c_size]),
    "lcb_ecdsa_verify_hashed_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_size,
                                                   ctypes.c_void_p, c_size, ctypes.c_void_p, ctypes.c_int,
                                                   ctypes.c_int32, ctypes.c_void_p]),
    "lcb_root_header_verify_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                                  c_size, ctypes.c_void_p, c_size, ctypes.c_void_p, ctypes.c_int,
                                                  ctypes.c_int32, ctypes.c_void_p]),
    "lcb_ecdsa_phase_ms": (ctypes.c_int, [ctypes.POINTER(ctypes.c_float)]),
    "lcb_ecdsa_pubkey_batch": (ctypes.c_int, [c_u8p, c_u8p, c_u8p, c_size]),
    "lcb_ecdsa_sign_hashed_batch": (ctypes.c_int, [c_u8p, c_u8p, c_u8p, c_u8p, c_u8p, c_size, ctypes.c_int,
                                                   ctypes.c_int32]),
    "lcb_ecdsa_pubkey_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_size, ctypes.c_void_p]),
    "lcb_ecdsa_sign_hashed_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, c_size, ctypes.c_int, ctypes.c_int32,
                                                 ctypes.c_void_p]),
    "lcb_ctx_create": (ctypes.c_void_p, []),
    "lcb_ctx_destroy": (None, [ctypes.c_void_p]),
    "lcb_ctx_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
}
# explicit-context forms: the context pointer first, then the same arguments as the context-less form
for _name in ("tpke_prepare_dev", "tpke_verify_prepared_dev", "tpke_verify_prepared_batched_dev", "tpke_batched_stats",
              "tpke_verify_shares_batched_dev", "ts_verify_prepared_batched_dev", "ts_verify_shares_batched_dev", "tpke_partial_decrypt_prepared_dev", "tpke_combine_dev",
              "tpke_verify_phase_ms", "ts_prepare_dev", "ts_verify_prepared_dev", "ts_assemble_dev", "g1_lagrange_dev",
              "g2_lagrange_dev", "g1_msm_dev", "g1_msm_glv_dev", "g1_msm_phase_ms", "g1_jac_sum_dev", "ecdsa_verify_hashed_dev",
              "root_header_verify_dev", "ecdsa_pubkey_dev", "ecdsa_sign_hashed_dev", "ecdsa_phase_ms", "batched_census",
              "tpke_combine_ordered_dev", "ts_assemble_ordered_dev"):
    _res, _args = _SIGS["lcb_" + _name]
    _SIGS["lcb_ctx_" + _name] = (_res, [ctypes.c_void_p] + list(_args))


def load(check_device=True):
    """Load the shared library; with check_device, also initialise the GPU (mclBn_init)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"{LIB_PATH} is not built (run __graft_entry__.build() or make -C lachain_amd/csrc)")
            lib_ = ctypes.CDLL(LIB_PATH)
            ab = bool(os.environ.get("LCB_LIB_PATH"))
            for name, (res, args) in _SIGS.items():
                try:
                    fn = getattr(lib_, name)
                except AttributeError:
                    if ab:          # an A/B build of an earlier revision may lack newer entry points
                        continue
                    raise
                fn.restype = res
                fn.argtypes = args
            _lib = lib_
        if check_device and not getattr(_lib, "_inited", False):
            rc = _lib.mclBn_init(MCL_BLS12_381, MCLBN_COMPILED_TIME_VAR)
            if rc != 0:
                raise RuntimeError("liblachain_bls: mclBn_init failed: " + _lib.lcb_last_error().decode())
            _lib._inited = True
    return _lib


def lib():
    return load(True)


def last_error():
    return lib().lcb_last_error().decode()


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"liblachain_bls {what} failed: {last_error()}")


def _bytes_ptr(b):
    """ctypes uint8 pointer to an immutable bytes object (read-only use)."""
    if not isinstance(b, (bytes, bytearray)):
        b = bytes(b)
    buf = (ctypes.c_uint8 * max(1, len(b))).from_buffer_copy(b if len(b) else b"\0")
    return buf, ctypes.cast(buf, c_u8p)


def _u32_ptr(vals):
    arr = (ctypes.c_uint32 * max(1, len(vals)))(*vals)
    return arr, ctypes.cast(arr, c_u32p)


def _out(n):
    buf = (ctypes.c_uint8 * max(1, n))()
    return buf, ctypes.cast(buf, c_u8p)


def _offsets(chunks):
    off = [0]
    for c in chunks:
        off.append(off[-1] + len(c))
    return off


# ---------------------------------------------------------------- batch wrappers (bytes in / bytes out)
def tpke_verify_shares(y_keys, cts, shares, batched=False, cached=False):
    """y_keys: list of 48-byte verification keys; cts: list of (U48, V, W96);
    shares: list of (ct_index, decryptor_index, Ui48).  Returns list of bools.  batched=True runs the randomized
    group check (lcb_tpke_verify_shares_batched: same decisions, false accept <= 2^-64 per group)."""
    n = len(shares)
    keep = []
    _, py = _bytes_ptr_keep(keep, b"".join(y_keys))
    _, pu = _bytes_ptr_keep(keep, b"".join(c[0] for c in cts))
    _, pw = _bytes_ptr_keep(keep, b"".join(c[2] for c in cts))
    _, pv = _bytes_ptr_keep(keep, b"".join(c[1] for c in cts))
    _, pvo = _u32_keep(keep, _offsets([c[1] for c in cts]))
    _, pct = _u32_keep(keep, [s[0] for s in shares])
    _, pdec = _u32_keep(keep, [s[1] for s in shares])
    _, pui = _bytes_ptr_keep(keep, b"".join(s[2] for s in shares))
    ob, po = _out(n)
    fn = (lib().lcb_tpke_verify_shares_batched if batched else
          lib().lcb_tpke_verify_shares_cached if cached else lib().lcb_tpke_verify_shares)
    _check(fn(po, n, py, len(y_keys), pu, pw, pv, pvo, len(cts), pct, pdec, pui), "tpke_verify_shares")
    return [bool(ob[i]) for i in range(n)]


def _bytes_ptr_keep(keep, b):
    buf, p = _bytes_ptr(b)
    keep.append(buf)
    return buf, p


def _u32_keep(keep, vals):
    arr, p = _u32_ptr(vals)
    keep.append(arr)
    return arr, p


def tpke_partial_decrypt(x32, cts):
    """cts: list of (U, V, W).  Returns list of (ok, Ui48)."""
    keep = []
    n = len(cts)
    _, px = _bytes_ptr_keep(keep, x32)
    _, pu = _bytes_ptr_keep(keep, b"".join(c[0] for c in cts))
    _, pw = _bytes_ptr_keep(keep, b"".join(c[2] for c in cts))
    _, pv = _bytes_ptr_keep(keep, b"".join(c[1] for c in cts))
    _, pvo = _u32_keep(keep, _offsets([c[1] for c in cts]))
    ob, po = _out(48 * n)
    sb, ps = _out(n)
    _check(lib().lcb_tpke_partial_decrypt(po, ps, px, pu, pw, pv, pvo, n), "tpke_partial_decrypt")
    raw = bytes(ob)
    return [(bool(sb[i]), raw[48 * i:48 * i + 48]) for i in range(n)]


def tpke_encrypt_phase1(y48, rs):
    keep = []
    n = len(rs)
    _, py = _bytes_ptr_keep(keep, y48)
    _, pr = _bytes_ptr_keep(keep, b"".join(rs))
    ub, pu = _out(48 * n)
    tb, pt = _out(48 * n)
    _check(lib().lcb_tpke_encrypt_phase1(pu, pt, py, pr, n), "tpke_encrypt_phase1")
    u, t = bytes(ub), bytes(tb)
    return [u[48 * i:48 * i + 48] for i in range(n)], [t[48 * i:48 * i + 48] for i in range(n)]


def tpke_encrypt_phase2(us, rs, vs):
    keep = []
    n = len(us)
    _, pu = _bytes_ptr_keep(keep, b"".join(us))
    _, pr = _bytes_ptr_keep(keep, b"".join(rs))
    _, pv = _bytes_ptr_keep(keep, b"".join(vs))
    _, pvo = _u32_keep(keep, _offsets(vs))
    wb, pw = _out(96 * n)
    _check(lib().lcb_tpke_encrypt_phase2(pw, pu, pr, pv, pvo, n), "tpke_encrypt_phase2")
    w = bytes(wb)
    return [w[96 * i:96 * i + 96] for i in range(n)]


def ts_verify_shares(pks, msgs, items, batched=False):
    """pks: list of 48-byte keys; msgs: list of bytes; items: list of (msg_index, pk_index, sig96).  batched=True runs
    the randomized group check (lcb_ts_verify_shares_batched)."""
    keep = []
    n = len(items)
    _, ppk = _bytes_ptr_keep(keep, b"".join(pks))
    _, psig = _bytes_ptr_keep(keep, b"".join(it[2] for it in items))
    _, pm = _bytes_ptr_keep(keep, b"".join(msgs))
    _, pmo = _u32_keep(keep, _offsets(msgs))
    _, pmi = _u32_keep(keep, [it[0] for it in items])
    _, ppi = _u32_keep(keep, [it[1] for it in items])
    ob, po = _out(n)
    fn = lib().lcb_ts_verify_shares_batched if batched else lib().lcb_ts_verify_shares
    _check(fn(po, n, ppk, len(pks), psig, pm, pmo, len(msgs), pmi, ppi), "ts_verify_shares")
    return [bool(ob[i]) for i in range(n)]


def ts_sign(sks, msgs, msg_idx):
    keep = []
    n = len(sks)
    _, psk = _bytes_ptr_keep(keep, b"".join(sks))
    _, pm = _bytes_ptr_keep(keep, b"".join(msgs))
    _, pmo = _u32_keep(keep, _offsets(msgs))
    _, pmi = _u32_keep(keep, msg_idx)
    ob, po = _out(96 * n)
    _check(lib().lcb_ts_sign(po, psk, pm, pmo, pmi, n), "ts_sign")
    o = bytes(ob)
    return [o[96 * i:96 * i + 96] for i in range(n)]


def lagrange_batch(group, problems):
    """group 1 or 2; problems: list of (xs: list of Fr32, ys: list of points).  Returns list of point|None."""
    keep = []
    pb = 48 if group == 1 else 96
    xs = [x for xs_, _ in problems for x in xs_]
    ys = [y for _, ys_ in problems for y in ys_]
    off = [0]
    for xs_, _ in problems:
        off.append(off[-1] + len(xs_))
    _, px = _bytes_ptr_keep(keep, b"".join(xs))
    _, py = _bytes_ptr_keep(keep, b"".join(ys))
    _, poff = _u32_keep(keep, off)
    np_ = len(problems)
    ob, po = _out(pb * np_)
    sb, ps = _out(np_)
    fn = lib().lcb_g1_lagrange_batch if group == 1 else lib().lcb_g2_lagrange_batch
    _check(fn(po, ps, px, py, poff, np_), "lagrange_batch")
    o = bytes(ob)
    return [o[pb * j:pb * j + pb] if sb[j] else None for j in range(np_)]


def g1_msm(points, scalars):
    keep = []
    _, pp = _bytes_ptr_keep(keep, b"".join(points))
    _, ps = _bytes_ptr_keep(keep, b"".join(scalars))
    ob, po = _out(48)
    _check(lib().lcb_g1_msm(po, pp, ps, len(points)), "g1_msm")
    return bytes(ob)


MSM_PHASES = ("digits", "sort", "bounds", "bucket_acc", "bucket_reduce", "combine")


def msm_phase_ms():
    """Device time (ms) of each phase of the last MSM (lcb_g1_msm_phase_ms)."""
    arr = (ctypes.c_float * len(MSM_PHASES))()
    _check(lib().lcb_g1_msm_phase_ms(arr, len(MSM_PHASES)), "msm_phase_ms")
    return dict(zip(MSM_PHASES, list(arr)))


def mul_batch(group, points, scalars, generator=False):
    keep = []
    pb = 48 if group == 1 else 96
    n = len(scalars)
    _, pp = _bytes_ptr_keep(keep, b"".join(points) if not generator else b"\0")
    _, ps = _bytes_ptr_keep(keep, b"".join(scalars))
    ob, po = _out(pb * n)
    fn = lib().lcb_g1_mul_batch if group == 1 else lib().lcb_g2_mul_batch
    _check(fn(po, pp, 1 if generator else 0, ps, n), "mul_batch")
    o = bytes(ob)
    return [o[pb * i:pb * i + pb] for i in range(n)]


def mul_batch_raw(group, points: bytes, scalars: bytes, n: int, generator=False) -> bytes:
    """Like mul_batch but with concatenated inputs/outputs (bulk synthetic-input generation)."""
    keep = []
    pb = 48 if group == 1 else 96
    _, pp = _bytes_ptr_keep(keep, points if not generator else b"\0")
    _, ps = _bytes_ptr_keep(keep, scalars)
    ob, po = _out(pb * n)
    fn = lib().lcb_g1_mul_batch if group == 1 else lib().lcb_g2_mul_batch
    _check(fn(po, pp, 1 if generator else 0, ps, n), "mul_batch")
    return bytes(ob)


def g2_hash_batch(msgs):
    keep = []
    n = len(msgs)
    _, pm = _bytes_ptr_keep(keep, b"".join(msgs))
    _, pmo = _u32_keep(keep, _offsets(msgs))
    ob, po = _out(96 * n)
    _check(lib().lcb_g2_hash_batch(po, pm, pmo, n), "g2_hash_batch")
    o = bytes(ob)
    return [o[96 * i:96 * i + 96] for i in range(n)]


def xor_with_hash(g1_48, data):
    keep = []
    _, pg = _bytes_ptr_keep(keep, g1_48)
    _, pd = _bytes_ptr_keep(keep, data)
    ob, po = _out(len(data))
    load(False).lcb_xor_with_hash(po, pg, pd, len(data))
    return bytes(ob)[: len(data)]


def _i32_keep(keep, vals):
    arr = (ctypes.c_int32 * max(1, len(vals)))(*vals)
    keep.append(arr)
    return ctypes.cast(arr, ctypes.POINTER(ctypes.c_int32))


def dkg_commitment_eval(commitments, degree, queries):
    """commitments: list of coefficient lists (serialized G1, Commitment's Index order); queries: (comm, x, y).
    -> list of 48-byte Commitment.Evaluate(x, y) or None (malformed)."""
    keep = []
    _, pc = _bytes_ptr_keep(keep, b"".join(b"".join(c) for c in commitments))
    _, pi = _u32_keep(keep, [q[0] for q in queries])
    px, py = _i32_keep(keep, [q[1] for q in queries]), _i32_keep(keep, [q[2] for q in queries])
    n = len(queries)
    ob, po = _out(48 * n)
    sb, ps = _out(n)
    _check(lib().lcb_dkg_commitment_eval(po, ps, pc, len(commitments), degree, pi, px, py, n), "dkg_commitment_eval")
    o = bytes(ob)
    return [o[48 * q:48 * q + 48] if sb[q] else None for q in range(n)]


def dkg_commitment_rows(commitments, degree, queries):
    """queries: (comm, x) -> list of degree+1 points (Commitment.Evaluate(x)) or None"""
    keep = []
    _, pc = _bytes_ptr_keep(keep, b"".join(b"".join(c) for c in commitments))
    _, pi = _u32_keep(keep, [q[0] for q in queries])
    px = _i32_keep(keep, [q[1] for q in queries])
    n, w = len(queries), degree + 1
    ob, po = _out(48 * n * w)
    sb, ps = _out(n)
    _check(lib().lcb_dkg_commitment_rows(po, ps, pc, len(commitments), degree, pi, px, n), "dkg_commitment_rows")
    o = bytes(ob)
    return [[o[48 * (q * w + i):48 * (q * w + i) + 48] for i in range(w)] if sb[q] else None for q in range(n)]


def g1_eval_poly_batch(coeffs, xs):
    keep = []
    _, pc = _bytes_ptr_keep(keep, b"".join(coeffs))
    px = _i32_keep(keep, xs)
    ob, po = _out(48 * len(xs))
    sb, ps = _out(len(xs))
    _check(lib().lcb_g1_eval_poly_batch(po, ps, pc, len(coeffs), px, len(xs)), "g1_eval_poly_batch")
    o = bytes(ob)
    return [o[48 * q:48 * q + 48] if sb[q] else None for q in range(len(xs))]


def rs_encode(data: bytes, n_shards: int, erasures: int) -> bytes:
    """ReliableBroadcast.ErasureCodingShards: all shards concatenated (len(data) divisible by the data shards)"""
    keep = []
    _, pd = _bytes_ptr_keep(keep, data)
    k = n_shards - erasures
    ob, po = _out(len(data) // k * n_shards if k > 0 else 0)
    _check(lib().lcb_rs_encode(po, pd, len(data), n_shards, erasures), "rs_encode")
    return bytes(ob)[: len(data) // k * n_shards]


def rs_decode(echos, shard_size: int, n_shards: int, erasures: int) -> bytes:
    """ReliableBroadcast.DecodeFromEchos: echos = [(from, shard bytes)] -> all shards concatenated"""
    keep = []
    _, pd = _bytes_ptr_keep(keep, b"".join(e[1] for e in echos))
    pf = _i32_keep(keep, [e[0] for e in echos])
    ob, po = _out(shard_size * n_shards)
    _check(lib().lcb_rs_decode(po, pd, pf, len(echos), shard_size, n_shards, erasures), "rs_decode")
    return bytes(ob)[: shard_size * n_shards]


# ---------------------------------------------------------------- secp256k1 ECDSA header signatures (§8f row 4)
def header_bytes(index: int, prev: bytes, merkle: bytes, state: bytes, nonce: int) -> bytes:
    """lcb_block_header record (112 B): u64 index | prev_block_hash | merkle_root | state_hash | u64 nonce"""
    assert len(prev) == len(merkle) == len(state) == 32
    return index.to_bytes(8, "little") + prev + merkle + state + nonce.to_bytes(8, "little")


def header_keccak_batch(headers: bytes) -> bytes:
    """HashUtils.Keccak(BlockHeader) of each 112-byte record"""
    n = len(headers) // 112
    keep = []
    _, ph = _bytes_ptr_keep(keep, headers)
    ob, po = _out(32 * n)
    _check(lib().lcb_header_keccak_batch(po, ph, n), "header_keccak_batch")
    return bytes(ob)[: 32 * n]


def ecdsa_verify_hashed_batch(hashes: bytes, sigs: bytes, sig_len: int, pubkeys: bytes, pk_len: int, key_idx,
                              use_new_chain_id: bool, chain_id: int) -> bytes:
    """DefaultCrypto.VerifySignatureHashed over a batch: one accept byte per signature"""
    n = len(hashes) // 32
    keep = []
    _, ph = _bytes_ptr_keep(keep, hashes)
    _, ps = _bytes_ptr_keep(keep, sigs)
    _, pk = _bytes_ptr_keep(keep, pubkeys)
    pi = _i32_keep(keep, key_idx)
    ob, po = _out(n)
    _check(lib().lcb_ecdsa_verify_hashed_batch(po, ph, ps, sig_len, pk, pk_len, len(pubkeys) // pk_len, pi, n,
                                               int(bool(use_new_chain_id)), chain_id), "ecdsa_verify_hashed_batch")
    return bytes(ob)[:n]


def root_header_verify_batch(headers: bytes, era: int, sigs: bytes, sig_len: int, pubkeys: bytes, pk_len: int, key_idx,
                             use_new_chain_id: bool, chain_id: int) -> bytes:
    """RootProtocol's SignedHeaderMessage check (index == era, header Keccak, VerifySignatureHashed)"""
    n = len(headers) // 112
    keep = []
    _, ph = _bytes_ptr_keep(keep, headers)
    _, ps = _bytes_ptr_keep(keep, sigs)
    _, pk = _bytes_ptr_keep(keep, pubkeys)
    pi = _i32_keep(keep, key_idx)
    ob, po = _out(n)
    _check(lib().lcb_root_header_verify_batch(po, ph, era, ps, sig_len, pk, pk_len, len(pubkeys) // pk_len, pi, n,
                                              int(bool(use_new_chain_id)), chain_id), "root_header_verify_batch")
    return bytes(ob)[:n]


def ecdsa_pubkey_batch(privs: bytes):
    """(compressed keys, ok) for 32-byte big-endian private keys"""
    n = len(privs) // 32
    keep = []
    _, pp = _bytes_ptr_keep(keep, privs)
    ob, po = _out(33 * n)
    okb, pok = _out(n)
    _check(lib().lcb_ecdsa_pubkey_batch(po, pok, pp, n), "ecdsa_pubkey_batch")
    return bytes(ob)[: 33 * n], bytes(okb)[:n]


def ecdsa_sign_hashed_batch(hashes: bytes, privs: bytes, nonces: bytes, use_new_chain_id: bool, chain_id: int):
    """(signatures, ok): r || s || v per DefaultCrypto.SignHashed's encoding, with the given nonces"""
    n = len(hashes) // 32
    L = 66 if use_new_chain_id else 65
    keep = []
    _, ph = _bytes_ptr_keep(keep, hashes)
    _, pp = _bytes_ptr_keep(keep, privs)
    _, pn = _bytes_ptr_keep(keep, nonces)
    ob, po = _out(L * n)
    okb, pok = _out(n)
    _check(lib().lcb_ecdsa_sign_hashed_batch(po, pok, ph, pp, pn, n, int(bool(use_new_chain_id)), chain_id),
           "ecdsa_sign_hashed_batch")
    return bytes(ob)[: L * n], bytes(okb)[:n]


class EcdsaKeySet:
    """lcb_ecdsa_keyset: validator keys resident on the device with their comb tables"""

    def __init__(self, pubkeys: bytes, pk_len: int):
        keep = []
        _, pk = _bytes_ptr_keep(keep, pubkeys)
        self.n = len(pubkeys) // pk_len
        self.h = lib().lcb_ecdsa_keyset_create(pk, pk_len, self.n)
        if not self.h:
            raise RuntimeError("lcb_ecdsa_keyset_create: " + lib().lcb_last_error().decode())

    def valid(self) -> bytes:
        ob, po = _out(self.n)
        _check(lib().lcb_ecdsa_keyset_valid(self.h, po), "keyset_valid")
        return bytes(ob)[: self.n]

    def close(self):
        if self.h:
            lib().lcb_ecdsa_keyset_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def coin_parity(sig: bytes) -> bool:
    """CoinResult.Parity of the combined signature bytes (src/Lachain.Consensus/CommonCoin/CoinResult.cs:16-20)."""
    keep = []
    _, p = _bytes_ptr_keep(keep, sig)
    return bool(load(False).lcb_coin_parity(p, len(sig)))


def coin_nonce(sig: bytes) -> int:
    """RootProtocol.GetNonceFromCoin (src/Lachain.Consensus/RootProtocol/RootProtocol.cs:316-322)."""
    keep = []
    _, p = _bytes_ptr_keep(keep, sig)
    return int(load(False).lcb_coin_nonce(p, len(sig)))


class BatchQueue:
    """lcb_queue (include/lachain_bls.h): single shares submitted from many threads run as aggregated GPU batches.

    submit_* return a ticket; wait(ticket) -> True / False (the share's decision); verify_* = submit + wait, the
    drop-in shape of PublicKey.VerifyShare (TPKE/PublicKey.cs:88-92) and ValidateSignature
    (ThresholdSignature/PublicKey.cs:16-21) for one-share-per-call callers."""

    def __init__(self, max_batch=4096, max_delay_ms=5.0, batched_min=0):
        self.ptr = lib().lcb_queue_create(max_batch, int(max_delay_ms * 1000))
        if not self.ptr:
            raise RuntimeError("lcb_queue_create failed")
        if batched_min:
            _check(lib().lcb_queue_set_batched(self.ptr, batched_min), "queue_set_batched")

    def submit_tpke(self, y48, u48, v, w96, ui48):
        t = lib().lcb_queue_tpke_verify(self.ptr, y48, u48, v, len(v), w96, ui48)
        if t <= 0:
            raise ValueError("lcb_queue_tpke_verify: bad arguments")
        return t

    def prepare_tpke(self, u48, v, w96):
        """prepare a ciphertext ahead of its shares (lcb_queue_tpke_prepare; HoneyBadger.cs:144-146 decrypts every
        ciphertext of the common subset before the other validators' shares for it arrive)"""
        if len(u48) != 48 or len(w96) != 96:
            raise ValueError("lcb_queue_tpke_prepare: U is 48 bytes, W 96")
        if lib().lcb_queue_tpke_prepare(self.ptr, u48, v, len(v), w96) != 0:
            raise ValueError("lcb_queue_tpke_prepare: bad arguments")

    def submit_ts(self, pk48, msg, sig96):
        t = lib().lcb_queue_ts_verify(self.ptr, pk48, msg, len(msg), sig96)
        if t <= 0:
            raise ValueError("lcb_queue_ts_verify: bad arguments")
        return t

    def wait(self, ticket) -> bool:
        r = lib().lcb_queue_wait(self.ptr, ticket)
        if r < 0:
            raise RuntimeError("lcb_queue batch failed: " + lib().lcb_queue_last_error(self.ptr).decode())
        return bool(r)

    def verify_tpke(self, y48, u48, v, w96, ui48) -> bool:
        return self.wait(self.submit_tpke(y48, u48, v, w96, ui48))

    def verify_ts(self, pk48, msg, sig96) -> bool:
        return self.wait(self.submit_ts(pk48, msg, sig96))

    def flush(self):
        lib().lcb_queue_flush(self.ptr)

    def stats(self):
        arr = (ctypes.c_uint64 * 3)()
        lib().lcb_queue_stats(self.ptr, arr)
        return dict(batches=int(arr[0]), shares=int(arr[1]), largest_batch=int(arr[2]))

    def close(self):
        if self.ptr:
            lib().lcb_queue_destroy(self.ptr)
            self.ptr = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class Context:
    """An explicit lcb_ctx (include/lachain_bls.h): private device workspaces, enqueue-ordered across streams."""

    def __init__(self):
        self.ptr = lib().lcb_ctx_create()
        if not self.ptr:
            raise RuntimeError("lcb_ctx_create failed: " + last_error())

    def synchronize(self):
        _check(lib().lcb_ctx_synchronize(self.ptr), "ctx_synchronize")

    def close(self):
        if self.ptr:
            lib().lcb_ctx_destroy(self.ptr)
            self.ptr = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def set_g2_sign_from_b(use_b):
    """the G2 wire flag's convention (include/lachain_bls.h lcb_set_g2_sign_from_b): parity of y.b instead of y.a"""
    _check(lib().lcb_set_g2_sign_from_b(1 if use_b else 0), "set_g2_sign_from_b")


def set_original_g2_cofactor(enable):
    lib().lcb_set_original_g2_cofactor(1 if enable else 0)


def set_batch_seed(seed32=None):
    """fixed ChaCha20 key for the batched verify's exponents (None: getrandom per call); the library honours it only
    when the process environment has LCB_ALLOW_FIXED_BATCH_SEED=1"""
    lib().lcb_set_batch_seed(seed32)


def set_batch_census(min_shares):
    """batched calls of >= min_shares shares start with the census of suspect keys (0 = never; default 16384)"""
    lib().lcb_set_batch_census(min_shares)


def _tuning(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: {last_error()} (tuning hooks are opt-in: LCB_ALLOW_TUNING=1)")


def error_count():
    """failures recorded on the calling thread (lcb_error_count): how the void mcl calls report failure"""
    return int(lib().lcb_error_count())


def inject_failure(site, count=1):
    """test hook (LCB_ALLOW_TEST_HOOKS=1): the next `count` passes through fault site `site` fail"""
    if lib().lcb_test_inject_failure(int(site), int(count)) != 0:
        raise RuntimeError("inject_failure: " + last_error())


def test_linesets(points, coop, force=None):
    """test hook (LCB_ALLOW_TEST_HOOKS=1): the line sets of G2 wire points on the five-lane (coop) or one-lane kernel;
    returns (uint32 array [n, 6592], the G2 flags of the odd-indexed points)"""
    import numpy as np
    n = len(points)
    force = bytes(force) if force is not None else bytes(n)
    out = np.zeros((n, 6592), dtype=np.uint32)
    g2f = np.zeros(max(1, n // 2), dtype=np.uint8)
    mode = coop if isinstance(coop, int) and not isinstance(coop, bool) else (1 if coop else 0)   # 2: the two-wave instance
    if lib().lcb_test_linesets(mode, b"".join(points), force, n, out.ctypes.data, g2f.ctypes.data) != 0:
        raise RuntimeError("test_linesets: " + last_error())
    return out, g2f[: n // 2]


def set_lines_coop_max(max_sets):
    """line sets of up to max_sets points per preparation on the five-lane kernel (-1: default)"""
    _tuning(lib().lcb_set_lines_coop_max(int(max_sets)), "set_lines_coop_max")


def set_keys_first(on):
    """fused batched calls: the key tables before the preparation fork (default on)"""
    _tuning(lib().lcb_set_keys_first(1 if on else 0), "set_keys_first")


def set_wave_priority(on):
    """latency-bound batched-check kernels at raised wave priority (default on)"""
    _tuning(lib().lcb_set_wave_priority(1 if on else 0), "set_wave_priority")


def set_msm_segments(max_segments):
    """MSM bucket-reduction lanes: the fewest segments up to max_segments (0: default rule)"""
    _tuning(lib().lcb_set_msm_segments(int(max_segments)), "set_msm_segments")


def set_msm_chunk(records_per_lane):
    """records per lane of the MSM bucket accumulation (0: one lane per bucket)"""
    _tuning(lib().lcb_set_msm_chunk(int(records_per_lane)), "set_msm_chunk")


def set_scratch_gate(nbytes):
    """launches whose full-device scratch exceeds nbytes run on the device's gate stream (-1 = off, 0 = every launch
    with scratch, < -1 = the model's per-queue share): include/lachain_bls.h lcb_set_scratch_gate"""
    _tuning(lib().lcb_set_scratch_gate(int(nbytes)), "set_scratch_gate")


def scratch_info():
    """the device's scratch model: dict(pool, bind_limit, slots, queues, per_queue, threshold) (lcb_scratch_info)"""
    out = (ctypes.c_uint64 * 6)()
    if lib().lcb_scratch_info(out) != 0:
        raise RuntimeError("lcb_scratch_info failed")
    keys = ("pool", "bind_limit", "slots", "queues", "per_queue", "threshold")
    return dict(zip(keys, (int(v) for v in out)))


def scratch_gate_stats():
    """(launches routed through the scratch gate, launches checked) since the process started"""
    a, b = ctypes.c_uint64(), ctypes.c_uint64()
    lib().lcb_scratch_gate_stats(ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def set_persist_blocks(max_blocks):
    """at most max_blocks blocks in the persistent table-walking grids (0 = as many as are resident)"""
    _tuning(lib().lcb_set_persist_blocks(int(max_blocks)), "set_persist_blocks")


def set_verify_chunk(checks):
    """checks per Miller + final-exponentiation launch pair (default 2^21; a test hook for chunk offsets)"""
    _tuning(lib().lcb_set_verify_chunk(int(checks)), "set_verify_chunk")


def set_coop_max(max_checks):
    """levels of <= max_checks group checks use the nine-lane cooperative kernels (0 = never; default 32768)"""
    _tuning(lib().lcb_set_coop_max(max_checks), "set_coop_max")


def set_coop_miller_max(max_checks):
    """levels of <= max_checks group checks run their Miller loops on the cooperative kernels"""
    _tuning(lib().lcb_set_coop_miller_max(max_checks), "set_coop_miller_max")


def set_fork_mode(mode):
    """stream layout of the fused batched verify (include/lachain_bls.h lcb_set_fork_mode): 0 = randomisation on a
    second stream, 1 = preparation chain on a high-priority stream, 2 = 1 with the preparation enqueued first,
    3 = 2 with the TPKE preparation split into hash / decode lanes on two more high-priority streams, 4 (default) = the
    split lanes in one dispatch on the one high-priority stream (one hardware queue per priority per context)"""
    _tuning(lib().lcb_set_fork_mode(mode), "set_fork_mode")


def debug_final_exp(values, coop):
    """final exponentiation of Fp12 values given as 144 u32 words each (Montgomery form) by the one-lane (coop=False)
    or the nine-lane (coop=True) kernel; returns the 144-word results"""
    n = len(values)
    a = (ctypes.c_uint32 * (144 * n))(*[w for v in values for w in v])
    out = (ctypes.c_uint32 * (144 * n))()
    _check(lib().lcb_debug_final_exp(a, n, out, 1 if coop else 0), "debug_final_exp")
    return [list(out[144 * i:144 * i + 144]) for i in range(n)]


def debug_coop_op(op, a_values, b_values):
    """one cooperative Fp12 operation (lcb_debug_coop_op) -> (cooperative results, one-lane results)"""
    n = len(a_values)
    a = (ctypes.c_uint32 * (144 * n))(*[w for v in a_values for w in v])
    b = (ctypes.c_uint32 * (144 * n))(*[w for v in b_values for w in v])
    out = (ctypes.c_uint32 * (144 * n))()
    ref = (ctypes.c_uint32 * (144 * n))()
    _check(lib().lcb_debug_coop_op(op, a, b, n, out, ref), "debug_coop_op")
    return ([list(out[144 * i:144 * i + 144]) for i in range(n)], [list(ref[144 * i:144 * i + 144]) for i in range(n)])


def batched_census():
    """{census shares, suspect keys, level-1 groups, level-1 entries after the split} of this thread's last batched
    verify"""
    out = (ctypes.c_uint32 * 4)()
    _check(lib().lcb_batched_census(out), "batched_census")
    return list(out)


def tpke_batched_stats():
    lv = (ctypes.c_uint32 * 8)()
    ms = (ctypes.c_float * 6)()
    k = lib().lcb_tpke_batched_stats(lv, ms)
    _check(0 if k >= 0 else k, "tpke_batched_stats")
    return list(lv[:k]), tuple(ms)


def set_line_mode(general):
    """general=True: later prepares mark every line set un-normalised, so the Miller loops take the on-the-fly
    fallback (pairing.hpp miller2_sets_fallback); False restores the normalised default"""
    _tuning(lib().lcb_set_line_mode(1 if general else 0), "set_line_mode")
