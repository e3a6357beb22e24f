#!/usr/bin/env python3
"""bench.py — BASELINE.json metric on MI355X: batched TPKE decryption-share verifications per second.

Workload (BASELINE.json configs[1]): 1,048,576 decryption shares of N=22, F=7
validators = 47,663 ciphertexts x 22 decryptors (the last ciphertext carries 12 shares), V = 32 bytes,
DKG-style keys of degree F, 1 % of shares corrupted (U_i + G) so the reject path is exercised.
One "step" = one pass of the hot path over the whole batch, inputs resident in HBM:
  lcb_tpke_prepare_dev          (k_g1_decompress: 22 keys; k_tpke_ct_prepare: per-ciphertext H(U||V) +
                                 Miller lines of H and W)
  lcb_tpke_verify_prepared_dev  (k_tpke_verify: per share, decompress U_i, 2-pair Miller loop, final exp)
Second line of the metric (BASELINE configs[3]): G1 Pippenger MSMs of 2^20 and 2^24 points in total, each
sharded over the ranks, reported under "msm" in the same JSON line with their own roofline and CPU baseline;
at N > 1 the per-GPU Jacobian partials are all-gathered over RCCL and summed on the GPU.
Launch: `python bench.py --gpus 1` or under torch.distributed.run with --gpus N (one rank per GPU, weak
scaling: every rank verifies its own 1M-share batch; no data-path collective).
Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
from lachain_amd import shard  # noqa: E402  (host-side partition / cross-rank reduction helpers, no GPU work)

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
SEED = 0x4C61636861696E

# Canonical Fp-mul counts (oracle/bls.c:orc_count_units; frozen in BASELINE.md §3) and MACs per Fp-mul
C = dict(C_ML1_EVAL=5192, C_ML2_EVAL=8116, C_LINES=2012, C_FE=8603, C_H2G2=7266, C_DEC1=611, C_DEC2=1837,
         C_MUL1=2835, C_MUL2=6908, C_AFF2=625)
MAC_PER_FPMUL = 300                      # 12x12 (a*b) + 12x12 (m*p) + 12 (m) 32-bit MACs, CIOS/FIPS Montgomery
# Round 2: precomputed line sets are normalised to A = 1 (pairing.hpp lineset_compute), so a line product costs
# 9 instead of 13 Fp2 products (-12 Fp-mul per line, 68 lines per set); normalising a set costs one Fp2
# inversion (C_FP2_INV) + 68 x (1 prefix product + 4 backward products) Fp2 products (3 Fp-mul each).
C["C_FP2_INV"] = 2 + 463 + 2 + 2                                      # norm, Fp inversion, 2 x (Fp2 x Fp)
C["C_NORM"] = C["C_FP2_INV"] + 68 * 5 * 3                            # per line set
# Round 2f: G2 decompression takes its square root with two exponentiations (field.hpp fp2_sqrt_any) instead of the
# mcl-order root measured above (sqrt of the norm, one or two Fp roots, an inversion): x^3 + b 5, norm 2, two
# exponentiations 2 x 463 + 1 check, c, u, b s / 2, c s 6, the y^2 == x check 2, parity 1
C["C_DEC2"] = 5 + 2 + 2 * 463 + 1 + 6 + 2 + 1
C["C_ML2_NORM2"] = C["C_ML2_EVAL"] - 2 * 68 * 12                     # TPKE: both sets normalised
C["C_ML2_NORM1"] = C["C_ML2_EVAL"] - 68 * 12                         # TS: message set normalised, share lines on the fly
W_VERIFY = C["C_DEC1"] + C["C_ML2_NORM2"] + C["C_FE"]                                  # per share
W_PREPARE = (C["C_DEC1"] + C["C_DEC2"] + C["C_H2G2"] + C["C_AFF2"] + 2 * C["C_LINES"]
             + 2 * C["C_NORM"])                                                        # per ciphertext
# gfx950 v_mad_u64_u32 is half rate: 64 lane-MACs / clk / CU (profiles/r01_valu_rates.jsonl)
PEAK_MAC32 = 256 * 64 * 2.4e9            # 3.93e13 MAC/s at the 2.4 GHz max clock
_T_START = time.perf_counter()


def progress(msg):
    """One stderr line per bench stage on rank 0 (the full run takes minutes; stdout carries only the result)."""
    if os.environ.get("RANK", "0") == "0":
        print(f"[bench {time.perf_counter() - _T_START:7.1f} s] {msg}", file=sys.stderr, flush=True)


def oracle_timing_lib():
    """The oracle built for timing on THIS host (oracle/liborc_native.so: gcc -O3 -march=native, so BMI2/ADX/AVX-512
    where the host has them), made on first use; the portable test build (-O2 -march=x86-64-v2) if no compiler."""
    import ctypes as ct
    import subprocess
    path = os.path.join(ROOT, "oracle", "liborc_native.so")
    if not os.path.exists(path):
        try:
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native"], check=True, timeout=180,
                           capture_output=True)
        except Exception:  # noqa: BLE001 — fall back to the portable build below
            pass
    if os.path.exists(path):
        lib = ct.CDLL(path)
        lib.orc_init()
        return lib, "oracle/liborc_native.so (gcc -O3 -march=native, built on this host)"
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as o
    return o.lib(), "oracle/liborc.so (gcc -O2 -march=x86-64-v2)"


def source_hash():
    """sha256 over the kernel / host sources (the GPU box has no .git): ties a committed PMC file to the build"""
    import glob
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "lachain_amd", "csrc")
    for f in sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.hpp")) +
                    glob.glob(os.path.join(csrc, "*.cpp")) + glob.glob(os.path.join(csrc, "*.h")) +
                    [os.path.join(csrc, "Makefile")]):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def cpu_threads():
    return max(1, min(16, os.cpu_count() or 1))   # the GPU box's CPU share is 16 threads


class Drbg:
    def __init__(self, seed: bytes):
        self.seed, self.ctr = seed, 0

    def block(self, n):
        out = bytearray()
        while len(out) < n:
            out += hashlib.sha256(self.seed + self.ctr.to_bytes(8, "little")).digest()
            self.ctr += 1
        return bytes(out[:n])

    def fr(self):
        return int.from_bytes(self.block(64), "little") % R


def make_inputs(nat, rank, n_shares, n_dec, f, vlen, corrupt_frac=0.01):
    """Synthetic TPKE batch generated with the product's own batch kernels (untimed)."""
    d = Drbg(SEED.to_bytes(8, "little") + rank.to_bytes(4, "little"))
    coeffs = [d.fr() for _ in range(f + 1)]

    def poly(x):
        acc = 0
        for c in reversed(coeffs):
            acc = (acc * x + c) % R
        return acc

    xs = [poly(i + 1) for i in range(n_dec)]
    y_secret = poly(0)
    n_cts = (n_shares + n_dec - 1) // n_dec
    rs = [d.fr() for _ in range(n_cts)]
    fr = lambda v: v.to_bytes(32, "little")
    y_keys = nat.mul_batch(1, None, [fr(x) for x in xs], generator=True)
    (y_pub,) = nat.mul_batch(1, None, [fr(y_secret)], generator=True)
    us, ts = nat.tpke_encrypt_phase1(y_pub, [fr(r) for r in rs])
    plain = d.block(vlen * n_cts)
    vs = [nat.xor_with_hash(ts[c], plain[c * vlen:(c + 1) * vlen]) for c in range(n_cts)]
    ws = nat.tpke_encrypt_phase2(us, [fr(r) for r in rs], vs)
    # shares: U_i = x_i U = (x_i r) G; corrupted: (x_i r + 1) G = U_i + G
    ct_idx = np.empty(n_shares, dtype=np.uint32)
    dec_idx = np.empty(n_shares, dtype=np.uint32)
    scal = bytearray(32 * n_shares)
    expect = np.ones(n_shares, dtype=np.uint8)
    # round(1 %) of the shares at seeded uniformly random positions (so some ciphertexts carry two or more bad shares,
    # the case the batched check's level-2 search cannot resolve alone)
    rng = np.random.default_rng(SEED + rank)
    expect[rng.choice(n_shares, size=int(round(corrupt_frac * n_shares)), replace=False)] = 0
    for i in range(n_shares):
        c, j = divmod(i, n_dec)
        ct_idx[i], dec_idx[i] = c, j
        s = xs[j] * rs[c] % R
        if not expect[i]:
            s = (s + 1) % R
        scal[32 * i:32 * i + 32] = s.to_bytes(32, "little")
    ui = nat.mul_batch_raw(1, b"", bytes(scal), n_shares, generator=True)
    v_off = np.arange(0, vlen * (n_cts + 1), vlen, dtype=np.uint32)
    return dict(y_keys=b"".join(y_keys), u=b"".join(us), w=b"".join(ws), v=b"".join(vs), v_off=v_off,
                ct_idx=ct_idx, dec_idx=dec_idx, ui=ui, expect=expect, n_cts=n_cts, n_dec=n_dec,
                keys_list=y_keys, cts_list=list(zip(us, vs, ws)), scal=bytes(scal))


# Byzantine patterns of the reference's own tests: a faulty validator corrupts its share in EVERY ciphertext
# (HoneyBadgerMalicious.cs:17-23 reverses the share bytes; validator 0 is the faulty one, HoneyBadgerTest.cs:75-94;
# HoneyBadgerSmartMalicious.cs:28-48 sends valid points that are not the share -> "wrong": U_i + G).
def byzantine_patterns(f):
    return {
        "random_1pct": None,                                   # the headline's pattern (make_inputs)
        "one_validator_reversed": ([0], "reversed"),
        "f_validators_reversed": (list(range(f)), "reversed"),
        "one_validator_wrong": ([0], "wrong"),
        "f_validators_wrong": (list(range(f)), "wrong"),
        "all_wrong": (None, "wrong"),
    }


def pattern_inputs(nat, inp, spec):
    """ui bytes and expected decisions of one pattern, from the batch's share scalars (wrong = scalar + 1)"""
    n = len(inp["expect"])
    if spec is None:
        return inp["ui"], inp["expect"]
    faulty, kind = spec
    scal = np.frombuffer(inp["scal"], dtype=np.uint8).reshape(n, 32)
    bad_scal = scal.copy()
    # the batch's 1 % corrupted shares carry scalar + 1: restore every share's good scalar first
    bad_idx = np.nonzero(inp["expect"] == 0)[0]
    good_scal = scal.copy()
    for i in bad_idx:
        v = (int.from_bytes(scal[i].tobytes(), "little") - 1) % R
        good_scal[i] = np.frombuffer(v.to_bytes(32, "little"), dtype=np.uint8)
    if "good_ui" not in inp:
        inp["good_ui"] = nat.mul_batch_raw(1, b"", good_scal.tobytes(), n, generator=True)
    ui = np.frombuffer(inp["good_ui"], dtype=np.uint8).reshape(n, 48).copy()
    sel = np.ones(n, dtype=bool) if faulty is None else np.isin(inp["dec_idx"], np.asarray(faulty, dtype=np.uint32))
    idx = np.nonzero(sel)[0]
    if kind == "reversed":
        ui[idx] = ui[idx, ::-1]
    else:
        for i in idx:
            v = (int.from_bytes(good_scal[i].tobytes(), "little") + 1) % R
            bad_scal[i] = np.frombuffer(v.to_bytes(32, "little"), dtype=np.uint8)
        ui[idx] = np.frombuffer(nat.mul_batch_raw(1, b"", bad_scal[idx].tobytes(), len(idx), generator=True),
                                dtype=np.uint8).reshape(len(idx), 48)
    expect = (~sel).astype(np.uint8)
    return ui.tobytes(), expect


def run_tpke_patterns(args, nat, torch, dev, world, inp, n, n_cts, n_dec):
    """The batched path (headline API) and the exact path on every Byzantine pattern of the reference's tests, same
    batch and timing discipline as the headline; decisions compared with the construction and with each other."""
    import torch.distributed as dist
    lib = nat.lib()
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    py, nk, pu, pw, pv, pvo, nc = PREP_ARGS[0]
    d_ct = to_dev(torch, dev, inp["ct_idx"])
    d_dec = to_dev(torch, dev, inp["dec_idx"])
    d_acc = torch.zeros(n, dtype=torch.uint8, device=dev)
    ctx = nat.Context()
    out = {}
    for name, spec in byzantine_patterns(args.f).items():
        if args.patterns and name not in args.patterns.split(","):
            continue
        ui_b, expect = pattern_inputs(nat, inp, spec)
        d_ui = to_dev(torch, dev, ui_b)

        def batched():
            rc = lib.lcb_ctx_tpke_verify_shares_batched_dev(ctx.ptr, d_acc.data_ptr(), n, py, nk, pu, pw, pv, pvo, nc,
                                                            d_ct.data_ptr(), d_dec.data_ptr(), d_ui.data_ptr(), sh)
            if rc != 0:
                raise RuntimeError(nat.last_error())

        def exact():
            rc = lib.lcb_ctx_tpke_prepare_dev(ctx.ptr, py, nk, pu, pw, pv, pvo, nc, sh)
            rc |= lib.lcb_ctx_tpke_verify_prepared_dev(ctx.ptr, d_acc.data_ptr(), n, nk, nc, d_ct.data_ptr(),
                                                       d_dec.data_ptr(), d_ui.data_ptr(), sh)
            if rc != 0:
                raise RuntimeError(nat.last_error())

        rec = {}
        got = {}
        for label, fn in (("batched", batched), ("exact", exact)):
            for _ in range(max(1, args.warmup)):
                fn()
            torch.cuda.synchronize(dev)
            got[label] = d_acc.cpu().numpy().copy()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(args.pattern_steps):
                fn()
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            el = time.perf_counter() - t0
            mism = int(np.sum(got[label] != expect)) + int(np.sum(d_acc.cpu().numpy() != expect))
            t = shard.max_time_sum(dist, torch, dev, el, mism)
            rec[label] = {"value": world * n * args.pattern_steps / float(t[0]),
                          "ms_per_step": 1e3 * float(t[0]) / args.pattern_steps, "decision_mismatches": int(t[1])}
            if label == "batched":
                lv = (ctypes.c_uint32 * 8)()
                m6 = (ctypes.c_float * 6)()
                k = lib.lcb_ctx_tpke_batched_stats(ctx.ptr, lv, m6)
                cs = (ctypes.c_uint32 * 4)()
                if lib.lcb_ctx_batched_census(ctx.ptr, cs) != 0:
                    raise RuntimeError(nat.last_error())
                rec[label]["levels"] = list(lv[:k])
                rec[label]["census"] = {"shares": cs[0], "suspect_keys": cs[1], "level1_groups": cs[2],
                                        "level1_entries_after_split": cs[3]}
        rec["rejected_shares"] = int(n - expect.sum())
        rec["batched_over_exact"] = rec["batched"]["value"] / rec["exact"]["value"]
        rec["batched_vs_exact_decisions_equal"] = bool(np.array_equal(got["batched"], got["exact"]))
        out[name] = rec
        del d_ui
    ctx.close()
    worst = min(out.values(), key=lambda r: r["batched_over_exact"]) if out else None
    return {"patterns": out,
            "worst_batched_over_exact": worst["batched_over_exact"] if worst else None,
            "note": ("reversed = the share's 48 bytes reversed (HoneyBadgerMalicious.cs:23; most do not decode and are "
                     "rejected without a pairing), wrong = a valid point that is not the share (U_i + G); faulty "
                     "validators 0..k-1 corrupt their share in every ciphertext; batched = "
                     "lcb_ctx_tpke_verify_shares_batched_dev (census of suspect keys + randomized group checks), "
                     "exact = lcb_ctx_tpke_prepare_dev + lcb_ctx_tpke_verify_prepared_dev; "
                     f"{args.pattern_steps} timed steps after {max(1, args.warmup)} warmup per path")}


def to_dev(torch, dev, b):
    if isinstance(b, np.ndarray):
        return torch.from_numpy(b.view(np.uint8).copy()).to(dev)
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)


def cpu_baseline(inp, target_s=12.0, batched=False):
    """configs[1] on host cores, two legs over the same shares (bounded samples, ~target_s each):
    amortized   — the GPU's algorithm: H(U||V) and the Miller lines of H and W once per ciphertext, one two-pair
                  Miller loop + ONE final exponentiation per share (orc_tpke_verify_batch_amortized);
    as_reference — what Lachain calls per share: G2.SetHashOf + two pairings + Equals (TPKE/PublicKey.cs:88-92,
                  orc_tpke_verify_batch).
    The amortized leg is the headline baseline (like-for-like algorithm); both run on the timing build."""
    lib, build = oracle_timing_lib()
    threads = cpu_threads()
    n_total, n_dec = len(inp["expect"]), inp["n_dec"]
    y, u, v, w, ui = inp["y_keys"], inp["u"], inp["v"], inp["w"], inp["ui"]
    vlen = int(inp["v_off"][1] - inp["v_off"][0])
    ct_all = np.ascontiguousarray(inp["ct_idx"], dtype=np.uint32)
    dec_all = np.ascontiguousarray(inp["dec_idx"], dtype=np.uint32)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)

    def run(n, amortized):
        n = max(n_dec, (n // n_dec) * n_dec)      # whole ciphertexts
        n_cts = n // n_dec
        acc = ctypes.create_string_buffer(n)
        ct, dc = ct_all[:n], dec_all[:n]
        t0 = time.perf_counter()
        if amortized == "rlc":
            rc = lib.orc_tpke_verify_batch_rlc(acc, ctypes.c_size_t(n), y, ctypes.c_size_t(n_dec), u, v,
                                               ctypes.c_size_t(vlen), w, ctypes.c_size_t(n_cts), p(ct), p(dc),
                                               ui[:48 * n], ctypes.c_uint64(int.from_bytes(os.urandom(8), "little")),
                                               threads)
        elif amortized:
            rc = lib.orc_tpke_verify_batch_amortized(acc, ctypes.c_size_t(n), y, ctypes.c_size_t(n_dec), u, v,
                                                     ctypes.c_size_t(vlen), w, ctypes.c_size_t(n_cts), p(ct), p(dc),
                                                     ui[:48 * n], threads)
        else:
            rc = lib.orc_tpke_verify_batch(acc, ctypes.c_size_t(n), y, u, v, ctypes.c_size_t(vlen), w, p(ct), p(dc),
                                           ui[:48 * n], threads)
        dt = time.perf_counter() - t0
        assert rc == 0
        mism = int(np.sum(np.frombuffer(acc.raw, dtype=np.uint8) != inp["expect"][:n]))
        return n, dt, mism

    legs = {}
    fn = {"rlc": "orc_tpke_verify_batch_rlc", True: "orc_tpke_verify_batch_amortized", False: "orc_tpke_verify_batch"}
    kinds = (("batched", "rlc"),) if batched else ()
    for name, am in kinds + (("amortized", True), ("as_reference", False)):
        n, dt, _ = run(8 * threads * n_dec if am else 4 * threads, am)
        n, dt, mism = run(int(min(n_total, max(n, n * target_s / max(dt, 1e-3)))), am)
        legs[name] = dict(value=n / dt, unit="share verifications/s", cores=threads, kind="port",
                          sample=f"first {n} shares ({n // n_dec} ciphertexts x {n_dec}) of the same batch, "
                                 f"{fn[am]}, {build}, "
                                 f"{threads} OpenMP threads, {dt:.1f} s, {mism} decision mismatches vs expected")
    if batched:       # like-for-like with the GPU headline: the same randomized batch algorithm on the host cores
        out = dict(legs["batched"])
        out["algorithm"] = "randomized batch check (the GPU's algorithm, k_batch.hip restated)"
        out["amortized_exact"] = dict(legs["amortized"], algorithm="exact per-share check, per-ciphertext lines")
    else:
        out = dict(legs["amortized"])
        out["algorithm"] = "amortized (the GPU's algorithm)"
    out["as_reference"] = legs["as_reference"]
    return out


# ------------------------------------------------------------------ G1 MSM (BASELINE configs[3])
R_TOP = R >> 192


def msm_inputs(nat, rank, n):
    """Points P_i = a_i G (a_i < 2^63, generated by the product's batch kernel), scalars uniform below r (top
    64-bit limb drawn below r's, so every value is < r).  Known answer: MSM = (sum a_i s_i mod r) G."""
    rng = np.random.default_rng([SEED, 0x4D534D, rank])
    a = rng.integers(1, 1 << 63, size=n, dtype=np.uint64)
    s = rng.integers(0, np.iinfo(np.uint64).max, size=(n, 4), dtype=np.uint64, endpoint=True)
    s[:, 3] = rng.integers(0, R_TOP, size=n, dtype=np.uint64)
    a_bytes = np.zeros((n, 4), dtype=np.uint64)
    a_bytes[:, 0] = a
    pts = nat.mul_batch_raw(1, b"", a_bytes.tobytes(), n, generator=True)
    # sum_i a_i s_i exactly: 16-bit limbs, every partial dot product stays below 2^58
    a16 = a.view(np.uint16).reshape(n, 4).astype(np.int64)
    s16 = s.view(np.uint16).reshape(n, 16).astype(np.int64)
    total = 0
    for k in range(4):
        for j in range(16):
            total += int(np.dot(a16[:, k], s16[:, j])) << (16 * (k + j))
    return pts, s.tobytes(), total % R


def msm_cpu_baseline(pts, scal, n_total, target_s=10.0):
    """The MSM CPU leg: the same algorithm as the GPU (signed-digit Pippenger, orc_g1_msm_pippenger) over the whole
    MSM, points decompressed beforehand (untimed, like the GPU's resident records); beside it the per-point
    multiplication MCL's LagrangeInterpolation does (orc_g1_msm_mt) on a bounded sample."""
    lib, build = oracle_timing_lib()
    threads = cpu_threads()
    lib.orc_g1_affine_bytes.restype = ctypes.c_size_t

    def run_ref(n):
        out = ctypes.create_string_buffer(48)
        t0 = time.perf_counter()
        rc = lib.orc_g1_msm_mt(out, pts[:48 * n], scal[:32 * n], ctypes.c_size_t(n), threads)
        assert rc == 0
        return time.perf_counter() - t0

    n = min(n_total, 64 * threads)
    dt = run_ref(n)
    n = int(min(n_total, max(n, n * (target_s / 2) / max(dt, 1e-3))))
    dt = run_ref(n)
    as_ref = dict(value=n / dt, unit="points/s", cores=threads, kind="port",
                  sample=f"first {n} points of the same MSM, orc_g1_msm_mt (one 255-bit var-base multiplication per "
                         f"point, as MCL's LagrangeInterpolation does), {build}, {threads} OpenMP threads, {dt:.1f} s")
    m = n_total
    aff = ctypes.create_string_buffer(lib.orc_g1_affine_bytes() * m)
    assert lib.orc_g1_affine_batch(aff, pts[:48 * m], ctypes.c_size_t(m), threads) == 0
    # window width minimising windows x (points + buckets)
    c = min(range(8, 19), key=lambda c: ((256 + c - 1) // c + 1) * (m + (1 << c)))
    out = ctypes.create_string_buffer(48)
    t0 = time.perf_counter()
    assert lib.orc_g1_msm_pippenger(out, aff, scal[:32 * m], ctypes.c_size_t(m), c, threads) == 0
    dt = time.perf_counter() - t0
    return dict(value=m / dt, unit="points/s", cores=threads, kind="port",
                sample=f"all {m} points of the same MSM, orc_g1_msm_pippenger (signed {c}-bit digits, Jacobian buckets "
                       f"with mixed additions, running-sum reduction, Horner over the windows: the GPU's plain-form "
                       f"algorithm; points decompressed beforehand), {build}, {threads} OpenMP threads, {dt:.2f} s",
                algorithm="Pippenger bucket method (same as the GPU)", as_reference=as_ref)


def run_msm_sizes(args, nat, torch, dev, rank, world, cpu):
    """configs[3]: one entry per total size in --msm-sizes (default 2^20 and 2^24 points), the points of each
    MSM sharded over the ranks (n / world per rank) with the RCCL all-gather of the 144-byte partials."""
    out = []
    for k, total in enumerate(int(x) for x in args.msm_sizes.split(",") if x):
        progress(f"MSM {total} points")
        r = run_msm(args, nat, torch, dev, rank, world, cpu and k == 0, max(1, total // world))
        if r is not None:
            r["total_points"] = total
            out.append(r)
        torch.cuda.empty_cache()
    return out


def run_msm(args, nat, torch, dev, rank, world, cpu, n):
    import torch.distributed as dist
    from lachain_amd import shard
    lib = nat.lib()
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    pts, scal, expect_local = msm_inputs(nat, rank, n)
    d_pts48 = to_dev(torch, dev, pts)
    d_aff = torch.empty(96 * n, dtype=torch.uint8, device=dev)
    d_ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_sc = to_dev(torch, dev, scal)
    d_jac = torch.zeros(144, dtype=torch.uint8, device=dev)
    d_out = torch.zeros(48, dtype=torch.uint8, device=dev)
    if lib.lcb_g1_to_affine_dev(d_aff.data_ptr(), d_ok.data_ptr(), d_pts48.data_ptr(), n, sh) != 0:
        raise RuntimeError(nat.last_error())
    del d_pts48
    # configs[3]'s points are a_i G (order r), so the GLV entry point applies; it keeps the plain form where that is
    # faster (large n) and reports that as a negative width
    msm_fn = lib.lcb_g1_msm_dev if args.msm_no_glv else lib.lcb_g1_msm_glv_dev
    c = lib.lcb_g1_msm_window(n) if args.msm_no_glv else lib.lcb_g1_msm_glv_window(n)
    glv = c > 0 and not args.msm_no_glv
    c = abs(c)
    wbits = 0
    if args.msm_glv_window > 0 and not args.msm_no_glv:     # A/B: the GLV form at an explicit width
        wbits, c, glv = args.msm_glv_window, args.msm_glv_window, True

    def sum_partials(allp, w):
        if lib.lcb_g1_jac_sum_dev(d_out.data_ptr(), None, allp.data_ptr(), w, sh) != 0:
            raise RuntimeError(nat.last_error())

    def step():
        if msm_fn(d_jac.data_ptr(), d_aff.data_ptr(), d_sc.data_ptr(), n, wbits, sh) != 0:
            raise RuntimeError(nat.last_error())
        # RCCL over xGMI: all-gather of the 144 B Jacobian partials, summed on the GPU (lachain_amd/shard.py)
        shard.msm_combine(dist, d_jac, world, sum_partials)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.msm_steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    phases = nat.msm_phase_ms()
    single_ms = 1e3 * elapsed / args.msm_steps
    # P independent MSMs in flight (the reference runs many LagrangeInterpolate-sized MSMs, one per ciphertext /
    # coin): one context and stream per slot, so one MSM's serial tails (bucket reduction, window combination) run
    # beside the next one's bucket accumulation; every slot's result is checked against the same known answer
    pipe = max(1, args.msm_pipeline)
    pipe_outs = []
    if pipe > 1:
        slots = []
        for _ in range(pipe):
            slots.append(dict(ctx=nat.Context(), st=torch.cuda.Stream(dev),
                              jac=torch.zeros(144, dtype=torch.uint8, device=dev),
                              out=torch.zeros(48, dtype=torch.uint8, device=dev)))
        pfn = lib.lcb_ctx_g1_msm_dev if args.msm_no_glv else lib.lcb_ctx_g1_msm_glv_dev
        torch.cuda.synchronize(dev)

        def pstep(k):
            sl = slots[k % pipe]
            st = sl["st"]
            with torch.cuda.stream(st):
                if pfn(sl["ctx"].ptr, sl["jac"].data_ptr(), d_aff.data_ptr(), d_sc.data_ptr(), n, wbits,
                       st.cuda_stream) != 0:
                    raise RuntimeError(nat.last_error())

                def psum(allp, w):
                    if lib.lcb_ctx_g1_jac_sum_dev(sl["ctx"].ptr, sl["out"].data_ptr(), None, allp.data_ptr(), w,
                                                  st.cuda_stream) != 0:
                        raise RuntimeError(nat.last_error())
                shard.msm_combine(dist, sl["jac"], world, psum)

        for k in range(max(args.warmup, 1) * pipe):
            pstep(k)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        kp = max(args.msm_steps, 2) * pipe
        t0 = time.perf_counter()
        for k in range(kp):
            pstep(k)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        elapsed_p = time.perf_counter() - t0
        if world > 1:
            elapsed_p = shard.max_time_sum(dist, torch, dev, elapsed_p)[0]
        pipe_outs = [bytes(sl["out"].cpu().numpy().tobytes()) for sl in slots]
        for sl in slots:
            sl["ctx"].close()
    # known answer over all ranks: (sum of the per-rank sums) G
    e = torch.tensor(list(expect_local.to_bytes(32, "little")), dtype=torch.uint8, device=dev)
    ok_pts = bool(d_ok.all().item())
    if world > 1:
        ge = shard.all_gather_fixed(dist, e, world)
        elapsed = shard.max_time_sum(dist, torch, dev, elapsed)[0]
        exp_total = sum(int.from_bytes(bytes(ge[32 * k:32 * k + 32].cpu().numpy().tobytes()), "little")
                        for k in range(world)) % R
    else:
        exp_total = expect_local
    if rank != 0:
        return None
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as o
    got = bytes(d_out.cpu().numpy().tobytes())
    want = o.g1_mul(o.g1_gen(), o.fr(exp_total))
    correct = ok_pts and got == want and all(p == want for p in pipe_outs)
    bits, npts = (128, 2 * n) if glv else (255, n)
    nwin = (128 + c - 1) // c if glv else 255 // c + 1
    t_acc = phases["bucket_acc"] * 1e-3
    fpmul_acc = npts * (bits / c) * 11     # mixed adds, one per nonzero digit (zero digits: 2^-c of them)
    fpmul_total = nwin * (npts * 11 + (1 << (c - 1)) * 2 * 16)
    bytes_acc = npts * (bits / c) * (96 + 4) + nwin * (1 << (c - 1)) * (8 + 144)
    single_value = n * world * args.msm_steps / elapsed
    w_msm = fpmul_total * MAC_PER_FPMUL          # SURVEY W(n): the whole MSM's algorithmic work
    res = dict(
        metric="BLS12-381 G1 MSM points/sec (Pippenger, sum_i s_i P_i)",
        value=n * world * kp / elapsed_p if pipe > 1 else single_value,
        unit="points/s", points_per_rank=n, window_bits=c, windows=nwin,
        steps=kp if pipe > 1 else args.msm_steps, in_flight=pipe,
        form="GLV: s = s1 + s2 lambda over P and phi(P) (points of order r)" if glv else "plain 255-bit digits",
        ms_per_step=1e3 * (elapsed_p / kp if pipe > 1 else elapsed / args.msm_steps), known_answer_ok=correct,
        single_msm=dict(value=single_value, ms=single_ms, steps=args.msm_steps,
                        frac_whole_msm=w_msm / (single_ms * 1e-3) / PEAK_MAC32),
        frac_whole_msm=w_msm / ((elapsed_p / kp if pipe > 1 else elapsed / args.msm_steps)) / PEAK_MAC32,
        phase_ms={k: round(v, 3) for k, v in phases.items()},
        roofline={"bound": "valu_int32", "kernel": "k_msm_bucket_acc",
                  "achieved": fpmul_acc * MAC_PER_FPMUL / t_acc / 1e12, "peak": PEAK_MAC32 / 1e12,
                  "unit": "Tmac32/s", "frac": fpmul_acc * MAC_PER_FPMUL / t_acc / PEAK_MAC32,
                  "hbm_gbs_bucket_phase": bytes_acc / t_acc / 1e9, "hbm_peak_gbs": 8000.0,
                  "algorithmic_fpmul_per_msm": fpmul_total},
        config="configs[3]: G1 Pippenger MSM, points sharded across ranks, RCCL all-gather of 144 B Jacobian partials",
    )
    if cpu:
        res["cpu_baseline"] = msm_cpu_baseline(pts, scal, n)
    return res


# ------------------------------------------------------------------ threshold signatures (BASELINE configs[2])
W_TS = C["C_DEC2"] + C["C_ML2_NORM1"] + C["C_LINES"] + C["C_FE"]  # per share: sig decompress, Miller (one side's
                                                                 # lines on the fly), final exponentiation


def coin_id(era, agreement, epoch):
    """CommonCoin message: CoinId.ToBytes() = Era || Agreement || Epoch, int64 LE (CoinId.cs:21-24)"""
    m64 = (1 << 64) - 1   # C# long.ToBytes(): two's complement, little-endian
    return b"".join((v & m64).to_bytes(8, "little") for v in (era, agreement, epoch))


def ts_inputs(nat, rank, rounds, n, f):
    d = Drbg(SEED.to_bytes(8, "little") + b"TS" + rank.to_bytes(4, "little"))
    coeffs = [d.fr() for _ in range(f + 1)]

    def poly(x):
        acc = 0
        for c in reversed(coeffs):
            acc = (acc * x + c) % R
        return acc

    sks = [poly(i + 1) for i in range(n)]
    shared_sk = poly(0)
    fr = lambda v: v.to_bytes(32, "little")
    pks = nat.mul_batch(1, None, [fr(x) for x in sks] + [fr(shared_sk)], generator=True)   # 100 shares + shared
    msgs = [coin_id(0, rank * rounds + r, 5) for r in range(rounds)]
    hs = np.frombuffer(b"".join(nat.g2_hash_batch(msgs)), dtype=np.uint8).reshape(rounds, 96)
    pts = np.repeat(hs, n, axis=0).tobytes()
    sk_arr = np.frombuffer(b"".join(fr(x) for x in sks), dtype=np.uint8).reshape(n, 32)
    sigs = bytearray(nat.mul_batch_raw(2, pts, np.tile(sk_arr, (rounds, 1)).tobytes(), rounds * n))
    good_sigs = bytes(sigs)
    # corrupt one share per round (1 %): share j of round r carries the signature of share j+1 (valid point,
    # wrong key); j = 7r mod n, so a third of the rounds lose one of their first F+1 shares
    expect = np.ones(rounds * n, dtype=np.uint8)
    for r in range(rounds):
        j = (7 * r) % n
        a, b = r * n + j, r * n + (j + 1) % n
        sigs[96 * a:96 * a + 96] = sigs[96 * b:96 * b + 96]
        expect[a] = 0
    midx = np.repeat(np.arange(rounds, dtype=np.uint32), n)
    pidx = np.tile(np.arange(n, dtype=np.uint32), rounds)
    moff = np.arange(0, 24 * (rounds + 1), 24, dtype=np.uint32)
    return dict(pks=b"".join(pks), msgs=b"".join(msgs), moff=moff, sigs=bytes(sigs), midx=midx, pidx=pidx,
                expect=expect, shared_sk=shared_sk, msg_list=msgs, good_sigs=good_sigs)


def ts_cpu_baseline(inp, n_total, n_per_round, target_s=10.0, batched=False):
    """configs[2] share verification on host cores: amortized (H(m) lines once per message, one final exp per
    share: orc_ts_validate_batch_amortized) and as-reference (hash + two pairings per ValidateSignature call,
    ThresholdSignature/PublicKey.cs:16-21: orc_ts_validate_batch)."""
    lib, build = oracle_timing_lib()
    threads = cpu_threads()
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    n_pks = len(inp["pks"]) // 48

    def run(k, am):
        k = max(n_per_round, (k // n_per_round) * n_per_round)
        acc = ctypes.create_string_buffer(k)
        mi = np.ascontiguousarray(inp["midx"][:k])
        pi = np.ascontiguousarray(inp["pidx"][:k])
        n_msgs = int(mi[-1]) + 1
        t0 = time.perf_counter()
        if am == "rlc":
            rc = lib.orc_ts_validate_batch_rlc(acc, ctypes.c_size_t(k), inp["pks"], ctypes.c_size_t(n_pks),
                                               inp["sigs"][:96 * k], inp["msgs"], p(inp["moff"]),
                                               ctypes.c_size_t(n_msgs), p(mi), p(pi),
                                               ctypes.c_uint64(int.from_bytes(os.urandom(8), "little")), threads)
        elif am:
            rc = lib.orc_ts_validate_batch_amortized(acc, ctypes.c_size_t(k), inp["pks"], ctypes.c_size_t(n_pks),
                                                     inp["sigs"][:96 * k], inp["msgs"], p(inp["moff"]),
                                                     ctypes.c_size_t(n_msgs), p(mi), p(pi), threads)
        else:
            rc = lib.orc_ts_validate_batch(acc, ctypes.c_size_t(k), inp["pks"], inp["sigs"][:96 * k], inp["msgs"],
                                           p(inp["moff"]), p(mi), p(pi), threads)
        dt = time.perf_counter() - t0
        assert rc == 0
        return k, dt, int(np.sum(np.frombuffer(acc.raw, dtype=np.uint8) != inp["expect"][:k]))

    legs = {}
    fn = {"rlc": "orc_ts_validate_batch_rlc", True: "orc_ts_validate_batch_amortized", False: "orc_ts_validate_batch"}
    kinds = (("batched", "rlc"),) if batched else ()
    for name, am in kinds + (("amortized", True), ("as_reference", False)):
        k, dt, _ = run(n_per_round * 2, am)
        k, dt, mism = run(int(min(n_total, max(k, k * target_s / max(dt, 1e-3)))), am)
        legs[name] = dict(value=k / dt, unit="share verifications/s", cores=threads, kind="port",
                          sample=f"first {k} shares ({k // n_per_round} rounds) of the same rounds, {fn[am]}, {build}, "
                                 f"{threads} OpenMP threads, {dt:.1f} s, {mism} decision mismatches vs expected")
    if batched:
        out = dict(legs["batched"])
        out["algorithm"] = "randomized batch check (the GPU's algorithm, k_batch.hip restated)"
        out["amortized_exact"] = dict(legs["amortized"], algorithm="exact per-share check, per-message lines")
    else:
        out = dict(legs["amortized"])
        out["algorithm"] = "amortized (the GPU's algorithm)"
    out["as_reference"] = legs["as_reference"]
    return out


def run_ts(args, nat, torch, dev, rank, world):
    """configs[2]: per step, prepare (keys, H(m) + lines) + verify every share, assemble the first F+1 valid shares
    per round (G2 Lagrange) and verify the combined signatures.  Timed twice on the same rounds: the randomized batch
    share check (lcb_ts_verify_shares_batched_dev: prepare + group checks in one call, the line's value) and the exact
    per-share check (lcb_ts_prepare_dev + lcb_ts_verify_prepared_dev, under "exact")."""
    import torch.distributed as dist
    lib = nat.lib()
    rounds, n, f = args.ts_rounds, args.ts_n, (args.ts_n - 1) // 3
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    t_gen = time.perf_counter()
    inp = ts_inputs(nat, rank, rounds, n, f)
    t_gen = time.perf_counter() - t_gen
    d_pks, d_msg, d_moff = to_dev(torch, dev, inp["pks"]), to_dev(torch, dev, inp["msgs"]), to_dev(torch, dev, inp["moff"])
    d_sigs, d_midx, d_pidx = to_dev(torch, dev, inp["sigs"]), to_dev(torch, dev, inp["midx"]), to_dev(torch, dev, inp["pidx"])
    d_acc = torch.zeros(rounds * n, dtype=torch.uint8, device=dev)
    d_comb = torch.zeros(96 * rounds, dtype=torch.uint8, device=dev)
    d_cst = torch.zeros(rounds, dtype=torch.uint8, device=dev)
    d_cacc = torch.zeros(rounds, dtype=torch.uint8, device=dev)
    d_ridx = torch.arange(rounds, dtype=torch.int32, device=dev)
    d_shared = torch.full((rounds,), n, dtype=torch.int32, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as o

    def run(batched):
        def step(timed=False):
            if timed:
                ev[0].record(stream)
            if batched:
                rc = lib.lcb_ts_verify_shares_batched_dev(d_acc.data_ptr(), rounds * n, d_pks.data_ptr(), n + 1,
                                                          d_sigs.data_ptr(), d_msg.data_ptr(), d_moff.data_ptr(),
                                                          rounds, d_midx.data_ptr(), d_pidx.data_ptr(), sh)
                if timed:
                    ev[1].record(stream)
            else:
                rc = lib.lcb_ts_prepare_dev(d_pks.data_ptr(), n + 1, d_msg.data_ptr(), d_moff.data_ptr(), rounds, sh)
                if timed:
                    ev[1].record(stream)
                rc |= lib.lcb_ts_verify_prepared_dev(d_acc.data_ptr(), rounds * n, n + 1, rounds, d_sigs.data_ptr(),
                                                     d_midx.data_ptr(), d_pidx.data_ptr(), sh)
            if timed:
                ev[2].record(stream)
            rc |= lib.lcb_ts_assemble_dev(d_comb.data_ptr(), d_cst.data_ptr(), d_acc.data_ptr(), d_sigs.data_ptr(), n,
                                          f + 1, rounds, sh)
            rc |= lib.lcb_ts_verify_prepared_dev(d_cacc.data_ptr(), rounds, n + 1, rounds, d_comb.data_ptr(),
                                                 d_ridx.data_ptr(), d_shared.data_ptr(), sh)
            if timed:
                ev[3].record(stream)
            if rc != 0:
                raise RuntimeError(nat.last_error())

        d_acc.fill_(7)
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        t_prep = t_ver = t_asm = 0.0
        for _ in range(args.ts_steps):
            step(True)
            torch.cuda.synchronize(dev)
            t_prep += ev[0].elapsed_time(ev[1])
            t_ver += ev[1].elapsed_time(ev[2])
            t_asm += ev[2].elapsed_time(ev[3])
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        levels = nat.tpke_batched_stats()[0] if batched else None
        mism = int(np.sum(d_acc.cpu().numpy() != inp["expect"]))
        comb_ok = int(d_cst.cpu().numpy().sum()) == rounds and int(d_cacc.cpu().numpy().sum()) == rounds
        # spot-check combined signatures against the oracle: sigma_r = shared_sk * H(msg_r) (ThresholdSignatureTest.cs)
        comb = d_comb.cpu().numpy().tobytes()
        for r in (0, 1, rounds - 1):
            comb_ok = comb_ok and comb[96 * r:96 * r + 96] == o.ts_sign(o.fr(inp["shared_sk"]), inp["msg_list"][r])
        t = shard.max_time_sum(dist, torch, dev, elapsed, mism, 0 if comb_ok else 1)
        per = args.ts_steps
        elapsed = float(t[0])
        out = dict(value=rounds * n * world * per / elapsed, unit="share verifications/s",
                   rounds_per_s=rounds * world * per / elapsed, ms_per_step=1e3 * elapsed / per,
                   decision_mismatches=int(t[1]), combined_ok=int(t[2]) == 0)
        if batched:
            out["phase_ms"] = {"prepare_and_verify_shares (one call)": (t_prep + t_ver) / per,
                               "assemble_and_verify_combined": t_asm / per}
            out["levels"] = levels
            out["api"] = "lcb_ts_verify_shares_batched_dev (prepare + randomized group checks)"
            step_fpmul = rounds * ts_round_fpmul(n, f + 1) + sum(levels or []) * C["C_TS_CHECK"]
            step_s = elapsed / per
            out["roofline"] = {"bound": "valu_int32",
                               "kernel": ("whole CommonCoin step: k_ts_rlc_points, message preparation, group checks, "
                                          "G2 Lagrange lanes, combined-signature checks"),
                               "achieved": step_fpmul * MAC_PER_FPMUL / step_s / 1e12, "peak": PEAK_MAC32 / 1e12,
                               "unit": "Tmac32/s", "frac": step_fpmul * MAC_PER_FPMUL / step_s / PEAK_MAC32,
                               "fpmul_per_step": step_fpmul,
                               "work_model": {k_: C[k_] for k_ in ("C_TS_POINTS", "C_GSUM_TS", "C_TS_CHECK",
                                                                  "C_MSG_PREP", "C_G2_LAG1", "C_G2_LAG2")}}
        else:
            ver_s = t_ver / per * 1e-3
            out["phase_ms"] = {"prepare": t_prep / per, "verify_shares": t_ver / per,
                               "assemble_and_verify_combined": t_asm / per}
            out["api"] = "lcb_ts_prepare_dev + lcb_ts_verify_prepared_dev"
            out["roofline"] = {"bound": "valu_int32", "kernel": "k_ts_miller + k_final_exp_check",
                               "achieved": rounds * n * W_TS * MAC_PER_FPMUL / ver_s / 1e12,
                               "peak": PEAK_MAC32 / 1e12, "unit": "Tmac32/s",
                               "frac": rounds * n * W_TS * MAC_PER_FPMUL / ver_s / PEAK_MAC32,
                               "work_per_share_fpmul": W_TS}
        return out

    bat = run(True) if args.ts_batched else None
    exact = run(False) if args.ts_exact else None

    def patterns():
        """faulty signers send a wrong share (the next signer's signature: a valid point) in EVERY round; the share
        checks alone (batched call vs exact prepare + verify), same rounds"""
        res = {}
        good = np.frombuffer(inp["good_sigs"], dtype=np.uint8).reshape(rounds, n, 96)
        for name, faulty in (("one_signer_wrong", [0]), ("f_signers_wrong", list(range(f)))):
            sg = good.copy()
            for j in faulty:
                sg[:, j] = good[:, (j + 1) % n] if (j + 1) % n not in faulty else good[:, (faulty[-1] + 1) % n]
            exp = np.ones((rounds, n), dtype=np.uint8)
            exp[:, faulty] = 0
            exp = exp.reshape(-1)
            d_sg = to_dev(torch, dev, sg.tobytes())
            rec = {}
            for label in ("batched", "exact"):
                def call():
                    if label == "batched":
                        rc = lib.lcb_ts_verify_shares_batched_dev(d_acc.data_ptr(), rounds * n, d_pks.data_ptr(),
                                                                  n + 1, d_sg.data_ptr(), d_msg.data_ptr(),
                                                                  d_moff.data_ptr(), rounds, d_midx.data_ptr(),
                                                                  d_pidx.data_ptr(), sh)
                    else:
                        rc = lib.lcb_ts_prepare_dev(d_pks.data_ptr(), n + 1, d_msg.data_ptr(), d_moff.data_ptr(),
                                                    rounds, sh)
                        rc |= lib.lcb_ts_verify_prepared_dev(d_acc.data_ptr(), rounds * n, n + 1, rounds,
                                                             d_sg.data_ptr(), d_midx.data_ptr(), d_pidx.data_ptr(), sh)
                    if rc != 0:
                        raise RuntimeError(nat.last_error())
                call()
                torch.cuda.synchronize(dev)
                mism = int(np.sum(d_acc.cpu().numpy() != exp))
                if world > 1:
                    dist.barrier()
                t0 = time.perf_counter()
                call()
                torch.cuda.synchronize(dev)
                if world > 1:
                    dist.barrier()
                el = time.perf_counter() - t0
                mism += int(np.sum(d_acc.cpu().numpy() != exp))
                t = shard.max_time_sum(dist, torch, dev, el, mism)
                rec[label] = {"value": rounds * n * world / float(t[0]), "ms_per_step": 1e3 * float(t[0]),
                              "decision_mismatches": int(t[1])}
                if label == "batched":
                    rec[label]["levels"] = nat.tpke_batched_stats()[0]
                    cs = nat.batched_census()
                    rec[label]["census"] = {"shares": cs[0], "suspect_keys": cs[1], "level1_groups": cs[2],
                                            "level1_entries_after_split": cs[3]}
            rec["batched_over_exact"] = rec["batched"]["value"] / rec["exact"]["value"]
            res[name] = rec
            del d_sg
        return res

    byz = patterns() if (args.pattern_steps > 0 and args.ts_batched and args.ts_exact) else None
    if rank != 0:
        return None
    head = bat or exact
    res = dict(
        metric="BLS12-381 threshold-signature share verifications/sec (ValidateSignature + AddShare assembly)",
        rounds_per_rank=rounds, shares_per_round=n, threshold_k=f + 1, steps=args.ts_steps,
        config=f"configs[2]: {rounds} rounds x N={n} F={f} CommonCoin shares per rank (one wrong share per round); "
               f"per round: {n} share verifications, G2 Lagrange over the first {f + 1} valid shares, "
               f"combined-signature verification",
        input_gen_s=t_gen,
        algorithm=("randomized batch check per round (e(sum s_i PK_i, H) == e(G, sum s_i sig_i), secret 64-bit "
                   "exponents; level 2 names a round's single bad share from gamma' = gamma^c)" if bat else
                   "exact per-share check"))
    res.update(head)
    if bat and exact:
        res["exact"] = exact
    res["byzantine"] = byz
    if world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = ts_cpu_baseline(inp, rounds * n, n, batched=bat is not None)
    return res


# ------------------------------------------------------------------ HoneyBadger epoch replay (BASELINE configs[4])
def replay_inputs(nat, n, f, n_coins, vlen=32):
    """One era of an N-node network: N ciphertexts (one proposal per node), every node's decryption share of
    every ciphertext, n_coins CommonCoin instances with every node's signature share.  One share per
    ciphertext and one per coin is corrupted (share j carries share j+1's value) so the reject and the
    first-F+1-valid selection paths run."""
    d = Drbg(SEED.to_bytes(8, "little") + b"REPLAY")
    fr = lambda v: v.to_bytes(32, "little")

    def keys():
        coeffs = [d.fr() for _ in range(f + 1)]
        poly = lambda x: sum(c * pow(x, i, R) for i, c in enumerate(coeffs)) % R
        return [poly(i + 1) for i in range(n)], poly(0)

    xs, y_secret = keys()
    y_keys = nat.mul_batch(1, None, [fr(x) for x in xs], generator=True)
    (y_pub,) = nat.mul_batch(1, None, [fr(y_secret)], generator=True)
    rs = [d.fr() for _ in range(n)]
    us, ts = nat.tpke_encrypt_phase1(y_pub, [fr(r) for r in rs])
    plain = d.block(vlen * n)
    vs = [nat.xor_with_hash(ts[c], plain[c * vlen:(c + 1) * vlen]) for c in range(n)]
    ws = nat.tpke_encrypt_phase2(us, [fr(r) for r in rs], vs)
    scal = bytearray(32 * n * n)
    expect_t = np.ones(n * n, dtype=np.uint8)
    for c in range(n):
        for j in range(n):
            sc = xs[j] * rs[c] % R
            if j == (7 * c) % n:
                sc = xs[(j + 1) % n] * rs[c] % R
                expect_t[c * n + j] = 0
            scal[32 * (c * n + j):32 * (c * n + j) + 32] = fr(sc)
    shares = nat.mul_batch_raw(1, b"", bytes(scal), n * n, generator=True)
    sks, shared_sk = keys()
    pks = nat.mul_batch(1, None, [fr(x) for x in sks] + [fr(shared_sk)], generator=True)
    msgs = [coin_id(0, m - 1, 0) for m in range(n_coins)]   # root coin (agreement -1) + one per agreement
    hs = np.frombuffer(b"".join(nat.g2_hash_batch(msgs)), dtype=np.uint8).reshape(n_coins, 96)
    sk_arr = np.frombuffer(b"".join(fr(x) for x in sks), dtype=np.uint8).reshape(n, 32)
    sigs = bytearray(nat.mul_batch_raw(2, np.repeat(hs, n, axis=0).tobytes(), np.tile(sk_arr, (n_coins, 1)).tobytes(),
                                       n_coins * n))
    expect_s = np.ones(n_coins * n, dtype=np.uint8)
    for m in range(n_coins):
        j = (3 * m) % n
        a, b = m * n + j, m * n + (j + 1) % n
        sigs[96 * a:96 * a + 96] = sigs[96 * b:96 * b + 96]
        expect_s[a] = 0
    return dict(xs=xs, y_keys=b"".join(y_keys), u=b"".join(us), w=b"".join(ws), v=b"".join(vs), plain=plain,
                shares=shares, expect_t=expect_t, pks=b"".join(pks), msgs=b"".join(msgs), msg_list=msgs,
                sigs=bytes(sigs), expect_s=expect_s, shared_sk=shared_sk)


def replay_cpu_baseline(inp, n, f, n_coins, target_s=3.0):
    """configs[4] on host cores, composed from bounded samples of the same era's inputs (every term measured here,
    all threads busy): per view = n^2 decryption-share verifications (the GPU's randomized batch check,
    orc_tpke_verify_batch_rlc, all n shares of a ciphertext in one group) + n partial decryptions (validity check + x U, orc_tpke_decrypt) + n FullDecrypt combinations
    (G1 Lagrange k = f+1) + n_coins x (n signature-share verifications (orc_ts_validate_batch_rlc) + G2 Lagrange k = f+1 + 1 combined
    check)."""
    from concurrent.futures import ThreadPoolExecutor
    lib, build = oracle_timing_lib()
    threads = cpu_threads()
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    vlen = len(inp["v"]) // n
    timings = {}

    def timed(fn, units):
        t0 = time.perf_counter()
        fn()
        return (time.perf_counter() - t0) / units

    # decryption shares: C ciphertexts x n shares
    def tpke(c):
        m = c * n
        acc = ctypes.create_string_buffer(m)
        ct = np.repeat(np.arange(c, dtype=np.uint32), n)
        dec = np.tile(np.arange(n, dtype=np.uint32), c)
        rc = lib.orc_tpke_verify_batch_rlc(acc, ctypes.c_size_t(m), inp["y_keys"], ctypes.c_size_t(n), inp["u"],
                                           inp["v"], ctypes.c_size_t(vlen), inp["w"], ctypes.c_size_t(c), p(ct),
                                           p(dec), inp["shares"][:48 * m], ctypes.c_uint64(SEED), threads)
        assert rc == 0 and acc.raw == bytes(inp["expect_t"][:m])
    c = max(1, threads // 8)
    t = timed(lambda: tpke(c), c * n)
    c = int(min(n, max(c, c * target_s / max(t * c * n, 1e-3))))
    timings["tpke_share"] = timed(lambda: tpke(c), c * n)

    def ts(mc):
        m = mc * n
        acc = ctypes.create_string_buffer(m)
        mi = np.repeat(np.arange(mc, dtype=np.uint32), n)
        pi = np.tile(np.arange(n, dtype=np.uint32), mc)
        moff = np.arange(0, 24 * (mc + 1), 24, dtype=np.uint32)
        rc = lib.orc_ts_validate_batch_rlc(acc, ctypes.c_size_t(m), inp["pks"], ctypes.c_size_t(n + 1),
                                           inp["sigs"][:96 * m], inp["msgs"], p(moff), ctypes.c_size_t(mc),
                                           p(mi), p(pi), ctypes.c_uint64(SEED), threads)
        assert rc == 0 and acc.raw == bytes(inp["expect_s"][:m])
    mc = max(1, threads // 8)
    t = timed(lambda: ts(mc), mc * n)
    mc = int(min(n_coins, max(mc, mc * target_s / max(t * mc * n, 1e-3))))
    timings["ts_share"] = timed(lambda: ts(mc), mc * n)

    fr = lambda v: v.to_bytes(32, "little")
    k = f + 1
    xs = b"".join(fr(i + 1) for i in range(k))
    g1s, g2s = inp["shares"][:48 * k], inp["sigs"][:96 * k]
    x0 = fr(inp["xs"][0])

    def pool(fn, jobs):
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(fn, range(jobs)))
    g1l = lambda _: lib.orc_g1_lagrange(ctypes.create_string_buffer(48), xs, g1s, ctypes.c_size_t(k))
    g2l = lambda _: lib.orc_g2_lagrange(ctypes.create_string_buffer(96), xs, g2s, ctypes.c_size_t(k))
    dec = lambda j: lib.orc_tpke_decrypt(ctypes.create_string_buffer(48), inp["u"][48 * j:48 * j + 48],
                                         inp["v"][vlen * j:vlen * j + vlen], ctypes.c_size_t(vlen),
                                         inp["w"][96 * j:96 * j + 96], x0)
    jobs = 2 * threads
    timings["g1_lagrange"] = timed(lambda: pool(g1l, jobs), jobs)
    timings["g2_lagrange"] = timed(lambda: pool(g2l, jobs), jobs)
    timings["partial_decrypt"] = timed(lambda: pool(dec, jobs), jobs)
    per_view = (n * n * timings["tpke_share"] + n * timings["partial_decrypt"] + n * timings["g1_lagrange"] +
                n_coins * ((n + 1) * timings["ts_share"] + timings["g2_lagrange"]))
    return dict(value=1.0 / per_view, unit="views/s", cores=threads, kind="port",
                per_item_ms={kk: round(v * 1e3, 4) for kk, v in timings.items()},
                sample=f"composed from measured samples of the same era ({c} ciphertexts x {n} decryption shares, "
                       f"{mc} coins x {n} signature shares, both through the GPU's randomized batch check (k_batch.hip restated), "
                       f"{jobs} G1 / G2 Lagrange "
                       f"problems at k={k} and {jobs} partial decryptions), {build}, {threads} threads")


def run_replay(args, nat, torch, dev, rank, world):
    """All N nodes' views of one era, views block-partitioned over the ranks (strong
    scaling: N views in total).  Per view: N ciphertext checks + the node's own partial decryptions, N*N
    decryption-share verifications, N FullDecrypt combinations (G1 Lagrange, k = F+1), and n_coins coins of
    N signature-share verifications + G2 Lagrange (k = F+1) + combined-signature check."""
    import torch.distributed as dist
    from lachain_amd import shard
    lib = nat.lib()
    n = args.replay_n
    f = (n - 1) // 3
    n_coins = n + 1
    v_lo, v_hi = shard.block_range(n, rank, world)
    V = v_hi - v_lo
    sh = torch.cuda.current_stream(dev).cuda_stream
    t_gen = time.perf_counter()
    inp = replay_inputs(nat, n, f, n_coins)
    t_gen = time.perf_counter() - t_gen
    tile = lambda b, reps: to_dev(torch, dev, b).repeat(reps)
    vlen = len(inp["v"]) // n
    d_y = to_dev(torch, dev, inp["y_keys"])
    d_u, d_w, d_v = tile(inp["u"], V), tile(inp["w"], V), tile(inp["v"], V)
    d_voff = to_dev(torch, dev, np.arange(0, vlen * (V * n + 1), vlen, dtype=np.uint32))
    x_views = np.frombuffer(b"".join(x.to_bytes(32, "little") for x in inp["xs"][v_lo:v_hi]), dtype=np.uint8)
    d_x = to_dev(torch, dev, np.repeat(x_views.reshape(V, 32), n, axis=0))   # view v decrypts with its own x
    d_own = torch.zeros(48 * V * n, dtype=torch.uint8, device=dev)
    d_own_st = torch.zeros(V * n, dtype=torch.uint8, device=dev)
    d_ct = to_dev(torch, dev, np.repeat(np.arange(V * n, dtype=np.uint32), n))
    d_dec = to_dev(torch, dev, np.tile(np.arange(n, dtype=np.uint32), V * n))
    d_sh = tile(inp["shares"], V)
    d_acc_t = torch.zeros(V * n * n, dtype=torch.uint8, device=dev)
    d_uc = torch.zeros(48 * V * n, dtype=torch.uint8, device=dev)
    d_ucst = torch.zeros(V * n, dtype=torch.uint8, device=dev)
    nm = V * n_coins
    d_pks = to_dev(torch, dev, inp["pks"])
    d_msg = tile(inp["msgs"], V)
    d_moff = to_dev(torch, dev, np.arange(0, 24 * (nm + 1), 24, dtype=np.uint32))
    d_sigs = tile(inp["sigs"], V)
    d_midx = to_dev(torch, dev, np.repeat(np.arange(nm, dtype=np.uint32), n))
    d_pidx = to_dev(torch, dev, np.tile(np.arange(n, dtype=np.uint32), nm))
    d_acc_s = torch.zeros(nm * n, dtype=torch.uint8, device=dev)
    d_comb = torch.zeros(96 * nm, dtype=torch.uint8, device=dev)
    d_cst = torch.zeros(nm, dtype=torch.uint8, device=dev)
    d_cacc = torch.zeros(nm, dtype=torch.uint8, device=dev)
    d_ridx = to_dev(torch, dev, np.arange(nm, dtype=np.uint32))
    d_shared = to_dev(torch, dev, np.full(nm, n, dtype=np.uint32))

    batched = not args.replay_exact
    # the era's TPKE decryptions and its coins are independent (HoneyBadger runs them in separate protocol
    # instances): with --replay-concurrent 1 they run side by side, each chain on its own host thread (so its own
    # default library context) and HIP stream, and one chain's latency-bound check levels overlap the other's bulk
    conc = args.replay_concurrent and batched
    s_tp = torch.cuda.Stream(dev) if conc else None
    s_ts = torch.cuda.Stream(dev) if conc else None

    def tpke_chain(sh):
        rc = lib.lcb_tpke_verify_shares_batched_dev(d_acc_t.data_ptr(), V * n * n, d_y.data_ptr(), n, d_u.data_ptr(),
                                                    d_w.data_ptr(), d_v.data_ptr(), d_voff.data_ptr(), V * n,
                                                    d_ct.data_ptr(), d_dec.data_ptr(), d_sh.data_ptr(), sh)
        rc |= lib.lcb_tpke_partial_decrypt_prepared_dev(d_own.data_ptr(), d_own_st.data_ptr(), d_x.data_ptr(), 1,
                                                        d_u.data_ptr(), V * n, sh)
        rc |= lib.lcb_tpke_combine_dev(d_uc.data_ptr(), d_ucst.data_ptr(), d_acc_t.data_ptr(), d_sh.data_ptr(), n,
                                       f + 1, V * n, sh)
        return rc

    def ts_chain(sh):
        rc = lib.lcb_ts_verify_shares_batched_dev(d_acc_s.data_ptr(), nm * n, d_pks.data_ptr(), n + 1,
                                                  d_sigs.data_ptr(), d_msg.data_ptr(), d_moff.data_ptr(), nm,
                                                  d_midx.data_ptr(), d_pidx.data_ptr(), sh)
        rc |= lib.lcb_ts_assemble_dev(d_comb.data_ptr(), d_cst.data_ptr(), d_acc_s.data_ptr(), d_sigs.data_ptr(), n,
                                      f + 1, nm, sh)
        rc |= lib.lcb_ts_verify_prepared_dev(d_cacc.data_ptr(), nm, n + 1, nm, d_comb.data_ptr(), d_ridx.data_ptr(),
                                             d_shared.data_ptr(), sh)
        return rc

    import concurrent.futures
    # one persistent thread per chain: each keeps its own default library context (and its workspaces) across steps
    pools = [concurrent.futures.ThreadPoolExecutor(max_workers=1) for _ in range(2)] if conc else []

    def run_chain(k):
        st = s_tp if k == 0 else s_ts
        rc = (tpke_chain if k == 0 else ts_chain)(st.cuda_stream)
        st.synchronize()
        return rc, (nat.last_error() if rc else "")

    def step_concurrent():
        torch.cuda.current_stream(dev).synchronize()    # inputs uploaded on the default stream are complete
        res = [f.result() for f in [pools[k].submit(run_chain, k) for k in range(2)]]
        for rc, err in res:
            if rc:
                raise RuntimeError(err)

    def step():
        if conc:
            return step_concurrent()
        if batched:      # prepare + randomized group checks in one call each (k_batch.hip)
            rc = lib.lcb_tpke_verify_shares_batched_dev(d_acc_t.data_ptr(), V * n * n, d_y.data_ptr(), n,
                                                        d_u.data_ptr(), d_w.data_ptr(), d_v.data_ptr(),
                                                        d_voff.data_ptr(), V * n, d_ct.data_ptr(), d_dec.data_ptr(),
                                                        d_sh.data_ptr(), sh)
        else:
            rc = lib.lcb_tpke_prepare_dev(d_y.data_ptr(), n, d_u.data_ptr(), d_w.data_ptr(), d_v.data_ptr(),
                                          d_voff.data_ptr(), V * n, sh)
        rc |= lib.lcb_tpke_partial_decrypt_prepared_dev(d_own.data_ptr(), d_own_st.data_ptr(), d_x.data_ptr(), 1,
                                                        d_u.data_ptr(), V * n, sh)
        if not batched:
            rc |= lib.lcb_tpke_verify_prepared_dev(d_acc_t.data_ptr(), V * n * n, n, V * n, d_ct.data_ptr(),
                                                   d_dec.data_ptr(), d_sh.data_ptr(), sh)
        rc |= lib.lcb_tpke_combine_dev(d_uc.data_ptr(), d_ucst.data_ptr(), d_acc_t.data_ptr(), d_sh.data_ptr(), n,
                                       f + 1, V * n, sh)
        if batched:
            rc |= lib.lcb_ts_verify_shares_batched_dev(d_acc_s.data_ptr(), nm * n, d_pks.data_ptr(), n + 1,
                                                       d_sigs.data_ptr(), d_msg.data_ptr(), d_moff.data_ptr(), nm,
                                                       d_midx.data_ptr(), d_pidx.data_ptr(), sh)
        else:
            rc |= lib.lcb_ts_prepare_dev(d_pks.data_ptr(), n + 1, d_msg.data_ptr(), d_moff.data_ptr(), nm, sh)
            rc |= lib.lcb_ts_verify_prepared_dev(d_acc_s.data_ptr(), nm * n, n + 1, nm, d_sigs.data_ptr(),
                                                 d_midx.data_ptr(), d_pidx.data_ptr(), sh)
        rc |= lib.lcb_ts_assemble_dev(d_comb.data_ptr(), d_cst.data_ptr(), d_acc_s.data_ptr(), d_sigs.data_ptr(), n,
                                      f + 1, nm, sh)
        rc |= lib.lcb_ts_verify_prepared_dev(d_cacc.data_ptr(), nm, n + 1, nm, d_comb.data_ptr(), d_ridx.data_ptr(),
                                             d_shared.data_ptr(), sh)
        if rc != 0:
            raise RuntimeError(nat.last_error())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.replay_steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    for pl in pools:
        pl.shutdown()
    # checks: bitmaps, every view decrypts every ciphertext and assembles every coin, spot values vs oracle
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as o
    bad = int(np.sum(d_acc_t.cpu().numpy() != np.tile(inp["expect_t"], V)))
    bad += int(np.sum(d_acc_s.cpu().numpy() != np.tile(inp["expect_s"], V)))
    bad += int(V * n - d_own_st.cpu().numpy().sum()) + int(V * n - d_ucst.cpu().numpy().sum())
    bad += int(nm - d_cst.cpu().numpy().sum()) + int(nm - d_cacc.cpu().numpy().sum())
    uc, own = d_uc.cpu().numpy().tobytes(), d_own.cpu().numpy().tobytes()
    for c in (0, n - 1):
        bad += o.xor_with_hash(uc[48 * c:48 * c + 48], inp["v"][vlen * c:vlen * c + vlen]) != \
            inp["plain"][vlen * c:vlen * c + vlen]
        exp_own = o.tpke_decrypt(inp["u"][48 * c:48 * c + 48], inp["v"][vlen * c:vlen * c + vlen],
                                 inp["w"][96 * c:96 * c + 96], o.fr(inp["xs"][v_lo]))
        bad += own[48 * c:48 * c + 48] != exp_own
    comb = d_comb.cpu().numpy().tobytes()
    bad += comb[:96] != o.ts_sign(o.fr(inp["shared_sk"]), inp["msg_list"][0])
    t = shard.max_time_sum(dist, torch, dev, elapsed, bad)
    if rank != 0:
        return None
    elapsed = float(t[0]) / args.replay_steps
    checks_per_view = n + n * n + n_coins * n + n_coins
    cpu = replay_cpu_baseline(inp, n, f, n_coins) if (world == 1 and not args.no_cpu_baseline) else None
    era_fpmul = n * replay_view_fpmul(n, f, n_coins)
    roof = {"bound": "valu_int32", "kernel": "whole era (every view): bench.py replay_view_fpmul",
            "achieved": era_fpmul * MAC_PER_FPMUL / elapsed / 1e12, "peak": PEAK_MAC32 / 1e12, "unit": "Tmac32/s",
            "frac": era_fpmul * MAC_PER_FPMUL / elapsed / PEAK_MAC32, "fpmul_per_era": era_fpmul}
    return dict(metric="HoneyBadgerBFT epoch crypto replay: node views/sec (TPKE + CommonCoin)", cpu_baseline=cpu,
                value=n / elapsed, unit="views/s", scaling="strong", views_total=n, n=n, f=f, coins=n_coins,
                roofline=roof,
                pairing_checks_per_s=n * checks_per_view / elapsed, ms_per_era=1e3 * elapsed,
                steps=args.replay_steps, mismatches=int(t[1]), input_gen_s=t_gen,
                share_checks=("randomized batch checks (lcb_tpke_verify_shares_batched_dev, "
                              "lcb_ts_verify_shares_batched_dev)" if batched else "exact per-share checks"),
                concurrent_chains=bool(conc),
                config=f"configs[4]: all {n} nodes' views of one era (N={n}, F={f}), views block-partitioned over "
                       f"ranks; per view {checks_per_view} pairing checks, {n} G1 and {n_coins} G2 Lagrange (k={f + 1})")


# ------------------------------------------------------------------ secp256k1 header signatures
W_ECDSA = 66 * 11 + 3        # Fp-mul per verification: <= 66 mixed additions (7M + 4S) + the r Z^2 comparison
MAC_PER_FPMUL_SECP = 72      # 8x8 32-bit product + 8 for the fold by 2^32 + 977 (p = 2^256 - 2^32 - 977)


def ecdsa_inputs(nat, rank, n, n_val, era, chain):
    """n SignedHeaderMessages of one era from n_val validators (RootProtocol.cs:91-105): random headers with Index =
    era, hashed and signed on the GPU with the product's own kernels (lcb_header_keccak_batch,
    lcb_ecdsa_sign_hashed_batch, new chain id); 1 % of the signatures get one bit of s flipped (must reject)."""
    rng = np.random.default_rng(0x4C61636861696E + 0x5EC + rank)

    def scalars(k):
        b = rng.integers(0, 256, (k, 32), dtype=np.uint8)
        b[:, 0] &= 0x7F                                 # < 2^255 < n
        b[:, 31] |= 1                                   # nonzero
        return b
    privs = scalars(n_val)
    keys, ok = nat.ecdsa_pubkey_batch(privs.tobytes())
    assert all(ok)
    hdr = rng.integers(0, 256, (n, 112), dtype=np.uint8)
    hdr[:, 0:8] = np.frombuffer(int(era).to_bytes(8, "little"), dtype=np.uint8)
    hashes = nat.header_keccak_batch(hdr.tobytes())
    idx = rng.integers(0, n_val, n, dtype=np.int32)
    sigs, sok = nat.ecdsa_sign_hashed_batch(hashes, privs[idx].tobytes(), scalars(n).tobytes(), True, chain)
    assert all(sok)
    sig = np.frombuffer(sigs, dtype=np.uint8).reshape(n, 66).copy()
    bad = rng.choice(n, max(1, n // 100), replace=False)
    sig[bad, 40] ^= 1
    expect = np.ones(n, dtype=np.uint8)
    expect[bad] = 0
    return dict(keys=keys, hdr=hdr.tobytes(), hashes=hashes, sigs=sig.tobytes(), idx=idx, expect=expect)


def ecdsa_cpu_baseline(inp, n_total, chain, target_s=8.0):
    lib, build = oracle_timing_lib()
    threads = cpu_threads()

    def run(m):
        out = ctypes.create_string_buffer(m)
        idx = np.ascontiguousarray(inp["idx"][:m])
        f = lib.orc_ecdsa_verify_batch_mt
        t0 = time.perf_counter()
        f(out, inp["hashes"][:32 * m], inp["sigs"][:66 * m], ctypes.c_size_t(66), inp["keys"], ctypes.c_size_t(33),
          ctypes.c_void_p(idx.ctypes.data), ctypes.c_size_t(len(inp["keys"]) // 33), ctypes.c_size_t(m), 1,
          ctypes.c_int32(chain), threads)
        dt = time.perf_counter() - t0
        assert out.raw[:m] == inp["expect"][:m].tobytes()
        return dt

    m = min(n_total, 32 * threads)
    dt = run(m)
    m = int(min(n_total, max(m, m * target_s / max(dt, 1e-3))))
    dt = run(m)
    return dict(value=m / dt, unit="header signatures/s", cores=threads, kind="port",
                sample=f"first {m} signatures of the same batch, orc_ecdsa_verify_batch_mt (libsecp256k1 verify "
                       f"semantics, Straus-Shamir 4-bit windows, 4x64-bit Montgomery; the header Keccak (~1 us) is not "
                       f"included), {build}, {threads} OpenMP threads, {dt:.1f} s")


def run_ecdsa(args, nat, torch, dev, rank, world, cpu):
    """RootProtocol header-signature checks: lcb_root_header_verify_dev over n headers of one era per rank (Keccak of
    the header, the Index == era check, VerifySignatureHashed) against a 256-validator key set resident on the GPU."""
    import torch.distributed as dist
    lib = nat.lib()
    n, era, chain = args.ecdsa_sigs, 4242, 225
    t_gen = time.perf_counter()
    inp = ecdsa_inputs(nat, rank, n, args.ecdsa_validators, era, chain)
    t_gen = time.perf_counter() - t_gen
    t_ks = time.perf_counter()
    ks = nat.EcdsaKeySet(inp["keys"], 33)
    t_ks = time.perf_counter() - t_ks
    sh = torch.cuda.current_stream(dev).cuda_stream
    d_hdr = to_dev(torch, dev, inp["hdr"])
    d_sig = to_dev(torch, dev, inp["sigs"])
    d_idx = torch.from_numpy(inp["idx"]).to(dev)
    d_acc = torch.zeros(n, dtype=torch.uint8, device=dev)

    def step():
        if lib.lcb_root_header_verify_dev(d_acc.data_ptr(), d_hdr.data_ptr(), era, d_sig.data_ptr(), 66,
                                          d_idx.data_ptr(), n, ks.h, 1, chain, sh) != 0:
            raise RuntimeError(nat.last_error())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.ecdsa_steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kms = (ctypes.c_float * 3)()
    if lib.lcb_ecdsa_phase_ms(kms) != 0:
        raise RuntimeError(nat.last_error())
    mism = int(np.sum(d_acc.cpu().numpy() != inp["expect"]))
    t = shard.max_time_sum(dist, torch, dev, elapsed, mism)
    elapsed = t[0]
    ks.close()
    if rank != 0:
        return None
    hash_ms, scal_ms, ver_ms = (float(x) for x in kms)
    achieved = n * W_ECDSA * MAC_PER_FPMUL_SECP / (ver_ms * 1e-3)
    res = dict(
        metric="secp256k1 ECDSA header-signature verifications/sec (RootProtocol SignedHeaderMessage check)",
        value=n * world * args.ecdsa_steps / elapsed, unit="header signatures/s", signatures_per_rank=n,
        validators=args.ecdsa_validators, steps=args.ecdsa_steps, ms_per_step=1e3 * elapsed / args.ecdsa_steps,
        decision_mismatches=int(t[1]), input_gen_s=t_gen, keyset_build_s=t_ks,
        kernel_ms={"k_secp_header_hash": hash_ms, "k_secp_scalars": scal_ms, "k_secp_verify": ver_ms},
        roofline={"bound": "valu_int32", "kernel": "k_secp_verify", "achieved": achieved / 1e12,
                  "peak": PEAK_MAC32 / 1e12, "unit": "Tmac32/s", "frac": achieved / PEAK_MAC32,
                  "work_per_signature_fpmul": W_ECDSA, "mac_per_fpmul": MAC_PER_FPMUL_SECP},
        config=f"SURVEY §8f row 4: {n} headers of one era per rank, {args.ecdsa_validators} validators' keys resident "
               f"with fixed-base comb tables, new chain id {chain}, 1% corrupted; shards by era (no collective)",
    )
    if cpu:
        res["cpu_baseline"] = ecdsa_cpu_baseline(inp, n, chain)
    return res


# ------------------------------------------------------------------ DKG G1 work and RBC erasure coding
def run_dkg(args, nat, rank):
    """Trustless-DKG value checks of one node (TrustlessKeygen.cs:150-152): Commitment.Evaluate(x, y) of all N dealers'
    commitments (degree F, (F+1)(F+2)/2 G1 coefficients each, generated as c_k G on the GPU) at x = the node's index,
    y = the dealer's.  Host-pointer API (lcb_dkg_commitment_eval): the rate includes the coefficient upload."""
    if rank != 0:
        return None
    n_val, deg = args.dkg_n, args.dkg_f
    ncoef = (deg + 1) * (deg + 2) // 2
    rng = np.random.default_rng(0x4C61636861696E + 0xD6)
    sc = rng.integers(0, 256, (n_val * ncoef, 32), dtype=np.uint8)
    sc[:, 31] &= 0x3F                                   # < 2^254 < r
    pts = nat.mul_batch_raw(1, None, sc.tobytes(), n_val * ncoef, generator=True)
    comms = [[pts[48 * (c * ncoef + k):48 * (c * ncoef + k) + 48] for k in range(ncoef)] for c in range(n_val)]
    queries = [(j, 1, j + 1) for j in range(n_val)]    # node 0's checks of every dealer's value
    nat.dkg_commitment_eval(comms, deg, queries[:2])   # warm-up (allocation)
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        got = nat.dkg_commitment_eval(comms, deg, queries)
    dt = (time.perf_counter() - t0) / reps
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as o
    t1 = time.perf_counter()
    m = 0
    while m < 4 and (m == 0 or time.perf_counter() - t1 < args.cpu_seconds / 3):
        assert o.dkg_commitment_eval(comms[m], deg, 1, m + 1) == got[m]
        m += 1
    cdt = (time.perf_counter() - t1) / m
    return dict(metric="Commitment.Evaluate(x, y) checks/sec (trustless DKG, one node's view of every dealer)",
                value=n_val / dt, unit="evaluations/s", dealers=n_val, degree=deg, ms_per_batch=1e3 * dt,
                api="lcb_dkg_commitment_eval (host pointers: includes the upload of the coefficients)",
                parity=f"first {m} results equal the oracle's literal (F+1)^2-product Commitment.Evaluate",
                cpu_baseline=dict(value=1.0 / cdt, unit="evaluations/s", cores=1, kind="port",
                                  sample=f"{m} evaluations, oracle orc_dkg_commitment_eval as the reference computes it "
                                         f"((F+1)^2 G1 x Fr products, Commitment.cs:23-37), one thread"))


def run_rs(args, nat, rank):
    """Reliable-broadcast erasure coding at N = 256 (F = 85: 86 data + 170 parity shards, ErasureCoding.cs:13):
    ErasureCodingShards of a payload and DecodeFromEchos from 86 random echoes (ReliableBroadcast.cs:393-446).
    Host-pointer API: the rate includes the payload / shard transfers."""
    if rank != 0:
        return None
    n_sh, era = args.rs_n, 2 * ((args.rs_n - 1) // 3)
    k = n_sh - era
    size = (args.rs_bytes // k) * k
    rng = np.random.default_rng(0x4C61636861696E + 0x125)
    data = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
    S = size // k
    nat.rs_encode(data[:k], n_sh, era)
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        enc = nat.rs_encode(data, n_sh, era)
    t_enc = (time.perf_counter() - t0) / reps
    keep = sorted(rng.choice(n_sh, k, replace=False).tolist())
    echos = [(j, enc[j * S:(j + 1) * S]) for j in keep]
    t0 = time.perf_counter()
    for _ in range(reps):
        dec = nat.rs_decode(echos, S, n_sh, era)
    t_dec = (time.perf_counter() - t0) / reps
    ok = dec == enc and enc[:size] == data
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as o
    sample = max(k, (min(size, 1 << 16) // k) * k)
    t1 = time.perf_counter()
    ref = o.rs_encode_shards(data[:sample], n_sh, era)
    c_enc = time.perf_counter() - t1
    s2 = sample // k
    assert ref == nat.rs_encode(data[:sample], n_sh, era)
    return dict(metric="Reed-Solomon erasure coding of reliable-broadcast payloads (N = %d shards, %d erasures)" % (n_sh, era),
                value=size / t_enc / 1e6, unit="payload MB/s (encode)", decode_mb_s=size / t_dec / 1e6,
                payload_bytes=size, shard_bytes=S, round_trip_exact=bool(ok),
                api="lcb_rs_encode / lcb_rs_decode (host pointers: includes the transfers)",
                cpu_baseline=dict(value=sample / c_enc / 1e6, unit="payload MB/s (encode)", cores=1, kind="port",
                                  sample=f"{sample} bytes ({s2} B shards), oracle orc_rs_encode_shards (ZXing-style "
                                         f"polynomial division per byte column), one thread; equal to the GPU shards"))

def run_mcl_latency(args, nat, rank):
    """Per-call latency of the mcl single-element surface (include/lachain_bls.h, the calls Lachain's protocol code
    makes one at a time): scalar Fr product and G1 / G2 addition / (de)serialization (host field code, fr_host.hpp /
    fp_host.hpp), G1 / G2 scalar products (k_ptmul.hip: GLV / GLS ladders on four lanes each, membership ladder beside),
    the pairing and the final exponentiation (nine-lane cooperative kernels), mulVec / Lagrange / Horner at the consensus sizes (N = 22,
    F = 7), and PublicKey.VerifyShare written as the reference writes it (HashToG2 + two GT.Pairing + Equals,
    TPKE/PublicKey.cs:88-92) beside the library's one-share batch call.  Median wall time per call from Python
    through ctypes (the ctypes overhead, ~1 us, is included); the oracle's single-threaded time for the same call
    beside the GPU-backed ones."""
    if rank != 0:
        return None
    from lachain_amd import mcl
    from lachain_amd.tpke import PublicKey, EncryptedShare, PartiallyDecryptedShare
    Fr, G1, G2, GT, M = mcl.Fr, mcl.G1, mcl.G2, mcl.GT, mcl.MclBls12381
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as o
    reps = args.mcl_reps

    def med(fn, r=reps):
        fn()
        ts = []
        for _ in range(r):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return 1e3 * ts[len(ts) // 2]

    a, b = Fr.GetRandom(), Fr.GetRandom()
    P, Q = G1.Generator() * a, G2.Generator() * b
    ab, bb, Pb, Qb = a.ToBytes(), b.ToBytes(), P.ToBytes(), Q.ToBytes()
    import itertools
    Qring = [G2.Generator() * Fr.GetRandom() for _ in range(40)]       # more than the 32-slot line-set cache
    qi = itertools.count()
    f = GT()
    mcl._f("mclBn_millerLoop", None, [ctypes.POINTER(type(f.v)), ctypes.POINTER(type(P.v)),
                                      ctypes.POINTER(type(Q.v))])(ctypes.byref(f.v), ctypes.byref(P.v), ctypes.byref(Q.v))
    fe = mcl._f("mclBn_finalExp", None, [ctypes.POINTER(type(f.v))] * 2)
    g = GT()
    xs = [Fr.FromInt(i + 1) for i in range(args.f + 1)]
    ys = [G1.Generator() * Fr.GetRandom() for _ in range(args.f + 1)]
    cs = [G1.Generator() * Fr.GetRandom() for _ in range(args.f + 1)]
    ys2 = [G2.Generator() * Fr.GetRandom() for _ in range(args.f + 1)]
    vs = [G1.Generator() * Fr.GetRandom() for _ in range(args.n)]
    ks = [Fr.GetRandom() for _ in range(args.n)]
    from lachain_amd.native import mclBnG1, mclBnFr
    pa = (mclBnG1 * args.n)(*[p.v for p in vs])
    sa = (mclBnFr * args.n)(*[k.v for k in ks])
    mv = mcl._f("mclBnG1_mulVec", None, [ctypes.POINTER(mclBnG1), ctypes.POINTER(mclBnG1), ctypes.POINTER(mclBnFr),
                                        ctypes.c_size_t])
    out = G1()
    # one TPKE share as the protocol sees it
    x = Fr.GetRandom()
    Y = (G1.Generator() * x).ToBytes()
    pk = PublicKey(Y, args.f + 1)
    r = Fr.GetRandom()
    U = (G1.Generator() * r).ToBytes()
    V = bytes(32)
    Hb = nat.g2_hash_batch([U + V])[0]
    W = (G2.FromBytes(Hb) * r).ToBytes()
    Ui = (G1.FromBytes(U) * x).ToBytes()
    share, ps = EncryptedShare(U, V, W, 0), PartiallyDecryptedShare(Ui, 0, 0)
    Ug, Yg, Wg, Uig = G1.FromBytes(U), G1.FromBytes(Y), G2.FromBytes(W), G1.FromBytes(Ui)

    def verify_mcl():
        h = G2()
        h.SetHashOf(U + V)
        return GT.Pairing(Uig, h) == GT.Pairing(Yg, Wg)

    assert verify_mcl() and pk.VerifyShare(share, ps)
    res = {
        "Fr_mul": 1e3 * med(lambda: a * b, 2000),
        "G1_add": 1e3 * med(lambda: P + P, 2000),
        "G2_add": 1e3 * med(lambda: Q + Q, 2000),
        "G1_deserialize": 1e3 * med(lambda: G1.FromBytes(Pb), 200),
        "G2_deserialize": 1e3 * med(lambda: G2.FromBytes(Qb), 200),
        "G1_mul": 1e3 * med(lambda: P * a),
        "G2_mul": 1e3 * med(lambda: Q * a),
        "pairing": 1e3 * med(lambda: GT.Pairing(P, Q)),
        "pairing_new_Q": 1e3 * med(lambda: GT.Pairing(P, Qring[next(qi) % len(Qring)])),
        "finalExp": 1e3 * med(lambda: fe(ctypes.byref(g.v), ctypes.byref(f.v))),
        "G1_mulVec_n%d" % args.n: 1e3 * med(lambda: mv(ctypes.byref(out.v), pa, sa, args.n)),
        "G1_Lagrange_k%d" % (args.f + 1): 1e3 * med(lambda: M.LagrangeInterpolate(xs, ys)),
        "G1_EvaluatePolynomial_n%d" % (args.f + 1): 1e3 * med(lambda: M.EvaluatePolynomial(cs, xs[3])),
        "G2_Lagrange_k%d" % (args.f + 1): 1e3 * med(lambda: M.LagrangeInterpolate(xs, ys2)),
        "VerifyShare_via_mcl": 1e3 * med(verify_mcl),
        "VerifyShare_batch_api_n1": 1e3 * med(lambda: pk.VerifyShare(share, ps)),
    }
    ref = {
        "Fr_mul": 1e3 * med(lambda: o.fr_mul(ab, bb), 2000),
        "G1_mul": 1e3 * med(lambda: o.g1_mul(Pb, ab)),
        "G2_mul": 1e3 * med(lambda: o.g2_mul(Qb, ab)),
        "pairing": 1e3 * med(lambda: o.pairing(Pb, Qb), max(3, reps // 3)),
    }
    return dict(metric="mcl single-call latency (median, one thread, through ctypes)", unit="us per call",
                gpu=res, oracle_cpu=ref,
                note="GPU-backed calls are a synchronous round trip each (launch + copies); Fr arithmetic and the "
                     "O(1) G1 / G2 field work (add, (de)serialize) are host code (fr_host.hpp, fp_host.hpp).  pairing: a repeated G2 argument (its line set cached per thread, as for "
                     "the H and W every share of a ciphertext is paired with); pairing_new_Q: 40 rotating G2 "
                     "arguments (every call computes its line set).  oracle_cpu: the oracle's plain-C routines "
                     "(portable build), one thread, same inputs")


C["C_MUL1_64"] = round(C["C_MUL1"] * 64 / 255)          # 64-bit var-base G1 multiplication (double-and-add)
C["C_MADD1"] = 11                                          # G1 mixed addition (7M + 4S)
C["C_JADD1"] = 16                                          # G1 Jacobian addition (11M + 5S)
C["C_DBL1"] = (C["C_MUL1"] - 127.5 * C["C_MADD1"]) / 255   # G1 doubling, from the 255-bit ladder's count
C["C_MUL_AB32"] = round(32 * C["C_DBL1"] + 32 * C["C_MADD1"]) + 1   # a P + b phi(P): 32 dbl, ~2 x 16 madds, beta x
C["C_KTAB"] = 7 * C["C_JADD1"] + 1                         # a Y + b phi(Y) from the key's byte tables
W_RLC_POINTS = C["C_DEC1"] + C["C_MUL_AB32"] + C["C_KTAB"]  # per share: decompress U_i, s_i U_i, s_i Y_i
# Round 5: whole-step work models of configs[2] and configs[4] from the same frozen counts.  G2 group
# operations in Fp-mul: a mixed addition is 7 Fp2 products + 4 squares (3 / 2 Fp-mul), a Jacobian addition 11 + 5; the
# doubling comes from the frozen 255-bit G2 ladder as C_DBL1 does from the G1 one.
C["C_MADD2"] = 7 * 3 + 4 * 2
C["C_JADD2"] = 11 * 3 + 5 * 2
C["C_DBL2"] = (C["C_MUL2"] - 127.5 * C["C_MADD2"]) / 255
# CommonCoin share randomisation (k_ts_rlc_points): decompress sigma, psi membership (63 doublings + 5 mixed additions
# + psi), a sigma + b psi^4(sigma) (32 doublings + ~32 mixed additions with the joint addend), the key's byte tables
C["C_TS_POINTS"] = round(C["C_DEC2"] + 63 * C["C_DBL2"] + 5 * C["C_MADD2"] + 10 + 32 * C["C_DBL2"]
                         + 32 * C["C_MADD2"] + C["C_KTAB"])
C["C_GSUM_TS"] = C["C_JADD1"] + C["C_JADD2"]              # per share: the group sums of both sides
C["C_GSUM_TPKE"] = 2 * C["C_JADD1"]
C["C_TS_CHECK"] = C["C_ML2_NORM1"] + C["C_LINES"] + C["C_FE"]   # a group check, the sigma side's lines on the fly
C["C_MSG_PREP"] = C["C_H2G2"] + C["C_LINES"] + C["C_NORM"]      # per message: hash to G2 + its normalised line set
# G2 Lagrange lanes (lanetab.hpp): GLS over the 15 sums of the psi-images, 64 doublings + 60 mixed additions (15 of 16
# digit columns nonzero) per table, the table's 1 + 9 additions, ~20 Fp-mul per entry of the batched affine conversion
# and one Fp2 inversion per lane; a pair of entries shares the doublings and the inversion
C["C_G2_LAG1"] = round(64 * C["C_DBL2"] + 60 * C["C_MADD2"] + C["C_MADD2"] + 9 * C["C_JADD2"] + 15 * 20 + C["C_FP2_INV"])
C["C_G2_LAG2"] = round(64 * C["C_DBL2"] + 120 * C["C_MADD2"] + 2 * (C["C_MADD2"] + 9 * C["C_JADD2"]) + 30 * 20
                       + C["C_FP2_INV"])


def ts_round_fpmul(n, k):
    """per CommonCoin round of n shares and threshold k: randomisation + group sums of every share, the message's
    preparation, the assembly's Lagrange lanes (k // 2 pairs + k % 2 single, the k - 1 additions and the affine output)
    and the combined signature's exact check; the group checks are counted separately (from the levels run)"""
    asm = (k // 2) * C["C_G2_LAG2"] + (k % 2) * C["C_G2_LAG1"] + (k - 1) * C["C_JADD2"] + C["C_AFF2"]
    return n * (C["C_TS_POINTS"] + C["C_GSUM_TS"]) + C["C_MSG_PREP"] + asm + W_TS


def replay_view_fpmul(n, f, n_coins):
    """per node view of configs[4] (all shares valid: level 1 only): the TPKE batch check of n x n shares (groups of
    <= 32) with the n ciphertexts' preparation, the node's partial decryptions (pairing check + x U), the n FullDecrypt
    G1 Lagrange combinations (k = f + 1 ladders of C_MUL1), and n_coins coins (batch check of n shares in groups of
    <= 128, assembly, combined check)"""
    k = f + 1
    tpke = n * n * (W_RLC_POINTS + C["C_GSUM_TPKE"]) + n * -(-n // 32) * (C["C_ML2_NORM2"] + C["C_FE"]) + n * W_PREPARE
    pdec = n * (C["C_DEC1"] + C["C_ML2_NORM2"] + C["C_FE"] + C["C_MUL1"])
    comb = n * (k * C["C_MUL1"] + (k - 1) * C["C_JADD1"] + C["C_AFF2"])
    coins = n_coins * ts_round_fpmul(n, k) + n_coins * -(-n // 128) * C["C_TS_CHECK"]
    return tpke + pdec + comb + coins


def run_tpke_batched(args, nat, torch, dev, world, inp, d_acc, dd, n, n_cts, n_dec, sh):
    """Randomized batch verify (lcb_ctx_tpke_verify_shares_batched_dev, k_batch.hip) of the same 1M-share batch: same
    timing discipline as the exact path (prepare + verify per step, warmup, barrier + synchronize).  With
    --tpke-streams K the batch is split by ciphertext into K contiguous parts verified concurrently, each by its own
    host thread, library context and HIP stream (the library is re-entrant per context): a part's splitting levels
    are latency-bound launches of < 1 wave per SIMD, and the other parts' randomisation fills the idle SIMDs."""
    import concurrent.futures
    import torch.distributed as dist
    lib = nat.lib()
    d_ct, d_dec, d_ui = dd
    py, nk, pu, pw, pv, pvo, nc = PREP_ARGS[0]
    K = max(1, args.tpke_streams)
    vlen = int(inp["v_off"][1] - inp["v_off"][0])
    bounds = [round(n_cts * k / K) for k in range(K + 1)]
    parts = []
    for k in range(K):
        c0, c1 = bounds[k], bounds[k + 1]
        s0, s1 = c0 * n_dec, min(n, c1 * n_dec)
        if s1 <= s0:
            continue
        ct_local = to_dev(torch, dev, np.ascontiguousarray(inp["ct_idx"][s0:s1] - c0, dtype=np.uint32))
        voff = to_dev(torch, dev, np.arange(0, vlen * (c1 - c0 + 1), vlen, dtype=np.uint32))
        ctx = nat.Context()
        st = torch.cuda.Stream(dev)
        parts.append(dict(c0=c0, nc=c1 - c0, s0=s0, ns=s1 - s0, ct=ct_local, voff=voff, ctx=ctx, stream=st))
    pool = concurrent.futures.ThreadPoolExecutor(max_workers=len(parts))

    single_stream = K > 1 and args.tpke_parts_single_stream

    def one(p):
        if single_stream:       # prepare + verify_prepared on the part's one stream (no second stream per context)
            rc = lib.lcb_ctx_tpke_prepare_dev(p["ctx"].ptr, py, nk, pu + 48 * p["c0"], pw + 96 * p["c0"],
                                              pv + vlen * p["c0"], p["voff"].data_ptr(), p["nc"],
                                              p["stream"].cuda_stream)
            rc |= lib.lcb_ctx_tpke_verify_prepared_batched_dev(
                p["ctx"].ptr, d_acc.data_ptr() + p["s0"], p["ns"], nk, p["nc"], p["ct"].data_ptr(),
                d_dec.data_ptr() + 4 * p["s0"], d_ui.data_ptr() + 48 * p["s0"], p["stream"].cuda_stream)
        else:
            rc = lib.lcb_ctx_tpke_verify_shares_batched_dev(
                p["ctx"].ptr, d_acc.data_ptr() + p["s0"], p["ns"], py, nk, pu + 48 * p["c0"], pw + 96 * p["c0"],
                pv + vlen * p["c0"], p["voff"].data_ptr(), p["nc"], p["ct"].data_ptr(), d_dec.data_ptr() + 4 * p["s0"],
                d_ui.data_ptr() + 48 * p["s0"], p["stream"].cuda_stream)
        if rc != 0:
            raise RuntimeError(nat.last_error())

    def step():
        for f in [pool.submit(one, p) for p in parts]:
            f.result()

    d_acc.fill_(7)
    torch.cuda.synchronize(dev)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    mism = int(np.sum(d_acc.cpu().numpy() != inp["expect"])) if args.warmup > 0 else 0
    d_acc.fill_(7)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    mism += int(np.sum(d_acc.cpu().numpy() != inp["expect"]))
    pool.shutdown()
    levels, ms = [], [0.0] * 6
    for p in parts:
        lv = (ctypes.c_uint32 * 8)()
        m6 = (ctypes.c_float * 6)()
        k = lib.lcb_ctx_tpke_batched_stats(p["ctx"].ptr, lv, m6)
        if k < 0:
            raise RuntimeError(nat.last_error())
        levels.append(list(lv[:k]))
        ms = [max(a, b) for a, b in zip(ms, m6)] if K > 1 else list(m6)
    for p in parts:
        p["ctx"].close()
    if K == 1:
        levels = levels[0]
    ms_points, ms_groups, ms_sum, ms_miller, ms_fe, ms_prep = ms
    t = shard.max_time_sum(dist, torch, dev, elapsed, mism, n)
    elapsed = t[0]
    checks = sum(sum(lv) for lv in levels) if K > 1 else sum(levels)
    ach_pair = checks * (C["C_ML2_NORM2"] + C["C_FE"]) * MAC_PER_FPMUL / ((ms_miller + ms_fe) * 1e-3)
    ach_pts = n * W_RLC_POINTS * MAC_PER_FPMUL / (ms_points * 1e-3)
    step_fpmul = n * W_RLC_POINTS + checks * (C["C_ML2_NORM2"] + C["C_FE"]) + n_cts * W_PREPARE
    step_ach = step_fpmul * MAC_PER_FPMUL / (elapsed / args.steps)
    return dict(
        metric="BLS12-381 TPKE decryption-share verifications/sec, randomized batch check (small-exponent test)",
        value=float(t[2]) * args.steps / elapsed, unit="share verifications/s", steps=args.steps,
        ms_per_step=1e3 * elapsed / args.steps, decision_mismatches=int(t[1]),
        algorithm=("per ciphertext group: e(sum s_i U_i, H) == e(sum s_i Y_i, W), secret s_i = a_i + b_i lambda "
                   "(32-bit a_i, b_i from ChaCha20 keyed by getrandom per call: 2^64 exponents); failed groups "
                   "located (one or two errors: a false location <= len^2 2^-64 per group) or checked singly; "
                   "other rejections exact, false accept <= 2^-64 per group"),
        api="lcb_ctx_tpke_verify_shares_batched_dev (prepare + verify, randomisation on a second stream)",
        concurrent_parts=K,
        levels=levels, group_checks_per_share=checks / n,
        device_ms={"randomise_and_group (beside prepare)": ms_points, "all_levels": ms_groups, "group_sums": ms_sum,
                   "k_tpke_rlc_miller": ms_miller, "k_final_exp_check": ms_fe,
                   "prepare_chain (fused, beside the randomisation)": ms_prep},
        roofline={"bound": "valu_int32",
                  "kernel": ("whole batched step: k_tpke_rlc_points + k_tpke_ct_prepare / k_lineset_fill + "
                             "k_tpke_rlc_miller / k_final_exp_check over all levels"),
                  "achieved": step_ach / 1e12, "peak": PEAK_MAC32 / 1e12, "unit": "Tmac32/s",
                  "frac": step_ach / PEAK_MAC32, "traffic": None, "mac_per_fpmul": MAC_PER_FPMUL,
                  "work_per_step_fpmul": step_fpmul,
                  "work_breakdown_fpmul": {"randomise (per share)": W_RLC_POINTS, "prepare (per ciphertext)": W_PREPARE,
                                           "group check (per group)": C["C_ML2_NORM2"] + C["C_FE"],
                                           "group_checks": checks},
                  "note": ("algorithmic Fp-mul of the step / step time; the splitting levels are launches of < 1 wave "
                           "per SIMD (latency-bound), which the concurrent parts overlap with the other parts' "
                           "randomisation; the full-occupancy rate of the same Miller / final-exponentiation code is "
                           "tpke_exact.roofline"),
                  "kernel_frac": ({"k_tpke_rlc_miller + k_final_exp_check (all levels, one part)": ach_pair / PEAK_MAC32,
                                   "k_tpke_rlc_points (+ k_rlc_groups), beside k_tpke_ct_prepare": ach_pts / PEAK_MAC32}
                                  if K == 1 else None)},
    )


PREP_ARGS = []


def run_tpke_pipelined(args, nat, torch, dev, world, inp, dd, n, n_cts, n_dec, P):
    """--tpke-pipeline P: P whole 1M-share batches in flight.  Each of P host threads owns a library context, a HIP
    stream and an accept buffer and verifies the full batch on its steps (thread t: steps t, t + P, ...); thread t
    starts t/P of a step after thread 0, so one batch's splitting levels (latency-bound launches of < 1 wave per SIMD)
    run beside another batch's randomisation and preparation.  Every step is the complete batched verify of the whole
    batch (prepare + all levels); the timed region covers all args.steps steps, bracketed like the other paths."""
    import concurrent.futures
    import threading
    import torch.distributed as dist
    lib = nat.lib()
    d_ct, d_dec, d_ui = dd
    py, nk, pu, pw, pv, pvo, nc = PREP_ARGS[0]
    lanes = []
    for t in range(P):
        lanes.append(dict(ctx=nat.Context(), stream=torch.cuda.Stream(dev),
                          acc=torch.full((n,), 7, dtype=torch.uint8, device=dev)))
    # every timed step's decisions are kept (one slot per step, copied on the lane's stream after its step) and all of
    # them are compared with the oracle's after the timed region (the last step of each lane only, before)
    slots = torch.full((max(1, args.steps), n), 7, dtype=torch.uint8, device=dev)

    def one(ln, step=None):
        rc = lib.lcb_ctx_tpke_verify_shares_batched_dev(
            ln["ctx"].ptr, ln["acc"].data_ptr(), n, py, nk, pu, pw, pv, pvo, nc, d_ct.data_ptr(), d_dec.data_ptr(),
            d_ui.data_ptr(), ln["stream"].cuda_stream)
        if rc != 0:
            raise RuntimeError(nat.last_error())
        if step is not None:
            with torch.cuda.stream(ln["stream"]):
                slots[step].copy_(ln["acc"], non_blocking=True)
        ln["stream"].synchronize()

    for ln in lanes:                      # warmup: every context once, alone
        for _ in range(max(1, args.warmup)):
            one(ln)
    torch.cuda.synchronize(dev)
    t_one = float("inf")                  # one batch alone, the least of three calls (host wall clock)
    for _ in range(3):
        t0 = time.perf_counter()
        one(lanes[0])
        t_one = min(t_one, time.perf_counter() - t0)
    mism = sum(int(np.sum(ln["acc"].cpu().numpy() != inp["expect"])) for ln in lanes)
    for ln in lanes:
        ln["acc"].fill_(7)
    go = threading.Barrier(P)

    def lane_run(t):
        ln = lanes[t]
        go.wait()
        time.sleep(t_one * t / P)
        for step in range(t, args.steps, P):
            one(ln, step)

    pool = concurrent.futures.ThreadPoolExecutor(max_workers=P)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for f in [pool.submit(lane_run, t) for t in range(P)]:
        f.result()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    pool.shutdown()
    expect_dev = torch.from_numpy(np.ascontiguousarray(inp["expect"]).astype(np.uint8)).to(dev)
    mism += int((slots[:args.steps] != expect_dev.unsqueeze(0)).sum().item())
    del slots
    levels = []
    for ln in lanes:
        lv = (ctypes.c_uint32 * 8)()
        m6 = (ctypes.c_float * 6)()
        k = lib.lcb_ctx_tpke_batched_stats(ln["ctx"].ptr, lv, m6)
        levels.append(list(lv[:max(k, 0)]))
        ln["ctx"].close()
    t = shard.max_time_sum(dist, torch, dev, elapsed, mism, n)
    elapsed = t[0]
    checks = sum(levels[0])
    step_fpmul = n * W_RLC_POINTS + checks * (C["C_ML2_NORM2"] + C["C_FE"]) + n_cts * W_PREPARE
    step_ach = step_fpmul * MAC_PER_FPMUL / (elapsed / args.steps)
    return dict(
        metric="BLS12-381 TPKE decryption-share verifications/sec, randomized batch check (small-exponent test)",
        value=float(t[2]) * args.steps / elapsed, unit="share verifications/s", steps=args.steps,
        ms_per_step=1e3 * elapsed / args.steps, decision_mismatches=int(t[1]),
        algorithm=("per ciphertext group: e(sum s_i U_i, H) == e(sum s_i Y_i, W), secret s_i = a_i + b_i lambda "
                   "(32-bit a_i, b_i from ChaCha20 keyed by getrandom per call: 2^64 exponents); failed groups "
                   "located (one or two errors: a false location <= len^2 2^-64 per group) or checked singly; "
                   "other rejections exact, false accept <= 2^-64 per group; every step's decisions checked"),
        api=f"lcb_ctx_tpke_verify_shares_batched_dev, {P} batches in flight (contexts / streams / host threads)",
        pipeline=P, single_batch_ms=1e3 * t_one, levels=levels[0],
        roofline={"bound": "valu_int32",
                  "kernel": ("whole batched step: k_tpke_rlc_points + k_tpke_ct_prepare_hw + coop Miller / "
                             "k_final_exp_check over all levels"),
                  "achieved": step_ach / 1e12, "peak": PEAK_MAC32 / 1e12, "unit": "Tmac32/s",
                  "frac": step_ach / PEAK_MAC32, "traffic": None, "mac_per_fpmul": MAC_PER_FPMUL,
                  "work_per_step_fpmul": step_fpmul})

LINE_MAX_BYTES = 6144    # the driver keeps only the tail of stdout (≈ 8 KB incl. stderr): the headline must fit in it


def _short(s, n=160):
    s = str(s)
    return s if len(s) <= n else s[:n - 3] + "..."


def _r(x, d=4):
    """Round a float for the compact line (relative precision: 6 significant digits)."""
    if isinstance(x, float):
        return float(f"{x:.6g}")
    return x


def _pick(d, *keys):
    if not d:
        return None
    return {k: _r(d[k]) for k in keys if k in d and d[k] is not None}


def compact_line(full):
    """The driver-facing headline: the contract keys, the headline roofline and CPU baseline, the exact path's
    like-for-like numbers, and one short summary per sub-bench.  Everything else stays in the detail record
    (`bench_detail_<hash>.json` and the `BENCH_DETAIL` stdout line printed before this one)."""
    rf = full.get("roofline") or {}
    cpu = full.get("cpu_baseline") or {}
    cfg = full.get("config") or {}
    line = {k: full[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                 "higher_is_better", "scaling", "vs_baseline", "dtype", "data") if k in full}
    line["config"] = {k: cfg[k] for k in ("workload", "shares_per_rank", "ciphertexts_per_rank", "decryptors",
                                          "degree", "corrupted_fraction", "parallelism", "decision_mismatches")
                      if k in cfg}
    if "algorithm" in cfg:
        line["config"]["algorithm"] = _short(cfg["algorithm"], 120)
    line["roofline"] = {k: _r(rf[k]) for k in ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic")
                        if k in rf}
    if "kernel" in rf:
        line["roofline"]["kernel"] = _short(rf["kernel"], 120)
    if rf.get("traffic_source"):
        line["roofline"]["traffic_source"] = _short(rf["traffic_source"], 100)
    if rf.get("kernel_frac"):
        line["roofline"]["kernel_frac"] = {_short(k, 48): _r(v) for k, v in rf["kernel_frac"].items()}
    if cpu:
        line["cpu_baseline"] = {k: _r(cpu[k]) for k in ("value", "unit", "cores", "kind") if k in cpu}
        line["cpu_baseline"]["sample"] = _short(cpu.get("sample", ""), 200)
        for k in ("amortized_exact", "as_reference"):
            if cpu.get(k):
                line["cpu_baseline"][k] = _r(cpu[k].get("value"))
    else:
        line["cpu_baseline"] = None
    line["source_hash"] = full.get("source_hash")
    ex = full.get("tpke_exact")
    if ex:
        exr = ex.get("roofline") or {}
        line["tpke_exact"] = {"value": _r(ex.get("value")), "ms_per_step": _r(ex.get("ms_per_step")),
                              "decision_mismatches": ex.get("decision_mismatches"),
                              "roofline": {"kernel": exr.get("kernel"), "frac": _r(exr.get("frac")),
                                           "traffic": _r(exr.get("traffic")),
                                           "kernel_ms": {k: _r(v) for k, v in (exr.get("kernel_ms") or {}).items()}}}
    else:
        line["tpke_exact"] = None
    tb = full.get("tpke_batched") or {}
    if tb.get("single_batch"):                # pipelined headline: the one-batch-at-a-time rate beside it
        sb = tb["single_batch"]
        line["tpke_single_batch"] = {k: _r(sb.get(k)) for k in ("value", "ms_per_step", "decision_mismatches",
                                                                "roofline_frac")}
        line["config"]["batches_in_flight"] = tb.get("pipeline")
        line["config"]["single_batch_latency_ms"] = _r(tb.get("single_batch_ms"))
    for k in ("hw_queues", "hw_queues_env"):
        if cfg.get(k):
            line["config"][k] = cfg[k]
    s = {}
    byz = full.get("tpke_byzantine")
    if byz:
        s["tpke_byzantine"] = {"worst_batched_over_exact": _r(byz.get("worst_batched_over_exact")),
                               "mismatches": sum(int((p.get("batched") or {}).get("decision_mismatches", 0)) +
                                                 int((p.get("exact") or {}).get("decision_mismatches", 0))
                                                 for p in (byz.get("patterns") or {}).values())}
    if full.get("msm"):
        s["msm"] = [{"points": m.get("total_points"), "value": _r(m.get("value")), "ms": _r(m.get("ms_per_step")),
                     "known_answer_ok": m.get("known_answer_ok"),
                     "frac": _r((m.get("roofline") or {}).get("frac"))} for m in full["msm"]]
    ts = full.get("threshold_signature")
    if ts:
        s["threshold_signature"] = {"value": _r(ts.get("value")), "unit": ts.get("unit"),
                                    "ms_per_step": _r(ts.get("ms_per_step")),
                                    "mismatches": ts.get("decision_mismatches"), "phase_ms": {
                                        _short(k, 24): _r(v) for k, v in (ts.get("phase_ms") or {}).items()},
                                    "exact": _r((ts.get("exact") or {}).get("value")),
                                    "cpu": _r((ts.get("cpu_baseline") or {}).get("value"))}
        if (ts.get("roofline") or {}).get("frac") is not None:
            s["threshold_signature"]["frac"] = _r(ts["roofline"]["frac"])
    for key, vk in (("epoch_replay", "mismatches"), ("ecdsa_headers", "decision_mismatches")):
        sub = full.get(key)
        if sub:
            s[key] = {"value": _r(sub.get("value")), "unit": sub.get("unit"), "mismatches": sub.get(vk),
                      "cpu": _r((sub.get("cpu_baseline") or {}).get("value"))}
            if (sub.get("roofline") or {}).get("frac") is not None:
                s[key]["frac"] = _r(sub["roofline"]["frac"])
    for key in ("dkg", "rbc_erasure_coding"):
        sub = full.get(key)
        if sub:
            s[key] = {"value": _r(sub.get("value")), "unit": sub.get("unit"),
                      "cpu": _r((sub.get("cpu_baseline") or {}).get("value"))}
    ml = full.get("mcl_latency")
    if ml:
        s["mcl_latency_us"] = {k: _r(v) for k, v in (ml.get("gpu") or {}).items()}
    line["summary"] = s
    text = json.dumps(line, separators=(",", ":"))
    if len(text) > LINE_MAX_BYTES:            # never let the line outgrow the driver's tail: drop the summaries
        line["summary"] = {"dropped": "line too long; see the BENCH_DETAIL record"}
    return line


def emit(full, write_file=True):
    """Print the detail record first (one line, prefixed so it never parses as the headline), write it under
    gpurun_out/ when that exists, then the compact headline as the LAST stdout line."""
    detail = json.dumps(full)
    print("BENCH_DETAIL " + detail, flush=True)
    out = os.path.join(ROOT, "gpurun_out")
    if write_file and os.path.isdir(out):
        try:
            with open(os.path.join(out, f"bench_detail_{full.get('source_hash')}.json"), "w") as fh:
                fh.write(detail + "\n")
        except OSError:
            pass
    sys.stderr.flush()
    print(json.dumps(compact_line(full), separators=(",", ":")), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=12,
                    help="timed TPKE steps (batches); 12 by default so that the default four batches in flight each run "
                         "three (at 3 steps one of the four contexts idles and the line under-reports the pipeline)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--shares", type=int, default=1048576)
    ap.add_argument("--n", type=int, default=22)
    ap.add_argument("--f", type=int, default=7)
    ap.add_argument("--vlen", type=int, default=32)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--tpke-batched", type=int, default=1, help="time the randomized batch verify (0 = skip)")
    ap.add_argument("--tpke-exact", type=int, default=1, help="time the exact per-share verify (0 = skip)")
    ap.add_argument("--tpke-parts-single-stream", type=int, default=0,
                    help="with --tpke-streams K > 1: each part prepares and verifies on one stream")
    ap.add_argument("--tpke-streams", type=int, default=1,
                    help="batched verify: concurrent parts (contexts / streams / host threads) per step; measured "
                         "no faster with 2 or 3 parts (147 - 159 vs 145 ms per 1M shares)")
    ap.add_argument("--hw-queues", type=int, default=int(os.environ.get("LCB_BENCH_HWQ", "0")),
                    help="GPU_MAX_HW_QUEUES for this process (0, the default: keep the environment's, the box's 4; "
                         "round 6 stopped overriding it: every hardware queue can hold a full-device scratch "
                         "reservation, DESIGN.md §14.1).  The environment's value is recorded in the line "
                         "(config.hw_queues_env) beside the one used (config.hw_queues)")
    ap.add_argument("--tpke-pipeline", type=int, default=4,
                    help="batched verify: whole batches in flight (each on its own context / stream / host thread); "
                         "round 4: 2 measured 12.3 vs 10.6 M shares/s for one at a time, 3 no better (profiles/r04/q1, "
                         "q2); round 5, with the preparation at 256 registers: 3 gives 14.98 vs 14.57 M/s for 2 "
                         "(profiles/r05/pipeline.txt); round 6, with the merged preparation (fork mode 4): 4 gives 17.14 vs 16.93 M/s "
                         "for 3, every pair of three (profiles/r06/ab_kernels/pipeline4.txt)")
    ap.add_argument("--headline", choices=("batched", "exact"), default="batched",
                    help="which TPKE path the line's value / roofline / cpu_baseline describe")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--pattern-steps", type=int, default=2,
                    help="timed steps per Byzantine pattern and path (0 = skip the patterns)")
    ap.add_argument("--patterns", default="", help="comma-separated subset of the Byzantine patterns (default all)")
    ap.add_argument("--coop-miller-max", type=int, default=-1,
                    help="levels of <= this many group checks run their Miller loops cooperatively (-1: default)")
    ap.add_argument("--fork-mode", type=int, default=-1,
                    help="fused batched verify stream layout (lcb_set_fork_mode; -1: library default)")
    ap.add_argument("--coop-max", type=int, default=-1,
                    help="levels of <= this many group checks on the nine-lane cooperative kernels (-1: library default)")
    ap.add_argument("--msm-sizes", default=f"{1 << 20},{1 << 24}",
                    help="total G1 MSM points per measurement, sharded over ranks (empty = skip)")
    ap.add_argument("--msm-steps", type=int, default=3)
    ap.add_argument("--msm-pipeline", type=int, default=2,
                    help="independent MSMs in flight (one context + stream each); 1 = one at a time")
    ap.add_argument("--msm-no-glv", action="store_true", help="plain 255-bit Pippenger instead of the GLV form")
    ap.add_argument("--msm-glv-window", type=int, default=0, help="A/B: the GLV form at this window width")
    ap.add_argument("--ts-rounds", type=int, default=65536, help="CommonCoin rounds per rank (0 = skip)")
    ap.add_argument("--ts-n", type=int, default=100)
    ap.add_argument("--ts-steps", type=int, default=1)
    ap.add_argument("--ts-batched", type=int, default=1, help="time the randomized batch share check (0 = skip)")
    ap.add_argument("--ts-exact", type=int, default=1, help="time the exact per-share check (0 = skip)")
    ap.add_argument("--replay-n", type=int, default=256, help="epoch-replay network size N (0 = skip)")
    ap.add_argument("--replay-steps", type=int, default=1)
    ap.add_argument("--replay-exact", type=int, default=0, help="epoch replay with the exact per-share checks")
    ap.add_argument("--replay-concurrent", type=int, default=1,
                    help="epoch replay: 1 = the TPKE and coin chains side by side (own host thread, context, stream); "
                         "0 = one after the other.  Round 4 kept this off after the CommonCoin assembly's 22.7 KB of "
                         "scratch per lane on two hardware queues aborted the process (HSA_STATUS_ERROR_OUT_OF_RESOURCES); "
                         "round 5 moved every multi-wave kernel to <= 4 KB (lanetab.hpp workspaces) and gates larger "
                         "reservations onto one stream per device (lcb_set_scratch_gate)")
    ap.add_argument("--ecdsa-sigs", type=int, default=1 << 20, help="header signatures per rank (0 = skip)")
    ap.add_argument("--ecdsa-validators", type=int, default=256)
    ap.add_argument("--ecdsa-steps", type=int, default=3)
    ap.add_argument("--dkg-n", type=int, default=256, help="DKG dealers (0 = skip)")
    ap.add_argument("--dkg-f", type=int, default=85)
    ap.add_argument("--rs-n", type=int, default=256, help="RBC shards (0 = skip)")
    ap.add_argument("--rs-bytes", type=int, default=1 << 24)
    ap.add_argument("--mcl-reps", type=int, default=30, help="per-call latency samples of the mcl surface (0 = skip)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    HWQ_ENV = os.environ.get("GPU_MAX_HW_QUEUES")
    if args.hw_queues > 0:
        # hardware queues per process, read when the HIP runtime starts (before torch / the library touch the GPU);
        # an A/B knob only (the default 0 keeps the environment's value), the line records both
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, args.hw_queues))
    import torch
    import torch.distributed as dist
    from lachain_amd import native as nat

    if world > 1:
        # RCCL over xGMI on the 8-GPU node; LCB_BENCH_BACKEND=gloo runs the same code with host collectives (the
        # world-size-2 test on a one-GPU box, where both ranks share the device)
        dist.init_process_group(os.environ.get("LCB_BENCH_BACKEND", "nccl"), init_method="env://")
    gpu = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    nat.load(False).lcb_set_device(gpu)
    nat.lib()
    if args.coop_max >= 0 or args.fork_mode >= 0 or args.coop_miller_max >= 0:
        os.environ["LCB_ALLOW_TUNING"] = "1"          # A/B runs only: the default line never touches the hooks
    if args.coop_max >= 0:
        nat.set_coop_max(args.coop_max)
    if args.fork_mode >= 0:
        nat.set_fork_mode(args.fork_mode)
    if args.coop_miller_max >= 0:
        nat.set_coop_miller_max(args.coop_miller_max)
    if os.environ.get("LCB_WAVE_PRIO"):           # A/B of the latency kernels' wave priority
        nat.set_wave_priority(int(os.environ["LCB_WAVE_PRIO"]))
    if os.environ.get("LCB_MSM_SEGS"):            # A/B of the bucket-reduction lane count
        nat.set_msm_segments(int(os.environ["LCB_MSM_SEGS"]))
    if os.environ.get("LCB_KEYS_FIRST"):          # A/B of the key tables' place in the fused batched calls
        nat.set_keys_first(int(os.environ["LCB_KEYS_FIRST"]))
    if os.environ.get("LCB_LINES_COOP"):          # A/B of the five-lane line-set kernel's size limit
        nat.set_lines_coop_max(int(os.environ["LCB_LINES_COOP"]))
    if os.environ.get("LCB_MSM_CHUNK"):           # A/B of the MSM bucket accumulation (0: one lane per bucket)
        nat.set_msm_chunk(int(os.environ["LCB_MSM_CHUNK"]))

    progress(f"inputs: {args.shares} TPKE shares")
    t_gen = time.perf_counter()
    inp = make_inputs(nat, rank, args.shares, args.n, args.f, args.vlen)
    t_gen = time.perf_counter() - t_gen
    n, n_cts, n_dec = args.shares, inp["n_cts"], inp["n_dec"]

    d_y = to_dev(torch, dev, inp["y_keys"])
    d_u = to_dev(torch, dev, inp["u"])
    d_w = to_dev(torch, dev, inp["w"])
    d_v = to_dev(torch, dev, inp["v"])
    d_voff = to_dev(torch, dev, inp["v_off"])
    d_ct = to_dev(torch, dev, inp["ct_idx"])
    d_dec = to_dev(torch, dev, inp["dec_idx"])
    d_ui = to_dev(torch, dev, inp["ui"])
    d_acc = torch.zeros(n, dtype=torch.uint8, device=dev)
    lib = nat.lib()
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    PREP_ARGS.append((d_y.data_ptr(), n_dec, d_u.data_ptr(), d_w.data_ptr(), d_v.data_ptr(), d_voff.data_ptr(), n_cts))

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        rc = lib.lcb_tpke_prepare_dev(d_y.data_ptr(), n_dec, d_u.data_ptr(), d_w.data_ptr(), d_v.data_ptr(),
                                      d_voff.data_ptr(), n_cts, sh)
        if ev is not None:
            ev[1].record(stream)
        rc |= lib.lcb_tpke_verify_prepared_dev(d_acc.data_ptr(), n, n_dec, n_cts, d_ct.data_ptr(), d_dec.data_ptr(),
                                               d_ui.data_ptr(), sh)
        if ev is not None:
            ev[2].record(stream)
        if rc != 0:
            raise RuntimeError(nat.last_error())

    exact = None
    if args.tpke_exact:
        progress("TPKE exact verify")
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize(dev)
        mismatches = 0
        if args.warmup > 0:
            got = d_acc.cpu().numpy()
            mismatches = int(np.sum(got != inp["expect"]))
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for k in range(args.steps):
            step(evs[k])
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        prep_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
        ver_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps
        kms = (ctypes.c_float * 2)()
        if lib.lcb_tpke_verify_phase_ms(kms) != 0:      # the two kernels of the last timed step (library events)
            raise RuntimeError(nat.last_error())
        miller_ms, fexp_ms = float(kms[0]), float(kms[1])
        got = d_acc.cpu().numpy()
        mismatches += int(np.sum(got != inp["expect"]))
        t = shard.max_time_sum(dist, torch, dev, elapsed, mismatches, n)
        elapsed = t[0]
        achieved = n * W_VERIFY * MAC_PER_FPMUL / (ver_ms * 1e-3)
        exact = dict(
            metric="BLS12-381 TPKE decryption-share verifications/sec, exact per-share check (the reference's "
                   "algorithm: one pairing-product check per share)",
            value=float(t[2]) * args.steps / float(t[0]), unit="share verifications/s", steps=args.steps,
            ms_per_step=1e3 * float(t[0]) / args.steps, decision_mismatches=int(t[1]),
            api="lcb_tpke_prepare_dev + lcb_tpke_verify_prepared_dev",
            roofline={"bound": "valu_int32", "kernel": "k_tpke_miller + k_final_exp_check",
                      "achieved": achieved / 1e12, "peak": PEAK_MAC32 / 1e12, "unit": "Tmac32/s",
                      "frac": achieved / PEAK_MAC32, "work_per_share_fpmul": W_VERIFY,
                      "mac_per_fpmul": MAC_PER_FPMUL, "verify_ms": ver_ms, "prepare_ms": prep_ms,
                      "kernel_ms": {"k_tpke_miller": miller_ms, "k_final_exp_check": fexp_ms},
                      "kernel_frac": {
                          "k_tpke_miller": n * (C["C_DEC1"] + C["C_ML2_NORM2"]) * MAC_PER_FPMUL
                          / (miller_ms * 1e-3) / PEAK_MAC32,
                          "k_final_exp_check": n * C["C_FE"] * MAC_PER_FPMUL / (fexp_ms * 1e-3) / PEAK_MAC32}})
    batched = None
    if args.tpke_batched:
        progress("TPKE batched verify")
        batched = run_tpke_batched(args, nat, torch, dev, world, inp, d_acc, (d_ct, d_dec, d_ui), n, n_cts, n_dec, sh)
        if args.tpke_pipeline > 1 and args.tpke_streams <= 1:
            # batches in flight: the headline is the pipelined rate; the one-batch-at-a-time rate stays in the record
            progress(f"TPKE batched verify, {args.tpke_pipeline} batches in flight")
            piped = run_tpke_pipelined(args, nat, torch, dev, world, inp, (d_ct, d_dec, d_ui), n, n_cts, n_dec,
                                       args.tpke_pipeline)
            piped["single_batch"] = {k: batched[k] for k in ("value", "ms_per_step", "decision_mismatches", "levels")
                                     if k in batched}
            piped["single_batch"]["roofline_frac"] = batched["roofline"]["frac"]
            piped["device_ms"] = batched.get("device_ms")
            batched = piped
    byz = None
    if args.pattern_steps > 0:
        progress("Byzantine patterns")
        byz = run_tpke_patterns(args, nat, torch, dev, world, inp, n, n_cts, n_dec)
    head = batched if (args.headline == "batched" and batched) else exact
    if head is None:
        raise SystemExit("nothing to report: --tpke-exact 0 and --tpke-batched 0")
    msm = ts = replay = ecdsa = dkg = rs = mcl_lat = None
    if args.mcl_reps > 0 and world == 1:
        progress("mcl latency")
        mcl_lat = run_mcl_latency(args, nat, rank)
    if args.dkg_n > 0 and world == 1:
        progress("DKG")
        dkg = run_dkg(args, nat, rank)
    if args.rs_n > 0 and world == 1:
        progress("RBC erasure coding")
        rs = run_rs(args, nat, rank)
    if args.ecdsa_sigs > 0:
        progress("ECDSA headers")
        ecdsa = run_ecdsa(args, nat, torch, dev, rank, world, cpu=(world == 1 and not args.no_cpu_baseline))
    if args.replay_n > 0:
        progress("epoch replay")
        replay = run_replay(args, nat, torch, dev, rank, world)
    if args.ts_rounds > 0:
        progress("threshold signatures")
        ts = run_ts(args, nat, torch, dev, rank, world)
    if args.msm_sizes:
        msm = run_msm_sizes(args, nat, torch, dev, rank, world, cpu=(world == 1 and not args.no_cpu_baseline))
    if rank == 0:
        # HBM bytes per launch of the group-check / verify pair from the committed PMC passes, only if they were taken
        # on THIS build (the file carries the source hash of the kernels it profiled; tools/pmc_to_json.py)
        traffic, traffic_note = None, "no PMC file for this build"
        src_hash = source_hash()
        pmc = os.path.join(ROOT, "profiles", "pmc_tpke_verify.json")
        if os.path.exists(pmc):
            with open(pmc) as fh:
                pj = json.load(fh)
            if pj.get("source_hash") == src_hash:
                traffic = pj.get("hbm_bytes_per_launch_at_bench_size")
                traffic_note = (f"{pmc[len(ROOT) + 1:]}: FETCH_SIZE x2 + WRITE_SIZE (KB->B) of k_tpke_miller + "
                                f"k_final_exp_check at the bench launch size, source hash {src_hash}")
            else:
                traffic_note = f"stale PMC file (profiled {pj.get('source_hash')}, this build {src_hash}): not reported"
        if exact is not None:
            exact["roofline"]["traffic"] = traffic
            exact["roofline"]["traffic_source"] = traffic_note
        if batched is not None:          # the whole batched step's HBM bytes (tools/pmc_batched_to_json.py)
            pmcb = os.path.join(ROOT, "profiles", "pmc_tpke_batched.json")
            bt, bnote = None, "no batched PMC file for this build"
            if os.path.exists(pmcb):
                with open(pmcb) as fh:
                    pb = json.load(fh)
                if pb.get("source_hash") == src_hash:
                    bt = pb.get("hbm_bytes_per_step")
                    bnote = (f"{pmcb[len(ROOT) + 1:]}: FETCH_SIZE x2 + WRITE_SIZE (KB->B) summed over the step's "
                             f"dispatches, source hash {src_hash}")
                else:
                    bnote = f"stale PMC file (profiled {pb.get('source_hash')}, this build {src_hash}): not reported"
            batched["roofline"]["traffic"] = bt
            batched["roofline"]["traffic_source"] = bnote
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            progress("TPKE CPU baseline")
            cpu = cpu_baseline(inp, args.cpu_seconds, batched=batched is not None)
        if head is batched:
            roofline = dict(batched.pop("roofline"))
            cpu_line = cpu
            algo = batched["algorithm"]
        else:
            roofline = dict(exact.pop("roofline"))
            cpu_line = cpu
            algo = "exact per-share check"
        line = {
            "metric": "BLS12-381 TPKE decryption-share verifications/sec (batched VerifyShare, N=22 F=7)",
            "value": head["value"], "unit": "share verifications/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": head["ms_per_step"], "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32 (381-bit Montgomery, 12x32-bit limbs)", "data": "synthetic",
            "config": {"workload": "configs[1]: 1M TPKE decryption shares, N=22 F=7 validators, one MI355X per rank",
                       "shares_per_rank": n, "ciphertexts_per_rank": n_cts, "decryptors": n_dec, "degree": args.f,
                       "v_bytes": args.vlen, "corrupted_fraction": 0.01, "parallelism": f"shard{world}",
                       "decision_mismatches": head["decision_mismatches"], "algorithm": algo, "api": head["api"],
                       "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"), "hw_queues_env": HWQ_ENV},
            "roofline": roofline,
            "source_hash": src_hash,
            "cpu_baseline": cpu_line,
            "tpke_batched": batched if head is batched else None,
            "tpke_exact": exact,
            "tpke_byzantine": byz,
            "input_gen_s": t_gen,
            "msm": msm,
            "threshold_signature": ts,
            "epoch_replay": replay,
            "ecdsa_headers": ecdsa,
            "dkg": dkg,
            "rbc_erasure_coding": rs,
            "mcl_latency": mcl_lat,
        }
        emit(line)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
