"""stage dumps of the TPKE two-error search (k_tpke_rlc_search2b) for the row-(ns + g) build and the
open-list-position build (-DLCB_SEARCH2B_BY_POSITION=1, tools/build_variant.sh), on the same batch with the same fixed
exponent key, so the gamma rows of both runs are the same field elements.

  run:      LCB_ALLOW_TEST_HOOKS=1 LCB_ALLOW_FIXED_BATCH_SEED=1 LCB_ALLOW_TUNING=1 python tools/debug/search2b_ab.py run TAG
            (LCB_LIB_PATH selects the build; dumps go to gpurun_out/s2b/TAG.{in,out}.N.bin)
  compare:  python tools/debug/search2b_ab.py compare gpurun_out/s2b/base gpurun_out/s2b/pos

The batch is the eight-ciphertext two-error pattern of tests/test_gpu_batched.py tiled `reps` times (N = 22, F = 7).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run(tag, reps=256):
    import torch
    from helpers import gpu_native
    import test_gpu_batched as tb
    nat = gpu_native()
    dev = torch.device("cuda", 0)
    out = os.path.join(ROOT, "gpurun_out", "s2b")
    os.makedirs(out, exist_ok=True)
    os.environ["LCB_DUMP_SEARCH2B"] = os.path.join(out, tag)
    b = tb.Batch(b"gpu-batched-two-errors", 22, 7, 8)
    rows = [list(r) for r in b.good]
    bad = {1: [5], 2: [0, 21], 3: [3, 4], 4: [1, 7, 12], 5: [9], 6: [10], 7: [6]}
    for r, pos in bad.items():
        for j in pos:
            rows[r][j] = b.bad[r][j]
    rows[5][2] = rows[5][2][::-1]
    rows[6][11] = rows[6][12]
    rows[7][17] = tb.off_subgroup_g1(b.d)
    base = [s for r in rows for s in r]
    expect = np.array([b.expect(i // 22, i % 22, base[i]) for i in range(len(base))], dtype=np.uint8)
    ct = np.tile(np.repeat(np.arange(8, dtype=np.uint32), 22), reps)
    dec = np.tile(np.arange(22, dtype=np.uint32), 8 * reps)
    nat.set_batch_census(0)
    nat.set_batch_seed(bytes(range(32)))
    res = []
    for it in range(int(os.environ.get("S2B_ITERS", "3"))):
        got = tb.run_dev(nat, (torch, dev), b, ct, dec, b"".join(base) * reps)
        levels, _ = nat.tpke_batched_stats()
        res.append(dict(iteration=it, levels=levels, mismatches=int(np.sum(got != np.tile(expect, reps)))))
        print(json.dumps(dict(tag=tag, by_position=int(nat.lib().lcbk_search2b_by_position()) if hasattr(
            nat.lib(), "lcbk_search2b_by_position") else None, **res[-1])), flush=True)
    return res


def load(path):
    raw = open(path, "rb").read()
    ns, no, n, bypos = np.frombuffer(raw[:16], dtype="<u4")
    o = 16
    op = np.frombuffer(raw[o:o + 4 * (no + 4)], dtype="<u4"); o += 4 * (no + 4)
    g0 = np.frombuffer(raw[o:o + 4 * ns * 144], dtype="<u4").reshape(ns, 144); o += 4 * ns * 144
    gg = np.frombuffer(raw[o:o + 8 * ns * 144], dtype="<u4").reshape(2 * ns, 144); o += 8 * ns * 144
    acc = np.frombuffer(raw[o:o + n], dtype=np.uint8)
    return dict(ns=int(ns), no=int(no), n=int(n), bypos=int(bypos), open=op[4:4 + no], count=int(op[0]), g0=g0,
                gg=gg, acc=acc)


def compare(pa, pb, call=0):
    A, B = load(f"{pa}.in.{call}.bin"), load(f"{pb}.in.{call}.bin")
    Ao, Bo = load(f"{pa}.out.{call}.bin"), load(f"{pb}.out.{call}.bin")
    rep = dict(ns=(A["ns"], B["ns"]), n_open=(A["no"], B["no"]), by_position=(A["bypos"], B["bypos"]))
    rep["open_sets_equal"] = bool(set(A["open"].tolist()) == set(B["open"].tolist()))
    rep["open_order_equal"] = bool(np.array_equal(A["open"], B["open"]))
    rep["gamma0_equal"] = bool(np.array_equal(A["g0"], B["g0"]))
    rep["gamma_c_equal"] = bool(np.array_equal(A["gg"][:A["ns"]], B["gg"][:B["ns"]]))

    def gt_rows(D):
        ns = D["ns"]
        return {int(g): D["gg"][ns + (k if D["bypos"] else g)] for k, g in enumerate(D["open"])}

    ra, rb = gt_rows(A), gt_rows(B)
    rep["gamma_t_equal_by_group"] = bool(all(np.array_equal(ra[g], rb[g]) for g in ra))
    rep["accept_in_equal"] = bool(np.array_equal(A["acc"], B["acc"]))
    rep["accept_out_equal"] = bool(np.array_equal(Ao["acc"], Bo["acc"]))
    rep["accept_out_rejects"] = (int(np.sum(Ao["acc"] == 0)), int(np.sum(Bo["acc"] == 0)))
    print(json.dumps(rep))
    return rep


# ---------------------------------------------------------------- in-kernel records (diagnostic builds)
def _fp12_words(gt):
    """canonical GT bytes (oracle) -> the device's 144 Montgomery words"""
    import oracle as o
    w = []
    for i in range(12):
        x = int.from_bytes(gt[48 * i:48 * i + 48], "little") * (1 << 384) % o.P
        w += [(x >> (32 * t)) & 0xffffffff for t in range(12)]
    return w


def _row_gt(row):
    import oracle as o
    rinv = pow(1 << 384, -1, o.P)
    out = b""
    for i in range(12):
        x = sum(int(row[12 * i + t]) << (32 * t) for t in range(12))
        out += (x * rinv % o.P).to_bytes(48, "little")
    return out


def _conj(gt):
    import oracle as o
    out = gt[:288]
    for i in range(6, 12):
        x = int.from_bytes(gt[48 * i:48 * i + 48], "little")
        out += ((o.P - x) % o.P).to_bytes(48, "little")
    return out


def _fpr(words):
    h = 0
    for w in words:
        h = (((h << 5) | (h >> 27)) & 0xffffffff) ^ w
    return h


def check_records(prefix, call=0, positions=3):
    """recompute D_j, E_j and gamma_c^-(c_j+1) from the dumped rows and compare their fingerprints with the kernel's"""
    import oracle as o
    raw = open(f"{prefix}.out.{call}.bin", "rb").read()
    D = load(f"{prefix}.out.{call}.bin")
    ns, no = D["ns"], D["no"]
    base = 16 + 4 * (no + 4) + 4 * ns * 144 + 8 * ns * 144 + D["n"]
    rec = np.frombuffer(raw[base:base + 4 * no * 32 * 8], dtype="<u4").reshape(no, 32, 8)
    Din = load(f"{prefix}.in.{call}.bin")
    report = []
    for k in range(positions):
        g = int(D["open"][k])
        g0, gc = _row_gt(Din["g0"][g]), _row_gt(Din["gg"][g])
        gt = _row_gt(Din["gg"][ns + (k if D["bypos"] else g)])
        p0, pc = g0, gc
        bad = []
        for j in range(22):
            cj = j + 1
            d_ = o.gt_mul(gc, _conj(p0))                       # gamma_c / gamma_0^(c_j)
            pc1 = o.gt_mul(pc, gc)                             # gamma_c^(c_j + 1)
            b_ = _conj(pc1)
            e_ = o.gt_mul(o.gt_mul(gt, gt), b_)
            want = (_fpr(_fp12_words(d_)), _fpr(_fp12_words(e_)), _fpr(_fp12_words(b_)), g)
            got = tuple(int(x) for x in rec[k, j, :4])
            if want != got:
                bad.append(dict(lane=j, want=[hex(x) for x in want], got=[hex(x) for x in got]))
            p0 = o.gt_mul(p0, g0)
            pc = o.gt_mul(pc, gc)
        found = [int(x) for x in rec[k, :22, 4]]
        report.append(dict(k=k, g=g, found=found, mismatched_lanes=len(bad), first=bad[:3]))
        print(json.dumps(report[-1]), flush=True)
    return report


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 256)
    elif sys.argv[1] == "records":
        check_records(sys.argv[2])
    else:
        compare(sys.argv[2], sys.argv[3], int(sys.argv[4]) if len(sys.argv) > 4 else 0)
