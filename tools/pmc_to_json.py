#!/usr/bin/env python3
"""Fold rocprofv3 --pmc passes (tools/pmc_round.sh) into profiles/<name>.json.

Corrections per /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are KB; gfx950 FETCH_SIZE
reports half the bytes of wide coalesced reads, so it is doubled.  The PMC launch verifies `--pmc-shares` shares;
per-launch figures are scaled to the bench launch (`--bench-shares`).  The verify phase of the bench is the
k_tpke_miller + k_final_exp_check pair; its HBM bytes per bench launch become bench.py's roofline.traffic.
Usage: pmc_to_json.py OUT.json PMC_SHARES BENCH_SHARES counter_collection.csv...
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import source_hash  # noqa: E402

out, pmc_n, bench_n, paths = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4:]
# per (kernel, grid size): the bench command launches the same kernels for several workloads (TPKE, CommonCoin,
# MSM), so counters are kept per dispatch shape; the verify phase is the TPKE launch of PMC_SHARES lanes
tot = collections.defaultdict(lambda: collections.defaultdict(float))
meta = {}
for path in paths:
    for r in csv.DictReader(open(path)):
        k = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size"]))
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[k] = {x: r.get(x) for x in ("VGPR_Count", "Accum_VGPR_Count", "Scratch_Size", "LDS_Block_Size")}
kernels = {f"{k[0]}@{k[1]}": dict(meta[k], grid_lanes=k[1], **c) for k, c in tot.items() if k[0].startswith("k_")}
scale = bench_n / pmc_n
verify = {}
for k in ("k_tpke_miller", "k_final_exp_check"):
    c = kernels.get(f"{k}@{pmc_n}", {})
    fetch = 2 * 1024 * c.get("FETCH_SIZE", 0.0)
    write = 1024 * c.get("WRITE_SIZE", 0.0)
    w = c.get("SQ_WAVES", 0.0) or 1.0
    verify[k] = {"fetch_bytes_corrected": fetch, "write_bytes": write,
                 "hbm_bytes_per_share": (fetch + write) / pmc_n,
                 "valu_insts_per_wave": c.get("SQ_INSTS_VALU", 0.0) / w,
                 "vmem_rd_per_wave": c.get("SQ_INSTS_VMEM_RD", 0.0) / w,
                 "vmem_wr_per_wave": c.get("SQ_INSTS_VMEM_WR", 0.0) / w,
                 "valu_active_frac_of_wave_cycles": c.get("SQ_ACTIVE_INST_VALU", 0.0) / (c.get("SQ_WAVE_CYCLES", 0.0) or 1.0),
                 "scratch_bytes_per_lane": float(c.get("Scratch_Size") or 0)}
per_launch = sum(v["fetch_bytes_corrected"] + v["write_bytes"] for v in verify.values()) * scale
doc = {"source": f"rocprofv3 --pmc, separate passes per counter group (tools/pmc_round.sh), one launch of "
                 f"{pmc_n} shares; per-launch bytes scaled x{scale:g} to the {bench_n}-share bench launch",
       "correction": "FETCH_SIZE x2 (gfx950 half-count of wide reads), KB -> B x1024",
       "source_hash": source_hash(),
       "kernels": kernels, "verify_phase": verify, "hbm_bytes_per_launch_at_bench_size": per_launch}
json.dump(doc, open(out, "w"), indent=1)
print(json.dumps({k: round(v["hbm_bytes_per_share"]) for k, v in verify.items()}), f"per_launch={per_launch:.3e}")
