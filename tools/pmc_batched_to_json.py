#!/usr/bin/env python3
"""Fold rocprofv3 --pmc passes of ONE batched TPKE step (bench.py --tpke-exact 0 --steps 1 --warmup 0, TPKE only) into
profiles/pmc_tpke_batched.json: per-dispatch counters of the step's kernels (the splitting levels launch the group
Miller loop / final exponentiation once per level) and the HBM bytes of the whole step (bench.py's roofline.traffic
for the batched headline).  Corrections per /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE
are KB; gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads (x2).
Usage: pmc_batched_to_json.py OUT.json counter_collection.csv...
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import source_hash  # noqa: E402

STEP_KERNELS = ("k_g1_decompress", "k_rlc_key_tables", "k_tpke_rlc_points", "k_rlc_groups", "k_tpke_ct_prepare",
                "k_tpke_ct_prepare_h", "k_tpke_ct_prepare_w", "k_tpke_ct_prepare_hw", "k_ct_ok_merge", "k_lineset_fill", "k_lineset_coop", "k_rlc_census_desc", "k_rlc_census_stats", "k_rlc_suspect_split",
                "k_tpke_rlc_sum", "k_tpke_rlc_wsum", "k_tpke_rlc_wsum2", "k_tpke_rlc_miller", "k_final_exp_check",
                "k_coop_tpke_miller", "k_rlc_miller_fallback", "k_coop_final_exp_check", "k_rlc_resolve",
                "k_rlc_search", "k_rlc_park_copy", "k_tpke_rlc_search2a", "k_tpke_rlc_search2b")
out, paths = sys.argv[1], sys.argv[2:]
disp = collections.defaultdict(lambda: collections.defaultdict(float))
meta = {}
seen = collections.defaultdict(set)
for path in paths:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0]
        if name not in STEP_KERNELS:
            continue
        k = (name, int(r["Grid_Size"]), int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0))
        disp[(name, int(r["Grid_Size"]))][r["Counter_Name"]] += float(r["Counter_Value"])
        seen[(name, int(r["Grid_Size"]))].add((path, k[2]))
        meta[(name, int(r["Grid_Size"]))] = {x: r.get(x) for x in ("VGPR_Count", "Accum_VGPR_Count", "Scratch_Size",
                                                                   "LDS_Block_Size")}
ndisp = {k: len({d for (pth, d) in v if pth == paths[0]}) for k, v in seen.items()}
# the PMC command may run several whole batches (one at a time, then the pipelined ones: bench.py --tpke-pipeline):
# per-step figures divide by the number of batches, counted as the dispatches of the randomisation at the batch size
steps = max(1, max((n for (name, g), n in ndisp.items() if name == "k_tpke_rlc_points"), default=1))
kernels = {}
step_bytes = 0.0
pair_bytes = 0.0
for (name, grid), c in sorted(disp.items()):
    fetch = 2 * 1024 * c.get("FETCH_SIZE", 0.0)
    write = 1024 * c.get("WRITE_SIZE", 0.0)
    w = c.get("SQ_WAVES", 0.0) or 1.0
    kernels[f"{name}@{grid}"] = dict(meta[(name, grid)], grid_lanes=grid, **c, fetch_bytes_corrected=fetch,
                                     write_bytes=write, hbm_bytes_per_lane=(fetch + write) / max(grid, 1),
                                     valu_insts_per_wave=c.get("SQ_INSTS_VALU", 0.0) / w)
    step_bytes += (fetch + write) / steps
    if name in ("k_tpke_rlc_miller", "k_final_exp_check"):
        pair_bytes += (fetch + write) / steps
doc = {"source": "rocprofv3 --pmc, separate passes per counter group (tools/pmc_round.sh with PMC_CMD = one batched "
                 "TPKE step of the bench batch), counters summed per (kernel, grid) over the step's dispatches",
       "correction": "FETCH_SIZE x2 (gfx950 half-count of wide reads), KB -> B x1024",
       "source_hash": source_hash(), "kernels": kernels,
       "batches_profiled": steps, "note": "kernels[]: counters summed over every profiled batch; hbm_bytes_*: per batch",
       "hbm_bytes_per_step": step_bytes, "hbm_bytes_group_checks_per_step": pair_bytes}
json.dump(doc, open(out, "w"), indent=1)
print(f"batches={steps} step_bytes={step_bytes:.3e} group_check_pair_bytes={pair_bytes:.3e}")
