#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection.csv files: per kernel, sum each counter over dispatches."""
import csv, sys, collections
tot = collections.defaultdict(lambda: collections.defaultdict(float))
meta = {}
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[k] = {x: r.get(x) for x in ("VGPR_Count", "Accum_VGPR_Count", "Scratch_Size", "LDS_Block_Size")}
for k, c in tot.items():
    if "k_" not in k:
        continue
    print(k, meta[k])
    for n, v in sorted(c.items()):
        print(f"   {n:22s} {v:,.0f}")
    if c.get("SQ_WAVES"):
        w = c["SQ_WAVES"]
        print(f"   valu/wave {c['SQ_INSTS_VALU']/w:,.0f}  vmem_rd/wave {c.get('SQ_INSTS_VMEM_RD',0)/w:,.0f}"
              f"  vmem_wr/wave {c.get('SQ_INSTS_VMEM_WR',0)/w:,.0f}  salu/wave {c.get('SQ_INSTS_SALU',0)/w:,.0f}"
              f"  active_valu/wave_cycles {c['SQ_ACTIVE_INST_VALU']/c['SQ_WAVE_CYCLES']:.3f}")
