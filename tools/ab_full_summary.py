"""summary of tools/ab_full.sh runs: python3 tools/ab_full_summary.py TAG N"""
import json
import sys

tag, n = sys.argv[1], int(sys.argv[2])
for k in range(1, n + 1):
    d = json.loads([l for l in open(f"gpurun_out/{tag}_{k}.json") if l.startswith("{")][-1])
    t, ex = d["tpke_batched"], d["tpke_exact"]
    pb, ts = d["tpke_byzantine"]["patterns"], d["threshold_signature"]
    print(k, "batched %.2f ms" % t["ms_per_step"], "exact %.1f" % ex["ms_per_step"],
          {p: round(v["batched"]["ms_per_step"], 1) for p, v in pb.items()},
          "worst/exact %.3f" % d["tpke_byzantine"]["worst_batched_over_exact"],
          "TS %.0f" % ts["ms_per_step"], {k2: round(v, 1) for k2, v in ts["phase_ms"].items()},
          {p: round(v["batched"]["ms_per_step"], 1) for p, v in ts["byzantine"].items()},
          "mism", t["decision_mismatches"], {k2: round(v, 1) for k2, v in t["device_ms"].items()})
