#!/bin/bash
# SQ counters of the nine-lane pairing kernels on the single-call path (mclBn_pairing / finalExp, one wave per launch)
set -o pipefail
TAG=${1:-pmccoop}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
CMD="$R/bench.py --shares 22528 --steps 1 --warmup 0 --tpke-pipeline 1 --no-cpu-baseline --tpke-exact 0 --pattern-steps 0 --mcl-reps 20 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0"
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/$TAG/p1 -o run -- python3 $CMD > $R/gpurun_out/$TAG/p1.log 2>&1 || { echo "PMC failed"; tail -5 $R/gpurun_out/$TAG/p1.log; exit 1; }
C2="SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES"
timeout -s KILL 200 rocprofv3 --pmc $C2 --output-format csv -d $R/gpurun_out/$TAG/p2 -o run -- python3 $CMD > $R/gpurun_out/$TAG/p2.log 2>&1 || { echo "PMC2 failed"; tail -5 $R/gpurun_out/$TAG/p2.log; exit 1; }
cd $R && python3 - $TAG <<'PY'
import csv, collections, sys, glob
tag = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob(f"gpurun_out/{tag}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0]
        g = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
        if k.startswith("k_coop") and g in ("64", 64):
            tot[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in tot.items():
    print(k, {n: "%.4g" % (sum(x) / len(x)) for n, x in sorted(c.items())})
PY
