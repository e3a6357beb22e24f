#!/bin/bash
# SQ stall counters of the exact TPKE pair (262,144 shares) for this build and lachain_amd/abfe (one PMC pass each)
set -o pipefail
TAG=${1:-pmcml}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
CMD="$R/bench.py --shares 262144 --steps 1 --warmup 0 --no-cpu-baseline --tpke-batched 0 --headline exact --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0"
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS"
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/$TAG/new -o run -- python3 $CMD > $R/gpurun_out/$TAG/new.log 2>&1 || { echo "PMC new failed"; tail -5 $R/gpurun_out/$TAG/new.log; exit 1; }
LCB_LIB_PATH=$R/lachain_amd/abfe/liblachain_bls.so timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/$TAG/old -o run -- python3 $CMD > $R/gpurun_out/$TAG/old.log 2>&1 || { echo "PMC old failed"; tail -5 $R/gpurun_out/$TAG/old.log; exit 1; }
cd $R && python3 - $TAG <<'PY'
import csv, collections, sys, glob
tag = sys.argv[1]
for v in ("new", "old"):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in glob.glob(f"gpurun_out/{tag}/{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0]
            if k in ("k_tpke_miller", "k_final_exp_check"):
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, c in tot.items():
        print(v, k, {n: "%.3g" % x for n, x in sorted(c.items())})
PY
