#!/bin/bash
# A/B of the batched TPKE step in one GPU call: the batch-check tests, the batched-only bench (one batch and two in
# flight), and a rocprofv3 kernel trace of a few steps.  Usage: bash tools/gpu_ab_tpke.sh TAG [pytest files...]
set -o pipefail
TAG=${1:-ab}
shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TESTS=${@:-"tests/test_gpu_batched.py tests/test_gpu_ts_batch.py"}
timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_tests.txt
B="--tpke-exact 0 --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline"
timeout -k 10 300 python3 -u bench.py $B --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.txt 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 - gpurun_out/${TAG}_bench.txt <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "single", d.get("tpke_single_batch"), "frac", d["roofline"]["frac"])
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_${TAG} -o run -- python3 $R/bench.py $B --steps 4 --warmup 1 > $R/gpurun_out/${TAG}_prof.txt 2>&1 || { echo "ROCPROF FAILED"; tail -5 $R/gpurun_out/${TAG}_prof.txt; exit 1; }
echo done
