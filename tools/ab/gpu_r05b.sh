#!/bin/bash
# Round 5 iteration: GPU suite, then the TPKE batched bench (driver step count, two batches in flight) and a rocprofv3
# kernel trace of single batches (timeline: tools/step_timeline.py).  Usage: bash tools/gpu_r05b.sh TAG [NOTESTS=1]
set -o pipefail
TAG=${1:-r05b}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.txt 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/$TAG/tests.txt; exit 1; }
  tail -2 gpurun_out/$TAG/tests.txt
fi
B="--tpke-exact 0 --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline"
timeout -k 10 300 python3 -u bench.py $B --steps 20 --warmup 2 > gpurun_out/$TAG/bench.txt 2> gpurun_out/$TAG/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/$TAG/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/bench.txt').read().strip().splitlines()[-1]); print('value', d['value'], 'ms', d['ms_per_step'], 'single', d.get('tpke_single_batch'), 'frac', d['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/prof -o run -- python3 $R/bench.py $B --tpke-pipeline 1 --steps 4 --warmup 1 > $R/gpurun_out/$TAG/bench_rocprof.txt 2>&1 || { echo "ROCPROF FAILED"; tail -5 $R/gpurun_out/$TAG/bench_rocprof.txt; exit 1; }
cd $R && python3 tools/step_timeline.py gpurun_out/$TAG/prof/run_kernel_trace.csv 2 > gpurun_out/$TAG/timeline.txt && grep -c . gpurun_out/$TAG/timeline.txt && grep -c fallback gpurun_out/$TAG/timeline.txt; rm -f gpurun_out/$TAG/prof/run_kernel_trace.csv.gz; echo done
