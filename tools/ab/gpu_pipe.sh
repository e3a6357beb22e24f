#!/bin/bash
# GPU suite, then the TPKE batched bench at the driver's step count with 2 and 3 batches in flight
set -o pipefail
TAG=${1:-pipe}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.txt 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/$TAG/tests.txt; exit 1; }
  tail -2 gpurun_out/$TAG/tests.txt
fi
B="--tpke-exact 0 --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline"
for P in 2 3; do
  timeout -k 10 300 python3 -u bench.py $B --steps 21 --warmup 2 --tpke-pipeline $P > gpurun_out/$TAG/bench_p$P.txt 2> gpurun_out/$TAG/bench_p$P.err || { echo "BENCH FAILED"; tail -20 gpurun_out/$TAG/bench_p$P.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/bench_p$P.txt').read().strip().splitlines()[-1]); print('P=$P value', d['value'], 'ms', d['ms_per_step'], 'mism', d['config']['decision_mismatches'], 'frac', d['roofline']['frac'])"
done
