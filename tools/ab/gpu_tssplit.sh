#!/bin/bash
# CommonCoin batched check: the split randomisation (default) vs the fused kernel (LCB_TS_SPLIT=0), twice each
set -o pipefail
TAG=${1:-tssplit}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
X="--shares 22528 --steps 1 --warmup 1 --tpke-pipeline 1 --tpke-exact 0 --pattern-steps 0 --mcl-reps 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --ts-exact 0 --ts-steps 2"
if [ -z "$NOTESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_batched_ts.py tests/test_gpu_scratch_gate.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/$TAG/tests.txt; exit 1; }
  tail -1 gpurun_out/$TAG/tests.txt
fi
for rep in 1 2; do
  for sp in 1 0; do
    LCB_TS_SPLIT=$sp timeout -k 10 300 python3 -u bench.py $X > gpurun_out/$TAG/s${sp}_$rep.txt 2>/dev/null || { echo "split=$sp failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/s${sp}_$rep.txt').read().strip().splitlines()[-1]); t=d['summary']['threshold_signature']; print('split=$sp', t['value'], t['ms_per_step'], t['phase_ms'], t['mismatches'])"
  done
done
