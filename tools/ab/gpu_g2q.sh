#!/bin/bash
# G2 Lagrange lanes with up to four entries per lane (default) vs the paired lanes (LCB_G2_LANES=2): the assembly /
# interpolation GPU tests, then configs[2] twice per setting
set -o pipefail
TAG=${1:-g2q}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd $R
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_ts_batch.py tests/test_gpu_batched_ts.py tests/test_gpu_parity.py tests/test_gpu_scratch_gate.py tests/test_gpu_sign_convention.py > gpurun_out/$TAG/tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/$TAG/tests.txt; exit 1; }
tail -1 gpurun_out/$TAG/tests.txt
XT="--shares 22528 --steps 1 --warmup 1 --tpke-pipeline 1 --pattern-steps 0 --mcl-reps 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --tpke-exact 0 --ts-exact 0 --ts-steps 3"
for rep in 1 2; do
  for v in 4 2; do
    LCB_ALLOW_TUNING=1 LCB_G2_LANES=$v timeout -k 10 300 python3 -u bench.py $XT > gpurun_out/$TAG/ts_${v}_$rep.txt 2> gpurun_out/$TAG/ts_${v}_$rep.err || { echo "TS BENCH FAILED"; tail -5 gpurun_out/$TAG/ts_${v}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$TAG/ts_${v}_$rep.txt').read().strip().splitlines()[-1]); t=d['summary'].get('threshold_signature'); print('lanes$v', t['value'], t['ms_per_step'], t['mismatches'], t['phase_ms'])"
  done
done
