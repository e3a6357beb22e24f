#!/bin/bash
# CommonCoin-only bench (configs[2]) for an A/B of the TS kernels, plus the TS GPU tests.  Usage: bash tools/gpu_ts_ab.sh TAG
set -o pipefail
TAG=${1:-ts}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ts_batch.py tests/test_gpu_batched_ts.py tests/test_gpu_configs.py -x -q --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_tests.txt
timeout -k 10 300 python3 -u bench.py --tpke-batched 0 --headline exact --shares 22000 --steps 1 --warmup 1 --pattern-steps 0 --mcl-reps 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --ts-steps 2 > gpurun_out/${TAG}_bench.txt 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/${TAG}_bench.txt') if l.startswith('BENCH_DETAIL')][-1][13:]); t=d['threshold_signature']
print('ts', round(t['value']/1e6, 3), 'M/s', round(t['ms_per_step'], 1), 'ms', t.get('phase_ms'), 'mism', t.get('decision_mismatches'), t.get('levels'))"
