#!/bin/bash
# A/B timing of the verify pair: bench with a small workload; writes gpurun_out/$1_*.txt
set -o pipefail
TAG=$1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ts_batch.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo TESTS FAILED; tail -20 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_tests.txt
timeout -k 10 300 python -u bench.py --shares 262144 --steps 2 --warmup 1 --no-cpu-baseline --ts-rounds 8192 --msm-points 0 --replay-n 0 > gpurun_out/${TAG}_bench.txt 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/${TAG}_bench.txt; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_bench.txt').read().strip().splitlines()[-1])
r=d['roofline']; print('value', round(d['value']), 'kernel_ms', r['kernel_ms'], 'frac', round(r['frac'],4), 'mism', d['config']['decision_mismatches'])
t=d['threshold_signature']; print('ts', round(t['value']), t['phase_ms'], 'mism', t['decision_mismatches'], t['combined_ok'])"
