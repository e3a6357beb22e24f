#!/bin/bash
# Cooperative point kernels (DPP exchange): their tests, the mcl single-call latencies and the MSM lines.
set -o pipefail
TAG=${1:-dpp}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ptmul.py tests/test_gpu_msm.py tests/test_gpu_mcl_surface.py tests/test_gpu_failures.py tests/test_gpu_sign_convention.py -x -q --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_tests.txt
timeout -k 10 300 python3 -u bench.py --tpke-exact 1 --tpke-batched 0 --headline exact --ts-rounds 0 --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --mcl-reps 30 --no-cpu-baseline --pattern-steps 0 --shares 22000 --steps 1 --warmup 1 --msm-steps 5 > gpurun_out/${TAG}_bench.txt 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/${TAG}_bench.txt') if l.startswith('BENCH_DETAIL')][-1][13:])
print(json.dumps({k: round(v, 1) for k, v in d['mcl_latency']['gpu'].items()}))
for m in d['msm']: print('msm', m['total_points'], round(m['value'] / 1e6, 1), 'M/s', m['ms_per_step'], m['phase_ms'], m['known_answer_ok'])"
