#!/bin/bash
# binary-GCD inversion in the nine-lane final exponentiation: the cooperative / mcl / queue GPU tests, the queue bench
# (1 ms deadline) and the mcl single-call latencies
set -o pipefail
TAG=${1:-fegcd}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd $R
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_coop.py tests/test_gpu_mcl_surface.py tests/test_gpu_queue.py tests/test_gpu_ct_cache.py > gpurun_out/$TAG/tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/$TAG/tests.txt; exit 1; }
tail -2 gpurun_out/$TAG/tests.txt
timeout -k 10 300 python3 -u tools/queue_bench.py --seconds 3 --deadlines 1 > gpurun_out/$TAG/queue_bench.jsonl 2> gpurun_out/$TAG/queue_bench.err || { echo "QUEUE BENCH FAILED"; tail -5 gpurun_out/$TAG/queue_bench.err; exit 1; }
cat gpurun_out/$TAG/queue_bench.jsonl
X="--shares 22528 --steps 1 --warmup 1 --tpke-pipeline 1 --pattern-steps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --tpke-exact 0 --mcl-reps 20"
timeout -k 10 300 python3 -u bench.py $X > gpurun_out/$TAG/mcl.txt 2> gpurun_out/$TAG/mcl.err || { echo "MCL BENCH FAILED"; tail -5 gpurun_out/$TAG/mcl.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/mcl.txt').read().strip().splitlines()[-1]); print(d['summary'].get('mcl_latency_us'))"
