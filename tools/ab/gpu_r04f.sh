#!/bin/bash
# Round-4 GPU call: the GPU suite, smoke, the mcl single-call latencies, the aggregation queue (prepare-ahead) and the
# batched-only TPKE bench.  Usage: bash tools/gpu_r04f.sh TAG
set -o pipefail
TAG=${1:-r04f}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -X faulthandler -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_tests.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
timeout -k 10 300 python3 -u bench.py --tpke-exact 0 --tpke-batched 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --mcl-reps 30 --no-cpu-baseline --pattern-steps 0 --shares 22000 --headline exact --tpke-exact 1 --steps 1 --warmup 1 > gpurun_out/${TAG}_mcl.txt 2> gpurun_out/${TAG}_mcl.err || { echo "MCL BENCH FAILED"; tail -20 gpurun_out/${TAG}_mcl.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/${TAG}_mcl.txt') if l.startswith('BENCH_DETAIL')][-1][13:]); print(json.dumps({k: round(v, 1) for k, v in d['mcl_latency']['gpu'].items()}))"
timeout -k 10 300 python3 -u tools/queue_bench.py --seconds 3 > gpurun_out/${TAG}_queue.jsonl 2> gpurun_out/${TAG}_queue.err || { echo "QUEUE BENCH FAILED"; tail -20 gpurun_out/${TAG}_queue.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/${TAG}_queue.jsonl'):
    d = json.loads(l); print(d['deadline_ms'], d['callers'], round(d['shares_per_s']), round(d['mean_batch'], 1), {k: round(v, 1) for k, v in d['latency_ms'].items()}, d['decision_mismatches'])"
B="--tpke-exact 0 --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline"
timeout -k 10 300 python3 -u bench.py $B --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.txt 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.txt').read().strip().splitlines()[-1]); print('value', d['value'], 'ms', d['ms_per_step'], 'single', d.get('tpke_single_batch'), 'frac', d['roofline']['frac'])"
echo done
