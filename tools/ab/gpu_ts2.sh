#!/bin/bash
# CommonCoin preparation at 256 registers ahead of the randomisation (+ GCD affine conversion in the hash lanes):
# the TS / TPKE batch GPU tests, the configs[2] step (twice) with a kernel trace, and the TPKE headline (3 in flight)
set -o pipefail
TAG=${1:-ts2}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd $R
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_batched_ts.py tests/test_gpu_ts_batch.py tests/test_gpu_batched.py > gpurun_out/$TAG/tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/$TAG/tests.txt; exit 1; }
tail -2 gpurun_out/$TAG/tests.txt
XT="--shares 22528 --steps 1 --warmup 1 --tpke-pipeline 1 --pattern-steps 0 --mcl-reps 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --tpke-exact 0 --ts-exact 0 --ts-steps 2"
timeout -k 10 300 python3 -u bench.py $XT > gpurun_out/$TAG/ts.txt 2> gpurun_out/$TAG/ts.err || { echo "TS BENCH FAILED"; tail -5 gpurun_out/$TAG/ts.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/$TAG/ts.txt').read().strip().splitlines()[-1]); print('ts', d['summary'].get('threshold_signature'))"
grep -o '\"phase_ms\": {[^}]*}' gpurun_out/$TAG/ts.txt | head -1
X="--pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --tpke-exact 0 --steps 21 --warmup 2"
timeout -k 10 300 python3 -u bench.py $X > gpurun_out/$TAG/tpke.txt 2> gpurun_out/$TAG/tpke.err || { echo "TPKE BENCH FAILED"; tail -5 gpurun_out/$TAG/tpke.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/tpke.txt').read().strip().splitlines()[-1]); print('tpke', '%.4g' % d['value'], '%.2f' % d['ms_per_step'], d['config']['decision_mismatches'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$TAG/rocprof -o run -- python3 $R/bench.py $XT --ts-steps 1 > $R/gpurun_out/$TAG/ts_prof.txt 2>&1 || { echo "PROF FAILED"; tail -5 $R/gpurun_out/$TAG/ts_prof.txt; exit 1; }
gzip -f $R/gpurun_out/$TAG/rocprof/run_kernel_trace.csv
echo ok
