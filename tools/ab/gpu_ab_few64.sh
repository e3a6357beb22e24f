#!/bin/bash
# A/B: the batched check's level-1 one-lane final exponentiation in 256-lane workgroups (LCB_FE_W64_MAX=0) or one-wave
# workgroups (default), one batch at a time and three in flight; then the kernel-resource and batched GPU tests
set -o pipefail
TAG=${1:-abfew64}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
B="--tpke-exact 0 --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --steps 21 --warmup 2"
run() {
  name=$1; shift
  env LCB_ALLOW_TUNING=1 "$@" > gpurun_out/$TAG/$name.txt 2> gpurun_out/$TAG/$name.err || { echo "$name FAILED"; tail -20 gpurun_out/$TAG/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/$name.txt').read().strip().splitlines()[-1]); print('$name', 'value %.4g' % d['value'], 'ms %.2f' % d['ms_per_step'], 'mism', d['config']['decision_mismatches'])"
}
for rep in 1 2; do
run base_p1_$rep env LCB_FE_W64_MAX=0 timeout -k 10 300 python3 -u bench.py $B --tpke-pipeline 1
run w64_p1_$rep timeout -k 10 300 python3 -u bench.py $B --tpke-pipeline 1
run base_p3_$rep env LCB_FE_W64_MAX=0 timeout -k 10 300 python3 -u bench.py $B --tpke-pipeline 3
run w64_p3_$rep timeout -k 10 300 python3 -u bench.py $B --tpke-pipeline 3
done
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batched.py tests/test_kernel_resources.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/$TAG/tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/$TAG/tests.txt; exit 1; }
tail -1 gpurun_out/$TAG/tests.txt
echo done
