#!/bin/bash
# Round 5: the assembly Fp12 products in the final exponentiation.  GPU suite, then exact and batched (three in
# flight) benches of this build and of the previous one (LCB_LIB_PATH=lachain_amd/abfe/...).  Usage: bash tools/gpu_fe.sh TAG
set -o pipefail
TAG=${1:-fe}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.txt 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/$TAG/tests.txt; exit 1; }
  tail -2 gpurun_out/$TAG/tests.txt
fi
X="--pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline"
run() {
  name=$1; shift
  "$@" > gpurun_out/$TAG/$name.txt 2> gpurun_out/$TAG/$name.err || { echo "$name FAILED"; tail -20 gpurun_out/$TAG/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/$name.txt').read().strip().splitlines()[-1]); r=d['roofline']; print('$name', 'value %.4g' % d['value'], 'ms %.2f' % d['ms_per_step'], 'mism', d['config'].get('decision_mismatches'), 'frac %.3f' % r['frac'], 'kms', r.get('kernel_ms'))"
}
OLD=lachain_amd/abfe/liblachain_bls.so
run exact_new timeout -k 10 300 python3 -u bench.py $X --tpke-batched 0 --headline exact --steps 3 --warmup 1
run exact_old env LCB_LIB_PATH=$OLD timeout -k 10 300 python3 -u bench.py $X --tpke-batched 0 --headline exact --steps 3 --warmup 1
run batched_new timeout -k 10 300 python3 -u bench.py $X --tpke-exact 0 --steps 21 --warmup 2
run batched_old env LCB_LIB_PATH=$OLD timeout -k 10 300 python3 -u bench.py $X --tpke-exact 0 --steps 21 --warmup 2
run batched_new2 timeout -k 10 300 python3 -u bench.py $X --tpke-exact 0 --steps 21 --warmup 2
