#!/bin/bash
# GPU suite, then this build vs lachain_amd/abfe (the previous commit): batched TPKE (three in flight), CommonCoin,
# exact TPKE.  Usage: bash tools/gpu_pow.sh TAG
set -o pipefail
TAG=${1:-pow}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.txt 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/$TAG/tests.txt; exit 1; }
  tail -2 gpurun_out/$TAG/tests.txt
fi
Z="--pattern-steps 0 --mcl-reps 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline"
run() {
  name=$1; shift
  "$@" > gpurun_out/$TAG/$name.txt 2> gpurun_out/$TAG/$name.err || { echo "$name FAILED"; tail -20 gpurun_out/$TAG/$name.err; exit 1; }
  python3 - $TAG $name <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/{sys.argv[1]}/{sys.argv[2]}.txt").read().strip().splitlines()[-1])
ts = (d.get("summary") or {}).get("threshold_signature") or {}
print(sys.argv[2], "value %.4g" % d["value"], "ms %.2f" % d["ms_per_step"], "mism", d["config"].get("decision_mismatches"),
      "ts", ts.get("value"), ts.get("ms_per_step"), ts.get("phase_ms"))
PY
}
OLD=lachain_amd/abfe/liblachain_bls.so
for rep in 1 2; do
  run new_$rep timeout -k 10 300 python3 -u bench.py $Z --ts-rounds 0 --tpke-exact 0 --steps 21 --warmup 2
  run old_$rep env LCB_LIB_PATH=$OLD timeout -k 10 300 python3 -u bench.py $Z --ts-rounds 0 --tpke-exact 0 --steps 21 --warmup 2
done
run ts_new timeout -k 10 300 python3 -u bench.py $Z --tpke-exact 0 --steps 1 --warmup 1 --ts-exact 0
run ts_old env LCB_LIB_PATH=$OLD timeout -k 10 300 python3 -u bench.py $Z --tpke-exact 0 --steps 1 --warmup 1 --ts-exact 0
run exact_new timeout -k 10 300 python3 -u bench.py $Z --ts-rounds 0 --tpke-batched 0 --headline exact --steps 3 --warmup 1
run exact_old env LCB_LIB_PATH=$OLD timeout -k 10 300 python3 -u bench.py $Z --ts-rounds 0 --tpke-batched 0 --headline exact --steps 3 --warmup 1
