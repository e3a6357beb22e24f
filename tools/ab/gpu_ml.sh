#!/bin/bash
# Round 5: the assembly Miller loop.  GPU suite, then exact TPKE (this build vs lachain_amd/abfe), batched three in
# flight with the level-1 Miller loop on the cooperative kernel (default) and on the one-lane assembly kernel
# (coop-miller-max 32768), and the CommonCoin line.  Usage: bash tools/gpu_ml.sh TAG
set -o pipefail
TAG=${1:-ml}
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
print(sys.argv[2], "value %.4g" % d["value"], "ms %.2f" % d["ms_per_step"], "mism", d["config"].get("decision_mismatches"),
      "frac %.3f" % d["roofline"]["frac"], "traffic", d["roofline"].get("traffic"))
PY
}
OLD=lachain_amd/abfe/liblachain_bls.so
run exact_new timeout -k 10 300 python3 -u bench.py $Z --ts-rounds 0 --tpke-batched 0 --headline exact --steps 3 --warmup 1
run exact_old env LCB_LIB_PATH=$OLD timeout -k 10 300 python3 -u bench.py $Z --ts-rounds 0 --tpke-batched 0 --headline exact --steps 3 --warmup 1
for rep in 1 2; do
  run bat_$rep timeout -k 10 300 python3 -u bench.py $Z --ts-rounds 0 --tpke-exact 0 --steps 21 --warmup 2
  run bat_ml32k_$rep timeout -k 10 300 python3 -u bench.py $Z --ts-rounds 0 --tpke-exact 0 --steps 21 --warmup 2 --coop-miller-max 32768
done
run bat_old env LCB_LIB_PATH=$OLD timeout -k 10 300 python3 -u bench.py $Z --ts-rounds 0 --tpke-exact 0 --steps 21 --warmup 2
