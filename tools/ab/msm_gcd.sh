#!/bin/bash
# GPU suite, then the 2^20 MSM one at a time (10 steps, three runs) after the binary-GCD serialisation change.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/msmgcd
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/msmgcd/gpu_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/msmgcd/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/msmgcd/gpu_tests.txt
X="--shares 22528 --steps 1 --warmup 1 --tpke-pipeline 1 --tpke-exact 0 --pattern-steps 0 --mcl-reps 300 --ts-rounds 0 --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --msm-sizes 1048576 --msm-steps 10"
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py $X > gpurun_out/msmgcd/b$i.txt 2> gpurun_out/msmgcd/b$i.err || { echo "BENCH FAILED"; tail -5 gpurun_out/msmgcd/b$i.err; exit 1; }
  python - gpurun_out/msmgcd/b$i.txt <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
def find(o, k):
    if isinstance(o, dict):
        if k in o: return o[k]
        for v in o.values():
            r = find(v, k)
            if r is not None: return r
    if isinstance(o, list):
        for v in o:
            r = find(v, k)
            if r is not None: return r
m = d["summary"].get("msm")
print("msm", m)
print("mcl", json.dumps(find(d, "mcl"))[:900])
PY
done
