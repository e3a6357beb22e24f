#!/bin/bash
# CommonCoin configs[2] with the paired G2 Lagrange lanes at 256 registers (two waves per SIMD; variant library in
# lachain_amd/abv) against this build, twice each
set -o pipefail
TAG=${1:-abg2w2}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd $R
XT="--shares 22528 --steps 1 --warmup 1 --tpke-pipeline 1 --pattern-steps 0 --mcl-reps 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --tpke-exact 0 --ts-exact 0 --ts-steps 3"
for rep in 1 2; do
  for v in base var; do
    if [ $v = var ]; then export LCB_LIB_PATH=$R/lachain_amd/abv/liblachain_bls.so; else unset LCB_LIB_PATH; fi
    timeout -k 10 300 python3 -u bench.py $XT > gpurun_out/$TAG/ts_${v}_$rep.txt 2> gpurun_out/$TAG/ts_${v}_$rep.err || { echo "TS BENCH FAILED"; tail -5 gpurun_out/$TAG/ts_${v}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$TAG/ts_${v}_$rep.txt').read().strip().splitlines()[-1]); t=d['summary'].get('threshold_signature'); print('$v', t['value'], t['ms_per_step'], t['mismatches'], t['phase_ms'])"
  done
done
