#!/bin/bash
# A/B of the exact TPKE verify pair: the in-tree library vs lachain_amd/ab/<VARIANT>/.  Usage: bash tools/gpu_exact_ab.sh VARIANT
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
B="--tpke-batched 0 --headline exact --pattern-steps 0 --mcl-reps 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --ts-rounds 0 --no-cpu-baseline --steps 5 --warmup 2"
for v in base $1; do
  if [ "$v" = "base" ]; then unset LCB_LIB_PATH; else export LCB_LIB_PATH=$GRAFT_REPO_ROOT/lachain_amd/ab/$v/liblachain_bls.so; fi
  timeout -k 10 300 python3 -u bench.py $B > gpurun_out/exact_$v.txt 2> gpurun_out/exact_$v.err || { echo "BENCH FAILED $v"; tail -5 gpurun_out/exact_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/exact_$v.txt').read().strip().splitlines()[-1]); e=d['tpke_exact']; print('$v', e['value'], e['ms_per_step'], e['decision_mismatches'], e['roofline'])"
done
