#!/bin/bash
# A/B of the batched TPKE step's stream layout / cooperative threshold / library build, no profiler (rocprofv3
# serializes the streams).  Usage: bash tools/ab_modes.sh TAG "args A" "args B" ...
# An argument "LCB_LIB_PATH=path@args" runs that case against another build of the library (e.g. lachain_amd/ab/...).
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
k=0
for a in "$@"; do
  k=$((k+1))
  lib=""
  if [[ "$a" == *@* ]]; then lib=${a%%@*}; lib=${lib#LCB_LIB_PATH=}; a=${a#*@}; fi
  LCB_LIB_PATH=$lib timeout -k 10 300 python3 -u bench.py --tpke-exact 0 --pattern-steps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --mcl-reps 0 --no-cpu-baseline --steps 5 $a > gpurun_out/${TAG}_$k.json 2> gpurun_out/${TAG}_$k.err || { echo "BENCH $k FAILED ($lib $a)"; tail -20 gpurun_out/${TAG}_$k.err; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/${TAG}_$k.json') if l.startswith('{')][-1]); t=d['tpke_batched']; print('$k', '$lib', '$a', round(d['value']/1e6,3), round(d['ms_per_step'],2), t['levels'], {k: round(v,1) for k,v in t['device_ms'].items()})"
done
