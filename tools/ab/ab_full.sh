#!/bin/bash
# Broad A/B (batched TPKE step, exact path, Byzantine patterns, CommonCoin) without the CPU baselines and the
# secondary sections.  Usage: bash tools/ab_full.sh TAG "args A" "args B" ...  ("LCB_LIB_PATH=path@args" as in
# tools/ab_modes.sh); summary: python3 tools/ab_full_summary.py TAG N
set -o pipefail
TAG=$1; shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
k=0
for a in "$@"; do
  k=$((k+1))
  lib=""
  if [[ "$a" == *@* ]]; then lib=${a%%@*}; lib=${lib#LCB_LIB_PATH=}; a=${a#*@}; fi
  LCB_LIB_PATH=$lib timeout -k 10 400 python3 -u bench.py --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --mcl-reps 0 --no-cpu-baseline --steps 3 $a > gpurun_out/${TAG}_$k.json 2> gpurun_out/${TAG}_$k.err || { echo "BENCH $k FAILED ($lib $a)"; tail -5 gpurun_out/${TAG}_$k.err; exit 1; }
  echo "done $k $lib $a"
done
