#!/bin/bash
# rocprofv3 kernel-trace stats of the bench (no CPU legs), then the PMC passes (tools/pmc_round.sh), each under its
# own time limit.  Usage: bash tools/prof_round.sh TAG
set -o pipefail
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG} -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/${TAG}_bench_rocprof.txt 2>&1 || { echo "ROCPROF FAILED"; tail -5 $R/gpurun_out/${TAG}_bench_rocprof.txt; exit 1; }
echo rocprof done
cd $R && bash tools/pmc_round.sh ${TAG}
