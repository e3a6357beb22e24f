#!/bin/bash
# Round-2c profiling of the current build: rocprofv3 kernel trace + stats of the bench (no CPU legs), then PMC passes
# of the exact TPKE verify (262,144 shares) and of one batched TPKE step (1M shares).  Usage: bash tools/prof_round2.sh TAG
set -o pipefail
TAG=${1:-r02c}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG} -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/${TAG}_bench_rocprof.txt 2>&1 || { echo "ROCPROF FAILED"; tail -5 $R/gpurun_out/${TAG}_bench_rocprof.txt; exit 1; }
echo rocprof done
cd $R
PMC_CMD="python3 $R/bench.py --shares 262144 --steps 1 --warmup 0 --no-cpu-baseline --tpke-batched 0 --ts-batched 0 --ts-rounds 4096 --msm-steps 1 --msm-sizes 1048576 --replay-n 0 --ecdsa-sigs 262144 --ecdsa-steps 1 --dkg-n 0 --rs-n 0" bash tools/pmc_round.sh ${TAG}_exact || exit 1
PMC_CMD="python3 $R/bench.py --tpke-exact 0 --steps 1 --warmup 0 --no-cpu-baseline --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0" bash tools/pmc_round.sh ${TAG}_batched || exit 1
echo all done
