#!/bin/bash
# Round-5 evidence, part 1 (one GPU call): the GPU suite, smoke, a rocprofv3 kernel trace + stats of the bench (TPKE,
# CommonCoin, MSM, replay, ECDSA, DKG, RS; no CPU legs) and a single-batch TPKE trace for the step timeline.
# Outputs under gpurun_out/<TAG>/.  Usage: bash tools/final_r05.sh TAG
set -o pipefail
TAG=${1:-r05f}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -X faulthandler -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/$TAG/gpu_tests.txt 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/$TAG/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/$TAG/gpu_tests.txt
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.txt 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/$TAG/smoke.txt; exit 1; }
tail -1 gpurun_out/$TAG/smoke.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/rocprof -o run -- python3 $R/bench.py --no-cpu-baseline --pattern-steps 1 --mcl-reps 10 > $R/gpurun_out/$TAG/bench_under_rocprof.txt 2>&1 || { echo "ROCPROF FAILED"; tail -5 $R/gpurun_out/$TAG/bench_under_rocprof.txt; exit 1; }
echo rocprof done
B="--tpke-exact 0 --pattern-steps 0 --mcl-reps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$TAG/single -o run -- python3 $R/bench.py $B --tpke-pipeline 1 --steps 4 --warmup 1 > $R/gpurun_out/$TAG/single_bench.txt 2>&1 || { echo "SINGLE ROCPROF FAILED"; tail -5 $R/gpurun_out/$TAG/single_bench.txt; exit 1; }
cd $R && python3 tools/step_timeline.py gpurun_out/$TAG/single/run_kernel_trace.csv 2 > gpurun_out/$TAG/batched_step_timeline.txt
gzip -f gpurun_out/$TAG/rocprof/run_kernel_trace.csv gpurun_out/$TAG/single/run_kernel_trace.csv
echo done
