set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r01b_gpu_tests.txt 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r01b_bench.txt 2>&1 && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r01b -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r01b_bench_rocprof.txt 2>&1)
