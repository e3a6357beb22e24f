set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/coop
timeout -k 10 300 python -u -m pytest tests/test_gpu_coop.py tests/test_gpu_parity.py tests/test_gpu_batched.py tests/test_gpu_mcl_surface.py tests/test_gpu_lines.py tests/test_gpu_batched_ts.py -x -q --timeout 150 --timeout-method thread > gpurun_out/coop/gpu_tests.txt 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/coop/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/coop/gpu_tests.txt
bash tools/ab_tpke.sh coop "base:" "l4:" "base:" "l4:" "base:--mcl-reps 300 --shares 4096 --tpke-pipeline 1" "l4:--mcl-reps 300 --shares 4096 --tpke-pipeline 1" "base:--mcl-reps 300 --shares 4096 --tpke-pipeline 1" "l4:--mcl-reps 300 --shares 4096 --tpke-pipeline 1"
