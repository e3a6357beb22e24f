set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/lf
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/lf/gpu_tests.txt 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/lf/gpu_tests.txt; exit 1; }
tail -1 gpurun_out/lf/gpu_tests.txt
bash tools/ab_tpke.sh lf "base:" "lf0:" "base:" "lf0:" "base:--ts-rounds 65536 --ts-exact 0 --shares 4096 --tpke-pipeline 1 --msm-sizes 1048576" "lf0:--ts-rounds 65536 --ts-exact 0 --shares 4096 --tpke-pipeline 1 --msm-sizes 1048576"
