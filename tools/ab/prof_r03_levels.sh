set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for CM in 32768 65536; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_cm$CM -o run -- python3 $R/bench.py --tpke-exact 0 --pattern-steps 0 --ts-rounds 0 --msm-sizes= --replay-n 0 --ecdsa-sigs 0 --dkg-n 0 --rs-n 0 --no-cpu-baseline --steps 3 --coop-max $CM > $R/gpurun_out/prof_cm$CM.json 2> $R/gpurun_out/prof_cm$CM.err || exit 1
done
echo done
