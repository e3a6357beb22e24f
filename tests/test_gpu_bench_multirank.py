"""bench.py's own N > 1 code at world size 2 on the GPU box: two ranks launched by torch.distributed.run exactly as
the driver launches the scaling runs, sharing the box's one GPU, with LCB_BENCH_BACKEND=gloo standing in for RCCL
(two ranks cannot hold one device under RCCL).  Exercises the process-group init, the barriers, the max-over-ranks
timing reduction (lachain_amd/shard.py max_time_sum), the ciphertext / round / era partitions and the MSM
all-gather of the partials, at small sizes; every section must report zero decision mismatches."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_world_size_two():
    # bench.py's default hardware queues (the environment's: HIP's default four per priority) and its default
    # concurrent epoch replay, two ranks on the one GPU.  Each process has its own 32 GiB scratch pool; the library's
    # gate keeps the bound reservations of its queues within it
    env = dict(os.environ, LCB_BENCH_BACKEND="gloo", OMP_NUM_THREADS="4")
    env.pop("GPU_MAX_HW_QUEUES", None)
    env.pop("LCB_BENCH_HWQ", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "1", "--shares", "8800", "--pattern-steps", "1",
           "--patterns", "f_validators_wrong", "--ts-rounds", "64", "--ts-n", "16", "--replay-n", "16",
           "--ecdsa-sigs", "4096", "--ecdsa-validators", "16", "--msm-sizes", "8192", "--msm-steps", "1",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    if r.returncode != 0 and os.path.isdir(os.path.join(ROOT, "gpurun_out")):
        with open(os.path.join(ROOT, "gpurun_out", "bench_multirank_failure.txt"), "w") as fh:
            fh.write(r.stdout + "\n----- stderr -----\n" + r.stderr)
    assert r.returncode == 0, r.stderr[:2000] + "\n...\n" + r.stderr[-2000:]
    lines = r.stdout.splitlines()
    head = json.loads([x for x in lines if x.startswith("{")][-1])
    assert lines[-1].startswith("{") and len(lines[-1]) <= 6144       # the compact headline is the last line
    assert head["summary"]["tpke_byzantine"]["mismatches"] == 0
    line = json.loads([x for x in lines if x.startswith("BENCH_DETAIL ")][-1][len("BENCH_DETAIL "):])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "shard2"
    assert line["config"]["decision_mismatches"] == 0
    assert line["tpke_exact"]["decision_mismatches"] == 0
    assert line["value"] > 0 and line["ms_per_step"] > 0
    for rec in line["tpke_byzantine"]["patterns"].values():
        assert rec["batched"]["decision_mismatches"] == 0 and rec["exact"]["decision_mismatches"] == 0
    ts = line["threshold_signature"]
    assert ts["decision_mismatches"] == 0 and ts["combined_ok"]
    assert line["epoch_replay"]["mismatches"] == 0
    assert line["ecdsa_headers"]["decision_mismatches"] == 0
    assert all(m["known_answer_ok"] for m in line["msm"])
