"""The headline line bench.py prints last must stay small enough for the driver's stdout tail (≈ 8 KB including
stderr; round 3's 20 KB line was not parsed) and carry the contract keys.  Built here from the round-3 full record
(profiles/r03/final3/bench_full.json), which holds every sub-bench section."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def _full():
    with open(os.path.join(ROOT, "profiles", "r03", "final3", "bench_full.json")) as fh:
        return json.load(fh)


def test_compact_line_size_and_keys():
    full = _full()
    line = bench.compact_line(full)
    text = json.dumps(line, separators=(",", ":"))
    assert len(text) <= bench.LINE_MAX_BYTES
    for k in REQUIRED:
        assert k in line, k
    assert line["value"] == full["value"]
    assert "workload" in line["config"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in line["roofline"], k
    assert abs(line["roofline"]["frac"] - full["roofline"]["frac"]) < 1e-5
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in line["cpu_baseline"], k
    ex = line["tpke_exact"]
    assert ex["value"] > 0 and ex["decision_mismatches"] == 0 and ex["roofline"]["frac"] > 0
    s = line["summary"]
    for k in ("tpke_byzantine", "msm", "threshold_signature", "epoch_replay", "ecdsa_headers", "dkg",
              "rbc_erasure_coding", "mcl_latency_us"):
        assert k in s, k


def test_emit_prints_headline_last(capsys):
    full = _full()
    bench.emit(full, write_file=False)
    out = capsys.readouterr().out.splitlines()
    assert out[0].startswith("BENCH_DETAIL ")
    assert json.loads(out[0][len("BENCH_DETAIL "):]) == full
    head = json.loads(out[-1])
    assert head["metric"] == full["metric"] and len(out[-1]) <= bench.LINE_MAX_BYTES


def test_oversized_summary_is_dropped():
    full = _full()
    full["mcl_latency"]["gpu"] = {f"op_{i}": float(i) for i in range(600)}
    line = bench.compact_line(full)
    assert len(json.dumps(line, separators=(",", ":"))) <= bench.LINE_MAX_BYTES
    assert line["roofline"]["frac"] > 0 and line["cpu_baseline"]["value"] > 0


def test_round4_driver_run_line_is_its_detail_compacted():
    """the final round-4 driver-command run (profiles/r04/final/bench_full.txt): its last stdout line is exactly
    compact_line() of the BENCH_DETAIL record printed above it, within the size limit, with the step's HBM traffic
    attached (the PMC files were taken on the same build)"""
    with open(os.path.join(ROOT, "profiles", "r04", "final", "bench_full.txt")) as fh:
        lines = fh.read().strip().splitlines()
    detail = json.loads([x for x in lines if x.startswith("BENCH_DETAIL ")][-1][len("BENCH_DETAIL "):])
    assert len(lines[-1]) <= bench.LINE_MAX_BYTES
    assert json.loads(lines[-1]) == json.loads(json.dumps(bench.compact_line(detail)))
    head = json.loads(lines[-1])
    assert head["roofline"]["traffic"] and head["n_gpus"] == 1 and head["config"]["decision_mismatches"] == 0
    assert head["source_hash"] == detail["source_hash"]
