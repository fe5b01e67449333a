"""bench.py's JSON line contract (the driver parses it): BASELINE.json's
metric, the roofline and cpu_baseline objects, and values that recompute from
the line's own fields.  GPU: one short C1 run."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_line_contract(gpu_available):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "c1", "--batch", "256",
                        "--steps", "3", "--warmup", "1", "--cpu-baseline-seconds", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == base["metric"] and d["unit"] == "info-bits/s"
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["vs_baseline"] is None
    assert d["dtype"] == "f64" and "synthetic" in d["data"]
    cfg = d["config"]
    assert cfg["workload"].startswith("C1") and cfg["batch_per_gpu"] == 256 and cfg["global_batch"] == 256
    # value = frames * info bits / wall; ms_per_step is the same wall over the steps
    frames = cfg["global_batch"] * d["steps"]
    assert d["value"] == pytest.approx(frames * cfg["info_bits_per_frame"] / (d["ms_per_step"] * d["steps"] / 1e3),
                                       rel=1e-9)
    rf = d["roofline"]
    assert rf["bound"] in ("hbm", "mfma") or rf["bound"].startswith("fp64")
    assert rf["unit"] and rf["peak"] > 0 and rf["achieved"] > 0
    assert rf["frac"] == pytest.approx(rf["achieved"] / rf["peak"], rel=1e-12)
    assert "traffic" in rf
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["unit"] == "info-bits/s" and cb["cores"] >= 1 and cb["kind"] in ("port", "reference")
    assert cb["sample"]
    assert 0.0 <= d["fer"] <= 1.0 and d["mean_iterations"] >= 1.0
