"""The benchmark's output contract (the driver parses bench.py's one JSON line every round): a short
cfg3 run in a subprocess, checked for every field the contract names and for internal consistency
(value = verified rows x steps / wall, roofline.frac = achieved / peak, workload from the
arguments)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_contract():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "cfg3", "--steps", "2",
           "--warmup", "1", "--no-cpu-baseline"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, out.stdout[-2000:]  # exactly one JSON line on stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] in ("weak", "strong")
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # value = whole-job verified matches per second of the timed steps
    v = d["verified_matches_per_step"] * 1e3 / d["ms_per_step"]
    assert abs(v - d["value"]) <= 1e-6 * d["value"]
    cfg = d["config"]
    assert "cfg3" in cfg["workload"] and "1225 unordered pairs" in cfg["workload"]
    assert cfg["n_img"] == 50 and cfg["k"] == 2048 and cfg["pairs_total"] == 1225
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] in ("hbm", "mfma")
    assert abs(r["frac"] - r["achieved"] / r["peak"]) <= 1e-9
    assert 0.0 < r["frac"] < 1.0
    # the cfg3 verified graph is fixed by the oracle-checked kernels (tests/test_gpu_fullsize.py)
    assert d["verified_matches_per_step"] == 554010
    assert isinstance(d["graph_checksum"], int) and 0 <= d["graph_checksum"] < 2147483647
