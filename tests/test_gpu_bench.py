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
    # the cfg3 verified graph is fixed by the oracle-checked kernels (tests/test_gpu_fullsize.py);
    # 554 010 before round 3's rank-2 step (8 squarings of adj(F^T F))
    assert d["verified_matches_per_step"] == 554009
    assert isinstance(d["graph_checksum"], int) and 0 <= d["graph_checksum"] < 2147483647


def test_bench_two_ranks_same_graph():
    """bench.py's N > 1 path (shard_range, per-rank K1 + K2, packed graph all-gather) as a 2-rank
    torch.distributed.run job (gloo, both ranks on GPU 0: RCCL cannot share a device) on cfg3:
    the gathered graph equals the single-process one (graph_checksum, verified count)."""
    import socket
    def run(extra, nproc):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        pre = ([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
                str(nproc), "--master-addr", "127.0.0.1", "--master-port", str(port)]
               if nproc > 1 else [sys.executable])
        cmd = pre + [os.path.join(ROOT, "bench.py"), "--config", "cfg3", "--steps", "1",
                     "--warmup", "1", "--no-cpu-baseline"] + extra
        out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600,
                             env=dict(os.environ, OMP_NUM_THREADS="4"))
        assert out.returncode == 0, out.stderr[-3000:]
        return json.loads([l for l in out.stdout.splitlines() if l.strip()][-1])
    one = run([], 1)
    two = run(["--gpus", "2", "--dist-backend", "gloo", "--device", "0"], 2)
    assert two["n_gpus"] == 2 and two["config"]["pairs_total"] == 1225
    assert two["verified_matches_per_step"] == one["verified_matches_per_step"] == 554009
    assert two["graph_checksum"] == one["graph_checksum"]
