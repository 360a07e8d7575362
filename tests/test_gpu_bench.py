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
    # the box's i8 ceiling measured in the same run, and K1 read against it
    c = d["calib"]
    assert 1000.0 < c["tops"] < r["peak"] and 1.0 < c["clock_ghz"] < 3.0 and c["ms"] > 50.0
    assert abs(r["practical_peak"] - c["tops"]) <= 1e-9
    assert abs(r["frac_of_practical"] - r["achieved"] / c["tops"]) <= 1e-9
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


def _bench(args, launcher=None, timeout=600):
    import socket
    pre = [sys.executable]
    if launcher:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        pre = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
               str(launcher), "--master-addr", "127.0.0.1", "--master-port", str(port)]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "SFM_BENCH_LAUNCHER")}
    env["OMP_NUM_THREADS"] = "4"
    return subprocess.run(pre + [os.path.join(ROOT, "bench.py")] + args, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout, env=env)


def test_bench_self_launch_two_ranks():
    """`bench.py --gpus 2` with NO torch.distributed.run starts
    its two ranks itself through the real count-then-spawn path (GPUs counted from the KFD
    topology; --ranks-per-gpu 2 puts both gloo ranks on GPU 0 of this 1-GPU box), the launcher
    never imports torch nor maps the HIP runtime, and the line has n_gpus 2 with the N = 1
    graph."""
    out = _bench(["--config", "cfg3", "--steps", "1", "--warmup", "1", "--no-cpu-baseline",
                  "--gpus", "2", "--dist-backend", "gloo", "--ranks-per-gpu", "2"])
    assert out.returncode == 0, out.stderr[-3000:]
    checks = [json.loads(l.split("launcher-selfcheck", 1)[1]) for l in out.stderr.splitlines()
              if "launcher-selfcheck" in l]
    assert [c["stage"] for c in checks] == ["spawned", "exit"], out.stderr[-3000:]
    for c in checks:
        assert c["torch_imported"] is False and c["hip_runtime_mapped"] is False, c
    assert checks[0]["count_source"] == "kfd-topology" and checks[0]["visible_gpus"] >= 1
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["distributed"]["launcher"] == "self"
    assert d["distributed"]["world"] == 2 and len(d["distributed"]["per_rank"]) == 2
    assert [r["rank"] for r in d["distributed"]["per_rank"]] == [0, 1]
    assert [r["device"] for r in d["distributed"]["per_rank"]] == [0, 0]
    assert sum(r["pairs"] for r in d["distributed"]["per_rank"]) == 1225
    assert d["verified_matches_per_step"] == 554009
    one = _bench(["--config", "cfg3", "--steps", "1", "--warmup", "1", "--no-cpu-baseline"])
    assert one.returncode == 0, one.stderr[-3000:]
    d1 = json.loads([l for l in one.stdout.splitlines() if l.strip()][-1])
    assert d1["n_gpus"] == 1 and d1["distributed"]["launcher"] == "none"
    assert d["graph_checksum"] == d1["graph_checksum"]


def test_bench_cfg4_line_carries_cfg5_at_two_ranks():
    """at N > 1 the cfg4 line runs its cfg5 leg (BASELINE configs[4]) on every
    rank — pair-sharded matching, point-sharded BA with the PCG branch from pcg_rule — so the
    driver's multi-GPU run times it.  A 2-rank gloo rehearsal through the self-launcher on small
    scenes: the N = 2 line's cfg5 reconstruction equals N = 1's bit for bit (points, registered
    views, median and mean reprojection error), and its BAs ran sharded."""
    base = ["--config", "cfg4", "--n-img", "12", "--k", "512", "--n-hyp", "1024", "--steps", "1",
            "--warmup", "1", "--no-cpu-baseline", "--no-fp64", "--no-cfg3", "--no-local",
            "--cfg5-n-img", "16", "--cfg5-k", "1024"]
    one = _bench(base)
    assert one.returncode == 0, one.stderr[-3000:]
    d1 = json.loads([l for l in one.stdout.splitlines() if l.strip()][-1])
    two = _bench(base + ["--gpus", "2", "--dist-backend", "gloo", "--ranks-per-gpu", "2"])
    assert two.returncode == 0, two.stderr[-3000:]
    d2 = json.loads([l for l in two.stdout.splitlines() if l.strip()][-1])
    c1, c2 = d1["cfg5"], d2["cfg5"]
    assert "error" not in c1 and "error" not in c2, (c1, c2)
    assert c1["n_gpus"] == 1 and c2["n_gpus"] == 2 and c2["shard_ba"] is True
    for key in ("points", "registered", "observations", "verified_matches", "median_reproj_px",
                "mean_reproj_px"):
        assert c1[key] == c2[key], (key, c1[key], c2[key])
    assert c1["registered"] >= 14 and c2["s_per_reconstruction"] > 0
    assert set(c2["pcg_branches"]) <= {"sharded", "replicated"}
    assert d2["graph_checksum"] == d1["graph_checksum"]


def test_bench_refuses_more_gpus_than_the_box_has():
    """`--gpus N` with fewer than N visible GPUs exits non-zero with a clear message and no JSON
    line (the box has one MI355X)."""
    import torch
    n = torch.cuda.device_count() + 1
    out = _bench(["--config", "cfg3", "--gpus", str(n)], timeout=300)
    assert out.returncode == 2, out.stderr[-2000:]
    assert f"needs {n} visible GPUs" in out.stderr and out.stdout.strip() == ""


def test_bench_cfg5_line_and_two_rank_rehearsal():
    """`--config cfg5` (a step = one whole incremental reconstruction) on a
    small scene: the line carries the end-to-end value, quality against the scene's truth, BA
    sizes / iterations and the PCG branch, and the K3 / CG-iteration HBM fractions; a 2-rank gloo
    rehearsal through the self-launcher (matching sharded, BA sharded, each PCG branch) returns
    the single-process reconstruction."""
    base = ["--config", "cfg5", "--n-img", "12", "--k", "1024", "--steps", "1", "--warmup", "1"]
    one = _bench(base)
    assert one.returncode == 0, one.stderr[-3000:]
    d1 = json.loads([l for l in one.stdout.splitlines() if l.strip()][-1])
    c1 = d1["cfg5"]
    assert d1["n_gpus"] == 1 and "BASELINE configs[4]" in d1["config"]["baseline_config"]
    assert c1["registered"] == 12 and c1["median_reproj_px"] < 0.8
    assert c1["max_centre_err_rel_radius"] < 0.02
    assert abs(d1["value"] - c1["verified_matches"] * 1e3 / d1["ms_per_step"]) <= 1e-6 * d1["value"]
    assert c1["pcg_branches"] == ["single"] and c1["lm_steps"] > 0 and c1["cg_iters"] > 0
    rf = c1["ba_rooflines"]
    assert 0 < rf["k3"]["frac"] < 1 and 0 < rf["cg_iteration"]["frac"] < 1
    assert d1["roofline"]["bound"] == "hbm" and abs(d1["roofline"]["frac"] - rf["k3"]["frac"]) < 1e-12
    for pcg in ("sharded", "replicated"):
        two = _bench(base + ["--gpus", "2", "--dist-backend", "gloo", "--device", "0",
                             "--ba-pcg", pcg])
        assert two.returncode == 0, two.stderr[-3000:]
        d2 = json.loads([l for l in two.stdout.splitlines() if l.strip()][-1])
        c2 = d2["cfg5"]
        assert d2["n_gpus"] == 2 and d2["distributed"]["launcher"] == "self"
        assert c2["pcg_branches"] == [pcg] and c2["shard_ba"] is True
        assert c2["verified_matches"] == c1["verified_matches"]
        assert c2["registered"] == c1["registered"]
        # sharding-invariant BA (reconstruction.BA_CHUNKS): the same reconstruction, bit for bit
        assert c2["points"] == c1["points"]
        assert c2["median_reproj_px"] == c1["median_reproj_px"]
        assert c2["mean_reproj_px"] == c1["mean_reproj_px"]


def test_bench_cfg4_local_leg():
    """the N = 1 cfg4 line carries `cfg4_local`, the same step on the cfg5
    local-visibility scene (most pairs fail verification, as in a real capture); small shape."""
    out = _bench(["--config", "cfg4", "--n-img", "24", "--k", "1024", "--steps", "1",
                  "--warmup", "1", "--no-cpu-baseline", "--no-cfg3", "--no-cfg5", "--no-fp64"])
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.strip()][-1])
    loc = d["cfg4_local"]
    assert "error" not in loc, loc
    assert loc["pairs"] == 276 and 0 < loc["verified_pairs"] < loc["pairs"]
    assert loc["verified_matches_per_step"] < d["verified_matches_per_step"]
    assert abs(loc["value"] - loc["verified_matches_per_step"] * 1e3 / loc["ms_per_step"]) \
        <= 1e-6 * loc["value"]
    assert 0 < loc["k2_executed_frac"] <= 1.0 and loc["match_ms"] > 0
