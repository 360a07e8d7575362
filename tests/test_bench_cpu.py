"""CPU: bench.py's launch contract and the BA shard/replicate rule (item 3).

`python bench.py --gpus N` must start N ranks itself when no launcher did, refuse (rc != 0, a
clear message, before any GPU call) when fewer than N GPUs are visible or when --gpus disagrees
with an external launcher's WORLD_SIZE, and fail as a whole when one of its ranks fails.  This
container has no GPU, so the refusals and the failure propagation are exercised here; the
successful N-rank run is tests/test_gpu_bench.py::test_bench_self_launch_two_ranks.
"""
import os
import subprocess
import sys

import pytest

import reconstruction as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "SFM_BENCH_LAUNCHER")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, cwd=ROOT, capture_output=True,
                          text=True, timeout=timeout, env=env)


@pytest.mark.skipif(__import__("torch").cuda.device_count() >= 2, reason="needs < 2 GPUs")
def test_bench_refuses_more_gpus_than_visible():
    r = _run(["--gpus", "2", "--config", "cfg3"])
    assert r.returncode == 2, r.stderr[-2000:]
    assert "needs 2 visible GPUs" in r.stderr
    assert r.stdout.strip() == ""


def test_bench_refuses_world_size_mismatch():
    r = _run(["--gpus", "3", "--config", "cfg3"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr, r.stderr[-2000:]


def test_bench_refuses_rccl_ranks_sharing_one_gpu():
    r = _run(["--gpus", "2", "--device", "0", "--dist-backend", "nccl", "--config", "cfg3"])
    assert r.returncode == 2 and "RCCL cannot" in r.stderr, r.stderr[-2000:]


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="CPU-only check")
def test_bench_self_launch_propagates_a_failing_rank(tmp_path):
    """Same-GPU gloo rehearsal form with no GPU present but a (fake) 1-GPU KFD topology: the
    launcher counts one GPU, starts both child ranks (it never touches the GPU itself), they fail
    at their first GPU call, and the parent exits non-zero without printing a JSON line."""
    r = _run(["--gpus", "2", "--ranks-per-gpu", "2", "--dist-backend", "gloo", "--config", "cfg3",
              "--steps", "1", "--warmup", "0", "--no-cpu-baseline"],
             {"SFM_BENCH_KFD_NODES": _fake_kfd(tmp_path, [0, 8])})
    assert r.returncode != 0
    assert '"torch_imported": false, "hip_runtime_mapped": false' in r.stderr, r.stderr[-2000:]
    assert "exited with" in r.stderr, r.stderr[-2000:]
    assert r.stdout.strip() == ""


def _fake_kfd(tmp_path, simd_counts):
    for i, s in enumerate(simd_counts):
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {s}\ngfx_target_version "
                                      f"{95000 if s else 0}\n")
    return str(tmp_path)


def test_visible_gpus_from_kfd_topology(tmp_path):
    """GPUs are counted from the KFD topology (CPU nodes have simd_count 0)
    with the runtimes' visibility variables applied, never through torch / HIP."""
    sys.path.insert(0, ROOT)
    import bench
    root = _fake_kfd(tmp_path, [0, 256, 256, 256, 0, 256])
    assert bench.visible_gpus(root, {}) == (4, "kfd-topology")
    assert bench.visible_gpus(root, {"HIP_VISIBLE_DEVICES": "1,3"})[0] == 2
    assert bench.visible_gpus(root, {"ROCR_VISIBLE_DEVICES": "0", "HIP_VISIBLE_DEVICES": "0"})[0] == 1
    assert bench.visible_gpus(root, {"ROCR_VISIBLE_DEVICES": "0",
                                     "HIP_VISIBLE_DEVICES": "1"})[0] == 0   # index past the list
    assert bench.visible_gpus(root, {"HIP_VISIBLE_DEVICES": ""})[0] == 4   # empty = default
    assert bench.visible_gpus(root, {"CUDA_VISIBLE_DEVICES": "-1"})[0] == 0
    assert bench.visible_gpus(root, {"ROCR_VISIBLE_DEVICES": "GPU-abc,GPU-def"})[0] == 2
    assert bench.visible_gpus(root, {"HIP_VISIBLE_DEVICES": "0,9,1"})[0] == 1   # stops at 9
    sel = bench.launcher_selfcheck()
    assert set(sel) == {"torch_imported", "hip_runtime_mapped"}


def test_launcher_never_imports_torch(tmp_path):
    """The self-launcher refuses a too-large --gpus before any rank starts, and its selfcheck
    says torch was never imported into it (run with a fake 1-GPU topology)."""
    r = _run(["--gpus", "4", "--ranks-per-gpu", "2", "--dist-backend", "gloo", "--config",
              "cfg3"])
    assert r.returncode == 2 and "needs 2 visible GPUs" in r.stderr, r.stderr[-2000:]
    code = ("import sys, json; sys.path.insert(0, %r); import bench; "
            "bench.KFD_NODES = %r; "
            "n = bench.visible_gpus(); "
            "print(json.dumps([n, bench.launcher_selfcheck()]))" % (ROOT, _fake_kfd(tmp_path, [0, 8])))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    import json
    (n, src), sel = json.loads(out.stdout)
    assert n == 1 and src == "kfd-topology"
    assert sel == {"torch_imported": False, "hip_runtime_mapped": False}


def test_pcg_rule_branches():
    """Small problems replicate (the per-iteration all-reduce costs more than the observation
    work it splits), large ones shard; a slow gather pushes mid-size problems to 'sharded'; an
    expensive all-reduce pushes them to 'replicated'; world size 1 never replicates for free."""
    small, _ = R.pcg_rule(17_641, 8_812, 500, 8, 18.0, 100e9)
    large, t = R.pcg_rule(1_430_000, 100_000, 500, 8, 18.0, 100e9)
    assert small == "replicated" and large == "sharded"
    assert t["sharded_us_per_step"] < t["replicated_us_per_step"]
    mid = (300_000, 60_000, 500, 8)
    assert R.pcg_rule(*mid, 18.0, 5e9)[0] == "sharded"
    assert R.pcg_rule(*mid, 400.0, 100e9)[0] == "replicated"
    # the model's terms are internally consistent
    _, t = R.pcg_rule(500_000, 100_000, 500, 8, 20.0, 50e9)
    it = t["iters_assumed"]
    tn = lambda n: R.PCG_FIXED_US + R.PCG_OBS_US * n
    assert abs(t["sharded_us_per_step"] - it * (tn(500_000 / 8) + R.PCG_SPLIT_US + 20.0)) < 1e-6
    assert abs(t["replicated_us_per_step"] - (it * tn(500_000) + t["gather_us"])) < 1e-6

