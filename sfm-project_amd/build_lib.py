"""Builds libsfmcore.so (all HIP kernels + the C-ABI) for gfx950 with hipcc, in-tree.

Used by __graft_entry__.build() and by the Python host on first import when the library is
missing.  The output lives in sfm-project_amd/lib/ (git-ignored, shipped to the GPU box).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libsfmcore.so")
SOURCES = ["capi.hip", "match_mfma.hip", "match_l2fr.hip", "match_hamming.hip", "ransac.hip", "ba.hip", "ba_solve.hip", "graph.hip", "tracks.hip", "triangulate.hip", "register.hip", "orb.hip", "calib.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -ffp-contract=off: RANSAC follows the oracle's op sequence bit-for-bit (explicit fmaf only).
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-fno-gpu-rdc", "-Wall", "-Wno-unused-function"]


# Per-file extra flags.  ransac.hip: no SLP vectorisation — on gfx950 v_pk_fma_f32 has the same
# FLOP rate as v_fma_f32 (MI355X_MICROARCH.md), so packing only adds operand-shuffle v_movs.
EXTRA = {"ransac.hip": ["-fno-slp-vectorize"]}


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    deps.append(os.path.join(HERE, "..", "include", "sfmcore.h"))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    objs = []
    procs = []
    for src in SOURCES:
        obj = os.path.join(LIB_DIR, src.replace(".hip", ".o"))
        cmd = [HIPCC, *FLAGS, *EXTRA.get(src, []), "-c", os.path.join(CSRC, src), "-o", obj]
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        objs.append(obj)
    for cmd, pr in procs:
        out, _ = pr.communicate()
        if pr.returncode != 0:
            sys.stderr.write(out.decode())
            raise RuntimeError("hipcc failed: " + " ".join(cmd))
        if verbose and out:
            sys.stderr.write(out.decode())
    tmp = LIB + ".tmp"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-o", tmp, *objs], check=True)
    os.replace(tmp, LIB)
    for o in objs:
        os.remove(o)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
