"""CPU: libsfmcore.so builds for gfx950, loads, and exports every entry point include/sfmcore.h
declares; argument validation runs host-side (no compute without a GPU)."""
import ctypes as C
import os
import re
import subprocess

import pytest

import sfmcore

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sfmcore.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|const char\*)\s+(sfm_\w+)\s*\(", src, re.M)))


def test_header_declares_the_abi():
    fns = declared_functions()
    assert set(fns) == set(sfmcore.EXPORTED)


def test_library_exports_every_declared_symbol():
    lib = sfmcore.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", sfmcore.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    for name in declared_functions():
        assert re.search(rf"\bT {name}\b", out), name


def test_library_targets_gfx950_only():
    data = open(sfmcore.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    for other in (b"gfx942", b"gfx90a", b"gfx908", b"sm_"):
        assert b"amdgcn-amd-amdhsa--" + other not in data


def test_version_and_errors_without_device():
    lib = sfmcore.load_library()
    assert lib.sfm_version() == 5   # 2: poll 0 = every 8; 3: BA chunk mode; 4: explicit Schur;
    # 5: sfm_ba_solve_params.poll_first
    prm = sfmcore.MatchParams(0, 1, 4, 5, -1)
    rc = lib.sfm_match_batch(None, None, None, 0, 0, 128, None, 1, C.byref(prm), None, None, None)
    assert rc == -1
    assert b"NULL" in lib.sfm_last_error()
    rp = sfmcore.RansacParams(4096, 15, 1.0, 0, 42)
    assert lib.sfm_ransac_f_batch(None, None, 0, 0, None, 1, None, None, C.byref(rp), None, None,
                                  None, None, None) == -1
    # the graph exchange entries refuse a NULL context and a packed layout they cannot encode
    assert lib.sfm_graph_rows_packed(None, 1, 16, None, None, None, None, 15, None, None) == -1
    assert b"sfm_graph_rows_packed" in lib.sfm_last_error()
    assert lib.sfm_graph_expand(None, 1, 0, None, None, None, None, None) == -1
    assert b"sfm_graph_expand" in lib.sfm_last_error()


def test_ctx_create_reports_missing_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    lib = sfmcore.load_library()
    h = C.c_void_p()
    rc = lib.sfm_ctx_create(0, C.byref(h))
    assert rc != 0 and not h.value
    assert len(lib.sfm_last_error()) > 0
    with pytest.raises(sfmcore.SfmCoreError):
        sfmcore.Context(0)
