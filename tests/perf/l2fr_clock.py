"""Where the forward scan's time goes, from in-kernel stamps (diagnostic build -DL2FR_CLOCK,
tools/build_variant.sh <name> -DL2FR_CLOCK; SFMCORE_LIB=.../libsfmcore_<name>.so).

Runs the scan-only launch (SFM_L2FR_DEBUG=1: prep + order + forward scan + dump) back to back for
>= 2 s on the cfg2/cfg3 workload (N_IMG, K override), then reads the last launch's per-block
stamps and reports: the kernel span, block life split into prologue (entry -> first stage landed),
train loop and epilogue, the per-chunk loop time and its MFMA efficiency (a SIMD runs 2 waves x
CHUNK/32 tiles x 16 MFMAs x 32 cycles per chunk), the in-kernel clock (memtime / realtime), and per
CU the idle time between consecutive blocks and after its last block (tail).
python tests/perf/l2fr_clock.py"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sfm-project_amd")]

import numpy as np
import torch

import sfmcore
import synth

W = 24


def main():
    n_img = int(os.environ.get("N_IMG", "50"))
    K = int(os.environ.get("K", "2048"))
    chunk = int(os.environ.get("CHUNK", "256"))
    s = synth.make_scene(n_img, K, seed=0)
    pairs = synth.unordered_pairs(n_img)
    ctx = sfmcore.context(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    desc, n_kp, pr = T(s["desc"]), T(s["n_kp"]), T(pairs)
    os.environ["SFM_L2FR_DEBUG"] = "1"
    out = ctx.match_batch(desc, n_kp, pr, cross_check=0, ratio=(4, 5))
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.time()
    while time.time() - t0 < 2.5:
        ev[0].record()
        for _ in range(20):
            out = ctx.match_batch(desc, n_kp, pr, cross_check=0, ratio=(4, 5), out=out)
        ev[1].record()
        torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / 20
    qb = int(os.environ.get("QB", "1024"))
    n_qblk = (K + qb - 1) // qb
    grid = 8 * ((len(pairs) + 7) // 8) * n_qblk
    buf = np.zeros(W * grid, np.uint64)
    L = sfmcore.load_library()
    L.sfm_debug_l2fr_stamps.argtypes = [C.c_void_p, C.c_int32]
    assert L.sfm_debug_l2fr_stamps(buf.ctypes.data_as(C.c_void_p), grid) == 0
    raw = buf.reshape(-1, W).astype(np.int64)
    raw = raw[raw[:, 21] > raw[:, 0]]
    rt = lambda i: raw[:, i].astype(np.float64) / 100.0          # realtime ticks (10 ns) -> us
    entry, pro, lend, ex = rt(0), rt(1), rt(20), rt(21)
    span = ex.max() - entry.min()
    clk = (raw[:, 19] - raw[:, 2]) / ((raw[:, 20] - raw[:, 1]) * 10e-9) / 1e9
    n_chunk = (K + chunk - 1) // chunk
    ch_end = np.stack([rt(3 + c) for c in range(min(n_chunk, 16))], 1)
    ch_t = np.diff(np.concatenate([pro[:, None], ch_end], 1), axis=1)
    mfma_cyc_chunk = int(os.environ.get("WPS", "2")) * (chunk // 32) * 16 * 32  # waves/SIMD of one block
    eff = mfma_cyc_chunk / (ch_t * np.median(clk) * 1e3)
    hw, xcc = raw[:, 22], raw[:, 23]
    cu_key = (xcc & 0xF) * 4096 + ((hw >> 13) & 0x7) * 256 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 0xF)
    gaps, tails, busy = [], [], []
    t_end = ex.max()
    for k in np.unique(cu_key):
        m = cu_key == k
        o = np.argsort(entry[m])
        e_, x_ = entry[m][o], ex[m][o]
        gaps.extend((e_[1:] - x_[:-1]).tolist())
        tails.append(t_end - x_[-1])
        busy.append((x_ - e_).sum())
    res = {
        "lib": os.path.basename(os.environ.get("SFMCORE_LIB", "base")),
        "n_img": n_img, "K": K, "blocks": int(len(raw)), "cus": int(len(np.unique(cu_key))),
        "launch_ms": ms, "span_us": span,
        "clock_ghz_median": float(np.median(clk)),
        "block_us": {"median": float(np.median(ex - entry)), "prologue": float(np.median(pro - entry)),
                     "loop": float(np.median(lend - pro)), "epilogue": float(np.median(ex - lend))},
        "chunk_us_median": [float(x) for x in np.median(ch_t, 0)],
        "chunk_mfma_eff_median": [float(x) for x in np.median(eff, 0)],
        "cu_gap_us": {"median": float(np.median(gaps)), "mean": float(np.mean(gaps)),
                      "sum_per_cu_mean": float(np.sum(gaps) / len(tails))},
        "cu_tail_us": {"median": float(np.median(tails)), "mean": float(np.mean(tails))},
        "cu_busy_frac_mean": float(np.mean(busy) / span),
        # matrix cycles of the whole launch per SIMD (4 i8 32x32x32 MFMAs of 32 cycles per 32x32
        # element tile) over the span at the in-kernel clock
        "kernel_mfma_eff": float(len(pairs) * (K // 32) ** 2 * 128 / 1024 / (span * np.median(clk) * 1e3)),
    }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
