"""In-kernel clock of the K1 mutual kernel (MI355X_MICROARCH.md "DVFS give-back" item 6): with the
diagnostic library (tools/build_variant.sh clock -DMU_CLOCK; SFMCORE_LIB=.../libsfmcore_clock.so)
every block stamps s_memtime / s_memrealtime around its train loop.  After >= 2 s of back-to-back
launches on the cfg3 workload (K=, N_IMG= override), the stamps of the last launch give the clock
(delta memtime / delta realtime x 100 MHz, median over blocks) and the shader cycles per 32-train
tile per wave.  Usage: SFMCORE_LIB=... python tests/perf/k1_clock.py"""
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


def main():
    n_img = int(os.environ.get("N_IMG", "50"))
    K = int(os.environ.get("K", "2048"))
    s = synth.make_scene(n_img, K, seed=0)
    pairs = synth.unordered_pairs(n_img)
    ctx = sfmcore.context(0)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    desc, n_kp, pr = T(s["desc"]), T(s["n_kp"]), T(pairs)
    out = ctx.match_batch(desc, n_kp, pr, ratio=(4, 5))
    torch.cuda.synchronize()
    t0, n = time.time(), 0
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    while time.time() - t0 < 2.5:
        ev[0].record()
        for _ in range(20):
            out = ctx.match_batch(desc, n_kp, pr, ratio=(4, 5), out=out)
        ev[1].record()
        torch.cuda.synchronize()
        n += 20
    ms = ev[0].elapsed_time(ev[1]) / 20
    qb = 512                                      # MU_WAVES (4) x QT (4) x 32 queries per block
    n_blk = len(pairs) * ((K + qb - 1) // qb)
    persist = os.environ.get("SFM_MU_PERSIST", "0") == "1"
    grid = 512 if persist else 8 * ((n_blk + 7) // 8)  # persistent: 2 blocks per CU x 256 CUs
    W = 8
    buf = np.zeros(W * grid, np.uint64)
    L = sfmcore.load_library()
    L.sfm_debug_clock_stamps.argtypes = [C.c_void_p, C.c_int32]
    assert L.sfm_debug_clock_stamps(buf.ctypes.data_as(C.c_void_p), grid) == 0
    raw = buf.reshape(-1, W)
    raw = raw[raw[:, 2] > raw[:, 0]]
    st = raw[:, :4].astype(np.float64)
    cyc = st[:, 2] - st[:, 0]
    wall = (st[:, 3] - st[:, 1]) / 100e6
    clk = cyc / wall
    # per wave: every train tile of the pair (one block per item), or the block's share of all
    # units x 4 tiles (persistent schedule)
    tiles = (n_blk * (K // 128) / grid * 4) if persist else K // 32
    res = {"workload": f"{len(pairs)} pairs x {K}", "persistent": persist, "launches": n, "launch_ms": ms,
           "blocks": int(len(st)), "clock_GHz_median": float(np.median(clk) / 1e9),
           "clock_GHz_p10_p90": [float(np.percentile(clk, 10) / 1e9),
                                 float(np.percentile(clk, 90) / 1e9)],
           "block_cycles_median": float(np.median(cyc)),
           "cycles_per_tile_wave_median": float(np.median(cyc) / tiles),
           "block_us_median": float(np.median(wall) * 1e6)}
    # whole-block lifetime (entry -> after the colpart store) and the per-CU timeline
    t_in, t_out = raw[:, 4].astype(np.int64), raw[:, 5].astype(np.int64)
    l0, l1 = raw[:, 1].astype(np.int64), raw[:, 3].astype(np.int64)
    cu = ((raw[:, 7].astype(np.int64) & 15) << 8) | ((raw[:, 6].astype(np.int64) >> 8) & 255)
    life = (t_out - t_in) / 100.0  # us
    res["block_life_us_median"] = float(np.median(life))
    res["block_life_us_p10_p90_max"] = [float(np.percentile(life, 10)), float(np.percentile(life, 90)),
                                        float(life.max())]
    xcc = raw[:, 7].astype(np.int64) & 15
    res["block_life_us_mean_by_xcc"] = [float(life[xcc == x].mean()) if (xcc == x).any() else None
                                        for x in range(8)]
    res["prologue_us_median"] = float(np.median((l0 - t_in) / 100.0))
    res["epilogue_us_median"] = float(np.median((t_out - l1) / 100.0))
    span = (t_out.max() - t_in.min()) / 100.0
    res["launch_span_us"] = float(span)
    ucu = np.unique(cu)
    res["cus_seen"] = int(len(ucu))
    occ, idle_gap = [], []
    for c in ucu:
        m = cu == c
        occ.append(life[m].sum() / span)
        a, b = np.sort(t_in[m]), np.sort(t_out[m])
        # slots: a block starts when another leaves; gaps = entry - the latest exit before it
        ex = np.sort(t_out[m])
        for t in a[2:]:
            k = np.searchsorted(ex, t) - 1
            if k >= 0:
                idle_gap.append((t - ex[k]) / 100.0)
    res["blocks_per_cu_mean"] = float(len(raw) / len(ucu))
    res["cu_block_occupancy_mean"] = float(np.mean(occ))  # sum of block lifetimes / span (2 = full)
    res["refill_gap_us_median"] = float(np.median(idle_gap)) if idle_gap else None
    first = np.sort(t_in)[:512]
    last = np.sort(t_out)[-512:]
    res["first_512_entries_spread_us"] = float((first.max() - first.min()) / 100.0)
    res["last_512_exits_spread_us"] = float((last.max() - last.min()) / 100.0)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
