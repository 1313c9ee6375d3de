"""Load balance of k_verify_rows: a build with -DREVEL_ROWS_WAVETIME records
each wave's start / end time (s_memrealtime, 100 MHz) and block count; this
runs bench.py's c3 image through the production verify a few times and
prints, for the last launch, the spread of the waves' end times against the
kernel's span (how much of the kernel is its tail).

    python tools/rows_wavetime.py --lib build/ab/wavetime.so [--shape zipf]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--shape", default="zipf")
    ap.add_argument("--gib", type=float, default=4.0)
    a = ap.parse_args()
    from revel_amd import _lib
    _lib.LIB_PATH = os.path.abspath(a.lib)
    import bench
    from revel_amd import gpu
    ctx = gpu.GpuContext(0)
    img, n, nrec = bench.c3_image(ctx, a.shape, 0x5EED0003 if a.shape == "zipf" else 0x5EED0005, a.gib)
    t, nphys, bad = bench.c3_verify_timed(ctx, img, n, nrec, 3)
    L = _lib.lib()
    f = L.revel_debug_rows_wavetime
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]
    buf = np.zeros(3 * 65536, np.uint64)
    assert f(buf.ctypes.data, buf.size) == 0
    w = buf.reshape(-1, 3)
    w = w[w[:, 1] > 0]
    start, end, nb = w[:, 0].astype(np.int64), w[:, 1].astype(np.int64), w[:, 2]
    t0 = start.min()
    us = lambda x: x / 100.0  # 100 MHz ticks -> us
    e = us(end - t0)
    s = us(start - t0)
    wid = np.flatnonzero(buf.reshape(-1, 3)[:, 1] > 0)  # global wave index w0
    wg = wid // 16
    by_xcd = {int(x): [round(float(np.median(e[(wg % 8) == x])), 1), round(float(e[(wg % 8) == x].max()), 1)]
              for x in range(8)}
    slot = wid % 16  # wave slot inside its workgroup
    by_slot = [round(float(np.median(e[slot == k])), 1) for k in range(16)]
    wg_med = np.array([np.median(e[wg == g]) for g in np.unique(wg)])
    print(json.dumps({"end_us_by_xcd_median_max": by_xcd, "end_us_by_wave_slot_median": by_slot,
                      "end_us_wg_median_p0_p50_p100": [round(float(np.min(wg_med)), 1), round(float(np.median(wg_med)), 1),
                                                        round(float(np.max(wg_med)), 1)],
                      "end_us_first_waves": [round(float(x), 1) for x in e[:20]]}), flush=True)
    print(json.dumps({"waves": int(len(w)), "bad_records": bad, "ms_calls": [round(x, 4) for x in t],
                      "span_us": round(float(e.max()), 1),
                      "start_us_p50_max": [round(float(np.median(s)), 1), round(float(s.max()), 1)],
                      "end_us_p0_p10_p50_p90_p99_max": [round(float(np.percentile(e, q)), 1) for q in (0, 10, 50, 90, 99, 100)],
                      "blocks_per_wave_min_p50_max": [int(nb.min()), int(np.median(nb)), int(nb.max())],
                      "tail_us_max_minus_p50": round(float(e.max() - np.median(e)), 1)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
