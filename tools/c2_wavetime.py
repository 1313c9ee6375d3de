"""Per-wave end times of the C2 kernel (k_full_blocks4) from a build with
-DREVEL_C2_WAVETIME, on bench.py's C2 workload: how the waves of a
workgroup finish by slot (the SIMD's arbiter favours older waves), by XCD,
and the kernel's tail.

    python tools/c2_wavetime.py --lib build/ab/c2wt.so [--blocks 1048576]
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
    ap.add_argument("--blocks", type=int, default=1 << 20)
    a = ap.parse_args()
    from revel_amd import _lib
    _lib.LIB_PATH = os.path.abspath(a.lib)
    import bench
    from revel_amd import BLOCK_SIZE, gpu
    ctx = gpu.GpuContext(0)
    n = a.blocks
    d, m, ok = ctx.alloc(n * BLOCK_SIZE), ctx.alloc(4 * n), ctx.alloc(n)
    ctx.synth_full_blocks(d, n, seed=bench.SEED)
    for _ in range(3):
        ctx.crc_full_blocks(d, n, m, ok)
    ctx.sync()
    f = _lib.lib().revel_debug_c2_wavetime
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64]
    buf = np.zeros(3 * 65536, np.uint64)
    assert f(buf.ctypes.data, buf.size) == 0
    w = buf.reshape(-1, 3)
    wid = np.flatnonzero(w[:, 1] > 0)
    start, end = w[wid, 0].astype(np.int64), w[wid, 1].astype(np.int64)
    e = (end - start.min()) / 100.0
    wg, slot = wid // 16, wid % 16
    print(json.dumps({"waves": int(len(wid)), "all_ok": bool(ctx.d2h(ok, n).all()),
                      "span_us": round(float(e.max()), 1),
                      "end_us_p0_p10_p50_p90_max": [round(float(np.percentile(e, q)), 1) for q in (0, 10, 50, 90, 100)],
                      "end_us_by_wave_slot_median": [round(float(np.median(e[slot == k])), 1) for k in range(16)],
                      "end_us_by_xcd_median": [round(float(np.median(e[(wg % 8) == x])), 1) for x in range(8)],
                      "end_us_by_xcd_max": [round(float(np.max(e[(wg % 8) == x])), 1) for x in range(8)],
                      "tail_us_max_minus_p50": round(float(e.max() - np.median(e)), 1)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
