"""The count pass alone (revel_gpu_count_records: k_count_hist) on bench.py's
c3 images, on any build of librevel_wal.so (probe builds by
tools/build_variant.sh), HIP events, median of --reps.

    python tools/count_ab.py [--lib build/ab/X.so] [--shapes zipf,small]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--shapes", default="zipf,small")
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    if a.lib:
        from revel_amd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    import bench
    from revel_amd import gpu
    from revel_amd._lib import check, lib
    L = lib()
    ctx = gpu.GpuContext(0)
    e0, e1 = ctx.event(), ctx.event()
    for shape in a.shapes.split(","):
        img, n, _ = bench.c3_image(ctx, shape, 0x5EED0003 if shape == "zipf" else 0x5EED0005, a.gib)
        nb = (n + 32767) // 32768
        cnt = ctx.alloc(4 * nb)
        ts = []
        for _ in range(a.reps + 3):
            e0.record()
            check(L.revel_gpu_count_records(ctx.handle, img.ptr, n, cnt.ptr, None))
            e1.record()
            ctx.sync()
            ts.append(e0.elapsed_ms(e1))
        ts = ts[3:]
        c = ctx.d2h(cnt, 4 * nb, np.uint32)
        print(json.dumps({"lib": a.lib or "in-tree", "shape": shape, "count_ms_median": round(float(np.median(ts)), 4),
                          "count_ms_min": round(min(ts), 4), "records": int(c.sum())}), flush=True)
        img.free()
        cnt.free()


if __name__ == "__main__":
    main()
