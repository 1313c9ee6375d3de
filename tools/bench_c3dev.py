"""bench.py's c3 / c3_small legs alone (the same device-framed images, the
same C-ABI calls and HIP-event timing), on any build of librevel_wal.so:
A/B runs of builds on exactly the image the driver's bench line measures.

    python tools/bench_c3dev.py [--lib A.so] [--shape zipf|small] [--gib 4] [--iters 9]

Prints one JSON line: median / min ms, algorithmic GB/s (image + 24 B per
physical record, as bench.py), and whether every record verified.
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
    ap.add_argument("--shape", choices=["zipf", "small"], default="zipf")
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--iters", type=int, default=9)
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--walk", type=int, default=None,
                    help="1: the fused pipeline (row stream walks the headers), 0: the count pass; default: the "
                         "context's (REVEL_C3_WALK)")
    a = ap.parse_args()
    if a.lib:
        from revel_amd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    import bench
    from revel_amd import gpu
    ctx = gpu.GpuContext(0)
    if a.walk is not None:
        ctx.set_c3_walk(a.walk)
    seed = 0x5EED0003 if a.shape == "zipf" else 0x5EED0005
    img, n, nrec = bench.c3_image(ctx, a.shape, seed, a.gib)
    times = []
    for _ in range(a.rounds):
        t, nphys, bad = bench.c3_verify_timed(ctx, img, n, nrec, a.iters)
        times += t
    ms = float(np.median(times))
    print(json.dumps({"lib": (a.lib or "in-tree") + ("" if a.walk is None else f":walk{a.walk}"), "shape": a.shape, "image_bytes": n, "physical_records": nphys,
                      "bad_records": bad, "ms_median": round(ms, 4), "ms_min": round(min(times), 4),
                      "ms_all": [round(x, 4) for x in times], "GiB_s": round(n / 2**30 / (ms / 1e3), 1),
                      "alg_GB_s": round((n + 24 * nphys) / (ms / 1e3) / 1e9, 1)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
