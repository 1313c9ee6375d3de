"""bench.py's c3 / c3_small legs alone (same images, same timing), for
kernel traces and A/B builds:  python tools/c3_legs.py [--shapes zipf,small] [--iters 9]"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="zipf,small")
    ap.add_argument("--iters", type=int, default=9)
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--warmup-calls", type=int, default=-1, help="untimed queued calls before the steady runs (default: bench.py's)")
    a = ap.parse_args()
    import bench
    from revel_amd import gpu
    ctx = gpu.GpuContext(0)
    for shape in a.shapes.split(","):
        seed = 0x5EED0003 if shape == "zipf" else 0x5EED0005
        img, n, nrec = bench.c3_image(ctx, shape, seed, a.gib)
        streamed = []
        times, nphys, bad = bench.c3_verify_timed(ctx, img, n, nrec, a.iters, stream=streamed, stream_runs=5,
                                                  stream_warmup=bench.C3_STREAM_WARMUP if a.warmup_calls < 0 else a.warmup_calls)
        img.free()
        print(json.dumps({"shape": shape, "ms_steady_median": round(float(np.median(streamed)), 4),
                          "ms_steady_runs": [round(x, 4) for x in streamed],
                          "ms_isolated_median": round(float(np.median(times)), 4), "nphys": nphys, "bad": bad,
                          "image_bytes": n, "warmup_calls": a.warmup_calls,
                          "env": {k: v for k, v in os.environ.items() if k.startswith("REVEL_")}}), flush=True)


if __name__ == "__main__":
    main()
