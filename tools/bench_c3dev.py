"""bench.py's c3 / c3_small legs alone (the same device-framed images, the
same C-ABI calls and HIP-event timing), on any build of librevel_wal.so:
A/B runs of builds on exactly the image the driver's bench line measures.

    python tools/bench_c3dev.py [--lib A.so] [--shape zipf|small] [--gib 4] [--iters 9]

Prints one JSON line: median / min ms of isolated calls, ms per call of
--iters calls queued back to back (ms_stream: bench.py's c3 "ms"),
algorithmic GB/s (image + 24 B per physical record, as bench.py), and
whether every record verified.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def walk_timed(ctx, img, n, nrec, iters):
    """bench.c3_verify_timed through the experiment module's fused pipeline."""
    from revel_amd._lib import check, experiments
    from revel_amd.gpu import RECORD_DTYPE
    X = experiments()
    nblocks = (n + 32767) // 32768
    counts, first = ctx.alloc(4 * nblocks), ctx.alloc(4 * nblocks)
    out = ctx.alloc((nrec + 2 * nblocks + 64) * RECORD_DTYPE.itemsize)
    e0, e1 = ctx.event(), ctx.event()
    times = []
    for _ in range(iters):
        e0.record()
        check(X.revel_x_walk_count_scan(ctx.handle, img.ptr, n, counts.ptr, first.ptr, None))
        check(X.revel_x_walk_verify(ctx.handle, img.ptr, n, 0, counts.ptr, first.ptr, out.ptr, None))
        e1.record()
        ctx.sync()
        times.append(e0.elapsed_ms(e1))
    nphys = int(ctx.d2h(first, 4 * nblocks, np.uint32)[-1]) + int(ctx.d2h(counts, 4 * nblocks, np.uint32)[-1])
    res = ctx.d2h(out, nphys * RECORD_DTYPE.itemsize).view(RECORD_DTYPE)
    return times, nphys, int((res["status"] != 0).sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--shape", choices=["zipf", "small"], default="zipf")
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--iters", type=int, default=9)
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--walk", type=int, default=0,
                    help="1: the fused pipeline of tools/experiments (x_verify_walk.inc) instead of the product's")
    a = ap.parse_args()
    if a.lib:
        from revel_amd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    import bench
    from revel_amd import gpu
    ctx = gpu.GpuContext(0)
    seed = 0x5EED0003 if a.shape == "zipf" else 0x5EED0005
    img, n, nrec = bench.c3_image(ctx, a.shape, seed, a.gib)
    times, streamed = [], []
    for _ in range(a.rounds):
        if a.walk:
            t, nphys, bad = walk_timed(ctx, img, n, nrec, a.iters)
        else:
            t, nphys, bad = bench.c3_verify_timed(ctx, img, n, nrec, a.iters, stream=streamed, stream_runs=5,
                                                      stream_warmup=bench.C3_STREAM_WARMUP)
        times += t
    ms = float(np.median(times))
    mss = float(np.median(streamed)) if streamed else None
    print(json.dumps({"lib": (a.lib or "in-tree") + (":walk" if a.walk else ""), "shape": a.shape, "image_bytes": n, "physical_records": nphys,
                      "bad_records": bad, "ms_median": round(ms, 4), "ms_min": round(min(times), 4),
                      "ms_all": [round(x, 4) for x in times], "GiB_s": round(n / 2**30 / (ms / 1e3), 1),
                      "alg_GB_s": round((n + 24 * nphys) / (ms / 1e3) / 1e9, 1),
                      "ms_stream": round(mss, 4) if mss else None,
                      "alg_GB_s_stream": round((n + 24 * nphys) / (mss / 1e3) / 1e9, 1) if mss else None}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
