"""A/B of two C3 verify pipelines on one box, alternating, through a debug
switch of the library (1 = arm A, 0 = arm B), on bench.py's 4 GiB Zipf and
small-record images; checks both give identical results on every image.
  --hook revel_debug_set_fused (default): the one-pass count + checksum path
    (k_walk_verify -> scan -> k_expand_fused, round 5) vs the two-read path;
  --hook revel_debug_set_dense_chunks: dense blocks by k_verify_dense_chunks
    (+ dense2 over the rest, round 5) vs dense2 over all of them (round 4).

    python tools/ab_fused.py [--hook NAME] [--gib 4] [--rounds 4] [--iters 9]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=9)
    ap.add_argument("--shapes", default="small,zipf")
    ap.add_argument("--hook", default="revel_debug_set_fused")
    ap.add_argument("--on", type=int, default=1, help="the hook's value for arm A (arm B: 0)")
    a = ap.parse_args()
    import bench
    from revel_amd import gpu
    from revel_amd._lib import lib
    from revel_amd.gpu import RECORD_DTYPE
    L = lib()
    import ctypes
    hook = getattr(L, a.hook)
    hook.restype = ctypes.c_int
    hook.argtypes = [ctypes.c_int]
    ctx = gpu.GpuContext(0)
    out = {}
    for shape in a.shapes.split(","):
        seed = 0x5EED0003 if shape == "zipf" else 0x5EED0005
        img, n, nrec = bench.c3_image(ctx, shape, seed, a.gib)
        res = {}
        digests = {}
        for r in range(a.rounds):
            for mode in (a.on, 0):
                hook(mode)
                mode = 1 if mode else 0
                streamed = []
                times, nphys, bad = bench.c3_verify_timed(ctx, img, n, nrec, a.iters, stream=streamed)
                res.setdefault(mode, {"iso": [], "steady": []})
                res[mode]["iso"].append(float(np.median(times)))
                res[mode]["steady"].append(streamed[0])
                if r == 0:
                    # full result digest of the last call (every field)
                    nblocks = (n + 32767) // 32768
                    counts, first = ctx.alloc(4 * nblocks), ctx.alloc(4 * nblocks)
                    o = ctx.alloc((nphys + 1) * RECORD_DTYPE.itemsize)
                    from revel_amd._lib import check
                    check(L.revel_gpu_count_scan_records(ctx.handle, img.ptr, n, counts.ptr, first.ptr, None))
                    check(L.revel_gpu_verify_records(ctx.handle, img.ptr, n, 0, first.ptr, o.ptr, None))
                    ctx.sync()
                    raw = ctx.d2h(o, nphys * RECORD_DTYPE.itemsize)
                    import hashlib
                    digests[mode] = (nphys, bad, hashlib.sha256(raw.tobytes()).hexdigest()[:16])
                    for b in (counts, first, o):
                        b.free()
                print(json.dumps({"shape": shape, "round": r, "arm_on": mode, "ms_iso": round(res[mode]["iso"][-1], 4),
                                  "ms_steady": round(res[mode]["steady"][-1], 4), "nphys": nphys, "bad": bad}),
                      flush=True)
        hook(-1)
        img.free()
        out[shape] = {
            "bytes": n,
            "hook": a.hook,
            "on_ms_steady_median": round(float(np.median(res[1]["steady"])), 4),
            "off_ms_steady_median": round(float(np.median(res[0]["steady"])), 4),
            "on_ms_iso_median": round(float(np.median(res[1]["iso"])), 4),
            "off_ms_iso_median": round(float(np.median(res[0]["iso"])), 4),
            "identical_results": digests.get(1) == digests.get(0),
            "digests": {str(k): v for k, v in digests.items()},
        }
        print(json.dumps({shape: out[shape]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
