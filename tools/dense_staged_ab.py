"""A/B of the dense kernels on bench.py's C3 images (round 6, x_verify_dense_staged.inc):
the production verify (count_scan -> verify_records: rows + expander + dense2) against
count_scan -> revel_x_verify_dense_variant(v) (the same split with another dense
kernel), same process, alternating arms, each a run of `iters` calls queued back to
back between two HIP events (ms per call), after untimed warm-up calls.  Every arm's
results are compared byte for byte with the production's first.
  python tools/dense_staged_ab.py [--shapes small,zipf] [--arms 4,5,6,7] [--rounds 5]"""
from __future__ import annotations

import argparse
import json
import os
import statistics as stat
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="small,zipf")
    ap.add_argument("--arms", default="4,5,6,7")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=9)
    ap.add_argument("--warmup", type=int, default=9)
    ap.add_argument("--gib", type=float, default=4.0)
    a = ap.parse_args()
    import bench
    from revel_amd import gpu
    from revel_amd._lib import check, experiments, lib
    from revel_amd.gpu import RECORD_DTYPE
    L, X = lib(), experiments()
    ctx = gpu.GpuContext(0)
    arms = ["product"] + [int(x) for x in a.arms.split(",") if x]
    for shape in a.shapes.split(","):
        seed = 0x5EED0003 if shape == "zipf" else 0x5EED0005
        img, n, nrec = bench.c3_image(ctx, shape, seed, a.gib)
        nblocks = (n + bench.BLOCK_SIZE - 1) // bench.BLOCK_SIZE
        counts, first = ctx.alloc(4 * nblocks), ctx.alloc(4 * nblocks)
        out = ctx.alloc((nrec + 2 * nblocks + 64) * RECORD_DTYPE.itemsize)

        def call(arm):
            check(L.revel_gpu_count_scan_records(ctx.handle, img.ptr, n, counts.ptr, first.ptr, None))
            if arm == "product":
                check(L.revel_gpu_verify_records(ctx.handle, img.ptr, n, 0, first.ptr, out.ptr, None))
            else:
                check(X.revel_x_verify_dense_variant(ctx.handle, arm, img.ptr, n, 0, first.ptr, out.ptr, None))

        def results():
            ctx.sync()
            nphys = int(ctx.d2h(first, 4 * nblocks, np.uint32)[-1]) + int(ctx.d2h(counts, 4 * nblocks, np.uint32)[-1])
            return ctx.d2h(out, nphys * RECORD_DTYPE.itemsize)

        ref = None
        ok = {}
        for arm in arms:
            ctx.memset(out, 0xA5, out.nbytes)
            call(arm)
            r = results()
            if ref is None:
                ref = r
            ok[str(arm)] = bool(r.size == ref.size and np.array_equal(r, ref))
        rec = ref.view(RECORD_DTYPE)
        print(json.dumps({"shape": shape, "image_bytes": n, "nphys": int(rec.size),
                          "not_ok": int((rec["status"] != 0).sum()), "identical": ok}), flush=True)
        e0, e1 = ctx.event(), ctx.event()
        times = {str(arm): [] for arm in arms}
        for _ in range(a.rounds):
            for arm in arms:
                for _ in range(a.warmup):
                    call(arm)
                e0.record()
                for _ in range(a.iters):
                    call(arm)
                e1.record()
                ctx.sync()
                times[str(arm)].append(e0.elapsed_ms(e1) / a.iters)
        print(json.dumps({"shape": shape, "ms_per_call_median": {k: round(stat.median(v), 4) for k, v in times.items()},
                          "runs": {k: [round(x, 4) for x in v] for k, v in times.items()}}), flush=True)
        for b in (counts, first, out, img):
            b.free()


if __name__ == "__main__":
    main()
