"""Block-order experiment for k_verify_rows: the same
qualifying blocks in different list orders, wave j taking list[j], list[j + W],
...  asc = block order, shuffle = random (what the atomic list build gives),
desc = by record count, most first (LPT-like), snake = desc with every other
stride of W reversed.  Times the rows kernel alone (HIP events), interleaved
rounds; checks every order reproduces the production results."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench_c3 import make_image  # noqa: E402
from revel_amd import BLOCK_SIZE, gpu  # noqa: E402
from revel_amd._lib import check, experiments, lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--tile", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--orders", default="asc,shuffle,desc,snake")
    a = ap.parse_args()
    ctx = gpu.GpuContext(0)
    img = make_image(a.bytes)
    whole = len(img) // BLOCK_SIZE * BLOCK_SIZE
    img = img[:whole] * a.tile
    n = len(img)
    d = ctx.upload(np.frombuffer(img, dtype=np.uint8))
    L, X = lib(), experiments()
    X.revel_x_rows_waves.restype = ctypes.c_int
    X.revel_x_rows_waves.argtypes = [ctypes.c_void_p]
    X.revel_x_verify_rows_list.restype = ctypes.c_int
    X.revel_x_verify_rows_list.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_size_t] + [ctypes.c_void_p] * 4
    W = X.revel_x_rows_waves(ctx.handle)
    nblocks = n // BLOCK_SIZE
    counts, first = ctx.alloc(4 * nblocks), ctx.alloc(4 * nblocks)

    def count():
        check(L.revel_gpu_count_records(ctx.handle, d.ptr, n, counts.ptr, None))
        check(L.revel_gpu_exclusive_scan_u32(ctx.handle, counts.ptr, first.ptr, nblocks, None))

    count()
    c = ctx.d2h(counts, 4 * nblocks, np.uint32)
    nrec = int(ctx.d2h(first, 4 * nblocks, np.uint32)[-1]) + int(c[-1])
    out = ctx.alloc(24 * nrec)
    check(L.revel_gpu_verify_records(ctx.handle, d.ptr, n, 0, first.ptr, out.ptr, None))
    ctx.sync()
    ref = ctx.d2h(out, 24 * nrec, np.uint8)
    q = np.nonzero((c >= 1) & (c <= 64))[0].astype(np.uint32)
    rng = np.random.default_rng(7)
    desc = q[np.argsort(-c[q].astype(np.int64), kind="stable")]
    snake = desc.copy()
    for k in range(0, len(desc), W):
        if (k // W) % 2:
            snake[k:k + W] = desc[k:k + W][::-1]
    lists = {"asc": q, "shuffle": rng.permutation(q), "desc": desc, "snake": snake}
    orders = a.orders.split(",")
    dl = {o: ctx.upload(np.concatenate([[len(lists[o])], lists[o]]).astype(np.uint32)) for o in orders}
    e0, e1 = ctx.event(), ctx.event()
    times = {o: [] for o in orders}
    ok = {o: True for o in orders}
    for _ in range(a.rounds):
        for o in orders:
            for _ in range(a.iters):
                count()
                e0.record()
                check(X.revel_x_verify_rows_list(ctx.handle, d.ptr, n, first.ptr, out.ptr, dl[o].ptr, None))
                e1.record()
                ctx.sync()
                times[o].append(e0.elapsed_ms(e1))
            ok[o] = ok[o] and bool(np.array_equal(ctx.d2h(out, 24 * nrec, np.uint8), ref))
    for o in orders:
        print(json.dumps({"order": o, "waves": W, "listed_blocks": int(len(q)), "blocks": nblocks,
                          "rows_ms_median": round(float(np.median(times[o])), 4),
                          "rows_ms_min": round(float(np.min(times[o])), 4), "matches_production": ok[o]}),
              flush=True)


if __name__ == "__main__":
    main()
