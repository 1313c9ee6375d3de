"""Config C3 throughput: Zipf-mixed 64 B..32 KiB records (FIRST/MIDDLE/LAST
fragments), written by the product log::Writer into a ~1 GiB image, copied to
HBM once, then device walk + segmented CRC verify timed with HIP events.

Record size = 64*k bytes, k in [1, 512] ~ Zipf(1.1) (seed 0x5EED0003).
Prints one JSON line.  Correctness here = every physical record verifies OK
against the CRC the host writer stored (the GPU tests check bit-exactness
against the oracle).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from revel_amd import BLOCK_SIZE, env, gpu, log  # noqa: E402
from revel_amd._lib import check, experiments, lib  # noqa: E402


def make_image(target: int, seed: int = 0x5EED0003) -> bytes:
    rng = np.random.default_rng(seed)
    k = np.arange(1, 513)
    p = k ** -1.1
    p /= p.sum()
    sizes = 64 * rng.choice(k, size=target // 2000 + 16, p=p)
    blob = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8).tobytes()
    f = env.MemoryWritableFile()
    w = log.Writer(f)
    off = 0
    for s in sizes:
        w.add_record(blob[off:off + int(s)])
        off += int(s)
        if f_size(f) >= target:
            break
    return f.contents()


def f_size(f) -> int:
    import ctypes
    p, n = ctypes.c_void_p(), ctypes.c_size_t()
    check(lib().revel_memory_writable_file_contents(f.handle, ctypes.byref(p), ctypes.byref(n)))
    return n.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=1 << 30, help="size of the written Zipf image")
    ap.add_argument("--tile", type=int, default=4, help="repeat the image's whole blocks this many times")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=1, help="interleaved rounds over the variants")
    ap.add_argument("--variants", default="0,15")
    ap.add_argument("--lib", default=None,
                    help="load this build of librevel_wal.so instead of the in-tree one (A/B of two builds)")
    ap.add_argument("--keep-tail", action="store_true",
                    help="end the tiled image with the writer's partial last block (as bench.py's c3 image does)")
    ap.add_argument("--image", choices=["zipf", "full"], default="zipf",
                    help="full = C2-style full blocks (1 record/block): the verify kernels' base cost")
    a = ap.parse_args()
    if a.lib:
        from revel_amd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    t0 = time.time()
    ctx = gpu.GpuContext(0)
    if a.image == "full":
        nb = a.bytes * max(1, a.tile) // BLOCK_SIZE
        n = nb * BLOCK_SIZE
        d = ctx.alloc(n)
        check(lib().revel_gpu_synth_full_blocks(ctx.handle, d.ptr, nb, 0x5EED0002, 0, None))
        ctx.sync()
    else:
        img = make_image(a.bytes)
        if a.tile > 1:  # whole blocks only, so the tiles stay block-aligned
            whole = len(img) // BLOCK_SIZE * BLOCK_SIZE
            img = img[:whole] * (a.tile - 1) + (img if a.keep_tail else img[:whole])
        n = len(img)
        d = ctx.upload(np.frombuffer(img, dtype=np.uint8))
    t_write = time.time() - t0
    res = ctx.verify_image(d, n)
    nrec = len(res)
    bad = int((res["status"] != 0).sum())
    nblocks = (n + BLOCK_SIZE - 1) // BLOCK_SIZE
    counts = ctx.alloc(4 * nblocks)
    first = ctx.alloc(4 * nblocks)
    out = ctx.alloc(nrec * 24)
    L = lib()
    e0, e1, e2 = ctx.event(), ctx.event(), ctx.event()
    variants = [int(v) for v in a.variants.split(",")]

    def run(variant):
        e0.record()
        check(L.revel_gpu_count_scan_records(ctx.handle, d.ptr, n, counts.ptr, first.ptr, None))
        e1.record()
        if variant == 0:  # production, from the product library
            check(L.revel_gpu_verify_records(ctx.handle, d.ptr, n, 0, first.ptr, out.ptr, None))
        elif variant >= 100:  # a production-library verify path (test hook), variant - 100
            check(L.revel_gpu_verify_records_path(ctx.handle, variant - 100, d.ptr, n, 0, first.ptr, out.ptr,
                                                  None))
        else:  # experiment arms (tools/experiments/libexperiments.so)
            check(experiments().revel_x_verify_records_variant(ctx.handle, variant, d.ptr, n, 0, first.ptr,
                                                               out.ptr, None))
        e2.record()
        ctx.sync()
        return e0.elapsed_ms(e2), e1.elapsed_ms(e2)

    # interleaved rounds (--rounds > 1): every variant once per round, so drift
    # (clock, temperature) spreads over all of them; medians per variant
    times = {v: ([], []) for v in variants}
    same_all = {v: True for v in variants}
    for _ in range(max(1, a.rounds)):
        for variant in variants:
            for _ in range(a.iters):
                ta, tv = run(variant)
                times[variant][0].append(ta)
                times[variant][1].append(tv)
            got = ctx.d2h(out, nrec * 24, np.uint8).view(res.dtype)
            same_all[variant] = same_all[variant] and bool(np.array_equal(got, res))
    for variant in variants:
        times_all, times_verify = times[variant]
        same = same_all[variant]
        ta, tv = float(np.median(times_all)), float(np.median(times_verify))
        print(json.dumps({
            "workload": ("C3 zipf 64B-32KiB records (1 GiB written by the host writer, whole blocks tiled"
                         + (", partial tail block kept" if a.keep_tail else "") + "), device walk + segmented CRC verify"
                         if a.image == "zipf" else "C2-layout full blocks through the C3 verify path"),
            "verify_variant": variant, "matches_production": same, "lib": a.lib or "in-tree",
            "image_bytes": n, "blocks": nblocks, "physical_records": nrec, "bad_records": bad,
            "types": {int(t): int((res["type"] == t).sum()) for t in (1, 2, 3, 4)},
            "host_write_s": round(t_write, 2),
            "ms_count_scan_verify": round(ta, 4), "ms_verify_only": round(tv, 4),
            "GiB_s_total": round(n / 2**30 / (ta / 1e3), 1), "GiB_s_verify": round(n / 2**30 / (tv / 1e3), 1),
        }), flush=True)


if __name__ == "__main__":
    main()
