"""Probe: does cutting a resident WAL image into block-aligned chunks and
pipelining the count pass of chunk c+1 against the verify of chunk c (two
contexts = two HIP streams) beat one count -> scan -> verify over the whole
image?  Uses only the public C-ABI (revel_gpu_count_scan_records /
revel_gpu_verify_records on sub-images; records never cross a block, so a
block-aligned chunk is an exact sub-problem, log_writer.rs:66-76).

For each chunking it prints the wall time per image (host clock around the
queued calls, both streams synchronised on both sides; median of --runs) and
whether the result arrays equal the whole-image call's byte for byte.

    python tools/pipeline_probe.py [--gib 4] [--shapes small,zipf] [--chunks 0,16,32,64] [--ctxs 1,2]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
BLOCK = 32768


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--shapes", default="small,zipf")
    ap.add_argument("--chunks", default="1,8,16,32,64")
    ap.add_argument("--ctxs", default="1,2,3")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--runs", type=int, default=3)
    a = ap.parse_args()
    import bench
    from revel_amd import gpu
    from revel_amd._lib import check, lib
    from revel_amd.gpu import RECORD_DTYPE
    L = lib()
    ctxs = [gpu.GpuContext(0) for _ in range(max(int(x) for x in a.ctxs.split(",")))]
    ctx = ctxs[0]
    for shape in a.shapes.split(","):
        seed = 0x5EED0003 if shape == "zipf" else 0x5EED0005
        img, n, nrec = bench.c3_image(ctx, shape, seed, a.gib)
        ctx.sync()
        nblocks = (n + BLOCK - 1) // BLOCK
        counts = ctx.alloc(4 * nblocks)
        first = ctx.alloc(4 * nblocks)
        cap = nrec + 2 * nblocks + 64
        out = ctx.alloc(cap * RECORD_DTYPE.itemsize)
        ref = None
        for nch in [int(x) for x in a.chunks.split(",")]:
            cb = (nblocks + nch - 1) // nch  # blocks per chunk
            spans = [(c * cb, min(nblocks, (c + 1) * cb)) for c in range(nch) if c * cb < nblocks]
            # per-chunk record totals (untimed) -> result offsets
            offs, tot = [], 0
            for (b0, b1) in spans:
                nb = min(n, b1 * BLOCK) - b0 * BLOCK
                check(L.revel_gpu_count_scan_records(ctx.handle, img.ptr + b0 * BLOCK, nb, counts.ptr + 4 * b0,
                                                     first.ptr + 4 * b0, None))
                ctx.sync()
                t = int(ctx.d2h(first, 4, np.uint32, src_offset=4 * (b1 - 1))[0]) + \
                    int(ctx.d2h(counts, 4, np.uint32, src_offset=4 * (b1 - 1))[0])
                offs.append(tot)
                tot += t
            assert tot <= cap

            def enqueue(k):
                for i, (b0, b1) in enumerate(spans):
                    c = ctxs[i % k]
                    nb = min(n, b1 * BLOCK) - b0 * BLOCK
                    check(L.revel_gpu_count_scan_records(c.handle, img.ptr + b0 * BLOCK, nb, counts.ptr + 4 * b0,
                                                         first.ptr + 4 * b0, None))
                    check(L.revel_gpu_verify_records(c.handle, img.ptr + b0 * BLOCK, nb, b0 * BLOCK,
                                                     first.ptr + 4 * b0, out.ptr + offs[i] * RECORD_DTYPE.itemsize,
                                                     None))

            for k in [int(x) for x in a.ctxs.split(",")]:
                if nch == 1 and k > 1:
                    continue
                for c in ctxs:
                    c.sync()
                enqueue(k)  # warm
                for c in ctxs:
                    c.sync()
                runs, enq = [], []
                for _ in range(a.runs):
                    t0 = time.perf_counter()
                    for _ in range(a.iters):
                        enqueue(k)
                    t1 = time.perf_counter()
                    for c in ctxs[:k]:
                        c.sync()
                    t2 = time.perf_counter()
                    runs.append((t2 - t0) * 1e3 / a.iters)
                    enq.append((t1 - t0) * 1e3 / a.iters)
                res = ctx.d2h(out, tot * RECORD_DTYPE.itemsize, np.uint8)
                if ref is None:
                    ref = res.copy()
                same = res.nbytes == ref.nbytes and bool(np.array_equal(res, ref))
                bad = int((res.view(RECORD_DTYPE)["status"] != 0).sum())
                print(f"{shape} chunks={len(spans)} ({cb} blocks = {cb * BLOCK / 2**20:.0f} MiB) ctxs={k}: "
                      f"ms/image median {np.median(runs):.4f} runs {[round(x, 4) for x in runs]} "
                      f"host enqueue {np.median(enq):.4f} ms  records {tot} bad {bad} same_as_whole {same}",
                      flush=True)
        for b in (counts, first, out, img):
            b.free()


if __name__ == "__main__":
    main()
