"""bench.py's C2 leg alone (1 M device-synthesised full blocks, K launches
between one pair of HIP events) on any build of librevel_wal.so, for A/B runs
of builds in alternating processes; checks the verify flags and the masked
CRCs of a sample of blocks against the first launch's.

    python tools/bench_c2dev.py [--lib A.so] [--blocks 1048576] [--steps 20] [--warmup 3]
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
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    if a.lib:
        from revel_amd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    import bench
    from revel_amd import BLOCK_SIZE, gpu
    ctx = gpu.GpuContext(0)
    n = a.blocks
    dblocks, masked, ok = ctx.alloc(n * BLOCK_SIZE), ctx.alloc(4 * n), ctx.alloc(n)
    ctx.synth_full_blocks(dblocks, n, seed=bench.SEED)
    ctx.sync()
    for _ in range(a.warmup):
        ctx.crc_full_blocks(dblocks, n, masked, ok)
    ctx.sync()
    all_ok = bool(ctx.d2h(ok, n).all())
    m0 = ctx.d2h(masked, 4 * n, np.uint32)
    e0, e1 = ctx.event(), ctx.event()
    e0.record()
    for _ in range(a.steps):
        ctx.crc_full_blocks(dblocks, n, masked, ok)
    e1.record()
    ctx.sync()
    ms = e0.elapsed_ms(e1) / a.steps
    same = bool(np.array_equal(ctx.d2h(masked, 4 * n, np.uint32), m0))
    print(json.dumps({"lib": a.lib or "in-tree", "blocks": n, "ms": round(ms, 4),
                      "GiB_s": round(n * BLOCK_SIZE / 2**30 / (ms / 1e3), 1),
                      "frac": round(n * (BLOCK_SIZE + 5) / (ms / 1e3) / 8e12, 4),
                      "all_ok": all_ok, "stable": same}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
