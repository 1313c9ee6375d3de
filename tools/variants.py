"""On-box experiment: C2 kernel variants vs the streaming-read ceiling.

For each variant: bit-exact check against variant 0 over all blocks (and
variant 0 against the oracle on a sample), then interleaved timing rounds
with HIP events on the context stream.  Prints one JSON line per variant.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from revel_amd import BLOCK_SIZE, gpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--variants", default="100,0,1,2,3,4,5,6,7")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--lib", default=None, help="load this build of librevel_wal.so (A/B of two builds)")
    args = ap.parse_args()
    if args.lib:
        from revel_amd import _lib
        _lib.LIB_PATH = os.path.abspath(args.lib)
    n = args.blocks
    variants = [int(v) for v in args.variants.split(",")]
    ctx = gpu.GpuContext(0)
    d = ctx.alloc(n * BLOCK_SIZE)
    t0 = time.time()
    ctx.synth_full_blocks(d, n, seed=0x5EED0002)
    ctx.sync()
    print(f"# synth {n} blocks in {time.time() - t0:.2f}s", flush=True)
    outs = {v: ctx.alloc(4 * n) for v in variants}
    ok = ctx.alloc(n)
    ctx.crc_full_blocks(d, n, outs[variants[-1] if 0 not in variants else 0], ok, variant=0)
    ctx.sync()
    ref = ctx.d2h(outs[0] if 0 in variants else outs[variants[-1]], 4 * n, np.uint32)
    okh = ctx.d2h(ok, n)
    sys.path.insert(0, ROOT)
    from oracle import oracle_c
    idx = np.arange(0, n, max(1, n // 128))
    sample = np.stack([ctx.d2h(d, BLOCK_SIZE, src_offset=int(i) * BLOCK_SIZE) for i in idx])
    oracle_ok = bool(np.array_equal(ref[idx], oracle_c.full_block_crcs(sample)))
    print(f"# variant0 vs oracle sample({len(idx)}): {oracle_ok}; ok flags all set: {bool(okh.all())}", flush=True)
    parity = {}
    for v in variants:
        ctx.crc_full_blocks(d, n, outs[v], None, variant=v)
        ctx.sync()
        got = ctx.d2h(outs[v], 4 * n, np.uint32)
        parity[v] = True if v == 100 else bool(np.array_equal(got, ref))
    times = {v: [] for v in variants}
    e0, e1 = ctx.event(), ctx.event()
    for r in range(args.rounds):
        for v in variants:
            ctx.crc_full_blocks(d, n, outs[v], None, variant=v)  # warm
            e0.record()
            for _ in range(args.iters):
                ctx.crc_full_blocks(d, n, outs[v], None, variant=v)
            e1.record()
            times[v].append(e0.elapsed_ms(e1) / args.iters)
    for v in variants:
        t = np.array(times[v])
        gib = n * BLOCK_SIZE / 2**30 / (np.median(t) / 1e3)
        gbs = n * (BLOCK_SIZE + 4) / 1e9 / (np.median(t) / 1e3)
        print(json.dumps({"variant": v, "parity": parity[v], "ms_median": float(np.median(t)),
                          "ms_min": float(t.min()), "GiB_s": round(gib, 1), "GB_s": round(gbs, 1),
                          "frac_8TBs": round(gbs / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
