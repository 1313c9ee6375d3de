"""End-to-end replay rate (config C5): host bytes -> pinned ring -> H2D ->
GPU verify -> summary D2H, PCIe-inclusive.

  --mode full     C2 layout (every block one FULL record), synthesised on
                  device in 1 GiB chunks and copied to a host RAM image
  --mode records  C3 layout (Zipf 64 B..32 KiB records by the host writer),
                  a 1 GiB image tiled to --gib
  --source memory replay from the host RAM image (pageable -> pinned ring)
  --source file   write the image to --path once, then replay it through the
                  page cache with pread
Prints one JSON line per configuration."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from revel_amd import BLOCK_SIZE, gpu  # noqa: E402


def host_image_full(ctx, gib):
    n = int(gib * (1 << 30)) // BLOCK_SIZE
    img = np.empty(n * BLOCK_SIZE, dtype=np.uint8)
    chunk = 32768  # blocks per 1 GiB
    d = ctx.alloc(chunk * BLOCK_SIZE)
    for b0 in range(0, n, chunk):
        k = min(chunk, n - b0)
        ctx.synth_full_blocks(d, k, seed=0x5EED0005, first=b0)
        ctx.sync()
        img[b0 * BLOCK_SIZE:(b0 + k) * BLOCK_SIZE] = ctx.d2h(d, k * BLOCK_SIZE)
    return img


def host_image_records(gib):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from bench_c3 import make_image
    one = np.frombuffer(make_image(1 << 30), dtype=np.uint8)
    one = one[:len(one) // BLOCK_SIZE * BLOCK_SIZE]      # whole blocks, so tiles stay aligned
    reps = max(1, int(round(gib * (1 << 30) / len(one))))
    return np.tile(one, reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=16.0)
    ap.add_argument("--mode", choices=["full", "records"], default="full")
    ap.add_argument("--source", choices=["memory", "file"], default="memory")
    ap.add_argument("--path", default="/tmp/revel_e2e.log")
    ap.add_argument("--window-mib", type=int, default=64)
    ap.add_argument("--nbuf", type=int, default=4)
    ap.add_argument("--threads", default="4,8,16")
    ap.add_argument("--io", default="mmap", help="file input methods: mmap,pread,direct")
    a = ap.parse_args()
    ctx = gpu.GpuContext(0)
    t0 = time.time()
    img = host_image_full(ctx, a.gib) if a.mode == "full" else host_image_records(a.gib)
    t_gen = time.time() - t0
    if a.source == "file":
        with open(a.path, "wb") as f:
            f.write(memoryview(img))
        del img
    runs = [(th, io) for io in (a.io.split(",") if a.source == "file" else ["-"]) for th in
            [int(t) for t in a.threads.split(",")]]
    for th, io in runs:
        kw = dict(full_blocks=a.mode == "full", window_bytes=a.window_mib << 20, nbuffers=a.nbuf, io_threads=th)
        st = ctx.replay_memory(img, **kw) if a.source == "memory" else ctx.replay_file(a.path, io=io, **kw)
        gib = st["bytes"] / 2**30
        print(json.dumps({
            "workload": f"C5 end-to-end replay, {a.mode} layout, source={a.source}",
            "GiB": round(gib, 2), "io": io, "io_threads": th, "window_MiB": a.window_mib, "nbuffers": a.nbuf,
            "end_to_end_GiB_s": round(gib / st["seconds"], 2),
            "h2d_GiB_s": round(gib / (st["h2d_ms"] / 1e3), 2),
            "host_fill_GiB_s": round(gib / st["read_seconds"], 2),
            "kernel_GiB_s": round(gib / (st["kernel_ms"] / 1e3), 1),
            "units": st["units"], "bad": st["bad"], "image_gen_s": round(t_gen, 1),
        }), flush=True)
    if a.source == "file":
        os.unlink(a.path)


if __name__ == "__main__":
    main()
