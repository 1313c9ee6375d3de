"""End-to-end replay rate (config C5): host bytes -> pinned ring -> H2D ->
GPU verify -> summary D2H, PCIe-inclusive.

  --mode full     C2 layout (every block one FULL record), synthesised on
                  device in 1 GiB chunks and copied to a host RAM image
  --mode records  C3 layout (Zipf 64 B..32 KiB records by the host writer),
                  a 1 GiB image tiled to --gib
  --source memory replay from the host RAM image (pageable -> pinned ring)
  --source file   write the image to --path once (streamed in 1 GiB pieces,
                  never held whole in RAM), then replay it through the page
                  cache
  --loader ring   revel_gpu_replay_file: pinned ring -> HBM windows -> verify
  --loader shard  revel_gpu_wal_shard_load: the whole file resident in HBM
                  (mmap -> pinned ring -> H2D, per-window count, one verify),
                  the C5 shard path of one GPU (REVEL_SHARD_VERIFY)
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


def write_file_full(ctx, gib, path):
    """C2-layout blocks synthesised on device, written 1 GiB at a time."""
    n = int(gib * (1 << 30)) // BLOCK_SIZE
    chunk = 32768
    d = ctx.alloc(chunk * BLOCK_SIZE)
    with open(path, "wb") as f:
        for b0 in range(0, n, chunk):
            k = min(chunk, n - b0)
            ctx.synth_full_blocks(d, k, seed=0x5EED0005, first=b0)
            ctx.sync()
            f.write(memoryview(ctx.d2h(d, k * BLOCK_SIZE)))
    d.free()
    return n * BLOCK_SIZE


def write_file_records(gib, path):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from bench_c3 import make_image
    one = make_image(1 << 30)
    one = one[:len(one) // BLOCK_SIZE * BLOCK_SIZE]
    reps = max(1, int(round(gib * (1 << 30) / len(one))))
    with open(path, "wb") as f:
        for _ in range(reps):
            f.write(one)
    return reps * len(one)


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
    ap.add_argument("--loader", default="ring", help="ring,shard (file source only for shard)")
    ap.add_argument("--repeat", type=int, default=1, help="runs per configuration (the first shard load also "
                                                          "allocates the context's pinned ring)")
    a = ap.parse_args()
    ctx = gpu.GpuContext(0)
    t0 = time.time()
    img = None
    if a.source == "file":
        nbytes = write_file_full(ctx, a.gib, a.path) if a.mode == "full" else write_file_records(a.gib, a.path)
    else:
        img = host_image_full(ctx, a.gib) if a.mode == "full" else host_image_records(a.gib)
        nbytes = img.nbytes
    t_gen = time.time() - t0
    runs = [(ld, th, io) for ld in a.loader.split(",")
            for io in (a.io.split(",") if a.source == "file" and ld == "ring" else ["-"])
            for th in [int(t) for t in a.threads.split(",")] for _ in range(a.repeat)]
    for ld, th, io in runs:
        if ld == "shard":
            from revel_amd import shard
            sh = shard.WalShard(ctx, 0, nbytes, path=a.path if a.source == "file" else None, image=img,
                                checksum=True, read=False, window_bytes=a.window_mib << 20, io_threads=th)
            inf = sh.info()
            sh.close()
            gib = nbytes / 2**30
            print(json.dumps({
                "workload": f"C5 end-to-end, {a.mode} layout, source={a.source}, loader=shard (whole file in HBM)",
                "GiB": round(gib, 2), "io": "mmap" if a.source == "file" else "memory", "io_threads": th,
                "window_MiB": a.window_mib, "nbuffers": 3,
                "end_to_end_GiB_s": round(gib / inf["seconds"], 2),
                "all_in_GiB_s": round(gib / (inf["seconds"] + inf["setup_seconds"]), 2),
                "setup_s": round(inf["setup_seconds"], 3),
                "h2d_GiB_s": round(gib / (inf["h2d_ms"] / 1e3), 2) if inf["h2d_ms"] else None,
                "host_fill_GiB_s": round(gib / inf["read_seconds"], 2) if inf["read_seconds"] else None,
                "kernel_GiB_s": round(gib / (inf["kernel_ms"] / 1e3), 1) if inf["kernel_ms"] else None,
                "units": inf["physical"], "bad": inf["bad"], "image_gen_s": round(t_gen, 1),
            }), flush=True)
            continue
        kw = dict(full_blocks=a.mode == "full", window_bytes=a.window_mib << 20, nbuffers=a.nbuf, io_threads=th)
        st = ctx.replay_memory(img, **kw) if a.source == "memory" else ctx.replay_file(a.path, io=io, **kw)
        gib = st["bytes"] / 2**30
        print(json.dumps({
            "workload": f"C5 end-to-end replay, {a.mode} layout, source={a.source}, loader=ring",
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
