"""WAL replay through WriteBatch decode on device, db_bench-shaped logs.

Workloads (synthetic, deterministic):
  fill1    -- one Put per batch, 16-B key, 100-B value (db_bench fillrandom,
              write_batch_size 1): 131-B logical records.
  fill100  -- 100 Puts per batch, same key/value shape: 11,912-B records.
The image is framed on the GPU by revel_gpu_append_records (bit-exact with
log::Writer, tests/test_gpu.py) from payloads built with numpy, then timed in
HBM: count+scan+verify -> reassemble -> decode, each bracketed by HIP events.
Prints one JSON line per workload.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from revel_amd import gpu  # noqa: E402
from revel_amd._lib import check, lib  # noqa: E402
from revel_amd.gpu import BATCH_ENTRY_DTYPE, BATCH_INFO_DTYPE, LOGICAL_DTYPE, RECORD_DTYPE  # noqa: E402


def make_reps(nbatches: int, per_batch: int, klen: int = 16, vlen: int = 100, seed: int = 7):
    rng = np.random.default_rng(seed)
    ent = 1 + 1 + klen + 1 + vlen
    size = 12 + per_batch * ent
    reps = np.zeros((nbatches, size), np.uint8)
    seq = 1 + per_batch * np.arange(nbatches, dtype=np.uint64)
    reps[:, 0:8] = seq.view(np.uint8).reshape(nbatches, 8)
    reps[:, 8:12] = np.full(nbatches, per_batch, np.uint32).view(np.uint8).reshape(nbatches, 4)
    body = reps[:, 12:].reshape(nbatches, per_batch, ent)
    body[:, :, 0] = 1
    body[:, :, 1] = klen
    body[:, :, 2:2 + klen] = rng.integers(0, 256, (nbatches, per_batch, klen), dtype=np.uint8)
    body[:, :, 2 + klen] = vlen
    body[:, :, 3 + klen:] = rng.integers(0, 256, (1, per_batch, vlen), dtype=np.uint8)  # value bytes shared
    return reps


def run(ctx, name, per_batch, target, iters):
    L = lib()
    size = 12 + per_batch * 119
    nb = max(1, target // (size + 7))
    reps = make_reps(nb, per_batch)
    dpay = ctx.upload(reps.reshape(-1))
    img, n, _ = ctx.append_records(dpay, np.full(nb, size, np.uint64))
    dpay.free()
    nblocks = (n + 32767) // 32768
    counts, first = ctx.alloc(4 * nblocks), ctx.alloc(4 * nblocks)
    # physical record count: run once
    check(L.revel_gpu_count_scan_records(ctx.handle, img.ptr, n, counts.ptr, first.ptr, None))
    ctx.sync()
    nphys = int(ctx.d2h(first, 4 * nblocks, np.uint32)[-1]) + int(ctx.d2h(counts, 4 * nblocks, np.uint32)[-1])
    phys = ctx.alloc(nphys * RECORD_DTYPE.itemsize)
    logical = ctx.alloc(nphys * LOGICAL_DTYPE.itemsize)
    payload = ctx.alloc(n)
    info = ctx.alloc(nphys * BATCH_INFO_DTYPE.itemsize)
    cap = n // 2
    ents = ctx.alloc(cap * BATCH_ENTRY_DTYPE.itemsize)
    ev = [ctx.event() for _ in range(4)]
    nl, pb, ne = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    t = {"verify": [], "reassemble": [], "decode": [], "total": []}
    for _ in range(iters):
        ev[0].record()
        check(L.revel_gpu_count_scan_records(ctx.handle, img.ptr, n, counts.ptr, first.ptr, None))
        check(L.revel_gpu_verify_records(ctx.handle, img.ptr, n, 0, first.ptr, phys.ptr, None))
        ev[1].record()
        check(L.revel_gpu_reassemble(ctx.handle, img.ptr, 0, n, phys.ptr, nphys, 1, logical.ptr, payload.ptr,
                                     ctypes.byref(nl), ctypes.byref(pb), None))
        ev[2].record()
        check(L.revel_gpu_decode_batches(ctx.handle, payload.ptr, pb.value, logical.ptr, nl.value, info.ptr,
                                         ents.ptr, cap, ctypes.byref(ne), None))
        ev[3].record()
        ctx.sync()
        t["verify"].append(ev[0].elapsed_ms(ev[1]))
        t["reassemble"].append(ev[1].elapsed_ms(ev[2]))
        t["decode"].append(ev[2].elapsed_ms(ev[3]))
        t["total"].append(ev[0].elapsed_ms(ev[3]))
    infos = ctx.d2h(info, nl.value * BATCH_INFO_DTYPE.itemsize).view(BATCH_INFO_DTYPE)
    e = ctx.d2h(ents, ne.value * BATCH_ENTRY_DTYPE.itemsize).view(BATCH_ENTRY_DTYPE)
    ok = bool((infos["status"] == 0).all() and nl.value == nb and ne.value == nb * per_batch
              and (e["sequence"] == np.arange(1, ne.value + 1, dtype=np.uint64)).all())
    med = {k: float(np.median(v)) for k, v in t.items()}
    return {
        "workload": name, "image_bytes": n, "batches": nb, "entries": int(ne.value), "physical_records": nphys,
        "all_ok_and_sequences_dense": ok,
        "ms": {k: round(v, 4) for k, v in med.items()},
        "GiB_s": {k: round(n / 2**30 / (v / 1e3), 1) for k, v in med.items()},
        "M_entries_s_total": round(ne.value / (med["total"] / 1e3) / 1e6, 1),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--lib", default=None, help="another build of librevel_wal.so (A/B)")
    a = ap.parse_args()
    if a.lib:
        from revel_amd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    ctx = gpu.GpuContext(0)
    for name, per in [("fill1", 1), ("fill100", 100)]:
        print(json.dumps(run(ctx, name, per, a.bytes, a.iters)), flush=True)


if __name__ == "__main__":
    main()
