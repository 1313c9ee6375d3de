"""Go / no-go probe for VERDICT r5 #1 (tools/experiments/x_stage_probe.hip):
the small-record verify as one coalesced read per block staged in LDS --
load, header walk and lane-per-record checksums all from the wave's 32 KiB
slot.  On bench.py's c3_small image (uniform 64..256-B records, 4 GiB,
framed on device) it times the probe kernel per mode (HIP events, median of
5), reads its per-phase shader cycles per block, and checks it: the counts
equal the production count pass's, and every record's computed CRC equals
its stored one (a fresh image has no bad record).  The production pipeline
(count_scan + verify) is timed on the same image for reference.

    make -C tools/experiments xst && python tools/stage_probe.py [--gib 4]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from revel_amd import gpu  # noqa: E402
from revel_amd._lib import check, lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--hybrid", action="store_true",
                    help="the production count pass over the first blocks beside k_scount over the rest, "
                         "on two streams at once")
    ap.add_argument("--scount", action="store_true",
                    help="time the scalar-load count pass probe (k_scount) on the small and Zipf images instead")
    a = ap.parse_args()
    if a.scount:
        return scount(a)
    if a.hybrid:
        return hybrid(a)
    X = ctypes.CDLL(os.path.join(ROOT, "tools", "experiments", "libxst.so"))
    X.xst_init.argtypes = [ctypes.c_void_p]
    X.xst_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    ctx = gpu.GpuContext(0)
    st = ctx.stream
    img, n, nrec = bench.c3_image(ctx, "small", 0x5EED0005, a.gib)
    nblocks = n // bench.BLOCK_SIZE  # whole blocks only (the probe has no partial-block path)
    print(f"image {n} B, {nblocks} whole blocks, {nrec} logical records", flush=True)
    # production reference: counts and time
    L = lib()
    counts_ref, first = ctx.alloc(4 * (nblocks + 1)), ctx.alloc(4 * (nblocks + 1))
    out = ctx.alloc((nrec + 2 * nblocks + 64) * 24)
    nb_all = (n + 32767) // 32768
    e0, e1 = ctx.event(), ctx.event()
    prod = []
    for _ in range(a.reps):
        e0.record()
        check(L.revel_gpu_count_scan_records(ctx.handle, img.ptr, n, counts_ref.ptr, first.ptr, None))
        check(L.revel_gpu_verify_records(ctx.handle, img.ptr, n, 0, first.ptr, out.ptr, None))
        e1.record()
        ctx.sync()
        prod.append(e0.elapsed_ms(e1))
    cref = ctx.d2h(counts_ref, 4 * nb_all, np.uint32)[:nblocks]
    print(f"production count_scan + verify: {np.median(prod):.4f} ms (median of {a.reps})", flush=True)
    out.free()
    counts = ctx.alloc(4 * nblocks)
    crcs = ctx.alloc(4 * 256 * nblocks)
    stats = ctx.alloc(8 * 8)
    check(X.xst_init(ctypes.c_void_p(st)))
    ctx.sync()
    ncu = 256
    results = {"image_bytes": n, "blocks": nblocks, "production_ms": float(np.median(prod))}
    for mode, ch in ((0, 1), (1, 1), (3, 1), (3, 2)):
        times = []
        for r in range(a.reps):
            ctx.memset(stats, 0, 64)
            e0.record()
            if X.xst_launch(mode, ch, ctypes.c_void_p(img.ptr), nblocks, ctypes.c_void_p(counts.ptr),
                            ctypes.c_void_p(crcs.ptr), ctypes.c_void_p(stats.ptr), ncu, ctypes.c_void_p(st)):
                raise SystemExit("launch failed")
            e1.record()
            ctx.sync()
            times.append(e0.elapsed_ms(e1))
        s = ctx.d2h(stats, 64, np.uint64)
        blk = max(1, int(s[3]))
        row = {"mode": mode, "ch": ch, "ms": round(float(np.median(times)), 4),
               "cycles_per_block": {"load": round(s[0] / blk), "walk": round(s[1] / blk), "crc": round(s[2] / blk)},
               "blocks": int(s[3]), "records": int(s[5]), "crc_mismatch": int(s[4])}
        if mode & 1:
            cnt = ctx.d2h(counts, 4 * nblocks, np.uint32)
            row["counts_equal_production"] = bool(np.array_equal(cnt, cref))
            row["records_expected"] = int(np.minimum(cref, 256).sum())
        print(json.dumps(row), flush=True)
        results[f"mode{mode}_ch{ch}"] = row
    print("RESULT " + json.dumps(results), flush=True)


def scount(a):
    """k_scount: the header walk on the scalar unit, C chains per wave, vs the
    production count pass (k_count_hist) on the same images: counts must be
    equal, times by HIP events (median of reps)."""
    X = ctypes.CDLL(os.path.join(ROOT, "tools", "experiments", "libxst.so"))
    X.xst_scount.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                             ctypes.c_void_p]
    ctx = gpu.GpuContext(0)
    st = ctx.stream
    L = lib()
    e0, e1 = ctx.event(), ctx.event()
    res = {}
    for shape, seed in (("small", 0x5EED0005), ("zipf", 0x5EED0003)):
        img, n, nrec = bench.c3_image(ctx, shape, seed, a.gib)
        nb = (n + 32767) // 32768
        cref, first, cnt = ctx.alloc(4 * nb), ctx.alloc(4 * nb), ctx.alloc(4 * nb)
        prod = []
        for _ in range(a.reps):
            e0.record()
            check(L.revel_gpu_count_records(ctx.handle, img.ptr, n, cref.ptr, None))
            e1.record()
            ctx.sync()
            prod.append(e0.elapsed_ms(e1))
        want = ctx.d2h(cref, 4 * nb, np.uint32)
        row = {"shape": shape, "blocks": nb, "production_count_ms": round(float(np.median(prod)), 4)}
        for c in (4, 8, 16):
            for wgs in (8, 16):
                ts = []
                for _ in range(a.reps):
                    ctx.memset(cnt, 0xFF, 4 * nb)
                    e0.record()
                    if X.xst_scount(c, ctypes.c_void_p(img.ptr), n, ctypes.c_void_p(cnt.ptr), 256 * wgs,
                                    ctypes.c_void_p(st)):
                        raise SystemExit("launch failed")
                    e1.record()
                    ctx.sync()
                    ts.append(e0.elapsed_ms(e1))
                got = ctx.d2h(cnt, 4 * nb, np.uint32)
                row[f"c{c}_wg{wgs}"] = {"ms": round(float(np.median(ts)), 4), "counts_equal": bool(np.array_equal(got, want))}
        print(json.dumps(row), flush=True)
        res[shape] = row
        for b in (img, cref, first, cnt):
            b.free()
    print("RESULT " + json.dumps(res), flush=True)


def hybrid(a):
    """Do the vector and scalar memory paths add up?  The production count
    pass (vector lanes, revel_gpu_count_records) over blocks [0, nV) on one
    context's stream and k_scount (scalar unit) over [nV, N) on a second
    context's stream, launched together; host wall time around both (median
    of reps), against each alone; the two count arrays together must equal
    the production pass over the whole image."""
    import time
    X = ctypes.CDLL(os.path.join(ROOT, "tools", "experiments", "libxst.so"))
    X.xst_scount.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                             ctypes.c_void_p]
    A, B = gpu.GpuContext(0), gpu.GpuContext(0)
    L = lib()
    res = {}
    for shape, seed in (("small", 0x5EED0005), ("zipf", 0x5EED0003)):
        img, n, nrec = bench.c3_image(A, shape, seed, a.gib)
        nb = (n + 32767) // 32768
        cref, cnt = A.alloc(4 * nb), A.alloc(4 * nb)
        check(L.revel_gpu_count_records(A.handle, img.ptr, n, cref.ptr, None))
        A.sync()
        want = A.d2h(cref, 4 * nb, np.uint32)
        row = {"shape": shape, "blocks": nb}

        def run(nv, vec, sca, c=8, wgs=8):
            A.sync()
            B.sync()
            t0 = time.perf_counter()
            if vec and nv:
                check(L.revel_gpu_count_records(A.handle, img.ptr, min(nv * 32768, n), cnt.ptr, None))
            if sca and nv < nb:
                if X.xst_scount(c, ctypes.c_void_p(img.ptr + nv * 32768), n - nv * 32768,
                                ctypes.c_void_p(cnt.ptr + 4 * nv), 256 * wgs, ctypes.c_void_p(B.stream)):
                    raise SystemExit("launch failed")
            A.sync()
            B.sync()
            return (time.perf_counter() - t0) * 1e3

        for f in (0.0, 0.2, 0.3, 0.4):
            nv = nb - int(f * nb)
            both = [run(nv, True, True) for _ in range(a.reps + 2)][2:]
            got = A.d2h(cnt, 4 * nb, np.uint32)
            vec = [run(nv, True, False) for _ in range(a.reps)]
            sca = [run(nv, False, True) for _ in range(a.reps)] if f else [0.0]
            row[f"f{f}"] = {"both_ms": round(float(np.median(both)), 4), "vector_alone_ms": round(float(np.median(vec)), 4),
                            "scalar_alone_ms": round(float(np.median(sca)), 4),
                            "counts_equal": bool(np.array_equal(got, want))}
        print(json.dumps(row), flush=True)
        res[shape] = row
        for b in (img, cref, cnt):
            b.free()
    print("RESULT " + json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
