"""Probe of the one-lane-per-block small-record verify (tools/experiments/x_lanewalk.hip,
libxlw.so): timing of its variants on bench.py's 4 GiB images, and its header-list entries,
counts and raw CRCs checked against the production pipeline's results on the same image
(clean, then with byte flips).

    python tools/lanewalk_probe.py [--gib 4] [--iters 10] [--shapes small,zipf] [--flips 300]
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
BLOCK = 32768
STRIDE = 257
CAP = 256


def unmask(m):
    m = np.asarray(m, dtype=np.uint64)
    rot = (m - np.uint64(0xA282EAD8)) & np.uint64(0xFFFFFFFF)
    return (((rot >> np.uint64(17)) | (rot << np.uint64(15))) & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", default="small,zipf")
    ap.add_argument("--flips", type=int, default=300)
    ap.add_argument("--variants", default="0:0,0:2,2:0,3:0,3:2")
    ap.add_argument("--check-var", type=int, default=3)
    ap.add_argument("--no-check", action="store_true")
    a = ap.parse_args()
    import bench
    from revel_amd import gpu
    from revel_amd._lib import check, lib
    from revel_amd.gpu import RECORD_DTYPE
    L = lib()
    X = ctypes.CDLL(os.path.join(ROOT, "tools", "experiments", "libxlw.so"))
    X.xlw_launch.restype = ctypes.c_int
    X.xlw_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    X.xlw_sink_words.restype = ctypes.c_uint64
    X.xlw_sink_words.argtypes = [ctypes.c_uint64]
    X.xlw_expand8.restype = ctypes.c_int
    X.xlw_expand8.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_void_p]
    X.xlw_init_xor.restype = ctypes.c_int
    X.xlw_init_xor.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    ctx = gpu.GpuContext(0)
    ixb = ctx.alloc(4 * (BLOCK + 2))
    assert X.xlw_init_xor(ixb.ptr, ctx.stream) == 0
    ctx.sync()
    ixor = ctx.d2h(ixb, 4 * (BLOCK + 2), np.uint32)
    ixb.free()

    for shape in a.shapes.split(","):
        seed = 0x5EED0003 if shape == "zipf" else 0x5EED0005
        img, n, nrec = bench.c3_image(ctx, shape, seed, a.gib)
        nb = n // BLOCK
        nbytes = nb * BLOCK
        counts_r, first_r = ctx.alloc(4 * nb), ctx.alloc(4 * nb)
        out = ctx.alloc((nrec + 2 * nb + 64) * RECORD_DTYPE.itemsize)
        counts, hl, hc = ctx.alloc(4 * nb), ctx.alloc(16 * STRIDE * nb), ctx.alloc(4 * STRIDE * nb)
        sink = ctx.alloc(4 * int(X.xlw_sink_words(nb)))
        e0, e1 = ctx.event(), ctx.event()

        def reference():
            check(L.revel_gpu_count_scan_records(ctx.handle, img.ptr, nbytes, counts_r.ptr, first_r.ptr, None))
            check(L.revel_gpu_verify_records(ctx.handle, img.ptr, nbytes, 0, first_r.ptr, out.ptr, None))

        def launch(var, mp):
            assert X.xlw_launch(var, mp, img.ptr, nb, counts.ptr, hl.ptr, hc.ptr, sink.ptr, ctx.stream) == 0

        def timed(fn, iters):
            fn()
            fn()
            ctx.sync()
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            ctx.sync()
            return e0.elapsed_ms(e1) / iters

        def compare(tag):
            reference()
            launch(a.check_var, 0)
            ctx.sync()
            cr = ctx.d2h(counts_r, 4 * nb, np.uint32)
            fr = ctx.d2h(first_r, 4 * nb, np.uint32)
            c = ctx.d2h(counts, 4 * nb, np.uint32)
            nphys = int(fr[-1]) + int(cr[-1])
            res = ctx.d2h(out, nphys * RECORD_DTYPE.itemsize).view(RECORD_DTYPE)
            if a.check_var in (8, 9, 12):  # captures: the expander computes the checksums
                oc = ctx.alloc(4 * (nphys + 64))
                assert X.xlw_expand8(hl.ptr, counts.ptr, first_r.ptr, oc.ptr, nb, ctx.stream) == 0
                ctx.sync()
                crc8 = ctx.d2h(oc, 4 * nphys, np.uint32)
                oc.free()
                E4 = ctx.d2h(hl, 16 * STRIDE * nb, np.uint32).reshape(nb, STRIDE, 4)
                H = E4[:, :, 0].astype(np.uint64) | ((E4[:, :, 1] & np.uint32(0xFFFFFF)).astype(np.uint64) << np.uint64(32))
                Hc = None
                Ho = (E4[:, :, 1] >> np.uint32(24)) | ((E4[:, :, 3] >> np.uint32(24)) << np.uint32(8))
            elif a.check_var == 7:  # 16-B entries {stored, len | type << 16, raw, offset}
                E4 = ctx.d2h(hl, 16 * STRIDE * nb, np.uint32).reshape(nb, STRIDE, 4)
                H = E4[:, :, 0].astype(np.uint64) | (E4[:, :, 1].astype(np.uint64) << np.uint64(32))
                Hc = E4[:, :, 2]
                Ho = E4[:, :, 3]
            else:
                H = ctx.d2h(hl, 8 * STRIDE * nb, np.uint64).reshape(nb, STRIDE)
                Hc = ctx.d2h(hc, 4 * STRIDE * nb, np.uint32).reshape(nb, STRIDE)
                Ho = None
            ok_counts = bool((c == cr).all())
            m = np.minimum(c, CAP).astype(np.int64)
            bidx = np.repeat(np.arange(nb), m)
            tidx = np.arange(int(m.sum())) - np.repeat(np.cumsum(m) - m, m)
            ent = H[bidx, tidx]
            r = res[fr[bidx].astype(np.int64) + tidx]
            stored = (ent & np.uint64(0xFFFFFFFF)).astype(np.uint32)
            ln = ((ent >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.uint32)
            ty = ((ent >> np.uint64(48)) & np.uint64(0xFF)).astype(np.uint8)
            ok_hdr = bool((stored == r["stored_crc"]).all() and (ln == r["length"]).all() and (ty == r["type"]).all())
            if Ho is not None:  # the in-block offsets too
                ok_hdr = ok_hdr and bool((bidx.astype(np.uint64) * np.uint64(BLOCK) + Ho[bidx, tidx] ==
                                          r["file_offset"]).all())
            crc_rec = r["status"] <= 1  # OK / BAD_CHECKSUM: a checksum was computed
            mism = int((r["status"] == 1).sum())
            if Hc is None:  # VAR 8: final checksums from the expander
                got = crc8[fr[bidx].astype(np.int64) + tidx]
                ok_raw = bool((got[crc_rec] == r["computed_crc"][crc_rec]).all())
                mism_x = int((got[crc_rec] != r["stored_crc"][crc_rec]).sum())
            else:
                raw = Hc[bidx, tidx]
                exp_raw = unmask(r["computed_crc"][crc_rec]) ^ ixor[r["length"][crc_rec] + 1]
                ok_raw = bool((raw[crc_rec] == exp_raw).all())
                mism_x = int((raw[crc_rec] != (unmask(r["stored_crc"][crc_rec]) ^ ixor[r["length"][crc_rec] + 1])).sum())
            rec = {"shape": shape, "check": tag, "var": a.check_var, "blocks": nb, "records": nphys, "listed": int(m.sum()),
                   "blocks_over_cap": int((c > CAP).sum()), "counts_equal": ok_counts, "headers_equal": ok_hdr,
                   "raw_crc_equal": ok_raw, "mismatches_ref": mism, "mismatches_lanewalk": mism_x,
                   "status_records": int((~crc_rec).sum())}
            print(json.dumps(rec), flush=True)
            return ok_counts and ok_hdr and ok_raw and mism == mism_x

        good = True if a.no_check else compare("clean")
        ms_ref = timed(reference, a.iters)
        print(json.dumps({"shape": shape, "pipeline": "production count+scan+verify", "bytes": nbytes,
                          "ms": round(ms_ref, 4)}), flush=True)
        for v in a.variants.split(","):
            var, mp = (int(x) for x in v.split(":"))
            ms = timed(lambda: launch(var, mp), a.iters)
            print(json.dumps({"shape": shape, "var": var, "map": mp, "bytes": nbytes, "ms": round(ms, 4),
                              "GB_s": round(nbytes / ms / 1e6, 1)}), flush=True)
        if a.flips and not a.no_check:
            rng = np.random.default_rng(7)
            for off in rng.integers(0, nbytes, a.flips):
                byte = ctx.d2h(img, 1, src_offset=int(off))
                ctx.h2d(img, byte ^ np.uint8(0x5A), dst_offset=int(off))
            good = compare("flipped") and good
        print(json.dumps({"shape": shape, "all_checks_pass": good}), flush=True)
        for bf in (img, counts_r, first_r, out, counts, hl, hc, sink):
            bf.free()


if __name__ == "__main__":
    main()
