"""Phase breakdown of k_walk_verify (round 5): a build with
-DREVEL_FUSED_PHASES sums each wave's shader-clock cycles per phase (loads
landed, walk, chains + captures, scan, records) over the last count pass;
this runs bench.py's image through the production count + verify and prints
the per-block averages.

    tools/build_variant.sh phases -DREVEL_FUSED_PHASES
    python tools/fused_phases.py --lib build/ab/phases.so [--shape small]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--shape", default="small")
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--kernel", choices=["fused", "fused2", "chunks"], default="fused",
                    help="fused: k_walk_verify (REVEL_FUSED=1); chunks: k_verify_dense_chunks (REVEL_DENSE_CHUNKS=1)")
    a = ap.parse_args()
    from revel_amd import _lib
    _lib.LIB_PATH = os.path.abspath(a.lib)
    import bench
    from revel_amd import gpu
    ctx = gpu.GpuContext(0)
    img, n, nrec = bench.c3_image(ctx, a.shape, 0x5EED0003 if a.shape == "zipf" else 0x5EED0005, a.gib)
    L = _lib.lib()
    f = L.revel_debug_fused_phases
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
    L.revel_debug_set_fused({"fused": 1, "fused2": 2}.get(a.kernel, 0))  # a one-pass path (opt-in)
    L.revel_debug_set_dense_chunks.restype, L.revel_debug_set_dense_chunks.argtypes = ctypes.c_int, [ctypes.c_int]
    L.revel_debug_set_dense_chunks(1 if a.kernel == "chunks" else -1)  # opt-in
    bench.c3_verify_timed(ctx, img, n, nrec, 1)  # warm
    assert f(None, 1) == 0
    t, nphys, bad = bench.c3_verify_timed(ctx, img, n, nrec, 1)
    buf = np.zeros(16, np.uint64)
    assert f(buf.ctypes.data, 0) == 0
    names = {0: "loads", 1: "walk_rest", 2: "chains", 3: "scan", 4: "records", 8: "detect", 9: "compact",
             10: "successors", 11: "doubling", 12: "chain_end", 13: "scalar_walk"}
    if a.kernel == "chunks":
        names = {0: "entries_issued", 1: "points_lookup", 2: "chains", 3: "scan", 4: "records"}
    if a.kernel == "fused2":
        names = {0: "stream", 1: "walk", 3: "scan", 4: "records"}
    blocks, recs, waves = int(buf[5]), int(buf[6]), int(buf[7])
    total = int(sum(int(buf[i]) for i in names))
    out = {"kernel": a.kernel, "shape": a.shape, "ms": round(t[0], 4), "blocks": blocks, "records": recs, "waves": waves,
           "cycles_per_block": {k: round(int(buf[i]) / max(1, blocks), 1) for i, k in names.items()},
           "share": {k: round(int(buf[i]) / max(1, total), 3) for i, k in names.items()},
           "wave_cycles_total_per_wave": round(total / max(1, waves)),
           "scalar_walks": {"continued": int(buf[14]), "from_start": int(buf[15]) & 0xFFFFFFFF,
                            "overflow": int(buf[15]) >> 32} if a.kernel == "fused" else
                           ({"scalar": int(buf[14]), "left_to_dense2": int(buf[15])} if a.kernel == "fused2" else None),
           "walk_cycles_per_record": round(sum(int(buf[i]) for i in (1, 8, 9, 10, 11, 12, 13)) / max(1, recs), 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
