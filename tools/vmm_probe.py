"""Diagnosis of the two round-3 guard-test wrong results (VERDICT r3 #2,
ADVICE r3): device memory mapped with the HIP virtual-memory API
(hipMemAddressReserve + hipMemCreate + hipMemMap, tests/test_gpu_guard.py's
GuardedImage) released while the next image is mapped.

Per iteration: image A is mapped, written by a kernel (synth + frame: pattern
X), read back; A is released according to the mode; image B (same size) is
mapped and its VA logged (reused = A's VA); then three views of B are checked:
  copy   -- host pattern Y copied in (hipMemcpyAsync H2D), read straight back
            (hipMemcpyAsync D2H): does the copy path see Y?
  kread  -- the C2 kernel's CRCs of B (a shader READ): Y's CRCs?  (the CRCs of
            an all-zero block or of X name what it read instead)
  kwrite -- a kernel writes pattern Z into B, D2H reads it back: Z?
Modes:
  nosync -- A unmapped / released / VA freed right after its last synchronous
            D2H (the round-3 test's GuardedImage.free before 8956d8f)
  sync   -- hipDeviceSynchronize() first, then the same
  keepva -- A unmapped + released, its VA range never freed (B gets a new VA)
  keepphys -- A unmapped, its VA freed (B may reuse it), its physical handle
            kept until the end (A's pages are neither freed nor wiped)
  plain  -- B is hipMalloc memory (control)
Reading the views: a stale GPU translation of a reused VA makes kernels see
A's pages (kread saw "X", or "zeros" once A's pages were wiped on release)
while the copies see B's; a stale runtime-side VA -> allocation lookup makes
the COPIES go to A's allocation while kernels see B's pages.

    python tools/vmm_probe.py [--iters 20] [--modes nosync,sync,keepva,plain]

Prints one JSON line per mode: iterations, VA reuses, mismatches per view and
what each mismatching read equalled.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--modes", default="nosync,sync,keepva,keepphys,plain")
    ap.add_argument("--blocks", type=int, default=2)
    a = ap.parse_args()
    from revel_amd import BLOCK_SIZE, gpu
    from oracle import oracle_c as oc
    from test_gpu_guard import GuardedImage, _guarded_nbytes
    hip = ctypes.CDLL("libamdhip64.so")
    ctx = gpu.GpuContext(0)
    nbytes = _guarded_nbytes(a.blocks)
    n = nbytes // BLOCK_SIZE
    zero_crc = oc.full_block_crcs(np.zeros((1, BLOCK_SIZE), np.uint8))[0]
    m, ok = ctx.alloc(4 * n), ctx.alloc(n)

    def crcs(buf):
        ctx.crc_full_blocks(buf, n, m, ok)
        ctx.sync()
        return ctx.d2h(m, 4 * n, np.uint32)

    for mode in a.modes.split(","):
        stats = {"mode": mode, "nbytes": nbytes, "iters": a.iters, "va_reused": 0, "a_mismatch": 0,
                 "copy_mismatch": 0, "kread_mismatch": 0, "kwrite_mismatch": 0, "kread_saw": [], "copy_saw": [],
                 "kwrite_saw": [], "events": []}
        kept, kept_phys = [], []
        prev = None  # (Z, Y, VA) of the previous iteration's image B
        for i in range(a.iters):
            sx, sz = 0x1000 + i, 0x9000 + i
            X = oc.synth_full_blocks(n, seed=sx).reshape(-1)
            A = GuardedImage(0, nbytes)
            ctx.synth_full_blocks(A, n, seed=sx)
            ctx.sync()
            got_a = ctx.d2h(A, nbytes)
            va_a = A.va
            if not np.array_equal(got_a, X):
                # which view is wrong: the kernel's (its CRCs of A) or the copy's
                ka = crcs(A)
                xs = oc.full_block_crcs(X.reshape(n, BLOCK_SIZE))
                stats["a_mismatch"] += 1
                stats.setdefault("a_saw", []).append({
                    "d2h": "prevZ" if prev is not None and np.array_equal(got_a, prev[0]) else
                           "prevY" if prev is not None and np.array_equal(got_a, prev[1]) else
                           "zeros" if not got_a.any() else "other",
                    "kernel_crcs_of_A": "X" if np.array_equal(ka, xs) else
                                        "zeros" if (ka == zero_crc).all() else "other",
                    "va_A": hex(va_a), "va_prev_B": hex(prev[2]) if prev is not None else None,
                    "A_overlaps_prev_B": bool(prev is not None and prev[2] <= va_a < prev[2] + nbytes)})
            if mode == "sync":
                hip.hipDeviceSynchronize()
            if mode == "keepva":
                A.hip.hipMemUnmap(A.va, A.nbytes)
                A.hip.hipMemRelease(A.handle)
                kept.append(A)
            elif mode == "keepphys":
                A.hip.hipMemUnmap(A.va, A.nbytes)
                A.hip.hipMemAddressFree(A.va, A.reserved)
                kept_phys.append(A)
            else:
                A.release()
            rng = np.random.default_rng(i)
            Y = rng.integers(0, 256, nbytes, dtype=np.uint8)
            B = ctx.alloc(nbytes) if mode == "plain" else GuardedImage(0, nbytes)
            va_b = B.ptr
            stats["va_reused"] += int(va_b == va_a)
            ctx.h2d(B, Y)
            got = ctx.d2h(B, nbytes)
            if not np.array_equal(got, Y):
                stats["copy_mismatch"] += 1
                stats["copy_saw"].append("X" if np.array_equal(got, X) else
                                         "zeros" if not got.any() else "other")
            want = oc.full_block_crcs(Y.reshape(n, BLOCK_SIZE))
            kr = crcs(B)
            if not np.array_equal(kr, want):
                stats["kread_mismatch"] += 1
                xs = oc.full_block_crcs(X.reshape(n, BLOCK_SIZE))
                stats["kread_saw"].append("X" if np.array_equal(kr, xs) else
                                          "zeros" if (kr == zero_crc).all() else "other")
            ctx.synth_full_blocks(B, n, seed=sz)
            ctx.sync()
            got = ctx.d2h(B, nbytes)
            Z = oc.synth_full_blocks(n, seed=sz).reshape(-1)
            if not np.array_equal(got, Z):
                stats["kwrite_mismatch"] += 1
                stats["kwrite_saw"].append("Y" if np.array_equal(got, Y) else
                                           "X" if np.array_equal(got, X) else
                                           "zeros" if not got.any() else "other")
            stats["events"].append([i, hex(va_a), hex(va_b)])
            prev = (Z, Y, va_b)
            if mode == "sync":
                hip.hipDeviceSynchronize()
            if mode == "plain":
                B.free()
            elif mode == "keepva":
                B.hip.hipMemUnmap(B.va, B.nbytes)
                B.hip.hipMemRelease(B.handle)
                kept.append(B)
            else:
                B.release()
        hip.hipDeviceSynchronize()
        for k in kept:
            k.hip.hipMemAddressFree(k.va, k.reserved)
        for k in kept_phys:
            k.hip.hipMemRelease(k.handle)
        stats["events"] = stats["events"][:6]
        stats["a_saw"] = stats.get("a_saw", [])[:6]
        print(json.dumps(stats), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
