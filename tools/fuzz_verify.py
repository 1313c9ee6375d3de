"""Randomised parity campaign for the C3 verify path (GPU box):
random WAL images -- record-size mixes from 0-byte to multi-block records,
block-edge sizes, dense small-record regions -- with structural corruptions
(bit flips, zeroed ranges, rewritten length / type bytes, truncation, garbage
blocks and tails), verified through the production C-ABI sequence
(revel_gpu_count_scan_records -> revel_gpu_verify_records) and, for the
smaller images, every test-hook verify path, each compared field by field
with the C oracle's walk (oracle/, the checker).

    python tools/fuzz_verify.py [--seconds 150] [--seed 1] [--max-mib 48]

Prints a progress line every ~20 s and one JSON summary line; on the first
mismatch it writes the image to gpurun_out/fuzz_fail_<seed>.bin and exits 1.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BLOCK = 32768
EDGE = np.array([0, 1, 2, 3, 4, 5, 6, 7, 8, 15, 16, 17, 32754, 32755, 32756, 32757, 32758, 32759, 32760, 32761,
                 32762, 32768, 65522, 65523, 98283])
PATHS = [None, 0, 1, 2, 3]


def sizes_of(rng, kind: str, target: int) -> np.ndarray:
    """Record payload sizes of one segment, about `target` image bytes."""
    if kind == "tiny":
        per = 7 + 8
        return rng.integers(0, 17, max(1, target // per))
    if kind == "small":
        m = int(rng.choice([32, 64, 128, 256, 512]))
        return rng.integers(0, m + 1, max(1, target // (7 + m // 2)))
    if kind == "zipf":
        k = np.arange(1, 513, dtype=np.float64)
        p = k ** -1.1
        p /= p.sum()
        n = max(1, target // 3400)
        return 64 * rng.choice(np.arange(1, 513), size=n, p=p)
    if kind == "big":
        return rng.integers(0, 200001, max(1, target // 100000))
    if kind == "edge":
        return rng.choice(EDGE, size=max(1, target // 20000))
    if kind == "periodic":
        return np.full(max(1, target // 120), int(rng.integers(0, 240)))
    raise ValueError(kind)


def make_image(rng, max_bytes: int):
    import oracle.oracle_c as oc
    target = int(np.exp(rng.uniform(np.log(1024), np.log(max_bytes))))
    kinds = ["tiny", "small", "zipf", "big", "edge", "periodic"]
    nseg = int(rng.integers(1, 5))
    parts = []
    for _ in range(nseg):
        parts.append(sizes_of(rng, str(rng.choice(kinds)), max(256, target // nseg)))
    sizes = np.concatenate(parts).astype(np.int64)
    blob = rng.integers(0, 256, int(sizes.sum()) + 1, dtype=np.uint8).tobytes()
    recs, o = [], 0
    for s in sizes:
        recs.append(blob[o:o + int(s)])
        o += int(s)
    img = bytearray(oc.write_image(recs))
    return img, len(sizes)


def corrupt(rng, img: bytearray, ref) -> list:
    """0..8 random structural corruptions, in place; returns their names."""
    ops = []
    for _ in range(int(rng.integers(0, 9))):
        if len(img) == 0:
            break
        op = int(rng.integers(0, 8))
        n = len(img)
        if op == 0:  # bit flip anywhere
            img[int(rng.integers(0, n))] ^= 1 << int(rng.integers(0, 8))
            ops.append("flip")
        elif op == 1:  # zeroed range (zero records / preallocated tail)
            a = int(rng.integers(0, n))
            k = min(n - a, int(rng.integers(1, 70000)))
            img[a:a + k] = bytes(k)
            ops.append("zero")
        elif op in (2, 3) and len(ref):  # a header's length or type byte rewritten
            r = ref[int(rng.integers(0, len(ref)))]
            p = int(r["file_offset"])
            if op == 2 and p + 6 <= n:
                v = int(rng.choice([0, 1, 6, 7, 32761, 32762, 65535, int(rng.integers(0, 65536))]))
                img[p + 4] = v & 0xFF
                img[p + 5] = v >> 8
                ops.append("len")
            elif op == 3 and p + 7 <= n:
                img[p + 6] = int(rng.choice([0, 5, 255, int(rng.integers(0, 256))]))
                ops.append("type")
        elif op == 4:  # truncation
            img[n - min(n, int(rng.integers(1, 40000))):] = b""
            ops.append("cut")
        elif op == 5:  # garbage tail
            img += rng.integers(0, 256, int(rng.integers(1, 50000)), dtype=np.uint8).tobytes()
            ops.append("tail")
        elif op == 6 and n >= BLOCK:  # one whole block of random bytes
            b = int(rng.integers(0, n // BLOCK))
            img[b * BLOCK:(b + 1) * BLOCK] = rng.integers(0, 256, BLOCK, dtype=np.uint8).tobytes()
            ops.append("garbage_block")
        elif op == 7:  # a trailer-sized hole: 1..6 bytes zeroed just before a block end
            if n >= BLOCK:
                e = BLOCK * int(rng.integers(1, n // BLOCK + 1))
                k = int(rng.integers(1, 7))
                img[e - k:e] = bytes(k)
                ops.append("trailer")
    return ops


def compare(res, ref) -> str:
    if len(res) != len(ref):
        return f"records {len(res)} vs {len(ref)}"
    for f in ("file_offset", "length", "type", "stored_crc", "computed_crc", "status"):
        if not np.array_equal(res[f].astype(np.uint64), ref[f].astype(np.uint64)):
            i = int(np.nonzero(res[f].astype(np.uint64) != ref[f].astype(np.uint64))[0][0])
            return f"field {f} record {i}: {int(res[f][i])} vs {int(ref[f][i])}"
    return ""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=150.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max-mib", type=float, default=48.0)
    ap.add_argument("--all-paths-below-mib", type=float, default=4.0)
    a = ap.parse_args()
    import oracle.oracle_c as oc  # the checker
    from revel_amd import gpu
    ctx = gpu.GpuContext(0)
    t0 = time.time()
    last = t0
    it = recs = phys = bytes_total = bad_total = 0
    kinds = {}
    while time.time() - t0 < a.seconds:
        seed = a.seed * 1_000_003 + it
        rng = np.random.default_rng(seed)
        img, nrec = make_image(rng, int(a.max_mib * (1 << 20)))
        ops = corrupt(rng, img, oc.walk(bytes(img), "sse42") if rng.random() < 0.7 else [])
        for o in ops:
            kinds[o] = kinds.get(o, 0) + 1
        data = bytes(img)
        it += 1
        if not data:
            continue
        ref = oc.walk(data, "bytewise" if len(data) < (8 << 20) else "sse42")
        # the device image at a random 16-B-aligned or unaligned offset inside its buffer
        shift = int(rng.choice([0, 0, 0, 16, 4, 1]))
        buf = ctx.alloc(len(data) + 64)
        ctx.h2d(buf, np.frombuffer(data, dtype=np.uint8), dst_offset=shift)

        class View:
            ptr, nbytes = buf.ptr + shift, len(data)
        paths = PATHS if len(data) <= a.all_paths_below_mib * (1 << 20) else [None]
        for p in paths:
            res = ctx.verify_image(View, len(data), path=p)
            msg = compare(res, ref)
            if msg:
                os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
                fn = os.path.join(ROOT, "gpurun_out", f"fuzz_fail_{seed}.bin")
                with open(fn, "wb") as f:
                    f.write(data)
                print(json.dumps({"fail": msg, "seed": seed, "path": p, "shift": shift, "bytes": len(data),
                                  "ops": ops, "image": fn}), flush=True)
                sys.exit(1)
        buf.free()
        recs += nrec
        phys += len(ref)
        bad_total += int((ref["status"] != 0).sum())
        bytes_total += len(data)
        if time.time() - last > 20:
            last = time.time()
            print(f"fuzz: {it} images, {bytes_total / 2**30:.2f} GiB, {phys} physical records, "
                  f"{bad_total} not OK, {time.time() - t0:.0f} s", flush=True)
    ctx.close()
    print(json.dumps({"images": it, "bytes": bytes_total, "logical_records": recs, "physical_records": phys,
                      "records_not_ok": bad_total, "corruptions": kinds, "seconds": round(time.time() - t0, 1),
                      "mismatches": 0, "paths": "production + test-hook paths 0-3 below %g MiB" % a.all_paths_below_mib,
                      "seed": a.seed}), flush=True)


if __name__ == "__main__":
    main()
