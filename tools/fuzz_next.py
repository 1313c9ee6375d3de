"""Randomised parity campaign for the SURVEY 8(f) rows on the GPU box (the
companion of tools/fuzz_verify.py, which covers the C3 verify path):
  * device append framing (revel_gpu_append_records) of random record-size
    sequences at random writer block offsets, byte for byte against the oracle
    writer (log_writer.rs:58-124) and its final block_offset;
  * device replay reassembly (revel_gpu_reassemble) of random, structurally
    corrupted images, event for event against the oracle reader's
    catch-and-continue sequence (log_reader.rs:76-153), checksum on and off;
  * device WriteBatch decode (revel_gpu_decode_batches) of random batch logs,
    malformed batches mixed in, entry for entry against the oracle's
    LevelDB-correct iterate (write_batch.rs:79-128).
The oracle (oracle/) is the checker only.

    python tools/fuzz_next.py [--seconds 150] [--seed 1]

Prints a progress line every ~20 s and one JSON summary line; on the first
mismatch it prints the failing case and exits 1.
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
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

BLOCK = 32768
OFFSETS = [0, 1, 5, 6, 7, 8, 100, 32754, 32755, 32760, 32761, 32762, 32767, 32768]


def fail(kind: str, seed: int, msg: str, **kw):
    print(json.dumps({"fail": kind, "seed": seed, "msg": msg, **kw}), flush=True)
    sys.exit(1)


def append_case(ctx, rng, seed):
    import oracle.oracle_c as oc
    from fuzz_verify import sizes_of
    target = int(np.exp(rng.uniform(np.log(256), np.log(6 << 20))))
    kinds = ["tiny", "small", "zipf", "big", "edge", "periodic"]
    sizes = np.concatenate([sizes_of(rng, str(rng.choice(kinds)), max(256, target // 2))
                            for _ in range(int(rng.integers(1, 4)))]).astype(np.int64)
    bo = int(rng.choice(OFFSETS)) if rng.random() < 0.6 else int(rng.integers(0, BLOCK + 1))
    blob = rng.integers(0, 256, max(1, int(sizes.sum())), dtype=np.uint8)
    recs, o = [], 0
    for s in sizes:
        recs.append(blob[o:o + int(s)].tobytes())
        o += int(s)
    d = ctx.upload(blob)
    img, n, nbo = ctx.append_records(d, [int(s) for s in sizes], bo)
    want = oc.write_image(recs, bo)
    # the writer's final block_offset (log_writer.rs:58-97's loop, framing only: a
    # trailer under 7 bytes starts a new block, every record emits at least one fragment)
    end = bo
    for s in sizes:
        left = int(s)
        while True:
            if BLOCK - end < 7:
                end = 0
            frag = min(left, BLOCK - end - 7)
            end += 7 + frag
            left -= frag
            if left == 0:
                break
    got = ctx.d2h(img, n).tobytes() if n else b""
    if n != len(want) or got != want:
        i = next((k for k in range(min(len(got), len(want))) if got[k] != want[k]), min(len(got), len(want)))
        fail("append", seed, f"image differs at byte {i} ({n} vs {len(want)} bytes)", block_offset=bo,
             records=len(sizes))
    if nbo != end:
        fail("append", seed, f"block_offset {nbo} vs {end}", block_offset=bo)
    img.free()
    d.free()
    return len(sizes), n


def reassembly_case(ctx, rng, seed):
    import oracle.crc32c_oracle as po
    import oracle.oracle_c as oc
    from fuzz_verify import corrupt, make_image
    img, nrec = make_image(rng, 3 << 20)
    corrupt(rng, img, oc.walk(bytes(img), "sse42") if rng.random() < 0.7 else [])
    data = bytes(img)
    if not data:
        return 0, 0
    d = ctx.upload(np.frombuffer(data, dtype=np.uint8))
    for checksum in (True, False):
        ev, payload, _ = ctx.reassemble(d, len(data), checksum=checksum)
        want = po.replay_events(data, checksum=checksum)
        if len(ev) != len(want):
            fail("reassembly", seed, f"events {len(ev)} vs {len(want)}", checksum=checksum, bytes=len(data))
        for k, (e, w) in enumerate(zip(ev, want)):
            ok = int(e["file_offset"]) == w[1]
            if ok and w[0] == "record":
                p0 = int(e["payload_offset"])
                ok = e["status"] == 0 and payload[p0:p0 + int(e["length"])].tobytes() == w[2]
            elif ok:
                ok = e["status"] != 0 and e["length"] == 0
            if not ok:
                fail("reassembly", seed, f"event {k}: {w[0]} at {w[1]}", checksum=checksum, bytes=len(data))
    d.free()
    return len(want), len(data)


def batches_case(ctx, rng, seed):
    import oracle.crc32c_oracle as po
    import oracle.oracle_c as oc
    from oracle import write_batch_oracle as wb
    from revel_amd._lib import BATCH_NOT_RECORD
    from tests_gen import batch_log, malformed_batches
    reps = batch_log(rng, int(rng.integers(1, 80)), max_entries=int(rng.integers(1, 60)),
                     max_key=int(rng.integers(1, 400)), max_value=int(rng.integers(1, 4000)),
                     big_every=int(rng.integers(5, 60)))
    bad = [r for _, r, _ in malformed_batches()]
    for _ in range(int(rng.integers(0, 6))):
        reps.insert(int(rng.integers(0, len(reps) + 1)), bad[int(rng.integers(0, len(bad)))])
    img = bytearray(oc.write_image(reps))
    if rng.random() < 0.4 and len(img):  # a few log-level corruptions too
        for _ in range(int(rng.integers(1, 4))):
            img[int(rng.integers(0, len(img)))] ^= 1 << int(rng.integers(0, 8))
    data = bytes(img)
    d = ctx.upload(np.frombuffer(data, dtype=np.uint8))
    ev, payload, infos, ents = ctx.replay_batches(d, len(data), checksum=True)
    want = po.replay_events(data, checksum=True)
    if not (len(ev) == len(want) == len(infos)):
        fail("batches", seed, f"events {len(ev)} / infos {len(infos)} vs {len(want)}")
    total = 0
    for i, w in enumerate(want):
        info = infos[i]
        if int(info["first_entry"]) != total:
            fail("batches", seed, f"batch {i}: first_entry {int(info['first_entry'])} vs {total}")
        if w[0] == "error":
            if info["status"] != BATCH_NOT_RECORD or info["nentries"] != 0:
                fail("batches", seed, f"batch {i}: error event not marked")
            continue
        st, sq, cnt, oents = wb.decode(w[2])
        if int(info["status"]) != st or int(info["nentries"]) != len(oents):
            fail("batches", seed, f"batch {i}: status {int(info['status'])} vs {st}, "
                                  f"entries {int(info['nentries'])} vs {len(oents)}")
        if st != wb.TOO_SMALL and (int(info["sequence"]) != sq or int(info["count"]) != cnt):
            fail("batches", seed, f"batch {i}: header")
        for k, (oseq, otype, okey, oval) in enumerate(oents):
            g = ents[total + k]
            k0, v0 = int(g["key_offset"]), int(g["value_offset"])
            if not (int(g["batch"]) == i and int(g["sequence"]) == oseq and int(g["type"]) == otype and
                    payload[k0:k0 + int(g["key_len"])].tobytes() == okey and
                    payload[v0:v0 + int(g["value_len"])].tobytes() == oval):
                fail("batches", seed, f"batch {i} entry {k}")
        total += len(oents)
    if len(ents) != total:
        fail("batches", seed, f"entries {len(ents)} vs {total}")
    d.free()
    return len(want), total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=150.0)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    from revel_amd import gpu
    ctx = gpu.GpuContext(0)
    t0 = last = time.time()
    stats = {"append": [0, 0, 0], "reassembly": [0, 0, 0], "batches": [0, 0, 0]}
    cases = [("append", append_case), ("reassembly", reassembly_case), ("batches", batches_case)]
    it = 0
    while time.time() - t0 < a.seconds:
        name, fn = cases[it % 3]
        seed = a.seed * 1_000_003 + it
        x, y = fn(ctx, np.random.default_rng(seed), seed)
        s = stats[name]
        s[0] += 1
        s[1] += x
        s[2] += y
        it += 1
        if time.time() - last > 20:
            last = time.time()
            print(f"fuzz_next: {it} cases, {time.time() - t0:.0f} s, {json.dumps(stats)}", flush=True)
    ctx.close()
    print(json.dumps({
        "append": {"cases": stats["append"][0], "records": stats["append"][1], "image_bytes": stats["append"][2]},
        "reassembly": {"cases": stats["reassembly"][0], "events": stats["reassembly"][1],
                       "image_bytes": stats["reassembly"][2], "checksum": "on and off"},
        "batches": {"cases": stats["batches"][0], "events": stats["batches"][1], "entries": stats["batches"][2]},
        "mismatches": 0, "seconds": round(time.time() - t0, 1), "seed": a.seed}), flush=True)


if __name__ == "__main__":
    main()
