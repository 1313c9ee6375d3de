"""Generate the committed golden fixtures under tests/golden/.

Sources:
* ``kat.json`` -- known answers copied as DATA from the reference's own tests
  (src/util/crc.rs:50-108 RFC 3720 B.4 vectors, src/log_reader.rs:231 golden
  WAL image).  These pin the oracle.
* ``edge_*.bin`` + ``edge_cases.json`` -- WAL images produced by the oracle's
  writer restatement (oracle/crc32c_oracle.py, log_writer.rs:58-124) for the
  edge cases the reference never tests, with the oracle's
  per-physical-record walk.
* ``c1_records.npz`` -- config C1 (10 000 x 4 KiB, splitmix64 seed 0x5EED0001)
  image digest + per-record list, from the C restatement (oracle/crc32c_oracle.c),
  cross-checked here against the Python restatement on its first records.

Run:  python tests/golden/make_golden.py   (needs `make -C oracle`)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import crc32c_oracle as po  # noqa: E402
from oracle import oracle_c as oc  # noqa: E402

BLOCK = po.BLOCK_SIZE


def payload(seed: int, n: int) -> bytes:
    return po.splitmix64_stream(seed, n)


def edge_cases():
    """name -> (records, block_offset, post-processing)"""
    cases = {}
    cases["hello_world"] = ([b"hello world"], 0, None)
    cases["empty_full"] = ([b""], 0, None)
    cases["one_byte"] = ([b"x"], 0, None)
    cases["exact_fill"] = ([payload(1, 32761)], 0, None)
    cases["exact_fill_x3"] = ([payload(2 + i, 32761) for i in range(3)], 0, None)
    cases["first_last"] = ([payload(5, 40000)], 0, None)
    cases["first_middle_last"] = ([payload(6, 100000)], 0, None)
    for t in range(1, 7):  # block trailers of 1..6 bytes are zero-padded
        cases[f"trailer_{t}"] = ([payload(10 + t, 32761 - 7 - t), payload(20 + t, 50)], 0, None)
    cases["trailer_7_exact_header"] = ([payload(30, 32761 - 7), b""], 0, None)
    cases["block_offset_32765"] = ([payload(31, 100), payload(32, 33000)], 32765, None)
    cases["many_small"] = ([payload(40 + i, i % 97) for i in range(600)], 0, None)
    cases["many_empty"] = ([b""] * 5000, 0, None)  # > 4681 physical records per block
    cases["zero_block"] = ([payload(50, 1000)], 0, "append_zero_block")
    cases["corrupt_bit"] = ([payload(60 + i, 3000) for i in range(20)], 0, "flip_bit")
    cases["truncated_tail"] = ([payload(70 + i, 9000) for i in range(5)], 0, "truncate")
    cases["mixed"] = ([payload(80 + i, (i * 7919) % 70000) for i in range(40)], 0, None)
    return cases


def post(image: bytes, how):
    if how is None:
        return image
    b = bytearray(image)
    if how == "append_zero_block":
        pad = (-len(b)) % BLOCK
        b += bytes(pad + BLOCK)
    elif how == "flip_bit":
        b[5 * 3007 + 1234] ^= 0x10   # inside the payload of record 5
    elif how == "truncate":
        b = b[:len(b) - 4321]
    return bytes(b)


def main() -> None:
    # ---- KATs (reference test data) ----
    kat = {
        "source": "src/util/crc.rs:50-108, src/log_reader.rs:229-241 (guimingyue/revel @ v0)",
        "value": [
            {"data_hex": bytes(32).hex(), "crc": 0x8A9136AA},
            {"data_hex": (b"\xff" * 32).hex(), "crc": 0x62A8AB43},
            {"data_hex": bytes(range(32)).hex(), "crc": 0x46DD794E},
            {"data_hex": bytes(range(31, -1, -1)).hex(), "crc": 0x113FDB5C},
            {"data_hex": bytes([0x01, 0xc0, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
                                0x00, 0x00, 0x00, 0x00, 0x14, 0x00, 0x00, 0x00, 0x00, 0x00, 0x04, 0x00,
                                0x00, 0x00, 0x00, 0x14, 0x00, 0x00, 0x00, 0x18, 0x28, 0x00, 0x00, 0x00,
                                0x00, 0x00, 0x00, 0x00, 0x02, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00]).hex(),
             "crc": 0xD9963A56},
        ],
        "check_123456789": 0xE3069283,
        "hello_world_image": [129, 221, 1, 7, 11, 0, 1, 104, 101, 108, 108, 111, 32, 119, 111, 114, 108, 100],
    }
    for v in kat["value"]:
        assert po.value(bytes.fromhex(v["data_hex"])) == v["crc"]
    assert bytes(kat["hello_world_image"]) == po.write_image([b"hello world"])
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)

    # ---- edge-case images ----
    index = {}
    for name, (recs, boff, how) in edge_cases().items():
        img_py = po.write_image(recs, block_offset=boff)
        img_c = oc.write_image(recs, block_offset=boff)
        assert img_py == img_c, name
        image = post(img_py, how)
        walk = po.walk_records(image)
        cw = oc.walk(image)
        assert len(cw) == len(walk), name
        for a, b in zip(walk, cw):
            assert (a.file_offset, a.length, a.rtype, a.stored, a.computed, a.status) == \
                (int(b["file_offset"]), int(b["length"]), int(b["type"]), int(b["stored_crc"]),
                 int(b["computed_crc"]), int(b["status"])), name
        fn = f"edge_{name}.bin"
        with open(os.path.join(HERE, fn), "wb") as f:
            f.write(image)
        try:
            logical = po.read_all(image, checksum=True)
            logical_err = None
        except po.CorruptionError as e:
            logical, logical_err = None, repr(e.args[0].status)
        index[name] = {
            "file": fn, "block_offset": boff, "post": how, "nbytes": len(image),
            "sha256": hashlib.sha256(image).hexdigest(),
            "records_in": [{"len": len(r), "sha256": hashlib.sha256(r).hexdigest()} for r in recs],
            "physical": [[p.file_offset, p.length, p.rtype, p.stored, p.computed, p.status] for p in walk],
            "logical_sha256": None if logical is None else [hashlib.sha256(x).hexdigest() for x in logical],
            "logical_error_status": logical_err,
        }
    with open(os.path.join(HERE, "edge_cases.json"), "w") as f:
        json.dump(index, f, indent=0)

    # ---- config C1: 10 000 x 4 KiB ----
    n, size, seed = 10000, 4096, 0x5EED0001
    words = po.splitmix64_np(np.uint64(seed) ^ np.arange(n, dtype=np.uint64), size // 8)
    recs = [words[i].tobytes() for i in range(n)]
    image = oc.write_image(recs)
    head = po.write_image(recs[:48])
    assert image[:len(head)] == head
    w = oc.walk(image)
    np.savez_compressed(os.path.join(HERE, "c1_records.npz"), file_offset=w["file_offset"], length=w["length"],
                        type=w["type"], stored_crc=w["stored_crc"], status=w["status"],
                        nbytes=np.array([len(image)]),
                        sha256=np.frombuffer(hashlib.sha256(image).digest(), dtype=np.uint8))
    print(f"C1 image {len(image)} bytes, {len(w)} physical records, {(len(image) + BLOCK - 1) // BLOCK} blocks")
    print(f"wrote {len(index)} edge cases")


if __name__ == "__main__":
    main()
