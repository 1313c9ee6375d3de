"""Pin the oracle to the reference's own known answers (CPU).

The reference (Rust) cannot be built here, so the oracle restatement is
pinned by the reference's tests as data:
  src/util/crc.rs:50-76   RFC 3720 B.4 vectors
  src/util/crc.rs:78-108  value/extend/mask/unmask identities
  src/log_reader.rs:229-241  golden 18-byte WAL image
and the Python and C restatements are checked against each other.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_image
from oracle import crc32c_oracle as po
from oracle import oracle_c as oc


@pytest.fixture(scope="module")
def kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


def test_crc_standard_results(kat):  # crc.rs:50-76
    for v in kat["value"]:
        data = bytes.fromhex(v["data_hex"])
        assert po.value(data) == v["crc"]
        assert oc.value(data) == v["crc"]
        for variant in ("bytewise", "slice16", "sse42"):
            fn = getattr(oc.lib(), {"bytewise": "oracle_crc_bytewise", "slice16": "oracle_crc_slice16",
                                    "sse42": "oracle_crc_sse42"}[variant])
            assert fn(0xFFFFFFFF, data, len(data)) ^ 0xFFFFFFFF == v["crc"], variant
    assert po.value(b"123456789") == kat["check_123456789"] == po.CHECK


def test_crc_values():  # crc.rs:78-81
    assert po.value(b"a") != po.value(b"foo")


def test_crc_extend():  # crc.rs:83-86: init is a prefix BYTE
    assert po.value(b"hello world") == po.extend(ord("h"), b"ello world")
    assert oc.value(b"hello world") == oc.extend(ord("h"), b"ello world")


def test_crc_mask():  # crc.rs:88-95
    crc = po.value(b"foo")
    assert crc != po.mask(crc)
    assert crc != po.mask(po.mask(crc))
    assert crc == po.unmask(po.mask(crc))
    assert crc == po.unmask(po.unmask(po.mask(po.mask(crc))))
    assert oc.mask(crc) == po.mask(crc)


def test_hello_world():  # crc.rs:97-108
    crc = po.extend(1, b"hello world")
    assert crc == po.crc_update(po.crc_update(po.INIT, b"\x01"), b"hello world") ^ po.XOROUT
    assert po.unmask(po.mask(crc)) == crc


def test_golden_wal_image(kat):  # log_reader.rs:229-241
    img = bytes(kat["hello_world_image"])
    assert po.write_image([b"hello world"]) == img
    assert oc.write_image([b"hello world"]) == img
    assert po.read_all(img) == [b"hello world"]
    # the header is mask(crc32c(0x01 || "hello world")) little-endian
    assert po.decode_fixed32(img[:4]) == po.mask(po.extend(1, b"hello world")) == 0x0701DD81


def test_combine_algebra():
    rng = np.random.default_rng(1)
    for _ in range(20):
        a = rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
        assert po.crc_combine(po.value(a), po.value(b), len(b)) == po.value(a + b)


def test_python_vs_c_random():
    rng = np.random.default_rng(2)
    for n in [0, 1, 2, 3, 7, 8, 15, 16, 17, 100, 1000, 4097]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert po.value(d) == oc.value(d)
        assert po.extend(3, d) == oc.extend(3, d)


def test_numpy_rows_matches_scalar():
    blocks = po.synth_full_blocks(3)
    want = [po.mask(po.value(bytes(b[6:]))) for b in blocks[:1]]
    assert po.full_block_masked_crcs(blocks[:1]).tolist() == want
    assert np.array_equal(oc.synth_full_blocks(3), blocks)
    assert np.array_equal(oc.full_block_crcs(blocks), po.full_block_masked_crcs(blocks))


def test_golden_edge_images_reproduce(golden_index):
    for name, ent in golden_index.items():
        img = golden_image(name)
        assert hashlib.sha256(img).hexdigest() == ent["sha256"], name
        walk = oc.walk(img)
        got = [[int(r["file_offset"]), int(r["length"]), int(r["type"]), int(r["stored_crc"]),
                int(r["computed_crc"]), int(r["status"])] for r in walk]
        assert got == ent["physical"], name


def test_golden_c1():
    z = np.load(os.path.join(GOLDEN, "c1_records.npz"))
    n, size, seed = 10000, 4096, 0x5EED0001
    words = po.splitmix64_np(np.uint64(seed) ^ np.arange(n, dtype=np.uint64), size // 8)
    image = oc.write_image([words[i].tobytes() for i in range(n)])
    assert len(image) == int(z["nbytes"][0]) == 41038750
    assert hashlib.sha256(image).digest() == z["sha256"].tobytes()
    w = oc.walk(image)
    assert np.array_equal(w["stored_crc"], z["stored_crc"])
    assert (w["status"] == 0).all()


def test_reader_semantics_edges(golden_index):
    assert po.read_all(golden_image("truncated_tail")) == \
        [po.splitmix64_stream(70 + i, 9000) for i in range(4)]
    with pytest.raises(po.CorruptionError):
        po.read_all(golden_image("corrupt_bit"))
    with pytest.raises(po.CorruptionError):
        po.read_all(golden_image("zero_block"))
    assert len(po.read_all(golden_image("corrupt_bit"), checksum=False)) == 20


# ---- WriteBatch / varint restatement (write_batch.rs, coding.rs) ----
from oracle import write_batch_oracle as wb  # noqa: E402


def test_varint32_roundtrip():  # coding.rs:173-191
    s = b"".join(wb.put_varint32(((i // 32) << (i % 32)) & 0xFFFFFFFF) for i in range(32 * 32))
    off = 0
    for i in range(32 * 32):
        v, used = wb.get_varint32(s, off, len(s))
        assert v == ((i // 32) << (i % 32)) & 0xFFFFFFFF
        assert used == len(wb.put_varint32(v))
        off += used
    assert off == len(s)


def test_varint32_overflow_and_truncation():  # coding.rs:193-212
    assert wb.get_varint32(bytes([129, 130, 131, 132, 133, 17]), 0, 6) is None
    big = wb.put_varint32((1 << 31) + 100)
    for n in range(len(big)):
        assert wb.get_varint32(big, 0, n) is None
    assert wb.get_varint32(big, 0, len(big)) == ((1 << 31) + 100, 5)


def test_write_batch_encode_decode():
    b = wb.WriteBatch()
    assert b.contents() == bytes(12) and b.count() == 0
    b.put(b"foo", b"bar")
    b.delete(b"box")
    b.put(b"baz", b"boo")
    b.set_sequence(100)
    rep = b.contents()
    assert rep[:12] == (100).to_bytes(8, "little") + (3).to_bytes(4, "little")
    assert rep[12:] == b"\x01\x03foo\x03bar\x00\x03box\x01\x03baz\x03boo"
    st, seq, cnt, ents = wb.decode(rep)
    assert (st, seq, cnt) == (wb.OK, 100, 3)
    assert ents == [(100, 1, b"foo", b"bar"), (101, 0, b"box", b""), (102, 1, b"baz", b"boo")]


def test_write_batch_malformed():
    from tests_gen import malformed_batches
    for name, rep, want in malformed_batches():
        assert wb.decode(rep)[0] == want, name
    # entries before an error are still reported (LevelDB hands them over)
    st, _, _, ents = wb.decode(dict((n, r) for n, r, _ in malformed_batches())["bad_tag"])
    assert st == wb.BAD_TAG and [e[2] for e in ents] == [b"k", b"gone"]


def test_batch_log_sequences_follow_db_write():  # db.rs:95-112
    from tests_gen import batch_log
    reps = batch_log(np.random.default_rng(1), 30, first_sequence=5)
    nxt = 5
    for r in reps:
        st, seq, cnt, ents = wb.decode(r)
        assert st == wb.OK and seq == nxt and len(ents) == cnt
        nxt += cnt
