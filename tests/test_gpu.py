"""GPU parity tests: every kernel through the C-ABI vs the oracle, bit-exact.

Config C2 (full-type blocks), config C3 (variable records via the device
walk + segmented CRC), the GPU-verified Reader, and size-independent
properties at larger sizes."""
import os

import numpy as np
import pytest

from revel_amd import BLOCK_SIZE, env, log
from revel_amd._lib import IO_ERROR, RevelError, check
from revel_amd.gpu import RECORD_DTYPE
from conftest import golden_image, trace
from oracle import crc32c_oracle as po
from oracle import oracle_c as oc

pytestmark = pytest.mark.gpu



class _View:
    """A device image at a byte offset inside a larger buffer."""

    def __init__(self, buf, off, nbytes):
        self.ptr, self.nbytes, self._buf = buf.ptr + off, nbytes, buf


def run_full(ctx, host_blocks, variant=None):
    n = host_blocks.shape[0]
    d = ctx.upload(host_blocks)
    m = ctx.alloc(4 * n)
    ok = ctx.alloc(n)
    ctx.crc_full_blocks(d, n, m, ok, variant=variant)
    ctx.sync()
    return ctx.d2h(m, 4 * n, np.uint32), ctx.d2h(ok, n)


def kat_blocks():
    """Whole-block patterns (0x00, 0xFF, byte ramps), random payloads and
    one-hot bits at lane / chunk edges, framed as FULL blocks."""
    rng = np.random.default_rng(11)
    pats = [np.zeros(BLOCK_SIZE, np.uint8), np.full(BLOCK_SIZE, 0xFF, np.uint8),
            np.arange(BLOCK_SIZE, dtype=np.uint32).astype(np.uint8),
            (np.arange(BLOCK_SIZE, dtype=np.uint32)[::-1]).astype(np.uint8)]
    for _ in range(12):
        pats.append(rng.integers(0, 256, BLOCK_SIZE, dtype=np.uint8))
    blocks = np.stack(pats)
    # one-hot bit blocks exercise every lane / byte position of the combine
    for pos in [6, 7, 8, 511, 512, 513, 4095, 16384, 32767]:
        b = np.zeros(BLOCK_SIZE, np.uint8)
        b[pos] = 0x80
        blocks = np.vstack([blocks, b[None]])
    blocks[:, 4] = 0xF9
    blocks[:, 5] = 0x7F
    blocks[:, 6] = 1
    crcs = oc.full_block_crcs(blocks)
    blocks[:, 0:4] = crcs.view(np.uint8).reshape(-1, 4)
    return blocks


@pytest.mark.parametrize("nrand", [0, 1, 15, 16, 17, 300, 4095, 4097])
def test_full_blocks_vs_oracle(gpu_ctx, nrand):
    """Every block count around the wave / workgroup / grid boundaries of the
    persistent 16-wave kernel (4096 resident waves on 256 CUs)."""
    blocks = np.vstack([kat_blocks(), oc.synth_full_blocks(nrand, seed=0x1234 + nrand)])
    got, ok = run_full(gpu_ctx, blocks)
    want = oc.full_block_crcs(blocks)
    assert np.array_equal(got, want)
    assert ok.all()


@pytest.mark.parametrize("shift", [1, 4, 8, 12])
def test_full_blocks_unaligned_base(gpu_ctx, shift):
    """Blocks at a device address that is not 16-B aligned (the C2 entry point
    accepts any base; the 16-B row loads are unaligned then): same CRCs."""
    blocks = np.vstack([kat_blocks(), oc.synth_full_blocks(40, seed=shift)])
    n = blocks.shape[0]
    buf = gpu_ctx.alloc(n * BLOCK_SIZE + 64)
    gpu_ctx.h2d(buf, blocks.reshape(-1), dst_offset=shift)
    m, ok = gpu_ctx.alloc(4 * n), gpu_ctx.alloc(n)
    gpu_ctx.crc_full_blocks(_View(buf, shift, n * BLOCK_SIZE), n, m, ok)
    gpu_ctx.sync()
    assert np.array_equal(gpu_ctx.d2h(m, 4 * n, np.uint32), oc.full_block_crcs(blocks))
    assert gpu_ctx.d2h(ok, n).all()


def test_full_blocks_flags_corruption(gpu_ctx):
    blocks = oc.synth_full_blocks(200, seed=99)
    rng = np.random.default_rng(12)
    bad = rng.choice(200, 40, replace=False)
    for i, b in enumerate(bad):
        kind = i % 4
        if kind == 0:
            blocks[b, 6 + int(rng.integers(1, 32762))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif kind == 1:
            blocks[b, 0] ^= 1            # stored crc
        elif kind == 2:
            blocks[b, 4] = 0x10          # length
        else:
            blocks[b, 6] = 2             # type byte (also changes the crc input)
    got, ok = run_full(gpu_ctx, blocks)
    assert np.array_equal(got, oc.full_block_crcs(blocks))
    want_ok = np.ones(200, bool)
    want_ok[bad] = False
    assert np.array_equal(ok.astype(bool), want_ok)


def test_synth_and_frame_match_oracle(gpu_ctx):
    n = 64
    d = gpu_ctx.alloc(n * BLOCK_SIZE)
    gpu_ctx.synth_full_blocks(d, n, seed=0x5EED0002, first=1000)
    gpu_ctx.sync()
    got = gpu_ctx.d2h(d, n * BLOCK_SIZE).reshape(n, BLOCK_SIZE)
    assert np.array_equal(got, oc.synth_full_blocks(n, seed=0x5EED0002, first=1000))
    # frame a payload-only buffer on device (GPU append framing)
    raw = got.copy()
    raw[:, :7] = 0xAB
    d2 = gpu_ctx.upload(raw)
    gpu_ctx.frame_full_blocks(d2, n)
    gpu_ctx.sync()
    assert np.array_equal(gpu_ctx.d2h(d2, n * BLOCK_SIZE).reshape(n, BLOCK_SIZE), got)


def test_full_blocks_large_property(gpu_ctx):
    """65 536 blocks (2 GiB): device synth -> all verify flags ok; CRCs of a
    1/64 sample equal the oracle's; a flipped block is caught."""
    n = 65536
    d = gpu_ctx.alloc(n * BLOCK_SIZE)
    gpu_ctx.synth_full_blocks(d, n, seed=0x5EED0002)
    m = gpu_ctx.alloc(4 * n)
    ok = gpu_ctx.alloc(n)
    gpu_ctx.crc_full_blocks(d, n, m, ok)
    gpu_ctx.sync()
    masked = gpu_ctx.d2h(m, 4 * n, np.uint32)
    assert gpu_ctx.d2h(ok, n).all()
    idx = np.arange(0, n, 64)
    sample = np.stack([gpu_ctx.d2h(d, BLOCK_SIZE, src_offset=int(i) * BLOCK_SIZE) for i in idx[:256]])
    assert np.array_equal(masked[idx[:256]], oc.full_block_crcs(sample))


def compare_walk(res, ref):
    assert len(res) == len(ref)
    for f in ("file_offset", "length", "type", "stored_crc", "computed_crc", "status"):
        assert np.array_equal(res[f].astype(np.uint64), ref[f].astype(np.uint64)), f


# Verify paths: None = the C-ABI call sequence revel_gpu_count_scan_records
# -> revel_gpu_verify_records (the production default: k_count_hist +
# k_scan_order, then k_verify_rows for blocks of up to 64 records and
# k_verify_records_dense2 for the rest); then the test hook after the count
# pass: 0 = the production verify, 1 = v3 walking the headers itself (verify
# without its count pass), 2 = v3 with the count pass's header lists
# (unaligned images), 3 = the round-4 split.  Round 5's small-record kernels
# (one-pass, coalesced dense, quad loads) left the product in round 6: the
# same tests run them over tools/experiments/libexperiments.so in
# test_experiments_gpu.py (-m experiment).
VERIFY_PATHS = [None, 0, 1, 2, 3]


@pytest.mark.parametrize("path", VERIFY_PATHS)
def test_verify_golden_images(gpu_ctx, golden_index, path):
    for name in golden_index:
        img = golden_image(name)
        dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
        res = gpu_ctx.verify_image(dimg, len(img), path=path)
        compare_walk(res, oc.walk(img))


def zipf_image(rng, nbytes_target):
    k = np.arange(1, 513)
    p = k ** -1.1
    p /= p.sum()
    recs = []
    total = 0
    while total < nbytes_target:
        s = 64 * int(rng.choice(k, p=p))
        recs.append(rng.integers(0, 256, s, dtype=np.uint8).tobytes())
        total += s + 7
    return recs


@pytest.mark.parametrize("path", VERIFY_PATHS)
def test_verify_zipf_and_corruption(gpu_ctx, path):
    rng = np.random.default_rng(13)
    recs = zipf_image(rng, 16 << 20)
    img = bytearray(oc.write_image(recs))
    ref = oc.walk(bytes(img))
    # flip one bit in 100 random records' payload
    okrecs = np.flatnonzero(ref["length"] > 0)
    victims = rng.choice(okrecs, 100, replace=False)
    for v in victims:
        off = int(ref["file_offset"][v]) + 7 + int(rng.integers(0, int(ref["length"][v])))
        img[off] ^= 1 << int(rng.integers(0, 8))
    img = bytes(img)
    dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    res = gpu_ctx.verify_image(dimg, len(img), base_offset=0, path=path)
    ref2 = oc.walk(img)
    compare_walk(res, ref2)
    assert sorted(np.flatnonzero(res["status"] == 1).tolist()) == sorted(victims.tolist())


@pytest.mark.parametrize("path", VERIFY_PATHS)
@pytest.mark.parametrize("cut", [1, 3, 6, 7, 8, 100, 32767, 32769, 40000])
def test_verify_partial_last_block(gpu_ctx, cut, path):
    rng = np.random.default_rng(cut)
    recs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in rng.integers(0, 9000, 30)]
    img = oc.write_image(recs)
    img = img[:min(len(img), cut + 65536)]
    dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    compare_walk(gpu_ctx.verify_image(dimg, len(img), path=path), oc.walk(img))


@pytest.mark.parametrize("tail_records", [1, 13, 63, 64, 65])
def test_verify_tail_block_cuts(gpu_ctx, tail_records):
    """The partial tail block goes through k_verify_rows with a length-bounded
    buffer resource: cuts at record ends, inside headers and payloads, at and
    around 16-B / 256-B / 1 KiB boundaries, a flipped bit in the tail; 64
    records = the rows kernel's limit, 65 = the dense kernel."""
    rng = np.random.default_rng(100 + tail_records)
    head = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in rng.integers(500, 9000, 8)]
    img0 = oc.write_image(head)
    pad = (-len(img0)) % 32768
    # fill to the block end with one record (or a trailer), then the tail records
    filler = [bytes(rng.integers(0, 256, pad - 7, dtype=np.uint8))] if pad >= 7 else []
    sizes = rng.integers(0, 380, tail_records)
    tail = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in sizes]
    img = oc.write_image(head + filler + tail)
    ends = oc.walk(img)
    base = (len(img) - 1) // 32768 * 32768
    rec_ends = [int(o) + 7 + int(n) for o, n in zip(ends["file_offset"], ends["length"]) if o >= base]
    cuts = set(rec_ends[-3:]) | {e - 1 for e in rec_ends[-3:]} | {e - 5 for e in rec_ends[-2:]}
    cuts |= {base + k for k in (1, 6, 7, 15, 16, 17, 255, 256, 257, 1023, 1024, 1025)}
    for cut in sorted(c for c in cuts if base < c <= len(img)):
        part = bytearray(img[:cut])
        if cut == len(img) and len(rec_ends) > 2:
            part[rec_ends[-2] - 3] ^= 0x10  # a payload bit of the second-to-last tail record
        part = bytes(part)
        dimg = gpu_ctx.upload(np.frombuffer(part, dtype=np.uint8))
        compare_walk(gpu_ctx.verify_image(dimg, len(part)), oc.walk(part))
        dimg.free()


@pytest.mark.parametrize("trailer", [0, 3, 6])
def test_verify_and_append_64_record_blocks(gpu_ctx, trailer):
    """Whole blocks with exactly 64 records (the rows kernel's limit: the end
    capture has no lane of its own), the last one ending `trailer` bytes before
    the block end, through verify and device append framing, plus a flipped
    bit in record 63."""
    rng = np.random.default_rng(640 + trailer)
    recs = []
    for _ in range(3):
        body = 32768 - trailer - 64 * 7
        cuts = np.sort(rng.choice(np.arange(1, body), 63, replace=False))
        sizes = np.diff(np.concatenate([[0], cuts, [body]]))
        recs += [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in sizes]
    img = oc.write_image(recs)
    assert len(img) == 3 * 32768 - trailer  # the writer leaves the last trailer out
    ref = oc.walk(img)
    assert len(ref) == 192
    dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    compare_walk(gpu_ctx.verify_image(dimg, len(img)), ref)
    bad = bytearray(img)
    bad[int(ref["file_offset"][63]) + 9] ^= 4
    bad = bytes(bad)
    dbad = gpu_ctx.upload(np.frombuffer(bad, dtype=np.uint8))
    res = gpu_ctx.verify_image(dbad, len(bad))
    compare_walk(res, oc.walk(bad))
    assert np.flatnonzero(res["status"] == 1).tolist() == [63]
    blob = np.frombuffer(b"".join(recs), dtype=np.uint8)
    d = gpu_ctx.upload(blob)
    out, n, _ = gpu_ctx.append_records(d, [len(r) for r in recs], 0)
    assert n == len(img)
    assert gpu_ctx.d2h(out, n).tobytes() == img


def test_expander_counts_1_to_64_with_flips(gpu_ctx):
    """k_expand_rows (round 3): the rows kernel leaves a mismatch mask per block
    and the expander writes the results, one lane per record across 16-block
    chunks in 64-record passes.  Blocks whose record counts cycle through
    1..64 (so chunks and passes split blocks everywhere, records 32..63 use the
    mask's high word) with ~1 record in 8 corrupted at a random byte, plus a
    torn last header: every field equals the oracle walk on every verify path."""
    rng = np.random.default_rng(6464)
    recs = []
    for nrec in list(range(1, 65)) + list(range(64, 0, -7)):
        body = 32768 - 7 * nrec - int(rng.integers(0, 7))  # a trailer of 0..6 bytes
        cuts = np.sort(rng.choice(np.arange(1, body), nrec - 1, replace=False)) if nrec > 1 else np.array([], int)
        sizes = np.diff(np.concatenate([[0], cuts, [body]]))
        recs += [rng.integers(0, 256, int(sz), dtype=np.uint8).tobytes() for sz in sizes]
    img = bytearray(oc.write_image(recs))
    ref0 = oc.walk(bytes(img))
    for i in np.flatnonzero(rng.random(len(ref0)) < 0.125):
        o, n = int(ref0["file_offset"][i]), int(ref0["length"][i])
        img[o + 7 + int(rng.integers(0, max(1, n)))] ^= 1 << int(rng.integers(0, 8))
    img = bytes(img) + bytes([0x11, 0x22, 0x33])  # a torn header at the end
    ref = oc.walk(img)
    assert int((ref["status"] == 1).sum()) > 100
    dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    for v in VERIFY_PATHS:
        compare_walk(gpu_ctx.verify_image(dimg, len(img), path=v), ref)


@pytest.mark.parametrize("plen", [123, 124, 126, 127, 128, 251, 254, 255, 256])
def test_verify_dense_word_stream_edges(gpu_ctx, plen):
    """Dense blocks of equal records whose CRC range (type + payload) is a
    multiple of 32 words or just off it, at every byte alignment of the type
    byte: the dense kernels' word-stream chunk boundaries (a 32-word record's
    last word takes a dword of the next chunk), a bit flipped in every 7th."""
    rng = np.random.default_rng(plen)
    recs = [rng.integers(0, 256, plen, dtype=np.uint8).tobytes() for _ in range(700)]
    img = bytearray(oc.write_image(recs))
    ref = oc.walk(bytes(img))
    for v in range(0, len(ref), 7):
        if ref["length"][v]:
            img[int(ref["file_offset"][v]) + 7 + int(rng.integers(0, int(ref["length"][v])))] ^= 0x10
    img = bytes(img)
    ref = oc.walk(img)
    dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    for v in VERIFY_PATHS:
        compare_walk(gpu_ctx.verify_image(dimg, len(img), path=v), ref)


def test_verify_small_records_dense(gpu_ctx):
    """Thousands of tiny records per block (many batches of the LDS record
    list, record starts/ends in every lane) in random bit positions."""
    rng = np.random.default_rng(15)
    recs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in rng.integers(0, 40, 20000)]
    img = oc.write_image(recs)
    dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    for v in VERIFY_PATHS:
        compare_walk(gpu_ctx.verify_image(dimg, len(img), path=v), oc.walk(img))


@pytest.mark.parametrize("rec_len", [24, 100, 124, 200])
def test_verify_multi_batch_lists(gpu_ctx, rec_len):
    """Blocks with 2..10 header-list batches of 64 records (the count pass
    lists 64, k_list_overflow the rest): bit flips in every batch, a zero
    record and a bad length deep in a block, all parity-checked."""
    rng = np.random.default_rng(rec_len)
    recs = [rng.integers(0, 256, rec_len + int(rng.integers(0, 8)), dtype=np.uint8).tobytes()
            for _ in range(6 * BLOCK_SIZE // (rec_len + 7))]
    img = bytearray(oc.write_image(recs))
    ref = oc.walk(bytes(img))
    # one flip per 37 records: every 64-record batch of every block gets some
    for v in range(5, len(ref) - 1, 37):
        off = int(ref["file_offset"][v]) + 7 + int(rng.integers(0, int(ref["length"][v])))
        img[off] ^= 1 << int(rng.integers(0, 8))
    # block 2: record #150 of the block becomes a zero record (ends the block)
    in_b2 = np.flatnonzero(ref["file_offset"] // BLOCK_SIZE == 2)
    if len(in_b2) > 150:
        z = int(ref["file_offset"][in_b2[150]])
        img[z:z + 7] = b"\0" * 7
    # block 4: record #100 gets a length past the block end
    in_b4 = np.flatnonzero(ref["file_offset"] // BLOCK_SIZE == 4)
    if len(in_b4) > 100:
        z = int(ref["file_offset"][in_b4[100]])
        img[z + 4:z + 6] = (0xFFF0).to_bytes(2, "little")
    img = bytes(img)
    dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    ref2 = oc.walk(img)
    for v in VERIFY_PATHS:
        compare_walk(gpu_ctx.verify_image(dimg, len(img), path=v), ref2)
    assert (ref2["status"] == 1).sum() > 10


def test_verify_batch_start_on_16_byte_boundary(gpu_ctx):
    """16-B records after a first record of every size 0..15: the first record
    of some list batch then starts exactly on a 16-B segment of a lane that has
    absorbed bytes of the previous batch's records (the fast path must not
    carry that register into the record; found by the dense append test)."""
    for period, l0 in [(p, l) for p in (32, 64) for l in range(16)]:
        # record k >= 1 starts at 7 + l0 + (k - 1) * period: with l0 = 3 the first
        # record of every 64- / 128-record batch starts 16 bytes before a
        # 512-B lane chunk ends (s = 4096 t - 16 for period 32)
        rng = np.random.default_rng(l0)
        recs = [rng.integers(0, 256, l0, dtype=np.uint8).tobytes()]
        recs += [rng.integers(0, 256, period - 7, dtype=np.uint8).tobytes() for _ in range(3000)]
        img = oc.write_image(recs)
        dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
        ref = oc.walk(img)
        for v in VERIFY_PATHS:
            compare_walk(gpu_ctx.verify_image(dimg, len(img), path=v), ref)


def _density_mix(seed, tail):
    """Blocks alternating dense (24..140-B records, > 64 per block) and sparse
    (2..30 KiB records) runs; `tail` picks the record sizes that end the image
    (a dense or a sparse partial last block)."""
    rng = np.random.default_rng(seed)
    recs = []
    for run in range(6):
        dense = run % 2 == 0
        total = 0
        while total < (BLOCK_SIZE if dense else 2 * BLOCK_SIZE):
            n = int(rng.integers(24, 140)) if dense else int(rng.integers(2000, 30000))
            recs.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
            total += n + 7
    for _ in range(200 if tail == "dense" else 1):
        n = int(rng.integers(10, 100)) if tail == "dense" else 9000
        recs.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    return oc.write_image(recs)


@pytest.mark.parametrize("tail", ["dense", "sparse"])
def test_verify_mixed_density(gpu_ctx, tail):
    """The production split (v3 over blocks with <= 64 records, the per-record
    dense kernel over the rest, partial last block by its density) on one
    image holding both kinds, with bit flips in both, vs the oracle."""
    img = bytearray(_density_mix(7 if tail == "dense" else 8, tail))
    ref = oc.walk(bytes(img))
    counts = np.bincount((ref["file_offset"] // BLOCK_SIZE).astype(np.int64))
    assert (counts > 64).any() and (counts <= 64).any()
    rng = np.random.default_rng(3)
    for v in rng.choice(len(ref) - 1, 40, replace=False):
        off = int(ref["file_offset"][v]) + 7 + int(rng.integers(0, max(1, int(ref["length"][v]))))
        if off < len(img):
            img[off] ^= 0x10
    img = bytes(img)
    ref = oc.walk(img)
    assert (ref["status"] == 1).sum() > 10
    dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    for v in VERIFY_PATHS:
        compare_walk(gpu_ctx.verify_image(dimg, len(img), path=v), ref)


@pytest.mark.parametrize("shift", [1, 4, 8, 12, 16])
def test_verify_unaligned_image_base(gpu_ctx, shift):
    """An image that does not start on a 16-B boundary: the split path reads
    aligned 16 B relative to the image, so such images take v3 (path 0 falls
    back to path 2); results unchanged."""
    img = _density_mix(11, "dense")
    buf = gpu_ctx.alloc(len(img) + 64)
    gpu_ctx.h2d(buf, np.frombuffer(img, dtype=np.uint8), dst_offset=shift)
    view = _View(buf, shift, len(img))
    ref = oc.walk(img)
    for v in VERIFY_PATHS:
        compare_walk(gpu_ctx.verify_image(view, len(img), path=v), ref)


def test_verify_base_offset_and_random_bytes(gpu_ctx):
    rng = np.random.default_rng(14)
    img = rng.integers(0, 256, 5 * BLOCK_SIZE + 123, dtype=np.uint8).tobytes()  # garbage headers
    dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    res = gpu_ctx.verify_image(dimg, len(img), base_offset=1 << 40)
    ref = oc.walk(img)
    ref["file_offset"] += np.uint64(1 << 40)
    compare_walk(res, ref)


def test_reader_checksum_gpu_golden(gpu_ctx, golden_index):
    for name in golden_index:
        img = golden_image(name)
        for window in (32768, 1 << 20):
            rd = log.Reader(env.MemorySequentialFile(img), checksum=True, gpu=gpu_ctx, window_bytes=window)
            try:
                got = list(rd)
            except RevelError as e:
                assert e.code == IO_ERROR
                got = "error"
            try:
                want = po.read_all(img, checksum=True)
            except po.CorruptionError:
                want = "error"
            assert got == want, (name, window)


def test_reader_checksum_gpu_c1(gpu_ctx):
    """Config C1 through the product writer and the GPU-verified reader."""
    words = po.splitmix64_np(np.uint64(0x5EED0001) ^ np.arange(10000, dtype=np.uint64), 512)
    recs = [words[i].tobytes() for i in range(10000)]
    f = env.MemoryWritableFile()
    w = log.Writer(f)
    for r in recs:
        w.add_record(r)
    img = f.contents()
    rd = log.Reader(env.MemorySequentialFile(img), checksum=True, gpu=gpu_ctx, window_bytes=8 << 20)
    got = list(rd)
    assert len(got) == 10000 and got == recs


def test_reader_continues_after_bad_record(gpu_ctx):
    recs = [bytes([i]) * 3000 for i in range(10)]
    img = bytearray(oc.write_image(recs))
    img[3 * 3007 + 100] ^= 0xFF
    rd = log.Reader(env.MemorySequentialFile(bytes(img)), checksum=True, gpu=gpu_ctx)
    out = []
    errors = 0
    while True:
        try:
            r = rd.read_record()
        except RevelError as e:
            assert e.code == IO_ERROR
            errors += 1
            continue
        if r is None:
            break
        out.append(r)
    assert errors == 1
    assert out == recs[:3] + recs[4:]


def drain(read_record, limit=100000):
    """Every result a reader yields until EOF, errors included as "E"."""
    out = []
    for _ in range(limit):
        try:
            r = read_record()
        except (RevelError, po.CorruptionError):
            out.append("E")
            continue
        if r is None:
            return out
        out.append(r)
    raise AssertionError("reader did not reach EOF")


@pytest.mark.parametrize("window", [32768, 1 << 20])
def test_reader_gpu_initial_offset_and_corruption(gpu_ctx, window):
    """GPU-verified reader vs the oracle LogReader: initial_offset at block
    edges, trailers and mid-record (SkipToInitialBlock + resync), with
    corrupted records in the stream."""
    rng = np.random.default_rng(71)
    recs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in rng.integers(0, 90000, 60)]
    img = bytearray(oc.write_image(recs))
    ref = oc.walk(bytes(img))
    for v in rng.choice(len(ref), 4, replace=False):
        if ref["length"][v] > 0:
            img[int(ref["file_offset"][v]) + 7 + int(rng.integers(0, int(ref["length"][v])))] ^= 0x08
    img = bytes(img)
    n = len(img)
    for off in [0, 1, 6, 7, 32761, 32762, 32767, 32768, 50000, 100003, n // 2, n - 1, n]:
        rd = log.Reader(env.MemorySequentialFile(img), checksum=True, gpu=gpu_ctx, initial_offset=off,
                        window_bytes=window)
        assert drain(rd.read_record) == drain(po.LogReader(img, True, off).read_record), off


# ---- end-to-end replay (host -> pinned ring -> HBM -> verify) ----
@pytest.mark.parametrize("window", [32768, 65536, 1 << 20])
def test_replay_memory_records_vs_oracle(gpu_ctx, golden_index, window):
    for name in golden_index:
        img = golden_image(name)
        ref = oc.walk(img)
        st = gpu_ctx.replay_memory(img, window_bytes=window, nbuffers=3, io_threads=3)
        bad = ref["status"] != 0
        assert st["bytes"] == len(img) and st["units"] == len(ref), name
        assert st["bad"] == int(bad.sum()), name
        want_first = int(ref["file_offset"][bad].min()) if bad.any() else 2**64 - 1
        assert st["first_bad_offset"] == want_first, name


def test_replay_full_blocks_and_file(gpu_ctx, tmp_path):
    blocks = oc.synth_full_blocks(300, seed=77)
    blocks[123, 5000] ^= 4
    blocks[250, 0] ^= 1
    img = blocks.tobytes()
    st = gpu_ctx.replay_memory(img, full_blocks=True, window_bytes=40 * BLOCK_SIZE, nbuffers=2, io_threads=4)
    assert (st["units"], st["bad"], st["first_bad_offset"]) == (300, 2, 123 * BLOCK_SIZE)
    path = str(tmp_path / "000007.log")
    with open(path, "wb") as f:
        f.write(img)
    st = gpu_ctx.replay_file(path, full_blocks=True, window_bytes=64 * BLOCK_SIZE, io_threads=4)
    assert (st["units"], st["bad"], st["first_bad_offset"]) == (300, 2, 123 * BLOCK_SIZE)
    # records mode on the same file: every block is one FULL record
    st = gpu_ctx.replay_file(path, offset=100 * BLOCK_SIZE, window_bytes=64 * BLOCK_SIZE, io_threads=2)
    assert (st["units"], st["bad"], st["first_bad_offset"]) == (200, 2, 123 * BLOCK_SIZE)


@pytest.mark.parametrize("io", ["pread", "mmap", "direct"])
def test_replay_file_io_methods(gpu_ctx, tmp_path, io):
    """Every input method sees the same bytes: a Zipf image with a ragged
    tail (not a page multiple, for O_DIRECT's rounded reads) and corruption."""
    from revel_amd._lib import NOT_SUPPORT
    rng = np.random.default_rng(61)
    img = bytearray(oc.write_image(zipf_image(rng, 3 << 20)))
    img = img[:len(img) - 1234]                  # torn tail inside the last block
    ref = oc.walk(bytes(img))
    for v in rng.choice(len(ref) - 1, 5, replace=False):
        img[int(ref["file_offset"][v]) + 7] ^= 0x20 if ref["length"][v] else 0
    img = bytes(img)
    want = oc.walk(img)
    path = str(tmp_path / "000009.log")
    with open(path, "wb") as f:
        f.write(img)
    bad = want["status"] != 0
    for off, win, th in [(0, 16 * BLOCK_SIZE, 3), (5 * BLOCK_SIZE, 7 * BLOCK_SIZE, 1), (0, 64 << 20, 8)]:
        try:
            st = gpu_ctx.replay_file(path, offset=off, window_bytes=win, io_threads=th, io=io)
        except RevelError as e:
            assert io == "direct" and e.code == NOT_SUPPORT  # file system refuses O_DIRECT: loud, not silent
            pytest.skip("O_DIRECT refused by this file system")
        sel = want["file_offset"] >= off
        assert st["bytes"] == len(img) - off
        assert st["units"] == int(sel.sum()) and st["bad"] == int((bad & sel).sum())
        first_bad = int(want["file_offset"][bad & sel].min()) if (bad & sel).any() else 2**64 - 1
        assert st["first_bad_offset"] == first_bad


# ---- device append framing (batch add_record) vs the oracle writer ----
@pytest.mark.parametrize("block_offset", [0, 1, 6, 7, 100, 32760, 32761, 32762, 32767, 32768])
def test_append_records_matches_writer(gpu_ctx, block_offset):
    rng = np.random.default_rng(block_offset + 1)
    sizes = list(rng.integers(0, 3000, 40)) + [0, 0, 32761, 32754, 70000, 1, 5] + list(rng.integers(0, 100, 300))
    recs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in sizes]
    blob = np.frombuffer(b"".join(recs), dtype=np.uint8)
    d = gpu_ctx.upload(blob if blob.size else np.zeros(1, np.uint8))
    img, n, bo = gpu_ctx.append_records(d, [len(r) for r in recs], block_offset)
    want = oc.write_image(recs, block_offset)
    w = po.LogWriter(block_offset=block_offset)
    for r in recs:
        w.add_record(r)
    assert bo == w.block_offset
    assert n == len(want)
    assert gpu_ctx.d2h(img, n).tobytes() == want


@pytest.mark.parametrize("block_offset", [0, 5, 32000])
def test_append_records_dense_blocks(gpu_ctx, block_offset):
    """~900 records per block: the framing header lists run in several
    128-record batches per whole block and 64-record batches in the lead and
    tail blocks."""
    rng = np.random.default_rng(block_offset + 77)
    recs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in rng.integers(0, 60, 4000)]
    blob = np.frombuffer(b"".join(recs), dtype=np.uint8)
    d = gpu_ctx.upload(blob)
    img, n, bo = gpu_ctx.append_records(d, [len(r) for r in recs], block_offset)
    want = oc.write_image(recs, block_offset)
    assert n == len(want)
    assert gpu_ctx.d2h(img, n).tobytes() == want


def test_append_records_c1_and_readback(gpu_ctx):
    words = po.splitmix64_np(np.uint64(0x5EED0001) ^ np.arange(10000, dtype=np.uint64), 512)
    d = gpu_ctx.upload(words.view(np.uint8).ravel())
    img, n, bo = gpu_ctx.append_records(d, [4096] * 10000, 0)
    assert n == 41038750
    host = gpu_ctx.d2h(img, n).tobytes()
    import hashlib
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "c1_records.npz"))
    assert hashlib.sha256(host).digest() == z["sha256"].tobytes()
    res = gpu_ctx.verify_image(img, n)
    assert len(res) == 11250 and (res["status"] == 0).all()


@pytest.mark.parametrize("n", [1, 2, 255, 1023, 1024, 1025, 4096, 131073, 1 << 20])
def test_exclusive_scan(gpu_ctx, n):
    from revel_amd._lib import check, lib
    rng = np.random.default_rng(n)
    a = rng.integers(0, 4682, n, dtype=np.uint32)
    din = gpu_ctx.upload(a)
    dout = gpu_ctx.alloc(4 * n)
    check(lib().revel_gpu_exclusive_scan_u32(gpu_ctx.handle, din.ptr, dout.ptr, n, None))
    gpu_ctx.sync()
    want = np.concatenate([[0], np.cumsum(a, dtype=np.uint64)[:-1]]).astype(np.uint32)
    assert np.array_equal(gpu_ctx.d2h(dout, 4 * n, np.uint32), want)


@pytest.mark.parametrize("nblocks", [1, 63, 64, 65, 1023, 1024, 1025, 4100])
def test_count_scan_records_and_general_scan(gpu_ctx, nblocks):
    """revel_gpu_count_scan_records (count + a scan whose first pass is the
    count pass's per-64-block sums) and the general revel_gpu_exclusive_scan_u32
    of the same counts, of a prefix of them, and of a counts buffer freed and
    reallocated (same size: a caching allocator hands back the same address)
    holding other data: all equal the oracle walk's counts scanned on the host.
    The general scan never takes the count pass's sums."""
    from revel_amd._lib import check, lib
    L = lib()
    rng = np.random.default_rng(nblocks)
    sizes = rng.integers(0, 3000, nblocks * 24)
    recs = [bytes(int(s)) for s in sizes]
    img = oc.write_image(recs)[:nblocks * BLOCK_SIZE - int(rng.integers(0, 100))]
    assert (len(img) + BLOCK_SIZE - 1) // BLOCK_SIZE == nblocks
    nb = (len(img) + BLOCK_SIZE - 1) // BLOCK_SIZE
    ref = oc.walk(img)
    want_counts = np.bincount(ref["file_offset"] // BLOCK_SIZE, minlength=nb).astype(np.uint32)
    want = np.concatenate([[0], np.cumsum(want_counts, dtype=np.uint64)[:-1]]).astype(np.uint32)
    d = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    counts, first, first2 = gpu_ctx.alloc(4 * nb), gpu_ctx.alloc(4 * nb), gpu_ctx.alloc(4 * nb)
    check(L.revel_gpu_count_scan_records(gpu_ctx.handle, d.ptr, len(img), counts.ptr, first.ptr, None))
    check(L.revel_gpu_exclusive_scan_u32(gpu_ctx.handle, counts.ptr, first2.ptr, nb, None))
    gpu_ctx.sync()
    assert np.array_equal(gpu_ctx.d2h(counts, 4 * nb, np.uint32), want_counts)
    assert np.array_equal(gpu_ctx.d2h(first, 4 * nb, np.uint32), want)
    assert np.array_equal(gpu_ctx.d2h(first2, 4 * nb, np.uint32), want)
    k = max(1, nb // 2)
    check(L.revel_gpu_count_records(gpu_ctx.handle, d.ptr, len(img), counts.ptr, None))
    check(L.revel_gpu_exclusive_scan_u32(gpu_ctx.handle, counts.ptr, first2.ptr, k, None))
    gpu_ctx.sync()
    assert np.array_equal(gpu_ctx.d2h(first2, 4 * k, np.uint32), want[:k])
    # count pass, free its counts, new counts buffer of the same size with other data, scan it
    check(L.revel_gpu_count_records(gpu_ctx.handle, d.ptr, len(img), counts.ptr, None))
    gpu_ctx.sync()
    counts.free()
    other = rng.integers(0, 4682, nb, dtype=np.uint32)
    counts2 = gpu_ctx.upload(other)
    check(L.revel_gpu_exclusive_scan_u32(gpu_ctx.handle, counts2.ptr, first2.ptr, nb, None))
    gpu_ctx.sync()
    want2 = np.concatenate([[0], np.cumsum(other, dtype=np.uint64)[:-1]]).astype(np.uint32)
    assert np.array_equal(gpu_ctx.d2h(first2, 4 * nb, np.uint32), want2)


# ---- device replay reassembly vs the oracle reader's event sequence ----
def check_reassembly(gpu_ctx, img, checksum=True):
    d = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    ev, payload, _ = gpu_ctx.reassemble(d, len(img), checksum=checksum)
    want = po.replay_events(img, checksum=checksum)
    assert len(ev) == len(want)
    for e, w in zip(ev, want):
        assert int(e["file_offset"]) == w[1]
        if w[0] == "record":
            assert e["status"] == 0
            p0 = int(e["payload_offset"])
            assert payload[p0:p0 + int(e["length"])].tobytes() == w[2]
        else:
            assert e["status"] != 0 and e["length"] == 0


@pytest.mark.parametrize("checksum", [True, False])
def test_reassemble_golden(gpu_ctx, golden_index, checksum):
    for name in golden_index:
        check_reassembly(gpu_ctx, golden_image(name), checksum)


def test_reassemble_gather_alignments(gpu_ctx):
    """Every payload length 0..99 plus 33-B multiples, so fragments start and
    end at every offset mod 16 in the image and in the gathered buffer."""
    rng = np.random.default_rng(32)
    sizes = list(range(100)) + [33 * k for k in range(1, 40)] + [32761, 32762, 40000, 65536]
    rng.shuffle(sizes)
    recs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in sizes]
    for boff in (0, 5):
        check_reassembly(gpu_ctx, oc.write_image(recs, boff) if boff == 0 else oc.write_image(recs), True)


def test_reassemble_mixed_corruption(gpu_ctx):
    rng = np.random.default_rng(31)
    recs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in rng.integers(0, 120000, 80)]
    img = bytearray(oc.write_image(recs))
    ref = oc.walk(bytes(img))
    for v in rng.choice(len(ref), 12, replace=False):       # flip payload / type bytes
        off = int(ref["file_offset"][v])
        if v % 3 == 0:
            img[off + 6] = 9                                  # unknown type
        elif ref["length"][v] > 0:
            img[off + 7 + int(rng.integers(0, int(ref["length"][v])))] ^= 0x40
    check_reassembly(gpu_ctx, bytes(img), True)
    check_reassembly(gpu_ctx, bytes(img), False)


# ---- device WriteBatch decode vs the oracle's LevelDB-correct iterate ----
from oracle import write_batch_oracle as wb  # noqa: E402
from revel_amd._lib import BATCH_NOT_RECORD  # noqa: E402


def check_batches(gpu_ctx, img, checksum=True):
    d = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    ev, payload, infos, ents = gpu_ctx.replay_batches(d, len(img), checksum=checksum)
    want = po.replay_events(img, checksum=checksum)
    assert len(ev) == len(want) == len(infos)
    total = 0
    for i, (e, w) in enumerate(zip(ev, want)):
        info = infos[i]
        assert int(info["first_entry"]) == total
        if w[0] == "error":
            assert info["status"] == BATCH_NOT_RECORD and info["nentries"] == 0
            continue
        st, seq, cnt, oents = wb.decode(w[2])
        assert int(info["status"]) == st, (i, st)
        assert int(info["nentries"]) == len(oents)
        if st != wb.TOO_SMALL:
            assert int(info["sequence"]) == seq and int(info["count"]) == cnt
        for k, (oseq, otype, okey, oval) in enumerate(oents):
            g = ents[total + k]
            assert int(g["batch"]) == i and int(g["sequence"]) == oseq and int(g["type"]) == otype
            k0, v0 = int(g["key_offset"]), int(g["value_offset"])
            assert payload[k0:k0 + int(g["key_len"])].tobytes() == okey
            assert payload[v0:v0 + int(g["value_len"])].tobytes() == oval
        total += len(oents)
    assert len(ents) == total
    return infos, ents


def test_decode_batches_random_log(gpu_ctx):
    from tests_gen import batch_log
    reps = batch_log(np.random.default_rng(41), 400, big_every=37)
    infos, ents = check_batches(gpu_ctx, oc.write_image(reps))
    assert (infos["status"] == 0).all() and len(ents) > 5000
    assert (np.diff(ents["sequence"].astype(np.int64)) == 1).all()  # one sequence per entry, db.rs:95-112


def test_decode_batches_malformed(gpu_ctx):
    from tests_gen import malformed_batches
    cases = malformed_batches()
    img = oc.write_image([r for _, r, _ in cases] * 3)
    infos, _ = check_batches(gpu_ctx, img)
    assert [int(s) for s in infos["status"][:len(cases)]] == [w for _, _, w in cases]


def test_decode_batches_after_log_corruption(gpu_ctx):
    from tests_gen import batch_log
    rng = np.random.default_rng(43)
    reps = batch_log(rng, 120, big_every=11)
    img = bytearray(oc.write_image(reps))
    ref = oc.walk(bytes(img))
    for v in rng.choice(len(ref), 6, replace=False):
        off = int(ref["file_offset"][v])
        if ref["length"][v] > 0:
            img[off + 7 + int(rng.integers(0, int(ref["length"][v])))] ^= 0x10
    infos, _ = check_batches(gpu_ctx, bytes(img), True)
    assert (infos["status"] == BATCH_NOT_RECORD).any()
    check_batches(gpu_ctx, bytes(img), False)  # unverified: corrupt batches decode or fail as bytes dictate


def test_decode_batches_many_batches(gpu_ctx):
    """9 000 small batches (35 scan tiles of the entry offsets) with malformed
    batches spread through the log and flipped payload bits, against the
    oracle; then a capacity cut two thirds in: infos complete, the total is
    reported, INVALID_ARGUMENT."""
    from tests_gen import batch_log, malformed_batches
    rng = np.random.default_rng(45)
    reps = batch_log(rng, 9000, max_entries=3, max_key=40, max_value=200, big_every=1501)
    cases = [r for _, r, _ in malformed_batches()]
    for k in range(0, len(cases) * 40, 40):
        reps.insert(k + 7, cases[(k // 40) % len(cases)])
    img = bytearray(oc.write_image(reps))
    ref = oc.walk(bytes(img))
    for v in rng.choice(len(ref), 25, replace=False):
        if ref["length"][v] > 0:
            img[int(ref["file_offset"][v]) + 7 + int(rng.integers(0, int(ref["length"][v])))] ^= 0x04
    img = bytes(img)
    infos, ents = check_batches(gpu_ctx, img)
    assert len(infos) > 8000 and (infos["status"] != 0).sum() > 10
    d = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    out, nl, pay, pb, _ = gpu_ctx.reassemble_device(d, len(img))
    with pytest.raises(RevelError):
        gpu_ctx.decode_batches_device(pay, pb, out, nl, entries_cap=len(ents) * 2 // 3)


def test_decode_batches_capacity(gpu_ctx):
    import ctypes
    from revel_amd._lib import INVALID_ARGUMENT, lib
    from tests_gen import batch_log
    img = oc.write_image(batch_log(np.random.default_rng(44), 20))
    d = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    out, nl, pay, pb, _ = gpu_ctx.reassemble_device(d, len(img))
    info, ent, ne = gpu_ctx.decode_batches_device(pay, pb, out, nl)
    with pytest.raises(RevelError) as e:
        gpu_ctx.decode_batches_device(pay, pb, out, nl, entries_cap=ne - 1)
    assert e.value.code == INVALID_ARGUMENT
    n = ctypes.c_uint64()
    with pytest.raises(RevelError):
        from revel_amd._lib import check
        check(lib().revel_gpu_decode_batches(gpu_ctx.handle, pay.ptr, pb, out.ptr, nl, info.ptr, ent.ptr, 3,
                                             ctypes.byref(n), None))
    assert n.value == ne


def test_gpu_entry_points_on_empty_inputs(gpu_ctx, tmp_path):
    """Zero-length images, files and record sets: no launch faults, empty results."""
    d = gpu_ctx.alloc(BLOCK_SIZE)
    assert len(gpu_ctx.verify_image(d, 0)) == 0
    ev, payload, phys = gpu_ctx.reassemble(d, 0)
    assert len(ev) == 0 and len(payload) == 0 and len(phys) == 0
    ev, payload, infos, ents = gpu_ctx.replay_batches(d, 0)
    assert len(infos) == 0 and len(ents) == 0
    path = str(tmp_path / "empty.log")
    open(path, "wb").close()
    for io in ("mmap", "pread"):
        st = gpu_ctx.replay_file(path, io=io)
        assert (st["bytes"], st["units"], st["bad"]) == (0, 0, 0)
    st = gpu_ctx.replay_memory(b"")
    assert (st["bytes"], st["units"]) == (0, 0)
    assert list(log.Reader(env.MemorySequentialFile(b""), checksum=True, gpu=gpu_ctx)) == []
    img, n, bo = gpu_ctx.append_records(d, [], block_offset=5)
    assert (n, bo) == (0, 5)
    # a lone trailer (< 7 bytes): no records
    assert len(gpu_ctx.verify_image(gpu_ctx.upload(np.zeros(6, np.uint8)), 6)) == 0


def test_property_random_streams_vs_oracle(gpu_ctx):
    """Hypothesis: random record streams (sizes clustered at the block-edge cases),
    optional bit flip and truncation -> device walk/verify, reassembly and the
    GPU reader all equal the oracle."""
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as hs
    edge = hs.sampled_from([0, 1, 2, 3, 4, 5, 6, 7, 8, 15, 16, 17, 32754, 32755, 32760, 32761, 32762, 32768, 65522])
    size = hs.one_of(edge, hs.integers(0, 70000))

    @settings(max_examples=40, deadline=None, suppress_health_check=list(HealthCheck), derandomize=True)
    @given(sizes=hs.lists(size, min_size=0, max_size=25), seed=hs.integers(0, 2**32 - 1),
           flip=hs.booleans(), cut=hs.integers(0, 40), off=hs.integers(0, 200000),
           window=hs.sampled_from([32768, 65536, 1 << 20]))
    def prop(sizes, seed, flip, cut, off, window):
        rng = np.random.default_rng(seed)
        img = bytearray(oc.write_image([rng.integers(0, 256, s, dtype=np.uint8).tobytes() for s in sizes]))
        if flip and len(img) > 0:
            img[int(rng.integers(0, len(img)))] ^= 1 << int(rng.integers(0, 8))
        if cut and len(img) > cut:
            img = img[:len(img) - cut]
        img = bytes(img)
        if img:
            d = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
            compare_walk(gpu_ctx.verify_image(d, len(img)), oc.walk(img))
            check_reassembly(gpu_ctx, img, True)
        rd = log.Reader(env.MemorySequentialFile(img), checksum=True, gpu=gpu_ctx, window_bytes=window)
        assert drain(rd.read_record) == drain(po.LogReader(img, True, 0).read_record)
        off = min(off, len(img))
        rd = log.Reader(env.MemorySequentialFile(img), checksum=True, gpu=gpu_ctx, initial_offset=off,
                        window_bytes=window)
        assert drain(rd.read_record) == drain(po.LogReader(img, True, off).read_record)

    prop()


def test_property_dense_streams_vs_oracle(gpu_ctx):
    """Hypothesis: dense streams (hundreds to thousands of small records, so
    blocks hold several header-list batches), a periodic tail that puts batch
    starts on fixed alignments, optional bit flips -> every verify path and
    the device append framing (at a random block offset) equal the oracle."""
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as hs

    @settings(max_examples=30, deadline=None, suppress_health_check=list(HealthCheck), derandomize=True)
    @given(n=hs.integers(100, 3000), maxlen=hs.integers(1, 120), period=hs.integers(0, 60),
           seed=hs.integers(0, 2**32 - 1), flips=hs.integers(0, 5), block_offset=hs.integers(0, 32768))
    def prop(n, maxlen, period, seed, flips, block_offset):
        rng = np.random.default_rng(seed)
        sizes = rng.integers(0, maxlen + 1, n)
        if period:
            sizes[n // 2:] = period
        recs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in sizes]
        img = bytearray(oc.write_image(recs))
        for _ in range(flips):
            img[int(rng.integers(0, len(img)))] ^= 1 << int(rng.integers(0, 8))
        img = bytes(img)
        d = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
        ref = oc.walk(img)
        for v in VERIFY_PATHS:
            compare_walk(gpu_ctx.verify_image(d, len(img), path=v), ref)
        blob = np.frombuffer(b"".join(recs) or b"\0", dtype=np.uint8)
        dp = gpu_ctx.upload(blob)
        fimg, fn, _ = gpu_ctx.append_records(dp, [len(r) for r in recs], block_offset)
        assert gpu_ctx.d2h(fimg, fn).tobytes() == oc.write_image(recs, block_offset)
        # the GPU reader (count -> scan -> verify per window) and the replay summary
        rd = log.Reader(env.MemorySequentialFile(img), checksum=True, gpu=gpu_ctx, window_bytes=65536)
        assert drain(rd.read_record) == drain(po.LogReader(img, True, 0).read_record)
        st = gpu_ctx.replay_memory(img, window_bytes=65536)
        assert (st["units"], st["bad"]) == (len(ref), int((ref["status"] != 0).sum()))

    prop()


def test_property_batch_decode_mutations(gpu_ctx):
    """Hypothesis: WriteBatch logs whose batch bytes are mutated before framing
    (valid log records carrying malformed batches) -> device decode == oracle."""
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as hs
    from tests_gen import batch_log

    @settings(max_examples=25, deadline=None, suppress_health_check=list(HealthCheck), derandomize=True)
    @given(seed=hs.integers(0, 2**32 - 1), nb=hs.integers(1, 30), nmut=hs.integers(0, 12),
           trunc=hs.integers(0, 3))
    def prop(seed, nb, nmut, trunc):
        rng = np.random.default_rng(seed)
        reps = [bytearray(r) for r in batch_log(rng, nb, max_entries=12, max_key=40, max_value=300)]
        for _ in range(nmut):
            r = reps[int(rng.integers(0, len(reps)))]
            if r:
                r[int(rng.integers(0, len(r)))] = int(rng.integers(0, 256))
        for _ in range(trunc):
            k = int(rng.integers(0, len(reps)))
            reps[k] = reps[k][:int(rng.integers(0, len(reps[k]) + 1))]
        check_batches(gpu_ctx, oc.write_image([bytes(r) for r in reps]))

    prop()


@pytest.mark.gpu
def test_c1_native_cabi_roundtrip():
    """Config C1 through the C-ABI from a native caller (tools/c1_native.cpp,
    built by __graft_entry__.build()): 10 000 x 4 KiB records appended and read
    back with checksum=1; the binary exits non-zero unless every record
    matches and the image is the 41 038 750-B image of SURVEY 8(a) a9."""
    import json
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "c1_native")
    assert os.path.exists(exe), "tools/c1_native not built (run __graft_entry__.build())"
    p = subprocess.run([exe, "1"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    out = json.loads(p.stdout)
    assert out["records_equal"] and out["image_bytes"] == 41038750


@pytest.mark.gpu
def test_reader_parked_window_buffers(gpu_ctx, golden_index):
    """Readers on one context reuse the window buffers the previous reader
    parked on it (same window size): sequential readers, overlapping readers
    (the second allocates its own) and a different window size all read every
    golden image exactly as the oracle reader does."""
    names = sorted(golden_index)
    want = {}
    for name in names:
        try:
            want[name] = po.read_all(golden_image(name), checksum=True)
        except po.CorruptionError:
            want[name] = "error"

    def read(rd):
        try:
            return list(rd)
        except RevelError as e:
            assert e.code == IO_ERROR
            return "error"

    for window in (65536, 65536, 1 << 20, 65536):
        for a, b in zip(names, names[1:] + names[:1]):
            ra = log.Reader(env.MemorySequentialFile(golden_image(a)), checksum=True, gpu=gpu_ctx, window_bytes=window)
            rb = log.Reader(env.MemorySequentialFile(golden_image(b)), checksum=True, gpu=gpu_ctx, window_bytes=window)
            assert read(rb) == want[b], (b, window)
            assert read(ra) == want[a], (a, window)
            del ra  # parks its buffers; rb's are freed (slot taken)
            del rb
            rc = log.Reader(env.MemorySequentialFile(golden_image(a)), checksum=True, gpu=gpu_ctx, window_bytes=window)
            assert read(rc) == want[a], (a, window)
            del rc


# ---- the reference's own vectors through the HIP kernels ----
def _kat():
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "kat.json")) as f:
        return json.load(f)


def kat_records_image(lead=0):
    """The five RFC 3720 B.4 vectors of crc.rs:50-76 framed as physical
    records: type byte = the vector's first byte, payload = the rest, so the
    record CRC crc32c(type || payload) (log_writer.rs:107-111) IS the vector's
    published CRC.  `lead` bytes of a zero-filled FULL record come first, to
    move the vectors across lane / row positions of the verify kernel."""
    import struct
    img = b""
    if lead:
        pad = bytes(lead)
        img += struct.pack("<IHB", po.mask(oc.extend(1, pad)), len(pad), 1) + pad
    want = []
    for v in _kat()["value"]:
        d = bytes.fromhex(v["data_hex"])
        want.append((len(img), v["crc"]))
        img += struct.pack("<IHB", po.mask(v["crc"]), len(d) - 1, d[0]) + d[1:]
    return img, want


@pytest.mark.parametrize("lead", [0, 1, 9, 57, 1000, 32768 - 7 - 206 - 7])
def test_rfc3720_kats_through_verify_kernel(gpu_ctx, lead):
    img, want = kat_records_image(lead)
    dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    res = gpu_ctx.verify_image(dimg, len(img))
    got = {int(r["file_offset"]): r for r in res}
    for off, kat_crc in want:
        r = got[off]
        assert int(r["computed_crc"]) == po.mask(kat_crc), (lead, off)
        assert po.unmask(int(r["computed_crc"])) == kat_crc
        assert int(r["status"]) == 0
    compare_walk(res, oc.walk(img))


ISCSI_HEX = "01c000000000000000000000000000001400000000000400000000140000001828000000000000000200000000000000"


def test_iscsi_pdu_and_hello_world_through_append_reader_verify(gpu_ctx):
    """crc.rs:66-74's 48-byte iSCSI PDU starts with 0x01 (FULL): appended as a
    47-byte record on the device, its stored header must be
    mask(0xd9963a56) LE, len 47, type 1; the GPU verify and the GPU-verified
    reader (explicit and default context) must accept it.  Same for the
    hello-world image of log_reader.rs:231."""
    pdu = bytes.fromhex(ISCSI_HEX)
    assert pdu[0] == 1
    hello_img = bytes(_kat()["hello_world_image"])
    for payload, kat_crc, golden in [(pdu[1:], 0xD9963A56, None), (b"hello world", None, hello_img)]:
        d = gpu_ctx.upload(np.frombuffer(payload, dtype=np.uint8))
        img_d, n, bo = gpu_ctx.append_records(d, [len(payload)], 0)
        img = gpu_ctx.d2h(img_d, n).tobytes()
        assert n == 7 + len(payload) and bo == n
        stored = int.from_bytes(img[:4], "little")
        if kat_crc is not None:
            assert stored == po.mask(kat_crc)
        if golden is not None:
            assert img == golden
        assert img[4:7] == bytes([len(payload) & 0xFF, len(payload) >> 8, 1])
        res = gpu_ctx.verify_image(img_d, n)
        assert len(res) == 1 and int(res["computed_crc"][0]) == stored and int(res["status"][0]) == 0
        for ctx in (gpu_ctx, None):
            rd = log.Reader(env.MemorySequentialFile(img), True, 0, gpu=ctx)
            assert list(rd) == [payload]


# ---- the drop-in: caller files + the 3-argument Reader::new ----
class _PySeq:
    def __init__(self, data, chunk=1 << 30):
        self.data, self.pos, self.chunk = data, 0, chunk

    def read(self, n):
        d = self.data[self.pos:self.pos + min(n, self.chunk)]
        self.pos += len(d)
        return d

    def skip(self, n):
        self.pos += n


def test_three_arg_reader_callbacks_every_golden(golden_index):
    """Reader::new(Box<dyn SequentialFile>, true, 0) (log_reader.rs:62): a
    caller-implemented file, checksum on, NO explicit context -- the thread's
    default context verifies on the GPU -- for every golden image."""
    for name in sorted(golden_index):
        img = golden_image(name)
        for chunk in (1 << 30, 4096):
            rd = log.Reader(env.CallbackSequentialFile(_PySeq(img, chunk)), True, 0)
            try:
                got = list(rd)
            except RevelError as e:
                assert e.code == IO_ERROR
                got = "error"
            try:
                want = po.read_all(img, checksum=True)
            except po.CorruptionError:
                want = "error"
            assert got == want, (name, chunk)


def test_read_record_into_gpu_verified_every_golden(golden_index):
    """read_record_into (the caller's scratch, log_reader.rs:76) on the
    3-argument GPU-verified reader: the same events as read_record, errors
    included, on every golden image through caller files."""
    from test_host_capi import reader_events
    for name in sorted(golden_index):
        img = golden_image(name)
        for chunk in (1 << 30, 4096):
            for start in (0, 64):
                a = log.Reader(env.CallbackSequentialFile(_PySeq(img, chunk)), True, 0)
                b = log.Reader(env.CallbackSequentialFile(_PySeq(img, chunk)), True, 0)
                assert reader_events(a, into=bytearray(start)) == reader_events(b), (name, chunk, start)


def test_callback_writer_then_three_arg_reader_roundtrip():
    """Writer::new(Rc<RefCell<dyn WritableFile>>) on a caller file, read back
    through Reader::new(file, true, initial_offset) with GPU verification."""
    class W:
        def __init__(self):
            self.b = bytearray()

        def append(self, d):
            self.b += d

        def flush(self):
            pass

        def close(self):
            pass

        def sync(self):
            pass
    rng = np.random.default_rng(99)
    recs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in rng.integers(0, 100000, 50)]
    w = W()
    wr = log.Writer(env.CallbackWritableFile(w))
    for r in recs:
        wr.add_record(r)
    img = bytes(w.b)
    assert img == oc.write_image(recs)
    for off in (0, 40000, len(img) // 2):
        rd = log.Reader(env.CallbackSequentialFile(_PySeq(img, 10000)), True, off)
        assert drain(rd.read_record) == drain(po.LogReader(img, True, off).read_record), off


def test_context_freed_before_its_reader():
    """revel_gpu_context_free while a reader still uses the context defers
    the release to the reader's free (was a use-after-free)."""
    from revel_amd import gpu as G
    rng = np.random.default_rng(5)
    recs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in rng.integers(0, 70000, 30)]
    img = oc.write_image(recs)
    for _ in range(3):
        ctx = G.GpuContext(0)
        rd = log.Reader(env.MemorySequentialFile(img), checksum=True, gpu=ctx, window_bytes=65536)
        first = rd.read_record()
        ctx.close()  # deferred: the reader pins the context
        assert [first] + list(rd) == recs
        del rd  # the last reader's release destroys the context
    ctx = G.GpuContext(0)
    rd = log.Reader(env.MemorySequentialFile(img), checksum=True, gpu=ctx)
    assert list(rd) == recs
    assert ctx.trim() is None
    del rd
    ctx.close()


# ---- one WAL across several GPU contexts (SURVEY 8(e), config C5 on N GPUs) ----
@pytest.fixture(scope="module")
def shard_ctxs():
    from revel_amd import gpu as G
    ctxs = [G.GpuContext(0) for _ in range(3)]
    yield ctxs
    for c in ctxs:
        c.close()


def _shard_images():
    rng = np.random.default_rng(123)
    imgs = {}
    recs = zipf_image(rng, 6 << 20)
    img = bytearray(oc.write_image(recs))
    ref = oc.walk(bytes(img))
    for v in rng.choice(np.flatnonzero(ref["length"] > 0), 25, replace=False):
        img[int(ref["file_offset"][v]) + 7 + int(rng.integers(0, int(ref["length"][v])))] ^= 0x40
    imgs["zipf_flips"] = bytes(img)
    big = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in rng.integers(0, 400000, 30)]
    imgs["big_records"] = oc.write_image(big)
    img = bytearray(oc.write_image(big[:12]))
    r2 = oc.walk(bytes(img))
    for v in rng.choice(len(r2), 4, replace=False):
        img[int(r2["file_offset"][v]) + 6] = 9  # unknown types inside fragments
    imgs["bad_types_torn"] = bytes(img[:-3])
    return imgs


def test_replay_sharded_matches_reader(shard_ctxs, golden_index, tmp_path):
    """revel_gpu_replay_sharded over 1..3 contexts (threads) on device 0: the
    stitched event stream equals the oracle Reader over the whole WAL
    (checksum on) for golden, corrupted Zipf, multi-block and torn images;
    the summary agrees; a file source gives the same result."""
    from revel_amd import shard
    imgs = {n: golden_image(n) for n in golden_index}
    imgs.update(_shard_images())
    for name, img in imgs.items():
        want = drain(po.LogReader(img, True).read_record)
        ref = oc.walk(img)
        for n in (1, 2, 3):
            r = shard.ShardedReplay(shard_ctxs[:n], image=img, checksum=True, window_bytes=65536, io_threads=2)
            got = drain(r.read_record)
            assert got == want, (name, n)
            s = r.summary()
            assert s["physical"] == len(ref) and s["bytes"] == len(img), (name, n)
            assert s["bad"] == int((ref["status"] != 0).sum()), (name, n)
            assert s["records"] == sum(1 for w in want if w != "E"), (name, n)
            assert s["errors"] == sum(1 for w in want if w == "E"), (name, n)
            r.close()
    img = imgs["zipf_flips"]
    path = str(tmp_path / "000007.log")
    with open(path, "wb") as f:
        f.write(img)
    r = shard.ShardedReplay(shard_ctxs, path=path, checksum=True, window_bytes=1 << 20)
    assert drain(r.read_record) == drain(po.LogReader(img, True).read_record)


def test_wal_shards_per_rank_and_stitch(shard_ctxs):
    """The one-process-per-GPU shape: each 'rank' loads its range
    (revel_gpu_wal_shard_load), exports its boundary blob, and one stitch
    of the blobs gives the whole-WAL counts; device verdicts per shard equal
    the oracle walk of that range."""
    from revel_amd import shard
    img = _shard_images()["big_records"]
    want = drain(po.LogReader(img, True).read_record)
    ref = oc.walk(img)
    for n in (2, 3):
        ranges = shard.block_ranges(len(img), n)
        shards = [shard.WalShard(shard_ctxs[k], s, e - s, image=img, window_bytes=3 * BLOCK_SIZE)
                  for k, (s, e) in enumerate(ranges)]
        for sh, (s, e) in zip(shards, ranges):
            inf = sh.info()
            part = ref[(ref["file_offset"] >= s) & (ref["file_offset"] < e)]
            assert inf["physical"] == len(part) and inf["bad"] == int((part["status"] != 0).sum())
        st = shard.Stitch([sh.boundary() for sh in shards])
        s = st.summary()
        assert s["records"] == len(want) and s["stitched"] >= 1
        assert s["payload_bytes"] == sum(len(w) for w in want)
        # the stitched payloads are among the whole-file records
        for _, p, _ in st.records():
            assert p in want


def test_replay_sharded_verify_mode_and_context_lifetime(shard_ctxs):
    from revel_amd import gpu as G
    from revel_amd import shard
    img = _shard_images()["zipf_flips"]
    ref = oc.walk(img)
    r = shard.ShardedReplay(shard_ctxs[:2], image=img, checksum=True, read=False)
    s = r.summary()
    assert s["physical"] == len(ref) and s["bad"] == 25 and s["records"] == 0
    with pytest.raises(RevelError):
        r.read_record()  # VERIFY keeps no logical records
    # a shard pins its context: closing the context first is deferred
    ctx = G.GpuContext(0)
    sh = shard.WalShard(ctx, 0, len(img) // BLOCK_SIZE * BLOCK_SIZE, image=img)
    ctx.close()
    assert sh.info()["physical"] > 0
    sh.close()
    with pytest.raises(RevelError):
        shard.ShardedReplay([shard_ctxs[0], shard_ctxs[0]], image=img)

@pytest.mark.parametrize("tail", [1, 3, 7, 11])
@pytest.mark.parametrize("slack", [0, 2, 6])
def test_dense_block_then_tiny_tail(gpu_ctx, tail, slack):
    """a dense block (> 64 records) whose last record ends 0-6 bytes
    before the block end, followed by a final block of 1..11 bytes (a torn
    header): the dense kernel's 16-B loads near that block's end may reach
    past the image end, so they must be range-checked per dword; every verify
    path equals the oracle walk, with a flipped bit in the dense block."""
    rng = np.random.default_rng(1000 * tail + slack)
    nrec = 150
    body = 32768 - 7 * nrec - slack
    cuts = np.sort(rng.choice(np.arange(1, body), nrec - 1, replace=False))
    sizes = np.diff(np.concatenate([[0], cuts, [body]]))
    recs = [rng.integers(0, 256, int(sz), dtype=np.uint8).tobytes() for sz in sizes]
    img = bytearray(oc.write_image(recs))
    img += bytes(slack)  # the writer leaves the last block's trailer out
    assert len(img) == 32768
    ref0 = oc.walk(bytes(img))
    last = int(ref0["file_offset"][-1]) + 7
    img[last + int(rng.integers(0, max(1, int(ref0["length"][-1]))))] ^= 0x40
    img += bytes(rng.integers(0, 256, tail, dtype=np.uint8))
    img = bytes(img)
    ref = oc.walk(img)
    assert int((ref["status"] == 1).sum()) == 1
    dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    for v in VERIFY_PATHS:
        compare_walk(gpu_ctx.verify_image(dimg, len(img), path=v), ref)


def test_record_index_guard_rejects_u32_wrap(gpu_ctx):
    """Record indices (d_first) are u32: the count calls and the shard loader
    refuse an image whose physical records reach 2^32 (an image of empty
    records past ~28 GiB) instead of wrapping -- the guard on a synthetic
    counts array: 917 535 blocks x 4681 records = 4 294 981 335 > 2^32 - 1,
    then 14 040 records fewer = exactly 2^32 - 1, which fits."""
    from revel_amd._lib import lib
    L = lib()
    nb = 917535
    counts = gpu_ctx.upload(np.full(nb, 4681, dtype=np.uint32))
    with pytest.raises(RevelError, match="u32"):
        check(L.revel_debug_check_record_index(gpu_ctx.handle, counts.ptr, nb))
    gpu_ctx.h2d(counts, np.array([0, 0, 3], dtype=np.uint32))
    check(L.revel_debug_check_record_index(gpu_ctx.handle, counts.ptr, nb))
    # images that cannot wrap (at most 917 503 blocks) are not checked (no synchronisation)
    gpu_ctx.h2d(counts, np.full(8, 0xFFFFFFFF, dtype=np.uint32))
    check(L.revel_debug_check_record_index(gpu_ctx.handle, counts.ptr, 917503))
    counts.free()


def _block_of_records(rng, nrec, body):
    """nrec records whose payloads fill `body` bytes (random cut points)."""
    cuts = np.sort(rng.choice(np.arange(1, body), nrec - 1, replace=False))
    sizes = np.diff(np.concatenate([[0], cuts, [body]]))
    return [rng.integers(0, 256, int(sz), dtype=np.uint8).tobytes() for sz in sizes]


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_dense_chunks_markers_and_reuse(gpu_ctx, seed):
    """Dense-block shapes against the oracle (written for round 5's
    k_verify_dense_chunks, now an experiment; its path re-runs this test in
    test_experiments_gpu.py): images that mix 120-220-record blocks with capture-dense blocks (a run of 20-40-B records,
    more than three record starts in some 128-B chunk: marked in slot 256),
    blocks past 256 records, sparse blocks, a zero record and a bad length
    ending dense blocks, and bit flips everywhere.  Two different images
    verified in turn on the SAME context (stale slot-256 values of the first
    must not change the second's results), every verify path."""
    rng = np.random.default_rng(4242 + seed)

    def image(order):
        recs = []
        for kind in order:
            if kind == "chunks":    # 120-220 records over a block: k_verify_dense_chunks
                n = int(rng.integers(120, 220))
                recs += _block_of_records(rng, n, 32768 - 7 * n)
            elif kind == "capdense":  # 90 records, a run of 30 tiny ones inside
                n = 90
                tiny = [rng.integers(0, 256, int(rng.integers(20, 40)), dtype=np.uint8).tobytes() for _ in range(30)]
                rest = _block_of_records(rng, n - 30, 32768 - 7 * n - sum(len(t) for t in tiny))
                recs += rest[:20] + tiny + rest[20:]
            elif kind == "over256":
                n = 300
                recs += _block_of_records(rng, n, 32768 - 7 * n)
            else:  # sparse
                n = 20
                recs += _block_of_records(rng, n, 32768 - 7 * n)
        img = bytearray(oc.write_image(recs))
        ref = oc.walk(bytes(img))
        for v in range(3, len(ref) - 1, 29):  # flips in every kind of block
            off = int(ref["file_offset"][v]) + 7 + int(rng.integers(0, max(1, int(ref["length"][v]))))
            img[off] ^= 1 << int(rng.integers(0, 8))
        # a dense-chunks block ends early twice: a zero record, a length past the block end
        for k, kind in enumerate(order):
            if kind != "chunks":
                continue
            inb = np.flatnonzero(ref["file_offset"] // BLOCK_SIZE == k)
            if len(inb) > 100:
                z = int(ref["file_offset"][inb[int(rng.integers(70, 100))]])
                if rng.integers(0, 2):
                    img[z:z + 7] = b"\0" * 7
                else:
                    img[z + 4:z + 6] = (0xFFF0).to_bytes(2, "little")
                break
        return bytes(img)

    kinds = ["chunks", "capdense", "chunks", "over256", "sparse", "chunks", "capdense", "chunks"]
    imgs = [image(kinds), image(kinds[::-1])]
    for img in imgs:
        ref = oc.walk(img)
        dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
        for v in VERIFY_PATHS:
            compare_walk(gpu_ctx.verify_image(dimg, len(img), path=v), ref)
        dimg.free()
