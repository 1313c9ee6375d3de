"""GPU parity at BASELINE.json's full sizes, through size-independent
properties (the oracle checks every value where it can in seconds):

* C2: 1 M blocks = 32 GiB synthesised + framed on the device, every masked
  CRC checked against the C oracle (SSE4.2 restatement, cross-checked with the
  bytewise one on a sample) over the whole 32 GiB, then 257 blocks corrupted
  -> exactly those flagged;
* C3: a 1 GiB Zipf image framed on the device (revel_gpu_append_records),
  verified: every record's offset, length, type, stored and computed CRC and
  status equal to the C oracle's walk of the same bytes copied back (SSE4.2
  over the whole GiB, bytewise on the first 16 MiB), record count = the host
  fragment layout; 1 000 payload bit flips -> exactly those records flagged and
  the oracle walk of the flipped bytes equal again;
* one WAL across 3 contexts at 256 MiB: the sharded replay's stream equals the
  oracle Reader's, and its counts equal the whole-image verify's."""
import numpy as np
import pytest

from revel_amd import BLOCK_SIZE, shard
from revel_amd._lib import RevelError
from oracle import crc32c_oracle as po
from oracle import oracle_c as oc

pytestmark = pytest.mark.gpu


def test_c2_full_size_every_crc_vs_oracle(gpu_ctx):
    n = 1 << 20
    d = gpu_ctx.alloc(n * BLOCK_SIZE)
    gpu_ctx.synth_full_blocks(d, n, seed=0x5EED0002)
    m, ok = gpu_ctx.alloc(4 * n), gpu_ctx.alloc(n)
    gpu_ctx.crc_full_blocks(d, n, m, ok)
    gpu_ctx.sync()
    got = gpu_ctx.d2h(m, 4 * n, np.uint32)
    assert gpu_ctx.d2h(ok, n).all()
    chunk = 32768  # 1 GiB of blocks per host pass
    for b0 in range(0, n, chunk):
        host = gpu_ctx.d2h(d, chunk * BLOCK_SIZE, src_offset=b0 * BLOCK_SIZE).reshape(chunk, BLOCK_SIZE)
        want = oc.full_block_crcs(host, "sse42")
        assert np.array_equal(got[b0:b0 + chunk], want), b0
        if b0 == 0:
            assert np.array_equal(want[:256], oc.full_block_crcs(host[:256], "bytewise"))
        # the stored header is what the writer would have stored
        assert np.array_equal(host[:, 0:4].copy().view(np.uint32).ravel(), want)
    # the same 32 GiB through the C3 record path (count -> scan -> verify): 16 384
    # 64-block chunks, so every count-pass wave walks several (kernel grid 4 096
    # waves), the scan runs over 512 tiles, and the u32 record-index guard sums
    # the counts (> 917 503 blocks); every block is one FULL record of 32 761 B
    res = gpu_ctx.verify_image(d, n * BLOCK_SIZE)
    assert len(res) == n
    assert np.array_equal(res["file_offset"], np.arange(n, dtype=np.uint64) * BLOCK_SIZE)
    assert (res["length"] == BLOCK_SIZE - 7).all() and (res["type"] == 1).all()
    assert np.array_equal(res["stored_crc"], got) and np.array_equal(res["computed_crc"], got)
    assert (res["status"] == 0).all()
    rng = np.random.default_rng(2)
    bad = np.sort(rng.choice(n, 257, replace=False))
    for b in bad:
        pos = int(rng.integers(6, BLOCK_SIZE))
        byte = gpu_ctx.d2h(d, 1, src_offset=int(b) * BLOCK_SIZE + pos)
        gpu_ctx.h2d(d, byte ^ np.uint8(1 << int(rng.integers(0, 8))), dst_offset=int(b) * BLOCK_SIZE + pos)
    gpu_ctx.crc_full_blocks(d, n, m, ok)
    gpu_ctx.sync()
    assert np.array_equal(np.flatnonzero(gpu_ctx.d2h(ok, n) == 0), bad)
    res = gpu_ctx.verify_image(d, n * BLOCK_SIZE)
    assert np.array_equal(np.flatnonzero(res["status"] != 0), bad)
    assert (res["status"][bad] == 1).all()  # REVEL_REC_BAD_CHECKSUM
    assert np.array_equal(res["stored_crc"], got)


def test_c3_full_size_append_verify_roundtrip(gpu_ctx):
    rng = np.random.default_rng(0x5EED0003)
    k = np.arange(1, 513)
    p = k ** -1.1
    p /= p.sum()
    target = 1 << 30
    sizes = (64 * rng.choice(k, size=target // 3000 + 4096, p=p)).astype(np.uint64)
    sizes = sizes[:int(np.searchsorted(np.cumsum(sizes + 7), target))]
    nb_pay = (int(sizes.sum()) + BLOCK_SIZE - 1) // BLOCK_SIZE
    pay = gpu_ctx.alloc(nb_pay * BLOCK_SIZE)
    gpu_ctx.synth_full_blocks(pay, nb_pay, seed=0x5EED0003)
    img, n, bo = gpu_ctx.append_records(pay, sizes)
    # the host layout (log_writer.rs:58-97) predicts the image size and the fragment count
    assert n == po_framed_size(sizes)
    nfrag = po_fragment_count(sizes)
    res = gpu_ctx.verify_image(img, n)
    assert len(res) == nfrag
    assert (res["status"] == 0).all()
    assert int(res["length"].astype(np.uint64).sum()) == int(sizes.sum())
    # every record against the C oracle's walk of the same 1 GiB (SSE4.2 CRC:
    # seconds; the bytewise table CRC -- the reference crate's algorithm class --
    # on the first 16 MiB)
    host = gpu_ctx.d2h(img, n)
    assert_walk_equal(res, oc.walk(host, "sse42"))
    head = 512 * BLOCK_SIZE
    assert_walk_equal(res[res["file_offset"] < head], oc.walk(host[:head], "bytewise"))
    # 1 000 payload bit flips -> exactly those records flagged, every field
    # again equal to the oracle's walk of the flipped image
    cand = np.flatnonzero(res["length"] > 0)
    victims = np.sort(rng.choice(cand, 1000, replace=False))
    for v in victims:
        off = int(res["file_offset"][v]) + 7 + int(rng.integers(0, int(res["length"][v])))
        byte = gpu_ctx.d2h(img, 1, src_offset=off)
        gpu_ctx.h2d(img, byte ^ np.uint8(0x20), dst_offset=off)
        host[off] ^= np.uint8(0x20)
    res2 = gpu_ctx.verify_image(img, n)
    assert np.array_equal(np.flatnonzero(res2["status"] != 0), victims)
    assert (res2["status"][victims] == 1).all()
    assert np.array_equal(gpu_ctx.d2h(img, n), host)
    assert_walk_equal(res2, oc.walk(host, "sse42"))


def assert_walk_equal(res, ref):
    """GPU verify results == the oracle walk, field by field (computed CRC
    only where the record's length is valid: the oracle leaves it 0 as the
    kernels do)."""
    assert len(res) == len(ref)
    for f in ("file_offset", "length", "type", "stored_crc", "computed_crc", "status"):
        assert np.array_equal(res[f], ref[f].astype(res[f].dtype)), f


def po_framed_size(sizes):
    import revel_amd
    return revel_amd.lib().revel_log_framed_size(np.ascontiguousarray(sizes, dtype=np.uint64).ctypes.data,
                                                 len(sizes), 0)


def po_fragment_count(sizes):
    """Physical records n successive add_record calls emit (log_writer.rs:58-97)."""
    boff, count = 0, 0
    for s in sizes.tolist():
        left, begin = s, True
        while True:
            if BLOCK_SIZE - boff < 7:
                boff = 0
            avail = BLOCK_SIZE - boff - 7
            frag = min(left, avail)
            count += 1
            boff += 7 + frag
            left -= frag
            if left == 0:
                break
    return count


def test_sharded_replay_256mib_three_contexts():
    from revel_amd import gpu as G
    rng = np.random.default_rng(77)
    k = np.arange(1, 513)
    p = k ** -1.1
    p /= p.sum()
    sizes = 64 * rng.choice(k, size=70000, p=p)
    blob = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8).tobytes()
    recs, off = [], 0
    for s in sizes:
        recs.append(blob[off:off + int(s)])
        off += int(s)
    img = bytearray(oc.write_image(recs))
    ref = oc.walk(bytes(img))
    for v in rng.choice(np.flatnonzero(ref["length"] > 0), 50, replace=False):
        img[int(ref["file_offset"][v]) + 7] ^= 1
    img = bytes(img)
    ctxs = [G.GpuContext(0) for _ in range(3)]
    try:
        r = shard.ShardedReplay(ctxs, image=img, checksum=True, window_bytes=8 << 20)
        got = []
        errors = 0
        while True:
            try:
                x = r.read_record()
            except RevelError:
                errors += 1
                continue
            if x is None:
                break
            got.append(x)
        rd = po.LogReader(img, True)
        want, werr = [], 0
        while True:
            try:
                x = rd.read_record()
            except po.CorruptionError:
                werr += 1
                continue
            if x is None:
                break
            want.append(x)
        assert got == want and errors == werr == 50
        s = r.summary()
        assert s["physical"] == len(ref) and s["bad"] == 50 and s["records"] == len(want)
        assert s["stitched"] >= 1
        r.close()
    finally:
        for c in ctxs:
            c.close()


def test_c3_small_shape_vs_oracle(gpu_ctx):
    """bench.py's c3_small image (64..256-B records, ~200 per block: every
    block takes the dense path; db_bench-shaped puts through DB::write ->
    add_record, db.rs:95-120, log_writer.rs:58-97) built by the bench's own
    helper at 256 MiB: every record against the C oracle's walk, then 500
    payload flips -> exactly those flagged and the walk equal again."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    img, n, nrec = bench.c3_image(gpu_ctx, "small", 0x5EED0005, 0.25)
    res = gpu_ctx.verify_image(img, n)
    assert len(res) == po_fragment_count(bench.c3_sizes("small", 0x5EED0005, int(0.25 * (1 << 30))))
    assert (res["status"] == 0).all() and len(res) >= nrec
    host = gpu_ctx.d2h(img, n)
    assert_walk_equal(res, oc.walk(host, "sse42"))
    assert_walk_equal(res[res["file_offset"] < 64 * BLOCK_SIZE], oc.walk(host[:64 * BLOCK_SIZE], "bytewise"))
    # ~200 records per whole block: the dense path, not the rows kernel
    per_block = np.bincount((res["file_offset"] // BLOCK_SIZE).astype(np.int64))
    assert np.median(per_block) > 64
    rng = np.random.default_rng(5)
    victims = np.sort(rng.choice(np.flatnonzero(res["length"] > 0), 500, replace=False))
    for v in victims:
        off = int(res["file_offset"][v]) + 7 + int(rng.integers(0, int(res["length"][v])))
        host[off] ^= np.uint8(0x08)
        gpu_ctx.h2d(img, host[off:off + 1], dst_offset=off)
    res2 = gpu_ctx.verify_image(img, n)
    assert np.array_equal(np.flatnonzero(res2["status"] != 0), victims)
    assert_walk_equal(res2, oc.walk(host, "sse42"))
    img.free()


def test_dense_batches_across_blocks_far_apart(gpu_ctx):
    """The dense kernel packs a wave's 64-record batches across its dense
    blocks only while they lie < kDensePackSpan (65 532) blocks apart (its
    buffer offsets stay in 31 bits).  A 2.2 GB image of full-type blocks with
    two dense blocks of 306 records (past the 256-entry header list: the
    overflow entries too) 69 632 blocks apart -- wave 0's consecutive dense
    blocks when the dense grid has 4 096 waves (256 CUs), else still two
    dense blocks far apart -- plus a third 4 096 blocks after the first (packed
    with it): every record against the C oracle's walk."""
    nb = 69633
    d = gpu_ctx.alloc(nb * BLOCK_SIZE)
    gpu_ctx.synth_full_blocks(d, nb, seed=0x5EED0009)
    rng = np.random.default_rng(9)
    for b in (0, 4096, nb - 1):
        recs = [rng.integers(0, 256, 100, dtype=np.uint8).tobytes() for _ in range(305)]
        recs.append(rng.integers(0, 256, 126, dtype=np.uint8).tobytes())
        blk = np.frombuffer(oc.write_image(recs), dtype=np.uint8)
        assert len(blk) == BLOCK_SIZE  # 305 * 107 + 133: the block exactly full
        gpu_ctx.h2d(d, blk, dst_offset=b * BLOCK_SIZE)
    gpu_ctx.sync()
    n = nb * BLOCK_SIZE
    res = gpu_ctx.verify_image(d, n)
    host = gpu_ctx.d2h(d, n)
    ref = oc.walk(host, "sse42")
    assert len(ref) == nb - 3 + 3 * 306
    assert_walk_equal(res, ref)
    assert (res["status"] == 0).all()
    # a flipped payload byte in each dense block's last record is found
    for b in (0, nb - 1):
        host_off = b * BLOCK_SIZE + BLOCK_SIZE - 1
        byte = host[host_off:host_off + 1] ^ np.uint8(0x40)
        gpu_ctx.h2d(d, byte, dst_offset=host_off)
    res2 = gpu_ctx.verify_image(d, n)
    bad = np.flatnonzero(res2["status"] != 0)
    assert len(bad) == 2 and (res2["file_offset"][bad] // BLOCK_SIZE).tolist() == [0, nb - 1]
    d.free()


@pytest.mark.parametrize("shape", ["zipf", "small"])
def test_bench_c3_legs_report_both_timings(gpu_ctx, shape, monkeypatch):
    """bench.py's c3 / c3_small legs on a 64 MiB image (single process): the
    steady-state `ms` (calls queued back to back) and the isolated per-call
    median are both reported, every record verifies, and the rate is the
    image over the steady-state time."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    r = bench.c3_records(gpu_ctx, bench.Dist(), 1 / 16, iters=3, shape=shape)
    assert r["bad_records"] == 0 and r["physical_records_rank0"] > 0
    assert r["ms"] > 0 and r["ms_isolated"] > 0
    assert abs(r["value"] - r["per_rank_bytes"] / 2**30 / (r["ms"] / 1e3)) <= 0.05 * r["value"]
    assert "back to back" in r["timing"]
    # the steady-state figure is the median of 5 runs (after bench.C3_STREAM_WARMUP
    # untimed queued calls), with their spread
    runs = r["ms_runs_rank0"]
    assert len(runs) == 5 and abs(r["ms"] - sorted(runs)[2]) <= 1e-3
    assert f"after {bench.C3_STREAM_WARMUP} untimed calls" in r["timing"]
    assert r["spread_pct_rank0"] >= 0.0
    # the leg's own roofline: image + 24 B per record over the steady-state time, against 8 TB/s
    rf = r["roofline"]
    alg = r["per_rank_bytes"] + 24 * r["physical_records_rank0"]
    assert rf["alg_bytes_per_call"] == alg and rf["bound"] == "hbm" and rf["peak"] == bench.PEAK_GBS
    # (kernel_ms is printed to 4 decimals: 0.1 % of a 64 MiB image's 0.05 ms)
    assert abs(rf["achieved"] - alg / (rf["kernel_ms"] / 1e3) / 1e9) <= 0.005 * rf["achieved"]
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) <= 1e-3
    # a 64 MiB image is not the committed PMC pass's: no traffic, and the reason says so
    assert rf["traffic"] is None and ("image" in rf["traffic_source"] or "build" in rf["traffic_source"])


def test_sharded_replay_one_context_per_device():
    """One WAL across one context PER VISIBLE DEVICE (distinct GPUs; the
    8-GPU node of the driver's round-end run): the stitched stream equals the
    oracle Reader's.  Every other sharded test runs its contexts on device 0,
    so this is the only test of distinct-device contexts; with one device
    visible it skips."""
    from revel_amd import gpu as G
    ndev = G.device_count()
    if ndev < 2:
        pytest.skip(f"{ndev} gfx950 device visible: distinct-device contexts need 2 or more")
    rng = np.random.default_rng(78)
    sizes = rng.integers(0, 20000, 9000)
    recs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in sizes]
    img = oc.write_image(recs)
    ctxs = [G.GpuContext(d) for d in range(ndev)]
    try:
        assert len({G.pci_bus_id(c.device) for c in ctxs}) == ndev
        r = shard.ShardedReplay(ctxs, image=img, checksum=True, window_bytes=8 << 20)
        got = []
        while True:
            x = r.read_record()
            if x is None:
                break
            got.append(x)
        assert got == recs
        s = r.summary()
        assert s["physical"] == len(oc.walk(img)) and s["bad"] == 0 and s["records"] == len(recs)
        r.close()
    finally:
        for c in ctxs:
            c.close()
