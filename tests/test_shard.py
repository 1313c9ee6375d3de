"""One WAL across several shards on the CPU: block ranges, the host boundary
walk and the host stitch (revel_wal_shard_boundary_host / revel_wal_stitch_*)
against the oracle reader over the whole file.  The GPU load of the same
shards is tested in test_gpu.py."""
import numpy as np
import pytest

from revel_amd import shard
from revel_amd._lib import RevelError
from conftest import golden_image
from oracle import crc32c_oracle as po
from oracle import oracle_c as oc

BS = 32768


def drain(read_record, limit=200000):
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
    raise AssertionError("no EOF")


def events_by_shards(img, ranges, stitched):
    """Global event order rebuilt from the shards: each shard's own events
    after the stitched records that complete in its head.  A shard's own
    events = an oracle reader started at the shard (outside any fragment: the
    resync of initial_offset skips the leading MIDDLE/LAST run) that stops at
    the shard end, the torn-tail rule still at the end of the WAL."""
    out = []
    for k, (s, e) in enumerate(ranges):
        out += [p for (_, p, before) in stitched if before == k]
        rd = po.LogReader(img, False, s)
        rd.records = [r for r in rd.records if r.file_offset < e]
        if e < len(img):
            rd.size = 1 << 64  # only the WAL's last record can be torn
        out += drain(rd.read_record)
    return out


def random_log(seed, n=60, maxlen=120000, small=False):
    rng = np.random.default_rng(seed)
    sizes = rng.integers(0, 200 if small else maxlen, n)
    return [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in sizes]


def check_split(img, ranges, read=True):
    blobs = [shard.boundary_host(img, s, e - s, read=read) for s, e in ranges]
    st = shard.Stitch(blobs)
    summ = st.summary()
    want = drain(po.LogReader(img, False).read_record)
    recs = st.records()
    assert summ["bytes"] == len(img)
    assert summ["physical"] == len(oc.walk(img))
    if read:
        assert events_by_shards(img, ranges, recs) == want
        assert summ["records"] == sum(1 for w in want if w != "E")
        assert summ["errors"] == sum(1 for w in want if w == "E")
        assert summ["payload_bytes"] == sum(len(w) for w in want if w != "E")
    else:
        assert all(p is None or len(p) == 0 for _, p, _ in recs)
    return summ


def test_block_ranges_cover_exactly():
    for n in [0, 1, BS, BS + 1, 10 * BS + 5, 1000 * BS]:
        for w in [1, 2, 3, 8]:
            rs = shard.block_ranges(n, w)
            assert len(rs) == w and rs[0][0] == 0 and rs[-1][1] == n
            for (a, b), (c, d) in zip(rs, rs[1:]):
                assert b == c
            assert all(a % BS == 0 or a == n for a, _ in rs)


@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_stitch_random_logs(world, seed):
    img = oc.write_image(random_log(seed))
    summ = check_split(img, shard.block_ranges(len(img), world))
    if world > 1:
        assert summ["stitched"] > 0


def test_stitch_every_block_split():
    """Two shards split at every block boundary of a log whose records span
    up to 4 blocks (boundaries inside FIRST / MIDDLE / LAST runs)."""
    img = oc.write_image(random_log(7, n=12, maxlen=130000))
    nb = (len(img) + BS - 1) // BS
    for cut in range(0, nb + 1):
        c = min(len(img), cut * BS)
        check_split(img, [(0, c), (c, len(img))])


def test_stitch_record_over_many_shards():
    """A 1 MiB record spans 33 blocks: with 1-block shards the fragment runs
    through shards of MIDDLEs only."""
    recs = [b"a" * 100, bytes(range(256)) * 4096, b"b" * 10, b"", b"c" * 70000]
    img = oc.write_image(recs)
    nb = (len(img) + BS - 1) // BS
    ranges = [(k * BS, min(len(img), (k + 1) * BS)) for k in range(nb)]
    summ = check_split(img, ranges)
    assert summ["records"] == len(recs) and summ["stitched"] >= 2


def test_stitch_with_errors_and_torn_tail():
    rng = np.random.default_rng(9)
    img = bytearray(oc.write_image(random_log(11, n=80, maxlen=50000)))
    ref = oc.walk(bytes(img))
    # unknown record types (errors) in the middle of fragments and elsewhere
    for v in rng.choice(len(ref), 8, replace=False):
        img[int(ref["file_offset"][v]) + 6] = 9
    img = bytes(img[:-5])  # a torn final record
    for world in (2, 3, 4, 7):
        check_split(img, shard.block_ranges(len(img), world))


def test_stitch_golden_images(golden_index):
    for name in golden_index:
        img = golden_image(name)
        for world in (1, 2, 3):
            check_split(img, shard.block_ranges(len(img), world))


def test_stitch_verify_mode_counts():
    img = oc.write_image(random_log(5))
    summ = check_split(img, shard.block_ranges(len(img), 4), read=False)
    assert summ["records"] == 0 and summ["stitched"] > 0


def test_stitch_rejects_non_contiguous_blobs():
    img = oc.write_image(random_log(3))
    rs = shard.block_ranges(len(img), 3)
    blobs = [shard.boundary_host(img, s, e - s) for s, e in rs]
    with pytest.raises(RevelError):
        shard.Stitch([blobs[0], blobs[2]])
    with pytest.raises(RevelError):
        shard.Stitch([blobs[0], b"garbage" * 20])
    with pytest.raises(RevelError):
        shard.boundary_host(img, 100, BS)  # not block-aligned
