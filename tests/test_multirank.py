"""World-size-2 gloo tests of the multi-GPU path on the CPU.

Each rank takes its block-aligned shard of one WAL and walks it through the
C-ABI (revel_wal_shard_boundary_host: no GPU, no CRC -- a Reader with
checksum == false), the ranks exchange only their boundary blobs, and rank 0
stitches them (revel_wal_stitch_new); the logical-record view must equal
reading the whole file.  Also checks bench.py's Dist helper (barrier / max /
sum over gloo)."""
import os
import socket

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, image, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    from revel_amd import shard
    D = bench.Dist()
    ranges = shard.block_ranges(len(image), world)
    s, e = ranges[rank]
    blob = shard.boundary_host(image, s, e - s)
    gathered = [None] * world
    D.dist.all_gather_object(gathered, blob)
    D.barrier()
    mx = D.max(float(rank + 1))
    sm = D.sum(1.0)
    if rank == 0:
        st = shard.Stitch(gathered)
        q.put((st.summary(), st.records(), ranges, mx, sm))
    D.close()


@pytest.mark.parametrize("world", [2])
def test_sharded_walk_and_stitch_gloo(world):
    import torch.multiprocessing as mp
    import numpy as np
    from oracle import crc32c_oracle as po
    from oracle import oracle_c as oc

    rng = np.random.default_rng(21)
    recs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in rng.integers(0, 50000, 60)]
    image = oc.write_image(recs)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, image, q)) for r in range(world)]
    for p in procs:
        p.start()
    summ, stitched, ranges, mx, sm = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from test_shard import events_by_shards
    assert recs == po.read_all(image, checksum=False)
    assert events_by_shards(image, ranges, stitched) == recs
    assert summ["records"] == len(recs) and summ["errors"] == 0 and summ["stitched"] >= 1
    assert summ["payload_bytes"] == sum(len(r) for r in recs)
    assert mx == float(world) and sm == float(world)


def _bench(args, devices, timeout=240):
    import subprocess
    import sys
    env = dict(os.environ, REVEL_BENCH_DEVICES=str(devices))
    env.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_bench_gpus_n_launches_n_ranks():
    """`bench.py --gpus 2` outside torch.distributed starts the 2 ranks itself
    (torch.distributed.run as a child process, gloo) and rank 0 prints one JSON
    line with n_gpus 2 and one `ranks` entry per rank (stub device count, no
    GPU work: --dry-run)."""
    import json
    p = _bench(["--gpus", "2", "--dry-run", "--blocks", "64"], devices=2)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["dry_run"]
    assert [r["rank"] for r in d["ranks"]] == [0, 1]
    assert [r["device"] for r in d["ranks"]] == [0, 1]
    assert d["config"]["distinct_devices"] == 2


def test_bench_refuses_more_gpus_than_visible():
    p = _bench(["--gpus", "4", "--blocks", "64"], devices=2, timeout=60)
    assert p.returncode == 2
    assert "2 gfx950 device(s) visible" in p.stderr


def _dry(args, devices, env_extra=None, timeout=300):
    import json
    env_extra = env_extra or {}
    old = {k: os.environ.get(k) for k in env_extra}
    os.environ.update(env_extra)
    try:
        p = _bench(args, devices=devices, timeout=timeout)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_gpus_8_dry_run(tmp_path):
    """The driver's N=8 scaling run, rehearsed on the CPU: 8 ranks (gloo), one
    `ranks` entry per rank on 8 distinct devices, and the end_to_end leg's
    shared file: rank 0 checks the free space for 8 x the per-rank part, every
    rank writes its part at rank x per, all ranks see the whole file.
    Partitioning: contiguous block-aligned parts (records never cross a block,
    log_writer.rs:66-76)."""
    d = _dry(["--gpus", "8", "--dry-run", "--blocks", "64", "--e2e-gib", str(16 * 32768 / 2**30)], devices=8,
             env_extra={"REVEL_BENCH_DIR": str(tmp_path)})
    assert d["n_gpus"] == 8 and d["dry_run"]
    assert [r["rank"] for r in d["ranks"]] == list(range(8))
    assert sorted(r["device"] for r in d["ranks"]) == list(range(8))
    assert d["config"]["distinct_devices"] == 8
    e = d["end_to_end"]
    assert e["skipped"] is None and e["per_rank_bytes"] == 16 * 32768 and e["file_bytes"] == 8 * 16 * 32768
    assert [r["file_size_seen"] for r in e["per_rank"]] == [8 * 16 * 32768] * 8
    assert not os.listdir(tmp_path)  # rank 0 removed the file


def test_bench_gpus_8_e2e_skips_together(tmp_path):
    """Free space short for 8 x the per-rank part, or one rank's write
    failing: every rank skips the end_to_end leg together and the line is
    still printed."""
    big = _dry(["--gpus", "8", "--dry-run", "--blocks", str(1 << 40), "--e2e-gib", "1000000"], devices=8,
               env_extra={"REVEL_BENCH_DIR": str(tmp_path)})
    e = big["end_to_end"]
    assert e["file_bytes"] == 8 * int(1000000 * (1 << 30)) // 32768 * 32768
    assert "MiB free <" in e["skipped"] and all(r["skipped"] for r in e["per_rank"])
    bad = _dry(["--gpus", "8", "--dry-run", "--blocks", "64", "--e2e-gib", str(4 * 32768 / 2**30)], devices=8,
               env_extra={"REVEL_BENCH_DIR": str(tmp_path), "REVEL_BENCH_E2E_FAIL_RANK": "5"})
    e = bad["end_to_end"]
    assert e["skipped"] and all(r["skipped"] for r in e["per_rank"])
    assert not os.listdir(tmp_path)


def test_bench_e2e_share_default_keeps_c5_file_size():
    """The end_to_end leg's default share: 100 / N GiB, so the shared file is
    BASELINE C5's 100 GiB at every N, one GPU included; an
    explicit --e2e-gib wins."""
    import sys
    sys.path.insert(0, ROOT)
    import bench

    class _D:
        def __init__(self, world):
            self.world = world

    dflt = bench.parse([])
    assert dflt.e2e_gib is None
    assert bench.e2e_share(dflt, _D(1)) == 100.0
    assert bench.e2e_share(dflt, _D(2)) == 50.0
    assert bench.e2e_share(dflt, _D(4)) == 25.0
    assert bench.e2e_share(dflt, _D(8)) == 12.5
    assert bench.e2e_share(bench.parse(["--e2e-gib", "0"]), _D(8)) == 0.0
    assert bench.e2e_share(bench.parse(["--e2e-gib", "3"]), _D(8)) == 3.0


def test_bench_e2e_part_repeats_the_image():
    """A rank's part of the end_to_end file larger than its device image
    repeats the image from byte 0 (whole blocks), piece by piece at any
    offset, including pieces that straddle the image's end."""
    import sys
    sys.path.insert(0, ROOT)
    import numpy as np

    import bench
    img = np.arange(5 * 32768, dtype=np.uint64).astype(np.uint8)  # a 5-block stand-in image
    read = lambda src, nb: img[src:src + nb].copy()  # noqa: E731
    whole = np.concatenate([img] * 4)
    for off, m in ((0, 32768), (3 * 32768, 4 * 32768), (5 * 32768 - 7, 20), (100, 15 * 32768 - 200)):
        got = bench.repeat_part(read, len(img), off, m)
        assert np.array_equal(got, whole[off:off + m])
