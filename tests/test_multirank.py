"""World-size-2 gloo tests of the multi-GPU path on the CPU.

Each rank takes its block-aligned shard of one WAL, walks it independently
(no data-path collective), and rank 0 stitches logical records across the
shard boundary; the result must equal reading the whole file.  Also checks
bench.py's Dist helper (barrier / max / sum over gloo)."""
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
    s, e = shard.block_ranges(len(image), world)[rank]
    recs = shard.physical_records(image[s:e], base_offset=s)
    gathered = [None] * world
    D.dist.all_gather_object(gathered, recs)
    D.barrier()
    mx = D.max(float(rank + 1))
    sm = D.sum(1.0)
    if rank == 0:
        q.put((shard.stitch(gathered), mx, sm, [len(g) for g in gathered]))
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
    got, mx, sm, counts = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(c > 0 for c in counts)
    assert got == recs == po.read_all(image, checksum=False)
    assert mx == float(world) and sm == float(world)


def test_block_ranges_cover_exactly():
    from revel_amd import shard
    for n in [0, 1, 32768, 32769, 10 * 32768 + 5]:
        for w in [1, 2, 3, 8]:
            rs = shard.block_ranges(n, w)
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (a, b), (c, d) in zip(rs, rs[1:]):
                assert b == c
            assert all(a % 32768 == 0 or a == n for a, _ in rs)
