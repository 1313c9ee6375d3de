"""Benchmark: CRC32C GiB/s on device-resident 32 KiB WAL blocks (config C2).

One step = one launch of the production CRC kernel over every block resident
in HBM (compute the masked CRC32C of type||payload of each full-type block and
verify it against the stored header).  Per rank: 1 M blocks = 32 GiB,
synthesised and framed on the device (splitmix64 payloads).  Ranks are
independent WAL streams, one per GPU, no collective on the data path
("scaling": "weak"); the barrier / max-over-ranks uses gloo on the host.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`--gpus N` with N > 1 outside torch.distributed (no WORLD_SIZE) launches the N
ranks itself: before anything touches a GPU it counts the visible gfx950
devices (KFD topology + *_VISIBLE_DEVICES; exits non-zero when there are fewer
than N), then runs `python -m torch.distributed.run --nproc-per-node N` on this
script as a child process and exits with its return code.  Each rank drives
GPU `LOCAL_RANK`; the JSON's `ranks` names every rank's device and PCI bus id
with its own kernel time, so a record shows that N distinct GPUs ran.

Prints one JSON line on rank 0.  The `cpu_baseline` leg (rank 0, N=1) times
the oracle's bytewise table CRC -- the reference crate's algorithm class --
on a bounded sample of the same blocks, on one host core, and checks the
GPU's CRCs for that sample against it.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import shutil
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BLOCK_SIZE = 32768  # log_format.rs:26 kBlockSize
METRIC = "CRC32C GiB/s on device-resident 32 KiB WAL blocks; % of HBM-read roofline"
PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SEED = 0x5EED0002


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--blocks", type=int, default=1 << 20, help="blocks per rank (default 1M = 32 GiB)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bound on the CPU baseline leg")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--variant", type=int, default=None, help="experiment kernel variant (default: production)")
    ap.add_argument("--e2e-gib", type=float, default=None,
                    help="per-rank share of the one-file WAL replayed for the end_to_end field (0 = skip; "
                         "a share larger than the --blocks image repeats it; default 100 / N: the 100 GiB "
                         "file of BASELINE config C5 at every N)")
    ap.add_argument("--c3-gib", type=float, default=4.0,
                    help="per-rank device-framed Zipf image for the c3 field (0 = skip)")
    ap.add_argument("--c3-small-gib", type=float, default=4.0,
                    help="per-rank device-framed image of 64..256 B records for the c3_small field (0 = skip)")
    ap.add_argument("--share-gpus", action="store_true",
                    help="rehearsal: allow more ranks than GPUs (rank r drives GPU r mod count)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/distributed plumbing only: no GPU work, values null (CPU tests)")
    return ap.parse_args(argv)


def progress(D, msg: str):
    """A progress line on stderr (rank 0): long legs (the 32 GiB end-to-end
    file) must not look hung to a supervisor watching the output."""
    if D.rank == 0:
        print(f"bench.py: {msg}", file=sys.stderr, flush=True)


def visible_gfx950() -> int:
    """gfx950 devices this process may use, counted WITHOUT initialising HIP
    (the launcher must not touch the GPU before it starts the ranks): KFD
    topology nodes with gfx_target_version 9.5.0, narrowed by the first of
    ROCR/HIP/CUDA_VISIBLE_DEVICES that is set.  REVEL_BENCH_DEVICES overrides
    the count (CPU tests of the launcher)."""
    if os.environ.get("REVEL_BENCH_DEVICES"):
        return int(os.environ["REVEL_BENCH_DEVICES"])
    n = 0
    for p in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties")):
        try:
            with open(p) as f:
                props = dict(line.split() for line in f if len(line.split()) == 2)
        except OSError:
            continue
        if props.get("gfx_target_version") == "90500":
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def launch_ranks(args, argv) -> int:
    """N ranks, one per GPU, under torch.distributed.run as a CHILD process
    (never exec: nothing here has touched the GPU, and the child is a fresh
    interpreter).  Rank 0's JSON line reaches stdout through the inherited
    descriptor; the return code is the launcher's."""
    have = visible_gfx950()
    if args.gpus > have and not args.share_gpus and not args.dry_run:
        print(f"bench.py: --gpus {args.gpus} but {have} gfx950 device(s) visible", file=sys.stderr, flush=True)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    return subprocess.run(cmd, env=env).returncode


class Dist:
    def __init__(self):
        self.rank = int(os.environ.get("RANK", 0))
        self.world = int(os.environ.get("WORLD_SIZE", 1))
        self.local = int(os.environ.get("LOCAL_RANK", 0))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist  # host-side gloo only; torch never touches the GPU here
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: float) -> float:
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def gather(self, obj):
        """Every rank's obj, in rank order (gloo all_gather_object)."""
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


PROD_KERNEL = "k_full_blocks4<1024, false>"  # the production C2 kernel (k_blocks.hip)


def library_sha256() -> str:
    import hashlib
    from revel_amd._lib import LIB_PATH
    with open(LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def pmc_traffic(nblocks: int):
    """HBM bytes per launch from the committed rocprofv3 PMC pass
    (profiles/pmc_c2.json, written by tools/pmc_summary.py) -- only when that
    pass measured THIS build: same kernel symbol, same librevel_wal.so
    SHA-256, same block count.  Returns (bytes or None, source note)."""
    path = os.path.join(ROOT, "profiles", "pmc_c2.json")
    try:
        with open(path) as f:
            p = json.load(f)
    except (OSError, ValueError):
        return None, "no PMC pass committed (profiles/pmc_c2.json)"
    if p.get("kernel") != PROD_KERNEL:
        return None, f"PMC pass was of {p.get('kernel')!r}, not the production {PROD_KERNEL!r}"
    if p.get("library_sha256") != library_sha256():
        return None, "PMC pass was taken on another build of librevel_wal.so"
    if int(p.get("blocks", -1)) != nblocks:
        return None, f"PMC pass was over {p.get('blocks')} blocks, not {nblocks}"
    return p.get("hbm_bytes_per_launch"), (f"profiles/pmc_c2.json: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes "
                                           f"of {PROD_KERNEL} on this librevel_wal.so "
                                           f"(sha256 {p['library_sha256'][:12]}), gfx950 FETCH_SIZE x2")


def pmc_leg_traffic(leg: str, image_bytes: int):
    """HBM bytes per call of a C3 leg (c3 / c3_small) from its committed
    rocprofv3 PMC passes (profiles/pmc_<leg>.json, tools/pmc_summary.py
    --pipeline): every dispatch of one count -> scan -> verify call, FETCH x2 +
    WRITE -- only when those passes measured THIS librevel_wal.so on an image
    of exactly these bytes.  Returns (bytes or None, source note)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{leg}.json")
    try:
        with open(path) as f:
            p = json.load(f)
    except (OSError, ValueError):
        return None, f"no PMC pass committed (profiles/pmc_{leg}.json)"
    if p.get("library_sha256") != library_sha256():
        return None, f"profiles/pmc_{leg}.json was taken on another build of librevel_wal.so"
    if int(p.get("image_bytes") or -1) != image_bytes:
        return None, f"profiles/pmc_{leg}.json was over a {p.get('image_bytes')} B image, not {image_bytes} B"
    return p.get("hbm_bytes_per_call"), (f"profiles/pmc_{leg}.json: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes "
                                          f"over {p.get('calls')} calls on this librevel_wal.so (sha256 "
                                          f"{p['library_sha256'][:12]}), every dispatch of a call, FETCH x2")


def cpu_baseline(ctx, dblocks, masked_dev, nblocks: int, seconds: float):
    """Oracle bytewise CRC (reference algorithm class) on one host core over a
    bounded sample of the same device blocks, repeated until ~`seconds` of CPU
    work; also the parity check of the GPU CRCs on that sample."""
    from oracle import oracle_c  # checker / baseline only

    nsample = min(nblocks, 8192)
    stride = max(1, nblocks // nsample)
    idx = np.arange(0, nblocks, stride)[:nsample]
    sample = np.empty((len(idx), BLOCK_SIZE), np.uint8)
    for j, i in enumerate(idx):
        sample[j] = ctx.d2h(dblocks, BLOCK_SIZE, src_offset=int(i) * BLOCK_SIZE)
    gpu_crc = ctx.d2h(masked_dev, 4 * nblocks, np.uint32)[idx]
    want = oracle_c.full_block_crcs(sample, "bytewise")          # parity (untimed)
    parity = bool(np.array_equal(want, gpu_crc))
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:                    # timed leg
        j = done % len(idx)
        k = min(256, len(idx) - j)
        oracle_c.full_block_crcs(sample[j:j + k], "bytewise")
        done += k
    t_byte = time.perf_counter() - t0
    ctxt = {}
    for v in ("slice16", "sse42"):
        t0 = time.perf_counter()
        got = oracle_c.full_block_crcs(sample, v)
        ctxt[v] = round(len(idx) * BLOCK_SIZE / 2**30 / (time.perf_counter() - t0), 3)
        parity = parity and bool(np.array_equal(got, gpu_crc))
    allcore = cpu_allcore(oracle_c, sample)
    c1 = c1_reference_path(oracle_c)
    return {
        "value": round(done * BLOCK_SIZE / 2**30 / t_byte, 4),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{len(idx)} of the {nblocks} benchmark blocks (every {stride}th, {len(idx) * BLOCK_SIZE >> 20} MiB)"
                  f" cycled for {t_byte:.1f} s = {done} block CRCs; oracle bytewise 256-entry table CRC "
                  f"(crate `crc` algorithm class), single thread",
        "context_GiB_s_1core": ctxt,
        "context_GiB_s_allcore": allcore,
        "host_cores_available": os.cpu_count(),
        "parity_vs_gpu": parity,
        "c1_reference_path": c1,
    }


def cpu_allcore(oracle_c, sample, seconds: float = 1.5):
    """SURVEY 8(d)'s all-core line: one independent block stream per host
    thread (the reference's Writer/Reader are single-threaded per stream), each
    thread cycling over its own slice of the sample for ~`seconds`, per CRC
    implementation.  Threads = the host CPUs this process may use, capped at
    16 (a one-GPU box's CPU share).  Context only: `value` stays one core."""
    import threading
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    nt = max(1, min(16, avail))
    out = {"threads": nt}
    for v in ("bytewise", "slice16", "sse42"):
        done = [0] * nt
        t_end = [0.0]

        per = max(1, len(sample) // nt)

        def work(t):
            lo = min(t * per, len(sample) - per)
            part = sample[lo:lo + per]  # contiguous: no copy inside the timed calls
            k, j, n = 0, 0, 0
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < seconds:
                m = min(64, len(part) - j)
                oracle_c.full_block_crcs(part[j:j + m], v)  # ctypes releases the GIL
                n += m
                j = (j + m) % len(part)
                k += 1
            done[t] = n

        ths = [threading.Thread(target=work, args=(t,)) for t in range(nt)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        t_end[0] = time.perf_counter() - t0
        out[v] = round(sum(done) * BLOCK_SIZE / 2**30 / t_end[0], 3)
    return out


def c1_reference_path(oracle_c):
    """Config C1 on the CPU: 10 000 x 4 KiB records appended with the oracle's
    writer restatement (log_writer.rs:58-124, bytewise CRC) and read back with
    its per-record CRC walk (log_reader.rs:200-206 made per record), one thread."""
    from oracle import crc32c_oracle as po
    words = po.splitmix64_np(np.uint64(0x5EED0001) ^ np.arange(10000, dtype=np.uint64), 512)
    recs = [words[i].tobytes() for i in range(10000)]
    t0 = time.perf_counter()
    image = oracle_c.write_image(recs)
    t_w = time.perf_counter() - t0
    t0 = time.perf_counter()
    walk = oracle_c.walk(image)
    t_r = time.perf_counter() - t0
    ok = bool((walk["status"] == 0).all()) and len(image) == 41038750
    mb = 10000 * 4096 / 1e6
    return {"records": 10000, "record_bytes": 4096, "image_bytes": len(image), "all_crc_ok": ok,
            "append_records_per_s": round(10000 / t_w), "append_MB_s": round(mb / t_w, 1),
            "readback_verify_records_per_s": round(10000 / t_r), "readback_verify_MB_s": round(mb / t_r, 1),
            "note": "reference's own reader cannot complete C1 (SURVEY App. A #1-3); LevelDB-correct walk timed"}


def e2e_file_path(D, total: int = 0) -> tuple:
    """(directory, path) of the one WAL file every rank of this job shares:
    REVEL_BENCH_DIR when set, else the first of the temp directory and
    /dev/shm with room for `total` bytes + 1 GiB (C5's 100 GiB file does not
    fit every box's root file system; it is read from the page cache either
    way), else the temp directory (the caller's free-space check then skips
    the leg with its reason).  Every rank computes the same choice before any
    byte is written (rank 0's truncate allocates nothing)."""
    import tempfile
    d = os.environ.get("REVEL_BENCH_DIR")
    if not d:
        cands = [tempfile.gettempdir(), "/dev/shm"]
        d = cands[0]
        for c in cands:
            try:
                if os.path.isdir(c) and shutil.disk_usage(c).free >= total + (1 << 30):
                    d = c
                    break
            except OSError:
                continue
    tag = os.environ.get("TORCHELASTIC_RUN_ID") or str(os.getppid() if D.world > 1 else os.getpid())
    return d, os.path.join(d, f"revel_bench_{os.environ.get('MASTER_PORT', 'solo')}_{tag}.log")


E2E_CHUNK = 1 << 30  # host bytes per piece of a rank's part (bounds the host copy at N ranks x 1 GiB)


def e2e_share(args, D) -> float:
    """GiB of the shared WAL file per rank: --e2e-gib, or by default 100 / N,
    so the file is BASELINE config C5's 100 GiB at every N (one GPU replays
    all of it).  A rank's part repeats its device-resident C2
    image when the part is larger than the image."""
    if args.e2e_gib is not None:
        return args.e2e_gib
    return 100.0 / D.world


def repeat_part(read, img_bytes: int, off: int, m: int) -> np.ndarray:
    """Bytes [off, off + m) of a rank's part of the end_to_end file: its
    device image (read(src_offset, nbytes) -> bytes), repeated from byte 0
    past the image's end.  The image is whole blocks, so every repeat is a
    valid WAL and the file is C5's size whatever the image's."""
    out = np.empty(m, np.uint8)
    done = 0
    while done < m:
        src = (off + done) % img_bytes
        take = min(m - done, img_bytes - src)
        out[done:done + take] = read(src, take)
        done += take
    return out


def e2e_write_file(D, per: int, part):
    """Write the shared WAL file for the end_to_end leg: rank 0 checks the
    free space for all ranks' parts (world x per bytes + 1 GiB) and creates
    the file, then every rank writes its part at rank x per, piece by piece
    (part(offset, nbytes) -> bytes of that piece, E2E_CHUNK at a time).  A failure anywhere makes EVERY rank skip the leg together
    (the headline value is already measured and must still be printed).
    Returns (path, None), or (None, reason) after removing the file.
    REVEL_BENCH_E2E_FAIL_RANK=r makes rank r's write fail (CPU tests)."""
    total = per * D.world
    d, path = e2e_file_path(D, total)
    why = ""
    if D.rank == 0:
        try:
            free = shutil.disk_usage(d).free
            if free < total + (1 << 30):
                why = f"{d}: {free >> 20} MiB free < {total >> 20} MiB file + 1 GiB"
            else:
                with open(path, "wb") as f:
                    f.truncate(total)
        except OSError as ex:
            why = f"create {path}: {ex}"
    if D.max(float(bool(why))) > 0:
        return None, why or "another rank could not write its part"
    ok = True
    try:
        if os.environ.get("REVEL_BENCH_E2E_FAIL_RANK") == str(D.rank):
            raise OSError(28, "injected write failure (REVEL_BENCH_E2E_FAIL_RANK)")
        fd = os.open(path, os.O_WRONLY)
        try:
            for off in range(0, per, E2E_CHUNK):
                m = min(E2E_CHUNK, per - off)
                view = memoryview(part(off, m))
                done = 0
                while done < m:
                    done += os.pwrite(fd, view[done:], D.rank * per + off + done)
                del view
        finally:
            os.close(fd)
    except OSError as ex:
        ok, why = False, f"rank {D.rank} write: {ex}"
    if D.max(float(not ok)) > 0:
        D.barrier()
        if D.rank == 0:
            try:
                os.unlink(path)
            except OSError:
                pass
        return None, why or "another rank could not write its part"
    return path, None


def end_to_end(ctx, D, dblocks, nblocks: int, gib: float):
    """Config C5, PCIe-inclusive (not `value`): ONE WAL file on the host holds
    every rank's blocks (rank r's `gib` GiB at offset r * gib); each rank loads
    its block-aligned shard of it onto its GPU (revel_gpu_wal_shard_load: mmap
    of the file -> 8 fill threads -> 3 x 64 MiB pinned ring -> H2D on a copy
    stream, records counted as each window lands -> verify of the resident
    shard), the ranks exchange their boundary blobs and rank 0 stitches them
    (revel_wal_stitch_new).  Rate = file bytes / max-over-ranks load time;
    file writing is outside the clock.  The file was just written, so it is
    read from the page cache.  `value` times the pipeline (first window read ->
    boundary blob); `all_in_GiB_s` adds the shard's HBM + pinned-ring setup."""
    from revel_amd import shard
    k = int(gib * (1 << 30)) // BLOCK_SIZE
    per = k * BLOCK_SIZE
    total = per * D.world
    img_bytes = nblocks * BLOCK_SIZE
    path, why = e2e_write_file(
        D, per, lambda off, m: repeat_part(lambda src, nb: ctx.d2h(dblocks, nb, src_offset=src), img_bytes, off, m))
    if path is None:
        return {"value": None, "skipped": why}
    D.barrier()
    s, e = shard.block_ranges(total, D.world)[D.rank]
    t0 = time.perf_counter()
    sh = shard.WalShard(ctx, s, e - s, path=path, file_bytes=total, checksum=True, read=False,
                        window_bytes=64 << 20, io_threads=8)
    t_all = time.perf_counter() - t0
    info = sh.info()
    t_load = info["seconds"]  # the pipeline: first window read -> boundary (HBM / pinned-ring setup excluded)
    blob = sh.boundary()
    sh.close()
    wall_max = D.max(t_load)
    all_in_max = D.max(t_all)
    blobs = [blob]
    if D.dist:
        blobs = [None] * D.world
        D.dist.all_gather_object(blobs, blob)
    D.barrier()
    if D.rank == 0:
        try:
            os.unlink(path)
        except OSError:
            pass
    summ = shard.Stitch(blobs).summary() if D.rank == 0 else {}
    per_rank = D.gather({"rank": D.rank, "load_s": round(t_load, 4), "all_in_s": round(t_all, 4),
                         "h2d_ms": round(info["h2d_ms"], 3), "verify_ms": round(info["kernel_ms"], 3)})
    return {
        "unit": "GiB/s",
        "value": round(total / 2**30 / wall_max, 2),
        "all_in_GiB_s": round(total / 2**30 / all_in_max, 2),
        "setup_s_rank0": round(info["setup_seconds"], 3),
        "file_GiB": round(total / 2**30, 2),
        "per_rank_GiB": round(per / 2**30, 2),
        "h2d_GiB_s_rank0": round((e - s) / 2**30 / (info["h2d_ms"] / 1e3), 2) if info["h2d_ms"] else None,
        "read_s_rank0": round(info["read_seconds"], 3),
        "verify_ms_rank0": round(info["kernel_ms"], 3),
        "per_rank": per_rank,
        "physical_records": summ.get("physical"),
        "bad_records": summ.get("bad"),
        "stitched": summ.get("stitched"),
        "source": f"one WAL file in {os.path.dirname(path)} (page cache: written just before), shared by all ranks",
        "path": "file mmap -> 8 fill threads -> 3 x 64 MiB pinned ring -> H2D (copy stream) + per-window record count "
                "-> verify of the HBM-resident shard -> boundary blob -> rank-0 stitch",
    }


def c3_sizes(shape: str, seed: int, target: int) -> np.ndarray:
    """Record sizes for the device-framed verify legs, until the framed image
    reaches `target` bytes.  zipf (C3): 64*k B, k in [1, 512] ~ Zipf(1.1);
    small: 64..256 B uniform -- the db_bench-shaped logs DB::put produces
    through DB::write -> Writer::add_record (db.rs:95-120, log_writer.rs:58-97),
    ~200 records per block, so nearly every block takes the dense path."""
    rng = np.random.default_rng(seed)
    if shape == "zipf":
        k = np.arange(1, 513)
        p = k ** -1.1
        p /= p.sum()
        sizes = (64 * rng.choice(k, size=target // 3000 + 4096, p=p)).astype(np.uint64)
    elif shape == "small":
        sizes = rng.integers(64, 257, size=target // 160 + 4096).astype(np.uint64)
    else:
        raise ValueError(shape)
    return sizes[:int(np.searchsorted(np.cumsum(sizes + 7), target))]


def c3_image(ctx, shape: str, seed: int, gib: float):
    """A device-framed WAL image: payload bytes synthesised on the device,
    framed by revel_gpu_append_records (bit-exact with log::Writer,
    tests/test_gpu.py).  Returns (image buffer, image bytes, record count)."""
    sizes = c3_sizes(shape, seed, int(gib * (1 << 30)))
    nb_pay = (int(sizes.sum()) + BLOCK_SIZE - 1) // BLOCK_SIZE
    pay = ctx.alloc(max(1, nb_pay) * BLOCK_SIZE)
    ctx.synth_full_blocks(pay, nb_pay, seed=seed)
    img, n, _ = ctx.append_records(pay, sizes)
    pay.free()
    return img, n, len(sizes)


def c3_verify_timed(ctx, img, n: int, nrec: int, iters: int, barrier=lambda: None, stream=None, stream_runs: int = 1,
                    stream_warmup: int = 0):
    """The production verify of a resident image through the C-ABI
    (revel_gpu_count_scan_records -> revel_gpu_verify_records), timed with
    HIP events around both calls, `iters` times, each call isolated (host
    sync after it).  With a list `stream`, then also `iters` calls queued back
    to back, `stream_runs` times (after `stream_warmup` untimed calls queued the same
    way), each run's ms per call appended to it.  Returns (per-iteration ms,
    physical records, records whose status is not OK: the last call's)."""
    from revel_amd._lib import check, lib
    from revel_amd.gpu import RECORD_DTYPE
    L = lib()
    nblocks = (n + BLOCK_SIZE - 1) // BLOCK_SIZE
    counts, first = ctx.alloc(4 * nblocks), ctx.alloc(4 * nblocks)
    cap = nrec + 2 * nblocks + 64           # records + FIRST/MIDDLE/LAST splits
    out = ctx.alloc(cap * RECORD_DTYPE.itemsize)
    e0, e1 = ctx.event(), ctx.event()
    times = []
    barrier()
    for _ in range(iters):
        e0.record()
        check(L.revel_gpu_count_scan_records(ctx.handle, img.ptr, n, counts.ptr, first.ptr, None))
        check(L.revel_gpu_verify_records(ctx.handle, img.ptr, n, 0, first.ptr, out.ptr, None))
        e1.record()
        ctx.sync()
        times.append(e0.elapsed_ms(e1))
    barrier()
    if stream is not None:
        # steady state: `iters` calls queued back to back (no host sync between
        # them, as a reader verifying window after window issues them), one
        # pair of events around all: per call = elapsed / iters, taken
        # `stream_runs` times (a median and its spread, not one
        # sample).  The isolated times above also hold the host's submission of
        # the first launch after e0 (~20 us on an idle stream: `gap before`
        # k_count_hist in the traces).
        # untimed: `stream_warmup` calls queued back to back first, so the
        # timed runs see the clocks of a sustained load (round 6: without it the
        # 3 runs fell monotonically, e.g. 0.815 / 0.795 / 0.788 ms on Zipf)
        for _ in range(stream_warmup):
            check(L.revel_gpu_count_scan_records(ctx.handle, img.ptr, n, counts.ptr, first.ptr, None))
            check(L.revel_gpu_verify_records(ctx.handle, img.ptr, n, 0, first.ptr, out.ptr, None))
        for _ in range(stream_runs):
            e0.record()
            for _ in range(iters):
                check(L.revel_gpu_count_scan_records(ctx.handle, img.ptr, n, counts.ptr, first.ptr, None))
                check(L.revel_gpu_verify_records(ctx.handle, img.ptr, n, 0, first.ptr, out.ptr, None))
            e1.record()
            ctx.sync()
            stream.append(e0.elapsed_ms(e1) / iters)
        barrier()
    nphys = int(ctx.d2h(first, 4 * nblocks, np.uint32)[-1]) + int(ctx.d2h(counts, 4 * nblocks, np.uint32)[-1])
    res = ctx.d2h(out, nphys * RECORD_DTYPE.itemsize).view(RECORD_DTYPE)
    bad = int((res["status"] != 0).sum())
    for b in (counts, first, out):
        b.free()
    return times, nphys, bad


C3_STREAM_WARMUP = 27  # ~22 ms of sustained verify before the steady-state runs


def c3_records(ctx, D, gib: float, iters: int = 9, shape: str = "zipf"):
    """Config C3 on every rank (shape zipf: Zipf(1.1) record sizes 64*k, k in
    [1, 512], seed 0x5EED0003 ^ rank; shape small: 64..256 B, the c3_small
    field), framed ON DEVICE, then the production verify path (count -> scan
    -> verify) timed with HIP events; all ranks start together, rate = total
    bytes / max-over-ranks median time."""
    seed = (0x5EED0003 if shape == "zipf" else 0x5EED0005) ^ D.rank
    img, n, nrec = c3_image(ctx, shape, seed, gib)
    streamed = []
    times, nphys, bad = c3_verify_timed(ctx, img, n, nrec, iters, D.barrier, stream=streamed, stream_runs=5,
                                        stream_warmup=C3_STREAM_WARMUP)
    img.free()
    bad = D.sum(float(bad))
    ms = float(np.median(streamed))
    ms_max = D.max(ms)
    iso_max = D.max(float(np.median(times)))
    alg = n + 24 * nphys  # image read + 24-B result per physical record (rank 0's image)
    traffic, traffic_source = pmc_leg_traffic("c3" if shape == "zipf" else "c3_small", n)
    return {
        "unit": "GiB/s",
        "value": round(n * D.world / 2**30 / (ms_max / 1e3), 1),
        "ms": round(ms_max, 4),
        "roofline": {
            "bound": "hbm",
            "achieved": round(alg / (ms / 1e3) / 1e9, 1),
            "peak": PEAK_GBS,
            "unit": "GB/s",
            "frac": round(alg / (ms / 1e3) / 1e9 / PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_over_alg": round(traffic / alg, 3) if traffic else None,
            "traffic_source": traffic_source,
            "kernel_ms": round(ms, 4),
            "kernel_ms_basis": "rank 0, steady state: the whole count -> scan -> verify call (all its launches)",
            "alg_bytes_per_call": alg,
        },
        "timing": f"median of {len(streamed)} runs of {iters} calls queued back to back between one pair of HIP "
                  f"events (steady state, ms per call), after {C3_STREAM_WARMUP} untimed calls queued the same way",
        "ms_runs_rank0": [round(x, 4) for x in streamed],
        "spread_pct_rank0": round(100.0 * (max(streamed) - min(streamed)) / ms, 2),
        "ms_isolated": round(iso_max, 4),
        "value_isolated": round(n * D.world / 2**30 / (iso_max / 1e3), 1),
        "per_rank_bytes": n,
        "physical_records_rank0": nphys,
        "bad_records": int(bad),
        "alg_GB_s_rank0": round((n + 24 * nphys) / (ms / 1e3) / 1e9, 1),
        "path": "count (per-block header walk + header list) -> scan -> verify (production: k_verify_rows over blocks "
                "with <= 64 records, k_verify_records_dense2 over denser ones)",
        "data": ("Zipf(1.1) 64 B..32 KiB records" if shape == "zipf" else "uniform 64..256 B records (db_bench-shaped)")
                + " framed on device by revel_gpu_append_records",
    }


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, argv)  # the parent never touches the GPU
    D = Dist()
    if D.world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={D.world}", file=sys.stderr, flush=True)
    if args.dry_run:
        return dry_run(args, D)
    from revel_amd import gpu  # the product library (and the HIP runtime) load here, in the ranks
    ndev = gpu.device_count()
    if ndev == 0:
        raise SystemExit("bench.py needs a gfx950 GPU (no fallback)")
    if D.world > ndev and not args.share_gpus:
        raise SystemExit(f"bench.py: {D.world} ranks but {ndev} gfx950 device(s) visible (--share-gpus to rehearse)")
    device = D.local % ndev  # distinct per rank unless --share-gpus
    ctx = gpu.GpuContext(device)
    n = args.blocks
    dblocks = ctx.alloc(n * BLOCK_SIZE)
    masked = ctx.alloc(4 * n)
    ok = ctx.alloc(n)
    ctx.synth_full_blocks(dblocks, n, seed=SEED ^ (D.rank << 40))
    ctx.sync()

    def step():
        ctx.crc_full_blocks(dblocks, n, masked, ok, variant=args.variant)

    for _ in range(args.warmup):
        step()
    ctx.sync()
    okh = ctx.d2h(ok, n)
    all_ok = D.sum(float(okh.all())) == D.world

    ev0, ev1 = ctx.event(), ctx.event()
    ctx.sync()
    D.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    ctx.sync()
    D.barrier()
    t1 = time.perf_counter()
    wall = D.max(t1 - t0)
    kern_ms = ev0.elapsed_ms(ev1) / args.steps
    kern_ms_max = D.max(kern_ms)
    ranks = D.gather({"rank": D.rank, "local_rank": D.local, "host": socket.gethostname(), "device": device,
                      "pci_bus_id": gpu.pci_bus_id(device), "kernel_ms": round(kern_ms, 4),
                      "wall_ms_per_step": round((t1 - t0) / args.steps * 1e3, 4),
                      "all_verify_flags_ok": bool(okh.all())})

    total_blocks = n * D.world
    value = total_blocks * BLOCK_SIZE / 2**30 / (wall / args.steps)
    alg_bytes = n * (BLOCK_SIZE + 4 + 1)          # read block, write masked CRC + ok flag
    achieved = alg_bytes / (kern_ms_max / 1e3) / 1e9
    traffic, traffic_source = pmc_traffic(n)

    progress(D, f"C2 {kern_ms_max:.3f} ms per launch")
    e2e = None
    e2e_gib = e2e_share(args, D)
    if e2e_gib > 0:
        progress(D, f"end_to_end: writing and replaying a {e2e_gib:g} GiB-per-rank WAL file")
        e2e = end_to_end(ctx, D, dblocks, n, e2e_gib)
        e2e["sizing"] = ("--e2e-gib" if args.e2e_gib is not None else
                         "default: 100 / N GiB per rank (BASELINE C5's 100 GiB file at every N)")
        progress(D, f"end_to_end: {e2e.get('value')} GiB/s")

    c3 = None
    if args.c3_gib > 0:
        c3 = c3_records(ctx, D, args.c3_gib)
        progress(D, f"c3: {c3['ms']} ms")
    c3_small = None
    if args.c3_small_gib > 0:
        c3_small = c3_records(ctx, D, args.c3_small_gib, shape="small")
        progress(D, f"c3_small: {c3_small['ms']} ms")

    cpu = None
    if D.rank == 0 and D.world == 1 and not args.no_cpu:
        progress(D, "cpu_baseline")
        cpu = cpu_baseline(ctx, dblocks, masked, n, args.cpu_seconds)

    if D.rank == 0:
        out = result_line(args, D, ranks, value=round(value, 1), ms=round(wall / args.steps * 1e3, 4))
        binfo = gpu.build_info()
        out["config"].update({"kernel_variant": "production" if args.variant is None else args.variant,
                              "all_verify_flags_ok": all_ok,
                              "library_sha256": library_sha256(),   # which binary ran (build provenance)
                              "build_info": binfo,
                              # XFLAGS builds (timing probes, A/B switches) are not the product
                              "diagnostic_build": "XFLAGS:" in binfo})
        if "XFLAGS:" in binfo:
            print(f"bench.py: WARNING: librevel_wal.so is a variant build ({binfo}); not a product measurement",
                  file=sys.stderr, flush=True)
        out["roofline"] = {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_source,
            "kernel_ms": round(kern_ms_max, 4),
            "alg_bytes_per_launch": alg_bytes,
        }
        out["cpu_baseline"] = cpu
        out["end_to_end"] = e2e
        out["c3"] = c3
        out["c3_small"] = c3_small
        print(json.dumps(out), flush=True)
    D.close()
    return 0


def result_line(args, D, ranks, value, ms):
    """The JSON line's contract fields (values filled by the caller)."""
    n = args.blocks
    distinct = len({(r["host"], r["pci_bus_id"]) for r in ranks})
    return {
        "metric": METRIC,
        "value": value,
        "unit": "GiB/s",
        "n_gpus": D.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: splitmix64 payloads generated + framed (masked CRC headers) on device",
        "config": {
            "workload": "C2: device-resident full-type 32 KiB WAL blocks, masked CRC32C(type||payload) "
                        "compute + verify vs stored header, one wavefront per block",
            "blocks_per_gpu": n,
            "bytes_per_gpu": n * BLOCK_SIZE,
            "parallelism": f"independent WAL stream per GPU x{D.world} (no collective)",
            "distinct_devices": distinct,
        },
        "ranks": ranks,
    }


def dry_run(args, D):
    """The launcher and the distributed plumbing without a GPU: every rank
    reports itself, rank 0 prints the line with null values.  With --e2e-gib
    the end_to_end leg's shared-file logic runs for real (free-space check of
    world x per-rank bytes, every rank's part written, the all-ranks skip on
    any failure) with zero bytes in place of the device blocks."""
    D.barrier()
    e2e = None
    e2e_gib = e2e_share(args, D)
    if e2e_gib > 0:
        k = int(e2e_gib * (1 << 30)) // BLOCK_SIZE
        per = k * BLOCK_SIZE
        path, why = e2e_write_file(D, per, lambda off, m: np.zeros(m, np.uint8))
        size = os.path.getsize(path) if path else None
        D.barrier()
        if path and D.rank == 0:
            os.unlink(path)
        e2e = {"file_bytes": per * D.world, "per_rank_bytes": per, "skipped": why,
               "per_rank": D.gather({"rank": D.rank, "skipped": path is None, "file_size_seen": size})}
    ranks = D.gather({"rank": D.rank, "local_rank": D.local, "host": socket.gethostname(), "device": D.local,
                      "pci_bus_id": f"dry-run-{D.local}", "kernel_ms": None})
    if D.rank == 0:
        out = result_line(args, D, ranks, value=None, ms=None)
        out["dry_run"] = True
        out["end_to_end"] = e2e
        print(json.dumps(out), flush=True)
    D.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
