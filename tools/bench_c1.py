"""Config C1 through the PRODUCT path: 10 000 x 4 KiB records appended by
revel_log_writer (host, SSE4.2 CRC, flush per physical record, memory or
posix file) and read back by revel_log_reader with checksum=true (CRC
verified on the GPU).  The reference-path (oracle) timing of the same
workload is in bench.py's cpu_baseline.c1_reference_path."""
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from revel_amd import env, gpu, log  # noqa: E402


def splitmix_records(n=10000, words=512, seed=0x5EED0001):
    with np.errstate(over="ignore"):
        x = (np.uint64(seed) ^ np.arange(n, dtype=np.uint64))[:, None] + \
            (np.arange(1, words + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))[None, :]
        z = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return [z[i].tobytes() for i in range(n)]


def main():
    recs = splitmix_records()
    mb = len(recs) * 4096 / 1e6
    ctx = gpu.GpuContext(0)
    out = {"workload": "C1 10000 x 4 KiB append + read-back, product path"}
    for kind in ("memory", "posix"):
        if kind == "memory":
            f = env.MemoryWritableFile()
        else:
            path = os.path.join(tempfile.gettempdir(), "revel_c1.log")
            f = env.PosixWritableFile(path)
        w = log.Writer(f)
        t0 = time.perf_counter()
        for r in recs:
            w.add_record(r)
        if kind == "posix":
            f.sync()
            f.close()
        tw = time.perf_counter() - t0
        src = env.MemorySequentialFile(f.contents()) if kind == "memory" else env.PosixSequentialFile(path)
        t0 = time.perf_counter()
        rd = log.Reader(src, checksum=True, gpu=ctx)
        got = list(rd)
        tr = time.perf_counter() - t0
        assert got == recs
        out[kind] = {"append_records_per_s": round(len(recs) / tw), "append_MB_s": round(mb / tw, 1),
                     "readback_gpu_verify_records_per_s": round(len(recs) / tr),
                     "readback_gpu_verify_MB_s": round(mb / tr, 1)}
        if kind == "posix":
            os.unlink(path)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
