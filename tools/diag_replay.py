"""Diagnosis: replay_memory of one property-test image (window 64 KiB), printing each step."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from revel_amd import _lib  # noqa: E402

if len(sys.argv) > 1:
    _lib.LIB_PATH = os.path.abspath(sys.argv[1])
from revel_amd import gpu  # noqa: E402
from oracle import oracle_c as oc  # noqa: E402

n, maxlen, period, seed, flips = 1472, 93, 29, 2056565109, 5
rng = np.random.default_rng(seed)
sizes = rng.integers(0, maxlen + 1, n)
sizes[n // 2:] = period
recs = [rng.integers(0, 256, int(s), dtype=np.uint8).tobytes() for s in sizes]
img = bytearray(oc.write_image(recs))
for _ in range(flips):
    img[int(rng.integers(0, len(img)))] ^= 1 << int(rng.integers(0, 8))
img = bytes(img)
ctx = gpu.GpuContext(0)
ref = oc.walk(img)
for w in (1 << 20, 65536):
    print("replay window", w, flush=True)
    st = ctx.replay_memory(img, window_bytes=w)
    print("units", st["units"], "bad", st["bad"], "want", len(ref), int((ref["status"] != 0).sum()), flush=True)
