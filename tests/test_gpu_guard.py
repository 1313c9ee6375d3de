"""Reads past the end of an image, made deterministic.

The round-2 out-of-bounds read of k_verify_records_dense (idle lanes formed
load addresses 16 B past a block whose data ran to the block end) faulted only
when the page after the window buffer happened to be unmapped.  Here the image
lives in device memory mapped with the HIP virtual-memory API at the START of
a reserved address range one mapping granule longer than the image: the
granule after the image is reserved but never mapped, so any load past the
image's last byte faults every time (a regression shows as a GPU memory
fault in this file, not as a flaky failure elsewhere).

The images end with a whole block whose data runs to the block's last byte:
a dense block (258 records: > 64 records -> the dense kernel, > 256 -> the
overflow header list) for record verify, append framing and reassembly, and
full-type blocks for the C2 kernel.  Every result is compared with the oracle.
"""
import ctypes
from ctypes import POINTER, Structure, byref, c_int, c_size_t, c_uint8, c_uint16, c_uint64, c_void_p

import numpy as np
import pytest

from revel_amd import BLOCK_SIZE, gpu
from revel_amd._lib import check, lib
from oracle import crc32c_oracle as po
from oracle import oracle_c as oc

pytestmark = pytest.mark.gpu


class _Loc(Structure):
    _fields_ = [("type", c_int), ("id", c_int)]


class _AllocFlags(Structure):
    _fields_ = [("compressionType", c_uint8), ("gpuDirectRDMACapable", c_uint8), ("usage", c_uint16)]


class _Prop(Structure):  # hipMemAllocationProp (hip_runtime_api.h)
    _fields_ = [("type", c_int), ("requestedHandleType", c_int), ("location", _Loc),
                ("win32HandleMetaData", c_void_p), ("allocFlags", _AllocFlags)]


class _Access(Structure):  # hipMemAccessDesc
    _fields_ = [("location", _Loc), ("flags", c_int)]


_PINNED, _LOC_DEVICE, _PROT_RW, _GRAN_MIN = 0x1, 1, 3, 0


class GuardedImage:
    """`nbytes` (a multiple of the mapping granularity) of device memory at
    the start of a reserved range whose next granule is left unmapped.  Has
    the `.ptr` / `.nbytes` of a DeviceBuffer."""

    def __init__(self, device: int, nbytes: int):
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.nbytes = nbytes
        prop = _Prop(_PINNED, 0, _Loc(_LOC_DEVICE, device), None, _AllocFlags(0, 0, 0))
        g = c_size_t()
        if self.hip.hipMemGetAllocationGranularity(byref(g), byref(prop), _GRAN_MIN) != 0:
            pytest.skip("no HIP virtual-memory management on this device")
        self.granule = g.value
        assert nbytes % self.granule == 0
        self.reserved = nbytes + self.granule
        self.hip.hipMemAddressReserve.argtypes = [POINTER(c_void_p), c_size_t, c_size_t, c_void_p, c_uint64]
        self.hip.hipMemCreate.argtypes = [POINTER(c_void_p), c_size_t, POINTER(_Prop), c_uint64]
        self.hip.hipMemMap.argtypes = [c_void_p, c_size_t, c_size_t, c_void_p, c_uint64]
        self.hip.hipMemSetAccess.argtypes = [c_void_p, c_size_t, POINTER(_Access), c_size_t]
        self.hip.hipMemUnmap.argtypes = [c_void_p, c_size_t]
        self.hip.hipMemRelease.argtypes = [c_void_p]
        self.hip.hipMemAddressFree.argtypes = [c_void_p, c_size_t]
        va, h = c_void_p(), c_void_p()
        assert self.hip.hipMemAddressReserve(byref(va), self.reserved, 0, None, 0) == 0
        self.va = va.value
        assert self.hip.hipMemCreate(byref(h), nbytes, byref(prop), 0) == 0
        self.handle = h.value
        assert self.hip.hipMemMap(self.va, nbytes, 0, self.handle, 0) == 0
        acc = _Access(_Loc(_LOC_DEVICE, device), _PROT_RW)
        assert self.hip.hipMemSetAccess(self.va, nbytes, byref(acc), 1) == 0
        self.ptr = self.va

    def free(self):
        """Deferred to the end of the module (release_all), so that no VA range
        is reserved and mapped a second time within the module.  Round 3 saw
        two wrong results in this file, and round 4 traced them to that reuse
        (tools/vmm_probe.py, profiles/r4/s3_vmm_probe_stale_translation_box.log;
        DESIGN.md 4.9): on one box, once ranges of this API had been unmapped,
        released and reserved again for new physical memory, KERNEL accesses
        and the runtime's COPIES to the same VA reached different memory (one
        side through a stale translation), while copies agreed with copies.
        A kernel write read back by a D2H copy then returns other bytes (the r3
        D2H after synth_full_blocks), and a kernel reading an H2D-copied image
        sees other pages (the r3 C2 launch that returned 2931026674 for two
        blocks: the masked CRC of an all-zero block).  It needed the reuse: no
        mismatch without it, none on the other boxes, and none ever with
        hipMalloc memory (the probe's plain mode and every other GPU test)."""
        _LIVE.append(self)

    def release(self):
        if self.va:
            self.hip.hipMemUnmap(self.va, self.nbytes)
            self.hip.hipMemRelease(self.handle)
            self.hip.hipMemAddressFree(self.va, self.reserved)
            self.va = self.ptr = None


_LIVE = []


@pytest.fixture(scope="module", autouse=True)
def release_all():
    yield
    import ctypes as _c
    _c.CDLL("libamdhip64.so").hipDeviceSynchronize()
    while _LIVE:
        _LIVE.pop().release()


def _guarded_nbytes(min_blocks: int) -> int:
    """Smallest multiple of both the granule and 32 KiB holding min_blocks blocks."""
    hip = ctypes.CDLL("libamdhip64.so")
    prop = _Prop(_PINNED, 0, _Loc(_LOC_DEVICE, 0), None, _AllocFlags(0, 0, 0))
    g = c_size_t()
    if hip.hipMemGetAllocationGranularity(byref(g), byref(prop), _GRAN_MIN) != 0:
        pytest.skip("no HIP virtual-memory management on this device")
    step = int(np.lcm(g.value, BLOCK_SIZE))
    return max(step, -(-min_blocks * BLOCK_SIZE // step) * step)


def dense_tail_records(nbytes: int):
    """Records whose image is exactly nbytes: FULL 32 761-B records for every
    block but the last, then 257 x 120 B + 1 x 122 B = 258 records filling the
    last block to its final byte (257 * 127 + 129 = 32 768)."""
    rng = np.random.default_rng(nbytes)
    nb = nbytes // BLOCK_SIZE
    recs = [rng.integers(0, 256, 32761, dtype=np.uint8).tobytes() for _ in range(nb - 1)]
    recs += [rng.integers(0, 256, 120, dtype=np.uint8).tobytes() for _ in range(257)]
    recs.append(rng.integers(0, 256, 122, dtype=np.uint8).tobytes())
    return recs


def test_full_blocks_end_at_unmapped_granule(gpu_ctx):
    """The C2 kernel's ring re-reads the last block past the end of the list:
    its loads stay inside the image."""
    nbytes = _guarded_nbytes(2)
    n = nbytes // BLOCK_SIZE
    # the blocks come from the host (the test is about the C2 kernel's loads);
    # with no VA range reused in this module (GuardedImage.free), the H2D copy
    # and the kernel see the same pages
    host = oc.synth_full_blocks(n, seed=0x5EED0002)
    g = GuardedImage(0, nbytes)
    try:
        gpu_ctx.h2d(g, host.reshape(-1))
        m, ok = gpu_ctx.alloc(4 * n), gpu_ctx.alloc(n)
        gpu_ctx.crc_full_blocks(g, n, m, ok)
        gpu_ctx.sync()
        assert np.array_equal(gpu_ctx.d2h(m, 4 * n, np.uint32), oc.full_block_crcs(host))
        assert gpu_ctx.d2h(ok, n).all()
    finally:
        g.free()


def test_dense_last_block_ends_at_unmapped_granule(gpu_ctx):
    nbytes = _guarded_nbytes(4)
    recs = dense_tail_records(nbytes)
    img = oc.write_image(recs)
    assert len(img) == nbytes
    ref = oc.walk(img)
    assert (ref["status"] == 0).all() and int((ref["file_offset"] >= nbytes - BLOCK_SIZE).sum()) == 258
    g = GuardedImage(0, nbytes)
    try:
        gpu_ctx.h2d(g, np.frombuffer(img, dtype=np.uint8))
        # the C-ABI sequence (dense blocks: the aligned-word-stream kernel);
        # production split, header walk, v3 with lists
        for path in (None, 0, 1, 2):
            res = gpu_ctx.verify_image(g, nbytes, path=path)
            for f in ("file_offset", "length", "stored_crc", "computed_crc", "status"):
                assert np.array_equal(res[f], ref[f].astype(res[f].dtype)), (path, f)
        ev, payload, _ = gpu_ctx.reassemble(g, nbytes)
        want = po.replay_events(img)
        assert len(ev) == len(want) == len(recs)
        assert bytes(payload) == b"".join(recs)
        gpu_ctx.sync()
    finally:
        g.free()
    # the replay's own window buffer: one window of exactly the image
    st = gpu_ctx.replay_memory(img, window_bytes=nbytes, nbuffers=2, io_threads=2)
    assert st["units"] == len(ref) and st["bad"] == 0


def test_append_framing_dense_last_block_into_guarded_image(gpu_ctx):
    """Device append framing (log_writer.rs:58-124) writing an image that ends
    at the unmapped granule: bytes equal the oracle writer's."""
    nbytes = _guarded_nbytes(4)
    recs = dense_tail_records(nbytes)
    want = oc.write_image(recs)
    lens = np.array([len(r) for r in recs], dtype=np.uint64)
    pay = gpu_ctx.upload(np.frombuffer(b"".join(recs), dtype=np.uint8))
    g = GuardedImage(0, nbytes)
    try:
        L = lib()
        bo, n = ctypes.c_uint64(0), ctypes.c_size_t()
        check(L.revel_gpu_append_records(gpu_ctx.handle, pay.ptr, lens.ctypes.data, len(lens), ctypes.byref(bo),
                                         g.ptr, nbytes, ctypes.byref(n), None))
        assert n.value == nbytes
        assert bytes(gpu_ctx.d2h(g, nbytes)) == want
    finally:
        g.free()
