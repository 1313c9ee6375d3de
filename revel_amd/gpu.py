"""Device-resident CRC engine (gfx950 HIP kernels) via the C-ABI.

Device memory is owned through :class:`DeviceBuffer`; host arrays are numpy.
No torch types cross the boundary: every call hands plain pointers to
``librevel_wal.so``.
"""
from __future__ import annotations

import ctypes
from ctypes import c_float, c_int, c_void_p
from typing import Optional, Tuple

import numpy as np

from ._lib import (BLOCK_SIZE, REPLAY_FULL_BLOCKS, REPLAY_IO, REPLAY_RECORDS, RecordResult, ReplayStats, check,
                   lib)

LOGICAL_DTYPE = np.dtype([("file_offset", "<u8"), ("payload_offset", "<u8"), ("length", "<u4"),
                          ("first_phys", "<u4"), ("last_phys", "<u4"), ("status", "u1"), ("reserved", "u1", (3,))])
BATCH_INFO_DTYPE = np.dtype([("sequence", "<u8"), ("first_entry", "<u8"), ("count", "<u4"), ("nentries", "<u4"),
                             ("status", "u1"), ("reserved", "u1", (7,))])
BATCH_ENTRY_DTYPE = np.dtype([("sequence", "<u8"), ("key_offset", "<u8"), ("value_offset", "<u8"),
                              ("key_len", "<u4"), ("value_len", "<u4"), ("batch", "<u4"), ("type", "u1"),
                              ("reserved", "u1", (3,))])
assert BATCH_INFO_DTYPE.itemsize == 32 and BATCH_ENTRY_DTYPE.itemsize == 40
RECORD_DTYPE = np.dtype([("file_offset", "<u8"), ("length", "<u4"), ("stored_crc", "<u4"),
                         ("computed_crc", "<u4"), ("type", "u1"), ("status", "u1"), ("reserved", "u1", (2,))])
assert RECORD_DTYPE.itemsize == ctypes.sizeof(RecordResult)

# verify paths of tools/experiments' revel_x_verify_dense_variant
_DENSE_VARIANTS = {"dense_chunks": 1, "dense_quad": 2, "dense_sorted": 3, "dense_staged": 5,
                   "dense_staged_1ch": 4, "dense_staged_12w": 7, "dense_staged_12w_1ch": 6,
                   "dense_staged_a16": 12, "dense_staged_a16_8w": 13, "dense_pairs": 16}


def device_count() -> int:
    n = c_int(0)
    check(lib().revel_gpu_device_count(ctypes.byref(n)))
    return n.value


def build_info() -> str:
    """The compiler (and target) that built librevel_wal.so's kernels."""
    return lib().revel_build_info().decode()


def pci_bus_id(device: int) -> str:
    """PCI bus id of a visible HIP device (which physical GPU ran)."""
    buf = ctypes.create_string_buffer(64)
    check(lib().revel_gpu_device_pci_bus_id(device, buf, 64))
    return buf.value.decode()


class DeviceBuffer:
    def __init__(self, ctx: "GpuContext", nbytes: int):
        self.ctx = ctx
        self.nbytes = nbytes
        p = c_void_p()
        check(lib().revel_gpu_malloc(ctx.handle, nbytes, ctypes.byref(p)))
        self.ptr = p.value

    def free(self) -> None:
        if self.ptr:
            check(lib().revel_gpu_free(self.ctx.handle, self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def offset(self, nbytes: int) -> int:
        return self.ptr + nbytes


class Event:
    def __init__(self, ctx: "GpuContext"):
        self.ctx = ctx
        p = c_void_p()
        check(lib().revel_gpu_event_new(ctx.handle, ctypes.byref(p)))
        self.ptr = p.value

    def record(self, stream: Optional[int] = None) -> None:
        check(lib().revel_gpu_event_record(self.ctx.handle, self.ptr, stream))

    def elapsed_ms(self, end: "Event") -> float:
        ms = c_float()
        check(lib().revel_gpu_event_elapsed_ms(self.ctx.handle, self.ptr, end.ptr, ctypes.byref(ms)))
        return ms.value

    def __del__(self):
        try:
            if self.ptr:
                lib().revel_gpu_event_free(self.ctx.handle, self.ptr)
                self.ptr = None
        except Exception:
            pass


class GpuContext:
    """One HIP device + stream (``revel_gpu_context``)."""

    def __init__(self, device: int = 0):
        p = c_void_p()
        check(lib().revel_gpu_context_new(device, ctypes.byref(p)))
        self._h = p.value
        self.device = device

    @property
    def handle(self) -> int:
        return self._h

    @property
    def stream(self) -> int:
        return lib().revel_gpu_context_stream(self._h)

    def trim(self) -> None:
        """Drop the window buffers parked by freed readers (revel_gpu_context_trim)."""
        check(lib().revel_gpu_context_trim(self.handle))

    def close(self) -> None:
        """revel_gpu_context_free: deferred to the last reader still using it."""
        if self._h:
            lib().revel_gpu_context_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- plumbing ----
    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def h2d(self, dst: DeviceBuffer, src: np.ndarray, dst_offset: int = 0) -> None:
        src = np.ascontiguousarray(src)
        check(lib().revel_gpu_memcpy_h2d(self._h, dst.ptr + dst_offset, src.ctypes.data, src.nbytes, None))
        self.sync()

    def d2h(self, src: DeviceBuffer, nbytes: int, dtype=np.uint8, src_offset: int = 0) -> np.ndarray:
        out = np.empty(nbytes // np.dtype(dtype).itemsize, dtype=dtype)
        check(lib().revel_gpu_memcpy_d2h(self._h, out.ctypes.data, src.ptr + src_offset, out.nbytes, None))
        self.sync()
        return out

    def upload(self, host: np.ndarray) -> DeviceBuffer:
        host = np.ascontiguousarray(host)
        buf = self.alloc(max(1, host.nbytes))
        if host.nbytes:
            self.h2d(buf, host)
        return buf

    def memset(self, dst: DeviceBuffer, value: int, nbytes: int) -> None:
        check(lib().revel_gpu_memset(self._h, dst.ptr, value, nbytes, None))

    def sync(self) -> None:
        check(lib().revel_gpu_stream_synchronize(self._h, None))

    def event(self) -> Event:
        return Event(self)

    # ---- kernels ----
    def crc_full_blocks(self, blocks: DeviceBuffer, nblocks: int, masked_out: DeviceBuffer,
                        ok_out: Optional[DeviceBuffer] = None, variant: Optional[int] = None) -> None:
        """Config C2: masked CRC of bytes [6:32768) of each full-type block."""
        if blocks.nbytes < nblocks * BLOCK_SIZE or masked_out.nbytes < 4 * nblocks:
            raise ValueError("buffer too small for nblocks")
        if ok_out is not None and ok_out.nbytes < nblocks:
            raise ValueError("ok buffer too small")
        ok = ok_out.ptr if ok_out is not None else None
        if variant is None or variant == 0:
            check(lib().revel_gpu_crc_full_blocks(self._h, blocks.ptr, nblocks, masked_out.ptr, ok, None))
        else:
            from ._lib import experiments  # kernel variants kept for the record (tools/experiments)
            check(experiments().revel_x_crc_full_blocks_variant(self._h, variant, blocks.ptr, nblocks,
                                                                masked_out.ptr, ok, None))

    def frame_full_blocks(self, blocks: DeviceBuffer, nblocks: int) -> None:
        if blocks.nbytes < nblocks * BLOCK_SIZE:
            raise ValueError("buffer too small for nblocks")
        check(lib().revel_gpu_frame_full_blocks(self._h, blocks.ptr, nblocks, None))

    def synth_full_blocks(self, blocks: DeviceBuffer, nblocks: int, seed: int, first: int = 0) -> None:
        if blocks.nbytes < nblocks * BLOCK_SIZE:
            raise ValueError("buffer too small for nblocks")
        check(lib().revel_gpu_synth_full_blocks(self._h, blocks.ptr, nblocks, seed, first, None))

    def verify_image(self, image: DeviceBuffer, nbytes: int, base_offset: int = 0,
                     variant: Optional[int] = None, path: Optional[int] = None) -> np.ndarray:
        """Config C3: walk + CRC every physical record of a device-resident
        WAL image.  Returns a structured array (RECORD_DTYPE) in file order.
        path: a verify path of the test hook after the count pass (0 =
        production split, 1 = header walk without the count pass's lists, 2 =
        v3 with the lists, 3 = the round-4 split); or one of round 5's
        small-record kernels, kept in tools/experiments/libexperiments.so
        (not the product): "one_pass" / "one_pass2"
        (the one-pass count + checksum pair revel_x_fused_count_scan ->
        revel_x_fused_verify), "dense_chunks" / "dense_quad" / "dense_sorted"
        (the production split with k_verify_dense_chunks, dense2's
        quad-coalesced loads or round 6's length-sorted batches for the dense
        blocks); variant: an experiment arm of tools/experiments
        (DESIGN.md 4.2)."""
        if nbytes == 0:
            return np.zeros(0, dtype=RECORD_DTYPE)
        if image.nbytes < nbytes:
            raise ValueError("image buffer smaller than nbytes")
        nblocks = (nbytes + BLOCK_SIZE - 1) // BLOCK_SIZE
        counts = self.alloc(4 * nblocks)
        first = self.alloc(4 * nblocks)
        L = lib()
        one_pass = path in ("one_pass", "one_pass2")
        if one_pass:
            from ._lib import experiments  # round 5's one-pass kernels (tools/experiments)
            check(experiments().revel_x_fused_count_scan(self._h, 2 if path == "one_pass2" else 1, image.ptr, nbytes,
                                                         counts.ptr, first.ptr, None))
        else:
            check(L.revel_gpu_count_scan_records(self._h, image.ptr, nbytes, counts.ptr, first.ptr, None))
        tail_first = self.d2h(first, 4, np.uint32, src_offset=4 * (nblocks - 1))[0]
        tail_count = self.d2h(counts, 4, np.uint32, src_offset=4 * (nblocks - 1))[0]
        total = int(tail_first) + int(tail_count)
        out = self.alloc(max(1, total) * RECORD_DTYPE.itemsize)
        if variant is not None:
            from ._lib import experiments  # kernel variants kept for the record (tools/experiments)
            check(experiments().revel_x_verify_records_variant(self._h, variant, image.ptr, nbytes, base_offset,
                                                               first.ptr, out.ptr, None))
        elif one_pass:
            from ._lib import experiments
            check(experiments().revel_x_fused_verify(self._h, image.ptr, nbytes, base_offset, counts.ptr, first.ptr,
                                                     out.ptr, None))
        elif path in _DENSE_VARIANTS:
            from ._lib import experiments
            check(experiments().revel_x_verify_dense_variant(self._h, _DENSE_VARIANTS[path], image.ptr, nbytes,
                                                             base_offset, first.ptr, out.ptr, None))
        elif path is not None:
            check(L.revel_gpu_verify_records_path(self._h, path, image.ptr, nbytes, base_offset, first.ptr, out.ptr,
                                                  None))
        else:
            check(L.revel_gpu_verify_records(self._h, image.ptr, nbytes, base_offset, first.ptr, out.ptr, None))
        self.sync()
        res = self.d2h(out, total * RECORD_DTYPE.itemsize, np.uint8).view(RECORD_DTYPE)
        return res

    # ---- end-to-end replay (host -> pinned -> HBM -> verify) ----
    def replay_memory(self, image, base_offset: int = 0, full_blocks: bool = False, window_bytes: int = 64 << 20,
                      nbuffers: int = 4, io_threads: int = 8) -> dict:
        arr = np.frombuffer(image, dtype=np.uint8) if isinstance(image, (bytes, bytearray)) else image
        st = ReplayStats()
        check(lib().revel_gpu_replay_memory(self._h, arr.ctypes.data, arr.nbytes, base_offset,
                                            REPLAY_FULL_BLOCKS if full_blocks else REPLAY_RECORDS,
                                            window_bytes, nbuffers, io_threads, ctypes.byref(st)))
        return st.as_dict()

    def replay_file(self, path: str, offset: int = 0, length: int = 0, full_blocks: bool = False,
                    window_bytes: int = 64 << 20, nbuffers: int = 4, io_threads: int = 8, io: str = "mmap") -> dict:
        """io: "mmap" (page cache copied by the io threads; default), "pread"
        (buffered) or "direct" (O_DIRECT; RevelError NOT_SUPPORT where refused)."""
        st = ReplayStats()
        check(lib().revel_gpu_replay_file(self._h, path.encode(), offset, length,
                                          (REPLAY_FULL_BLOCKS if full_blocks else REPLAY_RECORDS) | REPLAY_IO[io],
                                          window_bytes, nbuffers, io_threads, ctypes.byref(st)))
        return st.as_dict()

    # ---- device append framing (batch add_record) ----
    def append_records(self, payloads: DeviceBuffer, lens, block_offset: int = 0):
        """Frame records on the GPU as successive Writer.add_record calls
        would; returns (image DeviceBuffer, image_len, new block_offset)."""
        lens = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64))
        L = lib()
        size = L.revel_log_framed_size(lens.ctypes.data, len(lens), block_offset)
        img = self.alloc(max(1, size))
        bo = ctypes.c_uint64(block_offset)
        n = ctypes.c_size_t()
        check(L.revel_gpu_append_records(self._h, payloads.ptr, lens.ctypes.data, len(lens), ctypes.byref(bo),
                                         img.ptr, img.nbytes, ctypes.byref(n), None))
        return img, n.value, bo.value

    # ---- device replay reassembly ----
    def reassemble_device(self, image: DeviceBuffer, nbytes: int, base_offset: int = 0, checksum: bool = True):
        """Verify + reassemble a device-resident WAL image, leaving the results
        in HBM: (events DeviceBuffer, nlogical, payload DeviceBuffer,
        payload_bytes, phys host array)."""
        phys = self.verify_image(image, nbytes, base_offset)
        n = len(phys)
        out = self.alloc(max(1, n) * LOGICAL_DTYPE.itemsize)
        pay = self.alloc(max(1, nbytes))
        if n == 0:
            return out, 0, pay, 0, phys
        dphys = self.upload(phys.view(np.uint8))
        nl, pb = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib().revel_gpu_reassemble(self._h, image.ptr, base_offset, nbytes, dphys.ptr, n, 1 if checksum else 0,
                                         out.ptr, pay.ptr, ctypes.byref(nl), ctypes.byref(pb), None))
        return out, nl.value, pay, pb.value, phys

    def reassemble(self, image: DeviceBuffer, nbytes: int, base_offset: int = 0, checksum: bool = True):
        """Verify + reassemble a device-resident WAL image on the GPU.  Returns
        (events: LOGICAL_DTYPE array, payload bytes: np.uint8 array, phys)."""
        out, nl, pay, pb, phys = self.reassemble_device(image, nbytes, base_offset, checksum)
        ev = self.d2h(out, nl * LOGICAL_DTYPE.itemsize).view(LOGICAL_DTYPE) if nl else np.zeros(0, LOGICAL_DTYPE)
        payload = self.d2h(pay, pb) if pb else np.zeros(0, np.uint8)
        return ev, payload, phys

    # ---- device WriteBatch decode ----
    def decode_batches_device(self, payload: DeviceBuffer, payload_bytes: int, events: DeviceBuffer, nlogical: int,
                              entries_cap: Optional[int] = None):
        """Decode every logical record as a WriteBatch on the GPU:
        (info DeviceBuffer, entries DeviceBuffer, nentries)."""
        cap = payload_bytes // 2 if entries_cap is None else entries_cap
        info = self.alloc(max(1, nlogical) * BATCH_INFO_DTYPE.itemsize)
        ent = self.alloc(max(1, cap) * BATCH_ENTRY_DTYPE.itemsize)
        ne = ctypes.c_uint64()
        check(lib().revel_gpu_decode_batches(self._h, payload.ptr, payload_bytes, events.ptr, nlogical, info.ptr,
                                             ent.ptr, cap, ctypes.byref(ne), None))
        return info, ent, ne.value

    def replay_batches(self, image: DeviceBuffer, nbytes: int, base_offset: int = 0, checksum: bool = True):
        """WAL image in HBM -> verified, reassembled, decoded WriteBatches.
        Returns (events, payload, infos BATCH_INFO_DTYPE, entries
        BATCH_ENTRY_DTYPE) as host arrays."""
        out, nl, pay, pb, _ = self.reassemble_device(image, nbytes, base_offset, checksum)
        ev = self.d2h(out, nl * LOGICAL_DTYPE.itemsize).view(LOGICAL_DTYPE) if nl else np.zeros(0, LOGICAL_DTYPE)
        payload = self.d2h(pay, pb) if pb else np.zeros(0, np.uint8)
        if nl == 0:
            return ev, payload, np.zeros(0, BATCH_INFO_DTYPE), np.zeros(0, BATCH_ENTRY_DTYPE)
        info, ent, ne = self.decode_batches_device(pay, pb, out, nl)
        infos = self.d2h(info, nl * BATCH_INFO_DTYPE.itemsize).view(BATCH_INFO_DTYPE)
        ents = self.d2h(ent, ne * BATCH_ENTRY_DTYPE.itemsize).view(BATCH_ENTRY_DTYPE) if ne else \
            np.zeros(0, BATCH_ENTRY_DTYPE)
        return ev, payload, infos, ents
