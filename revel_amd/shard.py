"""One WAL across several GPUs (include/revel_wal.h, "one WAL across several
GPUs"; config C5 on N GPUs), via the C-ABI.

Physical records never cross a 32 KiB block (log_writer.rs:66-76), so a WAL
splits into contiguous block-aligned shards that are verified and reassembled
independently, one per GPU, with no collective.  Only logical records whose
fragments span a shard boundary need the neighbours: each shard keeps its
boundary records, and a host stitch folds them in file order with the reader's
rules (log_reader.rs:95-129).

* :func:`block_ranges`      -- ``revel_wal_shard_ranges``
* :class:`WalShard`         -- one shard loaded + verified (+ reassembled) on one GPU
* :func:`boundary_host`     -- a shard's boundary from a host header walk (no GPU, no CRC)
* :class:`Stitch`           -- the host stitch of the shards' boundary blobs
* :class:`ShardedReplay`    -- all shards in one process (one host thread per context),
  iterated like ``Reader.read_record``.
"""
from __future__ import annotations

import ctypes
from ctypes import c_int, c_size_t, c_uint64, c_void_p
from typing import List, Optional, Sequence, Tuple

import numpy as np

from ._lib import SHARD_READ, SHARD_VERIFY, ShardInfo, WalSummary, check, lib


def block_ranges(nbytes: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous block-aligned byte ranges, one per rank (some may be empty)."""
    offs = (c_uint64 * (world + 1))()
    check(lib().revel_wal_shard_ranges(nbytes, world, offs))
    return [(offs[k], offs[k + 1]) for k in range(world)]


def _src(image):
    if image is None:
        return None, None
    arr = np.frombuffer(image, dtype=np.uint8) if isinstance(image, (bytes, bytearray, memoryview)) else image
    return arr, arr.ctypes.data


def boundary_host(image, offset: int, length: int, read: bool = True) -> bytes:
    """Boundary blob of shard [offset, offset + length) of the WAL ``image``
    from a host header walk (a Reader with checksum == false)."""
    arr, ptr = _src(image)
    n = c_size_t()
    flags = SHARD_READ if read else SHARD_VERIFY
    check(lib().revel_wal_shard_boundary_host(ptr, arr.nbytes, offset, length, flags, None, 0, ctypes.byref(n)))
    buf = ctypes.create_string_buffer(n.value)
    check(lib().revel_wal_shard_boundary_host(ptr, arr.nbytes, offset, length, flags, buf, n.value, ctypes.byref(n)))
    return buf.raw[:n.value]


class Stitch:
    """Host stitch of boundary blobs given in file order."""

    def __init__(self, blobs: Sequence[bytes]):
        n = len(blobs)
        keep = [ctypes.create_string_buffer(b, len(b)) for b in blobs]
        ptrs = (c_void_p * n)(*[ctypes.addressof(k) for k in keep])
        sizes = (c_size_t * n)(*[len(b) for b in blobs])
        h = c_void_p()
        check(lib().revel_wal_stitch_new(ptrs, sizes, n, ctypes.byref(h)))
        self._h = h.value

    def summary(self) -> dict:
        s = WalSummary()
        check(lib().revel_wal_stitch_summary(self._h, ctypes.byref(s)))
        return s.as_dict()

    def records(self) -> List[Tuple[int, Optional[bytes], int]]:
        """(file_offset, payload or None in VERIFY mode, before_shard) per
        stitched record, in file order."""
        out = []
        for i in range(self.summary()["stitched"]):
            off, p, n, before = c_uint64(), c_void_p(), c_uint64(), c_int()
            check(lib().revel_wal_stitch_record(self._h, i, ctypes.byref(off), ctypes.byref(p), ctypes.byref(n),
                                                ctypes.byref(before)))
            data = ctypes.string_at(p.value, n.value) if p.value else (b"" if n.value == 0 else None)
            out.append((off.value, data, before.value))
        return out

    def __del__(self):
        if getattr(self, "_h", None):
            lib().revel_wal_stitch_free(self._h)
            self._h = None


class WalShard:
    """Shard [offset, offset + length) of a WAL (file ``path`` or host
    ``image``) loaded into HBM of ``ctx``'s GPU, verified, and with
    ``read=True`` reassembled (revel_gpu_wal_shard_load)."""

    def __init__(self, ctx, offset: int, length: int, path: Optional[str] = None, image=None, file_bytes: int = 0,
                 checksum: bool = True, read: bool = True, window_bytes: int = 0, io_threads: int = 8):
        self._ctx = ctx
        arr, ptr = _src(image)
        self._arr = arr
        if arr is not None and not file_bytes:
            file_bytes = arr.nbytes
        h = c_void_p()
        check(lib().revel_gpu_wal_shard_load(ctx.handle, path.encode() if path else None, ptr, file_bytes, offset,
                                             length, 1 if checksum else 0, SHARD_READ if read else SHARD_VERIFY,
                                             window_bytes, io_threads, ctypes.byref(h)))
        self._h = h.value

    def info(self) -> dict:
        s = ShardInfo()
        check(lib().revel_wal_shard_info_get(self._h, ctypes.byref(s)))
        return s.as_dict()

    def boundary(self) -> bytes:
        n = c_size_t()
        check(lib().revel_wal_shard_boundary(self._h, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value)
        check(lib().revel_wal_shard_boundary(self._h, buf, n.value, ctypes.byref(n)))
        return buf.raw[:n.value]

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().revel_wal_shard_free(self._h)
            self._h = None

    def __del__(self):
        self.close()


class ShardedReplay:
    """revel_gpu_replay_sharded: the WAL split over ``ctxs`` (one shard and host
    thread each) and stitched.  ``read_record`` / iteration return the logical
    records in file order as ``log.Reader`` does (RevelError(IOError) per
    error event, None at the end)."""

    def __init__(self, ctxs: Sequence, path: Optional[str] = None, image=None, file_bytes: int = 0,
                 checksum: bool = True, read: bool = True, window_bytes: int = 0, io_threads: int = 8):
        self._ctxs = list(ctxs)
        arr, ptr = _src(image)
        self._arr = arr
        if arr is not None and not file_bytes:
            file_bytes = arr.nbytes
        handles = (c_void_p * len(ctxs))(*[c.handle for c in ctxs])
        h = c_void_p()
        check(lib().revel_gpu_replay_sharded(handles, len(ctxs), path.encode() if path else None, ptr, file_bytes,
                                             1 if checksum else 0, SHARD_READ if read else SHARD_VERIFY,
                                             window_bytes, io_threads, ctypes.byref(h)))
        self._h = h.value

    def summary(self) -> dict:
        s = WalSummary()
        check(lib().revel_sharded_replay_summary(self._h, ctypes.byref(s)))
        return s.as_dict()

    def shard_info(self, k: int) -> dict:
        sh = lib().revel_sharded_replay_shard(self._h, k)
        if not sh:
            raise IndexError(k)
        s = ShardInfo()
        check(lib().revel_wal_shard_info_get(sh, ctypes.byref(s)))
        return s.as_dict()

    def read_record(self) -> Optional[bytes]:
        p, n, off = c_void_p(), c_size_t(), c_uint64()
        check(lib().revel_sharded_replay_next(self._h, ctypes.byref(p), ctypes.byref(n), ctypes.byref(off)))
        if not p.value:
            return None
        return ctypes.string_at(p.value, n.value) if n.value else b""

    def __iter__(self):
        while True:
            r = self.read_record()
            if r is None:
                return
            yield r

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().revel_sharded_replay_free(self._h)
            self._h = None

    def __del__(self):
        self.close()
