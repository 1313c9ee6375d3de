"""ctypes binding of ``librevel_wal.so`` (the C-ABI in include/revel_wal.h).

The library is built in-tree (``make -C revel_amd/csrc``, or
``__graft_entry__.build()``).  Loading fails loudly if it is missing: there
is no Python or CPU fallback for anything behind it.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, c_char_p, c_float, c_int, c_size_t, c_uint8, c_uint32,
                    c_uint64, c_void_p)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librevel_wal.so")

# status codes: src/error.rs:16-23
OK, NOT_FOUND, CORRUPTION, NOT_SUPPORT, INVALID_ARGUMENT, IO_ERROR = 0, 1, 2, 3, 4, 5
ERROR_NAMES = {1: "NotFound", 2: "Corruption", 3: "NotSupport", 4: "InvalidArgument", 5: "IOError"}

BLOCK_SIZE = 32768
HEADER_SIZE = 7
ZERO_TYPE, FULL_TYPE, FIRST_TYPE, MIDDLE_TYPE, LAST_TYPE = 0, 1, 2, 3, 4
REC_OK, REC_BAD_CHECKSUM, REC_BAD_LENGTH, REC_ZERO = 0, 1, 2, 3


class RecordResult(Structure):
    _fields_ = [("file_offset", c_uint64), ("length", c_uint32), ("stored_crc", c_uint32),
                ("computed_crc", c_uint32), ("type", c_uint8), ("status", c_uint8),
                ("reserved", c_uint8 * 2)]


assert ctypes.sizeof(RecordResult) == 24


class ReplayStats(Structure):
    _fields_ = [("bytes", c_uint64), ("windows", c_uint64), ("units", c_uint64), ("bad", c_uint64),
                ("first_bad_offset", c_uint64), ("seconds", ctypes.c_double), ("read_seconds", ctypes.c_double),
                ("h2d_ms", ctypes.c_double), ("kernel_ms", ctypes.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


REPLAY_RECORDS, REPLAY_FULL_BLOCKS = 0, 1
SHARD_VERIFY, SHARD_READ = 0, 1


class ShardInfo(Structure):
    _fields_ = [("device", c_int), ("checksum", c_int), ("offset", c_uint64), ("length", c_uint64),
                ("file_bytes", c_uint64), ("physical", c_uint64), ("bad", c_uint64), ("events", c_uint64),
                ("records", c_uint64), ("payload_bytes", c_uint64), ("d_image", c_void_p), ("d_phys", c_void_p),
                ("d_events", c_void_p), ("d_payload", c_void_p), ("setup_seconds", ctypes.c_double),
                ("seconds", ctypes.c_double),
                ("read_seconds", ctypes.c_double), ("h2d_ms", ctypes.c_double), ("kernel_ms", ctypes.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class WalSummary(Structure):
    _fields_ = [("bytes", c_uint64), ("physical", c_uint64), ("bad", c_uint64), ("records", c_uint64),
                ("errors", c_uint64), ("payload_bytes", c_uint64), ("stitched", c_uint64),
                ("seconds", ctypes.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}
REPLAY_IO = {"mmap": 0x00, "pread": 0x10, "direct": 0x20}


class LogicalRecord(Structure):
    _fields_ = [("file_offset", c_uint64), ("payload_offset", c_uint64), ("length", c_uint32),
                ("first_phys", c_uint32), ("last_phys", c_uint32), ("status", c_uint8), ("reserved", c_uint8 * 3)]


assert ctypes.sizeof(LogicalRecord) == 32
LOGICAL_OK, LOGICAL_BAD_TYPE = 0, 4
BATCH_HEADER = 12
TYPE_DELETION, TYPE_VALUE = 0, 1
BATCH_OK, BATCH_TOO_SMALL, BATCH_BAD_ENTRY, BATCH_BAD_TAG, BATCH_WRONG_COUNT, BATCH_NOT_RECORD = 0, 1, 2, 3, 4, 5

# callback types of the caller-implemented files (revel_wal.h)
APPEND_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p, c_size_t)
FILE_OP_FN = ctypes.CFUNCTYPE(c_int, c_void_p)
RELEASE_FN = ctypes.CFUNCTYPE(None, c_void_p)
READ_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p, c_size_t, POINTER(c_size_t))
SKIP_FN = ctypes.CFUNCTYPE(c_int, c_void_p, c_uint64)

# name -> (restype, argtypes); every symbol declared in include/revel_wal.h
SIGNATURES = {
    "revel_crc32c_value": (c_uint32, [c_void_p, c_size_t]),
    "revel_crc32c_extend": (c_uint32, [c_uint8, c_void_p, c_size_t]),
    "revel_crc32c_mask": (c_uint32, [c_uint32]),
    "revel_crc32c_unmask": (c_uint32, [c_uint32]),
    "revel_memory_writable_file_new": (c_void_p, []),
    "revel_posix_writable_file_new": (c_int, [c_char_p, POINTER(c_void_p)]),
    "revel_writable_file_append": (c_int, [c_void_p, c_void_p, c_size_t]),
    "revel_writable_file_flush": (c_int, [c_void_p]),
    "revel_writable_file_close": (c_int, [c_void_p]),
    "revel_writable_file_sync": (c_int, [c_void_p]),
    "revel_memory_writable_file_contents": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_size_t)]),
    "revel_writable_file_free": (None, [c_void_p]),
    "revel_writable_file_from_callbacks": (c_int, [c_void_p, APPEND_FN, FILE_OP_FN, FILE_OP_FN, FILE_OP_FN,
                                                   RELEASE_FN, POINTER(c_void_p)]),
    "revel_sequential_file_from_callbacks": (c_int, [c_void_p, READ_FN, SKIP_FN, RELEASE_FN, POINTER(c_void_p)]),
    "revel_memory_sequential_file_new": (c_void_p, [c_void_p, c_size_t]),
    "revel_posix_sequential_file_new": (c_int, [c_char_p, POINTER(c_void_p)]),
    "revel_sequential_file_read": (c_int, [c_void_p, c_void_p, c_size_t, POINTER(c_size_t)]),
    "revel_sequential_file_skip": (c_int, [c_void_p, c_uint64]),
    "revel_sequential_file_free": (None, [c_void_p]),
    "revel_log_writer_new": (c_void_p, [c_void_p, c_uint64]),
    "revel_log_writer_add_record": (c_int, [c_void_p, c_void_p, c_size_t]),
    "revel_log_writer_block_offset": (c_uint64, [c_void_p]),
    "revel_log_writer_free": (None, [c_void_p]),
    "revel_gpu_device_count": (c_int, [POINTER(c_int)]),
    "revel_gpu_context_new": (c_int, [c_int, POINTER(c_void_p)]),
    "revel_gpu_context_free": (None, [c_void_p]),
    "revel_gpu_context_stream": (c_void_p, [c_void_p]),
    "revel_gpu_context_trim": (c_int, [c_void_p]),
    "revel_log_reader_new": (c_int, [c_void_p, c_int, c_uint64, c_void_p, c_size_t, POINTER(c_void_p)]),
    "revel_log_reader_read_record": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_size_t)]),
    "revel_gpu_device_pci_bus_id": (c_int, [c_int, c_char_p, c_size_t]),
    "revel_build_info": (c_char_p, []),
    "revel_log_reader_read_record_into": (c_int, [c_void_p, c_void_p, c_size_t, POINTER(c_size_t), POINTER(c_int)]),
    "revel_log_reader_last_record_offset": (c_uint64, [c_void_p]),
    "revel_log_reader_free": (None, [c_void_p]),
    "revel_gpu_crc_full_blocks": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p]),
    "revel_gpu_frame_full_blocks": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "revel_gpu_count_records": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p, c_void_p]),
    "revel_gpu_count_scan_records": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p]),
    "revel_gpu_exclusive_scan_u32": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "revel_gpu_verify_records": (c_int, [c_void_p, c_void_p, c_size_t, c_uint64, c_void_p, c_void_p, c_void_p]),
    "revel_gpu_malloc": (c_int, [c_void_p, c_size_t, POINTER(c_void_p)]),
    "revel_gpu_free": (c_int, [c_void_p, c_void_p]),
    "revel_gpu_host_alloc": (c_int, [c_void_p, c_size_t, POINTER(c_void_p)]),
    "revel_gpu_host_free": (c_int, [c_void_p, c_void_p]),
    "revel_gpu_memcpy_h2d": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "revel_gpu_memcpy_d2h": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "revel_gpu_memset": (c_int, [c_void_p, c_void_p, c_int, c_size_t, c_void_p]),
    "revel_gpu_stream_synchronize": (c_int, [c_void_p, c_void_p]),
    "revel_gpu_device_synchronize": (c_int, [c_void_p]),
    "revel_gpu_synth_full_blocks": (c_int, [c_void_p, c_void_p, c_size_t, c_uint64, c_uint64, c_void_p]),
    "revel_gpu_event_new": (c_int, [c_void_p, POINTER(c_void_p)]),
    "revel_gpu_event_record": (c_int, [c_void_p, c_void_p, c_void_p]),
    "revel_gpu_event_elapsed_ms": (c_int, [c_void_p, c_void_p, c_void_p, POINTER(c_float)]),
    "revel_gpu_event_free": (c_int, [c_void_p, c_void_p]),
    "revel_last_error": (c_char_p, []),
    "revel_gpu_reassemble": (c_int, [c_void_p, c_void_p, c_uint64, c_uint64, c_void_p, c_size_t, c_int, c_void_p,
                                     c_void_p, POINTER(c_uint64), POINTER(c_uint64), c_void_p]),
    "revel_gpu_decode_batches": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_size_t, c_void_p, c_void_p,
                                         c_size_t, POINTER(c_uint64), c_void_p]),
    "revel_log_framed_size": (c_uint64, [c_void_p, c_size_t, c_uint64]),
    "revel_gpu_append_records": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, POINTER(c_uint64), c_void_p,
                                         c_size_t, POINTER(c_size_t), c_void_p]),
    "revel_gpu_replay_file": (c_int, [c_void_p, c_char_p, c_uint64, c_uint64, c_int, c_size_t, c_int, c_int,
                                      POINTER(ReplayStats)]),
    "revel_gpu_replay_memory": (c_int, [c_void_p, c_void_p, c_uint64, c_uint64, c_int, c_size_t, c_int, c_int,
                                        POINTER(ReplayStats)]),
    "revel_wal_shard_ranges": (c_int, [c_uint64, c_int, c_void_p]),
    "revel_gpu_wal_shard_load": (c_int, [c_void_p, c_char_p, c_void_p, c_uint64, c_uint64, c_uint64, c_int, c_int,
                                         c_size_t, c_int, POINTER(c_void_p)]),
    "revel_wal_shard_info_get": (c_int, [c_void_p, POINTER(ShardInfo)]),
    "revel_wal_shard_boundary": (c_int, [c_void_p, c_void_p, c_size_t, POINTER(c_size_t)]),
    "revel_wal_shard_free": (None, [c_void_p]),
    "revel_wal_shard_boundary_host": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_int, c_void_p, c_size_t,
                                              POINTER(c_size_t)]),
    "revel_wal_stitch_new": (c_int, [c_void_p, c_void_p, c_int, POINTER(c_void_p)]),
    "revel_wal_stitch_summary": (c_int, [c_void_p, POINTER(WalSummary)]),
    "revel_wal_stitch_record": (c_int, [c_void_p, c_size_t, POINTER(c_uint64), POINTER(c_void_p), POINTER(c_uint64),
                                        POINTER(c_int)]),
    "revel_wal_stitch_free": (None, [c_void_p]),
    "revel_gpu_replay_sharded": (c_int, [c_void_p, c_int, c_char_p, c_void_p, c_uint64, c_int, c_int, c_size_t, c_int,
                                         POINTER(c_void_p)]),
    "revel_sharded_replay_summary": (c_int, [c_void_p, POINTER(WalSummary)]),
    "revel_sharded_replay_shard": (c_void_p, [c_void_p, c_int]),
    "revel_sharded_replay_next": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_size_t), POINTER(c_uint64)]),
    "revel_sharded_replay_free": (None, [c_void_p]),
}

# exported test hooks (not part of the public header): the verify paths, the u32 record-index
# guard on a synthetic counts array, the one-pass / two-read A/B switch
EXTRA_SIGNATURES = {
    "revel_gpu_verify_records_path": (c_int, [c_void_p, c_int, c_void_p, c_size_t, c_uint64, c_void_p,
                                              c_void_p, c_void_p]),
    "revel_debug_check_record_index": (c_int, [c_void_p, c_void_p, c_size_t]),
}

# tools/experiments/libexperiments.so: kernel variants kept for the record
EXPERIMENT_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "experiments",
                               "libexperiments.so")
EXPERIMENT_SIGNATURES = {
    "revel_x_crc_full_blocks_variant": (c_int, [c_void_p, c_int, c_void_p, c_size_t, c_void_p, c_void_p,
                                                c_void_p]),
    "revel_x_verify_records_variant": (c_int, [c_void_p, c_int, c_void_p, c_size_t, c_uint64, c_void_p,
                                               c_void_p, c_void_p]),
    "revel_x_walk_count_scan": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p]),
    "revel_x_walk_verify": (c_int, [c_void_p, c_void_p, c_size_t, c_uint64, c_void_p, c_void_p, c_void_p,
                                    c_void_p]),
    "revel_x_fused_count_scan": (c_int, [c_void_p, c_int, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p]),
    "revel_x_fused_verify": (c_int, [c_void_p, c_void_p, c_size_t, c_uint64, c_void_p, c_void_p, c_void_p,
                                     c_void_p]),
    "revel_x_verify_dense_variant": (c_int, [c_void_p, c_int, c_void_p, c_size_t, c_uint64, c_void_p, c_void_p,
                                             c_void_p]),
}
_xlib = None


def experiments() -> ctypes.CDLL:
    """The experiment library (built by `make -C tools/experiments`); the
    product never loads it."""
    global _xlib
    if _xlib is None:
        if not os.path.exists(EXPERIMENT_PATH):
            raise RuntimeError(f"{EXPERIMENT_PATH} is missing: `make -C tools/experiments`")
        L = ctypes.CDLL(EXPERIMENT_PATH)
        for name, (res, args) in EXPERIMENT_SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _xlib = L
    return _xlib

_lib = None


class RevelError(RuntimeError):
    """A non-zero status from the C-ABI (codes of src/error.rs:16-23)."""

    def __init__(self, code: int, what: str = ""):
        self.code = code
        name = ERROR_NAMES.get(code, f"status {code}")
        super().__init__(f"{name}: {what}" if what else name)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `make -C revel_amd/csrc` or "
                "`python -c 'import __graft_entry__ as g; g.build()'` (there is no fallback)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in {**SIGNATURES, **EXTRA_SIGNATURES}.items():
            if name in EXTRA_SIGNATURES and not hasattr(L, name):
                continue  # a test / A-B hook an older build (tools/ab_libs_c3.sh) does not export
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != OK:
        msg = lib().revel_last_error()
        raise RevelError(rc, msg.decode() if msg else "")
