"""ctypes binding of oracle/build/liboracle.so (the plain-C restatement).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_int, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
_lib = None

VARIANTS = {"bytewise": 0, "slice16": 1, "sse42": 2}


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        for name in ("oracle_crc_bytewise", "oracle_crc_slice16", "oracle_crc_sse42"):
            getattr(L, name).restype = c_uint32
            getattr(L, name).argtypes = [c_uint32, c_void_p, c_size_t]
        L.oracle_value.restype = c_uint32
        L.oracle_value.argtypes = [c_void_p, c_size_t]
        L.oracle_extend.restype = c_uint32
        L.oracle_extend.argtypes = [c_uint8, c_void_p, c_size_t]
        L.oracle_mask.restype = c_uint32
        L.oracle_mask.argtypes = [c_uint32]
        L.oracle_unmask.restype = c_uint32
        L.oracle_unmask.argtypes = [c_uint32]
        L.oracle_full_block_crcs.restype = None
        L.oracle_full_block_crcs.argtypes = [c_void_p, c_size_t, c_void_p, c_int]
        L.oracle_write_image.restype = c_size_t
        L.oracle_write_image.argtypes = [c_void_p, c_void_p, c_size_t, POINTER(c_uint64), c_void_p, c_size_t]
        L.oracle_walk.restype = c_size_t
        L.oracle_walk.argtypes = [c_void_p, c_size_t] + [c_void_p] * 6 + [c_size_t]
        L.oracle_walk_v.restype = c_size_t
        L.oracle_walk_v.argtypes = [c_void_p, c_size_t] + [c_void_p] * 6 + [c_size_t, c_int]
        L.oracle_synth_full_blocks.restype = None
        L.oracle_synth_full_blocks.argtypes = [c_void_p, c_size_t, c_uint64, c_uint64]
        _lib = L
    return _lib


def value(data: bytes) -> int:
    return lib().oracle_value(data, len(data))


def extend(init: int, data: bytes) -> int:
    return lib().oracle_extend(init, data, len(data))


def mask(c: int) -> int:
    return lib().oracle_mask(c)


def full_block_crcs(blocks: np.ndarray, variant: str = "bytewise") -> np.ndarray:
    blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
    n = blocks.size // 32768
    out = np.empty(n, dtype=np.uint32)
    lib().oracle_full_block_crcs(blocks.ctypes.data, n, out.ctypes.data, VARIANTS[variant])
    return out


def write_image(records, block_offset: int = 0) -> bytes:
    payload = b"".join(records)
    lens = np.array([len(r) for r in records], dtype=np.uint64)
    cap = len(payload) + 7 * (len(records) + len(payload) // 32761 + 2) + 32768
    out = np.empty(cap, dtype=np.uint8)
    bo = c_uint64(block_offset)
    pbuf = np.frombuffer(payload, dtype=np.uint8) if payload else np.zeros(1, np.uint8)
    n = lib().oracle_write_image(pbuf.ctypes.data, lens.ctypes.data if len(lens) else None, len(records),
                                 ctypes.byref(bo), out.ctypes.data, cap)
    assert n != ctypes.c_size_t(-1).value
    return out[:n].tobytes()


WALK_DTYPE = np.dtype([("file_offset", "<u8"), ("length", "<u4"), ("type", "u1"), ("stored_crc", "<u4"),
                       ("computed_crc", "<u4"), ("status", "u1")])


def walk(image, variant: str = "bytewise") -> np.ndarray:
    """Every physical record: file_offset, length, type, stored, computed, status.
    image: bytes or a uint8 array; variant: the CRC implementation (bytewise =
    the reference crate's algorithm class; sse42 for GiB-sized images)."""
    if isinstance(image, np.ndarray):
        img = np.ascontiguousarray(image, dtype=np.uint8).ravel()
        n = img.size
    else:
        n = len(image)
        img = np.frombuffer(image, dtype=np.uint8) if image else None
    if n == 0:
        img = np.zeros(1, np.uint8)
    cap = max(1, n // 7 + 8)
    off = np.empty(cap, np.uint64); ln = np.empty(cap, np.uint32); ty = np.empty(cap, np.uint8)
    st = np.empty(cap, np.uint32); co = np.empty(cap, np.uint32); ss = np.empty(cap, np.uint8)
    k = lib().oracle_walk_v(img.ctypes.data, n, off.ctypes.data, ln.ctypes.data, ty.ctypes.data,
                            st.ctypes.data, co.ctypes.data, ss.ctypes.data, cap, VARIANTS[variant])
    assert k <= cap
    out = np.empty(k, dtype=WALK_DTYPE)
    out["file_offset"], out["length"], out["type"] = off[:k], ln[:k], ty[:k]
    out["stored_crc"], out["computed_crc"], out["status"] = st[:k], co[:k], ss[:k]
    return out


def synth_full_blocks(n: int, seed: int = 0x5EED0002, first: int = 0) -> np.ndarray:
    out = np.empty((n, 32768), dtype=np.uint8)
    lib().oracle_synth_full_blocks(out.ctypes.data, n, seed, first)
    return out
