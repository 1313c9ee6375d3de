"""CRC-32C surface of src/util/crc.rs:13-44, via the C-ABI."""
from __future__ import annotations

from ._lib import lib


def value(data: bytes) -> int:
    """crc.rs:17-19 ``value(data)``."""
    return lib().revel_crc32c_value(data, len(data))


def extend(init: int, data: bytes) -> int:
    """crc.rs:22-27 ``extend(init, data)`` -- ``init`` is a prefix byte."""
    return lib().revel_crc32c_extend(init & 0xFF, data, len(data))


def mask(crc: int) -> int:
    """crc.rs:36-38."""
    return lib().revel_crc32c_mask(crc & 0xFFFFFFFF)


def unmask(masked: int) -> int:
    """crc.rs:41-44."""
    return lib().revel_crc32c_unmask(masked & 0xFFFFFFFF)
