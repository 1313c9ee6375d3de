"""Block-aligned sharding of one WAL across GPUs and host-side stitching.

Physical records never cross a 32 KiB block (log_writer.rs:66-76), so any
block-aligned split is exact for CRC compute/verify: each rank verifies its
range independently (no collective).  Only logical-record reassembly crosses
shards (a FIRST in shard k whose LAST is in shard k+1); that is done on the
host over the ranks' physical-record lists concatenated in file order, with
the same FULL/FIRST/MIDDLE/LAST rules as log_reader.rs:95-129.
"""
from __future__ import annotations

from typing import Iterable, List, Sequence, Tuple

from ._lib import BLOCK_SIZE, FIRST_TYPE, FULL_TYPE, HEADER_SIZE, LAST_TYPE, MIDDLE_TYPE

PhysRec = Tuple[int, int, int, bytes]  # (file_offset, type, status, payload)


def block_ranges(nbytes: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous block-aligned byte ranges, one per rank (some may be empty)."""
    nblocks = (nbytes + BLOCK_SIZE - 1) // BLOCK_SIZE
    per = (nblocks + world - 1) // world if world else 0
    out = []
    for r in range(world):
        s = min(nbytes, r * per * BLOCK_SIZE)
        e = min(nbytes, (r + 1) * per * BLOCK_SIZE)
        out.append((s, e))
    return out


def physical_records(image: bytes, base_offset: int = 0) -> List[PhysRec]:
    """Host header walk (no CRC) of a block-aligned piece of a WAL; status as
    in revel_record_result (0 ok, 2 bad length, 3 zero record)."""
    out: List[PhysRec] = []
    n = len(image)
    for b in range(0, n, BLOCK_SIZE):
        bl = min(BLOCK_SIZE, n - b)
        off = 0
        while bl - off >= HEADER_SIZE:
            h = image[b + off:b + off + HEADER_SIZE]
            ln = h[4] | (h[5] << 8)
            t = h[6]
            if HEADER_SIZE + ln > bl - off:
                out.append((base_offset + b + off, t, 2, b""))
                break
            if t == 0 and ln == 0:
                out.append((base_offset + b + off, 0, 3, b""))
                break
            s = b + off + HEADER_SIZE
            out.append((base_offset + b + off, t, 0, bytes(image[s:s + ln])))
            off += HEADER_SIZE + ln
    return out


def reassemble(records: Iterable[PhysRec]) -> List[bytes]:
    """Logical records from physical ones in file order (bad records skipped)."""
    out: List[bytes] = []
    scratch = bytearray()
    in_frag = False
    for _, t, st, payload in records:
        if st != 0:
            in_frag = False
            scratch.clear()
            continue
        if t == FULL_TYPE:
            out.append(payload)
            in_frag = False
        elif t == FIRST_TYPE:
            scratch = bytearray(payload)
            in_frag = True
        elif t == MIDDLE_TYPE:
            if in_frag:
                scratch += payload
        elif t == LAST_TYPE:
            if in_frag:
                scratch += payload
                out.append(bytes(scratch))
            in_frag = False
    return out


def stitch(per_rank: Sequence[Sequence[PhysRec]]) -> List[bytes]:
    """Concatenate the ranks' physical records (rank order = file order)."""
    allrecs: List[PhysRec] = []
    for recs in per_rank:
        allrecs.extend(recs)
    return reassemble(allrecs)
