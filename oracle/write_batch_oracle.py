"""WriteBatch encode/decode restated from the reference -- TEST INFRASTRUCTURE ONLY.

Reference: guimingyue/revel @ v0, ``src/write_batch.rs``, ``src/coding.rs``,
``src/dbformat.rs``.

Layout (write_batch.rs:18-77, LevelDB's): ``rep[0:8]`` sequence (fixed64 LE,
set_sequence :67-69), ``rep[8:12]`` count (fixed32 LE, count/set_count
:160-166), then ``count`` entries: ``tag`` (dbformat.rs:24-38 ValueType:
1 = kTypeValue, 0 = kTypeDeletion), ``varint32 key_len, key`` and, for a value,
``varint32 value_len, value`` (put :44-49, delete :51-55;
put_length_prefixed_slice coding.rs:152-157; varints coding.rs:18-49,96-123).
Entry i is applied with sequence ``seq + i`` (MemTableInserter :148-158,
insert_into :178-181; db.rs:95-112 sets the sequence before logging).

Reference defects NOT reproduced (LevelDB semantics instead):
* ``sequence()`` decodes fixed64 at rep[8..] (write_batch.rs:168-170) -- the
  count field and 4 bytes past the header -- instead of offset 0.
* ``iterate`` (:79-128): the deletion branch parses the key from the TAG byte
  (``input.data()``, :112) and never advances (no remove_prefix) -> infinite
  loop; a Put whose key or value fails to parse never advances either; an
  unknown tag panics (dbformat.rs:36); a length past the end panics
  (coding.rs:161); the found != count check does nothing (:123-127).
  The restatement advances past every entry and reports errors as LevelDB's
  WriteBatch::Iterate does: too small (< 12 B), bad entry (key/value varint or
  length out of range), unknown tag, wrong count -- returning the entries
  decoded before the error, as LevelDB has already handed them to the
  memtable by then.
"""
from __future__ import annotations

import struct
from typing import List, Optional, Tuple

K_HEADER = 12
TYPE_DELETION, TYPE_VALUE = 0, 1
OK, TOO_SMALL, BAD_ENTRY, BAD_TAG, WRONG_COUNT = 0, 1, 2, 3, 4


def put_varint32(v: int) -> bytes:
    """coding.rs:18-49 (encode_varint32)."""
    out = bytearray()
    while v >= 128:
        out.append((v & 127) | 128)
        v >>= 7
    out.append(v)
    return bytes(out)


def get_varint32(buf: bytes, off: int, limit: int) -> Optional[Tuple[int, int]]:
    """coding.rs:96-123 -> (value, bytes used) or None."""
    result, shift, p = 0, 0, off
    while shift <= 28 and p < limit:
        b = buf[p]
        p += 1
        if b & 128:
            result |= (b & 127) << shift
        else:
            result |= b << shift
            return result & 0xFFFFFFFF, p - off
        shift += 7
    return None


class WriteBatch:
    def __init__(self):
        self.rep = bytearray(K_HEADER)

    def count(self) -> int:
        return struct.unpack_from("<I", self.rep, 8)[0]

    def _set_count(self, n: int) -> None:
        struct.pack_into("<I", self.rep, 8, n)

    def put(self, key: bytes, value: bytes) -> None:        # write_batch.rs:44-49
        self._set_count(self.count() + 1)
        self.rep.append(TYPE_VALUE)
        self.rep += put_varint32(len(key)) + key
        self.rep += put_varint32(len(value)) + value

    def delete(self, key: bytes) -> None:                    # write_batch.rs:51-55
        self._set_count(self.count() + 1)
        self.rep.append(TYPE_DELETION)
        self.rep += put_varint32(len(key)) + key

    def set_sequence(self, seq: int) -> None:                # write_batch.rs:67-69
        struct.pack_into("<Q", self.rep, 0, seq)

    def contents(self) -> bytes:
        return bytes(self.rep)


Entry = Tuple[int, int, bytes, bytes]  # (sequence, type, key, value)


def decode(rep: bytes) -> Tuple[int, int, int, List[Entry]]:
    """-> (status, sequence, count, entries), LevelDB WriteBatch::Iterate +
    MemTableInserter sequences."""
    if len(rep) < K_HEADER:
        return TOO_SMALL, 0, 0, []
    seq = struct.unpack_from("<Q", rep, 0)[0]
    count = struct.unpack_from("<I", rep, 8)[0]
    p, n = K_HEADER, len(rep)
    out: List[Entry] = []
    while p < n:
        tag = rep[p]
        p += 1
        if tag not in (TYPE_VALUE, TYPE_DELETION):
            return BAD_TAG, seq, count, out
        kv = get_varint32(rep, p, n)
        if kv is None or p + kv[1] + kv[0] > n:
            return BAD_ENTRY, seq, count, out
        klen, used = kv
        p += used
        key = bytes(rep[p:p + klen])
        p += klen
        val = b""
        if tag == TYPE_VALUE:
            vv = get_varint32(rep, p, n)
            if vv is None or p + vv[1] + vv[0] > n:
                return BAD_ENTRY, seq, count, out
            vlen, used = vv
            p += used
            val = bytes(rep[p:p + vlen])
            p += vlen
        out.append(((seq + len(out)) & 0xFFFFFFFFFFFFFFFF, tag, key, val))
    if len(out) != count:
        return WRONG_COUNT, seq, count, out
    return OK, seq, count, out
