"""CPU restatement of Revel's WAL CRC path -- TEST INFRASTRUCTURE ONLY.

This module is the parity *oracle*.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker.
The shipped product (``revel_amd`` + ``librevel_wal.so``) never imports,
links or calls anything under ``oracle/``.

What it restates (reference = guimingyue/revel @ v0, read-only at /root/reference):

* ``src/util/crc.rs:13-15``  -- ``Crc::<u32>::new(&CRC_32_ISCSI)`` from the
  third-party crate ``crc`` (``Cargo.toml:17-18``: ``crc="3.0.0"``, caret
  requirement, Cargo.lock not committed so the 3.x patch is unpinned; the
  crate source is NOT present here).  The published CRC_32_ISCSI catalogue
  entry is: width=32, poly=0x1EDC6F41, init=0xFFFFFFFF, refin=true,
  refout=true, xorout=0xFFFFFFFF, check("123456789")=0xE3069283.  The crate
  computes it with a 256-entry reflected lookup table, one byte per step;
  that is what ``_TABLE``/``value`` below do.
* ``src/util/crc.rs:17-19``  ``value``      -> :func:`value`
* ``src/util/crc.rs:21-27``  ``extend``     -> :func:`extend` (prefix *byte*,
  pinned by the reference test ``crc.rs:83-86``)
* ``src/util/crc.rs:29-44``  ``mask``/``unmask`` -> :func:`mask`/:func:`unmask`
* ``src/coding.rs:51-62`` ``encode_fixed32``, ``src/coding.rs:139-144``
  ``decode_fix32``
* ``src/log_format.rs:14-30`` record types / block + header sizes
* ``src/log_writer.rs:58-124`` ``Writer::add_record`` / ``emit_physical_record``
  -> :class:`LogWriter`
* ``src/log_reader.rs:76-216`` -> :func:`walk_records` / :class:`LogReader`,
  restated with LevelDB-correct semantics (CRC over ``type||payload[:len]`` of
  every physical record, every record of a block walked).  The reference's own
  reader is block-granular and checks ``buf[6..read_len]`` (SURVEY.md
  Appendix A, defects 1-3); on every input where the reference reader is
  well-defined (one physical record per block read, e.g. config C2 and the
  18-byte golden image of ``log_reader.rs:231``) both agree.

Parity is pinned by the reference's own known-answer tests
(``crc.rs:50-108``, ``log_reader.rs:229-241``), checked in
``tests/test_oracle.py``.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Iterable, List, Optional, Tuple

import numpy as np

# --- CRC_32_ISCSI parameters (crate `crc` catalogue; crc.rs:13-15) ----------
POLY = 0x1EDC6F41                   # normal form
POLY_REFLECTED = 0x82F63B78         # bit-reversed, what a refin/refout table uses
INIT = 0xFFFFFFFF
XOROUT = 0xFFFFFFFF
CHECK = 0xE3069283                  # CRC of b"123456789"

# --- log_format.rs:14-30 ----------------------------------------------------
ZERO_TYPE, FULL_TYPE, FIRST_TYPE, MIDDLE_TYPE, LAST_TYPE = 0, 1, 2, 3, 4
MAX_RECORD_TYPE = LAST_TYPE
BLOCK_SIZE = 32768
HEADER_SIZE = 7

# --- crc.rs:29 --------------------------------------------------------------
MASK_DELTA = 0xA282EAD8


def _make_table() -> List[int]:
    table = []
    for n in range(256):
        c = n
        for _ in range(8):
            c = (c >> 1) ^ POLY_REFLECTED if c & 1 else c >> 1
        table.append(c)
    return table


_TABLE = _make_table()
TABLE_NP = np.array(_TABLE, dtype=np.uint32)


def crc_update(state: int, data: bytes) -> int:
    """One-byte-per-step reflected table walk (the crate's algorithm class).

    ``state`` is the raw register (no init/xorout applied)."""
    t = _TABLE
    for b in data:
        state = t[(state ^ b) & 0xFF] ^ (state >> 8)
    return state


def value(data: bytes) -> int:
    """crc.rs:17-19 -- ``CASTAGNOLI.checksum(data)``."""
    return crc_update(INIT, data) ^ XOROUT


def extend(init: int, data: bytes) -> int:
    """crc.rs:21-27 -- digest.update(&[init]); digest.update(data); finalize.

    NOTE: unlike LevelDB's ``crc32c::Extend(crc, data, n)``, ``init`` is a
    *prefix byte* (record type), not a running CRC."""
    s = crc_update(INIT, bytes([init & 0xFF]))
    return crc_update(s, data) ^ XOROUT


def mask(crc: int) -> int:
    """crc.rs:36-38 -- rotate right by 15 bits and add a constant."""
    crc &= 0xFFFFFFFF
    return (((crc >> 15) | (crc << 17)) + MASK_DELTA) & 0xFFFFFFFF


def unmask(masked: int) -> int:
    """crc.rs:41-44."""
    rot = (masked - MASK_DELTA) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


def encode_fixed32(v: int) -> bytes:
    """coding.rs:51-62 (little endian)."""
    return struct.pack("<I", v & 0xFFFFFFFF)


def decode_fixed32(b: bytes) -> int:
    """coding.rs:139-144."""
    return b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24)


# --- GF(2) helpers (used by tests to check combine algebra, not by the walk) --
def multmodp(a: int, b: int) -> int:
    """a*b mod P in the reflected representation (bit 31 = x^0)."""
    p = 0
    m = 1 << 31
    while m:
        if a & m:
            p ^= b
        b = (b >> 1) ^ POLY_REFLECTED if b & 1 else b >> 1
        m >>= 1
    return p


def x8n(n: int) -> int:
    """x^(8n) mod P (reflected).  ``x^0`` is 0x80000000."""
    result = 1 << 31
    sq = 1 << 30  # x^1
    k = 8 * n
    while k:
        if k & 1:
            result = multmodp(sq, result)
        sq = multmodp(sq, sq)
        k >>= 1
    return result


def crc_combine(crc_a: int, crc_b: int, len_b: int) -> int:
    """crc(A||B) from crc(A), crc(B), |B| (zlib crc32_combine algebra)."""
    return multmodp(x8n(len_b), crc_a) ^ crc_b


# --- numpy vectorised walk (many equal-length messages at once) -------------
def crc_raw_rows(rows: np.ndarray, state: Optional[np.ndarray] = None) -> np.ndarray:
    """Bytewise table walk over every row of a 2-D uint8 array at once.

    Column j of every row is consumed in step j, so the cost is
    ``rows.shape[1]`` numpy steps of width ``rows.shape[0]``.  Returns the raw
    register (no xorout)."""
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    n = rows.shape[0]
    s = np.full(n, INIT, dtype=np.uint32) if state is None else state.astype(np.uint32).copy()
    cols = np.ascontiguousarray(rows.T).astype(np.uint32)
    for j in range(cols.shape[0]):
        s = TABLE_NP[(s ^ cols[j]) & 0xFF] ^ (s >> 8)
    return s


def value_rows(rows: np.ndarray) -> np.ndarray:
    return crc_raw_rows(rows) ^ np.uint32(XOROUT)


def mask_np(crc: np.ndarray) -> np.ndarray:
    crc = crc.astype(np.uint64)
    rot = ((crc >> 15) | (crc << 17)) & 0xFFFFFFFF
    return ((rot + MASK_DELTA) & 0xFFFFFFFF).astype(np.uint32)


def full_block_masked_crcs(blocks: np.ndarray) -> np.ndarray:
    """Masked CRC of ``type||payload`` = bytes [6, 32768) of full-type blocks.

    ``blocks`` is (n, 32768) uint8.  This is exactly what the writer stores
    for a FULL record of 32761 payload bytes (log_writer.rs:102-111) and, for
    such blocks, what the reference reader checks (log_reader.rs:200-206)."""
    assert blocks.ndim == 2 and blocks.shape[1] == BLOCK_SIZE
    return mask_np(value_rows(blocks[:, 6:]))


# --- Writer (log_writer.rs:25-124) ------------------------------------------
class LogWriter:
    """Restatement of ``log_writer::Writer`` writing into a bytearray, or into
    ``file`` -- any object with ``append(bytes)`` and ``flush()`` (the
    ``dyn WritableFile`` of env.rs:40-50) whose calls may raise.  A raising
    call propagates out of ``add_record`` at the point the reference's ``?``
    returns (log_writer.rs:70, :91, :114-119): the bytes already appended stay
    in the file and ``block_offset`` keeps the value it had at that point."""

    def __init__(self, dest: Optional[bytearray] = None, block_offset: int = 0, file=None):
        # log_writer.rs:45-53: block_offset is taken as given (no % kBlockSize)
        self.dest = dest if dest is not None else bytearray()
        self.file = file
        self.block_offset = block_offset
        self.type_crc = list(range(MAX_RECORD_TYPE + 1))  # init_type_crc, :33-37

    def _append(self, b: bytes) -> None:
        if self.file is None:
            self.dest += b
        else:
            self.file.append(bytes(b))

    def _flush(self) -> None:
        if self.file is not None:
            self.file.flush()

    def add_record(self, data: bytes) -> None:
        """log_writer.rs:58-97."""
        left = len(data)
        offset = 0
        begin = True
        while True:
            leftover = BLOCK_SIZE - self.block_offset
            if leftover < HEADER_SIZE:
                if leftover > 0:
                    self._append(bytes(leftover))         # :66-71 zero trailer (`?`: offset kept)
                self.block_offset = 0
            avail = BLOCK_SIZE - self.block_offset - HEADER_SIZE
            frag = left if left < avail else avail
            end = left == frag
            if begin and end:
                rtype = FULL_TYPE
            elif begin:
                rtype = FIRST_TYPE
            elif end:
                rtype = LAST_TYPE
            else:
                rtype = MIDDLE_TYPE
            self._emit(rtype, data[offset:offset + frag])
            offset += frag
            left -= frag
            begin = False
            if left <= 0:
                return

    def _emit(self, rtype: int, payload: bytes) -> None:
        """log_writer.rs:99-124."""
        n = len(payload)
        assert n <= 0xFFFF
        crc = mask(extend(self.type_crc[rtype], payload))
        self._append(encode_fixed32(crc) + bytes([n & 0xFF, n >> 8, rtype]))  # :114
        self._append(payload)                                                # :116
        self._flush()                                                        # :119
        self.block_offset += HEADER_SIZE + n                                 # :121, after every `?`


def write_image(records: Iterable[bytes], block_offset: int = 0) -> bytes:
    w = LogWriter(block_offset=block_offset)
    for r in records:
        w.add_record(r)
    return bytes(w.dest)


# --- Physical-record walk (LevelDB-correct restatement of log_reader.rs) -----
BAD_NONE, BAD_CHECKSUM, BAD_LENGTH, BAD_ZERO, BAD_TRUNCATED_HEADER = 0, 1, 2, 3, 4


@dataclass
class PhysicalRecord:
    file_offset: int      # offset of the 7-byte header in the file
    length: int
    rtype: int
    stored: int           # masked CRC as stored (decode_fix32 of header[0:4])
    computed: int         # mask(crc32c(type || payload[:length]))
    status: int           # BAD_* code

    @property
    def ok(self) -> bool:
        return self.status == BAD_NONE


def walk_block(block: bytes, base: int = 0) -> List[PhysicalRecord]:
    """Every physical record inside one block (<= 32768 bytes).

    Rules (log_reader.rs:180-212 made per-record, as LevelDB's
    ReadPhysicalRecord does):
      * fewer than 7 bytes left -> block trailer, stop;
      * type 0 and length 0 -> zero/preallocated region, stop the block
        (reported as BAD_ZERO, the reference's kBadRecord at :195-198);
      * 7+length past the block end -> BAD_LENGTH, stop the block;
      * otherwise CRC over block[off+6 : off+7+length] and compare.
    """
    out: List[PhysicalRecord] = []
    off = 0
    n = len(block)
    while n - off >= HEADER_SIZE:
        h = block[off:off + HEADER_SIZE]
        stored = decode_fixed32(h[0:4])
        length = h[4] | (h[5] << 8)
        rtype = h[6]
        if HEADER_SIZE + length > n - off:
            out.append(PhysicalRecord(base + off, length, rtype, stored, 0, BAD_LENGTH))
            break
        if rtype == ZERO_TYPE and length == 0:
            out.append(PhysicalRecord(base + off, 0, 0, stored, 0, BAD_ZERO))
            break
        computed = mask(value(block[off + 6: off + HEADER_SIZE + length]))
        st = BAD_NONE if computed == stored else BAD_CHECKSUM
        out.append(PhysicalRecord(base + off, length, rtype, stored, computed, st))
        off += HEADER_SIZE + length
    return out


def walk_records(image: bytes) -> List[PhysicalRecord]:
    out: List[PhysicalRecord] = []
    for b in range(0, len(image), BLOCK_SIZE):
        out.extend(walk_block(image[b:b + BLOCK_SIZE], b))
    return out


class LogReader:
    """Logical-record reassembly (log_reader.rs:76-153), LevelDB-correct.

    ``read_record`` returns the payload bytes, ``None`` at EOF (the reference
    returns an empty Slice, :140) and raises :class:`CorruptionError` where the
    reference returns ``Err(IOError)`` (:142-152).  Error rules, mirrored by the
    product reader:
      * BAD_CHECKSUM (when ``checksum``) -> error (:200-206);
      * BAD_ZERO -> error (kBadRecord, :195-198);
      * BAD_LENGTH of a record cut by the end of the file -> EOF (a torn final
        write; the reference returns kEof, :190-193), elsewhere -> error;
      * unknown type -> error (:126-128).
    After an error the next call continues with the following record."""

    def __init__(self, image: bytes, checksum: bool = True, initial_offset: int = 0):
        self.records = walk_records(image)
        self.size = len(image)
        self.checksum = checksum
        self.initial_offset = initial_offset
        self.resyncing = initial_offset > 0
        self._image = image
        # SkipToInitialBlock (LevelDB; the reference leaves it todo!()): reading
        # starts at the block holding initial_offset -- or the next one when only
        # a trailer (< 7 bytes) remains in it -- so records of earlier blocks are
        # never read, and their corruption never reported.
        in_block = initial_offset % BLOCK_SIZE
        start = initial_offset - in_block + (BLOCK_SIZE if in_block > BLOCK_SIZE - 6 else 0)
        self.i = 0
        while self.i < len(self.records) and self.records[self.i].file_offset < start:
            self.i += 1

    def read_record(self) -> Optional[bytes]:
        scratch = bytearray()
        in_frag = False
        while True:
            if self.i >= len(self.records):
                return None          # EOF; a partial fragment is dropped (:133-141)
            r = self.records[self.i]
            self.i += 1
            if r.status == BAD_LENGTH:
                if self.i == len(self.records) and r.file_offset + HEADER_SIZE + r.length > self.size:
                    self.i = len(self.records)
                    return None
                raise CorruptionError(r)
            if r.status == BAD_ZERO:
                raise CorruptionError(r)
            if self.checksum and r.status == BAD_CHECKSUM:
                raise CorruptionError(r)
            if r.file_offset < self.initial_offset:
                continue
            if self.resyncing:
                if r.rtype == MIDDLE_TYPE:
                    continue
                if r.rtype == LAST_TYPE:
                    self.resyncing = False
                    continue
                self.resyncing = False
            payload = self._payload(r)
            if r.rtype == FULL_TYPE:
                return payload
            if r.rtype == FIRST_TYPE:
                in_frag = True
                scratch = bytearray(payload)
            elif r.rtype == MIDDLE_TYPE:
                if in_frag:
                    scratch += payload
            elif r.rtype == LAST_TYPE:
                if in_frag:
                    scratch += payload
                    return bytes(scratch)
            else:
                raise CorruptionError(r)

    def _payload(self, r: PhysicalRecord) -> bytes:
        s = r.file_offset + HEADER_SIZE
        return bytes(self._image[s:s + r.length])


class CorruptionError(Exception):
    pass


def read_all(image: bytes, checksum: bool = True, initial_offset: int = 0) -> List[bytes]:
    rd = LogReader(image, checksum, initial_offset)
    out = []
    while True:
        rec = rd.read_record()
        if rec is None:
            return out
        out.append(rec)


# --- seeded synthetic payloads (shared with the C oracle and the product) ----
def splitmix64_stream(seed: int, nbytes: int) -> bytes:
    """Little-endian splitmix64 output words, truncated to ``nbytes``."""
    out = bytearray()
    x = seed & 0xFFFFFFFFFFFFFFFF
    while len(out) < nbytes:
        x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        z ^= z >> 31
        out += struct.pack("<Q", z)
    return bytes(out[:nbytes])


def splitmix64_np(seeds: np.ndarray, nwords: int) -> np.ndarray:
    """Vectorised splitmix64: row r = ``nwords`` words from seed ``seeds[r]``."""
    with np.errstate(over="ignore"):
        x = seeds.astype(np.uint64)[:, None] + (np.arange(1, nwords + 1, dtype=np.uint64)
                                                 * np.uint64(0x9E3779B97F4A7C15))[None, :]
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def synth_full_blocks(n: int, seed: int = 0x5EED0002, first: int = 0) -> np.ndarray:
    """Config C2 blocks: ``[mask(crc) LE][F9 7F][01][32761 payload bytes]``.

    Payload of block b = splitmix64(seed ^ b) bytes.  The header is filled by
    the oracle's own writer arithmetic (mask(extend(FULL, payload)))."""
    idx = np.arange(first, first + n, dtype=np.uint64)
    words = splitmix64_np(np.uint64(seed) ^ idx, BLOCK_SIZE // 8)
    blocks = words.view(np.uint8).reshape(n, BLOCK_SIZE).copy()
    blocks[:, 4] = 0xF9
    blocks[:, 5] = 0x7F
    blocks[:, 6] = FULL_TYPE
    crcs = full_block_masked_crcs(blocks)
    blocks[:, 0:4] = crcs.view(np.uint8).reshape(n, 4) if crcs.dtype.byteorder in "=<" else \
        crcs.astype("<u4").view(np.uint8).reshape(n, 4)
    return blocks


# --- batch replay events (LogReader semantics, restated for device parity) ---
EV_RECORD, EV_ERROR = 0, 1


def replay_events(image: bytes, checksum: bool = True):
    """The sequence a LogReader over ``image`` produces when every error is
    caught and reading continues: ("record", first_file_offset, payload) or
    ("error", file_offset, status).  Stops at EOF (incl. a torn tail).
    initial_offset = 0 (log_reader.rs:76-153 / LogReader above)."""
    rd = LogReader(image, checksum, 0)
    out = []
    while True:
        start = rd.i
        try:
            rec = rd.read_record()
        except CorruptionError as e:
            r = e.args[0]
            out.append(("error", r.file_offset, r.status))
            continue
        if rec is None:
            return out
        # first physical record of the returned logical record
        j = rd.i - 1
        phys = rd.records
        if phys[j].rtype == FULL_TYPE:
            first = phys[j].file_offset
        else:
            k = j
            while phys[k].rtype != FIRST_TYPE:
                k -= 1
            first = phys[k].file_offset
        out.append(("record", first, rec))
