"""Input records of the golden edge cases (regenerated deterministically by
the same code that made the fixtures, tests/golden/make_golden.py)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_golden  # noqa: E402

_CASES = None


def edge_records(name: str):
    global _CASES
    if _CASES is None:
        _CASES = make_golden.edge_cases()
    return _CASES[name][0]


def batch_log(rng, nbatches: int, max_entries: int = 40, max_key: int = 300, max_value: int = 6000,
              big_every: int = 0, first_sequence: int = 1):
    """WriteBatch reps as DB::write would log them (db.rs:95-112: sequence =
    last_sequence + 1, last_sequence += count).  Mixed puts and deletions;
    every big_every-th batch carries a value > 32 KiB (multi-fragment)."""
    from oracle import write_batch_oracle as wb
    reps, seq = [], first_sequence
    for b in range(nbatches):
        batch = wb.WriteBatch()
        for _ in range(int(rng.integers(1, max_entries + 1))):
            key = rng.integers(0, 256, int(rng.integers(0, max_key)), dtype="u1").tobytes()
            if rng.random() < 0.25:
                batch.delete(key)
            else:
                batch.put(key, rng.integers(0, 256, int(rng.integers(0, max_value)), dtype="u1").tobytes())
        if big_every and b % big_every == big_every - 1:
            batch.put(b"big", rng.integers(0, 256, 70000, dtype="u1").tobytes())
        batch.set_sequence(seq)
        seq += batch.count()
        reps.append(batch.contents())
    return reps


def malformed_batches():
    """(name, rep, expected status) for every WriteBatch error class."""
    import struct
    from oracle import write_batch_oracle as wb

    def hdr(seq, count):
        return struct.pack("<QI", seq, count)
    ok = wb.WriteBatch()
    ok.put(b"k", b"v")
    ok.delete(b"gone")
    ok.set_sequence(77)
    rep = ok.contents()
    return [
        ("empty", b"", wb.TOO_SMALL),
        ("eleven", b"\x01" * 11, wb.TOO_SMALL),
        ("header_only", hdr(5, 0), wb.OK),
        ("header_only_count1", hdr(5, 1), wb.WRONG_COUNT),
        ("ok", rep, wb.OK),
        ("count_high", hdr(77, 3) + rep[12:], wb.WRONG_COUNT),
        ("count_low", hdr(77, 1) + rep[12:], wb.WRONG_COUNT),
        ("bad_tag", rep + b"\x02\x01a", wb.BAD_TAG),
        ("bad_tag_first", hdr(1, 1) + b"\x07\x01a\x01b", wb.BAD_TAG),
        ("key_past_end", hdr(1, 1) + b"\x01\x05ab", wb.BAD_ENTRY),
        ("value_past_end", hdr(1, 1) + b"\x01\x01a\x09xyz", wb.BAD_ENTRY),
        ("varint_truncated", hdr(1, 1) + b"\x00\x80\x80", wb.BAD_ENTRY),
        ("varint_overflow", hdr(1, 1) + b"\x00" + bytes([129, 130, 131, 132, 133, 17]), wb.BAD_ENTRY),
        ("varint_nonminimal", hdr(9, 2) + b"\x01\x81\x00k\x80\x80\x00\x00\x80\x00", wb.OK),
        ("value_missing", hdr(1, 1) + b"\x01\x01a", wb.BAD_ENTRY),
        ("tag_only", hdr(1, 1) + b"\x00", wb.BAD_ENTRY),
        ("seq_wrap", hdr(2**64 - 1, 2) + b"\x00\x01a\x00\x01b", wb.OK),
        ("empty_key_value", hdr(3, 2) + b"\x01\x00\x00\x00\x00", wb.OK),
    ]
