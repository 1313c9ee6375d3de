"""CPU model of the fused C3 pipeline's arithmetic (tools/experiments/x_verify_walk.inc),
checked against the oracle walk (log_writer.rs:107-111 / log_reader.rs:200-206's
per-record CRC): it pins what the GPU kernels compute, independent of a GPU.

* row_header: the 7 header bytes taken out of a raw 1 KiB row held as 64
  lanes x 16 B (four dwords of lane o >> 4, two more of the next lane or of
  the next row's lane 0 when the type byte lies past the 16 B);
* the walk over those rows (count_block_wave's rules: a trailer < 7 B ends the
  block, a zero record or a length past the block end ends it, counted);
* the captures Q_p = P(y_p) x^(8 (S_p - y_p)) (P = zero-init raw CRC of the
  block bytes before y, S = the end of y's 256-B sub-row) at every valid
  record's type byte and at the end of the valid data, and k_expand_walk's
  finalizer: F_p = Q_p x^(-8 (S - off)) ^ w_p ^ h16_p x^-32 for a record
  start, Q_p x^(-8 (S - y)) for the end; crc_t = mask(F_{t+1} ^
  Q_t x^(8 (e_t - S_t)) ^ init_xor(len_t + 1)).
"""
import random

import pytest

from oracle import crc32c_oracle as po

POLY = 0x82F63B78
ONE = 0x80000000          # x^0, reflected
XINV = 0x05EC76F1         # x^-1 mod P, reflected
_T = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ POLY if _c & 1 else _c >> 1
    _T.append(_c)


def raw(data: bytes, c: int = 0) -> int:
    for b in data:
        c = _T[(c ^ b) & 0xFF] ^ (c >> 8)
    return c


def mul(a: int, b: int) -> int:
    m, p = 1 << 31, 0
    while m:
        if a & m:
            p ^= b
        m >>= 1
        b = (b >> 1) ^ POLY if b & 1 else b >> 1
    return p


def _pow(base: int, n: int) -> int:
    r = ONE
    while n:
        if n & 1:
            r = mul(r, base)
        base = mul(base, base)
        n >>= 1
    return r


X8 = 0x00800000                      # x^8
X8INV = _pow(XINV, 8)                # x^-8
x8n = lambda d: _pow(X8, d)          # noqa: E731
x8inv = lambda d: _pow(X8INV, d)     # noqa: E731
init_xor = lambda n: mul(x8n(n), 0xFFFFFFFF) ^ 0xFFFFFFFF  # noqa: E731
len_inv32 = lambda h16: mul(_pow(XINV, 32), h16)           # noqa: E731


def sub_row_end(y: int) -> int:
    return 32768 if y >= 32768 else (y | 255) + 1


def row_header(blk: bytes, K: int, o: int):
    """x_verify_walk.inc row_header: lane L = o >> 4 of the raw row at K."""
    row, nxt = blk[K:K + 1024], blk[K + 1024:K + 2048].ljust(1024, b"\0")
    L, q = o >> 4, o & 15

    def dw(buf, lane, c):
        return int.from_bytes(buf[16 * lane + 4 * c:16 * lane + 4 * c + 4], "little")

    d = [dw(row, L, c) for c in range(4)] + [0, 0]
    if q > 9:
        src, lane = (row, L + 1) if L < 63 else (nxt, 0)
        d[4], d[5] = dw(src, lane, 0), dw(src, lane, 1)
    j, sh = q >> 2, (q & 3) * 8
    a = (((d[j + 1] << 32) | d[j]) >> sh) & 0xFFFFFFFF
    b = (((d[j + 2] << 32) | d[j + 1]) >> sh) & 0xFFFFFFFF
    return a, b & 0xFFFF, (b >> 16) & 0xFF


def model_block(blk: bytes, bl: int):
    """Walk + captures + k_expand_walk's finalizer for one block; returns the
    header entries (offset, stored, len, type, ok) and the computed masked
    CRCs (None for a bad record, or for all of a dense block's)."""
    ents = []
    nv = 0
    if bl >= 7:
        wo = 0
        while True:
            K = wo & ~1023
            stored, ln, ty = row_header(blk, K, wo - K)
            ok = 7 + ln <= bl - wo and not (ty == 0 and ln == 0)
            ents.append((wo, stored, ln, ty, ok))
            nxt = wo + 7 + ln
            if not (ok and bl - nxt >= 7):
                nv = len(ents) if ok else len(ents) - 1
                break
            wo = nxt
    n = len(ents)
    if n > 64:
        return ents, [None] * n  # the dense kernel's blocks
    F, T = [], []
    for p in range(n + 1):  # slots: the records, then the end of the data
        valid = p < n and ents[p][4]
        off = ents[p][0] if p < n else (ents[-1][0] + 7 + ents[-1][2] if n else 0)
        y = off + 6 if valid else off
        S = sub_row_end(y)
        q = mul(raw(blk[:y]), x8n(S - y)) if p <= nv and nv else 0
        f = mul(q, x8inv(S - off if valid else (S - y if y <= S else 0)))
        t = 0
        if valid:
            f ^= ents[p][1] ^ len_inv32(ents[p][2])
            e = off + 7 + ents[p][2]
            t = mul(q, x8n(e - S) if e >= S else x8inv(S - e))
        F.append(f)
        T.append(t)
    crcs = [po.mask(F[i + 1] ^ T[i] ^ init_xor(ents[i][2] + 1)) if ents[i][4] else None for i in range(n)]
    return ents, crcs


@pytest.mark.parametrize("seed", range(6))
def test_walk_model_matches_oracle(seed):
    rng = random.Random(seed)
    checked = 0
    for trial in range(12):
        recs = [bytes(rng.randrange(256) for _ in range(rng.choice([0, 1, 5, 60, 64, 100, 200, 1000, 9000, 33000])))
                for _ in range(rng.randint(1, 14))]
        img = bytearray(po.write_image(recs))
        if trial % 3 == 0 and len(img) > 100:  # a flipped bit: payload, header or length
            i = rng.randrange(len(img))
            img[i] ^= 1 << rng.randrange(8)
        ref = po.walk_records(bytes(img))
        k = 0
        for b in range(0, len(img), 32768):
            blk = bytes(img[b:b + 32768])
            ents, crcs = model_block(blk + bytes(32768 + 2048 - len(blk)), len(blk))
            mine = [r for r in ref if b <= r.file_offset < b + 32768]
            assert len(ents) == len(mine)
            for e, c, r in zip(ents, crcs, mine):
                assert (b + e[0], e[1], e[2], e[3]) == (r.file_offset, r.stored, r.length, r.rtype)
                assert e[4] == (r.status in (po.BAD_NONE, po.BAD_CHECKSUM))
                if c is not None:
                    assert c == r.computed
                    checked += 1
            k += len(ents)
    assert checked > 20


def test_walk_model_dense_and_64_record_blocks():
    """Exactly 64 records (the end capture has index 64) and 65+ (dense:
    no captures) -- the walk's counts and entries still equal the oracle's."""
    for nrec, size in ((64, 500), (65, 400), (300, 90)):
        img = po.write_image([bytes([i % 251]) * size for i in range(nrec)])
        ents, crcs = model_block(img[:32768].ljust(32768 + 2048, b"\0"), min(32768, len(img)))
        ref = po.walk_block(img[:32768])
        assert [e[2] for e in ents] == [r.length for r in ref]
        if len(ents) <= 64:
            assert crcs == [r.computed for r in ref]
