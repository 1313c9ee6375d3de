/*
 * crc32c_oracle.c -- plain-C restatement of Revel's WAL CRC path.
 *
 * TEST INFRASTRUCTURE ONLY.  Linked/loaded exclusively by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg (as the checker or
 * as the timed CPU baseline).  The product library never links it.
 *
 * Reference: guimingyue/revel @ v0 (read-only at /root/reference).
 *   src/util/crc.rs:13-15   CRC_32_ISCSI via third-party crate `crc` ^3.0.0
 *                           (Cargo.toml:17-18; not vendored, 3.x patch
 *                           unpinned).  Published parameters: width 32,
 *                           poly 0x1EDC6F41 (reflected 0x82F63B78), init
 *                           0xFFFFFFFF, refin/refout, xorout 0xFFFFFFFF.
 *                           The crate walks a 256-entry table one byte per
 *                           step: oracle_crc_bytewise() below.
 *   src/util/crc.rs:17-44   value / extend / mask / unmask
 *   src/coding.rs:51-62,139-144  fixed32 little-endian header field
 *   src/log_format.rs:14-30 record types, kBlockSize, kHeaderSize
 *   src/log_writer.rs:58-124  add_record / emit_physical_record
 *   src/log_reader.rs:155-216 physical-record parse (LevelDB-correct walk,
 *                           see oracle/crc32c_oracle.py for the deviation
 *                           note and SURVEY.md Appendix A).
 *
 * slice-by-16 and SSE4.2 variants exist only as extra CPU-baseline context
 * lines; the reference-equivalent line is the bytewise one.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define ORACLE_POLY_REFLECTED 0x82F63B78u
#define ORACLE_MASK_DELTA 0xa282ead8u
#define ORACLE_BLOCK 32768u
#define ORACLE_HEADER 7u

static uint32_t T[16][256];
static int tables_ready = 0;

static void init_tables(void) {
    if (tables_ready) return;
    for (uint32_t n = 0; n < 256; ++n) {
        uint32_t c = n;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ ORACLE_POLY_REFLECTED : c >> 1;
        T[0][n] = c;
    }
    for (int t = 1; t < 16; ++t)
        for (uint32_t n = 0; n < 256; ++n)
            T[t][n] = (T[t - 1][n] >> 8) ^ T[0][T[t - 1][n] & 0xff];
    tables_ready = 1;
}

/* Raw register update, one byte per step (crate `crc` algorithm class). */
uint32_t oracle_crc_bytewise(uint32_t state, const uint8_t* p, size_t n) {
    init_tables();
    for (size_t i = 0; i < n; ++i) state = T[0][(state ^ p[i]) & 0xff] ^ (state >> 8);
    return state;
}

/* Context line: slice-by-16. */
uint32_t oracle_crc_slice16(uint32_t state, const uint8_t* p, size_t n) {
    init_tables();
    while (n >= 16) {
        uint32_t w0, w1, w2, w3;
        memcpy(&w0, p, 4); memcpy(&w1, p + 4, 4); memcpy(&w2, p + 8, 4); memcpy(&w3, p + 12, 4);
        w0 ^= state;
        state = T[15][w0 & 0xff] ^ T[14][(w0 >> 8) & 0xff] ^ T[13][(w0 >> 16) & 0xff] ^ T[12][w0 >> 24] ^
                T[11][w1 & 0xff] ^ T[10][(w1 >> 8) & 0xff] ^ T[9][(w1 >> 16) & 0xff] ^ T[8][w1 >> 24] ^
                T[7][w2 & 0xff] ^ T[6][(w2 >> 8) & 0xff] ^ T[5][(w2 >> 16) & 0xff] ^ T[4][w2 >> 24] ^
                T[3][w3 & 0xff] ^ T[2][(w3 >> 8) & 0xff] ^ T[1][(w3 >> 16) & 0xff] ^ T[0][w3 >> 24];
        p += 16; n -= 16;
    }
    return oracle_crc_bytewise(state, p, n);
}

/* Context line / second independent check: the x86 SSE4.2 crc32 instruction
 * computes exactly CRC-32C's raw register update. */
#if defined(__x86_64__)
__attribute__((target("sse4.2")))
uint32_t oracle_crc_sse42(uint32_t state, const uint8_t* p, size_t n) {
    uint64_t s = state;
    while (n >= 8) {
        uint64_t w; memcpy(&w, p, 8);
        s = __builtin_ia32_crc32di(s, w);
        p += 8; n -= 8;
    }
    uint32_t s32 = (uint32_t)s;
    while (n--) s32 = __builtin_ia32_crc32qi(s32, *p++);
    return s32;
}
#else
uint32_t oracle_crc_sse42(uint32_t state, const uint8_t* p, size_t n) {
    return oracle_crc_bytewise(state, p, n);
}
#endif

typedef uint32_t (*crc_fn)(uint32_t, const uint8_t*, size_t);
static crc_fn pick(int variant) {
    return variant == 2 ? oracle_crc_sse42 : variant == 1 ? oracle_crc_slice16 : oracle_crc_bytewise;
}

/* crc.rs:17-19 */
uint32_t oracle_value(const uint8_t* p, size_t n) { return oracle_crc_bytewise(0xFFFFFFFFu, p, n) ^ 0xFFFFFFFFu; }

/* crc.rs:21-27: init is a prefix BYTE */
uint32_t oracle_extend(uint8_t init, const uint8_t* p, size_t n) {
    uint32_t s = oracle_crc_bytewise(0xFFFFFFFFu, &init, 1);
    return oracle_crc_bytewise(s, p, n) ^ 0xFFFFFFFFu;
}

/* crc.rs:36-38 / 41-44 */
uint32_t oracle_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + ORACLE_MASK_DELTA; }
uint32_t oracle_unmask(uint32_t m) {
    uint32_t rot = m - ORACLE_MASK_DELTA;
    return (rot >> 17) | (rot << 15);
}

static uint32_t get32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static void put32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

/* Masked CRC of bytes [6, 32768) of each full-type block (config C2 unit).
 * variant: 0 bytewise (reference-equivalent), 1 slice-by-16, 2 SSE4.2. */
void oracle_full_block_crcs(const uint8_t* blocks, size_t nblocks, uint32_t* masked_out, int variant) {
    crc_fn f = pick(variant);
    for (size_t b = 0; b < nblocks; ++b) {
        const uint8_t* blk = blocks + b * (size_t)ORACLE_BLOCK;
        masked_out[b] = oracle_mask(f(0xFFFFFFFFu, blk + 6, ORACLE_BLOCK - 6) ^ 0xFFFFFFFFu);
    }
}

/* log_writer.rs:58-124 restated.  Appends the framed image of `nrec`
 * records (payloads concatenated in `payloads`, sizes in `lens`) to `out`
 * starting at *block_offset; returns bytes written, or (size_t)-1 if
 * `cap` would be exceeded. */
size_t oracle_write_image(const uint8_t* payloads, const uint64_t* lens, size_t nrec,
                          uint64_t* block_offset, uint8_t* out, size_t cap) {
    size_t pos = 0, src = 0;
    uint64_t boff = *block_offset;
    for (size_t r = 0; r < nrec; ++r) {
        const uint8_t* data = payloads + src;
        size_t left = (size_t)lens[r], off = 0;
        int begin = 1;
        src += left;
        for (;;) {
            size_t leftover = ORACLE_BLOCK - boff;
            if (leftover < ORACLE_HEADER) {
                if (leftover > 0) {
                    if (pos + leftover > cap) return (size_t)-1;
                    memset(out + pos, 0, leftover);
                    pos += leftover;
                }
                boff = 0;
            }
            size_t avail = ORACLE_BLOCK - boff - ORACLE_HEADER;
            size_t frag = left < avail ? left : avail;
            int end = left == frag;
            uint8_t type = (begin && end) ? 1 : begin ? 2 : end ? 4 : 3;
            if (pos + ORACLE_HEADER + frag > cap) return (size_t)-1;
            uint8_t* h = out + pos;
            h[4] = (uint8_t)(frag & 0xff);
            h[5] = (uint8_t)(frag >> 8);
            h[6] = type;
            memcpy(h + ORACLE_HEADER, data + off, frag);
            put32(h, oracle_mask(oracle_extend(type, data + off, frag)));
            pos += ORACLE_HEADER + frag;
            boff += ORACLE_HEADER + frag;
            off += frag;
            left -= frag;
            begin = 0;
            if (left == 0) break;
        }
    }
    *block_offset = boff;
    return pos;
}

/* Physical-record walk (same rules as walk_block() in crc32c_oracle.py).
 * Writes up to `cap` records; returns the number found (may exceed cap). */
size_t oracle_walk_v(const uint8_t* image, size_t n, uint64_t* rec_off, uint32_t* rec_len,
                     uint8_t* rec_type, uint32_t* rec_stored, uint32_t* rec_computed,
                     uint8_t* rec_status, size_t cap, int variant) {
    const crc_fn crc = pick(variant);
    size_t count = 0;
    for (size_t base = 0; base < n; base += ORACLE_BLOCK) {
        size_t bl = n - base < ORACLE_BLOCK ? n - base : ORACLE_BLOCK;
        const uint8_t* blk = image + base;
        size_t off = 0;
        while (bl - off >= ORACLE_HEADER) {
            const uint8_t* h = blk + off;
            uint32_t len = (uint32_t)h[4] | ((uint32_t)h[5] << 8);
            uint8_t type = h[6];
            uint32_t stored = get32(h), computed = 0;
            uint8_t status;
            int stop = 0;
            if (ORACLE_HEADER + len > bl - off) { status = 2; stop = 1; }
            else if (type == 0 && len == 0) { status = 3; stop = 1; }
            else {
                /* log_writer.rs:107-111: mask(crc of type || payload) */
                computed = oracle_mask(crc(0xFFFFFFFFu, h + 6, len + 1) ^ 0xFFFFFFFFu);
                status = computed == stored ? 0 : 1;
            }
            if (count < cap) {
                rec_off[count] = base + off; rec_len[count] = len; rec_type[count] = type;
                rec_stored[count] = stored; rec_computed[count] = computed; rec_status[count] = status;
            }
            ++count;
            if (stop) break;
            off += ORACLE_HEADER + len;
        }
    }
    return count;
}

size_t oracle_walk(const uint8_t* image, size_t n, uint64_t* rec_off, uint32_t* rec_len,
                   uint8_t* rec_type, uint32_t* rec_stored, uint32_t* rec_computed,
                   uint8_t* rec_status, size_t cap) {
    return oracle_walk_v(image, n, rec_off, rec_len, rec_type, rec_stored, rec_computed, rec_status, cap, 0);
}

/* Config C2 generator (identical bytes to synth_full_blocks() in Python and
 * to the product's device generator): splitmix64(seed ^ block_index). */
void oracle_synth_full_blocks(uint8_t* dst, size_t nblocks, uint64_t seed, uint64_t first) {
    for (size_t b = 0; b < nblocks; ++b) {
        uint64_t x = seed ^ (first + b);
        uint8_t* blk = dst + b * (size_t)ORACLE_BLOCK;
        for (size_t w = 0; w < ORACLE_BLOCK / 8; ++w) {
            x += 0x9E3779B97F4A7C15ull;
            uint64_t z = x;
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            z ^= z >> 31;
            memcpy(blk + 8 * w, &z, 8);
        }
        blk[4] = 0xF9; blk[5] = 0x7F; blk[6] = 1;
        put32(blk, oracle_mask(oracle_crc_bytewise(0xFFFFFFFFu, blk + 6, ORACLE_BLOCK - 6) ^ 0xFFFFFFFFu));
    }
}
