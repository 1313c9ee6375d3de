/*
 * revel_wal.h -- C-ABI drop-in boundary for Revel's write-ahead-log record
 * path, MI355X-native (gfx950).
 *
 * Reference: guimingyue/revel @ v0.  Each entry point names the reference
 * interface it replaces (file:line).  The reference is a Rust crate whose
 * WAL surface is crate-internal (lib.rs:24,33-38), so the binding a Revel
 * maintainer adds is the `extern "C"` block shown in INTEGRATION.md.
 *
 * Conventions
 *  - Plain pointers and sizes only; no C++ or torch types.
 *  - Status codes mirror `enum Error` (src/error.rs:16-23); 0 = Ok.
 *  - The caller owns every buffer it passes.  Opaque handles are owned by the
 *    caller after *_new and released with the matching *_free.
 *  - Handles are single-threaded, like the reference's Rc<RefCell<..>> types
 *    (log_writer.rs:26, log_reader.rs:44-56).  Use one writer/reader/GPU
 *    context per thread; distinct handles may be used concurrently.
 *  - Every GPU entry point fails loudly (REVEL_NOT_SUPPORT) when no gfx950
 *    device is present; there is no CPU fallback behind them.
 */
#ifndef REVEL_WAL_H_
#define REVEL_WAL_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes: src/error.rs:16-23 ---------------------------------- */
#define REVEL_OK 0
#define REVEL_NOT_FOUND 1
#define REVEL_CORRUPTION 2
#define REVEL_NOT_SUPPORT 3
#define REVEL_INVALID_ARGUMENT 4
#define REVEL_IO_ERROR 5

/* ---- on-disk format: src/log_format.rs:14-30 --------------------------- */
#define REVEL_BLOCK_SIZE 32768
#define REVEL_HEADER_SIZE 7
#define REVEL_ZERO_TYPE 0
#define REVEL_FULL_TYPE 1
#define REVEL_FIRST_TYPE 2
#define REVEL_MIDDLE_TYPE 3
#define REVEL_LAST_TYPE 4
#define REVEL_MAX_RECORD_TYPE 4
/* Payload bytes of a FULL record that fills one block exactly. */
#define REVEL_FULL_BLOCK_PAYLOAD (REVEL_BLOCK_SIZE - REVEL_HEADER_SIZE)

/* ---- CRC32C: src/util/crc.rs ------------------------------------------- */
/* crc.rs:17-19  `pub fn value(data: &[u8]) -> u32` */
uint32_t revel_crc32c_value(const uint8_t* data, size_t n);
/* crc.rs:22-27  `pub fn extend(init: u8, data: &[u8]) -> u32` -- CRC of the
 * single byte `init` followed by data (init is a prefix byte, NOT a crc). */
uint32_t revel_crc32c_extend(uint8_t init, const uint8_t* data, size_t n);
/* crc.rs:36-38  `pub const fn mask(crc: u32) -> u32` */
uint32_t revel_crc32c_mask(uint32_t crc);
/* crc.rs:41-44  `pub const fn unmask(masked_crc: u32) -> u32` */
uint32_t revel_crc32c_unmask(uint32_t masked_crc);

/* ---- files: src/env.rs -------------------------------------------------- */
typedef struct revel_writable_file revel_writable_file;
typedef struct revel_sequential_file revel_sequential_file;

/* env.rs:201-230 `MemoryWritableFile::new(Vec::new())` */
revel_writable_file* revel_memory_writable_file_new(void);
/* env.rs:25-38 `new_writable_file(filename)` (truncate|create|write). */
int revel_posix_writable_file_new(const char* path, revel_writable_file** out);
/* env.rs:40-50 `trait WritableFile { append, flush, close, sync }` */
int revel_writable_file_append(revel_writable_file* f, const uint8_t* data, size_t n);
int revel_writable_file_flush(revel_writable_file* f);
int revel_writable_file_close(revel_writable_file* f);
int revel_writable_file_sync(revel_writable_file* f);
/* Accessor the reference lacks (env.rs:201-204 keeps `memory` private):
 * borrow the bytes of a memory file; valid until the next append/free.
 * REVEL_INVALID_ARGUMENT for a posix file. */
int revel_memory_writable_file_contents(const revel_writable_file* f, const uint8_t** data, size_t* n);
void revel_writable_file_free(revel_writable_file* f);

/* Caller-implemented files: the adapter for a `dyn WritableFile` the caller
 * owns and shares (Writer::new(Rc<RefCell<dyn WritableFile>>),
 * log_writer.rs:26,41-45; db.rs:56-63 keeps a clone to sync it) -- every
 * call of the trait (env.rs:40-50) goes to the matching callback with `user`.
 * Callbacks return 0 for Ok or an error.rs code (1..5; anything else is
 * reported as REVEL_IO_ERROR), which the calling entry point returns.
 * append is required; flush/close/sync may be NULL (no-op, Ok).  release
 * (nullable) is called once by revel_writable_file_free, e.g. to drop the
 * Rc clone behind `user`.  On failure nothing is called and the caller keeps
 * `user`. */
typedef int (*revel_file_append_fn)(void* user, const uint8_t* data, size_t n);
typedef int (*revel_file_op_fn)(void* user);
typedef void (*revel_file_release_fn)(void* user);
int revel_writable_file_from_callbacks(void* user, revel_file_append_fn append, revel_file_op_fn flush,
                                       revel_file_op_fn close, revel_file_op_fn sync,
                                       revel_file_release_fn release, revel_writable_file** out);

/* The adapter for a caller's `Box<dyn SequentialFile>` (env.rs:52-57) handed
 * to Reader::new (log_reader.rs:40,62).  read fills up to n bytes of scratch
 * and stores the count in *got (0 = end of file); short counts are allowed,
 * the library calls again until n bytes or end of file (as it does for
 * read(2)).  skip(n) advances the position by n bytes (relative; the Posix
 * reference seeks absolute, env.rs:171-174, which is the same at the only
 * call, a reader's start); NULL = read and drop.  release (nullable) is called
 * once when the file is freed -- by revel_sequential_file_free or by the
 * reader that owns it -- e.g. to drop the Box behind `user`.  On failure
 * nothing is called and the caller keeps `user`. */
typedef int (*revel_file_read_fn)(void* user, uint8_t* scratch, size_t n, size_t* got);
typedef int (*revel_file_skip_fn)(void* user, uint64_t n);
int revel_sequential_file_from_callbacks(void* user, revel_file_read_fn read, revel_file_skip_fn skip,
                                         revel_file_release_fn release, revel_sequential_file** out);

/* env.rs:232-246 `MemorySequentialFile::new(Rc<Vec<u8>>)` -- copies data. */
revel_sequential_file* revel_memory_sequential_file_new(const uint8_t* data, size_t n);
/* Posix sequential file.  The reference declares PosixSequentialFile
 * (env.rs:153-175) but gives it no constructor. */
int revel_posix_sequential_file_new(const char* path, revel_sequential_file** out);
/* env.rs:52-57 `fn read(&self, scratch) -> Result<Slice>`: fills up to n
 * bytes of scratch, *got = bytes filled (0 at EOF). */
int revel_sequential_file_read(revel_sequential_file* f, uint8_t* scratch, size_t n, size_t* got);
/* env.rs:56 `fn skip(&self, n)`: RELATIVE skip for both kinds (the
 * reference's Posix impl seeks absolute, env.rs:171-174: App. A #6). */
int revel_sequential_file_skip(revel_sequential_file* f, uint64_t n);
void revel_sequential_file_free(revel_sequential_file* f);

/* ---- log writer: src/log_writer.rs -------------------------------------- */
typedef struct revel_log_writer revel_log_writer;
/* log_writer.rs:41-53 `Writer::new(dest)` / `new_with_block_offset(dest, off)`.
 * The writer borrows `dest` (the reference shares it via Rc, db.rs:56-63);
 * dest must outlive the writer.  block_offset is taken as given. */
revel_log_writer* revel_log_writer_new(revel_writable_file* dest, uint64_t block_offset);
/* log_writer.rs:58-97 `add_record(&mut self, slice) -> Result<()>`:
 * fragments into FULL/FIRST/MIDDLE/LAST physical records, zero-pads block
 * trailers < 7 bytes, header = [mask(crc32c(type||payload)) LE][len LE16][type],
 * flushes after every physical record (log_writer.rs:119). */
int revel_log_writer_add_record(revel_log_writer* w, const uint8_t* data, size_t n);
uint64_t revel_log_writer_block_offset(const revel_log_writer* w);
void revel_log_writer_free(revel_log_writer* w);

/* ---- GPU context -------------------------------------------------------- */
typedef struct revel_gpu_context revel_gpu_context;
/* Number of visible gfx950 devices (0 on a host without one). */
int revel_gpu_device_count(int* count);
/* PCI bus id ("dddd:bb:dd.f") of a visible HIP device: which physical GPU a
 * process drove (bench.py reports it per rank). */
int revel_gpu_device_pci_bus_id(int device, char* buf, size_t cap);
/* The compiler that built this library's gfx950 kernels (hipcc's clang
 * version string) and the offload target: build provenance for bench.py's
 * JSON line.  Static storage; never NULL. */
const char* revel_build_info(void);
/* One context per (thread, device): owns a HIP stream and scratch.  Every
 * GPU entry point binds the context's device for the duration of the call and
 * restores the calling thread's current device before it returns. */
int revel_gpu_context_new(int device, revel_gpu_context** out);
/* Readers created on a context pin it: freeing a context while readers
 * still use it is allowed and defers the release to the last reader's
 * revel_log_reader_free (the context must not be used for anything else
 * after this call). */
void revel_gpu_context_free(revel_gpu_context* ctx);
/* Drop the window buffers a freed reader parked on the context for the next
 * reader (pinned + device memory of about twice its window) and the pinned
 * ring a shard load keeps for the next one (3 windows). */
int revel_gpu_context_trim(revel_gpu_context* ctx);
/* The context's stream as an opaque hipStream_t. */
void* revel_gpu_context_stream(revel_gpu_context* ctx);

/* ---- log reader: src/log_reader.rs ------------------------------------- */
typedef struct revel_log_reader revel_log_reader;
/* log_reader.rs:62-74 `Reader::new(file, checksum, initial_offset)`:
 * revel_log_reader_new(file, checksum, initial_offset, NULL, 0, &r) is the
 * reference's 3-argument constructor.
 * The reader takes ownership of `file` (Box<dyn SequentialFile>) in every
 * case: on failure the file has been freed.
 * With checksum != 0 every physical record's CRC is verified ON THE GPU:
 * that of `gpu`, or with gpu == NULL of the calling thread's default context
 * (one per thread and current HIP device, created on first use, released when
 * the thread exits; REVEL_NOT_SUPPORT when the current device is not gfx950
 * -- there is no CPU fallback).  With checksum == 0 no GPU is used when gpu
 * is NULL.  The reader pins its context (see revel_gpu_context_free).
 * `window_bytes` = bytes read + verified per GPU batch (rounded up to a
 * block multiple; 0 = default 64 MiB). */
int revel_log_reader_new(revel_sequential_file* file, int checksum, uint64_t initial_offset,
                         revel_gpu_context* gpu, size_t window_bytes, revel_log_reader** out);
/* log_reader.rs:76-153 `read_record(&mut self, scratch) -> Result<Slice>`.
 * The returned bytes (data, n) borrow reader-owned memory valid until the next call (the
 * reference borrows the caller's scratch).  EOF: REVEL_OK with *n == 0 and
 * *data == NULL (the reference returns an empty Slice, :140).  A checksum
 * mismatch returns REVEL_IO_ERROR, as the reference does (:142-152). */
int revel_log_reader_read_record(revel_log_reader* r, const uint8_t** data, size_t* n);
/* log_reader.rs:76 with the reference's ownership: the record is written into
 * the caller's scratch (buf, cap) -- the `&mut Vec<u8>` the returned Slice
 * borrows -- and *n receives its length.  When cap is short the call returns
 * REVEL_INVALID_ARGUMENT with *n = the bytes needed and keeps the record: the
 * next read call (after the caller grows its scratch) returns it.  End of
 * file: REVEL_OK, *n == 0 and *eof = 1 (eof may be NULL: the reference's empty
 * Slice, :140, does not tell EOF from an empty record either).  Fragments are
 * assembled straight into buf while they fit, so a record is copied once. */
int revel_log_reader_read_record_into(revel_log_reader* r, uint8_t* buf, size_t cap, size_t* n, int* eof);
/* File offset of the first physical record of the last returned record. */
uint64_t revel_log_reader_last_record_offset(const revel_log_reader* r);
void revel_log_reader_free(revel_log_reader* r);

/* ---- device-resident CRC engine (the hot path) ------------------------- */
/* Per physical record result of revel_gpu_verify_records (24 bytes). */
typedef struct revel_record_result {
    uint64_t file_offset;   /* offset of the 7-byte header (base_offset + in-image offset) */
    uint32_t length;        /* payload length from the header */
    uint32_t stored_crc;    /* masked CRC stored in the header (coding.rs:139-144) */
    uint32_t computed_crc;  /* mask(crc32c(type || payload[:length])) */
    uint8_t type;           /* record type byte */
    uint8_t status;         /* REVEL_REC_* */
    uint8_t reserved[2];
} revel_record_result;

#define REVEL_REC_OK 0
#define REVEL_REC_BAD_CHECKSUM 1
#define REVEL_REC_BAD_LENGTH 2   /* 7 + length runs past the block end */
#define REVEL_REC_ZERO 3         /* type 0, length 0: preallocated region (log_reader.rs:195-198) */

/* Config C2 kernel.  d_blocks: nblocks * 32768 device bytes, every block one
 * FULL record of 32761 bytes.  d_masked_out[b] = mask(crc32c(block[6:32768]))
 * = the value log_writer.rs:107-111 stores for that payload;
 * d_ok[b] = (stored == computed && length == 32761 && type == FULL).
 * d_ok may be NULL.  Asynchronous on `stream` (NULL = context stream).
 * Alignment: any d_blocks is accepted and gives the same results; the
 * kernel's 16-byte loads run at full rate only when d_blocks is 16-byte
 * aligned (every revel_gpu_malloc / hipMalloc pointer is), an unaligned base
 * splits them (tests/test_gpu.py test_full_blocks_unaligned_base). */
int revel_gpu_crc_full_blocks(revel_gpu_context* ctx, const void* d_blocks, size_t nblocks,
                              uint32_t* d_masked_out, uint8_t* d_ok, void* stream);

/* GPU append framing for config C2 (log_writer.rs:99-124 on device): given
 * nblocks * 32768 bytes whose payload bytes [7:32768) are filled, write each
 * block's FULL header [mask(crc) LE][0xF9 0x7F][0x01] in place. */
int revel_gpu_frame_full_blocks(revel_gpu_context* ctx, void* d_blocks, size_t nblocks, void* stream);

/* Variable-layout verify (config C3).  Two steps so the caller sizes the
 * output:  (1) count physical records of each block of the image
 * (d_counts[nblocks]); (2) walk + CRC every record, writing record k of
 * block b to d_out[d_first[b] + k] where d_first is the exclusive prefix sum
 * of d_counts (revel_gpu_exclusive_scan_u32 computes it on device;
 * revel_gpu_count_scan_records does the count and the scan in one call, the
 * scan taking the count pass's per-64-block sums as its first pass).
 * nbytes need not be a block multiple (the last block may be partial).
 * The count pass also leaves per-block header lists in the context: a verify
 * of the same image on the same context uses them (for blocks with more than
 * 256 records it first lists the rest into their own d_out slots, which it
 * then overwrites with the results); without them verify walks the headers
 * itself, with the same results, slower.  A context's count -> verify pair
 * must not interleave with another on that context (use one context per
 * concurrent stream).  The verify pass reads the image itself: a change to
 * the image between the two calls is seen by verify (its records' checksums),
 * though the record layout comes from the count pass.
 * Record indices are u32: an image holding 2^32 or more physical records
 * (possible from ~28 GiB up: an empty record is 7 bytes, 4681 per block) is
 * refused by both count calls with REVEL_INVALID_ARGUMENT (the check sums the
 * counts in 64 bits and synchronises the stream; images of at most
 * 917503 blocks cannot wrap and are not checked).  Verify such a log in
 * pieces split at block boundaries. */
int revel_gpu_count_records(revel_gpu_context* ctx, const void* d_image, size_t nbytes,
                            uint32_t* d_counts, void* stream);
int revel_gpu_count_scan_records(revel_gpu_context* ctx, const void* d_image, size_t nbytes,
                                 uint32_t* d_counts, uint32_t* d_first, void* stream);
int revel_gpu_exclusive_scan_u32(revel_gpu_context* ctx, const uint32_t* d_in, uint32_t* d_out,
                                 size_t n, void* stream);
int revel_gpu_verify_records(revel_gpu_context* ctx, const void* d_image, size_t nbytes,
                             uint64_t base_offset, const uint32_t* d_first,
                             revel_record_result* d_out, void* stream);

/* ---- device replay reassembly (log_reader.rs:76-153 for a whole image) -- */
/* One entry per event a Reader produces while reading the image from its
 * start and continuing after every error: a logical record (FULL, or FIRST
 * MIDDLE* LAST, all valid) with its payload gathered contiguously, or an error
 * (the reader's Err(IOError)).  Incomplete fragments are dropped silently and
 * a torn final record ends the image, as the reader does. */
typedef struct revel_logical_record {
    uint64_t file_offset;     /* header offset of the first physical record */
    uint64_t payload_offset;  /* offset of the payload in the gathered buffer */
    uint32_t length;          /* payload bytes (0 for an error event) */
    uint32_t first_phys;      /* index range into the physical-record array */
    uint32_t last_phys;
    uint8_t status;           /* REVEL_LOGICAL_OK, or the REVEL_REC_* / BAD_TYPE error */
    uint8_t reserved[3];
} revel_logical_record;
#define REVEL_LOGICAL_OK 0
#define REVEL_LOGICAL_BAD_TYPE 4   /* record type outside FULL..LAST (log_reader.rs:126-128) */
/* d_phys: the nphys results of revel_gpu_verify_records for d_image (whose
 * byte 0 is file offset image_base, length image_len).  d_out needs nphys
 * entries, d_payload image_len bytes.  checksum = 0 ignores CRC mismatches.
 * Returns when done, with the event count in *nlogical and the gathered
 * payload bytes in *payload_bytes. */
int revel_gpu_reassemble(revel_gpu_context* ctx, const void* d_image, uint64_t image_base, uint64_t image_len,
                         const revel_record_result* d_phys, size_t nphys, int checksum,
                         revel_logical_record* d_out, void* d_payload, uint64_t* nlogical,
                         uint64_t* payload_bytes, void* stream);

/* ---- device WriteBatch decode (write_batch.rs:79-128 + insert_into :178-181)
 * Each reassembled logical record of a WAL is one WriteBatch rep:
 * [seq fixed64][count fixed32] then count x (tag, varint32 klen, key
 * [, varint32 vlen, value]).  Decoding is LevelDB-correct (the reference's
 * iterate() never advances past a deletion and sequence() reads offset 8; see
 * DESIGN.md section 4.8).  Entry i of a batch carries sequence seq + i
 * (MemTableInserter, write_batch.rs:148-158). */
#define REVEL_BATCH_HEADER 12
#define REVEL_TYPE_DELETION 0   /* dbformat.rs:24-28 ValueType */
#define REVEL_TYPE_VALUE 1
#define REVEL_BATCH_OK 0
#define REVEL_BATCH_TOO_SMALL 1    /* < 12 bytes */
#define REVEL_BATCH_BAD_ENTRY 2    /* key/value varint or length out of range */
#define REVEL_BATCH_BAD_TAG 3      /* tag not 0/1 (dbformat.rs:36 panics) */
#define REVEL_BATCH_WRONG_COUNT 4  /* decoded entries != header count */
#define REVEL_BATCH_NOT_RECORD 5   /* the logical event was a log error */
typedef struct revel_batch_info {
    uint64_t sequence;     /* header sequence (rep[0..8]) */
    uint64_t first_entry;  /* index of its first entry in the entry table */
    uint32_t count;        /* header count (rep[8..12]) */
    uint32_t nentries;     /* entries decoded (those before an error, on error) */
    uint8_t status;        /* REVEL_BATCH_* */
    uint8_t reserved[7];
} revel_batch_info;
typedef struct revel_batch_entry {
    uint64_t sequence;      /* batch sequence + entry index */
    uint64_t key_offset;    /* offsets into the gathered payload buffer */
    uint64_t value_offset;  /* (value_len 0 and offset past the key for a deletion) */
    uint32_t key_len;
    uint32_t value_len;
    uint32_t batch;         /* logical record index */
    uint8_t type;           /* REVEL_TYPE_VALUE / REVEL_TYPE_DELETION */
    uint8_t reserved[3];
} revel_batch_entry;
/* d_payload / d_logical: the outputs of revel_gpu_reassemble (nlogical
 * events over payload_bytes bytes).  d_info receives nlogical infos; entries
 * go to d_entries (capacity entries_cap; payload_bytes / 2 always suffices,
 * every entry being at least 2 bytes).  *nentries receives the total entry
 * count; REVEL_INVALID_ARGUMENT if it exceeds entries_cap (infos are still
 * written, entries past the cap are not).  Returns when done. */
int revel_gpu_decode_batches(revel_gpu_context* ctx, const void* d_payload, uint64_t payload_bytes,
                             const revel_logical_record* d_logical, size_t nlogical, revel_batch_info* d_info,
                             revel_batch_entry* d_entries, size_t entries_cap, uint64_t* nentries, void* stream);

/* ---- device append framing (log_writer.rs:58-124 for a whole batch) ----- */
/* Bytes that n successive add_record calls starting at block_offset would
 * append (headers, payloads, zero trailers). */
uint64_t revel_log_framed_size(const uint64_t* lens, size_t n, uint64_t block_offset);
/* Frame n records on the GPU exactly as n successive
 * Writer::add_record calls would (log_writer.rs:58-97): payloads are
 * concatenated in device memory (d_payloads), lengths on the host.  The
 * fragment layout is computed on the host; payload scatter, zero trailers and
 * every header's masked CRC32C are computed on the device.  The image (the
 * bytes the writer would append, starting at *block_offset within the current
 * block) goes to d_image (capacity image_cap); *image_len receives its size
 * and *block_offset is advanced like Writer::block_offset.  Returns when the
 * image is complete. */
int revel_gpu_append_records(revel_gpu_context* ctx, const void* d_payloads, const uint64_t* lens, size_t n,
                             uint64_t* block_offset, void* d_image, size_t image_cap, size_t* image_len,
                             void* stream);

/* ---- device plumbing (used by the reader, tests and bench) -------------- */
int revel_gpu_malloc(revel_gpu_context* ctx, size_t n, void** d_ptr);
int revel_gpu_free(revel_gpu_context* ctx, void* d_ptr);
int revel_gpu_host_alloc(revel_gpu_context* ctx, size_t n, void** h_pinned);
int revel_gpu_host_free(revel_gpu_context* ctx, void* h_pinned);
int revel_gpu_memcpy_h2d(revel_gpu_context* ctx, void* d_dst, const void* h_src, size_t n, void* stream);
int revel_gpu_memcpy_d2h(revel_gpu_context* ctx, void* h_dst, const void* d_src, size_t n, void* stream);
int revel_gpu_memset(revel_gpu_context* ctx, void* d_dst, int value, size_t n, void* stream);
int revel_gpu_stream_synchronize(revel_gpu_context* ctx, void* stream);
int revel_gpu_device_synchronize(revel_gpu_context* ctx);
/* Fill nblocks full-type blocks on device: payload = splitmix64(seed ^ (first+b))
 * (same bytes as oracle_synth_full_blocks), then frame the headers. */
int revel_gpu_synth_full_blocks(revel_gpu_context* ctx, void* d_blocks, size_t nblocks,
                                uint64_t seed, uint64_t first, void* stream);
/* HIP events for timing on a stream. */
int revel_gpu_event_new(revel_gpu_context* ctx, void** ev);
int revel_gpu_event_record(revel_gpu_context* ctx, void* ev, void* stream);
int revel_gpu_event_elapsed_ms(revel_gpu_context* ctx, void* start, void* stop, float* ms);
int revel_gpu_event_free(revel_gpu_context* ctx, void* ev);
/* Human-readable description of the last error on this thread. */
const char* revel_last_error(void);

/* ---- end-to-end replay: host bytes -> pinned ring -> HBM -> verify ------ */
/* Replays a WAL held in a host file (or host memory) through the GPU: a ring
 * of `nbuffers` pinned windows is filled by `io_threads` host threads (pread /
 * memcpy), each window is copied to HBM on a copy stream and verified on the
 * context's stream while the next windows are read and copied; only a small
 * per-window summary returns to the host.  This is the end-to-end rate of
 * log_reader.rs's path (env.rs:162-169 read(2) -> CRC), PCIe-inclusive.
 * mode REVEL_REPLAY_RECORDS verifies every physical record (config C3/C5
 * layout); REVEL_REPLAY_FULL_BLOCKS treats every block as one FULL record
 * (config C2 layout).  Windows are whole blocks; records never cross a block,
 * so window boundaries are exact.
 * For revel_gpu_replay_file, one REVEL_REPLAY_IO_* flag may be or-ed into mode
 * to choose how windows are read (SequentialFile::read, env.rs:162-169, in
 * bulk): a read-only MAP_SHARED mapping copied by the io threads (default;
 * the file must not shrink during the replay), buffered pread, or O_DIRECT
 * pread (REVEL_NOT_SUPPORT where the file system refuses O_DIRECT; there is
 * no silent fallback).  DESIGN.md section 4.4 has the measured rates. */
#define REVEL_REPLAY_RECORDS 0
#define REVEL_REPLAY_FULL_BLOCKS 1
#define REVEL_REPLAY_IO_MMAP 0x00
#define REVEL_REPLAY_IO_PREAD 0x10
#define REVEL_REPLAY_IO_DIRECT 0x20
typedef struct revel_replay_stats {
    uint64_t bytes;            /* bytes replayed */
    uint64_t windows;          /* windows processed */
    uint64_t units;            /* physical records (RECORDS) or blocks (FULL_BLOCKS) verified */
    uint64_t bad;              /* units whose CRC / header failed */
    uint64_t first_bad_offset; /* file offset of the first bad unit, UINT64_MAX if none */
    double seconds;            /* host wall time, first read to last verdict */
    double read_seconds;       /* summed host time spent filling pinned windows */
    double h2d_ms;             /* summed H2D copy time (HIP events) */
    double kernel_ms;          /* summed verify time (HIP events) */
} revel_replay_stats;
int revel_gpu_replay_file(revel_gpu_context* ctx, const char* path, uint64_t offset, uint64_t length, int mode,
                          size_t window_bytes, int nbuffers, int io_threads, revel_replay_stats* out);
int revel_gpu_replay_memory(revel_gpu_context* ctx, const uint8_t* image, uint64_t length, uint64_t base_offset,
                            int mode, size_t window_bytes, int nbuffers, int io_threads, revel_replay_stats* out);

/* ---- one WAL across several GPUs (config C5 on N GPUs) ----
 * Physical records never cross a 32 KiB block (log_writer.rs:66-76), so a WAL
 * splits into contiguous block-aligned shards that are verified (and
 * reassembled) independently, one per GPU, with no collective.  Only logical
 * records whose fragments span a shard boundary need the neighbours: each
 * shard keeps its boundary records (the leading MIDDLE/LAST run and the open
 * FIRST MIDDLE* tail), and a host stitch folds them in file order with the
 * reader's rules (log_reader.rs:95-129, LevelDB-correct as the replay reader).
 * In one process revel_gpu_replay_sharded drives n contexts on n host threads;
 * with one process per GPU each rank loads its shard, exports its boundary
 * (revel_wal_shard_boundary) and one rank stitches the gathered blobs. */
typedef struct revel_wal_shard revel_wal_shard;
/* offsets[0..n]: n contiguous block-aligned ranges covering [0, file_bytes)
 * (offsets[k+1] - offsets[k] = shard k's bytes; trailing shards may be empty). */
int revel_wal_shard_ranges(uint64_t file_bytes, int n, uint64_t* offsets);
#define REVEL_SHARD_VERIFY 0  /* load + verify every physical record, boundary records kept */
#define REVEL_SHARD_READ 1    /* + device reassembly: logical records and their payloads in HBM */
typedef struct revel_wal_shard_info {
    int device;
    int checksum;
    uint64_t offset, length;     /* the shard's byte range of the WAL */
    uint64_t file_bytes;         /* the WAL's size (torn-tail rule at its end) */
    uint64_t physical, bad;      /* physical records verified / not REVEL_REC_OK */
    uint64_t events, records;    /* READ: shard-local events (revel_gpu_reassemble), records among them */
    uint64_t payload_bytes;      /* READ: gathered payload bytes of those records */
    const void* d_image;         /* the shard's bytes in HBM (library-owned) */
    const revel_record_result* d_phys;
    const revel_logical_record* d_events;  /* READ */
    const void* d_payload;       /* READ */
    double setup_seconds;        /* allocating the shard's HBM buffers (+ the pinned ring, first load
                                    on a context only: the ring is kept on the context) */
    double seconds;              /* host wall time of the pipeline after setup: read + H2D + verify
                                    [+ reassembly] + boundary */
    double read_seconds;         /* summed host time filling pinned windows */
    double h2d_ms, kernel_ms;    /* summed H2D time / verify (+ reassembly) time, HIP events */
} revel_wal_shard_info;
/* Loads bytes [offset, offset + length) of the WAL at `path` (mmap'd; or of
 * the host `image` holding the whole WAL when path is NULL) into HBM of ctx's
 * device: io_threads fill a ring of pinned windows (window_bytes, 0 = 64 MiB),
 * each is copied on a copy stream and its records counted on the context
 * stream as it lands; then every physical record is verified (and with
 * REVEL_SHARD_READ reassembled) on the device.  offset must be block-aligned
 * and offset + length a block multiple or file_bytes.  The shard pins ctx. */
int revel_gpu_wal_shard_load(revel_gpu_context* ctx, const char* path, const uint8_t* image, uint64_t file_bytes,
                             uint64_t offset, uint64_t length, int checksum, int flags, size_t window_bytes,
                             int io_threads, revel_wal_shard** out);
int revel_wal_shard_info_get(const revel_wal_shard* s, revel_wal_shard_info* out);
/* The shard's boundary as a self-contained blob (records + their payloads
 * with REVEL_SHARD_READ): with buf NULL, *n = the size needed. */
int revel_wal_shard_boundary(const revel_wal_shard* s, uint8_t* buf, size_t cap, size_t* n);
void revel_wal_shard_free(revel_wal_shard* s);
/* The same boundary blob from a host header walk of the WAL bytes in host
 * memory (image = the whole WAL), for a Reader with checksum == false: no
 * CRC, no GPU (the CPU side of the one-process-per-GPU stitch, and its tests). */
int revel_wal_shard_boundary_host(const uint8_t* image, uint64_t file_bytes, uint64_t offset, uint64_t length,
                                  int flags, uint8_t* buf, size_t cap, size_t* n);

/* Host stitch of n shards' boundary blobs, in file order (contiguous). */
typedef struct revel_wal_stitch revel_wal_stitch;
typedef struct revel_wal_summary {
    uint64_t bytes;          /* WAL bytes covered */
    uint64_t physical, bad;  /* physical records verified / not REVEL_REC_OK */
    uint64_t records;        /* READ: logical records a Reader returns, stitched ones included */
    uint64_t errors;         /* READ: Err(IOError) events a Reader returns */
    uint64_t payload_bytes;  /* READ: their payload bytes; VERIFY: those of the stitched records only */
    uint64_t stitched;       /* logical records assembled across shard boundaries */
    double seconds;          /* revel_gpu_replay_sharded: wall time of the parallel loads + stitch */
} revel_wal_summary;
int revel_wal_stitch_new(const uint8_t* const* blobs, const size_t* sizes, int n, revel_wal_stitch** out);
int revel_wal_stitch_summary(const revel_wal_stitch* st, revel_wal_summary* out);
/* Stitched record i: header offset of its FIRST, payload (host, valid while
 * the stitch lives; NULL in VERIFY mode), and `before_shard` = the shard whose
 * own events it precedes in file order. */
int revel_wal_stitch_record(const revel_wal_stitch* st, size_t i, uint64_t* file_offset, const uint8_t** data,
                            uint64_t* n, int* before_shard);
void revel_wal_stitch_free(revel_wal_stitch* st);

/* One process, n GPUs: shard the WAL (revel_wal_shard_ranges), load shard k on
 * ctxs[k] on its own host thread, stitch.  With REVEL_SHARD_READ,
 * revel_sharded_replay_next then returns the logical records in file order
 * exactly as Reader::read_record would (log_reader.rs:76-153): REVEL_OK with
 * the payload (valid until the next call), REVEL_IO_ERROR for an error event
 * (continue calling), REVEL_OK with *data NULL at the end. */
typedef struct revel_sharded_replay revel_sharded_replay;
int revel_gpu_replay_sharded(revel_gpu_context* const* ctxs, int n, const char* path, const uint8_t* image,
                             uint64_t file_bytes, int checksum, int flags, size_t window_bytes, int io_threads,
                             revel_sharded_replay** out);
int revel_sharded_replay_summary(const revel_sharded_replay* r, revel_wal_summary* out);
const revel_wal_shard* revel_sharded_replay_shard(const revel_sharded_replay* r, int k);
int revel_sharded_replay_next(revel_sharded_replay* r, const uint8_t** data, size_t* n, uint64_t* file_offset);
void revel_sharded_replay_free(revel_sharded_replay* r);

#ifdef __cplusplus
}
#endif

#endif /* REVEL_WAL_H_ */
