// host_log.cpp -- host side of the WAL path behind include/revel_wal.h:
// CRC32C on the CPU for the writer, file abstractions, log::Writer and the
// GPU-verified log::Reader.
//
//   src/util/crc.rs:17-44     revel_crc32c_value/extend/mask/unmask
//   src/env.rs:25-266         revel_*_file_*
//   src/log_writer.rs:25-124  revel_log_writer_*
//   src/log_reader.rs:38-216  revel_log_reader_*
//
// The writer computes each record's CRC on the host (one record at a time,
// as log_writer.rs:107-111 does) with the x86 SSE4.2 crc32 instruction.  The
// reader verifies CRCs in bulk on the GPU: it reads a window of whole 32 KiB
// blocks into pinned memory, copies it to HBM, and runs the record-walk +
// segmented CRC kernels; read_record then reassembles logical records from
// the window with the per-record verdicts.
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <string>
#include <vector>

#include "crc32c_math.h"
#include "gpu_internal.h"
#include "revel_wal.h"

using revel::set_error;

// ===========================================================================
// CRC32C (host).  x86-64 SSE4.2 `crc32` computes the CRC-32C register update.
// ===========================================================================
namespace {

#if !defined(__x86_64__)
#error "host CRC path is written for x86-64 hosts (SSE4.2 crc32)"
#endif

__attribute__((target("sse4.2"))) uint32_t crc_update(uint32_t s, const uint8_t* p, size_t n) {
    uint64_t s64 = s;
    while (n >= 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        s64 = __builtin_ia32_crc32di(s64, w);
        p += 8;
        n -= 8;
    }
    uint32_t s32 = (uint32_t)s64;
    while (n--) s32 = __builtin_ia32_crc32qi(s32, *p++);
    return s32;
}

}  // namespace

extern "C" {

uint32_t revel_crc32c_value(const uint8_t* data, size_t n) {
    return crc_update(0xFFFFFFFFu, data, n) ^ 0xFFFFFFFFu;
}

uint32_t revel_crc32c_extend(uint8_t init, const uint8_t* data, size_t n) {
    uint32_t s = crc_update(0xFFFFFFFFu, &init, 1);
    return crc_update(s, data, n) ^ 0xFFFFFFFFu;
}

uint32_t revel_crc32c_mask(uint32_t crc) { return revel::mask(crc); }
uint32_t revel_crc32c_unmask(uint32_t masked) { return revel::unmask(masked); }

}  // extern "C"

// ===========================================================================
// Files (env.rs)
// ===========================================================================
struct revel_writable_file {
    enum Kind { MEMORY, POSIX, CALLBACK } kind = MEMORY;
    std::vector<uint8_t> mem;
    int fd = -1;
    std::vector<uint8_t> buf;  // posix write buffer, env.rs:69 kWritableFileBufferSize
    size_t pos = 0;
    std::string path;
    // CALLBACK: the caller's `dyn WritableFile` (env.rs:40-50)
    void* user = nullptr;
    revel_file_append_fn cb_append = nullptr;
    revel_file_op_fn cb_flush = nullptr, cb_close = nullptr, cb_sync = nullptr;
    revel_file_release_fn cb_release = nullptr;
};

struct revel_sequential_file {
    enum Kind { MEMORY, POSIX, CALLBACK } kind = MEMORY;
    std::vector<uint8_t> mem;
    size_t off = 0;
    int fd = -1;
    // CALLBACK: the caller's `dyn SequentialFile` (env.rs:52-57)
    void* user = nullptr;
    revel_file_read_fn cb_read = nullptr;
    revel_file_skip_fn cb_skip = nullptr;
    revel_file_release_fn cb_release = nullptr;
};

namespace {

constexpr size_t kWritableFileBufferSize = 65536;

int write_all(int fd, const uint8_t* p, size_t n) {
    while (n) {
        ssize_t w = ::write(fd, p, n);
        if (w < 0) {
            if (errno == EINTR) continue;
            return set_error(REVEL_IO_ERROR, "write: %s", strerror(errno));
        }
        p += w;
        n -= (size_t)w;
    }
    return REVEL_OK;
}

int posix_flush_buffer(revel_writable_file* f) {
    int rc = write_all(f->fd, f->buf.data(), f->pos);
    f->pos = 0;
    return rc;
}

// A caller callback's status: 0 = Ok, 1..5 = the error.rs code it returned,
// anything else is reported as IOError.
int callback_status(int rc, const char* what) {
    if (rc == REVEL_OK) return REVEL_OK;
    const int code = rc >= REVEL_NOT_FOUND && rc <= REVEL_IO_ERROR ? rc : REVEL_IO_ERROR;
    return set_error(code, "%s callback returned %d", what, rc);
}

int callback_op(revel_file_op_fn fn, void* user, const char* what) {
    return fn ? callback_status(fn(user), what) : REVEL_OK;
}

}  // namespace

extern "C" {

revel_writable_file* revel_memory_writable_file_new(void) { return new revel_writable_file; }

int revel_posix_writable_file_new(const char* path, revel_writable_file** out) {
    if (!path || !out) return set_error(REVEL_INVALID_ARGUMENT, "null path/out");
    *out = nullptr;
    int fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) return set_error(REVEL_IO_ERROR, "open(%s): %s", path, strerror(errno));
    auto* f = new revel_writable_file;
    f->kind = revel_writable_file::POSIX;
    f->fd = fd;
    f->buf.resize(kWritableFileBufferSize);
    f->path = path;
    *out = f;
    return REVEL_OK;
}

int revel_writable_file_from_callbacks(void* user, revel_file_append_fn append, revel_file_op_fn flush,
                                       revel_file_op_fn close, revel_file_op_fn sync, revel_file_release_fn release,
                                       revel_writable_file** out) {
    if (!out) return set_error(REVEL_INVALID_ARGUMENT, "null out");
    *out = nullptr;
    if (!append) return set_error(REVEL_INVALID_ARGUMENT, "append callback is required");
    auto* f = new revel_writable_file;
    f->kind = revel_writable_file::CALLBACK;
    f->user = user;
    f->cb_append = append;
    f->cb_flush = flush;
    f->cb_close = close;
    f->cb_sync = sync;
    f->cb_release = release;
    *out = f;
    return REVEL_OK;
}

// env.rs:116-136 intent: buffer small appends, write large ones directly.
int revel_writable_file_append(revel_writable_file* f, const uint8_t* data, size_t n) {
    if (!f || (!data && n)) return set_error(REVEL_INVALID_ARGUMENT, "null file/data");
    if (f->kind == revel_writable_file::MEMORY) {
        f->mem.insert(f->mem.end(), data, data + n);
        return REVEL_OK;
    }
    if (f->kind == revel_writable_file::CALLBACK) return callback_status(f->cb_append(f->user, data, n), "append");
    if (f->fd < 0) return set_error(REVEL_IO_ERROR, "append to closed file");
    size_t copy = std::min(n, kWritableFileBufferSize - f->pos);
    memcpy(f->buf.data() + f->pos, data, copy);
    f->pos += copy;
    data += copy;
    n -= copy;
    if (n == 0) return REVEL_OK;
    int rc = posix_flush_buffer(f);
    if (rc) return rc;
    if (n < kWritableFileBufferSize) {
        memcpy(f->buf.data(), data, n);
        f->pos = n;
        return REVEL_OK;
    }
    return write_all(f->fd, data, n);
}

int revel_writable_file_flush(revel_writable_file* f) {
    if (!f) return set_error(REVEL_INVALID_ARGUMENT, "null file");
    if (f->kind == revel_writable_file::MEMORY) return REVEL_OK;
    if (f->kind == revel_writable_file::CALLBACK) return callback_op(f->cb_flush, f->user, "flush");
    if (f->fd < 0) return set_error(REVEL_IO_ERROR, "flush of closed file");
    return posix_flush_buffer(f);
}

int revel_writable_file_close(revel_writable_file* f) {
    if (!f) return set_error(REVEL_INVALID_ARGUMENT, "null file");
    if (f->kind == revel_writable_file::CALLBACK) return callback_op(f->cb_close, f->user, "close");
    if (f->kind == revel_writable_file::MEMORY || f->fd < 0) return REVEL_OK;
    int rc = posix_flush_buffer(f);
    if (::close(f->fd) != 0 && rc == REVEL_OK) rc = set_error(REVEL_IO_ERROR, "close: %s", strerror(errno));
    f->fd = -1;
    return rc;
}

int revel_writable_file_sync(revel_writable_file* f) {
    if (!f) return set_error(REVEL_INVALID_ARGUMENT, "null file");
    if (f->kind == revel_writable_file::MEMORY) return REVEL_OK;
    if (f->kind == revel_writable_file::CALLBACK) return callback_op(f->cb_sync, f->user, "sync");
    if (f->fd < 0) return set_error(REVEL_IO_ERROR, "sync of closed file");
    int rc = posix_flush_buffer(f);
    if (rc) return rc;
    if (::fsync(f->fd) != 0) return set_error(REVEL_IO_ERROR, "fsync: %s", strerror(errno));
    return REVEL_OK;
}

int revel_memory_writable_file_contents(const revel_writable_file* f, const uint8_t** data, size_t* n) {
    if (!f || !data || !n) return set_error(REVEL_INVALID_ARGUMENT, "null argument");
    if (f->kind != revel_writable_file::MEMORY) return set_error(REVEL_INVALID_ARGUMENT, "not a memory file");
    *data = f->mem.data();
    *n = f->mem.size();
    return REVEL_OK;
}

void revel_writable_file_free(revel_writable_file* f) {
    if (!f) return;
    if (f->kind == revel_writable_file::POSIX && f->fd >= 0) (void)revel_writable_file_close(f);
    if (f->kind == revel_writable_file::CALLBACK && f->cb_release) f->cb_release(f->user);
    delete f;
}

revel_sequential_file* revel_memory_sequential_file_new(const uint8_t* data, size_t n) {
    auto* f = new revel_sequential_file;
    if (n) f->mem.assign(data, data + n);
    return f;
}

int revel_posix_sequential_file_new(const char* path, revel_sequential_file** out) {
    if (!path || !out) return set_error(REVEL_INVALID_ARGUMENT, "null path/out");
    *out = nullptr;
    int fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return set_error(errno == ENOENT ? REVEL_NOT_FOUND : REVEL_IO_ERROR, "open(%s): %s", path,
                                 strerror(errno));
    auto* f = new revel_sequential_file;
    f->kind = revel_sequential_file::POSIX;
    f->fd = fd;
    *out = f;
    return REVEL_OK;
}

int revel_sequential_file_from_callbacks(void* user, revel_file_read_fn read, revel_file_skip_fn skip,
                                         revel_file_release_fn release, revel_sequential_file** out) {
    if (!out) return set_error(REVEL_INVALID_ARGUMENT, "null out");
    *out = nullptr;
    if (!read) return set_error(REVEL_INVALID_ARGUMENT, "read callback is required");
    auto* f = new revel_sequential_file;
    f->kind = revel_sequential_file::CALLBACK;
    f->user = user;
    f->cb_read = read;
    f->cb_skip = skip;
    f->cb_release = release;
    *out = f;
    return REVEL_OK;
}

int revel_sequential_file_read(revel_sequential_file* f, uint8_t* scratch, size_t n, size_t* got) {
    if (!f || !got || (!scratch && n)) return set_error(REVEL_INVALID_ARGUMENT, "null argument");
    *got = 0;
    if (f->kind == revel_sequential_file::MEMORY) {
        size_t avail = f->off < f->mem.size() ? f->mem.size() - f->off : 0;
        size_t k = std::min(n, avail);
        if (k) memcpy(scratch, f->mem.data() + f->off, k);
        f->off += k;
        *got = k;
        return REVEL_OK;
    }
    // fill as much as the file has: read(2) and a caller's read may both
    // return short counts before the end of the file
    size_t total = 0;
    while (total < n) {
        if (f->kind == revel_sequential_file::CALLBACK) {
            size_t k = 0;
            int rc = callback_status(f->cb_read(f->user, scratch + total, n - total, &k), "read");
            if (rc) return rc;
            if (k > n - total) return set_error(REVEL_IO_ERROR, "read callback filled %zu of %zu bytes", k, n - total);
            if (k == 0) break;
            total += k;
            continue;
        }
        ssize_t r = ::read(f->fd, scratch + total, n - total);
        if (r < 0) {
            if (errno == EINTR) continue;
            return set_error(REVEL_IO_ERROR, "read: %s", strerror(errno));
        }
        if (r == 0) break;
        total += (size_t)r;
    }
    *got = total;
    return REVEL_OK;
}

int revel_sequential_file_skip(revel_sequential_file* f, uint64_t n) {
    if (!f) return set_error(REVEL_INVALID_ARGUMENT, "null file");
    if (f->kind == revel_sequential_file::MEMORY) {
        f->off += n;
        return REVEL_OK;
    }
    if (f->kind == revel_sequential_file::CALLBACK) {
        if (f->cb_skip) return callback_status(f->cb_skip(f->user, n), "skip");
        uint8_t sink[4096];  // no skip callback: read and drop
        while (n) {
            size_t k = 0;
            int rc = revel_sequential_file_read(f, sink, (size_t)std::min<uint64_t>(n, sizeof sink), &k);
            if (rc) return rc;
            if (k == 0) break;
            n -= k;
        }
        return REVEL_OK;
    }
    if (::lseek(f->fd, (off_t)n, SEEK_CUR) < 0) return set_error(REVEL_IO_ERROR, "lseek: %s", strerror(errno));
    return REVEL_OK;
}

void revel_sequential_file_free(revel_sequential_file* f) {
    if (!f) return;
    if (f->kind == revel_sequential_file::POSIX && f->fd >= 0) ::close(f->fd);
    if (f->kind == revel_sequential_file::CALLBACK && f->cb_release) f->cb_release(f->user);
    delete f;
}

}  // extern "C"

// ===========================================================================
// log::Writer (log_writer.rs:25-124)
// ===========================================================================
struct revel_log_writer {
    revel_writable_file* dest;
    uint64_t block_offset;
};

namespace {

int emit_physical_record(revel_log_writer* w, uint8_t type, const uint8_t* data, size_t n) {
    uint8_t hdr[REVEL_HEADER_SIZE];
    hdr[4] = (uint8_t)(n & 0xff);
    hdr[5] = (uint8_t)(n >> 8);
    hdr[6] = type;
    // log_writer.rs:107-111: extend(type_crc[type], data) with type_crc[t] = t
    const uint32_t crc = revel::mask(revel_crc32c_extend(type, data, n));
    hdr[0] = (uint8_t)crc;
    hdr[1] = (uint8_t)(crc >> 8);
    hdr[2] = (uint8_t)(crc >> 16);
    hdr[3] = (uint8_t)(crc >> 24);
    // log_writer.rs:114-121: each `?` returns before block_offset advances
    int rc = revel_writable_file_append(w->dest, hdr, REVEL_HEADER_SIZE);
    if (rc) return rc;
    rc = revel_writable_file_append(w->dest, data, n);
    if (rc) return rc;
    rc = revel_writable_file_flush(w->dest);  // log_writer.rs:119
    if (rc) return rc;
    w->block_offset += REVEL_HEADER_SIZE + n;
    return REVEL_OK;
}

}  // namespace

extern "C" {

revel_log_writer* revel_log_writer_new(revel_writable_file* dest, uint64_t block_offset) {
    if (!dest) return nullptr;
    return new revel_log_writer{dest, block_offset};
}

int revel_log_writer_add_record(revel_log_writer* w, const uint8_t* data, size_t n) {
    if (!w || (!data && n)) return set_error(REVEL_INVALID_ARGUMENT, "null writer/data");
    static const uint8_t kZeros[REVEL_HEADER_SIZE] = {0};
    size_t left = n, off = 0;
    bool begin = true;
    for (;;) {
        if (w->block_offset > REVEL_BLOCK_SIZE)
            return set_error(REVEL_INVALID_ARGUMENT, "block_offset %llu > block size",
                             (unsigned long long)w->block_offset);
        const size_t leftover = REVEL_BLOCK_SIZE - (size_t)w->block_offset;
        if (leftover < REVEL_HEADER_SIZE) {
            if (leftover > 0) {  // log_writer.rs:66-71: zero-fill the trailer
                int rc = revel_writable_file_append(w->dest, kZeros, leftover);
                if (rc) return rc;
            }
            w->block_offset = 0;
        }
        const size_t avail = REVEL_BLOCK_SIZE - (size_t)w->block_offset - REVEL_HEADER_SIZE;
        const size_t frag = left < avail ? left : avail;
        const bool end = left == frag;
        const uint8_t type = (begin && end) ? REVEL_FULL_TYPE
                             : begin        ? REVEL_FIRST_TYPE
                             : end          ? REVEL_LAST_TYPE
                                            : REVEL_MIDDLE_TYPE;
        int rc = emit_physical_record(w, type, data + off, frag);
        if (rc) return rc;
        off += frag;
        left -= frag;
        begin = false;
        if (left == 0) return REVEL_OK;
    }
}

uint64_t revel_log_writer_block_offset(const revel_log_writer* w) { return w ? w->block_offset : 0; }

}  // extern "C"

// Fragment layout of a batch of records (log_writer.rs:58-97, as the host
// writer above), for device append framing.
namespace {

uint64_t frame_layout(const uint64_t* lens, size_t n, uint64_t& boff, std::vector<revel::FragDesc>* frags) {
    uint64_t pos = 0, src = 0;
    for (size_t r = 0; r < n; ++r) {
        uint64_t left = lens[r], off = 0;
        bool begin = true;
        for (;;) {
            const uint64_t leftover = REVEL_BLOCK_SIZE - boff;
            if (leftover < REVEL_HEADER_SIZE) {
                if (leftover > 0) {
                    if (frags) frags->push_back({pos, 0, (uint32_t)leftover, revel::kTrailer});
                    pos += leftover;
                }
                boff = 0;
            }
            const uint64_t avail = REVEL_BLOCK_SIZE - boff - REVEL_HEADER_SIZE;
            const uint64_t frag = left < avail ? left : avail;
            const bool end = left == frag;
            const uint32_t type = (begin && end) ? REVEL_FULL_TYPE
                                  : begin        ? REVEL_FIRST_TYPE
                                  : end          ? REVEL_LAST_TYPE
                                                 : REVEL_MIDDLE_TYPE;
            if (frags) frags->push_back({pos, src + off, (uint32_t)frag, type});
            pos += REVEL_HEADER_SIZE + frag;
            boff += REVEL_HEADER_SIZE + frag;
            off += frag;
            left -= frag;
            begin = false;
            if (left == 0) break;
        }
        src += lens[r];
    }
    return pos;
}

}  // namespace

extern "C" {

uint64_t revel_log_framed_size(const uint64_t* lens, size_t n, uint64_t block_offset) {
    if ((!lens && n) || block_offset > REVEL_BLOCK_SIZE) return 0;
    uint64_t boff = block_offset;
    return frame_layout(lens, n, boff, nullptr);
}

int revel_gpu_append_records(revel_gpu_context* ctx, const void* d_payloads, const uint64_t* lens, size_t n,
                             uint64_t* block_offset, void* d_image, size_t image_cap, size_t* image_len,
                             void* stream) {
    if (!ctx || !block_offset || !image_len || (!lens && n)) return set_error(REVEL_INVALID_ARGUMENT, "null argument");
    if (*block_offset > REVEL_BLOCK_SIZE)
        return set_error(REVEL_INVALID_ARGUMENT, "block_offset %llu > block size", (unsigned long long)*block_offset);
    uint64_t boff = *block_offset;
    const uint32_t lead = (uint32_t)(boff % REVEL_BLOCK_SIZE);
    std::vector<revel::FragDesc> frags;
    const uint64_t len = frame_layout(lens, n, boff, &frags);
    *image_len = 0;
    if (len > image_cap) return set_error(REVEL_INVALID_ARGUMENT, "image capacity %zu < %llu", image_cap,
                                          (unsigned long long)len);
    if (len && (!d_image || (!d_payloads && frags.size()))) return set_error(REVEL_INVALID_ARGUMENT, "null device buffer");
    revel::DeviceGuard guard(ctx->di.device);
    if (guard.err() != hipSuccess) return set_error(REVEL_IO_ERROR, "hipSetDevice failed");
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    // Header lists for the device CRC pass: per virtual block (image byte 0 at
    // in-block offset `lead`) its record count and the fragment index of its
    // first record; the scatter kernel writes one entry per fragment.
    const uint64_t vblocks = (len + lead + REVEL_BLOCK_SIZE - 1) / REVEL_BLOCK_SIZE;
    std::vector<uint32_t> counts, first;
    const bool lists = !frags.empty() && frags.size() < (1ull << 32);
    if (lists) {
        counts.assign(vblocks, 0);
        first.assign(vblocks, 0);
        for (size_t f = 0; f < frags.size(); ++f) {
            if (frags[f].type == revel::kTrailer) continue;
            const uint64_t vb = (frags[f].dst + lead) / REVEL_BLOCK_SIZE;
            if (counts[vb]++ == 0) first[vb] = (uint32_t)f;
        }
    }
    revel::DeviceScratch scratch(&ctx->arena);
    revel::FragDesc* d_frags = nullptr;
    uint32_t *d_counts = nullptr, *d_first = nullptr;
    uint64_t* d_xlist = nullptr;
    uint32_t* d_blist = nullptr;
    hipError_t e = hipSuccess;
    if (!frags.empty()) {
        e = scratch.get(&d_frags, frags.size());
        if (e == hipSuccess)
            e = hipMemcpyAsync(d_frags, frags.data(), frags.size() * sizeof(revel::FragDesc), hipMemcpyHostToDevice, st);
    }
    if (lists) {
        if (e == hipSuccess) e = scratch.get(&d_counts, vblocks);
        if (e == hipSuccess) e = scratch.get(&d_first, vblocks);
        if (e == hipSuccess) e = scratch.get(&d_xlist, frags.size());
        if (e == hipSuccess) e = scratch.get(&d_blist, vblocks + revel::kBlockListAux);
        if (e == hipSuccess) e = hipMemcpyAsync(d_counts, counts.data(), vblocks * 4, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(d_first, first.data(), vblocks * 4, hipMemcpyHostToDevice, st);
    }
    if (e == hipSuccess)
        e = revel::frame_records(ctx->di, d_payloads, d_frags, frags.size(), d_image, len, lead, st, d_counts, d_first,
                                 d_xlist, d_blist);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        (void)hipStreamSynchronize(st);  // the context's scratch is free before the next call
        return set_error(REVEL_IO_ERROR, "append_records: %s", hipGetErrorString(e));
    }
    *image_len = len;
    *block_offset = boff;
    return REVEL_OK;
}

void revel_log_writer_free(revel_log_writer* w) { delete w; }

}  // extern "C"

// ===========================================================================
// log::Reader (log_reader.rs:38-216), GPU-verified.
// ===========================================================================
struct revel_log_reader {
    revel_sequential_file* file = nullptr;
    bool checksum = true;
    uint64_t initial_offset = 0;
    revel_gpu_context* gpu = nullptr;
    size_t window = 0;

    // current window of whole blocks
    uint8_t* win = nullptr;  // pinned host memory when gpu != nullptr
    std::vector<uint8_t> win_heap;
    size_t win_len = 0;
    uint64_t win_file_off = 0;  // file offset of win[0]
    uint64_t next_file_off = 0;
    bool file_eof = false;

    std::vector<revel_record_result> recs;
    size_t rec_i = 0;

    // device scratch
    void* d_win = nullptr;
    uint32_t* d_counts = nullptr;
    uint32_t* d_first = nullptr;
    revel_record_result* d_out = nullptr;
    size_t d_out_cap = 0;

    bool resyncing = false;
    uint64_t last_record_offset = 0;
    std::vector<uint8_t> scratch;

    // A record read_record_into could not deliver (the caller's buffer was too
    // short): handed out by the next read call, before anything else is read.
    const uint8_t* pending = nullptr;
    size_t pending_n = 0;
    bool has_pending = false;
};

namespace {

constexpr size_t kDefaultWindow = 64u << 20;

// Host-side header walk without CRC (checksum == false): same rules as the
// device walk so statuses other than BAD_CHECKSUM are identical.
}  // namespace

namespace revel {

void host_walk(const uint8_t* img, size_t n, uint64_t base, std::vector<revel_record_result>& out) {
    out.clear();
    for (size_t b = 0; b < n; b += REVEL_BLOCK_SIZE) {
        const size_t bl = std::min<size_t>(REVEL_BLOCK_SIZE, n - b);
        size_t off = 0;
        while (bl - off >= REVEL_HEADER_SIZE) {
            const uint8_t* h = img + b + off;
            revel_record_result r{};
            r.file_offset = base + b + off;
            r.length = (uint32_t)h[4] | ((uint32_t)h[5] << 8);
            r.type = h[6];
            r.stored_crc = (uint32_t)h[0] | ((uint32_t)h[1] << 8) | ((uint32_t)h[2] << 16) | ((uint32_t)h[3] << 24);
            r.computed_crc = 0;
            bool stop = false;
            if (REVEL_HEADER_SIZE + r.length > bl - off) {
                r.status = REVEL_REC_BAD_LENGTH;
                stop = true;
            } else if (r.type == 0 && r.length == 0) {
                r.status = REVEL_REC_ZERO;
                stop = true;
            } else {
                r.status = REVEL_REC_OK;
            }
            out.push_back(r);
            if (stop) break;
            off += REVEL_HEADER_SIZE + r.length;
        }
    }
}

}  // namespace revel

namespace {

int gpu_verify_window(revel_log_reader* r) {
    revel_gpu_context* g = r->gpu;
    void* st = revel_gpu_context_stream(g);
    const size_t nblocks = (r->win_len + REVEL_BLOCK_SIZE - 1) / REVEL_BLOCK_SIZE;
    int rc = revel_gpu_memcpy_h2d(g, r->d_win, r->win, r->win_len, st);
    if (!rc) rc = revel_gpu_count_scan_records(g, r->d_win, r->win_len, r->d_counts, r->d_first, st);
    uint32_t tail[2] = {0, 0};
    if (!rc) rc = revel_gpu_memcpy_d2h(g, &tail[0], r->d_first + (nblocks - 1), 4, st);
    if (!rc) rc = revel_gpu_memcpy_d2h(g, &tail[1], r->d_counts + (nblocks - 1), 4, st);
    if (!rc) rc = revel_gpu_stream_synchronize(g, st);
    if (rc) return rc;
    const size_t total = (size_t)tail[0] + tail[1];
    r->recs.clear();
    if (total == 0) return REVEL_OK;  // e.g. only a truncated header at the end of the file
    if (total > r->d_out_cap) {
        if (r->d_out) revel_gpu_free(g, r->d_out);
        r->d_out = nullptr;
        size_t cap = std::max(total, r->d_out_cap * 2);
        rc = revel_gpu_malloc(g, cap * sizeof(revel_record_result), reinterpret_cast<void**>(&r->d_out));
        if (rc) return rc;
        r->d_out_cap = cap;
    }
    r->recs.resize(total);
    rc = revel_gpu_verify_records(g, r->d_win, r->win_len, r->win_file_off, r->d_first, r->d_out, st);
    if (!rc) rc = revel_gpu_memcpy_d2h(g, r->recs.data(), r->d_out, total * sizeof(revel_record_result), st);
    if (!rc) rc = revel_gpu_stream_synchronize(g, st);
    return rc;
}

// Load the next window; returns REVEL_OK with r->recs possibly empty at EOF.
int load_window(revel_log_reader* r) {
    r->recs.clear();
    r->rec_i = 0;
    r->win_len = 0;
    if (r->file_eof) return REVEL_OK;
    size_t got = 0;
    int rc = revel_sequential_file_read(r->file, r->win, r->window, &got);
    if (rc) return rc;
    r->win_file_off = r->next_file_off;
    r->next_file_off += got;
    r->win_len = got;
    if (got < r->window) r->file_eof = true;
    if (got == 0) return REVEL_OK;
    if (r->gpu && r->checksum) return gpu_verify_window(r);
    revel::host_walk(r->win, r->win_len, r->win_file_off, r->recs);
    return REVEL_OK;
}

// Device + pinned bytes a parked reader may keep on its context: the window
// twice (pinned + device) plus results up to twice the window's bytes.
bool parkable(const revel_log_reader* r) {
    return r->d_out_cap * sizeof(revel_record_result) <= 2 * r->window;
}

void free_parked(revel_gpu_context* g) {
    auto& pr = g->parked_reader;
    if (pr.h_win) revel_gpu_host_free(g, pr.h_win);
    revel_gpu_free(g, pr.d_win);
    revel_gpu_free(g, pr.d_counts);
    revel_gpu_free(g, pr.d_first);
    revel_gpu_free(g, pr.d_out);
    pr = revel_gpu_context::ParkedReader{};
}

void reader_release(revel_log_reader* r) {
    revel_gpu_context* g = r->gpu;
    if (g && r->win && r->d_win && r->d_counts && r->d_first && parkable(r)) {
        bool closing;
        {
            std::lock_guard<std::mutex> lk(g->life_mu);
            closing = g->free_requested;
        }
        if (!closing) {  // park the window buffers for the next reader on this context
            free_parked(g);  // the newest window size wins the slot
            auto& pr = g->parked_reader;
            pr.window = r->window;
            pr.h_win = r->win;
            pr.d_win = r->d_win;
            pr.d_counts = r->d_counts;
            pr.d_first = r->d_first;
            pr.d_out = r->d_out;
            pr.d_out_cap = r->d_out_cap;
            r->win = nullptr;
            r->d_win = nullptr;
            r->d_counts = r->d_first = nullptr;
            r->d_out = nullptr;
            r->d_out_cap = 0;
        }
    }
    if (g) {
        if (r->win) revel_gpu_host_free(g, r->win);
        revel_gpu_free(g, r->d_win);
        revel_gpu_free(g, r->d_counts);
        revel_gpu_free(g, r->d_first);
        revel_gpu_free(g, r->d_out);
        r->gpu = nullptr;
        revel::context_unpin(g);  // may destroy a context freed while this reader lived
    }
    revel_sequential_file_free(r->file);
}

}  // namespace

extern "C" {

int revel_log_reader_new(revel_sequential_file* file, int checksum, uint64_t initial_offset, revel_gpu_context* gpu,
                         size_t window_bytes, revel_log_reader** out) {
    // the reader owns `file` from here on, also when construction fails
    // (Reader::new consumes its Box<dyn SequentialFile>, log_reader.rs:62)
    if (!out) {
        revel_sequential_file_free(file);
        return set_error(REVEL_INVALID_ARGUMENT, "null out");
    }
    *out = nullptr;
    if (!file) return set_error(REVEL_INVALID_ARGUMENT, "null file");
    if (checksum && !gpu) {
        // Reader::new(file, checksum, initial_offset): verify on the calling
        // thread's default context (current HIP device); no CPU fallback.
        int rc = revel::default_context(&gpu);
        if (rc) {
            revel_sequential_file_free(file);
            return rc;
        }
    }
    if (gpu) revel::context_pin(gpu);
    auto* r = new revel_log_reader;
    r->file = file;
    r->checksum = checksum != 0;
    r->initial_offset = initial_offset;
    r->gpu = gpu;
    size_t w = window_bytes ? window_bytes : kDefaultWindow;
    r->window = (w + REVEL_BLOCK_SIZE - 1) / REVEL_BLOCK_SIZE * REVEL_BLOCK_SIZE;
    const size_t nblocks = r->window / REVEL_BLOCK_SIZE;
    int rc = REVEL_OK;
    if (gpu && gpu->parked_reader.h_win && gpu->parked_reader.window == r->window) {
        auto& pr = gpu->parked_reader;  // the previous reader's buffers (same window)
        r->win = pr.h_win;
        r->d_win = pr.d_win;
        r->d_counts = pr.d_counts;
        r->d_first = pr.d_first;
        r->d_out = pr.d_out;
        r->d_out_cap = pr.d_out_cap;
        pr = revel_gpu_context::ParkedReader{};
    } else if (gpu) {
        rc = revel_gpu_host_alloc(gpu, r->window, reinterpret_cast<void**>(&r->win));
        if (!rc) rc = revel_gpu_malloc(gpu, r->window, &r->d_win);
        if (!rc) rc = revel_gpu_malloc(gpu, nblocks * 4, reinterpret_cast<void**>(&r->d_counts));
        if (!rc) rc = revel_gpu_malloc(gpu, nblocks * 4, reinterpret_cast<void**>(&r->d_first));
    } else {
        r->win_heap.resize(r->window);
        r->win = r->win_heap.data();
    }
    // SkipToInitialBlock (LevelDB semantics; the reference leaves it todo!(),
    // log_reader.rs:77): start at the block holding initial_offset, unless only
    // a trailer remains in it.
    if (!rc && initial_offset > 0) {
        uint64_t in_block = initial_offset % REVEL_BLOCK_SIZE;
        uint64_t block_start = initial_offset - in_block;
        if (in_block > REVEL_BLOCK_SIZE - 6) block_start += REVEL_BLOCK_SIZE;
        if (block_start > 0) rc = revel_sequential_file_skip(file, block_start);
        r->next_file_off = block_start;
        r->resyncing = true;
    }
    if (rc) {
        reader_release(r);
        delete r;
        return rc;
    }
    *out = r;
    return REVEL_OK;
}

}  // extern "C"

namespace {

// Where the bytes of a logical record are assembled: the caller's buffer
// (read_record_into) while they fit, else the reader's scratch (read_record:
// cap 0, always the scratch).  A FULL record is not assembled: its payload is
// handed out where it lies in the window.
struct Assembly {
    uint8_t* buf;
    size_t cap;
    size_t len = 0;
    bool in_buf = true;

    void reset(revel_log_reader* r) {
        len = 0;
        in_buf = true;
        r->scratch.clear();
    }
    void add(revel_log_reader* r, const uint8_t* p, size_t n) {
        if (in_buf && len + n <= cap) {
            memcpy(buf + len, p, n);
        } else {
            if (in_buf) r->scratch.assign(buf, buf + len);  // spill what the caller's buffer holds
            in_buf = false;
            r->scratch.insert(r->scratch.end(), p, p + n);
        }
        len += n;
    }
};

// log_reader.rs:76-153 (LevelDB-correct): the next logical record.  Returns
// REVEL_OK with *eof set at the end of the file; otherwise the record is
// either assembled in a.buf (*where == nullptr, a.len bytes) or lies at
// *where (window or scratch, *where_n bytes).
int next_logical(revel_log_reader* r, Assembly& a, const uint8_t** where, size_t* where_n, bool* eof) {
    *where = nullptr;
    *where_n = 0;
    *eof = false;
    a.reset(r);
    bool in_fragmented = false;
    uint64_t prospective = 0;
    for (;;) {
        if (r->rec_i >= r->recs.size()) {
            if (r->file_eof && r->rec_i >= r->recs.size() && r->win_len == 0) {  // EOF
                *eof = true;
                return REVEL_OK;
            }
            int rc = load_window(r);
            if (rc) return rc;
            if (r->recs.empty()) {
                // EOF: a partial fragmented record is dropped (log_reader.rs:133-141)
                a.reset(r);
                *eof = true;
                return REVEL_OK;
            }
            continue;
        }
        const revel_record_result rec = r->recs[r->rec_i++];
        if (rec.status == REVEL_REC_BAD_LENGTH) {
            // A record cut by the end of the file is a torn final write: EOF
            // (log_reader.rs:190-193 returns kEof).  Inside the file it is
            // corruption.
            const bool at_tail = r->file_eof && r->rec_i == r->recs.size() &&
                                 rec.file_offset + REVEL_HEADER_SIZE + rec.length > r->next_file_off;
            if (at_tail) {
                r->recs.clear();
                r->rec_i = 0;
                r->win_len = 0;
                a.reset(r);
                *eof = true;
                return REVEL_OK;
            }
            return set_error(REVEL_IO_ERROR, "bad record length at offset %llu", (unsigned long long)rec.file_offset);
        }
        if (rec.status == REVEL_REC_ZERO) {
            // log_reader.rs:195-198: kBadRecord -> Err(IOError)
            return set_error(REVEL_IO_ERROR, "zero-type record at offset %llu", (unsigned long long)rec.file_offset);
        }
        if (r->checksum && rec.status == REVEL_REC_BAD_CHECKSUM) {
            // log_reader.rs:200-206 + :142-152: checksum mismatch -> Err(IOError)
            return set_error(REVEL_IO_ERROR, "checksum mismatch at offset %llu (stored %08x computed %08x)",
                             (unsigned long long)rec.file_offset, rec.stored_crc, rec.computed_crc);
        }
        if (rec.file_offset < r->initial_offset) continue;
        if (r->resyncing) {
            if (rec.type == REVEL_MIDDLE_TYPE) continue;
            if (rec.type == REVEL_LAST_TYPE) {
                r->resyncing = false;
                continue;
            }
            r->resyncing = false;
        }
        const uint8_t* payload = r->win + (rec.file_offset - r->win_file_off) + REVEL_HEADER_SIZE;
        switch (rec.type) {
            case REVEL_FULL_TYPE:
                r->last_record_offset = rec.file_offset;
                a.reset(r);
                *where = payload;
                *where_n = rec.length;
                return REVEL_OK;
            case REVEL_FIRST_TYPE:
                in_fragmented = true;
                prospective = rec.file_offset;
                a.reset(r);
                a.add(r, payload, rec.length);
                break;
            case REVEL_MIDDLE_TYPE:
                if (in_fragmented) a.add(r, payload, rec.length);
                break;
            case REVEL_LAST_TYPE:
                if (in_fragmented) {
                    a.add(r, payload, rec.length);
                    r->last_record_offset = prospective;
                    if (!a.in_buf) {
                        *where = r->scratch.data();
                        *where_n = r->scratch.size();
                    }
                    return REVEL_OK;
                }
                break;
            default:
                // log_reader.rs:126-128: unknown type -> Err(IOError)
                return set_error(REVEL_IO_ERROR, "unknown record type %u at offset %llu", rec.type,
                                 (unsigned long long)rec.file_offset);
        }
    }
}

}  // namespace

extern "C" {

int revel_log_reader_read_record(revel_log_reader* r, const uint8_t** data, size_t* n) {
    if (!r || !data || !n) return set_error(REVEL_INVALID_ARGUMENT, "null argument");
    *data = nullptr;
    *n = 0;
    if (r->has_pending) {  // a record read_record_into could not deliver
        r->has_pending = false;
        *data = r->pending;
        *n = r->pending_n;
        return REVEL_OK;
    }
    Assembly a{nullptr, 0};  // no caller buffer: fragments go to the scratch
    const uint8_t* where;
    size_t wn;
    bool eof;
    int rc = next_logical(r, a, &where, &wn, &eof);
    if (rc || eof) return rc;
    *data = where;  // non-null: the window or the scratch
    *n = wn;
    return REVEL_OK;
}

int revel_log_reader_read_record_into(revel_log_reader* r, uint8_t* buf, size_t cap, size_t* n, int* eof) {
    if (!r || !n || (!buf && cap)) return set_error(REVEL_INVALID_ARGUMENT, "null argument");
    *n = 0;
    if (eof) *eof = 0;
    const uint8_t* where;
    size_t wn;
    if (r->has_pending) {
        where = r->pending;
        wn = r->pending_n;
    } else {
        Assembly a{buf, cap};
        bool at_eof;
        int rc = next_logical(r, a, &where, &wn, &at_eof);
        if (rc) return rc;
        if (at_eof) {
            if (eof) *eof = 1;
            return REVEL_OK;
        }
        if (!where) {  // assembled in the caller's buffer
            *n = a.len;
            return REVEL_OK;
        }
    }
    *n = wn;
    if (wn > cap) {  // keep it for the next call: the caller grows its buffer
        r->pending = where;
        r->pending_n = wn;
        r->has_pending = true;
        return set_error(REVEL_INVALID_ARGUMENT, "record of %zu bytes, buffer of %zu", wn, cap);
    }
    if (wn) memcpy(buf, where, wn);
    r->has_pending = false;
    return REVEL_OK;
}

uint64_t revel_log_reader_last_record_offset(const revel_log_reader* r) { return r ? r->last_record_offset : 0; }

void revel_log_reader_free(revel_log_reader* r) {
    if (!r) return;
    reader_release(r);
    delete r;
}

}  // extern "C"
