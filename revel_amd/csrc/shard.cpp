// shard.cpp -- one WAL across several GPUs (config C5 on N GPUs, SURVEY 8(e);
// include/revel_wal.h "one WAL across several GPUs").
//
// A shard is a contiguous block-aligned byte range of the WAL.  Its bytes are
// streamed into HBM through a ring of pinned windows (host fill threads ->
// H2D on a copy stream -> per-window record count on the context stream as
// each window lands), then every physical record is verified in one pass over
// the resident shard (k_verify_rows / dense / partial, as revel_gpu_verify_
// records) and, with REVEL_SHARD_READ, reassembled into logical records on the
// device (revel_gpu_reassemble's kernels with the torn-tail rule at the end of
// the WAL, not of the shard).
//
// Physical records never cross a block (log_writer.rs:66-76), so every
// shard-local verdict is exact.  Reassembly differs from a whole-file read
// only at the shard's edges: the reader's state entering the shard matters
// only for the leading run of MIDDLE/LAST records (up to the first LAST, or
// the first record that resets it -- FULL, FIRST or an error), and an open
// FIRST MIDDLE* run at the end continues into the next shard.  Both runs are
// kept on the host (the boundary); the stitch folds them in file order with
// log_reader.rs:95-129's rules (LevelDB-correct, as oracle LogReader):
// a carried fragment is extended by MIDDLEs, completed by a LAST, dropped by a
// reset or by the end of the WAL.
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "gpu_internal.h"
#include "host_io.h"
#include "revel_wal.h"

using revel::set_error;

namespace {

constexpr uint32_t kBlobMagic = 0x42535652u;  // "RVSB"
constexpr uint32_t kBlobVersion = 1;
enum HeadTerm : int32_t { HEAD_NONE = 0, HEAD_LAST = 1, HEAD_RESET = 2 };

struct BlobHeader {
    uint32_t magic, version;
    uint64_t offset, length, file_bytes;
    uint64_t physical, bad, events, records, payload_bytes;
    int32_t checksum, flags, head_term, reserved;
    uint64_t nhead, ntail, head_bytes, tail_bytes;
};

// A shard's boundary: the leading MIDDLE* [LAST] run and how it ends, the open
// FIRST MIDDLE* tail, and (READ) their payloads concatenated in record order.
struct Boundary {
    BlobHeader h{};
    std::vector<revel_record_result> head, tail;
    std::vector<uint8_t> head_bytes, tail_bytes;
};

// The reader's view of one physical record (k_reasm.hip reasm_is_error).
bool is_torn(const revel_record_result& r, uint64_t file_bytes, bool last) {
    return last && r.status == REVEL_REC_BAD_LENGTH && r.file_offset + REVEL_HEADER_SIZE + r.length > file_bytes;
}
bool is_error(const revel_record_result& r, bool checksum, bool torn) {
    if (r.status == REVEL_REC_ZERO) return true;
    if (r.status == REVEL_REC_BAD_LENGTH) return !torn;
    if (checksum && r.status == REVEL_REC_BAD_CHECKSUM) return true;
    return r.type < REVEL_FULL_TYPE || r.type > REVEL_LAST_TYPE;
}
bool valid_of_type(const revel_record_result& r, bool checksum, bool torn, uint8_t type) {
    return !torn && !is_error(r, checksum, torn) && r.type == type;
}

#define TRY(expr, what)                                                                                  \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess) return set_error(REVEL_IO_ERROR, "%s: %s", what, hipGetErrorString(e_));   \
    } while (0)

}  // namespace

struct revel_wal_shard {
    revel_gpu_context* ctx = nullptr;
    Boundary b;
    revel_wal_shard_info info{};
    void* d_image = nullptr;
    uint32_t* d_counts = nullptr;
    uint32_t* d_first = nullptr;
    uint64_t* d_hlist = nullptr;
    uint32_t* d_scan = nullptr;
    uint64_t* d_sum = nullptr;
    revel_record_result* d_phys = nullptr;
    revel_logical_record* d_events = nullptr;
    void* d_payload = nullptr;

    ~revel_wal_shard() {
        if (!ctx) return;
        revel::DeviceGuard guard(ctx->di.device);
        for (void* p : {d_image, (void*)d_counts, (void*)d_first, (void*)d_hlist, (void*)d_scan, (void*)d_sum,
                        (void*)d_phys, (void*)d_events, d_payload})
            if (p) (void)hipFree(p);
        revel::context_unpin(ctx);
    }
};

namespace {

// The context's cached pinned ring for a load with `window`-byte windows:
// (re)allocated when the window size changes; every slot's pending H2D is
// waited for when the load ends, successful or not.
int ring_for(revel_gpu_context* ctx, size_t window) {
    auto& R = ctx->shard_ring;
    if (R.copy && R.window == window) return REVEL_OK;
    revel::free_shard_ring(ctx);
    TRY(hipStreamCreateWithFlags(&R.copy, hipStreamNonBlocking), "hipStreamCreate(copy)");
    for (int i = 0; i < revel_gpu_context::ShardRing::kSlots; ++i) {
        TRY(hipHostMalloc(reinterpret_cast<void**>(&R.h[i]), window, hipHostMallocDefault), "hipHostMalloc(window)");
        TRY(hipEventCreate(&R.e0[i]), "hipEventCreate");
        TRY(hipEventCreate(&R.e1[i]), "hipEventCreate");
    }
    R.window = window;
    return REVEL_OK;
}

struct RingDrain {
    revel_gpu_context::ShardRing& R;
    bool used[revel_gpu_context::ShardRing::kSlots] = {};
    ~RingDrain() {
        for (int i = 0; i < revel_gpu_context::ShardRing::kSlots; ++i)
            if (used[i]) (void)hipEventSynchronize(R.e1[i]);
    }
};

// Where a shard's last record counts as a torn final write: only at the end of
// the WAL (a garbage length in an earlier shard is corruption, not EOF).
uint64_t torn_end(uint64_t offset, uint64_t length, uint64_t file_bytes) {
    return offset + length == file_bytes ? file_bytes : UINT64_MAX;
}

int fetch_records(revel_wal_shard* s, uint64_t i0, uint64_t n, std::vector<revel_record_result>& out) {
    out.resize(n);
    if (n) TRY(hipMemcpy(out.data(), s->d_phys + i0, n * sizeof(revel_record_result), hipMemcpyDeviceToHost),
               "hipMemcpy(records)");
    return REVEL_OK;
}

// Payload bytes of `recs` (all inside the shard) concatenated, from HBM.
int fetch_payloads(revel_wal_shard* s, const std::vector<revel_record_result>& recs, std::vector<uint8_t>& out) {
    uint64_t total = 0;
    for (const auto& r : recs) total += r.length;
    out.resize(total);
    uint64_t at = 0;
    for (const auto& r : recs) {
        const uint64_t src = r.file_offset - s->info.offset + REVEL_HEADER_SIZE;
        if (r.length)
            TRY(hipMemcpyAsync(out.data() + at, static_cast<const uint8_t*>(s->d_image) + src, r.length,
                               hipMemcpyDeviceToHost, s->ctx->stream),
                "hipMemcpyAsync(boundary payload)");
        at += r.length;
    }
    TRY(hipStreamSynchronize(s->ctx->stream), "hipStreamSynchronize");
    return REVEL_OK;
}

// The leading MIDDLE* [LAST] run and the open FIRST MIDDLE* tail of n
// physical records; fetch(i0, m, buf) reads records [i0, i0 + m), pay(recs,
// bytes) their payloads (READ only).
// fb = the torn-tail end: the WAL's size for its final shard, UINT64_MAX for
// the others (only the WAL's last record can be torn).
template <typename Fetch, typename Pay>
int boundary_scan(Boundary& B, uint64_t n, uint64_t fb, bool ck, Fetch&& fetch, Pay&& pay) {
    constexpr uint64_t kChunk = 256;
    std::vector<revel_record_result> buf;
    B.h.head_term = HEAD_NONE;
    int rc;
    for (uint64_t i = 0; i < n && B.h.head_term == HEAD_NONE; i += kChunk) {
        const uint64_t m = std::min(kChunk, n - i);
        if ((rc = fetch(i, m, buf))) return rc;
        for (uint64_t k = 0; k < m; ++k) {
            const revel_record_result& r = buf[k];
            const bool torn = is_torn(r, fb, i + k == n - 1);
            if (valid_of_type(r, ck, torn, REVEL_MIDDLE_TYPE)) {
                B.head.push_back(r);
            } else if (valid_of_type(r, ck, torn, REVEL_LAST_TYPE)) {
                B.head.push_back(r);
                B.h.head_term = HEAD_LAST;
                break;
            } else {
                B.h.head_term = HEAD_RESET;
                break;
            }
        }
    }
    if (B.h.head_term != HEAD_NONE) {  // a shard of MIDDLEs only has no tail of its own
        std::vector<revel_record_result> rev;
        bool open = false, stop = false;
        for (uint64_t j = n; j > 0 && !stop;) {
            const uint64_t i0 = j > kChunk ? j - kChunk : 0;
            if ((rc = fetch(i0, j - i0, buf))) return rc;
            for (uint64_t k = j - i0; k-- > 0;) {
                const revel_record_result& r = buf[k];
                const bool torn = is_torn(r, fb, i0 + k == n - 1);
                if (valid_of_type(r, ck, torn, REVEL_MIDDLE_TYPE)) {
                    rev.push_back(r);
                    continue;
                }
                if (valid_of_type(r, ck, torn, REVEL_FIRST_TYPE)) {
                    rev.push_back(r);
                    open = true;
                }
                stop = true;
                break;
            }
            j = i0;
        }
        if (open) B.tail.assign(rev.rbegin(), rev.rend());
    }
    if (B.h.flags & REVEL_SHARD_READ) {
        if ((rc = pay(B.head, B.head_bytes))) return rc;
        if ((rc = pay(B.tail, B.tail_bytes))) return rc;
    }
    B.h.nhead = B.head.size();
    B.h.ntail = B.tail.size();
    B.h.head_bytes = B.head_bytes.size();
    B.h.tail_bytes = B.tail_bytes.size();
    return REVEL_OK;
}

int find_boundary(revel_wal_shard* s) {
    return boundary_scan(
        s->b, s->info.physical, torn_end(s->info.offset, s->info.length, s->info.file_bytes), s->info.checksum != 0,
        [&](uint64_t i0, uint64_t m, std::vector<revel_record_result>& buf) { return fetch_records(s, i0, m, buf); },
        [&](const std::vector<revel_record_result>& recs, std::vector<uint8_t>& out) {
            return fetch_payloads(s, recs, out);
        });
}

size_t blob_size(const Boundary& B) {
    return sizeof(BlobHeader) + (B.head.size() + B.tail.size()) * sizeof(revel_record_result) + B.head_bytes.size() +
           B.tail_bytes.size();
}

void blob_write(const Boundary& B, uint8_t* q) {
    const size_t rs = sizeof(revel_record_result);
    memcpy(q, &B.h, sizeof B.h);
    q += sizeof B.h;
    if (!B.head.empty()) memcpy(q, B.head.data(), B.head.size() * rs);
    q += B.head.size() * rs;
    if (!B.tail.empty()) memcpy(q, B.tail.data(), B.tail.size() * rs);
    q += B.tail.size() * rs;
    if (!B.head_bytes.empty()) memcpy(q, B.head_bytes.data(), B.head_bytes.size());
    q += B.head_bytes.size();
    if (!B.tail_bytes.empty()) memcpy(q, B.tail_bytes.data(), B.tail_bytes.size());
}

// Load + verify (+ reassemble) shard bytes src[0, length) = WAL [offset, +length).
// release_src: src is the library's own mapping of the WAL file, whose
// consumed windows the fill threads release (host_io.h release_mapped).
int shard_load(revel_wal_shard* s, const uint8_t* src, size_t window_bytes, int io_threads, bool release_src) {
    revel_gpu_context* ctx = s->ctx;
    revel_wal_shard_info& I = s->info;
    revel::DeviceGuard guard(ctx->di.device);
    TRY(guard.err(), "hipSetDevice");
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t length = I.length;
    const uint64_t nblocks = (length + REVEL_BLOCK_SIZE - 1) / REVEL_BLOCK_SIZE;
    const int flags = s->b.h.flags;
    hipStream_t comp = ctx->stream;
    if (length) {
        revel::NodeBinding near_gpu(ctx->di.device);  // pinned ring + fill threads on the GPU's node
        TRY(hipMalloc(&s->d_image, length), "hipMalloc(shard image)");
        TRY(hipMalloc(reinterpret_cast<void**>(&s->d_counts), nblocks * 4), "hipMalloc(counts)");
        TRY(hipMalloc(reinterpret_cast<void**>(&s->d_first), nblocks * 4), "hipMalloc(first)");
        TRY(hipMalloc(reinterpret_cast<void**>(&s->d_hlist), revel::hlist_words(nblocks) * 8), "hipMalloc(hlist)");
        TRY(hipMalloc(reinterpret_cast<void**>(&s->d_scan), revel::scan_scratch_words(nblocks) * 4), "hipMalloc(scan)");
        TRY(hipMalloc(reinterpret_cast<void**>(&s->d_sum), 4 * sizeof(uint64_t)), "hipMalloc(summary)");
        size_t w = window_bytes ? window_bytes : (64u << 20);
        w = (w + REVEL_BLOCK_SIZE - 1) / REVEL_BLOCK_SIZE * REVEL_BLOCK_SIZE;
        w = (size_t)std::min<uint64_t>(w, nblocks * REVEL_BLOCK_SIZE);
        constexpr int nbuf = revel_gpu_context::ShardRing::kSlots;
        int rc0 = ring_for(ctx, w);
        if (rc0) return rc0;
        auto& R = ctx->shard_ring;
        RingDrain drain{R};
        const auto t_pipe = std::chrono::steady_clock::now();
        I.setup_seconds = std::chrono::duration<double>(t_pipe - t0).count();
        auto retire = [&](int slot) -> int {
            TRY(hipEventSynchronize(R.e1[slot]), "hipEventSynchronize(H2D)");
            float ms = 0;
            TRY(hipEventElapsedTime(&ms, R.e0[slot], R.e1[slot]), "hipEventElapsedTime");
            I.h2d_ms += ms;
            drain.used[slot] = false;
            return REVEL_OK;
        };
        const int threads = std::max(1, io_threads);
        uint64_t off = 0;
        for (uint64_t i = 0; off < length; ++i) {
            const int slot = (int)(i % nbuf);
            int rc;
            if (drain.used[slot] && (rc = retire(slot))) return rc;
            const uint64_t len = std::min<uint64_t>(w, length - off);
            uint8_t* h = R.h[slot];
            I.read_seconds += revel::parallel_fill(threads, len, [&](uint64_t o, uint64_t n) {
                memcpy(h + o, src + off + o, n);
                if (release_src) revel::release_mapped(src + off + o, n);
            });
            TRY(hipEventRecord(R.e0[slot], R.copy), "hipEventRecord");
            TRY(hipMemcpyAsync(static_cast<uint8_t*>(s->d_image) + off, h, len, hipMemcpyHostToDevice, R.copy),
                "hipMemcpyAsync(H2D)");
            TRY(hipEventRecord(R.e1[slot], R.copy), "hipEventRecord");
            drain.used[slot] = true;
            TRY(hipStreamWaitEvent(comp, R.e1[slot], 0), "hipStreamWaitEvent");
            const uint64_t b0 = off / REVEL_BLOCK_SIZE;
            TRY(revel::count_records(ctx->di, static_cast<uint8_t*>(s->d_image) + off, len, s->d_counts + b0,
                                     s->d_hlist + b0 * revel::kListStride, comp),
                "count_records");
            off += len;
        }
        for (int slot = 0; slot < nbuf; ++slot) {
            int rc;
            if (drain.used[slot] && (rc = retire(slot))) return rc;
        }
        hipEvent_t k0 = nullptr, k1 = nullptr;
        TRY(hipEventCreate(&k0), "hipEventCreate");
        TRY(hipEventCreate(&k1), "hipEventCreate");
        struct EvFree {
            hipEvent_t a, b;
            ~EvFree() {
                (void)hipEventDestroy(a);
                (void)hipEventDestroy(b);
            }
        } evfree{k0, k1};
        TRY(revel::exclusive_scan_u32(ctx->di, s->d_counts, s->d_first, nblocks, s->d_scan, comp), "scan");
        if (nblocks > revel::kNoWrapBlocks) {  // record indices are u32: a shard of 2^32 records or more is refused
            uint64_t total = 0;
            TRY(revel::total_records(ctx->di, s->d_counts, nblocks, reinterpret_cast<unsigned long long*>(s->d_sum),
                                     &total, comp),
                "total_records");
            if (total > 0xFFFFFFFFull)
                return set_error(REVEL_INVALID_ARGUMENT,
                                 "shard of %llu blocks holds %llu physical records: record indices are u32, load at "
                                 "most 4294967295 records per shard (use more shards)",
                                 (unsigned long long)nblocks, (unsigned long long)total);
        }
        uint32_t tail[2] = {0, 0};
        TRY(hipMemcpyAsync(&tail[0], s->d_first + nblocks - 1, 4, hipMemcpyDeviceToHost, comp), "hipMemcpyAsync");
        TRY(hipMemcpyAsync(&tail[1], s->d_counts + nblocks - 1, 4, hipMemcpyDeviceToHost, comp), "hipMemcpyAsync");
        TRY(hipStreamSynchronize(comp), "hipStreamSynchronize");
        I.physical = (uint64_t)tail[0] + tail[1];
        TRY(hipMalloc(reinterpret_cast<void**>(&s->d_phys), std::max<uint64_t>(1, I.physical) * sizeof(revel_record_result)),
            "hipMalloc(records)");
        TRY(hipEventRecord(k0, comp), "hipEventRecord");
        if (I.physical) {
            TRY(revel::verify_records(ctx->di, s->d_image, length, I.offset, s->d_first, s->d_phys, s->d_hlist,
                                      s->d_counts, comp),
                "verify_records");
        }
        TRY(hipMemsetAsync(s->d_sum, 0, 2 * sizeof(uint64_t), comp), "hipMemsetAsync");
        TRY(hipMemsetAsync(s->d_sum + 2, 0xFF, sizeof(uint64_t), comp), "hipMemsetAsync");
        TRY(hipMemsetAsync(s->d_sum + 3, 0, sizeof(uint64_t), comp), "hipMemsetAsync");
        TRY(revel::summarize_records(ctx->di, s->d_phys, s->d_first, s->d_counts, nblocks, s->d_sum, comp),
            "summarize_records");
        if ((flags & REVEL_SHARD_READ) && I.physical) {
            TRY(hipMalloc(reinterpret_cast<void**>(&s->d_events), I.physical * sizeof(revel_logical_record)),
                "hipMalloc(events)");
            TRY(hipMalloc(&s->d_payload, length), "hipMalloc(payload)");
            TRY(revel::reassemble_events(ctx, s->d_image, I.offset, torn_end(I.offset, I.length, I.file_bytes),
                                         s->d_phys, I.physical, I.checksum,
                                         s->d_events, s->d_payload, &I.events, &I.payload_bytes, comp),
                "reassemble");
            TRY(revel::count_ok_events(ctx->di, s->d_events, I.events, s->d_sum + 3, comp), "count_ok_events");
        }
        TRY(hipEventRecord(k1, comp), "hipEventRecord");
        uint64_t sum[4];
        TRY(hipMemcpyAsync(sum, s->d_sum, sizeof sum, hipMemcpyDeviceToHost, comp), "hipMemcpyAsync(summary)");
        TRY(hipStreamSynchronize(comp), "hipStreamSynchronize");
        float kms = 0;
        TRY(hipEventElapsedTime(&kms, k0, k1), "hipEventElapsedTime");
        I.kernel_ms = kms;
        I.bad = sum[1];
        I.records = sum[3];
        int rc = find_boundary(s);
        if (rc) return rc;
    }
    I.d_image = s->d_image;
    I.d_phys = s->d_phys;
    I.d_events = s->d_events;
    I.d_payload = s->d_payload;
    BlobHeader& H = s->b.h;
    H.offset = I.offset;
    H.length = I.length;
    H.file_bytes = I.file_bytes;
    H.physical = I.physical;
    H.bad = I.bad;
    H.events = I.events;
    H.records = I.records;
    H.payload_bytes = I.payload_bytes;
    H.checksum = I.checksum;
    I.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() - I.setup_seconds;
    return REVEL_OK;
}

int check_range(uint64_t file_bytes, uint64_t offset, uint64_t length) {
    if (offset % REVEL_BLOCK_SIZE && !(length == 0 && offset == file_bytes)) return set_error(REVEL_INVALID_ARGUMENT, "shard offset %llu not block-aligned",
                                                    (unsigned long long)offset);
    if (offset + length > file_bytes || offset + length < offset)
        return set_error(REVEL_INVALID_ARGUMENT, "shard [%llu, +%llu) past the WAL's %llu bytes",
                         (unsigned long long)offset, (unsigned long long)length, (unsigned long long)file_bytes);
    if ((offset + length) % REVEL_BLOCK_SIZE && offset + length != file_bytes)
        return set_error(REVEL_INVALID_ARGUMENT, "shard end %llu is neither block-aligned nor the end of the WAL",
                         (unsigned long long)(offset + length));
    return REVEL_OK;
}

// A read-only mapping of a WAL file (the whole file: shards index into it).
struct FileMap {
    int fd = -1;
    void* p = nullptr;
    uint64_t size = 0;
    ~FileMap() {
        if (p && size) ::munmap(p, size);
        if (fd >= 0) ::close(fd);
    }
    int open(const char* path) {
        fd = ::open(path, O_RDONLY | O_CLOEXEC);
        if (fd < 0) return set_error(errno == ENOENT ? REVEL_NOT_FOUND : REVEL_IO_ERROR, "open(%s): %s", path,
                                     strerror(errno));
        struct stat st;
        if (fstat(fd, &st) != 0) return set_error(REVEL_IO_ERROR, "fstat(%s): %s", path, strerror(errno));
        size = (uint64_t)st.st_size;
        if (size) {
            p = ::mmap(nullptr, size, PROT_READ, MAP_SHARED, fd, 0);
            if (p == MAP_FAILED) {
                p = nullptr;
                return set_error(REVEL_IO_ERROR, "mmap(%s): %s", path, strerror(errno));
            }
            (void)::madvise(p, size, MADV_SEQUENTIAL);
        }
        return REVEL_OK;
    }
};

int new_shard(revel_gpu_context* ctx, uint64_t file_bytes, uint64_t offset, uint64_t length, int checksum, int flags,
              revel_wal_shard** out) {
    *out = nullptr;
    if (!ctx) return set_error(REVEL_INVALID_ARGUMENT, "null revel_gpu_context");
    if (flags != REVEL_SHARD_VERIFY && flags != REVEL_SHARD_READ)
        return set_error(REVEL_INVALID_ARGUMENT, "bad shard flags %d", flags);
    int rc = check_range(file_bytes, offset, length);
    if (rc) return rc;
    auto* s = new revel_wal_shard;
    s->ctx = ctx;
    revel::context_pin(ctx);
    s->info.device = ctx->di.device;
    s->info.checksum = checksum ? 1 : 0;
    s->info.offset = offset;
    s->info.length = length;
    s->info.file_bytes = file_bytes;
    s->b.h.magic = kBlobMagic;
    s->b.h.version = kBlobVersion;
    s->b.h.flags = flags;
    *out = s;
    return REVEL_OK;
}

int parse_blob(const uint8_t* p, size_t n, Boundary& B) {
    if (!p || n < sizeof(BlobHeader)) return set_error(REVEL_INVALID_ARGUMENT, "shard boundary blob too small");
    memcpy(&B.h, p, sizeof B.h);
    if (B.h.magic != kBlobMagic || B.h.version != kBlobVersion)
        return set_error(REVEL_INVALID_ARGUMENT, "not a shard boundary blob");
    const uint64_t rs = sizeof(revel_record_result);
    const uint64_t need = sizeof(BlobHeader) + (B.h.nhead + B.h.ntail) * rs + B.h.head_bytes + B.h.tail_bytes;
    if (B.h.nhead > n || B.h.ntail > n || B.h.head_bytes > n || B.h.tail_bytes > n || need != n)
        return set_error(REVEL_INVALID_ARGUMENT, "shard boundary blob size mismatch");
    const uint8_t* q = p + sizeof(BlobHeader);
    B.head.resize(B.h.nhead);
    B.tail.resize(B.h.ntail);
    if (B.h.nhead) memcpy(B.head.data(), q, B.h.nhead * rs);
    q += B.h.nhead * rs;
    if (B.h.ntail) memcpy(B.tail.data(), q, B.h.ntail * rs);
    q += B.h.ntail * rs;
    B.head_bytes.assign(q, q + B.h.head_bytes);
    q += B.h.head_bytes;
    B.tail_bytes.assign(q, q + B.h.tail_bytes);
    return REVEL_OK;
}

}  // namespace

struct revel_wal_stitch {
    struct Rec {
        uint64_t file_offset = 0;
        uint64_t length = 0;
        std::vector<uint8_t> bytes;
        int before_shard = 0;
    };
    std::vector<Rec> recs;
    revel_wal_summary sum{};
};

namespace {

// Fold the boundaries in file order (log_reader.rs:95-129 across shards).
int stitch(const std::vector<const Boundary*>& bs, revel_wal_stitch* out) {
    revel_wal_summary& S = out->sum;
    S = revel_wal_summary{};
    const bool read = !bs.empty() && (bs[0]->h.flags & REVEL_SHARD_READ);
    for (size_t k = 0; k < bs.size(); ++k) {
        const BlobHeader& h = bs[k]->h;
        if (k && (h.offset != bs[k - 1]->h.offset + bs[k - 1]->h.length || h.file_bytes != bs[0]->h.file_bytes ||
                  h.checksum != bs[0]->h.checksum || h.flags != bs[0]->h.flags))
            return set_error(REVEL_INVALID_ARGUMENT, "shard %zu does not continue shard %zu of the same replay", k,
                             k - 1);
    }
    bool open = false;
    revel_wal_stitch::Rec cur;
    for (size_t k = 0; k < bs.size(); ++k) {
        const Boundary& B = *bs[k];
        S.bytes += B.h.length;
        S.physical += B.h.physical;
        S.bad += B.h.bad;
        S.records += B.h.records;
        S.errors += B.h.events - B.h.records;
        S.payload_bytes += B.h.payload_bytes;
        if (open) {
            for (const auto& r : B.head) cur.length += r.length;
            if (read) cur.bytes.insert(cur.bytes.end(), B.head_bytes.begin(), B.head_bytes.end());
            if (B.h.head_term == HEAD_LAST) {
                cur.before_shard = (int)k;
                out->recs.push_back(std::move(cur));
                cur = revel_wal_stitch::Rec{};
                open = false;
            } else if (B.h.head_term == HEAD_RESET) {
                cur = revel_wal_stitch::Rec{};  // FULL / FIRST / error: the fragment is dropped
                open = false;
            }  // HEAD_NONE: MIDDLEs only, the fragment runs on into the next shard
        }
        if (B.h.head_term != HEAD_NONE && !B.tail.empty()) {
            open = true;
            cur = revel_wal_stitch::Rec{};
            cur.file_offset = B.tail[0].file_offset;
            for (const auto& r : B.tail) cur.length += r.length;
            if (read) cur.bytes = B.tail_bytes;
        }
    }
    // an open fragment at the end of the WAL is dropped (log_reader.rs:133-141)
    S.stitched = out->recs.size();
    for (const auto& r : out->recs) {
        S.records += 1;
        S.payload_bytes += r.length;
    }
    if (!read) S.records = S.errors = 0;  // VERIFY keeps no logical view of the shards' interiors
    return REVEL_OK;
}

}  // namespace

struct revel_sharded_replay {
    std::vector<revel_wal_shard*> shards;
    revel_wal_stitch st;
    double seconds = 0;
    // revel_sharded_replay_next state
    int k = 0;
    bool pre_done = false;
    size_t next_stitch = 0;
    uint64_t ev_i = 0, ev_base = 0, pay_base = 0;
    std::vector<revel_logical_record> evs;
    std::vector<uint8_t> pay;

    ~revel_sharded_replay() {
        for (auto* s : shards) delete s;
    }
};

extern "C" {

int revel_wal_shard_ranges(uint64_t file_bytes, int n, uint64_t* offsets) {
    if (n <= 0 || !offsets) return set_error(REVEL_INVALID_ARGUMENT, "need n > 0 shards and an offsets array");
    const uint64_t nblocks = (file_bytes + REVEL_BLOCK_SIZE - 1) / REVEL_BLOCK_SIZE;
    const uint64_t per = (nblocks + n - 1) / n;
    for (int k = 0; k <= n; ++k) offsets[k] = std::min<uint64_t>(file_bytes, (uint64_t)k * per * REVEL_BLOCK_SIZE);
    return REVEL_OK;
}

int revel_gpu_wal_shard_load(revel_gpu_context* ctx, const char* path, const uint8_t* image, uint64_t file_bytes,
                             uint64_t offset, uint64_t length, int checksum, int flags, size_t window_bytes,
                             int io_threads, revel_wal_shard** out) {
    if (!out) return set_error(REVEL_INVALID_ARGUMENT, "null out");
    *out = nullptr;
    if (!path && !image && file_bytes) return set_error(REVEL_INVALID_ARGUMENT, "need a path or an image");
    FileMap fm;
    const uint8_t* src = image;
    if (path) {
        int rc = fm.open(path);
        if (rc) return rc;
        if (file_bytes == 0) file_bytes = fm.size;
        if (file_bytes > fm.size)
            return set_error(REVEL_INVALID_ARGUMENT, "file_bytes %llu > size of %s", (unsigned long long)file_bytes, path);
        src = static_cast<const uint8_t*>(fm.p);
    }
    revel_wal_shard* s = nullptr;
    int rc = new_shard(ctx, file_bytes, offset, length, checksum, flags, &s);
    if (rc) return rc;
    rc = shard_load(s, src ? src + offset : nullptr, window_bytes, io_threads, path != nullptr);
    if (rc) {
        delete s;
        return rc;
    }
    *out = s;
    return REVEL_OK;
}

int revel_wal_shard_info_get(const revel_wal_shard* s, revel_wal_shard_info* out) {
    if (!s || !out) return set_error(REVEL_INVALID_ARGUMENT, "null argument");
    *out = s->info;
    return REVEL_OK;
}

int revel_wal_shard_boundary(const revel_wal_shard* s, uint8_t* buf, size_t cap, size_t* n) {
    if (!s || !n) return set_error(REVEL_INVALID_ARGUMENT, "null argument");
    const size_t need = blob_size(s->b);
    *n = need;
    if (!buf) return REVEL_OK;
    if (cap < need) return set_error(REVEL_INVALID_ARGUMENT, "boundary blob needs %zu bytes, have %zu", need, cap);
    blob_write(s->b, buf);
    return REVEL_OK;
}

int revel_wal_shard_boundary_host(const uint8_t* image, uint64_t file_bytes, uint64_t offset, uint64_t length,
                                  int flags, uint8_t* buf, size_t cap, size_t* n) {
    if (!n || (!image && file_bytes)) return set_error(REVEL_INVALID_ARGUMENT, "null argument");
    if (flags != REVEL_SHARD_VERIFY && flags != REVEL_SHARD_READ)
        return set_error(REVEL_INVALID_ARGUMENT, "bad shard flags %d", flags);
    int rc = check_range(file_bytes, offset, length);
    if (rc) return rc;
    std::vector<revel_record_result> recs;
    revel::host_walk(image + offset, length, offset, recs);
    Boundary B;
    B.h.magic = kBlobMagic;
    B.h.version = kBlobVersion;
    B.h.flags = flags;
    B.h.checksum = 0;
    B.h.offset = offset;
    B.h.length = length;
    B.h.file_bytes = file_bytes;
    B.h.physical = recs.size();
    // the shard-local events of a reader with checksum == false (oracle
    // LogReader; k_reasm.hip's rules): entering outside a fragment, open tail dropped
    const uint64_t tend = torn_end(offset, length, file_bytes);
    bool in_frag = false;
    uint64_t acc = 0;
    for (size_t i = 0; i < recs.size(); ++i) {
        const revel_record_result& r = recs[i];
        if (r.status != REVEL_REC_OK) ++B.h.bad;
        const bool torn = is_torn(r, tend, i + 1 == recs.size());
        if (torn) break;
        if (is_error(r, false, torn)) {
            ++B.h.events;
            in_frag = false;
            continue;
        }
        if (!(flags & REVEL_SHARD_READ)) continue;
        if (r.type == REVEL_FULL_TYPE) {
            ++B.h.events;
            ++B.h.records;
            B.h.payload_bytes += r.length;
            in_frag = false;
        } else if (r.type == REVEL_FIRST_TYPE) {
            in_frag = true;
            acc = r.length;
        } else if (r.type == REVEL_MIDDLE_TYPE) {
            acc += in_frag ? r.length : 0;
        } else if (in_frag) {  // LAST
            ++B.h.events;
            ++B.h.records;
            B.h.payload_bytes += acc + r.length;
            in_frag = false;
        }
    }
    if (!(flags & REVEL_SHARD_READ)) B.h.events = 0;
    rc = boundary_scan(
        B, recs.size(), tend, false,
        [&](uint64_t i0, uint64_t m, std::vector<revel_record_result>& out) {
            out.assign(recs.begin() + i0, recs.begin() + i0 + m);
            return REVEL_OK;
        },
        [&](const std::vector<revel_record_result>& rs, std::vector<uint8_t>& out) {
            out.clear();
            for (const auto& r : rs)
                out.insert(out.end(), image + r.file_offset + REVEL_HEADER_SIZE,
                           image + r.file_offset + REVEL_HEADER_SIZE + r.length);
            return REVEL_OK;
        });
    if (rc) return rc;
    const size_t need = blob_size(B);
    *n = need;
    if (!buf) return REVEL_OK;
    if (cap < need) return set_error(REVEL_INVALID_ARGUMENT, "boundary blob needs %zu bytes, have %zu", need, cap);
    blob_write(B, buf);
    return REVEL_OK;
}

void revel_wal_shard_free(revel_wal_shard* s) { delete s; }

int revel_wal_stitch_new(const uint8_t* const* blobs, const size_t* sizes, int n, revel_wal_stitch** out) {
    if (!out) return set_error(REVEL_INVALID_ARGUMENT, "null out");
    *out = nullptr;
    if (n <= 0 || !blobs || !sizes) return set_error(REVEL_INVALID_ARGUMENT, "need n > 0 blobs");
    std::vector<Boundary> bs(n);
    std::vector<const Boundary*> ptrs(n);
    for (int k = 0; k < n; ++k) {
        int rc = parse_blob(blobs[k], sizes[k], bs[k]);
        if (rc) return rc;
        ptrs[k] = &bs[k];
    }
    auto* st = new revel_wal_stitch;
    int rc = stitch(ptrs, st);
    if (rc) {
        delete st;
        return rc;
    }
    *out = st;
    return REVEL_OK;
}

int revel_wal_stitch_summary(const revel_wal_stitch* st, revel_wal_summary* out) {
    if (!st || !out) return set_error(REVEL_INVALID_ARGUMENT, "null argument");
    *out = st->sum;
    return REVEL_OK;
}

int revel_wal_stitch_record(const revel_wal_stitch* st, size_t i, uint64_t* file_offset, const uint8_t** data,
                            uint64_t* n, int* before_shard) {
    if (!st || i >= st->recs.size()) return set_error(REVEL_INVALID_ARGUMENT, "no stitched record %zu", i);
    const auto& r = st->recs[i];
    if (file_offset) *file_offset = r.file_offset;
    if (data) *data = r.bytes.size() == r.length ? r.bytes.data() : nullptr;
    if (n) *n = r.length;
    if (before_shard) *before_shard = r.before_shard;
    return REVEL_OK;
}

void revel_wal_stitch_free(revel_wal_stitch* st) { delete st; }

int revel_gpu_replay_sharded(revel_gpu_context* const* ctxs, int n, const char* path, const uint8_t* image,
                             uint64_t file_bytes, int checksum, int flags, size_t window_bytes, int io_threads,
                             revel_sharded_replay** out) {
    if (!out) return set_error(REVEL_INVALID_ARGUMENT, "null out");
    *out = nullptr;
    if (n <= 0 || !ctxs) return set_error(REVEL_INVALID_ARGUMENT, "need n > 0 contexts");
    for (int k = 0; k < n; ++k) {
        if (!ctxs[k]) return set_error(REVEL_INVALID_ARGUMENT, "null context %d", k);
        for (int j = 0; j < k; ++j)  // a context is a single-threaded handle: one shard each
            if (ctxs[j] == ctxs[k]) return set_error(REVEL_INVALID_ARGUMENT, "context %d repeats context %d", k, j);
    }
    if (!path && !image && file_bytes) return set_error(REVEL_INVALID_ARGUMENT, "need a path or an image");
    const auto t0 = std::chrono::steady_clock::now();
    FileMap fm;
    const uint8_t* src = image;
    if (path) {
        int rc = fm.open(path);
        if (rc) return rc;
        if (file_bytes == 0) file_bytes = fm.size;
        if (file_bytes > fm.size)
            return set_error(REVEL_INVALID_ARGUMENT, "file_bytes %llu > size of %s", (unsigned long long)file_bytes, path);
        src = static_cast<const uint8_t*>(fm.p);
    }
    std::vector<uint64_t> offs(n + 1);
    revel_wal_shard_ranges(file_bytes, n, offs.data());
    auto* R = new revel_sharded_replay;
    R->shards.assign(n, nullptr);
    for (int k = 0; k < n; ++k) {
        int rc = new_shard(ctxs[k], file_bytes, offs[k], offs[k + 1] - offs[k], checksum, flags, &R->shards[k]);
        if (rc) {
            delete R;
            return rc;
        }
    }
    // one host thread per shard (each context is used by its own thread only)
    std::vector<int> rcs(n, REVEL_OK);
    std::vector<std::string> msgs(n);
    std::vector<std::thread> pool;
    for (int k = 0; k < n; ++k)
        pool.emplace_back([&, k] {
            rcs[k] = shard_load(R->shards[k], src ? src + offs[k] : nullptr, window_bytes, io_threads, path != nullptr);
            if (rcs[k]) msgs[k] = revel_last_error();
        });
    for (auto& t : pool) t.join();
    for (int k = 0; k < n; ++k)
        if (rcs[k]) {
            std::string m = msgs[k];
            delete R;
            return set_error(rcs[k], "shard %d: %s", k, m.c_str());
        }
    std::vector<const Boundary*> ptrs(n);
    for (int k = 0; k < n; ++k) ptrs[k] = &R->shards[k]->b;
    int rc = stitch(ptrs, &R->st);
    if (rc) {
        delete R;
        return rc;
    }
    R->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    R->st.sum.seconds = R->seconds;
    *out = R;
    return REVEL_OK;
}

int revel_sharded_replay_summary(const revel_sharded_replay* r, revel_wal_summary* out) {
    if (!r || !out) return set_error(REVEL_INVALID_ARGUMENT, "null argument");
    *out = r->st.sum;
    return REVEL_OK;
}

const revel_wal_shard* revel_sharded_replay_shard(const revel_sharded_replay* r, int k) {
    if (!r || k < 0 || k >= (int)r->shards.size()) return nullptr;
    return r->shards[k];
}

int revel_sharded_replay_next(revel_sharded_replay* r, const uint8_t** data, size_t* n, uint64_t* file_offset) {
    if (!r || !data || !n) return set_error(REVEL_INVALID_ARGUMENT, "null argument");
    *data = nullptr;
    *n = 0;
    static const uint8_t kEmpty = 0;  // a zero-length record is not the end
    const int nshards = (int)r->shards.size();
    if (nshards && !(r->shards[0]->b.h.flags & REVEL_SHARD_READ))
        return set_error(REVEL_INVALID_ARGUMENT, "replay was loaded without REVEL_SHARD_READ");
    for (;;) {
        if (r->k >= nshards) return REVEL_OK;
        if (!r->pre_done) {
            r->pre_done = true;
            if (r->next_stitch < r->st.recs.size() && r->st.recs[r->next_stitch].before_shard == r->k) {
                const auto& s = r->st.recs[r->next_stitch++];
                *data = s.bytes.empty() ? &kEmpty : s.bytes.data();
                *n = s.bytes.size();
                if (file_offset) *file_offset = s.file_offset;
                return REVEL_OK;
            }
        }
        revel_wal_shard* s = r->shards[r->k];
        if (r->ev_i >= s->info.events) {
            ++r->k;
            r->pre_done = false;
            r->ev_i = r->ev_base = r->pay_base = 0;
            r->evs.clear();
            r->pay.clear();
            continue;
        }
        if (r->ev_i < r->ev_base || r->ev_i >= r->ev_base + r->evs.size()) {
            // next batch of events + the payload span they cover
            revel::DeviceGuard guard(s->ctx->di.device);
            if (guard.err() != hipSuccess) return set_error(REVEL_IO_ERROR, "hipSetDevice failed");
            const uint64_t m = std::min<uint64_t>(4096, s->info.events - r->ev_i);
            r->evs.resize(m);
            TRY(hipMemcpy(r->evs.data(), s->d_events + r->ev_i, m * sizeof(revel_logical_record), hipMemcpyDeviceToHost),
                "hipMemcpy(events)");
            r->ev_base = r->ev_i;
            const auto& a = r->evs.front();
            const auto& b = r->evs.back();
            r->pay_base = a.payload_offset;
            const uint64_t span = b.payload_offset + b.length - a.payload_offset;
            r->pay.resize(span);
            if (span)
                TRY(hipMemcpy(r->pay.data(), static_cast<const uint8_t*>(s->d_payload) + a.payload_offset, span,
                              hipMemcpyDeviceToHost),
                    "hipMemcpy(payload)");
        }
        const revel_logical_record& e = r->evs[r->ev_i - r->ev_base];
        ++r->ev_i;
        if (file_offset) *file_offset = e.file_offset;
        if (e.status != REVEL_LOGICAL_OK)  // the reader's Err(IOError) (log_reader.rs:142-152); continue after it
            return set_error(REVEL_IO_ERROR, "record error %u at offset %llu", e.status,
                             (unsigned long long)e.file_offset);
        *data = e.length ? r->pay.data() + (e.payload_offset - r->pay_base) : &kEmpty;
        *n = e.length;
        return REVEL_OK;
    }
}

void revel_sharded_replay_free(revel_sharded_replay* r) { delete r; }

}  // extern "C"
