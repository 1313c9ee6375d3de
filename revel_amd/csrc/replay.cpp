// replay.cpp -- end-to-end WAL replay: host bytes -> pinned ring -> HBM ->
// GPU verify, PCIe-inclusive (config C5; log_reader.rs's read(2) + CRC path,
// env.rs:162-169, done in bulk).
//
// A ring of `nbuffers` windows, each = pinned host buffer + device buffer +
// per-window scratch.  For window i the host thread (1) waits until window
// i-nbuffers' verdict has come back, (2) fills the pinned buffer with
// `io_threads` parallel pread()/memcpy() calls, (3) enqueues H2D on the copy
// stream, and (4) makes the context stream wait for that copy and run the
// verify kernels + a summary kernel, then copies 24 summary bytes back.
// Reading window i+1 on the host therefore overlaps the H2D of window i and
// the verification of window i-1.
#include <ctype.h>
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "gpu_internal.h"
#include "host_io.h"
#include "revel_wal.h"

using revel::set_error;

namespace {

constexpr size_t kMaxRecordsPerBlock = REVEL_BLOCK_SIZE / REVEL_HEADER_SIZE + 1;

struct Window {
    uint8_t* h = nullptr;          // pinned host window
    void* d = nullptr;             // device window
    uint32_t* d_counts = nullptr;  // RECORDS
    uint32_t* d_first = nullptr;
    uint64_t* d_hlist = nullptr;
    uint32_t* d_scan = nullptr;
    revel_record_result* d_res = nullptr;
    uint32_t* d_masked = nullptr;  // FULL_BLOCKS
    uint8_t* d_ok = nullptr;
    uint64_t* d_sum = nullptr;
    uint64_t* h_sum = nullptr;     // pinned
    hipEvent_t e_h2d0{}, e_copied{}, e_k0{}, e_k1{}, e_done{};
    bool inflight = false;
    uint64_t len = 0;
};

struct Ring {
    revel_gpu_context* ctx;
    hipStream_t copy = nullptr;
    std::vector<Window> w;
    int mode;
    size_t window;

    ~Ring() {
        for (auto& x : w) {
            if (x.inflight) (void)hipEventSynchronize(x.e_done);
            if (x.h) (void)hipHostFree(x.h);
            if (x.h_sum) (void)hipHostFree(x.h_sum);
            for (void* p : {x.d, (void*)x.d_counts, (void*)x.d_first, (void*)x.d_hlist, (void*)x.d_scan, (void*)x.d_res,
                            (void*)x.d_masked, (void*)x.d_ok, (void*)x.d_sum})
                if (p) (void)hipFree(p);
            for (hipEvent_t e : {x.e_h2d0, x.e_copied, x.e_k0, x.e_k1, x.e_done})
                if (e) (void)hipEventDestroy(e);
        }
        if (copy) (void)hipStreamDestroy(copy);
    }
};

#define TRY(expr, what)                                                                          \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess) return set_error(REVEL_IO_ERROR, "%s: %s", what, hipGetErrorString(e_)); \
    } while (0)

int ring_init(Ring& R, int nbuf) {
    TRY(hipStreamCreateWithFlags(&R.copy, hipStreamNonBlocking), "hipStreamCreate(copy)");
    const size_t nblocks = R.window / REVEL_BLOCK_SIZE;
    R.w.resize(nbuf);
    for (auto& x : R.w) {
        TRY(hipHostMalloc(reinterpret_cast<void**>(&x.h), R.window, hipHostMallocDefault), "hipHostMalloc(window)");
        TRY(hipHostMalloc(reinterpret_cast<void**>(&x.h_sum), 4 * sizeof(uint64_t), hipHostMallocDefault),
            "hipHostMalloc(summary)");
        TRY(hipMalloc(&x.d, R.window), "hipMalloc(window)");
        TRY(hipMalloc(reinterpret_cast<void**>(&x.d_sum), 4 * sizeof(uint64_t)), "hipMalloc(summary)");
        if (R.mode == REVEL_REPLAY_RECORDS) {
            TRY(hipMalloc(reinterpret_cast<void**>(&x.d_counts), nblocks * 4), "hipMalloc(counts)");
            TRY(hipMalloc(reinterpret_cast<void**>(&x.d_first), nblocks * 4), "hipMalloc(first)");
            TRY(hipMalloc(reinterpret_cast<void**>(&x.d_hlist), revel::hlist_words(nblocks) * 8), "hipMalloc(hlist)");
            TRY(hipMalloc(reinterpret_cast<void**>(&x.d_scan), revel::scan_scratch_words(nblocks) * 4), "hipMalloc(scan)");
            TRY(hipMalloc(reinterpret_cast<void**>(&x.d_res), nblocks * kMaxRecordsPerBlock * sizeof(revel_record_result)),
                "hipMalloc(records)");
        } else {
            TRY(hipMalloc(reinterpret_cast<void**>(&x.d_masked), nblocks * 4), "hipMalloc(masked)");
            TRY(hipMalloc(reinterpret_cast<void**>(&x.d_ok), nblocks), "hipMalloc(ok)");
        }
        for (hipEvent_t* e : {&x.e_h2d0, &x.e_copied, &x.e_k0, &x.e_k1, &x.e_done})
            TRY(hipEventCreate(e), "hipEventCreate");
    }
    return REVEL_OK;
}

int tally(Window& x, revel_replay_stats* st) {
    TRY(hipEventSynchronize(x.e_done), "hipEventSynchronize");
    float h2d = 0, kms = 0;
    TRY(hipEventElapsedTime(&h2d, x.e_h2d0, x.e_copied), "hipEventElapsedTime(h2d)");
    TRY(hipEventElapsedTime(&kms, x.e_k0, x.e_k1), "hipEventElapsedTime(kernel)");
    st->h2d_ms += h2d;
    st->kernel_ms += kms;
    st->units += x.h_sum[0];
    st->bad += x.h_sum[1];
    st->first_bad_offset = std::min<uint64_t>(st->first_bad_offset, x.h_sum[2]);
    st->windows += 1;
    x.inflight = false;
    return REVEL_OK;
}

template <typename Fill>
int replay(revel_gpu_context* ctx, uint64_t length, uint64_t base_offset, int mode, size_t window_bytes, int nbuffers,
           int io_threads, revel_replay_stats* out, Fill&& fill) {
    if (!ctx || !out) return set_error(REVEL_INVALID_ARGUMENT, "null ctx/out");
    mode &= 0x0F;  // the IO flags were consumed by the caller
    if (mode != REVEL_REPLAY_RECORDS && mode != REVEL_REPLAY_FULL_BLOCKS)
        return set_error(REVEL_INVALID_ARGUMENT, "bad replay mode %d", mode);
    if (base_offset % REVEL_BLOCK_SIZE)
        return set_error(REVEL_INVALID_ARGUMENT, "replay must start on a block boundary");
    revel::DeviceGuard guard(ctx->di.device);
    TRY(guard.err(), "hipSetDevice");
    memset(out, 0, sizeof *out);
    out->first_bad_offset = UINT64_MAX;
    revel::NodeBinding near_gpu(ctx->di.device);  // before the ring: its pinned pages land on the GPU's node
    Ring R;
    R.ctx = ctx;
    R.mode = mode;
    size_t w = window_bytes ? window_bytes : (64u << 20);
    R.window = (w + REVEL_BLOCK_SIZE - 1) / REVEL_BLOCK_SIZE * REVEL_BLOCK_SIZE;
    nbuffers = std::max(2, nbuffers);
    io_threads = std::max(1, io_threads);
    int rc = ring_init(R, nbuffers);
    if (rc) return rc;
    hipStream_t comp = ctx->stream;
    auto t0 = std::chrono::steady_clock::now();
    uint64_t off = 0, nsub = 0;
    for (uint64_t i = 0; off < length; ++i, ++nsub) {
        Window& x = R.w[i % R.w.size()];
        if (x.inflight && (rc = tally(x, out))) return rc;
        x.len = std::min<uint64_t>(R.window, length - off);
        const uint8_t* h = x.h;
        out->read_seconds += revel::parallel_fill(io_threads, x.len, [&](uint64_t o, uint64_t n) {
            fill(const_cast<uint8_t*>(h) + o, off + o, n);
        });
        if (mode == REVEL_REPLAY_FULL_BLOCKS && x.len % REVEL_BLOCK_SIZE)
            return set_error(REVEL_INVALID_ARGUMENT, "FULL_BLOCKS replay needs whole blocks");
        TRY(hipEventRecord(x.e_h2d0, R.copy), "hipEventRecord");
        TRY(hipMemcpyAsync(x.d, x.h, x.len, hipMemcpyHostToDevice, R.copy), "hipMemcpyAsync(H2D)");
        TRY(hipEventRecord(x.e_copied, R.copy), "hipEventRecord");
        TRY(hipStreamWaitEvent(comp, x.e_copied, 0), "hipStreamWaitEvent");
        TRY(hipEventRecord(x.e_k0, comp), "hipEventRecord");
        TRY(hipMemsetAsync(x.d_sum, 0, 2 * sizeof(uint64_t), comp), "hipMemsetAsync");
        TRY(hipMemsetAsync(x.d_sum + 2, 0xFF, sizeof(uint64_t), comp), "hipMemsetAsync");
        const uint64_t nblocks = (x.len + REVEL_BLOCK_SIZE - 1) / REVEL_BLOCK_SIZE;
        if (mode == REVEL_REPLAY_RECORDS) {
            TRY(revel::count_records(ctx->di, x.d, x.len, x.d_counts, x.d_hlist, comp), "count_records");
            TRY(revel::exclusive_scan_u32(ctx->di, x.d_counts, x.d_first, nblocks, x.d_scan, comp), "scan");
            TRY(revel::verify_records(ctx->di, x.d, x.len, base_offset + off, x.d_first, x.d_res, x.d_hlist,
                                      x.d_counts, comp),
                "verify_records");
            TRY(revel::summarize_records(ctx->di, x.d_res, x.d_first, x.d_counts, nblocks, x.d_sum, comp),
                "summarize_records");
        } else {
            TRY(revel::crc_full_blocks(ctx->di, x.d, nblocks, x.d_masked, x.d_ok, comp), "crc_full_blocks");
            TRY(revel::summarize_blocks(ctx->di, x.d_ok, nblocks, base_offset + off, x.d_sum, comp),
                "summarize_blocks");
        }
        TRY(hipEventRecord(x.e_k1, comp), "hipEventRecord");
        TRY(hipMemcpyAsync(x.h_sum, x.d_sum, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, comp), "hipMemcpyAsync(D2H)");
        TRY(hipEventRecord(x.e_done, comp), "hipEventRecord");
        x.inflight = true;
        off += x.len;
        out->bytes += x.len;
    }
    const uint64_t nring = R.w.size();
    for (uint64_t j = nsub > nring ? nsub - nring : 0; j < nsub; ++j) {  // drain in submission order
        Window& x = R.w[j % nring];
        if (x.inflight && (rc = tally(x, out))) return rc;
    }
    out->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return REVEL_OK;
}

}  // namespace

extern "C" {

int revel_gpu_replay_file(revel_gpu_context* ctx, const char* path, uint64_t offset, uint64_t length, int mode,
                          size_t window_bytes, int nbuffers, int io_threads, revel_replay_stats* out) {
    if (!path) return set_error(REVEL_INVALID_ARGUMENT, "null path");
    const int io = mode & 0xF0;
    if (io != REVEL_REPLAY_IO_PREAD && io != REVEL_REPLAY_IO_MMAP && io != REVEL_REPLAY_IO_DIRECT)
        return set_error(REVEL_INVALID_ARGUMENT, "bad replay io flag 0x%x", io);
    int fd = ::open(path, O_RDONLY | O_CLOEXEC | (io == REVEL_REPLAY_IO_DIRECT ? O_DIRECT : 0));
    if (fd < 0 && io == REVEL_REPLAY_IO_DIRECT && errno == EINVAL)
        return set_error(REVEL_NOT_SUPPORT, "open(%s, O_DIRECT): not supported by this file system", path);
    if (fd < 0) return set_error(REVEL_NOT_FOUND, "open(%s): %s", path, strerror(errno));
    const off_t end = ::lseek(fd, 0, SEEK_END);
    if (length == 0) length = end > (off_t)offset ? (uint64_t)end - offset : 0;
    if (end < 0 || offset + length > (uint64_t)end) {
        ::close(fd);
        return set_error(REVEL_INVALID_ARGUMENT, "range [%llu, +%llu) past the end of %s", (unsigned long long)offset,
                         (unsigned long long)length, path);
    }
    std::atomic<bool> io_error{false};
    int rc;
    if (io == REVEL_REPLAY_IO_MMAP) {
        // offset is block- (hence page-) aligned; the io threads copy straight
        // from the page cache into the pinned window (no read(2) per piece)
        void* m = length ? ::mmap(nullptr, length, PROT_READ, MAP_SHARED, fd, (off_t)offset) : nullptr;
        if (m == MAP_FAILED) {
            ::close(fd);
            return set_error(REVEL_IO_ERROR, "mmap(%s): %s", path, strerror(errno));
        }
        if (m) (void)::madvise(m, length, MADV_SEQUENTIAL);
        const uint8_t* src = static_cast<const uint8_t*>(m);
        rc = replay(ctx, length, offset, mode, window_bytes, nbuffers, io_threads, out,
                    [&](uint8_t* dst, uint64_t rel, uint64_t n) {
                        memcpy(dst, src + rel, n);
                        revel::release_mapped(src + rel, n);  // the final munmap then has little to tear down
                    });
        if (m) ::munmap(m, length);
    } else {
        const uint64_t align = io == REVEL_REPLAY_IO_DIRECT ? 4096 : 1;
        rc = replay(ctx, length, offset, mode, window_bytes, nbuffers, io_threads, out,
                    [&](uint8_t* dst, uint64_t rel, uint64_t n) {
                        // O_DIRECT: pieces start page-aligned; the request is
                        // rounded up (the window has room: its size is whole
                        // blocks) and the kernel stops at end of file
                        const uint64_t want = (n + align - 1) / align * align;
                        uint64_t done = 0;
                        while (done < n) {
                            ssize_t r = ::pread(fd, dst + done, want - done, (off_t)(offset + rel + done));
                            if (r < 0 && errno == EINTR) continue;
                            if (r <= 0) {
                                memset(dst + done, 0, n - done);
                                io_error.store(true, std::memory_order_relaxed);
                                return;
                            }
                            done += (uint64_t)r;
                        }
                    });
    }
    ::close(fd);
    if (rc == REVEL_OK && io_error.load()) return set_error(REVEL_IO_ERROR, "short read from %s", path);
    return rc;
}

int revel_gpu_replay_memory(revel_gpu_context* ctx, const uint8_t* image, uint64_t length, uint64_t base_offset,
                            int mode, size_t window_bytes, int nbuffers, int io_threads, revel_replay_stats* out) {
    if (!image && length) return set_error(REVEL_INVALID_ARGUMENT, "null image");
    if (mode & 0xF0) return set_error(REVEL_INVALID_ARGUMENT, "io flags apply to revel_gpu_replay_file only");
    return replay(ctx, length, base_offset, mode, window_bytes, nbuffers, io_threads, out,
                  [&](uint8_t* dst, uint64_t rel, uint64_t n) { memcpy(dst, image + rel, n); });
}

}  // extern "C"
