// capi_gpu.cpp -- extern "C" GPU entry points of include/revel_wal.h.
// Every call validates its context and arguments, binds the context's device
// on the calling thread and launches on the given stream (NULL = the
// context's own).  There is no CPU fallback: without a gfx950 device every
// entry point returns REVEL_NOT_SUPPORT.
#include <hip/hip_runtime_api.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "gpu_internal.h"

namespace revel {

static thread_local std::string g_last_error;

int set_error(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

}  // namespace revel

using revel::set_error;

namespace revel {

void free_shard_ring(revel_gpu_context* ctx) {
    auto& R = ctx->shard_ring;
    if (R.copy) (void)hipStreamSynchronize(R.copy);
    for (int i = 0; i < revel_gpu_context::ShardRing::kSlots; ++i) {
        if (R.h[i]) (void)hipHostFree(R.h[i]);
        if (R.e0[i]) (void)hipEventDestroy(R.e0[i]);
        if (R.e1[i]) (void)hipEventDestroy(R.e1[i]);
    }
    if (R.copy) (void)hipStreamDestroy(R.copy);
    R = revel_gpu_context::ShardRing{};
}

void destroy_context(revel_gpu_context* ctx) {
    DeviceGuard guard(ctx->di.device);
    free_shard_ring(ctx);
    if (ctx->stream) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipStreamDestroy(ctx->stream);
    }
    if (ctx->hlist) (void)hipFree(ctx->hlist);
    if (ctx->scan_scratch) (void)hipFree(ctx->scan_scratch);
    if (ctx->wsums) (void)hipFree(ctx->wsums);
    if (ctx->small_scratch) (void)hipFree(ctx->small_scratch);
    if (ctx->arena.base) (void)hipFree(ctx->arena.base);
    auto& pr = ctx->parked_reader;
    if (pr.h_win) (void)hipHostFree(pr.h_win);
    if (pr.d_win) (void)hipFree(pr.d_win);
    if (pr.d_counts) (void)hipFree(pr.d_counts);
    if (pr.d_first) (void)hipFree(pr.d_first);
    if (pr.d_out) (void)hipFree(pr.d_out);
    delete ctx;
}

void context_pin(revel_gpu_context* ctx) {
    std::lock_guard<std::mutex> lk(ctx->life_mu);
    ++ctx->readers;
}

void context_unpin(revel_gpu_context* ctx) {
    bool destroy;
    {
        std::lock_guard<std::mutex> lk(ctx->life_mu);
        destroy = --ctx->readers == 0 && ctx->free_requested;
    }
    if (destroy) destroy_context(ctx);
}

namespace {
// One default context per (thread, device), released when the thread exits
// (deferred to the last reader, like any context).
struct ThreadDefaults {
    std::vector<revel_gpu_context*> by_device;
    ~ThreadDefaults() {
        for (revel_gpu_context* c : by_device)
            if (c) revel_gpu_context_free(c);
    }
};
thread_local ThreadDefaults t_defaults;
}  // namespace

int default_context(revel_gpu_context** out) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        return set_error(REVEL_NOT_SUPPORT, "no HIP device visible: checksum verification needs a gfx950 GPU");
    }
    auto& v = t_defaults.by_device;
    if ((size_t)dev < v.size() && v[dev]) {
        *out = v[dev];
        return REVEL_OK;
    }
    int rc = revel_gpu_context_new(dev, out);
    if (rc) return rc;
    if (v.size() <= (size_t)dev) v.resize(dev + 1, nullptr);
    v[dev] = *out;
    return REVEL_OK;
}

}  // namespace revel

namespace {

int hip_fail(hipError_t e, const char* what) {
    return set_error(REVEL_IO_ERROR, "%s: %s", what, hipGetErrorString(e));
}

bool is_gfx950(int dev) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) != hipSuccess) return false;
    return strncmp(p.gcnArchName, "gfx950", 6) == 0;
}

hipStream_t pick(const revel_gpu_context* c, void* stream) {
    return stream ? static_cast<hipStream_t>(stream) : c->stream;
}

// Validates the context and binds its device for the rest of the calling
// function (restoring the caller's device on return).
#define CHECK_CTX(ctx)                                                                     \
    if (!(ctx)) return set_error(REVEL_INVALID_ARGUMENT, "null revel_gpu_context");        \
    revel::DeviceGuard device_guard_((ctx)->di.device);                                     \
    if (device_guard_.err() != hipSuccess) return hip_fail(device_guard_.err(), "hipSetDevice")

#define HIP_TRY(expr, what)                          \
    do {                                             \
        hipError_t e_ = (expr);                      \
        if (e_ != hipSuccess) return hip_fail(e_, what); \
    } while (0)

}  // namespace

extern "C" {

const char* revel_last_error(void) { return revel::g_last_error.c_str(); }

int revel_gpu_device_count(int* count) {
    if (!count) return set_error(REVEL_INVALID_ARGUMENT, "null count");
    *count = 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return REVEL_OK;
    }
    int k = 0;
    for (int d = 0; d < n; ++d) k += is_gfx950(d) ? 1 : 0;
    *count = k;
    return REVEL_OK;
}

int revel_gpu_device_pci_bus_id(int device, char* buf, size_t cap) {
    if (!buf || cap == 0) return set_error(REVEL_INVALID_ARGUMENT, "null buffer");
    buf[0] = 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
        (void)hipGetLastError();
        return set_error(REVEL_INVALID_ARGUMENT, "device %d not visible", device);
    }
    char id[64] = {0};
    HIP_TRY(hipDeviceGetPCIBusId(id, (int)sizeof id, device), "hipDeviceGetPCIBusId");
    if (strlen(id) + 1 > cap) return set_error(REVEL_INVALID_ARGUMENT, "buffer of %zu bytes < %zu", cap, strlen(id) + 1);
    memcpy(buf, id, strlen(id) + 1);
    return REVEL_OK;
}

int revel_gpu_context_new(int device, revel_gpu_context** out) {
    if (!out) return set_error(REVEL_INVALID_ARGUMENT, "null out");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        (void)hipGetLastError();
        return set_error(REVEL_NOT_SUPPORT, "no HIP device visible: the CRC engine needs a gfx950 GPU");
    }
    if (device < 0 || device >= n) return set_error(REVEL_INVALID_ARGUMENT, "device %d out of range (0..%d)", device, n - 1);
    if (!is_gfx950(device)) return set_error(REVEL_NOT_SUPPORT, "device %d is not gfx950", device);
    revel::DeviceGuard guard(device);
    if (guard.err() != hipSuccess) return hip_fail(guard.err(), "hipSetDevice");
    auto* c = new revel_gpu_context;
    c->di.device = device;
    int cu = 0;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cu > 0) c->di.num_cu = cu;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return hip_fail(e, "hipStreamCreate");
    }
    *out = c;
    return REVEL_OK;
}

void revel_gpu_context_free(revel_gpu_context* ctx) {
    if (!ctx) return;
    {
        std::lock_guard<std::mutex> lk(ctx->life_mu);
        if (ctx->readers > 0) {  // the last reader's release destroys it
            ctx->free_requested = true;
            return;
        }
    }
    revel::destroy_context(ctx);
}

int revel_gpu_context_trim(revel_gpu_context* ctx) {
    CHECK_CTX(ctx);
    // free everything, forget it, then report the first failure: a buffer is
    // never left recorded after it was freed (destroy_context would free it again)
    auto& pr = ctx->parked_reader;
    hipError_t first = hipSuccess;
    auto note = [&](hipError_t e) {
        if (first == hipSuccess) first = e;
    };
    if (pr.h_win) note(hipHostFree(pr.h_win));
    if (pr.d_win) note(hipFree(pr.d_win));
    if (pr.d_counts) note(hipFree(pr.d_counts));
    if (pr.d_first) note(hipFree(pr.d_first));
    if (pr.d_out) note(hipFree(pr.d_out));
    pr = revel_gpu_context::ParkedReader{};
    revel::free_shard_ring(ctx);
    if (first != hipSuccess) return hip_fail(first, "revel_gpu_context_trim");
    return REVEL_OK;
}

void* revel_gpu_context_stream(revel_gpu_context* ctx) { return ctx ? ctx->stream : nullptr; }

int revel_gpu_crc_full_blocks(revel_gpu_context* ctx, const void* d_blocks, size_t nblocks, uint32_t* d_masked_out,
                              uint8_t* d_ok, void* stream) {
    CHECK_CTX(ctx);
    if (nblocks == 0) return REVEL_OK;
    if (!d_blocks || !d_masked_out) return set_error(REVEL_INVALID_ARGUMENT, "null device buffer");
    HIP_TRY(revel::crc_full_blocks(ctx->di, d_blocks, nblocks, d_masked_out, d_ok, pick(ctx, stream)),
            "crc_full_blocks launch");
    return REVEL_OK;
}

int revel_gpu_frame_full_blocks(revel_gpu_context* ctx, void* d_blocks, size_t nblocks, void* stream) {
    CHECK_CTX(ctx);
    if (nblocks == 0) return REVEL_OK;
    if (!d_blocks) return set_error(REVEL_INVALID_ARGUMENT, "null device buffer");
    HIP_TRY(revel::frame_full_blocks(ctx->di, d_blocks, nblocks, pick(ctx, stream)), "frame_full_blocks launch");
    return REVEL_OK;
}

int revel_gpu_synth_full_blocks(revel_gpu_context* ctx, void* d_blocks, size_t nblocks, uint64_t seed, uint64_t first,
                                void* stream) {
    CHECK_CTX(ctx);
    if (nblocks == 0) return REVEL_OK;
    if (!d_blocks) return set_error(REVEL_INVALID_ARGUMENT, "null device buffer");
    HIP_TRY(revel::synth_full_blocks(ctx->di, d_blocks, nblocks, seed, first, pick(ctx, stream)), "synth launch");
    return REVEL_OK;
}

namespace {
// The count pass of revel_gpu_count_records / revel_gpu_count_scan_records
// (k_count_hist): counts, the header lists (ctx->hlist, for the next verify of
// this image), the records per 64 blocks (ctx->wsums, the scan's first pass)
// and the block order's histogram rows (in the block-list area after the lists).
// The context's header-list buffer, grown to nblocks (grow-only).
int ensure_hlist(revel_gpu_context* ctx, uint64_t nblocks) {
    if (nblocks > ctx->hlist_cap_blocks) {
        if (ctx->hlist) (void)hipFree(ctx->hlist);
        ctx->hlist = nullptr;
        ctx->hlist_cap_blocks = 0;
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&ctx->hlist), revel::hlist_words(nblocks) * sizeof(uint64_t)),
                "hipMalloc(header list)");
        ctx->hlist_cap_blocks = nblocks;
    }
    return REVEL_OK;
}

int count_pass(revel_gpu_context* ctx, const void* d_image, size_t nbytes, uint32_t* d_counts, hipStream_t st) {
    const uint64_t nblocks = (nbytes + REVEL_BLOCK_SIZE - 1) / REVEL_BLOCK_SIZE;
    int rc0 = ensure_hlist(ctx, nblocks);
    if (rc0) return rc0;
    const uint64_t nw = revel::count_wave_sums(nblocks);
    if (nw > ctx->wsums_cap) {
        if (ctx->wsums) (void)hipFree(ctx->wsums);
        ctx->wsums = nullptr;
        ctx->wsums_cap = 0;
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&ctx->wsums), nw * sizeof(uint32_t)), "hipMalloc(wave sums)");
        ctx->wsums_cap = nw;
    }
    HIP_TRY(revel::count_hist(ctx->di, d_image, nbytes, d_counts, ctx->hlist, ctx->wsums,
                              revel::block_list_of(ctx->hlist, nblocks), st),
            "count_records launch");
    ctx->hlist_image = d_image;
    ctx->hlist_nbytes = nbytes;
    ctx->hlist_counts = d_counts;
    ctx->hlist_list_ready = false;
    return REVEL_OK;
}

int ensure_small_scratch(revel_gpu_context* ctx) {
    if (!ctx->small_scratch)
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&ctx->small_scratch), 4 * sizeof(uint32_t)), "hipMalloc(scratch)");
    return REVEL_OK;
}

// The u32 result index (d_first) of an image that could hold 2^32 or more
// physical records: sum the counts in 64 bits and reject it (synchronises).
int check_record_index(revel_gpu_context* ctx, const uint32_t* d_counts, uint64_t nblocks, hipStream_t st) {
    if (nblocks <= revel::kNoWrapBlocks) return REVEL_OK;
    int rc = ensure_small_scratch(ctx);
    if (rc) return rc;
    uint64_t total = 0;
    HIP_TRY(revel::total_records(ctx->di, d_counts, nblocks,
                                 reinterpret_cast<unsigned long long*>(ctx->small_scratch + 2), &total, st),
            "total_records");
    if (total > 0xFFFFFFFFull) {
        // a verify of this image must not take the count pass's lists: its
        // record slots (d_first) wrapped
        ctx->hlist_image = nullptr;
        ctx->hlist_list_ready = false;
        return set_error(REVEL_INVALID_ARGUMENT,
                         "image of %llu blocks holds %llu physical records: record indices (d_first) are u32, "
                         "verify at most 4294967295 records per call (split the image at a block boundary)",
                         (unsigned long long)nblocks, (unsigned long long)total);
    }
    return REVEL_OK;
}
}  // namespace

int revel_gpu_count_records(revel_gpu_context* ctx, const void* d_image, size_t nbytes, uint32_t* d_counts,
                            void* stream) {
    CHECK_CTX(ctx);
    if (nbytes == 0) return REVEL_OK;
    if (!d_image || !d_counts) return set_error(REVEL_INVALID_ARGUMENT, "null device buffer");
    const uint64_t nblocks = (nbytes + REVEL_BLOCK_SIZE - 1) / REVEL_BLOCK_SIZE;
    hipStream_t st = pick(ctx, stream);
    int rc = count_pass(ctx, d_image, nbytes, d_counts, st);
    if (rc) return rc;
    return check_record_index(ctx, d_counts, nblocks, st);
}

int revel_gpu_count_scan_records(revel_gpu_context* ctx, const void* d_image, size_t nbytes, uint32_t* d_counts,
                                 uint32_t* d_first, void* stream) {
    CHECK_CTX(ctx);
    if (nbytes == 0) return REVEL_OK;
    if (!d_image || !d_counts || !d_first) return set_error(REVEL_INVALID_ARGUMENT, "null device buffer");
    const uint64_t nblocks = (nbytes + REVEL_BLOCK_SIZE - 1) / REVEL_BLOCK_SIZE;
    hipStream_t st = pick(ctx, stream);
    int rc = count_pass(ctx, d_image, nbytes, d_counts, st);
    if (rc) return rc;
    // one launch for the scan (first pass: the count pass's per-64-block sums)
    // and verify's block list (from the count pass's histogram rows)
    HIP_TRY(revel::scan_order(ctx->di, nbytes, d_counts, ctx->wsums, d_first, revel::block_list_of(ctx->hlist, nblocks),
                              st),
            "scan launch");
    ctx->hlist_list_ready = true;
    return check_record_index(ctx, d_counts, nblocks, st);
}

int revel_gpu_exclusive_scan_u32(revel_gpu_context* ctx, const uint32_t* d_in, uint32_t* d_out, size_t n,
                                 void* stream) {
    CHECK_CTX(ctx);
    if (n == 0) return REVEL_OK;
    if (!d_in || !d_out) return set_error(REVEL_INVALID_ARGUMENT, "null device buffer");
    const uint64_t words = revel::scan_scratch_words(n);
    if (words > ctx->scan_scratch_cap) {
        if (ctx->scan_scratch) (void)hipFree(ctx->scan_scratch);
        ctx->scan_scratch = nullptr;
        ctx->scan_scratch_cap = 0;
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&ctx->scan_scratch), words * sizeof(uint32_t)), "hipMalloc(scan)");
        ctx->scan_scratch_cap = words;
    }
    HIP_TRY(revel::exclusive_scan_u32(ctx->di, d_in, d_out, n, ctx->scan_scratch, pick(ctx, stream)), "scan launch");
    return REVEL_OK;
}

int revel_gpu_verify_records(revel_gpu_context* ctx, const void* d_image, size_t nbytes, uint64_t base_offset,
                             const uint32_t* d_first, revel_record_result* d_out, void* stream) {
    CHECK_CTX(ctx);
    if (nbytes == 0) return REVEL_OK;
    if (!d_image || !d_first || !d_out) return set_error(REVEL_INVALID_ARGUMENT, "null device buffer");
    const bool memo = ctx->hlist && ctx->hlist_image == d_image && ctx->hlist_nbytes == nbytes;
    HIP_TRY(revel::verify_records(ctx->di, d_image, nbytes, base_offset, d_first, d_out, memo ? ctx->hlist : nullptr,
                                  memo ? ctx->hlist_counts : nullptr, pick(ctx, stream),
                                  memo && ctx->hlist_list_ready),
            "verify_records launch");
    ctx->hlist_image = nullptr;  // one count pass -> one verify
    return REVEL_OK;
}

// Test hook (not in the public header): the verify paths (0 = production,
// 1 = header walk without the count pass's lists, 2 = v3 with the count
// pass's lists, 3 = the round-4 split: k_verify_rows + k_verify_records_dense2,
// which is the production split since round 4).
int revel_gpu_verify_records_path(revel_gpu_context* ctx, int path, const void* d_image, size_t nbytes,
                                  uint64_t base_offset, const uint32_t* d_first, revel_record_result* d_out,
                                  void* stream) {
    CHECK_CTX(ctx);
    if (nbytes == 0) return REVEL_OK;
    if (!d_image || !d_first || !d_out) return set_error(REVEL_INVALID_ARGUMENT, "null device buffer");
    if (path < 0 || path > 3) return set_error(REVEL_INVALID_ARGUMENT, "verify path %d", path);
    const bool memo = ctx->hlist && ctx->hlist_image == d_image && ctx->hlist_nbytes == nbytes;
    HIP_TRY(revel::verify_records_path(ctx->di, path == 3 ? 0 : path, d_image, nbytes, base_offset, d_first, d_out,
                                       memo ? ctx->hlist : nullptr, memo ? ctx->hlist_counts : nullptr, pick(ctx, stream),
                                       memo && ctx->hlist_list_ready),
            "verify_records_path launch");
    ctx->hlist_image = nullptr;
    return REVEL_OK;
}

int revel_gpu_malloc(revel_gpu_context* ctx, size_t n, void** d_ptr) {
    CHECK_CTX(ctx);
    if (!d_ptr) return set_error(REVEL_INVALID_ARGUMENT, "null out");
    *d_ptr = nullptr;
    HIP_TRY(hipMalloc(d_ptr, n ? n : 1), "hipMalloc");
    return REVEL_OK;
}

int revel_gpu_free(revel_gpu_context* ctx, void* d_ptr) {
    CHECK_CTX(ctx);
    if (d_ptr) HIP_TRY(hipFree(d_ptr), "hipFree");
    return REVEL_OK;
}

int revel_gpu_host_alloc(revel_gpu_context* ctx, size_t n, void** h) {
    CHECK_CTX(ctx);
    if (!h) return set_error(REVEL_INVALID_ARGUMENT, "null out");
    *h = nullptr;
    HIP_TRY(hipHostMalloc(h, n ? n : 1, hipHostMallocDefault), "hipHostMalloc");
    return REVEL_OK;
}

int revel_gpu_host_free(revel_gpu_context* ctx, void* h) {
    CHECK_CTX(ctx);
    if (h) HIP_TRY(hipHostFree(h), "hipHostFree");
    return REVEL_OK;
}

int revel_gpu_memcpy_h2d(revel_gpu_context* ctx, void* d_dst, const void* h_src, size_t n, void* stream) {
    CHECK_CTX(ctx);
    if (n == 0) return REVEL_OK;
    HIP_TRY(hipMemcpyAsync(d_dst, h_src, n, hipMemcpyHostToDevice, pick(ctx, stream)), "hipMemcpyAsync H2D");
    return REVEL_OK;
}

int revel_gpu_memcpy_d2h(revel_gpu_context* ctx, void* h_dst, const void* d_src, size_t n, void* stream) {
    CHECK_CTX(ctx);
    if (n == 0) return REVEL_OK;
    HIP_TRY(hipMemcpyAsync(h_dst, d_src, n, hipMemcpyDeviceToHost, pick(ctx, stream)), "hipMemcpyAsync D2H");
    return REVEL_OK;
}

int revel_gpu_memset(revel_gpu_context* ctx, void* d_dst, int value, size_t n, void* stream) {
    CHECK_CTX(ctx);
    if (n == 0) return REVEL_OK;
    HIP_TRY(hipMemsetAsync(d_dst, value, n, pick(ctx, stream)), "hipMemsetAsync");
    return REVEL_OK;
}

int revel_gpu_stream_synchronize(revel_gpu_context* ctx, void* stream) {
    CHECK_CTX(ctx);
    HIP_TRY(hipStreamSynchronize(pick(ctx, stream)), "hipStreamSynchronize");
    return REVEL_OK;
}

int revel_gpu_device_synchronize(revel_gpu_context* ctx) {
    CHECK_CTX(ctx);
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    return REVEL_OK;
}

int revel_gpu_event_new(revel_gpu_context* ctx, void** ev) {
    CHECK_CTX(ctx);
    if (!ev) return set_error(REVEL_INVALID_ARGUMENT, "null out");
    hipEvent_t e;
    HIP_TRY(hipEventCreate(&e), "hipEventCreate");
    *ev = e;
    return REVEL_OK;
}

int revel_gpu_event_record(revel_gpu_context* ctx, void* ev, void* stream) {
    CHECK_CTX(ctx);
    HIP_TRY(hipEventRecord(static_cast<hipEvent_t>(ev), pick(ctx, stream)), "hipEventRecord");
    return REVEL_OK;
}

int revel_gpu_event_elapsed_ms(revel_gpu_context* ctx, void* start, void* stop, float* ms) {
    CHECK_CTX(ctx);
    HIP_TRY(hipEventSynchronize(static_cast<hipEvent_t>(stop)), "hipEventSynchronize");
    HIP_TRY(hipEventElapsedTime(ms, static_cast<hipEvent_t>(start), static_cast<hipEvent_t>(stop)),
            "hipEventElapsedTime");
    return REVEL_OK;
}

int revel_gpu_event_free(revel_gpu_context* ctx, void* ev) {
    CHECK_CTX(ctx);
    if (ev) HIP_TRY(hipEventDestroy(static_cast<hipEvent_t>(ev)), "hipEventDestroy");
    return REVEL_OK;
}

// Test hook (not in the public header): the u32 record-index guard of
// count_records / count_scan_records / the shard loader on a caller's counts
// array (a synthetic over-limit one: no 28 GiB image needed).
int revel_debug_check_record_index(revel_gpu_context* ctx, const uint32_t* d_counts, size_t nblocks) {
    CHECK_CTX(ctx);
    return check_record_index(ctx, d_counts, nblocks, ctx->stream);
}

}  // extern "C"
