// batch.cpp -- revel_gpu_decode_batches: the C-ABI driver of the device
// WriteBatch decode (count -> scan -> emit), write_batch.rs:79-128 +
// :178-181 made LevelDB-correct.
#include <hip/hip_runtime_api.h>

#include "gpu_internal.h"
#include "revel_wal.h"

using revel::set_error;

extern "C" int revel_gpu_decode_batches(revel_gpu_context* ctx, const void* d_payload, uint64_t payload_bytes,
                                        const revel_logical_record* d_logical, size_t nlogical,
                                        revel_batch_info* d_info, revel_batch_entry* d_entries, size_t entries_cap,
                                        uint64_t* nentries, void* stream) {
    if (!ctx || !nentries) return set_error(REVEL_INVALID_ARGUMENT, "null argument");
    *nentries = 0;
    if (nlogical == 0) return REVEL_OK;
    if (!d_payload || !d_logical || !d_info || (entries_cap && !d_entries))
        return set_error(REVEL_INVALID_ARGUMENT, "null device buffer");
    revel::DeviceGuard guard(ctx->di.device);
    if (guard.err() != hipSuccess) return set_error(REVEL_IO_ERROR, "hipSetDevice failed");
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    const uint64_t n = nlogical;
    revel::DeviceScratch S(&ctx->arena);
    uint64_t *nent, *first, *tiles;
    hipError_t e = S.get(&nent, n);
    if (e == hipSuccess) e = S.get(&first, n);
    if (e == hipSuccess) e = S.get(&tiles, revel::scan_scratch_words(n));
    if (e == hipSuccess) e = revel::batch_count(ctx->di, d_payload, payload_bytes, d_logical, n, d_info, nent, st);
    if (e == hipSuccess) e = revel::exclusive_scan_u64(ctx->di, nent, first, n, tiles, st);
    if (e == hipSuccess)
        e = revel::batch_emit(ctx->di, d_payload, payload_bytes, d_logical, n, first, d_info, d_entries, entries_cap,
                              st);
    uint64_t last_first = 0, last_n = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&last_first, first + n - 1, 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(&last_n, nent + n - 1, 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        (void)hipStreamSynchronize(st);  // the context's scratch is free before the next call
        return set_error(REVEL_IO_ERROR, "decode_batches: %s", hipGetErrorString(e));
    }
    *nentries = last_first + last_n;
    if (*nentries > entries_cap)
        return set_error(REVEL_INVALID_ARGUMENT, "decode_batches: %llu entries exceed capacity %zu",
                         (unsigned long long)*nentries, entries_cap);
    return REVEL_OK;
}
