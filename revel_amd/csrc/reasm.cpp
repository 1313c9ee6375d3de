// reasm.cpp -- revel_gpu_reassemble: the C-ABI driver of the device replay
// reassembly kernels (classify -> two scans -> emit -> gather).  The rules
// are log_reader.rs:76-153 made LevelDB-correct.
#include <hip/hip_runtime_api.h>
#include <string.h>

#include "gpu_internal.h"
#include "revel_wal.h"

using revel::set_error;

namespace revel {

// Classify -> scans -> emit -> gather on `st`; image_end = the file offset
// where a torn final record counts as EOF (the end of the WAL, which for a
// shard of it lies past the shard).  Synchronises st before returning.
hipError_t reassemble_events(revel_gpu_context* ctx, const void* d_image, uint64_t image_base, uint64_t image_end,
                             const revel_record_result* d_phys, uint64_t n, int checksum, revel_logical_record* d_out,
                             void* d_payload, uint64_t* nlogical, uint64_t* payload_bytes, hipStream_t st) {
    *nlogical = 0;
    *payload_bytes = 0;
    if (n == 0) return hipSuccess;
    const uint64_t tiles = scan_scratch_words(n);
    DeviceScratch S(&ctx->arena);
    uint32_t *flag, *end, *idx, *t32;
    uint64_t *len, *off, *dst, *t64;
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = S.get(&flag, n);
    if (e == hipSuccess) e = S.get(&end, n);
    if (e == hipSuccess) e = S.get(&idx, n);
    if (e == hipSuccess) e = S.get(&t32, tiles);
    if (e == hipSuccess) e = S.get(&len, n);
    if (e == hipSuccess) e = S.get(&off, n);
    if (e == hipSuccess) e = S.get(&dst, n);
    if (e == hipSuccess) e = S.get(&t64, tiles);
    if (e == hipSuccess) e = reasm_classify(ctx->di, d_phys, n, image_end, checksum, flag, len, end, st);
    if (e == hipSuccess) e = exclusive_scan_u32(ctx->di, flag, idx, n, t32, st);
    if (e == hipSuccess) e = exclusive_scan_u64(ctx->di, len, off, n, t64, st);
    if (e == hipSuccess) e = hipMemsetAsync(dst, 0xFF, n * sizeof(uint64_t), st);
    if (e == hipSuccess) e = reasm_emit(ctx->di, d_phys, n, image_end, checksum, flag, idx, off, end, d_out, dst, st);
    if (e == hipSuccess) e = reasm_gather(ctx->di, d_image, image_base, d_phys, n, dst, d_payload, st);
    uint32_t last_idx = 0, last_flag = 0;
    uint64_t last_off = 0, last_len = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&last_idx, idx + n - 1, 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(&last_flag, flag + n - 1, 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(&last_off, off + n - 1, 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(&last_len, len + n - 1, 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        (void)hipStreamSynchronize(st);  // the context's scratch is free before the next call
        return e;
    }
    *nlogical = (uint64_t)last_idx + last_flag;
    *payload_bytes = last_off + last_len;
    return hipSuccess;
}

}  // namespace revel

extern "C" int revel_gpu_reassemble(revel_gpu_context* ctx, const void* d_image, uint64_t image_base,
                                    uint64_t image_len, const revel_record_result* d_phys, size_t nphys, int checksum,
                                    revel_logical_record* d_out, void* d_payload, uint64_t* nlogical,
                                    uint64_t* payload_bytes, void* stream) {
    if (!ctx || !nlogical || !payload_bytes) return set_error(REVEL_INVALID_ARGUMENT, "null argument");
    *nlogical = 0;
    *payload_bytes = 0;
    if (nphys == 0) return REVEL_OK;
    if (!d_image || !d_phys || !d_out || !d_payload) return set_error(REVEL_INVALID_ARGUMENT, "null device buffer");
    revel::DeviceGuard guard(ctx->di.device);
    if (guard.err() != hipSuccess) return set_error(REVEL_IO_ERROR, "hipSetDevice failed");
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    hipError_t e = revel::reassemble_events(ctx, d_image, image_base, image_base + image_len, d_phys, nphys, checksum,
                                            d_out, d_payload, nlogical, payload_bytes, st);
    if (e != hipSuccess) return set_error(REVEL_IO_ERROR, "reassemble: %s", hipGetErrorString(e));
    return REVEL_OK;
}
