// k_reasm.hip -- device replay reassembly (log_reader.rs:76-153, LevelDB-correct):
// classify / emit / gather of logical records from the physical-record array.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <type_traits>

#include "device_common.h"

using namespace revel;

namespace {
// ---------------------------------------------------------------------------
// Device replay reassembly (log_reader.rs:76-153, LevelDB-correct; the rules
// of oracle LogReader / replay_events): physical records -> events in file
// order: RECORD (FULL, or FIRST MIDDLE* LAST all valid) or ERROR (zero record,
// length past the block that is not the torn tail of the image, checksum
// mismatch when checking, unknown type).
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool reasm_is_error(const revel_record_result& r, bool checksum, bool tail) {
    if (r.status == REVEL_REC_ZERO) return true;
    if (r.status == REVEL_REC_BAD_LENGTH) return !tail;
    if (checksum && r.status == REVEL_REC_BAD_CHECKSUM) return true;
    return r.type < REVEL_FULL_TYPE || r.type > REVEL_LAST_TYPE;
}

__global__ void k_reasm_classify(const revel_record_result* __restrict__ phys, uint64_t n, uint64_t image_end,
                                 int checksum, uint32_t* __restrict__ ev_flag, uint64_t* __restrict__ ev_len,
                                 uint32_t* __restrict__ ev_end) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const revel_record_result r = phys[i];
        auto tail_of = [&](uint64_t k, const revel_record_result& q) {
            return k == n - 1 && q.status == REVEL_REC_BAD_LENGTH && q.file_offset + kHeaderSize + q.length > image_end;
        };
        uint32_t flag = 0, end = (uint32_t)i;
        uint64_t len = 0;
        const bool tail = tail_of(i, r);
        if (reasm_is_error(r, checksum, tail)) {
            flag = 1;  // ERROR event
        } else if (!tail) {
            if (r.type == REVEL_FULL_TYPE) {
                flag = 1;
                len = r.length;
            } else if (r.type == REVEL_FIRST_TYPE) {
                uint64_t acc = r.length;
                for (uint64_t j = i + 1; j < n; ++j) {
                    const revel_record_result q = phys[j];
                    if (reasm_is_error(q, checksum, tail_of(j, q)) || tail_of(j, q)) break;
                    if (q.type == REVEL_MIDDLE_TYPE) {
                        acc += q.length;
                        continue;
                    }
                    if (q.type == REVEL_LAST_TYPE) {
                        flag = 1;
                        len = acc + q.length;
                        end = (uint32_t)j;
                    }
                    break;  // FULL / FIRST: this fragment is dropped
                }
            }
        }
        ev_flag[i] = flag;
        ev_len[i] = len;
        ev_end[i] = end;
    }
}

__global__ void k_reasm_emit(const revel_record_result* __restrict__ phys, uint64_t n, uint64_t image_end, int checksum,
                             const uint32_t* __restrict__ ev_flag, const uint32_t* __restrict__ ev_idx,
                             const uint64_t* __restrict__ pay_off, const uint32_t* __restrict__ ev_end,
                             revel_logical_record* __restrict__ out, uint64_t* __restrict__ frag_dst) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (!ev_flag[i]) continue;
        const revel_record_result r = phys[i];
        const bool tail = i == n - 1 && r.status == REVEL_REC_BAD_LENGTH &&
                          r.file_offset + kHeaderSize + r.length > image_end;
        revel_logical_record o;
        o.file_offset = r.file_offset;
        o.payload_offset = pay_off[i];
        o.first_phys = (uint32_t)i;
        o.last_phys = ev_end[i];
        o.reserved[0] = o.reserved[1] = o.reserved[2] = 0;
        if (reasm_is_error(r, checksum, tail)) {
            o.length = 0;
            o.status = r.status == REVEL_REC_OK || (!checksum && r.status == REVEL_REC_BAD_CHECKSUM)
                           ? REVEL_LOGICAL_BAD_TYPE
                           : r.status;
        } else {
            uint64_t acc = 0;
            for (uint64_t k = i; k <= ev_end[i]; ++k) {
                frag_dst[k] = pay_off[i] + acc;
                acc += phys[k].length;
            }
            o.length = (uint32_t)acc;
            o.status = REVEL_LOGICAL_OK;
        }
        out[ev_idx[i]] = o;
    }
}

// Fragments of emitted logical records, 32 per wave visit, 4 per 8-lane
// group.  Fragments of at most kTinyCopy bytes (small-record logs) are copied
// by their group with all four fragments' loads issued before any store, so a
// wave has 32 fragments' bytes in flight instead of 8 (the copy is latency-
// bound: profiles/r1s3_pmc_batches_summary.txt); fragments of at most
// kSmallFrag bytes then by their group one after another, larger ones one
// after another by the whole wave.
constexpr uint32_t kSmallFrag = 1024;
constexpr uint32_t kGatherFpg = 4;  // fragments per 8-lane group and visit
__global__ void k_reasm_gather(const uint8_t* __restrict__ image, uint64_t image_base,
                               const revel_record_result* __restrict__ phys, uint64_t n,
                               const uint64_t* __restrict__ frag_dst, uint8_t* __restrict__ payload) {
    const uint32_t lane = lane_id(), grp = lane >> 3, gl = lane & 7u;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t w0 = blockIdx.x * (uint64_t)(blockDim.x / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr uint64_t kVisit = 8u * kGatherFpg;
    // descriptors one visit ahead (fragment base + 8 j + grp of a visit: each j
    // reads 8 consecutive descriptors), clamped loads + a validity flag
    uint64_t dst_n[kGatherFpg], off_n[kGatherFpg];
    uint32_t len_n[kGatherFpg];
    auto fetch = [&](uint64_t base) {
#pragma unroll
        for (uint32_t j = 0; j < kGatherFpg; ++j) {
            const uint64_t k = base + 8u * j + grp;
            const uint64_t kc = k < n ? k : n - 1;
            const uint64_t d = frag_dst[kc];
            dst_n[j] = k < n ? d : ~0ull;
            off_n[j] = phys[kc].file_offset;
            len_n[j] = phys[kc].length;
        }
    };
    if (w0 * kVisit < n) fetch(w0 * kVisit);
    for (uint64_t base = w0 * kVisit; base < n; base += waves * kVisit) {
        uint64_t dst[kGatherFpg], src_off[kGatherFpg];
        uint32_t len[kGatherFpg];
#pragma unroll
        for (uint32_t j = 0; j < kGatherFpg; ++j) {
            dst[j] = dst_n[j];
            src_off[j] = off_n[j] - image_base + kHeaderSize;
            len[j] = len_n[j];
        }
        if (base + waves * kVisit < n) fetch(base + waves * kVisit);
        // tiny fragments: every load of the group's four, then the stores
        TinyCopy c[kGatherFpg];
#pragma unroll
        for (uint32_t j = 0; j < kGatherFpg; ++j) {
            const bool tiny = dst[j] != ~0ull && len[j] <= kTinyCopy;
            tiny_load(image + src_off[j], payload + (tiny ? dst[j] : 0u), tiny ? len[j] : 0u, gl, image, c[j]);
        }
#pragma unroll
        for (uint32_t j = 0; j < kGatherFpg; ++j)
            if (dst[j] != ~0ull && len[j] <= kTinyCopy) tiny_store(image + src_off[j], payload + dst[j], len[j], gl, c[j]);
#pragma unroll
        for (uint32_t j = 0; j < kGatherFpg; ++j) {
            const bool small = dst[j] != ~0ull && len[j] > kTinyCopy && len[j] <= kSmallFrag;
            if (small) group_copy<8>(image + src_off[j], payload + dst[j], len[j], gl);
            // large fragments: one bit per group (its lane 0), whole wave each
            uint64_t big = __ballot(dst[j] != ~0ull && len[j] > kSmallFrag && gl == 0);
            while (big) {
                const uint32_t l = (uint32_t)__builtin_ctzll(big);
                big &= big - 1;
                const uint64_t so = __shfl(src_off[j], l, 64), dd = __shfl(dst[j], l, 64);
                const uint32_t ln = __shfl(len[j], l, 64);
                group_copy<64>(image + so, payload + dd, ln, lane);
            }
        }
    }
}

// Events with status REVEL_LOGICAL_OK among n (the rest are errors): one
// atomic add per workgroup into *ok (zeroed by the caller).
__global__ __launch_bounds__(256) void k_count_ok_events(const revel_logical_record* __restrict__ ev, uint64_t n,
                                                         unsigned long long* __restrict__ ok) {
    __shared__ unsigned long long part[256];
    unsigned long long c = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        c += ev[i].status == REVEL_LOGICAL_OK ? 1u : 0u;
    part[threadIdx.x] = c;
    __syncthreads();
    for (uint32_t s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) part[threadIdx.x] += part[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0 && part[0]) atomicAdd(ok, part[0]);
}

}  // namespace

namespace revel {
hipError_t count_ok_events(const DeviceInfo& di, const revel_logical_record* d_ev, uint64_t n, uint64_t* d_ok,
                           hipStream_t st) {
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu * 4, (n + 255) / 256));
    hipLaunchKernelGGL(k_count_ok_events, dim3((uint32_t)grid), dim3(256), 0, st, d_ev, n,
                       reinterpret_cast<unsigned long long*>(d_ok));
    return hipGetLastError();
}

hipError_t reasm_classify(const DeviceInfo& di, const revel_record_result* d_phys, uint64_t n, uint64_t image_end,
                          int checksum, uint32_t* d_flag, uint64_t* d_len, uint32_t* d_end, hipStream_t st) {
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu * 8, (n + 255) / 256));
    hipLaunchKernelGGL(k_reasm_classify, dim3((uint32_t)grid), dim3(256), 0, st, d_phys, n, image_end, checksum, d_flag,
                       d_len, d_end);
    return hipGetLastError();
}

hipError_t reasm_emit(const DeviceInfo& di, const revel_record_result* d_phys, uint64_t n, uint64_t image_end,
                      int checksum, const uint32_t* d_flag, const uint32_t* d_idx, const uint64_t* d_off,
                      const uint32_t* d_end, revel_logical_record* d_out, uint64_t* d_frag_dst, hipStream_t st) {
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu * 8, (n + 255) / 256));
    hipLaunchKernelGGL(k_reasm_emit, dim3((uint32_t)grid), dim3(256), 0, st, d_phys, n, image_end, checksum, d_flag,
                       d_idx, d_off, d_end, d_out, d_frag_dst);
    return hipGetLastError();
}

hipError_t reasm_gather(const DeviceInfo& di, const void* d_image, uint64_t image_base,
                        const revel_record_result* d_phys, uint64_t n, const uint64_t* d_frag_dst, void* d_payload,
                        hipStream_t st) {
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu * 8, (n + 127) / 128));
    hipLaunchKernelGGL(k_reasm_gather, dim3((uint32_t)grid), dim3(256), 0, st, static_cast<const uint8_t*>(d_image),
                       image_base, d_phys, n, d_frag_dst, static_cast<uint8_t*>(d_payload));
    return hipGetLastError();
}

}  // namespace revel
