// batch.hip -- device WriteBatch decode for WAL replay (gfx950).
//
// Reference: write_batch.rs:79-128 (iterate), :148-158 (MemTableInserter:
// entry i gets sequence seq + i), :178-181 (insert_into), coding.rs:96-123
// (get_varint32) and :159-166 (get_length_prefixed_slice), made
// LevelDB-correct (DESIGN.md section 4.8 lists the reference's defects).
//
// Layout: one lane per logical record.  A batch is a sequential chain (entry
// k+1 starts where entry k's value ends), so the parallelism is across
// batches; two passes (count, then emit at the scanned entry index) keep the
// output dense without atomics.  The payload reads are a few header bytes per
// entry -- keys and values are located, never copied.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "gpu_internal.h"

namespace {

__device__ __forceinline__ bool get_varint32(const uint8_t* __restrict__ p, uint64_t& pos, uint64_t limit,
                                             uint32_t& v) {
    uint32_t result = 0;
    for (uint32_t shift = 0; shift <= 28 && pos < limit; shift += 7) {
        const uint32_t b = p[pos++];
        if (b & 128u) {
            result |= (b & 127u) << shift;
        } else {
            v = result | (b << shift);
            return true;
        }
    }
    return false;
}

__device__ __forceinline__ uint64_t load_le(const uint8_t* __restrict__ p, uint32_t nbytes) {
    uint64_t v = 0;
    for (uint32_t i = 0; i < nbytes; ++i) v |= uint64_t(p[i]) << (8 * i);
    return v;
}

// Walk one rep of n bytes; with EMIT, write entry k to out[first + k] when it
// is below cap.  Returns the REVEL_BATCH_* status; found = entries decoded.
template <bool EMIT>
__device__ uint8_t walk_batch(const uint8_t* __restrict__ rep, uint64_t rep_off, uint64_t n, uint64_t seq,
                              uint32_t count, uint32_t batch, uint32_t& found, revel_batch_entry* __restrict__ out,
                              uint64_t first, uint64_t cap) {
    uint64_t p = REVEL_BATCH_HEADER;
    found = 0;
    while (p < n) {
        const uint32_t tag = rep[p++];
        if (tag != REVEL_TYPE_VALUE && tag != REVEL_TYPE_DELETION) return REVEL_BATCH_BAD_TAG;
        uint32_t klen, vlen = 0;
        if (!get_varint32(rep, p, n, klen) || n - p < klen) return REVEL_BATCH_BAD_ENTRY;
        const uint64_t koff = p;
        p += klen;
        uint64_t voff = p;
        if (tag == REVEL_TYPE_VALUE) {
            if (!get_varint32(rep, p, n, vlen) || n - p < vlen) return REVEL_BATCH_BAD_ENTRY;
            voff = p;
            p += vlen;
        }
        if (EMIT && first + found < cap) {
            revel_batch_entry e;
            e.sequence = seq + found;
            e.key_offset = rep_off + koff;
            e.value_offset = rep_off + voff;
            e.key_len = klen;
            e.value_len = vlen;
            e.batch = batch;
            e.type = (uint8_t)tag;
            e.reserved[0] = e.reserved[1] = e.reserved[2] = 0;
            out[first + found] = e;
        }
        ++found;
    }
    return found == count ? REVEL_BATCH_OK : REVEL_BATCH_WRONG_COUNT;
}

__device__ __forceinline__ bool batch_span(const revel_logical_record& r, uint64_t payload_bytes) {
    return r.status == REVEL_LOGICAL_OK && r.payload_offset <= payload_bytes &&
           r.length <= payload_bytes - r.payload_offset;
}

__global__ void k_batch_count(const uint8_t* __restrict__ payload, uint64_t payload_bytes,
                              const revel_logical_record* __restrict__ logical, uint64_t n,
                              revel_batch_info* __restrict__ info, uint64_t* __restrict__ nent) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const revel_logical_record r = logical[i];
        revel_batch_info o;
        o.sequence = 0;
        o.first_entry = 0;
        o.count = 0;
        o.nentries = 0;
        for (int k = 0; k < 7; ++k) o.reserved[k] = 0;
        if (!batch_span(r, payload_bytes)) {
            o.status = REVEL_BATCH_NOT_RECORD;
        } else if (r.length < REVEL_BATCH_HEADER) {
            o.status = REVEL_BATCH_TOO_SMALL;
        } else {
            const uint8_t* rep = payload + r.payload_offset;
            o.sequence = load_le(rep, 8);
            o.count = (uint32_t)load_le(rep + 8, 4);
            o.status = walk_batch<false>(rep, r.payload_offset, r.length, o.sequence, o.count, (uint32_t)i, o.nentries,
                                         nullptr, 0, 0);
        }
        info[i] = o;
        nent[i] = o.nentries;
    }
}

__global__ void k_batch_emit(const uint8_t* __restrict__ payload, uint64_t payload_bytes,
                             const revel_logical_record* __restrict__ logical, uint64_t n,
                             const uint64_t* __restrict__ first, revel_batch_info* __restrict__ info,
                             revel_batch_entry* __restrict__ entries, uint64_t cap) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t f = first[i];
        info[i].first_entry = f;
        const revel_logical_record r = logical[i];
        if (!batch_span(r, payload_bytes) || r.length < REVEL_BATCH_HEADER) continue;
        const uint8_t* rep = payload + r.payload_offset;
        uint32_t found;
        walk_batch<true>(rep, r.payload_offset, r.length, load_le(rep, 8), (uint32_t)load_le(rep + 8, 4), (uint32_t)i,
                         found, entries, f, cap);
    }
}

uint32_t grid_for(const revel::DeviceInfo& di, uint64_t n) {
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu * 8, (n + 255) / 256));
}

}  // namespace

namespace revel {

hipError_t batch_count(const DeviceInfo& di, const void* d_payload, uint64_t payload_bytes,
                       const revel_logical_record* d_logical, uint64_t n, revel_batch_info* d_info, uint64_t* d_nent,
                       hipStream_t st) {
    hipLaunchKernelGGL(k_batch_count, dim3(grid_for(di, n)), dim3(256), 0, st, static_cast<const uint8_t*>(d_payload),
                       payload_bytes, d_logical, n, d_info, d_nent);
    return hipGetLastError();
}

hipError_t batch_emit(const DeviceInfo& di, const void* d_payload, uint64_t payload_bytes,
                      const revel_logical_record* d_logical, uint64_t n, const uint64_t* d_first,
                      revel_batch_info* d_info, revel_batch_entry* d_entries, uint64_t cap, hipStream_t st) {
    hipLaunchKernelGGL(k_batch_emit, dim3(grid_for(di, n)), dim3(256), 0, st, static_cast<const uint8_t*>(d_payload),
                       payload_bytes, d_logical, n, d_first, d_info, d_entries, cap);
    return hipGetLastError();
}

}  // namespace revel
