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
// entry, through a 48-B register window (RepWindow) -- keys and values are
// located, never copied.  A wave-per-batch walk from an LDS window measured
// 2.4x slower (the uniform walk is VALU-bound: DESIGN.md section 4.8).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "gpu_internal.h"

namespace {

// A lane's 48-B register window over its rep: three aligned 16-B chunks
// fetched together.  A byte chain walked through global byte loads costs one
// memory round trip per byte read (tag, key length, value length: three
// dependent trips per entry); through the window an entry whose header bytes
// share 48 B -- fill1's whole 31-B batch prefix, any 16-B-key entry's tag..vlen
// -- costs one.  Chunks are clamped to those holding rep bytes: an aligned
// 16 B never crosses a page, and bytes past the rep are never consumed (the
// walk checks every position against n).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // native vector: stays in registers

struct RepWindow {
    const u32x4* __restrict__ chunks;  // rep rounded down to 16 B
    uint64_t a0;                       // rep address & 15: virtual offset v = a0 + pos
    uint64_t last;                     // last chunk holding a rep byte
    uint64_t lo;                       // the window holds virtual bytes [lo, lo + 48)
    u32x4 c0, c1, c2;

    __device__ RepWindow(const uint8_t* rep, uint64_t n) {
        a0 = reinterpret_cast<uintptr_t>(rep) & 15u;
        chunks = reinterpret_cast<const u32x4*>(rep - a0);
        last = (a0 + n - 1) >> 4;
        fetch(a0);
    }
    __device__ __forceinline__ void fetch(uint64_t v) {
        const uint64_t c = v >> 4;
        lo = c << 4;
        c0 = chunks[c];  // c <= last: v is a rep byte
        c1 = chunks[c + 1 <= last ? c + 1 : c];
        c2 = chunks[c + 2 <= last ? c + 2 : c];
    }
    __device__ __forceinline__ uint32_t operator()(uint64_t pos) {
        const uint64_t v = a0 + pos;
        if (v - lo >= 48u) fetch(v);
        const uint32_t o = uint32_t(v - lo);
        // masks, not selects: the optimiser turns a select of loaded members
        // into a load from a selected address, which keeps the window in
        // memory (an alloca promoted to LDS) instead of registers
        const uint32_t m0 = o < 16u ? ~0u : 0u, m2 = o >= 32u ? ~0u : 0u, m1 = ~(m0 | m2);
        const u32x4 q = (c0 & m0) | (c1 & m1) | (c2 & m2);
        const uint32_t k = (o >> 2) & 3u;
        const uint32_t w = k == 0 ? q.x : k == 1 ? q.y : k == 2 ? q.z : q.w;
        return (w >> ((o & 3u) * 8u)) & 0xFFu;
    }
};

// Walk one rep of n >= REVEL_BATCH_HEADER bytes through get; reads the header
// into seq / count; with EMIT, writes entry k to out[first + k] when it is
// below cap.  Returns the REVEL_BATCH_* status; found = entries decoded.
template <bool EMIT>
__device__ __forceinline__ uint8_t walk_batch(RepWindow& get, uint64_t rep_off, uint64_t n, uint64_t& seq, uint32_t& count,
                              uint32_t batch, uint32_t& found, revel_batch_entry* __restrict__ out, uint64_t first,
                              uint64_t cap) {
    // get_varint32 (coding.rs:96-123) over the window, bounded by n
    auto varint = [&](uint64_t& pos, uint32_t& v) -> bool {
        uint32_t result = 0;
        for (uint32_t shift = 0; shift <= 28 && pos < n; shift += 7) {
            const uint32_t b = get(pos++);
            if (b & 128u) {
                result |= (b & 127u) << shift;
            } else {
                v = result | (b << shift);
                return true;
            }
        }
        return false;
    };
    seq = 0;
    count = 0;
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) seq |= uint64_t(get(q)) << (8 * q);
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) count |= get(8 + q) << (8 * q);
    uint64_t p = REVEL_BATCH_HEADER;
    found = 0;
    while (p < n) {
        const uint32_t tag = get(p++);
        if (tag != REVEL_TYPE_VALUE && tag != REVEL_TYPE_DELETION) return REVEL_BATCH_BAD_TAG;
        uint32_t klen, vlen = 0;
        if (!varint(p, klen) || n - p < klen) return REVEL_BATCH_BAD_ENTRY;
        const uint64_t koff = p;
        p += klen;
        uint64_t voff = p;
        if (tag == REVEL_TYPE_VALUE) {
            if (!varint(p, vlen) || n - p < vlen) return REVEL_BATCH_BAD_ENTRY;
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
            RepWindow win(payload + r.payload_offset, r.length);
            o.status = walk_batch<false>(win, r.payload_offset, r.length, o.sequence, o.count, (uint32_t)i, o.nentries,
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
        const revel_logical_record r = logical[i];
        if (batch_span(r, payload_bytes) && r.length >= REVEL_BATCH_HEADER) {
            RepWindow win(payload + r.payload_offset, r.length);
            uint64_t seq;
            uint32_t count, found;
            walk_batch<true>(win, r.payload_offset, r.length, seq, count, (uint32_t)i, found, entries, f, cap);
        }
        info[i].first_entry = f;  // stored last: loads and stores share vmcnt, no load waits for it
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
