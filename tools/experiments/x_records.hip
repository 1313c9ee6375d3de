// x_records.hip -- config C3 verify EXPERIMENT arms (not part of librevel_wal.so).
//
// This translation unit compiles the production k_records.hip (its kernels,
// tables and launchers) together with the verify kernels measured on the way
// to the production k_verify_rows: the round-1 kernel (v1), v2's boundary
// paths, v3's load shapes (quad transpose, 64-B rounds), v5 and the register
// ring.  Results: profiles/r1*_c3_*.txt, r2_c3_v7_vs_v3.txt; DESIGN.md section
// 4.2.  Since round 6 it also holds round 5's small-record kernels, moved out
// of the product: the one-pass count + checksum kernels
// (x_verify_fused.inc, x_verify_fused2.inc), the coalesced dense kernel
// (x_verify_chunks.inc) and dense2 with quad-coalesced loads
// (x_verify_dense_quad.inc), each behind a revel_x_* entry point instead of
// an environment switch.  Symbols are hidden except the revel_x_* functions;
// the device tables are this module's own copies (filled by its own
// k_init_len_tables).
#include <vector>

#include "k_records.hip"

namespace {
#include "x_verify_v1.inc"
#include "x_verify_ring.inc"
#include "x_verify5.inc"
#include "x_verify_walk.inc"
#include "x_verify_fused.inc"
#include "x_verify_chunks.inc"
#include "x_verify_fused2.inc"
#include "x_verify_dense_quad.inc"
#include "x_verify_dense_sorted.inc"
#include "x_verify_dense_staged.inc"
#include "x_verify_dense_pairs.inc"

// Header-list entries past kListCap of the blocks the one-pass kernels left
// (fb[0] counts them; none: the launch leaves at once).
__global__ void k_list_overflow_gated(const uint8_t* __restrict__ image, uint64_t nbytes,
                                      const uint32_t* __restrict__ counts, const uint32_t* __restrict__ first,
                                      const uint64_t* __restrict__ hlist, revel_record_result* __restrict__ out,
                                      const uint32_t* __restrict__ fb) {
    if (__builtin_amdgcn_readfirstlane(*fb) == 0u) return;
    const OverflowArgs ov{image, nbytes, first, hlist, out};
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < nblocks;
         b += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t n = counts[b];
        if (n > kListCap) list_overflow_block(ov, b, n);
    }
}
}  // namespace

namespace revel {
namespace {

template <bool FRAME, int BP>
hipError_t launch_verify2(uint64_t grid, bool partial, const uint8_t* img, uint64_t nbytes, uint64_t base_offset,
                          const uint32_t* d_first, revel_record_result* d_out, uint32_t lead, const uint64_t* hl,
                          const uint32_t* d_counts, hipStream_t st) {
    hipLaunchKernelGGL((k_verify_records2<FRAME, BP, BS_WHOLE>), dim3((uint32_t)grid), dim3(kVerify2Threads), 0, st,
                       img, nbytes, base_offset, d_first, d_out, lead, hl, d_counts,
                       reinterpret_cast<const uint64_t*>(d_out), 3u);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !partial) return e;
    hipLaunchKernelGGL((k_verify_records2<FRAME, BP, BS_PARTIAL>), dim3(1), dim3(kVerify2Threads), 0, st, img, nbytes,
                       base_offset, d_first, d_out, lead, hl, d_counts, reinterpret_cast<const uint64_t*>(d_out), 3u);
    return hipGetLastError();
}

uint32_t grid_for(const DeviceInfo& di, uint64_t n, uint64_t waves) {
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu, (n + waves - 1) / waves));
}

// k_verify_rows with another ring depth / workgroup size (production: 8 rows, 1024 threads)
template <int RING, int THREADS, int DIAG = 0, int NB = 4>
hipError_t launch_rows_shape(const DeviceInfo& di, const uint8_t* img, uint64_t nbytes, uint64_t base_offset,
                             const uint32_t* d_first, revel_record_result* d_out, const uint64_t* hl,
                             const uint32_t* d_counts, const uint64_t* xl, uint32_t xs, hipStream_t st,
                             revel_record_result* rows_out = nullptr) {
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    const uint64_t b_hi = nbytes / kBlockSize;
    uint32_t* d_blist = reinterpret_cast<uint32_t*>(const_cast<uint64_t*>(hl) + nblocks * kListStride);
    if (b_hi) {
        hipError_t e = launch_block_order(di, d_counts, 0u, (uint32_t)b_hi, d_blist, st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((k_verify_rows<false, RING, THREADS, DIAG, NB>), dim3((uint32_t)std::max(1, di.num_cu)),
                           dim3(THREADS), 0, st, img, base_offset, d_first, rows_out ? rows_out : d_out, 0u, hl,
                           d_counts, xl, d_blist + kBlockListAux, d_blist);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        if constexpr (DIAG == 0) {  // the production kernel leaves its results to the expander
            e = launch_expand_rows(di, base_offset, 0u, d_first, d_out, hl, d_counts, 0u, (uint32_t)b_hi, 0xFFFFFFFFu,
                                   kBlockSize, st);
            if (e != hipSuccess) return e;
        }
    }
    return launch_dense_and_partial<false>(di, img, nbytes, base_offset, d_first, d_out, 0u, hl, d_counts, xl, xs, st);
}

// ---- the fused pipeline (x_verify_walk.inc; round 4, measured slower than the count pass) ----
bool walk_supported(const void* d_image) { return aligned16(d_image); }

hipError_t walk_count_scan(const DeviceInfo& di, const void* d_image, uint64_t nbytes, uint32_t* d_counts,
                           uint32_t* d_first, uint64_t* d_hlist, hipStream_t st) {
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    if (nblocks == 0) return hipSuccess;
    // list positions and block indices in 32 bits (the position counter runs to P + W)
    if (nblocks > (1ull << 30) || !aligned16(d_image)) return hipErrorInvalidValue;
    hipError_t e = ensure_len_tables(di, st);
    if (e != hipSuccess) return e;
    uint64_t p = 1;
    while (p < nblocks) p <<= 1;
    hipLaunchKernelGGL((k_verify_walk<kRowsRing>), dim3((uint32_t)std::max(1, di.num_cu)), dim3(kRowsThreads), 0, st,
                       static_cast<const uint8_t*>(d_image), nbytes, d_counts, d_hlist, (uint32_t)(p - 1));
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    uint32_t* aux = block_list(d_hlist, nblocks);
    const uint64_t ntiles = (nblocks + kWalkTile - 1) / kWalkTile;
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ntiles, (uint64_t)std::max(1, di.num_cu) * 4));
    hipLaunchKernelGGL(k_walk_tiles, dim3(grid), dim3(256), 0, st, d_counts, (uint32_t)nblocks, aux + 3);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_walk_scan, dim3(grid), dim3(256), 0, st, d_counts, (uint32_t)nblocks, aux + 3, d_first, aux);
    return hipGetLastError();
}

hipError_t walk_verify(const DeviceInfo& di, const void* d_image, uint64_t nbytes, uint64_t base_offset,
                       const uint32_t* d_first, revel_record_result* d_out, const uint64_t* d_hlist,
                       const uint32_t* d_counts, hipStream_t st) {
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    if (nblocks == 0) return hipSuccess;
    const uint8_t* img = static_cast<const uint8_t*>(d_image);
    const uint32_t* aux = block_list(d_hlist, nblocks);
    const OverflowArgs ov{img, nbytes, d_first, d_hlist, d_out};
    const uint64_t nchunks = (nblocks + kExpandBatch - 1) / kExpandBatch;
    constexpr uint64_t kWaves = kExpandThreads / 64;
    const uint64_t grid = std::max<uint64_t>(
        1, std::min<uint64_t>((uint64_t)std::max(1, di.num_cu) * 8, (nchunks + kWaves - 1) / kWaves));
    hipLaunchKernelGGL(k_expand_walk, dim3((uint32_t)grid), dim3(kExpandThreads), 0, st, base_offset, d_first, d_out,
                       d_hlist, d_counts, (uint32_t)nblocks, (uint32_t)(nbytes % kBlockSize), ov, aux);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // dense blocks (the partial tail block too): their lists and the overflow entries in the result slots
    return launch_dense_and_partial<false>(di, img, nbytes, base_offset, d_first, d_out, 0u, d_hlist, d_counts,
                                           reinterpret_cast<const uint64_t*>(d_out),
                                           (uint32_t)(sizeof(revel_record_result) / 8), st, aux + 1, true);
}


hipError_t x_verify(const DeviceInfo& di, int variant, const void* d_image, uint64_t nbytes, uint64_t base_offset,
                    const uint32_t* d_first, revel_record_result* d_out, const uint64_t* d_hlist,
                    const uint32_t* d_counts, hipStream_t st) {
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    const uint8_t* img = static_cast<const uint8_t*>(d_image);
    if (variant == 1) {
        hipLaunchKernelGGL(k_verify_records, dim3(std::max<uint32_t>(1, std::min<uint64_t>((uint64_t)di.num_cu * 2,
                                                                                     (nblocks + 7) / 8))),
                           dim3(kVerifyThreads), 0, st, img, nbytes, base_offset, d_first, d_out);
        return hipGetLastError();
    }
    if (variant == 0) return verify_records_path(di, 0, d_image, nbytes, base_offset, d_first, d_out, d_hlist, d_counts, st);
    if (variant == 2) return verify_records_path(di, 1, d_image, nbytes, base_offset, d_first, d_out, d_hlist, d_counts, st);
    if (variant == 8) return verify_records_path(di, 2, d_image, nbytes, base_offset, d_first, d_out, d_hlist, d_counts, st);
    hipError_t e0 = ensure_len_tables(di, st);
    if (e0 != hipSuccess) return e0;
    const uint64_t grid = grid_for(di, nblocks, kVerify2Threads / 64);
    const uint64_t* hl = d_hlist;
    if (hl && d_counts) {
        const uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>(1u << 20, (nblocks + 63) / 64));
        hipLaunchKernelGGL(k_list_overflow, dim3((uint32_t)g), dim3(64), 0, st, img, nbytes, d_counts, d_first, hl,
                           d_out);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    const bool partial = nbytes % kBlockSize != 0;
    const bool lists = hl && d_counts && aligned16(img);
    const uint64_t* xl = reinterpret_cast<const uint64_t*>(d_out);
    const uint32_t xs = (uint32_t)(sizeof(revel_record_result) / 8);
    const uint64_t b_hi = nbytes / kBlockSize;
    switch (variant) {
        case 3: return launch_verify2<false, BP_MASK>(grid, partial, img, nbytes, base_offset, d_first, d_out, 0u, hl,
                                                      d_counts, st);
        case 4: return launch_verify2<false, BP_MASK_NOVOTE>(grid, partial, img, nbytes, base_offset, d_first, d_out,
                                                             0u, hl, d_counts, st);
        case 5:  // round-1 production: one kernel for whole and partial blocks
            hipLaunchKernelGGL((k_verify_records2<false, BP_BYTES, BS_ALL>), dim3((uint32_t)grid),
                               dim3(kVerify2Threads), 0, st, img, nbytes, base_offset, d_first, d_out, 0u, hl, d_counts,
                               xl, 3u);
            return hipGetLastError();
        case 6: return launch_verify2<false, BP_BYTES>(grid, partial, img, nbytes, base_offset, d_first, d_out, 0u,
                                                       hl, d_counts, st);
        case 7: {  // v5 over the sparse whole blocks
            if (!lists) return hipErrorInvalidValue;
            if (b_hi) {
                hipLaunchKernelGGL(k_verify_records5, dim3(grid_for(di, b_hi, kV5Threads / 64)), dim3(kV5Threads), 0,
                                   st, img, nbytes, base_offset, d_first, d_out, hl, d_counts);
                hipError_t e = hipGetLastError();
                if (e != hipSuccess) return e;
            }
            return launch_dense_and_partial<false>(di, img, nbytes, base_offset, d_first, d_out, 0u, hl, d_counts, xl,
                                                   xs, st);
        }
        case 9:  // v3 split with quad-coalesced loads + DPP transpose
            if (!lists) return hipErrorInvalidValue;
            return launch_verify_split<false, false, true>(di, img, nbytes, base_offset, d_first, d_out, 0u, hl,
                                                           d_counts, xl, xs, st);
        case 10:  // control for 9: the same 64-B rounds with lane-owned loads
            if (!lists) return hipErrorInvalidValue;
            return launch_verify_split<false, false, false, true>(di, img, nbytes, base_offset, d_first, d_out, 0u, hl,
                                                                  d_counts, xl, xs, st);
        case 14:  // variant 9's quad transpose with 128-B rounds
            if (!lists) return hipErrorInvalidValue;
            return launch_verify_split<false, false, true, false, true>(di, img, nbytes, base_offset, d_first, d_out,
                                                                        0u, hl, d_counts, xl, xs, st);
        case 20:  // rows, 16-row ring, 768 threads
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<16, 768>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 21:  // rows, 16-row ring, 512 threads
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<16, 512>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 22:  // rows, 8-row ring, 768 threads
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 768>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 23:  // rows, 16-row ring, 1024 threads
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<16, 1024>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 24:  // production shape through this module (control for 20-23)
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 25:  // DIAG: finalizer without multiplies (wrong CRCs, timing only)
        case 26:  // DIAG: no captures
        case 27:  // DIAG: both
        case 28:  // DIAG: captures without their reduction
        case 29:  // DIAG: captures without reduction, finalizer without multiplies
            if (!lists) return hipErrorInvalidValue;
            if (variant == 28)
                return launch_rows_shape<8, 1024, 4>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
            if (variant == 29)
                return launch_rows_shape<8, 1024, 5>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
            if (variant == 25)
                return launch_rows_shape<8, 1024, 1>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
            if (variant == 26)
                return launch_rows_shape<8, 1024, 2>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
            return launch_rows_shape<8, 1024, 3>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 31:  // DIAG: no captures, the row's table steps independent (latency probe)
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 10>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 32:  // DIAG: the row's table steps independent, captures on (latency probe)
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 8>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 33:  // DIAG: C2's block order (every block must qualify: probe images only)
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 64>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 34:  // DIAG: C2's block order, no captures
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 66>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 35:  // DIAG: loads + XOR fold only (no steps, captures or multiplies), 8-row ring
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 131>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 36:  // DIAG: loads + XOR fold only, 16-row ring
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<16, 1024, 131>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 37:  // DIAG: no row transposes
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 256>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 38:  // DIAG: no captures, 16-row ring (control: 26)
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<16, 1024, 2>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 39:  // DIAG: loads + XOR fold only, C2's block order (probe images only)
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 195>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 40:  // DIAG: loads + XOR fold only, global loads, 8-row ring
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 643>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 41:  // DIAG: loads + XOR fold only, global loads, 16-row ring
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<16, 1024, 643>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 42:  // DIAG: loads + XOR fold only, global loads, C2's block order
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 707>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 43:  // DIAG: the row loop alone (no per-block work), sorted order
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 7299>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 44:  // DIAG: the row loop alone, C2's order
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 7363>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 45:  // DIAG: the row loop alone, C2's order, 16-row ring
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<16, 1024, 7363>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 46:  // DIAG: loads-only, no finalizer (setup + prefetch kept)
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 1155>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 47:  // DIAG: loads-only, no setup / prefetch (finalizer kept)
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 6275>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 48:  // DIAG: loads-only, prefetch kept (no setup, no finalizer)
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 3203>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 49:  // part 0 peeled out of the part loop
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 8192>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 50:  // DIAG: loads-only, part 0 peeled
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 8323>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 51:  // DIAG: loads-only, no result stores
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 16515>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 52:  // DIAG: loads-only, no finalizer-constant gathers
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 32899>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 53:  // DIAG: loads-only, neither
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 49283>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 54:  // DIAG: full compute, no result stores
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 16384>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 55:  // result stores deferred into the next block's part 0
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 65536>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 56:  // DIAG: nontemporal result stores
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 131072>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 57:  // DIAG: 8 B per record stored
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 262144>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 58:  // DIAG: result stores into per-wave private slots
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 524288>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 59:  // DIAG: results into a private line-aligned 64-slot region per block, all 64 lanes (whole lines)
        case 60: {  // DIAG: the same region, lanes < n only (partial last line)
            if (!lists) return hipErrorInvalidValue;
            static revel_record_result* pad = nullptr;  // scratch of 64 results per block (timing only)
            static uint64_t pad_blocks = 0;
            if (pad_blocks < nblocks) {
                if (pad) (void)hipFree(pad);
                pad = nullptr;
                hipError_t e = hipMalloc(&pad, nblocks * 64 * sizeof(revel_record_result));
                if (e != hipSuccess) return e;
                pad_blocks = nblocks;
            }
            if (variant == 59)
                return launch_rows_shape<8, 1024, 1048576>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl,
                                                           xs, st, pad);
            return launch_rows_shape<8, 1024, 2097152>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs,
                                                       st, pad);
        }
        case 61:  // DIAG: 4 B per record into the block's spare header-list slots (timing only)
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 4194304>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 62:  // DIAG: 4 B per record, a contiguous u32 array in record order (timing only)
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 8388608>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 63: {  // DIAG: 4 B per record into a list-order staging array (offsets made on the host; timing only)
            if (!lists || !b_hi) return hipErrorInvalidValue;
            uint32_t* d_blist = block_list_of(const_cast<uint64_t*>(hl), nblocks);
            hipError_t e = launch_block_order(di, d_counts, 0u, (uint32_t)b_hi, d_blist, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) return e;
            uint32_t len = 0;
            e = hipMemcpy(&len, d_blist, 4, hipMemcpyDeviceToHost);
            if (e != hipSuccess) return e;
            std::vector<uint32_t> list(len), cnt(nblocks), off(len + 1);
            if (len) e = hipMemcpy(list.data(), d_blist + kBlockListAux, 4ull * len, hipMemcpyDeviceToHost);
            if (e == hipSuccess) e = hipMemcpy(cnt.data(), d_counts, 4ull * nblocks, hipMemcpyDeviceToHost);
            if (e != hipSuccess) return e;
            off[0] = 0;
            for (uint32_t k = 0; k < len; ++k) off[k + 1] = off[k] + cnt[list[k]];
            static uint32_t* d_off = nullptr;
            static uint64_t off_cap = 0;
            if (off_cap < len + 1) {
                if (d_off) (void)hipFree(d_off);
                d_off = nullptr;
                e = hipMalloc(&d_off, 4ull * (len + 1));
                if (e != hipSuccess) return e;
                off_cap = len + 1;
            }
            e = hipMemcpy(d_off, off.data(), 4ull * (len + 1), hipMemcpyHostToDevice);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL((k_verify_rows<false, 8, 1024, 16777216, 4>), dim3((uint32_t)std::max(1, di.num_cu)),
                               dim3(1024), 0, st, img, base_offset, d_first, d_out, 0u, hl, d_counts,
                               reinterpret_cast<const uint64_t*>(d_off), d_blist + kBlockListAux, d_blist);
            e = hipGetLastError();
            if (e != hipSuccess) return e;
            return launch_dense_and_partial<false>(di, img, nbytes, base_offset, d_first, d_out, 0u, hl, d_counts, xl, xs,
                                                   st);
        }
        case 30:  // rows with eight captures per flush
            if (!lists) return hipErrorInvalidValue;
            return launch_rows_shape<8, 1024, 0, 8>(di, img, nbytes, base_offset, d_first, d_out, hl, d_counts, xl, xs, st);
        case 15:  // session-5 production: v3 over the sparse whole blocks
            if (!lists) return hipErrorInvalidValue;
            return launch_verify_split<false, false>(di, img, nbytes, base_offset, d_first, d_out, 0u, hl, d_counts,
                                                     xl, xs, st);
        case 11:  // 16-slot ring, slots refilled in groups of 4 (11), 8 (12), 2 (13)
        case 12:
        case 13: {
            if (!lists) return hipErrorInvalidValue;
            if (b_hi) {
                const uint32_t g = grid_for(di, b_hi, kVerify2Threads / 64);
                if (variant == 11)
                    hipLaunchKernelGGL(k_verify_records3r<4>, dim3(g), dim3(kVerify2Threads), 0, st, img, nbytes,
                                       base_offset, d_first, d_out, 0u, hl, d_counts);
                else if (variant == 12)
                    hipLaunchKernelGGL(k_verify_records3r<8>, dim3(g), dim3(kVerify2Threads), 0, st, img, nbytes,
                                       base_offset, d_first, d_out, 0u, hl, d_counts);
                else
                    hipLaunchKernelGGL(k_verify_records3r<2>, dim3(g), dim3(kVerify2Threads), 0, st, img, nbytes,
                                       base_offset, d_first, d_out, 0u, hl, d_counts);
                hipError_t e = hipGetLastError();
                if (e != hipSuccess) return e;
            }
            return launch_dense_and_partial<false>(di, img, nbytes, base_offset, d_first, d_out, 0u, hl, d_counts, xl,
                                                   xs, st);
        }
        default: return hipErrorInvalidValue;
    }
}

// ---- round 5's one-pass count + checksum path (x_verify_fused.inc /
// x_verify_fused2.inc), moved out of the product in round 6 ----
hipError_t fused_count(const DeviceInfo& di, const void* d_image, uint64_t nbytes, uint32_t* d_counts,
                       uint64_t* d_hlist, uint32_t* d_fb, hipStream_t st, int variant) {
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    if (nblocks == 0) return hipSuccess;
    hipError_t e = ensure_len_tables(di, st);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(d_fb, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    if (variant == 2) {  // streamed: 12 waves per CU
        hipLaunchKernelGGL(k_walk_verify2, dim3(grid_for(di, nblocks, kF2Waves)), dim3(kF2Threads), 0, st,
                           static_cast<const uint8_t*>(d_image), nbytes, d_counts, d_hlist, d_fb);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_walk_verify, dim3(grid_for(di, nblocks, kFusedWaves)), dim3(kFusedThreads), 0, st,
                       static_cast<const uint8_t*>(d_image), nbytes, d_counts, d_hlist, d_fb);
    return hipGetLastError();
}

hipError_t fused_verify(const DeviceInfo& di, const void* d_image, uint64_t nbytes, uint64_t base_offset,
                        const uint32_t* d_first, revel_record_result* d_out, const uint64_t* d_hlist,
                        const uint32_t* d_counts, const uint32_t* d_fb, hipStream_t st) {
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    if (nblocks == 0) return hipSuccess;
    const uint8_t* img = static_cast<const uint8_t*>(d_image);
    // blocks with more than kListCap records: their entries past 256 into their result slots,
    // then k_verify_records_dense2 over exactly those blocks (both leave at once when fb[0] == 0)
    const uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(1, di.num_cu) * 4, (nblocks + 255) / 256));
    hipLaunchKernelGGL(k_list_overflow_gated, dim3((uint32_t)g), dim3(256), 0, st, img, nbytes, d_counts, d_first,
                       d_hlist, d_out, d_fb);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const uint64_t nchunks = (nblocks + kExpandBatch - 1) / kExpandBatch;
    constexpr uint64_t kWaves = kExpandThreads / 64;
    const uint64_t grid = std::max<uint64_t>(
        1, std::min<uint64_t>((uint64_t)std::max(1, di.num_cu) * 8, (nchunks + kWaves - 1) / kWaves));
    hipLaunchKernelGGL(k_expand_fused, dim3((uint32_t)grid), dim3(kExpandThreads), 0, st, img, nbytes, base_offset,
                       d_first, d_out, d_hlist, d_counts);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_verify_records_dense2<kFusedCap, true>), dim3(grid_for(di, nblocks, kDenseThreads / 64)),
                       dim3(kDenseThreads), 0, st, img, nbytes, base_offset, d_first, d_out, d_hlist, d_counts, d_fb);
    return hipGetLastError();
}

// The production split (k_verify_rows + expander over blocks of 1..64
// records, after count_scan_records' block order) with another dense kernel:
// dense = 1: k_verify_dense_chunks over blocks of 65..256 records, then
// dense2 over the rest (more than 256, or marked capture-dense); dense = 2:
// dense2 with quad-coalesced loads.  A 16-B aligned image only.
hipError_t verify_dense_variant(const DeviceInfo& di, int dense, const uint8_t* img, uint64_t nbytes,
                                uint64_t base_offset, const uint32_t* d_first, revel_record_result* d_out,
                                const uint64_t* hl, const uint32_t* d_counts, bool list_ready, hipStream_t st) {
    if (!aligned16(img) || !hl || !d_counts || dense < 1 || dense > 16) return hipErrorInvalidValue;
    hipError_t e = ensure_len_tables(di, st);
    if (e != hipSuccess) return e;
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    uint32_t* d_blist = block_list(hl, nblocks);
    const uint64_t* xl = reinterpret_cast<const uint64_t*>(d_out);
    const uint32_t tail_bl = (uint32_t)(nbytes % kBlockSize);
    uint64_t b_hi = nbytes / kBlockSize;
    const bool tail_in_rows = tail_bl != 0;
    const uint32_t tail_block = tail_in_rows ? (uint32_t)b_hi : 0xFFFFFFFFu;
    if (tail_in_rows) ++b_hi;
    const OverflowArgs ov{img, nbytes, d_first, hl, d_out};
    if (!list_ready) {
        e = launch_block_order(di, d_counts, 0u, (uint32_t)b_hi, d_blist, st);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((k_verify_rows<false, kRowsRing, kRowsThreads, 0>), dim3((uint32_t)std::max(1, di.num_cu)),
                       dim3(kRowsThreads), 0, st, img, base_offset, d_first, d_out, 0u, hl, d_counts, xl,
                       d_blist + kBlockListAux, d_blist, tail_block, tail_in_rows ? tail_bl : (uint32_t)kBlockSize, ov,
                       kRowsDyn ? d_blist + 3 : nullptr);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = launch_expand_rows(di, base_offset, 0u, d_first, d_out, hl, d_counts, 0u, (uint32_t)b_hi, tail_block,
                           tail_in_rows ? tail_bl : (uint32_t)kBlockSize, st);
    if (e != hipSuccess) return e;
    const uint32_t* dense_whole = d_blist + 1;
    const uint32_t grid = grid_for(di, nblocks, kDenseThreads / 64);
    if (dense == 1) {
        hipLaunchKernelGGL(k_verify_dense_chunks, dim3(grid_for(di, nblocks, kChunkWaves)), dim3(kChunkThreads), 0, st,
                           img, nbytes, base_offset, d_first, d_out, const_cast<uint64_t*>(hl), d_counts, dense_whole);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((k_verify_records_dense2<kListCap, true>), dim3(grid), dim3(kDenseThreads), 0, st, img,
                           nbytes, base_offset, d_first, d_out, hl, d_counts, dense_whole);
    } else if (dense == 2) {
        hipLaunchKernelGGL((k_verify_records_dense2q<>), dim3(grid), dim3(kDenseThreads), 0, st, img, nbytes,
                           base_offset, d_first, d_out, hl, d_counts, dense_whole);
    } else if (dense == 3) {
        hipLaunchKernelGGL(k_verify_records_dense3, dim3(grid), dim3(kDenseThreads), 0, st, img, nbytes, base_offset,
                           d_first, d_out, hl, d_counts, dense_whole);
    } else if (dense == 16) {
        // lane pairs on whole lines (x_verify_dense_pairs.inc)
        hipLaunchKernelGGL(k_verify_records_dense5, dim3(grid_for(di, nblocks, kPairThreads / 64)), dim3(kPairThreads),
                           0, st, img, nbytes, base_offset, d_first, d_out, hl, d_counts, dense_whole);
    } else {
        // 4..7: batch spans staged in LDS (x_verify_dense_staged.inc): 8 or 12 waves per CU, 1 or 2 chains per lane
        // (8..11: timing probes of 6 and 4, wrong results: loads only / checksums only)
#define XSG(NW, CH, P, ...)                                                                                             \
    hipLaunchKernelGGL((k_verify_records_dense4<NW, CH, P, ##__VA_ARGS__>), dim3(grid_for(di, nblocks, NW)),            \
                       dim3(SgCfg<NW>::threads), 0, st, img, nbytes, base_offset, d_first, d_out, hl, d_counts, dense_whole)
        if (dense == 4) XSG(8, 1, 0);
        else if (dense == 5) XSG(8, 2, 0);
        else if (dense == 6) XSG(12, 1, 0);
        else if (dense == 7) XSG(12, 2, 0);
        else if (dense == 8) XSG(12, 1, 1);
        else if (dense == 9) XSG(12, 1, 2);
        else if (dense == 10) XSG(8, 1, 1);
        else if (dense == 11) XSG(8, 1, 2);
        // 12..15: aligned groups read by ds_read_b128 (sg_crc16); 14 / 15 timing probes (checksums only)
        else if (dense == 12) XSG(12, 1, 0, true);
        else if (dense == 13) XSG(8, 1, 0, true);
        else if (dense == 14) XSG(12, 1, 2, true);
        else XSG(8, 1, 2, true);
#undef XSG
    }
    return hipGetLastError();
}

}  // namespace
}  // namespace revel

namespace {
hipStream_t x_stream(revel_gpu_context* ctx, void* stream) {
    return stream ? static_cast<hipStream_t>(stream) : ctx->stream;
}
int x_hlist(revel_gpu_context* ctx, uint64_t nblocks) {
    if (nblocks > ctx->hlist_cap_blocks) {
        if (ctx->hlist) (void)hipFree(ctx->hlist);
        ctx->hlist = nullptr;
        ctx->hlist_cap_blocks = 0;
        if (hipMalloc(reinterpret_cast<void**>(&ctx->hlist), revel::hlist_words(nblocks) * sizeof(uint64_t)) !=
            hipSuccess)
            return REVEL_IO_ERROR;
        ctx->hlist_cap_blocks = nblocks;
    }
    if (!ctx->small_scratch &&
        hipMalloc(reinterpret_cast<void**>(&ctx->small_scratch), 4 * sizeof(uint32_t)) != hipSuccess)
        return REVEL_IO_ERROR;
    return REVEL_OK;
}
}  // namespace

// Round 5's one-pass path (mode 1: k_walk_verify; 2: the streamed
// k_walk_verify2) on a product context, as the pair revel_x_fused_count_scan
// -> revel_x_fused_verify: the first call walks every block and checksums the
// records of blocks with at most 256 of them in one read of the image, the
// second expands the header lists into d_out and checks the blocks it left
// (the image must not change between them).  16-B aligned images only
// (REVEL_NOT_SUPPORT otherwise).  The product's verify cannot take these
// lists (its memo is cleared).
extern "C" __attribute__((visibility("default"))) int revel_x_fused_count_scan(
    revel_gpu_context* ctx, int mode, const void* d_image, size_t nbytes, uint32_t* d_counts, uint32_t* d_first,
    void* stream) {
    if (!ctx || !d_image || !d_counts || !d_first || mode < 1 || mode > 2) return REVEL_INVALID_ARGUMENT;
    if (nbytes == 0) return REVEL_OK;
    if ((reinterpret_cast<uintptr_t>(d_image) & 15u) != 0) return REVEL_NOT_SUPPORT;
    revel::DeviceGuard guard(ctx->di.device);
    if (guard.err() != hipSuccess) return REVEL_IO_ERROR;
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    int rc = x_hlist(ctx, nblocks);
    if (rc) return rc;
    hipStream_t st = x_stream(ctx, stream);
    hipError_t e = revel::fused_count(ctx->di, d_image, nbytes, d_counts, ctx->hlist, ctx->small_scratch, st, mode);
    if (e == hipSuccess) e = revel::exclusive_scan_t<uint32_t>(d_counts, d_first, nblocks,
                                                                 reinterpret_cast<uint32_t*>(ctx->hlist) +
                                                                     2 * nblocks * kListStride,
                                                                 st);
    ctx->hlist_image = nullptr;
    return e == hipSuccess ? REVEL_OK : REVEL_IO_ERROR;
}
extern "C" __attribute__((visibility("default"))) int revel_x_fused_verify(
    revel_gpu_context* ctx, const void* d_image, size_t nbytes, uint64_t base_offset, const uint32_t* d_counts,
    const uint32_t* d_first, revel_record_result* d_out, void* stream) {
    if (!ctx || !d_image || !d_counts || !d_first || !d_out) return REVEL_INVALID_ARGUMENT;
    if (nbytes == 0) return REVEL_OK;
    revel::DeviceGuard guard(ctx->di.device);
    if (guard.err() != hipSuccess) return REVEL_IO_ERROR;
    hipError_t e = revel::fused_verify(ctx->di, d_image, nbytes, base_offset, d_first, d_out, ctx->hlist, d_counts,
                                       ctx->small_scratch, x_stream(ctx, stream));
    return e == hipSuccess ? REVEL_OK : REVEL_IO_ERROR;
}

// The production split with another dense kernel (1: k_verify_dense_chunks +
// dense2 over the rest; 2: dense2 with quad-coalesced loads; 3: dense2 with
// length-sorted batches, x_verify_dense_sorted.inc; 4..7: batch spans staged in LDS,
// x_verify_dense_staged.inc), after
// revel_gpu_count_scan_records of the same image on this context (its header
// lists and block order).
extern "C" __attribute__((visibility("default"))) int revel_x_verify_dense_variant(
    revel_gpu_context* ctx, int dense, const void* d_image, size_t nbytes, uint64_t base_offset,
    const uint32_t* d_first, revel_record_result* d_out, void* stream) {
    if (!ctx || !d_image || !d_first || !d_out) return REVEL_INVALID_ARGUMENT;
    if (nbytes == 0) return REVEL_OK;
    revel::DeviceGuard guard(ctx->di.device);
    if (guard.err() != hipSuccess) return REVEL_IO_ERROR;
    const bool memo = ctx->hlist && ctx->hlist_image == d_image && ctx->hlist_nbytes == nbytes;
    if (!memo) return REVEL_INVALID_ARGUMENT;
    hipError_t e = revel::verify_dense_variant(ctx->di, dense, static_cast<const uint8_t*>(d_image), nbytes,
                                               base_offset, d_first, d_out, ctx->hlist, ctx->hlist_counts,
                                               ctx->hlist_list_ready, x_stream(ctx, stream));
    ctx->hlist_image = nullptr;
    if (e == hipErrorInvalidValue) return REVEL_INVALID_ARGUMENT;
    return e == hipSuccess ? REVEL_OK : REVEL_IO_ERROR;
}

#ifdef REVEL_FUSED_PHASES
// timing probe builds only (tools/fused_phases.py): k_walk_verify's summed
// cycles per phase (reset = 1 zeroes them first, no copy)
extern "C" __attribute__((visibility("default"))) int revel_x_fused_phases(uint64_t* host, int reset) {
    if (reset) {
        static const unsigned long long z[16] = {};
        return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_fused_phase), z, sizeof z, 0, hipMemcpyHostToDevice);
    }
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fused_phase), 16 * sizeof(uint64_t), 0, hipMemcpyDeviceToHost);
}
#endif

// Verify variant `variant` (numbering of DESIGN.md section 4.2) on a product
// context; uses the header lists of the context's last count pass when they
// belong to this image, like revel_gpu_verify_records.
extern "C" __attribute__((visibility("default"))) int revel_x_verify_records_variant(
    revel_gpu_context* ctx, int variant, const void* d_image, size_t nbytes, uint64_t base_offset,
    const uint32_t* d_first, revel_record_result* d_out, void* stream) {
    if (!ctx || !d_image || !d_first || !d_out) return REVEL_INVALID_ARGUMENT;
    if (nbytes == 0) return REVEL_OK;
    revel::DeviceGuard guard(ctx->di.device);
    if (guard.err() != hipSuccess) return REVEL_IO_ERROR;
    const bool memo = ctx->hlist && ctx->hlist_image == d_image && ctx->hlist_nbytes == nbytes;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    hipError_t e = revel::x_verify(ctx->di, variant, d_image, nbytes, base_offset, d_first, d_out,
                                   memo ? ctx->hlist : nullptr, memo ? ctx->hlist_counts : nullptr, st);
    ctx->hlist_image = nullptr;
    if (e == hipErrorInvalidValue) return REVEL_INVALID_ARGUMENT;
    return e == hipSuccess ? REVEL_OK : REVEL_IO_ERROR;
}

// Block-order experiment: k_verify_rows alone over a caller-built list of
// qualifying blocks (d_list[0] = count, then block indices), so the order the
// waves take blocks in (wave j: list[j], list[j + W], ...) can be measured.
// Uses the header lists of the context's last count pass; dense and partial
// blocks are not touched.  revel_x_rows_waves gives W.
extern "C" __attribute__((visibility("default"))) int revel_x_rows_waves(revel_gpu_context* ctx) {
    return ctx ? std::max(1, ctx->di.num_cu) * (kRowsThreads / 64) : 0;
}
extern "C" __attribute__((visibility("default"))) int revel_x_verify_rows_list(
    revel_gpu_context* ctx, const void* d_image, size_t nbytes, const uint32_t* d_first, revel_record_result* d_out,
    const uint32_t* d_list, void* stream) {
    if (!ctx || !d_image || !d_first || !d_out || !d_list) return REVEL_INVALID_ARGUMENT;
    revel::DeviceGuard guard(ctx->di.device);
    if (guard.err() != hipSuccess) return REVEL_IO_ERROR;
    if (!(ctx->hlist && ctx->hlist_image == d_image && ctx->hlist_nbytes == nbytes)) return REVEL_INVALID_ARGUMENT;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    hipError_t e = revel::ensure_len_tables(ctx->di, st);
    if (e != hipSuccess) return REVEL_IO_ERROR;
    hipLaunchKernelGGL((k_verify_rows<false, kRowsRing>), dim3((uint32_t)std::max(1, ctx->di.num_cu)),
                       dim3(kRowsThreads), 0, st, static_cast<const uint8_t*>(d_image), (uint64_t)0, d_first,
                       d_out, 0u, ctx->hlist, ctx->hlist_counts, reinterpret_cast<const uint64_t*>(d_out), d_list + 1,
                       d_list);
    ctx->hlist_image = nullptr;
    return hipGetLastError() == hipSuccess ? REVEL_OK : REVEL_IO_ERROR;
}

// The fused C3 pipeline (x_verify_walk.inc) on a product context: the row
// stream walks the headers itself (no count pass), then k_expand_walk.  Same
// contract as revel_gpu_count_scan_records / revel_gpu_verify_records (the
// second call uses the header lists and captures of the first, for the same
// image).  Round 4: parity-green, slower than the count pass.
extern "C" __attribute__((visibility("default"))) int revel_x_walk_count_scan(
    revel_gpu_context* ctx, const void* d_image, size_t nbytes, uint32_t* d_counts, uint32_t* d_first, void* stream) {
    if (!ctx || !d_image || !d_counts || !d_first) return REVEL_INVALID_ARGUMENT;
    if (nbytes == 0) return REVEL_OK;
    revel::DeviceGuard guard(ctx->di.device);
    if (guard.err() != hipSuccess) return REVEL_IO_ERROR;
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    if (nblocks > ctx->hlist_cap_blocks) {
        if (ctx->hlist) (void)hipFree(ctx->hlist);
        ctx->hlist = nullptr;
        ctx->hlist_cap_blocks = 0;
        if (hipMalloc(reinterpret_cast<void**>(&ctx->hlist), revel::hlist_words(nblocks) * sizeof(uint64_t)) !=
            hipSuccess)
            return REVEL_IO_ERROR;
        ctx->hlist_cap_blocks = nblocks;
    }
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    hipError_t e = revel::walk_count_scan(ctx->di, d_image, nbytes, d_counts, d_first, ctx->hlist, st);
    ctx->hlist_image = nullptr;  // the product's verify must not take these lists for a count pass's
    if (e == hipErrorInvalidValue) return REVEL_INVALID_ARGUMENT;
    return e == hipSuccess ? REVEL_OK : REVEL_IO_ERROR;
}
extern "C" __attribute__((visibility("default"))) int revel_x_walk_verify(
    revel_gpu_context* ctx, const void* d_image, size_t nbytes, uint64_t base_offset, const uint32_t* d_counts,
    const uint32_t* d_first, revel_record_result* d_out, void* stream) {
    if (!ctx || !d_image || !d_counts || !d_first || !d_out) return REVEL_INVALID_ARGUMENT;
    if (nbytes == 0) return REVEL_OK;
    revel::DeviceGuard guard(ctx->di.device);
    if (guard.err() != hipSuccess) return REVEL_IO_ERROR;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    hipError_t e = revel::walk_verify(ctx->di, d_image, nbytes, base_offset, d_first, d_out, ctx->hlist, d_counts, st);
    return e == hipSuccess ? REVEL_OK : REVEL_IO_ERROR;
}
