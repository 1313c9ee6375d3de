// k_records.hip -- config C3 kernels: per-block header walk (count + header
// list), exclusive scans, record verify (production k_verify_records3 and the
// experiment arms), device append framing and the replay summaries.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <type_traits>

#include "device_common.h"

using namespace revel;

namespace {
// The 7 header bytes at byte sh (0..5) of a 12-byte window w.
__device__ __forceinline__ Hdr header_in_window(uint3 w, uint32_t sh) {
    const uint32_t r = sh & 3u;
    const bool hi = sh >= 4u;
    const uint32_t lo0 = hi ? w.y : w.x, lo1 = hi ? w.z : w.y, lo2 = hi ? 0u : w.z;
    const uint32_t a = __builtin_amdgcn_alignbyte(lo1, lo0, r);  // bytes sh..sh+3
    const uint32_t b = __builtin_amdgcn_alignbyte(lo2, lo1, r);  // bytes sh+4..sh+7
    return {a, b & 0xFFFFu, (b >> 16) & 0xFFu};
}

// The header walk, one lane per block b = b_wave + lane of a whole wave (lanes
// past the image walk nothing): each block's number of physical records, and
// its header list -- the first kListCap headers (list_entry; the walk stops at
// the first bad header, so only the last entry can be bad), then the in-block
// offset of record kListCap when the block has more.
//
// A hop loads the 12-B window a = min(off & ~3, bl - 12) holding the next
// header (it never reaches past the block or the image end; off - a <= 5 keeps
// the 7 header bytes inside it), issued before anything else of the hop: loads
// and stores share vmcnt, so a store issued first would put its completion
// into the dependent walk.  The entries go to the wave's LDS slot row n % 16;
// every kStageHops hops (and at the end) the whole wave writes the group out:
// lane l stores 16 B (entries 2p, 2p + 1 of the group, p = l % 8) of block
// 8 i + l / 8, i = 0..7, so a store covers 8 blocks x 128 B -- whole lines,
// since kListStride keeps every list 128-B aligned -- instead of 64 scattered
// 16-B pieces every other hop.  Round 6 (profiles/r6/count_*.log, 4 GiB
// images): without any list stores the walk took 0.57 ms on small records and
// 34 us on Zipf against 0.93 ms / 48 us with per-lane stores; staged groups of
// 16 with aligned lists take 0.73 ms / 41 us (8-hop groups: 0.76 ms; unaligned
// lists: 0.75-0.84 ms).
constexpr uint32_t kStageHops = 16;
constexpr uint32_t kStageLanes = kStageHops / 2;     // lanes per block in a group's stores (16 B each)
constexpr uint32_t kStageBlocks = 64 / kStageLanes;  // blocks per store
constexpr uint32_t kStageRow = 65;  // u64 per LDS slot row: 64 lanes + 1 (spreads the transposed reads' banks)
constexpr uint32_t kStageWords = kStageHops * kStageRow;
static_assert(kListCap % kStageHops == 0, "a group never straddles kListCap");
static_assert((kListStride * 8u) % 128u == 0, "every block's header list starts on a 128-B line");
__device__ __forceinline__ uint32_t count_block_wave(const uint8_t* __restrict__ image, uint64_t nbytes,
                                                     uint64_t b_wave, uint64_t* __restrict__ hlist,
                                                     uint64_t* __restrict__ stage) {
    const uint32_t lane = lane_id();
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    const uint64_t b = b_wave + lane;
    const bool inb = b < nblocks;
    const uint64_t base = b * kBlockSize;
    const uint32_t bl = inb ? (uint32_t)std::min<uint64_t>(kBlockSize, nbytes - base) : 0u;
    uint32_t n = 0;
    bool walking = bl >= 12u;
    if (inb && !walking && bl >= kHeaderSize) {  // a last block of 7..11 bytes: one header at most
        const Hdr h = read_header(image + base, 0u, bl);
        hlist[b * kListStride] = list_entry(h);
        n = 1;
    }
    if (!__builtin_amdgcn_ballot_w64(walking)) return n;  // wave-uniform
    const bool staged = walking;  // (a 7..11-byte block's one entry is stored above)
    const uint8_t* const blk = image + base;
    const uint32_t cap = bl - 12u;
    uint32_t off = 0, a = 0;
    uint3 w{};
    if (walking) w = *reinterpret_cast<const uint3*>(blk);
    // the wave's 64 lists; a store whose offset lies past them is dropped
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        hlist + b_wave * kListStride, (short)0, (int)(64u * kListStride * 8u), 0x00020000);
    for (uint32_t g0 = 0;; g0 += kStageHops) {  // wave-uniform: a group of kStageHops hops
        // kStageHops hops for the wave, each lane's masked by its walk: no lane
        // leaves the loop, so the next window stays in flight in the register
        // the walk reads it from, across the group's stores
        for (uint32_t j = 0; j < kStageHops; ++j) {
            if (walking) {
                const Hdr h = header_in_window(w, off - a);
                const bool ok = classify(h, off, bl) == REVEL_REC_OK;
                const uint32_t next = off + kHeaderSize + h.len;  // <= bl when ok
                const bool more = ok && bl - next >= kHeaderSize;
                const uint32_t an = min(more ? next & ~3u : 0u, cap);
                const uint3 wn = *reinterpret_cast<const uint3*>(blk + an);
                if (n < kListCap) {
                    stage[(n % kStageHops) * kStageRow + lane] = list_entry(h);
                } else if (n == kListCap) {
                    hlist[b * kListStride + kListCap] = uint64_t(off);  // where record kListCap starts
                }
                ++n;
                walking = more;
                off = next;
                a = an;
                w = wn;
            }
        }
        if (g0 < kListCap) {
            // every lane: the group out, kStageLanes stores of 8 blocks x 128 B.
            // Unconditional (a lane with nothing to store points past the
            // resource): a fixed number of stores, so the compiler's wait for
            // the next window counts them exactly
            __builtin_amdgcn_wave_barrier();
            const uint32_t p = lane % kStageLanes;
            const uint32_t k = g0 + 2u * p;
#pragma unroll
            for (uint32_t i = 0; i < kStageLanes; ++i) {
                const uint32_t q = kStageBlocks * i + lane / kStageLanes;
                const uint32_t nq = (uint32_t)__shfl(staged ? min(n, kListCap) : 0u, q, 64);
                const uint64_t e0 = stage[(2u * p) * kStageRow + q];
                // (entry k + 1 past the count: a slot no reader takes)
                const uint64_t e1 = stage[(2u * p + 1u) * kStageRow + q];
                const u32x4 v = {(uint32_t)e0, (uint32_t)(e0 >> 32), (uint32_t)e1, (uint32_t)(e1 >> 32)};
                const uint32_t o = k < nq ? (q * kListStride + k) * 8u : 0x80000000u;
                __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)o, 0, 0);
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (!__builtin_amdgcn_ballot_w64(walking)) break;
    }
    return n;
}

// One lane per block.  With wsums (one wave per workgroup), wsums[w] = the
// records of blocks [64 w, 64 w + 64): the first pass of the exclusive scan
// that follows.  (The replay and shard loaders' count pass; the C-ABI's is
// k_count_hist, verify_rows.inc.)
__global__ __launch_bounds__(64) void k_count_records(const uint8_t* __restrict__ image, uint64_t nbytes,
                                                      uint32_t* __restrict__ counts, uint64_t* __restrict__ hlist,
                                                      uint32_t* __restrict__ wsums) {
    __shared__ uint64_t stage[kStageWords];
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    for (uint64_t b0 = blockIdx.x * 64ull; b0 < nblocks; b0 += gridDim.x * 64ull) {  // wave-uniform
        const uint64_t b = b0 + threadIdx.x;
        const uint32_t n = count_block_wave(image, nbytes, b0, hlist, stage);
        if (b < nblocks) counts[b] = n;
        if (wsums) {
            uint32_t t = n;
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) t += __shfl_xor(t, m, 64);
            if (threadIdx.x == 0) wsums[b0 / 64u] = t;
        }
    }
}

// Exclusive scan in two parallel passes over tiles of kScanTile elements
// (256 threads x 4): k_tile_sums writes each tile's sum; k_scan_apply adds the
// sums of the tiles before it and scans its own tile.
constexpr uint32_t kScanTile = 1024;

template <typename T>
__device__ __forceinline__ T block_reduce_256(T v, T* red) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    if (lane_id() == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    const T t = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    return t;
}

template <typename T>
__global__ __launch_bounds__(256) void k_tile_sums(const T* __restrict__ in, uint64_t n, T* __restrict__ tile_sums) {
    __shared__ T red[4];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
    T v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t i = base + k * 256 + threadIdx.x;
        v += i < n ? in[i] : T(0);
    }
    const T t = block_reduce_256<T>(v, red);
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = t;
}

// PARTS = partial sums per tile in `tile_sums` (1: k_tile_sums; kScanTile / 64:
// the per-wave sums of k_count_records).
template <typename T, uint32_t PARTS = 1>
__global__ __launch_bounds__(256) void k_scan_apply(const T* __restrict__ in, uint64_t n, const T* __restrict__ tile_sums,
                                                    T* __restrict__ out) {
    __shared__ T red[4];
    __shared__ T wsum[4];
    // offset of this tile = sum of the partial sums before it
    T pre = 0;
    for (uint32_t t = threadIdx.x; t < blockIdx.x * PARTS; t += 256) pre += tile_sums[t];
    const T tile_off = block_reduce_256<T>(pre, red);
    // each thread owns 4 consecutive elements
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * 4;
    T v[4], sum = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[k] = base + k < n ? in[base + k] : T(0);
        sum += v[k];
    }
    T x = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const T y = __shfl_up(x, d, 64);
        if ((int)lane_id() >= d) x += y;
    }
    const uint32_t w = threadIdx.x >> 6;
    if (lane_id() == 63) wsum[w] = x;
    __syncthreads();
    T run = tile_off + x - sum;
    for (uint32_t k = 0; k < w; ++k) run += wsum[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (base + k < n) out[base + k] = run;
        run += v[k];
    }
}


// x^(-8 pad) mod P for pad = 0..3 (x^-1 = (P+1)/x, reflected 0x05EC76F1).
struct InvPad {
    uint32_t v[4];
};
constexpr InvPad make_inv_pad() {
    InvPad s{};
    const uint32_t xinv = 0x05EC76F1u;
    uint32_t x8inv = 0x80000000u;
    for (int k = 0; k < 8; ++k) x8inv = multmodp(x8inv, xinv);
    uint32_t v = 0x80000000u;
    for (int p = 0; p < 4; ++p) {
        s.v[p] = v;
        v = multmodp(v, x8inv);
    }
    return s;
}
static_assert(multmodp(make_inv_pad().v[1], x8n(1)) == 0x80000000u, "x^-8 * x^8 == 1");
__constant__ InvPad c_inv_pad = make_inv_pad();


// ---------------------------------------------------------------------------
// Config C3, v2: S4R tables, 16 waves/CU, pipelined loads, wave-uniform fast
// path, exact tails.
// ---------------------------------------------------------------------------
constexpr int kVerify2Threads = 1024;
constexpr uint32_t kRecCap2 = 128;  // >= kListPerBlock

// Header-list entry k of block b.  Verify: the count pass kept k < kListCap in
// hlist, k_list_overflow wrote the rest into the result slots (xlist = out,
// xstride u64 apart).  FRAME: the framing list holds every entry in xlist.
template <bool FRAME>
__device__ __forceinline__ uint64_t list_at(const uint64_t* __restrict__ hlist, const uint64_t* __restrict__ xlist,
                                            uint32_t xstride, uint64_t b, uint32_t first_b, uint32_t k) {
    if (!FRAME && k < kListCap) return hlist[b * kListStride + k];
    return xlist[uint64_t(first_b + k) * xstride];
}

// x^(8d) and init_xor(d) for d = 0..32768, filled once per device.
__device__ uint32_t g_x8n_tab[kBlockSize + 1];
__device__ uint32_t g_init_xor_tab[kBlockSize + 1];

// x^(-8d) for d = 0..32768 (filled with the x^(8d) / init_xor tables).
__device__ uint32_t g_x8inv_tab[kBlockSize + 1];
// k_verify_rows' six inverse-shift tree levels (fill_inv_tree_tables layout),
// computed once here: the kernel copies them instead of 6 GF(2) multiplies per thread.
__device__ uint32_t g_shtab[6 * 1024];

struct InvShiftTables {
    uint32_t chunk[65];  // x^(-8*512*m)
    uint32_t byte[513];  // x^(-8*d)
};
constexpr InvShiftTables make_inv_shift_tables() {
    InvShiftTables s{};
    const uint32_t xinv8 = pow_modp(kXInv, 8);
    const uint32_t xinv4096 = pow_modp(xinv8, 512);
    uint32_t v = 0x80000000u;
    for (int m = 0; m <= 64; ++m) {
        s.chunk[m] = v;
        v = multmodp(v, xinv4096);
    }
    v = 0x80000000u;
    for (int d = 0; d <= 512; ++d) {
        s.byte[d] = v;
        v = multmodp(v, xinv8);
    }
    return s;
}
__constant__ InvShiftTables c_inv_shift = make_inv_shift_tables();
static_assert(multmodp(make_inv_shift_tables().byte[7], x8n(7)) == 0x80000000u, "x^-56 * x^56 == 1");

__device__ __forceinline__ uint32_t gf_x8inv_block(uint32_t n) {
    const uint32_t m = n >> 9, d = n & 511u;
    const uint32_t a = c_inv_shift.chunk[m];
    return d ? gf_mul(a, c_inv_shift.byte[d]) : a;
}

__global__ void k_init_len_tables() {
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d <= kBlockSize; d += gridDim.x * blockDim.x) {
        const uint32_t x = gf_x8n_block(d);
        g_x8n_tab[d] = x;
        g_init_xor_tab[d] = gf_mul(x, 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
        g_x8inv_tab[d] = gf_x8inv_block(d);
        if (d < 6u * 1024u) g_shtab[d] = gf_mul(c_inv_tree.c[d >> 10], (d & 255u) << (8u * ((d >> 8) & 3u)));
    }
}

// Record k's CRC range is [s, em1 + 1).  A bad header (always the last record
// of a list: the walk stops there) and the sentinel slot after the last
// record get s = em1 = 0xFFFF, a range no block position reaches, so lanes
// advance to the next record with two LDS reads and no bounds checks.
constexpr uint16_t kNoRange = 0xFFFFu;
struct VerifyWaveLds2 {
    uint16_t s[kRecCap2 + 1];
    uint16_t em1[kRecCap2 + 1];
    uint16_t off[kRecCap2];  // header offset
    uint32_t acc[kRecCap2];
    uint32_t hstored[kListPerBlock];  // headers of a list-built batch (v3/v4 finalize)
    uint32_t hlt[kListPerBlock];      // len | type << 16
    uint32_t nrec, more_off;
};

// One CRC step over a single byte with the S4R image's T0 (region 1, half 1).
__device__ __forceinline__ uint32_t byte_step_s4r(uint32_t state, uint32_t b, LaneConst L, const uint32_t* tab) {
    const uint32_t x = state ^ b;
    const uint32_t a = __builtin_amdgcn_perm(x, L.lc1, Sel<0>::v);
    return ldsw<128>(tab, a) ^ (state >> 8);
}

template <int TM>
__device__ __forceinline__ uint32_t byte_step_tm(uint32_t state, uint32_t b, LaneConst L, const uint32_t* tab) {
    if constexpr (TM == TM_S4R) {
        return byte_step_s4r(state, b, L, tab);
    } else {
        static_assert(TM == TM_S4, "byte steps: S4R or S4 tables");
        return tab[768 + ((state ^ b) & 0xffu)] ^ (state >> 8);  // T0 of the [T3|T2|T1|T0] image
    }
}

// FRAME = device append framing: headers hold length/type but no CRC yet;
// the kernel writes mask(crc32c(type||payload)) into bytes [off, off+4) of
// each header instead of emitting result records.  `lead` = in-block offset
// of image byte 0 (a batch appended to a partially written block).
template <int BP>
__device__ __forceinline__ uint32_t record_raw(uint32_t acc, uint32_t off, uint32_t len) {
    if constexpr (BP == 0) {
        return acc;
    } else {
        const uint32_t e = off + kHeaderSize + len;
        return gf_mul(c_inv_pad.v[((e + 3u) & ~3u) - e], acc);
    }
}

// Boundary paths (BP) for the 16-B steps that hold a record start or end:
//   BP_BYTES       exact: bytes past the end absorbed one at a time (v2)
//   BP_MASK        the word holding the end is absorbed with the bytes past e
//                  zeroed, so every flush is aligned to E = ceil4(e) (R * x^(8 pad));
//                  the finalizer multiplies by x^(-8 pad).  Branch-light: one
//                  masked absorb per word, the flush is the only divergence.
//   BP_MASK_NOVOTE same as BP_MASK without the wave-uniform interior fast path.
enum BoundaryPath : int { BP_BYTES = 0, BP_MASK = 1, BP_MASK_NOVOTE = 2 };

// WHICH: 0 = every block; 1 = whole blocks only (plain 16-B loads, no guards:
// the guarded loads of a partial block raise register pressure for the whole
// kernel); 2 = only the partial blocks (the first, when the image starts
// mid-block, and the last), launched as one extra workgroup.
enum BlockSet : int { BS_ALL = 0, BS_WHOLE = 1, BS_PARTIAL = 2 };

template <bool FRAME, int BP = BP_BYTES, int WHICH = BS_ALL, int TM = TM_S4R, int THREADS = kVerify2Threads,
          bool SPARSE_ONLY = false>
__global__ __launch_bounds__(THREADS) void k_verify_records2(const uint8_t* __restrict__ image, uint64_t nbytes,
                                                                     uint64_t base_offset,
                                                                     const uint32_t* __restrict__ first,
                                                                     revel_record_result* __restrict__ out,
                                                                     uint32_t lead,
                                                                     const uint64_t* __restrict__ hlist,
                                                                     const uint32_t* __restrict__ counts,
                                                                     const uint64_t* __restrict__ xlist = nullptr,
                                                                     uint32_t xstride = 3, uint32_t skip_tail = 0) {
    __shared__ uint32_t tab[TableCfg<TM>::bytes / 4];
    __shared__ VerifyWaveLds2 wl_all[THREADS / 64];
    fill_tables<TM>(tab);
    __syncthreads();
    VerifyWaveLds2& wl = wl_all[threadIdx.x >> 6];
    const LaneConst L = make_lane_const();
    const uint32_t lane = lane_id();
    const uint64_t vbytes = nbytes + lead;  // bytes of the virtual block-aligned image
    const uint64_t nblocks = (vbytes + kBlockSize - 1) / kBlockSize;
    const uint64_t waves_per_wg = THREADS / 64;
    const uint64_t gwave = blockIdx.x * waves_per_wg + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nwaves = gridDim.x * waves_per_wg;
    constexpr uint32_t kNone = 0xFFFFFFFFu;

    const uint64_t niter = WHICH == BS_PARTIAL ? std::min<uint64_t>(2, nblocks) : nblocks;
    for (uint64_t it = gwave; it < niter; it += nwaves) {
        const uint64_t b = WHICH == BS_PARTIAL && it == 1 ? nblocks - 1 : it;
        const uint64_t base = b * kBlockSize;  // virtual offset of the block
        const uint8_t* blk = image + base - lead;  // dereferenced only at [lo, bl)
        const uint32_t lo_b = b == 0 ? lead : 0u;
        const uint32_t bl = (uint32_t)std::min<uint64_t>(kBlockSize, vbytes - base);
        const bool full = WHICH == BS_WHOLE || (bl == kBlockSize && lo_b == 0);
        if constexpr (WHICH == BS_WHOLE) {
            if (bl != kBlockSize || lo_b != 0) continue;
        } else if constexpr (WHICH == BS_PARTIAL) {
            if (bl == kBlockSize && lo_b == 0) continue;
        }
        if constexpr (SPARSE_ONLY) {  // a dense partial block went to k_verify_records_dense
            if (counts[b] > kListPerBlock) continue;
        }
        if (skip_tail && b != 0 && b == nblocks - 1) continue;  // k_verify_rows took the tail block
        const uint32_t cs = lane * 512u, ce = cs + 512u;
        uint32_t out_base = FRAME ? 0u : first[b];
        uint32_t walk_from = lo_b;
        auto load_round = [&](uint4* v, int rr) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t pos = cs + rr * 128 + j * 16;
                v[j] = full ? ldg4_plain(reinterpret_cast<const uint4*>(blk + pos))
                            : (pos < bl ? load16_range(blk, pos, lo_b, bl) : make_uint4(0, 0, 0, 0));
            }
        };
        // the chunk's first round does not depend on the record list: issue it now
        uint4 cur[8], nxt[8];
        load_round(cur, 0);
        bool have_round0 = true;
        // header list from the count pass (parallel per-block walks) when it
        // covers the whole block; otherwise lane 0 walks here.
        // header lists: verify = the count pass's (records 0..63 in hlist, the rest
        // in the result slots, xlist = out, stride 3), only for images starting on
        // a block; FRAME = entry k of block b at xlist[first[b] + k], any lead
        const bool have_list = FRAME ? (counts && first && xlist) : (hlist && counts && xlist && lo_b == 0);
        const uint32_t nlist = have_list ? counts[b] : kNone;
        const uint32_t first_b = FRAME ? (have_list ? first[b] : 0u) : out_base;
        uint32_t lpass = 0, lpass_off = lo_b;  // list batches of kListPerBlock records
        uint64_t ent = 0;
        if (nlist != kNone && lane < nlist)
            ent = FRAME ? xlist[uint64_t(first_b) + lane] : hlist[b * kListStride + lane];
        for (;;) {
            const bool from_list = nlist != kNone;
            if (from_list) {
                const uint32_t k0 = lpass * kListPerBlock;
                const uint32_t np = min(nlist - k0, kListPerBlock);
                const Hdr h = list_header(ent);
                const uint32_t sz = lane < np ? kHeaderSize + h.len : 0u;
                const uint32_t off = lpass_off + wave_exclusive_sum(sz);
                if (lane < np) {
                    const bool bad = classify(h, off, bl) != REVEL_REC_OK;
                    wl.off[lane] = (uint16_t)off;
                    wl.s[lane] = bad ? kNoRange : (uint16_t)(off + 6);
                    wl.em1[lane] = bad ? kNoRange : (uint16_t)(off + kHeaderSize + h.len - 1u);
                    wl.acc[lane] = 0;
                }
                if (lane == 0) {
                    wl.s[np] = wl.em1[np] = kNoRange;
                    wl.nrec = np;
                    wl.more_off = k0 + np < nlist ? 1u : kNone;
                }
                lpass_off = __builtin_amdgcn_readlane(off + sz, np - 1u);
            } else if (lane == 0) {
                uint32_t off = walk_from, n = 0, cont = kNone;
                while (bl - off >= kHeaderSize) {
                    if (n == kRecCap2) { cont = off; break; }
                    const Hdr h = read_header_range(blk, off, lo_b, bl);
                    const uint32_t st = classify(h, off, bl);
                    const bool bad = st != REVEL_REC_OK;
                    wl.off[n] = (uint16_t)off;
                    wl.s[n] = bad ? kNoRange : (uint16_t)(off + 6);
                    wl.em1[n] = bad ? kNoRange : (uint16_t)(off + kHeaderSize + h.len - 1u);
                    wl.acc[n] = 0;
                    ++n;
                    if (bad) break;
                    off += kHeaderSize + h.len;
                }
                wl.s[n] = wl.em1[n] = kNoRange;
                wl.nrec = n;
                wl.more_off = cont;
            }
            wave_lds_sync();
            const uint32_t nrec = wl.nrec;
            const uint32_t cont = wl.more_off;
            auto load_rec = [&](uint32_t k, uint32_t& s, uint32_t& e) {
                s = wl.s[k];  // k <= nrec: the sentinel ends every list
                e = uint32_t(wl.em1[k]) + 1u;
            };
            uint32_t lo = 0, hi = nrec;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (uint32_t(wl.em1[mid]) + 1u > cs) hi = mid; else lo = mid + 1;
            }
            uint32_t r = lo, s, e;
            load_rec(r, s, e);
            const bool active = cs < bl && r < nrec && s < ce;
            uint32_t state = 0;
            if (__any(active)) {
                if (!have_round0) load_round(cur, 0);
#pragma unroll 1
                for (int rr = 0; rr < 4; ++rr) {
                    if (rr < 3) load_round(nxt, rr + 1);
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const uint32_t p16 = cs + rr * 128 + j * 16;
                        // don't-care bytes before the next record, or inside one
                        const bool interior = (p16 + 16u <= s) || (p16 >= s && p16 + 16u < e);
                        if (BP != BP_MASK_NOVOTE && __all(interior)) {
                            // a record starting exactly here: the register may hold garbage
                            // from don't-care bytes (bytes of records outside this list batch)
                            state = p16 == s ? 0u : state;
                            state = absorb4<TM>(state, cur[j], L, tab);
                        } else if constexpr (BP != BP_BYTES) {
                            const uint32_t ws[4] = {cur[j].x, cur[j].y, cur[j].z, cur[j].w};
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                const uint32_t p = p16 + q * 4u;
                                // a record starts / ends inside [p, p+4) (at most one of each:
                                // the next type byte is >= 6 bytes past an end)
                                // words before the start (header / gap) leave the register at 0,
                                // so a record starting on a 16-B boundary can take the fast path
                                const uint32_t ds = s - p, de = e - p - 1u;
                                const bool pre = s >= p, en_in = de < 4u;
                                uint32_t keep = ds < 4u ? (0xFFFFFFFFu << (8u * ds)) : (pre ? 0u : 0xFFFFFFFFu);
                                keep &= en_in ? (0xFFFFFFFFu >> (8u * (3u - de))) : 0xFFFFFFFFu;
                                state = pre ? 0u : state;
                                state = absorb<TM>(state, ws[q] & keep, L, tab);
                                if (en_in) {
                                    atomicXor(&wl.acc[r], state);  // = raw * x^(8 (E - e))
                                    state = 0;
                                    ++r;
                                    load_rec(r, s, e);
                                }
                            }
                        } else {
                            const uint32_t ws[4] = {cur[j].x, cur[j].y, cur[j].z, cur[j].w};
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                const uint32_t p = p16 + q * 4u;
                                const uint32_t w = ws[q];
                                if (s >= p + 4u) {
                                    // gap word (or no record left): state is don't-care
                                } else if (e > p + 4u) {
                                    // record continues past this word; maybe starts in it
                                    if (s >= p) state = 0;
                                    const uint32_t lb = s > p ? s - p : 0u;
                                    state = absorb<TM>(state, w & (0xFFFFFFFFu << (8u * lb)), L, tab);
                                } else if (e > p) {
                                    // record ends in this word (and may start in it)
                                    if (s >= p) state = 0;
                                    const uint32_t lb = s > p ? s - p : 0u;
                                    const uint32_t hb = e - p;
                                    if (lb == 0 && hb == 4) {
                                        state = absorb<TM>(state, w, L, tab);
                                    } else {
                                        for (uint32_t t = lb; t < hb; ++t)
                                            state = byte_step_tm<TM>(state, (w >> (8u * t)) & 0xffu, L, tab);
                                    }
                                    atomicXor(&wl.acc[r], state);
                                    state = 0;
                                    ++r;
                                    load_rec(r, s, e);
                                }
                            }
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int j = 0; j < 8; ++j) cur[j] = nxt[j];
                }
                // record still open at the chunk end: shift its partial register to e
                if (cs < bl && r < nrec && s < ce && e > ce) {
                    const uint32_t to = BP == BP_BYTES ? e : (e + 3u) & ~3u;
                    atomicXor(&wl.acc[r], gf_mul(g_x8n_tab[to - ce], state));
                }
            }
            have_round0 = false;
            wave_lds_sync();
            for (uint32_t k = lane; k < nrec; k += 64) {
                const uint32_t off = wl.off[k];
                const Hdr h = read_header_range(blk, off, lo_b, bl);
                const uint32_t st = classify(h, off, bl);
                if constexpr (FRAME) {
                    if (st == REVEL_REC_OK) {
                        const uint32_t m = mask(record_raw<BP>(wl.acc[k], off, h.len) ^ g_init_xor_tab[h.len + 1u]);
                        uint8_t* hp = const_cast<uint8_t*>(blk) + off;
                        hp[0] = (uint8_t)m;
                        hp[1] = (uint8_t)(m >> 8);
                        hp[2] = (uint8_t)(m >> 16);
                        hp[3] = (uint8_t)(m >> 24);
                    }
                } else {
                    revel_record_result res;
                    res.file_offset = base_offset + base - lead + off;
                    res.length = h.len;
                    res.stored_crc = h.stored;
                    res.type = (uint8_t)h.type;
                    res.reserved[0] = res.reserved[1] = 0;
                    if (st == REVEL_REC_OK) {
                        res.computed_crc = mask(record_raw<BP>(wl.acc[k], off, h.len) ^ g_init_xor_tab[h.len + 1u]);
                        res.status = res.computed_crc == res.stored_crc ? REVEL_REC_OK : REVEL_REC_BAD_CHECKSUM;
                    } else {
                        res.computed_crc = 0;
                        res.status = (uint8_t)st;
                    }
                    out[out_base + k] = res;
                }
            }
            out_base += nrec;
            wave_lds_sync();
            if (cont == kNone) break;
            if (from_list) {
                ++lpass;
                const uint32_t k0 = lpass * kListPerBlock;
                ent = k0 + lane < nlist ? list_at<FRAME>(hlist, xlist, xstride, b, first_b, k0 + lane) : 0ull;
            } else {
                walk_from = cont;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// The blocks b0, b0 + step, ... < hi of one wave whose record count is above
// MINN (DENSE) or at most MINN (!DENSE): one vector load of
// 64 candidates' counts, then one set bit of the ballot per block.  Every
// member is wave-uniform.
// ---------------------------------------------------------------------------
// MARK (the one-pass experiment, tools/experiments/x_verify_fused.inc): a block whose header list slot
// kListCap holds kCapMarker qualifies too (walked and listed only, <= MINN records).
constexpr uint64_t kCapMarker = ~0ull;
template <bool DENSE, uint32_t MINN = kListPerBlock, bool MARK = false>
struct BlockSeq {
    uint32_t scan;  // first candidate not yet in mask (block indices fit 32 bits: 128 TiB images)
    uint64_t mask;  // qualifying blocks among scan - 64 step .. scan - step
    __device__ explicit BlockSeq(uint64_t b0) : scan((uint32_t)b0), mask(0) {}
    __device__ uint64_t next(const uint32_t* __restrict__ counts, uint64_t step, uint64_t hi,
                             const uint64_t* __restrict__ hlist = nullptr) {
        while (mask == 0) {
            if (scan >= hi) return hi;
            const uint64_t c = scan + uint64_t(lane_id()) * step;
            bool sel = c < hi && ((counts[c] > MINN) == DENSE);
            if constexpr (MARK) sel = sel || (c < hi && hlist[c * kListStride + kListCap] == kCapMarker);
            mask = __ballot(sel);
            scan += (uint32_t)(64u * step);
        }
        const uint32_t i = (uint32_t)__builtin_ctzll(mask);
        mask &= mask - 1u;
        return scan - 64u * step + uint64_t(i) * step;
    }
};

// ---------------------------------------------------------------------------
// Config C3, v3 (production, whole blocks): v2's per-block work, software-
// pipelined across the blocks a wave visits.  After a block's main loop the
// wave issues the finalizer's header loads, then the NEXT block's round-0
// data, header list entry, record count and output slot, and only then waits
// for the headers: the next block's loads are in flight while this block is
// finalized, so a block no longer pays three global round trips in series.
// Partial blocks (first/last) still go through k_verify_records2<.., BS_PARTIAL>.
// ---------------------------------------------------------------------------
enum BlockSel : int { SEL_ALL = 0, SEL_DENSE = 1, SEL_SPARSE = 2 };

// TQ (variant 9 experiment): round loads coalesced per quad -- lane 4q+p loads
// 16-B piece p of each 64-B half of the four chunks 4q..4q+3 (16 TCP accesses
// per wave instruction instead of 64) -- and a 4x4 transpose of the 16-B
// pieces inside the quad (two DPP butterfly stages) hands every lane its own
// chunk's bytes, so the per-lane CRC logic is unchanged.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_qperm(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
template <int K, int CTRL, int H = 1>
__device__ __forceinline__ void quad_stage(uint4* v, bool bit) {
#pragma unroll
    for (int h = 0; h < H; ++h) {
#pragma unroll
        for (int r0 = 0; r0 < 4; ++r0) {
            if (r0 & K) continue;
            uint32_t* a = reinterpret_cast<uint32_t*>(&v[4 * h + r0]);
            uint32_t* b = reinterpret_cast<uint32_t*>(&v[4 * h + (r0 | K)]);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                // bit clear: keep a, b <- partner's a; bit set: keep b, a <- partner's b
                const uint32_t recv = dpp_qperm<CTRL>(bit ? a[c] : b[c]);
                a[c] = bit ? recv : a[c];
                b[c] = bit ? b[c] : recv;
            }
        }
    }
}
template <int H = 1>
__device__ __forceinline__ void quad_transpose(uint4* v, uint32_t lane) {
    quad_stage<1, 0xB1, H>(v, (lane & 1u) != 0);  // quad_perm [1,0,3,2]
    quad_stage<2, 0x4E, H>(v, (lane & 2u) != 0);  // quad_perm [2,3,0,1]
}

template <bool FRAME, int SEL = SEL_ALL, bool TQ = false, bool R64 = false, bool TQ8 = false>
__global__ __launch_bounds__(kVerify2Threads) void k_verify_records3(const uint8_t* __restrict__ image, uint64_t nbytes,
                                                                     uint64_t base_offset,
                                                                     const uint32_t* __restrict__ first,
                                                                     revel_record_result* __restrict__ out,
                                                                     uint32_t lead,
                                                                     const uint64_t* __restrict__ hlist,
                                                                     const uint32_t* __restrict__ counts,
                                                                     const uint64_t* __restrict__ xlist,
                                                                     uint32_t xstride) {
    __shared__ uint32_t tab[32768];
    __shared__ VerifyWaveLds2 wl_all[kVerify2Threads / 64];
    fill_tables<TM_S4R>(tab);
    __syncthreads();
    VerifyWaveLds2& wl = wl_all[threadIdx.x >> 6];
    const LaneConst L = make_lane_const();
    const uint32_t lane = lane_id();
    const uint64_t vbytes = nbytes + lead;
    const uint64_t b_lo = lead ? 1u : 0u, b_hi = vbytes / kBlockSize;  // whole blocks [b_lo, b_hi)
    const uint64_t waves_per_wg = kVerify2Threads / 64;
    const uint64_t nwaves = gridDim.x * waves_per_wg;
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    // header lists: verify = the count pass's (records 0..63 in hlist, the
    // rest listed by k_list_overflow into the result slots: xlist = out,
    // stride 3 u64); FRAME = entry k of block b at xlist[first[b] + k]
    // (written by k_scatter_fragments)
    const bool use_list = counts != nullptr && (FRAME ? xlist != nullptr : hlist != nullptr);
    const uint32_t cs = lane * 512u, ce = cs + 512u;

    // wave-uniform block index (readfirstlane: the compiler cannot prove that
    // threadIdx.x >> 6 is uniform, and would keep the block arithmetic in VGPRs)
    const uint32_t wave_in_wg = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // SEL_SPARSE / SEL_DENSE: only the blocks with at most / more than
    // kListPerBlock records (the others go to k_verify_records_dense / v5)
    BlockSeq<SEL == SEL_DENSE> seq(b_lo + blockIdx.x * waves_per_wg + wave_in_wg);
    uint64_t b = SEL != SEL_ALL ? seq.next(counts, nwaves, b_hi) : b_lo + blockIdx.x * waves_per_wg + wave_in_wg;
    if (b >= b_hi) return;  // wave-uniform; no workgroup barrier follows
    constexpr int kRoundLoads = ((TQ && !TQ8) || R64) ? 4 : 8, kRounds = 32 / kRoundLoads;  // 16-B loads per round, rounds per chunk
    uint4 cur[8], nxt[8];
    uint32_t pf_count = kNone, pf_first = 0;
    uint64_t pf_hl = 0;
    auto load_round = [&](const uint8_t* blk, uint4* v, int rr, bool own, uint32_t cs_ref) {
        if constexpr (TQ && TQ8) {
            // 128-B rounds: lane 4q+p loads piece p of each 64-B half of chunks 4q..4q+3
            const uint8_t* p = blk + (lane & ~3u) * 512u + rr * 128 + (lane & 3u) * 16u;
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    v[4 * h + j] = ldg4_plain(reinterpret_cast<const uint4*>(p + j * 512 + h * 64));
        } else if constexpr (TQ) {
            // every lane loads for its quad (own / cs_ref unused: all chunks read)
            // 64-B rounds: the quad transpose needs registers the 128-B rounds do not have
            const uint8_t* p = blk + (lane & ~3u) * 512u + rr * 64 + (lane & 3u) * 16u;
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = ldg4_plain(reinterpret_cast<const uint4*>(p + j * 512));
        } else {
            const uint8_t* p = blk + (own ? cs : cs_ref) + rr * (16 * kRoundLoads);
#pragma unroll
            for (int j = 0; j < kRoundLoads; ++j) v[j] = ldg4_plain(reinterpret_cast<const uint4*>(p + j * 16));
        }
    };
    // header list first: the list is needed before the data (loads return in order)
    auto prefetch = [&](uint64_t nb) {
        if (use_list) {
            pf_count = counts[nb];
            if constexpr (FRAME) {
                pf_first = first[nb];
                pf_hl = lane < pf_count ? xlist[uint64_t(pf_first) + lane] : 0ull;
            } else {
                pf_hl = hlist[nb * kListStride + lane];
            }
        }
        if constexpr (!FRAME) pf_first = first[nb];
        load_round(image + nb * kBlockSize - lead, cur, 0, true, 0u);
    };
    prefetch(b);
    while (b < b_hi) {
        const uint64_t base = b * kBlockSize;
        const uint8_t* blk = image + base - lead;
        const uint64_t bn = SEL != SEL_ALL ? seq.next(counts, nwaves, b_hi) : b + nwaves;
        const uint32_t nlist = pf_count;
        uint64_t ent = pf_hl;  // this lane's header-list entry of the current batch
        const uint32_t first_b = __builtin_amdgcn_readfirstlane(pf_first);
        uint32_t out_base = pf_first;
        uint32_t walk_from = 0;              // header walk (no list given)
        uint32_t lpass = 0, lpass_off = 0;   // list batches: records [128 lpass, +128), first header offset
        bool have_round0 = true;
        for (;;) {
            const bool from_list = use_list;
            if (from_list) {
                // headers come from the count pass (the first kListPerBlock) or
                // from k_list_overflow (the rest, in this block's result slots);
                // offsets by prefix sum; a batch is 128 records, two per lane
                // (entries lane and lane + 64); the finalizer reads the first
                // 64 headers back from LDS, the rest from the block
                const uint32_t k0 = lpass * kRecCap2;
                const uint32_t np = min(nlist - k0, kRecCap2);
                uint64_t ent_b = 0;
                if (np > 64u && k0 + 64u + lane < nlist)
                    ent_b = list_at<FRAME>(hlist, xlist, xstride, b, first_b, k0 + 64u + lane);
                const Hdr h = list_header(ent), hb = list_header(ent_b);
                const uint32_t sz = lane < np ? kHeaderSize + h.len : 0u;
                const uint32_t szb = lane + 64u < np ? kHeaderSize + hb.len : 0u;
                const uint32_t exa = wave_exclusive_sum(sz);
                const uint32_t off = lpass_off + exa;
                const uint32_t offb = lpass_off + __builtin_amdgcn_readlane(exa + sz, 63) + wave_exclusive_sum(szb);
                if (lane < np) {
                    const bool bad = classify(h, off, kBlockSize) != REVEL_REC_OK;
                    wl.off[lane] = (uint16_t)off;
                    wl.s[lane] = bad ? kNoRange : (uint16_t)(off + 6);
                    wl.em1[lane] = bad ? kNoRange : (uint16_t)(off + kHeaderSize + h.len - 1u);
                    wl.acc[lane] = 0;
                    wl.hstored[lane] = h.stored;
                    wl.hlt[lane] = h.len | (h.type << 16);
                }
                if (lane + 64u < np) {
                    const bool bad = classify(hb, offb, kBlockSize) != REVEL_REC_OK;
                    wl.off[lane + 64u] = (uint16_t)offb;
                    wl.s[lane + 64u] = bad ? kNoRange : (uint16_t)(offb + 6);
                    wl.em1[lane + 64u] = bad ? kNoRange : (uint16_t)(offb + kHeaderSize + hb.len - 1u);
                    wl.acc[lane + 64u] = 0;
                }
                if (lane == 0) {
                    wl.s[np] = wl.em1[np] = kNoRange;
                    wl.nrec = np;
                    wl.more_off = k0 + np < nlist ? 1u : kNone;
                }
                // header offset of the next batch
                lpass_off = np > 64u ? __builtin_amdgcn_readlane(offb + szb, np - 65u)
                                     : __builtin_amdgcn_readlane(off + sz, np - 1u);
            } else if (lane == 0) {
                uint32_t off = walk_from, n = 0, cont = kNone;
                while (kBlockSize - off >= kHeaderSize) {
                    if (n == kRecCap2) { cont = off; break; }
                    const Hdr h = read_header(blk, off, kBlockSize);
                    const uint32_t st = classify(h, off, kBlockSize);
                    const bool bad = st != REVEL_REC_OK;
                    wl.off[n] = (uint16_t)off;
                    wl.s[n] = bad ? kNoRange : (uint16_t)(off + 6);
                    wl.em1[n] = bad ? kNoRange : (uint16_t)(off + kHeaderSize + h.len - 1u);
                    wl.acc[n] = 0;
                    ++n;
                    if (bad) break;
                    off += kHeaderSize + h.len;
                }
                wl.s[n] = wl.em1[n] = kNoRange;
                wl.nrec = n;
                wl.more_off = cont;
            }
            wave_lds_sync();
            const uint32_t nrec = wl.nrec;
            const uint32_t cont = wl.more_off;
            auto load_rec = [&](uint32_t k, uint32_t& s, uint32_t& e) {
                s = wl.s[k];  // k <= nrec: the sentinel ends every list
                e = uint32_t(wl.em1[k]) + 1u;
            };
            uint32_t lo = 0, hi = nrec;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (uint32_t(wl.em1[mid]) + 1u > cs) hi = mid; else lo = mid + 1;
            }
            uint32_t r = lo, s, e;
            load_rec(r, s, e);
            const bool active = r < nrec && s < ce;
            uint32_t state = 0;
            const uint64_t act_mask = __ballot(active);
            if (act_mask) {
                // lanes with no record of this batch in their chunk load an
                // active lane's addresses instead (same lines, no traffic):
                // a block listed in several batches is not re-read whole
                const uint32_t cs_ref = (uint32_t)__builtin_ctzll(act_mask) * 512u;  // wave-uniform
                if (!have_round0) load_round(blk, cur, 0, active, cs_ref);
#pragma unroll 1
                for (int rr = 0; rr < kRounds; ++rr) {
                    // TQ8: transpose before the next round is issued (its 32 registers
                    // are not live yet: the transpose's temporaries fit)
                    if constexpr (TQ && TQ8) {
                        quad_transpose<2>(cur, lane);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    if (rr < kRounds - 1) load_round(blk, nxt, rr + 1, active, cs_ref);
                    __builtin_amdgcn_sched_barrier(0);
                    if constexpr (TQ && !TQ8) quad_transpose(cur, lane);
#pragma unroll
                    for (int j = 0; j < kRoundLoads; ++j) {
                        const uint32_t p16 = cs + rr * (16 * kRoundLoads) + j * 16;
                        // don't-care bytes before the next record, or inside one
                        const bool interior = (p16 + 16u <= s) || (p16 >= s && p16 + 16u < e);
                        if (__all(interior)) {
                            // a record starting exactly here: the register may hold garbage
                            // from don't-care bytes (bytes of records outside this list batch)
                            state = p16 == s ? 0u : state;
                            state = absorb4<TM_S4R>(state, cur[j], L, tab);
                        } else {
                            const uint32_t ws[4] = {cur[j].x, cur[j].y, cur[j].z, cur[j].w};
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                const uint32_t p = p16 + q * 4u;
                                const uint32_t w = ws[q];
                                if (s >= p + 4u) {
                                    // gap word (or no record left): state is don't-care
                                } else if (e > p + 4u) {
                                    // record continues past this word; maybe starts in it
                                    if (s >= p) state = 0;
                                    const uint32_t lb = s > p ? s - p : 0u;
                                    state = absorb<TM_S4R>(state, w & (0xFFFFFFFFu << (8u * lb)), L, tab);
                                } else if (e > p) {
                                    // record ends in this word (and may start in it)
                                    if (s >= p) state = 0;
                                    const uint32_t lb = s > p ? s - p : 0u;
                                    const uint32_t hb = e - p;
                                    if (lb == 0 && hb == 4) {
                                        state = absorb<TM_S4R>(state, w, L, tab);
                                    } else {
                                        for (uint32_t t = lb; t < hb; ++t)
                                            state = byte_step_s4r(state, (w >> (8u * t)) & 0xffu, L, tab);
                                    }
                                    atomicXor(&wl.acc[r], state);
                                    state = 0;
                                    ++r;
                                    load_rec(r, s, e);
                                }
                            }
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int j = 0; j < kRoundLoads; ++j) cur[j] = nxt[j];
                }
                // record still open at the chunk end: shift its partial register to e
                if (r < nrec && s < ce && e > ce) atomicXor(&wl.acc[r], gf_mul(g_x8n_tab[e - ce], state));
            }
            have_round0 = false;
            wave_lds_sync();
            // finalizer headers first, then the next block's loads, then wait
            const bool f0 = lane < nrec;
            const uint32_t off0 = f0 ? uint32_t(wl.off[lane]) : 0u;
            const Hdr h0 = from_list ? Hdr{wl.hstored[lane & (kListPerBlock - 1)], wl.hlt[lane & (kListPerBlock - 1)] & 0xFFFFu,
                                           wl.hlt[lane & (kListPerBlock - 1)] >> 16}
                                     : read_header(blk, off0, kBlockSize);
            if (cont == kNone && bn < b_hi) prefetch(bn);
            for (uint32_t k = lane; k < nrec; k += 64) {
                const uint32_t off = k == lane ? off0 : uint32_t(wl.off[k]);
                const Hdr h = k == lane ? h0 : read_header(blk, off, kBlockSize);
                const uint32_t st = classify(h, off, kBlockSize);
                if constexpr (FRAME) {
                    if (st == REVEL_REC_OK) {
                        const uint32_t m = mask(wl.acc[k] ^ g_init_xor_tab[h.len + 1u]);
                        uint8_t* hp = const_cast<uint8_t*>(blk) + off;
                        hp[0] = (uint8_t)m;
                        hp[1] = (uint8_t)(m >> 8);
                        hp[2] = (uint8_t)(m >> 16);
                        hp[3] = (uint8_t)(m >> 24);
                    }
                } else {
                    revel_record_result res;
                    res.file_offset = base_offset + base - lead + off;
                    res.length = h.len;
                    res.stored_crc = h.stored;
                    res.type = (uint8_t)h.type;
                    res.reserved[0] = res.reserved[1] = 0;
                    if (st == REVEL_REC_OK) {
                        res.computed_crc = mask(wl.acc[k] ^ g_init_xor_tab[h.len + 1u]);
                        res.status = res.computed_crc == res.stored_crc ? REVEL_REC_OK : REVEL_REC_BAD_CHECKSUM;
                    } else {
                        res.computed_crc = 0;
                        res.status = (uint8_t)st;
                    }
                    out[out_base + k] = res;
                }
            }
            out_base += nrec;
            wave_lds_sync();
            if (cont == kNone) break;
            if (from_list) {
                ++lpass;
                const uint32_t k0 = lpass * kRecCap2;
                ent = k0 + lane < nlist ? list_at<FRAME>(hlist, xlist, xstride, b, first_b, k0 + lane) : 0ull;
            } else {
                walk_from = cont;
            }
        }
        b = bn;
    }
}


#include "verify_dense.inc"
#include "verify_rows.inc"

// Header-list entries of records kListCap.. of the blocks that have more
// (small-record logs: a 131-B record gives ~250 per block), one lane per block,
// for the verify paths that do not order blocks (the split path walks them in
// k_order_hist).  Entry k of block b goes into the first 8 bytes of its own
// 24-byte result slot out[first[b] + k]: the verify pass that covers record k
// reads it before it writes the result there.
__global__ void k_list_overflow(const uint8_t* __restrict__ image, uint64_t nbytes, const uint32_t* __restrict__ counts,
                                const uint32_t* __restrict__ first, const uint64_t* __restrict__ hlist,
                                revel_record_result* __restrict__ out) {
    const OverflowArgs ov{image, nbytes, first, hlist, out};
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < nblocks;
         b += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t n = counts[b];
        if (n > kListCap) list_overflow_block(ov, b, n);
    }
}
#ifndef REVEL_ROWS_RING
#define REVEL_ROWS_RING 8
#endif
constexpr int kRowsRing = REVEL_ROWS_RING;  // rows in flight per wave in k_verify_rows (8 or 16)
#ifndef REVEL_ROWS_DIAG
#define REVEL_ROWS_DIAG 0  // timing probes only (k_verify_rows' DIAG bits; wrong results when != 0)
#endif

// ---------------------------------------------------------------------------
// Device append framing, step 1: scatter fragments (payload bytes + length
// and type header bytes, CRC left zero) and zero the block trailers.  The
// layout comes from the host (frame_layout()).
// ---------------------------------------------------------------------------
// FPG = fragments per 8-lane group and wave visit: 3 for small-record
// batches, 1 when fragments average over 1 KiB (whole-wave copies then get
// more waves instead of longer visits)
template <uint32_t kScatterFpg>
__global__ void k_scatter_fragments(const uint8_t* __restrict__ payloads, const revel::FragDesc* __restrict__ frags,
                                    uint64_t nfrags, uint8_t* __restrict__ image, uint64_t* __restrict__ xlist) {
    // 8 FPG fragments per wave visit, FPG per 8-lane group (fragment base +
    // 8 j + grp): payloads of at most kTinyCopy bytes are copied with all of
    // the group's loads issued before any store (the copy is latency-bound:
    // profiles/r1s3_pmc_batches_summary.txt), up to kSmallFragment bytes by
    // the group one after another, larger ones by the whole wave
    constexpr uint32_t kSmallFragment = 1024;
    constexpr uint64_t kVisit = 8u * kScatterFpg;
    const uint32_t lane = lane_id(), grp = lane >> 3, gl = lane & 7u;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t w0 = blockIdx.x * (uint64_t)(blockDim.x / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // descriptors one visit ahead (clamped loads: no branch around a load)
    revel::FragDesc dn[kScatterFpg];
    auto fetch = [&](uint64_t base) {
#pragma unroll
        for (uint32_t j = 0; j < kScatterFpg; ++j) {
            const uint64_t k = base + 8u * j + grp;
            dn[j] = frags[k < nfrags ? k : nfrags - 1];
        }
    };
    if (w0 * kVisit < nfrags) fetch(w0 * kVisit);
    for (uint64_t base = w0 * kVisit; base < nfrags; base += waves * kVisit) {
        revel::FragDesc d[kScatterFpg];
#pragma unroll
        for (uint32_t j = 0; j < kScatterFpg; ++j) d[j] = dn[j];
        if (base + waves * kVisit < nfrags) fetch(base + waves * kVisit);
        bool live[kScatterFpg], pay[kScatterFpg];
        TinyCopy c[kScatterFpg];
#pragma unroll
        for (uint32_t j = 0; j < kScatterFpg; ++j) {
            live[j] = base + 8u * j + grp < nfrags;
            pay[j] = live[j] && d[j].type != revel::kTrailer;
            const bool tiny = pay[j] && d[j].len <= kTinyCopy;
            tiny_load(payloads + d[j].src, image + d[j].dst + kHeaderSize, tiny ? d[j].len : 0u, gl, image, c[j]);
        }
#pragma unroll
        for (uint32_t j = 0; j < kScatterFpg; ++j) {
            const uint64_t f = base + 8u * j + grp;
            uint8_t* dst = image + d[j].dst;
            if (live[j]) {
                if (d[j].type == revel::kTrailer) {
                    if (gl < d[j].len) dst[gl] = 0;  // a trailer is < 7 bytes
                } else if (gl < kHeaderSize) {
                    const uint32_t hv = gl < 4 ? 0u : gl == 4 ? (d[j].len & 0xffu) : gl == 5 ? (d[j].len >> 8) : d[j].type;
                    dst[gl] = (uint8_t)hv;
                    // header-list entry of this record for the CRC pass (CRC still 0)
                    if (gl == 0 && xlist) xlist[f] = list_entry(Hdr{0u, d[j].len, d[j].type});
                }
            }
            if (pay[j] && d[j].len <= kTinyCopy) tiny_store(payloads + d[j].src, dst + kHeaderSize, d[j].len, gl, c[j]);
        }
#pragma unroll
        for (uint32_t j = 0; j < kScatterFpg; ++j) {
            const bool small = pay[j] && d[j].len > kTinyCopy && d[j].len <= kSmallFragment;
            if (small) group_copy<8>(payloads + d[j].src, image + d[j].dst + kHeaderSize, d[j].len, gl);
            uint64_t big = __ballot(pay[j] && d[j].len > kSmallFragment && gl == 0);
            while (big) {
                const uint32_t l = (uint32_t)__builtin_ctzll(big);
                big &= big - 1;
                const uint64_t so = __shfl(d[j].src, l, 64), dd = __shfl(d[j].dst, l, 64);
                const uint32_t ln = __shfl(d[j].len, l, 64);
                group_copy<64>(payloads + so, image + dd + kHeaderSize, ln, lane);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Per-window verdict summaries for the end-to-end replay: units, bad units and
// the smallest bad file offset (summary[0..2]; reset by the host to 0,0,~0).
// ---------------------------------------------------------------------------
__global__ void k_summary_records(const revel_record_result* __restrict__ res, const uint32_t* __restrict__ first,
                                  const uint32_t* __restrict__ counts, uint64_t nblocks,
                                  unsigned long long* __restrict__ summary) {
    const uint64_t total = uint64_t(first[nblocks - 1]) + counts[nblocks - 1];
    unsigned long long bad = 0, first_bad = ~0ull;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        if (res[i].status != REVEL_REC_OK) {
            ++bad;
            first_bad = min(first_bad, (unsigned long long)res[i].file_offset);
        }
    }
    if (bad) {
        atomicAdd(&summary[1], bad);
        atomicMin(&summary[2], first_bad);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&summary[0], (unsigned long long)total);
}

__global__ void k_summary_blocks(const uint8_t* __restrict__ ok, uint64_t nblocks, uint64_t base_offset,
                                 unsigned long long* __restrict__ summary) {
    unsigned long long bad = 0, first_bad = ~0ull;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nblocks; i += (uint64_t)gridDim.x * blockDim.x) {
        if (!ok[i]) {
            ++bad;
            first_bad = min(first_bad, (unsigned long long)(base_offset + i * kBlockSize));
        }
    }
    if (bad) {
        atomicAdd(&summary[1], bad);
        atomicMin(&summary[2], first_bad);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&summary[0], (unsigned long long)nblocks);
}

}  // namespace

namespace revel {
hipError_t count_records(const DeviceInfo& di, const void* d_image, uint64_t nbytes, uint32_t* d_counts,
                         uint64_t* d_hlist, hipStream_t st, uint32_t* d_wsums) {
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    // one lane per block: every header chain walks concurrently
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>(1u << 20, (nblocks + 63) / 64));
    hipLaunchKernelGGL(k_count_records, dim3((uint32_t)grid), dim3(64), 0, st,
                       static_cast<const uint8_t*>(d_image), nbytes, d_counts, d_hlist, d_wsums);
    return hipGetLastError();
}

uint64_t count_wave_sums(uint64_t nblocks) { return (nblocks + 63) / 64; }

template <typename T>
static hipError_t exclusive_scan_t(const T* d_in, T* d_out, uint64_t n, T* d_tile_scratch, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint64_t tiles = (n + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(k_tile_sums<T>, dim3((uint32_t)tiles), dim3(256), 0, st, d_in, n, d_tile_scratch);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_scan_apply<T>, dim3((uint32_t)tiles), dim3(256), 0, st, d_in, n, d_tile_scratch, d_out);
    return hipGetLastError();
}

hipError_t exclusive_scan_u32(const DeviceInfo&, const uint32_t* d_in, uint32_t* d_out, uint64_t n,
                              uint32_t* d_tile_scratch, hipStream_t st) {
    return exclusive_scan_t<uint32_t>(d_in, d_out, n, d_tile_scratch, st);
}

hipError_t exclusive_scan_u64(const DeviceInfo&, const uint64_t* d_in, uint64_t* d_out, uint64_t n,
                              uint64_t* d_tile_scratch, hipStream_t st) {
    return exclusive_scan_t<uint64_t>(d_in, d_out, n, d_tile_scratch, st);
}

uint64_t scan_scratch_words(uint64_t n) { return (n + kScanTile - 1) / kScanTile; }

uint64_t hlist_words(uint64_t nblocks) { return nblocks * kListStride + (nblocks + kBlockListAux + 1) / 2 + 1; }

// One-time per device (per thread): the x^(8d) / init_xor(d) tables.
static hipError_t ensure_len_tables(const DeviceInfo& di, hipStream_t st) {
    static thread_local int inited_dev = -1;
    if (inited_dev != di.device) {
        hipLaunchKernelGGL(k_init_len_tables, dim3(64), dim3(256), 0, st);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        inited_dev = di.device;
    }
    return hipSuccess;
}

// Whole blocks on `grid` workgroups, then (only if there is one) the partial
// first/last block on one more workgroup, same stream.
// Production: pipelined whole-block kernel + the partial blocks on one workgroup.
template <bool FRAME>
static hipError_t launch_verify3(uint64_t grid, bool partial, const uint8_t* img, uint64_t nbytes,
                                 uint64_t base_offset, const uint32_t* d_first, revel_record_result* d_out,
                                 uint32_t lead, const uint64_t* hl, const uint32_t* d_counts, hipStream_t st,
                                 const uint64_t* xlist = nullptr, uint32_t xstride = 1) {
    if (!FRAME) {  // entries past the first 64 of a block: in the result slots
        xlist = reinterpret_cast<const uint64_t*>(d_out);
        xstride = sizeof(revel_record_result) / 8;
    }
    hipLaunchKernelGGL((k_verify_records3<FRAME>), dim3((uint32_t)grid), dim3(kVerify2Threads), 0, st, img, nbytes,
                       base_offset, d_first, d_out, lead, hl, d_counts, xlist, xstride);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !partial) return e;
    // <= 2 partial blocks: one single-wave workgroup each, 4 KiB unreplicated tables
    // (a 128 KiB table fill and one latency-bound wave cost ~50 us per launch)
    hipLaunchKernelGGL((k_verify_records2<FRAME, BP_BYTES, BS_PARTIAL, TM_S4, 64>), dim3(2), dim3(64), 0, st, img,
                       nbytes, base_offset, d_first, d_out, lead, hl, d_counts, xlist, xstride);
    return hipGetLastError();
}

// The blocks the sparse-block kernels leave: every block with more than
// kListPerBlock records (partial first / last ones too) through
// k_verify_records_dense, then the sparse partial blocks through the
// single-wave verify2 launch.  Each kernel skips the others' blocks by count.
template <bool FRAME>
static hipError_t launch_dense_and_partial(const DeviceInfo& di, const uint8_t* img, uint64_t nbytes,
                                           uint64_t base_offset, const uint32_t* d_first, revel_record_result* d_out,
                                           uint32_t lead, const uint64_t* hl, const uint32_t* d_counts,
                                           const uint64_t* xl, uint32_t xs, hipStream_t st,
                                           const uint32_t* dense_whole = nullptr, bool tail_in_rows = false) {
    const uint64_t vbytes = nbytes + lead;
    const uint64_t nblocks = (vbytes + kBlockSize - 1) / kBlockSize;
    const uint64_t waves = kDenseThreads / 64;
    const uint32_t grid =
        (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu, (nblocks + waves - 1) / waves));
    if constexpr (!FRAME) {
        if (lead == 0) {  // verify of a whole image
            // the aligned-word-stream kernel over every dense block (round 4)
            hipLaunchKernelGGL(k_verify_records_dense2<>, dim3(grid), dim3(kDenseThreads), 0, st, img, nbytes,
                               base_offset, d_first, d_out, hl, d_counts, dense_whole);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess || vbytes % kBlockSize == 0 || tail_in_rows) return e;
            hipLaunchKernelGGL((k_verify_records2<FRAME, BP_BYTES, BS_PARTIAL, TM_S4, 64, true>), dim3(2), dim3(64), 0,
                               st, img, nbytes, base_offset, d_first, d_out, lead, hl, d_counts, xl, xs, 0u);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL(k_verify_records_dense<FRAME>, dim3(grid), dim3(kDenseThreads), 0, st, img, nbytes, base_offset,
                       d_first, d_out, lead, hl, d_counts, xl, xs, dense_whole);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || (lead == 0 && (vbytes % kBlockSize == 0 || tail_in_rows))) return e;
    hipLaunchKernelGGL((k_verify_records2<FRAME, BP_BYTES, BS_PARTIAL, TM_S4, 64, true>), dim3(2), dim3(64), 0, st, img,
                       nbytes, base_offset, d_first, d_out, lead, hl, d_counts, xl, xs, tail_in_rows ? 1u : 0u);
    return hipGetLastError();
}

// Verify (or FRAME: append framing) split by block density, from the
// per-block record counts.  Production (ROWS): the whole blocks with
// 1..kListPerBlock records are listed (count-sorted: k_scan_order, or
// launch_block_order) and verified by
// k_verify_rows; !ROWS = v3 over those blocks (experiments only, with its
// TQ / R64 / TQ8 load shapes).  Lists: verify = hlist + overflow entries in the
// result slots (xlist = out, 3 u64 apart); FRAME = framing list.
template <bool FRAME, bool ROWS = true, bool TQ = false, bool R64 = false, bool TQ8 = false, int ROWS_RING = kRowsRing>
static hipError_t launch_verify_split(const DeviceInfo& di, const uint8_t* img, uint64_t nbytes, uint64_t base_offset,
                                      const uint32_t* d_first, revel_record_result* d_out, uint32_t lead,
                                      const uint64_t* hl, const uint32_t* d_counts, const uint64_t* xl, uint32_t xs,
                                      hipStream_t st, uint32_t* d_blist = nullptr, const OverflowArgs* ov = nullptr,
                                      bool list_ready = false) {
    const uint64_t vbytes = nbytes + lead;
    const uint64_t b_lo = lead ? 1u : 0u;
    uint64_t b_hi = vbytes / kBlockSize;
    const uint32_t* dense_whole = nullptr;  // counted by k_order_hist when it runs
    // A partial tail block (not also the lead block) joins the rows kernel's
    // list when its 16-B groups are image-aligned: one single-wave launch fewer
    // (~50 us of latency-bound walk per verify, profiles/r2_s4_partial_tail.txt).
    const uint32_t tail_bl = (uint32_t)(vbytes % kBlockSize);
    const bool tail_in_rows = ROWS && tail_bl != 0 && b_hi >= b_lo && lead % 16u == 0;
    const uint32_t tail_block = tail_in_rows ? (uint32_t)b_hi : 0xFFFFFFFFu;
    if (tail_in_rows) ++b_hi;
    if (b_hi > b_lo) {
        if constexpr (ROWS) {
            // qualifying blocks listed first, most records first (block_order)
            // k_verify_rows' per-workgroup item counters: the block order's
            // histogram rows (aux[3..], dead once the list is built; each
            // workgroup zeroes its own at start)
            uint32_t* const cursor = d_blist + 3;
            if (!list_ready) {
                hipError_t e = launch_block_order(di, d_counts, (uint32_t)b_lo, (uint32_t)b_hi, d_blist, st);
                if (e != hipSuccess) return e;
            }
            hipLaunchKernelGGL((k_verify_rows<FRAME, ROWS_RING, kRowsThreads, FRAME ? 0 : REVEL_ROWS_DIAG>),
                               dim3((uint32_t)std::max(1, di.num_cu)), dim3(kRowsThreads), 0, st,
                               img, base_offset, d_first, d_out, lead, hl, d_counts, xl, d_blist + kBlockListAux,
                               d_blist, tail_block, tail_in_rows ? tail_bl : (uint32_t)kBlockSize,
                               ov ? *ov : OverflowArgs{}, kRowsDyn ? cursor : nullptr);
            dense_whole = d_blist + 1;
            if constexpr (!FRAME) {
                hipError_t e = launch_expand_rows(di, base_offset, lead, d_first, d_out, hl, d_counts, (uint32_t)b_lo,
                                                  (uint32_t)b_hi, tail_block, tail_in_rows ? tail_bl : (uint32_t)kBlockSize,
                                                  st);
                if (e != hipSuccess) return e;
            }
        } else {
            const uint64_t waves = kVerify2Threads / 64;
            const uint32_t grid = (uint32_t)std::max<uint64_t>(
                1, std::min<uint64_t>((uint64_t)di.num_cu, (b_hi - b_lo + waves - 1) / waves));
            hipLaunchKernelGGL((k_verify_records3<FRAME, SEL_SPARSE, TQ, R64, TQ8>), dim3(grid),
                               dim3(kVerify2Threads), 0, st, img, nbytes, base_offset, d_first, d_out, lead, hl,
                               d_counts, xl, xs);
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return launch_dense_and_partial<FRAME>(di, img, nbytes, base_offset, d_first, d_out, lead, hl, d_counts, xl, xs, st,
                                           dense_whole, tail_in_rows);
}

// the dense kernel reads aligned 16 B relative to the image start
static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// The qualifying-block list of verify lives after the header lists (hlist_words).
static uint32_t* block_list(const uint64_t* hl, uint64_t nblocks) {
    return reinterpret_cast<uint32_t*>(const_cast<uint64_t*>(hl) + nblocks * kListStride);
}

// Production verify paths (test hook `path`): 0 = production -- with the
// count pass's header lists and a 16-B aligned image, the density split
// (k_verify_rows + dense + partial), else v3 over every block; 1 = v3 forced
// to walk the headers itself (a verify without its count pass); 2 = v3 with
// the header lists (the unaligned-image path).  Experiment arms live in
// tools/experiments (x_records.hip).
hipError_t verify_records_path(const DeviceInfo& di, int path, const void* d_image, uint64_t nbytes,
                               uint64_t base_offset, const uint32_t* d_first, revel_record_result* d_out,
                               const uint64_t* d_hlist, const uint32_t* d_counts, hipStream_t st, bool list_ready) {
    if (path < 0 || path > 2) return hipErrorInvalidValue;
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    hipError_t e0 = ensure_len_tables(di, st);
    if (e0 != hipSuccess) return e0;
    const uint64_t waves = kVerify2Threads / 64;
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu, (nblocks + waves - 1) / waves));
    const uint64_t* hl = path == 1 ? nullptr : d_hlist;
    const uint32_t* counts = path == 1 ? nullptr : d_counts;
    const uint8_t* img = static_cast<const uint8_t*>(d_image);
    const bool split = path == 0 && hl && counts && aligned16(img);
    if (split) {
        // k_verify_rows' prologue lists the headers of blocks with more than
        // kListCap records: every block (lead 0, the partial tail included)
        const OverflowArgs ov{img, nbytes, d_first, hl, d_out};
        return launch_verify_split<false>(di, img, nbytes, base_offset, d_first, d_out, 0u, hl, counts,
                                          reinterpret_cast<const uint64_t*>(d_out),
                                          (uint32_t)(sizeof(revel_record_result) / 8), st, block_list(hl, nblocks),
                                          &ov, list_ready);
    }
    if (hl && counts) {
        // list the headers of blocks with more than kListCap records
        const uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>(1u << 20, (nblocks + 63) / 64));
        hipLaunchKernelGGL(k_list_overflow, dim3((uint32_t)g), dim3(64), 0, st, img, nbytes, counts, d_first, hl,
                           d_out);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    const bool partial = nbytes % kBlockSize != 0;
    return launch_verify3<false>(grid, partial, img, nbytes, base_offset, d_first, d_out, 0u, hl, counts, st);
}

hipError_t verify_records(const DeviceInfo& di, const void* d_image, uint64_t nbytes, uint64_t base_offset,
                          const uint32_t* d_first, revel_record_result* d_out, const uint64_t* d_hlist,
                          const uint32_t* d_counts, hipStream_t st, bool list_ready) {
    return verify_records_path(di, 0, d_image, nbytes, base_offset, d_first, d_out, d_hlist, d_counts, st,
                               list_ready);
}

uint32_t* block_list_of(uint64_t* d_hlist, uint64_t nblocks) { return block_list(d_hlist, nblocks); }

// Sum of the per-block counts in 64 bits (the u32 record-index guard).
__global__ void k_sum_counts(const uint32_t* __restrict__ counts, uint64_t n, unsigned long long* __restrict__ total) {
    unsigned long long s = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        s += counts[i];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
    if (lane_id() == 0 && s) atomicAdd(total, s);
}

hipError_t total_records(const DeviceInfo& di, const uint32_t* d_counts, uint64_t nblocks,
                         unsigned long long* d_total, uint64_t* total, hipStream_t st) {
    hipError_t e = hipMemsetAsync(d_total, 0, sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)std::max(1, di.num_cu) * 4, (nblocks + 255) / 256));
    hipLaunchKernelGGL(k_sum_counts, dim3((uint32_t)grid), dim3(256), 0, st, d_counts, nblocks, d_total);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    unsigned long long h = 0;
    e = hipMemcpyAsync(&h, d_total, sizeof h, hipMemcpyDeviceToHost, st);
    if (e != hipSuccess) return e;
    e = hipStreamSynchronize(st);
    *total = h;
    return e;
}

// The workgroup size of k_count_hist / k_scan_order: 1024 (16 waves) puts
// every chunk slot of an image up to 4096 chunks (128 Ki blocks) on its own
// wave (512 lets a wave walk two chunks in turn once the image passes 2048
// chunks; bench.py's 4 GiB images have 2049).  Round 5, kernel traces over
// four alternating processes (profiles/r5/late/count_wide_trace/): 930 vs
// 950 us on small records, 58.3 vs 59.5 us on Zipf.
static uint32_t count_threads() { return kCountThreadsWide; }

// The grid of k_count_hist and k_scan_order (they must agree: the same
// workgroup visits the same chunks in both) and the chunk visiting mask.
static void count_grid(const DeviceInfo& di, uint64_t nblocks, uint32_t threads, uint32_t* grid, uint32_t* cmask) {
    const uint64_t nchunks = (nblocks + 63) / 64;
    const uint64_t waves = threads / 64;
    uint64_t p = 1;
    while (p < nchunks) p <<= 1;
    *cmask = (uint32_t)(p - 1);
    *grid = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>(std::min<uint64_t>(kOrderMaxWG, (uint64_t)std::max(1, di.num_cu)), (p + waves - 1) / waves));
}

hipError_t count_hist(const DeviceInfo& di, const void* d_image, uint64_t nbytes, uint32_t* d_counts,
                      uint64_t* d_hlist, uint32_t* d_wsums, uint32_t* d_aux, hipStream_t st) {
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    if (nblocks == 0) return hipSuccess;
    const uint32_t threads = count_threads();
    uint32_t grid, cmask;
    count_grid(di, nblocks, threads, &grid, &cmask);
    hipLaunchKernelGGL(k_count_hist<kCountThreadsWide>, dim3(grid), dim3(threads), 0, st,
                       static_cast<const uint8_t*>(d_image), nbytes, d_counts, d_hlist, d_wsums, d_aux, cmask);
    return hipGetLastError();
}

hipError_t scan_order(const DeviceInfo& di, uint64_t nbytes, const uint32_t* d_counts, const uint32_t* d_wsums,
                      uint32_t* d_first, uint32_t* d_aux, hipStream_t st) {
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    if (nblocks == 0) return hipSuccess;
    const uint32_t threads = count_threads();
    uint32_t grid, cmask;
    count_grid(di, nblocks, threads, &grid, &cmask);
    hipLaunchKernelGGL(k_scan_order<kCountThreadsWide>, dim3(grid), dim3(threads), 0, st, nbytes, d_counts, d_wsums,
                       d_first, d_aux, cmask);
    return hipGetLastError();
}

hipError_t summarize_records(const DeviceInfo& di, const revel_record_result* d_res, const uint32_t* d_first,
                             const uint32_t* d_counts, uint64_t nblocks, uint64_t* d_summary, hipStream_t st) {
    hipLaunchKernelGGL(k_summary_records, dim3((uint32_t)std::max(1, di.num_cu)), dim3(256), 0, st, d_res, d_first,
                       d_counts, nblocks, reinterpret_cast<unsigned long long*>(d_summary));
    return hipGetLastError();
}

hipError_t summarize_blocks(const DeviceInfo& di, const uint8_t* d_ok, uint64_t nblocks, uint64_t base_offset,
                            uint64_t* d_summary, hipStream_t st) {
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu, (nblocks + 255) / 256));
    hipLaunchKernelGGL(k_summary_blocks, dim3((uint32_t)grid), dim3(256), 0, st, d_ok, nblocks, base_offset,
                       reinterpret_cast<unsigned long long*>(d_summary));
    return hipGetLastError();
}

hipError_t frame_records(const DeviceInfo& di, const void* d_payloads, const FragDesc* d_frags, uint64_t nfrags,
                         void* d_image, uint64_t image_len, uint32_t lead, hipStream_t st, const uint32_t* d_counts,
                         const uint32_t* d_first, uint64_t* d_xlist, uint32_t* d_blist) {
    if (nfrags) {
        const bool small = image_len / nfrags <= 1024u;
        const uint64_t per_wg = small ? 96 : 32;  // 4 waves x 8 groups x FPG
        const uint64_t grid =
            std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu * 8, (nfrags + per_wg - 1) / per_wg));
        if (small)
            hipLaunchKernelGGL(k_scatter_fragments<3>, dim3((uint32_t)grid), dim3(256), 0, st,
                               static_cast<const uint8_t*>(d_payloads), d_frags, nfrags, static_cast<uint8_t*>(d_image),
                               d_xlist);
        else
            hipLaunchKernelGGL(k_scatter_fragments<1>, dim3((uint32_t)grid), dim3(256), 0, st,
                               static_cast<const uint8_t*>(d_payloads), d_frags, nfrags, static_cast<uint8_t*>(d_image),
                               d_xlist);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (image_len == 0) return hipSuccess;
    hipError_t e = ensure_len_tables(di, st);
    if (e != hipSuccess) return e;
    const uint64_t nblocks = (image_len + lead + kBlockSize - 1) / kBlockSize;
    const uint64_t waves = kVerify2Threads / 64;
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu, (nblocks + waves - 1) / waves));
    const bool partial = lead != 0 || (image_len + lead) % kBlockSize != 0;
    const bool lists = d_counts && d_first && d_xlist;
    if (lists && aligned16(d_image) && d_blist)
        return launch_verify_split<true>(
            di, static_cast<const uint8_t*>(d_image), image_len, 0ull, d_first, nullptr, lead, nullptr, d_counts,
            d_xlist, 1u, st, d_blist);
    return launch_verify3<true>(grid, partial, static_cast<const uint8_t*>(d_image), image_len, 0ull,
                                lists ? d_first : nullptr, nullptr, lead, nullptr, lists ? d_counts : nullptr, st,
                                lists ? d_xlist : nullptr, 1u);
}

}  // namespace revel

#ifdef REVEL_ROWS_WAVETIME
// timing probe builds only (tools/rows_wavetime.py): k_verify_rows' per-wave
// start / end times and block counts of its last launch
extern "C" int revel_debug_rows_wavetime(uint64_t* host, uint64_t n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rows_wavetime), n * sizeof(uint64_t), 0,
                                    hipMemcpyDeviceToHost);
}
#endif
