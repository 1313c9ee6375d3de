// k_blocks.hip -- config C2 kernels: one FULL record per 32 KiB block (production
// k_full_blocks3 and the experiment arms of crc_full_blocks_variant), the
// streaming-read ceiling and the synthetic block generator.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <type_traits>

#include "device_common.h"

using namespace revel;

namespace {
// ---------------------------------------------------------------------------
// Config C2: one FULL record per block.
// ---------------------------------------------------------------------------
template <int TM, int THREADS, int LM, bool FRAME>
__global__ __launch_bounds__(THREADS) void k_full_blocks(const uint8_t* __restrict__ blocks, uint64_t nblocks,
                                                         uint32_t* __restrict__ masked_out,
                                                         uint8_t* __restrict__ ok_out, uint8_t* __restrict__ frame_dst) {
    __shared__ uint32_t tab[TableCfg<TM>::bytes / 4];
    constexpr int kStageWaves = LM == LM_STAGED ? THREADS / 64 : 1;
    __shared__ uint4 stage_all[kStageWaves][LM == LM_STAGED ? 512 : 1];
    uint4* stage = stage_all[LM == LM_STAGED ? (threadIdx.x >> 6) : 0];
    fill_tables<TM>(tab);
    __syncthreads();
    const LaneConst L = make_lane_const();
    const uint32_t my_shift = c_lane_shift.c[lane_id()];
    const uint64_t waves_per_wg = THREADS / 64;
    const uint64_t gwave = blockIdx.x * waves_per_wg + (threadIdx.x >> 6);
    const uint64_t nwaves = gridDim.x * waves_per_wg;
    for (uint64_t b = gwave; b < nblocks; b += nwaves) {
        const uint8_t* blk = blocks + b * kBlockSize;
        uint4 hdr;
        uint32_t r = full_block_lane_crc<TM, LM>(blk, L, tab, stage, &hdr, FRAME);
        r = xor_reduce_wave(gf_mul(my_shift, r));
        const uint32_t masked = mask(r ^ kFullInitXor);
        if (lane_id() == 0) {
            if constexpr (FRAME) {
                // header [mask(crc) LE][len LE16][type]; byte 7 is payload.
                uint2 h;
                h.x = masked;
                h.y = (hdr.y & 0xFF000000u) | (uint32_t(kFullTypeByte) << 16) | kFullPayload;
                *reinterpret_cast<uint2*>(frame_dst + b * kBlockSize) = h;
            } else {
                masked_out[b] = masked;
                if (ok_out) {
                    const bool ok = (hdr.x == masked) && ((hdr.y & 0xFFFFu) == kFullPayload) &&
                                    (((hdr.y >> 16) & 0xFFu) == kFullTypeByte);
                    ok_out[b] = ok ? 1 : 0;
                }
            }
        }
    }
}

// Read-only streaming ceiling with the same grid and block assignment:
// coalesced 16 B/lane loads of the whole block, xor-folded, 4 B written.
template <int THREADS, bool NT = true>
__global__ __launch_bounds__(THREADS) void k_stream_ceiling(const uint8_t* __restrict__ blocks, uint64_t nblocks,
                                                            uint32_t* __restrict__ out) {
    const uint64_t waves_per_wg = THREADS / 64;
    const uint64_t gwave = blockIdx.x * waves_per_wg + (threadIdx.x >> 6);
    const uint64_t nwaves = gridDim.x * waves_per_wg;
    for (uint64_t b = gwave; b < nblocks; b += nwaves) {
        const uint4* p = reinterpret_cast<const uint4*>(blocks + b * kBlockSize) + lane_id();
        uint4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            uint4 v = NT ? ldg4(p + k * 64) : ldg4_plain(p + k * 64);
            acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
        }
        uint32_t r = xor_reduce_wave(acc.x ^ acc.y ^ acc.z ^ acc.w);
        if (lane_id() == 0) out[b] = r;
    }
}

// ---------------------------------------------------------------------------
// Synthetic C2 payloads: block b = splitmix64(seed ^ (first + b)) words.
// ---------------------------------------------------------------------------
__global__ void k_synth(uint64_t* __restrict__ dst, uint64_t nblocks, uint64_t seed, uint64_t first) {
    const uint64_t words_per_block = kBlockSize / 8;
    const uint64_t total = nblocks * words_per_block;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t b = i / words_per_block, w = i % words_per_block;
        uint64_t z = (seed ^ (first + b)) + (w + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        dst[i] = z ^ (z >> 31);
    }
}

// ---------------------------------------------------------------------------
// Config C2, v2: software-pipelined across blocks, CHAINS independent CRC
// chains per lane (lane i's 512-byte chunk split into CHAINS contiguous
// sub-chunks that advance in lockstep), and the GF(2) combine done either by
// a per-lane multiply (EPI_GFMUL) or by a table-driven shift tree (EPI_TREE).
// ---------------------------------------------------------------------------
enum Epilogue : int { EPI_GFMUL = 0, EPI_TREE = 1 };

// x^(8 * 256 * 2^L) mod P, L = 0..6: the shift applied at tree level L.
struct TreeShiftConsts {
    uint32_t c[7];
};
constexpr TreeShiftConsts make_tree_shift() {
    TreeShiftConsts t{};
    for (int L = 0; L < 7; ++L) t.c[L] = x8n(256ull << L);
    return t;
}
__constant__ TreeShiftConsts c_tree_shift = make_tree_shift();
constexpr uint32_t kShift256 = x8n(256);

// shift tables: level L, byte k, entry e at shtab[L*1024 + k*256 + e] =
// (e << 8k) * x^(8 * 256 * 2^L) mod P.
__device__ void fill_shift_tables(uint32_t* shtab, int levels) {
    for (uint32_t d = threadIdx.x; d < uint32_t(levels) * 1024u; d += blockDim.x) {
        const uint32_t L = d >> 10, k = (d >> 8) & 3u, e = d & 255u;
        shtab[d] = gf_mul(c_tree_shift.c[L], e << (8u * k));
    }
}

template <int L>
__device__ __forceinline__ uint32_t tree_shift(const uint32_t* shtab, uint32_t v) {
    const uint32_t* t = shtab + L * 1024;
    return (t[v & 0xffu] ^ t[256 + ((v >> 8) & 0xffu)]) ^ (t[512 + ((v >> 16) & 0xffu)] ^ t[768 + (v >> 24)]);
}

template <int TM, int THREADS, int CHAINS, int EPI, bool FRAME>
__global__ __launch_bounds__(THREADS) void k_full_blocks2(const uint8_t* __restrict__ blocks, uint64_t nblocks,
                                                          uint32_t* __restrict__ masked_out,
                                                          uint8_t* __restrict__ ok_out, uint8_t* __restrict__ frame_dst) {
    static_assert(CHAINS == 1 || CHAINS == 2, "chains");
    constexpr int kLevels = EPI == EPI_TREE ? 7 : 0;
    constexpr int kL0 = 1;  // lane-tree level lv uses table lv + 1 (shift 512 * 2^lv)
    __shared__ uint32_t tab[TableCfg<TM>::bytes / 4];
    __shared__ uint32_t shtab[kLevels ? kLevels * 1024 : 1];
    fill_tables<TM>(tab);
    if constexpr (kLevels > 0) fill_shift_tables(shtab, kLevels);
    __syncthreads();
    const LaneConst L = make_lane_const();
    const uint32_t lane = lane_id();
    const bool l0 = lane == 0;
    const uint32_t my_shift = c_lane_shift.c[lane];
    const uint64_t waves_per_wg = THREADS / 64;
    const uint64_t gwave = blockIdx.x * waves_per_wg + (threadIdx.x >> 6);
    const uint64_t nwaves = gridDim.x * waves_per_wg;

    // round r of block b: CHAINS=1 -> bytes [512i + 128r, +128);
    // CHAINS=2 -> chain A [512i + 64r, +64) in v[0..3], chain B [512i + 256 + 64r, +64) in v[4..7]
    auto load_round = [&](uint4* v, uint64_t b, int r) {
        const uint8_t* base = blocks + b * kBlockSize + lane * 512u;
        if constexpr (CHAINS == 1) {
            const uint4* p = reinterpret_cast<const uint4*>(base + r * 128);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = ldg4_plain(p + j);
        } else {
            const uint4* pa = reinterpret_cast<const uint4*>(base + r * 64);
            const uint4* pb = reinterpret_cast<const uint4*>(base + 256 + r * 64);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = ldg4_plain(pa + j);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[4 + j] = ldg4_plain(pb + j);
        }
    };

    uint4 cur[8], nxt[8];
    uint64_t b = gwave;
    if (b < nblocks) load_round(cur, b, 0);
    for (; b < nblocks; b += nwaves) {
        uint32_t ca = 0, cb = 0;
        uint4 hdr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (r < 3) {
                load_round(nxt, b, r + 1);
            } else if (b + nwaves < nblocks) {
                load_round(nxt, b + nwaves, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            if (r == 0) zero_header_bytes(cur[0], l0, FRAME, &hdr);
            if constexpr (CHAINS == 1) {
#pragma unroll
                for (int j = 0; j < 8; ++j) ca = absorb4<TM>(ca, cur[j], L, tab);
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    ca = absorb4<TM>(ca, cur[j], L, tab);
                    cb = absorb4<TM>(cb, cur[4 + j], L, tab);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < 8; ++j) cur[j] = nxt[j];
        }
        // ---- combine: R(block) = XOR_i R_i * x^(8*512*(63-i)) ----
        uint32_t raw;
        if constexpr (EPI == EPI_GFMUL) {
            uint32_t v = CHAINS == 2 ? (gf_mul(kShift256, ca) ^ cb) : ca;
            raw = xor_reduce_wave(gf_mul(my_shift, v));
        } else {
            uint32_t v = ca;
            if constexpr (CHAINS == 2) v = tree_shift<0>(shtab, ca) ^ cb;
#pragma unroll
            for (int lv = 0; lv < 6; ++lv) {
                uint32_t sft;
                switch (lv) {  // table level = lane-tree level + kL0
                    case 0: sft = tree_shift<kL0 + 0>(shtab, v); break;
                    case 1: sft = tree_shift<kL0 + 1>(shtab, v); break;
                    case 2: sft = tree_shift<kL0 + 2>(shtab, v); break;
                    case 3: sft = tree_shift<kL0 + 3>(shtab, v); break;
                    case 4: sft = tree_shift<kL0 + 4>(shtab, v); break;
                    default: sft = tree_shift<kL0 + 5>(shtab, v); break;
                }
                const uint32_t up = __shfl_up(sft, 1u << lv, 64);
                const uint32_t m = (2u << lv) - 1u;
                v = ((lane & m) == m) ? (v ^ up) : v;
            }
            raw = __builtin_amdgcn_readlane(v, 63);
        }
        const uint32_t masked = mask(raw ^ kFullInitXor);
        if (l0) {
            if constexpr (FRAME) {
                uint2 h;
                h.x = masked;
                h.y = (hdr.y & 0xFF000000u) | (uint32_t(kFullTypeByte) << 16) | kFullPayload;
                *reinterpret_cast<uint2*>(frame_dst + b * kBlockSize) = h;
            } else {
                masked_out[b] = masked;
                if (ok_out) {
                    const bool ok = (hdr.x == masked) && ((hdr.y & 0xFFFFu) == kFullPayload) &&
                                    (((hdr.y >> 16) & 0xFFu) == kFullTypeByte);
                    ok_out[b] = ok ? 1 : 0;
                }
            }
        }
    }
}

template <int TM, int THREADS, int CHAINS, int EPI, bool FRAME>
hipError_t launch_full2(const DeviceInfo& di, const uint8_t* blocks, uint64_t n, uint32_t* masked, uint8_t* ok,
                        uint8_t* frame_dst, hipStream_t st) {
    auto kern = k_full_blocks2<TM, THREADS, CHAINS, EPI, FRAME>;
    const uint64_t wg_needed = (n + THREADS / 64 - 1) / (THREADS / 64);
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu, wg_needed));
    hipLaunchKernelGGL(kern, dim3((uint32_t)grid), dim3(THREADS), 0, st, blocks, n, masked, ok, frame_dst);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Config C2, v3: interleaved word streams with the gap folded into the tables.
//
// Stream s (s = 0..255) is the 32-bit words at byte offsets 4s + 1024k,
// k = 0..31; lane i owns streams 4i..4i+3, i.e. one 16-byte load per lane
// per 1 KiB: exactly the coalescing of a plain streaming read (1 KiB per
// wave instruction).  Consecutive words of a stream are 1024 bytes apart, so
// with tables T''m = x^(8*1020) * Tm the chain
//     U <- T''3[x0] ^ T''2[x1] ^ T''1[x2] ^ T''0[x3],   x = U ^ w
// absorbs a word AND the 1020 bytes of other streams' data that follow it in
// one step (shifting is linear, so it distributes over the table xor).  The
// four streams of a lane are four independent chains (ILP 4).  After its 32nd
// word, stream s stands at byte 32768 + 4s; the block register is
//     R = XOR_s  U_s * x^(-32 s)  mod P
// (x is invertible mod P since P(0) = 1), evaluated by an 8-level tree of
// inverse-shift tables: 2 levels inside the lane, 6 across lanes.
// ---------------------------------------------------------------------------
struct GapTables {
    uint32_t t[4][256];  // t[m][e] = x^(8*1020) * T_m[e]
};
constexpr GapTables make_gap_tables() {
    GapTables g{};
    const SliceTables st = make_slice_tables();
    const uint32_t c = x8n(1020);
    for (int m = 0; m < 4; ++m)
        for (int e = 0; e < 256; ++e) g.t[m][e] = multmodp(c, st.t[m][e]);
    return g;
}
__constant__ GapTables c_gap = make_gap_tables();

constexpr uint32_t pow_modp(uint32_t a, uint64_t n) {
    uint32_t r = 0x80000000u;
    while (n) {
        if (n & 1u) r = multmodp(r, a);
        a = multmodp(a, a);
        n >>= 1;
    }
    return r;
}
constexpr uint32_t kXInv = 0x05EC76F1u;  // x^-1 mod P, reflected
static_assert(multmodp(kXInv, 0x40000000u) == 0x80000000u, "x * x^-1 == 1");
// x^(-8 * 4 * 2^L): tree level L combines streams 2^L apart (4 * 2^L bytes)
struct InvTreeConsts {
    uint32_t c[8];
};
constexpr InvTreeConsts make_inv_tree() {
    InvTreeConsts t{};
    for (int L = 0; L < 8; ++L) t.c[L] = pow_modp(kXInv, 8ull * 4ull * (1ull << L));
    return t;
}
__constant__ InvTreeConsts c_inv_tree = make_inv_tree();
static_assert(multmodp(make_inv_tree().c[0], x8n(4)) == 0x80000000u, "inverse shift");

__device__ void fill_gap_tables(uint32_t* tab) {
    // S4R layout; byte0 -> T''3 (r0 h0), byte1 -> T''2 (r0 h1), byte2 -> T''1 (r1 h0), byte3 -> T''0 (r1 h1)
    for (uint32_t d = threadIdx.x; d < 32768u; d += blockDim.x) {
        const uint32_t r = d >> 14, e = (d >> 6) & 255u, h = (d >> 5) & 1u;
        tab[d] = c_gap.t[3 - (r * 2 + h)][e];
    }
}
__device__ void fill_inv_tree_tables(uint32_t* shtab) {
    for (uint32_t d = threadIdx.x; d < 8u * 1024u; d += blockDim.x) {
        const uint32_t L = d >> 10, k = (d >> 8) & 3u, e = d & 255u;
        shtab[d] = gf_mul(c_inv_tree.c[L], e << (8u * k));
    }
}

template <bool NT>
__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
    return NT ? ldg4(reinterpret_cast<const uint4*>(p)) : ldg4_plain(reinterpret_cast<const uint4*>(p));
}

// Block epilogue of the interleaved-stream kernels: R = XOR_s U_s x^(-32 s)
// by the 8-level inverse-shift tree (2 levels in-lane, 6 across lanes), then
// the masked CRC, the header check or the framed header.
template <bool FRAME>
__device__ __forceinline__ void finish_full_block(uint32_t u0, uint32_t u1, uint32_t u2, uint32_t u3, uint4 hdr,
                                                  uint64_t b, const uint32_t* shtab, uint32_t lane,
                                                  uint32_t* __restrict__ masked_out, uint8_t* __restrict__ ok_out,
                                                  uint8_t* __restrict__ frame_dst) {
    uint32_t v0 = u0 ^ tree_shift<0>(shtab, u1);
    uint32_t v1 = u2 ^ tree_shift<0>(shtab, u3);
    uint32_t v = v0 ^ tree_shift<1>(shtab, v1);
#pragma unroll
    for (int lv = 0; lv < 6; ++lv) {
        uint32_t t;
        switch (lv) {
            case 0: t = tree_shift<2>(shtab, v); break;
            case 1: t = tree_shift<3>(shtab, v); break;
            case 2: t = tree_shift<4>(shtab, v); break;
            case 3: t = tree_shift<5>(shtab, v); break;
            case 4: t = tree_shift<6>(shtab, v); break;
            default: t = tree_shift<7>(shtab, v); break;
        }
        const uint32_t dn = __shfl_down(t, 1u << lv, 64);
        const uint32_t m = (2u << lv) - 1u;
        v = ((lane & m) == 0u) ? (v ^ dn) : v;
    }
    const uint32_t raw = __builtin_amdgcn_readfirstlane(v);
    const uint32_t masked = mask(raw ^ kFullInitXor);
    if (lane == 0) {
        if constexpr (FRAME) {
            uint2 h;
            h.x = masked;
            h.y = (hdr.y & 0xFF000000u) | (uint32_t(kFullTypeByte) << 16) | kFullPayload;
            *reinterpret_cast<uint2*>(frame_dst + b * kBlockSize) = h;
        } else {
            masked_out[b] = masked;
            if (ok_out) {
                const bool ok = (hdr.x == masked) && ((hdr.y & 0xFFFFu) == kFullPayload) &&
                                (((hdr.y >> 16) & 0xFFu) == kFullTypeByte);
                ok_out[b] = ok ? 1 : 0;
            }
        }
    }
}

template <int THREADS, bool NT, bool FRAME, bool XS = false>
__global__ __launch_bounds__(THREADS) void k_full_blocks3(const uint8_t* __restrict__ blocks, uint64_t nblocks,
                                                          uint32_t* __restrict__ masked_out,
                                                          uint8_t* __restrict__ ok_out, uint8_t* __restrict__ frame_dst) {
    __shared__ uint32_t tab[32768];      // 128 KiB: T'' replicated 32x
    __shared__ uint32_t shtab[8 * 1024];  // 32 KiB: inverse-shift tree tables
    fill_gap_tables(tab);
    fill_inv_tree_tables(shtab);
    __syncthreads();
    const LaneConst L = make_lane_const();
    const uint32_t lane = lane_id();
    const bool l0 = lane == 0;
    const uint64_t waves_per_wg = THREADS / 64;
    const uint64_t gwave = blockIdx.x * waves_per_wg + (threadIdx.x >> 6);
    const uint64_t nwaves = gridDim.x * waves_per_wg;

    // round r (0..3) of block b: words of the 8 KiB [8192 r, +8192); lane i
    // loads 16 B at 1024 k + 16 i, k = 0..7
    auto load_round = [&](uint4* v, uint64_t b, int r) {
        const uint8_t* base = blocks + b * kBlockSize + r * 8192 + lane * 16u;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = ld16<NT>(base + k * 1024);
    };

    uint4 cur[8], nxt[8];
    uint64_t b = gwave;
    if (b < nblocks) load_round(cur, b, 0);
    for (; b < nblocks; b += nwaves) {
        uint32_t u0 = 0, u1 = 0, u2 = 0, u3 = 0;
        uint4 hdr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (r < 3) {
                load_round(nxt, b, r + 1);
            } else if (b + nwaves < nblocks) {
                load_round(nxt, b + nwaves, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            if (r == 0) {
                zero_header_bytes(cur[0], l0, FRAME, &hdr);
                if constexpr (XS) {
                    u0 = cur[0].x; u1 = cur[0].y; u2 = cur[0].z; u3 = cur[0].w;
                }
            }
            if constexpr (XS) {
                // u = crc ^ (word k); fold word k + 1 (next round's first, or 0 at the end)
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint4 wn = k < 7 ? cur[k + 1] : (r < 3 ? nxt[0] : make_uint4(0, 0, 0, 0));
                    u0 = step_x(u0, wn.x, L, tab);
                    u1 = step_x(u1, wn.y, L, tab);
                    u2 = step_x(u2, wn.z, L, tab);
                    u3 = step_x(u3, wn.w, L, tab);
                }
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    u0 = absorb<TM_S4R>(u0, cur[k].x, L, tab);
                    u1 = absorb<TM_S4R>(u1, cur[k].y, L, tab);
                    u2 = absorb<TM_S4R>(u2, cur[k].z, L, tab);
                    u3 = absorb<TM_S4R>(u3, cur[k].w, L, tab);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < 8; ++k) cur[k] = nxt[k];
        }
        finish_full_block<FRAME>(u0, u1, u2, u3, hdr, b, shtab, lane, masked_out, ok_out, frame_dst);
    }
}

template <int THREADS, bool NT, bool FRAME, bool XS = false>
hipError_t launch_full3(const DeviceInfo& di, const uint8_t* blocks, uint64_t n, uint32_t* masked, uint8_t* ok,
                        uint8_t* frame_dst, hipStream_t st) {
    auto kern = k_full_blocks3<THREADS, NT, FRAME, XS>;
    const uint64_t wg_needed = (n + THREADS / 64 - 1) / (THREADS / 64);
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu, wg_needed));
    hipLaunchKernelGGL(kern, dim3((uint32_t)grid), dim3(THREADS), 0, st, blocks, n, masked, ok, frame_dst);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Config C2, v4: v3's streams and x-state chains fed by a 16-slot load ring.
// Row g of a block (g = 0..31) is the 1 KiB [1024 g, +1024), 16 B per lane.
// v3 double-buffers whole 8 KiB rounds (cur / nxt), so while a round is folded
// only the next one is in flight.  Here the slot a row leaves is refilled at
// once with the row 16 ahead (into the next block at the end), so ~15 rows =
// 15 KiB per wave stay in flight with the same 64 VGPRs: HBM sees ~2x the
// bytes in flight per CU.  All loads are unconditional (rows past the last
// block re-read the last block), so the compiler's vmcnt counts stay exact.
// ---------------------------------------------------------------------------
template <int THREADS, bool FRAME>
__global__ __launch_bounds__(THREADS) void k_full_blocks4(const uint8_t* __restrict__ blocks, uint64_t nblocks,
                                                          uint32_t* __restrict__ masked_out,
                                                          uint8_t* __restrict__ ok_out, uint8_t* __restrict__ frame_dst) {
    __shared__ uint32_t tab[32768];      // 128 KiB: T'' replicated 32x
    __shared__ uint32_t shtab[8 * 1024];  // 32 KiB: inverse-shift tree tables
    fill_gap_tables(tab);
    fill_inv_tree_tables(shtab);
    __syncthreads();
    const LaneConst L = make_lane_const();
    const uint32_t lane = lane_id();
    const bool l0 = lane == 0;
    const uint64_t waves_per_wg = THREADS / 64;
    const uint64_t gwave = blockIdx.x * waves_per_wg + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nwaves = gridDim.x * waves_per_wg;
    if (gwave >= nblocks) return;
    const uint8_t* lane_base = blocks + lane * 16u;
    auto row = [&](uint64_t b, int g) {
        b = b < nblocks ? b : nblocks - 1;
        return ldg4(reinterpret_cast<const uint4*>(lane_base + b * kBlockSize + g * 1024));
    };
    uint4 ring[16];
#pragma unroll
    for (int g = 0; g < 16; ++g) ring[g] = row(gwave, g);
    for (uint64_t b = gwave; b < nblocks; b += nwaves) {
        uint32_t u0, u1, u2, u3;
        uint4 hdr;
#pragma unroll
        for (int g = 0; g < 32; ++g) {
            if (g == 0) {
                uint4 c = ring[0];
                zero_header_bytes(c, l0, FRAME, &hdr);
                u0 = c.x; u1 = c.y; u2 = c.z; u3 = c.w;
                ring[0] = row(b, 16);
            }
            // fold row g + 1 (0 after the last row): u = crc ^ (word g + 1)
            const uint4 wn = g < 31 ? ring[(g + 1) & 15] : make_uint4(0, 0, 0, 0);
            u0 = step_x(u0, wn.x, L, tab);
            u1 = step_x(u1, wn.y, L, tab);
            u2 = step_x(u2, wn.z, L, tab);
            u3 = step_x(u3, wn.w, L, tab);
            // row g + 1 has left its slot: refill with row g + 17
            if (g < 31) ring[(g + 1) & 15] = g + 17 < 32 ? row(b, g + 17) : row(b + nwaves, g + 17 - 32);
        }
        finish_full_block<FRAME>(u0, u1, u2, u3, hdr, b, shtab, lane, masked_out, ok_out, frame_dst);
    }
}

template <int THREADS, bool FRAME>
hipError_t launch_full4(const DeviceInfo& di, const uint8_t* blocks, uint64_t n, uint32_t* masked, uint8_t* ok,
                        uint8_t* frame_dst, hipStream_t st) {
    const uint64_t wg_needed = (n + THREADS / 64 - 1) / (THREADS / 64);
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu, wg_needed));
    hipLaunchKernelGGL((k_full_blocks4<THREADS, FRAME>), dim3((uint32_t)grid), dim3(THREADS), 0, st, blocks, n, masked,
                       ok, frame_dst);
    return hipGetLastError();
}

template <int TM, int THREADS, int LM, bool FRAME>
hipError_t launch_full(const DeviceInfo& di, int wg_per_cu, const uint8_t* blocks, uint64_t n, uint32_t* masked,
                       uint8_t* ok, uint8_t* frame_dst, hipStream_t st) {
    auto kern = k_full_blocks<TM, THREADS, LM, FRAME>;
    const uint64_t waves_needed = n;
    uint64_t grid = (uint64_t)di.num_cu * wg_per_cu;
    const uint64_t wg_needed = (waves_needed + THREADS / 64 - 1) / (THREADS / 64);
    grid = std::max<uint64_t>(1, std::min(grid, wg_needed));
    hipLaunchKernelGGL(kern, dim3((uint32_t)grid), dim3(THREADS), 0, st, blocks, n, masked, ok, frame_dst);
    return hipGetLastError();
}

template <int THREADS, bool NT>
hipError_t launch_stream(const DeviceInfo& di, int wg_per_cu, const uint8_t* b, uint64_t n, uint32_t* out,
                         hipStream_t st) {
    const uint64_t w = THREADS / 64;
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu * wg_per_cu, (n + w - 1) / w));
    hipLaunchKernelGGL((k_stream_ceiling<THREADS, NT>), dim3((uint32_t)grid), dim3(THREADS), 0, st, b, n, out);
    return hipGetLastError();
}

}  // namespace

namespace revel {
// Variant table used by the public entry point and by tools/variants.py.
hipError_t crc_full_blocks_variant(const DeviceInfo& di, int variant, const void* d_blocks, uint64_t n,
                                   uint32_t* d_masked, uint8_t* d_ok, hipStream_t st) {
    const uint8_t* b = static_cast<const uint8_t*>(d_blocks);
    switch (variant) {
        // production: v4 = v3 interleaved word streams (gap-folded tables, nt
        // loads) with x-state chains (3-input xors), fed by a 16-slot load ring
        case 0: return launch_full4<1024, false>(di, b, n, d_masked, d_ok, nullptr, st);
        case 9: return launch_full<TM_S4R, 1024, LM_DIRECT, false>(di, 1, b, n, d_masked, d_ok, nullptr, st);
        case 8: return launch_full<TM_S2R, 768, LM_STAGED, false>(di, 1, b, n, d_masked, d_ok, nullptr, st);
        // v2 (pipelined across blocks): chains x epilogue
        case 10: return launch_full2<TM_S4R, 1024, 1, EPI_GFMUL, false>(di, b, n, d_masked, d_ok, nullptr, st);
        case 11: return launch_full2<TM_S4R, 1024, 2, EPI_GFMUL, false>(di, b, n, d_masked, d_ok, nullptr, st);
        case 12: return launch_full2<TM_S4R, 1024, 1, EPI_TREE, false>(di, b, n, d_masked, d_ok, nullptr, st);
        case 13: return launch_full2<TM_S4R, 1024, 2, EPI_TREE, false>(di, b, n, d_masked, d_ok, nullptr, st);
        case 14: return launch_full2<TM_S2R, 1024, 2, EPI_TREE, false>(di, b, n, d_masked, d_ok, nullptr, st);
        // v3: interleaved word streams, gap folded into the tables
        case 20: return launch_full3<1024, true, false>(di, b, n, d_masked, d_ok, nullptr, st);
        case 21: return launch_full3<1024, false, false>(di, b, n, d_masked, d_ok, nullptr, st);
        // v3 with the x-state chain (3-input xors)
        case 22: return launch_full3<1024, true, false, true>(di, b, n, d_masked, d_ok, nullptr, st);
        // v4: v3 + x-state fed by a 16-slot load ring (~15 KiB in flight per wave) = production
        case 23: return launch_full4<1024, false>(di, b, n, d_masked, d_ok, nullptr, st);
        case 1: return launch_full<TM_S2R, 512, LM_STAGED, false>(di, 1, b, n, d_masked, d_ok, nullptr, st);
        case 2: return launch_full<TM_S4R, 256, LM_STAGED, false>(di, 1, b, n, d_masked, d_ok, nullptr, st);
        case 3: return launch_full<TM_S4, 1024, LM_STAGED, false>(di, 1, b, n, d_masked, d_ok, nullptr, st);
        case 4: return launch_full<TM_S2R, 512, LM_DIRECT, false>(di, 2, b, n, d_masked, d_ok, nullptr, st);
        case 5: return launch_full<TM_S4R, 1024, LM_DIRECT, false>(di, 1, b, n, d_masked, d_ok, nullptr, st);
        case 6: return launch_full<TM_S4, 512, LM_DIRECT, false>(di, 4, b, n, d_masked, d_ok, nullptr, st);
        case 7: return launch_full<TM_S2R, 512, LM_DIRECT_NT, false>(di, 2, b, n, d_masked, d_ok, nullptr, st);
        case 100: {
            const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu * 8, (n + 3) / 4));
            hipLaunchKernelGGL(k_stream_ceiling<256>, dim3((uint32_t)grid), dim3(256), 0, st, b, n, d_masked);
            return hipGetLastError();
        }
        // streaming-read ceiling shapes (experiment): plain loads; fewer / more waves per CU
        case 101: return launch_stream<256, false>(di, 8, b, n, d_masked, st);
        case 102: return launch_stream<256, true>(di, 4, b, n, d_masked, st);
        case 103: return launch_stream<256, true>(di, 2, b, n, d_masked, st);
        case 104: return launch_stream<1024, true>(di, 1, b, n, d_masked, st);
        case 105: return launch_stream<512, true>(di, 4, b, n, d_masked, st);
        case 106: return launch_stream<256, true>(di, 16, b, n, d_masked, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t frame_full_blocks(const DeviceInfo& di, void* d_blocks, uint64_t n, hipStream_t st) {
    uint8_t* b = static_cast<uint8_t*>(d_blocks);
    return launch_full4<1024, true>(di, b, n, nullptr, nullptr, b, st);
}

hipError_t synth_full_blocks(const DeviceInfo& di, void* d_blocks, uint64_t n, uint64_t seed, uint64_t first,
                             hipStream_t st) {
    const uint64_t words = n * (kBlockSize / 8);
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu * 16, (words + 255) / 256));
    hipLaunchKernelGGL(k_synth, dim3((uint32_t)grid), dim3(256), 0, st, static_cast<uint64_t*>(d_blocks), n, seed,
                       first);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return frame_full_blocks(di, d_blocks, n, st);
}

}  // namespace revel
