// x_blocks.hip -- config C2 EXPERIMENT arms (not part of librevel_wal.so).
//
// The kernels measured on the way to the production k_full_blocks4
// (revel_amd/csrc/k_blocks.hip): lane-owned 512-B chunks (v1, staged /
// direct / nontemporal loads), v2 (pipelined, 1-2 chains, GF-multiply or tree
// epilogue), v3 (interleaved word streams, double-buffered rounds, with and
// without x-state chains) and the streaming-read ceiling shapes.  Their results
// are in profiles/ (r1_variant_sweeps.txt, r1s2_*); DESIGN.md section 4.1 tells
// the story.  Built into tools/experiments/libexperiments.so by this directory's
// Makefile; tools/variants.py drives them.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <type_traits>

#include "device_common.h"

using namespace revel;

namespace {
// How a lane's 512-byte chunk reaches registers.
enum LoadMode : int {
    LM_DIRECT_NT = 0,     // lane loads its own chunk, nontemporal (64 lines per instruction)
    LM_DIRECT = 1,        // same, default cache policy
    LM_STAGED = 2,        // line-coalesced loads (8 whole lines per instruction) + LDS transpose
};

// Staging layout (one 8 KiB buffer per wave per round): piece t (16 B) of
// owner lane i sits in slot t*64 + (i ^ t).  ds_write_b128 by the loading
// lanes and ds_read_b128 by the owners are both bank-conflict-free.
__device__ __forceinline__ uint32_t stage_slot(uint32_t owner, uint32_t t) { return t * 64u + (owner ^ t); }

// Raw register of lane's 512-byte chunk of a full block (header bytes 0..5
// zeroed for lane 0, so the chunk set covers exactly block[6:32768)).
// Returns lane 0's first 16 bytes through *hdr.
template <int TM, int LM>
__device__ __forceinline__ uint32_t full_block_lane_crc(const uint8_t* blk, LaneConst L, const uint32_t* tab,
                                                        uint4* stage, uint4* hdr, bool force_type) {
    const uint32_t lane = lane_id();
    const bool l0 = lane == 0;
    uint32_t crc = 0;
    uint4 cur[8], nxt[8];
    // Round r covers bytes [512 i + 128 r, +128) of every lane i.
    auto load_round = [&](uint4* v, int r) {
        if constexpr (LM == LM_STAGED) {
            // instruction k: lanes 8m..8m+7 read the whole 128-B line of owner 8k+m
            const uint8_t* base = blk + (lane >> 3) * 512u + r * 128 + (lane & 7u) * 16u;
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = ldg4(reinterpret_cast<const uint4*>(base + k * 8 * 512));
        } else {
            const uint4* p = reinterpret_cast<const uint4*>(blk + lane * 512u + r * 128);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = LM == LM_DIRECT_NT ? ldg4(p + j) : ldg4_plain(p + j);
        }
    };
    load_round(cur, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        if (r < 3) load_round(nxt, r + 1);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (LM == LM_STAGED) {
#pragma unroll
            for (int k = 0; k < 8; ++k) stage[stage_slot(8u * k + (lane >> 3), lane & 7u)] = cur[k];
            wave_lds_sync();
#pragma unroll
            for (int t = 0; t < 8; ++t) cur[t] = stage[stage_slot(lane, t)];
            wave_lds_sync();
        }
        if (r == 0) zero_header_bytes(cur[0], l0, force_type, hdr);
#pragma unroll
        for (int j = 0; j < 8; ++j) crc = absorb4<TM>(crc, cur[j], L, tab);
        __builtin_amdgcn_sched_barrier(0);
        if (r < 3) {
#pragma unroll
            for (int j = 0; j < 8; ++j) cur[j] = nxt[j];
        }
    }
    return crc;
}

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
    __shared__ alignas(16) uint32_t tab[32768];// 128 KiB: T'' replicated 32x
    __shared__ uint32_t shtab[8 * 1024];  // 32 KiB: inverse-shift tree tables
    fill_gap_tables(tab, c_gap1020);
    fill_inv_tree_tables(shtab, 8);
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

// The production C2 kernel (k_blocks.hip k_full_blocks4) with a scheduling
// barrier after every row: each refill is issued in its own row, so ~15 rows
// stay in flight through the block end (the production build's scheduler sinks
// the last rows' refills to the block end, down to 4 in flight).
template <int THREADS>
__global__ __launch_bounds__(THREADS) void k_full_blocks4_sb(const uint8_t* __restrict__ blocks, uint64_t nblocks,
                                                             uint32_t* __restrict__ masked_out,
                                                             uint8_t* __restrict__ ok_out) {
    __shared__ alignas(16) uint32_t tab[32768];
    __shared__ uint32_t shtab[8 * 1024];
    fill_gap_tables(tab, c_gap1020);
    fill_inv_tree_tables(shtab, 8);
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
                zero_header_bytes(c, l0, false, &hdr);
                u0 = c.x; u1 = c.y; u2 = c.z; u3 = c.w;
                ring[0] = row(b, 16);
            }
            const uint4 wn = g < 31 ? ring[(g + 1) & 15] : make_uint4(0, 0, 0, 0);
            u0 = step_x(u0, wn.x, L, tab);
            u1 = step_x(u1, wn.y, L, tab);
            u2 = step_x(u2, wn.z, L, tab);
            u3 = step_x(u3, wn.w, L, tab);
            if (g < 31) ring[(g + 1) & 15] = g + 17 < 32 ? row(b, g + 17) : row(b + nwaves, g + 17 - 32);
            __builtin_amdgcn_sched_barrier(0);
        }
        finish_full_block<false>(u0, u1, u2, u3, hdr, b, shtab, lane, masked_out, ok_out, nullptr);
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


// Variant table of the experiment library (production = variant 0 of the
// product library, revel_gpu_crc_full_blocks).
extern "C" int revel_x_crc_full_blocks_variant(revel_gpu_context* ctx, int variant, const void* d_blocks,
                                               size_t n, uint32_t* d_masked, uint8_t* d_ok, void* stream) {
    if (!ctx || !d_blocks || !d_masked) return REVEL_INVALID_ARGUMENT;
    if (n == 0) return REVEL_OK;
    if (hipSetDevice(ctx->di.device) != hipSuccess) return REVEL_IO_ERROR;
    const DeviceInfo& di = ctx->di;
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    const uint8_t* b = static_cast<const uint8_t*>(d_blocks);
    hipError_t e;
    switch (variant) {
        case 9: e = launch_full<TM_S4R, 1024, LM_DIRECT, false>(di, 1, b, n, d_masked, d_ok, nullptr, st); break;
        case 8: e = launch_full<TM_S2R, 768, LM_STAGED, false>(di, 1, b, n, d_masked, d_ok, nullptr, st); break;
        // v2 (pipelined across blocks): chains x epilogue
        case 10: e = launch_full2<TM_S4R, 1024, 1, EPI_GFMUL, false>(di, b, n, d_masked, d_ok, nullptr, st); break;
        case 11: e = launch_full2<TM_S4R, 1024, 2, EPI_GFMUL, false>(di, b, n, d_masked, d_ok, nullptr, st); break;
        case 12: e = launch_full2<TM_S4R, 1024, 1, EPI_TREE, false>(di, b, n, d_masked, d_ok, nullptr, st); break;
        case 13: e = launch_full2<TM_S4R, 1024, 2, EPI_TREE, false>(di, b, n, d_masked, d_ok, nullptr, st); break;
        case 14: e = launch_full2<TM_S2R, 1024, 2, EPI_TREE, false>(di, b, n, d_masked, d_ok, nullptr, st); break;
        // v3: interleaved word streams, gap folded into the tables (nt / plain loads)
        case 20: e = launch_full3<1024, true, false>(di, b, n, d_masked, d_ok, nullptr, st); break;
        case 21: e = launch_full3<1024, false, false>(di, b, n, d_masked, d_ok, nullptr, st); break;
        // v3 with the x-state chain (3-input xors)
        case 22: e = launch_full3<1024, true, false, true>(di, b, n, d_masked, d_ok, nullptr, st); break;
        // production C2 with a scheduling barrier per row (constant ring depth)
        case 23: {
            const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu, (n + 15) / 16));
            hipLaunchKernelGGL(k_full_blocks4_sb<1024>, dim3((uint32_t)grid), dim3(1024), 0, st, b, n, d_masked, d_ok);
            e = hipGetLastError();
            break;
        }
        // v1: lane-owned 512-B chunks
        case 1: e = launch_full<TM_S2R, 512, LM_STAGED, false>(di, 1, b, n, d_masked, d_ok, nullptr, st); break;
        case 2: e = launch_full<TM_S4R, 256, LM_STAGED, false>(di, 1, b, n, d_masked, d_ok, nullptr, st); break;
        case 3: e = launch_full<TM_S4, 1024, LM_STAGED, false>(di, 1, b, n, d_masked, d_ok, nullptr, st); break;
        case 4: e = launch_full<TM_S2R, 512, LM_DIRECT, false>(di, 2, b, n, d_masked, d_ok, nullptr, st); break;
        case 5: e = launch_full<TM_S4R, 1024, LM_DIRECT, false>(di, 1, b, n, d_masked, d_ok, nullptr, st); break;
        case 6: e = launch_full<TM_S4, 512, LM_DIRECT, false>(di, 4, b, n, d_masked, d_ok, nullptr, st); break;
        case 7: e = launch_full<TM_S2R, 512, LM_DIRECT_NT, false>(di, 2, b, n, d_masked, d_ok, nullptr, st); break;
        case 100: {
            const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu * 8, (n + 3) / 4));
            hipLaunchKernelGGL(k_stream_ceiling<256>, dim3((uint32_t)grid), dim3(256), 0, st, b, n, d_masked);
            e = hipGetLastError();
            break;
        }
        // streaming-read ceiling shapes: plain loads; fewer / more waves per CU
        case 101: e = launch_stream<256, false>(di, 8, b, n, d_masked, st); break;
        case 102: e = launch_stream<256, true>(di, 4, b, n, d_masked, st); break;
        case 103: e = launch_stream<256, true>(di, 2, b, n, d_masked, st); break;
        case 104: e = launch_stream<1024, true>(di, 1, b, n, d_masked, st); break;
        case 105: e = launch_stream<512, true>(di, 4, b, n, d_masked, st); break;
        case 106: e = launch_stream<256, true>(di, 16, b, n, d_masked, st); break;
        default: return REVEL_INVALID_ARGUMENT;
    }
    return e == hipSuccess ? REVEL_OK : REVEL_IO_ERROR;
}
