// k_blocks.hip -- config C2 kernels: one FULL record per 32 KiB block
// (k_full_blocks4, verify and device framing) and the synthetic block generator.
// The experiment arms measured on the way (lane-owned chunks, v2, v3, the
// streaming-read ceiling) live in tools/experiments/x_blocks.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>

#include "device_common.h"

using namespace revel;

namespace {
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
// Config C2: interleaved word streams with the gap folded into the tables.
//
// Stream s (s = 0..255) is the 32-bit words at byte offsets 4s + 1024k,
// k = 0..31; lane i owns streams 4i..4i+3, i.e. one 16-byte load per lane
// per 1 KiB: exactly the coalescing of a plain streaming read (1 KiB per
// wave instruction).  Consecutive words of a stream are 1024 bytes apart, so
// the gap tables T'' = x^(8*1020) * T absorb a word and the 1020 bytes that
// follow it in one step (device_common.h).  The four streams of a lane are
// four independent chains (ILP 4).  After its 32nd word, stream s stands at
// byte 32768 + 4s; the block register is
//     R = XOR_s  U_s * x^(-32 s)  mod P
// (x is invertible mod P since P(0) = 1), evaluated by an 8-level tree of
// inverse-shift tables: 2 levels inside the lane, 6 across lanes.
// ---------------------------------------------------------------------------

// Block epilogue: R = XOR_s U_s x^(-32 s) by the 8-level inverse-shift tree
// (2 levels in-lane, 6 across lanes), then the masked CRC, the header check or
// the framed header.
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

// ---------------------------------------------------------------------------
// x-state chains fed by a 16-slot load ring.  Row g of a block (g = 0..31) is
// the 1 KiB [1024 g, +1024), 16 B per lane.  The slot a row leaves is refilled
// at once with the row 16 ahead (into the next block at the end), so ~15 rows =
// 15 KiB per wave stay in flight with 64 VGPRs.  All loads are unconditional
// (rows past the last block re-read the last block), so the compiler's vmcnt
// counts stay exact.  A chain carries x = U ^ (next word): the four table
// words and the next data word fold with two 3-input xors.
// ---------------------------------------------------------------------------
#ifdef REVEL_C2_WAVETIME
__device__ uint64_t g_c2_wavetime[3 * 65536];
#endif
template <int THREADS, bool FRAME>
__global__ __launch_bounds__(THREADS) void k_full_blocks4(const uint8_t* __restrict__ blocks, uint64_t nblocks,
                                                          uint32_t* __restrict__ masked_out,
                                                          uint8_t* __restrict__ ok_out, uint8_t* __restrict__ frame_dst) {
    __shared__ alignas(16) uint32_t tab[32768];  // 128 KiB: T'' replicated 32x
    __shared__ uint32_t shtab[8 * 1024];  // 32 KiB: inverse-shift tree tables
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
#ifdef REVEL_C2_WAVETIME  // timing probe: each wave's start / end (s_memrealtime, 100 MHz)
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
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
#ifdef REVEL_C2_WAVETIME
    if (lane == 0 && gwave < 65536u) {
        g_c2_wavetime[3u * gwave] = t_start;
        g_c2_wavetime[3u * gwave + 1u] = __builtin_amdgcn_s_memrealtime();
        g_c2_wavetime[3u * gwave + 2u] = (nblocks - gwave + nwaves - 1u) / nwaves;
    }
#endif
}

template <bool FRAME>
hipError_t launch_full4(const DeviceInfo& di, const uint8_t* blocks, uint64_t n, uint32_t* masked, uint8_t* ok,
                        uint8_t* frame_dst, hipStream_t st) {
    constexpr int kThreads = 1024;
    const uint64_t wg_needed = (n + kThreads / 64 - 1) / (kThreads / 64);
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu, wg_needed));
    hipLaunchKernelGGL((k_full_blocks4<kThreads, FRAME>), dim3((uint32_t)grid), dim3(kThreads), 0, st, blocks, n,
                       masked, ok, frame_dst);
    return hipGetLastError();
}

}  // namespace

namespace revel {

hipError_t crc_full_blocks(const DeviceInfo& di, const void* d_blocks, uint64_t n, uint32_t* d_masked, uint8_t* d_ok,
                           hipStream_t st) {
    return launch_full4<false>(di, static_cast<const uint8_t*>(d_blocks), n, d_masked, d_ok, nullptr, st);
}

hipError_t frame_full_blocks(const DeviceInfo& di, void* d_blocks, uint64_t n, hipStream_t st) {
    uint8_t* b = static_cast<uint8_t*>(d_blocks);
    return launch_full4<true>(di, b, n, nullptr, nullptr, b, st);
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

// Build provenance (revel_wal.h): hipcc's clang, which compiled this file's
// kernels, and the offload target.
// REVEL_BUILD_FLAGS: the Makefile's "--offload-arch=$(ARCH) $(XFLAGS)", so a
// variant build (timing probes, A/B switches: wrong results or other kernels)
// names its flags wherever bench.py prints the provenance.
#ifndef REVEL_BUILD_FLAGS
#define REVEL_BUILD_FLAGS "(flags unknown: built outside revel_amd/csrc/Makefile)"
#endif
extern "C" const char* revel_build_info(void) { return "hipcc clang " __clang_version__ "; " REVEL_BUILD_FLAGS; }

#ifdef REVEL_C2_WAVETIME
// timing probe builds only: k_full_blocks4's per-wave start / end times of its last launch
extern "C" int revel_debug_c2_wavetime(uint64_t* host, uint64_t n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_c2_wavetime), n * sizeof(uint64_t), 0, hipMemcpyDeviceToHost);
}
#endif
