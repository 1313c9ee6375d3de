// gpu_crc.hip -- CDNA4 (gfx950) CRC-32C engine for Revel's WAL record path.
//
// Hot path (reference guimingyue/revel @ v0):
//   log_writer.rs:107-111  crc = mask(extend(type, payload))  (writer side)
//   log_reader.rs:200-206  unmask(stored) == value(type||payload) (reader side)
//   util/crc.rs:13-44      CRC_32_ISCSI + mask/unmask
//
// Work decomposition: ONE WAVEFRONT PER 32 KiB LOG BLOCK.  Lane i owns the
// contiguous 512-byte chunk [512 i, 512 i + 512) of its block and runs a
// table-driven CRC over it from a zero register; the 64 partial registers are
// then combined by a wavefront GF(2) polynomial-shift reduction:
//     R(block) = XOR_i  R_i * x^(8*512*(63-i))  mod P
// (each lane multiplies by its own constant, then an xor-butterfly across the
// wave).  Init/xorout enter once per record as a length-dependent constant.
// No MFMA: this is GF(2) arithmetic, not a contraction.
//
// Lookup tables live in LDS, replicated 32x so that lane (l & 31) always hits
// bank (l & 31) for ds_read_b32: bank-conflict-free gathers whatever the data.
// The LDS byte address of entry e for lane l is (e << 8) | ((l & 31) << 2)
// | (region << 16), built by ONE v_perm_b32 per lookup.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <type_traits>
#include <string>
#include <vector>

#include "crc32c_math.h"
#include "gpu_internal.h"

using namespace revel;

namespace {

constexpr SliceTables kTables = make_slice_tables();

// ---------------------------------------------------------------------------
// Compile-time GF(2) constants
// ---------------------------------------------------------------------------
struct LaneShiftConsts {
    uint32_t c[64];  // x^(8*512*(63-i)) mod P
};
constexpr LaneShiftConsts make_lane_shift() {
    LaneShiftConsts s{};
    for (int i = 0; i < 64; ++i) s.c[i] = x8n(512ull * (63 - i));
    return s;
}
// x^(8*512*m) for m = 0..64 and x^(8*d) for d = 0..512: any shift inside a
// block is one multmodp of two table entries.
struct ShiftTables {
    uint32_t chunk[65];
    uint32_t byte[513];
};
constexpr ShiftTables make_shift_tables() {
    ShiftTables s{};
    for (int m = 0; m <= 64; ++m) s.chunk[m] = x8n(512ull * m);
    uint32_t v = 0x80000000u;  // x^0
    const uint32_t x8 = x8n(1);
    for (int d = 0; d <= 512; ++d) {
        s.byte[d] = v;
        v = multmodp(x8, v);
    }
    return s;
}

__constant__ SliceTables c_tables = kTables;
__constant__ LaneShiftConsts c_lane_shift = make_lane_shift();
__constant__ ShiftTables c_shift = make_shift_tables();

constexpr uint32_t kFullInitXor = init_xor(kFullCrcLen);
constexpr uint32_t kFullTypeByte = 1u;

// ---------------------------------------------------------------------------
// Device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Branch-free a*b mod P (reflected).  v_bfe_i32 turns a bit into 0/-1.
__device__ __forceinline__ uint32_t gf_mul(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        uint32_t am = (uint32_t)__builtin_amdgcn_sbfe((int)a, 31 - k, 1);
        p ^= b & am;
        uint32_t bm = (uint32_t)__builtin_amdgcn_sbfe((int)b, 0, 1);
        b = (b >> 1) ^ (kPolyReflected & bm);
    }
    return p;
}

// x^(8n) mod P for 0 <= n <= 32768 from the two shift tables.
__device__ __forceinline__ uint32_t gf_x8n_block(uint32_t n) {
    uint32_t m = n >> 9, d = n & 511u;
    uint32_t a = c_shift.chunk[m];
    return d ? gf_mul(a, c_shift.byte[d]) : a;
}

__device__ __forceinline__ uint32_t xor_reduce_wave(uint32_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v ^= __shfl_xor(v, m, 64);
    return v;
}

__device__ __forceinline__ uint32_t bytewise_step(uint32_t s, uint32_t b) {
    return c_tables.t[0][(s ^ b) & 0xffu] ^ (s >> 8);
}

// LDS byte-address load (ds_read_b32 with immediate offset).  The tables are
// a static __shared__ array, so its base folds into the instruction.
template <int OFF>
__device__ __forceinline__ uint32_t ldsw(const uint32_t* tab, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(tab) + byte_addr + OFF);
}

// v_perm_b32 selectors: result byte0 <- lanec byte0 (lane*4), byte1 <- x byte k,
// byte2 <- lanec byte2 (table region), byte3 <- 0.
template <int K>
struct Sel {
    static constexpr uint32_t v = 0x0C020000u | ((4u + K) << 8) | 0x00u;
};

// ---------------------------------------------------------------------------
// Table modes
// ---------------------------------------------------------------------------
enum TableMode : int {
    TM_S4R = 0,  // slice-by-4, 32x replicated, 128 KiB LDS
    TM_S2R = 1,  // slice-by-2, 32x replicated, 64 KiB LDS
    TM_S4 = 2,   // slice-by-4, unreplicated, 4 KiB LDS (bank conflicts)
};

template <int TM>
struct TableCfg;
template <>
struct TableCfg<TM_S4R> {
    static constexpr uint32_t bytes = 131072;
};
template <>
struct TableCfg<TM_S2R> {
    static constexpr uint32_t bytes = 65536;
};
template <>
struct TableCfg<TM_S4> {
    static constexpr uint32_t bytes = 4096;
};

// Fill the LDS image of the tables (cooperatively, whole workgroup).
template <int TM>
__device__ void fill_tables(uint32_t* tab) {
    const uint32_t ndw = TableCfg<TM>::bytes / 4;
    for (uint32_t d = threadIdx.x; d < ndw; d += blockDim.x) {
        uint32_t v;
        if constexpr (TM == TM_S4) {
            // [T3 | T2 | T1 | T0], 256 entries each: byte k of x indexes T(3-k)
            v = c_tables.t[3 - (d >> 8)][d & 255u];
        } else if constexpr (TM == TM_S4R) {
            // region r (16384 dw) -> row e (64 dw) -> half h (32 dw) -> copy c
            uint32_t r = d >> 14, e = (d >> 6) & 255u, h = (d >> 5) & 1u;
            // byte0 -> T3 (r0 h0), byte1 -> T2 (r0 h1), byte2 -> T1 (r1 h0), byte3 -> T0 (r1 h1)
            v = c_tables.t[3 - (r * 2 + h)][e];
        } else {
            // S2R: row e = [T1 x32 | T0 x32]
            uint32_t e = (d >> 6) & 255u, h = (d >> 5) & 1u;
            v = c_tables.t[1 - h][e];
        }
        tab[d] = v;
    }
}

struct LaneConst {
    uint32_t lc0, lc1;
};

__device__ __forceinline__ LaneConst make_lane_const() {
    uint32_t c4 = (lane_id() & 31u) << 2;
    return {c4, c4 | 0x10000u};
}

// Absorb one little-endian 32-bit word into the raw register.
template <int TM>
__device__ __forceinline__ uint32_t absorb(uint32_t crc, uint32_t w, LaneConst L, const uint32_t* tab) {
    uint32_t x = crc ^ w;
    if constexpr (TM == TM_S4R) {
        uint32_t a0 = __builtin_amdgcn_perm(x, L.lc0, Sel<0>::v);
        uint32_t a1 = __builtin_amdgcn_perm(x, L.lc0, Sel<1>::v);
        uint32_t a2 = __builtin_amdgcn_perm(x, L.lc1, Sel<2>::v);
        uint32_t a3 = __builtin_amdgcn_perm(x, L.lc1, Sel<3>::v);
        return (ldsw<0>(tab, a0) ^ ldsw<128>(tab, a1)) ^ (ldsw<0>(tab, a2) ^ ldsw<128>(tab, a3));
    } else if constexpr (TM == TM_S2R) {
        uint32_t a0 = __builtin_amdgcn_perm(x, L.lc0, Sel<0>::v);
        uint32_t a1 = __builtin_amdgcn_perm(x, L.lc0, Sel<1>::v);
        uint32_t c = ldsw<0>(tab, a0) ^ ldsw<128>(tab, a1) ^ (x >> 16);
        uint32_t a2 = __builtin_amdgcn_perm(c, L.lc0, Sel<0>::v);
        uint32_t a3 = __builtin_amdgcn_perm(c, L.lc0, Sel<1>::v);
        return ldsw<0>(tab, a2) ^ ldsw<128>(tab, a3) ^ (c >> 16);
    } else {
        return (tab[x & 0xffu] ^ tab[256 + ((x >> 8) & 0xffu)]) ^
               (tab[512 + ((x >> 16) & 0xffu)] ^ tab[768 + (x >> 24)]);
    }
}

template <int TM>
__device__ __forceinline__ uint32_t absorb4(uint32_t crc, uint4 v, LaneConst L, const uint32_t* tab) {
    crc = absorb<TM>(crc, v.x, L, tab);
    crc = absorb<TM>(crc, v.y, L, tab);
    crc = absorb<TM>(crc, v.z, L, tab);
    crc = absorb<TM>(crc, v.w, L, tab);
    return crc;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldg4(const uint4* p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 ldg4_plain(const uint4* p) { return *p; }

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
__device__ __forceinline__ void zero_header_bytes(uint4& v, bool l0, bool force_type, uint4* hdr) {
    *hdr = v;
    v.x = l0 ? 0u : v.x;
    const uint32_t y = force_type ? ((v.y & 0xFF000000u) | (uint32_t(kFullTypeByte) << 16)) : v.y;
    v.y = l0 ? (y & 0xFFFF0000u) : v.y;
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

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
template <int THREADS>
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
            uint4 v = ldg4(p + k * 64);
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
// Config C3: variable records (FULL/FIRST/MIDDLE/LAST mixes, padding, zeros).
// ---------------------------------------------------------------------------
struct Hdr {
    uint32_t stored, len, type;
};

// Bytes [off, off+7) of a block of length bl, never reading at or past bl
// (the image end need not be 4-byte aligned or padded).
__device__ __forceinline__ Hdr read_header(const uint8_t* base, uint32_t off, uint32_t bl) {
    const uint32_t a0 = off & ~3u;
    uint32_t w0, w1, w2 = 0;
    if (a0 + 12u <= bl) {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(base + a0);
        w0 = w[0]; w1 = w[1]; w2 = w[2];
    } else {
        uint8_t t[12];
        for (uint32_t k = 0; k < 12; ++k) t[k] = a0 + k < bl ? base[a0 + k] : 0;
        memcpy(&w0, t, 4); memcpy(&w1, t + 4, 4); memcpy(&w2, t + 8, 4);
    }
    const uint32_t sh = (off & 3u) * 8u;
    const uint64_t lo = (uint64_t(w1) << 32) | w0;
    const uint64_t hi = (uint64_t(w2) << 32) | w1;
    const uint32_t a = uint32_t(lo >> sh);  // bytes off..off+3
    const uint32_t b = uint32_t(hi >> sh);  // bytes off+4..off+7
    return {a, b & 0xFFFFu, (b >> 16) & 0xFFu};
}

// 16 bytes at block offset pos, zero outside [lo, bl) (lo > 0 only for the
// first block of an image that starts mid-block).
__device__ __forceinline__ uint4 load16_range(const uint8_t* blk, uint32_t pos, uint32_t lo, uint32_t bl) {
    if (pos >= lo && pos + 16u <= bl) return ldg4_plain(reinterpret_cast<const uint4*>(blk + pos));
    uint8_t t[16];
    for (uint32_t k = 0; k < 16; ++k) t[k] = (pos + k >= lo && pos + k < bl) ? blk[pos + k] : 0;
    uint4 v;
    memcpy(&v, t, 16);
    return v;
}

__device__ __forceinline__ Hdr read_header_range(const uint8_t* base, uint32_t off, uint32_t lo, uint32_t bl) {
    if ((off & ~3u) >= lo) return read_header(base, off, bl);
    uint8_t t[8];
    for (uint32_t k = 0; k < 7; ++k) t[k] = base[off + k];  // off >= lo, off + 7 <= bl
    t[7] = 0;
    uint32_t a, b;
    memcpy(&a, t, 4);
    memcpy(&b, t + 4, 4);
    return {a, b & 0xFFFFu, (b >> 16) & 0xFFu};
}

// 16 bytes at block offset pos, zero past bl.
__device__ __forceinline__ uint4 load16_guarded(const uint8_t* blk, uint32_t pos, uint32_t bl) {
    if (pos + 16u <= bl) return ldg4(reinterpret_cast<const uint4*>(blk + pos));
    uint8_t t[16];
    for (uint32_t k = 0; k < 16; ++k) t[k] = pos + k < bl ? blk[pos + k] : 0;
    uint4 v;
    memcpy(&v, t, 16);
    return v;
}

// One step of the physical-record walk (oracle walk_block rules).
__device__ __forceinline__ uint32_t classify(const Hdr& h, uint32_t off, uint32_t bl) {
    if (kHeaderSize + h.len > bl - off) return REVEL_REC_BAD_LENGTH;
    if (h.type == 0 && h.len == 0) return REVEL_REC_ZERO;
    return REVEL_REC_OK;
}

// Header-list entry: the 7 header bytes as read (stored CRC | len << 32 |
// type << 48).  Offsets are not stored: entry k sits at the sum of 7 + len of
// the entries before it (a wave prefix sum in the consumer).
__device__ __forceinline__ uint64_t list_entry(const Hdr& h) {
    return uint64_t(h.stored) | (uint64_t(h.len | (h.type << 16)) << 32);
}
__device__ __forceinline__ Hdr list_header(uint64_t e) {
    const uint32_t hi = uint32_t(e >> 32);
    return {uint32_t(e), hi & 0xFFFFu, (hi >> 16) & 0xFFu};
}
// Wave-wide exclusive prefix sum (lanes >= n contribute 0).
__device__ __forceinline__ uint32_t wave_exclusive_sum(uint32_t v) {
    uint32_t incl = v;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(incl, d, 64);
        incl += lane_id() >= d ? t : 0u;
    }
    return incl - v;
}

// Per block (one lane each): number of physical records and, when list is
// non-null, the first kListPerBlock headers (list_entry; the walk stops at the
// first bad header, so only the last entry can be bad).
__global__ void k_count_records(const uint8_t* __restrict__ image, uint64_t nbytes, uint32_t* __restrict__ counts,
                                uint64_t* __restrict__ hlist) {
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < nblocks;
         b += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t base = b * kBlockSize;
        const uint32_t bl = (uint32_t)std::min<uint64_t>(kBlockSize, nbytes - base);
        const uint8_t* blk = image + base;
        uint32_t off = 0, n = 0;
        while (bl - off >= kHeaderSize) {
            const Hdr h = read_header(blk, off, bl);
            const bool ok = classify(h, off, bl) == REVEL_REC_OK;
            if (hlist && n < kListPerBlock) hlist[b * kListPerBlock + n] = list_entry(h);
            ++n;
            if (!ok) break;
            off += kHeaderSize + h.len;
        }
        counts[b] = n;
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

template <typename T>
__global__ __launch_bounds__(256) void k_scan_apply(const T* __restrict__ in, uint64_t n, const T* __restrict__ tile_sums,
                                                    T* __restrict__ out) {
    __shared__ T red[4];
    __shared__ T wsum[4];
    // offset of this tile = sum of the tile sums before it
    T pre = 0;
    for (uint32_t t = threadIdx.x; t < blockIdx.x; t += 256) pre += tile_sums[t];
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

constexpr int kVerifyThreads = 512;
constexpr uint32_t kRecCap = 256;  // records per LDS batch per wave

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

struct VerifyWaveLds {
    uint16_t s[kRecCap];    // start of the CRC range (= header offset + 6)
    uint16_t em1[kRecCap];  // end of the range minus one (off + 7 + len - 1 <= 32767); s - 1 for bad headers
    uint32_t acc[kRecCap];  // xor of lane contributions, aligned to E = ceil4(end)
    uint32_t nrec;
    uint32_t more_off;
};

// Per-lane segmented CRC.  Every record's contributions are aligned to its
// word-aligned range end E = ceil4(e): the lane holding e absorbs the final
// word with the bytes past e zeroed (that is R * x^(8 pad)), lanes ending
// earlier shift their partial register by E - chunk_end; the finalizer
// multiplies by x^(-8 pad).  Records whose header is bad get an empty range.
__global__ __launch_bounds__(kVerifyThreads) void k_verify_records(const uint8_t* __restrict__ image, uint64_t nbytes,
                                                                   uint64_t base_offset,
                                                                   const uint32_t* __restrict__ first,
                                                                   revel_record_result* __restrict__ out) {
    constexpr int TM = TM_S2R;
    __shared__ uint32_t tab[TableCfg<TM>::bytes / 4];
    fill_tables<TM>(tab);
    __shared__ VerifyWaveLds wl_all[kVerifyThreads / 64];
    __syncthreads();
    VerifyWaveLds& wl = wl_all[threadIdx.x >> 6];
    const LaneConst L = make_lane_const();
    const uint32_t lane = lane_id();
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    const uint64_t waves_per_wg = kVerifyThreads / 64;
    const uint64_t gwave = blockIdx.x * waves_per_wg + (threadIdx.x >> 6);
    const uint64_t nwaves = gridDim.x * waves_per_wg;

    for (uint64_t b = gwave; b < nblocks; b += nwaves) {
        const uint64_t base = b * kBlockSize;
        const uint8_t* blk = image + base;
        const uint32_t bl = (uint32_t)std::min<uint64_t>(kBlockSize, nbytes - base);
        const uint32_t cs = lane * 512u, ce = cs + 512u;
        uint32_t out_base = first[b];
        uint32_t walk_from = 0;
        for (;;) {
            // ---- lane 0 walks up to kRecCap records into LDS ----
            if (lane == 0) {
                uint32_t off = walk_from, n = 0, cont = 0xFFFFFFFFu;
                while (bl - off >= kHeaderSize) {
                    if (n == kRecCap) { cont = off; break; }
                    const Hdr h = read_header(blk, off, bl);
                    const uint32_t st = classify(h, off, bl);
                    wl.s[n] = (uint16_t)(off + 6);
                    wl.em1[n] = (uint16_t)(st == REVEL_REC_OK ? off + kHeaderSize + h.len - 1u : off + 5u);
                    wl.acc[n] = 0;
                    ++n;
                    if (st != REVEL_REC_OK) break;
                    off += kHeaderSize + h.len;
                }
                wl.nrec = n;
                wl.more_off = cont;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            const uint32_t nrec = wl.nrec;
            const uint32_t cont = wl.more_off;

            // Range of record k as [s, e) with exact e; E = aligned end.
            // Bad records: s = e (empty).
            auto load_rec = [&](uint32_t k, uint32_t& s, uint32_t& e, uint32_t& E) {
                if (k >= nrec) { s = e = E = 0xFFFFFFFFu; return; }
                s = wl.s[k];
                e = uint32_t(wl.em1[k]) + 1u;
                E = (e + 3u) & ~3u;
            };
            // first record whose range ends after cs (ranges are increasing)
            uint32_t lo = 0, hi = nrec;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (uint32_t(wl.em1[mid]) + 1u > cs) hi = mid; else lo = mid + 1;
            }
            uint32_t r = lo, s, e, E;
            load_rec(r, s, e, E);
            while (r < nrec && s == e) { ++r; load_rec(r, s, e, E); }

            uint32_t state = 0;
            if (cs < bl && s < ce) {
#pragma unroll 2
                for (uint32_t t = 0; t < 32; ++t) {
                    const uint32_t p16 = cs + t * 16u;
                    if (p16 >= bl || s >= ce) break;  // nothing of this batch left in the chunk
                    const uint4 v = load16_guarded(blk, p16, bl);
                    if (p16 >= s && p16 + 16u < e) {
                        state = absorb4<TM>(state, v, L, tab);  // interior: no boundary in these 16 bytes
                    } else {
                        const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const uint32_t p = p16 + q * 4u;
                            // keep bytes of [s, e) inside [p, p+4)
                            const uint32_t lo_b = s > p ? min(s - p, 4u) : 0u;
                            const uint32_t hi_b = e > p ? min(e - p, 4u) : 0u;
                            uint32_t keep = hi_b >= 4u ? 0xFFFFFFFFu : ((1u << (8u * hi_b)) - 1u);
                            keep &= lo_b >= 4u ? 0u : (0xFFFFFFFFu << (8u * lo_b));
                            state = absorb<TM>(state, ws[q] & keep, L, tab);
                            if (e > p && e <= p + 4u) {  // record ends in this word: flush
                                atomicXor(&wl.acc[r], state);
                                state = 0;
                                do { ++r; load_rec(r, s, e, E); } while (r < nrec && s == e);
                            }
                        }
                    }
                }
                // a record still open at the chunk end: shift to its aligned end
                if (r < nrec && s < ce && e > ce) {
                    atomicXor(&wl.acc[r], gf_mul(gf_x8n_block(E - ce), state));
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();

            // ---- finalize: one lane per record ----
            for (uint32_t k = lane; k < nrec; k += 64) {
                const uint32_t off = uint32_t(wl.s[k]) - 6u;
                const Hdr h = read_header(blk, off, bl);
                const uint32_t st = classify(h, off, bl);
                revel_record_result res;
                res.file_offset = base_offset + base + off;
                res.length = h.len;
                res.stored_crc = h.stored;
                res.type = (uint8_t)h.type;
                res.reserved[0] = res.reserved[1] = 0;
                if (st == REVEL_REC_OK) {
                    const uint32_t n = h.len + 1u;  // type byte + payload
                    const uint32_t e = off + kHeaderSize + h.len;
                    const uint32_t pad = ((e + 3u) & ~3u) - e;
                    const uint32_t raw = gf_mul(c_inv_pad.v[pad], wl.acc[k]);
                    const uint32_t ix = gf_mul(gf_x8n_block(n), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
                    res.computed_crc = mask(raw ^ ix);
                    res.status = res.computed_crc == res.stored_crc ? REVEL_REC_OK : REVEL_REC_BAD_CHECKSUM;
                } else {
                    res.computed_crc = 0;
                    res.status = (uint8_t)st;
                }
                out[out_base + k] = res;
            }
            out_base += nrec;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (cont == 0xFFFFFFFFu) break;
            walk_from = cont;
        }
    }
}

// ---------------------------------------------------------------------------
// Config C3, v2: S4R tables, 16 waves/CU, pipelined loads, wave-uniform fast
// path, exact tails.
// ---------------------------------------------------------------------------
constexpr int kVerify2Threads = 1024;
constexpr uint32_t kRecCap2 = 128;  // >= kListPerBlock

// x^(8d) and init_xor(d) for d = 0..32768, filled once per device.
__device__ uint32_t g_x8n_tab[kBlockSize + 1];
__device__ uint32_t g_init_xor_tab[kBlockSize + 1];

__global__ void k_init_len_tables() {
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d <= kBlockSize; d += gridDim.x * blockDim.x) {
        const uint32_t x = gf_x8n_block(d);
        g_x8n_tab[d] = x;
        g_init_xor_tab[d] = gf_mul(x, 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
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

template <bool FRAME, int BP = BP_BYTES, int WHICH = BS_ALL, int TM = TM_S4R, int THREADS = kVerify2Threads>
__global__ __launch_bounds__(THREADS) void k_verify_records2(const uint8_t* __restrict__ image, uint64_t nbytes,
                                                                     uint64_t base_offset,
                                                                     const uint32_t* __restrict__ first,
                                                                     revel_record_result* __restrict__ out,
                                                                     uint32_t lead,
                                                                     const uint64_t* __restrict__ hlist,
                                                                     const uint32_t* __restrict__ counts) {
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
        const uint32_t nlist = (hlist && counts) ? counts[b] : kNone;
        for (;;) {
            if (walk_from == lo_b && nlist <= kListPerBlock) {
                const Hdr h = list_header(lane < nlist ? hlist[b * kListPerBlock + lane] : 0ull);
                const uint32_t off = lo_b + wave_exclusive_sum(lane < nlist ? kHeaderSize + h.len : 0u);
                if (lane < nlist) {
                    const bool bad = classify(h, off, bl) != REVEL_REC_OK;
                    wl.off[lane] = (uint16_t)off;
                    wl.s[lane] = bad ? kNoRange : (uint16_t)(off + 6);
                    wl.em1[lane] = bad ? kNoRange : (uint16_t)(off + kHeaderSize + h.len - 1u);
                    wl.acc[lane] = 0;
                }
                if (lane == 0) {
                    wl.s[nlist] = wl.em1[nlist] = kNoRange;
                    wl.nrec = nlist;
                    wl.more_off = kNone;
                }
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
                        // don't-care gap before the next record, or strictly inside one
                        const bool interior = (p16 + 16u <= s) || (p16 >= s && p16 + 16u < e);
                        if (BP != BP_MASK_NOVOTE && __all(interior)) {
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
            walk_from = cont;
        }
    }
}

// ---------------------------------------------------------------------------
// Config C3, v3 (production, whole blocks): v2's per-block work, software-
// pipelined across the blocks a wave visits.  After a block's main loop the
// wave issues the finalizer's header loads, then the NEXT block's round-0
// data, header list entry, record count and output slot, and only then waits
// for the headers: the next block's loads are in flight while this block is
// finalized, so a block no longer pays three global round trips in series.
// Partial blocks (first/last) still go through k_verify_records2<.., BS_PARTIAL>.
// ---------------------------------------------------------------------------
template <bool FRAME>
__global__ __launch_bounds__(kVerify2Threads) void k_verify_records3(const uint8_t* __restrict__ image, uint64_t nbytes,
                                                                     uint64_t base_offset,
                                                                     const uint32_t* __restrict__ first,
                                                                     revel_record_result* __restrict__ out,
                                                                     uint32_t lead,
                                                                     const uint64_t* __restrict__ hlist,
                                                                     const uint32_t* __restrict__ counts) {
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
    const bool use_list = hlist != nullptr && counts != nullptr;
    const uint32_t cs = lane * 512u, ce = cs + 512u;

    // wave-uniform block index (readfirstlane: the compiler cannot prove that
    // threadIdx.x >> 6 is uniform, and would keep the block arithmetic in VGPRs)
    const uint32_t wave_in_wg = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint64_t b = b_lo + blockIdx.x * waves_per_wg + wave_in_wg;
    if (b >= b_hi) return;  // wave-uniform; no workgroup barrier follows
    uint4 cur[8], nxt[8];
    uint32_t pf_count = kNone, pf_first = 0;
    uint64_t pf_hl = 0;
    auto load_round = [&](const uint8_t* blk, uint4* v, int rr) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = ldg4_plain(reinterpret_cast<const uint4*>(blk + cs + rr * 128 + j * 16));
    };
    // header list first: the list is needed before the data (loads return in order)
    auto prefetch = [&](uint64_t nb) {
        if (use_list) {
            pf_count = counts[nb];
            pf_hl = hlist[nb * kListPerBlock + lane];
        }
        if constexpr (!FRAME) pf_first = first[nb];
        load_round(image + nb * kBlockSize - lead, cur, 0);
    };
    prefetch(b);
    while (b < b_hi) {
        const uint64_t base = b * kBlockSize;
        const uint8_t* blk = image + base - lead;
        const uint64_t bn = b + nwaves;
        const uint32_t nlist = pf_count;
        const uint64_t hl_e = pf_hl;
        uint32_t out_base = pf_first;
        uint32_t walk_from = 0;
        bool have_round0 = true;
        for (;;) {
            const bool from_list = walk_from == 0 && nlist <= kListPerBlock;
            if (from_list) {
                // headers come from the count pass; offsets by prefix sum; the
                // finalizer reads them back from LDS (no global header reads)
                const Hdr h = list_header(hl_e);
                const uint32_t off = wave_exclusive_sum(lane < nlist ? kHeaderSize + h.len : 0u);
                if (lane < nlist) {
                    const bool bad = classify(h, off, kBlockSize) != REVEL_REC_OK;
                    wl.off[lane] = (uint16_t)off;
                    wl.s[lane] = bad ? kNoRange : (uint16_t)(off + 6);
                    wl.em1[lane] = bad ? kNoRange : (uint16_t)(off + kHeaderSize + h.len - 1u);
                    wl.acc[lane] = 0;
                    wl.hstored[lane] = h.stored;
                    wl.hlt[lane] = h.len | (h.type << 16);
                }
                if (lane == 0) {
                    wl.s[nlist] = wl.em1[nlist] = kNoRange;
                    wl.nrec = nlist;
                    wl.more_off = kNone;
                }
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
            if (__any(active)) {
                if (!have_round0) load_round(blk, cur, 0);
#pragma unroll 1
                for (int rr = 0; rr < 4; ++rr) {
                    if (rr < 3) load_round(blk, nxt, rr + 1);
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const uint32_t p16 = cs + rr * 128 + j * 16;
                        // don't-care gap before the next record, or strictly inside one
                        const bool interior = (p16 + 16u <= s) || (p16 >= s && p16 + 16u < e);
                        if (__all(interior)) {
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
                    for (int j = 0; j < 8; ++j) cur[j] = nxt[j];
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
            walk_from = cont;
        }
        b = bn;
    }
}

// ---------------------------------------------------------------------------
// Device append framing, step 1: scatter fragments (payload bytes + length
// and type header bytes, CRC left zero) and zero the block trailers.  One
// wave per fragment; the layout comes from the host (frame_layout()).
// ---------------------------------------------------------------------------
__global__ void k_scatter_fragments(const uint8_t* __restrict__ payloads, const revel::FragDesc* __restrict__ frags,
                                    uint64_t nfrags, uint8_t* __restrict__ image) {
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
    for (uint64_t f = blockIdx.x * (uint64_t)(blockDim.x / 64) + (threadIdx.x >> 6); f < nfrags; f += waves) {
        const revel::FragDesc d = frags[f];
        uint8_t* dst = image + d.dst;
        const uint32_t lane = lane_id();
        if (d.type == revel::kTrailer) {
            for (uint32_t i = lane; i < d.len; i += 64) dst[i] = 0;
            continue;
        }
        if (lane < 7) {
            const uint8_t hv[7] = {0, 0, 0, 0, (uint8_t)(d.len & 0xffu), (uint8_t)(d.len >> 8), (uint8_t)d.type};
            dst[lane] = hv[lane];
        }
        const uint8_t* src = payloads + d.src;
        uint8_t* pd = dst + kHeaderSize;
        for (uint32_t i = lane * 4; i < d.len; i += 256) {
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k)
                if (i + k < d.len) pd[i + k] = src[i + k];
        }
    }
}

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

// One wave copies len bytes src -> dst, any byte alignment of either: a byte
// head up to dst's next 16-B boundary, then aligned 16-B stores whose source
// bytes are funnel-shifted (v_alignbyte) out of 4-B-aligned dword loads (never
// reading past the source range), then a byte tail.  Coalesced both ways.
__device__ __forceinline__ void wave_copy(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint32_t len) {
    const uint32_t lane = lane_id();
    const uint32_t head = min(len, (16u - uint32_t(reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u);
    if (lane < head) dst[lane] = src[lane];
    const uint8_t* s = src + head;
    uint8_t* d = dst + head;
    const uint32_t n = len - head;
    const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(s) & 3u);
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(s - sh);
    // vector v reads s4[4v .. 4v+3] (+ s4[4v+4] when sh != 0): stay inside [s, s+n)
    const uint32_t nvec = sh == 0 ? n / 16u : (n + sh >= 20u ? (n + sh - 20u) / 16u + 1u : 0u);
    for (uint32_t v = lane; v < nvec; v += 64) {
        const uint32_t* q = s4 + 4u * v;
        const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = sh ? q[4] : 0u;
        uint4 o;
        o.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
        o.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
        o.z = __builtin_amdgcn_alignbyte(w3, w2, sh);
        o.w = __builtin_amdgcn_alignbyte(w4, w3, sh);
        *reinterpret_cast<uint4*>(d + 16u * v) = o;
    }
    for (uint32_t i = nvec * 16u + lane; i < n; i += 64) d[i] = s[i];
}

// One wave per physical record that belongs to an emitted logical record.
__global__ void k_reasm_gather(const uint8_t* __restrict__ image, uint64_t image_base,
                               const revel_record_result* __restrict__ phys, uint64_t n,
                               const uint64_t* __restrict__ frag_dst, uint8_t* __restrict__ payload) {
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t w0 = blockIdx.x * (uint64_t)(blockDim.x / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint64_t k = w0; k < n; k += waves) {
        const uint64_t dst = frag_dst[k];
        if (dst == ~0ull) continue;
        const revel_record_result r = phys[k];
        wave_copy(image + (r.file_offset - image_base) + kHeaderSize, payload + dst, r.length);
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

// ---------------------------------------------------------------------------
// Launch helpers
// ---------------------------------------------------------------------------
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

template <int THREADS, bool NT, bool FRAME>
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
            if (r == 0) zero_header_bytes(cur[0], l0, FRAME, &hdr);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                u0 = absorb<TM_S4R>(u0, cur[k].x, L, tab);
                u1 = absorb<TM_S4R>(u1, cur[k].y, L, tab);
                u2 = absorb<TM_S4R>(u2, cur[k].z, L, tab);
                u3 = absorb<TM_S4R>(u3, cur[k].w, L, tab);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < 8; ++k) cur[k] = nxt[k];
        }
        // ---- tree combine: R = XOR_s U_s x^(-32 s) ----
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

template <int THREADS, bool NT, bool FRAME>
hipError_t launch_full3(const DeviceInfo& di, const uint8_t* blocks, uint64_t n, uint32_t* masked, uint8_t* ok,
                        uint8_t* frame_dst, hipStream_t st) {
    auto kern = k_full_blocks3<THREADS, NT, FRAME>;
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

}  // namespace

// ===========================================================================
// Internal entry points (declared in gpu_internal.h)
// ===========================================================================
namespace revel {

// Variant table used by the public entry point and by tools/variants.py.
hipError_t crc_full_blocks_variant(const DeviceInfo& di, int variant, const void* d_blocks, uint64_t n,
                                   uint32_t* d_masked, uint8_t* d_ok, hipStream_t st) {
    const uint8_t* b = static_cast<const uint8_t*>(d_blocks);
    switch (variant) {
        // production: v3 interleaved word streams (gap-folded tables), nt loads
        case 0: return launch_full3<1024, true, false>(di, b, n, d_masked, d_ok, nullptr, st);
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
        default: return hipErrorInvalidValue;
    }
}

hipError_t frame_full_blocks(const DeviceInfo& di, void* d_blocks, uint64_t n, hipStream_t st) {
    uint8_t* b = static_cast<uint8_t*>(d_blocks);
    return launch_full3<1024, true, true>(di, b, n, nullptr, nullptr, b, st);
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

hipError_t count_records(const DeviceInfo& di, const void* d_image, uint64_t nbytes, uint32_t* d_counts,
                         uint64_t* d_hlist, hipStream_t st) {
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    // one lane per block: every header chain walks concurrently
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>(1u << 20, (nblocks + 63) / 64));
    hipLaunchKernelGGL(k_count_records, dim3((uint32_t)grid), dim3(64), 0, st,
                       static_cast<const uint8_t*>(d_image), nbytes, d_counts, d_hlist);
    return hipGetLastError();
}

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
                                 uint32_t lead, const uint64_t* hl, const uint32_t* d_counts, hipStream_t st) {
    hipLaunchKernelGGL((k_verify_records3<FRAME>), dim3((uint32_t)grid), dim3(kVerify2Threads), 0, st, img, nbytes,
                       base_offset, d_first, d_out, lead, hl, d_counts);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !partial) return e;
    // <= 2 partial blocks: one single-wave workgroup each, 4 KiB unreplicated tables
    // (a 128 KiB table fill and one latency-bound wave cost ~50 us per launch)
    hipLaunchKernelGGL((k_verify_records2<FRAME, BP_BYTES, BS_PARTIAL, TM_S4, 64>), dim3(2), dim3(64), 0, st, img,
                       nbytes, base_offset, d_first, d_out, lead, hl, d_counts);
    return hipGetLastError();
}

template <bool FRAME, int BP>
static hipError_t launch_verify2(uint64_t grid, bool partial, const uint8_t* img, uint64_t nbytes,
                                 uint64_t base_offset, const uint32_t* d_first, revel_record_result* d_out,
                                 uint32_t lead, const uint64_t* hl, const uint32_t* d_counts, hipStream_t st) {
    hipLaunchKernelGGL((k_verify_records2<FRAME, BP, BS_WHOLE>), dim3((uint32_t)grid), dim3(kVerify2Threads), 0, st,
                       img, nbytes, base_offset, d_first, d_out, lead, hl, d_counts);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !partial) return e;
    hipLaunchKernelGGL((k_verify_records2<FRAME, BP, BS_PARTIAL>), dim3(1), dim3(kVerify2Threads), 0, st, img, nbytes,
                       base_offset, d_first, d_out, lead, hl, d_counts);
    return hipGetLastError();
}

hipError_t verify_records_variant(const DeviceInfo& di, int variant, const void* d_image, uint64_t nbytes,
                                  uint64_t base_offset, const uint32_t* d_first, revel_record_result* d_out,
                                  const uint64_t* d_hlist, const uint32_t* d_counts, hipStream_t st) {
    const uint64_t nblocks = (nbytes + kBlockSize - 1) / kBlockSize;
    if (variant == 1) {
        const uint64_t waves = kVerifyThreads / 64;
        const uint64_t grid =
            std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu * 2, (nblocks + waves - 1) / waves));
        hipLaunchKernelGGL(k_verify_records, dim3((uint32_t)grid), dim3(kVerifyThreads), 0, st,
                           static_cast<const uint8_t*>(d_image), nbytes, base_offset, d_first, d_out);
        return hipGetLastError();
    }
    hipError_t e0 = ensure_len_tables(di, st);
    if (e0 != hipSuccess) return e0;
    const uint64_t waves = kVerify2Threads / 64;
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu, (nblocks + waves - 1) / waves));
    const uint64_t* hl = variant == 2 ? nullptr : d_hlist;
    const uint8_t* img = static_cast<const uint8_t*>(d_image);
    const bool partial = nbytes % kBlockSize != 0;
    switch (variant) {
        case 3: return launch_verify2<false, BP_MASK>(grid, partial, img, nbytes, base_offset, d_first, d_out, 0u, hl,
                                                      d_counts, st);
        case 4: return launch_verify2<false, BP_MASK_NOVOTE>(grid, partial, img, nbytes, base_offset, d_first, d_out,
                                                             0u, hl, d_counts, st);
        case 5:  // round-1 production: one kernel for whole and partial blocks
            hipLaunchKernelGGL((k_verify_records2<false, BP_BYTES, BS_ALL>), dim3((uint32_t)grid),
                               dim3(kVerify2Threads), 0, st, img, nbytes, base_offset, d_first, d_out, 0u, hl, d_counts);
            return hipGetLastError();
        case 6: return launch_verify2<false, BP_BYTES>(grid, partial, img, nbytes, base_offset, d_first, d_out, 0u,
                                                       hl, d_counts, st);
        case 0:
        case 2: return launch_verify3<false>(grid, partial, img, nbytes, base_offset, d_first, d_out, 0u, hl,
                                             d_counts, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t verify_records(const DeviceInfo& di, const void* d_image, uint64_t nbytes, uint64_t base_offset,
                          const uint32_t* d_first, revel_record_result* d_out, const uint64_t* d_hlist,
                          const uint32_t* d_counts, hipStream_t st) {
    return verify_records_variant(di, 0, d_image, nbytes, base_offset, d_first, d_out, d_hlist, d_counts, st);
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
                         void* d_image, uint64_t image_len, uint32_t lead, hipStream_t st) {
    if (nfrags) {
        const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu * 8, (nfrags + 3) / 4));
        hipLaunchKernelGGL(k_scatter_fragments, dim3((uint32_t)grid), dim3(256), 0, st,
                           static_cast<const uint8_t*>(d_payloads), d_frags, nfrags, static_cast<uint8_t*>(d_image));
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
    return launch_verify3<true>(grid, partial, static_cast<const uint8_t*>(d_image), image_len, 0ull, nullptr, nullptr,
                                lead, nullptr, nullptr, st);
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
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)di.num_cu * 8, (n + 3) / 4));
    hipLaunchKernelGGL(k_reasm_gather, dim3((uint32_t)grid), dim3(256), 0, st, static_cast<const uint8_t*>(d_image),
                       image_base, d_phys, n, d_frag_dst, static_cast<uint8_t*>(d_payload));
    return hipGetLastError();
}

}  // namespace revel
