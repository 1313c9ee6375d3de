// device_common.h -- device helpers shared by the gfx950 kernel files
// (k_blocks.hip, k_records.hip, k_reasm.hip).  Everything here has internal
// linkage (anonymous namespace): each translation unit gets its own copy of
// the constant tables, so no relocatable device code is needed.
//
// The CRC-32C engine for Revel's WAL record path (CDNA4 / gfx950).
//
// Hot path (reference guimingyue/revel @ v0):
//   log_writer.rs:107-111  crc = mask(extend(type, payload))  (writer side)
//   log_reader.rs:200-206  unmask(stored) == value(type||payload) (reader side)
//   util/crc.rs:13-44      CRC_32_ISCSI + mask/unmask
//
// Work decomposition: ONE WAVEFRONT PER 32 KiB LOG BLOCK, read as 32 coalesced
// 1 KiB rows (lane i loads the 16 B at 1024 g + 16 i of row g, through a
// register ring of rows in flight).
//  * C2 (k_full_blocks4, k_blocks.hip): INTERLEAVED WORD STREAMS.  Stream s
//    (0..255) is the 32-bit words at 4 s + 1024 g; lane i owns streams
//    4i..4i+3 (the four words of its 16-B load), four independent CRC chains.
//    Consecutive words of a stream are 1024 B apart, so the slice-by-4 tables
//    are premultiplied by x^(8*1020) (GAP-FOLDED TABLES, GapTables below): one
//    table step absorbs a word AND the 1020 bytes of other streams after it.
//    At the block end the 256 stream registers are combined by an
//    INVERSE-SHIFT TREE: R = XOR_s U_s * x^(-32 s) mod P, 8 levels of 4 table
//    lookups (2 in-lane, 6 across lanes; x is invertible mod P since P(0) = 1).
//  * C3 (k_verify_rows, verify_rows.inc): the same rows, transposed by
//    permlane swaps so lane i owns ONE 4-byte column of each 256-B sub-row (a
//    single chain per lane, 252-B gap tables), with prefix captures at record
//    boundaries reduced by the same kind of inverse-shift tree (the file
//    header of verify_rows.inc has the algebra).
// Init/xorout enter once per record as a length-dependent constant.  No MFMA:
// this is GF(2) arithmetic, not a contraction.
//
// Lookup tables live in LDS, replicated 32x so that lane (l & 31) always hits
// bank (l & 31) for ds_read_b32: bank-conflict-free gathers whatever the data.
// The LDS byte address of entry e for lane l is (e << 8) | ((l & 31) << 2)
// | (region << 16), built by ONE v_perm_b32 per lookup.  The 128 KiB of
// replicated tables (plus the tree tables) fill the CU's LDS, which is why the
// rows are staged in a VGPR ring rather than in LDS.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>

#include "crc32c_math.h"
#include "gpu_internal.h"

namespace {
using namespace revel;

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
        p = __builtin_amdgcn_bitop3_b32(p, b, (uint32_t)__builtin_amdgcn_sbfe((int)a, 31 - k, 1), 0x78);
        if (k < 31) {
            const uint32_t bm = (uint32_t)__builtin_amdgcn_sbfe((int)b, 0, 1);
            b = __builtin_amdgcn_bitop3_b32(b >> 1, bm, kPolyReflected, 0x78);  // s0 ^ (s1 & s2)
        }
    }
    return p;
}

// p1 = a1*b, p2 = a2*b: one shared chain b*x^k, two masked accumulations
// 7 VALU per bit for both products: three v_bitop3 (0x78 = s0 ^ (s1 & s2)),
// three v_bfe, one shift.  The builtins keep the compiler from re-associating
// the chain into a longer form.
__device__ __forceinline__ void gf_mul2(uint32_t b, uint32_t a1, uint32_t a2, uint32_t& p1, uint32_t& p2) {
    uint32_t q1 = 0, q2 = 0;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        q1 = __builtin_amdgcn_bitop3_b32(q1, b, (uint32_t)__builtin_amdgcn_sbfe((int)a1, 31 - k, 1), 0x78);
        q2 = __builtin_amdgcn_bitop3_b32(q2, b, (uint32_t)__builtin_amdgcn_sbfe((int)a2, 31 - k, 1), 0x78);
        if (k < 31) {
            const uint32_t bm = (uint32_t)__builtin_amdgcn_sbfe((int)b, 0, 1);
            b = __builtin_amdgcn_bitop3_b32(b >> 1, bm, kPolyReflected, 0x78);
        }
    }
    p1 = q1;
    p2 = q2;
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
    TM_S4H = 3,  // slice-by-4, 16x replicated, 64 KiB LDS (2-way conflicts, one stage per word; round 5)
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
template <>
struct TableCfg<TM_S4H> {
    static constexpr uint32_t bytes = 65536;
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
        } else if constexpr (TM == TM_S4H) {
            // row e (64 dw = 256 B) -> table slot k (16 dw) -> copy c (lane & 15): byte k of x -> T(3-k)
            uint32_t e = d >> 6, k = (d >> 4) & 3u;
            v = c_tables.t[3 - k][e];
        } else {
            // S2R: row e = [T1 x32 | T0 x32]
            uint32_t e = (d >> 6) & 255u, h = (d >> 5) & 1u;
            v = c_tables.t[1 - h][e];
        }
        tab[d] = v;
    }
}


// Wave priority rotation (s_setprio, an immediate 0..3): the SIMD issues the
// highest-priority ready wave first, then the oldest, so with equal
// priorities a workgroup's older waves run ahead of its younger ones (the C2
// kernel's waves finished at 2.6 / 3.5 / 4.4 / 4.9 ms of 5.2 by age rank,
// profiles/r4/s20_*).  rotate_prio(r) sets priority r & 3; a wave calling it
// with (its age rank + blocks done) takes every priority in turn.  A wave keeps
// its last priority until it exits (a new wave starts at 0).  The gain was
// measured with the verify kernels alone on their stream (DESIGN.md 4.2,
// round 4).  With other work beside them (C5 replay: window i's verify while
// window i+1 lands on the copy stream) the rotation measured neutral: 8 GiB
// records-layout replay, rotation on / off (-DREVEL_DENSE_PRIO=0
// -DREVEL_ROWS_PRIO=0), 6 alternating runs each: ring loader 50.1 / 50.4
// GiB/s end to end, verify 585 / 580 GiB/s; whole-shard verify 5 652 / 5 458
// GiB/s (profiles/r5/late/prio_e2e/).
__device__ __forceinline__ void rotate_prio(uint32_t r) {
    switch (__builtin_amdgcn_readfirstlane(r) & 3u) {
        case 0: __builtin_amdgcn_s_setprio(0); break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        default: __builtin_amdgcn_s_setprio(3); break;
    }
}

struct LaneConst {
    uint32_t lc0, lc1;
};

__device__ __forceinline__ LaneConst make_lane_const() {
    uint32_t c4 = (lane_id() & 31u) << 2;
    return {c4, c4 | 0x10000u};
}
// TM_S4H: the lane's copy among 16
__device__ __forceinline__ LaneConst make_lane_const_h() {
    const uint32_t c4 = (lane_id() & 15u) << 2;
    return {c4, c4};
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
    } else if constexpr (TM == TM_S4H) {
        // address = x_k << 8 | (lane & 15) << 2 (L.lc0 from make_lane_const_h), table k at +64 k
        constexpr uint32_t s0 = 0x0C0C0400u, s1 = 0x0C0C0500u, s2 = 0x0C0C0600u, s3 = 0x0C0C0700u;
        const uint32_t a0 = __builtin_amdgcn_perm(x, L.lc0, s0);
        const uint32_t a1 = __builtin_amdgcn_perm(x, L.lc0, s1);
        const uint32_t a2 = __builtin_amdgcn_perm(x, L.lc0, s2);
        const uint32_t a3 = __builtin_amdgcn_perm(x, L.lc0, s3);
        return (ldsw<0>(tab, a0) ^ ldsw<64>(tab, a1)) ^ (ldsw<128>(tab, a2) ^ ldsw<192>(tab, a3));
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

// x-state form of an S4R step: the chain carries x = crc ^ (next word), so
// the four table words and the following data word fold with two 3-input
// xors (v_bitop3_b32, truth table 0x96) instead of four v_xor_b32.  wn = the
// stream's next word (0 after the last one: then the result is the crc).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t step_x(uint32_t x, uint32_t wn, LaneConst L, const uint32_t* tab) {
    const uint32_t a0 = __builtin_amdgcn_perm(x, L.lc0, Sel<0>::v);
    const uint32_t a1 = __builtin_amdgcn_perm(x, L.lc0, Sel<1>::v);
    const uint32_t a2 = __builtin_amdgcn_perm(x, L.lc1, Sel<2>::v);
    const uint32_t a3 = __builtin_amdgcn_perm(x, L.lc1, Sel<3>::v);
    return xor3(xor3(ldsw<0>(tab, a0), ldsw<128>(tab, a1), ldsw<0>(tab, a2)), ldsw<128>(tab, a3), wn);
}

// The same step with ONE wait for its four lookups: an explicit lgkmcnt(0)
// after the reads, before the first xor (the compiler otherwise waits twice,
// lgkmcnt(1) then lgkmcnt(0)).  For a single dependent chain whose waves are
// bound by instruction issue (k_verify_rows): one s_waitcnt fewer per step.
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }  // lgkmcnt(0) only
__device__ __forceinline__ uint32_t step_x1(uint32_t x, uint32_t wn, LaneConst L, const uint32_t* tab) {
    const uint32_t a0 = __builtin_amdgcn_perm(x, L.lc0, Sel<0>::v);
    const uint32_t a1 = __builtin_amdgcn_perm(x, L.lc0, Sel<1>::v);
    const uint32_t a2 = __builtin_amdgcn_perm(x, L.lc1, Sel<2>::v);
    const uint32_t a3 = __builtin_amdgcn_perm(x, L.lc1, Sel<3>::v);
    const uint32_t t0 = ldsw<0>(tab, a0), t1 = ldsw<128>(tab, a1), t2 = ldsw<0>(tab, a2), t3 = ldsw<128>(tab, a3);
    wait_lgkm0();
    return xor3(xor3(t0, t1, t2), t3, wn);
}

// ---------------------------------------------------------------------------
// Interleaved word streams with the gap folded into the tables (C2 k_full_blocks4,
// C3 k_verify_rows).  A stream is the 32-bit words of a block at a fixed offset
// within every row of ROW bytes; consecutive words of a stream are ROW bytes
// apart, so with T''m = x^(8*(ROW-4)) * Tm one x-state step
//     U <- T''3[x0] ^ T''2[x1] ^ T''1[x2] ^ T''0[x3],   x = U ^ w
// absorbs a word AND the ROW-4 bytes of other streams that follow it (shifting
// is linear, so it distributes over the table xor): T''(v) = v * x^(8*ROW).
// ---------------------------------------------------------------------------
struct GapTables {
    uint32_t t[4][256];  // t[m][e] = x^(8*gap) * T_m[e]
};
constexpr GapTables make_gap_tables(uint32_t gap) {
    GapTables g{};
    const SliceTables st = make_slice_tables();
    const uint32_t c = x8n(gap);
    for (int m = 0; m < 4; ++m)
        for (int e = 0; e < 256; ++e) g.t[m][e] = multmodp(c, st.t[m][e]);
    return g;
}
__constant__ GapTables c_gap1020 = make_gap_tables(1020);  // 1 KiB rows (C2)
__constant__ GapTables c_gap252 = make_gap_tables(252);    // 256-B rows (C3)

constexpr uint32_t pow_modp(uint32_t a, uint64_t n) {
    uint32_t r = 0x80000000u;
    while (n) {
        if (n & 1u) r = multmodp(r, a);
        a = multmodp(a, a);
        n >>= 1;
    }
    return r;
}
constexpr uint32_t kXInv = 0x05EC76F1u;  // x^-1 mod P, reflected (P(0) = 1, so x is invertible)
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

// S4R image of a gap table set (128 KiB, replicated 32x):
// byte0 -> T''3 (r0 h0), byte1 -> T''2 (r0 h1), byte2 -> T''1 (r1 h0), byte3 -> T''0 (r1 h1)
// Four words per ds_write_b128 (the 32 copies of an entry are consecutive
// words, so a 16-B group holds one value): a quarter of the loads and LDS
// writes of a word-by-word fill.  tab must be 16-B aligned.
__device__ void fill_gap_tables(uint32_t* tab, const GapTables& g) {
    for (uint32_t q = threadIdx.x; q < 8192u; q += blockDim.x) {
        const uint32_t d = 4u * q;
        const uint32_t r = d >> 14, e = (d >> 6) & 255u, h = (d >> 5) & 1u;
        const uint32_t v = g.t[3 - (r * 2 + h)][e];
        reinterpret_cast<uint4*>(tab)[q] = make_uint4(v, v, v, v);
    }
}
// Inverse-shift tables, `levels` x 4 KiB unreplicated: level L, byte k, entry e at
// shtab[L*1024 + k*256 + e] = (e << 8k) * x^(-32 * 2^L) mod P.
__device__ void fill_inv_tree_tables(uint32_t* shtab, int levels) {
    for (uint32_t d = threadIdx.x; d < uint32_t(levels) * 1024u; d += blockDim.x) {
        const uint32_t L = d >> 10, k = (d >> 8) & 3u, e = d & 255u;
        shtab[d] = gf_mul(c_inv_tree.c[L], e << (8u * k));
    }
}
// v * (the level-L constant of shtab), four unreplicated lookups.
// acc ^ v * (the level-L constant): two 3-input xors.
template <int L>
__device__ __forceinline__ uint32_t tree_shift_xor(const uint32_t* shtab, uint32_t v, uint32_t acc) {
    const uint32_t* t = shtab + L * 1024;
    return __builtin_amdgcn_bitop3_b32(
        __builtin_amdgcn_bitop3_b32(t[v & 0xffu], t[256 + ((v >> 8) & 0xffu)], t[512 + ((v >> 16) & 0xffu)], 0x96),
        t[768 + (v >> 24)], acc, 0x96);
}
template <int L>
__device__ __forceinline__ uint32_t tree_shift(const uint32_t* shtab, uint32_t v) {
    return tree_shift_xor<L>(shtab, v, 0u);
}
// tree_shift_xor with one wait for its four lookups (see step_x1).
template <int L>
__device__ __forceinline__ uint32_t tree_shift_xor1(const uint32_t* shtab, uint32_t v, uint32_t acc) {
    const uint32_t* t = shtab + L * 1024;
    const uint32_t t0 = t[v & 0xffu], t1 = t[256 + ((v >> 8) & 0xffu)], t2 = t[512 + ((v >> 16) & 0xffu)],
                   t3 = t[768 + (v >> 24)];
    wait_lgkm0();
    return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(t0, t1, t2, 0x96), t3, acc, 0x96);
}
template <int L>
__device__ __forceinline__ uint32_t tree_shift1(const uint32_t* shtab, uint32_t v) {
    return tree_shift_xor1<L>(shtab, v, 0u);
}

template <int TM>
__device__ __forceinline__ uint32_t absorb4(uint32_t crc, uint4 v, LaneConst L, const uint32_t* tab) {
    if constexpr (TM == TM_S4R) {
        // x-state chain over the four words: 1 xor + 7 three-input xors
        // instead of 16 two-input ones
        uint32_t x = crc ^ v.x;
        x = step_x(x, v.y, L, tab);
        x = step_x(x, v.z, L, tab);
        x = step_x(x, v.w, L, tab);
        return step_x(x, 0u, L, tab);
    }
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

// Lane 0 keeps a copy of the block's first 16 bytes (*hdr) and zeroes header
// bytes 0..5 (force_type: the type byte becomes FULL), so the chunk set covers
// exactly block[6:32768).
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

// G lanes (gl = 0..G-1 within the group) copy len bytes src -> dst, any byte
// alignment of either: a byte head up to dst's next 16-B boundary, then
// aligned 16-B stores whose source bytes are funnel-shifted (v_alignbyte) out
// of 4-B-aligned dword loads (never reading past the source range), then a
// byte tail.  Coalesced both ways.  G = 64: the whole wave.
template <uint32_t G>
__device__ __forceinline__ void group_copy(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint32_t len,
                                           uint32_t gl) {
    const uint32_t head = min(len, (16u - uint32_t(reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u);
    for (uint32_t i = gl; i < head; i += G) dst[i] = src[i];
    const uint8_t* s = src + head;
    uint8_t* d = dst + head;
    const uint32_t n = len - head;
    const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(s) & 3u);
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(s - sh);
    // vector v reads s4[4v .. 4v+3] (+ s4[4v+4] when sh != 0): stay inside [s, s+n)
    const uint32_t nvec = sh == 0 ? n / 16u : (n + sh >= 20u ? (n + sh - 20u) / 16u + 1u : 0u);
    for (uint32_t v = gl; v < nvec; v += G) {
        const uint32_t* q = s4 + 4u * v;
        const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = sh ? q[4] : 0u;
        uint4 o;
        o.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
        o.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
        o.z = __builtin_amdgcn_alignbyte(w3, w2, sh);
        o.w = __builtin_amdgcn_alignbyte(w4, w3, sh);
        *reinterpret_cast<uint4*>(d + 16u * v) = o;
    }
    for (uint32_t i = nvec * 16u + gl; i < n; i += G) d[i] = s[i];
}

// A copy of at most kTinyCopy bytes by an 8-lane group, split into a load
// phase and a store phase so that a caller can have several fragments' loads
// in flight before their dependent stores (small-record logs: with one ~131-B
// fragment per group and visit, the copies waited on memory ~90 % of the
// time).  Same layout as group_copy<8>: byte head to dst's 16-B boundary, at
// most one aligned 16-B store per lane funnel-shifted from dwords, byte tail.
// Every load is unconditional (no branch around a load: exact vmcnt waits),
// its address clamped into the source range, or `safe` (4-B aligned, at
// least 4 readable bytes) when that range is empty.
constexpr uint32_t kTinyCopy = 140;  // head <= 15, <= 8 vectors, tail <= 18
struct TinyCopy {
    uint32_t hb[2];  // head bytes gl, gl + 8
    uint32_t w[5];   // source dwords of the lane's 16-B store
    uint32_t tb[3];  // tail bytes gl, gl + 8, gl + 16
};
struct TinyShape {
    uint32_t head, n, sh, nvec;
};
__device__ __forceinline__ TinyShape tiny_shape(const uint8_t* src, const uint8_t* dst, uint32_t len) {
    TinyShape t;
    t.head = min(len, (16u - uint32_t(reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u);
    t.n = len - t.head;
    t.sh = uint32_t(reinterpret_cast<uintptr_t>(src + t.head) & 3u);
    // vector v reads s4[4v .. 4v+3] (+ s4[4v+4] when sh != 0): stay inside [s, s+n)
    t.nvec = t.sh == 0 ? t.n / 16u : (t.n + t.sh >= 20u ? (t.n + t.sh - 20u) / 16u + 1u : 0u);
    return t;
}
__device__ __forceinline__ void tiny_load(const uint8_t* __restrict__ src, const uint8_t* dst, uint32_t len,
                                          uint32_t gl, const uint8_t* safe, TinyCopy& c) {
    const TinyShape t = tiny_shape(src, dst, len);
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) c.hb[k] = len ? src[min(gl + 8u * k, len - 1u)] : safe[0];
    const uint8_t* s = src + t.head;
    const uint32_t* q = t.nvec ? reinterpret_cast<const uint32_t*>(s - t.sh) + 4u * min(gl, t.nvec - 1u)
                               : reinterpret_cast<const uint32_t*>(safe);
    const uint32_t lastw = t.nvec ? (t.sh ? 4u : 3u) : 0u;
#pragma unroll
    for (uint32_t k = 0; k < 5; ++k) c.w[k] = q[min(k, lastw)];
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) c.tb[k] = t.n ? s[min(16u * t.nvec + gl + 8u * k, t.n - 1u)] : safe[0];
}
__device__ __forceinline__ void tiny_store(const uint8_t* src, uint8_t* __restrict__ dst, uint32_t len, uint32_t gl,
                                           const TinyCopy& c) {
    const TinyShape t = tiny_shape(src, dst, len);
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k)
        if (gl + 8u * k < t.head) dst[gl + 8u * k] = (uint8_t)c.hb[k];
    uint8_t* d = dst + t.head;
    if (gl < t.nvec) {
        uint4 o;
        o.x = __builtin_amdgcn_alignbyte(c.w[1], c.w[0], t.sh);
        o.y = __builtin_amdgcn_alignbyte(c.w[2], c.w[1], t.sh);
        o.z = __builtin_amdgcn_alignbyte(c.w[3], c.w[2], t.sh);
        o.w = __builtin_amdgcn_alignbyte(c.w[4], c.w[3], t.sh);
        *reinterpret_cast<uint4*>(d + 16u * gl) = o;
    }
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) {
        const uint32_t i = 16u * t.nvec + gl + 8u * k;
        if (i < t.n) d[i] = (uint8_t)c.tb[k];
    }
}

}  // namespace
