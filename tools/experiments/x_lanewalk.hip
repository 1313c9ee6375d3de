// x_lanewalk.hip -- probe (round 6): ONE LANE PER BLOCK for the small-record
// C3 verify.  Every lane streams its own 32 KiB block in 128-B rounds (one
// lane-owned line per 8-load burst) and runs the reader's header walk AND the
// record checksums in the same pass, one raw dword per step:
//   * the words of a record are aligned to its END e (word [lo, lo + 4) with
//     lo = e mod 4), so its last word ends exactly at e: no pad to take off;
//   * its first word starts up to 3 bytes before the type byte s; the chain
//     starts from those header bytes in position, so they cancel (C ^ w);
//   * when a lane's record ends, the raw CRC is compared with
//     unmask(stored) ^ init_xor(len + 1) (looked up when the header was read),
//     the header-list entry is written, and the next header -- the 7 bytes
//     right after e, in the lane's next three dwords -- is parsed.
// No count pass, no cross-lane combining.  Variants for the probe:
//   VAR 0: the loads only (lane-per-block memory pattern), MAP 0 contiguous
//          blocks per wave, MAP 1 strided;
//   VAR 1: loads + one CRC chain per lane over the whole block;
//   VAR 2: the full walk + checksums (entries, counts);
//   VAR 3: VAR 2 with the record's steps as u = K + negF in [0, nwm1] (fewer instructions);
//   VAR 4-6: timing probes of the chain: no loads / 2 / 4 independent chains per lane;
//   VAR 8: one continuous chain over the raw dwords + header captures (k_lw8_expand finishes);
//   VAR 9: VAR 8 with the headers handled once per 4-dword batch;
//   VAR 10-12: VAR 0 / 1 / 9 with quad-coalesced loads + DPP transpose;
//   VAR 7: branch-free steps (the next header parsed by every lane while the lookups are in
//          flight), 16-B entries {stored, len | type << 16, raw CRC, offset} in hlist.
// Built into tools/experiments/libxlw.so (make -C tools/experiments xlw).
#include "device_common.h"

namespace {

constexpr int kLwThreads = 512;  // 8 waves: one workgroup per CU beside the 128 KiB tables

__device__ uint32_t g_lw_init_xor[kBlockSize + 2];  // init_xor(n): the raw CRC of n bytes vs crc32c's
__device__ uint32_t g_lw_x8n[kBlockSize + 2];       // x^(8 n) mod P

__global__ void k_lw_init() {
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d <= kBlockSize + 1u; d += gridDim.x * blockDim.x) {
        uint32_t x = 0x80000000u;  // x^(8 d)
        const uint32_t x8 = x8n(1);
        uint32_t a = x8, n = d;
        while (n) {
            if (n & 1u) x = multmodp(x, a);
            a = multmodp(a, a);
            n >>= 1;
        }
        g_lw_init_xor[d] = multmodp(x, 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
        g_lw_x8n[d] = x;
    }
}

template <int VAR, int NBUF, bool QUAD = false>
__global__ __launch_bounds__(kLwThreads) void k_lw(const uint8_t* __restrict__ image, uint64_t nblocks,
                                                  uint32_t* __restrict__ counts, uint64_t* __restrict__ hlist,
                                                  uint32_t* __restrict__ hcrc, uint32_t* __restrict__ sink,
                                                  uint32_t map) {
    __shared__ uint32_t tab[VAR >= 1 ? 32768 : 1];
    if constexpr (VAR >= 1) {
        fill_tables<TM_S4R>(tab);
        __syncthreads();
    }
    const LaneConst L = make_lane_const();
    const uint32_t lane = lane_id();
    const uint64_t gw = (uint64_t(blockIdx.x) * kLwThreads + threadIdx.x) >> 6;
    const uint64_t nw = uint64_t(gridDim.x) * (kLwThreads / 64);
    const uint64_t b = map == 0 ? gw * 64u + lane : uint64_t(lane) * nw + gw;
    const bool live = b < nblocks;
    // per-lane global loads (a buffer resource per lane would be a waterfall loop); rounds past
    // the block re-read its last one (wave-uniform clamp), lanes past the image read block 0
    const u32x4* const src = reinterpret_cast<const u32x4*>(image + (live ? b * kBlockSize : 0));
    u32x4 V[NBUF][8];
    // QUAD: instruction (g, k) has lane 4Q+p load piece 4g+p of the block of lane 4Q+k (64
    // contiguous bytes per quad: 16 lines per instruction instead of 64); settle() transposes
    // the 4x4 pieces inside the quad (two DPP butterfly stages) before the round is used
    const uint32_t qp = lane & 3u;
    typedef __attribute__((address_space(1))) const u32x4 gu32x4;  // global, not flat (flat loads count in lgkmcnt too)
    gu32x4* srcq[4] = {(gu32x4*)src, (gu32x4*)src, (gu32x4*)src, (gu32x4*)src};
    if constexpr (QUAD) {
        const uint64_t sv = reinterpret_cast<uint64_t>(src);
        const uint32_t lo = uint32_t(sv), hi = uint32_t(sv >> 32);
#define LW_BQ(k, ctrl)                                                                                        \
    srcq[k] = (gu32x4*)(                                                                                      \
        (uint64_t(uint32_t(__builtin_amdgcn_mov_dpp((int)hi, ctrl, 0xF, 0xF, true))) << 32) |                 \
        uint32_t(__builtin_amdgcn_mov_dpp((int)lo, ctrl, 0xF, 0xF, true)));
        LW_BQ(0, 0x00) LW_BQ(1, 0x55) LW_BQ(2, 0xAA) LW_BQ(3, 0xFF)
#undef LW_BQ
    }
    auto load = [&](u32x4* v, uint32_t r) {
        const uint32_t rr = r < kBlockSize / 128u ? r : kBlockSize / 128u - 1u;
        if constexpr (QUAD) {
#pragma unroll
            for (int g = 0; g < 2; ++g)
#pragma unroll
                for (int k = 0; k < 4; ++k) v[4 * g + k] = srcq[k][8u * rr + 4u * uint32_t(g) + qp];
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = src[8u * rr + uint32_t(i)];
        }
    };
    auto settle = [&](u32x4* v) __attribute__((always_inline)) {
        if constexpr (QUAD) {
#pragma unroll
            for (int g = 0; g < 2; ++g) {
#define LW_QSTAGE(S, CTRL)                                                                           \
    _Pragma("unroll") for (int k0 = 0; k0 < 4; ++k0) {                                               \
        if (k0 & (S)) continue;                                                                      \
        const int k1 = k0 | (S);                                                                     \
        const bool hi_ = (qp & (S)) != 0u;                                                           \
        u32x4& r0 = v[4 * g + k0];                                                                   \
        u32x4& r1 = v[4 * g + k1];                                                                   \
        const u32x4 snd = {hi_ ? r0.x : r1.x, hi_ ? r0.y : r1.y, hi_ ? r0.z : r1.z, hi_ ? r0.w : r1.w}; \
        const u32x4 rcv = {(uint32_t)__builtin_amdgcn_mov_dpp((int)snd.x, CTRL, 0xF, 0xF, true),      \
                           (uint32_t)__builtin_amdgcn_mov_dpp((int)snd.y, CTRL, 0xF, 0xF, true),      \
                           (uint32_t)__builtin_amdgcn_mov_dpp((int)snd.z, CTRL, 0xF, 0xF, true),      \
                           (uint32_t)__builtin_amdgcn_mov_dpp((int)snd.w, CTRL, 0xF, 0xF, true)};     \
        r0 = hi_ ? rcv : r0;                                                                         \
        r1 = hi_ ? r1 : rcv;                                                                         \
    }
                LW_QSTAGE(1, 0xB1)
                LW_QSTAGE(2, 0x4E)
#undef LW_QSTAGE
            }
        }
    };
    uint32_t acc = 0, acc2 = 0, acc3 = 0, acc4 = 0;
    uint64_t* const hl = hlist + (live ? b : 0) * kListStride;
    uint32_t* const hc = hcrc + (live ? b : 0) * kListStride;
    uint32_t t = 0, C = 0, sh = 0, h0 = 0, hi = 0;
    // VAR 2 state: CRC range [s, e) of the open record
    uint32_t s = 0xFFFFFFFFu, e = 0xFFFFFFFFu;
    // VAR 3 state: the record's words are absorbed at steps K with u = K + negF in [0, nwm1]
    uint32_t negF = 0x80000000u, nwm1 = 0;
    // VAR 7 state: u = K + 1 - G in [0, nwm1]; pc = the record's header offset
    uint32_t G = 0x40000000u, pc = 0;
    u32x4* const he = reinterpret_cast<u32x4*>(hlist) + (live ? b : 0) * kListStride;
    // VAR 8 state: the next header at np, in dword npK (walk ended: ~0)
    uint32_t np = 0, npK = live ? 0u : 0xFFFFFFFFu;
    // header at p (bytes p..p+7 = a | b << 32): a record (its range, C from its lead bytes), a
    // status record (bad length / zero: listed, the walk ends), or the block's trailer
    auto parse = [&](uint32_t p, uint32_t a, uint32_t bb) __attribute__((always_inline)) {
        const uint32_t len = bb & 0xFFFFu;
        const uint32_t ne = p + kHeaderSize + len;
        const bool fits = p <= kBlockSize - kHeaderSize;
        const bool bad = fits && (ne > kBlockSize || (bb & 0xFFFFFFu) == 0u);
        const bool ok = fits && !bad;
        h0 = a;
        hi = bb & 0xFFFFFFu;
        if (__builtin_expect(bad, 0)) {
            const uint32_t ts = t < kListCap ? t : kListCap;
            hl[ts] = uint64_t(a) | (uint64_t(hi) << 32);
            hc[ts] = 0u;
            ++t;
        }
        // the first word starts 3 - (len & 3) bytes before the type byte: those header bytes,
        // in position, are the chain's start (they cancel in C ^ w)
        const uint32_t o = (len & 3u) << 3;
        C = __builtin_amdgcn_ubfe(__builtin_amdgcn_alignbyte(bb, a, 3u), o, 24u - o);
        sh = ne & 3u;
        if constexpr (VAR == 2) {
            s = ok ? p + 6u : 0xFFFFFFFFu;
            e = ok ? ne : 0xFFFFFFFFu;
        } else {
            const uint32_t w1 = len >> 2;  // words - 1
            nwm1 = ok ? w1 : 0u;
            negF = ok ? w1 + 1u - (ne >> 2) : 0x80000000u;
        }
    };
    auto finish = [&]() __attribute__((always_inline)) {
        // the raw CRC goes out beside the entry: the expander compares it with
        // unmask(stored) ^ init_xor(len + 1)
        const uint32_t ts = t < kListCap ? t : kListCap;
        hl[ts] = uint64_t(h0) | (uint64_t(hi) << 32);
        hc[ts] = C;
        ++t;
    };
    auto step = [&](uint32_t K, uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3) __attribute__((always_inline)) {
        if constexpr (VAR == 0) {
            acc ^= d0;
        } else if constexpr (VAR == 1) {
            acc = absorb<TM_S4R>(acc, d0, L, tab);
        } else if constexpr (VAR == 4) {  // chain only: data from the step index (no loads used)
            acc = absorb<TM_S4R>(acc, K * 0x9E3779B1u, L, tab);
        } else if constexpr (VAR == 5) {  // two independent chains per lane (even / odd steps), loads used
            if (K & 1u) acc2 = absorb<TM_S4R>(acc2, d0, L, tab);
            else acc = absorb<TM_S4R>(acc, d0, L, tab);
        } else if constexpr (VAR == 6) {  // four independent chains per lane
            if ((K & 3u) == 0u) acc = absorb<TM_S4R>(acc, d0, L, tab);
            else if ((K & 3u) == 1u) acc2 = absorb<TM_S4R>(acc2, d0, L, tab);
            else if ((K & 3u) == 2u) acc3 = absorb<TM_S4R>(acc3, d0, L, tab);
            else acc4 = absorb<TM_S4R>(acc4, d0, L, tab);
        } else if constexpr (VAR == 8) {
            // ONE chain per lane over the raw dwords (no restarts, no alignment): C = S(4K), the
            // raw CRC of the block's bytes [0, 4K).  The walk only captures S at each header's
            // dword, with the bytes of that dword before the header; the expander turns two
            // consecutive captures into the record's checksum (linearity).
            const uint32_t Cb = C;
            C = absorb<TM_S4R>(C, d0, L, tab);
            if (K == npK) {
                const uint32_t j = np & 3u;
                const uint32_t st = __builtin_amdgcn_alignbyte(d1, d0, j);
                const uint32_t lt = __builtin_amdgcn_alignbyte(d2, d1, j);
                const uint32_t pre = __builtin_amdgcn_ubfe(d0, 0u, 8u * j);
                const uint32_t len = lt & 0xFFFFu, h24 = lt & 0xFFFFFFu;
                const bool fits = np <= kBlockSize - kHeaderSize;
                const uint32_t ne = np + kHeaderSize + len;
                const bool ok = fits && ne <= kBlockSize && h24 != 0u;
                // a record's entry, or the walk's end (not counted): {stored, len | type << 16 |
                // p << 24, S(p & ~3), bytes [p & ~3, p) | (p >> 8) << 24}
                he[t < kListCap ? t : kListCap] = u32x4{st, h24 | (np << 24), Cb, pre | ((np >> 8) << 24)};
                t += fits ? 1u : 0u;
                np = ne;
                npK = ok ? ne >> 2 : 0xFFFFFFFFu;
            }
        } else if constexpr (VAR == 7) {
            // branch-free: the table lookups issue first; everything that does not need the chain
            // (the header after this word, the next record's state) is computed for every lane
            // while they are in flight (sched_barrier + the asm pin keep it there); the new state
            // is selected where the record ends
            const uint32_t u = K + 1u - G;
            const bool in = u <= nwm1, done = u == nwm1;
            const uint32_t x = C ^ __builtin_amdgcn_alignbyte(d1, d0, sh);
            const uint32_t a0 = __builtin_amdgcn_perm(x, L.lc0, Sel<0>::v);
            const uint32_t a1 = __builtin_amdgcn_perm(x, L.lc0, Sel<1>::v);
            const uint32_t a2 = __builtin_amdgcn_perm(x, L.lc1, Sel<2>::v);
            const uint32_t a3 = __builtin_amdgcn_perm(x, L.lc1, Sel<3>::v);
            const uint32_t t0 = ldsw<0>(tab, a0), t1 = ldsw<128>(tab, a1), t2 = ldsw<0>(tab, a2), t3 = ldsw<128>(tab, a3);
            __builtin_amdgcn_sched_barrier(0);
            uint32_t a = __builtin_amdgcn_alignbyte(d2, d1, sh), bb = __builtin_amdgcn_alignbyte(d3, d2, sh);
            uint32_t p = 4u * K + 4u + sh;
            const uint32_t len = bb & 0xFFFFu;
            uint32_t nhi = bb & 0xFFFFFFu;
            const uint32_t ne = p + kHeaderSize + len;
            const bool fits = p <= kBlockSize - kHeaderSize;
            const bool okx = fits && ne <= kBlockSize && nhi != 0u;
            uint32_t stat = fits && !okx ? 1u : 0u;
            const uint32_t o = (len & 3u) << 3;
            uint32_t cinit = __builtin_amdgcn_ubfe(__builtin_amdgcn_alignbyte(bb, a, 3u), o, 24u - o);
            uint32_t nG = okx ? (ne >> 2) - (len >> 2) : 0x40000000u;
            uint32_t nn = okx ? (len >> 2) : 0u;
            uint32_t nsh = ne & 3u;
            asm volatile("" : "+v"(a), "+v"(nhi), "+v"(p), "+v"(cinit), "+v"(nG), "+v"(nn), "+v"(nsh), "+v"(stat));
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t nc = xor3(t0, t1, t2) ^ t3;
            const uint32_t Cn = in ? nc : C;
            if (done) {
                he[t < kListCap ? t : kListCap] = u32x4{h0, hi, Cn, pc};
                ++t;
                if (__builtin_expect(stat != 0u, 0)) {  // bad length / zero: a status record ends the walk
                    he[t < kListCap ? t : kListCap] = u32x4{a, nhi, 0u, p};
                    ++t;
                }
            }
            C = done ? cinit : Cn;
            G = done ? nG : G;
            nwm1 = done ? nn : nwm1;
            sh = done ? nsh : sh;
            h0 = done ? a : h0;
            hi = done ? nhi : hi;
            pc = done ? p : pc;
        } else if constexpr (VAR == 2) {
            const uint32_t lo4 = 4u * K + 4u + sh;  // the end of this step's word
            const uint32_t w = __builtin_amdgcn_alignbyte(d1, d0, sh);
            const bool in = lo4 > s && lo4 <= e;
            const uint32_t nc = absorb<TM_S4R>(C, w, L, tab);
            C = in ? nc : C;
            if (lo4 == e) {
                finish();
                // the next header: bytes e.. = byte sh of d1 on
                parse(lo4, __builtin_amdgcn_alignbyte(d2, d1, sh), __builtin_amdgcn_alignbyte(d3, d2, sh));
            }
        } else {
            const uint32_t u = K + negF;
            const uint32_t w = __builtin_amdgcn_alignbyte(d1, d0, sh);
            const uint32_t nc = absorb<TM_S4R>(C, w, L, tab);
            C = u <= nwm1 ? nc : C;
            if (u == nwm1) {
                finish();
                const uint32_t p = 4u * K + 4u + sh;
                parse(p, __builtin_amdgcn_alignbyte(d2, d1, sh), __builtin_amdgcn_alignbyte(d3, d2, sh));
            }
        }
    };
    // VAR 9: batches of four dwords (16 B): one chain step per dword, and the headers that
    // start in the batch handled once per batch (a select of the dword among four), not per step
    auto sel4 = [](uint32_t i, uint32_t a, uint32_t b_, uint32_t c, uint32_t d) __attribute__((always_inline)) {
        const uint32_t lo = (i & 1u) ? b_ : a, hi2 = (i & 1u) ? d : c;
        return (i & 2u) ? hi2 : lo;
    };
    auto batch = [&](uint32_t m, const uint32_t* d) __attribute__((always_inline)) {
        const uint32_t c0 = C;
        const uint32_t c1 = absorb<TM_S4R>(c0, d[0], L, tab);
        const uint32_t c2 = absorb<TM_S4R>(c1, d[1], L, tab);
        const uint32_t c3 = absorb<TM_S4R>(c2, d[2], L, tab);
        C = absorb<TM_S4R>(c3, d[3], L, tab);
        // at most three headers start in 16 B (7-byte records): three straight-line passes, the
        // later ones skipped unless a lane has another header in the batch (no loop: a loop
        // around the stores made the compiler wait for every load in flight)
#pragma unroll
        for (int rep = 0; rep < 3; ++rep) {
            if ((np >> 4) == m && npK != 0xFFFFFFFFu) {
                const uint32_t i = (np >> 2) & 3u, j = np & 3u;
                const uint32_t x0 = sel4(i, d[0], d[1], d[2], d[3]);
                const uint32_t x1 = sel4(i, d[1], d[2], d[3], d[4]);
                const uint32_t x2 = sel4(i, d[2], d[3], d[4], d[5]);
                const uint32_t cap = sel4(i, c0, c1, c2, c3);
                const uint32_t st = __builtin_amdgcn_alignbyte(x1, x0, j);
                const uint32_t lt = __builtin_amdgcn_alignbyte(x2, x1, j);
                const uint32_t pre = __builtin_amdgcn_ubfe(x0, 0u, 8u * j);
                const uint32_t len = lt & 0xFFFFu, h24 = lt & 0xFFFFFFu;
                const bool fits = np <= kBlockSize - kHeaderSize;
                const uint32_t ne = np + kHeaderSize + len;
                const bool ok = fits && ne <= kBlockSize && h24 != 0u;
                he[t < kListCap ? t : kListCap] = u32x4{st, h24 | (np << 24), cap, pre | ((np >> 8) << 24)};
                t += fits ? 1u : 0u;
                np = ne;
                npK = ok ? ne >> 2 : 0xFFFFFFFFu;
            }
        }
    };
    // round r's 32 dwords in cur, round r + 1's in nxt (the window's last three dwords)
#define LW_ROUND(cur, nxt, r)                                                                                      \
    {                                                                                                              \
        uint32_t D_[36];                                                                                           \
        _Pragma("unroll") for (int i = 0; i < 8; ++i) {                                                            \
            D_[4 * i] = cur[i].x;                                                                                  \
            D_[4 * i + 1] = cur[i].y;                                                                              \
            D_[4 * i + 2] = cur[i].z;                                                                              \
            D_[4 * i + 3] = cur[i].w;                                                                              \
        }                                                                                                          \
        D_[32] = nxt[0].x;                                                                                         \
        D_[33] = nxt[0].y;                                                                                         \
        D_[34] = nxt[0].z;                                                                                         \
        D_[35] = nxt[0].w;                                                                                         \
        if constexpr (VAR == 9) {                                                                                  \
            _Pragma("unroll") for (int k = 0; k < 8; ++k) batch(8u * (r) + uint32_t(k), &D_[4 * k]);                 \
        } else {                                                                                                   \
            _Pragma("unroll") for (int k = 0; k < 32; ++k) step(32u * (r) + uint32_t(k), D_[k], D_[k + 1], D_[k + 2], D_[k + 3]); \
        }                                                                                                          \
    }
#pragma unroll
    for (int j = 0; j + 1 < NBUF; ++j) load(V[j], uint32_t(j));
    settle(V[0]);
    if constexpr (VAR == 2 || VAR == 3) {
        // the first header (round 0 must have landed)
        if (live) parse(0u, V[0][0].x, V[0][0].y);
    }
    if constexpr (VAR == 7) {
        const uint32_t a = V[0][0].x, bb = V[0][0].y;
        const uint32_t len = bb & 0xFFFFu, nhi = bb & 0xFFFFFFu, ne = kHeaderSize + len;
        const bool okx = ne <= kBlockSize && nhi != 0u;
        if (live && !okx) {
            he[0] = u32x4{a, nhi, 0u, 0u};
            t = 1;
        }
        const uint32_t o = (len & 3u) << 3;
        C = __builtin_amdgcn_ubfe(__builtin_amdgcn_alignbyte(bb, a, 3u), o, 24u - o);
        G = live && okx ? (ne >> 2) - (len >> 2) : 0x40000000u;
        nwm1 = live && okx ? (len >> 2) : 0u;
        sh = ne & 3u;
        h0 = a;
        hi = nhi;
        pc = 0;
    }
    constexpr uint32_t R = kBlockSize / 128u;  // 256 rounds
    // sched_barrier: each round's eight loads issue together, NBUF - 1 rounds ahead of their use
    // (without it the scheduler spread them through the round with vmcnt waits between)
    for (uint32_t r = 0; r < R; r += NBUF) {
#pragma unroll
        for (int j = 0; j < NBUF; ++j) {
            __builtin_amdgcn_sched_barrier(0);
            load(V[(j + NBUF - 1) % NBUF], r + uint32_t(j + NBUF - 1));
            __builtin_amdgcn_sched_barrier(0);
            settle(V[(j + 1) % NBUF]);  // the next round (its first dwords end this one)
            LW_ROUND(V[j], V[(j + 1) % NBUF], r + uint32_t(j))
            if (r + uint32_t(j) + 1u >= R) break;
        }
    }
#undef LW_ROUND
    if constexpr (VAR == 8 || VAR == 9) {
        // a walk that reached the block end exactly: its end capture is the chain's total
        if (npK == kBlockSize / 4u) he[t < kListCap ? t : kListCap] = u32x4{0u, 0u, C, (kBlockSize >> 8) << 24};
    }
    if constexpr (VAR == 2 || VAR == 3 || VAR >= 7) {
        if (live) counts[b] = t;
    } else {
        sink[gw * 64u + lane] = acc ^ acc2 ^ acc3 ^ acc4;
    }
}

// VAR 8's expander (probe): record t of block b from entries t and t + 1 -> its crc32c
__device__ __forceinline__ uint32_t lw_byte(uint32_t c, uint32_t byte) {
    return c_tables.t[0][(c ^ byte) & 0xFFu] ^ (c >> 8);
}
__global__ void k_lw8_expand(const uint64_t* __restrict__ hlist, const uint32_t* __restrict__ counts,
                             const uint32_t* __restrict__ first, uint32_t* __restrict__ out, uint64_t nblocks) {
    const u32x4* const he = reinterpret_cast<const u32x4*>(hlist);
    const uint32_t lane = lane_id();
    for (uint64_t b = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6; b < nblocks;
         b += (uint64_t(gridDim.x) * blockDim.x) >> 6) {
        const uint32_t n = counts[b], f = first[b];
        for (uint32_t t = lane; t < n && t < kListCap; t += 64u) {
            const u32x4 E = he[b * kListStride + t], F = he[b * kListStride + t + 1u];
            const uint32_t p = (E.y >> 24) | ((E.w >> 24) << 8), len = E.y & 0xFFFFu;
            uint32_t crc = 0;
            if (p + kHeaderSize + len <= kBlockSize && (E.y & 0xFFFFFFu) != 0u) {
                // S(p + 6): the capture, then the bytes before the header, then 6 header bytes
                uint32_t c = E.z;
                const uint32_t j = p & 3u;
                for (uint32_t i = 0; i < j; ++i) c = lw_byte(c, E.w >> (8u * i));
                for (uint32_t i = 0; i < 4u; ++i) c = lw_byte(c, E.x >> (8u * i));
                c = lw_byte(c, len);
                c = lw_byte(c, len >> 8);
                // S(e): the next capture and the bytes before the next header
                const uint32_t pn = (F.y >> 24) | ((F.w >> 24) << 8);
                uint32_t se = F.z;
                for (uint32_t i = 0; i < (pn & 3u); ++i) se = lw_byte(se, F.w >> (8u * i));
                const uint32_t raw = se ^ gf_mul(c, g_lw_x8n[len + 1u]);
                crc = mask(raw ^ g_lw_init_xor[len + 1u]);
            }
            out[f + t] = crc;
        }
    }
}

}  // namespace

extern "C" {
// init_xor(n) for n = 0..32769 into dst (the checker's table: raw CRC ^ init_xor(n) = crc32c)
int xlw_init_xor(uint32_t* dst, void* stream) {
    hipLaunchKernelGGL(k_lw_init, dim3(64), dim3(256), 0, (hipStream_t)stream);
    if (hipGetLastError() != hipSuccess) return -1;
    return hipMemcpyFromSymbolAsync(dst, HIP_SYMBOL(g_lw_init_xor), sizeof(g_lw_init_xor), 0, hipMemcpyDeviceToDevice,
                                    (hipStream_t)stream) == hipSuccess ? 0 : -1;
}
// var 0/1/2, map 0/1 (var 0 only); nblocks whole 32 KiB blocks; sink: one u32 per lane of the grid
// var 0..3 (VAR 0: map 0/1), nbuf 3 or 4 round buffers; nblocks whole 32 KiB blocks;
// sink: one u32 per lane of the grid
int xlw_launch(int var, int map, const void* image, uint64_t nblocks, uint32_t* counts, uint64_t* hlist,
               uint32_t* hcrc, uint32_t* sink, void* stream) {
    const uint64_t waves = (nblocks + 63) / 64;
    const uint32_t grid = (uint32_t)((waves + (kLwThreads / 64) - 1) / (kLwThreads / 64));
    const hipStream_t st = (hipStream_t)stream;
    const uint8_t* img = static_cast<const uint8_t*>(image);
    const uint32_t mp = (uint32_t)(map & 1);
    const int nbuf = map >> 1 ? 4 : 3;  // map bit 1: four round buffers
#define XLW(V, N) hipLaunchKernelGGL((k_lw<V, N>), dim3(grid), dim3(kLwThreads), 0, st, img, nblocks, counts, hlist, hcrc, sink, mp)
    if (var >= 10) {  // QUAD loads: 10 = loads only, 11 = + one chain, 12 = the batched walk
#define XLWQ(V, N) hipLaunchKernelGGL((k_lw<V, N, true>), dim3(grid), dim3(kLwThreads), 0, st, img, nblocks, counts, hlist, hcrc, sink, mp)
        if (var == 10) XLWQ(0, 3); else if (var == 11) XLWQ(1, 3); else XLWQ(9, 3);
#undef XLWQ
    } else if (var == 9) {
        if (nbuf == 3) XLW(9, 3); else XLW(9, 4);
    } else if (var == 8) {
        if (nbuf == 3) XLW(8, 3); else XLW(8, 4);
    } else if (var == 7) {
        if (nbuf == 3) XLW(7, 3); else XLW(7, 4);
    } else if (var >= 4) {
        if (var == 4) XLW(4, 3); else if (var == 5) XLW(5, 3); else XLW(6, 3);
    } else if (nbuf == 3) {
        if (var == 0) XLW(0, 3); else if (var == 1) XLW(1, 3); else if (var == 2) XLW(2, 3); else XLW(3, 3);
    } else {
        if (var == 0) XLW(0, 4); else if (var == 1) XLW(1, 4); else if (var == 2) XLW(2, 4); else XLW(3, 4);
    }
#undef XLW
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
// VAR 8's expander: crc32c of every listed record into out[first[b] + t]
int xlw_expand8(const void* hlist, const uint32_t* counts, const uint32_t* first, uint32_t* out, uint64_t nblocks,
                void* stream) {
    hipLaunchKernelGGL(k_lw8_expand, dim3(2048), dim3(256), 0, (hipStream_t)stream, (const uint64_t*)hlist, counts,
                       first, out, nblocks);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
uint64_t xlw_sink_words(uint64_t nblocks) {
    const uint64_t waves = (nblocks + 63) / 64;
    const uint64_t grid = (waves + (kLwThreads / 64) - 1) / (kLwThreads / 64);
    return grid * kLwThreads;
}
}
