// crc32c_math.h -- compile-time CRC-32C tables and GF(2) helpers shared by the
// host library and the gfx950 kernels.
//
// Parameter set: CRC_32_ISCSI as used by src/util/crc.rs:13-15 (crate `crc`
// ^3.0.0): reflected polynomial 0x82F63B78, init 0xFFFFFFFF, xorout
// 0xFFFFFFFF.  Everything here is constexpr so the device tables are
// constant-initialised and the per-lane combine constants are folded.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define REVEL_HD __host__ __device__
#else
#define REVEL_HD
#endif

namespace revel {

constexpr uint32_t kPolyReflected = 0x82F63B78u;
constexpr uint32_t kMaskDelta = 0xa282ead8u;       // crc.rs:29
constexpr uint32_t kBlockSize = 32768u;            // log_format.rs:27
constexpr uint32_t kHeaderSize = 7u;               // log_format.rs:30
constexpr uint32_t kFullPayload = kBlockSize - kHeaderSize;  // 32761
constexpr uint32_t kFullCrcLen = kFullPayload + 1;           // type byte + payload

// Slicing tables: T[0] is the classic bytewise table; T[k][n] is the register
// contribution of byte n followed by k zero bytes.
struct SliceTables {
    uint32_t t[8][256];
};

constexpr SliceTables make_slice_tables() {
    SliceTables s{};
    for (uint32_t n = 0; n < 256; ++n) {
        uint32_t c = n;
        for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ kPolyReflected : (c >> 1);
        s.t[0][n] = c;
    }
    for (int k = 1; k < 8; ++k)
        for (uint32_t n = 0; n < 256; ++n)
            s.t[k][n] = (s.t[k - 1][n] >> 8) ^ s.t[0][s.t[k - 1][n] & 0xffu];
    return s;
}

// a * b mod P, reflected representation (bit 31 = coefficient of x^0).
REVEL_HD constexpr uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (int k = 0; k < 32; ++k) {
        if (a & (0x80000000u >> k)) p ^= b;
        b = (b & 1u) ? (b >> 1) ^ kPolyReflected : (b >> 1);
    }
    return p;
}

// x^(8n) mod P.
REVEL_HD constexpr uint32_t x8n(uint64_t n) {
    uint32_t result = 0x80000000u;  // x^0
    uint32_t sq = 0x40000000u;      // x^1
    uint64_t k = 8 * n;
    while (k) {
        if (k & 1u) result = multmodp(sq, result);
        sq = multmodp(sq, sq);
        k >>= 1;
    }
    return result;
}

// Register-domain shift: the raw state after `s` is followed by n zero bytes.
REVEL_HD constexpr uint32_t shift_bytes(uint32_t s, uint64_t n) { return multmodp(x8n(n), s); }

// crc(msg) = R(msg, 0) ^ init_xor(len) where R is the zero-initialised raw
// register walk: init_xor(n) = shift(0xFFFFFFFF, n) ^ 0xFFFFFFFF.
REVEL_HD constexpr uint32_t init_xor(uint64_t n) { return shift_bytes(0xFFFFFFFFu, n) ^ 0xFFFFFFFFu; }

REVEL_HD constexpr uint32_t mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + kMaskDelta; }
REVEL_HD constexpr uint32_t unmask(uint32_t m) {
    uint32_t rot = m - kMaskDelta;
    return (rot >> 17) | (rot << 15);
}

static_assert(make_slice_tables().t[0][1] == 0xF26B8303u, "CRC-32C table");
static_assert(init_xor(0) == 0u, "empty message");

}  // namespace revel
