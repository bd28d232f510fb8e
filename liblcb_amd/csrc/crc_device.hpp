// crc_device.hpp — CRC-32 family of include/math/crc32.h on gfx950.
//
// One lane per buffer (the register chain is serial, like the digests).  The
// reference runs one byte per step through a 256-entry table
// (crc32_normal8 crc32.h:61-73, crc32_reflect8 crc32.h:101-113; its 4-bit
// tables below 64 bytes compute the same function).  Here the same recurrence
// is applied 8 bytes at a time (slicing-by-8): table k holds the register
// contribution of a byte followed by k zero bytes, so one step XORs eight
// lookups.  The eight 1 KiB tables of the variant's polynomial are generated
// at compile time from the polynomial (pinned against the reference's tables
// by tests/test_crc32_gpu.py) and staged into LDS per workgroup.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hash_device.hpp"

namespace lcbgpu {

struct CrcTables {
    uint32_t t[8][256];
};

constexpr uint32_t crc_bitrev32(uint32_t x) {
    uint32_t r = 0;
    for (int i = 0; i < 32; ++i)
        if ((x >> i) & 1u) r |= 1u << (31 - i);
    return r;
}

// t[0]: the reference's byte table (bit-serial definition of each rule);
// t[k]: t[k-1] advanced by one zero byte.
constexpr CrcTables make_crc_tables(uint32_t poly, bool reflect) {
    CrcTables T{};
    const uint32_t rp = crc_bitrev32(poly);
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = reflect ? i : i << 24;
        for (int k = 0; k < 8; ++k) {
            if (reflect) c = (c & 1u) ? (c >> 1) ^ rp : c >> 1;
            else c = (c & 0x80000000u) ? (c << 1) ^ poly : c << 1;
        }
        T.t[0][i] = c;
    }
    for (int k = 1; k < 8; ++k)
        for (int i = 0; i < 256; ++i) {
            const uint32_t p = T.t[k - 1][i];
            T.t[k][i] = reflect ? (p >> 8) ^ T.t[0][p & 0xffu] : (p << 8) ^ T.t[0][p >> 24];
        }
    return T;
}

// Table families: the five (polynomial, bit order) pairs of crc32.h:126-494.
__device__ const CrcTables kCrcTabDev[5] = {
    make_crc_tables(0x04c11db7u, false),   // crc32_tbl256_04c11db7
    make_crc_tables(0x04c11db7u, true),    // crc32_tbl256_edb88320
    make_crc_tables(0x1edc6f41u, true),    // crc32_tbl256_1edc6f41
    make_crc_tables(0xa833982bu, true),    // crc32_tbl256_a833982b
    make_crc_tables(0x814141abu, false),   // crc32_tbl256_814141ab
};

// Variant v (ids of include/lcb_crc32_gpu.h) -> crc32.h:501-576:
//   X_update(c, d, n) = inv ? ~rule(~c) : rule(c);  X(d, n) = X_update(oneshot, d, n).
template <int V>
struct CrcVar {
    static constexpr int kFam = V <= 3 ? 0 : V <= 5 ? 1 : V == 6 ? 2 : V == 7 ? 3 : 4;
    static constexpr bool kRefl = kFam >= 1 && kFam <= 3;
    static constexpr bool kInv = V == 1 || V == 2 || V == 4 || V == 6 || V == 7;
    static constexpr uint32_t kOneshot = (V == 2 || V == 3 || V == 5) ? 0xffffffffu : 0u;
};

__device__ __forceinline__ void crc_stage_tables(uint32_t* lds, int fam) {
    const uint4* src = reinterpret_cast<const uint4*>(&kCrcTabDev[fam].t[0][0]);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (int i = threadIdx.x; i < 512; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

template <bool kRefl>
struct CrcRule {
    const uint32_t* T;  // LDS [8][256]

    __device__ __forceinline__ uint32_t at(int k, uint32_t b) const { return T[k * 256 + b]; }

    // 8 message bytes = raw LE words w0, w1.
    __device__ __forceinline__ uint32_t step8(uint32_t r, uint32_t w0, uint32_t w1) const {
        if (kRefl) {
            const uint32_t x = r ^ w0;
            return xor3(xor3(at(7, x & 255u), at(6, (x >> 8) & 255u), at(5, (x >> 16) & 255u)),
                        xor3(at(4, x >> 24), at(3, w1 & 255u), at(2, (w1 >> 8) & 255u)),
                        at(1, (w1 >> 16) & 255u) ^ at(0, w1 >> 24));
        } else {
            const uint32_t x = r ^ bswap32(w0), y = bswap32(w1);
            return xor3(xor3(at(7, x >> 24), at(6, (x >> 16) & 255u), at(5, (x >> 8) & 255u)),
                        xor3(at(4, x & 255u), at(3, y >> 24), at(2, (y >> 16) & 255u)),
                        at(1, (y >> 8) & 255u) ^ at(0, y & 255u));
        }
    }
    // 4 message bytes = raw LE word w.
    __device__ __forceinline__ uint32_t step4(uint32_t r, uint32_t w) const {
        if (kRefl) {
            const uint32_t x = r ^ w;
            return xor3(at(3, x & 255u), at(2, (x >> 8) & 255u), at(1, (x >> 16) & 255u)) ^ at(0, x >> 24);
        } else {
            const uint32_t x = r ^ bswap32(w);
            return xor3(at(3, x >> 24), at(2, (x >> 16) & 255u), at(1, (x >> 8) & 255u)) ^ at(0, x & 255u);
        }
    }
    // One byte b: crc32.h:110 / crc32.h:70.
    __device__ __forceinline__ uint32_t step1(uint32_t r, uint32_t b) const {
        if (kRefl) return (r >> 8) ^ at(0, (r ^ b) & 255u);
        return (r << 8) ^ at(0, ((r >> 24) ^ b) & 255u);
    }
};

// Register value after the whole message (before the variant's output ~).
template <class Rule>
__device__ __forceinline__ uint32_t crc_message(const Rule& R, uint32_t r, const uint8_t* msg, uint64_t len) {
    const uint8_t* p = msg;
    const uint64_t nline = len >> 7;
    for (uint64_t k = 0; k < nline; ++k, p += 128) {
        uint32_t a[16], b[16];
        load_full128(p, a, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) r = R.step8(r, a[2 * j], a[2 * j + 1]);
#pragma unroll
        for (int j = 0; j < 8; ++j) r = R.step8(r, b[2 * j], b[2 * j + 1]);
    }
    uint32_t rem = (uint32_t)(len & 127u);
    if (rem >= 64) {
        uint32_t w[16];
        load_full64(p, w);
#pragma unroll
        for (int j = 0; j < 8; ++j) r = R.step8(r, w[2 * j], w[2 * j + 1]);
        p += 64;
        rem -= 64;
    }
    if (rem) {
        uint32_t w[16];
        load_tail64(p, rem, w);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int valid = (int)rem - 4 * k;
            if (valid >= 4) {
                r = R.step4(r, w[k]);
            } else if (valid > 0) {
#pragma unroll
                for (int b = 0; b < 3; ++b)
                    if (b < valid) r = R.step1(r, (w[k] >> (8 * b)) & 255u);
            }
        }
    }
    return r;
}

}  // namespace lcbgpu
