// hash_device.hpp — per-lane compression functions and message drivers for
// the MI355X (gfx950) batch digest kernels.
//
// Mapping: ONE LANE PER MESSAGE.  Merkle-Damgard (MD5/SHA) and Streebog chain
// every block through the previous state, so the 64 lanes of a wavefront each
// carry an independent message ("one wavefront per buffer" vs the
// serial chain).  All state lives in VGPRs; rounds are fully unrolled with
// compile-time indices so nothing spills to scratch.  The only memory traffic
// is the message bytes (read once) and the digest (written once).
//
// Bit-exactness notes:
//  * message words are loaded as raw little-endian u32; SHA policies byte-swap
//    them (v_perm_b32) inside compress();
//  * counts are bytes; bit length = bytes << 3 (md5.h:282, sha2.h:725-731);
//  * GOST pads with 0x01 and never emits a length block
//    (gost3411-2012.h:1820-1837).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

namespace lcbgpu {

// ------------------------------------------------------------ primitives
// Mark a kernel-argument pointer as global memory.  Pointers read out of the
// by-value KArgs struct are otherwise generic, and generic loads compile to
// flat_load, which also counts against lgkmcnt: every wait for an LDS table
// read would then wait for outstanding HBM loads as well.  The address-space
// cast lets the compiler's address-space inference turn them into
// global_load.
template <class T>
__device__ __forceinline__ T* gptr(T* p) {
    return (T*)(__attribute__((address_space(1))) T*)p;
}

__device__ __forceinline__ uint32_t rotl32(uint32_t x, uint32_t n) {
    return __builtin_amdgcn_alignbit(x, x, 32u - n);  // v_alignbit_b32
}
__device__ __forceinline__ uint32_t rotr32(uint32_t x, uint32_t n) {
    return __builtin_amdgcn_alignbit(x, x, n);
}
__device__ __forceinline__ uint64_t rotr64(uint64_t x, uint32_t n) {
    return (x >> n) | (x << (64u - n));
}
__device__ __forceinline__ uint32_t bswap32(uint32_t x) {
    return __builtin_amdgcn_perm(0u, x, 0x00010203u);  // v_perm_b32
}
// Any 3-input boolean function in one VALU op (gfx950 v_bitop3_b32); the
// immediate is the truth table over (a, b, c) = (0xf0, 0xcc, 0xaa).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t ch3(uint32_t x, uint32_t y, uint32_t z) {   // (x & y) | (~x & z)
    return __builtin_amdgcn_bitop3_b32(x, y, z, 0xca);
}
__device__ __forceinline__ uint32_t maj3(uint32_t x, uint32_t y, uint32_t z) {  // majority
    return __builtin_amdgcn_bitop3_b32(x, y, z, 0xe8);
}
// Plain-C forms for wave-uniform operands: no VALU-only builtins, so values
// derived from kernel arguments stay on the scalar ALU (s_lshr/s_lshl/s_or).
// (A 32-bit rotate written as shifts is re-formed into rotr, which only has a
// VALU pattern; the 64-bit shift of the doubled word keeps it scalar.)
__device__ __forceinline__ uint32_t srotr32(uint32_t x, uint32_t n) {
    return (uint32_t)((((uint64_t)x << 32) | x) >> n);
}
__device__ __forceinline__ uint64_t srotr64(uint64_t x, uint32_t n) { return (x >> n) | (x << (64u - n)); }

// 64-bit values as explicit (lo, hi) halves so rotates are v_alignbit pairs.
struct u64p {
    uint32_t lo, hi;
};
__device__ __forceinline__ u64p mk64(uint64_t v) { return u64p{(uint32_t)v, (uint32_t)(v >> 32)}; }
__device__ __forceinline__ uint64_t v64(u64p a) { return ((uint64_t)a.hi << 32) | a.lo; }
template <int N>
__device__ __forceinline__ u64p rotr64p(u64p x) {
    if (N < 32) return u64p{__builtin_amdgcn_alignbit(x.hi, x.lo, N), __builtin_amdgcn_alignbit(x.lo, x.hi, N)};
    return u64p{__builtin_amdgcn_alignbit(x.lo, x.hi, N - 32), __builtin_amdgcn_alignbit(x.hi, x.lo, N - 32)};
}
template <int N>  // N < 32
__device__ __forceinline__ u64p shr64p(u64p x) {
    return u64p{__builtin_amdgcn_alignbit(x.hi, x.lo, N), x.hi >> N};
}
__device__ __forceinline__ u64p xor3p(u64p a, u64p b, u64p c) {
    return u64p{xor3(a.lo, b.lo, c.lo), xor3(a.hi, b.hi, c.hi)};
}
__device__ __forceinline__ u64p add64p(u64p a, u64p b) { return mk64(v64(a) + v64(b)); }
// 64-bit add as one v_lshl_add_u64 on register pairs.  Written as asm because
// the compiler otherwise splits ((hi << 32) | lo) + y into a zero-extended low
// add, a separate 32-bit high add and pair-building moves (measured on the
// SHA-512 block: 1096 v_lshl_add_u64 + 542 v_mov_b32 + 108 v_add_u32 where
// 752 adds suffice).
__device__ __forceinline__ uint64_t add64(uint64_t a, uint64_t b) {
    uint64_t r;
    asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ uint64_t add64k(uint64_t a, uint64_t k) {  // k wave-uniform
    uint64_t r;
    asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(a), "s"(k));
    return r;
}

// ------------------------------------------------------- block loading
// Bytes [p, p+64) of a message that has at least 64 bytes left, as 16 raw LE
// words.  Any alignment.  Every dword loaded contains >= 1 message byte, so
// no access leaves the buffer the caller described.
__device__ __forceinline__ void load_full64(const uint8_t* p, uint32_t w[16]) {
    const uintptr_t ip = reinterpret_cast<uintptr_t>(p);
    if ((ip & 15u) == 0) {
        const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 v = q[k];
            w[4 * k + 0] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
        }
    } else if ((ip & 3u) == 0) {
        const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = q[k];
    } else {
        const uint32_t sh = (uint32_t)(ip & 3u);
        const uint32_t* q = reinterpret_cast<const uint32_t*>(p - sh);
        uint32_t d[17];
#pragma unroll
        for (int k = 0; k < 17; ++k) d[k] = q[k];
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
    }
}

// Bytes [p, p+128) of a message with >= 128 bytes left: one whole cache line
// per lane when 16-B aligned (both halves requested together, so the line is
// fetched from HBM once even when L2 is under pressure).
__device__ __forceinline__ void load_full128(const uint8_t* p, uint32_t w0[16], uint32_t w1[16]) {
    const uintptr_t ip = reinterpret_cast<uintptr_t>(p);
    if ((ip & 15u) == 0) {
        const uint4* q = reinterpret_cast<const uint4*>(p);
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = q[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            w0[4 * k + 0] = v[k].x; w0[4 * k + 1] = v[k].y; w0[4 * k + 2] = v[k].z; w0[4 * k + 3] = v[k].w;
            w1[4 * k + 0] = v[k + 4].x; w1[4 * k + 1] = v[k + 4].y; w1[4 * k + 2] = v[k + 4].z;
            w1[4 * k + 3] = v[k + 4].w;
        }
    } else {
        load_full64(p, w0);
        load_full64(p + 64, w1);
    }
}

// Bytes [p, p+rem) (0 <= rem < 64) as raw LE words; bytes >= rem are zero.
__device__ __forceinline__ void load_tail64(const uint8_t* p, uint32_t rem, uint32_t w[16]) {
    const uintptr_t ip = reinterpret_cast<uintptr_t>(p);
    const uint32_t sh = (uint32_t)(ip & 3u);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p - sh);
    const uint32_t lim = rem + sh;  // aligned dword j holds a message byte iff 4j < lim
    uint32_t d[17];
#pragma unroll
    for (int k = 0; k < 17; ++k) d[k] = (4u * k < lim) ? q[k] : 0u;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t v = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
        const int valid = (int)rem - 4 * k;  // bytes of word k inside the message
        const uint32_t mask = valid >= 4 ? 0xffffffffu
                            : (valid <= 0 ? 0u : (0xffffffffu >> (32 - 8 * valid)));
        w[k] = v & mask;
    }
}

// OR the bytes p[lo .. hi) (0 <= lo <= hi <= 64) into raw LE byte positions
// lo .. hi of w.  `p` itself may lie outside the caller's buffer: only the
// aligned dwords holding at least one byte of [p + lo, p + hi) are loaded.
__device__ __forceinline__ void or_window64(const uint8_t* p, uint32_t lo, uint32_t hi, uint32_t w[16]) {
    const uintptr_t ip = reinterpret_cast<uintptr_t>(p);
    const uint32_t sh = (uint32_t)(ip & 3u);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p - sh);
    // aligned dword k holds p bytes [4k - sh, 4k + 4 - sh)
    uint32_t d[17];
#pragma unroll
    for (int k = 0; k < 17; ++k) d[k] = (4u * k < hi + sh && 4u * k + 4u > lo + sh) ? q[k] : 0u;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t v = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
        // bytes of word k inside [lo, hi)
        const int b0 = (int)lo - 4 * k, b1 = (int)hi - 4 * k;
        const uint32_t mlo = b0 <= 0 ? 0xffffffffu : (b0 >= 4 ? 0u : (0xffffffffu << (8 * b0)));
        const uint32_t mhi = b1 >= 4 ? 0xffffffffu : (b1 <= 0 ? 0u : (0xffffffffu >> (32 - 8 * b1)));
        w[k] |= v & mlo & mhi;
    }
}

// or_window64 for a buffer padded by at least 68 readable bytes before and
// after the window (the device key table, lcb_hash_gpu.cpp key_table): the
// 68-byte span is read with four 16-B loads and one dword, unconditionally,
// instead of 17 predicated dword loads.
__device__ __forceinline__ void or_window64_padded(const uint8_t* p, uint32_t lo, uint32_t hi, uint32_t w[16]) {
    typedef uint32_t v4a __attribute__((ext_vector_type(4), aligned(4)));
    const uintptr_t ip = reinterpret_cast<uintptr_t>(p);
    const uint32_t sh = (uint32_t)(ip & 3u);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p - sh);
    uint32_t d[17];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const v4a v = *reinterpret_cast<const v4a*>(q + 4 * k);
        d[4 * k] = v.x; d[4 * k + 1] = v.y; d[4 * k + 2] = v.z; d[4 * k + 3] = v.w;
    }
    d[16] = q[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t v = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
        const int b0 = (int)lo - 4 * k, b1 = (int)hi - 4 * k;
        const uint32_t mlo = b0 <= 0 ? 0xffffffffu : (b0 >= 4 ? 0u : (0xffffffffu << (8 * b0)));
        const uint32_t mhi = b1 >= 4 ? 0xffffffffu : (b1 <= 0 ? 0u : (0xffffffffu >> (32 - 8 * b1)));
        w[k] |= v & mlo & mhi;
    }
}

// Bytes [pos, pos + 64) of the virtual message V = A[0, la) || B[0, lb) as
// raw LE words; bytes at or past la + lb are zero.  Keyed batches
// (lcb_hash_batch_keyed) hash key || message and message || key this way
// without a copy of either.
__device__ __forceinline__ void load_vblock64(const uint8_t* A, uint64_t la, const uint8_t* B, uint64_t lb,
                                              uint64_t pos, uint32_t w[16]) {
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = 0u;
    if (pos < la) {
        const uint64_t n = la - pos;
        or_window64(A + pos, 0, n < 64 ? (uint32_t)n : 64u, w);
    }
    const uint64_t end = la + lb;
    if (pos + 64 > la && pos < end) {
        const uint64_t b = pos > la ? pos : la;       // first V byte taken from B
        const uint32_t s0 = (uint32_t)(b - pos);
        const uint64_t e = pos + 64 < end ? pos + 64 : end;
        or_window64(B + (b - la) - s0, s0, (uint32_t)(e - pos), w);
    }
}

// OR byte value `b` into raw LE byte position `pos` (0..63) of w.
__device__ __forceinline__ void put_byte(uint32_t w[16], uint32_t pos, uint32_t b) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
        w[k] |= ((pos >> 2) == (uint32_t)k) ? (b << (8u * (pos & 3u))) : 0u;
}

// ================================================================== MD5
// md5.h:137-229.  Round functions in their bitop3-friendly forms.
struct Md5 {
    // kOcc: waves per SIMD (second __launch_bounds__ argument of the
    // per-lane kernel).  kPairLoad: read whole 128-B lines (both halves
    // requested together).  kLdsStream: fixed-stride batches take the LDS-DMA
    // line stream.  kScalarPad: the pad-only block's schedule runs on the
    // SALU (md_pad_only).
    static constexpr int kBlock = 64, kDigest = 16, kLenBytes = 8, kWords = 16, kOcc = 8;
    static constexpr bool kPairLoad = true;   // HBM-bound: read whole 128-B lines
    static constexpr bool kLdsStream = true;
    static constexpr bool kScalarPad = false;  // no schedule to move: pad block via compress()
    static constexpr int kTileOcc = 4;         // md_tiles_kernel: waves per SIMD (0: not used)
    uint32_t s[4];
    __device__ __forceinline__ void init() {
        s[0] = 0x67452301u; s[1] = 0xefcdab89u; s[2] = 0x98badcfeu; s[3] = 0x10325476u;
    }
    // x + T as one v_add_u32 with T as an inline literal, the asm hiding the
    // constant from loop-invariant code motion: in a kernel with several
    // inlined compressions in loops (md_tiles_kernel) the compiler otherwise
    // parks all 64 T in SGPRs, which pushed its other scalars into VGPR lanes
    // and its VGPRs into scratch.
    template <uint32_t T>
    __device__ __forceinline__ static uint32_t addk(uint32_t x) {
        uint32_t r;
        asm("v_add_u32 %0, %1, %2" : "=v"(r) : "i"(T), "v"(x));
        return r;
    }
#define LCB_MD5_STEP(f, a, b, c, d, x, t, r) \
    a = b + rotl32(kLit ? addk<t>(a + (f) + (x)) : a + (f) + (x) + (t), r)
    // kLit: T added last through addk (see there; after a + F + x, so the asm
    // cannot be hoisted ahead of its step either).
    template <bool kLit = true>
    __device__ __forceinline__ void compress(const uint32_t* w) {
        uint32_t a = s[0], b = s[1], c = s[2], d = s[3];
#define F1(b, c, d) ch3((b), (c), (d))
#define F2(b, c, d) ch3((d), (b), (c))
#define F3(b, c, d) xor3((b), (c), (d))
#define F4(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0x39)
        LCB_MD5_STEP(F1(b, c, d), a, b, c, d, w[0], 0xd76aa478u, 7);
        LCB_MD5_STEP(F1(a, b, c), d, a, b, c, w[1], 0xe8c7b756u, 12);
        LCB_MD5_STEP(F1(d, a, b), c, d, a, b, w[2], 0x242070dbu, 17);
        LCB_MD5_STEP(F1(c, d, a), b, c, d, a, w[3], 0xc1bdceeeu, 22);
        LCB_MD5_STEP(F1(b, c, d), a, b, c, d, w[4], 0xf57c0fafu, 7);
        LCB_MD5_STEP(F1(a, b, c), d, a, b, c, w[5], 0x4787c62au, 12);
        LCB_MD5_STEP(F1(d, a, b), c, d, a, b, w[6], 0xa8304613u, 17);
        LCB_MD5_STEP(F1(c, d, a), b, c, d, a, w[7], 0xfd469501u, 22);
        LCB_MD5_STEP(F1(b, c, d), a, b, c, d, w[8], 0x698098d8u, 7);
        LCB_MD5_STEP(F1(a, b, c), d, a, b, c, w[9], 0x8b44f7afu, 12);
        LCB_MD5_STEP(F1(d, a, b), c, d, a, b, w[10], 0xffff5bb1u, 17);
        LCB_MD5_STEP(F1(c, d, a), b, c, d, a, w[11], 0x895cd7beu, 22);
        LCB_MD5_STEP(F1(b, c, d), a, b, c, d, w[12], 0x6b901122u, 7);
        LCB_MD5_STEP(F1(a, b, c), d, a, b, c, w[13], 0xfd987193u, 12);
        LCB_MD5_STEP(F1(d, a, b), c, d, a, b, w[14], 0xa679438eu, 17);
        LCB_MD5_STEP(F1(c, d, a), b, c, d, a, w[15], 0x49b40821u, 22);

        LCB_MD5_STEP(F2(b, c, d), a, b, c, d, w[1], 0xf61e2562u, 5);
        LCB_MD5_STEP(F2(a, b, c), d, a, b, c, w[6], 0xc040b340u, 9);
        LCB_MD5_STEP(F2(d, a, b), c, d, a, b, w[11], 0x265e5a51u, 14);
        LCB_MD5_STEP(F2(c, d, a), b, c, d, a, w[0], 0xe9b6c7aau, 20);
        LCB_MD5_STEP(F2(b, c, d), a, b, c, d, w[5], 0xd62f105du, 5);
        LCB_MD5_STEP(F2(a, b, c), d, a, b, c, w[10], 0x02441453u, 9);
        LCB_MD5_STEP(F2(d, a, b), c, d, a, b, w[15], 0xd8a1e681u, 14);
        LCB_MD5_STEP(F2(c, d, a), b, c, d, a, w[4], 0xe7d3fbc8u, 20);
        LCB_MD5_STEP(F2(b, c, d), a, b, c, d, w[9], 0x21e1cde6u, 5);
        LCB_MD5_STEP(F2(a, b, c), d, a, b, c, w[14], 0xc33707d6u, 9);
        LCB_MD5_STEP(F2(d, a, b), c, d, a, b, w[3], 0xf4d50d87u, 14);
        LCB_MD5_STEP(F2(c, d, a), b, c, d, a, w[8], 0x455a14edu, 20);
        LCB_MD5_STEP(F2(b, c, d), a, b, c, d, w[13], 0xa9e3e905u, 5);
        LCB_MD5_STEP(F2(a, b, c), d, a, b, c, w[2], 0xfcefa3f8u, 9);
        LCB_MD5_STEP(F2(d, a, b), c, d, a, b, w[7], 0x676f02d9u, 14);
        LCB_MD5_STEP(F2(c, d, a), b, c, d, a, w[12], 0x8d2a4c8au, 20);

        LCB_MD5_STEP(F3(b, c, d), a, b, c, d, w[5], 0xfffa3942u, 4);
        LCB_MD5_STEP(F3(a, b, c), d, a, b, c, w[8], 0x8771f681u, 11);
        LCB_MD5_STEP(F3(d, a, b), c, d, a, b, w[11], 0x6d9d6122u, 16);
        LCB_MD5_STEP(F3(c, d, a), b, c, d, a, w[14], 0xfde5380cu, 23);
        LCB_MD5_STEP(F3(b, c, d), a, b, c, d, w[1], 0xa4beea44u, 4);
        LCB_MD5_STEP(F3(a, b, c), d, a, b, c, w[4], 0x4bdecfa9u, 11);
        LCB_MD5_STEP(F3(d, a, b), c, d, a, b, w[7], 0xf6bb4b60u, 16);
        LCB_MD5_STEP(F3(c, d, a), b, c, d, a, w[10], 0xbebfbc70u, 23);
        LCB_MD5_STEP(F3(b, c, d), a, b, c, d, w[13], 0x289b7ec6u, 4);
        LCB_MD5_STEP(F3(a, b, c), d, a, b, c, w[0], 0xeaa127fau, 11);
        LCB_MD5_STEP(F3(d, a, b), c, d, a, b, w[3], 0xd4ef3085u, 16);
        LCB_MD5_STEP(F3(c, d, a), b, c, d, a, w[6], 0x04881d05u, 23);
        LCB_MD5_STEP(F3(b, c, d), a, b, c, d, w[9], 0xd9d4d039u, 4);
        LCB_MD5_STEP(F3(a, b, c), d, a, b, c, w[12], 0xe6db99e5u, 11);
        LCB_MD5_STEP(F3(d, a, b), c, d, a, b, w[15], 0x1fa27cf8u, 16);
        LCB_MD5_STEP(F3(c, d, a), b, c, d, a, w[2], 0xc4ac5665u, 23);

        LCB_MD5_STEP(F4(b, c, d), a, b, c, d, w[0], 0xf4292244u, 6);
        LCB_MD5_STEP(F4(a, b, c), d, a, b, c, w[7], 0x432aff97u, 10);
        LCB_MD5_STEP(F4(d, a, b), c, d, a, b, w[14], 0xab9423a7u, 15);
        LCB_MD5_STEP(F4(c, d, a), b, c, d, a, w[5], 0xfc93a039u, 21);
        LCB_MD5_STEP(F4(b, c, d), a, b, c, d, w[12], 0x655b59c3u, 6);
        LCB_MD5_STEP(F4(a, b, c), d, a, b, c, w[3], 0x8f0ccc92u, 10);
        LCB_MD5_STEP(F4(d, a, b), c, d, a, b, w[10], 0xffeff47du, 15);
        LCB_MD5_STEP(F4(c, d, a), b, c, d, a, w[1], 0x85845dd1u, 21);
        LCB_MD5_STEP(F4(b, c, d), a, b, c, d, w[8], 0x6fa87e4fu, 6);
        LCB_MD5_STEP(F4(a, b, c), d, a, b, c, w[15], 0xfe2ce6e0u, 10);
        LCB_MD5_STEP(F4(d, a, b), c, d, a, b, w[6], 0xa3014314u, 15);
        LCB_MD5_STEP(F4(c, d, a), b, c, d, a, w[13], 0x4e0811a1u, 21);
        LCB_MD5_STEP(F4(b, c, d), a, b, c, d, w[4], 0xf7537e82u, 6);
        LCB_MD5_STEP(F4(a, b, c), d, a, b, c, w[11], 0xbd3af235u, 10);
        LCB_MD5_STEP(F4(d, a, b), c, d, a, b, w[2], 0x2ad7d2bbu, 15);
        LCB_MD5_STEP(F4(c, d, a), b, c, d, a, w[9], 0xeb86d391u, 21);
#undef F1
#undef F2
#undef F3
#undef F4
        s[0] += a; s[1] += b; s[2] += c; s[3] += d;
    }
#undef LCB_MD5_STEP
    // md5.h:282: LE u64 bit length in bytes 56..63.
    __device__ __forceinline__ static void put_length(uint32_t* w, uint64_t bytes) {
        const uint64_t bits = bytes << 3;
        w[14] = (uint32_t)bits; w[15] = (uint32_t)(bits >> 32);
    }
    // md5.h:285: state bytes LE.
    __device__ __forceinline__ void digest_words(uint32_t* out) const {
#pragma unroll
        for (int i = 0; i < 4; ++i) out[i] = s[i];
    }
};

// ================================================================ SHA-1
// sha1.h:220-292 with a 16-word rolling schedule.
struct Sha1 {
    static constexpr int kBlock = 64, kDigest = 20, kLenBytes = 8, kWords = 16, kOcc = 8;
    static constexpr bool kPairLoad = true;
    static constexpr bool kLdsStream = true;
    static constexpr bool kScalarPad = true;
    // Ragged batches: the tile kernel at 2 waves per SIMD (182-192 VGPRs, no
    // scratch; at 3 or 4 it spills): packets 2-3 % faster than per-lane, C4 equal
    // (profiles/r3_sha_tiles_ab.txt).
    static constexpr int kTileOcc = 2;
    uint32_t s[5];
    __device__ __forceinline__ void init() {
        s[0] = 0x67452301u; s[1] = 0xefcdab89u; s[2] = 0x98badcfeu; s[3] = 0x10325476u;
        s[4] = 0xc3d2e1f0u;
    }
    __device__ __forceinline__ void compress(const uint32_t* raw) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = bswap32(raw[i]);
        rounds<false>(w);
    }
    // Pad-only block (0x80, zeros, BE bit length) from a wave-uniform length:
    // the schedule is scalar work (see md_pad_only).
    __device__ __forceinline__ void compress_pad(uint64_t bytes) {
        uint32_t w[16] = {0x80000000u};
        w[14] = (uint32_t)(bytes >> 29); w[15] = (uint32_t)(bytes << 3);
        rounds<true>(w);
    }
    template <bool kUniform>  // w: BE words
    __device__ __forceinline__ void rounds(uint32_t (&w)[16]) {
        uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4];
#pragma unroll
        for (int i = 0; i < 80; ++i) {
            uint32_t x;
            if (i < 16) {
                x = w[i];
            } else {
                if (kUniform) {
                    const uint32_t y = w[(i - 3) & 15] ^ w[(i - 8) & 15] ^ w[(i - 14) & 15] ^ w[i & 15];
                    x = srotr32(y, 31);
                } else {
                    x = rotl32(xor3(w[(i - 3) & 15], w[(i - 8) & 15], w[(i - 14) & 15] ^ w[i & 15]), 1);
                }
                w[i & 15] = x;
            }
            uint32_t f, k;
            if (i < 20) { f = ch3(b, c, d); k = 0x5a827999u; }
            else if (i < 40) { f = xor3(b, c, d); k = 0x6ed9eba1u; }
            else if (i < 60) { f = maj3(b, c, d); k = 0x8f1bbcdcu; }
            else { f = xor3(b, c, d); k = 0xca62c1d6u; }
            const uint32_t t = kUniform ? rotl32(a, 5) + f + e + (k + x) : rotl32(a, 5) + f + e + k + x;
            e = d; d = c; c = rotl32(b, 30); b = a; a = t;
        }
        s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e;
    }
    // sha1.h:833: BE u64 bit length.
    __device__ __forceinline__ static void put_length(uint32_t* w, uint64_t bytes) {
        const uint64_t bits = bytes << 3;
        w[14] = bswap32((uint32_t)(bits >> 32)); w[15] = bswap32((uint32_t)bits);
    }
    // sha1.h:837: BE state.
    __device__ __forceinline__ void digest_words(uint32_t* out) const {
#pragma unroll
        for (int i = 0; i < 5; ++i) out[i] = bswap32(s[i]);
    }
};

// ============================================================ SHA-224/256
// sha2.h:260-327.
__constant__ static const uint32_t kSha256K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

template <bool k224>
struct Sha256 {
    static constexpr int kBlock = 64, kDigest = k224 ? 28 : 32, kLenBytes = 8, kWords = 16, kOcc = 4;
    static constexpr bool kPairLoad = false;  // VALU-bound: fewer live VGPRs
    // Line stream on: 2.4 % faster than direct loads (profiles/r1_sha2_lds_ab.txt).
    static constexpr bool kLdsStream = true;
    static constexpr bool kScalarPad = true;
    // Ragged batches: the tile kernel at 2 waves per SIMD (179-194 VGPRs, no
    // scratch): C4 6 % faster than per-lane, packets 2 % slower
    // (profiles/r3_sha_tiles_ab.txt).
    static constexpr int kTileOcc = 2;
    uint32_t s[8];
    __device__ __forceinline__ void init() {
        if (k224) {  // sha2.h:129-132
            s[0] = 0xc1059ed8u; s[1] = 0x367cd507u; s[2] = 0x3070dd17u; s[3] = 0xf70e5939u;
            s[4] = 0xffc00b31u; s[5] = 0x68581511u; s[6] = 0x64f98fa7u; s[7] = 0xbefa4fa4u;
        } else {     // sha2.h:134-137
            s[0] = 0x6a09e667u; s[1] = 0xbb67ae85u; s[2] = 0x3c6ef372u; s[3] = 0xa54ff53au;
            s[4] = 0x510e527fu; s[5] = 0x9b05688cu; s[6] = 0x1f83d9abu; s[7] = 0x5be0cd19u;
        }
    }
    __device__ __forceinline__ void compress(const uint32_t* raw) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = bswap32(raw[i]);
        rounds<false>(w);
    }
    // Pad-only block from a wave-uniform length (scalar schedule, md_pad_only).
    __device__ __forceinline__ void compress_pad(uint64_t bytes) {
        uint32_t w[16] = {0x80000000u};
        w[14] = (uint32_t)(bytes >> 29); w[15] = (uint32_t)(bytes << 3);
        rounds<true>(w);
    }
    template <bool kUniform>  // w: BE words
    __device__ __forceinline__ void rounds(uint32_t (&w)[16]) {
        uint32_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
        for (int i = 0; i < 64; ++i) {
            uint32_t x;
            if (i < 16) {
                x = w[i];
            } else {
                const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
                uint32_t s0, s1;
                if (kUniform) {
                    s0 = srotr32(w15, 7) ^ srotr32(w15, 18) ^ (w15 >> 3);
                    s1 = srotr32(w2, 17) ^ srotr32(w2, 19) ^ (w2 >> 10);
                } else {
                    s0 = xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
                    s1 = xor3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
                }
                x = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
                w[i & 15] = x;
            }
            const uint32_t S1 = xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
            const uint32_t ch = ch3(e, f, g);
            const uint32_t t1 = kUniform ? h + S1 + ch + (kSha256K[i] + x) : h + S1 + ch + kSha256K[i] + x;
            const uint32_t S0 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
            const uint32_t mj = maj3(a, b, c);
            h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
        }
        s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
    }
    __device__ __forceinline__ static void put_length(uint32_t* w, uint64_t bytes) {
        const uint64_t bits = bytes << 3;  // sha2.h:726
        w[14] = bswap32((uint32_t)(bits >> 32)); w[15] = bswap32((uint32_t)bits);
    }
    __device__ __forceinline__ void digest_words(uint32_t* out) const {
#pragma unroll
        for (int i = 0; i < kDigest / 4; ++i) out[i] = bswap32(s[i]);  // sha2.h:735-736
    }
};

// ============================================================ SHA-384/512
// sha2.h:531-613; 64-bit words emulated on the 32-bit VALU (v_alignbit pairs,
// v_add_co/addc or v_lshl_add_u64).  Raw words: 32 LE u32 per 128-B block.

constexpr uint64_t kSha512Kc[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
    0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
    0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
    0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
    0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
    0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
    0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
    0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
    0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
    0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
    0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
    0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
    0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
    0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
    0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
    0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
    0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};

template <bool k384>
struct Sha512 {
    static constexpr int kBlock = 128, kDigest = k384 ? 48 : 64, kLenBytes = 16, kWords = 32, kOcc = 4;
    static constexpr bool kPairLoad = false;  // 128-B blocks already
    // Line stream off: 2.5-4 % slower (3 waves per SIMD at 139 VGPRs instead
    // of 4; profiles/r1_sha2_lds_ab.txt, profiles/r1_fixed_occ_ab.txt).
    static constexpr bool kLdsStream = false;
    static constexpr bool kScalarPad = true;
    static constexpr int kTileOcc = 0;   // VALU-bound: ragged batches take the per-lane kernel
    uint64_t s[8];
    __device__ __forceinline__ void init() {
        if (k384) {  // sha2.h:139-143
            s[0] = 0xcbbb9d5dc1059ed8ull; s[1] = 0x629a292a367cd507ull; s[2] = 0x9159015a3070dd17ull;
            s[3] = 0x152fecd8f70e5939ull; s[4] = 0x67332667ffc00b31ull; s[5] = 0x8eb44a8768581511ull;
            s[6] = 0xdb0c2e0d64f98fa7ull; s[7] = 0x47b5481dbefa4fa4ull;
        } else {     // sha2.h:144-148
            s[0] = 0x6a09e667f3bcc908ull; s[1] = 0xbb67ae8584caa73bull; s[2] = 0x3c6ef372fe94f82bull;
            s[3] = 0xa54ff53a5f1d36f1ull; s[4] = 0x510e527fade682d1ull; s[5] = 0x9b05688c2b3e6c1full;
            s[6] = 0x1f83d9abfb41bd6bull; s[7] = 0x5be0cd19137e2179ull;
        }
    }
    struct Vars {
        u64p w[16];
        u64p a, b, c, d, e, f, g, h;
    };
    // One round with a compile-time index (the 80 rounds are expanded by a
    // fold expression, so every w[] index is static and w stays in VGPRs).
    template <int i>
    __device__ __forceinline__ static void round(Vars& v) {
        u64p x;
        if constexpr (i < 16) {
            x = v.w[i];
        } else {
            const u64p w15 = v.w[(i - 15) & 15], w2 = v.w[(i - 2) & 15];
            const u64p s0 = xor3p(rotr64p<1>(w15), rotr64p<8>(w15), shr64p<7>(w15));
            const u64p s1 = xor3p(rotr64p<19>(w2), rotr64p<61>(w2), shr64p<6>(w2));
            x = mk64(add64(add64(v64(v.w[i & 15]), v64(s0)), add64(v64(v.w[(i - 7) & 15]), v64(s1))));
            v.w[i & 15] = x;
        }
        const u64p S1 = xor3p(rotr64p<14>(v.e), rotr64p<18>(v.e), rotr64p<41>(v.e));
        const u64p ch = u64p{ch3(v.e.lo, v.f.lo, v.g.lo), ch3(v.e.hi, v.f.hi, v.g.hi)};
        const uint64_t t1 = add64(add64(add64k(v64(v.h), kSha512Kc[i]), v64(x)), add64(v64(S1), v64(ch)));
        const u64p S0 = xor3p(rotr64p<28>(v.a), rotr64p<34>(v.a), rotr64p<39>(v.a));
        const u64p mj = u64p{maj3(v.a.lo, v.b.lo, v.c.lo), maj3(v.a.hi, v.b.hi, v.c.hi)};
        v.h = v.g; v.g = v.f; v.f = v.e; v.e = mk64(add64(v64(v.d), t1)); v.d = v.c; v.c = v.b; v.b = v.a;
        v.a = mk64(add64(t1, add64(v64(S0), v64(mj))));
    }
    template <int... I>
    __device__ __forceinline__ static void rounds(Vars& v, std::integer_sequence<int, I...>) {
        (round<I>(v), ...);
    }
    // Pad-only block from a wave-uniform length: the 80-word schedule is
    // computed in plain 64-bit C (scalar ALU) and K[i] + W[i] is folded into
    // one wave-uniform operand (md_pad_only).
    struct UVars {
        uint64_t w[16];
        u64p a, b, c, d, e, f, g, h;
    };
    template <int i>
    __device__ __forceinline__ static void uround(UVars& v) {
        uint64_t x;
        if constexpr (i < 16) {
            x = v.w[i];
        } else {
            const uint64_t w15 = v.w[(i - 15) & 15], w2 = v.w[(i - 2) & 15];
            const uint64_t s0 = srotr64(w15, 1) ^ srotr64(w15, 8) ^ (w15 >> 7);
            const uint64_t s1 = srotr64(w2, 19) ^ srotr64(w2, 61) ^ (w2 >> 6);
            x = v.w[i & 15] + s0 + v.w[(i - 7) & 15] + s1;
            v.w[i & 15] = x;
        }
        const u64p S1 = xor3p(rotr64p<14>(v.e), rotr64p<18>(v.e), rotr64p<41>(v.e));
        const u64p ch = u64p{ch3(v.e.lo, v.f.lo, v.g.lo), ch3(v.e.hi, v.f.hi, v.g.hi)};
        const uint64_t t1 = add64(add64k(v64(v.h), kSha512Kc[i] + x), add64(v64(S1), v64(ch)));
        const u64p S0 = xor3p(rotr64p<28>(v.a), rotr64p<34>(v.a), rotr64p<39>(v.a));
        const u64p mj = u64p{maj3(v.a.lo, v.b.lo, v.c.lo), maj3(v.a.hi, v.b.hi, v.c.hi)};
        v.h = v.g; v.g = v.f; v.f = v.e; v.e = mk64(add64(v64(v.d), t1)); v.d = v.c; v.c = v.b; v.b = v.a;
        v.a = mk64(add64(t1, add64(v64(S0), v64(mj))));
    }
    template <int... I>
    __device__ __forceinline__ static void urounds(UVars& v, std::integer_sequence<int, I...>) {
        (uround<I>(v), ...);
    }
    __device__ __forceinline__ void compress_pad(uint64_t bytes) {
        UVars v;
#pragma unroll
        for (int i = 0; i < 16; ++i) v.w[i] = 0;
        v.w[0] = 0x8000000000000000ull;
        v.w[14] = bytes >> 61; v.w[15] = bytes << 3;
        v.a = mk64(s[0]); v.b = mk64(s[1]); v.c = mk64(s[2]); v.d = mk64(s[3]);
        v.e = mk64(s[4]); v.f = mk64(s[5]); v.g = mk64(s[6]); v.h = mk64(s[7]);
        urounds(v, std::make_integer_sequence<int, 80>{});
        s[0] += v64(v.a); s[1] += v64(v.b); s[2] += v64(v.c); s[3] += v64(v.d);
        s[4] += v64(v.e); s[5] += v64(v.f); s[6] += v64(v.g); s[7] += v64(v.h);
    }
    __device__ __forceinline__ void compress(const uint32_t* raw) {
        Vars v;
#pragma unroll
        for (int i = 0; i < 16; ++i)  // BE u64 words (sha2.h:582)
            v.w[i] = u64p{bswap32(raw[2 * i + 1]), bswap32(raw[2 * i])};
        v.a = mk64(s[0]); v.b = mk64(s[1]); v.c = mk64(s[2]); v.d = mk64(s[3]);
        v.e = mk64(s[4]); v.f = mk64(s[5]); v.g = mk64(s[6]); v.h = mk64(s[7]);
        rounds(v, std::make_integer_sequence<int, 80>{});
        s[0] += v64(v.a); s[1] += v64(v.b); s[2] += v64(v.c); s[3] += v64(v.d);
        s[4] += v64(v.e); s[5] += v64(v.f); s[6] += v64(v.g); s[7] += v64(v.h);
    }
    // sha2.h:727-730: 128-bit BE bit length in bytes 112..127 (hi 64 bits =
    // bytes >> 61 for any length below 2^64 bytes).
    __device__ __forceinline__ static void put_length(uint32_t* w, uint64_t bytes) {
        const uint64_t lo = bytes << 3, hi = bytes >> 61;
        w[28] = bswap32((uint32_t)(hi >> 32)); w[29] = bswap32((uint32_t)hi);
        w[30] = bswap32((uint32_t)(lo >> 32)); w[31] = bswap32((uint32_t)lo);
    }
    __device__ __forceinline__ void digest_words(uint32_t* out) const {  // sha2.h:738
#pragma unroll
        for (int i = 0; i < kDigest / 8; ++i) {
            out[2 * i] = bswap32((uint32_t)(s[i] >> 32));
            out[2 * i + 1] = bswap32((uint32_t)s[i]);
        }
    }
};

// HMAC mid-state save/load (state words only; the prefix length is implied).
template <int N>
__device__ __forceinline__ void save_words(const uint32_t (&s)[N], uint32_t* p) {
#pragma unroll
    for (int i = 0; i < N; ++i) p[i] = s[i];
}
template <int N>
__device__ __forceinline__ void save_words(const uint64_t (&s)[N], uint32_t* p) {
#pragma unroll
    for (int i = 0; i < N; ++i) { p[2 * i] = (uint32_t)s[i]; p[2 * i + 1] = (uint32_t)(s[i] >> 32); }
}
template <int N>
__device__ __forceinline__ void load_words(uint32_t (&s)[N], const uint32_t* p) {
#pragma unroll
    for (int i = 0; i < N; ++i) s[i] = p[i];
}
template <int N>
__device__ __forceinline__ void load_words(uint64_t (&s)[N], const uint32_t* p) {
#pragma unroll
    for (int i = 0; i < N; ++i) s[i] = (uint64_t)p[2 * i] | ((uint64_t)p[2 * i + 1] << 32);
}

// ------------------------------------------------- MD-family message driver
// Loads block `blk` (kBlock bytes) of a message with `avail` >= kBlock bytes.
template <class H>
__device__ __forceinline__ void load_block_full(const uint8_t* p, uint32_t* w) {
#pragma unroll
    for (int h = 0; h < H::kBlock / 64; ++h) load_full64(p + 64 * h, w + 16 * h);
}
// Tail block: rem (< kBlock) message bytes, zero fill.
template <class H>
__device__ __forceinline__ void load_block_tail(const uint8_t* p, uint32_t rem, uint32_t* w) {
#pragma unroll
    for (int h = 0; h < H::kBlock / 64; ++h) {
        const int r = (int)rem - 64 * h;
        if (r >= 64) {
            load_full64(p + 64 * h, w + 16 * h);
        } else if (r > 0) {
            load_tail64(p + 64 * h, (uint32_t)r, w + 16 * h);
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) w[16 * h + k] = 0u;
        }
    }
}

// Processes a whole message of `len` bytes starting from state `st`, whose
// compressed prefix is `prefix` bytes long (0, or the block for HMAC inner),
// then pads (md5.h:266-288 / sha1.h:816-840 / sha2.h:706-742).
// Per-wave LDS-DMA line stream over 64 fixed-stride records (the fixed-stride
// fast paths of lcb_kernels.hip and crc_kernels.hip).  The per-lane loads of
// the generic kernels touch 64 different 128-B lines per wave-instruction;
// here line L of the wave's 64 records moves into a slab of LDS with 8
// coalesced LDS-DMA instructions (global_load_lds_dwordx4: one instruction =
// 8 records x one whole 128-B line), every lane copies its own 128 B into
// VGPRs (take), and the caller issues line L+1 before computing line L.
// Instruction g carries records j with j & 7 == g (lane group q = j >> 3,
// chunk c = lane & 7) and lands at slab + g * kSlabRow, kSlabRow = 1,040:
// record j's row starts at (j & 7) * 1040 + (j >> 3) * 128, in bank group
// ((j & 7) + 8 (j >> 3)) mod 16, so the 16 lanes of every ds_read_b128 group
// start in 16 different bank groups and take() reads chunk k at row + 16 k,
// one base and immediate offsets (round 4's 8 KiB slabs XOR-swizzled the
// chunks: one v_xor per chunk, 8 VALU per line).
// The fixed-stride stream (LdsStridedStream) always covers 64 whole records;
// the ragged one (GatherLineStream) repeats a record's last line once it has
// run out.  The fixed-stride DMA carries the nt cache policy (every byte is
// read once; kLdsAux).
constexpr uint32_t kSlabRow = 1040;                     // LDS bytes per DMA instruction (padded)
constexpr uint32_t kSlabBytes = 7 * kSlabRow + 1024;     // one wave's slab (8,304 B)
// Default cache policy of the ragged (gather) line stream: a record of a
// packed ragged batch need not start on a 128-B line, so one streamed "line"
// can span two cache lines; with nt the second is gone before the record's
// next line asks for it (64 KiB records at a 64-B phase: 5.95 ms with nt,
// 4.70 default; profiles/r2_c4_tiles_ab.txt).  Tiles whose records share
// a 0 or 64-B phase stream whole cache lines with nt instead (md_tile_stream).
constexpr int kGatherAux = 0;
#ifndef LCB_LDS_AUX
#define LCB_LDS_AUX 2
#endif
constexpr int kLdsAux = LCB_LDS_AUX;  // cache policy of the LDS-DMA stream: nt (every byte is read once)
// The slab side shared by the line streams: take() copies this lane's 128 B
// of the landed line into VGPRs.
struct LdsLineSlab {
    uint8_t* slab;
    uint32_t lane;
    // Waits for the issued line, copies this lane's 128 B (raw LE words);
    // the slab is free again on return.
    __device__ __forceinline__ void take(uint32_t w0[16], uint32_t w1[16]) const {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        using lds_cu4 = __attribute__((address_space(3))) const v4u;
        // The row base (one VGPR); the 8 chunks at immediate offsets.
        const uint32_t b = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t*)slab) +
                           (lane & 7u) * kSlabRow + (lane >> 3) * 128u;
        lds_cu4* row = (lds_cu4*)(uintptr_t)b;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const v4u v = row[k];
            uint32_t* d = (k < 4) ? (w0 + 4 * k) : (w1 + 4 * (k - 4));
            d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slab free again
    }
};

// Fixed-stride stream with a wave-uniform base: instruction g of line L reads
// from (wave base + g stride + 128 L) — a scalar address — plus one per-lane
// 32-bit offset (record 8 (lane >> 3) of the 8 the instruction carries, and
// the chunk lane & 7), i.e. the saddr form of global_load_lds with 1 VGPR of
// addressing instead of 8 64-bit pointers.  The wave covers 64 whole records
// (the caller shifts a partial last wave back over its predecessor's
// records), so there is no per-lane clamp.  Needs 56 * stride + 128 < 2^32
// (fixed_stride_lines: stride < 2^26).
struct LdsStridedStream : LdsLineSlab {
    const uint8_t* wbase;   // wave-uniform
    uint64_t stride1;       // wave-uniform: one record
    uint32_t voff;
    __device__ __forceinline__ void init(const uint8_t* data, uint64_t stride, uint64_t wave_first, uint32_t ln,
                                         uint8_t* my_slab) {
        lane = ln;
        slab = my_slab;
        wbase = data + wave_first * stride;
        stride1 = stride;
        voff = (ln >> 3) * 8u * (uint32_t)stride + (ln & 7) * 16;
    }
    template <int kAux = kLdsAux>
    __device__ __forceinline__ void issue(uint64_t L) {
        // Offset re-defined in place (no copy): zero-extended at each use, so
        // every DMA takes the saddr + 32-bit vaddr form.
        asm volatile("" : "+v"(voff));
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            // Opaque scalar: keeps the loop optimiser from turning the
            // address into a per-lane 64-bit induction variable.
            uint64_t so = (uint64_t)g * stride1 + L * 128;
            asm volatile("" : "+s"(so));
            const uint8_t* sb = wbase + so;
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(sb + voff),
                                             (__attribute__((address_space(3))) void*)(slab + g * kSlabRow), 16, 0,
                                             kAux);
        }
    }
};

// Ragged variant: record j of the wave streams from its own base pointer
// (any 16-B aligned start), re-reading its last whole line once it runs out
// (the data is discarded; every DMA stays inside the record).  Bases and
// limits are exchanged across lanes once, at init.
struct GatherLineStream : LdsLineSlab {
    const uint8_t* src[8];  // instruction g: this lane's chunk of local record g + 8 (lane >> 3)
    uint32_t rem[8];   // advances left: lines of the record after the current one
    __device__ __forceinline__ void init_gather(const uint8_t* base, uint32_t last_line, uint32_t ln,
                                                uint8_t* my_slab) {
        lane = ln;
        slab = my_slab;
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            const int j = g + 8 * (int)(ln >> 3);
            const uint64_t b = __shfl((unsigned long long)reinterpret_cast<uintptr_t>(base), j, 64);
            rem[g] = (uint32_t)__shfl((int)last_line, j, 64);
            src[g] = reinterpret_cast<const uint8_t*>(b) + (ln & 7) * 16;
        }
    }
    // Issues the next line of every record, then steps each record's pointer
    // to its following line while it has one (a record that has run out
    // re-reads its last line; the data is discarded).  Pointers advance in
    // place: no per-issue address temporaries next to the line in VGPRs.
    // All records have the same number of lines: no clamping, no rem[].
    // kAux: cache policy (kGatherAux, or kLdsAux when every streamed line is a
    // whole 128-B cache line read once).
    template <int kAux = kGatherAux>
    __device__ __forceinline__ void issue_next_uniform() {
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src[g],
                                             (__attribute__((address_space(3))) void*)(slab + g * kSlabRow), 16, 0,
                                             kAux);
            src[g] += 128;
        }
    }
    __device__ __forceinline__ void issue_next() {
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src[g],
                                             (__attribute__((address_space(3))) void*)(slab + g * kSlabRow), 16, 0,
                                             kGatherAux);
            const bool more = rem[g] != 0;
            src[g] += more ? 128 : 0;
            rem[g] -= more ? 1u : 0u;
        }
    }
};

// 128 message bytes as raw LE words (a0 = bytes 0..63, a1 = 64..127):
// two 64-B blocks, or one 128-B block.
template <class H>
__device__ __forceinline__ void md_compress128(H& st, const uint32_t* a0, const uint32_t* a1) {
    if constexpr (H::kBlock == 128) {
        uint32_t w[32];
#pragma unroll
        for (int k = 0; k < 16; ++k) { w[k] = a0[k]; w[16 + k] = a1[k]; }
        st.compress(w);
    } else {
        st.compress(a0);
        st.compress(a1);
    }
}

// Compresses `nfull` whole blocks starting at p; returns the pointer after them.
// kPf: latency form for batches too small to fill the chip -- the loads of
// the next 128 B are in flight while the current 128 B are compressed (two
// register sets, fewer waves per SIMD); otherwise occupancy hides the load
// latency and one set is kept.
// Workgroup blockIdx.x of a fixed-stride grid -> the record group it hashes:
// workgroups are dealt to the 8 XCDs round robin (b % 8), so XCD x gets the
// contiguous x-th eighth of the records (one stream per XCD's L2 and TLB)
// instead of every eighth group.  Identity when the grid is not a multiple
// of 8.  MD5 fixed stride -1.6 %, SHA-1 -0.8 % (profiles/r4_fixed_waves_ab.txt).
__device__ __forceinline__ uint32_t xcd_block() {
    uint32_t b = blockIdx.x;
    if ((gridDim.x & 7u) == 0) b = (b & 7u) * (gridDim.x >> 3) + (b >> 3);
    return b;
}

#ifndef LCB_LANE_PRIO
#define LCB_LANE_PRIO 1
#endif
// Wave priority by the bytes its (first active) lane has left, longest
// remaining first: s_setprio 3 / 2 / 1 / 0 at >= 48 / 32 / 16 KiB / less.
// Among a SIMD's waves the arbiter otherwise favours the oldest, so in a
// bucketed ragged batch (C4: 1/3 of the messages 64 KiB) the youngest long
// waves end last and run alone at the end (md_tiles.hpp tile_prio: the
// same rule in 128-B lines).
__device__ __forceinline__ void wave_prio_left(uint64_t left) {
    const uint32_t k = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(left >> 14 < 3 ? left >> 14 : 3));
    if (k >= 3) __builtin_amdgcn_s_setprio(3);
    else if (k == 2) __builtin_amdgcn_s_setprio(2);
    else if (k == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

// kPrio: the per-lane loop sets the wave priority by the bytes left
// (LCB_LANE_PRIO); off where the caller keeps its own priority (the resident
// grid's chunks-left priority in md_fixed_finish).
template <class H, bool kPf = false, bool kPrio = true>
__device__ __forceinline__ const uint8_t* md_full_blocks(H& st, const uint8_t* p, uint64_t nfull) {
    uint32_t w[H::kWords];
    uint64_t b = 0;
    if constexpr (kPf) {  // 128 B per stage: two 64-B blocks or one 128-B block
        constexpr int kPer = 128 / H::kBlock;
        const uint64_t nl = nfull / kPer;
        uint32_t a0[16], a1[16], b0[16], b1[16];
        if (nl) load_full128(p, a0, a1);
        uint64_t L = 0;
        for (; L + 2 <= nl; L += 2) {
            load_full128(p + 128 * (L + 1), b0, b1);
            md_compress128(st, a0, a1);
            if (L + 2 < nl) load_full128(p + 128 * (L + 2), a0, a1);
            md_compress128(st, b0, b1);
        }
        if (L < nl) md_compress128(st, a0, a1);
        b = nl * kPer;
        p += 128 * nl;
    }
    if (H::kPairLoad && !kPf) {  // two blocks = one 128-B line per iteration
        uint32_t w1[16];
        for (; b + 2 <= nfull; b += 2, p += 128) {
            load_full128(p, w, w1);
            st.compress(w);
            st.compress(w1);
        }
    }
    for (; b < nfull; ++b, p += H::kBlock) {
#if LCB_LANE_PRIO
        if (kPrio && (b & 15) == 0) wave_prio_left((nfull - b) * (uint64_t)H::kBlock);
#endif
        load_block_full<H>(p, w);
        st.compress(w);
    }
    return p;
}

// Last block: w holds the final rem (< kBlock) message bytes, zero filled;
// appends 0x80, zeros and the length of all `total` bytes (md5.h:266-288 /
// sha1.h:816-840 / sha2.h:706-742).
template <class H>
__device__ __forceinline__ void md_pad_tail(H& st, uint32_t* w, uint32_t rem, uint64_t total) {
    // 0x80 terminator at byte `rem` (of a 64- or 128-byte block).
#pragma unroll
    for (int h = 0; h < H::kBlock / 64; ++h)
        if ((rem >> 6) == (uint32_t)h) put_byte(w + 16 * h, rem & 63u, 0x80u);
    if (rem + 1 + H::kLenBytes > (uint32_t)H::kBlock) {  // no room for the length
        st.compress(w);
#pragma unroll
        for (int k = 0; k < H::kWords; ++k) w[k] = 0u;
    }
    H::put_length(w, total);
    st.compress(w);
}

template <class H, bool kPf = false, bool kPrio = true>
__device__ __forceinline__ void md_message(H& st, const uint8_t* msg, uint64_t len, uint64_t prefix) {
    uint32_t w[H::kWords];
    const uint64_t nfull = len / H::kBlock;
    const uint8_t* p = md_full_blocks<H, kPf, kPrio>(st, msg, nfull);
    const uint32_t rem = (uint32_t)(len - nfull * H::kBlock);
    load_block_tail<H>(p, rem, w);
    md_pad_tail(st, w, rem, len + prefix);
}

// Whole virtual message A[0, la) || B[0, lb) from state `st` after `prefix`
// bytes: A's whole blocks straight from A, the block(s) holding the seam
// assembled word by word, then the rest straight from B (any alignment).
template <class H>
__device__ __forceinline__ void md_message2(H& st, const uint8_t* A, uint64_t la, const uint8_t* B, uint64_t lb,
                                            uint64_t prefix) {
    const uint64_t nA = la / H::kBlock;
    md_full_blocks(st, A, nA);
    uint64_t done = nA * H::kBlock;
    const uint64_t total = la + lb;
    uint32_t w[H::kWords];
    while (done < la && done + H::kBlock <= total) {   // a whole block across the seam
#pragma unroll
        for (int h = 0; h < H::kBlock / 64; ++h) load_vblock64(A, la, B, lb, done + 64 * h, w + 16 * h);
        st.compress(w);
        done += H::kBlock;
    }
    if (done >= la) {                                  // the rest lies in B
        md_message(st, B + (done - la), total - done, prefix + done);
        return;
    }
    // the final, partial block still holds bytes of A
#pragma unroll
    for (int h = 0; h < H::kBlock / 64; ++h) load_vblock64(A, la, B, lb, done + 64 * h, w + 16 * h);
    md_pad_tail(st, w, (uint32_t)(total - done), total + prefix);
}

// Final block of a message whose length is a whole number of blocks: 0x80,
// zeros, length (md5.h:271-283, sha1.h:816-834, sha2.h:714-733).  Equal to
// md_message(st, p, 0, total) but built from `total` alone, so when `total`
// is wave-uniform (fixed-length batches) the block and the SHA message
// schedule derived from it live in SGPRs and run on the scalar ALU, leaving
// the VALU only the rounds.
template <class H>
__device__ __forceinline__ void md_pad_only(H& st, uint64_t total) {
    if constexpr (H::kScalarPad) {
        st.compress_pad(total);
    } else {
        uint32_t w[H::kWords];
#pragma unroll
        for (int k = 0; k < H::kWords; ++k) w[k] = 0u;
        w[0] = 0x80u;
        H::put_length(w, total);
        st.compress(w);
    }
}

// Outer HMAC pass over an inner digest held in registers (digest words are
// raw LE byte order): one block = digest || 0x80 || zeros || length(B + D).
template <class H>
__device__ __forceinline__ void md_outer(H& st, const uint32_t* dig) {
    uint32_t w[H::kWords];
#pragma unroll
    for (int k = 0; k < H::kWords; ++k) w[k] = (k < H::kDigest / 4) ? dig[k] : 0u;
    w[H::kDigest / 4] = 0x80u;  // D is a multiple of 4: terminator starts a fresh word
    H::put_length(w, (uint64_t)H::kBlock + H::kDigest);
    st.compress(w);
}

// Stores D digest bytes (raw LE word order) at out (any alignment).
template <int D>
__device__ __forceinline__ void store_digest(uint8_t* out, const uint32_t* dw) {
    if ((reinterpret_cast<uintptr_t>(out) & 3u) == 0) {
        uint32_t* o = reinterpret_cast<uint32_t*>(out);
        if ((D % 16) == 0 && (reinterpret_cast<uintptr_t>(out) & 15u) == 0) {
#pragma unroll
            for (int i = 0; i < D / 16; ++i)
                reinterpret_cast<uint4*>(out)[i] = make_uint4(dw[4 * i], dw[4 * i + 1], dw[4 * i + 2], dw[4 * i + 3]);
        } else {
#pragma unroll
            for (int i = 0; i < D / 4; ++i) o[i] = dw[i];
        }
    } else {
#pragma unroll
        for (int i = 0; i < D; ++i) out[i] = (uint8_t)(dw[i >> 2] >> (8 * (i & 3)));
    }
}

}  // namespace lcbgpu
