// gost_device.hpp — GOST R 34.11-2012 (Streebog, RFC 6986) per-lane device
// code for the MI355X batch kernels.
//
// One lane per message (as the MD family).  The LPS transform uses the
// big-table form of the reference (gost3411-2012.h:1071-1099):
//     dst[i] = XOR_{j=0..7} Ax[j][ byte i of src[j] ]
// with the 8 x 256 x u64 = 16 KiB table held in LDS — in the batch kernels
// as a 64 KiB lane-rotated, bank-sliced image (GostRot below) whose gathers
// are bank-conflict-free — so LPS is 64 ds_read_b64 + XORs per 512-bit
// transform and a 64-byte block costs 25 LPS (gost3411-2012.h:1129-1142).  The table is generated at
// COMPILE TIME from the RFC 6986 S-box pi and the 64 rows of the linear map A,
// following the reference's small-table definition (gost3411-2012.h:1032-1067),
// and pinned against the reference's gost3411_2012_Ax by a test.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "hash_device.hpp"

namespace lcbgpu {

struct GostConsts {
    uint8_t pi[256];
    uint64_t A[64];
    uint64_t C[12][8];
};

// RFC 6986 section 6: pi, A, C.
constexpr GostConsts kGostConsts = {
    {0xfc, 0xee, 0xdd, 0x11, 0xcf, 0x6e, 0x31, 0x16, 0xfb, 0xc4, 0xfa, 0xda, 0x23, 0xc5, 0x04, 0x4d,
     0xe9, 0x77, 0xf0, 0xdb, 0x93, 0x2e, 0x99, 0xba, 0x17, 0x36, 0xf1, 0xbb, 0x14, 0xcd, 0x5f, 0xc1,
     0xf9, 0x18, 0x65, 0x5a, 0xe2, 0x5c, 0xef, 0x21, 0x81, 0x1c, 0x3c, 0x42, 0x8b, 0x01, 0x8e, 0x4f,
     0x05, 0x84, 0x02, 0xae, 0xe3, 0x6a, 0x8f, 0xa0, 0x06, 0x0b, 0xed, 0x98, 0x7f, 0xd4, 0xd3, 0x1f,
     0xeb, 0x34, 0x2c, 0x51, 0xea, 0xc8, 0x48, 0xab, 0xf2, 0x2a, 0x68, 0xa2, 0xfd, 0x3a, 0xce, 0xcc,
     0xb5, 0x70, 0x0e, 0x56, 0x08, 0x0c, 0x76, 0x12, 0xbf, 0x72, 0x13, 0x47, 0x9c, 0xb7, 0x5d, 0x87,
     0x15, 0xa1, 0x96, 0x29, 0x10, 0x7b, 0x9a, 0xc7, 0xf3, 0x91, 0x78, 0x6f, 0x9d, 0x9e, 0xb2, 0xb1,
     0x32, 0x75, 0x19, 0x3d, 0xff, 0x35, 0x8a, 0x7e, 0x6d, 0x54, 0xc6, 0x80, 0xc3, 0xbd, 0x0d, 0x57,
     0xdf, 0xf5, 0x24, 0xa9, 0x3e, 0xa8, 0x43, 0xc9, 0xd7, 0x79, 0xd6, 0xf6, 0x7c, 0x22, 0xb9, 0x03,
     0xe0, 0x0f, 0xec, 0xde, 0x7a, 0x94, 0xb0, 0xbc, 0xdc, 0xe8, 0x28, 0x50, 0x4e, 0x33, 0x0a, 0x4a,
     0xa7, 0x97, 0x60, 0x73, 0x1e, 0x00, 0x62, 0x44, 0x1a, 0xb8, 0x38, 0x82, 0x64, 0x9f, 0x26, 0x41,
     0xad, 0x45, 0x46, 0x92, 0x27, 0x5e, 0x55, 0x2f, 0x8c, 0xa3, 0xa5, 0x7d, 0x69, 0xd5, 0x95, 0x3b,
     0x07, 0x58, 0xb3, 0x40, 0x86, 0xac, 0x1d, 0xf7, 0x30, 0x37, 0x6b, 0xe4, 0x88, 0xd9, 0xe7, 0x89,
     0xe1, 0x1b, 0x83, 0x49, 0x4c, 0x3f, 0xf8, 0xfe, 0x8d, 0x53, 0xaa, 0x90, 0xca, 0xd8, 0x85, 0x61,
     0x20, 0x71, 0x67, 0xa4, 0x2d, 0x2b, 0x09, 0x5b, 0xcb, 0x9b, 0x25, 0xd0, 0xbe, 0xe5, 0x6c, 0x52,
     0x59, 0xa6, 0x74, 0xd2, 0xe6, 0xf4, 0xb4, 0xc0, 0xd1, 0x66, 0xaf, 0xc2, 0x39, 0x4b, 0x63, 0xb6},
    {0x8e20faa72ba0b470ull, 0x47107ddd9b505a38ull, 0xad08b0e0c3282d1cull, 0xd8045870ef14980eull,
     0x6c022c38f90a4c07ull, 0x3601161cf205268dull, 0x1b8e0b0e798c13c8ull, 0x83478b07b2468764ull,
     0xa011d380818e8f40ull, 0x5086e740ce47c920ull, 0x2843fd2067adea10ull, 0x14aff010bdd87508ull,
     0x0ad97808d06cb404ull, 0x05e23c0468365a02ull, 0x8c711e02341b2d01ull, 0x46b60f011a83988eull,
     0x90dab52a387ae76full, 0x486dd4151c3dfdb9ull, 0x24b86a840e90f0d2ull, 0x125c354207487869ull,
     0x092e94218d243cbaull, 0x8a174a9ec8121e5dull, 0x4585254f64090fa0ull, 0xaccc9ca9328a8950ull,
     0x9d4df05d5f661451ull, 0xc0a878a0a1330aa6ull, 0x60543c50de970553ull, 0x302a1e286fc58ca7ull,
     0x18150f14b9ec46ddull, 0x0c84890ad27623e0ull, 0x0642ca05693b9f70ull, 0x0321658cba93c138ull,
     0x86275df09ce8aaa8ull, 0x439da0784e745554ull, 0xafc0503c273aa42aull, 0xd960281e9d1d5215ull,
     0xe230140fc0802984ull, 0x71180a8960409a42ull, 0xb60c05ca30204d21ull, 0x5b068c651810a89eull,
     0x456c34887a3805b9ull, 0xac361a443d1c8cd2ull, 0x561b0d22900e4669ull, 0x2b838811480723baull,
     0x9bcf4486248d9f5dull, 0xc3e9224312c8c1a0ull, 0xeffa11af0964ee50ull, 0xf97d86d98a327728ull,
     0xe4fa2054a80b329cull, 0x727d102a548b194eull, 0x39b008152acb8227ull, 0x9258048415eb419dull,
     0x492c024284fbaec0ull, 0xaa16012142f35760ull, 0x550b8e9e21f7a530ull, 0xa48b474f9ef5dc18ull,
     0x70a6a56e2440598eull, 0x3853dc371220a247ull, 0x1ca76e95091051adull, 0x0edd37c48a08a6d8ull,
     0x07e095624504536cull, 0x8d70c431ac02a736ull, 0xc83862965601dd1bull, 0x641c314b2b8ee083ull},
    {{0xdd806559f2a64507ull, 0x05767436cc744d23ull, 0xa2422a08a460d315ull, 0x4b7ce09192676901ull,
      0x714eb88d7585c4fcull, 0x2f6a76432e45d016ull, 0xebcb2f81c0657c1full, 0xb1085bda1ecadae9ull},
     {0xe679047021b19bb7ull, 0x55dda21bd7cbcd56ull, 0x5cb561c2db0aa7caull, 0x9ab5176b12d69958ull,
      0x61d55e0f16b50131ull, 0xf3feea720a232b98ull, 0x4fe39d460f70b5d7ull, 0x6fa3b58aa99d2f1aull},
     {0x991e96f50aba0ab2ull, 0xc2b6f443867adb31ull, 0xc1c93a376062db09ull, 0xd3e20fe490359eb1ull,
      0xf2ea7514b1297b7bull, 0x06f15e5f529c1f8bull, 0x0a39fc286a3d8435ull, 0xf574dcac2bce2fc7ull},
     {0x220cbebc84e3d12eull, 0x3453eaa193e837f1ull, 0xd8b71333935203beull, 0xa9d72c82ed03d675ull,
      0x9d721cad685e353full, 0x488e857e335c3c7dull, 0xf948e1a05d71e4ddull, 0xef1fdfb3e81566d2ull},
     {0x601758fd7c6cfe57ull, 0x7a56a27ea9ea63f5ull, 0xdfff00b723271a16ull, 0xbfcd1747253af5a3ull,
      0x359e35d7800fffbdull, 0x7f151c1f1686104aull, 0x9a3f410c6ca92363ull, 0x4bea6bacad474799ull},
     {0xfa68407a46647d6eull, 0xbf71c57236904f35ull, 0x0af21f66c2bec6b6ull, 0xcffaa6b71c9ab7b4ull,
      0x187f9ab49af08ec6ull, 0x2d66c4f95142a46cull, 0x6fa4c33b7a3039c0ull, 0xae4faeae1d3ad3d9ull},
     {0x8886564d3a14d493ull, 0x3517454ca23c4af3ull, 0x06476983284a0504ull, 0x0992abc52d822c37ull,
      0xd3473e33197a93c9ull, 0x399ec6c7e6bf87c9ull, 0x51ac86febf240954ull, 0xf4c70e16eeaac5ecull},
     {0xa47f0dd4bf02e71eull, 0x36acc2355951a8d9ull, 0x69d18d2bd1a5c42full, 0xf4892bcb929b0690ull,
      0x89b4443b4ddbc49aull, 0x4eb7f8719c36de1eull, 0x03e7aa020c6e4141ull, 0x9b1f5b424d93c9a7ull},
     {0x7261445183235adbull, 0x0e38dc92cb1f2a60ull, 0x7b2b8a9aa6079c54ull, 0x800a440bdbb2ceb1ull,
      0x3cd955b7e00d0984ull, 0x3a7d3a1b25894224ull, 0x944c9ad8ec165fdeull, 0x378f5a541631229bull},
     {0x74b4c7fb98459cedull, 0x3698fad1153bb6c3ull, 0x7a1e6c303b7652f4ull, 0x9fe76702af69334bull,
      0x1fffe18a1b336103ull, 0x8941e71cff8a78dbull, 0x382ae548b2e4f3f3ull, 0xabbedea680056f52ull},
     {0x6bcaa4cd81f32d1bull, 0xdea2594ac06fd85dull, 0xefbacd1d7d476e98ull, 0x8a1d71efea48b9caull,
      0x2001802114846679ull, 0xd8fa6bbbebab0761ull, 0x3002c6cd635afe94ull, 0x7bcd9ed0efc889fbull},
     {0x48bc924af11bd720ull, 0xfaf417d5d9b21b99ull, 0xe71da4aa88e12852ull, 0x5d80ef9d1891cc86ull,
      0xf82012d430219f9bull, 0xcda43c32bcdf1d77ull, 0xd21380b00449b17aull, 0x378ee767f11631baull}}};

struct GostAx {
    uint64_t t[8][256];
};

// Ax[j][b] = L(pi[b] placed in byte j): bit s of byte j is bit 8j+s of the
// 64-bit row, which selects A[63 - 8j - s] (MSB-first, gost3411-2012.h:1056-1064).
constexpr GostAx make_gost_ax() {
    GostAx r{};
    for (int j = 0; j < 8; ++j)
        for (int b = 0; b < 256; ++b) {
            uint64_t c = 0;
            const unsigned v = kGostConsts.pi[b];
            for (int s = 0; s < 8; ++s)
                if ((v >> s) & 1u) c ^= kGostConsts.A[63 - 8 * j - s];
            r.t[j][b] = c;
        }
    return r;
}

constexpr GostAx kGostAxHost = make_gost_ax();
__device__ const GostAx kGostAxDev = make_gost_ax();
__constant__ const uint64_t kGostC[12][8] = {
#define LCB_C(i) {kGostConsts.C[i][0], kGostConsts.C[i][1], kGostConsts.C[i][2], kGostConsts.C[i][3], \
                  kGostConsts.C[i][4], kGostConsts.C[i][5], kGostConsts.C[i][6], kGostConsts.C[i][7]}
    LCB_C(0), LCB_C(1), LCB_C(2), LCB_C(3), LCB_C(4), LCB_C(5),
    LCB_C(6), LCB_C(7), LCB_C(8), LCB_C(9), LCB_C(10), LCB_C(11)
#undef LCB_C
};

// Cooperative copy of the 16 KiB table into LDS (call by every thread, then barrier).
__device__ __forceinline__ void gost_stage_table(uint64_t* lds) {
    const uint4* src = reinterpret_cast<const uint4*>(&kGostAxDev.t[0][0]);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

// LPS(x) (gost3411-2012.h:1071-1090).
__device__ __forceinline__ void gost_lps(uint64_t o[8], const uint64_t x[8], const uint64_t* __restrict__ T) {
    uint32_t lo[8], hi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { lo[j] = (uint32_t)x[j]; hi[j] = (uint32_t)(x[j] >> 32); }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint64_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t src = (i < 4) ? lo[j] : hi[j];
            const uint32_t b = __builtin_amdgcn_ubfe(src, 8u * (i & 3), 8u);
            v[j] = T[j * 256 + b];
        }
        // 8-way XOR as bitop3 xor3 on each half: 4 ops per half instead of 7.
        uint32_t l = xor3(xor3((uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2]),
                          xor3((uint32_t)v[3], (uint32_t)v[4], (uint32_t)v[5]),
                          (uint32_t)v[6] ^ (uint32_t)v[7]);
        uint32_t h = xor3(xor3((uint32_t)(v[0] >> 32), (uint32_t)(v[1] >> 32), (uint32_t)(v[2] >> 32)),
                          xor3((uint32_t)(v[3] >> 32), (uint32_t)(v[4] >> 32), (uint32_t)(v[5] >> 32)),
                          (uint32_t)(v[6] >> 32) ^ (uint32_t)(v[7] >> 32));
        o[i] = ((uint64_t)h << 32) | l;
    }
}

// The flat table (one 16 KiB copy, entry (j, b) at T[j * 256 + b]): the
// one-lane HMAC key-schedule prep kernel.
// gost_g's hooks for tables whose LPS works on words in natural order: the
// round constants are wave-uniform (scalar loads), N is added to word 0.
struct GostNaturalOrder {
    __device__ __forceinline__ static void to_lane(uint64_t o[8], const uint64_t v[8]) {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = v[i];
    }
    __device__ __forceinline__ static void from_lane(uint64_t o[8], const uint64_t v[8]) { to_lane(o, v); }
    __device__ __forceinline__ static void xor_n(uint64_t x[8], uint64_t n0) { x[0] ^= n0; }
    __device__ __forceinline__ static void xor_c(uint64_t x[8], const uint64_t k[8], int r) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = k[i] ^ kGostC[r][i];
    }
};

struct GostFlat : GostNaturalOrder {
    const uint64_t* T;
    __device__ __forceinline__ void lps(uint64_t o[8], const uint64_t x[8]) const { gost_lps(o, x, T); }
};

// Lane-rotated, bank-sliced LPS table (the batch kernels).
//
// With the flat table the 64 data-dependent ds_read_b64 of an LPS land on
// random bank pairs: a 32-lane group meets ~3.4 distinct entries on its
// busiest bank pair, ~6.5 LDS cycles per wave-instruction instead of 2
// (DESIGN.md 5).  Here the LDS holds 4 replicas of the 8 tables, table j of
// replica c alone in bank pair 8c + j (entry b at byte b * 256 + (8c + j) * 8,
// 64 KiB), and lane l (c = (l & 31) >> 3, r = l & 7) takes the 8 input words
// of an LPS in the rotated order j = (j' + r) & 7 at static step j'.  At every
// step the 32 lanes of a ds_read_b64 group then read 32 different bank
// pairs: conflict-free whatever the data.  The rotation is a 3-stage barrel
// over the lane's 8 input words (bit-selects); a lookup address is ONE
// v_perm_b32 (table byte -> address bits 8-15, the lane's bank-pair offset
// -> bits 0-7), one instruction fewer than the flat form's extract + shift.
using lds_u8 = __attribute__((address_space(3))) const uint8_t;
#ifndef LCB_GOST_FENCE
#define LCB_GOST_FENCE 4
#endif
constexpr int kGostLpsFence = LCB_GOST_FENCE;
using lds_u64 = __attribute__((address_space(3))) const uint64_t;

template <int kFence>
struct GostRotF : GostNaturalOrder {
    lds_u8* L;
    // Byte j & 3 of offp[j >> 2] = (8c + ((j' + r) & 7)) * 8 (< 256): the lane's
    // bank-pair offsets for the 8 steps, packed 4 to a VGPR (v_perm picks the
    // byte), 6 VGPRs fewer than one per step.
    uint32_t offp[2];
    // Bits 0 / 1 / 2 of r as all-ones word masks (the barrel's bit-selects are
    // v_bitop3; as SGPR lane masks feeding v_cndmask the kernel measured ~5 %
    // slower, tools/ab_gost3.sh).
    uint32_t m1, m2, m4;
    __device__ __forceinline__ void init(lds_u8* lds) {
        L = lds;
        const uint32_t l = threadIdx.x & 31u, c = l >> 3, r = l & 7u;
        offp[0] = offp[1] = 0u;
#pragma unroll
        for (int j = 0; j < 8; ++j) offp[j >> 2] |= ((8u * c + (((uint32_t)j + r) & 7u)) * 8u) << (8 * (j & 3));
        m1 = (r & 1u) ? 0xffffffffu : 0u;
        m2 = (r & 2u) ? 0xffffffffu : 0u;
        m4 = (r & 4u) ? 0xffffffffu : 0u;
    }
    template <int S>
    __device__ __forceinline__ static void rot(uint32_t (&v)[8], uint32_t m) {  // v[j] <- v[(j + S) & 7] where m
        uint32_t t[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) t[j] = ch3(m, v[(j + S) & 7], v[j]);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = t[j];
    }
    // LPS(x) (gost3411-2012.h:1071-1090): o[i] = XOR_j Ax[j][byte i of x[j]].
    __device__ __forceinline__ void lps(uint64_t o[8], const uint64_t x[8]) const {
        uint32_t lo[8], hi[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { lo[j] = (uint32_t)x[j]; hi[j] = (uint32_t)(x[j] >> 32); }
        rot<1>(lo, m1); rot<1>(hi, m1);
        rot<2>(lo, m2); rot<2>(hi, m2);
        rot<4>(lo, m4); rot<4>(hi, m4);   // lo/hi[j'] = word (j' + r) & 7
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            uint64_t v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                // address bytes: [0] = step j's offset (S1 byte j & 3), [1] = byte
                // i & 3 of the word (S0), [2,3] = 0
                const uint32_t sel = 0x0c0c0000u | ((4u + (uint32_t)(i & 3)) << 8) | (uint32_t)(j & 3);
                const uint32_t a = __builtin_amdgcn_perm((i < 4) ? lo[j] : hi[j], offp[j >> 2], sel);
                v[j] = *reinterpret_cast<lds_u64*>(L + a);
            }
            uint32_t l = xor3(xor3((uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2]),
                              xor3((uint32_t)v[3], (uint32_t)v[4], (uint32_t)v[5]),
                              (uint32_t)v[6] ^ (uint32_t)v[7]);
            uint32_t h = xor3(xor3((uint32_t)(v[0] >> 32), (uint32_t)(v[1] >> 32), (uint32_t)(v[2] >> 32)),
                              xor3((uint32_t)(v[3] >> 32), (uint32_t)(v[4] >> 32), (uint32_t)(v[5] >> 32)),
                              (uint32_t)(v[6] >> 32) ^ (uint32_t)(v[7] >> 32));
            o[i] = ((uint64_t)h << 32) | l;
            // Scheduling fence after every kGostLpsFence output words: bounds
            // the ds_read lookahead, which otherwise grows until the 128-VGPR
            // budget of the 4-waves-per-SIMD kernels spills (kernel_resources test).
            if (kFence && (i + 1) % kFence == 0) __builtin_amdgcn_sched_barrier(0);
        }
    }
};
// The Sigma-in-LDS kernels (HMAC, keyed) keep the fence; the two-pass plain
// kernel (no Sigma live through the chain) fits 128 VGPRs without it.
using GostRot = GostRotF<kGostLpsFence>;

// Fills the 64 KiB rotated image (every thread, then barrier).
__device__ __forceinline__ void gost_stage_rot(uint64_t* lds) {
    for (int i = threadIdx.x; i < 256 * 32; i += blockDim.x) lds[i] = kGostAxDev.t[i & 7][i >> 5];
    __syncthreads();
}

// g_N(h, m) for a counter N whose upper 448 bits are zero (messages shorter
// than 2^61 bytes; the ABI caps lengths at 2^32): gost3411-2012.h:1110-1144.
// h and m in the table's lane order (natural order for GostFlat / GostRot;
// the hooks let tools/gost_half.hpp's lane-ordered layout run the same code).
#ifndef LCB_GOST_G_ROLLED
#define LCB_GOST_G_ROLLED 1
#endif
using lds_u64w = __attribute__((address_space(3))) uint64_t;
// ff (optional): LDS slots (stride ff_stride) that hold the feed-forward
// h ^ m through the 25 LPS instead of 16 VGPRs (the final g_0(h, Sigma),
// whose Sigma slots are free by then).  Read back volatile, so the compiler
// does not keep the stored words in registers anyway.
#if LCB_GOST_G_ROLLED
template <class Tab>
__device__ __forceinline__ void gost_g(uint64_t h[8], uint64_t n0, const uint64_t m[8], const Tab& T,
                                       lds_u64w* ff = nullptr, int ff_stride = 0) {
    // E(K, m) as 12 (K, t) steps plus the last key, from K_0 = h, t_0 = m:
    //   step r: K_{r+1} = LPS(K_r ^ c_r), t_{r+1} = LPS(t_r ^ K_{r+1}),
    //   c_0 = N, c_r = C_{r-1};  K_13 = LPS(K_12 ^ C_11) (step 12, no t).
    // One rolled loop: two LPS bodies per kernel instead of five, so every
    // g in a kernel shares one register allocation.
    uint64_t k[8], t[8], x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        k[i] = h[i];
        t[i] = m[i];
        h[i] ^= m[i];   // the feed-forward h ^ m of :1142, taken now: m and the old h die here
        if (ff) ff[i * ff_stride] = h[i];
    }
#pragma unroll 1
    for (int r = 0; r < 13; ++r) {
        if (r == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = k[i];
            T.xor_n(x, n0);
        } else {
            T.xor_c(x, k, r - 1);
        }
        T.lps(k, x);                                     // K_{r+1} = LPS(K_r ^ c_r)
        if (r == 12) break;
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = t[i] ^ k[i];
        T.lps(t, x);                                     // t_{r+1} = LPS(t_r ^ K_{r+1})
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (ff) h[i] = *(volatile lds_u64w*)&ff[i * ff_stride];
        h[i] ^= t[i] ^ k[i];                             // :1142 (h already holds h ^ m)
    }
}

#else
// Unrolled head and tail (round 2's form): K_1, t_1 and K_13 outside the
// 11-round loop.
template <class Tab>
__device__ __forceinline__ void gost_g(uint64_t h[8], uint64_t n0, const uint64_t m[8], const Tab& T,
                                       lds_u64w* = nullptr, int = 0) {
    uint64_t k[8], t[8], x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = h[i];
    T.xor_n(x, n0);
    T.lps(k, x);                                         // K = LPS(h ^ N)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        x[i] = k[i] ^ m[i];
        h[i] ^= m[i];
    }
    T.lps(t, x);                                         // t = LPS(K ^ m)
#pragma unroll 1
    for (int r = 0; r < 11; ++r) {
        T.xor_c(x, k, r);
        T.lps(k, x);                                     // K = LPS(K ^ C_r)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = t[i] ^ k[i];
        T.lps(t, x);                                     // t = LPS(t ^ K)
    }
    T.xor_c(x, k, 11);
    T.lps(k, x);                                         // K13 = LPS(K ^ C_11)
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] ^= t[i] ^ k[i];     // :1142
}
#endif

// The chaining value h is kept in the table's lane order between blocks
// (natural for the product's tables); Sigma and N in natural order.  The IV (all words equal) reads the
// same in every order.
//
// kSgLds words of Sigma (the last ones; 0, 4 or 8) live in LDS: word i of
// thread x at sgl_base[(i - (8 - kSgLds)) * kSgStride + x] (bind_sigma), not
// in VGPRs.  Sigma is touched once per block, and its 16 VGPRs are what
// pushed the batch kernels (4 waves per SIMD, 128 VGPRs) into scratch spills.
template <bool k256, int kSgStride = 0, int kSgLds = 0>
struct Gost {
    static constexpr int kBlock = 64, kDigest = k256 ? 32 : 64, kWords = 16;
    static constexpr int kSgReg = 8 - kSgLds;   // Sigma words 0 .. kSgReg-1 in VGPRs
    // kSgLds == 8: the counter N lives in LDS too (word 8 of the lane's slots).
    static constexpr bool kNLds = kSgLds == 8;
    uint64_t h[8], n0, sg[kSgReg ? kSgReg : 1];
    lds_u64w* sgl;   // kSgLds: this thread's LDS Sigma words (stride kSgStride)
    __device__ __forceinline__ void bind_sigma(lds_u64w* base) {
        if constexpr (kSgLds > 0) sgl = base + threadIdx.x;
    }
    __device__ __forceinline__ uint64_t sigma(int i) const {
        if (i >= kSgReg) return sgl[(i - kSgReg) * kSgStride];
        return sg[i];
    }
    // Sigma for the final g_0(h, Sigma), LDS words read back volatile: else
    // the compiler forwards the words just stored and keeps them in VGPRs
    // through g_0(h, N), which spilled.
    __device__ __forceinline__ uint64_t sigma_final(int i) const {
        if (i >= kSgReg) return *(volatile lds_u64w*)&sgl[(i - kSgReg) * kSgStride];
        return sg[i];
    }
    __device__ __forceinline__ uint64_t get_n() const {
        if constexpr (kNLds) return sgl[8 * kSgStride];
        else return n0;
    }
    __device__ __forceinline__ void set_n(uint64_t v) {
        if constexpr (kNLds) sgl[8 * kSgStride] = v;
        else n0 = v;
    }
    __device__ __forceinline__ void set_sigma(int i, uint64_t v) {
        if (i >= kSgReg) sgl[(i - kSgReg) * kSgStride] = v;
        else sg[i] = v;
    }
    __device__ __forceinline__ void init() {  // gost3411-2012.h:1713-1729
        // GOST-256's IV word made in place (volatile asm): as a plain constant
        // the compiler hoists it out of the persistent kernels' message loop
        // and then spills it.
        uint32_t iv = 0u;
        if (k256) asm volatile("v_mov_b32 %0, 0x1010101" : "=v"(iv));
#pragma unroll
        for (int i = 0; i < 8; ++i) { h[i] = ((uint64_t)iv << 32) | iv; set_sigma(i, 0); }
        set_n(0);
    }
    // One g_N step over raw LE words w (gost3411-2012.h:1129-1131).
    // Sigma += m mod 2^512 (gost3411-2012.h:996-1013).
    __device__ __forceinline__ void add_sigma(const uint64_t m[8]) {
        uint32_t carry = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint64_t s1 = sigma(i) + m[i];
            const uint32_t c1 = s1 < m[i];
            const uint64_t s2 = s1 + carry;
            carry = c1 | (s2 < s1);
            set_sigma(i, s2);
        }
    }
    template <class Tab>
    __device__ __forceinline__ void block(const uint32_t* w, uint64_t bits, const Tab& T) {
        uint64_t m[8], ml[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) m[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
        // Sigma first, so that only the lane-ordered copy of m stays live through g_N.
        add_sigma(m);
        T.to_lane(ml, m);
        gost_g(h, get_n(), ml, T);
        set_n(get_n() + bits);
    }
    // Tail + finalisation (gost3411-2012.h:1820-1839).
    template <class Tab>
    __device__ __forceinline__ void finish(uint32_t* w, uint32_t rem, const Tab& T) {
        put_byte(w, rem, 0x01u);
        block(w, (uint64_t)rem * 8u, T);
        uint64_t m[8], ml[8];
        m[0] = get_n();
#pragma unroll
        for (int i = 1; i < 8; ++i) m[i] = 0;
        T.to_lane(ml, m);
        gost_g(h, 0, ml, T);   // g_0(h, N)
#pragma unroll
        for (int i = 0; i < 8; ++i) m[i] = sigma_final(i);
        T.to_lane(ml, m);
        if constexpr (kSgLds == 8) gost_g(h, 0, ml, T, sgl, kSgStride);   // g_0(h, Sigma), h ^ Sigma in the Sigma slots
        else gost_g(h, 0, ml, T);   // g_0(h, Sigma)
    }
    // g_N alone (the two-pass form, gost_run2): Sigma is added up afterwards.
    template <class Tab>
    __device__ __forceinline__ void chain(const uint32_t* w, uint64_t bits, const Tab& T) {
        uint64_t m[8], ml[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) m[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
        T.to_lane(ml, m);
        gost_g(h, get_n(), ml, T);
        set_n(get_n() + bits);
    }
    template <class Tab>
    __device__ __forceinline__ void digest_words(uint32_t* out, const Tab& T) const {
        constexpr int first = 8 - kDigest / 8;  // last D bytes of h
        uint64_t hn[8];
        T.from_lane(hn, h);
#pragma unroll
        for (int i = 0; i < kDigest / 8; ++i) {
            out[2 * i] = (uint32_t)hn[first + i];
            out[2 * i + 1] = (uint32_t)(hn[first + i] >> 32);
        }
    }
    template <class Tab>
    __device__ __forceinline__ void save(uint32_t* p, const Tab& T) const {
        uint64_t hn[8];
        T.from_lane(hn, h);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            p[2 * i] = (uint32_t)hn[i]; p[2 * i + 1] = (uint32_t)(hn[i] >> 32);
            p[18 + 2 * i] = (uint32_t)sigma(i); p[19 + 2 * i] = (uint32_t)(sigma(i) >> 32);
        }
        const uint64_t n = get_n();
        p[16] = (uint32_t)n; p[17] = (uint32_t)(n >> 32);
    }
    template <class Tab>
    __device__ __forceinline__ void load(const uint32_t* p, const Tab& T) {
        uint64_t hn[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            hn[i] = (uint64_t)p[2 * i] | ((uint64_t)p[2 * i + 1] << 32);
            set_sigma(i, (uint64_t)p[18 + 2 * i] | ((uint64_t)p[19 + 2 * i] << 32));
        }
        T.to_lane(h, hn);
        set_n((uint64_t)p[16] | ((uint64_t)p[17] << 32));
    }
};

// Message sources of gost_run: whole 64-B block j (j < nfull) and the
// zero-filled tail of r = rem() < 64 bytes (tail_n), as raw LE words.
// opaque(): the same source with its pointers passed through an empty asm,
// so a second pass's loads are not merged with the first pass's (which would
// keep the first pass's tail block live across the chain: 104 B/lane spilled).
__device__ __forceinline__ const uint8_t* opaque_ptr(const uint8_t* p) {
    asm volatile("" : "+v"(p));
    return gptr(p);   // still global memory: global_load, not flat_load
}
struct GostPlainSrc {   // msg[0, len)
    const uint8_t* p;
    uint64_t len;
    __device__ __forceinline__ GostPlainSrc opaque() const { return {opaque_ptr(p), len}; }
    __device__ __forceinline__ uint64_t nfull() const { return len >> 6; }
    __device__ __forceinline__ uint32_t rem() const { return (uint32_t)(len & 63u); }
    __device__ __forceinline__ void block(uint64_t j, uint32_t w[16]) const { load_full64(p + 64 * j, w); }
    __device__ __forceinline__ void tail_n(uint32_t w[16], uint32_t r) const { load_tail64(p + (len & ~63ull), r, w); }
};
struct GostVirtSrc {    // A[0, la) || B[0, lb) (keyed batches), nothing copied
    const uint8_t* A;
    uint64_t la;
    const uint8_t* B;
    uint64_t lb;
    __device__ __forceinline__ GostVirtSrc opaque() const { return {opaque_ptr(A), la, opaque_ptr(B), lb}; }
    __device__ __forceinline__ uint64_t nfull() const { return (la + lb) >> 6; }
    __device__ __forceinline__ uint32_t rem() const { return (uint32_t)((la + lb) & 63u); }
    __device__ __forceinline__ void block(uint64_t j, uint32_t w[16]) const {
        const uint64_t pos = 64 * j;
        if (pos + 64 <= la) load_full64(A + pos, w);
        else if (pos >= la) load_full64(B + (pos - la), w);
        else load_vblock64(A, la, B, lb, pos, w);     // the seam block
    }
    __device__ __forceinline__ void tail_n(uint32_t w[16], uint32_t r) const {   // r == rem()
        const uint64_t pos = (la + lb) & ~63ull;
        if (pos >= la) load_tail64(B + (pos - la), r, w);
        else load_vblock64(A, la, B, lb, pos, w);     // zero fill past la + lb
    }
};

// One whole message through a GOST state (gost3411_2012_update + _final,
// gost3411-2012.h:1743-1843): the whole blocks, then the tail || 0x01 and the
// two g_0 steps (Gost::finish).
template <class G, class Src, class Tab>
__device__ __forceinline__ void gost_run(G& st, const Src& src, const Tab& T) {
    uint32_t w[16];
    const uint64_t nfull = src.nfull();
    for (uint64_t j = 0; j < nfull; ++j) {
        src.block(j, w);
        st.block(w, 512, T);
    }
    const uint32_t rem = src.rem();
    src.tail_n(w, rem);
    st.finish(w, rem, T);
}

// Sigma += m mod 2^512 on a register Sigma (gost3411-2012.h:996-1013).
__device__ __forceinline__ void gost_sigma_add(uint64_t sg[8], const uint32_t w[16]) {
    uint32_t carry = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint64_t m = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
        const uint64_t s1 = sg[i] + m;
        const uint32_t c1 = s1 < m;
        const uint64_t s2 = s1 + carry;
        carry = c1 | (s2 < s1);
        sg[i] = s2;
    }
}

// The two-pass form of gost_run (plain batches, Sigma starting at zero):
// Sigma = the sum of the message's blocks is independent of the g_N chain
// (gost3411-2012.h:1129-1142: Sigma += m beside h = g_N(h, m)), so the chain
// runs first with no Sigma at all -- whole blocks, the tail || 0x01 block,
// then g_0(h, N) (:1836) -- and a second pass over the message adds Sigma up
// from the bytes again (re-read: L2 / Infinity-Cache resident by then, the
// kernel is LDS-bound at ~0.04 of HBM) right before the last g_0(h, Sigma)
// (:1837).  Sigma costs no VGPRs and no LDS through the 19 g's of a 1 KiB
// message, and nothing is live across g_0(h, N) but h.
// The two-pass form in two parts, for segmented long waves (gost_seg_kernel):
// the chain over whole blocks [j0, j1) ...
template <class G, class Src, class Tab>
__device__ __forceinline__ void gost_chain_blocks(G& st, const Src& src, const Tab& T, uint64_t j0, uint64_t j1) {
    uint32_t w[16];
    for (uint64_t j = j0; j < j1; ++j) {
#if LCB_LANE_PRIO
        if ((j & 15) == 0) wave_prio_left((j1 - j) * 64u);
#endif
        src.block(j, w);
        st.chain(w, 512, T);
    }
}
// ... and the rest after the last whole block: the tail || 0x01 block,
// g_0(h, N), the Sigma pass over the whole message, g_0(h, Sigma).
template <class G, class Src, class Tab>
__device__ __forceinline__ void gost_run2_final(G& st, const Src& src, const Tab& T) {
    uint32_t w[16];
    const uint64_t nfull = src.nfull();
    const uint32_t rem = src.rem();
    src.tail_n(w, rem);
    put_byte(w, rem, 0x01u);
    st.chain(w, (uint64_t)rem * 8u, T);
    {
        uint64_t m[8], ml[8];
        m[0] = st.get_n();
#pragma unroll
        for (int i = 1; i < 8; ++i) m[i] = 0;
        T.to_lane(ml, m);
        gost_g(st.h, 0, ml, T);                   // g_0(h, N)
    }
    uint64_t sg[8], sl[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) sg[i] = 0;
    const Src s2 = src.opaque();
    for (uint64_t j = 0; j < nfull; ++j) {
        s2.block(j, w);
        gost_sigma_add(sg, w);
    }
    // The tail's byte masks re-formed from an opaque copy of rem: else they
    // are computed once and kept (spilled) across the chain.
    uint32_t r2 = rem;
    asm volatile("" : "+v"(r2));
    s2.tail_n(w, r2);
    put_byte(w, r2, 0x01u);
    gost_sigma_add(sg, w);
    T.to_lane(sl, sg);
    gost_g(st.h, 0, sl, T);                       // g_0(h, Sigma)
}
// gost_run2 = gost_chain_blocks(0, nfull) + gost_run2_final, written out
// as one body: that is the machine code the plain kernel was tuned on (the
// split form compiles to different code at the same 124 VGPRs).
template <class G, class Src, class Tab>
__device__ __forceinline__ void gost_run2(G& st, const Src& src, const Tab& T) {
    uint32_t w[16];
    const uint64_t nfull = src.nfull();
    for (uint64_t j = 0; j < nfull; ++j) {
#if LCB_LANE_PRIO
        if ((j & 15) == 0) wave_prio_left((nfull - j) * 64u);
#endif
        src.block(j, w);
        st.chain(w, 512, T);
    }
    const uint32_t rem = src.rem();
    src.tail_n(w, rem);
    put_byte(w, rem, 0x01u);
    st.chain(w, (uint64_t)rem * 8u, T);
    {
        uint64_t m[8], ml[8];
        m[0] = st.get_n();
#pragma unroll
        for (int i = 1; i < 8; ++i) m[i] = 0;
        T.to_lane(ml, m);
        gost_g(st.h, 0, ml, T);                   // g_0(h, N)
    }
    uint64_t sg[8], sl[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) sg[i] = 0;
    const Src s2 = src.opaque();
    for (uint64_t j = 0; j < nfull; ++j) {
        s2.block(j, w);
        gost_sigma_add(sg, w);
    }
    uint32_t r2 = rem;
    asm volatile("" : "+v"(r2));
    s2.tail_n(w, r2);
    put_byte(w, r2, 0x01u);
    gost_sigma_add(sg, w);
    T.to_lane(sl, sg);
    gost_g(st.h, 0, sl, T);                       // g_0(h, Sigma)
}

// HMAC outer pass (gost3411-2012.h:1902-1934): the D-byte inner digest dw
// hashed from the state after K ^ opad (mid_outer).
template <class G, class Tab>
__device__ __forceinline__ void gost_outer(G& o, const uint32_t* dw, const uint32_t* mid_outer, const Tab& T) {
    o.load(mid_outer, T);
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = (i < G::kDigest / 4) ? dw[i] : 0u;
    if (G::kDigest == 64) {       // a 64-byte digest is a full block, then an
        o.block(w, 512, T);       // empty pad block (gost3411-2012.h:1783-1793)
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = 0u;
        o.finish(w, 0, T);
    } else {
        o.finish(w, G::kDigest, T);  // 32 bytes: the digest is the tail block
    }
}

template <class G, class Tab>
__device__ __forceinline__ void gost_message(G& st, const uint8_t* msg, uint64_t len, const Tab& T) {
    gost_run(st, GostPlainSrc{msg, len}, T);
}

}  // namespace lcbgpu
