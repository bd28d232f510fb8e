// gost_half.hpp — EXPERIMENT (not product code): a lane-ordered GOST LPS
// layout measured against the product's GostRot by tools/gost_lanes_ab.hip
// and tools/lds_rate.hip (GOST A/B).  Plugs into the product's
// Gost<k256> / gost_g through their table hooks (to_lane, from_lane, xor_n,
// xor_c, lps).
#pragma once
#include "../liblcb_amd/csrc/gost_device.hpp"

namespace lcbgpu {

// Lane-ordered, half-rotated LPS (the batch kernels): no word rotation at all.
//
// GostRot spends 48 of its ~185 VALU per LPS rotating the 8 input words into
// the lane's bank order.  Here each lane keeps every 512-bit value of g_N in
// its own word order instead -- position j' holds word pi(j') =
// (j' & 4) | ((j' + rho) & 3), a rotation by rho = lane & 3 inside each half --
// and LPS maps that order to itself: output position i' is word pi(i'), i.e.
// byte pi(i') of every input word, whose half (i' >> 2) is static and whose
// byte inside the half is the lane's perm selector.  Lookups stay one
// v_perm_b32 each (table byte -> address bits 8-15, bank-pair offset -> bits
// 0-7, half of the table index -> bit 16).  At static step j' the 32 lanes of
// a ds_read_b64 group read tables pi(j') -- 4 distinct tables of one half --
// so the LDS holds 8 replicas c of the 8 tables: table j of replica c alone in
// bank pair 4c + (j & 3), rows (j >> 2) * 256 + b (128 KiB), lane l taking
// rho = l & 3, c = (l & 31) >> 2: 32 different bank pairs per group,
// conflict-free whatever the data.  LPS = 64 perm + 64 XOR (bitop3 xor3).
// The round constants, permuted per rho, sit after the image (4 x 784 B,
// the stride putting the four copies in different banks); N is added to the
// position of word 0 under a per-lane mask; the message and the chaining
// value are permuted in and out once per g_N (gost_g).
constexpr uint32_t kGostHalfImage = 131072;           // bytes of the 8-replica image
constexpr uint32_t kGostHalfCStride = 784;            // bytes per rho copy of the constants
constexpr uint32_t kGostHalfLdsU64 = (kGostHalfImage + 4 * kGostHalfCStride) / 8;

struct GostHalf {
    lds_u8* L;
    uint32_t off[8];     // ((j' >> 2) << 16) | (4c + ((j' + rho) & 3)) * 8
    uint32_t sel[4];     // perm selector: byte (q + rho) & 3 of the source half -> bits 8-15
    uint32_t rho;        // this rho's constants: C[r][pi(j')] at kGostHalfImage + rho * 784 + 64 r + 8 j'
    __device__ __forceinline__ void init(lds_u8* lds) {
        L = lds;
        const uint32_t l = threadIdx.x & 31u, c = l >> 2;
        rho = l & 3u;
#pragma unroll
        for (int j = 0; j < 8; ++j) off[j] = ((uint32_t)(j >> 2) << 16) | ((4u * c + (((uint32_t)j + rho) & 3u)) * 8u);
#pragma unroll
        for (int q = 0; q < 4; ++q) sel[q] = 0x0c020000u | ((4u + (((uint32_t)q + rho) & 3u)) << 8);
    }
    __device__ __forceinline__ uint32_t m1() const { return (rho & 1u) ? 0xffffffffu : 0u; }
    __device__ __forceinline__ uint32_t m2() const { return (rho & 2u) ? 0xffffffffu : 0u; }
    template <int S>
    __device__ __forceinline__ static void hrot(uint32_t (&v)[8], uint32_t m) {  // v[j] <- v[(j & 4) | ((j + S) & 3)] where m
        uint32_t t[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) t[j] = ch3(m, v[(j & 4) | ((j + S) & 3)], v[j]);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = t[j];
    }
    // natural -> lane order: o[j'] = v[pi(j')]
    __device__ __forceinline__ void to_lane(uint64_t o[8], const uint64_t v[8]) const {
        uint32_t lo[8], hi[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { lo[j] = (uint32_t)v[j]; hi[j] = (uint32_t)(v[j] >> 32); }
        const uint32_t a = m1(), b = m2();
        hrot<1>(lo, a); hrot<1>(hi, a);
        hrot<2>(lo, b); hrot<2>(hi, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = ((uint64_t)hi[j] << 32) | lo[j];
    }
    // lane -> natural order: o[pi(j')] = v[j'] (rotation by -rho)
    __device__ __forceinline__ void from_lane(uint64_t o[8], const uint64_t v[8]) const {
        uint32_t lo[8], hi[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { lo[j] = (uint32_t)v[j]; hi[j] = (uint32_t)(v[j] >> 32); }
        const uint32_t a = m1(), b = m2();
        hrot<3>(lo, a); hrot<3>(hi, a);
        hrot<2>(lo, b); hrot<2>(hi, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = ((uint64_t)hi[j] << 32) | lo[j];
    }
    // x ^= N (N < 2^64: word 0 only, at the position j' with pi(j') = 0)
    __device__ __forceinline__ void xor_n(uint64_t x[8], uint64_t n0) const {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t e = (((uint32_t)j + rho) & 3u) == 0u ? n0 : 0ull;
            x[j] ^= e;
        }
    }
    __device__ __forceinline__ void xor_c(uint64_t x[8], const uint64_t k[8], int r) const {
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        using lds_v4u = __attribute__((address_space(3))) const v4u;
        const lds_v4u* c = reinterpret_cast<const lds_v4u*>(L + kGostHalfImage + rho * kGostHalfCStride + 64 * r);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const v4u v = c[q];
            x[2 * q] = k[2 * q] ^ (((uint64_t)v[1] << 32) | v[0]);
            x[2 * q + 1] = k[2 * q + 1] ^ (((uint64_t)v[3] << 32) | v[2]);
        }
    }
    // LPS in lane order: o[i'] = XOR_j' Ax[pi(j')][byte pi(i') of x[j']].
    __device__ __forceinline__ void lps(uint64_t o[8], const uint64_t x[8]) const {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            uint64_t v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t a = __builtin_amdgcn_perm((i < 4) ? (uint32_t)x[j] : (uint32_t)(x[j] >> 32), off[j],
                                                         sel[i & 3]);
                v[j] = *reinterpret_cast<lds_u64*>(L + a);
            }
            uint32_t l = xor3(xor3((uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2]),
                              xor3((uint32_t)v[3], (uint32_t)v[4], (uint32_t)v[5]),
                              (uint32_t)v[6] ^ (uint32_t)v[7]);
            uint32_t h = xor3(xor3((uint32_t)(v[0] >> 32), (uint32_t)(v[1] >> 32), (uint32_t)(v[2] >> 32)),
                              xor3((uint32_t)(v[3] >> 32), (uint32_t)(v[4] >> 32), (uint32_t)(v[5] >> 32)),
                              (uint32_t)(v[6] >> 32) ^ (uint32_t)(v[7] >> 32));
            o[i] = ((uint64_t)h << 32) | l;
        }
    }
};

// Fills the 8-replica image and the permuted constants (every thread, then barrier).
__device__ __forceinline__ void gost_stage_half(uint64_t* lds) {
    for (int i = threadIdx.x; i < 16384; i += blockDim.x) {
        const int j = ((i >> 13) << 2) | (i & 3), b = (i >> 5) & 255;
        lds[i] = kGostAxDev.t[j][b];
    }
    for (int i = threadIdx.x; i < 4 * 96; i += blockDim.x) {
        const int rho = i / 96, r = (i % 96) >> 3, jp = i & 7;
        lds[kGostHalfImage / 8 + rho * (kGostHalfCStride / 8) + r * 8 + jp] = kGostC[r][(jp & 4) | ((jp + rho) & 3)];
    }
    __syncthreads();
}

}  // namespace lcbgpu
