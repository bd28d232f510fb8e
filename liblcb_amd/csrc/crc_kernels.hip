// crc_kernels.hip — batched CRC-32 (include/lcb_crc32_gpu.h) for gfx950.
//
// Grid as the digest kernels: one lane per buffer, 256-thread workgroups,
// optional length-bucketing permutation.  The variant's slicing-by-8 tables
// (8 KiB) are staged into LDS; every lookup is a ds_read_b32 at a
// data-dependent address.  Fixed-stride batches of whole 128-B lines take the
// LDS-DMA line stream (crc_fixed_lds_kernel), everything else the per-lane
// kernel; both run at about the HBM rate on 1 KiB buffers.
#include <hip/hip_runtime.h>
#include "crc_device.hpp"
#include "lcb_internal.hpp"


namespace lcbgpu {

template <int V>
__global__ __launch_bounds__(256) void crc_batch_kernel(KArgs a) {
    using Var = CrcVar<V>;
    __shared__ uint32_t T[8 * 256];
    crc_stage_tables(T, Var::kFam);  // before any early return: it synchronises
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.count) return;
    const uint64_t idx = a.order ? (uint64_t)gptr(a.order)[i] : i;
    const uint8_t* msg = gptr(a.data) + (a.offsets ? gptr(a.offsets)[idx] : idx * a.stride);
    const uint64_t len = a.lengths ? (uint64_t)gptr(a.lengths)[idx] : (uint64_t)a.fixed_len;
    const uint32_t c = a.init ? gptr(a.init)[idx] : Var::kOneshot;
    CrcRule<Var::kRefl> R{T};
    uint32_t r = crc_message(R, Var::kInv ? ~c : c, msg, len);
    gptr(reinterpret_cast<uint32_t*>(a.digests))[idx] = Var::kInv ? ~r : r;
}

// Fixed-stride batches (lcb_internal.hpp fixed_stride_lines): the 128-B lines
// arrive through the per-wave LDS-DMA line stream (LdsStridedStream,
// hash_device.hpp), line L+1 in flight while line L is folded in.
// kAux: the line stream's cache policy, chosen by alignment as for the digest
// kernels (md_fixed_lds_kernel).
#ifndef LCB_CRC_XCD
#define LCB_CRC_XCD 1
#endif
template <int V, int kAux>
__global__ __launch_bounds__(256) void crc_fixed_lds_kernel(KArgs a) {
    using Var = CrcVar<V>;
    __shared__ uint32_t T[8 * 256];
    __shared__ __attribute__((aligned(16))) uint8_t slab[4][kSlabBytes];
    crc_stage_tables(T, Var::kFam);  // before any early return: it synchronises
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint64_t wave_first = ((uint64_t)(LCB_CRC_XCD ? xcd_block() : blockIdx.x) * 4 + wv) * 64;
    if (wave_first >= a.count) return;  // wave-uniform
    // A partial last wave moves back over its predecessor's records (count
    // >= 64) and stores only its own.
    const uint64_t last = a.count - 1, nlines = a.fixed_len / 128;
    const uint32_t skip = wave_first + 63 > last ? (uint32_t)(wave_first + 63 - last) : 0u;
    wave_first -= skip;
    LdsStridedStream ls;
    ls.init(a.data, a.stride, wave_first, lane, &slab[wv][0]);
    const uint64_t i = wave_first + lane;
    const uint32_t c = a.init ? gptr(a.init)[i] : Var::kOneshot;
    const CrcRule<Var::kRefl> R{T};
    uint32_t r = Var::kInv ? ~c : c;
    if (nlines) ls.issue<kAux>(0);
    for (uint64_t L = 0; L < nlines; ++L) {
        uint32_t w0[16], w1[16];
        ls.take(w0, w1);
        if (L + 1 < nlines) ls.issue<kAux>(L + 1);
#pragma unroll
        for (int j = 0; j < 8; ++j) r = R.step8(r, w0[2 * j], w0[2 * j + 1]);
#pragma unroll
        for (int j = 0; j < 8; ++j) r = R.step8(r, w1[2 * j], w1[2 * j + 1]);
    }
    if (lane < skip) return;
    r = crc_message(R, r, gptr(a.data) + i * a.stride + nlines * 128, (uint64_t)a.fixed_len - nlines * 128);
    gptr(reinterpret_cast<uint32_t*>(a.digests))[i] = Var::kInv ? ~r : r;
}

template <int V>
static void launch_crc_v(const KArgs& a, hipStream_t s) {
    const uint64_t blocks = (a.count + 255) / 256;
    if (!fixed_stride_lines(a))
        hipLaunchKernelGGL(crc_batch_kernel<V>, dim3((unsigned)blocks), dim3(256), 0, s, a);
    else if (a.stride % 128 == 0 && reinterpret_cast<uintptr_t>(a.data) % 128 == 0)
        hipLaunchKernelGGL((crc_fixed_lds_kernel<V, kLdsAux>), dim3((unsigned)blocks), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((crc_fixed_lds_kernel<V, kGatherAux>), dim3((unsigned)blocks), dim3(256), 0, s, a);
}

void launch_crc(int variant, const KArgs& a, hipStream_t s) {
    switch (variant) {
    case 1: launch_crc_v<1>(a, s); break;
    case 2: launch_crc_v<2>(a, s); break;
    case 3: launch_crc_v<3>(a, s); break;
    case 4: launch_crc_v<4>(a, s); break;
    case 5: launch_crc_v<5>(a, s); break;
    case 6: launch_crc_v<6>(a, s); break;
    case 7: launch_crc_v<7>(a, s); break;
    case 8: launch_crc_v<8>(a, s); break;
    }
}

// Host copy of the compile-time tables (tests pin table 0 of each family
// against the reference's crc32_tbl256_* arrays).
void crc_table_host(int variant, uint32_t* out /* 8 x 256 */) {
    static constexpr CrcTables kHost[5] = {
        make_crc_tables(0x04c11db7u, false), make_crc_tables(0x04c11db7u, true),
        make_crc_tables(0x1edc6f41u, true),  make_crc_tables(0xa833982bu, true),
        make_crc_tables(0x814141abu, false)};
    static constexpr int kFam[9] = {0, CrcVar<1>::kFam, CrcVar<2>::kFam, CrcVar<3>::kFam, CrcVar<4>::kFam,
                                    CrcVar<5>::kFam, CrcVar<6>::kFam, CrcVar<7>::kFam, CrcVar<8>::kFam};
    const CrcTables& t = kHost[kFam[variant]];
    for (int k = 0; k < 8; ++k)
        for (int b = 0; b < 256; ++b) out[k * 256 + b] = t.t[k][b];
}

}  // namespace lcbgpu
