// crc_kernels.hip — batched CRC-32 (include/lcb_crc32_gpu.h) for gfx950.
//
// Grid as the digest kernels: one lane per buffer, 256-thread workgroups,
// optional length-bucketing permutation.  The variant's slicing-by-8 tables
// (8 KiB) are staged into LDS; every lookup is a ds_read_b32 at a
// data-dependent address, so the kernel is bound by HBM streaming or LDS
// bank conflicts, whichever is slower.
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

template <int V>
static void launch_crc_v(const KArgs& a, hipStream_t s) {
    const uint64_t blocks = (a.count + 255) / 256;
    hipLaunchKernelGGL(crc_batch_kernel<V>, dim3((unsigned)blocks), dim3(256), 0, s, a);
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
