// lds_rate.hip — is the GOST LPS bound by the LDS or by the VALU?
// A chain of LPS transforms (tools/gost_half.hpp GostHalf: 64 conflict-free
// data-dependent ds_read_b64 + 64 v_perm_b32 + 64 xor per LPS per lane) with
// E extra independent v_xor_b32 per LPS added beside it.  If the time per LPS
// does not move as E grows the LPS is LDS-bound; the slope is the VALU cost.
// Also: reads only (address from the previous read, no perm), to get the
// bare ds_read_b64 rate of this access pattern.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "gost_half.hpp"

using namespace lcbgpu;

template <int kExtra>
__global__ __launch_bounds__(1024) void k_lps(uint64_t* out, int iters) {
    __shared__ __attribute__((aligned(256))) uint64_t Timg[kGostHalfLdsU64];
    gost_stage_half(Timg);
    GostHalf T;
    T.init((lds_u8*)Timg);
    uint64_t x[8], o[8];
    for (int i = 0; i < 8; ++i) x[i] = 0x9e3779b97f4a7c15ull * (threadIdx.x + 7 * blockIdx.x + 13 * i + 1);
    uint32_t d0 = threadIdx.x, d1 = blockIdx.x;
    for (int it = 0; it < iters; ++it) {
        T.lps(o, x);
#pragma unroll
        for (int e = 0; e < kExtra; e += 2) {
            d0 ^= (d1 + e);
            d1 ^= (d0 + e);
            asm volatile("" : "+v"(d0), "+v"(d1));
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = o[i];
    }
    uint64_t a = d0 ^ d1;
    for (int i = 0; i < 8; ++i) a ^= x[i];
    out[blockIdx.x * 1024 + threadIdx.x] = a;
}

// reads only: 8 chains of 8 reads, next address = low bits of the value read
__global__ __launch_bounds__(1024) void k_reads(uint64_t* out, int iters) {
    __shared__ __attribute__((aligned(256))) uint64_t Timg[kGostHalfLdsU64];
    gost_stage_half(Timg);
    const uint32_t l = threadIdx.x & 31u, off = (l & 31u) * 8u;
    uint32_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = ((threadIdx.x * 37u + 11u * i) & 0x1ff) << 8 | off;
    uint64_t acc = 0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            uint64_t v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<lds_u64*>((lds_u8*)Timg + (a[j] ^ (uint32_t)(i << 9)));
            uint64_t s = v[0] ^ v[1] ^ v[2] ^ v[3] ^ v[4] ^ v[5] ^ v[6] ^ v[7];
            acc ^= s;
            a[i] = (((uint32_t)s & 0x1ff) << 8) | off;
        }
    }
    out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

template <class F>
static float best(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    float m = 1e30f;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(a, 0);
        f();
        hipEventRecord(b, 0);
        if (hipEventSynchronize(b) != hipSuccess || hipGetLastError() != hipSuccess) { printf("failed\n"); exit(1); }
        float ms;
        hipEventElapsedTime(&ms, a, b);
        m = ms < m ? ms : m;
    }
    return m;
}

int main() {
    const int blocks = 256 * 4, iters = 2000;
    uint64_t* out;
    hipMalloc(&out, (size_t)blocks * 1024 * 8);
    // per CU: blocks/256 workgroups x 16 waves x iters LPS x 64 ds_read_b64
    const double reads_per_cu = (double)blocks / 256 * 16 * iters * 64;
    auto rep = [&](const char* n, float ms, double valu_per_lps) {
        const double cyc = ms * 1e-3 * 2.4e9;
        printf("%-26s %.3f ms  %.2f cycles per ds_read_b64 per CU (2.4 GHz)  ~%.0f VALU/LPS\n", n, ms, cyc / reads_per_cu,
               valu_per_lps);
    };
    rep("lps", best([&] { hipLaunchKernelGGL(k_lps<0>, dim3(blocks), dim3(1024), 0, 0, out, iters); }), 128);
    rep("lps + 32 xor", best([&] { hipLaunchKernelGGL(k_lps<32>, dim3(blocks), dim3(1024), 0, 0, out, iters); }), 160);
    rep("lps + 64 xor", best([&] { hipLaunchKernelGGL(k_lps<64>, dim3(blocks), dim3(1024), 0, 0, out, iters); }), 192);
    rep("lps + 128 xor", best([&] { hipLaunchKernelGGL(k_lps<128>, dim3(blocks), dim3(1024), 0, 0, out, iters); }), 256);
    rep("lps + 256 xor", best([&] { hipLaunchKernelGGL(k_lps<256>, dim3(blocks), dim3(1024), 0, 0, out, iters); }), 384);
    rep("reads only (+xor)", best([&] { hipLaunchKernelGGL(k_reads, dim3(blocks), dim3(1024), 0, 0, out, iters); }), 72);
    return 0;
}
