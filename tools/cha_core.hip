// cha_core.hip — register-only ChaCha double-round throughput on gfx950,
// to separate the VALU bound of the ChaCha kernels from their memory side.
// Variants: one lane per block (LANE, 4 independent quarter-round chains per
// lane) with 1 or 2 blocks per lane, and the quad/DPP layout (QUAD, one
// chain per lane) with 1 or 2 blocks per lane.  Reports ns per block-double-
// round over the whole device, at 1..8 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/cha_core tools/cha_core.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#ifndef ROT
#define ROT 0
#endif
__device__ __forceinline__ uint32_t rotl(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, 32u - n); }
// ROT 0: every rotate is v_alignbit_b32 x, x, n.  ROT 1: byte rotates (16, 8)
// as v_perm_b32.  ROT 2: 16/8 as v_perm, 12/7 as shift + v_lshl_or.
__device__ __forceinline__ uint32_t rot16(uint32_t x) {
#if ROT >= 1
    return __builtin_amdgcn_perm(x, x, 0x01000302u);
#else
    return rotl(x, 16);
#endif
}
__device__ __forceinline__ uint32_t rot8(uint32_t x) {
#if ROT >= 1
    return __builtin_amdgcn_perm(x, x, 0x02010003u);
#else
    return rotl(x, 8);
#endif
}
template <int N> __device__ __forceinline__ uint32_t rotn(uint32_t x) {
#if ROT >= 2
    return (x << N) | (x >> (32 - N));
#else
    return rotl(x, N);
#endif
}
__device__ __forceinline__ void qr(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
    a += b; d = rot16(d ^ a);
    c += d; b = rotn<12>(b ^ c);
    a += b; d = rot8(d ^ a);
    c += d; b = rotn<7>(b ^ c);
}
template <int C> __device__ __forceinline__ uint32_t qp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, C, 0xf, 0xf, true);
}
__device__ __forceinline__ void dr_full(uint32_t* x) {
    qr(x[0], x[4], x[8], x[12]); qr(x[1], x[5], x[9], x[13]);
    qr(x[2], x[6], x[10], x[14]); qr(x[3], x[7], x[11], x[15]);
    qr(x[0], x[5], x[10], x[15]); qr(x[1], x[6], x[11], x[12]);
    qr(x[2], x[7], x[8], x[13]); qr(x[3], x[4], x[9], x[14]);
}
__device__ __forceinline__ void dr_quad(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
    qr(a, b, c, d);
    b = qp<0x39>(b); c = qp<0x4E>(c); d = qp<0x93>(d);
    qr(a, b, c, d);
    b = qp<0x93>(b); c = qp<0x4E>(c); d = qp<0x39>(d);
}

template <int NB>
__global__ __launch_bounds__(256) void k_lane(uint32_t* out, int iters) {
    uint32_t x[NB][16];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int k = 0; k < 16; ++k) x[j][k] = threadIdx.x * 16 + k + j;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < NB; ++j) dr_full(x[j]);
    }
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int k = 0; k < 16; ++k) r ^= x[j][k];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int NB>
__global__ __launch_bounds__(256) void k_quad(uint32_t* out, int iters) {
    uint32_t a[NB], b[NB], c[NB], d[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) { a[j] = threadIdx.x + j; b[j] = a[j] * 3; c[j] = a[j] * 5; d[j] = a[j] * 7; }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < NB; ++j) dr_quad(a[j], b[j], c[j], d[j]);
    }
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < NB; ++j) r ^= a[j] ^ b[j] ^ c[j] ^ d[j];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

typedef void (*kfn)(uint32_t*, int);

int main() {
    uint32_t* out;
    hipMalloc(&out, 256 * 256 * 16 * sizeof(uint32_t));
    struct { const char* name; kfn f; int blocks_per_lane_x4; } ks[] = {
        {"lane x1 (1 block/lane)", k_lane<1>, 4}, {"lane x2 (2 blocks/lane)", k_lane<2>, 8},
        {"quad x1 (1/4 block/lane)", k_quad<1>, 1}, {"quad x2", k_quad<2>, 2}, {"quad x4", k_quad<4>, 4}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 2000;
    for (auto& k : ks) {
        for (int w = 1; w <= 8; w *= 2) {
            const int grid = 256 * w;  // w workgroups of 4 waves per CU = w waves per SIMD
            hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), 0, 0, out, 10);
            hipDeviceSynchronize();
            hipEventRecord(e0, 0);
            hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), 0, 0, out, iters);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            // blocks processed: threads * blocks_per_lane_x4 / 4
            const double blocks = (double)grid * 256 * k.blocks_per_lane_x4 / 4.0;
            const double ndr = blocks * iters;
            printf("%-26s waves/SIMD %d  %.3f ms  %.3f ns per block-double-round x1e3 (device)  "
                   "=> ChaCha20 1GiB: %.1f us\n",
                   k.name, w, ms, ms * 1e6 / ndr * 1e3, ms * 1e3 / ndr * 10 * 16777216.0);
        }
    }
    return 0;
}
