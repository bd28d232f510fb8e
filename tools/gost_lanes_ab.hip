// gost_lanes_ab.hip — A/B of two GOST R 34.11-2012 layouts on MI355X
// (VERDICT r1 item 6): 1 Mi messages of 1 KiB,
// GOST-512, device-resident, digests compared between the layouts.
//
//   lane   one lane per message, the product's form (gost_device.hpp GostRot:
//          64 KiB lane-rotated bank-sliced LPS image, 192 VALU + 64 ds_read_b64
//          per LPS per message); workgroups of 256 (2 per CU, the product
//          kernel's shape) and of 512 threads (the launch bound lets the
//          compiler use 128 VGPRs: 4 waves per SIMD)
//   oct    eight lanes per message, lane r holding state word r: the lane
//          looks up table r (no rotation needed for conflict-free banks) with
//          the byte order permuted per lane so that the 8 -> 1 XOR
//          reduce-scatter over the 8 lanes is three static DPP butterflies
//          (row_half_mirror, quad_perm xor-2, quad_perm xor-1) with no
//          selects: 26 VALU per lane per LPS = 208 per message; the state
//          needs 2 VGPRs per 512-bit value instead of 16, so the occupancy
//          is set by the LDS image, not by registers
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gost_lanes_ab.hip -o build_exp/gost_lanes_ab
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <vector>

#include "gost_half.hpp"

using namespace lcbgpu;

constexpr uint64_t kLen = 1024;

// ------------------------------------------------------------ one lane per message
template <int kThreads, int kMinBlocks>
__global__ __launch_bounds__(kThreads, kMinBlocks) void k_lane(const uint8_t* data, uint64_t n, uint64_t* out) {
    __shared__ __attribute__((aligned(256))) uint64_t Timg[256 * 32];
    gost_stage_rot(Timg);
    GostRot T;
    T.init((lds_u8*)Timg);
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    Gost<false> st;
    st.init();
    gost_message(st, data + i * kLen, kLen, T);
    uint32_t dw[16];
    st.digest_words(dw, T);
    for (int w = 0; w < 8; ++w) out[i * 8 + w] = (uint64_t)dw[2 * w] | ((uint64_t)dw[2 * w + 1] << 32);
}

// ------------------------------------------------------------ lane-ordered, half-rotated (GostHalf)
template <int kThreads>
__global__ __launch_bounds__(kThreads) void k_half(const uint8_t* data, uint64_t n, uint64_t* out) {
    __shared__ __attribute__((aligned(256))) uint64_t Timg[kGostHalfLdsU64];
    gost_stage_half(Timg);
    GostHalf T;
    T.init((lds_u8*)Timg);
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    Gost<false> st;
    st.init();
    gost_message(st, data + i * kLen, kLen, T);
    uint32_t dw[16];
    st.digest_words(dw, T);
    for (int w = 0; w < 8; ++w) out[i * 8 + w] = (uint64_t)dw[2 * w] | ((uint64_t)dw[2 * w + 1] << 32);
}

// ------------------------------------------------------------ eight lanes per message
template <int C>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, C, 0xf, 0xf, false);
}
constexpr int kHalfMirror = 0x141, kXor2 = 0x4E, kXor1 = 0xB1;

struct Oct {
    lds_u8* L;
    uint32_t off;       // (8c + r) * 8: table r of replica c
    uint32_t selq[4];   // perm selector: byte ((r ^ q) & 3) of the source -> address bits 8-15
    uint32_t swap;      // all-ones where bit 2 of r is set
    __device__ __forceinline__ void init(lds_u8* lds) {
        L = lds;
        const uint32_t l = threadIdx.x & 31u, c = l >> 3, r = l & 7u;
        off = (8u * c + r) * 8u;
#pragma unroll
        for (int q = 0; q < 4; ++q) selq[q] = 0x0c0c0000u | ((4u + ((r ^ (uint32_t)q) & 3u)) << 8);
        swap = (r & 4u) ? 0xffffffffu : 0u;
    }
    // Lane r: in = word r of x, out = word r of LPS(x).  Slot s holds the
    // contribution to output word r ^ t(s), t = {0,1,2,3,7,6,5,4}.
    __device__ __forceinline__ void lps(uint32_t& lo, uint32_t& hi) const {
        const uint32_t a = ch3(swap, hi, lo), b = ch3(swap, lo, hi);
        uint32_t ul[8], uh[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const uint32_t ad = __builtin_amdgcn_perm(s < 4 ? a : b, off, selq[s < 4 ? s : 7 - s]);
            const uint64_t v = *reinterpret_cast<lds_u64*>(L + ad);
            ul[s] = (uint32_t)v;
            uh[s] = (uint32_t)(v >> 32);
        }
        uint32_t al[4], ah[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) { al[s] = ul[s] ^ dpp<kHalfMirror>(ul[s + 4]); ah[s] = uh[s] ^ dpp<kHalfMirror>(uh[s + 4]); }
        uint32_t bl[2], bh[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) { bl[s] = al[s] ^ dpp<kXor2>(al[s + 2]); bh[s] = ah[s] ^ dpp<kXor2>(ah[s + 2]); }
        lo = bl[0] ^ dpp<kXor1>(bl[1]);
        hi = bh[0] ^ dpp<kXor1>(bh[1]);
    }
};

struct W64 { uint32_t lo, hi; };
__device__ __forceinline__ W64 wx(W64 a, W64 b) { return W64{a.lo ^ b.lo, a.hi ^ b.hi}; }

// g_N(h, m) on lane r's words (gost3411-2012.h:1110-1144); n = N on lane 0, 0 elsewhere.
__device__ __forceinline__ void g_oct(W64& h, W64 n, W64 m, const Oct& T, const uint64_t* Cw, uint32_t r) {
    W64 k = wx(h, n);
    T.lps(k.lo, k.hi);
    W64 t = wx(k, m);
    T.lps(t.lo, t.hi);
#pragma unroll 1
    for (int q = 0; q < 11; ++q) {
        const uint64_t c = Cw[q * 8 + r];
        k.lo ^= (uint32_t)c; k.hi ^= (uint32_t)(c >> 32);
        T.lps(k.lo, k.hi);
        t = wx(t, k);
        T.lps(t.lo, t.hi);
    }
    const uint64_t c = Cw[11 * 8 + r];
    k.lo ^= (uint32_t)c; k.hi ^= (uint32_t)(c >> 32);
    T.lps(k.lo, k.hi);
    h = wx(h, wx(m, wx(t, k)));
}

__device__ __forceinline__ uint64_t u64(W64 a) { return (uint64_t)a.lo | ((uint64_t)a.hi << 32); }

// Sigma += m mod 2^512 across the 8 lanes (carry-lookahead over the group).
__device__ __forceinline__ void sigma_add(W64& sg, W64 m, uint32_t r) {
    const uint64_t s = u64(sg) + u64(m);
    uint32_t G = s < u64(m), P = s == ~0ull;
#pragma unroll
    for (int d = 1; d < 8; d <<= 1) {
        const uint32_t gs = __shfl_up(G, d, 8), ps = __shfl_up(P, d, 8);
        if (r >= (uint32_t)d) { G |= P & gs; P &= ps; }
    }
    uint32_t cin = __shfl_up(G, 1, 8);
    if (r == 0) cin = 0;
    const uint64_t v = s + cin;
    sg = W64{(uint32_t)v, (uint32_t)(v >> 32)};
}

template <int kThreads>
__global__ __launch_bounds__(kThreads) void k_oct(const uint8_t* data, uint64_t n, uint64_t* out) {
    __shared__ __attribute__((aligned(256))) uint64_t Timg[256 * 32];
    __shared__ uint64_t Cw[12 * 8];
    for (int i = threadIdx.x; i < 96; i += kThreads) Cw[i] = kGostC[i / 8][i % 8];
    gost_stage_rot(Timg);
    Oct T;
    T.init((lds_u8*)Timg);
    const uint64_t g = ((uint64_t)blockIdx.x * kThreads + threadIdx.x) >> 3;
    const uint32_t r = threadIdx.x & 7u;
    if (g >= n) return;   // whole groups of 8 exit together
    const uint64_t* p = reinterpret_cast<const uint64_t*>(data + g * kLen) + r;
    W64 h{0, 0}, sg{0, 0};
    uint64_t n0 = 0;
    uint64_t nx = __builtin_nontemporal_load(p);
    for (uint32_t b = 0; b < kLen / 64; ++b) {
        const W64 m{(uint32_t)nx, (uint32_t)(nx >> 32)};
        if (b + 1 < kLen / 64) nx = __builtin_nontemporal_load(p + 8 * (b + 1));
        g_oct(h, r == 0 ? W64{(uint32_t)n0, (uint32_t)(n0 >> 32)} : W64{0, 0}, m, T, Cw, r);
        n0 += 512;
        sigma_add(sg, m, r);
    }
    // 1024 is a whole number of blocks: the tail block is 0x01 then zeros (rem 0).
    const W64 pad = r == 0 ? W64{1, 0} : W64{0, 0};
    g_oct(h, r == 0 ? W64{(uint32_t)n0, (uint32_t)(n0 >> 32)} : W64{0, 0}, pad, T, Cw, r);
    sigma_add(sg, pad, r);
    g_oct(h, W64{0, 0}, r == 0 ? W64{(uint32_t)n0, (uint32_t)(n0 >> 32)} : W64{0, 0}, T, Cw, r);
    g_oct(h, W64{0, 0}, sg, T, Cw, r);
    out[g * 8 + r] = u64(h);
}

// ------------------------------------------------------------ driver
template <class F>
static float time_best(F launch, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int i = 0; i < reps; ++i) {
        hipEventRecord(a, 0);
        launch();
        hipEventRecord(b, 0);
        if (hipEventSynchronize(b) != hipSuccess || hipGetLastError() != hipSuccess) {
            printf("launch failed\n");
            exit(1);
        }
        float ms;
        hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
    }
    return best;
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 0) : (1ull << 20);
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    std::vector<uint8_t> h(n * kLen);
    uint64_t x = 0x9e3779b97f4a7c15ull;
    for (size_t i = 0; i < h.size(); i += 8) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        memcpy(&h[i], &x, 8);
    }
    uint8_t* d;
    uint64_t *o1, *o2, *o3, *o4;
    hipMalloc(&d, h.size());
    hipMalloc(&o1, n * 64); hipMalloc(&o2, n * 64); hipMalloc(&o3, n * 64); hipMalloc(&o4, n * 64);
    hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice);
    const double gib = (double)(n * kLen) / (1 << 30);
    float t1 = time_best([&] { hipLaunchKernelGGL((k_lane<256, 2>), dim3((n + 255) / 256), dim3(256), 0, 0, d, n, o1); }, reps);
    float t2 = time_best([&] { hipLaunchKernelGGL((k_lane<512, 1>), dim3((n + 511) / 512), dim3(512), 0, 0, d, n, o2); }, reps);
    float t3 = time_best([&] { hipLaunchKernelGGL((k_oct<512>), dim3((n * 8 + 511) / 512), dim3(512), 0, 0, d, n, o3); }, reps);
    float t4 = time_best([&] { hipLaunchKernelGGL((k_oct<1024>), dim3((n * 8 + 1023) / 1024), dim3(1024), 0, 0, d, n, o4); }, reps);
    uint64_t* o5;
    hipMalloc(&o5, n * 64);
    float t5 = time_best([&] { hipLaunchKernelGGL((k_half<1024>), dim3((n + 1023) / 1024), dim3(1024), 0, 0, d, n, o5); }, reps);
    float t6 = time_best([&] { hipLaunchKernelGGL((k_half<512>), dim3((n + 511) / 512), dim3(512), 0, 0, d, n, o5); }, reps);
    float t7 = time_best([&] { hipLaunchKernelGGL((k_half<768>), dim3((n + 767) / 768), dim3(768), 0, 0, d, n, o5); }, reps);

    std::vector<uint64_t> r1(n * 8), r2(n * 8), r3(n * 8), r4(n * 8);
    hipMemcpy(r1.data(), o1, n * 64, hipMemcpyDeviceToHost);
    hipMemcpy(r2.data(), o2, n * 64, hipMemcpyDeviceToHost);
    hipMemcpy(r3.data(), o3, n * 64, hipMemcpyDeviceToHost);
    hipMemcpy(r4.data(), o4, n * 64, hipMemcpyDeviceToHost);
    std::vector<uint64_t> r5(n * 8);
    hipMemcpy(r5.data(), o5, n * 64, hipMemcpyDeviceToHost);
    const bool e2 = r1 == r2, e3 = r1 == r3, e4 = r1 == r4, e5 = r1 == r5;
    printf("GOST-512, %llu messages x 1 KiB (%.3f GiB), best of %d\n", (unsigned long long)n, gib, reps);
    printf("lane  256 thr x 2 WG/CU : %.4f ms  %.3f ms/GiB\n", t1, t1 / gib);
    printf("lane  512 thr           : %.4f ms  %.3f ms/GiB  digests %s\n", t2, t2 / gib, e2 ? "equal" : "DIFFER");
    printf("oct   512 thr           : %.4f ms  %.3f ms/GiB  digests %s\n", t3, t3 / gib, e3 ? "equal" : "DIFFER");
    printf("oct  1024 thr           : %.4f ms  %.3f ms/GiB  digests %s\n", t4, t4 / gib, e4 ? "equal" : "DIFFER");
    printf("half 1024 thr (1 WG/CU) : %.4f ms  %.3f ms/GiB  digests %s\n", t5, t5 / gib, e5 ? "equal" : "DIFFER");
    printf("half  512 thr (1 WG/CU) : %.4f ms  %.3f ms/GiB\n", t6, t6 / gib);
    printf("half  768 thr (1 WG/CU) : %.4f ms  %.3f ms/GiB\n", t7, t7 / gib);
    return (e2 && e3 && e4 && e5) ? 0 : 1;
}
