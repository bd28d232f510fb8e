// Probe: does global_load_lds_dwordx4 (the LDS-DMA the tile kernel streams
// with) return the right bytes from a byte-unaligned global address on
// gfx950, and at what rate?  If it does at full rate, the tile stream could
// fetch each record from its own first byte (no per-lane rotation, dword
// phase or v_alignbyte; md_tiles.hpp) instead of from its 128-B line.
//   hipcc --offload-arch=gfx950 -O3 -o tools/dma_unaligned tools/dma_unaligned.hip
//   tools/dma_unaligned        (one JSON line per probe)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__host__ __device__ __forceinline__ uint8_t pat(uint64_t i) { return (uint8_t)(i * 7u + (i >> 9) + 3u); }

__global__ void fill_kernel(uint8_t* p, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = pat(i);
}

// Correctness: lane l DMAs 16 B from src + l * 16 + sh into LDS, then copies
// its 16 LDS bytes out.
__global__ __launch_bounds__(64) void dma_check_kernel(const uint8_t* src, uint32_t sh, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[256];
    buf[threadIdx.x * 4] = 0; buf[threadIdx.x * 4 + 1] = 0; buf[threadIdx.x * 4 + 2] = 0; buf[threadIdx.x * 4 + 3] = 0;
    __syncthreads();
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src + threadIdx.x * 16 + sh),
                                     (__attribute__((address_space(3))) void*)buf, 16, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);   // vmcnt(0) lgkmcnt(0)
    __syncthreads();
    for (int k = 0; k < 4; ++k) out[threadIdx.x * 4 + k] = buf[threadIdx.x * 4 + k];
}

// Throughput, the tile kernel's pattern: a wave streams 64 records (ragged
// starts, `gap` bytes apart) of `lines` 128-B lines each; per line, 8 DMA
// instructions, lane group q of instruction g carrying record 8q + g.
//   mode 0: from the record's 128-B line (start & ~127), as today
//   mode 1: from the record's own first byte (start), byte-unaligned
__global__ __launch_bounds__(256) void dma_stream_kernel(const uint8_t* base, uint64_t gap, uint32_t lines,
                                                         uint32_t mode, uint32_t* sink, uint32_t work) {
    __shared__ __attribute__((aligned(16))) uint8_t slab[4][8 * 1040];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + wv;
    uint8_t* s = &slab[wv][0];
    uint64_t src[8];
    for (int g = 0; g < 8; ++g) {
        const uint64_t j = wave * 64 + g + 8 * (lane >> 3);
        const uint64_t st = j * gap + 5;                       // ragged start
        src[g] = (mode ? st : (st & ~127ull)) + (lane & 7) * 16;
    }
    uint32_t acc = 0;
    if (!work) {
        for (uint32_t L = 0; L < lines; ++L) {
#pragma unroll
            for (int g = 0; g < 8; ++g)
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(base + src[g] + L * 128u),
                                                 (__attribute__((address_space(3))) void*)(s + g * 1040), 16, 0, 2);
            __builtin_amdgcn_s_waitcnt(0);
            const uint32_t* r = (const uint32_t*)(s + (lane & 7) * 1040 + (lane >> 3) * 16);
            acc ^= r[0] ^ r[1] ^ r[2] ^ r[3];
        }
        sink[wave * 64 + lane] = acc;
        return;
    }
    // With the tile kernel's compute: take line L (32 words per lane from
    // the slab), issue line L + 1, then two MD5-sized rounds of VALU on it
    // (128 steps, about 5 VALU each) `work` times.
#pragma unroll
    for (int g = 0; g < 8; ++g)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(base + src[g]),
                                         (__attribute__((address_space(3))) void*)(s + g * 1040), 16, 0, 2);
    uint32_t a = lane, b = 1, c = 2, d = 3;
    for (uint32_t L = 0; L < lines; ++L) {
        __builtin_amdgcn_s_waitcnt(0);
        uint32_t w[32];
        const uint8_t* row = s + (lane & 7) * 1040 + (lane >> 3) * 128;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t* q = (const uint32_t*)(row + 16 * k);
            w[4 * k] = q[0]; w[4 * k + 1] = q[1]; w[4 * k + 2] = q[2]; w[4 * k + 3] = q[3];
        }
        __builtin_amdgcn_s_waitcnt(0);
        if (L + 1 < lines) {
#pragma unroll
            for (int g = 0; g < 8; ++g)
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(base + src[g] + (L + 1) * 128u),
                                                 (__attribute__((address_space(3))) void*)(s + g * 1040), 16, 0, 2);
        }
        for (uint32_t rr = 0; rr < work; ++rr)
#pragma unroll
        for (int r = 0; r < 128; ++r) {
            const uint32_t f = (b & c) | (~b & d);
            const uint32_t t = a + f + w[r & 31] + 0x5a827999u * (uint32_t)(r + 1);
            a = d; d = c; c = b;
            b = b + __builtin_rotateleft32(t, (r * 7 + 5) & 31);
        }
    }
    sink[wave * 64 + lane] = a ^ b ^ c ^ d;
}

int main() {
    const uint64_t gap = 1031, lines = 8;
    const uint64_t waves = 16384, recs = waves * 64;
    const uint64_t bytes = recs * gap + 4096;
    uint8_t* d;
    uint32_t *d_out, *d_sink;
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMalloc(&d_out, 64 * 16));
    CHECK(hipMalloc(&d_sink, recs * 4));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, d, bytes);
    CHECK(hipDeviceSynchronize());
    for (uint32_t sh = 0; sh < 16; ++sh) {
        hipLaunchKernelGGL(dma_check_kernel, dim3(1), dim3(64), 0, 0, d + 4096, sh, d_out);
        CHECK(hipDeviceSynchronize());
        uint8_t h[64 * 16];
        CHECK(hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost));
        int bad = 0;
        for (int l = 0; l < 64; ++l) {
            uint8_t e[16];
            for (int k = 0; k < 16; ++k) e[k] = pat(4096 + l * 16 + sh + k);
            if (memcmp(h + l * 16, e, 16)) ++bad;
        }
        printf("{\"probe\": \"dma_check\", \"shift\": %u, \"lanes_wrong\": %d}\n", sh, bad);
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (uint32_t work = 0; work < 4; work += (work ? 2 : 1))
    for (int rep = 0; rep < 3; ++rep)
        for (uint32_t mode = 0; mode < 2; ++mode) {
            hipLaunchKernelGGL(dma_stream_kernel, dim3(waves / 4), dim3(256), 0, 0, d, gap, (uint32_t)lines, mode, d_sink, work);
            CHECK(hipEventRecord(e0, 0));
            for (int it = 0; it < 10; ++it)
                hipLaunchKernelGGL(dma_stream_kernel, dim3(waves / 4), dim3(256), 0, 0, d, gap, (uint32_t)lines, mode, d_sink, work);
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 100.0;   // per launch
            printf("{\"probe\": \"dma_stream\", \"valu_work\": %u, \"mode\": \"%s\", \"rep\": %d, \"us_per_launch\": %.1f, \"GBps_streamed\": %.0f}\n",
                   work, mode ? "record_start_unaligned" : "line_aligned", rep, us, recs * lines * 128.0 / us / 1e3);
        }
    return 0;
}
