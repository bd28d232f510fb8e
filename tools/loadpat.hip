// loadpat.hip — HBM read rate of the access patterns a per-lane digest
// kernel can use on 1M x 1 KiB rows (no hashing; XOR-reduce, 16 B out/row).
//  row:   lane = row, 8 x dwordx4 per 128-B line, line by line (current kernels)
//  coal:  fully coalesced stream (lane i reads 16 B at 16*i), same bytes
//  ldsdma: coalesced global_load_lds_dwordx4 of 8 rows x 128 B per wave-instr
//          into a per-wave LDS slab, then each lane reads its own row
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(256) void k_row(const uint4* __restrict__ d, uint4* out, int rows) {
    int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= rows) return;
    const uint4* p = d + (size_t)r * 64;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int line = 0; line < 8; ++line) {
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = p[line * 8 + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) { acc.x ^= v[k].x; acc.y ^= v[k].y; acc.z ^= v[k].z; acc.w ^= v[k].w; }
    }
    out[r] = acc;
}

__global__ __launch_bounds__(256) void k_coal(const uint4* __restrict__ d, uint4* out, size_t n16) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (; i < n16; i += (size_t)gridDim.x * 256) {
        uint4 v = d[i];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// Each wave: 64 rows; per 128-B line index L, 8 LDS-DMA instructions each
// moving 8 rows' line L (1 KiB) into the wave's 8 KiB slab, then lane m reads
// its 128 B (XOR-swizzled 16-B chunks to spread banks).
__global__ __launch_bounds__(256) void k_ldsdma(const uint8_t* __restrict__ d, uint4* out, int rows) {
    __shared__ __attribute__((aligned(16))) uint8_t slab[4][8192];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int row0 = (blockIdx.x * 4 + w) * 64;
    if (row0 >= rows) return;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int L = 0; L < 8; ++L) {
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            const int m = g * 8 + (lane >> 3);            // row within the wave
            const int c = (lane & 7) ^ (m & 7);           // swizzled chunk
            const uint8_t* src = d + (size_t)(row0 + m) * 1024 + L * 128 + c * 16;
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src, (__attribute__((address_space(3))) void*)&slab[w][g * 1024], 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const uint4 v = *reinterpret_cast<const uint4*>(&slab[w][lane * 128 + ((c ^ (lane & 7)) * 16)]);
            acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
        }
        __builtin_amdgcn_wave_barrier();
    }
    out[row0 + lane] = acc;
}

int main() {
    const int rows = 1 << 20;
    const size_t bytes = (size_t)rows * 1024;
    uint8_t* d; uint4* out;
    const int coal_blocks = 2048 * 4;
    const size_t out_n = (size_t)coal_blocks * 256 > (size_t)rows ? (size_t)coal_blocks * 256 : (size_t)rows;
    hipMalloc(&d, bytes); hipMalloc(&out, out_n * 16);  // k_coal writes one uint4 per thread
    hipMemset(d, 1, bytes);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int pass = 0; pass < 3; ++pass) {
        for (int k = 0; k < 3; ++k) {
            float best = 1e9;
            for (int it = 0; it < 60; ++it) {
                hipEventRecord(a, 0);
                if (k == 0) hipLaunchKernelGGL(k_row, dim3(rows / 256), dim3(256), 0, 0, (const uint4*)d, out, rows);
                if (k == 1) hipLaunchKernelGGL(k_coal, dim3(coal_blocks), dim3(256), 0, 0, (const uint4*)d, out, bytes / 16);
                if (k == 2) hipLaunchKernelGGL(k_ldsdma, dim3(rows / 256), dim3(256), 0, 0, (const uint8_t*)d, out, rows);
                hipEventRecord(b, 0);
                if (hipEventSynchronize(b) != hipSuccess || hipGetLastError() != hipSuccess) {
                    printf("kernel %d failed\n", k);
                    return 1;
                }
                float ms; hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
            }
            printf("pass %d %-7s best %.4f ms  %.0f GB/s\n", pass, k == 0 ? "row" : k == 1 ? "coal" : "ldsdma",
                   best, bytes / (best * 1e-3) / 1e9);
        }
    }
    return 0;
}
