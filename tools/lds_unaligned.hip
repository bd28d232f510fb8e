// Probe: do byte-unaligned LDS reads (ds_read_b32 / ds_read_b128) return the
// right bytes on gfx950, and what do they cost?  A lane-varying byte shift of
// the tile kernel's stream (md_tiles.hpp) is one v_alignbyte per word today;
// an unaligned LDS read would move it into the LDS path.
//   hipcc --offload-arch=gfx950 -O3 -o tools/lds_unaligned tools/lds_unaligned.hip
//   tools/lds_unaligned        (prints one JSON line per probe)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__host__ __device__ __forceinline__ uint8_t pat(uint32_t i) { return (uint8_t)(i * 7u + 3u); }

// Every lane reads 16 B at LDS byte (lane * 16 + sh) with ONE ds_read_b128
// and 4 B at (lane * 4 + sh) with ONE ds_read_b32 (inline asm: the compiler
// would split an unaligned access), and writes them out.
__global__ __launch_bounds__(64) void lds_read_kernel(uint32_t sh, uint32_t* out, uint32_t iters, uint64_t* cyc) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[2048];
    for (int i = threadIdx.x; i < 2048; i += 64) buf[i] = pat(i);
    __syncthreads();
    const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)buf;
    uint32_t a16 = base + threadIdx.x * 16 + sh;
    uint32_t a4 = base + threadIdx.x * 4 + sh;
    v4u v;
    uint32_t w;
    asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a16) : "memory");
    asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(a4) : "memory");
    out[threadIdx.x * 5 + 0] = v.x;
    out[threadIdx.x * 5 + 1] = v.y;
    out[threadIdx.x * 5 + 2] = v.z;
    out[threadIdx.x * 5 + 3] = v.w;
    out[threadIdx.x * 5 + 4] = w;
    // Throughput: `iters` rounds of 8 independent ds_read_b128 at this shift.
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    v4u acc = {0, 0, 0, 0};
    for (uint32_t it = 0; it < iters; ++it) {
        v4u r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t a = base + ((threadIdx.x * 16 + k * 1024 + sh) & 1023);
            asm volatile("ds_read_b128 %0, %1" : "=v"(r[k]) : "v"(a) : "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= r[k];
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
    if (acc.x == 0x12345678u) out[0] = acc.y;   // keep the loop
}

int main() {
    uint32_t* d_out;
    uint64_t* d_cyc;
    CHECK(hipMalloc(&d_out, 64 * 5 * 4));
    CHECK(hipMalloc(&d_cyc, 8));
    uint64_t base_cyc = 0;
    for (uint32_t sh = 0; sh < 16; ++sh) {
        hipLaunchKernelGGL(lds_read_kernel, dim3(1), dim3(64), 0, 0, sh, d_out, 2000u, d_cyc);
        CHECK(hipDeviceSynchronize());
        uint32_t h[64 * 5];
        uint64_t cyc;
        CHECK(hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost));
        int bad16 = 0, bad4 = 0;
        for (int l = 0; l < 64; ++l) {
            uint8_t e16[16], e4[4];
            for (int k = 0; k < 16; ++k) e16[k] = pat(l * 16 + sh + k);
            for (int k = 0; k < 4; ++k) e4[k] = pat(l * 4 + sh + k);
            if (l * 16 + sh + 16 <= 2048 && memcmp(&h[l * 5], e16, 16)) ++bad16;
            if (memcmp(&h[l * 5 + 4], e4, 4)) ++bad4;
        }
        if (sh == 0) base_cyc = cyc;
        printf("{\"probe\": \"ds_read\", \"shift\": %u, \"b128_lanes_wrong\": %d, \"b32_lanes_wrong\": %d, "
               "\"b128_x8_loop_memtime\": %llu, \"rel_to_aligned\": %.3f}\n",
               sh, bad16, bad4, (unsigned long long)cyc, base_cyc ? (double)cyc / base_cyc : 1.0);
    }
    return 0;
}
