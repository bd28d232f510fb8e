// Probe: what do blocks that exit at once cost?  The tile kernel's grid is an
// upper bound (the tile count is known on the device only): its surplus
// one-wave workgroups read the entry count and leave.  Times a kernel of N
// such blocks (no real work), and the same N appended to a kernel whose
// first blocks do some work.
//   hipcc --offload-arch=gfx950 -O3 -o tools/empty_grid tools/empty_grid.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(64) void tiles_like(const uint32_t* ntiles, uint32_t iters, uint32_t* sink) {
    __shared__ uint32_t slab[2048];
    const uint32_t n = ntiles[0];
    if (blockIdx.x >= n) return;
    uint32_t a = threadIdx.x, b = blockIdx.x;
    for (uint32_t i = 0; i < iters; ++i) { a = a * 1664525u + b; b ^= a >> 7; }
    slab[threadIdx.x] = a;
    __syncthreads();
    sink[blockIdx.x * 64 + threadIdx.x] = slab[(threadIdx.x + 1) & 63] ^ b;
}

int main() {
    uint32_t *d_n, *d_sink;
    CHECK(hipMalloc(&d_n, 4));
    CHECK(hipMalloc(&d_sink, (size_t)80000 * 64 * 4));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const uint32_t work[2] = {0u, 17000u};     // live blocks
    for (int w = 0; w < 2; ++w) {
        CHECK(hipMemcpy(d_n, &work[w], 4, hipMemcpyHostToDevice));
        for (uint32_t extra = 0; extra <= 64000; extra += 16000) {
            const uint32_t grid = work[w] + extra;
            if (grid == 0) continue;
            hipLaunchKernelGGL(tiles_like, dim3(grid), dim3(64), 0, 0, d_n, 20000u, d_sink);
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0, 0));
            for (int it = 0; it < 20; ++it)
                hipLaunchKernelGGL(tiles_like, dim3(grid), dim3(64), 0, 0, d_n, 20000u, d_sink);
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            printf("{\"live_blocks\": %u, \"exiting_blocks\": %u, \"us_per_launch\": %.2f}\n", work[w], extra, ms * 50.0);
        }
    }
    return 0;
}
