// gather_rate.hip — random 8-byte table gathers from a 16 KiB table (the
// GOST LPS access pattern): LDS ds_read_b64 vs global loads served by L1 vs a
// mix, to see whether the vector-memory path can take part of the lookups.
// Each lane chases a data-dependent index chain (next index from the loaded
// value), 8 independent chains per lane, like the 8 lookups feeding one
// LPS output word.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int kMode>  // 0: all LDS, 1: all global, 2: 6 LDS + 2 global, 3: 5 LDS + 3 global, 4: 7 LDS + 1 global
__global__ __launch_bounds__(256) void k_gather(const uint64_t* __restrict__ gtab, uint64_t* out, int iters) {
    __shared__ uint64_t T[2048];
    for (int i = threadIdx.x; i < 2048; i += 256) T[i] = gtab[i];
    __syncthreads();
    uint32_t idx[8];
    for (int c = 0; c < 8; ++c) idx[c] = (threadIdx.x * 131 + blockIdx.x * 7 + c * 977) & 255;
    uint64_t acc = 0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const bool glob = (kMode == 1) || (kMode == 2 && c >= 6) || (kMode == 3 && c >= 5) ||
                              (kMode == 4 && c >= 7);
            const uint64_t v = glob ? gtab[c * 256 + idx[c]] : T[c * 256 + idx[c]];
            acc ^= v;
            idx[c] = (uint32_t)(v >> (8 * (it & 7))) & 255;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    uint64_t h[2048];
    uint64_t x = 0x9e3779b97f4a7c15ull;
    for (int i = 0; i < 2048; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = x; }
    uint64_t *gtab, *out;
    const int blocks = 256 * 8;  // 8 blocks/CU of 256 threads (LDS 16 KiB each)
    hipMalloc(&gtab, sizeof(h));
    hipMalloc(&out, (size_t)blocks * 256 * 8);
    hipMemcpy(gtab, h, sizeof(h), hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int iters = 512;
    const char* names[5] = {"lds", "global(L1)", "6 lds+2 glob", "5 lds+3 glob", "7 lds+1 glob"};
    for (int pass = 0; pass < 2; ++pass)
        for (int m = 0; m < 5; ++m) {
            float best = 1e9;
            for (int r = 0; r < 5; ++r) {
                hipEventRecord(a, 0);
                if (m == 0) hipLaunchKernelGGL(k_gather<0>, dim3(blocks), dim3(256), 0, 0, gtab, out, iters);
                if (m == 1) hipLaunchKernelGGL(k_gather<1>, dim3(blocks), dim3(256), 0, 0, gtab, out, iters);
                if (m == 2) hipLaunchKernelGGL(k_gather<2>, dim3(blocks), dim3(256), 0, 0, gtab, out, iters);
                if (m == 3) hipLaunchKernelGGL(k_gather<3>, dim3(blocks), dim3(256), 0, 0, gtab, out, iters);
                if (m == 4) hipLaunchKernelGGL(k_gather<4>, dim3(blocks), dim3(256), 0, 0, gtab, out, iters);
                hipEventRecord(b, 0);
                if (hipEventSynchronize(b) != hipSuccess || hipGetLastError() != hipSuccess) {
                    printf("failed\n");
                    return 1;
                }
                float ms;
                hipEventElapsedTime(&ms, a, b);
                best = ms < best ? ms : best;
            }
            // wave-instructions of 8-byte gathers per CU
            const double wi = (double)blocks * 4 * iters * 8 / 256;
            printf("%-14s %.3f ms  %.2f ns per gather-instr per CU  (%.1f G lookups/s)\n", names[m], best,
                   best * 1e6 / wi, (double)blocks * 256 * iters * 8 / (best * 1e-3) / 1e9);
        }
    return 0;
}
