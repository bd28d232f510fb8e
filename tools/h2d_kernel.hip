// Probe: host -> device bandwidth of a copy KERNEL reading pinned host memory
// over the link, against hipMemcpyAsync (the copy engine), for the ingestion
// queue's batch sizes (round 7: the queue's gather-copy kernel moved 19-24
// GiB/s against the copy engine's 25-38 in tools/queue_bench).  Sources:
// hipHostMalloc'd memory and malloc'd memory registered with hipHostRegister;
// kernel loads: plain dwordx4, nontemporal, and system-coherent (sc0 sc1);
// 8 loads in flight per thread, grids of 128..1024 blocks of 256 threads.
//   hipcc --offload-arch=gfx950 -O3 -o tools/h2d_kernel tools/h2d_kernel.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int kMode>
__global__ __launch_bounds__(256) void copy_kernel(const uint4* src, uint4* dst, uint64_t n) {
    constexpr int kU = 8;
    const uint64_t step = (uint64_t)gridDim.x * 256;
    for (uint64_t w0 = (uint64_t)blockIdx.x * 256 + threadIdx.x; w0 < n; w0 += step * kU) {
        uint4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint64_t w = w0 + u * step;
            if (w < n) {
                if constexpr (kMode == 0) v[u] = src[w];
                else if constexpr (kMode == 1) {
                    const v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src + w));
                    v[u] = make_uint4(t.x, t.y, t.z, t.w);
                }
                else asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(v[u]) : "v"(src + w) : "memory");
            }
        }
        if constexpr (kMode == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint64_t w = w0 + u * step;
            if (w < n) dst[w] = v[u];
        }
    }
}

int main() {
    const size_t max_bytes = 64u << 20;
    uint8_t* hm = nullptr;
    CHECK(hipHostMalloc(reinterpret_cast<void**>(&hm), max_bytes, hipHostMallocDefault));
    uint8_t* hr = static_cast<uint8_t*>(aligned_alloc(4096, max_bytes));
    memset(hm, 1, max_bytes);
    memset(hr, 2, max_bytes);
    CHECK(hipHostRegister(hr, max_bytes, hipHostRegisterDefault));
    void* hrd = nullptr;
    CHECK(hipHostGetDevicePointer(&hrd, hr, 0));
    void* hmd = nullptr;
    CHECK(hipHostGetDevicePointer(&hmd, hm, 0));
    uint8_t* d = nullptr;
    CHECK(hipMalloc(reinterpret_cast<void**>(&d), max_bytes));
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const size_t sizes[2] = {11u << 20, 64u << 20};
    const char* srcn[2] = {"hostmalloc", "registered"};
    const void* srch[2] = {hm, hr};
    const void* srcd[2] = {hmd, hrd};
    const int reps = 20;
    for (int si = 0; si < 2; ++si) {
        for (int z = 0; z < 2; ++z) {
            const size_t bytes = sizes[z];
            float ms;
            // copy engine
            CHECK(hipMemcpyAsync(d, srch[si], bytes, hipMemcpyHostToDevice, s));
            CHECK(hipStreamSynchronize(s));
            CHECK(hipEventRecord(e0, s));
            for (int r = 0; r < reps; ++r) CHECK(hipMemcpyAsync(d, srch[si], bytes, hipMemcpyHostToDevice, s));
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            printf("{\"src\": \"%s\", \"bytes\": %zu, \"how\": \"hipMemcpyAsync\", \"GiB_s\": %.2f}\n", srcn[si], bytes,
                   bytes * (double)reps / (ms * 1e-3) / (1 << 30));
            fflush(stdout);
            const uint64_t n = bytes / 16;
            for (int mode = 0; mode < 3; ++mode) {
                for (unsigned grid : {128u, 256u, 512u, 1024u}) {
                    auto launch = [&]() {
                        const uint4* sp = static_cast<const uint4*>(srcd[si]);
                        uint4* dp = reinterpret_cast<uint4*>(d);
                        if (mode == 0) hipLaunchKernelGGL(copy_kernel<0>, dim3(grid), dim3(256), 0, s, sp, dp, n);
                        else if (mode == 1) hipLaunchKernelGGL(copy_kernel<1>, dim3(grid), dim3(256), 0, s, sp, dp, n);
                        else hipLaunchKernelGGL(copy_kernel<2>, dim3(grid), dim3(256), 0, s, sp, dp, n);
                    };
                    launch();
                    CHECK(hipStreamSynchronize(s));
                    CHECK(hipEventRecord(e0, s));
                    for (int r = 0; r < reps; ++r) launch();
                    CHECK(hipEventRecord(e1, s));
                    CHECK(hipEventSynchronize(e1));
                    CHECK(hipEventElapsedTime(&ms, e0, e1));
                    static const char* mn[3] = {"plain", "nontemporal", "sc0sc1"};
                    printf("{\"src\": \"%s\", \"bytes\": %zu, \"how\": \"kernel_%s\", \"grid\": %u, \"GiB_s\": %.2f}\n",
                           srcn[si], bytes, mn[mode], grid, bytes * (double)reps / (ms * 1e-3) / (1 << 30));
                    fflush(stdout);
                }
            }
        }
    }
    return 0;
}
