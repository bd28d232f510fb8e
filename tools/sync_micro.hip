// Probe: what do the pieces of a one-kernel bucketing cost on gfx950?
// (VERDICT r5 item 1 asks for <= 14 us per 1M-packet bucketing; the three
// kernels take 25 us, count 8.2 + base 5.7 + place 11.1.)  Each case is a
// 1,024-thread-block kernel launched 200 times back to back on one stream;
// the period per launch (HIP events) is printed, beside the same grid doing
// nothing.  Cases:
//   empty        the launch itself
//   ticket       thread 0 of every block: one relaxed agent-scope fetch_add
//                on ONE word (the one-kernel form's ticket counter)
//   hist_dense   threads < 488 of every block: a returning relaxed agent
//                fetch_add on word t of a 488-word histogram
//   hist_padded  the same, one histogram word per 128-B line
//   bar_counter  grid barrier: every block adds 1 to one counter and thread 0
//                polls it until it reaches (launch + 1) x grid
//   bar_flags    grid barrier: block b stores the launch's epoch into its own
//                flag line; thread t < grid polls flag t (no shared word)
//   load16       the count kernel's reads: 4 x (8-B offset + 8-B length) per
//                thread, 1M messages, no sync
// A poll gives up after 100 ms (1e7 ticks of the 100 MHz clock): the grid
// is one block per CU and nothing else runs, so a well-formed run never
// gets there; the "valve" count says if one did.
//   hipcc --offload-arch=gfx950 -O3 -o tools/sync_micro tools/sync_micro.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int kKeys = 488;

__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
    return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct Args {
    uint32_t* words;     // counters, histogram, flags
    uint32_t* sink;
    const uint64_t* off;
    const uint64_t* len;
    uint32_t epoch;
    uint32_t n;          // messages (load16)
};

template <int kCase>
__global__ __launch_bounds__(1024) void probe(Args a) {
    __shared__ uint32_t misc[2];
    const uint32_t t = threadIdx.x;
    uint32_t acc = 0;
    if constexpr (kCase == 1) {
        if (t == 0) acc = __hip_atomic_fetch_add(a.words, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if constexpr (kCase == 2 || kCase == 3) {
        const uint32_t stride = kCase == 2 ? 1u : 32u;
        if (t < (uint32_t)kKeys)
            acc = __hip_atomic_fetch_add(a.words + 64 + t * stride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if constexpr (kCase == 4) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) {
            __hip_atomic_fetch_add(a.words + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t target = (a.epoch + 1) * gridDim.x;
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            misc[0] = 0;
            while (ld_agent(a.words + 1) < target) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > 10000000ull) { misc[0] = 1; break; }
            }
            if (misc[0]) __hip_atomic_fetch_add(a.words + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
    } else if constexpr (kCase == 5) {
        uint32_t* flags = a.words + 1024;   // one 128-B line per block
        if (t == 0) st_agent(flags + blockIdx.x * 32, a.epoch + 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool valve = false;
        for (;;) {
            const bool ok = t >= gridDim.x || ld_agent(flags + t * 32) == a.epoch + 1;
            if (__syncthreads_and(ok)) break;
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 10000000ull) { valve = true; break; }
        }
        if (valve && t == 0) __hip_atomic_fetch_add(a.words + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if constexpr (kCase == 6) {
        const uint32_t per = (a.n + gridDim.x - 1) / gridDim.x;
        const uint32_t lo = blockIdx.x * per, hi = lo + per < a.n ? lo + per : a.n;
        for (uint32_t i0 = lo + t; i0 < hi; i0 += 4 * blockDim.x) {
            uint64_t o[4], l[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t i = i0 + u * blockDim.x;
                o[u] = i < hi ? a.off[i] : 0;
                l[u] = i < hi ? a.len[i] : 0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) acc += (uint32_t)(o[u] ^ l[u]);
        }
    }
    if (acc == 0xdeadbeefu) a.sink[blockIdx.x] = acc;   // keep the loads
}

template <int kCase>
static int run(const char* name, Args a, uint32_t grid, hipStream_t s, hipEvent_t e0, hipEvent_t e1, uint32_t* ep) {
    const int iters = 200;
    for (int w = 0; w < 10; ++w) {
        a.epoch = (*ep)++;
        hipLaunchKernelGGL(probe<kCase>, dim3(grid), dim3(1024), 0, s, a);
    }
    CHECK(hipStreamSynchronize(s));
    CHECK(hipEventRecord(e0, s));
    for (int it = 0; it < iters; ++it) {
        a.epoch = (*ep)++;
        hipLaunchKernelGGL(probe<kCase>, dim3(grid), dim3(1024), 0, s, a);
    }
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    uint32_t valve = 0;
    CHECK(hipMemcpy(&valve, a.words + 2, 4, hipMemcpyDeviceToHost));
    printf("{\"case\": \"%s\", \"grid\": %u, \"us_per_launch\": %.2f, \"valve\": %u}\n", name, grid,
           ms * 1000.0 / iters, valve);
    fflush(stdout);
    return 0;
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t n = 1u << 20;
    Args a{};
    CHECK(hipMalloc(&a.words, 1 << 20));
    CHECK(hipMemset(a.words, 0, 1 << 20));
    CHECK(hipMalloc(&a.sink, 1 << 16));
    uint64_t *off, *len;
    CHECK(hipMalloc(&off, (size_t)n * 8));
    CHECK(hipMalloc(&len, (size_t)n * 8));
    CHECK(hipMemset(off, 1, (size_t)n * 8));
    CHECK(hipMemset(len, 2, (size_t)n * 8));
    a.off = off;
    a.len = len;
    a.n = n;
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const uint32_t grids[3] = {64u, 128u, (uint32_t)cus};
    for (int g = 0; g < 3; ++g) {
        const uint32_t grid = grids[g];
        // the barrier cases count epochs from 0 on fresh words
        CHECK(hipMemset(a.words, 0, 1 << 20));
        uint32_t ep = 0;
        if (run<0>("empty", a, grid, s, e0, e1, &ep)) return 1;
        if (run<1>("ticket", a, grid, s, e0, e1, &ep)) return 1;
        if (run<2>("hist_dense", a, grid, s, e0, e1, &ep)) return 1;
        if (run<3>("hist_padded", a, grid, s, e0, e1, &ep)) return 1;
        if (run<6>("load16", a, grid, s, e0, e1, &ep)) return 1;
        CHECK(hipMemset(a.words, 0, 1 << 20));
        ep = 0;
        if (run<4>("bar_counter", a, grid, s, e0, e1, &ep)) return 1;
        CHECK(hipMemset(a.words, 0, 1 << 20));
        ep = 0;
        if (run<5>("bar_flags", a, grid, s, e0, e1, &ep)) return 1;
    }
    return 0;
}
