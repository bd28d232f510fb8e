// H2D copy rate from hipHostMalloc'd memory vs malloc'd memory registered with
// hipHostRegister (the zero-copy queue's receive-buffer case), 64 MiB copies.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
static double rate(void* src, void* dst, size_t n, hipStream_t s) {
    for (int i = 0; i < 3; ++i) (void)hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s);
    (void)hipStreamSynchronize(s);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 20; ++i) (void)hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s);
    (void)hipStreamSynchronize(s);
    double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return 20.0 * n / t / (1 << 30);
}
int main() {
    const size_t n = 64u << 20;
    void *d = nullptr, *h = nullptr;
    hipStream_t s;
    if (hipMalloc(&d, n) != hipSuccess || hipStreamCreate(&s) != hipSuccess) return 1;
    if (hipHostMalloc(&h, n, hipHostMallocDefault) != hipSuccess) return 1;
    memset(h, 1, n);
    printf("{\"hostmalloc_GiB_s\": %.2f", rate(h, d, n, s));
    void* m = aligned_alloc(4096, n);
    memset(m, 1, n);
    if (hipHostRegister(m, n, hipHostRegisterDefault) != hipSuccess) return 1;
    printf(", \"registered_GiB_s\": %.2f", rate(m, d, n, s));
    // 8 runs of 8 MiB each (one batch's producer runs)
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < 20; ++r)
        for (int k = 0; k < 8; ++k)
            (void)hipMemcpyAsync((char*)d + k * (n / 8), (char*)m + k * (n / 8), n / 8, hipMemcpyHostToDevice, s);
    (void)hipStreamSynchronize(s);
    double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf(", \"registered_8runs_GiB_s\": %.2f}\n", 20.0 * n / t / (1 << 30));
    return 0;
}
