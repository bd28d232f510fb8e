// queue_bench.cpp — throughput and latency of the asynchronous ingestion queue
// (include/lcb_hash_queue.h) with native producer threads, the way a
// thread pool's packet callbacks would feed it.
//
// Packets: packet i = `size` bytes at pool + i*size, pool = the splitmix64
// stream of SURVEY.md §8d (byte b = byte (b&7) of mix64(seed ^ (b>>3))), so
// the digests are reproducible by oracle/pyoracle.gen_stream.
//
// Output: one JSON line {packets, bytes, seconds, packets_per_s, GiB_s,
// lat_us_p50/p99/max (submit -> callback), queue stats}
// and, with --out FILE, the packed digests (for the oracle comparison).
//
// usage: queue_bench [--alg 1] [--packets 1048576] [--size 1024] [--threads 8]
//                    [--flush-us 200] [--batch-msgs 65536] [--batch-bytes 67108864]
//                    [--slots 4] [--align 16] [--key HEX] [--cb 1] [--pool-mib 0] [--out FILE]
//                    [--rate PACKETS_PER_S] [--zerocopy 1]
//
// --zerocopy: the pool is page-locked (hipHostRegister) and registered with
// the queue (lcb_hash_queue_register); packets are submitted with
// LCB_HASH_Q_F_ZEROCOPY, so the queue records (address, length) and the
// kernel reads them from host memory in place -- no producer memcpy.
//
// --rate: open loop.  Producer t's k-th packet is due at t0 + (k * threads + t)
// / rate (an aggregate rate of `rate`); a producer spins until it is due and the
// latency is counted from the DUE time, so a producer running late (the
// queue pushing back) adds its lateness to the latency instead of hiding it.
// Without --rate the producers submit as fast as they can (saturation: the
// latency then includes the time blocked waiting for a free slot).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include <emmintrin.h>

#include <hip/hip_runtime_api.h>

#include "../include/lcb_hash_gpu.h"
#include "../include/lcb_hash_queue.h"

static uint64_t mix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Ctx {
    std::vector<int64_t>* t_sub;
    std::vector<int64_t>* t_done;
    std::atomic<uint64_t>* errors;
};
static Ctx g_ctx;

// Completion callback (runs on the queue's completion thread); udata is the
// packet index.
static void on_done(void* udata, int error, const uint8_t*, size_t) {
    const uint64_t i = (uint64_t)(uintptr_t)udata;
    (*g_ctx.t_done)[i] = now_ns();
    if (error) g_ctx.errors->fetch_add(1);
}

int main(int argc, char** argv) {
    int alg = 1, threads = 8;
    uint64_t packets = 1 << 20, size = 1024, seed = 0x6C62636861736821ull;
    lcb_hash_queue_settings_t cfg;
    lcb_hash_queue_settings_def(&cfg);
    cfg.max_batch_bytes = 64u << 20;
    std::string keyhex, out;
    bool use_cb = true;
    bool copy_only = false;  // baseline: producers only memcpy into a private arena
    uint64_t pool_mib = 0;  // 0: every packet distinct (cold source); else cycle a pool this big
    double rate = 0;        // packets/s offered (open loop); 0: as fast as possible
    bool zerocopy = false;  // submit from a registered page-locked pool, no copy
    for (int i = 1; i + 1 < argc; i += 2) {
        std::string a = argv[i], v = argv[i + 1];
        if (a == "--alg") alg = atoi(v.c_str());
        else if (a == "--packets") packets = strtoull(v.c_str(), nullptr, 0);
        else if (a == "--size") size = strtoull(v.c_str(), nullptr, 0);
        else if (a == "--threads") threads = atoi(v.c_str());
        else if (a == "--flush-us") cfg.flush_usec = (uint32_t)atoi(v.c_str());
        else if (a == "--batch-msgs") cfg.max_batch_msgs = strtoull(v.c_str(), nullptr, 0);
        else if (a == "--batch-bytes") cfg.max_batch_bytes = strtoull(v.c_str(), nullptr, 0);
        else if (a == "--slots") cfg.batches = (uint32_t)atoi(v.c_str());
        else if (a == "--align") cfg.align = (uint32_t)atoi(v.c_str());
        else if (a == "--key") keyhex = v;
        else if (a == "--out") out = v;
        else if (a == "--cb") use_cb = atoi(v.c_str()) != 0;
        else if (a == "--pool-mib") pool_mib = strtoull(v.c_str(), nullptr, 0);
        else if (a == "--copy-only") copy_only = atoi(v.c_str()) != 0;
        else if (a == "--rate") rate = atof(v.c_str());
        else if (a == "--zerocopy") zerocopy = atoi(v.c_str()) != 0;
        else { fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
    }
    const size_t D = lcb_hash_digest_size(alg);
    if (!D || threads < 1 || threads > 64) { fprintf(stderr, "bad arguments\n"); return 2; }
    std::vector<uint8_t> key;
    for (size_t k = 0; k + 1 < keyhex.size(); k += 2) key.push_back((uint8_t)strtoul(keyhex.substr(k, 2).c_str(), nullptr, 16));

    // Packet pool (the synthetic stream), generated in parallel.
    const uint64_t nbytes = packets * size;
    const uint64_t pool_pk = pool_mib ? std::max<uint64_t>(1, (pool_mib << 20) / size) : packets;
    std::vector<uint8_t> pool(std::min(packets, pool_pk) * size + 8);
    {
        std::vector<std::thread> th;
        const uint64_t words = (pool.size() - 8 + 7) / 8;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t] {
                for (uint64_t w = words * t / threads; w < words * (t + 1) / threads; ++w) {
                    const uint64_t v = mix64(seed ^ w);
                    memcpy(&pool[w * 8], &v, 8);
                }
            });
        for (auto& x : th) x.join();
    }
    if (zerocopy && hipHostRegister(pool.data(), pool.size(), hipHostRegisterDefault) != hipSuccess) {
        fprintf(stderr, "hipHostRegister failed\n");
        return 1;
    }
    const uint32_t sflags = zerocopy ? LCB_HASH_Q_F_ZEROCOPY : 0u;
    auto attach = [&](lcb_hash_queue_p qq) { return zerocopy ? lcb_hash_queue_register(qq, pool.data(), pool.size()) : 0; };
    std::vector<uint8_t> digests(packets * D);
    std::vector<int64_t> t_sub(packets), t_done(packets);
    std::atomic<uint64_t> errors{0};
    g_ctx = Ctx{&t_sub, &t_done, &errors};

    if (copy_only) {
        // Host-side ceiling for the producers: the same loop, memcpy only.
        std::vector<uint8_t> arena(nbytes);
        memset(arena.data(), 0, arena.size());
        const int64_t c0 = now_ns();
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t] {
                const uint64_t lo = packets * t / threads, hi = packets * (t + 1) / threads;
                for (uint64_t i = lo; i < hi; ++i) {
                    t_sub[i] = now_ns();
                    memcpy(&arena[i * size], &pool[(i % pool_pk) * size], size);
                }
            });
        for (auto& x : th) x.join();
        const double sec = (now_ns() - c0) * 1e-9;
        printf("{\"copy_only\": 1, \"packets\": %llu, \"size\": %llu, \"threads\": %d, \"pool_mib\": %llu, "
               "\"seconds\": %.4f, \"packets_per_s\": %.0f, \"GiB_s\": %.3f}\n",
               (unsigned long long)packets, (unsigned long long)size, threads, (unsigned long long)pool_mib, sec,
               packets / sec, nbytes / sec / (1ull << 30));
        return 0;
    }

    lcb_hash_queue_p q = nullptr;
    const uint8_t* kp = key.empty() && keyhex.empty() ? nullptr : key.data();
    int rc = lcb_hash_queue_create(alg, kp, key.size(), &cfg, &q);
    if (!rc) rc = attach(q);
    if (rc) { fprintf(stderr, "create: %s\n", lcb_hash_strerror(rc)); return 1; }

    // Warm-up on a throwaway queue: batches through the whole pipeline (first
    // launches, clocks), so the measured queue's stats hold the run alone.
    {
        std::vector<uint8_t> wd(std::min<uint64_t>(packets, 16384) * D);
        for (uint64_t i = 0; i < wd.size() / D; ++i)
            lcb_hash_queue_submit(q, &pool[(i % pool_pk) * size], size, &wd[i * D], nullptr, nullptr, sflags);
        lcb_hash_queue_wait(q);
        lcb_hash_queue_destroy(q);
        q = nullptr;
        rc = lcb_hash_queue_create(alg, kp, key.size(), &cfg, &q);
        if (!rc) rc = attach(q);
        if (rc) { fprintf(stderr, "create: %s\n", lcb_hash_strerror(rc)); return 1; }
    }
    lcb_hash_queue_stats_t st0;
    lcb_hash_queue_stats(q, &st0);

    std::atomic<int> fail{0};
    // The producers are started first and released together: t0 is taken
    // when every one of them is running (round 5 took it before spawning
    // them, so the last producer's first packets were already late by the
    // threads' start-up -- charged to the queue as latency: worst_at 0.875,
    // the 8th producer's first packet, in every run).
    std::atomic<int> ready{0}, go{0};
    std::atomic<int64_t> t0a{0};
    int64_t t0 = 0;
    {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t] {
                ready.fetch_add(1);
                while (!go.load(std::memory_order_acquire)) _mm_pause();
                const int64_t t0 = t0a.load(std::memory_order_relaxed);
                if (rate > 0) {
                    // contiguous packets per producer (as without --rate); the
                    // k-th packet of producer t is due at (k * threads + t) / rate
                    const double gap = 1e9 / rate;
                    const uint64_t lo = packets * t / threads, hi = packets * (t + 1) / threads;
                    for (uint64_t i = lo; i < hi; ++i) {
                        const int64_t due = t0 + (int64_t)(((i - lo) * threads + t) * gap);
                        while (now_ns() < due) _mm_pause();
                        t_sub[i] = due;
                        int r = lcb_hash_queue_submit(q, &pool[(i % pool_pk) * size], size, &digests[i * D],
                                                      use_cb ? on_done : nullptr, (void*)(uintptr_t)i, sflags);
                        if (r) { fail.store(r); return; }
                    }
                    return;
                }
                const uint64_t lo = packets * t / threads, hi = packets * (t + 1) / threads;
                for (uint64_t i = lo; i < hi; ++i) {
                    t_sub[i] = now_ns();
                    int r = lcb_hash_queue_submit(q, &pool[(i % pool_pk) * size], size, &digests[i * D],
                                                  use_cb ? on_done : nullptr, (void*)(uintptr_t)i, sflags);
                    if (r) { fail.store(r); return; }
                }
            });
        while (ready.load() < threads) _mm_pause();
        t0 = now_ns();
        t0a.store(t0, std::memory_order_relaxed);
        go.store(1, std::memory_order_release);
        for (auto& x : th) x.join();
    }
    rc = lcb_hash_queue_wait(q);
    const int64_t t1 = now_ns();
    lcb_hash_queue_stats_t st;
    lcb_hash_queue_stats(q, &st);
    lcb_hash_queue_destroy(q);
    if (fail.load() || rc || errors.load()) {
        fprintf(stderr, "failed: submit %d wait %d cb-errors %llu\n", fail.load(), rc,
                (unsigned long long)errors.load());
        return 1;
    }
    std::vector<double> lat(packets);
    for (uint64_t i = 0; i < packets; ++i) lat[i] = use_cb ? (t_done[i] - t_sub[i]) * 1e-3 : 0.0;
    // the second half of the run alone (start-up effects excluded)
    std::vector<double> lat2(lat.begin() + packets / 2, lat.end());
    std::sort(lat2.begin(), lat2.end());
    // where the worst packet sits in the run (fraction of the submit order)
    const uint64_t worst = std::max_element(lat.begin(), lat.end()) - lat.begin();
    std::sort(lat.begin(), lat.end());
    const double sec = (t1 - t0) * 1e-9;
    printf("{\"alg\": %d, \"zerocopy\": %d, \"rate\": %.0f, \"lat_us_p999\": %.1f, \"late_half_p99\": %.1f, \"late_half_max\": %.1f, "
           "\"worst_at\": %.4f, \"packets\": %llu, \"size\": %llu, \"threads\": %d, \"flush_usec\": %u, "
           "\"batch_msgs\": %llu, \"batch_bytes\": %llu, \"slots\": %u, \"pool_mib\": %llu, \"seconds\": %.4f, "
           "\"packets_per_s\": %.0f, \"GiB_s\": %.3f, \"lat_us_p50\": %.1f, \"lat_us_p99\": %.1f, "
           "\"lat_us_max\": %.1f, \"batches\": %llu, \"sealed_full\": %llu, \"sealed_timer\": %llu, "
           "\"sealed_flush\": %llu, \"submit_waits\": %llu, \"cb\": %d, \"drain_ms\": %.2f, \"launch_ms\": %.2f, "
           "\"completer_busy_ms\": %.2f, \"gpu_wait_ms\": %.2f, \"max_fill_us\": %.1f, \"max_launch_us\": %.1f, "
           "\"max_gpu_us\": %.1f, \"max_callback_us\": %.1f, \"max_submit_wait_us\": %.1f, "
           "\"max_launch_steps_us\": {\"reopen\": %.1f, \"drain\": %.1f, \"rebase\": %.1f, \"copies\": %.1f, "
           "\"runs\": %.1f, \"kernels\": %.1f, \"event\": %.1f}}\n",
           alg, (int)zerocopy, rate, lat[packets * 999 / 1000], lat2[lat2.size() * 99 / 100], lat2.back(), (double)worst / packets,
           (unsigned long long)packets, (unsigned long long)size, threads, cfg.flush_usec,
           (unsigned long long)cfg.max_batch_msgs, (unsigned long long)cfg.max_batch_bytes, cfg.batches, (unsigned long long)pool_mib, sec,
           packets / sec, nbytes / sec / (1ull << 30), lat[packets / 2], lat[packets * 99 / 100],
           lat[packets - 1], (unsigned long long)(st.batches - st0.batches),
           (unsigned long long)(st.sealed_full - st0.sealed_full),
           (unsigned long long)(st.sealed_timer - st0.sealed_timer),
           (unsigned long long)(st.sealed_flush - st0.sealed_flush),
           (unsigned long long)(st.submit_waits - st0.submit_waits), (int)use_cb,
           (st.flusher_drain_ns - st0.flusher_drain_ns) * 1e-6, (st.flusher_launch_ns - st0.flusher_launch_ns) * 1e-6, (st.completer_busy_ns - st0.completer_busy_ns) * 1e-6,
           (st.gpu_wait_ns - st0.gpu_wait_ns) * 1e-6, st.max_fill_ns * 1e-3, st.max_launch_ns * 1e-3,
           st.max_gpu_ns * 1e-3, st.max_callback_ns * 1e-3, st.max_submit_wait_ns * 1e-3,
           st.max_launch_steps_ns[0] * 1e-3, st.max_launch_steps_ns[1] * 1e-3, st.max_launch_steps_ns[2] * 1e-3,
           st.max_launch_steps_ns[3] * 1e-3, st.max_launch_steps_ns[4] * 1e-3, st.max_launch_steps_ns[5] * 1e-3,
           st.max_launch_steps_ns[6] * 1e-3);
    if (!out.empty()) {
        FILE* f = fopen(out.c_str(), "wb");
        if (!f || fwrite(digests.data(), 1, digests.size(), f) != digests.size()) return 1;
        fclose(f);
    }
    return 0;
}
