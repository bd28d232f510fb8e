// lcb_hash_multi.cpp — one batch over several MI355X devices
// (include/lcb_hash_gpu.h: lcb_hash_partition, lcb_hash_batch_multi).
//
// every buffer is independent, so a batch shards with no
// data-path collective.  The batch is cut into contiguous message ranges
// balanced by compression work (message bytes + one padding block each) at
// the k/N quantiles of the prefix sum; part p runs on devs[p].
//
//   host mode    one worker thread per part, each running the host pipeline
//                (pinned staging, H2D -> kernel -> D2H) on its device from a
//                pooled staging context; digests land in the caller's array.
//   device mode  the batch lives on devs[0].  Parts on devs[0] hash in place;
//                a part on another device is copied peer-to-peer over xGMI
//                (hipMemcpyPeerAsync: its byte span, and its rebased offsets),
//                hashed there, and its digests are copied back next to the
//                others on devs[0] — the scatter/gather of SURVEY 8(e) as
//                point-to-point DMA on each link, no collective.
#include <errno.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/lcb_hash_gpu.h"
#include "lcb_internal.hpp"

using namespace lcbgpu;

namespace {

// Work of message i: its bytes plus one 64-B block (every message ends in a
// padding compression, so empty messages are not free).
constexpr uint64_t kMsgOverhead = 64;

void partition(const uint32_t* lengths, size_t count, uint32_t fixed_len, size_t nparts, uint64_t* first) {
    first[0] = 0;
    first[nparts] = count;
    if (!lengths) {  // equal work per message: equal counts
        for (size_t p = 1; p < nparts; ++p) first[p] = (uint64_t)((unsigned __int128)count * p / nparts);
        return;
    }
    uint64_t total = 0;
    for (size_t i = 0; i < count; ++i) total += (uint64_t)lengths[i] + kMsgOverhead;
    // first[p] = the first message whose work prefix reaches p/nparts of the total.
    uint64_t acc = 0;
    size_t i = 0;
    for (size_t p = 1; p < nparts; ++p) {
        const uint64_t target = (uint64_t)((unsigned __int128)total * p / nparts);
        while (i < count && acc + ((uint64_t)lengths[i] + kMsgOverhead) / 2 < target) {
            acc += (uint64_t)lengths[i] + kMsgOverhead;
            ++i;
        }
        first[p] = i;
    }
}

struct Part {
    int dev;
    uint64_t lo, hi;
    int rc = 0;
};

int multi_host(const std::vector<Part>& parts_in, int alg, const uint8_t* key, size_t key_len,
               const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths, uint64_t stride,
               uint32_t fixed_len, uint8_t* digests) {
    std::vector<Part> parts = parts_in;
    const size_t D = dsize(alg);
    auto run = [&](Part& p) {
        if (p.hi <= p.lo) return;
        if (hipSetDevice(p.dev) != hipSuccess) { p.rc = ENODEV; return; }
        Stage* st = stage_acquire(p.dev);
        // Without offsets message lo + k starts at data + (lo + k) * stride.
        p.rc = batch_host(alg, key, key_len, offsets ? data : data + p.lo * stride,
                          offsets ? offsets + p.lo : nullptr, lengths ? lengths + p.lo : nullptr,
                          p.hi - p.lo, stride, fixed_len, digests + p.lo * D, nullptr, st);
        stage_release(st);
    };
    if (parts.size() == 1) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        run(parts[0]);
        (void)hipSetDevice(cur);
    } else {
        std::vector<std::thread> th;
        for (Part& p : parts) th.emplace_back(run, std::ref(p));
        for (auto& t : th) t.join();
    }
    for (const Part& p : parts)
        if (p.rc) return p.rc;
    return 0;
}

// ------------------------------------------------ device-mode resources
// Part slots: a persistent non-blocking stream and a growable buffer on one
// device, pooled across calls (r4 created and destroyed a stream and four
// buffers per part per call).  A call holds its slots until every part has
// been waited for, so a slot's buffer is idle whenever it is acquired.
struct PartSlot {
    int dev = -1;
    hipStream_t s = nullptr;
    uint8_t* p = nullptr;
    size_t bytes = 0;
    bool busy = false;
};
std::mutex g_ps_mu;
std::vector<PartSlot*> g_ps;

PartSlot* slot_acquire(int dev) {
    std::lock_guard<std::mutex> lk(g_ps_mu);
    for (PartSlot* x : g_ps)
        if (x->dev == dev && !x->busy) {
            x->busy = true;
            return x;
        }
    PartSlot* x = new PartSlot();
    x->dev = dev;
    if (hipStreamCreateWithFlags(&x->s, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        delete x;
        return nullptr;
    }
    x->busy = true;
    g_ps.push_back(x);
    return x;
}
void slot_release(PartSlot* x) {
    std::lock_guard<std::mutex> lk(g_ps_mu);
    x->busy = false;
}
// The slot's buffer holds `bytes` (current device = the slot's); the slot is
// idle (its last use was waited for), so growing frees at once.
hipError_t slot_reserve(PartSlot* x, size_t bytes) {
    if (x->bytes >= bytes && x->p) return hipSuccess;
    if (x->p) (void)hipFree(x->p);
    x->p = nullptr;
    x->bytes = 0;
    const size_t nb = std::max<size_t>(bytes + bytes / 8, 1u << 20);
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&x->p), nb);
    if (e == hipSuccess) x->bytes = nb;
    return e;
}

// Peer access from `dev` to `home` (both directions of a part's traffic run
// on dev's stream: its copy engine reads the home buffer and writes the
// digests back), enabled once per pair.
std::mutex g_peer_mu;
uint8_t g_peer[64][64];   // 0 unknown, 1 enabled, 2 unavailable
std::atomic<uint64_t> g_st_calls{0}, g_st_remote{0}, g_st_before_wait{0};

void ensure_peer(int dev, int home) {
    if (dev == home) return;
    std::lock_guard<std::mutex> lk(g_peer_mu);
    if (g_peer[dev][home]) return;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, dev, home) != hipSuccess || !can) {
        (void)hipGetLastError();
        g_peer[dev][home] = 2;
        return;
    }
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(dev);
    const hipError_t e = hipDeviceEnablePeerAccess(home, 0);
    (void)hipSetDevice(cur);
    if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) {
        (void)hipGetLastError();
        g_peer[dev][home] = 1;
    } else {
        (void)hipGetLastError();
        g_peer[dev][home] = 2;
    }
}

// Pinned result buffers of the device split (device mode), pooled: a
// hipHostMalloc per call would cost more than the split.
struct SplitHost {
    uint64_t* h = nullptr;          // pinned, coherent: [result words | epoch word]
    uint32_t epoch = 0;
    bool busy = false;
};
std::mutex g_sh_mu;
std::vector<SplitHost*> g_sh;
constexpr size_t kSplitWords = 4 * 64 + 2;   // device result block (+ ticket); host: + epoch word

SplitHost* split_host_acquire() {
    std::lock_guard<std::mutex> lk(g_sh_mu);
    for (SplitHost* x : g_sh)
        if (!x->busy) {
            x->busy = true;
            return x;
        }
    SplitHost* x = new SplitHost();
    if (hipHostMalloc(reinterpret_cast<void**>(&x->h), kSplitWords * 8, hipHostMallocCoherent) != hipSuccess) {
        (void)hipGetLastError();
        delete x;
        return nullptr;
    }
    memset(x->h, 0, kSplitWords * 8);
    x->busy = true;
    g_sh.push_back(x);
    return x;
}
void split_host_release(SplitHost* x) {
    std::lock_guard<std::mutex> lk(g_sh_mu);
    x->busy = false;
}

std::atomic<uint64_t> g_st_host_ns{0}, g_st_split_ns{0}, g_st_splits{0};

inline uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

// `ready`: an event on the home device recorded on the caller's stream at
// entry; every part's stream waits on it before touching the batch, so the
// parts run after the caller's earlier work on its stream (ABI v4).
// A remote part (another device, or every part but the first with
// COPY_PARTS) gets, on its own slot stream and without any host wait: its
// byte span [base[k], end[k]) (from the split: no host pass over the
// messages), its offsets and lengths (peer copies from the home buffers;
// the data pointer is rebased instead of the offsets: a.data = copy - base),
// the batch, and the copy of its digests back.  The host waits for the
// parts only after the last one is enqueued; *t_enq = when that was.
int multi_device(const std::vector<Part>& parts, int alg, const uint8_t* key, size_t key_len,
                 const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths, uint64_t stride,
                 uint32_t fixed_len, uint8_t* digests, const std::vector<uint64_t>& base_of,
                 const std::vector<uint64_t>& end_of, bool copy_all, hipEvent_t ready, uint64_t* t_enq) {
    const size_t D = dsize(alg);
    const int home = parts[0].dev;
    std::vector<PartSlot*> slots(parts.size(), nullptr);
    std::vector<uint64_t> enq_at(parts.size(), 0);
    int rc = 0;
    int cur = 0;
    (void)hipGetDevice(&cur);
    auto fail = [&](hipError_t e) { if (!rc && e != hipSuccess) rc = map_err(e); return e != hipSuccess; };
    uint64_t remote = 0;
    g_st_calls.fetch_add(1, std::memory_order_relaxed);
    for (size_t k = 0; k < parts.size() && !rc; ++k) {
        const Part& p = parts[k];
        if (p.hi <= p.lo) continue;
        const uint64_t n = p.hi - p.lo;
        ensure_peer(p.dev, home);
        if (fail(hipSetDevice(p.dev))) break;
        PartSlot* q = slot_acquire(p.dev);
        if (!q) { rc = ENOMEM; break; }
        slots[k] = q;
        if (fail(hipStreamWaitEvent(q->s, ready, 0))) break;
        if (p.dev == home && !(copy_all && k > 0)) {  // in place on the home device
            rc = batch_device(alg, key, key_len, offsets ? data : data + p.lo * stride,
                              offsets ? offsets + p.lo : nullptr, lengths ? lengths + p.lo : nullptr, n,
                              stride, fixed_len, digests + p.lo * D, q->s, nullptr);
            continue;
        }
        // Remote part: its byte span [base, end) of the home buffer.
        const uint64_t base = base_of[k], end = end_of[k];
        const uint64_t span = end > base ? end - base : 0;
        // Slot buffer: [data span | offsets | lengths | digests], 256-B aligned
        // pieces.  A copy part on the home device itself (COPY_PARTS) reads
        // the offsets and lengths where they are: copying them within one
        // device buys nothing (two enqueues per part less).
        const bool idx_copy = p.dev != home;
        auto up = [](uint64_t x) { return (x + 255) & ~(uint64_t)255; };
        const uint64_t o_data = 0, o_off = up(std::max<uint64_t>(span, 1));
        const uint64_t o_len = o_off + (offsets && idx_copy ? up(n * 8) : 0);
        const uint64_t o_dig = o_len + (lengths && idx_copy ? up(n * 4) : 0);
        if (fail(slot_reserve(q, o_dig + up(n * D)))) break;
        uint8_t* qd = q->p + o_data;
        const uint64_t* qo = offsets ? (idx_copy ? reinterpret_cast<uint64_t*>(q->p + o_off) : offsets + p.lo) : nullptr;
        const uint32_t* ql = lengths ? (idx_copy ? reinterpret_cast<uint32_t*>(q->p + o_len) : lengths + p.lo) : nullptr;
        uint8_t* qg = q->p + o_dig;
        if (span && fail(hipMemcpyPeerAsync(qd, p.dev, data + base, home, span, q->s))) break;
        if (qo && idx_copy &&
            fail(hipMemcpyPeerAsync(const_cast<uint64_t*>(qo), p.dev, offsets + p.lo, home, n * 8, q->s)))
            break;
        if (ql && idx_copy &&
            fail(hipMemcpyPeerAsync(const_cast<uint32_t*>(ql), p.dev, lengths + p.lo, home, n * 4, q->s)))
            break;
        if (offsets) {
            // message i at (qd - base) + offsets[i]: the copy of the span.
            rc = batch_device(alg, key, key_len, qd - base, qo, ql, n, 0, fixed_len, qg, q->s, nullptr);
        } else {
            rc = batch_device(alg, key, key_len, qd, nullptr, ql, n, stride, fixed_len, qg, q->s, nullptr);
        }
        if (!rc && !fail(hipMemcpyPeerAsync(digests + p.lo * D, home, qg, p.dev, n * D, q->s))) {
            ++remote;
            enq_at[k] = now_ns();
        }
    }
    *t_enq = now_ns();
    g_st_remote.fetch_add(remote, std::memory_order_relaxed);
    bool waited = false;
    uint64_t t_wait = 0, before = 0;
    for (size_t k = 0; k < parts.size(); ++k) {
        PartSlot* q = slots[k];
        if (!q) continue;
        (void)hipSetDevice(q->dev);
        if (!waited) {
            // the remote parts whose copies, batch and copy-back were all
            // enqueued before this first wait (their enqueue timestamps)
            t_wait = now_ns();
            waited = true;
            for (size_t j = 0; j < parts.size(); ++j) before += enq_at[j] && enq_at[j] <= t_wait;
        }
        fail(hipStreamSynchronize(q->s));
        slot_release(q);
    }
    if (!rc) g_st_before_wait.fetch_add(before, std::memory_order_relaxed);
    (void)hipSetDevice(cur);
    return rc;
}

}  // namespace

extern "C" {

int lcb_hash_partition(const uint32_t* lengths, size_t count, uint32_t fixed_len, size_t nparts,
                       uint64_t* first) {
    if (nparts == 0 || !first) return EINVAL;
    partition(lengths, count, fixed_len, nparts, first);
    return 0;
}

int lcb_hash_batch_multi(const int* devs, int ndev, int alg, const uint8_t* key, size_t key_len,
                         const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths, size_t count,
                         uint64_t stride, uint32_t fixed_len, uint8_t* digests, uint32_t flags, void* stream) {
    if (!devs || ndev <= 0 || ndev > 64) return EINVAL;
    if (alg < LCB_HASH_MD5 || alg > LCB_HASH_GOST512) return EINVAL;
    if (flags & ~(LCB_HASH_F_DEVICE | LCB_HASH_F_COPY_PARTS)) return EINVAL;
    if ((flags & LCB_HASH_F_COPY_PARTS) && !(flags & LCB_HASH_F_DEVICE)) return EINVAL;
    if (count == 0) return 0;
    if (!data || !digests) return EINVAL;
    if (key == nullptr && key_len != 0) return EINVAL;
    if (int rc = ensure_init()) return rc;
    int ndevices = 0;
    if (hipGetDeviceCount(&ndevices) != hipSuccess) return ENODEV;
    // (ordinals index the 64 x 64 peer table too)
    for (int k = 0; k < ndev; ++k)
        if (devs[k] < 0 || devs[k] >= ndevices || devs[k] >= 64) return ENODEV;
    const bool dev_mode = flags & LCB_HASH_F_DEVICE;
    std::vector<uint64_t> first(ndev + 1);
    if (!dev_mode) {
        partition(lengths, count, fixed_len, (size_t)ndev, first.data());
        std::vector<Part> parts(ndev);
        for (int k = 0; k < ndev; ++k) parts[k] = Part{devs[k], first[k], first[k + 1]};
        return multi_host(parts, alg, key, key_len, data, offsets, lengths, stride, fixed_len, digests);
    }
    // Device mode.  The batch is on devs[0], written by the caller's earlier
    // work on `stream`; an event recorded there gates every part (ABI v4).
    // A ragged batch (or one with offsets) is split on devs[0] by
    // launch_multi_split behind that work -- the split and every part's
    // byte span, a few hundred bytes read back -- instead of copying all
    // offsets and lengths to the host and scanning them there (VERDICT r5
    // item 3: 12 MB and two O(count) host passes for a 1M batch).
    const uint64_t t0 = now_ns();
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (hipSetDevice(devs[0]) != hipSuccess) return ENODEV;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    hipEvent_t ready = nullptr;
    hipError_t e = hipEventCreateWithFlags(&ready, hipEventDisableTiming);
    std::vector<uint64_t> base(ndev, 0), end(ndev, 0);
    const bool split_dev = ndev > 1 && (lengths || offsets);
    SplitHost* sh = nullptr;
    uint64_t split_ns = 0;
    if (e == hipSuccess && split_dev) {
        const uint64_t nb = (count + split_chunk(count) - 1) / split_chunk(count);
        uint64_t* dbuf = nullptr;
        sh = split_host_acquire();
        if (!sh) e = hipErrorOutOfMemory;
        if (e == hipSuccess) e = scratch_alloc(reinterpret_cast<void**>(&dbuf), (nb + kSplitWords) * 8, s);
        if (e == hipSuccess) {
            sh->epoch = (sh->epoch + 1) ? sh->epoch + 1 : 1;
            launch_multi_split(lengths, offsets, stride, fixed_len, count, (uint32_t)ndev, dbuf, dbuf + nb, sh->h,
                               sh->epoch, s);
            e = hipGetLastError();
            (void)scratch_free(dbuf, s);
        }
    }
    if (e == hipSuccess) e = hipEventRecord(ready, s);
    if (e == hipSuccess && split_dev) {
        // The split's last block writes the result and then this call's
        // epoch into the pinned word: spin on it, then poll with short
        // sleeps; a stream that has drained without it is an error.
        const uint32_t* flag = reinterpret_cast<const uint32_t*>(sh->h + 4 * 64 + 1);
        for (uint64_t it = 0;; ++it) {
            if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == sh->epoch) break;
            if (it < 20000) {
                __builtin_ia32_pause();
                continue;
            }
            if ((it & 63) == 0) {
                const hipError_t q = hipEventQuery(ready);
                if (q == hipSuccess && __atomic_load_n(flag, __ATOMIC_ACQUIRE) != sh->epoch) {
                    e = hipErrorUnknown;
                    break;
                }
                if (q != hipSuccess && q != hipErrorNotReady) {
                    e = q;
                    break;
                }
                (void)hipGetLastError();
            }
            std::this_thread::sleep_for(std::chrono::microseconds(5));
        }
        if (e == hipSuccess) {
            for (int k = 0; k <= ndev; ++k) first[k] = sh->h[k];
            for (int k = 0; k < ndev; ++k) {
                base[k] = sh->h[ndev + 1 + k];
                end[k] = sh->h[2 * ndev + 1 + k];
            }
        }
        split_ns = now_ns() - t0;
    }
    if (sh) split_host_release(sh);
    (void)hipSetDevice(cur);
    if (e != hipSuccess) {
        if (ready) (void)hipEventDestroy(ready);
        return map_err(e);
    }
    if (!split_dev) {
        partition(nullptr, count, fixed_len, (size_t)ndev, first.data());   // equal work per message
        for (int k = 0; k < ndev; ++k)
            if (first[k + 1] > first[k] && !offsets) {
                base[k] = first[k] * stride;
                end[k] = (first[k + 1] - 1) * stride + fixed_len;
            }
    }
    std::vector<Part> parts(ndev);
    for (int k = 0; k < ndev; ++k) parts[k] = Part{devs[k], first[k], first[k + 1]};
    uint64_t t_enq = 0;
    const int rc = multi_device(parts, alg, key, key_len, data, offsets, lengths, stride, fixed_len, digests, base,
                                end, flags & LCB_HASH_F_COPY_PARTS, ready, &t_enq);
    (void)hipEventDestroy(ready);   // every part has been synchronised
    g_st_host_ns.fetch_add(t_enq - t0, std::memory_order_relaxed);
    g_st_split_ns.fetch_add(split_ns, std::memory_order_relaxed);
    if (split_dev) g_st_splits.fetch_add(1, std::memory_order_relaxed);
    return rc;
}

int lcb_hash_multi_stats(lcb_hash_multi_stats_t* out) {
    if (!out) return EINVAL;
    memset(out, 0, sizeof(*out));
    out->calls = g_st_calls.load();
    out->remote_parts = g_st_remote.load();
    out->parts_enqueued_before_wait = g_st_before_wait.load();
    out->host_ns = g_st_host_ns.load();
    out->split_ns = g_st_split_ns.load();
    out->device_splits = g_st_splits.load();
    std::lock_guard<std::mutex> lk(g_peer_mu);
    for (int a = 0; a < 64; ++a)
        for (int b = 0; b < 64; ++b) {
            out->peer_enabled += g_peer[a][b] == 1;
            out->peer_unavailable += g_peer[a][b] == 2;
        }
    return 0;
}

}  // extern "C"
