// lcb_hash_queue.cpp — asynchronous packet ingestion (include/lcb_hash_queue.h).
//
// Structure:
//   slots      `batches` staging slots, each a page-locked arena (data,
//              offsets, lengths, digests) + its HBM mirror + a stream/event.
//   open       the slot producers currently append to.  A producer reserves
//              (count, bytes) with one CAS on the slot's 64-bit state word
//              [sealed:1 | count:23 | bytes:40], copies its packet outside any
//              lock, and leaves; `writers` counts producers between their
//              reservation and the end of their copy.
//   flusher    seals the open slot (full / flush_usec / flush request), waits
//              for writers to drain, installs a free slot as the new open one,
//              and enqueues H2D -> batch kernel -> D2H on the sealed slot's
//              stream.
//   completer  waits for launched slots in order, hands each digest to its
//              submitter (copy to `digest`, then `cb`), returns the slot.
//
// Reference shape being batched: tp_task_pkt_rcvr_handler()
// (src/threadpool/threadpool_task.c:661-725) delivers one io_buf per
// datagram to a callback that hashes it (include/proto/radius.h:776-830);
// completion mirrors tpt_msg_send() (src/threadpool/threadpool_msg_sys.c:279).
#include <errno.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/lcb_hash_gpu.h"
#include "../../include/lcb_hash_queue.h"
#include "lcb_internal.hpp"

using namespace lcbgpu;

namespace {

using Clock = std::chrono::steady_clock;

constexpr uint64_t kSealed = 1ull << 63;
constexpr int kCountShift = 40;
constexpr uint64_t kBytesMask = (1ull << kCountShift) - 1;
constexpr uint64_t kCountMask = (1ull << 23) - 1;
constexpr size_t kMaxMsgs = kCountMask;          // per batch
constexpr size_t kMaxBytes = 1ull << 36;         // per batch (64 GiB)

inline uint64_t st_count(uint64_t s) { return (s >> kCountShift) & kCountMask; }
inline uint64_t st_bytes(uint64_t s) { return s & kBytesMask; }

struct Meta {
    uint8_t* digest;
    lcb_hash_done_cb cb;
    void* udata;
};

enum SealWhy { kSealFull = 1, kSealTimer = 2, kSealFlush = 3 };

struct Slot {
    std::atomic<uint64_t> state{0};
    std::atomic<int> writers{0};
    std::atomic<int64_t> t_first{0};        // ns since clock epoch of packet 0; 0 = empty
    uint8_t* h_data = nullptr;
    uint64_t* h_off = nullptr;
    uint32_t* h_len = nullptr;
    uint8_t* h_dig = nullptr;
    Meta* meta = nullptr;
    uint8_t* d_data = nullptr;
    uint64_t* d_off = nullptr;
    uint32_t* d_len = nullptr;
    uint8_t* d_dig = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    size_t n = 0, bytes = 0, payload = 0;   // final shape of a sealed batch
    int launch_err = 0;
};

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}

}  // namespace

struct lcb_hash_queue_s {
    int alg = 0;
    size_t D = 0;
    int device = 0;
    lcb_hash_queue_settings_t cfg{};
    std::vector<Slot> slots;
    uint32_t* mid = nullptr;                 // HMAC mid-states (device), or null

    std::atomic<Slot*> open{nullptr};
    std::mutex m;
    std::condition_variable cv_flusher;      // flusher: work may be due
    std::condition_variable cv_open;         // producers: a new open slot
    std::condition_variable cv_complete;     // completer: a slot was launched
    std::condition_variable cv_done;         // waiters: packets completed
    std::condition_variable cv_free;         // flusher: a slot was returned
    std::deque<Slot*> free_slots, inflight;
    bool stop = false;                       // flusher: drain the open slot and exit
    bool completer_stop = false;             // completer: exit once inflight is empty
    std::atomic<bool> flush_req{false};

    std::atomic<uint64_t> submitted{0}, completed{0}, completed_bytes{0};
    std::atomic<uint64_t> batches{0}, sealed_full{0}, sealed_timer{0}, sealed_flush{0};
    std::atomic<uint64_t> max_batch{0}, submit_waits{0};
    std::atomic<int> first_error{0};

    std::thread flusher, completer;

    void flusher_main();
    void completer_main();
    void launch(Slot* b, int why);
    void release_all();
};

namespace {

// Seal `b` (idempotent); returns true if this call sealed it.
bool seal(Slot* b) {
    uint64_t s = b->state.load(std::memory_order_acquire);
    while (!(s & kSealed))
        if (b->state.compare_exchange_weak(s, s | kSealed, std::memory_order_acq_rel)) return true;
    return false;
}

// Reopen a drained slot.  `writers` is NOT reset: a producer holding a stale
// pointer to this slot may have incremented it and will decrement it again.
void reset_slot(Slot* b) {
    b->t_first.store(0, std::memory_order_relaxed);
    b->n = b->bytes = b->payload = 0;
    b->launch_err = 0;
    b->state.store(0, std::memory_order_release);
}

}  // namespace

// Enqueue one sealed, writer-free slot: H2D, kernel, D2H, completion event.
void lcb_hash_queue_s::launch(Slot* b, int why) {
    const uint64_t s = b->state.load(std::memory_order_acquire);
    b->n = st_count(s);
    b->bytes = st_bytes(s);
    size_t payload = 0;
    for (size_t i = 0; i < b->n; ++i) payload += b->h_len[i];
    b->payload = payload;
    hipStream_t st = b->stream;
    KArgs a;
    a.data = b->d_data; a.offsets = b->d_off; a.lengths = b->d_len; a.order = nullptr;
    a.count = b->n; a.stride = 0; a.fixed_len = 0; a.digests = b->d_dig; a.mid = mid;
    int rc = 0;
    if (hipMemcpyAsync(b->d_off, b->h_off, b->n * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(b->d_len, b->h_len, b->n * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
        (b->bytes && hipMemcpyAsync(b->d_data, b->h_data, b->bytes, hipMemcpyHostToDevice, st) != hipSuccess))
        rc = EIO;
    if (!rc) rc = launch_ordered(alg, a, st);
    if (!rc && hipMemcpyAsync(b->h_dig, b->d_dig, b->n * D, hipMemcpyDeviceToHost, st) != hipSuccess)
        rc = EIO;
    if (!rc && hipEventRecord(b->done, st) != hipSuccess) rc = EIO;
    b->launch_err = rc;
    batches.fetch_add(1, std::memory_order_relaxed);
    uint64_t mb = max_batch.load(std::memory_order_relaxed);
    while (b->n > mb && !max_batch.compare_exchange_weak(mb, b->n)) {}
    switch (why) {
    case kSealFull: sealed_full.fetch_add(1, std::memory_order_relaxed); break;
    case kSealTimer: sealed_timer.fetch_add(1, std::memory_order_relaxed); break;
    default: sealed_flush.fetch_add(1, std::memory_order_relaxed); break;
    }
    {
        std::lock_guard<std::mutex> lk(m);
        inflight.push_back(b);
    }
    cv_complete.notify_one();
}

void lcb_hash_queue_s::flusher_main() {
    (void)hipSetDevice(device);
    const auto window = std::chrono::microseconds(cfg.flush_usec);
    for (;;) {
        Slot* b = open.load(std::memory_order_acquire);
        int why = 0;
        {
            std::unique_lock<std::mutex> lk(m);
            for (;;) {
                const uint64_t s = b->state.load(std::memory_order_acquire);
                const int64_t t0 = b->t_first.load(std::memory_order_acquire);
                if (s & kSealed) { why = kSealFull; break; }
                if (st_count(s) > 0 && flush_req.load(std::memory_order_acquire)) { why = kSealFlush; break; }
                if (stop) {
                    if (st_count(s) > 0) { why = kSealFlush; break; }
                    return;
                }
                if (st_count(s) == 0) flush_req.store(false, std::memory_order_release);
                if (t0 != 0) {
                    const auto due = Clock::time_point(std::chrono::nanoseconds(t0)) + window;
                    if (Clock::now() >= due) { why = kSealTimer; break; }
                    cv_flusher.wait_until(lk, due);
                } else {
                    cv_flusher.wait_for(lk, std::chrono::milliseconds(50));
                }
            }
        }
        seal(b);  // no-op when a producer already sealed it as full
        flush_req.store(false, std::memory_order_release);
        // Producers that reserved a slot finish their copies.
        while (b->writers.load(std::memory_order_acquire) != 0) std::this_thread::yield();
        launch(b, why);
        // Install the next open slot (waits while every slot is in flight).
        Slot* next = nullptr;
        {
            std::unique_lock<std::mutex> lk(m);
            cv_free.wait(lk, [&] { return !free_slots.empty(); });
            next = free_slots.front();
            free_slots.pop_front();
            reset_slot(next);
            open.store(next, std::memory_order_release);
        }
        cv_open.notify_all();
    }
}

void lcb_hash_queue_s::completer_main() {
    (void)hipSetDevice(device);
    for (;;) {
        Slot* b = nullptr;
        {
            std::unique_lock<std::mutex> lk(m);
            cv_complete.wait(lk, [&] { return !inflight.empty() || completer_stop; });
            if (inflight.empty()) return;
            b = inflight.front();
        }
        int err = b->launch_err;
        if (!err) err = map_err(hipEventSynchronize(b->done));
        for (size_t i = 0; i < b->n; ++i) {
            const Meta& mt = b->meta[i];
            const uint8_t* dg = b->h_dig + i * D;
            if (!err && mt.digest) memcpy(mt.digest, dg, D);
            if (mt.cb) mt.cb(mt.udata, err, err ? nullptr : dg, D);
        }
        if (err) {
            int z = 0;
            first_error.compare_exchange_strong(z, err);
        }
        completed_bytes.fetch_add(b->payload, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> lk(m);
            inflight.pop_front();
            free_slots.push_back(b);
            completed.fetch_add(b->n, std::memory_order_release);
        }
        cv_free.notify_one();
        cv_done.notify_all();
    }
}

namespace {

int validate(const lcb_hash_queue_settings_t& c) {
    if (c.max_batch_msgs == 0 || c.max_batch_msgs > kMaxMsgs) return EINVAL;
    if (c.max_batch_bytes == 0 || c.max_batch_bytes > kMaxBytes) return EINVAL;
    if (c.batches < 2 || c.batches > 16) return EINVAL;
    if (c.align == 0 || c.align > 4096 || (c.align & (c.align - 1))) return EINVAL;
    if (c.flags != 0) return EINVAL;
    return 0;
}

int alloc_slot(Slot& b, size_t msgs, size_t bytes, size_t D) {
#define Q_TRY(x) do { if ((x) != hipSuccess) return ENOMEM; } while (0)
    Q_TRY(hipStreamCreateWithFlags(&b.stream, hipStreamNonBlocking));
    Q_TRY(hipEventCreateWithFlags(&b.done, hipEventDisableTiming));
    Q_TRY(hipHostMalloc(reinterpret_cast<void**>(&b.h_data), bytes, hipHostMallocDefault));
    Q_TRY(hipHostMalloc(reinterpret_cast<void**>(&b.h_off), msgs * 8, hipHostMallocDefault));
    Q_TRY(hipHostMalloc(reinterpret_cast<void**>(&b.h_len), msgs * 4, hipHostMallocDefault));
    Q_TRY(hipHostMalloc(reinterpret_cast<void**>(&b.h_dig), msgs * D, hipHostMallocDefault));
    Q_TRY(hipMalloc(reinterpret_cast<void**>(&b.d_data), bytes));
    Q_TRY(hipMalloc(reinterpret_cast<void**>(&b.d_off), msgs * 8));
    Q_TRY(hipMalloc(reinterpret_cast<void**>(&b.d_len), msgs * 4));
    Q_TRY(hipMalloc(reinterpret_cast<void**>(&b.d_dig), msgs * D));
#undef Q_TRY
    b.meta = new (std::nothrow) Meta[msgs];
    return b.meta ? 0 : ENOMEM;
}

void free_slot(Slot& b) {
    if (b.h_data) (void)hipHostFree(b.h_data);
    if (b.h_off) (void)hipHostFree(b.h_off);
    if (b.h_len) (void)hipHostFree(b.h_len);
    if (b.h_dig) (void)hipHostFree(b.h_dig);
    if (b.d_data) (void)hipFree(b.d_data);
    if (b.d_off) (void)hipFree(b.d_off);
    if (b.d_len) (void)hipFree(b.d_len);
    if (b.d_dig) (void)hipFree(b.d_dig);
    if (b.done) (void)hipEventDestroy(b.done);
    if (b.stream) (void)hipStreamDestroy(b.stream);
    delete[] b.meta;
    b.h_data = nullptr; b.h_off = nullptr; b.h_len = nullptr; b.h_dig = nullptr; b.meta = nullptr;
    b.d_data = nullptr; b.d_off = nullptr; b.d_len = nullptr; b.d_dig = nullptr;
    b.done = nullptr; b.stream = nullptr;
}

}  // namespace

void lcb_hash_queue_s::release_all() {
    for (Slot& b : slots) free_slot(b);
    if (mid) (void)hipFree(mid);
    mid = nullptr;
}

extern "C" {

void lcb_hash_queue_settings_def(lcb_hash_queue_settings_p s) {
    if (!s) return;
    s->max_batch_msgs = 65536;
    s->max_batch_bytes = 16u << 20;
    s->flush_usec = 200;
    s->batches = 4;
    s->align = 16;
    s->flags = 0;
}

int lcb_hash_queue_create(int alg, const uint8_t* key, size_t key_len, const lcb_hash_queue_settings_t* s,
                          lcb_hash_queue_p* q_out) {
    if (!q_out) return EINVAL;
    *q_out = nullptr;
    if (dsize(alg) == 0) return EINVAL;
    if (key == nullptr && key_len != 0) return EINVAL;
    lcb_hash_queue_settings_t cfg;
    lcb_hash_queue_settings_def(&cfg);
    if (s) cfg = *s;
    if (int rc = validate(cfg)) return rc;
    if (int rc = ensure_init()) return rc;

    lcb_hash_queue_s* q = new (std::nothrow) lcb_hash_queue_s();
    if (!q) return ENOMEM;
    q->alg = alg;
    q->D = dsize(alg);
    q->cfg = cfg;
    if (hipGetDevice(&q->device) != hipSuccess) { delete q; return ENODEV; }
    q->slots = std::vector<Slot>(cfg.batches);
    int rc = 0;
    for (Slot& b : q->slots)
        if ((rc = alloc_slot(b, cfg.max_batch_msgs, cfg.max_batch_bytes, q->D))) break;
    if (!rc && key) {
        // HMAC mid-states once per queue (the key is fixed for its lifetime).
        hipStream_t st = q->slots[0].stream;
        uint32_t* mid = nullptr;
        uint8_t* dkey = nullptr;
        rc = hmac_setup(alg, key, key_len, st, &mid, &dkey);
        if (!rc) {
            uint32_t* keep = nullptr;
            if (hipMalloc(reinterpret_cast<void**>(&keep), 2 * kMidWords * sizeof(uint32_t)) != hipSuccess ||
                hipMemcpyAsync(keep, mid, 2 * kMidWords * sizeof(uint32_t), hipMemcpyDeviceToDevice, st) !=
                    hipSuccess)
                rc = ENOMEM;
            (void)hipFreeAsync(mid, st);
            if (dkey) (void)hipFreeAsync(dkey, st);
            if (hipStreamSynchronize(st) != hipSuccess && !rc) rc = EIO;
            q->mid = keep;
        }
    }
    if (rc) {
        q->release_all();
        delete q;
        return rc;
    }
    for (size_t i = 1; i < q->slots.size(); ++i) q->free_slots.push_back(&q->slots[i]);
    reset_slot(&q->slots[0]);
    q->open.store(&q->slots[0], std::memory_order_release);
    q->flusher = std::thread([q] { q->flusher_main(); });
    q->completer = std::thread([q] { q->completer_main(); });
    *q_out = q;
    return 0;
}

int lcb_hash_queue_submitv(lcb_hash_queue_p q, const lcb_hash_seg_t* segs, size_t nsegs, uint8_t* digest,
                           lcb_hash_done_cb cb, void* udata, uint32_t flags) {
    if (!q || (nsegs && !segs) || (flags & ~LCB_HASH_Q_F_NOWAIT)) return EINVAL;
    size_t len = 0;
    for (size_t k = 0; k < nsegs; ++k) {
        if (segs[k].size && !segs[k].data) return EINVAL;
        len += segs[k].size;
    }
    if (len > UINT32_MAX || len > q->cfg.max_batch_bytes) return EMSGSIZE;
    const uint64_t A = q->cfg.align;
    bool waited = false;
    for (;;) {
        Slot* b = q->open.load(std::memory_order_acquire);
        b->writers.fetch_add(1, std::memory_order_acq_rel);
        uint64_t s = b->state.load(std::memory_order_acquire);
        uint64_t idx = 0, pos = 0;
        bool got = false;
        while (!(s & kSealed)) {
            const uint64_t cnt = st_count(s), used = st_bytes(s);
            pos = (used + A - 1) & ~(A - 1);
            if (cnt + 1 > q->cfg.max_batch_msgs || pos + len > q->cfg.max_batch_bytes) {
                if (seal(b)) {
                    { std::lock_guard<std::mutex> lk(q->m); }
                    q->cv_flusher.notify_one();
                }
                break;
            }
            const uint64_t ns = ((cnt + 1) << kCountShift) | (pos + len);
            if (b->state.compare_exchange_weak(s, ns, std::memory_order_acq_rel)) {
                idx = cnt;
                got = true;
                break;
            }
        }
        if (!got) {
            // Sealed: wait until the flusher installs a new open slot.
            b->writers.fetch_sub(1, std::memory_order_release);
            std::unique_lock<std::mutex> lk(q->m);
            if (q->open.load(std::memory_order_acquire) == b) {
                if (flags & LCB_HASH_Q_F_NOWAIT) return EAGAIN;
                if (!waited) { q->submit_waits.fetch_add(1, std::memory_order_relaxed); waited = true; }
                q->cv_open.wait(lk, [&] { return q->open.load(std::memory_order_acquire) != b; });
            }
            continue;
        }
        uint8_t* dst = b->h_data + pos;
        for (size_t k = 0; k < nsegs; ++k) {
            if (segs[k].size) memcpy(dst, segs[k].data, segs[k].size);
            dst += segs[k].size;
        }
        b->h_off[idx] = pos;
        b->h_len[idx] = (uint32_t)len;
        b->meta[idx] = Meta{digest, cb, udata};
        q->submitted.fetch_add(1, std::memory_order_relaxed);
        if (idx == 0) {
            b->t_first.store(now_ns(), std::memory_order_release);
            b->writers.fetch_sub(1, std::memory_order_release);
            { std::lock_guard<std::mutex> lk(q->m); }
            q->cv_flusher.notify_one();
        } else {
            b->writers.fetch_sub(1, std::memory_order_release);
        }
        return 0;
    }
}

int lcb_hash_queue_submit(lcb_hash_queue_p q, const uint8_t* data, size_t size, uint8_t* digest,
                          lcb_hash_done_cb cb, void* udata, uint32_t flags) {
    if (size && !data) return EINVAL;
    lcb_hash_seg_t seg{data, size};
    return lcb_hash_queue_submitv(q, &seg, 1, digest, cb, udata, flags);
}

int lcb_hash_queue_flush(lcb_hash_queue_p q) {
    if (!q) return EINVAL;
    {
        std::lock_guard<std::mutex> lk(q->m);
        q->flush_req.store(true, std::memory_order_release);
    }
    q->cv_flusher.notify_one();
    return 0;
}

int lcb_hash_queue_wait(lcb_hash_queue_p q) {
    if (!q) return EINVAL;
    const uint64_t target = q->submitted.load(std::memory_order_acquire);
    std::unique_lock<std::mutex> lk(q->m);
    while (q->completed.load(std::memory_order_acquire) < target) {
        q->flush_req.store(true, std::memory_order_release);
        q->cv_flusher.notify_one();
        q->cv_done.wait_for(lk, std::chrono::milliseconds(1));
    }
    return q->first_error.load();
}

int lcb_hash_queue_stats(lcb_hash_queue_p q, lcb_hash_queue_stats_t* st) {
    if (!q || !st) return EINVAL;
    st->packets = q->completed.load();
    st->bytes = q->completed_bytes.load();
    st->batches = q->batches.load();
    st->sealed_full = q->sealed_full.load();
    st->sealed_timer = q->sealed_timer.load();
    st->sealed_flush = q->sealed_flush.load();
    st->max_batch_msgs = q->max_batch.load();
    st->submit_waits = q->submit_waits.load();
    return 0;
}

void lcb_hash_queue_destroy(lcb_hash_queue_p q) {
    if (!q) return;
    (void)lcb_hash_queue_wait(q);
    {
        std::lock_guard<std::mutex> lk(q->m);
        q->stop = true;
    }
    q->cv_flusher.notify_all();
    q->flusher.join();
    {
        std::lock_guard<std::mutex> lk(q->m);
        q->completer_stop = true;
    }
    q->cv_complete.notify_all();
    q->completer.join();
    q->release_all();
    delete q;
}

}  // extern "C"
