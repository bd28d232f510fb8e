// lcb_hash_queue.cpp — asynchronous packet ingestion (include/lcb_hash_queue.h).
//
// Structure:
//   slots      `batches` staging slots, each a page-locked arena (data,
//              offsets, lengths, digests) + its HBM mirror + a stream/event.
//   open       the slot producers currently append to.
//   leases     a producer thread reserves a LEASE of `lease_msgs` message
//              indices and a run of arena bytes with one CAS on the slot's
//              state word [sealed:1 | count:23 | bytes:40], then fills it
//              packet by packet without writing shared cache lines: per packet
//              it raises/lowers its lease record's `busy` count around the copy
//              (a Dekker handshake with the flusher's seal) and publishes
//              `done` (packets written).  Indices a lease did not fill become
//              holes: zero-length entries that nobody waits for.
//   flusher    seals the open slot (full / flush_usec / flush request),
//              installs a free slot as the new open one at once, then waits
//              for the sealed slot's leases to go idle, turns their unused
//              indices into holes and enqueues H2D -> batch kernel -> D2H.
//   completer  waits for launched slots in order, hands each digest to its
//              submitter (copy to `digest`, then `cb`), returns the slot.
//
// Reference shape being batched: tp_task_pkt_rcvr_handler()
// (src/threadpool/threadpool_task.c:661-725) delivers one io_buf per
// datagram to a callback that hashes it (include/proto/radius.h:776-830);
// completion mirrors tpt_msg_send() (src/threadpool/threadpool_msg_sys.c:279).
#include <errno.h>
#include <execinfo.h>
#include <unistd.h>
#include <pthread.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include <emmintrin.h>
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
constexpr uint32_t kLeaseMsgs = 32;              // message indices per lease
constexpr size_t kLeaseBytes = 32u << 10;        // arena bytes per lease, at least

inline uint64_t st_count(uint64_t s) { return (s >> kCountShift) & kCountMask; }
// h_off entry of a zero-copy packet: this bit | its device address (user
// addresses are far below 2^63); arena packets hold their arena position.
constexpr uint64_t kZeroCopyTag = 1ull << 63;
// Zero-copy runs per batch moved by bulk H2D copies, and the largest gap
// between two packets of one run (bytes copied but never hashed).
constexpr int kZcRuns = 32;
constexpr uint64_t kZcGap = 256;
// LCB_QUEUE_TRACE (read once): 1 logs every stall over 1 ms on stderr (a
// slow launch step, a batch picked up late by the completion thread, the
// flusher waiting for a free slot, a submit waiting for an open slot, a
// batch slower than 1 ms end to end); 2 also starts a watchdog that samples
// the flusher's stack (SIGUSR2, taken for the whole process) while one
// launch's enqueues take over 2 ms.  Diagnostics only.
int trace_level() {
    static const int lv = [] {
        const char* e = getenv("LCB_QUEUE_TRACE");
        return e ? atoi(e) : 0;
    }();
    return lv;
}
inline uint64_t st_bytes(uint64_t s) { return s & kBytesMask; }

struct Meta {
    uint8_t* digest;
    lcb_hash_done_cb cb;
    void* udata;
    uint32_t real;          // 0: hole (index reserved by a lease, never filled)
};

struct alignas(64) LeaseRec {
    // Producers between their seal check and publish.  A COUNTER, not a flag:
    // a producer still holding a lease of an older generation of this slot
    // announces itself here too (then sees the gen mismatch and leaves), and
    // must not clear the announcement of the record's current owner.
    std::atomic<uint32_t> busy{0};
    std::atomic<uint32_t> done{0};   // packets written into this lease
    // Written by the lease's owner before it publishes `done`: the payload
    // bytes of its packets and whether one of them is zero-copy, so the
    // launch sums per lease instead of walking every packet.
    std::atomic<uint64_t> payload{0};
    std::atomic<uint32_t> zc{0};
};

enum SealWhy { kSealFull = 1, kSealTimer = 2, kSealFlush = 3 };

struct Slot {
    alignas(64) std::atomic<uint64_t> state{0};
    alignas(64) std::atomic<uint32_t> gen{0};    // bumped each time the slot reopens
    std::atomic<uint32_t> closed{0};             // read-mostly copy of the seal for lease holders
    std::atomic<int64_t> t_first{0};             // ns timestamp of the first packet; 0 = none
    int64_t t_seal = 0, t_launch = 0;            // flusher: sealed / enqueued (ns)
    uint64_t seq = 0;                            // open order (wait() bookkeeping)
    uint8_t* h_data = nullptr;
    uint64_t* h_off = nullptr;
    uint32_t* h_len = nullptr;
    uint8_t* h_dig = nullptr;
    Meta* meta = nullptr;
    uint8_t* zrun = nullptr;                     // launch: run of each zero-copy packet (kZcRuns = none)
    LeaseRec* leases = nullptr;
    size_t nleases = 0;
    uint8_t* d_data = nullptr;
    uint64_t* d_off = nullptr;
    uint32_t* d_len = nullptr;
    uint32_t* d_work = nullptr;                  // bucketing scratch (launch_ordered)
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    size_t n = 0, bytes = 0, payload = 0, packets = 0;  // final shape of a sealed batch
    int launch_err = 0;
};

// Copy into the staging arena with streaming stores: the arena is only read
// again by the DMA engine, so write-allocating its lines in the producer's
// cache (a read for ownership per line) is wasted memory traffic.  `dst`
// 16-byte aligned; the caller fences (sfence) before publishing.
inline void stream_copy(uint8_t* dst, const uint8_t* src, size_t n) {
    if (n < 256 || (reinterpret_cast<uintptr_t>(dst) & 15)) {
        memcpy(dst, src, n);
        return;
    }
    size_t i = 0;
    for (; i + 64 <= n; i += 64) {
        const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
        const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
        const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
        const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
    }
    if (i < n) memcpy(dst + i, src + i, n - i);
}

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}

void note_max(std::atomic<uint64_t>& m, int64_t v) {
    if (v <= 0) return;
    uint64_t cur = m.load(std::memory_order_relaxed);
    while ((uint64_t)v > cur && !m.compare_exchange_weak(cur, (uint64_t)v, std::memory_order_relaxed)) {}
}

// A producer thread's current lease in one queue.
struct Lease {
    uint64_t qid = 0;           // queue identity (0 = unused entry)
    Slot* slot = nullptr;
    uint32_t gen = 0;
    uint32_t rec = 0;
    uint64_t idx = 0, idx_end = 0;
    uint64_t pos = 0, pos_end = 0;
    bool valid = false;
};
constexpr int kTlsLeases = 8;
thread_local Lease t_leases[kTlsLeases];
std::atomic<uint64_t> g_next_qid{1};

}  // namespace

struct lcb_hash_queue_s {
    int alg = 0;
    size_t D = 0;
    int device = 0;
    uint64_t qid = 0;
    uint32_t lease_msgs = 0;
    size_t lease_bytes = 0;
    lcb_hash_queue_settings_t cfg{};
    std::vector<Slot> slots;
    uint32_t* mid = nullptr;                 // HMAC mid-states (device), or null

    std::atomic<Slot*> open{nullptr};
    std::mutex m;
    std::condition_variable cv_flusher;      // flusher: work may be due
    std::condition_variable cv_open;         // producers: a new open slot
    std::condition_variable cv_complete;     // completer: a slot was launched
    std::condition_variable cv_done;         // waiters: a slot completed
    std::condition_variable cv_free;         // flusher: a slot was returned
    std::deque<Slot*> free_slots, inflight;
    bool stop = false;                       // flusher: drain the open slot and exit
    bool completer_stop = false;             // completer: exit once inflight is empty
    std::atomic<bool> flush_req{false};
    uint64_t next_seq = 1;                   // under m
    std::atomic<uint64_t> completed_seq{0};  // seq of the last completed slot

    std::atomic<uint64_t> completed{0}, completed_bytes{0};
    std::atomic<uint64_t> batches{0}, sealed_full{0}, sealed_timer{0}, sealed_flush{0};
    std::atomic<uint64_t> max_batch{0}, submit_waits{0};
    const int64_t t_create = now_ns();   // trace timestamps are relative to it
    std::atomic<uint64_t> drain_ns{0}, launch_ns{0}, completer_ns{0}, gpu_wait_ns{0};
    std::atomic<uint64_t> max_fill{0}, max_launch{0}, max_gpu{0}, max_cb{0}, max_submit_wait{0};
    std::atomic<uint64_t> max_steps[7] = {};   // the steps of the max_launch batch
    std::atomic<int> first_error{0};

    // Zero-copy packet sources (lcb_hash_queue_register): append-only, read
    // lock-free by submitters once `nregions` covers an entry.
    struct Region {
        const uint8_t* host;
        size_t size;
        uint64_t dev;   // device address of host[0]
    };
    static constexpr int kMaxRegions = 16;
    Region regions[kMaxRegions];
    std::atomic<int> nregions{0};

    std::thread flusher, completer;
    // LCB_QUEUE_TRACE=2: a watchdog samples the flusher's stack while one
    // launch's enqueues take over 2 ms (what a blocking enqueue waits in).
    std::thread watchdog;
    std::atomic<int64_t> enq_t0{0};          // flusher: start of the current launch's enqueues, 0 outside
    std::atomic<bool> watchdog_stop{false};
    pthread_t flusher_tid{};
    void watchdog_main();

    void flusher_main();
    void completer_main();
    void drain_leases(Slot* b);
    void launch(Slot* b, int why, int64_t* steps);
    void release_all();
    void install_open(Slot* b);      // under m
};

namespace {

// Seal `b` (idempotent); returns true if this call sealed it.  The sealed bit
// in `state` stops new leases; `closed` (a line lease holders only read) stops
// packets in existing leases.  Its seq_cst store is the sealer's half of the
// Dekker handshake with `busy` (drain_leases reads `busy` after it).
bool seal(Slot* b) {
    uint64_t s = b->state.load(std::memory_order_seq_cst);
    bool mine = false;
    while (!(s & kSealed))
        if (b->state.compare_exchange_weak(s, s | kSealed, std::memory_order_seq_cst)) { mine = true; break; }
    b->closed.store(1, std::memory_order_seq_cst);
    return mine;
}

}  // namespace

// Reopen a drained slot as a new generation (under m).
void lcb_hash_queue_s::install_open(Slot* b) {
    for (size_t r = 0; r < b->nleases; ++r) {
        b->leases[r].done.store(0, std::memory_order_relaxed);
        b->leases[r].payload.store(0, std::memory_order_relaxed);
        b->leases[r].zc.store(0, std::memory_order_relaxed);
    }
    b->t_first.store(0, std::memory_order_relaxed);
    b->closed.store(0, std::memory_order_relaxed);
    b->n = b->bytes = b->payload = b->packets = 0;
    b->launch_err = 0;
    b->seq = next_seq++;
    b->gen.fetch_add(1, std::memory_order_release);
    b->state.store(0, std::memory_order_release);
    open.store(b, std::memory_order_release);
}

// After the seal: wait until no producer is inside any of the slot's leases,
// then turn every index a lease did not fill into a hole.
void lcb_hash_queue_s::drain_leases(Slot* b) {
    std::atomic_thread_fence(std::memory_order_seq_cst);
    const uint64_t count = st_count(b->state.load(std::memory_order_acquire));
    const uint64_t nrec = (count + lease_msgs - 1) / lease_msgs;
    for (uint64_t r = 0; r < nrec; ++r) {
        LeaseRec& L = b->leases[r];
        while (L.busy.load(std::memory_order_seq_cst) != 0) std::this_thread::yield();
        const uint64_t lo = r * lease_msgs + L.done.load(std::memory_order_acquire);
        const uint64_t hi = std::min<uint64_t>(count, (r + 1) * lease_msgs);
        const uint64_t arena = (uint64_t)reinterpret_cast<uintptr_t>(b->d_data);
        for (uint64_t i = lo; i < hi; ++i) {
            b->h_off[i] = arena;   // an empty message at the arena's start
            b->h_len[i] = 0;
            b->meta[i] = Meta{nullptr, nullptr, nullptr, 0};
        }
    }
}

// Enqueue one sealed, drained slot: H2D, kernel, completion event.
// steps[0..4]: ns spent rebasing, enqueueing the index/length/arena copies,
// the zero-copy run copies, the kernels, the event.
void lcb_hash_queue_s::launch(Slot* b, int why, int64_t* steps) {
    int64_t tt[6];
    tt[0] = now_ns();
    const uint64_t s = b->state.load(std::memory_order_acquire);
    b->n = st_count(s);
    b->bytes = st_bytes(s);
    // Packets, payload and zero-copy presence from the leases' own sums
    // (the launch walked every packet -- up to 64K -- on
    // the flusher's seal-to-launch path).
    size_t payload = 0, packets = 0;
    bool any_zc = false;
    const uint64_t nrec = (b->n + lease_msgs - 1) / lease_msgs;
    for (uint64_t r = 0; r < nrec; ++r) {
        const LeaseRec& L = b->leases[r];
        packets += L.done.load(std::memory_order_acquire);
        payload += L.payload.load(std::memory_order_relaxed);
        any_zc |= L.zc.load(std::memory_order_relaxed) != 0;
    }
    // Copied packets hold their device address in the arena already (the
    // producer wrote it); the arena copy covers the bytes the leases
    // reserved.  Zero-copy packets: every producer submits from its own
    // receive buffers in address order, so a batch's zero-copy packets form
    // a few contiguous RUNS (one per producer stream; gaps up to kZcGap
    // bytes are bridged).  Runs that lie in one registered region and fit
    // the slot's device arena beside the copied packets move with one H2D
    // copy each, at the link's bulk rate, and are hashed from device memory;
    // a packet outside them is read by the kernel where it lies, over the
    // link.  Only a batch with zero-copy packets walks its packets.
    const uint64_t arena = (uint64_t)reinterpret_cast<uintptr_t>(b->d_data);
    struct Run { uint64_t lo, hi; };
    Run run[kZcRuns];
    int nrun = 0, last = -1;
    uint64_t aused = b->bytes;
    uint64_t rpos[kZcRuns];
    const uint8_t* rhost[kZcRuns];
    if (any_zc) {
        aused = 0;
        for (size_t i = 0; i < b->n; ++i) {
            const uint64_t o = b->h_off[i];
            b->zrun[i] = kZcRuns;
            if (!(o & kZeroCopyTag)) {
                aused = std::max<uint64_t>(aused, o - arena + b->h_len[i]);
                continue;
            }
            const uint64_t d = o & ~kZeroCopyTag, e = d + b->h_len[i];
            int r = -1;
            if (last >= 0 && d >= run[last].hi && d <= run[last].hi + kZcGap) r = last;
            for (int k = 0; k < nrun && r < 0; ++k)
                if (d >= run[k].hi && d <= run[k].hi + kZcGap) r = k;
            if (r < 0 && nrun < kZcRuns) { r = nrun++; run[r].lo = d; run[r].hi = d; }
            if (r < 0) continue;                       // too many runs: read in place
            run[r].hi = e;
            b->zrun[i] = (uint8_t)r;
            last = r;
        }
        // Arena position of each run (after the copied packets, 256-B
        // aligned); runs that do not fit or leave every registered region
        // stay in place.
        uint64_t pos = (aused + 255) & ~255ull;
        const int nr = nregions.load(std::memory_order_acquire);
        for (int k = 0; k < nrun; ++k) {
            rhost[k] = nullptr;
            const uint64_t len = run[k].hi - run[k].lo;
            if (pos + len > cfg.max_batch_bytes) continue;
            for (int g = 0; g < nr && !rhost[k]; ++g)
                if (run[k].lo >= regions[g].dev && run[k].hi <= regions[g].dev + regions[g].size)
                    rhost[k] = regions[g].host + (run[k].lo - regions[g].dev);
            if (rhost[k]) { rpos[k] = pos; pos = (pos + len + 255) & ~255ull; }
        }
        for (size_t i = 0; i < b->n; ++i) {
            const uint64_t o = b->h_off[i];
            if (!(o & kZeroCopyTag)) continue;
            const int r = b->zrun[i];
            if (r < kZcRuns && rhost[r]) b->h_off[i] = arena + rpos[r] + ((o & ~kZeroCopyTag) - run[r].lo);
            else b->h_off[i] = o & ~kZeroCopyTag;
        }
    }
    b->payload = payload;
    b->packets = packets;
    hipStream_t st = b->stream;
    KArgs a;
    a.data = nullptr; a.offsets = b->d_off; a.lengths = b->d_len; a.order = nullptr;
    // The batch kernel stores the digests straight into the slot's pinned,
    // coherent host buffer: no device -> host copy command per batch.  (The
    // copy's enqueue blocked the flusher for 8-10 ms once per zero-copy run
    // -- the p99 half-load tail of BENCH_r04 -- LCB_QUEUE_TRACE)
    a.count = b->n; a.stride = 0; a.fixed_len = 0; a.digests = b->h_dig; a.mid = mid;
    int rc = 0;
    tt[1] = now_ns();
    enq_t0.store(tt[1], std::memory_order_release);
    if (hipMemcpyAsync(b->d_off, b->h_off, b->n * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(b->d_len, b->h_len, b->n * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
        (aused && hipMemcpyAsync(b->d_data, b->h_data, aused, hipMemcpyHostToDevice, st) != hipSuccess))
        rc = EIO;
    tt[2] = now_ns();
    for (int k = 0; k < nrun && !rc; ++k)
        if (rhost[k] && run[k].hi > run[k].lo &&
            hipMemcpyAsync(b->d_data + rpos[k], rhost[k], run[k].hi - run[k].lo, hipMemcpyHostToDevice, st) != hipSuccess)
            rc = EIO;
    tt[3] = now_ns();
    if (!rc) rc = launch_ordered(alg, a, st, b->d_work);
    tt[4] = now_ns();
    if (!rc && hipEventRecord(b->done, st) != hipSuccess) rc = EIO;
    tt[5] = now_ns();
    enq_t0.store(0, std::memory_order_release);
    for (int k = 0; k < 5; ++k) steps[k] = tt[k + 1] - tt[k];
    // LCB_QUEUE_TRACE=1: report any launch over 1 ms on stderr as well.
    const bool trace = trace_level() > 0;
    if (trace && tt[5] - tt[0] > 1000000)
        fprintf(stderr, "lcb_hash_queue: slow launch seq=%llu n=%zu runs=%d aused=%llu: rebase %.0f us, "
                "idx/len %.0f us, runs %.0f us, kernel %.0f us, event %.0f us\n", (unsigned long long)b->seq, b->n,
                nrun, (unsigned long long)aused, steps[0] * 1e-3, steps[1] * 1e-3, steps[2] * 1e-3, steps[3] * 1e-3,
                steps[4] * 1e-3);
    b->launch_err = rc;
    b->t_launch = now_ns();
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
                    if (Clock::now() >= due) {
                        why = kSealTimer;
                        break;
                    }
                    cv_flusher.wait_until(lk, due);
                } else {
                    cv_flusher.wait_for(lk, std::chrono::milliseconds(50));
                }
            }
        }
        seal(b);  // no-op when a producer already sealed it as full
        b->t_seal = now_ns();
        // A slot can be sealed full while a lease holder has not published its
        // first packet yet (t_first still 0): no fill time to report then.
        const int64_t t_first = b->t_first.load(std::memory_order_relaxed);
        if (t_first != 0) note_max(max_fill, b->t_seal - t_first);
        flush_req.store(false, std::memory_order_release);
        // Reopen at once when a slot is free (producers then wait only for the
        // install, never for the launch below).  When every other slot is still
        // in flight, launch the sealed slot FIRST: waiting for a free slot
        // before its launch would hold the batch back for a whole GPU round.
        bool reopened = false;
        {
            std::unique_lock<std::mutex> lk(m);
            if (!free_slots.empty()) {
                Slot* next = free_slots.front();
                free_slots.pop_front();
                install_open(next);
                reopened = true;
            }
        }
        if (reopened) cv_open.notify_all();
        const int64_t t_busy = now_ns();
        drain_leases(b);
        const int64_t t_launch = now_ns();
        const bool trace = trace_level() > 0;
        if (trace && (t_launch - t_busy > 1000000 || t_busy - b->t_seal > 1000000))
            fprintf(stderr, "lcb_hash_queue: slow seal -> launch: reopen %.0f us, drain %.0f us\n",
                    (t_busy - b->t_seal) * 1e-3, (t_launch - t_busy) * 1e-3);
        const int64_t t_seal = b->t_seal;
        int64_t steps[7] = {t_busy - t_seal, t_launch - t_busy, 0, 0, 0, 0, 0};
        launch(b, why, steps + 2);   // b may complete and be reused from here on: no access
        const int64_t t_end = now_ns();
        if (t_end - t_seal > (int64_t)max_launch.load(std::memory_order_relaxed)) {
            // (the flusher is the only writer)
            for (int k = 0; k < 7; ++k) max_steps[k].store((uint64_t)steps[k], std::memory_order_relaxed);
            max_launch.store((uint64_t)(t_end - t_seal), std::memory_order_relaxed);
        }
        drain_ns.fetch_add(t_launch - t_busy, std::memory_order_relaxed);
        launch_ns.fetch_add(t_end - t_launch, std::memory_order_relaxed);
        if (!reopened) {
            const int64_t t_fw = now_ns();
            size_t nin = 0;
            {
                std::unique_lock<std::mutex> lk(m);
                nin = inflight.size();
                cv_free.wait(lk, [&] { return !free_slots.empty(); });
                Slot* next = free_slots.front();
                free_slots.pop_front();
                install_open(next);
            }
            cv_open.notify_all();
            if (trace && now_ns() - t_fw > 1000000)
                fprintf(stderr, "lcb_hash_queue: t=%.0f us flusher waited %.0f us for a free slot (%zu in flight)\n",
                        (t_fw - t_create) * 1e-3, (now_ns() - t_fw) * 1e-3, nin);
        }
    }
}

namespace {
void stack_sample_handler(int) {
    void* fr[48];
    const int n = backtrace(fr, 48);
    static const char hdr[] = "lcb_hash_queue: flusher stack while an enqueue blocks:\n";
    (void)!write(2, hdr, sizeof hdr - 1);
    backtrace_symbols_fd(fr, n, 2);
}
}  // namespace

void lcb_hash_queue_s::watchdog_main() {
    void* warm[4];
    (void)backtrace(warm, 4);   // load the unwinder outside the signal handler
    int64_t sampled_t0 = 0;
    int samples = 0;
    while (!watchdog_stop.load(std::memory_order_acquire)) {
        std::this_thread::sleep_for(std::chrono::microseconds(500));
        const int64_t t0 = enq_t0.load(std::memory_order_acquire);
        if (t0 == 0) continue;
        if (t0 != sampled_t0) { sampled_t0 = t0; samples = 0; }
        const int64_t age = now_ns() - t0;
        // up to 3 samples per blocked launch, 2 ms apart, from 2 ms on
        if (samples < 3 && age > 2000000ll * (samples + 1)) {
            fprintf(stderr, "lcb_hash_queue: t=%.0f us launch enqueues blocked %.0f us, sampling the flusher\n",
                    (t0 - t_create) * 1e-3, age * 1e-3);
            pthread_kill(flusher_tid, SIGUSR2);
            ++samples;
        }
    }
}

void lcb_hash_queue_s::completer_main() {
    (void)hipSetDevice(device);
    int64_t prev_end = 0;
    for (;;) {
        Slot* b = nullptr;
        {
            std::unique_lock<std::mutex> lk(m);
            cv_complete.wait(lk, [&] { return !inflight.empty() || completer_stop; });
            if (inflight.empty()) return;
            b = inflight.front();
        }
        const int64_t t_wait = now_ns();
        const bool trace = trace_level() > 0;
        if (trace && t_wait - std::max(prev_end, b->t_launch) > 1000000)
            fprintf(stderr, "lcb_hash_queue: t=%.0f us completer took batch seq=%llu up %.0f us late\n",
                    (t_wait - t_create) * 1e-3, (unsigned long long)b->seq,
                    (t_wait - std::max(prev_end, b->t_launch)) * 1e-3);
        int err = b->launch_err;
        if (!err) err = map_err(hipEventSynchronize(b->done));
        const int64_t t_cb = now_ns();
        gpu_wait_ns.fetch_add(t_cb - t_wait, std::memory_order_relaxed);
        note_max(max_gpu, t_cb - std::max(t_wait, b->t_launch));
        if (trace && t_cb - std::max(t_wait, b->t_launch) > 1000000)
            fprintf(stderr, "lcb_hash_queue: slow batch seq=%llu n=%zu bytes=%zu packets=%zu: launched %.0f us after "
                    "its seal, done %.0f us after launch (completer free %.0f us after launch)\n",
                    (unsigned long long)b->seq, b->n, b->bytes, b->packets, (b->t_launch - b->t_seal) * 1e-3,
                    (t_cb - b->t_launch) * 1e-3, (t_wait - b->t_launch) * 1e-3);
        for (size_t i = 0; i < b->n; ++i) {
            const Meta& mt = b->meta[i];
            if (!mt.real) continue;
            const uint8_t* dg = b->h_dig + i * D;
            if (!err && mt.digest) memcpy(mt.digest, dg, D);
            if (mt.cb) mt.cb(mt.udata, err, err ? nullptr : dg, D);
        }
        if (err) {
            int z = 0;
            first_error.compare_exchange_strong(z, err);
        }
        const int64_t t_end = now_ns();
        completer_ns.fetch_add(t_end - t_cb, std::memory_order_relaxed);
        note_max(max_cb, t_end - t_cb);
        completed.fetch_add(b->packets, std::memory_order_relaxed);
        completed_bytes.fetch_add(b->payload, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> lk(m);
            inflight.pop_front();
            completed_seq.store(b->seq, std::memory_order_release);
            free_slots.push_back(b);
        }
        cv_free.notify_one();
        cv_done.notify_all();
        prev_end = now_ns();
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

int alloc_slot(Slot& b, int alg, size_t msgs, size_t bytes, size_t D, size_t nleases) {
#define Q_TRY(x) do { if ((x) != hipSuccess) return ENOMEM; } while (0)
    Q_TRY(hipStreamCreateWithFlags(&b.stream, hipStreamNonBlocking));
    Q_TRY(hipEventCreateWithFlags(&b.done, hipEventDisableTiming));
    Q_TRY(hipHostMalloc(reinterpret_cast<void**>(&b.h_data), bytes, hipHostMallocDefault));
    Q_TRY(hipHostMalloc(reinterpret_cast<void**>(&b.h_off), msgs * 8, hipHostMallocDefault));
    Q_TRY(hipHostMalloc(reinterpret_cast<void**>(&b.h_len), msgs * 4, hipHostMallocDefault));
    // Fine-grained (coherent): the batch kernels write it over the link.
    Q_TRY(hipHostMalloc(reinterpret_cast<void**>(&b.h_dig), msgs * D, hipHostMallocCoherent));
    Q_TRY(hipMalloc(reinterpret_cast<void**>(&b.d_data), bytes));
    Q_TRY(hipMalloc(reinterpret_cast<void**>(&b.d_off), msgs * 8));
    Q_TRY(hipMalloc(reinterpret_cast<void**>(&b.d_len), msgs * 4));
    Q_TRY(hipMalloc(reinterpret_cast<void**>(&b.d_work), bucket_scratch_words(alg, msgs) * sizeof(uint32_t)));
#undef Q_TRY
    b.meta = new (std::nothrow) Meta[msgs];
    b.zrun = new (std::nothrow) uint8_t[msgs];
    if (!b.zrun) return ENOMEM;
    b.leases = new (std::nothrow) LeaseRec[nleases];
    b.nleases = nleases;
    if (!b.meta || !b.leases) return ENOMEM;
    // Touch every buffer once through the path a batch takes (host arena ->
    // HBM by DMA, digests back): first use of fresh device pages and DMA
    // mappings cost milliseconds, which would otherwise land on the first
    // full-size batches' packets.
    memset(b.h_off, 0, msgs * 8);
    memset(b.h_len, 0, msgs * 4);
    if (hipMemcpyAsync(b.d_data, b.h_data, bytes, hipMemcpyHostToDevice, b.stream) != hipSuccess ||
        hipMemcpyAsync(b.d_off, b.h_off, msgs * 8, hipMemcpyHostToDevice, b.stream) != hipSuccess ||
        hipMemcpyAsync(b.d_len, b.h_len, msgs * 4, hipMemcpyHostToDevice, b.stream) != hipSuccess ||
        hipMemsetAsync(b.d_work, 0, bucket_scratch_words(alg, msgs) * sizeof(uint32_t), b.stream) != hipSuccess ||
        hipStreamSynchronize(b.stream) != hipSuccess)
        return EIO;
    return 0;
}

void free_slot(Slot& b) {
    if (b.h_data) (void)hipHostFree(b.h_data);
    if (b.h_off) (void)hipHostFree(b.h_off);
    if (b.h_len) (void)hipHostFree(b.h_len);
    if (b.h_dig) (void)hipHostFree(b.h_dig);
    if (b.d_data) (void)hipFree(b.d_data);
    if (b.d_off) (void)hipFree(b.d_off);
    if (b.d_len) (void)hipFree(b.d_len);
    if (b.d_work) (void)hipFree(b.d_work);
    if (b.done) (void)hipEventDestroy(b.done);
    if (b.stream) (void)hipStreamDestroy(b.stream);
    delete[] b.meta;
    delete[] b.zrun;
    delete[] b.leases;
    b.h_data = nullptr; b.h_off = nullptr; b.h_len = nullptr; b.h_dig = nullptr; b.meta = nullptr; b.zrun = nullptr;
    b.d_data = nullptr; b.d_off = nullptr; b.d_len = nullptr; b.d_work = nullptr;
    b.done = nullptr; b.stream = nullptr; b.leases = nullptr; b.nleases = 0;
}

// This thread's lease entry for queue `qid` (a free or evicted entry if none).
// Evicting an entry abandons its lease: the unused indices become holes.
Lease& tls_lease(uint64_t qid) {
    Lease* victim = &t_leases[qid % kTlsLeases];
    for (Lease& L : t_leases) {
        if (L.qid == qid) return L;
        if (L.qid == 0) victim = &L;
    }
    *victim = Lease();
    victim->qid = qid;
    return *victim;
}

}  // namespace

void lcb_hash_queue_s::release_all() {
    for (Slot& b : slots) free_slot(b);
    if (mid) {   // the queue's HMAC mid-states are as good as its key: zeroed first
        (void)hipMemset(mid, 0, 2 * kMidWords * sizeof(uint32_t));
        (void)hipDeviceSynchronize();
        (void)hipFree(mid);
    }
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
    q->qid = g_next_qid.fetch_add(1);
    q->lease_msgs = (uint32_t)std::min<size_t>(kLeaseMsgs, cfg.max_batch_msgs);
    q->lease_bytes = std::min<size_t>(kLeaseBytes, cfg.max_batch_bytes);
    if (hipGetDevice(&q->device) != hipSuccess) { delete q; return ENODEV; }
    q->slots = std::vector<Slot>(cfg.batches);
    const size_t nleases = (cfg.max_batch_msgs + q->lease_msgs - 1) / q->lease_msgs;
    int rc = 0;
    for (Slot& b : q->slots)
        if ((rc = alloc_slot(b, alg, cfg.max_batch_msgs, cfg.max_batch_bytes, q->D, nleases))) break;
    if (!rc && key) {
        // HMAC mid-states once per queue (the key is fixed for its lifetime).
        hipStream_t st = q->slots[0].stream;
        const uint32_t* mid = nullptr;
        KeyRef kref;
        rc = hmac_setup(alg, key, key_len, st, &mid, &kref);
        if (!rc) {
            uint32_t* keep = nullptr;
            if (hipMalloc(reinterpret_cast<void**>(&keep), 2 * kMidWords * sizeof(uint32_t)) != hipSuccess ||
                hipMemcpyAsync(keep, mid, 2 * kMidWords * sizeof(uint32_t), hipMemcpyDeviceToDevice, st) !=
                    hipSuccess)
                rc = ENOMEM;
            key_release(kref, st, true);
            if (hipStreamSynchronize(st) != hipSuccess && !rc) rc = EIO;
            q->mid = keep;
        }
    }
    if (!rc) {
        // Empty messages through the batch paths a batch takes: the first
        // launch of a kernel loads its code object (4-5 ms for the first,
        // LCB_QUEUE_TRACE), which would otherwise land on the first batches'
        // packets -- one message (the per-lane kernel), then a bucketed
        // batch (the bucketing and tile kernels: their first launch on a
        // full batch held the flusher 0.9 ms, BENCH r7b max_launch_steps_us
        // "kernels", and the packets of that batch made the p999).
        Slot& b = q->slots[0];
        const uint64_t warm[2] = {1, std::min<uint64_t>(cfg.max_batch_msgs, kBucketMinCount)};
        for (int w = 0; w < 2 && !rc; ++w) {
            const uint64_t n = warm[w];
            if (w == 1 && n < kBucketMinCount) break;
            for (uint64_t i = 0; i < n; ++i) {
                b.h_off[i] = (uint64_t)reinterpret_cast<uintptr_t>(b.d_data);
                b.h_len[i] = 0;
            }
            KArgs a;
            a.data = nullptr; a.offsets = b.d_off; a.lengths = b.d_len; a.order = nullptr;
            a.count = n; a.stride = 0; a.fixed_len = 0; a.digests = b.h_dig; a.mid = q->mid;
            if (hipMemcpyAsync(b.d_off, b.h_off, n * 8, hipMemcpyHostToDevice, b.stream) != hipSuccess ||
                hipMemcpyAsync(b.d_len, b.h_len, n * 4, hipMemcpyHostToDevice, b.stream) != hipSuccess ||
                launch_ordered(alg, a, b.stream, b.d_work) != 0 || hipStreamSynchronize(b.stream) != hipSuccess)
                rc = EIO;
        }
    }
    if (rc) {
        q->release_all();
        delete q;
        return rc;
    }
    for (size_t i = 1; i < q->slots.size(); ++i) q->free_slots.push_back(&q->slots[i]);
    {
        std::lock_guard<std::mutex> lk(q->m);
        q->install_open(&q->slots[0]);
    }
    q->flusher = std::thread([q] { q->flusher_main(); });
    q->completer = std::thread([q] { q->completer_main(); });
    {
        if (trace_level() >= 2) {
            struct sigaction sa {};
            sa.sa_handler = stack_sample_handler;
            sigemptyset(&sa.sa_mask);
            sa.sa_flags = SA_RESTART;
            sigaction(SIGUSR2, &sa, nullptr);
            q->flusher_tid = q->flusher.native_handle();
            q->watchdog = std::thread([q] { q->watchdog_main(); });
        }
    }
    *q_out = q;
    return 0;
}

int lcb_hash_queue_submitv(lcb_hash_queue_p q, const lcb_hash_seg_t* segs, size_t nsegs, uint8_t* digest,
                           lcb_hash_done_cb cb, void* udata, uint32_t flags) {
    if (!q || (nsegs && !segs) || (flags & ~(LCB_HASH_Q_F_NOWAIT | LCB_HASH_Q_F_ZEROCOPY))) return EINVAL;
    size_t len = 0;
    for (size_t k = 0; k < nsegs; ++k) {
        if (segs[k].size && !segs[k].data) return EINVAL;
        len += segs[k].size;
    }
    if (len > UINT32_MAX || len > q->cfg.max_batch_bytes) return EMSGSIZE;
    // Zero copy: the packet's device address in a registered region; it
    // takes a batch index but no staging bytes.
    uint64_t zc = 0;
    if (flags & LCB_HASH_Q_F_ZEROCOPY) {
        if (nsegs != 1) return EINVAL;
        const uint8_t* p = segs[0].data;
        const int nr = q->nregions.load(std::memory_order_acquire);
        for (int r = 0; r < nr && !zc; ++r) {
            const auto& R = q->regions[r];
            if (p >= R.host && (size_t)(p - R.host) <= R.size && len <= R.size - (size_t)(p - R.host))
                zc = kZeroCopyTag | (R.dev + (uint64_t)(p - R.host));
        }
        if (!zc) return EINVAL;
    }
    const size_t clen = zc ? 0 : len;   // staging bytes the packet takes
    const uint64_t A = q->cfg.align;
    const uint64_t cap_m = q->cfg.max_batch_msgs, cap_b = q->cfg.max_batch_bytes, LM = q->lease_msgs;
    Lease& L = tls_lease(q->qid);
    bool waited = false;
    for (;;) {
        if (L.valid) {
            Slot* b = L.slot;
            LeaseRec& r = b->leases[L.rec];
            // Dekker with the flusher: announce, then check the seal.
            r.busy.fetch_add(1, std::memory_order_relaxed);
            std::atomic_thread_fence(std::memory_order_seq_cst);
            const bool live = b->gen.load(std::memory_order_relaxed) == L.gen &&
                              !b->closed.load(std::memory_order_relaxed);
            const uint64_t pos = zc ? L.pos : (L.pos + A - 1) & ~(A - 1);
            if (live && L.idx < L.idx_end && pos + clen <= L.pos_end) {
                if (!zc) {
                    uint8_t* dst = b->h_data + pos;
                    for (size_t k = 0; k < nsegs; ++k) {
                        if (segs[k].size) stream_copy(dst, segs[k].data, segs[k].size);
                        dst += segs[k].size;
                    }
                    _mm_sfence();  // streaming stores before the release of `done`
                }
                const uint64_t i = L.idx;
                // copied packets: their device address in the arena already
                // (no rebase pass at launch)
                b->h_off[i] = zc ? zc : (uint64_t)reinterpret_cast<uintptr_t>(b->d_data) + pos;
                b->h_len[i] = (uint32_t)len;
                b->meta[i] = Meta{digest, cb, udata, 1};
                r.payload.store(r.payload.load(std::memory_order_relaxed) + len, std::memory_order_relaxed);
                if (zc) r.zc.store(1, std::memory_order_relaxed);
                L.idx = i + 1;
                L.pos = pos + clen;
                r.done.store((uint32_t)(L.idx - (uint64_t)L.rec * LM), std::memory_order_release);
                r.busy.fetch_sub(1, std::memory_order_release);
                if (b->t_first.load(std::memory_order_relaxed) == 0) {
                    int64_t z = 0;
                    if (b->t_first.compare_exchange_strong(z, now_ns(), std::memory_order_acq_rel)) {
                        { std::lock_guard<std::mutex> lk(q->m); }
                        q->cv_flusher.notify_one();
                    }
                }
                return 0;
            }
            r.busy.fetch_sub(1, std::memory_order_release);
            L.valid = false;
        }
        // New lease on the open slot: LM indices and room for LM packets of
        // this size (at least kLeaseBytes), shrunk to what the slot has left.
        Slot* b = q->open.load(std::memory_order_acquire);
        const uint32_t g = b->gen.load(std::memory_order_acquire);
        uint64_t s = b->state.load(std::memory_order_acquire);
        bool got = false;
        uint64_t cnt = 0, pos0 = 0, nbytes = 0;
        while (!(s & kSealed)) {
            cnt = st_count(s);
            pos0 = (st_bytes(s) + A - 1) & ~(A - 1);
            const uint64_t room = cap_b > pos0 ? cap_b - pos0 : 0;
            if (cnt + LM > cap_m || room < clen) {  // an empty slot always fits
                if (seal(b)) {
                    { std::lock_guard<std::mutex> lk(q->m); }
                    q->cv_flusher.notify_one();
                }
                break;
            }
            const uint64_t want = std::max<uint64_t>(q->lease_bytes,
                                                     std::min<uint64_t>(LM * (clen + A), cap_b / 8));
            nbytes = std::min<uint64_t>(std::max<uint64_t>(want, clen), room);
            const uint64_t ns = ((cnt + LM) << kCountShift) | (pos0 + nbytes);
            if (b->state.compare_exchange_weak(s, ns, std::memory_order_acq_rel)) {
                got = true;
                break;
            }
        }
        if (got) {
            L.slot = b;
            L.gen = g;
            L.rec = (uint32_t)(cnt / LM);
            L.idx = cnt;
            L.idx_end = cnt + LM;
            L.pos = pos0;
            L.pos_end = pos0 + nbytes;
            L.valid = true;
            continue;
        }
        // Sealed: wait until the flusher installs a new open slot.  The
        // install normally follows the seal within a microsecond or two: spin
        // that long before sleeping on the condition variable (a futex
        // wake-up costs tens of microseconds).
        if (flags & LCB_HASH_Q_F_NOWAIT) {
            if (q->open.load(std::memory_order_acquire) == b) return EAGAIN;
            continue;
        }
        const int64_t t_w = now_ns();
        for (int k = 0; k < 2000 && q->open.load(std::memory_order_acquire) == b; ++k) _mm_pause();
        if (q->open.load(std::memory_order_acquire) != b) continue;
        std::unique_lock<std::mutex> lk(q->m);
        if (q->open.load(std::memory_order_acquire) == b) {
            if (!waited) { q->submit_waits.fetch_add(1, std::memory_order_relaxed); waited = true; }
            q->cv_open.wait(lk, [&] { return q->open.load(std::memory_order_acquire) != b; });
            const int64_t t_ww = now_ns();
            note_max(q->max_submit_wait, t_ww - t_w);
            const bool trace = trace_level() > 0;
            if (trace && t_ww - t_w > 1000000)
                fprintf(stderr, "lcb_hash_queue: t=%.0f us a submit waited %.0f us for an open slot\n",
                        (t_w - q->t_create) * 1e-3, (t_ww - t_w) * 1e-3);
        }
    }
}

int lcb_hash_queue_submit(lcb_hash_queue_p q, const uint8_t* data, size_t size, uint8_t* digest,
                          lcb_hash_done_cb cb, void* udata, uint32_t flags) {
    if (size && !data) return EINVAL;
    lcb_hash_seg_t seg{data, size};
    return lcb_hash_queue_submitv(q, &seg, 1, digest, cb, udata, flags);
}

int lcb_hash_queue_register(lcb_hash_queue_p q, const void* base, size_t size) {
    if (!q || !base || size == 0) return EINVAL;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, base) != hipSuccess) {
        (void)hipGetLastError();
        return EINVAL;   // pageable memory
    }
    if (attr.type != hipMemoryTypeHost || !attr.devicePointer) return EINVAL;
    const void* last = static_cast<const uint8_t*>(base) + size - 1;
    hipPointerAttribute_t al;
    if (hipPointerGetAttributes(&al, last) != hipSuccess || al.type != hipMemoryTypeHost ||
        static_cast<const uint8_t*>(al.devicePointer) != static_cast<const uint8_t*>(attr.devicePointer) + size - 1) {
        (void)hipGetLastError();
        return EINVAL;   // not one page-locked allocation
    }
    std::lock_guard<std::mutex> lk(q->m);
    const int n = q->nregions.load(std::memory_order_relaxed);
    if (n >= lcb_hash_queue_s::kMaxRegions) return ENOMEM;
    q->regions[n] = {static_cast<const uint8_t*>(base), size, (uint64_t)reinterpret_cast<uintptr_t>(attr.devicePointer)};
    q->nregions.store(n + 1, std::memory_order_release);
    return 0;
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
    std::unique_lock<std::mutex> lk(q->m);
    // Every packet whose submit returned lives in the open slot or an older
    // one (slots complete in open order); an empty open slot needs no flush.
    Slot* b = q->open.load(std::memory_order_acquire);
    const bool empty = st_count(b->state.load(std::memory_order_acquire)) == 0;
    const uint64_t target = empty ? b->seq - 1 : b->seq;
    while (q->completed_seq.load(std::memory_order_acquire) < target) {
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
    st->flusher_drain_ns = q->drain_ns.load();
    st->flusher_launch_ns = q->launch_ns.load();
    st->completer_busy_ns = q->completer_ns.load();
    st->gpu_wait_ns = q->gpu_wait_ns.load();
    st->max_fill_ns = q->max_fill.load();
    st->max_launch_ns = q->max_launch.load();
    st->max_gpu_ns = q->max_gpu.load();
    st->max_callback_ns = q->max_cb.load();
    st->max_submit_wait_ns = q->max_submit_wait.load();
    for (int k = 0; k < 7; ++k) st->max_launch_steps_ns[k] = q->max_steps[k].load();
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
    q->watchdog_stop.store(true, std::memory_order_release);
    if (q->watchdog.joinable()) q->watchdog.join();
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
