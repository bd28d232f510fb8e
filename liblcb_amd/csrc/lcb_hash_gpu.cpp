// lcb_hash_gpu.cpp — the exported C-ABI (include/lcb_hash_gpu.h).
//
// Device mode enqueues on the caller's stream and never synchronises (except
// to stage a long HMAC key, see hmac_setup).  Host mode runs a double-buffered
// pipeline on two private streams: H2D -> kernel -> D2H per chunk, chunk c+1's
// upload overlapping chunk c's kernel; page-locked input is DMA'd directly,
// pageable input is gathered into pinned staging by up to 8 host threads.  Every HIP failure maps to an errno code; nothing falls back to the
// CPU.
#include <errno.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <mutex>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/lcb_crc32_gpu.h"
#include "../../include/lcb_hash_gpu.h"
#include "lcb_internal.hpp"

namespace lcbgpu {

size_t dsize(int alg) {
    if (is_crc_alg(alg)) return 4;  // CRC-32: one uint32 per buffer
    static const size_t ds[9] = {0, 16, 20, 28, 32, 48, 64, 32, 64};
    return (alg >= 1 && alg <= 8) ? ds[alg] : 0;
}
size_t bsize(int alg) {
    if (alg < 1 || alg > 8) return 0;
    return (alg == LCB_HASH_SHA384 || alg == LCB_HASH_SHA512) ? 128 : 64;
}

int map_err(hipError_t e) {
    switch (e) {
    case hipSuccess: return 0;
    case hipErrorOutOfMemory: return ENOMEM;
    case hipErrorNoDevice:
    case hipErrorInvalidDevice:
    case hipErrorInsufficientDriver: return ENODEV;
    default: return EIO;
    }
}

#define LCB_TRY(expr)                        \
    do {                                     \
        hipError_t _e = (expr);              \
        if (_e != hipSuccess) return map_err(_e); \
    } while (0)

// ------------------------------------------------------------ scratch pool
namespace {
std::mutex g_scratch_mu;
hipMemPool_t g_scratch[64];
}  // namespace

static hipMemPool_t scratch_pool(int dev) {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    if (g_scratch[dev]) return g_scratch[dev];
    hipMemPoolProps props;
    memset(&props, 0, sizeof(props));
    props.allocType = hipMemAllocationTypePinned;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = dev;
    hipMemPool_t pool = nullptr;
    if (hipMemPoolCreate(&pool, &props) != hipSuccess) return nullptr;
    int off = 0;
    uint64_t keep = UINT64_MAX;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolReuseFollowEventDependencies, &off);
    (void)hipMemPoolSetAttribute(pool, hipMemPoolReuseAllowOpportunistic, &off);
    (void)hipMemPoolSetAttribute(pool, hipMemPoolReuseAllowInternalDependencies, &off);
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    g_scratch[dev] = pool;
    return pool;
}

hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t s) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    hipMemPool_t pool = scratch_pool(dev);
    if (!pool) return hipErrorOutOfMemory;
    return hipMallocFromPoolAsync(p, bytes, pool, s);
}

hipError_t scratch_free(void* p, hipStream_t s) { return hipFreeAsync(p, s); }

// ------------------------------------------------------ per-stream scratch
// Every stream-ordered allocation, free or event record costs ~6.5 us of the
// stream's timeline (the marker packet it enqueues; rocprofv3 traces of the
// 1M-packet pass, profiles/r5_pkt_gaps.txt: 6.6 us of idle before the first
// bucketing kernel with one allocation, 12.2 us with two, 6.2 us after an
// hipEventRecord), i.e. 1-2 % of a packet pass.  Each (device, stream)
// keeps ONE buffer instead, reused by the batches enqueued on that stream:
// the stream's order puts every use after the previous one, so nothing is
// recorded per call.  A call holds the buffer exclusively while it enqueues
// (another thread enqueueing on the same stream at that moment takes the
// pool path).  Streams are told apart by handle: a destroyed stream's object
// is released only once its work has completed, so a later stream that
// reuses the handle finds the buffer idle (hipStreamPerThread names a
// different stream in every thread: it takes the pool path).  Buffers are
// never evicted: past kStreamScratchMax streams, new ones take the pool
// path.  A buffer that grows is retired with an event (the one record) and
// freed once that event has completed.
// Header (kStreamScratchHeader bytes): word 0 = the key-index check's flag
// (the call's epoch when an index is bad), word 1 = the check kernel's
// block counter (monotonic; the host tracks its expected value).
struct StreamScratch {
    int dev = -1;
    hipStream_t sid = nullptr;
    uint8_t* p = nullptr;          // device: [header | payload]
    size_t bytes = 0;              // payload bytes
    uint32_t* hflag = nullptr;     // pinned coherent host word: check result (epoch | bad bit)
    uint32_t epoch = 0;            // last check epoch used on this buffer (< 2^31)
    uint32_t ctr = 0;              // expected value of header word 1
    bool busy = false;
};
constexpr size_t kStreamScratchHeader = 256;
constexpr size_t kStreamScratchMax = 16;

namespace {
std::mutex g_ss_mu;
std::vector<StreamScratch*> g_ss;
std::vector<std::pair<uint8_t*, hipEvent_t>> g_ss_retired;

void ss_reap_locked() {
    for (size_t k = 0; k < g_ss_retired.size();) {
        if (hipEventQuery(g_ss_retired[k].second) == hipSuccess) {
            (void)hipFree(g_ss_retired[k].first);
            (void)hipEventDestroy(g_ss_retired[k].second);
            g_ss_retired.erase(g_ss_retired.begin() + k);
        } else {
            (void)hipGetLastError();
            ++k;
        }
    }
}
}  // namespace

StreamScratch* stream_scratch_acquire(hipStream_t s, size_t bytes) {
    int dev = 0;
    if (s == hipStreamPerThread || hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_ss_mu);
    if (!g_ss_retired.empty()) ss_reap_locked();
    StreamScratch* e = nullptr;
    for (StreamScratch* x : g_ss)
        if (x->dev == dev && x->sid == s) { e = x; break; }
    if (e && e->busy) return nullptr;   // another thread is enqueueing on this stream
    if (!e) {
        if (g_ss.size() >= kStreamScratchMax) return nullptr;
        e = new StreamScratch();
        if (hipHostMalloc(reinterpret_cast<void**>(&e->hflag), 64, hipHostMallocCoherent) != hipSuccess) {
            (void)hipGetLastError();
            delete e;
            return nullptr;
        }
        *e->hflag = 0;
        e->dev = dev;
        e->sid = s;
        g_ss.push_back(e);
    }
    if (e->bytes < bytes || !e->p) {
        // Grow (to 1.25x, so a slowly growing batch does not reallocate every
        // call); the old buffer is freed once the work enqueued so far is done.
        if (e->p) {
            hipEvent_t ev = nullptr;
            if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
                hipEventRecord(ev, s) != hipSuccess) {
                (void)hipGetLastError();
                if (ev) (void)hipEventDestroy(ev);
                return nullptr;
            }
            g_ss_retired.emplace_back(e->p, ev);
            e->p = nullptr;
            e->bytes = 0;
        }
        const size_t nb = std::max<size_t>(bytes + bytes / 4, 1u << 20);
        if (hipMalloc(reinterpret_cast<void**>(&e->p), nb + kStreamScratchHeader) != hipSuccess) {
            (void)hipGetLastError();
            e->p = nullptr;
            return nullptr;
        }
        // Header zeroed in stream order: flag 0 (epochs start at 1), counter
        // 0; and the bucketing head of the payload (the one-kernel
        // bucketing's sync words start at zero and stay so between uses).
        if (hipMemsetAsync(e->p, 0, kStreamScratchHeader + kBucketWork * sizeof(uint32_t), s) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipFree(e->p);
            e->p = nullptr;
            return nullptr;
        }
        e->bytes = nb;
        e->ctr = 0;
    }
    e->busy = true;
    return e;
}

uint8_t* stream_scratch_payload(StreamScratch* e) { return e->p + kStreamScratchHeader; }

void stream_scratch_release(StreamScratch* e) {
    if (!e) return;
    std::lock_guard<std::mutex> lk(g_ss_mu);
    e->busy = false;
}

// ------------------------------------------------------------- key cache
// Key tables of keyed batches (lcb_hash_batch_keyed) and single HMAC keys
// (lcb_hash_batch with a key), uploaded and prepared (mid-states) once per
// device and reused while the same keys come back: a RADIUS server signs
// every batch with the same table of peer secrets (radius_client.c:242,886,
// 1025), and the upload (three pageable copies) plus the prep kernel cost
// ~30 us of stream time per call (r5 trace).  Entries are looked up by their
// exact bytes; an entry is immutable once prepared; a stream other than the
// one that prepared it waits on its `ready` event.
//
// The cache holds secrets (the key bytes on the host and the device, and the
// ipad/opad mid-states, which are as good as the key), so:
//  * at most kKeyCacheMax entries, least recently used evicted first;
//  * an evicted or flushed entry's device buffer is zeroed in stream order
//    after every use of it before it returns to the pool, and its host copy
//    is zeroed (md5.h:337,358 zeroise the reference's pads the same way);
//  * lcb_hash_key_cache_flush() drops every entry; LCB_HASH_KEY_CACHE=0
//    turns the cache off (every call uploads its keys to a per-call buffer,
//    zeroed before it is freed).
// An entry is pinned while a call holds it (from the lookup until its batch
// is enqueued, KeyRef); device-mode calls note the stream they used: an
// entry only ever used on the evicting call's stream is zeroed in that
// stream's order, any other after a device synchronisation.
struct KeyCacheEntry {
    int dev = -1;
    int alg = 0;
    int kind = 0;                    // LCB_HASH_KEY_* of a table, or 0: one HMAC key
    std::vector<uint8_t> sig;        // key bytes + lengths (the lookup key)
    uint8_t* dbuf = nullptr;         // [pad | key bytes | key offsets | key lengths | mid-states]
    size_t dbytes = 0;
    KeyTable kt;
    hipEvent_t ready = nullptr;
    hipStream_t sid = nullptr;       // stream that prepared it
    uint32_t inflight = 0;           // calls between lookup and release
    uint64_t tick = 0;               // last use (LRU)
    std::vector<hipStream_t> users;  // streams of device-mode uses since it was prepared
    bool many = false;               // more users than kKeyUsersMax
};
constexpr size_t kKeyCacheMax = 16;
constexpr size_t kKeyUsersMax = 8;
namespace {
std::mutex g_kc_mu;
std::vector<KeyCacheEntry*> g_kc;
uint64_t g_kc_tick = 0;

bool key_cache_on() {
    const char* ev = getenv("LCB_HASH_KEY_CACHE");
    return !(ev && ev[0] == '0');
}

void wipe_host(std::vector<uint8_t>& v) {
    if (!v.empty()) {
        volatile uint8_t* p = v.data();
        for (size_t i = 0; i < v.size(); ++i) p[i] = 0;
    }
    v.clear();
}

// Zero and free an idle entry's device buffer (caller holds g_kc_mu).  When
// every device-mode use was on `s` (the evicting call's stream, on the
// entry's device), in stream order behind them; otherwise -- other streams,
// which may be gone by now, so nothing is enqueued on them -- after a
// synchronisation of the entry's device.
void entry_destroy_locked(KeyCacheEntry* e, hipStream_t s, bool sync) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    bool done = false;
    if (!sync && cur == e->dev && !e->many) {
        bool only_s = true;
        for (hipStream_t u : e->users) only_s = only_s && u == s;
        if (only_s && hipMemsetAsync(e->dbuf, 0, e->dbytes, s) == hipSuccess && scratch_free(e->dbuf, s) == hipSuccess)
            done = true;
        (void)hipGetLastError();
    }
    if (!done) {
        if (cur != e->dev) (void)hipSetDevice(e->dev);
        (void)hipDeviceSynchronize();
        (void)hipMemset(e->dbuf, 0, e->dbytes);
        (void)hipDeviceSynchronize();
        (void)hipFree(e->dbuf);
        (void)hipGetLastError();
        if (cur != e->dev) (void)hipSetDevice(cur);
    }
    if (e->ready) (void)hipEventDestroy(e->ready);
    wipe_host(e->sig);
    delete e;
}

// Host copies of the secrets are wiped at exit (device memory goes with
// the process; the runtime may be gone by then).
struct KeyCacheAtExit {
    ~KeyCacheAtExit() {
        std::lock_guard<std::mutex> lk(g_kc_mu);
        for (KeyCacheEntry* e : g_kc) wipe_host(e->sig);
    }
} g_kc_atexit;
}  // namespace

void key_release(KeyRef& r, hipStream_t s, bool async_use) {
    if (r.temp) {
        // per-call buffer: zeroed behind the batch that read it, then freed
        (void)hipMemsetAsync(r.temp, 0, r.temp_bytes, s);
        (void)scratch_free(r.temp, s);
        (void)hipGetLastError();
        r.temp = nullptr;
    }
    if (r.entry) {
        std::lock_guard<std::mutex> lk(g_kc_mu);
        KeyCacheEntry* e = static_cast<KeyCacheEntry*>(r.entry);
        if (async_use && !e->many && std::find(e->users.begin(), e->users.end(), s) == e->users.end()) {
            if (e->users.size() < kKeyUsersMax) e->users.push_back(s);
            else e->many = true;
        }
        --e->inflight;
        r.entry = nullptr;
    }
}

// The device key table of (alg, kind, keys): cached or built on `s`; the
// caller passes `ref` to key_release once its batch is enqueued.
static int key_table(int alg, int kind, const std::vector<uint8_t>& blob, const std::vector<uint32_t>& koff,
                     const std::vector<uint32_t>& klen, const KeyBlock* kb, hipStream_t s, KeyTable* out,
                     KeyRef* ref) {
    *ref = KeyRef();
    int dev = 0;
    LCB_TRY(hipGetDevice(&dev));
    const hipStream_t sid = s;
    std::vector<uint8_t> sig(blob.begin(), blob.end());
    sig.insert(sig.end(), reinterpret_cast<const uint8_t*>(klen.data()),
               reinterpret_cast<const uint8_t*>(klen.data() + klen.size()));
    struct Wipe {
        std::vector<uint8_t>& v;
        ~Wipe() { wipe_host(v); }
    } wipe_sig{sig};
    const bool use_cache = key_cache_on();
    std::lock_guard<std::mutex> lk(g_kc_mu);
    if (use_cache) {
        for (KeyCacheEntry* e : g_kc) {
            if (e->dev != dev || e->alg != alg || e->kind != kind || e->sig != sig) continue;
            if (e->sid != sid || s == hipStreamPerThread) {
                if (hipEventQuery(e->ready) != hipSuccess) {
                    (void)hipGetLastError();
                    LCB_TRY(hipStreamWaitEvent(s, e->ready, 0));
                }
            }
            e->tick = ++g_kc_tick;
            ++e->inflight;
            ref->entry = e;
            *out = e->kt;
            return 0;
        }
    }
    const size_t nkeys = klen.size();
    const size_t blob_b = (blob.size() + 15) & ~(size_t)15, tab_b = (nkeys * 4 + 15) & ~(size_t)15;
    const size_t mid_b = nkeys * 2 * kMidWords * sizeof(uint32_t);
    // One host image of [pad | key bytes | offsets | lengths] and ONE copy;
    // the key bytes have >= 68 readable bytes on both sides (kKeyPad before,
    // the tables and mid-states after: or_window64_padded reads a window's
    // whole 68-byte span).
    constexpr size_t kKeyPad = 128;
    static_assert(2 * 16 + 2 * kMidWords * sizeof(uint32_t) >= 68, "readable bytes after the key bytes");
    std::vector<uint8_t> img(kKeyPad + blob_b + 2 * tab_b, 0);
    struct Wipe wipe_img{img};
    if (!blob.empty()) memcpy(img.data() + kKeyPad, blob.data(), blob.size());
    memcpy(img.data() + kKeyPad + blob_b, koff.data(), nkeys * 4);
    memcpy(img.data() + kKeyPad + blob_b + tab_b, klen.data(), nkeys * 4);
    bool cache = use_cache;
    if (cache && g_kc.size() >= kKeyCacheMax) {
        // Evict the least recently used idle entry.
        KeyCacheEntry* v = nullptr;
        for (KeyCacheEntry* e : g_kc)
            if (e->inflight == 0 && (!v || e->tick < v->tick)) v = e;
        if (v) {
            g_kc.erase(std::find(g_kc.begin(), g_kc.end(), v));
            entry_destroy_locked(v, s, false);
        } else {
            cache = false;   // every entry is in use: this call takes the per-call path
        }
    }
    const size_t dbytes = img.size() + mid_b;
    uint8_t* dbuf = nullptr;
    LCB_TRY(scratch_alloc(reinterpret_cast<void**>(&dbuf), dbytes, s));
    // Pageable source: the copy returns once the bytes are staged, so the
    // host image may die on return.
    hipError_t e = hipMemcpyAsync(dbuf, img.data(), img.size(), hipMemcpyHostToDevice, s);
    KeyTable kt;
    kt.mode = (uint32_t)kind;
    kt.keys = dbuf + kKeyPad;
    kt.key_off = reinterpret_cast<const uint32_t*>(dbuf + kKeyPad + blob_b);
    kt.key_len = reinterpret_cast<const uint32_t*>(dbuf + kKeyPad + blob_b + tab_b);
    kt.nkeys = (uint32_t)nkeys;
    kt.mid = reinterpret_cast<const uint32_t*>(dbuf + kKeyPad + blob_b + 2 * tab_b);
    if (e == hipSuccess) {
        if (kind == 0) {
            // One HMAC key: the key block by value (short key) or H(key) of the
            // uploaded bytes (long key), as hmac_setup always did.
            launch_hmac_prep(alg, *kb, blob.size() > bsize(alg) ? dbuf + kKeyPad : nullptr, blob.size(),
                             const_cast<uint32_t*>(kt.mid), s);
        } else if (kind != LCB_HASH_KEY_SUFFIX) {
            KArgs a;
            a.key_mode = kt.mode; a.keys = kt.keys; a.key_off = kt.key_off; a.key_len = kt.key_len;
            a.nkeys = kt.nkeys;
            launch_key_prep(alg, a, const_cast<uint32_t*>(kt.mid), s);
        }
        e = hipGetLastError();
    }
    hipEvent_t ready = nullptr;
    if (e == hipSuccess && cache) {
        e = hipEventCreateWithFlags(&ready, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventRecord(ready, s);
    }
    if (e != hipSuccess) {
        if (ready) (void)hipEventDestroy(ready);
        (void)hipMemsetAsync(dbuf, 0, dbytes, s);
        (void)scratch_free(dbuf, s);
        (void)hipGetLastError();
        return map_err(e);
    }
    if (cache) {
        KeyCacheEntry* ce = new KeyCacheEntry();
        ce->dev = dev; ce->alg = alg; ce->kind = kind; ce->sig.swap(sig);
        ce->dbuf = dbuf; ce->dbytes = dbytes; ce->kt = kt; ce->ready = ready; ce->sid = sid;
        ce->tick = ++g_kc_tick;
        ce->inflight = 1;
        g_kc.push_back(ce);
        ref->entry = ce;
    } else {
        ref->temp = dbuf;
        ref->temp_bytes = dbytes;
    }
    *out = kt;
    return 0;
}

// HMAC mid-states of one key on `s` (cached, see key_table); key_release
// `ref` once the batch reading them is enqueued.
int hmac_setup(int alg, const uint8_t* key, size_t key_len, hipStream_t s, const uint32_t** mid, KeyRef* ref) {
    KeyBlock kb;
    memset(&kb, 0, sizeof(kb));
    if (key_len > UINT32_MAX) return EINVAL;
    if (key_len <= bsize(alg) && key_len) memcpy(kb.w, key, key_len);
    std::vector<uint8_t> blob(key, key + key_len);
    std::vector<uint32_t> koff(1, 0u), klen(1, (uint32_t)key_len);
    KeyTable kt;
    const int rc = key_table(alg, 0, blob, koff, klen, &kb, s, &kt, ref);
    wipe_host(blob);
    volatile uint32_t* kw = kb.w;
    for (int i = 0; i < 32; ++i) kw[i] = 0;
    if (rc) return rc;
    *mid = kt.mid;
    return 0;
}

// Segmented long waves of a bucketed batch: the wave capacity its scratch
// holds (0: this batch is never segmented).  The tile kernel's plain MD5 /
// SHA-1 / SHA-256 digests and HMAC-MD5 (md_tiles.hpp: segmented copies cost
// code size) and md_lines_kernel (SHA-384/512, plain and HMAC) take
// segmented waves;
// batches of other modes get no state region (every ragged
// batch paid 64 B per message for it).  LCB_TILE_SEGS=0 in the environment
// turns segmenting off (read per call: the tests compare both forms in one
// process).
static uint32_t seg_capacity(int alg, const KArgs& a) {
    if (!a.lengths || a.order != nullptr || a.count < kBucketMinCount || a.count >= kBucketMaxCount) return 0;
    const bool tiles = tiles_take(alg, a);
    const bool seg_kernel = tiles ? a.key_mode == kKeyNone && alg >= 1 && alg <= 4
                                  : a.key_mode == kKeyNone && (alg == 5 || alg == 6 ||
                                                               ((alg == 7 || alg == 8) && a.mid == nullptr));
    if (!seg_kernel) return 0;
    const char* ev = getenv("LCB_TILE_SEGS");
    if (ev && ev[0] == '0') return 0;
    return bucket_seg_cap(a.count, tile_slots(alg));
}

// The take-over test (LCB_SEG_TAKEOVER=1, tests only): segmented jobs run in
// reverse segment order with no wait, and after each such batch the host
// reads its segment header (synchronising the stream) into g_seg_last.
namespace {
std::mutex g_seg_mu;
uint32_t g_seg_last[4];
}  // namespace
static bool seg_takeover_test() {
    const char* ev = getenv("LCB_SEG_TAKEOVER");
    return ev && ev[0] == '1';
}

// Launch the batch kernel, bucketing a large ragged batch by length first
// (no synchronisation).  Bucketing scratch: work_buf (at least
// ordered_words(alg, a) words), else a stream-ordered allocation.
int launch_ordered(int alg, KArgs a, hipStream_t s, uint32_t* work_buf) {
    uint32_t* work = nullptr;
    // The bucketing permutation holds message indices as uint32 and, padded
    // per key to whole tiles, up to 63 pad entries (kOrderPad = 2^32 - 1) per
    // key: its length, the scan and the tile count must stay below 2^32.
    if (a.lengths && a.order == nullptr && a.count >= kBucketMaxCount) return EINVAL;
    bool pooled = false;
    bool seg_test = false;
    if (a.lengths && a.order == nullptr && a.count >= kBucketMinCount) {
        // work: [key totals | spare | spare | entry count | order | ... | segments]
        const uint32_t cap = seg_capacity(alg, a);
        const size_t bytes = bucket_words(a.count, cap) * sizeof(uint32_t);
        if (work_buf) {
            work = work_buf;
        } else {
            LCB_TRY(scratch_alloc(reinterpret_cast<void**>(&work), bytes, s));
            pooled = true;
            // a pool block: the bucketing's sync words must start at zero
            LCB_TRY(hipMemsetAsync(work + kBucketSync, 0, kBucketSyncWords * sizeof(uint32_t), s));
        }
        const bool tiles = tiles_take(alg, a);
        const uint32_t seg_min = cap ? tile_slots(alg) : 0u;
        if (seg_min) {
            a.seg = work + bucket_seg_offset(a.count);
            a.seg_cap = cap;
            seg_test = seg_takeover_test();
        }
        launch_bucketing(a, work, work + kBucketWork, tiles, seg_min, seg_test, s);
        a.order = work + kBucketWork;
        if (tiles) a.tile_next = work + kBucketHead;
    }
    launch_batch(alg, a, s);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && seg_test) {
        // {segmented waves, taken over, published by their last segment, other}
        uint32_t nseg = 0;
        e = hipMemcpyAsync(&nseg, a.seg, 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        // (the whole segment region: the flags sit one per 4,352-B block)
        std::vector<uint32_t> reg((size_t)nseg * kSegBlockWords + 1);
        if (e == hipSuccess && nseg)
            e = hipMemcpyAsync(reg.data(), a.seg + kSegHead, (size_t)nseg * kSegBlockWords * 4, hipMemcpyDeviceToHost,
                               s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        uint32_t h[4] = {nseg, 0, 0, 0};
        for (uint32_t i = 0; i < nseg && e == hipSuccess; ++i) {
            const uint32_t f = reg[(size_t)i * kSegBlockWords + 64 * kSegStateWords];
            ++h[f == kSegTaken ? 1 : f == (uint32_t)kSegs - 1 ? 2 : 3];
            if (f != kSegTaken && f != (uint32_t)kSegs - 1 && h[3] == 1)
                fprintf(stderr, "lcb seg take-over test: wave %u flag %#x\n", i, f);
        }
        std::lock_guard<std::mutex> lk(g_seg_mu);
        memcpy(g_seg_last, h, sizeof(h));
    }
    if (pooled) (void)scratch_free(work, s);
    return map_err(e);
}

size_t bucket_scratch_words(int alg, uint64_t count) {
    KArgs a;
    a.lengths = reinterpret_cast<const uint32_t*>(&a);   // any ragged plain batch of `count`
    a.order = nullptr;
    a.count = count < kBucketMinCount ? kBucketMinCount : count;
    return bucket_words(a.count, seg_capacity(alg, a));
}

// Bucketing scratch words of a batch (0: not bucketed).
static size_t ordered_words(int alg, const KArgs& a) {
    return (a.lengths && a.order == nullptr && a.count >= kBucketMinCount && a.count < kBucketMaxCount)
               ? bucket_words(a.count, seg_capacity(alg, a))
               : 0;
}

int device_cu_count() {
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    int n = cache[dev].load(std::memory_order_relaxed);
    if (n <= 0) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cache[dev].store(n, std::memory_order_relaxed);
    }
    return n;
}

std::once_flag g_init_flag;
int g_init_rc = 0;

int ensure_init() {
    std::call_once(g_init_flag, [] {
        int n = 0;
        g_init_rc = (hipGetDeviceCount(&n) != hipSuccess || n <= 0) ? ENODEV : 0;
    });
    return g_init_rc;
}

// True when `p` is page-locked host memory the DMA engines can read directly
// (hipHostMalloc / hipHostRegister, e.g. torch's pin_memory()).
bool is_pinned(const void* p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory reports an error: clear it
        return false;
    }
    return attr.type == hipMemoryTypeHost;
}

// memcpy of many (dst, src, n) pieces, split over up to 8 host threads when
// the chunk is large (the single-thread staging copy was the host-path bound).
void parallel_copy(const std::vector<Piece>& pieces, size_t bytes) {
    const size_t nt = bytes >= (8u << 20) ? std::min<size_t>(8, pieces.size()) : 1;
    if (nt <= 1) {
        for (const Piece& p : pieces) memcpy(p.dst, p.src, p.n);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (pieces.size() + nt - 1) / nt;
    for (size_t t = 0; t < nt; ++t) {
        const size_t lo = t * per, hi = std::min(pieces.size(), lo + per);
        if (lo >= hi) break;
        th.emplace_back([&pieces, lo, hi] {
            for (size_t k = lo; k < hi; ++k) memcpy(pieces[k].dst, pieces[k].src, pieces[k].n);
        });
    }
    for (auto& x : th) x.join();
}

}  // namespace lcbgpu

namespace lcbgpu {

static void set_keys(KArgs& a, const KeyTable* kt, const uint32_t* index) {
    if (!kt) return;
    a.key_mode = kt->mode; a.keys = kt->keys; a.key_off = kt->key_off; a.key_len = kt->key_len;
    a.nkeys = kt->nkeys; a.mid = kt->mid; a.key_index = index;
}

int batch_device(int alg, const uint8_t* key, size_t key_len, const uint8_t* data,
                 const uint64_t* offsets, const uint32_t* lengths, size_t count, uint64_t stride,
                 uint32_t fixed_len, uint8_t* digests, hipStream_t s, const uint32_t* init,
                 const KeyTable* kt, const KeyCheck* kc) {
    KArgs a;
    a.data = data; a.offsets = offsets; a.lengths = lengths; a.order = nullptr;
    a.count = count; a.stride = stride; a.fixed_len = fixed_len; a.digests = digests;
    a.mid = nullptr;
    a.init = init;
    set_keys(a, kt, kt ? kt->index : nullptr);
    if (kc) {
        a.bad = kc->dflag;
        a.bad_epoch = kc->epoch;
        a.check_host = kc->fused_host;
    }
    KeyRef kref;
    if (key) {
        const uint32_t* mid = nullptr;
        int rc = hmac_setup(alg, key, key_len, s, &mid, &kref);
        if (rc) return rc;
        a.mid = mid;
    }
    int rc;
    const size_t words = ordered_words(alg, a);
    // A fused check needs this batch's bucketing on the keyed call's scratch.
    if (kc && kc->fused_host && (words == 0 || kc->work_words < words)) {
        rc = EINVAL;
    } else if (kc && kc->work_words >= words) {
        rc = launch_ordered(alg, a, s, kc->work);   // the keyed call's stream scratch
    } else if (words) {
        StreamScratch* ss = stream_scratch_acquire(s, words * sizeof(uint32_t));
        rc = launch_ordered(alg, a, s, ss ? reinterpret_cast<uint32_t*>(stream_scratch_payload(ss)) : nullptr);
        stream_scratch_release(ss);
    } else {
        rc = launch_ordered(alg, a, s);
    }
    key_release(kref, s, true);
    return rc;
}

// ------------------------------------------------------------ host mode
// Per-thread staging context for the current device.
struct Stage {
    int device = -1;
    size_t cap = 0;                 // data bytes per buffer
    size_t mcap = 0;                // messages per buffer
    hipStream_t st[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    uint8_t* h_data[2] = {nullptr, nullptr};
    uint64_t* h_off[2] = {nullptr, nullptr};
    uint32_t* h_len[2] = {nullptr, nullptr};
    uint32_t* h_init[2] = {nullptr, nullptr};   // CRC X_update() values of the chunk
    uint8_t* h_dig[2] = {nullptr, nullptr};
    uint8_t* d_data[2] = {nullptr, nullptr};
    uint64_t* d_off[2] = {nullptr, nullptr};
    uint32_t* d_len[2] = {nullptr, nullptr};
    uint32_t* d_init[2] = {nullptr, nullptr};
    uint8_t* d_dig[2] = {nullptr, nullptr};
    // pending chunk per buffer (digests to copy out once `done` fires)
    size_t pend_first[2] = {0, 0}, pend_n[2] = {0, 0};
    bool busy[2] = {false, false};

    void release() {
        for (int b = 0; b < 2; ++b) {
            if (h_data[b]) (void)hipHostFree(h_data[b]);
            if (h_off[b]) (void)hipHostFree(h_off[b]);
            if (h_len[b]) (void)hipHostFree(h_len[b]);
            if (h_init[b]) (void)hipHostFree(h_init[b]);
            if (h_dig[b]) (void)hipHostFree(h_dig[b]);
            if (d_data[b]) (void)hipFree(d_data[b]);
            if (d_off[b]) (void)hipFree(d_off[b]);
            if (d_len[b]) (void)hipFree(d_len[b]);
            if (d_init[b]) (void)hipFree(d_init[b]);
            if (d_dig[b]) (void)hipFree(d_dig[b]);
            if (done[b]) (void)hipEventDestroy(done[b]);
            if (st[b]) (void)hipStreamDestroy(st[b]);
            h_data[b] = nullptr; h_off[b] = nullptr; h_len[b] = nullptr; h_dig[b] = nullptr;
            d_data[b] = nullptr; d_off[b] = nullptr; d_len[b] = nullptr; d_dig[b] = nullptr;
            h_init[b] = nullptr; d_init[b] = nullptr;
            done[b] = nullptr; st[b] = nullptr;
        }
        cap = mcap = 0;
        device = -1;
    }
    ~Stage() { release(); }

    int ensure(int dev, size_t need_bytes, size_t need_msgs) {
        if (device == dev && cap >= need_bytes && mcap >= need_msgs) return 0;
        size_t nb = std::max(need_bytes, cap), nm = std::max(need_msgs, mcap);
        release();
        device = dev;
        for (int b = 0; b < 2; ++b) {
            LCB_TRY(hipStreamCreateWithFlags(&st[b], hipStreamNonBlocking));
            LCB_TRY(hipEventCreateWithFlags(&done[b], hipEventDisableTiming));
            LCB_TRY(hipHostMalloc(reinterpret_cast<void**>(&h_data[b]), nb, hipHostMallocDefault));
            LCB_TRY(hipHostMalloc(reinterpret_cast<void**>(&h_off[b]), nm * 8, hipHostMallocDefault));
            LCB_TRY(hipHostMalloc(reinterpret_cast<void**>(&h_len[b]), nm * 4, hipHostMallocDefault));
            LCB_TRY(hipHostMalloc(reinterpret_cast<void**>(&h_init[b]), nm * 4, hipHostMallocDefault));
            LCB_TRY(hipHostMalloc(reinterpret_cast<void**>(&h_dig[b]), nm * 64, hipHostMallocDefault));
            LCB_TRY(hipMalloc(reinterpret_cast<void**>(&d_data[b]), nb));
            LCB_TRY(hipMalloc(reinterpret_cast<void**>(&d_off[b]), nm * 8));
            LCB_TRY(hipMalloc(reinterpret_cast<void**>(&d_len[b]), nm * 4));
            LCB_TRY(hipMalloc(reinterpret_cast<void**>(&d_init[b]), nm * 4));
            LCB_TRY(hipMalloc(reinterpret_cast<void**>(&d_dig[b]), nm * 64));
        }
        cap = nb;
        mcap = nm;
        return 0;
    }
};

thread_local Stage g_stage;
constexpr size_t kChunkBytes = 64ull << 20;   // 64 MiB per in-flight chunk
constexpr size_t kChunkMsgs = 1u << 18;       // 256 K messages per chunk

// Staging contexts for worker threads of the multi-device path: a pool per
// device, so repeated lcb_hash_batch_multi calls reuse their pinned buffers.
std::mutex g_pool_m;
std::vector<Stage*> g_pool;

Stage* stage_acquire(int dev) {
    std::lock_guard<std::mutex> lk(g_pool_m);
    for (size_t k = 0; k < g_pool.size(); ++k)
        if (g_pool[k]->device == dev) {
            Stage* st = g_pool[k];
            g_pool.erase(g_pool.begin() + k);
            return st;
        }
    return new Stage();
}
void stage_release(Stage* st) {
    std::lock_guard<std::mutex> lk(g_pool_m);
    g_pool.push_back(st);
}

int batch_host(int alg, const uint8_t* key, size_t key_len, const uint8_t* data,
               const uint64_t* offsets, const uint32_t* lengths, size_t count, uint64_t stride,
               uint32_t fixed_len, uint8_t* digests, const uint32_t* init, Stage* stage,
               const KeyTable* kt) {
    int dev = 0;
    LCB_TRY(hipGetDevice(&dev));
    Stage& S = stage ? *stage : g_stage;
    const size_t D = dsize(alg);
    const bool fixed = (offsets == nullptr && lengths == nullptr);
    auto off_of = [&](size_t i) -> uint64_t { return offsets ? offsets[i] : (uint64_t)i * stride; };
    auto len_of = [&](size_t i) -> uint64_t { return lengths ? lengths[i] : fixed_len; };

    // Largest single message decides the minimum buffer.
    uint64_t maxlen = fixed_len;
    if (lengths) {
        maxlen = 0;
        for (size_t i = 0; i < count; ++i) maxlen = std::max<uint64_t>(maxlen, lengths[i]);
    }
    int rc = S.ensure(dev, std::max<size_t>(kChunkBytes, maxlen), kChunkMsgs);
    if (rc) return rc;
    const bool src_pinned = is_pinned(data);
    const bool dig_pinned = is_pinned(digests);

    const uint32_t* mid = nullptr;
    KeyRef kref;
    if (key) {
        rc = hmac_setup(alg, key, key_len, S.st[0], &mid, &kref);
        if (rc) return rc;
        if (hipStreamSynchronize(S.st[0]) != hipSuccess) {   // mid-states visible to both streams
            key_release(kref, S.st[0], false);
            (void)hipStreamSynchronize(S.st[0]);
            return EIO;
        }
    }

    auto drain = [&](int b) -> int {
        if (!S.busy[b]) return 0;
        LCB_TRY(hipEventSynchronize(S.done[b]));
        if (!dig_pinned) memcpy(digests + S.pend_first[b] * D, S.h_dig[b], S.pend_n[b] * D);
        S.busy[b] = false;
        return 0;
    };

    std::vector<Piece> pieces;
    size_t i = 0;
    int b = 0;
    while (i < count) {
        if ((rc = drain(b))) break;
        hipStream_t s = S.st[b];
        // Choose messages [i, j): their bytes must fit one staging buffer.
        size_t j = i;
        uint64_t base = 0, span = 0, total = 0;
        if (fixed) {
            // Direct DMA copies the span [i*stride, (j-1)*stride + fixed_len);
            // the gather path packs (j-i) * fixed_len bytes.  Both must fit
            // one staging buffer (stride < fixed_len, e.g. 0 or overlapping
            // records, makes the packed size the larger one).
            size_t per = stride ? std::max<size_t>(1, (S.cap - fixed_len) / stride + 1) : S.mcap;
            if (!src_pinned) per = std::min<size_t>(per, fixed_len ? S.cap / fixed_len : S.mcap);
            j = std::min(count, i + std::min(per, S.mcap));
            base = (uint64_t)i * stride;
            span = (uint64_t)(j - i - 1) * stride + fixed_len;
            total = (uint64_t)(j - i) * fixed_len;
        } else {
            uint64_t lo = UINT64_MAX, hi = 0;
            while (j < count && j - i < S.mcap) {
                const uint64_t o = off_of(j), n = len_of(j);
                const uint64_t nlo = std::min(lo, o), nhi = std::max(hi, o + n);
                if (j > i && (nhi - nlo > S.cap || total + n > S.cap)) break;
                lo = nlo; hi = nhi; total += n;
                ++j;
            }
            base = lo;
            span = hi - lo;
        }
        const size_t n = j - i;
        // Direct DMA from pinned input when the chunk's bytes are dense enough;
        // otherwise gather the messages into pinned staging first.
        const bool direct = src_pinned && span <= S.cap && (fixed || span <= 2 * total + 4096);
        KArgs a;
        a.order = nullptr; a.count = n; a.digests = S.d_dig[b]; a.mid = mid;
        bool ok = true;
        // One uint32 per message rides along with the chunk: the CRC
        // X_update() values, or the key index of a keyed batch.
        const uint32_t* per_msg = init ? init : (kt ? kt->index : nullptr);
        if (per_msg) {
            memcpy(S.h_init[b], per_msg + i, n * 4);
            ok = hipMemcpyAsync(S.d_init[b], S.h_init[b], n * 4, hipMemcpyHostToDevice, s) == hipSuccess;
            if (init) a.init = S.d_init[b];
        }
        set_keys(a, kt, kt && kt->index ? S.d_init[b] : nullptr);
        if (!ok) {
        } else if (direct) {
            ok = hipMemcpyAsync(S.d_data[b], data + base, span ? span : 1, hipMemcpyHostToDevice, s) == hipSuccess;
            if (fixed) {
                a.data = S.d_data[b]; a.offsets = nullptr; a.lengths = nullptr;
                a.stride = stride; a.fixed_len = fixed_len;
            } else {
                for (size_t k = 0; k < n; ++k) {
                    S.h_off[b][k] = off_of(i + k) - base;
                    S.h_len[b][k] = (uint32_t)len_of(i + k);
                }
                a.data = S.d_data[b]; a.offsets = S.d_off[b]; a.lengths = S.d_len[b];
                a.stride = 0; a.fixed_len = 0;
            }
        } else {
            pieces.clear();
            uint64_t pos = 0;
            for (size_t k = 0; k < n; ++k) {
                const uint64_t ln = len_of(i + k);
                pieces.push_back(Piece{S.h_data[b] + pos, data + off_of(i + k), (size_t)ln});
                S.h_off[b][k] = pos;
                S.h_len[b][k] = (uint32_t)ln;
                pos += ln;
            }
            parallel_copy(pieces, pos);
            ok = hipMemcpyAsync(S.d_data[b], S.h_data[b], pos ? pos : 1, hipMemcpyHostToDevice, s) == hipSuccess;
            a.data = S.d_data[b]; a.offsets = S.d_off[b]; a.lengths = S.d_len[b];
            a.stride = 0; a.fixed_len = 0;
        }
        if (ok && a.offsets) {
            ok = hipMemcpyAsync(S.d_off[b], S.h_off[b], n * 8, hipMemcpyHostToDevice, s) == hipSuccess &&
                 hipMemcpyAsync(S.d_len[b], S.h_len[b], n * 4, hipMemcpyHostToDevice, s) == hipSuccess;
        }
        if (!ok || launch_ordered(alg, a, s) != 0 ||
            hipMemcpyAsync(dig_pinned ? digests + i * D : S.h_dig[b], S.d_dig[b], n * D,
                           hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipEventRecord(S.done[b], s) != hipSuccess) {
            rc = EIO;
            break;
        }
        S.pend_first[b] = i;
        S.pend_n[b] = n;
        S.busy[b] = true;
        i = j;
        b ^= 1;
    }
    int rc2 = drain(0);
    int rc3 = drain(1);
    if (key) {  // both streams are drained: release the HMAC state (a per-call one is zeroed)
        key_release(kref, S.st[0], false);
        (void)hipStreamSynchronize(S.st[0]);
    }
    if (rc) return rc;
    if (rc2) return rc2;
    return rc3;
}

}  // namespace lcbgpu

using namespace lcbgpu;

// ================================================================== ABI
extern "C" {

int lcb_hash_gpu_abi_version(void) { return LCB_HASH_GPU_ABI_VERSION; }
size_t lcb_hash_digest_size(int alg) { return dsize(alg); }
size_t lcb_hash_block_size(int alg) { return bsize(alg); }

int lcb_hash_gpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* lcb_hash_strerror(int error) {
    switch (error) {
    case 0: return "success";
    case EINVAL: return "invalid argument";
    case ENOMEM: return "out of device or pinned memory";
    case ENODEV: return "no usable MI355X / HIP device";
    case EIO: return "HIP launch or copy failure";
    case EMSGSIZE: return "packet larger than a queue batch";
    case EAGAIN: return "no free queue staging slot";
    case EBUSY: return "resource in use by a call in progress";
    default: return "unknown error";
    }
}

int lcb_hash_batch(int alg, const uint8_t* key, size_t key_len, const uint8_t* data,
                   const uint64_t* offsets, const uint32_t* lengths, size_t count, uint64_t stride,
                   uint32_t fixed_len, uint8_t* digests, uint32_t flags, void* stream) {
    if (alg < LCB_HASH_MD5 || alg > LCB_HASH_GOST512) return EINVAL;
    if (flags & ~LCB_HASH_F_DEVICE) return EINVAL;
    if (count == 0) return 0;
    if (!data || !digests) return EINVAL;
    if (key == nullptr && key_len != 0) return EINVAL;
    if (int rc = ensure_init()) return rc;
    if (flags & LCB_HASH_F_DEVICE)
        return batch_device(alg, key, key_len, data, offsets, lengths, count, stride, fixed_len,
                            digests, reinterpret_cast<hipStream_t>(stream), nullptr);
    return batch_host(alg, key, key_len, data, offsets, lengths, count, stride, fixed_len, digests,
                      nullptr, nullptr);
}

int lcb_hash_batch_keyed(int alg, int key_mode, const uint8_t* keys, const uint64_t* key_offsets,
                         const uint32_t* key_lengths, size_t nkeys, const uint32_t* key_index,
                         const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths, size_t count,
                         uint64_t stride, uint32_t fixed_len, uint8_t* digests, uint32_t flags, void* stream) {
    static_assert(LCB_HASH_KEY_HMAC == kKeyHmac && LCB_HASH_KEY_PREFIX == kKeyPrefix &&
                  LCB_HASH_KEY_SUFFIX == kKeySuffix, "key mode ids");
    if (alg < LCB_HASH_MD5 || alg > LCB_HASH_GOST512) return EINVAL;
    if (key_mode < LCB_HASH_KEY_HMAC || key_mode > LCB_HASH_KEY_SUFFIX) return EINVAL;
    if (flags & ~LCB_HASH_F_DEVICE) return EINVAL;
    if (nkeys == 0 || nkeys > UINT32_MAX || !key_lengths) return EINVAL;
    if (count == 0) return 0;
    if (!data || !digests) return EINVAL;
    const bool dev_mode = flags & LCB_HASH_F_DEVICE;
    // Pack the key table (host memory) into one blob.
    std::vector<uint32_t> koff(nkeys), klen(nkeys);
    uint64_t total = 0;
    for (size_t k = 0; k < nkeys; ++k) {
        if (key_lengths[k] && !keys) return EINVAL;
        koff[k] = (uint32_t)total;
        klen[k] = key_lengths[k];
        total += key_lengths[k];
        if (total > UINT32_MAX) return EINVAL;
    }
    if (!dev_mode && key_index)
        for (size_t i = 0; i < count; ++i)
            if (key_index[i] >= nkeys) return EINVAL;
    if (int rc = ensure_init()) return rc;
    std::vector<uint8_t> blob(total ? total : 1);
    for (size_t k = 0; k < nkeys; ++k)
        if (klen[k]) memcpy(blob.data() + koff[k], keys + (key_offsets ? key_offsets[k] : 0), klen[k]);
    hipStream_t s = dev_mode ? reinterpret_cast<hipStream_t>(stream) : nullptr;
    // The device key table (bytes, offsets, lengths, mid-states): cached
    // across calls with the same keys (key_table), else built on `s`.
    KeyTable kt;
    KeyRef kref;
    int rc = key_table(alg, key_mode, blob, koff, klen, nullptr, s, &kt, &kref);
    wipe_host(blob);
    if (rc) return rc;
    kt.index = key_index;
    if (!dev_mode) {
        // Host mode: the pipeline's own streams read the table; wait for it.
        rc = hipStreamSynchronize(s) == hipSuccess ? 0 : EIO;
        if (!rc) rc = batch_host(alg, nullptr, 0, data, offsets, lengths, count, stride, fixed_len, digests,
                                 nullptr, nullptr, &kt);
        key_release(kref, s, false);
        (void)hipStreamSynchronize(s);
        return rc;
    }
    if (!key_index) {
        rc = batch_device(alg, nullptr, 0, data, offsets, lengths, count, stride, fixed_len, digests, s, nullptr,
                          &kt);
        key_release(kref, s, true);
        return rc;
    }
    // Device mode with per-message key indices: an index >= nkeys is EINVAL
    // and no digest is written, as in host mode.  The check kernel runs
    // first: a block that finds a bad index writes this call's epoch into
    // the stream scratch's flag word, and the last of its blocks (a counter
    // in the same header) writes epoch | bad bit into a pinned host word.
    // The batch is enqueued right behind the check with every digest store
    // gated on the device flag (batch_aborted); only then does the host wait,
    // for the check's host word, not for the batch.  The GPU never idles for
    // the host's round trip, and nothing is recorded on the stream (r4: three
    // key uploads, a memset, a read-back and 40 us of idle stream per keyed
    // call; an event record costs 6.5 us: profiles/r5_pkt_gaps.txt).
    KArgs probe;
    probe.lengths = lengths; probe.order = nullptr; probe.count = count; probe.key_mode = (uint32_t)key_mode;
    const size_t words = ordered_words(alg, probe);
    StreamScratch* ss = stream_scratch_acquire(s, std::max<size_t>(words, 1) * sizeof(uint32_t));
    if (ss) {
        ss->epoch = (ss->epoch + 1) & 0x7fffffffu;
        if (ss->epoch == 0) ss->epoch = 1;
        KeyCheck kc;
        kc.dflag = reinterpret_cast<const uint32_t*>(ss->p);
        kc.epoch = ss->epoch;
        kc.work = reinterpret_cast<uint32_t*>(stream_scratch_payload(ss));
        kc.work_words = ss->bytes / sizeof(uint32_t);
        if (words && kc.work_words >= words) {
            // Bucketed: the count kernel checks the indices (bucket_count_kernel<true>).
            kc.fused_host = ss->hflag;
        } else {
            const uint32_t nblk = launch_key_check(key_index, count, (uint32_t)nkeys,
                                                   reinterpret_cast<uint32_t*>(ss->p), ss->hflag, kc.epoch, ss->ctr, s);
            // The host's expected block count advances only with a launch
            // that happened (a failed launch left it ahead for
            // good and every later keyed call on the stream returned EIO).
            rc = map_err(hipGetLastError());
            if (!rc) ss->ctr += nblk;
        }
        if (!rc)
            rc = batch_device(alg, nullptr, 0, data, offsets, lengths, count, stride, fixed_len, digests, s, nullptr,
                              &kt, &kc);
        key_release(kref, s, true);
        if (!rc) {
            // Spin on the host word for a while, then poll with short sleeps;
            // a stream that has drained without the word is an error.
            for (uint64_t it = 0;; ++it) {
                const uint32_t v = __atomic_load_n(ss->hflag, __ATOMIC_ACQUIRE);
                if ((v & 0x7fffffffu) == kc.epoch) {
                    if (v >> 31) rc = EINVAL;
                    break;
                }
                if (it < 20000) {
                    __builtin_ia32_pause();
                    continue;
                }
                if ((it & 63) == 0) {
                    const hipError_t q = hipStreamQuery(s);
                    if (q == hipSuccess &&
                        (__atomic_load_n(ss->hflag, __ATOMIC_ACQUIRE) & 0x7fffffffu) != kc.epoch) {
                        rc = EIO;
                        break;
                    }
                    if (q != hipSuccess && q != hipErrorNotReady) {
                        rc = map_err(q);
                        break;
                    }
                    (void)hipGetLastError();
                }
                std::this_thread::sleep_for(std::chrono::microseconds(5));
            }
        }
        stream_scratch_release(ss);   // held until the host word was read (epochs are per buffer)
        return rc;
    }
    // No stream scratch free (another thread enqueues on this stream): the
    // check's flag in a pooled word, read back before the batch.
    uint32_t* d_bad = nullptr;
    uint32_t h_bad = 0;
    if (scratch_alloc(reinterpret_cast<void**>(&d_bad), 16, s) != hipSuccess) rc = ENOMEM;
    if (!rc && hipMemsetAsync(d_bad, 0, 4, s) != hipSuccess) rc = EIO;
    if (!rc) {
        (void)launch_key_check(key_index, count, (uint32_t)nkeys, d_bad, nullptr, 1u, 0u, s);
        if (hipGetLastError() != hipSuccess || hipMemcpyAsync(&h_bad, d_bad, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            rc = EIO;
    }
    if (!rc && h_bad) rc = EINVAL;
    if (!rc) rc = batch_device(alg, nullptr, 0, data, offsets, lengths, count, stride, fixed_len, digests, s, nullptr, &kt);
    if (d_bad) (void)scratch_free(d_bad, s);
    key_release(kref, s, true);
    return rc;
}

int md5_get_digest_batch(const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths,
                         size_t count, uint64_t stride, uint32_t fixed_len, uint8_t* digests,
                         uint32_t flags, void* stream) {
    return lcb_hash_batch(LCB_HASH_MD5, nullptr, 0, data, offsets, lengths, count, stride, fixed_len,
                          digests, flags, stream);
}
int md5_hmac_get_digest_batch(const uint8_t* key, size_t key_size, const uint8_t* data,
                              const uint64_t* offsets, const uint32_t* lengths, size_t count,
                              uint64_t stride, uint32_t fixed_len, uint8_t* digests, uint32_t flags,
                              void* stream) {
    static const uint8_t empty = 0;
    return lcb_hash_batch(LCB_HASH_MD5, key ? key : &empty, key_size, data, offsets, lengths, count,
                          stride, fixed_len, digests, flags, stream);
}
int sha1_get_digest_batch(const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths,
                          size_t count, uint64_t stride, uint32_t fixed_len, uint8_t* digests,
                          uint32_t flags, void* stream) {
    return lcb_hash_batch(LCB_HASH_SHA1, nullptr, 0, data, offsets, lengths, count, stride, fixed_len,
                          digests, flags, stream);
}
int sha1_hmac_get_digest_batch(const uint8_t* key, size_t key_size, const uint8_t* data,
                               const uint64_t* offsets, const uint32_t* lengths, size_t count,
                               uint64_t stride, uint32_t fixed_len, uint8_t* digests, uint32_t flags,
                               void* stream) {
    static const uint8_t empty = 0;
    return lcb_hash_batch(LCB_HASH_SHA1, key ? key : &empty, key_size, data, offsets, lengths, count,
                          stride, fixed_len, digests, flags, stream);
}

// sha2_init's bits convention (sha2.h:217-241): bits or bytes.
static int sha2_alg(size_t bits) {
    switch (bits) {
    case 224: case 28: return LCB_HASH_SHA224;
    case 256: case 32: return LCB_HASH_SHA256;
    case 384: case 48: return LCB_HASH_SHA384;
    case 512: case 64: return LCB_HASH_SHA512;
    }
    return 0;
}
// gost3411_2012_init (gost3411-2012.h:1715-1729): 256/32 -> 256, else 512.
static int gost_alg(size_t bits) {
    return (bits == 256 || bits == 32) ? LCB_HASH_GOST256 : LCB_HASH_GOST512;
}

int sha2_get_digest_batch(size_t bits, const uint8_t* data, const uint64_t* offsets,
                          const uint32_t* lengths, size_t count, uint64_t stride, uint32_t fixed_len,
                          uint8_t* digests, size_t* digest_size, uint32_t flags, void* stream) {
    const int alg = sha2_alg(bits);
    if (!alg) return EINVAL;
    if (digest_size) *digest_size = dsize(alg);
    return lcb_hash_batch(alg, nullptr, 0, data, offsets, lengths, count, stride, fixed_len, digests,
                          flags, stream);
}
int sha2_hmac_get_digest_batch(size_t bits, const uint8_t* key, size_t key_size, const uint8_t* data,
                               const uint64_t* offsets, const uint32_t* lengths, size_t count,
                               uint64_t stride, uint32_t fixed_len, uint8_t* digests,
                               size_t* digest_size, uint32_t flags, void* stream) {
    static const uint8_t empty = 0;
    const int alg = sha2_alg(bits);
    if (!alg) return EINVAL;
    if (digest_size) *digest_size = dsize(alg);
    return lcb_hash_batch(alg, key ? key : &empty, key_size, data, offsets, lengths, count, stride,
                          fixed_len, digests, flags, stream);
}
int gost3411_2012_get_digest_batch(size_t bits, const uint8_t* data, const uint64_t* offsets,
                                   const uint32_t* lengths, size_t count, uint64_t stride,
                                   uint32_t fixed_len, uint8_t* digests, size_t* digest_size,
                                   uint32_t flags, void* stream) {
    const int alg = gost_alg(bits);
    if (digest_size) *digest_size = dsize(alg);
    return lcb_hash_batch(alg, nullptr, 0, data, offsets, lengths, count, stride, fixed_len, digests,
                          flags, stream);
}
int gost3411_2012_hmac_get_digest_batch(size_t bits, const uint8_t* key, size_t key_size,
                                        const uint8_t* data, const uint64_t* offsets,
                                        const uint32_t* lengths, size_t count, uint64_t stride,
                                        uint32_t fixed_len, uint8_t* digests, size_t* digest_size,
                                        uint32_t flags, void* stream) {
    static const uint8_t empty = 0;
    const int alg = gost_alg(bits);
    if (digest_size) *digest_size = dsize(alg);
    return lcb_hash_batch(alg, key ? key : &empty, key_size, data, offsets, lengths, count, stride,
                          fixed_len, digests, flags, stream);
}

int lcb_hash_gen_synthetic(uint64_t seed, uint64_t start, uint8_t* dev_out, size_t n, void* stream) {
    if (n == 0) return 0;
    if (!dev_out) return EINVAL;
    launch_gen(seed, start, dev_out, n, reinterpret_cast<hipStream_t>(stream));
    return map_err(hipGetLastError());
}

size_t lcb_hash_gpu_probe_sink_words(int mode, size_t count) {
    if (mode == LCB_PROBE_RECORDS || mode == LCB_PROBE_GOST_LPS) return count;
    if (ensure_init()) return 0;
    return (size_t)8 * device_cu_count() * 256;
}

int lcb_hash_gpu_read_probe(int mode, const uint8_t* dev_data, size_t count, uint64_t stride, uint32_t fixed_len,
                            uint32_t* dev_sink, void* stream) {
    if (int rc = ensure_init()) return rc;
    if (mode == LCB_PROBE_GOST_LPS) {
        if (!dev_sink || count == 0 || count > UINT32_MAX) return EINVAL;
        launch_gost_lps_probe(count, fixed_len, dev_sink, reinterpret_cast<hipStream_t>(stream));
        return map_err(hipGetLastError());
    }
    if (!dev_data || !dev_sink || count == 0) return EINVAL;
    KArgs a{};
    a.data = dev_data;
    a.count = count;
    a.stride = stride;
    a.fixed_len = fixed_len;
    if (mode == LCB_PROBE_RECORDS) {
        if (!fixed_stride_lines(a)) return EINVAL;
    } else if (mode == LCB_PROBE_LINEAR) {
        if ((count * stride) % 16 || (reinterpret_cast<uintptr_t>(dev_data) & 15u)) return EINVAL;
    } else {
        return EINVAL;
    }
    launch_probe(mode, a, dev_sink, reinterpret_cast<hipStream_t>(stream));
    return map_err(hipGetLastError());
}

int lcb_hash_gpu_clock_stamp(uint64_t* dev_out, size_t slots, void* stream) {
    if (int rc = ensure_init()) return rc;
    if (!dev_out || slots == 0 || slots > 4096 || slots % 8 || (reinterpret_cast<uintptr_t>(dev_out) & 7u))
        return EINVAL;
    launch_clock_stamp(dev_out, (uint32_t)slots, reinterpret_cast<hipStream_t>(stream));
    return map_err(hipGetLastError());
}

int lcb_hash_key_cache_flush(void) {
    if (int rc = ensure_init()) return rc;
    std::lock_guard<std::mutex> lk(g_kc_mu);
    int rc = 0;
    for (size_t k = 0; k < g_kc.size();) {
        KeyCacheEntry* e = g_kc[k];
        if (e->inflight) {   // a call in progress holds it
            rc = EBUSY;
            ++k;
            continue;
        }
        g_kc.erase(g_kc.begin() + k);
        entry_destroy_locked(e, nullptr, true);
    }
    return rc;
}

size_t lcb_hash_key_cache_entries(void) {
    std::lock_guard<std::mutex> lk(g_kc_mu);
    return g_kc.size();
}

int lcb_hash_gpu_seg_last(uint32_t* out) {
    if (!out) return EINVAL;
    std::lock_guard<std::mutex> lk(g_seg_mu);
    memcpy(out, g_seg_last, sizeof(g_seg_last));
    return 0;
}

int lcb_hash_gpu_gost_table(uint64_t* out) {
    if (!out) return EINVAL;
    gost_table_host(out);
    return 0;
}

}  // extern "C"

// ================================================================ CRC-32
extern "C" {

int lcb_crc32_batch(int variant, const uint32_t* init, const uint8_t* data, const uint64_t* offsets,
                    const uint32_t* lengths, size_t count, uint64_t stride, uint32_t fixed_len,
                    uint32_t* crcs, uint32_t flags, void* stream) {
    if (variant < LCB_CRC32A || variant > LCB_CRC32Q) return EINVAL;
    if (flags & ~LCB_HASH_F_DEVICE) return EINVAL;
    if (count == 0) return 0;
    if (!data || !crcs || (reinterpret_cast<uintptr_t>(crcs) & 3u)) return EINVAL;
    if (int rc = ensure_init()) return rc;
    const int alg = kCrcAlgBase + variant;
    uint8_t* out = reinterpret_cast<uint8_t*>(crcs);
    if (flags & LCB_HASH_F_DEVICE)
        return batch_device(alg, nullptr, 0, data, offsets, lengths, count, stride, fixed_len, out,
                            reinterpret_cast<hipStream_t>(stream), init);
    return batch_host(alg, nullptr, 0, data, offsets, lengths, count, stride, fixed_len, out, init, nullptr);
}

#define LCB_CRC_ENTRY(name, id)                                                                       \
    int name##_batch(const uint32_t* init, const uint8_t* data, const uint64_t* offsets,              \
                     const uint32_t* lengths, size_t count, uint64_t stride, uint32_t fixed_len,      \
                     uint32_t* crcs, uint32_t flags, void* stream) {                                  \
        return lcb_crc32_batch(id, init, data, offsets, lengths, count, stride, fixed_len, crcs,       \
                               flags, stream);                                                        \
    }
LCB_CRC_ENTRY(crc32a, LCB_CRC32A)
LCB_CRC_ENTRY(crc32cksum, LCB_CRC32CKSUM)
LCB_CRC_ENTRY(crc32mpeg2, LCB_CRC32MPEG2)
LCB_CRC_ENTRY(crc32b, LCB_CRC32B)
LCB_CRC_ENTRY(crc32jamcrc, LCB_CRC32JAMCRC)
LCB_CRC_ENTRY(crc32c, LCB_CRC32C)
LCB_CRC_ENTRY(crc32d, LCB_CRC32D)
LCB_CRC_ENTRY(crc32q, LCB_CRC32Q)
#undef LCB_CRC_ENTRY

int lcb_crc32_gpu_tables(int variant, uint32_t* out) {
    if (variant < LCB_CRC32A || variant > LCB_CRC32Q || !out) return EINVAL;
    crc_table_host(variant, out);
    return 0;
}

}  // extern "C"
