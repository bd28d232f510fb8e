// lcb_internal.hpp — types shared by the kernel TU and the C-ABI TU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace lcbgpu {

// Device-side description of one batch (see include/lcb_hash_gpu.h).
struct KArgs {
    const uint8_t* data;
    const uint64_t* offsets;   // nullptr: i * stride
    const uint32_t* lengths;   // nullptr: fixed_len
    const uint32_t* order;     // nullptr: identity; else bucketing permutation
    uint64_t count;
    uint64_t stride;
    uint32_t fixed_len;
    uint8_t* digests;          // packed count x D (CRC: count x uint32)
    const uint32_t* mid;       // HMAC mid-states (nullptr: plain digest)
    const uint32_t* init = nullptr;  // CRC: per-buffer X_update() value (nullptr: one-shot X())
    // Bucketed batches for the tile kernel (set with a padded `order`):
    // [1] = entries of `order`, pads included.
    uint32_t* tile_next = nullptr;
    // Keyed batches (lcb_hash_batch_keyed): per-message key index into a key
    // table on the device; `mid` then holds 2 * kMidWords words per key.
    uint32_t key_mode = 0;           // kKeyNone / kKeyHmac / kKeyPrefix / kKeySuffix
    const uint32_t* key_index = nullptr;  // nullptr: key 0 for every message
    const uint8_t* keys = nullptr;   // key bytes
    const uint32_t* key_off = nullptr;
    const uint32_t* key_len = nullptr;
    uint32_t nkeys = 0;
    // Keyed device batches: the key-index check's flag word; a digest is
    // stored only while *bad != bad_epoch (batch_aborted).
    const uint32_t* bad = nullptr;
    uint32_t bad_epoch = 0;
    // Set when the check runs inside the bucketing (launch_bucketing): the
    // count kernel checks the indices and sets *bad, the base kernel writes
    // the result to this pinned host word (no separate check kernel).
    uint32_t* check_host = nullptr;
    // Segmented long tiles (md_tiles.hpp): header, then per segmented wave
    // its saved states and flag (bucket_seg_words); nullptr: no tile is
    // segmented.  seg_cap: the waves that may be cut (the grid's extra jobs).
    uint32_t* seg = nullptr;
    uint32_t seg_cap = 0;
};

// True when the key-index check of this keyed batch found an index >= nkeys
// (lcb_hash_batch_keyed, device mode): its kernels then store no digest.
__device__ __forceinline__ bool batch_aborted(const KArgs& a) {
    if (!a.bad) return false;
    return *(const __attribute__((address_space(1))) uint32_t*)(uintptr_t)a.bad == a.bad_epoch;
}

// KArgs::key_mode.  kKeyNone: plain digest, or single-key HMAC when mid is
// set (lcb_hash_batch).  The others take key k = key_index[i]:
//   kKeyHmac    HMAC(K_k, m_i)            mid[k]: states after K^ipad, K^opad
//   kKeyPrefix  H(K_k || m_i)             mid[k]: state after K_k's whole blocks
//   kKeySuffix  H(m_i || K_k)
enum { kKeyNone = 0, kKeyHmac = 1, kKeyPrefix = 2, kKeySuffix = 3 };

// Fixed-stride batch of at least 64 16-B aligned records with at least one
// whole 128-B line each and a stride below 64 MiB: the shape the LDS-DMA
// line-stream kernels accept (LdsStridedStream: whole 64-record waves, one
// 32-bit per-lane offset up to 56 strides).
inline bool fixed_stride_lines(const KArgs& a) {
    return !a.offsets && !a.lengths && !a.order && (a.stride % 16) == 0 &&
           (reinterpret_cast<uintptr_t>(a.data) % 16) == 0 && a.fixed_len >= 128 && a.stride >= a.fixed_len &&
           a.count >= 64 && a.stride < (1ull << 26);
}

// Words reserved per HMAC mid-state (GOST needs 34: h, N, Sigma).
constexpr int kMidWords = 64;

// Short HMAC key, zero padded to 128 bytes, passed by value.
struct KeyBlock {
    uint32_t w[32];
};

// Bucket keys of ragged-batch bucketing (see lcb_kernels.hip): a length
// class (< 122) times 4 start phases: the start's dword inside its 16-B chunk,
// (start >> 2) & 3 (the tile kernel's uniform block-window shift).
constexpr int kBucketClasses = 122;
constexpr int kBucketPhases = 4;
constexpr int kBucketKeys = kBucketClasses * kBucketPhases;
// Bucketing scratch ahead of the permutation: per-key totals, a spare
// block, a spare word, the number of `order` entries (uint32 words).
// After the permutation: the per-block key counts, their per-block bases
// (bucket_blocks(count) x kBucketKeys words each) and one 16-bit key per
// message.
constexpr int kBucketHead = 2 * kBucketKeys;
constexpr int kBucketNTiles = 2 * kBucketKeys + 1;   // entries of `order`, pads included
// The one-kernel bucketing's synchronisation words (bucket_fused_kernel):
// zero between uses (its last block resets them; a fresh scratch buffer is
// zeroed once), then `order`.
constexpr int kBucketSync = 2 * kBucketKeys + 2;
constexpr int kBucketSyncWords = 64;
constexpr int kBucketWork = 2 * kBucketKeys + 2 + kBucketSyncWords;
// Groups of chunks of the one-kernel bucketing (at most kBucketGroupsMax):
// the last chunk counted in a group scans the group's counts.
constexpr uint32_t kBucketGroupsMax = 56;
// Messages per bucketing block: count / 1024, clamped to [4096, 8192] (the
// placement sorts a block's whole chunk in LDS).
constexpr uint64_t kBucketBlocksTarget = 1024;
constexpr uint64_t kBucketChunkMin = 4096;
constexpr uint64_t kBucketChunkMax = 8192;
inline uint64_t bucket_chunk(uint64_t count) {
    uint64_t c = (count + kBucketBlocksTarget - 1) / kBucketBlocksTarget;
    return c < kBucketChunkMin ? kBucketChunkMin : (c > kBucketChunkMax ? kBucketChunkMax : c);
}
inline uint64_t bucket_blocks(uint64_t count) { return (count + bucket_chunk(count) - 1) / bucket_chunk(count); }
// Ragged batches at least this large are bucketed by length first.
constexpr uint64_t kBucketMinCount = 4096;
// When every key has enough messages (count >= kBucketPadRatio * 64 * keys
// in use), each key's run of `order` is padded to a whole number of tiles
// with kOrderPad entries, so no tile mixes keys (at most 63 per key).
constexpr uint32_t kOrderPad = 0xffffffffu;
constexpr uint64_t kBucketPadRatio = 16;
// Largest ragged batch the uint32 permutation can describe, pads included.
constexpr uint64_t kBucketMaxCount = 0xffffffffull - 63ull * kBucketKeys;
// Words of `order`: the entries (count + at most 63 pads per key), rounded
// up to the tile kernel's whole grid, (count + 63) / 64 + kBucketKeys tiles
// of 64 -- it loads a tile's entries before it knows the entry count and
// ignores those past it.
inline size_t bucket_order_words(uint64_t count) { return (size_t)count + 64ull * (kBucketKeys + 1); }
// uint32 words of bucketing scratch for a batch of `count` messages:
// [work | permutation | per-block counts | per-block bases | 16-bit keys].
// Segmented long tiles (md_tiles.hpp): when a large batch's longest keys
// (records of at least kSegMinClass's length, 32 KiB) fill at least one
// generation of the tile kernel's wave slots, each of their tiles runs as
// kSegs jobs of a third of its lines, the state handed on through memory.
// The tile count of a batch is then kSegs x (long tiles) + the rest, fine
// enough to spread over the SIMDs: a long class of 5,461 tiles is 5.33
// tiles per SIMD, 6 when whole, 16 thirds when cut.
constexpr int kSegs = 3;
constexpr uint32_t kSegMinClass = 67;            // len_class: >= 512 blocks
constexpr uint32_t kSegStateWords = 16;          // hash state words saved per lane (SHA-512: 8 x 64 bits)
constexpr uint32_t kLinesOcc = 4;                // md_lines_kernel (SHA-384/512 ragged): waves per SIMD
constexpr uint64_t kSegMinCount = 131072;        // 2 x 4 x 256 SIMD slots of 64 records
// At most kSegMaxGens generations of the kernel's wave slots are cut (a
// longer class loses little to whole waves: ceil(n / S) against n / S); the
// scratch holds states for that many waves only, whatever the batch size
// (sizing them by the message count cost 64 B per message).
constexpr uint32_t kSegMaxGens = 4;
// Segment header words (a.seg[..]): the segmented waves (nseg), the wait
// before a take-over in 100-MHz ticks (0: kSegWaitTicks), 1 = jobs in
// reverse segment order (the take-over test, LCB_SEG_TAKEOVER); then one
// block per segmented wave: its saved states (kSegStateWords x 64 words,
// word-major) and its flag, in a 256-B line of its own.
constexpr uint32_t kSegHead = 64;
enum { kSegHdrCount = 0, kSegHdrWait = 1, kSegHdrReverse = 3 };
constexpr uint32_t kSegBlockWords = 64 * kSegStateWords + 64;
constexpr uint32_t kSegTaken = 0x80000000u;      // a wave's flag once a job took it over (seg_jobs.hpp)
__host__ __device__ inline uint64_t bucket_tiles_max(uint64_t count) { return (count + 63) / 64 + kBucketKeys; }
// Segmented-wave capacity of a batch (the tile kernel's or md_lines_kernel's
// wave slots `slots`): 0 below kSegMinCount.
inline uint32_t bucket_seg_cap(uint64_t count, uint32_t slots) {
    if (count < kSegMinCount || slots == 0) return 0;
    const uint64_t cap = (uint64_t)kSegMaxGens * slots, tiles = bucket_tiles_max(count);
    return (uint32_t)(cap < tiles ? cap : tiles);
}
inline size_t bucket_seg_words(uint32_t seg_cap) {
    return seg_cap ? (size_t)kSegHead + (size_t)seg_cap * kSegBlockWords : 0;
}
inline size_t bucket_seg_offset(uint64_t count) {
    const size_t w = (size_t)kBucketWork + bucket_order_words(count) + 2 * bucket_blocks(count) * kBucketKeys +
                     (count + 1) / 2 + (size_t)kBucketGroupsMax * kBucketKeys;   // ... group sums
    return (w + 63) / 64 * 64;
}
inline size_t bucket_words(uint64_t count, uint32_t seg_cap = 0) {
    return bucket_seg_offset(count) + bucket_seg_words(seg_cap);
}

// CRC-32 variants travel through the batch machinery as alg ids
// kCrcAlgBase + variant (variant ids of include/lcb_crc32_gpu.h).
constexpr int kCrcAlgBase = 100;
inline bool is_crc_alg(int alg) { return alg > kCrcAlgBase && alg <= kCrcAlgBase + 8; }

// Device-side description of one ChaCha batch (see include/lcb_chacha_gpu.h).
struct ChaArgs {
    const uint8_t* src = nullptr;         // nullptr: write the keystream itself
    uint8_t* dst = nullptr;
    const uint64_t* offsets = nullptr;    // nullptr: i * stride
    const uint32_t* lengths = nullptr;    // nullptr: fixed_len
    const uint64_t* blk_start = nullptr;  // ragged: exclusive block prefix (count + 1)
    const uint32_t* counters = nullptr;   // 2 LE words per buffer, nullptr: 0
    const uint32_t* ivs = nullptr;        // iv_words per buffer, nullptr: 0
    const uint32_t* subkeys = nullptr;    // xchacha: 8 words per buffer
    uint64_t count = 0, stride = 0;
    uint64_t total_blocks = 0;            // fixed layout: count * bpb
    uint32_t fixed_len = 0, bpb = 1;
    uint32_t iv_words = 2, iv_at = 0;     // chacha 2,0; xchacha 6,4
    uint32_t dr = 10;                     // double rounds = ceil(rounds / 2)
    uint32_t stream = 0;                  // dense aligned whole blocks: block g at byte 64 g
    uint32_t key[8] = {};                 // state words 4..11
    uint32_t cst[4] = {};                 // state words 0..3 of the block function
    uint32_t hcst[4] = {};                // state words 0..3 of hchacha (xchacha)
};

void launch_batch(int alg, const KArgs& a, hipStream_t s);
// Per-algorithm launchers, one translation unit each (k_<alg>.hip,
// gost_kernels.hip); launch_batch / launch_key_prep / launch_hmac_prep
// dispatch to them by alg id.
#define LCB_DECLARE_FAMILY(tag)                                                                       \
    void launch_plain_##tag(const KArgs& a, bool hmac, hipStream_t s);                               \
    void launch_keyed_##tag(const KArgs& a, hipStream_t s);                                          \
    void launch_key_prep_##tag(const KArgs& a, uint32_t* mid, hipStream_t s);                        \
    void launch_hmac_prep_##tag(const KeyBlock& kb, const uint8_t* dkey, uint64_t key_len, uint32_t* mid, \
                                hipStream_t s);
LCB_DECLARE_FAMILY(md5)
LCB_DECLARE_FAMILY(sha1)
LCB_DECLARE_FAMILY(sha224)
LCB_DECLARE_FAMILY(sha256)
LCB_DECLARE_FAMILY(sha384)
LCB_DECLARE_FAMILY(sha512)
LCB_DECLARE_FAMILY(gost256)
LCB_DECLARE_FAMILY(gost512)
#undef LCB_DECLARE_FAMILY
// ChaCha: ragged scan (parts: (count+1023)/1024 words, blk_start: count+1),
// xchacha subkey prep (subkeys: 8 words per buffer), then the block kernel.
void launch_chacha(const ChaArgs& a, uint64_t nparts, uint64_t* parts, uint64_t* blk_start,
                   uint32_t* subkeys, hipStream_t s);
void launch_crc(int variant, const KArgs& a, hipStream_t s);
void crc_table_host(int variant, uint32_t* out);
// Bucketing permutation of the ragged batch `a` (reads data/offsets/stride/
// lengths/count) into `order` (bucket_order_words(count) words); `work` =
// kBucketWork words (key totals, entry count).  tiles: the tile kernel's
// form, each key's run padded to whole tiles when the batch is large.
// seg_min > 0 (a.seg set): segment the waves of the longest keys when there
// are at least 1.25 x seg_min (wave slots) and at most a.seg_cap of them
// and cutting them evens the SIMDs' load (a.seg[0] = their count, else 0;
// their flags zeroed).  seg_test: the take-over test (jobs in reverse
// segment order, no wait before taking a tile over).
void launch_bucketing(const KArgs& a, uint32_t* work, uint32_t* order, bool tiles, uint32_t seg_min,
                      bool seg_test, hipStream_t s);
// The tile kernel's wave slots of alg on this device (0: no tile kernel).
uint32_t tile_slots(int alg);
// True when launch_batch(alg, a) runs the tile kernel on a bucketed batch:
// only then may `order` hold pad entries (every other kernel reads it per lane).
bool tiles_take(int alg, const KArgs& a);
void launch_hmac_prep(int alg, const KeyBlock& kb, const uint8_t* dkey, uint64_t key_len,
                      uint32_t* mid, hipStream_t s);
// Key-table prep of a keyed batch: mid[k] for every key (kKeyHmac, kKeyPrefix).
void launch_key_prep(int alg, const KArgs& a, uint32_t* mid, hipStream_t s);
void launch_gen(uint64_t seed, uint64_t start, uint8_t* out, uint64_t n, hipStream_t s);
// *bad |= 1 if any of idx[0..count) >= nkeys (bad zeroed by the caller).
// bad[0] = epoch if any of idx[0..count) >= nkeys.  With a pinned host word
// hbad: bad[1] counts the kernel's finished blocks (it holds ctr before the
// launch) and the last block writes epoch | (bad ? 1 << 31 : 0) to *hbad.
// Returns the kernel's block count (the host adds it to its ctr).
uint32_t launch_key_check(const uint32_t* idx, uint64_t count, uint32_t nkeys, uint32_t* bad, uint32_t* hbad,
                          uint32_t epoch, uint32_t ctr, hipStream_t s);
// HBM read probes (lcb_hash_gpu_read_probe): mode 0 = the fixed-stride line
// stream alone over `a`'s records, mode 1 = linear coalesced read of
// count * stride bytes; sink: one uint32 per record (0) / per thread (1).
void launch_probe(int mode, const KArgs& a, uint32_t* sink, hipStream_t s);
// mode 2: the plain GOST kernel's LDS gathers alone (count lanes, the LPS
// count of a fixed_len-byte message each); sink: one uint32 per lane.
void launch_gost_lps_probe(uint64_t count, uint32_t fixed_len, uint32_t* sink, hipStream_t s);
// lcb_hash_batch_multi device mode: the work-balanced split of a batch of
// `count` messages into nparts (<= 64) and each part's byte span, on `s`:
// res (device, 4 x 64 + 2 words) = [first 0..n | base 0..n-1 | end 0..n-1 |
// targets ... | ticket], bsum: (count + split_chunk - 1) / split_chunk
// words.  The first 3 n + 1 words land in hres (pinned, coherent host
// memory), then hres word 4 x 64 + 1 (as uint32) = epoch.
uint64_t split_chunk(uint64_t count);
void launch_multi_split(const uint32_t* lengths, const uint64_t* offsets, uint64_t stride, uint32_t fixed_len,
                        uint64_t count, uint32_t nparts, uint64_t* bsum, uint64_t* res, uint64_t* hres,
                        uint32_t epoch, hipStream_t s);
// lcb_hash_gpu_clock_stamp: `slots` one-wave workgroups, 3 uint64 each.
void launch_clock_stamp(uint64_t* out, uint32_t slots, hipStream_t s);
void gost_table_host(uint64_t* out);

// Shared by the C-ABI TUs (lcb_hash_gpu.cpp).
size_t dsize(int alg);                  // digest bytes, 0 for an unknown alg
size_t bsize(int alg);                  // block bytes (HMAC key block)
int map_err(hipError_t e);              // HIP error -> liblcb errno code
int ensure_init();                      // 0, or ENODEV without a usable device
int device_cu_count();                  // compute units of the current device (cached)
// Stream-ordered scratch from the library's own pool on the current device
// (one per device).  The pool reuses freed memory only on the stream that
// freed it: the default pool's cross-stream reuse handed one live
// bucketing buffer to two batches running concurrently on different streams
// (the ingestion queue's slots).  Memory stays in the pool.
hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t s);
hipError_t scratch_free(void* p, hipStream_t s);
// A call's hold on its device key table (lcb_hash_gpu.cpp key_table): a
// cache entry, pinned until released, or a per-call buffer.
struct KeyRef {
    void* entry = nullptr;
    uint8_t* temp = nullptr;
    size_t temp_bytes = 0;
};
// Once the batch that reads the keys is enqueued on `s`: a per-call buffer
// is zeroed and freed in stream order, a cache entry unpinned (async_use:
// the batch reads it later on `s`, so evicting it must wait for `s`).
void key_release(KeyRef& r, hipStream_t s, bool async_use);
// HMAC mid-states of one key, prepared on `s` and cached by the key's bytes;
// key_release(*ref) after the batch using them is enqueued.
int hmac_setup(int alg, const uint8_t* key, size_t key_len, hipStream_t s, const uint32_t** mid, KeyRef* ref);
// Batch kernel launch, bucketing a large ragged batch by length first.
// work_buf: optional caller-owned device buffer of bucket_words(count)
// uint32 for the bucketing of a ragged batch; null = stream-ordered allocation.
int launch_ordered(int alg, KArgs a, hipStream_t s, uint32_t* work_buf = nullptr);
// Words of a work_buf that serves any ragged plain batch of alg of up to
// `count` messages (segment states included where alg can be segmented).
size_t bucket_scratch_words(int alg, uint64_t count);

// The two batch paths of lcb_hash_batch (lcb_hash_gpu.cpp), on the current
// device.  batch_device enqueues on `s`; batch_host stages through `stage`
// (nullptr: the calling thread's own staging context).  `init`: CRC
// X_update() values (nullptr otherwise).
struct Stage;
// Key table of a keyed batch on the device (lcb_hash_batch_keyed), with the
// per-message key index kept where the caller gave it.
struct KeyTable {
    uint32_t mode = 0;                 // kKeyHmac / kKeyPrefix / kKeySuffix
    const uint8_t* keys = nullptr;     // device: packed key bytes
    const uint32_t* key_off = nullptr; // device
    const uint32_t* key_len = nullptr; // device
    uint32_t nkeys = 0;
    const uint32_t* mid = nullptr;     // device: 2 * kMidWords words per key
    const uint32_t* index = nullptr;   // per message (device or host memory, as the batch), or nullptr
};
// Key-index check of a keyed device batch (lcb_hash_batch_keyed): the flag
// word the check kernel sets to `epoch`, and the stream scratch the call
// holds (bucketing work words, reused by the batch).
struct KeyCheck {
    const uint32_t* dflag = nullptr;
    uint32_t epoch = 0;
    uint32_t* work = nullptr;
    size_t work_words = 0;
    // Non-null: the batch is bucketed and its count kernel runs the check
    // (one kernel less per keyed call); the result goes to this host word.
    uint32_t* fused_host = nullptr;
};
int batch_device(int alg, const uint8_t* key, size_t key_len, const uint8_t* data,
                 const uint64_t* offsets, const uint32_t* lengths, size_t count, uint64_t stride,
                 uint32_t fixed_len, uint8_t* digests, hipStream_t s, const uint32_t* init,
                 const KeyTable* kt = nullptr, const KeyCheck* kc = nullptr);
int batch_host(int alg, const uint8_t* key, size_t key_len, const uint8_t* data,
               const uint64_t* offsets, const uint32_t* lengths, size_t count, uint64_t stride,
               uint32_t fixed_len, uint8_t* digests, const uint32_t* init, Stage* stage,
               const KeyTable* kt = nullptr);
Stage* stage_acquire(int dev);      // pooled staging context (multi-device workers)
void stage_release(Stage* st);

// Host-memory helpers shared by the host-mode pipelines.
bool is_pinned(const void* p);  // page-locked (DMA-able) host memory
struct Piece {
    uint8_t* dst;
    const uint8_t* src;
    size_t n;
};
void parallel_copy(const std::vector<Piece>& pieces, size_t bytes);  // up to 8 threads

}  // namespace lcbgpu
