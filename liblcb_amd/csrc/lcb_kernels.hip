// lcb_kernels.hip — dispatch of the batch digest kernels (one translation unit
// per algorithm: k_<alg>.hip, gost_kernels.hip) and the shared utility
// kernels: synthetic input, HBM read probes, length bucketing.
#include <hip/hip_runtime.h>
#include "hash_device.hpp"
#include "lcb_internal.hpp"

namespace lcbgpu {

// ------------------------------------------------------ synthetic input
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// Thread t writes stream word (start/8 + t) — the bytes of it that fall in
// [start, start + n) — to out[word*8 - start ...].
__global__ __launch_bounds__(256) void gen_kernel(uint64_t seed, uint64_t start, uint8_t* out, uint64_t n) {
    const uint64_t w0 = start >> 3;
    const uint64_t nw = ((start + n + 7) >> 3) - w0;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nw;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t word = w0 + t;
        const uint64_t v = mix64(seed ^ word);
        const uint64_t b0 = word << 3;
        if (b0 >= start && b0 + 8 <= start + n && ((reinterpret_cast<uintptr_t>(out + (b0 - start)) & 7u) == 0)) {
            *reinterpret_cast<uint64_t*>(out + (b0 - start)) = v;
        } else {
            for (int k = 0; k < 8; ++k) {
                const uint64_t b = b0 + k;
                if (b >= start && b < start + n) out[b - start] = (uint8_t)(v >> (8 * k));
            }
        }
    }
}

// ------------------------------------------------- HBM read probes
// Achievable read bandwidth on the box, measured beside the
// digest kernels by bench.py: no compression, the same bytes.
//   records: md_fixed_lds_kernel's stream exactly (LdsStridedStream over
//            fixed-stride records, 4 waves x 5 workgroups per CU, one line in
//            flight per wave), each lane folding its 128 B into one word;
//   linear:  plain coalesced 16-B-per-lane loads over the whole range, 4 in
//            flight per lane, grid of 8 workgroups per CU (8 in flight
//            measured slower: 5.3 against 5.6 TB/s).
// One uint32 per record / per thread goes to `sink` so nothing is dead.
__global__ __launch_bounds__(256) void probe_records_kernel(KArgs a, uint32_t* sink) {
    __shared__ __attribute__((aligned(16))) uint8_t slab[4][8192];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint64_t wave_first = ((uint64_t)blockIdx.x * 4 + wv) * 64;
    if (wave_first >= a.count) return;
    const uint64_t last = a.count - 1;
    const uint32_t skip = wave_first + 63 > last ? (uint32_t)(wave_first + 63 - last) : 0u;
    wave_first -= skip;
    const uint64_t nlines = a.fixed_len / 128;
    LdsStridedStream ls;
    ls.init(a.data, a.stride, wave_first, lane, &slab[wv][0]);
    uint32_t acc = 0;
    if (nlines) ls.issue(0);
    for (uint64_t L = 0; L < nlines; ++L) {
        uint32_t w[32];
        ls.take(w, w + 16);
        if (L + 1 < nlines) ls.issue(L + 1);
#pragma unroll
        for (int k = 0; k < 32; k += 2) acc = xor3(acc, w[k], w[k + 1]);
    }
    if (lane >= skip) gptr(sink)[wave_first + lane] = acc;
}

typedef unsigned int probe_v4u __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void probe_linear_kernel(const probe_v4u* data, uint64_t n16, uint32_t* sink) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    uint64_t i = tid;
    for (; i + 3 * nth < n16; i += 4 * nth) {
        probe_v4u v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = __builtin_nontemporal_load(gptr(data) + i + k * nth);
#pragma unroll
        for (int k = 0; k < 4; ++k) acc = xor3(acc, xor3(v[k].x, v[k].y, v[k].z), v[k].w);
    }
    for (; i < n16; i += nth) {
        const probe_v4u v = gptr(data)[i];
        acc = xor3(acc, xor3(v.x, v.y, v.z), v.w);
    }
    gptr(sink)[tid] = acc;
}

void launch_probe(int mode, const KArgs& a, uint32_t* sink, hipStream_t s) {
    if (mode == 0) {
        hipLaunchKernelGGL(probe_records_kernel, dim3((unsigned)((a.count + 255) / 256)), dim3(256), 0, s, a, sink);
    } else {
        const uint64_t n16 = a.count * a.stride / 16;
        hipLaunchKernelGGL(probe_linear_kernel, dim3((unsigned)(8 * device_cu_count())), dim3(256), 0, s,
                           reinterpret_cast<const probe_v4u*>(a.data), n16, sink);
    }
}

// ---------------------------------------------------- length bucketing
// Ragged batches: lanes of one wavefront run until the longest lane's message
// is done, so a random mix of 64 B and 64 KiB messages would make almost
// every wave as slow as a 64 KiB one.  These kernels compute a permutation
// `order` that groups messages by key = length class x start phase, highest
// key (longest class) first (a counting sort; order inside a key is arbitrary
// and does not affect any digest, which is always written at the message's
// own index):
//   class(len) = nb for nb = len/64 + 1 < 64, else 58 + floor(log2(nb))
//   (exact block counts up to 4 KiB, power-of-two bins above), and
//   phase     = (start >> 2) & 3: the start's dword inside its 16-B chunk,
//               which the tile kernel's block window needs uniform per wave
//               (the rest of the start's offset inside its 128-B line is
//               applied per lane: md_tiles.hpp).
// Tiles of 64 consecutive `order` entries then share their key.  For a large
// batch every key's run is padded to whole tiles with kOrderPad entries.
__device__ __forceinline__ uint32_t len_class(uint64_t len) {
    const uint64_t nb = (len >> 6) + 1;
    if (nb < 64) return (uint32_t)nb;
    return 58u + (63u - (uint32_t)__clzll((long long)nb));
}

__device__ __forceinline__ uint32_t bucket_key(const KArgs& a, uint64_t i) {
    const uint64_t off = a.offsets ? gptr(a.offsets)[i] : i * a.stride;
    const uint32_t p = (uint32_t)(reinterpret_cast<uintptr_t>(a.data) + off);
    return len_class(gptr(a.lengths)[i]) * kBucketPhases + ((p >> 2) & 3u);
}

// Few, large blocks (kBucketBlocks x 1024 threads): every block adds its LDS
// histogram to the global one with one atomic per key it saw, and the
// atomics on a hot key serialise (one word takes ~88 per us,
// MI355X_MICROARCH.md): 4096 blocks of 256 cost ~50 us on a 3-length batch.
constexpr uint32_t kBucketBlocks = 512;

__global__ __launch_bounds__(1024) void bucket_hist_kernel(KArgs a, uint32_t* hist) {
    __shared__ uint32_t h[kBucketKeys];
    for (int c = threadIdx.x; c < kBucketKeys; c += blockDim.x) h[c] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.count;
         i += (uint64_t)gridDim.x * blockDim.x)
        atomicAdd(&h[bucket_key(a, i)], 1u);
    __syncthreads();
    for (int c = threadIdx.x; c < kBucketKeys; c += blockDim.x)
        if (h[c]) atomicAdd(&hist[c], h[c]);
}

static_assert(kBucketKeys <= 1024, "one scan element per thread");

// Block b owns the contiguous chunk [b * chunk, (b + 1) * chunk).  Every block
// derives the start of each key's run (DESCENDING key order, runs padded to
// whole tiles when the batch is large) from the global histogram with one
// 1024-wide LDS scan, counts its own keys, reserves one range per key (fill
// counter atomics), then places its indices (LDS atomics give the rank inside
// the block's range).  Block 0 also writes the pad entries and the tile count.
__global__ __launch_bounds__(1024) void bucket_scatter_kernel(KArgs a, const uint32_t* hist, uint32_t* fill,
                                                             uint32_t* ntiles, uint32_t* order, uint64_t chunk,
                                                             bool allow_pad) {
    __shared__ uint32_t h[kBucketKeys];
    __shared__ uint32_t base[1024];
    const uint32_t t = threadIdx.x;
    // Scan element t = key kBucketKeys - 1 - t (descending), padded count.
    const int kt = (int)kBucketKeys - 1 - (int)t;
    const uint32_t hk = kt >= 0 ? hist[kt] : 0u;
    const int used = __syncthreads_count(hk != 0);
    const bool pad = allow_pad && a.count >= kBucketPadRatio * 64 * (uint64_t)used;
    const uint32_t len = pad ? (hk + 63u) & ~63u : hk;
    base[t] = len;
    for (int c = t; c < kBucketKeys; c += blockDim.x) h[c] = 0;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {     // inclusive scan (Hillis-Steele)
        const uint32_t v = t >= d ? base[t - d] : 0u;
        __syncthreads();
        base[t] += v;
        __syncthreads();
    }
    const uint32_t start = base[t] - len;          // exclusive
    __syncthreads();
    if (kt >= 0) {
        if (blockIdx.x == 0) {
            for (uint32_t e = start + hk; e < start + len; ++e) order[e] = kOrderPad;
            if (t == 0) *ntiles = base[1023];   // entries of `order`, pads included
        }
        base[t] = start;                           // base of key kt at scan slot t
    }
    const uint64_t lo = (uint64_t)blockIdx.x * chunk;
    const uint64_t hi = lo + chunk < a.count ? lo + chunk : a.count;
    for (uint64_t i = lo + t; i < hi; i += blockDim.x) atomicAdd(&h[bucket_key(a, i)], 1u);
    __syncthreads();
    for (int k = t; k < kBucketKeys; k += blockDim.x) {
        const uint32_t slot = (uint32_t)(kBucketKeys - 1 - k);
        if (h[k]) base[slot] += atomicAdd(&fill[k], h[k]);
        h[k] = 0;
    }
    __syncthreads();
    for (uint64_t i = lo + t; i < hi; i += blockDim.x) {
        const uint32_t k = bucket_key(a, i);
        order[base[kBucketKeys - 1 - k] + atomicAdd(&h[k], 1u)] = (uint32_t)i;
    }
}

void launch_bucketing(const KArgs& a, uint32_t* work, uint32_t* order, bool allow_pad, hipStream_t s) {
    // work: histogram | fill counters | tile-queue head | tile count, zeroed
    // here; order: bucket_words(count) - kBucketWork uint32.
    // Rounded up to 16 B: one fill kernel instead of a body and a tail (the
    // bytes past kBucketWork are `order` entries the scatter writes anyway).
    (void)hipMemsetAsync(work, 0, (kBucketWork * sizeof(uint32_t) + 15) & ~(size_t)15, s);
    uint64_t nb = (a.count + 1023) / 1024;
    if (nb > kBucketBlocks) nb = kBucketBlocks;
    const uint64_t chunk = (a.count + nb - 1) / nb;
    hipLaunchKernelGGL(bucket_hist_kernel, dim3((unsigned)nb), dim3(1024), 0, s, a, work);
    hipLaunchKernelGGL(bucket_scatter_kernel, dim3((unsigned)((a.count + chunk - 1) / chunk)), dim3(1024), 0, s, a,
                       work, work + kBucketKeys, work + kBucketNTiles, order, chunk, allow_pad);
}

// ------------------------------------------------------------- dispatch
#define LCB_ALG_SWITCH(fn, ...)                                   \
    switch (alg) {                                                \
    case 1: fn##_md5(__VA_ARGS__); break;                         \
    case 2: fn##_sha1(__VA_ARGS__); break;                        \
    case 3: fn##_sha224(__VA_ARGS__); break;                      \
    case 4: fn##_sha256(__VA_ARGS__); break;                      \
    case 5: fn##_sha384(__VA_ARGS__); break;                      \
    case 6: fn##_sha512(__VA_ARGS__); break;                      \
    case 7: fn##_gost256(__VA_ARGS__); break;                     \
    case 8: fn##_gost512(__VA_ARGS__); break;                     \
    default: break;                                               \
    }

// Keyed batches, device mode: flags an out-of-range key index before the
// batch runs (lcb_hash_batch_keyed returns EINVAL then and writes no digest,
// as host mode does).  One global atomic OR per offending lane.
__global__ __launch_bounds__(256) void key_index_check_kernel(const uint32_t* idx, uint64_t count, uint32_t nkeys,
                                                              uint32_t* bad) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count;
         i += (uint64_t)gridDim.x * blockDim.x)
        if (gptr(idx)[i] >= nkeys) __hip_atomic_fetch_or(gptr(bad), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

void launch_key_check(const uint32_t* idx, uint64_t count, uint32_t nkeys, uint32_t* bad, hipStream_t s) {
    uint64_t blocks = (count + 255) / 256;
    const uint64_t cap = (uint64_t)4 * device_cu_count();
    if (blocks > cap) blocks = cap;
    hipLaunchKernelGGL(key_index_check_kernel, dim3((unsigned)(blocks ? blocks : 1)), dim3(256), 0, s, idx, count,
                       nkeys, bad);
}

// The hashes with a tile kernel (kTileOcc > 0): MD5, SHA-1, SHA-224/256.
static_assert(Md5::kTileOcc > 0 && Sha1::kTileOcc > 0 && Sha256<true>::kTileOcc > 0 &&
                  Sha256<false>::kTileOcc > 0 && Sha512<true>::kTileOcc == 0 && Sha512<false>::kTileOcc == 0,
              "tiles_take must list exactly the hashes with a tile kernel");

bool tiles_take(int alg, const KArgs& a) {
    // Their plain, HMAC, keyed HMAC and keyed suffix batches (md_kernels.hpp
    // launch_md*) run the tile kernel: its runs are padded to whole tiles.
    return alg >= 1 && alg <= 4 && a.key_mode != kKeyPrefix;
}

void launch_key_prep(int alg, const KArgs& a, uint32_t* mid, hipStream_t s) {
    LCB_ALG_SWITCH(launch_key_prep, a, mid, s)
}

void launch_batch(int alg, const KArgs& a, hipStream_t s) {
    if (a.key_mode != kKeyNone) {
        LCB_ALG_SWITCH(launch_keyed, a, s)
        return;
    }
    if (is_crc_alg(alg)) {
        launch_crc(alg - kCrcAlgBase, a, s);
        return;
    }
    const bool hmac = a.mid != nullptr;
    LCB_ALG_SWITCH(launch_plain, a, hmac, s)
}

void launch_hmac_prep(int alg, const KeyBlock& kb, const uint8_t* dkey, uint64_t key_len,
                      uint32_t* mid, hipStream_t s) {
    LCB_ALG_SWITCH(launch_hmac_prep, kb, dkey, key_len, mid, s)
}

void launch_gen(uint64_t seed, uint64_t start, uint8_t* out, uint64_t n, hipStream_t s) {
    const uint64_t nw = ((start + n + 7) >> 3) - (start >> 3);
    uint64_t blocks = (nw + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(gen_kernel, dim3((unsigned)blocks), dim3(256), 0, s, seed, start, out, n);
}

}  // namespace lcbgpu
