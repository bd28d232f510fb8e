// lcb_kernels.hip — dispatch of the batch digest kernels (one translation unit
// per algorithm: k_<alg>.hip, gost_kernels.hip) and the shared utility
// kernels: synthetic input, HBM read probes, length bucketing.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <algorithm>
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
    __shared__ __attribute__((aligned(16))) uint8_t slab[4][kSlabBytes];
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

// ------------------------------------------------- engine-clock stamps
// lcb_hash_gpu_clock_stamp: lane 0 of every one-wave workgroup writes
// {XCC_ID << 32 | HW_ID, s_memtime (shader cycles), s_memrealtime (100 MHz)}
// to out[3 b ..] (vector stores).  Two stamps launched on a stream around a
// run of kernels give the engine clock of that run per XCD: Δ cycles ÷
// Δ real time.  The workgroups are dealt round robin to the XCDs, so a grid
// of 8 k puts k on each.
__global__ __launch_bounds__(64) void clock_stamp_kernel(uint64_t* out) {
    if (threadIdx.x != 0) return;
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const uint64_t t = __builtin_amdgcn_s_memtime();
    const uint64_t r = __builtin_amdgcn_s_memrealtime();
    uint64_t* o = gptr(out) + 3ull * blockIdx.x;
    o[0] = ((uint64_t)xcc << 32) | hw;
    o[1] = t;
    o[2] = r;
}

void launch_clock_stamp(uint64_t* out, uint32_t slots, hipStream_t s) {
    hipLaunchKernelGGL(clock_stamp_kernel, dim3(slots), dim3(64), 0, s, out);
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

// A counting sort in three kernels with no global atomics (round 3's two
// kernels took 13 + 23.5 us on 1M packets, about 7 % of a packet pass, much
// of it the serialised per-key atomics of 512 blocks on a few hundred
// counters; profiles/r4_bucketing_ab.txt).  Block b of nb owns the
// contiguous chunk [b * chunk, (b + 1) * chunk):
//   bucket_count_kernel  key of every message (16 bits, kept for the last
//                        pass) and the block's key counts -> cnt[k][b]
//                        (key-major: one key's counts are contiguous);
//   bucket_base_kernel   one wave per key: base[k][b] = sum of cnt[k][b' < b]
//                        (coalesced loads, a wave scan), tot[k] = all of them;
//   bucket_place_kernel  every block scans the key totals in DESCENDING key
//                        order (one wave; runs padded to whole tiles for a
//                        large batch) and places its messages at
//                        start[k] + base[k][b] + rank (LDS atomics); block 0
//                        writes the pad entries and the entry count.
// Messages per thread in one unrolled step of the bucketing kernels (their
// loads issued together, not one round trip per message).
constexpr int kBucketUnroll = 4;

// kCheck: a keyed device batch's key-index check rides along (the indices
// are read with the lengths; a block that finds one >= nkeys sets *a.bad to
// the call's epoch) and bucket_base_kernel, the next kernel on the stream,
// reports the flag to the host word: one kernel launch less than
// key_index_check_kernel + bucketing (8.3 us per keyed packet pass).
template <bool kCheck>
__global__ __launch_bounds__(1024) void bucket_count_kernel(KArgs a, uint64_t chunk, uint32_t nb, uint32_t* cnt,
                                                           uint16_t* keys) {
    __shared__ uint32_t h[kBucketKeys];
    for (int c = threadIdx.x; c < kBucketKeys; c += blockDim.x) h[c] = 0;
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * chunk;
    const uint64_t hi = lo + chunk < a.count ? lo + chunk : a.count;
    bool bad = false;
    for (uint64_t i0 = lo + threadIdx.x; i0 < hi; i0 += kBucketUnroll * blockDim.x) {
        uint32_t k[kBucketUnroll], ki[kBucketUnroll];
#pragma unroll
        for (int u = 0; u < kBucketUnroll; ++u) {
            const uint64_t i = i0 + (uint64_t)u * blockDim.x;
            k[u] = i < hi ? bucket_key(a, i) : 0u;
            if constexpr (kCheck) ki[u] = i < hi ? gptr(a.key_index)[i] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kBucketUnroll; ++u) {
            const uint64_t i = i0 + (uint64_t)u * blockDim.x;
            if (i < hi) {
                gptr(keys)[i] = (uint16_t)k[u];
                atomicAdd(&h[k[u]], 1u);
                if constexpr (kCheck) bad |= ki[u] >= a.nkeys;
            }
        }
    }
    if constexpr (kCheck) {
        bad = __syncthreads_or(bad);
        if (bad && threadIdx.x == 0)
            __hip_atomic_store(const_cast<uint32_t*>(gptr(a.bad)), a.bad_epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    } else {
        __syncthreads();
    }
    for (int c = threadIdx.x; c < kBucketKeys; c += blockDim.x) gptr(cnt)[(uint64_t)c * nb + blockIdx.x] = h[c];
}

static_assert(kBucketKeys <= 1024, "one scan element per thread");

// Inclusive scan of v over the wave (6 ds_bpermute steps).
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t v, uint32_t lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t u = (uint32_t)__shfl_up((int)v, d, 64);
        if (lane >= (uint32_t)d) v += u;
    }
    return v;
}

// hbad: the fused key-index check's host word (bucket_count_kernel<true>):
// every count block has finished, so *bad is final; one system-scope
// release store of epoch | bad bit.
__global__ __launch_bounds__(256) void bucket_base_kernel(const uint32_t* cnt, uint32_t nb, uint32_t* base,
                                                          uint32_t* tot, const uint32_t* bad, uint32_t* hbad,
                                                          uint32_t epoch) {
    if (hbad && blockIdx.x == 0 && threadIdx.x == 0) {
        const uint32_t b = __hip_atomic_load(gptr(bad), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(hbad, epoch | (b == epoch ? 0x80000000u : 0u), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t k = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= (uint32_t)kBucketKeys) return;   // wave-uniform
    const uint32_t* c = gptr(cnt) + (uint64_t)k * nb;
    uint32_t* o = gptr(base) + (uint64_t)k * nb;
    uint32_t run = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += 256) {   // 4 counts per lane per round
        uint32_t v[4], s = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t b = b0 + 4 * lane + u;
            v[u] = b < nb ? c[b] : 0u;
            s += v[u];
        }
        const uint32_t incl = wave_scan_incl(s, lane);
        uint32_t e = run + incl - s;              // exclusive prefix of this lane's first count
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t b = b0 + 4 * lane + u;
            if (b < nb) o[b] = e;
            e += v[u];
        }
        run += (uint32_t)__shfl((int)incl, 63, 64);
    }
    if (lane == 0) gptr(tot)[k] = run;
}

// The block sorts its chunk by key in LDS first (local offsets from its own
// counts), then writes `order` in sorted order: consecutive threads write
// consecutive entries of one key's run, so a wave's 64 stores cover a few
// contiguous runs instead of 64 scattered dwords (each a partial-line write).
// kTiles: the tile kernel's form, runs padded to whole tiles (large
// batches).
static_assert(kBucketChunkMax <= 8192, "a block's chunk sorts in LDS");
template <bool kTiles>
__global__ __launch_bounds__(1024) void bucket_place_kernel(KArgs a, uint64_t chunk, uint32_t nb,
                                                            const uint32_t* cnt, const uint32_t* base,
                                                            const uint32_t* tot, const uint16_t* keys,
                                                            uint32_t* work, uint32_t* order, uint32_t seg_min,
                                                            uint32_t seg_simds, uint32_t* seg_flags, uint32_t seg_cap,
                                                            uint32_t seg_test) {
    __shared__ uint32_t h[kBucketKeys];        // run start in `order` of this block's entries, per key
    __shared__ uint32_t loc[kBucketKeys];      // local (sorted) offset per key, then the fill cursor
    __shared__ uint32_t len_s[kBucketKeys];
    __shared__ uint32_t sidx[kBucketChunkMax];
    __shared__ uint16_t skey[kBucketChunkMax];
    __shared__ uint32_t misc[2];
    const uint32_t t = threadIdx.x;
    const uint64_t lo = (uint64_t)blockIdx.x * chunk;
    const uint64_t hi = lo + chunk < a.count ? lo + chunk : a.count;
    // Every global load the block needs is issued here, together (the key
    // totals, this block's bases and counts, the first step's message keys):
    // one memory round trip instead of four in a row (r4: 10.4-11.9 us).
    const uint32_t hk = t < (uint32_t)kBucketKeys ? gptr(tot)[t] : 0u;
    const uint32_t bk = t < (uint32_t)kBucketKeys ? gptr(base)[(uint64_t)t * nb + blockIdx.x] : 0u;
    constexpr int kPer = (kBucketKeys + 63) / 64;
    uint32_t cv[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
        const int k = kPer * (int)(t - 64) + u;
        cv[u] = (t >= 64 && t < 128 && k < kBucketKeys) ? gptr(cnt)[(uint64_t)k * nb + blockIdx.x] : 0u;
    }
    uint32_t k0[kBucketUnroll];
#pragma unroll
    for (int u = 0; u < kBucketUnroll; ++u) {
        const uint64_t i = lo + t + (uint64_t)u * blockDim.x;
        k0[u] = i < hi ? gptr(keys)[i] : 0u;
    }
    // Padded run lengths, then one wave scans them in DESCENDING key order
    // (the longest class first): lane l owns keys K-1-8l .. K-8-8l; wave 1
    // scans the block's own counts (ascending: any order works locally).
    const int used = __syncthreads_count(hk != 0);
    const bool pad = kTiles && a.count >= kBucketPadRatio * 64 * (uint64_t)used;
    if (t < (uint32_t)kBucketKeys) len_s[t] = pad ? (hk + 63u) & ~63u : hk;
    __syncthreads();
    if (t < 64) {
        uint32_t v[kPer], s = 0;
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int k = kBucketKeys - 1 - (kPer * (int)t + u);
            v[u] = k >= 0 ? len_s[k] : 0u;
            s += v[u];
        }
        const uint32_t incl = wave_scan_incl(s, t);
        uint32_t e = incl - s;
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int k = kBucketKeys - 1 - (kPer * (int)t + u);
            if (k >= 0) h[k] = e;                // start of key k's run
            e += v[u];
        }
        if (t == 63) misc[0] = incl;             // entries of `order`, pads included
    } else if (t < 128) {
        const uint32_t l = t - 64;
        uint32_t s = 0;
#pragma unroll
        for (int u = 0; u < kPer; ++u) s += cv[u];
        uint32_t e = wave_scan_incl(s, l) - s;
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int k = kPer * (int)l + u;
            if (k < kBucketKeys) loc[k] = e;
            e += cv[u];
        }
    }
    __syncthreads();
    constexpr uint32_t kSegKey = kSegMinClass * kBucketPhases;
    static_assert(kSegKey >= 1 && kSegKey < (uint32_t)kBucketKeys, "segment class inside the key range");
    if (t < (uint32_t)kBucketKeys) {
        const uint32_t start = h[t];
        if (blockIdx.x == 0)
            for (uint32_t e = start + hk; e < start + len_s[t]; ++e) gptr(order)[e] = kOrderPad;
        // Segmented waves: the runs of every key >= kSegKey (the longest
        // classes) come first, so the first start / 64 waves hold only their
        // records (whole tiles when the runs are padded), the next one some.
        // Cut them only where it pays: n whole tiles over the SIMDs end at
        // ceil(n / simds) tiles per SIMD, thirds at ceil(3 n / simds) / 3
        // (5,461 tiles: 6 against 5.33); at least 1.25 generations of wave
        // slots, so a segment's predecessor has had a generation to finish
        // (4,096 MD5 tiles cut in thirds ran 17 % slower than whole).
        if (t == kSegKey - 1) {
            // (rounded up: an unpadded order's wave that mixes the last long
            // records with shorter ones is a job too -- segment 0 runs it
            // whole, at the front of the grid; left at the back of the
            // segmented jobs its 21 long records ran alone for 2 ms of C4.)
            const uint64_t n = (start + 63) / 64, sm = seg_simds ? seg_simds : 1;
            const uint64_t a0 = (n + sm - 1) / sm * sm, a3 = (kSegs * n + sm - 1) / sm * sm;
            const bool pays = 100 * kSegs * a0 > 103 * a3 && 4 * n >= 5 * (uint64_t)seg_min;
            misc[1] = (seg_min && seg_simds && pays && n <= seg_cap) ? (uint32_t)n : 0u;
        }
        // order position of the key's first local entry, minus its local offset
        h[t] = start + bk - loc[t];
    }
    if (blockIdx.x == 0 && t == 0) gptr(work)[kBucketNTiles] = misc[0];
    __syncthreads();
    if (seg_min) {
        // Every block zeroes its share of the segment flags (read by the
        // batch kernel, next on the stream); block 0 publishes the count.
        const uint32_t nseg = misc[1];
        for (uint32_t i = blockIdx.x * blockDim.x + t; i < nseg; i += nb * blockDim.x)
            gptr(seg_flags)[kSegHead + (uint64_t)i * kSegBlockWords + 64 * kSegStateWords] = 0u;
        if (blockIdx.x == 0 && t < 4) {
            const uint32_t hv[4] = {nseg, seg_test ? 1u : 0u, 0u, seg_test ? 1u : 0u};
            gptr(seg_flags)[t] = hv[t];   // kSegHdrCount, kSegHdrWait, (spare), kSegHdrReverse
        }
    }
    // chunk <= kBucketChunkMax (bucket_chunk): the whole chunk sorts in LDS.
    for (uint64_t i0 = lo + t; i0 < hi; i0 += kBucketUnroll * blockDim.x) {
        uint32_t k[kBucketUnroll];
        if (i0 == lo + t) {   // the first step's keys were loaded up front
#pragma unroll
            for (int u = 0; u < kBucketUnroll; ++u) k[u] = k0[u];
        } else {
#pragma unroll
            for (int u = 0; u < kBucketUnroll; ++u) {
                const uint64_t i = i0 + (uint64_t)u * blockDim.x;
                k[u] = i < hi ? gptr(keys)[i] : 0u;
            }
        }
#pragma unroll
        for (int u = 0; u < kBucketUnroll; ++u) {
            const uint64_t i = i0 + (uint64_t)u * blockDim.x;
            if (i < hi) {
                const uint32_t p = atomicAdd(&loc[k[u]], 1u);
                sidx[p] = (uint32_t)i;
                skey[p] = (uint16_t)k[u];
            }
        }
    }
    __syncthreads();
    const uint32_t n = (uint32_t)(hi - lo);
    for (uint32_t p = t; p < n; p += blockDim.x) gptr(order)[h[skey[p]] + p] = sidx[p];
}

// ------------------------------------------------ one-kernel bucketing
// The same counting sort as one kernel (the three
// kernels above spend 24.5 us per packet pass, most of it three kernels'
// fixed start and end costs).  Its blocks take work by TICKET, not by
// blockIdx: tickets 0..nb-1 count chunk t, tickets nb..2nb-1 place chunk
// t - nb.  A placing block waits for every chunk's count, and every count
// ticket was drawn before any place ticket, i.e. by a block that is
// running (counting never waits): no grid size or co-residency can
// deadlock it.  Chunks form `ng` groups of G; the block that counts a
// group's last chunk scans the group's counts (per key: the exclusive
// prefix over the group's chunks, and the group total), so what is serial
// after the last count is one group's scan; each placing block adds the
// group totals itself (ng x 488 words), recomputes its messages' keys
// (12 B of offset + length each, rather than a key array written by one
// block and read by another) and then places as bucket_place_kernel.
// Cross-block words (counts, prefixes, group totals) move as agent-scope
// atomic stores and loads, each writer waiting for its stores (vmcnt)
// before it bumps a counter -- no release / acquire fences, which write
// back and invalidate a whole XCD's L2 each (a first form with them ran the
// packet pass 120 us slower).  The sync words (kBucketSync: ticket, groups
// done, one counter per group) are zero at entry; the block that draws the
// last ticket of all resets them.
struct BucketSync {
    uint32_t* w;
    __device__ uint32_t* ticket() const { return w; }
    __device__ uint32_t* groups_done() const { return w + 1; }
    __device__ uint32_t* group(uint32_t g) const { return w + 8 + g; }
};
static_assert(8 + kBucketGroupsMax <= (uint32_t)kBucketSyncWords, "sync words");

__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
    __hip_atomic_store(gptr(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
    return __hip_atomic_load(const_cast<uint32_t*>(gptr(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool kTiles, bool kCheck>
__global__ __launch_bounds__(1024) void bucket_fused_kernel(KArgs a, uint64_t chunk, uint32_t nb, uint32_t G,
                                                            uint32_t ng, uint32_t* cnt, uint32_t* inb, uint32_t* gsum,
                                                            uint32_t* work, uint32_t* order, uint32_t seg_min,
                                                            uint32_t seg_simds, uint32_t* seg_flags, uint32_t seg_cap,
                                                            uint32_t seg_test) {
    __shared__ uint32_t h[kBucketKeys];        // count: histogram; place: run start of this chunk's entries
    __shared__ uint32_t loc[kBucketKeys];      // place: local (sorted) offset per key, then the fill cursor
    __shared__ uint32_t len_s[kBucketKeys];
    __shared__ uint32_t sidx[kBucketChunkMax];
    __shared__ uint16_t skey[kBucketChunkMax];
    __shared__ uint32_t misc[4];
    const uint32_t t = threadIdx.x;
    const BucketSync sy{gptr(work) + kBucketSync};
    constexpr int kPer = (kBucketKeys + 63) / 64;
    for (;;) {
        if (t == 0) misc[2] = __hip_atomic_fetch_add(sy.ticket(), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const uint32_t tk = misc[2];
        __syncthreads();
        if (tk >= 2 * nb) {
            // Every block draws exactly one ticket past the work; the one
            // that draws the last leaves the sync words zero for the next use
            // (no other block touches them any more).
            if (tk == 2 * nb + gridDim.x - 1 && t < (uint32_t)kBucketSyncWords) st_agent(sy.w + t, 0u);
            return;
        }
        const uint32_t c = tk < nb ? tk : tk - nb;
        const uint64_t lo = (uint64_t)c * chunk;
        const uint64_t hi = lo + chunk < a.count ? lo + chunk : a.count;
        const uint32_t g = c / G;
        if (tk < nb) {
            // ------------------------------------------------ count chunk c
            for (uint32_t k = t; k < (uint32_t)kBucketKeys; k += blockDim.x) h[k] = 0;
            __syncthreads();
            bool bad = false;
            for (uint64_t i0 = lo + t; i0 < hi; i0 += kBucketUnroll * blockDim.x) {
                uint32_t k[kBucketUnroll], ki[kBucketUnroll];
#pragma unroll
                for (int u = 0; u < kBucketUnroll; ++u) {
                    const uint64_t i = i0 + (uint64_t)u * blockDim.x;
                    k[u] = i < hi ? bucket_key(a, i) : 0u;
                    if constexpr (kCheck) ki[u] = i < hi ? gptr(a.key_index)[i] : 0u;
                }
#pragma unroll
                for (int u = 0; u < kBucketUnroll; ++u) {
                    const uint64_t i = i0 + (uint64_t)u * blockDim.x;
                    if (i < hi) {
                        atomicAdd(&h[k[u]], 1u);
                        if constexpr (kCheck) bad |= ki[u] >= a.nkeys;
                    }
                }
            }
            if constexpr (kCheck) {
                bad = __syncthreads_or(bad);
                if (bad && t == 0) st_agent(const_cast<uint32_t*>(a.bad), a.bad_epoch);
            } else {
                __syncthreads();
            }
            for (uint32_t k = t; k < (uint32_t)kBucketKeys; k += blockDim.x)
                st_agent(cnt + (uint64_t)c * kBucketKeys + k, h[k]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's stores done
            __syncthreads();                                    // ... and every thread's
            const uint32_t gsz = (g + 1) * G <= nb ? G : nb - g * G;
            if (t == 0)
                misc[3] = __hip_atomic_fetch_add(sy.group(g), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 == gsz;
            __syncthreads();
            if (!misc[3]) continue;
            // The group's last chunk: per key, the exclusive prefix over the
            // group's chunks (inb) and the group total (gsum).
            if (t < (uint32_t)kBucketKeys) {
                uint32_t v[16];
                uint32_t run = 0;
                for (uint32_t j0 = 0; j0 < gsz; j0 += 16) {   // 16 loads in flight per thread
#pragma unroll
                    for (int u = 0; u < 16; ++u)
                        v[u] = j0 + u < gsz ? ld_agent(cnt + (uint64_t)(g * G + j0 + u) * kBucketKeys + t) : 0u;
#pragma unroll
                    for (int u = 0; u < 16; ++u) {
                        if (j0 + u < gsz) st_agent(inb + (uint64_t)(g * G + j0 + u) * kBucketKeys + t, run);
                        run += v[u];
                    }
                }
                st_agent(gsum + (uint64_t)g * kBucketKeys + t, run);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (t == 0) {
                const uint32_t done = __hip_atomic_fetch_add(sy.groups_done(), 1u, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT) + 1;
                if (kCheck && done == ng && a.check_host) {
                    // every chunk counted: the fused key-index check is final
                    const uint32_t bv = ld_agent(a.bad);
                    __hip_atomic_store(a.check_host, a.bad_epoch | (bv == a.bad_epoch ? 0x80000000u : 0u),
                                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
            continue;
        }
        // ------------------------------------------------ place chunk c
        // This chunk's first keys do not depend on the other chunks: their
        // loads go out before the wait.  (A safety valve, never reached by a
        // well-formed launch: after 1 s -- 10^8 ticks of the 100 MHz clock
        // -- the block gives its chunk up rather than spin for ever, so a
        // corrupted sync word cannot hang the GPU; the last block still
        // resets the words.)
        uint32_t k0[kBucketUnroll];
#pragma unroll
        for (int u = 0; u < kBucketUnroll; ++u) {
            const uint64_t i = lo + t + (uint64_t)u * blockDim.x;
            k0[u] = i < hi ? bucket_key(a, i) : 0u;
        }
        if (t == 0) {
            misc[3] = 0;
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            uint32_t spins = 0;
            while (ld_agent(sy.groups_done()) < ng) {
                if (++spins > 4) __builtin_amdgcn_s_sleep(2);
                if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {
                    misc[3] = 1;
                    break;
                }
            }
        }
        __syncthreads();
        if (misc[3]) {
            __syncthreads();
            continue;
        }
        // Per key: this chunk's count, the total (all groups) and this
        // chunk's base (the groups before its own, plus its prefix inside it).
        // (16 loads in flight per thread: the group totals are ng rows)
        uint32_t hk = 0, bk = 0, ck = 0;
        if (t < (uint32_t)kBucketKeys) {
            ck = ld_agent(cnt + (uint64_t)c * kBucketKeys + t);
            bk = ld_agent(inb + (uint64_t)c * kBucketKeys + t);
            for (uint32_t q0 = 0; q0 < ng; q0 += 16) {
                uint32_t v[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) v[u] = q0 + u < ng ? ld_agent(gsum + (uint64_t)(q0 + u) * kBucketKeys + t) : 0u;
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    hk += v[u];
                    bk += q0 + u < g ? v[u] : 0u;
                }
            }
        }
        // (from here as bucket_place_kernel, chunk c)
        const int used = __syncthreads_count(hk != 0);
        const bool pad = kTiles && a.count >= kBucketPadRatio * 64 * (uint64_t)used;
        if (t < (uint32_t)kBucketKeys) {
            len_s[t] = pad ? (hk + 63u) & ~63u : hk;
            loc[t] = ck;     // this chunk's counts (scanned below)
        }
        __syncthreads();
        if (t < 64) {
            uint32_t v[kPer], sm = 0;
#pragma unroll
            for (int u = 0; u < kPer; ++u) {
                const int k = kBucketKeys - 1 - (kPer * (int)t + u);
                v[u] = k >= 0 ? len_s[k] : 0u;
                sm += v[u];
            }
            const uint32_t incl = wave_scan_incl(sm, t);
            uint32_t e = incl - sm;
#pragma unroll
            for (int u = 0; u < kPer; ++u) {
                const int k = kBucketKeys - 1 - (kPer * (int)t + u);
                if (k >= 0) h[k] = e;
                e += v[u];
            }
            if (t == 63) misc[0] = incl;
        } else if (t < 128) {
            const uint32_t l = t - 64;
            uint32_t cv[kPer], sm = 0;
#pragma unroll
            for (int u = 0; u < kPer; ++u) {
                const int k = kPer * (int)l + u;
                cv[u] = k < kBucketKeys ? loc[k] : 0u;
                sm += cv[u];
            }
            uint32_t e = wave_scan_incl(sm, l) - sm;
#pragma unroll
            for (int u = 0; u < kPer; ++u) {
                const int k = kPer * (int)l + u;
                if (k < kBucketKeys) loc[k] = e;
                e += cv[u];
            }
        }
        __syncthreads();
        constexpr uint32_t kSegKey = kSegMinClass * kBucketPhases;
        if (t < (uint32_t)kBucketKeys) {
            const uint32_t start = h[t];
            if (c == 0)
                for (uint32_t e = start + hk; e < start + len_s[t]; ++e) gptr(order)[e] = kOrderPad;
            if (t == kSegKey - 1) {
                const uint64_t n = (start + 63) / 64, sm = seg_simds ? seg_simds : 1;
                const uint64_t a0 = (n + sm - 1) / sm * sm, a3 = (kSegs * n + sm - 1) / sm * sm;
                const bool pays = 100 * kSegs * a0 > 103 * a3 && 4 * n >= 5 * (uint64_t)seg_min;
                misc[1] = (seg_min && seg_simds && pays && n <= seg_cap) ? (uint32_t)n : 0u;
            }
            h[t] = start + bk - loc[t];
        }
        if (c == 0 && t == 0) gptr(work)[kBucketNTiles] = misc[0];
        __syncthreads();
        if (seg_min) {
            const uint32_t nseg = misc[1];
            for (uint32_t i = c * blockDim.x + t; i < nseg; i += nb * blockDim.x)
                gptr(seg_flags)[kSegHead + (uint64_t)i * kSegBlockWords + 64 * kSegStateWords] = 0u;
            if (c == 0 && t < 4) {
                const uint32_t hv[4] = {nseg, seg_test ? 1u : 0u, 0u, seg_test ? 1u : 0u};
                gptr(seg_flags)[t] = hv[t];
            }
        }
        for (uint64_t i0 = lo + t; i0 < hi; i0 += kBucketUnroll * blockDim.x) {
            uint32_t k[kBucketUnroll];
            if (i0 == lo + t) {
#pragma unroll
                for (int u = 0; u < kBucketUnroll; ++u) k[u] = k0[u];
            } else {
#pragma unroll
                for (int u = 0; u < kBucketUnroll; ++u) {
                    const uint64_t i = i0 + (uint64_t)u * blockDim.x;
                    k[u] = i < hi ? bucket_key(a, i) : 0u;
                }
            }
#pragma unroll
            for (int u = 0; u < kBucketUnroll; ++u) {
                const uint64_t i = i0 + (uint64_t)u * blockDim.x;
                if (i < hi) {
                    const uint32_t p = atomicAdd(&loc[k[u]], 1u);
                    sidx[p] = (uint32_t)i;
                    skey[p] = (uint16_t)k[u];
                }
            }
        }
        __syncthreads();
        const uint32_t n = (uint32_t)(hi - lo);
        for (uint32_t p = t; p < n; p += blockDim.x) gptr(order)[h[skey[p]] + p] = sidx[p];
        __syncthreads();
    }
}

void launch_bucketing(const KArgs& a, uint32_t* work, uint32_t* order, bool tiles, uint32_t seg_min, bool seg_test,
                      hipStream_t s) {
    // work: [tot | spare | spare | entry count] then `order`
    // (bucket_order_words), then cnt, base (nb x kBucketKeys each) and the
    // 16-bit keys; every word the kernels read is written
    // first by an earlier kernel of the three (no memset).
    const uint64_t chunk = bucket_chunk(a.count);
    const uint32_t nb = (uint32_t)bucket_blocks(a.count);
    uint32_t* cnt = order + bucket_order_words(a.count);
    uint32_t* base = cnt + (uint64_t)nb * kBucketKeys;
    uint16_t* keys = reinterpret_cast<uint16_t*>(base + (uint64_t)nb * kBucketKeys);
    // LCB_BUCKET_FUSED=1 in the environment: the one-kernel form.  Not the
    // default: same-process A/Bs with rocprofv3 kernel traces measured it at
    // 26.3 us median per 1M-packet bucketing against 25.1 for the three
    // kernels (profiles/r7_bucket_fused_ab.txt) -- the serial
    // chain inside one kernel (count, a group's scan, the wait, the place)
    // costs what the two kernel boundaries cost.
    const char* fe = getenv("LCB_BUCKET_FUSED");
    if (fe && fe[0] == '1') {
        uint32_t* gsum = reinterpret_cast<uint32_t*>(keys) + (a.count + 1) / 2;
        uint32_t G = 1;
        while (G * G < nb) ++G;                                            // ~sqrt(nb) chunks per group
        if ((nb + G - 1) / G > kBucketGroupsMax) G = (nb + kBucketGroupsMax - 1) / kBucketGroupsMax;
        const uint32_t ng = (nb + G - 1) / G;
        const uint32_t simds = 4u * (uint32_t)device_cu_count();
        // one block per CU (97 VGPRs x 16 waves: one 1,024-thread block fits a
        // CU): each block then counts a chunk and places one, and only the
        // grid's own blocks draw the exit tickets (a grid of 2 nb dispatched
        // a second round of blocks just to exit)
        const uint32_t grid = std::min<uint32_t>(nb, (uint32_t)device_cu_count());
        const uint32_t sm = a.seg ? seg_min : 0u, st = seg_test ? 1u : 0u;
#define LCB_FUSED(T, C)                                                                                      \
    hipLaunchKernelGGL((bucket_fused_kernel<T, C>), dim3(grid), dim3(1024), 0, s, a, chunk, nb, G, ng, cnt, base, \
                       gsum, work, order, sm, simds, a.seg, a.seg_cap, st)
        if (tiles) {
            if (a.check_host) LCB_FUSED(true, true); else LCB_FUSED(true, false);
        } else {
            if (a.check_host) LCB_FUSED(false, true); else LCB_FUSED(false, false);
        }
#undef LCB_FUSED
        return;
    }
    if (a.check_host)
        hipLaunchKernelGGL(bucket_count_kernel<true>, dim3(nb), dim3(1024), 0, s, a, chunk, nb, cnt, keys);
    else
        hipLaunchKernelGGL(bucket_count_kernel<false>, dim3(nb), dim3(1024), 0, s, a, chunk, nb, cnt, keys);
    hipLaunchKernelGGL(bucket_base_kernel, dim3((kBucketKeys + 3) / 4), dim3(256), 0, s, cnt, nb, base, work, a.bad,
                       a.check_host, a.bad_epoch);
    if (!a.seg) seg_min = 0;
    const uint32_t simds = 4u * (uint32_t)device_cu_count();
    if (tiles)
        hipLaunchKernelGGL(bucket_place_kernel<true>, dim3(nb), dim3(1024), 0, s, a, chunk, nb, cnt, base, work, keys,
                           work, order, seg_min, simds, a.seg, a.seg_cap, seg_test ? 1u : 0u);
    else
        hipLaunchKernelGGL(bucket_place_kernel<false>, dim3(nb), dim3(1024), 0, s, a, chunk, nb, cnt, base, work, keys,
                           work, order, seg_min, simds, a.seg, a.seg_cap, seg_test ? 1u : 0u);
}

uint32_t tile_slots(int alg) {
    // 4 SIMDs per CU x the batch kernel's waves per SIMD: the tile kernel's,
    // md_lines_kernel's for SHA-384/512, the plain GOST kernels'.
    uint32_t occ = 0;
    switch (alg) {
    case 1: occ = Md5::kTileOcc; break;
    case 2: occ = Sha1::kTileOcc; break;
    case 3: occ = Sha256<true>::kTileOcc; break;
    case 4: occ = Sha256<false>::kTileOcc; break;
    case 5:
    case 6: occ = kLinesOcc; break;
    case 7:
    case 8: occ = 4; break;   // gost_plain2_kernel / gost_seg_kernel: 2 x 512-thread workgroups per CU
    default: break;
    }
    return occ * 4u * (uint32_t)device_cu_count();
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

// Keyed batches, device mode: flags an out-of-range key index (lcb_hash_batch_keyed
// returns EINVAL then and no digest is written, as in host mode).  The flag
// takes the call's epoch, so it needs no clearing between calls; it gates
// the batch's digest stores (batch_aborted).  With a host word: every block
// counts itself in bad[1] (agent-scope acq_rel add: the last block sees
// every earlier block's flag store), and the last one writes the result to
// the pinned host word with a system-scope store -- the host polls that word
// instead of recording an event (6.5 us of stream time each).
__global__ __launch_bounds__(256) void key_index_check_kernel(const uint32_t* idx, uint64_t count, uint32_t nkeys,
                                                              uint32_t* bad, uint32_t* hbad, uint32_t epoch,
                                                              uint32_t target) {
    bool any = false;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 7 * step < count; i += 8 * step) {   // 8 independent loads in flight
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = gptr(idx)[i + u * step];
#pragma unroll
        for (int u = 0; u < 8; ++u) any |= v[u] >= nkeys;
    }
    for (; i < count; i += step) any |= gptr(idx)[i] >= nkeys;
    any = __syncthreads_or(any);
    if (threadIdx.x != 0) return;
    if (any) __hip_atomic_store(gptr(bad), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!hbad) return;
    const uint32_t done = __hip_atomic_fetch_add(gptr(bad) + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1;
    if (done != target) return;
    const uint32_t b = __hip_atomic_load(gptr(bad), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(hbad, epoch | (b == epoch ? 0x80000000u : 0u), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

uint32_t launch_key_check(const uint32_t* idx, uint64_t count, uint32_t nkeys, uint32_t* bad, uint32_t* hbad,
                          uint32_t epoch, uint32_t ctr, hipStream_t s) {
    // Few blocks: each ends in one agent-scope acq_rel add on one counter
    // (1,024 blocks took 28 us, 128 take a few: the adds serialise).
    uint64_t blocks = (count + 2047) / 2048;
    const uint64_t cap = (uint64_t)device_cu_count() / 2;
    if (blocks > cap) blocks = cap;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(key_index_check_kernel, dim3((unsigned)blocks), dim3(256), 0, s, idx, count, nkeys, bad, hbad,
                       epoch, ctr + (uint32_t)blocks);
    return (uint32_t)blocks;
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


// ------------------------------------- multi-device split on the home device
// lcb_hash_batch_multi, device mode: the work-balanced
// split of a ragged batch (lcb_hash_partition's rule: first[p] is the first
// message whose work midpoint, prefix + (len + 64) / 2, reaches p/N of the
// total work) and each part's byte span [min offset, max offset + length),
// computed where the offsets and lengths are, into `res` (uint64):
//   [0, n]          first[0..n]
//   [n+1, 2n]       base[p] (UINT64_MAX for an empty part)
//   [2n+1, 3n]      end[p]
//   [3n+1, 4n)      targets T_1..T_{n-1} (internal)
// Three kernels: per-block work sums, one block scanning them (totals,
// targets, initial values), then each block recomputing its messages'
// prefixes, the part of every message (targets in LDS) and the spans (LDS
// reduction, one global min / max per part per block).  Without lengths
// every message costs the same: first[] is the equal-count split (as the
// host rule) and only the spans are computed.
constexpr uint32_t kSplitThreads = 1024;

__device__ __forceinline__ uint64_t split_work(const uint32_t* lengths, uint32_t fixed_len, uint64_t i) {
    return (uint64_t)(lengths ? gptr(lengths)[i] : fixed_len) + 64u;
}

__global__ __launch_bounds__(kSplitThreads) void split_sum_kernel(const uint32_t* lengths, uint32_t fixed_len,
                                                                  uint64_t count, uint64_t chunk, uint64_t* bsum) {
    __shared__ uint64_t red[kSplitThreads / 64];
    const uint64_t lo = (uint64_t)blockIdx.x * chunk;
    const uint64_t hi = lo + chunk < count ? lo + chunk : count;
    uint64_t s = 0;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += kSplitThreads) s += split_work(lengths, fixed_len, i);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += (uint64_t)__shfl_xor((unsigned long long)s, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (uint32_t k = 0; k < kSplitThreads / 64; ++k) t += red[k];
        gptr(bsum)[blockIdx.x] = t;
    }
}

// One block: bsum[b] -> exclusive prefix (in place); res initialised.
__global__ __launch_bounds__(kSplitThreads) void split_scan_kernel(uint64_t* bsum, uint32_t nb, uint64_t count,
                                                                   uint32_t n, bool ragged, uint64_t* res) {
    __shared__ uint64_t part[kSplitThreads];
    const uint32_t t = threadIdx.x;
    const uint64_t v = t < nb ? gptr(bsum)[t] : 0;   // nb <= kSplitThreads
    part[t] = v;
    __syncthreads();
    for (uint32_t d = 1; d < kSplitThreads; d <<= 1) {   // Hillis-Steele inclusive scan
        const uint64_t x = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
    if (t < nb) gptr(bsum)[t] = part[t] - v;
    const uint64_t W = part[kSplitThreads - 1];
    uint64_t* r = gptr(res);
    if (t <= n) r[t] = t == 0 ? 0 : (ragged || t == n ? count : (count / n) * t + (count % n) * t / n);
    if (t < n) {
        r[n + 1 + t] = ~0ull;
        r[2 * n + 1 + t] = 0;
    }
    if (t >= 1 && t < n) {   // T_t = floor(W t / n), exactly: (W / n) t + (W % n) t / n
        r[3 * n + t] = (W / n) * t + (W % n) * t / n;
    }
    if (t == 0) r[4 * 64 + 1] = 0;   // the place kernel's ticket
}

__global__ __launch_bounds__(kSplitThreads) void split_place_kernel(const uint32_t* lengths, const uint64_t* offsets,
                                                                    uint64_t stride, uint32_t fixed_len,
                                                                    uint64_t count, uint64_t chunk,
                                                                    const uint64_t* bbase, uint32_t n, uint64_t* res,
                                                                    uint32_t* ticket, uint64_t* hres, uint32_t epoch) {
    __shared__ uint64_t tg[64];         // targets T_1..T_{n-1} (ragged) or first[0..n] (equal work)
    __shared__ unsigned long long lmin[64], lmax[64];
    __shared__ uint64_t wsum[kSplitThreads / 64];
    __shared__ uint64_t carry_s;
    const uint32_t t = threadIdx.x;
    const bool ragged = lengths != nullptr;
    uint64_t* r = gptr(res);
    if (t < 64) {
        tg[t] = ragged ? (t >= 1 && t < n ? r[3 * n + t] : 0) : (t <= n ? r[t] : count);
        lmin[t] = ~0ull;
        lmax[t] = 0;
    }
    if (t == 0) carry_s = gptr(bbase)[blockIdx.x];
    __syncthreads();
    // part of message i: ragged, the targets at or below its midpoint m;
    // equal work, the last p with first[p] <= i
    auto part_of = [&](uint64_t key) {
        uint32_t p = 0;
        for (uint32_t k = 1; k < n; ++k) p += tg[k] <= key;
        return p;
    };
    const uint64_t lo = (uint64_t)blockIdx.x * chunk;
    const uint64_t hi = lo + chunk < count ? lo + chunk : count;
    for (uint64_t i0 = lo; i0 < hi; i0 += kSplitThreads) {
        const uint64_t i = i0 + t;
        const bool in = i < hi;
        const uint64_t w = in ? split_work(lengths, fixed_len, i) : 0;
        // block-wide inclusive scan of w (wave scan + wave totals)
        uint64_t x = w;
        const uint32_t lane = t & 63;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = (uint64_t)__shfl_up((unsigned long long)x, d, 64);
            if (lane >= (uint32_t)d) x += y;
        }
        if (lane == 63) wsum[t >> 6] = x;
        __syncthreads();
        uint64_t before = carry_s;
        for (uint32_t k = 0; k < (t >> 6); ++k) before += wsum[k];
        const uint64_t acc = before + x - w;       // work prefix of message i
        __syncthreads();
        if (t == kSplitThreads - 1) carry_s = before + x;
        if (in) {
            const uint32_t pi = part_of(ragged ? acc + w / 2 : i);
            // first[p] = i for the parts (part(i - 1), part(i)]
            uint32_t pp = 0;
            if (i > 0) {
                if (ragged) {
                    const uint64_t wp = split_work(lengths, fixed_len, i - 1);
                    pp = part_of(acc - wp + wp / 2);
                } else {
                    pp = part_of(i - 1);
                }
            }
            if (ragged)
                for (uint32_t p = pp + 1; p <= pi; ++p) r[p] = i;
            const uint64_t off = offsets ? gptr(offsets)[i] : i * stride;
            const uint64_t len = lengths ? gptr(lengths)[i] : fixed_len;
            atomicMin(&lmin[pi], (unsigned long long)off);
            atomicMax(&lmax[pi], (unsigned long long)(off + len));
        }
        __syncthreads();
    }
    if (t < n && lmin[t] != ~0ull) {
        atomicMin(reinterpret_cast<unsigned long long*>(gptr(r) + n + 1 + t), lmin[t]);
        atomicMax(reinterpret_cast<unsigned long long*>(gptr(r) + 2 * n + 1 + t), lmax[t]);
    }
    // The last block to finish hands the result to the host's pinned,
    // coherent buffer (system-scope stores, then the call's epoch released
    // after them): the host polls one word instead of a copy command and
    // an event (host time per call).
    __shared__ uint32_t last_s;
    __syncthreads();
    if (t == 0) {
        __threadfence();
        last_s = __hip_atomic_fetch_add(gptr(ticket), 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1 == gridDim.x;
    }
    __syncthreads();
    if (!last_s) return;
    __threadfence();
    if (t <= 3 * n)
        __hip_atomic_store(hres + t, __hip_atomic_load(gptr(r) + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    if (t == 0) {
        __threadfence_system();
        __hip_atomic_store(reinterpret_cast<uint32_t*>(hres + 4 * 64 + 1), epoch, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

uint64_t split_chunk(uint64_t count) {
    uint64_t c = (count + kSplitThreads - 1) / kSplitThreads;
    if (c < 8192) c = 8192;
    return (c + kSplitThreads - 1) / kSplitThreads * kSplitThreads;
}

void launch_multi_split(const uint32_t* lengths, const uint64_t* offsets, uint64_t stride, uint32_t fixed_len,
                        uint64_t count, uint32_t nparts, uint64_t* bsum, uint64_t* res, uint64_t* hres,
                        uint32_t epoch, hipStream_t s) {
    const uint64_t chunk = split_chunk(count);
    const uint32_t nb = (uint32_t)((count + chunk - 1) / chunk);
    hipLaunchKernelGGL(split_sum_kernel, dim3(nb), dim3(kSplitThreads), 0, s, lengths, fixed_len, count, chunk, bsum);
    hipLaunchKernelGGL(split_scan_kernel, dim3(1), dim3(kSplitThreads), 0, s, bsum, nb, count, nparts,
                       lengths != nullptr, res);
    hipLaunchKernelGGL(split_place_kernel, dim3(nb), dim3(kSplitThreads), 0, s, lengths, offsets, stride, fixed_len,
                       count, chunk, bsum, nparts, res, reinterpret_cast<uint32_t*>(res + 4 * 64 + 1), hres, epoch);
}

}  // namespace lcbgpu
