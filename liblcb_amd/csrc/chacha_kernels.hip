// chacha_kernels.hip — batched ChaCha / XChaCha (include/lcb_chacha_gpu.h)
// for gfx950.
//
// Unlike the digests, ChaCha is a counter-mode keystream: every 64-byte
// block of every buffer is independent (chacha.h:423-446 — the state only
// differs in the 64-bit block counter).  So the unit of work is a BLOCK, not
// a buffer.
//
// chacha_lane_kernel (the product): ONE LANE PER BLOCK, the whole 4x4 state
// in 16 VGPRs, 80 quarter rounds with 4-way ILP inside the lane and no
// cross-lane traffic — the minimum VALU work per block.  Register-only
// throughput (tools/cha_core.hip on MI355X) is ~0.41-0.45 ms of ChaCha20 per
// GiB whatever the layout, so ChaCha20 is VALU-bound and ChaCha8/12 are
// HBM-bound.  For the memory side, a dense batch of whole aligned blocks
// (the bench layout) takes the STREAM path: the wave's 64 blocks = 4 KiB
// are read and written by four coalesced 1 KiB instructions (16 B per
// lane), and the keystream is redistributed lane-per-block -> lane-per-16-B
// through a bank-conflict-free swizzled LDS slab.  Other layouts (ragged,
// misaligned, partial blocks) go through per-lane 16-B / dword-slot /
// byte paths.  Waves grid-stride over 64-block tiles, a few tiles each, and
// every wave's exit condition is the block total it reads.
//
// A four-lanes-per-block formulation (DPP quad rotations, round 1) ran at
// the same register-only VALU rate with more per-block overhead (0.59-0.67
// ms ChaCha20 against 0.55); it is gone from the source (git history,
// profiles/r1_chacha_bench_v*.txt).
//
// Block -> buffer: fixed-length batches divide once per wave and then step
// (bpb blocks per buffer); ragged batches search an exclusive prefix of
// blocks per buffer built on the device by chacha_scan_* (a 64-ary wave
// search for the tile's first buffer, then a short per-lane gallop).
//
// Buffers at any byte alignment: 16-B aligned full slices use dwordx4; other
// slices use aligned dword slots with v_alignbyte funnel shifts and byte
// stores only at the buffer edges.  No byte outside a described buffer is
// read past its containing dword, and none is written.
#include <hip/hip_runtime.h>

#include "hash_device.hpp"
#include "lcb_internal.hpp"


namespace lcbgpu {

// Double-round counts up to this prefetch the next tile's input while the
// current one computes (the short ciphers are HBM-bound; ChaCha20 is not).
constexpr int kChaPrefetchMaxDr = 6;

// chacha.h:125-130
__device__ __forceinline__ void cha_qr(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
    a += b; d = rotl32(d ^ a, 16);
    c += d; b = rotl32(b ^ c, 12);
    a += b; d = rotl32(d ^ a, 8);
    c += d; b = rotl32(b ^ c, 7);
}

// Whole-state double round in one lane (hchacha prep).
__device__ __forceinline__ void cha_dround_full(uint32_t* x) {
    cha_qr(x[0], x[4], x[8], x[12]); cha_qr(x[1], x[5], x[9], x[13]);
    cha_qr(x[2], x[6], x[10], x[14]); cha_qr(x[3], x[7], x[11], x[15]);
    cha_qr(x[0], x[5], x[10], x[15]); cha_qr(x[1], x[6], x[11], x[12]);
    cha_qr(x[2], x[7], x[8], x[13]); cha_qr(x[3], x[4], x[9], x[14]);
}

// ----------------------------------------------------------- hchacha prep
// xchacha: subkey_i = hchacha(key, iv_i[0:16]) (chacha.h:361-401), one lane
// per buffer; the block kernel then runs chacha with that 256-bit key.
__global__ __launch_bounds__(256) void hchacha_kernel(ChaArgs a, uint32_t* subkeys) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.count) return;
    uint32_t x[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = a.hcst[k];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[4 + k] = a.key[k];
    const uint32_t* iv = a.ivs ? gptr(a.ivs) + i * a.iv_words : nullptr;
#pragma unroll
    for (int k = 0; k < 4; ++k) x[12 + k] = iv ? iv[k] : 0u;
    for (uint32_t r = 0; r < a.dr; ++r) cha_dround_full(x);
    uint32_t* o = gptr(subkeys) + i * 8;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        o[k] = x[k];
        o[4 + k] = x[12 + k];
    }
}

// ------------------------------------------------- ragged: block prefix
// blk_start[i] = sum_{k<i} ceil(len_k / 64), blk_start[count] = total.
// Three passes of 1024 buffers per workgroup (4 per thread).
constexpr int kScanPer = 1024;

__device__ __forceinline__ uint64_t blocks_of(uint32_t len) { return ((uint64_t)len + 63u) >> 6; }

// Inclusive scan of one value per thread over the 256-thread workgroup.
__device__ __forceinline__ uint64_t wg_inclusive_scan(uint64_t v, uint64_t* sh) {
    sh[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t d = 1; d < 256; d <<= 1) {
        const uint64_t add = threadIdx.x >= d ? sh[threadIdx.x - d] : 0u;
        __syncthreads();
        v += add;
        sh[threadIdx.x] = v;
        __syncthreads();
    }
    return v;
}

__global__ __launch_bounds__(256) void chacha_scan_reduce(const uint32_t* lengths, uint64_t count,
                                                          uint64_t* parts) {
    __shared__ uint64_t sh[256];
    const uint64_t base = (uint64_t)blockIdx.x * kScanPer + threadIdx.x * 4u;
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (base + k < count) s += blocks_of(gptr(lengths)[base + k]);
    const uint64_t inc = wg_inclusive_scan(s, sh);
    if (threadIdx.x == 255) gptr(parts)[blockIdx.x] = inc;
}

// One workgroup: exclusive scan of the per-workgroup sums, in place.
__global__ __launch_bounds__(256) void chacha_scan_parts(uint64_t* parts, uint64_t nparts) {
    __shared__ uint64_t sh[256];
    uint64_t carry = 0;
    for (uint64_t b = 0; b < nparts; b += 256) {
        const uint64_t i = b + threadIdx.x;
        const uint64_t v = i < nparts ? gptr(parts)[i] : 0u;
        const uint64_t inc = wg_inclusive_scan(v, sh);
        if (i < nparts) gptr(parts)[i] = carry + inc - v;
        carry += sh[255];
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void chacha_scan_final(const uint32_t* lengths, uint64_t count,
                                                         const uint64_t* parts, uint64_t* blk_start) {
    __shared__ uint64_t sh[256];
    const uint64_t base = (uint64_t)blockIdx.x * kScanPer + threadIdx.x * 4u;
    uint64_t b[4], s = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        b[k] = base + k < count ? blocks_of(gptr(lengths)[base + k]) : 0u;
        s += b[k];
    }
    const uint64_t inc = wg_inclusive_scan(s, sh);
    uint64_t run = gptr(parts)[blockIdx.x] + inc - s;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (base + k < count) gptr(blk_start)[base + k] = run;
        run += b[k];
        if (base + k + 1 == count) gptr(blk_start)[count] = run;
    }
}

// ------------------------------------------------------------ block kernel
// Ragged batches: largest i with blk_start[i] <= g0 for a wave-uniform g0
// (blk_start[count] = total > g0; a zero-length buffer shares its start with
// the next one and is skipped).  64-ary search: each step the wave loads 64
// evenly spaced prefix entries of the live interval and a ballot picks the
// sub-interval, so 1M buffers take 4 vector loads instead of 20 dependent
// ones.
__device__ __forceinline__ uint64_t cha_wave_search(const uint64_t* bs, uint64_t count, uint64_t g0,
                                                    uint32_t lane) {
    uint64_t lo = 0, hi = count;
    while (hi - lo > 1) {
        const uint64_t step = (hi - lo + 63) >> 6;
        const uint64_t idx = lo + (uint64_t)lane * step;
        const bool le = idx < hi && bs[idx] <= g0;  // a prefix of the lanes (bs is sorted)
        const uint32_t k = (uint32_t)__popcll(__ballot(le)) - 1u;  // lane 0 always qualifies
        lo = lo + (uint64_t)k * step;
        const uint64_t nh = lo + step;
        hi = nh < hi ? nh : hi;
    }
    return lo;
}

// Per lane: the buffer holding block g >= blk_start[lo], galloping forward
// from the tile's first buffer then bisecting (blocks of one tile are
// consecutive, so the distance is small unless many buffers are empty).
__device__ __forceinline__ uint64_t cha_lane_search(const uint64_t* bs, uint64_t count, uint64_t lo, uint64_t g) {
    uint64_t hi = count;
    for (uint64_t s = 1;; s <<= 1) {
        const uint64_t c = lo + s;
        if (c >= count) break;
        if (bs[c] > g) {
            hi = c;
            break;
        }
        lo = c;
    }
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (bs[mid] <= g) lo = mid; else hi = mid;
    }
    return lo;
}

// XOR keystream slice K (bytes [0,16) of the lane's slice) into dst[0, n)
// (src NULL: store K itself), at any alignment, touching only those bytes.
__device__ __forceinline__ void cha_store_slice(uint8_t* d, const uint8_t* s, uint32_t n, const uint32_t K[4]) {
    const uintptr_t ad = reinterpret_cast<uintptr_t>(d), as = reinterpret_cast<uintptr_t>(s);
    if (n == 16 && ((ad | as) & 15u) == 0) {
        uint4 v = s ? *reinterpret_cast<const uint4*>(s) : make_uint4(0, 0, 0, 0);
        v.x ^= K[0]; v.y ^= K[1]; v.z ^= K[2]; v.w ^= K[3];
        *reinterpret_cast<uint4*>(d) = v;
        return;
    }
    if (s && ((ad ^ as) & 3u)) {  // src and dst misaligned differently: bytes
        for (uint32_t b = 0; b < n; ++b) d[b] = s[b] ^ (uint8_t)(K[b >> 2] >> (8u * (b & 3u)));
        return;
    }
    // Dword slots k = 0..4 of the aligned window starting at d - sh.  Slot k
    // holds slice bytes [4k - sh, 4k - sh + 4).
    const uint32_t sh = (uint32_t)(ad & 3u);
    uint8_t* db = d - sh;
    const uint8_t* sb = s ? s - sh : nullptr;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const int first = 4 * k - (int)sh;
        const int lo = first < 0 ? 0 : first;
        const int hi = (first + 4) < (int)n ? first + 4 : (int)n;
        if (lo >= hi) continue;
        const uint32_t kh = k < 4 ? K[k] : 0u, kl = k > 0 ? K[k - 1] : 0u;
        const uint32_t kw = sh ? __builtin_amdgcn_alignbyte(kh, kl, 4u - sh) : kh;
        const uint32_t v = (sb ? *reinterpret_cast<const uint32_t*>(sb + 4 * k) : 0u) ^ kw;
        if (lo == first && hi == first + 4) {
            *reinterpret_cast<uint32_t*>(db + 4 * k) = v;
        } else {
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (first + b >= lo && first + b < hi) db[4 * k + b] = (uint8_t)(v >> (8 * b));
        }
    }
}

// ------------------------------------------------- lane-per-block kernel
// One lane per 64-byte block: the whole 4x4 state in 16 VGPRs, no
// cross-lane traffic.  Per block this is the minimum VALU work (80 quarter
// rounds, 4-way ILP inside the lane) — the quad/DPP kernel above spends
// ~30-50 % more VALU per block on DPP-carrying ops and its transpose.  The
// src block is loaded before the rounds so its latency hides behind them.
template <int DR>
__global__ __launch_bounds__(256) void chacha_lane_kernel(ChaArgs a) {
    __shared__ uint4 cha_lds[4][256];  // per wave: 64 blocks x 4 slices of keystream
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave0 = (uint64_t)blockIdx.x * (blockDim.x >> 6) +
                           (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    uint64_t total = a.total_blocks;
    if (a.lengths) {
        const uint64_t tv = gptr(a.blk_start)[a.count];
        total = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(tv >> 32)) << 32) |
                (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)tv);
    }
    constexpr uint64_t kTile = 64;
    const uint64_t bpb = a.bpb;
    const uint64_t gstep = nwaves * kTile;
    uint64_t buf0 = 0, jb0 = 0, sdiv = 0, smod = 0;
    if (!a.lengths) {
        if (total <= 0xffffffffull && gstep <= 0xffffffffull) {  // wave-uniform: 32-bit divisions
            const uint32_t q0 = (uint32_t)(wave0 * kTile) / (uint32_t)bpb, q1 = (uint32_t)gstep / (uint32_t)bpb;
            buf0 = q0;
            sdiv = q1;
        } else {
            buf0 = (wave0 * kTile) / bpb;
            sdiv = gstep / bpb;
        }
        jb0 = wave0 * kTile - buf0 * bpb;
        smod = gstep - sdiv * bpb;
    }
    for (uint64_t t = wave0; t * kTile < total; t += nwaves) {
        const uint64_t g0 = t * kTile;
        uint64_t g = g0 + lane, buf, jb;
        const bool live = g < total;
        if (!live) g = total - 1;
        if (a.lengths) {
            buf0 = cha_wave_search(gptr(a.blk_start), a.count, g0, lane);
            buf = cha_lane_search(gptr(a.blk_start), a.count, buf0, g);
            jb = g - gptr(a.blk_start)[buf];
        } else if (bpb >= kTile) {
            jb = jb0 + lane;
            buf = buf0;
            if (jb >= bpb) {
                jb -= bpb;
                ++buf;
            }
            if (buf >= a.count) buf = a.count - 1;
        } else {
            const uint32_t r = (uint32_t)jb0 + lane;
            const uint32_t k = r / (uint32_t)bpb;
            buf = buf0 + k;
            jb = r - k * (uint32_t)bpb;
            if (buf >= a.count) buf = a.count - 1;
        }
        const uint64_t off = a.offsets ? gptr(a.offsets)[buf] : buf * a.stride;
        const uint64_t len = a.lengths ? (uint64_t)gptr(a.lengths)[buf] : (uint64_t)a.fixed_len;
        const uint64_t p = jb * 64u;
        const uint32_t n = (live && len > p) ? (uint32_t)(len - p < 64u ? len - p : 64u) : 0u;
        uint8_t* dp = gptr(a.dst) + off + p;
        const uint8_t* sp = a.src ? gptr(a.src) + off + p : nullptr;
        // Stream tile (wave-uniform): the batch is one dense 16-B aligned run
        // of whole blocks (block g at byte 64 g) and this tile is full, so
        // the wave's 4 KiB are read and written by 4 coalesced 1 KiB
        // instructions (lane l <-> bytes 1024 k + 16 l); the keystream is
        // redistributed through LDS (below).
        const bool stream = a.stream && g0 + kTile <= total;
        const bool fast = !stream && n == 64 &&
                          ((reinterpret_cast<uintptr_t>(dp) | reinterpret_cast<uintptr_t>(sp)) & 15u) == 0;
        // Prefetch the source before the rounds when they are short (the
        // memory-bound ChaCha8/12); for long rounds load after them and keep
        // the 16 VGPRs for occupancy instead.
        constexpr bool kPrefetch = DR != 0 && DR <= kChaPrefetchMaxDr;
        uint4 in[4] = {};
        if (kPrefetch && stream && a.src) {
            const uint4* sb = reinterpret_cast<const uint4*>(gptr(a.src) + g0 * 64u);
#pragma unroll
            for (int k = 0; k < 4; ++k) in[k] = sb[64 * k + lane];
        } else if (kPrefetch && fast && sp) {
#pragma unroll
            for (int k = 0; k < 4; ++k) in[k] = reinterpret_cast<const uint4*>(sp)[k];
        }
        // State (chacha.h:69-75): constants, key, 64-bit counter + jb, IV.
        uint32_t s[16], x[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) s[k] = a.cst[k];
        if (a.subkeys) {
            const uint4* sk = reinterpret_cast<const uint4*>(gptr(a.subkeys) + 8 * buf);
            const uint4 u = sk[0], v = sk[1];
            s[4] = u.x; s[5] = u.y; s[6] = u.z; s[7] = u.w;
            s[8] = v.x; s[9] = v.y; s[10] = v.z; s[11] = v.w;
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) s[4 + k] = a.key[k];
        }
        uint64_t ctr = jb;
        if (a.counters) {
            const uint32_t* c = gptr(a.counters) + 2 * buf;
            ctr += (uint64_t)c[0] | ((uint64_t)c[1] << 32);
        }
        s[12] = (uint32_t)ctr;
        s[13] = (uint32_t)(ctr >> 32);
        if (a.ivs) {
            const uint32_t* iv = gptr(a.ivs) + buf * a.iv_words + a.iv_at;
            s[14] = iv[0];
            s[15] = iv[1];
        } else {
            s[14] = s[15] = 0u;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = s[k];
        if (DR) {
#pragma unroll
            for (int r = 0; r < DR; ++r) cha_dround_full(x);
        } else {
            for (uint32_t r = 0; r < a.dr; ++r) cha_dround_full(x);
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] += s[k];  // chacha.h:143-161
        if (stream) {
            // Keystream block `lane`, slice i -> LDS slot 4 lane + (i ^ h),
            // h = (lane >> 1) & 3: conflict-free for the 8-lane groups of
            // ds_write_b128 and for the 16-lane groups of ds_read_b128 below
            // (MI355X_MICROARCH.md LDS lane groups).  Wave-private region.
            uint4* L = cha_lds[threadIdx.x >> 6];
            const uint32_t h = (lane >> 1) & 3u;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                L[4 * lane + ((uint32_t)i ^ h)] = make_uint4(x[4 * i], x[4 * i + 1], x[4 * i + 2], x[4 * i + 3]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (!kPrefetch && a.src) {
                const uint4* sb = reinterpret_cast<const uint4*>(gptr(a.src) + g0 * 64u);
#pragma unroll
                for (int k = 0; k < 4; ++k) in[k] = sb[64 * k + lane];
            }
            uint4* db = reinterpret_cast<uint4*>(gptr(a.dst) + g0 * 64u);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t b = 16u * k + (lane >> 2), sl = lane & 3u;
                const uint4 kv = L[4 * b + (sl ^ ((b >> 1) & 3u))];
                uint4 v = in[k];
                v.x ^= kv.x; v.y ^= kv.y; v.z ^= kv.z; v.w ^= kv.w;
                db[64 * k + lane] = v;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else if (fast) {
            if (!kPrefetch && sp) {
#pragma unroll
                for (int k = 0; k < 4; ++k) in[k] = reinterpret_cast<const uint4*>(sp)[k];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint4 v = in[k];
                v.x ^= x[4 * k]; v.y ^= x[4 * k + 1]; v.z ^= x[4 * k + 2]; v.w ^= x[4 * k + 3];
                reinterpret_cast<uint4*>(dp)[k] = v;
            }
        } else if (n) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int nk = (int)n - 16 * k;
                if (nk > 0) cha_store_slice(dp + 16 * k, sp ? sp + 16 * k : nullptr, nk < 16 ? nk : 16, &x[4 * k]);
            }
        }
        if (!a.lengths) {
            buf0 += sdiv;
            jb0 += smod;
            if (jb0 >= bpb) {
                jb0 -= bpb;
                ++buf0;
            }
        }
    }
}


// Workgroups that are resident at once on the whole device for kernel K
// (CUs x occupancy), cached per device: the persistent grid is sized to it so
// every wave runs from start to end and no partial second batch of waves
// idles most SIMDs at the tail.
template <class K>
static uint64_t resident_grid(K kernel) {
    static int cache[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    if (cache[dev] <= 0) {
        int cus = 0, per = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 256, 0) != hipSuccess || per <= 0) per = 4;
        cache[dev] = cus * per;
    }
    return (uint64_t)cache[dev];
}

// Grid: each wave takes ~kTilesPerWave tiles (grid-stride), so a launch is
// many short waves rather than exactly one resident batch — the hardware
// dispatcher then evens out the tail, and nothing depends on the occupancy
// API (which can over-count residency by one workgroup per CU at some SGPR
// counts, MI355X_MICROARCH.md 'Residency').  Ragged batches (total unknown on
// the host) launch 8x the resident count and grid-stride.
constexpr uint64_t kChaTilesPerWave = 4;
template <int DR>
static void launch_cha_dr(const ChaArgs& a, uint64_t need_tiles, hipStream_t s) {
    auto kern = chacha_lane_kernel<DR>;
    uint64_t grid = need_tiles == UINT64_MAX
                        ? 8 * resident_grid(kern)
                        : (need_tiles + 4 * kChaTilesPerWave - 1) / (4 * kChaTilesPerWave);
    grid = std::min<uint64_t>(std::max<uint64_t>(grid, 1), 1u << 20);
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256), 0, s, a);
}

void launch_chacha(const ChaArgs& a, uint64_t nparts, uint64_t* parts, uint64_t* blk_start,
                   uint32_t* subkeys, hipStream_t s) {
    ChaArgs k = a;
    if (a.lengths) {
        const unsigned nb = (unsigned)((a.count + kScanPer - 1) / kScanPer);
        hipLaunchKernelGGL(chacha_scan_reduce, dim3(nb), dim3(256), 0, s, a.lengths, a.count, parts);
        hipLaunchKernelGGL(chacha_scan_parts, dim3(1), dim3(256), 0, s, parts, nparts);
        hipLaunchKernelGGL(chacha_scan_final, dim3(nb), dim3(256), 0, s, a.lengths, a.count,
                           (const uint64_t*)parts, blk_start);
        k.blk_start = blk_start;
    }
    if (subkeys) {
        hipLaunchKernelGGL(hchacha_kernel, dim3((unsigned)((a.count + 255) / 256)), dim3(256), 0, s, a,
                           subkeys);
        k.subkeys = subkeys;
    }
    // Grid sizing: see launch_cha_dr.
    constexpr uint64_t kTile = 64u;
    uint64_t need = UINT64_MAX;  // tiles
    if (!a.lengths) need = (a.total_blocks + kTile - 1) / kTile;
    switch (a.dr) {
    case 4: launch_cha_dr<4>(k, need, s); break;     // ChaCha8
    case 6: launch_cha_dr<6>(k, need, s); break;     // ChaCha12
    case 10: launch_cha_dr<10>(k, need, s); break;   // ChaCha20
    default: launch_cha_dr<0>(k, need, s); break;
    }
}

}  // namespace lcbgpu
