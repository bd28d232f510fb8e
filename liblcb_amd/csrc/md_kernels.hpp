// md_kernels.hpp — MD-family (MD5, SHA-1, SHA-2) batch kernels and their
// launchers, instantiated once per algorithm by the k_<alg>.hip translation
// units (LCB_MD_FAMILY below), so the library's kernels compile in parallel.
//
// Grid: one lane per message, 256-thread workgroups (4 waves), message index
// = blockIdx.x * 256 + threadIdx.x, optionally through a bucketing
// permutation `order` (ragged batches: similar lengths share a wavefront).
// No inter-workgroup communication; every message is independent.
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>

#include "hash_device.hpp"
#include "lcb_internal.hpp"
#include "seg_jobs.hpp"

namespace lcbgpu {

static inline dim3 grid_for(uint64_t count) { return dim3((unsigned)((count + 255) / 256)); }

__device__ __forceinline__ bool msg_at(const KArgs& a, uint64_t& idx, const uint8_t*& msg, uint64_t& len) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.count) return false;
    idx = a.order ? (uint64_t)gptr(a.order)[i] : i;
    msg = gptr(a.data) + (a.offsets ? gptr(a.offsets)[idx] : idx * a.stride);
    len = a.lengths ? (uint64_t)gptr(a.lengths)[idx] : (uint64_t)a.fixed_len;
    return true;
}

// ------------------------------------------------------------- MD family
// Message body: fixed-length batches of whole blocks take the pad-only final
// block from the kernel-argument length (wave-uniform, scalar schedule).
template <class H, bool kPf>
__device__ __forceinline__ void md_body(H& st, const KArgs& a, const uint8_t* msg, uint64_t len,
                                        uint64_t prefix) {
    if (!a.lengths && a.fixed_len % H::kBlock == 0) {
        md_full_blocks<H, kPf>(st, msg, (uint64_t)a.fixed_len / H::kBlock);
        md_pad_only(st, (uint64_t)a.fixed_len + prefix);
    } else {
        md_message<H, kPf>(st, msg, len, prefix);
    }
}

// kPf: small batches (fewer than kPfMaxCount messages: at most one wave per
// SIMD, so occupancy cannot hide the load latency) take the prefetching
// message loop with the whole register file available (two 128-B stages
// stay in VGPRs); otherwise the occupancy-bound loop at H::kOcc waves per
// SIMD.
constexpr uint64_t kPfMaxCount = 16384;
template <class H, bool kHmac, bool kPf = false>
__global__ __launch_bounds__(256, kPf ? 1 : H::kOcc) void md_batch_kernel(KArgs a) {
    uint64_t idx, len;
    const uint8_t* msg;
    if (!msg_at(a, idx, msg, len)) return;
    H st;
    uint32_t dw[H::kDigest / 4];
    if (kHmac) {
        load_words(st.s, a.mid);                       // state after K ^ ipad
        md_body<H, kPf>(st, a, msg, len, (uint64_t)H::kBlock);
        st.digest_words(dw);
        H o;
        load_words(o.s, a.mid + kMidWords);            // state after K ^ opad
        md_outer(o, dw);
        o.digest_words(dw);
    } else {
        st.init();
        md_body<H, kPf>(st, a, msg, len, 0);
        st.digest_words(dw);
    }
    store_digest<H::kDigest>(a.digests + idx * H::kDigest, dw);
}

// ------------------------------------------- MD family, fixed-stride fast path
// Fixed-stride batches with 16-B aligned records of >= 128 bytes (the bench
// workload and any array of equal-size records): each wave streams line L+1
// of its 64 records into LDS (LdsStridedStream, hash_device.hpp: scalar base
// + two per-lane offsets, no VALU per DMA) while the two 64-B blocks of line
// L are compressed.  Bytes after the last whole line go through the generic
// loader.  One line in flight per wave (8 KiB of LDS), 4 waves per workgroup,
// 4 workgroups per CU (128 KiB; a fifth is never placed); deeper per-wave buffering,
// half-line stages and taking the next line mid-way through the current one
// (two line registers sets: 4 waves/SIMD) measured slower
// (profiles/r1_lds_depth_ab.txt, r1_lds_half_ab.txt, r2_fixed_stream_ab.txt).
// kAux: cache policy of the line stream -- nt when every record starts on a
// 128-B line (each streamed line is one cache line, read once); default
// otherwise, so the second cache line of a straddling 128-B line is still
// in L2 when the record's next line asks for it.
// LCB_TILE_TRACE (diagnostic builds only, tools/build_variant.sh): lane 0
// of every wave records, per tile, 8 words at g_tile_trace[8 t] -- the
// 100 MHz real-time clock at the tile's start, after its geometry, at its
// first and last take and after its digests, the hardware id, the tile's
// line count | wave id << 16, and the shader cycles over the tile
// (tools/tile_trace.py reads them).  The fixed-stride kernel records the
// same per wave at g_fixed_trace[8 w].  Vector stores only.
#ifdef LCB_TILE_TRACE
__device__ uint64_t* g_tile_trace;
__device__ uint64_t* g_fixed_trace;
__device__ __forceinline__ uint64_t trace_now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ uint64_t trace_hwid() {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    return (uint64_t)hw | ((uint64_t)xcc << 32);
}
struct TileTrace {
    uint64_t w[8];
    __device__ __forceinline__ void mark(int i) { w[i] = trace_now(); }
    __device__ __forceinline__ void put(uint64_t* buf, uint64_t idx, uint32_t lane) {
        if (buf && lane == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) buf[idx * 8 + i] = w[i];
        }
    }
};
#define LCB_TRACE(...) __VA_ARGS__
#else
#define LCB_TRACE(...)
#endif

#ifndef LCB_FIXED_WAVES
#define LCB_FIXED_WAVES 4
#endif
// XCD-contiguous record ranges (xcd_block).
#ifndef LCB_FIXED_XCD
#define LCB_FIXED_XCD 1
#endif
// Resident-grid form (MD5; LCB_FIXED_PERSIST = workgroups per CU, 0 = off):
// the grid is exactly the workgroups that fit at once (4 x 32 KiB per CU, the
// fifth is never placed: DESIGN.md 9.5), XCD x owns the x-th eighth of the
// 64-record chunks and its waves sweep it together (chunk = base + slot +
// j * slots, so every SIMD hashes the same number of chunks), the next
// chunk's line 0 is issued while the current chunk's last line is
// compressed, and each wave's priority is the chunks it has left
// (LCB_FIXED_PPRIO: the arbiter otherwise favours the oldest wave, which
// ends first and leaves its SIMD one wave short at the end).  Same-process
// A/B against the one-generation-per-workgroup kernel (profiles/
// r4_fixed_persist_ab.txt): MD5 -1.9 %; contiguous runs per wave -0.4 %,
// without the priority +1.2 / +1.7 %; SHA-1 / SHA-256 +-0.2 % (not used).
#ifndef LCB_FIXED_PERSIST
#define LCB_FIXED_PERSIST 4
#endif
// SHA-1 on the resident grid too (A/B builds only, tools/build_variant.sh
// -DLCB_PERSIST_SHA1=1).
#ifndef LCB_PERSIST_SHA1
#define LCB_PERSIST_SHA1 0
#endif
#ifndef LCB_FIXED_PPRIO
#define LCB_FIXED_PPRIO 1
#endif
#ifndef LCB_FIXED_PINTER
#define LCB_FIXED_PINTER 1
#endif
constexpr int kFixedWaves = LCB_FIXED_WAVES;   // waves (8 KiB slabs) per workgroup
constexpr int kFixedPersist = LCB_FIXED_PERSIST;

template <class H, bool kHmac>
__device__ __forceinline__ void md_fixed_finish(H& st, const KArgs& a, const uint8_t* data, uint64_t stride,
                                                uint32_t fixed_len, uint64_t nlines, uint64_t prefix,
                                                uint64_t wave_first, uint32_t skip, uint32_t lane) {
    if (lane < skip) return;
    const uint64_t i = wave_first + lane;
    const uint8_t* msg = data + i * stride + nlines * 128;
    const uint64_t tail = (uint64_t)fixed_len - nlines * 128;
    if (tail == 0)  // wave-uniform: schedule of the pad block on the SALU
        md_pad_only(st, prefix + nlines * 128);
    else   // the resident grid's chunks-left priority stays (no per-lane bytes-left priority)
        md_message<H, false, false>(st, msg, tail, prefix + nlines * 128);
    uint32_t dw[H::kDigest / 4];
    st.digest_words(dw);
    if (kHmac) {
        H o;
        load_words(o.s, a.mid + kMidWords);
        md_outer(o, dw);
        o.digest_words(dw);
    }
    store_digest<H::kDigest>(a.digests + i * H::kDigest, dw);
}

template <class H, bool kHmac, int kAux>
__global__ __launch_bounds__(64 * kFixedWaves) void md_fixed_persist_kernel(KArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t slab[kFixedWaves][kSlabBytes];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint8_t* data = a.data;
    uint64_t count = a.count, stride = a.stride;
    uint32_t fixed_len = a.fixed_len;
    asm volatile("" : "+s"(data), "+s"(count), "+s"(stride), "+s"(fixed_len));
    // Balanced contiguous chunk range of this wave slot.
    const uint64_t nch = (count + 63) / 64;
#if LCB_FIXED_PINTER
    // Interleaved: XCD x owns the x-th eighth of the chunks; its waves sweep
    // it together (chunk base + slot + j * slots).
    const uint64_t xcd = blockIdx.x & 7u, nbx = gridDim.x >> 3;
    const uint64_t xb = xcd * nch / 8, xe = (xcd + 1) * nch / 8;
    const uint64_t lslots = nbx * kFixedWaves;
    const uint64_t ls0 = (uint64_t)(blockIdx.x >> 3) * kFixedWaves + wv;
    uint64_t c = xb + ls0;
    const uint64_t cstep = lslots;
    if (c >= xe) return;  // wave-uniform
    uint32_t nleft = (uint32_t)((xe - 1 - c) / cstep + 1);   // chunks left, this one included
#else
    const uint64_t slots = (uint64_t)gridDim.x * kFixedWaves;
    const uint64_t s = (uint64_t)xcd_block() * kFixedWaves + wv;
    uint64_t c = s * nch / slots;
    const uint64_t c_end = (s + 1) * nch / slots;
    constexpr uint64_t cstep = 1;
    if (c >= c_end) return;  // wave-uniform
    uint32_t nleft = (uint32_t)(c_end - c);
#endif
    const uint64_t last = count - 1;
    const uint32_t nlines = fixed_len / 128;
    // A partial last chunk moves back over its predecessor's records (count
    // >= 64) and stores only its own.
    auto first_of = [&](uint64_t ch, uint32_t& sk) {
        uint64_t f = ch * 64;
        sk = f + 63 > last ? (uint32_t)(f + 63 - last) : 0u;
        return f - sk;
    };
    uint32_t skip;
    uint64_t wave_first = first_of(c, skip);
    LdsStridedStream ls;
    ls.init(data, stride, wave_first, lane, &slab[wv][0]);
    ls.issue<kAux>(0);
    for (;;) {
        H st;
        uint64_t prefix = 0;
        if (kHmac) {
            load_words(st.s, a.mid);
            prefix = H::kBlock;
        } else {
            st.init();
        }
        const bool more = nleft > 1;
        uint32_t nskip = 0;
        const uint64_t next_first = more ? first_of(c + cstep, nskip) : 0;
        if (LCB_FIXED_PPRIO) {  // once per chunk: the chunks left after this one
            if (nleft > 3) __builtin_amdgcn_s_setprio(3);
            else if (nleft == 3) __builtin_amdgcn_s_setprio(2);
            else if (nleft == 2) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
        for (uint32_t L = 0; L < nlines; ++L) {
            uint32_t w[32];
            ls.take(w, w + 16);
            if (L + 1 < nlines) {
                ls.issue<kAux>(L + 1);
            } else if (more) {                  // the next chunk's line 0
                ls.wbase = data + next_first * stride;
                ls.issue<kAux>(0);
            }
            if constexpr (H::kBlock == 128) {
                st.compress(w);
            } else {
                st.compress(w);
                st.compress(w + 16);
            }
        }
        md_fixed_finish<H, kHmac>(st, a, data, stride, fixed_len, nlines, prefix, wave_first, skip, lane);
        if (!more) break;
        --nleft;
        c += cstep;
        wave_first = next_first;
        skip = nskip;
    }
}

template <class H, bool kHmac, int kAux>
__global__ __launch_bounds__(64 * kFixedWaves) void md_fixed_lds_kernel(KArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t slab[kFixedWaves][kSlabBytes];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint64_t wave_first = ((uint64_t)(LCB_FIXED_XCD ? xcd_block() : blockIdx.x) * kFixedWaves + wv) * 64;
    // The arguments line 0's issue needs, loaded together (one scalar round
    // trip; the compiler otherwise loads the count, branches, then loads the
    // rest: two round trips before every wave's first line).
    const uint8_t* data = a.data;
    uint64_t count = a.count, stride = a.stride;
    uint32_t fixed_len = a.fixed_len;
    asm volatile("" : "+s"(data), "+s"(count), "+s"(stride), "+s"(fixed_len));
    if (wave_first >= count) return;  // wave-uniform
    LCB_TRACE(TileTrace tr; const uint64_t trw = wave_first / 64; const uint64_t trc = __builtin_amdgcn_s_memtime();
              tr.mark(0); tr.w[1] = tr.w[0]; tr.w[5] = trace_hwid(); tr.w[6] = fixed_len / 128;)
    // A partial last wave moves back over its predecessor's records (count >=
    // 64, fixed_stride_lines) and stores only its own: no per-lane clamping.
    const uint64_t last = count - 1;
    const uint32_t skip = wave_first + 63 > last ? (uint32_t)(wave_first + 63 - last) : 0u;
    wave_first -= skip;
    const uint64_t nlines = fixed_len / 128;
    LdsStridedStream ls;
    ls.init(data, stride, wave_first, lane, &slab[wv][0]);
    H st;
    uint64_t prefix = 0;
    if (kHmac) {
        load_words(st.s, a.mid);
        prefix = H::kBlock;
    } else {
        st.init();
    }
    if (nlines) ls.issue<kAux>(0);
    for (uint64_t L = 0; L < nlines; ++L) {
        uint32_t w[32];
        ls.take(w, w + 16);                 // line L -> VGPRs, its buffer free again
        LCB_TRACE(if (L == 0) tr.mark(2); if (L + 1 == nlines) tr.mark(3);)
        if (L + 1 < nlines) ls.issue<kAux>(L + 1);
        if constexpr (H::kBlock == 128) {
            st.compress(w);                 // one SHA-384/512 block per line
        } else {
            st.compress(w);                 // two 64-B blocks per line
            st.compress(w + 16);
        }
    }
    if (lane < skip) return;
    const uint64_t i = wave_first + lane;
    const uint8_t* msg = data + i * stride + nlines * 128;
    const uint64_t tail = (uint64_t)fixed_len - nlines * 128;
    if (tail == 0)  // wave-uniform: schedule of the pad block on the SALU
        md_pad_only(st, prefix + nlines * 128);
    else
        md_message(st, msg, tail, prefix + nlines * 128);
    uint32_t dw[H::kDigest / 4];
    st.digest_words(dw);
    if (kHmac) {
        H o;
        load_words(o.s, a.mid + kMidWords);
        md_outer(o, dw);
        o.digest_words(dw);
    }
    store_digest<H::kDigest>(a.digests + i * H::kDigest, dw);
    LCB_TRACE(tr.mark(4); tr.w[7] = __builtin_amdgcn_s_memtime() - trc;
              tr.put(g_fixed_trace, trw, lane == skip ? 0u : 1u);)
}

// ------------------------- ragged 128-B-block batches (SHA-384/512), streamed
// A bucketed ragged batch (order by length class) of a 128-B-block hash: wave
// = 64 consecutive order entries, lane = message.  When every record of the
// wave starts 16-B aligned, the first nmin lines (nmin = the wave's smallest
// whole-line count; every record has them) stream through the wave's LDS
// slab with coalesced LDS-DMA (GatherLineStream: 8 records x one 128-B line
// per instruction, line L + 1 issued while line L is compressed: one line =
// one SHA-512 block); the rest of each message (further whole blocks, tail,
// padding) takes the per-lane loop.  The per-lane loop alone (md_batch_kernel
// over the order) streams each lane's message from its own address: with
// C4's 64 KiB records every lane of a wave reads a different page per block.
// Default cache policy: a record at a 64-B offset straddles cache lines, the
// second half stays in L2 for the record's next line.
#ifndef LCB_LINES128
#define LCB_LINES128 1
#endif
// One-wave workgroups (as the tile kernel), kLinesOcc per SIMD.  Segmented
// long waves (a.seg, seg_jobs.hpp): the first kSegs x nseg workgroups run
// thirds of the first nseg waves' line loops, handing the state on.
template <class H, bool kHmac>
__global__ __launch_bounds__(64, kLinesOcc) void md_lines_kernel(KArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t slab[kSlabBytes];
    const uint32_t lane = threadIdx.x & 63;
    TileSeg js;
    const uint64_t first = seg_job(a, blockIdx.x, js) * 64;
    if (first >= a.count) return;  // wave-uniform
    const uint64_t i = first + lane;
    const bool valid = i < a.count;
    // A lane past the batch end takes the wave's first record (no pad entries:
    // the order of a 128-B-block batch is unpadded), so every DMA address is a
    // record's own line.
    const uint64_t idx = gptr(a.order)[valid ? i : first];
    const uint8_t* msg = gptr(a.data) + (a.offsets ? gptr(a.offsets)[idx] : idx * a.stride);
    const uint64_t len = gptr(a.lengths)[idx];
    // Wave minimum of the whole-line counts (0 unless every record is 16-B
    // aligned), every lane active.
    uint32_t m = (reinterpret_cast<uintptr_t>(msg) & 15u) ? 0u : (uint32_t)(len >> 7);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t t = (uint32_t)__shfl_xor((int)m, o, 64);
        m = t < m ? t : m;
    }
    const uint32_t nmin = (uint32_t)__builtin_amdgcn_readfirstlane(m);
    // Longest record of the wave, in lines (segmented jobs only): a wave
    // whose streamed part is not most of its work is not cut.
    uint32_t mx = 0;
    if (js.nsegs > 1) {
        mx = (uint32_t)(len >> 7);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const uint32_t t = (uint32_t)__shfl_xor((int)mx, o, 64);
            mx = t > mx ? t : mx;
        }
        mx = (uint32_t)__builtin_amdgcn_readfirstlane(mx);
    }
    H st;
    uint64_t prefix = 0;
    if (kHmac) {
        load_words(st.s, a.mid);
        prefix = H::kBlock;
    } else {
        st.init();
    }
    // This job's lines [Lb, Le) of the streamed nmin.
    uint32_t Lb = 0, Le = nmin;
    bool suspend = false;
    if (js.nsegs > 1) {
        // Too short to cut, or most of a lane's work is its per-lane tail (the
        // wave that mixes the last long records with short ones: cut, its
        // last segment ran 21 long records per lane, alone, behind every
        // other job -- +3 ms on C4): segment 0 runs it whole, up front.
        if (nmin < (uint32_t)js.nsegs + 2u || 8ull * nmin < 7ull * mx) {
            if (js.seg != 0) return;
        } else {
            bool whole = false;
            if (js.seg > 0) {
                if (!seg_wait(js, &whole)) return;
                if (!whole) {
                    Lb = nmin * js.seg / js.nsegs;
                    seg_load(st.s, js.lane_state());
                }
            }
            if (!whole && js.seg + 1 < js.nsegs) {
                Le = nmin * (js.seg + 1) / js.nsegs;
                suspend = true;
            }
        }
    }
    if (Le > Lb) {
        GatherLineStream ls;
        ls.init_gather(msg + (uint64_t)Lb * 128, Le - Lb - 1, lane, slab);
        ls.issue_next_uniform<kGatherAux>();
        for (uint32_t L = Lb; L < Le; ++L) {
#if LCB_LANE_PRIO
            // (not in segmented jobs: same-process A/B on C4, 20.6 -> 19.9 ms
            // with segmenting on, and the build ran the unsegmented C4 4 %
            // faster too, 19.6 -> 18.8: profiles/r5_c4_segs_ab.txt)
            if (js.nsegs == 1 && ((L - Lb) & 15) == 0) wave_prio_left((uint64_t)(nmin - L) * 128);
#endif
            uint32_t w[32];
            ls.take(w, w + 16);
            if (L + 1 < Le) ls.issue_next_uniform<kGatherAux>();
            st.compress(w);
            if (suspend && L + 1 == Le) {   // (here, not after the loop: 4 VGPRs less at its exit)
                seg_save(st.s, js.lane_state());
                seg_publish(js.flag, js.seg);
            }
        }
    }
    if (suspend) return;
    if (!valid) return;
    // The record's address and length read again (L2-hot) rather than held
    // in 4 VGPRs through the line loop: the index is made opaque so the
    // loads are not merged with the first ones.
    uint64_t ix = idx;
    asm volatile("" : "+v"(ix));
    const uint8_t* msg2 = gptr(a.data) + (a.offsets ? gptr(a.offsets)[ix] : ix * a.stride);
    const uint64_t len2 = gptr(a.lengths)[ix];
    const uint64_t done = (uint64_t)nmin * 128;
    md_message(st, msg2 + done, len2 - done, prefix + done);
    uint32_t dw[H::kDigest / 4];
    st.digest_words(dw);
    if (kHmac) {
        H o;
        load_words(o.s, a.mid + kMidWords);
        md_outer(o, dw);
        o.digest_words(dw);
    }
    store_digest<H::kDigest>(a.digests + ix * H::kDigest, dw);
}

}  // namespace lcbgpu
#include "md_tiles.hpp"
namespace lcbgpu {

// HMAC key schedule on the device (RFC 2104, md5.h:309-338): key block =
// key (<= B bytes, passed by value) or H(key) (long key in device memory);
// mid[0..] = state after (K ^ ipad), mid[kMidWords..] = state after (K ^ opad).
template <class H>
__global__ __launch_bounds__(64) void md_hmac_prep_kernel(KeyBlock kb, const uint8_t* dkey, uint64_t key_len, uint32_t* mid) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint32_t k[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) k[i] = kb.w[i];
    if (dkey) {
        H st;
        st.init();
        md_message(st, dkey, key_len, 0);
        uint32_t dw[H::kDigest / 4];
        st.digest_words(dw);
#pragma unroll
        for (int i = 0; i < 32; ++i) k[i] = (i < H::kDigest / 4) ? dw[i] : 0u;
    }
    uint32_t w[H::kWords];
    H st;
#pragma unroll
    for (int i = 0; i < H::kWords; ++i) w[i] = k[i] ^ 0x36363636u;
    st.init();
    st.compress(w);
    save_words(st.s, mid);
#pragma unroll
    for (int i = 0; i < H::kWords; ++i) w[i] = k[i] ^ 0x5c5c5c5cu;
    st.init();
    st.compress(w);
    save_words(st.s, mid + kMidWords);
}

// --------------------------------------------------- keyed batches (MD family)
// lcb_hash_batch_keyed: message i uses key k = key_index[i] of a key table
// (RADIUS: one shared secret per peer, radius_client.c:242,886,1025).
// kKeyHmac  HMAC(K_k, m_i): mid[k] holds the states after K^ipad / K^opad
//           (md5.h:309-338), computed once per key by md_key_prep_kernel;
// kKeyPrefix H(K_k || m_i): mid[k] holds the state after K_k's whole blocks,
//           the rest of K_k and m_i are hashed as one virtual message
//           (radius.h:774-789: the key-prefixed MD5 context copied per block);
// kKeySuffix H(m_i || K_k) (radius.h:1334-1336, 1346-1352).

template <class H, int kMode>
__global__ __launch_bounds__(256, H::kBlock == 128 ? 3 : (H::kOcc < 4 ? H::kOcc : 4)) void md_keyed_kernel(KArgs a) {
    uint64_t idx, len;
    const uint8_t* msg;
    if (!msg_at(a, idx, msg, len)) return;
    const uint32_t k = key_of(a, idx);
    const uint32_t* mid = gptr(a.mid) + (uint64_t)k * 2 * kMidWords;
    const uint8_t* K = gptr(a.keys) + gptr(a.key_off)[k];
    const uint64_t kl = gptr(a.key_len)[k];
    H st;
    uint32_t dw[H::kDigest / 4];
    if (kMode == kKeyHmac) {
        load_words(st.s, mid);
        md_message(st, msg, len, (uint64_t)H::kBlock);
        st.digest_words(dw);
        H o;
        load_words(o.s, mid + kMidWords);
        md_outer(o, dw);
        o.digest_words(dw);
    } else if (kMode == kKeyPrefix) {
        const uint64_t full = kl / H::kBlock * H::kBlock;
        load_words(st.s, mid);
        md_message2(st, K + full, kl - full, msg, len, full);
        st.digest_words(dw);
    } else {
        st.init();
        md_message2(st, msg, len, K, kl, 0);
        st.digest_words(dw);
    }
    if (batch_aborted(a)) return;
    store_digest<H::kDigest>(a.digests + idx * H::kDigest, dw);
}

// One lane per key: the mid-states of a keyed batch.
template <class H>
__global__ __launch_bounds__(64) void md_key_prep_kernel(KArgs a, uint32_t* mid) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.nkeys) return;
    const uint8_t* K = gptr(a.keys) + gptr(a.key_off)[k];
    const uint64_t kl = gptr(a.key_len)[k];
    uint32_t* m = mid + k * 2 * kMidWords;
    H st;
    st.init();
    if (a.key_mode == kKeyPrefix) {
        md_full_blocks(st, K, kl / H::kBlock);
        save_words(st.s, m);
        return;
    }
    // HMAC: key block = K zero padded, or H(K) for a key longer than a block.
    uint32_t w[H::kWords];
    if (kl > (uint64_t)H::kBlock) {
        md_message(st, K, kl, 0);
        uint32_t dw[H::kDigest / 4];
        st.digest_words(dw);
#pragma unroll
        for (int i = 0; i < H::kWords; ++i) w[i] = i < H::kDigest / 4 ? dw[i] : 0u;
    } else if (kl == (uint64_t)H::kBlock) {
        load_block_full<H>(K, w);
    } else {
        load_block_tail<H>(K, (uint32_t)kl, w);
    }
    uint32_t x[H::kWords];
#pragma unroll
    for (int i = 0; i < H::kWords; ++i) x[i] = w[i] ^ 0x36363636u;
    st.init();
    st.compress(x);
    save_words(st.s, m);
#pragma unroll
    for (int i = 0; i < H::kWords; ++i) x[i] = w[i] ^ 0x5c5c5c5cu;
    st.init();
    st.compress(x);
    save_words(st.s, m + kMidWords);
}

// ------------------------------------------------------------- launchers
template <class H>
void launch_md(const KArgs& a, bool hmac, hipStream_t s) {
    if constexpr (H::kLdsStream) {
        // LDS-DMA fast path: fixed-stride, 16-B aligned records of at least one
        // whole 128-B line.
        if (fixed_stride_lines(a)) {
            constexpr unsigned T = 64 * kFixedWaves;
            const dim3 grid((unsigned)((a.count + T - 1) / T));
            if constexpr (kFixedPersist > 0 && (std::is_same<H, Md5>::value ||
                                                (LCB_PERSIST_SHA1 && std::is_same<H, Sha1>::value))) {
                const uint64_t cap = (uint64_t)kFixedPersist * device_cu_count();
                if (grid.x > cap && cap % 8 == 0) {
                    const dim3 pg((unsigned)cap);
                    if (a.stride % 128 == 0 && reinterpret_cast<uintptr_t>(a.data) % 128 == 0) {
                        if (hmac) hipLaunchKernelGGL((md_fixed_persist_kernel<H, true, kLdsAux>), pg, dim3(T), 0, s, a);
                        else hipLaunchKernelGGL((md_fixed_persist_kernel<H, false, kLdsAux>), pg, dim3(T), 0, s, a);
                    } else {
                        if (hmac) hipLaunchKernelGGL((md_fixed_persist_kernel<H, true, kGatherAux>), pg, dim3(T), 0, s, a);
                        else hipLaunchKernelGGL((md_fixed_persist_kernel<H, false, kGatherAux>), pg, dim3(T), 0, s, a);
                    }
                    return;
                }
            }
            if (a.stride % 128 == 0 && reinterpret_cast<uintptr_t>(a.data) % 128 == 0) {
                if (hmac) hipLaunchKernelGGL((md_fixed_lds_kernel<H, true, kLdsAux>), grid, dim3(T), 0, s, a);
                else hipLaunchKernelGGL((md_fixed_lds_kernel<H, false, kLdsAux>), grid, dim3(T), 0, s, a);
            } else {
                if (hmac) hipLaunchKernelGGL((md_fixed_lds_kernel<H, true, kGatherAux>), grid, dim3(T), 0, s, a);
                else hipLaunchKernelGGL((md_fixed_lds_kernel<H, false, kGatherAux>), grid, dim3(T), 0, s, a);
            }
            return;
        }
    }
    if (a.order && a.tile_next) {  // bucketed ragged batch: the tile kernel
        if (hmac ? launch_tiles<H, kTileHmac>(a, s) : launch_tiles<H, kTilePlain>(a, s)) return;
    }
    if constexpr (H::kBlock == 128 && LCB_LINES128) {
        // bucketed (unpadded order) 128-B-block batch: the streamed line loop
        if (a.order && a.lengths && !a.tile_next && a.count >= kPfMaxCount) {
            const dim3 grid((unsigned)((a.count + 63) / 64 + (a.seg ? (uint64_t)(kSegs - 1) * a.seg_cap : 0)));
            if (hmac) hipLaunchKernelGGL((md_lines_kernel<H, true>), grid, dim3(64), 0, s, a);
            else hipLaunchKernelGGL((md_lines_kernel<H, false>), grid, dim3(64), 0, s, a);
            return;
        }
    }
    if (a.count < kPfMaxCount) {
        if (hmac) hipLaunchKernelGGL((md_batch_kernel<H, true, true>), grid_for(a.count), dim3(256), 0, s, a);
        else hipLaunchKernelGGL((md_batch_kernel<H, false, true>), grid_for(a.count), dim3(256), 0, s, a);
        return;
    }
    if (hmac) hipLaunchKernelGGL((md_batch_kernel<H, true>), grid_for(a.count), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((md_batch_kernel<H, false>), grid_for(a.count), dim3(256), 0, s, a);
}

template <class H>
void launch_md_keyed(const KArgs& a, hipStream_t s) {
    if (a.order && a.tile_next) {  // bucketed ragged batch: the tile kernel's keyed modes
        if (a.key_mode == kKeyHmac && launch_tiles<H, kTileKeyedHmac>(a, s)) return;
        if (a.key_mode == kKeySuffix && launch_tiles<H, kTileKeyedSuffix>(a, s)) return;
    }
    switch (a.key_mode) {
    case kKeyHmac: hipLaunchKernelGGL((md_keyed_kernel<H, kKeyHmac>), grid_for(a.count), dim3(256), 0, s, a); break;
    case kKeyPrefix: hipLaunchKernelGGL((md_keyed_kernel<H, kKeyPrefix>), grid_for(a.count), dim3(256), 0, s, a); break;
    case kKeySuffix: hipLaunchKernelGGL((md_keyed_kernel<H, kKeySuffix>), grid_for(a.count), dim3(256), 0, s, a); break;
    }
}

// One algorithm's launchers (declared in lcb_internal.hpp).
#define LCB_MD_FAMILY(H, tag)                                                                        \
    void launch_plain_##tag(const KArgs& a, bool hmac, hipStream_t s) { launch_md<H>(a, hmac, s); }  \
    void launch_keyed_##tag(const KArgs& a, hipStream_t s) { launch_md_keyed<H>(a, s); }             \
    void launch_key_prep_##tag(const KArgs& a, uint32_t* mid, hipStream_t s) {                      \
        hipLaunchKernelGGL(md_key_prep_kernel<H>, dim3((unsigned)((a.nkeys + 63) / 64)), dim3(64), 0, s, a, mid); \
    }                                                                                                \
    void launch_hmac_prep_##tag(const KeyBlock& kb, const uint8_t* dkey, uint64_t key_len, uint32_t* mid, \
                                hipStream_t s) {                                                     \
        hipLaunchKernelGGL(md_hmac_prep_kernel<H>, dim3(1), dim3(64), 0, s, kb, dkey, key_len, mid);  \
    }

}  // namespace lcbgpu
