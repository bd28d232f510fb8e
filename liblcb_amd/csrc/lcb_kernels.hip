// lcb_kernels.hip — MI355X (gfx950) batch digest kernels and their launchers.
//
// Grid: one lane per message, 256-thread workgroups (4 waves), message index
// = blockIdx.x * 256 + threadIdx.x, optionally through a bucketing
// permutation `order` (ragged batches: similar lengths share a wavefront).
// No inter-workgroup communication; every message is independent.
#include <hip/hip_runtime.h>
#include "hash_device.hpp"
#include "gost_device.hpp"
#include "lcb_internal.hpp"

namespace lcbgpu {

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
// 5 workgroups per CU (the whole 160 KiB); deeper per-wave buffering,
// half-line stages and taking the next line mid-way through the current one
// (two line registers sets: 4 waves/SIMD) measured slower
// (profiles/r1_lds_depth_ab.txt, r1_lds_half_ab.txt, r2_fixed_stream_ab.txt).
// kAux: cache policy of the line stream -- nt when every record starts on a
// 128-B line (each streamed line is one cache line, read once); default
// otherwise, so the second cache line of a straddling 128-B line is still
// in L2 when the record's next line asks for it.
template <class H, bool kHmac, int kAux>
__global__ __launch_bounds__(256) void md_fixed_lds_kernel(KArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t slab[4][8192];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint64_t wave_first = ((uint64_t)blockIdx.x * 4 + wv) * 64;
    if (wave_first >= a.count) return;  // wave-uniform
    // A partial last wave moves back over its predecessor's records (count >=
    // 64, fixed_stride_lines) and stores only its own: no per-lane clamping.
    const uint64_t last = a.count - 1;
    const uint32_t skip = wave_first + 63 > last ? (uint32_t)(wave_first + 63 - last) : 0u;
    wave_first -= skip;
    const uint64_t nlines = a.fixed_len / 128;
    LdsStridedStream ls;
    ls.init(a.data, a.stride, wave_first, lane, &slab[wv][0]);
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
    const uint8_t* msg = a.data + i * a.stride + nlines * 128;
    const uint64_t tail = (uint64_t)a.fixed_len - nlines * 128;
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
}

// ------------------------------------- MD family, bucketed ragged batches
// A length-bucketed batch (`order` lists messages longest class first) is cut
// into TILES of 64 consecutive `order` entries, one tile per wave at a time,
// in a persistent grid of 5-wave workgroups sized to what is resident
// (5 per CU: 25 waves):
//   waves 0..3  STREAM waves: when every record of the tile has the same
//               number of whole 128-B lines (a length bucket) and starts 16-B
//               aligned, the lines move through an 8 KiB LDS slab per wave
//               by coalesced LDS-DMA (GatherLineStream: 8 records x one line
//               per instruction); other tiles load per lane;
//   wave 4      a DIRECT wave: per-lane 128-B line loads, no LDS.
// LDS holds 4 x 5 = 20 stream waves per CU (5,120 on the chip); a C4 batch
// (1M records of {64 B, 1 KiB, 64 KiB}) has 5,461 tiles of
// 64 KiB records, so with stream waves alone the last 341 long tiles start
// only when the first ones end (profiles/r1_gather_ab.txt).  Here every
// wave's FIRST tile is static — stream waves take tiles 0 .. S-1, direct
// waves S .. S+D-1 (S, D = resident stream / direct waves) — so all 5,461
// long chains start at once, and later tiles come from one device-scope
// atomic queue head, longest first.  Every wave leaves the loop once the
// queue is past the last tile.  Measured on C4 (MD5, profiles/r2_c4_tiles_ab.txt):
// 4.81 ms against 5.20-5.25 for the per-lane kernel and 4.92 for stream
// waves alone; 6-wave workgroups (5 + 1, 80 VGPRs) 5.54.
template <class H, bool kHmac>
__device__ __forceinline__ void md_tile_finish(const KArgs& a, H& st, uint64_t idx, const uint8_t* msg, uint64_t len,
                                               uint64_t done, uint64_t prefix) {
    md_message(st, msg + done, len - done, prefix + done);
    uint32_t dw[H::kDigest / 4];
    st.digest_words(dw);
    if (kHmac) {
        H o;
        load_words(o.s, a.mid + kMidWords);
        md_outer(o, dw);
        o.digest_words(dw);
    }
    store_digest<H::kDigest>(a.digests + idx * H::kDigest, dw);
}

// One 128-B line: two 64-B blocks, or one SHA-384/512 block.
template <class H>
__device__ __forceinline__ void md_compress_line(H& st, const uint32_t* w) {
    if constexpr (H::kBlock == 128) {
        st.compress(w);
    } else {
        st.compress(w);
        st.compress(w + 16);
    }
}

// Record `i` (clamped to the batch) of a bucketed batch: index, start, length.
__device__ __forceinline__ void tile_record(const KArgs& a, uint64_t i, uint64_t& idx, const uint8_t*& msg,
                                            uint64_t& len) {
    const uint64_t last = a.count - 1;
    idx = gptr(a.order)[i > last ? last : i];
    msg = gptr(a.data) + (a.offsets ? gptr(a.offsets)[idx] : idx * a.stride);
    len = a.lengths ? (uint64_t)gptr(a.lengths)[idx] : (uint64_t)a.fixed_len;
}

template <class H, bool kHmac>
__device__ __forceinline__ void md_tile_stream(const KArgs& a, uint64_t first, uint32_t lane, uint8_t* slab) {
    const uint64_t last = a.count - 1, i = first + lane;
    uint64_t idx, len;
    const uint8_t* msg;
    tile_record(a, i, idx, msg, len);
    H st;
    uint64_t prefix = 0;
    if (kHmac) {
        load_words(st.s, a.mid);
        prefix = H::kBlock;
    } else {
        st.init();
    }
    // Lines streamed per record; lanes past the end repeat the last record
    // (clamped above) and discard it.
    const uint32_t nl = (uint32_t)((len >> 7) < 0xffffffu ? (len >> 7) : 0xffffffu);
    // Stream when every record of the tile has the same number (> 0) of
    // whole lines and starts 16-B aligned (a length bucket: C4's 64 KiB
    // tiles); otherwise every lane loads its own bytes.
    const bool ok = nl > 0 && (reinterpret_cast<uintptr_t>(msg) & 15u) == 0 &&
                    nl == (uint32_t)__builtin_amdgcn_readfirstlane(nl);
    uint64_t done = 0;
    if (__all(ok)) {  // wave-uniform
        const uint32_t nlu = (uint32_t)__builtin_amdgcn_readfirstlane(nl);
        // Half-line phase of the tile (bucketing groups it): 0 when every
        // record starts on a 128-B line, 1 when every record starts 64 B into
        // one, 2 otherwise.
        const uint32_t ma = (uint32_t)reinterpret_cast<uintptr_t>(msg) & 127u;
        const uint32_t ma0 = (uint32_t)__builtin_amdgcn_readfirstlane(ma);
        const uint32_t ph = (__all(ma == ma0) && (ma0 & 63u) == 0) ? (ma0 >> 6) : 2u;
        GatherLineStream gs;
        if (H::kBlock == 64 && ph < 2) {
            // Whole cache lines: a 64-B-phase tile streams the nlu + 1 lines
            // its records overlap (line L = blocks 2L-1 and 2L of the record;
            // the bytes before its first block and after its last whole line
            // share those cache lines and are discarded), so no line is read
            // twice and the stream carries the read-once (nt) policy.
            const uint32_t n = nlu + ph;
            gs.init_gather(msg - 64 * ph, n - 1, lane, slab);
            gs.issue_next_uniform<kLdsAux>();
            for (uint32_t L = 0; L < n; ++L) {
                uint32_t w[32];
                gs.take(w, w + 16);
                if (L + 1 < n) gs.issue_next_uniform<kLdsAux>();
                if (ph == 0 || L > 0) st.compress(w);
                if (ph == 0 || L < nlu) st.compress(w + 16);
            }
        } else {
            gs.init_gather(msg, nlu - 1, lane, slab);
            gs.issue_next_uniform();
            for (uint32_t L = 0; L < nlu; ++L) {
                uint32_t w[32];
                gs.take(w, w + 16);
                if (L + 1 < nlu) gs.issue_next_uniform();
                md_compress_line(st, w);
            }
        }
        done = (uint64_t)nlu * 128;
    }
    if (i > last) return;
    tile_record(a, i, idx, msg, len);   // reloaded: not kept live across the line loop
    md_tile_finish<H, kHmac>(a, st, idx, msg, len, done, prefix);
}

template <class H, bool kHmac>
__device__ __forceinline__ void md_tile_direct(const KArgs& a, uint64_t first, uint32_t lane) {
    const uint64_t i = first + lane;
    if (i >= a.count) return;
    const uint64_t idx = gptr(a.order)[i];
    const uint8_t* msg = gptr(a.data) + (a.offsets ? gptr(a.offsets)[idx] : idx * a.stride);
    const uint64_t len = a.lengths ? (uint64_t)gptr(a.lengths)[idx] : (uint64_t)a.fixed_len;
    H st;
    uint64_t prefix = 0;
    if (kHmac) {
        load_words(st.s, a.mid);
        prefix = H::kBlock;
    } else {
        st.init();
    }
    md_tile_finish<H, kHmac>(a, st, idx, msg, len, 0, prefix);
}

constexpr int kTileWaves = 5;         // waves per workgroup: 4 stream waves (32 KiB LDS) + 1 direct wave
constexpr int kTileStreamWaves = 4;
constexpr int kTileWgPerCu = 5;       // 160 KiB of LDS / 32 KiB; 25 waves per CU (7 on one SIMD)

template <class H, bool kHmac>
__global__ __launch_bounds__(64 * kTileWaves, H::kTileOcc) void md_tiles_kernel(KArgs a, uint32_t nstream, uint32_t nwaves) {
    __shared__ __attribute__((aligned(16))) uint8_t slab[kTileStreamWaves][8192];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const bool stream = wv < (uint32_t)kTileStreamWaves;   // wave-uniform
    const uint64_t ntiles = (a.count + 63) / 64;
    uint64_t t = stream ? (uint64_t)blockIdx.x * kTileStreamWaves + wv
                        : (uint64_t)nstream + (uint64_t)blockIdx.x * (kTileWaves - kTileStreamWaves) + (wv - kTileStreamWaves);
    while (t < ntiles) {
        if (stream) md_tile_stream<H, kHmac>(a, t * 64, lane, &slab[wv][0]);
        else md_tile_direct<H, kHmac>(a, t * 64, lane);
        uint32_t c = 0;
        if (lane == 0) c = atomicAdd(a.tile_next, 1u);   // device scope, returns the old head
        t = (uint64_t)nwaves + __builtin_amdgcn_readfirstlane(c);
    }
}

// HMAC key schedule on the device (RFC 2104, md5.h:309-338): key block =
// key (<= B bytes, passed by value) or H(key) (long key in device memory);
// mid[0..] = state after (K ^ ipad), mid[kMidWords..] = state after (K ^ opad).
template <class H>
__global__ void md_hmac_prep_kernel(KeyBlock kb, const uint8_t* dkey, uint64_t key_len, uint32_t* mid) {
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
__device__ __forceinline__ uint32_t key_of(const KArgs& a, uint64_t idx) {
    const uint32_t k = a.key_index ? gptr(a.key_index)[idx] : 0u;
    return k < a.nkeys ? k : a.nkeys - 1;   // out of range: the last key (documented)
}

template <class H, int kMode>
__global__ __launch_bounds__(256, H::kOcc < 4 ? H::kOcc : 4) void md_keyed_kernel(KArgs a) {
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

// ------------------------------------------------------------------ GOST
// Four waves per SIMD: the 64 KiB rotated LPS image (gost_device.hpp GostRot)
// leaves room for two 512-thread workgroups per CU, and the launch bound caps
// the state at 128 VGPRs.  (Two 256-thread workgroups at up to 256 VGPRs:
// 2-3 % slower; tools/gost_lanes_ab.hip)
constexpr int kGostThreads = 512;
template <bool k256, bool kHmac>
__global__ __launch_bounds__(kGostThreads, 4) void gost_batch_kernel(KArgs a) {
    __shared__ __attribute__((aligned(256))) uint64_t Timg[256 * 32];  // 64 KiB rotated image
    gost_stage_rot(Timg);
    GostRot T;
    T.init((lds_u8*)Timg);
    uint64_t idx, len;
    const uint8_t* msg;
    if (!msg_at(a, idx, msg, len)) return;
    using G = Gost<k256>;
    G st;
    uint32_t dw[G::kDigest / 4];
    if (kHmac) {
        st.load(a.mid, T);
        gost_message(st, msg, len, T);
        st.digest_words(dw, T);
        // Outer pass: fresh state after K ^ opad, message = inner digest.
        G o;
        o.load(a.mid + kMidWords, T);
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = (i < G::kDigest / 4) ? dw[i] : 0u;
        if (G::kDigest == 64) {       // a 64-byte digest is a full block, then an
            o.block(w, 512, T);       // empty pad block (gost3411-2012.h:1783-1793)
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] = 0u;
            o.finish(w, 0, T);
        } else {
            o.finish(w, G::kDigest, T);  // 32 bytes: the digest is the tail block
        }
        o.digest_words(dw, T);
    } else {
        st.init();
        gost_message(st, msg, len, T);
        st.digest_words(dw, T);
    }
    store_digest<G::kDigest>(a.digests + idx * G::kDigest, dw);
}

// Keyed GOST batches (see md_keyed_kernel).
template <bool k256, int kMode>
__global__ __launch_bounds__(kGostThreads, 4) void gost_keyed_kernel(KArgs a) {
    __shared__ __attribute__((aligned(256))) uint64_t Timg[256 * 32];
    gost_stage_rot(Timg);
    GostRot T;
    T.init((lds_u8*)Timg);
    uint64_t idx, len;
    const uint8_t* msg;
    if (!msg_at(a, idx, msg, len)) return;
    using G = Gost<k256>;
    const uint32_t k = key_of(a, idx);
    const uint32_t* mid = gptr(a.mid) + (uint64_t)k * 2 * kMidWords;
    const uint8_t* K = gptr(a.keys) + gptr(a.key_off)[k];
    const uint64_t kl = gptr(a.key_len)[k];
    G st;
    uint32_t dw[G::kDigest / 4];
    if (kMode == kKeyHmac) {
        st.load(mid, T);
        gost_message(st, msg, len, T);
        st.digest_words(dw, T);
        G o;
        o.load(mid + kMidWords, T);
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = (i < G::kDigest / 4) ? dw[i] : 0u;
        if (G::kDigest == 64) {
            o.block(w, 512, T);
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] = 0u;
            o.finish(w, 0, T);
        } else {
            o.finish(w, G::kDigest, T);
        }
        o.digest_words(dw, T);
    } else if (kMode == kKeyPrefix) {
        const uint64_t full = kl / 64 * 64;
        st.load(mid, T);
        gost_message2(st, K + full, kl - full, msg, len, T);
        st.digest_words(dw, T);
    } else {
        st.init();
        gost_message2(st, msg, len, K, kl, T);
        st.digest_words(dw, T);
    }
    store_digest<G::kDigest>(a.digests + idx * G::kDigest, dw);
}

// One lane per key (flat table; the whole block stages it first).
template <bool k256>
__global__ __launch_bounds__(256) void gost_key_prep_kernel(KArgs a, uint32_t* mid) {
    __shared__ __attribute__((aligned(16))) uint64_t Timg[8 * 256];
    gost_stage_table(Timg);
    const GostFlat T{{}, Timg};
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= a.nkeys) return;
    using G = Gost<k256>;
    const uint8_t* K = gptr(a.keys) + gptr(a.key_off)[k];
    const uint64_t kl = gptr(a.key_len)[k];
    uint32_t* m = mid + k * 2 * kMidWords;
    G st;
    st.init();
    uint32_t w[16];
    if (a.key_mode == kKeyPrefix) {
        for (uint64_t b = 0; b < kl / 64; ++b) {
            load_full64(K + 64 * b, w);
            st.block(w, 512, T);
        }
        st.save(m, T);
        return;
    }
    if (kl > 64) {  // gost3411-2012.h:1873-1878: long key -> its digest
        gost_message(st, K, kl, T);
        uint32_t dw[G::kDigest / 4];
        st.digest_words(dw, T);
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = (i < G::kDigest / 4) ? dw[i] : 0u;
    } else if (kl == 64) {
        load_full64(K, w);
    } else {
        load_tail64(K, (uint32_t)kl, w);
    }
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = w[i] ^ 0x36363636u;
    st.init();
    st.block(x, 512, T);
    st.save(m, T);
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = w[i] ^ 0x5c5c5c5cu;
    st.init();
    st.block(x, 512, T);
    st.save(m + kMidWords, T);
}

template <bool k256>
__global__ void gost_hmac_prep_kernel(KeyBlock kb, const uint8_t* dkey, uint64_t key_len, uint32_t* mid) {
    __shared__ __attribute__((aligned(16))) uint64_t Timg[8 * 256];
    gost_stage_table(Timg);
    const GostFlat T{{}, Timg};
    if (threadIdx.x != 0) return;
    using G = Gost<k256>;
    uint32_t k[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) k[i] = kb.w[i];
    if (dkey) {  // gost3411-2012.h:1873-1878: long key -> its digest
        G st;
        st.init();
        gost_message(st, dkey, key_len, T);
        uint32_t dw[G::kDigest / 4];
        st.digest_words(dw, T);
#pragma unroll
        for (int i = 0; i < 16; ++i) k[i] = (i < G::kDigest / 4) ? dw[i] : 0u;
    }
    uint32_t w[16];
    G st;
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = k[i] ^ 0x36363636u;
    st.init();
    st.block(w, 512, T);
    st.save(mid, T);
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = k[i] ^ 0x5c5c5c5cu;
    st.init();
    st.block(w, 512, T);
    st.save(mid + kMidWords, T);
}

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
// `order` that groups messages by block-count class, longest class first
// (a counting sort; order inside a class is arbitrary and does not affect
// any digest, which is always written at the message's own index).
//   class(len) = nb for nb = len/64 + 1 < 64, else 58 + floor(log2(nb))
// i.e. exact block counts up to 4 KiB, power-of-two bins above.  Inside a
// class, records whose start lies in the first half of a 128-B line come
// after those in the second half (key = class * 2 + half): tiles of 64
// consecutive entries then share their half-line phase, and the tile kernel
// streams a 64-B-phase tile as whole cache lines (md_tile_stream).
__device__ __forceinline__ uint32_t len_class(uint64_t len) {
    const uint64_t nb = (len >> 6) + 1;
    if (nb < 64) return (uint32_t)nb;
    return 58u + (63u - (uint32_t)__clzll((long long)nb));
}

__device__ __forceinline__ uint32_t bucket_key(const KArgs& a, uint64_t i) {
    const uint64_t off = a.offsets ? gptr(a.offsets)[i] : i * a.stride;
    const uint32_t half = (uint32_t)(((reinterpret_cast<uintptr_t>(a.data) + off) >> 6) & 1u);
    return (len_class(gptr(a.lengths)[i]) << 1) | half;
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

// Block b owns the contiguous chunk [b * chunk, (b + 1) * chunk): it counts
// its keys, reserves one range per key (start of the key in DESCENDING key
// order, from the global histogram, + a per-key fill counter), then places
// its indices (LDS atomics give the rank inside the block's range).
__global__ __launch_bounds__(1024) void bucket_scatter_kernel(KArgs a, const uint32_t* hist, uint32_t* fill,
                                                             uint32_t* order, uint64_t chunk) {
    __shared__ uint32_t h[kBucketKeys];
    __shared__ uint32_t base[kBucketKeys];
    for (int c = threadIdx.x; c < kBucketKeys; c += blockDim.x) h[c] = 0;
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * chunk;
    const uint64_t hi = lo + chunk < a.count ? lo + chunk : a.count;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) atomicAdd(&h[bucket_key(a, i)], 1u);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int c = kBucketKeys - 1; c >= 0; --c) {
            base[c] = run;
            run += hist[c];
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kBucketKeys; k += blockDim.x) {
        if (h[k]) base[k] += atomicAdd(&fill[k], h[k]);
        h[k] = 0;
    }
    __syncthreads();
    for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        const uint32_t k = bucket_key(a, i);
        order[base[k] + atomicAdd(&h[k], 1u)] = (uint32_t)i;
    }
}

void launch_bucketing(const KArgs& a, uint32_t* work, uint32_t* order, hipStream_t s) {
    // work: histogram | fill counters | tile-queue head, zeroed here; order:
    // count uint32.
    (void)hipMemsetAsync(work, 0, kBucketWork * sizeof(uint32_t), s);
    uint64_t nb = (a.count + 1023) / 1024;
    if (nb > kBucketBlocks) nb = kBucketBlocks;
    const uint64_t chunk = (a.count + nb - 1) / nb;
    hipLaunchKernelGGL(bucket_hist_kernel, dim3((unsigned)nb), dim3(1024), 0, s, a, work);
    hipLaunchKernelGGL(bucket_scatter_kernel, dim3((unsigned)((a.count + chunk - 1) / chunk)), dim3(1024), 0, s, a,
                       work, work + kBucketKeys, order, chunk);
}

// ------------------------------------------------------------- launchers
static inline dim3 grid_for(uint64_t count) { return dim3((unsigned)((count + 255) / 256)); }

template <class H>
static void launch_md(const KArgs& a, bool hmac, hipStream_t s) {
    if constexpr (H::kLdsStream) {
        // LDS-DMA fast path: fixed-stride, 16-B aligned records of at least one
        // whole 128-B line.
        if (fixed_stride_lines(a)) {
            const dim3 grid((unsigned)((a.count + 255) / 256));
            if (a.stride % 128 == 0 && reinterpret_cast<uintptr_t>(a.data) % 128 == 0) {
                if (hmac) hipLaunchKernelGGL((md_fixed_lds_kernel<H, true, kLdsAux>), grid, dim3(256), 0, s, a);
                else hipLaunchKernelGGL((md_fixed_lds_kernel<H, false, kLdsAux>), grid, dim3(256), 0, s, a);
            } else {
                if (hmac) hipLaunchKernelGGL((md_fixed_lds_kernel<H, true, kGatherAux>), grid, dim3(256), 0, s, a);
                else hipLaunchKernelGGL((md_fixed_lds_kernel<H, false, kGatherAux>), grid, dim3(256), 0, s, a);
            }
            return;
        }
    }
    if constexpr (H::kTileOcc > 0) {
        if (a.order && a.tile_next) {  // bucketed ragged batch: persistent tile queue
            auto kern = hmac ? md_tiles_kernel<H, true> : md_tiles_kernel<H, false>;
            int per_cu = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * kTileWaves, 0) != hipSuccess || per_cu <= 0)
                per_cu = 1;
            per_cu = per_cu > kTileWgPerCu ? kTileWgPerCu : per_cu;
            const uint64_t ntiles = (a.count + 63) / 64;
            uint64_t grid = (uint64_t)per_cu * device_cu_count();
            const uint64_t need = (ntiles + kTileWaves - 1) / kTileWaves;
            if (grid > need) grid = need > 0 ? need : 1;
            hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * kTileWaves), 0, s, a,
                               (uint32_t)(grid * kTileStreamWaves), (uint32_t)(grid * kTileWaves));
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
template <bool k256>
static void launch_gost(const KArgs& a, bool hmac, hipStream_t s) {
    const dim3 g((unsigned)((a.count + kGostThreads - 1) / kGostThreads));
    if (hmac) hipLaunchKernelGGL((gost_batch_kernel<k256, true>), g, dim3(kGostThreads), 0, s, a);
    else hipLaunchKernelGGL((gost_batch_kernel<k256, false>), g, dim3(kGostThreads), 0, s, a);
}

template <class H>
static void launch_md_keyed(const KArgs& a, hipStream_t s) {
    switch (a.key_mode) {
    case kKeyHmac: hipLaunchKernelGGL((md_keyed_kernel<H, kKeyHmac>), grid_for(a.count), dim3(256), 0, s, a); break;
    case kKeyPrefix: hipLaunchKernelGGL((md_keyed_kernel<H, kKeyPrefix>), grid_for(a.count), dim3(256), 0, s, a); break;
    case kKeySuffix: hipLaunchKernelGGL((md_keyed_kernel<H, kKeySuffix>), grid_for(a.count), dim3(256), 0, s, a); break;
    }
}
template <bool k256>
static void launch_gost_keyed(const KArgs& a, hipStream_t s) {
    const dim3 g((unsigned)((a.count + kGostThreads - 1) / kGostThreads));
    switch (a.key_mode) {
    case kKeyHmac: hipLaunchKernelGGL((gost_keyed_kernel<k256, kKeyHmac>), g, dim3(kGostThreads), 0, s, a); break;
    case kKeyPrefix: hipLaunchKernelGGL((gost_keyed_kernel<k256, kKeyPrefix>), g, dim3(kGostThreads), 0, s, a); break;
    case kKeySuffix: hipLaunchKernelGGL((gost_keyed_kernel<k256, kKeySuffix>), g, dim3(kGostThreads), 0, s, a); break;
    }
}

void launch_key_prep(int alg, const KArgs& a, uint32_t* mid, hipStream_t s) {
    const dim3 g((unsigned)((a.nkeys + 63) / 64)), gg((unsigned)((a.nkeys + 255) / 256));
    switch (alg) {
    case 1: hipLaunchKernelGGL(md_key_prep_kernel<Md5>, g, dim3(64), 0, s, a, mid); break;
    case 2: hipLaunchKernelGGL(md_key_prep_kernel<Sha1>, g, dim3(64), 0, s, a, mid); break;
    case 3: hipLaunchKernelGGL(md_key_prep_kernel<Sha256<true>>, g, dim3(64), 0, s, a, mid); break;
    case 4: hipLaunchKernelGGL(md_key_prep_kernel<Sha256<false>>, g, dim3(64), 0, s, a, mid); break;
    case 5: hipLaunchKernelGGL(md_key_prep_kernel<Sha512<true>>, g, dim3(64), 0, s, a, mid); break;
    case 6: hipLaunchKernelGGL(md_key_prep_kernel<Sha512<false>>, g, dim3(64), 0, s, a, mid); break;
    case 7: hipLaunchKernelGGL(gost_key_prep_kernel<true>, gg, dim3(256), 0, s, a, mid); break;
    case 8: hipLaunchKernelGGL(gost_key_prep_kernel<false>, gg, dim3(256), 0, s, a, mid); break;
    }
}

void launch_batch(int alg, const KArgs& a, hipStream_t s) {
    const bool hmac = a.mid != nullptr;
    if (a.key_mode != kKeyNone) {
        switch (alg) {
        case 1: launch_md_keyed<Md5>(a, s); break;
        case 2: launch_md_keyed<Sha1>(a, s); break;
        case 3: launch_md_keyed<Sha256<true>>(a, s); break;
        case 4: launch_md_keyed<Sha256<false>>(a, s); break;
        case 5: launch_md_keyed<Sha512<true>>(a, s); break;
        case 6: launch_md_keyed<Sha512<false>>(a, s); break;
        case 7: launch_gost_keyed<true>(a, s); break;
        case 8: launch_gost_keyed<false>(a, s); break;
        }
        return;
    }
    switch (alg) {
    case 1: launch_md<Md5>(a, hmac, s); break;
    case 2: launch_md<Sha1>(a, hmac, s); break;
    case 3: launch_md<Sha256<true>>(a, hmac, s); break;
    case 4: launch_md<Sha256<false>>(a, hmac, s); break;
    case 5: launch_md<Sha512<true>>(a, hmac, s); break;
    case 6: launch_md<Sha512<false>>(a, hmac, s); break;
    case 7: launch_gost<true>(a, hmac, s); break;
    case 8: launch_gost<false>(a, hmac, s); break;
    default:
        if (is_crc_alg(alg)) launch_crc(alg - kCrcAlgBase, a, s);
        break;
    }
}

void launch_hmac_prep(int alg, const KeyBlock& kb, const uint8_t* dkey, uint64_t key_len,
                      uint32_t* mid, hipStream_t s) {
    switch (alg) {
    case 1: hipLaunchKernelGGL(md_hmac_prep_kernel<Md5>, dim3(1), dim3(64), 0, s, kb, dkey, key_len, mid); break;
    case 2: hipLaunchKernelGGL(md_hmac_prep_kernel<Sha1>, dim3(1), dim3(64), 0, s, kb, dkey, key_len, mid); break;
    case 3: hipLaunchKernelGGL(md_hmac_prep_kernel<Sha256<true>>, dim3(1), dim3(64), 0, s, kb, dkey, key_len, mid); break;
    case 4: hipLaunchKernelGGL(md_hmac_prep_kernel<Sha256<false>>, dim3(1), dim3(64), 0, s, kb, dkey, key_len, mid); break;
    case 5: hipLaunchKernelGGL(md_hmac_prep_kernel<Sha512<true>>, dim3(1), dim3(64), 0, s, kb, dkey, key_len, mid); break;
    case 6: hipLaunchKernelGGL(md_hmac_prep_kernel<Sha512<false>>, dim3(1), dim3(64), 0, s, kb, dkey, key_len, mid); break;
    case 7: hipLaunchKernelGGL(gost_hmac_prep_kernel<true>, dim3(1), dim3(256), 0, s, kb, dkey, key_len, mid); break;
    case 8: hipLaunchKernelGGL(gost_hmac_prep_kernel<false>, dim3(1), dim3(256), 0, s, kb, dkey, key_len, mid); break;
    }
}

void launch_gen(uint64_t seed, uint64_t start, uint8_t* out, uint64_t n, hipStream_t s) {
    const uint64_t nw = ((start + n + 7) >> 3) - (start >> 3);
    uint64_t blocks = (nw + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(gen_kernel, dim3((unsigned)blocks), dim3(256), 0, s, seed, start, out, n);
}

void gost_table_host(uint64_t* out) {
    for (int j = 0; j < 8; ++j)
        for (int b = 0; b < 256; ++b) out[j * 256 + b] = kGostAxHost.t[j][b];
}

}  // namespace lcbgpu
