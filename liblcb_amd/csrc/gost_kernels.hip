// gost_kernels.hip — GOST R 34.11-2012 (Streebog) batch kernels and their
// launchers (gost_device.hpp holds the per-lane transform).
#include <hip/hip_runtime.h>
#include "gost_device.hpp"
#include "hash_device.hpp"
#include "lcb_internal.hpp"
#include "seg_jobs.hpp"

namespace lcbgpu {

__device__ __forceinline__ void msg_at(const KArgs& a, uint64_t i, uint64_t& idx, const uint8_t*& msg,
                                       uint64_t& len) {
    idx = a.order ? (uint64_t)gptr(a.order)[i] : i;
    msg = gptr(a.data) + (a.offsets ? gptr(a.offsets)[idx] : idx * a.stride);
    len = a.lengths ? (uint64_t)gptr(a.lengths)[idx] : (uint64_t)a.fixed_len;
}

__device__ __forceinline__ uint32_t key_of(const KArgs& a, uint64_t idx) {
    const uint32_t k = a.key_index ? gptr(a.key_index)[idx] : 0u;
    // Required for memory safety: a device-mode batch with a bad index runs
    // (only its digest stores are gated, batch_aborted); the clamp keeps its
    // key-table and mid-state reads in bounds (md_tiles.hpp key_of).
    return k < a.nkeys ? k : a.nkeys - 1;
}

// Message index of message i, re-derived where the digest is stored (i's
// lane part passes through an empty asm, so the compiler reloads the index
// instead of keeping it live through the whole message: two VGPRs of the 128
// the GOST kernels may use).
__device__ __forceinline__ uint64_t store_index(const KArgs& a, uint64_t base) {
    uint32_t t = threadIdx.x;
    asm volatile("" : "+v"(t));
    const uint64_t i = base + t;
    return a.order ? (uint64_t)gptr(a.order)[i] : i;
}

// The digest words made final here (empty asm): else the compiler sinks
// the last LPS's XORs past store_index's branch and keeps its 8-byte table
// words live across it, which spilled GOST-256 (28 B per lane).
template <int N>
__device__ __forceinline__ void settle_words(uint32_t (&w)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+v"(w[i]));
}

// ------------------------------------------------------------------ GOST
// HMAC and keyed batches: one 1024-thread workgroup per CU (16 waves: four per SIMD, so at most 128
// VGPRs per lane) sharing ONE 64 KiB rotated LPS image (gost_device.hpp
// GostRot), and every lane's Sigma in the LDS beside it (64 KiB, Gost<k256,
// kGostThreads>): 128 KiB of the CU's 160.  Round 2 ran two 512-thread
// workgroups per CU, each with its own image and Sigma in VGPRs: at 128 VGPRs
// that spilled 12-68 B per lane to scratch (1.45-1.58x the algorithmic HBM
// traffic).  (Two 256-thread workgroups at up to 256 VGPRs were 2-3 %
// slower; tools/gost_lanes_ab.hip)
#ifndef LCB_GOST_THREADS
#define LCB_GOST_THREADS 1024
#endif
constexpr int kGostThreads = LCB_GOST_THREADS;
// Sigma words in LDS: all 8 with one 1024-thread workgroup per CU (64 KiB
// image + 64 KiB Sigma), the last 4 with two 512-thread workgroups (2 x 80 KiB).
constexpr int kGostSgLds = kGostThreads >= 1024 ? 8 : 4;
// The grid is persistent: one workgroup per CU stages the image once and
// walks the batch in strides of (grid x 1024) messages, so no CU idles at a
// workgroup boundary while its 16 waves drain and the next workgroup stages
// its table (one resident workgroup per CU: nothing else would fill in).
#define LCB_GOST_FOR_EACH(a, base)                                                                   \
    for (uint64_t base = (uint64_t)blockIdx.x * kGostThreads; base < (a).count;                      \
         base += (uint64_t)gridDim.x * kGostThreads)                                                 \
        if (base + threadIdx.x < (a).count)
template <bool k256>
__global__ __launch_bounds__(kGostThreads) void gost_hmac_kernel(KArgs a) {
    __shared__ __attribute__((aligned(256))) uint64_t Timg[256 * 32];  // 64 KiB rotated image
    __shared__ __attribute__((aligned(16))) uint64_t Sg[(kGostSgLds + (kGostSgLds == 8)) * kGostThreads];  // Sigma of every lane
    gost_stage_rot(Timg);
    GostRot T;
    T.init((lds_u8*)Timg);
    LCB_GOST_FOR_EACH(a, base) {
    uint64_t idx, len;
    const uint8_t* msg;
    msg_at(a, base + threadIdx.x, idx, msg, len);
    using G = Gost<k256, kGostThreads, kGostSgLds>;
    G st;
    st.bind_sigma((lds_u64w*)Sg);
    uint32_t dw[G::kDigest / 4];
    st.load(a.mid, T);   // state after K ^ ipad; the outer pass from K ^ opad
    gost_run(st, GostPlainSrc{msg, len}, T);
    st.digest_words(dw, T);
    gost_outer(st, dw, a.mid + kMidWords, T);
    st.digest_words(dw, T);
    settle_words<G::kDigest / 4>(dw);
    store_digest<G::kDigest>(a.digests + store_index(a, base) * G::kDigest, dw);
    }
}

// Plain GOST batches: the two-pass form (gost_run2: Sigma added up by a
// second pass over the message after the g_N chain), so neither the LDS nor
// the VGPRs hold Sigma through the chain and the LDS holds only the 64 KiB
// rotated image; an ordinary grid of 512-thread workgroups (one message per
// lane, two workgroups per CU at 4 waves per SIMD, no LPS scheduling fence).
// Measured against the persistent 1,024-thread Sigma-in-LDS form (the HMAC
// and keyed kernels below), same box, 1M x 1 KiB (profiles/r4_gost_ab.txt):
// 2.76-2.80 against 3.02-3.04 ms.  The persistent one-workgroup-per-CU grid
// keeps all 16 waves of a CU in step, so they wait on their block loads
// together while the CU's LDS, which bounds GOST, idles; independent
// workgroups drift apart.  (Persistent 2-pass 2.93 ms, 1,024-thread
// workgroups 2.93 ms, block prefetch by LDS-DMA 3.14 ms.)
constexpr int kGostPlainThreads = 512;
template <bool k256>
__global__ __launch_bounds__(kGostPlainThreads, 4) void gost_plain2_kernel(KArgs a) {
    __shared__ __attribute__((aligned(256))) uint64_t Timg[256 * 32];  // 64 KiB rotated image
    gost_stage_rot(Timg);
    GostRotF<0> T;
    T.init((lds_u8*)Timg);
    const uint64_t base = (uint64_t)blockIdx.x * kGostPlainThreads;
    if (base + threadIdx.x >= a.count) return;
    uint64_t idx, len;
    const uint8_t* msg;
    msg_at(a, base + threadIdx.x, idx, msg, len);
    using G = Gost<k256>;
    G st;
    uint32_t dw[G::kDigest / 4];
    st.init();
    gost_run2(st, GostPlainSrc{msg, len}, T);
    st.digest_words(dw, T);
    settle_words<G::kDigest / 4>(dw);
    store_digest<G::kDigest>(a.digests + store_index(a, base) * G::kDigest, dw);
}

// Plain GOST batches with segmented long waves (a.seg: the bucketing cut
// the longest class's waves into kSegs jobs, seg_jobs.hpp).  C4 (a third of
// 1M records 64 KiB long) ran 0.89 of the fixed-stride rate per compression
// unsegmented: 5,468 waves of 64 KiB records over 4,096 wave slots end in a
// partly filled second generation.  Job j of the grid is wave-level (8 per
// workgroup); a segment chains its lanes' whole blocks [n s / S, n (s + 1)
// / S) -- per lane, n = that lane's whole blocks -- and hands h (16 words)
// on; N = 512 x the blocks before it, so only h travels.  The last segment
// also runs the tail, g_0(h, N) and the Sigma pass over the whole message
// (gost_run2_final).  The same occupancy as gost_plain2_kernel; a separate
// kernel so that the plain one keeps its machine code.
template <bool k256>
__global__ __launch_bounds__(kGostPlainThreads, 4) void gost_seg_kernel(KArgs a) {
    __shared__ __attribute__((aligned(256))) uint64_t Timg[256 * 32];  // 64 KiB rotated image
    gost_stage_rot(Timg);
    GostRotF<0> T;
    T.init((lds_u8*)Timg);
    TileSeg js;
    const uint64_t wv = seg_job(a, (uint64_t)blockIdx.x * (kGostPlainThreads / 64) + (threadIdx.x >> 6), js);
    if (wv * 64 >= a.count) return;   // wave-uniform: the grid is an upper bound
    const uint64_t i = wv * 64 + (threadIdx.x & 63);
    const bool valid = i < a.count;
    uint64_t idx = 0, len = 0;
    const uint8_t* msg = gptr(a.data);
    if (valid) msg_at(a, i, idx, msg, len);
    using G = Gost<k256>;
    G st;
    st.init();
    const GostPlainSrc src{msg, len};
    const uint64_t nfull = src.nfull();
    uint64_t j0 = 0, j1 = nfull;
    bool last = true;
    if (js.nsegs > 1) {
        bool whole = false;
        if (js.seg > 0) {
            if (!seg_wait(js, &whole)) return;   // taken over by another job
            if (!whole) {
                j0 = nfull * js.seg / js.nsegs;
                seg_load(st.h, js.lane_state());
                st.set_n(512 * j0);
            }
        }
        if (!whole && js.seg + 1 < js.nsegs) {
            j1 = nfull * (js.seg + 1) / js.nsegs;
            last = false;
        }
    }
    gost_chain_blocks(st, src, T, j0, j1);
    if (!last) {
        seg_save(st.h, js.lane_state());
        seg_publish(js.flag, js.seg);
        return;
    }
    gost_run2_final(st, src, T);
    uint32_t dw[G::kDigest / 4];
    st.digest_words(dw, T);
    settle_words<G::kDigest / 4>(dw);
    if (valid) store_digest<G::kDigest>(a.digests + idx * G::kDigest, dw);
}

// Diagnostic (lcb_hash_gpu_read_probe LCB_PROBE_GOST_LPS): the bound of the
// plain kernel -- its LDS gathers alone.  The same grid, workgroups, table
// image and occupancy as gost_plain2_kernel; each lane runs the plain
// kernel's number of LPS transforms for a fixed_len-byte message (19 g of 25
// LPS for 1 KiB) as ONE dependent chain (each g's 25 LPS are a chain: t
// needs the new K), with no block loads, no Sigma and no feed-forward.  The
// bench reports lds_frac = this time / the kernel's.
__global__ __launch_bounds__(kGostPlainThreads, 4) void gost_lps_probe_kernel(uint64_t count, uint32_t nlps,
                                                                              uint32_t* sink) {
    __shared__ __attribute__((aligned(256))) uint64_t Timg[256 * 32];
    gost_stage_rot(Timg);
    GostRotF<0> T;
    T.init((lds_u8*)Timg);
    const uint64_t i = (uint64_t)blockIdx.x * kGostPlainThreads + threadIdx.x;
    if (i >= count) return;
    uint64_t x[8], o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = 0x9e3779b97f4a7c15ull * (i * 8 + k + 1);
#pragma unroll 1
    for (uint32_t r = 0; r < nlps; ++r) {
        T.lps(o, x);
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = o[k] ^ (uint64_t)(r + k);   // the chain's round-constant XOR
    }
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= x[k];
    gptr(sink)[i] = (uint32_t)acc ^ (uint32_t)(acc >> 32);
}

void launch_gost_lps_probe(uint64_t count, uint32_t fixed_len, uint32_t* sink, hipStream_t s) {
    const uint32_t nlps = (fixed_len / 64 + 1 + 2) * 25;   // g_N per whole block + tail, g_0 twice
    hipLaunchKernelGGL(gost_lps_probe_kernel, dim3((unsigned)((count + kGostPlainThreads - 1) / kGostPlainThreads)),
                       dim3(kGostPlainThreads), 0, s, count, nlps, sink);
}

// Keyed GOST batches (see md_keyed_kernel).
template <bool k256, int kMode>
__global__ __launch_bounds__(kGostThreads) void gost_keyed_kernel(KArgs a) {
    __shared__ __attribute__((aligned(256))) uint64_t Timg[256 * 32];
    __shared__ __attribute__((aligned(16))) uint64_t Sg[(kGostSgLds + (kGostSgLds == 8)) * kGostThreads];
    gost_stage_rot(Timg);
    GostRot T;
    T.init((lds_u8*)Timg);
    LCB_GOST_FOR_EACH(a, base) {
    uint64_t idx, len;
    const uint8_t* msg;
    msg_at(a, base + threadIdx.x, idx, msg, len);
    using G = Gost<k256, kGostThreads, kGostSgLds>;
    const uint32_t k = key_of(a, idx);
    const uint32_t* mid = gptr(a.mid) + (uint64_t)k * 2 * kMidWords;
    const uint8_t* K = gptr(a.keys) + gptr(a.key_off)[k];
    const uint64_t kl = gptr(a.key_len)[k];
    G st;
    st.bind_sigma((lds_u64w*)Sg);
    uint32_t dw[G::kDigest / 4];
    if (kMode == kKeyHmac) {
        st.load(mid, T);
        gost_run(st, GostPlainSrc{msg, len}, T);
        st.digest_words(dw, T);
        // The key's outer mid-state, looked up again (not kept live through the message).
        const uint64_t i2 = store_index(a, base);
        gost_outer(st, dw, gptr(a.mid) + (uint64_t)key_of(a, i2) * 2 * kMidWords + kMidWords, T);
    } else if (kMode == kKeyPrefix) {
        // State after K's whole blocks; the rest of K and the message as one
        // virtual message (radius.h:774-789 copies the keyed context the same way).
        const uint64_t full = kl / 64 * 64;
        st.load(mid, T);
        gost_run(st, GostVirtSrc{K + full, kl - full, msg, len}, T);
    } else {
        st.init();
        gost_run(st, GostVirtSrc{msg, len, K, kl}, T);
    }
    st.digest_words(dw, T);
    settle_words<G::kDigest / 4>(dw);
    if (!batch_aborted(a)) store_digest<G::kDigest>(a.digests + store_index(a, base) * G::kDigest, dw);
    }
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
__global__ __launch_bounds__(256) void gost_hmac_prep_kernel(KeyBlock kb, const uint8_t* dkey, uint64_t key_len, uint32_t* mid) {
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

// Persistent grid: as many workgroups as fit on the chip at once (the LDS of
// the image + Sigma and the VGPRs decide how many per CU).
template <class K>
static dim3 gost_grid(K kern, uint64_t count, int threads = kGostThreads) {
    const uint64_t need = (count + threads - 1) / threads;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, 0) != hipSuccess || per_cu <= 0)
        per_cu = 1;
    const uint64_t slots = (uint64_t)per_cu * device_cu_count();
    return dim3((unsigned)(need < slots ? need : slots));
}
template <bool k256>
void launch_gost(const KArgs& a, bool hmac, hipStream_t s) {
    if (hmac) {
        auto k = gost_hmac_kernel<k256>;
        hipLaunchKernelGGL(k, gost_grid(k, a.count), dim3(kGostThreads), 0, s, a);
    } else if (a.seg) {
        // waves + (kSegs - 1) x the segment capacity: an upper bound of the jobs
        const uint64_t jobs = (a.count + 63) / 64 + (uint64_t)(kSegs - 1) * a.seg_cap;
        const dim3 g((unsigned)((jobs + kGostPlainThreads / 64 - 1) / (kGostPlainThreads / 64)));
        hipLaunchKernelGGL(gost_seg_kernel<k256>, g, dim3(kGostPlainThreads), 0, s, a);
    } else {
        const dim3 g((unsigned)((a.count + kGostPlainThreads - 1) / kGostPlainThreads));
        hipLaunchKernelGGL(gost_plain2_kernel<k256>, g, dim3(kGostPlainThreads), 0, s, a);
    }
}
template <bool k256, int kMode>
static void launch_gost_keyed_mode(const KArgs& a, hipStream_t s) {
    auto k = gost_keyed_kernel<k256, kMode>;
    hipLaunchKernelGGL(k, gost_grid(k, a.count), dim3(kGostThreads), 0, s, a);
}
template <bool k256>
void launch_gost_keyed(const KArgs& a, hipStream_t s) {
    switch (a.key_mode) {
    case kKeyHmac: launch_gost_keyed_mode<k256, kKeyHmac>(a, s); break;
    case kKeyPrefix: launch_gost_keyed_mode<k256, kKeyPrefix>(a, s); break;
    case kKeySuffix: launch_gost_keyed_mode<k256, kKeySuffix>(a, s); break;
    }
}

#define LCB_GOST_FAMILY(k256, tag)                                                                   \
    void launch_plain_##tag(const KArgs& a, bool hmac, hipStream_t s) { launch_gost<k256>(a, hmac, s); } \
    void launch_keyed_##tag(const KArgs& a, hipStream_t s) { launch_gost_keyed<k256>(a, s); }        \
    void launch_key_prep_##tag(const KArgs& a, uint32_t* mid, hipStream_t s) {                      \
        hipLaunchKernelGGL(gost_key_prep_kernel<k256>, dim3((unsigned)((a.nkeys + 255) / 256)), dim3(256), 0, s, a, mid); \
    }                                                                                                \
    void launch_hmac_prep_##tag(const KeyBlock& kb, const uint8_t* dkey, uint64_t key_len, uint32_t* mid, \
                                hipStream_t s) {                                                     \
        hipLaunchKernelGGL(gost_hmac_prep_kernel<k256>, dim3(1), dim3(256), 0, s, kb, dkey, key_len, mid); \
    }
LCB_GOST_FAMILY(true, gost256)
LCB_GOST_FAMILY(false, gost512)

void gost_table_host(uint64_t* out) {
    for (int j = 0; j < 8; ++j)
        for (int b = 0; b < 256; ++b) out[j * 256 + b] = kGostAxHost.t[j][b];
}

}  // namespace lcbgpu
