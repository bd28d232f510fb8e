// lcb_chacha_gpu.cpp — exported C-ABI of the batched ChaCha / XChaCha
// (include/lcb_chacha_gpu.h).
//
// Device mode enqueues the (ragged scan,) (hchacha prep,) block kernel on the
// caller's stream with stream-ordered scratch and never synchronises.  Host
// mode runs a double-buffered pipeline on two private streams: pack chunk
// c+1's buffers into page-locked staging while chunk c is on the GPU, then
// H2D -> kernel -> D2H and scatter the output back to the caller's offsets.
// Dense fixed-stride batches whose src/dst are already page-locked are DMA'd
// directly.  Nothing falls back to the CPU.
#include <errno.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/lcb_chacha_gpu.h"
#include "../../include/lcb_hash_gpu.h"
#include "lcb_internal.hpp"

using namespace lcbgpu;

namespace {

#define CHA_TRY(expr)                             \
    do {                                          \
        hipError_t _e = (expr);                   \
        if (_e != hipSuccess) return map_err(_e); \
    } while (0)

// chacha.h:110-117
const uint32_t kSigma[4] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};  // "expand 32-byte k"
const uint32_t kTau[4] = {0x61707865u, 0x3120646eu, 0x79622d36u, 0x6b206574u};    // "expand 16-byte k"

// Largest `rounds` accepted: the reference loops `rounds` times without
// bound (chacha.h:432); a GPU kernel must finish, so absurd values are EINVAL.
constexpr size_t kMaxRounds = 1024;

uint32_t le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// Key, constants and rounds of one batch (chacha.h:286-316, 404-421).
ChaArgs make_args(bool x, const uint8_t* key, size_t key_size, size_t rounds) {
    ChaArgs a;
    const bool big = (key_size == 256 || key_size == 32);
    for (int k = 0; k < 4; ++k) a.hcst[k] = big ? kSigma[k] : kTau[k];
    for (int k = 0; k < 8; ++k) a.key[k] = le32(key + 4 * (big ? k : (k & 3)));
    // xchacha's block function always runs with the 256-bit subkey.
    for (int k = 0; k < 4; ++k) a.cst[k] = x ? kSigma[k] : a.hcst[k];
    a.dr = (uint32_t)((rounds + 1) / 2);
    a.iv_words = x ? 6 : 2;
    a.iv_at = x ? 4 : 0;
    return a;
}

// Enqueue one batch whose every pointer is on the device.
int cha_enqueue(ChaArgs a, bool x, hipStream_t s) {
    if (a.count == 0) return 0;
    if (!a.lengths) {
        if (a.fixed_len == 0) return 0;
        a.bpb = (uint32_t)((a.fixed_len + 63u) / 64u);
        a.total_blocks = (uint64_t)a.count * a.bpb;
        // One dense run of whole, 16-B aligned blocks: the kernel's
        // coalesced stream path applies to every full wave tile.
        const uintptr_t al = reinterpret_cast<uintptr_t>(a.dst) | reinterpret_cast<uintptr_t>(a.src);
        a.stream = (!a.offsets && a.stride == a.fixed_len && a.fixed_len % 64u == 0 && (al & 15u) == 0) ? 1u : 0u;
    }
    uint64_t* scan = nullptr;
    uint32_t* subkeys = nullptr;
    const uint64_t nparts = (a.count + 1023) / 1024;
    if (a.lengths)
        CHA_TRY(scratch_alloc(reinterpret_cast<void**>(&scan), (nparts + a.count + 1) * 8, s));
    if (x) {
        hipError_t e = scratch_alloc(reinterpret_cast<void**>(&subkeys), a.count * 32, s);
        if (e != hipSuccess) {
            if (scan) (void)scratch_free(scan, s);
            return map_err(e);
        }
    }
    launch_chacha(a, nparts, scan, scan ? scan + nparts : nullptr, subkeys, s);
    hipError_t e = hipGetLastError();
    if (scan) (void)scratch_free(scan, s);
    if (subkeys) (void)scratch_free(subkeys, s);
    return map_err(e);
}

// ------------------------------------------------------------ host mode
struct ChaStage {
    int device = -1;
    size_t cap = 0, mcap = 0;  // bytes / buffers per slot
    hipStream_t st[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    uint8_t* h_in[2] = {nullptr, nullptr};
    uint8_t* h_out[2] = {nullptr, nullptr};
    uint8_t* h_meta[2] = {nullptr, nullptr};  // offsets | lengths | counters | ivs
    uint8_t* d_in[2] = {nullptr, nullptr};
    uint8_t* d_out[2] = {nullptr, nullptr};
    uint8_t* d_meta[2] = {nullptr, nullptr};
    // pending output of a slot: buffers [first, first + n) packed in h_out
    size_t pend_first[2] = {0, 0}, pend_n[2] = {0, 0};
    bool pend_direct[2] = {false, false}, busy[2] = {false, false};

    static size_t meta_bytes(size_t m) { return m * (8 + 4 + 8 + 24); }

    void release() {
        for (int b = 0; b < 2; ++b) {
            if (h_in[b]) (void)hipHostFree(h_in[b]);
            if (h_out[b]) (void)hipHostFree(h_out[b]);
            if (h_meta[b]) (void)hipHostFree(h_meta[b]);
            if (d_in[b]) (void)hipFree(d_in[b]);
            if (d_out[b]) (void)hipFree(d_out[b]);
            if (d_meta[b]) (void)hipFree(d_meta[b]);
            if (done[b]) (void)hipEventDestroy(done[b]);
            if (st[b]) (void)hipStreamDestroy(st[b]);
            h_in[b] = h_out[b] = h_meta[b] = d_in[b] = d_out[b] = d_meta[b] = nullptr;
            done[b] = nullptr;
            st[b] = nullptr;
            busy[b] = false;
        }
        cap = mcap = 0;
        device = -1;
    }
    ~ChaStage() { release(); }

    int ensure(int dev, size_t need_bytes, size_t need_msgs) {
        if (device == dev && cap >= need_bytes && mcap >= need_msgs) return 0;
        const size_t nb = std::max(need_bytes, cap), nm = std::max(need_msgs, mcap);
        release();
        device = dev;
        for (int b = 0; b < 2; ++b) {
            CHA_TRY(hipStreamCreateWithFlags(&st[b], hipStreamNonBlocking));
            CHA_TRY(hipEventCreateWithFlags(&done[b], hipEventDisableTiming));
            CHA_TRY(hipHostMalloc(reinterpret_cast<void**>(&h_in[b]), nb, hipHostMallocDefault));
            CHA_TRY(hipHostMalloc(reinterpret_cast<void**>(&h_out[b]), nb, hipHostMallocDefault));
            CHA_TRY(hipHostMalloc(reinterpret_cast<void**>(&h_meta[b]), meta_bytes(nm), hipHostMallocDefault));
            CHA_TRY(hipMalloc(reinterpret_cast<void**>(&d_in[b]), nb));
            CHA_TRY(hipMalloc(reinterpret_cast<void**>(&d_out[b]), nb));
            CHA_TRY(hipMalloc(reinterpret_cast<void**>(&d_meta[b]), meta_bytes(nm)));
        }
        cap = nb;
        mcap = nm;
        return 0;
    }
};

thread_local ChaStage g_cha;
constexpr size_t kChaChunkBytes = 64ull << 20;
constexpr size_t kChaChunkMsgs = 1u << 18;

int chacha_host(bool x, const ChaArgs& proto, const uint8_t* counters, const uint8_t* ivs,
                const uint8_t* src, uint8_t* dst, const uint64_t* offsets, const uint32_t* lengths,
                size_t count, uint64_t stride, uint32_t fixed_len) {
    int dev = 0;
    CHA_TRY(hipGetDevice(&dev));
    auto off_of = [&](size_t i) -> uint64_t { return offsets ? offsets[i] : (uint64_t)i * stride; };
    auto len_of = [&](size_t i) -> uint64_t { return lengths ? lengths[i] : fixed_len; };
    uint64_t maxlen = fixed_len;
    if (lengths) {
        maxlen = 0;
        for (size_t i = 0; i < count; ++i) maxlen = std::max<uint64_t>(maxlen, lengths[i]);
    }
    int rc = g_cha.ensure(dev, std::max<size_t>(kChaChunkBytes, maxlen), kChaChunkMsgs);
    if (rc) return rc;
    ChaStage& S = g_cha;
    const size_t ivl = x ? 24 : 8;
    // Dense fixed stride with page-locked src/dst: no staging copies at all.
    const bool dense = !offsets && !lengths && stride == fixed_len;
    const bool direct = dense && is_pinned(dst) && (src == nullptr || is_pinned(src));

    auto drain = [&](int b) -> int {
        if (!S.busy[b]) return 0;
        CHA_TRY(hipEventSynchronize(S.done[b]));
        S.busy[b] = false;
        if (S.pend_direct[b]) return 0;
        std::vector<Piece> pieces;
        uint64_t pos = 0, bytes = 0;
        for (size_t k = 0; k < S.pend_n[b]; ++k) {
            const size_t i = S.pend_first[b] + k;
            const uint64_t ln = len_of(i);
            if (ln) pieces.push_back(Piece{dst + off_of(i), S.h_out[b] + pos, (size_t)ln});
            pos += ln;
            bytes += ln;
        }
        parallel_copy(pieces, bytes);
        return 0;
    };

    std::vector<Piece> pieces;
    size_t i = 0;
    int b = 0;
    while (i < count) {
        if ((rc = drain(b))) break;
        hipStream_t s = S.st[b];
        // Buffers [i, j) whose packed bytes fit one slot.
        size_t j = i;
        uint64_t total = 0;
        while (j < count && j - i < S.mcap) {
            const uint64_t n = len_of(j);
            if (j > i && total + n > S.cap) break;
            total += n;
            ++j;
        }
        const size_t n = j - i;
        ChaArgs a = proto;
        a.count = n;
        uint8_t* hm = S.h_meta[b];
        uint8_t* dm = S.d_meta[b];
        uint64_t* h_off = reinterpret_cast<uint64_t*>(hm);
        uint32_t* h_len = reinterpret_cast<uint32_t*>(hm + n * 8);
        uint8_t* h_ctr = hm + n * 12;
        uint8_t* h_iv = h_ctr + n * 8;
        bool ok = true;
        if (direct) {
            if (src) ok = hipMemcpyAsync(S.d_in[b], src + (uint64_t)i * stride, total ? total : 1,
                                         hipMemcpyHostToDevice, s) == hipSuccess;
        } else {
            pieces.clear();
            uint64_t pos = 0;
            for (size_t k = 0; k < n; ++k) {
                const uint64_t ln = len_of(i + k);
                if (src && ln) pieces.push_back(Piece{S.h_in[b] + pos, src + off_of(i + k), (size_t)ln});
                h_off[k] = pos;
                h_len[k] = (uint32_t)ln;
                pos += ln;
            }
            if (src) {
                parallel_copy(pieces, pos);
                ok = hipMemcpyAsync(S.d_in[b], S.h_in[b], pos ? pos : 1, hipMemcpyHostToDevice, s) == hipSuccess;
            }
        }
        if (dense) {
            a.offsets = nullptr; a.lengths = nullptr; a.stride = fixed_len; a.fixed_len = fixed_len;
        } else {
            a.offsets = reinterpret_cast<const uint64_t*>(dm);
            a.lengths = reinterpret_cast<const uint32_t*>(dm + n * 8);
            a.stride = 0; a.fixed_len = 0;
        }
        if (counters) memcpy(h_ctr, counters + i * 8, n * 8);
        if (ivs) memcpy(h_iv, ivs + i * ivl, n * ivl);
        if (ok && !dense)
            ok = hipMemcpyAsync(dm, hm, n * 12, hipMemcpyHostToDevice, s) == hipSuccess;
        if (ok && counters)
            ok = hipMemcpyAsync(dm + n * 12, h_ctr, n * 8, hipMemcpyHostToDevice, s) == hipSuccess;
        if (ok && ivs)
            ok = hipMemcpyAsync(dm + n * 20, h_iv, n * ivl, hipMemcpyHostToDevice, s) == hipSuccess;
        a.counters = counters ? reinterpret_cast<const uint32_t*>(dm + n * 12) : nullptr;
        a.ivs = ivs ? reinterpret_cast<const uint32_t*>(dm + n * 20) : nullptr;
        a.src = src ? S.d_in[b] : nullptr;
        a.dst = S.d_out[b];
        uint8_t* out = direct ? dst + (uint64_t)i * stride : S.h_out[b];
        if (!ok || cha_enqueue(a, x, s) != 0 ||
            (total && hipMemcpyAsync(out, S.d_out[b], total, hipMemcpyDeviceToHost, s) != hipSuccess) ||
            hipEventRecord(S.done[b], s) != hipSuccess) {
            rc = EIO;
            break;
        }
        S.pend_first[b] = i;
        S.pend_n[b] = n;
        S.pend_direct[b] = direct;
        S.busy[b] = true;
        i = j;
        b ^= 1;
    }
    const int rc2 = drain(0);
    const int rc3 = drain(1);
    if (rc) return rc;
    return rc2 ? rc2 : rc3;
}

}  // namespace

extern "C" {

int lcb_chacha_batch(int xchacha, const uint8_t* key, size_t key_size, const uint8_t* counters,
                     const uint8_t* ivs, size_t rounds, const uint8_t* src, uint8_t* dst,
                     const uint64_t* offsets, const uint32_t* lengths, size_t count, uint64_t stride,
                     uint32_t fixed_len, uint32_t flags, void* stream) {
    if (flags & ~LCB_HASH_F_DEVICE) return EINVAL;
    if (rounds > kMaxRounds) return EINVAL;
    if (count == 0) return 0;
    if (!key || !dst) return EINVAL;
    if (int rc = ensure_init()) return rc;
    const bool x = xchacha != 0;
    ChaArgs a = make_args(x, key, key_size, rounds);
    if (flags & LCB_HASH_F_DEVICE) {
        if ((reinterpret_cast<uintptr_t>(counters) | reinterpret_cast<uintptr_t>(ivs)) & 3u) return EINVAL;
        a.src = src; a.dst = dst; a.offsets = offsets; a.lengths = lengths;
        a.counters = reinterpret_cast<const uint32_t*>(counters);
        a.ivs = reinterpret_cast<const uint32_t*>(ivs);
        a.count = count; a.stride = stride; a.fixed_len = fixed_len;
        return cha_enqueue(a, x, reinterpret_cast<hipStream_t>(stream));
    }
    return chacha_host(x, a, counters, ivs, src, dst, offsets, lengths, count, stride, fixed_len);
}

int chacha_batch(const uint8_t* key, size_t key_size, const uint8_t* counters, const uint8_t* ivs,
                 size_t rounds, const uint8_t* src, uint8_t* dst, const uint64_t* offsets,
                 const uint32_t* lengths, size_t count, uint64_t stride, uint32_t fixed_len, uint32_t flags,
                 void* stream) {
    return lcb_chacha_batch(0, key, key_size, counters, ivs, rounds, src, dst, offsets, lengths, count, stride,
                            fixed_len, flags, stream);
}

int xchacha_batch(const uint8_t* key, size_t key_size, const uint8_t* counters, const uint8_t* ivs,
                  size_t rounds, const uint8_t* src, uint8_t* dst, const uint64_t* offsets,
                  const uint32_t* lengths, size_t count, uint64_t stride, uint32_t fixed_len, uint32_t flags,
                  void* stream) {
    return lcb_chacha_batch(1, key, key_size, counters, ivs, rounds, src, dst, offsets, lengths, count, stride,
                            fixed_len, flags, stream);
}

}  // extern "C"
