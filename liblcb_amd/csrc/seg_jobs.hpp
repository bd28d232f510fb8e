// seg_jobs.hpp -- segmented long tiles: one wave's share of a ragged batch
// (64 records of the longest length class) cut into kSegs jobs that hand the
// hash state on through memory (lcb_internal.hpp kSegs; used by the tile
// kernel, md_tiles.hpp, and the 128-B-block line kernel, md_kernels.hpp).
//
// Why: a long class of n waves over the chip's S SIMDs takes ceil(n / S)
// wave-times on its busiest SIMD, since a wave cannot be split: C4's 5,461
// waves of 64 KiB records are 5.33 per SIMD, 6 on a third of them (SHA-512
// 5,461 waves: 18.7 ms, 6,144 waves: 17.9 ms; tools/long_waves.py).  Thirds
// of a wave spread as 16 per SIMD.
#pragma once
#include <hip/hip_runtime.h>

#include "hash_device.hpp"
#include "lcb_internal.hpp"

namespace lcbgpu {

// A job of a segmented long tile (lcb_internal.hpp kSegs): segment `seg` of
// `nsegs` runs the tile's whole-block lines [B(seg), B(seg + 1)), B(s) =
// 1 + (LF - 1) s / nsegs, the last segment also the tail.  A segment hands
// the hash state on through `state` (kSegStateWords words per lane) and
// the tile's flag (segments done, agent-scope release / acquire); the
// next segment re-reads line B - 1 for its carry.  Jobs are ordered
// seg-major (every tile's segment 0 first), one generation of wave slots
// apart at least (launch_ordered), so a segment's predecessor has normally
// finished when it starts.  A job that has waited kSegWaitTicks anyway
// (100 ms of the 100-MHz constant clock) takes the tile over -- flag
// kSegTaken, the whole tile from line 0 -- so no dispatch order can leave
// a wave spinning forever; the others then leave (the predecessor's
// publish fails, later segments see kSegTaken).  The take-over test
// (LCB_SEG_TAKEOVER, launch_ordered) sets the wait to one tick and deals
// the jobs in reverse segment order, so every cut tile's last segment
// starts first and takes it over (each taken tile's flag stays kSegTaken,
// which the test reads back).
#ifndef LCB_TILE_SEG
#define LCB_TILE_SEG 1
#endif
constexpr uint64_t kSegWaitTicks = 10000000ull;
struct TileSeg {
    uint32_t seg = 0, nsegs = 1;
    uint32_t* flag = nullptr;
    uint32_t wait = 0;              // ticks before a take-over
    // The wave's saved states (wave-uniform base), word-major: word k of
    // lane l at state[64 k + l], so each store instruction writes 256
    // contiguous bytes (lane-major, 16-B per-lane runs, every dword store
    // was 64 partial-sector writes: C4 wrote 7.1x its digest bytes).
    uint32_t* state = nullptr;
    // This lane's word 0, its address formed where used (not held in VGPRs
    // through the line loop).
    __device__ __forceinline__ uint32_t* lane_state() const {
        uint32_t ln = threadIdx.x & 63u;
        asm volatile("" : "+v"(ln));
        return state + ln;
    }
};
__device__ __forceinline__ uint32_t seg_line(uint32_t LF, uint32_t s, uint32_t n) { return 1u + (LF - 1u) * s / n; }
// The hand-off: coherent stores, then (seg_publish) every store complete
// before the flag; coherent loads after the flag was seen.  p: this lane's
// word 0; word i at p[64 i].
template <int N>
__device__ __forceinline__ void seg_save(const uint32_t (&s)[N], uint32_t* p) {
#pragma unroll
    for (int i = 0; i < N; ++i) __hip_atomic_store(gptr(p) + 64 * i, s[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int N>
__device__ __forceinline__ void seg_load(uint32_t (&s)[N], const uint32_t* p) {
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < N; ++i)
        s[i] = __hip_atomic_load(const_cast<uint32_t*>(gptr(p)) + 64 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int N>
__device__ __forceinline__ void seg_save(const uint64_t (&s)[N], uint32_t* p) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
        __hip_atomic_store(gptr(p) + 128 * i, (uint32_t)s[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(gptr(p) + 128 * i + 64, (uint32_t)(s[i] >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
template <int N>
__device__ __forceinline__ void seg_load(uint64_t (&s)[N], const uint32_t* p) {
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const uint32_t lo = __hip_atomic_load(const_cast<uint32_t*>(gptr(p)) + 128 * i, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t hi = __hip_atomic_load(const_cast<uint32_t*>(gptr(p)) + 128 * i + 64, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
        s[i] = (uint64_t)lo | ((uint64_t)hi << 32);
    }
}
__device__ __forceinline__ void seg_publish(uint32_t* flag, uint32_t seg) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63) == 0) {
        uint32_t e = seg;
        (void)__hip_atomic_compare_exchange_strong(gptr(flag), &e, seg + 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
    }
}
// Wait until segment s - 1 has published (true), or the tile was taken
// over by another job (false: leave).  A wait past kSegWaitTicks takes the
// tile over (*whole = true, returns true).
__device__ __forceinline__ bool seg_wait(const TileSeg& js, bool* whole) {
    uint32_t* const flag = js.flag;
    const uint32_t s = js.seg;
    *whole = false;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        // Relaxed polls: the state travels by coherent (agent-scope atomic)
        // stores and loads, ordered by waiting for the stores before the
        // flag is published -- no release / acquire fence, which on gfx950
        // writes back / invalidates the XCD's whole L2 (buffer_wbl2 /
        // buffer_inv): with them segmented MD5 ran 17 % slower.
        // (readfirstlane: the wave's branches on it stay uniform)
        const uint32_t f = (uint32_t)__builtin_amdgcn_readfirstlane(
            __hip_atomic_load(gptr(flag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (f == kSegTaken) return false;
        if (f >= s) return true;   // (the state is read with coherent loads: seg_load)
        if (__builtin_amdgcn_s_memrealtime() - t0 >= js.wait) {
            // One lane exchanges (64 lanes on one word: which would win is
            // unspecified), the wave follows its result.
            int won = 0;
            if ((threadIdx.x & 63) == 0) {
                uint32_t e = f;
                won = __hip_atomic_compare_exchange_strong(gptr(flag), &e, kSegTaken, __ATOMIC_ACQ_REL,
                                                           __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (__builtin_amdgcn_readfirstlane(won)) {
                *whole = true;
                return true;
            }
            continue;   // it moved on meanwhile: read it again
        }
        __builtin_amdgcn_s_sleep(16);
    }
}

// The job of workgroup `blk` when the first nseg waves (in `order`) are
// segmented: jobs segment-major (every wave's segment 0 first), then the
// other waves in order.  Returns the wave index; js describes the job.
__device__ __forceinline__ uint64_t seg_job(const KArgs& a, uint64_t blk, TileSeg& js) {
    if (!a.seg) return blk;
    const uint32_t nseg = gptr(a.seg)[kSegHdrCount];
    if (blk < (uint64_t)kSegs * nseg) {
        const uint32_t sj = (uint32_t)(blk / nseg);
        const uint64_t w = blk - (uint64_t)sj * nseg;
        // (readfirstlane: the header words are uniform, and the line bounds
        // derived from the segment go into SGPR operands)
        const uint32_t rev = (uint32_t)__builtin_amdgcn_readfirstlane(gptr(a.seg)[kSegHdrReverse]);
        js.seg = rev ? kSegs - 1u - sj : sj;
        js.nsegs = kSegs;
        const uint32_t wt = (uint32_t)__builtin_amdgcn_readfirstlane(gptr(a.seg)[kSegHdrWait]);
        js.wait = wt ? wt : (uint32_t)kSegWaitTicks;
        js.state = a.seg + kSegHead + w * kSegBlockWords;
        js.flag = js.state + 64 * kSegStateWords;
        return w;
    }
    return blk - (uint64_t)(kSegs - 1) * nseg;
}

}  // namespace lcbgpu
