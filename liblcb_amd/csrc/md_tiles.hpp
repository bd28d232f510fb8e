// md_tiles.hpp — the tile kernel of bucketed ragged MD-family batches (the
// 64-byte-block hashes: MD5, SHA-1, SHA-224/256), included by md_kernels.hpp.
//
// A length-bucketed batch (lcb_kernels.hip launch_bucketing: `order` lists
// messages by key = length class x start phase, longest class first, every
// key's run padded to whole tiles for a large batch) is cut into TILES of 64
// consecutive `order` entries; one wave hashes one tile, lane = message.
// One-wave workgroups, one per tile, each with its 8 KiB LDS slab: the
// hardware dispatcher hands out the tiles in order (longest first) and a
// finished wave's slot takes the next tile at once.  MD5 at 108-123 VGPRs
// runs 4 waves per SIMD (H::kTileOcc), SHA-1 / SHA-224/256 at 156-194 VGPRs
// run 2 (they spill at 3; being VALU-bound they lose nothing by it).
//
// THE WHOLE-LINE STREAM.  The records of a tile share their length class
// (their 64-B block counts differ by at most one) and the dword phase
// R = (start >> 2) & 3 of their start inside its 16-B chunk, so one wave
// moves them through its slab by coalesced LDS-DMA as in the fixed-stride
// kernel (8 records x one 128-B line per global_load_lds_dwordx4).  Every
// record streams its own whole 128-B cache lines (base = start rounded down
// to 128 B, nt policy: each cache line is read once), whatever its start:
// with off = start & 127 = 64 h + 16 m + 4 R + sh,
//   * m (the start's chunk inside its 64-B half) is applied by the DMA: the
//     lane that fills slot k of the record's slab row loads the record's
//     chunk (k + m) & 7, so a lane's take() of line L reads the line rotated
//     by m chunks -- the words of the record's 16-B-aligned stream, the
//     chunks that wrapped round being the start of line L + 1's part;
//   * R is the tile's (uniform) dword shift of the 16-word block window and
//     sh the lane's byte shift, one v_alignbyte per word;
//   * h (the start's half of its line) offsets the lane's block numbering:
//     line L completes blocks 2L - 1 - h (from the carry, the last 16 words
//     of line L - 1, merged with line L's wrapped chunks) and 2L - h.
// No streamed line straddles two cache lines (a 16-B aligned stream base
// made every 128-B line two cache-line requests: 17 % of the packet stream,
// profiles/r3_tile_diag_ab.txt), and the bucketing key needs only the 4
// dword phases.  The stream carries every byte of the record, the last
// partial line included: a chunk is fetched only if its cache line holds a
// byte of its record (the line, and so its page, is the record's), so no
// per-lane global load remains and the tail, the 0x80 / length padding and
// the key bytes of a secret-suffix message are assembled in registers.
//
// Tiles that mix phases (small unpadded batches only) take the per-lane
// message loop (md_tile_direct).
//
// Modes (template kMode):
//   kTilePlain      H(m)
//   kTileHmac       HMAC(K, m), one key: mid-states at a.mid (md5.h:309-369)
//   kTileKeyedHmac  HMAC(K_k, m), k = key_index[i] (lcb_hash_batch_keyed)
//   kTileKeyedSuffix H(m || K_k) (radius.h:1315-1377, the packet authenticator)
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "hash_device.hpp"
#include "lcb_internal.hpp"
#include "seg_jobs.hpp"

namespace lcbgpu {

enum { kTilePlain = 0, kTileHmac = 1, kTileKeyedHmac = 2, kTileKeyedSuffix = 3 };


// __builtin_amdgcn_readfirstlane is 32-bit: a 64-bit value goes as two halves.
__device__ __forceinline__ uint64_t readfirstlane64(uint64_t v) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
}

// The key of message idx.  The clamp is REQUIRED for memory safety: device
// mode enqueues the batch right behind the index check (the check kernel,
// or bucket_count_kernel<true>) and gates only the digest stores on its
// flag (batch_aborted), so with a bad index the batch still runs, and the
// clamp is what keeps its key-table and mid-state reads inside the table.
// (Host mode rejects a bad index before any kernel runs.)
__device__ __forceinline__ uint32_t key_of(const KArgs& a, uint64_t idx) {
    const uint32_t k = a.key_index ? gptr(a.key_index)[idx] : 0u;
    return k < a.nkeys ? k : a.nkeys - 1;
}

// One lane's record of a tile.  A pad entry (kOrderPad, or past the last
// entry) takes lane 0's record (never a pad: a tile starts a key's run or
// continues it) so every DMA address stays inside the batch; its digest is
// not stored.
struct TileRec {
    const uint8_t* p;
    uint32_t idx;
    uint32_t len;
    bool valid;
};

// Message geometry / key of a lane for the tile modes.
template <class H, int kMode>
struct TileMsg {
    uint64_t total;     // bytes hashed after the state's prefix (message [+ suffix key])
    uint64_t prefix;    // bytes already in the state (HMAC: one block)
    const uint8_t* K;   // suffix key
    uint32_t kl;
};

// One block from the stream window X = c[0..15] ++ y[0..15] (c: the carry
// merged with line L's wrapped chunks, y: line L, for the carry block; c = y
// = line L for the line's own block): X[R + k] byte-shifted by sh, k = 0..15,
// i.e. the 16 raw LE words of the block.
// kA16: every record of the tile starts on a 16-B boundary (sh = 0, R = 0):
// the window is the words themselves, no v_alignbyte.
template <int R, bool kA16 = false>
__device__ __forceinline__ void tile_shift(const uint32_t* c, const uint32_t* y, uint32_t sh, uint32_t w[16]) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int j = R + k;
        const uint32_t lo = j < 16 ? c[j] : y[j - 16];
        const uint32_t hi = j + 1 < 16 ? c[j + 1] : y[j + 1 - 16];
        w[k] = kA16 ? lo : __builtin_amdgcn_alignbyte(hi, lo, sh);
    }
}
// The carry block's first 16 words: word j of the lane's rotated stream is
// still the carry (dwords 16..31 of line L - 1) while its chunk j >> 2 + m
// lies below 4, else it wrapped round into line L (y[16 + j]).  Chunk 0 is
// always kept (m <= 3); the three keep masks of chunks 1..3 (m < 3, m < 2,
// m < 1) are lane masks computed once per tile (TileKeep): 12 v_cndmask per
// line and no per-line compares.
struct TileKeep {
    bool k1, k2, k3;
    __device__ __forceinline__ void init(uint32_t m) {
        k1 = m < 3u;
        k2 = m < 2u;
        k3 = m < 1u;
    }
};
__device__ __forceinline__ void tile_merge(uint32_t* c, const uint32_t* y, const TileKeep& kp) {
#pragma unroll
    for (int q = 1; q < 4; ++q) {
        const bool keep = q == 1 ? kp.k1 : (q == 2 ? kp.k2 : kp.k3);
#pragma unroll
        for (int i = 0; i < 4; ++i) c[4 * q + i] = keep ? c[4 * q + i] : y[16 + 4 * q + i];
    }
}

// Compression inside the tile kernel: MD5 with its T constants as inline
// literals (Md5::addk), other hashes as they are.
template <class H>
__device__ __forceinline__ void tile_compress(H& st, const uint32_t* w) {
    if constexpr (std::is_same<H, Md5>::value) st.template compress<true>(w);
    else st.compress(w);
}

// Block b of a lane's (virtual) message from the streamed words w: whole
// message blocks go straight to compress; the block holding the message's
// end gets its bytes past the end cleared, the 0x80 terminator and, in the last block, the bit length of
// prefix + total (md5.h:266-288).  Lanes whose message has fewer blocks do
// nothing (b = 2^32 - 1: a lane whose first block starts in the next line).
// whole: every lane's block b is a whole message block (uniform fast path).
template <class H, int kMode>
__device__ __forceinline__ void tile_block(H& st, uint32_t b, uint32_t* w, uint64_t len, const TileMsg<H, kMode>& m,
                                           uint32_t nblk, bool whole) {
    if (whole) {                   // wave-uniform: every lane has a whole message block here
        tile_compress(st, w);
        return;
    }
    if (b >= nblk) return;         // this lane is done (or has no block here: b = -1)
    const uint64_t pos = (uint64_t)b * 64;
    if (pos + 64 > len) {          // the block holds the end of the message
        const uint32_t rb = pos >= len ? 0u : (uint32_t)(len - pos);   // message bytes in the block
        // Words below the end word e are message words, words above it
        // zero; word e keeps its rb & 3 message bytes and takes the 0x80
        // terminator after them when the message (m.total == len: every mode
        // but the keyed suffix, whose tail is not assembled here) ends in
        // this block: 5 VALU per word (was 10, with put_byte's pass).
        const uint32_t e = rb >> 2, sb = 8u * (rb & 3u);
        const uint32_t pm = (1u << sb) - 1u;
        const uint32_t pb = (m.total == len && len >= pos) ? (0x80u << sb) : 0u;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t part = (w[k] & pm) | pb;
            w[k] = e > (uint32_t)k ? w[k] : (e == (uint32_t)k ? part : 0u);
        }
        if constexpr (kMode == kTileKeyedSuffix) {
            // The key K (the message's suffix: virtual bytes len .. total)
            // ORed in where it falls in this block (per-lane loads of the
            // small key table, L2-resident), then its 0x80 terminator.
            if (pos < m.total) {
                const uint64_t kb = pos > len ? pos : len;       // first block byte taken from K
                const uint32_t s0 = (uint32_t)(kb - pos);
                const uint64_t e = pos + 64 < m.total ? pos + 64 : m.total;
                or_window64_padded(m.K + (kb - len) - s0, s0, (uint32_t)(e - pos), w);
            }
            if (m.total >= pos && m.total < pos + 64) put_byte(w, (uint32_t)(m.total - pos), 0x80u);
        }
        if (b + 1 == nblk) H::put_length(w, m.total + m.prefix);
    }
    tile_compress(st, w);
}

// Initial state, materialised where the line loop starts (as plain
// constants they were hoisted and held in registers across the loop).
template <class H>
__device__ __forceinline__ void tile_init(H& st) {
    if constexpr (std::is_same<H, Md5>::value) {
        asm volatile("v_mov_b32 %0, 0x67452301" : "=v"(st.s[0]));
        asm volatile("v_mov_b32 %0, 0xefcdab89" : "=v"(st.s[1]));
        asm volatile("v_mov_b32 %0, 0x98badcfe" : "=v"(st.s[2]));
        asm volatile("v_mov_b32 %0, 0x10325476" : "=v"(st.s[3]));
    } else {
        st.init();
    }
}

// The HMAC mid-state pointer re-defined per use: its words (wave-uniform
// for one key) are loaded where needed instead of being hoisted into 8
// SGPRs held across the line loop.
__device__ __forceinline__ const uint32_t* tile_mid(const KArgs& a) {
    const uint32_t* mid = a.mid;
    asm volatile("" : "+s"(mid));
    return gptr(mid);
}

template <class H, int kMode>
__device__ __forceinline__ void tile_finish(const KArgs& a, H& st, const TileRec& r) {
    uint32_t dw[H::kDigest / 4];
    st.digest_words(dw);
    if (kMode == kTileHmac || kMode == kTileKeyedHmac) {
        const uint32_t* mid = tile_mid(a);
        if (kMode == kTileKeyedHmac) mid += (uint64_t)key_of(a, r.idx) * 2 * kMidWords;
        H o;
        load_words(o.s, mid + kMidWords);   // state after K ^ opad
        md_outer(o, dw);
        o.digest_words(dw);
    }
    bool store = r.valid;
    if constexpr (kMode == kTileKeyedHmac || kMode == kTileKeyedSuffix) store = store && !batch_aborted(a);
    if (store) store_digest<H::kDigest>(a.digests + (uint64_t)r.idx * H::kDigest, dw);
}

template <class H, int kMode>
__device__ __forceinline__ void tile_state(const KArgs& a, const TileRec& r, H& st, TileMsg<H, kMode>& m) {
    m.prefix = 0;
    m.total = r.len;
    m.K = nullptr;
    m.kl = 0;
    if (kMode == kTileHmac || kMode == kTileKeyedHmac) {
        const uint32_t* mid = tile_mid(a);
        if (kMode == kTileKeyedHmac) mid += (uint64_t)key_of(a, r.idx) * 2 * kMidWords;
        load_words(st.s, mid);              // state after K ^ ipad
        m.prefix = H::kBlock;
    } else {
        tile_init(st);
    }
    if (kMode == kTileKeyedSuffix) {
        const uint32_t k = key_of(a, r.idx);
        m.K = gptr(a.keys) + gptr(a.key_off)[k];
        m.kl = gptr(a.key_len)[k];
        m.total += m.kl;
    }
}

// Per-lane message loop for a tile whose records do not share a phase.
template <class H, int kMode>
__device__ __forceinline__ void md_tile_direct(const KArgs& a, const TileRec& r) {
    H st;
    TileMsg<H, kMode> m;
    tile_state(a, r, st, m);
    if (kMode == kTileKeyedSuffix) md_message2(st, r.p, r.len, m.K, m.kl, 0);
    else md_message(st, r.p, r.len, m.prefix);
    tile_finish<H, kMode>(a, st, r);
}

// Wave-level reductions by DPP (no LDS round trips): the 16-lane rows by
// quad_perm xor 1, xor 2, row_half_mirror and row_mirror (each lane ends
// with its row's result), the four rows combined on the SALU.  The tile
// geometry's seven reductions were 6-deep ds_bpermute chains (r3: ~2 us per
// tile with no line in flight, tools/tile_trace.py).
constexpr int kDppQuadXor1 = 0xB1, kDppQuadXor2 = 0x4E, kDppRowHalfMirror = 0x141, kDppRowMirror = 0x140;
template <int kCtrl>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v, uint32_t ident) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)v, kCtrl, 0xf, 0xf, false);
}
template <class Op>
__device__ __forceinline__ uint32_t wave_reduce(uint32_t v, uint32_t ident, Op op) {
    v = op(v, dpp_mov<kDppQuadXor1>(v, ident));
    v = op(v, dpp_mov<kDppQuadXor2>(v, ident));
    v = op(v, dpp_mov<kDppRowHalfMirror>(v, ident));
    v = op(v, dpp_mov<kDppRowMirror>(v, ident));
    const uint32_t r0 = __builtin_amdgcn_readlane(v, 0), r1 = __builtin_amdgcn_readlane(v, 16);
    const uint32_t r2 = __builtin_amdgcn_readlane(v, 32), r3 = __builtin_amdgcn_readlane(v, 48);
    return op(op(r0, r1), op(r2, r3));
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    return wave_reduce(v, 0u, [](uint32_t x, uint32_t y) { return x > y ? x : y; });
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    return wave_reduce(v, ~0u, [](uint32_t x, uint32_t y) { return x < y ? x : y; });
}
__device__ __forceinline__ int32_t wave_max_i32(int32_t v) {
    return (int32_t)wave_reduce((uint32_t)v, 0x80000000u,
                                [](uint32_t x, uint32_t y) { return (int32_t)x > (int32_t)y ? x : y; });
}
__device__ __forceinline__ int32_t wave_min_i32(int32_t v) {
    return (int32_t)wave_reduce((uint32_t)v, 0x7fffffffu,
                                [](uint32_t x, uint32_t y) { return (int32_t)x < (int32_t)y ? x : y; });
}
// OR over the lane's group of 8 (lanes 8q .. 8q + 7): quad xor 1, xor 2,
// then row_half_mirror pairs the two quads.
__device__ __forceinline__ uint32_t group8_or(uint32_t v) {
    v |= dpp_mov<kDppQuadXor1>(v, 0u);
    v |= dpp_mov<kDppQuadXor2>(v, 0u);
    v |= dpp_mov<kDppRowHalfMirror>(v, 0u);
    return v;
}

// The tile's line stream: line L of the 64 records moves into the wave's
// 8 KiB slab with 8 global_load_lds_dwordx4.  Lane group q (lanes 8q ..
// 8q + 7) carries, in instruction g, the whole 128-B cache line L of record
// j = 8q + g (one of its own lanes' records), lane 8q + c the record's chunk
// c + m_j (mod 8; m_j: record j's chunk rotation): the texture unit sees 8
// whole cache lines per instruction.  Instruction g lands at slab + g * kRow
// (kRow = 1,040: 1 KiB plus one 16-B slot), so record j's row starts at
// (j & 7) * 1040 + (j >> 3) * 128, in bank group ((j & 7) + 8 (j >> 3)) mod 16,
// and its rotated chunk k is the row's slot k: the 16 lanes of every
// ds_read_b128 group start in 16 different bank groups, and take() reads
// the 8 chunks at one base plus immediate offsets (no per-chunk address
// VALU; the XOR-swizzled rows of 8 KiB slabs took 8 v_xor per line).
// Addressing: the saddr form, a wave-uniform scalar
// base (the tile's lowest stream base + 128 L) plus one 32-bit offset per
// instruction (8 VGPRs; md_tile_stream checks that the tile spans less than
// 4 GiB).  In the last lines (masked) a chunk past its record's last byte is
// fetched from the record's first chunk instead (the data never used).
// Which chunks are valid comes from one word per group per line: every
// lane's count of valid chunks in the line, 4 bits each, OR-reduced in the
// group; the group's rotations travel the same way, 2 bits each, once.
#ifndef LCB_TILE_SKIP
#define LCB_TILE_SKIP 1
#endif
constexpr uint32_t kTileRow = kSlabRow;     // the padded rows of the shared line slab (hash_device.hpp)
constexpr uint32_t kTileSlab = kSlabBytes;
struct TileGatherStream {
    uint8_t* slab;
    uint32_t lane;
    const uint8_t* tb;      // wave-uniform: the tile's lowest stream base
    uint32_t voff[8];       // instruction g: this lane's chunk of record 8 (lane >> 3) + g, bytes from tb
    // The rotations of the lane's group of 8 records, 2 bits each.
    __device__ __forceinline__ static uint32_t group_rot(uint32_t m, uint32_t ln) {
        return group8_or(m << (2u * (ln & 7u)));
    }
    __device__ __forceinline__ void init(const uint8_t* tile_base, uint32_t rel, uint32_t m, uint32_t ln,
                                         uint8_t* my_slab) {
        lane = ln;
        slab = my_slab;
        tb = tile_base;
        const uint32_t mpk = group_rot(m, ln);
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            const uint32_t rj = (uint32_t)__shfl((int)rel, (int)(ln & ~7u) + g, 64);
            const uint32_t mj = (mpk >> (2 * g)) & 3u;
            voff[g] = rj + (((ln & 7u) + mj) & 7u) * 16u;
        }
    }
    __device__ __forceinline__ void issue(uint32_t L) {
        asm volatile("" : "+v"(voff[0]), "+v"(voff[1]), "+v"(voff[2]), "+v"(voff[3]), "+v"(voff[4]),
                     "+v"(voff[5]), "+v"(voff[6]), "+v"(voff[7]));
        uint64_t so = (uint64_t)L * 128u;
        asm volatile("" : "+s"(so));
        const uint8_t* sb = tb + so;
#pragma unroll
        for (int g = 0; g < 8; ++g)
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(sb + voff[g]),
                                             (__attribute__((address_space(3))) void*)(slab + g * kTileRow), 16, 0,
                                             kLdsAux);
    }
    // lastc: index of this lane's last stream chunk holding a record byte;
    // first: its first chunk holding a record byte in line L (line 0 only,
    // kFirst: start >> 4 & 7; later lines 0).  The chunk k this lane fetches
    // for instruction g is voff[g]'s chunk field ((voff[g] >> 4) & 7: the
    // record's row offset is a multiple of 128), so the group's rotations
    // need no exchange here (r4 rebuilt them with 3 DPP per call and 3 VALU
    // per instruction).
    template <bool kFirst>
    __device__ __forceinline__ void issue_masked(uint32_t L, uint32_t lastc, uint32_t first = 0) {
        // The lane id re-defined per call: the per-lane chunk numbers below
        // are not hoisted out of the tile loop (16 VGPRs held all along).
        uint32_t ln = lane;
        asm volatile("" : "+v"(ln));
        int n = (int)lastc - 8 * (int)L + 1;                    // valid chunks of line L
        n = n < 0 ? 0 : (n > 8 ? 8 : n);
        const uint32_t nv = group8_or((uint32_t)n << (4u * (ln & 7u)));
#if LCB_TILE_SKIP
        uint32_t fv = 0;
        if constexpr (kFirst) fv = group8_or(first << (4u * (ln & 7u)));   // every lane active (DPP)
#endif
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            const uint32_t k = (voff[g] >> 4) & 7u;                      // chunk of the line
#if LCB_TILE_SKIP
            // Only the chunks that hold record bytes are fetched: a lane whose
            // chunk lies past its record's last byte (or, in line 0, before
            // its first) loads the nearest chunk of the line that does
            // instead -- a 16-B piece of a line the other lanes of the same
            // instruction fetch anyway, so no extra memory sector -- and the
            // lanes of a record that ended in an earlier line load nothing
            // (EXEC off: reloading any of its lines re-read HBM).  (Redirecting to the record's first chunk re-read line
            // 0 from HBM; lanes switched off by EXEC cost the branches and the
            // saddr form: profiles/r4_tile_skip_ab.txt.)  1M packets: HBM
            // reads 1.237 -> 1.15 x the algorithmic bytes.
            const uint32_t nk = (nv >> (4 * g)) & 15u;
            uint32_t t = k < nk ? k : nk - 1u;
            if constexpr (kFirst) {
                const uint32_t fk = (fv >> (4 * g)) & 15u;
                t = k < fk ? fk : t;
            }
            const uint32_t v = voff[g] + L * 128u + 16u * t - 16u * k;
            if (nk != 0)   // the record has bytes in line L (uniform in the lane's group)
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(tb + v),
                                                 (__attribute__((address_space(3))) void*)(slab + g * kTileRow), 16, 0,
                                                 kLdsAux);
#else
            const uint32_t v = k < ((nv >> (4 * g)) & 15u) ? voff[g] + L * 128u : voff[g] - 16u * k;
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(tb + v),
                                             (__attribute__((address_space(3))) void*)(slab + g * kTileRow), 16, 0,
                                             kLdsAux);
#endif
        }
    }
    // Waits for the issued line, copies this lane's 128 B (raw LE words, the
    // record's chunks rotated by its m); the slab is free again on return.
    __device__ __forceinline__ void take(uint32_t y[32]) const {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        using lds_cu4 = __attribute__((address_space(3))) const v4u;
        // The row base (one VGPR); the 8 chunks at immediate offsets.
        const uint32_t b = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint8_t*)slab) +
                           (lane & 7u) * kTileRow + (lane >> 3) * 128u;
        lds_cu4* row = (lds_cu4*)(uintptr_t)b;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const v4u v = row[k];
            y[4 * k] = v.x; y[4 * k + 1] = v.y; y[4 * k + 2] = v.z; y[4 * k + 3] = v.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
};

#ifndef LCB_TILE_PRIO
#define LCB_TILE_PRIO 1
#endif
// Segmented jobs run without the priority (equal jobs in dispatch order;
// C4 same-process A/B: SHA-1 -1.3 %, MD5 and SHA-256 within 0.2 %,
// profiles/r5_c4_segs_ab.txt), as in md_lines_kernel.
#ifndef LCB_TILE_ONECOPY
#define LCB_TILE_ONECOPY 0
#endif
#ifndef LCB_TILE_SEG_PRIO
#define LCB_TILE_SEG_PRIO 0
#endif
// Wave priority by remaining lines, longest remaining first (set every 16
// lines; tiles under 128 lines stay at 0).  Among a SIMD's waves the arbiter
// otherwise favours the oldest, so of two long tiles the younger, with more
// left to do, ends last: in C4 the first round of 64 KiB tiles ended between
// 1.1 and 2.9 ms, the second round's last tiles ran alone for the last
// 0.8 ms (tools/tile_trace.py).  C4 4.54 -> 4.35 ms, packets and 1 KiB
// records unchanged (profiles/r4_tile_prio_ab.txt).
__device__ __forceinline__ void tile_prio(uint32_t left) {
    if (left >= 384) __builtin_amdgcn_s_setprio(3);
    else if (left >= 256) __builtin_amdgcn_s_setprio(2);
    else if (left >= 128) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

// Tiles whose records all start on a 16-B boundary (R = 0, no byte shift:
// C4's packed 64 B / 1 KiB / 64 KiB records, arrays of aligned records) run
// a copy of the line loop without the per-word v_alignbyte (32 VALU per
// line): C4 4.21 -> 4.05 ms, 1 KiB records -1.5 %, packets unchanged
// (profiles/r4_tile_a16_ab.txt).
#ifndef LCB_TILE_A16
#define LCB_TILE_A16 1
#endif
// kSeg: the copy that runs segmented jobs (js.nsegs > 1); the other is
// compiled without any segment path, as the packet tiles were before
// segments (same-process A/B: one copy with both paths ran packets 0.5 %
// slower).
template <class H, int kMode, int kR, bool kA16, bool kSeg>
__device__ __forceinline__ void md_tile_stream(const KArgs& a, const TileRec& r, uint32_t lane, uint8_t* slab,
                                               const TileSeg& js LCB_TRACE(, TileTrace& tr)) {
    const uint32_t p32 = (uint32_t)reinterpret_cast<uintptr_t>(r.p);
    const uint32_t sh = p32 & 3u;
    const uint32_t off = p32 & 127u;              // stream offset of the record's first byte
    const uint32_t h = off >> 6, m = (off >> 4) & 3u;
    // h re-derived from the start at each use (one v_bfe), not held in a
    // VGPR through the line loop.
    auto half = [&]() { uint32_t v = p32; asm volatile("" : "+v"(v)); return (v >> 6) & 1u; };
    const uint64_t len = r.len;
    H st;
    TileMsg<H, kMode> m_;
    tile_state(a, r, st, m_);
    // Geometry: lines holding record bytes (max, and min of lines wholly
    // inside the record), blocks of the padded (virtual) message + h (max),
    // lines whose two blocks are whole message blocks (min), whole message
    // blocks (min).
    const uint64_t end = off + len;                          // record end, in stream bytes
    // The tile's stream bases: 32-bit offsets from the lowest (saddr form)
    // when the tile spans less than 4 GiB, else the per-lane loop.  Bases
    // are compared as signed 128-B line deltas from lane 0's, so each bound
    // is one 32-bit reduction.  These three reductions come first: line 0
    // is issued (masked: it is right for any record) before the rest of
    // the geometry, whose reductions then run under its latency.
    const uint32_t NL = wave_max_u32((uint32_t)((end + 127u) >> 7));
    const uint64_t base = (uint64_t)reinterpret_cast<uintptr_t>(r.p) - off;
    const uint64_t b0 = readfirstlane64(base);
    const int64_t d = (int64_t)(base - b0);
    const bool near = d > -(1ll << 38) && d < (1ll << 38);
    const int32_t dl = (int32_t)(d >> 7);
    const int32_t dmin = wave_min_i32(dl), dmax = wave_max_i32(dl);
    const uint64_t lo = b0 + (uint64_t)((int64_t)dmin * 128);
    // The span in lines, in 64 bits (dmax - dmin of two int32 may exceed int32).
    const uint64_t span_lines = (uint64_t)((int64_t)dmax - (int64_t)dmin);
    if (!__all(near) || (span_lines + NL + 1) * 128u >= (1ull << 32) || !__all(end != off)) {
        if (kSeg && js.seg != 0) return;     // segment 0 of a segmented tile runs it whole
        if (kMode == kTileKeyedSuffix) md_message2(st, r.p, r.len, m_.K, m_.kl, 0);
        else md_message(st, r.p, r.len, m_.prefix);
        tile_finish<H, kMode>(a, st, r);
        return;
    }
    const uint32_t lastc = (uint32_t)((end - 1) >> 4);
    TileGatherStream ls;
    ls.init(reinterpret_cast<const uint8_t*>(lo), (uint32_t)(dl - dmin) * 128u, m, lane, slab);
    auto issue0 = [&]() {
        if (__all(lastc >= 7u && off < 16u)) ls.issue(0);           // every lane's whole line 0
        else ls.issue_masked<true>(0, lastc, off >> 4);
    };
    if (!kSeg || js.seg == 0) issue0();
    // The rest of the geometry: lines wholly inside every record (min),
    // blocks of the padded (virtual) message + h (max), lines whose two
    // blocks are whole message blocks (min), whole message blocks (min).
    const uint32_t nblk = (uint32_t)((m_.total + 8u) >> 6) + 1u;
    const uint32_t nf = r.len >> 6;
    const uint32_t NS = wave_min_u32((uint32_t)(end >> 7));
    const uint32_t NB = wave_max_u32(nblk + h), NF = wave_min_u32(nf);
    uint32_t LF = wave_min_u32((nf + h + 1u) >> 1);
    if (LF > NL) LF = NL;
    LCB_TRACE(tr.mark(1); tr.w[6] = NL;)
    // No lane's chunks rotated (every start on a 64-B half line, as in C4):
    // the carry needs no merge (wave-uniform).
    const bool rotated = !__all(m == 0);
    auto issue = [&](uint32_t L) {
        if (L >= NS) ls.issue_masked<false>(L, lastc);
        else ls.issue(L);
    };
    // This job's whole-block lines [Lb, Le); a segment before the last
    // stops there (suspend) and streams no further line.
    uint32_t Lb = 0, Le = LF;
    bool suspend = false;
    // (Not in the keyed-suffix mode: its MD5 kernel is at 128 VGPRs without
    // the segment paths; launch_ordered segments no suffix batch.)
    constexpr bool kSegOK = kSeg && LCB_TILE_SEG && kMode != kTileKeyedSuffix;
    if constexpr (kSegOK) {
        // too short to cut, or lines past the whole-block ones are much of
        // the tile (mixed lengths: the last segment would run them behind
        // every other job): segment 0 runs it whole, up front
        if (LF < (uint32_t)js.nsegs + 2u || 8ull * LF < 7ull * NL) {
            if (js.seg != 0) return;
        } else {
            bool whole = false;
            if (js.seg > 0) {
                if (!seg_wait(js, &whole)) return;
                if (whole) issue0();
                else Lb = seg_line(LF, js.seg, js.nsegs);
            }
            if (!whole && js.seg + 1 < js.nsegs) {
                Le = seg_line(LF, js.seg + 1, js.nsegs);
                suspend = true;
            }
        }
    }
    const uint32_t LE = kSegOK && suspend ? Le : NL;   // lines streamed
    TileKeep kp;      // the merge's keep masks (lane masks, once per tile)
    kp.init(m);
    uint32_t c[16];   // dwords 16..31 of the previous (rotated) line: the carry
    // Whole-block lines: both blocks of line L (2L - 1 - h and 2L - h) are
    // whole message blocks of every lane.  Two line buffers in turn, the
    // loop unrolled by two so that which buffer holds the carry is fixed at
    // compile time: line L lands in one buffer while the other's upper half
    // (dwords 16..31 of line L - 1) is the carry, merged in place -- no
    // per-line copy of the carry (16 v_mov per line before).  MD5 only: the
    // unrolled loop of SHA-1 / SHA-224/256 (~45 KiB of code per dword phase,
    // four phases hot at once) ran 2.7-2.9 % slower on packets than the
    // rolled one despite 1.2 % fewer VALU (instruction cache), and their
    // carry copy is 0.6 % of a line's VALU (profiles/r5_tile_ab.txt).
    constexpr bool kTwoBuf = std::is_same<H, Md5>::value;
    // Resume: the saved state, and line Lb - 1 again for the carry.
    auto resume = [&](uint32_t* yprev) {
        if constexpr (kSegOK) {
            seg_load(st.s, js.lane_state());
            issue(Lb - 1u);
            ls.take(yprev);
            if (Lb < LE) issue(Lb);
        }
    };
    uint32_t L = Lb;
    if constexpr (!kTwoBuf) {
        if (kSegOK && Lb > 0) {
            uint32_t y[32];
            resume(y);
#pragma unroll
            for (int k = 0; k < 16; ++k) c[k] = y[16 + k];
        }
        for (; L < Le; ++L) {
            uint32_t y[32];
#if LCB_TILE_PRIO
            if ((!kSeg || LCB_TILE_SEG_PRIO) && (L & 15u) == 0) tile_prio(NL - L);
#endif
            ls.take(y);
            LCB_TRACE(if (L == 0) tr.mark(2); if (L + 1 == NL) tr.mark(3);)
            if (L + 1 < LE) issue(L + 1);
            uint32_t w[16];
            if (L > 0) {   // block 2L - 1 - h: the carry merged with this line's wrapped chunks
                if (rotated) tile_merge(c, y, kp);
                tile_shift<kR, kA16>(c, y, sh, w);
                tile_compress(st, w);
            }
            tile_shift<kR, kA16>(y, y + 16, sh, w);   // block 2L - h: the rotated line's words R..R+16
            if (L > 0 || half() == 0) tile_compress(st, w);
#pragma unroll
            for (int k = 0; k < 16; ++k) c[k] = y[16 + k];
        }
    } else if (Le) {
        uint32_t ya[32], yb[32];
        // Line L into y, cr = the other buffer's upper half (the carry).
        auto whole_line = [&](uint32_t Ln, uint32_t* y, uint32_t* cr) {
#if LCB_TILE_PRIO
            if ((!kSeg || LCB_TILE_SEG_PRIO) && (Ln & 15u) == 0) tile_prio(NL - Ln);
#endif
            ls.take(y);
            LCB_TRACE(if (Ln + 1 == NL) tr.mark(3);)
            if (Ln + 1 < LE) issue(Ln + 1);
            uint32_t w[16];
            // block 2L - 1 - h: the carry merged with this line's wrapped chunks
            if (rotated) tile_merge(cr, y, kp);
            tile_shift<kR, kA16>(cr, y, sh, w);
            tile_compress(st, w);
            tile_shift<kR, kA16>(y, y + 16, sh, w);   // block 2L - h: the rotated line's words R..R+16
            tile_compress(st, w);
        };
        if (!kSegOK || Lb == 0) {   // line 0: no carry block; its own block only when the record starts in the first half
#if LCB_TILE_PRIO
            if (!kSeg || LCB_TILE_SEG_PRIO) tile_prio(NL);
#endif
            ls.take(ya);
            LCB_TRACE(tr.mark(2); if (NL == 1) tr.mark(3);)
            if (1 < LE) issue(1);
            uint32_t w[16];
            tile_shift<kR, kA16>(ya, ya + 16, sh, w);
            if (half() == 0) tile_compress(st, w);
            L = 1;
        } else {
            resume(ya);
        }
        for (; L + 1 < Le; L += 2) {
            whole_line(L, yb, ya + 16);
            whole_line(L + 1, ya, yb + 16);
        }
        if (L < Le) {
            whole_line(L, yb, ya + 16);
            ++L;
#pragma unroll
            for (int k = 0; k < 16; ++k) c[k] = yb[16 + k];
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) c[k] = ya[16 + k];
        }
    }
    if constexpr (kSegOK) {
        if (suspend) {
            // Hand the state on, then publish: segment seg + 1 may start.  (A
            // failed exchange: the tile was taken over, nothing to hand on.)
            seg_save(st.s, js.lane_state());
            seg_publish(js.flag, js.seg);
            return;
        }
    }
    // The rest, line by line (tile_block: ends of messages, a keyed suffix,
    // padding, length);
    // lines past the last streamed one are zeros (those bytes lie past every
    // record's end).
    for (; 2 * L <= NB; ++L) {   // block 2L - 1 - h < nblk for some lane
        uint32_t y[32];
        if (L < NL) {
            ls.take(y);
            LCB_TRACE(if (L == 0) tr.mark(2); if (L + 1 == NL) tr.mark(3);)
            if (L + 1 < NL) issue(L + 1);
        } else {
#pragma unroll
            for (int k = 0; k < 32; ++k) y[k] = 0u;
        }
        uint32_t w[16];
        if (L > 0) {
            if (rotated) tile_merge(c, y, kp);
            tile_shift<kR, kA16>(c, y, sh, w);
            tile_block<H, kMode>(st, 2 * L - 1 - half(), w, len, m_, nblk, 2 * L - 1 < NF);
        }
        if (2 * L < NB) {
            tile_shift<kR, kA16>(y, y + 16, sh, w);
            tile_block<H, kMode>(st, 2 * L - half(), w, len, m_, nblk, 2 * L < NF && L > 0);
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) c[k] = y[16 + k];
    }
    tile_finish<H, kMode>(a, st, r);
}

// One copy of the line loop per dword phase R: the block window's word
// selection is static (no per-call dispatch and the register moves that
// merge its cases).  kSeg: the copy for segmented jobs.
template <class H, int kMode, bool kSeg>
__device__ __forceinline__ void md_tile_phase(const KArgs& a, const TileRec& r, uint32_t lane, uint8_t* slab,
                                              const TileSeg& js, uint32_t R LCB_TRACE(, TileTrace& tr)) {
    switch (R) {
    case 0:
        if (LCB_TILE_A16 && __all((reinterpret_cast<uintptr_t>(r.p) & 15u) == 0))
            md_tile_stream<H, kMode, 0, true, kSeg>(a, r, lane, slab, js LCB_TRACE(, tr));
        else
            md_tile_stream<H, kMode, 0, false, kSeg>(a, r, lane, slab, js LCB_TRACE(, tr));
        break;
    case 1: md_tile_stream<H, kMode, 1, false, kSeg>(a, r, lane, slab, js LCB_TRACE(, tr)); break;
    case 2: md_tile_stream<H, kMode, 2, false, kSeg>(a, r, lane, slab, js LCB_TRACE(, tr)); break;
    default: md_tile_stream<H, kMode, 3, false, kSeg>(a, r, lane, slab, js LCB_TRACE(, tr)); break;
    }
}

// One tile per wave: the hardware dispatcher hands the tiles out in
// blockIdx order (longest class first), one-wave workgroups (8 KiB of LDS
// each, so a finished wave's slot is free at once).  A persistent grid with
// a tile queue (round 3) ran 4-15 % slower: its waves keep their age for
// the whole kernel and the SIMD's arbiter favours the oldest, so the
// youngest wave of a SIMD ran 2.5x slower per line than the oldest and
// the kernel ended with the starved waves' tiles (tools/tile_trace.py;
// profiles/r4_tile_np_ab.txt).
template <class H, int kMode>
__global__ __launch_bounds__(64, H::kTileOcc) void md_tiles_kernel(KArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t slab[kTileSlab];
    const uint32_t lane = threadIdx.x & 63;
    // The entry count and the tile's `order` entries load together (`order`
    // covers the whole grid, bucket_order_words): three round trips to the
    // first line's issue (kernel arguments, entries, offsets and lengths)
    // instead of five.  The asm keeps the entry load above the exit branch.
    // (16-B records written by the bucketing -- address, length, index --
    // save one more round trip but cost the bucketing a gather and 12 B
    // more per entry: 2 % slower on the packets, profiles/r4_tile_rec_ab.txt.)
    // Segmented long tiles (a.seg): the first kSegs x nseg blocks are their
    // jobs, segment-major; the rest are the other tiles, in order.
    TileSeg js;
    const uint64_t t = seg_job(a, blockIdx.x, js);
    // (the entry load stays inside `order`, which covers the unsegmented grid)
    const uint64_t tmax = bucket_tiles_max(a.count) - 1;
    uint32_t ent = gptr(a.order)[(t < tmax ? t : tmax) * 64 + lane];
    uint32_t norder = gptr(a.tile_next)[1];   // entries (pads included), from the bucketing
    asm volatile("" : "+v"(ent), "+s"(norder));
    const uint64_t ntiles = (norder + 63) / 64;
    if (t >= ntiles) return;                   // the grid is an upper bound
    TileRec r;
    r.valid = t * 64 + lane < norder && ent != kOrderPad;
    // lane 0's entry, read with every lane active (never a pad: t < ntiles)
    const uint32_t ent0 = (uint32_t)__builtin_amdgcn_readfirstlane(ent);
    r.idx = r.valid ? ent : ent0;
    r.p = gptr(a.data) + (a.offsets ? gptr(a.offsets)[r.idx] : (uint64_t)r.idx * a.stride);
    r.len = a.lengths ? gptr(a.lengths)[r.idx] : a.fixed_len;
    LCB_TRACE(TileTrace tr; tr.w[1] = tr.w[2] = tr.w[3] = 0; tr.w[6] = 0;
              const uint64_t trc = __builtin_amdgcn_s_memtime(); tr.mark(0); tr.w[5] = trace_hwid();)
    // The tile's dword phase R (uniform after the bucketing), or a mixed tile.
    const uint32_t Rl = ((uint32_t)reinterpret_cast<uintptr_t>(r.p) >> 2) & 3u;
    const uint32_t R = (uint32_t)__builtin_amdgcn_readfirstlane(Rl);
    // Segmented jobs: plain and HMAC digests of MD5, SHA-1 and SHA-224/256
    // (launch_ordered; not the keyed modes).  Each segmented copy of the
    // line loop adds about as much machine code as the unsegmented one, and
    // the code object's size showed in the headline: a library with
    // segmented copies for every mode (33 MB) ran its first 20 timed
    // fixed-stride steps 7 % slower than one without (18 MB), the same
    // kernel, fresh processes alternating (profiles/r6_codesize_headline.txt).
    // HMAC and plain SHA-224 take segmented jobs through
    // ONE copy of their line loop, the segmented one, for segmented and
    // whole tiles alike: no second copy, so no code growth (their packet
    // tiles pay the segment paths' registers: one copy with both paths ran
    // the plain MD5 packets 0.5 % slower).  Plain MD5, SHA-1 and SHA-256
    // keep two copies (the packet rows run the unsegmented one).
    constexpr bool kSha224 = std::is_same<H, Sha256<true>>::value;
    constexpr bool kOneCopy = kMode == kTileHmac || (kMode == kTilePlain && kSha224);
    constexpr bool kSegMode = kMode == kTilePlain || kOneCopy;
    const bool uniform = __all(Rl == R);
    if (js.nsegs > 1 && (!kSegMode || !uniform)) {
        // a segmented tile that cannot be cut: segment 0 runs it whole (one
        // call site per copy below: a second one inlined the copy twice)
        if (js.seg != 0) return;
        js.nsegs = 1;
    }
    if (uniform) {
        if constexpr (kSegMode && (LCB_TILE_ONECOPY || kOneCopy)) {
            md_tile_phase<H, kMode, true>(a, r, lane, slab, js, R LCB_TRACE(, tr));
        } else if constexpr (kSegMode) {
            if (js.nsegs > 1) md_tile_phase<H, kMode, true>(a, r, lane, slab, js, R LCB_TRACE(, tr));
            else md_tile_phase<H, kMode, false>(a, r, lane, slab, js, R LCB_TRACE(, tr));
        } else {
            md_tile_phase<H, kMode, false>(a, r, lane, slab, js, R LCB_TRACE(, tr));
        }
    } else {
        md_tile_direct<H, kMode>(a, r);
    }
    LCB_TRACE(tr.mark(4); tr.w[6] |= t << 16; tr.w[7] = __builtin_amdgcn_s_memtime() - trc;
              tr.put(g_tile_trace, t, lane);)
}

// Launch of the tile kernel on a bucketed batch (a.order, a.tile_next set);
// false if this hash has no tile kernel.
template <class H, int kMode>
__host__ bool launch_tiles(const KArgs& a, hipStream_t s) {
    if constexpr (H::kTileOcc > 0) {
        // One wave per tile; the tile count is known on the device only, so
        // the grid is its upper bound (extra waves leave at once).
        const uint64_t ntiles = bucket_tiles_max(a.count) + (a.seg ? (uint64_t)(kSegs - 1) * a.seg_cap : 0);
        hipLaunchKernelGGL((md_tiles_kernel<H, kMode>), dim3((unsigned)ntiles), dim3(64), 0, s, a);
        return true;
    } else {
        (void)a;
        (void)s;
        return false;
    }
}

}  // namespace lcbgpu
