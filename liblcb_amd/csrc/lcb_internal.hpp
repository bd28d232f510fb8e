// lcb_internal.hpp — types shared by the kernel TU and the C-ABI TU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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
};

// Words reserved per HMAC mid-state (GOST needs 34: h, N, Sigma).
constexpr int kMidWords = 64;

// Short HMAC key, zero padded to 128 bytes, passed by value.
struct KeyBlock {
    uint32_t w[32];
};

// Length classes for ragged-batch bucketing (see lcb_kernels.hip).
constexpr int kLenClasses = 128;
// Ragged batches at least this large are bucketed by length first.
constexpr uint64_t kBucketMinCount = 4096;

// CRC-32 variants travel through the batch machinery as alg ids
// kCrcAlgBase + variant (variant ids of include/lcb_crc32_gpu.h).
constexpr int kCrcAlgBase = 100;
inline bool is_crc_alg(int alg) { return alg > kCrcAlgBase && alg <= kCrcAlgBase + 8; }

void launch_batch(int alg, const KArgs& a, hipStream_t s);
void launch_crc(int variant, const KArgs& a, hipStream_t s);
void crc_table_host(int variant, uint32_t* out);
void launch_bucketing(const uint32_t* lengths, uint64_t count, uint32_t* work, uint32_t* order,
                      hipStream_t s);
void launch_hmac_prep(int alg, const KeyBlock& kb, const uint8_t* dkey, uint64_t key_len,
                      uint32_t* mid, hipStream_t s);
void launch_gen(uint64_t seed, uint64_t start, uint8_t* out, uint64_t n, hipStream_t s);
void gost_table_host(uint64_t* out);

// Shared by the C-ABI TUs (lcb_hash_gpu.cpp).
size_t dsize(int alg);                  // digest bytes, 0 for an unknown alg
size_t bsize(int alg);                  // block bytes (HMAC key block)
int map_err(hipError_t e);              // HIP error -> liblcb errno code
int ensure_init();                      // 0, or ENODEV without a usable device
// Enqueue the HMAC mid-state prep; *mid / *dkey are stream-ordered
// allocations the caller releases with hipFreeAsync after its last use.
int hmac_setup(int alg, const uint8_t* key, size_t key_len, hipStream_t s, uint32_t** mid,
               uint8_t** dkey_out);
// Batch kernel launch, bucketing a large ragged batch by length first.
int launch_ordered(int alg, KArgs a, hipStream_t s);

}  // namespace lcbgpu
