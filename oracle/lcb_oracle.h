/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C CPU restatement of liblcb's include/crypto/hash path, used as the
 * CHECKER for the MI355X batch kernels.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product (liblcb_amd and
 * the C-ABI library) never links, calls or falls back to anything here.
 *
 * Parity pin: tests/test_oracle_golden.py checks every function below against
 * the reference's own known-answer tables (extracted into tests/golden/kat.json)
 * and against digests produced by the reference itself compiled from
 * /root/reference (oracle/_ref, see oracle/Makefile and tests/golden/make_golden.py).
 *
 * Algorithm ids are shared with include/lcb_hash_gpu.h.
 */
#ifndef LCB_ORACLE_H
#define LCB_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
	OR_MD5 = 1, OR_SHA1 = 2, OR_SHA224 = 3, OR_SHA256 = 4,
	OR_SHA384 = 5, OR_SHA512 = 6, OR_GOST256 = 7, OR_GOST512 = 8
};

/* Digest / block size in bytes; 0 for an unknown id. */
size_t or_digest_size(int alg);
size_t or_block_size(int alg);

/* Streaming context (one struct for every algorithm). */
typedef struct or_ctx_s {
	int alg;
	size_t used;              /* bytes buffered in buf */
	uint64_t count, count_hi; /* message length in bytes (128-bit for SHA-384/512) */
	uint32_t h32[8];          /* MD5 / SHA-1 / SHA-224/256 state */
	uint64_t h64[8];          /* SHA-384/512 state, GOST h */
	uint64_t gn[8], gs[8];    /* GOST counter N and sigma */
	uint8_t buf[128];
} or_ctx_t;

int  or_init(or_ctx_t *c, int alg);                 /* 0 or -1 (unknown alg) */
void or_update(or_ctx_t *c, const uint8_t *d, size_t n);
void or_final(or_ctx_t *c, uint8_t *digest);

/* One-shot digest and RFC 2104 HMAC (block 64, or 128 for SHA-384/512). */
int or_digest(int alg, const uint8_t *d, size_t n, uint8_t *digest);
int or_hmac(int alg, const uint8_t *key, size_t key_len,
    const uint8_t *d, size_t n, uint8_t *digest);

/*
 * Batch helpers with the same buffer-description convention as the GPU ABI:
 * message i starts at base + (offsets ? offsets[i] : i * stride) and is
 * (lengths ? lengths[i] : fixed_len) bytes long; digests are packed
 * count x digest_size.  key == NULL selects the plain digest.
 */
int or_batch(int alg, const uint8_t *key, size_t key_len,
    const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths,
    size_t count, uint64_t stride, uint32_t fixed_len, uint8_t *digests);

/* Keyed batches, as lcb_hash_batch_keyed: mode 1 HMAC(K, m), 2 H(K || m),
 * 3 H(m || K) with K = key key_index[i] (NULL: key 0); -1 on a bad index. */
int or_batch_keyed(int alg, int mode, const uint8_t *keys, const uint64_t *key_offsets,
    const uint32_t *key_lengths, size_t nkeys, const uint32_t *key_index,
    const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths,
    size_t count, uint64_t stride, uint32_t fixed_len, uint8_t *digests);

/*
 * CRC-32 family of include/math/crc32.h (oracle/crc32_oracle.c).  Variant
 * ids are shared with include/lcb_crc32_gpu.h.
 */
enum {
	OR_CRC32A = 1, OR_CRC32CKSUM = 2, OR_CRC32MPEG2 = 3, OR_CRC32B = 4,
	OR_CRC32JAMCRC = 5, OR_CRC32C = 6, OR_CRC32D = 7, OR_CRC32Q = 8
};
int      or_crc32_valid(int variant);
uint32_t or_crc32_table(int variant, int i);	/* byte table entry */
uint32_t or_crc32_update(int variant, uint32_t crc, const uint8_t *d, size_t n);
uint32_t or_crc32(int variant, const uint8_t *d, size_t n);
/* init == NULL: crcs[i] = X(msg i); else crcs[i] = X_update(init[i], msg i). */
int or_crc32_batch(int variant, const uint32_t *init, const uint8_t *base,
    const uint64_t *offsets, const uint32_t *lengths, size_t count,
    uint64_t stride, uint32_t fixed_len, uint32_t *crcs);

/*
 * ChaCha of include/crypto/cipher/chacha.h (oracle/chacha_oracle.c).
 * key_size: 256 or 32 -> 256-bit key, anything else -> 128-bit (chacha.h:289).
 * counter8 / iv8 / iv24 may be NULL (zero).  src NULL -> keystream.
 */
void or_hchacha(const uint8_t *key, size_t key_size, const uint8_t *iv16, size_t rounds, uint8_t *out32);
void or_chacha(const uint8_t *key, size_t key_size, const uint8_t *counter8, const uint8_t *iv8,
    size_t rounds, const uint8_t *src, size_t n, uint8_t *dst);
void or_xchacha(const uint8_t *key, size_t key_size, const uint8_t *counter8, const uint8_t *iv24,
    size_t rounds, const uint8_t *src, size_t n, uint8_t *dst);
/* Buffer i (same layout in src and dst): counters + 8*i, ivs + (x ? 24 : 8)*i. */
int or_chacha_batch(const uint8_t *key, size_t key_size, size_t rounds, int x,
    const uint8_t *counters, const uint8_t *ivs, const uint8_t *src, uint8_t *dst,
    const uint64_t *offsets, const uint32_t *lengths, size_t count, uint64_t stride,
    uint32_t fixed_len);

/* Synthetic-input generator: byte b of the stream is byte
 * (b & 7) of splitmix64_mix(seed ^ (b >> 3)).  Writes n bytes starting at
 * stream byte position `start`. */
uint64_t or_mix64(uint64_t x);
void or_gen_bytes(uint64_t seed, uint64_t start, uint8_t *out, size_t n);

#ifdef __cplusplus
}
#endif
#endif
