/*
 * lcb_hash_gpu.h — C-ABI of the MI355X batch digest engine (liblcb_hash_gpu.so).
 *
 * liblcb's hash API (include/crypto/hash/ in the reference) is one
 * message per call, header-only, `static inline`: there is no exported symbol
 * or FFI a batch engine could hook.  The drop-in boundary is therefore:
 *
 *   1. include/crypto/hash/{md5,sha1,sha2,gost3411-2012}.h in THIS repo —
 *      source-compatible restatements of the reference headers (same macros,
 *      types and static inline prototypes), so existing callers such as the
 *      reference's include/proto/radius.h:53 compile unchanged;
 *   2. this header — exported batch counterparts of the reference one-shot
 *      functions.  Each entry point computes, for every message i,
 *      exactly the bytes the named reference function writes.
 *
 * Buffer description (all entry points):
 *   message i starts at  data + (offsets ? offsets[i] : i * stride)
 *   and is               (lengths ? lengths[i] : fixed_len) bytes long;
 *   any byte alignment is accepted (the reference accepts any alignment:
 *   md5.h:146-151, gost3411-2012.h:1123-1128).
 *   digests are packed: digest i occupies digests[i*D .. i*D+D-1],
 *   D = lcb_hash_digest_size(alg).
 *
 * Memory modes (flags):
 *   LCB_HASH_F_DEVICE  data/offsets/lengths/digests are device pointers on the
 *                      current HIP device; the work is enqueued on `stream`
 *                      (a hipStream_t, NULL = default stream) and the call
 *                      returns without waiting.
 *   0                  host pointers; the call stages through pinned memory
 *                      (H2D -> kernel -> D2H, double-buffered) and returns
 *                      when the digests are in `digests`.  `stream` ignored.
 *
 * HMAC: key/key_len are always host memory (RFC 2104 as the reference:
 * a key longer than the block is first replaced by its digest).
 *
 * Errors are liblcb-style errno codes: 0, EINVAL (bad alg/bits/arguments),
 * ENOMEM, ENODEV (no usable MI355X / HIP runtime), EIO (HIP launch or copy
 * failure).  On error no digest is reported as valid.  There is no CPU
 * fallback: the product path fails loudly instead.
 */
#ifndef LCB_HASH_GPU_H
#define LCB_HASH_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LCB_HASH_GPU_ABI_VERSION	1

/* Algorithm ids. */
#define LCB_HASH_MD5		1	/* md5.h */
#define LCB_HASH_SHA1		2	/* sha1.h */
#define LCB_HASH_SHA224		3	/* sha2.h, bits 224 */
#define LCB_HASH_SHA256		4	/* sha2.h, bits 256 */
#define LCB_HASH_SHA384		5	/* sha2.h, bits 384 */
#define LCB_HASH_SHA512		6	/* sha2.h, bits 512 */
#define LCB_HASH_GOST256	7	/* gost3411-2012.h, bits 256 */
#define LCB_HASH_GOST512	8	/* gost3411-2012.h, bits 512 */

/* Flags. */
#define LCB_HASH_F_DEVICE	0x0001u

/* Information. */
int	lcb_hash_gpu_abi_version(void);
size_t	lcb_hash_digest_size(int alg);		/* 0 for an unknown alg */
size_t	lcb_hash_block_size(int alg);		/* 64 or 128; 0 unknown */
int	lcb_hash_gpu_device_count(void);	/* <= 0: no usable device */
const char *lcb_hash_strerror(int error);

/*
 * Generic entry point.  key == NULL: plain digest; key != NULL: HMAC.
 * Replaces `count` calls of the reference's *_get_digest / *_hmac_get_digest.
 */
int	lcb_hash_batch(int alg, const uint8_t *key, size_t key_len,
	    const uint8_t *data, const uint64_t *offsets, const uint32_t *lengths,
	    size_t count, uint64_t stride, uint32_t fixed_len,
	    uint8_t *digests, uint32_t flags, void *stream);

/* Reference-named batch entry points. ---------------------------------- */

/* md5_get_digest(data, data_size, digest)            md5.h:396-402 */
int	md5_get_digest_batch(const uint8_t *data, const uint64_t *offsets,
	    const uint32_t *lengths, size_t count, uint64_t stride,
	    uint32_t fixed_len, uint8_t *digests, uint32_t flags, void *stream);
/* md5_hmac_get_digest(key, key_size, data, data_size, digest)   md5.h:419-425 */
int	md5_hmac_get_digest_batch(const uint8_t *key, size_t key_size,
	    const uint8_t *data, const uint64_t *offsets, const uint32_t *lengths,
	    size_t count, uint64_t stride, uint32_t fixed_len,
	    uint8_t *digests, uint32_t flags, void *stream);

/* sha1_get_digest(data, data_size, digest)           sha1.h:946-954 */
int	sha1_get_digest_batch(const uint8_t *data, const uint64_t *offsets,
	    const uint32_t *lengths, size_t count, uint64_t stride,
	    uint32_t fixed_len, uint8_t *digests, uint32_t flags, void *stream);
/* sha1_hmac_get_digest(key, key_size, data, data_size, digest)  sha1.h:969-975 */
int	sha1_hmac_get_digest_batch(const uint8_t *key, size_t key_size,
	    const uint8_t *data, const uint64_t *offsets, const uint32_t *lengths,
	    size_t count, uint64_t stride, uint32_t fixed_len,
	    uint8_t *digests, uint32_t flags, void *stream);

/* sha2_get_digest(bits, data, data_size, digest, digest_size)   sha2.h:854-865.
 * bits: 224/28, 256/32, 384/48, 512/64 as sha2_init (sha2.h:213-251); any
 * other value is EINVAL (the reference leaves it undefined).  digest_size
 * (may be NULL) receives the per-message digest size. */
int	sha2_get_digest_batch(size_t bits, const uint8_t *data,
	    const uint64_t *offsets, const uint32_t *lengths, size_t count,
	    uint64_t stride, uint32_t fixed_len, uint8_t *digests,
	    size_t *digest_size, uint32_t flags, void *stream);
/* sha2_hmac_get_digest(bits, key, key_size, data, data_size, digest, digest_size)
 * sha2.h:887-894 */
int	sha2_hmac_get_digest_batch(size_t bits, const uint8_t *key,
	    size_t key_size, const uint8_t *data, const uint64_t *offsets,
	    const uint32_t *lengths, size_t count, uint64_t stride,
	    uint32_t fixed_len, uint8_t *digests, size_t *digest_size,
	    uint32_t flags, void *stream);

/* gost3411_2012_get_digest(bits, data, data_size, digest, digest_size)
 * gost3411-2012.h:1962-1973.  bits: 256/32 -> 256; anything else -> 512,
 * exactly as gost3411_2012_init (gost3411-2012.h:1715-1729). */
int	gost3411_2012_get_digest_batch(size_t bits, const uint8_t *data,
	    const uint64_t *offsets, const uint32_t *lengths, size_t count,
	    uint64_t stride, uint32_t fixed_len, uint8_t *digests,
	    size_t *digest_size, uint32_t flags, void *stream);
/* gost3411_2012_hmac_get_digest(bits, key, key_size, data, data_size, digest, digest_size)
 * gost3411-2012.h:1996-2004 */
int	gost3411_2012_hmac_get_digest_batch(size_t bits, const uint8_t *key,
	    size_t key_size, const uint8_t *data, const uint64_t *offsets,
	    const uint32_t *lengths, size_t count, uint64_t stride,
	    uint32_t fixed_len, uint8_t *digests, size_t *digest_size,
	    uint32_t flags, void *stream);

/* Synthetic input: writes bytes [start, start+n) of the stream
 * whose u64 word k (little-endian) is mix64(seed ^ k), into device memory. */
int	lcb_hash_gen_synthetic(uint64_t seed, uint64_t start, uint8_t *dev_out,
	    size_t n, void *stream);

/* Diagnostics: copies the 8 x 256 GOST LPS lookup table the kernels use
 * (generated from the RFC 6986 pi / A constants) to host memory `out`
 * (2048 uint64_t), so tests can pin it against the reference's
 * gost3411_2012_Ax (gost3411-2012.h:184-882). */
int	lcb_hash_gpu_gost_table(uint64_t *out);

#ifdef __cplusplus
}
#endif
#endif /* LCB_HASH_GPU_H */
