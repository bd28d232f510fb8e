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

#define LCB_HASH_GPU_ABI_VERSION	6

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
/* lcb_hash_batch_multi, device mode, diagnostics: parts 1..ndev-1 take the
 * peer-copy path even when they run on devs[0] (a same-device copy), so one
 * GPU exercises the scatter/gather code. */
#define LCB_HASH_F_COPY_PARTS	0x0100u

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

/*
 * Keyed batches: message i uses key k = key_index[i] (NULL: key 0) of a key
 * table — the RADIUS shapes, one shared secret per peer
 * (src/proto/radius_client.c:242,886,1025):
 *   LCB_HASH_KEY_HMAC    digest_i = HMAC(K_k, m_i)   RFC 2104 as the
 *                        *_hmac_get_digest functions; Message-Authenticator
 *                        (include/proto/radius.h:850-919)
 *   LCB_HASH_KEY_PREFIX  digest_i = H(K_k || m_i)    User-Password hiding
 *                        (radius.h:745-830: MD5(secret || authenticator)
 *                        and MD5(secret || c_j) from a copied key context)
 *   LCB_HASH_KEY_SUFFIX  digest_i = H(m_i || K_k)    packet authenticator
 *                        (radius.h:1315-1377: MD5(packet || secret))
 * Key k = keys + (key_offsets ? key_offsets[k] : 0), key_lengths[k] bytes;
 * keys, key_offsets and key_lengths are HOST memory.  key_index lives where
 * the batch does (device memory with LCB_HASH_F_DEVICE).  Per-key state
 * (HMAC ipad/opad mid-states, the prefix's whole-block state) is computed
 * once per key on the device, and kept on the device for later calls with
 * the same key bytes (a per-device cache of up to 16 tables; HMAC keys of
 * lcb_hash_batch share it).  An index >= nkeys is EINVAL in both modes and
 * no digest is written: device mode checks the indices on the device ahead
 * of the batch and gates every digest store on the result; the call waits
 * for that check (so for the work already on `stream`), not for the batch,
 * which stays asynchronous on `stream`.  The host arrays may be released on
 * return.
 */
#define LCB_HASH_KEY_HMAC	1
#define LCB_HASH_KEY_PREFIX	2
#define LCB_HASH_KEY_SUFFIX	3
int	lcb_hash_batch_keyed(int alg, int key_mode, const uint8_t *keys,
	    const uint64_t *key_offsets, const uint32_t *key_lengths, size_t nkeys,
	    const uint32_t *key_index, const uint8_t *data, const uint64_t *offsets,
	    const uint32_t *lengths, size_t count, uint64_t stride,
	    uint32_t fixed_len, uint8_t *digests, uint32_t flags, void *stream);

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

/* Multi-device batches. ---------------------------------
 *
 * lcb_hash_partition: cut a batch into `nparts` contiguous message ranges of
 * balanced work (message bytes + one 64-B padding block each; lengths NULL:
 * equal counts).  Part p = messages [first[p], first[p+1]); `first` holds
 * nparts + 1 entries, lengths are HOST memory.  The bench's one-process-per-
 * GPU mode shards with the same rule.
 *
 * lcb_hash_batch_multi: lcb_hash_batch with the batch split by
 * lcb_hash_partition over devs[0..ndev-1] (HIP device ordinals; repeats
 * allowed), all parts concurrently; returns when every digest is written.
 *   flags 0                 host memory, one staging pipeline per part;
 *                           `stream` ignored;
 *   flags LCB_HASH_F_DEVICE data/offsets/lengths/digests are device memory on
 *                           devs[0]; a part on another device is copied peer-
 *                           to-peer (xGMI), hashed there, and its digests are
 *                           copied back into `digests` on devs[0].  `stream`
 *                           (a hipStream_t of devs[0], NULL = its default
 *                           stream) orders the call: every part starts after
 *                           the work enqueued on `stream` before the call (an
 *                           event recorded there at entry), so the caller may
 *                           write the batch asynchronously on it and call
 *                           without a host synchronisation (ABI v4; v3 had no
 *                           `stream` and required complete inputs).
 * LCB_HASH_F_COPY_PARTS without LCB_HASH_F_DEVICE is EINVAL.
 * With devs = {d} it equals lcb_hash_batch on device d.  Errors: EINVAL,
 * ENODEV (an ordinal out of range), ENOMEM, EIO.
 * Device mode enables peer access from every device to devs[0] once
 * (hipDeviceEnablePeerAccess) and enqueues every remote part's copies
 * before it waits for any part; part streams and buffers are pooled per
 * device.  A ragged (or offsets) batch is split on devs[0] itself, behind
 * the caller's work on `stream`: the parts and each part's byte span are
 * computed there and only they are read back (ABI v6; v5 copied every
 * offset and length to the host).  lcb_hash_multi_stats reports what the
 * device-mode calls did (ABI v5, host time v6). */
int	lcb_hash_partition(const uint32_t *lengths, size_t count,
	    uint32_t fixed_len, size_t nparts, uint64_t *first);
int	lcb_hash_batch_multi(const int *devs, int ndev, int alg,
	    const uint8_t *key, size_t key_len, const uint8_t *data,
	    const uint64_t *offsets, const uint32_t *lengths, size_t count,
	    uint64_t stride, uint32_t fixed_len, uint8_t *digests, uint32_t flags,
	    void *stream);
typedef struct lcb_hash_multi_stats_s {
	uint64_t	calls;		/* device-mode lcb_hash_batch_multi calls */
	uint64_t	remote_parts;	/* parts hashed on a copy (another device, or COPY_PARTS) */
	uint64_t	parts_enqueued_before_wait; /* remote parts whose copies, batch and
					 * digest copy-back were all enqueued before the
					 * call's first wait on any part */
	uint64_t	peer_enabled;	/* device pairs (d -> devs[0]) with peer access on */
	uint64_t	peer_unavailable; /* pairs where hipDeviceCanAccessPeer said no:
					 * the runtime stages their copies */
	uint64_t	host_ns;	/* host time of the device-mode calls from entry
					 * until every part was enqueued (ABI v6) */
	uint64_t	split_ns;	/* of which the split on devs[0] and its read-back */
	uint64_t	device_splits;	/* calls split on devs[0] (ragged or offsets) */
} lcb_hash_multi_stats_t;
int	lcb_hash_multi_stats(lcb_hash_multi_stats_t *out);

/* Key cache (ABI v6).  Key tables of keyed batches and single HMAC keys
 * are uploaded, prepared (mid-states) and cached per device by their bytes,
 * at most 16 entries, least recently used evicted first.  The cache holds
 * secrets: an evicted entry's device buffer is zeroed before it is freed and
 * its host copy wiped (the reference zeroises its pads, md5.h:337,358).
 * lcb_hash_key_cache_flush drops and zeroes every entry (it synchronises the
 * devices that hold one; EBUSY if a call in progress holds an entry, which
 * then stays); lcb_hash_key_cache_entries counts the live entries.  The
 * environment variable LCB_HASH_KEY_CACHE=0 turns the cache off: every call
 * uploads its keys to a per-call buffer, zeroed before it is freed. */
int	lcb_hash_key_cache_flush(void);
size_t	lcb_hash_key_cache_entries(void);

/* Synthetic input: writes bytes [start, start+n) of the stream
 * whose u64 word k (little-endian) is mix64(seed ^ k), into device memory. */
int	lcb_hash_gen_synthetic(uint64_t seed, uint64_t start, uint8_t *dev_out,
	    size_t n, void *stream);

/* Diagnostics: HBM read probe (achievable read bandwidth on
 * the box, measured next to the digest kernels; no reference counterpart).
 * Reads `count` records of `fixed_len` bytes at `stride` from device memory
 * `dev_data` without hashing them.  mode LCB_PROBE_RECORDS: the LDS-DMA line
 * stream of the fixed-stride digest kernels (fixed_len >= 128, stride and
 * dev_data 16-B aligned, count >= 64); `dev_sink` receives count uint32.
 * mode LCB_PROBE_LINEAR: coalesced 16-B loads over count * stride bytes
 * (a multiple of 16); `dev_sink` receives lcb_hash_gpu_probe_sink_words()
 * uint32.  mode LCB_PROBE_GOST_LPS: no memory read at all -- the plain GOST
 * kernel's table gathers alone (its grid and LDS image; per lane the LPS
 * count of a fixed_len-byte message as one dependent chain, dev_data
 * unused): the LDS bound of GOST beside its kernel time; `dev_sink`
 * receives count uint32.  Asynchronous on `stream`.  EINVAL on a shape the
 * mode cannot read. */
#define LCB_PROBE_RECORDS	0
#define LCB_PROBE_LINEAR	1
#define LCB_PROBE_GOST_LPS	2
int	lcb_hash_gpu_read_probe(int mode, const uint8_t *dev_data, size_t count,
	    uint64_t stride, uint32_t fixed_len, uint32_t *dev_sink, void *stream);
size_t	lcb_hash_gpu_probe_sink_words(int mode, size_t count);

/* Diagnostics: engine-clock stamps (no reference
 * counterpart).  Enqueues on `stream` a grid of `slots` one-wave workgroups
 * (a multiple of 8, at most 4096; dealt round robin to the 8 XCDs); lane 0
 * of workgroup b writes three uint64 to dev_out[3 b ..]: XCC_ID << 32 |
 * HW_ID, s_memtime (shader-clock cycles) and s_memrealtime (100 MHz ticks).
 * Two stamps around a run of kernels on the same stream give that run's
 * engine clock per XCD (bench.py clock_window).  EINVAL on a bad shape. */
int	lcb_hash_gpu_clock_stamp(uint64_t *dev_out, size_t slots, void *stream);

/* Diagnostics (tests only): with LCB_SEG_TAKEOVER=1 in the environment, a
 * ragged batch whose long waves are cut into segmented jobs
 * runs those jobs in reverse segment order with no wait, so every cut wave
 * is taken over by its last segment -- the path that keeps a job from
 * waiting forever -- and the call synchronises and reads the waves' flags
 * back.  out[4] = {cut waves, taken over, completed in segment order,
 * other} of the last such batch. */
int	lcb_hash_gpu_seg_last(uint32_t *out);

/* Diagnostics: copies the 8 x 256 GOST LPS lookup table the kernels use
 * (generated from the RFC 6986 pi / A constants) to host memory `out`
 * (2048 uint64_t), so tests can pin it against the reference's
 * gost3411_2012_Ax (gost3411-2012.h:184-882). */
int	lcb_hash_gpu_gost_table(uint64_t *out);

#ifdef __cplusplus
}
#endif
#endif /* LCB_HASH_GPU_H */
