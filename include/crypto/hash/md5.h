/*
 * crypto/hash/md5.h — source-compatible drop-in for liblcb's md5.h
 * (reference include/crypto/hash/md5.h), clean-room.
 *
 * Same macros, types and `static inline` prototypes as the reference
 * (md5.h:50-435), so callers such as include/proto/radius.h compile
 * unchanged.  This is the one-message CPU path (per-packet, latency-bound);
 * batches of buffers go to the MI355X through include/lcb_hash_gpu.h.
 * Behaviour notes kept from the reference:
 *   - ctx->count counts BYTES (md5.h:113 says bits, the code uses bytes);
 *   - *_final() zeroizes the context (md5.h:287) — re-init before reuse;
 *   - contexts are plain copyable structs (radius.h snapshots mid-states).
 * RFC 1321 (MD5), RFC 2104 (HMAC).
 */
#ifndef __MD5_H__INCLUDED__
#define __MD5_H__INCLUDED__

#include <sys/param.h>
#include <sys/types.h>
#include <string.h>
#include <inttypes.h>

#ifndef nitems
#	define nitems(__val)	(sizeof(__val) / sizeof(__val[0]))
#endif

#define MD5_HASH_SIZE		16
#define MD5_HASH_STR_SIZE	(MD5_HASH_SIZE * 2)
#define MD5_MSG_BLK_SIZE	64
#define MD5_MSG_BLK_SIZE_MASK	(MD5_MSG_BLK_SIZE - 1)
#define MD5_MSG_BLK_64CNT	(MD5_MSG_BLK_SIZE / sizeof(uint64_t))

typedef struct md5_ctx_s {
	uint32_t hash[(MD5_HASH_SIZE / sizeof(uint32_t))];
	uint64_t count;				/* bytes hashed so far */
	uint64_t buffer[MD5_MSG_BLK_64CNT];	/* partial block */
} md5_ctx_t, *md5_ctx_p;

typedef struct hmac_md5_ctx_s {
	md5_ctx_t ctx;
	uint64_t k_opad[MD5_MSG_BLK_64CNT];
} hmac_md5_ctx_t, *hmac_md5_ctx_p;

/* Zeroization the optimiser cannot drop. */
static void *(*volatile md5_wipe_fn)(void *, int, size_t) = memset;

static inline uint32_t
md5_rol32(const uint32_t x, const unsigned n) {
	return ((x << n) | (x >> (32 - n)));
}

static inline void
md5_init(md5_ctx_p ctx) {
	ctx->hash[0] = 0x67452301;
	ctx->hash[1] = 0xefcdab89;
	ctx->hash[2] = 0x98badcfe;
	ctx->hash[3] = 0x10325476;
	ctx->count = 0;
}

/* One 64-byte block, any alignment. */
static inline void
md5_transform(md5_ctx_p ctx, const uint8_t *block) {
	static const uint32_t T[64] = {
		0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
		0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
		0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
		0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
		0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
		0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
		0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
		0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391
	};
	static const uint8_t S[16] = { 7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21 };
	uint32_t x[16], v[4], a, t;
	size_t i, g;

	memcpy(x, block, sizeof(x));	/* little-endian words, any alignment */
#if defined(__BYTE_ORDER__) && (__BYTE_ORDER__ == __ORDER_BIG_ENDIAN__)
	for (i = 0; i < 16; i ++) {
		x[i] = __builtin_bswap32(x[i]);
	}
#endif
	memcpy(v, ctx->hash, sizeof(v));
	/* Four 16-step rounds, each a loop the compiler fully unrolls so the
	 * word index, constant and rotation fold to immediates.  Each step
	 * starts from a + (x[g] + T[i]), which does not wait for the previous
	 * step, so only the round function, one add, the rotate and the add of
	 * b sit on the chain; round 2's G is added as its two disjoint terms
	 * (c & ~d) + (b & d), the first of which does not wait for b either. */
#define MD5_ROUND(__r, __g, __fn) do {						\
	_Pragma("GCC unroll 16")						\
	for (i = 16 * (__r); i < 16 * (__r) + 16; i ++) {			\
		g = (__g);							\
		a = v[0] + (x[g] + T[i]);					\
		__fn;								\
		t = v[3];							\
		v[3] = v[2];							\
		v[2] = v[1];							\
		v[1] += md5_rol32(a, S[4 * (__r) + (i & 3)]);			\
		v[0] = t;							\
	}									\
} while (0)
	MD5_ROUND(0, i, a += (v[3] ^ (v[1] & (v[2] ^ v[3]))));
	MD5_ROUND(1, ((5 * i + 1) & 15), (a += (v[2] & ~v[3]), a += (v[1] & v[3])));
	MD5_ROUND(2, ((3 * i + 5) & 15), a += (v[1] ^ v[2] ^ v[3]));
	MD5_ROUND(3, ((7 * i) & 15), a += (v[2] ^ (v[1] | ~v[3])));
#undef MD5_ROUND
	for (i = 0; i < 4; i ++) {
		ctx->hash[i] += v[i];
	}
}

static inline void
md5_update(md5_ctx_p ctx, const uint8_t *data, const size_t data_size) {
	size_t used = (size_t)(ctx->count & MD5_MSG_BLK_SIZE_MASK), n = data_size, take;

	ctx->count += data_size;
	if (0 != used) {
		take = (MD5_MSG_BLK_SIZE - used);
		if (take > n) {
			take = n;
		}
		memcpy(((uint8_t*)ctx->buffer) + used, data, take);
		used += take;
		data += take;
		n -= take;
		if (MD5_MSG_BLK_SIZE != used)
			return;
		md5_transform(ctx, (const uint8_t*)ctx->buffer);
	}
	for (; n >= MD5_MSG_BLK_SIZE; n -= MD5_MSG_BLK_SIZE, data += MD5_MSG_BLK_SIZE) {
		md5_transform(ctx, data);
	}
	if (0 != n) {
		memcpy(ctx->buffer, data, n);
	}
}

static inline void
md5_final(md5_ctx_p ctx, uint8_t *digest) {
	uint8_t *buf = (uint8_t*)ctx->buffer;
	size_t used = (size_t)(ctx->count & MD5_MSG_BLK_SIZE_MASK), i;
	uint64_t bits = (ctx->count << 3);

	buf[used ++] = 0x80;
	if (used > (MD5_MSG_BLK_SIZE - 8)) {
		memset(buf + used, 0x00, (MD5_MSG_BLK_SIZE - used));
		md5_transform(ctx, buf);
		used = 0;
	}
	memset(buf + used, 0x00, ((MD5_MSG_BLK_SIZE - 8) - used));
	for (i = 0; i < 8; i ++) {	/* little-endian bit count */
		buf[(MD5_MSG_BLK_SIZE - 8) + i] = (uint8_t)(bits >> (8 * i));
	}
	md5_transform(ctx, buf);
	for (i = 0; i < MD5_HASH_SIZE; i ++) {
		digest[i] = (uint8_t)(ctx->hash[i >> 2] >> (8 * (i & 3)));
	}
	md5_wipe_fn(ctx, 0x00, sizeof(md5_ctx_t));
}

static inline void
hmac_md5_init(const uint8_t *key, const size_t key_len, hmac_md5_ctx_p hctx) {
	uint8_t k[MD5_MSG_BLK_SIZE];
	size_t i;

	memset(k, 0x00, sizeof(k));
	if (key_len > MD5_MSG_BLK_SIZE) {	/* long key -> MD5(key) */
		md5_init(&hctx->ctx);
		md5_update(&hctx->ctx, key, key_len);
		md5_final(&hctx->ctx, k);
	} else if (0 != key_len) {
		memcpy(k, key, key_len);
	}
	for (i = 0; i < MD5_MSG_BLK_SIZE; i ++) {
		((uint8_t*)hctx->k_opad)[i] = (k[i] ^ 0x5c);
		k[i] ^= 0x36;
	}
	md5_init(&hctx->ctx);
	md5_update(&hctx->ctx, k, sizeof(k));
	md5_wipe_fn(k, 0x00, sizeof(k));
}

static inline void
hmac_md5_update(hmac_md5_ctx_p hctx, const uint8_t *data, const size_t data_size) {

	md5_update(&hctx->ctx, data, data_size);
}

static inline void
hmac_md5_final(hmac_md5_ctx_p hctx, uint8_t *digest) {

	md5_final(&hctx->ctx, digest);		/* inner */
	md5_init(&hctx->ctx);
	md5_update(&hctx->ctx, (const uint8_t*)hctx->k_opad, MD5_MSG_BLK_SIZE);
	md5_update(&hctx->ctx, digest, MD5_HASH_SIZE);
	md5_final(&hctx->ctx, digest);		/* outer */
	md5_wipe_fn(hctx->k_opad, 0x00, sizeof(hctx->k_opad));
}

static inline void
hmac_md5(const uint8_t *key, const size_t key_len, const uint8_t *data,
    const size_t data_size, uint8_t *digest) {
	hmac_md5_ctx_t hctx;

	hmac_md5_init(key, key_len, &hctx);
	hmac_md5_update(&hctx, data, data_size);
	hmac_md5_final(&hctx, digest);
}

/* Lowercase hex + NUL (hex needs MD5_HASH_STR_SIZE + 1 bytes). */
static inline void
md5_cvt_hex(const uint8_t *bin, uint8_t *hex) {
	static const char digits[] = "0123456789abcdef";
	size_t i;

	for (i = 0; i < MD5_HASH_SIZE; i ++) {
		hex[2 * i] = (uint8_t)digits[bin[i] >> 4];
		hex[2 * i + 1] = (uint8_t)digits[bin[i] & 0x0f];
	}
	hex[2 * MD5_HASH_SIZE] = 0;
}

static inline void
md5_cvt_str(const uint8_t *digest, char *digest_str) {

	md5_cvt_hex(digest, (uint8_t*)digest_str);
}

static inline void
md5_get_digest(const void *data, const size_t data_size, uint8_t *digest) {
	md5_ctx_t ctx;

	md5_init(&ctx);
	md5_update(&ctx, (const uint8_t*)data, data_size);
	md5_final(&ctx, digest);
}

static inline void
md5_get_digest_str(const char *data, const size_t data_size, char *digest_str) {
	uint8_t digest[MD5_HASH_SIZE];

	md5_get_digest(data, data_size, digest);
	md5_cvt_str(digest, digest_str);
}

static inline void
md5_hmac_get_digest(const void *key, const size_t key_size,
    const void *data, const size_t data_size, uint8_t *digest) {

	hmac_md5((const uint8_t*)key, key_size, (const uint8_t*)data, data_size, digest);
}

static inline void
md5_hmac_get_digest_str(const char *key, size_t key_size,
    const char *data, size_t data_size, char *digest_str) {
	uint8_t digest[MD5_HASH_SIZE];

	md5_hmac_get_digest(key, key_size, data, data_size, digest);
	md5_cvt_str(digest, digest_str);
}

#ifdef MD5_SELF_TEST
/* 0 - OK; 1 - digest KAT failed; 2 - HMAC KAT failed.
 * Vectors: RFC 1321 appendix A.5 and RFC 2202 section 2. */
static inline int
md5_self_test(void) {
	static const struct { const char *msg; const char *md; } kat[] = {
		{ "", "d41d8cd98f00b204e9800998ecf8427e" },
		{ "a", "0cc175b9c0f1b6a831c399e269772661" },
		{ "abc", "900150983cd24fb0d6963f7d28e17f72" },
		{ "message digest", "f96b697d7cb7938d525a2f31aaf161d0" },
		{ "abcdefghijklmnopqrstuvwxyz", "c3fcd3d76192e4007dfb496cca67e13b" },
		{ "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789",
		  "d174ab98d277d9f5a5611c2c9f419d9f" },
		{ "1234567890123456789012345678901234567890"
		  "1234567890123456789012345678901234567890", "57edf4a22be3c955ac49da2e2107b67a" },
	};
	char str[MD5_HASH_STR_SIZE + 1];
	size_t i;

	for (i = 0; i < nitems(kat); i ++) {
		md5_get_digest_str(kat[i].msg, strlen(kat[i].msg), str);
		if (0 != memcmp(str, kat[i].md, MD5_HASH_STR_SIZE))
			return (1);
	}
	/* RFC 2202 test case 2 and 6 (80-byte key, hashed first). */
	md5_hmac_get_digest_str("Jefe", 4, "what do ya want for nothing?", 28, str);
	if (0 != memcmp(str, "750c783e6ab0b503eaa86e310a5db738", MD5_HASH_STR_SIZE))
		return (2);
	{
		char key[80];
		memset(key, 0xaa, sizeof(key));
		md5_hmac_get_digest_str(key, sizeof(key),
		    "Test Using Larger Than Block-Size Key - Hash Key First", 54, str);
		if (0 != memcmp(str, "6b1ab7fe4bd7bf8f0b62e6ce61b9d0cd", MD5_HASH_STR_SIZE))
			return (2);
	}
	return (0);
}
#endif

#endif /* __MD5_H__INCLUDED__ */
