/*
 * crypto/hash/sha1.h — source-compatible drop-in for liblcb's sha1.h
 * (reference include/crypto/hash/sha1.h), clean-room.
 *
 * Same macros, types and `static inline` prototypes as the reference
 * (sha1.h:105-985).  Portable C only: no SSE/SHA-NI variants and no per-init
 * cpuid (the reference executes cpuid in every sha1_init in SIMD builds,
 * sha1.h:186-202), so the context layout does not change with ISA flags.
 * One-message CPU path; batches go through include/lcb_hash_gpu.h.
 * FIPS 180-4 (SHA-1), RFC 2104 (HMAC).
 */
#ifndef __SHA1_H__INCLUDED__
#define __SHA1_H__INCLUDED__

#include <sys/param.h>
#include <sys/types.h>
#include <string.h>
#include <inttypes.h>

#ifndef nitems
#	define nitems(__val)	(sizeof(__val) / sizeof(__val[0]))
#endif

#define SHA1_HASH_SIZE		((size_t)20)
#define SHA1_HASH_STR_SIZE	(SHA1_HASH_SIZE * 2)
#define SHA1_MSG_BLK_SIZE	((size_t)64)
#define SHA1_MSG_BLK_SIZE_MASK	(SHA1_MSG_BLK_SIZE - 1)
#define SHA1_MSG_BLK_64CNT	(SHA1_MSG_BLK_SIZE / sizeof(uint64_t))

#define SHA1_ALIGN(__n)	__attribute__ ((aligned(__n)))
#if defined(__SHA__) && defined(__SSSE3__) && defined(__SSE4_1__)
#	define SHA1_ENABLE_SIMD	1	/* layout only: this header has no SIMD path */
#endif

/* Field for field the reference's layout (sha1.h:128-139), including the
 * build-dependent tail, so sizeof / offsetof agree in every build and mixed
 * translation units see one struct (tests/test_dropin_headers.py). */
typedef struct sha1_ctx_s {
	uint64_t count;				/* bytes hashed so far */
	SHA1_ALIGN(32) uint32_t hash[(SHA1_HASH_SIZE / sizeof(uint32_t))];
	SHA1_ALIGN(32) uint64_t buffer[SHA1_MSG_BLK_64CNT];	/* partial block */
	SHA1_ALIGN(32) uint32_t W[80];		/* message schedule scratch */
#ifdef __SSE2__
	int use_sse;				/* layout only */
#endif
#ifdef SHA1_ENABLE_SIMD
	int use_simd;				/* layout only */
#endif
} sha1_ctx_t, *sha1_ctx_p;

typedef struct hmac_sha1_ctx_s {
	sha1_ctx_t ctx;
	SHA1_ALIGN(32) uint64_t k_opad[SHA1_MSG_BLK_64CNT];
} hmac_sha1_ctx_t, *hmac_sha1_ctx_p;

static void *(*volatile sha1_wipe_fn)(void *, int, size_t) = memset;

static inline uint32_t
sha1_rol32(const uint32_t x, const unsigned n) {
	return ((x << n) | (x >> (32 - n)));
}

static inline uint32_t
sha1_load_be32(const uint8_t *p) {
	return (((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) |
	    ((uint32_t)p[2] << 8) | (uint32_t)p[3]);
}

static inline void
sha1_init(sha1_ctx_p ctx) {
	ctx->hash[0] = 0x67452301;
	ctx->hash[1] = 0xefcdab89;
	ctx->hash[2] = 0x98badcfe;
	ctx->hash[3] = 0x10325476;
	ctx->hash[4] = 0xc3d2e1f0;
	ctx->count = 0;
}

/* Compress every 64-byte block in [blocks, blocks_max), any alignment. */
static inline void
sha1_transform(sha1_ctx_p ctx, const uint8_t *blocks, const uint8_t *blocks_max) {
	uint32_t w[16], a, b, c, d, e, f, k, t;
	size_t i;

	for (; blocks < blocks_max; blocks += SHA1_MSG_BLK_SIZE) {
		for (i = 0; i < 16; i ++) {
			w[i] = sha1_load_be32(blocks + 4 * i);
		}
		a = ctx->hash[0]; b = ctx->hash[1]; c = ctx->hash[2];
		d = ctx->hash[3]; e = ctx->hash[4];
#pragma GCC unroll 80
		for (i = 0; i < 80; i ++) {
			if (i >= 16) {	/* rolling 16-word schedule */
				w[i & 15] = sha1_rol32((w[(i + 13) & 15] ^ w[(i + 8) & 15] ^
				    w[(i + 2) & 15] ^ w[i & 15]), 1);
			}
			if (i < 20) {
				f = (d ^ (b & (c ^ d)));
				k = 0x5a827999;
			} else if (i < 40) {
				f = (b ^ c ^ d);
				k = 0x6ed9eba1;
			} else if (i < 60) {
				f = ((b & c) | (d & (b | c)));
				k = 0x8f1bbcdc;
			} else {
				f = (b ^ c ^ d);
				k = 0xca62c1d6;
			}
			t = (sha1_rol32(a, 5) + f + e + k + w[i & 15]);
			e = d;
			d = c;
			c = sha1_rol32(b, 30);
			b = a;
			a = t;
		}
		ctx->hash[0] += a; ctx->hash[1] += b; ctx->hash[2] += c;
		ctx->hash[3] += d; ctx->hash[4] += e;
	}
}

static inline void
sha1_update(sha1_ctx_p ctx, const uint8_t *data, size_t data_size) {
	size_t used = (size_t)(ctx->count & SHA1_MSG_BLK_SIZE_MASK), take, whole;

	ctx->count += data_size;
	if (0 != used) {
		take = (SHA1_MSG_BLK_SIZE - used);
		if (take > data_size) {
			take = data_size;
		}
		memcpy(((uint8_t*)ctx->buffer) + used, data, take);
		used += take;
		data += take;
		data_size -= take;
		if (SHA1_MSG_BLK_SIZE != used)
			return;
		sha1_transform(ctx, (const uint8_t*)ctx->buffer,
		    ((const uint8_t*)ctx->buffer) + SHA1_MSG_BLK_SIZE);
	}
	whole = (data_size & ~SHA1_MSG_BLK_SIZE_MASK);
	if (0 != whole) {
		sha1_transform(ctx, data, (data + whole));
	}
	if (data_size != whole) {
		memcpy(ctx->buffer, data + whole, (data_size - whole));
	}
}

static inline void
sha1_final(sha1_ctx_p ctx, uint8_t *digest) {
	uint8_t *buf = (uint8_t*)ctx->buffer;
	size_t used = (size_t)(ctx->count & SHA1_MSG_BLK_SIZE_MASK), i;
	uint64_t bits = (ctx->count << 3);

	buf[used ++] = 0x80;
	if (used > (SHA1_MSG_BLK_SIZE - 8)) {
		memset(buf + used, 0x00, (SHA1_MSG_BLK_SIZE - used));
		sha1_transform(ctx, buf, (buf + SHA1_MSG_BLK_SIZE));
		used = 0;
	}
	memset(buf + used, 0x00, ((SHA1_MSG_BLK_SIZE - 8) - used));
	for (i = 0; i < 8; i ++) {	/* big-endian bit count */
		buf[(SHA1_MSG_BLK_SIZE - 1) - i] = (uint8_t)(bits >> (8 * i));
	}
	sha1_transform(ctx, buf, (buf + SHA1_MSG_BLK_SIZE));
	for (i = 0; i < SHA1_HASH_SIZE; i ++) {
		digest[i] = (uint8_t)(ctx->hash[i >> 2] >> (24 - 8 * (i & 3)));
	}
	sha1_wipe_fn(ctx, 0x00, sizeof(sha1_ctx_t));
}

static inline void
hmac_sha1_init(const uint8_t *key, size_t key_len, hmac_sha1_ctx_p hctx) {
	uint8_t k[SHA1_MSG_BLK_SIZE];
	size_t i;

	memset(k, 0x00, sizeof(k));
	if (key_len > SHA1_MSG_BLK_SIZE) {
		sha1_init(&hctx->ctx);
		sha1_update(&hctx->ctx, key, key_len);
		sha1_final(&hctx->ctx, k);
	} else if (0 != key_len) {
		memcpy(k, key, key_len);
	}
	for (i = 0; i < SHA1_MSG_BLK_SIZE; i ++) {
		((uint8_t*)hctx->k_opad)[i] = (k[i] ^ 0x5c);
		k[i] ^= 0x36;
	}
	sha1_init(&hctx->ctx);
	sha1_update(&hctx->ctx, k, sizeof(k));
	sha1_wipe_fn(k, 0x00, sizeof(k));
}

static inline void
hmac_sha1_update(hmac_sha1_ctx_p hctx, const uint8_t *data, size_t data_size) {

	sha1_update(&hctx->ctx, data, data_size);
}

static inline void
hmac_sha1_final(hmac_sha1_ctx_p hctx, uint8_t *digest) {

	sha1_final(&hctx->ctx, digest);
	sha1_init(&hctx->ctx);
	sha1_update(&hctx->ctx, (const uint8_t*)hctx->k_opad, SHA1_MSG_BLK_SIZE);
	sha1_update(&hctx->ctx, digest, SHA1_HASH_SIZE);
	sha1_final(&hctx->ctx, digest);
	sha1_wipe_fn(hctx->k_opad, 0x00, sizeof(hctx->k_opad));
}

static inline void
hmac_sha1(const uint8_t *key, size_t key_len, const uint8_t *data,
    size_t data_size, uint8_t *digest) {
	hmac_sha1_ctx_t hctx;

	hmac_sha1_init(key, key_len, &hctx);
	hmac_sha1_update(&hctx, data, data_size);
	hmac_sha1_final(&hctx, digest);
}

static inline void
sha1_cvt_hex(const uint8_t *bin, uint8_t *hex) {
	static const char digits[] = "0123456789abcdef";
	size_t i;

	for (i = 0; i < SHA1_HASH_SIZE; i ++) {
		hex[2 * i] = (uint8_t)digits[bin[i] >> 4];
		hex[2 * i + 1] = (uint8_t)digits[bin[i] & 0x0f];
	}
	hex[2 * SHA1_HASH_SIZE] = 0;
}

static inline void
sha1_cvt_str(const uint8_t *digest, char *digest_str) {

	sha1_cvt_hex(digest, (uint8_t*)digest_str);
}

static inline void
sha1_get_digest(const void *data, size_t data_size, uint8_t *digest) {
	sha1_ctx_t ctx;

	sha1_init(&ctx);
	sha1_update(&ctx, (const uint8_t*)data, data_size);
	sha1_final(&ctx, digest);
}

static inline void
sha1_get_digest_str(const char *data, size_t data_size, char *digest_str) {
	uint8_t digest[SHA1_HASH_SIZE];

	sha1_get_digest(data, data_size, digest);
	sha1_cvt_str(digest, digest_str);
}

static inline void
sha1_hmac_get_digest(const void *key, size_t key_size,
    const void *data, size_t data_size, uint8_t *digest) {

	hmac_sha1((const uint8_t*)key, key_size, (const uint8_t*)data, data_size, digest);
}

static inline void
sha1_hmac_get_digest_str(const char *key, size_t key_size,
    const char *data, size_t data_size, char *digest_str) {
	uint8_t digest[SHA1_HASH_SIZE];

	sha1_hmac_get_digest(key, key_size, data, data_size, digest);
	sha1_cvt_str(digest, digest_str);
}

#ifdef SHA1_SELF_TEST
/* 0 - OK; 1 - digest KAT failed; 2 - HMAC KAT failed.
 * Vectors: FIPS 180 examples (incl. one million 'a' fed byte by byte) and
 * RFC 2202 section 3. */
static inline int
sha1_self_test(void) {
	static const struct { const char *msg; const char *md; } kat[] = {
		{ "", "da39a3ee5e6b4b0d3255bfef95601890afd80709" },
		{ "abc", "a9993e364706816aba3e25717850c26c9cd0d89d" },
		{ "abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
		  "84983e441c3bd26ebaae4aa1f95129e5e54670f1" },
	};
	char str[SHA1_HASH_STR_SIZE + 1];
	uint8_t digest[SHA1_HASH_SIZE];
	sha1_ctx_t ctx;
	size_t i;

	for (i = 0; i < nitems(kat); i ++) {
		sha1_get_digest_str(kat[i].msg, strlen(kat[i].msg), str);
		if (0 != memcmp(str, kat[i].md, SHA1_HASH_STR_SIZE))
			return (1);
	}
	sha1_init(&ctx);
	for (i = 0; i < 1000000; i ++) {
		sha1_update(&ctx, (const uint8_t*)"a", 1);
	}
	sha1_final(&ctx, digest);
	sha1_cvt_str(digest, str);
	if (0 != memcmp(str, "34aa973cd4c4daa4f61eeb2bdbad27316534016f", SHA1_HASH_STR_SIZE))
		return (1);
	sha1_hmac_get_digest_str("Jefe", 4, "what do ya want for nothing?", 28, str);
	if (0 != memcmp(str, "effcdf6ae5eb2fa2d27416d5f184df9c259a7c79", SHA1_HASH_STR_SIZE))
		return (2);
	return (0);
}
#endif

#endif /* __SHA1_H__INCLUDED__ */
