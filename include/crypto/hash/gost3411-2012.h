/*
 * crypto/hash/gost3411-2012.h — source-compatible drop-in for liblcb's
 * gost3411-2012.h (reference include/crypto/hash/gost3411-2012.h), clean-room.
 *
 * GOST R 34.11-2012 "Streebog" 256/512 (RFC 6986) and its HMAC (RFC 7836,
 * 64-byte block) behind the reference API (gost3411-2012.h:91-2020):
 * gost3411_2012_init(bits, ctx) with 256|32 -> 256-bit and ANY other value
 * -> 512-bit, exactly as the reference.
 *
 * The LPS lookup table (8 x 256 x u64) is read-only data generated from the
 * S-box pi and the linear map A (gost3411-2012-lps.h, tools/gen_gost_table.py):
 * no mutable global, as the reference.  Portable C only:
 * the use_sse/use_avx fields exist for source compatibility and are ignored.
 * One-message CPU path; batches go through include/lcb_hash_gpu.h.
 */
#ifndef __GOST3411_2012_H__INCLUDED__
#define __GOST3411_2012_H__INCLUDED__

#include <sys/param.h>
#include <sys/types.h>
#include <string.h>
#include <inttypes.h>

#ifndef nitems
#	define nitems(__val)	(sizeof(__val) / sizeof(__val[0]))
#endif

#define GOST3411_2012_256_HASH_SIZE	((size_t)32)
#define GOST3411_2012_512_HASH_SIZE	((size_t)64)
#define GOST3411_2012_HASH_MAX_SIZE	GOST3411_2012_512_HASH_SIZE
#define GOST3411_2012_HASH_MAX_64CNT	(GOST3411_2012_HASH_MAX_SIZE / sizeof(uint64_t))

#define GOST3411_2012_256_HASH_STR_SIZE	(GOST3411_2012_256_HASH_SIZE * 2)
#define GOST3411_2012_512_HASH_STR_SIZE	(GOST3411_2012_512_HASH_SIZE * 2)
#define GOST3411_2012_HASH_STR_MAX_SIZE	GOST3411_2012_512_HASH_STR_SIZE

#define GOST3411_2012_MSG_BLK_SIZE	((size_t)64)
#define GOST3411_2012_MSG_BLK_SIZE_MASK	(GOST3411_2012_MSG_BLK_SIZE - 1)
#define GOST3411_2012_MSG_BLK_BITS	(GOST3411_2012_MSG_BLK_SIZE * 8)
#define GOST3411_2012_MSG_BLK_64CNT	(GOST3411_2012_MSG_BLK_SIZE / sizeof(uint64_t))
#define GOST3411_2012_ROUNDS_COUNT	((size_t)12)

#define GOST3411_2012_ALIGN(__n) __attribute__ ((aligned(__n)))

/* Field for field the reference's layout (gost3411-2012.h:953-965), so
 * sizeof / offsetof agree (tests/test_dropin_headers.py). */
typedef struct gost3411_2012_ctx_s {
	size_t hash_size;	/* 32 or 64 */
	size_t buffer_usage;	/* bytes in buffer, always < 64 between calls */
	int use_sse;		/* source compatibility only */
	int use_avx;		/* source compatibility only */
	GOST3411_2012_ALIGN(32) uint64_t hash[GOST3411_2012_HASH_MAX_64CNT];	/* h */
	GOST3411_2012_ALIGN(32) uint64_t counter[GOST3411_2012_MSG_BLK_64CNT];	/* N: bits processed */
	GOST3411_2012_ALIGN(32) uint64_t sigma[GOST3411_2012_MSG_BLK_64CNT];	/* Sigma: sum of blocks */
	GOST3411_2012_ALIGN(32) uint64_t buffer[GOST3411_2012_MSG_BLK_64CNT];	/* partial block */
	GOST3411_2012_ALIGN(8) uint64_t kbuf[GOST3411_2012_MSG_BLK_64CNT];	/* layout only */
	GOST3411_2012_ALIGN(8) uint64_t tbuf[GOST3411_2012_MSG_BLK_64CNT];	/* layout only */
	GOST3411_2012_ALIGN(8) uint64_t sbuf[GOST3411_2012_MSG_BLK_64CNT];	/* layout only */
} gost3411_2012_ctx_t, *gost3411_2012_ctx_p;

typedef struct hmac_gost3411_2012_ctx_s {
	gost3411_2012_ctx_t ctx;
	GOST3411_2012_ALIGN(32) uint64_t k_opad[GOST3411_2012_MSG_BLK_64CNT];
} hmac_gost3411_2012_ctx_t, *hmac_gost3411_2012_ctx_p;

static void *(*volatile gost3411_2012_wipe_fn)(void *, int, size_t) = memset;

/* RFC 6986 section 6.4: iteration constants C_1..C_12 (little-endian words). */
static const uint64_t gost3411_2012_C[GOST3411_2012_ROUNDS_COUNT][GOST3411_2012_MSG_BLK_64CNT] = {
	{ 0xdd806559f2a64507ull, 0x05767436cc744d23ull, 0xa2422a08a460d315ull, 0x4b7ce09192676901ull,
	  0x714eb88d7585c4fcull, 0x2f6a76432e45d016ull, 0xebcb2f81c0657c1full, 0xb1085bda1ecadae9ull },
	{ 0xe679047021b19bb7ull, 0x55dda21bd7cbcd56ull, 0x5cb561c2db0aa7caull, 0x9ab5176b12d69958ull,
	  0x61d55e0f16b50131ull, 0xf3feea720a232b98ull, 0x4fe39d460f70b5d7ull, 0x6fa3b58aa99d2f1aull },
	{ 0x991e96f50aba0ab2ull, 0xc2b6f443867adb31ull, 0xc1c93a376062db09ull, 0xd3e20fe490359eb1ull,
	  0xf2ea7514b1297b7bull, 0x06f15e5f529c1f8bull, 0x0a39fc286a3d8435ull, 0xf574dcac2bce2fc7ull },
	{ 0x220cbebc84e3d12eull, 0x3453eaa193e837f1ull, 0xd8b71333935203beull, 0xa9d72c82ed03d675ull,
	  0x9d721cad685e353full, 0x488e857e335c3c7dull, 0xf948e1a05d71e4ddull, 0xef1fdfb3e81566d2ull },
	{ 0x601758fd7c6cfe57ull, 0x7a56a27ea9ea63f5ull, 0xdfff00b723271a16ull, 0xbfcd1747253af5a3ull,
	  0x359e35d7800fffbdull, 0x7f151c1f1686104aull, 0x9a3f410c6ca92363ull, 0x4bea6bacad474799ull },
	{ 0xfa68407a46647d6eull, 0xbf71c57236904f35ull, 0x0af21f66c2bec6b6ull, 0xcffaa6b71c9ab7b4ull,
	  0x187f9ab49af08ec6ull, 0x2d66c4f95142a46cull, 0x6fa4c33b7a3039c0ull, 0xae4faeae1d3ad3d9ull },
	{ 0x8886564d3a14d493ull, 0x3517454ca23c4af3ull, 0x06476983284a0504ull, 0x0992abc52d822c37ull,
	  0xd3473e33197a93c9ull, 0x399ec6c7e6bf87c9ull, 0x51ac86febf240954ull, 0xf4c70e16eeaac5ecull },
	{ 0xa47f0dd4bf02e71eull, 0x36acc2355951a8d9ull, 0x69d18d2bd1a5c42full, 0xf4892bcb929b0690ull,
	  0x89b4443b4ddbc49aull, 0x4eb7f8719c36de1eull, 0x03e7aa020c6e4141ull, 0x9b1f5b424d93c9a7ull },
	{ 0x7261445183235adbull, 0x0e38dc92cb1f2a60ull, 0x7b2b8a9aa6079c54ull, 0x800a440bdbb2ceb1ull,
	  0x3cd955b7e00d0984ull, 0x3a7d3a1b25894224ull, 0x944c9ad8ec165fdeull, 0x378f5a541631229bull },
	{ 0x74b4c7fb98459cedull, 0x3698fad1153bb6c3ull, 0x7a1e6c303b7652f4ull, 0x9fe76702af69334bull,
	  0x1fffe18a1b336103ull, 0x8941e71cff8a78dbull, 0x382ae548b2e4f3f3ull, 0xabbedea680056f52ull },
	{ 0x6bcaa4cd81f32d1bull, 0xdea2594ac06fd85dull, 0xefbacd1d7d476e98ull, 0x8a1d71efea48b9caull,
	  0x2001802114846679ull, 0xd8fa6bbbebab0761ull, 0x3002c6cd635afe94ull, 0x7bcd9ed0efc889fbull },
	{ 0x48bc924af11bd720ull, 0xfaf417d5d9b21b99ull, 0xe71da4aa88e12852ull, 0x5d80ef9d1891cc86ull,
	  0xf82012d430219f9bull, 0xcda43c32bcdf1d77ull, 0xd21380b00449b17aull, 0x378ee767f11631baull }
};

/* LPS table: T[j][b] = L(pi[b] in byte j), generated from RFC 6986 pi / A by
 * tools/gen_gost_table.py into read-only data. */
#include "gost3411-2012-lps.h"

/* dst = LPS(a ^ b); dst may alias a or b. */
static inline void
gost3411_2012_xlps(uint64_t *dst, const uint64_t *a, const uint64_t *b) {
	uint64_t x[8], r[8];
	size_t i, j;

	for (j = 0; j < 8; j ++) {
		x[j] = (a[j] ^ b[j]);
	}
#pragma GCC unroll 8
	for (i = 0; i < 8; i ++) {
		r[i] = 0;
#pragma GCC unroll 8
		for (j = 0; j < 8; j ++) {
			r[i] ^= gost3411_2012_T[j][(x[j] >> (8 * i)) & 0xff];
		}
	}
	memcpy(dst, r, sizeof(r));
}

/* g_N(h, m): h = E(LPS(h ^ N), m) ^ h ^ m. */
static inline void
gost3411_2012_g(uint64_t *h, const uint64_t *n, const uint64_t *m) {
	uint64_t k[8], t[8];
	size_t i;

	gost3411_2012_xlps(k, h, n);
	gost3411_2012_xlps(t, k, m);
	for (i = 0; i < GOST3411_2012_ROUNDS_COUNT; i ++) {
		gost3411_2012_xlps(k, k, gost3411_2012_C[i]);
		if ((GOST3411_2012_ROUNDS_COUNT - 1) != i) {
			gost3411_2012_xlps(t, t, k);
		}
	}
	for (i = 0; i < 8; i ++) {
		h[i] ^= (t[i] ^ k[i] ^ m[i]);
	}
}

static inline void
gost3411_2012_add512(uint64_t *a, const uint64_t *b) {
	uint64_t s, c = 0;
	size_t i;

	for (i = 0; i < 8; i ++) {
		s = (a[i] + b[i]);
		a[i] = (s + c);
		c = ((s < b[i]) | (a[i] < s));
	}
}

static inline uint64_t
gost3411_2012_load_le64(const uint8_t *p) {
	uint64_t v = 0;
	size_t i;

	for (i = 0; i < 8; i ++) {
		v |= ((uint64_t)p[i] << (8 * i));
	}
	return (v);
}

/* Process blocks in [blocks, blocks_max), each adding block_size_bits to N. */
static inline void
gost3411_2012_transform_n(gost3411_2012_ctx_p ctx, const size_t block_size_bits,
    const uint8_t *blocks, const uint8_t *blocks_max) {
	uint64_t m[8], nb[8];
	size_t i;

	memset(nb, 0x00, sizeof(nb));
	nb[0] = block_size_bits;
	for (; blocks < blocks_max; blocks += GOST3411_2012_MSG_BLK_SIZE) {
		for (i = 0; i < 8; i ++) {
			m[i] = gost3411_2012_load_le64(blocks + 8 * i);
		}
		gost3411_2012_g(ctx->hash, ctx->counter, m);
		gost3411_2012_add512(ctx->counter, nb);
		gost3411_2012_add512(ctx->sigma, m);
	}
}

/* g_0(h, block). */
static inline void
gost3411_2012_transform_1(gost3411_2012_ctx_p ctx, const uint64_t *block) {
	static const uint64_t zero[8];

	gost3411_2012_g(ctx->hash, zero, block);
}

static inline void
gost3411_2012_init(const size_t bits, gost3411_2012_ctx_p ctx) {

	memset(ctx, 0x00, sizeof(gost3411_2012_ctx_t));
	if (256 == bits || GOST3411_2012_256_HASH_SIZE == bits) {
		ctx->hash_size = GOST3411_2012_256_HASH_SIZE;
		memset(ctx->hash, 0x01, sizeof(ctx->hash));	/* IV 0x01..01 */
	} else {
		ctx->hash_size = GOST3411_2012_512_HASH_SIZE;	/* IV 0 */
	}
}

static inline void
gost3411_2012_update(gost3411_2012_ctx_p ctx, const uint8_t *data, const size_t data_size) {
	size_t n = data_size, take, whole;

	if (0 != ctx->buffer_usage) {
		take = (GOST3411_2012_MSG_BLK_SIZE - ctx->buffer_usage);
		if (take > n) {
			take = n;
		}
		memcpy(((uint8_t*)ctx->buffer) + ctx->buffer_usage, data, take);
		ctx->buffer_usage += take;
		data += take;
		n -= take;
		if (GOST3411_2012_MSG_BLK_SIZE != ctx->buffer_usage)
			return;
		gost3411_2012_transform_n(ctx, GOST3411_2012_MSG_BLK_BITS,
		    (const uint8_t*)ctx->buffer, ((const uint8_t*)ctx->buffer) + GOST3411_2012_MSG_BLK_SIZE);
		ctx->buffer_usage = 0;
	}
	whole = (n & ~GOST3411_2012_MSG_BLK_SIZE_MASK);
	if (0 != whole) {
		gost3411_2012_transform_n(ctx, GOST3411_2012_MSG_BLK_BITS, data, (data + whole));
	}
	if (n != whole) {
		memcpy(ctx->buffer, data + whole, (n - whole));
		ctx->buffer_usage = (n - whole);
	}
}

static inline void
gost3411_2012_final(gost3411_2012_ctx_p ctx, uint8_t *digest) {
	uint8_t *buf = (uint8_t*)ctx->buffer;
	uint64_t n[8], s[8];
	size_t used = ctx->buffer_usage, i;

	memset(buf + used, 0x00, (GOST3411_2012_MSG_BLK_SIZE - used));
	buf[used] = 0x01;
	gost3411_2012_transform_n(ctx, (used * 8), buf, (buf + GOST3411_2012_MSG_BLK_SIZE));
	memcpy(n, ctx->counter, sizeof(n));
	memcpy(s, ctx->sigma, sizeof(s));
	gost3411_2012_transform_1(ctx, n);
	gost3411_2012_transform_1(ctx, s);
	for (i = 0; i < ctx->hash_size; i ++) {	/* last hash_size bytes of h */
		size_t k = (GOST3411_2012_HASH_MAX_SIZE - ctx->hash_size + i);
		digest[i] = (uint8_t)(ctx->hash[k >> 3] >> (8 * (k & 7)));
	}
	gost3411_2012_wipe_fn(ctx, 0x00, sizeof(gost3411_2012_ctx_t));
}

static inline void
hmac_gost3411_2012_init(const size_t bits, const uint8_t *key, const size_t key_len,
    hmac_gost3411_2012_ctx_p hctx) {
	uint8_t k[GOST3411_2012_MSG_BLK_SIZE];
	size_t i;

	memset(k, 0x00, sizeof(k));
	gost3411_2012_init(bits, &hctx->ctx);
	if (key_len > GOST3411_2012_MSG_BLK_SIZE) {
		gost3411_2012_update(&hctx->ctx, key, key_len);
		gost3411_2012_final(&hctx->ctx, k);
		gost3411_2012_init(bits, &hctx->ctx);
	} else if (0 != key_len) {
		memcpy(k, key, key_len);
	}
	for (i = 0; i < GOST3411_2012_MSG_BLK_SIZE; i ++) {
		((uint8_t*)hctx->k_opad)[i] = (k[i] ^ 0x5c);
		k[i] ^= 0x36;
	}
	gost3411_2012_update(&hctx->ctx, k, sizeof(k));
	gost3411_2012_wipe_fn(k, 0x00, sizeof(k));
}

static inline void
hmac_gost3411_2012_update(hmac_gost3411_2012_ctx_p hctx, const uint8_t *data,
    const size_t data_size) {

	gost3411_2012_update(&hctx->ctx, data, data_size);
}

static inline void
hmac_gost3411_2012_final(hmac_gost3411_2012_ctx_p hctx, uint8_t *digest,
    size_t *digest_size) {
	size_t hs = hctx->ctx.hash_size;

	gost3411_2012_final(&hctx->ctx, digest);
	gost3411_2012_init(hs, &hctx->ctx);
	gost3411_2012_update(&hctx->ctx, (const uint8_t*)hctx->k_opad, GOST3411_2012_MSG_BLK_SIZE);
	gost3411_2012_update(&hctx->ctx, digest, hs);
	if (NULL != digest_size) {
		(*digest_size) = hs;
	}
	gost3411_2012_final(&hctx->ctx, digest);
	gost3411_2012_wipe_fn(hctx->k_opad, 0x00, sizeof(hctx->k_opad));
}

static inline void
hmac_gost3411_2012(const size_t bits, const uint8_t *key, const size_t key_len,
    const uint8_t *data, const size_t data_size, uint8_t *digest, size_t *digest_size) {
	hmac_gost3411_2012_ctx_t hctx;

	hmac_gost3411_2012_init(bits, key, key_len, &hctx);
	hmac_gost3411_2012_update(&hctx, data, data_size);
	hmac_gost3411_2012_final(&hctx, digest, digest_size);
}

static inline void
gost3411_2012_cvt_hex(const uint8_t *bin, const size_t bin_size, uint8_t *hex) {
	static const char digits[] = "0123456789abcdef";
	size_t i;

	for (i = 0; i < bin_size; i ++) {
		hex[2 * i] = (uint8_t)digits[bin[i] >> 4];
		hex[2 * i + 1] = (uint8_t)digits[bin[i] & 0x0f];
	}
	hex[2 * bin_size] = 0;
}

static inline void
gost3411_2012_cvt_str(const uint8_t *digest, const size_t digest_size, char *digest_str) {

	gost3411_2012_cvt_hex(digest, digest_size, (uint8_t*)digest_str);
}

static inline void
gost3411_2012_get_digest(const size_t bits, const void *data, const size_t data_size,
    uint8_t *digest, size_t *digest_size) {
	gost3411_2012_ctx_t ctx;

	gost3411_2012_init(bits, &ctx);
	gost3411_2012_update(&ctx, (const uint8_t*)data, data_size);
	if (NULL != digest_size) {
		(*digest_size) = ctx.hash_size;
	}
	gost3411_2012_final(&ctx, digest);
}

static inline void
gost3411_2012_get_digest_str(const size_t bits, const char *data, const size_t data_size,
    char *digest_str, size_t *digest_str_size) {
	uint8_t digest[GOST3411_2012_HASH_MAX_SIZE];
	size_t ds = 0;

	gost3411_2012_get_digest(bits, data, data_size, digest, &ds);
	gost3411_2012_cvt_str(digest, ds, digest_str);
	if (NULL != digest_str_size) {
		(*digest_str_size) = (ds * 2);
	}
}

static inline void
gost3411_2012_hmac_get_digest(const size_t bits, const void *key, const size_t key_size,
    const void *data, const size_t data_size, uint8_t *digest, size_t *digest_size) {

	hmac_gost3411_2012(bits, (const uint8_t*)key, key_size, (const uint8_t*)data,
	    data_size, digest, digest_size);
}

static inline void
gost3411_2012_hmac_get_digest_str(size_t bits, const char *key, const size_t key_size,
    const char *data, const size_t data_size, char *digest_str, size_t *digest_str_size) {
	uint8_t digest[GOST3411_2012_HASH_MAX_SIZE];
	size_t ds = 0;

	hmac_gost3411_2012(bits, (const uint8_t*)key, key_size, (const uint8_t*)data,
	    data_size, digest, &ds);
	gost3411_2012_cvt_str(digest, ds, digest_str);
	if (NULL != digest_str_size) {
		(*digest_str_size) = (ds * 2);
	}
}

#ifdef GOST3411_2012_SELF_TEST
/* 0 - OK; 1/2 - 256/512-bit digest KAT failed; 3 - chunked update failed;
 * 5/6 - HMAC 256/512 failed.  Vectors: RFC 6986 example M1 (63 bytes) and
 * RFC 7836 section 4.1.1 HMAC. */
static inline int
gost3411_2012_self_test(void) {
	static const char m1[] = "012345678901234567890123456789012345678901234567890123456789012";
	static const char *m1_256 = "9d151eefd8590b89daa6ba6cb74af9275dd051026bb149a452fd84e5e57b5500";
	static const char *m1_512 = "1b54d01a4af5b9d5cc3d86d68d285462b19abc2475222f35c085122be4ba1ffa"
	    "00ad30f8767b3a82384c6574f024c311e2a481332b08ef7f41797891c1646f48";
	static const uint8_t hk[32] = {
		0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15,
		16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31 };
	static const uint8_t hm[16] = {
		0x01, 0x26, 0xbd, 0xb8, 0x78, 0x00, 0xaf, 0x21, 0x43, 0x41, 0x45, 0x65, 0x63, 0x78, 0x01, 0x00 };
	static const char *h256 = "a1aa5f7de402d7b3d323f2991c8d4534013137010a83754fd0af6d7cd4922ed9";
	static const char *h512 = "a59bab22ecae19c65fbde6e5f4e9f5d8549d31f037f9df9b905500e171923a77"
	    "3d5f1530f2ed7e964cb2eedc29e9ad2f3afe93b2814f79f5000ffc0366c251e6";
	char str[GOST3411_2012_HASH_STR_MAX_SIZE + 1];
	uint8_t digest[GOST3411_2012_HASH_MAX_SIZE];
	gost3411_2012_ctx_t ctx;
	size_t n, i, j;

	gost3411_2012_get_digest_str(256, m1, 63, str, &n);
	if (64 != n || 0 != memcmp(str, m1_256, n))
		return (1);
	gost3411_2012_get_digest_str(512, m1, 63, str, &n);
	if (128 != n || 0 != memcmp(str, m1_512, n))
		return (2);
	for (j = 1; j < 63; j ++) {	/* every update chunk size */
		gost3411_2012_init(512, &ctx);
		for (i = 0; i < 63; i += j) {
			gost3411_2012_update(&ctx, (const uint8_t*)m1 + i, ((63 - i) < j ? (63 - i) : j));
		}
		gost3411_2012_final(&ctx, digest);
		gost3411_2012_cvt_str(digest, 64, str);
		if (0 != memcmp(str, m1_512, 128))
			return (3);
	}
	gost3411_2012_hmac_get_digest_str(256, (const char*)hk, sizeof(hk), (const char*)hm,
	    sizeof(hm), str, &n);
	if (64 != n || 0 != memcmp(str, h256, n))
		return (5);
	gost3411_2012_hmac_get_digest_str(512, (const char*)hk, sizeof(hk), (const char*)hm,
	    sizeof(hm), str, &n);
	if (128 != n || 0 != memcmp(str, h512, n))
		return (6);
	return (0);
}
#endif

#endif /* __GOST3411_2012_H__INCLUDED__ */
