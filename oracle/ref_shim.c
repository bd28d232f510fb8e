/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Thin C wrapper that compiles the REFERENCE's own hash headers, where they
 * lie under /root/reference/include (nothing is copied), into
 * oracle/_ref/libref_hash*.so.  Used (a) to validate the oracle restatement
 * and generate golden fixtures (tests/golden/make_golden.py) and (b) as the
 * timed "reference CPU path" in bench.py's cpu_baseline leg.
 *
 * Build variants (oracle/Makefile):
 *   libref_hash.so       generic, exactly as tests/hash/main.c:36 builds it
 *                        (#undef __SSE2__): generic SHA-1 / GOST paths.
 *   libref_hash_simd.so  REF_SIMD=1: SSE4.1/SSSE3/SHA-NI/AVX2 code paths of
 *                        sha1.h / sha2.h / gost3411-2012.h enabled; the
 *                        reference still picks them per ctx with cpuid.
 */
#include <sys/param.h>
#include <sys/types.h>
#include <inttypes.h>
#include <stdio.h>

#ifdef REF_SIMD
#	include <immintrin.h>   /* sha1.h:91 / sha2.h:50 need it first */
#else
#	undef __SSE2__          /* tests/hash/main.c:36 */
#endif

#define MD5_SELF_TEST 1
#define SHA1_SELF_TEST 1
#define SHA2_SELF_TEST 1
#define GOST3411_2012_SELF_TEST 1

#include "crypto/hash/md5.h"
#include "crypto/hash/sha1.h"
#include "crypto/hash/sha2.h"
#include "crypto/hash/gost3411-2012.h"

#ifndef nitems			/* BSD sys/param.h macro used by crc32.h:619 */
#	define nitems(x)	(sizeof((x)) / sizeof((x)[0]))
#endif
#define CRC32_SELF_TEST 1
#include "math/crc32.h"
#include <errno.h>
#define CHACHA_SELF_TEST 1
#include "crypto/cipher/chacha.h"

enum { A_MD5 = 1, A_SHA1, A_SHA224, A_SHA256, A_SHA384, A_SHA512, A_GOST256, A_GOST512 };

static size_t
ref_bits(int alg) {
	static const size_t b[9] = { 0, 0, 0, 224, 256, 384, 512, 256, 512 };
	return (alg >= 1 && alg <= 8) ? b[alg] : 0;
}

/* tests/hash/main.c:53-82: first failing self test's code, else 0. */
int
ref_self_test(void) {
	int e;
	if ((e = md5_self_test())) return 100 + e;
	if ((e = sha1_self_test())) return 200 + e;
	if ((e = sha2_self_test())) return 300 + e;
	if ((e = gost3411_2012_self_test())) return 400 + e;
	return 0;
}

/* One digest through the reference's one-shot API. */
static int
ref_one(int alg, const uint8_t *d, size_t n, uint8_t *out) {
	switch (alg) {
	case A_MD5: md5_get_digest(d, n, out); return 0;
	case A_SHA1: sha1_get_digest(d, n, out); return 0;
	case A_SHA224: case A_SHA256: case A_SHA384: case A_SHA512:
		sha2_get_digest(ref_bits(alg), d, n, out, NULL); return 0;
	case A_GOST256: case A_GOST512:
		gost3411_2012_get_digest(ref_bits(alg), d, n, out, NULL); return 0;
	}
	return -1;
}

static int
ref_one_hmac(int alg, const uint8_t *k, size_t kl, const uint8_t *d, size_t n,
    uint8_t *out) {
	switch (alg) {
	case A_MD5: md5_hmac_get_digest(k, kl, d, n, out); return 0;
	case A_SHA1: sha1_hmac_get_digest(k, kl, d, n, out); return 0;
	case A_SHA224: case A_SHA256: case A_SHA384: case A_SHA512:
		sha2_hmac_get_digest(ref_bits(alg), k, kl, d, n, out, NULL); return 0;
	case A_GOST256: case A_GOST512:
		gost3411_2012_hmac_get_digest(ref_bits(alg), k, kl, d, n, out, NULL); return 0;
	}
	return -1;
}

static size_t
ref_dsize(int alg) {
	static const size_t ds[9] = { 0, 16, 20, 28, 32, 48, 64, 32, 64 };
	return (alg >= 1 && alg <= 8) ? ds[alg] : 0;
}

/* Batch loop: message i at base + (offsets ? offsets[i] : i*stride), length
 * (lengths ? lengths[i] : fixed_len); key != NULL selects HMAC. */
int
ref_batch(int alg, const uint8_t *key, size_t key_len, const uint8_t *base,
    const uint64_t *offsets, const uint32_t *lengths, size_t count,
    uint64_t stride, uint32_t fixed_len, uint8_t *digests) {
	size_t i, ds = ref_dsize(alg);

	if (0 == ds)
		return -1;
	for (i = 0; i < count; i ++) {
		const uint8_t *p = base + (offsets ? offsets[i] : (uint64_t)i * stride);
		size_t n = (lengths ? lengths[i] : fixed_len);
		if (key)
			ref_one_hmac(alg, key, key_len, p, n, digests + i * ds);
		else
			ref_one(alg, p, n, digests + i * ds);
	}
	return 0;
}

/* H(A || B) through the reference's streaming calls: init, update(A),
 * update(B), final (the keyed-prefix and secret-suffix shapes of RADIUS,
 * radius.h:774-789 and :1334-1352). */
static int
ref_two(int alg, const uint8_t *a, size_t la, const uint8_t *b, size_t lb,
    uint8_t *out) {
	switch (alg) {
	case A_MD5: {
		md5_ctx_t c;
		md5_init(&c); md5_update(&c, a, la); md5_update(&c, b, lb);
		md5_final(&c, out);
		return 0;
	}
	case A_SHA1: {
		sha1_ctx_t c;
		sha1_init(&c); sha1_update(&c, a, la); sha1_update(&c, b, lb);
		sha1_final(&c, out);
		return 0;
	}
	case A_SHA224: case A_SHA256: case A_SHA384: case A_SHA512: {
		sha2_ctx_t c;
		sha2_init(ref_bits(alg), &c); sha2_update(&c, a, la);
		sha2_update(&c, b, lb); sha2_final(&c, out);
		return 0;
	}
	case A_GOST256: case A_GOST512: {
		gost3411_2012_ctx_t c;
		gost3411_2012_init(ref_bits(alg), &c);
		gost3411_2012_update(&c, a, la); gost3411_2012_update(&c, b, lb);
		gost3411_2012_final(&c, out);
		return 0;
	}
	}
	return -1;
}

/* Keyed batch (the shapes of lcb_hash_batch_keyed): message i uses key
 * key_index[i] (NULL: 0); mode 1 HMAC (the reference's *_hmac_get_digest),
 * 2 H(K || m), 3 H(m || K).  -2 for a key index out of range. */
int
ref_batch_keyed(int alg, int mode, const uint8_t *keys, const uint64_t *key_off,
    const uint32_t *key_len, size_t nkeys, const uint32_t *key_index,
    const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths,
    size_t count, uint64_t stride, uint32_t fixed_len, uint8_t *digests) {
	size_t i, ds = ref_dsize(alg);

	if (0 == ds || mode < 1 || mode > 3)
		return -1;
	for (i = 0; i < count; i ++) {
		const uint8_t *p = base + (offsets ? offsets[i] : (uint64_t)i * stride);
		size_t n = (lengths ? lengths[i] : fixed_len);
		uint32_t k = (key_index ? key_index[i] : 0);
		const uint8_t *K;

		if (k >= nkeys)
			return -2;
		K = keys + (key_off ? key_off[k] : 0);
		if (1 == mode)
			ref_one_hmac(alg, K, key_len[k], p, n, digests + i * ds);
		else if (2 == mode)
			ref_two(alg, K, key_len[k], p, n, digests + i * ds);
		else
			ref_two(alg, p, n, K, key_len[k], digests + i * ds);
	}
	return 0;
}

/* Streaming with fixed-size update chunks (chunk 0 = whole message);
 * exercises *_update buffering like gost3411-2012.h:2162-2230. */
int
ref_chunked(int alg, const uint8_t *d, size_t n, size_t chunk, uint8_t *out) {
	size_t i, c;

	if (0 == chunk)
		chunk = (n ? n : 1);
	switch (alg) {
	case A_MD5: { md5_ctx_t x; md5_init(&x);
		for (i = 0; i < n; i += c) { c = MIN(chunk, n - i); md5_update(&x, d + i, c); }
		md5_final(&x, out); return 0; }
	case A_SHA1: { sha1_ctx_t x; sha1_init(&x);
		for (i = 0; i < n; i += c) { c = MIN(chunk, n - i); sha1_update(&x, d + i, c); }
		sha1_final(&x, out); return 0; }
	case A_SHA224: case A_SHA256: case A_SHA384: case A_SHA512: {
		sha2_ctx_t x; sha2_init(ref_bits(alg), &x);
		for (i = 0; i < n; i += c) { c = MIN(chunk, n - i); sha2_update(&x, d + i, c); }
		sha2_final(&x, out); return 0; }
	case A_GOST256: case A_GOST512: {
		gost3411_2012_ctx_t x; gost3411_2012_init(ref_bits(alg), &x);
		for (i = 0; i < n; i += c) { c = MIN(chunk, n - i); gost3411_2012_update(&x, d + i, c); }
		gost3411_2012_final(&x, out); return 0; }
	}
	return -1;
}

/* GOST big-table export, so tests can pin the generated Ax tables
 * (liblcb_amd) against gost3411-2012.h:184-882. */
int
ref_gost_ax(uint64_t *out /* 8*256 */) {
	memcpy(out, gost3411_2012_Ax, sizeof(gost3411_2012_Ax));
	return (int)sizeof(gost3411_2012_Ax);
}

/* ---------------------------------------------------------------- CRC-32
 * include/math/crc32.h, variant ids as include/lcb_crc32_gpu.h:
 * 1 crc32a, 2 cksum, 3 mpeg2, 4 crc32b, 5 jamcrc, 6 crc32c, 7 crc32d, 8 crc32q. */
int
ref_crc32_self_test(void) {
	return crc32_self_test();	/* crc32.h:581-657 */
}

static uint32_t
ref_crc32_one(int v, int upd, uint32_t c, const uint8_t *p, size_t n) {
	switch (v) {
	case 1: return upd ? crc32a_update(c, p, n) : crc32a(p, n);
	case 2: return upd ? crc32cksum_update(c, p, n) : crc32cksum(p, n);
	case 3: return upd ? crc32mpeg2_update(c, p, n) : crc32mpeg2(p, n);
	case 4: return upd ? crc32b_update(c, p, n) : crc32b(p, n);
	case 5: return upd ? crc32jamcrc_update(c, p, n) : crc32jamcrc(p, n);
	case 6: return upd ? crc32c_update(c, p, n) : crc32c(p, n);
	case 7: return upd ? crc32d_update(c, p, n) : crc32d(p, n);
	case 8: return upd ? crc32q_update(c, p, n) : crc32q(p, n);
	}
	return 0;
}

/* init == NULL: crcs[i] = X(msg i); else X_update(init[i], msg i). */
int
ref_crc32_batch(int v, const uint32_t *init, const uint8_t *base,
    const uint64_t *offsets, const uint32_t *lengths, size_t count,
    uint64_t stride, uint32_t fixed_len, uint32_t *crcs) {
	size_t i;

	if (v < 1 || v > 8)
		return -1;
	for (i = 0; i < count; i ++) {
		const uint8_t *p = base + (offsets ? offsets[i] : (uint64_t)i * stride);
		size_t n = (lengths ? lengths[i] : fixed_len);
		crcs[i] = ref_crc32_one(v, init != NULL, init ? init[i] : 0, p, n);
	}
	return 0;
}

/* The reference's 256-entry byte table used by variant v (crc32.h:128-494). */
int
ref_crc32_table(int v, uint32_t *out) {
	const uint32_t *t;

	switch (v) {
	case 1: case 2: case 3: t = crc32_tbl256_04c11db7; break;
	case 4: case 5: t = crc32_tbl256_edb88320; break;
	case 6: t = crc32_tbl256_1edc6f41; break;
	case 7: t = crc32_tbl256_a833982b; break;
	case 8: t = crc32_tbl256_814141ab; break;
	default: return -1;
	}
	memcpy(out, t, 256 * sizeof(uint32_t));
	return 0;
}

/* ---------------------------------------------------------------- ChaCha
 * include/crypto/cipher/chacha.h one-shot chacha() / xchacha() per buffer. */
int
ref_chacha_self_test(void) {
	return chacha_self_test();	/* chacha.h:1061-1160 */
}

int
ref_chacha_batch(const uint8_t *key, size_t key_size, size_t rounds, int x,
    const uint8_t *counters, const uint8_t *ivs, const uint8_t *src, uint8_t *dst,
    const uint64_t *offsets, const uint32_t *lengths, size_t count, uint64_t stride,
    uint32_t fixed_len) {
	size_t i, ivlen = (x ? 24 : 8);

	for (i = 0; i < count; i ++) {
		uint64_t o = (offsets ? offsets[i] : (uint64_t)i * stride);
		size_t n = (lengths ? lengths[i] : fixed_len);
		const uint8_t *c = (counters ? counters + 8 * i : NULL);
		const uint8_t *v = (ivs ? ivs + ivlen * i : NULL);
		if (x)
			xchacha(key, key_size, c, v, rounds, (src ? src + o : NULL), n, dst + o);
		else
			chacha(key, key_size, c, v, rounds, (src ? src + o : NULL), n, dst + o);
	}
	return 0;
}

/* The self test's first table (chacha.h:709-...), decoded exactly as
 * chacha_self_test does: vector i -> key (32), count (8, NULL -> flag 0),
 * iv (8), rounds, data size, expected output, plaintext (NULL -> keystream
 * test).  Returns -1 past the end. */
int
ref_chacha_kat(size_t i, uint8_t *key, size_t *key_size, uint8_t *count, int *has_count,
    uint8_t *iv, int *has_iv, size_t *rounds, size_t *data_size, uint8_t *expected,
    uint8_t *plain, int *has_plain) {
	size_t n;

	for (n = 0; 0 != chacha_tst1v[n].rounds; n ++)
		;
	if (i >= n)
		return -1;
	memset(key, 0, CHACHA_KEY_256_LEN);
	chacha_import_le_hex(key, CHACHA_KEY_256_LEN, chacha_tst1v[i].key, chacha_tst1v[i].key_size);
	*key_size = chacha_tst1v[i].key_size / 2;
	*has_count = (NULL != chacha_tst1v[i].count);
	memset(count, 0, 8);
	if (*has_count)
		chacha_import_be_hex(count, 8, chacha_tst1v[i].count, 16);
	*has_iv = (NULL != chacha_tst1v[i].iv);
	memset(iv, 0, 8);
	if (*has_iv)
		chacha_import_le_hex(iv, 8, chacha_tst1v[i].iv, 16);
	*rounds = chacha_tst1v[i].rounds;
	*data_size = chacha_tst1v[i].data_size / 2;
	chacha_import_le_hex(expected, CHACHA_TEST_LEN, chacha_tst1v[i].encrypted,
	    chacha_tst1v[i].data_size);
	*has_plain = (NULL != chacha_tst1v[i].plain);
	memset(plain, 0, CHACHA_TEST_LEN);
	if (*has_plain)
		chacha_import_le_hex(plain, CHACHA_TEST_LEN, chacha_tst1v[i].plain,
		    chacha_tst1v[i].data_size);
	return 0;
}
