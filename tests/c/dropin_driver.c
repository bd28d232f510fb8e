/*
 * Drives the drop-in headers (include/crypto/hash/) through their full
 * streaming API for tests/test_dropin_headers.py.
 * stdin lines:  <alg> <key-hex|-|=> <msg-hex|-> <repeat> <chunk>
 *   key "-" = plain digest, "=" = HMAC with an empty key; msg "-" = empty.
 *   alg: md5 sha1 sha224 sha256 sha384 sha512 gost256 gost512
 *   chunk 0 = one update per repetition, else fixed-size updates.
 * stdout: one digest (lowercase hex) per line.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "crypto/hash/md5.h"
#include "crypto/hash/sha1.h"
#include "crypto/hash/sha2.h"
#include "crypto/hash/gost3411-2012.h"

static size_t
unhex(const char *s, uint8_t *out) {
	size_t n = 0;
	unsigned v;

	if (0 == strcmp(s, "-") || 0 == strcmp(s, "="))
		return (0);
	while (s[0] && s[1] && 1 == sscanf(s, "%2x", &v)) {
		out[n ++] = (uint8_t)v;
		s += 2;
	}
	return (n);
}

static void
feed(void (*upd)(void *, const uint8_t *, size_t), void *ctx, const uint8_t *m,
    size_t n, size_t repeat, size_t chunk) {
	size_t r, i, c;
	uint8_t *all;

	if (0 == chunk) {
		for (r = 0; r < repeat; r ++)
			upd(ctx, m, n);
		return;
	}
	all = malloc(n * repeat + 1);
	for (r = 0; r < repeat; r ++)
		memcpy(all + r * n, m, n);
	for (i = 0; i < n * repeat; i += c) {
		c = ((n * repeat - i) < chunk ? (n * repeat - i) : chunk);
		upd(ctx, all + i, c);
	}
	free(all);
}

static void u_md5(void *c, const uint8_t *d, size_t n) { md5_update(c, d, n); }
static void u_sha1(void *c, const uint8_t *d, size_t n) { sha1_update(c, d, n); }
static void u_sha2(void *c, const uint8_t *d, size_t n) { sha2_update(c, d, n); }
static void u_gost(void *c, const uint8_t *d, size_t n) { gost3411_2012_update(c, d, n); }
static void u_hmd5(void *c, const uint8_t *d, size_t n) { hmac_md5_update(c, d, n); }
static void u_hsha1(void *c, const uint8_t *d, size_t n) { hmac_sha1_update(c, d, n); }
static void u_hsha2(void *c, const uint8_t *d, size_t n) { hmac_sha2_update(c, d, n); }
static void u_hgost(void *c, const uint8_t *d, size_t n) { hmac_gost3411_2012_update(c, d, n); }

int
main(void) {
	static char alg[32], khex[4096], mhex[1 << 20];
	static uint8_t key[2048], msg[1 << 19];
	size_t repeat, chunk, kn, mn, ds = 0;
	uint8_t dig[64];
	char str[129];

	while (5 == scanf("%31s %4095s %1048575s %zu %zu", alg, khex, mhex, &repeat, &chunk)) {
		int hm = strcmp(khex, "-");
		kn = unhex(khex, key);
		mn = unhex(mhex, msg);
		if (0 == strcmp(alg, "md5")) {
			if (hm) { hmac_md5_ctx_t c; hmac_md5_init(key, kn, &c);
				feed(u_hmd5, &c, msg, mn, repeat, chunk); hmac_md5_final(&c, dig); }
			else { md5_ctx_t c; md5_init(&c); feed(u_md5, &c, msg, mn, repeat, chunk); md5_final(&c, dig); }
			ds = MD5_HASH_SIZE;
		} else if (0 == strcmp(alg, "sha1")) {
			if (hm) { hmac_sha1_ctx_t c; hmac_sha1_init(key, kn, &c);
				feed(u_hsha1, &c, msg, mn, repeat, chunk); hmac_sha1_final(&c, dig); }
			else { sha1_ctx_t c; sha1_init(&c); feed(u_sha1, &c, msg, mn, repeat, chunk); sha1_final(&c, dig); }
			ds = SHA1_HASH_SIZE;
		} else if (0 == strncmp(alg, "sha", 3)) {
			size_t bits = (size_t)atoi(alg + 3);
			if (hm) { hmac_sha2_ctx_t c; hmac_sha2_init(bits, key, kn, &c);
				feed(u_hsha2, &c, msg, mn, repeat, chunk); hmac_sha2_final(&c, dig, &ds); }
			else { sha2_ctx_t c; sha2_init(bits, &c); ds = c.hash_size;
				feed(u_sha2, &c, msg, mn, repeat, chunk); sha2_final(&c, dig); }
		} else {
			size_t bits = (size_t)atoi(alg + 4);
			if (hm) { hmac_gost3411_2012_ctx_t c; hmac_gost3411_2012_init(bits, key, kn, &c);
				feed(u_hgost, &c, msg, mn, repeat, chunk); hmac_gost3411_2012_final(&c, dig, &ds); }
			else { gost3411_2012_ctx_t c; gost3411_2012_init(bits, &c); ds = c.hash_size;
				feed(u_gost, &c, msg, mn, repeat, chunk); gost3411_2012_final(&c, dig); }
		}
		sha2_cvt_hex(dig, ds, (uint8_t*)str);
		printf("%s\n", str);
	}
	return (0);
}
