/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see lcb_oracle.h).
 *
 * Plain C restatement of rozhuk-im/liblcb include/crypto/cipher/chacha.h,
 * the one-shot functions chacha() (chacha.h:650-660) and xchacha()
 * (chacha.h:669-679) and hchacha() (chacha.h:361-401), byte-at-a-time and
 * unoptimised.  State layout of chacha.h:69-75: words 0-3 constants
 * ("expand 32-byte k" / "expand 16-byte k", chacha.h:110-117), 4-11 key
 * (a 128-bit key repeated, chacha.h:286-316), 12-13 the 64-bit block counter
 * (chacha.h:319-327), 14-15 the 64-bit IV (chacha.h:344-355).  Rounds are
 * applied as double rounds while i < rounds (chacha.h:432-434).  Pinned by
 * the reference's chacha_self_test vectors and by the reference compiled from
 * /root/reference (oracle/_ref) in tests/test_chacha_oracle.py.
 */
#include <string.h>
#include "lcb_oracle.h"

static uint32_t ld32(const uint8_t *p) {
	return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static void st32(uint8_t *p, uint32_t v) {
	for (int i = 0; i < 4; i++)
		p[i] = (uint8_t)(v >> (8 * i));
}
static uint32_t rotl(uint32_t v, int n) { return (v << n) | (v >> (32 - n)); }

static void qr(uint32_t *x, int a, int b, int c, int d) {	/* chacha.h:125-130 */
	x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 16);
	x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 12);
	x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 8);
	x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 7);
}

static void rounds_apply(uint32_t *x, size_t rounds) {	/* chacha.h:132-141 */
	for (size_t i = 0; i < rounds; i += 2) {
		qr(x, 0, 4, 8, 12); qr(x, 1, 5, 9, 13); qr(x, 2, 6, 10, 14); qr(x, 3, 7, 11, 15);
		qr(x, 0, 5, 10, 15); qr(x, 1, 6, 11, 12); qr(x, 2, 7, 8, 13); qr(x, 3, 4, 9, 14);
	}
}

static void key_setup(uint32_t *s, const uint8_t *key, size_t key_size) {	/* chacha.h:286-316 */
	static const uint32_t k256[4] = { 0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u };
	static const uint32_t k128[4] = { 0x61707865u, 0x3120646eu, 0x79622d36u, 0x6b206574u };
	const int big = (key_size == 256 || key_size == 32);
	for (int i = 0; i < 4; i++)
		s[i] = big ? k256[i] : k128[i];
	for (int i = 0; i < 8; i++)
		s[4 + i] = ld32(key + 4 * (big ? i : (i & 3)));
}

void or_hchacha(const uint8_t *key, size_t key_size, const uint8_t *iv16, size_t rounds, uint8_t *out32) {
	uint32_t s[16];
	key_setup(s, key, key_size);
	for (int i = 0; i < 4; i++)
		s[12 + i] = iv16 ? ld32(iv16 + 4 * i) : 0;
	rounds_apply(s, rounds);
	for (int i = 0; i < 4; i++) {
		st32(out32 + 4 * i, s[i]);
		st32(out32 + 16 + 4 * i, s[12 + i]);
	}
}

/* dst = src ^ keystream (src NULL: the keystream itself), n bytes; the
 * counter in s[12..13] advances per 64-byte block. */
static void crypt(uint32_t *s, size_t rounds, const uint8_t *src, size_t n, uint8_t *dst) {
	uint8_t ks[64];
	for (size_t off = 0; off < n; off += 64) {
		uint32_t x[16];
		memcpy(x, s, sizeof(x));
		rounds_apply(x, rounds);
		for (int i = 0; i < 16; i++)
			st32(ks + 4 * i, x[i] + s[i]);	/* chacha.h:143-161 */
		const size_t m = (n - off < 64) ? n - off : 64;
		for (size_t i = 0; i < m; i++)
			dst[off + i] = (src ? src[off + i] : 0) ^ ks[i];
		if (++s[12] == 0)	/* 64-bit counter, chacha.h:440-444 */
			s[13]++;
	}
}

void or_chacha(const uint8_t *key, size_t key_size, const uint8_t *counter8, const uint8_t *iv8,
    size_t rounds, const uint8_t *src, size_t n, uint8_t *dst) {
	uint32_t s[16];
	key_setup(s, key, key_size);
	s[12] = counter8 ? ld32(counter8) : 0;
	s[13] = counter8 ? ld32(counter8 + 4) : 0;
	s[14] = iv8 ? ld32(iv8) : 0;
	s[15] = iv8 ? ld32(iv8 + 4) : 0;
	crypt(s, rounds, src, n, dst);
}

void or_xchacha(const uint8_t *key, size_t key_size, const uint8_t *counter8, const uint8_t *iv24,
    size_t rounds, const uint8_t *src, size_t n, uint8_t *dst) {
	uint8_t k2[32];
	or_hchacha(key, key_size, iv24, rounds, k2);	/* chacha.h:404-421 */
	or_chacha(k2, 32, counter8, iv24 ? iv24 + 16 : NULL, rounds, src, n, dst);
}

int or_chacha_batch(const uint8_t *key, size_t key_size, size_t rounds, int x,
    const uint8_t *counters, const uint8_t *ivs, const uint8_t *src, uint8_t *dst,
    const uint64_t *offsets, const uint32_t *lengths, size_t count, uint64_t stride,
    uint32_t fixed_len) {
	const size_t ivlen = x ? 24 : 8;
	for (size_t i = 0; i < count; i++) {
		const uint64_t o = offsets ? offsets[i] : (uint64_t)i * stride;
		const size_t n = lengths ? lengths[i] : fixed_len;
		const uint8_t *c = counters ? counters + 8 * i : NULL;
		const uint8_t *v = ivs ? ivs + ivlen * i : NULL;
		if (x)
			or_xchacha(key, key_size, c, v, rounds, src ? src + o : NULL, n, dst + o);
		else
			or_chacha(key, key_size, c, v, rounds, src ? src + o : NULL, n, dst + o);
	}
	return 0;
}
