/*
 * crypto/hash/sha2.h — source-compatible drop-in for liblcb's sha2.h
 * (reference include/crypto/hash/sha2.h), clean-room.
 *
 * SHA-224/256 (64-byte blocks) and SHA-384/512 (128-byte blocks) behind the
 * reference's `bits` convention (sha2.h:213-251): 224|28, 256|32, 384|48,
 * 512|64.  Unlike the reference (which leaves the context uninitialised), an
 * unknown `bits` value selects nothing: hash_size and block_size are set to 0
 * and update/final become no-ops that write no digest.
 * Portable C only (no SHA-NI, no per-init cpuid).  One-message CPU path;
 * batches go through include/lcb_hash_gpu.h.  FIPS 180-4, RFC 2104.
 */
#ifndef __SHA2_H__INCLUDED__
#define __SHA2_H__INCLUDED__

#include <sys/param.h>
#include <sys/types.h>
#include <string.h>
#include <inttypes.h>

#ifndef nitems
#	define nitems(__val)	(sizeof(__val) / sizeof(__val[0]))
#endif

#define SHA2_224_HASH_SIZE	((size_t)28)
#define SHA2_256_HASH_SIZE	((size_t)32)
#define SHA2_384_HASH_SIZE	((size_t)48)
#define SHA2_512_HASH_SIZE	((size_t)64)
#define SHA2_HASH_MAX_SIZE	SHA2_512_HASH_SIZE

#define SHA2_224_HASH_STR_SIZE	(SHA2_224_HASH_SIZE * 2)
#define SHA2_256_HASH_STR_SIZE	(SHA2_256_HASH_SIZE * 2)
#define SHA2_384_HASH_STR_SIZE	(SHA2_384_HASH_SIZE * 2)
#define SHA2_512_HASH_STR_SIZE	(SHA2_512_HASH_SIZE * 2)
#define SHA2_HASH_STR_MAX_SIZE	SHA2_512_HASH_STR_SIZE

#define SHA2_256_MSG_BLK_SIZE	((size_t)64)
#define SHA2_512_MSG_BLK_SIZE	((size_t)128)
#define SHA2_MSG_BLK_MAX_SIZE	SHA2_512_MSG_BLK_SIZE
#define SHA2_256_MSG_BLK_64CNT	(SHA2_256_MSG_BLK_SIZE / sizeof(uint64_t))
#define SHA2_512_MSG_BLK_64CNT	(SHA2_512_MSG_BLK_SIZE / sizeof(uint64_t))
#define SHA2_MSG_BLK_MAX_64CNT	(SHA2_MSG_BLK_MAX_SIZE / sizeof(uint64_t))

/* Initial hash values (FIPS 180-4 5.3). */
static const uint32_t SHA2_224_H0[8] = {
	0xc1059ed8, 0x367cd507, 0x3070dd17, 0xf70e5939,
	0xffc00b31, 0x68581511, 0x64f98fa7, 0xbefa4fa4 };
static const uint32_t SHA2_256_H0[8] = {
	0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
	0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19 };
static const uint64_t SHA2_384_H0[8] = {
	0xcbbb9d5dc1059ed8ull, 0x629a292a367cd507ull, 0x9159015a3070dd17ull, 0x152fecd8f70e5939ull,
	0x67332667ffc00b31ull, 0x8eb44a8768581511ull, 0xdb0c2e0d64f98fa7ull, 0x47b5481dbefa4fa4ull };
static const uint64_t SHA2_512_H0[8] = {
	0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull, 0xa54ff53a5f1d36f1ull,
	0x510e527fade682d1ull, 0x9b05688c2b3e6c1full, 0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull };

#define SHA2_ALIGN(__n)	__attribute__ ((aligned(__n)))
#if defined(__SHA__) && defined(__SSSE3__) && defined(__SSE4_1__) && \
    (defined(__x86_64__) || defined(__i386__))
/* Built with the SHA extensions enabled (as the reference's SIMD build):
 * SHA-224/256 blocks go through the SHA-NI instructions when the CPU has
 * them (checked once per context by sha2_init, like the reference's
 * use_simd). */
#	define SHA2_ENABLE_SIMD	1
#	include <immintrin.h>
#	include <cpuid.h>
#endif

/* Field for field the reference's layout (sha2.h:152-163), including the
 * build-dependent tail (tests/test_dropin_headers.py pins sizeof / offsetof). */
typedef struct sha2_ctx_s {
	SHA2_ALIGN(32) uint64_t hash[(SHA2_HASH_MAX_SIZE / sizeof(uint64_t))]; /* 224/256: 8 x u32 packed */
	SHA2_ALIGN(32) uint64_t buffer[SHA2_MSG_BLK_MAX_64CNT];	/* partial block */
	SHA2_ALIGN(32) uint64_t W[80];	/* message schedule scratch */
	uint64_t count;		/* bytes hashed, low 64 bits */
	uint64_t count_hi;	/* bytes hashed, high 64 bits */
	size_t hash_size;	/* 28, 32, 48 or 64 (0: invalid bits) */
	size_t block_size;	/* 64 or 128 */
#ifdef SHA2_ENABLE_SIMD
	int use_simd;		/* SHA-NI available (sha2_init) */
#endif
} sha2_ctx_t, *sha2_ctx_p;

typedef struct hmac_sha2_ctx_s {
	sha2_ctx_t ctx;
	SHA2_ALIGN(32) uint64_t k_opad[SHA2_MSG_BLK_MAX_64CNT];
} hmac_sha2_ctx_t, *hmac_sha2_ctx_p;

static void *(*volatile sha2_wipe_fn)(void *, int, size_t) = memset;

static inline uint32_t
sha2_ror32(const uint32_t x, const unsigned n) {
	return ((x >> n) | (x << (32 - n)));
}

static inline uint64_t
sha2_ror64(const uint64_t x, const unsigned n) {
	return ((x >> n) | (x << (64 - n)));
}

static inline uint64_t
sha2_load_be(const uint8_t *p, const size_t n) {
	uint64_t v = 0;
	size_t i;

	for (i = 0; i < n; i ++) {
		v = ((v << 8) | p[i]);
	}
	return (v);
}

#ifdef SHA2_ENABLE_SIMD
/* SHA-NI usable on this CPU (SHA, SSSE3, SSE4.1). */
static inline int
sha2_cpu_has_sha_ni(void) {
#if defined(__GNUC__) && !defined(__clang__) && (__GNUC__ >= 11)
	/* libgcc's cpu model, filled in at program start: no cpuid per call. */
	return (__builtin_cpu_supports("sha") && __builtin_cpu_supports("ssse3") &&
	    __builtin_cpu_supports("sse4.1"));
#else
	unsigned int a, b, c, d;

	if (0 == __get_cpuid(1, &a, &b, &c, &d) ||
	    0 == (c & (1u << 9)) || 0 == (c & (1u << 19)))	/* SSSE3, SSE4.1 */
		return (0);
	if (0 == __get_cpuid_count(7, 0, &a, &b, &c, &d))
		return (0);
	return (0 != (b & (1u << 29)));				/* SHA */
#endif
}
#endif

static inline void
sha2_init(const size_t bits, sha2_ctx_p ctx) {

	memset(ctx, 0x00, sizeof(sha2_ctx_t));
	switch (bits) {
	case 224:
	case SHA2_224_HASH_SIZE:
		ctx->hash_size = SHA2_224_HASH_SIZE;
		ctx->block_size = SHA2_256_MSG_BLK_SIZE;
		memcpy(ctx->hash, SHA2_224_H0, sizeof(SHA2_224_H0));
		break;
	case 256:
	case SHA2_256_HASH_SIZE:
		ctx->hash_size = SHA2_256_HASH_SIZE;
		ctx->block_size = SHA2_256_MSG_BLK_SIZE;
		memcpy(ctx->hash, SHA2_256_H0, sizeof(SHA2_256_H0));
		break;
	case 384:
	case SHA2_384_HASH_SIZE:
		ctx->hash_size = SHA2_384_HASH_SIZE;
		ctx->block_size = SHA2_512_MSG_BLK_SIZE;
		memcpy(ctx->hash, SHA2_384_H0, sizeof(SHA2_384_H0));
		break;
	case 512:
	case SHA2_512_HASH_SIZE:
		ctx->hash_size = SHA2_512_HASH_SIZE;
		ctx->block_size = SHA2_512_MSG_BLK_SIZE;
		memcpy(ctx->hash, SHA2_512_H0, sizeof(SHA2_512_H0));
		break;
	}
#ifdef SHA2_ENABLE_SIMD
	ctx->use_simd = sha2_cpu_has_sha_ni();
#endif
}

static inline void
sha2_transform_block64(sha2_ctx_p ctx, const uint8_t *blk) {
	static const uint32_t K[64] = {
		0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
		0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
		0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
		0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
		0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
		0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
		0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
		0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2
	};
	uint32_t *h = (uint32_t*)ctx->hash, w[16], s[8], t1, t2, x, y, ab, bc;
	size_t i;

	for (i = 0; i < 16; i ++) {
		w[i] = (uint32_t)sha2_load_be(blk + 4 * i, 4);
	}
	memcpy(s, h, sizeof(s));
	bc = (s[1] ^ s[2]);
#pragma GCC unroll 64
	for (i = 0; i < 64; i ++) {
		if (i >= 16) {
			x = w[(i + 1) & 15];	/* W[i-15] */
			y = w[(i + 14) & 15];	/* W[i-2] */
			w[i & 15] += ((sha2_ror32(x, 7) ^ sha2_ror32(x, 18) ^ (x >> 3)) +
			    w[(i + 9) & 15] +
			    (sha2_ror32(y, 17) ^ sha2_ror32(y, 19) ^ (y >> 10)));
		}
		/* h + K + W does not wait for this round's e; Maj(a, b, c) =
		 * b ^ ((a ^ b) & (b ^ c)), and a ^ b is the next round's b ^ c. */
		t1 = ((s[7] + (K[i] + w[i & 15])) + (s[6] ^ (s[4] & (s[5] ^ s[6]))) +
		    (sha2_ror32(s[4], 6) ^ sha2_ror32(s[4], 11) ^ sha2_ror32(s[4], 25)));
		ab = (s[0] ^ s[1]);
		t2 = ((sha2_ror32(s[0], 2) ^ sha2_ror32(s[0], 13) ^ sha2_ror32(s[0], 22)) +
		    (s[1] ^ (ab & bc)));
		bc = ab;
		s[7] = s[6]; s[6] = s[5]; s[5] = s[4]; s[4] = s[3] + t1;
		s[3] = s[2]; s[2] = s[1]; s[1] = s[0]; s[0] = (t1 + t2);
	}
	for (i = 0; i < 8; i ++) {
		h[i] += s[i];
	}
}

static inline void
sha2_transform_block128(sha2_ctx_p ctx, const uint8_t *blk) {
	static const uint64_t K[80] = {
		0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
		0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
		0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
		0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
		0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
		0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
		0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
		0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
		0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
		0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
		0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
		0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
		0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
		0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
		0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
		0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
		0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
		0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
		0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
		0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull
	};
	uint64_t *h = ctx->hash, w[16], s[8], t1, t2, x, y, ab, bc;
	size_t i;

	for (i = 0; i < 16; i ++) {
		w[i] = sha2_load_be(blk + 8 * i, 8);
	}
	memcpy(s, h, sizeof(s));
	bc = (s[1] ^ s[2]);
#pragma GCC unroll 80
	for (i = 0; i < 80; i ++) {
		if (i >= 16) {
			x = w[(i + 1) & 15];
			y = w[(i + 14) & 15];
			w[i & 15] += ((sha2_ror64(x, 1) ^ sha2_ror64(x, 8) ^ (x >> 7)) +
			    w[(i + 9) & 15] +
			    (sha2_ror64(y, 19) ^ sha2_ror64(y, 61) ^ (y >> 6)));
		}
		t1 = ((s[7] + (K[i] + w[i & 15])) + (s[6] ^ (s[4] & (s[5] ^ s[6]))) +
		    (sha2_ror64(s[4], 14) ^ sha2_ror64(s[4], 18) ^ sha2_ror64(s[4], 41)));
		ab = (s[0] ^ s[1]);
		t2 = ((sha2_ror64(s[0], 28) ^ sha2_ror64(s[0], 34) ^ sha2_ror64(s[0], 39)) +
		    (s[1] ^ (ab & bc)));	/* Maj, as in the 64-byte block */
		bc = ab;
		s[7] = s[6]; s[6] = s[5]; s[5] = s[4]; s[4] = s[3] + t1;
		s[3] = s[2]; s[2] = s[1]; s[1] = s[0]; s[0] = (t1 + t2);
	}
	for (i = 0; i < 8; i ++) {
		h[i] += s[i];
	}
}

#ifdef SHA2_ENABLE_SIMD
/* SHA-224/256 blocks with the SHA-NI instructions.  The state is kept as
 * the two lane groups the instructions use, {A, B, E, F} and {C, D, G, H};
 * each sha256rnds2 does two rounds, the message schedule four words at a
 * time (sha256msg1: W[t-16] + sigma0(W[t-15]); + W[t-7]; sha256msg2 adds
 * sigma1 of the last two words). */
__attribute__((target("sha,ssse3,sse4.1")))
static inline void
sha2_transform_block64_shani(sha2_ctx_p ctx, const uint8_t *blocks, const uint8_t *blocks_max) {
	static const uint32_t K4[64] SHA2_ALIGN(16) = {
		0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
		0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
		0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
		0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
		0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
		0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
		0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
		0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2
	};
	const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bll, 0x0405060700010203ll);
	uint32_t *h = (uint32_t*)ctx->hash;
	__m128i t, abef, cdgh, abef0, cdgh0, wk, m[4];
	size_t g;

	t = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)(const void*)&h[0]), 0xb1);	/* C D A B */
	cdgh = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)(const void*)&h[4]), 0x1b);	/* H G F E */
	abef = _mm_alignr_epi8(t, cdgh, 8);						/* A B E F */
	cdgh = _mm_blend_epi16(cdgh, t, 0xf0);						/* C D G H */
	for (; blocks < blocks_max; blocks += SHA2_256_MSG_BLK_SIZE) {
		abef0 = abef;
		cdgh0 = cdgh;
#pragma GCC unroll 16
		for (g = 0; g < 16; g ++) {	/* four rounds per step */
			if (g < 4) {
				m[g] = _mm_shuffle_epi8(_mm_loadu_si128(
				    (const __m128i*)(const void*)(blocks + 16 * g)), bswap);
			} else {
				m[g & 3] = _mm_sha256msg2_epu32(_mm_add_epi32(
				    _mm_sha256msg1_epu32(m[g & 3], m[(g + 1) & 3]),
				    _mm_alignr_epi8(m[(g + 3) & 3], m[(g + 2) & 3], 4)), m[(g + 3) & 3]);
			}
			wk = _mm_add_epi32(m[g & 3], _mm_load_si128((const __m128i*)(const void*)&K4[4 * g]));
			cdgh = _mm_sha256rnds2_epu32(cdgh, abef, wk);
			abef = _mm_sha256rnds2_epu32(abef, cdgh, _mm_shuffle_epi32(wk, 0x0e));
		}
		abef = _mm_add_epi32(abef, abef0);
		cdgh = _mm_add_epi32(cdgh, cdgh0);
	}
	t = _mm_shuffle_epi32(abef, 0x1b);					/* F E B A */
	cdgh = _mm_shuffle_epi32(cdgh, 0xb1);					/* D C H G */
	_mm_storeu_si128((__m128i*)(void*)&h[0], _mm_blend_epi16(t, cdgh, 0xf0));	/* D C B A */
	_mm_storeu_si128((__m128i*)(void*)&h[4], _mm_alignr_epi8(cdgh, t, 8));	/* H G F E */
}
#endif

/* Compress every block in [blocks, blocks_max) (any alignment). */
static inline void
sha2_transform(sha2_ctx_p ctx, const uint8_t *blocks, const uint8_t *blocks_max) {

	if (0 == ctx->block_size)
		return;
#ifdef SHA2_ENABLE_SIMD
	if (0 != ctx->use_simd && SHA2_256_MSG_BLK_SIZE == ctx->block_size) {
		sha2_transform_block64_shani(ctx, blocks, blocks_max);
		return;
	}
#endif
	for (; blocks < blocks_max; blocks += ctx->block_size) {
		if (SHA2_256_MSG_BLK_SIZE == ctx->block_size) {
			sha2_transform_block64(ctx, blocks);
		} else {
			sha2_transform_block128(ctx, blocks);
		}
	}
}

static inline void
sha2_update(sha2_ctx_p ctx, const uint8_t *data, size_t data_size) {
	size_t bs = ctx->block_size, used, take, whole;

	if (0 == bs || 0 == data_size)
		return;
	used = (size_t)(ctx->count & (bs - 1));
	ctx->count += data_size;
	if (ctx->count < data_size) {
		ctx->count_hi ++;
	}
	if (0 != used) {
		take = (bs - used);
		if (take > data_size) {
			take = data_size;
		}
		memcpy(((uint8_t*)ctx->buffer) + used, data, take);
		used += take;
		data += take;
		data_size -= take;
		if (bs != used)
			return;
		sha2_transform(ctx, (const uint8_t*)ctx->buffer, ((const uint8_t*)ctx->buffer) + bs);
	}
	whole = (data_size & ~(bs - 1));
	if (0 != whole) {
		sha2_transform(ctx, data, (data + whole));
	}
	if (data_size != whole) {
		memcpy(ctx->buffer, data + whole, (data_size - whole));
	}
}

static inline void
sha2_final(sha2_ctx_p ctx, uint8_t *digest) {
	uint8_t *buf = (uint8_t*)ctx->buffer;
	size_t bs = ctx->block_size, lenlen, used, i;
	uint64_t lo, hi;

	if (0 == bs)
		return;
	lenlen = ((SHA2_256_MSG_BLK_SIZE == bs) ? 8 : 16);
	used = (size_t)(ctx->count & (bs - 1));
	lo = (ctx->count << 3);
	hi = ((ctx->count_hi << 3) | (ctx->count >> 61));
	buf[used ++] = 0x80;
	if (used > (bs - lenlen)) {
		memset(buf + used, 0x00, (bs - used));
		sha2_transform(ctx, buf, (buf + bs));
		used = 0;
	}
	memset(buf + used, 0x00, (bs - used));
	for (i = 0; i < 8; i ++) {	/* big-endian bit count (128-bit for 384/512) */
		buf[(bs - 1) - i] = (uint8_t)(lo >> (8 * i));
		if (16 == lenlen) {
			buf[(bs - 9) - i] = (uint8_t)(hi >> (8 * i));
		}
	}
	sha2_transform(ctx, buf, (buf + bs));
	for (i = 0; i < ctx->hash_size; i ++) {
		if (SHA2_256_MSG_BLK_SIZE == bs) {
			digest[i] = (uint8_t)(((uint32_t*)ctx->hash)[i >> 2] >> (24 - 8 * (i & 3)));
		} else {
			digest[i] = (uint8_t)(ctx->hash[i >> 3] >> (56 - 8 * (i & 7)));
		}
	}
	sha2_wipe_fn(ctx, 0x00, sizeof(sha2_ctx_t));
}

static inline void
hmac_sha2_init(const size_t bits, const uint8_t *key, const size_t key_len,
    hmac_sha2_ctx_p hctx) {
	uint8_t k[SHA2_MSG_BLK_MAX_SIZE];
	size_t bs, i;

	memset(k, 0x00, sizeof(k));
	sha2_init(bits, &hctx->ctx);
	bs = hctx->ctx.block_size;
	if (key_len > bs) {
		sha2_update(&hctx->ctx, key, key_len);
		sha2_final(&hctx->ctx, k);
		sha2_init(bits, &hctx->ctx);
	} else if (0 != key_len) {
		memcpy(k, key, key_len);
	}
	for (i = 0; i < SHA2_MSG_BLK_MAX_SIZE; i ++) {
		((uint8_t*)hctx->k_opad)[i] = (k[i] ^ 0x5c);
		k[i] ^= 0x36;
	}
	sha2_update(&hctx->ctx, k, bs);
	sha2_wipe_fn(k, 0x00, sizeof(k));
}

static inline void
hmac_sha2_update(hmac_sha2_ctx_p hctx, const uint8_t *data, const size_t data_size) {

	sha2_update(&hctx->ctx, data, data_size);
}

static inline void
hmac_sha2_final(hmac_sha2_ctx_p hctx, uint8_t *digest, size_t *digest_size) {
	size_t hs = hctx->ctx.hash_size;

	sha2_final(&hctx->ctx, digest);
	sha2_init(hs, &hctx->ctx);
	sha2_update(&hctx->ctx, (const uint8_t*)hctx->k_opad, hctx->ctx.block_size);
	sha2_update(&hctx->ctx, digest, hs);
	if (NULL != digest_size) {
		(*digest_size) = hs;
	}
	sha2_final(&hctx->ctx, digest);
	sha2_wipe_fn(hctx->k_opad, 0x00, sizeof(hctx->k_opad));
}

static inline void
hmac_sha2(const size_t bits, const uint8_t *key, const size_t key_len,
    const uint8_t *data, const size_t data_size,
    uint8_t *digest, size_t *digest_size) {
	hmac_sha2_ctx_t hctx;

	hmac_sha2_init(bits, key, key_len, &hctx);
	hmac_sha2_update(&hctx, data, data_size);
	hmac_sha2_final(&hctx, digest, digest_size);
}

static inline void
sha2_cvt_hex(const uint8_t *bin, const size_t bin_size, uint8_t *hex) {
	static const char digits[] = "0123456789abcdef";
	size_t i;

	for (i = 0; i < bin_size; i ++) {
		hex[2 * i] = (uint8_t)digits[bin[i] >> 4];
		hex[2 * i + 1] = (uint8_t)digits[bin[i] & 0x0f];
	}
	hex[2 * bin_size] = 0;
}

static inline void
sha2_cvt_str(const uint8_t *digest, const size_t digest_size, char *digest_str) {

	sha2_cvt_hex(digest, digest_size, (uint8_t*)digest_str);
}

static inline void
sha2_get_digest(const size_t bits, const void *data, const size_t data_size,
    uint8_t *digest, size_t *digest_size) {
	sha2_ctx_t ctx;

	sha2_init(bits, &ctx);
	sha2_update(&ctx, (const uint8_t*)data, data_size);
	if (NULL != digest_size) {
		(*digest_size) = ctx.hash_size;
	}
	sha2_final(&ctx, digest);
}

static inline void
sha2_get_digest_str(const size_t bits, const char *data, const size_t data_size,
    char *digest_str, size_t *digest_str_size) {
	uint8_t digest[SHA2_HASH_MAX_SIZE];
	size_t ds = 0;

	sha2_get_digest(bits, data, data_size, digest, &ds);
	sha2_cvt_str(digest, ds, digest_str);
	if (NULL != digest_str_size) {
		(*digest_str_size) = (ds * 2);
	}
}

static inline void
sha2_hmac_get_digest(const size_t bits, const void *key, const size_t key_size,
    const void *data, const size_t data_size, uint8_t *digest,
    size_t *digest_size) {

	hmac_sha2(bits, (const uint8_t*)key, key_size, (const uint8_t*)data, data_size,
	    digest, digest_size);
}

static inline void
sha2_hmac_get_digest_str(const size_t bits, const char *key, const size_t key_size,
    const char *data, const size_t data_size,
    char *digest_str, size_t *digest_str_size) {
	uint8_t digest[SHA2_HASH_MAX_SIZE];
	size_t ds = 0;

	hmac_sha2(bits, (const uint8_t*)key, key_size, (const uint8_t*)data, data_size,
	    digest, &ds);
	sha2_cvt_str(digest, ds, digest_str);
	if (NULL != digest_str_size) {
		(*digest_str_size) = (ds * 2);
	}
}

#ifdef SHA2_SELF_TEST
/* 0 - OK; 1..4 - SHA-224/256/384/512 digest KAT failed; 5..7 - HMAC
 * SHA-256/384/512 failed.  Vectors: FIPS 180 "abc" and RFC 4231 test case 2. */
static inline int
sha2_self_test(void) {
	static const char *abc[4] = {
		"23097d223405d8228642a477bda255b32aadbce4bda0b3f7e36c9da7",
		"ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad",
		"cb00753f45a35e8bb5a03d699ac65007272c32ab0eded1631a8b605a43ff5bed"
		"8086072ba1e7cc2358baeca134c825a7",
		"ddaf35a193617abacc417349ae20413112e6fa4e89a97ea20a9eeee64b55d39a"
		"2192992a274fc1a836ba3c23a3feebbd454d4423643ce80e2a9ac94fa54ca49f"
	};
	static const char *jefe[3] = {
		"5bdcc146bf60754e6a042426089575c75a003f089d2739839dec58b964ec3843",
		"af45d2e376484031617f78d2b58a6b1b9c7ef464f5a01b47e42ec3736322445e"
		"8e2240ca5e69e2c78b3239ecfab21649",
		"164b7a7bfcf819e2e395fbe73b56e0a387bd64222e831fd610270cd7ea250554"
		"9758bf75c05a994a6d034f65f8f0e6fdcaeab1a34d4a6b4b636e070a38bce737"
	};
	static const size_t bits[4] = { 224, 256, 384, 512 };
	char str[SHA2_HASH_STR_MAX_SIZE + 1];
	size_t i, n;

	for (i = 0; i < 4; i ++) {
		sha2_get_digest_str(bits[i], "abc", 3, str, &n);
		if (n != strlen(abc[i]) || 0 != memcmp(str, abc[i], n))
			return ((int)i + 1);
	}
	for (i = 0; i < 3; i ++) {
		sha2_hmac_get_digest_str((256 + 128 * i), "Jefe", 4,
		    "what do ya want for nothing?", 28, str, &n);
		if (n != strlen(jefe[i]) || 0 != memcmp(str, jefe[i], n))
			return ((int)i + 5);
	}
	return (0);
}
#endif

#endif /* __SHA2_H__INCLUDED__ */
