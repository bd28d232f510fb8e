/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see lcb_oracle.h).
 *
 * Plain, unoptimised C restatement of rozhuk-im/liblcb include/crypto/hash.
 * Every routine names the reference lines it follows; the constants are the
 * published FIPS 180 / RFC 1321 / RFC 6986 values.  Parity is pinned against
 * the reference's own KAT tables and against the compiled reference
 * (oracle/_ref) by tests/test_oracle_golden.py.
 */
#include <string.h>
#include "lcb_oracle.h"

static uint32_t rol32(uint32_t x, unsigned n) { return (x << n) | (x >> (32 - n)); }
static uint32_t ror32(uint32_t x, unsigned n) { return (x >> n) | (x << (32 - n)); }
static uint64_t ror64(uint64_t x, unsigned n) { return (x >> n) | (x << (64 - n)); }
static uint32_t ld_le32(const uint8_t *p) {
	return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static uint32_t ld_be32(const uint8_t *p) {
	return (uint32_t)p[3] | ((uint32_t)p[2] << 8) | ((uint32_t)p[1] << 16) | ((uint32_t)p[0] << 24);
}
static uint64_t ld_be64(const uint8_t *p) {
	return ((uint64_t)ld_be32(p) << 32) | ld_be32(p + 4);
}
static uint64_t ld_le64(const uint8_t *p) {
	return ((uint64_t)ld_le32(p + 4) << 32) | ld_le32(p);
}
static void st_le32(uint8_t *p, uint32_t v) { for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (8 * i)); }
static void st_be32(uint8_t *p, uint32_t v) { for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (24 - 8 * i)); }
static void st_be64(uint8_t *p, uint64_t v) { for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (56 - 8 * i)); }
static void st_le64(uint8_t *p, uint64_t v) { for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i)); }

size_t or_digest_size(int alg) {
	static const size_t ds[9] = { 0, 16, 20, 28, 32, 48, 64, 32, 64 };
	return (alg >= 1 && alg <= 8) ? ds[alg] : 0;
}
size_t or_block_size(int alg) {
	if (alg < 1 || alg > 8) return 0;
	return (alg == OR_SHA384 || alg == OR_SHA512) ? 128 : 64;
}

/* ------------------------------------------------------------------ MD5 */
/* md5.h:137-229 (md5_transform): 64 steps, round functions md5.h:77-86,
 * shifts md5.h:59-74.  The per-step additive constants are RFC 1321 T[i]. */
static const uint32_t md5_T[64] = {
	0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
	0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
	0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
	0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
	0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
	0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
	0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
	0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391
};
static const uint8_t md5_R[4][4] = { {7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21} };

static void md5_compress(uint32_t h[4], const uint8_t *blk) {
	uint32_t x[16], a = h[0], b = h[1], c = h[2], d = h[3];
	for (int i = 0; i < 16; i++) x[i] = ld_le32(blk + 4 * i);   /* LE words, md5.h:146-151 */
	for (int i = 0; i < 64; i++) {
		uint32_t f; int g, r = i >> 4;
		switch (r) {
		case 0: f = (b & c) | (~b & d); g = i; break;             /* MD5_F */
		case 1: f = (b & d) | (c & ~d); g = (5 * i + 1) & 15; break; /* MD5_G */
		case 2: f = b ^ c ^ d; g = (3 * i + 5) & 15; break;       /* MD5_H */
		default: f = c ^ (b | ~d); g = (7 * i) & 15; break;       /* MD5_I */
		}
		uint32_t t = d;
		d = c; c = b;
		b = b + rol32(a + f + x[g] + md5_T[i], md5_R[r][i & 3]);
		a = t;
	}
	h[0] += a; h[1] += b; h[2] += c; h[3] += d;
}

/* ---------------------------------------------------------------- SHA-1 */
/* sha1.h:220-292 (sha1_transform_generic): BE load :239, expansion :242-244,
 * four 20-round groups with K :223. */
static void sha1_compress(uint32_t h[5], const uint8_t *blk) {
	uint32_t w[80], a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
	for (int i = 0; i < 16; i++) w[i] = ld_be32(blk + 4 * i);
	for (int i = 16; i < 80; i++) w[i] = rol32(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
	for (int i = 0; i < 80; i++) {
		uint32_t f, k;
		if (i < 20) { f = (b & c) | (~b & d); k = 0x5a827999; }
		else if (i < 40) { f = b ^ c ^ d; k = 0x6ed9eba1; }
		else if (i < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8f1bbcdc; }
		else { f = b ^ c ^ d; k = 0xca62c1d6; }
		uint32_t t = rol32(a, 5) + f + e + k + w[i];
		e = d; d = c; c = rol32(b, 30); b = a; a = t;
	}
	h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

/* -------------------------------------------------------------- SHA-256 */
/* sha2.h:260-327 (sha2_transform_block64_generic); sigma macros sha2.h:100-107. */
static const uint32_t sha256_K[64] = {
	0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
	0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
	0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
	0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
	0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
	0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
	0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
	0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2
};
static void sha256_compress(uint32_t h[8], const uint8_t *blk) {
	uint32_t w[64], s[8];
	for (int i = 0; i < 16; i++) w[i] = ld_be32(blk + 4 * i);
	for (int i = 16; i < 64; i++) {
		uint32_t s0 = ror32(w[i - 15], 7) ^ ror32(w[i - 15], 18) ^ (w[i - 15] >> 3);
		uint32_t s1 = ror32(w[i - 2], 17) ^ ror32(w[i - 2], 19) ^ (w[i - 2] >> 10);
		w[i] = w[i - 16] + s0 + w[i - 7] + s1;
	}
	memcpy(s, h, sizeof(s));
	for (int i = 0; i < 64; i++) {
		uint32_t S1 = ror32(s[4], 6) ^ ror32(s[4], 11) ^ ror32(s[4], 25);
		uint32_t ch = (s[4] & s[5]) | (~s[4] & s[6]);
		uint32_t t1 = s[7] + S1 + ch + sha256_K[i] + w[i];
		uint32_t S0 = ror32(s[0], 2) ^ ror32(s[0], 13) ^ ror32(s[0], 22);
		uint32_t mj = (s[0] & s[1]) | (s[0] & s[2]) | (s[1] & s[2]);
		memmove(s + 1, s, 7 * sizeof(uint32_t));
		s[4] += t1;
		s[0] = t1 + S0 + mj;
	}
	for (int i = 0; i < 8; i++) h[i] += s[i];
}

/* -------------------------------------------------------------- SHA-512 */
/* sha2.h:531-613 (sha2_transform_block128_generic); sigma macros sha2.h:109-116. */
static const uint64_t sha512_K[80] = {
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
static void sha512_compress(uint64_t h[8], const uint8_t *blk) {
	uint64_t w[80], s[8];
	for (int i = 0; i < 16; i++) w[i] = ld_be64(blk + 8 * i);
	for (int i = 16; i < 80; i++) {
		uint64_t s0 = ror64(w[i - 15], 1) ^ ror64(w[i - 15], 8) ^ (w[i - 15] >> 7);
		uint64_t s1 = ror64(w[i - 2], 19) ^ ror64(w[i - 2], 61) ^ (w[i - 2] >> 6);
		w[i] = w[i - 16] + s0 + w[i - 7] + s1;
	}
	memcpy(s, h, sizeof(s));
	for (int i = 0; i < 80; i++) {
		uint64_t S1 = ror64(s[4], 14) ^ ror64(s[4], 18) ^ ror64(s[4], 41);
		uint64_t ch = (s[4] & s[5]) | (~s[4] & s[6]);
		uint64_t t1 = s[7] + S1 + ch + sha512_K[i] + w[i];
		uint64_t S0 = ror64(s[0], 28) ^ ror64(s[0], 34) ^ ror64(s[0], 39);
		uint64_t mj = (s[0] & s[1]) | (s[0] & s[2]) | (s[1] & s[2]);
		memmove(s + 1, s, 7 * sizeof(uint64_t));
		s[4] += t1;
		s[0] = t1 + S0 + mj;
	}
	for (int i = 0; i < 8; i++) h[i] += s[i];
}

/* IVs: md5.h:126-134, sha1.h:177-181, sha2.h:129-148. */
static const uint32_t iv_sha224[8] = {
	0xc1059ed8, 0x367cd507, 0x3070dd17, 0xf70e5939, 0xffc00b31, 0x68581511, 0x64f98fa7, 0xbefa4fa4 };
static const uint32_t iv_sha256[8] = {
	0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19 };
static const uint64_t iv_sha384[8] = {
	0xcbbb9d5dc1059ed8ull, 0x629a292a367cd507ull, 0x9159015a3070dd17ull, 0x152fecd8f70e5939ull,
	0x67332667ffc00b31ull, 0x8eb44a8768581511ull, 0xdb0c2e0d64f98fa7ull, 0x47b5481dbefa4fa4ull };
static const uint64_t iv_sha512[8] = {
	0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull, 0xa54ff53a5f1d36f1ull,
	0x510e527fade682d1ull, 0x9b05688c2b3e6c1full, 0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull };

/* ------------------------------------------------ GOST R 34.11-2012 */
/* RFC 6986 pi (S-box), the linear map A (64 rows) and the 12 iteration
 * constants C; the reference holds the same values at
 * gost3411-2012.h:108-141 (sbox), :161-178 (A), :887-949 (C). */
static const char gost_pi_hex[] =
	"fceedd11cf6e3116fbc4fada23c5044de977f0db932e99ba1736f1bb14cd5fc1"
	"f918655ae25cef21811c3c428b018e4f058402aee36a8fa0060bed987fd4d31f"
	"eb342c51eac848abf22a68a2fd3aceccb5700e56080c7612bf7213479cb75d87"
	"15a19629107b9ac7f391786f9d9eb2b13275193dff358a7e6d54c680c3bd0d57"
	"dff524a93ea843c9d779d6f67c22b903e00fecde7a94b0bcdce828504e330a4a"
	"a79760731e0062441ab83882649f2641ad454692275e552f8ca3a57d69d5953b"
	"0758b34086ac1df730376be488d9e789e11b83494c3ff8fe8d53aa90cad88561"
	"207167a42d2b095bcb9b25d0bee56c5259a674d2e6f4b4c0d166afc2394b63b6";
static const uint64_t gost_A[64] = {
	0x8E20FAA72BA0B470u, 0x47107DDD9B505A38u, 0xAD08B0E0C3282D1Cu, 0xD8045870EF14980Eu,
	0x6C022C38F90A4C07u, 0x3601161CF205268Du, 0x1B8E0B0E798C13C8u, 0x83478B07B2468764u,
	0xA011D380818E8F40u, 0x5086E740CE47C920u, 0x2843FD2067ADEA10u, 0x14AFF010BDD87508u,
	0x0AD97808D06CB404u, 0x05E23C0468365A02u, 0x8C711E02341B2D01u, 0x46B60F011A83988Eu,
	0x90DAB52A387AE76Fu, 0x486DD4151C3DFDB9u, 0x24B86A840E90F0D2u, 0x125C354207487869u,
	0x092E94218D243CBAu, 0x8A174A9EC8121E5Du, 0x4585254F64090FA0u, 0xACCC9CA9328A8950u,
	0x9D4DF05D5F661451u, 0xC0A878A0A1330AA6u, 0x60543C50DE970553u, 0x302A1E286FC58CA7u,
	0x18150F14B9EC46DDu, 0x0C84890AD27623E0u, 0x0642CA05693B9F70u, 0x0321658CBA93C138u,
	0x86275DF09CE8AAA8u, 0x439DA0784E745554u, 0xAFC0503C273AA42Au, 0xD960281E9D1D5215u,
	0xE230140FC0802984u, 0x71180A8960409A42u, 0xB60C05CA30204D21u, 0x5B068C651810A89Eu,
	0x456C34887A3805B9u, 0xAC361A443D1C8CD2u, 0x561B0D22900E4669u, 0x2B838811480723BAu,
	0x9BCF4486248D9F5Du, 0xC3E9224312C8C1A0u, 0xEFFA11AF0964EE50u, 0xF97D86D98A327728u,
	0xE4FA2054A80B329Cu, 0x727D102A548B194Eu, 0x39B008152ACB8227u, 0x9258048415EB419Du,
	0x492C024284FBAEC0u, 0xAA16012142F35760u, 0x550B8E9E21F7A530u, 0xA48B474F9EF5DC18u,
	0x70A6A56E2440598Eu, 0x3853DC371220A247u, 0x1CA76E95091051ADu, 0x0EDD37C48A08A6D8u,
	0x07E095624504536Cu, 0x8D70C431AC02A736u, 0xC83862965601DD1Bu, 0x641C314B2B8EE083u
};
static const uint64_t gost_C[12][8] = {
	{ 0xDD806559F2A64507u, 0x05767436CC744D23u, 0xA2422A08A460D315u, 0x4B7CE09192676901u,
	  0x714EB88D7585C4FCu, 0x2F6A76432E45D016u, 0xEBCB2F81C0657C1Fu, 0xB1085BDA1ECADAE9u },
	{ 0xE679047021B19BB7u, 0x55DDA21BD7CBCD56u, 0x5CB561C2DB0AA7CAu, 0x9AB5176B12D69958u,
	  0x61D55E0F16B50131u, 0xF3FEEA720A232B98u, 0x4FE39D460F70B5D7u, 0x6FA3B58AA99D2F1Au },
	{ 0x991E96F50ABA0AB2u, 0xC2B6F443867ADB31u, 0xC1C93A376062DB09u, 0xD3E20FE490359EB1u,
	  0xF2EA7514B1297B7Bu, 0x06F15E5F529C1F8Bu, 0x0A39FC286A3D8435u, 0xF574DCAC2BCE2FC7u },
	{ 0x220CBEBC84E3D12Eu, 0x3453EAA193E837F1u, 0xD8B71333935203BEu, 0xA9D72C82ED03D675u,
	  0x9D721CAD685E353Fu, 0x488E857E335C3C7Du, 0xF948E1A05D71E4DDu, 0xEF1FDFB3E81566D2u },
	{ 0x601758FD7C6CFE57u, 0x7A56A27EA9EA63F5u, 0xDFFF00B723271A16u, 0xBFCD1747253AF5A3u,
	  0x359E35D7800FFFBDu, 0x7F151C1F1686104Au, 0x9A3F410C6CA92363u, 0x4BEA6BACAD474799u },
	{ 0xFA68407A46647D6Eu, 0xBF71C57236904F35u, 0x0AF21F66C2BEC6B6u, 0xCFFAA6B71C9AB7B4u,
	  0x187F9AB49AF08EC6u, 0x2D66C4F95142A46Cu, 0x6FA4C33B7A3039C0u, 0xAE4FAEAE1D3AD3D9u },
	{ 0x8886564D3A14D493u, 0x3517454CA23C4AF3u, 0x06476983284A0504u, 0x0992ABC52D822C37u,
	  0xD3473E33197A93C9u, 0x399EC6C7E6BF87C9u, 0x51AC86FEBF240954u, 0xF4C70E16EEAAC5ECu },
	{ 0xA47F0DD4BF02E71Eu, 0x36ACC2355951A8D9u, 0x69D18D2BD1A5C42Fu, 0xF4892BCB929B0690u,
	  0x89B4443B4DDBC49Au, 0x4EB7F8719C36DE1Eu, 0x03E7AA020C6E4141u, 0x9B1F5B424D93C9A7u },
	{ 0x7261445183235ADBu, 0x0E38DC92CB1F2A60u, 0x7B2B8A9AA6079C54u, 0x800A440BDBB2CEB1u,
	  0x3CD955B7E00D0984u, 0x3A7D3A1B25894224u, 0x944C9AD8EC165FDEu, 0x378F5A541631229Bu },
	{ 0x74B4C7FB98459CEDu, 0x3698FAD1153BB6C3u, 0x7A1E6C303B7652F4u, 0x9FE76702AF69334Bu,
	  0x1FFFE18A1B336103u, 0x8941E71CFF8A78DBu, 0x382AE548B2E4F3F3u, 0xABBEDEA680056F52u },
	{ 0x6BCAA4CD81F32D1Bu, 0xDEA2594AC06FD85Du, 0xEFBACD1D7D476E98u, 0x8A1D71EFEA48B9CAu,
	  0x2001802114846679u, 0xD8FA6BBBEBAB0761u, 0x3002C6CD635AFE94u, 0x7BCD9ED0EFC889FBu },
	{ 0x48BC924AF11BD720u, 0xFAF417D5D9B21B99u, 0xE71DA4AA88E12852u, 0x5D80EF9D1891CC86u,
	  0xF82012D430219F9Bu, 0xCDA43C32BCDF1D77u, 0xD21380B00449B17Au, 0x378EE767F11631BAu }
};

static uint8_t gost_pi[256];
static uint64_t gost_ax[8][256];
static int gost_ready;

/* L() of a single 64-bit row, most significant bit selecting A[0]
 * (small-table form, gost3411-2012.h:1056-1064). */
static uint64_t gost_L(uint64_t v) {
	uint64_t c = 0;
	for (int b = 0; b < 64; b++, v <<= 1)
		if (v & 0x8000000000000000ull) c ^= gost_A[b];
	return c;
}

/* The small-table LPS (gost3411-2012.h:1032-1067) is linear in the
 * pi-substituted bytes, so it is tabulated once: Ax[j][b] = L(pi[b] << 8j)
 * — the big-table form of gost3411-2012.h:1071-1090. */
static void gost_setup(void) {
	if (gost_ready) return;
	for (int i = 0; i < 256; i++) {
		int hi = gost_pi_hex[2 * i], lo = gost_pi_hex[2 * i + 1];
		hi = (hi <= '9') ? hi - '0' : hi - 'a' + 10;
		lo = (lo <= '9') ? lo - '0' : lo - 'a' + 10;
		gost_pi[i] = (uint8_t)((hi << 4) | lo);
	}
	for (int j = 0; j < 8; j++)
		for (int b = 0; b < 256; b++)
			gost_ax[j][b] = gost_L((uint64_t)gost_pi[b] << (8 * j));
	gost_ready = 1;
}

/* LPS: byte k = 8*j + i of the LE state (byte i of word j) goes through pi
 * and lands at tau(k) = 8*i + j, then L() per output word. */
static void gost_lps(uint64_t dst[8], const uint64_t src[8]) {
	for (int i = 0; i < 8; i++) {
		uint64_t c = 0;
		for (int j = 0; j < 8; j++)
			c ^= gost_ax[j][(src[j] >> (8 * i)) & 0xff];
		dst[i] = c;
	}
}

/* 512-bit little-endian add with carry (gost3411-2012.h:996-1013). */
static void gost_add512(uint64_t a[8], const uint64_t b[8]) {
	unsigned carry = 0;
	for (int i = 0; i < 8; i++) {
		uint64_t s = a[i] + b[i];
		unsigned c1 = s < a[i];
		uint64_t s2 = s + carry;
		unsigned c2 = s2 < s;
		a[i] = s2;
		carry = c1 | c2;
	}
}

/* g_N(h, m) with optional counter update (gost3411-2012.h:1110-1167):
 * K = LPS(h ^ N); E(K, m) = 12 rounds of X, LPS with key schedule
 * K_{i+1} = LPS(K_i ^ C_i); h ^= E ^ m ^ ...  (final XOR :1142). */
static void gost_g(uint64_t h[8], const uint64_t N[8], const uint64_t m[8]) {
	uint64_t k[8], t[8], x[8];
	for (int i = 0; i < 8; i++) x[i] = h[i] ^ N[i];
	gost_lps(k, x);
	for (int i = 0; i < 8; i++) x[i] = k[i] ^ m[i];
	gost_lps(t, x);
	for (int r = 0; r < 12; r++) {
		for (int i = 0; i < 8; i++) x[i] = k[i] ^ gost_C[r][i];
		gost_lps(k, x);
		if (r < 11) {
			for (int i = 0; i < 8; i++) x[i] = t[i] ^ k[i];
			gost_lps(t, x);
		}
	}
	for (int i = 0; i < 8; i++) h[i] ^= m[i] ^ t[i] ^ k[i];
}

static void gost_block(or_ctx_t *c, const uint8_t *blk, uint64_t bits) {
	uint64_t m[8], add[8] = { 0 };
	for (int i = 0; i < 8; i++) m[i] = ld_le64(blk + 8 * i);  /* native LE words, :1123-1128 */
	gost_g(c->h64, c->gn, m);
	add[0] = bits;
	gost_add512(c->gn, add);     /* N += bits, :1130 */
	gost_add512(c->gs, m);       /* Sigma += m, :1131 */
}

/* --------------------------------------------------- streaming core */
static void compress_blk(or_ctx_t *c, const uint8_t *blk) {
	switch (c->alg) {
	case OR_MD5: md5_compress(c->h32, blk); break;
	case OR_SHA1: sha1_compress(c->h32, blk); break;
	case OR_SHA224: case OR_SHA256: sha256_compress(c->h32, blk); break;
	case OR_SHA384: case OR_SHA512: sha512_compress(c->h64, blk); break;
	default: gost_block(c, blk, 512); break;
	}
}

int or_init(or_ctx_t *c, int alg) {
	memset(c, 0, sizeof(*c));
	c->alg = alg;
	switch (alg) {
	case OR_MD5: case OR_SHA1:
		c->h32[0] = 0x67452301; c->h32[1] = 0xefcdab89; c->h32[2] = 0x98badcfe;
		c->h32[3] = 0x10325476; c->h32[4] = 0xc3d2e1f0; break;
	case OR_SHA224: memcpy(c->h32, iv_sha224, 32); break;
	case OR_SHA256: memcpy(c->h32, iv_sha256, 32); break;
	case OR_SHA384: memcpy(c->h64, iv_sha384, 64); break;
	case OR_SHA512: memcpy(c->h64, iv_sha512, 64); break;
	case OR_GOST256: memset(c->h64, 0x01, 64); gost_setup(); break;  /* gost3411-2012.h:1717-1722 */
	case OR_GOST512: gost_setup(); break;                             /* IV 0, :1723-1728 */
	default: return -1;
	}
	return 0;
}

/* Block buffering as md5_update (md5.h:233-262), sha2_update (sha2.h:647-681)
 * and gost3411_2012_update (gost3411-2012.h:1767-1799). */
void or_update(or_ctx_t *c, const uint8_t *d, size_t n) {
	size_t bs = or_block_size(c->alg);
	uint64_t old = c->count;
	c->count += n;
	if (c->count < old) c->count_hi++;
	while (n > 0) {
		size_t take = bs - c->used;
		if (take > n) take = n;
		memcpy(c->buf + c->used, d, take);
		c->used += take; d += take; n -= take;
		if (c->used == bs) { compress_blk(c, c->buf); c->used = 0; }
	}
}

void or_final(or_ctx_t *c, uint8_t *digest) {
	size_t bs = or_block_size(c->alg), ds = or_digest_size(c->alg);
	if (c->alg == OR_GOST256 || c->alg == OR_GOST512) {
		/* gost3411-2012.h:1820-1843: 0x01 then zeros, g_N with N += used*8,
		 * then g_0(h, N), g_0(h, Sigma); digest = last ds bytes of h. */
		uint64_t zero[8] = { 0 }, n[8], s[8];
		uint64_t used = c->used;
		memset(c->buf + used, 0, 64 - used);
		c->buf[used] = 0x01;
		gost_block(c, c->buf, used * 8);
		memcpy(n, c->gn, 64); memcpy(s, c->gs, 64);
		gost_g(c->h64, zero, n);
		gost_g(c->h64, zero, s);
		uint8_t full[64];
		for (int i = 0; i < 8; i++) st_le64(full + 8 * i, c->h64[i]);
		memcpy(digest, full + 64 - ds, ds);
		memset(c, 0, sizeof(*c));
		return;
	}
	/* md5.h:266-288 / sha1.h:816-840 / sha2.h:706-742. */
	size_t lenoff = bs - ((bs == 128) ? 16 : 8);
	c->buf[c->used++] = 0x80;
	if (c->used > lenoff) {
		memset(c->buf + c->used, 0, bs - c->used);
		compress_blk(c, c->buf);
		c->used = 0;
	}
	memset(c->buf + c->used, 0, bs - c->used);
	uint64_t bits = c->count << 3;
	if (c->alg == OR_MD5) {
		st_le64(c->buf + 56, bits);
	} else if (bs == 64) {
		st_be64(c->buf + 56, bits);
	} else {
		st_be64(c->buf + 112, (c->count_hi << 3) | (c->count >> 61));
		st_be64(c->buf + 120, bits);
	}
	compress_blk(c, c->buf);
	switch (c->alg) {
	case OR_MD5: for (int i = 0; i < 4; i++) st_le32(digest + 4 * i, c->h32[i]); break;
	case OR_SHA1: case OR_SHA224: case OR_SHA256: {
		uint8_t full[32];
		for (int i = 0; i < 8; i++) st_be32(full + 4 * i, c->h32[i]);
		memcpy(digest, full, ds);
		break;
	}
	default: {
		uint8_t full[64];
		for (int i = 0; i < 8; i++) st_be64(full + 8 * i, c->h64[i]);
		memcpy(digest, full, ds);
		break;
	}
	}
	memset(c, 0, sizeof(*c));
}

int or_digest(int alg, const uint8_t *d, size_t n, uint8_t *digest) {
	or_ctx_t c;
	if (or_init(&c, alg)) return -1;
	or_update(&c, d, n);
	or_final(&c, digest);
	return 0;
}

/* RFC 2104 as hmac_md5_init/final (md5.h:309-359), hmac_sha2_* (sha2.h:763-828),
 * hmac_gost3411_2012_* (gost3411-2012.h:1864-1934): a key longer than the
 * block is replaced by its digest, zero-padded to the block, ipad 0x36, opad 0x5c. */
int or_hmac(int alg, const uint8_t *key, size_t key_len,
    const uint8_t *d, size_t n, uint8_t *digest) {
	size_t bs = or_block_size(alg), ds = or_digest_size(alg);
	uint8_t k[128] = { 0 }, pad[128], inner[64];
	or_ctx_t c;
	if (bs == 0) return -1;
	if (key_len > bs) or_digest(alg, key, key_len, k);
	else memcpy(k, key, key_len);
	for (size_t i = 0; i < bs; i++) pad[i] = k[i] ^ 0x36;
	or_init(&c, alg); or_update(&c, pad, bs); or_update(&c, d, n); or_final(&c, inner);
	for (size_t i = 0; i < bs; i++) pad[i] = k[i] ^ 0x5c;
	or_init(&c, alg); or_update(&c, pad, bs); or_update(&c, inner, ds); or_final(&c, digest);
	return 0;
}

int or_batch(int alg, const uint8_t *key, size_t key_len,
    const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths,
    size_t count, uint64_t stride, uint32_t fixed_len, uint8_t *digests) {
	size_t ds = or_digest_size(alg);
	if (ds == 0) return -1;
	for (size_t i = 0; i < count; i++) {
		const uint8_t *p = base + (offsets ? offsets[i] : (uint64_t)i * stride);
		size_t n = lengths ? lengths[i] : fixed_len;
		if (key) or_hmac(alg, key, key_len, p, n, digests + i * ds);
		else or_digest(alg, p, n, digests + i * ds);
	}
	return 0;
}

/* Keyed batches (lcb_hash_batch_keyed): message i with key k = key_index[i]
 * (NULL: 0) of the table keys + key_offsets[k] (NULL: 0), key_lengths[k]:
 *   mode 1  HMAC(K, m)                 radius.h:850-919 (hmac_md5_*)
 *   mode 2  H(K || m)                  radius.h:774-789 (md5_update(key) then
 *                                      (authenticator | c_j) from a ctx copy)
 *   mode 3  H(m || K)                  radius.h:1331-1336, 1346-1352 */
int or_batch_keyed(int alg, int mode, const uint8_t *keys, const uint64_t *key_offsets,
    const uint32_t *key_lengths, size_t nkeys, const uint32_t *key_index,
    const uint8_t *base, const uint64_t *offsets, const uint32_t *lengths,
    size_t count, uint64_t stride, uint32_t fixed_len, uint8_t *digests) {
	size_t ds = or_digest_size(alg);
	if (ds == 0 || nkeys == 0 || mode < 1 || mode > 3) return -1;
	for (size_t i = 0; i < count; i++) {
		const uint8_t *p = base + (offsets ? offsets[i] : (uint64_t)i * stride);
		size_t n = lengths ? lengths[i] : fixed_len;
		size_t k = key_index ? key_index[i] : 0;
		if (k >= nkeys) return -1;
		const uint8_t *K = keys + (key_offsets ? key_offsets[k] : 0);
		size_t kl = key_lengths[k];
		or_ctx_t c;
		if (mode == 1) {
			or_hmac(alg, K, kl, p, n, digests + i * ds);
			continue;
		}
		or_init(&c, alg);
		if (mode == 2) { or_update(&c, K, kl); or_update(&c, p, n); }
		else { or_update(&c, p, n); or_update(&c, K, kl); }
		or_final(&c, digests + i * ds);
	}
	return 0;
}

/* ------------------------------------------------- synthetic input */
uint64_t or_mix64(uint64_t x) {
	uint64_t z = x + 0x9e3779b97f4a7c15ull;
	z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
	z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
	return z ^ (z >> 31);
}

void or_gen_bytes(uint64_t seed, uint64_t start, uint8_t *out, size_t n) {
	for (size_t i = 0; i < n; i++) {
		uint64_t b = start + i;
		out[i] = (uint8_t)(or_mix64(seed ^ (b >> 3)) >> (8 * (b & 7)));
	}
}
