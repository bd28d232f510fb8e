/* Single-thread speed of the one-shot *_get_digest over 1 KiB messages,
 * every algorithm: built once against the reference's headers and once
 * against this repo's drop-in headers with the same flags
 * (tools/dropin_speed.sh) — the SURVEY.md 8(d) calibration of the drop-in
 * CPU path against the reference.  Prints "alg MiB/s checksum". */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#ifdef SPEED_SIMD
#	include <immintrin.h>
#else
#	undef __SSE2__		/* as tests/hash/main.c:36 */
#endif
#include "crypto/hash/md5.h"
#include "crypto/hash/sha1.h"
#include "crypto/hash/sha2.h"
#include "crypto/hash/gost3411-2012.h"

static double
now(void) {
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ((double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec);
}

int
main(int argc, char **argv) {
	const size_t len = 1024;
	size_t n = (argc > 1 ? strtoul(argv[1], NULL, 10) : 16384), i, k;
	uint8_t *buf = malloc(n * len), d[64];
	const char *names[] = { "md5", "sha1", "sha224", "sha256", "sha384", "sha512", "gost256", "gost512" };
	uint64_t x = 0x6c62636861736821ull;

	for (i = 0; i < n * len; i ++) {
		x = x * 6364136223846793005ull + 1442695040888963407ull;
		buf[i] = (uint8_t)(x >> 56);
	}
	for (k = 0; k < 8; k ++) {
		size_t m = (k >= 6 ? n / 4 : n);	/* GOST is ~8x slower */
		uint32_t sum = 0;
		double t0 = now();
		for (i = 0; i < m; i ++) {
			const uint8_t *p = buf + i * len;
			switch (k) {
			case 0: md5_get_digest(p, len, d); break;
			case 1: sha1_get_digest(p, len, d); break;
			case 2: sha2_get_digest(224, p, len, d, NULL); break;
			case 3: sha2_get_digest(256, p, len, d, NULL); break;
			case 4: sha2_get_digest(384, p, len, d, NULL); break;
			case 5: sha2_get_digest(512, p, len, d, NULL); break;
			case 6: gost3411_2012_get_digest(256, p, len, d, NULL); break;
			case 7: gost3411_2012_get_digest(512, p, len, d, NULL); break;
			}
			sum = sum * 31 + d[0] + ((uint32_t)d[5] << 8);
		}
		printf("%s %.1f %08x\n", names[k], (double)(m * len) / (now() - t0) / 1048576.0, sum);
	}
	free(buf);
	return (0);
}
