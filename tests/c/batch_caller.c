/*
 * A plain C caller of the batch C-ABI (include/lcb_hash_gpu.h), the way a
 * liblcb maintainer would wire it next to the per-packet code
 * (INTEGRATION.md 2): ragged packets in ordinary (pageable) host memory at
 * any byte alignment, hashed by the reference-named *_get_digest_batch entry
 * points in host mode, every digest compared with the single-message call of
 * the drop-in headers (include/crypto/hash/, the CPU path callers already
 * compile).  Built with gcc by tests/test_c_caller_gpu.py.
 * stdout: "OK <messages> <checks>", or the first mismatch (exit 1).
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "crypto/hash/md5.h"
#include "crypto/hash/sha1.h"
#include "crypto/hash/sha2.h"
#include "crypto/hash/gost3411-2012.h"
#include "lcb_hash_gpu.h"

#define NMSG	3000

static uint64_t rng = 0x9e3779b97f4a7c15ull;

static uint32_t
next32(void) {
	rng ^= rng << 13;
	rng ^= rng >> 7;
	rng ^= rng << 17;
	return ((uint32_t)(rng >> 16));
}

static int
check(const char *what, size_t i, const uint8_t *got, const uint8_t *exp, size_t n) {
	if (0 == memcmp(got, exp, n))
		return (0);
	printf("MISMATCH %s message %zu\n", what, i);
	return (1);
}

int
main(void) {
	uint64_t *offs = malloc(NMSG * sizeof(uint64_t));
	uint32_t *lens = malloc(NMSG * sizeof(uint32_t));
	uint8_t *data, *dig = malloc((size_t)NMSG * 64);
	const uint8_t key[] = "radius-shared-secret-of-a-peer";
	uint8_t exp[64];
	size_t total = 0, i, ds = 0, checks = 0;
	int rc, bad = 0;

	for (i = 0; i < NMSG; i ++) {
		lens[i] = (i % 97 == 0) ? 0 : (next32() % 2100);
		total += (next32() & 15);	/* any byte alignment */
		offs[i] = total;
		total += lens[i];
	}
	data = malloc(total + 1);
	for (i = 0; i < total; i ++)
		data[i] = (uint8_t)next32();

	if (lcb_hash_gpu_device_count() <= 0) {
		printf("NODEV\n");
		return (2);
	}
	rc = md5_get_digest_batch(data, offs, lens, NMSG, 0, 0, dig, 0, NULL);
	if (rc) { printf("md5 rc %d (%s)\n", rc, lcb_hash_strerror(rc)); return (1); }
	for (i = 0; i < NMSG && !bad; i ++, checks ++) {
		md5_get_digest(data + offs[i], lens[i], exp);
		bad = check("md5", i, dig + i * MD5_HASH_SIZE, exp, MD5_HASH_SIZE);
	}
	rc = md5_hmac_get_digest_batch(key, sizeof(key) - 1, data, offs, lens, NMSG, 0, 0, dig, 0, NULL);
	if (rc) { printf("hmac-md5 rc %d\n", rc); return (1); }
	for (i = 0; i < NMSG && !bad; i ++, checks ++) {
		md5_hmac_get_digest(key, sizeof(key) - 1, data + offs[i], lens[i], exp);
		bad = check("hmac-md5", i, dig + i * MD5_HASH_SIZE, exp, MD5_HASH_SIZE);
	}
	rc = sha1_get_digest_batch(data, offs, lens, NMSG, 0, 0, dig, 0, NULL);
	if (rc) { printf("sha1 rc %d\n", rc); return (1); }
	for (i = 0; i < NMSG && !bad; i ++, checks ++) {
		sha1_get_digest(data + offs[i], lens[i], exp);
		bad = check("sha1", i, dig + i * SHA1_HASH_SIZE, exp, SHA1_HASH_SIZE);
	}
	rc = sha2_get_digest_batch(256, data, offs, lens, NMSG, 0, 0, dig, &ds, 0, NULL);
	if (rc || ds != SHA2_256_HASH_SIZE) { printf("sha256 rc %d ds %zu\n", rc, ds); return (1); }
	for (i = 0; i < NMSG && !bad; i ++, checks ++) {
		sha2_get_digest(256, data + offs[i], lens[i], exp, NULL);
		bad = check("sha256", i, dig + i * ds, exp, ds);
	}
	rc = sha2_get_digest_batch(384, data, offs, lens, NMSG, 0, 0, dig, &ds, 0, NULL);
	if (rc || ds != SHA2_384_HASH_SIZE) { printf("sha384 rc %d ds %zu\n", rc, ds); return (1); }
	for (i = 0; i < NMSG && !bad; i ++, checks ++) {
		sha2_get_digest(384, data + offs[i], lens[i], exp, NULL);
		bad = check("sha384", i, dig + i * ds, exp, ds);
	}
	rc = gost3411_2012_get_digest_batch(512, data, offs, lens, NMSG, 0, 0, dig, &ds, 0, NULL);
	if (rc || ds != GOST3411_2012_512_HASH_SIZE) { printf("gost512 rc %d ds %zu\n", rc, ds); return (1); }
	for (i = 0; i < NMSG && !bad; i ++, checks ++) {
		gost3411_2012_get_digest(512, data + offs[i], lens[i], exp, NULL);
		bad = check("gost512", i, dig + i * ds, exp, ds);
	}
	/* Fixed stride: every 1 KiB record of the same buffer. */
	rc = md5_get_digest_batch(data, NULL, NULL, total / 1024, 1024, 1024, dig, 0, NULL);
	if (rc) { printf("md5 fixed rc %d\n", rc); return (1); }
	for (i = 0; i < total / 1024 && !bad; i ++, checks ++) {
		md5_get_digest(data + i * 1024, 1024, exp);
		bad = check("md5 fixed", i, dig + i * MD5_HASH_SIZE, exp, MD5_HASH_SIZE);
	}
	/* Argument errors are reported, not UB. */
	if (EINVAL != sha2_get_digest_batch(100, data, offs, lens, NMSG, 0, 0, dig, &ds, 0, NULL)) {
		printf("sha2 bits 100 not EINVAL\n");
		return (1);
	}
	if (bad)
		return (1);
	printf("OK %d %zu\n", NMSG, checks);
	free(data);
	free(dig);
	free(offs);
	free(lens);
	return (0);
}
