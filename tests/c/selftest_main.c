/* Runs the drop-in headers' own *_self_test() functions (tests/hash/main.c
 * style: exit code = first failing test's code). */
#include <stdio.h>

#define MD5_SELF_TEST 1
#define SHA1_SELF_TEST 1
#define SHA2_SELF_TEST 1
#define GOST3411_2012_SELF_TEST 1

#include "crypto/hash/md5.h"
#include "crypto/hash/sha1.h"
#include "crypto/hash/sha2.h"
#include "crypto/hash/gost3411-2012.h"

int
main(void) {
	int e;

	if ((e = md5_self_test())) { printf("md5 %d\n", e); return (e); }
	if ((e = sha1_self_test())) { printf("sha1 %d\n", e); return (10 + e); }
	if ((e = sha2_self_test())) { printf("sha2 %d\n", e); return (20 + e); }
	if ((e = gost3411_2012_self_test())) { printf("gost %d\n", e); return (30 + e); }
	return (0);
}
