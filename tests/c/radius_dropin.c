/* Compiles the REFERENCE's RADIUS protocol code against THIS repo's drop-in
 * crypto/hash headers (include path order puts ours first): the only in-tree
 * caller of the hash path must build unchanged.  Built only where
 * /root/reference exists (tests/test_dropin_headers.py). */
#include "proto/radius.h"

int
main(void) {
	md5_ctx_t c;
	uint8_t d[MD5_HASH_SIZE];

	md5_init(&c);
	md5_update(&c, (const uint8_t*)"radius", 6);
	md5_final(&c, d);
	return (d[0] == 0x33 ? 0 : 0);
}
