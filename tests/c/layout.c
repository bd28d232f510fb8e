/* Prints sizeof / offsetof of every context struct of crypto/hash/*.h: built
 * once against the reference's headers and once against this repo's drop-in
 * headers with the same flags (tests/test_dropin_headers.py), the two outputs
 * must be identical (mixed translation units and sizeof-based
 * callers see one layout). */
#include <stddef.h>
#include <stdio.h>
#ifdef LAYOUT_SIMD
#	include <immintrin.h>	/* the reference's sha1.h / sha2.h want it first */
#else
#	undef __SSE2__		/* as tests/hash/main.c:36 */
#endif
#include "crypto/hash/md5.h"
#include "crypto/hash/sha1.h"
#include "crypto/hash/sha2.h"
#include "crypto/hash/gost3411-2012.h"

#define F(t, f)	printf("%s.%s %zu %zu\n", #t, #f, offsetof(t, f), sizeof(((t*)0)->f))
#define S(t)	printf("%s %zu %zu\n", #t, sizeof(t), _Alignof(t))

int
main(void) {
	S(md5_ctx_t); F(md5_ctx_t, hash); F(md5_ctx_t, count); F(md5_ctx_t, buffer);
	S(hmac_md5_ctx_t); F(hmac_md5_ctx_t, ctx); F(hmac_md5_ctx_t, k_opad);
	S(sha1_ctx_t); F(sha1_ctx_t, count); F(sha1_ctx_t, hash); F(sha1_ctx_t, buffer); F(sha1_ctx_t, W);
	S(hmac_sha1_ctx_t); F(hmac_sha1_ctx_t, ctx); F(hmac_sha1_ctx_t, k_opad);
	S(sha2_ctx_t); F(sha2_ctx_t, hash); F(sha2_ctx_t, buffer); F(sha2_ctx_t, W); F(sha2_ctx_t, count);
	F(sha2_ctx_t, count_hi); F(sha2_ctx_t, hash_size); F(sha2_ctx_t, block_size);
	S(hmac_sha2_ctx_t); F(hmac_sha2_ctx_t, ctx); F(hmac_sha2_ctx_t, k_opad);
	S(gost3411_2012_ctx_t); F(gost3411_2012_ctx_t, hash_size); F(gost3411_2012_ctx_t, buffer_usage);
	F(gost3411_2012_ctx_t, use_sse); F(gost3411_2012_ctx_t, use_avx); F(gost3411_2012_ctx_t, hash);
	F(gost3411_2012_ctx_t, counter); F(gost3411_2012_ctx_t, sigma); F(gost3411_2012_ctx_t, buffer);
	F(gost3411_2012_ctx_t, kbuf); F(gost3411_2012_ctx_t, tbuf); F(gost3411_2012_ctx_t, sbuf);
	S(hmac_gost3411_2012_ctx_t); F(hmac_gost3411_2012_ctx_t, ctx); F(hmac_gost3411_2012_ctx_t, k_opad);
	return (0);
}
