/*
 * lcb_hash_batch_multi's stream contract (include/lcb_hash_gpu.h, ABI v4)
 * from a plain C caller: the batch is written on the device asynchronously
 * on the caller's non-default stream (behind a long memset that delays it),
 * then hashed over two parts (devs {0, 0}, LCB_HASH_F_COPY_PARTS: the
 * peer-copy path on one GPU) with NO host synchronisation in between; every
 * digest must equal the drop-in md5.h single-message call on the bytes the
 * stream wrote.  Built with gcc by tests/test_c_caller_gpu.py.
 * stdout: "OK <messages>", or the first mismatch (exit 1).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "crypto/hash/md5.h"
#include "lcb_hash_gpu.h"

#define NMSG	65536
#define MSGLEN	1000		/* ragged description, unaligned records */
#define DELAY_BYTES	((size_t)2 << 30)

int
main(void) {
	hipStream_t s;
	uint8_t *d_data = NULL, *d_dig = NULL, *d_delay = NULL, *h_data, *h_dig;
	uint64_t *h_off, *d_off = NULL;
	uint32_t *h_len, *d_len = NULL;
	int devs[2] = {0, 0}, err;
	size_t i, total = (size_t)NMSG * MSGLEN + 7;
	uint8_t md[MD5_HASH_SIZE];

	if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
	    hipMalloc((void**)&d_data, total) != hipSuccess ||
	    hipMalloc((void**)&d_dig, (size_t)NMSG * 16) != hipSuccess ||
	    hipMalloc((void**)&d_off, (size_t)NMSG * 8) != hipSuccess ||
	    hipMalloc((void**)&d_len, (size_t)NMSG * 4) != hipSuccess ||
	    hipMalloc((void**)&d_delay, DELAY_BYTES) != hipSuccess) {
		printf("HIP allocation failed\n");
		return (1);
	}
	h_data = malloc(total);
	h_dig = malloc((size_t)NMSG * 16);
	h_off = malloc((size_t)NMSG * 8);
	h_len = malloc((size_t)NMSG * 4);
	for (i = 0; i < NMSG; i ++) {
		h_off[i] = 7 + (uint64_t)i * MSGLEN;	/* odd start: every alignment */
		h_len[i] = MSGLEN - (uint32_t)(i % 3);
	}
	/* Stale bytes first, synchronously: what a racing batch would see. */
	if (hipMemset(d_data, 0xa5, total) != hipSuccess ||
	    hipMemcpy(d_off, h_off, (size_t)NMSG * 8, hipMemcpyHostToDevice) != hipSuccess ||
	    hipMemcpy(d_len, h_len, (size_t)NMSG * 4, hipMemcpyHostToDevice) != hipSuccess ||
	    hipDeviceSynchronize() != hipSuccess) {
		printf("HIP setup failed\n");
		return (1);
	}
	/* Asynchronous on `s`: a long memset, then the real batch bytes. */
	if (hipMemsetAsync(d_delay, 1, DELAY_BYTES, s) != hipSuccess ||
	    hipMemsetAsync(d_delay, 2, DELAY_BYTES, s) != hipSuccess) {
		printf("hipMemsetAsync failed\n");
		return (1);
	}
	err = lcb_hash_gen_synthetic(0x5eedull, 0, d_data, total, s);
	if (0 == err)
		err = lcb_hash_batch_multi(devs, 2, LCB_HASH_MD5, NULL, 0, d_data, d_off, d_len,
		    NMSG, 0, 0, d_dig, LCB_HASH_F_DEVICE | LCB_HASH_F_COPY_PARTS, s);
	if (0 != err) {
		printf("error %d (%s)\n", err, lcb_hash_strerror(err));
		return (1);
	}
	if (hipStreamSynchronize(s) != hipSuccess ||
	    hipMemcpy(h_data, d_data, total, hipMemcpyDeviceToHost) != hipSuccess ||
	    hipMemcpy(h_dig, d_dig, (size_t)NMSG * 16, hipMemcpyDeviceToHost) != hipSuccess) {
		printf("HIP readback failed\n");
		return (1);
	}
	for (i = 0; i < NMSG; i ++) {
		md5_get_digest(h_data + h_off[i], h_len[i], md);
		if (memcmp(md, h_dig + i * 16, 16)) {
			printf("MISMATCH message %zu\n", i);
			return (1);
		}
	}
	printf("OK %d\n", NMSG);
	return (0);
}
