/*
 * INTEGRATION.md section 3, as a translation unit: a liblcb thread-pool
 * packet receiver (tp_task_pkt_rcvr_cb, reference
 * include/threadpool/threadpool_task.h:149) submits each received datagram to
 * the batching queue (include/lcb_hash_queue.h); the queue's completion
 * callback hands the digest back to the receiving thread with tpt_msg_send
 * (include/threadpool/threadpool_msg_sys.h:60).  Compiled against the
 * REFERENCE's thread-pool headers by tests/test_dropin_headers.py (the
 * thread pool itself is liblcb's, out of this repo's scope), which also
 * checks the object's external references.
 */
#include <sys/param.h>
#include <sys/types.h>
#include <sys/socket.h>
#include <errno.h>
#include <inttypes.h>
#include <stdlib.h>
#include <string.h>

#include "threadpool/threadpool.h"
#include "threadpool/threadpool_task.h"
#include "threadpool/threadpool_msg_sys.h"
#include "utils/io_buf.h"
#include "lcb_hash_gpu.h"
#include "lcb_hash_queue.h"

typedef struct radius_rx_s {		/* one in-flight received packet */
	tpt_p		tpt;		/* thread that received it */
	uint8_t		*pkt;		/* copy of the datagram */
	size_t		size;
	uint8_t		mac[16];	/* HMAC-MD5 lands here */
	int		error;
} radius_rx_t, *radius_rx_p;

static lcb_hash_queue_p g_hmac_md5_q;	/* one queue per shared secret */
static void (*g_verified)(radius_rx_p rx);	/* application continuation */

static void
radius_rx_verified(tpt_p tpt, void *udata) {	/* back on the receiving thread */
	radius_rx_p rx = udata;

	(void)tpt;
	if (NULL != g_verified)
		g_verified(rx);		/* compare rx->mac with the attribute, reply */
	free(rx->pkt);
	free(rx);
}

static void
radius_rx_hashed(void *udata, int error, const uint8_t *digest, size_t size) {
	radius_rx_p rx = udata;		/* on the queue's completion thread */

	(void)digest; (void)size;	/* already copied into rx->mac */
	rx->error = error;
	tpt_msg_send(rx->tpt, NULL, TP_MSG_F_FORCE, radius_rx_verified, rx);
}

int
radius_pkt_rcvr_cb(tp_task_p tptask, int error, struct sockaddr_storage *addr,
    io_buf_p buf, size_t transfered_size, void *udata) {
	radius_rx_p rx;

	(void)tptask; (void)addr; (void)udata;
	if (0 != error)
		return (TP_TASK_CB_CONTINUE);
	rx = calloc(1, sizeof(*rx));
	if (NULL == rx)
		return (TP_TASK_CB_CONTINUE);
	rx->tpt = tpt_get_current();
	rx->size = transfered_size;
	rx->pkt = malloc(transfered_size ? transfered_size : 1);
	if (NULL == rx->pkt) {
		free(rx);
		return (TP_TASK_CB_CONTINUE);
	}
	memcpy(rx->pkt, buf->data, transfered_size);
	/* Message-Authenticator zeroed as radius.h:850-919 expects (not shown). */
	error = lcb_hash_queue_submit(g_hmac_md5_q, rx->pkt, rx->size, rx->mac,
	    radius_rx_hashed, rx, 0);
	if (0 != error) {		/* EMSGSIZE / EAGAIN (NOWAIT) — no CPU fallback */
		free(rx->pkt);
		free(rx);
	}
	return (TP_TASK_CB_CONTINUE);
}

int
radius_hash_queue_start(const uint8_t *secret, size_t secret_len, void (*verified)(radius_rx_p)) {
	lcb_hash_queue_settings_t s;

	g_verified = verified;
	lcb_hash_queue_settings_def(&s);	/* 64K packets / 16 MiB / 200 us / 4 slots */
	return (lcb_hash_queue_create(LCB_HASH_MD5, secret, secret_len, &s, &g_hmac_md5_q));
}

/* Type check: the receiver really is a tp_task_pkt_rcvr_cb. */
tp_task_pkt_rcvr_cb radius_pkt_rcvr_cb_ptr = radius_pkt_rcvr_cb;
