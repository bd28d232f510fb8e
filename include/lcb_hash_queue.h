/*
 * lcb_hash_queue.h — asynchronous packet ingestion for the MI355X batch digest
 * engine (liblcb_hash_gpu.so), SURVEY.md §8(f) row 2.
 *
 * In the reference, packets arrive one at a time on thread-pool threads:
 * tp_task_pkt_rcvr_handler() (src/threadpool/threadpool_task.c:661-725)
 * recvfrom()s each datagram into the task's io_buf (include/utils/io_buf.h:
 * 40-47) and calls the task callback, which hashes it with a one-message
 * call (e.g. include/proto/radius.h:776-830, md5 / hmac-md5 per packet).
 * A GPU cannot usefully take one 1-4 KiB message per call, so this queue
 * turns those per-packet calls into batches without changing the callers'
 * shape:
 *
 *   - any number of threads call lcb_hash_queue_submit() with a packet
 *     (or lcb_hash_queue_submitv() with segments, e.g. packet || secret as
 *     radius.h:776-789 hashes it); the bytes are copied into the open
 *     batch's page-locked staging arena (lock-free slot reservation), and
 *     the call returns;
 *   - a flusher thread seals the open batch when it is full
 *     (max_batch_msgs / max_batch_bytes) or its first packet is flush_usec
 *     old, DMAs it to HBM, runs the batch kernel and copies the digests back
 *     (with every staging slot in flight, the sealed batch is launched first
 *     and producers wait for the next slot to be returned);
 *   - a completion thread delivers every digest: it is copied to the
 *     submitter's `digest` pointer (if any) and `cb(udata, error, digest,
 *     size)` is called (if any).  The callback runs on the queue's
 *     completion thread, exactly like a tpt_msg_cb delivered by
 *     tpt_msg_send() (src/threadpool/threadpool_msg_sys.c:279): a thread-pool
 *     caller forwards it to the submitting thread with tpt_msg_send(), see
 *     INTEGRATION.md.
 *
 * Digests equal the reference one-shot function of the queue's algorithm
 * (md5_get_digest, md5_hmac_get_digest, ...) over the submitted bytes.
 * Batches complete in submission order; within a batch callbacks run in
 * slot order.  Errors are liblcb errno codes as in lcb_hash_gpu.h, plus
 * EMSGSIZE (packet larger than a batch) and EAGAIN (LCB_HASH_Q_F_NOWAIT and
 * no free staging slot).  There is no CPU fallback.
 */
#ifndef LCB_HASH_QUEUE_H
#define LCB_HASH_QUEUE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lcb_hash_queue_s *lcb_hash_queue_p;

/* Completion: error 0 and digest != NULL, or error != 0 and digest NULL. */
typedef void (*lcb_hash_done_cb)(void *udata, int error, const uint8_t *digest,
    size_t digest_size);

typedef struct lcb_hash_queue_settings_s {
	size_t	max_batch_msgs;	/* Seal a batch at this many packets. */
	size_t	max_batch_bytes; /* ... or this many staged bytes. */
	uint32_t flush_usec;	/* ... or when its first packet is this old. */
	uint32_t batches;	/* Staging slots (in flight + open), 2..16. */
	uint32_t align;		/* Packet start alignment in staging, 1..4096, power of 2. */
	uint32_t flags;		/* Reserved, 0. */
} lcb_hash_queue_settings_t, *lcb_hash_queue_settings_p;

/* Segment of a packet for lcb_hash_queue_submitv(). */
typedef struct lcb_hash_seg_s {
	const uint8_t	*data;
	size_t		size;
} lcb_hash_seg_t;

typedef struct lcb_hash_queue_stats_s {
	uint64_t	packets;	/* Completed packets. */
	uint64_t	bytes;		/* Completed payload bytes. */
	uint64_t	batches;	/* Launched batches. */
	uint64_t	sealed_full;	/* ... sealed because full. */
	uint64_t	sealed_timer;	/* ... sealed by flush_usec. */
	uint64_t	sealed_flush;	/* ... sealed by flush()/wait(). */
	uint64_t	max_batch_msgs;	/* Largest launched batch. */
	uint64_t	submit_waits;	/* Submits that had to wait for a slot. */
	uint64_t	flusher_drain_ns; /* Flusher: waiting for leases, filling holes. */
	uint64_t	flusher_launch_ns; /* Flusher: enqueueing copies and kernels. */
	uint64_t	completer_busy_ns; /* Completer: digest copies + callbacks. */
	uint64_t	gpu_wait_ns;	/* Completer: waiting for launched batches. */
	/* Worst single batch / submit seen, per pipeline stage (ns): */
	uint64_t	max_fill_ns;	/* first packet in a slot -> its seal. */
	uint64_t	max_launch_ns;	/* seal -> copies and kernel enqueued. */
	uint64_t	max_gpu_ns;	/* enqueued (or the completer free) -> done. */
	uint64_t	max_callback_ns; /* a batch's digest copies + callbacks. */
	uint64_t	max_submit_wait_ns; /* a submit blocked for an open slot. */
	/* The steps of the launch that set max_launch_ns (ns): reopen (install
	 * the next open slot), drain (wait for the leases, fill holes), rebase
	 * (only batches with zero-copy packets: coalesce their runs, rebase
	 * their addresses), index/length + arena copies enqueued, zero-copy run
	 * copies enqueued, bucketing + batch kernels enqueued, completion event
	 * recorded.  Their sum is max_launch_ns. */
	uint64_t	max_launch_steps_ns[7];
} lcb_hash_queue_stats_t;

/* Submit flags. */
#define LCB_HASH_Q_F_NOWAIT	0x0001u	/* EAGAIN instead of waiting for a slot. */
/* Zero copy: the packet lies in a page-locked region registered with
 * lcb_hash_queue_register() (e.g. the thread pool's receive io_bufs,
 * include/utils/io_buf.h:40-47, recvfrom()'d in place,
 * src/threadpool/threadpool_task.c:692-721): the producer copies nothing,
 * the queue records the packet's address and length.  When the batch
 * launches, its zero-copy packets are coalesced into runs (a packet that
 * follows the end of a run within 256 B extends it); every run that lies in
 * one registered region and fits the slot's device arena moves to the device
 * with ONE bulk host-to-device copy, and only a packet outside such a run is
 * read by the kernel in place over PCIe (GOST reads each message twice, in
 * its Sigma pass and its compression pass: such a packet crosses PCIe twice).
 * The bytes must stay unchanged until the packet's completion (digest
 * written / callback called).  One segment
 * only (lcb_hash_queue_submitv with nsegs == 1); EINVAL if
 * [data, data + size) is not inside one registered region. */
#define LCB_HASH_Q_F_ZEROCOPY	0x0002u

/* Defaults: 65536 packets, 16 MiB, 200 us, 4 slots, 16-byte alignment. */
void	lcb_hash_queue_settings_def(lcb_hash_queue_settings_p s);

/* key == NULL: plain digests; key != NULL: HMAC with that key (copied). */
int	lcb_hash_queue_create(int alg, const uint8_t *key, size_t key_len,
	    const lcb_hash_queue_settings_t *s, lcb_hash_queue_p *q_out);
/* Waits for every submitted packet, then frees the queue. */
void	lcb_hash_queue_destroy(lcb_hash_queue_p q);

int	lcb_hash_queue_submit(lcb_hash_queue_p q, const uint8_t *data,
	    size_t size, uint8_t *digest, lcb_hash_done_cb cb, void *udata,
	    uint32_t flags);
int	lcb_hash_queue_submitv(lcb_hash_queue_p q, const lcb_hash_seg_t *segs,
	    size_t nsegs, uint8_t *digest, lcb_hash_done_cb cb, void *udata,
	    uint32_t flags);

/* Register page-locked host memory (hipHostMalloc / hipHostRegister) as a
 * zero-copy packet source, for the queue's lifetime; up to 16 regions.
 * EINVAL if [base, base + size) is not page-locked memory of one allocation,
 * ENOMEM when the table is full.  Call before the submits that use it.
 * There is no unregister: a registered region must stay allocated and
 * page-locked until lcb_hash_queue_destroy() has returned (submits validate
 * against the table lock-free, so freeing a region while the queue lives
 * would let a later submit in that address range pass validation). */
int	lcb_hash_queue_register(lcb_hash_queue_p q, const void *base, size_t size);

/* Seal the open batch now (returns at once). */
int	lcb_hash_queue_flush(lcb_hash_queue_p q);
/* Flush and wait until every packet submitted before the call completed;
 * returns the first error any batch reported (0 if none). */
int	lcb_hash_queue_wait(lcb_hash_queue_p q);
int	lcb_hash_queue_stats(lcb_hash_queue_p q, lcb_hash_queue_stats_t *st);

/* Diagnostics (environment, read once per process): LCB_QUEUE_TRACE=1 logs
 * every stall over 1 ms to stderr (a slow launch step, a batch the
 * completion thread picked up late, the flusher waiting for a free slot, a
 * submit waiting for an open slot, a batch slower than 1 ms end to end);
 * LCB_QUEUE_TRACE=2 also samples the flusher's stack (it takes SIGUSR2 for
 * the process) while one launch's enqueues take over 2 ms. */

#ifdef __cplusplus
}
#endif

#endif /* LCB_HASH_QUEUE_H */
