/*
 * lcb_crc32_gpu.h — batched CRC-32 on the MI355X (liblcb_hash_gpu.so),
 * SURVEY.md §8(f) row 3.
 *
 * The reference's CRC-32 family (include/math/crc32.h) is a set of header
 * macros, one buffer per call, e.g. crc32c(data, size) and
 * crc32c_update(crc, data, size) (crc32.h:501-576).  Each entry point here
 * computes, for every buffer i, exactly the value the named reference macro
 * returns:
 *
 *   init == NULL:  crcs[i] = X(msg_i, len_i)                 (one-shot form)
 *   init != NULL:  crcs[i] = X_update(init[i], msg_i, len_i) (chained form,
 *                  e.g. a packet split over several io_bufs)
 *
 * Buffer description, memory modes (LCB_HASH_F_DEVICE), errors and the
 * absence of any CPU fallback are as in lcb_hash_gpu.h; in device mode
 * `init` and `crcs` are device pointers too.  `crcs` must be 4-byte aligned.
 */
#ifndef LCB_CRC32_GPU_H
#define LCB_CRC32_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Variant ids (crc32.h macro, catalogue name). */
#define LCB_CRC32A		1	/* crc32a       CRC-32/BZIP2    crc32.h:505-508 */
#define LCB_CRC32CKSUM		2	/* crc32cksum   CRC-32/CKSUM    crc32.h:514-517 */
#define LCB_CRC32MPEG2		3	/* crc32mpeg2   CRC-32/MPEG-2   crc32.h:522-525 */
#define LCB_CRC32B		4	/* crc32b       CRC-32/ISO-HDLC crc32.h:532-535 */
#define LCB_CRC32JAMCRC		5	/* crc32jamcrc  CRC-32/JAMCRC   crc32.h:541-544 */
#define LCB_CRC32C		6	/* crc32c       CRC-32/ISCSI    crc32.h:551-554 */
#define LCB_CRC32D		7	/* crc32d       CRC-32/BASE91-D crc32.h:561-564 */
#define LCB_CRC32Q		8	/* crc32q       CRC-32/AIXM     crc32.h:571-574 */

int	lcb_crc32_batch(int variant, const uint32_t *init, const uint8_t *data,
	    const uint64_t *offsets, const uint32_t *lengths, size_t count,
	    uint64_t stride, uint32_t fixed_len, uint32_t *crcs, uint32_t flags,
	    void *stream);

/* Reference-named entry points (same arguments minus the variant). */
int	crc32a_batch(const uint32_t *init, const uint8_t *data,
	    const uint64_t *offsets, const uint32_t *lengths, size_t count,
	    uint64_t stride, uint32_t fixed_len, uint32_t *crcs, uint32_t flags,
	    void *stream);
int	crc32cksum_batch(const uint32_t *init, const uint8_t *data,
	    const uint64_t *offsets, const uint32_t *lengths, size_t count,
	    uint64_t stride, uint32_t fixed_len, uint32_t *crcs, uint32_t flags,
	    void *stream);
int	crc32mpeg2_batch(const uint32_t *init, const uint8_t *data,
	    const uint64_t *offsets, const uint32_t *lengths, size_t count,
	    uint64_t stride, uint32_t fixed_len, uint32_t *crcs, uint32_t flags,
	    void *stream);
int	crc32b_batch(const uint32_t *init, const uint8_t *data,
	    const uint64_t *offsets, const uint32_t *lengths, size_t count,
	    uint64_t stride, uint32_t fixed_len, uint32_t *crcs, uint32_t flags,
	    void *stream);
int	crc32jamcrc_batch(const uint32_t *init, const uint8_t *data,
	    const uint64_t *offsets, const uint32_t *lengths, size_t count,
	    uint64_t stride, uint32_t fixed_len, uint32_t *crcs, uint32_t flags,
	    void *stream);
int	crc32c_batch(const uint32_t *init, const uint8_t *data,
	    const uint64_t *offsets, const uint32_t *lengths, size_t count,
	    uint64_t stride, uint32_t fixed_len, uint32_t *crcs, uint32_t flags,
	    void *stream);
int	crc32d_batch(const uint32_t *init, const uint8_t *data,
	    const uint64_t *offsets, const uint32_t *lengths, size_t count,
	    uint64_t stride, uint32_t fixed_len, uint32_t *crcs, uint32_t flags,
	    void *stream);
int	crc32q_batch(const uint32_t *init, const uint8_t *data,
	    const uint64_t *offsets, const uint32_t *lengths, size_t count,
	    uint64_t stride, uint32_t fixed_len, uint32_t *crcs, uint32_t flags,
	    void *stream);

/* The eight slicing tables (8 x 256) the kernels use for `variant`; table 0
 * is the reference's crc32_tbl256_* of that variant (tests pin it). */
int	lcb_crc32_gpu_tables(int variant, uint32_t *out);

#ifdef __cplusplus
}
#endif

#endif /* LCB_CRC32_GPU_H */
