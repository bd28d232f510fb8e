/*
 * lcb_chacha_gpu.h — batched ChaCha / XChaCha on the MI355X
 * (liblcb_hash_gpu.so), SURVEY.md §8(f) row 4.
 *
 * The reference's cipher (include/crypto/cipher/chacha.h) is header-only and
 * one buffer per call; its one-shot forms are
 *
 *   chacha(key, key_size, counter, iv, rounds, src, bytes, dst)   chacha.h:662-674
 *   xchacha(key, key_size, counter, iv, rounds, src, bytes, dst)  chacha.h:681-693
 *
 * Each entry point here computes, for every buffer i, exactly the bytes the
 * reference writes for
 *
 *   chacha(key, key_size,
 *          counters ? counters + 8*i : NULL,        (8-byte LE block counter)
 *          ivs ? ivs + IVL*i : NULL,                (IVL = 8, or 24 for xchacha)
 *          rounds,
 *          src ? src + off_i : NULL,                (NULL: the keystream itself)
 *          len_i,
 *          dst + off_i)
 *
 * with off_i = offsets ? offsets[i] : i * stride and
 * len_i = lengths ? lengths[i] : fixed_len.  One key per batch (host memory,
 * 32 bytes read when key_size is 256 or 32, else 16 bytes used as a 128-bit
 * key: chacha.h:286-316); any `rounds` value behaves as the reference's
 * `for (i = 0; i < rounds; i += 2)` double-round loop (chacha.h:432-434).
 * Block j of buffer i uses counter + j with a 64-bit carry
 * (chacha.h:440-444).  src may equal dst (in place).  Bytes of dst outside
 * the described buffers are never written; buffers must not overlap.
 *
 * Memory modes (flags): LCB_HASH_F_DEVICE (include/lcb_hash_gpu.h) — src,
 * dst, offsets, lengths, counters and ivs are device pointers, counters and
 * ivs 4-byte aligned, the work is enqueued on `stream` without waiting;
 * 0 — host pointers, staged through page-locked memory, returns when dst is
 * written.  Errors: 0, EINVAL, ENOMEM, ENODEV, EIO (no CPU fallback).
 */
#ifndef LCB_CHACHA_GPU_H
#define LCB_CHACHA_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* xchacha == 0: chacha(); != 0: xchacha() (24-byte ivs). */
int	lcb_chacha_batch(int xchacha, const uint8_t *key, size_t key_size,
	    const uint8_t *counters, const uint8_t *ivs, size_t rounds,
	    const uint8_t *src, uint8_t *dst, const uint64_t *offsets,
	    const uint32_t *lengths, size_t count, uint64_t stride,
	    uint32_t fixed_len, uint32_t flags, void *stream);

/* Reference-named entry points (chacha.h:662, chacha.h:681), batched. */
int	chacha_batch(const uint8_t *key, size_t key_size,
	    const uint8_t *counters, const uint8_t *ivs, size_t rounds,
	    const uint8_t *src, uint8_t *dst, const uint64_t *offsets,
	    const uint32_t *lengths, size_t count, uint64_t stride,
	    uint32_t fixed_len, uint32_t flags, void *stream);
int	xchacha_batch(const uint8_t *key, size_t key_size,
	    const uint8_t *counters, const uint8_t *ivs, size_t rounds,
	    const uint8_t *src, uint8_t *dst, const uint64_t *offsets,
	    const uint32_t *lengths, size_t count, uint64_t stride,
	    uint32_t fixed_len, uint32_t flags, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* LCB_CHACHA_GPU_H */
