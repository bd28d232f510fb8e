/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Thin C wrapper that compiles the REFERENCE's RADIUS packet code
 * (/root/reference/include/proto/radius.h, by path, nothing copied) into
 * oracle/_ref/libref_radius.so.  tests/golden/make_golden_radius.py drives it
 * to produce the RADIUS fixtures (tests/golden/radius.json) that pin the keyed
 * batch modes of the GPU library (lcb_hash_batch_keyed) against the
 * reference's own radius_pkt_sign / radius_pkt_verify /
 * radius_pkt_authenticator_calc / radius_pkt_attr_msg_authenticator_calc.
 *
 * Built with the CMake HAVE_* probes glibc needs (SURVEY.md 8(c) caveat 3).
 * Compiled a second time against THIS repo's drop-in include/crypto/hash/md5.h
 * (include order: ours first) by tests/test_dropin_headers.py, so the same
 * packets can be signed by both builds and compared byte for byte.
 */
#include <sys/param.h>
#include <sys/types.h>
#include <errno.h>
#include <inttypes.h>
#include <stdio.h>
#include <string.h>

#include "proto/radius.h"

/* Attribute TLVs: blob of (type, len, data[len]) records, len = data bytes. */
static int
add_attrs(rad_pkt_hdr_p pkt, size_t buf_size, const uint8_t *tlv, size_t tlv_len) {
	size_t i = 0;
	int error;

	while (i + 2 <= tlv_len) {
		uint8_t type = tlv[i], len = tlv[i + 1];
		if (i + 2 + len > tlv_len)
			return (EINVAL);
		error = radius_pkt_attr_add(pkt, buf_size, NULL, type, len,
		    (uint8_t*)(tlv + i + 2), NULL);
		if (0 != error)
			return (error);
		i += 2 + (size_t)len;
	}
	return (0);
}

/*
 * A request (code Access-Request, Accounting-Request, ...; id; the random
 * authenticator of an Access-Request) with a User-Password (pwd != NULL) and
 * the attribute TLVs, optionally a Message-Authenticator, signed by
 * radius_pkt_sign (radius.h:1487).  pre: the packet as built, before signing.
 * Returns 0 or the reference's error code.
 */
int
ref_rad_request(uint8_t code, uint8_t id, const uint8_t *auth16, const uint8_t *pwd, size_t pwd_len,
    const uint8_t *tlv, size_t tlv_len, const uint8_t *key, size_t key_len, int add_msg_authr,
    uint8_t *pre, size_t *pre_len, uint8_t *out, size_t *out_len) {
	uint8_t buf[RADIUS_PKT_MAX_SIZE];
	rad_pkt_hdr_p pkt = (rad_pkt_hdr_p)buf;
	size_t sz = 0;
	int error;

	memset(buf, 0, sizeof(buf));
	error = radius_pkt_init(pkt, sizeof(buf), NULL, code, id, (uint8_t*)auth16);
	if (0 != error)
		return (error);
	if (NULL != pwd) {
		/* radius_pkt_attr_add(User-Password) cannot succeed in the
		 * reference: its size probe (radius.h:1052-1055) calls
		 * radius_pkt_attr_password_encode with buf_size 0, which returns
		 * EOVERFLOW (:762-763) for every length.  Lay the attribute out as
		 * it intends (:1056-1063) with the reference's own allocator. */
		rad_pkt_attr_p attr = NULL;
		size_t tm = (0 != pwd_len) ? ((pwd_len + (MD5_HASH_SIZE - 1)) & ~((size_t)(MD5_HASH_SIZE - 1))) :
		    MD5_HASH_SIZE;
		if (RADIUS_A_T_USER_PASSWORD_MAX_LEN < pwd_len)
			return (EINVAL);
		error = radius_pkt_attr_alloc_raw(pkt, sizeof(buf), NULL, RADIUS_ATTR_TYPE_USER_PASSWORD,
		    (uint8_t)tm, &attr, NULL);
		if (0 != error)
			return (error);
		memcpy(RADIUS_PKT_ATTR_DATA(attr), pwd, pwd_len);
		memset((RADIUS_PKT_ATTR_DATA(attr) + pwd_len), 0x00, (tm - pwd_len));
	}
	error = add_attrs(pkt, sizeof(buf), tlv, tlv_len);
	if (0 != error)
		return (error);
	if (add_msg_authr) {
		error = radius_pkt_attr_add(pkt, sizeof(buf), NULL, RADIUS_ATTR_TYPE_MSG_AUTHENTIC, 0,
		    NULL, NULL);
		if (0 != error)
			return (error);
	}
	*pre_len = RADIUS_PKT_HDR_LEN_GET(pkt);
	memcpy(pre, buf, *pre_len);
	error = radius_pkt_sign(pkt, sizeof(buf), &sz, (uint8_t*)key, key_len, 0);
	if (0 != error)
		return (error);
	*out_len = RADIUS_PKT_HDR_LEN_GET(pkt);
	memcpy(out, buf, *out_len);
	return (0);
}

/* A reply to `req` (radius_pkt_reply_init, radius.h:1472), attributes,
 * optional Message-Authenticator, signed by radius_pkt_sign. */
int
ref_rad_reply(uint8_t code, const uint8_t *req, const uint8_t *tlv, size_t tlv_len,
    const uint8_t *key, size_t key_len, int add_msg_authr,
    uint8_t *pre, size_t *pre_len, uint8_t *out, size_t *out_len) {
	uint8_t buf[RADIUS_PKT_MAX_SIZE];
	rad_pkt_hdr_p pkt = (rad_pkt_hdr_p)buf;
	size_t sz = 0;
	int error;

	memset(buf, 0, sizeof(buf));
	error = radius_pkt_reply_init(pkt, sizeof(buf), NULL, code, (rad_pkt_hdr_p)req);
	if (0 != error)
		return (error);
	error = add_attrs(pkt, sizeof(buf), tlv, tlv_len);
	if (0 != error)
		return (error);
	if (add_msg_authr) {
		error = radius_pkt_attr_add(pkt, sizeof(buf), NULL, RADIUS_ATTR_TYPE_MSG_AUTHENTIC, 0,
		    NULL, NULL);
		if (0 != error)
			return (error);
	}
	*pre_len = RADIUS_PKT_HDR_LEN_GET(pkt);
	memcpy(pre, buf, *pre_len);
	error = radius_pkt_sign(pkt, sizeof(buf), &sz, (uint8_t*)key, key_len, 0);
	if (0 != error)
		return (error);
	*out_len = RADIUS_PKT_HDR_LEN_GET(pkt);
	memcpy(out, buf, *out_len);
	return (0);
}

/* radius_pkt_sign (radius.h:1487, add_msg_authr = 0) of a copy of an
 * already built packet `pkt_in`; `out` receives the signed packet. */
int
ref_rad_sign(const uint8_t *pkt_in, size_t len, const uint8_t *key, size_t key_len, uint8_t *out,
    size_t *out_len) {
	uint8_t buf[RADIUS_PKT_MAX_SIZE];
	rad_pkt_hdr_p pkt = (rad_pkt_hdr_p)buf;
	size_t sz = 0;
	int error;

	if (len > sizeof(buf))
		return (EINVAL);
	memset(buf, 0, sizeof(buf));
	memcpy(buf, pkt_in, len);
	error = radius_pkt_sign(pkt, sizeof(buf), &sz, (uint8_t*)key, key_len, 0);
	if (0 != error)
		return (error);
	*out_len = RADIUS_PKT_HDR_LEN_GET(pkt);
	memcpy(out, buf, *out_len);
	return (0);
}

/* radius_pkt_chk + radius_pkt_verify (radius.h:1535) of a copy of `pkt`
 * (req may be NULL); `out` receives the packet after verification (User-
 * Password decoded in place).  Returns the reference's result. */
int
ref_rad_verify(const uint8_t *pkt_in, size_t len, const uint8_t *key, size_t key_len,
    const uint8_t *req, uint8_t *out) {
	uint8_t buf[RADIUS_PKT_MAX_SIZE];
	int error;

	if (len > sizeof(buf))
		return (EINVAL);
	memcpy(buf, pkt_in, len);
	error = radius_pkt_chk((rad_pkt_hdr_p)buf, len);
	if (0 != error)
		return (error);
	error = radius_pkt_verify((rad_pkt_hdr_p)buf, (uint8_t*)key, key_len, (rad_pkt_hdr_p)req);
	memcpy(out, buf, len);
	return (error);
}

/* radius_pkt_authenticator_calc (radius.h:1315) on a copy of `pkt`. */
int
ref_rad_authenticator_calc(const uint8_t *pkt_in, size_t len, const uint8_t *key, size_t key_len,
    int inside, const uint8_t *req, uint8_t *out16) {
	uint8_t buf[RADIUS_PKT_MAX_SIZE];

	if (len > sizeof(buf))
		return (EINVAL);
	memcpy(buf, pkt_in, len);
	return (radius_pkt_authenticator_calc((rad_pkt_hdr_p)buf, (uint8_t*)key, key_len, inside,
	    (rad_pkt_hdr_p)req, out16));
}

/* radius_pkt_attr_msg_authenticator_calc (radius.h:850) for the packet's
 * Message-Authenticator attribute, on a copy of `pkt`. */
int
ref_rad_msg_authenticator_calc(const uint8_t *pkt_in, size_t len, const uint8_t *key, size_t key_len,
    int inside, const uint8_t *req, uint8_t *out16) {
	uint8_t buf[RADIUS_PKT_MAX_SIZE];
	rad_pkt_attr_p attr = NULL;
	int error;

	if (len > sizeof(buf))
		return (EINVAL);
	memcpy(buf, pkt_in, len);
	error = radius_pkt_attr_find_raw((rad_pkt_hdr_p)buf, 0, RADIUS_ATTR_TYPE_MSG_AUTHENTIC, &attr, NULL);
	if (0 != error)
		return (error);
	return (radius_pkt_attr_msg_authenticator_calc((rad_pkt_hdr_p)buf, attr, (uint8_t*)key, key_len,
	    inside, (rad_pkt_hdr_p)req, out16));
}

/* radius_pkt_attr_password_encode / _decode (radius.h:745, 795). */
int
ref_rad_password_encode(const uint8_t *auth16, const uint8_t *pwd, size_t pwd_len, const uint8_t *key,
    size_t key_len, uint8_t *out, size_t out_size, size_t *out_len) {
	return (radius_pkt_attr_password_encode((uint8_t*)auth16, (uint8_t*)pwd, pwd_len, (uint8_t*)key,
	    key_len, out, out_size, out_len));
}

int
ref_rad_password_decode(const uint8_t *auth16, const uint8_t *enc, size_t enc_len, const uint8_t *key,
    size_t key_len, uint8_t *out, size_t out_size, size_t *out_len) {
	return (radius_pkt_attr_password_decode((uint8_t*)auth16, (uint8_t*)enc, enc_len, (uint8_t*)key,
	    key_len, out, out_size, out_len));
}
