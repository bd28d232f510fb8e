/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see lcb_oracle.h).
 *
 * Plain C restatement of rozhuk-im/liblcb include/math/crc32.h: the eight
 * CRC-32 variants defined there (crc32.h:501-576) over the two register
 * update rules crc32_normal8 (MSB first, crc32.h:61-73) and crc32_reflect8
 * (LSB first, crc32.h:101-113).  The reference switches to its 4-bit tables
 * below 64 bytes (crc32.h:42, 75-83, 115-123); that is the same function
 * (the 4-bit steps compose to the 8-bit table), so one byte-wise rule is
 * restated here.  The byte tables are derived from the polynomial by the
 * bit-serial definition, not copied; tests/test_crc32.py pins them against
 * the reference's tables and KATs (crc32.h:581-657) compiled from
 * /root/reference into oracle/_ref.
 */
#include <string.h>
#include "lcb_oracle.h"

/* One variant of crc32.h:501-576: polynomial, bit order, and whether the
 * macro wraps the register in ~ on the way in and out. */
typedef struct crc_variant_s {
	uint32_t poly;		/* normal (MSB-first) form */
	int reflect;		/* crc32_reflect vs crc32_normal */
	int inv;		/* X_update(c) = ~rule(~c) (1) or rule(c) (0) */
	uint32_t oneshot_c;	/* the c that X(data, size) passes to X_update */
} crc_variant_t;

static const crc_variant_t crc_var[9] = {
	{ 0, 0, 0, 0 },
	{ 0x04c11db7u, 0, 1, 0x00000000u },	/* crc32a  BZIP2   crc32.h:505-508 */
	{ 0x04c11db7u, 0, 1, 0xffffffffu },	/* cksum   CKSUM   crc32.h:514-517 */
	{ 0x04c11db7u, 0, 0, 0xffffffffu },	/* mpeg2   MPEG-2  crc32.h:522-525 */
	{ 0x04c11db7u, 1, 1, 0x00000000u },	/* crc32b  ISO-HDLC crc32.h:532-535 */
	{ 0x04c11db7u, 1, 0, 0xffffffffu },	/* jamcrc  JAMCRC  crc32.h:541-544 */
	{ 0x1edc6f41u, 1, 1, 0x00000000u },	/* crc32c  ISCSI   crc32.h:551-554 */
	{ 0xa833982bu, 1, 1, 0x00000000u },	/* crc32d  BASE91-D crc32.h:561-564 */
	{ 0x814141abu, 0, 0, 0x00000000u },	/* crc32q  AIXM    crc32.h:571-574 */
};

static uint32_t bitrev32(uint32_t x) {
	uint32_t r = 0;
	for (int i = 0; i < 32; i++)
		if (x >> i & 1u)
			r |= 1u << (31 - i);
	return r;
}

/* Byte table by the bit-serial definition of each rule. */
static void crc_table(int v, uint32_t t[256]) {
	const crc_variant_t *cv = &crc_var[v];
	const uint32_t rp = bitrev32(cv->poly);
	for (uint32_t i = 0; i < 256; i++) {
		uint32_t c;
		if (cv->reflect) {
			c = i;
			for (int k = 0; k < 8; k++)
				c = (c & 1u) ? (c >> 1) ^ rp : c >> 1;
		} else {
			c = i << 24;
			for (int k = 0; k < 8; k++)
				c = (c & 0x80000000u) ? (c << 1) ^ cv->poly : c << 1;
		}
		t[i] = c;
	}
}

static uint32_t g_tab[9][256];
static int g_tab_ready[9];

static const uint32_t *tab(int v) {
	if (!g_tab_ready[v]) {	/* benign race: every writer stores the same values */
		crc_table(v, g_tab[v]);
		g_tab_ready[v] = 1;
	}
	return g_tab[v];
}

int or_crc32_valid(int variant) { return variant >= OR_CRC32A && variant <= OR_CRC32Q; }

uint32_t or_crc32_table(int variant, int i) {
	return or_crc32_valid(variant) ? tab(variant)[i & 255] : 0;
}

/* X_update(crc, d, n) of crc32.h for variant X. */
uint32_t or_crc32_update(int variant, uint32_t crc, const uint8_t *d, size_t n) {
	if (!or_crc32_valid(variant))
		return 0;
	const crc_variant_t *cv = &crc_var[variant];
	const uint32_t *t = tab(variant);
	uint32_t r = cv->inv ? ~crc : crc;
	if (cv->reflect) {	/* crc32.h:109-111 */
		for (size_t i = 0; i < n; i++)
			r = (r >> 8) ^ t[(r ^ d[i]) & 0xffu];
	} else {		/* crc32.h:69-71 */
		for (size_t i = 0; i < n; i++)
			r = (r << 8) ^ t[((r >> 24) ^ d[i]) & 0xffu];
	}
	return cv->inv ? ~r : r;
}

/* X(d, n) of crc32.h. */
uint32_t or_crc32(int variant, const uint8_t *d, size_t n) {
	if (!or_crc32_valid(variant))
		return 0;
	return or_crc32_update(variant, crc_var[variant].oneshot_c, d, n);
}

int or_crc32_batch(int variant, const uint32_t *init, const uint8_t *base,
    const uint64_t *offsets, const uint32_t *lengths, size_t count,
    uint64_t stride, uint32_t fixed_len, uint32_t *crcs) {
	if (!or_crc32_valid(variant))
		return -1;
	for (size_t i = 0; i < count; i++) {
		const uint8_t *m = base + (offsets ? offsets[i] : (uint64_t)i * stride);
		const size_t n = lengths ? lengths[i] : fixed_len;
		crcs[i] = init ? or_crc32_update(variant, init[i], m, n) : or_crc32(variant, m, n);
	}
	return 0;
}
