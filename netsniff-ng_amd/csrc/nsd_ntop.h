// nsd_ntop.h - inet_ntop(AF_INET / AF_INET6) output without libc's sprintf.
//
// The reference prints addresses with inet_ntop (proto_ipv4.c:53-54,
// 189-190, proto_ipv6.c:41-42, 106-107, proto_ipv6_mobility_hdr.c); glibc's inet_ntop
// (resolv/inet_ntop.c, the BIND 4.9.4 code) formats with sprintf, which
// serialises threads: eight formatter threads ran no faster than one.  These
// produce the same text:
//   IPv4: the dotted quad, each byte in decimal;
//   IPv6: eight 16-bit words in lowercase hex without leading zeros, ':'
//         separated; the first longest run of two or more zero words
//         written as "::"; an address whose first 6 words are zero (the run
//         is exactly words 0..5) or whose first 5 are zero and word 5 is
//         0xffff (IPv4-compatible / IPv4-mapped) ends in the dotted quad of
//         its last 4 bytes.
// tests/test_ntop.py pins both against the C library's inet_ntop.
#pragma once
#include <stdint.h>

namespace nsd {

// writes the text and its NUL, returns a pointer to the NUL
static inline char *ntop4_to(const uint8_t *a, char *p)
{
	for (int i = 0; i < 4; i++) {
		if (i)
			*p++ = '.';
		unsigned v = a[i];
		if (v >= 100) {
			*p++ = (char)('0' + v / 100);
			v %= 100;
			*p++ = (char)('0' + v / 10);
			*p++ = (char)('0' + v % 10);
		} else if (v >= 10) {
			*p++ = (char)('0' + v / 10);
			*p++ = (char)('0' + v % 10);
		} else {
			*p++ = (char)('0' + v);
		}
	}
	*p = 0;
	return p;
}

// dst: at least INET6_ADDRSTRLEN (46) bytes
static inline char *ntop6_to(const uint8_t *src, char *p)
{
	static const char hx[] = "0123456789abcdef";
	unsigned w[8];
	for (int i = 0; i < 8; i++)
		w[i] = (unsigned)src[2 * i] << 8 | src[2 * i + 1];
	int best = -1, blen = 0, cur = -1, clen = 0;
	for (int i = 0; i < 8; i++) {
		if (w[i] == 0) {
			if (cur < 0) {
				cur = i;
				clen = 1;
			} else {
				clen++;
			}
		} else if (cur >= 0) {
			if (best < 0 || clen > blen) {
				best = cur;
				blen = clen;
			}
			cur = -1;
		}
	}
	if (cur >= 0 && (best < 0 || clen > blen)) {
		best = cur;
		blen = clen;
	}
	if (best >= 0 && blen < 2)
		best = -1;
	for (int i = 0; i < 8; i++) {
		if (best >= 0 && i >= best && i < best + blen) {
			if (i == best)
				*p++ = ':';
			continue;
		}
		if (i != 0)
			*p++ = ':';
		if (i == 6 && best == 0 && (blen == 6 || (blen == 5 && w[5] == 0xffff)))
			return ntop4_to(src + 12, p);
		const unsigned v = w[i];
		if (v >= 0x1000)
			*p++ = hx[v >> 12];
		if (v >= 0x100)
			*p++ = hx[(v >> 8) & 15];
		if (v >= 0x10)
			*p++ = hx[(v >> 4) & 15];
		*p++ = hx[v & 15];
	}
	if (best >= 0 && best + blen == 8)
		*p++ = ':';
	*p = 0;
	return p;
}

} // namespace nsd
