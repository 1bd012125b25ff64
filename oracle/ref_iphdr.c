/*
 * ref_iphdr.c - the parts of the reference's IPv4 / IPv6 layers that compile
 * as they lie, exported for the parity tests.  TEST INFRASTRUCTURE ONLY
 * (built by oracle/Makefile "ref" into oracle/_ref/libnsdrefip.so).
 *
 * proto_ipv4.c / proto_ipv6.c themselves include geoip.h -> config.h (which
 * this image cannot generate), but what they compute with comes from three
 * headers that include only system headers and built_in.h, compiled here
 * from /root/reference:
 *   csum.h:12-39  csum / calc_csum (the IPv4 header checksum of
 *                 proto_ipv4.c:51 and the ICMPv4 checksum of
 *                 proto_icmpv4.c:42) and csum_expected (the "should be"
 *                 value, proto_ipv4.c:86-88);
 *   ipv4.h:8-27   struct ipv4hdr: the bitfield / field layout the IPv4 line
 *                 prints from (proto_ipv4.c:49-50, 69-84);
 *   ipv6.h:14-30  struct ipv6hdr (proto_ipv6.c:36-52).
 * The few expressions proto_ipv4.c / proto_ipv6.c apply to those fields
 * (the FRAG_OFF_* masks, proto_ipv4.c:26-29; the traffic class / flow
 * label of proto_ipv6.c:36-39) are restated below, marked as such.
 */
#include <stdint.h>
#include <string.h>

#include "csum.h"
#include "ipv4.h"
#include "ipv6.h"

/* calc_csum(buf, len) over a copy (csum reads u16 words through a cast) */
uint16_t nsref_calc_csum(const uint8_t *buf, size_t len)
{
	uint16_t tmp[32768 + 1];

	if (len > sizeof(tmp))
		return 0;
	memset(tmp, 0, sizeof(tmp));
	memcpy(tmp, buf, len);
	return calc_csum(tmp, len);
}

uint16_t nsref_csum_expected(uint16_t sum, uint16_t computed)
{
	return csum_expected(sum, computed);
}

/* proto_ipv4.c:49-51, 69-88 over struct ipv4hdr at hdr (60 readable bytes,
 * zero past the capture): out[] = {version, ihl, tos, tot_len (ntohs), id
 * (ntohs), res, nofrag, morefrag, fragoff, ttl, protocol, check (ntohs),
 * csum = calc_csum(ip, ihl * 4), should_be = csum_expected(h_check, csum),
 * saddr, daddr (as stored)} */
void nsref_ipv4_fields(const uint8_t *hdr, uint32_t *out)
{
	uint8_t buf[64];
	struct ipv4hdr ip;
	uint16_t frag_off, csum;

	memcpy(buf, hdr, 60);
	memset(buf + 60, 0, 4);
	memcpy(&ip, buf, sizeof(ip));
	frag_off = ntohs(ip.h_frag_off);
	csum = nsref_calc_csum(buf, ip.h_ihl * 4);
	out[0] = ip.h_version;
	out[1] = ip.h_ihl;
	out[2] = ip.h_tos;
	out[3] = ntohs(ip.h_tot_len);
	out[4] = ntohs(ip.h_id);
	/* FRAG_OFF_* (proto_ipv4.c:26-29, restated) */
	out[5] = (frag_off & 0x8000) ? 1 : 0;
	out[6] = (frag_off & 0x4000) ? 1 : 0;
	out[7] = (frag_off & 0x2000) ? 1 : 0;
	out[8] = frag_off & 0x1fff;
	out[9] = ip.h_ttl;
	out[10] = ip.h_protocol;
	out[11] = ntohs(ip.h_check);
	out[12] = csum;
	out[13] = csum_expected(ip.h_check, csum);
	out[14] = ip.h_saddr;
	out[15] = ip.h_daddr;
}

/* proto_ipv6.c:36-52 over struct ipv6hdr: out[] = {version, traffic class,
 * flow label (the reference's expressions, restated: its flow label ORs
 * overlapping shifts), payload_len (ntohs), nexthdr, hop_limit} */
void nsref_ipv6_fields(const uint8_t *hdr, uint32_t *out)
{
	struct ipv6hdr ip;

	memcpy(&ip, hdr, sizeof(ip));
	out[0] = ip.version;
	out[1] = (uint8_t)((ip.priority << 4) | ((ip.flow_lbl[0] & 0xF0) >> 4));
	out[2] = ((ip.flow_lbl[0] & 0x0F) << 8) | (ip.flow_lbl[1] << 4) | ip.flow_lbl[2];
	out[3] = ntohs(ip.payload_len);
	out[4] = ip.nexthdr;
	out[5] = ip.hop_limit;
}
