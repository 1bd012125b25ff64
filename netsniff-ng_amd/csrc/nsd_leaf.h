// nsd_leaf.h - where the leaf parsers whose fields the host renders leave
// the pkt_buff cursor: ARP, DCCP, IGMP, LLDP and the ICMPv6 message bodies
// of types 130-154 (MLD, Neighbor Discovery and its options, Router
// Renumbering, Node Information, MLDv2, Mobile IPv6, SEND, MRD, FMIPv6).
//
// The chain walk (gen_step, nsd_walk.h) runs these on the device and on the
// host CPU, so a record's data_off is the leaf's end - where the exit op's
// dump starts - exactly as each reference parser's pulls leave it (a failed
// pull does not advance, pkt_buff.h:50-64).  Each function follows the
// reference function cited above it; the host text renderers
// (nsd_format_leaves.h, nsd_format_icmpv6.h) print the same pulls and the
// formatter checks the two agree.  S is a byte source with b(o) and
// be16(o); bytes at offsets >= caplen read as zero.
#pragma once
#include <stdint.h>

namespace nsd {

// pkt_buff cursor [data, tail)
struct LCur {
	uint32_t data, tail;
	NSD_HD uint32_t len() const { return tail - data; }
	NSD_HD bool pull(uint32_t n)
	{
		if (n > len())
			return false;
		data += n;
		return true;
	}
	NSD_HD bool pull(uint32_t n, uint32_t &at)
	{
		at = data;
		return pull(n);
	}
	// n one-byte pulls (the %x / %c loops): false once one fails
	NSD_HD bool pull_bytes(int64_t n)
	{
		if (n <= 0)
			return true;
		if ((uint64_t)n <= len()) {
			data += (uint32_t)n;
			return true;
		}
		data = tail;
		return false;
	}
	// print_ipv6_addr_list (proto_icmpv6.c:283-299): nr 16-byte pulls
	NSD_HD bool addrs(uint8_t nr)
	{
		const uint32_t k = len() / 16 < nr ? len() / 16 : nr;
		data += 16 * k;
		return k == nr;
	}
};

// proto_arp.c:80-196: one pull of struct arphdr (28 bytes), both modes
template <class S>
NSD_HD uint32_t leaf_arp(const S &, uint32_t a, uint32_t tail)
{
	return tail - a >= 28 ? a + 28 : a;
}

// proto_dccp.c:70-148
template <class S>
NSD_HD uint32_t leaf_dccp(const S &s, uint32_t h, uint32_t tail, int mode)
{
	if (tail - h < 12)
		return h;
	if (mode != PRINT_NORM)
		return h + 12;
	uint32_t d = h + 12;
	const uint32_t b8 = s.b(h + 8);
	const bool x = b8 & 1;
	const uint32_t type = (b8 >> 1) & 15;
	if (x) {
		if (tail - d < 4)
			return d;
		d += 4;
	}
	if (type >= 1 && type <= 9) {
		const uint32_t need = x ? 8u : 4u;
		if (tail - d < need)
			return d;
		d += need;
	}
	return d;
}

// proto_igmp.c:452-493 picks the dissector (0..3, -1 none); print_less
// pulls nothing (:495-554)
template <class S>
NSD_HD uint32_t leaf_igmp(const S &s, uint32_t m, uint32_t tail, int mode)
{
	if (mode != PRINT_NORM)
		return m;
	const uint32_t t = s.b(m), plen = tail - m;
	uint32_t d;
	switch (t) {
	case 0x01: case 0x02: case 0x03: case 0x04: case 0x05: case 0x06: case 0x07: case 0x08:
		return plen == 20 ? m + 20 : m;   // dissect_igmp_v0
	case 0x12: case 0xFF: case 0xFE: case 0xFD: case 0xFC: case 0x16: case 0x17:
		return plen == 8 ? m + 8 : m;     // v1 / v2
	case 0x11:
		if (plen == 8)
			return m + 8;             // v1 / v2 query
		if (plen < 12)
			return m;
		d = m + 12;                       // v3 query (:334-385)
		{
			const uint32_t n = s.be16(m + 10);
			const uint32_t k = (tail - d) / 4 < n ? (tail - d) / 4 : n;
			return d + 4 * k;
		}
	case 0x22: {                              // v3 report (:387-450)
		if (plen < 8)
			return m;
		d = m + 8;
		uint32_t nrec = s.be16(m + 6);
		while (nrec--) {
			if (tail - d < 8)
				break;
			const uint32_t n = s.be16(d + 2);
			d += 8;
			const uint32_t k = (tail - d) / 4 < n ? (tail - d) / 4 : n;
			d += 4 * k;
		}
		return d;
	}
	}
	return m;
}

// lldp_print_net_addr (proto_lldp.c:88-131): false = -EINVAL
template <class S>
NSD_HD bool lldp_addr_ok(const S &s, uint32_t a, uint32_t alen)
{
	if (alen < 1)
		return false;
	const uint32_t af = s.b(a);
	alen--;
	return af == 1 ? alen >= 4 : af == 2 ? alen >= 16 : af == 6 ? alen >= 6 : true;
}

// lldp (proto_lldp.c:161-455) / lldp_less (:457-488).  Quirk kept: `len`
// only loses the 2-byte TLV headers in print_full
template <class S>
NSD_HD uint32_t leaf_lldp(const S &s, uint32_t d, uint32_t tail, int mode)
{
	uint32_t len = tail - d, n_tlv = 0;
	if (mode != PRINT_NORM) {
		while (len >= 2) {
			const uint32_t hdr = s.be16(d);
			d += 2;
			len -= 2;
			const uint32_t type = hdr >> 9, tlen = hdr & 0x1FF;
			if (type == 0 || tlen == 0 || len < tlen)
				break;
			d += tlen;
			len -= tlen;
		}
		return d;
	}
	while (len >= 2) {
		if (tail - d < 2)
			return d;
		const uint32_t hdr = s.be16(d);
		d += 2;
		len -= 2;
		const uint32_t type = hdr >> 9, tlen = hdr & 0x1FF;
		if (type == 0 && tlen == 0)
			return d;
		if (len < tlen)
			return d;
		switch (type) {
		case 1:
		case 2: {
			if (n_tlv != type - 1 || tlen < 2 || tail - d < tlen)
				return d;
			const uint32_t at = d;
			d += tlen;
			const uint32_t sub = s.b(at);
			if (sub == (type == 1 ? 4u : 3u)) {
				if (tlen < 7)
					return d;
			} else if (sub == (type == 1 ? 5u : 4u)) {
				if (!lldp_addr_ok(s, at + 1, tlen))   // the TLV length, as the reference
					return d;
			}
			break;
		}
		case 3:
			if (n_tlv != 2 || tlen != 2 || tail - d < 2)
				return d;
			d += 2;
			break;
		case 4:
		case 5:
		case 6:
			if (tail - d >= tlen)
				d += tlen;
			break;
		case 7:
			if (tlen != 4 || tail - d < 4)
				return d;
			d += 4;
			break;
		case 8: {
			if (tlen < 9 || tlen > 167 || tail - d < tlen)
				return d;
			uint32_t p = d;
			d += tlen;
			const uint32_t alen = s.b(p);
			p++;
			if (tlen - 1 < alen || !lldp_addr_ok(s, p, alen))
				return d;
			p += alen + 1;
			if (tlen - alen < 4)
				return d;
			p += 4;
			const uint32_t oidlen = s.b(p);
			if (tlen - alen - 4 < 3 || tlen - alen - 4 - 3 < oidlen)
				return d;
			break;
		}
		case 127:
			if (tlen < 4 || tail - d < 4)
				return d;
			d += 4;
			if (tail - d >= tlen - 4)
				d += tlen - 4;
			break;
		default:
			if (tail - d >= tlen)
				d += tlen;
			break;
		}
		n_tlv++;
	}
	return d;
}

// one Neighbor Discovery option body (proto_icmpv6.c:372-806); `len` is the
// option's payload length (ssize_t): each fixed pull, then `len -= sizeof`,
// a negative remainder failing after the pull advanced
template <class S>
NSD_HD bool i6_nd_opt_end(const S &s, LCur &c, uint32_t type, int64_t len)
{
	uint32_t a;
	switch (type) {
	case 1: case 2:
		return c.pull_bytes(len);
	case 3:
		return c.pull(30) && (len -= 30) >= 0;
	case 4:
		if (!c.pull(6) || (len -= 6) < 0)
			return false;
		return c.pull_bytes(len);
	case 5:
		return c.pull(6) && (len -= 6) >= 0;
	case 9: case 10:
		if (!c.pull(6) || (len -= 6) < 0)
			return false;
		return c.addrs((uint8_t)(len / 16));
	case 15: {   // the header's pad_len is a size_t read in host (little-endian) order
		if (!c.pull(9, a) || (len -= 9) < 0)
			return false;
		uint64_t pad = 0;
		for (int k = 7; k >= 0; k--)
			pad = pad << 8 | s.b(a + 1 + k);
		if (pad > (uint64_t)len) {
			c.pull((uint32_t)len);
			return true;
		}
		if (!c.pull_bytes(len - (int64_t)pad))
			return false;
		c.pull_bytes((int64_t)pad);   // a failed padding pull only ends its loop
		return true;
	}
	case 16:
		if (!c.pull(2) || (len -= 2) < 0)
			return false;
		c.pull_bytes(len);
		return true;
	case 17:
		if (!c.pull(2) || (len -= 2) < 0)
			return false;
		if (len == 20)
			return c.pull(20);
		if (len == 16)
			return c.pull(16);
		c.pull_bytes(len);
		return true;
	case 19:
		if (!c.pull(1) || (len -= 1) < 0)
			return false;
		return c.pull_bytes(len);
	}
	c.pull((uint32_t)len);
	return true;
}

// dissect_neighb_disc_ops (proto_icmpv6.c:808-911)
template <class S>
NSD_HD bool i6_nd_ops_end(const S &s, LCur &c)
{
	while (c.len()) {
		uint32_t a;
		if (!c.pull(2, a))
			return false;
		const uint32_t type = s.b(a), l8 = s.b(a + 1);
		const int64_t payl = (int64_t)(uint16_t)(l8 * 8) - 2;
		if (payl > (int64_t)c.len() || payl < 0)
			return false;
		if (!i6_nd_opt_end(s, c, type, payl))
			return false;
	}
	return true;
}

// dissect_icmpv6_mcast_rec (proto_icmpv6.c:310-370)
template <class S>
NSD_HD bool i6_mcast_rec_end(const S &s, LCur &c, uint32_t nr_rec)
{
	while (nr_rec--) {
		uint32_t r;
		if (!c.pull(20, r))
			return false;
		const uint32_t aux_bytes = (uint16_t)(s.b(r + 1) * 4);
		const uint32_t nr_src = s.be16(r + 2);
		if (aux_bytes > c.len() || !c.addrs((uint8_t)nr_src) || aux_bytes > c.len() ||
		    !c.pull_bytes(aux_bytes))
			return false;
	}
	return true;
}

// icmpv6 (proto_icmpv6.c:1667-1688) over a type 130-154 message: the header
// pull, then the body's pulls (:1023-1474)
template <class S>
NSD_HD uint32_t leaf_icmpv6_body(const S &s, uint32_t h, uint32_t tail)
{
	LCur c{ h, tail };
	uint32_t a;
	if (!c.pull(4))
		return h;
	switch (s.b(h)) {
	case 130:
		if (c.pull(20) && c.len() >= 4 && c.pull(4, a))
			c.addrs((uint8_t)s.be16(a + 2));
		break;
	case 131: case 132:
		c.pull(20);
		break;
	case 138: case 139: case 140:
		c.pull(12);
		break;
	case 133: case 141: case 142: case 147: case 148: case 154:
		if (c.pull(4))
			i6_nd_ops_end(s, c);
		break;
	case 134:
		if (c.pull(12))
			i6_nd_ops_end(s, c);
		break;
	case 135: case 136:
		if (c.pull(20))
			i6_nd_ops_end(s, c);
		break;
	case 137:
		if (c.pull(36))
			i6_nd_ops_end(s, c);
		break;
	case 143:
		if (c.pull(4, a))
			i6_mcast_rec_end(s, c, s.be16(a + 2));
		break;
	case 144: case 146: case 150: case 151:
		c.pull(4);
		break;
	case 145:
		if (c.pull(4))
			c.addrs((uint8_t)(c.len() / 16));
		break;
	case 149:
		if (c.pull(8))
			i6_nd_ops_end(s, c);
		break;
	}
	return c.data;
}

// the leaf end of ops `id` run at `start` (ids without pulls: start)
template <int MODE, class S>
NSD_HD uint32_t leaf_end(const S &s, int id, uint32_t start, uint32_t tail)
{
	switch (id) {
	case NSD_OPS_ARP:
		return leaf_arp(s, start, tail);
	case NSD_OPS_LLDP:
		return leaf_lldp(s, start, tail, MODE);
	case NSD_OPS_IGMP:
		return leaf_igmp(s, start, tail, MODE);
	case NSD_OPS_DCCP:
		return leaf_dccp(s, start, tail, MODE);
	case NSD_OPS_ICMPV6:
		return MODE == PRINT_NORM ? leaf_icmpv6_body(s, start, tail) : start;
	}
	return start;
}

} // namespace nsd
