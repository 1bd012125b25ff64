// nsd_format_icmpv6.h - host renderer of the ICMPv6 message bodies with a
// variable length (types 130-154: MLD, Neighbor Discovery and its options,
// Router Renumbering, Node Information, MLDv2 reports, Mobile IPv6, SEND,
// Multicast Router Discovery, FMIPv6).  Included by nsd_format.cpp after the
// leaf renderers.
//
// The device classifies these messages and stops the chain at the ICMPv6
// header with the cursor at its start (NSD_F_HOST, PRINT_NORM only); this
// file runs icmpv6() (proto_icmpv6.c:1667-1688) from there, header pull and
// body parsers included, and returns where the cursor ended: the exit op's
// dump starts there.  Every function follows the reference function cited
// above it, pull for pull (a failed pull does not advance, pkt_buff.h:50-64);
// bytes at offsets >= caplen read as zero (parity domain).

// pkt_buff cursor (pkt_buff.h:15-64)
struct Cur {
	const Frame &f;
	uint32_t data, tail;
	uint32_t len() const { return tail - data; }
	// pkt_pull: `n` is the reference's unsigned int argument
	bool pull(uint32_t n, uint32_t &at)
	{
		if (n > len())
			return false;
		at = data;
		data += n;
		return true;
	}
	bool pull(uint32_t n)
	{
		uint32_t at;
		return pull(n, at);
	}
};

static void i6_addr(Out &o, const Frame &f, uint32_t off)
{
	char b[INET6_ADDRSTRLEN];
	ntop6(f, off, b);
	o << b;
}

static const char I6_INVALID_OPEN[] = "\033[30;41mINVALID\033[0m";

// print_ipv6_addr_list (proto_icmpv6.c:283-299); nr_addr is a uint8_t
static bool i6_addr_list(Out &o, Cur &c, uint8_t nr)
{
	while (nr--) {
		uint32_t a;
		if (!c.pull(16, a))
			return false;
		o << "\n\t   Address: ";
		i6_addr(o, c.f, a);
	}
	return true;
}

// the body bytes printed "%x" one by one, each pulled (the loops of
// proto_icmpv6.c:387-398 and the like); false if a pull fails
static bool i6_hex_bytes(Out &o, Cur &c, int64_t n)
{
	while (n-- > 0) {
		uint32_t a;
		if (!c.pull(1, a)) {
			o << I6_INVALID_OPEN;
			return false;
		}
		o.x(c.f.b(a));
	}
	return true;
}

// dissect_icmpv6_mcast_rec (proto_icmpv6.c:310-370)
static const char *const i6_mcast_rec_types[] = {
	"MODE_IS_INCLUDE", "MODE_IS_EXCLUDE", "CHANGE_TO_INCLUDE_MODE",
	"CHANGE_TO_EXCLUDE_MODE", "ALLOW_NEW_SOURCES", "BLOCK_OLD_SOURCES",
};

static bool i6_mcast_rec(Out &o, Cur &c, uint16_t nr_rec)
{
	while (nr_rec--) {
		uint32_t r;
		if (!c.pull(20, r))
			return false;
		const uint8_t type = c.f.b(r), aux = c.f.b(r + 1);
		const uint16_t aux_bytes = (uint16_t)(aux * 4);
		const uint16_t nr_src = c.f.be16(r + 2);
		const size_t ti = (size_t)((int)type - 1);
		o << ", Rec Type " << (ti < 6 ? i6_mcast_rec_types[ti] : "Unknown") << " (";
		o.u(type) << ")";
		if (aux_bytes > c.len()) {
			o << ", Aux Data Len (";
			o.u(aux) << ", ";
			o.u(aux_bytes) << " bytes) " << C_RED << "invalid" << C_END;
			return false;
		}
		o << ", Aux Data Len (";
		o.u(aux) << ", ";
		o.u(aux_bytes) << " bytes)";
		o << ", Nr. of Sources (";
		o.u(nr_src) << ")";
		o << ", Address: ";
		i6_addr(o, c.f, r + 4);
		if (!i6_addr_list(o, c, (uint8_t)nr_src))
			return false;
		if (aux_bytes > c.len()) {
			o << "\nAux Data Len " << C_RED << "invalid" << C_END;
			return false;
		}
		o << ", Aux Data: ";
		if (!i6_hex_bytes(o, c, aux_bytes))
			return false;
	}
	return true;
}

// ---- Neighbor Discovery options (proto_icmpv6.c:372-911) ---------------------
static const char *const i6_nd15_names[] = { "DER Encoded X.501 Name", "FQDN" };
static const char *const i6_nd17_codes[] = {
	"Old Care-of Address", "New Care-of Address", "NAR's IP address", "NAR's Prefix",
};
// the reference's literals continue lines with a backslash, keeping the next
// line's indentation inside the string (proto_icmpv6.c:712-725)
static const char *const i6_nd19_codes[] = {
	"Wildcard requesting resolution for all nearby access points",
	"Link-Layer Address of the New Access Point",
	"Link-Layer Address of the MN",
	"Link-Layer Address of the NAR",
	"Link-Layer Address of the source of RtSolPr or PrRtAdv          message",
	"The access point identified by the LLA belongs to the          current interface of the router",
	"No prefix information available for the access point          identified by the LLA",
	"No fast handover support available for the access point          identified by the LLA",
};

// icmpv6_neighb_disc_ops (proto_icmpv6.c:764-806)
static const char *i6_nd_name(uint8_t t)
{
	switch (t) {
	case 1: return "Source Link-Layer Address";
	case 2: return "Target Link-Layer Address";
	case 3: case 23: return "Prefix Information";
	case 4: case 24: return "Redirected Header";
	case 5: case 25: return "MTU";
	case 6: case 26: return "NBMA Shortcut Limit Option";
	case 7: case 27: return "Advertisement Interval Option";
	case 8: case 28: return "Home Agent Information Option";
	case 9: case 29: return "Source Address List";
	case 10: case 30: return "Target Address List";
	case 11: return "CGA option";
	case 12: return "RSA Signature option";
	case 13: return "Timestamp option";
	case 14: return "Nonce option";
	case 15: return "Trust Anchor option";
	case 16: return "Certificate option";
	case 17: return "IP Address/Prefix Option";
	case 18: return "New Router Prefix Information Option";
	case 19: return "Link-layer Address Option";
	case 20: return "Neighbor Advertisement Acknowledgment Option";
	case 31: return "DNS Search List Option";
	case 32: return "Proxy Signature (PS)";
	case 138: return "CARD Request option";
	case 139: return "CARD Reply option";
	case 253: return "RFC3692-style Experiment 1";
	case 254: return "RFC3692-style Experiment 2";
	}
	return nullptr;
}

// one option body; `len` = the option's payload length (ssize_t in the
// reference).  Each starts with its fixed pull, then `len -= sizeof` and a
// negative remainder fails after the pull already advanced.
static bool i6_nd_opt(Out &o, Cur &c, uint8_t type, int64_t len)
{
	uint32_t a;
	switch (type) {
	case 1: case 2:   // dissect_neighb_disc_ops_1/_2 (:372-406)
		o << "Address 0x";
		return i6_hex_bytes(o, c, len);
	case 3:           // :408-437
		if (!c.pull(30, a) || (len -= 30) < 0)
			return false;
		{
			const uint8_t la = c.f.b(a + 1);
			o << "Prefix Len (";
			o.u(c.f.b(a)) << ") ";
			o << "L (";
			o.u(la >> 7) << ") A (";
			o.u((la >> 7) & 1) << ") Res1 (0x";
			o.x(la & 0x3F) << ") ";
			o << "Valid Lifetime (";
			o.u(c.f.be32(a + 2)) << "s) ";
			o << "Preferred Lifetime (";
			o.u(c.f.be32(a + 6)) << "s) ";
			o << "Reserved2 (0x";
			o.x(c.f.be32(a + 10)) << ") ";
			o << "Prefix: ";
			i6_addr(o, c.f, a + 14);
			o << " ";
		}
		return true;
	case 4:           // :439-469
		if (!c.pull(6, a) || (len -= 6) < 0)
			return false;
		o << "Reserved 1 (0x";
		o.x(c.f.be16(a)) << ") ";
		o << "Reserved 2 (0x";
		o.x(c.f.be32(a + 2)) << ") ";
		o << "IP header + data ";
		return i6_hex_bytes(o, c, len);
	case 5:           // :471-488
		if (!c.pull(6, a) || (len -= 6) < 0)
			return false;
		o << "Reserved (0x";
		o.x(c.f.be16(a)) << ") ";
		o << "MTU (";
		o.u(c.f.be32(a + 2)) << ")";
		return true;
	case 9: case 10:  // :490-513
		if (!c.pull(6, a) || (len -= 6) < 0)
			return false;
		o << "Reserved 1 (0x";
		o.x(c.f.be16(a)) << ") ";
		o << "Reserved 2 (0x";
		o.x(c.f.be32(a + 2)) << ") ";
		return i6_addr_list(o, c, (uint8_t)(len / 16));
	case 15: {        // :520-584; the header's pad_len is a size_t (9-byte packed struct)
		if (!c.pull(9, a) || (len -= 9) < 0)
			return false;
		const uint8_t nt = c.f.b(a);
		uint64_t pad = 0;
		for (int k = 7; k >= 0; k--)
			pad = pad << 8 | c.f.b(a + 1 + k);   // host (little-endian) order
		const size_t ni = (size_t)((int)nt - 1);
		o << "Name Type " << (ni < 2 ? i6_nd15_names[ni] : "Unknown") << " (";
		o.u(nt) << ") ";
		if (pad > (uint64_t)len) {
			o << "Pad Len (";
			o.u(pad) << ", invalid)\n" << C_RED << "Skip Option" << C_END;
			c.pull((uint32_t)len);
			return true;
		}
		o << "Pad Len (";
		o.u(pad) << ") ";
		int64_t name_len = len - (int64_t)pad;
		o << "Name (";
		while (name_len--) {
			if (!c.pull(1, a)) {
				o << I6_INVALID_OPEN;
				return false;
			}
			o.c((char)c.f.b(a));
		}
		o << ") ";
		o << "Padding (";
		while (pad--) {
			if (!c.pull(1, a)) {
				o << I6_INVALID_OPEN;
				break;
			}
			o.x(c.f.b(a));
		}
		o << ")";
		return true;
	}
	case 16: {        // :590-626
		if (!c.pull(2, a) || (len -= 2) < 0)
			return false;
		const uint8_t ct = c.f.b(a);
		o << "Cert Type " << ((size_t)((int)ct - 1) < 1 ? "X.509v3 Certificate" : "Unknown") << " (";
		o.u(ct) << ") ";
		o << "Res (0x";
		o.x(c.f.b(a + 1)) << ") ";
		o << "Certificate + Padding (";
		i6_hex_bytes(o, c, len);   // a failed pull breaks the loop, the option still succeeds
		o << ") ";
		return true;
	}
	case 17: {        // :635-710
		if (!c.pull(2, a) || (len -= 2) < 0)
			return false;
		const uint8_t oc = c.f.b(a);
		const size_t oi = (size_t)((int)oc - 1);
		o << "Opt Code " << (oi < 4 ? i6_nd17_codes[oi] : "Unknown") << " (";
		o.u(oc) << ") ";
		o << "Prefix Len (";
		o.u(c.f.b(a + 1)) << ") ";
		if (len == 20) {
			if (!c.pull(20, a))
				return false;
			o << "Res (0x";
			o.x(c.f.le32(a)) << ") ";   // printed without ntohl
			o << "Addr: ";
			i6_addr(o, c.f, a + 4);
			o << " ";
		} else if (len == 16) {
			if (!c.pull(16, a))
				return false;
			o << "Addr: ";
			i6_addr(o, c.f, a);
			o << " ";
		} else {
			o << C_RED << "Error Wrong Length. Skip Option" << C_END << " (";
			i6_hex_bytes(o, c, len);
			o << ") ";
		}
		return true;
	}
	case 19: {        // :727-762
		if (!c.pull(1, a) || (len -= 1) < 0)
			return false;
		const uint8_t oc = c.f.b(a);
		o << "Opt Code " << (oc < 8 ? i6_nd19_codes[oc] : "Unknown") << " (";
		o.u(oc) << ") ";
		o << "LLA (";
		if (!i6_hex_bytes(o, c, len))
			return false;
		o << ") ";
		return true;
	}
	default:
		c.pull((uint32_t)len);
		return true;
	}
}

// dissect_neighb_disc_ops (proto_icmpv6.c:808-911)
static bool i6_nd_ops(Out &o, Cur &c)
{
	while (c.len()) {
		uint32_t a;
		if (!c.pull(2, a))
			return false;
		const uint8_t type = c.f.b(a), l8 = c.f.b(a + 1);
		const uint16_t total = (uint16_t)(l8 * 8);
		const int64_t payl = (int64_t)total - 2;   // pad_bytes = total % 8 = 0
		const char *nm = i6_nd_name(type);
		o << "\n\tOption " << (nm ? nm : "Type Unknown") << " (";
		o.u(type) << ") ";
		if (payl > (int64_t)c.len() || payl < 0) {
			o << "Length (";
			o.u(l8) << ", ";
			o.u(total) << " bytes, " << C_RED << "invalid" << C_END << ") ";
			return false;
		}
		o << "Length (";
		o.u(l8) << ", ";
		o.u(total) << " bytes) ";
		if (!i6_nd_opt(o, c, type, payl))
			return false;
	}
	return true;
}

// ---- message bodies (proto_icmpv6.c:1023-1474) ---------------------------------
static bool i6_body(Out &o, Cur &c, uint8_t type)
{
	const Frame &f = c.f;
	uint32_t a;
	switch (type) {
	case 130: {   // :1023-1070
		if (!c.pull(20, a))
			return false;
		const uint16_t mrd = f.be16(a);
		const bool v2 = c.len() >= 4;
		if (v2) {
			o << ", MLDv2, Max Resp Delay (";
			o.u(mrd >> 15 ? (uint32_t)(((mrd & 0xFFF) | 0x1000) << (((mrd >> 12) & 0x3) + 3)) : mrd) << "ms)";
		} else {
			o << ", Max Resp Delay (";
			o.u(mrd) << "ms)";
		}
		o << ", Res (0x";
		o.x(f.be16(a + 2)) << ")";
		o << ", Address: ";
		i6_addr(o, f, a + 4);
		if (v2) {
			if (!c.pull(4, a))
				return false;
			const uint8_t sq = f.b(a);
			const uint16_t nr = f.be16(a + 2);
			o << ", Resv (0x";
			o.x(sq >> 4) << ")";
			o << ", S (";
			o.u((sq >> 3) & 1) << ")";
			o << ", QRV (0x";
			o.x(sq & 3) << ")";
			o << ", QQIC (";
			o.u(f.b(a + 1)) << ")";
			o << ", Nr Src (";
			o.u(nr) << ")";
			return i6_addr_list(o, c, (uint8_t)nr);
		}
		return true;
	}
	case 131: case 132:   // :1072-1094
		if (!c.pull(20, a))
			return false;
		o << ", Max Resp Delay (";
		o.u(f.be16(a)) << "ms)";
		o << ", Res (0x";
		o.x(f.be16(a + 2)) << ")";
		o << ", Address: ";
		i6_addr(o, f, a + 4);
		return true;
	case 133: case 141: case 142:   // :1096-1108, 1292-1300
		if (!c.pull(4, a))
			return false;
		o << ", Reserved (0x";
		o.x(f.be32(a)) << ")";
		return i6_nd_ops(o, c);
	case 134: {   // :1110-1127
		if (!c.pull(12, a))
			return false;
		const uint8_t mo = f.b(a + 1);
		o << ", Cur Hop Limit (";
		o.u(f.b(a)) << ")";
		o << ", M (";
		o.u(mo >> 7) << ") O (";
		o.u((mo >> 6) & 1) << ")";
		o << ", Router Lifetime (";
		o.u(f.be16(a + 2)) << "s)";
		o << ", Reachable Time (";
		o.u(f.be32(a + 4)) << "ms)";
		o << ", Retrans Timer (";
		o.u(f.be32(a + 8)) << "ms)";
		return i6_nd_ops(o, c);
	}
	case 135:   // :1129-1145
		if (!c.pull(20, a))
			return false;
		o << ", Reserved (0x";
		o.x(f.be32(a)) << ")";
		o << ", Target Address: ";
		i6_addr(o, f, a + 4);
		return i6_nd_ops(o, c);
	case 136: {   // :1147-1167
		if (!c.pull(20, a))
			return false;
		const uint32_t r = f.be32(a);
		o << ", R (";
		o.u(r >> 31) << ") S (";
		o.u((r >> 30) & 1) << ") O (";
		o.u((r >> 29) & 1) << ") Reserved (0x";
		o.x(r & 0x1FFFFFFF) << ")";
		o << ", Target Address: ";
		i6_addr(o, f, a + 4);
		return i6_nd_ops(o, c);
	}
	case 137:   // :1169-1188 (Reserved printed without ntohl)
		if (!c.pull(36, a))
			return false;
		o << ", Reserved (0x";
		o.x(f.le32(a)) << ")";
		o << ", Target Address: ";
		i6_addr(o, f, a + 4);
		o << ", Dest Address: ";
		i6_addr(o, f, a + 20);
		return i6_nd_ops(o, c);
	case 138: {   // :1210-1231 (+ dissect_icmpv6_rr_body :1190-1198)
		if (!c.pull(12, a))
			return false;
		const uint8_t fl = f.b(a + 5);
		o << ", Sequence Nr. (";
		o.u(f.be32(a)) << ")";
		o << ", Segment Nr. (";
		o.u(f.b(a + 4)) << ")";
		o << ", T (";
		o.u(fl >> 7) << ") R (";
		o.u((fl >> 6) & 1) << ") A (";
		o.u((fl >> 5) & 1) << ") S (";
		o.u((fl >> 4) & 1) << ") P (";
		o.u((fl >> 3) & 1) << ") Res \t\t(0x";   // a continued string literal
		o.x(fl & 7) << ") ";
		o << ", Max Delay (";
		o.u(f.be16(a + 6)) << "ms)";
		o << ", Res (0x";
		o.x(f.be32(a + 8)) << ")";
		if (c.len())
			o << " Message Body recognized";
		return true;
	}
	case 139: case 140: {   // :1257-1279 (+ dissect_icmpv6_node_inf_data :1233-1241)
		static const char *const qtypes[] = { "NOOP", "unused", "Node Name", "Node Addresses",
						      "IPv4 Addresses " };
		if (!c.pull(12, a))
			return false;
		const uint16_t qt = f.be16(a);
		o << ", Qtype " << (qt < 5 ? qtypes[qt] : "Unknown") << " (";
		o.u(qt) << ")";
		o << ", Flags (0x";
		o.x(f.be16(a + 2)) << ")";
		o << ", Nonce (0x";
		o.x(f.be64(a + 4)) << ")";
		if (c.len())
			o << " Data recognized";
		return true;
	}
	case 143: {   // :1302-1317
		if (!c.pull(4, a))
			return false;
		const uint16_t nr = f.be16(a + 2);
		o << ", Res (0x";
		o.x(f.be16(a)) << ")";
		o << ", Nr. Mcast Addr Records (";
		o.u(nr) << ")";
		return i6_mcast_rec(o, c, nr);
	}
	case 144: case 146:   // :1319-1332, 1350-1353
		if (!c.pull(4, a))
			return false;
		o << ", ID (";
		o.u(f.be16(a)) << ")";
		o << ", Res (0x";
		o.x(f.be16(a + 2)) << ")";
		return true;
	case 145:   // :1334-1348
		if (!c.pull(4, a))
			return false;
		o << ", ID (";
		o.u(f.be16(a)) << ")";
		o << ", Res (0x";
		o.x(f.be16(a + 2)) << ")";
		return i6_addr_list(o, c, (uint8_t)(c.len() / 16));
	case 147: {   // :1355-1371
		if (!c.pull(4, a))
			return false;
		const uint16_t m = f.be16(a + 2);
		o << ", ID (";
		o.u(f.be16(a)) << ")";
		o << ", M (";
		o.u(m >> 15) << ") O (";
		o.u((m >> 14) & 1) << ") Res (0x";
		o.x(m & 0x3FFF) << ")";
		return i6_nd_ops(o, c);
	}
	case 148:   // :1373-1386
		if (!c.pull(4, a))
			return false;
		o << ", ID (";
		o.u(f.be16(a)) << ")";
		o << ", Component (";
		o.u(f.be16(a + 2)) << ")";
		return i6_nd_ops(o, c);
	case 149:   // :1388-1403
		if (!c.pull(8, a))
			return false;
		o << ", ID (";
		o.u(f.be16(a)) << ")";
		o << ", All Components (";
		o.u(f.be16(a + 2)) << ")";
		o << ", Component (";
		o.u(f.be16(a + 4)) << ")";
		o << ", Res (0x";
		o.x(f.be16(a + 6)) << ")";
		return i6_nd_ops(o, c);
	case 150:   // :1405-1419: little-endian bitfields over the raw u32
		if (!c.pull(4, a))
			return false;
		o << ", Subtype (";
		o.u(f.b(a + 3)) << ")";
		o << ", Res (0x";
		o.x(f.le32(a) & 0xFFFFFF) << ")";
		o << ", Options in Payload";
		return true;
	case 151:   // :1421-1434
		if (!c.pull(4, a))
			return false;
		o << ", Query Interval (";
		o.u(f.be16(a)) << "s)";
		o << ", Robustness Variable  (";
		o.u(f.be16(a + 2)) << ")";
		return true;
	case 152: case 153:   // :1436-1458: empty structs
		return true;
	case 154:   // :1460-1474
		if (!c.pull(4, a))
			return false;
		o << ", Subtype (";
		o.u(f.b(a)) << ")";
		o << ", Res (0x";
		o.x(f.b(a + 1)) << ")";
		o << ", ID (";
		o.u(f.be16(a + 2)) << ")";
		return i6_nd_ops(o, c);
	}
	return true;
}

// icmpv6_process names for types 130-154 (proto_icmpv6.c:1538-1649)
static void i6_names_130(uint8_t t, uint8_t code, const char *&ts, const char *&cs)
{
	static const char *const c139[] = { "Data contains IPv6 Address", "Data contains Name or nothing",
					    "Data contains IPv4 Address" };
	static const char *const c140[] = { "Successful reply", "Responder refuses answer",
					    "Qtype is unknown to the Responder" };
	cs = "Unknown Code";
	switch (t) {
	case 130: ts = "Multicast Listener Query"; break;
	case 131: ts = "Multicast Listener Report"; break;
	case 132: ts = "Multicast Listener Done"; break;
	case 133: ts = "Router Solicitation"; break;
	case 134: ts = "Router Advertisement"; break;
	case 135: ts = "Neighbor Solicitation"; break;
	case 136: ts = "Neighbor Advertisement"; break;
	case 137: ts = "Redirect Message"; break;
	case 138:
		ts = "Router Renumbering";
		if (code == 1) cs = "Router Renumbering Command";
		else if (code == 2) cs = "Router Renumbering Result";
		else if (code == 255) cs = "Sequence Number Reset";
		break;
	case 139: ts = "ICMP Node Information Query"; if (code < 3) cs = c139[code]; break;
	case 140: ts = "ICMP Node Information Response"; if (code < 3) cs = c140[code]; break;
	case 141: ts = "Inverse Neighbor Discovery Solicitation Message"; break;
	case 142: ts = "Inverse Neighbor Discovery Advertisement Message"; break;
	case 143: ts = "Multicast Listener Report v2"; break;
	case 144: ts = "Home Agent Address Discovery Request Message"; break;
	case 145: ts = "Home Agent Address Discovery Reply Message"; break;
	case 146: ts = "Mobile Prefix Solicitation"; break;
	case 147: ts = "Mobile Prefix Advertisement"; break;
	case 148: ts = "Certification Path Solicitation"; break;
	case 149: ts = "Certification Path Advertisement"; break;
	case 150: ts = "ICMP messages utilized by experimental mobility protocols such as Seamoby"; break;
	case 151: ts = "Multicast Router Advertisement"; cs = "Ad. Interval"; break;
	case 152: ts = "Multicast Router Solicitation"; cs = "Reserved"; break;
	case 153: ts = "Multicast Router Termination"; cs = "Reserved"; break;
	default: ts = "FMIPv6 Messages"; break;   // 154
	}
}

// icmpv6 (proto_icmpv6.c:1667-1688) for a type 130-154 message, from the
// header the device left the cursor at
static Done r_icmpv6_host(Out &o, const Frame &f, const Layer &L)
{
	Cur c{ f, L.start, L.tail };
	uint32_t h;
	if (!c.pull(4, h))
		return { L.start, L.tail, false, true };
	const uint8_t type = f.b(h), code = f.b(h + 1);
	const char *ts, *cs;
	i6_names_130(type, code, ts, cs);
	o << " [ ICMPv6 " << ts << " (";
	o.u(type) << "), " << cs << " (";
	o.u(code) << "), Chks (0x";
	o.x(f.be16(h + 2)) << ")";
	if (!i6_body(o, c, type))
		o << "\n" << C_RED << "Failed to dissect Message" << C_END;
	o << " ]\n";
	return { c.data, c.tail, false, true };
}
