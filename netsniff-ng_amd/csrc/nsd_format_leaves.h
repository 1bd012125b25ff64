// nsd_format_leaves.h - host renderers of the leaf parsers the device only
// classifies (records flagged NSD_F_HOST): ARP, LLDP, IGMP, DCCP.  Included
// by nsd_format.cpp after its Out / Frame / Layer / Done helpers.
//
// The device stops such a chain at the leaf with the cursor at the leaf's
// start; the renderer runs the leaf's print function from there (pulls
// included) and returns where the cursor ended, which is where the exit op's
// dump starts.  Each function follows the reference parser cited above it;
// bytes at offsets >= caplen read as zero (parity domain).

// calc_csum (csum.h:12-27): ~fold(sum of len >> 1 little-endian u16 words)
static uint16_t leaf_csum(const Frame &f, uint64_t off, uint64_t len)
{
	uint64_t sum = 0;
	for (uint64_t w = 0; w < (len >> 1); w++)
		sum += f.le16(off + 2 * w);
	sum = (sum >> 16) + (sum & 0xffff);
	sum += (sum >> 16);
	return (uint16_t)~sum;
}

// tputs_safe / tputchar_safe (tprintf.c:164-180)
static void tputs_safe(Out &o, const Frame &f, uint64_t off, uint64_t len)
{
	for (uint64_t i = 0; i < len; i++) {
		const uint8_t c = f.b(off + i);
		if (c >= 0x20 && c < 0x7f) {
			o.c((char)c);
		} else {
			o << "\\0x";
			o.xn(c, 2);
		}
	}
}

static void ip4(Out &o, const Frame &f, uint64_t off)
{
	quad(o, f, off);
}

// ---- ARP (proto_arp.c:52-196) -------------------------------------------------
static const char *arp_opcode(uint16_t op)
{
	switch (op) {
	case 1: return "ARP request";
	case 2: return "ARP reply";
	case 3: return "RARP request";
	case 4: return "RARP reply";
	case 8: return "InARP request";
	case 9: return "InARP reply";
	case 10: return "(ATM) ARP NAK";
	}
	return "Unknown";
}

static Done r_arp(Out &o, const Frame &f, const Layer &L, int mode)
{
	if (L.tail - L.start < 28)
		return { L.start, L.tail, false, true };
	const uint32_t a = L.start;
	const uint16_t hrd = f.be16(a), pro = f.be16(a + 2), op = f.be16(a + 6);
	if (mode != PRINT_NORM) {
		o << " Op " << arp_opcode(op);
		return { a + 28, L.tail, false, true };
	}
	const char *hn;
	switch (hrd) {
	case 1: hn = "Ethernet"; break;
	case 6: hn = "IEEE 802"; break;
	case 7: hn = "ARCNET"; break;
	case 16: case 19: case 21: hn = "ATM"; break;
	case 20: hn = "Serial Line"; break;
	case 24: hn = "IEEE 1394.1995"; break;
	default: hn = "Unknown";
	}
	const char *pn = lookup_ether_type(pro);
	o << " [ ARP Format HA (";
	o.u(hrd) << " => " << hn << "), Format Proto (0x";
	o.xn(pro, 4) << " => " << (pn ? pn : "Unknown") << "), HA Len (";
	o.u(f.b(a + 4)) << "), Proto Len (";
	o.u(f.b(a + 5)) << "), Opcode (";
	o.u(op) << " => " << arp_opcode(op) << ")";
	for (int t = 0; t < 2; t++) {   // arp_print_addrs: sender, then target
		const char *dir = t ? "Target" : "Sender";
		if (hrd == 1) {
			o << ", " << dir << " MAC (";
			mac(o, f, a + (t ? 18 : 8));
			o << ")";
		}
		if (pro == 0x0800) {
			o << ", " << dir << " IP (";
			ip4(o, f, a + (t ? 24 : 14));
			o << ")";
		}
	}
	o << " ]\n";
	return { a + 28, L.tail, false, true };
}

// ---- DCCP (proto_dccp.c:53-148) -----------------------------------------------
static const char *dccp_type(uint32_t t)
{
	static const char *const names[] = { "Request", "Response", "Data", "Ack", "DataAck",
					     "CloseReq", "Close", "Reset", "Sync", "SyncAck" };
	return t < 10 ? names[t] : "Reserved";   // 10..15 (the type is 4 bits)
}

static Done r_dccp(Out &o, const Frame &f, const Layer &L, int mode)
{
	const uint32_t h = L.start;
	if (L.tail - h < 12)
		return { h, L.tail, false, true };
	const uint16_t sp = f.be16(h), dp = f.be16(h + 2);
	if (mode != PRINT_NORM) {
		o << " DCCP ";
		o.u(sp) << "/";
		o.u(dp);
		return { h + 12, L.tail, false, true };
	}
	uint32_t d = h + 12;
	// little-endian bitfields of byte 8: x (bit 0), type (bits 1..4); sqnr is
	// the 24-bit field of bytes 9..11 passed through ntohl
	const uint8_t b8 = f.b(h + 8);
	const bool x = b8 & 1;
	const uint32_t type = (b8 >> 1) & 15;
	uint64_t seq = (uint32_t)f.b(h + 9) << 24 | (uint32_t)f.b(h + 10) << 16 | (uint32_t)f.b(h + 11) << 8;
	if (x) {
		if (L.tail - d < 4)
			return { d, L.tail, false, true };
		seq = seq << 24 | f.be32(d);
		d += 4;
	}
	int64_t ack = -1;
	if (type >= 1 && type <= 9) {
		if (x) {
			if (L.tail - d < 8)
				return { d, L.tail, false, true };
			ack = (int64_t)((uint64_t)f.be16(d + 2) << 32 | f.be32(d + 4));
			d += 8;
		} else {
			if (L.tail - d < 4)
				return { d, L.tail, false, true };
			ack = (int64_t)((uint32_t)f.b(d + 1) << 24 | (uint32_t)f.b(d + 2) << 16 |
					(uint32_t)f.b(d + 3) << 8);
			d += 4;
		}
	}
	o << " [ DCCP Port (";
	o.u(sp) << " => ";
	o.u(dp) << "), Header Len (";
	o.u((uint32_t)f.b(h + 4) * 4) << " Bytes), Type: " << dccp_type(type) << ", Seqnr:";
	o.u(seq);
	if (ack > 0) {
		o << ", AckNr:";
		o.u((uint64_t)ack);
	}
	o << " ]\n";
	return { d, L.tail, false, true };
}

// ---- IGMP (proto_igmp.c:137-554) ----------------------------------------------
static const char *igmp_type_name(uint8_t t)
{
	switch (t) {
	case 0x01: return "Create Group Request";
	case 0x02: return "Create Group Reply";
	case 0x03: return "Join Group Request";
	case 0x04: return "Join Group Reply";
	case 0x05: return "Leave Group Request";
	case 0x06: return "Leave Group Reply";
	case 0x07: return "Confirm Group Request";
	case 0x08: return "Confirm Group Reply";
	case 0x11: return "Membership Query";
	case 0x12: case 0x16: case 0x22: return "Membership Report";
	case 0x17: return "Leave Group";
	case 0xFF: return "Hello";
	case 0xFE: return "Bye";
	case 0xFD: return "Join Group";
	case 0xFC: return "Leave Group";
	}
	return nullptr;
}

static void igmp_type(Out &o, uint8_t t)   // PRINT_FRIENDLY_NAMED_MSG_TYPE
{
	const char *nm = igmp_type_name(t);
	o << "  Type (0x";
	o.xn(t, 2);
	if (nm)
		o << ", " << nm;
	o << ")";
}

static const char *igmp_group_rec_name(uint8_t t)
{
	static const char *const names[] = { "Mode Is Include", "Mode Is Exclude", "Change To Include Mode",
					     "Change To Exclude Mode", "Allow New Sources", "Block Old Sources" };
	return t >= 1 && t <= 6 ? names[t - 1] : nullptr;
}

// ", CSum (0x..) is ok|bogus" over [m, m + len)
static void igmp_csum(Out &o, const Frame &f, uint32_t m, uint32_t len)
{
	const uint16_t cs = leaf_csum(f, m, len);
	o << ", CSum (0x";
	o.xn(f.be16(m + 2), 4) << ") is ";
	if (cs) {
		o << C_RED << "bogus (!)" << C_END << " - " << C_RED << " should be ";   // " - %s should be %x%s"
		o.x(csum_expected(f.le16(m + 2), cs)) << C_END;
	} else {
		o << "ok";
	}
}

static uint32_t igmp_decode_code(uint8_t x)   // DECODE_MAX_RESP_CODE / DECODE_QQIC
{
	return x < 128 ? x : ((uint32_t)(x & 0x0F) | 0x10) << (((x & 0x70) >> 4) + 3);
}

// ", Src Addr (a, b, ...)" over n sources pulled one by one
static void igmp_sources(Out &o, const Frame &f, uint32_t &d, uint32_t tail, uint32_t n)
{
	if (!n--)
		return;
	if (tail - d < 4)
		return;
	o << ", Src Addr (";
	ip4(o, f, d);
	d += 4;
	while (n--) {
		if (tail - d < 4)
			break;
		o << ", ";
		ip4(o, f, d);
		d += 4;
	}
	o << ")";
}

// which dissector igmp() picks (proto_igmp.c:452-493): 0..3, or -1 for none
static int igmp_version(const Frame &f, const Layer &L)
{
	const uint8_t t = f.b(L.start);
	const uint32_t plen = L.tail - L.start;
	switch (t) {
	case 0x01: case 0x02: case 0x03: case 0x04: case 0x05: case 0x06: case 0x07: case 0x08:
		return plen == 20 ? 0 : -1;
	case 0x11:
		if (plen >= 12)
			return 3;
		if (plen == 8 && f.b(L.start + 1))
			return 2;
		return plen == 8 ? 1 : -1;
	case 0x12:
		return plen == 8 ? 1 : -1;
	case 0xFF: case 0xFE: case 0xFD: case 0xFC: case 0x16: case 0x17:
		return plen == 8 ? 2 : -1;
	case 0x22:
		return plen >= 8 ? 3 : -1;
	}
	return -1;
}

static Done r_igmp(Out &o, const Frame &f, const Layer &L, int mode)
{
	const uint32_t m = L.start, tail = L.tail;
	const uint8_t t = f.b(m);
	const int ver = igmp_version(f, L);
	const bool rgmp = t >= 0xFC;
	if (mode != PRINT_NORM) {
		// igmp_less (proto_igmp.c:495-554): no pull
		if (ver < 0)
			return { m, tail, false, true };
		if (rgmp) {
			o << " IGMPv2 (RGMP)";
		} else {
			o << " IGMPv";
			o.u((uint32_t)ver);
		}
		igmp_type(o, t);
		return { m, tail, false, true };
	}
	if (ver < 0)
		return { m, tail, false, true };
	const uint8_t code = f.b(m + 1);
	uint32_t d;
	if (ver == 0) {   // dissect_igmp_v0 (:212-272)
		static const char *const reply[] = { "Request Granted", "Request Denied, No Resources",
						     "Request Denied, Invalid Code",
						     "Request Denied, Invalid Group Address",
						     "Request Denied, Invalid Access Key" };
		const bool is_reply = t == 0x02 || t == 0x04 || t == 0x06 || t == 0x08;
		d = m + 20;
		o << " [ IGMPv0";
		igmp_type(o, t);
		o << ", Code (";
		o.u(code);
		if (t == 0x01 && code <= 1) {
			o << ", " << (code ? "Private" : "Public");
		} else if (is_reply && code < 5) {
			o << ", " << reply[code];
		} else if (is_reply) {
			o << ", Request Pending, Retry In ";
			o.u(code) << " Seconds";
		}
		o << ")";
		igmp_csum(o, f, m, 20 + (tail - d));
		o << ", Id (";
		o.u(f.be16(m + 4)) << "), Group Addr (";   // ntohs of the u32 identifier's low half
		ip4(o, f, m + 8);
		o << "), Access Key (0x";
		o.xn((uint64_t)f.le32(m + 12) | (uint64_t)f.le32(m + 16) << 32, 16) << ") ]\n";
		return { d, tail, false, true };
	}
	if (ver == 1) {   // dissect_igmp_v1 (:274-296)
		d = m + 8;
		o << " [ IGMPv1";
		igmp_type(o, t);
		igmp_csum(o, f, m, 8 + (tail - d));
		o << ", Group Addr (";
		ip4(o, f, m + 4);
		o << ") ]\n";
		return { d, tail, false, true };
	}
	if (ver == 2) {   // dissect_igmp_v2 (:298-332)
		d = m + 8;
		o << (rgmp ? " [ IGMPv2 (RGMP)" : " [ IGMPv2");
		igmp_type(o, t);
		o << ", Max Resp Time (";
		o.u(code) << ")";
		igmp_csum(o, f, m, 8 + (tail - d));
		o << ", Group Addr (";
		ip4(o, f, m + 4);
		o << ") ]\n";
		return { d, tail, false, true };
	}
	if (t == 0x11) {   // dissect_igmp_v3_membership_query (:334-385)
		d = m + 12;
		const uint8_t b8 = f.b(m + 8), qqic = f.b(m + 9);
		const uint32_t n = f.be16(m + 10);
		o << " [ IGMPv3";
		igmp_type(o, t);
		o << ", Max Resp Code (0x";
		o.xn(code, 2) << " => ";
		o.u(igmp_decode_code(code)) << ")";
		igmp_csum(o, f, m, 12 + (tail - d));
		o << ", Suppress (";
		o.u((b8 >> 3) & 1) << "), QRV (";
		o.u(b8 & 7) << "), QQIC (0x";
		o.xn(qqic, 2) << " => ";
		o.u(igmp_decode_code(qqic)) << "), Group Addr (";
		ip4(o, f, m + 4);
		o << "), Num Src (";
		o.u(n) << ")";
		igmp_sources(o, f, d, tail, n);
		o << " ]\n";
		return { d, tail, false, true };
	}
	// dissect_igmp_v3_membership_report (:387-450)
	d = m + 8;
	uint32_t nrec = f.be16(m + 6);
	o << " [ IGMPv3";
	igmp_type(o, t);
	igmp_csum(o, f, m, 8 + (tail - d));
	o << ", Num Group Rec (";
	o.u(nrec) << ") ]\n";
	while (nrec--) {
		if (tail - d < 8)
			break;
		const uint32_t r = d;
		d += 8;
		const uint8_t rt = f.b(r);
		const char *rn = igmp_group_rec_name(rt);
		const uint32_t n = f.be16(r + 2);
		o << "   [ Group Record  Type (";
		o.u(rt);
		if (rn)
			o << ", " << rn;
		o << "), Num Src (";
		o.u(n) << "), Multicast Addr (";
		ip4(o, f, r + 4);
		o << ")";
		igmp_sources(o, f, d, tail, n);
		o << " ]\n";
	}
	o << "\n";
	return { d, tail, false, true };
}

// ---- LLDP (proto_lldp.c:88-488) -----------------------------------------------
// lldp_print_net_addr (:88-131); false = -EINVAL
static bool lldp_net_addr(Out &o, const Frame &f, uint64_t a, uint64_t alen)
{
	if (alen < 1)
		return false;
	const uint8_t af = f.b(a);
	a++;
	alen--;
	switch (af) {
	case 1:
		if (alen < 4)
			return false;
		ip4(o, f, a);
		break;
	case 2: {
		if (alen < 16)
			return false;
		char b[INET6_ADDRSTRLEN];
		ntop6(f, a, b);
		o << b;
		break;
	}
	case 6:
		if (alen < 6)
			return false;
		mac(o, f, (uint32_t)a);
		break;
	default:
		o << "unknown address family";
	}
	return true;
}

static void lldp_caps(Out &o, uint16_t cap)   // lldp_print_cap (:133-159)
{
	static const char *const names[] = { "Other", "Repeater", "Bridge", "WLAN AP", "Router", "Telephone",
					     "DOCSIS", "Station only" };
	bool prev = false;
	for (int i = 0; i < 8; i++) {
		if (!((cap >> i) & 1))
			continue;
		if (prev)
			o << ", ";
		o << names[i];
		prev = true;
	}
}

static Done r_lldp(Out &o, const Frame &f, const Layer &L, int mode)
{
	uint32_t d = L.start;
	const uint32_t tail = L.tail;
	uint32_t len = tail - d;
	uint32_t n_tlv = 0;
	if (mode != PRINT_NORM) {
		// lldp_less (:457-488): len follows pkt_len exactly, so its pulls succeed
		while (len >= 2) {
			const uint16_t hdr = f.be16(d);
			d += 2;
			const uint32_t type = hdr >> 9, tlen = hdr & 0x1FF;
			n_tlv++;
			len -= 2;
			if (type == 0 || tlen == 0)
				break;
			if (len < tlen)
				break;
			d += tlen;
			len -= tlen;
		}
		o << " ";
		o.u(n_tlv) << " TLV" << (n_tlv == 1 ? "" : "s");
		return { d, tail, false, true };
	}
	// lldp (:161-455).  Quirk kept: `len` only loses the 2-byte TLV headers,
	// so once the TLVs are used up the next header pull fails -> INVALID
	if (len == 0)
		return { d, tail, false, true };
	o << " [ LLDP ";
	auto invalid = [&]() -> Done {
		o << " " << C_RED << "INVALID" << C_END << " ]\n";
		return { d, tail, false, true };
	};
	while (len >= 2) {
		if (tail - d < 2)
			return invalid();
		const uint16_t hdr = f.be16(d);
		d += 2;
		const uint32_t type = hdr >> 9, tlen = hdr & 0x1FF;
		len -= 2;
		if (type == 0 && tlen == 0) {
			if (n_tlv < 3)
				return invalid();
			break;
		}
		if (len < tlen)
			return invalid();
		switch (type) {
		case 1:     // Chassis ID
		case 2: {   // Port ID
			if (n_tlv != type - 1)
				return invalid();
			o << (type == 1 ? "Chassis ID" : ", Port ID");
			if (tlen < 2)
				return invalid();
			if (tail - d < tlen)
				return invalid();
			const uint32_t s = d;
			d += tlen;
			const uint8_t sub = f.b(s);
			o << " (Subtype ";
			o.u(sub) << " => ";
			const uint8_t mac_sub = type == 1 ? 4 : 3, net_sub = type == 1 ? 5 : 4;
			const bool str = type == 1 ? (sub == 1 || sub == 2 || sub == 3 || sub == 6 || sub == 7)
						   : (sub == 1 || sub == 2 || sub == 5 || sub == 6 || sub == 7);
			if (sub == mac_sub) {
				if (tlen < 7)
					return invalid();
				mac(o, f, s + 1);
			} else if (sub == net_sub) {
				if (!lldp_net_addr(o, f, s + 1, tlen))   // the TLV length, as the reference
					return invalid();
			} else if (str) {
				tputs_safe(o, f, s + 1, tlen - 1);
			} else {
				o << "Reserved";
			}
			o << ")";
			break;
		}
		case 3:     // TTL
			if (n_tlv != 2)
				return invalid();
			o << ", TTL";
			if (tlen != 2)
				return invalid();
			if (tail - d < 2)
				return invalid();
			o << " (";
			o.u(f.be16(d)) << ")";
			d += 2;
			break;
		case 4:
		case 5:
		case 6:
			o << (type == 4 ? ", Port desc (" : type == 5 ? ", Sys name (" : ", Sys desc (");
			if (tail - d < tlen) {
				o << "none";
			} else {
				tputs_safe(o, f, d, tlen);
				d += tlen;
			}
			o << ")";
			break;
		case 7:
			o << ", Sys Cap";
			if (tlen != 4)
				return invalid();
			if (tail - d < 4)
				return invalid();
			o << " (";
			lldp_caps(o, f.be16(d));
			o << ") Ena Cap (";
			lldp_caps(o, f.be16(d + 2));
			o << ")";
			d += 4;
			break;
		case 8: {   // Management address
			o << ", Mgmt Addr (";
			if (tlen < 9 || tlen > 167)
				return invalid();
			if (tail - d < tlen)
				return invalid();
			uint32_t p = d;
			d += tlen;
			const uint32_t alen = f.b(p);
			p++;
			if (tlen - 1 < alen)
				return invalid();
			if (!lldp_net_addr(o, f, p, alen))
				return invalid();
			p += alen;
			const uint8_t ist = f.b(p);
			o << ", Iface Subtype ";
			o.u(ist) << "/" << (ist == 2 ? "ifIndex" : ist == 3 ? "System Port Number" : "Unknown");
			p++;
			if (tlen - alen < 4)
				return invalid();
			o << ", Iface Number ";
			o.u(f.be32(p));
			p += 4;
			const uint32_t oidlen = f.b(p);
			if (tlen - alen - 4 < 3 || tlen - alen - 4 - 3 < oidlen)
				return invalid();
			if (oidlen > 0) {
				o << ", OID ";
				tputs_safe(o, f, p + 1, oidlen);
			}
			o << ")";
			break;
		}
		case 127: {   // Organizationally specific
			o << ", Org specific";
			if (tlen < 4)
				return invalid();
			if (tail - d < 4)
				return invalid();
			const uint32_t v = f.be32(d);
			d += 4;
			const char *vn = lookup_vendor(v >> 8);
			o << " (OUI " << (vn ? vn : "Unknown") << ", Subtype ";
			o.u(v & 0xff) << ")";
			if (tail - d >= tlen - 4)   // "eat it up"; a failed pull does not advance
				d += tlen - 4;
			break;
		}
		default:
			o << ", Unknown TLV ";
			o.u(type);
			if (tail - d >= tlen)
				d += tlen;
			break;
		}
		n_tlv++;
	}
	o << " ]\n";
	return { d, tail, false, true };
}
