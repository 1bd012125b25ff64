// nsd_format.cpp - host formatter: renders a device chain record + the raw
// frame bytes into the exact text the reference dissector chain hands to
// tprintf for that packet ("printed records out").
//
// The device decides the chain (which ops ran, where each layer starts, the
// final cursor, the checksums); this file only renders each layer's fields,
// following the print functions of the reference parsers (cited per layer).
// It also re-derives each layer's end from the bytes and checks it against
// the next layer's recorded start, so a record that disagrees with the bytes
// is reported (NSD_ERR_FORMAT) instead of rendered wrong.
//
// No printf on this path: fields are appended with small integer formatters.
#include <arpa/inet.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/netsniff_dissect.h"
#include "nsd_lookup.h"
#include "nsd_ntop.h"

// as dissector.h:29 declares it (net/if.h and linux/if.h do not mix)
extern "C" char *if_indextoname(unsigned ifindex, char *ifname);

namespace nsd {

static const char C_BOLD[] = "\033[1m";
static const char C_RED[] = "\033[30;41m";
static const char C_END[] = "\033[0m";

// The text sink: appends go to a small buffer on the stack and reach the
// string a few KiB at a time (std::string::append per field costs a call and
// a capacity check; a packet is ~80 fields).  One Out per string at a time:
// its destructor flushes, so the string is complete when the entry returns.
struct Out {
	std::string &s;
	char *w;
	char buf[4096];
	explicit Out(std::string &str) : s(str), w(buf) {}
	Out(const Out &) = delete;
	Out &operator=(const Out &) = delete;
	~Out() { flush(); }
	void flush()
	{
		if (w != buf)
			s.append(buf, (size_t)(w - buf));
		w = buf;
	}
	// the text so far, and dropping what came after `mark` of it
	size_t size() const { return s.size() + (size_t)(w - buf); }
	void cut(size_t mark)
	{
		flush();
		s.resize(mark);
	}
	// room for n <= sizeof(buf) bytes at w
	char *room(size_t n)
	{
		if ((size_t)(buf + sizeof(buf) - w) < n)
			flush();
		return w;
	}
	// literal-sized appends inline to a few stores; the rare flush / long
	// append is out of line
	__attribute__((always_inline)) Out &put(const char *t, size_t n)
	{
		if (__builtin_expect((size_t)(buf + sizeof(buf) - w) < n, 0))
			return put_slow(t, n);
		memcpy(w, t, n);
		w += n;
		return *this;
	}
	__attribute__((noinline)) Out &put_slow(const char *t, size_t n)
	{
		flush();
		if (n > sizeof(buf) / 2) {
			s.append(t, n);
			return *this;
		}
		memcpy(w, t, n);
		w += n;
		return *this;
	}
	__attribute__((always_inline)) Out &operator<<(const char *t) { return put(t, strlen(t)); }
	Out &c(char ch)
	{
		*room(1) = ch;
		w++;
		return *this;
	}
	// %u (two digits per step, written in place)
	Out &u(uint64_t v)
	{
		static const char d2[201] = "00010203040506070809101112131415161718192021222324252627282930313233343536373839"
					    "40414243444546474849505152535455565758596061626364656667686970717273747576777879"
					    "8081828384858687888990919293949596979899";
		static const uint64_t p10[20] = { 1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull,
			10000000ull, 100000000ull, 1000000000ull, 10000000000ull, 100000000000ull, 1000000000000ull,
			10000000000000ull, 100000000000000ull, 1000000000000000ull, 10000000000000000ull,
			100000000000000000ull, 1000000000000000000ull, 10000000000000000000ull };
		char *p = room(20);
		if (v < 10) {
			*p = (char)('0' + v);
			w = p + 1;
			return *this;
		}
		// digits = floor(log10 v) + 1 from the bit length
		int n = ((64 - __builtin_clzll(v)) * 1233) >> 12;
		n += v >= p10[n];
		char *e = p + n;
		w = e;
		while (v >= 100) {
			const uint32_t r = (uint32_t)(v % 100);
			v /= 100;
			e -= 2;
			memcpy(e, d2 + 2 * r, 2);
		}
		if (v >= 10)
			memcpy(e - 2, d2 + 2 * v, 2);
		else
			e[-1] = (char)('0' + v);
		return *this;
	}
	// %d / %zd
	Out &d(int64_t v)
	{
		if (v < 0) { c('-'); return u((uint64_t)(-(v + 1)) + 1); }
		return u((uint64_t)v);
	}
	// %x
	Out &x(uint64_t v)
	{
		static const char hx[] = "0123456789abcdef";
		char b[16];
		int i = 16;
		do { b[--i] = hx[v & 15]; v >>= 4; } while (v);
		return put(b + i, (size_t)(16 - i));
	}
	// %.Nx (zero padded to at least N digits)
	Out &xn(uint64_t v, int n)
	{
		static const char hx[] = "0123456789abcdef";
		const int bits = v ? 64 - __builtin_clzll(v) : 1;
		int k = (bits + 3) >> 2;
		if (k < n)
			k = n;
		char *p = room((size_t)k);
		w = p + k;
		for (int i = k - 1; i >= 0; i--, v >>= 4)
			p[i] = hx[v & 15];
		return *this;
	}
};

// bytes of one frame; offsets >= caplen read as zero (parity domain)
struct Frame {
	const uint8_t *p;
	uint32_t caplen;
	uint8_t b(uint64_t o) const { return o < caplen ? p[o] : 0; }
	uint16_t be16(uint64_t o) const { return (uint16_t)(b(o) << 8 | b(o + 1)); }
	uint16_t le16(uint64_t o) const { return (uint16_t)(b(o) | b(o + 1) << 8); }
	uint32_t be32(uint64_t o) const { return (uint32_t)be16(o) << 16 | be16(o + 2); }
	uint32_t le32(uint64_t o) const { return (uint32_t)le16(o) | (uint32_t)le16(o + 2) << 16; }
	uint64_t be64(uint64_t o) const { return (uint64_t)be32(o) << 32 | be32(o + 4); }
};

struct Layer {
	int id;
	uint32_t start;   // pkt->data when the layer's process() ran
	uint32_t tail;    // pkt->tail at that point
};

// What a layer did: where its cursor ended and whether it chained on.
struct Done {
	uint32_t data, tail;
	bool next;        // called pkt_set_dissector with a key present in the table
	bool ok;          // false: cannot render (host-only body)
};

static bool lay2_has(uint32_t k)
{
	switch (k) {
	case 0x0806: case 0x88cc: case 0x8100: case 0x0800: case 0x86DD: case 0x88a8: case 0x8847:
		return true;
	}
	return false;
}

static bool lay3_has(uint32_t k)
{
	switch (k) {
	case 1: case 58: case 2: case 51: case 50: case 60: case 44: case 0: case 41: case 135:
	case 59: case 43: case 6: case 17: case 33:
		return true;
	}
	return false;
}

// each byte value as " %.2x" and "%.2x:" in the low 3 bytes of a word
// (little endian: stored as 4 bytes, the next store 3 further on overwrites
// the 4th)
struct HexText {
	uint32_t sp[256], colon[256];
	constexpr HexText() : sp(), colon()
	{
		const char hx[] = "0123456789abcdef";
		for (int v = 0; v < 256; v++) {
			const uint32_t hi = (uint8_t)hx[v >> 4], lo = (uint8_t)hx[v & 15];
			sp[v] = (uint32_t)' ' | hi << 8 | lo << 16;
			colon[v] = hi | lo << 8 | (uint32_t)':' << 16;
		}
	}
};
static constexpr HexText k_hex{};

// decimal text of each octet value, its length in the 4th byte
struct OctetText {
	char t[256][4];
	constexpr OctetText() : t()
	{
		for (int v = 0; v < 256; v++) {
			int n = 0;
			if (v >= 100) t[v][n++] = (char)('0' + v / 100);
			if (v >= 10) t[v][n++] = (char)('0' + v / 10 % 10);
			t[v][n++] = (char)('0' + v % 10);
			t[v][3] = (char)n;
		}
	}
};
static constexpr OctetText k_octet{};

// the IPv4 address at off as inet_ntop prints it, straight into the sink
static void quad(Out &o, const Frame &f, uint64_t off)
{
	char *w = o.room(16);   // 4 x 4-byte stores, the last may run 1 past the text
	for (int i = 0; i < 4; i++) {
		const char *t = k_octet.t[f.b(off + i)];
		memcpy(w, t, 4);
		w += (uint8_t)t[3];
		if (i < 3)
			*w++ = '.';
	}
	o.w = w;
}

static void ntop6(const Frame &f, uint64_t off, char *buf)
{
	uint8_t a[16];
	for (int i = 0; i < 16; i++) a[i] = f.b(off + i);
	ntop6_to(a, buf);
}

// ether_lookup_addr (proto_ethernet.c:33-46)
static const char *ether_class(const Frame &f, uint32_t mac)
{
	uint8_t m0 = f.b(mac);
	if (m0 & 0x01) {
		if ((m0 & f.b(mac + 1) & f.b(mac + 2) & f.b(mac + 3) & f.b(mac + 4) & f.b(mac + 5)) == 0xff)
			return "Broadcast";
		return "Multicast";
	}
	if (m0 & 0x02)
		return "Locally Administered";
	const char *v = lookup_vendor((uint32_t)m0 << 16 | (uint32_t)f.b(mac + 1) << 8 | f.b(mac + 2));
	return v ? v : "Unknown";
}

// "%.2x:%.2x:%.2x:%.2x:%.2x:%.2x" in one write
static void mac(Out &o, const Frame &f, uint32_t m)
{
	char *w = o.room(20);   // (4-byte stores, 3 apart; the 6th ':' is not kept)
	for (int i = 0; i < 6; i++)
		memcpy(w + 3 * i, &k_hex.colon[f.b(m + i)], 4);
	o.w = w + 17;
}

// ---- layers --------------------------------------------------------------

// proto_ethernet.c:48-97
static Done r_ethernet(Out &o, const Frame &f, const Layer &L, int mode)
{
	if (L.tail - L.start < 14)
		return { L.start, L.tail, false, true };
	const uint32_t e = L.start;
	const uint16_t proto = f.be16(e + 12);
	const char *type = lookup_ether_type(proto);
	if (mode == PRINT_NORM) {
		o << " [ Eth MAC (";
		mac(o, f, e + 6);
		o << " => ";
		mac(o, f, e);
		o << "), Proto (0x";
		o.xn(proto, 4);
		if (type)
			o << ", " << C_BOLD << type << C_END;
		o << ") ]\n [ Vendor (" << ether_class(f, e + 6) << " => " << ether_class(f, e) << ") ]\n";
	} else {
		o << " " << ether_class(f, e + 6) << " => " << ether_class(f, e) << " " << C_BOLD
		  << (type ? type : "(null)") << C_END;
	}
	return { e + 14, L.tail, lay2_has(proto), true };
}

// proto_vlan.c:22-40 (vlan) and proto_vlan_q_in_q.c:23-41 (QinQ)
static Done r_vlan(Out &o, const Frame &f, const Layer &L, int mode, bool qinq)
{
	if (L.tail - L.start < 4)
		return { L.start, L.tail, false, true };
	const uint16_t tci = f.be16(L.start), inner = f.be16(L.start + 2);
	if (mode == PRINT_NORM) {
		o << (qinq ? " [ VLAN QinQ Prio (" : " [ VLAN Prio (");
		o.u((tci & 0xe000) >> 13) << (qinq ? "), DEI (" : "), CFI (");
		o.u((tci & 0x1000) >> 12) << "), ID (";
		o.u(tci & 0x0fff) << "), Proto (0x";
		o.xn(inner, 4) << ") ]\n";
	} else {
		o << " VLAN";
		o.u(tci & 0x0fff);
	}
	return { L.start + 4, L.tail, lay2_has(inner), true };
}

// proto_mpls_unicast.c:49-102
static Done r_mpls(Out &o, const Frame &f, const Layer &L, int mode)
{
	uint32_t d = L.start;
	for (;;) {
		if (L.tail - d < 4)
			return { d, L.tail, false, true };
		const uint32_t v = f.be32(d);
		const uint32_t s = (v >> 8) & 1;
		d += 4;
		if (mode == PRINT_NORM) {
			o << " [ MPLS Label (";
			o.u(v >> 12) << "), Exp (";
			o.u((v >> 9) & 7) << "), S (";
			o.u(s) << "), TTL (";
			o.u(v & 0xFF) << ") ]\n";
		} else {
			o << " MPLS/";
			o.u(v >> 12);
		}
		if (s)
			break;
	}
	bool next = false;
	if (L.tail - d) {
		const uint8_t nib = f.b(d) >> 4;
		next = nib == 4 || nib == 6;
	}
	return { d, L.tail, next, true };
}

// csum_expected (csum.h:29-39)
static uint16_t csum_expected(uint16_t sum, uint16_t computed)
{
	uint32_t s = sum;
	s += (uint16_t)((computed >> 8) | (computed << 8));
	s = (s & 0xFFFF) + (s >> 16);
	s = (s & 0xFFFF) + (s >> 16);
	return (uint16_t)s;
}

// proto_ipv4.c:34-204
static Done r_ipv4(Out &o, const Frame &f, const Layer &L, int mode, uint16_t ip_csum)
{
	if (L.tail - L.start < 20)
		return { L.start, L.tail, false, true };
	const uint32_t ip = L.start;
	const uint8_t ihl = f.b(ip) & 0xF;
	const uint16_t tot_len = f.be16(ip + 2);
	const uint8_t proto = f.b(ip + 9);
	uint32_t data = ip + 20, tail = L.tail;
	const uint32_t opts_len = (ihl > 5 ? ihl : 5) * 4u - 20u;

	if (mode != PRINT_NORM) {
		o << " ";
		quad(o, f, ip + 12);
		o << "/";
		quad(o, f, ip + 16);
		o << " Len ";
		o.u(tot_len);
		if (opts_len <= tail - data)
			data += opts_len;
		return { data, tail, lay3_has(proto), true };
	}

	// trailer: t bytes ending 20 B past the tail, printed %x (:56-67)
	{
		const uint64_t plen = tail - data;
		if (plen + 20 > tot_len) {
			uint32_t t = (uint32_t)(plen + 20 - tot_len);
			const uint64_t end = (uint64_t)data + tot_len + t;
			o << " [ Eth trailer ";
			while (t--)
				o.x(f.b(end - t));
			o << " ]\n";
		}
	}
	const uint16_t frag = f.be16(ip + 6);
	o << " [ IPv4 Addr (";
	quad(o, f, ip + 12);
	o << " => ";
	quad(o, f, ip + 16);
	o << "), Proto (";
	o.u(proto) << "), TTL (";
	o.u(f.b(ip + 8)) << "), TOS (";
	o.u(f.b(ip + 1)) << "), Ver (";
	o.u(f.b(ip) >> 4) << "), IHL (";
	o.u(ihl) << "), Tlen (";
	o.u(tot_len) << "), ID (";
	o.u(f.be16(ip + 4)) << "), Res (";
	o.u((frag & 0x8000) ? 1 : 0) << "), NoFrag (";
	o.u((frag & 0x4000) ? 1 : 0) << "), MoreFrag (";
	o.u((frag & 0x2000) ? 1 : 0) << "), FragOff (";
	o.u(frag & 0x1fff) << "), CSum (0x";
	o.xn(f.be16(ip + 10), 4) << ") is ";
	if (ip_csum) {
		o << C_RED << "bogus (!)" << C_END << C_RED << " should be 0x";
		o.xn(csum_expected(f.le16(ip + 10), ip_csum), 4) << C_END;
	} else {
		o << "ok";
	}
	o << " ]\n";

	// options (:133-169)
	if (opts_len <= tail - data) {
		uint64_t op = data;
		int64_t left = opts_len;
		data += opts_len;
		for (; left > 0; op++) {
			const uint8_t c = f.b(op);
			o << "   [ Option  Copied (";
			o.u((c & 0x80) ? 1 : 0) << "), Class (";
			o.u((c & 0x60) >> 5) << "), Number (";
			o.u(c & 0x1F) << ")";
			if (c == 0 || c == 1) {
				o << " ]\n";
				left--;
				continue;
			}
			int64_t olen = f.b(++op);
			if (olen < 2 || olen > left) {
				o << ", Len (";
				o.d(olen) << ", invalid) ]\n";
				break;
			}
			o << ", Len (";
			o.d(olen) << ") ]\n";
			left -= olen;
			o << "     [ Data hex ";
			for (olen -= 2; olen > 0; olen--) {
				o << " ";
				o.xn(f.b(++op), 2);
			}
			o << " ]\n";
		}
	}
	// trim (:174-175)
	{
		const int64_t x = (int64_t)tot_len - (int64_t)ihl * 4;
		if (x >= 0 && (uint64_t)x < tail - data)
			tail = data + (uint32_t)x;
	}
	return { data, tail, lay3_has(proto), true };
}

// proto_ipv6.c:22-105
static Done r_ipv6(Out &o, const Frame &f, const Layer &L, int mode)
{
	if (L.tail - L.start < 40)
		return { L.start, L.tail, false, true };
	const uint32_t ip = L.start;
	char s[INET6_ADDRSTRLEN], dd[INET6_ADDRSTRLEN];
	ntop6(f, ip + 8, s);
	ntop6(f, ip + 24, dd);
	const uint8_t nh = f.b(ip + 6);
	if (mode == PRINT_NORM) {
		const uint8_t b0 = f.b(ip), f0 = f.b(ip + 1), f1 = f.b(ip + 2), f2 = f.b(ip + 3);
		const uint8_t tc = (uint8_t)(((b0 & 0xF) << 4) | ((f0 & 0xF0) >> 4));
		const uint32_t flow = ((uint32_t)(f0 & 0x0F) << 8) | ((uint32_t)f1 << 4) | f2;  // :38-39 as written
		o << " [ IPv6 Addr (" << s << " => " << dd << "), Version (";
		o.u(b0 >> 4) << "), TrafficClass (";
		o.u(tc) << "), FlowLabel (";
		o.u(flow) << "), Len (";
		o.u(f.be16(ip + 4)) << "), NextHdr (";
		o.u(nh) << "), HopLimit (";
		o.u(f.b(ip + 7)) << ") ]\n";
	} else {
		o << " " << s << "/" << dd << " Len ";
		o.u(f.be16(ip + 4));
	}
	return { ip + 40, L.tail, lay3_has(nh), true };
}

// proto_ipv6_hop_by_hop.c:39-94, proto_ipv6_dest_opts.c:40-95
static Done r_v6opts(Out &o, const Frame &f, const Layer &L, int mode, bool dest)
{
	if (L.tail - L.start < 2)
		return { L.start, L.tail, false, true };
	const uint8_t nh = f.b(L.start), hl = f.b(L.start + 1);
	const uint32_t hdr_ext_len = (hl + 1u) * 8u, opt_len = hdr_ext_len - 2u;
	const uint32_t d = L.start + 2;
	const bool bad = opt_len > L.tail - d;
	if (mode == PRINT_NORM) {
		o << (dest ? "\t [ Destination Options NextHdr (" : "\t [ Hop-by-Hop Options NextHdr (");
		o.u(nh) << "), HdrExtLen (";
		o.u(hl) << ", ";
		o.u(hdr_ext_len);
		if (bad) {
			o << " Bytes, " << C_RED << "invalid" << C_END << ")";
			return { d, L.tail, false, true };
		}
		o << " Bytes)";
		if (opt_len)
			o << ", Option(s) recognized ";
		o << " ]\n";
	} else {
		if (bad)
			return { d, L.tail, false, true };
		o << (dest ? " Dest Ops" : " Hop Ops");
	}
	return { d + opt_len, L.tail, lay3_has(nh), true };
}

// proto_ipv6_routing.c:33-156
static Done r_routing(Out &o, const Frame &f, const Layer &L, int mode)
{
	if (L.tail - L.start < 4)
		return { L.start, L.tail, false, true };
	const uint32_t r = L.start;
	const uint8_t nh = f.b(r), hl = f.b(r + 1), type = f.b(r + 2), left = f.b(r + 3);
	const uint32_t hdr_ext_len = (hl + 1u) * 8u;
	int64_t data_len = (int64_t)hdr_ext_len - 4;
	uint32_t d = r + 4;
	auto bad = [&]() { return data_len > (int64_t)(L.tail - d) || data_len < 0; };

	if (mode == PRINT_NORM) {
		o << "\t [ Routing NextHdr (";
		o.u(nh) << "), HdrExtLen (";
		o.u(hl) << ", ";
		o.u(hdr_ext_len);
		if (bad()) {
			o << " Bytes " << C_RED << "invalid" << C_END << "), ";
			return { d, L.tail, false, true };
		}
		o << " Bytes), Type (";
		o.u(type) << "), Left (";
		o.u(left) << "), ";
		if (type == 0) {
			const bool pulled = L.tail - d >= 4;
			const uint32_t res = f.le32(d);   // printed in host order (:51)
			if (pulled) d += 4;
			data_len -= 4;
			if (pulled && !bad()) {
				o << "Res (0x";
				o.x(res) << ")";
				uint8_t num = (uint8_t)(data_len / 16);
				while (num--) {
					const bool ok = L.tail - d >= 16;
					const uint32_t a = d;
					if (ok) d += 16;
					data_len -= 16;
					if (!ok || bad())
						break;
					char buf[INET6_ADDRSTRLEN];
					ntop6(f, a, buf);
					o << "\n\t   Address: " << buf;
				}
			}
		} else {
			o << "Type ";
			o.u(type) << " is unknown";
		}
		o << " ]\n";
	} else {
		if (bad())
			return { d, L.tail, false, true };
		o << " Routing ";
		if (type == 0) {
			const bool pulled = L.tail - d >= 4;
			if (pulled) d += 4;
			data_len -= 4;
			if (pulled && !bad()) {
				o << "Addresses (";
				o.u((uint64_t)data_len / 16) << ")";
			}
		} else {
			o << "Type ";
			o.u(type) << " is unknown";
		}
	}
	if (bad())
		return { d, L.tail, false, true };
	return { d + (uint32_t)data_len, L.tail, lay3_has(nh), true };
}

// proto_ipv6_fragm.c:25-63
static Done r_fragm(Out &o, const Frame &f, const Layer &L, int mode)
{
	if (L.tail - L.start < 8)
		return { L.start, L.tail, false, true };
	const uint32_t g = L.start;
	const uint16_t w = f.be16(g + 2);
	if (mode == PRINT_NORM) {
		o << "\t [ Fragment NextHdr (";
		o.u(f.b(g)) << "), Reserved (";
		o.u(f.b(g + 1)) << "), Offset (";
		o.u(w >> 3) << "), Res (";
		o.u((w >> 1) & 3) << "), M flag (";
		o.u(w & 1) << "), Identification (";
		o.u(f.be32(g + 4)) << ") ]\n";
	} else {
		o << " FragmOffs ";
		o.u(w >> 3);
	}
	return { g + 8, L.tail, lay3_has(f.b(g)), true };
}

// proto_ip_authentication_hdr.c:26-88
static Done r_auth(Out &o, const Frame &f, const Layer &L, int mode)
{
	if (L.tail - L.start < 12)
		return { L.start, L.tail, false, true };
	const uint32_t a = L.start;
	const uint8_t nh = f.b(a), plen = f.b(a + 1);
	const uint32_t hdr_len = plen * 4u + 8u;
	uint32_t d = a + 12;
	if (hdr_len > L.tail - d) {
		if (mode == PRINT_NORM) {
			o << " [ Authentication Header NextHdr (";
			o.u(nh) << "), HdrLen (";
			o.u(plen) << ", ";
			o.u(hdr_len) << " Bytes " << C_RED << "invalid" << C_END << "), ";
		}
		return { d, L.tail, false, true };
	}
	if (mode == PRINT_NORM) {
		o << " [ Authentication Header NextHdr (";
		o.u(nh) << "), HdrLen (";
		o.u(plen) << ", ";
		o.u(hdr_len) << " Bytes), Reserved (0x";
		o.x(f.be16(a + 2)) << "), SPI (0x";
		o.x(f.be32(a + 4)) << "), SNF (0x";
		o.x(f.be32(a + 8)) << "), ICV 0x";
		for (uint32_t i = 12; i < hdr_len; i++)
			o.xn(f.b(d++), 2);
		o << " ]\n";
	} else {
		o << " AH";
		if (hdr_len >= 12)
			d += hdr_len - 12;
	}
	return { d, L.tail, lay3_has(nh), true };
}

// proto_ip_esp.c:23-46
static Done r_esp(Out &o, const Frame &f, const Layer &L, int mode)
{
	if (L.tail - L.start < 8)
		return { L.start, L.tail, false, true };
	if (mode == PRINT_NORM) {
		o << " [ ESP SPI (0x";
		o.x(f.be32(L.start)) << "), SN (0x";
		o.x(f.be32(L.start + 4)) << ") ]\n";
	} else {
		o << " ESP";
	}
	return { L.start + 8, L.tail, false, true };
}

// proto_ipv6_no_nxt_hdr.c:17-34
static Done r_nonext(Out &o, const Layer &L, int mode)
{
	o << (mode == PRINT_NORM ? " [ No Next Header ]\n" : " No Next Header");
	return { L.start, L.tail, false, true };
}

// proto_ipv6_mobility_hdr.c:81-309
static Done r_mobility(Out &o, const Frame &f, const Layer &L, int mode)
{
	if (L.tail - L.start < 6)
		return { L.start, L.tail, false, true };
	const uint32_t m = L.start;
	const uint8_t nh = f.b(m), hl = f.b(m + 1), type = f.b(m + 2);
	const uint32_t hdr_ext_len = (hl + 1u) * 8u;
	int64_t mdl = (int64_t)hdr_ext_len - 6;
	uint32_t d = m + 6;
	auto bad = [&]() { return mdl > (int64_t)(L.tail - d) || mdl < 0; };

	if (mode != PRINT_NORM) {
		if (bad())
			return { d, L.tail, false, true };
		o << " Mobility Type (";
		o.u(type) << "), ";
		return { d + (uint32_t)mdl, L.tail, lay3_has(nh), true };
	}
	o << "\t [ Mobility NextHdr (";
	o.u(nh) << "), HdrExtLen (";
	o.u(hl) << ", ";
	o.u(hdr_ext_len);
	if (bad()) {
		o << " Bytes " << C_RED << "invalid" << C_END << "), ";
		return { d, L.tail, false, true };
	}
	o << " Bytes), MH Type (";
	o.u(type) << "), Res (0x";
	o.x(f.b(m + 3)) << "), Chks (0x";
	o.x(f.be16(m + 4)) << "), MH Data ";
	auto opts = [&]() { if (mdl) o << "MH Option(s) recognized "; };
	// get_mh_type (:206-245): pull a fixed part, then print if the rest fits
	auto sub = [&](uint32_t n, bool dec_on_fail) -> int64_t {
		const bool ok = L.tail - d >= n;
		const uint32_t at = d;
		if (ok) d += n;
		if (ok || dec_on_fail) mdl -= n;
		if (!ok) return -1;
		return at;
	};
	switch (type) {
	case 0: {
		o << "Binding Refresh Request Message ";
		int64_t at = sub(2, true);
		if (at >= 0 && !bad()) opts();
		break;
	}
	case 1: case 2: {
		o << (type == 1 ? "Home Test Init Message " : "Care-of Test Init Message ");
		int64_t at = sub(10, true);
		if (at >= 0 && !bad()) {
			o << "Init Cookie (0x";
			o.x(f.be64(at + 2)) << ")";
			opts();
		}
		break;
	}
	case 3: case 4: {
		o << "Binding Refresh Request Message ";
		int64_t at = sub(18, true);
		if (at >= 0 && !bad()) {
			o << "HN Index (";
			o.u(f.be16(at)) << ") Init Cookie (0x";
			o.x(f.be64(at + 2)) << ") Keygen Token (0x";
			o.x(f.be64(at + 10)) << ")";
			opts();
		}
		break;
	}
	case 5: {
		o << "Binding Refresh Request Message ";
		int64_t at = sub(6, true);
		if (at >= 0 && !bad()) {
			o << "Sequence (0x";
			o.x(f.be16(at)) << ") A|H|L|K (0x";
			o.x(f.be16(at + 2) >> 12) << ") Lifetime (";
			o.u(f.be16(at + 4) * 4u) << "s)";
			opts();
		}
		break;
	}
	case 6: {
		o << "Binding Refresh Request Message ";
		int64_t at = sub(6, false);
		if (at >= 0 && !bad()) {
			o << "Status (0x";
			o.x(f.b(at)) << ") K (";
			o.u(f.b(at + 1) >> 7) << ") Sequence (0x";
			o.x(f.be16(at + 2)) << ")Lifetime (";
			o.u(f.be16(at + 4) * 4u) << "s)";
			opts();
		}
		break;
	}
	case 7: {
		o << "Binding Refresh Request Message ";
		int64_t at = sub(10, false);
		if (at >= 0 && !bad()) {
			// :194-201 reads 8 stack bytes past a u64: outside the parity
			// domain; rendered with those bytes as zero
			uint8_t a[16] = { 0 };
			uint64_t v = f.be64(at + 2);
			memcpy(a, &v, 8);
			char buf[INET6_ADDRSTRLEN];
			ntop6_to(a, buf);
			o << "Status (0x";
			o.x(f.b(at)) << ") Home Addr (" << buf << ")";
			opts();
		}
		break;
	}
	default:
		o << "Type ";
		o.u(type) << " is unknown. Error";
	}
	o << " ]\n";
	if (bad())
		return { d, L.tail, false, true };
	return { d + (uint32_t)mdl, L.tail, lay3_has(nh), true };
}

// proto_tcp.c:63-151
static Done r_tcp(Out &o, const Frame &f, const Layer &L, int mode)
{
	if (L.tail - L.start < 20)
		return { L.start, L.tail, false, true };
	static const char *const names[8] = { "FIN", "SYN", "RST", "PSH", "ACK", "URG", "ECE", "CWR" };
	const uint32_t t = L.start;
	const uint16_t sp = f.be16(t), dp = f.be16(t + 2);
	const uint8_t b12 = f.b(t + 12), fl = f.b(t + 13);
	const char *sn = lookup_port_tcp(sp), *dn = lookup_port_tcp(dp);
	if (mode == PRINT_NORM) {
		o << " [ TCP Port (";
		o.u(sp);
		if (sn) o << " (" << C_BOLD << sn << C_END << ")";
		o << " => ";
		o.u(dp);
		if (dn) o << " (" << C_BOLD << dn << C_END << ")";
		o << "), SN (0x";
		o.x(f.be32(t + 4)) << "), AN (0x";
		o.x(f.be32(t + 8)) << "), DataOff (";
		o.u(b12 >> 4) << "), Res (";
		o.u(b12 & 15) << "), Flags (";
		// tprintf_flag (:56-63) resets the separator after an unset flag
		bool v = false;
		for (int i = 0; i < 8; i++) {
			const bool set = (fl >> i) & 1;
			if (set) {
				if (v) o.c(' ');
				o << names[i];
			}
			v = set;
		}
		o << "), Window (";
		o.u(f.be16(t + 14)) << "), CSum (0x";
		o.xn(f.be16(t + 16), 4) << "), UrgPtr (";
		o.u(f.be16(t + 18)) << ") ]\n";
	} else {
		o << " TCP ";
		o.u(sp);
		if (sn) o << "(" << C_BOLD << sn << C_END << ")";
		o << "/";
		o.u(dp);
		if (dn) o << "(" << C_BOLD << dn << C_END << ")";
		o << " F" << C_BOLD;
		for (int i = 0; i < 8; i++)
			if ((fl >> i) & 1)
				o << " " << names[i];
		o << C_END << " Win ";
		o.u(f.be16(t + 14)) << " S/A 0x";
		o.x(f.be32(t + 4)) << "/0x";
		o.x(f.be32(t + 8));
	}
	return { t + 20, L.tail, false, true };
}

// proto_udp.c:23-83
static Done r_udp(Out &o, const Frame &f, const Layer &L, int mode)
{
	if (L.tail - L.start < 8)
		return { L.start, L.tail, false, true };
	const uint32_t u = L.start;
	const uint16_t sp = f.be16(u), dp = f.be16(u + 2), ulen = f.be16(u + 4);
	const char *sn = lookup_port_udp(sp), *dn = lookup_port_udp(dp);
	if (mode == PRINT_NORM) {
		const int64_t len = (int64_t)ulen - 8;
		o << " [ UDP Port (";
		o.u(sp);
		if (sn) o << " (" << C_BOLD << sn << C_END << ")";
		o << " => ";
		o.u(dp);
		if (dn) o << " (" << C_BOLD << dn << C_END << ")";
		o << "), ";
		if (len > (int64_t)(L.tail - u - 8) || len < 0) {
			o << "Len (";
			o.u(ulen) << ") " << C_RED << "invalid" << C_END << ", ";
		}
		o << "Len (";
		o.u(ulen) << " Bytes, ";
		o.d(len) << " Bytes Data), CSum (0x";
		o.xn(f.be16(u + 6), 4) << ") ]\n";
	} else {
		o << " UDP ";
		o.u(sp);
		if (sn) o << "(" << C_BOLD << sn << C_END << ")";
		o << "/";
		o.u(dp);
		if (dn) o << "(" << C_BOLD << dn << C_END << ")";
	}
	return { u + 8, L.tail, false, true };
}

// proto_icmpv4.c:34-61
static Done r_icmp(Out &o, const Frame &f, const Layer &L, int mode, bool bad)
{
	if (L.tail - L.start < 8)
		return { L.start, L.tail, false, true };
	const uint32_t c = L.start;
	if (mode == PRINT_NORM) {
		o << " [ ICMP Type (";
		o.u(f.b(c)) << "), Code (";
		o.u(f.b(c + 1)) << "), CSum (0x";
		o.xn(f.be16(c + 2), 4) << ") is ";
		if (bad) o << C_RED << "bogus (!)" << C_END;
		else o << "ok";
		o << " ]\n";
	} else {
		o << " Type ";
		o.u(f.b(c)) << " Code ";
		o.u(f.b(c + 1));
	}
	return { c + 8, L.tail, false, true };
}

// ICMPv6 names (proto_icmpv6.c:912-1021, icmpv6_process :1492-1665)
static const char *const v6_t1[] = {
	"No route to destination",
	"Communication with destination administratively prohibited",
	"Beyond scope of source address", "Address unreachable", "Port unreachable",
	"Source address failed ingress/egress policy", "Reject route to destination",
	"Error in Source Routing Header",
};
static const char *const v6_t3[] = { "Hop limit exceeded in transit",
				     "Fragment reassembly time exceeded" };
static const char *const v6_t4[] = { "Erroneous header field encountered",
				     "Unrecognized Next Header type encountered",
				     "Unrecognized IPv6 option encountered" };

static void icmpv6_names(uint8_t t, uint8_t c, const char *&ts, const char *&cs, int &body)
{
	ts = "Unknown Type";
	cs = "Unknown Code";
	body = 0;
	switch (t) {
	case 1: ts = "Destination Unreachable"; if (c < 8) cs = v6_t1[c]; body = 1; break;
	case 2: ts = "Packet Too Big"; body = 2; break;
	case 3: ts = "Time Exceeded"; if (c < 2) cs = v6_t3[c]; body = 3; break;
	case 4: ts = "Parameter Problem"; if (c < 3) cs = v6_t4[c]; body = 4; break;
	case 100: case 101: case 200: case 201: ts = "Private experimation"; break;
	case 127: case 255: ts = "Reserved for expansion of ICMPv6 error messages"; break;
	case 128: ts = "Echo Request"; body = 128; break;
	case 129: ts = "Echo Reply"; body = 129; break;
	case 155:
		ts = "RPL Control Message";
		switch (c) {
		case 0x00: cs = "DODAG Information Solicitation"; break;
		case 0x01: cs = "DODAG Information Object"; break;
		case 0x02: cs = "Destination Advertisement Object"; break;
		case 0x03: cs = "Destination Advertisement Object Acknowledgment"; break;
		case 0x80: cs = "Secure DODAG Information Solicitation"; break;
		case 0x81: cs = "Secure DODAG Information Object"; break;
		case 0x82: cs = "Secure Destination Advertisement Object"; break;
		case 0x83: cs = "Secure Destination Advertisement Object Acknowledgment"; break;
		case 0x8A: cs = "Consistency Check"; break;
		}
		break;
	default:
		if (t >= 130 && t <= 154)
			body = -1;   // variable-length body
	}
}

static Done r_icmpv6_host(Out &o, const Frame &f, const Layer &L);

// proto_icmpv6.c:1667-1699
static Done r_icmpv6(Out &o, const Frame &f, const Layer &L, int mode)
{
	if (L.tail - L.start < 4)
		return { L.start, L.tail, false, true };
	const uint32_t h = L.start;
	const uint8_t type = f.b(h), code = f.b(h + 1);
	if (mode != PRINT_NORM) {
		o << " ICMPv6 Type (";
		o.u(type) << ") Code (";
		o.u(code) << ")";
		return { h + 4, L.tail, false, true };
	}
	const char *ts, *cs;
	int body;
	icmpv6_names(type, code, ts, cs, body);
	if (body < 0)
		return r_icmpv6_host(o, f, L);   // types 130-154 (NSD_F_HOST), nsd_format_icmpv6.h
	uint32_t d = h + 4;
	o << " [ ICMPv6 " << ts << " (";
	o.u(type) << "), " << cs << " (";
	o.u(code) << "), Chks (0x";
	o.x(f.be16(h + 2)) << ")";
	if (body) {
		if (L.tail - d < 4) {
			o << "\n" << C_RED << "Failed to dissect Message" << C_END;
		} else {
			const uint32_t b = d;
			d += 4;
			switch (body) {
			case 1: case 3:
				o << ", Unused (0x";
				o.x(f.be32(b)) << ") Payload include as much of invoking packet";
				break;
			case 2:
				o << ", MTU (0x";
				o.x(f.be32(b)) << ") Payload include as much of invoking packet";
				break;
			case 4:
				o << ", Pointer (0x";
				o.x(f.be32(b)) << ") Payload include as much of invoking packet";
				break;
			default:
				o << ", ID (0x";
				o.x(f.be16(b)) << "), Seq. Nr. (";
				o.u(f.be16(b + 2)) << ") Payload include Data";
			}
		}
	}
	o << " ]\n";
	return { d, L.tail, false, true };
}

// proto_none.c:17-72
static void dump_ascii(Out &o, const Frame &f, uint32_t from, uint32_t len)
{
	if (!len)
		return;
	o << " [ Chr ";
	const bool inside = (uint64_t)from + len <= f.caplen;   // (bytes past caplen read as zero)
	for (uint32_t i0 = 0; i0 < len; i0 += 1024) {
		const uint32_t m = len - i0 < 1024 ? len - i0 : 1024;
		char *w = o.room(m);
		if (inside) {
			const uint8_t *q = f.p + from + i0;
			for (uint32_t i = 0; i < m; i++)
				w[i] = (q[i] >= 0x20 && q[i] < 0x7f) ? (char)q[i] : '.';
		} else {
			for (uint32_t i = 0; i < m; i++) {
				const uint8_t c = f.b(from + i0 + i);
				w[i] = (c >= 0x20 && c < 0x7f) ? (char)c : '.';
			}
		}
		o.w += m;
	}
	o << " ]\n";
}

static void dump_hex(Out &o, const Frame &f, uint32_t from, uint32_t len)
{
	if (!len)
		return;
	o << " [ Hex ";
	const bool inside = (uint64_t)from + len <= f.caplen;   // (bytes past caplen read as zero)
	for (uint32_t i0 = 0; i0 < len; i0 += 512) {
		const uint32_t m = len - i0 < 512 ? len - i0 : 512;
		char *w = o.room(3 * (size_t)m + 1);   // (4-byte stores, 3 apart)
		for (uint32_t i = 0; i < m; i++) {
			const uint8_t c = inside ? f.p[from + i0 + i] : f.b(from + i0 + i);
			memcpy(w + 3 * i, &k_hex.sp[c], 4);
		}
		o.w += 3 * (size_t)m;
	}
	o << " ]\n";
}

#include "nsd_format_leaves.h"
#include "nsd_format_icmpv6.h"
#include "nsd_format_sll.h"

static bool is_lt(int lt, uint32_t v) { return (uint32_t)lt == v || (uint32_t)lt == __builtin_bswap32(v); }

// The print function of ops L.id over [L.start, L.tail): its text, and where
// the reference parser leaves the cursor (Done)
static Done render_one(Out &o, const Frame &f, const Layer &L, int mode, uint16_t ip_csum, bool icmp_bad,
		       const nsd_sll_t *sll)
{
	switch (L.id) {
	case NSD_OPS_ETHERNET:       return r_ethernet(o, f, L, mode);
	case NSD_OPS_VLAN:           return r_vlan(o, f, L, mode, false);
	case NSD_OPS_QINQ:           return r_vlan(o, f, L, mode, true);
	case NSD_OPS_MPLS_UC:        return r_mpls(o, f, L, mode);
	case NSD_OPS_IPV4:           return r_ipv4(o, f, L, mode, ip_csum);
	case NSD_OPS_IPV6:
	case NSD_OPS_IPV6_IN_IPV4:   return r_ipv6(o, f, L, mode);
	case NSD_OPS_IPV6_HOP_BY_HOP:return r_v6opts(o, f, L, mode, false);
	case NSD_OPS_IPV6_DEST_OPTS: return r_v6opts(o, f, L, mode, true);
	case NSD_OPS_IPV6_ROUTING:   return r_routing(o, f, L, mode);
	case NSD_OPS_IPV6_FRAGM:     return r_fragm(o, f, L, mode);
	case NSD_OPS_IP_AUTH:        return r_auth(o, f, L, mode);
	case NSD_OPS_IP_ESP:         return r_esp(o, f, L, mode);
	case NSD_OPS_IPV6_NO_NEXT:   return r_nonext(o, L, mode);
	case NSD_OPS_IPV6_MOBILITY:  return r_mobility(o, f, L, mode);
	case NSD_OPS_TCP:            return r_tcp(o, f, L, mode);
	case NSD_OPS_UDP:            return r_udp(o, f, L, mode);
	case NSD_OPS_ICMPV4:         return r_icmp(o, f, L, mode, icmp_bad);
	case NSD_OPS_ICMPV6:         return r_icmpv6(o, f, L, mode);
	// leaves the device classifies and the host renders (NSD_F_HOST)
	case NSD_OPS_ARP:            return r_arp(o, f, L, mode);
	case NSD_OPS_LLDP:           return r_lldp(o, f, L, mode);
	case NSD_OPS_IGMP:           return r_igmp(o, f, L, mode);
	case NSD_OPS_DCCP:           return r_dccp(o, f, L, mode);
	case NSD_OPS_SLL:            return r_sll(o, L, mode, sll);
	}
	return { L.start, L.tail, false, false };   // 802.11, netlink heads
}

bool render_layer(std::string &s, const uint8_t *pkt, uint32_t caplen, int id, uint32_t start, uint32_t tail,
		  int mode, uint16_t ip_csum, bool icmp_bad, const nsd_sll_t *sll, uint32_t &data,
		  uint32_t &ntail, bool &next)
{
	Out o(s);
	Frame f{ pkt, caplen };
	Layer L{ id, start, tail };
	const Done dn = render_one(o, f, L, mode, ip_csum, icmp_bad, sll);
	data = dn.data;
	ntail = dn.tail;
	next = dn.next;
	return dn.ok;
}

// proto_none.c: _hex / _ascii over [from, from + len) (empty for len 0)
void render_hex(std::string &s, const uint8_t *pkt, uint32_t caplen, uint32_t from, uint32_t len)
{
	Out o(s);
	dump_hex(o, Frame{ pkt, caplen }, from, len);
}

void render_ascii(std::string &s, const uint8_t *pkt, uint32_t caplen, uint32_t from, uint32_t len)
{
	Out o(s);
	dump_ascii(o, Frame{ pkt, caplen }, from, len);
}

// PRINT_HEX / _ASCII / _HEX_ASCII: every process() is NULL (dissector.c:26-38,
// 108-118); true when `mode` is one of those (or PRINT_NONE) and was handled
static bool format_no_chain(Out &o, const Frame &f, uint32_t caplen, int mode)
{
	if (mode == PRINT_NONE)
		return true;
	if (mode == PRINT_NORM || mode == PRINT_LESS)
		return false;
	if (mode == PRINT_HEX) {
		if (caplen) { dump_hex(o, f, 0, caplen); o << "\n"; }
	} else if (mode == PRINT_ASCII) {
		if (caplen) { dump_ascii(o, f, 0, caplen); o << "\n"; }
	} else {
		if (caplen) { dump_ascii(o, f, 0, caplen); dump_hex(o, f, 0, caplen); }
		o << "\n";
	}
	return true;
}

// The chain's text: layers ids[0..n) as dissector_main runs them, then the
// exit op.  offs: the layer starts the walk recorded (each layer's print must
// end exactly where the next one starts), or NULL: each layer starts where
// the previous print left the cursor (compact records).  end: the walk's
// final {data, tail} to check, or NULL.
static int format_chain(Out &o, const Frame &f, int linktype, int mode, uint32_t n, const uint8_t *ids,
			const uint16_t *offs, const uint32_t *end, uint16_t ip_csum, uint8_t nflags,
			const nsd_sll_t *sll, uint32_t leaf_end = 0xFFFFFFFFu)
{
	const bool host = nflags & NSD_F_HOST;
	if (n == 0 && is_lt(linktype, NSD_LINKTYPE_EN10MB))
		return NSD_ERR_FORMAT;
	if (host && n == 0)
		return NSD_ERR_FORMAT;
	uint32_t tail = f.caplen, data = 0;
	for (uint32_t k = 0; k < n; k++) {
		Layer L{ ids[k], offs ? offs[k] : data, tail };
		if (L.start > tail)
			return NSD_ERR_FORMAT;
		const Done dn = render_one(o, f, L, mode, ip_csum, nflags & NSD_F_ICMP_BAD, sll);
		if (!dn.ok)
			return NSD_ERR_FORMAT;
		// consistency with the walk: the chain goes on exactly while it has
		// layers, and (16-byte records, ext entries) ends where it recorded
		// (for a host-rendered leaf too: the walk kept where its pulls end)
		if (k + 1 < n) {
			if (!dn.next || (offs && dn.data != offs[k + 1]))
				return NSD_ERR_FORMAT;
		} else {
			if (dn.next || (end && (dn.data != end[0] || dn.tail != end[1])))
				return NSD_ERR_FORMAT;
			// compact records: the device's end of a host-rendered leaf
			if (leaf_end != 0xFFFFFFFFu && dn.data != leaf_end)
				return NSD_ERR_FORMAT;
		}
		tail = dn.tail;
		data = dn.data;
	}
	// exit op (dissector.c:60-61) over what the last layer left
	if (mode == PRINT_NORM) {
		const uint32_t len = tail - data;
		if (len) {
			dump_ascii(o, f, data, len);
			dump_hex(o, f, data, len);
		}
	}
	o << "\n";
	return NSD_OK;
}

// the ext entry's chain (NSD_ERR_FORMAT when there is none)
static int ext_chain(const uint32_t *ext_pool, uint32_t slot, uint8_t nflags, uint32_t &n, uint8_t *ids,
		     uint16_t *offs)
{
	if (!ext_pool || slot == 0xFFFFFFFFu || (nflags & NSD_F_OVERFLOW))
		return NSD_ERR_FORMAT;
	n = NSD_EXT_NLAYERS(ext_pool, slot);
	if (n > NSD_EXT_MAX_LAYERS)
		return NSD_ERR_FORMAT;
	for (uint32_t k = 0; k < n; k++) {
		ids[k] = (uint8_t)NSD_EXT_ID(ext_pool, slot, k);
		offs[k] = (uint16_t)NSD_EXT_OFF(ext_pool, slot, k);
	}
	return NSD_OK;
}

// Render one packet; returns NSD_OK or NSD_ERR_FORMAT (text so far kept).
int format_packet(std::string &s, const uint8_t *pkt, uint32_t caplen, int linktype, int mode,
		  const nsd_rec &rec, const uint32_t *ext_pool, const nsd_sll_t *sll)
{
	Out o(s);
	Frame f{ pkt, caplen };
	if (format_no_chain(o, f, caplen, mode))
		return NSD_OK;
	// the chain as the device recorded it
	uint32_t n = rec.nflags & 7u;
	uint8_t ids[NSD_EXT_MAX_LAYERS];
	uint16_t offs[NSD_EXT_MAX_LAYERS];
	if (n == NSD_N_EXT) {
		uint32_t slot;
		memcpy(&slot, rec.off2, 4);
		if (ext_chain(ext_pool, slot, rec.nflags, n, ids, offs) != NSD_OK)
			return NSD_ERR_FORMAT;
	} else {
		for (uint32_t k = 0; k < n; k++) {
			ids[k] = (uint8_t)((rec.chain >> (5 * k)) & 31);
			offs[k] = k ? (uint16_t)(rec.off2[k - 1] * 2u) : 0;
		}
	}
	const uint32_t end[2] = { rec.data_off, rec.tail_off };
	return format_chain(o, f, linktype, mode, n, ids, offs, end, rec.ip_csum, rec.nflags, sll);
}

// the same over compact record i: the layer starts come from the prints
static int packet_compact(Out &o, const uint8_t *pkt, uint32_t caplen, int linktype, int mode, const nsd_crec &rec,
			  uint32_t i, const uint32_t *ext_pool, const nsd_sll_t *sll)
{
	Frame f{ pkt, caplen };
	if (format_no_chain(o, f, caplen, mode))
		return NSD_OK;
	uint32_t n = rec.nflags & 7u;
	uint8_t ids[NSD_EXT_MAX_LAYERS];
	uint16_t offs[NSD_EXT_MAX_LAYERS];
	if (n == NSD_N_EXT && rec.nlayers) {
		// 7..12 layers: ids 6.. in the packet's side word (pool word i)
		if (!ext_pool || (rec.nflags & NSD_F_OVERFLOW) || rec.nlayers <= NSD_REC_MAX_LAYERS ||
		    rec.nlayers > NSD_CREC_MAX_LAYERS)
			return NSD_ERR_FORMAT;
		n = rec.nlayers;
		for (uint32_t k = 0; k < n; k++)
			ids[k] = (uint8_t)(k < NSD_REC_MAX_LAYERS ? (rec.chain >> (5 * k)) & 31
								  : (ext_pool[i] >> (5 * (k - NSD_REC_MAX_LAYERS))) & 31);
		return format_chain(o, f, linktype, mode, n, ids, nullptr, nullptr, rec.ip_csum, rec.nflags, sll);
	}
	const bool le = (rec.nflags & (NSD_F_HOST | NSD_F_LEAF_END)) == (NSD_F_HOST | NSD_F_LEAF_END);
	if (le && !ext_pool)
		return NSD_ERR_FORMAT;
	if (n == NSD_N_EXT) {
		// (a compact chain's entry holds ids only; a host leaf's end in word 2)
		if (ext_chain(ext_pool, rec.chain, rec.nflags, n, ids, offs) != NSD_OK)
			return NSD_ERR_FORMAT;
		return format_chain(o, f, linktype, mode, n, ids, nullptr, nullptr, rec.ip_csum, rec.nflags, sll,
				    le ? ext_pool[rec.chain + 2] & 0xFFFF : 0xFFFFFFFFu);
	}
	for (uint32_t k = 0; k < n; k++)
		ids[k] = (uint8_t)((rec.chain >> (5 * k)) & 31);
	return format_chain(o, f, linktype, mode, n, ids, nullptr, nullptr, rec.ip_csum, rec.nflags, sll,
			    le ? ext_pool[i] & 0xFFFF : 0xFFFFFFFFu);
}

int format_packet_compact(std::string &s, const uint8_t *pkt, uint32_t caplen, int linktype, int mode,
			  const nsd_crec &rec, uint32_t i, const uint32_t *ext_pool, const nsd_sll_t *sll)
{
	Out o(s);
	return packet_compact(o, pkt, caplen, linktype, mode, rec, i, ext_pool, sll);
}

// hex() / ascii() / hex_ascii() over [from, to) (proto_none.c:28-72)
void format_post_dump(std::string &s, const uint8_t *pkt, uint32_t caplen, int mode, uint32_t from,
		      uint32_t to)
{
	Out o(s);
	Frame f{ pkt, caplen };
	const uint32_t len = to - from;
	if (mode == PRINT_HEX) {
		if (len) { dump_hex(o, f, from, len); o << "\n"; }
	} else if (mode == PRINT_ASCII) {
		if (len) { dump_ascii(o, f, from, len); o << "\n"; }
	} else if (mode == PRINT_HEX_ASCII) {
		if (len) { dump_ascii(o, f, from, len); dump_hex(o, f, from, len); }
		o << "\n";
	}
}

// ---- show_frame_hdr (dissector.h:31-116) ----------------------------------

// if_indextoname (dissector.h:82, 89), cached per interface index: the
// reference asks the kernel for every packet (a socket and an ioctl).  The
// lookup runs outside the cache's lock; only names that exist are cached
// (at most IF_CACHE_MAX indexes: a file of many distinct indexes pays the
// lookups past that, as the reference does), and a failed lookup is kept
// only as the thread's last one, so an interface that appears later is
// seen.  nsd_if_cache_reset() (each replay, dissector_cleanup_all) drops the
// cache: renamed interfaces are seen by the next replay.  Index 0 names no
// interface.  Copies the name into b (IF_NAMESIZE bytes); false where there
// is none.
namespace {
constexpr size_t IF_NAME_MAX = 16;   // IF_NAMESIZE
constexpr size_t IF_CACHE_MAX = 4096;
std::mutex g_if_mu;
std::unordered_map<uint32_t, std::string> g_if_names;
std::atomic<uint32_t> g_if_gen{ 1 };
} // namespace

extern "C" __attribute__((visibility("hidden"))) void nsd_if_cache_reset(void)
{
	std::lock_guard<std::mutex> g(g_if_mu);
	g_if_names.clear();
	g_if_gen.fetch_add(1, std::memory_order_relaxed);
}

static bool if_name(uint32_t idx, char *b)
{
	thread_local uint32_t t_idx = 0, t_gen = 0;
	thread_local bool t_ok = false;
	thread_local char t_name[IF_NAME_MAX];
	if (idx == 0)
		return false;
	const uint32_t gen = g_if_gen.load(std::memory_order_relaxed);
	if (idx == t_idx && gen == t_gen) {
		if (t_ok)
			memcpy(b, t_name, IF_NAME_MAX);
		return t_ok;
	}
	bool ok = false, cached = false;
	{
		std::lock_guard<std::mutex> g(g_if_mu);
		auto it = g_if_names.find(idx);
		if (it != g_if_names.end()) {
			snprintf(b, IF_NAME_MAX, "%s", it->second.c_str());
			ok = cached = true;
		}
	}
	if (!cached) {
		ok = if_indextoname(idx, b) != nullptr;
		if (ok) {
			std::lock_guard<std::mutex> g(g_if_mu);
			if (g_if_names.size() < IF_CACHE_MAX)
				g_if_names.emplace(idx, b);
		}
	}
	t_idx = idx;
	t_gen = gen;
	t_ok = ok;
	if (ok)
		memcpy(t_name, b, IF_NAME_MAX);
	return ok;
}

static void frame_hdr(Out &o, const nsd_frame_hdr_t &fh, const nsd_sll_t *sll, const uint8_t *pkt, uint32_t caplen,
		      int linktype, int mode, uint64_t count)
{
	// packet_types[] (dissector.h:31-39)
	static const char *const types[8] = { "<", "B", "M", "P", ">", nullptr, "K->U", "U->K" };
	static const uint8_t type_len[8] = { 1, 1, 1, 1, 1, 0, 4, 4 };
	if (mode == PRINT_NONE)
		return;
	uint8_t pkttype = sll ? sll->pkttype : 0;
	// nlmon captures: sll_pkttype is PACKET_OUTGOING for every packet; the
	// nlmsg_pid tells kernel from user (dissector.h:71-75; the link type
	// compared as passed, unswapped)
	if ((uint32_t)linktype == NSD_LINKTYPE_NETLINK && caplen >= 16 && pkttype == 4) {
		uint32_t pid;
		memcpy(&pid, pkt + 12, 4);
		pkttype = pid == 0 ? 7 : 6;
	}
	if (pkttype < 8 && types[pkttype])
		o.put(types[pkttype], type_len[pkttype]);
	else
		o << "?";
	char ifb[IF_NAME_MAX];
	if (if_name(sll ? (uint32_t)sll->ifindex : 0, ifb))
		o << " " << ifb << " ";
	else
		o << " ? ";
	o.u(fh.len);
	if (mode == PRINT_LESS) {
		o << " #";
		o.u(count);
		return;
	}
	o << " ";
	o.u(fh.sec) << "s.";
	o.u(fh.nsec) << "ns #";
	o.u(count).c(' ');
	if (!fh.v3) {
		// __show_ts_source (dissector.h:41-51)
		if (fh.status & 0x80000000u)
			o << "(raw hw ts)";
		else if (fh.status & 0x40000000u)
			o << "(sys hw ts)";
		else if (fh.status & 0x20000000u)
			o << "(sw ts)";
	}
	o.c('\n');
	// tpacket_has_vlan_info (ring.h:71-84): TP_STATUS_VLAN_VALID (1 << 4) |
	// TP_STATUS_VLAN_TPID_VALID (1 << 6) of the tpacket3_hdr view's tp_status,
	// which for a tpacket2_hdr is its tp_nsec; the tci / tpid helpers give 0
	// for v2 (ring.h:51-69)
	const uint32_t st = fh.v3 ? fh.status : fh.nsec;
	if (st & 0x50u) {
		const uint16_t tci = fh.v3 ? (uint16_t)fh.vlan_tci : 0;
		const uint16_t tpid = fh.v3 ? fh.vlan_tpid : 0;
		o << " [ tpacketv3 VLAN Prio (";
		o.u((tci & 0xe000u) >> 13) << "), CFI (";
		o.u((tci & 0x1000u) >> 12) << "), ID (";
		o.u(tci & 0x0fffu) << "), Proto (0x";
		o.xn(tpid, 4) << ") ]\n";
	}
}

void format_frame_hdr(std::string &s, const nsd_frame_hdr_t &fh, const nsd_sll_t *sll, const uint8_t *pkt,
		      uint32_t caplen, int linktype, int mode, uint64_t count)
{
	Out o(s);
	frame_hdr(o, fh, sll, pkt, caplen, linktype, mode, count);
}

int render_packet_cpu(std::string &text, const uint8_t *packet, size_t len, int linktype, int mode,
		      const nsd_sll_t *sll);

// The replay's formatter job (netsniff-ng.c:732-737 per record): packets
// [lo, hi) of a batch, show_frame_hdr then the entry point's text, into s
// through one sink.  A record that could not hold its chain (NSD_F_OVERFLOW:
// more than NSD_EXT_MAX_LAYERS layers, or the ext pool was full) is rendered
// by the per-packet path, which has no layer budget; any other status is an
// error.
int format_replay_part(std::string &s, const uint8_t *frames, const nsd_desc_t *desc, const nsd_frame_hdr_t *fh,
		       const nsd_sll_t *sll, const nsd_crec *rec, const uint32_t *ext, uint64_t count0, uint32_t lo,
		       uint32_t hi, int linktype, int mode)
{
	Out o(s);
	for (uint32_t k = lo; k < hi; k++) {
		const uint64_t d = desc[k];
		const uint8_t *const pkt = frames + NSD_DESC_OFF(d);
		const uint32_t caplen = (uint32_t)NSD_DESC_CAPLEN(d);
		frame_hdr(o, fh[k], sll + k, pkt, caplen, linktype, mode, count0 + k);
		const size_t mark = o.size();
		const int r = packet_compact(o, pkt, caplen, linktype, mode, rec[k], k, ext, sll + k);
		if (r == NSD_OK)
			continue;
		if (!(rec[k].nflags & NSD_F_OVERFLOW))
			return NSD_ERR_FORMAT;
		o.cut(mark);
		const int r2 = render_packet_cpu(s, pkt, caplen, linktype, mode, sll + k);
		if (r2 != NSD_OK)
			return r2;
	}
	return NSD_OK;
}

} // namespace nsd

extern "C" long nsd_format_frame_hdr(const nsd_frame_hdr_t *fh, const nsd_sll_t *sll, const uint8_t *pkt,
				     uint32_t caplen, int linktype, int mode, uint64_t count, char *out, size_t cap)
{
	if (!fh || (!pkt && caplen))
		return NSD_ERR_ARG;
	std::string s;
	nsd::format_frame_hdr(s, *fh, sll, pkt, caplen, linktype, mode, count);
	if (out && cap) {
		const size_t k = s.size() < cap - 1 ? s.size() : cap - 1;
		memcpy(out, s.data(), k);
		out[k] = 0;
	}
	return (long)s.size();
}

extern "C" long nsd_format_packet(const uint8_t *pkt, uint32_t caplen, int linktype, int mode,
				  const nsd_rec *rec, const uint32_t *ext_pool, char *out, size_t cap)
{
	return nsd_format_packet_sll(pkt, caplen, linktype, mode, rec, ext_pool, nullptr, out, cap);
}

extern "C" long nsd_format_packet_sll(const uint8_t *pkt, uint32_t caplen, int linktype, int mode,
				      const nsd_rec *rec, const uint32_t *ext_pool, const nsd_sll_t *sll,
				      char *out, size_t cap)
{
	if (!pkt && caplen)
		return NSD_ERR_ARG;
	if (!rec)
		return NSD_ERR_ARG;
	std::string s;
	s.reserve(256 + 6 * (size_t)caplen);
	int rc = nsd::format_packet(s, pkt, caplen, linktype, mode, *rec, ext_pool, sll);
	if (out && cap) {
		size_t k = s.size() < cap - 1 ? s.size() : cap - 1;
		memcpy(out, s.data(), k);
		out[k] = 0;
	}
	if (rc != NSD_OK)
		return rc;
	return (long)s.size();
}

// Batch formatter: renders packets [0, n) into one buffer; per-packet end
// offsets in ends[] (so callers can split), status per packet in rc[] (may be
// NULL).  Returns total bytes, or -needed when cap is too small.
extern "C" long nsd_format_batch_sll(const uint8_t *frames, const nsd_desc_t *desc,
				     const nsd_sll_t *sll, uint32_t n, int linktype, int mode,
				     const nsd_rec *rec, const uint32_t *ext_pool, char *out, size_t cap,
				     uint64_t *ends, int8_t *rc);

extern "C" long nsd_format_batch(const uint8_t *frames, const nsd_desc_t *desc, uint32_t n,
				 int linktype, int mode, const nsd_rec *rec, const uint32_t *ext_pool,
				 char *out, size_t cap, uint64_t *ends, int8_t *rc)
{
	return nsd_format_batch_sll(frames, desc, nullptr, n, linktype, mode, rec, ext_pool, out, cap, ends, rc);
}

// same, with one sockaddr_ll per packet (SLL link types; may be NULL)
extern "C" long nsd_format_batch_sll(const uint8_t *frames, const nsd_desc_t *desc,
				     const nsd_sll_t *sll, uint32_t n, int linktype, int mode,
				     const nsd_rec *rec, const uint32_t *ext_pool, char *out, size_t cap,
				     uint64_t *ends, int8_t *rc)
{
	std::string s;
	s.reserve(cap ? cap : 4096);
	for (uint32_t i = 0; i < n; i++) {
		const uint64_t d = desc[i];
		int r = nsd::format_packet(s, frames + NSD_DESC_OFF(d), NSD_DESC_CAPLEN(d), linktype,
					   mode, rec[i], ext_pool, sll ? sll + i : nullptr);
		if (rc)
			rc[i] = (int8_t)r;
		if (ends)
			ends[i] = s.size();
	}
	if (s.size() > cap)
		return -(long)s.size();
	memcpy(out, s.data(), s.size());
	return (long)s.size();
}

extern "C" long nsd_format_batch_compact(const uint8_t *frames, const nsd_desc_t *desc, const nsd_sll_t *sll,
					 uint32_t n, int linktype, int mode, const nsd_crec *crec,
					 const uint32_t *ext_pool, char *out, size_t cap, uint64_t *ends,
					 int8_t *rc)
{
	return nsd_format_range_compact(frames, desc, sll, 0, n, linktype, mode, crec, ext_pool, out, cap, ends, rc);
}

extern "C" long nsd_format_range_compact(const uint8_t *frames, const nsd_desc_t *desc, const nsd_sll_t *sll,
					 uint32_t lo, uint32_t hi, int linktype, int mode, const nsd_crec *crec,
					 const uint32_t *ext_pool, char *out, size_t cap, uint64_t *ends, int8_t *rc)
{
	return nsd_format_range_compact_fh(frames, desc, sll, nullptr, 0, lo, hi, linktype, mode, crec, ext_pool, out,
					   cap, ends, rc);
}

extern "C" long nsd_format_range_compact_fh(const uint8_t *frames, const nsd_desc_t *desc, const nsd_sll_t *sll,
					    const nsd_frame_hdr_t *fh, uint64_t first_count, uint32_t lo, uint32_t hi,
					    int linktype, int mode, const nsd_crec *crec, const uint32_t *ext_pool,
					    char *out, size_t cap, uint64_t *ends, int8_t *rc)
{
	if (hi < lo || (hi > lo && (!frames || !desc || !crec)))
		return NSD_ERR_ARG;
	// a per-thread buffer that keeps its capacity across calls (reserving
	// `cap` per call faulted in fresh pages every time: threads formatting
	// ranges in parallel then queued on the process's page-table lock);
	// given back when it grew far past what this call needed
	static thread_local std::string t_buf;
	std::string &s = t_buf;
	s.clear();
	{
		nsd::Out o(s);
		for (uint32_t i = lo; i < hi; i++) {
			const uint64_t d = desc[i];
			const uint8_t *pkt = frames + NSD_DESC_OFF(d);
			if (fh)
				nsd::frame_hdr(o, fh[i], sll ? sll + i : nullptr, pkt, NSD_DESC_CAPLEN(d), linktype, mode,
					       first_count + i);
			int r = nsd::packet_compact(o, pkt, NSD_DESC_CAPLEN(d), linktype, mode, crec[i], i, ext_pool,
						    sll ? sll + i : nullptr);
			if (rc)
				rc[i - lo] = (int8_t)r;
			if (ends)
				ends[i - lo] = o.size();
		}
	}
	const long total = (long)s.size();
	if (s.size() <= cap)
		memcpy(out, s.data(), s.size());
	if (s.capacity() > ((size_t)64 << 20) && s.capacity() > 4 * s.size())
		std::string().swap(s);
	return total <= (long)cap ? total : -total;
}
