// nsd_proto.cpp - the reference's per-packet surface: dissector_init_all /
// dissector_entry_point / dissector_cleanup_all / dissector_set_print_type
// (dissector.h:118-122, dissector.c:22-138) over proto-ops objects with the
// reference's names, keys and layout (protos.h:6-31, proto.h:18-33,
// pkt_buff.h:15-24).
//
// dissector_entry_point runs the reference's own control flow: a pkt_buff
// over the frame, the link type's start / exit ops, dissector_main's loop
// (`for (d = start; d; ) d->process(pkt)`), then the post-chain dump of
// PRINT_HEX / ASCII / HEX_ASCII and tprintf_flush.  Each Ethernet-chain
// ops' process() is one layer of this library: nsd::cpu_step (gen_step of
// nsd_walk.h, the layer step the device's general walk runs) decides the
// cursor and the next ops, nsd::render_layer (nsd_format.cpp, the renderer
// the batch path's records go through) prints the layer, and the two are
// required to agree on where the layer ends (bug_on, like pkt_buff.h's
// invariants).  It runs on the host CPU: SURVEY 8b keeps the per-packet
// entry there (a launch per packet would be all latency); batches of frames
// go to the device through the batch extension.
//
// The 802.11 and netlink heads stay the reference's objects
// (dissector_80211.o / proto_80211_mac_hdr.o, dissector_netlink.o /
// proto_nlmsg.o): when linked, their ops and initialisers are found through
// weak references and run inside the same loop, with this library's
// none_ops as their exit.
#include <arpa/inet.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ioctl.h>
#include <unistd.h>

#include <string>

#include "../../include/netsniff_dissect.h"
#include "nsd_lookup.h"

namespace nsd {
bool render_layer(std::string &s, const uint8_t *pkt, uint32_t caplen, int id, uint32_t start, uint32_t tail,
		  int mode, uint16_t ip_csum, bool icmp_bad, const nsd_sll_t *sll, uint32_t &data,
		  uint32_t &ntail, bool &next);
void render_hex(std::string &s, const uint8_t *pkt, uint32_t caplen, uint32_t from, uint32_t len);
void render_ascii(std::string &s, const uint8_t *pkt, uint32_t caplen, uint32_t from, uint32_t len);
int cpu_step(int mode, const uint8_t *pkt, uint32_t caplen, int id, uint32_t &data, uint32_t &tail,
	     uint16_t &ip_csum, uint8_t &flags, const nsd_sll_t *sll);
int render_packet_cpu(std::string &text, const uint8_t *packet, size_t len, int linktype, int mode,
		      const nsd_sll_t *sll);
}

extern "C" __attribute__((visibility("hidden"))) void nsd_device_ctx_release(void);
extern "C" __attribute__((visibility("hidden"))) void nsd_replay_release(void);
extern "C" __attribute__((visibility("hidden"))) void nsd_if_cache_reset(void);

#ifndef NSD_ETCDIRE
#define NSD_ETCDIRE "/etc/netsniff-ng"
#endif

// ---- output: the executable's tprintf when it has one (netsniff-ng links
// tprintf.o), else stdout through the wrap emulation ------------------------
extern "C" {
void tprintf(char *msg, ...) __attribute__((weak));
void tprintf_flush(void) __attribute__((weak));
}

namespace {

std::string g_out;          // text of the current packet when there is no tprintf
long g_line_count = 0;      // __tprintf_flush's line counter for that case
thread_local std::string *t_capture = nullptr;   // render_packet_cpu's sink

int tty_cols()
{
	struct winsize ts;
	return ioctl(0, TIOCGWINSZ, &ts) == 0 ? ts.ws_col : 80;   // DEFAULT_TTY_SIZE
}

// one piece of text, as one or more tprintf calls: the reference's buffer is
// 1 KiB and panics on a single call longer than that (tprintf.c:126-162).
// A NUL byte (a "%c" of packet data, e.g. proto_icmpv6.c:563) goes in as
// its own "%c" call: "%.*s" would stop at it
void out(const char *p, size_t n)
{
	if (!n)
		return;
	if (t_capture) {
		t_capture->append(p, n);
		return;
	}
	if (tprintf) {
		for (size_t i = 0; i < n;) {
			if (!p[i]) {
				tprintf((char *)"%c", 0);
				i++;
				continue;
			}
			size_t k = strnlen(p + i, n - i < 256 ? n - i : 256);
			tprintf((char *)"%.*s", (int)k, p + i);
			i += k;
		}
		return;
	}
	g_out.append(p, n);
}

void out(const std::string &s) { out(s.data(), s.size()); }

void flush()
{
	if (tprintf_flush) {
		tprintf_flush();
		return;
	}
	if (g_out.empty())
		return;
	std::string w(2 * g_out.size() + 16, '\0');
	const long k = nsd_tprintf_wrap(g_out.data(), g_out.size(), tty_cols(), &g_line_count, &w[0], w.size());
	if (k > 0)
		fwrite(w.data(), 1, (size_t)k, stdout);
	fflush(stdout);
	g_out.clear();
}

// the frame dissector_entry_point is walking: bytes at offsets >= caplen read
// as zero (the parity domain; the IPv4 checksum and trailer read past tail)
struct FrameCtx {
	const uint8_t *head = nullptr;
	uint32_t caplen = 0;
};
thread_local FrameCtx t_frame;

[[noreturn]] void bug(const char *what, int id)
{
	fprintf(stderr, "netsniff-dissect: BUG: %s (ops %d)\n", what, id);
	abort();   // bug_on() (built_in.h:174)
}

} // namespace

// ---- proto.h:28-33: the exit op's dumps -----------------------------------
namespace {

size_t pkt_len(const struct pkt_buff *pkt) { return (size_t)(pkt->tail - pkt->data); }

void hex_bytes(const uint8_t *ptr, size_t len)
{
	std::string s;
	nsd::render_hex(s, ptr, (uint32_t)len, 0, (uint32_t)len);
	out(s);
}

void ascii_bytes(const uint8_t *ptr, size_t len)
{
	std::string s;
	nsd::render_ascii(s, ptr, (uint32_t)len, 0, (uint32_t)len);
	out(s);
}

// proto_none.c:30-38
void hex_impl(struct pkt_buff *pkt)
{
	const size_t len = pkt_len(pkt);
	if (!len)
		return;
	const uint8_t *p = pkt->data;
	pkt->data += len;
	hex_bytes(p, len);
	out("\n", 1);
}

// proto_none.c:50-58
void ascii_impl(struct pkt_buff *pkt)
{
	const size_t len = pkt_len(pkt);
	if (!len)
		return;
	const uint8_t *p = pkt->data;
	pkt->data += len;
	ascii_bytes(p, len);
	out("\n", 1);
}

// proto_none.c:61-72
void hex_ascii_impl(struct pkt_buff *pkt)
{
	const size_t len = pkt_len(pkt);
	const uint8_t *p = pkt->data;
	pkt->data += len;
	if (len) {
		ascii_bytes(p, len);
		hex_bytes(p, len);
	}
	out("\n", 1);
}

// proto_none.c:74-77
void none_less(struct pkt_buff *) { out("\n", 1); }

} // namespace

extern "C" void empty(struct pkt_buff *) {}
extern "C" void _hex(uint8_t *ptr, size_t len) { if (ptr) hex_bytes(ptr, len); }
extern "C" void hex(struct pkt_buff *pkt) { hex_impl(pkt); }
extern "C" void _ascii(uint8_t *ptr, size_t len) { if (ptr) ascii_bytes(ptr, len); }
extern "C" void ascii(struct pkt_buff *pkt) { ascii_impl(pkt); }
extern "C" void hex_ascii(struct pkt_buff *pkt) { hex_ascii_impl(pkt); }

// ---- the ops objects -------------------------------------------------------
namespace {
struct protocol *ops_of(int id);

// ops `id`'s process() in `mode`: one layer at the pkt_buff cursor.  A walk
// and renderer that disagree are a bug: process() aborts (the reference's
// bug_on), render_packet_cpu (strict false) gets false back and reports it
bool run_layer(struct pkt_buff *pkt, int id, int mode, bool strict = true)
{
	const uint8_t *head = pkt->head;
	const uint32_t caplen = t_frame.head == head ? t_frame.caplen : (uint32_t)(pkt->tail - head);
	const uint32_t start = (uint32_t)(pkt->data - head), tail = (uint32_t)(pkt->tail - head);
	nsd_sll_t ll;
	const nsd_sll_t *sll = nullptr;
	if (pkt->sll) {
		memcpy(&ll, pkt->sll, sizeof(ll));   // struct sockaddr_ll: the same 20 bytes
		sll = &ll;
	}
	uint32_t data = start, ntail = tail;
	uint16_t csum = 0;
	uint8_t flags = 0;
	const int next = nsd::cpu_step(mode, head, caplen, id, data, ntail, csum, flags, sll);
	std::string s;
	uint32_t rdata, rtail;
	bool rnext;
	if (!nsd::render_layer(s, head, caplen, id, start, tail, mode, csum, flags & NSD_F_ICMP_BAD, sll, rdata,
			       rtail, rnext)) {
		if (!strict)
			return false;
		bug("layer cannot be rendered", id);
	}
	if (rdata != data || rtail != ntail || rnext != (next != 0)) {
		if (!strict)
			return false;
		bug("walk and renderer disagree on the layer's end", id);
	}
	out(s);
	pkt->data = pkt->head + data;
	pkt->tail = pkt->head + ntail;
	if (next)
		pkt->dissector = ops_of(next);   // pkt_set_dissector (pkt_buff.h:102-110)
	return true;
}

template <int ID>
void print_full(struct pkt_buff *pkt) { run_layer(pkt, ID, PRINT_NORM); }
template <int ID>
void print_less(struct pkt_buff *pkt) { run_layer(pkt, ID, PRINT_LESS); }

} // namespace

#define NSD_OPS_OBJECT(name, key, id) \
	extern "C" struct protocol name = { key, print_full<id>, print_less<id>, nullptr, nullptr };

// keys as in each proto_*.c's ops definition (identity is the ops
// object, several share a key)
NSD_OPS_OBJECT(ethernet_ops, 0, NSD_OPS_ETHERNET)                  // proto_ethernet.c:99
NSD_OPS_OBJECT(vlan_ops, 0x8100, NSD_OPS_VLAN)                     // proto_vlan.c:57
NSD_OPS_OBJECT(QinQ_ops, 0x88a8, NSD_OPS_QINQ)                     // proto_vlan_q_in_q.c:58
NSD_OPS_OBJECT(mpls_uc_ops, 0x8847, NSD_OPS_MPLS_UC)               // proto_mpls_unicast.c:104
NSD_OPS_OBJECT(arp_ops, 0x0806, NSD_OPS_ARP)                       // proto_arp.c:198
NSD_OPS_OBJECT(lldp_ops, 0x88cc, NSD_OPS_LLDP)                     // proto_lldp.c:490
NSD_OPS_OBJECT(ipv4_ops, 0x0800, NSD_OPS_IPV4)                     // proto_ipv4.c:206
NSD_OPS_OBJECT(ipv6_ops, 0x86DD, NSD_OPS_IPV6)                     // proto_ipv6.c:115
NSD_OPS_OBJECT(ipv6_in_ipv4_ops, 0x29, NSD_OPS_IPV6_IN_IPV4)       // proto_ipv6_in_ipv4.c:20
NSD_OPS_OBJECT(icmpv4_ops, 0x01, NSD_OPS_ICMPV4)                   // proto_icmpv4.c:63
NSD_OPS_OBJECT(icmpv6_ops, 0x3A, NSD_OPS_ICMPV6)                   // proto_icmpv6.c:1701
NSD_OPS_OBJECT(igmp_ops, 0x02, NSD_OPS_IGMP)                       // proto_igmp.c:556
NSD_OPS_OBJECT(ip_auth_ops, 0x33, NSD_OPS_IP_AUTH)                 // proto_ip_authentication_hdr.c:90
NSD_OPS_OBJECT(ip_esp_ops, 0x32, NSD_OPS_IP_ESP)                   // proto_ip_esp.c:48
NSD_OPS_OBJECT(ipv6_dest_opts_ops, 0x3C, NSD_OPS_IPV6_DEST_OPTS)   // proto_ipv6_dest_opts.c:97
NSD_OPS_OBJECT(ipv6_fragm_ops, 0x2C, NSD_OPS_IPV6_FRAGM)           // proto_ipv6_fragm.c:65
NSD_OPS_OBJECT(ipv6_hop_by_hop_ops, 0x00, NSD_OPS_IPV6_HOP_BY_HOP) // proto_ipv6_hop_by_hop.c:96
NSD_OPS_OBJECT(ipv6_mobility_ops, 0x87, NSD_OPS_IPV6_MOBILITY)     // proto_ipv6_mobility_hdr.c:311
NSD_OPS_OBJECT(ipv6_no_next_header_ops, 0x3B, NSD_OPS_IPV6_NO_NEXT) // proto_ipv6_no_nxt_hdr.c:36
NSD_OPS_OBJECT(ipv6_routing_ops, 0x2B, NSD_OPS_IPV6_ROUTING)       // proto_ipv6_routing.c:158
NSD_OPS_OBJECT(tcp_ops, 0x06, NSD_OPS_TCP)                         // proto_tcp.c:153
NSD_OPS_OBJECT(udp_ops, 0x11, NSD_OPS_UDP)                         // proto_udp.c:85
NSD_OPS_OBJECT(dccp_ops, 0x21, NSD_OPS_DCCP)                       // proto_dccp.c:150
NSD_OPS_OBJECT(sll_ops, 0, NSD_OPS_SLL)                            // dissector_sll.c:84

// proto_none.c:79-83
extern "C" struct protocol none_ops = { 0x01, hex_ascii_impl, none_less, nullptr, nullptr };

// the reference objects this library does not replace (weak: present when
// netsniff-ng links them, as it does by default)
extern "C" {
extern struct protocol ieee80211_ops __attribute__((weak));   // proto_80211_mac_hdr.c:3269
extern struct protocol nlmsg_ops __attribute__((weak));       // proto_nlmsg.c:1058
void dissector_init_ieee80211(int fnttype) __attribute__((weak));
void dissector_cleanup_ieee80211(void) __attribute__((weak));
void dissector_init_netlink(int fnttype) __attribute__((weak));
void dissector_cleanup_netlink(void) __attribute__((weak));
}

namespace {

struct protocol *ops_of(int id)
{
	switch (id) {
	case NSD_OPS_ETHERNET: return &ethernet_ops;
	case NSD_OPS_VLAN: return &vlan_ops;
	case NSD_OPS_QINQ: return &QinQ_ops;
	case NSD_OPS_MPLS_UC: return &mpls_uc_ops;
	case NSD_OPS_ARP: return &arp_ops;
	case NSD_OPS_LLDP: return &lldp_ops;
	case NSD_OPS_IPV4: return &ipv4_ops;
	case NSD_OPS_IPV6: return &ipv6_ops;
	case NSD_OPS_IPV6_IN_IPV4: return &ipv6_in_ipv4_ops;
	case NSD_OPS_ICMPV4: return &icmpv4_ops;
	case NSD_OPS_ICMPV6: return &icmpv6_ops;
	case NSD_OPS_IGMP: return &igmp_ops;
	case NSD_OPS_IP_AUTH: return &ip_auth_ops;
	case NSD_OPS_IP_ESP: return &ip_esp_ops;
	case NSD_OPS_IPV6_DEST_OPTS: return &ipv6_dest_opts_ops;
	case NSD_OPS_IPV6_FRAGM: return &ipv6_fragm_ops;
	case NSD_OPS_IPV6_HOP_BY_HOP: return &ipv6_hop_by_hop_ops;
	case NSD_OPS_IPV6_MOBILITY: return &ipv6_mobility_ops;
	case NSD_OPS_IPV6_NO_NEXT: return &ipv6_no_next_header_ops;
	case NSD_OPS_IPV6_ROUTING: return &ipv6_routing_ops;
	case NSD_OPS_TCP: return &tcp_ops;
	case NSD_OPS_UDP: return &udp_ops;
	case NSD_OPS_DCCP: return &dccp_ops;
	case NSD_OPS_SLL: return &sll_ops;
	case NSD_OPS_NLMSG: return &nlmsg_ops;            // NULL unless linked: the chain ends
	case NSD_OPS_IEEE80211: return &ieee80211_ops;
	}
	return nullptr;
}

bool is_lt(int lt, uint32_t v) { return (uint32_t)lt == v || (uint32_t)lt == __builtin_bswap32(v); }

// the ops id of one of this library's ops objects, 0 for others
int id_of(const struct protocol *p)
{
	for (int id = 1; id < NSD_OPS_COUNT; id++)
		if (id != NSD_OPS_NLMSG && id != NSD_OPS_IEEE80211 && ops_of(id) == p)
			return id;
	return 0;
}

// start / exit ops per link type (dissector.c:75-104; byte-swapped link
// types match too, :79)
void start_end(int linktype, struct protocol *&start, struct protocol *&end)
{
	end = &none_ops;
	if (is_lt(linktype, NSD_LINKTYPE_EN10MB)) {
		start = &ethernet_ops;
	} else if (is_lt(linktype, NSD_LINKTYPE_IEEE802_11_RADIOTAP) || is_lt(linktype, NSD_LINKTYPE_IEEE802_11)) {
		start = &ieee80211_ops;
	} else if (is_lt(linktype, NSD_LINKTYPE_NETLINK)) {
		start = &nlmsg_ops;
	} else if (is_lt(linktype, NSD_LINKTYPE_LINUX_SLL)) {
		start = &sll_ops;
	} else {
		start = &none_ops;
		end = nullptr;
	}
}

std::string g_etcdir = NSD_ETCDIRE;

} // namespace

// ---- dissector.c ---------------------------------------------------------
extern "C" int dissector_set_print_type(void *ptr, int type)
{
	for (struct protocol *p = (struct protocol *)ptr; p; p = p->next) {
		switch (type) {
		case PRINT_NORM: p->process = p->print_full; break;
		case PRINT_LESS: p->process = p->print_less; break;
		default: p->process = nullptr; break;
		}
	}
	return 0;
}

extern "C" void nsd_set_etcdir(const char *dir) { g_etcdir = dir ? dir : NSD_ETCDIRE; }

// dissector.c:124-130: dissector_init_ethernet (entry, eth_lay2, eth_lay3 and
// exit ops, dissector_eth.c:64-75, + the four name tables), the 802.11 and
// netlink initialisers, dissector_init_sll (dissector_sll.c:100-105)
extern "C" void dissector_init_all(int fnttype)
{
	static const int eth_chain[] = {
		NSD_OPS_ETHERNET, NSD_OPS_ARP, NSD_OPS_LLDP, NSD_OPS_VLAN, NSD_OPS_IPV4, NSD_OPS_IPV6,
		NSD_OPS_QINQ, NSD_OPS_MPLS_UC, NSD_OPS_ICMPV4, NSD_OPS_ICMPV6, NSD_OPS_IGMP, NSD_OPS_IP_AUTH,
		NSD_OPS_IP_ESP, NSD_OPS_IPV6_DEST_OPTS, NSD_OPS_IPV6_FRAGM, NSD_OPS_IPV6_HOP_BY_HOP,
		NSD_OPS_IPV6_IN_IPV4, NSD_OPS_IPV6_MOBILITY, NSD_OPS_IPV6_NO_NEXT, NSD_OPS_IPV6_ROUTING,
		NSD_OPS_TCP, NSD_OPS_UDP, NSD_OPS_DCCP,
	};
	for (int id : eth_chain)
		dissector_set_print_type(ops_of(id), fnttype);
	dissector_set_print_type(&none_ops, fnttype);
	nsd::lookup_init_reporting(g_etcdir.c_str());
	if (dissector_init_ieee80211)
		dissector_init_ieee80211(fnttype);
	if (dissector_init_netlink)
		dissector_init_netlink(fnttype);
	dissector_set_print_type(&sll_ops, fnttype);
	dissector_set_print_type(&none_ops, fnttype);
}

// dissector.c:132-138
extern "C" void dissector_cleanup_all(void)
{
	nsd_lookup_cleanup();
	if (dissector_cleanup_ieee80211)
		dissector_cleanup_ieee80211();
	if (dissector_cleanup_netlink)
		dissector_cleanup_netlink();
	nsd_device_ctx_release();
	nsd_replay_release();
	nsd_if_cache_reset();
}

// dissector.c:43-62
static void dissector_main(struct pkt_buff *pkt, struct protocol *start, struct protocol *end)
{
	if (!start)
		return;
	for (pkt->dissector = start; pkt->dissector;) {
		if (!pkt->dissector->process)
			break;
		struct protocol *d = pkt->dissector;
		pkt->dissector = nullptr;
		d->process(pkt);
	}
	if (end && end->process)
		end->process(pkt);
}

// dissector.c:64-122
extern "C" void dissector_entry_point(uint8_t *packet, size_t len, int linktype, int mode,
				      struct sockaddr_ll *sll)
{
	if (mode == PRINT_NONE)
		return;
	struct pkt_buff pkt;
	pkt.head = packet;
	pkt.data = packet;
	pkt.tail = packet + len;
	pkt.dissector = nullptr;
	pkt.link_type = (uint32_t)linktype;
	pkt.sll = sll;
	t_frame.head = packet;
	t_frame.caplen = (uint32_t)len;

	struct protocol *start, *end;
	start_end(linktype, start, end);
	dissector_main(&pkt, start, end);

	switch (mode) {
	case PRINT_HEX: hex_impl(&pkt); break;
	case PRINT_ASCII: ascii_impl(&pkt); break;
	case PRINT_HEX_ASCII: hex_ascii_impl(&pkt); break;
	}
	flush();
	t_frame.head = nullptr;
}

// One packet's text as dissector_entry_point prints it when every ops object
// is set to `mode` (dissector_init_all(mode) + dissector_entry_point(...,
// mode, ...), as read_pcap calls them), appended to out instead of going to
// tprintf.  The pcap replay uses it for the records a batch cannot carry: a
// frame above NSD_MAX_CAPLEN, or a chain the record and its ext pool could
// not hold (NSD_F_OVERFLOW).  It depends on no global print type: this
// library's ops run their layer in `mode`, none_ops as the start op (an
// unknown link type, dissector.c:100-103) prints what its process() would in
// `mode` (hex_ascii / none_less, proto_none.c:61-83).  The reference's own
// 802.11 / netlink objects print through tprintf, outside this text: a chain
// that reaches one returns NSD_ERR_UNSUPPORTED, and a walk / renderer
// disagreement NSD_ERR_FORMAT (the text so far stays in `text`).
int nsd::render_packet_cpu(std::string &text, const uint8_t *packet, size_t len, int linktype, int mode,
			   const nsd_sll_t *sll)
{
	if (mode == PRINT_NONE)
		return NSD_OK;
	struct sockaddr_ll *ll = (struct sockaddr_ll *)sll;
	struct pkt_buff pkt;
	pkt.head = (uint8_t *)packet;
	pkt.data = (uint8_t *)packet;
	pkt.tail = (uint8_t *)packet + len;
	pkt.dissector = nullptr;
	pkt.link_type = (uint32_t)linktype;
	pkt.sll = ll;
	const FrameCtx saved = t_frame;
	std::string *const saved_cap = t_capture;
	t_frame.head = packet;
	t_frame.caplen = (uint32_t)len;
	t_capture = &text;
	int rc = NSD_OK;
	struct protocol *start, *end;
	start_end(linktype, start, end);
	if (mode == PRINT_NORM || mode == PRINT_LESS) {
		for (pkt.dissector = start; pkt.dissector;) {
			struct protocol *d = pkt.dissector;
			pkt.dissector = nullptr;
			const int id = id_of(d);
			if (id) {
				if (!run_layer(&pkt, id, mode, false)) {
					rc = NSD_ERR_FORMAT;
					break;
				}
			} else if (d == &none_ops) {
				(mode == PRINT_NORM ? hex_ascii_impl : none_less)(&pkt);
			} else {
				rc = NSD_ERR_UNSUPPORTED;
				break;
			}
		}
		if (rc == NSD_OK && end == &none_ops)
			(mode == PRINT_NORM ? hex_ascii_impl : none_less)(&pkt);
	}
	if (rc == NSD_OK) {
		switch (mode) {
		case PRINT_HEX: hex_impl(&pkt); break;
		case PRINT_ASCII: ascii_impl(&pkt); break;
		case PRINT_HEX_ASCII: hex_ascii_impl(&pkt); break;
		}
	}
	t_capture = saved_cap;
	t_frame = saved;
	return rc;
}
