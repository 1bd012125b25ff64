// nsd_format_sll.h - host renderer of the LINKTYPE_LINUX_SLL head
// (dissector_sll.c:39-82) over the packet's struct sockaddr_ll.  Included by
// nsd_format.cpp after its Out / Frame / Layer / Done helpers.
//
// dissector_sll.c includes dissector.h -> ring.h -> the configure-generated
// config.h and is unbuildable here, so this text is pinned by the CPU
// restatement (oracle/nsd_oracle.c); the name tables it prints
// (device_type2str, device_addr2str, dev.c:252-422) compile from the
// reference and pin the tables (tests/test_sll.py).

#include <net/if_arp.h>
// newer ARPHRD values glibc's net/if_arp.h lacks (linux/if_arp.h)
#ifndef ARPHRD_PHONET
#define ARPHRD_PHONET 820
#endif
#ifndef ARPHRD_PHONET_PIPE
#define ARPHRD_PHONET_PIPE 821
#endif
#ifndef ARPHRD_CAIF
#define ARPHRD_CAIF 822
#endif
#ifndef ARPHRD_IP6GRE
#define ARPHRD_IP6GRE 823
#endif
#ifndef ARPHRD_NETLINK
#define ARPHRD_NETLINK 824
#endif

// pkt_type2str (dissector_sll.c:17-37)
static const char *sll_pkt_type(uint8_t t)
{
	switch (t) {
	case 0: return "host";
	case 1: return "broadcast";
	case 2: return "multicast";
	case 3: return "other host";
	case 4: return "outgoing";
	case 6: return "user";
	case 7: return "kernel";
	}
	return "Unknown";
}

// device_type2str (dev.c:252-402)
static const char *sll_dev_type(uint16_t type)
{
	switch (type) {
	case ARPHRD_ETHER: return "ether";
	case ARPHRD_EETHER: return "eether";
	case ARPHRD_AX25: return "ax25";
	case ARPHRD_PRONET: return "pronet";
	case ARPHRD_CHAOS: return "chaos";
	case ARPHRD_IEEE802: return "ieee802";
	case ARPHRD_ARCNET: return "arcnet";
	case ARPHRD_APPLETLK: return "appletlk";
	case ARPHRD_DLCI: return "dlci";
	case ARPHRD_ATM: return "atm";
	case ARPHRD_METRICOM: return "metricom";
	case ARPHRD_IEEE1394: return "ieee1394";
	case ARPHRD_INFINIBAND: return "infiniband";
	case ARPHRD_SLIP: return "slip";
	case ARPHRD_CSLIP: return "cslip";
	case ARPHRD_SLIP6: return "slip6";
	case ARPHRD_CSLIP6: return "cslip6";
	case ARPHRD_RSRVD: return "RSRVD";
	case ARPHRD_ADAPT: return "adapt";
	case ARPHRD_ROSE: return "rose";
	case ARPHRD_X25: return "x25";
	case ARPHRD_HWX25: return "hwx25";
	case ARPHRD_CAN: return "can";
	case ARPHRD_PPP: return "ppp";
	case ARPHRD_HDLC: return "hdlc";
	case ARPHRD_LAPB: return "lapb";
	case ARPHRD_DDCMP: return "ddcmp";
	case ARPHRD_RAWHDLC: return "rawhdlc";
	case ARPHRD_TUNNEL: return "tunnel";
	case ARPHRD_TUNNEL6: return "tunnel6";
	case ARPHRD_FRAD: return "frad";
	case ARPHRD_SKIP: return "skip";
	case ARPHRD_LOOPBACK: return "loopback";
	case ARPHRD_LOCALTLK: return "localtlk";
	case ARPHRD_FDDI: return "fddi";
	case ARPHRD_BIF: return "bif";
	case ARPHRD_SIT: return "sit";
	case ARPHRD_IPDDP: return "ipddp";
	case ARPHRD_IPGRE: return "ipgre";
	case ARPHRD_PIMREG: return "pimreg";
	case ARPHRD_HIPPI: return "hippi";
	case ARPHRD_ASH: return "ash";
	case ARPHRD_ECONET: return "econet";
	case ARPHRD_IRDA: return "irda";
	case ARPHRD_FCPP: return "fcpp";
	case ARPHRD_FCAL: return "fcal";
	case ARPHRD_FCPL: return "fcpl";
	case ARPHRD_IEEE802_TR: return "ieee802_tr";
	case ARPHRD_IEEE80211: return "ieee80211";
	case ARPHRD_IEEE80211_PRISM: return "ieee80211_prism";
	case ARPHRD_IEEE80211_RADIOTAP: return "ieee80211_radiotap";
	case ARPHRD_IEEE802154: return "ieee802154";
	case ARPHRD_PHONET: return "phonet";
	case ARPHRD_PHONET_PIPE: return "phonet_pipe";
	case ARPHRD_CAIF: return "caif";
	case ARPHRD_IP6GRE: return "ip6gre";
	case ARPHRD_NETLINK: return "netlink";
	case ARPHRD_NONE: return "none";
	case ARPHRD_VOID: return "void";
	}
	if (type >= ARPHRD_FCFABRIC && type <= ARPHRD_FCFABRIC + 12) {
		static const char *const fc[] = { "fcfb0", "fcfb1", "fcfb2", "fcfb3", "fcfb4", "fcfb5", "fcfb6",
						  "fcfb7", "fcfb8", "fcfb9", "fcfb10", "fcfb11", "fcfb12" };
		return fc[type - ARPHRD_FCFABRIC];
	}
	return "Unknown";
}

// device_addr2str (dev.c:405-422) into a 40-byte buffer (sll_print_full's
// addr_str): "%02x" then ":%02x" while the written length stays below 40,
// the last piece cut by snprintf.  Address bytes past sll_addr[8] (the
// reference reads on past the struct for halen > 8 and for TUNNEL6's 16
// bytes) read as zero, as everywhere outside the parity domain.
static void sll_dev_addr(Out &o, const uint8_t *addr8, int alen, int type)
{
	uint8_t a[256] = {};
	memcpy(a, addr8, 8);
	char buf[64];
	if (alen == 4 && (type == ARPHRD_TUNNEL || type == ARPHRD_SIT || type == ARPHRD_IPGRE)) {
		inet_ntop(AF_INET, a, buf, 40);
		o << buf;
		return;
	}
	if (alen == 16 && type == ARPHRD_TUNNEL6) {
		inet_ntop(AF_INET6, a, buf, 40);
		o << buf;
		return;
	}
	static const char hx[] = "0123456789abcdef";
	std::string t;
	t.push_back(hx[a[0] >> 4]);
	t.push_back(hx[a[0] & 15]);
	for (int i = 1, l = 2; i < alen && l < 40; i++, l += 3) {
		t.push_back(':');
		t.push_back(hx[a[i] >> 4]);
		t.push_back(hx[a[i] & 15]);
	}
	if (t.size() > 39)
		t.resize(39);
	o << t.c_str();
}

// pcap_devtype_to_linktype (pcap_io.h:205-267), the two classes the head
// dispatches on: 1 = LINKTYPE_EN10MB, 2 = LINKTYPE_NETLINK, 0 = other
static int sll_link_class(uint16_t hatype)
{
	switch (hatype) {
	case ARPHRD_TUNNEL: case ARPHRD_TUNNEL6: case ARPHRD_LOOPBACK: case ARPHRD_SIT:
	case ARPHRD_IPDDP: case ARPHRD_IPGRE: case ARPHRD_IP6GRE: case ARPHRD_ETHER:
		return 1;
	case ARPHRD_NETLINK:
		return 2;
	}
	return 0;
}

// sll_print_full / sll_print_less (dissector_sll.c:39-82); pulls nothing
static Done r_sll(Out &o, const Layer &L, int mode, const nsd_sll_t *sll)
{
	nsd_sll_t z;
	memset(&z, 0, sizeof(z));
	const nsd_sll_t &s = sll ? *sll : z;
	const uint16_t proto = (uint16_t)((s.protocol >> 8) | (s.protocol << 8));
	if (mode == PRINT_NORM)
		o << " [ Linux \"cooked\"";
	o << " Pkt Type ";
	o.u(s.pkttype) << " (" << sll_pkt_type(s.pkttype) << ")";
	o << ", If Type ";
	o.u(s.hatype) << " (" << sll_dev_type(s.hatype) << ")";
	o << ", Addr Len ";
	o.u(s.halen) << ", Src (";
	sll_dev_addr(o, s.addr, s.halen, s.hatype);
	o << "), Proto 0x";
	o.x(proto);
	if (mode != PRINT_NORM)
		return { L.start, L.tail, false, true };
	o << " ]\n";
	const int cls = sll_link_class(s.hatype);
	if (cls == 0)
		o << " [ Unknown protocol ]\n";
	const bool next = (cls == 1 && lay2_has(proto)) || cls == 2;
	return { L.start, L.tail, next, true };
}
