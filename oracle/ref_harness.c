/*
 * ref_harness.c - drives the REFERENCE's own parser objects (compiled from
 * /root/reference by oracle/Makefile ("make ref") into oracle/_ref/) over a pcap and
 * prints through the reference's real tprintf.c.  TEST INFRASTRUCTURE ONLY.
 *
 * What comes from the reference (object files built from its sources as they
 * lie): every proto_*.c parser except proto_ipv4.c / proto_ipv6.c, hash.c,
 * lookup.c, tprintf.c, xmalloc.c, str.c, die.c, and the inline pkt_buff.h /
 * hash.h helpers.
 *
 * What this file supplies, and why:
 *   - the chain loop and entry point, restating dissector.c:43-122 for the
 *     Ethernet link type (dissector.c itself includes ring.h -> config.h);
 *   - the eth_lay2 / eth_lay3 tables, built with the reference's own
 *     insert_hash / INSERT_HASH_PROTOS in dissector_eth.c:30-62 order
 *     (dissector_eth.c includes dissector.h -> ring.h -> config.h);
 *   - dissector_set_print_type, restating dissector.c:22-41;
 *   - ipv4_ops / ipv6_ops / ipv6() / ipv6_less(): proto_ipv4.c and
 *     proto_ipv6.c include geoip.h -> config.h, a configure-generated header
 *     this image cannot produce (configure needs pkg-config).  Those layers
 *     therefore run the oracle restatement (nsd_oracle.c) and are NOT pinned
 *     by this harness.
 *
 *   - the LINKTYPE_LINUX_SLL head (-f / -F only), restating
 *     dissector_sll.c:17-63 (dissector.h -> ring.h -> config.h) over the
 *     reference's own device_type2str / device_addr2str (dev.c) and
 *     pcap_devtype_to_linktype (pcap_io.h, included as it lies);
 *   - show_frame_hdr / __show_frame_hdr (dissector.h:31-116, same reason),
 *     restated below and fed by the reference's own pcap code.
 *
 * With -f / -F the record loop is read_pcap's (netsniff-ng.c:659-737) over
 * the REFERENCE's pcap objects: pcap_rw_ops (pcap_rw.c, the `-c` reader:
 * pcap_generic_pull_fhdr -> pcap_validate_header incl. the *_LL remap,
 * pcap_rw_read), pcap_get_length and pcap_pkthdr_to_tpacket_hdr
 * (pcap_io.h:322-347, 594-709) into a zeroed struct frame_map, the packet
 * counter, then show_frame_hdr and the dissector.  (The default reader, SG,
 * reads the same records for files below its 12 MiB of iovecs.)
 *
 * Usage: nsref [-m mode] [-n] [-w cols] [-i index_out] [-f|-F] file.pcap
 *   -w 0    : stdin from /dev/null -> tprintf wraps at DEFAULT_TTY_SIZE (80)
 *   -w N>0  : stdin is a pty N columns wide (N=65535: effectively unwrapped)
 *   -i F    : write one u64 stdout byte offset per packet boundary to F
 *   -f      : `netsniff-ng --in file.pcap`: frame header line + dissector
 *   -F      : frame header lines only (no dissector; any link type)
 * Without -f / -F every record (zero-length ones too) goes to the entry
 * point alone, the per-packet surface the entry-point tests pin.
 * Bytes past caplen are zero (parity domain).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ioctl.h>
#include <termios.h>
#include <unistd.h>
#include <arpa/inet.h>

#include "hash.h"
#include "proto.h"
#include "protos.h"
#include "pkt_buff.h"
#include "tprintf.h"
#include "lookup.h"

#include "pcap_io.h"

#include "nsd_oracle.h"

/* as dissector.h:29 declares it (net/if.h and linux/if.h do not mix) */
extern char *if_indextoname(unsigned ifindex, char *ifname);

/* dev.c (compiles from the reference as it lies): the tables the SLL head
 * prints through (dissector_sll.c:48-51) */
const char *device_type2str(uint16_t type);
const char *device_addr2str(const unsigned char *addr, int alen, int type, char *buf, int blen);

/* -T: dump device_type2str for every hatype that has a name, and
 * device_addr2str for a fixed 8-byte address at every (alen, type) the
 * formatter distinguishes, into a 40-byte buffer as sll_print_full does */
static int dump_dev_tables(void)
{
	static const unsigned char addr[32] = { 0xde, 0xad, 0xbe, 0xef, 0x01, 0x02, 0x03, 0x04 };
	static const int types[] = { 1, 768, 769, 776, 778, 772, 824, 0 };
	char buf[40];
	for (unsigned t = 0; t < 65536; t++) {
		const char *s = device_type2str((uint16_t)t);
		if (strcmp(s, "Unknown"))
			printf("T %u %s\n", t, s);
	}
	for (size_t k = 0; k < sizeof(types) / sizeof(types[0]); k++)
		for (int alen = 0; alen <= 8; alen++) {
			memset(buf, 0, sizeof(buf));
			printf("A %d %d %s\n", types[k], alen, device_addr2str(addr, alen, types[k], buf, sizeof(buf)));
		}
	return 0;
}

struct hash_table eth_lay2;
struct hash_table eth_lay3;

static int g_mode;
static uint32_t g_caplen;
static struct protocol sll_ops_h;   /* the SLL head, below */

/* dissector.c:22-41 */
int dissector_set_print_type(void *ptr, int type)
{
	struct protocol *proto;

	for (proto = ptr; proto; proto = proto->next) {
		switch (type) {
		case PRINT_NORM: proto->process = proto->print_full; break;
		case PRINT_LESS: proto->process = proto->print_less; break;
		default:         proto->process = NULL; break;
		}
	}
	return 0;
}

/* ---- IPv4 / IPv6 via the restatement (see header comment) --------------- */
static void emit_tprintf(void *ctx, const char *s, size_t n)
{
	(void)ctx;
	/* tprintf's 1 KiB buffer: hand over in pieces well below it */
	while (n) {
		size_t k = n > 256 ? 256 : n;
		tprintf("%.*s", (int)k, s);
		s += k;
		n -= k;
	}
}

static void run_oracle_layer(struct pkt_buff *pkt, int ops_id)
{
	uint32_t data = pkt->data - pkt->head, tail = pkt->tail - pkt->head;
	int next = nsor_run_layer(ops_id, g_mode, pkt->head, g_caplen, &data, &tail,
				  emit_tprintf, NULL);
	pkt->data = pkt->head + data;
	pkt->tail = pkt->head + tail;
	if (next) {
		/* map back to the key the reference would have looked up */
		unsigned key = 0;
		struct hash_table *tab = &eth_lay3;
		switch (next) {
		case NSD_OPS_ICMPV4: key = 1; break;
		case NSD_OPS_ICMPV6: key = 58; break;
		case NSD_OPS_IGMP: key = 2; break;
		case NSD_OPS_IP_AUTH: key = 51; break;
		case NSD_OPS_IP_ESP: key = 50; break;
		case NSD_OPS_IPV6_DEST_OPTS: key = 60; break;
		case NSD_OPS_IPV6_FRAGM: key = 44; break;
		case NSD_OPS_IPV6_HOP_BY_HOP: key = 0; break;
		case NSD_OPS_IPV6_IN_IPV4: key = 41; break;
		case NSD_OPS_IPV6_MOBILITY: key = 135; break;
		case NSD_OPS_IPV6_NO_NEXT: key = 59; break;
		case NSD_OPS_IPV6_ROUTING: key = 43; break;
		case NSD_OPS_TCP: key = 6; break;
		case NSD_OPS_UDP: key = 17; break;
		case NSD_OPS_DCCP: key = 33; break;
		default: tab = NULL;
		}
		if (tab)
			pkt_set_dissector(pkt, tab, key);
	}
}

static void h_ipv4(struct pkt_buff *pkt) { run_oracle_layer(pkt, NSD_OPS_IPV4); }
void ipv6(struct pkt_buff *pkt) { run_oracle_layer(pkt, NSD_OPS_IPV6); }
void ipv6_less(struct pkt_buff *pkt) { run_oracle_layer(pkt, NSD_OPS_IPV6); }

struct protocol ipv4_ops = { .key = 0x0800, .print_full = h_ipv4, .print_less = h_ipv4 };
struct protocol ipv6_ops = { .key = 0x86DD, .print_full = ipv6, .print_less = ipv6_less };

/* ---- tables: dissector_eth.c:30-62 -------------------------------------- */
static void init_tables(int type)
{
	dissector_set_print_type(&ethernet_ops, type);
	init_hash(&eth_lay2);
	INSERT_HASH_PROTOS(arp_ops, eth_lay2);
	INSERT_HASH_PROTOS(lldp_ops, eth_lay2);
	INSERT_HASH_PROTOS(vlan_ops, eth_lay2);
	INSERT_HASH_PROTOS(ipv4_ops, eth_lay2);
	INSERT_HASH_PROTOS(ipv6_ops, eth_lay2);
	INSERT_HASH_PROTOS(QinQ_ops, eth_lay2);
	INSERT_HASH_PROTOS(mpls_uc_ops, eth_lay2);
	for_each_hash_int(&eth_lay2, dissector_set_print_type, type);

	init_hash(&eth_lay3);
	INSERT_HASH_PROTOS(icmpv4_ops, eth_lay3);
	INSERT_HASH_PROTOS(icmpv6_ops, eth_lay3);
	INSERT_HASH_PROTOS(igmp_ops, eth_lay3);
	INSERT_HASH_PROTOS(ip_auth_ops, eth_lay3);
	INSERT_HASH_PROTOS(ip_esp_ops, eth_lay3);
	INSERT_HASH_PROTOS(ipv6_dest_opts_ops, eth_lay3);
	INSERT_HASH_PROTOS(ipv6_fragm_ops, eth_lay3);
	INSERT_HASH_PROTOS(ipv6_hop_by_hop_ops, eth_lay3);
	INSERT_HASH_PROTOS(ipv6_in_ipv4_ops, eth_lay3);
	INSERT_HASH_PROTOS(ipv6_mobility_ops, eth_lay3);
	INSERT_HASH_PROTOS(ipv6_no_next_header_ops, eth_lay3);
	INSERT_HASH_PROTOS(ipv6_routing_ops, eth_lay3);
	INSERT_HASH_PROTOS(tcp_ops, eth_lay3);
	INSERT_HASH_PROTOS(udp_ops, eth_lay3);
	INSERT_HASH_PROTOS(dccp_ops, eth_lay3);
	for_each_hash_int(&eth_lay3, dissector_set_print_type, type);

	dissector_set_print_type(&none_ops, type);
	dissector_set_print_type(&sll_ops_h, type);
}

/* ---- chain loop + entry: dissector.c:43-122 (Ethernet link type) -------- */
static void dissector_main(struct pkt_buff *pkt, struct protocol *start, struct protocol *end)
{
	struct protocol *d;

	if (!start)
		return;
	for (pkt->dissector = start; pkt->dissector; ) {
		if (!pkt->dissector->process)
			break;
		d = pkt->dissector;
		pkt->dissector = NULL;
		d->process(pkt);
	}
	if (end && end->process)
		end->process(pkt);
}

/* ---- LINKTYPE_LINUX_SLL head: dissector_sll.c:17-63 --------------------- */
static char *pkt_type2str(uint8_t pkttype)
{
	switch (pkttype) {
	case PACKET_HOST: return "host";
	case PACKET_BROADCAST: return "broadcast";
	case PACKET_MULTICAST: return "multicast";
	case PACKET_OTHERHOST: return "other host";
	case PACKET_OUTGOING: return "outgoing";
	case PACKET_USER: return "user";
	case PACKET_KERNEL: return "kernel";
	}
	return "Unknown";
}

static int g_sll_unsupported;

static void sll_print_full(struct pkt_buff *pkt)
{
	struct sockaddr_ll *sll = pkt->sll;
	char addr_str[40] = {};

	tprintf(" [ Linux \"cooked\"");
	tprintf(" Pkt Type %d (%s)", sll->sll_pkttype, pkt_type2str(sll->sll_pkttype));
	tprintf(", If Type %d (%s)", sll->sll_hatype, device_type2str(sll->sll_hatype));
	tprintf(", Addr Len %d", sll->sll_halen);
	tprintf(", Src (%s)", device_addr2str(sll->sll_addr, sll->sll_halen, sll->sll_hatype,
					       addr_str, sizeof(addr_str)));
	tprintf(", Proto 0x%x", ntohs(sll->sll_protocol));
	tprintf(" ]\n");
	switch (pcap_devtype_to_linktype(sll->sll_hatype)) {
	case LINKTYPE_EN10MB:
		pkt_set_dissector(pkt, &eth_lay2, ntohs(sll->sll_protocol));
		break;
	case LINKTYPE_NETLINK:
		g_sll_unsupported = 1;   /* dissector_netlink (libnl, config.h): not built here */
		break;
	default:
		tprintf(" [ Unknown protocol ]\n");
	}
}

static void sll_print_less(struct pkt_buff *pkt)
{
	struct sockaddr_ll *sll = pkt->sll;
	char addr_str[40] = {};

	tprintf(" Pkt Type %d (%s)", sll->sll_pkttype, pkt_type2str(sll->sll_pkttype));
	tprintf(", If Type %d (%s)", sll->sll_hatype, device_type2str(sll->sll_hatype));
	tprintf(", Addr Len %d", sll->sll_halen);
	tprintf(", Src (%s)", device_addr2str(sll->sll_addr, sll->sll_halen, sll->sll_hatype,
					       addr_str, sizeof(addr_str)));
	tprintf(", Proto 0x%x", ntohs(sll->sll_protocol));
}

static struct protocol sll_ops_h = { .key = 0, .print_full = sll_print_full, .print_less = sll_print_less };

static void entry(uint8_t *packet, size_t len, int linktype, int mode, struct sockaddr_ll *sll)
{
	struct pkt_buff *pkt;

	if (mode == PRINT_NONE)
		return;
	pkt = pkt_alloc(packet, len);
	pkt->link_type = linktype;
	pkt->sll = sll;
	if (linktype == 1 || (uint32_t)linktype == 0x01000000u)
		dissector_main(pkt, &ethernet_ops, &none_ops);
	else if (sll && (linktype == LINKTYPE_LINUX_SLL || (uint32_t)linktype == 0x71000000u))
		dissector_main(pkt, &sll_ops_h, &none_ops);
	else
		dissector_main(pkt, &none_ops, NULL);
	switch (mode) {
	case PRINT_HEX: hex(pkt); break;
	case PRINT_ASCII: ascii(pkt); break;
	case PRINT_HEX_ASCII: hex_ascii(pkt); break;
	}
	tprintf_flush();
	pkt_free(pkt);
}

static int setup_stdin(int cols)
{
	int fd;

	if (cols <= 0) {
		fd = open("/dev/null", O_RDONLY);
	} else {
		struct winsize ws = { .ws_row = 24, .ws_col = (unsigned short)cols };
		int m = posix_openpt(O_RDWR | O_NOCTTY);
		if (m < 0 || grantpt(m) || unlockpt(m))
			return -1;
		fd = open(ptsname(m), O_RDWR | O_NOCTTY);
		if (fd < 0 || ioctl(fd, TIOCSWINSZ, &ws))
			return -1;
	}
	if (fd < 0 || dup2(fd, 0) < 0)
		return -1;
	return 0;
}

static uint32_t sw32(uint32_t v, int swap) { return swap ? __builtin_bswap32(v) : v; }

/* ---- show_frame_hdr: dissector.h:31-116 (+ ring.h:34-84 helpers) ----------
 * Only the TPACKET_V2 form read_pcap uses (v3 false, raw_hdr = the zeroed
 * frame_map's tp_h).  ring.h is built with HAVE_TPACKET3 (configure:334-360
 * finds it on any kernel with tpacket_v3), so tpacket_has_vlan_info reads
 * the status through the tpacket3_hdr view of this tpacket2_hdr
 * (tpacket_uhdr(*hdr, tp_status, true), ring.h:83): offset 20, which in a
 * tpacket2_hdr is tp_nsec; the VLAN tci / tpid helpers return 0 for v2. */
static const char *const packet_types[256] = {
	[PACKET_HOST] = "<", [PACKET_BROADCAST] = "B", [PACKET_MULTICAST] = "M",
	[PACKET_OTHERHOST] = "P", [PACKET_OUTGOING] = ">", [PACKET_USER] = "K->U",
	[PACKET_KERNEL] = "U->K",
};

static const char *show_ts_source(uint32_t status)
{
	if (status & TP_STATUS_TS_RAW_HARDWARE)
		return "(raw hw ts)";
	else if (status & TP_STATUS_TS_SYS_HARDWARE)
		return "(sys hw ts)";
	else if (status & TP_STATUS_TS_SOFTWARE)
		return "(sw ts)";
	return "";
}

static void show_frame_hdr_v2(uint8_t *packet, size_t len, int linktype, struct sockaddr_ll *s_ll,
			      struct tpacket2_hdr *h2, int mode, unsigned long count)
{
	char tmp[IFNAMSIZ];
	uint8_t pkttype = s_ll->sll_pkttype;
	const char *ifn;
	uint32_t st3;

	if (mode == PRINT_NONE)
		return;
	if (linktype == LINKTYPE_NETLINK && len >= 16 && pkttype == PACKET_OUTGOING) {
		uint32_t pid;
		memcpy(&pid, packet + 12, 4);   /* struct nlmsghdr.nlmsg_pid */
		pkttype = pid == 0 ? PACKET_KERNEL : PACKET_USER;
	}
	ifn = if_indextoname(s_ll->sll_ifindex, tmp);
	switch (mode) {
	case PRINT_LESS:
		tprintf("%s %s %u #%lu", packet_types[pkttype] ? : "?", ifn ? : "?", h2->tp_len, count);
		break;
	default:
		tprintf("%s %s %u %us.%uns #%lu %s\n", packet_types[pkttype] ? : "?", ifn ? : "?",
			h2->tp_len, h2->tp_sec, h2->tp_nsec, count, show_ts_source(h2->tp_status));
		st3 = ((struct tpacket3_hdr *)(void *)h2)->tp_status;
		if (st3 & (TP_STATUS_VLAN_VALID | TP_STATUS_VLAN_TPID_VALID)) {
			uint16_t tci = 0;
			tprintf(" [ tpacketv3 VLAN ");
			tprintf("Prio (%u), ", (tci & 0xe000) >> 13);
			tprintf("CFI (%u), ", (tci & 0x1000) >> 12);
			tprintf("ID (%u), ", tci & 0x0fff);
			tprintf("Proto (0x%.4x)", 0);
			tprintf(" ]\n");
		}
		break;
	}
}

/* struct frame_map (ring.h:86-89; ring.h needs config.h) */
struct frame_map {
	struct tpacket2_hdr tp_h;
	struct sockaddr_ll s_ll;
};

/* read_pcap's loop (netsniff-ng.c:659-737) over the reference's RW reader */
static int replay(const char *path, int mode, int frames_only, FILE *fi)
{
	const struct pcap_file_ops *io = &pcap_rw_ops;
	uint32_t magic, link_type;
	unsigned long count = 0;
	pcap_pkthdr_t phdr;
	struct frame_map fm;
	size_t out_len = 1 << 20, hw = 0;
	uint8_t *out;
	int fd, ret;

	fd = open(path, O_RDONLY);
	if (fd < 0)
		return 1;
	if (io->pull_fhdr_pcap(fd, &magic, &link_type))
		return 1;
	memset(&fm, 0, sizeof(fm));
	out = calloc(1, out_len + 4096);
	for (;;) {
		uint32_t caplen;
		uint64_t pos;

		ret = io->read_pcap(fd, &phdr, magic, out, out_len);
		if (ret < 0)
			break;
		caplen = pcap_get_length(&phdr, magic);
		if (caplen == 0)
			continue;   /* unreachable: the reader returns -EINVAL first */
		/* parity domain: bytes past caplen read as zero */
		if (hw > caplen)
			memset(out + caplen, 0, hw - caplen);
		hw = caplen;
		pcap_pkthdr_to_tpacket_hdr(&phdr, magic, &fm.tp_h, &fm.s_ll);
		count++;
		show_frame_hdr_v2(out, fm.tp_h.tp_snaplen, link_type, &fm.s_ll, &fm.tp_h, mode, count);
		if (!frames_only) {
			g_caplen = fm.tp_h.tp_snaplen;
			entry(out, fm.tp_h.tp_snaplen, (int)link_type, mode, &fm.s_ll);
			if (g_sll_unsupported)
				return 3;
		} else {
			tprintf_flush();
		}
		if (fi) {
			fflush(stdout);
			pos = (uint64_t)ftello(stdout);
			fwrite(&pos, 8, 1, fi);
		}
	}
	fflush(stdout);
	close(fd);
	free(out);
	return 0;
}

int main(int argc, char **argv)
{
	int opt, cols = 0, names = 0, fh_mode = 0;
	const char *index_out = NULL;
	FILE *f, *fi = NULL;
	uint32_t fh[6];
	int swap;
	uint8_t *buf;
	static char outbuf[1 << 20];

	g_mode = PRINT_NORM;
	if (argc > 1 && !strcmp(argv[1], "-T"))
		return dump_dev_tables();
	while ((opt = getopt(argc, argv, "m:nw:i:fF")) != -1) {
		switch (opt) {
		case 'f': fh_mode = 1; break;
		case 'F': fh_mode = 2; break;
		case 'm': g_mode = atoi(optarg); break;
		case 'n': names = 1; break;
		case 'w': cols = atoi(optarg); break;
		case 'i': index_out = optarg; break;
		default:
			fprintf(stderr, "usage: %s [-m mode] [-n] [-w cols] [-i idx] file.pcap\n", argv[0]);
			return 2;
		}
	}
	if (optind >= argc)
		return 2;
	if (setup_stdin(cols)) {
		fprintf(stderr, "stdin setup failed: %s\n", strerror(errno));
		return 1;
	}
	/* tprintf_init initialises the buffer spinlock and makes stdout
	 * unbuffered (tprintf.c:112-118); re-buffer stdout before any output:
	 * the bytes are the same, only faster */
	tprintf_init();
	setvbuf(stdout, outbuf, _IOFBF, sizeof(outbuf));
	if (names) {
		lookup_init(LT_PORTS_UDP);
		lookup_init(LT_PORTS_TCP);
		lookup_init(LT_ETHERTYPES);
		lookup_init(LT_OUI);
	}
	init_tables(g_mode);

	if (fh_mode) {
		int rc;
		if (index_out)
			fi = fopen(index_out, "wb");
		rc = replay(argv[optind], g_mode, fh_mode == 2, fi);
		if (fi)
			fclose(fi);
		return rc;
	}

	f = fopen(argv[optind], "rb");
	if (!f || fread(fh, 4, 6, f) != 6) {
		fprintf(stderr, "cannot read %s\n", argv[optind]);
		return 1;
	}
	swap = fh[0] == 0xd4c3b2a1u || fh[0] == 0x4d3cb2a1u;
	if (index_out)
		fi = fopen(index_out, "wb");
	/* read_pcap's reused 1 MiB `out` buffer (netsniff-ng.c:680-681) */
	buf = calloc(1, (1 << 20) + 4096);
	for (;;) {
		uint32_t rh[4], caplen;
		uint64_t pos;
		if (fread(rh, 4, 4, f) != 4)
			break;
		caplen = sw32(rh[2], swap);
		if (caplen > (1 << 20))
			return 1;
		memset(buf, 0, caplen + 4096);
		if (fread(buf, 1, caplen, f) != caplen)
			break;
		g_caplen = caplen;
		entry(buf, caplen, (int)sw32(fh[5], swap), g_mode, NULL);
		if (fi) {
			fflush(stdout);
			pos = (uint64_t)ftello(stdout);
			fwrite(&pos, 8, 1, fi);
		}
	}
	fflush(stdout);
	if (fi)
		fclose(fi);
	fclose(f);
	return 0;
}
