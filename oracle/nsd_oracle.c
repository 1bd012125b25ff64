/*
 * nsd_oracle.c - CPU restatement of netsniff-ng's per-packet dissector chain.
 *
 * TEST INFRASTRUCTURE ONLY (see nsd_oracle.h): the checker for the HIP path,
 * and the "port" CPU baseline timed by bench.py.  Never linked by the product.
 *
 * Restates, function by function:
 *   pkt_buff cursor ops ............. pkt_buff.h:50-100
 *   dispatch tables ................. dissector_eth.c:30-62 (+ hash.c exact-key lookup)
 *   chain loop / entry point ........ dissector.c:43-122
 *   parsers ......................... proto_*.c (cited per function below)
 *   name tables ..................... lookup.c:33-158
 * Bytes at offsets >= caplen read as zero (the parity domain).
 */
#define _GNU_SOURCE
#include "nsd_oracle.h"

#include <arpa/inet.h>
#include <ctype.h>
#include <inttypes.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* text sink                                                                */
/* ------------------------------------------------------------------------ */
void nsor_text_init(nsor_text *t) { memset(t, 0, sizeof(*t)); }
void nsor_text_free(nsor_text *t) { free(t->buf); memset(t, 0, sizeof(*t)); }
void nsor_text_reset(nsor_text *t) { t->len = 0; t->unsupported = 0; if (t->buf) t->buf[0] = 0; }

static void text_append(nsor_text *t, const char *s, size_t n)
{
	if (t->len + n + 1 > t->cap) {
		size_t nc = t->cap ? t->cap : 4096;
		while (t->len + n + 1 > nc)
			nc *= 2;
		t->buf = realloc(t->buf, nc);
		if (!t->buf)
			abort();
		t->cap = nc;
	}
	memcpy(t->buf + t->len, s, n);
	t->len += n;
	t->buf[t->len] = 0;
}

/* colours (colors.h:26-28) */
#define C_BOLD   "\033[1m"
#define C_RED    "\033[30;41m"
#define C_END    "\033[0m"

/* ------------------------------------------------------------------------ */
/* walk state = struct pkt_buff (pkt_buff.h:15-24) as offsets               */
/* ------------------------------------------------------------------------ */
typedef struct P {
	const uint8_t *p;
	uint32_t caplen;
	uint32_t data, tail;
	int      mode;
	/* outputs */
	uint16_t ip_csum;
	int      icmp_bad;
	int      host;
	uint32_t extent;          /* furthest checksum byte (for W) */
	/* text */
	nsor_text   *t;
	nsor_emit_fn emit;
	void        *ectx;
} P;

static inline int texting(const P *k) { return k->t || k->emit; }

static void E(P *k, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
static void E(P *k, const char *fmt, ...)
{
	char tmp[512];
	va_list vl;
	int n;

	if (!texting(k))
		return;
	va_start(vl, fmt);
	n = vsnprintf(tmp, sizeof(tmp), fmt, vl);
	va_end(vl);
	if (n < 0)
		abort();
	if ((size_t)n >= sizeof(tmp)) {
		char *big = malloc(n + 1);
		va_start(vl, fmt);
		vsnprintf(big, n + 1, fmt, vl);
		va_end(vl);
		if (k->t) text_append(k->t, big, n);
		else k->emit(k->ectx, big, n);
		free(big);
		return;
	}
	if (k->t) text_append(k->t, tmp, n);
	else k->emit(k->ectx, tmp, n);
}

static inline uint8_t B(const P *k, uint64_t off)
{
	return off < k->caplen ? k->p[off] : 0;
}
static inline uint16_t BE16(const P *k, uint64_t o) { return (uint16_t)(B(k, o) << 8 | B(k, o + 1)); }
static inline uint16_t LE16(const P *k, uint64_t o) { return (uint16_t)(B(k, o) | B(k, o + 1) << 8); }
static inline uint32_t BE32(const P *k, uint64_t o) { return (uint32_t)BE16(k, o) << 16 | BE16(k, o + 2); }
static inline uint32_t LE32(const P *k, uint64_t o) { return (uint32_t)LE16(k, o) | (uint32_t)LE16(k, o + 2) << 16; }
static inline uint64_t BE64(const P *k, uint64_t o) { return (uint64_t)BE32(k, o) << 32 | BE32(k, o + 4); }

static inline uint32_t pkt_len(const P *k) { return k->tail - k->data; }          /* pkt_buff.h:36-41 */

/* pkt_pull (pkt_buff.h:43-57): on success *at = old data, data += len */
static inline int pull(P *k, uint32_t len, uint32_t *at)
{
	if (len <= pkt_len(k)) {
		if (at)
			*at = k->data;
		k->data += len;
		return 1;
	}
	return 0;
}

/* pkt_trim (pkt_buff.h:66-79) */
static inline void trim(P *k, uint32_t len)
{
	if (len <= pkt_len(k))
		k->tail -= len;
}

/* ------------------------------------------------------------------------ */
/* name tables: lookup.c:33-158                                             */
/* ------------------------------------------------------------------------ */
typedef struct { uint32_t id; char *s; } oui_ent;
static char   *lt_udp[65536], *lt_tcp[65536], *lt_eth[65536];
static oui_ent *lt_oui; static size_t lt_noui;

static int u64_cmp(const void *a, const void *b)
{
	uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
	return x < y ? -1 : x > y;
}

void nsor_lookup_clear(void)
{
	for (int i = 0; i < 65536; i++) {
		free(lt_udp[i]); free(lt_tcp[i]); free(lt_eth[i]);
		lt_udp[i] = lt_tcp[i] = lt_eth[i] = NULL;
	}
	for (size_t i = 0; i < lt_noui; i++)
		free(lt_oui[i].s);
	free(lt_oui);
	lt_oui = NULL;
	lt_noui = 0;
}

/* strtrim_right (str.c:75-90) */
static char *strtrim_right(char *p, char c)
{
	size_t len = strlen(p);
	while (*p && len) {
		char *end = p + len - 1;
		if (c == *end)
			*end = 0;
		else
			break;
		len = strlen(p);
	}
	return p;
}

/* one table; later lines shadow earlier ones with the same id, since
 * lookup_init prepends duplicates (lookup.c:84-88) and __lookup_inline
 * returns the first match (lookup.c:130-138). */
static int load_table(const char *path, int which)
{
	char buff[128], *ptr, *end;
	FILE *fp = fopen(path, "r");
	size_t oui_cap = 0;

	if (!fp)
		return 0;
	memset(buff, 0, sizeof(buff));
	while (fgets(buff, sizeof(buff), fp) != NULL) {
		unsigned int id;
		buff[sizeof(buff) - 1] = 0;
		ptr = buff;
		id = (unsigned int)strtol(ptr, &end, 0);
		if (id == 0 && end == ptr)
			continue;
		ptr = strstr(buff, ", ");
		if (!ptr)
			continue;
		ptr += 2;
		ptr = strtrim_right(ptr, '\n');
		ptr = strtrim_right(ptr, ' ');
		if (which < 3) {
			char **tab = which == 0 ? lt_udp : which == 1 ? lt_tcp : lt_eth;
			if (id < 65536) {
				free(tab[id]);
				tab[id] = strdup(ptr);
			}
		} else if (id <= 0xFFFFFF) {
			if (lt_noui == oui_cap) {
				oui_cap = oui_cap ? 2 * oui_cap : 1024;
				lt_oui = realloc(lt_oui, oui_cap * sizeof(*lt_oui));
			}
			lt_oui[lt_noui].id = id;
			lt_oui[lt_noui].s = strdup(ptr);
			lt_noui++;
		}
		memset(buff, 0, sizeof(buff));
	}
	fclose(fp);
	if (which == 3 && lt_noui) {
		/* keep the LAST line per id: sort by (id, line index), keep last */
		uint64_t *keys = malloc(lt_noui * sizeof(uint64_t));
		oui_ent *sorted = malloc(lt_noui * sizeof(oui_ent));
		size_t m = 0;
		for (size_t i = 0; i < lt_noui; i++)
			keys[i] = ((uint64_t)lt_oui[i].id << 32) | i;
		qsort(keys, lt_noui, sizeof(uint64_t), u64_cmp);
		for (size_t i = 0; i < lt_noui; i++) {
			oui_ent e = lt_oui[keys[i] & 0xFFFFFFFFu];
			if (m && sorted[m - 1].id == e.id) {
				free(sorted[m - 1].s);
				sorted[m - 1] = e;
			} else {
				sorted[m++] = e;
			}
		}
		free(keys);
		free(lt_oui);
		lt_oui = sorted;
		lt_noui = m;
	}
	return 1;
}

int nsor_lookup_init(const char *dir)
{
	static const char *files[4] = { "udp.conf", "tcp.conf", "ether.conf", "oui.conf" };
	char path[4096];
	int n = 0;

	nsor_lookup_clear();
	if (!dir)
		return 0;
	for (int i = 0; i < 4; i++) {
		snprintf(path, sizeof(path), "%s/%s", dir, files[i]);
		n += load_table(path, i);
	}
	return n;
}

static const char *lookup_port_udp(unsigned id) { return id < 65536 ? lt_udp[id] : NULL; }
static const char *lookup_port_tcp(unsigned id) { return id < 65536 ? lt_tcp[id] : NULL; }
static const char *lookup_ether_type(unsigned id) { return id < 65536 ? lt_eth[id] : NULL; }
static const char *lookup_vendor_str(unsigned id)          /* lookup.h:17-20 */
{
	size_t lo = 0, hi = lt_noui;
	while (lo < hi) {
		size_t mid = (lo + hi) / 2;
		if (lt_oui[mid].id < id) lo = mid + 1;
		else hi = mid;
	}
	if (lo < lt_noui && lt_oui[lo].id == id)
		return lt_oui[lo].s;
	return "Unknown";
}

/* ------------------------------------------------------------------------ */
/* dispatch tables: dissector_eth.c:30-62                                   */
/* ------------------------------------------------------------------------ */
static int lay2(unsigned key)
{
	switch (key) {
	case 0x0806: return NSD_OPS_ARP;
	case 0x88cc: return NSD_OPS_LLDP;
	case 0x8100: return NSD_OPS_VLAN;
	case 0x0800: return NSD_OPS_IPV4;
	case 0x86DD: return NSD_OPS_IPV6;
	case 0x88a8: return NSD_OPS_QINQ;
	case 0x8847: return NSD_OPS_MPLS_UC;
	}
	return 0;
}

static int lay3(unsigned key)
{
	switch (key) {
	case 1:   return NSD_OPS_ICMPV4;
	case 58:  return NSD_OPS_ICMPV6;
	case 2:   return NSD_OPS_IGMP;
	case 51:  return NSD_OPS_IP_AUTH;
	case 50:  return NSD_OPS_IP_ESP;
	case 60:  return NSD_OPS_IPV6_DEST_OPTS;
	case 44:  return NSD_OPS_IPV6_FRAGM;
	case 0:   return NSD_OPS_IPV6_HOP_BY_HOP;
	case 41:  return NSD_OPS_IPV6_IN_IPV4;
	case 135: return NSD_OPS_IPV6_MOBILITY;
	case 59:  return NSD_OPS_IPV6_NO_NEXT;
	case 43:  return NSD_OPS_IPV6_ROUTING;
	case 6:   return NSD_OPS_TCP;
	case 17:  return NSD_OPS_UDP;
	case 33:  return NSD_OPS_DCCP;
	}
	return 0;
}

/* ------------------------------------------------------------------------ */
/* parsers                                                                  */
/* ------------------------------------------------------------------------ */

/* ether_lookup_addr (proto_ethernet.c:33-46) */
static const char *ether_lookup_addr(const P *k, uint32_t mac)
{
	uint8_t m0 = B(k, mac);
	if (m0 & 0x01) {
		if ((m0 & B(k, mac + 1) & B(k, mac + 2) & B(k, mac + 3) & B(k, mac + 4) &
		     B(k, mac + 5)) == 0xff)
			return "Broadcast";
		return "Multicast";
	} else if (m0 & 0x02) {
		return "Locally Administered";
	}
	return lookup_vendor_str((unsigned)m0 << 16 | (unsigned)B(k, mac + 1) << 8 | B(k, mac + 2));
}

/* ethernet / ethernet_less (proto_ethernet.c:48-97) */
static int L_ethernet(P *k)
{
	uint32_t eth;
	uint16_t proto;

	if (!pull(k, 14, &eth))
		return 0;
	proto = BE16(k, eth + 12);
	if (texting(k)) {
		uint32_t src = eth + 6, dst = eth;
		if (k->mode == PRINT_NORM) {
			const char *type = lookup_ether_type(proto);
			E(k, " [ Eth ");
			E(k, "MAC (%.2x:%.2x:%.2x:%.2x:%.2x:%.2x => ", B(k, src), B(k, src + 1),
			  B(k, src + 2), B(k, src + 3), B(k, src + 4), B(k, src + 5));
			E(k, "%.2x:%.2x:%.2x:%.2x:%.2x:%.2x), ", B(k, dst), B(k, dst + 1),
			  B(k, dst + 2), B(k, dst + 3), B(k, dst + 4), B(k, dst + 5));
			E(k, "Proto (0x%.4x", proto);
			if (type)
				E(k, ", %s%s%s", C_BOLD, type, C_END);
			E(k, ") ]\n");
			E(k, " [ Vendor ");
			E(k, "(%s => %s)", ether_lookup_addr(k, src), ether_lookup_addr(k, dst));
			E(k, " ]\n");
		} else {
			const char *type = lookup_ether_type(proto);
			E(k, " %s => %s ", ether_lookup_addr(k, src), ether_lookup_addr(k, dst));
			E(k, "%s%s%s", C_BOLD, type ? type : "(null)", C_END);
		}
	}
	return lay2(proto);
}

/* vlan / vlan_less (proto_vlan.c:22-56) */
static int L_vlan(P *k)
{
	uint32_t v;
	uint16_t tci, inner;

	if (!pull(k, 4, &v))
		return 0;
	tci = BE16(k, v);
	inner = BE16(k, v + 2);
	if (k->mode == PRINT_NORM) {
		E(k, " [ VLAN ");
		E(k, "Prio (%d), ", (tci & 0xe000) >> 13);
		E(k, "CFI (%d), ", (tci & 0x1000) >> 12);
		E(k, "ID (%d), ", tci & 0x0fff);
		E(k, "Proto (0x%.4x)", inner);
		E(k, " ]\n");
	} else {
		E(k, " VLAN%d", tci & 0x0FFF);
	}
	return lay2(inner);
}

/* QinQ_full / QinQ_less (proto_vlan_q_in_q.c:23-56) */
static int L_qinq(P *k)
{
	uint32_t v;
	uint16_t tci, tpid;

	if (!pull(k, 4, &v))
		return 0;
	tci = BE16(k, v);
	tpid = BE16(k, v + 2);
	if (k->mode == PRINT_NORM) {
		E(k, " [ VLAN QinQ ");
		E(k, "Prio (%d), ", (tci & 0xE000) >> 13);
		E(k, "DEI (%d), ", (tci & 0x1000) >> 12);
		E(k, "ID (%d), ", tci & 0x0FFF);
		E(k, "Proto (0x%.4x)", tpid);
		E(k, " ]\n");
	} else {
		E(k, " VLAN%d", tci & 0x0FFF);
	}
	return lay2(tpid);
}

/* mpls_uc_full / mpls_uc_less (proto_mpls_unicast.c:23-102) */
static int L_mpls(P *k)
{
	uint32_t m, d;
	uint8_t s;

	do {
		if (!pull(k, 4, &m))
			return 0;
		d = BE32(k, m);
		s = (d >> 8) & 1;
		if (k->mode == PRINT_NORM) {
			E(k, " [ MPLS ");
			E(k, "Label (%u), ", d >> 12);
			E(k, "Exp (%u), ", (d >> 9) & 0x7);
			E(k, "S (%u), ", s);
			E(k, "TTL (%u)", d & 0xFF);
			E(k, " ]\n");
		} else {
			E(k, " MPLS/%u", d >> 12);
		}
	} while (!s);

	/* mpls_uc_next_proto (proto_mpls_unicast.c:23-47) */
	if (!pkt_len(k))
		return 0;
	switch (B(k, k->data) >> 4) {
	case 4: return lay2(0x0800);
	case 6: return lay2(0x86DD);
	}
	return 0;
}

static void ntop4(const P *k, uint32_t off, char *buf)
{
	uint8_t a[4];
	for (int i = 0; i < 4; i++)
		a[i] = B(k, off + i);
	inet_ntop(AF_INET, a, buf, INET_ADDRSTRLEN);
}

static void ntop6(const P *k, uint32_t off, char *buf)
{
	uint8_t a[16];
	for (int i = 0; i < 16; i++)
		a[i] = B(k, off + i);
	inet_ntop(AF_INET6, a, buf, INET6_ADDRSTRLEN);
}

/* csum / calc_csum (csum.h:12-27): ~fold(sum of host-order (LE) u16 words),
 * len >> 1 words, so an odd trailing byte is dropped. */
static uint16_t calc_csum(const P *k, uint32_t off, uint64_t len)
{
	unsigned long sum = 0;
	uint64_t nwords = len >> 1;
	for (uint64_t i = 0; i < nwords; i++)
		sum += LE16(k, off + 2 * i);
	sum = (sum >> 16) + (sum & 0xffff);
	sum += (sum >> 16);
	return (uint16_t)~sum;
}

/* csum_expected (csum.h:29-39) */
static uint16_t csum_expected(uint16_t sum, uint16_t computed)
{
	uint32_t s = sum;
	s += (uint16_t)((computed >> 8) | (computed << 8));
	s = (s & 0xFFFF) + (s >> 16);
	s = (s & 0xFFFF) + (s >> 16);
	return (uint16_t)s;
}

/* ipv4 / ipv4_less (proto_ipv4.c:34-204) */
static int L_ipv4(P *k)
{
	uint32_t ip;
	uint8_t ihl, proto;
	uint16_t tot_len;

	if (!pull(k, 20, &ip))
		return 0;
	ihl = B(k, ip) & 0xF;
	tot_len = BE16(k, ip + 2);
	proto = B(k, ip + 9);

	if (k->mode != PRINT_NORM) {
		if (texting(k)) {
			char s[INET_ADDRSTRLEN], d[INET_ADDRSTRLEN];
			ntop4(k, ip + 12, s);
			ntop4(k, ip + 16, d);
			E(k, " %s/%s Len %u", s, d, tot_len);
		}
		/* pull options, no trim (proto_ipv4.c:196-202) */
		pull(k, (uint32_t)((ihl > 5 ? ihl : 5) * 4 - 20), NULL);
		return lay3(proto);
	}

	/* checksum over ihl*4 bytes, also past the captured end (quirk 1) */
	k->ip_csum = calc_csum(k, ip, (uint64_t)ihl * 4);
	{
		uint64_t ce = (uint64_t)ip + (uint64_t)ihl * 4;
		if (ce > k->caplen) ce = k->caplen;
		if (ce > k->extent) k->extent = (uint32_t)ce;
	}

	if (texting(k)) {
		char s[INET_ADDRSTRLEN], d[INET_ADDRSTRLEN];
		uint16_t frag = BE16(k, ip + 6);
		uint16_t raw_check = LE16(k, ip + 10);
		uint32_t trailer_len = 0;

		ntop4(k, ip + 12, s);
		ntop4(k, ip + 16, d);
		/* trailer (proto_ipv4.c:56-67): window ending 20 B past the tail */
		if ((uint64_t)pkt_len(k) + 20 > tot_len) {
			trailer_len = pkt_len(k) + 20 - tot_len;
		}
		if (trailer_len) {
			uint64_t trailer = (uint64_t)k->data + tot_len + trailer_len;
			E(k, " [ Eth trailer ");
			while (trailer_len--)
				E(k, "%x", B(k, trailer - trailer_len));
			E(k, " ]\n");
		}
		E(k, " [ IPv4 ");
		E(k, "Addr (%s => %s), ", s, d);
		E(k, "Proto (%u), ", proto);
		E(k, "TTL (%u), ", B(k, ip + 8));
		E(k, "TOS (%u), ", B(k, ip + 1));
		E(k, "Ver (%u), ", B(k, ip) >> 4);
		E(k, "IHL (%u), ", ihl);
		E(k, "Tlen (%u), ", tot_len);
		E(k, "ID (%u), ", BE16(k, ip + 4));
		E(k, "Res (%u), NoFrag (%u), MoreFrag (%u), FragOff (%u), ",
		  (frag & 0x8000) ? 1 : 0, (frag & 0x4000) ? 1 : 0, (frag & 0x2000) ? 1 : 0,
		  frag & 0x1fff);
		E(k, "CSum (0x%.4x) is %s", BE16(k, ip + 10),
		  k->ip_csum ? C_RED "bogus (!)" C_END : "ok");
		if (k->ip_csum)
			E(k, "%s should be 0x%.4x%s", C_RED, csum_expected(raw_check, k->ip_csum), C_END);
		E(k, " ]\n");
	}

	/* options walk (proto_ipv4.c:133-169): pull first, then print */
	{
		int64_t opts_len = (int64_t)(ihl > 5 ? ihl : 5) * 4 - 20;
		uint32_t opt;
		int ok = pull(k, (uint32_t)opts_len, &opt);
		if (ok && texting(k)) {
			uint64_t o = opt;
			for (; opts_len > 0; o++) {
				uint8_t c = B(k, o);
				E(k, "   [ Option  Copied (%u), Class (%u), Number (%u)",
				  (c & 0x80) ? 1 : 0, (c & 0x60) >> 5, c & 0x1F);
				if (c == 0x00 || c == 0x01) {
					E(k, " ]\n");
					opts_len--;
				} else {
					int64_t opt_len = B(k, ++o);
					if (opt_len < 2 || opt_len > opts_len) {
						E(k, ", Len (%" PRId64 ", invalid) ]\n", opt_len);
						break;
					}
					E(k, ", Len (%" PRId64 ") ]\n", opt_len);
					opts_len -= opt_len;
					E(k, "     [ Data hex ");
					for (opt_len -= 2; opt_len > 0; opt_len--)
						E(k, " %.2x", B(k, ++o));
					E(k, " ]\n");
				}
			}
		}
	}

	/* trim (proto_ipv4.c:174-175), evaluated in size_t: negative => no trim */
	{
		uint64_t x = (uint64_t)((int64_t)tot_len - (int64_t)ihl * 4);
		uint32_t len = pkt_len(k);
		uint64_t m = len < x ? len : x;
		trim(k, (uint32_t)(len - m));
	}
	return lay3(proto);
}

/* ipv6 / ipv6_less (proto_ipv6.c:22-113); also ipv6_in_ipv4_ops */
static int L_ipv6(P *k)
{
	uint32_t ip;
	uint8_t nh;

	if (!pull(k, 40, &ip))
		return 0;
	nh = B(k, ip + 6);
	if (texting(k)) {
		char s[INET6_ADDRSTRLEN], d[INET6_ADDRSTRLEN];
		ntop6(k, ip + 8, s);
		ntop6(k, ip + 24, d);
		if (k->mode == PRINT_NORM) {
			uint8_t b0 = B(k, ip), f0 = B(k, ip + 1), f1 = B(k, ip + 2), f2 = B(k, ip + 3);
			uint8_t tc = (uint8_t)(((b0 & 0xF) << 4) | ((f0 & 0xF0) >> 4));
			/* overlapping ORs, as written (proto_ipv6.c:38-39) */
			uint32_t flow = ((uint32_t)(f0 & 0x0F) << 8) | ((uint32_t)f1 << 4) | f2;
			E(k, " [ IPv6 ");
			E(k, "Addr (%s => %s), ", s, d);
			E(k, "Version (%u), ", b0 >> 4);
			E(k, "TrafficClass (%u), ", tc);
			E(k, "FlowLabel (%u), ", flow);
			E(k, "Len (%u), ", BE16(k, ip + 4));
			E(k, "NextHdr (%u), ", nh);
			E(k, "HopLimit (%u)", B(k, ip + 7));
			E(k, " ]\n");
		} else {
			E(k, " %s/%s Len %u", s, d, BE16(k, ip + 4));
		}
	}
	return lay3(nh);
}

/* hop_by_hop & dest_opts (proto_ipv6_hop_by_hop.c:39-94,
 * proto_ipv6_dest_opts.c:40-95): same shape, different labels */
static int L_v6opts(P *k, int dest)
{
	uint32_t h;
	uint8_t nh, hl;
	uint16_t hdr_ext_len;
	int64_t opt_len;

	if (!pull(k, 2, &h))
		return 0;
	nh = B(k, h);
	hl = B(k, h + 1);
	hdr_ext_len = (uint16_t)((hl + 1) * 8);
	opt_len = (int64_t)hdr_ext_len - 2;

	if (k->mode == PRINT_NORM) {
		E(k, dest ? "\t [ Destination Options " : "\t [ Hop-by-Hop Options ");
		E(k, "NextHdr (%u), ", nh);
		if (opt_len > (int64_t)pkt_len(k) || opt_len < 0) {
			E(k, "HdrExtLen (%u, %u Bytes, %s)", hl, hdr_ext_len, C_RED "invalid" C_END);
			return 0;
		}
		E(k, "HdrExtLen (%u, %u Bytes)", hl, hdr_ext_len);
		if (opt_len)
			E(k, ", Option(s) recognized ");
		E(k, " ]\n");
	} else {
		if (opt_len > (int64_t)pkt_len(k) || opt_len < 0)
			return 0;
		E(k, dest ? " Dest Ops" : " Hop Ops");
	}
	pull(k, (uint32_t)opt_len, NULL);
	return lay3(nh);
}

/* routing / routing_less (proto_ipv6_routing.c:33-156) */
static int L_routing(P *k)
{
	uint32_t r, tmp;
	uint8_t nh, hl, type, left;
	uint16_t hdr_ext_len;
	int64_t data_len;

	if (!pull(k, 4, &r))
		return 0;
	nh = B(k, r);
	hl = B(k, r + 1);
	type = B(k, r + 2);
	left = B(k, r + 3);
	hdr_ext_len = (uint16_t)((hl + 1) * 8);
	data_len = (int64_t)hdr_ext_len - 4;

	if (k->mode == PRINT_NORM) {
		E(k, "\t [ Routing ");
		E(k, "NextHdr (%u), ", nh);
		if (data_len > (int64_t)pkt_len(k) || data_len < 0) {
			E(k, "HdrExtLen (%u, %u Bytes %s), ", hl, hdr_ext_len, C_RED "invalid" C_END);
			return 0;
		}
		E(k, "HdrExtLen (%u, %u Bytes), ", hl, hdr_ext_len);
		E(k, "Type (%u), ", type);
		E(k, "Left (%u), ", left);
		if (type == 0) {
			/* dissect_routinghdr_type_0 (proto_ipv6_routing.c:33-65), norm */
			int ok = pull(k, 4, &tmp);
			data_len -= 4;
			if (ok && !(data_len > (int64_t)pkt_len(k) || data_len < 0)) {
				uint8_t num_addr;
				/* reserved u32 printed in host (LE) order, not ntohl (:51) */
				E(k, "Res (0x%x)", LE32(k, tmp));
				num_addr = (uint8_t)(data_len / 16);
				while (num_addr--) {
					uint32_t a;
					int aok = pull(k, 16, &a);
					data_len -= 16;
					if (!aok || data_len > (int64_t)pkt_len(k) || data_len < 0)
						break;
					if (texting(k)) {
						char s[INET6_ADDRSTRLEN];
						ntop6(k, a, s);
						E(k, "\n\t   Address: %s", s);
					}
				}
			}
		} else {
			E(k, "Type %u is unknown", type);
		}
		E(k, " ]\n");
	} else {
		if (data_len > (int64_t)pkt_len(k) || data_len < 0)
			return 0;
		E(k, " Routing ");
		if (type == 0) {
			int ok = pull(k, 4, &tmp);
			data_len -= 4;
			if (ok && !(data_len > (int64_t)pkt_len(k) || data_len < 0))
				E(k, "Addresses (%zu)", (size_t)data_len / 16);
		} else {
			E(k, "Type %u is unknown", type);
		}
	}
	if (data_len > (int64_t)pkt_len(k) || data_len < 0)
		return 0;
	pull(k, (uint32_t)data_len, NULL);
	return lay3(nh);
}

/* fragm / fragm_less (proto_ipv6_fragm.c:25-63) */
static int L_fragm(P *k)
{
	uint32_t f;
	uint16_t w;

	if (!pull(k, 8, &f))
		return 0;
	w = BE16(k, f + 2);
	if (k->mode == PRINT_NORM) {
		E(k, "\t [ Fragment ");
		E(k, "NextHdr (%u), ", B(k, f));
		E(k, "Reserved (%u), ", B(k, f + 1));
		E(k, "Offset (%u), ", w >> 3);
		E(k, "Res (%u), ", (w >> 1) & 0x3);
		E(k, "M flag (%u), ", w & 0x1);
		E(k, "Identification (%u)", BE32(k, f + 4));
		E(k, " ]\n");
	} else {
		E(k, " FragmOffs %u", w >> 3);
	}
	return lay3(B(k, f));
}

/* auth_hdr / auth_hdr_less (proto_ip_authentication_hdr.c:26-88) */
static int L_auth(P *k)
{
	uint32_t a;
	uint8_t nh, plen;

	if (!pull(k, 12, &a))
		return 0;
	nh = B(k, a);
	plen = B(k, a + 1);
	if (k->mode == PRINT_NORM) {
		uint64_t hdr_len = (uint64_t)plen * 4 + 8, i;
		E(k, " [ Authentication Header ");
		E(k, "NextHdr (%u), ", nh);
		if (hdr_len > pkt_len(k)) {
			E(k, "HdrLen (%u, %zd Bytes %s), ", plen, (ssize_t)hdr_len, C_RED "invalid" C_END);
			return 0;
		}
		E(k, "HdrLen (%u, %zd Bytes), ", plen, (ssize_t)hdr_len);
		E(k, "Reserved (0x%x), ", BE16(k, a + 2));
		E(k, "SPI (0x%x), ", BE32(k, a + 4));
		E(k, "SNF (0x%x), ", BE32(k, a + 8));
		E(k, "ICV 0x");
		for (i = 12; i < hdr_len; i++) {
			uint32_t d;
			if (!pull(k, 1, &d)) {
				E(k, "%sinvalid%s", C_RED, C_END);
				break;
			}
			E(k, "%02x", B(k, d));
		}
		E(k, " ]\n");
	} else {
		int64_t hdr_len = (int64_t)plen * 4 + 8;
		if (hdr_len > (int64_t)pkt_len(k) || hdr_len < 0)
			return 0;
		E(k, " AH");
		/* hdr_len - 12 in size_t, truncated to unsigned int by pkt_pull */
		pull(k, (uint32_t)(uint64_t)(hdr_len - 12), NULL);
	}
	return lay3(nh);
}

/* esp / esp_less (proto_ip_esp.c:23-46): leaf */
static int L_esp(P *k)
{
	uint32_t e;

	if (!pull(k, 8, &e))
		return 0;
	if (k->mode == PRINT_NORM) {
		E(k, " [ ESP ");
		E(k, "SPI (0x%x), ", BE32(k, e));
		E(k, "SN (0x%x)", BE32(k, e + 4));
		E(k, " ]\n");
	} else {
		E(k, " ESP");
	}
	return 0;
}

/* no_next_header (proto_ipv6_no_nxt_hdr.c:17-34): leaf, no pull */
static int L_nonext(P *k)
{
	if (k->mode == PRINT_NORM) {
		E(k, " [ No Next Header");
		E(k, " ]\n");
	} else {
		E(k, " No Next Header");
	}
	return 0;
}

/* mobility (proto_ipv6_mobility_hdr.c:81-309) */
static void mob_options(P *k, int64_t mdl)
{
	if (mdl)
		E(k, "MH Option(s) recognized ");
}

static int L_mobility(P *k)
{
	uint32_t m, s;
	uint8_t nh, hl, type;
	uint16_t hdr_ext_len;
	int64_t mdl;

	if (!pull(k, 6, &m))
		return 0;
	nh = B(k, m);
	hl = B(k, m + 1);
	type = B(k, m + 2);
	hdr_ext_len = (uint16_t)((hl + 1) * 8);
	mdl = (int64_t)hdr_ext_len - 6;

	if (k->mode != PRINT_NORM) {
		if (mdl > (int64_t)pkt_len(k) || mdl < 0)
			return 0;
		E(k, " Mobility Type (%u), ", type);
		pull(k, (uint32_t)mdl, NULL);
		return lay3(nh);
	}

	E(k, "\t [ Mobility ");
	E(k, "NextHdr (%u), ", nh);
	if (mdl > (int64_t)pkt_len(k) || mdl < 0) {
		E(k, "HdrExtLen (%u, %u Bytes %s), ", hl, hdr_ext_len, C_RED "invalid" C_END);
		return 0;
	}
	E(k, "HdrExtLen (%u, %u Bytes), ", hl, hdr_ext_len);
	E(k, "MH Type (%u), ", type);
	E(k, "Res (0x%x), ", B(k, m + 3));
	E(k, "Chks (0x%x), ", BE16(k, m + 4));
	E(k, "MH Data ");

	/* get_mh_type (:206-245) */
	switch (type) {
	case 0: {
		int ok;
		E(k, "Binding Refresh Request Message ");
		ok = pull(k, 2, &s);
		mdl -= 2;
		if (ok && !(mdl > (int64_t)pkt_len(k) || mdl < 0))
			mob_options(k, mdl);
		break;
	}
	case 1: case 2: {
		int ok;
		E(k, type == 1 ? "Home Test Init Message " : "Care-of Test Init Message ");
		ok = pull(k, 10, &s);
		mdl -= 10;
		if (ok && !(mdl > (int64_t)pkt_len(k) || mdl < 0)) {
			E(k, "Init Cookie (0x%" PRIx64 ")", BE64(k, s + 2));
			mob_options(k, mdl);
		}
		break;
	}
	case 3: case 4: {
		int ok;
		E(k, "Binding Refresh Request Message ");
		ok = pull(k, 18, &s);
		mdl -= 18;
		if (ok && !(mdl > (int64_t)pkt_len(k) || mdl < 0)) {
			E(k, "HN Index (%u) ", BE16(k, s));
			E(k, "Init Cookie (0x%" PRIx64 ") ", BE64(k, s + 2));
			E(k, "Keygen Token (0x%" PRIx64 ")", BE64(k, s + 10));
			mob_options(k, mdl);
		}
		break;
	}
	case 5: {
		int ok;
		E(k, "Binding Refresh Request Message ");
		ok = pull(k, 6, &s);
		mdl -= 6;
		if (ok && !(mdl > (int64_t)pkt_len(k) || mdl < 0)) {
			E(k, "Sequence (0x%x) ", BE16(k, s));
			E(k, "A|H|L|K (0x%x) ", BE16(k, s + 2) >> 12);
			E(k, "Lifetime (%us)", BE16(k, s + 4) * 4);
			mob_options(k, mdl);
		}
		break;
	}
	case 6: {
		E(k, "Binding Refresh Request Message ");
		if (!pull(k, 6, &s))
			break;
		mdl -= 6;
		if (mdl > (int64_t)pkt_len(k) || mdl < 0)
			break;
		E(k, "Status (0x%x) ", B(k, s));
		E(k, "K (%u) ", B(k, s + 1) >> 7);
		E(k, "Sequence (0x%x)", BE16(k, s + 2));
		E(k, "Lifetime (%us)", BE16(k, s + 4) * 4);
		mob_options(k, mdl);
		break;
	}
	case 7: {
		E(k, "Binding Refresh Request Message ");
		if (!pull(k, 10, &s))
			break;
		mdl -= 10;
		if (mdl > (int64_t)pkt_len(k) || mdl < 0)
			break;
		E(k, "Status (0x%x) ", B(k, s));
		/* (:194-201) inet_ntop(AF_INET6) over an 8-byte stack u64: the upper
		 * 8 bytes are stack garbage -> outside the parity domain.  Render
		 * with those 8 bytes as zero. */
		if (texting(k)) {
			uint8_t a[16] = {0};
			char buf[INET6_ADDRSTRLEN];
			uint64_t addr = BE64(k, s + 2);
			memcpy(a, &addr, 8);
			inet_ntop(AF_INET6, a, buf, sizeof(buf));
			E(k, "Home Addr (%s)", buf);
		}
		mob_options(k, mdl);
		break;
	}
	default:
		E(k, "Type %u is unknown. Error", type);
	}
	E(k, " ]\n");
	if (mdl > (int64_t)pkt_len(k) || mdl < 0)
		return 0;
	pull(k, (uint32_t)mdl, NULL);
	return lay3(nh);
}

/* tcp / tcp_less (proto_tcp.c:63-151): leaf, options not pulled */
static int L_tcp(P *k)
{
	uint32_t t;

	if (!pull(k, 20, &t))
		return 0;
	if (texting(k)) {
		uint16_t src = BE16(k, t), dst = BE16(k, t + 2);
		uint8_t b12 = B(k, t + 12), fl = B(k, t + 13);
		const char *sn = lookup_port_tcp(src), *dn = lookup_port_tcp(dst);
		static const char *names[8] = { "FIN", "SYN", "RST", "PSH", "ACK", "URG", "ECE", "CWR" };
		if (k->mode == PRINT_NORM) {
			int v = 0;
			E(k, " [ TCP ");
			E(k, "Port (%u", src);
			if (sn)
				E(k, " (%s%s%s)", C_BOLD, sn, C_END);
			E(k, " => %u", dst);
			if (dn)
				E(k, " (%s%s%s)", C_BOLD, dn, C_END);
			E(k, "), ");
			E(k, "SN (0x%x), ", BE32(k, t + 4));
			E(k, "AN (0x%x), ", BE32(k, t + 8));
			E(k, "DataOff (%u), ", b12 >> 4);
			E(k, "Res (%u), ", b12 & 0xF);
			E(k, "Flags (");
			/* tprintf_flag (proto_tcp.c:56-63) returns false for an unset
			 * flag, so the separator only follows an immediately preceding
			 * set flag: FIN..ACK + CWR prints "ACKCWR" */
			for (int i = 0; i < 8; i++) {
				int set = (fl >> i) & 1;
				if (set)
					E(k, "%s%s", v ? " " : "", names[i]);
				v = set;
			}
			E(k, "), ");
			E(k, "Window (%u), ", BE16(k, t + 14));
			E(k, "CSum (0x%.4x), ", BE16(k, t + 16));
			E(k, "UrgPtr (%u)", BE16(k, t + 18));
			E(k, " ]\n");
		} else {
			E(k, " TCP %u", src);
			if (sn)
				E(k, "(%s%s%s)", C_BOLD, sn, C_END);
			E(k, "/%u", dst);
			if (dn)
				E(k, "(%s%s%s)", C_BOLD, dn, C_END);
			E(k, " F%s", C_BOLD);
			for (int i = 0; i < 8; i++)
				if (fl & (1u << i))
					E(k, " %s", names[i]);
			E(k, "%s Win %u S/A 0x%x/0x%x", C_END, BE16(k, t + 14), BE32(k, t + 4),
			  BE32(k, t + 8));
		}
	}
	return 0;
}

/* udp / udp_less (proto_udp.c:23-83): leaf */
static int L_udp(P *k)
{
	uint32_t u;

	if (!pull(k, 8, &u))
		return 0;
	if (texting(k)) {
		uint16_t src = BE16(k, u), dst = BE16(k, u + 2), ulen = BE16(k, u + 4);
		const char *sn = lookup_port_udp(src), *dn = lookup_port_udp(dst);
		if (k->mode == PRINT_NORM) {
			int64_t len = (int64_t)ulen - 8;  /* ssize_t after size_t wrap */
			E(k, " [ UDP ");
			E(k, "Port (%u", src);
			if (sn)
				E(k, " (%s%s%s)", C_BOLD, sn, C_END);
			E(k, " => %u", dst);
			if (dn)
				E(k, " (%s%s%s)", C_BOLD, dn, C_END);
			E(k, "), ");
			if (len > (int64_t)pkt_len(k) || len < 0)
				E(k, "Len (%u) %s, ", ulen, C_RED "invalid" C_END);
			E(k, "Len (%u Bytes, %" PRId64 " Bytes Data), ", ulen, len);
			E(k, "CSum (0x%.4x)", BE16(k, u + 6));
			E(k, " ]\n");
		} else {
			E(k, " UDP %u", src);
			if (sn)
				E(k, "(%s%s%s)", C_BOLD, sn, C_END);
			E(k, "/%u", dst);
			if (dn)
				E(k, "(%s%s%s)", C_BOLD, dn, C_END);
		}
	}
	return 0;
}

/* icmp / icmp_less (proto_icmpv4.c:34-61): leaf; checksum over the whole
 * remaining (post-trim) payload, odd byte dropped */
static int L_icmp(P *k)
{
	uint32_t c;

	if (!pull(k, 8, &c))
		return 0;
	if (k->mode == PRINT_NORM) {
		uint16_t cs = calc_csum(k, c, (uint64_t)pkt_len(k) + 8);
		k->icmp_bad = cs != 0;
		if (k->tail > k->extent)
			k->extent = k->tail;
		E(k, " [ ICMP ");
		E(k, "Type (%u), ", B(k, c));
		E(k, "Code (%u), ", B(k, c + 1));
		E(k, "CSum (0x%.4x) is %s", BE16(k, c + 2), cs ? C_RED "bogus (!)" C_END : "ok");
		E(k, " ]\n");
	} else {
		E(k, " Type %u Code %u", B(k, c), B(k, c + 1));
	}
	return 0;
}

/* icmpv6 type/code strings (proto_icmpv6.c:912-1490, icmpv6_process :1492-1665) */
static const char *icmpv6_type_1_codes[] = {
	"No route to destination",
	"Communication with destination administratively prohibited",
	"Beyond scope of source address",
	"Address unreachable",
	"Port unreachable",
	"Source address failed ingress/egress policy",
	"Reject route to destination",
	"Error in Source Routing Header",
};
static const char *icmpv6_type_3_codes[] = {
	"Hop limit exceeded in transit",
	"Fragment reassembly time exceeded",
};
static const char *icmpv6_type_4_codes[] = {
	"Erroneous header field encountered",
	"Unrecognized Next Header type encountered",
	"Unrecognized IPv6 option encountered",
};
static const char *icmpv6_type_139_codes[] = {
	"Data contains IPv6 Address",
	"Data contains Name or nothing",
	"Data contains IPv4 Address",
};
static const char *icmpv6_type_140_codes[] = {
	"Successful reply",
	"Responder refuses answer",
	"Qtype is unknown to the Responder",
};
#define ASZ(a) (sizeof(a) / sizeof((a)[0]))

static const char *icmpv6_138_code(uint8_t c)
{
	switch (c) {
	case 1: return "Router Renumbering Command";
	case 2: return "Router Renumbering Result";
	case 255: return "Sequence Number Reset";
	}
	return NULL;
}
static const char *icmpv6_155_code(uint8_t c)
{
	switch (c) {
	case 0x00: return "DODAG Information Solicitation";
	case 0x01: return "DODAG Information Object";
	case 0x02: return "Destination Advertisement Object";
	case 0x03: return "Destination Advertisement Object Acknowledgment";
	case 0x80: return "Secure DODAG Information Solicitation";
	case 0x81: return "Secure DODAG Information Object";
	case 0x82: return "Secure Destination Advertisement Object";
	case 0x83: return "Secure Destination Advertisement Object Acknowledgment";
	case 0x8A: return "Consistency Check";
	}
	return NULL;
}

/* body: 0 none, 1..4 types 1-4, 128/129 echo, -1 host-rendered (130-154) */
static void icmpv6_process(uint8_t type, uint8_t code, const char **ts, const char **cs, int *body)
{
	*ts = "Unknown Type";
	*cs = "Unknown Code";
	*body = 0;
	switch (type) {
	case 1: *ts = "Destination Unreachable";
		if (code < ASZ(icmpv6_type_1_codes)) *cs = icmpv6_type_1_codes[code];
		*body = 1; return;
	case 2: *ts = "Packet Too Big"; *body = 2; return;
	case 3: *ts = "Time Exceeded";
		if (code < ASZ(icmpv6_type_3_codes)) *cs = icmpv6_type_3_codes[code];
		*body = 3; return;
	case 4: *ts = "Parameter Problem";
		if (code < ASZ(icmpv6_type_4_codes)) *cs = icmpv6_type_4_codes[code];
		*body = 4; return;
	case 100: case 101: case 200: case 201: *ts = "Private experimation"; return;
	case 127: case 255: *ts = "Reserved for expansion of ICMPv6 error messages"; return;
	case 128: *ts = "Echo Request"; *body = 128; return;
	case 129: *ts = "Echo Reply"; *body = 129; return;
	case 130: *ts = "Multicast Listener Query"; *body = -1; return;
	case 131: *ts = "Multicast Listener Report"; *body = -1; return;
	case 132: *ts = "Multicast Listener Done"; *body = -1; return;
	case 133: *ts = "Router Solicitation"; *body = -1; return;
	case 134: *ts = "Router Advertisement"; *body = -1; return;
	case 135: *ts = "Neighbor Solicitation"; *body = -1; return;
	case 136: *ts = "Neighbor Advertisement"; *body = -1; return;
	case 137: *ts = "Redirect Message"; *body = -1; return;
	case 138: *ts = "Router Renumbering";
		if (icmpv6_138_code(code)) *cs = icmpv6_138_code(code);
		*body = -1; return;
	case 139: *ts = "ICMP Node Information Query";
		if (code < ASZ(icmpv6_type_139_codes)) *cs = icmpv6_type_139_codes[code];
		*body = -1; return;
	case 140: *ts = "ICMP Node Information Response";
		if (code < ASZ(icmpv6_type_140_codes)) *cs = icmpv6_type_140_codes[code];
		*body = -1; return;
	case 141: *ts = "Inverse Neighbor Discovery Solicitation Message"; *body = -1; return;
	case 142: *ts = "Inverse Neighbor Discovery Advertisement Message"; *body = -1; return;
	case 143: *ts = "Multicast Listener Report v2"; *body = -1; return;
	case 144: *ts = "Home Agent Address Discovery Request Message"; *body = -1; return;
	case 145: *ts = "Home Agent Address Discovery Reply Message"; *body = -1; return;
	case 146: *ts = "Mobile Prefix Solicitation"; *body = -1; return;
	case 147: *ts = "Mobile Prefix Advertisement"; *body = -1; return;
	case 148: *ts = "Certification Path Solicitation"; *body = -1; return;
	case 149: *ts = "Certification Path Advertisement"; *body = -1; return;
	case 150: *ts = "ICMP messages utilized by experimental mobility protocols such as Seamoby";
		*body = -1; return;
	case 151: *ts = "Multicast Router Advertisement"; *cs = "Ad. Interval"; *body = -1; return;
	case 152: *ts = "Multicast Router Solicitation"; *cs = "Reserved"; *body = -1; return;
	case 153: *ts = "Multicast Router Termination"; *cs = "Reserved"; *body = -1; return;
	case 154: *ts = "FMIPv6 Messages"; *body = -1; return;
	case 155: *ts = "RPL Control Message";
		if (icmpv6_155_code(code)) *cs = icmpv6_155_code(code);
		return;
	}
}

static void C_icmpv6_body(P *k);

/* icmpv6 / icmpv6_less (proto_icmpv6.c:1667-1699): leaf */
static int L_icmpv6(P *k, uint32_t layer_start)
{
	uint32_t h;
	uint8_t type, code;

	if (!pull(k, 4, &h))
		return 0;
	type = B(k, h);
	code = B(k, h + 1);
	if (k->mode != PRINT_NORM) {
		E(k, " ICMPv6 Type (%u) Code (%u)", type, code);
		return 0;
	}
	{
		const char *ts, *cs;
		int body;
		icmpv6_process(type, code, &ts, &cs, &body);
		if (body < 0) {
			/* variable-length body: rendered on the host (NSD_F_HOST);
			 * the walk keeps where its pulls end */
			k->host = 1;
			k->data = layer_start;
			C_icmpv6_body(k);
			if (k->t)
				k->t->unsupported = 1;
			return 0;
		}
		E(k, " [ ICMPv6 ");
		E(k, "%s (%u), ", ts, type);
		E(k, "%s (%u), ", cs, code);
		E(k, "Chks (0x%x)", BE16(k, h + 2));
		if (body) {
			uint32_t b;
			if (!pull(k, 4, &b)) {
				E(k, "\n%s%s%s", C_RED, "Failed to dissect Message", C_END);
			} else {
				switch (body) {
				case 1: case 3:
					E(k, ", Unused (0x%x)", BE32(k, b));
					E(k, " Payload include as much of invoking packet");
					break;
				case 2:
					E(k, ", MTU (0x%x)", BE32(k, b));
					E(k, " Payload include as much of invoking packet");
					break;
				case 4:
					E(k, ", Pointer (0x%x)", BE32(k, b));
					E(k, " Payload include as much of invoking packet");
					break;
				default:
					E(k, ", ID (0x%x)", BE16(k, b));
					E(k, ", Seq. Nr. (%u)", BE16(k, b + 2));
					E(k, " Payload include Data");
				}
			}
		}
		E(k, " ]\n");
	}
	return 0;
}

/* run one ops' process() */
/* ---- LINKTYPE_LINUX_SLL head (dissector_sll.c:17-82) ---------------------
 * The packet's struct sockaddr_ll comes from nsor_set_sll (thread-local;
 * NULL = zeros, like a zeroed pkt->sll). */
static __thread const nsd_sll_t *g_sll;

void nsor_set_sll(const nsd_sll_t *sll) { g_sll = sll; }

static const char *sll_pkt_type2str(unsigned t)          /* dissector_sll.c:17-37 */
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

static const char *sll_device_type2str(unsigned t)       /* dev.c:252-402 */
{
	static const struct { unsigned t; const char *s; } tab[] = {
		{1, "ether"}, {2, "eether"}, {3, "ax25"}, {4, "pronet"}, {5, "chaos"},
		{6, "ieee802"}, {7, "arcnet"}, {8, "appletlk"}, {15, "dlci"}, {19, "atm"},
		{23, "metricom"}, {24, "ieee1394"}, {32, "infiniband"}, {256, "slip"},
		{257, "cslip"}, {258, "slip6"}, {259, "cslip6"}, {260, "RSRVD"}, {264, "adapt"},
		{270, "rose"}, {271, "x25"}, {272, "hwx25"}, {280, "can"}, {512, "ppp"},
		{513, "hdlc"}, {516, "lapb"}, {517, "ddcmp"}, {518, "rawhdlc"}, {768, "tunnel"},
		{769, "tunnel6"}, {770, "frad"}, {771, "skip"}, {772, "loopback"},
		{773, "localtlk"}, {774, "fddi"}, {775, "bif"}, {776, "sit"}, {777, "ipddp"},
		{778, "ipgre"}, {779, "pimreg"}, {780, "hippi"}, {781, "ash"}, {782, "econet"},
		{783, "irda"}, {784, "fcpp"}, {785, "fcal"}, {786, "fcpl"}, {787, "fcfb0"},
		{788, "fcfb1"}, {789, "fcfb2"}, {790, "fcfb3"}, {791, "fcfb4"}, {792, "fcfb5"},
		{793, "fcfb6"}, {794, "fcfb7"}, {795, "fcfb8"}, {796, "fcfb9"}, {797, "fcfb10"},
		{798, "fcfb11"}, {799, "fcfb12"}, {800, "ieee802_tr"}, {801, "ieee80211"},
		{802, "ieee80211_prism"}, {803, "ieee80211_radiotap"}, {804, "ieee802154"},
		{820, "phonet"}, {821, "phonet_pipe"}, {822, "caif"}, {823, "ip6gre"},
		{824, "netlink"}, {0xFFFE, "none"}, {0xFFFF, "void"},
	};
	for (size_t i = 0; i < sizeof(tab) / sizeof(tab[0]); i++)
		if (tab[i].t == t)
			return tab[i].s;
	return "Unknown";
}

/* device_addr2str (dev.c:405-422) into sll_print_full's 40-byte buffer;
 * bytes past sll_addr[8] read as zero (parity domain) */
static void sll_device_addr2str(const uint8_t *addr8, int alen, int type, char *buf)
{
	uint8_t a[256];
	memset(a, 0, sizeof(a));
	memcpy(a, addr8, 8);
	if (alen == 4 && (type == 768 || type == 776 || type == 778)) {
		inet_ntop(AF_INET, a, buf, 40);
		return;
	}
	if (alen == 16 && type == 769) {
		inet_ntop(AF_INET6, a, buf, 40);
		return;
	}
	snprintf(buf, 40, "%02x", a[0]);
	for (int i = 1, l = 2; i < alen && l < 40; i++, l += 3)
		snprintf(buf + l, 40 - l, ":%02x", a[i]);
}

static int L_sll(P *k)
{
	nsd_sll_t z;
	const nsd_sll_t *s = g_sll;
	char addr[64];
	unsigned proto;
	int cls;

	if (!s) {
		memset(&z, 0, sizeof(z));
		s = &z;
	}
	proto = (unsigned)((s->protocol >> 8) | ((s->protocol & 0xFF) << 8));
	memset(addr, 0, sizeof(addr));
	sll_device_addr2str(s->addr, s->halen, s->hatype, addr);
	if (k->mode == PRINT_NORM)
		E(k, " [ Linux \"cooked\"");
	E(k, " Pkt Type %d (%s)", s->pkttype, sll_pkt_type2str(s->pkttype));
	E(k, ", If Type %d (%s)", s->hatype, sll_device_type2str(s->hatype));
	E(k, ", Addr Len %d", s->halen);
	E(k, ", Src (%s)", addr);
	E(k, ", Proto 0x%x", proto);
	if (k->mode != PRINT_NORM)
		return 0;                    /* sll_print_less dispatches nothing */
	E(k, " ]\n");
	/* pcap_devtype_to_linktype (pcap_io.h:205-267) */
	switch (s->hatype) {
	case 768: case 769: case 772: case 776: case 777: case 778: case 823: case 1:
		cls = 1; break;
	case 824:
		cls = 2; break;
	default:
		cls = 0;
	}
	if (cls == 1)
		return lay2(proto);
	if (cls == 2)
		return NSD_OPS_NLMSG;
	E(k, " [ Unknown protocol ]\n");
	return 0;
}

/* ---- host-rendered leaves: the pulls only ---------------------------------
 * The text of ARP, DCCP, IGMP, LLDP and the ICMPv6 130-154 bodies is the
 * host renderer's (pinned by the reference objects' goldens); the walk
 * records where each parser leaves the cursor, which the exit op's dump
 * starts from.  A failed pull does not advance (pkt_buff.h:43-57). */

/* arp (proto_arp.c:80-196) / arp_less: one struct arphdr */
static void C_arp(P *k)
{
	pull(k, 28, NULL);
}

/* dccp (proto_dccp.c:70-133) / dccp_less (:135-148) */
static void C_dccp(P *k)
{
	uint32_t h;
	uint8_t b8;

	if (!pull(k, 12, &h) || k->mode != PRINT_NORM)
		return;
	b8 = B(k, h + 8);                  /* x: bit 0, type: bits 1..4 */
	if ((b8 & 1) && !pull(k, 4, NULL))
		return;
	if (((b8 >> 1) & 15) >= 1 && ((b8 >> 1) & 15) <= 9)
		pull(k, (b8 & 1) ? 8 : 4, NULL);
}

/* the v3 source list: n pulls of 4 bytes, ending at the first that fails
 * (proto_igmp.c:368-383, 430-445) */
static void C_igmp_sources(P *k, size_t n)
{
	while (n--)
		if (!pull(k, 4, NULL))
			break;
}

/* igmp (proto_igmp.c:452-493); igmp_less pulls nothing (:495-554) */
static void C_igmp(P *k)
{
	uint32_t len = pkt_len(k), m;
	uint8_t t = B(k, k->data);
	size_t nrec;

	if (k->mode != PRINT_NORM)
		return;
	switch (t) {
	case 0x01: case 0x02: case 0x03: case 0x04:
	case 0x05: case 0x06: case 0x07: case 0x08:
		if (len == 20)
			pull(k, 20, NULL);                 /* dissect_igmp_v0 */
		return;
	case 0x11:
		if (len >= 12) {                           /* v3 query (:334-385) */
			pull(k, 12, &m);
			C_igmp_sources(k, BE16(k, m + 10));
		} else if (len == 8) {
			pull(k, 8, NULL);                  /* v2 / v1 */
		}
		return;
	case 0x12: case 0xFF: case 0xFE: case 0xFD: case 0xFC: case 0x16: case 0x17:
		if (len == 8)
			pull(k, 8, NULL);
		return;
	case 0x22:                                         /* v3 report (:387-450) */
		if (len < 8)
			return;
		pull(k, 8, &m);
		nrec = BE16(k, m + 6);
		while (nrec--) {
			uint32_t r;
			if (!pull(k, 8, &r))
				break;
			C_igmp_sources(k, BE16(k, r + 2));
		}
		return;
	}
}

/* lldp_print_net_addr (proto_lldp.c:88-131): 0 ok, -1 invalid */
static int C_lldp_addr(const P *k, uint32_t a, uint32_t alen)
{
	uint8_t af;

	if (alen < 1)
		return -1;
	af = B(k, a);
	alen--;
	if ((af == 1 && alen < 4) || (af == 2 && alen < 16) || (af == 6 && alen < 6))
		return -1;
	return 0;
}

/* lldp (proto_lldp.c:161-455) / lldp_less (:457-488).  print_full's `len`
 * only loses the TLV headers (:187), not the TLV bodies */
static void C_lldp(P *k)
{
	unsigned int len = pkt_len(k), n_tlv = 0, type, tlen;
	uint32_t h, s;

	if (k->mode != PRINT_NORM) {
		while (len >= 2) {
			if (!pull(k, 2, &h))
				break;
			type = BE16(k, h) >> 9;
			tlen = BE16(k, h) & 0x1FF;
			len -= 2;
			if (type == 0 || tlen == 0 || len < tlen)
				break;
			pull(k, tlen, NULL);
			len -= tlen;
		}
		return;
	}
	while (len >= 2) {
		if (!pull(k, 2, &h))
			return;
		type = BE16(k, h) >> 9;
		tlen = BE16(k, h) & 0x1FF;
		len -= 2;
		if (type == 0 && tlen == 0)
			return;
		if (len < tlen)
			return;
		switch (type) {
		case 1:                 /* Chassis ID / Port ID (:200-295) */
		case 2:
			if (n_tlv != type - 1 || tlen < 2 || !pull(k, tlen, &s))
				return;
			if (B(k, s) == (type == 1 ? 4 : 3)) {
				if (tlen < 7)
					return;
			} else if (B(k, s) == (type == 1 ? 5 : 4)) {
				if (C_lldp_addr(k, s + 1, tlen))
					return;
			}
			break;
		case 3:                 /* TTL (:296-314) */
			if (n_tlv != 2 || tlen != 2 || !pull(k, 2, NULL))
				return;
			break;
		case 7:                 /* System capabilities (:348-368) */
			if (tlen != 4 || !pull(k, 4, NULL))
				return;
			break;
		case 8: {               /* Management address (:369-418) */
			uint32_t alen, oidlen;
			if (tlen < 9 || tlen > 167 || !pull(k, tlen, &s))
				return;
			alen = B(k, s);
			if (tlen - 1 < alen || C_lldp_addr(k, s + 1, alen))
				return;
			if (tlen - alen < 4)
				return;
			oidlen = B(k, s + 1 + alen + 1 + 4);
			if (tlen - alen - 4 < 3 || tlen - alen - 4 - 3 < oidlen)
				return;
			break;
		}
		case 127:               /* Organizationally specific (:419-437) */
			if (tlen < 4 || !pull(k, 4, NULL))
				return;
			pull(k, tlen - 4, NULL);
			break;
		default:                /* descriptions (:315-347), unknown TLVs (:438-441) */
			pull(k, tlen, NULL);
			break;
		}
		n_tlv++;
	}
}

/* `n` one-byte pulls, as the %x / %c loops of proto_icmpv6.c take them */
static int C_bytes(P *k, int64_t n)
{
	while (n-- > 0)
		if (!pull(k, 1, NULL))
			return 0;
	return 1;
}

/* print_ipv6_addr_list (proto_icmpv6.c:283-299) */
static int C_addrs(P *k, uint8_t nr)
{
	while (nr--)
		if (!pull(k, 16, NULL))
			return 0;
	return 1;
}

/* the Neighbor Discovery option bodies (proto_icmpv6.c:372-806): each pulls
 * its fixed part, then `len -= sizeof(*part)` (ssize_t), a negative
 * remainder failing after the pull */
static int C_nd_opt(P *k, uint8_t type, ssize_t len)
{
	uint32_t a;

	switch (type) {
	case 1: case 2:                      /* link-layer address (:372-406) */
		return C_bytes(k, len);
	case 3:                              /* prefix information (:408-437) */
		return pull(k, 30, NULL) && (len -= 30) >= 0;
	case 4:                              /* redirected header (:439-469) */
		if (!pull(k, 6, NULL) || (len -= 6) < 0)
			return 0;
		return C_bytes(k, len);
	case 5:                              /* MTU (:471-488) */
		return pull(k, 6, NULL) && (len -= 6) >= 0;
	case 9: case 10:                     /* address lists (:490-513) */
		if (!pull(k, 6, NULL) || (len -= 6) < 0)
			return 0;
		return C_addrs(k, (uint8_t)(len / 16));
	case 15: {                           /* naming (:520-584): packed {u8; size_t} */
		uint64_t pad = 0;
		ssize_t name_len;
		if (!pull(k, 9, &a) || (len -= 9) < 0)
			return 0;
		for (int i = 7; i >= 0; i--)
			pad = pad << 8 | B(k, a + 1 + i);
		if (pad > (uint64_t)len) {
			pull(k, (uint32_t)len, NULL);
			return 1;
		}
		name_len = len - (ssize_t)pad;
		if (!C_bytes(k, name_len))
			return 0;
		while (pad--)
			if (!pull(k, 1, NULL))
				break;
		return 1;
	}
	case 16:                             /* certificate (:590-626) */
		if (!pull(k, 2, NULL) || (len -= 2) < 0)
			return 0;
		C_bytes(k, len);
		return 1;
	case 17:                             /* IP address / prefix (:635-710) */
		if (!pull(k, 2, NULL) || (len -= 2) < 0)
			return 0;
		if (len == 20)
			return pull(k, 20, NULL);
		if (len == 16)
			return pull(k, 16, NULL);
		C_bytes(k, len);
		return 1;
	case 19:                             /* link-layer address (:727-762) */
		if (!pull(k, 1, NULL) || (len -= 1) < 0)
			return 0;
		return C_bytes(k, len);
	default:                             /* the rest skip the option (:786-806) */
		pull(k, (uint32_t)len, NULL);
		return 1;
	}
}

/* dissect_neighb_disc_ops (proto_icmpv6.c:808-911) */
static int C_nd_ops(P *k)
{
	while (pkt_len(k)) {
		uint32_t a;
		ssize_t payl;
		if (!pull(k, 2, &a))
			return 0;
		payl = (ssize_t)(uint16_t)(B(k, a + 1) * 8) - 2;
		if (payl > (ssize_t)pkt_len(k) || payl < 0)
			return 0;
		if (!C_nd_opt(k, B(k, a), payl))
			return 0;
	}
	return 1;
}

/* dissect_icmpv6_mcast_rec (proto_icmpv6.c:310-370) */
static int C_mcast_recs(P *k, uint16_t nr)
{
	while (nr--) {
		uint32_t r;
		uint16_t aux;
		if (!pull(k, 20, &r))
			return 0;
		aux = (uint16_t)(B(k, r + 1) * 4);
		if (aux > pkt_len(k) || !C_addrs(k, (uint8_t)BE16(k, r + 2)) || aux > pkt_len(k) ||
		    !C_bytes(k, aux))
			return 0;
	}
	return 1;
}

/* icmpv6 (proto_icmpv6.c:1667-1688) for the types whose bodies
 * icmpv6_process dissects at variable length (130-154, :1023-1474) */
static void C_icmpv6_body(P *k)
{
	uint32_t h, a;

	if (!pull(k, 4, &h))
		return;
	switch (B(k, h)) {
	case 130:                                    /* MLD query, MLDv2 (:1023-1070) */
		if (pull(k, 20, NULL) && pkt_len(k) >= 4 && pull(k, 4, &a))
			C_addrs(k, (uint8_t)BE16(k, a + 2));
		break;
	case 131: case 132:                          /* :1072-1094 */
		pull(k, 20, NULL);
		break;
	case 133: case 141: case 142: case 147: case 148: case 154:
		if (pull(k, 4, NULL))                /* :1096-1108, 1292-1300, 1355-1386, 1460-1474 */
			C_nd_ops(k);
		break;
	case 134:                                    /* :1110-1127 */
		if (pull(k, 12, NULL))
			C_nd_ops(k);
		break;
	case 135: case 136:                          /* :1129-1167 */
		if (pull(k, 20, NULL))
			C_nd_ops(k);
		break;
	case 137:                                    /* :1169-1188 */
		if (pull(k, 36, NULL))
			C_nd_ops(k);
		break;
	case 138: case 139: case 140:                /* :1210-1279 */
		pull(k, 12, NULL);
		break;
	case 143:                                    /* MLDv2 report (:1302-1317) */
		if (pull(k, 4, &a))
			C_mcast_recs(k, BE16(k, a + 2));
		break;
	case 144: case 146: case 150: case 151:      /* :1319-1332, 1350-1353, 1405-1434 */
		pull(k, 4, NULL);
		break;
	case 145:                                    /* :1334-1348 */
		if (pull(k, 4, NULL))
			C_addrs(k, (uint8_t)(pkt_len(k) / 16));
		break;
	case 149:                                    /* :1388-1403 */
		if (pull(k, 8, NULL))
			C_nd_ops(k);
		break;
	}
}

static int run_layer(P *k, int id)
{
	uint32_t start = k->data;

	switch (id) {
	case NSD_OPS_ETHERNET:       return L_ethernet(k);
	case NSD_OPS_VLAN:           return L_vlan(k);
	case NSD_OPS_QINQ:           return L_qinq(k);
	case NSD_OPS_MPLS_UC:        return L_mpls(k);
	case NSD_OPS_IPV4:           return L_ipv4(k);
	case NSD_OPS_IPV6:
	case NSD_OPS_IPV6_IN_IPV4:   return L_ipv6(k);
	case NSD_OPS_IPV6_HOP_BY_HOP:return L_v6opts(k, 0);
	case NSD_OPS_IPV6_DEST_OPTS: return L_v6opts(k, 1);
	case NSD_OPS_IPV6_ROUTING:   return L_routing(k);
	case NSD_OPS_IPV6_FRAGM:     return L_fragm(k);
	case NSD_OPS_IP_AUTH:        return L_auth(k);
	case NSD_OPS_IP_ESP:         return L_esp(k);
	case NSD_OPS_IPV6_NO_NEXT:   return L_nonext(k);
	case NSD_OPS_IPV6_MOBILITY:  return L_mobility(k);
	case NSD_OPS_TCP:            return L_tcp(k);
	case NSD_OPS_UDP:            return L_udp(k);
	case NSD_OPS_ICMPV4:         return L_icmp(k);
	case NSD_OPS_ICMPV6:         return L_icmpv6(k, start);
	case NSD_OPS_SLL:            return L_sll(k);
	default:
		/* ARP, LLDP, IGMP, DCCP (and non-Ethernet heads): host-rendered
		 * leaves, the cursor where their pulls end */
		k->host = 1;
		k->data = start;
		if (id == NSD_OPS_ARP)
			C_arp(k);
		else if (id == NSD_OPS_LLDP)
			C_lldp(k);
		else if (id == NSD_OPS_IGMP)
			C_igmp(k);
		else if (id == NSD_OPS_DCCP)
			C_dccp(k);
		if (k->t)
			k->t->unsupported = 1;
		return 0;
	}
}

/* exit op and post-mode dumps (proto_none.c:17-77, dissector.c:106-118) */
static void dump_ascii(P *k, uint32_t from, uint32_t len)
{
	char *buf;
	if (!len || !texting(k))
		return;
	E(k, " [ Chr ");
	buf = malloc(len);
	for (uint32_t i = 0; i < len; i++) {
		uint8_t c = B(k, from + i);
		buf[i] = (c >= 0x20 && c < 0x7f) ? (char)c : '.';
	}
	if (k->t) text_append(k->t, buf, len);
	else k->emit(k->ectx, buf, len);
	free(buf);
	E(k, " ]\n");
}

static void dump_hex(P *k, uint32_t from, uint32_t len)
{
	static const char hx[] = "0123456789abcdef";
	char *buf;
	if (!len || !texting(k))
		return;
	E(k, " [ Hex ");
	buf = malloc(3 * (size_t)len);
	for (uint32_t i = 0; i < len; i++) {
		uint8_t c = B(k, from + i);
		buf[3 * i] = ' ';
		buf[3 * i + 1] = hx[c >> 4];
		buf[3 * i + 2] = hx[c & 15];
	}
	if (k->t) text_append(k->t, buf, 3 * (size_t)len);
	else k->emit(k->ectx, buf, 3 * (size_t)len);
	free(buf);
	E(k, " ]\n");
}

int nsor_run_layer(int ops_id, int mode, const uint8_t *pkt, uint32_t caplen,
		   uint32_t *data, uint32_t *tail, nsor_emit_fn emit, void *ctx)
{
	P k;
	int next;

	memset(&k, 0, sizeof(k));
	k.p = pkt;
	k.caplen = caplen;
	k.data = *data;
	k.tail = *tail;
	k.mode = mode;
	k.emit = emit;
	k.ectx = ctx;
	next = run_layer(&k, ops_id);
	*data = k.data;
	*tail = k.tail;
	return next;
}

static int is_linktype(int lt, uint32_t v)
{
	return (uint32_t)lt == v || (uint32_t)lt == __builtin_bswap32(v);
}

void nsor_dissect(const uint8_t *pkt, uint32_t caplen, int linktype, int mode,
		  nsor_text *text, nsd_rec *rec, nsor_info *info)
{
	P k;
	nsor_info local;
	nsor_info *in = info ? info : &local;
	int id = 0;

	memset(&k, 0, sizeof(k));
	k.p = pkt;
	k.caplen = caplen;
	k.data = 0;
	k.tail = caplen;
	k.mode = mode;
	k.t = text;
	in->nlayers = 0;
	in->overflow = 0;

	if (mode == PRINT_NONE)      /* dissector.c:70-71 */
		goto done;

	if (mode == PRINT_NORM || mode == PRINT_LESS) {
		if (is_linktype(linktype, NSD_LINKTYPE_EN10MB)) {
			id = NSD_OPS_ETHERNET;
		} else if (is_linktype(linktype, NSD_LINKTYPE_LINUX_SLL)) {
			id = NSD_OPS_SLL;
		} else if (is_linktype(linktype, NSD_LINKTYPE_IEEE802_11) ||
			   is_linktype(linktype, NSD_LINKTYPE_IEEE802_11_RADIOTAP)) {
			id = NSD_OPS_IEEE80211;
		} else if (is_linktype(linktype, NSD_LINKTYPE_NETLINK)) {
			id = NSD_OPS_NLMSG;
		}
		/* chain loop (dissector.c:51-58) */
		while (id) {
			if (in->nlayers < NSD_EXT_MAX_LAYERS) {
				in->id[in->nlayers] = (uint8_t)id;
				in->off[in->nlayers] = (uint16_t)k.data;
			} else {
				in->overflow = 1;
			}
			in->nlayers++;
			id = run_layer(&k, id);
		}
		/* exit op (dissector.c:60-61) */
		if (!k.host) {
			if (mode == PRINT_NORM) {
				uint32_t len = k.tail - k.data;
				if (len) {
					dump_ascii(&k, k.data, len);
					dump_hex(&k, k.data, len);
				}
				E(&k, "\n");
			} else {
				E(&k, "\n");
			}
		}
	} else {
		uint32_t len = caplen;
		switch (mode) {     /* dissector.c:108-118 */
		case PRINT_HEX:
			if (len) { dump_hex(&k, 0, len); E(&k, "\n"); }
			break;
		case PRINT_ASCII:
			if (len) { dump_ascii(&k, 0, len); E(&k, "\n"); }
			break;
		case PRINT_HEX_ASCII:
			if (len) { dump_ascii(&k, 0, len); dump_hex(&k, 0, len); }
			E(&k, "\n");
			break;
		}
	}
done:
	in->data = k.data;
	in->tail = k.tail;
	{
		uint32_t e = k.data > k.extent ? k.data : k.extent;
		uint32_t w;
		if (caplen <= 64)
			w = caplen;
		else {
			w = (e + 63) & ~63u;
			if (w > caplen) w = caplen;
		}
		in->w_bytes = (mode == PRINT_NONE) ? 0 : w;
	}
	if (rec) {
		uint32_t n = in->nlayers;
		int ext = n > NSD_REC_MAX_LAYERS || in->overflow;
		memset(rec, 0, sizeof(*rec));
		for (uint32_t i = 0; i < n && i < NSD_REC_MAX_LAYERS; i++) {
			rec->chain |= (uint32_t)in->id[i] << (5 * i);
			if (i >= 1 && in->off[i] > 510)
				ext = 1;
		}
		rec->data_off = (uint16_t)k.data;
		rec->tail_off = (uint16_t)k.tail;
		rec->ip_csum = k.ip_csum;
		rec->nflags = (uint8_t)((ext ? NSD_N_EXT : n) |
			(k.icmp_bad ? NSD_F_ICMP_BAD : 0) | (k.host ? NSD_F_HOST : 0) |
			(in->overflow ? NSD_F_OVERFLOW : 0));
		if (!ext)
			for (uint32_t i = 1; i < n; i++)
				rec->off2[i - 1] = (uint8_t)(in->off[i] >> 1);
	}
}

/* ------------------------------------------------------------------------ */
/* batch forms                                                              */
/* ------------------------------------------------------------------------ */
static void count(uint64_t *c, const nsd_rec *r, const nsor_info *in, uint32_t caplen)
{
	uint32_t n = in->nlayers < NSD_EXT_MAX_LAYERS ? in->nlayers : NSD_EXT_MAX_LAYERS;
	for (uint32_t i = 0; i < n; i++)
		c[NSD_CNT_OPS + in->id[i]]++;
	c[NSD_CNT_PKTS]++;
	c[NSD_CNT_BYTES] += caplen;
	if (r->ip_csum) c[NSD_CNT_IP_BAD]++;
	if (r->nflags & NSD_F_ICMP_BAD) c[NSD_CNT_ICMP_BAD]++;
	if (r->nflags & NSD_F_HOST) c[NSD_CNT_HOST]++;
	if ((r->nflags & 7) == NSD_N_EXT) c[NSD_CNT_EXT]++;
	if (r->nflags & NSD_F_OVERFLOW) c[NSD_CNT_OVERFLOW]++;
	if (r->tail_off < caplen) c[NSD_CNT_TRIM]++;
}

uint64_t nsor_dissect_batch(const uint8_t *frames, const nsd_desc_t *desc, uint32_t n,
			    int linktype, int mode, nsd_rec *rec, uint32_t *ext,
			    uint32_t ext_words, uint32_t *ext_used, uint64_t *counters)
{
	return nsor_dissect_batch_sll(frames, desc, NULL, n, linktype, mode, rec, ext, ext_words,
				      ext_used, counters);
}

uint64_t nsor_dissect_batch_sll(const uint8_t *frames, const nsd_desc_t *desc, const nsd_sll_t *sll,
				uint32_t n, int linktype, int mode, nsd_rec *rec, uint32_t *ext,
				uint32_t ext_words, uint32_t *ext_used, uint64_t *counters)
{
	uint64_t sw = 0;
	nsor_info in;
	nsd_rec r;

	for (uint32_t i = 0; i < n; i++) {
		uint64_t d = desc[i];
		uint32_t caplen = NSD_DESC_CAPLEN(d);
		g_sll = sll ? sll + i : NULL;
		nsor_dissect(frames + NSD_DESC_OFF(d), caplen, linktype, mode, NULL, &r, &in);
		if ((r.nflags & 7) == NSD_N_EXT) {
			/* dense pool entries in packet order (layout: netsniff_dissect.h) */
			const uint32_t m = in.nlayers < NSD_EXT_MAX_LAYERS ? in.nlayers : NSD_EXT_MAX_LAYERS;
			const uint32_t words = NSD_EXT_WORDS(m);
			uint32_t slot = UINT32_MAX;
			if (ext_used) {
				const uint32_t at = *ext_used;
				*ext_used += words;
				if (ext && (uint64_t)at + words <= ext_words)
					slot = at;
			}
			if (slot != UINT32_MAX) {
				uint32_t *e = ext + slot;
				memset(e, 0, words * sizeof(uint32_t));
				e[0] = i;
				e[1] = m;
				for (uint32_t k = 0; k < m; k++)
					e[NSD_EXT_HDR_WORDS + k] = in.id[k] | (uint32_t)in.off[k] << 16;
			} else {
				r.nflags |= NSD_F_OVERFLOW;
			}
			memcpy(r.off2, &slot, 4);
			r.off2[4] = 0;
		}
		if (rec)
			rec[i] = r;
		if (counters)
			count(counters, &r, &in, caplen);
		sw += in.w_bytes;
	}
	g_sll = NULL;
	return sw;
}

uint64_t nsor_dissect_batch_text(const uint8_t *frames, const nsd_desc_t *desc,
				 uint32_t n, int linktype, int mode, nsor_text *text)
{
	uint64_t sw = 0;
	nsor_info in;
	for (uint32_t i = 0; i < n; i++) {
		uint64_t d = desc[i];
		nsor_dissect(frames + NSD_DESC_OFF(d), NSD_DESC_CAPLEN(d), linktype, mode, text,
			     NULL, &in);
		sw += in.w_bytes;
	}
	return sw;
}

/* ---- show_frame_hdr (dissector.h:31-116) ---------------------------------
 * The line every capture loop prints before the entry point.  The header
 * view: a tpacket2_hdr (v3 0, read_pcap's zeroed frame_map) or the frame's
 * tpacket3_hdr (v3 1, walk_t3_block).  ring.h is built with HAVE_TPACKET3,
 * so tpacket_has_vlan_info reads tp_status through the tpacket3_hdr view
 * (ring.h:71-84): for a tpacket2_hdr that is the word at offset 20, tp_nsec;
 * tpacket_uhdr_vlan_tci / _proto return 0 when v3 is false (ring.h:51-69). */
extern char *if_indextoname(unsigned ifindex, char *ifname);

static const char *const fh_packet_types[256] = {
	[0] = "<", [1] = "B", [2] = "M", [3] = "P", [4] = ">", [6] = "K->U", [7] = "U->K",
};

static const char *fh_ts_source(uint32_t status)      /* dissector.h:41-51 */
{
	if (status & (1u << 31))
		return "(raw hw ts)";
	else if (status & (1u << 30))
		return "(sys hw ts)";
	else if (status & (1u << 29))
		return "(sw ts)";
	return "";
}

static void T(nsor_text *t, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
static void T(nsor_text *t, const char *fmt, ...)
{
	char tmp[256];
	va_list vl;
	int n;
	va_start(vl, fmt);
	n = vsnprintf(tmp, sizeof(tmp), fmt, vl);
	va_end(vl);
	if (n > 0)
		text_append(t, tmp, (size_t)n);
}

void nsor_frame_hdr(const nsd_frame_hdr_t *fh, const nsd_sll_t *sll, const uint8_t *pkt, uint32_t caplen,
		    int linktype, int mode, uint64_t count, nsor_text *t)
{
	char tmp[64];
	nsd_sll_t z;
	uint8_t pkttype;
	const char *ifn;

	if (mode == PRINT_NONE)
		return;
	if (!sll) {
		memset(&z, 0, sizeof(z));
		sll = &z;
	}
	pkttype = sll->pkttype;
	if (linktype == NSD_LINKTYPE_NETLINK && caplen >= 16 && pkttype == 4) {
		uint32_t pid;
		memcpy(&pid, pkt + 12, 4);                   /* nlmsghdr.nlmsg_pid */
		pkttype = pid == 0 ? 7 : 6;                  /* PACKET_KERNEL : PACKET_USER */
	}
	/* if_indextoname (dissector.h:82, 89), the last answer kept per thread:
	 * the reference asks the kernel for every packet (a socket and an
	 * ioctl), which would make the timed CPU baseline a syscall benchmark;
	 * the name of an index does not change while a capture runs */
	{
		static __thread int last_idx = -1, last_ok;
		static __thread char last_name[64];
		if (sll->ifindex != last_idx) {
			const char *r = if_indextoname((unsigned)sll->ifindex, tmp);
			last_idx = sll->ifindex;
			last_ok = r != NULL;
			if (r)
				snprintf(last_name, sizeof(last_name), "%s", r);
		}
		ifn = last_ok ? last_name : NULL;
	}
	switch (mode) {
	case PRINT_LESS:
		T(t, "%s %s %u #%lu", fh_packet_types[pkttype] ? fh_packet_types[pkttype] : "?", ifn ? ifn : "?",
		  fh->len, (unsigned long)count);
		break;
	default:
		T(t, "%s %s %u %us.%uns #%lu %s\n", fh_packet_types[pkttype] ? fh_packet_types[pkttype] : "?",
		  ifn ? ifn : "?", fh->len, fh->sec, fh->nsec, (unsigned long)count,
		  fh->v3 ? "" : fh_ts_source(fh->status));
		if ((fh->v3 ? fh->status : fh->nsec) & ((1u << 4) | (1u << 6))) {
			uint16_t tci = fh->v3 ? (uint16_t)fh->vlan_tci : 0;
			T(t, " [ tpacketv3 VLAN ");
			T(t, "Prio (%u), ", (tci & 0xe000) >> 13);
			T(t, "CFI (%u), ", (tci & 0x1000) >> 12);
			T(t, "ID (%u), ", tci & 0x0fff);
			T(t, "Proto (0x%.4x)", fh->v3 ? fh->vlan_tpid : 0);
			T(t, " ]\n");
		}
		break;
	}
}

/* ---- pcap records -> the frame_map read_pcap prints from ------------------
 * pcap_validate_header (pcap_io.h:874-911: magic, version, the *_LL remap
 * for SLL / netlink link types), the record sizes (pcap_get_hdr_length
 * :429-453), pcap_rw_read's end rules (pcap_rw.c:38-55: a short header or
 * body, caplen 0 or above the 1 MiB buffer end the replay) and
 * pcap_pkthdr_to_tpacket_hdr (:594-709) into a frame_map zeroed once
 * (netsniff-ng.c:672).  Fills up to max records' fh / sll / caplen (each may
 * be NULL); returns the records, or -1 for a file read_pcap refuses. */
long nsor_pcap_meta(const char *path, nsd_frame_hdr_t *fh, nsd_sll_t *sll, uint32_t *caplen, uint32_t max)
{
	FILE *f = fopen(path, "rb");
	uint8_t h[24], r[32];
	uint32_t magic, lt, m;
	uint16_t vmaj, vmin;
	int swapped = 0, ll = 0, hdrsize = 16, usec;
	nsd_sll_t s;
	long n = 0;

	if (!f)
		return -1;
	if (fread(h, 1, 24, f) != 24) {
		fclose(f);
		return -1;
	}
	memcpy(&magic, h, 4);
	memcpy(&vmaj, h + 4, 2);
	memcpy(&vmin, h + 6, 2);
	memcpy(&lt, h + 20, 4);
	m = magic;
	if (m == 0xd4c3b2a1u || m == 0x4d3cb2a1u || m == 0x34cdb2a1u || m == 0x12cbe2a1u) {
		swapped = 1;
		m = __builtin_bswap32(m);
	}
	if ((m != 0xa1b2c3d4u && m != 0xa1b23c4du && m != 0xa1b2cd34u && m != 0xa1e2cb12u) ||
	    (vmaj != 2 && __builtin_bswap16(vmaj) != 2) || (vmin != 4 && __builtin_bswap16(vmin) != 4)) {
		fclose(f);
		return -1;
	}
	if (swapped)
		lt = __builtin_bswap32(lt);
	if ((lt == 113 || lt == 253) && (m == 0xa1b2c3d4u || m == 0xa1b23c4du)) {
		ll = 1;
		hdrsize = 32;
	}
	if (m == 0xa1b2cd34u || m == 0xa1e2cb12u)
		hdrsize = 24;
	usec = m == 0xa1b2c3d4u || m == 0xa1b2cd34u;
	memset(&s, 0, sizeof(s));
	while ((uint32_t)n < max) {
		uint32_t v[4], cl;
		int k;
		if (fread(r, 1, hdrsize, f) != (size_t)hdrsize)
			break;
		memcpy(v, r, 16);
		for (k = 0; k < 4; k++)
			if (swapped)
				v[k] = __builtin_bswap32(v[k]);
		cl = v[2] - (ll ? 16 : 0);
		if (cl == 0 || cl > (1u << 20))
			break;
		if (fseek(f, cl, SEEK_CUR) != 0)
			break;
		{
			/* a body cut short by the end of the file ends the replay */
			long pos = ftell(f), end;
			fseek(f, 0, SEEK_END);
			end = ftell(f);
			if (pos > end)
				break;
			fseek(f, pos, SEEK_SET);
		}
		if (fh) {
			memset(&fh[n], 0, sizeof(fh[n]));
			fh[n].sec = v[0];
			fh[n].nsec = usec ? v[1] * 1000u : v[1];
			fh[n].len = v[3] - (ll ? 16 : 0);
		}
		if (ll) {                                     /* ll_to_sockaddr :182-191 */
			s.pkttype = (uint8_t)(r[16] << 8 | r[17]);
			s.hatype = (uint16_t)(r[18] << 8 | r[19]);
			s.halen = (uint8_t)(r[20] << 8 | r[21]);
			memcpy(s.addr, r + 22, 8);
			memcpy(&s.protocol, r + 30, 2);
		} else if (m == 0xa1b2cd34u) {                /* struct pcap_pkthdr_kuz */
			uint32_t ifi;
			uint16_t pr;
			memcpy(&ifi, r + 16, 4);
			memcpy(&pr, r + 20, 2);
			s.ifindex = (int32_t)(swapped ? __builtin_bswap32(ifi) : ifi);
			s.protocol = swapped ? __builtin_bswap16(pr) : pr;
			s.pkttype = r[22];
		} else if (m == 0xa1e2cb12u) {                /* struct pcap_pkthdr_bkm */
			uint16_t ifi, pr;
			memcpy(&ifi, r + 18, 2);
			memcpy(&pr, r + 20, 2);
			s.ifindex = swapped ? __builtin_bswap16(ifi) : ifi;
			s.protocol = swapped ? __builtin_bswap16(pr) : pr;
			s.hatype = r[22];
			s.pkttype = r[23];
		}
		if (sll)
			sll[n] = s;
		if (caplen)
			caplen[n] = cl;
		n++;
	}
	fclose(f);
	return n;
}

typedef struct {
	const uint8_t *frames;
	const nsd_desc_t *desc;
	const nsd_frame_hdr_t *fh;
	const nsd_sll_t *sll;
	uint64_t first_count;
	uint32_t lo, hi;
	int linktype, mode;
	nsd_rec *rec;
	uint64_t counters[NSD_NCOUNTERS];
	uint64_t sw;
	uint64_t text_bytes;
} mt_job;

/* fields + text (what the reference always does: it prints as it parses)
 * per packet into a thread-local sink that is reset after every packet, as
 * tprintf_flush empties the reference's buffer (tprintf.c:105-110) */
static void *mt_text_worker(void *arg)
{
	mt_job *j = arg;
	nsor_info in;
	nsor_text t;
	nsor_text_init(&t);
	for (uint32_t i = j->lo; i < j->hi; i++) {
		uint64_t d = j->desc[i];
		const nsd_sll_t *sl = j->sll ? j->sll + i : NULL;
		if (j->fh)
			nsor_frame_hdr(j->fh + i, sl, j->frames + NSD_DESC_OFF(d), NSD_DESC_CAPLEN(d), j->linktype,
				       j->mode, j->first_count + i, &t);
		g_sll = sl;
		nsor_dissect(j->frames + NSD_DESC_OFF(d), NSD_DESC_CAPLEN(d), j->linktype, j->mode, &t,
			     NULL, &in);
		j->text_bytes += t.len;
		j->sw += in.w_bytes;
		nsor_text_reset(&t);
	}
	nsor_text_free(&t);
	return NULL;
}

uint64_t nsor_dissect_batch_text_mt(const uint8_t *frames, const nsd_desc_t *desc, uint32_t n,
				    int linktype, int mode, int nthreads, uint64_t *text_bytes)
{
	return nsor_dissect_batch_text_fh_mt(frames, desc, NULL, NULL, 0, n, linktype, mode, nthreads, text_bytes);
}

uint64_t nsor_dissect_batch_text_fh_mt(const uint8_t *frames, const nsd_desc_t *desc, const nsd_frame_hdr_t *fh,
				       const nsd_sll_t *sll, uint64_t first_count, uint32_t n, int linktype,
				       int mode, int nthreads, uint64_t *text_bytes)
{
	pthread_t th[256];
	mt_job *jobs;
	uint64_t sw = 0, tb = 0;

	if (nthreads < 1) nthreads = 1;
	if (nthreads > 256) nthreads = 256;
	jobs = calloc(nthreads, sizeof(*jobs));
	for (int t = 0; t < nthreads; t++) {
		jobs[t].frames = frames;
		jobs[t].desc = desc;
		jobs[t].lo = (uint32_t)((uint64_t)n * t / nthreads);
		jobs[t].hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
		jobs[t].linktype = linktype;
		jobs[t].mode = mode;
		jobs[t].fh = fh;
		jobs[t].sll = sll;
		jobs[t].first_count = first_count;
		pthread_create(&th[t], NULL, mt_text_worker, &jobs[t]);
	}
	for (int t = 0; t < nthreads; t++) {
		pthread_join(th[t], NULL);
		sw += jobs[t].sw;
		tb += jobs[t].text_bytes;
	}
	free(jobs);
	if (text_bytes)
		*text_bytes = tb;
	return sw;
}

static void *mt_worker(void *arg)
{
	mt_job *j = arg;
	nsor_info in;
	nsd_rec r;
	for (uint32_t i = j->lo; i < j->hi; i++) {
		uint64_t d = j->desc[i];
		uint32_t caplen = NSD_DESC_CAPLEN(d);
		nsor_dissect(j->frames + NSD_DESC_OFF(d), caplen, j->linktype, j->mode, NULL, &r, &in);
		if (j->rec)
			j->rec[i] = r;
		count(j->counters, &r, &in, caplen);
		j->sw += in.w_bytes;
	}
	return NULL;
}

uint64_t nsor_dissect_batch_mt(const uint8_t *frames, const nsd_desc_t *desc, uint32_t n,
			       int linktype, int mode, nsd_rec *rec, uint64_t *counters,
			       int nthreads)
{
	pthread_t th[256];
	mt_job *jobs;
	uint64_t sw = 0;

	if (nthreads < 1) nthreads = 1;
	if (nthreads > 256) nthreads = 256;
	jobs = calloc(nthreads, sizeof(*jobs));
	for (int t = 0; t < nthreads; t++) {
		jobs[t].frames = frames;
		jobs[t].desc = desc;
		jobs[t].lo = (uint32_t)((uint64_t)n * t / nthreads);
		jobs[t].hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
		jobs[t].linktype = linktype;
		jobs[t].mode = mode;
		jobs[t].rec = rec;
		pthread_create(&th[t], NULL, mt_worker, &jobs[t]);
	}
	for (int t = 0; t < nthreads; t++) {
		pthread_join(th[t], NULL);
		if (counters)
			for (int c = 0; c < NSD_NCOUNTERS; c++)
				counters[c] += jobs[t].counters[c];
		sw += jobs[t].sw;
	}
	free(jobs);
	return sw;
}

/* The line floor of a batch (TEST / MEASUREMENT INFRASTRUCTURE, bench.py's
 * roofline): the distinct 128-byte lines of the frame buffer that hold the
 * bytes the chain must inspect, [off, off + W(pkt)) per packet (W as
 * nsor_dissect's w_bytes: the algorithmic read extent).  An HBM read moves
 * whole 128-byte lines, so no schedule that reads each needed line once can
 * fetch less: the floor the measured traffic is compared with (plus 8 bytes
 * of descriptor per packet).  Packets in order of offset (the synthetic
 * batches); each thread walks a contiguous range, and a line two ranges
 * share is counted once. */
typedef struct {
	const uint8_t *frames;
	const nsd_desc_t *desc;
	uint32_t lo, hi;
	int linktype, mode;
	uint64_t lines, first, last;   /* distinct lines; the range's first and last line (UINT64_MAX: none) */
} lf_job;

static void *lf_worker(void *arg)
{
	lf_job *j = arg;
	nsor_info in;
	nsd_rec r;
	uint64_t last = UINT64_MAX;
	j->first = UINT64_MAX;
	for (uint32_t i = j->lo; i < j->hi; i++) {
		const uint64_t d = j->desc[i], off = NSD_DESC_OFF(d);
		nsor_dissect(j->frames + off, NSD_DESC_CAPLEN(d), j->linktype, j->mode, NULL, &r, &in);
		if (!in.w_bytes)
			continue;
		uint64_t a = off >> 7;
		const uint64_t b = (off + in.w_bytes - 1) >> 7;
		if (j->first == UINT64_MAX)
			j->first = a;
		if (last != UINT64_MAX && a <= last)
			a = last + 1;
		if (b >= a)
			j->lines += b - a + 1;
		if (last == UINT64_MAX || b > last)
			last = b;
	}
	j->last = last;
	return NULL;
}

uint64_t nsor_line_floor_mt(const uint8_t *frames, const nsd_desc_t *desc, uint32_t n, int linktype, int mode,
			    int nthreads)
{
	pthread_t th[256];
	lf_job *jobs;
	uint64_t lines = 0, prev_last = UINT64_MAX;

	if (nthreads < 1) nthreads = 1;
	if (nthreads > 256) nthreads = 256;
	jobs = calloc(nthreads, sizeof(*jobs));
	for (int t = 0; t < nthreads; t++) {
		jobs[t].frames = frames;
		jobs[t].desc = desc;
		jobs[t].lo = (uint32_t)((uint64_t)n * t / nthreads);
		jobs[t].hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
		jobs[t].linktype = linktype;
		jobs[t].mode = mode;
		pthread_create(&th[t], NULL, lf_worker, &jobs[t]);
	}
	for (int t = 0; t < nthreads; t++) {
		pthread_join(th[t], NULL);
		lines += jobs[t].lines;
		if (jobs[t].first != UINT64_MAX && jobs[t].first == prev_last)
			lines--;   /* the line the previous range ended in */
		if (jobs[t].last != UINT64_MAX)
			prev_last = jobs[t].last;
	}
	free(jobs);
	return lines;
}

