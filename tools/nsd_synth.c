/*
 * nsd_synth.c - deterministic synthetic frame generators for the BASELINE
 * configs, seeded splitmix64, one independent stream per packet
 * index so any index range (a shard) can be generated on its own.
 *
 *   NSD_SYN_UDP64  (C1/C2) Eth/IPv4/UDP 64 B: IHL 5, tot_len 50, DF, TTL 64,
 *                  valid csum, src 10.0.0.0|i, sport 1024+i%1000, dport 53,
 *                  UDP len 30, 22 zero payload bytes.
 *   NSD_SYN_IMIX   (C3/C5) sizes {64:7, 576:4, 1500:1}, 50% 802.1Q,
 *                  L4 uniform over {TCP(20B), UDP, ICMP echo}, tot_len
 *                  consistent with the frame (no trailers), valid checksums.
 *   NSD_SYN_IPV6X  (C4) Eth/IPv6 + 0..6 extension headers drawn from
 *                  {HBH, DestOpts, Routing(type 0 with 0..4 addrs, type 4),
 *                  Fragment, AH, Mobility(types 0..6)}, hdr_ext_len 0..3,
 *                  terminal {TCP, UDP, ICMPv6 echo, NoNext, ESP}, ~1% of
 *                  packets with one deliberately invalid ext length,
 *                  frame sizes drawn from 64..1500.
 *
 * Not part of the product and not the oracle: input generation for tests and
 * bench.py.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include "../include/netsniff_dissect.h"

enum { NSD_SYN_UDP64 = 1, NSD_SYN_IMIX = 3, NSD_SYN_IPV6X = 4 };

typedef struct { uint64_t s; } rng;
static inline uint64_t next(rng *r)
{
	uint64_t z = (r->s += 0x9E3779B97F4A7C15ull);
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}
static inline rng seed_for(uint64_t seed, uint64_t i)
{
	rng r = { seed ^ (i * 0xD1342543DE82EF95ull) };
	next(&r);
	return r;
}
static inline uint32_t rnd(rng *r, uint32_t n) { return (uint32_t)(next(r) % n); }

static inline void put16(uint8_t *p, uint16_t v) { p[0] = v >> 8; p[1] = (uint8_t)v; }
static inline void put32(uint8_t *p, uint32_t v) { put16(p, v >> 16); put16(p + 2, (uint16_t)v); }

/* one's complement checksum in network order over len bytes */
static uint16_t inet_csum(const uint8_t *p, size_t len)
{
	uint32_t sum = 0;
	for (size_t i = 0; i + 1 < len; i += 2)
		sum += (uint32_t)p[i] << 8 | p[i + 1];
	if (len & 1)
		sum += (uint32_t)p[len - 1] << 8;
	while (sum >> 16)
		sum = (sum & 0xffff) + (sum >> 16);
	return (uint16_t)~sum;
}

static void fill_random(rng *r, uint8_t *p, size_t n)
{
	size_t i = 0;
	while (i + 8 <= n) {
		uint64_t v = next(r);
		memcpy(p + i, &v, 8);
		i += 8;
	}
	if (i < n) {
		uint64_t v = next(r);
		memcpy(p + i, &v, n - i);
	}
}

static void eth_hdr(uint8_t *p, rng *r, uint16_t type, int fixed)
{
	static const uint8_t dst[6] = { 0x3c, 0xfd, 0xfe, 0x00, 0x00, 0x02 };
	static const uint8_t src[6] = { 0x00, 0x1b, 0x21, 0x00, 0x00, 0x01 };
	memcpy(p, dst, 6);
	memcpy(p + 6, src, 6);
	if (!fixed) {
		uint64_t v = next(r);
		p[3] = (uint8_t)v; p[4] = (uint8_t)(v >> 8); p[5] = (uint8_t)(v >> 16);
		p[9] = (uint8_t)(v >> 24); p[10] = (uint8_t)(v >> 32); p[11] = (uint8_t)(v >> 40);
		/* ~1/16 multicast / broadcast destinations exercise the vendor class */
		if (((v >> 48) & 15) == 0) { p[0] = 0x01; p[1] = 0x00; p[2] = 0x5e; }
		if (((v >> 48) & 15) == 1) memset(p, 0xff, 6);
		if (((v >> 48) & 15) == 2) p[6] = 0x02;
	}
	put16(p + 12, type);
}

static void ipv4_hdr(uint8_t *p, uint16_t tot_len, uint16_t id, uint8_t ttl, uint8_t proto,
		     uint32_t saddr, uint32_t daddr, uint8_t tos)
{
	p[0] = 0x45; p[1] = tos;
	put16(p + 2, tot_len);
	put16(p + 4, id);
	put16(p + 6, 0x4000);
	p[8] = ttl; p[9] = proto;
	put16(p + 10, 0);
	put32(p + 12, saddr);
	put32(p + 16, daddr);
	put16(p + 10, inet_csum(p, 20));
}

/* C1/C2 */
static uint32_t gen_udp64(uint64_t seed, uint64_t i, uint8_t *p)
{
	(void)seed;
	if (!p)
		return 64;
	memset(p, 0, 64);
	eth_hdr(p, NULL, 0x0800, 1);
	ipv4_hdr(p + 14, 50, (uint16_t)i, 64, 17, 0x0A000000u | (uint32_t)(i & 0xFFFFFF), 0xC0A80101u, 0);
	put16(p + 34, (uint16_t)(1024 + i % 1000));
	put16(p + 36, 53);
	put16(p + 38, 30);
	put16(p + 40, 0);
	return 64;
}

/* C3/C5 */
static uint32_t gen_imix(uint64_t seed, uint64_t i, uint8_t *p)
{
	rng r = seed_for(seed, i);
	uint32_t sz, k = rnd(&r, 12);
	int vlan, l4;
	uint32_t l3, l4o, tot;

	sz = k < 7 ? 64 : k < 11 ? 576 : 1500;
	vlan = rnd(&r, 2);
	l4 = rnd(&r, 3);   /* 0 TCP, 1 UDP, 2 ICMP */
	if (!p)
		return sz;

	fill_random(&r, p, sz);
	eth_hdr(p, &r, vlan ? 0x8100 : 0x0800, 0);
	l3 = 14;
	if (vlan) {
		uint16_t tci = (uint16_t)next(&r);
		put16(p + 14, tci);
		put16(p + 16, 0x0800);
		l3 = 18;
	}
	tot = sz - l3;
	ipv4_hdr(p + l3, (uint16_t)tot, (uint16_t)next(&r), (uint8_t)(1 + rnd(&r, 255)),
		 l4 == 0 ? 6 : l4 == 1 ? 17 : 1, (uint32_t)next(&r), (uint32_t)next(&r),
		 (uint8_t)rnd(&r, 4) << 2);
	l4o = l3 + 20;
	if (l4 == 0) {
		p[l4o + 12] = 0x50;             /* doff 5, res 0 */
		p[l4o + 13] = (uint8_t)next(&r);
	} else if (l4 == 1) {
		put16(p + l4o + 4, (uint16_t)(tot - 20));
	} else {
		p[l4o] = rnd(&r, 2) ? 8 : 0;    /* echo request / reply */
		p[l4o + 1] = 0;
		put16(p + l4o + 2, 0);
		/* valid checksum over the whole ICMP message; the dissector folds
		 * LE words and drops an odd byte, so make the message even */
		put16(p + l4o + 2, inet_csum(p + l4o, tot - 20));
		if (rnd(&r, 64) == 0)
			p[l4o + 2] ^= 0x5a;         /* ~1.5% bogus */
	}
	return sz;
}

/* C4 ---------------------------------------------------------------------- */
enum { X_HBH, X_DST, X_RT, X_FRAG, X_AH, X_MOB, X_N };
static const uint8_t x_proto[X_N] = { 0, 60, 43, 44, 51, 135 };

typedef struct {
	int kind;
	uint32_t len;       /* bytes of this header */
	uint8_t hl;         /* hdr_ext_len / payload_len field */
	uint8_t sub;        /* routing type / mobility type */
	uint8_t naddr;
} xhdr;

static uint32_t gen_ipv6x(uint64_t seed, uint64_t i, uint8_t *p)
{
	rng r = seed_for(seed, i);
	xhdr x[6];
	int depth = (int)rnd(&r, 7), term = (int)rnd(&r, 5), bad = rnd(&r, 100) == 0;
	int badk = depth ? (int)rnd(&r, depth) : 0;
	uint32_t hdr = 14 + 40, sz, want = 64 + rnd(&r, 1500 - 64 + 1);
	static const uint8_t t_proto[5] = { 6, 17, 58, 59, 50 };
	static const uint32_t t_len[5] = { 20, 8, 8, 0, 8 };

	for (int k = 0; k < depth; k++) {
		xhdr *h = &x[k];
		h->kind = (int)rnd(&r, X_N);
		h->sub = 0;
		h->naddr = 0;
		switch (h->kind) {
		case X_HBH: case X_DST:
			h->hl = (uint8_t)rnd(&r, 4);
			h->len = (h->hl + 1u) * 8;
			break;
		case X_RT:
			if (rnd(&r, 2)) {
				h->sub = 0;
				h->naddr = (uint8_t)rnd(&r, 5);
				h->hl = (uint8_t)(2 * h->naddr);
			} else {
				h->sub = 4;
				h->hl = (uint8_t)rnd(&r, 4);
			}
			h->len = (h->hl + 1u) * 8;
			break;
		case X_FRAG:
			h->hl = 0;
			h->len = 8;
			break;
		case X_AH:
			h->hl = (uint8_t)(1 + rnd(&r, 6));   /* hdr_len = hl*4+8 >= 12 */
			h->len = h->hl * 4u + 8;
			break;
		case X_MOB: {
			static const uint8_t minhl[7] = { 0, 1, 1, 2, 2, 1, 1 };
			h->sub = (uint8_t)rnd(&r, 7);
			h->hl = (uint8_t)(minhl[h->sub] + rnd(&r, 4 - minhl[h->sub]));
			h->len = (h->hl + 1u) * 8;
			break;
		}
		}
		hdr += h->len;
	}
	hdr += t_len[term];
	sz = want > hdr ? want : hdr;
	if (sz & 1)
		sz++;                       /* keep ICMPv6/ICMP sums simple */
	if (!p)
		return sz;

	fill_random(&r, p, sz);
	eth_hdr(p, &r, 0x86DD, 0);
	{
		uint8_t *ip = p + 14;
		uint64_t v = next(&r);
		ip[0] = (uint8_t)(0x60 | (v & 0xF));
		ip[1] = (uint8_t)(v >> 8); ip[2] = (uint8_t)(v >> 16); ip[3] = (uint8_t)(v >> 24);
		put16(ip + 4, (uint16_t)(sz - 54));
		ip[6] = depth ? x_proto[x[0].kind] : t_proto[term];
		ip[7] = 64;
		/* addresses with zero runs so inet_ntop's "::" compression shows */
		memset(ip + 8, 0, 32);
		put16(ip + 8, 0x2001); put16(ip + 10, 0x0db8);
		put16(ip + 22, (uint16_t)v); put32(ip + 20, (uint32_t)(v >> 16));
		put16(ip + 24, 0xfe80);
		if ((v >> 40) & 1)
			put32(ip + 36, (uint32_t)next(&r));
		else {
			put16(ip + 34, 0xffff);
			put32(ip + 36, (uint32_t)next(&r));
			memset(ip + 24, 0, 10);
		}
	}
	{
		uint32_t o = 54;
		for (int k = 0; k < depth; k++) {
			xhdr *h = &x[k];
			uint8_t *q = p + o;
			uint8_t nh = k + 1 < depth ? x_proto[x[k + 1].kind] : t_proto[term];
			q[0] = nh;
			switch (h->kind) {
			case X_HBH: case X_DST:
				q[1] = h->hl;
				break;
			case X_RT:
				q[1] = h->hl; q[2] = h->sub; q[3] = (uint8_t)rnd(&r, 5);
				if (h->sub == 0)
					for (int a = 0; a < h->naddr; a++) {
						uint8_t *ad = q + 8 + 16 * a;
						memset(ad, 0, 16);
						put16(ad, 0x2001); put16(ad + 2, 0x0db8);
						put16(ad + 14, (uint16_t)(a + 1));
					}
				break;
			case X_FRAG:
				q[1] = 0;
				break;
			case X_AH:
				q[1] = h->hl;
				break;
			case X_MOB:
				q[1] = h->hl; q[2] = h->sub;
				break;
			}
			if (bad && k == badk)
				q[1] = (uint8_t)(200 + rnd(&r, 56));  /* length beyond the frame */
			o += h->len;
		}
		if (term == 2) {                 /* ICMPv6 echo */
			p[o] = rnd(&r, 2) ? 128 : 129;
			p[o + 1] = 0;
		}
	}
	return sz;
}

static uint32_t gen(int cfg, uint64_t seed, uint64_t i, uint8_t *p)
{
	switch (cfg) {
	case NSD_SYN_UDP64: return gen_udp64(seed, i, p);
	case NSD_SYN_IMIX:  return gen_imix(seed, i, p);
	case NSD_SYN_IPV6X: return gen_ipv6x(seed, i, p);
	}
	return 0;
}

/* Descriptors for packets [lo, lo+n): frames packed at `align`-byte
 * boundaries (align a power of two >= 1) starting at byte `base`.
 * Returns the end offset (buffer bytes needed, without NSD_FRAME_PAD). */
uint64_t nsd_synth_layout(int cfg, uint64_t seed, uint64_t lo, uint64_t n,
			  uint32_t align, uint64_t base, nsd_desc_t *desc)
{
	uint64_t off = base;
	if (!align)
		align = 1;
	for (uint64_t k = 0; k < n; k++) {
		uint32_t sz = gen(cfg, seed, lo + k, NULL);
		off = (off + align - 1) & ~(uint64_t)(align - 1);
		if (desc)
			desc[k] = NSD_DESC(off, sz);
		off += sz;
	}
	return off;
}

typedef struct {
	int cfg;
	uint64_t seed, lo, a, b;
	uint8_t *frames;
	const nsd_desc_t *desc;
} fill_job;

static void *fill_worker(void *arg)
{
	fill_job *j = arg;
	for (uint64_t k = j->a; k < j->b; k++)
		gen(j->cfg, j->seed, j->lo + k, j->frames + NSD_DESC_OFF(j->desc[k]));
	return NULL;
}

/* Fill the frames of packets [lo, lo+n) at the offsets in desc. */
void nsd_synth_fill(int cfg, uint64_t seed, uint64_t lo, uint64_t n, uint8_t *frames,
		    const nsd_desc_t *desc, int nthreads)
{
	pthread_t th[64];
	fill_job jobs[64];
	if (nthreads < 1) nthreads = 1;
	if (nthreads > 64) nthreads = 64;
	for (int t = 0; t < nthreads; t++) {
		jobs[t] = (fill_job){ cfg, seed, lo, n * t / nthreads, n * (t + 1) / nthreads, frames, desc };
		pthread_create(&th[t], NULL, fill_worker, &jobs[t]);
	}
	for (int t = 0; t < nthreads; t++)
		pthread_join(th[t], NULL);
}

/* Write packets [lo, lo+n) as a classic LE pcap (magic 0xa1b2c3d4, v2.4,
 * linktype 1), ts = (i, 0). Returns bytes written or 0 on error. */
uint64_t nsd_synth_pcap(int cfg, uint64_t seed, uint64_t lo, uint64_t n, const char *path)
{
	FILE *f = fopen(path, "wb");
	uint8_t buf[2048];
	uint64_t total = 0;
	struct { uint32_t magic; uint16_t vmaj, vmin; int32_t zone; uint32_t sig, snap, lt; } fh =
		{ 0xa1b2c3d4u, 2, 4, 0, 0, 65535, 1 };
	if (!f)
		return 0;
	fwrite(&fh, sizeof(fh), 1, f);
	total += sizeof(fh);
	for (uint64_t k = 0; k < n; k++) {
		uint32_t sz = gen(cfg, seed, lo + k, buf);
		uint32_t rh[4] = { (uint32_t)(lo + k), 0, sz, sz };
		fwrite(rh, sizeof(rh), 1, f);
		fwrite(buf, 1, sz, f);
		total += sizeof(rh) + sz;
	}
	fclose(f);
	return total;
}
