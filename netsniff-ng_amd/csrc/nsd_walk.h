// nsd_walk.h - the device chain walk: one lane walks one packet through the
// netsniff-ng dissector chain and produces the 16-byte chain record.
//
// This is the parse semantics of the reference parsers without their text
// (text is rendered on the host from record + raw bytes, nsd_format.cpp):
// per layer it advances the pkt_buff cursor exactly as the reference does,
// computes the values that decide later output (IPv4 header checksum,
// ICMPv4 checksum, IPv4 tail trim) and looks up the next ops by key.
// References are given per layer (file:line of the reference parser).
//
// The byte source is a template parameter (Src) so the same walk runs over an
// LDS-staged header window with a global-memory fallback.
#pragma once
#include <stdint.h>
#include "../../include/netsniff_dissect.h"

namespace nsd {

// dissector_eth.c:30-39 (eth_lay2): exact-key map -> ops id
__device__ __forceinline__ int lay2(uint32_t key)
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

// dissector_eth.c:44-60 (eth_lay3) as a 256-entry table in constant memory
__constant__ uint8_t c_lay3[256] = {
	/*   0 */ NSD_OPS_IPV6_HOP_BY_HOP, NSD_OPS_ICMPV4, NSD_OPS_IGMP, 0, 0, 0, NSD_OPS_TCP, 0,
	/*   8 */ 0, 0, 0, 0, 0, 0, 0, 0,
	/*  16 */ 0, NSD_OPS_UDP, 0, 0, 0, 0, 0, 0,
	/*  24 */ 0, 0, 0, 0, 0, 0, 0, 0,
	/*  32 */ 0, NSD_OPS_DCCP, 0, 0, 0, 0, 0, 0,
	/*  40 */ 0, NSD_OPS_IPV6_IN_IPV4, 0, NSD_OPS_IPV6_ROUTING, NSD_OPS_IPV6_FRAGM, 0, 0, 0,
	/*  48 */ 0, 0, NSD_OPS_IP_ESP, NSD_OPS_IP_AUTH, 0, 0, 0, 0,
	/*  56 */ 0, 0, NSD_OPS_ICMPV6, NSD_OPS_IPV6_NO_NEXT, NSD_OPS_IPV6_DEST_OPTS, 0, 0, 0,
	/*  64 */ 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
	/*  80 */ 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
	/*  96 */ 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
	/* 112 */ 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
	/* 128 */ 0, 0, 0, 0, 0, 0, 0, NSD_OPS_IPV6_MOBILITY, 0, 0, 0, 0, 0, 0, 0, 0,
};

// the walk looks eth_lay3 up through its byte source (s.lay3(key)), which
// serves it from an LDS copy of c_lay3: a per-lane constant-memory read would
// be a vector-memory load inside the walk

// Per-packet walk output (kept in registers).
struct WalkOut {
	uint32_t data, tail;
	uint32_t n;          // layers run
	uint32_t chain;      // first 6 ids, 5 bits each
	uint64_t offA;       // offsets of layers 0..3 (16 bits each)
	uint32_t offB;       // offsets of layers 4..5
	uint16_t ip_csum;
	uint8_t  flags;      // NSD_F_*
	bool     need_ext;   // more than 6 layers or a layer start > 510
	uint32_t slot;       // ext slot (valid when ext_on)
	bool     ext_on;
	int      id;         // next ops to run (0 = chain ended)
	bool     icmp_pend;  // ICMPv4 checksum left to the wave-cooperative pass
	uint32_t icmp_off, icmp_len;
};

// Ext spill: the first time a packet needs the ext form it takes a slot in
// its block's scratch table (LDS counter, one add per group of lanes reaching
// that point together) and copies the layers collected so far; later layers
// go straight to the slot.  The block compacts its scratch entries into the
// caller's ext table when it finishes (one global atomic per block, see
// ext_compact in nsd_kernels.hip): a global slot counter bumped per wave
// serialises every wave of the chip on one word.
struct ExtSink {
	nsd_ext *scr;        // this block's scratch entries (room for every packet it walks)
	uint32_t *s_n;       // LDS: scratch entries taken
};

__device__ __forceinline__ uint16_t off_of(const WalkOut &w, uint32_t k)
{
	return k < 4 ? (uint16_t)(w.offA >> (16 * k)) : (uint16_t)(w.offB >> (16 * (k - 4)));
}

__device__ __forceinline__ void record_layer(WalkOut &w, int id, const ExtSink &es)
{
	const uint32_t k = w.n;
	if (k < NSD_REC_MAX_LAYERS) {
		w.chain |= (uint32_t)id << (5 * k);
		if (k < 4)
			w.offA |= (uint64_t)(w.data & 0xFFFF) << (16 * k);
		else
			w.offB |= (w.data & 0xFFFF) << (16 * (k - 4));
		if (k >= 1 && w.data > 510)
			w.need_ext = true;
	} else {
		w.need_ext = true;
	}
	// scratch slot: one LDS atomic per group of lanes reaching this point
	// together (ballot / shfl / mbcnt over the active lanes).  Only the used
	// prefix of the entry is written (the layers past nlayers are undefined).
	const bool want = w.need_ext && !w.ext_on;
	const uint64_t wm = __ballot(want);
	if (wm) {
		const int leader = __ffsll((unsigned long long)wm) - 1;
		uint32_t sb = 0;
		if ((int)__lane_id() == leader)
			sb = atomicAdd(es.s_n, (uint32_t)__popcll(wm));
		sb = __shfl(sb, leader, 64);
		sb += __builtin_amdgcn_mbcnt_hi((uint32_t)(wm >> 32),
						__builtin_amdgcn_mbcnt_lo((uint32_t)wm, 0));
		if (want) {
			nsd_ext *e = es.scr + sb;
			const uint32_t m = k < NSD_REC_MAX_LAYERS ? k : NSD_REC_MAX_LAYERS;
			for (uint32_t j = 0; j < m; j++) {
				e->id[j] = (uint8_t)((w.chain >> (5 * j)) & 31);
				e->off[j] = off_of(w, j);
			}
			w.slot = sb;
			w.ext_on = true;
		}
	}
	if (w.ext_on) {
		if (k < NSD_EXT_MAX_LAYERS) {
			es.scr[w.slot].id[k] = (uint8_t)id;
			es.scr[w.slot].off[k] = (uint16_t)w.data;
		} else {
			w.flags |= NSD_F_OVERFLOW;
		}
	}
	w.n = k + 1;
}

// csum() (csum.h:12-22) over `nwords` little-endian u16 words from `off`
template <class Src>
__device__ __forceinline__ uint16_t calc_csum(const Src &s, uint32_t off, uint32_t nwords)
{
	uint32_t sum = s.sum16(off, nwords);   // <= 32767 words * 0xffff fits in 32 bits
	sum = (sum >> 16) + (sum & 0xffff);
	sum += (sum >> 16);
	return (uint16_t)~sum;
}

// Walk state initialisation (pkt_alloc: data = head, tail = head + len).
__device__ __forceinline__ void walk_init(WalkOut &w, uint32_t caplen, int start_id)
{
	w.data = 0;
	w.tail = caplen;
	w.n = 0;
	w.chain = 0;
	w.offA = 0;
	w.offB = 0;
	w.ip_csum = 0;
	w.flags = 0;
	w.need_ext = false;
	w.ext_on = false;
	w.slot = 0;
	w.id = start_id;
	w.icmp_pend = false;
	w.icmp_off = 0;
	w.icmp_len = 0;
}

// The walk (dissector_main's loop, dissector.c:51-58).  MODE is PRINT_NORM
// or PRINT_LESS (parse semantics differ).  Runs layers until the chain ends
// or, when `resumable`, until the next layer starts too close to the end of
// the source's staged window (returns true: restage at w.data and call again).
// Cnt: per-ops counter hook cnt(id).
//
// FAST (the first-pass kernel): instead of suspending, spilling to the ext
// table or deferring an ICMP checksum, the walk gives up (returns true) and
// the packet is queued for the general kernel, which walks it from scratch;
// counting is left to the caller (from the finished record).
template <int MODE, bool FAST, class Src, class Cnt>
__device__ __forceinline__ bool walk(const Src &s, uint32_t caplen, const ExtSink &es, WalkOut &w,
				     Cnt &&cnt)
{
	(void)caplen;
	while (w.id) {
		const int id = w.id;
		if (s.near_end(w.data, id))
			return true;
		if constexpr (FAST) {
			if (w.n >= NSD_REC_MAX_LAYERS || (w.n >= 1 && w.data > 510))
				return true;
			w.chain |= (uint32_t)id << (5 * w.n);
			if (w.n < 4)
				w.offA |= (uint64_t)w.data << (16 * w.n);
			else
				w.offB |= w.data << (16 * (w.n - 4));
			w.n++;
		} else {
			record_layer(w, id, es);
			cnt(w.n <= NSD_EXT_MAX_LAYERS ? id : -1);   // the oracle counts the first 64 layers
		}
		const uint32_t start = w.data;
		const uint32_t len = w.tail - w.data;   // pkt_len (pkt_buff.h:36-41)
		int next = 0;
		switch (id) {
		case NSD_OPS_ETHERNET:      // proto_ethernet.c:48-79
			if (len >= 14) {
				next = lay2(s.be16(start + 12));
				w.data = start + 14;
			}
			break;
		case NSD_OPS_VLAN:          // proto_vlan.c:22-40
		case NSD_OPS_QINQ:          // proto_vlan_q_in_q.c:23-41
			if (len >= 4) {
				next = lay2(s.be16(start + 2));
				w.data = start + 4;
			}
			break;
		case NSD_OPS_MPLS_UC: {     // proto_mpls_unicast.c:49-77
			uint32_t d = start, l = len;
			bool ok = true;
			for (;;) {
				if (l < 4) { ok = false; break; }
				uint8_t sbit = s.b(d + 2) & 1;
				d += 4; l -= 4;
				if (sbit) break;
			}
			w.data = d;
			if (ok && l) {
				uint8_t nib = s.b(d) >> 4;   // mpls_uc_next_proto :23-47
				next = nib == 4 ? NSD_OPS_IPV4 : nib == 6 ? NSD_OPS_IPV6 : 0;
			}
			break;
		}
		case NSD_OPS_IPV4: {        // proto_ipv4.c:34-178 / 180-204
			if (len < 20)
				break;
			const uint8_t ihl = s.b(start) & 0xF;
			const uint32_t proto = s.b(start + 9);
			uint32_t d = start + 20, l = len - 20;
			const uint32_t opts = (ihl > 5 ? ihl : 5) * 4u - 20u;
			if (MODE == PRINT_NORM) {
				// checksum over ihl*4 bytes, past the frame too (bytes >= caplen are 0)
				w.ip_csum = calc_csum(s, start, ihl * 2u);
			}
			if (opts <= l) { d += opts; l -= opts; }
			w.data = d;
			if (MODE == PRINT_NORM) {
				// trim to tot_len - ihl*4, evaluated in size_t (:174-175)
				const int64_t x = (int64_t)s.be16(start + 2) - (int64_t)ihl * 4;
				if (x >= 0 && (uint64_t)x < l)
					w.tail = d + (uint32_t)x;
			}
			next = s.lay3(proto);
			break;
		}
		case NSD_OPS_IPV6:          // proto_ipv6.c:22-105
		case NSD_OPS_IPV6_IN_IPV4:  // proto_ipv6_in_ipv4.c:20-24
			if (len >= 40) {
				next = s.lay3(s.b(start + 6));
				w.data = start + 40;
			}
			break;
		case NSD_OPS_IPV6_HOP_BY_HOP:   // proto_ipv6_hop_by_hop.c:39-71
		case NSD_OPS_IPV6_DEST_OPTS: {  // proto_ipv6_dest_opts.c:40-72
			if (len < 2)
				break;
			const uint32_t opt_len = (s.b(start + 1) + 1u) * 8u - 2u;
			w.data = start + 2;
			if (opt_len <= len - 2) {
				w.data += opt_len;
				next = s.lay3(s.b(start));
			}
			break;
		}
		case NSD_OPS_IPV6_ROUTING: {    // proto_ipv6_routing.c:79-122
			if (len < 4)
				break;
			const uint32_t data_len = (s.b(start + 1) + 1u) * 8u - 4u;
			w.data = start + 4;
			if (data_len <= len - 4) {
				// type 0 pulls reserved + addresses, then the rest: same total
				w.data += data_len;
				next = s.lay3(s.b(start));
			}
			break;
		}
		case NSD_OPS_IPV6_FRAGM:    // proto_ipv6_fragm.c:25-47
			if (len >= 8) {
				next = s.lay3(s.b(start));
				w.data = start + 8;
			}
			break;
		case NSD_OPS_IP_AUTH: {     // proto_ip_authentication_hdr.c:26-69
			if (len < 12)
				break;
			const uint32_t hdr_len = s.b(start + 1) * 4u + 8u;
			w.data = start + 12;
			if (hdr_len <= len - 12) {
				if (hdr_len > 12)
					w.data += hdr_len - 12;   // ICV bytes pulled one by one
				next = s.lay3(s.b(start));
			}
			break;
		}
		case NSD_OPS_IP_ESP:        // proto_ip_esp.c:23-35: leaf
			if (len >= 8)
				w.data = start + 8;
			break;
		case NSD_OPS_IPV6_NO_NEXT:  // proto_ipv6_no_nxt_hdr.c:17-29: leaf, no pull
			break;
		case NSD_OPS_IPV6_MOBILITY: {   // proto_ipv6_mobility_hdr.c:247-309
			if (len < 6)
				break;
			const int32_t hdr_ext_len = (s.b(start + 1) + 1) * 8;
			int32_t mdl = hdr_ext_len - 6;
			uint32_t d = start + 6, l = len - 6;
			if (mdl > (int32_t)l)
				{ w.data = d; break; }
			if (MODE == PRINT_NORM) {
				// get_mh_type (:206-245): subtype pull, then the length check
				const uint8_t type = s.b(start + 2);
				int32_t sub = 0;
				bool dec_on_fail = true;
				switch (type) {
				case 0: sub = 2; break;
				case 1: case 2: sub = 10; break;
				case 3: case 4: sub = 18; break;
				case 5: sub = 6; break;
				case 6: sub = 6; dec_on_fail = false; break;
				case 7: sub = 10; dec_on_fail = false; break;
				}
				if (sub) {
					const bool ok = (uint32_t)sub <= l;
					if (ok) { d += sub; l -= sub; }
					if (ok || dec_on_fail)
						mdl -= sub;
				}
				if (mdl > (int32_t)l || mdl < 0)
					{ w.data = d; break; }
			}
			w.data = d + (uint32_t)mdl;
			next = s.lay3(s.b(start));
			break;
		}
		case NSD_OPS_TCP:           // proto_tcp.c:63-107: leaf, options not pulled
			if (len >= 20)
				w.data = start + 20;
			break;
		case NSD_OPS_UDP:           // proto_udp.c:23-58: leaf
			if (len >= 8)
				w.data = start + 8;
			break;
		case NSD_OPS_ICMPV4:        // proto_icmpv4.c:34-51: leaf
			if (len >= 8) {
				w.data = start + 8;
				if (MODE == PRINT_NORM) {
					// calc_csum(icmp, pkt_len + 8): the whole (post-trim)
					// message, odd trailing byte dropped (csum.h:24-27).
					// Short messages inside the staged window are summed
					// here; longer ones by the whole wave afterwards.
					if (s.in_window(start, len & ~1u)) {
						if (calc_csum(s, start, len >> 1))
							w.flags |= NSD_F_ICMP_BAD;
					} else if constexpr (FAST) {
						return true;
					} else {
						w.icmp_pend = true;
						w.icmp_off = start;
						w.icmp_len = len;
					}
				}
			}
			break;
		case NSD_OPS_ICMPV6: {      // proto_icmpv6.c:1667-1699: leaf
			if (len < 4)
				break;
			w.data = start + 4;
			if (MODE == PRINT_NORM) {
				const uint8_t type = s.b(start);
				if (type >= 130 && type <= 154) {
					// variable-length body (:372-911, :1023-1490): host renders
					w.flags |= NSD_F_HOST;
					w.data = start;
				} else if ((type >= 1 && type <= 4) || type == 128 || type == 129) {
					if (len - 4 >= 4)
						w.data = start + 8;
				}
			}
			break;
		}
		default:
			// ARP, LLDP, IGMP, DCCP and non-Ethernet heads: host-rendered leaves
			w.flags |= NSD_F_HOST;
			w.data = start;
			break;
		}
		if constexpr (FAST) {
			if (s.missed())   // a byte outside the staged window was needed
				return true;
		}
		w.id = next;
	}
	return false;
}

// Straight-line walk for the common chains (pass 1): Ethernet, up to two
// 802.1Q / 802.1ad tags, IPv4 or IPv6, then TCP / UDP / ICMPv4 / ICMPv6 /
// ESP / NoNext (or a host-rendered leaf: ARP, LLDP, IGMP, DCCP).  Same
// semantics as walk() for every packet it finishes (the per-layer comments
// there cite the reference); anything else (MPLS, deeper tag stacks,
// extension headers, IPv6-in-IPv4, bytes past the staged window) returns true
// and the packet goes to pass 2.  No loop, no per-layer dispatch switch.
template <int MODE, class Src>
__device__ __forceinline__ bool fast_walk(const Src &s, uint32_t caplen, WalkOut &w)
{
	uint32_t n = 0;
	auto rec = [&](int id, uint32_t at) {
		w.chain |= (uint32_t)id << (5 * n);
		if (n < 4)
			w.offA |= (uint64_t)at << (16 * n);
		else
			w.offB |= at << (16 * (n - 4));
		n++;
	};
	if (w.id != NSD_OPS_ETHERNET)
		return true;   // other link types: pass 2
	rec(NSD_OPS_ETHERNET, 0);
	if (caplen < 14) {
		w.n = n;
		return false;
	}
	uint32_t d = 14;
	int next = lay2(s.be16(12));
#pragma unroll
	for (int t = 0; t < 2; t++) {
		if (next != NSD_OPS_VLAN && next != NSD_OPS_QINQ)
			break;
		rec(next, d);
		if (caplen - d < 4) {
			w.data = d;
			w.n = n;
			return s.missed();
		}
		next = lay2(s.be16(d + 2));
		d += 4;
	}
	w.data = d;
	uint32_t d2;
	int l4;
	if (next == NSD_OPS_IPV4) {
		rec(NSD_OPS_IPV4, d);
		if (caplen - d < 20) {
			w.n = n;
			return s.missed();
		}
		const uint32_t ihl = s.b(d) & 0xF;
		const uint32_t proto = s.b(d + 9);
		if (MODE == PRINT_NORM) {
			if (!s.in_window(d, ihl * 4u))
				return true;
			w.ip_csum = calc_csum(s, d, ihl * 2u);
		}
		d2 = d + 20;
		uint32_t l = caplen - d2;
		const uint32_t opts = (ihl > 5 ? ihl : 5) * 4u - 20u;
		if (opts <= l) { d2 += opts; l -= opts; }
		if (MODE == PRINT_NORM) {
			const int32_t x = (int32_t)s.be16(d + 2) - (int32_t)(ihl * 4);
			if (x >= 0 && (uint32_t)x < l)
				w.tail = d2 + (uint32_t)x;
		}
		l4 = s.lay3(proto);
	} else if (next == NSD_OPS_IPV6) {
		rec(NSD_OPS_IPV6, d);
		if (caplen - d < 40) {
			w.n = n;
			return s.missed();
		}
		d2 = d + 40;
		l4 = s.lay3(s.b(d + 6));
	} else if (next == NSD_OPS_ARP || next == NSD_OPS_LLDP) {
		rec(next, d);
		w.flags |= NSD_F_HOST;
		w.n = n;
		return s.missed();
	} else if (next == 0) {
		w.n = n;
		return s.missed();
	} else {
		return true;   // MPLS, a third tag
	}
	w.data = d2;
	const uint32_t len = w.tail - d2;
	switch (l4) {
	case 0:
		break;
	case NSD_OPS_TCP:
		rec(l4, d2);
		if (len >= 20) w.data = d2 + 20;
		break;
	case NSD_OPS_UDP:
	case NSD_OPS_IP_ESP:
		rec(l4, d2);
		if (len >= 8) w.data = d2 + 8;
		break;
	case NSD_OPS_IPV6_NO_NEXT:
		rec(l4, d2);
		break;
	case NSD_OPS_ICMPV4:
		rec(l4, d2);
		if (len >= 8) {
			w.data = d2 + 8;
			if (MODE == PRINT_NORM) {
				if (!s.in_window(d2, len & ~1u)) {
					// message past the window: the wave sums it after the walk
					w.icmp_pend = true;
					w.icmp_off = d2;
					w.icmp_len = len;
				} else if (calc_csum(s, d2, len >> 1)) {
					w.flags |= NSD_F_ICMP_BAD;
				}
			}
		}
		break;
	case NSD_OPS_ICMPV6:
		rec(l4, d2);
		if (len >= 4) {
			w.data = d2 + 4;
			if (MODE == PRINT_NORM) {
				const uint8_t type = s.b(d2);
				if (type >= 130 && type <= 154) {
					w.flags |= NSD_F_HOST;
					w.data = d2;
				} else if (((type >= 1 && type <= 4) || type == 128 || type == 129) && len - 4 >= 4) {
					w.data = d2 + 8;
				}
			}
		}
		break;
	case NSD_OPS_IGMP:
	case NSD_OPS_DCCP:
		rec(l4, d2);
		w.flags |= NSD_F_HOST;
		break;
	default:
		return true;   // extension headers, AH, IPv6-in-IPv4
	}
	w.n = n;
	return s.missed();
}

} // namespace nsd
