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
// The byte source (Src) and the sink for what a layer records (Sink) are
// template parameters, so the same layer step runs
//   * on the device over an LDS-staged header window (the general walk of
//     nsd_kernels.hip: wave-level sinks, ballots, LDS counters), and
//   * on the host over the whole frame (nsd_cpu.hip: the per-packet entry
//     point dissector_entry_point and the exported proto-ops objects, which
//     SURVEY 8b keeps on the CPU: one packet per call is all launch latency).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>
#include "../../include/netsniff_dissect.h"

#define NSD_HD __host__ __device__ __forceinline__

#include "nsd_leaf.h"

namespace nsd {

// dissector_eth.c:30-39 (eth_lay2): exact-key map -> ops id
NSD_HD int lay2(uint32_t key)
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

// dissector_eth.c:44-60 (eth_lay3) as a 256-entry table: constant memory on
// the device, a plain array on the host (same initialiser)
#define NSD_LAY3_TABLE { \
	/*   0 */ NSD_OPS_IPV6_HOP_BY_HOP, NSD_OPS_ICMPV4, NSD_OPS_IGMP, 0, 0, 0, NSD_OPS_TCP, 0, \
	/*   8 */ 0, 0, 0, 0, 0, 0, 0, 0, \
	/*  16 */ 0, NSD_OPS_UDP, 0, 0, 0, 0, 0, 0, \
	/*  24 */ 0, 0, 0, 0, 0, 0, 0, 0, \
	/*  32 */ 0, NSD_OPS_DCCP, 0, 0, 0, 0, 0, 0, \
	/*  40 */ 0, NSD_OPS_IPV6_IN_IPV4, 0, NSD_OPS_IPV6_ROUTING, NSD_OPS_IPV6_FRAGM, 0, 0, 0, \
	/*  48 */ 0, 0, NSD_OPS_IP_ESP, NSD_OPS_IP_AUTH, 0, 0, 0, 0, \
	/*  56 */ 0, 0, NSD_OPS_ICMPV6, NSD_OPS_IPV6_NO_NEXT, NSD_OPS_IPV6_DEST_OPTS, 0, 0, 0, \
	/*  64 */ 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, \
	/*  80 */ 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, \
	/*  96 */ 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, \
	/* 112 */ 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, \
	/* 128 */ 0, 0, 0, 0, 0, 0, 0, NSD_OPS_IPV6_MOBILITY, 0, 0, 0, 0, 0, 0, 0, 0, \
}
static __constant__ uint8_t c_lay3[256] = NSD_LAY3_TABLE;
static const uint8_t h_lay3[256] = NSD_LAY3_TABLE;

// the walk looks eth_lay3 up through its byte source (s.lay3(key)), which
// serves it from an LDS copy of c_lay3: a per-lane constant-memory read would
// be a vector-memory load inside the walk

// Per-packet walk output (kept in registers).
struct WalkOut {
	uint32_t data, tail;
	uint32_t n;          // layers run
	uint32_t chain;      // first 6 ids, 5 bits each
	uint64_t offA;       // offsets of layers 0..3 (16 bits each)
	uint32_t offB;       // offsets of layers 4..5; compact records (no offsets):
	                     // ids 6..11, 5 bits each (the side word)
	uint16_t ip_csum;
	uint8_t  flags;      // NSD_F_*
	bool     need_ext;   // more than 6 layers or a layer start > 510
	uint32_t slot;       // ext slot (valid when ext_on)
	bool     ext_on;
	int      id;         // next ops to run (0 = chain ended)
	bool     icmp_pend;  // ICMPv4 checksum left to the wave-cooperative pass
	uint32_t icmp_off, icmp_len;
	uint32_t icmp_sum;   // split schedule: sum of the message words before icmp_off (fast_walk<.., true>)
	int      leaf;       // device: a host-rendered leaf at w.data whose end is still to walk
};

// Where the general walk puts what it records beyond the record's 6 layers:
// 16-byte records (CR false) keep layers 6 .. 6+NSD_LDS_LAYERS-1 (id and
// start) in a per-lane LDS list, written out with the packet's pool entry
// when its walk ends; compact records (CR) keep no layer starts at all (the
// renderer re-derives them), so their ids 6..11 stay in a register
// (offB, free in that form: the side word).  Deeper layers go straight into the packet's pool
// entry (taken when the chain reaches that depth).  Pool words come from
// per-wave chunks (ext_take).
#define NSD_LDS_LAYERS 6
template <bool CR>
struct GenSink {
	static constexpr bool OFFS = !CR;   // the walk tracks layer starts
	uint32_t *pool;               // the ext pool
	uint32_t pool_words;
	uint32_t *used;               // pool words handed out (global)
	uint32_t chunk;               // words per chunk request
	uint32_t *wc;                 // LDS: this wave's chunk {next word, words left}
	uint32_t *s_ops;              // LDS: block per-ops layer counts
	uint32_t *lay;                // LDS: this wave's layer lists, [j * 64 + lane]
	uint32_t sbase;               // first pool word handed out (compact records: the
	                              // side words [0, n) come first)
	uint32_t *side;               // compact records: side word of packet i (or null)

	// a chain reaching layer 6 + NSD_LDS_LAYERS takes its pool entry now (rare)
	__device__ __forceinline__ void take_deep(bool deep_first, WalkOut &w) const;
	// count layer k (ops id, start offset) and keep it beyond the record
	__device__ __forceinline__ void layer(const WalkOut &w, uint32_t k, int id, uint32_t start) const;
	// a host-rendered leaf ends the chain: its pulls are walked once the
	// lane's chain is done (emit_general), where fewer registers are live
	template <int MODE, class Src>
	__device__ __forceinline__ uint32_t leaf(const Src &, bool lw, WalkOut &w, int id, uint32_t, uint32_t nd) const
	{
		w.leaf = lw ? id : w.leaf;
		return nd;
	}
};

// Wave-uniform call: every lane with `want` gets a pool entry of `words`
// words (consecutive lanes, consecutive entries) from the wave's chunk; a new
// chunk is taken with one global atomic when the current one is short (its
// tail is left unused).  Returns the entry's word index, or 0xFFFFFFFF when
// it does not fit in the pool (or !want).
template <class G>
__device__ __forceinline__ uint32_t ext_take(const G &g, bool want, uint32_t words)
{
	const uint64_t m = __ballot(want);
	if (!m)
		return 0xFFFFFFFFu;
	const int leader = __ffsll((unsigned long long)m) - 1;
	const uint32_t need = (uint32_t)__popcll(m) * words;
	uint32_t base = g.wc[0], left = g.wc[1];
	if (left < need) {
		// +3: the caller's running offset may not be a multiple of 4 (entries
		// are written with 16-byte stores)
		const uint32_t chunk = (g.chunk > need ? g.chunk : need) + 3;
		uint32_t b = 0xFFFFFFFFu;
		// a full pool takes no more chunks, so the counter cannot wrap round
		// into it (the launcher caps pool_words well below 2^32)
		if ((int)__lane_id() == leader &&
		    __hip_atomic_load(g.used, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + g.sbase < g.pool_words)
			b = atomicAdd(g.used, chunk) + g.sbase;
		b = __shfl(b, leader, 64);
		if (b == 0xFFFFFFFFu)
			return 0xFFFFFFFFu;   // the wave's chunk state stays empty
		base = (b + 3) & ~3u;
		left = chunk - (base - b);
	}
	if ((int)__lane_id() == leader) {
		g.wc[0] = base + need;
		g.wc[1] = left - need;
	}
	const uint32_t s = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
							 __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0)) * words;
	return want && (uint64_t)s + words <= g.pool_words ? s : 0xFFFFFFFFu;
}

// the sink's layer store: (16-byte records) layers 6..11 in the wave's LDS
// list, deeper ones in the packet's pool entry (taken by take_deep);
// compact records store only the deeper ones' ids
template <bool CR>
__device__ __forceinline__ void GenSink<CR>::layer(const WalkOut &w, uint32_t k, int id, uint32_t start) const
{
	constexpr uint32_t DEEP = NSD_REC_MAX_LAYERS + NSD_LDS_LAYERS;
	atomicAdd(&s_ops[id], 1u);   // the oracle counts the first 64 layers
	const uint32_t lv = CR ? (uint32_t)id : (uint32_t)id | start << 16;
	if (!CR && k >= NSD_REC_MAX_LAYERS && k < DEEP)
		lay[(k - NSD_REC_MAX_LAYERS) * 64 + __lane_id()] = lv;
	else if (k >= DEEP && w.slot != 0xFFFFFFFFu)
		pool[w.slot + NSD_EXT_HDR_WORDS + k] = lv;
}

template <bool CR>
__device__ __forceinline__ void GenSink<CR>::take_deep(bool deep_first, WalkOut &w) const
{
	if (__ballot(deep_first)) {
		// room for every layer the record may hold (the chain's length is not
		// known yet); the wave-uniform test leaves the entry test to here
		deep_first = deep_first && !w.ext_on;
		const uint32_t sb = ext_take(*this, deep_first, NSD_EXT_WORDS(NSD_EXT_MAX_LAYERS));
		if (deep_first) {
			w.slot = sb;
			w.ext_on = true;
		}
	}
}

// The host walk's sink: every layer into the caller's arrays (the host
// keeps the whole chain, so nothing is taken from a pool while walking)
struct HostSink {
	static constexpr bool OFFS = true;
	uint8_t *ids;                 // [NSD_EXT_MAX_LAYERS]
	uint16_t *offs;               // [NSD_EXT_MAX_LAYERS]
	uint64_t *counters;           // NSD_NCOUNTERS, or NULL

	__host__ void take_deep(bool, WalkOut &) const {}
	__host__ void layer(const WalkOut &, uint32_t k, int id, uint32_t start) const
	{
		ids[k] = (uint8_t)id;
		offs[k] = (uint16_t)start;
		if (counters)
			counters[NSD_CNT_OPS + id]++;
	}
	template <int MODE, class Src>
	__host__ uint32_t leaf(const Src &s, bool lw, WalkOut &w, int id, uint32_t start, uint32_t nd) const
	{
		return lw ? leaf_end<MODE>(s, id, start, w.tail) : nd;
	}
};

NSD_HD uint16_t off_of(const WalkOut &w, uint32_t k)
{
	return k < 4 ? (uint16_t)(w.offA >> (16 * k)) : (uint16_t)(w.offB >> (16 * (k - 4)));
}

// csum() (csum.h:12-22) over `nwords` little-endian u16 words from `off`
template <class Src>
NSD_HD uint16_t calc_csum(const Src &s, uint32_t off, uint32_t nwords)
{
	uint32_t sum = s.sum16(off, nwords);   // <= 32767 words * 0xffff fits in 32 bits
	sum = (sum >> 16) + (sum & 0xffff);
	sum += (sum >> 16);
	return (uint16_t)~sum;
}

// Walk state initialisation (pkt_alloc: data = head, tail = head + len).
NSD_HD void walk_init(WalkOut &w, uint32_t caplen, int start_id)
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
	w.icmp_sum = 0;
	w.leaf = 0;
}

// Per-ops step table for the general walk: the first pull (minl), the fixed
// advance, the rule kind, the byte offset of the next-ops key (kpos; a
// big-endian u16 ethertype looked up in eth_lay2 when kw16, else a u8 looked
// up in eth_lay3) and `need`, the bytes from the layer start its parse
// reads (a lane whose window ends earlier suspends and is restaged; longer
// reads such as IPv4 options or deep MPLS stacks use the byte source's
// global fallback).  Per-ops semantics are cited in gen_step.
enum : uint32_t {
	K_HOST = 0,   // host-rendered leaf: ARP, LLDP, IGMP, DCCP, non-Ethernet heads
	K_CONT = 1,   // fixed pull, continue with the key's ops
	K_LEAF = 2,   // fixed pull, chain ends
	K_IPV4 = 3,
	K_T8 = 4,     // HBH / DestOpts / Routing: (hdr_ext_len + 1) * 8
	K_AH = 5,
	K_MOB = 6,
	K_ICMP6 = 7,
	K_MPLS = 8,
};
#define NSD_STEP(minl, adv, kind, kpos, kw16, need) \
	((minl) | (adv) << 8 | (kind) << 16 | (kpos) << 20 | (kw16) << 24 | (uint32_t)(need) << 25)
#define NSD_STEP_TABLE { \
	/*  0 invalid   */ NSD_STEP(0, 0, K_HOST, 0, 0, 0), \
	/*  1 ethernet  */ NSD_STEP(14, 14, K_CONT, 12, 1, 14), /* proto_ethernet.c:48-79 */ \
	/*  2 vlan      */ NSD_STEP(4, 4, K_CONT, 2, 1, 4), /* proto_vlan.c:22-40 */ \
	/*  3 qinq      */ NSD_STEP(4, 4, K_CONT, 2, 1, 4), /* proto_vlan_q_in_q.c:23-41 */ \
	/*  4 mpls      */ NSD_STEP(0, 0, K_MPLS, 0, 0, 16), /* proto_mpls_unicast.c:49-77 */ \
	/*  5 arp       */ NSD_STEP(0, 0, K_HOST, 0, 0, 0), \
	/*  6 lldp      */ NSD_STEP(0, 0, K_HOST, 0, 0, 0), \
	/*  7 ipv4      */ NSD_STEP(20, 20, K_IPV4, 9, 0, 20), /* proto_ipv4.c:34-178 */ \
	/*  8 ipv6      */ NSD_STEP(40, 40, K_CONT, 6, 0, 8), /* proto_ipv6.c:22-105 */ \
	/*  9 ipv6inv4  */ NSD_STEP(40, 40, K_CONT, 6, 0, 8), /* proto_ipv6_in_ipv4.c:20-24 */ \
	/* 10 icmpv4    */ NSD_STEP(8, 8, K_LEAF, 0, 0, 0), /* proto_icmpv4.c:34-51 */ \
	/* 11 icmpv6    */ NSD_STEP(4, 4, K_ICMP6, 0, 0, 4), /* proto_icmpv6.c:1667-1699 */ \
	/* 12 igmp      */ NSD_STEP(0, 0, K_HOST, 0, 0, 0), \
	/* 13 ah        */ NSD_STEP(12, 12, K_AH, 0, 0, 4), /* proto_ip_authentication_hdr.c:26-69 */ \
	/* 14 esp       */ NSD_STEP(8, 8, K_LEAF, 0, 0, 0), /* proto_ip_esp.c:23-35 */ \
	/* 15 destopts  */ NSD_STEP(2, 2, K_T8, 0, 0, 4), /* proto_ipv6_dest_opts.c:40-72 */ \
	/* 16 fragm     */ NSD_STEP(8, 8, K_CONT, 0, 0, 4), /* proto_ipv6_fragm.c:25-47 */ \
	/* 17 hopbyhop  */ NSD_STEP(2, 2, K_T8, 0, 0, 4), /* proto_ipv6_hop_by_hop.c:39-71 */ \
	/* 18 mobility  */ NSD_STEP(6, 6, K_MOB, 0, 0, 4), /* proto_ipv6_mobility_hdr.c:247-309 */ \
	/* 19 nonext    */ NSD_STEP(0, 0, K_LEAF, 0, 0, 0), /* proto_ipv6_no_nxt_hdr.c:17-29 */ \
	/* 20 routing   */ NSD_STEP(4, 4, K_T8, 0, 0, 4), /* proto_ipv6_routing.c:79-122 */ \
	/* 21 tcp       */ NSD_STEP(20, 20, K_LEAF, 0, 0, 0), /* proto_tcp.c:63-107 (options not pulled) */ \
	/* 22 udp       */ NSD_STEP(8, 8, K_LEAF, 0, 0, 0), /* proto_udp.c:23-58 */ \
	/* 23..31: dccp, none, sll, 802.11, nlmsg, unused: host leaves */ \
}
static __constant__ uint32_t c_step[32] = NSD_STEP_TABLE;
static const uint32_t h_step[32] = NSD_STEP_TABLE;

// eth_lay2 (dissector_eth.c:30-39) as a 32-entry perfect hash for the
// general walk: slot ((key * 0x156) & 0xFFFF) >> 11 holds key | ops << 16
// (one LDS read + compare instead of a 7-way compare tree)
#define NSD_L2H(key) ((((key) * 0x156u) & 0xFFFFu) >> 11)
#define NSD_L2E(key, ops) (NSD_L2H(key) == i ? (key) | (ops) << 16 : 0u)
struct Lay2Hash {
	uint32_t e[32];
	constexpr Lay2Hash() : e()
	{
		for (uint32_t i = 0; i < 32; i++)
			e[i] = NSD_L2E(0x0806, NSD_OPS_ARP) | NSD_L2E(0x88cc, NSD_OPS_LLDP) |
			       NSD_L2E(0x8100, NSD_OPS_VLAN) | NSD_L2E(0x0800, NSD_OPS_IPV4) |
			       NSD_L2E(0x86DD, NSD_OPS_IPV6) | NSD_L2E(0x88a8, NSD_OPS_QINQ) |
			       NSD_L2E(0x8847, NSD_OPS_MPLS_UC);
	}
};
static_assert(NSD_L2H(0x0806) != NSD_L2H(0x88cc) && NSD_L2H(0x8100) != NSD_L2H(0x0800) &&
	      NSD_L2H(0x86DD) != NSD_L2H(0x88a8), "eth_lay2 hash must be perfect");
static __constant__ Lay2Hash c_lay2h;
static constexpr Lay2Hash h_lay2h;

// record words of a finished walk (layout of nsd_rec)
NSD_HD uint4 pack_record(const WalkOut &w)
{
	uint4 r;
	const uint32_t nf = (w.need_ext ? NSD_N_EXT : w.n) | w.flags;
	r.x = w.chain;
	r.y = (w.data & 0xFFFF) | (w.tail << 16);
	if (w.need_ext) {
		const uint32_t slot = w.ext_on ? w.slot : 0xFFFFFFFFu;
		r.z = w.ip_csum | (nf << 16) | ((slot & 0xFF) << 24);
		r.w = slot >> 8;
	} else {
		// layer k start / 2 for k = 1..5 (all even)
		const uint32_t o1 = (uint32_t)(w.offA >> 16) & 0xFFFF, o2 = (uint32_t)(w.offA >> 32) & 0xFFFF;
		const uint32_t o3 = (uint32_t)(w.offA >> 48), o4 = w.offB & 0xFFFF, o5 = w.offB >> 16;
		r.z = w.ip_csum | (nf << 16) | ((o1 >> 1) << 24);
		r.w = (o2 >> 1) | ((o3 >> 1) << 8) | ((o4 >> 1) << 16) | ((o5 >> 1) << 24);
	}
	return r;
}

// The LINKTYPE_LINUX_SLL head's next ops (dissector_sll.c:39-82): in
// print_full a hatype that pcap_devtype_to_linktype (pcap_io.h:205-267) maps
// to LINKTYPE_EN10MB continues in eth_lay2 with ntohs(sll_protocol),
// ARPHRD_NETLINK continues with the netlink ops (a host leaf), anything else
// ends the chain; print_less dispatches nothing.  e2 = the eth_lay2 hash
// entry at NSD_L2H(proto).
NSD_HD int sll_next(uint32_t hatype, uint32_t proto, int mode, uint32_t e2)
{
	if (mode != PRINT_NORM)
		return 0;
	const bool eth = hatype == 1 || hatype == 768 || hatype == 769 || hatype == 772 || hatype == 776 ||
			 hatype == 777 || hatype == 778 || hatype == 823;
	return eth ? ((e2 & 0xFFFF) == proto ? (int)(e2 >> 16) : 0) : hatype == 824 ? NSD_OPS_NLMSG : 0;
}

// get_mh_type's subtype pull sizes for mobility types 0..7
// (proto_ipv6_mobility_hdr.c:206-245), one byte per type
#define NSD_MH_SUB 0x0A060612120A0A02ull

// The general walk (the walkers of nsd_kernels.hip), one layer per call for
// every lane of the wave:
// dissector_main's loop body (dissector.c:51-58) for the ops `w.id`,
// computed as straight-line selects over a per-ops rule table rather than a
// switch, so a wave whose lanes sit at different layers runs one instruction
// stream (a divergent switch runs every case body present plus its exec-mask
// bookkeeping, which made the scalar unit the bottleneck).  The rules of the
// less common kinds and the rare heavy bodies (IPv4 header checksum, ICMPv4
// checksum, MPLS label walk) are branches only the lanes on such a layer take
// (the wave skips a body none of its lanes needs; as wave-uniform ballot
// tests they cost C4 2 % more).  `act`: the lane runs a layer in this call.  Per
// layer: record the ops (chain word / offsets, or the ext pool entry once
// the chain needs the ext form), count it, advance the pkt_buff cursor
// exactly as the reference parser does, look up the next ops.
// `info0`: the ops' rule word s.step(w.id), when the caller has read it.
// Record the layer the lane runs (`act`: ops w.id at w.data): the first 6 in
// the record; more than 6, or a layer past byte 510, forces the ext form
template <class Sink>
NSD_HD void record_layer(bool act, WalkOut &w, const Sink &g)
{
	const int id = act ? w.id : 0;
	const uint32_t start = w.data;
	const uint32_t k = w.n;
	constexpr uint32_t DEEP = NSD_REC_MAX_LAYERS + NSD_LDS_LAYERS;
	const bool need_now = act && (k >= NSD_REC_MAX_LAYERS || (k >= 1 && start > 510));
	g.take_deep(act && k == DEEP, w);   // (entry taken unless ext_on)
	const uint32_t kk = k < 8 ? k : 7;   // keeps the shifts below defined
	w.need_ext = w.need_ext || need_now;
	w.chain |= act && k < NSD_REC_MAX_LAYERS ? (uint32_t)id << (5 * kk) : 0u;
	if constexpr (Sink::OFFS) {
		w.offA |= act && k < 4 ? (uint64_t)(start & 0xFFFF) << (16 * (kk & 3)) : 0ull;
		w.offB |= act && k >= 4 && k < NSD_REC_MAX_LAYERS ? (start & 0xFFFF) << (16 * (kk & 1)) : 0u;
	} else {
		w.offB |= act && k >= NSD_REC_MAX_LAYERS && k < DEEP
				    ? (uint32_t)id << (5 * ((k - NSD_REC_MAX_LAYERS) & 7)) : 0u;
	}
	w.flags |= act && k >= NSD_EXT_MAX_LAYERS ? NSD_F_OVERFLOW : 0;
	if (act && k < NSD_EXT_MAX_LAYERS)
		g.layer(w, k, id, start);
	w.n = act ? k + 1 : k;
}

template <int MODE, class Src, class Sink>
NSD_HD void gen_step(const Src &s, bool act, WalkOut &w, const Sink &g, uint32_t info0)
{
	const int id = act ? w.id : 0;
	const uint32_t start = w.data;
	const uint32_t info = act ? info0 : 0u;
	record_layer(act, w, g);

	// ---- parse.  Every use of the layer's bytes (B0, KD) is gated by the
	// first pull (pulled), so bytes past the frame, which the device's
	// continuation rows do not mask, never reach a result.  The common rules are
	// computed for every lane and selected by the rule kind (boolean terms
	// combined with & and | so the compiler keeps them as selects).
	const uint32_t len = w.tail - start;   // pkt_len (pkt_buff.h:36-41)
	const uint32_t minl = info & 0xFF, fadv = (info >> 8) & 0xFF, kind = (info >> 16) & 0xF,
		       kpos = (info >> 20) & 0xF;
	const bool kw16 = (info >> 24) & 1;
	const uint32_t B0 = s.dword_at(start);          // layer bytes 0..3
	// the next-ops key's bytes: the layer's first byte for the extension
	// headers (kpos 0), a second read only when a lane's key sits further on
	uint32_t KD = B0;
	if (act & (kpos != 0))
		KD = s.dword_at(start + kpos);
	const uint32_t b0 = B0 & 0xFF, b1 = (B0 >> 8) & 0xFF, b2 = (B0 >> 16) & 0xFF;
	// eth_lay2 (a 16-bit ethertype; the perfect hash) / eth_lay3 (dissector_eth.c:30-62)
	int nx = s.lay3(KD & 0xFF);
	if (act & kw16) {
		const uint32_t key16 = __builtin_bswap16((uint16_t)KD);
		const uint32_t e2 = s.l2h(NSD_L2H(key16));
		nx = (e2 & 0xFFFF) == key16 ? (int)(e2 >> 16) : 0;
	}
	const uint32_t T8 = (b1 + 1u) * 8u;             // (hdr_ext_len + 1) * 8
	const bool pulled = len >= minl;

	// HBH / DestOpts: opt_len = T8 - 2 <= pkt_len after the 2-byte pull;
	// Routing: data_len = T8 - 4 <= pkt_len after the 4-byte pull.  These,
	// AH, the fixed pulls and the leaves are the common case; the other
	// kinds' rules run only when a lane of the wave is on such a layer
	// (instruction issue bounds the general walk)
	// AH (proto_ip_authentication_hdr.c:26-69): hdr_len = plen*4 + 8,
	// checked against pkt_len after the 12-byte pull (hdr_len + 12 <= len),
	// the ICV pulled when hdr_len > 12: the same rule with b1*4 + 8 and the
	// check offset by 12
	const bool isah = kind == K_AH;
	const bool var = (kind == K_T8) | isah;
	const uint32_t VL = (b1 << (isah ? 2u : 3u)) + 8u;
	const bool vok = VL + (isah ? 12u : 0u) <= len;
	uint32_t adv = var ? (vok ? (VL > minl ? VL : minl) : minl) : fadv;
	bool cont = (kind == K_CONT) | (var & vok);
	bool host = kind == K_HOST;
	const bool isv4 = act & (kind == K_IPV4);
	uint32_t ihl = 0;
	if (isv4) {
		// IPv4: options pulled if present, else data stays (proto_ipv4.c:136)
		ihl = b0 & 0xF;
		const uint32_t opts = (ihl > 5 ? ihl : 5) * 4u - 20u;
		const uint32_t v4adv = 20 + (opts <= len - 20 ? opts : 0);
		adv = v4adv;
		cont = true;
		if (MODE == PRINT_NORM) {
			// tail trim to tot_len - ihl*4, evaluated in size_t (:174-175)
			const uint32_t k2 = __builtin_bswap16((uint16_t)(B0 >> 16));   // tot_len
			const int64_t x = (int64_t)k2 - (int64_t)ihl * 4;
			const bool trim = pulled & (x >= 0) & ((uint64_t)x < len - v4adv);
			w.tail = trim ? start + v4adv + (uint32_t)x : w.tail;
		}
	}
	const bool ismob = act & (kind == K_MOB);
	if (ismob) {
		// Mobility: msg_len check, then (PRINT_NORM) get_mh_type's subtype
		// pull and the second check
		const int32_t mdl0 = (int32_t)T8 - 6;
		const uint32_t l0 = len - 6;
		const bool mok1 = mdl0 <= (int32_t)l0;
		const uint32_t sub = b2 < 8 ? (uint32_t)(NSD_MH_SUB >> (8 * b2)) & 0xFF : 0u;
		const bool sok = sub <= l0;
		const uint32_t sp = sok ? sub : 0u;
		const int32_t mdl = mdl0 - ((sok | (b2 <= 5)) ? (int32_t)sub : 0);
		const bool mok2 = (mdl <= (int32_t)(l0 - sp)) & (mdl >= 0);
		const bool mobok = MODE == PRINT_NORM ? mok1 & mok2 : mok1;
		const uint32_t mobadv =
			!mok1 ? 6u : MODE != PRINT_NORM ? T8 : mok2 ? 6 + sp + (uint32_t)mdl : 6 + sp;
		adv = mobadv;
		cont = mobok;
	}
	const bool isi6 = act & (kind == K_ICMP6);
	if (isi6) {
		// ICMPv6 (PRINT_NORM): types 130-154 have variable-length bodies
		// (leaf walk); types 1-4 / 128 / 129 pull a 4-byte body
		const bool i6host = MODE == PRINT_NORM && b0 - 130u <= 24u;
		const bool i6body = MODE == PRINT_NORM && ((b0 - 1u <= 3u) | ((b0 & 0xFE) == 128)) & (len >= 8);
		adv = i6host ? 0u : i6body ? 8u : 4u;
		host = i6host;
	}
	host = host & pulled;
	const bool upd = act & (kind != K_MPLS);
	// the new cursor and ops are stored last, after every use of the old
	// ones (start, id): the walkers' loop then carries them in place
	uint32_t nd = start + ((upd & pulled) ? adv : 0u);
	int nid = upd ? ((pulled & cont) ? nx : 0) : w.id;
	w.flags |= (upd & host) ? NSD_F_HOST : 0;
	// a host-rendered leaf: where its parser's pulls leave the cursor
	// (nsd_leaf.h), so the exit op's dump starts from the record; the
	// sink decides when (the device walks it after the chain, emit_general)
	nd = g.template leaf<MODE>(s, upd & host, w, id, start, nd);
	// ---- the rare heavy bodies
	const bool v4 = upd && kind == K_IPV4 && pulled;
	if (MODE == PRINT_NORM && v4) {
		// checksum over ihl*4 bytes, past the frame too (bytes >= caplen are 0)
		w.ip_csum = calc_csum(s, start, ihl * 2u);
	}
	const bool i4 = upd && id == NSD_OPS_ICMPV4 && pulled;
	if (MODE == PRINT_NORM && i4) {
		// calc_csum(icmp, pkt_len + 8): the whole (post-trim) message, odd
		// trailing byte dropped (csum.h:24-27); past the window: pending
		if (s.in_window(start, len & ~1u)) {
			if (calc_csum(s, start, len >> 1))
				w.flags |= NSD_F_ICMP_BAD;
		} else {
			w.icmp_pend = true;
			w.icmp_off = start;
			w.icmp_len = len;
		}
	}
	const bool mp = act && kind == K_MPLS;
	if (mp) {                                     // proto_mpls_unicast.c:49-77
		{
			uint32_t d = start, l = len;
			bool ok = true;
			for (;;) {
				if (l < 4) { ok = false; break; }
				const uint8_t sbit = s.b(d + 2) & 1;
				d += 4; l -= 4;
				if (sbit) break;
			}
			nd = d;
			int nxt = 0;
			if (ok && l) {
				const uint8_t nib = s.b(d) >> 4;   // mpls_uc_next_proto :23-47
				nxt = nib == 4 ? NSD_OPS_IPV4 : nib == 6 ? NSD_OPS_IPV6 : 0;
			}
			nid = nxt;
		}
	}
	w.data = nd;
	w.id = nid;
}
template <int MODE, class Src, class Sink>
NSD_HD void gen_step(const Src &s, bool act, WalkOut &w, const Sink &g)
{
	gen_step<MODE>(s, act, w, g, s.step(w.id));
}

// Straight-line walk for the common chains (pass 1): Ethernet, up to two
// 802.1Q / 802.1ad tags, IPv4 or IPv6, then TCP / UDP / ICMPv4 / ICMPv6 /
// ESP / NoNext (or the host-rendered leaves ARP and DCCP).  Same semantics
// as gen_step() for every packet it finishes (the c_step table cites the
// reference per ops); anything else (MPLS, deeper tag stacks, extension
// headers, IPv6-in-IPv4, the looping leaves LLDP / IGMP / ICMPv6 130-154,
// bytes past the staged window) goes to the general walk.  No loop, no per-layer
// dispatch switch.
// Returns FW_DONE, FW_RESTART (the general walk takes the packet from its start) or
// FW_RESUME (the chain reached an extension header / AH / IPv6-in-IPv4 ops
// at w.data with layers 0..w.n-1 recorded: the general walk resumes there with w.id).
// FOLD (the split schedule's fast kernel): an ICMPv4 message that runs past
// the window has its words inside the window summed here, from LDS (w.icmp_sum),
// and only the rest [icmp_off, icmp_off + icmp_len) left to the checksum pass.
// EXT (the fused kernel): Hop-by-Hop / DestOpts / Routing / Fragment / AH /
// Mobility headers whose needed bytes (c_step's `need`: next header, length,
// MH type) lie in the window are stepped here too, by gen_step's rules for
// their kinds,
// so a chain of a few short extension headers finishes in the fast walk and
// a longer one reaches the general walk further on (C4, line model: 0.74
// deferred packets instead of 0.86, 0.86 staged windows instead of 1.09).
enum : uint32_t { FW_DONE = 0, FW_RESTART = 1, FW_RESUME = 2 };
// the most layers a deferred packet carries into the general walk: the SLL
// head, Ethernet, two tags (the loop below) and IP.  The hand-over packs the
// layer count into 3 bits and the next ops id into 5 (take(), fast_tiles).
constexpr uint32_t FW_MAX_LAYERS = 5;
static_assert(FW_MAX_LAYERS < 8 && NSD_OPS_COUNT <= 32, "a deferred walk state packs n in 3 bits and id in 5");
template <int MODE, bool FOLD = false, bool EXT = false, class Src>
__device__ __forceinline__ uint32_t fast_walk(const Src &s, uint32_t caplen, WalkOut &w)
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
		return FW_RESTART;   // other link types: the general walk
	rec(NSD_OPS_ETHERNET, 0);
	if (caplen < 14) {
		w.n = n;
		return FW_DONE;
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
			return s.missed() ? FW_RESTART : FW_DONE;
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
			return s.missed() ? FW_RESTART : FW_DONE;
		}
		const uint32_t ihl = s.b(d) & 0xF;
		const uint32_t proto = s.b(d + 9);
		if (MODE == PRINT_NORM) {
			if (!s.in_window(d, ihl * 4u))
				return FW_RESTART;
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
			return s.missed() ? FW_RESTART : FW_DONE;
		}
		d2 = d + 40;
		l4 = s.lay3(s.b(d + 6));
	} else if (next == NSD_OPS_ARP) {
		rec(next, d);
		w.flags |= NSD_F_HOST;
		w.data = leaf_arp(s, d, caplen);
		w.n = n;
		return s.missed() ? FW_RESTART : FW_DONE;
	} else if (next == NSD_OPS_LLDP) {
		// the TLV walk reads past the window: the general walk runs it
		if (s.missed())
			return FW_RESTART;
		w.n = n;
		w.id = next;
		return FW_RESUME;
	} else if (next == 0) {
		w.n = n;
		return s.missed() ? FW_RESTART : FW_DONE;
	} else {
		return FW_RESTART;   // MPLS, a third tag
	}
	if constexpr (EXT) {
		for (;;) {
			const bool t8 = l4 == NSD_OPS_IPV6_HOP_BY_HOP || l4 == NSD_OPS_IPV6_DEST_OPTS ||
					l4 == NSD_OPS_IPV6_ROUTING;
			const bool fr = l4 == NSD_OPS_IPV6_FRAGM, ah = l4 == NSD_OPS_IP_AUTH;
			const bool mob = l4 == NSD_OPS_IPV6_MOBILITY;
			if (!(t8 || fr || ah || mob) || n >= FW_MAX_LAYERS || !s.in_window(d2, 4))
				break;
			rec(l4, d2);
			const uint32_t l = w.tail - d2;   // pkt_len
			const uint32_t minl = t8 ? (l4 == NSD_OPS_IPV6_ROUTING ? 4u : 2u) : fr ? 8u : mob ? 6u : 12u;
			if (l < minl) {
				// the pull fails: the chain ends, data stays (pkt_buff.h:50-64)
				w.data = d2;
				w.n = n;
				return s.missed() ? FW_RESTART : FW_DONE;
			}
			const uint32_t b0 = s.b(d2), b1 = s.b(d2 + 1);
			uint32_t adv;
			bool cont;
			if (t8) {
				// (hdr_ext_len + 1) * 8 bytes, or the chain ends after the
				// fixed pull (proto_ipv6_hop_by_hop.c:56-60, _dest_opts.c,
				// _routing.c:89-92)
				const uint32_t T8 = (b1 + 1u) * 8u;
				cont = T8 <= l;
				adv = cont ? T8 : minl;
			} else if (fr) {
				adv = 8;   // proto_ipv6_fragm.c:25-47: always continues
				cont = true;
			} else if (mob) {
				// Mobility: the message length check, then (PRINT_NORM)
				// get_mh_type's subtype pull and the second check
				// (proto_ipv6_mobility_hdr.c:247-286, gen_step's K_MOB)
				const uint32_t b2 = s.b(d2 + 2);
				const int32_t mdl0 = (int32_t)((b1 + 1u) * 8u) - 6;
				const uint32_t l0 = l - 6;
				const bool mok1 = mdl0 <= (int32_t)l0;
				const uint32_t sub = b2 < 8 ? (uint32_t)(NSD_MH_SUB >> (8 * b2)) & 0xFF : 0u;
				const bool sok = sub <= l0;
				const uint32_t sp = sok ? sub : 0u;
				const int32_t mdl = mdl0 - ((sok | (b2 <= 5)) ? (int32_t)sub : 0);
				const bool mok2 = (mdl <= (int32_t)(l0 - sp)) & (mdl >= 0);
				cont = MODE == PRINT_NORM ? mok1 & mok2 : mok1;
				adv = !mok1 ? 6u : MODE != PRINT_NORM ? (b1 + 1u) * 8u : mok2 ? 6 + sp + (uint32_t)mdl : 6 + sp;
			} else {
				// AH: plen * 4 + 8, checked after the 12-byte pull
				// (proto_ip_authentication_hdr.c:40-52)
				const uint32_t hl = b1 * 4u + 8u;
				cont = hl <= l - 12;
				adv = 12 + ((cont && hl > 12) ? hl - 12 : 0u);
			}
			d2 += adv;
			if (!cont) {
				w.data = d2;
				w.n = n;
				return s.missed() ? FW_RESTART : FW_DONE;
			}
			l4 = s.lay3(b0);
		}
		// an ICMPv6 type past the window, or a next layer past byte 510 (its
		// start needs the ext form, gen_step): the general walk resumes there
		if ((l4 == NSD_OPS_ICMPV6 && !s.in_window(d2, 1)) || (l4 != 0 && d2 > 510)) {
			if (s.missed())
				return FW_RESTART;
			w.data = d2;
			w.n = n;
			w.id = l4;
			return FW_RESUME;
		}
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
					if (FOLD) {
						// the words inside the window summed here (kw < len >> 1:
						// the message does not fit); the pass sums the rest
						const uint32_t kw = s.window_bytes(d2) >> 1;
						w.icmp_sum = s.sum16(d2, kw);
						w.icmp_off = d2 + 2 * kw;
						w.icmp_len = (len & ~1u) - 2 * kw;
					}
				} else if (calc_csum(s, d2, len >> 1)) {
					w.flags |= NSD_F_ICMP_BAD;
				}
			}
		}
		break;
	case NSD_OPS_ICMPV6: {
		const uint8_t type = s.b(d2);
		if (MODE == PRINT_NORM && len >= 4 && type >= 130 && type <= 154)
			goto resume;   // variable-length bodies (MLD, ND options, ...)
		rec(l4, d2);
		if (len >= 4) {
			w.data = d2 + 4;
			if (MODE == PRINT_NORM && ((type >= 1 && type <= 4) || type == 128 || type == 129) &&
			    len - 4 >= 4)
				w.data = d2 + 8;
		}
		break;
	}
	case NSD_OPS_DCCP:
		rec(l4, d2);
		w.flags |= NSD_F_HOST;
		w.data = leaf_dccp(s, d2, w.tail, MODE);
		break;
	default:
	resume:
		// IGMP (its v3 lists run past the window), the ICMPv6 bodies above,
		// extension headers, AH, IPv6-in-IPv4: the general walk resumes at d2
		if (s.missed())
			return FW_RESTART;
		w.n = n;
		w.id = l4;
		return FW_RESUME;
	}
	w.n = n;
	return s.missed() ? FW_RESTART : FW_DONE;
}

} // namespace nsd
