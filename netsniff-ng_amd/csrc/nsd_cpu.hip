// nsd_cpu.hip - the dissector chain walk on the host CPU, for the per-packet
// surface only ("the per-packet entry point stays a CPU
// implementation ... routing single packets to the GPU is a non-goal": one
// packet per launch would be all launch latency).  Batches always go to the
// device (nsd_kernels.hip); nothing here is a fallback for them.
//
// This is the product's own layer step, gen_step() of nsd_walk.h (the code
// general walk of the device kernel runs), instantiated with a host byte source
// over the whole frame and a sink that keeps the chain in arrays:
//   * nsd_walk_packet_cpu: one packet -> the record (+ ext entry) the device
//     writes for it;
//   * nsd::cpu_step: one layer at a pkt_buff cursor, for the exported
//     proto-ops objects (nsd_proto.cpp), whose process() functions run it
//     and then render the layer's text.
#include <string.h>

#include "nsd_walk.h"

namespace nsd {

// bytes of one frame, zero at offsets >= caplen (the parity domain); the
// whole frame is "in the window", so every layer runs in one gen_step
struct HSrc {
	const uint8_t *p;
	uint32_t caplen;

	__host__ uint8_t b(uint32_t o) const { return o < caplen ? p[o] : 0; }
	__host__ uint16_t le16(uint32_t o) const { return (uint16_t)(b(o) | b(o + 1) << 8); }
	__host__ uint16_t be16(uint32_t o) const { return (uint16_t)(b(o) << 8 | b(o + 1)); }
	__host__ uint32_t dword_at(uint32_t o) const
	{
		if (o + 4 <= caplen && o + 4 > o) {
			uint32_t v;
			memcpy(&v, p + o, 4);
			return v;
		}
		return (uint32_t)b(o) | (uint32_t)b(o + 1) << 8 | (uint32_t)b(o + 2) << 16 | (uint32_t)b(o + 3) << 24;
	}
	__host__ bool in_window(uint32_t, uint32_t) const { return true; }
	__host__ uint32_t sum16(uint32_t o, uint32_t nwords) const
	{
		uint32_t sum = 0;
		for (uint32_t i = 0; i < nwords; i++)
			sum += le16(o + 2 * i);
		return sum;
	}
	__host__ int lay3(uint32_t key) const { return h_lay3[key & 255]; }
	__host__ uint32_t step(int id) const { return h_step[id & 31]; }
	__host__ uint32_t l2h(uint32_t h) const { return h_lay2h.e[h & 31]; }
};

// per-packet flag counters, as the device's FlagCnt::add counts them
static void count_flags(uint64_t *c, const WalkOut &w, uint32_t caplen)
{
	c[NSD_CNT_PKTS]++;
	c[NSD_CNT_BYTES] += caplen;
	c[NSD_CNT_IP_BAD] += w.ip_csum != 0;
	c[NSD_CNT_ICMP_BAD] += (w.flags & NSD_F_ICMP_BAD) != 0;
	c[NSD_CNT_HOST] += (w.flags & NSD_F_HOST) != 0;
	c[NSD_CNT_EXT] += w.need_ext;
	c[NSD_CNT_OVERFLOW] += (w.flags & NSD_F_OVERFLOW) != 0;
	c[NSD_CNT_TRIM] += w.tail < caplen;
}

// the whole chain from the link type's start ops (dissector_main's loop,
// dissector.c:51-58); layers k < NSD_EXT_MAX_LAYERS land in ids / offs
template <int MODE>
static void walk_packet(const uint8_t *pkt, uint32_t caplen, int start_id, const nsd_sll_t *sll, WalkOut &w,
			uint8_t *ids, uint16_t *offs, uint64_t *counters)
{
	const HSrc s{ pkt, caplen };
	const HostSink g{ ids, offs, counters };
	walk_init(w, caplen, start_id);
	if (start_id == NSD_OPS_SLL) {
		// the SLL head pulls nothing and dispatches on pkt->sll (the device's
		// sll_head, nsd_kernels.hip)
		const uint32_t proto = sll ? __builtin_bswap16(sll->protocol) : 0u;
		g.layer(w, 0, NSD_OPS_SLL, 0);
		w.chain = NSD_OPS_SLL;
		w.n = 1;
		w.id = sll_next(sll ? sll->hatype : 0u, proto, MODE, h_lay2h.e[NSD_L2H(proto)]);
	}
	while (w.id != 0)
		gen_step<MODE>(s, true, w, g);
}

// One layer of the chain at the cursor [data, tail) of a frame of caplen
// bytes: ops `id` pulls and validates its header exactly as on the device;
// returns the next ops (0: the chain ends) and the new cursor, the IPv4
// header checksum and the NSD_F_* flags the layer raised.  The SLL head
// reads only sll (pkt->sll).
void cpu_count_packet(const uint8_t *pkt, uint32_t caplen, int linktype, int mode, const nsd_sll_t *sll,
		      uint64_t *counters);

int cpu_step(int mode, const uint8_t *pkt, uint32_t caplen, int id, uint32_t &data, uint32_t &tail,
	     uint16_t &ip_csum, uint8_t &flags, const nsd_sll_t *sll)
{
	ip_csum = 0;
	flags = 0;
	if (id == NSD_OPS_SLL) {
		// pulls nothing, dispatches on pkt->sll (dissector_sll.c:39-67)
		const uint32_t proto = sll ? __builtin_bswap16(sll->protocol) : 0u;
		return sll_next(sll ? sll->hatype : 0u, proto, mode, h_lay2h.e[NSD_L2H(proto)]);
	}
	const HSrc s{ pkt, caplen };
	uint8_t ids[NSD_EXT_MAX_LAYERS];
	uint16_t offs[NSD_EXT_MAX_LAYERS];
	const HostSink g{ ids, offs, nullptr };
	WalkOut w;
	walk_init(w, caplen, id);
	w.data = data;
	w.tail = tail;
	if (mode == PRINT_NORM)
		gen_step<PRINT_NORM>(s, true, w, g);
	else
		gen_step<PRINT_LESS>(s, true, w, g);
	data = w.data;
	tail = w.tail;
	ip_csum = w.ip_csum;
	flags = w.flags;
	return w.id;
}

} // namespace nsd

__attribute__((visibility("hidden"))) int nsd_start_for(int linktype);   // nsd_host.cpp

// The counters the device adds for one packet, from the host walk, for frames
// the batch path cannot carry (caplen above NSD_MAX_CAPLEN: the pcap replay
// renders those through the per-packet path)
void nsd::cpu_count_packet(const uint8_t *pkt, uint32_t caplen, int linktype, int mode, const nsd_sll_t *sll,
			   uint64_t *counters)
{
	WalkOut w;
	uint8_t ids[NSD_EXT_MAX_LAYERS];
	uint16_t offs[NSD_EXT_MAX_LAYERS];
	if (mode == PRINT_NORM || mode == PRINT_LESS) {
		const int start = nsd_start_for(linktype);
		if (mode == PRINT_NORM)
			walk_packet<PRINT_NORM>(pkt, caplen, start, sll, w, ids, offs, counters);
		else
			walk_packet<PRINT_LESS>(pkt, caplen, start, sll, w, ids, offs, counters);
		count_flags(counters, w, caplen);
	} else {
		counters[NSD_CNT_PKTS]++;
		counters[NSD_CNT_BYTES] += caplen;
	}
}

// One packet through the host walk: the record the device writes for it; a
// chain that needs the ext form gets its entry at word 0 of ext (its
// "packet index" is 0) when ext_words allows, else NSD_F_OVERFLOW.
extern "C" int nsd_walk_packet_cpu(const uint8_t *pkt, uint32_t caplen, int linktype, int mode,
				   const nsd_sll_t *sll, nsd_rec *rec, uint32_t *ext, uint32_t ext_words,
				   uint64_t *counters)
{
	using namespace nsd;
	if ((!pkt && caplen) || !rec || caplen > NSD_MAX_CAPLEN || mode < PRINT_NORM || mode > PRINT_NONE)
		return NSD_ERR_ARG;
	WalkOut w;
	if (mode != PRINT_NORM && mode != PRINT_LESS) {
		// every process() is NULL: no chain (dissector.c:51-53)
		walk_init(w, caplen, 0);
		const uint4 r = pack_record(w);
		memcpy(rec, &r, sizeof(*rec));
		if (counters) {
			counters[NSD_CNT_PKTS]++;
			counters[NSD_CNT_BYTES] += caplen;
		}
		return NSD_OK;
	}
	uint8_t ids[NSD_EXT_MAX_LAYERS];
	uint16_t offs[NSD_EXT_MAX_LAYERS];
	const int start = nsd_start_for(linktype);
	if (mode == PRINT_NORM)
		walk_packet<PRINT_NORM>(pkt, caplen, start, sll, w, ids, offs, counters);
	else
		walk_packet<PRINT_LESS>(pkt, caplen, start, sll, w, ids, offs, counters);
	if (w.need_ext) {
		const uint32_t nl = w.n < NSD_EXT_MAX_LAYERS ? w.n : NSD_EXT_MAX_LAYERS;
		const uint32_t words = NSD_EXT_WORDS(nl);
		if (ext && ext_words >= words) {
			memset(ext, 0, words * sizeof(uint32_t));
			ext[0] = 0;
			ext[1] = nl;
			for (uint32_t k = 0; k < nl; k++)
				ext[NSD_EXT_HDR_WORDS + k] = ids[k] | (uint32_t)offs[k] << 16;
			w.ext_on = true;
			w.slot = 0;
		} else {
			w.flags |= NSD_F_OVERFLOW;
		}
	}
	if (counters)
		count_flags(counters, w, caplen);
	const uint4 r = pack_record(w);
	memcpy(rec, &r, sizeof(*rec));
	return NSD_OK;
}
