// nsd_kernels.hip - CDNA4 (gfx950) kernels for the netsniff-ng dissector chain.
//
// One lane walks one packet (nsd_walk.h).  Layout in HBM:
//   frames  : one byte buffer, frames at arbitrary offsets (16-byte aligned
//             frames take the dwordx4 fast path)
//   desc    : u64 per packet (bits 0..39 offset, 40..63 caplen)
//   rec     : 16-byte chain record per packet (nsd_rec), one dwordx4 store per
//             lane -> 1 KiB contiguous per wave
//   ext     : overflow records for deep chains, slots by atomic counter
//   counters: u64[64] per-ops / flag counts
//
// Header bytes are staged through LDS: each wave copies the first WIN bytes of
// its 64 packets into an LDS window (16-byte chunks, WIN/16 consecutive lanes
// per packet so each packet's header is read as one contiguous segment), and
// the walk reads the window; bytes beyond WIN (deep IPv6 chains, long ICMP
// payloads) come from global memory.  Bytes >= caplen read as zero.
//
// Counting is wave-aggregated: per layer step the active lanes are grouped by
// ops id with ballot / readfirstlane, one lane adds the popcount into the
// block's LDS counters, and each block adds its counters to HBM once.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nsd_walk.h"

namespace nsd {

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;

// LDS window + global fallback.  The window holds bytes [0, WIN) of the
// frame with bytes >= caplen already zeroed.  Stored transposed by dword:
// dword j of lane l's packet lives at win[j * 64 + l], so the 64 lanes of a
// wave reading the same header offset hit 64 consecutive dwords (no bank
// conflicts).
template <int WIN>
struct LSrc {
	const uint32_t *win;   // this wave's window base + lane
	const uint8_t *p;      // frame in HBM (fallback outside the window)
	uint32_t caplen;
	uint32_t base;         // frame offset of window byte 0 (multiple of 16)
	__device__ __forceinline__ uint32_t dw(uint32_t j) const { return win[j * 64]; }
	__device__ __forceinline__ uint8_t b(uint32_t o) const
	{
		const uint32_t r = o - base;
		if (r < WIN)
			return (uint8_t)(dw(r >> 2) >> ((r & 3) * 8));
		return o < caplen ? p[o] : 0;
	}
	__device__ __forceinline__ uint16_t le16(uint32_t o) const
	{
		const uint32_t r = o - base;
		if (r + 1 < WIN && (r & 3) != 3)
			return (uint16_t)(dw(r >> 2) >> ((r & 3) * 8));
		return (uint16_t)(b(o) | b(o + 1) << 8);
	}
	__device__ __forceinline__ uint16_t be16(uint32_t o) const
	{
		return (uint16_t)__builtin_bswap16(le16(o));
	}
	__device__ __forceinline__ bool in_window(uint32_t o, uint32_t nbytes) const
	{
		return o >= base && o + nbytes <= base + WIN;
	}
	// the next layer would read past the staged window (bytes a layer's
	// process() inspects, counted from its start; longer reads such as
	// IPv4 options or routing addresses use the global fallback)
	__device__ __forceinline__ bool near_end(uint32_t o, int id) const
	{
		uint32_t need;
		switch (id) {
		case NSD_OPS_ETHERNET: need = 14; break;
		case NSD_OPS_IPV4: need = 20; break;
		case NSD_OPS_MPLS_UC: need = 16; break;
		case NSD_OPS_IPV6: case NSD_OPS_IPV6_IN_IPV4: need = 8; break;
		case NSD_OPS_VLAN: case NSD_OPS_QINQ: case NSD_OPS_IPV6_HOP_BY_HOP:
		case NSD_OPS_IPV6_DEST_OPTS: case NSD_OPS_IPV6_ROUTING: case NSD_OPS_IPV6_FRAGM:
		case NSD_OPS_IP_AUTH: case NSD_OPS_IPV6_MOBILITY: case NSD_OPS_ICMPV6: need = 4; break;
		default: need = 0;
		}
		return need && o < caplen && o + need > base + WIN;
	}
	// sum of `nwords` little-endian u16 words from `o` (csum.h:16-17)
	__device__ __forceinline__ uint32_t sum16(uint32_t o, uint32_t nwords) const
	{
		uint32_t sum = 0;
		if (!(o & 1) && in_window(o, 2 * nwords)) {
			uint32_t j = (o - base) >> 2, k = nwords;
			if ((o & 2) && k) { sum += dw(j) >> 16; j++; k--; }
			for (; k >= 2; k -= 2, j++) { const uint32_t v = dw(j); sum += (v & 0xFFFF) + (v >> 16); }
			if (k) sum += dw(j) & 0xFFFF;
			return sum;
		}
		for (uint32_t i = 0; i < nwords; i++)
			sum += le16(o + 2 * i);
		return sum;
	}
};

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Wave-aggregated counting into the block's LDS counters: the active lanes
// are grouped by value; the group leader adds the group's size.
struct WaveCnt {
	unsigned long long *s_cnt;
	__device__ __forceinline__ void operator()(int id) const
	{
		int my = id;
		for (;;) {
			const uint64_t pend = __ballot(my >= 0);
			if (!pend)
				break;
			const int leader = __ffsll((unsigned long long)pend) - 1;
			const int lid = __shfl(my, leader, 64);
			const uint64_t m = __ballot(my == lid);
			if (lane_id() == leader)
				atomicAdd(&s_cnt[NSD_CNT_OPS + lid], (unsigned long long)__popcll(m));
			if (my == lid)
				my = -1;
		}
	}
};

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v)
{
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		v += __shfl_xor(v, o, 64);
	return v;
}

// Stage WIN bytes of each participating packet of the wave into LDS, from
// frame offset my_base (a multiple of 16).  Chunk c (16 bytes at window
// offset 16c) of packet q is loaded by lane (q * CPP + c) % 64 in round
// (q * CPP + c) / 64, CPP = WIN / 16: the CPP chunks of one packet are read
// by consecutive lanes as one contiguous segment.  Bytes at frame offsets
// >= caplen are written as zero.
template <int WIN>
__device__ __forceinline__ void stage(uint32_t *wwin, const uint8_t *frames, uint64_t my_off,
				      uint32_t my_cap, uint32_t my_base, bool my_part, int lane)
{
	constexpr int CPP = WIN / 16;
#pragma unroll
	for (int r = 0; r < CPP; r++) {
		const int t = r * 64 + lane;
		const int q = t / CPP;
		const int c = t % CPP;
		const uint64_t off = __shfl(my_off, q, 64);
		const uint32_t cap = __shfl(my_cap, q, 64);
		const uint32_t wb = __shfl(my_base, q, 64);
		const bool part = __shfl((int)my_part, q, 64);
		if (!part)
			continue;
		const uint32_t fo = wb + (uint32_t)c * 16;   // frame offset of this chunk
		uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
		if (fo < cap) {
			const uint64_t a = off + fo;
			if ((a & 15) == 0) {
				const uint4 v = *(const uint4 *)(frames + a);
				w0 = v.x; w1 = v.y; w2 = v.z; w3 = v.w;
			} else {
				const uint32_t mis = (uint32_t)(a & 3);
				const uint32_t *src = (const uint32_t *)(frames + (a - mis));
				uint32_t d0 = src[0], d1 = src[1], d2 = src[2], d3 = src[3];
				if (mis) {
					const uint32_t d4 = src[4], sh = mis * 8;
					d0 = (d0 >> sh) | (d1 << (32 - sh));
					d1 = (d1 >> sh) | (d2 << (32 - sh));
					d2 = (d2 >> sh) | (d3 << (32 - sh));
					d3 = (d3 >> sh) | (d4 << (32 - sh));
				}
				w0 = d0; w1 = d1; w2 = d2; w3 = d3;
			}
			if (fo + 16 > cap) {   // zero bytes at frame offsets >= caplen
				const uint32_t keep = cap - fo;   // 1..15 bytes
				auto mask = [&](uint32_t &w, uint32_t bo) {
					if (bo >= keep) w = 0;
					else if (bo + 4 > keep) w &= (1u << ((keep - bo) * 8)) - 1u;
				};
				mask(w0, 0); mask(w1, 4); mask(w2, 8); mask(w3, 12);
			}
		}
		uint32_t *dst = wwin + (c * 4) * 64 + q;
		dst[0] = w0;
		dst[64] = w1;
		dst[128] = w2;
		dst[192] = w3;
	}
}

// Wave-cooperative ICMPv4 checksum (calc_csum over [a, a + nbytes), nbytes
// even, csum.h:24-27): the wave reads the message as consecutive dwords
// (lane l takes dwords l, l+64, ...: 256 contiguous bytes per load
// instruction).  Each byte is weighted by the parity of its distance from `a`
// (1 for the low byte of an LE word, 256 for the high byte), which makes the
// sum independent of the message's alignment.  `a` is wave-uniform.  Returns
// the folded one's-complement result in every lane.
__device__ __forceinline__ uint16_t wave_csum(const uint8_t *frames, uint64_t a, uint32_t nbytes, int lane)
{
	const uint32_t alo = __builtin_amdgcn_readfirstlane((uint32_t)a);
	const uint32_t ahi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
	const uint64_t au = ((uint64_t)ahi << 32) | alo;
	const uint32_t *p = (const uint32_t *)(frames + (au & ~3ull));
	const uint32_t s0 = alo & 3, endb = s0 + nbytes;   // byte range [s0, endb) of p
	const bool odd = alo & 1;
	uint32_t sum = 0;
	for (uint32_t j = lane; 4 * j < endb; j += 64) {
		uint32_t x = p[j];
		const uint32_t lo = 4 * j;
		if (lo < s0)
			x &= 0xFFFFFFFFu << (8 * s0);
		if (lo + 4 > endb)
			x &= 0xFFFFFFFFu >> (8 * (lo + 4 - endb));
		const uint32_t ev = (x & 0x00FF00FFu), od = (x >> 8) & 0x00FF00FFu;
		const uint32_t e2 = (ev & 0xFFFF) + (ev >> 16), o2 = (od & 0xFFFF) + (od >> 16);
		sum += odd ? (e2 << 8) + o2 : e2 + (o2 << 8);
	}
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		sum += __shfl_xor(sum, o, 64);
	sum = (sum >> 16) + (sum & 0xffff);
	sum += (sum >> 16);
	return (uint16_t)~sum;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m)
{
	return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// record words of a finished walk (layout of nsd_rec)
__device__ __forceinline__ uint4 pack_record(const WalkOut &w)
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

struct FlagCnt {
	uint32_t pkts = 0, ipbad = 0, icmpbad = 0, host = 0, ext = 0, ovf = 0, trim = 0;
	uint64_t bytes = 0;
	__device__ __forceinline__ void add(const WalkOut &w, uint32_t caplen)
	{
		pkts++;
		bytes += caplen;
		ipbad += w.ip_csum != 0;
		icmpbad += (w.flags & NSD_F_ICMP_BAD) != 0;
		host += (w.flags & NSD_F_HOST) != 0;
		ext += w.need_ext;
		ovf += (w.flags & NSD_F_OVERFLOW) != 0;
		trim += w.tail < caplen;
	}
	// wave reduce -> block LDS counters
	__device__ __forceinline__ void flush(unsigned long long *s_cnt, int lane) const
	{
		const uint32_t vals[7] = { pkts, ipbad, icmpbad, host, ext, ovf, trim };
		const int idx[7] = { NSD_CNT_PKTS, NSD_CNT_IP_BAD, NSD_CNT_ICMP_BAD, NSD_CNT_HOST,
				     NSD_CNT_EXT, NSD_CNT_OVERFLOW, NSD_CNT_TRIM };
#pragma unroll
		for (int k = 0; k < 7; k++) {
			const uint64_t v = wave_sum64(vals[k]);
			if (lane == 0 && v)
				atomicAdd(&s_cnt[idx[k]], (unsigned long long)v);
		}
		const uint64_t b = wave_sum64(bytes);
		if (lane == 0 && b)
			atomicAdd(&s_cnt[NSD_CNT_BYTES], (unsigned long long)b);
	}
};

__device__ __forceinline__ void block_flush(unsigned long long *s_cnt, unsigned long long *counters)
{
	__syncthreads();
	for (int k = threadIdx.x; k < NSD_NCOUNTERS; k += BLOCK)
		if (s_cnt[k])
			atomicAdd(&counters[k], s_cnt[k]);
}

// Pass 1: every packet whose chain resolves inside its first WIN bytes
// (<= 6 layers, checksummed bytes inside the window) is finished here; the
// others are appended to `queue` (wave-aggregated: one atomic per wave, slots
// by mbcnt prefix) for dissect_general.
template <int MODE, int WIN>
__global__ __launch_bounds__(BLOCK) void dissect_fast(
	const uint8_t *__restrict__ frames, const uint64_t *__restrict__ desc, uint32_t n,
	int start_id, uint4 *__restrict__ rec, unsigned long long *__restrict__ counters,
	uint32_t *__restrict__ queue, uint32_t *__restrict__ qcount)
{
	__shared__ uint32_t s_win[WAVES][(WIN / 4) * 64];
	__shared__ unsigned long long s_cnt[NSD_NCOUNTERS];

	const int lane = threadIdx.x & 63;
	const int wv = threadIdx.x >> 6;
	for (int k = threadIdx.x; k < NSD_NCOUNTERS; k += BLOCK)
		s_cnt[k] = 0;
	__syncthreads();

	const ExtSink es{ nullptr, 0, nullptr };
	const uint32_t stride = gridDim.x * BLOCK;
	FlagCnt fc;

	for (uint32_t base = blockIdx.x * BLOCK + wv * 64; base < n; base += stride) {
		const uint32_t i = base + lane;
		const bool valid = i < n;
		const uint64_t d = valid ? desc[i] : 0;
		const uint64_t off = NSD_DESC_OFF(d);
		const uint32_t caplen = NSD_DESC_CAPLEN(d);

		if (MODE != PRINT_NORM && MODE != PRINT_LESS) {
			// every process() is NULL: no chain (dissector.c:51-53)
			if (valid) {
				rec[i] = make_uint4(0, caplen << 16, 0, 0);
				fc.pkts++;
				fc.bytes += caplen;
			}
			continue;
		}

		stage<WIN>(&s_win[wv][0], frames, off, caplen, 0, valid, lane);
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
		WalkOut w;
		walk_init(w, caplen, valid ? start_id : 0);
		bool deferred = false;
		if (valid) {
			const LSrc<WIN> src{ &s_win[wv][lane], frames + off, caplen, 0 };
			deferred = walk<MODE, true>(src, caplen, es, w, 0);
		}
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();

		const uint64_t dm = __ballot(deferred);
		if (dm) {
			uint32_t qb = 0;
			if (lane == __ffsll((unsigned long long)dm) - 1)
				qb = atomicAdd(qcount, (uint32_t)__popcll(dm));
			qb = __shfl(qb, __ffsll((unsigned long long)dm) - 1, 64);
			if (deferred)
				queue[qb + lanes_below(dm)] = i;
		}
		const bool done = valid && !deferred;
		// per-ops counts from the finished chains, grouped by chain value
		{
			// ids are >= 1, so equal chain words imply equal layer counts
			uint32_t key = done ? w.chain : 0xFFFFFFFFu;
			for (;;) {
				const uint64_t pend = __ballot(key != 0xFFFFFFFFu);
				if (!pend)
					break;
				const int leader = __ffsll((unsigned long long)pend) - 1;
				const uint32_t lk = __shfl(key, leader, 64);
				const uint64_t m = __ballot(key == lk);
				if (lane == leader) {
					const uint32_t cnt = (uint32_t)__popcll(m);
					for (uint32_t k = 0, nl = w.n; k < nl; k++)
						atomicAdd(&s_cnt[NSD_CNT_OPS + ((lk >> (5 * k)) & 31)], (unsigned long long)cnt);
				}
				if (key == lk)
					key = 0xFFFFFFFFu;
			}
		}
		if (done) {
			rec[i] = pack_record(w);
			fc.add(w, caplen);
		}
	}
	fc.flush(s_cnt, lane);
	block_flush(s_cnt, counters);
}

// Pass 2: the queued packets, one lane each (compacted), walked from scratch
// with per-lane window restaging, ext spill and wave-cooperative ICMPv4
// checksums.
template <int MODE, int WIN>
__global__ __launch_bounds__(BLOCK) void dissect_general(
	const uint8_t *__restrict__ frames, const uint64_t *__restrict__ desc, int start_id,
	uint4 *__restrict__ rec, nsd_ext *__restrict__ ext, uint32_t ext_cap,
	uint32_t *__restrict__ ext_count, unsigned long long *__restrict__ counters,
	const uint32_t *__restrict__ queue, const uint32_t *__restrict__ qcount)
{
	__shared__ uint32_t s_win[WAVES][(WIN / 4) * 64];
	__shared__ unsigned long long s_cnt[NSD_NCOUNTERS];

	const int lane = threadIdx.x & 63;
	const int wv = threadIdx.x >> 6;
	for (int k = threadIdx.x; k < NSD_NCOUNTERS; k += BLOCK)
		s_cnt[k] = 0;
	__syncthreads();

	const uint32_t nq = *qcount;
	const WaveCnt wc{ s_cnt };
	const ExtSink es{ ext, ext_cap, ext_count };
	const uint32_t stride = gridDim.x * BLOCK;
	FlagCnt fc;

	for (uint32_t base = blockIdx.x * BLOCK + wv * 64; base < nq; base += stride) {
		const uint32_t k = base + lane;
		const bool valid = k < nq;
		const uint32_t i = valid ? queue[k] : 0;
		const uint64_t d = valid ? desc[i] : 0;
		const uint64_t off = NSD_DESC_OFF(d);
		const uint32_t caplen = NSD_DESC_CAPLEN(d);

		WalkOut w;
		walk_init(w, caplen, valid ? start_id : 0);
		uint32_t wbase = 0;
		bool part = valid;
		// lanes whose next header lies past their window suspend; the wave
		// restages those windows at the lanes' cursors and resumes them
		for (;;) {
			stage<WIN>(&s_win[wv][0], frames, off, caplen, wbase, part, lane);
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
			bool susp = false;
			if (part) {
				const LSrc<WIN> src{ &s_win[wv][lane], frames + off, caplen, wbase };
				susp = walk<MODE, false>(src, caplen, es, w, wc);
			}
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			if (!__ballot(susp))
				break;
			part = susp;
			if (susp)
				wbase = w.data & ~15u;
		}
		if (MODE == PRINT_NORM) {
			uint64_t pend = __ballot(w.icmp_pend);
			while (pend) {
				const int l = __ffsll((unsigned long long)pend) - 1;
				pend &= pend - 1;
				const uint64_t a = __shfl(off, l, 64) + __shfl(w.icmp_off, l, 64);
				const uint32_t nb = __shfl(w.icmp_len, l, 64) & ~1u;
				const uint16_t cs = wave_csum(frames, a, nb, lane);
				if (lane == l && cs)
					w.flags |= NSD_F_ICMP_BAD;
			}
		}
		if (!valid)
			continue;
		if (w.ext_on) {
			nsd_ext *e = ext + w.slot;
			e->pkt = i;
			e->nlayers = (uint16_t)(w.n < NSD_EXT_MAX_LAYERS ? w.n : NSD_EXT_MAX_LAYERS);
		}
		rec[i] = pack_record(w);
		fc.add(w, caplen);
	}
	fc.flush(s_cnt, lane);
	block_flush(s_cnt, counters);
}

} // namespace nsd

// ---- launchers (C ABI, called by nsd_host.cpp) ------------------------------
// workspace: [0, 64) queue counter (zeroed here), [64, 64 + 4n) queue
extern "C" size_t nsd_launch_workspace_bytes(uint32_t n) { return 64 + 4 * (size_t)n; }

extern "C" int nsd_launch_dissect(const uint8_t *d_frames, const uint64_t *d_desc, uint32_t n,
				  int start_id, int mode, nsd_rec *d_rec, nsd_ext *d_ext,
				  uint32_t ext_cap, uint32_t *d_ext_count, uint64_t *d_counters,
				  void *d_ws, int grid, hipStream_t stream)
{
	using namespace nsd;
	static int s_cus = 0;
	if (n == 0)
		return 0;
	if (!s_cus) {
		int dev = 0;
		if (hipGetDevice(&dev) != hipSuccess ||
		    hipDeviceGetAttribute(&s_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
			s_cus = 256;
	}
	const uint32_t waves = (n + 63) / 64;
	uint32_t blocks = (waves + WAVES - 1) / WAVES;
	// persistent grid: enough resident blocks to fill every CU, the rest
	// grid-strides (counters then cost one flush per block)
	const uint32_t cap_blocks = grid > 0 ? (uint32_t)grid : (uint32_t)s_cus * 8;
	if (blocks > cap_blocks)
		blocks = cap_blocks;
	const uint32_t gblocks = (uint32_t)s_cus * 4;
	unsigned long long *cnt = (unsigned long long *)d_counters;
	uint4 *rec = (uint4 *)d_rec;
	uint32_t *qcount = (uint32_t *)d_ws;
	uint32_t *queue = (uint32_t *)((uint8_t *)d_ws + 64);
	if (hipMemsetAsync(qcount, 0, 64, stream) != hipSuccess)
		return -2;
	switch (mode) {
	case PRINT_NORM:
		hipLaunchKernelGGL((dissect_fast<PRINT_NORM, 64>), dim3(blocks), dim3(BLOCK), 0, stream,
				   d_frames, d_desc, n, start_id, rec, cnt, queue, qcount);
		hipLaunchKernelGGL((dissect_general<PRINT_NORM, 64>), dim3(gblocks), dim3(BLOCK), 0, stream,
				   d_frames, d_desc, start_id, rec, d_ext, ext_cap, d_ext_count, cnt, queue, qcount);
		break;
	case PRINT_LESS:
		hipLaunchKernelGGL((dissect_fast<PRINT_LESS, 64>), dim3(blocks), dim3(BLOCK), 0, stream,
				   d_frames, d_desc, n, start_id, rec, cnt, queue, qcount);
		hipLaunchKernelGGL((dissect_general<PRINT_LESS, 64>), dim3(gblocks), dim3(BLOCK), 0, stream,
				   d_frames, d_desc, start_id, rec, d_ext, ext_cap, d_ext_count, cnt, queue, qcount);
		break;
	default:
		hipLaunchKernelGGL((dissect_fast<PRINT_HEX, 64>), dim3(blocks), dim3(BLOCK), 0, stream,
				   d_frames, d_desc, n, start_id, rec, cnt, queue, qcount);
		break;
	}
	return hipGetLastError() == hipSuccess ? 0 : -2;
}
