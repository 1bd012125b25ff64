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
	const uint8_t *p;      // frame in HBM (fallback past WIN)
	uint32_t caplen;
	__device__ __forceinline__ uint32_t dw(uint32_t j) const { return win[j * 64]; }
	__device__ __forceinline__ uint8_t b(uint32_t o) const
	{
		if (o < WIN)
			return (uint8_t)(dw(o >> 2) >> ((o & 3) * 8));
		return o < caplen ? p[o] : 0;
	}
	__device__ __forceinline__ uint16_t le16(uint32_t o) const
	{
		if (o + 1 < WIN && (o & 3) != 3)
			return (uint16_t)(dw(o >> 2) >> ((o & 3) * 8));
		return (uint16_t)(b(o) | b(o + 1) << 8);
	}
	__device__ __forceinline__ uint16_t be16(uint32_t o) const
	{
		return (uint16_t)__builtin_bswap16(le16(o));
	}
	// sum of `nwords` little-endian u16 words from `o` (csum.h:16-17)
	__device__ __forceinline__ uint32_t sum16(uint32_t o, uint32_t nwords) const
	{
		uint32_t sum = 0;
		if (!(o & 1) && o + 2 * nwords <= WIN) {
			uint32_t j = o >> 2, k = nwords;
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

// Stage the first WIN bytes of each of the wave's 64 packets into LDS.
// Chunk c (16 bytes at frame offset 16c) of packet q is loaded by lane
// (q * CPP + c) % 64 in round (q * CPP + c) / 64, CPP = WIN / 16.
template <int WIN>
__device__ __forceinline__ void stage(uint32_t *wwin, const uint8_t *frames, uint64_t my_off,
				      uint32_t my_cap, int lane)
{
	constexpr int CPP = WIN / 16;
#pragma unroll
	for (int r = 0; r < CPP; r++) {
		const int t = r * 64 + lane;
		const int q = t / CPP;
		const int c = t % CPP;
		const uint64_t off = __shfl(my_off, q, 64);
		const uint32_t cap = __shfl(my_cap, q, 64);   // 0 for lanes past n
		const uint32_t fo = (uint32_t)c * 16;
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
				auto mask = [&](uint32_t &w, uint32_t base) {
					if (base >= keep) w = 0;
					else if (base + 4 > keep) w &= (1u << ((keep - base) * 8)) - 1u;
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

template <int MODE, int WIN>
__global__ __launch_bounds__(BLOCK) void dissect_kernel(
	const uint8_t *__restrict__ frames, const uint64_t *__restrict__ desc, uint32_t n,
	int start_id, uint4 *__restrict__ rec, nsd_ext *__restrict__ ext, uint32_t ext_cap,
	uint32_t *__restrict__ ext_count, unsigned long long *__restrict__ counters)
{
	__shared__ uint32_t s_win[WAVES][(WIN / 4) * 64];
	__shared__ unsigned long long s_cnt[NSD_NCOUNTERS];

	const int lane = threadIdx.x & 63;
	const int wv = threadIdx.x >> 6;
	for (int i = threadIdx.x; i < NSD_NCOUNTERS; i += BLOCK)
		s_cnt[i] = 0;
	__syncthreads();

	const WaveCnt wc{ s_cnt };
	const ExtSink es{ ext, ext_cap, ext_count };
	const uint32_t stride = gridDim.x * BLOCK;
	uint32_t c_pkts = 0, c_ipbad = 0, c_icmpbad = 0, c_host = 0, c_ext = 0, c_ovf = 0, c_trim = 0;
	uint64_t c_bytes = 0;

	// whole waves iterate together (staging uses cross-lane shuffles)
	for (uint32_t base = blockIdx.x * BLOCK + wv * 64; base < n; base += stride) {
		const uint32_t i = base + lane;
		const bool valid = i < n;
		const uint64_t d = valid ? desc[i] : 0;
		const uint64_t off = NSD_DESC_OFF(d);
		const uint32_t caplen = NSD_DESC_CAPLEN(d);
		uint4 r;

		if (MODE == PRINT_NORM || MODE == PRINT_LESS) {
			stage<WIN>(&s_win[wv][0], frames, off, caplen, lane);
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
			WalkOut w;
			if (valid) {
				const LSrc<WIN> src{ &s_win[wv][lane], frames + off, caplen };
				walk<MODE>(src, caplen, start_id, es, w, wc);
			}
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			if (!valid)
				continue;
			const bool ext_form = w.need_ext;
			const uint32_t nf = (ext_form ? NSD_N_EXT : w.n) | w.flags;
			r.x = w.chain;
			r.y = (w.data & 0xFFFF) | (w.tail << 16);
			if (ext_form) {
				const uint32_t slot = w.ext_on ? w.slot : 0xFFFFFFFFu;
				r.z = w.ip_csum | (nf << 16) | ((slot & 0xFF) << 24);
				r.w = slot >> 8;
				if (w.ext_on) {
					nsd_ext *e = ext + w.slot;
					e->pkt = i;
					e->nlayers = (uint16_t)(w.n < NSD_EXT_MAX_LAYERS ? w.n : NSD_EXT_MAX_LAYERS);
				}
			} else {
				// layer k start / 2 for k = 1..5 (all even)
				const uint32_t o1 = (uint32_t)(w.offA >> 16) & 0xFFFF, o2 = (uint32_t)(w.offA >> 32) & 0xFFFF;
				const uint32_t o3 = (uint32_t)(w.offA >> 48), o4 = w.offB & 0xFFFF, o5 = w.offB >> 16;
				r.z = w.ip_csum | (nf << 16) | ((o1 >> 1) << 24);
				r.w = (o2 >> 1) | ((o3 >> 1) << 8) | ((o4 >> 1) << 16) | ((o5 >> 1) << 24);
			}
			c_ipbad += w.ip_csum != 0;
			c_icmpbad += (w.flags & NSD_F_ICMP_BAD) != 0;
			c_host += (w.flags & NSD_F_HOST) != 0;
			c_ext += ext_form;
			c_ovf += (w.flags & NSD_F_OVERFLOW) != 0;
			c_trim += w.tail < caplen;
		} else {
			if (!valid)
				continue;
			r.x = 0;
			r.y = caplen << 16;
			r.z = 0;
			r.w = 0;
		}
		c_pkts++;
		c_bytes += caplen;
		rec[i] = r;
	}

	// flags: wave reduce -> LDS -> one global atomic per counter per block
	{
		const uint32_t vals[7] = { c_pkts, c_ipbad, c_icmpbad, c_host, c_ext, c_ovf, c_trim };
		const int idx[7] = { NSD_CNT_PKTS, NSD_CNT_IP_BAD, NSD_CNT_ICMP_BAD, NSD_CNT_HOST,
				     NSD_CNT_EXT, NSD_CNT_OVERFLOW, NSD_CNT_TRIM };
#pragma unroll
		for (int k = 0; k < 7; k++) {
			const uint64_t v = wave_sum64(vals[k]);
			if (lane == 0 && v)
				atomicAdd(&s_cnt[idx[k]], (unsigned long long)v);
		}
		const uint64_t b = wave_sum64(c_bytes);
		if (lane == 0 && b)
			atomicAdd(&s_cnt[NSD_CNT_BYTES], (unsigned long long)b);
	}
	__syncthreads();
	for (int k = threadIdx.x; k < NSD_NCOUNTERS; k += BLOCK)
		if (s_cnt[k])
			atomicAdd(&counters[k], s_cnt[k]);
}

} // namespace nsd

// ---- launcher (C ABI, called by nsd_host.cpp) -------------------------------
extern "C" int nsd_launch_dissect(const uint8_t *d_frames, const uint64_t *d_desc, uint32_t n,
				  int start_id, int mode, nsd_rec *d_rec, nsd_ext *d_ext,
				  uint32_t ext_cap, uint32_t *d_ext_count, uint64_t *d_counters,
				  int grid, hipStream_t stream)
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
	// grid-strides (counters then cost one flush per block, not per 256 pkts)
	const uint32_t cap_blocks = grid > 0 ? (uint32_t)grid : (uint32_t)s_cus * 8;
	if (blocks > cap_blocks)
		blocks = cap_blocks;
	unsigned long long *cnt = (unsigned long long *)d_counters;
	uint4 *rec = (uint4 *)d_rec;
	switch (mode) {
	case PRINT_NORM:
		hipLaunchKernelGGL((dissect_kernel<PRINT_NORM, 64>), dim3(blocks), dim3(BLOCK), 0, stream,
				   d_frames, d_desc, n, start_id, rec, d_ext, ext_cap, d_ext_count, cnt);
		break;
	case PRINT_LESS:
		hipLaunchKernelGGL((dissect_kernel<PRINT_LESS, 64>), dim3(blocks), dim3(BLOCK), 0, stream,
				   d_frames, d_desc, n, start_id, rec, d_ext, ext_cap, d_ext_count, cnt);
		break;
	default:
		hipLaunchKernelGGL((dissect_kernel<PRINT_HEX, 64>), dim3(blocks), dim3(BLOCK), 0, stream,
				   d_frames, d_desc, n, start_id, rec, d_ext, ext_cap, d_ext_count, cnt);
		break;
	}
	return hipGetLastError() == hipSuccess ? 0 : -2;
}
