// nsd_kernels.hip - CDNA4 (gfx950) kernels for the netsniff-ng dissector chain.
//
// One lane walks one packet (nsd_walk.h).  Layout in HBM:
//   frames  : one byte buffer, frames at arbitrary offsets
//   desc    : u64 per packet (bits 0..39 offset, 40..63 caplen)
//   rec     : 16-byte chain record per packet (nsd_rec), written as one
//             dwordx4 store per lane -> fully coalesced 1 KiB per wave
//   ext     : overflow records for deep chains, slots by atomic counter
//   counters: u64[64] per-ops / flag counts
//
// Header bytes are staged through LDS: each wave copies the first WIN bytes
// of its 64 packets into an LDS window (16-byte chunk loads, several lanes per
// packet, so each packet's header is read as whole contiguous segments), and
// the walk reads the window; bytes beyond WIN (deep IPv6 chains, long ICMP
// payloads) come from global memory.  Bytes >= caplen read as zero.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nsd_walk.h"

namespace nsd {

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;

// Global-memory byte source (bounds-checked; zero past caplen).
struct GSrc {
	const uint8_t *p;
	uint32_t caplen;
	__device__ __forceinline__ uint8_t b(uint32_t o) const { return o < caplen ? p[o] : 0; }
	__device__ __forceinline__ uint16_t be16(uint32_t o) const { return (uint16_t)(b(o) << 8 | b(o + 1)); }
	__device__ __forceinline__ uint16_t le16(uint32_t o) const { return (uint16_t)(b(o) | b(o + 1) << 8); }
};

// LDS window + global fallback.  The window holds bytes [0, WIN) of the
// frame with bytes >= caplen already zeroed.  Stored transposed by dword:
// dword j of lane l's packet lives at win[j * 64 + l], so the 64 lanes of a
// wave reading the same header offset hit 64 consecutive dwords (no bank
// conflicts).
template <int WIN>
struct LSrc {
	const uint32_t *win;   // this wave's window base + lane
	const uint8_t *p;
	uint32_t caplen;
	__device__ __forceinline__ uint32_t dw(uint32_t j) const { return win[j * 64]; }
	__device__ __forceinline__ uint8_t b(uint32_t o) const
	{
		if (o < WIN)
			return (uint8_t)(dw(o >> 2) >> ((o & 3) * 8));
		return o < caplen ? p[o] : 0;
	}
	__device__ __forceinline__ uint16_t be16(uint32_t o) const
	{
		if (o + 1 < WIN && (o & 3) != 3) {
			uint32_t v = dw(o >> 2) >> ((o & 3) * 8);
			return (uint16_t)((v & 0xFF) << 8 | ((v >> 8) & 0xFF));
		}
		return (uint16_t)(b(o) << 8 | b(o + 1));
	}
	__device__ __forceinline__ uint16_t le16(uint32_t o) const
	{
		if (o + 1 < WIN && (o & 3) != 3)
			return (uint16_t)(dw(o >> 2) >> ((o & 3) * 8));
		return (uint16_t)(b(o) | b(o + 1) << 8);
	}
};

// Per-lane counters; indices are compile-time constants inside the walk's
// switch, so they stay in registers.
struct LaneCnt {
	uint32_t ops[NSD_OPS_COUNT];
	template <int ID> __device__ __forceinline__ void inc() { ops[ID]++; }
	__device__ __forceinline__ void any(int id)   // rare (host-rendered) ids
	{
#pragma unroll
		for (int i = 1; i < NSD_OPS_COUNT; i++)
			if (id == i)
				ops[i]++;
	}
};

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		v += __shfl_xor(v, o, 64);
	return v;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v)
{
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		v += __shfl_xor(v, o, 64);
	return v;
}

// Stage the first WIN bytes of each of the wave's 64 packets into LDS.
// Chunk c (16 bytes at frame offset 16c) of packet q is loaded by lane
// (q * CPP + c) % 64 in round (q * CPP + c) / 64, CPP = WIN / 16 chunks per
// packet: consecutive lanes read consecutive 16-byte pieces of one packet.
// Frames may start at any byte; chunks are fetched 16-byte aligned and the
// bytes are shifted into place.
template <int WIN>
__device__ __forceinline__ void stage(uint32_t *wwin, const uint8_t *frames, uint64_t my_off,
				      uint32_t my_cap, bool my_valid, int lane)
{
	constexpr int CPP = WIN / 16;            // chunks per packet
	constexpr int ROUNDS = CPP;              // 64 packets * CPP chunks / 64 lanes
#pragma unroll
	for (int r = 0; r < ROUNDS; r++) {
		const int t = r * 64 + lane;
		const int q = t / CPP;               // packet (lane) whose chunk this is
		const int c = t % CPP;
		const uint64_t off = __shfl(my_off, q, 64);
		const uint32_t cap = __shfl(my_cap, q, 64);
		const bool valid = __shfl((int)my_valid, q, 64);
		const uint32_t fo = (uint32_t)c * 16;   // frame offset of this chunk
		uint32_t w[4] = { 0, 0, 0, 0 };
		if (valid && fo < cap) {
			const uint64_t a = off + fo;
			const uint32_t mis = (uint32_t)(a & 3);
			const uint32_t *src = (const uint32_t *)(frames + (a - mis));
			// 5 dwords cover 16 bytes at any dword misalignment
			uint32_t d0 = src[0], d1 = src[1], d2 = src[2], d3 = src[3], d4 = mis ? src[4] : 0;
			if (mis) {
				const uint32_t sh = mis * 8;
				d0 = (d0 >> sh) | (d1 << (32 - sh));
				d1 = (d1 >> sh) | (d2 << (32 - sh));
				d2 = (d2 >> sh) | (d3 << (32 - sh));
				d3 = (d3 >> sh) | (d4 << (32 - sh));
			}
			w[0] = d0; w[1] = d1; w[2] = d2; w[3] = d3;
			// zero bytes at frame offsets >= caplen
			if (fo + 16 > cap) {
#pragma unroll
				for (int j = 0; j < 4; j++) {
					const uint32_t base = fo + 4 * j;
					if (base >= cap)
						w[j] = 0;
					else if (base + 4 > cap)
						w[j] &= (1u << ((cap - base) * 8)) - 1u;
				}
			}
		}
#pragma unroll
		for (int j = 0; j < 4; j++)
			wwin[(c * 4 + j) * 64 + q] = w[j];
	}
}

template <int MODE, int WIN>
__global__ __launch_bounds__(BLOCK) void dissect_kernel(
	const uint8_t *__restrict__ frames, const uint64_t *__restrict__ desc, uint32_t n,
	int start_id, nsd_rec *__restrict__ rec, nsd_ext *__restrict__ ext, uint32_t ext_cap,
	uint32_t *__restrict__ ext_count, unsigned long long *__restrict__ counters)
{
	__shared__ uint32_t s_win[WAVES][(WIN / 4) * 64];
	__shared__ unsigned long long s_cnt[NSD_NCOUNTERS];

	const int lane = threadIdx.x & 63;
	const int wv = threadIdx.x >> 6;
	for (int i = threadIdx.x; i < NSD_NCOUNTERS; i += BLOCK)
		s_cnt[i] = 0;

	LaneCnt lc;
#pragma unroll
	for (int i = 0; i < NSD_OPS_COUNT; i++)
		lc.ops[i] = 0;
	uint32_t c_ipbad = 0, c_icmpbad = 0, c_host = 0, c_ext = 0, c_ovf = 0, c_trim = 0, c_pkts = 0;
	uint64_t c_bytes = 0;

	const ExtSink es{ ext, ext_cap, ext_count };
	const uint32_t stride = gridDim.x * BLOCK;
	// whole waves iterate together (staging uses cross-lane shuffles)
	for (uint32_t base = blockIdx.x * BLOCK + wv * 64; base < n; base += stride) {
		const uint32_t i = base + lane;
		const bool valid = i < n;
		const uint64_t d = valid ? desc[i] : 0;
		const uint64_t off = NSD_DESC_OFF(d);
		const uint32_t caplen = NSD_DESC_CAPLEN(d);

		nsd_rec r;
		if (MODE == PRINT_NORM || MODE == PRINT_LESS) {
			stage<WIN>(&s_win[wv][0], frames, off, caplen, valid, lane);
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			WalkOut w;
			if (valid) {
				LSrc<WIN> src{ &s_win[wv][lane], frames + off, caplen };
				walk<MODE>(src, caplen, start_id, es, w, lc);
			}
			__builtin_amdgcn_wave_barrier();
			if (!valid)
				continue;
			const bool ext_form = w.need_ext;
			r.chain = w.chain;
			r.data_off = (uint16_t)w.data;
			r.tail_off = (uint16_t)w.tail;
			r.ip_csum = w.ip_csum;
			r.nflags = (uint8_t)((ext_form ? NSD_N_EXT : w.n) | w.flags);
			if (ext_form) {
				const uint32_t slot = w.ext_on ? w.slot : 0xFFFFFFFFu;
				r.off2[0] = (uint8_t)slot;
				r.off2[1] = (uint8_t)(slot >> 8);
				r.off2[2] = (uint8_t)(slot >> 16);
				r.off2[3] = (uint8_t)(slot >> 24);
				r.off2[4] = 0;
				if (w.ext_on) {
					nsd_ext *e = ext + w.slot;
					e->pkt = i;
					e->nlayers = (uint16_t)(w.n < NSD_EXT_MAX_LAYERS ? w.n : NSD_EXT_MAX_LAYERS);
					e->rsvd = 0;
				}
			} else {
#pragma unroll
				for (int k = 0; k < 5; k++)
					r.off2[k] = (uint8_t)(off_of(w, k + 1) >> 1);
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
			r.chain = 0;
			r.data_off = 0;
			r.tail_off = (uint16_t)caplen;
			r.ip_csum = 0;
			r.nflags = 0;
			r.off2[0] = r.off2[1] = r.off2[2] = r.off2[3] = r.off2[4] = 0;
		}
		c_pkts++;
		c_bytes += caplen;
		rec[i] = r;
	}

	// counters: wave reduce -> LDS -> one global atomic per counter per block
	__syncthreads();
#pragma unroll
	for (int k = 1; k < NSD_OPS_COUNT; k++) {
		uint32_t v = wave_sum(lc.ops[k]);
		if (lane == 0 && v)
			atomicAdd(&s_cnt[NSD_CNT_OPS + k], (unsigned long long)v);
	}
	{
		uint32_t v;
		v = wave_sum(c_pkts);    if (lane == 0 && v) atomicAdd(&s_cnt[NSD_CNT_PKTS], (unsigned long long)v);
		v = wave_sum(c_ipbad);   if (lane == 0 && v) atomicAdd(&s_cnt[NSD_CNT_IP_BAD], (unsigned long long)v);
		v = wave_sum(c_icmpbad); if (lane == 0 && v) atomicAdd(&s_cnt[NSD_CNT_ICMP_BAD], (unsigned long long)v);
		v = wave_sum(c_host);    if (lane == 0 && v) atomicAdd(&s_cnt[NSD_CNT_HOST], (unsigned long long)v);
		v = wave_sum(c_ext);     if (lane == 0 && v) atomicAdd(&s_cnt[NSD_CNT_EXT], (unsigned long long)v);
		v = wave_sum(c_ovf);     if (lane == 0 && v) atomicAdd(&s_cnt[NSD_CNT_OVERFLOW], (unsigned long long)v);
		v = wave_sum(c_trim);    if (lane == 0 && v) atomicAdd(&s_cnt[NSD_CNT_TRIM], (unsigned long long)v);
		uint64_t b = wave_sum64(c_bytes);
		if (lane == 0 && b) atomicAdd(&s_cnt[NSD_CNT_BYTES], (unsigned long long)b);
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
	if (n == 0)
		return 0;
	const uint32_t waves = (n + 63) / 64;
	uint32_t blocks = (waves + WAVES - 1) / WAVES;
	if (grid > 0 && blocks > (uint32_t)grid)
		blocks = (uint32_t)grid;
	unsigned long long *cnt = (unsigned long long *)d_counters;
	switch (mode) {
	case PRINT_NORM:
		hipLaunchKernelGGL((dissect_kernel<PRINT_NORM, 64>), dim3(blocks), dim3(BLOCK), 0, stream,
				   d_frames, d_desc, n, start_id, d_rec, d_ext, ext_cap, d_ext_count, cnt);
		break;
	case PRINT_LESS:
		hipLaunchKernelGGL((dissect_kernel<PRINT_LESS, 64>), dim3(blocks), dim3(BLOCK), 0, stream,
				   d_frames, d_desc, n, start_id, d_rec, d_ext, ext_cap, d_ext_count, cnt);
		break;
	default:
		hipLaunchKernelGGL((dissect_kernel<PRINT_HEX, 64>), dim3(blocks), dim3(BLOCK), 0, stream,
				   d_frames, d_desc, n, start_id, d_rec, d_ext, ext_cap, d_ext_count, cnt);
		break;
	}
	return hipGetLastError() == hipSuccess ? 0 : -2;
}
