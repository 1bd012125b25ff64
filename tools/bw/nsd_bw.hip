// nsd_bw.hip - the read ceiling bench.py measures beside the dissect kernels
// (not product code): a streaming read of a device buffer at the rate this
// device reaches (bw.hip found 6.32 TB/s read-only at 4
// blocks of 256 per CU).  Each lane keeps four 16-byte loads in flight per
// round; plain or nontemporal loads; the grid is blocks_per_cu per CU.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ v4u ld(const v4u *p)
{
	if (NT)
		return __builtin_nontemporal_load(p);
	return *p;
}

template <bool NT>
__global__ __launch_bounds__(256) void k_read(const v4u *__restrict__ a, size_t n, uint32_t *sink)
{
	const size_t step = (size_t)gridDim.x * blockDim.x;
	size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
	v4u acc = { 0, 0, 0, 0 };
	for (; i + 3 * step < n; i += 4 * step) {
		const v4u x0 = ld<NT>(a + i), x1 = ld<NT>(a + i + step);
		const v4u x2 = ld<NT>(a + i + 2 * step), x3 = ld<NT>(a + i + 3 * step);
		acc ^= x0 ^ x1 ^ x2 ^ x3;
	}
	for (; i < n; i += step)
		acc ^= ld<NT>(a + i);
	if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u)   // keeps the loads; never true in practice
		sink[0] = acc.x;
}

// reads `bytes` (a multiple of 16) of buf on `stream`; returns 0 or -1
extern "C" int nsd_bw_read(const void *buf, size_t bytes, int blocks_per_cu, int nontemporal, void *stream,
			   uint32_t *sink)
{
	int dev = 0, cus = 0;
	if (hipGetDevice(&dev) != hipSuccess ||
	    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
		return -1;
	const dim3 grid((unsigned)(cus * (blocks_per_cu > 0 ? blocks_per_cu : 4)));
	const size_t n = bytes / 16;
	if (nontemporal)
		hipLaunchKernelGGL(k_read<true>, grid, dim3(256), 0, (hipStream_t)stream, (const v4u *)buf, n, sink);
	else
		hipLaunchKernelGGL(k_read<false>, grid, dim3(256), 0, (hipStream_t)stream, (const v4u *)buf, n, sink);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The fast walk's access shape alone: every packet's first 64 bytes (from
// the 16-byte aligned address at or below its start) as four 16-byte loads
// by four consecutive lanes, a wave per tile of 64 packets, one tile of
// loads in flight per wave, plus the descriptor loads; nothing computed.
// What the tile phase of the dissect kernels could reach on a batch's
// layout (IMIX: one or two lines every 5 - 12 lines).
template <bool NT>
__global__ __launch_bounds__(256) void k_windows(const uint8_t *__restrict__ frames, const uint64_t *__restrict__ desc,
						 uint32_t n, uint32_t *sink)
{
	const uint32_t lane = threadIdx.x & 63;
	const uint32_t stride = gridDim.x * blockDim.x;
	v4u acc = { 0, 0, 0, 0 };
	for (uint32_t base = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < n; base += stride) {
		const uint64_t d = base + lane < n ? desc[base + lane] : 0;
		const uint64_t a = (uint64_t)(uintptr_t)frames + ((d & ((1ull << 40) - 1)) & ~15ull);
#pragma unroll
		for (int r = 0; r < 4; r++) {
			const int q = r * 16 + (int)(lane >> 2);
			const uint64_t aq = (uint64_t)__shfl((uint32_t)a, q, 64) | (uint64_t)__shfl((uint32_t)(a >> 32), q, 64) << 32;
			acc ^= ld<NT>((const v4u *)(uintptr_t)(aq + 16 * (lane & 3)));
		}
	}
	if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u)
		sink[0] = acc.x;
}

extern "C" int nsd_bw_windows(const void *frames, const void *desc, uint32_t n, int blocks_per_cu, int nontemporal,
			      void *stream, uint32_t *sink)
{
	int dev = 0, cus = 0;
	if (hipGetDevice(&dev) != hipSuccess ||
	    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
		return -1;
	const dim3 grid((unsigned)(cus * (blocks_per_cu > 0 ? blocks_per_cu : 4)));
	if (nontemporal)
		hipLaunchKernelGGL(k_windows<true>, grid, dim3(256), 0, (hipStream_t)stream, (const uint8_t *)frames,
				   (const uint64_t *)desc, n, sink);
	else
		hipLaunchKernelGGL(k_windows<false>, grid, dim3(256), 0, (hipStream_t)stream, (const uint8_t *)frames,
				   (const uint64_t *)desc, n, sink);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The ICMPv4 checksum pass's access shape alone: the
// pending messages of a batch as per-wave lists of {message's byte offset
// in the frame buffer (bits 0..39) | length << 48}; block b's four waves
// take its lists 4b .. 4b+3 in 64-entry pieces round-robin (as icmp_pass
// does), register-allocated for 4 waves per SIMD like the fused kernel.
// LANES lanes per message (64 / LANES messages per group), U 16-byte loads
// per lane per group.  Layout 0 (the pass): chunks counted from the
// message's 16-byte aligned start, sub-lanes 0 / 1 take the first / last
// chunk masked, the interior chunks 1 + sub + LANES t unmasked.  Layout 1
// (ALIGN): chunks counted from the 128-byte line holding the first byte,
// chunk j on sub-lane j % LANES (each 8-lane group instruction reads one
// whole line), the message's first and last chunk masked, chunks before
// it skipped.  PIPE: the next group's loads issued (unconditional, clamped
// indexes) before the current group is summed.  Long messages: the chunks
// past the first LANES * U per lane in a plain loop.
template <bool NT>
__device__ __forceinline__ uint4 ldc(const uint4 *p)
{
	const v4u x = ld<NT>((const v4u *)p);
	return make_uint4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ uint32_t mmask(uint32_t p, uint32_t s0, uint32_t endb)
{
	uint32_t m = 0xFFFFFFFFu;
	if (s0 > p)
		m = s0 >= p + 4 ? 0u : m << (8 * (s0 - p));
	if (endb < p + 4)
		m = endb <= p ? 0u : m & (0xFFFFFFFFu >> (8 * (p + 4 - endb)));
	return m;
}
__device__ __forceinline__ uint32_t sum4(const uint4 &v, uint32_t acc)
{
	acc = __builtin_amdgcn_sad_u16(v.x, 0u, acc);
	acc = __builtin_amdgcn_sad_u16(v.y, 0u, acc);
	acc = __builtin_amdgcn_sad_u16(v.z, 0u, acc);
	return __builtin_amdgcn_sad_u16(v.w, 0u, acc);
}
__device__ __forceinline__ uint4 masked(const uint4 &v, uint32_t lo, uint32_t s0, uint32_t endb)
{
	return make_uint4(v.x & mmask(lo, s0, endb), v.y & mmask(lo + 4, s0, endb), v.z & mmask(lo + 8, s0, endb),
			  v.w & mmask(lo + 12, s0, endb));
}

struct MsgG {
	const uint4 *base;
	uint32_t s0, endb, c0, nch;   // chunks [c0, nch) hold message bytes [s0, endb)
};

template <bool ALIGN>
__device__ __forceinline__ MsgG msg_group(const uint8_t *frames, uint64_t e, uint32_t q, uint32_t k0, uint32_t cnt,
					  uint32_t grp)
{
	const int src = (int)((q + grp) & 63);
	const uint32_t alo = __shfl((uint32_t)e, src, 64), ahi = __shfl((uint32_t)(e >> 32), src, 64);
	const bool mon = q < 64 && k0 + q + grp < cnt;
	const uint64_t a = (uint64_t)alo | (uint64_t)(ahi & 0xFF) << 32;
	const uint32_t len = (ahi >> 16) & ~1u;
	MsgG g;
	g.s0 = ALIGN ? (alo & 127) : (alo & 15);
	g.base = (const uint4 *)(frames + (a & (ALIGN ? ~127ull : ~15ull)));
	g.endb = g.s0 + len;
	g.c0 = g.s0 >> 4;
	g.nch = mon ? (g.endb + 15) >> 4 : 0u;
	return g;
}

// chunk of slot u on this sub-lane
template <int LANES, bool ALIGN>
__device__ __forceinline__ uint32_t msg_chunk(uint32_t sub, int u)
{
	return ALIGN ? sub + LANES * u : 1 + sub + LANES * u;
}

template <int LANES, int U, bool ALIGN, bool NT, bool CLAMP>
__device__ __forceinline__ void msg_issue(const MsgG &g, uint32_t sub, uint4 (&v)[U], uint4 &edge)
{
	if (!ALIGN) {
		// sub-lane 0: chunk 0, sub-lane 1: chunk nch - 1 (both masked later)
		const uint32_t je = sub == 0 || g.nch < 2 ? 0u : g.nch - 1;
		if (CLAMP || (sub == 0 && g.nch > 0) || (sub == 1 && g.nch > 1))
			edge = ldc<NT>(g.base + je);
	}
#pragma unroll
	for (int u = 0; u < U; u++) {
		const uint32_t j = msg_chunk<LANES, ALIGN>(sub, u);
		const bool in = ALIGN ? (j >= g.c0 && j < g.nch) : j + 1 < g.nch;
		if (CLAMP)
			v[u] = ldc<NT>(g.base + (in ? j : 0u));
		else
			v[u] = in ? ldc<NT>(g.base + j) : make_uint4(0, 0, 0, 0);
	}
}

template <int LANES, int U, bool ALIGN>
__device__ __forceinline__ uint32_t msg_sum(const MsgG &g, uint32_t sub, const uint4 (&v)[U], const uint4 &edge)
{
	uint32_t s = 0;
	if (!ALIGN && ((sub == 0 && g.nch > 0) || (sub == 1 && g.nch > 1))) {
		const uint32_t je = sub == 0 ? 0u : g.nch - 1;
		s = sum4(masked(edge, 16 * je, g.s0, g.endb), s);
	}
#pragma unroll
	for (int u = 0; u < U; u++) {
		const uint32_t j = msg_chunk<LANES, ALIGN>(sub, u);
		const bool in = ALIGN ? (j >= g.c0 && j < g.nch) : j + 1 < g.nch;
		uint4 x = in ? v[u] : make_uint4(0, 0, 0, 0);
		if (ALIGN && (j == g.c0 || j + 1 == g.nch))
			x = masked(x, 16 * j, g.s0, g.endb);
		s = sum4(x, s);
	}
	return s;
}

template <int LANES, int U, bool ALIGN, bool NT>
__device__ __forceinline__ uint32_t msg_rest(const MsgG &g, uint32_t sub)
{
	uint32_t s = 0;
	for (uint32_t j0 = msg_chunk<LANES, ALIGN>(sub, U); __ballot(j0 + (ALIGN ? 0 : 1) < g.nch); j0 += LANES * U) {
		uint4 v[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t j = j0 + LANES * u;
			const bool in = ALIGN ? j < g.nch : j + 1 < g.nch;
			v[u] = in ? ldc<NT>(g.base + j) : make_uint4(0, 0, 0, 0);
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t j = j0 + LANES * u;
			uint4 x = v[u];
			if (ALIGN && j + 1 == g.nch)
				x = masked(x, 16 * j, g.s0, g.endb);
			s = sum4(x, s);
		}
	}
	return s;
}

template <int LANES, int U, bool ALIGN, bool PIPE, bool NT>
__global__ __launch_bounds__(256, 4) void k_msgs(const uint8_t *__restrict__ frames, const uint64_t *__restrict__ ents,
						 const uint32_t *__restrict__ loff, const uint32_t *__restrict__ lcnt,
						 uint32_t nlists, uint32_t *sink)
{
	constexpr uint32_t GPW = 64 / LANES;
	const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	const uint32_t sub = lane % LANES, grp = lane / LANES;
	uint32_t acc = 0;
	for (uint32_t l = 0; l < 4; l++) {
		const uint32_t li = blockIdx.x * 4 + l;
		if (li >= nlists)
			break;
		const uint32_t cnt = lcnt[li];
		const uint64_t *list = ents + loff[li];
		for (uint32_t k0 = 64 * ((wv + l) % 4); k0 < cnt; k0 += 256) {
			const uint64_t e = k0 + lane < cnt ? list[k0 + lane] : 0;
			if (!PIPE) {
				for (uint32_t q = 0; q < 64 && k0 + q < cnt; q += GPW) {
					const MsgG g = msg_group<ALIGN>(frames, e, q, k0, cnt, grp);
					uint4 v[U], ed = make_uint4(0, 0, 0, 0);
					msg_issue<LANES, U, ALIGN, NT, false>(g, sub, v, ed);
					acc += msg_sum<LANES, U, ALIGN>(g, sub, v, ed) + msg_rest<LANES, U, ALIGN, NT>(g, sub);
				}
			} else {
				uint32_t q = 0;
				MsgG ga = msg_group<ALIGN>(frames, e, q, k0, cnt, grp);
				uint4 va[U], vb[U], ea = make_uint4(0, 0, 0, 0), eb = make_uint4(0, 0, 0, 0);
				msg_issue<LANES, U, ALIGN, NT, true>(ga, sub, va, ea);
				for (;;) {
					const bool more_b = q + GPW < 64 && k0 + q + GPW < cnt;
					MsgG gb = msg_group<ALIGN>(frames, e, q + GPW, k0, cnt, grp);
					if (more_b)
						msg_issue<LANES, U, ALIGN, NT, true>(gb, sub, vb, eb);
					acc += msg_sum<LANES, U, ALIGN>(ga, sub, va, ea) + msg_rest<LANES, U, ALIGN, NT>(ga, sub);
					if (!more_b)
						break;
					q += GPW;
					const bool more_a = q + GPW < 64 && k0 + q + GPW < cnt;
					ga = msg_group<ALIGN>(frames, e, q + GPW, k0, cnt, grp);
					if (more_a)
						msg_issue<LANES, U, ALIGN, NT, true>(ga, sub, va, ea);
					acc += msg_sum<LANES, U, ALIGN>(gb, sub, vb, eb) + msg_rest<LANES, U, ALIGN, NT>(gb, sub);
					if (!more_a)
						break;
					q += GPW;
				}
			}
		}
	}
	if (acc == 0x9E3779B9u)
		sink[0] = acc;
}

// variant: bit 0 ALIGN, bit 1 PIPE, bits 8..15 LANES (4 / 8 / 16), bits 16..23 U
extern "C" int nsd_bw_msgs(const void *frames, const void *ents, const void *loff, const void *lcnt,
			   uint32_t nlists, int variant, int nontemporal, void *stream, uint32_t *sink)
{
	const uint32_t blocks = (nlists + 3) / 4;
	const bool al = variant & 1, pi = variant & 2;
	const int lanes = (variant >> 8) & 0xFF, u = (variant >> 16) & 0xFF;
	// bit 2: 40 KB of dynamic LDS per block, so 4 blocks per CU at most (the fused kernel's residency)
	const size_t lds = (variant & 4) ? 40 * 1024 : 0;
#define NSD_K(L, UU, A, P)                                                                                         \
	if (lanes == L && u == UU && al == A && pi == P) {                                                         \
		if (nontemporal)                                                                                  \
			hipLaunchKernelGGL((k_msgs<L, UU, A, P, true>), dim3(blocks), dim3(256), lds, (hipStream_t)stream, \
					   (const uint8_t *)frames, (const uint64_t *)ents, (const uint32_t *)loff,     \
					   (const uint32_t *)lcnt, nlists, sink);                                        \
		else                                                                                              \
			hipLaunchKernelGGL((k_msgs<L, UU, A, P, false>), dim3(blocks), dim3(256), lds, (hipStream_t)stream, \
					   (const uint8_t *)frames, (const uint64_t *)ents, (const uint32_t *)loff,     \
					   (const uint32_t *)lcnt, nlists, sink);                                        \
		return hipGetLastError() == hipSuccess ? 0 : -1;                                                   \
	}
#define NSD_KA(L, UU) NSD_K(L, UU, false, false) NSD_K(L, UU, true, false) NSD_K(L, UU, false, true) NSD_K(L, UU, true, true)
	NSD_KA(8, 12)
	NSD_KA(8, 8)
	NSD_KA(8, 6)
	NSD_KA(16, 6)
	NSD_KA(16, 8)
	NSD_KA(4, 12)
#undef NSD_KA
#undef NSD_K
	return -2;
}
