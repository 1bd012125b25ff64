// bw3.hip - the fast kernel's access shape staged by LDS-DMA instead of
// registers: each wave streams 64-packet tiles (64-B frames, one 8-B
// descriptor per packet) through B LDS tile buffers with
// global_load_lds_dwordx4 (nontemporal), descriptors through LDS too (a
// register load's use would drain every LDS-DMA in flight), counted
// s_waitcnt vmcnt(N) waits, the tile "walked" from LDS (SPIN dependent VALU
// ops per lane), one 8-B record per packet stored nontemporally.
// Against bw2 (the same shape with the next tile in registers).
// Build: hipcc --offload-arch=gfx950 -O3 tools/bw/bw3.hip -o tools/bw/bw3
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef uint32_t v2u __attribute__((ext_vector_type(2)));
#define LDS(p) ((__attribute__((address_space(3))) void *)(p))

// LDS-DMA of 16 B per lane to LDS byte address `lds` (wave-uniform) + 16 *
// lane, as inline asm: the compiler then neither drains it at LDS reads
// (hipcc waits vmcnt(0) before any ds_read while a builtin LDS-DMA is
// pending) nor counts it; the waits are ours (wait_vm)
template <int AUX>
__device__ __forceinline__ void glds16(const void *g, uint32_t lds)
{
	uint32_t keep;
	if (AUX)
		asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
			     : "=&s"(keep) : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
	else
		asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
			     : "=&s"(keep) : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void *p)
{
	return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

template <int N>
__device__ __forceinline__ void wait_vm()
{
	asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// per wave: B tile buffers of 4 KiB frames, B + 2 slots of 512 B descriptors.
// Op order per iteration t: wait, D(t+B+1) (descriptors two iterations ahead
// of their frames), F(t+B-1) (4 ops), the walk of tile t, S(t) (the record
// store; on gfx9 stores count in vmcnt too).  F(t) was issued at iteration
// t-B+1; after it come S(t-B+1) and (B-2) x [D, 4 F, S]: vmcnt(1 + 6 (B-2));
// for B = 4 the descriptors D(t+3) of F(t+3) (issued at t-2, after F(t))
// bound it: vmcnt(11).  The first B-1 iterations wait for everything.
template <int B, int SPIN, int AUX>
__global__ __launch_bounds__(256) void k_glds(const uint8_t *__restrict__ frames, const uint64_t *__restrict__ desc,
					      v2u *__restrict__ rec, uint32_t npkt)
{
	constexpr int DS = B + 2;
	extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	uint32_t *const fb = lds + wv * B * 1024;                                   // frames [B][1024 dwords]
	uint64_t *const db = (uint64_t *)(lds + 4 * B * 1024) + wv * DS * 64;      // descriptors [DS][64]
	const uint32_t stride = gridDim.x * 256;
	const uint32_t base0 = blockIdx.x * 256 + wv * 64;
	const uint32_t nt = base0 < npkt ? (npkt - base0 + stride - 1) / stride : 0;
	auto issue_desc = [&](uint32_t t) {
		const uint32_t b = base0 + t * stride;
		if (t < nt && lane < 32)
			glds16<AUX>((const void *)(desc + b + 2 * lane), lds_addr(db + (t % DS) * 64));
	};
	auto issue_frames = [&](uint32_t t) {
		const uint64_t *d = db + (t % DS) * 64;
#pragma unroll
		for (int r = 0; r < 4; r++) {
			const int q = 16 * r + (lane >> 2), c = lane & 3;
			const uint64_t dq = d[q];
			if (t < nt)
				glds16<AUX>((const void *)(frames + (dq & 0xFFFFFFFFFFull) + 16 * c),
					    lds_addr(fb + (t % B) * 1024 + r * 256));
		}
	};
	if (!nt)
		return;
	for (uint32_t t = 0; t <= B; t++)
		issue_desc(t);
	wait_vm<0>();
	for (uint32_t t = 0; t + 1 < B; t++)
		issue_frames(t);
	for (uint32_t t = 0; t < nt; t++) {
		if (t + 1 < B)
			wait_vm<0>();
		else if (B == 2)
			wait_vm<1>();
		else if (B == 3)
			wait_vm<7>();
		else
			wait_vm<11>();
		issue_desc(t + B + 1);
		issue_frames(t + B - 1);
		const uint32_t *row = fb + (t % B) * 1024 + lane * 16;
		uint32_t acc = 0;
#pragma unroll
		for (int j = 0; j < 16; j += 4) {
			const uint4 v = *(const uint4 *)(row + j);
			acc ^= v.x ^ v.y ^ v.z ^ v.w;
		}
		uint32_t x = acc ^ (uint32_t)db[(t % DS) * 64 + lane];
#pragma unroll 1
		for (int s = 0; s < SPIN; s++)
			x = x * 0x9E3779B1u + (x >> 7);
		const uint32_t i = base0 + t * stride + lane;
		const v2u v = { x, acc };
		if (i < npkt)
			__builtin_nontemporal_store(v, rec + i);
	}
	wait_vm<0>();
}

int main()
{
	const uint32_t npkt = 1u << 24;
	uint8_t *a;
	uint64_t *d;
	v2u *rec;
	CHECK(hipMalloc(&a, (size_t)npkt * 64 + 4096));
	CHECK(hipMalloc(&d, (size_t)npkt * 8 + 4096));
	CHECK(hipMalloc(&rec, (size_t)npkt * 8));
	CHECK(hipMemset(a, 1, (size_t)npkt * 64));
	{
		uint64_t *h = (uint64_t *)malloc((size_t)npkt * 8);
		for (uint32_t i = 0; i < npkt; i++)
			h[i] = (uint64_t)i * 64 | (uint64_t)64 << 40;
		CHECK(hipMemcpy(d, h, (size_t)npkt * 8, hipMemcpyHostToDevice));
		free(h);
	}
	int cus = 0;
	CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
	hipEvent_t e0, e1;
	CHECK(hipEventCreate(&e0));
	CHECK(hipEventCreate(&e1));
	typedef void (*kf)(const uint8_t *, const uint64_t *, v2u *, uint32_t);
	struct V {
		int B, spin, aux;
		kf f;
	} vs[] = {
		{ 2, 0, 2, k_glds<2, 0, 2> },   { 3, 0, 2, k_glds<3, 0, 2> },   { 4, 0, 2, k_glds<4, 0, 2> },
		{ 3, 0, 0, k_glds<3, 0, 0> },   { 3, 64, 2, k_glds<3, 64, 2> }, { 4, 64, 2, k_glds<4, 64, 2> },
		{ 3, 128, 2, k_glds<3, 128, 2> },
	};
	for (const V &v : vs) {
		const size_t lds = (size_t)4 * (v.B * 4096 + (v.B + 2) * 512);
		for (int b = 1; b <= 8; b++) {
			if ((size_t)b * lds > 160 * 1024)
				break;
			const int grid = cus * b;
			float ms = 0;
			for (int rep = 0; rep < 30; rep++) {
				if (rep == 10)
					CHECK(hipEventRecord(e0));
				hipLaunchKernelGGL(v.f, dim3(grid), dim3(256), lds, 0, a, d, rec, npkt);
			}
			CHECK(hipEventRecord(e1));
			CHECK(hipEventSynchronize(e1));
			CHECK(hipEventElapsedTime(&ms, e0, e1));
			const double t = ms / 20;
			printf("{\"B\": %d, \"spin\": %d, \"aux\": %d, \"blocks_per_cu\": %d, \"ms_per_16M\": %.4f, \"gbs\": %.1f}\n",
			       v.B, v.spin, v.aux, b, t, (double)npkt * 80 / (t * 1e-3) / 1e9);
		}
	}
	return 0;
}
