// bw2.hip - the split schedule's fast-kernel access shape against
// occupancy: a persistent grid of B blocks per CU (B = 4..8, all resident),
// each wave grid-striding over 64-packet tiles of 64-B frames, the next
// tile's four 16-B chunks per lane in flight (registers) while the current
// tile is "walked" (SPIN dependent VALU ops per lane), one 8-B record per
// packet stored nontemporally.  The ceiling dissect_fast's C2 launch can
// reach at each occupancy.
// Build: hipcc --offload-arch=gfx950 -O3 tools/bw/bw2.hip -o tools/bw/bw2
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

template <int SPIN>
__global__ __launch_bounds__(256, 8) void k_pref(const uint4 *__restrict__ frames, const uint64_t *__restrict__ desc,
						 v2u *__restrict__ rec, uint32_t npkt)
{
	const int lane = threadIdx.x & 63;
	const uint32_t stride = gridDim.x * 256;
	uint32_t base = blockIdx.x * 256 + (threadIdx.x & ~63u);
	if (base >= npkt)
		return;
	v4u ch[4];
#pragma unroll
	for (int r = 0; r < 4; r++)
		ch[r] = __builtin_nontemporal_load((const v4u *)(frames + (size_t)base * 4 + r * 64 + lane));
	uint64_t d0 = desc[base + lane];
	for (; base < npkt; base += stride) {
		uint32_t acc = 0;
#pragma unroll
		for (int r = 0; r < 4; r++)
			acc ^= ch[r].x ^ ch[r].y ^ ch[r].z ^ ch[r].w;
		const uint32_t nb = base + stride;
		uint64_t d1 = 0;
		if (nb < npkt) {
#pragma unroll
			for (int r = 0; r < 4; r++)
				ch[r] = __builtin_nontemporal_load((const v4u *)(frames + (size_t)nb * 4 + r * 64 + lane));
			d1 = desc[nb + lane];
		}
		// the walk: SPIN dependent integer ops
		uint32_t x = acc ^ (uint32_t)d0;
#pragma unroll 1
		for (int s = 0; s < SPIN; s++)
			x = x * 0x9E3779B1u + (x >> 7);
		const v2u v = { x, acc };
		__builtin_nontemporal_store(v, rec + base + lane);
		d0 = d1;
	}
}

// the same with two tiles in flight per wave (two register sets, the loop
// unrolled by two so the sets swap roles without copies)
template <int SPIN>
__global__ __launch_bounds__(256, 4) void k_pref2(const uint4 *__restrict__ frames, const uint64_t *__restrict__ desc,
						  v2u *__restrict__ rec, uint32_t npkt)
{
	const int lane = threadIdx.x & 63;
	const uint32_t stride = gridDim.x * 256;
	uint32_t base = blockIdx.x * 256 + (threadIdx.x & ~63u);
	if (base >= npkt)
		return;
	v4u A[4], B[4];
	auto ld = [&](v4u *c, uint32_t b) {
		if (b < npkt) {
#pragma unroll
			for (int r = 0; r < 4; r++)
				c[r] = __builtin_nontemporal_load((const v4u *)(frames + (size_t)b * 4 + r * 64 + lane));
		}
	};
	auto tile = [&](v4u *c, uint32_t b, uint64_t d) {
		uint32_t acc = 0;
#pragma unroll
		for (int r = 0; r < 4; r++)
			acc ^= c[r].x ^ c[r].y ^ c[r].z ^ c[r].w;
		ld(c, b + 2 * stride);
		uint32_t x = acc ^ (uint32_t)d;
#pragma unroll 1
		for (int s = 0; s < SPIN; s++)
			x = x * 0x9E3779B1u + (x >> 7);
		const v2u v = { x, acc };
		__builtin_nontemporal_store(v, rec + b + lane);
	};
	ld(A, base);
	ld(B, base + stride);
	uint64_t d0 = desc[base + lane];
	for (;;) {
		const uint64_t d1 = base + stride < npkt ? desc[base + stride + lane] : 0;
		tile(A, base, d0);
		base += stride;
		if (base >= npkt)
			break;
		d0 = base + stride < npkt ? desc[base + stride + lane] : 0;
		tile(B, base, d1);
		base += stride;
		if (base >= npkt)
			break;
	}
}

int main()
{
	const uint32_t npkt = 1u << 24;
	uint4 *a;
	uint64_t *d;
	v2u *rec;
	CHECK(hipMalloc(&a, (size_t)npkt * 64));
	CHECK(hipMalloc(&d, (size_t)npkt * 8));
	CHECK(hipMalloc(&rec, (size_t)npkt * 8));
	CHECK(hipMemset(a, 1, (size_t)npkt * 64));
	CHECK(hipMemset(d, 0, (size_t)npkt * 8));
	int cus = 0;
	CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
	hipEvent_t e0, e1;
	CHECK(hipEventCreate(&e0));
	CHECK(hipEventCreate(&e1));
	for (int spin : { 0, 64, 128, 256 }) {
		for (int b = 2; b <= 8; b++) {
			const int grid = cus * b;
			float ms = 0;
			for (int rep = 0; rep < 40; rep++) {
				if (rep == 20)
					CHECK(hipEventRecord(e0));
				if (spin == 0) hipLaunchKernelGGL(k_pref<0>, dim3(grid), dim3(256), 0, 0, a, d, rec, npkt);
				if (spin == 64) hipLaunchKernelGGL(k_pref<64>, dim3(grid), dim3(256), 0, 0, a, d, rec, npkt);
				if (spin == 128) hipLaunchKernelGGL(k_pref<128>, dim3(grid), dim3(256), 0, 0, a, d, rec, npkt);
				if (spin == 256) hipLaunchKernelGGL(k_pref<256>, dim3(grid), dim3(256), 0, 0, a, d, rec, npkt);
			}
			CHECK(hipEventRecord(e1));
			CHECK(hipEventSynchronize(e1));
			CHECK(hipEventElapsedTime(&ms, e0, e1));
			const double t = ms / 20;
			printf("{\"spin\": %d, \"blocks_per_cu\": %d, \"ms_per_16M\": %.4f, \"gbs\": %.1f}\n", spin, b, t,
			       (double)npkt * 80 / (t * 1e-3) / 1e9);
		}
	}
	for (int spin : { 0, 64, 128 }) {
		for (int b = 2; b <= 4; b++) {
			const int grid = cus * b;
			float ms = 0;
			for (int rep = 0; rep < 40; rep++) {
				if (rep == 20)
					CHECK(hipEventRecord(e0));
				if (spin == 0) hipLaunchKernelGGL(k_pref2<0>, dim3(grid), dim3(256), 0, 0, a, d, rec, npkt);
				if (spin == 64) hipLaunchKernelGGL(k_pref2<64>, dim3(grid), dim3(256), 0, 0, a, d, rec, npkt);
				if (spin == 128) hipLaunchKernelGGL(k_pref2<128>, dim3(grid), dim3(256), 0, 0, a, d, rec, npkt);
			}
			CHECK(hipEventRecord(e1));
			CHECK(hipEventSynchronize(e1));
			CHECK(hipEventElapsedTime(&ms, e0, e1));
			const double t = ms / 20;
			printf("{\"depth\": 2, \"spin\": %d, \"blocks_per_cu\": %d, \"ms_per_16M\": %.4f, \"gbs\": %.1f}\n", spin, b, t,
			       (double)npkt * 80 / (t * 1e-3) / 1e9);
		}
	}
	return 0;
}
