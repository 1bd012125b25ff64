// bw.hip - achievable HBM streaming rates on this device (read-only,
// write-only, copy, and the dissector's pass-1 shape: 72 B read + 16 B
// written per 64 B packet), for the roofline notes in DESIGN.md.
// Build: hipcc --offload-arch=gfx950 -O3 tools/bw/bw.hip -o tools/bw/bw
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_read(const uint4 *__restrict__ a, size_t n, uint32_t *out)
{
	uint32_t acc = 0;
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
		const uint4 v = a[i];
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (acc == 0x12345678u)
		out[0] = acc;
}

__global__ void k_write(uint4 *__restrict__ a, size_t n)
{
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
		a[i] = make_uint4((uint32_t)i, 0, 0, 0);
}

__global__ void k_copy(const uint4 *__restrict__ a, uint4 *__restrict__ b, size_t n)
{
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
		b[i] = a[i];
}

// pass-1 shape: per packet 8 B descriptor + 64 B frame read, 16 B record written
__global__ void k_shape(const uint4 *__restrict__ frames, const uint64_t *__restrict__ desc,
			uint4 *__restrict__ rec, size_t npkt)
{
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < npkt; i += (size_t)gridDim.x * blockDim.x) {
		const uint64_t d = desc[i];
		const uint4 *f = frames + 4 * i;
		const uint4 a = f[0], b = f[1], c = f[2], e = f[3];
		rec[i] = make_uint4(a.x ^ b.y ^ (uint32_t)d, c.z ^ e.w, a.y ^ e.x, b.w ^ c.x);
	}
}

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ntl(const uint4 *p)
{
	const v4u v = __builtin_nontemporal_load((const v4u *)p);
	return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nts(uint4 r, uint4 *p)
{
	v4u v = { r.x, r.y, r.z, r.w };
	__builtin_nontemporal_store(v, (v4u *)p);
}
// the same with nontemporal loads (NTL) and/or stores (NTS)
template <bool NTL, bool NTS>
__global__ void k_shape_nt(const uint4 *__restrict__ frames, const uint64_t *__restrict__ desc,
			   uint4 *__restrict__ rec, size_t npkt)
{
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < npkt; i += (size_t)gridDim.x * blockDim.x) {
		const uint64_t d = NTL ? __builtin_nontemporal_load(desc + i) : desc[i];
		const uint4 *f = frames + 4 * i;
		uint4 a, b, c, e;
		if (NTL) {
			a = ntl(f); b = ntl(f + 1); c = ntl(f + 2); e = ntl(f + 3);
		} else {
			a = f[0]; b = f[1]; c = f[2]; e = f[3];
		}
		const uint4 r = make_uint4(a.x ^ b.y ^ (uint32_t)d, c.z ^ e.w, a.y ^ e.x, b.w ^ c.x);
		if (NTS)
			nts(r, rec + i);
		else
			rec[i] = r;
	}
}

// the dissect kernel's staging order: per wave instruction, 4 consecutive
// lanes read one packet's 4 chunks (1 KiB contiguous per instruction), one
// record per packet stored by the lane that owns it; REC = 16 or 8 bytes
template <int REC>
__global__ void k_shape_coal(const uint4 *__restrict__ frames, const uint64_t *__restrict__ desc,
			     uint4 *__restrict__ rec, size_t npkt)
{
	const int lane = threadIdx.x & 63;
	for (size_t base = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) & ~(size_t)63; base < npkt;
	     base += (size_t)gridDim.x * blockDim.x) {
		uint32_t acc = 0;
#pragma unroll
		for (int r = 0; r < 4; r++) {
			const size_t t = base * 4 + r * 64 + lane;   // chunk index
			if (t < npkt * 4) {
				const uint4 v = ntl(frames + t);
				acc ^= v.x ^ v.y ^ v.z ^ v.w;
			}
		}
		acc ^= __shfl_xor(acc, 1, 64) ^ __shfl_xor(acc, 2, 64);
		const size_t i = base + lane;
		if (i < npkt) {
			const uint64_t d = desc[i];
			if (REC == 16) {
				nts(make_uint4(acc ^ (uint32_t)d, acc, 0, 0), rec + i);
			} else {
				typedef uint32_t v2u __attribute__((ext_vector_type(2)));
				const v2u v = { acc ^ (uint32_t)d, acc };
				__builtin_nontemporal_store(v, (v2u *)rec + i);
			}
		}
	}
}

int main()
{
	const size_t bytes = 1ull << 30;
	const size_t n = bytes / 16;
	uint4 *a, *b;
	uint64_t *d;
	uint32_t *o;
	CHECK(hipMalloc(&a, bytes));
	CHECK(hipMalloc(&b, bytes));
	CHECK(hipMalloc(&d, bytes / 8));
	CHECK(hipMalloc(&o, 4));
	CHECK(hipMemset(a, 1, bytes));
	CHECK(hipMemset(b, 2, bytes));
	CHECK(hipMemset(d, 0, bytes / 8));
	int cus = 0;
	CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
	hipEvent_t e0, e1;
	CHECK(hipEventCreate(&e0));
	CHECK(hipEventCreate(&e1));
	const int grids[] = { 4, 8, 16, 32 };
	for (int gi = 0; gi < 4; gi++) {
		const int grid = cus * grids[gi];
		float ms;
		double gbs[4];
		for (int kind = 0; kind < 4; kind++) {
			for (int rep = 0; rep < 6; rep++) {
				if (rep == 1)
					CHECK(hipEventRecord(e0));
				if (kind == 0) hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, n, o);
				if (kind == 1) hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, b, n);
				if (kind == 2) hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, a, b, n);
				if (kind == 3) hipLaunchKernelGGL(k_shape, dim3(grid), dim3(256), 0, 0, a, d, b, n / 4);
			}
			CHECK(hipEventRecord(e1));
			CHECK(hipEventSynchronize(e1));
			CHECK(hipEventElapsedTime(&ms, e0, e1));
			const double t = ms / 5 * 1e-3;
			const double moved = kind == 0 ? bytes : kind == 1 ? bytes : kind == 2 ? 2.0 * bytes
					     : (double)(n / 4) * (64 + 8 + 16);
			gbs[kind] = moved / t / 1e9;
		}
		double nt[3];
		for (int v = 0; v < 3; v++) {
			for (int rep = 0; rep < 6; rep++) {
				if (rep == 1)
					CHECK(hipEventRecord(e0));
				if (v == 0) hipLaunchKernelGGL((k_shape_nt<true, false>), dim3(grid), dim3(256), 0, 0, a, d, b, n / 4);
				if (v == 1) hipLaunchKernelGGL((k_shape_nt<false, true>), dim3(grid), dim3(256), 0, 0, a, d, b, n / 4);
				if (v == 2) hipLaunchKernelGGL((k_shape_nt<true, true>), dim3(grid), dim3(256), 0, 0, a, d, b, n / 4);
			}
			CHECK(hipEventRecord(e1));
			CHECK(hipEventSynchronize(e1));
			CHECK(hipEventElapsedTime(&ms, e0, e1));
			nt[v] = (double)(n / 4) * 88 / (ms / 5 * 1e-3) / 1e9;
		}
		double co[2];
		for (int v = 0; v < 2; v++) {
			for (int rep = 0; rep < 6; rep++) {
				if (rep == 1)
					CHECK(hipEventRecord(e0));
				if (v == 0) hipLaunchKernelGGL((k_shape_coal<16>), dim3(grid), dim3(256), 0, 0, a, d, b, n / 4);
				if (v == 1) hipLaunchKernelGGL((k_shape_coal<8>), dim3(grid), dim3(256), 0, 0, a, d, b, n / 4);
			}
			CHECK(hipEventRecord(e1));
			CHECK(hipEventSynchronize(e1));
			CHECK(hipEventElapsedTime(&ms, e0, e1));
			co[v] = (double)(n / 4) * (v == 0 ? 88 : 80) / (ms / 5 * 1e-3) / 1e9;
		}
		printf("{\"blocks_per_cu\": %d, \"read_gbs\": %.1f, \"write_gbs\": %.1f, \"copy_gbs\": %.1f, \"pass1_shape_gbs\": %.1f, \"shape_ntload\": %.1f, \"shape_ntstore\": %.1f, \"shape_nt_both\": %.1f, \"coal_rec16_gbs\": %.1f, \"coal_rec8_gbs\": %.1f, \"coal_rec16_ms_per_16M\": %.4f, \"coal_rec8_ms_per_16M\": %.4f}\n",
		       grids[gi], gbs[0], gbs[1], gbs[2], gbs[3], nt[0], nt[1], nt[2], co[0], co[1],
		       16777216.0 * 88 / co[0] / 1e6, 16777216.0 * 80 / co[1] / 1e6);
	}
	return 0;
}
