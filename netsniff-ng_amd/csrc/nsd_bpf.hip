// nsd_bpf.hip - classic BPF on the device ("BPF on device").
//
// netsniff-ng filters every record before it dissects it: read_pcap
// (netsniff-ng.c:707-725) runs bpf_run_filter (bpf.c:508-705) over the frame
// and skips the record when it returns 0; programs come from
// bpf_parse_rules (bpf.c:707-766) and must pass __bpf_validate
// (bpf.c:388-506).  Here a whole batch is filtered at once: one lane per
// packet interprets the program (decoded once on the host, kept in LDS) over
// its frame in HBM.  The kernel writes the u32 verdict per packet and,
// optionally, the descriptors of the accepted packets in batch order - the
// dissect kernels' input, so a filtered capture goes frames -> filter ->
// dissect without leaving the device.
//
// Roofline: HBM-bound integer work.  Per packet: the 8-B descriptor, the
// frame bytes the program reads (for header filters: the first 64-B line),
// the 4-B verdict; the compaction adds 12 B read + 8 B per accepted packet.
#include <hip/hip_runtime.h>

#include <mutex>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <new>

#include "../../include/netsniff_dissect.h"

namespace nsdbpf {

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;
constexpr uint32_t ROUNDS = 4;                     // packets per lane per tile (compaction)
constexpr uint32_t TILE = ROUNDS * BLOCK;          // packets per block (compaction)
constexpr uint32_t MEMWORDS = 16;                  // BPF_MEMWORDS (bpf.c:30)
constexpr uint32_t MAXINSNS = 4096;                // BPF_MAXINSNS (bpf_insns.h:5)

// Decoded instruction: word x = kind | F_X | F_IND | size << 8 | jt << 16 |
// jf << 24, word y = k.  The host maps each 16-bit code bpf_run_filter's
// switch accepts to one kind; every other code is K_BAD, which returns 0
// like the switch's default (bpf.c:528-529).
enum : uint32_t {
	K_BAD, K_RETK, K_RETA, K_LDP, K_MSH, K_LEN, K_IMM, K_MEM, K_ST, K_JA, K_JGT, K_JGE, K_JEQ,
	K_JSET, K_ADD, K_SUB, K_MUL, K_DIV, K_MOD, K_AND, K_OR, K_XOR, K_LSH, K_RSH, K_NEG, K_TAX,
	K_TXA
};
constexpr uint32_t F_X = 1u << 5;     // X instead of K (operand) / A (destination, ST source)
constexpr uint32_t F_IND = 1u << 6;   // packet offset X + k (BPF_IND)

// code -> kind | flags | size << 8, following bpf_run_filter's cases
static uint32_t decode(uint16_t code)
{
	switch (code) {
	case 0x06: return K_RETK;                           // RET K
	case 0x16: return K_RETA;                           // RET A
	case 0x20: return K_LDP | 4u << 8;                  // LD W ABS
	case 0x28: return K_LDP | 2u << 8;                  // LD H ABS
	case 0x30: return K_LDP | 1u << 8;                  // LD B ABS
	case 0x40: return K_LDP | F_IND | 4u << 8;          // LD W IND
	case 0x48: return K_LDP | F_IND | 2u << 8;          // LD H IND
	case 0x50: return K_LDP | F_IND | 1u << 8;          // LD B IND
	case 0xb1: return K_MSH;                            // LDX B MSH
	case 0x80: return K_LEN;                            // LD W LEN
	case 0x81: return K_LEN | F_X;                      // LDX W LEN
	case 0x00: return K_IMM;                            // LD IMM
	case 0x01: return K_IMM | F_X;                      // LDX IMM
	case 0x60: return K_MEM;                            // LD MEM
	case 0x61: return K_MEM | F_X;                      // LDX MEM
	case 0x02: return K_ST;                             // ST
	case 0x03: return K_ST | F_X;                       // STX
	case 0x05: return K_JA;
	case 0x25: return K_JGT;   case 0x2d: return K_JGT | F_X;
	case 0x35: return K_JGE;   case 0x3d: return K_JGE | F_X;
	case 0x15: return K_JEQ;   case 0x1d: return K_JEQ | F_X;
	case 0x45: return K_JSET;  case 0x4d: return K_JSET | F_X;
	case 0x04: return K_ADD;   case 0x0c: return K_ADD | F_X;
	case 0x14: return K_SUB;   case 0x1c: return K_SUB | F_X;
	case 0x24: return K_MUL;   case 0x2c: return K_MUL | F_X;
	case 0x34: return K_DIV;   case 0x3c: return K_DIV | F_X;
	case 0x94: return K_MOD;   case 0x9c: return K_MOD | F_X;
	case 0x54: return K_AND;   case 0x5c: return K_AND | F_X;
	case 0x44: return K_OR;    case 0x4c: return K_OR | F_X;
	case 0xa4: return K_XOR;   case 0xac: return K_XOR | F_X;
	case 0x64: return K_LSH;   case 0x6c: return K_LSH | F_X;
	case 0x74: return K_RSH;   case 0x7c: return K_RSH | F_X;
	case 0x84: return K_NEG;
	case 0x07: return K_TAX;
	case 0x87: return K_TXA;
	}
	return K_BAD;
}

// big-endian `size`-byte value at p + off (the caller checked off + size <=
// caplen): two aligned dword loads and a byte funnel; the second dword may
// lie up to 7 bytes past the frame, inside the batch's NSD_FRAME_PAD
__device__ __forceinline__ uint32_t pkt_load(const uint8_t *p, uint32_t off, uint32_t size)
{
	const uintptr_t a = (uintptr_t)p + off;
	const uint32_t *q = (const uint32_t *)(a & ~(uintptr_t)3);
	const uint32_t v = __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(a & 3));
	const uint32_t be = __builtin_bswap32(v);
	return size == 4 ? be : size == 2 ? be >> 16 : be >> 24;
}

// Each packet's first 64 bytes, from the 16-byte aligned address at or
// below its start, are staged in LDS before the program runs: a wave's 64
// frames are fetched by four coalesced 16-byte loads per lane (lane L loads
// chunk L & 3 of packet 16 t + L / 4), so a header filter's loads are LDS
// reads instead of a chain of dependent HBM loads per instruction.  A row is
// 16 dwords; chunk c of packet q sits in slot c ^ (q & 3) (lanes reading one
// header offset spread over the banks).  Loads that reach past the row read
// the frame in HBM (pkt_load).
constexpr uint32_t ROWW = 16;

// big-endian `size`-byte value at row position r (r + size <= 64)
__device__ __forceinline__ uint32_t row_load(const uint32_t *row, uint32_t sw, uint32_t r, uint32_t size)
{
	const uint32_t j = r >> 2;
	// (when j + 1 is 16 the bytes lie in dword j alone: the other word is any)
	const uint32_t v = __builtin_amdgcn_alignbyte(row[((j + 1) & 15) ^ sw], row[j ^ sw], r & 3);
	const uint32_t be = __builtin_bswap32(v);
	return size == 4 ? be : size == 2 ? be >> 16 : be >> 24;
}

// bpf_run_filter (bpf.c:508-705) for one packet per lane.  Every program the
// loader accepts jumps forward only, so it retires within `len` steps; the
// step bound is the loop's exit condition regardless.  mem: this lane's
// scratch words M[j] at mem[j * BLOCK]; row / sw / m: the staged first bytes
// (row position = packet offset + m).
__device__ __forceinline__ uint32_t run_one(const uint2 *prog, uint32_t len, uint32_t *mem,
					    bool usesmem, const uint8_t *p, uint32_t plen, bool on,
					    const uint32_t *row, uint32_t sw, uint32_t m)
{
	if (usesmem)
		for (uint32_t j = 0; j < MEMWORDS; j++)
			mem[j * BLOCK] = 0;   // M[] starts zeroed per packet (bpf.c:515)
	uint32_t A = 0, X = 0, pc = 0, ret = 0;
	bool run = on;
	for (uint32_t step = 0; step < len && __ballot(run); step++) {
		if (!run)
			continue;
		const uint2 in = prog[pc];
		pc++;
		const uint32_t kind = in.x & 31, k = in.y;
		const bool fx = in.x & F_X;
		const uint32_t B = fx ? X : k;
		const uint32_t jt = (in.x >> 16) & 0xFF, jf = in.x >> 24;
		switch (kind) {
		case K_RETK: ret = k; run = false; break;
		case K_RETA: ret = A; run = false; break;
		case K_LDP: {
			const uint32_t size = (in.x >> 8) & 7;
			const uint32_t off = ((in.x & F_IND) ? X : 0u) + k;   // IND wraps in 32 bits (bpf.c:562)
			if ((uint64_t)off + size > plen) {
				ret = 0;
				run = false;
			} else {
				const uint32_t r = off + m;   // (off < plen <= 65535)
				A = r + size <= 4 * ROWW ? row_load(row, sw, r, size) : pkt_load(p, off, size);
			}
			break;
		}
		case K_MSH:
			if (k >= plen) {
				ret = 0;
				run = false;
			} else {
				const uint32_t r = k + m;
				X = ((r < 4 * ROWW ? row_load(row, sw, r, 1) : pkt_load(p, k, 1)) & 0xf) << 2;
			}
			break;
		case K_LEN: if (fx) X = plen; else A = plen; break;
		case K_IMM: if (fx) X = k; else A = k; break;
		case K_MEM: {
			const uint32_t v = mem[(k & 15) * BLOCK];
			if (fx) X = v; else A = v;
			break;
		}
		case K_ST: mem[(k & 15) * BLOCK] = fx ? X : A; break;
		case K_JA: pc += k; break;
		case K_JGT: pc += A > B ? jt : jf; break;
		case K_JGE: pc += A >= B ? jt : jf; break;
		case K_JEQ: pc += A == B ? jt : jf; break;
		case K_JSET: pc += (A & B) ? jt : jf; break;
		case K_ADD: A += B; break;
		case K_SUB: A -= B; break;
		case K_MUL: A *= B; break;
		case K_DIV: if (!B) { ret = 0; run = false; } else { A /= B; } break;
		case K_MOD: if (!B) { ret = 0; run = false; } else { A %= B; } break;
		case K_AND: A &= B; break;
		case K_OR: A |= B; break;
		case K_XOR: A ^= B; break;
		case K_LSH: A <<= (B & 31); break;   // the x86 build's shl/shr mask the count
		case K_RSH: A >>= (B & 31); break;
		case K_NEG: A = 0u - A; break;
		case K_TAX: X = A; break;
		case K_TXA: A = X; break;
		default: ret = 0; run = false; break;   // K_BAD
		}
		if (run && pc >= len) {   // cannot happen for a loaded program
			ret = 0;
			run = false;
		}
	}
	return run ? 0u : ret;
}

typedef uint32_t bv4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const bv4u gbv4u;

__device__ __forceinline__ void wave_lds_sync()
{
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// dynamic LDS of a bpf_filter block: the program, the staged rows, and the
// scratch words when the program uses them
__host__ __device__ constexpr size_t prog_bytes(uint32_t len) { return ((size_t)len * 8 + 15) & ~(size_t)15; }
__host__ __device__ constexpr size_t filter_lds(uint32_t len, bool usesmem)
{
	return prog_bytes(len) + (size_t)BLOCK * ROWW * 4 + (usesmem ? (size_t)MEMWORDS * BLOCK * 4 : 0);
}
static_assert(filter_lds(MAXINSNS, true) <= 65536, "a bpf_filter block's LDS");

// One tile of R * BLOCK packets per block: verdicts, and the tile's accepted
// count when compacting.
template <bool COUNT, uint32_t R>
__global__ __launch_bounds__(BLOCK) void bpf_filter(const uint2 *__restrict__ gprog, uint32_t len,
						    uint32_t usesmem, const uint8_t *__restrict__ frames,
						    const uint64_t *__restrict__ desc, uint32_t n,
						    uint32_t *__restrict__ verdict, uint32_t *__restrict__ tile_cnt)
{
	extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
	uint2 *const prog = (uint2 *)lds;
	uint32_t *const rows = (uint32_t *)(lds + prog_bytes(len));
	uint32_t *const mem = rows + BLOCK * ROWW;
	uint32_t *const wcnt = rows;   // (after the rounds; the largest program fills 64 KiB exactly)
	for (uint32_t j = threadIdx.x; j < len; j += BLOCK)
		prog[j] = gprog[j];
	__syncthreads();
	const uint32_t lane = threadIdx.x & 63;
	uint32_t *const wrows = rows + (threadIdx.x & ~63u) * ROWW;
	const uint32_t *const row = wrows + lane * ROWW;
	const uint32_t sw = (lane & 3) << 2;
	uint32_t acc = 0;
	const uint64_t base = (uint64_t)blockIdx.x * (R * BLOCK);
#pragma unroll 1
	for (uint32_t r = 0; r < R; r++) {
		const uint64_t i = base + r * BLOCK + threadIdx.x;
		const bool on = i < n;
		const uint64_t d = on ? desc[i] : 0;
		const uint64_t a = (uint64_t)(uintptr_t)frames + NSD_DESC_OFF(d);
		// the wave's 64 first windows (past the batch: frames[0, 64), readable)
		bv4u v[4];
#pragma unroll
		for (uint32_t t = 0; t < 4; t++) {
			const int q = (int)(16 * t + (lane >> 2));
			const uint64_t aq = (uint64_t)__shfl((uint32_t)a, q, 64) | (uint64_t)__shfl((uint32_t)(a >> 32), q, 64) << 32;
			v[t] = __builtin_nontemporal_load((gbv4u *)(uintptr_t)((aq & ~15ull) + 16 * (lane & 3)));
		}
		wave_lds_sync();   // (the previous round's reads of the rows are done)
#pragma unroll
		for (uint32_t t = 0; t < 4; t++) {
			const uint32_t q = 16 * t + (lane >> 2);
			*(bv4u *)(wrows + q * ROWW + (((lane & 3) ^ (q & 3)) << 2)) = v[t];
		}
		wave_lds_sync();
		const uint32_t vd = run_one(prog, len, mem + threadIdx.x, usesmem != 0, frames + NSD_DESC_OFF(d),
					    NSD_DESC_CAPLEN(d), on, row, sw, (uint32_t)(a & 15));
		if (on)
			verdict[i] = vd;
		acc += (on && vd != 0) ? 1u : 0u;
	}
	if (COUNT) {
		for (int s = 32; s; s >>= 1)
			acc += __shfl_xor(acc, s, 64);
		__syncthreads();   // every wave is done with its rows
		if (lane == 0)
			wcnt[threadIdx.x >> 6] = acc;
		__syncthreads();
		if (threadIdx.x == 0) {
			uint32_t t = 0;
			for (int w = 0; w < WAVES; w++)
				t += wcnt[w];
			tile_cnt[blockIdx.x] = t;
		}
	}
}

// Exclusive scan of the tile counts in place (one block), total to *count.
__global__ __launch_bounds__(1024) void bpf_scan(uint32_t *__restrict__ tile_cnt, uint32_t tiles,
						 uint32_t *__restrict__ count)
{
	__shared__ uint32_t part[16];
	__shared__ uint32_t carry;
	const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	if (threadIdx.x == 0)
		carry = 0;
	__syncthreads();
	for (uint32_t b = 0; b < tiles; b += 1024) {
		const uint32_t i = b + threadIdx.x;
		const uint32_t v = i < tiles ? tile_cnt[i] : 0;
		uint32_t x = v;   // inclusive wave scan
		for (int s = 1; s < 64; s <<= 1) {
			const uint32_t y = __shfl_up(x, s, 64);
			if (lane >= (uint32_t)s)
				x += y;
		}
		if (lane == 63)
			part[wv] = x;
		__syncthreads();
		uint32_t before = carry;
		for (uint32_t w = 0; w < wv; w++)
			before += part[w];
		if (i < tiles)
			tile_cnt[i] = before + x - v;
		__syncthreads();
		if (threadIdx.x == 0) {
			uint32_t t = 0;
			for (int w = 0; w < 16; w++)
				t += part[w];
			carry += t;
		}
		__syncthreads();
	}
	if (threadIdx.x == 0)
		*count = carry;
}

// Accepted descriptors to desc_out[tile offset + rank], in batch order.
__global__ __launch_bounds__(BLOCK) void bpf_compact(const uint32_t *__restrict__ verdict,
						     const uint64_t *__restrict__ desc, uint32_t n,
						     const uint32_t *__restrict__ tile_off,
						     uint64_t *__restrict__ desc_out)
{
	__shared__ uint32_t wcnt[WAVES];
	const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	uint32_t at = tile_off[blockIdx.x];
	const uint64_t base = (uint64_t)blockIdx.x * TILE;
#pragma unroll 1
	for (uint32_t r = 0; r < ROUNDS; r++) {
		const uint64_t i = base + r * BLOCK + threadIdx.x;
		const bool keep = i < n && verdict[i] != 0;
		const uint64_t m = __ballot(keep);
		if (lane == 0)
			wcnt[wv] = (uint32_t)__popcll(m);
		__syncthreads();
		uint32_t before = 0, total = 0;
		for (uint32_t w = 0; w < (uint32_t)WAVES; w++) {
			before += w < wv ? wcnt[w] : 0;
			total += wcnt[w];
		}
		const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
								__builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
		if (keep)
			desc_out[at + before + rank] = desc[i];
		at += total;
		__syncthreads();   // wcnt is reused by the next round
	}
}

} // namespace nsdbpf

// ---- host side: program objects and launches (C ABI) ----------------------
using namespace nsdbpf;

struct nsd_bpf_prog {
	uint32_t len = 0;
	uint32_t usesmem = 0;
	uint2 *d_prog = nullptr;   // decoded program, device memory
	// nsd_bpf_filter_batch's device buffers, kept and grown across calls (a
	// hipFree per batch would synchronise the device under the replay's
	// pipelined batches)
	std::mutex mu;
	uint8_t *d_frames = nullptr;
	size_t frames_cap = 0;
	uint64_t *d_desc = nullptr;
	uint32_t *d_verdict = nullptr;
	size_t n_cap = 0;
};

static bool hip_ok(hipError_t e, const char *what)
{
	if (e != hipSuccess) {
		fprintf(stderr, "netsniff-dissect bpf: %s: %s\n", what, hipGetErrorString(e));
		return false;
	}
	return true;
}

// __bpf_validate (bpf.c:388-506), returning 1 / 0 like the reference
extern "C" int nsd_bpf_validate(const nsd_bpf_insn *prog, uint32_t len)
{
	if (!prog || len < 1)
		return 0;
	for (uint32_t i = 0; i < len; i++) {
		const nsd_bpf_insn &p = prog[i];
		const uint32_t from = i + 1;
		const uint32_t cls = p.code & 0x07, mode = p.code & 0xe0, op = p.code & 0xf0;
		switch (cls) {
		case 0x00:   // LD
		case 0x01:   // LDX
			if (mode == 0x60 && p.k >= MEMWORDS)
				return 0;
			if (mode != 0x00 && mode != 0x20 && mode != 0x40 && mode != 0xa0 && mode != 0x60 &&
			    mode != 0x80)
				return 0;
			break;
		case 0x02:   // ST
		case 0x03:   // STX
			if (p.k >= MEMWORDS)
				return 0;
			break;
		case 0x04:   // ALU: constant division by zero, unknown ops
			if (op == 0x30 || op == 0x90) {
				if ((p.code & 0x18) == 0 && p.k == 0)
					return 0;
			} else if (op != 0x00 && op != 0x10 && op != 0x20 && op != 0x40 && op != 0xa0 &&
				   op != 0x50 && op != 0x60 && op != 0x70 && op != 0x80) {
				return 0;
			}
			break;
		case 0x05:   // JMP: targets checked in 32-bit arithmetic, as the reference
			if (op == 0x00) {
				if ((uint32_t)(from + p.k) >= len)
					return 0;
			} else if (op == 0x10 || op == 0x20 || op == 0x30 || op == 0x40) {
				if (from + p.jt >= len || from + p.jf >= len)
					return 0;
			} else {
				return 0;
			}
			break;
		default:     // RET, MISC
			break;
		}
	}
	return (prog[len - 1].code & 0x07) == 0x06;
}

extern "C" nsd_bpf_prog *nsd_bpf_load(const nsd_bpf_insn *prog, uint32_t len)
{
	if (!nsd_bpf_validate(prog, len) || len > MAXINSNS)
		return nullptr;
	static thread_local uint2 dec[MAXINSNS];
	uint32_t usesmem = 0;
	for (uint32_t i = 0; i < len; i++) {
		const nsd_bpf_insn &p = prog[i];
		// a JA whose target overflows 32 bits passes __bpf_validate and makes
		// the reference jump off the program: refused here
		if ((p.code & 0x07) == 0x05 && (p.code & 0xf0) == 0x00 && (uint64_t)i + 1 + p.k >= len)
			return nullptr;
		// division by a constant 0 passes __bpf_validate too (its check reads
		// BPF_RVAL, bpf.c:447) and traps in the reference: refused here
		if ((p.code == 0x34 || p.code == 0x94) && p.k == 0)
			return nullptr;
		const uint32_t dk = decode(p.code);
		const uint32_t kind = dk & 31;
		usesmem |= (kind == K_MEM || kind == K_ST) ? 1u : 0u;
		dec[i] = make_uint2(dk | (uint32_t)p.jt << 16 | (uint32_t)p.jf << 24, p.k);
	}
	nsd_bpf_prog *h = new (std::nothrow) nsd_bpf_prog;
	if (!h)
		return nullptr;
	h->len = len;
	h->usesmem = usesmem;
	if (!hip_ok(hipMalloc(&h->d_prog, (size_t)len * sizeof(uint2)), "hipMalloc") ||
	    !hip_ok(hipMemcpy(h->d_prog, dec, (size_t)len * sizeof(uint2), hipMemcpyHostToDevice), "H2D")) {
		if (h->d_prog)
			(void)hipFree(h->d_prog);
		delete h;
		return nullptr;
	}
	return h;
}

extern "C" void nsd_bpf_free(nsd_bpf_prog *prog)
{
	if (!prog)
		return;
	if (prog->d_prog)
		(void)hipFree(prog->d_prog);
	if (prog->d_frames)
		(void)hipFree(prog->d_frames);
	if (prog->d_desc)
		(void)hipFree(prog->d_desc);
	if (prog->d_verdict)
		(void)hipFree(prog->d_verdict);
	delete prog;
}

static uint32_t tiles_for(uint32_t n) { return (uint32_t)(((uint64_t)n + TILE - 1) / TILE); }

extern "C" size_t nsd_bpf_workspace_bytes(uint32_t n) { return (size_t)tiles_for(n) * 4 + 256; }

extern "C" int nsd_bpf_filter_device(const nsd_bpf_prog *prog, const uint8_t *d_frames,
				     const nsd_desc_t *d_desc, uint32_t n, uint32_t *d_verdict,
				     nsd_desc_t *d_desc_out, uint32_t *d_count, void *d_workspace,
				     void *stream)
{
	if (!prog || (n && (!d_frames || !d_desc || !d_verdict)))
		return NSD_ERR_ARG;
	const bool compact = d_desc_out != nullptr;
	if ((compact || d_count) && (!d_desc_out || !d_count || !d_workspace))
		return NSD_ERR_ARG;
	hipStream_t s = (hipStream_t)stream;
	if (n == 0) {
		if (compact && !hip_ok(hipMemsetAsync(d_count, 0, 4, s), "memset"))
			return NSD_ERR_HIP;
		return NSD_OK;
	}
	const uint32_t tiles = tiles_for(n);
	uint32_t *tile_cnt = (uint32_t *)d_workspace;
	const size_t lds = filter_lds(prog->len, prog->usesmem != 0);
	if (compact) {
		hipLaunchKernelGGL((bpf_filter<true, ROUNDS>), dim3(tiles), dim3(BLOCK), lds, s, prog->d_prog, prog->len,
				   prog->usesmem, d_frames, (const uint64_t *)d_desc, n, d_verdict, tile_cnt);
		hipLaunchKernelGGL(bpf_scan, dim3(1), dim3(1024), 0, s, tile_cnt, tiles, d_count);
		hipLaunchKernelGGL(bpf_compact, dim3(tiles), dim3(BLOCK), 0, s, (const uint32_t *)d_verdict,
				   (const uint64_t *)d_desc, n, (const uint32_t *)tile_cnt, (uint64_t *)d_desc_out);
	} else {
		// verdicts only: a block per 256 packets (C3 -5 % against 1,024; the
		// compaction keeps 1,024-packet tiles for its one-block scan)
		const uint32_t blocks = (uint32_t)(((uint64_t)n + BLOCK - 1) / BLOCK);
		hipLaunchKernelGGL((bpf_filter<false, 1>), dim3(blocks), dim3(BLOCK), lds, s, prog->d_prog, prog->len,
				   prog->usesmem, d_frames, (const uint64_t *)d_desc, n, d_verdict, nullptr);
	}
	return hip_ok(hipGetLastError(), "launch") ? NSD_OK : NSD_ERR_HIP;
}

// Host-memory batch: H2D, filter, D2H of the verdicts.  Synchronous.
extern "C" int nsd_bpf_filter_batch(const nsd_bpf_prog *prog, const uint8_t *frames, size_t frames_len,
				    const nsd_desc_t *desc, uint32_t n, uint32_t *verdict)
{
	if (!prog || (n && (!frames || !desc || !verdict)))
		return NSD_ERR_ARG;
	if (n == 0)
		return NSD_OK;
	for (uint32_t i = 0; i < n; i++)
		if (NSD_DESC_OFF(desc[i]) + NSD_DESC_CAPLEN(desc[i]) > frames_len)
			return NSD_ERR_ARG;
	nsd_bpf_prog *h = const_cast<nsd_bpf_prog *>(prog);
	std::lock_guard<std::mutex> lk(h->mu);
	bool ok = true;
	if (frames_len + NSD_FRAME_PAD > h->frames_cap) {
		if (h->d_frames)
			(void)hipFree(h->d_frames);
		h->d_frames = nullptr;
		h->frames_cap = 0;
		const size_t want = frames_len + frames_len / 4 + NSD_FRAME_PAD;
		ok = hip_ok(hipMalloc(&h->d_frames, want), "hipMalloc");
		if (ok)
			h->frames_cap = want;
	}
	if (ok && n > h->n_cap) {
		if (h->d_desc)
			(void)hipFree(h->d_desc);
		if (h->d_verdict)
			(void)hipFree(h->d_verdict);
		h->d_desc = nullptr;
		h->d_verdict = nullptr;
		h->n_cap = 0;
		const size_t want = n + n / 4 + 64;
		ok = hip_ok(hipMalloc(&h->d_desc, want * 8), "hipMalloc") &&
		     hip_ok(hipMalloc(&h->d_verdict, want * 4), "hipMalloc");
		if (ok)
			h->n_cap = want;
	}
	ok = ok && hip_ok(hipMemcpy(h->d_frames, frames, frames_len, hipMemcpyHostToDevice), "H2D") &&
	     hip_ok(hipMemset(h->d_frames + frames_len, 0, NSD_FRAME_PAD), "memset") &&
	     hip_ok(hipMemcpy(h->d_desc, desc, (size_t)n * 8, hipMemcpyHostToDevice), "H2D");
	ok = ok && nsd_bpf_filter_device(prog, h->d_frames, (const nsd_desc_t *)h->d_desc, n, h->d_verdict, nullptr,
					 nullptr, nullptr, nullptr) == NSD_OK;
	ok = ok && hip_ok(hipMemcpy(verdict, h->d_verdict, (size_t)n * 4, hipMemcpyDeviceToHost), "D2H");
	return ok ? NSD_OK : NSD_ERR_HIP;
}
