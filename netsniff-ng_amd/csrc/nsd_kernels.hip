// nsd_kernels.hip - CDNA4 (gfx950) kernels for the netsniff-ng dissector chain.
//
// One lane walks one packet (nsd_walk.h).  Layout in HBM:
//   frames  : one byte buffer, frames at arbitrary offsets
//   desc    : u64 per packet (bits 0..39 offset, 40..63 caplen)
//   rec     : 16-byte chain record per packet (nsd_rec), one dwordx4 store per
//             lane -> 1 KiB contiguous per wave
//   ext     : overflow records for deep chains, slots by wave-aggregated atomic
//   counters: u64[64] per-ops / flag counts
//
// Header windows are staged through LDS in "aligned coordinates": a frame at
// byte offset `off` is read from A = off & ~15 in whole 16-byte chunks (every
// load a global_load_dwordx4, whatever the frame's alignment; AF_PACKET rings
// put the MAC header at 2 mod 16), and frame byte o sits at window position
// o + m, m = off & 15.  Window bytes at frame offsets >= caplen are zeroed.
// Each lane's fast-walk window is one LDS row of 20 dwords: 16-byte aligned
// rows take one ds_write_b128 per chunk, and 32 lanes reading the same
// header offset meet at most 2-way in a bank (an odd 17-dword stride was
// conflict-free but needed 4 ds_write_b32 per chunk: 1.3 % slower on C2).
//
// The fast walk finishes every packet whose chain resolves inside its first
// 64 bytes, with the next tile's chunks and the tile after next's descriptors
// in flight while the current tile is walked from LDS only.  The tile's
// other packets go to the wave's walkers, the general walk (walkers):
// per-lane windows staged at each walker's cursor, idle walkers refilled,
// ext spill; ICMPv4 payload checksums longer than a window are summed by the
// block at the end.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <mutex>

#include "nsd_walk.h"

namespace nsd {

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;

// Summed over launches on this device and sampled now and then by the
// launcher to choose the schedule (split or fused, nsd_launch_dissect_rec):
// [0] packets the fast walk handed to the general walk, [1] ICMPv4 messages
// left to a checksum pass (longer than their window)
constexpr int WIN1 = 64;         // bytes per staged window, pass 1
#ifndef NSD_WIN2
#define NSD_WIN2 128
#endif
constexpr int WIN2 = NSD_WIN2;   // bytes per staged window, general-walk continuation
// fast-walk window row stride in dwords (16-byte aligned rows, see top)
constexpr int row_of(int W) { return W / 4 + 4; }
#ifndef NSD_CSUM_U
#define NSD_CSUM_U 12              // interior chunk loads in flight per lane (icmp_pass)
#endif
#ifndef NSD_GROUP_TILES
#define NSD_GROUP_TILES 1          // fused waves take their tiles at run time from a counter per CU group
#endif
#ifndef NSD_GROUP_BLOCKS
#define NSD_GROUP_BLOCKS 4u        // blocks sharing a tile counter (4: one CU's; 8: two CUs of one XCD)
#endif
#ifndef NSD_PRIO
#define NSD_PRIO 1                 // fused waves' issue priority by their tile progress (walk_tiles)
#endif
#ifndef NSD_CSUM_LANES
#define NSD_CSUM_LANES 8           // lanes per message in icmp_pass (each group instruction: 8 = one 128-B line)
#endif
#ifndef NSD_MINW
#define NSD_MINW 4                 // waves per SIMD the fused kernel is register-allocated for
#endif
#ifndef NSD_L2PF
#define NSD_L2PF 16                // a tile with this many deferred packets is walker-heavy (NSD_LATE)
#endif
#ifndef NSD_LATE
#define NSD_LATE 1                 // a walker-heavy tile's successor loads its chunks after the walkers (0: before, with L2 touches)
#endif
#ifndef NSD_FAST_EXT
#define NSD_FAST_EXT 1             // the fused kernel's fast walk steps extension headers in its window
#endif
#ifndef NSD_WIN_NT
#define NSD_WIN_NT 1               // the walkers' window loads nontemporal (stage_glds)
#endif
#ifndef NSD_RING
#define NSD_RING 1                 // the fused kernel's compact records through the per-wave record ring (RingSt)
#endif
#ifndef NSD_CSUM_SPLIT
#define NSD_CSUM_SPLIT 1           // dissect_icmp blocks per pass-1 block
#endif

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
// a chunk in global memory: an address rebuilt from shuffled integers is a
// generic pointer, which compiles to flat_load; flat loads count in lgkmcnt
// too, so every LDS wait of the walk would also wait for the next tile's
// chunks.  Loads through this type are global_load.
typedef __attribute__((address_space(1))) const v4u gv4u;
__device__ __forceinline__ uint32_t lanes_below(uint64_t m)
{
	return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v)
{
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		v += __shfl_xor(v, o, 64);
	return v;
}

// The frame's bytes straight from HBM (zero past caplen), for the leaf walks
struct HbmBytes {
	const uint8_t *p;
	uint32_t caplen;
	__device__ __forceinline__ uint8_t b(uint32_t o) const { return o < caplen ? p[o] : 0; }
	__device__ __forceinline__ uint16_t be16(uint32_t o) const { return (uint16_t)(b(o) << 8 | b(o + 1)); }
};

// Byte source over an LDS window (aligned coordinates, see top).
// FAST (the fast walk): the window is a zero-padded row (bytes past caplen
// zeroed by stage_write; 20-dword rows, or the split schedule's 16-dword rows
// with their 16-byte slots XOR-swizzled by sw); bytes outside it are not fetched, the
// source records the miss and the walk gives the packet up to the general
// walk.  Otherwise (the general walk's continuation windows, stage_glds): a
// row of up to WIN bytes filled by LDS-DMA with its 16-byte slots
// XOR-swizzled (dword j at j ^ sw) and nothing zeroed, so every read masks
// the bytes at offsets >= caplen itself; only its first wl bytes are staged
// (a walker's window ends at a line boundary, walkers()), and bytes outside
// them come from HBM.
template <bool FAST, int WIN>
struct LSrc {
	const uint32_t *win;     // this lane's window row
	const uint8_t *lay3t;    // LDS copy of eth_lay3
	const uint32_t *stept;   // LDS copy of c_step, then c_lay2h (general walk)
	const uint8_t *p;        // frame in HBM
	uint32_t caplen;
	uint32_t m;              // off & 15
	uint32_t wb;             // aligned position of window byte 0 (multiple of 16)
	mutable bool miss;
	uint32_t sw;             // continuation rows: slot swizzle (dword index xor)
	uint32_t wl = WIN;       // bytes of the row staged from wb (continuation rows; FAST: WIN)

	__device__ __forceinline__ uint32_t dw(uint32_t j) const { return win[j ^ sw]; }
	__device__ __forceinline__ int lay3(uint32_t key) const { return lay3t[key & 255]; }
	__device__ __forceinline__ uint32_t step(int id) const { return stept[id & 31]; }
	__device__ __forceinline__ uint32_t l2h(uint32_t h) const { return stept[32 + (h & 31)]; }
	// bytes o .. o+3 (little-endian) from the window row: two dwords and a
	// byte funnel shift.  Meaningful only for bytes inside the window (a
	// near_end() budget covers them).  FAST: zero at offsets >= caplen.  The
	// continuation rows are not zeroed past caplen and this read does not
	// mask them: it serves gen_step's layer bytes (B0, the next-ops key) only,
	// every use of which is gated by the layer's first pull succeeding
	// (pulled: the bytes it reads lie before tail <= caplen), so a byte past
	// the frame never reaches a result (C4 -1.4 %: 6 VALU per read).
	__device__ __forceinline__ uint32_t dword_at(uint32_t o) const
	{
		const uint32_t r = o + m - wb;
		uint32_t j = r >> 2;
		j = j > WIN / 4 - 1 ? WIN / 4 - 1 : j;
		const uint32_t v = __builtin_amdgcn_alignbyte(dw(j + 1), dw(j), r & 3);
		if constexpr (FAST)
			return o >= caplen ? 0u : v;
		return v;
	}
	__device__ __forceinline__ bool missed() const { return miss; }
	__device__ __forceinline__ uint8_t b(uint32_t o) const
	{
		const uint32_t r = o + m - wb;
		if constexpr (FAST) {
			if (r < WIN)
				return (uint8_t)(dw(r >> 2) >> ((r & 3) * 8));
			if (o < caplen)
				miss = true;
			return 0;
		} else {
			if (o >= caplen)
				return 0;
			return r < wl ? (uint8_t)(dw(r >> 2) >> ((r & 3) * 8)) : p[o];
		}
	}
	__device__ __forceinline__ uint16_t le16(uint32_t o) const
	{
		const uint32_t r = o + m - wb;
		if (r + 1 < wl && (r & 3) != 3 && (FAST || o + 2 <= caplen))
			return (uint16_t)(dw(r >> 2) >> ((r & 3) * 8));
		return (uint16_t)(b(o) | b(o + 1) << 8);
	}
	__device__ __forceinline__ uint16_t be16(uint32_t o) const
	{
		return (uint16_t)__builtin_bswap16(le16(o));
	}
	// bytes o .. o+15 as four little-endian dwords (5 window dwords + byte
	// funnel shifts).  Only the bytes the caller's near_end() budget covers
	// are meaningful (later ones may come from the next window row); bytes
	// at offsets >= caplen are zero.
	__device__ __forceinline__ void bytes16(uint32_t o, uint32_t &B0, uint32_t &B1, uint32_t &B2,
						uint32_t &B3) const
	{
		const uint32_t r = o + m - wb;
		uint32_t j = r >> 2;
		j = j > WIN / 4 - 1 ? WIN / 4 - 1 : j;
		const uint32_t sh = r & 3;
		const uint32_t w0 = dw(j), w1 = dw(j + 1), w2 = dw(j + 2), w3 = dw(j + 3), w4 = dw(j + 4);
		const bool z = o >= caplen;
		B0 = z ? 0u : __builtin_amdgcn_alignbyte(w1, w0, sh);
		B1 = z ? 0u : __builtin_amdgcn_alignbyte(w2, w1, sh);
		B2 = z ? 0u : __builtin_amdgcn_alignbyte(w3, w2, sh);
		B3 = z ? 0u : __builtin_amdgcn_alignbyte(w4, w3, sh);
	}
	__device__ __forceinline__ bool in_window(uint32_t o, uint32_t nbytes) const
	{
		const uint32_t r = o + m - wb;
		return r < wl && r + nbytes <= wl;
	}
	// window bytes from frame offset o to the window's end
	__device__ __forceinline__ uint32_t window_bytes(uint32_t o) const
	{
		const uint32_t r = o + m - wb;
		return r < wl ? wl - r : 0u;
	}
	// the next layer would read past the staged window (the bytes its parse
	// inspects from its start, c_step's `need`): general walk only
	__device__ __forceinline__ bool near_end(uint32_t o, int id) const
	{
		return near_end_i(o, step(id));
	}
	// the same from the ops' rule word
	__device__ __forceinline__ bool near_end_i(uint32_t o, uint32_t info) const
	{
		const uint32_t need = info >> 25;
		return need && o < caplen && o + m + need > wb + wl;
	}
	// sum of `nwords` little-endian u16 words from `o` (csum.h:16-17)
	__device__ __forceinline__ uint32_t sum16(uint32_t o, uint32_t nwords) const
	{
		uint32_t sum = 0;
		const uint32_t r = o + m - wb;
		if (FAST && !(r & 1)) {
			// the fast walk sums only inside the window (its callers check
			// in_window).  Even start: a leading half, whole dwords four
			// reads at a time (independent LDS reads, one wait per four:
			// an IPv4 header of 20 bytes is one round), a trailing half.
			// Reads past the count are selected away (they stay in LDS).
			uint32_t j = r >> 2, k = nwords;
			if ((r & 2) && k) { sum += dw(j) >> 16; j++; k--; }
			const uint32_t nd = k >> 1;
			for (uint32_t t = 0; t < nd; t += 4) {
				const uint32_t v0 = dw(j + t), v1 = dw(j + t + 1), v2 = dw(j + t + 2), v3 = dw(j + t + 3);
				sum = __builtin_amdgcn_sad_u16(v0, 0u, sum);
				sum = __builtin_amdgcn_sad_u16(t + 1 < nd ? v1 : 0u, 0u, sum);
				sum = __builtin_amdgcn_sad_u16(t + 2 < nd ? v2 : 0u, 0u, sum);
				sum = __builtin_amdgcn_sad_u16(t + 3 < nd ? v3 : 0u, 0u, sum);
			}
			if (k & 1) sum += dw(j + nd) & 0xFFFF;
			return sum;
		}
		if (FAST) {
			// odd start (frames at odd offsets): the dword at window position
			// r, funnel-shifted out of two row dwords, holds the words at o
			// and o + 2; two per round, then a trailing word
			const uint32_t j = r >> 2, sh = r & 3, nd = nwords >> 1;
			for (uint32_t t = 0; t < nd; t += 2) {
				const uint32_t v0 = dw(j + t), v1 = dw(j + t + 1), v2 = dw(j + t + 2);
				sum = __builtin_amdgcn_sad_u16(__builtin_amdgcn_alignbyte(v1, v0, sh), 0u, sum);
				sum = __builtin_amdgcn_sad_u16(t + 1 < nd ? __builtin_amdgcn_alignbyte(v2, v1, sh) : 0u, 0u,
							       sum);
			}
			if (nwords & 1)
				sum += __builtin_amdgcn_alignbyte(dw(j + nd + 1), dw(j + nd), sh) & 0xFFFF;
			return sum;
		}
		if (!(r & 1) && in_window(o, 2 * nwords) && o + 2 * nwords <= caplen) {
			uint32_t j = r >> 2, k = nwords;
			if ((r & 2) && k) { sum += dw(j) >> 16; j++; k--; }
			for (; k >= 2; k -= 2, j++)
				sum = __builtin_amdgcn_sad_u16(dw(j), 0u, sum);   // + both 16-bit halves
			if (k) sum += dw(j) & 0xFFFF;
			return sum;
		}
		for (uint32_t i = 0; i < nwords; i++)
			sum += le16(o + 2 * i);
		return sum;
	}
};

// ---- staging ---------------------------------------------------------------
// Chunk r of the wave: lane (q * CPP + c) % 64 in round (q * CPP + c) / 64
// loads chunk c of packet q's window, so the CPP chunks of one packet are
// read by consecutive lanes as one contiguous, 16-byte aligned segment.

template <int WIN>
struct Chunks {
	static constexpr int CPP = WIN / 16;   // 16-byte chunks per window
	static_assert(CPP <= 4 && WIN <= 255, "a chunk's valid count per byte of nv");
	uint4 v[CPP];
	uint32_t nv;   // valid bytes of chunk r (0..16) in byte r
};

// issue the loads (no wait): in round r, lane (q * CPP + c) % 64 loads chunk
// c of packet q's window = aligned bytes [A_q + 16c, +16), skipped when the
// chunk lies wholly past caplen.  Each lane prepares its own packet's
// aligned start address and frame end once; two shuffles per round hand
// them to the loading lanes (the end, capped at 255 - the window is shorter
// - rides in the address's high dword, a 48-bit VA leaves its top byte
// free).  The count of valid bytes per chunk is kept for stage_write.
// ALL (the split fast loop): every chunk load is issued, chunks wholly past
// caplen too (stage_write zeroes them; a 64-byte window always lies inside
// the frame buffer's NSD_FRAME_PAD): a load under a branch leaves hipcc
// unsure whether it is pending, and it then waits vmcnt(0) for the chunks.
// NT: streaming loads; false where the general walk re-reads the lines soon.
template <int WIN, bool ALL = false, bool NT = true>
__device__ __forceinline__ void stage_load(Chunks<WIN> &ch, const uint8_t *frames, uint64_t my_desc, int lane)
{
	constexpr int CPP = Chunks<WIN>::CPP;
	const uint64_t a = (uint64_t)frames + (NSD_DESC_OFF(my_desc) & ~15ull);
	const uint32_t lim = (uint32_t)NSD_DESC_CAPLEN(my_desc) + ((uint32_t)my_desc & 15);
	const uint32_t hr = (uint32_t)(a >> 32) | (lim < 255u ? lim : 255u) << 24;
	ch.nv = 0;
#pragma unroll
	for (int r = 0; r < CPP; r++) {
		const int t = r * 64 + lane;
		const int q = t / CPP, c = t % CPP;
		const uint32_t alo = __shfl((uint32_t)a, q, 64), ahr = __shfl(hr, q, 64);
		const uint32_t pos = 16u * c, qlim = ahr >> 24;
		const uint32_t nv = qlim > pos ? min(qlim - pos, 16u) : 0u;
		if (ALL || nv) {
			// streaming loads (nt): C2 -9 %, C3 -2 %; C4 +5 % (its general
			// walk re-reads the first line from HBM rather than L2)
			const uint64_t src = ((uint64_t)(ahr & 0xFFFFFFu) << 32 | alo) + pos;
			v4u t4;
			if constexpr (NT)
				t4 = __builtin_nontemporal_load((const gv4u *)src);
			else
				t4 = *(const gv4u *)src;
			ch.v[r] = make_uint4(t4.x, t4.y, t4.z, t4.w);
		} else {
			ch.v[r] = make_uint4(0, 0, 0, 0);
		}
		ch.nv |= nv << (8 * r);
	}
}

// write the chunks to the window rows (row q, dwords 4c..4c+3), zeroing the
// bytes at frame offsets >= caplen
template <int WIN>
__device__ __forceinline__ void stage_write(uint32_t *wwin, const Chunks<WIN> &ch, int lane)
{
	constexpr int CPP = Chunks<WIN>::CPP, ROW = row_of(WIN);
#pragma unroll
	for (int r = 0; r < CPP; r++) {
		const int t = r * 64 + lane;
		const int q = t / CPP, c = t % CPP;
		const uint32_t nv = (ch.nv >> (8 * r)) & 0xFF;
		uint32_t w[4] = { ch.v[r].x, ch.v[r].y, ch.v[r].z, ch.v[r].w };
		if (nv < 16) {
#pragma unroll
			for (int j = 0; j < 4; j++) {
				const uint32_t bp = 4 * j;
				if (bp >= nv)
					w[j] = 0;
				else if (bp + 4 > nv)
					w[j] &= (1u << ((nv - bp) * 8)) - 1u;
			}
		}
		*(uint4 *)(wwin + q * ROW + c * 4) = make_uint4(w[0], w[1], w[2], w[3]);
	}
}

// The continuation windows (WIN bytes per lane, CPP = WIN / 16 slots) by
// LDS-DMA: wave-instruction r's lane l fills slot l % CPP of row
// q = r * (64 / CPP) + l / CPP (the destination is lane-linear), loading
// chunk (l % CPP) ^ swz(q) of packet q's window, so row q holds its chunk c
// in slot c ^ swz(q) and the lanes reading one window offset spread over
// the banks (dword j of row q at j ^ (swz(q) << 2)).  No VGPR holds the
// window on the way.  Chunks wholly past the frame are not loaded (the
// source masks the bytes past caplen instead).  The loads are nontemporal
// (NSD_WIN_NT): a window's lines are read once, and as L2-allocating loads
// they pushed out the packets' first lines that the late chunk loads had
// just brought in for the walkers (C4: 308.6 -> 259.4 B/packet read, 40.5M
// -> 34.0M 128-byte requests per launch against a line floor of 262.9;
// kernel time unchanged).  abase: this lane's aligned
// window start in HBM; rem: bytes from there to the frame's aligned end (0:
// the lane takes no window).
__device__ __forceinline__ uint32_t swz_of(uint32_t q, int cpp) { return (q >> 1) & (uint32_t)(cpp - 1); }

template <int WIN>
__device__ __forceinline__ void stage_glds(uint32_t *wwin, uint64_t abase, uint32_t rem, int lane)
{
	constexpr int CPP = WIN / 16, PER = 64 / CPP;
	static_assert(CPP * PER == 64, "a window size whose slots tile a wave");
	const uint32_t lo = (uint32_t)abase;
	// the high address dword (a 48-bit VA) shares its word with min(rem, 0xFFFF)
	const uint32_t hr = (uint32_t)(abase >> 32) | (rem < 0xFFFFu ? rem : 0xFFFFu) << 16;
#pragma unroll 2
	for (int r = 0; r < CPP; r++) {
		const int q = r * PER + lane / CPP;
		const uint32_t alo = __shfl(lo, q, 64), ahr = __shfl(hr, q, 64);
		const uint32_t c = ((uint32_t)lane % CPP) ^ swz_of((uint32_t)q, CPP);
		if (16 * c < (ahr >> 16)) {
			const uint64_t a = ((uint64_t)(ahr & 0xFFFFu) << 32 | alo) + 16 * c;
			__builtin_amdgcn_global_load_lds((const void *)a,
							 (__attribute__((address_space(3))) void *)(wwin + r * 256), 16, 0,
							 NSD_WIN_NT ? 2 : 0);
		}
	}
	// the DMA's LDS writes are ordered for this wave's reads by its vmcnt only
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Touch the first line(s) of a packet's fast window so a later load of it
// hits L2: one 4-byte LDS-DMA load per line (64 lanes write 256 bytes of
// `dummy`, an LDS area nothing reads, so no VGPR waits for the line).  Both
// lines when the window straddles a 128-byte line.
__device__ __forceinline__ void l2_touch(const uint8_t *frames, uint64_t d, uint32_t *dummy, bool on)
{
	const uint64_t a = (uint64_t)frames + NSD_DESC_OFF(d);
	const uint32_t span = NSD_DESC_CAPLEN(d) < 64 ? (uint32_t)NSD_DESC_CAPLEN(d) : 64u;
	if (on)
		__builtin_amdgcn_global_load_lds((const void *)(a & ~127ull),
						 (__attribute__((address_space(3))) void *)dummy, 4, 0, 0);
	if (on && (a & 127) + span > 128)
		__builtin_amdgcn_global_load_lds((const void *)((a & ~127ull) + 128),
						 (__attribute__((address_space(3))) void *)dummy, 4, 0, 0);
}

__device__ __forceinline__ void wave_sync_lds()
{
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ICMPv4 checksum helpers (calc_csum over the whole message, csum.h:12-27).
// Only whether the checksum is zero is kept (NSD_F_ICMP_BAD).  Sums run over
// the 16-bit halves of 16-byte aligned loads with the bytes outside the
// message masked off.  For a message at an odd address that weights every
// byte by 256 relative to the reference's LE words, i.e. multiplies the sum
// by 256 mod 0xFFFF (65536 = 1), so the folded sum is 0xFFFF exactly when the
// reference's is (RFC 1071 byte-order independence) and the checksum is zero
// exactly when the reference's is.  Partial sums may be folded early: folding
// keeps the value mod 0xFFFF and keeps it non-zero.

// byte mask of the dword at aligned position p for message bytes [s0, endb)
__device__ __forceinline__ uint32_t msg_mask(uint32_t p, uint32_t s0, uint32_t endb)
{
	uint32_t m = 0xFFFFFFFFu;
	if (s0 > p)
		m = s0 >= p + 4 ? 0u : m << (8 * (s0 - p));
	if (endb < p + 4)
		m = endb <= p ? 0u : m & (0xFFFFFFFFu >> (8 * (p + 4 - endb)));
	return m;
}

// acc + low half + high half (v_sad_u16 against zero)
__device__ __forceinline__ uint32_t sum_halves(uint32_t x, uint32_t acc)
{
	return __builtin_amdgcn_sad_u16(x, 0u, acc);
}

// chunk at aligned position lo, bytes outside [s0, endb) masked per lane
__device__ __forceinline__ uint32_t csum_chunk(const uint4 &v, uint32_t lo, uint32_t s0, uint32_t endb)
{
	uint32_t acc = sum_halves(v.x & msg_mask(lo, s0, endb), 0u);
	acc = sum_halves(v.y & msg_mask(lo + 4, s0, endb), acc);
	acc = sum_halves(v.z & msg_mask(lo + 8, s0, endb), acc);
	return sum_halves(v.w & msg_mask(lo + 12, s0, endb), acc);
}

__device__ __forceinline__ uint16_t csum_final(uint32_t sum)
{
	sum = (sum >> 16) + (sum & 0xffff);
	sum += (sum >> 16);
	return (uint16_t)~sum;
}

// Streaming record store: nontemporal (written once, read by the host or a
// later kernel), measured 6 % faster than a plain store in the pass-1 access
// shape (tools/bw: 72 B read + 16 B written per packet).
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void store_rec(uint4 *rec, uint32_t i, uint4 r)
{
	const v4u v = { r.x, r.y, r.z, r.w };
	__builtin_nontemporal_store(v, (v4u *)(rec + i));
}

// The record of packet i in the launch's record form: the 16-byte nsd_rec,
// or (CR) the 8-byte nsd_crec - the same results without the cursors a
// renderer re-derives from the bytes: the first 6 ids, the layer count in
// nlayers for 7..12 layers (ids 6..11 in the packet's side word), or the ext
// slot of a longer chain
__device__ __forceinline__ uint2 crec_of(const WalkOut &w)
{
	const bool more = w.n > NSD_REC_MAX_LAYERS;
	const uint32_t nf = (more ? NSD_N_EXT : w.n) | w.flags;
	const uint32_t rs = more && !w.ext_on ? w.n : 0u;
	return make_uint2(w.ext_on ? w.slot : w.chain, w.ip_csum | nf << 16 | rs << 24);
}

template <bool CR>
__device__ __forceinline__ void put_rec(void *rec, uint32_t i, const WalkOut &w)
{
	if constexpr (CR) {
		const uint2 r = crec_of(w);
		__builtin_nontemporal_store(v2u{ r.x, r.y }, (v2u *)rec + i);
	} else {
		store_rec((uint4 *)rec, i, pack_record(w));
	}
}

// The fused tile loop's pending-list entries and, without the record ring
// (NSD_RING 0: r05's schedule), its compact records, held one tile: a
// tile's stores are issued after the next tile's
// chunk wait and before its prefetch loads, so the wait that precedes each
// tile (vmcnt(0): its chunks are the youngest loads) finds them issued a
// whole tile earlier (C3 -1 %).  (Nontemporal stores: as sc1 stores, the
// split kernel's choice below, C3 ran 1.5 % slower.)  Measured on the C3
// tile phase without its walk: the record stores cost 0.07
// of its 0.35 ms however they are issued - every tile or every fourth in 4x
// larger pieces, 8 or 16 bytes per lane, held or not - i.e. the writes'
// interleaving with the scattered window reads in HBM, not a wait in this
// loop.  The 16-byte form stores at once (held, its four words spill the
// fused kernel's registers).
template <bool CR>
struct HeldSt {
	uint2 r;          // the compact record (nsd_crec)
	uint32_t ri;      // packet index of the record; ~0: none
	uint64_t pe;      // pending-list entry
	uint32_t pp;      // its slot; ~0: none
	__device__ __forceinline__ void hold_rec(uint32_t i, uint2 rv, bool on)
	{
		ri = on ? i : 0xFFFFFFFFu;
		r = rv;
	}
	__device__ __forceinline__ void hold_pend(uint64_t *wq, uint64_t e, uint32_t slot)
	{
		if constexpr (!CR) {
			if (slot != 0xFFFFFFFFu)
				wq[slot] = e;   // (not held either, as the 16-byte record)
			return;
		}
		pe = e;
		pp = slot;
	}
	__device__ __forceinline__ void flush(void *rec, uint64_t *wq)
	{
		if constexpr (!CR)
			return;
		if (ri != 0xFFFFFFFFu)
			__builtin_nontemporal_store(v2u{ r.x, r.y }, (v2u *)rec + ri);
		if (pp != 0xFFFFFFFFu)
			wq[pp] = pe;
		ri = pp = 0xFFFFFFFFu;
	}
};

// The split fast loop's stores.  With NSD_FAST_ASMST they are inline-asm
// vector stores: hipcc's waitcnt pass treats the vector-memory counter as
// out of order while loads and stores are both pending and then waits
// vmcnt(0) for a tile's chunks - for every later chunk load and every store
// too, which defeats a deeper prefetch.  It does not see these stores, so its
// waits count the loop's loads alone; loads complete in order among
// themselves, so a wait that leaves N later loads outstanding still covers
// the load it waits for, whatever the stores do.  Their completion is ours:
// drain_stores() before anything reads what they wrote.  The compact record
// stores use the sc1 policy (written through, the line dropped from the
// XCD's L2; MI355X_MICROARCH.md "stores of each flavour"): C2 0.2069 - 0.2092
// -> 0.2036 - 0.2049 ms against nontemporal stores on one box (records are
// read by the host or another kernel, never by this wave again); the 16-byte
// records stay nontemporal (sc1 there: +12 %).  A store of more
// than 8 bytes reads its data registers over two cycles, and hipcc's hazard
// recognizer does not know an asm statement is such a store: the next VALU
// could overwrite the data before it is read (gfx9's 12-dword store hazard;
// without the wait state a depth-3 build wrote corrupt list entries and
// faulted the GPU).  The 16-byte forms end in s_nop 1.
#ifndef NSD_FAST_DEPTH
#define NSD_FAST_DEPTH 2           // tiles of chunks in flight per fast wave (1..3)
#endif
#ifndef NSD_FAST_ASMST
#define NSD_FAST_ASMST (NSD_FAST_DEPTH > 1)
#endif
__device__ __forceinline__ void st_b32(uint32_t *p, uint32_t v)
{
	if (NSD_FAST_ASMST)
		asm volatile("global_store_dword %0, %1, off" ::"v"(p), "v"(v) : "memory");
	else
		*p = v;
}
__device__ __forceinline__ void st_b128(uint4 *p, uint4 x)
{
	if (NSD_FAST_ASMST) {
		const v4u v = { x.x, x.y, x.z, x.w };
		asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
	} else {
		*p = x;
	}
}
__device__ __forceinline__ void drain_stores()
{
	if (NSD_FAST_ASMST)
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
template <bool CR>
__device__ __forceinline__ void put_rec_st(void *rec, uint32_t i, const WalkOut &w)
{
	if (!NSD_FAST_ASMST) {
		put_rec<CR>(rec, i, w);
	} else if constexpr (CR) {
		const uint2 r = crec_of(w);
		const v2u v = { r.x, r.y };
		asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"((v2u *)rec + i), "v"(v) : "memory");
	} else {
		const uint4 r = pack_record(w);
		const v4u v = { r.x, r.y, r.z, r.w };
		// (16-byte records stay nontemporal: with sc1 0.2667 - 0.2677 ms
		// against 0.2370 - 0.2378)
		asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" ::"v"((uint4 *)rec + i), "v"(v) : "memory");
	}
}

// byte offset of packet i's nflags in the record array
template <bool CR>
__device__ __forceinline__ size_t nflags_at(uint32_t i)
{
	return CR ? (size_t)i * 8 + 6 : (size_t)i * 16 + 10;
}

// Per-wave flag counters: wave-uniform (ballot + popcount, scalar registers);
// only the byte count is per lane.
struct FlagCnt {
	uint32_t pkts = 0, ipbad = 0, icmpbad = 0, host = 0, ext = 0, ovf = 0, trim = 0;
	uint64_t bytes = 0;
	__device__ __forceinline__ static uint32_t pc(bool c) { return (uint32_t)__popcll(__ballot(c)); }
	__device__ __forceinline__ void add(const WalkOut &w, uint32_t caplen, bool on)
	{
		pkts += pc(on);
		ipbad += pc(on && w.ip_csum != 0);
		icmpbad += pc(on && (w.flags & NSD_F_ICMP_BAD));
		host += pc(on && (w.flags & NSD_F_HOST));
		ext += pc(on && w.need_ext);
		ovf += pc(on && (w.flags & NSD_F_OVERFLOW));
		trim += pc(on && w.tail < caplen);
		if (on)
			bytes += caplen;
	}
	// -> block LDS counters
	__device__ __forceinline__ void flush(unsigned long long *s_cnt, int lane) const
	{
		const uint32_t vals[7] = { pkts, ipbad, icmpbad, host, ext, ovf, trim };
		const int idx[7] = { NSD_CNT_PKTS, NSD_CNT_IP_BAD, NSD_CNT_ICMP_BAD, NSD_CNT_HOST,
				     NSD_CNT_EXT, NSD_CNT_OVERFLOW, NSD_CNT_TRIM };
		if (lane == 0) {
#pragma unroll
			for (int k = 0; k < 7; k++)
				if (vals[k])
					atomicAdd(&s_cnt[idx[k]], (unsigned long long)vals[k]);
		}
		const uint64_t b = wave_sum64(bytes);
		if (lane == 0 && b)
			atomicAdd(&s_cnt[NSD_CNT_BYTES], (unsigned long long)b);
	}
};

__device__ __forceinline__ void block_init(unsigned long long *s_cnt, uint8_t *s_lay3)
{
	for (int k = threadIdx.x; k < NSD_NCOUNTERS; k += BLOCK)
		s_cnt[k] = 0;
	for (int k = threadIdx.x; k < 256; k += BLOCK)
		s_lay3[k] = c_lay3[k];
	__syncthreads();
}

__device__ __forceinline__ void block_flush(unsigned long long *s_cnt, unsigned long long *counters)
{
	__syncthreads();
	for (int k = threadIdx.x; k < NSD_NCOUNTERS; k += BLOCK)
		if (s_cnt[k])
			atomicAdd(&counters[k], s_cnt[k]);
}

// Pending ICMPv4 checksums: entry = packet index | message offset << 32 |
// message length << 48 (offsets and lengths are < 65536).  Each wave of a
// block keeps one list (room for every packet it visits).
__device__ __forceinline__ uint64_t pend_entry(uint32_t i, uint32_t off, uint32_t len)
{
	return (uint64_t)i | (uint64_t)(off & 0xFFFF) << 32 | (uint64_t)(len & 0xFFFF) << 48;
}

// ---- the fused kernel ---------------------------------------------------------
// Block-level shared state of one dissect launch.
// a wave's window area: the fast walk's 20-dword rows, then (same words) the
// continuation's WIN2-byte rows
constexpr int WINWORDS = 64 * row_of(WIN1) > 16 * WIN2 ? 64 * row_of(WIN1) : 16 * WIN2;
struct Shared {
	alignas(16) uint32_t win[WAVES][WINWORDS];              // staged windows (fast walk, then continuations)
	unsigned long long cnt[NSD_NCOUNTERS];      // block counters
	uint32_t ops[32];                           // block per-ops layer counts (32-bit LDS atomics)
	uint8_t lay3[256];                          // eth_lay3
	uint32_t step[64];                          // c_step, c_lay2h (general walk)
	uint32_t wc[WAVES][2];                      // per-wave ext pool chunk {next word, words left}
	uint32_t pcnt[WAVES];                       // pending checksums per wave
	// general-walk layer lists (layers 6..11, 16-byte records); compact
	// records keep no layer starts, and the fused kernel's waves use the
	// words as their record rings (RecRing)
	alignas(16) uint32_t lay[WAVES][NSD_LDS_LAYERS * 64];
	uint8_t tmap[WAVES][64];                    // take(): pending lane of each rank
};

// The fused kernel's record ring (compact records of walker-heavy batches:
// a build of its own, dissect_all<MODE, true, true>, which the launcher runs
// when the schedule sample defers more than a quarter of the packets; the
// plain build holds a tile's records one tile in registers, HeldSt, which do
// not fit beside the ring's code: 11 VGPRs spilled, C3 +28 %, and stored
// right after the fast walk instead C3 ran 4 % slower).  In the ring build
// a tile whose packets the fast walk all finishes stores its records at
// once, right after its fast walk.  A tile with deferred packets has its
// records written
// twice over: by the fast walk (the packets it finishes) and later by the
// walkers' sessions (each session's finished packets), often across two
// tiles.  Stored to HBM as they came, a 128-byte line of records (16
// packets) was written in two or three pieces microseconds apart, and the
// XCD's L2 had let the line go in between, so each piece cost its own
// partial-line writes (C4: 17.4 B/packet written for 8 B of records, and
// 6.3 more for the side words' 4-byte stores; TCC_EA0_WRREQ: 37 % of the
// requests 32-byte ones).  Here each wave keeps two such tiles' records and
// side words in LDS (the compact form's unused layer-list words: 2 x 64 x 8
// B + 2 x 64 x 4 B = 1,536 B a wave) and stores a tile's records in one
// coalesced wave store (512 B, whole lines) once its last packet is
// finished; its side words likewise (256 B) when any packet of the tile has
// one (C4), zero for the tile's packets without one.  A slot needed by a new
// tile while packets of its old tile are still held by walkers (walked
// across two more tiles) stores the finished ones at once, and those
// walkers store theirs directly (the tile has left the ring).  The state is
// wave-uniform and lives in scalar registers (a round trip to LDS for it
// before each tile's prefetch loads cost 5 %).  C4: 23.7 -> 12.2 B/packet
// written per launch, kernel time within the box's noise (+-1 %: C4's
// walker steps, not its bytes, set its time).
constexpr uint32_t RING_NONE = 0xFFFFFFFFu;
struct RingSt {
	// (scalars, never an array indexed at run time: that would go to scratch)
	uint32_t tb0, tb1;       // the tile (first packet) of slot 0 / 1, RING_NONE: free
	uint32_t left0, left1;   // its packets not yet finished
	uint32_t any;            // bit s: a packet of slot s's tile has a side word
	uint32_t next;           // the slot the next tile with deferrals takes
	__device__ __forceinline__ void init()
	{
		tb0 = tb1 = RING_NONE;
		left0 = left1 = any = next = 0;
	}
	__device__ __forceinline__ uint32_t tb(int s) const { return s ? tb1 : tb0; }
	__device__ __forceinline__ uint32_t left(int s) const { return s ? left1 : left0; }
	__device__ __forceinline__ void set(int s, uint32_t t, uint32_t l)
	{
		if (s) {
			tb1 = t;
			left1 = l;
		} else {
			tb0 = t;
			left0 = l;
		}
	}
};
// this wave's slots (addresses recomputed at each use: nothing of them stays
// live across the walker engine, whose registers are at their limit)
__device__ __forceinline__ uint2 *ring_rec(Shared &sh)
{
	return (uint2 *)&sh.lay[__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))][0];
}
__device__ __forceinline__ uint32_t *ring_side(Shared &sh)
{
	return &sh.lay[__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))][256];
}
static_assert(NSD_LDS_LAYERS * 64 >= 2 * 64 * 2 + 2 * 64, "two tiles of compact records and side words");

// Lanes with fin finished packet i with record r and side word sv (0:
// none): into its tile's slot, or straight to HBM when the tile is not in
// the ring.  Wave-uniform call.
__device__ __forceinline__ void ring_put(Shared &sh, RingSt &rs, bool fin, uint32_t i, uint2 r, uint32_t sv,
					 void *__restrict__ rec, uint32_t *__restrict__ side)
{
	const uint32_t tb = i & ~63u;
	const int sl = !fin ? -1 : tb == rs.tb0 ? 0 : tb == rs.tb1 ? 1 : -1;
	if (sl >= 0) {
		ring_rec(sh)[sl * 64 + (i & 63)] = r;
		ring_side(sh)[sl * 64 + (i & 63)] = sv;
	} else if (fin) {
		__builtin_nontemporal_store(v2u{ r.x, r.y }, (v2u *)rec + i);
		if (sv)
			side[i] = sv;
	}
	rs.left0 -= (uint32_t)__popcll(__ballot(sl == 0));
	rs.left1 -= (uint32_t)__popcll(__ballot(sl == 1));
	rs.any |= (__ballot(sl == 0 && sv != 0) ? 1u : 0u) | (__ballot(sl == 1 && sv != 0) ? 2u : 0u);
}

// Store slot s's tile - the records of its packets (lane k: packet tb + k;
// `held`: still on a walker, not stored) in one wave store, its side words
// in another when any is set - and free the slot.  Wave-uniform call.
__device__ __forceinline__ void ring_store(Shared &sh, RingSt &rs, int s, bool held, void *__restrict__ rec,
					   uint32_t *__restrict__ side, uint32_t n, int lane)
{
	wave_sync_lds();
	const uint32_t i = rs.tb(s) + (uint32_t)lane;
	const bool on = !held && i < n;
	const uint2 r = ring_rec(sh)[s * 64 + lane];
	if (on)
		__builtin_nontemporal_store(v2u{ r.x, r.y }, (v2u *)rec + i);
	if (rs.any & (1u << s)) {
		const uint32_t sv = ring_side(sh)[s * 64 + lane];
		if (on)
			side[i] = sv;
	}
	wave_sync_lds();   // (the slot's next writes after these reads)
	rs.set(s, RING_NONE, 0);
	rs.any &= ~(1u << s);
}

// A tile with `nd` deferred packets (nd > 0) takes the next slot (free:
// ring_turn) with the records of the packets the fast walk finished (`done`)
__device__ __forceinline__ void ring_open(Shared &sh, RingSt &rs, uint32_t base, uint32_t nd, bool done, uint2 r,
					  uint32_t sv, int lane)
{
	const int s = (int)rs.next;
	if (done) {
		ring_rec(sh)[s * 64 + lane] = r;
		ring_side(sh)[s * 64 + lane] = sv;
	}
	rs.set(s, base, nd);
	rs.any |= __ballot(done && sv != 0) ? 1u << s : 0u;
	rs.next ^= 1u;
}

// The LINKTYPE_LINUX_SLL head (dissector_sll.c:39-82): pulls nothing; in
// print_full the next ops come from the packet's sockaddr_ll (sll_next).
template <int MODE>
__device__ __forceinline__ void sll_head(Shared &sh, WalkOut &w, const uint32_t *__restrict__ sll, uint32_t i)
{
	const uint32_t w0 = sll ? sll[5 * (size_t)i] : 0u;       // sll_family | sll_protocol << 16
	const uint32_t w2 = sll ? sll[5 * (size_t)i + 2] : 0u;   // sll_hatype | pkttype << 16 | halen << 24
	const uint32_t hatype = w2 & 0xFFFF;
	const uint32_t proto = __builtin_bswap16((uint16_t)(w0 >> 16));
	w.chain = NSD_OPS_SLL;
	w.n = 1;
	atomicAdd(&sh.ops[NSD_OPS_SLL], 1u);
	w.id = sll_next(hatype, proto, MODE, sh.step[32 + NSD_L2H(proto)]);
}

// A wave's pending list (wq, `wcap` slots: one per packet the wave visits)
// holds the ICMPv4 checksums left to icmp_pass from the front (npend) and
// the host-rendered leaves left to leaf_pass from the back (nleaf); a packet
// ends in at most one of the two.
struct Pending {
	uint64_t *wq;
	uint32_t wcap;
	uint32_t npend, nleaf;
};

// leaf entry: packet index | leaf start << 32 | ops id << 48 (16-byte
// records), packet index | leaf start << 32 | tail << 48 (compact records,
// whose record has no tail; the id is the chain's last)
__device__ __forceinline__ uint64_t leaf_entry(uint32_t i, uint32_t start, int id)
{
	return (uint64_t)i | (uint64_t)(start & 0xFFFF) << 32 | (uint64_t)id << 48;
}
__device__ __forceinline__ uint64_t leaf_entry_c(uint32_t i, uint32_t start, uint32_t tail)
{
	return (uint64_t)i | (uint64_t)(start & 0xFFFF) << 32 | (uint64_t)(tail & 0xFFFF) << 48;
}

// What a lane whose general walk ended leaves behind (wave-uniform call):
// an ICMPv4 message past its windows and a host-rendered leaf go to the
// wave's pending list, an ext chain to the pool (layers 0..5 from the record
// registers, 6..11 from the wave's LDS list, deeper ones already in the
// entry), then the record and the flag counts.  Compact records keep a
// chain of 7..12 layers in the packet's side word (ids 6..11, 5 bits each:
// one coalesced 4-byte store instead of a pool entry, C4 -25 %); only
// longer chains (entry taken at layer 12 by take_deep) write an entry, with
// ids only.
template <int MODE, bool CR, bool RING>
__device__ __forceinline__ void emit_general(Shared &sh, RingSt &rs, bool fin, WalkOut &w, uint32_t i,
					     uint32_t caplen, const GenSink<CR> &g, void *__restrict__ rec, Pending &pq,
					     FlagCnt &fc, int lane)
{
	// a host-rendered leaf's end is walked by the leaf pass: into the 16-byte
	// record's cursor, or (compact records with side words) into the side
	// word of a chain of up to 6 layers or word 2 of an entry past 12 layers
	const bool lf = fin && w.leaf != 0 &&
			(!CR || (g.side && (w.n <= NSD_REC_MAX_LAYERS || (w.ext_on && w.slot != 0xFFFFFFFFu &&
									   w.n <= NSD_EXT_MAX_LAYERS))));
	const uint64_t lm = __ballot(lf);
	if (lf) {
		pq.wq[pq.wcap - 1 - (pq.nleaf + lanes_below(lm))] =
			CR ? leaf_entry_c(i, w.data, w.tail) : leaf_entry(i, w.data, w.leaf);
		if (CR)
			w.flags |= NSD_F_LEAF_END;
	}
	pq.nleaf += (uint32_t)__popcll(lm);
	uint64_t *const wq = pq.wq;
	uint32_t &npend = pq.npend;
	if (MODE == PRINT_NORM) {
		const bool pnd = fin && w.icmp_pend;
		const uint64_t pm = __ballot(pnd);
		if (pnd)
			wq[npend + lanes_below(pm)] = pend_entry(i, w.icmp_off, w.icmp_len);
		npend += (uint32_t)__popcll(pm);
	}
	constexpr uint32_t DEEP = NSD_REC_MAX_LAYERS + NSD_LDS_LAYERS;
	static_assert(DEEP == NSD_CREC_MAX_LAYERS, "side words hold the LDS-listed layers");
	// (a 7..12-layer chain's side word: ids 6..11, never 0)
	const bool sw = CR && fin && w.n > NSD_REC_MAX_LAYERS && !w.ext_on;
	if constexpr (CR) {
		if (sw && g.side && !RING)
			g.side[i] = w.offB;
		if (sw && !g.side)
			w.flags |= NSD_F_OVERFLOW;   // no side words: the pool is smaller than the batch
	}
	const bool ex = fin && (CR ? w.ext_on : w.need_ext);
	if (__ballot(ex)) {
		const bool tk = ex && !w.ext_on;
		if (!CR) {
			const uint32_t sb = ext_take(g, tk, NSD_EXT_WORDS(DEEP));
			if (tk) {
				w.slot = sb;
				w.ext_on = true;
			}
		}
		if (ex && w.slot == 0xFFFFFFFFu)
			w.flags |= NSD_F_OVERFLOW;   // the pool is full
		if (ex && w.slot != 0xFFFFFFFFu) {
			uint32_t *e = g.pool + w.slot;
			const uint32_t nl = w.n < NSD_EXT_MAX_LAYERS ? w.n : NSD_EXT_MAX_LAYERS;
			auto lv = [&](uint32_t j) -> uint32_t {
				if (CR)   // ids only
					return j < NSD_REC_MAX_LAYERS ? (w.chain >> (5 * j)) & 31
								      : (w.offB >> (5 * (j - NSD_REC_MAX_LAYERS))) & 31;
				if (j < NSD_REC_MAX_LAYERS)
					return ((w.chain >> (5 * j)) & 31) | (uint32_t)off_of(w, j) << 16;
				return j < nl ? g.lay[(j - NSD_REC_MAX_LAYERS) * 64 + lane] : 0u;
			};
			// layers 0 .. DEEP-1 (deeper ones are in the entry already)
			static_assert(DEEP % 4 == 0 && DEEP <= 16, "whole uint4 groups of a short entry");
			*(uint4 *)e = make_uint4(i, nl, 0, 0);
#pragma unroll
			for (uint32_t g0 = 0; g0 < DEEP; g0 += 4)
				if (g0 == 0 || nl > g0)
					*(uint4 *)(e + 4 + g0) = make_uint4(lv(g0), lv(g0 + 1), lv(g0 + 2), lv(g0 + 3));
		}
	}
	if (CR && RING)
		ring_put(sh, rs, fin, i, crec_of(w), sw && g.side ? w.offB : 0u, rec, g.side);
	else if (fin)
		put_rec<CR>(rec, i, w);
	fc.add(w, caplen, fin);
}

// The general walk's pool: every lane of a wave is also a walker that holds
// (at most) one packet the fast walk could not finish.  A tile's deferred
// packets are handed to free walkers in lane order; a session stages the
// windows of the walkers that need one (new, or suspended at the end of
// their window) and steps every walker that can step.  While packets are
// still waiting for a walker, a session stops as soon as NSD_REFILL walkers
// are idle, to take them; the tile's last session runs until every walker
// is done or suspended, and the suspended ones are carried to the next
// tile's session (their next window would be restaged anyway).  So a tile
// costs one window wait (1.15 sessions per C4 tile against 2 rounds) and
// its steps run with refilled lanes (7.2 layer steps per C4 tile against 9.8
// when each tile's deferred lanes are walked to their ends).
#ifndef NSD_REFILL
#define NSD_REFILL 16   // idle walkers at which a session stops to take waiting packets
#endif
struct Walker {
	WalkOut w;
	uint64_t d;       // its packet's descriptor
	uint32_t i;       // its packet's index
	uint32_t wb;      // aligned position of its staged window
	uint32_t wl;      // bytes of it staged
	bool have;        // holds a packet
	bool stage;       // its window must be (re)staged before it steps again
};

// The ring at the point where the previous tile's held stores go out
// (walk_tiles, before the next tile's loads): every tile whose packets are
// all finished is stored, and the slot the next tile with deferrals takes,
// if its tile still has packets on walkers (walked across two more tiles),
// stores the finished ones and leaves the ring.
__device__ __forceinline__ void ring_turn(Shared &sh, RingSt &rs, const Walker &wk, void *__restrict__ rec,
					  uint32_t *__restrict__ side, uint32_t n, int lane)
{
#pragma unroll
	for (int k = 0; k < 2; k++)
		if (rs.tb(k) != RING_NONE && rs.left(k) == 0)
			ring_store(sh, rs, k, false, rec, side, n, lane);
	const int s = (int)rs.next;
	if (rs.tb(s) != RING_NONE) {
		// which of the tile's packets walkers hold: a byte per packet in the
		// wave's take() map (free outside take)
		const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
		sh.tmap[wv][lane] = 0;
		wave_sync_lds();
		if (wk.have && (wk.i & ~63u) == rs.tb(s))
			sh.tmap[wv][wk.i & 63] = 1;
		wave_sync_lds();
		const bool held = sh.tmap[wv][lane] != 0;
		ring_store(sh, rs, s, held, rec, side, n, lane);
	}
}

// How much of a walker's window to stage (walkers()).  An HBM read costs
// whole 128-byte lines, and a chain's later layers need only a few bytes
// each (c_step's `need`: 4 for an extension header, none for a leaf), so a
// window that runs into the next line past the chain's end fetches a line
// nothing reads.  The window ends at the end of the line holding the next
// layer's needed bytes, or of the line after it when fewer than
// NSD_WIN_AHEAD bytes of that line would be left past them (the chain then
// likely goes on there); a walker whose next layer needs no bytes (a leaf)
// stages nothing.  C4 (line model over the oracle's layer starts): 1.09
// staged windows per packet against 0.93, 233 against 279 distinct bytes
// per packet.
#ifndef NSD_WIN_LINES
#define NSD_WIN_LINES 1
#endif
#ifndef NSD_WIN_AHEAD
#define NSD_WIN_AHEAD 32
#endif
__device__ __forceinline__ uint32_t window_len(uint64_t abs_wb, uint64_t abs_cur, uint32_t need)
{
	if (!NSD_WIN_LINES)
		return WIN2;
	if (!need)
		return 0;
	uint64_t le = ((abs_cur + need - 1) | 127) + 1;
	if (le - (abs_cur + need) < NSD_WIN_AHEAD)
		le += 128;
	const uint64_t l = le - abs_wb;
	return l < WIN2 ? (uint32_t)l : (uint32_t)WIN2;
}

// Hand the waiting packets (lanes with pnd: the tile's deferred packets, walk
// state pw after walk_init / the fast walk's layers) to free walkers: the
// waiting lane of rank r goes to the free walker of rank r (a lane map in
// LDS, then one shuffle per state word).
template <bool CR>
__device__ __forceinline__ void take(Shared &sh, Walker &wk, bool &pnd, const WalkOut &pw, uint32_t pi, uint64_t pd,
				     int lane, int wv);

template <int MODE, bool CR, bool RING>
__device__ __forceinline__ void walkers(Shared &sh, RingSt &rs, const uint8_t *__restrict__ frames, void *__restrict__ rec,
					const GenSink<CR> &g, Pending &pq, FlagCnt &fc, Walker &wk, bool &pnd,
					const WalkOut &pw, uint32_t pi, uint64_t pd, bool drain)
{
	constexpr int ROW = WIN2 / 4;
	const int lane = threadIdx.x & 63;
	const int wv = threadIdx.x >> 6;
	for (;;) {
		take<CR>(sh, wk, pnd, pw, pi, pd, lane, wv);
		if (!__ballot(wk.have))
			break;
		const bool more = __ballot(pnd) != 0;
		// ---- a session
		const uint64_t off = NSD_DESC_OFF(wk.d);
		const uint32_t caplen = NSD_DESC_CAPLEN(wk.d), m = (uint32_t)off & 15;
		const bool st = wk.have && wk.stage;
		const uint64_t fbase = (uint64_t)(frames + (off & ~15ull));
		if (st) {
			wk.wb = (wk.w.data + m) & ~15u;
			wk.wl = window_len(fbase + wk.wb, fbase + wk.w.data + m, sh.step[wk.w.id & 31] >> 25);
		}
		if (__ballot(st)) {
			// (the window's HBM address and extent are recomputed from the
			// descriptor rather than kept live across the walk: registers)
			const uint32_t lim = caplen + m;   // first aligned position past the frame
			uint32_t rem = st && wk.wb < lim ? lim - wk.wb : 0u;
			rem = rem < wk.wl ? rem : wk.wl;
			stage_glds<WIN2>(&sh.win[wv][0], fbase + wk.wb, rem, lane);
		}
		const LSrc<false, WIN2> src{ &sh.win[wv][lane * ROW], sh.lay3, sh.step, frames + off,
					     caplen, m, wk.wb, false, swz_of((uint32_t)lane, WIN2 / 16) << 2, wk.wl };
		bool susp, act;
		uint32_t info;   // the stepping ops' rule word (gen_step reuses it)
		auto ready = [&](uint32_t inf) {
			const bool run = wk.have && wk.w.id != 0;
			info = inf;
			susp = run && src.near_end_i(wk.w.data, info);
			act = run && !susp;
			const uint64_t am = __ballot(act);
			// stop when no walker can step, or enough are idle to take
			// waiting packets
			return am != 0 && !(more && __popcll(am) <= 64 - NSD_REFILL);
		};
		// (a plain leaf - TCP / UDP / ESP / NoNext, no byte read - run in
		// the step that reached it, so its chain ends an iteration earlier:
		// C4 1.002 against 0.956 ms, r06 gpu_s8; every iteration pays the
		// fold's record code)
		auto step = [&]() -> uint32_t {
			gen_step<MODE>(src, act, wk.w, g, info);
			return src.step(wk.w.id);
		};
		if constexpr (CR) {
			// one exit, at the bottom: the exits of a loop that tests at the
			// top merge into one latch, where the compiler copied 13 walk
			// state registers per step (C4 -1.3 %; the 16-byte form's
			// walkers spill this way: 1.73 against 1.70 ms)
			if (ready(src.step(wk.w.id))) {
				do {
				} while (ready(step()));
			}
		} else {
			for (uint32_t inf = src.step(wk.w.id); ready(inf);)
				inf = step();
		}
		wave_sync_lds();
		const bool fin = wk.have && wk.w.id == 0;
		emit_general<MODE, CR, RING>(sh, rs, fin, wk.w, wk.i, caplen, g, rec, pq, fc, lane);
		wk.have = wk.have && !fin;
		wk.stage = susp;
		if (!drain && !more)
			break;   // every walker is done or suspended: the next tile
	}
}

template <bool CR>
__device__ __forceinline__ void take(Shared &sh, Walker &wk, bool &pnd, const WalkOut &pw, uint32_t pi, uint64_t pd,
				     int lane, int wv)
{
	const uint64_t P = __ballot(pnd), F = __ballot(!wk.have);
	if (!P || !F)
		return;
	const uint32_t rp = lanes_below(P), rf = lanes_below(F);
	const uint32_t np = (uint32_t)__popcll(P), nf = (uint32_t)__popcll(F);
	if (pnd && rp < nf)
		sh.tmap[wv][rp] = (uint8_t)lane;
	wave_sync_lds();
	const bool get = !wk.have && rf < np;
	const int src = get ? (int)sh.tmap[wv][rf] : lane;
	const uint32_t x0 = __shfl(pi, src, 64);
	const uint32_t x1 = __shfl((uint32_t)pd, src, 64);
	const uint32_t x2 = __shfl((uint32_t)(pd >> 32), src, 64);
	const uint32_t x3 = __shfl(pw.data | pw.tail << 16, src, 64);
	// (a deferred chain has at most 4 layers: Ethernet, 2 tags, IP)
	const uint32_t x4 = __shfl((uint32_t)pw.ip_csum | (uint32_t)pw.flags << 16 | pw.n << 24 | (uint32_t)pw.id << 27,
				   src, 64);
	const uint32_t x5 = __shfl(pw.chain, src, 64);
	uint32_t x6 = 0, x7 = 0, x8 = 0;
	if (!CR) {
		x6 = __shfl((uint32_t)pw.offA, src, 64);
		x7 = __shfl((uint32_t)(pw.offA >> 32), src, 64);
		x8 = __shfl(pw.offB, src, 64);
	}
	if (get) {
		wk.i = x0;
		wk.d = x1 | (uint64_t)x2 << 32;
		walk_init(wk.w, x3 >> 16, (int)(x4 >> 27));
		wk.w.data = x3 & 0xFFFF;
		wk.w.ip_csum = (uint16_t)x4;
		wk.w.flags = (uint8_t)(x4 >> 16);
		wk.w.n = (x4 >> 24) & 7;
		wk.w.chain = x5;
		if (!CR) {
			wk.w.offA = x6 | (uint64_t)x7 << 32;
			wk.w.offB = x8;
		}
	}
	wk.have = wk.have || get;
	wk.stage = wk.stage || get;
	pnd = pnd && rp >= nf;
}

// plain_walk maps protocols 6 / 17 without the eth_lay3
// lookup fast_walk makes: the table must agree
constexpr uint8_t k_plain_lay3[256] = NSD_LAY3_TABLE;

// ---- pending ICMPv4 checksums -------------------------------------------------
// Runs after both passes (the records are final): the block's waves take its
// lists in 64-entry pieces and patch the flags byte of the records whose sum
// is bad.  Eight lanes per message, 8 messages per wave at a time: lane
// `sub` of a group sums the interior chunks 1 + sub + 8t (whole 16-byte
// loads, no masking; each group instruction reads 128 contiguous bytes, a
// line, where four lanes read half a line per instruction: C3 -1.6 %), U of
// them in flight per lane; sub-lanes 0 and 1 also take the message's first
// and last chunk with the bytes outside the message masked.  A message then
// costs a few wave instructions per KiB instead of one wave per message.
template <int U, bool CR, int L = NSD_CSUM_LANES>
__device__ __forceinline__ void icmp_pass(Shared &sh, const uint8_t *__restrict__ frames,
					  const uint64_t *__restrict__ desc, void *__restrict__ rec,
					  const uint64_t *__restrict__ pend, uint32_t region)
{
	const int lane = threadIdx.x & 63;
	const int wv = threadIdx.x >> 6;
	static_assert(L == 4 || L == 8 || L == 16, "lanes per message");
	const uint32_t sub = lane & (L - 1), grp = lane / L;
	uint32_t bad = 0;
	for (int l = 0; l < WAVES; l++) {
		const uint32_t cnt = sh.pcnt[l];
		const uint64_t *list = pend + ((size_t)blockIdx.x * WAVES + l) * (region / WAVES);
		// the block's waves split each list in 64-entry pieces
		for (uint32_t k0 = 64 * ((wv + l) % WAVES); k0 < cnt; k0 += 64 * WAVES) {
			const bool on = k0 + lane < cnt;
			const uint64_t e = on ? list[k0 + lane] : 0;
			const uint32_t i = (uint32_t)e;
			const uint32_t moff = (uint32_t)(e >> 32) & 0xFFFF, mlen = (uint32_t)(e >> 48);
			const uint64_t a = (on ? NSD_DESC_OFF(desc[i]) : 0) + moff;
			const uint32_t nb = on ? (mlen & ~1u) : 0u;
			for (uint32_t q = 0; q < 64 && k0 + q < cnt; q += 64 / L) {
				const int src = (int)(q + grp);
				const uint32_t alo = __shfl((uint32_t)a, src, 64);
				const uint32_t ahi = __shfl((uint32_t)(a >> 32), src, 64);
				const uint32_t mnb = __shfl(nb, src, 64);
				const bool mon = k0 + (uint32_t)src < cnt;
				const uint32_t s0 = alo & 15, endb = s0 + mnb;
				const uint32_t nch = mon ? (endb + 15) >> 4 : 0u;
				const uint4 *base = (const uint4 *)(frames + ((((uint64_t)ahi << 32) | alo) & ~15ull));
				// edge chunks, masked: chunk 0 on sub-lane 0, chunk nch-1 on sub-lane 1
				uint32_t sum = 0;
				const uint32_t je = sub == 0 ? 0u : nch - 1;
				if ((sub == 0 && nch > 0) || (sub == 1 && nch > 1))
					sum = csum_chunk(base[je], 16 * je, s0, endb);
				// interior chunks [1, nch - 1)
				for (uint32_t j = 1 + sub; __ballot(j + 1 < nch); j += L * U) {
					uint4 v[U];
#pragma unroll
					for (int u = 0; u < U; u++) {
						const uint32_t jj = j + L * u;
						v[u] = jj + 1 < nch ? base[jj] : make_uint4(0, 0, 0, 0);
					}
#pragma unroll
					for (int u = 0; u < U; u++) {
						sum = sum_halves(v[u].x, sum);
						sum = sum_halves(v[u].y, sum);
						sum = sum_halves(v[u].z, sum);
						sum = sum_halves(v[u].w, sum);
					}
				}
				sum = (sum >> 16) + (sum & 0xffff);   // folding keeps the zero test
#pragma unroll
				for (int x = 1; x < L; x <<= 1)
					sum += __shfl_xor(sum, x, 64);
				const uint32_t mi = __shfl(i, src, 64);
				const bool isbad = mon && sub == 0 && csum_final(sum) != 0;
				if (isbad) {
					uint8_t *nf = (uint8_t *)rec + nflags_at<CR>(mi);
					*nf = *nf | NSD_F_ICMP_BAD;
				}
				bad += FlagCnt::pc(isbad);
			}
		}
	}
	if (lane == 0 && bad)
		atomicAdd(&sh.cnt[NSD_CNT_ICMP_BAD], (unsigned long long)bad);
}

// ---- the walk ------------------------------------------------------------------
// Every packet of the block's grid-stride tiles, one wave per 64-packet tile:
// the fast walk over each packet's first 64 bytes, then the general walk's
// walkers take the packets it could not finish (walkers); ICMPv4 messages
// past the windows and host-rendered leaves go to the wave's pending list
// (pq).
// A wave's issue priority (s_setprio) from its progress: level 0 (the first
// quarter of its tiles) issues first, level 3 last.  The SIMD arbiter
// otherwise favours the oldest waves, and a CU's blocks arrive in rounds of
// one block per CU: with 4 blocks per CU the first round finished its tiles
// 20 % ahead of the fourth (C4: 835 against 1031 us; C3: 305 against 422),
// whose waves then ran the launch's tail with the CU a quarter full.
// (Priority by round alone only swapped which round lagged.)  Since the
// group tiles balance a CU's blocks, it still gives C3 0.7 % but costs
// walker-heavy batches 1 % (C4): the launcher turns it off for those
// (`prio`, from the schedule sample).
__device__ __forceinline__ void prio_level(uint32_t lvl)
{
	if (lvl == 0)
		__builtin_amdgcn_s_setprio(3);
	else if (lvl == 1)
		__builtin_amdgcn_s_setprio(2);
	else if (lvl == 2)
		__builtin_amdgcn_s_setprio(1);
	else
		__builtin_amdgcn_s_setprio(0);
}

template <int MODE, bool CR, bool RING>
__device__ __forceinline__ void walk_tiles(Shared &sh, const uint8_t *__restrict__ frames,
					   const uint64_t *__restrict__ desc, uint32_t n, int start_id,
					   void *__restrict__ rec, uint32_t *__restrict__ ext, uint32_t ext_words,
					   uint32_t *__restrict__ ext_used, uint32_t chunk,
					   const uint32_t *__restrict__ sll, Pending &pq,
					   unsigned long long *__restrict__ sched, uint32_t *__restrict__ gtiles,
					   uint32_t prio)
{
	constexpr int ROW = row_of(WIN1);
	auto &s_win = sh.win;
	unsigned long long *const s_cnt = sh.cnt;
	const uint8_t *const s_lay3 = sh.lay3;
	const int lane = threadIdx.x & 63;
	const int wv = threadIdx.x >> 6;

	const uint32_t stride = gridDim.x * BLOCK;
	uint64_t *const wq = pq.wq;
	// compact records: pool words [0, n) are the packets' side words (when the
	// pool has them), entries come after
	const bool side = CR && ext_words >= n;
	const GenSink<CR> g{ ext, ext_words, ext_used, chunk, &sh.wc[wv][0], sh.ops, &sh.lay[wv][0],
			 side ? n : 0u, side ? ext : nullptr };
	FlagCnt fc;
	uint32_t ndefer = 0;
	uint32_t base = blockIdx.x * BLOCK + wv * 64;   // this wave's tile; whole waves iterate

	if (MODE != PRINT_NORM && MODE != PRINT_LESS) {
		// every process() is NULL: no chain (dissector.c:51-53)
		for (; base < n; base += stride) {
			const uint32_t i = base + lane;
			fc.pkts += FlagCnt::pc(i < n);
			if (i < n) {
				const uint32_t caplen = NSD_DESC_CAPLEN(desc[i]);
				if constexpr (CR)
					__builtin_nontemporal_store(v2u{ 0u, 0u }, (v2u *)rec + i);
				else
					store_rec((uint4 *)rec, i, make_uint4(0, caplen << 16, 0, 0));
				fc.bytes += caplen;
			}
		}
		fc.flush(s_cnt, lane);
		return;
	}

	// Tiles of a CU group.  A launch of 4 blocks per CU places blocks b,
	// b + G, b + 2G, b + 3G (G = grid / 4) on one CU, and the SIMD arbiter
	// runs the first-placed block's waves ahead of the later ones (C4: the
	// rounds ended their tiles at 835 / 881 / 945 / 1031 us).  So the group's
	// 16 waves share its grid-stride tiles: the group's j-th tile is row
	// j / 16 of the grid stride, block b + ((j / 4) % 4) G, wave j % 4 (the
	// static order, so the waves still sweep the batch front to back, and
	// tile numbers grow with j), and a wave takes the next j from the
	// group's counter (a line of its own in the workspace, zeroed before
	// each launch by zero_tiles; one counter for the whole grid serialised
	// its atomics: 2.3x slower).
	// The atomic for tile t+2 is issued a tile ahead and its return read then
	// (hipcc's atomic optimizer would wait for it at once: the offset it
	// cannot prove uniform).  A wave asks only while its pending list has
	// room for an entry from every packet of the tiles it holds, the new one
	// and its walkers: the lists hold twice a wave's even share plus four
	// tiles (region_for_fused), so a group's waves cannot all stop for room
	// while its tiles are left.  Grids that are not 4 blocks per CU share
	// per block.  Compact records only (the 16-byte form's walk state leaves
	// no registers for it: 12 VGPRs spilled).
	constexpr bool DYN = NSD_GROUP_TILES && CR;
	const uint32_t ntiles = (n + 63) / 64;
	const uint32_t nw = gridDim.x * WAVES;
	const bool grp4 = gridDim.x % NSD_GROUP_BLOCKS == 0;
	const uint32_t G = grp4 ? gridDim.x / NSD_GROUP_BLOCKS : gridDim.x, R = grp4 ? NSD_GROUP_BLOCKS : 1u;
	const uint32_t grp = blockIdx.x % G;
	uint32_t *const gctr = gtiles + 32 * grp;
	auto tile_of = [&](uint32_t j) -> uint32_t {   // the group's j-th tile's first packet (n: none)
		const uint32_t k = j / (4 * R), r = (j / 4) % R, w = j % 4;
		const uint64_t t = (uint64_t)k * nw + (grp + r * G) * 4 + w;
		return t < ntiles ? (uint32_t)t * 64 : n;
	};
	uint32_t gv = 0;
	bool asked = false;
	auto ask = [&](uint32_t held) {
		const uint32_t used = pq.npend + pq.nleaf;
		asked = used + 64u * (held + 2) <= pq.wcap;
		if (asked && lane == 0) {
			uint32_t z;
			asm volatile("v_mov_b32 %0, 0" : "=v"(z));
			gv = atomicAdd(gctr + z, 1u);
		}
	};
	auto take = [&]() -> uint32_t {   // the asked tile (n: none)
		if (!asked)
			return n;
		asked = false;
		return tile_of((uint32_t)__builtin_amdgcn_readfirstlane((int)gv));
	};
	uint32_t nb1 = n, nb2 = n;
	if constexpr (DYN) {
		ask(0);
		base = take();
		if (base < n) {
			ask(1);
			nb1 = take();
			if (nb1 < n)
				ask(2);   // for tile t+2, read when tile t is walked
		}
	} else {
		nb1 = base + stride < n ? base + stride : n;
	}
	// software pipeline: tile t walked while tile t+1's chunks and tile t+2's
	// descriptors are in flight
	if (base >= n)
		return;
	uint64_t d0 = (base + lane < n) ? desc[base + lane] : 0;
	uint64_t d1 = (nb1 < n && nb1 + lane < n) ? desc[nb1 + lane] : 0;
	Chunks<WIN1> ch;
	stage_load<WIN1>(ch, frames, d0, lane);
	Walker wk;
	walk_init(wk.w, 0, 0);
	wk.d = 0;
	wk.i = 0;
	wk.wb = 0;
	wk.wl = 0;
	wk.have = false;
	wk.stage = false;

	// late: the next tile's chunks load after this tile's walkers (this tile's
	// predecessor was walker-heavy: NSD_LATE, below)
	bool late = false;
	HeldSt<CR> hs;   // the previous tile's record / pending-list stores
	hs.ri = hs.pp = 0xFFFFFFFFu;
	// compact records: the wave's record ring (RecRing), slot rs for the
	// next tile
	constexpr bool RG = CR && RING;
	RingSt rs;
	rs.init();
	// (one more pass after the last tile drains the walkers: the engine is
	// inlined once)
	// this wave's even share of tiles and the ones walked, for prio_level
	const uint32_t share = (ntiles + nw - 1) / nw;
	uint32_t done = 0, lvl = 0xFFu;
	for (;;) {
		if (NSD_PRIO && CR && prio) {   // (the 16-byte form's walk state leaves no registers for it)
			const uint32_t l = done < share ? 4u * done / share : 3u;
			if (l != lvl) {
				lvl = l;
				prio_level(l);
			}
			done++;
		}
		const bool last = base >= n;
		const uint32_t i = base + lane;
		const bool valid = i < n;
		const uint64_t off = NSD_DESC_OFF(d0);
		const uint32_t caplen = NSD_DESC_CAPLEN(d0);
		WalkOut w;
		walk_init(w, caplen, valid ? start_id : 0);
		bool deferred = false;
		uint64_t d2 = 0;
		if (!last) {
			stage_write(&s_win[wv][0], ch, lane);
			hs.flush(rec, wq);   // tile t-1's stores, before tile t+1's loads
			if (RG)
				ring_turn(sh, rs, wk, rec, g.side, n, lane);
			// prefetch: descriptors of tile t+2, chunks of tile t+1
			if constexpr (DYN) {
				nb2 = take();
				if (nb2 < n)
					ask(3);   // tiles t .. t+2 held
			}
			const uint32_t b2 = DYN ? nb2 : base + 2 * stride;
			d2 = (b2 < n && b2 + lane < n) ? desc[b2 + lane] : 0;
			const uint32_t b1 = DYN ? nb1 : base + stride;
			if (b1 < n && !late)
				stage_load<WIN1>(ch, frames, d1, lane);
			wave_sync_lds();

			uint32_t fw = FW_DONE;
			const LSrc<true, WIN1> src{ &s_win[wv][lane * ROW], s_lay3, nullptr, frames + off, caplen,
						    (uint32_t)off & 15, 0, false };
			if (valid)
				fw = fast_walk<MODE, false, NSD_FAST_EXT != 0>(src, caplen, w);
			deferred = fw != FW_DONE;
			ndefer += FlagCnt::pc(deferred);
			wave_sync_lds();
			const bool done = valid && !deferred;
			if (MODE == PRINT_NORM) {
				// ICMPv4 messages past the window: listed for the checksum pass, which
				// patches the record if the sum is bad
				const bool pnd = w.icmp_pend && done;
				const uint64_t pmask = __ballot(pnd);
				hs.hold_pend(wq, pend_entry(i, w.icmp_off, w.icmp_len),
					     pnd ? pq.npend + lanes_below(pmask) : 0xFFFFFFFFu);
				pq.npend += (uint32_t)__popcll(pmask);
			}
			// per-ops counts from the finished chains, grouped by chain word
			// (ids are >= 1, so equal chain words imply equal layer counts) for
			// the first two distinct chains of the tile (C2: one), the rest per
			// lane (C3: -4.5 % against looping over every distinct chain)
			{
				uint32_t key = done ? w.chain : 0xFFFFFFFFu;
				for (int it = 0;; it++) {
					const uint64_t pm = __ballot(key != 0xFFFFFFFFu);
					if (!pm)
						break;
					if (it == 2) {
						// more than two distinct chains in the tile: the rest
						// count their own layers (the LDS serialises them)
						if (key != 0xFFFFFFFFu)
							for (uint32_t k = 0; k < w.n; k++)
								atomicAdd(&sh.ops[(key >> (5 * k)) & 31], 1u);
						break;
					}
					const int leader = __ffsll((unsigned long long)pm) - 1;
					const uint32_t lk = __shfl(key, leader, 64);
					const uint64_t m = __ballot(key == lk);
					if (lane == leader) {
						const uint32_t cnt = (uint32_t)__popcll(m);
						for (uint32_t k = 0, nl = w.n; k < nl; k++)
							atomicAdd(&sh.ops[(lk >> (5 * k)) & 31], cnt);
					}
					if (key == lk)
						key = 0xFFFFFFFFu;
				}
			}
			// a leaf the fast walk finished (ARP, DCCP): its end in the side word
			const bool lend = CR && g.side && done && (w.flags & NSD_F_HOST);
			if (lend)
				w.flags |= NSD_F_LEAF_END;
			const uint32_t nd = (uint32_t)__popcll(__ballot(deferred));
			if (RG && nd) {
				ring_open(sh, rs, base, nd, done, crec_of(w), lend ? w.data : 0u, lane);
			} else if (CR && !RG) {
				if (lend)
					g.side[i] = w.data;
				hs.hold_rec(i, crec_of(w), done);
			} else {
				if (lend)
					g.side[i] = w.data;
				if (done)
					put_rec<CR>(rec, i, w);
			}
			fc.add(w, caplen, done);
			// the deferred packets' walk state for the general walk: from the
			// start (FW_RESTART: other link types, MPLS, deeper tag stacks, bytes
			// past the first window) or from where the fast walk stopped
			// (FW_RESUME: its layers recorded; its finished chains are counted by
			// chain word, these are counted here)
			if (deferred) {
				if (fw == FW_RESTART) {
					walk_init(w, caplen, start_id);
					if (start_id == NSD_OPS_SLL)
						sll_head<MODE>(sh, w, sll, i);
				} else {
					for (uint32_t k = 0; k < w.n; k++)
						atomicAdd(&sh.ops[(w.chain >> (5 * k)) & 31], 1u);
				}
			}
		}
		// (the walkers carried over are suspended: their windows are
		// restaged anyway, so this tile's staging may reuse their rows)
		bool pnd = deferred;
		const bool many = __popcll(__ballot(pnd)) >= NSD_L2PF;
		if (__ballot(pnd || wk.have)) {
			// (the walkers wait for their windows anyway: the held stores go
			// first, and nothing is held across the engine's registers)
			hs.flush(rec, wq);
			walkers<MODE, CR, RG>(sh, rs, frames, rec, g, pq, fc, wk, pnd, w, i, d0, last);
		}
		if (last) {
			hs.flush(rec, wq);
			if (RG)
				ring_turn(sh, rs, wk, rec, g.side, n, lane);   // every walker is done: the ring's last tiles
			break;
		}
		// After a walker-heavy tile (C4) the next tile's chunks load here, with
		// L2-allocating loads, rather than a tile ahead: its walkers' first
		// windows then find the packets' first lines in L2 (loaded a tile
		// ahead, those lines had left L2 by the time the walkers staged them:
		// C4 400 -> 349 B/packet, 1.152 -> 1.107 ms on one box).  The chunk
		// registers are dead during the walkers either way.
		if (late && (DYN ? nb1 : base + stride) < n)
			stage_load<WIN1, false, false>(ch, frames, d1, lane);
		// (NSD_LATE 0: the chunks load a tile ahead, and while the walkers are
		// busy the lines of tile t+2 go into L2 now, so the next iteration's
		// loads of them wait for L2 rather than HBM: C4 1.45 -> 1.32 ms then.
		// Not for tiles the fast walk finishes (C2, C3): there the next loads
		// would wait for the touches (vector memory counts in order; C2
		// +12 %).  The LDS-DMA target is window words past the fast rows.)
		{
			const uint32_t b2 = DYN ? nb2 : base + 2 * stride;
			if (!NSD_LATE && many && b2 < n)
				l2_touch(frames, d2, &s_win[wv][64 * ROW], b2 + lane < n);
		}
		late = NSD_LATE && many;
		d0 = d1;
		d1 = d2;
		if constexpr (DYN) {
			base = nb1;
			nb1 = nb2;
			nb2 = n;
		} else {
			base += stride;
		}
	}
	if (NSD_PRIO && CR && prio)
		__builtin_amdgcn_s_setprio(0);   // the leaf and checksum passes at the neutral level
	fc.flush(s_cnt, lane);
	// the pending list held every entry (ask()'s room rule: a packet adds at
	// most one, ICMPv4 from the front or leaf from the back, and the lists
	// hold two shares plus four tiles); a broken invariant overwrote the next
	// wave's list: counted, and the counters then differ from any oracle's
	if (lane == 0 && pq.npend + pq.nleaf > pq.wcap)
		atomicAdd(&s_cnt[NSD_CNT_LISTOVF], 1ull);
	// the schedule sample (a launch the launcher samples passes its pair)
	if (sched && lane == 0 && ndefer)
		atomicAdd(&sched[0], (unsigned long long)ndefer);
	if (sched && lane == 0 && pq.npend)
		atomicAdd(&sched[1], (unsigned long long)pq.npend);
}

// ---- host-rendered leaves -------------------------------------------------------
// The leaves the wave's general walk ended in (ARP / LLDP / IGMP / DCCP /
// ICMPv6 130-154; ARP and DCCP inside the fast window finish in fast_walk):
// one lane per entry walks the leaf parser's pulls over the frame in HBM
// (nsd_leaf.h) and rewrites the record's cursor word.  A pass of its own,
// after the tiles, so the LLDP TLV and ND-option loops do not add to the
// walk's register peak.  The wave reads back only what it wrote itself.
template <int MODE, bool CR>
__device__ __forceinline__ void leaf_pass(const uint8_t *__restrict__ frames, const uint64_t *__restrict__ desc,
					  void *__restrict__ rec, uint32_t *__restrict__ pool, const Pending &pq)
{
	if (!pq.nleaf)
		return;
	__threadfence();   // the wave's record and list stores complete before its loads below
	for (uint32_t k = threadIdx.x & 63; k < pq.nleaf; k += 64) {
		const uint64_t e = pq.wq[pq.wcap - 1 - k];
		const uint32_t i = (uint32_t)e, start = (uint32_t)(e >> 32) & 0xFFFF;
		const uint64_t d = desc[i];
		const HbmBytes src{ frames + NSD_DESC_OFF(d), NSD_DESC_CAPLEN(d) };
		if constexpr (!CR) {
			const int id = (int)(e >> 48);
			uint32_t *const y = (uint32_t *)((uint4 *)rec + i) + 1;   // data_off | tail_off << 16
			const uint32_t tail = __hip_atomic_load(y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 16;
			*y = leaf_end<MODE>(src, id, start, tail) | tail << 16;
		} else {
			// the leaf is the chain's last layer: its id from the record (inline
			// ids) or the entry (ids only); its end into the side word or entry
			const uint32_t tail = (uint32_t)(e >> 48);
			const uint64_t rv = __hip_atomic_load((uint64_t *)rec + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			const uint2 r = make_uint2((uint32_t)rv, (uint32_t)(rv >> 32));
			const uint32_t nf = (r.y >> 16) & 0xFF, n = nf & 7;
			uint32_t *loc;
			int id;
			if (n != NSD_N_EXT) {
				id = (int)((r.x >> (5 * (n - 1))) & 31);
				loc = pool + i;
			} else {
				const uint32_t nl = __hip_atomic_load(pool + r.x + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xFFFF;
				id = (int)(__hip_atomic_load(pool + r.x + NSD_EXT_HDR_WORDS + nl - 1, __ATOMIC_RELAXED,
							     __HIP_MEMORY_SCOPE_AGENT) & 31);
				loc = pool + r.x + 2;
			}
			*loc = leaf_end<MODE>(src, id, start, tail);
		}
	}
}

// One launch per batch.  Each block of the persistent grid walks its
// grid-stride tiles (fast walk + continuations), walks the leaves its waves
// left pending, then sums the ICMPv4 messages they left pending; a later
// phase reads only what the same block wrote (its pending lists), so the
// phases need a block barrier, not a grid-wide one.
// the fused launch's group tile counters (walk_tiles): word 0 of each
// 128-byte line.  A kernel rather than hipMemsetAsync: with the memset
// captured into a HIP graph the counters held garbage from the second
// replay on (tools/dbg_graph.py), so no tile was walked.
__global__ void zero_tiles(uint32_t *__restrict__ gtiles, uint32_t groups)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < groups)
		gtiles[32 * i] = 0;
}

template <int MODE, bool CR, bool RING = false>
__global__ __launch_bounds__(BLOCK, NSD_MINW) void dissect_all(
	const uint8_t *__restrict__ frames, const uint64_t *__restrict__ desc, uint32_t n, int start_id,
	void *__restrict__ rec, uint32_t *__restrict__ ext, uint32_t ext_words,
	uint32_t *__restrict__ ext_used, uint32_t chunk, unsigned long long *__restrict__ counters,
	uint64_t *__restrict__ pend, uint32_t region, const uint32_t *__restrict__ sll,
	unsigned long long *__restrict__ sched, uint32_t *__restrict__ gtiles, uint32_t prio)
{
	__shared__ Shared sh;
	if (threadIdx.x < 64)
		sh.step[threadIdx.x] = threadIdx.x < 32 ? c_step[threadIdx.x] : c_lay2h.e[threadIdx.x - 32];
	if (threadIdx.x < 32)
		sh.ops[threadIdx.x] = 0;
	if (threadIdx.x < 2 * WAVES)
		sh.wc[threadIdx.x >> 1][threadIdx.x & 1] = 0;
	block_init(sh.cnt, sh.lay3);   // (its barrier orders the stores above too)

	// this wave's pending list (a wave visits region / WAVES packets)
	Pending pq{ pend + ((size_t)blockIdx.x * WAVES + (threadIdx.x >> 6)) * (region / WAVES), region / WAVES, 0,
		    0 };
	walk_tiles<MODE, CR, RING>(sh, frames, desc, n, start_id, rec, ext, ext_words, ext_used, chunk, sll, pq,
				   sched, gtiles, prio);
	if (MODE == PRINT_NORM || MODE == PRINT_LESS)
		leaf_pass<MODE, CR>(frames, desc, rec, ext, pq);
	if ((threadIdx.x & 63) == 0)
		sh.pcnt[threadIdx.x >> 6] = pq.npend;
	if (MODE == PRINT_NORM) {
		__syncthreads();   // records final, pending lists and counts complete
		icmp_pass<NSD_CSUM_U, CR>(sh, frames, desc, rec, pend, region);
	}
	block_flush(sh.cnt, counters);
	if (threadIdx.x < 32 && sh.ops[threadIdx.x])
		atomicAdd(&counters[NSD_CNT_OPS + threadIdx.x], (unsigned long long)sh.ops[threadIdx.x]);
}


// ==== the split schedule ===========================================================
// Two launches per batch.  dissect_fast runs the fast walk of every tile at
// high occupancy (8 waves per SIMD: its registers and LDS are only what the
// fast walk needs), writes the records of the packets it finishes, sums the
// ICMPv4 messages they leave pending and appends every packet it cannot
// finish to its wave's deferral list; dissect_walk runs the walker pool
// (walkers(), the general walk) over those lists.  The fused kernel's
// register peak is the walker pool's (119 VGPRs: 4 waves per SIMD), which
// C2 and C3 - nearly nothing deferred - paid for in latency hiding.
//
// A fast wave's list (`cap` slots of 32 bytes):
//   deferrals from the front: { packet, data | tail << 16,
//     ip_csum | flags << 16 | n << 24 | id << 27, chain },
//     { descriptor, starts of layers 1..4 (a byte each: the fast window) }
//   pending ICMPv4 checksums from the back: { packet, off | len << 16,
//     the message's words before off, summed and weighted like the pass
//     (below) }, { descriptor }
// and its counts at cnts[wave] = { deferrals, checksums }.  The descriptor
// rides along so the walker kernel and the checksum pass read no desc[]
// (and the walker kernel knows the next chunk's window addresses early).

constexpr int FROW = WIN1 / 4;   // fast rows: 16 dwords, 16-byte slots XOR-swizzled by swz_of(q, 4)
#ifndef NSD_FAST_MINW
#define NSD_FAST_MINW (NSD_FAST_DEPTH > 1 ? 4 : 6)   // waves per SIMD dissect_fast is register-allocated for (compact records)
#endif
#ifndef NSD_FAST_MINW_FULL
#define NSD_FAST_MINW_FULL (NSD_FAST_DEPTH > 1 ? 4 : 5)   // the same for 16-byte records (the deferral entries carry layer starts)
#endif
#ifndef NSD_PLAIN_COUNT
#define NSD_PLAIN_COUNT 1          // plain tiles count from three ballots (dissect_fast)
#endif
#ifndef NSD_FAST_BPC
#define NSD_FAST_BPC (NSD_FAST_DEPTH > 1 ? 3 : 0)   // resident fast blocks per CU (0: as many as fit)
#endif
#ifndef NSD_SPLIT_TAIL
#define NSD_SPLIT_TAIL 1           // the fast kernel's blocks walk their own deferrals (no walker launch)
#endif
#ifndef NSD_FAST_CSUM_U
#define NSD_FAST_CSUM_U 8        // interior chunk loads in flight per lane (fast_icmp_pass; 4: C3 split +4 %)
#endif

struct FastShared {
	alignas(16) uint32_t win[WAVES][64 * FROW];   // fast rows
	unsigned long long cnt[NSD_NCOUNTERS];        // block counters
	uint32_t ops[32];                             // block per-ops layer counts
	uint8_t lay3[256];                            // eth_lay3
	uint32_t pcnt[WAVES];                         // pending checksums per wave
};

// stage_write into the split schedule's rows: chunk c of packet q at slot
// c ^ swz(q) of its 16-dword row (ds_write_b128; the 8 lanes of a store
// group cover two whole rows: no bank conflict)
__device__ __forceinline__ void stage_write_sw(uint32_t *wwin, const Chunks<WIN1> &ch, int lane)
{
#pragma unroll
	for (int r = 0; r < 4; r++) {
		const int t = r * 64 + lane;
		const int q = t / 4, c = t % 4;
		const uint32_t nv = (ch.nv >> (8 * r)) & 0xFF;
		uint32_t w[4] = { ch.v[r].x, ch.v[r].y, ch.v[r].z, ch.v[r].w };
		if (nv < 16) {
#pragma unroll
			for (int j = 0; j < 4; j++) {
				const uint32_t bp = 4 * j;
				if (bp >= nv)
					w[j] = 0;
				else if (bp + 4 > nv)
					w[j] &= (1u << ((nv - bp) * 8)) - 1u;
			}
		}
		*(uint4 *)(wwin + q * FROW + ((c ^ swz_of((uint32_t)q, 4)) << 2)) = make_uint4(w[0], w[1], w[2], w[3]);
	}
}

// a folded 16-bit partial sum in the pass's byte weighting: the pass sums a
// message's bytes as aligned little-endian halves, which weights them by 256
// (mod 0xFFFF) against the reference's words when the message starts at an
// odd address (see the ICMPv4 checksum helpers above); so is the partial
__device__ __forceinline__ uint32_t fold_weighted(uint32_t sum, bool odd)
{
	sum = (sum >> 16) + (sum & 0xFFFF);
	sum = (sum >> 16) + (sum & 0xFFFF);
	return odd ? ((sum & 0xFF) << 8 | sum >> 8) : sum;
}

// The plain IPv4 chain (PRINT_NORM, split schedule): Ethernet (type 0x0800,
// no tag), IPv4 without options (first byte 0x45), then TCP or UDP, in a
// frame of at least 42 bytes.  For such a packet fast_walk (nsd_walk.h) reads
// bytes 12..33 and nothing past them, all inside the window, and ends with
// the chain Ethernet, IPv4, TCP / UDP at offsets 0 / 14 / 34 (proto_ethernet.c,
// proto_ipv4.c:34-204 incl. the total-length trim, proto_tcp.c / proto_udp.c).
// plain_is tells from bytes 12..23 whether the packet is one; plain_walk
// then reads bytes 12..35 (7 row dwords, byte funnel shifts) and gives
// fast_walk's result from them alone (re-read rather than kept: registers).
// A tile takes this path only when every valid lane's packet is plain
// (wave-uniform), so a mixed tile runs fast_walk alone.
// plain_is / plain_walk map protocol 6 / 17 to TCP / UDP without the eth_lay3
// lookup fast_walk makes: the table must agree
static_assert(k_plain_lay3[6] == NSD_OPS_TCP && k_plain_lay3[17] == NSD_OPS_UDP,
	      "plain_walk's protocol map differs from eth_lay3");

__device__ __forceinline__ bool plain_is(const LSrc<true, WIN1> &s, uint32_t caplen)
{
	const uint32_t r = s.m + 12, j = r >> 2, sh = r & 3;
	const uint32_t d12 = __builtin_amdgcn_alignbyte(s.dw(j + 1), s.dw(j), sh);
	const uint32_t d20 = __builtin_amdgcn_alignbyte(s.dw(j + 3), s.dw(j + 2), sh);
	const uint32_t proto = d20 >> 24;
	return caplen >= 42 && (d12 & 0xFFFFFFu) == 0x450008u && (proto == 6 || proto == 17);
}

__device__ __forceinline__ void plain_walk(const LSrc<true, WIN1> &s, uint32_t caplen, WalkOut &w)
{
	const uint32_t r = s.m + 12, j = r >> 2, sh = r & 3;   // j + 6 <= 12: inside the 16-dword row
	const uint32_t w0 = s.dw(j), w1 = s.dw(j + 1), w2 = s.dw(j + 2), w3 = s.dw(j + 3), w4 = s.dw(j + 4),
		       w5 = s.dw(j + 5), w6 = s.dw(j + 6);
	const uint32_t d12 = __builtin_amdgcn_alignbyte(w1, w0, sh), d16 = __builtin_amdgcn_alignbyte(w2, w1, sh),
		       d20 = __builtin_amdgcn_alignbyte(w3, w2, sh), d24 = __builtin_amdgcn_alignbyte(w4, w3, sh),
		       d28 = __builtin_amdgcn_alignbyte(w5, w4, sh), d32 = __builtin_amdgcn_alignbyte(w6, w5, sh);
	// calc_csum over the 10 header words at 14..32 (csum.h:12-27)
	uint32_t sum = (d12 >> 16) + (d32 & 0xFFFF);
	sum = __builtin_amdgcn_sad_u16(d16, 0u, sum);
	sum = __builtin_amdgcn_sad_u16(d20, 0u, sum);
	sum = __builtin_amdgcn_sad_u16(d24, 0u, sum);
	sum = __builtin_amdgcn_sad_u16(d28, 0u, sum);
	sum = (sum >> 16) + (sum & 0xffff);
	sum += sum >> 16;
	w.ip_csum = (uint16_t)~sum;
	// the total-length trim (ihl 5: no options)
	const int32_t x = (int32_t)__builtin_bswap16((uint16_t)d16) - 20;
	if (x >= 0 && (uint32_t)x < caplen - 34)
		w.tail = 34 + (uint32_t)x;
	const bool tcp = (d20 >> 24) == 6;
	const int l4 = tcp ? NSD_OPS_TCP : NSD_OPS_UDP;
	w.chain = NSD_OPS_ETHERNET | NSD_OPS_IPV4 << 5 | (uint32_t)l4 << 10;
	w.offA = (uint64_t)14 << 16 | (uint64_t)34 << 32;
	w.n = 3;
	const uint32_t len = w.tail - 34, hl = tcp ? 20u : 8u;
	w.data = len >= hl ? 34 + hl : 34;
}

template <int MODE, bool CR>
__device__ __forceinline__ void fast_tiles(FastShared &sh, const uint8_t *__restrict__ frames,
					   const uint64_t *__restrict__ desc, uint32_t n, int start_id,
					   void *__restrict__ rec, const uint32_t *__restrict__ sll, uint32_t *__restrict__ side,
					   uint4 *__restrict__ list, uint32_t cap, uint32_t &ndef, uint32_t &nicmp)
{
	constexpr int SW = 2;
	const int lane = threadIdx.x & 63;
	const int wv = threadIdx.x >> 6;
	const uint32_t stride = gridDim.x * BLOCK;
	FlagCnt fc;
	uint32_t base = blockIdx.x * BLOCK + wv * 64;

	if (MODE != PRINT_NORM && MODE != PRINT_LESS) {
		// every process() is NULL: no chain (dissector.c:51-53)
		for (; base < n; base += stride) {
			const uint32_t i = base + lane;
			fc.pkts += FlagCnt::pc(i < n);
			if (i < n) {
				const uint32_t caplen = NSD_DESC_CAPLEN(desc[i]);
				if constexpr (CR)
					__builtin_nontemporal_store(v2u{ 0u, 0u }, (v2u *)rec + i);
				else
					store_rec((uint4 *)rec, i, make_uint4(0, caplen << 16, 0, 0));
				fc.bytes += caplen;
			}
		}
		fc.flush(sh.cnt, lane);
		return;
	}
	if (base >= n)
		return;
	uint32_t *const rows = &sh.win[wv][0];
	// Descriptors (a lane past the batch: 0).  With a deeper prefetch they
	// are loaded unconditionally, from a clamped index (a load under a branch
	// leaves hipcc unsure whether it is pending, and it then waits vmcnt(0)
	// for the chunks, i.e. for every load in flight); a lane past the batch
	// then keeps the last packet's descriptor: it only stages that frame's
	// window, it walks nothing (valid is false) and counts nothing.
	// The product build runs depth 2 (inline-asm stores, 3 blocks per CU).
	auto dsc = [&](uint32_t b) -> uint64_t {
		if (NSD_FAST_DEPTH == 1)
			return b < n && b + lane < n ? desc[b + lane] : 0;
		return desc[b < n && b + lane < n ? b + lane : n - 1];
	};
	// One tile at `base` whose chunks are in `ch` (descriptors d0): write them
	// to the rows, reuse `ch` for the chunks of the tile NSD_FAST_DEPTH
	// strides on (descriptors dpre), walk the tile.
	auto tile = [&](Chunks<WIN1> &ch, const uint64_t d0, const uint64_t dpre) {
		const uint32_t i = base + lane;
		const bool valid = i < n;
		const uint64_t off = NSD_DESC_OFF(d0);
		const uint32_t caplen = NSD_DESC_CAPLEN(d0);
		WalkOut w;
		walk_init(w, caplen, valid ? start_id : 0);
		stage_write_sw(rows, ch, lane);
		// (deeper prefetch: issued past the batch's last tile too, from the
		// clamped descriptor - loads skipped on some paths also make hipcc
		// wait vmcnt(0))
		if (NSD_FAST_DEPTH == 1) {
			if (base + stride < n)
				stage_load<WIN1>(ch, frames, dpre, lane);
		} else {
			stage_load<WIN1, true>(ch, frames, dpre, lane);
		}
		wave_sync_lds();
		uint32_t fw = FW_DONE;
		const LSrc<true, WIN1> src{ rows + lane * FROW, sh.lay3, nullptr, frames + off, caplen,
					    (uint32_t)off & 15, 0, false, swz_of((uint32_t)lane, 4) << 2 };
		// (every lane's row is staged, a lane past the batch from the clamped descriptor)
		const bool plain = MODE == PRINT_NORM && start_id == NSD_OPS_ETHERNET &&
				   __ballot(valid && !plain_is(src, caplen)) == 0;
		if (plain) {
			if (valid)
				plain_walk(src, caplen, w);
		} else if (valid) {
			fw = fast_walk<MODE, true>(src, caplen, w);
		}
		const bool deferred = fw != FW_DONE;
		wave_sync_lds();
		const bool done = valid && !deferred;
		if (NSD_PLAIN_COUNT && plain) {
			// a plain tile (Ethernet / IPv4 / TCP or UDP, every packet done, no
			// ICMPv4, no leaf, no deferral): its counts straight from three
			// ballots - packets, bad IPv4 sums, trims - and the TCP share
			const uint64_t vm = __ballot(valid), tm = __ballot(valid && w.chain >> 10 == NSD_OPS_TCP);
			const uint32_t nv = (uint32_t)__popcll(vm), nt = (uint32_t)__popcll(tm);
			if (lane == 0) {
				atomicAdd(&sh.ops[NSD_OPS_ETHERNET], nv);
				atomicAdd(&sh.ops[NSD_OPS_IPV4], nv);
				if (nt)
					atomicAdd(&sh.ops[NSD_OPS_TCP], nt);
				if (nv - nt)
					atomicAdd(&sh.ops[NSD_OPS_UDP], nv - nt);
			}
			if (valid)
				put_rec_st<CR>(rec, i, w);
			fc.pkts += nv;
			fc.ipbad += FlagCnt::pc(valid && w.ip_csum != 0);
			fc.trim += FlagCnt::pc(valid && w.tail < caplen);
			if (valid)
				fc.bytes += caplen;
			return;
		}
		if (MODE == PRINT_NORM) {
			// ICMPv4 messages past the window, from the back of the list
			const bool pnd = w.icmp_pend && done;
			const uint64_t pm = __ballot(pnd);
			if (pnd) {
				const uint32_t part = fold_weighted(w.icmp_sum, ((uint32_t)off + w.icmp_off) & 1);
				uint4 *e = list + (size_t)(cap - 1 - (nicmp + lanes_below(pm))) * SW;
				st_b128(e, make_uint4(i, w.icmp_off | w.icmp_len << 16, part, 0));
				st_b128(e + 1, make_uint4((uint32_t)d0, (uint32_t)(d0 >> 32), 0, 0));
			}
			nicmp += (uint32_t)__popcll(pm);
		}
		// per-ops counts of the finished chains, grouped by chain word (as
		// walk_tiles)
		{
			uint32_t key = done ? w.chain : 0xFFFFFFFFu;
			for (int it = 0;; it++) {
				const uint64_t pm = __ballot(key != 0xFFFFFFFFu);
				if (!pm)
					break;
				if (it == 2) {
					if (key != 0xFFFFFFFFu)
						for (uint32_t k = 0; k < w.n; k++)
							atomicAdd(&sh.ops[(key >> (5 * k)) & 31], 1u);
					break;
				}
				const int leader = __ffsll((unsigned long long)pm) - 1;
				const uint32_t lk = __shfl(key, leader, 64);
				const uint64_t m = __ballot(key == lk);
				if (lane == leader) {
					const uint32_t cnt = (uint32_t)__popcll(m);
					for (uint32_t k = 0, nl = w.n; k < nl; k++)
						atomicAdd(&sh.ops[(lk >> (5 * k)) & 31], cnt);
				}
				if (key == lk)
					key = 0xFFFFFFFFu;
			}
		}
		if (CR && side && done && (w.flags & NSD_F_HOST)) {
			// a leaf the fast walk finished (ARP, DCCP): its end in the side word
			st_b32(side + i, w.data);
			w.flags |= NSD_F_LEAF_END;
		}
		if (done)
			put_rec_st<CR>(rec, i, w);
		fc.add(w, caplen, done);
		// the deferred packets' walk state, for dissect_walk: from the start
		// (FW_RESTART; the SLL head is run here) or where the fast walk stopped
		// (FW_RESUME: its layers are counted here)
		const uint64_t dm = __ballot(deferred);
		if (dm) {
			if (deferred) {
				if (fw == FW_RESTART) {
					walk_init(w, caplen, start_id);
					if (start_id == NSD_OPS_SLL) {
						const uint32_t w0 = sll ? sll[5 * (size_t)i] : 0u;
						const uint32_t w2 = sll ? sll[5 * (size_t)i + 2] : 0u;
						const uint32_t proto = __builtin_bswap16((uint16_t)(w0 >> 16));
						w.chain = NSD_OPS_SLL;
						w.n = 1;
						atomicAdd(&sh.ops[NSD_OPS_SLL], 1u);
						w.id = sll_next(w2 & 0xFFFF, proto, MODE, c_lay2h.e[NSD_L2H(proto)]);
					}
				} else {
					for (uint32_t k = 0; k < w.n; k++)
						atomicAdd(&sh.ops[(w.chain >> (5 * k)) & 31], 1u);
				}
				// (n < 8 and id < 32: a deferred chain holds at most the SLL
				// head, Ethernet, 2 tags and IP, layer 0 at 0 and the others
				// inside the 64-byte window)
				uint4 *e = list + (size_t)(ndef + lanes_below(dm)) * SW;
				st_b128(e, make_uint4(i, w.data | w.tail << 16,
						      (uint32_t)w.ip_csum | (uint32_t)w.flags << 16 | w.n << 24 |
							      (uint32_t)w.id << 27,
						      w.chain));
				const uint32_t offs = CR ? 0u
							 : ((uint32_t)(w.offA >> 16) & 0xFF) | ((uint32_t)(w.offA >> 32) & 0xFF) << 8 |
								   ((uint32_t)(w.offA >> 48) & 0xFF) << 16 | (w.offB & 0xFF) << 24;
				st_b128(e + 1, make_uint4((uint32_t)d0, (uint32_t)(d0 >> 32), offs, 0));
			}
			ndef += (uint32_t)__popcll(dm);
		}
	};
#if NSD_FAST_DEPTH == 1
	// software pipeline: tile t walked while tile t+1's chunks and tile t+2's
	// descriptors are in flight
	uint64_t d0 = dsc(base), d1 = dsc(base + stride);
	Chunks<WIN1> ch;
	stage_load<WIN1>(ch, frames, d0, lane);
	for (; base < n; base += stride) {
		const uint64_t d2 = dsc(base + 2 * stride);
		tile(ch, d0, d1);
		d0 = d1;
		d1 = d2;
	}
#elif NSD_FAST_DEPTH == 3
	// three tiles' chunks in flight while one is walked: three register sets
	// in turn (the loop unrolled by three), descriptors four tiles ahead
	uint64_t d0 = dsc(base), d1 = dsc(base + stride), d2 = dsc(base + 2 * stride), d3 = dsc(base + 3 * stride);
	Chunks<WIN1> chA, chB, chC;
	stage_load<WIN1, true>(chA, frames, d0, lane);
	stage_load<WIN1, true>(chB, frames, d1, lane);
	stage_load<WIN1, true>(chC, frames, d2, lane);
	for (;;) {
		uint64_t d4 = dsc(base + 4 * stride);
		tile(chA, d0, d3);
		d0 = d1;
		d1 = d2;
		d2 = d3;
		d3 = d4;
		base += stride;
		if (base >= n)
			break;
		d4 = dsc(base + 4 * stride);
		tile(chB, d0, d3);
		d0 = d1;
		d1 = d2;
		d2 = d3;
		d3 = d4;
		base += stride;
		if (base >= n)
			break;
		d4 = dsc(base + 4 * stride);
		tile(chC, d0, d3);
		d0 = d1;
		d1 = d2;
		d2 = d3;
		d3 = d4;
		base += stride;
		if (base >= n)
			break;
	}
#else
	// two tiles' chunks in flight while one is walked: two register sets that
	// swap roles (the loop unrolled by two), descriptors three tiles ahead
	static_assert(NSD_FAST_DEPTH == 2, "prefetch depth 1, 2 or 3");
	uint64_t d0 = dsc(base), d1 = dsc(base + stride), d2 = dsc(base + 2 * stride);
	Chunks<WIN1> chA, chB;
	stage_load<WIN1, true>(chA, frames, d0, lane);
	stage_load<WIN1, true>(chB, frames, d1, lane);
	for (;;) {
		uint64_t d3 = dsc(base + 3 * stride);
		tile(chA, d0, d2);
		d0 = d1;
		d1 = d2;
		d2 = d3;
		base += stride;
		if (base >= n)
			break;
		d3 = dsc(base + 3 * stride);
		tile(chB, d0, d2);
		d0 = d1;
		d1 = d2;
		d2 = d3;
		base += stride;
		if (base >= n)
			break;
	}
#endif
	drain_stores();   // the loop's records, list entries and side words are complete
	fc.flush(sh.cnt, lane);
}

// The fast kernel's pending ICMPv4 checksums (fast_tiles' list backs): as
// icmp_pass, four lanes per message; the remainder [off, off + len) is summed
// from HBM and the partial sum of the words before it added.
template <int U, bool CR>
__device__ __forceinline__ void fast_icmp_pass(FastShared &sh, const uint8_t *__restrict__ frames,
					       const uint64_t *__restrict__ desc, void *__restrict__ rec,
					       const uint4 *__restrict__ lists, uint32_t cap)
{
	constexpr int SW = 2;
	const int lane = threadIdx.x & 63;
	const int wv = threadIdx.x >> 6;
	const uint32_t sub = lane & 3, grp = lane >> 2;
	uint32_t bad = 0;
	for (int l = 0; l < WAVES; l++) {
		const uint32_t cnt = sh.pcnt[l];
		const uint4 *list = lists + ((size_t)blockIdx.x * WAVES + l) * cap * SW;
		for (uint32_t k0 = 64 * ((wv + l) % WAVES); k0 < cnt; k0 += 64 * WAVES) {
			const bool on = k0 + lane < cnt;
			const uint4 *ep = list + (size_t)(cap - 1 - (k0 + lane)) * SW;
			const uint4 e = on ? ep[0] : make_uint4(0, 0, 0, 0);
			const uint32_t i = e.x;
			const uint64_t a = (on ? NSD_DESC_OFF((uint64_t)ep[1].y << 32 | ep[1].x) : 0) + (e.y & 0xFFFF);
			const uint32_t nb = e.y >> 16;
			for (uint32_t q = 0; q < 64 && k0 + q < cnt; q += 16) {
				const int src = (int)(q + grp);
				const uint32_t alo = __shfl((uint32_t)a, src, 64);
				const uint32_t ahi = __shfl((uint32_t)(a >> 32), src, 64);
				const uint32_t mnb = __shfl(nb, src, 64);
				const uint32_t part = __shfl(e.z, src, 64);
				const bool mon = k0 + (uint32_t)src < cnt;
				const uint32_t s0 = alo & 15, endb = s0 + mnb;
				const uint32_t nch = mon ? (endb + 15) >> 4 : 0u;
				const uint4 *base = (const uint4 *)(frames + ((((uint64_t)ahi << 32) | alo) & ~15ull));
				uint32_t sum = sub == 0 ? part : 0u;
				const uint32_t je = sub == 0 ? 0u : nch - 1;
				if ((sub == 0 && nch > 0) || (sub == 1 && nch > 1))
					sum += csum_chunk(base[je], 16 * je, s0, endb);
				for (uint32_t j = 1 + sub; __ballot(j + 1 < nch); j += 4 * U) {
					uint4 v[U];
#pragma unroll
					for (int u = 0; u < U; u++) {
						const uint32_t jj = j + 4 * u;
						v[u] = jj + 1 < nch ? base[jj] : make_uint4(0, 0, 0, 0);
					}
#pragma unroll
					for (int u = 0; u < U; u++) {
						sum = sum_halves(v[u].x, sum);
						sum = sum_halves(v[u].y, sum);
						sum = sum_halves(v[u].z, sum);
						sum = sum_halves(v[u].w, sum);
					}
				}
				sum = (sum >> 16) + (sum & 0xffff);
				sum += __shfl_xor(sum, 1, 64);
				sum += __shfl_xor(sum, 2, 64);
				const uint32_t mi = __shfl(i, src, 64);
				const bool isbad = mon && sub == 0 && csum_final(sum) != 0;
				if (isbad) {
					uint8_t *nf = (uint8_t *)rec + nflags_at<CR>(mi);
					*nf = *nf | NSD_F_ICMP_BAD;
				}
				bad += FlagCnt::pc(isbad);
			}
		}
	}
	if (lane == 0 && bad)
		atomicAdd(&sh.cnt[NSD_CNT_ICMP_BAD], (unsigned long long)bad);
}

template <int MODE, bool CR>
__device__ __forceinline__ void walk_lists(Shared &sh, uint32_t *s_touch, const uint8_t *__restrict__ frames,
					   const uint64_t *__restrict__ desc, uint32_t n, void *__restrict__ rec,
					   uint32_t *__restrict__ ext, uint32_t ext_words, uint32_t *__restrict__ ext_used,
					   uint32_t chunk, unsigned long long *__restrict__ counters,
					   const uint4 *__restrict__ lists, uint32_t cap, const uint2 *__restrict__ cnts,
					   uint32_t nlists, uint32_t nw, uint64_t *__restrict__ pend, uint32_t region);

// The split schedule's fast kernel.  `tail` (NSD_SPLIT_TAIL): a block whose
// waves deferred packets walks them itself after its tiles (walk_lists over
// its own four lists, the walker pool's LDS in the same words as the fast
// rows), so a batch the fast walk finishes takes one launch instead of two
// (C2: the walker kernel's empty launch cost 4.9 us of 205, at any grid).
template <int MODE, bool CR>
__global__ __launch_bounds__(BLOCK, CR ? NSD_FAST_MINW : NSD_FAST_MINW_FULL) void dissect_fast(
	const uint8_t *__restrict__ frames, const uint64_t *__restrict__ desc, uint32_t n, int start_id,
	void *__restrict__ rec, unsigned long long *__restrict__ counters, uint4 *__restrict__ lists, uint32_t cap,
	uint2 *__restrict__ cnts, const uint32_t *__restrict__ sll, uint32_t *__restrict__ side,
	unsigned long long *__restrict__ sched, uint32_t *__restrict__ ext, uint32_t ext_words,
	uint32_t *__restrict__ ext_used, uint32_t chunk, uint64_t *__restrict__ pend, uint32_t region, uint32_t tail)
{
	constexpr int SW = 2;
	union FastLds {
		FastShared f;
		Shared w;
	};
	__shared__ FastLds su;
	FastShared &sh = su.f;
	if (threadIdx.x < 32)
		sh.ops[threadIdx.x] = 0;
	block_init(sh.cnt, sh.lay3);
	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	const uint32_t gw = blockIdx.x * WAVES + wv;
	uint32_t ndef = 0, nicmp = 0;
	fast_tiles<MODE, CR>(sh, frames, desc, n, start_id, rec, sll, side, lists + (size_t)gw * cap * SW, cap, ndef,
			     nicmp);
	if (lane == 0) {
		cnts[gw] = make_uint2(ndef, nicmp);
		sh.pcnt[wv] = nicmp;
		if (sched && ndef)
			atomicAdd(&sched[0], (unsigned long long)ndef);
		if (sched && nicmp)
			atomicAdd(&sched[1], (unsigned long long)nicmp);
	}
	if (MODE == PRINT_NORM) {
		__syncthreads();   // records final, the block's pending lists and counts complete
		fast_icmp_pass<NSD_FAST_CSUM_U, CR>(sh, frames, desc, rec, lists, cap);
	}
	block_flush(sh.cnt, counters);
	if (threadIdx.x < 32 && sh.ops[threadIdx.x])
		atomicAdd(&counters[NSD_CNT_OPS + threadIdx.x], (unsigned long long)sh.ops[threadIdx.x]);
	if constexpr (NSD_SPLIT_TAIL && (MODE == PRINT_NORM || MODE == PRINT_LESS)) {
		// (the barrier also orders the flush's LDS reads before the walker
		// pool's set-up in the same words)
		if (__syncthreads_or(tail && ndef != 0)) {
			__shared__ uint32_t s_touch[64];
			walk_lists<MODE, CR>(su.w, s_touch, frames, desc, n, rec, ext, ext_words, ext_used, chunk, counters,
					     lists, cap, cnts, gridDim.x * WAVES, gridDim.x * WAVES, pend, region);
		}
	}
}

// The walker kernel: wave g of the grid takes the fast kernel's lists g,
// g + W, g + 2W, ... (W = this grid's waves), 64 deferrals (a chunk) at a
// time, and hands them to its walker pool (walkers()); then, as the fused
// kernel, the leaves and ICMPv4 checksums its walks left pending (its own
// lists, `region` / WAVES slots per wave).  Chunk entries are loaded two
// chunks ahead, and while chunk c's walkers run, the first windows of chunk
// c + 1 (at each packet's cursor) are touched into L2 by 4-byte LDS-DMA loads
// (no VGPR waits for them): its sessions then stage from L2.
// The walker pool over the fast kernel's deferral lists: wave gw takes lists
// gw, gw + nw, ... (nw: the list stride; the fast kernel's own tail passes
// nlists, so each wave takes its own list only), then the block's leaves and
// ICMPv4 checksums.  s_touch: the L2 touches' LDS-DMA target (never read).
template <int MODE, bool CR>
__device__ __forceinline__ void walk_lists(Shared &sh, uint32_t *s_touch, const uint8_t *__restrict__ frames,
					   const uint64_t *__restrict__ desc, uint32_t n, void *__restrict__ rec,
					   uint32_t *__restrict__ ext, uint32_t ext_words, uint32_t *__restrict__ ext_used,
					   uint32_t chunk, unsigned long long *__restrict__ counters,
					   const uint4 *__restrict__ lists, uint32_t cap, const uint2 *__restrict__ cnts,
					   uint32_t nlists, uint32_t nw, uint64_t *__restrict__ pend, uint32_t region)
{
	constexpr int SW = 2;
	if (threadIdx.x < 64)
		sh.step[threadIdx.x] = threadIdx.x < 32 ? c_step[threadIdx.x] : c_lay2h.e[threadIdx.x - 32];
	if (threadIdx.x < 32)
		sh.ops[threadIdx.x] = 0;
	if (threadIdx.x < 2 * WAVES)
		sh.wc[threadIdx.x >> 1][threadIdx.x & 1] = 0;
	block_init(sh.cnt, sh.lay3);
	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	const uint32_t gw = blockIdx.x * WAVES + wv;
	Pending pq{ pend + (size_t)gw * (region / WAVES), region / WAVES, 0, 0 };
	const bool side = CR && ext_words >= n;
	const GenSink<CR> g{ ext, ext_words, ext_used, chunk, &sh.wc[wv][0], sh.ops, &sh.lay[wv][0],
			     side ? n : 0u, side ? ext : nullptr };
	FlagCnt fc;
	Walker wk;
	walk_init(wk.w, 0, 0);
	wk.d = 0;
	wk.i = 0;
	wk.wb = 0;
	wk.wl = 0;
	wk.have = false;
	wk.stage = false;
	WalkOut pw;
	walk_init(pw, 0, 0);
	RingSt rs;   // (unused: the walker kernel stores its records at once)
	rs.init();

	// chunk positions (wave-uniform): list L, first entry k0, the list's count
	struct Pos {
		uint32_t L, k0, cnt;
	};
	auto adv = [&](Pos p) -> Pos {
		p.k0 += 64;
		while (p.L < nlists && p.k0 >= p.cnt) {
			p.L += nw;
			p.k0 = 0;
			p.cnt = p.L < nlists ? min(cnts[p.L].x, cap) : 0u;
		}
		return p;
	};
	auto load = [&](const Pos &p, uint4 &x0, uint4 &x1) {
		x0 = x1 = make_uint4(0, 0, 0, 0);
		if (p.L < nlists && p.k0 + lane < p.cnt) {
			const uint4 *e = lists + ((size_t)p.L * cap + p.k0 + lane) * SW;
			x0 = e[0];
			x1 = e[1];
		}
	};
	Pos p0 = adv(Pos{ gw, 0u - 64u, gw < nlists ? min(cnts[gw].x, cap) : 0u });
	Pos p1 = adv(p0);
	uint4 c0, c1, n0, n1;
	load(p0, c0, c1);
	load(p1, n0, n1);
	while (p0.L < nlists) {
		const Pos p2 = adv(p1);
		{
			// the next chunk's first windows into L2: [cursor, +WIN2) in aligned
			// coordinates, one or two 128-byte lines
			const uint64_t d = (uint64_t)n1.y << 32 | n1.x;
			const uint32_t m = (uint32_t)NSD_DESC_OFF(d) & 15, caplen = NSD_DESC_CAPLEN(d);
			const uint32_t wb = ((n0.y & 0xFFFF) + m) & ~15u;
			const bool on = p1.L < nlists && p1.k0 + lane < p1.cnt && wb < caplen + m;
			const uint64_t a = (uint64_t)frames + (NSD_DESC_OFF(d) & ~15ull) + wb;
			const bool two = on && (a & 127) != 0 && wb + (128 - (uint32_t)(a & 127)) < caplen + m;
			if (on)
				__builtin_amdgcn_global_load_lds((const void *)(a & ~127ull),
								 (__attribute__((address_space(3))) void *)s_touch, 4, 0, 0);
			if (two)
				__builtin_amdgcn_global_load_lds((const void *)((a & ~127ull) + 128),
								 (__attribute__((address_space(3))) void *)s_touch, 4, 0, 0);
		}
		uint4 m0, m1;
		load(p2, m0, m1);
		bool pnd = p0.k0 + lane < p0.cnt;
		const uint32_t pi = c0.x;
		const uint64_t pd = (uint64_t)c1.y << 32 | c1.x;
		walk_init(pw, c0.y >> 16, (int)(c0.z >> 27));
		pw.data = c0.y & 0xFFFF;
		pw.ip_csum = (uint16_t)c0.z;
		pw.flags = (uint8_t)(c0.z >> 16);
		pw.n = (c0.z >> 24) & 7;
		pw.chain = c0.w;
		if (!CR) {
			// layer starts 1..4 (layer 0 at 0)
			pw.offA = (uint64_t)(c1.z & 0xFF) << 16 | (uint64_t)((c1.z >> 8) & 0xFF) << 32 |
				  (uint64_t)((c1.z >> 16) & 0xFF) << 48;
			pw.offB = c1.z >> 24;
		}
		walkers<MODE, CR, false>(sh, rs, frames, rec, g, pq, fc, wk, pnd, pw, pi, pd, false);
		c0 = n0;
		c1 = n1;
		n0 = m0;
		n1 = m1;
		p0 = p1;
		p1 = p2;
	}
	{
		bool none = false;
		if (__ballot(wk.have))
			walkers<MODE, CR, false>(sh, rs, frames, rec, g, pq, fc, wk, none, pw, 0, 0, true);
	}
	fc.flush(sh.cnt, lane);
	leaf_pass<MODE, CR>(frames, desc, rec, ext, pq);
	if (lane == 0)
		sh.pcnt[wv] = pq.npend;
	if (MODE == PRINT_NORM) {
		__syncthreads();
		icmp_pass<NSD_CSUM_U, CR>(sh, frames, desc, rec, pend, region);
	}
	block_flush(sh.cnt, counters);
	if (threadIdx.x < 32 && sh.ops[threadIdx.x])
		atomicAdd(&counters[NSD_CNT_OPS + threadIdx.x], (unsigned long long)sh.ops[threadIdx.x]);
}

template <int MODE, bool CR>
__global__ __launch_bounds__(BLOCK, NSD_MINW) void dissect_walk(
	const uint8_t *__restrict__ frames, const uint64_t *__restrict__ desc, uint32_t n,
	void *__restrict__ rec, uint32_t *__restrict__ ext, uint32_t ext_words,
	uint32_t *__restrict__ ext_used, uint32_t chunk, unsigned long long *__restrict__ counters,
	const uint4 *__restrict__ lists, uint32_t cap, const uint2 *__restrict__ cnts, uint32_t nlists,
	uint64_t *__restrict__ pend, uint32_t region)
{
	__shared__ Shared sh;
	__shared__ uint32_t s_touch[64];
	{
		// nothing deferred to this block's waves (the common case of traffic
		// the fast walk finishes): leave before any set-up
		const uint32_t nw = gridDim.x * WAVES;
		bool any = false;
		for (uint32_t L = blockIdx.x * WAVES + (threadIdx.x % WAVES) + (threadIdx.x / WAVES) * nw; L < nlists;
		     L += (BLOCK / WAVES) * nw)
			any = any || cnts[L].x != 0;
		if (!__syncthreads_or(any))
			return;
	}
	walk_lists<MODE, CR>(sh, s_touch, frames, desc, n, rec, ext, ext_words, ext_used, chunk, counters, lists, cap,
			     cnts, nlists, gridDim.x * WAVES, pend, region);
}

} // namespace nsd

// ---- launcher (C ABI, called by nsd_host.cpp / nsd_pipe.cpp) -----------------
// A persistent grid of at most NSD_MAX_GRID blocks; block b owns pending
// lists b (room for every packet it visits).
constexpr uint32_t NSD_MAX_GRID = 4096;

static uint32_t region_for(uint32_t n, uint32_t blocks)
{
	const uint64_t stride = (uint64_t)blocks * nsd::BLOCK;
	return (uint32_t)(((n + stride - 1) / stride) * nsd::BLOCK);
}
// the fused kernel's pending-list slots per block: its waves take their
// group's tiles at run time (walk_tiles, compact records), so each list holds twice a wave's
// even share plus four tiles (8 bytes a slot: within the workspace's first
// 32 bytes per region slot, sched_pair_at)
// (Each packet a wave visits adds at most one pending-list entry - an ICMPv4
// message past its windows from the front, or a host-rendered leaf from the
// back, never both: a leaf ends a chain that has no ICMPv4 layer - and
// walk_tiles asks for a tile only while the list has room for every packet
// of the tiles it holds; a wave that found its list overrun counts it in
// NSD_CNT_LISTOVF.)
static uint32_t region_for_fused(uint32_t n, uint32_t blocks, bool compact)
{
	return NSD_GROUP_TILES && compact ? 2 * region_for(n, blocks) + nsd::WAVES * 4 * 64 : region_for(n, blocks);
}

// worst case over grids: sum of regions <= n + blocks * BLOCK
static size_t region_slots(uint32_t n)
{
	return ((size_t)n + (size_t)NSD_MAX_GRID * nsd::BLOCK + 1) & ~(size_t)1;
}

// ---- the schedule -------------------------------------------------------------
// split (dissect_fast + dissect_walk) or fused (dissect_all).  The split
// schedule runs the fast walk at 6 waves per SIMD instead of 4 and wins when
// the fast walk finishes nearly every packet and few ICMPv4 messages run
// past their windows (C2 16M x 64 B: 0.233 against 0.249 ms).  When many
// packets need the general walk (C4's IPv6 extension chains) the fused
// kernel wins by far (1.17 against 1.88 ms): its walkers take a tile's
// packets while their first lines are still on chip, where the walker
// kernel re-reads them and the fast kernel writes a list entry per packet.
// When many ICMPv4 checksums are left to a pass (C3 IMIX: about a fifth of
// the packets) the fused kernel wins too (0.70 - 0.75 against 0.73 - 0.81
// ms on the same boxes, r03): its checksum pass streams at 4 waves per SIMD
// with 8 loads in flight per lane.  Adaptive (the default): every
// NSD_SCHED_SAMPLE launches on a device, one launch is sampled: its kernels
// count the packets the fast walk handed over and the ICMPv4 messages left
// to a pass into a pair at the end of that launch's own workspace (zeroed
// before it, copied to pinned host memory after it, on its stream), so
// launches on other streams or pipes never mix into the sample.  Once the
// copy has landed, the two shares of that launch's packets pick the
// schedule for the launches after it, with hysteresis (fused above 15 %
// deferred or 10 % pending checksums, split again below 5 % of both).  A
// capture's traffic mix changes slowly against batches of a few
// milliseconds; both schedules give identical results.  nsd_set_schedule
// forces one (tests).  The same sample brings back the launch's packet and
// byte counts (the counter vector before and after it): when its frames
// average at most NSD_SMALL_FRAME bytes, the fast kernel runs
// NSD_FAST_BPC_SMALL blocks per CU instead of NSD_FAST_BPC (C2's 64-byte
// frames stream from few waves: 0.217 -> 0.207 ms at 2 blocks per CU on one
// box, where IMIX frames need the third: 0.78 against 0.92 ms); and when
// more than a quarter of its packets went to the walkers, the fused kernel
// runs without the progress priority (walk_tiles: C4 -1 % without it, C3
// +0.7 %, in the same kernel) and with the record ring (RingSt: C4's writes
// halved, C3 +3 % with it; on until the first sample is read).  State is per
// device.
#ifndef NSD_SCHED_SAMPLE
#define NSD_SCHED_SAMPLE 32
#endif
namespace {
constexpr int MAX_DEV = 16;
#ifndef NSD_SMALL_FRAME
#define NSD_SMALL_FRAME 128
#endif
#ifndef NSD_FAST_BPC_SMALL
#define NSD_FAST_BPC_SMALL 2
#endif
struct Sched {
	bool init = false, fused = false, pending = false, small = false;
	bool walky = false;                    // the sample's deferred share above 25 % (no progress priority)
	bool sampled_once = false;             // a sample has been read
	bool recorded = false;                 // the pending sample's event is recorded (sched_sampled)
	bool discard = false;                  // the pending sample failed: wait for its copies, use nothing
	int launches = 0, last = 0;
	uint64_t sampled = 0;                  // packets of the sampled launch in flight
	unsigned long long *host = nullptr;    // its pair, then its counters [32, 34) before and after
	hipEvent_t ev = nullptr;
	int cus = 0;                           // compute units of the device
};
Sched g_sched[MAX_DEV];
std::mutex g_sched_mu;
int g_sched_force = 0;   // 0 adaptive, NSD_SCHED_SPLIT, NSD_SCHED_FUSED
int g_ring_force = 0;    // nsd_set_record_ring: 0 adaptive, 1 on, 2 off
std::atomic<int> g_grid_cap{ 0 };   // nsd_set_grid_cap

int cur_dev()
{
	int d = 0;
	if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= MAX_DEV)
		d = 0;
	return d;
}

// The plan of one launch of n packets on the current device: the schedule,
// and whether this launch is the sample (then its pair is zeroed on
// `stream` here and copied back by sched_sampled after the kernels).
struct Plan {
	bool fused, sample, small, prio, ring;
	int cus;
};
Plan sched_plan(uint32_t n, unsigned long long *pair, const uint64_t *counters, hipStream_t stream)
{
	std::lock_guard<std::mutex> g(g_sched_mu);
	const int dev = cur_dev();
	Sched &S = g_sched[dev];
	if (!S.cus) {
		int cus = 0;
		if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
			cus = 256;
		S.cus = cus;
	}
	Plan p{ false, false, false, true, true, S.cus };
	// a launch captured into a graph takes the schedule as it stands and is
	// never the sample (an event query or a host copy would break the
	// capture; the graph replays this plan)
	hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
	const bool capturing = hipStreamIsCapturing(stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
	// (a sample is read only once sched_sampled has recorded its event: between
	// the plan and that record, the event still stands for an older sample, and
	// another stream's launch must not take the copies in flight for it)
	if (!capturing && S.pending && S.recorded && hipEventQuery(S.ev) == hipSuccess && S.discard) {
		S.pending = S.recorded = S.discard = false;
	} else if (!capturing && S.pending && S.recorded && hipEventQuery(S.ev) == hipSuccess) {
		const double rd = S.sampled ? (double)S.host[0] / (double)S.sampled : 0.0;
		const double ri = S.sampled ? (double)S.host[1] / (double)S.sampled : 0.0;
		S.fused = S.fused ? rd > 0.05 || ri > 0.05 : rd > 0.15 || ri > 0.10;
		const uint64_t pk = S.host[4] - S.host[2], by = S.host[5] - S.host[3];
		if (pk)
			S.small = by <= (uint64_t)NSD_SMALL_FRAME * pk;
		S.walky = rd > 0.25;
		S.sampled_once = true;
		S.pending = false;
		S.recorded = false;
	}
	if (!S.init && !capturing) {
		S.init = true;
		if (hipHostMalloc((void **)&S.host, 64, hipHostMallocDefault) != hipSuccess ||
		    hipEventCreateWithFlags(&S.ev, hipEventDisableTiming) != hipSuccess)
			S.host = nullptr;
	}
	p.fused = g_sched_force ? g_sched_force == NSD_SCHED_FUSED : S.fused;
	p.small = S.small;
	p.prio = !S.walky;
	// the record ring until a sample shows a quarter or less of the packets
	// deferred (C3: +3 % with it; C4: writes 23.7 -> 12.2 B/packet)
	p.ring = g_ring_force ? g_ring_force == 1 : !S.sampled_once || S.walky;
	if (!capturing && ++S.launches >= NSD_SCHED_SAMPLE && !S.pending && S.host && pair && counters &&
	    hipMemsetAsync(pair, 0, 16, stream) == hipSuccess &&
	    hipMemcpyAsync(S.host + 2, counters + NSD_CNT_PKTS, 16, hipMemcpyDeviceToHost, stream) == hipSuccess) {
		p.sample = true;
		S.launches = 0;
		S.sampled = n;
		S.pending = true;   // (until its copy lands)
		S.recorded = false;
	}
	S.last = p.fused ? NSD_SCHED_FUSED : NSD_SCHED_SPLIT;
	return p;
}

// A failed sample (under the lock): copies queued for it may still be in
// flight into S.host, so the sample stays pending - no later sample queues
// copies into the same words - until an event behind them completes, and
// its values are discarded then (sched_plan).  Without an event, the stream
// is drained here instead.
void sched_fail(Sched &S, hipStream_t stream)
{
	S.discard = true;
	if (hipEventRecord(S.ev, stream) == hipSuccess) {
		S.recorded = true;
		return;
	}
	(void)hipStreamSynchronize(stream);
	S.pending = S.recorded = S.discard = false;
}

// after the sampled launch's kernels on `stream`: bring its pair and
// counters back
void sched_sampled(unsigned long long *pair, const uint64_t *counters, hipStream_t stream)
{
	std::lock_guard<std::mutex> g(g_sched_mu);
	Sched &S = g_sched[cur_dev()];
	if (hipMemcpyAsync(S.host, pair, 16, hipMemcpyDeviceToHost, stream) != hipSuccess ||
	    hipMemcpyAsync(S.host + 4, counters + NSD_CNT_PKTS, 16, hipMemcpyDeviceToHost, stream) != hipSuccess ||
	    hipEventRecord(S.ev, stream) != hipSuccess) {
		sched_fail(S, stream);
		return;
	}
	S.recorded = true;
}

// the sampled launch's kernels failed to launch: drop the sample (once the
// copies sched_plan queued for it have landed)
void sched_abort(hipStream_t stream)
{
	std::lock_guard<std::mutex> g(g_sched_mu);
	sched_fail(g_sched[cur_dev()], stream);
}
} // namespace

extern "C" int nsd_set_schedule(int sched)
{
	if (sched != NSD_SCHED_ADAPTIVE && sched != NSD_SCHED_SPLIT && sched != NSD_SCHED_FUSED)
		return NSD_ERR_ARG;
	std::lock_guard<std::mutex> g(g_sched_mu);
	const int prev = g_sched_force;
	g_sched_force = sched;
	return prev;
}

extern "C" int nsd_set_record_ring(int mode)
{
	if (mode < 0 || mode > 2)
		return NSD_ERR_ARG;
	std::lock_guard<std::mutex> g(g_sched_mu);
	const int prev = g_ring_force;
	g_ring_force = mode;
	return prev;
}

extern "C" int nsd_set_grid_cap(int blocks)
{
	if (blocks < 0)
		return NSD_ERR_ARG;
	return g_grid_cap.exchange(blocks);
}

extern "C" int nsd_last_schedule(void)
{
	std::lock_guard<std::mutex> g(g_sched_mu);
	return g_sched[cur_dev()].last;
}

// workspace: the fused kernel's pending lists (u64 per slot); the split
// schedule's fast lists (up to 32 bytes per slot), their counts and the
// walker kernel's pending lists (u64 per slot, up to two per packet slot)
static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
// (the last 256 bytes: the schedule sample's pair, at sched_pair_at)
// (then the fused kernel's group tile counters: a 128-byte line per block
// at most, gtiles_at)
static size_t gtiles_at(uint32_t n)
{
	const size_t slots = region_slots(n);
	return align256(align256(32 * slots) + align256((size_t)NSD_MAX_GRID * nsd::WAVES * 8) + 16 * slots);
}
static size_t sched_pair_at(uint32_t n)
{
	return gtiles_at(n) + (size_t)NSD_MAX_GRID * 128;
}
extern "C" size_t nsd_launch_workspace_bytes(uint32_t n)
{
	return sched_pair_at(n) + 256;
}

extern "C" int nsd_launch_dissect_rec(const uint8_t *d_frames, const uint64_t *d_desc, const void *d_sll,
				      uint32_t n, int start_id, int mode, void *d_rec, int compact, uint32_t *d_ext,
				      uint32_t ext_words, uint32_t *d_ext_used, uint64_t *d_counters, void *d_ws,
				      int grid, hipStream_t stream);

extern "C" int nsd_launch_dissect(const uint8_t *d_frames, const uint64_t *d_desc, uint32_t n,
				  int start_id, int mode, nsd_rec *d_rec, uint32_t *d_ext,
				  uint32_t ext_words, uint32_t *d_ext_used, uint64_t *d_counters,
				  void *d_ws, int grid, hipStream_t stream)
{
	return nsd_launch_dissect_rec(d_frames, d_desc, nullptr, n, start_id, mode, d_rec, 0, d_ext, ext_words,
				      d_ext_used, d_counters, d_ws, grid, stream);
}

extern "C" int nsd_launch_dissect_sll(const uint8_t *d_frames, const uint64_t *d_desc, const void *d_sll,
				      uint32_t n, int start_id, int mode, nsd_rec *d_rec, uint32_t *d_ext,
				      uint32_t ext_words, uint32_t *d_ext_used, uint64_t *d_counters,
				      void *d_ws, int grid, hipStream_t stream)
{
	return nsd_launch_dissect_rec(d_frames, d_desc, d_sll, n, start_id, mode, d_rec, 0, d_ext, ext_words,
				      d_ext_used, d_counters, d_ws, grid, stream);
}

// d_sll: one struct sockaddr_ll (nsd_sll_t, 20 bytes) per packet, or NULL
// (read as zeros); used by the LINKTYPE_LINUX_SLL head only.  d_rec: n
// nsd_rec (16 B), or n nsd_crec (8 B) when `compact`.
extern "C" int nsd_launch_dissect_rec(const uint8_t *d_frames, const uint64_t *d_desc, const void *d_sll,
				      uint32_t n, int start_id, int mode, void *d_rec, int compact, uint32_t *d_ext,
				      uint32_t ext_words, uint32_t *d_ext_used, uint64_t *d_counters, void *d_ws,
				      int grid, hipStream_t stream)
{
	using namespace nsd;
	if (n == 0)
		return 0;
	const int mi = mode == PRINT_NORM ? 0 : mode == PRINT_LESS ? 1 : 2;
	const int ci = compact ? 1 : 0;
	const uint32_t waves = (n + 63) / 64;
	const uint32_t want = (waves + WAVES - 1) / WAVES;
	// ext pool chunk per request: half the pool spread over the waves, so the
	// unused chunk tails the waves keep at the end waste at most half of it
	// (a pool of 2x the words the chains need never overflows), within
	// [1 deep entry, 512 short entries]
	if (ext_words > NSD_EXT_POOL_MAX_WORDS)
		ext_words = NSD_EXT_POOL_MAX_WORDS;
	auto chunk_for = [&](uint32_t blocks) {
		const uint64_t per = (uint64_t)ext_words / (2ull * blocks * WAVES);
		const uint32_t lo = NSD_EXT_WORDS(NSD_EXT_MAX_LAYERS), hi = 512 * NSD_EXT_WORDS(16);
		return (uint32_t)(per < lo ? lo : per > hi ? hi : per) & ~3u;
	};
	// persistent grids: exactly the blocks that are resident together (CUs x
	// the kernel's occupancy), so no block waits for a second round; every
	// block grid-strides (counters then cost one flush per block).  The
	// occupancy of a kernel is a property of its code (one gfx950 build):
	// cached once, racing callers store the same value.
	auto occupancy = [&](const void *f, std::atomic<int> &slot, int dflt) {
		int occ = slot.load(std::memory_order_relaxed);
		if (!occ) {
			if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, f, BLOCK, 0) != hipSuccess || occ < 1)
				occ = dflt;
			slot.store(occ, std::memory_order_relaxed);
		}
		return occ;
	};
	if (grid <= 0)
		grid = g_grid_cap.load(std::memory_order_relaxed);
	unsigned long long *const pair = d_ws ? (unsigned long long *)((uint8_t *)d_ws + sched_pair_at(n)) : nullptr;
	const Plan plan = sched_plan(n, mi != 2 ? pair : nullptr, d_counters, stream);
	const int s_cus = plan.cus;
	unsigned long long *const sched = plan.sample ? pair : nullptr;
	const bool fused = mi != 2 && plan.fused;
	if (fused) {
	typedef void (*kfn)(const uint8_t *, const uint64_t *, uint32_t, int, void *, uint32_t *, uint32_t,
			    uint32_t *, uint32_t, unsigned long long *, uint64_t *, uint32_t, const uint32_t *,
			    unsigned long long *, uint32_t *, uint32_t);
	static const kfn kernels[2][3] = {
		{ dissect_all<PRINT_NORM, false>, dissect_all<PRINT_LESS, false>, dissect_all<PRINT_HEX, false> },
		{ dissect_all<PRINT_NORM, true>, dissect_all<PRINT_LESS, true>, dissect_all<PRINT_HEX, true> },
	};
	// compact records of walker-heavy batches: the record ring's build (an
	// instantiation of its own: beside the ring's code, the records held one
	// tile in registers spill, and without them C3 runs 4 % slower)
	static const kfn ring_kernels[2] = { dissect_all<PRINT_NORM, true, true>, dissect_all<PRINT_LESS, true, true> };
	static std::atomic<int> s_occ[2][3], s_rocc[2];
	const bool ring = NSD_RING && plan.ring && ci == 1 && mi < 2;
	const kfn f = ring ? ring_kernels[mi] : kernels[ci][mi];
	std::atomic<int> &occ_slot = ring ? s_rocc[mi] : s_occ[ci][mi];
	uint32_t cap_blocks = grid > 0 ? (uint32_t)grid : (uint32_t)(s_cus * occupancy((const void *)f, occ_slot, 4));
	if (cap_blocks > NSD_MAX_GRID)
		cap_blocks = NSD_MAX_GRID;
	const uint32_t blocks = want < cap_blocks ? want : cap_blocks;
	// the CU groups' tile counters (walk_tiles), a 128-byte line each, zeroed
	// on the launch's stream
	uint32_t *const gtiles = (uint32_t *)((uint8_t *)d_ws + gtiles_at(n));
	if (NSD_GROUP_TILES && compact) {
		hipLaunchKernelGGL(zero_tiles, dim3((blocks + 255) / 256), dim3(256), 0, stream, gtiles, blocks);
		if (hipGetLastError() != hipSuccess) {
			if (sched)
				sched_abort(stream);
			return -2;
		}
	}
	hipLaunchKernelGGL(f, dim3(blocks), dim3(BLOCK), 0, stream, d_frames, d_desc, n, start_id, d_rec, d_ext,
			   ext_words, d_ext_used, chunk_for(blocks), (unsigned long long *)d_counters, (uint64_t *)d_ws,
			   region_for_fused(n, blocks, compact), (const uint32_t *)d_sll, sched, gtiles,
			   plan.prio ? 1u : 0u);
	if (hipGetLastError() != hipSuccess) {
		if (sched)
			sched_abort(stream);
		return -2;
	}
	if (sched)
		sched_sampled(sched, d_counters, stream);
	return 0;
	}
	typedef void (*ffn)(const uint8_t *, const uint64_t *, uint32_t, int, void *, unsigned long long *, uint4 *,
			    uint32_t, uint2 *, const uint32_t *, uint32_t *, unsigned long long *, uint32_t *, uint32_t,
			    uint32_t *, uint32_t, uint64_t *, uint32_t, uint32_t);
	typedef void (*wfn)(const uint8_t *, const uint64_t *, uint32_t, void *, uint32_t *, uint32_t, uint32_t *,
			    uint32_t, unsigned long long *, const uint4 *, uint32_t, const uint2 *, uint32_t, uint64_t *,
			    uint32_t);
	static const ffn fast[2][3] = {
		{ dissect_fast<PRINT_NORM, false>, dissect_fast<PRINT_LESS, false>, dissect_fast<PRINT_HEX, false> },
		{ dissect_fast<PRINT_NORM, true>, dissect_fast<PRINT_LESS, true>, dissect_fast<PRINT_HEX, true> },
	};
	static const wfn walk[2][2] = {
		{ dissect_walk<PRINT_NORM, false>, dissect_walk<PRINT_LESS, false> },
		{ dissect_walk<PRINT_NORM, true>, dissect_walk<PRINT_LESS, true> },
	};
	static std::atomic<int> s_focc[2][3], s_wocc[2][2];
	// grid > 0 (tests): both kernels' grids capped at `grid` blocks
	uint32_t fcap = grid > 0 ? (uint32_t)grid
				 : (uint32_t)(s_cus * occupancy((const void *)fast[ci][mi], s_focc[ci][mi], 8));
	// with two tiles in flight per wave, 3 blocks per CU outrun the 4 that
	// fit (HBM serves fewer concurrent streams better), and 2
	// the 3 when the frames are small (the sample, sched_plan)
	const int bpc = plan.small ? NSD_FAST_BPC_SMALL : NSD_FAST_BPC;
	if (grid <= 0 && bpc > 0 && fcap > (uint32_t)(s_cus * bpc))
		fcap = (uint32_t)(s_cus * bpc);
	if (fcap > NSD_MAX_GRID)
		fcap = NSD_MAX_GRID;
	const uint32_t fblocks = want < fcap ? want : fcap;
	const uint32_t cap = region_for(n, fblocks) / WAVES;   // slots per fast wave
	const uint32_t nlists = fblocks * WAVES;
	const size_t slotb = 32;   // a list slot: two uint4 (fast_tiles)
	uint8_t *ws = (uint8_t *)d_ws;
	uint4 *lists = (uint4 *)ws;
	uint2 *cnts = (uint2 *)(ws + align256(slotb * nlists * cap));
	uint64_t *pend = (uint64_t *)((uint8_t *)cnts + align256((size_t)nlists * 8));
	// compact records: the pool's side words (when it has them), for leaf ends
	uint32_t *side = compact && d_ext && ext_words >= n ? d_ext : nullptr;
	// NSD_SPLIT_TAIL: each fast block walks its own deferrals, one list per
	// wave (`region` = cap slots of walker pending entries per wave)
	const bool tail = NSD_SPLIT_TAIL && mi != 2;
	hipLaunchKernelGGL(fast[ci][mi], dim3(fblocks), dim3(BLOCK), 0, stream, d_frames, d_desc, n, start_id, d_rec,
			   (unsigned long long *)d_counters, lists, cap, cnts, (const uint32_t *)d_sll, side, sched, d_ext,
			   ext_words, d_ext_used, chunk_for(fblocks), pend, cap * WAVES, tail ? 1u : 0u);
	if (hipGetLastError() != hipSuccess) {
		if (sched)
			sched_abort(stream);
		return -2;
	}
	if (mi == 2 || tail) {
		if (sched && tail)
			sched_sampled(sched, d_counters, stream);
		return 0;   // no chains: nothing deferred; or the fast blocks walked their own
	}
	uint32_t wcap = grid > 0 ? (uint32_t)grid
				 : (uint32_t)(s_cus * occupancy((const void *)walk[ci][mi], s_wocc[ci][mi], 4));
#ifdef NSD_WALK_GRID_CAP
	if (wcap > NSD_WALK_GRID_CAP)
		wcap = NSD_WALK_GRID_CAP;
#endif
	const uint32_t wblocks = fblocks < wcap ? fblocks : wcap;
	const uint32_t per_wave = (nlists + wblocks * WAVES - 1) / (wblocks * WAVES);   // lists per walker wave
	hipLaunchKernelGGL(walk[ci][mi], dim3(wblocks), dim3(BLOCK), 0, stream, d_frames, d_desc, n, d_rec, d_ext,
			   ext_words, d_ext_used, chunk_for(wblocks), (unsigned long long *)d_counters, lists, cap, cnts,
			   nlists, pend, per_wave * cap * WAVES);
	if (hipGetLastError() != hipSuccess) {
		if (sched)
			sched_abort(stream);
		return -2;
	}
	if (sched)
		sched_sampled(sched, d_counters, stream);
	return 0;
}

