// nsd_pipe.cpp - pipelined host-batch path (include/netsniff_dissect.h,
// nsd_pipe_*): the capture side of SURVEY 8f.2.  A batch (one TPACKET_V3
// block, walk_t3_block netsniff-ng.c:991-1039, or a run of pcap records,
// read_pcap netsniff-ng.c:700-760) goes H2D, through the dissect kernels and
// D2H on its own stream slot; `depth` slots rotate, so batch k's copies
// overlap batch k+1's walk and the H2D / D2H engines run concurrently.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/netsniff_dissect.h"

extern "C" int nsd_launch_dissect_rec(const uint8_t *d_frames, const uint64_t *d_desc, const void *d_sll,
				      uint32_t n, int start_id, int mode, void *d_rec, int compact, uint32_t *d_ext,
				      uint32_t ext_words, uint32_t *d_ext_used, uint64_t *d_counters, void *d_ws,
				      int grid, hipStream_t stream);
extern "C" size_t nsd_launch_workspace_bytes(uint32_t n);
int nsd_start_for(int linktype);

namespace {
constexpr int MAX_DEPTH = 8;

bool ok(hipError_t e, const char *what)
{
	if (e != hipSuccess) {
		fprintf(stderr, "netsniff-dissect pipe: %s: %s\n", what, hipGetErrorString(e));
		return false;
	}
	return true;
}

// makes the pipe's device current for a scope (a caller that switched device
// since the pipe was created still runs the pipe's batches where its buffers
// are, and the launch's per-device schedule state is the pipe's device's)
struct OnDevice {
	int prev = -1;
	explicit OnDevice(int dev)
	{
		if (hipGetDevice(&prev) != hipSuccess || prev == dev)
			prev = -1;
		else if (hipSetDevice(dev) != hipSuccess)
			prev = -1;
	}
	~OnDevice()
	{
		if (prev >= 0)
			(void)hipSetDevice(prev);
	}
};

struct Slot {
	hipStream_t stream = nullptr;
	hipEvent_t done = nullptr;
	uint8_t *frames = nullptr;
	uint64_t *desc = nullptr;
	nsd_sll_t *sll = nullptr;    // per-packet sockaddr_ll (SLL link types)
	nsd_rec *rec = nullptr;
	uint32_t *ext = nullptr;
	uint32_t *small = nullptr;   // ext_count at +0, counters at +64 (device)
	uint64_t *small_h = nullptr; // pinned host copy of the same 576 bytes
	void *ws = nullptr;
	// the batch in flight
	bool busy = false;
	int status = NSD_OK;
	uint32_t n = 0;
	void *rec_out = nullptr;
	uint32_t *ext_out = nullptr;
	uint32_t *ext_count_out = nullptr;
	uint64_t *counters_out = nullptr;
	int *status_out = nullptr;
};
} // namespace

struct nsd_pipe {
	uint32_t max_pkts = 0;
	size_t max_bytes = 0;
	uint32_t ext_cap = 0;   // ext pool words per batch
	int depth = 0;
	int start_id = 0;
	int mode = 0;
	int device = 0;         // the device current at creation: its streams and buffers
	bool compact = false;   // nsd_crec records (nsd_pipe_create_compact)
	int head = 0;    // oldest in flight
	int count = 0;   // in flight
	Slot slot[MAX_DEPTH];
};

static void slot_free(Slot &s)
{
	if (s.stream) (void)hipStreamDestroy(s.stream);
	if (s.done) (void)hipEventDestroy(s.done);
	if (s.frames) (void)hipFree(s.frames);
	if (s.desc) (void)hipFree(s.desc);
	if (s.sll) (void)hipFree(s.sll);
	if (s.rec) (void)hipFree(s.rec);
	if (s.ext) (void)hipFree(s.ext);
	if (s.small) (void)hipFree(s.small);
	if (s.small_h) (void)hipHostFree(s.small_h);
	if (s.ws) (void)hipFree(s.ws);
	s = Slot();
}

extern "C" void nsd_pipe_destroy(nsd_pipe *p)
{
	if (!p)
		return;
	const OnDevice on(p->device);
	nsd_pipe_drain(p);
	for (int k = 0; k < p->depth; k++)
		slot_free(p->slot[k]);
	delete p;
}

static nsd_pipe *pipe_create(uint32_t max_pkts, size_t max_frame_bytes, uint32_t ext_cap, int depth, int linktype,
			     int mode, bool compact);

extern "C" nsd_pipe *nsd_pipe_create(uint32_t max_pkts, size_t max_frame_bytes, uint32_t ext_cap,
				     int depth, int linktype, int mode)
{
	return pipe_create(max_pkts, max_frame_bytes, ext_cap, depth, linktype, mode, false);
}

extern "C" nsd_pipe *nsd_pipe_create_compact(uint32_t max_pkts, size_t max_frame_bytes, uint32_t ext_cap,
					     int depth, int linktype, int mode)
{
	return pipe_create(max_pkts, max_frame_bytes, ext_cap, depth, linktype, mode, true);
}

static nsd_pipe *pipe_create(uint32_t max_pkts, size_t max_frame_bytes, uint32_t ext_cap, int depth, int linktype,
			     int mode, bool compact)
{
	if (!max_pkts || !max_frame_bytes || depth < 1 || depth > MAX_DEPTH || mode < PRINT_NORM ||
	    mode > PRINT_NONE)
		return nullptr;
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
		return nullptr;
	int dev = 0;
	if (hipGetDevice(&dev) != hipSuccess)
		return nullptr;
	nsd_pipe *p = new nsd_pipe;
	p->device = dev;
	p->max_pkts = max_pkts;
	p->max_bytes = max_frame_bytes;
	p->ext_cap = ext_cap;
	p->depth = depth;
	p->start_id = nsd_start_for(linktype);
	p->mode = mode;
	p->compact = compact;
	for (int k = 0; k < depth; k++) {
		Slot &s = p->slot[k];
		bool good = ok(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking), "stream") &&
			    ok(hipEventCreateWithFlags(&s.done, hipEventDisableTiming), "event") &&
			    ok(hipMalloc(&s.frames, max_frame_bytes + NSD_FRAME_PAD), "hipMalloc") &&
			    ok(hipMalloc(&s.desc, (size_t)max_pkts * 8), "hipMalloc") &&
			    ok(hipMalloc(&s.sll, (size_t)max_pkts * sizeof(nsd_sll_t)), "hipMalloc") &&
			    ok(hipMalloc(&s.rec, (size_t)max_pkts * sizeof(nsd_rec)), "hipMalloc") &&
			    (!ext_cap || ok(hipMalloc(&s.ext, (size_t)ext_cap * 4), "hipMalloc")) &&
			    ok(hipMalloc(&s.small, 64 + NSD_NCOUNTERS * 8), "hipMalloc") &&
			    ok(hipHostMalloc(&s.small_h, 64 + NSD_NCOUNTERS * 8, hipHostMallocDefault), "hipHostMalloc") &&
			    ok(hipMalloc(&s.ws, nsd_launch_workspace_bytes(max_pkts)), "hipMalloc");
		if (!good) {
			nsd_pipe_destroy(p);
			return nullptr;
		}
	}
	return p;
}

// complete the oldest batch
static int complete_oldest(nsd_pipe *p)
{
	Slot &s = p->slot[p->head];
	int st = s.status;
	if (st == NSD_OK && !ok(hipEventSynchronize(s.done), "batch"))
		st = NSD_ERR_HIP;
	if (st == NSD_OK) {
		const uint32_t used = (uint32_t)s.small_h[0];
		if (s.counters_out)
			memcpy(s.counters_out, s.small_h + 8, NSD_NCOUNTERS * 8);
		if (s.ext_count_out)
			*s.ext_count_out = used;
		// compact records: the side words [0, n) and the entries after them,
		// only when a record of the batch needs either (a chain in the ext
		// form, or a host-rendered leaf's end)
		const bool side = s.small_h[8 + NSD_CNT_EXT] || s.small_h[8 + NSD_CNT_HOST];
		const uint64_t need = p->compact ? (side ? (uint64_t)s.n + used : 0) : used;
		const uint32_t k = need < p->ext_cap ? (uint32_t)need : p->ext_cap;
		if (k && s.ext_out &&
		    !ok(hipMemcpyAsync(s.ext_out, s.ext, (size_t)k * 4, hipMemcpyDeviceToHost,
				       s.stream), "ext D2H"))
			st = NSD_ERR_HIP;
		if (k && s.ext_out && st == NSD_OK && !ok(hipStreamSynchronize(s.stream), "ext D2H"))
			st = NSD_ERR_HIP;
	}
	if (s.status_out)
		*s.status_out = st;
	s.busy = false;
	p->head = (p->head + 1) % p->depth;
	p->count--;
	return st;
}

extern "C" int nsd_pipe_wait(nsd_pipe *p)
{
	if (!p)
		return NSD_ERR_ARG;
	if (!p->count)
		return 1;
	const OnDevice on(p->device);
	return complete_oldest(p);
}

extern "C" int nsd_pipe_drain(nsd_pipe *p)
{
	if (!p)
		return NSD_ERR_ARG;
	const OnDevice on(p->device);
	int st = NSD_OK;
	while (p->count) {
		int r = complete_oldest(p);
		if (r != NSD_OK && st == NSD_OK)
			st = r;
	}
	return st;
}

extern "C" int nsd_pipe_submit(nsd_pipe *p, const uint8_t *frames, size_t frames_len,
			       const nsd_desc_t *desc, uint32_t n, nsd_rec *rec, uint32_t *ext,
			       uint32_t *ext_count, uint64_t *counters, int *status)
{
	return nsd_pipe_submit_sll(p, frames, frames_len, desc, nullptr, n, rec, ext, ext_count, counters,
				   status);
}

// same, with one sockaddr_ll per packet (pkt->sll of the SLL heads; the
// *_LL pcap record's cooked header or the RX ring's per-frame sockaddr_ll);
// sll may be NULL (the heads read zeros)
static int pipe_submit(nsd_pipe *p, const uint8_t *frames, size_t frames_len, const nsd_desc_t *desc,
		       const nsd_sll_t *sll, uint32_t n, void *rec, uint32_t *ext, uint32_t *ext_count,
		       uint64_t *counters, int *status);

extern "C" int nsd_pipe_submit_sll(nsd_pipe *p, const uint8_t *frames, size_t frames_len,
				   const nsd_desc_t *desc, const nsd_sll_t *sll, uint32_t n, nsd_rec *rec,
				   uint32_t *ext, uint32_t *ext_count, uint64_t *counters, int *status)
{
	if (p && p->compact)
		return NSD_ERR_ARG;
	return pipe_submit(p, frames, frames_len, desc, sll, n, rec, ext, ext_count, counters, status);
}

extern "C" int nsd_pipe_submit_compact(nsd_pipe *p, const uint8_t *frames, size_t frames_len,
				       const nsd_desc_t *desc, const nsd_sll_t *sll, uint32_t n, nsd_crec *crec,
				       uint32_t *ext, uint32_t *ext_count, uint64_t *counters, int *status)
{
	if (p && !p->compact)
		return NSD_ERR_ARG;
	return pipe_submit(p, frames, frames_len, desc, sll, n, crec, ext, ext_count, counters, status);
}

static int pipe_submit(nsd_pipe *p, const uint8_t *frames, size_t frames_len, const nsd_desc_t *desc,
		       const nsd_sll_t *sll, uint32_t n, void *rec, uint32_t *ext, uint32_t *ext_count,
		       uint64_t *counters, int *status)
{
	if (!p || (n && (!frames || !desc || !rec)) || (p->ext_cap && !ext && n))
		return NSD_ERR_ARG;
	if (n > p->max_pkts || frames_len > p->max_bytes)
		return NSD_ERR_ARG;
	const OnDevice on(p->device);
	for (uint32_t i = 0; i < n; i++) {
		const uint64_t cap = NSD_DESC_CAPLEN(desc[i]);
		if (cap > NSD_MAX_CAPLEN)
			return NSD_ERR_CAPLEN;
		if (NSD_DESC_OFF(desc[i]) + cap > frames_len)
			return NSD_ERR_ARG;
	}
	if (p->count == p->depth)
		complete_oldest(p);   // its status goes to its own *status
	const int k = (p->head + p->count) % p->depth;
	Slot &s = p->slot[k];
	s.busy = true;
	s.n = n;
	s.rec_out = rec;
	s.ext_out = ext;
	s.ext_count_out = ext_count;
	s.counters_out = counters;
	s.status_out = status;
	s.status = NSD_OK;
	p->count++;
	const hipStream_t st = s.stream;
	const size_t rb = p->compact ? sizeof(nsd_crec) : sizeof(nsd_rec);
	bool good = ok(hipMemsetAsync(s.small, 0, 64 + NSD_NCOUNTERS * 8, st), "memset");
	if (good && n) {
		good = ok(hipMemcpyAsync(s.frames, frames, frames_len, hipMemcpyHostToDevice, st), "H2D") &&
		       ok(hipMemsetAsync(s.frames + frames_len, 0, NSD_FRAME_PAD, st), "memset") &&
		       ok(hipMemcpyAsync(s.desc, desc, (size_t)n * 8, hipMemcpyHostToDevice, st), "H2D") &&
		       (!sll || ok(hipMemcpyAsync(s.sll, sll, (size_t)n * sizeof(nsd_sll_t), hipMemcpyHostToDevice,
						  st), "H2D"));
		good = good && nsd_launch_dissect_rec(s.frames, s.desc, sll ? s.sll : nullptr, n, p->start_id,
						      p->mode, s.rec, p->compact ? 1 : 0, p->ext_cap ? s.ext : nullptr,
						      p->ext_cap, s.small, (uint64_t *)((uint8_t *)s.small + 64), s.ws, 0,
						      st) == 0;
		good = good && ok(hipMemcpyAsync(rec, s.rec, (size_t)n * rb, hipMemcpyDeviceToHost, st), "D2H");
	}
	good = good && ok(hipMemcpyAsync(s.small_h, s.small, 64 + NSD_NCOUNTERS * 8, hipMemcpyDeviceToHost,
					 st), "D2H") &&
	       ok(hipEventRecord(s.done, st), "event");
	if (!good)
		s.status = NSD_ERR_HIP;
	return good ? NSD_OK : NSD_ERR_HIP;
}

// point an idle pipe at another link type / print mode (the pcap replay keeps
// one pipe for the process, nsd_pcap.cpp); 1 when the pipe lives on another
// device than the current one (the replay then builds a set on this one)
extern "C" __attribute__((visibility("hidden"))) int nsd_pipe_retarget(nsd_pipe *p, int linktype, int mode)
{
	if (!p || p->count || mode < PRINT_NORM || mode > PRINT_NONE)
		return NSD_ERR_ARG;
	int dev = 0;
	if (hipGetDevice(&dev) != hipSuccess)
		return NSD_ERR_HIP;
	if (dev != p->device)
		return 1;
	p->start_id = nsd_start_for(linktype);
	p->mode = mode;
	return NSD_OK;
}

extern "C" void *nsd_host_alloc(size_t len)
{
	void *p = nullptr;
	if (!len || hipHostMalloc(&p, len, hipHostMallocDefault) != hipSuccess)
		return nullptr;
	return p;
}

extern "C" void nsd_host_free(void *ptr)
{
	if (ptr)
		(void)hipHostFree(ptr);
}

extern "C" int nsd_host_register(void *ptr, size_t len)
{
	if (!ptr || !len)
		return NSD_ERR_ARG;
	return hipHostRegister(ptr, len, hipHostRegisterDefault) == hipSuccess ? NSD_OK : NSD_ERR_HIP;
}

extern "C" int nsd_host_unregister(void *ptr)
{
	if (!ptr)
		return NSD_ERR_ARG;
	return hipHostUnregister(ptr) == hipSuccess ? NSD_OK : NSD_ERR_HIP;
}
