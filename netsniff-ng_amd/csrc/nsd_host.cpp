// nsd_host.cpp - C ABI of the batch path (include/netsniff_dissect.h):
// nsd_dissect_device[_ws|_sll] / dissector_entry_batch[_sll] launch the HIP
// kernels of nsd_kernels.hip over a batch of frames.  There is no CPU walk
// behind these entries: without a usable GPU they fail loudly (NSD_ERR_HIP).
// The reference's per-packet surface lives in nsd_proto.cpp.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ioctl.h>
#include <unistd.h>

#include <mutex>
#include <string>

#include "../../include/netsniff_dissect.h"

extern "C" int nsd_launch_dissect_sll(const uint8_t *d_frames, const uint64_t *d_desc, const void *d_sll,
				      uint32_t n, int start_id, int mode, nsd_rec *d_rec, uint32_t *d_ext,
				      uint32_t ext_words, uint32_t *d_ext_used, uint64_t *d_counters,
				      void *d_ws, int grid, hipStream_t stream);
extern "C" int nsd_launch_dissect(const uint8_t *d_frames, const uint64_t *d_desc, uint32_t n,
				  int start_id, int mode, nsd_rec *d_rec, uint32_t *d_ext,
				  uint32_t ext_cap, uint32_t *d_ext_count, uint64_t *d_counters,
				  void *d_ws, int grid, hipStream_t stream);
extern "C" int nsd_launch_dissect_rec(const uint8_t *d_frames, const uint64_t *d_desc, const void *d_sll,
				      uint32_t n, int start_id, int mode, void *d_rec, int compact, uint32_t *d_ext,
				      uint32_t ext_words, uint32_t *d_ext_used, uint64_t *d_counters, void *d_ws,
				      int grid, hipStream_t stream);
extern "C" size_t nsd_launch_workspace_bytes(uint32_t n);

// ---- device context ----------------------------------------------------
namespace {
struct DevCtx {
	std::mutex mu;
	bool init = false;
	int dev = -1;
	int cus = 0;
	hipStream_t stream = nullptr;
	uint8_t *frames = nullptr; size_t frames_cap = 0;
	uint64_t *desc = nullptr; size_t desc_cap = 0;
	nsd_rec *rec = nullptr; size_t rec_cap = 0;
	uint32_t *ext = nullptr; size_t ext_cap = 0;   // ext pool (words)
	uint32_t *ext_count = nullptr;
	uint64_t *counters = nullptr;
	uint8_t *ws = nullptr; size_t ws_cap = 0;          // queue for entry_batch
	uint8_t *dev_ws = nullptr; size_t dev_ws_cap = 0;  // nsd_dissect_device's own
	uint8_t *sll = nullptr; size_t sll_cap = 0;        // per-packet sockaddr_ll (SLL heads)
};
DevCtx g_ctx;

bool hip_ok(hipError_t e, const char *what)
{
	if (e != hipSuccess) {
		fprintf(stderr, "netsniff-dissect: %s: %s\n", what, hipGetErrorString(e));
		return false;
	}
	return true;
}

bool ctx_init(DevCtx &c)
{
	if (c.init)
		return true;
	int n = 0;
	if (!hip_ok(hipGetDeviceCount(&n), "hipGetDeviceCount") || n == 0)
		return false;
	if (!hip_ok(hipGetDevice(&c.dev), "hipGetDevice"))
		return false;
	hipDeviceProp_t prop;
	if (!hip_ok(hipGetDeviceProperties(&prop, c.dev), "hipGetDeviceProperties"))
		return false;
	c.cus = prop.multiProcessorCount;
	if (!hip_ok(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking), "hipStreamCreate"))
		return false;
	if (!hip_ok(hipMalloc(&c.ext_count, 1024), "hipMalloc"))
		return false;
	c.counters = (uint64_t *)((uint8_t *)c.ext_count + 64);
	c.init = true;
	return true;
}

template <class T>
bool grow(T *&p, size_t &cap, size_t need)
{
	if (need <= cap)
		return true;
	if (p)
		(void)hipFree(p);
	p = nullptr;
	size_t want = need + need / 4 + 64;
	if (!hip_ok(hipMalloc(&p, want * sizeof(T)), "hipMalloc"))
		return false;
	cap = want;
	return true;
}

} // namespace

// linktype -> first ops (dissector.c:75-103); shared with nsd_pipe.cpp
__attribute__((visibility("hidden"))) int nsd_start_for(int linktype)
{
	auto is = [&](uint32_t v) { return (uint32_t)linktype == v || (uint32_t)linktype == __builtin_bswap32(v); };
	if (is(NSD_LINKTYPE_EN10MB)) return NSD_OPS_ETHERNET;
	if (is(NSD_LINKTYPE_LINUX_SLL)) return NSD_OPS_SLL;
	if (is(NSD_LINKTYPE_IEEE802_11) || is(NSD_LINKTYPE_IEEE802_11_RADIOTAP)) return NSD_OPS_IEEE80211;
	if (is(NSD_LINKTYPE_NETLINK)) return NSD_OPS_NLMSG;
	return 0;   // unknown link type: start at none_ops (dissector.c:100-103)
}

namespace {
int start_for(int linktype) { return nsd_start_for(linktype); }
} // namespace

// ---- batch extension ---------------------------------------------------
extern "C" size_t nsd_workspace_bytes(uint32_t n) { return nsd_launch_workspace_bytes(n); }

static int check_device_args(const uint8_t *d_frames, const nsd_desc_t *d_desc, const nsd_rec *d_rec,
			     const uint32_t *d_ext, uint32_t ext_cap, const uint32_t *d_ext_count,
			     const uint64_t *d_counters, int mode)
{
	if (!d_frames || !d_desc || !d_rec || !d_ext_count || !d_counters)
		return NSD_ERR_ARG;
	if (ext_cap && !d_ext)
		return NSD_ERR_ARG;
	if (mode < PRINT_NORM || mode > PRINT_NONE)
		return NSD_ERR_ARG;
	return NSD_OK;
}

extern "C" int nsd_dissect_device_ws(const uint8_t *d_frames, const nsd_desc_t *d_desc, uint32_t n,
				     int linktype, int mode, nsd_rec *d_rec, uint32_t *d_ext,
				     uint32_t ext_cap, uint32_t *d_ext_count, uint64_t *d_counters,
				     void *d_workspace, void *stream)
{
	if (n == 0)
		return NSD_OK;
	int rc = check_device_args(d_frames, d_desc, d_rec, d_ext, ext_cap, d_ext_count, d_counters, mode);
	if (rc || !d_workspace)
		return rc ? rc : NSD_ERR_ARG;
	rc = nsd_launch_dissect(d_frames, d_desc, n, start_for(linktype), mode, d_rec, d_ext, ext_cap,
				d_ext_count, d_counters, d_workspace, 0, (hipStream_t)stream);
	return rc ? NSD_ERR_HIP : NSD_OK;
}

// grid override for experiments (0 = default)
extern "C" int nsd_dissect_device_grid(const uint8_t *d_frames, const nsd_desc_t *d_desc,
				       uint32_t n, int linktype, int mode, nsd_rec *d_rec,
				       uint32_t *d_ext, uint32_t ext_cap, uint32_t *d_ext_count,
				       uint64_t *d_counters, void *d_workspace, int grid, void *stream)
{
	if (n == 0)
		return NSD_OK;
	int rc = check_device_args(d_frames, d_desc, d_rec, d_ext, ext_cap, d_ext_count, d_counters, mode);
	if (rc || !d_workspace)
		return rc ? rc : NSD_ERR_ARG;
	rc = nsd_launch_dissect(d_frames, d_desc, n, start_for(linktype), mode, d_rec, d_ext, ext_cap,
				d_ext_count, d_counters, d_workspace, grid, (hipStream_t)stream);
	return rc ? NSD_ERR_HIP : NSD_OK;
}

// Without a caller workspace the library keeps one per process (allocated on
// first use and grown on demand: that call is not graph-capturable).
extern "C" int nsd_dissect_device(const uint8_t *d_frames, const nsd_desc_t *d_desc, uint32_t n,
				  int linktype, int mode, nsd_rec *d_rec, uint32_t *d_ext,
				  uint32_t ext_cap, uint32_t *d_ext_count, uint64_t *d_counters,
				  void *stream)
{
	if (n == 0)
		return NSD_OK;
	int rc = check_device_args(d_frames, d_desc, d_rec, d_ext, ext_cap, d_ext_count, d_counters, mode);
	if (rc)
		return rc;
	DevCtx &c = g_ctx;
	std::lock_guard<std::mutex> lk(c.mu);
	if (!grow(c.dev_ws, c.dev_ws_cap, nsd_launch_workspace_bytes(n)))
		return NSD_ERR_NOMEM;
	rc = nsd_launch_dissect(d_frames, d_desc, n, start_for(linktype), mode, d_rec, d_ext, ext_cap,
				d_ext_count, d_counters, c.dev_ws, 0, (hipStream_t)stream);
	return rc ? NSD_ERR_HIP : NSD_OK;
}

extern "C" int nsd_dissect_device_sll(const uint8_t *d_frames, const nsd_desc_t *d_desc,
				      const nsd_sll_t *d_sll, uint32_t n, int linktype, int mode,
				      nsd_rec *d_rec, uint32_t *d_ext, uint32_t ext_cap,
				      uint32_t *d_ext_count, uint64_t *d_counters, void *d_workspace,
				      void *stream)
{
	if (n == 0)
		return NSD_OK;
	int rc = check_device_args(d_frames, d_desc, d_rec, d_ext, ext_cap, d_ext_count, d_counters, mode);
	if (rc || !d_workspace)
		return rc ? rc : NSD_ERR_ARG;
	rc = nsd_launch_dissect_sll(d_frames, d_desc, d_sll, n, start_for(linktype), mode, d_rec, d_ext,
				    ext_cap, d_ext_count, d_counters, d_workspace, 0, (hipStream_t)stream);
	return rc ? NSD_ERR_HIP : NSD_OK;
}

extern "C" int nsd_dissect_device_compact(const uint8_t *d_frames, const nsd_desc_t *d_desc,
					  const nsd_sll_t *d_sll, uint32_t n, int linktype, int mode,
					  nsd_crec *d_crec, uint32_t *d_ext, uint32_t ext_words,
					  uint32_t *d_ext_used, uint64_t *d_counters, void *d_workspace,
					  void *stream)
{
	if (n == 0)
		return NSD_OK;
	int rc = check_device_args(d_frames, d_desc, (const nsd_rec *)d_crec, d_ext, ext_words, d_ext_used,
				   d_counters, mode);
	if (rc || !d_workspace)
		return rc ? rc : NSD_ERR_ARG;
	rc = nsd_launch_dissect_rec(d_frames, d_desc, d_sll, n, start_for(linktype), mode, d_crec, 1, d_ext,
				    ext_words, d_ext_used, d_counters, d_workspace, 0, (hipStream_t)stream);
	return rc ? NSD_ERR_HIP : NSD_OK;
}

extern "C" int dissector_entry_batch(const uint8_t *frames, size_t frames_len,
				     const nsd_desc_t *desc, uint32_t n, int linktype, int mode,
				     nsd_rec *rec, uint32_t *ext, uint32_t ext_cap,
				     uint32_t *ext_count, uint64_t *counters)
{
	return dissector_entry_batch_sll(frames, frames_len, desc, nullptr, n, linktype, mode, rec, ext,
					 ext_cap, ext_count, counters);
}

extern "C" int dissector_entry_batch_sll(const uint8_t *frames, size_t frames_len,
					 const nsd_desc_t *desc, const nsd_sll_t *sll, uint32_t n,
					 int linktype, int mode, nsd_rec *rec, uint32_t *ext,
					 uint32_t ext_cap, uint32_t *ext_count, uint64_t *counters)
{
	if (n == 0)
		return NSD_OK;
	if (!frames || !desc || !rec || (ext_cap && !ext))
		return NSD_ERR_ARG;
	for (uint32_t i = 0; i < n; i++) {
		if (NSD_DESC_CAPLEN(desc[i]) > NSD_MAX_CAPLEN)
			return NSD_ERR_CAPLEN;
		if (NSD_DESC_OFF(desc[i]) + NSD_DESC_CAPLEN(desc[i]) > frames_len)
			return NSD_ERR_ARG;
	}
	DevCtx &c = g_ctx;
	std::lock_guard<std::mutex> lk(c.mu);
	if (!ctx_init(c))
		return NSD_ERR_HIP;
	if (!grow(c.frames, c.frames_cap, frames_len + NSD_FRAME_PAD) || !grow(c.desc, c.desc_cap, n) ||
	    !grow(c.rec, c.rec_cap, n) || (ext_cap && !grow(c.ext, c.ext_cap, ext_cap)) ||
	    !grow(c.ws, c.ws_cap, nsd_launch_workspace_bytes(n)) ||
	    (sll && !grow(c.sll, c.sll_cap, (size_t)n * sizeof(nsd_sll_t))))
		return NSD_ERR_NOMEM;
	hipStream_t s = c.stream;
	if (sll && !hip_ok(hipMemcpyAsync(c.sll, sll, (size_t)n * sizeof(nsd_sll_t), hipMemcpyHostToDevice, s),
			   "H2D"))
		return NSD_ERR_HIP;
	bool ok = hip_ok(hipMemcpyAsync(c.frames, frames, frames_len, hipMemcpyHostToDevice, s), "H2D") &&
		  hip_ok(hipMemsetAsync(c.frames + frames_len, 0, NSD_FRAME_PAD, s), "memset") &&
		  hip_ok(hipMemcpyAsync(c.desc, desc, n * sizeof(uint64_t), hipMemcpyHostToDevice, s), "H2D") &&
		  hip_ok(hipMemsetAsync(c.ext_count, 0, 64 + NSD_NCOUNTERS * 8, s), "memset");
	if (!ok)
		return NSD_ERR_HIP;
	if (nsd_launch_dissect_sll(c.frames, c.desc, sll ? c.sll : nullptr, n, start_for(linktype), mode, c.rec,
				   ext_cap ? c.ext : nullptr, ext_cap, c.ext_count, c.counters, c.ws, 0, s))
		return NSD_ERR_HIP;
	uint32_t used = 0;
	ok = hip_ok(hipMemcpyAsync(rec, c.rec, n * sizeof(nsd_rec), hipMemcpyDeviceToHost, s), "D2H") &&
	     hip_ok(hipMemcpyAsync(&used, c.ext_count, 4, hipMemcpyDeviceToHost, s), "D2H");
	if (ok && counters)
		ok = hip_ok(hipMemcpyAsync(counters, c.counters, NSD_NCOUNTERS * 8, hipMemcpyDeviceToHost, s), "D2H");
	ok = ok && hip_ok(hipStreamSynchronize(s), "sync");
	if (ok && ext_cap) {
		uint32_t k = used < ext_cap ? used : ext_cap;
		if (k)
			ok = hip_ok(hipMemcpy(ext, c.ext, (size_t)k * 4, hipMemcpyDeviceToHost), "D2H");
	}
	if (ext_count)
		*ext_count = used;
	return ok ? NSD_OK : NSD_ERR_HIP;
}

// __tprintf_flush (tprintf.c:65-103) applied to one flushed buffer
extern "C" long nsd_tprintf_wrap(const char *in, size_t len, int cols, long *state, char *out,
				 size_t cap)
{
	const long term_start = 3;
	long term_len = cols - 5;
	long line_count = state ? *state : 0;
	long color_open = 0;
	size_t o = 0;
	if (!out || cap < 2 * len + 16)
		return NSD_ERR_ARG;
	for (size_t i = 0; i < len; ++i) {
		if (in[i] == '\n') {
			term_len = cols - 5;
			line_count = -1;
		}
		if (in[i] == 033 && i + 1 < len && in[i + 1] == '[')
			color_open++;
		if (color_open == 0 && line_count >= term_len) {
			out[o++] = '\n';
			for (long k = 0; k < term_start; k++)
				out[o++] = ' ';
			line_count = term_start;
			while (i < len && (in[i] == ' ' || in[i] == ','))
				i++;
		}
		// at i == len the reference reads buffer[buffer_use], the NUL that
		// vsnprintf left there
		const char ch = i < len ? in[i] : '\0';
		if (color_open > 0 && ch == 'm')
			color_open--;
		out[o++] = ch;
		line_count++;
	}
	if (state)
		*state = line_count;
	return (long)o;
}

// the device context of the host-memory batch entry (dissector_cleanup_all
// frees it, nsd_proto.cpp)
extern "C" __attribute__((visibility("hidden"))) void nsd_device_ctx_release(void)
{
	DevCtx &c = g_ctx;
	std::lock_guard<std::mutex> lk(c.mu);
	if (!c.init)
		return;
	(void)hipFree(c.frames); (void)hipFree(c.desc); (void)hipFree(c.rec); (void)hipFree(c.ext);
	(void)hipFree(c.ext_count); (void)hipFree(c.ws); (void)hipFree(c.dev_ws); (void)hipFree(c.sll);
	c.ws = c.dev_ws = nullptr;
	c.ws_cap = c.dev_ws_cap = 0;
	(void)hipStreamDestroy(c.stream);
	c.frames = nullptr; c.desc = nullptr; c.rec = nullptr; c.ext = nullptr; c.sll = nullptr;
	c.frames_cap = c.desc_cap = c.rec_cap = c.ext_cap = c.sll_cap = 0;
	c.ext_count = nullptr; c.counters = nullptr; c.stream = nullptr;
	c.init = false;
}

extern "C" const char *nsd_version(void) { return "netsniff-dissect 0.2 (gfx950)"; }

#ifndef NSD_BUILD_INFO
#define NSD_BUILD_INFO "unknown"
#endif
extern "C" const char *nsd_build_info(void) { return NSD_BUILD_INFO; }

extern "C" int nsd_device_count(void)
{
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess)
		return 0;
	return n;
}
