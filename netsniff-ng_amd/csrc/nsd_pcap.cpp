// nsd_pcap.cpp - the pcap replay front end of the dissector path
// (`netsniff-ng --in file.pcap`, read_pcap netsniff-ng.c:640-770): a pcap
// reader that packs records into batches (frames + nsd_desc_t), and a replay
// driver that feeds them through the optional device BPF filter and the
// pipelined device walk (nsd_pipe_*) and writes the formatted text.
//
// Reader semantics follow pcap_io.h and pcap_sg.c:
//   - file header validation and the *_LL remap for SLL / netlink files
//     (pcap_validate_header, pcap_io.h:874-908); the link type handed to the
//     dissector is the header field as stored, so a byte-swapped file passes
//     a byte-swapped link type (pcap_generic_pull_fhdr :910-928), which the
//     entry point matches either way (dissector.c:79);
//   - record header sizes per format (pcap_get_hdr_length :429-452: 16 for
//     usec / nsec, 32 for the *_LL forms whose 16-byte cooked header is not
//     packet data, 24 for the Kuznetzov / Borkmann forms), the caplen field
//     byte-swapped for swapped files and minus 16 for *_LL
//     (pcap_get_length :322-352);
//   - a record with caplen 0 or above the 1 MiB replay buffer ends the
//     replay, as pcap_sg_read's -EINVAL does (pcap_sg.c:121-123), and so
//     does a short read at the end of the file;
//   - a record longer than a batch can carry (NSD_MAX_CAPLEN < caplen <=
//     1 MiB: tcpdump's default snaplen is 262144, GRO frames are long) ends
//     the batch before it; the batch reader reports NSD_ERR_CAPLEN when it
//     is the next record, and the replay dissects it through the per-packet
//     path (nsd_proto.cpp), in file order.
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/uio.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/netsniff_dissect.h"

namespace nsd {
void format_frame_hdr(std::string &s, const nsd_frame_hdr_t &fh, const nsd_sll_t *sll, const uint8_t *pkt,
		      uint32_t caplen, int linktype, int mode, uint64_t count);
int render_packet_cpu(std::string &text, const uint8_t *packet, size_t len, int linktype, int mode,
		      const nsd_sll_t *sll);
int format_replay_part(std::string &s, const uint8_t *frames, const nsd_desc_t *desc, const nsd_frame_hdr_t *fh,
		       const nsd_sll_t *sll, const nsd_crec *rec, const uint32_t *ext, uint64_t count0, uint32_t lo,
		       uint32_t hi, int linktype, int mode);
int format_packet_compact(std::string &s, const uint8_t *pkt, uint32_t caplen, int linktype, int mode,
			  const nsd_crec &rec, uint32_t i, const uint32_t *ext_pool, const nsd_sll_t *sll);
void cpu_count_packet(const uint8_t *pkt, uint32_t caplen, int linktype, int mode, const nsd_sll_t *sll,
		      uint64_t *counters);
}

extern "C" __attribute__((visibility("hidden"))) int nsd_pipe_retarget(nsd_pipe *p, int linktype, int mode);

namespace {

constexpr uint32_t TCPDUMP = 0xa1b2c3d4, NSEC = 0xa1b23c4d, KUZ = 0xa1b2cd34, BKM = 0xa1e2cb12;
constexpr uint32_t LT_LINUX_SLL = 113, LT_NETLINK = 253;
constexpr uint32_t REPLAY_BUF = 1024 * 1024;   // read_pcap's `out` buffer (netsniff-ng.c:680)

uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }
uint16_t bswap16(uint16_t v) { return __builtin_bswap16(v); }

} // namespace

struct nsd_pcap {
	int fd = -1;
	bool swapped = false;
	uint32_t hdrsize = 16;   // record header bytes (pcap_get_hdr_length)
	uint32_t ll_extra = 0;   // cooked-header bytes counted in caplen (*_LL)
	uint32_t linktype = 0;   // as stored in the file header
	uint32_t magic_raw = 0;  // as stored in the file header
	uint32_t magic = 0;      // in host order
	bool nsec = false;
	bool eof = false;
	// buffered reader (the scatter-gather reader's iovecs, pcap_sg.c), or a
	// regular file mapped whole (pcap_mm.c's way; the replay's reader then
	// only scans the record headers and the pool copies the bodies)
	std::vector<uint8_t> buf;
	const uint8_t *map = nullptr;
	size_t pos = 0, len = 0;
	// a mapped file's record index, one window at a time (RecIndex below):
	// the records' header offsets and caplens, ix_i the next one; ix_end =
	// the walk ended inside the indexed window (no records past the last)
	std::vector<uint64_t> ix_off;
	std::vector<uint32_t> ix_cap;
	size_t ix_i = 0;
	bool ix_end = false;

	const uint8_t *data() const { return map ? map : buf.data(); }
	bool fill(size_t need)
	{
		if (len - pos >= need)
			return true;
		if (map)
			return false;
		if (pos) {
			memmove(buf.data(), buf.data() + pos, len - pos);
			len -= pos;
			pos = 0;
		}
		if (buf.size() < need)
			buf.resize(need);
		while (len < need) {
			ssize_t r = read(fd, buf.data() + len, buf.size() - len);
			if (r < 0 && errno == EINTR)
				continue;
			if (r <= 0)
				return false;
			len += (size_t)r;
		}
		return true;
	}
};

extern "C" nsd_pcap *nsd_pcap_open(const char *path)
{
	if (!path)
		return nullptr;
	int fd = open(path, O_RDONLY);
	if (fd < 0)
		return nullptr;
	nsd_pcap *p = new nsd_pcap;
	p->fd = fd;
	struct stat sb;
	const char *mm = getenv("NSD_PCAP_MMAP");
	if (!(mm && mm[0] == '0') && fstat(fd, &sb) == 0 && S_ISREG(sb.st_mode) && sb.st_size >= 24) {
		void *m = mmap(nullptr, (size_t)sb.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
		if (m != MAP_FAILED) {
			(void)madvise(m, (size_t)sb.st_size, MADV_SEQUENTIAL);
			p->map = (const uint8_t *)m;
			p->len = (size_t)sb.st_size;
		}
	}
	if (!p->map)
		p->buf.resize(4 << 20);
	uint8_t h[24];
	if (!p->fill(24)) {
		nsd_pcap_close(p);
		return nullptr;
	}
	memcpy(h, p->data(), 24);
	p->pos = 24;
	uint32_t magic, lt;
	memcpy(&magic, h, 4);
	memcpy(&lt, h + 20, 4);
	uint16_t vmaj, vmin;
	memcpy(&vmaj, h + 4, 2);
	memcpy(&vmin, h + 6, 2);
	// pcap_check_magic (pcap_io.h:286-320)
	p->magic_raw = magic;
	uint32_t m = magic;
	if (m == bswap32(TCPDUMP) || m == bswap32(NSEC) || m == bswap32(KUZ) || m == bswap32(BKM)) {
		p->swapped = true;
		m = bswap32(m);
	}
	if (m != TCPDUMP && m != NSEC && m != KUZ && m != BKM) {
		nsd_pcap_close(p);
		return nullptr;
	}
	// pcap_validate_header: version 2.4 in either byte order
	if ((vmaj != 2 && bswap16(vmaj) != 2) || (vmin != 4 && bswap16(vmin) != 4)) {
		nsd_pcap_close(p);
		return nullptr;
	}
	const uint32_t lt_host = p->swapped ? bswap32(lt) : lt;
	p->linktype = lt;
	p->magic = m;
	p->nsec = m == NSEC || m == BKM;
	if (m == KUZ || m == BKM) {
		p->hdrsize = 24;
	} else if (lt_host == LT_LINUX_SLL || lt_host == LT_NETLINK) {
		p->hdrsize = 32;   // *_LL: the cooked header follows the record header
		p->ll_extra = 16;
	}
	return p;
}

extern "C" int nsd_pcap_linktype(const nsd_pcap *p) { return p ? (int)p->linktype : -1; }

extern "C" void nsd_pcap_close(nsd_pcap *p)
{
	if (!p)
		return;
	if (p->map)
		munmap((void *)p->map, p->len);
	if (p->fd >= 0)
		close(p->fd);
	delete p;
}

// Read up to max_n records into frames[0, cap): frames packed at 16-byte
// aligned offsets (TPACKET_ALIGNMENT, as in the RX ring), NSD_FRAME_PAD bytes
// kept free past the last one.  desc[k] = NSD_DESC(offset, caplen);
// wire_len[k] (may be NULL) = the record's original length, ts_ns[k] (may be
// NULL) = its timestamp in ns.  Returns the records read (0 at the end of the
// replay), or NSD_ERR_ARG.
extern "C" long nsd_pcap_read_batch(nsd_pcap *p, uint8_t *frames, size_t cap, nsd_desc_t *desc,
				    uint32_t max_n, uint32_t *wire_len, uint64_t *ts_ns)
{
	return nsd_pcap_read_batch_sll(p, frames, cap, desc, nullptr, max_n, wire_len, ts_ns);
}

// What read_pcap's pcap_pkthdr_to_tpacket_hdr (pcap_io.h:594-709) makes of
// one record header h (as stored) in its frame_map, zeroed once
// (netsniff-ng.c:672) and overwritten field by field per record:
//   tp_sec = ts.tv_sec; tp_nsec = tv_usec * 1000 (usec, *_LL, Kuznetzov) or
//   the ns field (nsec, Borkmann); tp_len = len, minus the cooked header for
//   *_LL; all byte-swapped for swapped files (the usec product in 32 bits);
//   sll: the cooked header (*_LL: ll_to_sockaddr, pcap_io.h:182-191:
//   pkttype / hatype / halen from be16, protocol as stored, addr), or the
//   Kuznetzov ifindex / protocol / pkttype, or the Borkmann ifindex (u16) /
//   protocol / hatype / pkttype; every other field stays 0.
static void record_meta(const nsd_pcap *p, const uint8_t *h, nsd_sll_t *sll, nsd_frame_hdr_t *fh)
{
	const bool sw = p->swapped;
	auto r32 = [&](int o) { uint32_t v; memcpy(&v, h + o, 4); return sw ? bswap32(v) : v; };
	auto r16 = [&](int o) { uint16_t v; memcpy(&v, h + o, 2); return sw ? bswap16(v) : v; };
	if (fh) {
		memset(fh, 0, sizeof(*fh));
		fh->sec = r32(0);
		const uint32_t frac = r32(4);
		fh->nsec = p->nsec ? frac : frac * 1000u;
		fh->len = r32(12) - p->ll_extra;
	}
	if (!sll)
		return;
	nsd_sll_t ll;
	memset(&ll, 0, sizeof(ll));
	if (p->ll_extra) {
		const uint8_t *c = h + 16;   // struct pcap_ll, big-endian fields
		ll.pkttype = (uint8_t)(((uint32_t)c[0] << 8) | c[1]);
		ll.hatype = (uint16_t)(((uint32_t)c[2] << 8) | c[3]);
		ll.halen = (uint8_t)(((uint32_t)c[4] << 8) | c[5]);
		memcpy(ll.addr, c + 6, 8);
		memcpy(&ll.protocol, c + 14, 2);
	} else if (p->magic == KUZ) {
		// struct pcap_pkthdr_kuz {ts, caplen, len, u32 ifindex, u16 protocol, u8 pkttype}
		ll.ifindex = (int32_t)r32(16);
		ll.protocol = r16(20);
		ll.pkttype = h[22];
	} else if (p->magic == BKM) {
		// struct pcap_pkthdr_bkm {ts, caplen, len, u16 tsource, u16 ifindex,
		// u16 protocol, u8 hatype, u8 pkttype}
		ll.ifindex = r16(18);
		ll.protocol = r16(20);
		ll.hatype = h[22];
		ll.pkttype = h[23];
	}
	*sll = ll;
}

// same, also filling sll[k] (may be NULL) the way read_pcap fills fm.s_ll
// (netsniff-ng.c:672, 727): zeroed once, then for *_LL records
// pcap_pkthdr_to_tpacket_hdr -> ll_to_sockaddr (pcap_io.h:182-191, 594-660)
// from the cooked header after the record header (struct pcap_ll
// {pkttype, hatype, len, addr[8], protocol}, every field big-endian in either
// file byte order): pkttype / hatype / halen from be16, protocol kept as
// stored (be16), addr copied; family and ifindex stay 0.
static long read_batch(nsd_pcap *p, uint8_t *frames, size_t cap, nsd_desc_t *desc, nsd_sll_t *sll,
		       nsd_frame_hdr_t *fh, uint32_t max_n, uint32_t *wire_len, uint64_t *ts_ns, uint8_t *rhdr);

extern "C" long nsd_pcap_read_batch_sll(nsd_pcap *p, uint8_t *frames, size_t cap, nsd_desc_t *desc,
					nsd_sll_t *sll, uint32_t max_n, uint32_t *wire_len, uint64_t *ts_ns)
{
	return read_batch(p, frames, cap, desc, sll, nullptr, max_n, wire_len, ts_ns, nullptr);
}

extern "C" long nsd_pcap_read_batch_fh(nsd_pcap *p, uint8_t *frames, size_t cap, nsd_desc_t *desc,
				       nsd_sll_t *sll, nsd_frame_hdr_t *fh, uint32_t max_n)
{
	return read_batch(p, frames, cap, desc, sll, fh, max_n, nullptr, nullptr, nullptr);
}

// rhdr (may be NULL): each record's header bytes as stored (hdrsize <= 32,
// 32-byte stride), for the pcap write-out
static long read_batch(nsd_pcap *p, uint8_t *frames, size_t cap, nsd_desc_t *desc, nsd_sll_t *sll,
		       nsd_frame_hdr_t *fh, uint32_t max_n, uint32_t *wire_len, uint64_t *ts_ns, uint8_t *rhdr)
{
	if (!p || !frames || !desc || cap < NSD_FRAME_PAD)
		return NSD_ERR_ARG;
	size_t off = 0;
	uint32_t n = 0;
	while (n < max_n && !p->eof) {
		if (!p->fill(p->hdrsize)) {
			p->eof = true;
			break;
		}
		const uint8_t *h = p->data() + p->pos;
		uint32_t sec, frac, cl, wl;
		memcpy(&sec, h, 4);
		memcpy(&frac, h + 4, 4);
		memcpy(&cl, h + 8, 4);
		memcpy(&wl, h + 12, 4);
		if (p->swapped) {
			sec = bswap32(sec);
			frac = bswap32(frac);
			cl = bswap32(cl);
			wl = bswap32(wl);
		}
		const uint32_t caplen = cl - p->ll_extra;   // unsigned, as the reference computes it
		if (caplen == 0 || caplen > REPLAY_BUF) {
			p->eof = true;   // pcap_sg_read: -EINVAL ends read_pcap's loop
			break;
		}
		if (caplen > NSD_MAX_CAPLEN) {
			if (n == 0)
				return NSD_ERR_CAPLEN;   // the next record does not fit a batch
			break;
		}
		const size_t at = (off + 15) & ~(size_t)15;
		if (at + caplen + NSD_FRAME_PAD > cap) {
			if (n == 0)
				return NSD_ERR_ARG;   // one record does not fit the batch buffer
			break;                        // next batch
		}
		if (!p->fill((size_t)p->hdrsize + caplen)) {
			p->eof = true;
			break;
		}
		h = p->data() + p->pos;
		memcpy(frames + at, h + p->hdrsize, caplen);
		p->pos += p->hdrsize + caplen;
		desc[n] = NSD_DESC(at, caplen);
		if (rhdr)
			memcpy(rhdr + 32 * (size_t)n, h, p->hdrsize);
		if (sll || fh)
			record_meta(p, h, sll ? sll + n : nullptr, fh ? fh + n : nullptr);
		if (wire_len)
			wire_len[n] = wl;
		if (ts_ns)
			ts_ns[n] = (uint64_t)sec * 1000000000ull + (p->nsec ? frac : (uint64_t)frac * 1000ull);
		off = at + caplen;
		n++;
	}
	memset(frames + off, 0, NSD_FRAME_PAD);
	return n;
}

// A mapped file's next batch, as read_batch lays it out (same checks, same
// stops), without touching the bodies: desc[k] = the record's place in the
// batch buffer, src[k] = its header's offset in the file.  fill_range copies
// a range of the batch afterwards (the replay runs those on its pool).
// *end = the bytes the batch uses.
static long scan_batch(nsd_pcap *p, size_t cap, nsd_desc_t *desc, uint64_t *src, uint32_t max_n, size_t *end)
{
	size_t off = 0;
	uint32_t n = 0;
	const uint32_t hs = p->hdrsize;
	*end = 0;
	if (p->eof)
		return 0;
	// (a record read past the index by read_one)
	while (p->ix_i < p->ix_off.size() && p->ix_off[p->ix_i] < p->pos)
		p->ix_i++;
	// (locals: the stores to desc / src could alias p's fields)
	const uint64_t *const ixo = p->ix_off.data();
	const uint32_t *const ixc = p->ix_cap.data();
	const size_t ixn = p->ix_off.size();
	size_t i = p->ix_i;
	long rc = 0;
	while (n < max_n) {
		if (i == ixn) {
			if (p->ix_end)
				p->eof = true;
			break;   // (the caller builds the next window)
		}
		const uint32_t caplen = ixc[i];
		if (caplen > NSD_MAX_CAPLEN) {
			if (n == 0)
				rc = NSD_ERR_CAPLEN;
			break;
		}
		const size_t at = (off + 15) & ~(size_t)15;
		if (at + caplen + NSD_FRAME_PAD > cap) {
			if (n == 0)
				rc = NSD_ERR_ARG;
			break;
		}
		src[n] = ixo[i];
		desc[n] = NSD_DESC(at, caplen);
		i++;
		off = at + caplen;
		n++;
	}
	if (n) {
		p->pos = ixo[i - 1] + hs + ixc[i - 1];
		p->ix_i = i;
	}
	*end = off;
	return rc ? rc : n;
}

// the index window under p->pos is used up (and the walk goes on)
static bool ix_need(const nsd_pcap *p)
{
	size_t i = p->ix_i;
	while (i < p->ix_off.size() && p->ix_off[i] < p->pos)
		i++;
	return i == p->ix_off.size() && !p->ix_end && !p->eof;
}

static void fill_range(const nsd_pcap *p, uint8_t *frames, const nsd_desc_t *desc, const uint64_t *src,
		       uint32_t lo, uint32_t hi, nsd_sll_t *sll, nsd_frame_hdr_t *fh, uint8_t *rhdr)
{
	const uint32_t hs = p->hdrsize;
	for (uint32_t k = lo; k < hi; k++) {
		const uint8_t *h = p->map + src[k];
		memcpy(frames + NSD_DESC_OFF(desc[k]), h + hs, NSD_DESC_CAPLEN(desc[k]));
		if (rhdr)
			memcpy(rhdr + 32 * (size_t)k, h, hs);
		record_meta(p, h, sll + k, fh + k);
	}
}

// ---- a mapped file's record index, built in parallel ----------------------
// The record walk (each header's caplen gives the next header) is one
// dependent load per record: walked by one thread it bounds the replay's
// reader (a 64-byte frame every 80 bytes touches every line of the file).
// A window of the file is cut into chunks; chunk 0 is walked from the exact
// record start, every later chunk from a guess (the first offset from which
// several headers in a row look like records); the exact walk then runs
// through the chunks' results: the exact offset X where it enters chunk c is
// looked up among the offsets chunk c visited, and from there chunk c's walk
// IS the exact walk (a walk is determined by its start).  A chunk whose walk
// never met X (a wrong guess that did not fall into step) is walked again
// from X.  The end rule is read_batch's: a header past the file end, caplen 0
// or > the 1 MiB replay buffer, or a body past the file end ends the walk.
struct IxChunk {
	std::vector<uint64_t> off;
	std::vector<uint32_t> cap;
	size_t next = 0;     // where the walk stopped (its last record's end)
	bool ended = false;  // stopped by the end rule, not at the chunk's end
};

// caplen of the header at pos, or 0 when the end rule stops there
static uint32_t rec_caplen(const nsd_pcap *p, size_t pos)
{
	const uint32_t hs = p->hdrsize;
	if (p->len - pos < hs)
		return 0;
	uint32_t cl;
	memcpy(&cl, p->map + pos + 8, 4);
	if (p->swapped)
		cl = bswap32(cl);
	const uint32_t caplen = cl - p->ll_extra;
	if (caplen == 0 || caplen > REPLAY_BUF || p->len - pos - hs < caplen)
		return 0;
	return caplen;
}

// the walk from pos while pos < stop_at, appended to c
static void ix_walk(const nsd_pcap *p, size_t pos, size_t stop_at, IxChunk &c)
{
	const uint32_t hs = p->hdrsize;
	c.ended = false;
	while (pos < stop_at) {
		if (p->len - pos > 4096 + 64)
			__builtin_prefetch(p->map + pos + 4096);
		const uint32_t caplen = rec_caplen(p, pos);
		if (!caplen) {
			c.ended = true;
			break;
		}
		c.off.push_back(pos);
		c.cap.push_back(caplen);
		pos += hs + caplen;
	}
	c.next = pos;
}

// a record start for a walk from inside [lo, hi): the first offset whose next
// 8 headers pass the end rule with a plausible fraction-of-second field (or
// reach the file end exactly); hi when there is none
static size_t ix_guess(const nsd_pcap *p, size_t lo, size_t hi)
{
	const uint32_t hs = p->hdrsize;
	const uint32_t frac_max = p->nsec ? 1000000000u : 1000000u;
	for (size_t o = lo; o < hi; o++) {
		size_t q = o;
		int k = 0;
		for (; k < 8; k++) {
			if (q == p->len)
				break;
			const uint32_t caplen = rec_caplen(p, q);
			if (!caplen)
				break;
			uint32_t frac;
			memcpy(&frac, p->map + q + 4, 4);
			if ((p->swapped ? bswap32(frac) : frac) >= frac_max)
				break;
			q += hs + caplen;
		}
		if (k == 8 || (k > 0 && q == p->len))
			return o;
	}
	return hi;
}

// chunk c of the window [b[0], b[nc]): walked from its guess to b[c + 1]
static void ix_chunk(const nsd_pcap *p, const std::vector<size_t> &b, int c, IxChunk &out)
{
	out.off.clear();
	out.cap.clear();
	const size_t from = c == 0 ? b[0] : ix_guess(p, b[c], b[c + 1]);
	out.next = from;
	out.ended = false;
	if (from < b[c + 1])
		ix_walk(p, from, b[c + 1], out);
}

// the window's chunk bounds from the exact record start `start`
static std::vector<size_t> ix_bounds(const nsd_pcap *p, size_t start, size_t window, int nc)
{
	const size_t end = p->len - start < window ? p->len : start + window;
	std::vector<size_t> b(nc + 1);
	for (int c = 0; c <= nc; c++)
		b[c] = start + (end - start) * (size_t)c / (size_t)nc;
	b[nc] = end;
	return b;
}

// the exact walk through the chunks' results into p's index
static void ix_splice(nsd_pcap *p, const std::vector<size_t> &b, std::vector<IxChunk> &ch)
{
	const int nc = (int)ch.size();
	p->ix_off.clear();
	p->ix_cap.clear();
	p->ix_i = 0;
	p->ix_end = false;
	size_t x = b[0];
	for (int c = 0; c < nc; c++) {
		if (x >= b[c + 1])
			continue;   // a record across the whole chunk
		IxChunk &k = ch[c];
		const auto it = std::lower_bound(k.off.begin(), k.off.end(), (uint64_t)x);
		if (!(it != k.off.end() && *it == x) && !(k.ended && k.next == x)) {
			// the guess never fell into step: walk the chunk again from x
			k.off.clear();
			k.cap.clear();
			ix_walk(p, x, b[c + 1], k);
			p->ix_off.insert(p->ix_off.end(), k.off.begin(), k.off.end());
			p->ix_cap.insert(p->ix_cap.end(), k.cap.begin(), k.cap.end());
		} else {
			const size_t i = (size_t)(it - k.off.begin());
			p->ix_off.insert(p->ix_off.end(), k.off.begin() + (long)i, k.off.end());
			p->ix_cap.insert(p->ix_cap.end(), k.cap.begin() + (long)i, k.cap.end());
		}
		x = k.next;
		if (k.ended) {
			p->ix_end = true;
			return;
		}
	}
	// the window reached the file end: the walk ends there
	if (b[nc] == p->len && x >= p->len)
		p->ix_end = true;
}

// the index window from p->pos, chunks run by run(nc, fn) (fn(c) for each
// chunk c, in any order and on any threads)
template <class Run>
static void ix_build(nsd_pcap *p, size_t window, int nc, std::vector<IxChunk> &ch, Run run)
{
	const std::vector<size_t> b = ix_bounds(p, p->pos, window, nc);
	if ((int)ch.size() != nc)
		ch.resize(nc);
	run(nc, std::function<void(int)>([&](int c) { ix_chunk(p, b, c, ch[c]); }));
	ix_splice(p, b, ch);
}

// the index window (bytes of file per build; NSD_PCAP_IX_WINDOW overrides,
// for tests)
static size_t ix_window()
{
	const char *e = getenv("NSD_PCAP_IX_WINDOW");
	const long long v = e ? atoll(e) : 0;
	return v > 0 ? (size_t)v : (size_t)16 << 20;
}

// The record index of a mapped file (the replay reader's, windows of
// `window` bytes, 0 = the replay's, cut into `chunks` walked from guesses and
// spliced): the first max_n records' header offsets and caplens into off /
// caplen.  Returns the records the walk finds (read_batch's end rule), or
// NSD_ERR_ARG (not a pcap file, or not a regular file).
extern "C" long nsd_pcap_index(const char *path, uint64_t window, int chunks, uint64_t *off, uint32_t *caplen,
			       size_t max_n)
{
	nsd_pcap *p = nsd_pcap_open(path);
	if (!p)
		return NSD_ERR_ARG;
	if (!p->map || (max_n && (!off || !caplen))) {
		nsd_pcap_close(p);
		return NSD_ERR_ARG;
	}
	std::vector<IxChunk> ch;
	size_t n = 0;
	while (ix_need(p)) {
		// (chunks run last to first: the splice does not depend on the order)
		ix_build(p, window ? (size_t)window : ix_window(), chunks < 1 ? 1 : chunks, ch,
			 [](int nc, const std::function<void(int)> &fn) {
				 for (int c = nc - 1; c >= 0; c--)
					 fn(c);
			 });
		for (size_t i = 0; i < p->ix_off.size(); i++, n++)
			if (n < max_n) {
				off[n] = p->ix_off[i];
				caplen[n] = p->ix_cap[i];
			}
		if (!p->ix_off.empty())
			p->pos = p->ix_off.back() + p->hdrsize + p->ix_cap.back();
		p->ix_i = p->ix_off.size();
	}
	nsd_pcap_close(p);
	return (long)n;
}

// The next record whatever its length (<= the 1 MiB replay buffer), for the
// records a batch cannot carry: its bytes into `frame`, its header as stored
// into rhdr (may be NULL), its sockaddr_ll / frame header fields into *sll /
// *fh (record_meta).  Returns caplen, 0 at the end of the replay.
static long read_one(nsd_pcap *p, std::vector<uint8_t> &frame, nsd_sll_t *sll, nsd_frame_hdr_t *fh,
		     uint8_t *rhdr)
{
	if (p->eof || !p->fill(p->hdrsize)) {
		p->eof = true;
		return 0;
	}
	const uint8_t *h = p->data() + p->pos;
	uint32_t cl;
	memcpy(&cl, h + 8, 4);
	if (p->swapped)
		cl = bswap32(cl);
	const uint32_t caplen = cl - p->ll_extra;
	if (caplen == 0 || caplen > REPLAY_BUF || !p->fill((size_t)p->hdrsize + caplen)) {
		p->eof = true;
		return 0;
	}
	h = p->data() + p->pos;
	frame.assign(h + p->hdrsize, h + p->hdrsize + caplen);
	frame.resize((size_t)caplen + NSD_FRAME_PAD, 0);
	if (rhdr)
		memcpy(rhdr, h, p->hdrsize);
	record_meta(p, h, sll, fh);
	p->pos += p->hdrsize + caplen;
	return caplen;
}

// The replay loop: read -> [BPF filter on the device] -> device walk (pipelined,
// `depth` batches in flight) -> host formatter -> [tprintf wrap] -> out_fd.
// Writes the text dissector_entry_point prints for each accepted record, in
// file order.  `filter` may be NULL (every record passes, bpf.c:711).
// `cols` > 0 wraps like tprintf at that width, 0 writes the unwrapped stream.
// counters (may be NULL) accumulates the per-protocol counter vector.
// `threads` host threads render each batch (<= 0: up to 16 by the hardware).
// Returns the records printed, or a negative NSD_ERR_*.
extern "C" long nsd_replay_pcap(const char *path, int mode, const nsd_bpf_prog *filter, int out_fd,
				int cols, uint64_t *counters, int threads)
{
	return nsd_replay_pcap_out(path, mode, filter, out_fd, cols, counters, threads, -1);
}

static bool write_all(int fd, const void *buf, size_t n)
{
	const uint8_t *w = (const uint8_t *)buf;
	while (n) {
		ssize_t r = write(fd, w, n);
		if (r < 0 && errno == EINTR)
			continue;
		if (r <= 0)
			return false;
		w += r;
		n -= (size_t)r;
	}
	return true;
}

// pcap_generic_push_fhdr -> pcap_prepare_header (pcap_io.h:813-843, 936-950)
// with the replayed file's magic and link type as read_pcap holds them
// (ctx->magic / ctx->link_type, netsniff-ng.c:694-695): the *_LL remap undone
// (the stored magic), version 2.4, thiszone 0, sigfigs 0, snaplen 65535,
// link type swapped once more when the magic is a swapped one (as the
// reference does with the as-stored value).  A swapped SLL / netlink file
// holds the remapped magic swab32(*_MAGIC_LL), which pcap_magic_is_swapped
// does not recognise (pcap_io.h:307-320): its header is written unswapped,
// the link type as stored.
static bool push_fhdr(const nsd_pcap *p, int fd)
{
	uint8_t h[24];
	const bool sw = p->swapped && p->ll_extra == 0;
	const uint16_t vmaj = sw ? bswap16(2) : 2, vmin = sw ? bswap16(4) : 4;
	const uint32_t zero = 0, snap = sw ? bswap32(65535) : 65535;
	const uint32_t lt = sw ? bswap32(p->linktype) : p->linktype;
	memcpy(h, &p->magic_raw, 4);
	memcpy(h + 4, &vmaj, 2);
	memcpy(h + 6, &vmin, 2);
	memcpy(h + 8, &zero, 4);
	memcpy(h + 12, &zero, 4);
	memcpy(h + 16, &snap, 4);
	memcpy(h + 20, &lt, 4);
	return write_all(fd, h, sizeof(h));
}

// The replay's staging: pinned host buffers per batch slot and the device pipe.
namespace {
constexpr uint32_t BATCH = 1u << 16;
constexpr size_t FRAME_BYTES = 32ull << 20;
constexpr int DEPTH = 3;           // batches on the device
constexpr int NSLOT = DEPTH + 4;   // + being copied, being rendered, rendered, being written
// the side words and room for a quarter of a batch to take a deep (> 12
// layer) entry; a chain the pool cannot hold is rendered per packet
constexpr uint32_t EXT_WORDS = BATCH + BATCH / 4 * NSD_EXT_WORDS(NSD_EXT_MAX_LAYERS);

// one formatter part's text: a cache line of its own, as every append writes
// the string's length (adjacent std::strings shared lines between the pool's
// threads: per-packet false sharing that cost the 16-thread pool 3x per record)
struct alignas(64) TextPart {
	std::string s;
};

struct ReplayRes {
	nsd_pipe *pipe = nullptr;
	struct {
		uint8_t *frames;
		nsd_desc_t *desc;
		nsd_sll_t *sll;
		nsd_crec *rec;
		uint32_t *ext;
	} buf[NSLOT] = {};
	// each record's frame header fields (show_frame_hdr)
	std::vector<nsd_frame_hdr_t> fh[NSLOT];
	// a mapped file's record offsets (scan_batch)
	std::vector<uint64_t> src[NSLOT];
	// the formatter parts' text buffers per slot, kept with their capacity:
	// regrown per replay they faulted in hundreds of MB of fresh pages,
	// with the formatter threads queued on the page-table lock
	std::vector<TextPart> part[NSLOT];
	bool ready() const { return pipe != nullptr; }
	long create(int lt, int mode)
	{
		pipe = nsd_pipe_create_compact(BATCH, FRAME_BYTES, EXT_WORDS, DEPTH, lt, mode);
		if (!pipe)
			return NSD_ERR_HIP;
		for (auto &x : buf) {
			x.frames = (uint8_t *)nsd_host_alloc(FRAME_BYTES);
			x.desc = (nsd_desc_t *)nsd_host_alloc(BATCH * sizeof(nsd_desc_t));
			x.sll = (nsd_sll_t *)nsd_host_alloc(BATCH * sizeof(nsd_sll_t));
			x.rec = (nsd_crec *)nsd_host_alloc(BATCH * sizeof(nsd_crec));
			x.ext = (uint32_t *)nsd_host_alloc(EXT_WORDS * sizeof(uint32_t));
			if (!x.frames || !x.desc || !x.sll || !x.rec || !x.ext) {
				release();
				return NSD_ERR_NOMEM;
			}
		}
		for (auto &v : fh)
			v.resize(BATCH);
		for (auto &v : src)
			v.resize(BATCH);
		return NSD_OK;
	}
	void release()
	{
		for (auto &x : buf) {
			nsd_host_free(x.frames);
			nsd_host_free(x.desc);
			nsd_host_free(x.sll);
			nsd_host_free(x.rec);
			nsd_host_free(x.ext);
			x = {};
		}
		for (auto &v : part)
			std::vector<TextPart>().swap(v);
		for (auto &v : fh)
			std::vector<nsd_frame_hdr_t>().swap(v);
		for (auto &v : src)
			std::vector<uint64_t>().swap(v);
		nsd_pipe_destroy(pipe);
		pipe = nullptr;
	}
};
std::mutex g_replay_mu;
ReplayRes g_replay;

// The CPUs the formatter pool runs on: one per physical core (an SMT
// sibling formats at a fraction of a core's rate), those of the calling
// thread's NUMA node first, of the CPUs this process may use.  Empty when
// the topology cannot be read (then nothing is pinned), or NSD_REPLAY_PIN=0.
// The topology is read from /sys once per process.
struct CpuTopo {
	int cpu;
	long pkg, core;
	int node;
};
const std::vector<CpuTopo> &cpu_topology()
{
	static const std::vector<CpuTopo> topo = [] {
		std::vector<CpuTopo> t;
		auto rd = [](int cpu, const char *what) -> long {
			char path[128];
			snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/%s", cpu, what);
			FILE *f = fopen(path, "r");
			if (!f)
				return -1;
			long v = -1;
			if (fscanf(f, "%ld", &v) != 1)
				v = -1;
			fclose(f);
			return v;
		};
		for (int c = 0; c < CPU_SETSIZE; c++) {
			const long pkg = rd(c, "topology/physical_package_id"), core = rd(c, "topology/core_id");
			if (pkg < 0 || core < 0)
				continue;
			int node = 0;
			for (int n = 0; n < 64; n++) {
				char path[128];
				snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/node%d", c, n);
				if (access(path, F_OK) == 0) {
					node = n;
					break;
				}
			}
			t.push_back({ c, pkg, core, node });
		}
		return t;
	}();
	return topo;
}

std::vector<int> pool_cpus()
{
	std::vector<int> out;
	const char *e = getenv("NSD_REPLAY_PIN");
	if (e && e[0] == '0')
		return out;
	cpu_set_t set;
	if (sched_getaffinity(0, sizeof(set), &set) != 0)
		return out;
	const std::vector<CpuTopo> &topo = cpu_topology();
	const int me = sched_getcpu();
	const CpuTopo *mine = nullptr;
	for (const CpuTopo &t : topo)
		if (t.cpu == me)
			mine = &t;
	std::vector<std::pair<long, long>> seen;   // (package, core)
	std::vector<int> near, far;
	int first = -1;                            // the caller's core
	for (const CpuTopo &t : topo) {
		if (!CPU_ISSET(t.cpu, &set))
			continue;
		bool dup = false;
		for (auto &x : seen)
			dup = dup || (x.first == t.pkg && x.second == t.core);
		if (dup)
			continue;
		seen.emplace_back(t.pkg, t.core);
		if (mine && t.pkg == mine->pkg && t.core == mine->core)
			first = t.cpu;
		else
			(!mine || t.node == mine->node ? near : far).push_back(t.cpu);
	}
	// the caller's core first (the pool leaves it to the reader)
	if (first >= 0)
		out.push_back(first);
	out.insert(out.end(), near.begin(), near.end());
	out.insert(out.end(), far.begin(), far.end());
	return out;
}

// Stage times of one replay, printed to stderr when NSD_REPLAY_STATS is set
// in the environment (the pipeline's balance on a given host): the reader,
// the device waits, the formatter jobs (summed over the pool), the writer,
// and the reader's waits for a free slot.
struct ReplayStats {
	std::atomic<uint64_t> read{ 0 }, scan{ 0 }, ix{ 0 }, dev{ 0 }, fmt{ 0 }, write{ 0 }, slot{ 0 }, jobs{ 0 };
	static uint64_t now()
	{
		return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
			       std::chrono::steady_clock::now().time_since_epoch())
			.count();
	}
};
} // namespace

// As nsd_replay_pcap; with pcap_fd >= 0 also the `--out f.pcap` write-out
// of read_pcap (netsniff-ng.c:636, 693-697, 739-746): the file header, then
// every record that passed the filter exactly as it was read (record header
// incl. the *_LL cooked header, then its bytes: write_pcap(fdo, &phdr, magic,
// out, pcap_get_length) of pcap_sg.c / pcap_rw.c), in file order.
//
// Three stages run at once over a ring of batch slots (pinned host buffers):
//   - this thread reads a batch, filters it and submits it to the device
//     pipe (compact records, DEPTH batches in flight); when the pipe is full
//     it completes the oldest batch and queues its render jobs;
//   - `threads` formatter threads (a pool for the whole replay) render the
//     batch's contiguous packet ranges, each into its own text buffer;
//   - a writer thread writes each batch's buffers in file order (writev, or
//     through the tprintf wrap when cols > 0), then the pcap write-out, and
//     frees the slot.
// So reading and walking batch k+1 overlap the rendering of batch k and the
// writing of batch k-1.  A record above NSD_MAX_CAPLEN waits for everything
// before it to be written, then goes through the per-packet path.
extern "C" __attribute__((visibility("hidden"))) void nsd_if_cache_reset(void);   // nsd_format.cpp

extern "C" long nsd_replay_pcap_out(const char *path, int mode, const nsd_bpf_prog *filter, int out_fd,
				    int cols, uint64_t *counters, int threads, int pcap_fd)
{
	if (threads <= 0) {
		const unsigned hc = std::thread::hardware_concurrency();
		threads = hc ? (int)(hc < 16 ? hc : 16) : 1;
	}
	if (threads > 64)
		threads = 64;
	nsd_pcap *p = nsd_pcap_open(path);
	if (!p)
		return NSD_ERR_ARG;
	nsd_if_cache_reset();   // interface names as they are now (renames since an earlier replay)
	const int lt = (int)p->linktype;
	// the dissector's SLL head reads the sockaddr_ll: an *_LL file's cooked
	// headers, or a Kuznetzov / Borkmann file of an SLL link type (the frame
	// headers read it for every file)
	const bool has_ll = p->ll_extra != 0 || p->linktype == LT_LINUX_SLL || p->linktype == bswap32(LT_LINUX_SLL);
	if (pcap_fd >= 0 && !push_fhdr(p, pcap_fd)) {
		nsd_pcap_close(p);
		return NSD_ERR_ARG;
	}
	// the pinned staging and the device pipe (hundreds of MB: their set-up
	// costs about as much as replaying a million records) are kept for the
	// process and reused by the next replay; a replay running beside another
	// gets its own
	std::unique_lock<std::mutex> cache_lk(g_replay_mu, std::try_to_lock);
	ReplayRes own;
	ReplayRes &res = cache_lk.owns_lock() ? g_replay : own;
	long rc = res.ready() ? (long)nsd_pipe_retarget(res.pipe, lt, mode) : (long)res.create(lt, mode);
	if (rc == 1) {
		// the cached set was made on another device than the current one
		res.release();
		rc = res.create(lt, mode);
	}
	if (rc != NSD_OK) {
		nsd_pcap_close(p);
		return rc;
	}
	nsd_pipe *const pipe = res.pipe;
	struct Slot {
		uint8_t *frames = nullptr;
		nsd_desc_t *desc = nullptr;
		nsd_sll_t *sll = nullptr;
		uint8_t *rhdr = nullptr;   // record headers as read (pcap write-out)
		nsd_frame_hdr_t *fh = nullptr;
		uint64_t *src = nullptr;   // record offsets in a mapped file
		int fill_left = 0;         // copy jobs of the batch not done
		uint64_t count0 = 0;       // the packet counter of the batch's first record
		nsd_crec *rec = nullptr;
		uint32_t *ext = nullptr;
		uint32_t *verdict = nullptr;
		uint32_t ext_used = 0, n = 0;
		uint64_t cnt[NSD_NCOUNTERS];
		int status = 0;
		uint64_t seq = 0;
		int parts = 0, left = 0;   // render jobs, jobs not done
		std::vector<TextPart> *part = nullptr;   // res.part[slot]
		long prc = NSD_OK;         // first render error
	};
	std::vector<Slot> b(NSLOT);
	std::vector<uint32_t> verdicts(filter ? (size_t)NSLOT * BATCH : 0);
	std::vector<uint8_t> rhdrs(pcap_fd >= 0 ? (size_t)NSLOT * BATCH * 32 : 0);
	for (int k = 0; k < NSLOT; k++) {
		Slot &x = b[k];
		x.frames = res.buf[k].frames;
		x.desc = res.buf[k].desc;
		x.rec = res.buf[k].rec;
		x.ext = res.buf[k].ext;
		x.sll = res.buf[k].sll;
		x.fh = res.fh[k].data();
		x.src = res.src[k].data();
		x.verdict = filter ? &verdicts[(size_t)k * BATCH] : nullptr;
		x.rhdr = pcap_fd >= 0 ? &rhdrs[(size_t)k * BATCH * 32] : nullptr;
		x.part = &res.part[k];
		if (x.part->size() < (size_t)threads)
			x.part->resize(threads);
	}

	std::mutex mu;
	std::condition_variable cv_job, cv_write, cv_free, cv_fill;
	ReplayStats st;
	const bool stats = getenv("NSD_REPLAY_STATS") != nullptr;
	const uint64_t t_start = ReplayStats::now();
	// (slot, part, parts): render jobs, and the jobs of a mapped file's
	// reader (copies of a batch, parts > 0; record index chunks, slot -1),
	// which the pool takes first, in the order given
	struct Job {
		int slot, part, parts;
	};
	std::deque<Job> jobs, fills;
	std::vector<int> free_slots;
	for (int k = NSLOT - 1; k >= 0; k--)
		free_slots.push_back(k);
	std::deque<int> to_write;               // slots in file order, waiting for their render
	uint64_t next_seq = 0, written = 0;     // batches handed to the writer / written
	long err = rc;                          // first error of any stage
	bool stop = false;
	long printed = 0;
	uint64_t counted = 0;                   // read_pcap's ctx->tx_packets (netsniff-ng.c:730)
	long wrap_state = 0;
	std::string wrapped;

	// the writer's output of one piece of text (wrapped when cols > 0)
	auto put_text = [&](const std::string &t) -> long {
		if (cols > 0 && !t.empty()) {
			wrapped.resize(2 * t.size() + 16);
			const long k = nsd_tprintf_wrap(t.data(), t.size(), cols, &wrap_state, &wrapped[0], wrapped.size());
			if (k < 0)
				return k;
			return write_all(out_fd, wrapped.data(), (size_t)k) ? NSD_OK : NSD_ERR_ARG;
		}
		return write_all(out_fd, t.data(), t.size()) ? NSD_OK : NSD_ERR_ARG;
	};
	auto put_parts = [&](const Slot &x) -> long {
		if (cols > 0) {
			for (int t = 0; t < x.parts; t++) {
				const long r = put_text((*x.part)[t].s);
				if (r != NSD_OK)
					return r;
			}
			return NSD_OK;
		}
		std::vector<struct iovec> iov;
		for (int t = 0; t < x.parts; t++)
			if (!(*x.part)[t].s.empty())
				iov.push_back({ (void *)(*x.part)[t].s.data(), (*x.part)[t].s.size() });
		size_t k = 0;
		while (k < iov.size()) {
			const int cnt = (int)(iov.size() - k < 512 ? iov.size() - k : 512);
			ssize_t w = writev(out_fd, &iov[k], cnt);
			if (w < 0 && errno == EINTR)
				continue;
			if (w <= 0)
				return NSD_ERR_ARG;
			while (w > 0 && k < iov.size()) {   // advance past what was written
				if ((size_t)w >= iov[k].iov_len) {
					w -= (ssize_t)iov[k].iov_len;
					k++;
				} else {
					iov[k].iov_base = (uint8_t *)iov[k].iov_base + w;
					iov[k].iov_len -= (size_t)w;
					w = 0;
				}
			}
		}
		return NSD_OK;
	};
	auto put_records = [&](const Slot &x) -> long {
		if (pcap_fd < 0)
			return NSD_OK;
		std::string recs;
		for (uint32_t k = 0; k < x.n; k++) {
			recs.append((const char *)x.rhdr + 32 * (size_t)k, p->hdrsize);
			recs.append((const char *)x.frames + NSD_DESC_OFF(x.desc[k]), NSD_DESC_CAPLEN(x.desc[k]));
		}
		return write_all(pcap_fd, recs.data(), recs.size()) ? NSD_OK : NSD_ERR_ARG;
	};

	// formatter pool: part t of a slot = its packets [n t / parts, n (t+1) / parts)
	auto render = [&](Slot &x, int t) -> long {
		const uint32_t lo = (uint32_t)((uint64_t)x.n * t / x.parts), hi = (uint32_t)((uint64_t)x.n * (t + 1) / x.parts);
		std::string &s = (*x.part)[t].s;
		s.clear();
		return nsd::format_replay_part(s, x.frames, x.desc, x.fh, x.sll, x.rec, x.ext, x.count0, lo, hi, lt, mode);
	};
	// copy job `q` of `parts` of a mapped file's batch
	auto fill_part = [&](Slot &x, int q, int parts) {
		const uint32_t lo = (uint32_t)((uint64_t)x.n * q / parts), hi = (uint32_t)((uint64_t)x.n * (q + 1) / parts);
		fill_range(p, x.frames, x.desc, x.src, lo, hi, x.sll, x.fh, x.rhdr);
	};
	// the copy of a scanned batch (x.n records in slot k) goes to the pool
	// while the reader scans the next batch; wait_fill joins it (the reader
	// takes the batch's parts still queued)
	auto start_fill = [&](Slot &x, int k) {
		const int parts = x.n < 4096 ? 1 : (int)std::min<uint32_t>((uint32_t)threads + 1, x.n / 2048);
		std::lock_guard<std::mutex> g(mu);
		x.fill_left = parts;
		for (int q = 0; q < parts; q++)
			fills.push_back({ k, q, parts });
		cv_job.notify_all();
	};
	// the record index's chunk jobs (slot -1) of the window being built
	std::function<void(int)> ix_fn;
	int ix_left = 0;
	std::vector<IxChunk> ix_chunks;
	// the front copy job, taken with mu held (returns with it held)
	auto run_fill = [&](std::unique_lock<std::mutex> &lk) {
		const Job j = fills.front();
		fills.pop_front();
		lk.unlock();
		if (j.slot < 0)
			ix_fn(j.part);
		else
			fill_part(b[j.slot], j.part, j.parts);
		lk.lock();
		if (j.slot < 0 ? --ix_left == 0 : --b[j.slot].fill_left == 0)
			cv_fill.notify_all();
	};
	auto wait_fill = [&](Slot &x) {
		std::unique_lock<std::mutex> lk(mu);
		while (x.fill_left > 0) {
			if (!fills.empty())
				run_fill(lk);   // (in file order: this batch's or an earlier one's)
			else
				cv_fill.wait(lk);
		}
	};
	// a mapped file's index windows: the chunks of the window after the one
	// the reader scans run on the pool meanwhile (a window's start is the end
	// of the one before, known once that one is spliced)
	std::vector<size_t> ix_b;
	bool ix_flight = false;
	auto ix_launch = [&](size_t start) {
		const int nc = threads + 1;
		ix_b = ix_bounds(p, start, ix_window(), nc);
		if ((int)ix_chunks.size() != nc)
			ix_chunks.resize(nc);
		std::lock_guard<std::mutex> g(mu);
		ix_fn = [&](int c) { ix_chunk(p, ix_b, c, ix_chunks[c]); };
		ix_left = nc;
		for (int c = 0; c < nc; c++)
			fills.push_back({ -1, c, nc });
		ix_flight = true;
		cv_job.notify_all();
	};
	auto ix_join = [&]() {
		std::unique_lock<std::mutex> lk(mu);
		while (ix_left > 0) {
			if (!fills.empty())
				run_fill(lk);
			else
				cv_fill.wait(lk);
		}
		ix_flight = false;
	};
	auto build_index = [&]() {
		if (!ix_flight)
			ix_launch(p->pos);
		ix_join();
		ix_splice(p, ix_b, ix_chunks);
		if (!p->ix_end)
			ix_launch(p->ix_off.empty() ? ix_b[0] : p->ix_off.back() + p->hdrsize + p->ix_cap.back());
	};
	std::vector<std::thread> pool;
	const std::vector<int> cpus = pool_cpus();
	for (int t = 0; t < threads; t++)
		pool.emplace_back([&, t]() {
			if (!cpus.empty()) {
				// one formatter per physical core, near the caller; the
				// caller's own core (the reader) is left out while others remain
				cpu_set_t one;
				CPU_ZERO(&one);
				const size_t k = cpus.size() > 1 ? 1 + (size_t)t % (cpus.size() - 1) : 0;
				CPU_SET(cpus[k], &one);
				(void)pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
			}
			std::unique_lock<std::mutex> lk(mu);
			for (;;) {
				cv_job.wait(lk, [&] { return stop || !jobs.empty() || !fills.empty(); });
				if (jobs.empty() && fills.empty())
					return;
				if (!fills.empty()) {
					run_fill(lk);
					continue;
				}
				const Job j = jobs.front();
				jobs.pop_front();
				lk.unlock();
				const uint64_t t0 = stats ? ReplayStats::now() : 0;
				const long r = render(b[j.slot], j.part);
				if (stats) {
					st.fmt += ReplayStats::now() - t0;
					st.jobs++;
				}
				lk.lock();
				Slot &x = b[j.slot];
				if (r != NSD_OK && x.prc == NSD_OK)
					x.prc = r;
				if (--x.left == 0)
					cv_write.notify_all();
			}
		});
	std::thread writer([&]() {
		std::unique_lock<std::mutex> lk(mu);
		for (;;) {
			cv_write.wait(lk, [&] { return (!to_write.empty() && b[to_write.front()].left == 0) ||
						       (stop && to_write.empty()); });
			if (to_write.empty())
				return;
			const int k = to_write.front();
			to_write.pop_front();
			Slot &x = b[k];
			long r = x.prc;
			const bool skip = err != NSD_OK;
			lk.unlock();
			const uint64_t t0 = stats ? ReplayStats::now() : 0;
			if (!skip && r == NSD_OK)
				r = put_parts(x);
			if (!skip && r == NSD_OK)
				r = put_records(x);
			if (stats)
				st.write += ReplayStats::now() - t0;
			lk.lock();
			if (r != NSD_OK && err == NSD_OK)
				err = r;
			if (!skip && r == NSD_OK)
				printed += x.n;
			written++;
			free_slots.push_back(k);
			cv_free.notify_all();
		}
	});

	// the device batch in slot k completed: queue its render jobs
	std::deque<int> on_device;
	auto complete_oldest = [&]() -> long {
		const int k = on_device.front();
		on_device.pop_front();
		Slot &x = b[k];
		const uint64_t t0 = stats ? ReplayStats::now() : 0;
		const int ws = nsd_pipe_wait(pipe);
		if (stats)
			st.dev += ReplayStats::now() - t0;
		long r = ws != NSD_OK ? (ws < 0 ? ws : NSD_ERR_HIP) : x.status;
		if (r == NSD_OK && counters)
			for (int c = 0; c < NSD_NCOUNTERS; c++)
				counters[c] += x.cnt[c];
		std::lock_guard<std::mutex> g(mu);
		x.parts = x.n < 2048 ? 1 : threads;
		x.left = x.parts;
		x.prc = r;
		x.seq = next_seq++;
		to_write.push_back(k);
		if (r == NSD_OK) {
			for (int t = 0; t < x.parts; t++)
				jobs.push_back({ k, t, 0 });
			cv_job.notify_all();
		} else {
			x.left = 0;
			cv_write.notify_all();
		}
		return r;
	};
	// everything read so far through the device, rendered and written
	auto flush_all = [&]() -> long {
		while (!on_device.empty())
			complete_oldest();
		std::unique_lock<std::mutex> lk(mu);
		cv_free.wait(lk, [&] { return written == next_seq; });
		return err;
	};
	// a record longer than a batch can carry: after the batches before it,
	// filtered and dissected on its own through the per-packet path
	std::vector<uint8_t> big;
	auto one_big = [&]() -> long {
		long r = flush_all();
		if (r != NSD_OK)
			return r;
		nsd_sll_t ll;
		nsd_frame_hdr_t fh;
		uint8_t hdr[32];
		const long caplen = read_one(p, big, &ll, &fh, hdr);
		if (caplen <= 0)
			return NSD_OK;
		if (filter) {
			const nsd_desc_t d = NSD_DESC(0, caplen);
			uint32_t v = 0;
			r = nsd_bpf_filter_batch(filter, big.data(), (size_t)caplen, &d, 1, &v);
			if (r != NSD_OK)
				return r;
			if (!v)
				return NSD_OK;
		}
		if (counters)
			nsd::cpu_count_packet(big.data(), (uint32_t)caplen, lt, mode, has_ll ? &ll : nullptr, counters);
		std::string text;
		nsd::format_frame_hdr(text, fh, &ll, big.data(), (uint32_t)caplen, lt, mode, ++counted);
		r = nsd::render_packet_cpu(text, big.data(), (size_t)caplen, lt, mode, &ll);
		if (r != NSD_OK)
			return r;
		// (the writer is idle: every batch before this record is written)
		r = put_text(text);
		if (r == NSD_OK && pcap_fd >= 0 &&
		    !(write_all(pcap_fd, hdr, p->hdrsize) && write_all(pcap_fd, big.data(), (size_t)caplen)))
			r = NSD_ERR_ARG;
		if (r == NSD_OK)
			printed++;
		return r;
	};

	// slot k's n records read: filtered (bpf_run_filter per record before the
	// dissector, netsniff-ng.c:723-725) and submitted to the device
	auto give_back = [&](int slot) {
		std::lock_guard<std::mutex> g(mu);
		free_slots.push_back(slot);
	};
	auto submit_slot = [&](int k, long n) -> long {
		Slot &x = b[k];
		size_t used = 0;
		for (long j = 0; j < n; j++) {
			const size_t e = NSD_DESC_OFF(x.desc[j]) + NSD_DESC_CAPLEN(x.desc[j]);
			used = e > used ? e : used;
		}
		if (filter) {
			// bpf_run_filter per record before the dissector (netsniff-ng.c:723-725)
			int r = nsd_bpf_filter_batch(filter, x.frames, used, x.desc, (uint32_t)n, x.verdict);
			if (r != NSD_OK) {
				give_back(k);
				return r;
			}
			long m = 0;
			for (long j = 0; j < n; j++)
				if (x.verdict[j]) {
					x.sll[m] = x.sll[j];
					x.fh[m] = x.fh[j];
					if (x.rhdr && m != j)
						memcpy(x.rhdr + 32 * (size_t)m, x.rhdr + 32 * (size_t)j, 32);
					x.desc[m++] = x.desc[j];
				}
			n = m;
			if (n == 0) {
				give_back(k);
				return NSD_OK;
			}
		}
		if ((int)on_device.size() == DEPTH)
			complete_oldest();
		x.n = (uint32_t)n;
		x.count0 = counted + 1;
		counted += x.n;
		x.status = NSD_OK;
		memset(x.cnt, 0, sizeof(x.cnt));
		int r = nsd_pipe_submit_compact(pipe, x.frames, used, x.desc, has_ll ? x.sll : nullptr, x.n, x.rec, x.ext,
						&x.ext_used, x.cnt, &x.status);
		if (r != NSD_OK) {
			give_back(k);
			return r;
		}
		on_device.push_back(k);
		return NSD_OK;
	};
	int pend = -1;     // a mapped file's batch whose copy is on the pool
	long pend_n = 0;
	while (rc == NSD_OK) {
		int k;
		{
			std::unique_lock<std::mutex> lk(mu);
			if (err != NSD_OK) {
				rc = err;
				break;
			}
			if (free_slots.empty()) {
				lk.unlock();
				if (!on_device.empty()) {
					complete_oldest();
					continue;
				}
				lk.lock();
				const uint64_t t0 = stats ? ReplayStats::now() : 0;
				cv_free.wait(lk, [&] { return !free_slots.empty(); });
				if (stats)
					st.slot += ReplayStats::now() - t0;
			}
			k = free_slots.back();
			free_slots.pop_back();
		}
		Slot &x = b[k];
		const uint64_t tr = stats ? ReplayStats::now() : 0;
		long n;
		if (p->map) {
			size_t end = 0;
			if (ix_need(p)) {
				build_index();
				if (stats)
					st.ix += ReplayStats::now() - tr;
			}
			n = scan_batch(p, FRAME_BYTES, x.desc, x.src, BATCH, &end);
			if (stats)
				st.scan += ReplayStats::now() - tr;
			if (n > 0) {
				x.n = (uint32_t)n;
				memset(x.frames + end, 0, NSD_FRAME_PAD);
				start_fill(x, k);
			}
		} else {
			n = read_batch(p, x.frames, FRAME_BYTES, x.desc, x.sll, x.fh, BATCH, nullptr, nullptr, x.rhdr);
		}
		// the mapped batch before this one: its copy done, on to the device
		// (file order)
		if (pend >= 0) {
			const int j = pend;
			pend = -1;
			wait_fill(b[j]);
			const long r = submit_slot(j, pend_n);
			if (r != NSD_OK) {
				if (n > 0 && p->map)
					wait_fill(x);
				give_back(k);
				rc = r;
				break;
			}
		}
		if (stats)
			st.read += ReplayStats::now() - tr;
		if (n == NSD_ERR_CAPLEN) {
			give_back(k);
			rc = one_big();
			continue;
		}
		if (n <= 0) {
			give_back(k);
			if (n < 0)
				rc = n;
			break;
		}
		if (p->map) {
			pend = k;
			pend_n = n;
			continue;
		}
		const long r = submit_slot(k, n);
		if (r != NSD_OK) {
			rc = r;
			break;
		}
	}
	if (ix_flight)
		ix_join();   // (an index window no scan reached)
	if (pend >= 0) {
		// (left by an error: its copy drains before the slots go away)
		wait_fill(b[pend]);
		std::lock_guard<std::mutex> g(mu);
		free_slots.push_back(pend);
	}
	{
		const long r = flush_all();
		if (rc == NSD_OK)
			rc = r;
	}
	{
		std::lock_guard<std::mutex> g(mu);
		stop = true;
	}
	cv_job.notify_all();
	cv_write.notify_all();
	for (auto &t : pool)
		t.join();
	writer.join();
	if (stats)
		fprintf(stderr,
			"nsd_replay: %ld records, %d threads, %.1f ms: read %.1f (scan %.1f, index %.1f), device waits %.1f, slot waits %.1f, "
			"format %.1f (%llu jobs, %.1f per thread), write %.1f ms\n",
			printed, threads, (ReplayStats::now() - t_start) / 1e6, st.read / 1e6, st.scan / 1e6, st.ix / 1e6, st.dev / 1e6, st.slot / 1e6,
			st.fmt / 1e6, (unsigned long long)st.jobs.load(), st.fmt / 1e6 / threads, st.write / 1e6);
	// (an error leaves batches in the pipe: drop the cached set then)
	if (&res == &own || rc != NSD_OK)
		res.release();
	nsd_pcap_close(p);
	return rc == NSD_OK ? printed : rc;
}

// dissector_cleanup_all (nsd_proto.cpp) frees the replay's cached buffers
extern "C" __attribute__((visibility("hidden"))) void nsd_replay_release(void)
{
	std::lock_guard<std::mutex> g(g_replay_mu);
	g_replay.release();
}

// ---- TPACKET_V3 ring front end (walk_t3_block, netsniff-ng.c:990-1039) ------
// A retired RX ring block (struct block_desc, netsniff-ng.c:1061-1066 =
// tpacket_block_desc: version, offset_to_priv, tpacket_hdr_v1 {block_status,
// num_pkts, offset_to_first_pkt, blk_len, seq_num, ts_first, ts_last}) is
// turned into descriptors that point into the block itself, so the block
// is the batch's frame buffer (zero copy on the host; nsd_pipe_submit(block,
// block_len, desc, n, ...)).  Per frame: tpacket3_hdr {tp_next_offset,
// tp_sec, tp_nsec, tp_snaplen, tp_len, tp_status, tp_mac, tp_net, ...} with the
// sockaddr_ll at TPACKET_ALIGN(sizeof(tpacket3_hdr)) = 48 after it; the packet
// is at hdr + tp_mac, tp_snaplen bytes.  skip_packet (netsniff-ng.c:425-442):
// with packet_type >= 0 only frames of that sll_pkttype are kept; otherwise
// frames on the loopback ifindex `lo_ifindex` with PACKET_OUTGOING (4) are
// dropped.  Returns the frames described, or NSD_ERR_ARG for a block whose
// headers point outside it (or a frame above NSD_MAX_CAPLEN).
extern "C" long nsd_t3_block_desc(const uint8_t *block, size_t block_len, int packet_type,
				  int lo_ifindex, nsd_desc_t *desc, uint32_t max_n)
{
	return nsd_t3_block_desc_sll(block, block_len, packet_type, lo_ifindex, desc, nullptr, max_n);
}

// same, also copying each kept frame's sockaddr_ll (hdr + 48, the `sll`
// walk_t3_block hands to dissector_entry_point, netsniff-ng.c:1011-1025)
// into sll[k] (may be NULL): the per-packet input of the SLL heads
extern "C" long nsd_t3_block_desc_sll(const uint8_t *block, size_t block_len, int packet_type,
				      int lo_ifindex, nsd_desc_t *desc, nsd_sll_t *sll, uint32_t max_n)
{
	return nsd_t3_block_desc_fh(block, block_len, packet_type, lo_ifindex, desc, sll, nullptr, max_n);
}

// same, also the frame header fields walk_t3_block's __show_frame_hdr reads
// from each kept frame's tpacket3_hdr (netsniff-ng.c:1021; v3 true):
// tp_sec +4, tp_nsec +8, tp_len +16, tp_status +20, hv1.tp_vlan_tci +32,
// hv1.tp_vlan_tpid +36
extern "C" long nsd_t3_block_desc_fh(const uint8_t *block, size_t block_len, int packet_type, int lo_ifindex,
				     nsd_desc_t *desc, nsd_sll_t *sll, nsd_frame_hdr_t *fh, uint32_t max_n)
{
	if (!block || !desc || block_len < 48)
		return NSD_ERR_ARG;
	uint32_t num_pkts, first;
	memcpy(&num_pkts, block + 12, 4);
	memcpy(&first, block + 16, 4);
	size_t h = first;
	uint32_t n = 0;
	for (uint32_t i = 0; i < num_pkts; i++) {
		if (h + 48 + 20 > block_len)
			return NSD_ERR_ARG;
		uint32_t next, snaplen;
		uint16_t mac;
		int32_t ifindex;
		memcpy(&next, block + h, 4);
		memcpy(&snaplen, block + h + 12, 4);
		memcpy(&mac, block + h + 24, 2);
		memcpy(&ifindex, block + h + 48 + 4, 4);
		const uint8_t pkttype = block[h + 48 + 10];
		const bool skip = packet_type >= 0 ? pkttype != (uint8_t)packet_type
						   : (ifindex == lo_ifindex && pkttype == 4);
		if (!skip) {
			if (h + mac + (size_t)snaplen > block_len || snaplen > NSD_MAX_CAPLEN || n >= max_n)
				return NSD_ERR_ARG;
			if (sll)
				memcpy(&sll[n], block + h + 48, sizeof(nsd_sll_t));
			if (fh) {
				nsd_frame_hdr_t &f = fh[n];
				memset(&f, 0, sizeof(f));
				memcpy(&f.sec, block + h + 4, 4);
				memcpy(&f.nsec, block + h + 8, 4);
				memcpy(&f.len, block + h + 16, 4);
				memcpy(&f.status, block + h + 20, 4);
				memcpy(&f.vlan_tci, block + h + 32, 4);
				memcpy(&f.vlan_tpid, block + h + 36, 2);
				f.v3 = 1;
			}
			desc[n++] = NSD_DESC(h + mac, snaplen);
		}
		if (i + 1 < num_pkts) {
			if (next == 0)
				return NSD_ERR_ARG;
			h += next;
		}
	}
	return n;
}
