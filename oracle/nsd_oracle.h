/*
 * nsd_oracle.h - CPU restatement of netsniff-ng's dissector chain.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker the device path is compared
 * against; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it.  The product library (netsniff-ng_amd/) never links it.
 *
 * Parity pin: every parser except IPv4/IPv6 is pinned against the
 * reference's own parser objects compiled from /root/reference (oracle/_ref,
 * "make -C oracle ref"); IPv4/IPv6 cannot be compiled from the reference
 * here (proto_ipv4.c/proto_ipv6.c include geoip.h -> the configure-generated
 * config.h, which this image cannot produce), so their text is pinned by the
 * restatement plus known-answer checks only.  See DESIGN.md "Oracle".
 */
#ifndef NSD_ORACLE_H
#define NSD_ORACLE_H

#include <stddef.h>
#include <stdint.h>
#include "../include/netsniff_dissect.h"

#ifdef __cplusplus
extern "C" {
#endif

/* growable text sink; pass NULL for fields-only walks */
typedef struct nsor_text {
	char  *buf;
	size_t len, cap;
	int    unsupported;   /* set when a host-only body (ARP, LLDP, ...) was hit */
} nsor_text;

void nsor_text_init(nsor_text *t);
void nsor_text_free(nsor_text *t);
void nsor_text_reset(nsor_text *t);

/* per-packet walk result beyond the record */
typedef struct nsor_info {
	uint32_t nlayers;
	uint8_t  id[NSD_EXT_MAX_LAYERS];
	uint16_t off[NSD_EXT_MAX_LAYERS];
	uint32_t data, tail;
	uint32_t w_bytes;      /* algorithmic read bytes W(pkt) */
	int      overflow;
} nsor_info;

/* Dissect one packet (bytes past caplen read as zero).
 * mode: PRINT_* ; linktype as in dissector_entry_point.
 * text may be NULL (no formatting).  rec/info may be NULL. */
void nsor_dissect(const uint8_t *pkt, uint32_t caplen, int linktype, int mode,
		  nsor_text *text, nsd_rec *rec, nsor_info *info);

/* The struct sockaddr_ll the LINKTYPE_LINUX_SLL head prints and dispatches
 * on, for the next nsor_dissect calls of this thread (NULL = zeros). */
void nsor_set_sll(const nsd_sll_t *sll);

/* Batch form producing exactly what the device produces.  Ext pool entries
 * are packed densely in packet order (the device hands them out in
 * arbitrary order from per-wave chunks; tests compare through the slot
 * indirection).  *ext_used accumulates the words taken; counters
 * accumulate.  Returns sum W. */
uint64_t nsor_dissect_batch(const uint8_t *frames, const nsd_desc_t *desc, uint32_t n,
			    int linktype, int mode, nsd_rec *rec, uint32_t *ext,
			    uint32_t ext_words, uint32_t *ext_used, uint64_t *counters);

/* Same, with one struct sockaddr_ll per packet (SLL link types; may be NULL). */
uint64_t nsor_dissect_batch_sll(const uint8_t *frames, const nsd_desc_t *desc, const nsd_sll_t *sll,
				uint32_t n, int linktype, int mode, nsd_rec *rec, uint32_t *ext,
				uint32_t ext_words, uint32_t *ext_used, uint64_t *counters);

/* Same walk, text for every packet appended to *text (fields+text baseline). */
uint64_t nsor_dissect_batch_text(const uint8_t *frames, const nsd_desc_t *desc,
				 uint32_t n, int linktype, int mode, nsor_text *text);

/* Multi-threaded fields-only walk over contiguous shards (CPU baseline). */
/* Distinct 128-byte lines holding the bytes the chain must inspect,
 * [off, off + W) per packet (the batch's line floor; bench.py's roofline) */
uint64_t nsor_line_floor_mt(const uint8_t *frames, const nsd_desc_t *desc, uint32_t n, int linktype, int mode,
			    int nthreads);

uint64_t nsor_dissect_batch_mt(const uint8_t *frames, const nsd_desc_t *desc, uint32_t n,
			       int linktype, int mode, nsd_rec *rec, uint64_t *counters,
			       int nthreads);

/* Multi-threaded fields + text walk (text per packet into a per-thread sink,
 * discarded after each packet: the formatted CPU baseline); *text_bytes
 * receives the text length.  Returns sum W. */
uint64_t nsor_dissect_batch_text_mt(const uint8_t *frames, const nsd_desc_t *desc, uint32_t n,
				    int linktype, int mode, int nthreads, uint64_t *text_bytes);

/* The same with each packet's frame header line in front of its text
 * (fh / sll per packet, counter first_count + i; fh NULL: none). */
uint64_t nsor_dissect_batch_text_fh_mt(const uint8_t *frames, const nsd_desc_t *desc, const nsd_frame_hdr_t *fh,
				       const nsd_sll_t *sll, uint64_t first_count, uint32_t n, int linktype,
				       int mode, int nthreads, uint64_t *text_bytes);

/* show_frame_hdr (dissector.h:31-116) restated: the line for one packet. */
void nsor_frame_hdr(const nsd_frame_hdr_t *fh, const nsd_sll_t *sll, const uint8_t *pkt, uint32_t caplen,
		    int linktype, int mode, uint64_t count, nsor_text *t);

/* read_pcap's record loop restated (pcap_io.h / pcap_rw.c): each record's
 * frame header fields, sockaddr_ll and caplen (any may be NULL) for up to
 * max records; returns the records, -1 for a refused file. */
long nsor_pcap_meta(const char *path, nsd_frame_hdr_t *fh, nsd_sll_t *sll, uint32_t *caplen, uint32_t max);

/* Name tables (lookup.c:33-95 restated).  dir NULL => clear (names off). */
int  nsor_lookup_init(const char *dir);
void nsor_lookup_clear(void);

/* Per-layer entry for the oracle/_ref hybrid harness: run one ops' print
 * function on [*data, *tail) of pkt, return next ops ID (0 = chain ends).
 * emit receives the text pieces in order. */
typedef void (*nsor_emit_fn)(void *ctx, const char *s, size_t n);
int nsor_run_layer(int ops_id, int mode, const uint8_t *pkt, uint32_t caplen,
		   uint32_t *data, uint32_t *tail, nsor_emit_fn emit, void *ctx);

#ifdef __cplusplus
}
#endif
#endif
