/*
 * netsniff_dissect.h - C ABI of the MI355X-native netsniff-ng dissection path.
 *
 * Drop-in boundary for netsniff-ng's per-packet dissector chain
 * (reference: dissector.h:118-122, dissector.c:22-138, dissector_eth.c:17-86,
 * proto.h:18-26, pkt_buff.h:15-110).  Two surfaces:
 *
 *   1. The reference surface, same names / argument meaning / behaviour:
 *        dissector_init_all        <- dissector.h:118 / dissector.c:124-130
 *        dissector_entry_point     <- dissector.h:119 / dissector.c:64-122
 *        dissector_cleanup_all     <- dissector.h:121 / dissector.c:132-138
 *        dissector_set_print_type  <- dissector.h:122 / dissector.c:22-41
 *        struct protocol / pkt_buff and the protos.h ops objects
 *      The per-packet entry point runs on the host CPU.
 *
 *   2. The batch extension (new): a packed batch of frames is
 *      walked by hand-written CDNA4 kernels, one lane per packet, producing
 *      a 16-byte chain record per packet, an overflow table for deep chains
 *      and a per-protocol counter vector.
 *
 * Plain C types only (no torch / HIP types); a stream is passed as void *
 * (a hipStream_t, NULL = the null stream).
 */
#ifndef NETSNIFF_DISSECT_H
#define NETSNIFF_DISSECT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- print modes (dissector.h:22-27) ---------------------------------- */
#define PRINT_NORM      0
#define PRINT_LESS      1
#define PRINT_HEX       2
#define PRINT_ASCII     3
#define PRINT_HEX_ASCII 4
#define PRINT_NONE      5

/* ---- link types the entry point switches on (linktype.h, dissector.c:77-104) */
#define NSD_LINKTYPE_EN10MB            1
#define NSD_LINKTYPE_IEEE802_11        105
#define NSD_LINKTYPE_LINUX_SLL         113
#define NSD_LINKTYPE_IEEE802_11_RADIOTAP 127
#define NSD_LINKTYPE_NETLINK           253

/* ---- protocol-chain IDs: one per ops object (protos.h:6-31) -------------
 * Identity is the ops struct, not the hash key: none_ops and icmpv4_ops share
 * key 0x01, ethernet_ops and ipv6_hop_by_hop_ops share key 0. */
enum nsd_ops_id {
	NSD_OPS_INVALID        = 0,
	NSD_OPS_ETHERNET       = 1,   /* proto_ethernet.c:99      key 0      */
	NSD_OPS_VLAN           = 2,   /* proto_vlan.c:57          0x8100     */
	NSD_OPS_QINQ           = 3,   /* proto_vlan_q_in_q.c:58   0x88a8     */
	NSD_OPS_MPLS_UC        = 4,   /* proto_mpls_unicast.c:104  0x8847     */
	NSD_OPS_ARP            = 5,   /* proto_arp.c:198          0x0806     */
	NSD_OPS_LLDP           = 6,   /* proto_lldp.c:490         0x88cc     */
	NSD_OPS_IPV4           = 7,   /* proto_ipv4.c:206         0x0800     */
	NSD_OPS_IPV6           = 8,   /* proto_ipv6.c:115         0x86DD     */
	NSD_OPS_IPV6_IN_IPV4   = 9,   /* proto_ipv6_in_ipv4.c:20  41         */
	NSD_OPS_ICMPV4         = 10,  /* proto_icmpv4.c:63        1          */
	NSD_OPS_ICMPV6         = 11,  /* proto_icmpv6.c:1701      58         */
	NSD_OPS_IGMP           = 12,  /* proto_igmp.c:556         2          */
	NSD_OPS_IP_AUTH        = 13,  /* proto_ip_authentication_hdr.c:90  51 */
	NSD_OPS_IP_ESP         = 14,  /* proto_ip_esp.c:48        50         */
	NSD_OPS_IPV6_DEST_OPTS = 15,  /* proto_ipv6_dest_opts.c:97  60       */
	NSD_OPS_IPV6_FRAGM     = 16,  /* proto_ipv6_fragm.c:65    44         */
	NSD_OPS_IPV6_HOP_BY_HOP= 17,  /* proto_ipv6_hop_by_hop.c:96  0       */
	NSD_OPS_IPV6_MOBILITY  = 18,  /* proto_ipv6_mobility_hdr.c:311 135   */
	NSD_OPS_IPV6_NO_NEXT   = 19,  /* proto_ipv6_no_nxt_hdr.c:36  59      */
	NSD_OPS_IPV6_ROUTING   = 20,  /* proto_ipv6_routing.c:158 43         */
	NSD_OPS_TCP            = 21,  /* proto_tcp.c:153          6          */
	NSD_OPS_UDP            = 22,  /* proto_udp.c:85           17         */
	NSD_OPS_DCCP           = 23,  /* proto_dccp.c:150         33         */
	NSD_OPS_NONE           = 24,  /* proto_none.c:79          exit op    */
	NSD_OPS_SLL            = 25,  /* dissector_sll.c:84       (host)     */
	NSD_OPS_IEEE80211      = 26,  /* proto_80211_mac_hdr.c:3269 (host)     */
	NSD_OPS_NLMSG          = 27,  /* proto_nlmsg.c:1058       (host)     */
	NSD_OPS_COUNT          = 28
};

/* ---- batch input --------------------------------------------------------
 * Frames live in one byte buffer; packet i is described by one 64-bit word:
 * bits 0..39 = byte offset of the frame in the buffer (any alignment),
 * bits 40..63 = caplen (tp_snaplen).  caplen must be <= NSD_MAX_CAPLEN.
 * The buffer must stay readable for NSD_FRAME_PAD bytes past its last frame
 * (the kernel loads whole 16-byte chunks and masks bytes >= caplen to zero).
 * Bytes at offsets >= caplen read as zero: this is the parity domain's
 * definition of out-of-frame bytes (SURVEY §8a "Parity domain"). */
typedef uint64_t nsd_desc_t;
#define NSD_DESC(off, caplen)   ((((uint64_t)(caplen)) << 40) | ((uint64_t)(off) & 0xFFFFFFFFFFull))
#define NSD_DESC_OFF(d)         ((uint64_t)(d) & 0xFFFFFFFFFFull)
#define NSD_DESC_CAPLEN(d)      ((uint32_t)((uint64_t)(d) >> 40))
#define NSD_MAX_CAPLEN          65535u
#define NSD_FRAME_PAD           64u

/* ---- per-packet chain record (16 bytes, written by the device) ----------
 * chain   : ops ID of layer k in bits [5k, 5k+5), k = 0..5.
 * data_off: final pkt->data; the exit op (none_ops) covers [data_off, tail_off).
 * tail_off: final pkt->tail (caplen unless the IPv4 trim, proto_ipv4.c:174, cut it).
 * ip_csum : IPv4 header checksum as the reference computes it
 *           (calc_csum over ihl*4 bytes, proto_ipv4.c:51); 0 means "ok".
 *           Only computed in PRINT_NORM; 0 otherwise.
 * nflags  : bits 0..2 = number of layers run (0..6), 7 = NSD_N_EXT (the full
 *           chain is in the ext pool, slot = off2[0..3] little-endian u32);
 *           bits 3..7 = NSD_F_* flags.
 * off2[k-1]: start offset of layer k divided by 2, k = 1..5 (layer 0 starts
 *           at 0). Every layer start is even, and offsets > 510
 *           force the ext form.
 */
typedef struct nsd_rec {
	uint32_t chain;
	uint16_t data_off;
	uint16_t tail_off;
	uint16_t ip_csum;
	uint8_t  nflags;
	uint8_t  off2[5];
} nsd_rec;

#define NSD_REC_MAX_LAYERS   6
#define NSD_N_EXT            7
#define NSD_F_ICMP_BAD       0x08  /* ICMPv4 checksum nonzero: "bogus (!)" (proto_icmpv4.c:74-81) */
#define NSD_F_HOST           0x10  /* last layer's fields are printed by the host renderer
                                      (ICMPv6 130-154, ARP, LLDP, IGMP, DCCP, non-Ethernet link
                                      types); data_off is still where that parser's pulls end */
#define NSD_F_OVERFLOW       0x20  /* chain longer than NSD_EXT_MAX_LAYERS or ext pool full:
                                      record holds the first layers only */
#define NSD_F_LEAF_END       0x40  /* compact records (nsd_crec) of an NSD_F_HOST leaf: where the
                                      leaf's pulls end (the 16-byte record's data_off) is in the
                                      packet's side word (chains up to 6 layers) or in word 2 of
                                      its ext entry (chains past 12 layers), bits 0..15 */

#define NSD_REC_NLAYERS(r)   ((r)->nflags & 7u)
#define NSD_REC_ID(r, k)     (((r)->chain >> (5u * (k))) & 31u)

/* ---- ext pool: chains the 16-byte record cannot hold --------------------
 * Chains longer than NSD_REC_MAX_LAYERS layers, or with a layer starting past
 * byte 510, keep their full layer list in a pool of u32 words; the record's
 * slot (off2[0..3], little-endian) is the entry's word index s:
 *   pool[s + 0]     packet index within the batch
 *   pool[s + 1]     nlayers
 *   pool[s + 2..3]  reserved
 *   pool[s + 4 + k] ops ID (bits 0..7) | start offset of layer k (bits 16..31),
 *                   k < nlayers (at most NSD_EXT_MAX_LAYERS)
 * An entry occupies NSD_EXT_WORDS(nlayers) words.  The device hands pool
 * words out in per-wave chunks, so *ext_used (the words handed out) can
 * exceed the words holding entries; an entry that does not fit in the pool
 * leaves its record with NSD_F_OVERFLOW and slot 0xFFFFFFFF.  Entry order is
 * unspecified (follow the records' slots).  Sizing: the unused chunk tails
 * cost at most half the pool, so a pool of twice the words the batch's
 * chains need never overflows; NSD_EXT_POOL_WORDS(n) is that for n packets
 * whose chains are at most 16 layers, plus room for a few deeper ones.
 * Pools are capped at NSD_EXT_POOL_MAX_WORDS words. */
#define NSD_EXT_MAX_LAYERS   64
#define NSD_EXT_HDR_WORDS    4u
#define NSD_EXT_WORDS(nl)    ((nl) <= 16u ? NSD_EXT_HDR_WORDS + 16u : NSD_EXT_HDR_WORDS + NSD_EXT_MAX_LAYERS)
#define NSD_EXT_POOL_WORDS(n)   (48ull * (n) + 4096u)
#define NSD_EXT_POOL_MAX_WORDS  0xF0000000u
#define NSD_EXT_PKT(pool, s)      ((pool)[(s)])
#define NSD_EXT_NLAYERS(pool, s)  ((pool)[(s) + 1] & 0xFFFFu)
#define NSD_EXT_ID(pool, s, k)    ((pool)[(s) + NSD_EXT_HDR_WORDS + (k)] & 0xFFu)
#define NSD_EXT_OFF(pool, s, k)   ((pool)[(s) + NSD_EXT_HDR_WORDS + (k)] >> 16)

/* ---- per-protocol counter vector (u64, summed over the batch) ----------- */
enum nsd_counter {
	NSD_CNT_OPS       = 0,   /* [0, NSD_OPS_COUNT): layer instances per ops ID */
	NSD_CNT_PKTS      = 32,  /* packets walked */
	NSD_CNT_BYTES     = 33,  /* sum of caplen */
	NSD_CNT_IP_BAD    = 34,  /* IPv4 header checksum bogus (PRINT_NORM) */
	NSD_CNT_ICMP_BAD  = 35,  /* ICMPv4 checksum bogus (PRINT_NORM) */
	NSD_CNT_HOST      = 36,  /* records flagged NSD_F_HOST */
	NSD_CNT_EXT       = 37,  /* records using the ext pool */
	NSD_CNT_OVERFLOW  = 38,  /* records flagged NSD_F_OVERFLOW */
	NSD_CNT_TRIM      = 39,  /* IPv4 tail trims (tail_off < caplen) */
	NSD_CNT_LISTOVF   = 40,  /* waves whose pending list overran its slots: a kernel
	                            invariant broken, never expected (results unreliable) */
	NSD_NCOUNTERS     = 64
};

/* ---- status codes ------------------------------------------------------ */
#define NSD_OK               0
#define NSD_ERR_ARG         -1
#define NSD_ERR_HIP         -2
#define NSD_ERR_CAPLEN      -3
#define NSD_ERR_NOMEM       -4
#define NSD_ERR_FORMAT      -5
#define NSD_ERR_UNSUPPORTED -6   /* a chain reaches a reference object (802.11 / netlink)
                                    that prints through tprintf (pcap replay) */

/* ---- reference surface (dissector.h:118-122) ----------------------------
 * The per-packet entry runs on the host CPU, as SURVEY 8b plans it (one
 * packet per launch would be all launch latency): dissector_main's loop
 * (dissector.c:43-62) over the ops objects below, whose process() functions
 * run this library's layer step (nsd_walk.h gen_step, the code the device's
 * general walk runs) and render that layer's text through the caller's
 * tprintf.  Batches go to the device (the batch extension further down).
 *   dissector_init_all(fnttype)  dissector.c:124-130 + dissector_eth.c:64-75
 *       + dissector_sll.c:100-105: print types of every ops object, the
 *       802.11 / netlink initialisers when those reference objects are
 *       linked, and the four name tables from ETCDIRE (NSD_ETCDIRE at build
 *       time, "/etc/netsniff-ng" by default, or nsd_set_etcdir()).
 *   dissector_entry_point        dissector.c:64-122 (any frame length)
 *   dissector_cleanup_all        dissector.c:132-138
 *   dissector_set_print_type     dissector.c:22-41 */
struct sockaddr_ll;
void dissector_init_all(int fnttype);
void dissector_entry_point(uint8_t *packet, size_t len, int linktype, int mode,
			   struct sockaddr_ll *sll);
void dissector_cleanup_all(void);
int  dissector_set_print_type(void *ptr, int type);
/* the directory dissector_init_all loads udp.conf / tcp.conf / ether.conf /
 * oui.conf from (the reference's compile-time ETCDIRE_STRING, lookup.c:20-25);
 * NULL restores the build default */
void nsd_set_etcdir(const char *dir);

/* ---- proto-ops objects (proto.h:18-33, pkt_buff.h:15-24, protos.h:6-31) --
 * Same layouts and names as the reference, so the reference objects that
 * stay in netsniff-ng's link when this library replaces the Ethernet chain
 * (dissector_80211.o, dissector_netlink.o, proto_80211_mac_hdr.o and, with
 * libnl, proto_nlmsg.o / mac80211.o: INTEGRATION.md) find none_ops,
 * dissector_set_print_type and the proto.h dump helpers here, and their
 * ieee80211_ops / nlmsg_ops chains run inside dissector_entry_point.
 * Skipped when the reference's own headers were included first. */
#ifndef PROTO_H
struct pkt_buff;
struct protocol {
	const unsigned int key;
	void (*print_full)(struct pkt_buff *pkt);
	void (*print_less)(struct pkt_buff *pkt);
	struct protocol *next;
	void (*process)(struct pkt_buff *pkt);
};
void empty(struct pkt_buff *pkt);
void _hex(uint8_t *ptr, size_t len);
void hex(struct pkt_buff *pkt);
void _ascii(uint8_t *ptr, size_t len);
void ascii(struct pkt_buff *pkt);
void hex_ascii(struct pkt_buff *pkt);
#endif
#ifndef PKT_BUFF_H
struct pkt_buff {
	uint8_t *head;
	uint8_t *data;
	uint8_t *tail;
	struct protocol *dissector;
	uint32_t link_type;
	struct sockaddr_ll *sll;
};
#endif
#ifndef PROTOS_H
extern struct protocol arp_ops, ethernet_ops, icmpv4_ops, icmpv6_ops, igmp_ops, ip_auth_ops,
	ip_esp_ops, ipv4_ops, ipv6_ops, ipv6_dest_opts_ops, ipv6_fragm_ops, ipv6_hop_by_hop_ops,
	ipv6_in_ipv4_ops, ipv6_mobility_ops, ipv6_no_next_header_ops, ipv6_routing_ops, lldp_ops,
	none_ops, tcp_ops, udp_ops, dccp_ops, vlan_ops, QinQ_ops, mpls_uc_ops;
#endif
extern struct protocol sll_ops;   /* dissector_sll.c:84 */


/* ---- batch extension ---------------------------------------------------- */

/* Device-resident walk: every pointer is device memory, the call only
 * enqueues work on `stream` (no host synchronisation, graph-capturable).
 * `d_ext` is the ext pool of `ext_words` u32 words (may be NULL when 0);
 * `d_ext_used` (one u32, the pool words handed out) is a running offset: set
 * it to 0 before a batch that starts a fresh pool.  `d_counters`
 * (NSD_NCOUNTERS u64) is accumulated into, not overwritten.  `mode` selects
 * the parse semantics (print_full vs print_less chains differ, SURVEY §8a
 * quirk 7 / mobility).  Returns NSD_OK or an error without launching. */
int nsd_dissect_device(const uint8_t *d_frames, const nsd_desc_t *d_desc, uint32_t n,
		       int linktype, int mode,
		       nsd_rec *d_rec, uint32_t *d_ext, uint32_t ext_words,
		       uint32_t *d_ext_used, uint64_t *d_counters, void *stream);

/* Same, with a caller-provided device workspace of nsd_workspace_bytes(n)
 * bytes (the deferral queue and pending-checksum lists between the kernel's
 * phases): no allocation inside, so the call can be captured in a hipGraph.
 * nsd_dissect_device uses a library-owned workspace grown on demand. */
size_t nsd_workspace_bytes(uint32_t n);
int nsd_dissect_device_ws(const uint8_t *d_frames, const nsd_desc_t *d_desc, uint32_t n,
			  int linktype, int mode, nsd_rec *d_rec, uint32_t *d_ext,
			  uint32_t ext_words, uint32_t *d_ext_used, uint64_t *d_counters,
			  void *d_workspace, void *stream);

/* Host-memory batch: stages frames/descriptors to HBM, runs
 * nsd_dissect_device with a fresh pool, copies records / the used pool words
 * / counters back.  Synchronous.  `counters` may be NULL; `ext` may be NULL
 * when ext_words == 0; *ext_used (may be NULL) receives the pool words
 * handed out. */
int dissector_entry_batch(const uint8_t *frames, size_t frames_len,
			  const nsd_desc_t *desc, uint32_t n, int linktype, int mode,
			  nsd_rec *rec, uint32_t *ext, uint32_t ext_words,
			  uint32_t *ext_used, uint64_t *counters);

/* Host formatter: renders one record + its raw frame bytes into the exact
 * text the reference dissector chain prints (unwrapped tprintf stream, i.e.
 * what dissector_entry_point hands to tprintf for this packet).
 * `ext_pool` is the pool the record's slot refers to (may be NULL if the
 * record has no ext slot).  Writes at most `cap` bytes (NUL-terminated when
 * room), returns the full text length, or a negative NSD_ERR_*. */
long nsd_format_packet(const uint8_t *pkt, uint32_t caplen, int linktype, int mode,
		       const nsd_rec *rec, const uint32_t *ext_pool,
		       char *out, size_t cap);

/* Name tables (lookup.c:33-95): load udp.conf / tcp.conf / ether.conf /
 * oui.conf from `dir` (the reference's ETCDIRE_STRING).  NULL or a missing
 * file leaves that table empty (names not printed, vendor "Unknown").
 * Returns the number of tables loaded. */
int nsd_lookup_init(const char *dir);
void nsd_lookup_cleanup(void);

/* tprintf wrap emulation (tprintf.c:65-103): rewrap an unwrapped text
 * stream for a terminal `cols` wide, carrying the line counter in *state
 * (start with 0).  Returns bytes written to out (cap must be >= 2*len+16). */
long nsd_tprintf_wrap(const char *in, size_t len, int cols, long *state,
		      char *out, size_t cap);

/* Pipelined host-batch path (the RX loop's batches, SURVEY 8f.2: e.g. one
 * TPACKET_V3 block per batch, walk_t3_block netsniff-ng.c:991-1039).  Each
 * submitted batch is copied to the device, walked and its records copied
 * back on its own stream slot; up to `depth` batches are in flight, so the
 * copies of one batch overlap the walk of another.  The caller's buffers
 * belong to the pipe from submit until the batch completes (nsd_pipe_wait);
 * pinned buffers (nsd_host_alloc / nsd_host_register) make the copies
 * asynchronous, pageable ones still work but serialise them.
 * Batches complete in submission order.
 *
 * nsd_pipe_create: capacities per batch (packets, frame bytes, ext pool words),
 * 1 <= depth <= 8.  NULL on failure (no GPU, no memory, bad arguments).
 * nsd_pipe_submit: validates like dissector_entry_batch, then enqueues; when
 * all slots are busy it first completes the oldest batch (its status is
 * returned through that batch's *status, see below).  rec[n] receives the
 * records, ext[ext_words] / *ext_used the ext pool, counters[64] (may
 * be NULL) this batch's counters, *status (may be NULL) the batch's final
 * status.  Returns NSD_OK if enqueued, else NSD_ERR_*.
 * nsd_pipe_wait: completes the oldest in-flight batch, returns its status,
 * or 1 when nothing is in flight.  nsd_pipe_drain: completes all. */
typedef struct nsd_pipe nsd_pipe;
nsd_pipe *nsd_pipe_create(uint32_t max_pkts, size_t max_frame_bytes, uint32_t ext_words,
			  int depth, int linktype, int mode);
int nsd_pipe_submit(nsd_pipe *p, const uint8_t *frames, size_t frames_len,
		    const nsd_desc_t *desc, uint32_t n, nsd_rec *rec, uint32_t *ext,
		    uint32_t *ext_used, uint64_t *counters, int *status);
int nsd_pipe_wait(nsd_pipe *p);
int nsd_pipe_drain(nsd_pipe *p);
void nsd_pipe_destroy(nsd_pipe *p);

/* ---- LINKTYPE_LINUX_SLL heads (dissector_sll.c:39-82) -----------------------
 * The SLL "cooked" head prints the packet's struct sockaddr_ll (pkt->sll,
 * dissector.c:74: the RX ring's per-frame sockaddr_ll, or the *_LL pcap
 * record's cooked header) and, in print_full, continues in eth_lay2 with
 * sll_protocol when the hatype maps to Ethernet (pcap_devtype_to_linktype).
 * nsd_sll_t is struct sockaddr_ll's layout (20 bytes).  Batches of an SLL
 * link type pass one per packet (NULL reads as zeros). */
typedef struct nsd_sll {
	uint16_t family;
	uint16_t protocol;   /* network byte order */
	int32_t  ifindex;
	uint16_t hatype;
	uint8_t  pkttype;
	uint8_t  halen;
	uint8_t  addr[8];
} nsd_sll_t;
int nsd_dissect_device_sll(const uint8_t *d_frames, const nsd_desc_t *d_desc,
			   const nsd_sll_t *d_sll, uint32_t n, int linktype, int mode,
			   nsd_rec *d_rec, uint32_t *d_ext, uint32_t ext_words,
			   uint32_t *d_ext_used, uint64_t *d_counters, void *d_workspace,
			   void *stream);
int dissector_entry_batch_sll(const uint8_t *frames, size_t frames_len,
			      const nsd_desc_t *desc, const nsd_sll_t *sll, uint32_t n,
			      int linktype, int mode, nsd_rec *rec, uint32_t *ext,
			      uint32_t ext_words, uint32_t *ext_used, uint64_t *counters);
long nsd_format_packet_sll(const uint8_t *pkt, uint32_t caplen, int linktype, int mode,
			   const nsd_rec *rec, const uint32_t *ext_pool, const nsd_sll_t *sll,
			   char *out, size_t cap);
/* nsd_format_batch_sll: packets [0, n) into one buffer (per-packet end
 * offsets in ends[], status in rc[], both may be NULL); returns total bytes
 * or -needed when cap is too small.  nsd_pipe_submit_sll: nsd_pipe_submit
 * with one sockaddr_ll per packet (the pipe's link type is an SLL one). */
long nsd_format_batch_sll(const uint8_t *frames, const nsd_desc_t *desc, const nsd_sll_t *sll,
			  uint32_t n, int linktype, int mode, const nsd_rec *rec,
			  const uint32_t *ext_pool, char *out, size_t cap, uint64_t *ends, int8_t *rc);
int nsd_pipe_submit_sll(nsd_pipe *p, const uint8_t *frames, size_t frames_len,
			const nsd_desc_t *desc, const nsd_sll_t *sll, uint32_t n, nsd_rec *rec,
			uint32_t *ext, uint32_t *ext_used, uint64_t *counters, int *status);

/* The per-packet entry's walk alone (no text): one packet -> the record the
 * device writes for it (a chain that needs the ext form gets its pool
 * entry at word 0 of ext, record slot 0, when ext_words allows; else
 * NSD_F_OVERFLOW); counters (may be NULL) accumulate.  Host CPU, the same
 * layer step as the device's general walk. */
int nsd_walk_packet_cpu(const uint8_t *pkt, uint32_t caplen, int linktype, int mode,
			const nsd_sll_t *sll, nsd_rec *rec, uint32_t *ext, uint32_t ext_words,
			uint64_t *counters);

/* ---- compact records (8 bytes per packet) ---------------------------------
 * The walk's results without the cursors: the ops ids, the IPv4 header
 * checksum and the flags, but no layer offsets, final data / tail cursor.
 * A renderer re-derives each of those from the bytes as it prints the
 * layer (every proto_*.c print pulls its own header), so a consumer that
 * renders, as the reference does for every packet, loses nothing; the
 * 16-byte nsd_rec additionally lets it cross-check the device's cursors.
 * Layout (no layer offsets, so a layer past byte 510 needs no ext form):
 *  - up to 6 layers: chain = the ops ids as in nsd_rec, nflags & 7 = count;
 *  - 7..NSD_CREC_MAX_LAYERS layers: chain = ids 0..5, nflags & 7 =
 *    NSD_N_EXT, nlayers = the count, and the batch's ext pool word i (the
 *    packet's side word) holds ids 6.. (5 bits each).  Words [0, n) of the
 *    pool are the side words when ext_words >= n (otherwise such records get
 *    NSD_F_OVERFLOW); pool entries start at word n + *d_ext_used;
 *  - longer chains: chain = the ext pool slot (0xFFFFFFFF with
 *    NSD_F_OVERFLOW: pool full), nflags & 7 = NSD_N_EXT, nlayers = 0; the
 *    entry keeps the ids (offset bits 0: no cursors in this form either).
 * Host-rendered leaves (NSD_F_HOST) also get their end cursor when the pool
 * has side words: NSD_F_LEAF_END, the cursor in the side word (up to 6
 * layers) or in the entry's word 2 (past 12 layers; a 7..12-layer chain's
 * side word holds ids, so its leaf has no recorded end).
 * nflags (besides the count), ip_csum: as in nsd_rec.  The counters are the
 * same as for 16-byte records (NSD_CNT_EXT counts the chains that need the
 * 16-byte record's ext form). */
#define NSD_CREC_MAX_LAYERS  12
typedef struct nsd_crec {
	uint32_t chain;
	uint16_t ip_csum;
	uint8_t  nflags;
	uint8_t  nlayers;
} nsd_crec;

/* nsd_dissect_device_ws / _sll writing n compact records; d_sll as in
 * nsd_dissect_device_sll (NULL: zeros), d_workspace of nsd_workspace_bytes(n) */
int nsd_dissect_device_compact(const uint8_t *d_frames, const nsd_desc_t *d_desc,
			       const nsd_sll_t *d_sll, uint32_t n, int linktype, int mode,
			       nsd_crec *d_crec, uint32_t *d_ext, uint32_t ext_words,
			       uint32_t *d_ext_used, uint64_t *d_counters, void *d_workspace,
			       void *stream);
/* nsd_format_batch_sll over compact records: each layer starts where the
 * previous one's print left the cursor.  A record without its chain (NSD_F_OVERFLOW)
 * gets rc NSD_ERR_FORMAT (render it per packet: dissector_entry_point).
 * Packet i's side word is ext_pool[i]: the call covers a whole launch's
 * batch (for a part of one: nsd_format_range_compact). */
long nsd_format_batch_compact(const uint8_t *frames, const nsd_desc_t *desc, const nsd_sll_t *sll,
			      uint32_t n, int linktype, int mode, const nsd_crec *crec,
			      const uint32_t *ext_pool, char *out, size_t cap, uint64_t *ends,
			      int8_t *rc);

/* Kernel schedule of the batch walks.  NSD_SCHED_SPLIT: a fast kernel
 * (fast walk of every packet at high occupancy) plus a walker kernel over
 * the packets it defers; NSD_SCHED_FUSED: one kernel doing both; results
 * are identical.  NSD_SCHED_ADAPTIVE (the default) picks per device from the
 * recently observed share of deferred packets (split for traffic the fast
 * walk finishes, fused for deep chains).  nsd_set_schedule returns the
 * previous setting (or NSD_ERR_ARG); nsd_last_schedule the schedule of the
 * last launch (NSD_SCHED_SPLIT / _FUSED, 0 before any). */
#define NSD_SCHED_ADAPTIVE 0
#define NSD_SCHED_SPLIT    1
#define NSD_SCHED_FUSED    2
int nsd_set_schedule(int sched);
int nsd_last_schedule(void);
/* nsd_set_grid_cap caps every batch walk's grid at `blocks` blocks (0: none,
 * the default; tests use it to give small batches several tiles per wave).
 * Process-wide; returns the previous cap, or NSD_ERR_ARG. */
int nsd_set_grid_cap(int blocks);
/* nsd_set_record_ring: whether the fused kernel's compact records of tiles
 * with deferred packets go through its per-wave record ring (coalesced
 * stores once a tile is finished; results identical either way): 0
 * adaptive (the default: on for batches whose schedule sample defers more
 * than a quarter of the packets, and until the first sample), 1 on, 2 off.
 * Process-wide (tests); returns the previous setting, or NSD_ERR_ARG. */
int nsd_set_record_ring(int mode);

/* Compact-record pipe: nsd_pipe_create_compact as nsd_pipe_create, its
 * batches walked into nsd_crec records.  The pool needs ext_words >=
 * max_pkts + the entries (its words [0, n) are the batch's side words).
 * nsd_pipe_submit_compact as nsd_pipe_submit_sll with crec[n]: ext[0, n +
 * *ext_used) receives the side words and the entries only when a record of
 * the batch needs either (its counters[NSD_CNT_EXT] or [NSD_CNT_HOST] > 0;
 * otherwise ext is left as it was).  Each submit form refuses the other kind
 * of pipe. */
nsd_pipe *nsd_pipe_create_compact(uint32_t max_pkts, size_t max_frame_bytes, uint32_t ext_words,
				  int depth, int linktype, int mode);
int nsd_pipe_submit_compact(nsd_pipe *p, const uint8_t *frames, size_t frames_len,
			    const nsd_desc_t *desc, const nsd_sll_t *sll, uint32_t n, nsd_crec *crec,
			    uint32_t *ext, uint32_t *ext_used, uint64_t *counters, int *status);
/* nsd_format_batch_compact over packets [lo, hi) of a launch's batch: desc,
 * sll (may be NULL) and crec are the whole batch's arrays and ext_pool its
 * pool, so a range's side words are found at their batch index (what lets
 * a caller split one batch over threads; nsd_format_batch_compact itself
 * must be given the whole batch).  ends[k - lo] / rc[k - lo] per packet. */
long nsd_format_range_compact(const uint8_t *frames, const nsd_desc_t *desc, const nsd_sll_t *sll,
			      uint32_t lo, uint32_t hi, int linktype, int mode, const nsd_crec *crec,
			      const uint32_t *ext_pool, char *out, size_t cap, uint64_t *ends, int8_t *rc);

/* ---- the frame header line (show_frame_hdr / __show_frame_hdr,
 * dissector.h:31-116) ----------------------------------------------------------
 * Every capture loop prints it right before it calls dissector_entry_point
 * for a packet: read_pcap (netsniff-ng.c:732), walk_t3_block (:1021), the
 * TPACKET_V2 ring loop (:1153), the forwarding loops (:368, :538).
 * nsd_frame_hdr_t holds what __show_frame_hdr reads from the tpacket header:
 *   - v3 == 0: a struct tpacket2_hdr, as read_pcap fills its frame_map
 *     (zeroed once, netsniff-ng.c:672) with pcap_pkthdr_to_tpacket_hdr
 *     (pcap_io.h:594-709): tp_len, tp_sec, tp_nsec per record format,
 *     tp_status 0.  Built with HAVE_TPACKET3, tpacket_has_vlan_info reads
 *     the status through the tpacket3_hdr view (ring.h:71-84), i.e. this
 *     header's tp_nsec: a nsec value with bit 4 or 6 set prints the
 *     " [ tpacketv3 VLAN ... ]" line with tci 0 / proto 0;
 *   - v3 == 1: the frame's struct tpacket3_hdr in a TPACKET_V3 block
 *     (tp_len, tp_sec, tp_nsec, tp_status, hv1.tp_vlan_tci / tp_vlan_tpid).
 * The sockaddr_ll gives the packet type ("<", "B", "M", "P", ">", "K->U",
 * "U->K", else "?") and the interface (if_indextoname, "?" when it fails);
 * a LINKTYPE_NETLINK packet of >= 16 bytes marked PACKET_OUTGOING is shown
 * as kernel / user by its nlmsg_pid (dissector.h:71-75).
 * nsd_format_frame_hdr: the line for one packet (`count` = the loop's
 * packet counter, 1 for the first); NUL-terminated when room, returns its
 * length (PRINT_NONE: 0).
 * nsd_format_range_compact_fh: nsd_format_range_compact with each packet's
 * frame header in front of its text (fh[i], sll[i] (NULL: zeros), count
 * first_count + i); fh NULL = nsd_format_range_compact. */
typedef struct nsd_frame_hdr {
	uint32_t len;        /* tp_len */
	uint32_t sec;        /* tp_sec */
	uint32_t nsec;       /* tp_nsec */
	uint32_t status;     /* tp_status */
	uint32_t vlan_tci;   /* v3: hv1.tp_vlan_tci */
	uint16_t vlan_tpid;  /* v3: hv1.tp_vlan_tpid */
	uint8_t  v3;         /* 1: tpacket3_hdr (walk_t3_block), 0: tpacket2_hdr */
	uint8_t  reserved;
} nsd_frame_hdr_t;
long nsd_format_frame_hdr(const nsd_frame_hdr_t *fh, const nsd_sll_t *sll, const uint8_t *pkt,
			  uint32_t caplen, int linktype, int mode, uint64_t count, char *out, size_t cap);
long nsd_format_range_compact_fh(const uint8_t *frames, const nsd_desc_t *desc, const nsd_sll_t *sll,
				 const nsd_frame_hdr_t *fh, uint64_t first_count, uint32_t lo, uint32_t hi,
				 int linktype, int mode, const nsd_crec *crec, const uint32_t *ext_pool,
				 char *out, size_t cap, uint64_t *ends, int8_t *rc);

/* ---- pcap replay front end (`netsniff-ng --in f.pcap`, read_pcap
 * netsniff-ng.c:640-770; pcap_io.h / pcap_sg.c record formats) ---------------
 * nsd_pcap_open: validates the file header (tcpdump usec / nsec, Kuznetzov,
 * Borkmann magics, either byte order, version 2.4; SLL / netlink files use the
 * *_LL record form), NULL on error.  nsd_pcap_linktype: the header's link
 * type as stored (byte-swapped files pass it swapped, as the reference does).
 * nsd_pcap_read_batch: reads up to max_n records into frames[0, cap) at
 * 16-byte aligned offsets (NSD_FRAME_PAD zero bytes kept after the last),
 * desc[k] = NSD_DESC(offset, caplen); wire_len / ts_ns (may be NULL) receive
 * the record lengths and timestamps.  Returns the records read, 0 at the end
 * (a record with caplen 0 or above 1 MiB ends the replay like pcap_sg_read's
 * -EINVAL), or NSD_ERR_ARG.
 * nsd_replay_pcap: the whole replay loop: read -> optional device BPF filter
 * -> pipelined device walk -> formatter -> [tprintf wrap at `cols` > 0] ->
 * out_fd, in file order (a *_LL file's cooked headers reach the SLL head as
 * each packet's sockaddr_ll); counters (may be NULL) accumulates the counter
 * vector; `threads` host threads format each batch (<= 0: up to 16).
 * Returns the records printed or a negative NSD_ERR_*.
 * A regular file is mapped whole at nsd_pcap_open (pcap_mm.c's way): the
 * replay is a snapshot of the file as it was at open - records appended
 * later are not read, and a truncation by another process while it is
 * replayed faults the reader (SIGBUS), as the reference's mapped reader
 * would.  NSD_PCAP_MMAP=0 in the environment reads with read() instead
 * (pcap_sg.c's way: a growing file is followed to its current end).
 * Interface names (the frame header line) are looked up afresh by each
 * replay. */
typedef struct nsd_pcap nsd_pcap;
struct nsd_bpf_prog;
nsd_pcap *nsd_pcap_open(const char *path);
int nsd_pcap_linktype(const nsd_pcap *p);
long nsd_pcap_read_batch(nsd_pcap *p, uint8_t *frames, size_t cap, nsd_desc_t *desc,
			 uint32_t max_n, uint32_t *wire_len, uint64_t *ts_ns);
/* as nsd_pcap_read_batch, also filling sll[k] (may be NULL) as read_pcap
 * fills fm.s_ll (netsniff-ng.c:672, 727; pcap_pkthdr_to_tpacket_hdr ->
 * ll_to_sockaddr, pcap_io.h:182-191, 594-660): every sockaddr_ll field that
 * conversion sets - the *_LL record's cooked header; ifindex / protocol /
 * pkttype (Kuznetzov); ifindex / protocol / hatype / pkttype (Borkmann) -
 * and zeros elsewhere (r04: Kuznetzov / Borkmann records used to leave
 * zeros; read_batch_fh below fills the same fields). */
long nsd_pcap_read_batch_sll(nsd_pcap *p, uint8_t *frames, size_t cap, nsd_desc_t *desc,
			     nsd_sll_t *sll, uint32_t max_n, uint32_t *wire_len, uint64_t *ts_ns);
/* as nsd_pcap_read_batch_sll, also filling fh[k] (may be NULL) with the
 * tpacket2_hdr fields read_pcap prints (pcap_pkthdr_to_tpacket_hdr,
 * pcap_io.h:594-709: tp_nsec = usec * 1000 for the usec and Kuznetzov
 * forms, the ns field for nsec / Borkmann, byte-swapped files swapped, *_LL
 * lengths minus the 16-byte cooked header), and sll[k] with every field that
 * conversion sets: the cooked header (*_LL), ifindex / protocol / pkttype
 * (Kuznetzov), ifindex / protocol / hatype / pkttype (Borkmann). */
long nsd_pcap_read_batch_fh(nsd_pcap *p, uint8_t *frames, size_t cap, nsd_desc_t *desc,
			    nsd_sll_t *sll, nsd_frame_hdr_t *fh, uint32_t max_n);
void nsd_pcap_close(nsd_pcap *p);
/* nsd_pcap_index: a mapped pcap file's record walk (the one read_pcap's
 * readers take record by record, pcap_mm.c:67 pcap_mm_read) as the replay
 * reader builds it (windows of `window` bytes, 0 = the replay's; each cut into
 * `chunks` walked in parallel from guessed record starts and spliced onto
 * the exact walk): the first max_n records' header offsets and caplens.
 * Returns the records found (read_batch's end rule) or NSD_ERR_ARG. */
long nsd_pcap_index(const char *path, uint64_t window, int chunks, uint64_t *off, uint32_t *caplen,
		    size_t max_n);
long nsd_replay_pcap(const char *path, int mode, const struct nsd_bpf_prog *filter, int out_fd,
		     int cols, uint64_t *counters, int threads);
/* nsd_replay_pcap plus `--out f.pcap` (read_pcap netsniff-ng.c:636, 693-697,
 * 739-746): with pcap_fd >= 0 writes the file header pcap_generic_push_fhdr
 * writes for the replayed file's magic / link type, then every record that
 * passed the filter exactly as read (record header, *_LL cooked header,
 * bytes), in file order; pcap_fd < 0 is nsd_replay_pcap. */
long nsd_replay_pcap_out(const char *path, int mode, const struct nsd_bpf_prog *filter, int out_fd,
			 int cols, uint64_t *counters, int threads, int pcap_fd);

/* ---- TPACKET_V3 RX ring front end (walk_t3_block, netsniff-ng.c:990-1039) --
 * nsd_t3_block_desc: descriptors for the frames of one retired ring block
 * (tpacket_block_desc + tpacket3_hdr chain), pointing into the block itself:
 * submit the block as the batch's frame buffer (nsd_pipe_submit(block,
 * block_len, desc, n, ...)) and hand it back to the kernel when that batch
 * completes (the reference hands it back after the whole block,
 * netsniff-ng.c:1121).  skip_packet (netsniff-ng.c:425-442): packet_type >= 0
 * keeps only that sll_pkttype, else loopback (lo_ifindex) PACKET_OUTGOING
 * frames are dropped.  Returns the frames described, or NSD_ERR_ARG for an
 * inconsistent block or more than max_n frames. */
long nsd_t3_block_desc(const uint8_t *block, size_t block_len, int packet_type, int lo_ifindex,
		       nsd_desc_t *desc, uint32_t max_n);
/* as nsd_t3_block_desc, also copying each kept frame's struct sockaddr_ll
 * (hdr + 48) into sll[k] (may be NULL), for the SLL heads */
long nsd_t3_block_desc_sll(const uint8_t *block, size_t block_len, int packet_type,
			   int lo_ifindex, nsd_desc_t *desc, nsd_sll_t *sll, uint32_t max_n);
/* as nsd_t3_block_desc_sll, also filling fh[k] (may be NULL) from each kept
 * frame's tpacket3_hdr (v3 = 1), what walk_t3_block's __show_frame_hdr
 * prints (netsniff-ng.c:1021) */
long nsd_t3_block_desc_fh(const uint8_t *block, size_t block_len, int packet_type, int lo_ifindex,
			  nsd_desc_t *desc, nsd_sll_t *sll, nsd_frame_hdr_t *fh, uint32_t max_n);

/* ---- classic BPF on the device --------------------------------
 * The capture loop filters every record before dissecting it (read_pcap
 * netsniff-ng.c:707-725: bpf_run_filter, bpf.c:508-705, skips the record on
 * 0).  Programs are struct sock_filter arrays (linux/filter.h), as
 * bpf_parse_rules (bpf.c:707-766) reads them.
 *
 * nsd_bpf_validate: __bpf_validate (bpf.c:388-506), 1 = valid, 0 = not.
 * nsd_bpf_load: validates, decodes and uploads a program; NULL if it is
 * invalid, longer than 4096 instructions (BPF_MAXINSNS), has a jump whose
 * target leaves the program in 64-bit arithmetic (which __bpf_validate's
 * 32-bit check lets through and the reference then runs off its program),
 * or there is no device.
 * nsd_bpf_filter_device: device pointers, enqueued on `stream`; d_verdict[i]
 * = bpf_run_filter's return for packet i (0 = drop).  With d_desc_out (and
 * d_count, d_workspace of nsd_bpf_workspace_bytes(n) bytes) the descriptors
 * of the accepted packets are packed in batch order into d_desc_out and
 * their number written to *d_count: the dissect kernels' input.
 * nsd_bpf_filter_batch: host memory in and out, synchronous. */
typedef struct nsd_bpf_insn {
	uint16_t code;
	uint8_t  jt;
	uint8_t  jf;
	uint32_t k;
} nsd_bpf_insn;
typedef struct nsd_bpf_prog nsd_bpf_prog;
int nsd_bpf_validate(const nsd_bpf_insn *prog, uint32_t len);
nsd_bpf_prog *nsd_bpf_load(const nsd_bpf_insn *prog, uint32_t len);
void nsd_bpf_free(nsd_bpf_prog *prog);
size_t nsd_bpf_workspace_bytes(uint32_t n);
int nsd_bpf_filter_device(const nsd_bpf_prog *prog, const uint8_t *d_frames,
			  const nsd_desc_t *d_desc, uint32_t n, uint32_t *d_verdict,
			  nsd_desc_t *d_desc_out, uint32_t *d_count, void *d_workspace,
			  void *stream);
int nsd_bpf_filter_batch(const nsd_bpf_prog *prog, const uint8_t *frames, size_t frames_len,
			 const nsd_desc_t *desc, uint32_t n, uint32_t *verdict);

/* Pinned host memory for the pipe's buffers. */
void *nsd_host_alloc(size_t len);
void nsd_host_free(void *ptr);
int nsd_host_register(void *ptr, size_t len);
int nsd_host_unregister(void *ptr);

/* Library / device info. */
const char *nsd_version(void);
/* the compile line the library was built with (bench lines record it) */
const char *nsd_build_info(void);
int nsd_device_count(void);

#ifdef __cplusplus
}
#endif

#endif /* NETSNIFF_DISSECT_H */
