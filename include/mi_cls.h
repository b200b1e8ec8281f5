/*
 * mi_cls.h -- thin C ABI between the (C) ODP host side and the hand-written
 * gfx950 HIP kernels of the MI355X packet parse + PMR classify path.
 *
 * This ABI is the device-side, batch form of the two per-packet internal
 * calls that every linux-generic pktio driver's .recv op makes
 * (pktio_if_ops_t.recv, platform/linux-generic/include/odp_packet_io_internal.h:222;
 * loop driver: platform/linux-generic/pktio/loop.c:253-384):
 *
 *   _odp_packet_parse_common()   platform/linux-generic/include/odp_parse_internal.h:80-112
 *   _odp_cls_classify_packet()   platform/linux-generic/odp_classification.c:1742-1771
 *
 * One call of mi_cls_classify() replaces the per-packet pair for a whole
 * batch of contiguous packets already resident in device memory.  All
 * pointers are plain device pointers; the caller owns every buffer.  Every
 * entry point returns 0 on success or a negative errno.
 *
 * Threading: one mi_cls_ctx_t per GPU; calls on one context are
 * serialised by the caller (mirrors the reference's lock-free data plane
 * reading rule tables that the control plane snapshots, odp_classification.c:1373).
 */
#ifndef MI_CLS_H_
#define MI_CLS_H_

#ifndef __HIPCC_RTC__
#include <stddef.h>
#endif
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------
 * Per-packet result record (16 bytes, written by the kernel).
 * Mirrors the packet-header fields the reference fills in
 * (odp_packet_hdr_t.p / .cos / .dst_queue / .cls_mark,
 *  platform/linux-generic/include/odp_packet_internal.h:55-70,112,116,139):
 *   in_flags  - low 32 bits of packet_parser_t.input_flags.all (bits >= 32
 *               are never set by this path; layout: packet_inline_types.h:60-107)
 *   err       - flags.all.error, 7 bits: snap_len, ip, l3_chksum, tcp, udp,
 *               sctp, l4_chksum (packet_inline_types.h:152-165)
 *   outcome   - MI_CLS_OUT_* below (the 0 / 1 / -1 return protocol of
 *               _odp_packet_parse_common and _odp_cls_classify_packet)
 *   cos       - CoS index (cos_t.index, the slot number), 0xFF when none
 *   hops      - number of PMR matches on the CoS descent (diagnostic)
 *   queue     - queue slot inside the CoS: 0 for a single-queue CoS, the
 *               Toeplitz hash slot for a hash-queue CoS (get_dest_queue,
 *               odp_classification.c:395-405); the host maps (cos, slot) to
 *               the odp_queue_t handle
 *   mark      - hdr->cls_mark (valid when in_flags bit 0, cls_mark, is set)
 *   l3/l4     - packet_parser_t.l3_offset / l4_offset (0xFFFF = invalid);
 *               l2_offset is always 0 on this path and is not stored.
 * ---------------------------------------------------------------------- */
typedef struct mi_cls_result {
	uint32_t in_flags;
	uint8_t  err;
	uint8_t  outcome;
	uint8_t  cos;
	uint8_t  hops;
	uint16_t queue;
	uint16_t mark;
	uint16_t l3_offset;
	uint16_t l4_offset;
} mi_cls_result_t;

enum {
	MI_CLS_OUT_ENQ        = 0, /* classify returned 0: enqueue to (cos, queue)        */
	MI_CLS_OUT_COS_DROP   = 1, /* classify returned 1: CoS action DROP (silent drop)   */
	MI_CLS_OUT_DISCARD    = 2, /* classify returned -1: no CoS (in_discards++)         */
	MI_CLS_OUT_PARSE_DROP = 3, /* parse returned -1: truncated L4 header (in_errors++) */
	MI_CLS_OUT_LOOP       = 4  /* CoS graph cycle: the reference never returns here    */
};

/* ------------------------------------------------------------------------
 * Compiled rule table ("snapshot" of the control-plane CoS/PMR tables,
 * platform/linux-generic/include/odp_classification_datamodel.h:126-206).
 * One contiguous, position-independent little-endian blob of 32-bit words:
 *   mi_tbl_hdr_t | mi_cos_t[num_cos] | mi_rule_t[num_rules] | mi_term_t[num_terms]
 * Rules of a CoS are stored contiguously in cos->pmr[] order (the order the
 * reference scans them, match_pmr_cos, odp_classification.c:1631), with
 * entries whose linked CoS is invalid already removed (:1635-1636).
 * ---------------------------------------------------------------------- */
#define MI_CLS_TBL_MAGIC   0x534C434Du /* "MCLS" */
#define MI_CLS_TBL_VERSION 1u

typedef struct mi_tbl_hdr {
	uint32_t magic;
	uint32_t version;
	uint32_t total_bytes;
	uint32_t num_cos;       /* CoS slots described (= max slot used + 1)          */
	uint32_t num_rules;
	uint32_t num_terms;
	int32_t  default_cos;   /* slot, -1 = none (classifier_t.default_cos)         */
	int32_t  error_cos;     /* slot, -1 = none (classifier_t.error_cos)           */
	uint32_t default_valid; /* default_cos->valid at snapshot time (:1712)        */
	uint32_t used_kinds;    /* bit per MI_K_* present anywhere in the table       */
	uint32_t max_hops;      /* descent bound (cycle guard)                        */
	uint32_t cos_off;       /* byte offsets of the three arrays from the header   */
	uint32_t rule_off;
	uint32_t term_off;
	uint32_t generation;    /* control-plane generation this snapshot reflects    */
	uint32_t rsv;
} mi_tbl_hdr_t;

typedef struct mi_cos {
	uint32_t rule_begin;
	uint32_t num_rules;
	uint8_t  action;        /* 0 enqueue, 1 drop (odp_cos_action_t)              */
	uint8_t  num_queue;     /* 1..32                                             */
	uint8_t  hash_proto;    /* cos_t.hash_proto: bit0 ipv4, 1 ipv6, 2 udp, 3 tcp */
	uint8_t  index;         /* cos_t.index                                       */
	uint32_t valid;
} mi_cos_t;

typedef struct mi_rule {
	uint32_t term_begin;
	uint16_t num_terms;     /* 0..8; 0 matches everything                       */
	uint16_t mark;
	uint32_t dst_cos;       /* linked CoS slot                                  */
	uint32_t rsv;
} mi_rule_t;

/* Compiled term kinds (one per verify_pmr_<term>, odp_classification.c:931-1357) */
enum {
	MI_K_LEN = 0,      /* frame_len (host order) & mask == value                 */
	MI_K_ETH0,         /* raw bytes at l2+12, gate eth                           */
	MI_K_ETHX,         /* raw bytes at l2+16 / +20 (qinq), gate vlan|qinq        */
	MI_K_VID0,         /* raw tci at l2+14 & be16(0x0fff), gate eth&vlan         */
	MI_K_VIDX,         /* raw tci at l2+14 / +18, & be16(0x0fff), gate vlan|qinq */
	MI_K_PCP0,         /* tci>>13 (host order), gate eth&vlan                    */
	MI_K_DMAC,         /* 6 raw bytes at l2, gate eth                            */
	MI_K_PROTO,        /* ipv4 proto / ipv6 fixed next_hdr, gate ipv4|ipv6       */
	MI_K_DSCP,         /* tos>>2 / (vtf&0x0fc00000)>>22, gate ipv4|ipv6          */
	MI_K_UDP_DPORT,
	MI_K_TCP_DPORT,
	MI_K_UDP_SPORT,
	MI_K_TCP_SPORT,
	MI_K_SIP,
	MI_K_DIP,
	MI_K_SIP6,
	MI_K_DIP6,
	MI_K_SPI,          /* l4+4 (AH) / l4+0 (ESP)                                 */
	MI_K_NEVER,        /* LD_VNI: accepted at create, never matches (:1250)      */
	MI_K_CUSTOM_FRAME, /* bytes at offset, gate len > offset+size                */
	MI_K_CUSTOM_L3,    /* bytes at l3+offset, gate l2 & l3 valid & len > ...     */
	MI_K_ALWAYS,       /* INNER_HDR_OFF: always passes (:1504)                   */
	MI_K_COUNT
};

typedef struct mi_term {
	uint8_t  kind;          /* MI_K_*                                            */
	uint8_t  size;          /* val_sz                                            */
	uint16_t rsv0;
	uint32_t offset;        /* custom offset                                     */
	uint32_t rsv1[2];
	uint32_t mask[4];       /* little-endian packing of the mask bytes           */
	uint32_t value[4];      /* pre-masked value bytes (pmr_create_term, :757)    */
} mi_term_t;

/* ------------------------------------------------------------------------
 * Context and entry points
 * ---------------------------------------------------------------------- */
typedef struct mi_cls_ctx mi_cls_ctx_t;

/* Number of visible HIP devices (>= 0), or a negative errno. */
int mi_cls_device_count(void);

/* Create a classification context bound to HIP device `device`. */
int mi_cls_ctx_create(int device, mi_cls_ctx_t **ctx);
int mi_cls_ctx_destroy(mi_cls_ctx_t *ctx);

/* Upload a compiled rule table (host memory, mi_tbl_hdr_t blob) to the
 * context's device copy, stream-ordered on `stream` (hipStream_t, NULL =
 * default stream).  Validates the blob; -EINVAL on a malformed table. */
int mi_cls_rules_load(mi_cls_ctx_t *ctx, const void *tbl, size_t bytes, void *stream);

/* Parse + classify n packets.
 *   pkts_dev  packed packet bytes; each packet starts at pkts_dev + off_dev[i]
 *             (any alignment).  Loads are 16-B pieces at frame-relative
 *             offsets, so the buffer must be readable up to
 *             off_dev[i] + round_up(len_dev[i], 16) for every packet: when
 *             off_dev[i] is not a multiple of 16 that is up to 15 bytes past
 *             the next 16-byte boundary after the packet (a batch whose
 *             allocation ends right after its last frame needs 16 B of slack).
 *   off_dev   uint32 byte offsets, len_dev uint16 frame lengths (FCS stripped)
 *   out_dev   n result records
 * Stream-ordered on `stream`; returns after the launch is enqueued. */
int mi_cls_classify(mi_cls_ctx_t *ctx, const uint8_t *pkts_dev, const uint32_t *off_dev,
		    const uint16_t *len_dev, uint32_t n, mi_cls_result_t *out_dev,
		    void *stream);

/* Host-memory batch (the pktio receive path, loop.c:253-384 / pcap.c:280-401):
 * classifies n frames packed at pkts_host (offsets relative to it, every
 * frame inside `bytes`), writes the n records to out_host and waits.
 * When pkts_host, off_host, len_host and out_host are all page-locked
 * (mi_cls_host_alloc, hipHostMalloc, hipHostRegister) the kernel reads the
 * frames' header windows and the descriptors in place and writes the records
 * in place (zero copy: only the bytes it touches cross the host link);
 * otherwise the frames and descriptors are copied to the context's device
 * staging buffers on its own stream and the records copied back. */
int mi_cls_classify_host(mi_cls_ctx_t *ctx, const uint8_t *pkts_host, size_t bytes,
			 const uint32_t *off_host, const uint16_t *len_host, uint32_t n,
			 mi_cls_result_t *out_host);

/* Pipelined form of mi_cls_classify_host: enqueue the batch on the context's
 * stream and return a ticket (0 for n == 0); mi_cls_classify_host_wait(ticket)
 * returns once its records are in out_host.  The caller leaves all four
 * buffers untouched in between.  Up to 8 batches may be in flight; batches
 * complete in submission order.  A rule load waits for the batches in
 * flight, which classify under the rules they were submitted with.
 * Replaces nothing in the reference (its receive burst parses
 * synchronously, pktio/loop.c:253-384): it lets the runtime overlap one
 * burst's classification with delivering the previous one. */
int mi_cls_classify_host_submit(mi_cls_ctx_t *ctx, const uint8_t *pkts_host, size_t bytes,
				const uint32_t *off_host, const uint16_t *len_host, uint32_t n,
				mi_cls_result_t *out_host, uint64_t *ticket);
int mi_cls_classify_host_wait(mi_cls_ctx_t *ctx, uint64_t ticket);

/* Program-specialised kernel of the loaded rules.  A program whose default
 * CoS has a classification block and whose rules do not form a CoS tree
 * gets a kernel with that block compiled in as constants (hipRTC, in the
 * background after mi_cls_rules_load; launches use the generic kernel until
 * it is ready -- the records are the same either way).  Blocks until the
 * compilation of the loaded program's kernel has ended: 0 = the specialised
 * kernel is in use, 1 = none (no such block, a CoS tree, disabled by
 * MI_CLS_JIT=0, or it failed to compile), -EINVAL = no rules loaded. */
int mi_cls_spec_wait(mi_cls_ctx_t *ctx);

/* Host-only (no device needed): compile the specialised kernel of a
 * compiled table's program for block shape nw (4, 12, 16) synchronously
 * (the tree form for CoS trees, which the data path does not use).
 * 0 compiled, 1 the default CoS has no classification block, < 0 error
 * (-ENOEXEC: the compile failed).  Tests use it to check the embedded
 * kernel sources build. */
int mi_cls_spec_compile(const void *tbl, size_t bytes, int nw);

/* State of the specialised-kernel compiler (host only): *running = compiler
 * processes alive (at most 1: one compile at a time), *queued = 1 if a
 * request waits to start (a newer request replaces it), *cached = distinct
 * programs kept (at most 64; later programs run the generic kernels).
 * Returns 1 while the compile thread is active, else 0. */
int mi_cls_spec_pending(uint32_t *running, uint32_t *queued, uint32_t *cached);

/* The kernel instantiation the context's last mi_cls_classify launched
 * (diagnostics: bench lines and fault records name it).  info[0] waves per
 * block, [1] 1 if the hot region was in LDS, [2] 1 if the per-lane CoS-tree
 * rounds were compiled in (DIV), [3] flat engine + 1 (0: not a flat
 * kernel), [4] 1 if program-specialised, [5] 1 if the pktin-option kernel
 * (CK), [6] grid (blocks).  All zero before the first launch.  Returns the
 * number of words written (min(n, MI_CLS_LAUNCH_INFO_WORDS)) or -EINVAL. */
#define MI_CLS_LAUNCH_INFO_WORDS 7
int mi_cls_last_launch(const mi_cls_ctx_t *ctx, uint32_t *info, uint32_t n);

/* ------------------------------------------------------------------------
 * Multi-GPU: one host batch over several devices.
 * The batch shards with no exchange step: mi_cls_shard cuts it into
 * contiguous slices balanced by the bytes the kernel reads per packet
 * (min(len,128) + 6 B descriptor + 16 B record); each slice is staged,
 * classified and copied back on its own context and stream, all devices in
 * flight at once; the records land at their packets' positions in `out`, so
 * the result is the single-device result and per-queue arrival order is the
 * one the reference's _odp_cls_enq runs see
 * (platform/linux-generic/include/odp_classification_internal.h:208-236).
 * Replaces running the per-burst loopback_recv (pktio/loop.c:253-384) once
 * per device.
 * ---------------------------------------------------------------------- */
typedef struct mi_cls_group mi_cls_group_t;

/* begin[0..nshards]: slice k is packets [begin[k], begin[k+1]). */
int mi_cls_shard(const uint16_t *len, uint32_t n, uint32_t nshards, uint32_t *begin);

/* One context per entry of devices[] (an id may repeat: several contexts on
 * one device). */
int mi_cls_group_create(const int *devices, uint32_t n, mi_cls_group_t **group);
int mi_cls_group_destroy(mi_cls_group_t *group);
uint32_t mi_cls_group_size(const mi_cls_group_t *group);
mi_cls_ctx_t *mi_cls_group_ctx(mi_cls_group_t *group, uint32_t i);
/* The rule table replicated to every device (synchronous). */
int mi_cls_group_rules_load(mi_cls_group_t *group, const void *tbl, size_t bytes);
int mi_cls_group_pktin_opt_set(mi_cls_group_t *group, uint64_t opt);
/* As mi_cls_classify_host, sharded over the group's devices; returns when
 * every record is in out_host.  Pinned input (mi_cls_host_alloc) lets the
 * devices' copies overlap. */
int mi_cls_group_classify_host(mi_cls_group_t *group, const uint8_t *pkts_host, size_t bytes,
			       const uint32_t *off_host, const uint16_t *len_host, uint32_t n,
			       mi_cls_result_t *out_host);

/* Pipelined form of mi_cls_group_classify_host (the multi-GPU receive
 * path's submit / wait, as mi_cls_classify_host_submit for one context):
 * every device's slice is put in flight and a ticket returned;
 * mi_cls_group_classify_host_wait(ticket) returns once all records are in
 * out_host.  Batch, descriptors and records must be page-locked
 * (mi_cls_host_alloc) to be read and written in place; otherwise the batch
 * is classified synchronously and *ticket is 0 (done).  Up to 8 batches in
 * flight, completed in submission order.  Replaces running the receive
 * burst (pktio/loop.c:253-384) once per device, synchronously. */
int mi_cls_group_classify_host_submit(mi_cls_group_t *group, const uint8_t *pkts_host, size_t bytes,
				      const uint32_t *off_host, const uint16_t *len_host, uint32_t n,
				      mi_cls_result_t *out_host, uint64_t *ticket);
int mi_cls_group_classify_host_wait(mi_cls_group_t *group, uint64_t ticket);

/* pktin parse options for the following classify calls on this context:
 * odp_pktin_config_opt_t.all_bits (include/odp_rt.h; reference
 * include/odp/api/spec/packet_io.h odp_pktin_config_opt_t).  Bits 2-5
 * validate the IPv4 header / UDP / TCP / SCTP checksums (odp_parse.c:134-141,
 * 298-313, odp_packet.c:2065-2138: l3/l4_chksum_done in in_flags bits 30/31,
 * l3/l4_chksum_err in err bits 2/6), bits 6-10 drop packets with IPv4 /
 * IPv6 / UDP / TCP / SCTP errors (MI_CLS_OUT_PARSE_DROP).  0 (the default)
 * is the plain parse.  Replaces the `opt` argument of
 * _odp_packet_parse_common (include/odp_parse_internal.h:80-112). */
int mi_cls_pktin_opt_set(mi_cls_ctx_t *ctx, uint64_t opt);

/* ------------------------------------------------------------------------
 * Receive delivery on the GPU: the host steps of loopback_recv /
 * pcapif_recv_pkt after classification (pktio/loop.c:308-373, pcap.c:
 * 330-352) for packets whose headers and buffers are in page-locked host
 * memory the device addresses at the host's addresses: each packet's
 * metadata (_odp_packet_parse_common's result at the pktio's parser layer,
 * hdr->cos / cls_mark / dst_queue of _odp_cls_classify_packet, input pktio)
 * written into its header, its frame copied into its buffer (pcap frames,
 * pool switch, _odp_pktio_packet_to_pool), and the stable group-by-queue
 * permutation of _odp_cls_enq's runs (include/odp_classification_internal.h:
 * 208-236: each queue receives its packets in arrival order).
 * ---------------------------------------------------------------------- */

/* The receive-path fields of a packet header (the runtime's packet header
 * embeds this block; odp_packet_hdr_t.p / cos / cls_mark / dst_queue /
 * input, platform/linux-generic/include/odp_packet_internal.h:55-70,112-139). */
typedef struct mi_cls_pkt_meta {
	uint32_t data_off;      /* headroom                                        */
	uint32_t len;
	uint64_t in_flags;      /* packet_parser_t.input_flags                      */
	uint8_t  err;           /* flags.all.error                                  */
	uint8_t  cos;           /* 0xFF none                                        */
	uint16_t cls_mark;
	uint16_t l2, l3, l4;
	uint16_t rsv0;
	uint32_t rsv1;
	uint64_t dst_queue;     /* odp_queue_t                                      */
	uint64_t input;         /* odp_pktio_t                                      */
	uint64_t user_ptr;
	uint64_t rsv2;
} mi_cls_pkt_meta_t;    /* 64 B: one cache line of the header, written whole */

/* One delivered packet (host-written, 48 B). */
typedef struct mi_cls_dlv {
	uint64_t meta;          /* address of its mi_cls_pkt_meta_t (64-B aligned)   */
	uint64_t dst_queue;     /* queue written into meta when the classifier is on */
	uint64_t user_ptr;      /* kept user pointer (not MI_CLS_DLV_FRESH)          */
	uint32_t src;           /* frame offset from the batch base (MI_CLS_DLV_COPY) */
	uint32_t rec;           /* index of its record                              */
	uint16_t len;           /* frame length                                     */
	uint8_t  flags;         /* MI_CLS_DLV_*                                     */
	uint8_t  qid;           /* queue group 0..MI_CLS_DLV_GROUPS-1, 0xFF none    */
	uint32_t data_off;      /* the packet's headroom (kept: not MI_CLS_DLV_FRESH) */
	uint64_t rsv;
} mi_cls_dlv_t;

#define MI_CLS_DLV_FRESH 0x01u  /* newly allocated: initialise every field     */
#define MI_CLS_DLV_COPY  0x02u  /* copy the frame into meta + data_from_meta    */
#define MI_CLS_DLV_CLS   0x04u  /* classifier on: cos / cls_mark / dst_queue    */
#define MI_CLS_DLV_GROUPS 64
/* Entries one delivery groups at most: a burst with more entries must give
 * every entry qid 0xFF (mi_cls_deliver_submit rejects it otherwise). */
#define MI_CLS_DLV_GROUP_MAX 8192

typedef struct mi_cls_dlv_args {
	const uint8_t *base;    /* the classified batch's base (host VA)           */
	const mi_cls_result_t *res;   /* its records                              */
	const mi_cls_dlv_t *dlv;
	uint32_t n;             /* entries of dlv                                   */
	uint32_t layer;         /* parser layer (ODP_PROTO_LAYER_L2..ALL = 1..4)    */
	uint64_t input;         /* odp_pktio_t written into meta                    */
	uint32_t headroom;      /* data_off of fresh packets                        */
	uint32_t data_from_meta;/* bytes from a meta block to the packet's data     */
	uint32_t *perm;         /* out: entry indexes grouped by qid (stable)       */
	uint32_t *gcnt;         /* out: MI_CLS_DLV_GROUPS entry counts per qid       */
} mi_cls_dlv_args_t;

/* Submit the delivery of a classified burst on the context's stream (after
 * its classification) and return a ticket for mi_cls_classify_host_wait.
 * Every pointer is host memory the device reads and writes in place
 * (mi_cls_host_alloc); entries with qid 0xFF are left out of perm.  More
 * than MI_CLS_DLV_GROUP_MAX entries with a queue group: -E2BIG. */
int mi_cls_deliver_submit(mi_cls_ctx_t *ctx, const mi_cls_dlv_args_t *args, uint64_t *ticket);

/* ------------------------------------------------------------------------
 * The receive chain: classification, the per-frame decisions and the
 * delivery of one burst submitted at once, with no host step between them.
 * The host's per-frame decide step of mi_cls_deliver_submit (parse drop,
 * CoS drop / discard, destination pool, too long for the pool, queue group)
 * runs on the device from a per-generation table of the control plane
 * (mi_cls_rxtab_t: CoS -> pool slot, queues, queue groups), and each frame
 * takes its packet from packets the host took from the pools before the
 * submit (pool slot k: got[got_base[k] .. + have[k]), used in arrival order).
 * A burst whose frames need more packets of a slot than were taken reports
 * `short_pool` and is delivered again by the host (nothing it would deliver
 * differently has been enqueued).  Reference steps: loop.c:308-373,
 * pcap.c:330-352, include/odp_packet_io_internal.h:352-371,
 * odp_classification.c:1742-1771, include/odp_classification_internal.h:
 * 142-236.
 * ---------------------------------------------------------------------- */
#define MI_CLS_RX_POOLS 16
#define MI_CLS_RX_QENT 1024
#define MI_CLS_RXT_CLS   0x1u   /* classifier on                               */
#define MI_CLS_RXT_GROUP 0x2u   /* every CoS enqueues plainly to <= 64 queues:   */
				/* group by queue (qg) for one enqueue per queue */
typedef struct mi_cls_rxtab {
	uint32_t flags;               /* MI_CLS_RXT_*                               */
	uint32_t npool;               /* pool slots (slot 0: the pktio's pool)      */
	uint32_t pool_cap[MI_CLS_RX_POOLS];   /* data capacity of each slot's packets */
	uint8_t  rt_slot[64];         /* runtime pool index -> slot + 1 (0: none)   */
	uint8_t  cos_pool[256];       /* CoS index -> pool slot                     */
	uint8_t  cos_nq[256];         /* queues of the CoS                          */
	uint16_t cos_q0[256];         /* its first entry of qh / qg                 */
	uint8_t  rt_pinned[64];       /* runtime pool index -> 1: page-locked pool   */
	uint64_t qh[MI_CLS_RX_QENT];  /* odp_queue_t per (CoS, queue slot)          */
	uint8_t  qg[MI_CLS_RX_QENT];  /* its queue group 0..63 (MI_CLS_RXT_GROUP)   */
	uint64_t stamp;               /* new value whenever the table is rewritten: */
				      /* the device keeps a copy per stamp          */
} mi_cls_rxtab_t;

typedef struct mi_cls_rx_out {
	uint64_t in_errors, in_discards, packets, octets;
	uint32_t used[MI_CLS_RX_POOLS];   /* packets taken of each slot              */
	uint32_t need[MI_CLS_RX_POOLS];   /* frames that wanted a packet of the slot */
	uint32_t short_pool;          /* 1: a slot had too few packets (host redo)  */
	uint32_t not_in_place;        /* loop staging (stage): a packet outside the  */
				      /* page-locked arena (host redo)              */
	uint32_t rsv[2];
} mi_cls_rx_out_t;

/* Frame decision word (dec[i]): fate in bits 0-1, pool slot in bits 2-6,
 * queue group in bits 8-14 (0x7F none), rank among the slot's frames in
 * bits 16-31. */
#define MI_CLS_RXF_DROP    0u   /* parse drop or CoS drop: nothing delivered  */
#define MI_CLS_RXF_DISCARD 1u   /* counted in in_discards                      */
#define MI_CLS_RXF_FRESH   2u   /* a packet of its slot (frame copied)         */
#define MI_CLS_RXF_INPLACE 3u   /* a loop packet received in its own buffer    */

typedef struct mi_cls_rxc_args {
	const uint8_t *base;          /* the burst's frames (soff[i] from here)     */
	const uint32_t *soff;
	const uint16_t *slen;
	mi_cls_result_t *res;         /* records (every frame's, when the ticket is done) */
	uint32_t n;                   /* frames (<= MI_CLS_DLV_GROUP_MAX)           */
	uint32_t layer;               /* parser layer (ODP_PROTO_LAYER_L2..ALL)     */
	uint64_t input;               /* odp_pktio_t written into meta              */
	uint32_t headroom;            /* data_off of fresh packets                  */
	uint32_t data_from_meta;      /* bytes from a meta block to its data        */
	const mi_cls_rxtab_t *tab;
	const uint64_t *got;          /* packets taken per slot (odp_packet_t)      */
	uint32_t got_base[MI_CLS_RX_POOLS], have[MI_CLS_RX_POOLS];
	const uint64_t *pk;           /* loop: each frame's packet, else NULL       */
	const uint8_t *ppool;         /* loop: its runtime pool index + 1           */
	const uint16_t *pdoff;        /* loop: its headroom                         */
	uint32_t meta_off;            /* bytes from a packet handle to its meta     */
	uint32_t stage;               /* loop: the device builds soff / slen / ppool */
				      /* from the packets' headers (pk) first       */
	uint16_t head_off;            /* stage: offset of a header's buffer pointer */
	uint16_t pool_off;            /* stage: offset of its u16 pool index        */
	/* outputs */
	uint32_t *dec;                /* per frame: decision word                   */
	uint64_t *ent;                /* per frame: the delivered packet (0: none)  */
	uint32_t *perm;               /* frames grouped by queue group (stable)     */
	uint32_t *gcnt;               /* MI_CLS_DLV_GROUPS counts                   */
	mi_cls_rx_out_t *out;
} mi_cls_rxc_args_t;

/* Submit a host batch's classification (as mi_cls_classify_host_submit)
 * followed by the decisions and the delivery of args; one ticket for all
 * (mi_cls_classify_host_wait).  Every pointer of args is page-locked host
 * memory the device addresses in place; res / soff / slen / base are the
 * classification's.  -EINVAL: not so, or n too large. */
int mi_cls_rx_chain_submit(mi_cls_ctx_t *ctx, const uint8_t *pkts, size_t bytes,
			   const mi_cls_rxc_args_t *args, uint64_t *ticket);

/* 1 if p lies in page-locked host memory that the device addresses at the
 * same address (the receive delivery's requirement), else 0. */
int mi_cls_host_mapped(const void *p);

/* Pinned (page-locked) host memory for staging; NULL on failure. */
void *mi_cls_host_alloc(size_t bytes);
void mi_cls_host_free(void *p);

/* Per-CoS packet counters with the reference's per-hop counting rule
 * (odp_classification.c:1646-1647, 1721-1723): when enabled, each
 * mi_cls_classify() adds into a device array of num_cos uint64 counters
 * for CoS slots whose stats are enabled (stats_mask bit per slot, up to 256).
 * mi_cls_stats_read copies the counters to host memory (synchronous). */
int mi_cls_stats_enable(mi_cls_ctx_t *ctx, const uint32_t stats_mask[8]);
int mi_cls_stats_read(mi_cls_ctx_t *ctx, uint64_t *host_counters, uint32_t num);
int mi_cls_stats_reset(mi_cls_ctx_t *ctx);

/* Host-only (no device needed): assemble a compiled table into the private
 * device encoding and describe it.  info[0] total 32-bit words, [1] words of
 * the per-lane "hot" region (copied to LDS when it fits), [2] CoS with a
 * classification block, [3..6] blocks per engine (direct, candidate,
 * bitmap, wide bitmap), [7] 1 if some rule leads to a CoS with rules,
 * [8] single-candidate blocks, [9] (when n >= 10) 0 if the program is not
 * flat (decided on the default CoS in one round), else its engine + 1,
 * [10] (n >= 11) CoS whose rules need a chain of blocks (more key classes
 * than one block holds; [2..8] count their first blocks).
 * n >= 9.  Used by tests and tools to check engine selection on the CPU. */
int mi_cls_program_info(const void *tbl, size_t bytes, uint32_t *info, uint32_t n);

/* Last error string for the context (static storage, never NULL). */
const char *mi_cls_strerror(int err);

#ifdef __cplusplus
}
#endif

#endif /* MI_CLS_H_ */
