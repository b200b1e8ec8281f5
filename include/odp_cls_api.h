/*
 * odp_cls_api.h -- the ODP classification API surface served by the MI355X
 * build (libodp_cls.so).  Names, argument meaning, handle conventions and
 * error behaviour follow the reference API:
 *
 *   include/odp/api/spec/classification.h        (types :55-770, functions :779-1158)
 *   include/odp/api/spec/packet_io.h:695-747     (pktio-side CoS setters)
 *   platform/linux-generic/odp_classification.c  (linux-generic semantics)
 *
 * Handles are index+1 and the INVALID handle is 0 (odp_classification.c:60-78).
 * Creation returns INVALID on failure; *_multi returns the number created or -1
 * when the first fails; destroy returns 0 / -1.  The library owns the rule
 * tables; value/mask buffers are copied at create time.
 *
 * Base types, queue / pool handles and odp_queue_param_t come from odp_rt.h
 * (the runtime subset); hash-queue CoS create their queues with
 * odp_queue_create() as the reference does (odp_classification.c:318-341).
 */
#ifndef ODP_AMD_CLS_API_H_
#define ODP_AMD_CLS_API_H_

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#include "odp_rt.h"

#ifdef __cplusplus
extern "C" {
#endif

/* classification.h:55-137 -- enum order is ABI */
typedef enum {
	ODP_PMR_LEN,
	ODP_PMR_ETHTYPE_0,
	ODP_PMR_ETHTYPE_X,
	ODP_PMR_VLAN_ID_0,
	ODP_PMR_VLAN_ID_X,
	ODP_PMR_VLAN_PCP_0,
	ODP_PMR_DMAC,
	ODP_PMR_IPPROTO,
	ODP_PMR_IP_DSCP,
	ODP_PMR_UDP_DPORT,
	ODP_PMR_TCP_DPORT,
	ODP_PMR_UDP_SPORT,
	ODP_PMR_TCP_SPORT,
	ODP_PMR_SIP_ADDR,
	ODP_PMR_DIP_ADDR,
	ODP_PMR_SIP6_ADDR,
	ODP_PMR_DIP6_ADDR,
	ODP_PMR_IPSEC_SPI,
	ODP_PMR_LD_VNI,
	ODP_PMR_CUSTOM_FRAME,
	ODP_PMR_CUSTOM_L3,
	ODP_PMR_IGMP_GRP_ADDR,
	ODP_PMR_ICMP_ID,
	ODP_PMR_ICMP_TYPE,
	ODP_PMR_ICMP_CODE,
	ODP_PMR_SCTP_SPORT,
	ODP_PMR_SCTP_DPORT,
	ODP_PMR_GTPV1_TEID,
	ODP_PMR_INNER_HDR_OFF = 32
} odp_cls_pmr_term_t;

typedef union odp_cls_pmr_terms_t {
	struct {
		uint64_t len:1;
		uint64_t ethtype_0:1;
		uint64_t ethtype_x:1;
		uint64_t vlan_id_0:1;
		uint64_t vlan_id_x:1;
		uint64_t vlan_pcp_0:1;
		uint64_t dmac:1;
		uint64_t ip_proto:1;
		uint64_t ip_dscp:1;
		uint64_t udp_dport:1;
		uint64_t tcp_dport:1;
		uint64_t udp_sport:1;
		uint64_t tcp_sport:1;
		uint64_t sip_addr:1;
		uint64_t dip_addr:1;
		uint64_t sip6_addr:1;
		uint64_t dip6_addr:1;
		uint64_t ipsec_spi:1;
		uint64_t ld_vni:1;
		uint64_t custom_frame:1;
		uint64_t custom_l3:1;
		uint64_t igmp_grp_addr:1;
		uint64_t icmp_id:1;
		uint64_t icmp_type:1;
		uint64_t icmp_code:1;
		uint64_t sctp_sport:1;
		uint64_t sctp_dport:1;
		uint64_t gtpv1_teid:1;
	} bit;
	uint64_t all_bits;
} odp_cls_pmr_terms_t;

/* classification.h:278-321 */
typedef struct odp_pmr_param_t {
	odp_cls_pmr_term_t term;
	odp_bool_t range_term;
	union {
		struct {
			const void *value;
			const void *mask;
		} match;
		struct {
			const void *val_start;
			const void *val_end;
		} range;
	};
	uint32_t val_sz;
	uint32_t offset;
} odp_pmr_param_t;

typedef struct odp_pmr_create_opt_t {
	odp_pmr_param_t *terms;
	int num_terms;
	uint64_t mark;
	uint32_t priority;
} odp_pmr_create_opt_t;

typedef struct odp_threshold_types_t {
	uint8_t all_bits;
} odp_threshold_types_t;

typedef struct odp_cls_cos_stats_t {
	uint64_t octets;
	uint64_t packets;
	uint64_t discards;
	uint64_t errors;
} odp_cls_cos_stats_t;

typedef struct odp_cls_queue_stats_t {
	uint64_t octets;
	uint64_t packets;
	uint64_t discards;
	uint64_t errors;
} odp_cls_queue_stats_t;

typedef struct odp_cls_stats_capability_t {
	struct {
		union {
			struct {
				uint64_t octets   : 1;
				uint64_t packets  : 1;
				uint64_t discards : 1;
				uint64_t errors   : 1;
			} counter;
			uint64_t all_counters;
		};
	} cos;
	struct {
		union {
			struct {
				uint64_t octets   : 1;
				uint64_t packets  : 1;
				uint64_t discards : 1;
				uint64_t errors   : 1;
			} counter;
			uint64_t all_counters;
		};
	} queue;
} odp_cls_stats_capability_t;

typedef struct odp_cls_capability_t {
	odp_cls_pmr_terms_t supported_terms;
	uint32_t max_pmr;
	uint32_t max_pmr_per_cos;
	uint32_t max_terms_per_pmr;
	uint32_t max_pmr_priority;
	uint32_t max_cos;
	uint32_t max_cos_stats;
	uint32_t max_hash_queues;
	odp_pktin_hash_proto_t hash_protocols;
	odp_bool_t pmr_range_supported;
	odp_support_t random_early_detection;
	odp_threshold_types_t threshold_red;
	odp_support_t back_pressure;
	odp_threshold_types_t threshold_bp;
	uint64_t max_mark;
	odp_cls_stats_capability_t stats;
} odp_cls_capability_t;

typedef enum {
	ODP_COS_ACTION_ENQUEUE,
	ODP_COS_ACTION_DROP,
} odp_cos_action_t;

typedef struct odp_red_param_t {
	odp_bool_t enable;
	uint64_t threshold;
} odp_red_param_t;

typedef struct odp_bp_param_t {
	odp_bool_t enable;
	uint64_t threshold;
	uint8_t pfc_level;
} odp_bp_param_t;

/* classification.h:647-770 -- queue and {queue_param, hash_proto} share a union */
typedef struct odp_cls_cos_param {
	odp_cos_action_t action;
	odp_bool_t stats_enable;
	uint32_t num_queue;
	union {
		odp_queue_t queue;
		struct {
			odp_queue_param_t queue_param;
			odp_pktin_hash_proto_t hash_proto;
		};
	};
	odp_pool_t pool;
	odp_red_param_t red;
	odp_bp_param_t bp;
	odp_pktin_vector_config_t vector;
	odp_aggr_enq_profile_t aggr_enq_profile;
} odp_cls_cos_param_t;

/* ---------------------------------------------------------------- API */
void odp_cls_cos_param_init(odp_cls_cos_param_t *param);
int odp_cls_capability(odp_cls_capability_t *capability);
odp_cos_t odp_cls_cos_create(const char *name, const odp_cls_cos_param_t *param);
int odp_cls_cos_create_multi(const char *name[], const odp_cls_cos_param_t param[],
			     odp_cos_t cos[], int num);
int odp_cos_destroy(odp_cos_t cos);
int odp_cos_destroy_multi(odp_cos_t cos[], int num);
int odp_cos_queue_set(odp_cos_t cos, odp_queue_t queue);
odp_queue_t odp_cos_queue(odp_cos_t cos);
uint32_t odp_cls_cos_num_queue(odp_cos_t cos);
uint32_t odp_cls_cos_queues(odp_cos_t cos, odp_queue_t queue[], uint32_t num);
int odp_cls_cos_stats(odp_cos_t cos, odp_cls_cos_stats_t *stats);
int odp_cls_queue_stats(odp_cos_t cos, odp_queue_t queue, odp_cls_queue_stats_t *stats);
void odp_cls_pmr_param_init(odp_pmr_param_t *param);
void odp_cls_pmr_create_opt_init(odp_pmr_create_opt_t *opt);
odp_pmr_t odp_cls_pmr_create(const odp_pmr_param_t *terms, int num_terms,
			     odp_cos_t src_cos, odp_cos_t dst_cos);
odp_pmr_t odp_cls_pmr_create_opt(const odp_pmr_create_opt_t *opt,
				 odp_cos_t src_cos, odp_cos_t dst_cos);
int odp_cls_pmr_create_multi(const odp_pmr_create_opt_t opt[], odp_cos_t src_cos[],
			     odp_cos_t dst_cos[], odp_pmr_t pmr[], int num);
int odp_cls_pmr_destroy(odp_pmr_t pmr);
int odp_cls_pmr_destroy_multi(odp_pmr_t pmr[], int num);
int odp_cls_cos_pool_set(odp_cos_t cos, odp_pool_t pool_id);
odp_pool_t odp_cls_cos_pool(odp_cos_t cos);
uint64_t odp_cos_to_u64(odp_cos_t cos);
uint64_t odp_pmr_to_u64(odp_pmr_t pmr);
void odp_cls_print_all(void);

/* packet_io.h:695-747 */
int odp_pktio_default_cos_set(odp_pktio_t pktio, odp_cos_t default_cos);
int odp_pktio_error_cos_set(odp_pktio_t pktio, odp_cos_t error_cos);
int odp_pktio_skip_set(odp_pktio_t pktio, uint32_t offset);
int odp_pktio_headroom_set(odp_pktio_t pktio, uint32_t headroom);

/* ------------------------------------------------------------------
 * MI355X build extensions (not in the ODP spec).
 * ---------------------------------------------------------------- */

/* Table limits.  The stock linux-generic limits are 64 CoS / 256 PMR /
 * 8 PMR per CoS (odp_classification_datamodel.h:32-40); this build defaults
 * to the raised limits the BASELINE configs need (255 / 8192 / 4096), with
 * unchanged lookup semantics.  Must be called before any other cls call. */
int odp_amd_cls_limits_set(uint32_t max_cos, uint32_t max_pmr, uint32_t max_pmr_per_cos);
/* Reset all classifier state (tables, pktio bindings); test helper. */
void odp_amd_cls_reset(void);

/* A classifier-enabled receive endpoint bound to one GPU: the classifier_t
 * of a pktio entry (odp_classification_datamodel.h:176-181) plus its device
 * context.  odp_pktio_open() of the ODP runtime layer creates these. */
odp_pktio_t odp_amd_cls_pktio_create(int gpu);
/* Classifier endpoint whose host bursts are sharded over gpus[0..n) (n <= 16;
 * ids may repeat); the runtime opens pktios this way when ODP_AMD_GPUS is set. */
odp_pktio_t odp_amd_cls_pktio_create_multi(const int *gpus, int n);
int odp_amd_cls_pktio_destroy(odp_pktio_t pktio);

/* Snapshot ("compile") the current tables into the mi_cls.h blob format.
 * Returns the blob size; writes at most cap bytes into buf (buf may be NULL
 * to query the size). */
long odp_amd_cls_compile(odp_pktio_t pktio, void *buf, size_t cap);

/* Receive-path batch classify: parse + classify n packets already resident
 * in device memory (layout: include/mi_cls.h).  Recompiles and uploads the
 * rule snapshot when the control plane changed since the last call. */
int odp_amd_cls_classify(odp_pktio_t pktio, const uint8_t *pkts_dev, const uint32_t *off_dev,
			 const uint16_t *len_dev, uint32_t n, void *out_dev, void *stream);

/* Host-memory form for the pktio receive path: stage, classify, copy the
 * records back (synchronous).  parse_only = 1 parses without classifying
 * (classifier disabled on the pktio): records carry the parse result with
 * outcome DISCARD (or PARSE_DROP). */
int odp_amd_cls_classify_host(odp_pktio_t pktio, const uint8_t *pkts, size_t bytes,
			      const uint32_t *off, const uint16_t *len, uint32_t n, void *out,
			      int parse_only);

/* Pipelined form (classifier enabled): submit a burst, wait for it later
 * (mi_cls_classify_host_submit / _wait).  A multi-GPU pktio classifies the
 * burst synchronously and returns ticket 0. */
int odp_amd_cls_classify_host_submit(odp_pktio_t pktio, const uint8_t *pkts, size_t bytes,
				     const uint32_t *off, const uint16_t *len, uint32_t n,
				     void *out, uint64_t *ticket);
int odp_amd_cls_classify_host_wait(odp_pktio_t pktio, uint64_t ticket);
/* Snapshot the current rules into the pktio's GPU context(s) and wait for
 * their program-specialised kernel (mi_cls_spec_wait): 0 in use, 1 none,
 * < 0 error. */
int odp_amd_cls_spec_wait(odp_pktio_t pktio);

/* The kernel instantiation of the pktio's last device launch
 * (mi_cls_last_launch: waves per block, LDS hot region, DIV, flat engine + 1,
 * specialised, pktin-option kernel, grid). */
int odp_amd_cls_last_launch(odp_pktio_t pktio, uint32_t *info, uint32_t n);

/* GPU receive delivery of a classified burst on the pktio's device
 * (mi_cls_deliver_submit; the runtime's receive path after classification,
 * pktio/loop.c:308-373).  Wait with odp_amd_cls_deliver_wait. */
struct mi_cls_dlv_args;
int odp_amd_cls_deliver(odp_pktio_t pktio, const struct mi_cls_dlv_args *args, uint64_t *ticket);
int odp_amd_cls_deliver_wait(odp_pktio_t pktio, uint64_t ticket);

/* Create the device context, upload the current rule snapshot and run a
 * warm-up launch (odp_pktio_start). */
int odp_amd_cls_prepare(odp_pktio_t pktio, int parse_only);

/* pktin parse options of the pktio (odp_pktin_config_opt_t.all_bits, from
 * odp_pktio_config(): checksum validation and drop-on-error bits), applied
 * by every later classify call: the `opt` that loop.c:271/310 hands to
 * _odp_packet_parse_common (include/odp_parse_internal.h:80-112). */
int odp_amd_cls_pktin_opt_set(odp_pktio_t pktio, uint64_t opt);

/* Enqueue-stage counters of a (CoS, queue slot) (odp_cls_queue_stats). */
void odp_amd_cls_queue_stats_add(uint32_t cos_index, uint32_t slot, uint64_t packets,
				 uint64_t discards);

/* 1 when every valid CoS has a pool of its own other than pktio_pool (no
 * classified packet comes from the pktio's pool), else 0. */
int odp_amd_cls_all_cos_pooled(odp_pool_t pktio_pool);

/* The receive chain's per-generation table of the control plane for a
 * pktio whose pool is pktio_pool (mi_cls_rxtab_t; pool_cap / rt_slot are the
 * caller's); -1 when it does not fit. */
struct mi_cls_rxtab;
int odp_amd_cls_rxtab_fill(odp_pool_t pktio_pool, struct mi_cls_rxtab *tab, odp_pool_t pools[],
			   uint32_t *npool, uint64_t *gen);

/* One burst's receive chain: classification, decisions and delivery
 * submitted at once on the pktio's GPU (mi_cls_rx_chain_submit); wait with
 * odp_amd_cls_deliver_wait.  -ENOTSUP on pktios over several GPUs. */
struct mi_cls_rxc_args;
int odp_amd_cls_rx_chain(odp_pktio_t pktio, const uint8_t *pkts, size_t bytes,
			 const struct mi_cls_rxc_args *args, uint64_t *ticket);

/* cos->pool of a CoS index (pool switch of the receive path). */
odp_pool_t odp_amd_cls_pool_of(uint32_t cos_index);

/* Enqueue flavour of a CoS index (cos->vector): returns use_std_enq (1 plain
 * enqueue, 0 packet vectors from *vec_pool of up to *vec_max packets), and
 * *use_aggr (hash-queue runs go to odp_queue_aggr(dst, 0)); -1 if invalid. */
int odp_amd_cls_cos_enq_mode(uint32_t cos_index, odp_pool_t *vec_pool, uint32_t *vec_max,
			     int *use_aggr);

/* packet_rss_hash (odp_classification.c:1773-1839) on a parsed frame;
 * hp = bit0 ipv4, bit1 ipv6, bit2 udp, bit3 tcp. */
uint32_t odp_amd_cls_rss_hash(const uint8_t *base, uint64_t in_flags, uint32_t l3, uint32_t l4,
			      uint32_t hp);

/* classification.h:851 */
odp_queue_t odp_cls_hash_result(odp_cos_t cos, odp_packet_t packet);

/* Map a result record's (cos index, queue slot) to the odp_queue_t handle
 * (queue_grp_tbl / cos->queue lookup of get_dest_queue, :395-405). */
odp_queue_t odp_amd_cls_queue_of(uint32_t cos_index, uint32_t queue_slot);

/* Control-plane generation counter (bumped by every table change). */
uint64_t odp_amd_cls_generation(void);

/* sizeof / offsetof of the ABI structs (binding self-check). */
size_t odp_amd_cls_abi_size(int which);

#ifdef __cplusplus
}
#endif

#endif /* ODP_AMD_CLS_API_H_ */
