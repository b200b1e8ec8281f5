/*
 * odp_rt_internal.h -- private structures shared by the runtime sources
 * (odp_rt.c: init/shm/pools/packets/events/queues/scheduler,
 *  odp_pktio.c: packet I/O drivers and the GPU receive path).
 */
#ifndef ODP_AMD_RT_INTERNAL_H_
#define ODP_AMD_RT_INTERNAL_H_

#include <pthread.h>

#include "odp_api.h"
#include "mi_cls.h"

#define RT_MAX_POOLS   64
#define RT_MAX_QUEUES  1024
#define RT_MAX_PKTIO   64
#define RT_MAX_AGGR    4
/* CONFIG_PACKET_HEADROOM (platform/linux-generic/include/odp_config_internal.h:105) */
/* odp_pktin_config_opt_t bits the receive path implements: ipv4/udp/tcp/
 * sctp checksum validation and the five drop-on-error options */
#define RT_PKTIN_OPT_MASK 0x7FCull
#define RT_PKT_HEADROOM 128
#define RT_PKT_TAILROOM 64

#define RT_ERR(...) fprintf(stderr, "odp: " __VA_ARGS__)

/* common event header: packets and event vectors start with it */
typedef struct ev_hdr {
	uint8_t type;           /* odp_event_type_t */
	uint8_t subtype;
	uint16_t pool;          /* pool index */
	uint32_t index;         /* element index in the pool */
	struct ev_hdr *next;
} ev_hdr_t;

/* packet metadata: the fields odp_packet_hdr_t carries on the receive path
 * (platform/linux-generic/include/odp_packet_internal.h:55-70,112-139).
 * From data_off on they are mi_cls_pkt_meta_t, the block the GPU receive
 * delivery writes (mi_cls_deliver_submit). */
typedef struct pkt_hdr {
	ev_hdr_t ev;
	uint8_t *head;          /* buffer start */
	uint32_t buf_len;       /* headroom + data capacity + tailroom */
	uint32_t rsv;
	/* the metadata block fills the header's second cache line: the GPU
	 * writes it whole, and the line the pool and queues use stays the
	 * host's */
	uint8_t pad[32];
	union {
		mi_cls_pkt_meta_t meta;
		struct {
			uint32_t data_off;      /* current headroom */
			uint32_t len;
			uint64_t in_flags;      /* packet_parser_t.input_flags */
			uint8_t err;            /* flags.all.error (7 bits) */
			uint8_t cos;            /* CoS index, 0xff none */
			uint16_t cls_mark;
			uint16_t l2, l3, l4;
			uint16_t rsv0;
			uint32_t rsv1;
			odp_queue_t dst_queue;
			odp_pktio_t input;
			const void *user_ptr;
			uint64_t rsv2;
		};
	};
} pkt_hdr_t;

_Static_assert(sizeof(((pkt_hdr_t *)0)->meta) == 64 && __builtin_offsetof(pkt_hdr_t, meta) == 64 &&
	       __builtin_offsetof(pkt_hdr_t, user_ptr) - __builtin_offsetof(pkt_hdr_t, meta) ==
	       __builtin_offsetof(mi_cls_pkt_meta_t, user_ptr) &&
	       __builtin_offsetof(pkt_hdr_t, dst_queue) - __builtin_offsetof(pkt_hdr_t, meta) ==
	       __builtin_offsetof(mi_cls_pkt_meta_t, dst_queue) &&
	       __builtin_offsetof(pkt_hdr_t, l4) - __builtin_offsetof(pkt_hdr_t, meta) ==
	       __builtin_offsetof(mi_cls_pkt_meta_t, l4) &&
	       __builtin_offsetof(pkt_hdr_t, in_flags) - __builtin_offsetof(pkt_hdr_t, meta) ==
	       __builtin_offsetof(mi_cls_pkt_meta_t, in_flags),
	       "pkt_hdr_t fields must overlay mi_cls_pkt_meta_t");

typedef struct evv_hdr {
	ev_hdr_t ev;
	uint32_t size;
	uint32_t max_size;
	odp_event_t tbl[];
} evv_hdr_t;

typedef struct rt_pool {
	int used;
	char name[ODP_POOL_NAME_LEN];
	odp_pool_param_t param;
	uint8_t *mem;
	size_t elem_size;
	uint32_t num;
	uint32_t data_cap;      /* packet data capacity (excl. head/tailroom) */
	ev_hdr_t **free_stk;    /* free events: a stack of pointers (bulk take / give
				 * copy pointers; no walk through the events) */
	uint32_t num_free;      /* on free_stk (thread caches not counted) */
	uint32_t gen;           /* creation number: tags the thread caches */
	int pinned;             /* mem is page-locked and device-addressed at its host
				 * addresses (GPU receive delivery reads / writes it) */
	odp_spinlock_t lock;
} rt_pool_t;

typedef struct rt_queue rt_queue_t;

struct rt_queue {
	int used;
	char name[ODP_QUEUE_NAME_LEN];
	odp_queue_param_t param;
	odp_spinlock_t lock;
	odp_event_t *ring;
	uint32_t cap, head, count;
	void *context;
	int owner;              /* atomic/ordered context holder: thread id + 1 */
	int sched_slot;         /* index in the scheduler list, -1 none */
	/* event aggregation (queue_types.h num_aggr / odp_queue_aggr) */
	uint32_t num_aggr;
	rt_queue_t *aggr[RT_MAX_AGGR];
	int is_aggr;
	rt_queue_t *base;
	odp_event_aggr_config_t aggr_cfg;
	evv_hdr_t *cur_vec;
	uint64_t cur_t0;
	/* plain pktin queue (ODP_PKTIN_MODE_QUEUE): pktio to poll when empty */
	int pktin_idx;          /* pktio index + 1, 0 none */
};

/* runtime-private entry points */
pkt_hdr_t *rt_pkt_hdr(odp_packet_t pkt);
rt_pool_t *rt_pool(odp_pool_t pool);
/* free events of a pool this thread can allocate: its free list plus the
 * calling thread's cache */
uint32_t rt_pool_avail(odp_pool_t pool);
/* up to num packets of a pool whose buffers hold len bytes, headers NOT
 * initialised (rt_packet_init does that, e.g. after a prefetch); returns the
 * count taken */
int rt_packet_alloc_raw(odp_pool_t pool, uint32_t len, odp_packet_t pkt[], int num);
void rt_packet_init(odp_packet_t pkt, uint32_t len);
/* packets taken with rt_packet_alloc_raw and not used, back to their pool */
void rt_packet_return_raw(odp_pool_t pool, const odp_packet_t pkt[], int num);
int rt_queue_enq_multi(rt_queue_t *q, const odp_event_t ev[], int num);
int rt_queue_deq_multi_raw(rt_queue_t *q, odp_event_t ev[], int num);
int rt_thread_id(void);
/* scheduler hooks for SCHED-mode packet input (odp_pktio.c) */
int rt_pktio_sched_poll(void);
int rt_pktio_poll_index(int idx);
uint32_t rt_gpu_index(void);
int rt_queue_is_valid(odp_queue_t h);
/* the address range spanned by the pinned packet pools ([*lo, *lo + *bytes));
 * 0 when there is none */
int rt_pinned_arena(uint8_t **lo, size_t *bytes);
/* 1 when every handle of pk[0..n) is a header in a page-locked pool (the
 * GPU may read it): the handles' addresses against the pools' ranges */
int rt_pinned_handles(const odp_packet_t pk[], int n);
/* bytes from a packet header's metadata block to its data at the default
 * headroom (fixed by the pool layout) */
uint32_t rt_data_from_meta(void);

#endif /* ODP_AMD_RT_INTERNAL_H_ */
