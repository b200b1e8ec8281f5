/*
 * odp_cls.c -- ODP classification control plane for the MI355X build.
 *
 * Implements the odp_cls_* / odp_pktio_*_cos_set API of include/odp_cls_api.h
 * with linux-generic's semantics (platform/linux-generic/odp_classification.c):
 *   - CoS and PMR slots are taken lowest-free-first (:292-295, :447-449), so a
 *     CoS index equals its slot; handles are slot+1 (:60-78);
 *   - PMRs are appended to the source CoS list; destroying one moves the
 *     last PMR of that list into its slot and always decrements the count
 *     (:765-793), so scan order is NOT creation order after deletes;
 *   - destroying a CoS only clears its valid flag (:487-501): PMRs pointing
 *     at it are skipped by the data plane (:1635-1636) and a re-created CoS
 *     in the same slot is picked up again.
 *
 * The data plane does not read these tables: a change bumps a generation
 * counter, and the next batch classify call snapshots ("compiles") the
 * tables into the flat mi_cls.h blob and uploads it to the GPU.  This is the
 * device-side counterpart of the reference's lock-free readers
 * ("indeterminate during a PMR change", :1373-1374).
 */
#include <errno.h>
#include <inttypes.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "odp_cls_api.h"
#include "mi_cls.h"

/* runtime (odp_rt.c): a handle of a queue the runtime created */
int rt_queue_is_valid(odp_queue_t h);

#define COS_QUEUE_MAX 32
#define PMR_TERM_MAX 8
#define MAX_MARK 0xFFFFu
#define MAX_PKTIO 64

typedef struct {
	odp_cls_pmr_term_t term;
	uint8_t value[16];     /* pre-masked */
	uint8_t mask[16];
	uint32_t offset;
	uint32_t val_sz;
} term_t;

typedef struct {
	int valid;
	uint32_t num_terms;
	uint16_t mark;
	term_t t[PMR_TERM_MAX];
	int src_cos;           /* slot */
} pmr_t;

typedef struct {
	int valid;
	uint32_t num_rule;
	int *pmr;              /* pmr slots, max_per_cos */
	int *linked;           /* cos slots */
	int stats_enable;
	odp_cos_action_t action;
	odp_queue_t queue;
	uint32_t num_queue;
	odp_pool_t pool;
	uint8_t index;
	int queue_group;
	uint32_t hash_proto;   /* bit0 ipv4, bit1 ipv6, bit2 udp, bit3 tcp */
	odp_queue_t hq[COS_QUEUE_MAX];
	char name[ODP_COS_NAME_LEN];
	uint64_t stats_discards;
	/* per-queue enqueue counters (_odp_cos_queue_stats_add,
	 * odp_classification_internal.h:60-81), maintained by the host
	 * enqueue stage of the receive path */
	uint64_t q_packets[COS_QUEUE_MAX];
	uint64_t q_discards[COS_QUEUE_MAX];
	/* cos->vector (odp_classification_datamodel.h:145-151): packet vector
	 * delivery, or event-aggregator enqueue of hash-queue runs */
	odp_pool_t vec_pool;
	uint32_t vec_max;
	int use_std_enq;
	int use_aggr;
} cos_t;

typedef struct {
	int used;
	int gpu;
	int default_cos;       /* slot, -1 none */
	int error_cos;
	uint32_t headroom;
	mi_cls_ctx_t *ctx;       /* device 0 of the pktio (the group's first context) */
	mi_cls_ctx_t *pctx;      /* parse-only context (empty table) */
	/* multi-GPU receive (odp_amd_cls_pktio_create_multi): host bursts are
	 * sharded over these devices (mi_cls_group_classify_host) */
	mi_cls_group_t *grp;
	int ngpu;
	int gpus[16];
	uint64_t compiled_gen;
	void *blob;
	size_t blob_cap;
	uint32_t stats_mask[8];
	uint64_t pktin_opt;      /* odp_pktin_config_opt_t.all_bits */
} pktio_t;

static struct {
	int init;
	uint32_t max_cos, max_pmr, max_per_cos;
	cos_t *cos;
	pmr_t *pmr;
	pktio_t pktio[MAX_PKTIO];
	uint64_t gen;
	uint64_t hq_seq;
	pthread_mutex_t lock;
} G = { .max_cos = 255, .max_pmr = 8192, .max_per_cos = 4096,
	.lock = PTHREAD_MUTEX_INITIALIZER };

#define ERR(...) fprintf(stderr, "odp_cls: " __VA_ARGS__)

static void free_tables(void)
{
	uint32_t i;

	if (G.cos) {
		for (i = 0; i < G.max_cos; i++) {
			if (G.cos[i].valid && G.cos[i].queue_group)
				for (uint32_t j = 0; j < G.cos[i].num_queue; j++)
					odp_queue_destroy(G.cos[i].hq[j]);
			free(G.cos[i].pmr);
			free(G.cos[i].linked);
		}
	}
	free(G.cos);
	free(G.pmr);
	G.cos = NULL;
	G.pmr = NULL;
	G.init = 0;
}

static int ensure_init(void)
{
	uint32_t i;

	if (G.init)
		return 0;
	G.cos = calloc(G.max_cos, sizeof(cos_t));
	G.pmr = calloc(G.max_pmr, sizeof(pmr_t));
	if (!G.cos || !G.pmr)
		goto fail;
	for (i = 0; i < G.max_cos; i++) {
		G.cos[i].pmr = malloc(G.max_per_cos * sizeof(int));
		G.cos[i].linked = malloc(G.max_per_cos * sizeof(int));
		if (!G.cos[i].pmr || !G.cos[i].linked)
			goto fail;
	}
	G.init = 1;
	return 0;
fail:
	free_tables();
	return -1;
}

int odp_amd_cls_limits_set(uint32_t max_cos, uint32_t max_pmr, uint32_t max_pmr_per_cos)
{
	/* cos index is a u8 in the packet header, 0xFF marks "no CoS" in records */
	if (max_cos < 1 || max_cos > 255 || max_pmr < 1 || max_pmr_per_cos < 1)
		return -1;
	pthread_mutex_lock(&G.lock);
	free_tables();
	G.max_cos = max_cos;
	G.max_pmr = max_pmr;
	G.max_per_cos = max_pmr_per_cos;
	G.gen++;
	pthread_mutex_unlock(&G.lock);
	return 0;
}

void odp_amd_cls_reset(void)
{
	pthread_mutex_lock(&G.lock);
	free_tables();
	for (int i = 0; i < MAX_PKTIO; i++) {
		G.pktio[i].default_cos = -1;
		G.pktio[i].error_cos = -1;
	}
	G.gen++;
	pthread_mutex_unlock(&G.lock);
}

uint64_t odp_amd_cls_generation(void)
{
	return G.gen;
}

static inline uint32_t cos_ndx(odp_cos_t h)
{
	return (uint32_t)((uintptr_t)h - 1);
}

static inline odp_cos_t cos_hdl(uint32_t ndx)
{
	return (odp_cos_t)(uintptr_t)(ndx + 1);
}

/* get_cos_entry (:462-472) */
static cos_t *get_cos(odp_cos_t h)
{
	uint32_t i = cos_ndx(h);

	if (!G.init || h == ODP_COS_INVALID || i >= G.max_cos || !G.cos[i].valid)
		return NULL;
	return &G.cos[i];
}

static pmr_t *get_pmr(odp_pmr_t h)
{
	uint32_t i = (uint32_t)((uintptr_t)h - 1);

	if (!G.init || h == ODP_PMR_INVALID || i >= G.max_pmr || !G.pmr[i].valid)
		return NULL;
	return &G.pmr[i];
}

void odp_cls_cos_param_init(odp_cls_cos_param_t *param)
{
	memset(param, 0, sizeof(*param));
	param->queue = ODP_QUEUE_INVALID;
	param->pool = ODP_POOL_INVALID;
	param->num_queue = 1;
	param->vector.enable = false;
}

void odp_cls_pmr_param_init(odp_pmr_param_t *param)
{
	memset(param, 0, sizeof(*param));
}

void odp_cls_pmr_create_opt_init(odp_pmr_create_opt_t *opt)
{
	opt->terms = NULL;
	opt->num_terms = 0;
	opt->mark = 0;
	opt->priority = 0;
}

/* odp_cls_capability (:153-202) with this build's table limits */
int odp_cls_capability(odp_cls_capability_t *c)
{
	memset(c, 0, sizeof(*c));
	c->max_pmr = G.max_pmr;
	c->max_pmr_per_cos = G.max_per_cos;
	c->max_terms_per_pmr = PMR_TERM_MAX;
	c->max_pmr_priority = 0;
	c->max_cos = G.max_cos;
	c->max_cos_stats = G.max_cos;
	c->pmr_range_supported = false;
	c->supported_terms.bit.len = 1;
	c->supported_terms.bit.ethtype_0 = 1;
	c->supported_terms.bit.ethtype_x = 1;
	c->supported_terms.bit.vlan_id_0 = 1;
	c->supported_terms.bit.vlan_id_x = 1;
	c->supported_terms.bit.vlan_pcp_0 = 1;
	c->supported_terms.bit.dmac = 1;
	c->supported_terms.bit.ip_proto = 1;
	c->supported_terms.bit.ip_dscp = 1;
	c->supported_terms.bit.udp_dport = 1;
	c->supported_terms.bit.udp_sport = 1;
	c->supported_terms.bit.tcp_dport = 1;
	c->supported_terms.bit.tcp_sport = 1;
	c->supported_terms.bit.sip_addr = 1;
	c->supported_terms.bit.dip_addr = 1;
	c->supported_terms.bit.sip6_addr = 1;
	c->supported_terms.bit.dip6_addr = 1;
	c->supported_terms.bit.ipsec_spi = 1;
	c->supported_terms.bit.custom_frame = 1;
	c->supported_terms.bit.custom_l3 = 1;
	c->random_early_detection = ODP_SUPPORT_NO;
	c->back_pressure = ODP_SUPPORT_NO;
	c->max_hash_queues = COS_QUEUE_MAX;
	c->hash_protocols.proto.ipv4_udp = 1;
	c->hash_protocols.proto.ipv4_tcp = 1;
	c->hash_protocols.proto.ipv4 = 1;
	c->hash_protocols.proto.ipv6_udp = 1;
	c->hash_protocols.proto.ipv6_tcp = 1;
	c->hash_protocols.proto.ipv6 = 1;
	c->max_mark = MAX_MARK;
	c->stats.cos.counter.discards = 1;
	c->stats.cos.counter.packets = 1;
	c->stats.queue.counter.discards = 1;
	c->stats.queue.counter.packets = 1;
	return 0;
}

/* _odp_cls_update_hash_proto (:212-225) */
static uint32_t fold_hash_proto(odp_pktin_hash_proto_t h)
{
	uint32_t r = 0;

	if (h.proto.ipv4 || h.proto.ipv4_tcp || h.proto.ipv4_udp)
		r |= 1;
	if (h.proto.ipv6 || h.proto.ipv6_tcp || h.proto.ipv6_udp)
		r |= 2;
	if (h.proto.ipv4_tcp || h.proto.ipv6_tcp)
		r |= 8;
	if (h.proto.ipv4_udp || h.proto.ipv6_udp)
		r |= 4;
	return r;
}

/* odp_cls_cos_create (:233-370) */
odp_cos_t odp_cls_cos_create(const char *name, const odp_cls_cos_param_t *param_in)
{
	odp_cls_cos_param_t param = *param_in;
	odp_cos_t ret = ODP_COS_INVALID;
	uint32_t i, j;

	if (param.action == ODP_COS_ACTION_DROP) {
		param.num_queue = 1;
		param.queue = ODP_QUEUE_INVALID;
		param.pool = ODP_POOL_INVALID;
		param.vector.enable = false;
	} else if (param.num_queue == 1 && param.queue == ODP_QUEUE_INVALID) {
		return ODP_COS_INVALID;
	}
	if (param.num_queue > COS_QUEUE_MAX || param.num_queue < 1)
		return ODP_COS_INVALID;
	/* event aggregation: the CoS queue is an aggregator, or its hash queues
	 * get aggregators (:256-259) */
	const int event_aggr_enabled =
		(param.num_queue == 1 && param.queue != ODP_QUEUE_INVALID &&
		 rt_queue_is_valid(param.queue) && odp_queue_type(param.queue) == ODP_QUEUE_TYPE_AGGR) ||
		(param.num_queue > 1 && param.queue_param.num_aggr);

	/* packet vector parameters (:261-288) */
	if (param.vector.enable) {
		odp_pool_info_t pool_info;

		if (event_aggr_enabled) {
			ERR("Packet and event vectoring enabled simultaneously\n");
			return ODP_COS_INVALID;
		}
		if (param.vector.pool == ODP_POOL_INVALID ||
		    odp_pool_info(param.vector.pool, &pool_info)) {
			ERR("invalid packet vector pool\n");
			return ODP_COS_INVALID;
		}
		if (pool_info.params.type != ODP_POOL_VECTOR) {
			ERR("wrong pool type\n");
			return ODP_COS_INVALID;
		}
		if (param.vector.max_size == 0) {
			ERR("vector.max_size is zero\n");
			return ODP_COS_INVALID;
		}
		if (param.vector.max_size > pool_info.params.vector.max_size) {
			ERR("vector.max_size larger than pool max vector size\n");
			return ODP_COS_INVALID;
		}
	}
	if (param.aggr_enq_profile.type != ODP_AEP_TYPE_NONE)
		return ODP_COS_INVALID;

	pthread_mutex_lock(&G.lock);
	if (ensure_init())
		goto out;
	for (i = 0; i < G.max_cos; i++) {
		cos_t *c = &G.cos[i];

		if (c->valid)
			continue;
		if (name == NULL) {
			c->name[0] = 0;
		} else {
			strncpy(c->name, name, ODP_COS_NAME_LEN - 1);
			c->name[ODP_COS_NAME_LEN - 1] = 0;
		}
		for (j = 0; j < G.max_per_cos; j++) {
			c->pmr[j] = -1;
			c->linked[j] = -1;
		}
		c->num_queue = param.num_queue;
		if (param.num_queue > 1) {
			c->queue_group = 1;
			c->queue = ODP_QUEUE_INVALID;
			c->hash_proto = fold_hash_proto(param.hash_proto);
			/* implementation-created hash queues (:310-330) */
			for (j = 0; j < param.num_queue; j++) {
				char hq_name[ODP_QUEUE_NAME_LEN];

				snprintf(hq_name, sizeof(hq_name), "_odp_cos_hq_%u_%u", i, j);
				c->hq[j] = odp_queue_create(hq_name, &param.queue_param);
				if (c->hq[j] == ODP_QUEUE_INVALID) {
					while (j--)
						odp_queue_destroy(c->hq[j]);
					goto out;
				}
			}
		} else {
			c->queue_group = 0;
			c->hash_proto = 0;
			c->queue = param.queue;
		}
		c->stats_discards = 0;
		memset(c->q_packets, 0, sizeof(c->q_packets));
		memset(c->q_discards, 0, sizeof(c->q_discards));
		c->action = param.action;
		c->pool = param.pool;
		c->valid = 1;
		c->num_rule = 0;
		c->index = (uint8_t)i;
		c->vec_pool = param.vector.enable ? param.vector.pool : ODP_POOL_INVALID;
		c->vec_max = param.vector.enable ? param.vector.max_size : 0;
		c->use_std_enq = !param.vector.enable;
		c->use_aggr = event_aggr_enabled && param.num_queue > 1;
		c->stats_enable = param.stats_enable;
		G.gen++;
		ret = cos_hdl(i);
		goto out;
	}
	ERR("CLS_COS_MAX_ENTRY reached\n");
out:
	pthread_mutex_unlock(&G.lock);
	return ret;
}

int odp_cls_cos_create_multi(const char *name[], const odp_cls_cos_param_t param[],
			     odp_cos_t cos[], int num)
{
	int i;

	for (i = 0; i < num; i++) {
		odp_cos_t c = odp_cls_cos_create(name ? name[i] : NULL, &param[i]);

		if (c == ODP_COS_INVALID)
			return i == 0 ? -1 : i;
		cos[i] = c;
	}
	return i;
}

int odp_cos_destroy(odp_cos_t h)
{
	int rc = -1;

	pthread_mutex_lock(&G.lock);
	cos_t *c = get_cos(h);

	if (c) {
		/* :494-495 */
		if (c->queue_group)
			for (uint32_t j = 0; j < c->num_queue; j++)
				odp_queue_destroy(c->hq[j]);
		c->valid = 0;
		G.gen++;
		rc = 0;
	} else {
		ERR("Invalid odp_cos_t handle\n");
	}
	pthread_mutex_unlock(&G.lock);
	return rc;
}

int odp_cos_destroy_multi(odp_cos_t cos[], int num)
{
	int i;

	for (i = 0; i < num; i++) {
		int r = odp_cos_destroy(cos[i]);

		if (r)
			return i == 0 ? r : i;
	}
	return i;
}

int odp_cos_queue_set(odp_cos_t h, odp_queue_t q)
{
	cos_t *c = get_cos(h);

	if (!c || q == ODP_QUEUE_INVALID || c->num_queue != 1)
		return -1;
	c->queue = q;
	G.gen++;
	return 0;
}

odp_queue_t odp_cos_queue(odp_cos_t h)
{
	cos_t *c = get_cos(h);

	return c ? c->queue : ODP_QUEUE_INVALID;
}

uint32_t odp_cls_cos_num_queue(odp_cos_t h)
{
	cos_t *c = get_cos(h);

	return c ? c->num_queue : 0;
}

/* odp_cls_cos_queues (:569-601) */
uint32_t odp_cls_cos_queues(odp_cos_t h, odp_queue_t queue[], uint32_t num)
{
	cos_t *c = get_cos(h);
	uint32_t i, n;

	if (!c)
		return 0;
	if (c->num_queue == 1) {
		if (num == 0)
			return 1;
		queue[0] = c->queue;
		return 1;
	}
	n = num < c->num_queue ? num : c->num_queue;
	for (i = 0; i < n; i++)
		queue[i] = c->hq[i];
	return c->num_queue;
}

int odp_cls_cos_pool_set(odp_cos_t h, odp_pool_t pool)
{
	cos_t *c = get_cos(h);

	if (!c)
		return -1;
	c->pool = pool;
	return 0;
}

odp_pool_t odp_cls_cos_pool(odp_cos_t h)
{
	cos_t *c = get_cos(h);

	return c ? c->pool : ODP_POOL_INVALID;
}

uint64_t odp_cos_to_u64(odp_cos_t h)
{
	return (uint64_t)(uintptr_t)h;
}

uint64_t odp_pmr_to_u64(odp_pmr_t h)
{
	return (uint64_t)(uintptr_t)h;
}

/* pmr_create_term (:670-763) */
static int create_term(term_t *v, const odp_pmr_param_t *p)
{
	uint32_t size, i;
	int custom = 0;

	if (p->range_term) {
		ERR("PMR value range not supported\n");
		return -1;
	}
	switch (p->term) {
	case ODP_PMR_VLAN_PCP_0:
	case ODP_PMR_IPPROTO:
	case ODP_PMR_IP_DSCP:
		size = 1;
		break;
	case ODP_PMR_ETHTYPE_0:
	case ODP_PMR_ETHTYPE_X:
	case ODP_PMR_VLAN_ID_0:
	case ODP_PMR_VLAN_ID_X:
	case ODP_PMR_UDP_DPORT:
	case ODP_PMR_TCP_DPORT:
	case ODP_PMR_UDP_SPORT:
	case ODP_PMR_TCP_SPORT:
		size = 2;
		break;
	case ODP_PMR_LEN:
	case ODP_PMR_SIP_ADDR:
	case ODP_PMR_DIP_ADDR:
	case ODP_PMR_IPSEC_SPI:
	case ODP_PMR_LD_VNI:
		size = 4;
		break;
	case ODP_PMR_DMAC:
		size = 6;
		break;
	case ODP_PMR_SIP6_ADDR:
	case ODP_PMR_DIP6_ADDR:
		size = 16;
		break;
	case ODP_PMR_CUSTOM_FRAME:
	case ODP_PMR_CUSTOM_L3:
		custom = 1;
		size = 16;
		break;
	default:
		ERR("Bad PMR term\n");
		return -1;
	}
	if ((!custom && p->val_sz != size) || (custom && p->val_sz > size)) {
		ERR("Bad PMR value size: %u\n", p->val_sz);
		return -1;
	}
	memset(v, 0, sizeof(*v));
	v->term = p->term;
	memcpy(v->value, p->match.value, p->val_sz);
	memcpy(v->mask, p->match.mask, p->val_sz);
	for (i = 0; i < p->val_sz; i++)
		v->value[i] &= v->mask[i];
	v->offset = p->offset;
	v->val_sz = p->val_sz;
	return 0;
}

/* cls_pmr_create (:812-858) */
static odp_pmr_t pmr_create(const odp_pmr_param_t *terms, int num_terms, uint16_t mark,
			    odp_cos_t src, odp_cos_t dst)
{
	odp_pmr_t ret = ODP_PMR_INVALID;
	uint32_t p;
	int i;

	pthread_mutex_lock(&G.lock);
	cos_t *cs = get_cos(src), *cd = get_cos(dst);

	if (!cs || !cd) {
		ERR("Invalid odp_cos_t handle\n");
		goto out;
	}
	if (num_terms > PMR_TERM_MAX) {
		ERR("no of terms greater than supported CLS_PMRTERM_MAX\n");
		goto out;
	}
	if (cs->num_rule == G.max_per_cos)
		goto out;
	for (p = 0; p < G.max_pmr; p++)
		if (!G.pmr[p].valid)
			break;
	if (p == G.max_pmr) {
		ERR("CLS_PMR_MAX_ENTRY reached\n");
		goto out;
	}
	pmr_t *r = &G.pmr[p];

	for (i = 0; i < num_terms; i++)
		if (create_term(&r->t[i], &terms[i]))
			goto out;
	r->valid = 1;
	r->num_terms = (uint32_t)num_terms;
	r->mark = mark;
	cs->pmr[cs->num_rule] = (int)p;
	cs->linked[cs->num_rule] = (int)cd->index;
	cs->num_rule++;
	r->src_cos = cs->index;
	G.gen++;
	ret = (odp_pmr_t)(uintptr_t)(p + 1);
out:
	pthread_mutex_unlock(&G.lock);
	return ret;
}

odp_pmr_t odp_cls_pmr_create(const odp_pmr_param_t *terms, int num_terms,
			     odp_cos_t src_cos, odp_cos_t dst_cos)
{
	return pmr_create(terms, num_terms, 0, src_cos, dst_cos);
}

odp_pmr_t odp_cls_pmr_create_opt(const odp_pmr_create_opt_t *opt,
				 odp_cos_t src_cos, odp_cos_t dst_cos)
{
	if (opt == NULL) {
		ERR("Bad parameter\n");
		return ODP_PMR_INVALID;
	}
	if (opt->mark > MAX_MARK) {
		ERR("Too large mark value: %" PRIu64 "\n", opt->mark);
		return ODP_PMR_INVALID;
	}
	return pmr_create(opt->terms, opt->num_terms, (uint16_t)opt->mark, src_cos, dst_cos);
}

int odp_cls_pmr_create_multi(const odp_pmr_create_opt_t opt[], odp_cos_t src_cos[],
			     odp_cos_t dst_cos[], odp_pmr_t pmr[], int num)
{
	int i;

	for (i = 0; i < num; i++) {
		odp_pmr_t p = odp_cls_pmr_create_opt(&opt[i], src_cos[i], dst_cos[i]);

		if (p == ODP_PMR_INVALID)
			return i == 0 ? -1 : i;
		pmr[i] = p;
	}
	return i;
}

/* odp_cls_pmr_destroy (:765-793) */
int odp_cls_pmr_destroy(odp_pmr_t h)
{
	int rc = -1;

	pthread_mutex_lock(&G.lock);
	pmr_t *r = get_pmr(h);

	if (r && r->src_cos >= 0) {
		cos_t *c = &G.cos[r->src_cos];
		int p = (int)((uintptr_t)h - 1);
		uint32_t loc = c->num_rule, i;

		if (loc != 0) {
			loc -= 1;
			for (i = 0; i <= loc; i++) {
				if (c->pmr[i] == p) {
					c->pmr[i] = c->pmr[loc];
					c->linked[i] = c->linked[loc];
				}
			}
			c->num_rule--;
		}
		r->valid = 0;
		G.gen++;
		rc = 0;
	}
	pthread_mutex_unlock(&G.lock);
	return rc;
}

int odp_cls_pmr_destroy_multi(odp_pmr_t pmr[], int num)
{
	int i;

	for (i = 0; i < num; i++) {
		int r = odp_cls_pmr_destroy(pmr[i]);

		if (r)
			return i == 0 ? r : i;
	}
	return i;
}

/* ----------------------------------------------------------------- pktio */
static pktio_t *get_pktio(odp_pktio_t h)
{
	uintptr_t i = (uintptr_t)h;

	if (i == 0 || i > MAX_PKTIO || !G.pktio[i - 1].used)
		return NULL;
	return &G.pktio[i - 1];
}

odp_pktio_t odp_amd_cls_pktio_create(int gpu)
{
	int i;

	pthread_mutex_lock(&G.lock);
	for (i = 0; i < MAX_PKTIO; i++) {
		if (!G.pktio[i].used) {
			pktio_t *e = &G.pktio[i];

			memset(e, 0, sizeof(*e));
			e->used = 1;
			e->gpu = gpu;
			e->default_cos = -1;
			e->error_cos = -1;
			e->compiled_gen = ~0ull;
			pthread_mutex_unlock(&G.lock);
			return (odp_pktio_t)(uintptr_t)(i + 1);
		}
	}
	pthread_mutex_unlock(&G.lock);
	return ODP_PKTIO_INVALID;
}

/* A classifier endpoint whose host bursts are sharded over several GPUs
 * (SURVEY.md §8(e)); gpus[0] also serves the device-pointer entry. */
odp_pktio_t odp_amd_cls_pktio_create_multi(const int *gpus, int n)
{
	if (!gpus || n < 1 || n > 16)
		return ODP_PKTIO_INVALID;
	odp_pktio_t h = odp_amd_cls_pktio_create(gpus[0]);
	pktio_t *e = get_pktio(h);

	if (!e)
		return ODP_PKTIO_INVALID;
	e->ngpu = n;
	memcpy(e->gpus, gpus, (size_t)n * sizeof(int));
	return h;
}

int odp_amd_cls_pktio_destroy(odp_pktio_t h)
{
	pktio_t *e = get_pktio(h);

	if (!e)
		return -1;
	if (e->grp)
		mi_cls_group_destroy(e->grp);   /* owns e->ctx */
	else if (e->ctx)
		mi_cls_ctx_destroy(e->ctx);
	if (e->pctx)
		mi_cls_ctx_destroy(e->pctx);
	free(e->blob);
	memset(e, 0, sizeof(*e));
	return 0;
}

/* odp_pktio_default_cos_set / error_cos_set (:603-647) */
int odp_pktio_default_cos_set(odp_pktio_t h, odp_cos_t cos)
{
	pktio_t *e = get_pktio(h);
	int slot = -1;

	if (!e) {
		ERR("Invalid odp_pktio_t handle\n");
		return -1;
	}
	if (cos != ODP_COS_INVALID) {
		cos_t *c = get_cos(cos);

		if (!c) {
			ERR("Invalid odp_cos_t handle\n");
			return -1;
		}
		slot = c->index;
	}
	e->default_cos = slot;
	G.gen++;
	return 0;
}

int odp_pktio_error_cos_set(odp_pktio_t h, odp_cos_t cos)
{
	pktio_t *e = get_pktio(h);
	int slot = -1;

	if (!e) {
		ERR("Invalid odp_pktio_t handle\n");
		return -1;
	}
	if (cos != ODP_COS_INVALID) {
		cos_t *c = get_cos(cos);

		if (!c) {
			ERR("Invalid odp_cos_t handle\n");
			return -1;
		}
		slot = c->index;
	}
	e->error_cos = slot;
	G.gen++;
	return 0;
}

int odp_pktio_skip_set(odp_pktio_t h, uint32_t offset)
{
	(void)h;
	(void)offset;
	return -ENOTSUP;   /* :649-656 */
}

int odp_pktio_headroom_set(odp_pktio_t h, uint32_t headroom)
{
	pktio_t *e = get_pktio(h);

	if (!e)
		return -1;
	e->headroom = headroom;
	return 0;
}

/* --------------------------------------------------------------- compile */
static uint32_t le_word(const uint8_t *b, uint32_t n)
{
	uint32_t v = 0, i;

	for (i = 0; i < n && i < 4; i++)
		v |= (uint32_t)b[i] << (8 * i);
	return v;
}

/* term -> mi_term_t; field packing documented in mi_cls.h / mi_cls.hip */
static void compile_term(const term_t *t, mi_term_t *o)
{
	uint32_t i;

	memset(o, 0, sizeof(*o));
	o->size = (uint8_t)t->val_sz;
	o->offset = t->offset;
	for (i = 0; i < 4; i++) {
		o->mask[i] = le_word(t->mask + 4 * i, 4);
		o->value[i] = le_word(t->value + 4 * i, 4);
	}
	switch (t->term) {
	case ODP_PMR_LEN:          o->kind = MI_K_LEN; break;
	case ODP_PMR_ETHTYPE_0:    o->kind = MI_K_ETH0; break;
	case ODP_PMR_ETHTYPE_X:    o->kind = MI_K_ETHX; break;
	case ODP_PMR_VLAN_ID_0:    o->kind = MI_K_VID0; break;
	case ODP_PMR_VLAN_ID_X:    o->kind = MI_K_VIDX; break;
	case ODP_PMR_VLAN_PCP_0:   o->kind = MI_K_PCP0; break;
	case ODP_PMR_DMAC:         o->kind = MI_K_DMAC; break;
	case ODP_PMR_IPPROTO:      o->kind = MI_K_PROTO; break;
	case ODP_PMR_IP_DSCP:      o->kind = MI_K_DSCP; break;
	case ODP_PMR_SIP_ADDR:     o->kind = MI_K_SIP; break;
	case ODP_PMR_DIP_ADDR:     o->kind = MI_K_DIP; break;
	case ODP_PMR_SIP6_ADDR:    o->kind = MI_K_SIP6; break;
	case ODP_PMR_DIP6_ADDR:    o->kind = MI_K_DIP6; break;
	case ODP_PMR_IPSEC_SPI:    o->kind = MI_K_SPI; break;
	case ODP_PMR_LD_VNI:       o->kind = MI_K_NEVER; break;
	case ODP_PMR_CUSTOM_FRAME: o->kind = MI_K_CUSTOM_FRAME; break;
	case ODP_PMR_CUSTOM_L3:    o->kind = MI_K_CUSTOM_L3; break;
	case ODP_PMR_INNER_HDR_OFF: o->kind = MI_K_ALWAYS; break;
	/* ports: the kernel holds {sport, dport} as one raw 32-bit word read at
	 * l4; the destination port is the upper half */
	case ODP_PMR_UDP_SPORT:    o->kind = MI_K_UDP_SPORT; break;
	case ODP_PMR_TCP_SPORT:    o->kind = MI_K_TCP_SPORT; break;
	case ODP_PMR_UDP_DPORT:
	case ODP_PMR_TCP_DPORT:
		o->kind = t->term == ODP_PMR_UDP_DPORT ? MI_K_UDP_DPORT : MI_K_TCP_DPORT;
		o->mask[0] <<= 16;
		o->value[0] <<= 16;
		break;
	default:                   o->kind = MI_K_NEVER; break;
	}
}

static long compile_locked(pktio_t *e, void *buf, size_t cap)
{
	uint32_t ncos = 0, nrules = 0, nterms = 0, s, i, t, used = 0;

	if (ensure_init())
		return -ENOMEM;
	/* slots described: every slot up to the highest one that is valid or
	 * referenced as default / error CoS */
	for (s = 0; s < G.max_cos; s++)
		if (G.cos[s].valid)
			ncos = s + 1;
	if (e->default_cos >= 0 && (uint32_t)e->default_cos + 1 > ncos)
		ncos = (uint32_t)e->default_cos + 1;
	if (e->error_cos >= 0 && (uint32_t)e->error_cos + 1 > ncos)
		ncos = (uint32_t)e->error_cos + 1;
	for (s = 0; s < ncos; s++) {
		const cos_t *c = &G.cos[s];

		if (!c->valid)
			continue;
		for (i = 0; i < c->num_rule; i++) {
			const pmr_t *r = &G.pmr[c->pmr[i]];

			if (!G.cos[c->linked[i]].valid || !r->valid)
				continue;
			nrules++;
			nterms += r->num_terms;
		}
	}
	size_t bytes = sizeof(mi_tbl_hdr_t) + (size_t)ncos * sizeof(mi_cos_t) +
		       (size_t)nrules * sizeof(mi_rule_t) + (size_t)nterms * sizeof(mi_term_t);

	if (!buf || cap < bytes)
		return (long)bytes;
	memset(buf, 0, bytes);
	mi_tbl_hdr_t *h = buf;
	mi_cos_t *co = (mi_cos_t *)((uint8_t *)buf + sizeof(*h));
	mi_rule_t *ro = (mi_rule_t *)(co + ncos);
	mi_term_t *to = (mi_term_t *)(ro + nrules);
	uint32_t rn = 0, tn = 0;

	h->magic = MI_CLS_TBL_MAGIC;
	h->version = MI_CLS_TBL_VERSION;
	h->total_bytes = (uint32_t)bytes;
	h->num_cos = ncos;
	h->num_rules = nrules;
	h->num_terms = nterms;
	h->default_cos = e->default_cos;
	h->error_cos = e->error_cos;
	h->default_valid = e->default_cos >= 0 && G.cos[e->default_cos].valid;
	h->max_hops = G.max_cos;
	h->cos_off = sizeof(*h);
	h->rule_off = (uint32_t)((uint8_t *)ro - (uint8_t *)buf);
	h->term_off = (uint32_t)((uint8_t *)to - (uint8_t *)buf);
	h->generation = (uint32_t)G.gen;
	for (s = 0; s < ncos; s++) {
		const cos_t *c = &G.cos[s];

		co[s].rule_begin = rn;
		co[s].action = (uint8_t)(c->action == ODP_COS_ACTION_DROP);
		co[s].num_queue = (uint8_t)(c->num_queue ? c->num_queue : 1);
		co[s].hash_proto = (uint8_t)c->hash_proto;
		co[s].index = (uint8_t)s;
		co[s].valid = (uint32_t)c->valid;
		if (!c->valid)
			continue;
		for (i = 0; i < c->num_rule; i++) {
			const pmr_t *r = &G.pmr[c->pmr[i]];

			if (!G.cos[c->linked[i]].valid || !r->valid)
				continue;
			ro[rn].term_begin = tn;
			ro[rn].num_terms = (uint16_t)r->num_terms;
			ro[rn].mark = r->mark;
			ro[rn].dst_cos = (uint32_t)c->linked[i];
			for (t = 0; t < r->num_terms; t++) {
				compile_term(&r->t[t], &to[tn]);
				used |= 1u << to[tn].kind;
				tn++;
			}
			rn++;
		}
		co[s].num_rules = rn - co[s].rule_begin;
	}
	h->used_kinds = used;
	/* stats bitmap: CoS slots with stats_enable */
	memset(e->stats_mask, 0, sizeof(e->stats_mask));
	for (s = 0; s < ncos; s++)
		if (G.cos[s].stats_enable)
			e->stats_mask[s >> 5] |= 1u << (s & 31);
	return (long)bytes;
}

long odp_amd_cls_compile(odp_pktio_t h, void *buf, size_t cap)
{
	pktio_t *e = get_pktio(h);
	long r;

	if (!e)
		return -EINVAL;
	pthread_mutex_lock(&G.lock);
	r = compile_locked(e, buf, cap);
	pthread_mutex_unlock(&G.lock);
	return r;
}

static int ensure_ctx(pktio_t *e);
static int sync_rules(pktio_t *e, void *stream);

int odp_amd_cls_classify(odp_pktio_t h, const uint8_t *pkts_dev, const uint32_t *off_dev,
			 const uint16_t *len_dev, uint32_t n, void *out_dev, void *stream)
{
	pktio_t *e = get_pktio(h);
	int rc;

	if (!e)
		return -EINVAL;
	rc = ensure_ctx(e);
	if (rc)
		return rc;
	/* the options before the rules: a program load specialises the kernel
	 * of the options in force (the option kernel when they are on) */
	mi_cls_pktin_opt_set(e->ctx, e->pktin_opt);
	rc = sync_rules(e, stream);
	if (rc)
		return rc;
	return mi_cls_classify(e->ctx, pkts_dev, off_dev, len_dev, n, (mi_cls_result_t *)out_dev,
			       stream);
}

/* The pktio's pktin parse options (odp_pktio_config() -> config.pktin,
 * used by the receive path as _odp_packet_parse_common's `opt`). */
int odp_amd_cls_pktin_opt_set(odp_pktio_t h, uint64_t opt)
{
	pktio_t *e = get_pktio(h);

	if (!e)
		return -EINVAL;
	e->pktin_opt = opt;
	return 0;
}

odp_queue_t odp_amd_cls_queue_of(uint32_t cos_index, uint32_t slot)
{
	if (!G.init || cos_index >= G.max_cos)
		return ODP_QUEUE_INVALID;
	const cos_t *c = &G.cos[cos_index];

	if (c->queue_group)
		return slot < c->num_queue ? c->hq[slot] : ODP_QUEUE_INVALID;
	return c->queue;
}

/* CoS stats: device per-hop packet counters summed over every pktio that
 * classified with stats enabled (odp_classification.c:1850-1869). */
int odp_cls_cos_stats(odp_cos_t h, odp_cls_cos_stats_t *stats)
{
	cos_t *c = get_cos(h);
	uint64_t buf[256];
	int i;

	if (!c || !stats)
		return -1;
	memset(stats, 0, sizeof(*stats));
	stats->discards = c->stats_discards;
	for (i = 0; i < MAX_PKTIO; i++) {
		pktio_t *e = &G.pktio[i];

		if (!e->used || !e->ctx)
			continue;
		uint32_t nc = e->grp ? mi_cls_group_size(e->grp) : 1u;

		for (uint32_t k = 0; k < nc; k++) {
			mi_cls_ctx_t *x = e->grp ? mi_cls_group_ctx(e->grp, k) : e->ctx;

			if (mi_cls_stats_read(x, buf, 256) == 0)
				stats->packets += buf[c->index];
		}
	}
	return 0;
}

int odp_cls_queue_stats(odp_cos_t h, odp_queue_t q, odp_cls_queue_stats_t *stats)
{
	cos_t *c = get_cos(h);
	uint32_t i, slot = COS_QUEUE_MAX;

	if (!c || !stats)
		return -1;
	if (c->queue_group) {
		for (i = 0; i < c->num_queue; i++)
			if (c->hq[i] == q)
				slot = i;
	} else if (c->queue == q) {
		slot = 0;
	}
	if (slot == COS_QUEUE_MAX) {
		ERR("Invalid odp_queue_t handle\n");
		return -1;
	}
	/* :1871-1898: packets / discards of the enqueue stage */
	memset(stats, 0, sizeof(*stats));
	stats->packets = __atomic_load_n(&c->q_packets[slot], __ATOMIC_RELAXED);
	stats->discards = __atomic_load_n(&c->q_discards[slot], __ATOMIC_RELAXED);
	return 0;
}

static const char *term_name(odp_cls_pmr_term_t t)
{
	static const char *n[] = {
		"PMR_LEN", "PMR_ETHTYPE_0", "PMR_ETHTYPE_X", "PMR_VLAN_ID_0", "PMR_VLAN_ID_X",
		"PMR_VLAN_PCP_0", "PMR_DMAC", "PMR_IPPROTO", "PMR_IP_DSCP", "PMR_UDP_DPORT",
		"PMR_TCP_DPORT", "PMR_UDP_SPORT", "PMR_TCP_SPORT", "PMR_SIP_ADDR", "PMR_DIP_ADDR",
		"PMR_SIP6_ADDR", "PMR_DIP6_ADDR", "PMR_IPSEC_SPI", "PMR_LD_VNI",
		"PMR_CUSTOM_FRAME", "PMR_CUSTOM_L3",
	};

	if ((unsigned)t < sizeof(n) / sizeof(n[0]))
		return n[t];
	return "unknown";
}

static void print_cos_ident(const cos_t *c)
{
	if (c->name[0])
		printf("%s", c->name);
	printf("(%" PRIu64 ")\n", odp_cos_to_u64(cos_hdl(c->index)));
}

/* odp_cls_print_all (:1989-2003) */
void odp_cls_print_all(void)
{
	uint32_t s, j, k, b;

	printf("\nClassifier info\n---------------\n\n");
	if (!G.init)
		return;
	for (s = 0; s < G.max_cos; s++) {
		const cos_t *c = &G.cos[s];
		int first = 1;

		if (!c->valid)
			continue;
		printf("cos: ");
		print_cos_ident(c);
		printf("    queues:\n");
		if (!c->queue_group) {
			if (c->queue == ODP_QUEUE_INVALID)
				printf("        none\n");
			else
				printf("        %" PRIx64 "\n", (uint64_t)(uintptr_t)c->queue);
		} else {
			for (j = 0; j < c->num_queue; j++)
				printf("        %" PRIx64 "\n", (uint64_t)(uintptr_t)c->hq[j]);
		}
		for (j = 0; j < c->num_rule; j++) {
			const pmr_t *r = &G.pmr[c->pmr[j]];

			for (k = 0; k < r->num_terms; k++) {
				const term_t *v = &r->t[k];

				printf(first ? "    rules: " : "           ");
				first = 0;
				printf("%s: ", term_name(v->term));
				if (v->term == ODP_PMR_CUSTOM_FRAME || v->term == ODP_PMR_CUSTOM_L3)
					printf("offset:%" PRIu32 " ", v->offset);
				for (b = 0; b < v->val_sz; b++)
					printf("%02x", v->value[b]);
				printf(" ");
				for (b = 0; b < v->val_sz; b++)
					printf("%02x", v->mask[b]);
				printf(" -> ");
				if (r->mark)
					printf("mark:%u ", r->mark);
				print_cos_ident(&G.cos[c->linked[j]]);
			}
		}
	}
}

/* ABI self-description for binding checks (tests compare these against the
 * ctypes mirrors in odp_amd/cls.py). */
size_t odp_amd_cls_abi_size(int which)
{
	switch (which) {
	case 0: return sizeof(odp_pmr_param_t);
	case 1: return sizeof(odp_pmr_create_opt_t);
	case 2: return sizeof(odp_cls_cos_param_t);
	case 3: return sizeof(odp_cls_capability_t);
	case 4: return sizeof(odp_cls_cos_stats_t);
	case 5: return sizeof(mi_cls_result_t);
	case 6: return sizeof(mi_tbl_hdr_t);
	case 7: return sizeof(mi_cos_t);
	case 8: return sizeof(mi_rule_t);
	case 9: return sizeof(mi_term_t);
	case 100: return offsetof(odp_cls_cos_param_t, pool);
	case 101: return offsetof(odp_cls_cos_param_t, vector);
	case 102: return offsetof(odp_cls_cos_param_t, aggr_enq_profile);
	case 103: return offsetof(odp_cls_capability_t, max_mark);
	case 104: return offsetof(odp_pmr_param_t, val_sz);
	case 105: return offsetof(odp_cls_cos_param_t, hash_proto);
	default: return 0;
	}
}

/* ------------------------------------------------ receive-path host side */

/* _odp_cos_queue_stats_add (odp_classification_internal.h:60-81) */
void odp_amd_cls_queue_stats_add(uint32_t cos_index, uint32_t slot, uint64_t packets,
				 uint64_t discards)
{
	if (!G.init || cos_index >= G.max_cos || slot >= COS_QUEUE_MAX)
		return;
	cos_t *c = &G.cos[cos_index];

	if (packets)
		__atomic_fetch_add(&c->q_packets[slot], packets, __ATOMIC_RELAXED);
	if (discards)
		__atomic_fetch_add(&c->q_discards[slot], discards, __ATOMIC_RELAXED);
}

/* The enqueue flavour of a CoS (cos->vector, odp_classification.c:362-365):
 * *vec_pool / *vec_max for packet vector delivery (use_std_enq == 0),
 * *use_aggr for hash-queue runs redirected to odp_queue_aggr(dst, 0).
 * Returns use_std_enq, or -1 for an invalid index. */
int odp_amd_cls_cos_enq_mode(uint32_t cos_index, odp_pool_t *vec_pool, uint32_t *vec_max,
			     int *use_aggr)
{
	if (!G.init || cos_index >= G.max_cos)
		return -1;
	const cos_t *c = &G.cos[cos_index];

	*vec_pool = c->vec_pool;
	*vec_max = c->vec_max;
	*use_aggr = c->use_aggr;
	return c->use_std_enq;
}

/* 1 when every valid CoS has a pool of its own, other than the pktio's
 * pool: classified packets never come from the pktio's pool (the receive
 * path's pcap burst bound).  A CoS whose pool is the pktio's pool counts as
 * unpooled. */
int odp_amd_cls_all_cos_pooled(odp_pool_t pktio_pool)
{
	int all = 1, any = 0;

	pthread_mutex_lock(&G.lock);
	for (uint32_t i = 0; G.init && i < G.max_cos; i++)
		if (G.cos[i].valid && G.cos[i].action != ODP_COS_ACTION_DROP) {
			/* (a drop CoS never takes a packet) */
			any = 1;
			if (G.cos[i].pool == ODP_POOL_INVALID || G.cos[i].pool == pktio_pool)
				all = 0;
		}
	pthread_mutex_unlock(&G.lock);
	return any && all;
}

/* The receive chain's table (mi_cls_rxtab_t, mi_cls.h) for a pktio whose
 * own pool is pktio_pool: per CoS index its pool slot (slot 0: the pktio's
 * pool; a CoS without a pool of its own takes it, _odp_cls_classify_packet
 * :1760-1764), its queues (get_dest_queue, :395-405) and their queue groups
 * (every enqueueing CoS with the plain enqueue -- no packet vectors, no
 * aggregators -- and at most 64 queues in all: one group per queue).
 * pools[] / *npool: each slot's pool; *gen: the generation the table
 * reflects.  The caller fills pool_cap / rt_slot (runtime pools).  -1 when
 * the control plane does not fit the table. */
int odp_amd_cls_rxtab_fill(odp_pool_t pktio_pool, struct mi_cls_rxtab *tab, odp_pool_t pools[],
			   uint32_t *npool, uint64_t *gen)
{
	odp_queue_t gq[MI_CLS_DLV_GROUPS];
	uint32_t np = 1, nq = 0, ng = 0;
	int plain = 1, rc = 0;

	memset(tab, 0, sizeof(*tab));
	pools[0] = pktio_pool;
	pthread_mutex_lock(&G.lock);
	*gen = G.gen;
	for (uint32_t i = 0; G.init && i < G.max_cos && i < 256 && rc == 0; i++) {
		const cos_t *c = &G.cos[i];

		if (!c->valid)
			continue;
		const odp_pool_t pool = c->pool != ODP_POOL_INVALID ? c->pool : pktio_pool;
		uint32_t k = 0;

		while (k < np && pools[k] != pool)
			k++;
		if (k == np) {
			if (np == MI_CLS_RX_POOLS) {
				rc = -1;
				break;
			}
			pools[np++] = pool;
		}
		const uint32_t n = c->queue_group ? c->num_queue : 1u;

		if (nq + n > MI_CLS_RX_QENT) {
			rc = -1;
			break;
		}
		tab->cos_pool[i] = (uint8_t)k;
		tab->cos_nq[i] = (uint8_t)n;
		tab->cos_q0[i] = (uint16_t)nq;
		for (uint32_t j = 0; j < n; j++) {
			const odp_queue_t q = c->queue_group ? c->hq[j] : c->queue;
			uint32_t g = 0;

			while (g < ng && gq[g] != q)
				g++;
			if (g == ng && c->action == ODP_COS_ACTION_ENQUEUE) {
				if (ng == MI_CLS_DLV_GROUPS)
					plain = 0;
				else
					gq[ng++] = q;
			}
			tab->qh[nq + j] = (uint64_t)(uintptr_t)q;
			tab->qg[nq + j] = (uint8_t)(g < ng ? g : 0xFFu);
		}
		nq += n;
		if (c->action == ODP_COS_ACTION_ENQUEUE && (c->use_std_enq <= 0 || c->use_aggr))
			plain = 0;
	}
	pthread_mutex_unlock(&G.lock);
	tab->flags = MI_CLS_RXT_CLS | (plain ? MI_CLS_RXT_GROUP : 0u);
	tab->npool = np;
	*npool = np;
	return rc;
}

/* One burst's receive chain (mi_cls_rx_chain_submit) on the pktio's
 * context, under the current rules.  -ENOTSUP for pktios over several
 * devices (they take the host-decided delivery). */
int odp_amd_cls_rx_chain(odp_pktio_t h, const uint8_t *pkts, size_t bytes,
			 const struct mi_cls_rxc_args *args, uint64_t *ticket)
{
	pktio_t *e = get_pktio(h);
	int rc;

	if (!e || !ticket)
		return -EINVAL;
	*ticket = 0;
	if (e->grp)
		return -ENOTSUP;
	rc = ensure_ctx(e);
	if (rc)
		return rc;
	mi_cls_pktin_opt_set(e->ctx, e->pktin_opt);
	rc = sync_rules(e, NULL);
	if (rc)
		return rc;
	return mi_cls_rx_chain_submit(e->ctx, pkts, bytes, args, ticket);
}

/* cos->pool of the final CoS (_odp_cls_classify_packet, :1760-1764) */
odp_pool_t odp_amd_cls_pool_of(uint32_t cos_index)
{
	if (!G.init || cos_index >= G.max_cos)
		return ODP_POOL_INVALID;
	return G.cos[cos_index].pool;
}

static int ensure_ctx(pktio_t *e)
{
	if (e->ctx)
		return 0;
	if (e->ngpu > 1) {
		int rc = mi_cls_group_create(e->gpus, (uint32_t)e->ngpu, &e->grp);

		if (rc)
			return rc;
		e->ctx = mi_cls_group_ctx(e->grp, 0);
		return 0;
	}
	return mi_cls_ctx_create(e->gpu, &e->ctx);
}

/* snapshot + upload when the control plane changed (caller: data path) */
static int sync_rules(pktio_t *e, void *stream)
{
	if (e->compiled_gen == G.gen)
		return 0;
	pthread_mutex_lock(&G.lock);
	uint64_t gen = G.gen;
	long need = compile_locked(e, NULL, 0);

	if (need < 0) {
		pthread_mutex_unlock(&G.lock);
		return (int)need;
	}
	if ((size_t)need > e->blob_cap) {
		free(e->blob);
		e->blob = malloc((size_t)need);
		e->blob_cap = e->blob ? (size_t)need : 0;
		if (!e->blob) {
			pthread_mutex_unlock(&G.lock);
			return -ENOMEM;
		}
	}
	compile_locked(e, e->blob, e->blob_cap);
	pthread_mutex_unlock(&G.lock);
	int rc = e->grp ? mi_cls_group_rules_load(e->grp, e->blob, (size_t)need)
			: mi_cls_rules_load(e->ctx, e->blob, (size_t)need, stream);

	if (rc)
		return rc;
	int any = 0;

	for (int i = 0; i < 8; i++)
		any |= e->stats_mask[i] != 0;
	if (e->grp) {
		for (uint32_t k = 0; k < mi_cls_group_size(e->grp); k++)
			mi_cls_stats_enable(mi_cls_group_ctx(e->grp, k), any ? e->stats_mask : NULL);
	} else {
		mi_cls_stats_enable(e->ctx, any ? e->stats_mask : NULL);
	}
	e->compiled_gen = gen;
	return 0;
}

/* Parse-only context: an empty table (no default / error CoS), so every
 * record carries the parse result and outcome DISCARD / PARSE_DROP. */
static int ensure_parse_ctx(pktio_t *e)
{
	if (e->pctx)
		return 0;
	int rc = mi_cls_ctx_create(e->gpu, &e->pctx);

	if (rc)
		return rc;
	mi_tbl_hdr_t h;

	memset(&h, 0, sizeof(h));
	h.magic = MI_CLS_TBL_MAGIC;
	h.version = MI_CLS_TBL_VERSION;
	h.total_bytes = sizeof(h);
	h.default_cos = -1;
	h.error_cos = -1;
	h.max_hops = 1;
	h.cos_off = h.rule_off = h.term_off = sizeof(h);
	rc = mi_cls_rules_load(e->pctx, &h, sizeof(h), NULL);
	if (rc) {
		mi_cls_ctx_destroy(e->pctx);
		e->pctx = NULL;
	}
	return rc;
}

int odp_amd_cls_classify_host(odp_pktio_t h, const uint8_t *pkts, size_t bytes,
			      const uint32_t *off, const uint16_t *len, uint32_t n, void *out,
			      int parse_only)
{
	pktio_t *e = get_pktio(h);
	int rc;

	if (!e)
		return -EINVAL;
	if (parse_only) {
		rc = ensure_parse_ctx(e);
		if (rc)
			return rc;
		mi_cls_pktin_opt_set(e->pctx, e->pktin_opt);
		return mi_cls_classify_host(e->pctx, pkts, bytes, off, len, n,
					    (mi_cls_result_t *)out);
	}
	rc = ensure_ctx(e);
	if (rc)
		return rc;
	if (!e->grp)
		mi_cls_pktin_opt_set(e->ctx, e->pktin_opt);
	rc = sync_rules(e, NULL);
	if (rc)
		return rc;
	if (e->grp) {
		mi_cls_group_pktin_opt_set(e->grp, e->pktin_opt);
		return mi_cls_group_classify_host(e->grp, pkts, bytes, off, len, n,
						  (mi_cls_result_t *)out);
	}
	mi_cls_pktin_opt_set(e->ctx, e->pktin_opt);
	return mi_cls_classify_host(e->ctx, pkts, bytes, off, len, n, (mi_cls_result_t *)out);
}

int odp_amd_cls_classify_host_submit(odp_pktio_t h, const uint8_t *pkts, size_t bytes,
				     const uint32_t *off, const uint16_t *len, uint32_t n,
				     void *out, uint64_t *ticket)
{
	pktio_t *e = get_pktio(h);
	int rc;

	if (!e || !ticket)
		return -EINVAL;
	*ticket = 0;
	rc = ensure_ctx(e);
	if (rc)
		return rc;
	if (!e->grp)
		mi_cls_pktin_opt_set(e->ctx, e->pktin_opt);
	rc = sync_rules(e, NULL);
	if (rc)
		return rc;
	if (e->grp) {
		/* every device's slice in flight (page-locked bursts; pageable
		 * ones complete here with ticket 0) */
		mi_cls_group_pktin_opt_set(e->grp, e->pktin_opt);
		return mi_cls_group_classify_host_submit(e->grp, pkts, bytes, off, len, n,
							 (mi_cls_result_t *)out, ticket);
	}
	mi_cls_pktin_opt_set(e->ctx, e->pktin_opt);
	return mi_cls_classify_host_submit(e->ctx, pkts, bytes, off, len, n,
					   (mi_cls_result_t *)out, ticket);
}

int odp_amd_cls_classify_host_wait(odp_pktio_t h, uint64_t ticket)
{
	pktio_t *e = get_pktio(h);

	if (!e)
		return -EINVAL;
	if (ticket == 0)
		return 0;
	if (e->grp)
		return mi_cls_group_classify_host_wait(e->grp, ticket);
	return e->ctx ? mi_cls_classify_host_wait(e->ctx, ticket) : -EINVAL;
}

/* GPU receive delivery of a classified burst (mi_cls_deliver_submit) on the
 * pktio's (first) device; waited for with odp_amd_cls_classify_host_wait. */
int odp_amd_cls_deliver(odp_pktio_t h, const mi_cls_dlv_args_t *args, uint64_t *ticket)
{
	pktio_t *e = get_pktio(h);
	int rc;

	if (!e || !ticket)
		return -EINVAL;
	*ticket = 0;
	rc = ensure_ctx(e);
	if (rc)
		return rc;
	return mi_cls_deliver_submit(e->ctx, args, ticket);
}

/* Wait for a delivery ticket (the first device's ring, also for pktios over
 * several devices, whose classify tickets belong to the group). */
int odp_amd_cls_deliver_wait(odp_pktio_t h, uint64_t ticket)
{
	pktio_t *e = get_pktio(h);

	if (!e || !e->ctx)
		return -EINVAL;
	return ticket ? mi_cls_classify_host_wait(e->ctx, ticket) : 0;
}

/* Kernel instantiation of the pktio's last device launch (mi_cls_last_launch). */
int odp_amd_cls_last_launch(odp_pktio_t h, uint32_t *info, uint32_t n)
{
	pktio_t *e = get_pktio(h);

	if (!e || !e->ctx)
		return -EINVAL;
	return mi_cls_last_launch(e->ctx, info, n);
}

int odp_amd_cls_spec_wait(odp_pktio_t h)
{
	pktio_t *e = get_pktio(h);
	int rc;

	if (!e)
		return -EINVAL;
	rc = ensure_ctx(e);
	if (rc)
		return rc;
	if (!e->grp)
		mi_cls_pktin_opt_set(e->ctx, e->pktin_opt);   /* the options' kernel */
	rc = sync_rules(e, NULL);
	if (rc)
		return rc;
	if (!e->grp)
		return mi_cls_spec_wait(e->ctx);
	for (uint32_t k = 0; k < mi_cls_group_size(e->grp); k++) {
		rc = mi_cls_spec_wait(mi_cls_group_ctx(e->grp, k));
		if (rc)
			return rc;
	}
	return 0;
}

/* pktio start: device context, rule snapshot and a warm-up launch, so the
 * first received burst does not pay for GPU initialisation. */
int odp_amd_cls_prepare(odp_pktio_t h, int parse_only)
{
	static const uint8_t frame[64];
	const uint32_t off = 0;
	const uint16_t len = 60;
	mi_cls_result_t r;

	return odp_amd_cls_classify_host(h, frame, sizeof(frame), &off, &len, 1, &r, parse_only);
}

/* ---- odp_cls_hash_result (:407-437): the host form of get_dest_queue ---- */
static const uint32_t rss_key[10] = {
	0x6d5a56dau, 0x255b0ec2u, 0x4167253du, 0x43a38fb0u, 0xd0ca2bcbu,
	0xae7b30b4u, 0x77cb2da3u, 0x8030f20cu, 0x6a42b73bu, 0xbeac01fau,
};

/* thash_softrss (protocols/thash.h:82-99), one tuple word */
static uint32_t thash_word(uint32_t w, uint32_t j)
{
	uint32_t h = 0, i;

	for (i = 0; i < 32; i++)
		if (w & (1u << (31 - i)))
			h ^= (rss_key[j] << i) | (i ? rss_key[j + 1] >> (32 - i) : 0u);
	return h;
}

static uint32_t rd32(const uint8_t *p)
{
	uint32_t v;

	memcpy(&v, p, 4);
	return v;
}

/* packet_rss_hash (:1773-1839) over a parsed frame */
uint32_t odp_amd_cls_rss_hash(const uint8_t *base, uint64_t in_flags, uint32_t l3, uint32_t l4,
			      uint32_t hp)
{
	const uint64_t F_IPV4 = 1ull << 13, F_IPV6 = 1ull << 14, F_UDP = 1ull << 22,
		       F_TCP = 1ull << 23;
	uint32_t h = 0, j = 0, i;
	int l4on = ((in_flags & F_TCP) && (hp & 8u)) || ((in_flags & F_UDP) && (hp & 4u));

	if (in_flags & F_IPV4) {
		if (hp & 1u) {
			h ^= thash_word(rd32(base + l3 + 12), 0);
			h ^= thash_word(rd32(base + l3 + 16), 1);
			j = 2;
		}
		if (l4on && j == 2)   /* L4 without L3: undefined in the reference */
			h ^= thash_word(rd32(base + l4), 2);
	} else if (in_flags & F_IPV6) {
		if (hp & 2u) {
			for (i = 0; i < 4; i++) {
				h ^= thash_word(__builtin_bswap32(rd32(base + l3 + 8 + 4 * i)), i);
				h ^= thash_word(__builtin_bswap32(rd32(base + l3 + 24 + 4 * i)), 4 + i);
			}
			j = 8;
		}
		if (l4on && j == 8)
			h ^= thash_word(rd32(base + l4), 8);
	}
	return h;
}

/* runtime accessor (odp_rt.c) */
int _odp_amd_packet_parse_info(odp_packet_t pkt, const uint8_t **data, uint64_t *in_flags,
			       uint32_t *l3, uint32_t *l4);

odp_queue_t odp_cls_hash_result(odp_cos_t h, odp_packet_t packet)
{
	cos_t *c = get_cos(h);
	const uint8_t *data;
	uint64_t fl;
	uint32_t l3, l4;

	if (!c || packet == ODP_PACKET_INVALID)
		return ODP_QUEUE_INVALID;
	if (c->num_queue == 1)
		return c->queue;
	if (_odp_amd_packet_parse_info(packet, &data, &fl, &l3, &l4))
		return ODP_QUEUE_INVALID;
	uint32_t hash = odp_amd_cls_rss_hash(data, fl, l3, l4, c->hash_proto) & (COS_QUEUE_MAX - 1);

	return c->hq[hash % c->num_queue];
}
