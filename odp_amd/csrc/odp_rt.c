/*
 * odp_rt.c -- the ODP runtime subset around the MI355X classifier receive
 * path: init/term, threads, time, cpumask, system info, shared memory,
 * pools, packets, events, event vectors, queues (plain, scheduled,
 * aggregator) and the scheduler.
 *
 * Scope: what an ODP application on top of the
 * classifier needs -- example/classifier/odp_classifier.c compiles and runs
 * against this unchanged.  Semantics follow the API spec
 * (include/odp/api/spec/ headers); the linux-generic implementation
 * (platform/linux-generic/odp_{init,shared_memory,pool,packet,queue_basic,
 * schedule_basic,event_vector,time,cpumask}.c) is the behavioural
 * reference.  Everything here is host C: the data-plane compute
 * (parse + classify) runs on the GPU behind odp_pktio.c.
 *
 * Design notes:
 *  - packets are single-segment: one pool element holds the header, a
 *    128 B headroom (odp_config_internal.h:105), the data capacity of the
 *    pool (max(pkt.len, pkt.seg_len)) and a tailroom;
 *  - queues are spinlocked growable rings; scheduled queues sit on one
 *    scheduler list scanned by priority (higher value = higher priority,
 *    schedule.h odp_schedule_max_prio) with a rotating start per thread;
 *  - ATOMIC queues are held by one thread from the schedule call that
 *    returned their events until its next schedule call (or
 *    odp_schedule_release_atomic); ORDERED queues are scheduled the same way
 *    (atomic scheduling satisfies the ordered guarantees);
 *  - SCHED-mode packet input is polled from odp_schedule*(): a started
 *    pktio is received in GPU-sized bursts by whichever thread gets its
 *    receive lock (the reference scheduler's pktin poll command,
 *    schedule_basic.c sched_cb_pktin_poll).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <inttypes.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "odp_rt_internal.h"

/* ================================================================ globals */
static struct {
	int init;
	odp_init_t param;
	int thr_count;
	odp_spinlock_t lock;        /* pool / queue / shm table changes */
	rt_pool_t pool[RT_MAX_POOLS];
	rt_queue_t queue[RT_MAX_QUEUES];
	/* scheduler list */
	rt_queue_t *sched[RT_MAX_QUEUES];
	int num_sched;
	odp_spinlock_t sched_lock;
	int sched_configured;
} RT;

static void pool_cache_flush(int idx);
static __thread int tls_thr_id = -1;
static __thread odp_thread_type_t tls_thr_type = ODP_THREAD_CONTROL;
static __thread rt_queue_t *tls_atomic;     /* held atomic/ordered queue */
static __thread uint32_t tls_rr;
static __thread int tls_paused;

int rt_thread_id(void)
{
	return tls_thr_id < 0 ? 0 : tls_thr_id;
}

/* ================================================================ init */
void odp_init_param_init(odp_init_t *param)
{
	memset(param, 0, sizeof(*param));
	param->mem_model = ODP_MEM_MODEL_THREAD;
}

int odp_init_global(odp_instance_t *instance, const odp_init_t *params,
		    const odp_platform_init_t *platform_params)
{
	(void)platform_params;
	if (!instance)
		return -1;
	if (params)
		RT.param = *params;
	else
		odp_init_param_init(&RT.param);
	odp_spinlock_init(&RT.lock);
	odp_spinlock_init(&RT.sched_lock);
	RT.init = 1;
	*instance = (odp_instance_t)0x0dbadf00dull;
	return 0;
}

int odp_init_local(odp_instance_t instance, odp_thread_type_t thr_type)
{
	(void)instance;
	if (tls_thr_id >= 0) {
		RT_ERR("thread already initialised\n");
		return -1;
	}
	tls_thr_id = __atomic_fetch_add(&RT.thr_count, 1, __ATOMIC_RELAXED);
	if (tls_thr_id >= ODP_THREAD_COUNT_MAX) {
		__atomic_fetch_sub(&RT.thr_count, 1, __ATOMIC_RELAXED);
		tls_thr_id = -1;
		return -1;
	}
	tls_thr_type = thr_type;
	return 0;
}

int odp_term_local(void)
{
	if (tls_thr_id < 0)
		return -1;
	odp_schedule_release_atomic();
	for (int i = 0; i < RT_MAX_POOLS; i++)
		pool_cache_flush(i);
	tls_thr_id = -1;
	/* returns the number of threads still running (init.h) */
	return __atomic_sub_fetch(&RT.thr_count, 1, __ATOMIC_RELAXED) > 0;
}

int odp_term_global(odp_instance_t instance)
{
	(void)instance;
	RT.init = 0;
	return 0;
}

int odp_thread_id(void)
{
	return rt_thread_id();
}

int odp_thread_count(void)
{
	return __atomic_load_n(&RT.thr_count, __ATOMIC_RELAXED);
}

int odp_thread_count_max(void)
{
	return ODP_THREAD_COUNT_MAX;
}

odp_thread_type_t odp_thread_type(void)
{
	return tls_thr_type;
}

int odp_cpu_id(void)
{
	int c = sched_getcpu();

	return c < 0 ? 0 : c;
}

int odp_cpu_count(void)
{
	cpu_set_t s;

	if (sched_getaffinity(0, sizeof(s), &s))
		return 1;
	return CPU_COUNT(&s);
}

/* ================================================================ time */
static uint64_t now_ns(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * ODP_TIME_SEC_IN_NS + (uint64_t)ts.tv_nsec;
}

odp_time_t odp_time_local(void) { odp_time_t t; t.nsec = now_ns(); return t; }
odp_time_t odp_time_global(void) { return odp_time_local(); }
uint64_t odp_time_local_ns(void) { return now_ns(); }
uint64_t odp_time_global_ns(void) { return now_ns(); }
odp_time_t odp_time_diff(odp_time_t t2, odp_time_t t1) { odp_time_t t; t.nsec = t2.nsec - t1.nsec; return t; }
uint64_t odp_time_diff_ns(odp_time_t t2, odp_time_t t1) { return t2.nsec - t1.nsec; }
odp_time_t odp_time_sum(odp_time_t t1, odp_time_t t2) { odp_time_t t; t.nsec = t1.nsec + t2.nsec; return t; }
uint64_t odp_time_to_ns(odp_time_t time) { return time.nsec; }
odp_time_t odp_time_local_from_ns(uint64_t ns) { odp_time_t t; t.nsec = ns; return t; }
int odp_time_cmp(odp_time_t t2, odp_time_t t1) { return t2.nsec > t1.nsec ? 1 : (t2.nsec < t1.nsec ? -1 : 0); }
uint64_t odp_time_local_res(void) { return ODP_TIME_SEC_IN_NS; }

void odp_time_wait_ns(uint64_t ns)
{
	struct timespec ts = { (time_t)(ns / ODP_TIME_SEC_IN_NS), (long)(ns % ODP_TIME_SEC_IN_NS) };

	nanosleep(&ts, NULL);
}

/* ================================================================ cpumask */
void odp_cpumask_zero(odp_cpumask_t *m) { memset(m, 0, sizeof(*m)); }
void odp_cpumask_set(odp_cpumask_t *m, int c) { if (c >= 0 && c < ODP_CPUMASK_SIZE) m->bits[c / 64] |= 1ull << (c % 64); }
void odp_cpumask_clr(odp_cpumask_t *m, int c) { if (c >= 0 && c < ODP_CPUMASK_SIZE) m->bits[c / 64] &= ~(1ull << (c % 64)); }
int odp_cpumask_isset(const odp_cpumask_t *m, int c) { return c >= 0 && c < ODP_CPUMASK_SIZE && ((m->bits[c / 64] >> (c % 64)) & 1); }
void odp_cpumask_copy(odp_cpumask_t *d, const odp_cpumask_t *s) { *d = *s; }

void odp_cpumask_setall(odp_cpumask_t *m)
{
	odp_cpumask_all_available(m);
}

int odp_cpumask_count(const odp_cpumask_t *m)
{
	int n = 0;

	for (int i = 0; i < ODP_CPUMASK_SIZE / 64; i++)
		n += __builtin_popcountll(m->bits[i]);
	return n;
}

int odp_cpumask_next(const odp_cpumask_t *m, int cpu)
{
	for (int c = cpu + 1; c < ODP_CPUMASK_SIZE; c++)
		if (odp_cpumask_isset(m, c))
			return c;
	return -1;
}

int odp_cpumask_first(const odp_cpumask_t *m)
{
	return odp_cpumask_next(m, -1);
}

int odp_cpumask_last(const odp_cpumask_t *m)
{
	for (int c = ODP_CPUMASK_SIZE - 1; c >= 0; c--)
		if (odp_cpumask_isset(m, c))
			return c;
	return -1;
}

/* hex string, most significant nibble first, "0x" prefix (cpumask.h) */
int32_t odp_cpumask_to_str(const odp_cpumask_t *m, char *str, int32_t size)
{
	int last = odp_cpumask_last(m);
	int nib = last < 0 ? 1 : last / 4 + 1;

	if (size < nib + 3)
		return -1;
	str[0] = '0';
	str[1] = 'x';
	for (int i = 0; i < nib; i++) {
		int n = nib - 1 - i, v = 0;

		for (int b = 0; b < 4; b++)
			v |= odp_cpumask_isset(m, n * 4 + b) << b;
		str[2 + i] = "0123456789abcdef"[v];
	}
	str[2 + nib] = 0;
	return nib + 3;
}

void odp_cpumask_from_str(odp_cpumask_t *m, const char *str)
{
	odp_cpumask_zero(m);
	if (!str)
		return;
	if (str[0] == '0' && (str[1] == 'x' || str[1] == 'X'))
		str += 2;
	int len = (int)strlen(str);

	for (int i = 0; i < len; i++) {
		char ch = str[len - 1 - i];
		int v = (ch >= '0' && ch <= '9') ? ch - '0' :
			(ch >= 'a' && ch <= 'f') ? ch - 'a' + 10 :
			(ch >= 'A' && ch <= 'F') ? ch - 'A' + 10 : -1;

		if (v < 0)
			return;
		for (int b = 0; b < 4; b++)
			if (v & (1 << b))
				odp_cpumask_set(m, i * 4 + b);
	}
}

int odp_cpumask_all_available(odp_cpumask_t *m)
{
	cpu_set_t s;

	odp_cpumask_zero(m);
	if (sched_getaffinity(0, sizeof(s), &s)) {
		odp_cpumask_set(m, 0);
		return 1;
	}
	for (int c = 0; c < CPU_SETSIZE && c < ODP_CPUMASK_SIZE; c++)
		if (CPU_ISSET(c, &s))
			odp_cpumask_set(m, c);
	return odp_cpumask_count(m);
}

/* linux-generic keeps the first CPU for control threads when it can
 * (odp_cpumask_task.c); workers get the rest, lowest first. */
int odp_cpumask_default_worker(odp_cpumask_t *mask, int num)
{
	odp_cpumask_t all;
	int avail = odp_cpumask_all_available(&all), first = odp_cpumask_first(&all), n = 0;

	if (avail > 1)
		odp_cpumask_clr(&all, first);
	if (num <= 0 || num > odp_cpumask_count(&all))
		num = odp_cpumask_count(&all);
	odp_cpumask_zero(mask);
	for (int c = odp_cpumask_first(&all); c >= 0 && n < num; c = odp_cpumask_next(&all, c)) {
		odp_cpumask_set(mask, c);
		n++;
	}
	return n;
}

int odp_cpumask_default_control(odp_cpumask_t *mask, int num)
{
	odp_cpumask_t all;

	(void)num;
	odp_cpumask_all_available(&all);
	odp_cpumask_zero(mask);
	odp_cpumask_set(mask, odp_cpumask_first(&all));
	return 1;
}

/* ================================================================ system */
const char *odp_version_api_str(void) { return "1.50.0"; }
const char *odp_version_impl_name(void) { return "odp-amd-mi355x"; }
const char *odp_version_impl_str(void) { return "odp-amd-mi355x 0.1 (gfx950 parse+classify receive path)"; }
uint64_t odp_sys_page_size(void) { return (uint64_t)sysconf(_SC_PAGESIZE); }
int odp_sys_cache_line_size(void) { return ODP_CACHE_LINE_SIZE; }

void odp_sys_info_print(void)
{
	char model[128] = "unknown";
	FILE *f = fopen("/proc/cpuinfo", "r");

	if (f) {
		char line[256];

		while (fgets(line, sizeof(line), f)) {
			if (strncmp(line, "model name", 10) == 0) {
				char *p = strchr(line, ':');

				if (p) {
					p += 2;
					p[strcspn(p, "\n")] = 0;
					snprintf(model, sizeof(model), "%s", p);
				}
				break;
			}
		}
		fclose(f);
	}
	printf("\nODP system info\n---------------\n"
	       "ODP API version: %s\nODP impl name:   %s\nODP impl details: %s\n"
	       "CPU model:       %s\nCPU count:       %i\nCache line size: %i\n"
	       "Packet path:     parse + classify on GPU %u (gfx950)\n\n",
	       odp_version_api_str(), odp_version_impl_name(), odp_version_impl_str(),
	       model, odp_cpu_count(), ODP_CACHE_LINE_SIZE, rt_gpu_index());
}

/* ================================================================ shm */
typedef struct {
	int used;
	char name[ODP_SHM_NAME_LEN];
	void *addr;
	uint64_t size;
	uint32_t flags;
} rt_shm_t;

#define RT_MAX_SHM 256
static rt_shm_t shm_tbl[RT_MAX_SHM];
static odp_spinlock_t shm_lock;

odp_shm_t odp_shm_reserve(const char *name, uint64_t size, uint64_t align, uint32_t flags)
{
	odp_shm_t h = ODP_SHM_INVALID;

	if (align < ODP_CACHE_LINE_SIZE)
		align = ODP_CACHE_LINE_SIZE;
	odp_spinlock_lock(&shm_lock);
	for (int i = 0; i < RT_MAX_SHM; i++) {
		if (shm_tbl[i].used)
			continue;
		void *p = NULL;

		if (posix_memalign(&p, (size_t)align, (size_t)(size ? size : 1)))
			break;
		memset(p, 0, (size_t)(size ? size : 1));
		shm_tbl[i].used = 1;
		shm_tbl[i].addr = p;
		shm_tbl[i].size = size;
		shm_tbl[i].flags = flags;
		snprintf(shm_tbl[i].name, sizeof(shm_tbl[i].name), "%s", name ? name : "");
		h = (odp_shm_t)(uintptr_t)(i + 1);
		break;
	}
	odp_spinlock_unlock(&shm_lock);
	return h;
}

static rt_shm_t *get_shm(odp_shm_t h)
{
	uintptr_t i = (uintptr_t)h;

	if (i == 0 || i > RT_MAX_SHM || !shm_tbl[i - 1].used)
		return NULL;
	return &shm_tbl[i - 1];
}

int odp_shm_free(odp_shm_t h)
{
	odp_spinlock_lock(&shm_lock);
	rt_shm_t *s = get_shm(h);

	if (!s) {
		odp_spinlock_unlock(&shm_lock);
		return -1;
	}
	free(s->addr);
	memset(s, 0, sizeof(*s));
	odp_spinlock_unlock(&shm_lock);
	return 0;
}

odp_shm_t odp_shm_lookup(const char *name)
{
	for (int i = 0; i < RT_MAX_SHM; i++)
		if (shm_tbl[i].used && name && strcmp(shm_tbl[i].name, name) == 0)
			return (odp_shm_t)(uintptr_t)(i + 1);
	return ODP_SHM_INVALID;
}

void *odp_shm_addr(odp_shm_t h)
{
	rt_shm_t *s = get_shm(h);

	return s ? s->addr : NULL;
}

int odp_shm_info(odp_shm_t h, odp_shm_info_t *info)
{
	rt_shm_t *s = get_shm(h);

	if (!s || !info)
		return -1;
	info->name = s->name;
	info->addr = s->addr;
	info->size = s->size;
	info->page_size = odp_sys_page_size();
	info->flags = s->flags;
	info->num_seg = 1;
	return 0;
}

uint64_t odp_shm_to_u64(odp_shm_t h) { return (uint64_t)(uintptr_t)h; }

void odp_shm_print_all(void)
{
	printf("\nShared memory blocks\n");
	for (int i = 0; i < RT_MAX_SHM; i++)
		if (shm_tbl[i].used)
			printf("  %2i %-32s %" PRIu64 " B\n", i, shm_tbl[i].name, shm_tbl[i].size);
}

/* ================================================================ pools */
rt_pool_t *rt_pool(odp_pool_t h)
{
	uintptr_t i = (uintptr_t)h;

	if (i == 0 || i > RT_MAX_POOLS || !RT.pool[i - 1].used)
		return NULL;
	return &RT.pool[i - 1];
}

void odp_pool_param_init(odp_pool_param_t *p)
{
	memset(p, 0, sizeof(*p));
	p->pkt.headroom = RT_PKT_HEADROOM;
	p->buf.align = ODP_CACHE_LINE_SIZE;
}

int odp_pool_capability(odp_pool_capability_t *capa)
{
	memset(capa, 0, sizeof(*capa));
	capa->max_pools = RT_MAX_POOLS;
	capa->pkt.max_pools = RT_MAX_POOLS;
	capa->pkt.max_len = 65535;
	capa->pkt.max_num = 1u << 22;
	capa->pkt.max_headroom = RT_PKT_HEADROOM;
	capa->pkt.min_headroom = RT_PKT_HEADROOM;
	capa->pkt.max_segs_per_pkt = 1;
	capa->pkt.min_seg_len = 64;
	capa->pkt.max_seg_len = 65535;
	capa->event_vector.max_pools = RT_MAX_POOLS;
	capa->event_vector.max_num = 1u << 20;
	capa->event_vector.max_size = 4096;
	return 0;
}

static size_t align_up(size_t v, size_t a)
{
	return (v + a - 1) / a * a;
}

static int pinned_pools(void)
{
	static int on = -1;

	if (on < 0) {
		const char *v = getenv("ODP_AMD_PINNED_POOLS");

		on = !(v && v[0] == '0');
	}
	return on;
}

/* ODP_AMD_PAGEABLE_POOLS=<name>[,<name>...]: packet pools of these names in
 * ordinary memory (the others page-locked), so one receive burst can take
 * the GPU delivery and the next the host's */
static int pool_pageable(const char *name)
{
	const char *v = getenv("ODP_AMD_PAGEABLE_POOLS");
	const size_t n = name ? strlen(name) : 0;

	while (v && *v && n) {
		const char *c = strchr(v, ',');
		const size_t l = c ? (size_t)(c - v) : strlen(v);

		if (l == n && strncmp(v, name, n) == 0)
			return 1;
		v = c ? c + 1 : NULL;
	}
	return 0;
}

/* 1 when every packet handle of pk[0..n) is a header inside a page-locked
 * pool's memory (the GPU may then read it), else 0.  Only the handles are
 * compared against the pools' address ranges: no header is read. */
int rt_pinned_handles(const odp_packet_t pk[], int n)
{
	uintptr_t lo[RT_MAX_POOLS], hi[RT_MAX_POOLS];
	int np = 0, last = 0;

	for (int i = 0; i < RT_MAX_POOLS; i++) {
		const rt_pool_t *p = &RT.pool[i];

		if (p->used && p->pinned && p->mem) {
			lo[np] = (uintptr_t)p->mem;
			hi[np] = (uintptr_t)p->mem + p->elem_size * p->num;
			np++;
		}
	}
	for (int i = 0; i < n; i++) {
		const uintptr_t a = (uintptr_t)pk[i];

		if (np && a >= lo[last] && a + sizeof(pkt_hdr_t) <= hi[last])
			continue;
		int k = 0;

		while (k < np && !(a >= lo[k] && a + sizeof(pkt_hdr_t) <= hi[k]))
			k++;
		if (k == np)
			return 0;
		last = k;
	}
	return 1;
}

int rt_pinned_arena(uint8_t **lo, size_t *bytes)
{
	uint8_t *a = NULL, *b = NULL;

	for (int i = 0; i < RT_MAX_POOLS; i++) {
		const rt_pool_t *p = &RT.pool[i];

		if (!p->used || !p->pinned || !p->mem)
			continue;
		if (!a || p->mem < a)
			a = p->mem;
		if (!b || p->mem + p->elem_size * p->num > b)
			b = p->mem + p->elem_size * p->num;
	}
	*lo = a;
	*bytes = a ? (size_t)(b - a) : 0;
	return a != NULL;
}

uint32_t rt_data_from_meta(void)
{
	return (uint32_t)(align_up(sizeof(pkt_hdr_t), 64) + RT_PKT_HEADROOM -
			  __builtin_offsetof(pkt_hdr_t, meta));
}

odp_pool_t odp_pool_create(const char *name, const odp_pool_param_t *param)
{
	size_t esz;
	uint32_t num, cap = 0;

	if (!param)
		return ODP_POOL_INVALID;
	switch (param->type) {
	case ODP_POOL_PACKET: {
		uint32_t len = param->pkt.len > param->pkt.seg_len ? param->pkt.len : param->pkt.seg_len;

		if (param->pkt.max_len > len)
			len = param->pkt.max_len;
		if (len == 0)
			len = 1856;
		if (len > 65535 || param->pkt.num == 0) {
			RT_ERR("pool %s: unsupported packet pool parameters\n", name ? name : "");
			return ODP_POOL_INVALID;
		}
		cap = (uint32_t)align_up(len, 64);
		esz = align_up(sizeof(pkt_hdr_t), 64) + RT_PKT_HEADROOM + cap + RT_PKT_TAILROOM;
		num = param->pkt.num;
		break;
	}
	case ODP_POOL_EVENT_VECTOR:
	case ODP_POOL_VECTOR: {
		uint32_t ms = param->type == ODP_POOL_EVENT_VECTOR ? param->event_vector.max_size
								  : param->vector.max_size;
		num = param->type == ODP_POOL_EVENT_VECTOR ? param->event_vector.num : param->vector.num;
		if (ms == 0 || num == 0)
			return ODP_POOL_INVALID;
		cap = ms;
		esz = align_up(sizeof(evv_hdr_t) + (size_t)ms * sizeof(odp_event_t), 64);
		break;
	}
	default:
		RT_ERR("pool type %d is not supported by this build\n", (int)param->type);
		return ODP_POOL_INVALID;
	}

	odp_spinlock_lock(&RT.lock);
	int idx = -1;

	for (int i = 0; i < RT_MAX_POOLS; i++)
		if (!RT.pool[i].used) {
			idx = i;
			break;
		}
	if (idx < 0) {
		odp_spinlock_unlock(&RT.lock);
		return ODP_POOL_INVALID;
	}
	rt_pool_t *p = &RT.pool[idx];

	static uint32_t pool_gen;

	memset(p, 0, sizeof(*p));
	p->used = 1;
	p->gen = ++pool_gen;
	odp_spinlock_unlock(&RT.lock);

	void *mem = NULL;

	/* packet pools in page-locked memory the GPU addresses at the same
	 * addresses: the receive path then classifies loop packets in place and
	 * the GPU writes received packets' metadata and frames into them
	 * (ODP_AMD_PINNED_POOLS=0: ordinary memory, host delivery) */
	if (param->type == ODP_POOL_PACKET && pinned_pools() && !pool_pageable(name)) {
		mem = mi_cls_host_alloc(esz * num);
		if (mem && !mi_cls_host_mapped(mem)) {
			mi_cls_host_free(mem);
			mem = NULL;
		}
		p->pinned = mem != NULL;
	}
	if (!mem && posix_memalign(&mem, 64, esz * num)) {
		p->used = 0;
		return ODP_POOL_INVALID;
	}
	p->mem = mem;
	p->elem_size = esz;
	p->num = num;
	p->data_cap = cap;
	p->param = *param;
	snprintf(p->name, sizeof(p->name), "%s", name ? name : "");
	odp_spinlock_init(&p->lock);
	p->free_stk = malloc((size_t)num * sizeof(ev_hdr_t *));
	if (!p->free_stk) {
		if (p->pinned)
			mi_cls_host_free(p->mem);
		else
			free(p->mem);
		p->used = 0;
		return ODP_POOL_INVALID;
	}
	for (uint32_t i = num; i-- > 0;) {
		ev_hdr_t *e = (ev_hdr_t *)(p->mem + (size_t)i * esz);

		memset(e, 0, sizeof(*e));
		e->pool = (uint16_t)idx;
		e->index = i;
		e->type = param->type == ODP_POOL_PACKET ? ODP_EVENT_PACKET :
			  param->type == ODP_POOL_VECTOR ? ODP_EVENT_PACKET_VECTOR : ODP_EVENT_VECTOR;
		if (param->type == ODP_POOL_PACKET) {
			pkt_hdr_t *h = (pkt_hdr_t *)e;

			h->head = (uint8_t *)e + align_up(sizeof(pkt_hdr_t), 64);
			h->buf_len = RT_PKT_HEADROOM + cap + RT_PKT_TAILROOM;
		} else {
			((evv_hdr_t *)e)->max_size = cap;
		}
		/* the stack's top is element 0 (taken first) */
		p->free_stk[num - 1 - i] = e;
	}
	p->num_free = num;
	return (odp_pool_t)(uintptr_t)(idx + 1);
}

int odp_pool_destroy(odp_pool_t h)
{
	rt_pool_t *p = rt_pool(h);

	if (!p)
		return -1;
	pool_cache_flush((int)(p - RT.pool));
	if (p->num_free != p->num)
		RT_ERR("pool %s destroyed with %u events in use\n", p->name, p->num - p->num_free);
	if (p->pinned)
		mi_cls_host_free(p->mem);
	else
		free(p->mem);
	free(p->free_stk);
	odp_spinlock_lock(&RT.lock);
	memset(p, 0, sizeof(*p));
	odp_spinlock_unlock(&RT.lock);
	return 0;
}

odp_pool_t odp_pool_lookup(const char *name)
{
	for (int i = 0; i < RT_MAX_POOLS; i++)
		if (RT.pool[i].used && name && strcmp(RT.pool[i].name, name) == 0)
			return (odp_pool_t)(uintptr_t)(i + 1);
	return ODP_POOL_INVALID;
}

int odp_pool_info(odp_pool_t h, odp_pool_info_t *info)
{
	rt_pool_t *p = rt_pool(h);

	if (!p || !info)
		return -1;
	memset(info, 0, sizeof(*info));
	info->type = p->param.type;
	info->name = p->name;
	info->params = p->param;
	info->min_data_addr = (uint64_t)(uintptr_t)p->mem;
	info->max_data_addr = (uint64_t)(uintptr_t)(p->mem + p->elem_size * p->num - 1);
	return 0;
}

static const char *pool_type_str(odp_pool_type_t t)
{
	switch (t) {
	case ODP_POOL_PACKET: return "packet";
	case ODP_POOL_EVENT_VECTOR: return "event vector";
	case ODP_POOL_VECTOR: return "packet vector";
	default: return "other";
	}
}

void odp_pool_print(odp_pool_t h)
{
	rt_pool_t *p = rt_pool(h);

	if (!p)
		return;
	printf("Pool info\n---------\n  pool            %" PRIu64 "\n  name            %s\n"
	       "  pool type       %s\n  num             %u\n  free            %u\n"
	       "  data capacity   %u\n  element size    %zu\n\n",
	       odp_pool_to_u64(h), p->name, pool_type_str(p->param.type), p->num, p->num_free,
	       p->data_cap, p->elem_size);
}

void odp_pool_print_all(void)
{
	int n = 0;

	for (int i = 0; i < RT_MAX_POOLS; i++)
		n += RT.pool[i].used;
	printf("\nList of all pools\n-----------------\n  num of pools: %i\n"
	       "  id name                             type          num      free\n", n);
	for (int i = 0; i < RT_MAX_POOLS; i++) {
		rt_pool_t *p = &RT.pool[i];

		if (p->used)
			printf("  %2i %-32s %-13s %-8u %u\n", i + 1, p->name, pool_type_str(p->param.type),
			       p->num, p->num_free);
	}
	printf("\n");
}

uint64_t odp_pool_to_u64(odp_pool_t h) { return (uint64_t)(uintptr_t)h; }
int odp_pool_index(odp_pool_t h) { return rt_pool(h) ? (int)((uintptr_t)h - 1) : -1; }
unsigned int odp_pool_max_index(void) { return RT_MAX_POOLS - 1; }

static int pool_take(rt_pool_t *p, ev_hdr_t *out[], int num)
{
	odp_spinlock_lock(&p->lock);
	const int n = num < (int)p->num_free ? num : (int)p->num_free;

	p->num_free -= (uint32_t)n;
	memcpy(out, p->free_stk + p->num_free, (size_t)n * sizeof(ev_hdr_t *));
	odp_spinlock_unlock(&p->lock);
	return n;
}

static void pool_give(rt_pool_t *p, ev_hdr_t *const e[], int num)
{
	if (num <= 0)
		return;
	odp_spinlock_lock(&p->lock);
	if (p->num_free + (uint32_t)num > p->num) {
		/* more events returned than the pool owns: a double free by the
		 * application -- the excess is dropped, the free stack never grows
		 * past the pool */
		const uint32_t room = p->num - p->num_free;

		RT_ERR("pool %s: %d events freed, room for %u (double free?)\n", p->name, num, room);
		num = (int)room;
	}
	memcpy(p->free_stk + p->num_free, e, (size_t)num * sizeof(ev_hdr_t *));
	p->num_free += (uint32_t)num;
	odp_spinlock_unlock(&p->lock);
}

/* Per-thread cache of free events in front of a large pool's locked free
 * list (as a DPDK mempool cache): allocations and frees take the pool lock
 * once per PC_BATCH events instead of per event.  Pools below PC_MIN_POOL
 * events are not cached (a thread's cache would hold a noticeable share of
 * them away from the others).  Entries are tagged with the pool's creation
 * number; odp_term_local() and odp_pool_destroy() return the calling
 * thread's cached events. */
#define PC_SIZE 512
#define PC_BATCH 256
#define PC_MIN_POOL 4096u
typedef struct {
	uint32_t gen;
	int n;
	ev_hdr_t *e[PC_SIZE];
} pool_cache_t;
/* The thread's caches, one slot per pool, allocated on first use: the TLS
 * itself is one pointer, so the library builds with the initial-exec TLS
 * model (a register-relative load instead of a __tls_get_addr call per
 * packet allocation and free) and still fits the static TLS surplus when it
 * is dlopen()ed. */
static __thread pool_cache_t **tls_pc;

static pool_cache_t *pool_cache(rt_pool_t *p)
{
	const int idx = (int)(p - RT.pool);
	if (p->num < PC_MIN_POOL)
		return NULL;
	if (!tls_pc) {
		tls_pc = calloc(RT_MAX_POOLS, sizeof(*tls_pc));
		if (!tls_pc)
			return NULL;
	}
	pool_cache_t *c = tls_pc[idx];

	if (!c) {
		c = calloc(1, sizeof(*c));
		if (!c)
			return NULL;
		c->gen = p->gen;
		tls_pc[idx] = c;
	}
	if (c->gen != p->gen) {   /* cache of a destroyed pool in this slot */
		c->n = 0;
		c->gen = p->gen;
	}
	return c;
}

static void pool_cache_flush(int idx)
{
	pool_cache_t *c = tls_pc ? tls_pc[idx] : NULL;

	if (c && c->n && RT.pool[idx].used && c->gen == RT.pool[idx].gen)
		pool_give(&RT.pool[idx], c->e, c->n);
	if (c)
		c->n = 0;
}

uint32_t rt_pool_avail(odp_pool_t h)
{
	rt_pool_t *p = rt_pool(h);

	if (!p)
		return 0;
	const pool_cache_t *c = tls_pc ? tls_pc[p - RT.pool] : NULL;

	return p->num_free + (c && c->gen == p->gen ? (uint32_t)c->n : 0u);
}

static int pool_alloc(rt_pool_t *p, ev_hdr_t *out[], int num)
{
	pool_cache_t *c = pool_cache(p);
	int n = 0;

	if (!c)
		return pool_take(p, out, num);
	while (n < num) {
		if (c->n == 0) {
			c->n = pool_take(p, c->e, PC_BATCH);
			if (c->n == 0)
				break;
		}
		int take = num - n < c->n ? num - n : c->n;

		memcpy(out + n, c->e + c->n - take, (size_t)take * sizeof(ev_hdr_t *));
		c->n -= take;
		n += take;
	}
	return n;
}

static void pool_free(ev_hdr_t *e)
{
	rt_pool_t *p = &RT.pool[e->pool];
	pool_cache_t *c = pool_cache(p);

	if (!c) {
		pool_give(p, &e, 1);
		return;
	}
	if (c->n == PC_SIZE) {
		pool_give(p, c->e + PC_SIZE - PC_BATCH, PC_BATCH);
		c->n -= PC_BATCH;
	}
	c->e[c->n++] = e;
}

/* ================================================================ packets */
pkt_hdr_t *rt_pkt_hdr(odp_packet_t pkt)
{
	return (pkt_hdr_t *)(void *)pkt;
}

/* packet_init + packet_parse_reset(hdr, 1) (odp_packet_internal.h:468-479) */
static void pkt_init(pkt_hdr_t *h, uint32_t len)
{
	h->data_off = RT_PKT_HEADROOM;
	h->len = len;
	h->in_flags = 0;
	h->err = 0;
	h->cos = 0xff;
	h->cls_mark = 0;
	h->l2 = 0;   /* odp_packet_alloc sets l2 = 0 (packet.c packet_init) */
	h->l3 = ODP_PACKET_OFFSET_INVALID;
	h->l4 = ODP_PACKET_OFFSET_INVALID;
	h->dst_queue = ODP_QUEUE_INVALID;
	h->input = ODP_PKTIO_INVALID;
	h->user_ptr = NULL;
}

int odp_packet_alloc_multi(odp_pool_t pool, uint32_t len, odp_packet_t pkt[], int num)
{
	rt_pool_t *p = rt_pool(pool);
	ev_hdr_t *e[256];
	int done = 0;

	if (!p || p->param.type != ODP_POOL_PACKET || len > p->data_cap)
		return -1;
	while (done < num) {
		int want = num - done > 256 ? 256 : num - done;
		int got = pool_alloc(p, e, want);

		for (int i = 0; i < got; i++) {
			pkt_init((pkt_hdr_t *)e[i], len);
			pkt[done + i] = (odp_packet_t)(void *)e[i];
		}
		done += got;
		if (got < want)
			break;
	}
	return done;
}

int rt_packet_alloc_raw(odp_pool_t pool, uint32_t len, odp_packet_t pkt[], int num)
{
	rt_pool_t *p = rt_pool(pool);

	if (!p || p->param.type != ODP_POOL_PACKET || len > p->data_cap || num <= 0)
		return 0;
	return pool_alloc(p, (ev_hdr_t **)(void *)pkt, num);
}

/* Packets of one pool back to it at once (taken with rt_packet_alloc_raw and
 * not used): into the calling thread's cache while it has room, the rest
 * onto the pool's stack in one locked copy. */
void rt_packet_return_raw(odp_pool_t pool, const odp_packet_t pkt[], int num)
{
	rt_pool_t *p = rt_pool(pool);

	if (!p || num <= 0)
		return;
	ev_hdr_t *const *e = (ev_hdr_t *const *)(const void *)pkt;
	pool_cache_t *c = pool_cache(p);

	if (c) {
		const int room = PC_SIZE - c->n;
		const int k = num < room ? num : room;

		memcpy(c->e + c->n, e, (size_t)k * sizeof(ev_hdr_t *));
		c->n += k;
		e += k;
		num -= k;
	}
	pool_give(p, e, num);
}

void rt_packet_init(odp_packet_t pkt, uint32_t len)
{
	pkt_init(rt_pkt_hdr(pkt), len);
}

odp_packet_t odp_packet_alloc(odp_pool_t pool, uint32_t len)
{
	odp_packet_t p;

	return odp_packet_alloc_multi(pool, len, &p, 1) == 1 ? p : ODP_PACKET_INVALID;
}

void odp_packet_free(odp_packet_t pkt)
{
	if (pkt != ODP_PACKET_INVALID)
		pool_free(&rt_pkt_hdr(pkt)->ev);
}

void odp_packet_free_multi(const odp_packet_t pkt[], int num)
{
	for (int i = 0; i < num; i++)
		odp_packet_free(pkt[i]);
}

odp_packet_t odp_packet_from_event(odp_event_t ev) { return (odp_packet_t)(void *)ev; }
odp_event_t odp_packet_to_event(odp_packet_t pkt) { return (odp_event_t)(void *)pkt; }

void odp_packet_from_event_multi(odp_packet_t pkt[], const odp_event_t ev[], int num)
{
	for (int i = 0; i < num; i++)
		pkt[i] = odp_packet_from_event(ev[i]);
}

void odp_packet_to_event_multi(const odp_packet_t pkt[], odp_event_t ev[], int num)
{
	for (int i = 0; i < num; i++)
		ev[i] = odp_packet_to_event(pkt[i]);
}

uint32_t odp_packet_len(odp_packet_t pkt) { return rt_pkt_hdr(pkt)->len; }
uint32_t odp_packet_seg_len(odp_packet_t pkt) { return rt_pkt_hdr(pkt)->len; }
uint32_t odp_packet_buf_len(odp_packet_t pkt) { return rt_pkt_hdr(pkt)->buf_len; }
uint32_t odp_packet_headroom(odp_packet_t pkt) { return rt_pkt_hdr(pkt)->data_off; }
void *odp_packet_data(odp_packet_t pkt) { pkt_hdr_t *h = rt_pkt_hdr(pkt); return h->head + h->data_off; }
void *odp_packet_head(odp_packet_t pkt) { return rt_pkt_hdr(pkt)->head; }
int odp_packet_num_segs(odp_packet_t pkt) { (void)pkt; return 1; }
int odp_packet_is_segmented(odp_packet_t pkt) { (void)pkt; return 0; }
odp_pool_t odp_packet_pool(odp_packet_t pkt) { return (odp_pool_t)(uintptr_t)(rt_pkt_hdr(pkt)->ev.pool + 1); }
odp_pktio_t odp_packet_input(odp_packet_t pkt) { return rt_pkt_hdr(pkt)->input; }
int odp_packet_input_index(odp_packet_t pkt) { return rt_pkt_hdr(pkt)->input ? (int)((uintptr_t)rt_pkt_hdr(pkt)->input - 1) : -1; }
void *odp_packet_user_ptr(odp_packet_t pkt) { return (void *)(uintptr_t)rt_pkt_hdr(pkt)->user_ptr; }
void odp_packet_user_ptr_set(odp_packet_t pkt, const void *p) { rt_pkt_hdr(pkt)->user_ptr = p; }
uint64_t odp_packet_to_u64(odp_packet_t hdl) { return (uint64_t)(uintptr_t)hdl; }

uint32_t odp_packet_tailroom(odp_packet_t pkt)
{
	pkt_hdr_t *h = rt_pkt_hdr(pkt);

	return h->buf_len - h->data_off - h->len;
}

void *odp_packet_tail(odp_packet_t pkt)
{
	pkt_hdr_t *h = rt_pkt_hdr(pkt);

	return h->head + h->data_off + h->len;
}

void *odp_packet_offset(odp_packet_t pkt, uint32_t offset, uint32_t *len, void *seg)
{
	pkt_hdr_t *h = rt_pkt_hdr(pkt);

	(void)seg;
	if (offset >= h->len)
		return NULL;
	if (len)
		*len = h->len - offset;
	return h->head + h->data_off + offset;
}

void *odp_packet_push_head(odp_packet_t pkt, uint32_t len)
{
	pkt_hdr_t *h = rt_pkt_hdr(pkt);

	if (len > h->data_off)
		return NULL;
	h->data_off -= len;
	h->len += len;
	return h->head + h->data_off;
}

void *odp_packet_pull_head(odp_packet_t pkt, uint32_t len)
{
	pkt_hdr_t *h = rt_pkt_hdr(pkt);

	if (len >= h->len)
		return NULL;
	h->data_off += len;
	h->len -= len;
	return h->head + h->data_off;
}

void *odp_packet_push_tail(odp_packet_t pkt, uint32_t len)
{
	pkt_hdr_t *h = rt_pkt_hdr(pkt);
	void *t = odp_packet_tail(pkt);

	if (len > odp_packet_tailroom(pkt))
		return NULL;
	h->len += len;
	return t;
}

void *odp_packet_pull_tail(odp_packet_t pkt, uint32_t len)
{
	pkt_hdr_t *h = rt_pkt_hdr(pkt);

	if (len >= h->len)
		return NULL;
	h->len -= len;
	return odp_packet_tail(pkt);
}

int odp_packet_copy_to_mem(odp_packet_t pkt, uint32_t offset, uint32_t len, void *dst)
{
	pkt_hdr_t *h = rt_pkt_hdr(pkt);

	if ((uint64_t)offset + len > h->len)
		return -1;
	memcpy(dst, h->head + h->data_off + offset, len);
	return 0;
}

int odp_packet_copy_from_mem(odp_packet_t pkt, uint32_t offset, uint32_t len, const void *src)
{
	pkt_hdr_t *h = rt_pkt_hdr(pkt);

	if ((uint64_t)offset + len > h->len)
		return -1;
	memcpy(h->head + h->data_off + offset, src, len);
	return 0;
}

/* full copy with metadata into another pool (_odp_pktio_packet_to_pool,
 * odp_packet_io_internal.h:352-371, uses odp_packet_copy) */
odp_packet_t odp_packet_copy(odp_packet_t pkt, odp_pool_t pool)
{
	pkt_hdr_t *s = rt_pkt_hdr(pkt);
	odp_packet_t n = odp_packet_alloc(pool, s->len);

	if (n == ODP_PACKET_INVALID)
		return n;
	pkt_hdr_t *d = rt_pkt_hdr(n);

	memcpy(d->head + d->data_off, s->head + s->data_off, s->len);
	d->in_flags = s->in_flags;
	d->err = s->err;
	d->cos = s->cos;
	d->cls_mark = s->cls_mark;
	d->l2 = s->l2;
	d->l3 = s->l3;
	d->l4 = s->l4;
	d->dst_queue = s->dst_queue;
	d->input = s->input;
	d->user_ptr = s->user_ptr;
	return n;
}

int odp_packet_is_valid(odp_packet_t pkt)
{
	if (pkt == ODP_PACKET_INVALID)
		return 0;
	pkt_hdr_t *h = rt_pkt_hdr(pkt);

	return h->ev.type == ODP_EVENT_PACKET && h->ev.pool < RT_MAX_POOLS && RT.pool[h->ev.pool].used;
}

static void *layer_ptr(odp_packet_t pkt, uint16_t off, uint32_t *len)
{
	pkt_hdr_t *h = rt_pkt_hdr(pkt);

	if (off == ODP_PACKET_OFFSET_INVALID || off >= h->len)
		return NULL;
	if (len)
		*len = h->len - off;
	return h->head + h->data_off + off;
}

void *odp_packet_l2_ptr(odp_packet_t pkt, uint32_t *len) { return layer_ptr(pkt, rt_pkt_hdr(pkt)->l2, len); }
void *odp_packet_l3_ptr(odp_packet_t pkt, uint32_t *len) { return layer_ptr(pkt, rt_pkt_hdr(pkt)->l3, len); }
void *odp_packet_l4_ptr(odp_packet_t pkt, uint32_t *len) { return layer_ptr(pkt, rt_pkt_hdr(pkt)->l4, len); }
uint32_t odp_packet_l2_offset(odp_packet_t pkt) { return rt_pkt_hdr(pkt)->l2; }
uint32_t odp_packet_l3_offset(odp_packet_t pkt) { return rt_pkt_hdr(pkt)->l3; }
uint32_t odp_packet_l4_offset(odp_packet_t pkt) { return rt_pkt_hdr(pkt)->l4; }

static int set_off(odp_packet_t pkt, uint16_t *f, uint32_t off)
{
	if (off >= rt_pkt_hdr(pkt)->len)
		return -1;
	*f = (uint16_t)off;
	return 0;
}

int odp_packet_l2_offset_set(odp_packet_t pkt, uint32_t o) { return set_off(pkt, &rt_pkt_hdr(pkt)->l2, o); }
int odp_packet_l3_offset_set(odp_packet_t pkt, uint32_t o) { return set_off(pkt, &rt_pkt_hdr(pkt)->l3, o); }
int odp_packet_l4_offset_set(odp_packet_t pkt, uint32_t o) { return set_off(pkt, &rt_pkt_hdr(pkt)->l4, o); }

uint64_t odp_packet_cls_mark(odp_packet_t pkt)
{
	pkt_hdr_t *h = rt_pkt_hdr(pkt);

	return (h->in_flags & 1u) ? h->cls_mark : 0;
}

/* packet_flags.h over input_flags (packet_inline_types.h:60-107) and the
 * error bits (:152-165: snap_len, ip, l3_chksum, tcp, udp, sctp, l4_chksum) */
#define FLAG(name, bit) \
	int odp_packet_has_##name(odp_packet_t pkt) { return (int)((rt_pkt_hdr(pkt)->in_flags >> (bit)) & 1u); }
FLAG(flow_hash, 1)
FLAG(ts, 2)
FLAG(l2, 3)
FLAG(l3, 4)
FLAG(l4, 5)
FLAG(eth, 6)
FLAG(eth_bcast, 7)
FLAG(eth_mcast, 8)
FLAG(jumbo, 9)
FLAG(vlan, 10)
FLAG(vlan_qinq, 11)
FLAG(arp, 12)
FLAG(ipv4, 13)
FLAG(ipv6, 14)
FLAG(ip_bcast, 15)
FLAG(ip_mcast, 16)
FLAG(ipfrag, 17)
FLAG(ipopt, 18)
FLAG(ipsec, 19)
FLAG(udp, 22)
FLAG(tcp, 23)
FLAG(sctp, 24)
FLAG(icmp, 25)
#undef FLAG

int odp_packet_has_error(odp_packet_t pkt) { return rt_pkt_hdr(pkt)->err != 0; }
int odp_packet_has_l2_error(odp_packet_t pkt) { return (rt_pkt_hdr(pkt)->err & 0x01) != 0; }
int odp_packet_has_l3_error(odp_packet_t pkt) { return (rt_pkt_hdr(pkt)->err & 0x06) != 0; }
int odp_packet_has_l4_error(odp_packet_t pkt) { return (rt_pkt_hdr(pkt)->err & 0x78) != 0; }

/* packet_inlines.h:389-420: input_flags l3/l4_chksum_done (bits 30/31),
 * error bits l3_chksum_err (2) / l4_chksum_err (6) */
odp_packet_chksum_status_t odp_packet_l3_chksum_status(odp_packet_t pkt)
{
	const pkt_hdr_t *h = rt_pkt_hdr(pkt);

	if (!((h->in_flags >> 30) & 1u))
		return ODP_PACKET_CHKSUM_UNKNOWN;
	return (h->err & 0x04) ? ODP_PACKET_CHKSUM_BAD : ODP_PACKET_CHKSUM_OK;
}

odp_packet_chksum_status_t odp_packet_l4_chksum_status(odp_packet_t pkt)
{
	const pkt_hdr_t *h = rt_pkt_hdr(pkt);

	if (!((h->in_flags >> 31) & 1u))
		return ODP_PACKET_CHKSUM_UNKNOWN;
	return (h->err & 0x40) ? ODP_PACKET_CHKSUM_BAD : ODP_PACKET_CHKSUM_OK;
}

/* accessor for odp_cls_hash_result (odp_cls.c) */
int _odp_amd_packet_parse_info(odp_packet_t pkt, const uint8_t **data, uint64_t *in_flags,
			       uint32_t *l3, uint32_t *l4)
{
	pkt_hdr_t *h = rt_pkt_hdr(pkt);

	*data = h->head + h->data_off;
	*in_flags = h->in_flags;
	*l3 = h->l3;
	*l4 = h->l4;
	return 0;
}

void odp_packet_print_data(odp_packet_t pkt, uint32_t offset, uint32_t len)
{
	pkt_hdr_t *h = rt_pkt_hdr(pkt);
	const uint8_t *d = h->head + h->data_off;

	if ((uint64_t)offset + len > h->len) {
		printf("  bad offset or len\n");
		return;
	}
	printf("Packet data\n-----------\n  handle   0x%" PRIx64 "\n  offset   %u\n  length   %u\n",
	       odp_packet_to_u64(pkt), offset, len);
	for (uint32_t i = 0; i < len; i += 16) {
		printf(" ");
		for (uint32_t j = i; j < i + 16 && j < len; j++)
			printf(" %02x", d[offset + j]);
		printf("\n");
	}
}

void odp_packet_print(odp_packet_t pkt)
{
	pkt_hdr_t *h = rt_pkt_hdr(pkt);

	printf("Packet info\n-----------\n  handle         0x%" PRIx64 "\n  pool           %u\n"
	       "  input_flags    0x%" PRIx64 "\n  error_flags    0x%x\n  l2_offset      %u\n"
	       "  l3_offset      %u\n  l4_offset      %u\n  frame_len      %u\n  headroom       %u\n"
	       "  tailroom       %u\n  cos            %u\n", odp_packet_to_u64(pkt), h->ev.pool + 1,
	       h->in_flags, h->err, h->l2, h->l3, h->l4, h->len, h->data_off,
	       odp_packet_tailroom(pkt), h->cos);
}

/* ================================================================ events */
static ev_hdr_t *ev_hdr(odp_event_t ev)
{
	return (ev_hdr_t *)(void *)ev;
}

odp_event_type_t odp_event_type(odp_event_t ev) { return (odp_event_type_t)ev_hdr(ev)->type; }
odp_event_subtype_t odp_event_subtype(odp_event_t ev)
{
	return ev_hdr(ev)->type == ODP_EVENT_PACKET ? ODP_EVENT_PACKET_BASIC : ODP_EVENT_NO_SUBTYPE;
}

odp_event_type_t odp_event_types(odp_event_t ev, odp_event_subtype_t *subtype)
{
	if (subtype)
		*subtype = odp_event_subtype(ev);
	return odp_event_type(ev);
}

odp_pool_t odp_event_pool(odp_event_t ev) { return (odp_pool_t)(uintptr_t)(ev_hdr(ev)->pool + 1); }
uint64_t odp_event_to_u64(odp_event_t hdl) { return (uint64_t)(uintptr_t)hdl; }

int odp_event_is_valid(odp_event_t ev)
{
	if (ev == ODP_EVENT_INVALID)
		return 0;
	ev_hdr_t *e = ev_hdr(ev);

	return e->pool < RT_MAX_POOLS && RT.pool[e->pool].used;
}

void odp_event_free(odp_event_t ev)
{
	if (ev == ODP_EVENT_INVALID)
		return;
	pool_free(ev_hdr(ev));
}

void odp_event_free_multi(const odp_event_t ev[], int num)
{
	for (int i = 0; i < num; i++)
		odp_event_free(ev[i]);
}

/* event vectors (event_vector.h) */
odp_event_vector_t odp_event_vector_from_event(odp_event_t ev) { return (odp_event_vector_t)(void *)ev; }
odp_event_t odp_event_vector_to_event(odp_event_vector_t v) { return (odp_event_t)(void *)v; }
static evv_hdr_t *evv(odp_event_vector_t v) { return (evv_hdr_t *)(void *)v; }

odp_event_vector_t odp_event_vector_alloc(odp_pool_t pool)
{
	rt_pool_t *p = rt_pool(pool);
	ev_hdr_t *e;

	if (!p || (p->param.type != ODP_POOL_EVENT_VECTOR && p->param.type != ODP_POOL_VECTOR))
		return ODP_EVENT_VECTOR_INVALID;
	if (pool_alloc(p, &e, 1) != 1)
		return ODP_EVENT_VECTOR_INVALID;
	((evv_hdr_t *)e)->size = 0;
	return (odp_event_vector_t)(void *)e;
}

void odp_event_vector_free(odp_event_vector_t v)
{
	if (v != ODP_EVENT_VECTOR_INVALID)
		pool_free(&evv(v)->ev);
}

uint32_t odp_event_vector_tbl(odp_event_vector_t v, odp_event_t **tbl)
{
	*tbl = evv(v)->tbl;
	return evv(v)->size;
}

uint32_t odp_event_vector_size(odp_event_vector_t v) { return evv(v)->size; }
void odp_event_vector_size_set(odp_event_vector_t v, uint32_t size) { evv(v)->size = size; }
odp_pool_t odp_event_vector_pool(odp_event_vector_t v) { return (odp_pool_t)(uintptr_t)(evv(v)->ev.pool + 1); }

odp_event_type_t odp_event_vector_type(odp_event_vector_t v)
{
	evv_hdr_t *h = evv(v);

	if (h->size == 0)
		return ODP_EVENT_BUFFER;   /* undefined for an empty vector */
	odp_event_type_t t = odp_event_type(h->tbl[0]);

	for (uint32_t i = 1; i < h->size; i++)
		if (odp_event_type(h->tbl[i]) != t)
			return (odp_event_type_t)0;   /* ODP_EVENT_ANY */
	return t;
}

/* packet vectors (packet.h): event vectors of packets drawn from
 * ODP_POOL_VECTOR pools; odp_packet_t and odp_event_t share their handles, so
 * the vector's table serves both */
odp_packet_vector_t odp_packet_vector_from_event(odp_event_t ev) { return (odp_packet_vector_t)(void *)ev; }
odp_event_t odp_packet_vector_to_event(odp_packet_vector_t v) { return (odp_event_t)(void *)v; }

odp_packet_vector_t odp_packet_vector_alloc(odp_pool_t pool)
{
	rt_pool_t *p = rt_pool(pool);

	if (!p || p->param.type != ODP_POOL_VECTOR)
		return ODP_PACKET_VECTOR_INVALID;
	return (odp_packet_vector_t)(void *)odp_event_vector_alloc(pool);
}

void odp_packet_vector_free(odp_packet_vector_t v)
{
	odp_event_vector_free((odp_event_vector_t)(void *)v);
}

uint32_t odp_packet_vector_tbl(odp_packet_vector_t v, odp_packet_t **tbl)
{
	*tbl = (odp_packet_t *)(void *)evv((odp_event_vector_t)(void *)v)->tbl;
	return evv((odp_event_vector_t)(void *)v)->size;
}

uint32_t odp_packet_vector_size(odp_packet_vector_t v)
{
	return evv((odp_event_vector_t)(void *)v)->size;
}

void odp_packet_vector_size_set(odp_packet_vector_t v, uint32_t size)
{
	evv((odp_event_vector_t)(void *)v)->size = size;
}

odp_pool_t odp_packet_vector_pool(odp_packet_vector_t v)
{
	return odp_event_vector_pool((odp_event_vector_t)(void *)v);
}

int odp_packet_vector_valid(odp_packet_vector_t v)
{
	if (v == ODP_PACKET_VECTOR_INVALID)
		return 0;
	const ev_hdr_t *h = &evv((odp_event_vector_t)(void *)v)->ev;

	return h->type == ODP_EVENT_PACKET_VECTOR &&
	       evv((odp_event_vector_t)(void *)v)->size <= evv((odp_event_vector_t)(void *)v)->max_size;
}

/* ================================================================ queues */
static rt_queue_t *rtq(odp_queue_t h)
{
	return (rt_queue_t *)(void *)h;
}

/* a handle of a queue this runtime created (the classifier is also driven
 * with foreign queue handles by tests and applications of its C ABI) */
int rt_queue_is_valid(odp_queue_t h)
{
	const rt_queue_t *q = rtq(h);

	return q >= &RT.queue[0] && q < &RT.queue[RT_MAX_QUEUES] &&
	       ((uintptr_t)q - (uintptr_t)&RT.queue[0]) % sizeof(rt_queue_t) == 0 && q->used;
}

void odp_queue_param_init(odp_queue_param_t *p)
{
	memset(p, 0, sizeof(*p));
	p->type = ODP_QUEUE_TYPE_PLAIN;
	p->enq_mode = ODP_QUEUE_OP_MT;
	p->deq_mode = ODP_QUEUE_OP_MT;
	p->sched.prio = odp_schedule_default_prio();
	p->sched.sync = ODP_SCHED_SYNC_PARALLEL;
	p->sched.group = ODP_SCHED_GROUP_ALL;
	p->order = ODP_QUEUE_ORDER_KEEP;
	p->nonblocking = ODP_BLOCKING;
}

int odp_queue_capability(odp_queue_capability_t *capa)
{
	memset(capa, 0, sizeof(*capa));
	capa->max_queues = RT_MAX_QUEUES;
	capa->plain.max_num = RT_MAX_QUEUES;
	capa->plain.max_size = 0;   /* limited by memory only */
	return 0;
}

static rt_queue_t *queue_alloc(void)
{
	rt_queue_t *q = NULL;

	odp_spinlock_lock(&RT.lock);
	for (int i = 0; i < RT_MAX_QUEUES; i++)
		if (!RT.queue[i].used) {
			q = &RT.queue[i];
			memset(q, 0, sizeof(*q));
			q->used = 1;
			q->sched_slot = -1;
			break;
		}
	odp_spinlock_unlock(&RT.lock);
	return q;
}

static void sched_add(rt_queue_t *q)
{
	odp_spinlock_lock(&RT.sched_lock);
	q->sched_slot = RT.num_sched;
	RT.sched[RT.num_sched++] = q;
	odp_spinlock_unlock(&RT.sched_lock);
}

static void sched_remove(rt_queue_t *q)
{
	odp_spinlock_lock(&RT.sched_lock);
	if (q->sched_slot >= 0) {
		int s = q->sched_slot;

		RT.sched[s] = RT.sched[--RT.num_sched];
		RT.sched[s]->sched_slot = s;
		q->sched_slot = -1;
	}
	odp_spinlock_unlock(&RT.sched_lock);
}

odp_queue_t odp_queue_create(const char *name, const odp_queue_param_t *param)
{
	odp_queue_param_t def;

	if (!param) {
		odp_queue_param_init(&def);
		param = &def;
	}
	if (param->num_aggr > RT_MAX_AGGR) {
		RT_ERR("queue %s: num_aggr %u > %u\n", name ? name : "", param->num_aggr, RT_MAX_AGGR);
		return ODP_QUEUE_INVALID;
	}
	if (param->type == ODP_QUEUE_TYPE_SCHED &&
	    (param->sched.prio < odp_schedule_min_prio() || param->sched.prio > odp_schedule_max_prio())) {
		RT_ERR("queue %s: bad priority %d\n", name ? name : "", param->sched.prio);
		return ODP_QUEUE_INVALID;
	}
	rt_queue_t *q = queue_alloc();

	if (!q)
		return ODP_QUEUE_INVALID;
	snprintf(q->name, sizeof(q->name), "%s", name ? name : "");
	q->param = *param;
	q->param.aggr = NULL;
	q->context = param->context;
	odp_spinlock_init(&q->lock);
	q->cap = 256;
	q->ring = malloc(q->cap * sizeof(odp_event_t));
	if (!q->ring) {
		q->used = 0;
		return ODP_QUEUE_INVALID;
	}
	/* aggregator queues: enqueue-only front ends producing event vectors
	 * into this queue (queue_types.h num_aggr / aggr) */
	for (uint32_t i = 0; i < param->num_aggr; i++) {
		rt_queue_t *a = queue_alloc();

		if (!a || !param->aggr || !rt_pool(param->aggr[i].pool)) {
			if (a)
				a->used = 0;
			for (uint32_t j = 0; j < i; j++)
				q->aggr[j]->used = 0;
			free(q->ring);
			q->used = 0;
			RT_ERR("queue %s: bad aggregator config %u\n", q->name, i);
			return ODP_QUEUE_INVALID;
		}
		snprintf(a->name, sizeof(a->name), "%.24s_aggr%u", q->name, i);
		a->param.type = ODP_QUEUE_TYPE_PLAIN;
		a->is_aggr = 1;
		a->base = q;
		a->aggr_cfg = param->aggr[i];
		odp_spinlock_init(&a->lock);
		q->aggr[i] = a;
	}
	q->num_aggr = param->num_aggr;
	if (param->type == ODP_QUEUE_TYPE_SCHED)
		sched_add(q);
	return (odp_queue_t)(void *)q;
}

static void aggr_flush_locked(rt_queue_t *a);

int odp_queue_destroy(odp_queue_t h)
{
	rt_queue_t *q = rtq(h);

	if (!q || !q->used || q->is_aggr)
		return -1;
	for (uint32_t i = 0; i < q->num_aggr; i++) {
		rt_queue_t *a = q->aggr[i];

		if (a->cur_vec) {
			odp_event_vector_free((odp_event_vector_t)(void *)a->cur_vec);
			a->cur_vec = NULL;
		}
		a->used = 0;
	}
	if (q->count) {
		RT_ERR("queue %s destroyed with %u events\n", q->name, q->count);
	}
	sched_remove(q);
	odp_spinlock_lock(&q->lock);
	free(q->ring);
	q->ring = NULL;
	q->used = 0;
	odp_spinlock_unlock(&q->lock);
	return 0;
}

odp_queue_t odp_queue_lookup(const char *name)
{
	for (int i = 0; i < RT_MAX_QUEUES; i++)
		if (RT.queue[i].used && name && strcmp(RT.queue[i].name, name) == 0)
			return (odp_queue_t)(void *)&RT.queue[i];
	return ODP_QUEUE_INVALID;
}

odp_queue_t odp_queue_aggr(odp_queue_t h, uint32_t idx)
{
	rt_queue_t *q = rtq(h);

	if (!q || idx >= q->num_aggr)
		return ODP_QUEUE_INVALID;
	return (odp_queue_t)(void *)q->aggr[idx];
}

/* ring operations; caller holds q->lock */
static int ring_put(rt_queue_t *q, const odp_event_t ev[], int num)
{
	if (q->count + (uint32_t)num > q->cap) {
		uint32_t ncap = q->cap;

		while (ncap < q->count + (uint32_t)num)
			ncap *= 2;
		odp_event_t *nr = malloc(ncap * sizeof(odp_event_t));

		if (!nr)
			return -1;
		for (uint32_t i = 0; i < q->count; i++)
			nr[i] = q->ring[(q->head + i) % q->cap];
		free(q->ring);
		q->ring = nr;
		q->cap = ncap;
		q->head = 0;
	}
	for (int i = 0; i < num; i++)
		q->ring[(q->head + q->count + (uint32_t)i) % q->cap] = ev[i];
	q->count += (uint32_t)num;
	return num;
}

static int ring_get(rt_queue_t *q, odp_event_t ev[], int num)
{
	int n = (uint32_t)num < q->count ? num : (int)q->count;

	for (int i = 0; i < n; i++)
		ev[i] = q->ring[(q->head + (uint32_t)i) % q->cap];
	q->head = (q->head + (uint32_t)n) % q->cap;
	q->count -= (uint32_t)n;
	return n;
}

int rt_queue_enq_multi(rt_queue_t *q, const odp_event_t ev[], int num)
{
	int r;

	odp_spinlock_lock(&q->lock);
	r = q->used ? ring_put(q, ev, num) : -1;
	odp_spinlock_unlock(&q->lock);
	return r;
}

/* aggregator: close the current vector into the base queue; a->lock held */
static void aggr_flush_locked(rt_queue_t *a)
{
	if (!a->cur_vec)
		return;
	odp_event_t e = (odp_event_t)(void *)a->cur_vec;

	a->cur_vec = NULL;
	if (rt_queue_enq_multi(a->base, &e, 1) != 1)
		odp_event_free(e);
}

static int aggr_enq(rt_queue_t *a, const odp_event_t ev[], int num)
{
	int n = 0;

	odp_spinlock_lock(&a->lock);
	while (n < num) {
		if (!a->cur_vec) {
			odp_event_vector_t v = odp_event_vector_alloc(a->aggr_cfg.pool);

			if (v == ODP_EVENT_VECTOR_INVALID)
				break;
			a->cur_vec = evv(v);
			a->cur_t0 = now_ns();
		}
		evv_hdr_t *v = a->cur_vec;
		uint32_t lim = a->aggr_cfg.max_size && a->aggr_cfg.max_size < v->max_size ?
			       a->aggr_cfg.max_size : v->max_size;

		v->tbl[v->size++] = ev[n++];
		if (v->size >= lim)
			aggr_flush_locked(a);
	}
	odp_spinlock_unlock(&a->lock);
	return n;
}

/* close aggregation vectors older than max_tmo_ns (scheduler tick) */
static void aggr_timeouts(rt_queue_t *q)
{
	uint64_t t = 0;

	for (uint32_t i = 0; i < q->num_aggr; i++) {
		rt_queue_t *a = q->aggr[i];

		if (!__atomic_load_n(&a->cur_vec, __ATOMIC_RELAXED))
			continue;
		if (!t)
			t = now_ns();
		odp_spinlock_lock(&a->lock);
		if (a->cur_vec && t - a->cur_t0 >= a->aggr_cfg.max_tmo_ns)
			aggr_flush_locked(a);
		odp_spinlock_unlock(&a->lock);
	}
}

int odp_queue_enq_multi(odp_queue_t h, const odp_event_t ev[], int num)
{
	rt_queue_t *q = rtq(h);

	if (!q || num < 0)
		return -1;
	if (num == 0)
		return 0;
	if (q->is_aggr)
		return aggr_enq(q, ev, num);
	return rt_queue_enq_multi(q, ev, num);
}

int odp_queue_enq(odp_queue_t h, odp_event_t ev)
{
	return odp_queue_enq_multi(h, &ev, 1) == 1 ? 0 : -1;
}

int rt_queue_deq_multi_raw(rt_queue_t *q, odp_event_t ev[], int num)
{
	int r;

	odp_spinlock_lock(&q->lock);
	r = ring_get(q, ev, num);
	odp_spinlock_unlock(&q->lock);
	/* the caller reads every event's first header line next (type, pool):
	 * start all of those misses now (a packet's header was last written
	 * by the GPU receive delivery or another core) */
	for (int i = 0; i < r; i++)
		__builtin_prefetch((const void *)ev[i]);
	return r;
}

int odp_queue_deq_multi(odp_queue_t h, odp_event_t ev[], int num)
{
	rt_queue_t *q = rtq(h);

	if (!q || q->is_aggr || q->param.type != ODP_QUEUE_TYPE_PLAIN)
		return -1;
	if (q->num_aggr)
		aggr_timeouts(q);
	if (q->pktin_idx && __atomic_load_n(&q->count, __ATOMIC_RELAXED) == 0)
		rt_pktio_poll_index(q->pktin_idx - 1);   /* ODP_PKTIN_MODE_QUEUE */
	return rt_queue_deq_multi_raw(q, ev, num);
}

odp_event_t odp_queue_deq(odp_queue_t h)
{
	odp_event_t e;

	return odp_queue_deq_multi(h, &e, 1) == 1 ? e : ODP_EVENT_INVALID;
}

odp_queue_type_t odp_queue_type(odp_queue_t h)
{
	return rtq(h)->is_aggr ? ODP_QUEUE_TYPE_AGGR : rtq(h)->param.type;
}
odp_schedule_sync_t odp_queue_sched_type(odp_queue_t h) { return rtq(h)->param.sched.sync; }
odp_schedule_prio_t odp_queue_sched_prio(odp_queue_t h) { return rtq(h)->param.sched.prio; }
void *odp_queue_context(odp_queue_t h) { return rtq(h)->context; }
uint64_t odp_queue_to_u64(odp_queue_t h) { return (uint64_t)(uintptr_t)h; }

int odp_queue_context_set(odp_queue_t h, void *ctx, uint32_t len)
{
	(void)len;
	if (!h)
		return -1;
	rtq(h)->context = ctx;
	return 0;
}

int odp_queue_info(odp_queue_t h, odp_queue_info_t *info)
{
	rt_queue_t *q = rtq(h);

	if (!q || !q->used || !info)
		return -1;
	memset(info, 0, sizeof(*info));
	info->name = q->name;
	info->type = q->param.type;
	info->param = q->param;
	if (q->is_aggr)
		info->aggr_config = q->aggr_cfg;
	return 0;
}

static const char *sync_str(int s)
{
	return s == ODP_SCHED_SYNC_ATOMIC ? "atomic" : s == ODP_SCHED_SYNC_ORDERED ? "ordered" : "parallel";
}

void odp_queue_print(odp_queue_t h)
{
	rt_queue_t *q = rtq(h);

	if (!q || !q->used)
		return;
	printf("Queue info\n----------\n  handle          %p\n  name            %s\n"
	       "  type            %s\n  sync            %s\n  priority        %d\n"
	       "  num_aggr        %u\n  events          %u\n\n", (void *)q, q->name,
	       q->param.type == ODP_QUEUE_TYPE_SCHED ? "scheduled" : "plain",
	       sync_str(q->param.sched.sync), q->param.sched.prio, q->num_aggr, q->count);
}

void odp_queue_print_all(void)
{
	int n = 0;

	for (int i = 0; i < RT_MAX_QUEUES; i++)
		n += RT.queue[i].used && !RT.queue[i].is_aggr;
	printf("\nList of all queues\n------------------\n  Max queues: %d, current: %d\n"
	       "  idx %-32s type   sync     prio  events\n", RT_MAX_QUEUES, n, "name");
	for (int i = 0; i < RT_MAX_QUEUES; i++) {
		rt_queue_t *q = &RT.queue[i];

		if (!q->used || q->is_aggr)
			continue;
		printf("  %3i %-32s %-6s %-8s %4d  %u\n", i, q->name,
		       q->param.type == ODP_QUEUE_TYPE_SCHED ? "sched" : "plain",
		       q->param.type == ODP_QUEUE_TYPE_SCHED ? sync_str(q->param.sched.sync) : "-",
		       q->param.type == ODP_QUEUE_TYPE_SCHED ? q->param.sched.prio : 0, q->count);
	}
	printf("\n");
}

/* ================================================================ scheduler */
void odp_schedule_config_init(odp_schedule_config_t *c)
{
	memset(c, 0, sizeof(*c));
	c->num_queues = RT_MAX_QUEUES;
	c->queue_size = 0;
	c->sched_group.all = 1;
	c->sched_group.control = 1;
	c->sched_group.worker = 1;
}

int odp_schedule_config(const odp_schedule_config_t *c)
{
	(void)c;
	if (RT.sched_configured) {
		RT_ERR("scheduler already configured\n");
		return -1;
	}
	RT.sched_configured = 1;
	return 0;
}

int odp_schedule_min_prio(void) { return 0; }
int odp_schedule_max_prio(void) { return ODP_SCHED_MAX_PRIOS - 1; }
int odp_schedule_default_prio(void) { return (ODP_SCHED_MAX_PRIOS - 1) / 2; }
int odp_schedule_num_prio(void) { return ODP_SCHED_MAX_PRIOS; }
uint64_t odp_schedule_wait_time(uint64_t ns) { return ns; }
void odp_schedule_pause(void) { tls_paused = 1; }
void odp_schedule_resume(void) { tls_paused = 0; }
void odp_schedule_release_ordered(void) { odp_schedule_release_atomic(); }

void odp_schedule_release_atomic(void)
{
	rt_queue_t *q = tls_atomic;

	if (q) {
		__atomic_store_n(&q->owner, 0, __ATOMIC_RELEASE);
		tls_atomic = NULL;
	}
}

/* One pass over the scheduled queues: highest priority first, rotating start
 * within a priority level.  Returns events taken from a single queue. */
static int sched_try(odp_queue_t *from, odp_event_t ev[], int num)
{
	const int me = rt_thread_id() + 1;
	rt_queue_t *cand[RT_MAX_QUEUES];
	int n, best = -1;

	odp_spinlock_lock(&RT.sched_lock);
	n = RT.num_sched;
	memcpy(cand, RT.sched, (size_t)n * sizeof(cand[0]));
	odp_spinlock_unlock(&RT.sched_lock);
	if (n == 0)
		return 0;
	uint32_t start = tls_rr++;

	for (int prio = odp_schedule_max_prio(); prio >= odp_schedule_min_prio(); prio--) {
		for (int k = 0; k < n; k++) {
			rt_queue_t *q = cand[(start + (uint32_t)k) % (uint32_t)n];

			if (q->param.sched.prio != prio)
				continue;
			if (q->num_aggr)
				aggr_timeouts(q);
			if (__atomic_load_n(&q->count, __ATOMIC_RELAXED) == 0)
				continue;
			int sync = q->param.sched.sync;

			if (sync != ODP_SCHED_SYNC_PARALLEL) {
				int free_ = 0;

				if (!__atomic_compare_exchange_n(&q->owner, &free_, me, 0,
								 __ATOMIC_ACQUIRE, __ATOMIC_RELAXED))
					continue;
			}
			int got = rt_queue_deq_multi_raw(q, ev, num);

			if (got <= 0) {
				if (sync != ODP_SCHED_SYNC_PARALLEL)
					__atomic_store_n(&q->owner, 0, __ATOMIC_RELEASE);
				continue;
			}
			if (sync != ODP_SCHED_SYNC_PARALLEL)
				tls_atomic = q;
			if (from)
				*from = (odp_queue_t)(void *)q;
			best = got;
			return best;
		}
	}
	return 0;
}

static __thread uint64_t tls_last_poll;

int odp_schedule_multi(odp_queue_t *from, uint64_t wait, odp_event_t ev[], int num)
{
	uint64_t t_end = 0;
	int got;

	odp_schedule_release_atomic();
	if (num <= 0 || tls_paused)
		return 0;
	for (;;) {
		/* Queued events first; packet input (a GPU burst of up to 4096 frames
		 * into the CoS queues) when they are drained, or at least every
		 * millisecond so a busy event loop does not starve packet input.
		 * Polling on every call would pile bursts up faster than the
		 * application consumes them and run the pools dry. */
		uint64_t t0 = now_ns();

		got = sched_try(from, ev, num);
		if (got <= 0 || t0 - tls_last_poll > 1000000) {
			tls_last_poll = t0;
			rt_pktio_sched_poll();
			if (got <= 0)
				got = sched_try(from, ev, num);
		}
		if (got > 0)
			return got;
		if (wait == ODP_SCHED_NO_WAIT)
			return 0;
		uint64_t t = now_ns();

		if (!t_end)
			t_end = wait == ODP_SCHED_WAIT ? UINT64_MAX : t + wait;
		if (t >= t_end)
			return 0;
		odp_time_wait_ns(20 * ODP_TIME_USEC_IN_NS);
	}
}

odp_event_t odp_schedule(odp_queue_t *from, uint64_t wait)
{
	odp_event_t e;

	return odp_schedule_multi(from, wait, &e, 1) == 1 ? e : ODP_EVENT_INVALID;
}

int odp_schedule_multi_wait(odp_queue_t *from, odp_event_t ev[], int num)
{
	return odp_schedule_multi(from, ODP_SCHED_WAIT, ev, num);
}

int odp_schedule_multi_no_wait(odp_queue_t *from, odp_event_t ev[], int num)
{
	return odp_schedule_multi(from, ODP_SCHED_NO_WAIT, ev, num);
}
