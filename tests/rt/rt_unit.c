/*
 * rt_unit.c -- unit checks of the ODP runtime subset (no GPU): pools and
 * packets, queues (FIFO order, growth, info), the scheduler (priority order,
 * ATOMIC ownership, release), event aggregation into vectors (size and
 * timeout), cpumask, shm, time and the helper's parsers / threads.
 * Prints "ok <name>" / "FAIL <name>: why" lines; exit status 1 on failure.
 * Test infrastructure only.
 */
#define _GNU_SOURCE
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "odp/helper/odph_api.h"

static int fails;

#define CHECK(name, cond) do { \
	if (cond) printf("ok %s\n", name); \
	else { printf("FAIL %s: %s (line %d)\n", name, #cond, __LINE__); fails++; } \
} while (0)

static odp_pool_t pkt_pool(const char *name, uint32_t num, uint32_t len)
{
	odp_pool_param_t p;

	odp_pool_param_init(&p);
	p.type = ODP_POOL_PACKET;
	p.pkt.num = num;
	p.pkt.len = len;
	return odp_pool_create(name, &p);
}

static void t_pool_packet(void)
{
	odp_pool_t pool = pkt_pool("p", 8, 1500);
	odp_packet_t pk[10];
	int n = odp_packet_alloc_multi(pool, 100, pk, 10);

	CHECK("pool.alloc_limit", n == 8);
	CHECK("pool.lookup", odp_pool_lookup("p") == pool);
	CHECK("packet.len", odp_packet_len(pk[0]) == 100);
	CHECK("packet.headroom", odp_packet_headroom(pk[0]) == 128);
	CHECK("packet.pool", odp_packet_pool(pk[0]) == pool);
	CHECK("packet.event_type", odp_event_type(odp_packet_to_event(pk[0])) == ODP_EVENT_PACKET);
	uint8_t buf[100];

	for (int i = 0; i < 100; i++)
		buf[i] = (uint8_t)i;
	CHECK("packet.copy_from", odp_packet_copy_from_mem(pk[0], 0, 100, buf) == 0);
	CHECK("packet.copy_oob", odp_packet_copy_from_mem(pk[0], 50, 51, buf) < 0);
	odp_packet_t c = ODP_PACKET_INVALID;

	odp_packet_free(pk[7]);
	c = odp_packet_copy(pk[0], pool);
	CHECK("packet.copy", c != ODP_PACKET_INVALID &&
	      memcmp(odp_packet_data(c), buf, 100) == 0);
	CHECK("packet.push_head", odp_packet_push_head(pk[1], 14) != NULL && odp_packet_len(pk[1]) == 114);
	CHECK("packet.pull_tail", odp_packet_pull_tail(pk[1], 14) != NULL && odp_packet_len(pk[1]) == 100);
	CHECK("packet.no_parse", !odp_packet_has_eth(pk[0]) && !odp_packet_has_error(pk[0]) &&
	      odp_packet_l3_offset(pk[0]) == ODP_PACKET_OFFSET_INVALID);
	odp_packet_free(c);
	odp_packet_free_multi(pk, 7);
	CHECK("pool.realloc", odp_packet_alloc_multi(pool, 1500, pk, 10) == 8);
	CHECK("pool.too_long", odp_packet_alloc(pool, 70000) == ODP_PACKET_INVALID);
	odp_packet_free_multi(pk, 8);
	CHECK("pool.destroy", odp_pool_destroy(pool) == 0);
}

static odp_event_t mk_ev(odp_pool_t pool, uint8_t tag)
{
	odp_packet_t p = odp_packet_alloc(pool, 1);

	*(uint8_t *)odp_packet_data(p) = tag;
	return odp_packet_to_event(p);
}

static uint8_t tag_of(odp_event_t ev)
{
	return *(uint8_t *)odp_packet_data(odp_packet_from_event(ev));
}

static void t_queue(odp_pool_t pool)
{
	odp_queue_param_t qp;
	odp_queue_info_t info;

	odp_queue_param_init(&qp);
	odp_queue_t q = odp_queue_create("plainq", &qp);

	CHECK("queue.create", q != ODP_QUEUE_INVALID);
	CHECK("queue.info", odp_queue_info(q, &info) == 0 && strcmp(info.name, "plainq") == 0 &&
	      info.type == ODP_QUEUE_TYPE_PLAIN);
	/* FIFO across ring growth (initial capacity 256) */
	int ok = 1;

	for (int i = 0; i < 600; i++) {
		odp_event_t e = mk_ev(pool, (uint8_t)i);

		ok &= odp_queue_enq(q, e) == 0;
	}
	for (int i = 0; i < 600; i++) {
		odp_event_t e = odp_queue_deq(q);

		ok &= e != ODP_EVENT_INVALID && tag_of(e) == (uint8_t)i;
		odp_event_free(e);
	}
	CHECK("queue.fifo_growth", ok);
	CHECK("queue.empty", odp_queue_deq(q) == ODP_EVENT_INVALID);
	CHECK("queue.lookup", odp_queue_lookup("plainq") == q);
	CHECK("queue.destroy", odp_queue_destroy(q) == 0);
}

static void t_sched(odp_pool_t pool)
{
	odp_queue_param_t qp;
	odp_queue_t lo, hi, at;
	odp_event_t ev[8];
	odp_queue_t from;

	odp_queue_param_init(&qp);
	qp.type = ODP_QUEUE_TYPE_SCHED;
	qp.sched.prio = odp_schedule_min_prio();
	lo = odp_queue_create("lo", &qp);
	qp.sched.prio = odp_schedule_max_prio();
	hi = odp_queue_create("hi", &qp);
	qp.sched.prio = odp_schedule_default_prio();
	qp.sched.sync = ODP_SCHED_SYNC_ATOMIC;
	at = odp_queue_create("at", &qp);
	odp_queue_enq(lo, mk_ev(pool, 1));
	odp_queue_enq(hi, mk_ev(pool, 2));
	odp_queue_enq(at, mk_ev(pool, 3));
	odp_queue_enq(at, mk_ev(pool, 4));
	int n = odp_schedule_multi(&from, ODP_SCHED_NO_WAIT, ev, 8);

	CHECK("sched.prio_first", n == 1 && from == hi && tag_of(ev[0]) == 2);
	odp_event_free(ev[0]);
	n = odp_schedule_multi(&from, ODP_SCHED_NO_WAIT, ev, 1);
	CHECK("sched.prio_second", n == 1 && from == at && tag_of(ev[0]) == 3);
	odp_event_free(ev[0]);
	n = odp_schedule_multi(&from, ODP_SCHED_NO_WAIT, ev, 8);
	CHECK("sched.atomic_fifo", n == 1 && from == at && tag_of(ev[0]) == 4);
	odp_event_free(ev[0]);
	n = odp_schedule_multi(&from, ODP_SCHED_NO_WAIT, ev, 8);
	CHECK("sched.prio_last", n == 1 && from == lo);
	odp_event_free(ev[0]);
	odp_time_t t0 = odp_time_local();

	n = odp_schedule_multi(&from, odp_schedule_wait_time(20 * ODP_TIME_MSEC_IN_NS), ev, 8);
	uint64_t dt = odp_time_diff_ns(odp_time_local(), t0);

	CHECK("sched.wait_timeout", n == 0 && dt >= 20 * ODP_TIME_MSEC_IN_NS);
	odp_queue_destroy(lo);
	odp_queue_destroy(hi);
	odp_queue_destroy(at);
}

/* atomic ownership: a second thread cannot take events of a queue the first
 * thread holds until it calls schedule again (or releases) */
static odp_queue_t g_atq;
static int g_got;

static int other_thread(void *arg)
{
	odp_event_t ev;
	odp_queue_t from;

	(void)arg;
	g_got = odp_schedule_multi(&from, ODP_SCHED_NO_WAIT, &ev, 1);
	if (g_got > 0)
		odp_event_free(ev);
	return 0;
}

static void t_atomic(odp_instance_t inst, odp_pool_t pool)
{
	odp_queue_param_t qp;
	odp_event_t ev;
	odp_queue_t from;
	odph_thread_t thr;
	odph_thread_common_param_t cp;
	odph_thread_param_t tp;

	odp_queue_param_init(&qp);
	qp.type = ODP_QUEUE_TYPE_SCHED;
	qp.sched.sync = ODP_SCHED_SYNC_ATOMIC;
	g_atq = odp_queue_create("atomic2", &qp);
	odp_queue_enq(g_atq, mk_ev(pool, 1));
	odp_queue_enq(g_atq, mk_ev(pool, 2));
	CHECK("atomic.take", odp_schedule_multi(&from, ODP_SCHED_NO_WAIT, &ev, 1) == 1);
	odp_event_free(ev);
	odph_thread_common_param_init(&cp);
	odph_thread_param_init(&tp);
	cp.instance = inst;
	tp.start = other_thread;
	tp.thr_type = ODP_THREAD_WORKER;
	CHECK("thread.create", odph_thread_create(&thr, &cp, &tp, 1) == 1);
	CHECK("thread.join", odph_thread_join(&thr, 1) == 1);
	CHECK("atomic.held", g_got == 0);
	odp_schedule_release_atomic();
	CHECK("thread.create2", odph_thread_create(&thr, &cp, &tp, 1) == 1);
	odph_thread_join(&thr, 1);
	CHECK("atomic.released", g_got == 1);
	odp_queue_destroy(g_atq);
}

static void t_aggr(odp_pool_t pool)
{
	odp_pool_param_t vp;
	odp_queue_param_t qp;
	odp_event_aggr_config_t ac;
	odp_event_t ev[4];
	odp_queue_t from;

	odp_pool_param_init(&vp);
	vp.type = ODP_POOL_EVENT_VECTOR;
	vp.event_vector.num = 8;
	vp.event_vector.max_size = 4;
	odp_pool_t vpool = odp_pool_create("vec", &vp);

	odp_queue_param_init(&qp);
	qp.type = ODP_QUEUE_TYPE_SCHED;
	memset(&ac, 0, sizeof(ac));
	ac.pool = vpool;
	ac.max_size = 3;
	ac.max_tmo_ns = 5 * ODP_TIME_MSEC_IN_NS;
	ac.event_type = ODP_EVENT_PACKET;
	qp.num_aggr = 1;
	qp.aggr = &ac;
	odp_queue_t q = odp_queue_create("aggq", &qp);
	odp_queue_t a = odp_queue_aggr(q, 0);

	CHECK("aggr.handle", a != ODP_QUEUE_INVALID && odp_queue_aggr(q, 1) == ODP_QUEUE_INVALID);
	for (int i = 0; i < 4; i++)
		odp_queue_enq(a, mk_ev(pool, (uint8_t)(10 + i)));
	int n = odp_schedule_multi(&from, ODP_SCHED_NO_WAIT, ev, 4);
	int ok = n == 1 && odp_event_type(ev[0]) == ODP_EVENT_VECTOR;

	if (ok) {
		odp_event_vector_t v = odp_event_vector_from_event(ev[0]);
		odp_event_t *tbl;
		uint32_t sz = odp_event_vector_tbl(v, &tbl);

		ok = sz == 3 && tag_of(tbl[0]) == 10 && tag_of(tbl[2]) == 12;
		odp_event_free_multi(tbl, (int)sz);
		odp_event_vector_free(v);
	}
	CHECK("aggr.full_vector", ok);
	/* the 4th event is flushed by the timeout */
	n = odp_schedule_multi(&from, odp_schedule_wait_time(50 * ODP_TIME_MSEC_IN_NS), ev, 4);
	ok = n == 1 && odp_event_type(ev[0]) == ODP_EVENT_VECTOR;
	if (ok) {
		odp_event_vector_t v = odp_event_vector_from_event(ev[0]);
		odp_event_t *tbl;

		ok = odp_event_vector_tbl(v, &tbl) == 1 && tag_of(tbl[0]) == 13;
		odp_event_free(tbl[0]);
		odp_event_vector_free(v);
	}
	CHECK("aggr.timeout_flush", ok);
	odp_queue_destroy(q);
	odp_pool_destroy(vpool);
}

static void t_misc(void)
{
	odp_cpumask_t m;
	char s[ODP_CPUMASK_STR_SIZE];
	uint32_t ip;
	odph_ethaddr_t mac;

	odp_cpumask_zero(&m);
	odp_cpumask_set(&m, 1);
	odp_cpumask_set(&m, 5);
	odp_cpumask_to_str(&m, s, sizeof(s));
	CHECK("cpumask.str", strcmp(s, "0x22") == 0);
	CHECK("cpumask.count", odp_cpumask_count(&m) == 2 && odp_cpumask_first(&m) == 1 &&
	      odp_cpumask_next(&m, 1) == 5 && odp_cpumask_last(&m) == 5);
	odp_cpumask_from_str(&m, "0x5");
	CHECK("cpumask.from_str", odp_cpumask_isset(&m, 0) && odp_cpumask_isset(&m, 2) &&
	      odp_cpumask_count(&m) == 2);
	int w = odp_cpumask_default_worker(&m, 0);

	CHECK("cpumask.default_worker", w >= 1 && odp_cpumask_count(&m) == w);
	CHECK("helper.ipv4", odph_ipv4_addr_parse(&ip, "10.10.10.0") == 0 && ip == 0x0a0a0a00u);
	CHECK("helper.ipv4_bad", odph_ipv4_addr_parse(&ip, "10.10.300.0") != 0 &&
	      odph_ipv4_addr_parse(&ip, "10.10") != 0);
	CHECK("helper.mac", odph_eth_addr_parse(&mac, "11:22:33:44:55:66") == 0 &&
	      mac.addr[0] == 0x11 && mac.addr[5] == 0x66);
	CHECK("helper.mac_bad", odph_eth_addr_parse(&mac, "11:22:33") != 0);
	odp_shm_t shm = odp_shm_reserve("blk", 1000, 256, 0);

	CHECK("shm.reserve", shm != ODP_SHM_INVALID && ((uintptr_t)odp_shm_addr(shm) & 255) == 0);
	CHECK("shm.lookup", odp_shm_lookup("blk") == shm);
	CHECK("shm.free", odp_shm_free(shm) == 0 && odp_shm_addr(shm) == NULL);
	odp_time_t t0 = odp_time_local();

	odp_time_wait_ns(2 * ODP_TIME_MSEC_IN_NS);
	CHECK("time.diff", odp_time_diff_ns(odp_time_local(), t0) >= 2 * ODP_TIME_MSEC_IN_NS);
	CHECK("byteorder", odp_cpu_to_be_16(0x1234) == 0x3412 &&
	      odp_be_to_cpu_32(0x11223344) == 0x44332211u);
}

/* packet vectors (packet.h) and CoS vector parameter validation
 * (odp_cls_cos_create, odp_classification.c:256-288) */
static void t_vectors(odp_pool_t pool)
{
	odp_pool_param_t vp;

	odp_pool_param_init(&vp);
	vp.type = ODP_POOL_VECTOR;
	vp.vector.num = 2;
	vp.vector.max_size = 8;
	odp_pool_t vpool = odp_pool_create("pktv", &vp);
	odp_packet_vector_t v1 = odp_packet_vector_alloc(vpool), v2 = odp_packet_vector_alloc(vpool);

	CHECK("pktv.alloc", v1 != ODP_PACKET_VECTOR_INVALID && v2 != ODP_PACKET_VECTOR_INVALID);
	CHECK("pktv.exhausted", odp_packet_vector_alloc(vpool) == ODP_PACKET_VECTOR_INVALID);
	CHECK("pktv.event_type",
	      odp_event_type(odp_packet_vector_to_event(v1)) == ODP_EVENT_PACKET_VECTOR);
	CHECK("pktv.from_event",
	      odp_packet_vector_from_event(odp_packet_vector_to_event(v1)) == v1);
	odp_packet_t *tbl;

	CHECK("pktv.empty", odp_packet_vector_tbl(v1, &tbl) == 0 && odp_packet_vector_valid(v1));
	tbl[0] = odp_packet_alloc(pool, 60);
	tbl[1] = odp_packet_alloc(pool, 60);
	odp_packet_vector_size_set(v1, 2);
	CHECK("pktv.size", odp_packet_vector_size(v1) == 2 && odp_packet_vector_pool(v1) == vpool);
	odp_packet_free_multi(tbl, 2);
	odp_packet_vector_free(v1);
	odp_packet_vector_free(v2);
	/* a packet pool is no vector pool */
	CHECK("pktv.wrong_pool", odp_packet_vector_alloc(pool) == ODP_PACKET_VECTOR_INVALID);

	/* CoS vector parameters */
	odp_queue_param_t qp;
	odp_cls_cos_param_t cp;

	odp_queue_param_init(&qp);
	qp.type = ODP_QUEUE_TYPE_SCHED;
	odp_queue_t q = odp_queue_create("vq", &qp);

	odp_cls_cos_param_init(&cp);
	cp.queue = q;
	cp.vector.enable = true;
	cp.vector.pool = ODP_POOL_INVALID;
	cp.vector.max_size = 4;
	CHECK("cosv.no_pool", odp_cls_cos_create("v0", &cp) == ODP_COS_INVALID);
	cp.vector.pool = pool;
	CHECK("cosv.wrong_pool_type", odp_cls_cos_create("v1", &cp) == ODP_COS_INVALID);
	cp.vector.pool = vpool;
	cp.vector.max_size = 0;
	CHECK("cosv.max_size_zero", odp_cls_cos_create("v2", &cp) == ODP_COS_INVALID);
	cp.vector.max_size = 9;
	CHECK("cosv.max_size_above_pool", odp_cls_cos_create("v3", &cp) == ODP_COS_INVALID);
	cp.vector.max_size = 8;
	odp_cos_t ok = odp_cls_cos_create("v4", &cp);

	CHECK("cosv.ok", ok != ODP_COS_INVALID);
	odp_cos_destroy(ok);
	/* packet vectors together with event aggregation (hash queues with
	 * aggregators) */
	odp_pool_param_t ep;
	odp_event_aggr_config_t ac;

	odp_pool_param_init(&ep);
	ep.type = ODP_POOL_EVENT_VECTOR;
	ep.event_vector.num = 4;
	ep.event_vector.max_size = 4;
	memset(&ac, 0, sizeof(ac));
	ac.pool = odp_pool_create("evq", &ep);
	ac.max_size = 4;
	ac.event_type = ODP_EVENT_PACKET;
	odp_cls_cos_param_init(&cp);
	cp.num_queue = 4;
	cp.queue_param = qp;
	cp.queue_param.num_aggr = 1;
	cp.queue_param.aggr = &ac;
	cp.vector.enable = true;
	cp.vector.pool = vpool;
	cp.vector.max_size = 4;
	CHECK("cosv.pktv_and_aggr", odp_cls_cos_create("v5", &cp) == ODP_COS_INVALID);
	cp.vector.enable = false;
	ok = odp_cls_cos_create("v6", &cp);
	CHECK("cosv.aggr_hash_queues", ok != ODP_COS_INVALID);
	odp_cos_destroy(ok);
	odp_queue_destroy(q);
	odp_pool_destroy(vpool);
	odp_pool_destroy(ac.pool);
}

int main(int argc, char *argv[])
{
	odp_instance_t inst;

	argc = odph_parse_options(argc, argv);
	(void)argc;
	if (odp_init_global(&inst, NULL, NULL) || odp_init_local(inst, ODP_THREAD_CONTROL)) {
		printf("FAIL init\n");
		return 1;
	}
	CHECK("thread.id", odp_thread_id() == 0);
	odp_schedule_config(NULL);
	t_pool_packet();
	odp_pool_t pool = pkt_pool("evpool", 2048, 64);

	t_queue(pool);
	t_sched(pool);
	t_atomic(inst, pool);
	t_aggr(pool);
	t_vectors(pool);
	t_misc();
	odp_pool_destroy(pool);
	odp_term_local();
	odp_term_global(inst);
	return fails ? 1 : 0;
}
