/*
 * rx_driver.c -- test driver for the ODP runtime + GPU receive path.
 *
 * Replays a rule program (text form of odp_amd.rules programs, written by
 * tests/rt_helpers.py) through the odp_cls_* API, opens a pktio, runs the
 * receive path and prints every packet that reaches a queue, in arrival
 * order per queue, with its metadata.  tests/test_runtime*.py compare the
 * output against the CPU oracle.  Test infrastructure only.
 *
 * usage: rx_driver <pktio> <rules|-> <sched|direct|queue> <layer 0-4>
 *                  <cos_pools 0|1> <cls 0|1> [source pcap for loop]
 *   <pktio> = "pcap:in=FILE..." or "loop" (then the frames of the source
 *   pcap are read through a second, parse-less pcap pktio and sent into the
 *   loop interface).
 * environment: RX_PKTV=<max_size>,<vectors>  every enqueue CoS delivers packet
 *   vectors (cls_cos_param.vector) from a vector pool of that size;
 *   RX_AGGR=<max_size>  hash-queue CoS get one event aggregator per queue
 *   (queue_param.num_aggr), so their runs go to odp_queue_aggr(q, 0).
 * output lines:
 *   V <queue> <size> / E <queue> <size>   a packet / event vector; its
 *                                         packets follow as P lines
 *   P <queue> <pool> <in_flags> <err> <l3> <l4> <cos> <mark> <hex frame>
 *   S <in_packets> <in_errors> <in_discards> <in_octets>
 *   Q <cos> <slot> <packets> <discards>     (odp_cls_queue_stats)
 * RX_COUNT_ONLY=1: no P lines; "R <packets delivered> <ns>" (receive-path
 *   rate, bench.py's runtime e2e: from odp_pktio_start to the last packet).
 * RX_SWITCH_RULES=<rules file> (direct mode): replayed after the first
 *   odp_pktin_recv call (RX_SWITCH_AFTER=k: after the k-th), while earlier
 *   bursts are still in flight on the GPU -- classification or delivery
 *   (control-plane change between two receive calls).
 */
#define _GNU_SOURCE
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "odp_api.h"

#define MAX_COS 256
#define MAX_PMR 8192

static odp_cos_t cos_h[MAX_COS];
static odp_queue_t cos_q[MAX_COS];
static odp_pool_t cos_pool[MAX_COS];
static char cos_name[MAX_COS][ODP_COS_NAME_LEN];
static int ncos;
static odp_pmr_t pmr_h[MAX_PMR];
static int npmr;
static odp_pool_t pktv_pool = ODP_POOL_INVALID, evv_pool = ODP_POOL_INVALID;
static uint32_t pktv_max, aggr_max;
static odp_event_aggr_config_t aggr_cfg;

static int hexval(char c)
{
	return c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : -1;
}

static int unhex(const char *s, uint8_t *out, int max)
{
	int n = 0;

	if (strcmp(s, "-") == 0)
		return 0;
	while (s[0] && s[1] && n < max) {
		out[n++] = (uint8_t)(hexval(s[0]) << 4 | hexval(s[1]));
		s += 2;
	}
	return n;
}

static odp_pool_t mkpool(const char *name)
{
	odp_pool_param_t p;

	odp_pool_param_init(&p);
	p.type = ODP_POOL_PACKET;
	p.pkt.len = 1856;
	/* RX_SEG_LEN: a first-segment length below the frame sizes (the
	 * runtime still keeps every packet in one segment, seg_len being the
	 * minimum the spec asks for) */
	p.pkt.seg_len = getenv("RX_SEG_LEN") ? (uint32_t)atoi(getenv("RX_SEG_LEN")) : 1856;
	/* RX_POOL_NUM: packets per pool (rate runs hold a whole capture) */
	p.pkt.num = getenv("RX_POOL_NUM") ? (uint32_t)atoi(getenv("RX_POOL_NUM")) : 20000;
	return odp_pool_create(name, &p);
}

static int replay(FILE *f, odp_pktio_t pktio, int cos_pools)
{
	char line[65536];

	while (fgets(line, sizeof(line), f)) {
		char *save = NULL, *tok = strtok_r(line, " \n", &save);

		if (!tok)
			continue;
		if (strcmp(tok, "cos") == 0) {
			/* cos <name> <action> <num_queue> <hash_proto> <stats> */
			char *name = strtok_r(NULL, " \n", &save);
			int action = atoi(strtok_r(NULL, " \n", &save));
			int nq = atoi(strtok_r(NULL, " \n", &save));
			unsigned hp = (unsigned)strtoul(strtok_r(NULL, " \n", &save), NULL, 0);
			int stats = atoi(strtok_r(NULL, " \n", &save));
			odp_cls_cos_param_t cp;
			odp_queue_param_t qp;

			odp_cls_cos_param_init(&cp);
			odp_queue_param_init(&qp);
			qp.type = ODP_QUEUE_TYPE_SCHED;
			cp.action = action ? ODP_COS_ACTION_DROP : ODP_COS_ACTION_ENQUEUE;
			cp.stats_enable = stats;
			cp.num_queue = (uint32_t)nq;
			snprintf(cos_name[ncos], ODP_COS_NAME_LEN, "%s", name);
			if (!action) {
				if (pktv_pool != ODP_POOL_INVALID) {
					cp.vector.enable = true;
					cp.vector.pool = pktv_pool;
					cp.vector.max_size = pktv_max;
				}
				if (nq > 1) {
					if (evv_pool != ODP_POOL_INVALID) {
						qp.num_aggr = 1;
						qp.aggr = &aggr_cfg;
					}
					cp.queue_param = qp;
					cp.hash_proto.all_bits = hp;
				} else {
					cos_q[ncos] = odp_queue_create(name, &qp);
					cp.queue = cos_q[ncos];
				}
				if (cos_pools) {
					char pn[ODP_POOL_NAME_LEN];

					snprintf(pn, sizeof(pn), "%.24sPool", name);
					cos_pool[ncos] = mkpool(pn);
					cp.pool = cos_pool[ncos];
				}
			}
			cos_h[ncos++] = odp_cls_cos_create(name, &cp);
		} else if (strcmp(tok, "pmr") == 0) {
			/* pmr <src> <dst> <mark> <nterms> {<term> <val> <mask> <offset>} */
			int src = atoi(strtok_r(NULL, " \n", &save));
			int dst = atoi(strtok_r(NULL, " \n", &save));
			uint64_t mark = strtoull(strtok_r(NULL, " \n", &save), NULL, 0);
			int nt = atoi(strtok_r(NULL, " \n", &save));
			odp_pmr_param_t t[8];
			uint8_t val[8][16], msk[8][16];
			odp_pmr_create_opt_t opt;

			for (int i = 0; i < nt && i < 8; i++) {
				odp_cls_pmr_param_init(&t[i]);
				t[i].term = (odp_cls_pmr_term_t)atoi(strtok_r(NULL, " \n", &save));
				t[i].val_sz = (uint32_t)unhex(strtok_r(NULL, " \n", &save), val[i], 16);
				unhex(strtok_r(NULL, " \n", &save), msk[i], 16);
				t[i].offset = (uint32_t)atoi(strtok_r(NULL, " \n", &save));
				t[i].match.value = val[i];
				t[i].match.mask = msk[i];
			}
			odp_cls_pmr_create_opt_init(&opt);
			opt.terms = t;
			opt.num_terms = nt;
			opt.mark = mark;
			pmr_h[npmr++] = odp_cls_pmr_create_opt(&opt, cos_h[src], cos_h[dst]);
		} else if (strcmp(tok, "pmr_destroy") == 0) {
			odp_cls_pmr_destroy(pmr_h[atoi(strtok_r(NULL, " \n", &save))]);
		} else if (strcmp(tok, "cos_destroy") == 0) {
			odp_cos_destroy(cos_h[atoi(strtok_r(NULL, " \n", &save))]);
		} else if (strcmp(tok, "default") == 0 || strcmp(tok, "error") == 0) {
			int i = atoi(strtok_r(NULL, " \n", &save));
			odp_cos_t c = i < 0 ? ODP_COS_INVALID : cos_h[i];

			if (tok[0] == 'd')
				odp_pktio_default_cos_set(pktio, c);
			else
				odp_pktio_error_cos_set(pktio, c);
		}
	}
	return 0;
}

static const char *qname(odp_queue_t q)
{
	odp_queue_info_t info;

	return odp_queue_info(q, &info) == 0 ? info.name : "?";
}

static const char *poolname(odp_pool_t p)
{
	odp_pool_info_t info;

	return odp_pool_info(p, &info) == 0 ? info.name : "?";
}

static void print_pkt(const char *q, odp_packet_t pkt);

/* one received event: a packet, or a packet / event vector of packets */
static void print_ev(const char *q, odp_event_t ev)
{
	if (odp_event_type(ev) == ODP_EVENT_PACKET_VECTOR) {
		odp_packet_vector_t v = odp_packet_vector_from_event(ev);
		odp_packet_t *tbl;
		uint32_t n = odp_packet_vector_tbl(v, &tbl);

		printf("V %s %u\n", q, n);
		for (uint32_t i = 0; i < n; i++) {
			print_pkt(q, tbl[i]);
			odp_packet_free(tbl[i]);
		}
		odp_packet_vector_free(v);
		return;
	}
	if (odp_event_type(ev) == ODP_EVENT_VECTOR) {
		odp_event_vector_t v = odp_event_vector_from_event(ev);
		odp_event_t *tbl;
		uint32_t n = odp_event_vector_tbl(v, &tbl);

		printf("E %s %u\n", q, n);
		for (uint32_t i = 0; i < n; i++) {
			print_pkt(q, odp_packet_from_event(tbl[i]));
			odp_event_free(tbl[i]);
		}
		odp_event_vector_free(v);
		return;
	}
	print_pkt(q, odp_packet_from_event(ev));
	odp_event_free(ev);
}

static int count_only;
static uint64_t delivered, recv_ns, drain_ns;

static void print_pkt(const char *q, odp_packet_t pkt)
{
	if (count_only) {
		delivered++;
		return;
	}
	uint32_t len = odp_packet_len(pkt);
	const uint8_t *d = odp_packet_data(pkt);
	uint64_t fl = 0;

	/* reassemble the input_flags word from the packet_flags.h accessors */
	static int (*const fn[])(odp_packet_t) = {
		NULL, odp_packet_has_flow_hash, odp_packet_has_ts, odp_packet_has_l2,
		odp_packet_has_l3, odp_packet_has_l4, odp_packet_has_eth, odp_packet_has_eth_bcast,
		odp_packet_has_eth_mcast, odp_packet_has_jumbo, odp_packet_has_vlan,
		odp_packet_has_vlan_qinq, odp_packet_has_arp, odp_packet_has_ipv4,
		odp_packet_has_ipv6, odp_packet_has_ip_bcast, odp_packet_has_ip_mcast,
		odp_packet_has_ipfrag, odp_packet_has_ipopt, odp_packet_has_ipsec, NULL, NULL,
		odp_packet_has_udp, odp_packet_has_tcp, odp_packet_has_sctp, odp_packet_has_icmp };
	for (unsigned b = 0; b < sizeof(fn) / sizeof(fn[0]); b++)
		if (fn[b] && fn[b](pkt))
			fl |= 1ull << b;
	/* checksum statuses (0 unknown, 1 bad, 2 ok) in bits 40-41 / 42-43 */
	fl |= (uint64_t)odp_packet_l3_chksum_status(pkt) << 40;
	fl |= (uint64_t)odp_packet_l4_chksum_status(pkt) << 42;
	if (odp_packet_num_segs(pkt) != 1 || odp_packet_seg_len(pkt) != len)
		printf("SEGMENTED %s\n", q);   /* never expected: tests fail on it */
	printf("P %s %s %" PRIx64 " %d %u %u %" PRIu64 " %u ", q, poolname(odp_packet_pool(pkt)), fl,
	       odp_packet_has_error(pkt), odp_packet_l3_offset(pkt), odp_packet_l4_offset(pkt),
	       odp_packet_cls_mark(pkt), len);
	for (uint32_t i = 0; i < len; i++)
		printf("%02x", d[i]);
	printf("\n");
}

/* Send the source capture's frames into the loop interface through a
 * parse-less pcap pktio (the loop "wire"); returns the frames sent. */
static long feed_loop(const char *src_pcap, odp_pool_t pool, odp_pktio_t pktio)
{
	char src[512];
	odp_pktio_param_t sp;
	odp_pktio_config_t sc;
	odp_pktin_queue_t inq;
	odp_pktout_queue_t outq;
	odp_packet_t pk[256];
	int n;
	long sent = 0;

	snprintf(src, sizeof(src), "pcap:in=%s", src_pcap);
	odp_pktio_param_init(&sp);
	odp_pktio_t sio = odp_pktio_open(src, pool, &sp);

	if (sio == ODP_PKTIO_INVALID || odp_pktin_queue_config(sio, NULL))
		return -1;
	odp_pktio_promisc_mode_set(sio, 1);
	odp_pktio_config_init(&sc);
	sc.parser.layer = ODP_PROTO_LAYER_NONE;
	odp_pktio_config(sio, &sc);
	if (odp_pktio_start(sio) || odp_pktin_queue(sio, &inq, 1) != 1 ||
	    odp_pktout_queue(pktio, &outq, 1) < 1)
		return -1;
	while ((n = odp_pktin_recv(inq, pk, 256)) > 0) {
		if (odp_pktout_send(outq, pk, n) != n)
			return -1;
		sent += n;
	}
	odp_pktio_stop(sio);
	odp_pktio_close(sio);
	return sent;
}

int main(int argc, char *argv[])
{
	odp_instance_t inst;
	odp_pktio_param_t pp;
	odp_pktin_queue_param_t iq;
	odp_pktout_queue_param_t oq;
	odp_pktio_config_t cfg;
	const char *mode;
	int layer, cos_pools, cls;

	if (argc < 7) {
		fprintf(stderr, "usage: %s <pktio> <rules|-> <sched|direct|queue> <layer> "
			"<cos_pools> <cls> [source pcap]\n", argv[0]);
		return 2;
	}
	mode = argv[3];
	layer = atoi(argv[4]);
	cos_pools = atoi(argv[5]);
	cls = atoi(argv[6]);
	if (odp_init_global(&inst, NULL, NULL) || odp_init_local(inst, ODP_THREAD_CONTROL))
		return 3;
	odp_schedule_config(NULL);
	odp_pool_t pool = mkpool("pktio_pool");
	/* RX_HOLD_PKTIO_POOL=1: every packet of the pktio's pool is held by the
	 * application for the run (classified frames then need CoS pools) */
	odp_packet_t *held = NULL;
	int nheld = 0;

	if (getenv("RX_HOLD_PKTIO_POOL")) {
		held = malloc(sizeof(odp_packet_t) * 1048576);
		odp_packet_t pk;

		while (held && nheld < 1048576 && (pk = odp_packet_alloc(pool, 64)) != ODP_PACKET_INVALID)
			held[nheld++] = pk;
	}

	if (getenv("RX_PKTV")) {
		odp_pool_param_t vp;
		unsigned mx = 0, num = 0;

		sscanf(getenv("RX_PKTV"), "%u,%u", &mx, &num);
		odp_pool_param_init(&vp);
		vp.type = ODP_POOL_VECTOR;
		vp.vector.num = num;
		vp.vector.max_size = mx;
		pktv_pool = odp_pool_create("pktv_pool", &vp);
		pktv_max = mx;
		if (pktv_pool == ODP_POOL_INVALID)
			return 12;
	}
	if (getenv("RX_AGGR")) {
		odp_pool_param_t vp;

		aggr_max = (uint32_t)atoi(getenv("RX_AGGR"));
		odp_pool_param_init(&vp);
		vp.type = ODP_POOL_EVENT_VECTOR;
		vp.event_vector.num = 20000;
		vp.event_vector.max_size = aggr_max;
		evv_pool = odp_pool_create("evv_pool", &vp);
		if (evv_pool == ODP_POOL_INVALID)
			return 13;
		memset(&aggr_cfg, 0, sizeof(aggr_cfg));
		aggr_cfg.pool = evv_pool;
		aggr_cfg.max_size = aggr_max;
		aggr_cfg.max_tmo_ns = 1000;
		aggr_cfg.event_type = ODP_EVENT_PACKET;
	}

	odp_pktio_param_init(&pp);
	pp.in_mode = strcmp(mode, "sched") == 0 ? ODP_PKTIN_MODE_SCHED :
		     strcmp(mode, "queue") == 0 ? ODP_PKTIN_MODE_QUEUE : ODP_PKTIN_MODE_DIRECT;
	odp_pktio_t pktio = odp_pktio_open(argv[1], pool, &pp);

	if (pktio == ODP_PKTIO_INVALID)
		return 4;
	odp_pktin_queue_param_init(&iq);
	iq.classifier_enable = cls;
	if (odp_pktin_queue_config(pktio, &iq))
		return 5;
	odp_pktout_queue_param_init(&oq);
	if (odp_pktout_queue_config(pktio, &oq))
		return 5;
	if (!getenv("RX_NO_PROMISC"))
		odp_pktio_promisc_mode_set(pktio, 1);
	odp_pktio_config_init(&cfg);
	cfg.parser.layer = (odp_proto_layer_t)layer;
	/* RX_PKTIN_OPT: odp_pktin_config_opt_t.all_bits (checksum / drop options) */
	if (getenv("RX_PKTIN_OPT"))
		cfg.pktin.all_bits = strtoull(getenv("RX_PKTIN_OPT"), NULL, 0);
	if (odp_pktio_config(pktio, &cfg))
		return 6;
	if (strcmp(argv[2], "-") != 0) {
		FILE *f = fopen(argv[2], "r");

		if (!f)
			return 7;
		replay(f, pktio, cos_pools);
		fclose(f);
	}
	count_only = getenv("RX_COUNT_ONLY") != NULL;
	if (odp_pktio_start(pktio))
		return 8;
	fprintf(stderr, "T started\n");
	/* rate runs time the steady state: GPU context, rule upload and the
	 * warm-up launch happen in odp_pktio_start */
	odp_time_t t_start = odp_time_local();

	/* loop: feed the source frames through a parse-less pcap pktio.
	 * RX_LOOP_ROUNDS=R (rate runs, direct mode): R rounds of "send the
	 * capture into the loop (not timed), receive and drain it (timed)" */
	const int is_loop = strncmp(argv[1], "loop", 4) == 0 && argc > 7;
	int rounds = getenv("RX_LOOP_ROUNDS") ? atoi(getenv("RX_LOOP_ROUNDS")) : 1;
	uint64_t timed_ns = 0;

	/* RX_FEED_POOL=1: the loop "wire" sends packets of a pool of its own
	 * ("feedPool"; with ODP_AMD_PAGEABLE_POOLS=feedPool in ordinary memory,
	 * outside the page-locked arena the GPU stages loop packets in) */
	odp_pool_t feed_pool = getenv("RX_FEED_POOL") ? mkpool("feedPool") : pool;

	if (is_loop && feed_loop(argv[7], feed_pool, pktio) < 0)
		return 9;
	if (is_loop && rounds > 1)
		t_start = odp_time_local();
again:

	if (pp.in_mode == ODP_PKTIN_MODE_DIRECT) {
		odp_pktin_queue_t inq;
		odp_packet_t pk[512];
		int n, idle = 0;

		if (odp_pktin_queue(pktio, &inq, 1) != 1)
			return 11;
		const char *sw = getenv("RX_SWITCH_RULES");
		int sw_after = getenv("RX_SWITCH_AFTER") ? atoi(getenv("RX_SWITCH_AFTER")) : 1;

		while (idle < 3) {
			odp_time_t t0 = odp_time_local();

			n = odp_pktin_recv(inq, pk, 512);
			odp_time_t t1 = odp_time_local();

			recv_ns += odp_time_diff_ns(t1, t0);
			if (sw && --sw_after <= 0) {
				FILE *f = fopen(sw, "r");

				if (!f)
					return 7;
				replay(f, pktio, cos_pools);
				fclose(f);
				sw = NULL;
			}
			for (int i = 0; i < n; i++) {
				print_pkt("pktin", pk[i]);
				odp_packet_free(pk[i]);
			}
			int m = 0;

			if (count_only) {
				/* rate runs: drain the CoS queues as the bursts come */
				odp_event_t ev[256];
				odp_queue_t from;

				while ((m = odp_schedule_multi(&from, ODP_SCHED_NO_WAIT, ev, 256)) > 0)
					for (int i = 0; i < m; i++)
						print_ev("-", ev[i]);
			}
			drain_ns += odp_time_diff_ns(odp_time_local(), t1);
			idle = (n == 0 && odp_amd_pktio_rx_idle(pktio) == 1) ? idle + 1 : 0;
		}
		/* classified packets went to CoS queues: drain them */
		for (;;) {
			odp_event_t ev[64];
			odp_queue_t from;

			n = odp_schedule_multi(&from, ODP_SCHED_NO_WAIT, ev, 64);
			if (n <= 0)
				break;
			for (int i = 0; i < n; i++)
				print_ev(qname(from), ev[i]);
		}
		if (is_loop && --rounds > 0) {
			timed_ns += odp_time_diff_ns(odp_time_local(), t_start);
			if (feed_loop(argv[7], feed_pool, pktio) < 0)
				return 9;
			t_start = odp_time_local();
			goto again;
		}
	} else {
		int idle = 0;
		odp_queue_t pin = ODP_QUEUE_INVALID;

		odp_pktin_event_queue(pktio, &pin, 1);
		while (idle < 3) {
			odp_event_t ev[64];
			odp_queue_t from;
			int n;

			if (pp.in_mode == ODP_PKTIN_MODE_QUEUE) {
				n = odp_queue_deq_multi(pin, ev, 64);
				from = pin;
				if (n <= 0)
					n = odp_schedule_multi(&from, ODP_SCHED_NO_WAIT, ev, 64);
			} else {
				n = odp_schedule_multi(&from, ODP_SCHED_NO_WAIT, ev, 64);
			}
			for (int i = 0; i < n; i++)
				print_ev(qname(from), ev[i]);
			idle = (n <= 0 && odp_amd_pktio_rx_idle(pktio) == 1) ? idle + 1 : 0;
			if (n <= 0 && evv_pool != ODP_POOL_INVALID)
				usleep(2000);   /* let the aggregators' max_tmo_ns pass */
		}
	}
	if (count_only) {
		printf("R %" PRIu64 " %" PRIu64 "\n", delivered,
		       timed_ns + odp_time_diff_ns(odp_time_local(), t_start));
		/* direct mode: time in odp_pktin_recv vs draining the CoS queues */
		fprintf(stderr, "RXLOOP recv_ns %" PRIu64 " drain_ns %" PRIu64 "\n", recv_ns, drain_ns);
	}
	odp_pktio_stats_t st;

	odp_pktio_stats(pktio, &st);
	printf("S %" PRIu64 " %" PRIu64 " %" PRIu64 " %" PRIu64 "\n", st.in_packets, st.in_errors,
	       st.in_discards, st.in_octets);
	for (int c = 0; c < ncos; c++) {
		odp_queue_t qs[32];
		uint32_t nq = odp_cls_cos_queues(cos_h[c], qs, 32);

		for (uint32_t s = 0; s < nq && s < 32; s++) {
			odp_cls_queue_stats_t qs_;

			if (odp_cls_queue_stats(cos_h[c], qs[s], &qs_) == 0)
				printf("Q %s %u %" PRIu64 " %" PRIu64 "\n", cos_name[c], s, qs_.packets,
				       qs_.discards);
		}
	}
	fprintf(stderr, "T loop done %.1f ms\n", odp_time_diff_ns(odp_time_local(), t_start) / 1e6);
	odp_pktio_stop(pktio);
	fprintf(stderr, "T stopped %.1f ms\n", odp_time_diff_ns(odp_time_local(), t_start) / 1e6);
	if (held) {
		odp_packet_free_multi(held, nheld);
		free(held);
	}
	odp_pktio_close(pktio);
	fprintf(stderr, "T closed %.1f ms\n", odp_time_diff_ns(odp_time_local(), t_start) / 1e6);
	return 0;
}
