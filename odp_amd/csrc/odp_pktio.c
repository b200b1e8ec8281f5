/*
 * odp_pktio.c -- packet I/O for the MI355X build: the "loop" and "pcap"
 * drivers and the GPU receive path they share.
 *
 * Reference behaviour:
 *   platform/linux-generic/odp_packet_io.c  (open/config/start/stop/close,
 *                                            pktin/pktout queue config)
 *   platform/linux-generic/pktio/loop.c:253-384   loopback_recv
 *   platform/linux-generic/pktio/pcap.c:90-401    devname parsing, promisc
 *                                                 filter, pcapif_recv_pkt
 *   include/odp_classification_internal.h:142-236 _odp_cls_enq run batching
 *
 * The receive path replaces the reference's per-packet
 *   _odp_packet_parse_common() + _odp_cls_classify_packet()
 * with ONE batched GPU launch per burst: the burst's frames are packed into a
 * pinned staging buffer at 64-byte aligned offsets, parsed and classified by
 * mi_cls_kernel (odp_amd_cls_classify_host -> mi_cls_classify_host), and the
 * 16-byte result records drive the host side exactly as the reference's
 * return codes do:
 *   parse != 0            -> in_errors++        (loop.c:311-312)
 *   parse  < 0            -> drop               (loop.c:314-317)
 *   classify < 0          -> in_discards++, drop (loop.c:324-330)
 *   classify > 0 (DROP)   -> drop
 *   pool switch           -> copy into the CoS pool (loop.c:332-337)
 *   no error flags        -> in_packets / in_octets (loop.c:352-355)
 *   enqueue               -> runs of equal (dst_queue, cos) in arrival order
 *                            (_odp_cls_enq / _odp_cos_enq + queue stats)
 * The pcap reader (classic pcap and pcapng, both byte orders) replaces
 * libpcap, which this image does not have.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <x86intrin.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <time.h>

#include "odp_rt_internal.h"
#include "mi_cls.h"

static int rx_prof = -1;   /* ODP_AMD_RX_PROF set: receive-path phase times */

static uint64_t prof_ns(void)
{
	struct timespec ts;

	if (rx_prof <= 0)
		return 0;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

enum { DRV_LOOP = 1, DRV_PCAP, DRV_NULL };
enum { ST_OPENED = 0, ST_STARTED, ST_STOPPED };

#define RX_BURST_DEFAULT 4096
/* staging sets per pktio: one burst staged and classified, one whose GPU
 * delivery is in flight, one being staged */
/* receive pipeline depth (pktio_recv): classifications and GPU deliveries
 * in flight */
#define RX_CLS_DEPTH 1
#define RX_DLV_DEPTH 3
#define RX_SETS (1 + RX_CLS_DEPTH + RX_DLV_DEPTH)
/* in-place loop bursts: offsets from the pinned arena's base stay below the
 * kernel's out-of-range offset */
#define OOB_SPAN ((size_t)0xF0000000u)
#define PCAP_MTU_MAX (64 * 1024)

/* Per-chunk pktio counters of a delivery. */
typedef struct {
	uint64_t in_errors, in_discards, octets, packets;
} rx_cnt_t;

/* One receive burst on its way through the GPU. */
typedef struct {
	uint8_t *stage;         /* copies of the frames (64 B aligned offsets) */
	size_t stage_cap;
	int stage_pinned;
	const uint8_t *base;    /* the burst's frames: base + soff[i], slen[i] bytes */
	size_t bytes;
	uint32_t *soff;
	uint16_t *slen;
	mi_cls_result_t *res;
	odp_packet_t *pk;       /* loop driver: the packets themselves */
	odp_packet_t *tmp;      /* delivery: packets grouped by queue */
	uint32_t tmp_cap;
	uint32_t n_cap;
	int arr_pinned;
	/* GPU delivery (mi_cls_deliver_submit): entries, permutation and
	 * group counts in page-locked memory; the packet of each entry */
	mi_cls_dlv_t *dlv;
	uint32_t *perm;
	uint32_t *gcnt;
	odp_packet_t *ent;      /* delivered packet per entry */
	odp_packet_t *old;      /* loop packets whose frames the GPU copies out (pool switch) */
	uint8_t *ppool;         /* loop: each packet's pool index + 1 (read at staging) */
	uint16_t *pdoff;        /* loop: each packet's headroom */
	const void **pup;       /* loop: each packet's user pointer */
	int dlv_pinned;
	/* a GPU delivery in flight (rx_dlv_start .. rx_dlv_end) */
	int delivering;
	uint64_t dticket;
	int derr;               /* the submit failed */
	uint32_t ne;            /* entries */
	int nold, grouped, ng;
	odp_queue_t gq[MI_CLS_DLV_GROUPS];
	rx_cnt_t cnt;
	int n;
	int pending;            /* staged (and submitted), not delivered */
	uint64_t ticket;        /* odp_amd_cls_classify_host_submit, 0 = done */
	uint64_t gen;           /* control-plane generation the set was submitted under */
	uint64_t dgen;          /* generation its delivery was decided under (rx_dlv_start) */
	/* receive chain (rxc_submit .. rxc_end): the burst classified, decided
	 * and delivered by the GPU from one submission, `delivering` from it */
	int chain;
	int gstage;             /* loop burst staged by the GPU (only pk[] is set) */
	int pk_pinned;          /* pk / ppool page-locked */
	int rxc_pinned;         /* dec / cent / got / rxo page-locked */
	uint32_t *dec;          /* per frame: decision word (MI_CLS_RXF_*, mi_cls.h) */
	uint64_t *cent;         /* per frame: its packet, 0 none */
	uint64_t *got;          /* packets taken for the burst, per pool slot */
	uint32_t got_cap;
	mi_cls_rx_out_t *rxo;
	uint32_t cnp, cbase[MI_CLS_RX_POOLS], chave[MI_CLS_RX_POOLS];
	odp_pool_t cpool[MI_CLS_RX_POOLS];
} rx_set_t;

typedef struct {
	int used;
	char name[ODP_PKTIO_NAME_LEN];
	int drv;
	odp_pktio_t hdl;
	odp_pool_t pool;
	odp_pktio_param_t param;
	odp_pktio_config_t config;
	odp_pktin_queue_param_t inq_param;
	odp_queue_t inq;            /* SCHED / QUEUE mode input queue */
	int inq_configured;
	uint32_t num_out;
	int state;
	int cls_enabled;
	odp_proto_layer_t parse_layer;
	int promisc;
	odp_spinlock_t rxl;
	odp_atomic_u64_t in_octets, in_packets, in_discards, in_errors;
	odp_atomic_u64_t out_octets, out_packets, out_discards;
	/* pcap */
	uint8_t *fbuf;
	uint32_t *foff;
	uint16_t *flen;
	uint32_t nframes, next;
	int loops, loop_cnt, eof;
	FILE *tx;
	/* loop */
	odp_queue_t loopq;
	size_t fbuf_bytes;      /* frame store size incl. 64 B of zero padding */
	int fbuf_pinned;        /* page-locked: the GPU reads frames in place */
	/* GPU bursts: two staging sets, so one burst is classified while the
	 * previous one is delivered (pipelined receive) */
	rx_set_t rs[RX_SETS];
	int cur;                /* set the next burst is staged into */
	/* receive chain: the control plane's table (per generation), the pools
	 * of its slots and how many packets of each a burst is given */
	mi_cls_rxtab_t *rxtab;
	int rxtab_pinned, rxtab_ok;
	uint64_t rxtab_gen;
	odp_pool_t rx_pools[MI_CLS_RX_POOLS];
	uint32_t rx_np, rx_want[MI_CLS_RX_POOLS];
	uint64_t prof[14];      /* ODP_AMD_RX_PROF: ns staging / classifying / delivering, bursts,
				 * then of delivering: ns preparing / enqueueing, TSC ticks in
				 * packet allocation / frame copies; GPU delivery: ns deciding +
				 * taking packets + entries, ns in the delivery kernel (submit to
				 * wait), ns enqueueing, bursts; receive chain: ns in its
				 * submit call (odp_amd_cls_rx_chain) */
} rt_pktio_t;

static void rx_sets_free(rt_pktio_t *e);
static void fbuf_free(rt_pktio_t *e);
static int rx_finish(rt_pktio_t *e, rx_set_t *s, odp_packet_t out[], int max_out);
static int rx_dlv_end(rt_pktio_t *e, rx_set_t *s, odp_packet_t out[], int max_out);
static rx_set_t *rx_age(rt_pktio_t *e, int k);
static int stage_reserve(rx_set_t *s, uint32_t n, size_t bytes);
static int rxc_loop_stage_ok(rt_pktio_t *e, rx_set_t *s, uint32_t max);
static int loop_stage_hdrs(rt_pktio_t *e, rx_set_t *s, uint32_t n);

static rt_pktio_t PK[RT_MAX_PKTIO];
static odp_spinlock_t pk_lock;
/* started SCHED-mode pktios, polled from odp_schedule*() */
static int sched_list[RT_MAX_PKTIO];
static int num_sched_pktio;

static const uint8_t pcap_mac[6] = { 0x02, 0x00, 0x00, 0x00, 0x00, 0x02 };
static const uint8_t loop_mac[6] = { 0x02, 0xe9, 0x34, 0x80, 0x73, 0x01 };

uint32_t rt_gpu_index(void)
{
	const char *e = getenv("ODP_AMD_GPU");

	return e ? (uint32_t)atoi(e) : 0u;
}

static uint32_t rx_burst(void)
{
	static uint32_t b;

	if (!b) {
		const char *e = getenv("ODP_AMD_RX_BURST");

		b = e && atoi(e) > 0 ? (uint32_t)atoi(e) : RX_BURST_DEFAULT;
	}
	return b;
}

static rt_pktio_t *get_pk(odp_pktio_t h)
{
	uintptr_t i = (uintptr_t)h;

	if (i == 0 || i > RT_MAX_PKTIO || !PK[i - 1].used)
		return NULL;
	return &PK[i - 1];
}

/* ============================================================ pcap reader */
static uint32_t rd32s(const uint8_t *p, int swap)
{
	uint32_t v;

	memcpy(&v, p, 4);
	return swap ? __builtin_bswap32(v) : v;
}

static uint16_t rd16s(const uint8_t *p, int swap)
{
	uint16_t v;

	memcpy(&v, p, 2);
	return swap ? __builtin_bswap16(v) : v;
}

/* append one frame to the packed, 64 B aligned frame store */
static int frame_add(rt_pktio_t *e, const uint8_t *d, uint32_t caplen, size_t *cap_b,
		     uint32_t *cap_n, size_t *used_b)
{
	if (caplen > 65535 || caplen == 0)
		return 0;   /* longer than the u16 descriptor: not received */
	if (e->nframes == *cap_n) {
		uint32_t nn = *cap_n ? *cap_n * 2 : 1024;
		uint32_t *o = realloc(e->foff, nn * sizeof(uint32_t));
		uint16_t *l = o ? realloc(e->flen, nn * sizeof(uint16_t)) : NULL;

		if (!o || !l)
			return -1;
		e->foff = o;
		e->flen = l;
		*cap_n = nn;
	}
	size_t need = *used_b + ((caplen + 63u) & ~63u);

	if (need > *cap_b) {
		size_t nb = *cap_b ? *cap_b : (1u << 20);

		while (nb < need)
			nb *= 2;
		uint8_t *b = realloc(e->fbuf, nb);

		if (!b)
			return -1;
		memset(b + *cap_b, 0, nb - *cap_b);
		e->fbuf = b;
		*cap_b = nb;
	}
	memcpy(e->fbuf + *used_b, d, caplen);
	e->foff[e->nframes] = (uint32_t)*used_b;
	e->flen[e->nframes] = (uint16_t)caplen;
	e->nframes++;
	*used_b = need;
	return 0;
}

/* Classic pcap (0xa1b2c3d4 / 0xa1b23c4d, either byte order) and pcapng
 * (SHB / IDB / EPB / SPB / PB blocks).  Only DLT_EN10MB (1) is accepted,
 * as in _pcapif_init_rx (pcap.c:130-134).  Returns 0 / -1. */
static int pcap_load(rt_pktio_t *e, const char *fname)
{
	FILE *f = fopen(fname, "rb");
	uint8_t *buf = NULL;
	long sz;
	size_t cap_b = 0, used_b = 0;
	uint32_t cap_n = 0;
	int rc = -1;

	if (!f) {
		RT_ERR("failed to open pcap file %s (%s)\n", fname, strerror(errno));
		return -1;
	}
	if (fseek(f, 0, SEEK_END) || (sz = ftell(f)) < 0 || fseek(f, 0, SEEK_SET))
		goto out;
	buf = malloc((size_t)sz + 1);
	if (!buf || fread(buf, 1, (size_t)sz, f) != (size_t)sz)
		goto out;
	if (sz < 24)
		goto bad;
	uint32_t m = rd32s(buf, 0);

	if (m == 0xa1b2c3d4u || m == 0xa1b23c4du || m == 0xd4c3b2a1u || m == 0x4d3cb2a1u) {
		int sw = (m == 0xd4c3b2a1u || m == 0x4d3cb2a1u);

		if ((rd32s(buf + 20, sw) & 0x0fffffffu) != 1u) {
			RT_ERR("unsupported datalink type: %u\n", rd32s(buf + 20, sw));
			goto out;
		}
		for (long p = 24; p + 16 <= sz;) {
			uint32_t incl = rd32s(buf + p + 8, sw);

			if (p + 16 + (long)incl > sz)
				break;
			if (frame_add(e, buf + p + 16, incl, &cap_b, &cap_n, &used_b))
				goto out;
			p += 16 + incl;
		}
		rc = 0;
	} else if (m == 0x0a0d0d0au) {
		int sw = 0;
		uint32_t link[64], nif = 0, snap[64];

		for (long p = 0; p + 12 <= sz;) {
			uint32_t type = rd32s(buf + p, sw);

			if (type == 0x0a0d0d0au) {   /* section header: byte order */
				uint32_t bom;

				memcpy(&bom, buf + p + 8, 4);
				sw = bom == 0x4d3c2b1au;
				nif = 0;
			}
			uint32_t blen = rd32s(buf + p + 4, sw);

			if (blen < 12 || p + (long)blen > sz)
				break;
			const uint8_t *b = buf + p + 8;

			if (type == 1 && nif < 64) {             /* interface description */
				link[nif] = rd16s(b, sw);
				snap[nif] = rd32s(b + 4, sw);
				nif++;
			} else if (type == 6 && blen >= 32) {   /* enhanced packet */
				uint32_t ifc = rd32s(b, sw), cap = rd32s(b + 12, sw);

				if (ifc < nif && link[ifc] != 1)
					goto bad_link;
				if (20 + cap <= blen - 12 &&
				    frame_add(e, b + 20, cap, &cap_b, &cap_n, &used_b))
					goto out;
			} else if (type == 3 && blen >= 16) {   /* simple packet */
				uint32_t olen = rd32s(b, sw), cap = olen;

				if (nif && link[0] != 1)
					goto bad_link;
				if (nif && snap[0] && cap > snap[0])
					cap = snap[0];
				if (4 + cap <= blen - 12 &&
				    frame_add(e, b + 4, cap, &cap_b, &cap_n, &used_b))
					goto out;
			} else if (type == 2 && blen >= 32) {   /* obsolete packet block */
				uint32_t ifc = rd16s(b, sw), cap = rd32s(b + 12, sw);

				if (ifc < nif && link[ifc] != 1)
					goto bad_link;
				if (20 + cap <= blen - 12 &&
				    frame_add(e, b + 20, cap, &cap_b, &cap_n, &used_b))
					goto out;
			}
			p += blen;
		}
		rc = 0;
	} else {
		goto bad;
	}
	goto out;
bad_link:
	RT_ERR("unsupported datalink type in %s\n", fname);
	goto out;
bad:
	RT_ERR("%s: not a pcap / pcapng file\n", fname);
out:
	if (rc == 0 && e->fbuf) {
		/* page-locked frame store: the GPU reads the bursts' header windows
		 * in place (zero copy, mi_cls_classify_host) and no staging copy is
		 * made.  ODP_AMD_RX_INPLACE=0 keeps the staged copies (A/B runs). */
		const char *v = getenv("ODP_AMD_RX_INPLACE");
		uint8_t *pb = v && v[0] == '0' ? NULL : mi_cls_host_alloc(used_b + 64);

		e->fbuf_bytes = used_b + 64;
		if (pb) {
			memcpy(pb, e->fbuf, used_b);
			memset(pb + used_b, 0, 64);
			free(e->fbuf);
			e->fbuf = pb;
			e->fbuf_pinned = 1;
		}
	}
	free(buf);
	fclose(f);
	return rc;
}

static int pcap_dump_open(rt_pktio_t *e, const char *fname)
{
	const uint32_t hdr[6] = { 0xa1b2c3d4u, 0x00040002u, 0, 0, PCAP_MTU_MAX, 1 };

	e->tx = fopen(fname, "wb");
	if (!e->tx) {
		RT_ERR("failed to open dump file %s\n", fname);
		return -1;
	}
	fwrite(hdr, sizeof(hdr), 1, e->tx);
	fflush(e->tx);
	return 0;
}

static void pcap_dump(rt_pktio_t *e, odp_packet_t pkt)
{
	struct timeval tv;
	uint32_t h[4];
	pkt_hdr_t *p = rt_pkt_hdr(pkt);

	gettimeofday(&tv, NULL);
	h[0] = (uint32_t)tv.tv_sec;
	h[1] = (uint32_t)tv.tv_usec;
	h[2] = h[3] = p->len;
	fwrite(h, sizeof(h), 1, e->tx);
	fwrite(p->head + p->data_off, 1, p->len, e->tx);
	fflush(e->tx);
}

/* _pcapif_parse_devname (pcap.c:90-117) */
static int pcap_open(rt_pktio_t *e, const char *devname)
{
	char in[ODP_PKTIO_NAME_LEN], *tok, *save = NULL;
	char *rx = NULL, *txn = NULL;
	int rc = 0;

	snprintf(in, sizeof(in), "%s", devname);
	e->loops = 1;
	e->loop_cnt = 1;
	for (tok = strtok_r(in + 5, ":", &save); tok; tok = strtok_r(NULL, ":", &save)) {
		if (strncmp(tok, "in=", 3) == 0 && !rx) {
			rx = strdup(tok + 3);
		} else if (strncmp(tok, "out=", 4) == 0 && !txn) {
			txn = strdup(tok + 4);
		} else if (strncmp(tok, "loops=", 6) == 0) {
			e->loops = atoi(tok + 6);
			if (e->loops < 0) {
				RT_ERR("invalid loop count\n");
				rc = -1;
			}
		}
	}
	if (!rc && rx)
		rc = pcap_load(e, rx);
	if (!rc && txn)
		rc = pcap_dump_open(e, txn);
	if (!rc && !rx && !txn)
		rc = -1;
	free(rx);
	free(txn);
	e->promisc = 0;   /* pcapif_init sets promisc off (pcap.c:232) */
	return rc;
}

/* BPF "ether dst <pcap_mac> or broadcast or multicast" (pcap.c:176-186) */
static int pcap_filter_pass(const rt_pktio_t *e, const uint8_t *d, uint32_t len)
{
	if (e->promisc)
		return 1;
	if (len < 6)
		return 0;
	return memcmp(d, pcap_mac, 6) == 0 || (d[0] & 1u);
}

/* ============================================================ open / config */
void odp_pktio_param_init(odp_pktio_param_t *p)
{
	memset(p, 0, sizeof(*p));
	p->in_mode = ODP_PKTIN_MODE_DIRECT;
	p->out_mode = ODP_PKTOUT_MODE_DIRECT;
}

void odp_pktin_queue_param_init(odp_pktin_queue_param_t *p)
{
	memset(p, 0, sizeof(*p));
	p->op_mode = ODP_PKTIO_OP_MT;
	p->num_queues = 1;
	p->classifier_enable = 0;
	odp_queue_param_init(&p->queue_param);
	p->queue_param.type = ODP_QUEUE_TYPE_SCHED;
}

void odp_pktout_queue_param_init(odp_pktout_queue_param_t *p)
{
	memset(p, 0, sizeof(*p));
	p->op_mode = ODP_PKTIO_OP_MT;
	p->num_queues = 1;
}

void odp_pktio_config_init(odp_pktio_config_t *c)
{
	memset(c, 0, sizeof(*c));
	c->parser.layer = ODP_PROTO_LAYER_ALL;
	c->reassembly.max_num_frags = 2;
}

odp_pktio_t odp_pktio_open(const char *name, odp_pool_t pool, const odp_pktio_param_t *param)
{
	odp_pktio_param_t def;
	int drv;

	if (!name)
		return ODP_PKTIO_INVALID;
	if (strncmp(name, "pcap:", 5) == 0)
		drv = DRV_PCAP;
	else if (strncmp(name, "loop", 4) == 0)
		drv = DRV_LOOP;
	else if (strncmp(name, "null", 4) == 0)
		drv = DRV_NULL;
	else {
		RT_ERR("pktio %s: no driver (this build has loop, pcap:in=/out=, null)\n", name);
		return ODP_PKTIO_INVALID;
	}
	rt_pool_t *pp = rt_pool(pool);

	if (!pp || pp->param.type != ODP_POOL_PACKET) {
		RT_ERR("pktio %s: invalid packet pool\n", name);
		return ODP_PKTIO_INVALID;
	}
	if (!param) {
		odp_pktio_param_init(&def);
		param = &def;
	}
	if (odp_pktio_lookup(name) != ODP_PKTIO_INVALID) {
		RT_ERR("pktio %s already open\n", name);
		return ODP_PKTIO_INVALID;
	}
	/* the classifier endpoint (classifier_t + device context) gives the
	 * handle; ODP_AMD_GPUS="0,1,..." shards each receive burst over several
	 * GPUs (mi_cls_group_classify_host), otherwise ODP_AMD_GPU picks one */
	int gpus[16], ngpu = 0;
	const char *ge = getenv("ODP_AMD_GPUS");

	while (ge && *ge && ngpu < 16) {
		char *end;
		long v = strtol(ge, &end, 10);

		if (end == ge)
			break;
		gpus[ngpu++] = (int)v;
		ge = *end == ',' ? end + 1 : end;
	}
	odp_pktio_t h = ngpu > 1 ? odp_amd_cls_pktio_create_multi(gpus, ngpu)
				 : odp_amd_cls_pktio_create(ngpu == 1 ? gpus[0] : (int)rt_gpu_index());

	if (h == ODP_PKTIO_INVALID)
		return h;
	rt_pktio_t *e = &PK[(uintptr_t)h - 1];

	odp_spinlock_lock(&pk_lock);
	memset(e, 0, sizeof(*e));
	e->used = 1;
	odp_spinlock_unlock(&pk_lock);
	snprintf(e->name, sizeof(e->name), "%s", name);
	e->drv = drv;
	e->hdl = h;
	e->pool = pool;
	e->param = *param;
	odp_pktio_config_init(&e->config);
	odp_spinlock_init(&e->rxl);
	e->state = ST_OPENED;
	e->promisc = 1;
	if (drv == DRV_PCAP && pcap_open(e, name)) {
		fbuf_free(e);
		free(e->foff);
		free(e->flen);
		e->used = 0;
		odp_amd_cls_pktio_destroy(h);
		return ODP_PKTIO_INVALID;
	}
	if (drv == DRV_LOOP) {
		odp_queue_param_t qp;
		char qn[ODP_QUEUE_NAME_LEN];

		odp_queue_param_init(&qp);
		snprintf(qn, sizeof(qn), "%.20s_loopq", name);
		e->loopq = odp_queue_create(qn, &qp);
		if (e->loopq == ODP_QUEUE_INVALID) {
			e->used = 0;
			odp_amd_cls_pktio_destroy(h);
			return ODP_PKTIO_INVALID;
		}
	}
	/* default queue config as odp_pktio_open does for DISABLED-less modes */
	odp_pktin_queue_param_init(&e->inq_param);
	return h;
}

odp_pktio_t odp_pktio_lookup(const char *name)
{
	for (int i = 0; i < RT_MAX_PKTIO; i++)
		if (PK[i].used && name && strcmp(PK[i].name, name) == 0)
			return PK[i].hdl;
	return ODP_PKTIO_INVALID;
}

int odp_pktio_capability(odp_pktio_t h, odp_pktio_capability_t *c)
{
	rt_pktio_t *e = get_pk(h);

	if (!e || !c)
		return -1;
	memset(c, 0, sizeof(*c));
	c->max_input_queues = 1;
	c->max_output_queues = e->drv == DRV_LOOP ? ODP_PKTOUT_MAX_QUEUES : 1;
	c->max_input_queue_size = 0;
	c->max_output_queue_size = 0;
	odp_pktio_config_init(&c->config);
	c->config.parser.layer = ODP_PROTO_LAYER_ALL;
	c->config.pktin.all_bits = RT_PKTIN_OPT_MASK;
	c->config.enable_loop = 0;
	c->set_op.op.promisc_mode = e->drv == DRV_PCAP;
	c->maxlen.equal = 1;
	c->maxlen.min_input = c->maxlen.min_output = 68 + 14;
	c->maxlen.max_input = c->maxlen.max_output = 65535;
	c->loop_supported = ODP_SUPPORT_NO;
	return 0;
}

int odp_pktio_config(odp_pktio_t h, const odp_pktio_config_t *config)
{
	rt_pktio_t *e = get_pk(h);
	odp_pktio_config_t def;

	if (!e)
		return -1;
	if (!config) {
		odp_pktio_config_init(&def);
		config = &def;
	}
	/* parser options, pktin checksum validation and drop-on-error options
	 * (bits 2-10); no timestamps, pktout offloads, IPsec or LSO */
	if ((config->pktin.all_bits & ~RT_PKTIN_OPT_MASK) || config->pktout.all_bits ||
	    config->enable_loop || config->inbound_ipsec || config->outbound_ipsec ||
	    config->enable_lso) {
		RT_ERR("pktio %s: unsupported configuration option\n", e->name);
		return -1;
	}
	if (e->state == ST_STARTED)
		return -1;
	e->config = *config;
	return 0;
}

int odp_pktin_queue_config(odp_pktio_t h, const odp_pktin_queue_param_t *param)
{
	rt_pktio_t *e = get_pk(h);
	odp_pktin_queue_param_t def;

	if (!e || e->state == ST_STARTED)
		return -1;
	if (!param) {
		odp_pktin_queue_param_init(&def);
		param = &def;
	}
	if (e->param.in_mode == ODP_PKTIN_MODE_DISABLED)
		return -1;
	if (param->num_queues > 1 || (param->num_queues == 0 && !param->classifier_enable)) {
		RT_ERR("pktio %s: %u input queues requested, 1 supported\n", e->name,
		       param->num_queues);
		return -1;
	}
	if (param->vector.enable) {
		RT_ERR("pktio %s: packet vectors are not supported\n", e->name);
		return -1;
	}
	if (e->inq != ODP_QUEUE_INVALID) {
		odp_queue_destroy(e->inq);
		e->inq = ODP_QUEUE_INVALID;
	}
	e->inq_param = *param;
	e->cls_enabled = param->classifier_enable;
	if (e->param.in_mode == ODP_PKTIN_MODE_SCHED || e->param.in_mode == ODP_PKTIN_MODE_QUEUE) {
		odp_queue_param_t qp = param->queue_param;
		char qn[ODP_QUEUE_NAME_LEN];

		qp.type = e->param.in_mode == ODP_PKTIN_MODE_SCHED ? ODP_QUEUE_TYPE_SCHED
								    : ODP_QUEUE_TYPE_PLAIN;
		snprintf(qn, sizeof(qn), "odp-pktin-%d-0", (int)((uintptr_t)h - 1));
		e->inq = odp_queue_create(qn, &qp);
		if (e->inq == ODP_QUEUE_INVALID)
			return -1;
		if (e->param.in_mode == ODP_PKTIN_MODE_QUEUE)
			((rt_queue_t *)(void *)e->inq)->pktin_idx = (int)(uintptr_t)h;
	}
	e->inq_configured = 1;
	return 0;
}

int odp_pktout_queue_config(odp_pktio_t h, const odp_pktout_queue_param_t *param)
{
	rt_pktio_t *e = get_pk(h);
	odp_pktio_capability_t c;

	if (!e || e->state == ST_STARTED || odp_pktio_capability(h, &c))
		return -1;
	uint32_t n = param ? param->num_queues : 1;

	if (n == 0 || n > c.max_output_queues)
		return -1;
	e->num_out = n;
	return 0;
}

int odp_pktin_queue(odp_pktio_t h, odp_pktin_queue_t q[], int num)
{
	rt_pktio_t *e = get_pk(h);

	if (!e || e->param.in_mode != ODP_PKTIN_MODE_DIRECT)
		return -1;
	if (num > 0 && q) {
		q[0].q = (_odp_pktin_hdl_t)(uintptr_t)h;
		q[0].index = 0;
		q[0].pktio = h;
	}
	return 1;
}

int odp_pktin_event_queue(odp_pktio_t h, odp_queue_t q[], int num)
{
	rt_pktio_t *e = get_pk(h);

	if (!e || (e->param.in_mode != ODP_PKTIN_MODE_SCHED &&
		   e->param.in_mode != ODP_PKTIN_MODE_QUEUE))
		return -1;
	if (num > 0 && q)
		q[0] = e->inq;
	return e->inq != ODP_QUEUE_INVALID ? 1 : 0;
}

int odp_pktout_queue(odp_pktio_t h, odp_pktout_queue_t q[], int num)
{
	rt_pktio_t *e = get_pk(h);

	if (!e || e->param.out_mode != ODP_PKTOUT_MODE_DIRECT)
		return -1;
	if (!e->num_out)
		e->num_out = 1;
	for (int i = 0; i < num && (uint32_t)i < e->num_out; i++) {
		q[i].q = (void *)(uintptr_t)h;
		q[i].index = i;
		q[i].pktio = h;
	}
	return (int)e->num_out;
}

int odp_pktio_start(odp_pktio_t h)
{
	rt_pktio_t *e = get_pk(h);

	if (!e)
		return -1;
	if (e->state == ST_STARTED) {
		RT_ERR("Already started\n");
		return -1;
	}
	if (!e->inq_configured && e->param.in_mode != ODP_PKTIN_MODE_DISABLED &&
	    odp_pktin_queue_config(h, NULL))
		return -1;
	/* odp_packet_io.c:675-677 */
	e->parse_layer = e->cls_enabled ? ODP_PROTO_LAYER_ALL : e->config.parser.layer;
	/* GPU context, rule snapshot and a warm-up launch before traffic */
	if (e->param.in_mode != ODP_PKTIN_MODE_DISABLED && e->parse_layer != ODP_PROTO_LAYER_NONE) {
		/* the options of the layers that are parsed: L3 takes the IPv4
		 * header checksum and the IP drops, L4 everything (odp_parse.c:
		 * 372-414 stop before the rest) */
		uint64_t opt = e->config.pktin.all_bits & RT_PKTIN_OPT_MASK;

		if (e->parse_layer < ODP_PROTO_LAYER_L3)
			opt = 0;
		else if (e->parse_layer == ODP_PROTO_LAYER_L3)
			opt &= (1u << 2) | (1u << 6) | (1u << 7);
		odp_amd_cls_pktin_opt_set(h, opt);
		int rc = odp_amd_cls_prepare(h, !e->cls_enabled);

		if (rc) {
			RT_ERR("pktio %s: GPU receive path unavailable (%s)\n", e->name,
			       mi_cls_strerror(rc));
			return -1;
		}
		/* the burst sets' page-locked arrays too: made here, not by the
		 * first bursts (each page-locked allocation is a runtime call) */
		for (int k = 0; k < RX_SETS; k++)
			(void)stage_reserve(&e->rs[k], rx_burst(), 0);
	}
	e->state = ST_STARTED;
	if (e->param.in_mode == ODP_PKTIN_MODE_SCHED) {
		odp_spinlock_lock(&pk_lock);
		sched_list[num_sched_pktio++] = (int)((uintptr_t)h - 1);
		odp_spinlock_unlock(&pk_lock);
	}
	return 0;
}

static void sched_list_remove(int idx)
{
	odp_spinlock_lock(&pk_lock);
	for (int i = 0; i < num_sched_pktio; i++)
		if (sched_list[i] == idx) {
			sched_list[i] = sched_list[--num_sched_pktio];
			break;
		}
	odp_spinlock_unlock(&pk_lock);
}

int odp_pktio_stop(odp_pktio_t h)
{
	rt_pktio_t *e = get_pk(h);

	if (!e || e->state != ST_STARTED) {
		RT_ERR("Not started\n");
		return -1;
	}
	sched_list_remove((int)((uintptr_t)h - 1));
	odp_spinlock_lock(&e->rxl);   /* wait for an in-flight burst */
	/* bursts still on the GPU were received before the stop: deliver them,
	 * oldest first */
	for (int k = 1; k <= RX_SETS; k++) {
		rx_set_t *s = &e->rs[(e->cur + k) % RX_SETS];

		if (s->delivering)
			(void)rx_dlv_end(e, s, NULL, 0);
		if (s->pending)
			(void)rx_finish(e, s, NULL, 0);
	}
	e->state = ST_STOPPED;
	odp_spinlock_unlock(&e->rxl);
	return 0;
}

int odp_pktio_close(odp_pktio_t h)
{
	rt_pktio_t *e = get_pk(h);

	if (!e)
		return -1;
	if (e->state == ST_STARTED) {
		RT_ERR("pktio %s: close while started\n", e->name);
		return -1;
	}
	if (rx_prof > 0 && e->prof[3])
		fprintf(stderr, "RXPROF %s bursts %" PRIu64 " stage_ns %" PRIu64 " classify_ns %" PRIu64
			" deliver_ns %" PRIu64 " (prepare_ns %" PRIu64 " enqueue_ns %" PRIu64
			" alloc_tsc %" PRIu64 " copy_tsc %" PRIu64 ") gpu_bursts %" PRIu64
			" (decide_ns %" PRIu64 " submit_ns %" PRIu64 " kernel_ns %" PRIu64 " enqueue_ns %" PRIu64
			") chain_submit_ns %" PRIu64 "\n", e->name,
			e->prof[3], e->prof[0], e->prof[1], e->prof[2], e->prof[4], e->prof[5], e->prof[6],
			e->prof[7], e->prof[11], e->prof[8], e->prof[12], e->prof[9], e->prof[10], e->prof[13]);
	if (e->inq != ODP_QUEUE_INVALID) {
		odp_event_t ev[64];
		int n;

		while ((n = rt_queue_deq_multi_raw((rt_queue_t *)(void *)e->inq, ev, 64)) > 0)
			odp_event_free_multi(ev, n);
		odp_queue_destroy(e->inq);
	}
	if (e->loopq != ODP_QUEUE_INVALID) {
		odp_event_t ev[64];
		int n;

		while ((n = rt_queue_deq_multi_raw((rt_queue_t *)(void *)e->loopq, ev, 64)) > 0)
			odp_event_free_multi(ev, n);
		odp_queue_destroy(e->loopq);
	}
	if (e->tx)
		fclose(e->tx);
	fbuf_free(e);
	free(e->foff);
	free(e->flen);
	rx_sets_free(e);
	odp_spinlock_lock(&pk_lock);
	memset(e, 0, sizeof(*e));
	odp_spinlock_unlock(&pk_lock);
	return odp_amd_cls_pktio_destroy(h);
}

/* ============================================================ receive */
/* Host memory the GPU can read in place (page-locked) where there is a GPU,
 * ordinary memory otherwise (parse layer NONE needs none). */
static void *hmem_alloc(size_t bytes, int *pinned)
{
	void *p = mi_cls_host_alloc(bytes);

	*pinned = p != NULL;
	return p ? p : malloc(bytes);
}

static void hmem_free(void *p, int pinned)
{
	if (pinned)
		mi_cls_host_free(p);
	else
		free(p);
}

static void fbuf_free(rt_pktio_t *e)
{
	hmem_free(e->fbuf, e->fbuf_pinned);
	e->fbuf = NULL;
	e->fbuf_pinned = 0;
}

static void rx_set_arrays_free(rx_set_t *s)
{
	hmem_free(s->soff, s->arr_pinned);
	hmem_free(s->slen, s->arr_pinned);
	hmem_free(s->res, s->arr_pinned);
	hmem_free(s->dlv, s->dlv_pinned);
	hmem_free(s->perm, s->dlv_pinned);
	hmem_free(s->gcnt, s->dlv_pinned);
	free(s->ent);
	free(s->old);
	hmem_free(s->ppool, s->pk_pinned);
	free(s->pdoff);
	free(s->pup);
	s->pup = NULL;
	s->dlv = NULL;
	s->perm = NULL;
	s->gcnt = NULL;
	s->ent = NULL;
	s->old = NULL;
	s->ppool = NULL;
	s->pdoff = NULL;
	s->dlv_pinned = 0;
	hmem_free(s->pk, s->pk_pinned);
	hmem_free(s->dec, s->rxc_pinned);
	hmem_free(s->cent, s->rxc_pinned);
	hmem_free(s->got, s->rxc_pinned);
	hmem_free(s->rxo, s->rxc_pinned);
	s->dec = NULL;
	s->cent = NULL;
	s->got = NULL;
	s->rxo = NULL;
	s->got_cap = 0;
	s->rxc_pinned = 0;
	free(s->tmp);
	s->tmp = NULL;
	s->tmp_cap = 0;
	s->soff = NULL;
	s->slen = NULL;
	s->res = NULL;
	s->pk = NULL;
	s->n_cap = 0;
}

static void rx_sets_free(rt_pktio_t *e)
{
	hmem_free(e->rxtab, e->rxtab_pinned);
	e->rxtab = NULL;
	e->rxtab_pinned = 0;
	e->rxtab_ok = 0;
	e->rxtab_gen = 0;
	e->rx_np = 0;
	for (int k = 0; k < RX_SETS; k++) {
		rx_set_t *s = &e->rs[k];

		hmem_free(s->stage, s->stage_pinned);
		rx_set_arrays_free(s);
		memset(s, 0, sizeof(*s));
	}
}

/* descriptor arrays for n frames; stage bytes grow keeping the contents */
static int stage_reserve(rx_set_t *s, uint32_t n, size_t bytes)
{
	if (n > s->n_cap) {
		uint32_t c = n < 256 ? 256 : n;
		int p1, p2, p3;

		rx_set_arrays_free(s);
		s->soff = hmem_alloc(c * sizeof(uint32_t), &p1);
		s->slen = hmem_alloc(c * sizeof(uint16_t), &p2);
		s->res = hmem_alloc(c * sizeof(mi_cls_result_t), &p3);
		s->arr_pinned = p1;
		int k1, k2;

		s->pk = hmem_alloc(c * sizeof(odp_packet_t), &k1);
		s->ppool = hmem_alloc(c, &k2);
		s->pk_pinned = k1 && k2;
		if (k1 != k2 && s->pk && s->ppool) {   /* mixed: ordinary copies */
			hmem_free(s->pk, k1);
			hmem_free(s->ppool, k2);
			s->pk = malloc(c * sizeof(odp_packet_t));
			s->ppool = malloc(c);
		}
		if (p1 != p2 || p1 != p3) {   /* mixed: keep the pageable copies */
			hmem_free(s->soff, p1);
			hmem_free(s->slen, p2);
			hmem_free(s->res, p3);
			s->soff = malloc(c * sizeof(uint32_t));
			s->slen = malloc(c * sizeof(uint16_t));
			s->res = malloc(c * sizeof(mi_cls_result_t));
			s->arr_pinned = 0;
		}
		if (!s->soff || !s->slen || !s->res || !s->pk) {
			rx_set_arrays_free(s);
			return -1;
		}
		/* GPU delivery arrays: only when all three are page-locked */
		int q1, q2, q3;

		s->dlv = hmem_alloc(c * sizeof(mi_cls_dlv_t), &q1);
		s->perm = hmem_alloc(c * sizeof(uint32_t), &q2);
		s->gcnt = hmem_alloc(MI_CLS_DLV_GROUPS * sizeof(uint32_t), &q3);
		s->ent = malloc(c * sizeof(odp_packet_t));
		s->old = malloc(c * sizeof(odp_packet_t));
		s->pdoff = malloc(c * sizeof(uint16_t));
		s->pup = malloc(c * sizeof(void *));
		if (!s->ppool || !s->pdoff || !s->pup) {
			rx_set_arrays_free(s);
			return -1;
		}
		/* receive chain arrays (page-locked or none) */
		{
			int r1, r2, r3, r4;

			s->dec = hmem_alloc(c * sizeof(uint32_t), &r1);
			s->cent = hmem_alloc(c * sizeof(uint64_t), &r2);
			s->got = hmem_alloc((size_t)4 * c * sizeof(uint64_t), &r3);
			s->rxo = hmem_alloc(sizeof(mi_cls_rx_out_t), &r4);
			s->rxc_pinned = r1 && r2 && r3 && r4;
			s->got_cap = 4u * c;
			if (!s->rxc_pinned) {
				hmem_free(s->dec, r1);
				hmem_free(s->cent, r2);
				hmem_free(s->got, r3);
				hmem_free(s->rxo, r4);
				s->dec = NULL;
				s->cent = NULL;
				s->got = NULL;
				s->rxo = NULL;
				s->got_cap = 0;
			}
		}
		s->dlv_pinned = q1 && q2 && q3 && s->dlv && s->perm && s->gcnt && s->ent && s->old;
		if (!s->dlv_pinned) {
			hmem_free(s->dlv, q1);
			hmem_free(s->perm, q2);
			hmem_free(s->gcnt, q3);
			free(s->ent);
			free(s->old);
			s->dlv = NULL;
			s->perm = NULL;
			s->gcnt = NULL;
			s->ent = NULL;
			s->old = NULL;
		}
		s->n_cap = c;
	}
	if (bytes > s->stage_cap) {
		size_t c = s->stage_cap ? s->stage_cap : (4u << 20);
		int pinned;

		while (c < bytes)
			c *= 2;
		uint8_t *ns = hmem_alloc(c, &pinned);

		if (!ns)
			return -1;
		if (s->stage) {
			memcpy(ns, s->stage, s->stage_cap);
			hmem_free(s->stage, s->stage_pinned);
		}
		s->stage = ns;
		s->stage_pinned = pinned;
		s->stage_cap = c;
	}
	return 0;
}

/* Host-side masking for parser layers below L4 (odp_parse.c:372-414): the
 * L2 / L3 parts of the full parse are identical at any layer; the layer only
 * cuts what is recorded and whether an L4 truncation drops. */
static void apply_layer(mi_cls_result_t *r, odp_proto_layer_t layer)
{
	/* l2 l3 eth eth_bcast eth_mcast jumbo vlan vlan_qinq */
	const uint32_t L2F = (1u << 3) | (0x3fu << 6);
	/* + l3 arp ipv4 ipv6 ip_bcast ip_mcast ipfrag ipopt */
	const uint32_t L3F = L2F | (1u << 4) | (0x7fu << 12);

	if (layer >= ODP_PROTO_LAYER_L4)
		return;
	/* an L4 truncation does not drop below L4; a drop_ipv4/6_err drop
	 * (ip_err set, L3 options) does */
	if (r->outcome == MI_CLS_OUT_PARSE_DROP && !(layer == ODP_PROTO_LAYER_L3 && (r->err & 0x02)))
		r->outcome = MI_CLS_OUT_DISCARD;
	if (layer == ODP_PROTO_LAYER_L2) {
		r->in_flags &= L2F;
		r->err &= 0x01;     /* snap_len_err */
		r->l4_offset = ODP_PACKET_OFFSET_INVALID;
	} else {
		r->in_flags &= L3F | (1u << 30);   /* + l3_chksum_done */
		r->err &= 0x07;     /* snap_len_err, ip_err, l3_chksum_err */
	}
}

/* Enqueue a run of classified packets (_odp_cos_enq,
 * odp_classification_internal.h:171-201) */
/* Queue slot of dst inside the CoS (_odp_cos_queue_idx,
 * odp_classification_internal.h:49-65): 0 for a single-queue CoS. */
static uint32_t cos_slot_of(uint32_t cos_index, odp_queue_t dst)
{
	odp_cos_t cos = (odp_cos_t)(uintptr_t)(cos_index + 1u);
	uint32_t nq = odp_cls_cos_num_queue(cos), slot = 0;

	if (nq > 1) {
		odp_queue_t qs[32];

		odp_cls_cos_queues(cos, qs, 32);
		for (uint32_t i = 0; i < nq; i++)
			if (qs[i] == dst)
				slot = i;
	}
	return slot;
}

/* _odp_cos_vector_enq (odp_classification_internal.h:83-137): the run goes
 * into ceil(num / max_size) packet vectors, all full but the last; what the
 * vector pool cannot hold is counted as discards.  (The reference leaves the
 * packets it could not place unreferenced; here they are freed.) */
static void cos_vector_enq(odp_queue_t queue, odp_packet_t pk[], int num, uint32_t cos,
			   odp_pool_t vpool, uint32_t max_size)
{
	const uint32_t slot = cos_slot_of(cos, queue);
	int num_pktv = (int)(((uint32_t)num + max_size - 1) / max_size);
	odp_event_t ev[num_pktv];
	odp_packet_vector_t pv[num_pktv];
	int i;

	for (i = 0; i < num_pktv; i++) {
		pv[i] = odp_packet_vector_alloc(vpool);
		if (pv[i] == ODP_PACKET_VECTOR_INVALID)
			break;
		ev[i] = odp_packet_vector_to_event(pv[i]);
	}
	if (i == 0) {
		odp_packet_free_multi(pk, num);
		odp_amd_cls_queue_stats_add(cos, slot, 0, (uint64_t)num);
		return;
	}
	num_pktv = i;
	uint32_t num_enq = 0;

	for (i = 0; i < num_pktv; i++) {
		odp_packet_t *tbl;
		uint32_t sz = max_size;

		if (num_enq + max_size > (uint32_t)num)
			sz = (uint32_t)num - num_enq;
		odp_packet_vector_tbl(pv[i], &tbl);
		memcpy(tbl, &pk[num_enq], sz * sizeof(odp_packet_t));
		odp_packet_vector_size_set(pv[i], sz);
		num_enq += sz;
	}
	if (num_enq < (uint32_t)num)
		odp_packet_free_multi(&pk[num_enq], num - (int)num_enq);
	int ret = odp_queue_enq_multi(queue, ev, num_pktv);

	if (ret == num_pktv) {
		odp_amd_cls_queue_stats_add(cos, slot, num_enq, (uint64_t)num - num_enq);
		return;
	}
	if (ret < 0)
		ret = 0;
	uint32_t enqueued = max_size * (uint32_t)ret;

	odp_amd_cls_queue_stats_add(cos, slot, enqueued, (uint64_t)num - enqueued);
	for (i = ret; i < num_pktv; i++) {
		odp_packet_t *tbl;
		uint32_t sz = odp_packet_vector_tbl(pv[i], &tbl);

		odp_packet_free_multi(tbl, (int)sz);
		odp_packet_vector_free(pv[i]);
	}
}

/* One enqueue run (equal dst_queue and cos): _odp_cos_enq
 * (odp_classification_internal.h:142-167).  Single packets and CoS without
 * packet vectors take the plain enqueue -- to odp_queue_aggr(dst, 0) for a
 * hash-queue CoS with event aggregators -- others go into packet vectors;
 * queue stats are kept on the CoS queue (dst). */
static void cos_enq_run(odp_packet_t pk[], int num)
{
	pkt_hdr_t *h = rt_pkt_hdr(pk[0]);
	const uint32_t cos = h->cos;
	odp_queue_t dst = h->dst_queue;
	odp_pool_t vpool = ODP_POOL_INVALID;
	uint32_t vmax = 0;
	int use_aggr = 0;
	const int std = odp_amd_cls_cos_enq_mode(cos, &vpool, &vmax, &use_aggr);

	if (num < 2 || std != 0) {
		odp_queue_t q = use_aggr ? odp_queue_aggr(dst, 0) : dst;
		int r = q == ODP_QUEUE_INVALID ? -1
			: odp_queue_enq_multi(q, (const odp_event_t *)(void *)pk, num);

		if (r < 0)
			r = 0;
		if (r != num)
			odp_packet_free_multi(&pk[r], num - r);
		odp_amd_cls_queue_stats_add(cos, cos_slot_of(cos, dst), (uint64_t)r,
					    (uint64_t)(num - r));
		return;
	}
	cos_vector_enq(dst, pk, num, cos, vpool, vmax);
}

/* The host's staging of n loop packets already in s->pk: lengths, pools,
 * headrooms, user pointers and the descriptors.  Packets of page-locked
 * pools are classified in place: the descriptors are their data addresses
 * relative to the lowest pinned pool (one base for the burst; the GPU
 * addresses that memory at the host's addresses).  A burst with a packet
 * outside that range is copied into the stage instead.  0, or -1 when the
 * stage cannot grow. */
static int loop_stage_hdrs(rt_pktio_t *e, rx_set_t *s, uint32_t n)
{
	uint8_t *lo = NULL;
	size_t span = 0, off = 0;
	int in_place = s->arr_pinned && rt_pinned_arena(&lo, &span) && span < OOB_SPAN;
	uint8_t pinned_of[RT_MAX_POOLS];

	(void)e;
	for (int k = 0; k < RT_MAX_POOLS; k++) {
		rt_pool_t *rp = rt_pool((odp_pool_t)(uintptr_t)(k + 1));

		pinned_of[k] = rp && rp->pinned;
	}
	/* header prefetch distance (ODP_AMD_LOOP_PF, A/B; 16 -> 96: loop receive
	 * 17.5 -> 20.0 Mpkt/s, profiles/r04pf_loop_prefetch_ab.txt) */
	static int pf = -1;

	if (pf < 0)
		pf = getenv("ODP_AMD_LOOP_PF") ? atoi(getenv("ODP_AMD_LOOP_PF")) : 96;
	for (uint32_t i = 0; i < n; i++) {
		if (i + pf < n) {   /* both header lines (the sender wrote them) */
			const uint8_t *nh = (const uint8_t *)rt_pkt_hdr(s->pk[i + pf]);

			__builtin_prefetch(nh);
			__builtin_prefetch(nh + 64);
		}
		pkt_hdr_t *h = rt_pkt_hdr(s->pk[i]);
		const uint8_t *d = h->head + h->data_off;
		uint32_t l = h->len > 65535 ? 65535 : h->len;
		const uint32_t pi = h->ev.pool;

		s->slen[i] = (uint16_t)l;
		s->ppool[i] = (uint8_t)(pi + 1u);
		s->pdoff[i] = (uint16_t)h->data_off;
		s->pup[i] = h->user_ptr;
		if (in_place && pinned_of[pi] && d >= lo && (size_t)(d - lo) + l + 16u <= span)
			s->soff[i] = (uint32_t)(d - lo);
		else
			in_place = 0;
	}
	if (in_place) {
		s->base = lo;
		s->bytes = span;
		return 0;
	}
	for (uint32_t i = 0; i < n; i++) {
		pkt_hdr_t *h = rt_pkt_hdr(s->pk[i]);
		const uint32_t l = s->slen[i];

		if (stage_reserve(s, n, off + l + 64))
			return -1;
		memcpy(s->stage + off, h->head + h->data_off, l);
		s->soff[i] = (uint32_t)off;
		off += (l + 63u) & ~63u;
	}
	s->base = s->stage;
	s->bytes = off + 64;
	return 0;
}

/* Pull up to `max` frames from the driver into staging set s.  pcap frames
 * in a page-locked frame store are not copied: the set points at the store
 * (the GPU reads them there) and they are copied once, into their packets,
 * at delivery.  Other pcap frames are copied into the stage (64 B aligned
 * offsets) and allocated later, directly from the final pool; loop frames
 * keep their packets in s->pk.  Returns the frame count. */
static int stage_frames(rt_pktio_t *e, rx_set_t *s, uint32_t max)
{
	uint32_t n = 0;
	size_t off = 0;

	if (stage_reserve(s, max, 0))
		return -1;
	s->base = s->stage;
	if (e->drv == DRV_PCAP) {
		/* in place only when the descriptor / record arrays are page-locked
		 * too: otherwise mi_cls stages the whole frame store every burst */
		const int in_place = e->fbuf_pinned && s->arr_pinned;

		if (in_place)
			s->base = e->fbuf;
		while (n < max) {
			if (e->next >= e->nframes) {
				if (e->nframes == 0 || e->eof)
					break;
				/* _pcapif_reopen (pcap.c:257-278): note loop_cnt starts at 1 */
				if (e->loops != 0 && ++e->loop_cnt >= e->loops) {
					e->eof = 1;
					break;
				}
				e->next = 0;
			}
			const uint32_t fo = e->foff[e->next];
			const uint8_t *d = e->fbuf + fo;
			uint16_t l = e->flen[e->next];

			e->next++;
			if (!pcap_filter_pass(e, d, l))
				continue;
			if (in_place) {
				s->soff[n] = fo;
			} else {
				if (stage_reserve(s, max, off + l + 64))
					return -1;
				s->base = s->stage;
				memcpy(s->stage + off, d, l);
				s->soff[n] = (uint32_t)off;
				off += ((uint32_t)l + 63u) & ~63u;
			}
			s->slen[n] = l;
			n++;
		}
		s->bytes = in_place ? e->fbuf_bytes : off + 64;
	} else if (e->drv == DRV_LOOP) {
		/* the receive chain stages the burst on the GPU from the packets'
		 * headers (rxc_submit): only the handles are taken here */
		const int gstage = rxc_loop_stage_ok(e, s, max);

		while (n < max) {
			odp_event_t *ev = (odp_event_t *)(void *)(s->pk + n);
			int want = (int)(max - n);
			int got = rt_queue_deq_multi_raw((rt_queue_t *)(void *)e->loopq, ev, want);

			if (got <= 0)
				break;
			n += (uint32_t)got;
			if (got < want)
				break;
		}
		/* the GPU reads the headers: only of packets in page-locked pools
		 * (a packet of a pool in ordinary memory is staged by the host) */
		s->gstage = gstage && n > 0 && rt_pinned_handles(s->pk, (int)n);
		if (s->gstage) {
			uint8_t *lo = NULL;
			size_t span = 0;

			(void)rt_pinned_arena(&lo, &span);
			s->base = lo;
			s->bytes = span;
		} else if (n > 0 && loop_stage_hdrs(e, s, n)) {
			odp_packet_free_multi(s->pk, (int)n);
			return -1;
		}
	}
	return (int)n;
}

/* more frames ready at the driver right now (a burst in flight can wait) */
static int rx_more(rt_pktio_t *e)
{
	if (e->drv == DRV_PCAP)
		return e->nframes && !e->eof &&
		       (e->next < e->nframes || e->loops == 0 || e->loop_cnt + 1 < e->loops);
	if (e->drv == DRV_LOOP)
		return ((rt_queue_t *)(void *)e->loopq)->count > 0;
	return 0;
}

/* ODP_AMD_RX_PIPELINE=0: classify each burst synchronously */
static int rx_pipeline(void)
{
	static int on = -1;

	if (on < 0) {
		const char *v = getenv("ODP_AMD_RX_PIPELINE");

		on = !(v && v[0] == '0');
	}
	return on;
}

static void rx_drop(rt_pktio_t *e, rx_set_t *s, int rc)
{
	RT_ERR("pktio %s: GPU classify failed (%s), burst of %d dropped\n", e->name,
	       mi_cls_strerror(rc), s->n);
	if (e->drv == DRV_LOOP)
		odp_packet_free_multi(s->pk, s->n);
	odp_atomic_add_u64(&e->in_discards, (uint64_t)s->n);
	s->pending = 0;
}

/* Classify set s: submitted to the GPU (pipelined) or done on return.  On
 * failure the burst is dropped and counted; returns 0 / -1. */
static int rx_classify(rt_pktio_t *e, rx_set_t *s, int pipe)
{
	int rc = 0;

	s->ticket = 0;
	s->pending = 1;
	if (e->parse_layer == ODP_PROTO_LAYER_NONE)
		return 0;
	s->gen = odp_amd_cls_generation();
	if (pipe)
		rc = odp_amd_cls_classify_host_submit(e->hdl, s->base, s->bytes, s->soff, s->slen,
						      (uint32_t)s->n, s->res, &s->ticket);
	else
		rc = odp_amd_cls_classify_host(e->hdl, s->base, s->bytes, s->soff, s->slen,
					       (uint32_t)s->n, s->res, !e->cls_enabled);
	if (rc) {
		rx_drop(e, s, rc);
		return -1;
	}
	return 0;
}

/* The host steps of loopback_recv / pcapif_recv_pkt for frames [lo, hi) of
 * set s (loop.c:253-384, pcap.c:299-352; _odp_packet_parse_common's result
 * applied at the pktio's layer, _odp_cls_classify_packet's outcome, the
 * packet in its final pool, _odp_pktio_packet_to_pool): s->pk[i] becomes the
 * packet to deliver, or ODP_PACKET_INVALID.  (Preparing chunks of a burst on
 * helper threads measured slower -- 14.3 -> 6.4 Mpkt/s with four helpers,
 * profiles/r03g_rx_helpers_ab.txt: each packet's header line then moves between cores
 * on its way to the queue and the consumer -- so one thread does it.) */
static void rx_prepare_each(rt_pktio_t *e, rx_set_t *s, int lo, int hi, rx_cnt_t *c)
{
	const odp_proto_layer_t layer = e->parse_layer;

	for (int i = lo; i < hi; i++) {
		mi_cls_result_t r;
		odp_packet_t pkt = e->drv == DRV_LOOP ? s->pk[i] : ODP_PACKET_INVALID;
		uint32_t len = s->slen[i];

		s->pk[i] = ODP_PACKET_INVALID;
		if (i + 16 < hi)    /* records written by the GPU: not in the CPU caches */
			__builtin_prefetch(&s->res[i + 16]);
		if (i + 8 < hi) {   /* frames read in place are cold in the CPU caches */
			const uint8_t *nf = s->base + s->soff[i + 8];
			const uint32_t nl = s->slen[i + 8];

			for (uint32_t b = 0; b < nl; b += 64)
				__builtin_prefetch(nf + b);
		}
		if (layer != ODP_PROTO_LAYER_NONE) {
			r = s->res[i];
			apply_layer(&r, layer);
			if (r.err || r.outcome == MI_CLS_OUT_PARSE_DROP)
				c->in_errors++;
			if (r.outcome == MI_CLS_OUT_PARSE_DROP) {
				odp_packet_free(pkt);
				continue;
			}
		} else {
			memset(&r, 0, sizeof(r));
			r.cos = 0xff;
		}
		odp_pool_t pool = e->pool;

		if (e->cls_enabled) {
			if (r.outcome == MI_CLS_OUT_DISCARD || r.outcome == MI_CLS_OUT_LOOP)
				c->in_discards++;
			if (r.outcome != MI_CLS_OUT_ENQ) {
				odp_packet_free(pkt);
				continue;
			}
			odp_pool_t cp = odp_amd_cls_pool_of(r.cos);

			if (cp != ODP_POOL_INVALID)
				pool = cp;
		}
		/* packet in the final pool (_odp_pktio_packet_to_pool) */
		if (pkt == ODP_PACKET_INVALID) {
			const uint64_t ta = rx_prof > 0 ? __rdtsc() : 0;

			pkt = odp_packet_alloc(pool, len);
			if (pkt == ODP_PACKET_INVALID) {
				if (e->cls_enabled)
					c->in_discards++;
				continue;
			}
			const uint64_t tb = rx_prof > 0 ? __rdtsc() : 0;

			memcpy(odp_packet_data(pkt), s->base + s->soff[i], len);
			if (rx_prof > 0) {
				e->prof[6] += tb - ta;
				e->prof[7] += __rdtsc() - tb;
			}
		} else if (odp_packet_pool(pkt) != pool) {
			odp_packet_t np = odp_packet_alloc(pool, len);

			if (np == ODP_PACKET_INVALID) {
				odp_packet_free(pkt);
				c->in_discards++;
				continue;
			}
			pkt_hdr_t *sh = rt_pkt_hdr(pkt);

			memcpy(odp_packet_data(np), sh->head + sh->data_off, len);
			rt_pkt_hdr(np)->user_ptr = sh->user_ptr;
			odp_packet_free(pkt);
			pkt = np;
		}
		pkt_hdr_t *h = rt_pkt_hdr(pkt);

		if (layer != ODP_PROTO_LAYER_NONE) {
			h->in_flags = r.in_flags;
			h->err = r.err;
			h->l2 = 0;
			h->l3 = r.l3_offset;
			h->l4 = r.l4_offset;
		} else {
			h->in_flags = 0;
			h->err = 0;
		}
		h->input = e->hdl;
		if (!h->err) {
			c->octets += len;
			c->packets++;
		}
		if (e->cls_enabled) {
			h->cos = r.cos;
			h->cls_mark = r.mark;
			h->dst_queue = odp_amd_cls_queue_of(r.cos, r.queue);
		}
		s->pk[i] = pkt;
	}
}


/* Packet metadata of a delivered frame from its record. */
static inline void rx_fill(rt_pktio_t *e, pkt_hdr_t *h, const mi_cls_result_t *r, uint32_t len,
			   rx_cnt_t *c)
{
	if (e->parse_layer != ODP_PROTO_LAYER_NONE) {
		h->in_flags = r->in_flags;
		h->err = r->err;
		h->l2 = 0;
		h->l3 = r->l3_offset;
		h->l4 = r->l4_offset;
	} else {
		h->in_flags = 0;
		h->err = 0;
	}
	h->input = e->hdl;
	if (!h->err) {
		c->octets += len;
		c->packets++;
	}
	if (e->cls_enabled) {
		h->cos = r->cos;
		h->cls_mark = r->mark;
		h->dst_queue = odp_amd_cls_queue_of(r->cos, r->queue);
	}
}

/* rx_prepare for pcap frames: the same steps in three passes, so packets
 * are taken from each pool in bulk and their headers prefetched before they
 * are written (a per-frame odp_packet_alloc spent most of its time on the
 * cold header line).  Pass 1 decides each frame (parse drop, CoS discard, or
 * the pool it goes to), pass 2 takes every pool's packets at once -- frames
 * of one pool get them in arrival order, so when a pool runs short the same
 * frames are discarded as frame-by-frame allocation would -- and pass 3
 * initialises the headers, copies the frames and writes the metadata.
 * `slot` (one byte per frame) and `got` (n_cap packets) are the set's
 * delivery scratch; more than RX_MAX_POOLS distinct pools in a burst fall
 * back to rx_prepare_each. */
#define RX_MAX_POOLS 16
static void rx_prepare(rt_pktio_t *e, rx_set_t *s, int lo, int hi, rx_cnt_t *c)
{
	const odp_proto_layer_t layer = e->parse_layer;
	uint8_t *slot = s->tmp ? (uint8_t *)(void *)(s->tmp + s->tmp_cap) : NULL;
	odp_packet_t *got = s->tmp;
	struct {
		odp_pool_t pool;
		uint32_t cap;
		int cnt, base, have, used;
	} pl[RX_MAX_POOLS];
	int npl = 0;

	if (e->drv != DRV_PCAP || !slot) {
		rx_prepare_each(e, s, lo, hi, c);
		return;
	}
	/* pass 1: the decision per frame */
	for (int i = lo; i < hi; i++) {
		if (i + 16 < hi)
			__builtin_prefetch(&s->res[i + 16]);
		mi_cls_result_t r;
		const uint32_t len = s->slen[i];

		s->pk[i] = ODP_PACKET_INVALID;
		slot[i] = 0xff;
		if (layer != ODP_PROTO_LAYER_NONE) {
			r = s->res[i];
			apply_layer(&r, layer);
			if (r.err || r.outcome == MI_CLS_OUT_PARSE_DROP)
				c->in_errors++;
			if (r.outcome == MI_CLS_OUT_PARSE_DROP)
				continue;
		} else {
			memset(&r, 0, sizeof(r));
		}
		odp_pool_t pool = e->pool;

		if (e->cls_enabled) {
			if (r.outcome == MI_CLS_OUT_DISCARD || r.outcome == MI_CLS_OUT_LOOP)
				c->in_discards++;
			if (r.outcome != MI_CLS_OUT_ENQ)
				continue;
			odp_pool_t cp = odp_amd_cls_pool_of(r.cos);

			if (cp != ODP_POOL_INVALID)
				pool = cp;
		}
		int k = 0;

		while (k < npl && pl[k].pool != pool)
			k++;
		if (k == npl) {
			rt_pool_t *rp = rt_pool(pool);

			if (npl == RX_MAX_POOLS) {   /* start over frame by frame */
				memset(c, 0, sizeof(*c));
				rx_prepare_each(e, s, lo, hi, c);
				return;
			}
			pl[k].pool = pool;
			pl[k].cap = rp && rp->param.type == ODP_POOL_PACKET ? rp->data_cap : 0u;
			pl[k].cnt = 0;
			npl++;
		}
		if (len > pl[k].cap) {   /* odp_packet_alloc fails: no packet taken */
			if (e->cls_enabled)
				c->in_discards++;
			continue;
		}
		slot[i] = (uint8_t)k;
		pl[k].cnt++;
	}
	/* pass 2: each pool's packets at once */
	int at = lo;

	for (int k = 0; k < npl; k++) {
		pl[k].base = at;
		pl[k].have = pl[k].cnt ? rt_packet_alloc_raw(pl[k].pool, 0, &got[at], pl[k].cnt) : 0;
		pl[k].used = 0;
		at += pl[k].cnt;
	}
	/* pass 3: headers, frames, metadata */
	for (int i = lo; i < hi; i++) {
		if (i + 8 < hi) {   /* frames read in place are cold in the CPU caches */
			const uint8_t *nf = s->base + s->soff[i + 8];
			const uint32_t nl = s->slen[i + 8];

			for (uint32_t b = 0; b < nl; b += 64)
				__builtin_prefetch(nf + b);
		}
		const int k = slot[i];

		if (k == 0xff)
			continue;
		const int j = pl[k].used++;

		if (j >= pl[k].have) {   /* the pool ran short */
			if (e->cls_enabled)
				c->in_discards++;
			continue;
		}
		if (j + 4 < pl[k].have) {   /* a later packet of this pool: its header */
			const pkt_hdr_t *nh = rt_pkt_hdr(got[pl[k].base + j + 4]);

			/* the buffer follows the 64-B aligned header (odp_rt.c pool
			 * layout): its first data line, without reading the header */
			__builtin_prefetch(nh, 1);
			__builtin_prefetch((const uint8_t *)nh + ((sizeof(pkt_hdr_t) + 63u) & ~(size_t)63u) +
					   RT_PKT_HEADROOM, 1);
		}
		const odp_packet_t pkt = got[pl[k].base + j];
		const uint32_t len = s->slen[i];
		mi_cls_result_t r;

		if (layer != ODP_PROTO_LAYER_NONE) {
			r = s->res[i];
			apply_layer(&r, layer);
		} else {
			memset(&r, 0, sizeof(r));
			r.cos = 0xff;
		}
		const uint64_t ta = rx_prof > 0 ? __rdtsc() : 0;

		rt_packet_init(pkt, len);
		const uint64_t tb = rx_prof > 0 ? __rdtsc() : 0;

		memcpy(odp_packet_data(pkt), s->base + s->soff[i], len);
		if (rx_prof > 0) {
			e->prof[6] += tb - ta;
			e->prof[7] += __rdtsc() - tb;
		}
		rx_fill(e, rt_pkt_hdr(pkt), &r, len, c);
		s->pk[i] = pkt;
	}
}

/* Enqueue the delivered packets pk[0..n) in arrival order.  _odp_cls_enq
 * (odp_classification_internal.h:171-201) enqueues runs of equal
 * (dst_queue, CoS); when every run of the burst takes the plain enqueue (no
 * packet vectors, no aggregator), the runs of one queue are joined into one
 * enqueue call per queue instead -- each queue still receives its packets in
 * arrival order, and nothing outside the burst can tell the two apart (the
 * whole burst is enqueued before the receive call returns).  Per-CoS queue
 * statistics are kept as per run.  Runs of CoS with packet vectors or
 * aggregators keep the reference's per-run form (their vector boundaries
 * depend on it). */
#define RX_GROUP_MAXQ 64
#define RX_GROUP_HASH 256      /* open-addressing slots: queue -> group */
static inline uint32_t rx_qhash(odp_queue_t q)
{
	const uint64_t x = (uint64_t)(uintptr_t)q * 0x9E3779B97F4A7C15ull;

	return (uint32_t)(x >> 56);   /* 8 bits: RX_GROUP_HASH slots */
}

static void rx_enqueue(odp_packet_t pk[], int n, odp_packet_t *tmp, uint8_t *gidx)
{
	struct {
		odp_queue_t q;
		int cnt, fill;
	} g[RX_GROUP_MAXQ];
	int ng = 0, plain = 1;
	int8_t mode_of_cos[256];   /* 1 plain, 0 not, -1 unknown */
	uint8_t slot_grp[RX_GROUP_HASH];   /* group + 1, 0 empty */

	memset(mode_of_cos, -1, sizeof(mode_of_cos));
	memset(slot_grp, 0, sizeof(slot_grp));
	for (int i = 0; i < n; i++) {
		pkt_hdr_t *h = rt_pkt_hdr(pk[i]);
		const uint32_t cos = h->cos & 0xffu;

		if (mode_of_cos[cos] < 0) {
			odp_pool_t vp = ODP_POOL_INVALID;
			uint32_t vmax = 0;
			int aggr = 0;
			const int std = odp_amd_cls_cos_enq_mode(cos, &vp, &vmax, &aggr);

			mode_of_cos[cos] = std > 0 && !aggr;
		}
		if (!mode_of_cos[cos]) {
			plain = 0;
			break;
		}
		uint32_t sl = rx_qhash(h->dst_queue);

		while (slot_grp[sl] && g[slot_grp[sl] - 1].q != h->dst_queue)
			sl = (sl + 1) & (RX_GROUP_HASH - 1);
		if (!slot_grp[sl]) {
			if (ng == RX_GROUP_MAXQ) {
				plain = 0;
				break;
			}
			g[ng].q = h->dst_queue;
			g[ng].cnt = 0;
			slot_grp[sl] = (uint8_t)++ng;
		}
		gidx[i] = (uint8_t)(slot_grp[sl] - 1);
		g[slot_grp[sl] - 1].cnt++;
	}
	if (!plain) {
		/* the reference's form: one enqueue per run */
		int nrun = 0;

		for (int i = 0; i < n; i++) {
			if (nrun) {
				pkt_hdr_t *ph = rt_pkt_hdr(pk[i - 1]), *h = rt_pkt_hdr(pk[i]);

				if (ph->dst_queue != h->dst_queue || ph->cos != h->cos) {
					cos_enq_run(&pk[i - nrun], nrun);
					nrun = 0;
				}
			}
			nrun++;
		}
		if (nrun)
			cos_enq_run(&pk[n - nrun], nrun);
		return;
	}
	/* counting sort by queue, stable: each group's packets in arrival order */
	int at = 0;

	for (int k = 0; k < ng; k++) {
		g[k].fill = at;
		at += g[k].cnt;
	}
	for (int i = 0; i < n; i++)
		tmp[g[gidx[i]].fill++] = pk[i];
	at = 0;
	for (int k = 0; k < ng; k++) {
		odp_packet_t *gp = tmp + at;
		const int num = g[k].cnt;
		int r = odp_queue_enq_multi(g[k].q, (const odp_event_t *)(void *)gp, num);

		at += num;
		if (r < 0)
			r = 0;
		if (r != num)
			odp_packet_free_multi(&gp[r], num - r);
		/* queue statistics as per run of the reference: per CoS of the queue */
		int done = 0;

		for (int j = 0; j < num && done < num; j++) {
			const uint32_t cos = rt_pkt_hdr(gp[j])->cos;
			int first = 1;

			for (int t = 0; t < j && first; t++)
				first = rt_pkt_hdr(gp[t])->cos != cos;
			if (!first)
				continue;
			uint64_t ok = 0, bad = 0;

			for (int t = j; t < num; t++)
				if (rt_pkt_hdr(gp[t])->cos == cos) {
					if (t < r)
						ok++;
					else
						bad++;
				}
			done += (int)(ok + bad);
			odp_amd_cls_queue_stats_add(cos, cos_slot_of(cos, g[k].q), ok, bad);
		}
	}
}

/* ODP_AMD_RX_GPU_DELIVER=0: host delivery only */
static int gpu_deliver_on(void)
{
	static int on = -1;

	if (on < 0) {
		const char *v = getenv("ODP_AMD_RX_GPU_DELIVER");

		on = !(v && v[0] == '0');
	}
	return on;
}

/* Enqueue the grouped packets of a GPU delivery: group g (queue gq[g]) holds
 * entries perm[at .. at + gcnt[g]) in arrival order; queue statistics per
 * CoS of the queue as per run of the reference. */
static void rx_enqueue_groups(rx_set_t *s, const odp_queue_t *gq, int ng, odp_packet_t *tmp)
{
	uint32_t at = 0;

	for (int g = 0; g < ng; g++) {
		const uint32_t num = s->gcnt[g];
		uint64_t ok[256], bad[256];
		uint8_t seen[256];
		int ncos = 0;
		uint8_t cl[256];

		if (!num)
			continue;
		for (uint32_t k = 0; k < num; k++)
			tmp[k] = s->ent[s->perm[at + k]];
		int r = odp_queue_enq_multi(gq[g], (const odp_event_t *)(void *)tmp, (int)num);

		if (r < 0)
			r = 0;
		if ((uint32_t)r != num)
			odp_packet_free_multi(&tmp[r], (int)num - r);
		memset(seen, 0, sizeof(seen));
		for (uint32_t k = 0; k < num; k++) {
			const uint32_t cos = s->res[s->dlv[s->perm[at + k]].rec].cos;

			if (!seen[cos]) {
				seen[cos] = 1;
				cl[ncos++] = (uint8_t)cos;
				ok[cos] = 0;
				bad[cos] = 0;
			}
			if (k < (uint32_t)r)
				ok[cos]++;
			else
				bad[cos]++;
		}
		for (int k = 0; k < ncos; k++)
			odp_amd_cls_queue_stats_add(cl[k], cos_slot_of(cl[k], gq[g]), ok[cl[k]],
						    bad[cl[k]]);
		at += num;
	}
}

/* Delivery of set s on the GPU (mi_cls_deliver_submit): the host decides
 * every frame from its record (parse drop, CoS drop / discard, destination
 * pool: the same decisions and counters as rx_prepare), takes the packets
 * from each pool at once, and hands the GPU one entry per delivered packet;
 * the GPU writes the packets' metadata, copies frames that change buffers
 * (pcap frames, loop packets switching pools) and groups the packets by
 * queue; the host then enqueues each queue's packets with one call.  The
 * host touches no packet header or frame byte on this path.  This starts
 * it: the decisions, the packets, the entries, the kernel submitted (the set
 * is then `delivering` until rx_dlv_end).  Returns 0, or -1 when the burst
 * needs the host path (a destination pool not page-locked, more than
 * RX_MAX_POOLS pools, frames the GPU cannot address) -- nothing has been
 * done then. */
static int rx_dlv_start(rt_pktio_t *e, rx_set_t *s, rx_cnt_t *c)
{
	const odp_proto_layer_t layer = e->parse_layer;
	uint8_t *slot = s->tmp ? (uint8_t *)(void *)(s->tmp + s->tmp_cap) : NULL;
	odp_packet_t *got = s->tmp;
	struct {
		odp_pool_t pool;
		uint32_t cap;
		int cnt, base, have, used;
	} pl[RX_MAX_POOLS];
	int npl = 0;
	enum { A_NONE = 0xff, A_INPLACE = 0xfe };   /* else: index of the pool */

	if (!gpu_deliver_on() || !s->dlv_pinned || !slot || layer == ODP_PROTO_LAYER_NONE ||
	    !mi_cls_host_mapped(s->base))
		return -1;
	const uint64_t td0 = prof_ns();
	s->dgen = odp_amd_cls_generation();
	/* per-burst caches of the CoS lookups (pool, queue of slot 0) */
	odp_pool_t cpool[256];
	odp_queue_t cq0[256];
	uint8_t cseen[256];

	memset(cseen, 0, sizeof(cseen));
#define COS_SEEN(cos)                                                                  \
	do {                                                                           \
		if (!cseen[cos]) {                                                     \
			cseen[cos] = 1;                                                \
			cpool[cos] = odp_amd_cls_pool_of(cos);                         \
			cq0[cos] = odp_amd_cls_queue_of(cos, 0);                       \
		}                                                                      \
	} while (0)
	/* pass 1: the decision per frame, no side effects yet */
	for (int i = 0; i < s->n; i++) {
		mi_cls_result_t r = s->res[i];
		odp_pool_t pool = e->pool;

		if (i + 16 < s->n)
			__builtin_prefetch(&s->res[i + 16]);
		slot[i] = A_NONE;
		apply_layer(&r, layer);
		if (r.outcome == MI_CLS_OUT_PARSE_DROP)
			continue;
		if (e->cls_enabled) {
			if (r.outcome != MI_CLS_OUT_ENQ)
				continue;
			COS_SEEN(r.cos);
			if (cpool[r.cos] != ODP_POOL_INVALID)
				pool = cpool[r.cos];
		}
		if (e->drv == DRV_LOOP && (odp_pool_t)(uintptr_t)s->ppool[i] == pool) {
			/* the GPU writes the packet's own header */
			if (!rt_pool(pool)->pinned)
				return -1;
			slot[i] = A_INPLACE;
			continue;
		}
		int k = 0;

		while (k < npl && pl[k].pool != pool)
			k++;
		if (k == npl) {
			rt_pool_t *rp = rt_pool(pool);

			if (npl == RX_MAX_POOLS || !rp || !rp->pinned)
				return -1;
			pl[k].pool = pool;
			pl[k].cap = rp->param.type == ODP_POOL_PACKET ? rp->data_cap : 0u;
			pl[k].cnt = 0;
			npl++;
		}
		if (s->slen[i] > pl[k].cap)   /* odp_packet_alloc fails: discarded */
			continue;
		slot[i] = (uint8_t)k;
		pl[k].cnt++;
	}
	/* pass 2: each pool's packets at once */
	int at = 0;

	for (int k = 0; k < npl; k++) {
		pl[k].base = at;
		pl[k].have = pl[k].cnt ? rt_packet_alloc_raw(pl[k].pool, 0, &got[at], pl[k].cnt) : 0;
		pl[k].used = 0;
		at += pl[k].cnt;
	}
	/* pass 3: counters, drops, entries (queue groups: every plain-enqueue
	 * queue of the burst, at most MI_CLS_DLV_GROUPS) */
	odp_queue_t gq[MI_CLS_DLV_GROUPS];
	int ng = 0, grouped = e->cls_enabled, nold = 0;
	int8_t mode_of_cos[256];
	uint8_t slot_grp[RX_GROUP_HASH];
	uint32_t ne = 0;

	memset(mode_of_cos, -1, sizeof(mode_of_cos));
	memset(slot_grp, 0, sizeof(slot_grp));
	for (int i = 0; i < s->n; i++) {
		mi_cls_result_t r = s->res[i];
		const uint32_t len = s->slen[i];
		const int k = slot[i];
		odp_packet_t pkt = e->drv == DRV_LOOP ? s->pk[i] : ODP_PACKET_INVALID;

		s->pk[i] = ODP_PACKET_INVALID;
		apply_layer(&r, layer);
		if (r.err || r.outcome == MI_CLS_OUT_PARSE_DROP)
			c->in_errors++;
		if (r.outcome == MI_CLS_OUT_PARSE_DROP) {
			odp_packet_free(pkt);
			continue;
		}
		if (e->cls_enabled && (r.outcome == MI_CLS_OUT_DISCARD || r.outcome == MI_CLS_OUT_LOOP))
			c->in_discards++;
		if (e->cls_enabled && r.outcome != MI_CLS_OUT_ENQ) {
			odp_packet_free(pkt);
			continue;
		}
		uint8_t fl = MI_CLS_DLV_FRESH | MI_CLS_DLV_COPY;
		odp_packet_t dst;

		if (k == A_INPLACE) {
			dst = pkt;
			fl = 0;
		} else if (k == A_NONE || pl[k].used >= pl[k].have) {
			/* too long for the pool, or the pool ran short (a loop
			 * packet's failed pool switch is a discard either way) */
			if (k != A_NONE)
				pl[k].used++;
			if (e->cls_enabled || pkt != ODP_PACKET_INVALID)
				c->in_discards++;
			odp_packet_free(pkt);
			continue;
		} else {
			dst = got[pl[k].base + pl[k].used++];
			if (pkt != ODP_PACKET_INVALID)
				s->old[nold++] = pkt;   /* freed once the GPU copied it */
		}
		if (!r.err) {
			c->octets += len;
			c->packets++;
		}
		mi_cls_dlv_t *d = &s->dlv[ne];
		uint8_t qid = 0xff;

		d->meta = (uint64_t)(uintptr_t)&rt_pkt_hdr(dst)->meta;
		d->data_off = k == A_INPLACE ? s->pdoff[i] : RT_PKT_HEADROOM;
		/* the metadata line is written whole: a packet received in place
		 * keeps its user pointer (read with its headroom at staging) */
		d->user_ptr = k == A_INPLACE ? (uint64_t)(uintptr_t)s->pup[i] : 0u;
		d->dst_queue = 0;
		d->src = s->soff[i];
		d->rec = (uint32_t)i;
		d->len = (uint16_t)len;
		if (e->cls_enabled) {
			const odp_queue_t q = r.queue == 0 ? cq0[r.cos] : odp_amd_cls_queue_of(r.cos, r.queue);

			fl |= MI_CLS_DLV_CLS;
			d->dst_queue = (uint64_t)(uintptr_t)q;
			if (grouped && mode_of_cos[r.cos] < 0) {
				odp_pool_t vp = ODP_POOL_INVALID;
				uint32_t vmax = 0;
				int aggr = 0;
				const int std = odp_amd_cls_cos_enq_mode(r.cos, &vp, &vmax, &aggr);

				mode_of_cos[r.cos] = std > 0 && !aggr;
			}
			if (grouped && mode_of_cos[r.cos]) {
				uint32_t sl = rx_qhash(q);

				while (slot_grp[sl] && gq[slot_grp[sl] - 1] != q)
					sl = (sl + 1) & (RX_GROUP_HASH - 1);
				if (!slot_grp[sl]) {
					if (ng == MI_CLS_DLV_GROUPS) {
						grouped = 0;
					} else {
						gq[ng] = q;
						slot_grp[sl] = (uint8_t)++ng;
					}
				}
				if (grouped)
					qid = (uint8_t)(slot_grp[sl] - 1);
			} else {
				grouped = 0;
			}
		}
		d->flags = fl;
		d->qid = qid;
		s->ent[ne++] = dst;
	}
#undef COS_SEEN
	/* the pools' packets nobody took back */
	for (int k = 0; k < npl; k++)
		if (pl[k].used < pl[k].have)
			odp_packet_free_multi(&got[pl[k].base + pl[k].used], pl[k].have - pl[k].used);
	if (ne > MI_CLS_DLV_GROUP_MAX)   /* larger than the device grouping serves */
		grouped = 0;
	if (!grouped)   /* per-run enqueue (vectors, aggregators, > 64 queues) */
		for (uint32_t j = 0; j < ne; j++)
			s->dlv[j].qid = 0xff;
	s->ne = ne;
	s->nold = nold;
	s->grouped = grouped;
	s->ng = ng;
	memcpy(s->gq, gq, (size_t)ng * sizeof(odp_queue_t));
	s->cnt = *c;
	s->dticket = 0;
	s->delivering = 1;
	e->prof[8] += prof_ns() - td0;
	e->prof[11]++;
	if (ne) {
		mi_cls_dlv_args_t a;

		a.base = s->base;
		a.res = s->res;
		a.dlv = s->dlv;
		a.n = ne;
		a.layer = (uint32_t)layer;
		a.input = (uint64_t)(uintptr_t)e->hdl;
		a.headroom = RT_PKT_HEADROOM;
		a.data_from_meta = rt_data_from_meta();
		a.perm = s->perm;
		a.gcnt = s->gcnt;
		s->dticket = 0;
		const uint64_t ts0 = prof_ns();
		int rc = odp_amd_cls_deliver(e->hdl, &a, &s->dticket);

		e->prof[12] += prof_ns() - ts0;

		if (rc) {
			s->dticket = 0;
			s->derr = rc;   /* rx_dlv_end drops the packets */
		}
	}
	return 0;
}

/* The control plane changed while set s's GPU delivery was in flight: its
 * packets' CoS, queues and pools were settled under the old tables, and a
 * queue destroyed since may have had its slot reused by a new one.  The burst
 * is classified again under the current tables and each delivered packet
 * re-resolved from its new record -- what a receive call made after the
 * change delivers: a packet whose outcome is no longer an enqueue is freed
 * (CoS discards counted, and it leaves in_packets / in_octets), one whose CoS
 * pool changed is copied into that pool, and every packet takes its CoS, mark
 * and queue from the new record.  The burst is then enqueued per run. */
static void rx_dlv_regen(rt_pktio_t *e, rx_set_t *s, rx_cnt_t *c)
{
	const odp_proto_layer_t layer = e->parse_layer;
	uint32_t m = 0;
	int rc = odp_amd_cls_classify_host(e->hdl, s->base, s->bytes, s->soff, s->slen, (uint32_t)s->n,
					   s->res, 0);

	s->grouped = 0;
	if (rc) {
		RT_ERR("pktio %s: GPU classify failed (%s), %u packets dropped\n", e->name,
		       mi_cls_strerror(rc), s->ne);
		odp_packet_free_multi(s->ent, (int)s->ne);
		c->in_discards += s->ne;
		s->ne = 0;
		return;
	}
	for (uint32_t j = 0; j < s->ne; j++) {
		odp_packet_t pkt = s->ent[j];
		mi_cls_result_t r = s->res[s->dlv[j].rec];
		const uint32_t len = s->dlv[j].len;

		apply_layer(&r, layer);
		if (r.outcome != MI_CLS_OUT_ENQ) {
			if (r.outcome == MI_CLS_OUT_DISCARD || r.outcome == MI_CLS_OUT_LOOP)
				c->in_discards++;
			if (!r.err) {
				c->packets--;
				c->octets -= len;
			}
			odp_packet_free(pkt);
			continue;
		}
		odp_pool_t pool = odp_amd_cls_pool_of(r.cos);

		if (pool == ODP_POOL_INVALID)
			pool = e->pool;
		if (odp_packet_pool(pkt) != pool) {
			/* _odp_pktio_packet_to_pool under the new CoS */
			odp_packet_t np = odp_packet_alloc(pool, len);

			if (np == ODP_PACKET_INVALID) {
				c->in_discards++;
				if (!r.err) {
					c->packets--;
					c->octets -= len;
				}
				odp_packet_free(pkt);
				continue;
			}
			pkt_hdr_t *oh = rt_pkt_hdr(pkt), *nh = rt_pkt_hdr(np);

			memcpy(odp_packet_data(np), oh->head + oh->data_off, len);
			nh->in_flags = oh->in_flags;
			nh->err = oh->err;
			nh->l2 = oh->l2;
			nh->l3 = oh->l3;
			nh->l4 = oh->l4;
			nh->input = oh->input;
			nh->user_ptr = oh->user_ptr;
			odp_packet_free(pkt);
			pkt = np;
		}
		pkt_hdr_t *h = rt_pkt_hdr(pkt);

		h->in_flags = r.in_flags;
		h->cos = r.cos;
		h->cls_mark = r.mark;
		h->dst_queue = odp_amd_cls_queue_of(r.cos, r.queue);
		s->ent[m++] = pkt;
	}
	s->ne = m;
}

/* End the GPU delivery of set s (rx_dlv_start): wait for the kernel, give
 * pool-switched packets their user pointers, enqueue (classifier on) or
 * return the packets in out[] (at most max_out), add the counters.
 * Returns the packets placed in out[]. */
static int rxc_end(rt_pktio_t *e, rx_set_t *s, odp_packet_t out[], int max_out);

static int rx_dlv_end(rt_pktio_t *e, rx_set_t *s, odp_packet_t out[], int max_out)
{
	if (s->chain)
		return rxc_end(e, s, out, max_out);
	const uint64_t tk0 = prof_ns();
	rx_cnt_t *c = &s->cnt;
	int num_rx = 0, rc = s->derr;

	if (!rc && s->dticket)
		rc = odp_amd_cls_deliver_wait(e->hdl, s->dticket);
	s->delivering = 0;
	s->dticket = 0;
	s->derr = 0;
	if (rc) {
		RT_ERR("pktio %s: GPU delivery failed (%s), %u packets dropped\n", e->name,
		       mi_cls_strerror(rc), s->ne);
		odp_packet_free_multi(s->ent, (int)s->ne);
		odp_packet_free_multi(s->old, s->nold);
		c->in_discards += s->ne;
		s->ne = 0;
		s->nold = 0;
	}
	/* pool switch: the new packet keeps the user pointer */
	if (s->nold) {
		int o = 0;

		for (uint32_t j = 0; j < s->ne && o < s->nold; j++)
			if (s->dlv[j].flags & MI_CLS_DLV_FRESH)
				rt_pkt_hdr(s->ent[j])->user_ptr = rt_pkt_hdr(s->old[o++])->user_ptr;
		odp_packet_free_multi(s->old, s->nold);
		s->nold = 0;
	}
	if (e->cls_enabled && s->ne && s->dgen != odp_amd_cls_generation())
		rx_dlv_regen(e, s, c);
	const uint64_t tk1 = prof_ns();

	if (!e->cls_enabled) {
		for (uint32_t j = 0; j < s->ne; j++) {
			if (num_rx < max_out)
				out[num_rx++] = s->ent[j];
			else
				odp_packet_free(s->ent[j]);
		}
	} else if (s->grouped) {
		rx_enqueue_groups(s, s->gq, s->ng, s->tmp);
	} else if (s->ne) {
		rx_enqueue(s->ent, (int)s->ne, s->tmp, (uint8_t *)(void *)(s->tmp + s->tmp_cap));
	}
	s->ne = 0;
	e->prof[9] += tk1 - tk0;
	e->prof[10] += prof_ns() - tk1;
	if (c->in_errors)
		odp_atomic_add_u64(&e->in_errors, c->in_errors);
	if (c->in_discards)
		odp_atomic_add_u64(&e->in_discards, c->in_discards);
	odp_atomic_add_u64(&e->in_octets, c->octets);
	odp_atomic_add_u64(&e->in_packets, c->packets);
	return num_rx;
}

/* Delivery of set s on the host: rx_prepare, then the delivered packets,
 * compacted in arrival order, to their queues or out[]. */
static int rx_deliver_host(rt_pktio_t *e, rx_set_t *s, rx_cnt_t *c, odp_packet_t out[], int max_out,
			   uint64_t t2)
{
	int nd = 0, num_rx = 0;

	rx_prepare(e, s, 0, s->n, c);
	const uint64_t t3 = prof_ns();

	e->prof[4] += t3 - t2;
	for (int i = 0; i < s->n; i++)
		if (s->pk[i] != ODP_PACKET_INVALID)
			s->pk[nd++] = s->pk[i];
	if (e->cls_enabled) {
		if (s->tmp) {
			rx_enqueue(s->pk, nd, s->tmp, (uint8_t *)(void *)(s->tmp + s->tmp_cap));
		} else {
			for (int i = 0; i < nd; i++)
				cos_enq_run(&s->pk[i], 1);
		}
	} else {
		for (int i = 0; i < nd; i++) {
			if (num_rx < max_out)
				out[num_rx++] = s->pk[i];
			else
				odp_packet_free(s->pk[i]);
		}
	}
	e->prof[5] += prof_ns() - t3;
	return num_rx;
}

/* Wait for set s's records and deliver its packets: classified ones to their
 * CoS queues, the rest (classifier disabled) into out[] (at most max_out).
 * Returns the packets placed in out[]. */
/* Wait for set s's classification; a burst that was in flight while the
 * control plane changed is classified again.  Returns 0, or -1 when the
 * burst was dropped (rx_drop). */
static int rx_classified(rt_pktio_t *e, rx_set_t *s)
{
	const odp_proto_layer_t layer = e->parse_layer;
	uint64_t t1 = prof_ns();

	if (s->ticket) {
		int rc = odp_amd_cls_classify_host_wait(e->hdl, s->ticket);

		s->ticket = 0;
		if (rc) {
			rx_drop(e, s, rc);
			return -1;
		}
	}
	/* The control plane changed while the burst was in flight (a CoS
	 * destroyed, its queues or pool changed, PMRs added or removed): its
	 * records name CoS indexes of the old rule snapshot, so classify it again
	 * under the current one -- what the synchronous path, which has no gap
	 * between classify and enqueue, would deliver on this call. */
	if (layer != ODP_PROTO_LAYER_NONE && e->cls_enabled && s->gen != odp_amd_cls_generation()) {
		int rc = odp_amd_cls_classify_host(e->hdl, s->base, s->bytes, s->soff, s->slen,
						   (uint32_t)s->n, s->res, 0);

		if (rc) {
			rx_drop(e, s, rc);
			return -1;
		}
	}
	e->prof[1] += prof_ns() - t1;
	s->pending = 0;
	if (!s->tmp || s->tmp_cap < s->n_cap) {
		/* delivery scratch: packets (bulk allocation, then grouping by
		 * queue), then one byte per frame (its pool, then its queue group) */
		free(s->tmp);
		s->tmp = malloc(s->n_cap * (sizeof(odp_packet_t) + 1u));
		s->tmp_cap = s->tmp ? s->n_cap : 0;
	}
	return 0;
}

/* Deliver set s on the host (the burst needs the host path). */
static int rx_finish_host(rt_pktio_t *e, rx_set_t *s, rx_cnt_t *c, odp_packet_t out[], int max_out,
			  uint64_t t2)
{
	const int num_rx = rx_deliver_host(e, s, c, out, max_out, t2);

	e->prof[2] += prof_ns() - t2;
	if (c->in_errors)
		odp_atomic_add_u64(&e->in_errors, c->in_errors);
	if (c->in_discards)
		odp_atomic_add_u64(&e->in_discards, c->in_discards);
	odp_atomic_add_u64(&e->in_octets, c->octets);
	odp_atomic_add_u64(&e->in_packets, c->packets);
	return num_rx;
}

/* Wait for set s's records and deliver its packets now: classified ones to
 * their CoS queues, the rest (classifier disabled) into out[] (at most
 * max_out).  Returns the packets placed in out[]. */
static int rx_finish(rt_pktio_t *e, rx_set_t *s, odp_packet_t out[], int max_out)
{
	rx_cnt_t c;

	if (rx_classified(e, s))
		return 0;
	const uint64_t t2 = prof_ns();

	memset(&c, 0, sizeof(c));
	if (rx_dlv_start(e, s, &c) == 0) {
		const int num_rx = rx_dlv_end(e, s, out, max_out);

		e->prof[2] += prof_ns() - t2;
		return num_rx;
	}
	return rx_finish_host(e, s, &c, out, max_out, t2);
}

/* Classifier on: wait for set s's records and start its GPU delivery,
 * leaving it in flight (rx_dlv_end on a later call); a burst that needs the
 * host path is delivered now. */
static void rx_finish_start(rt_pktio_t *e, rx_set_t *s)
{
	rx_cnt_t c;

	if (rx_classified(e, s))
		return;
	const uint64_t t2 = prof_ns();

	memset(&c, 0, sizeof(c));
	if (rx_dlv_start(e, s, &c) == 0) {
		e->prof[2] += prof_ns() - t2;
		return;
	}
	/* the host path delivers s now: every older burst still in its GPU
	 * delivery is enqueued first, oldest first (arrival order per queue) */
	for (int k = RX_SETS - 1; k > RX_CLS_DEPTH; k--) {
		rx_set_t *b = rx_age(e, k);

		if (b->delivering)
			(void)rx_dlv_end(e, b, NULL, 0);
	}
	(void)rx_finish_host(e, s, &c, NULL, 0, t2);
}

/* ------------------------------------------------------- receive chain
 * One submission per burst (mi_cls_rx_chain_submit): the classification,
 * the per-frame decisions of rx_dlv_start (parse drop, CoS drop / discard,
 * destination pool, too long for its pool, queue group) and the delivery
 * run on the GPU one after the other, with no host step between them.  The
 * packets the frames go into are taken from the pools before the submit (as
 * many per pool as the previous bursts used, plus a margin); a burst that
 * needs more of a pool than it was given is delivered again on the host
 * (rxc_end), so every outcome stays the reference's
 * (pktio/loop.c:253-384, pcap.c:299-352).  ODP_AMD_RX_CHAIN=0 turns it off. */
static int rx_chain_on(void)
{
	static int on = -1;

	if (on < 0) {
		const char *v = getenv("ODP_AMD_RX_CHAIN");

		on = !(v && v[0] == '0');
	}
	return on;
}

/* The chain's table for the current control-plane generation: refilled when
 * it changed; 0 when the chain can serve this pktio (every pool of the
 * table page-locked). */
static int rxc_table(rt_pktio_t *e)
{
	const uint64_t g = odp_amd_cls_generation();

	if (e->rxtab && e->rxtab_gen == g)
		return e->rxtab_ok ? 0 : -1;
	if (!e->rxtab) {
		e->rxtab = hmem_alloc(sizeof(mi_cls_rxtab_t), &e->rxtab_pinned);
		if (!e->rxtab)
			return -1;
	}
	uint64_t tg = 0;
	uint32_t np = 0;
	int ok = e->rxtab_pinned &&
		 odp_amd_cls_rxtab_fill(e->pool, e->rxtab, e->rx_pools, &np, &tg) == 0;

	for (uint32_t k = 0; ok && k < np; k++) {
		rt_pool_t *rp = rt_pool(e->rx_pools[k]);
		const int idx = odp_pool_index(e->rx_pools[k]);

		ok = rp && rp->pinned && rp->param.type == ODP_POOL_PACKET && idx >= 0 && idx < 64;
		if (ok) {
			e->rxtab->pool_cap[k] = rp->data_cap;
			e->rxtab->rt_slot[idx] = (uint8_t)(k + 1u);
		}
	}
	for (int k = 0; ok && k < RT_MAX_POOLS && k < 64; k++) {
		rt_pool_t *rp = rt_pool((odp_pool_t)(uintptr_t)(k + 1));

		e->rxtab->rt_pinned[k] = rp && rp->pinned;
	}
	if (e->rx_np != np)
		memset(e->rx_want, 0, sizeof(e->rx_want));   /* first bursts: as many as frames */
	e->rx_np = np;
	e->rxtab_gen = tg;
	{
		/* a new stamp per rewrite: the device's copies follow it */
		static uint64_t stamps;

		e->rxtab->stamp = __atomic_add_fetch(&stamps, 1, __ATOMIC_RELAXED);
	}
	e->rxtab_ok = ok && tg == g;
	return e->rxtab_ok ? 0 : -1;
}

/* Submit set s's burst as a chain: 1, or 0 when it takes the other path
 * (nothing done then). */
/* Whether this pktio's loop bursts can be staged by the GPU (the chain's
 * conditions, and an arena of page-locked pools to address them in). */
static int rxc_loop_stage_ok(rt_pktio_t *e, rx_set_t *s, uint32_t max)
{
	uint8_t *lo = NULL;
	size_t span = 0;

	return rx_chain_on() && gpu_deliver_on() && e->cls_enabled && e->parse_layer == ODP_PROTO_LAYER_ALL &&
	       s->rxc_pinned && s->dlv_pinned && s->arr_pinned && s->pk_pinned && max > 0 &&
	       max <= MI_CLS_DLV_GROUP_MAX && rt_pinned_arena(&lo, &span) && span < OOB_SPAN &&
	       rxc_table(e) == 0;
}

/* A burst that does not take the chain: a loop burst left for the GPU to
 * stage is staged by the host now (the classic path reads its descriptors). */
static int rxc_no(rt_pktio_t *e, rx_set_t *s)
{
	if (s->gstage) {
		s->gstage = 0;
		if (loop_stage_hdrs(e, s, (uint32_t)s->n)) {
			rx_drop(e, s, -ENOMEM);
			s->n = 0;
		}
	}
	return 0;
}

static int rxc_submit(rt_pktio_t *e, rx_set_t *s)
{
	const uint32_t n = (uint32_t)s->n;

	if (!rx_chain_on() || !gpu_deliver_on() || !e->cls_enabled || e->parse_layer != ODP_PROTO_LAYER_ALL ||
	    !s->rxc_pinned || !s->dlv_pinned || !s->arr_pinned || n == 0 || n > MI_CLS_DLV_GROUP_MAX ||
	    (e->drv == DRV_LOOP && !s->pk_pinned) || !mi_cls_host_mapped(s->base) || rxc_table(e))
		return rxc_no(e, s);
	/* the packets of each pool slot, in the order the frames take them */
	uint32_t at = 0;

	s->cnp = e->rx_np;
	for (uint32_t k = 0; k < s->cnp; k++) {
		uint32_t want = e->rx_want[k] ? e->rx_want[k] : n;

		if (want > n)
			want = n;
		if (at + want > s->got_cap)
			want = s->got_cap - at;
		s->cpool[k] = e->rx_pools[k];
		s->cbase[k] = at;
		s->chave[k] = want ? (uint32_t)rt_packet_alloc_raw(s->cpool[k], 0,
								   (odp_packet_t *)(void *)(s->got + at),
								   (int)want) : 0u;
		at += s->chave[k];
	}
	mi_cls_rxc_args_t a;

	memset(&a, 0, sizeof(a));
	a.base = s->base;
	a.soff = s->soff;
	a.slen = s->slen;
	a.res = s->res;
	a.n = n;
	a.layer = (uint32_t)e->parse_layer;
	a.input = (uint64_t)(uintptr_t)e->hdl;
	a.headroom = RT_PKT_HEADROOM;
	a.data_from_meta = rt_data_from_meta();
	a.tab = e->rxtab;
	a.got = s->got;
	memcpy(a.got_base, s->cbase, sizeof(a.got_base));
	memcpy(a.have, s->chave, sizeof(a.have));
	if (e->drv == DRV_LOOP) {
		/* the GPU reads the loop packets' metadata (a pool switch takes the
		 * old packet's user pointer): every packet in a page-locked pool
		 * (checked by address for a GPU-staged burst, by pool here) */
		if (!s->gstage)
			for (uint32_t i = 0; i < n; i++)
				if (!s->ppool[i] || !e->rxtab->rt_pinned[(s->ppool[i] - 1u) & 63u]) {
					for (uint32_t k = 0; k < s->cnp; k++)
						rt_packet_return_raw(s->cpool[k],
								     (const odp_packet_t *)(const void *)(s->got +
													   s->cbase[k]),
								     (int)s->chave[k]);
					return rxc_no(e, s);
				}
		a.pk = (const uint64_t *)(const void *)s->pk;
		a.ppool = s->ppool;
		a.stage = (uint32_t)s->gstage;
		a.head_off = (uint16_t)__builtin_offsetof(pkt_hdr_t, head);
		a.pool_off = (uint16_t)__builtin_offsetof(pkt_hdr_t, ev.pool);
	}
	a.meta_off = (uint32_t)__builtin_offsetof(pkt_hdr_t, meta);
	s->rxo->not_in_place = 0;
	a.dec = s->dec;
	a.ent = s->cent;
	a.perm = s->perm;
	a.gcnt = s->gcnt;
	a.out = s->rxo;
	s->gen = odp_amd_cls_generation();
	s->dgen = e->rxtab_gen;
	s->dticket = 0;
	const uint64_t tc = prof_ns();
	const int crc = odp_amd_cls_rx_chain(e->hdl, s->base, s->bytes, &a, &s->dticket);

	e->prof[13] += prof_ns() - tc;
	if (crc != 0) {
		for (uint32_t k = 0; k < s->cnp; k++)
			rt_packet_return_raw(s->cpool[k], (const odp_packet_t *)(const void *)(s->got + s->cbase[k]),
					     (int)s->chave[k]);
		s->dticket = 0;
		return rxc_no(e, s);
	}
	s->chain = 1;
	s->ticket = 0;
	s->pending = 0;
	s->delivering = 1;
	s->derr = 0;
	return 1;
}

/* End set s's chain: wait for it, give back the packets no frame took, free
 * the loop packets that were dropped or copied into another pool, enqueue
 * (one enqueue per queue group, else runs in arrival order), add the
 * counters.  A burst that was short of packets, or that the control plane
 * changed under, is finished on the host instead.  Returns the packets
 * placed in out[] (none: the classifier is on). */
static int rxc_end(rt_pktio_t *e, rx_set_t *s, odp_packet_t out[], int max_out)
{
	const uint64_t tk0 = prof_ns();
	int rc = odp_amd_cls_deliver_wait(e->hdl, s->dticket);
	const mi_cls_rx_out_t *o = s->rxo;

	s->delivering = 0;
	s->chain = 0;
	s->dticket = 0;
	e->prof[9] += prof_ns() - tk0;
	if (!rc) {
		/* the next bursts' packets per slot: this one's need plus a margin */
		for (uint32_t k = 0; k < s->cnp && k < e->rx_np; k++)
			e->rx_want[k] = o->need[k] + o->need[k] / 4u + 32u;
	}
	if (rc || o->short_pool || o->not_in_place || s->dgen != odp_amd_cls_generation()) {
		/* every packet taken for the burst back; the host path then
		 * decides, allocates and delivers from the records (the classify
		 * records are valid; a control-plane change re-classifies).  A loop
		 * burst the GPU staged is staged and classified again by the host
		 * (its headrooms and user pointers are the host path's inputs; a
		 * packet outside the page-locked arena is copied) */
		for (uint32_t k = 0; k < s->cnp; k++)
			rt_packet_return_raw(s->cpool[k], (const odp_packet_t *)(const void *)(s->got + s->cbase[k]),
					     (int)s->chave[k]);
		if (rc) {
			s->gstage = 0;
			rx_drop(e, s, rc);
			return 0;
		}
		if (s->gstage) {
			s->gstage = 0;
			if (loop_stage_hdrs(e, s, (uint32_t)s->n) || rx_classify(e, s, 0))
				return 0;   /* dropped and counted */
		}
		s->pending = 1;
		return rx_finish(e, s, out, max_out);
	}
	s->gstage = 0;
	const uint64_t tk1 = prof_ns();

	for (uint32_t k = 0; k < s->cnp; k++)
		if (o->used[k] < s->chave[k])
			rt_packet_return_raw(s->cpool[k],
					     (const odp_packet_t *)(const void *)(s->got + s->cbase[k] + o->used[k]),
					     (int)(s->chave[k] - o->used[k]));
	if (e->drv == DRV_LOOP) {
		/* loop packets not delivered in their own buffer: dropped,
		 * discarded, or copied into a packet of their CoS pool */
		for (int i = 0; i < s->n; i++)
			if ((s->dec[i] & 3u) != MI_CLS_RXF_INPLACE)
				odp_packet_free(s->pk[i]);
	}
	odp_packet_t *tmp = s->tmp;

	if (!tmp || s->tmp_cap < s->n_cap) {
		free(s->tmp);
		s->tmp = malloc(s->n_cap * (sizeof(odp_packet_t) + 1u));
		s->tmp_cap = s->tmp ? s->n_cap : 0;
		tmp = s->tmp;
	}
	if ((e->rxtab->flags & MI_CLS_RXT_GROUP) && tmp) {
		/* group g holds frames perm[at .. at + gcnt[g]) of the queue whose
		 * entries carry group g; queue stats per CoS of the queue */
		uint32_t at = 0;

		for (int g = 0; g < MI_CLS_DLV_GROUPS; g++) {
			const uint32_t num = s->gcnt[g];

			if (!num)
				continue;
			const uint32_t i0 = s->perm[at];
			const mi_cls_result_t *r0 = &s->res[i0];
			const odp_queue_t q = (odp_queue_t)(uintptr_t)
				e->rxtab->qh[e->rxtab->cos_q0[r0->cos] + r0->queue];
			uint64_t ok[256], bad[256];
			uint8_t seen[256], cl[256];
			int ncos = 0;

			for (uint32_t k = 0; k < num; k++)
				tmp[k] = (odp_packet_t)(uintptr_t)s->cent[s->perm[at + k]];
			int r = odp_queue_enq_multi(q, (const odp_event_t *)(void *)tmp, (int)num);

			if (r < 0)
				r = 0;
			if ((uint32_t)r != num)
				odp_packet_free_multi(&tmp[r], (int)num - r);
			memset(seen, 0, sizeof(seen));
			for (uint32_t k = 0; k < num; k++) {
				const uint32_t cos = s->res[s->perm[at + k]].cos;

				if (!seen[cos]) {
					seen[cos] = 1;
					cl[ncos++] = (uint8_t)cos;
					ok[cos] = 0;
					bad[cos] = 0;
				}
				if (k < (uint32_t)r)
					ok[cos]++;
				else
					bad[cos]++;
			}
			for (int j = 0; j < ncos; j++)
				odp_amd_cls_queue_stats_add(cl[j], cos_slot_of(cl[j], q), ok[cl[j]], bad[cl[j]]);
			at += num;
		}
	} else {
		/* runs of equal (queue, CoS) in arrival order (_odp_cls_enq) */
		int nd = 0;

		for (int i = 0; i < s->n; i++)
			if (s->cent[i])
				s->pk[nd++] = (odp_packet_t)(uintptr_t)s->cent[i];
		if (tmp)
			rx_enqueue(s->pk, nd, tmp, (uint8_t *)(void *)(tmp + s->tmp_cap));
		else
			for (int i = 0; i < nd; i++)
				cos_enq_run(&s->pk[i], 1);
	}
	if (o->in_errors)
		odp_atomic_add_u64(&e->in_errors, o->in_errors);
	if (o->in_discards)
		odp_atomic_add_u64(&e->in_discards, o->in_discards);
	odp_atomic_add_u64(&e->in_octets, o->octets);
	odp_atomic_add_u64(&e->in_packets, o->packets);
	e->prof[10] += prof_ns() - tk1;
	(void)out;
	(void)max_out;
	return 0;
}

/* Set of age k: staged k calls ago (age 0: this call). */
static rx_set_t *rx_age(rt_pktio_t *e, int k)
{
	return &e->rs[(e->cur + RX_SETS - k) % RX_SETS];
}

/* One receive call.  With the classifier enabled and more frames waiting at
 * the driver, bursts stream through RX_SETS sets by age: staged and
 * submitted for classification (age 0), classification in flight (ages 1 ..
 * RX_CLS_DEPTH), decided from their records and GPU delivery started (age
 * RX_CLS_DEPTH), delivery in flight (older), enqueued (the oldest).  Each
 * GPU step then has that many calls of host work to run behind before a
 * call waits for it (a delivery copies ~1.5 MB of frames over PCIe per
 * 4096-frame burst).  A call with nothing more at the driver delivers
 * everything, oldest first.  Unclassified packets are returned in out[] (at
 * most max_out); classified ones are enqueued to their CoS queues. */
static int pktio_recv(rt_pktio_t *e, odp_packet_t out[], int max_out)
{
	rx_set_t *s = rx_age(e, 0);
	long pending_n = 0;   /* frames staged, not yet taken from pools */
	int in_flight = 0;

	for (int k = 1; k < RX_SETS; k++) {
		const rx_set_t *o = rx_age(e, k);

		pending_n += o->pending ? (long)o->n : 0;
		in_flight |= o->pending || o->delivering;
	}
	const int pipe = e->cls_enabled && e->parse_layer != ODP_PROTO_LAYER_NONE &&
			 rx_pipeline();
	uint32_t burst = rx_burst();
	int num_rx = 0;

	if (rx_prof < 0)
		rx_prof = getenv("ODP_AMD_RX_PROF") != NULL;
	if (!e->cls_enabled && (uint32_t)max_out < burst)
		burst = (uint32_t)max_out;
	if (e->drv == DRV_PCAP) {
		/* pcap frames become packets of the pktio's pool at delivery: stage
		 * no more than the pool can still hold after the bursts in flight,
		 * so a packet allocation never fails on a staged frame (frames not
		 * staged stay in the store for the next call; the reference instead
		 * consumes the frame and stops on a failed allocation, pcap.c:324-327) */
		/* (frames that all go to CoS with pools of their own never take a
		 * packet of the pktio's pool: no bound then) */
		if (rt_pool(e->pool) && !(e->cls_enabled && odp_amd_cls_all_cos_pooled(e->pool))) {
			long room = (long)rt_pool_avail(e->pool) - pending_n;

			if (room < (long)burst)
				burst = room > 0 ? (uint32_t)room : 0u;
		}
	}
	uint64_t t0 = prof_ns();
	int n = stage_frames(e, s, burst);
	uint64_t t1 = prof_ns();

	e->prof[0] += t1 - t0;
	if (n < 0 && !in_flight)
		return n;
	s->n = n > 0 ? n : 0;
	if (n > 0) {
		e->prof[3]++;
		if (!(pipe && rxc_submit(e, s)) && rx_classify(e, s, pipe))
			n = 0;
		e->prof[1] += prof_ns() - t1;
	}
	/* bursts are delivered in arrival order: the oldest first */
	rx_set_t *z = rx_age(e, RX_SETS - 1);

	if (z->delivering)
		num_rx += rx_dlv_end(e, z, out, max_out);
	/* only a burst really in flight streams (a multi-GPU pktio's submit
	 * completes before it returns: ticket 0) */
	if (n > 0 && pipe && (s->ticket || s->chain) && rx_more(e)) {
		rx_set_t *q = rx_age(e, RX_CLS_DEPTH);

		if (q->pending)
			rx_finish_start(e, q);
		e->cur = (e->cur + 1) % RX_SETS;
		return num_rx;
	}
	/* the rest in arrival order: deliveries in flight, then the bursts
	 * still pending, then s */
	for (int k = RX_SETS - 2; k >= 1; k--) {
		rx_set_t *b = rx_age(e, k);

		if (b->delivering)
			num_rx += rx_dlv_end(e, b, out + num_rx, max_out - num_rx);
		if (b->pending)
			num_rx += rx_finish(e, b, out + num_rx, max_out - num_rx);
	}
	if (n > 0) {
		if (s->delivering)
			num_rx += rx_dlv_end(e, s, out + num_rx, max_out - num_rx);
		else
			num_rx += rx_finish(e, s, out + num_rx, max_out - num_rx);
	}
	return num_rx;
}

/* receive into the pktin queue (SCHED / QUEUE modes) */
static int poll_into_inq(rt_pktio_t *e)
{
	odp_packet_t pk[RX_BURST_DEFAULT];
	int n;

	if (!odp_spinlock_trylock(&e->rxl))
		return 0;
	if (e->state != ST_STARTED) {
		odp_spinlock_unlock(&e->rxl);
		return 0;
	}
	n = pktio_recv(e, pk, RX_BURST_DEFAULT);
	odp_spinlock_unlock(&e->rxl);
	if (n > 0) {
		int r = odp_queue_enq_multi(e->inq, (const odp_event_t *)(void *)pk, n);

		if (r < 0)
			r = 0;
		if (r < n) {
			odp_packet_free_multi(&pk[r], n - r);
			odp_atomic_add_u64(&e->in_discards, (uint64_t)(n - r));
		}
	}
	return n;
}

int rt_pktio_sched_poll(void)
{
	int idx[RT_MAX_PKTIO], n, total = 0;

	if (!__atomic_load_n(&num_sched_pktio, __ATOMIC_RELAXED))
		return 0;
	odp_spinlock_lock(&pk_lock);
	n = num_sched_pktio;
	memcpy(idx, sched_list, (size_t)n * sizeof(int));
	odp_spinlock_unlock(&pk_lock);
	for (int i = 0; i < n; i++)
		total += poll_into_inq(&PK[idx[i]]);
	return total;
}

int rt_pktio_poll_index(int idx)
{
	if (idx < 0 || idx >= RT_MAX_PKTIO || !PK[idx].used)
		return 0;
	return poll_into_inq(&PK[idx]);
}

int odp_pktin_recv(odp_pktin_queue_t q, odp_packet_t pkts[], int num)
{
	rt_pktio_t *e = get_pk(q.pktio);
	int n;

	if (!e || num < 0)
		return -1;
	if (e->state != ST_STARTED)
		return 0;
	odp_spinlock_lock(&e->rxl);
	n = e->state == ST_STARTED ? pktio_recv(e, pkts, num) : 0;
	odp_spinlock_unlock(&e->rxl);
	return n;
}

uint64_t odp_pktin_wait_time(uint64_t nsec)
{
	return nsec;
}

int odp_pktin_recv_tmo(odp_pktin_queue_t q, odp_packet_t pkts[], int num, uint64_t wait)
{
	odp_time_t t0 = odp_time_local();

	for (;;) {
		int n = odp_pktin_recv(q, pkts, num);

		if (n != 0 || wait == ODP_PKTIN_NO_WAIT)
			return n;
		if (wait != ODP_PKTIN_WAIT &&
		    odp_time_diff_ns(odp_time_local(), t0) >= wait)
			return 0;
		odp_time_wait_ns(10 * ODP_TIME_USEC_IN_NS);
	}
}

/* ============================================================ transmit */
int odp_pktout_send(odp_pktout_queue_t q, const odp_packet_t pkts[], int num)
{
	rt_pktio_t *e = get_pk(q.pktio);

	if (!e || num < 0)
		return -1;
	if (e->state != ST_STARTED)
		return -1;
	uint64_t octets = 0;

	for (int i = 0; i < num; i++)
		octets += odp_packet_len(pkts[i]);
	if (e->drv == DRV_LOOP) {
		int r = odp_queue_enq_multi(e->loopq, (const odp_event_t *)(const void *)pkts, num);

		if (r < 0)
			return -1;
		odp_atomic_add_u64(&e->out_packets, (uint64_t)r);
		odp_atomic_add_u64(&e->out_octets, octets);
		return r;
	}
	for (int i = 0; i < num; i++) {
		if (e->tx)
			pcap_dump(e, pkts[i]);
		odp_packet_free(pkts[i]);
	}
	odp_atomic_add_u64(&e->out_packets, (uint64_t)num);
	odp_atomic_add_u64(&e->out_octets, octets);
	return num;
}

/* ============================================================ misc */
int odp_pktio_promisc_mode(odp_pktio_t h)
{
	rt_pktio_t *e = get_pk(h);

	if (!e)
		return -1;
	return e->drv == DRV_PCAP ? e->promisc : 1;
}

int odp_pktio_promisc_mode_set(odp_pktio_t h, odp_bool_t enable)
{
	rt_pktio_t *e = get_pk(h);

	if (!e || e->drv != DRV_PCAP || e->state == ST_STARTED)
		return -1;
	e->promisc = enable;
	return 0;
}

int odp_pktio_mac_addr(odp_pktio_t h, void *mac, int size)
{
	rt_pktio_t *e = get_pk(h);

	if (!e || size < 6)
		return -1;
	memcpy(mac, e->drv == DRV_PCAP ? pcap_mac : loop_mac, 6);
	return 6;
}

uint32_t odp_pktio_mtu(odp_pktio_t h)
{
	rt_pktio_t *e = get_pk(h);

	return e ? (e->drv == DRV_PCAP ? PCAP_MTU_MAX : 9216) : 0;
}

int odp_pktio_stats(odp_pktio_t h, odp_pktio_stats_t *s)
{
	rt_pktio_t *e = get_pk(h);

	if (!e || !s)
		return -1;
	memset(s, 0, sizeof(*s));
	s->in_octets = odp_atomic_load_u64(&e->in_octets);
	s->in_packets = odp_atomic_load_u64(&e->in_packets);
	s->in_discards = odp_atomic_load_u64(&e->in_discards);
	s->in_errors = odp_atomic_load_u64(&e->in_errors);
	s->out_octets = odp_atomic_load_u64(&e->out_octets);
	s->out_packets = odp_atomic_load_u64(&e->out_packets);
	s->out_discards = odp_atomic_load_u64(&e->out_discards);
	return 0;
}

int odp_pktio_stats_reset(odp_pktio_t h)
{
	rt_pktio_t *e = get_pk(h);

	if (!e)
		return -1;
	odp_atomic_init_u64(&e->in_octets, 0);
	odp_atomic_init_u64(&e->in_packets, 0);
	odp_atomic_init_u64(&e->in_discards, 0);
	odp_atomic_init_u64(&e->in_errors, 0);
	odp_atomic_init_u64(&e->out_octets, 0);
	odp_atomic_init_u64(&e->out_packets, 0);
	odp_atomic_init_u64(&e->out_discards, 0);
	return 0;
}

int odp_pktio_info(odp_pktio_t h, odp_pktio_info_t *info)
{
	rt_pktio_t *e = get_pk(h);

	if (!e || !info)
		return -1;
	info->name = e->name;
	info->drv_name = e->drv == DRV_PCAP ? "pcap" : e->drv == DRV_LOOP ? "loop" : "null";
	info->pool = e->pool;
	info->param = e->param;
	return 0;
}

int odp_pktio_index(odp_pktio_t h)
{
	return get_pk(h) ? (int)((uintptr_t)h - 1) : -1;
}

uint64_t odp_pktio_to_u64(odp_pktio_t h)
{
	return (uint64_t)(uintptr_t)h;
}

void odp_pktio_print(odp_pktio_t h)
{
	rt_pktio_t *e = get_pk(h);
	odp_pktio_stats_t s;

	if (!e)
		return;
	odp_pktio_stats(h, &s);
	printf("Pktio info\n----------\n  name            %s\n  driver          %s\n"
	       "  classifier      %s\n  frames (pcap)   %u\n  in_packets      %" PRIu64 "\n"
	       "  in_errors       %" PRIu64 "\n  in_discards     %" PRIu64 "\n\n", e->name,
	       e->drv == DRV_PCAP ? "pcap" : e->drv == DRV_LOOP ? "loop" : "null",
	       e->cls_enabled ? "enabled (GPU)" : "disabled", e->nframes, s.in_packets,
	       s.in_errors, s.in_discards);
}

/* Build extension: 1 when the driver has no more input and no receive burst
 * is in flight (pcap past EOF, loop queue empty); 0 otherwise; -1 bad handle. */
int odp_amd_pktio_rx_idle(odp_pktio_t h)
{
	rt_pktio_t *e = get_pk(h);
	int idle;

	if (!e)
		return -1;
	odp_spinlock_lock(&e->rxl);
	idle = 1;
	for (int k = 0; k < RX_SETS; k++)
		if (e->rs[k].pending || e->rs[k].delivering)
			idle = 0;
	if (!idle)
		;
	else if (e->drv == DRV_PCAP)
		idle = e->eof || e->nframes == 0 || (e->next >= e->nframes && e->loops == 1);
	else if (e->drv == DRV_LOOP)
		idle = ((rt_queue_t *)(void *)e->loopq)->count == 0;
	else
		idle = 1;
	odp_spinlock_unlock(&e->rxl);
	return idle;
}
