/*
 * odp_cls_oracle.c -- CPU restatement of OpenDataPlane linux-generic's packet
 * parser + PMR classifier, used ONLY as test infrastructure.
 *
 *   *** TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT ***
 *   Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 *   load this library, and only as the checker / the timed CPU baseline.  The
 *   product path (odp_amd/, libodp_cls.so, libmi_cls.so) never links it.
 *
 * Parity status: PINNED by the reference's own fixtures (see DESIGN.md
 * "Oracle"): udp64.pcap + the example's rule (pktio_env:21-23), the parser
 * frames of test/common/test_packet_*.h with the flag assertions of
 * test/validation/api/packet/packet.c:3745-4560, the per-term MATCH/NO_MATCH
 * cases of odp_classification_test_pmr.c, and the input_flags words the
 * survey observed from the reference build.
 * The reference itself cannot be built here (it needs configure-generated
 * autoheaders and ~20 library stand-ins), so it is not linked.
 *
 * Everything below is a plain scalar restatement, written from the behaviour
 * of the reference (file:line citations are relative to
 * platform/linux-generic/ of the reference tree).  Bytes at or beyond
 * frame_len read as zero (the reference reads whatever follows the frame in
 * its buffer; our fixtures zero-pad, which makes the two identical).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

/* ------------------------------------------------------------------ flags */
/* input_flags bit numbers: include/odp/api/plat/packet_inline_types.h:66-107 */
#define IF_CLS_MARK   (1ull << 0)
#define IF_L2         (1ull << 3)
#define IF_L3         (1ull << 4)
#define IF_L4         (1ull << 5)
#define IF_ETH        (1ull << 6)
#define IF_ETH_BCAST  (1ull << 7)
#define IF_ETH_MCAST  (1ull << 8)
#define IF_JUMBO      (1ull << 9)
#define IF_VLAN       (1ull << 10)
#define IF_VLAN_QINQ  (1ull << 11)
#define IF_ARP        (1ull << 12)
#define IF_IPV4       (1ull << 13)
#define IF_IPV6       (1ull << 14)
#define IF_IP_BCAST   (1ull << 15)
#define IF_IP_MCAST   (1ull << 16)
#define IF_IPFRAG     (1ull << 17)
#define IF_IPOPT      (1ull << 18)
#define IF_IPSEC      (1ull << 19)
#define IF_IPSEC_AH   (1ull << 20)
#define IF_IPSEC_ESP  (1ull << 21)
#define IF_UDP        (1ull << 22)
#define IF_TCP        (1ull << 23)
#define IF_SCTP       (1ull << 24)
#define IF_ICMP       (1ull << 25)
#define IF_NO_NEXT    (1ull << 26)

/* error flags, as the 7-bit group flags.all.error (packet_inline_types.h:152-165) */
#define ER_SNAP_LEN   (1u << 0)
#define ER_IP         (1u << 1)
#define ER_L3_CHKSUM  (1u << 2)
#define ER_TCP        (1u << 3)
#define ER_UDP        (1u << 4)
#define ER_SCTP       (1u << 5)
#define ER_L4_CHKSUM  (1u << 6)

/* PMR terms: include/odp/api/spec/classification.h:55-137 (enum order) */
enum {
	T_LEN, T_ETHTYPE_0, T_ETHTYPE_X, T_VLAN_ID_0, T_VLAN_ID_X, T_VLAN_PCP_0,
	T_DMAC, T_IPPROTO, T_IP_DSCP, T_UDP_DPORT, T_TCP_DPORT, T_UDP_SPORT,
	T_TCP_SPORT, T_SIP_ADDR, T_DIP_ADDR, T_SIP6_ADDR, T_DIP6_ADDR,
	T_IPSEC_SPI, T_LD_VNI, T_CUSTOM_FRAME, T_CUSTOM_L3, T_IGMP_GRP_ADDR,
	T_ICMP_ID, T_ICMP_TYPE, T_ICMP_CODE, T_SCTP_SPORT, T_SCTP_DPORT,
	T_GTPV1_TEID, T_INNER_HDR_OFF = 32
};

/* result record: same 16-byte layout as include/mi_cls.h (mi_cls_result_t) */
typedef struct {
	uint32_t in_flags;
	uint8_t  err;
	uint8_t  outcome;
	uint8_t  cos;
	uint8_t  hops;
	uint16_t queue;
	uint16_t mark;
	uint16_t l3_offset;
	uint16_t l4_offset;
} orc_result_t;

_Static_assert(sizeof(orc_result_t) == 16, "result record is 16 bytes");

enum { OUT_ENQ = 0, OUT_COS_DROP = 1, OUT_DISCARD = 2, OUT_PARSE_DROP = 3, OUT_LOOP = 4 };

typedef struct {
	uint64_t input_flags;
	uint32_t err;
	uint16_t l2, l3, l4;
} orc_parser_t;

/* ---------------------------------------------------------- byte access */
typedef struct {
	const uint8_t *p;
	uint32_t len;
} pkt_t;

static inline uint32_t B(const pkt_t *k, uint32_t i)
{
	return i < k->len ? k->p[i] : 0u;
}

static inline uint32_t be16(const pkt_t *k, uint32_t i)
{
	return (B(k, i) << 8) | B(k, i + 1);
}

static inline uint32_t be32(const pkt_t *k, uint32_t i)
{
	return (B(k, i) << 24) | (B(k, i + 1) << 16) | (B(k, i + 2) << 8) | B(k, i + 3);
}

/* little-endian load of network bytes == the reference's raw struct load */
static inline uint32_t raw16(const pkt_t *k, uint32_t i)
{
	return B(k, i) | (B(k, i + 1) << 8);
}

static inline uint32_t raw32(const pkt_t *k, uint32_t i)
{
	return B(k, i) | (B(k, i + 1) << 8) | (B(k, i + 2) << 16) | (B(k, i + 3) << 24);
}

/* ----------------------------------------------------------------- parse */
/* _odp_parse_eth, odp_parse.c:23-105 */
static uint32_t parse_eth(orc_parser_t *prs, const pkt_t *k, uint32_t *offset)
{
	uint64_t f = IF_L2 | IF_ETH;
	uint32_t frame_len = k->len;
	uint32_t ethtype;

	if (frame_len - *offset > 1514)
		f |= IF_JUMBO;
	uint32_t mac0 = be16(k, 0);
	if ((mac0 & 0x0100) == 0x0100)
		f |= IF_ETH_MCAST;
	if (mac0 == 0xffff && be16(k, 2) == 0xffff && be16(k, 4) == 0xffff)
		f |= IF_ETH_BCAST;

	ethtype = be16(k, 12);
	*offset += 14;

	if (ethtype < 1514) {
		if (ethtype > frame_len - *offset) {
			prs->err |= ER_SNAP_LEN;
			ethtype = 0;
			goto error;
		}
		ethtype = be16(k, *offset + 6);
		*offset += 8;
	}
	if (ethtype == 0x88A8) {
		f |= IF_VLAN_QINQ | IF_VLAN;
		ethtype = be16(k, *offset + 2);
		*offset += 4;
	}
	if (ethtype == 0x8100) {
		f |= IF_VLAN;
		ethtype = be16(k, *offset + 2);
		*offset += 4;
	}
	if (*offset > frame_len) {
		f = IF_L2;
		ethtype = 0;
	}
error:
	prs->input_flags |= f;
	return ethtype;
}

/* ------------------------------------------------------ pktin options */
/* odp_pktin_config_opt_t.all_bits (include/odp/api/spec/packet_io.h) */
#define O_IPV4_CK    (1ull << 2)
#define O_UDP_CK     (1ull << 3)
#define O_TCP_CK     (1ull << 4)
#define O_SCTP_CK    (1ull << 5)
#define O_DROP_V4    (1ull << 6)
#define O_DROP_V6    (1ull << 7)
#define O_DROP_UDP   (1ull << 8)
#define O_DROP_TCP   (1ull << 9)
#define O_DROP_SCTP  (1ull << 10)
#define IF_L3_CHKSUM_DONE  (1ull << 30)
#define IF_L4_CHKSUM_DONE  (1ull << 31)
#define IF_UDP_CHKSUM_ZERO (1ull << 32)

static uint64_t g_opt;   /* pktio_entry->config.pktin of the receive path */

void orc_pktin_opt_set(uint64_t opt)
{
	g_opt = opt;
}

/* chksum_partial, include/odp_chksum_internal.h (the unaligned-access form;
 * every caller here starts at an even offset from L3): 32-bit little-endian
 * words, then a 16-bit word, then a last byte as the low byte. */
static uint64_t chksum_partial(const pkt_t *k, uint32_t o, uint32_t len)
{
	uint64_t sum = 0;

	while (len >= 4) {
		sum += raw32(k, o);
		o += 4;
		len -= 4;
	}
	if (len > 1) {
		sum += raw16(k, o);
		o += 2;
		len -= 2;
	}
	if (len)
		sum += B(k, o);   /* odp_cpu_to_be_16(b << 8) on a little-endian CPU */
	return sum;
}

/* chksum_finalize, include/odp_chksum_internal.h */
static uint16_t chksum_finalize(uint64_t sum)
{
	sum = (sum >> 32) + (sum & 0xffffffff);
	sum = (sum >> 16) + (sum & 0xffff);
	return (uint16_t)((sum >> 16) + sum);
}

/* odp_hash_crc32c (arch/default/odp_hash_crc32.c): reflected CRC-32C,
 * caller-supplied init, no final inversion; byte at a time. */
static uint32_t crc32c_bytes(uint32_t crc, const pkt_t *k, uint32_t o, uint32_t len)
{
	for (uint32_t i = 0; i < len; i++) {
		crc ^= B(k, o + i);
		for (int b = 0; b < 8; b++)
			crc = (crc & 1) ? (crc >> 1) ^ 0x82F63B78u : crc >> 1;
	}
	return crc;
}

/* parse_ipv4, odp_parse.c:112-173 */
static uint32_t parse_ipv4(orc_parser_t *prs, const pkt_t *k, uint32_t *offset, int *non_first,
			   uint64_t *l4_part_sum)
{
	uint32_t o = *offset, frame_len = k->len;
	uint32_t dst = be32(k, o + 16);
	uint32_t l3_len = be16(k, o + 2);
	uint32_t frag = be16(k, o + 6);
	uint32_t ver = B(k, o) >> 4, ihl = B(k, o) & 0xf;

	if ((prs->err & ER_L3_CHKSUM) || ihl < 5 || ver != 4 || 20 > frame_len - o ||
	    l3_len > frame_len - o) {
		prs->err |= ER_IP;
		return 0;
	}
	if (g_opt & O_IPV4_CK) {
		prs->input_flags |= IF_L3_CHKSUM_DONE;
		if (chksum_finalize(chksum_partial(k, o, ihl * 4)) != 0xffff) {
			prs->err |= ER_IP | ER_L3_CHKSUM;
			return 0;
		}
	}
	*offset += ihl * 4;
	if (g_opt & (O_UDP_CK | O_TCP_CK))
		*l4_part_sum = chksum_partial(k, o + 12, 8);   /* src + dst address */
	if (ihl > 5)
		prs->input_flags |= IF_IPOPT;
	if (frag & 0x3fff) {
		prs->input_flags |= IF_IPFRAG;
		if (frag & 0x1fff)
			*non_first = 1;
	}
	if (dst == 0xffffffffu)
		prs->input_flags |= IF_IP_BCAST;
	if ((dst >> 28) == 0xe)
		prs->input_flags |= IF_IP_MCAST;
	return B(k, o + 9);
}

/* parse_ipv6, odp_parse.c:183-249 */
static uint32_t parse_ipv6(orc_parser_t *prs, const pkt_t *k, uint32_t *offset, uint32_t seg_end,
			   uint64_t *l4_part_sum)
{
	uint32_t o = *offset, frame_len = k->len;
	uint32_t dst0 = be32(k, o + 24);
	uint32_t plen = be16(k, o + 4);
	uint32_t l3_len = plen + 40;

	if ((prs->err & ER_L3_CHKSUM) || (be32(k, o) >> 28) != 6 || 40 > frame_len - o ||
	    l3_len > frame_len - o) {
		prs->err |= ER_IP;
		return 0;
	}
	if ((dst0 & 0xff000000u) == 0xff000000u)
		prs->input_flags |= IF_IP_MCAST;
	else
		prs->input_flags &= ~IF_IP_MCAST;
	prs->input_flags &= ~IF_IP_BCAST;

	*offset += 40;
	if (g_opt & (O_UDP_CK | O_TCP_CK))
		*l4_part_sum = chksum_partial(k, o + 8, 32);   /* src + dst address */
	uint32_t nh = B(k, o + 6);
	if (nh == 0 || nh == 43) {
		uint32_t ext, nxt;

		prs->input_flags |= IF_IPOPT;
		do {
			ext = *offset;
			*offset += 8 + B(k, ext + 1) * 8;
			nxt = B(k, ext);
		} while ((nxt == 0 || nxt == 43) && *offset < seg_end);

		if (*offset >= prs->l3 + plen) {
			prs->err |= ER_IP;
			return 0;
		}
		if (nxt == 44)
			prs->input_flags |= IF_IPFRAG;
		return nxt;
	}
	if (nh == 44)
		prs->input_flags |= IF_IPOPT | IF_IPFRAG;
	return nh;
}

/* _odp_packet_l4_chksum, odp_packet.c:2065-2138 (contiguous packet:
 * packet_sum over [l4, frame_len) from the even offset l4 - l3). */
static int l4_chksum(const pkt_t *k, orc_parser_t *prs, uint64_t l4_part_sum)
{
	uint32_t frame_len = k->len, l4 = prs->l4;

	if (prs->input_flags & IF_IPFRAG)
		return prs->err != 0;
	if ((g_opt & O_UDP_CK) && (prs->input_flags & IF_UDP) &&
	    !(prs->input_flags & IF_UDP_CHKSUM_ZERO)) {
		uint16_t sum = (uint16_t)~chksum_finalize(l4_part_sum +
							  chksum_partial(k, l4, frame_len - l4));

		prs->input_flags |= IF_L4_CHKSUM_DONE;
		if (sum != 0) {
			prs->err |= ER_L4_CHKSUM | ER_UDP;
			if (g_opt & O_DROP_UDP)
				return -1;
		}
	} else if ((g_opt & O_TCP_CK) && (prs->input_flags & IF_TCP)) {
		uint16_t sum = (uint16_t)~chksum_finalize(l4_part_sum +
							  chksum_partial(k, l4, frame_len - l4));

		prs->input_flags |= IF_L4_CHKSUM_DONE;
		if (sum != 0) {
			prs->err |= ER_L4_CHKSUM | ER_TCP;
			if (g_opt & O_DROP_TCP)
				return -1;
		}
	} else if ((g_opt & O_SCTP_CK) && (prs->input_flags & IF_SCTP)) {
		uint32_t sum = ~crc32c_bytes((uint32_t)l4_part_sum, k, l4 + 12, frame_len - l4 - 12);

		prs->input_flags |= IF_L4_CHKSUM_DONE;
		if (sum != raw32(k, l4 + 8)) {
			prs->err |= ER_L4_CHKSUM | ER_SCTP;
			if (g_opt & O_DROP_SCTP)
				return -1;
		}
	}
	return prs->err != 0;
}

/* packet_parse_reset(all=1) + _odp_packet_parse_common (layer ALL, the
 * pktin options set by orc_pktin_opt_set):
 * odp_packet_internal.h:468-479, odp_parse_internal.h:80-112,
 * odp_parse.c:362-488.  Returns 0 ok, 1 error flags set, -1 drop. */
static int parse_l3_l4(const pkt_t *kp, orc_parser_t *prs, uint64_t *l4_part_sum);

int orc_parse(const uint8_t *p, uint32_t frame_len, orc_parser_t *prs)
{
	pkt_t k = { p, frame_len };
	uint64_t l4_part_sum = 0;
	int r;

	prs->input_flags = 0;
	prs->err = 0;
	prs->l2 = prs->l3 = prs->l4 = 0xFFFF;
	r = parse_l3_l4(&k, prs, &l4_part_sum);
	if (!r && (g_opt & (O_UDP_CK | O_TCP_CK | O_SCTP_CK)))
		r = l4_chksum(&k, prs, l4_part_sum);
	prs->input_flags &= ~IF_UDP_CHKSUM_ZERO;   /* internal: not in the record */
	return r;
}

static int parse_l3_l4(const pkt_t *kp, orc_parser_t *prs, uint64_t *l4_part_sum)
{
	pkt_t k = *kp;
	uint32_t frame_len = k.len;
	uint32_t seg_end = frame_len;   /* contiguous packet: seg_len == frame_len */
	uint32_t offset = 0, ip_proto = 255, ethtype;
	int non_first = 0;

	prs->l2 = 0;
	ethtype = parse_eth(prs, &k, &offset);

	prs->l3 = (uint16_t)offset;
	prs->input_flags |= IF_L3;
	switch (ethtype) {
	case 0x0800:
		prs->input_flags |= IF_IPV4;
		ip_proto = parse_ipv4(prs, &k, &offset, &non_first, l4_part_sum);
		if (!(prs->err & ER_IP))
			prs->l4 = (uint16_t)offset;
		else if (g_opt & O_DROP_V4)
			return -1;
		break;
	case 0x86DD:
		prs->input_flags |= IF_IPV6;
		ip_proto = parse_ipv6(prs, &k, &offset, seg_end, l4_part_sum);
		if (!(prs->err & ER_IP))
			prs->l4 = (uint16_t)offset;
		else if (g_opt & O_DROP_V6)
			return -1;
		break;
	case 0x0806:
		prs->input_flags |= IF_ARP;
		ip_proto = 255;
		break;
	default:
		prs->input_flags &= ~IF_L3;
		ip_proto = 255;
	}

	prs->input_flags |= IF_L4;
	switch (ip_proto) {
	case 1:
	case 58:
		prs->input_flags |= IF_ICMP;
		break;
	case 4:
		break;
	case 6:
		prs->input_flags |= IF_TCP;
		if (non_first)
			return prs->err != 0;
		if (offset + 20 > seg_end)
			return -1;
		/* parse_tcp, odp_parse.c:256-278 */
		if ((B(&k, offset + 12) >> 4) < 5)
			prs->err |= ER_TCP;
		if ((g_opt & O_TCP_CK) && !(prs->input_flags & IF_IPFRAG)) {
			uint16_t tcp_len = (uint16_t)(frame_len - prs->l4);

			*l4_part_sum += (uint16_t)((tcp_len >> 8) | (tcp_len << 8));   /* cpu_to_be_16 */
			*l4_part_sum += 6 << 8;
		}
		if ((prs->err & ER_TCP) && (g_opt & O_DROP_TCP))
			return -1;
		break;
	case 17:
		prs->input_flags |= IF_UDP;
		if (non_first)
			return prs->err != 0;
		if (offset + 8 > seg_end)
			return -1;
		/* parse_udp, odp_parse.c:285-327 */
		{
			uint32_t udplen = be16(&k, offset + 4);

			if (udplen < 8) {
				prs->err |= ER_UDP;
			} else {
				if ((g_opt & O_UDP_CK) && !(prs->input_flags & IF_IPFRAG)) {
					if (raw16(&k, offset + 6) == 0) {
						prs->input_flags |= IF_L4_CHKSUM_DONE;
						if (!(prs->input_flags & IF_IPV4))
							prs->err |= ER_L4_CHKSUM;
						prs->input_flags |= IF_UDP_CHKSUM_ZERO;
					} else {
						*l4_part_sum += raw16(&k, offset + 4);   /* udp->length */
						*l4_part_sum += 17 << 8;
					}
				}
				if (be16(&k, offset + 2) == 4500 && udplen > 4 &&
				    raw32(&k, offset + 8) != 0)
					prs->input_flags |= IF_IPSEC;
			}
		}
		if ((prs->err & ER_UDP) && (g_opt & O_DROP_UDP))
			return -1;
		break;
	case 51:
		prs->input_flags |= IF_IPSEC | IF_IPSEC_AH;
		break;
	case 50:
		prs->input_flags |= IF_IPSEC | IF_IPSEC_ESP;
		break;
	case 132:
		prs->input_flags |= IF_SCTP;
		if (non_first)
			return prs->err != 0;
		if (offset + 12 > seg_end)
			return -1;
		/* parse_sctp, odp_parse.c:334-356 */
		if ((uint16_t)(frame_len - prs->l4) < 12) {
			prs->err |= ER_SCTP;
		} else if ((g_opt & O_SCTP_CK) && !(prs->input_flags & IF_IPFRAG)) {
			uint32_t crc = crc32c_bytes(~0u, &k, offset, 8);
			static const uint8_t zero4[4];
			pkt_t z = { zero4, 4 };

			*l4_part_sum = crc32c_bytes(crc, &z, 0, 4);
		}
		if ((prs->err & ER_SCTP) && (g_opt & O_DROP_SCTP))
			return -1;
		break;
	case 59:
		prs->input_flags |= IF_NO_NEXT;
		break;
	default:
		prs->input_flags &= ~IF_L4;
		break;
	}
	return prs->err != 0;
}

/* -------------------------------------------------------- control plane */
/* Restates the table model of odp_classification.c:137-930 with pointer
 * semantics kept as slot indices. */
typedef struct {
	int term;
	uint8_t value[16];
	uint8_t mask[16];
	uint32_t val_sz;
	uint32_t offset;
} orc_term_t;

typedef struct orc_pmr {
	int valid;
	int num_terms;
	uint16_t mark;
	orc_term_t t[8];
	int src_cos;            /* slot, -1 none */
} orc_pmr_t;

typedef struct orc_cos {
	int valid;
	uint32_t num_rule;
	int *pmr;               /* slots, size max_pmr_per_cos */
	int *linked;            /* slots */
	int action;             /* 0 enqueue, 1 drop */
	uint32_t num_queue;
	uint32_t hash_proto;    /* bit0 ipv4, bit1 ipv6, bit2 udp, bit3 tcp (cos->hash_proto) */
	int stats_enable;
	uint8_t index;
	uint64_t stats_packets;
} orc_cos_t;

static struct {
	uint32_t max_cos, max_pmr, max_per_cos;
	orc_cos_t *cos;
	orc_pmr_t *pmr;
	int default_cos;        /* slot or -1 (entry->cls.default_cos) */
	int error_cos;
} G;

void orc_reset(uint32_t max_cos, uint32_t max_pmr, uint32_t max_per_cos)
{
	uint32_t i;

	if (G.cos) {
		for (i = 0; i < G.max_cos; i++) {
			free(G.cos[i].pmr);
			free(G.cos[i].linked);
		}
		free(G.cos);
		free(G.pmr);
	}
	G.max_cos = max_cos;
	G.max_pmr = max_pmr;
	G.max_per_cos = max_per_cos;
	G.cos = calloc(max_cos, sizeof(orc_cos_t));
	G.pmr = calloc(max_pmr, sizeof(orc_pmr_t));
	for (i = 0; i < max_cos; i++) {
		G.cos[i].pmr = calloc(max_per_cos, sizeof(int));
		G.cos[i].linked = calloc(max_per_cos, sizeof(int));
	}
	G.default_cos = -1;
	G.error_cos = -1;
}

/* odp_cls_cos_create (odp_classification.c:233-370), hash-proto folding :212-225.
 * hash_proto_in uses odp_pktin_hash_proto_t bits: ipv4_udp=0, ipv4_tcp=1,
 * ipv4=2, ipv6_udp=3, ipv6_tcp=4, ipv6=5. Returns handle (slot+1) or 0. */
int orc_cos_create(int action, uint32_t num_queue, int has_queue,
		   uint32_t hash_proto_in, int stats_enable)
{
	uint32_t i, j;

	if (action == 1) {
		num_queue = 1;
	} else if (num_queue == 1 && !has_queue) {
		return 0;
	}
	if (num_queue > 32 || num_queue < 1)
		return 0;
	for (i = 0; i < G.max_cos; i++) {
		orc_cos_t *c = &G.cos[i];

		if (c->valid)
			continue;
		for (j = 0; j < G.max_per_cos; j++) {
			c->pmr[j] = -1;
			c->linked[j] = -1;
		}
		c->num_queue = num_queue;
		c->hash_proto = 0;
		if (num_queue > 1) {
			uint32_t h = hash_proto_in;

			if (h & ((1u << 2) | (1u << 1) | (1u << 0)))
				c->hash_proto |= 1;
			if (h & ((1u << 5) | (1u << 4) | (1u << 3)))
				c->hash_proto |= 2;
			if (h & ((1u << 1) | (1u << 4)))
				c->hash_proto |= 8;
			if (h & ((1u << 0) | (1u << 3)))
				c->hash_proto |= 4;
		}
		c->stats_packets = 0;
		c->action = action;
		c->valid = 1;
		c->num_rule = 0;
		c->index = (uint8_t)i;
		c->stats_enable = stats_enable;
		return (int)i + 1;
	}
	return 0;
}

/* odp_cos_destroy (:487-501): only clears valid */
int orc_cos_destroy(int h)
{
	int s = h - 1;

	if (h == 0 || s < 0 || (uint32_t)s >= G.max_cos || !G.cos[s].valid)
		return -1;
	G.cos[s].valid = 0;
	return 0;
}

/* pmr_create_term (:670-763) value-size validation per term */
static int term_size_ok(const orc_term_t *t)
{
	uint32_t size;
	int custom = 0;

	switch (t->term) {
	case T_VLAN_PCP_0: case T_IPPROTO: case T_IP_DSCP:
		size = 1; break;
	case T_ETHTYPE_0: case T_ETHTYPE_X: case T_VLAN_ID_0: case T_VLAN_ID_X:
	case T_UDP_DPORT: case T_TCP_DPORT: case T_UDP_SPORT: case T_TCP_SPORT:
		size = 2; break;
	case T_LEN: case T_SIP_ADDR: case T_DIP_ADDR: case T_IPSEC_SPI: case T_LD_VNI:
		size = 4; break;
	case T_DMAC:
		size = 6; break;
	case T_SIP6_ADDR: case T_DIP6_ADDR:
		size = 16; break;
	case T_CUSTOM_FRAME: case T_CUSTOM_L3:
		custom = 1; size = 16; break;
	default:
		return 0;
	}
	if ((!custom && t->val_sz != size) || (custom && t->val_sz > size))
		return 0;
	return 1;
}

/* cls_pmr_create (:812-858).  Returns handle (slot+1) or 0. */
int orc_pmr_create(const orc_term_t *terms, int num_terms, uint32_t mark, int src, int dst)
{
	int s = src - 1, d = dst - 1, i;
	uint32_t p, b;

	if (src == 0 || dst == 0 || (uint32_t)s >= G.max_cos || (uint32_t)d >= G.max_cos ||
	    !G.cos[s].valid || !G.cos[d].valid)
		return 0;
	if (num_terms > 8)
		return 0;
	if (mark > 0xFFFF)
		return 0;
	if (G.cos[s].num_rule == G.max_per_cos)
		return 0;
	for (p = 0; p < G.max_pmr; p++)
		if (!G.pmr[p].valid)
			break;
	if (p == G.max_pmr)
		return 0;
	orc_pmr_t *r = &G.pmr[p];

	for (i = 0; i < num_terms; i++) {
		if (!term_size_ok(&terms[i]))
			return 0;
	}
	r->valid = 1;
	r->num_terms = num_terms;
	for (i = 0; i < num_terms; i++) {
		orc_term_t *t = &r->t[i];

		memset(t, 0, sizeof(*t));
		t->term = terms[i].term;
		t->val_sz = terms[i].val_sz;
		t->offset = terms[i].offset;
		memcpy(t->value, terms[i].value, t->val_sz);
		memcpy(t->mask, terms[i].mask, t->val_sz);
		for (b = 0; b < t->val_sz; b++)
			t->value[b] &= t->mask[b];
	}
	r->mark = (uint16_t)mark;
	G.cos[s].pmr[G.cos[s].num_rule] = (int)p;
	G.cos[s].linked[G.cos[s].num_rule] = d;
	G.cos[s].num_rule++;
	r->src_cos = s;
	return (int)p + 1;
}

/* odp_cls_pmr_destroy (:765-793): swap-with-last, unconditional decrement */
int orc_pmr_destroy(int h)
{
	int p = h - 1;
	uint32_t i, loc;

	if (h == 0 || (uint32_t)p >= G.max_pmr || !G.pmr[p].valid || G.pmr[p].src_cos < 0)
		return -1;
	orc_cos_t *c = &G.cos[G.pmr[p].src_cos];

	loc = c->num_rule;
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
	G.pmr[p].valid = 0;
	return 0;
}

int orc_default_cos_set(int h)
{
	if (h != 0 && ((uint32_t)(h - 1) >= G.max_cos || !G.cos[h - 1].valid))
		return -1;
	G.default_cos = h - 1;
	return 0;
}

int orc_error_cos_set(int h)
{
	if (h != 0 && ((uint32_t)(h - 1) >= G.max_cos || !G.cos[h - 1].valid))
		return -1;
	G.error_cos = h - 1;
	return 0;
}

uint64_t orc_cos_stats_packets(int h)
{
	return G.cos[h - 1].stats_packets;
}

/* ------------------------------------------------------------- classify */
static int bytes_match(const pkt_t *k, uint32_t o, const orc_term_t *t)
{
	uint32_t i;

	for (i = 0; i < t->val_sz; i++)
		if ((B(k, o + i) & t->mask[i]) != t->value[i])
			return 0;
	return 1;
}

/* Work counters of the reference's linear scan on this thread: PMRs
 * verify_pmr was called on, and terms it evaluated (its loop stops at the
 * first failing term, :1386-1512).  Read by orc_eval_counts() for bench.py's
 * compute roof ("reference-equivalent term evaluations"). */
static __thread uint64_t n_rules_tested, n_terms_tested;

void orc_eval_counts(uint64_t *rules, uint64_t *terms)
{
	*rules = n_rules_tested;
	*terms = n_terms_tested;
	n_rules_tested = n_terms_tested = 0;
}

/* verify_pmr (:1363-1515) with the verify_pmr_<term> helpers (:931-1357) */
static int verify_pmr(const orc_pmr_t *r, const pkt_t *k, const orc_parser_t *prs)
{
	uint64_t f = prs->input_flags;
	int i;

	n_rules_tested++;
	if (!r->valid)
		return 0;
	for (i = 0; i < r->num_terms; i++) {
		const orc_term_t *t = &r->t[i];
		int ok;

		n_terms_tested++;

		switch (t->term) {
		case T_LEN: {
			uint32_t v, m;

			memcpy(&v, t->value, 4);
			memcpy(&m, t->mask, 4);
			ok = (k->len & m) == v;
			break;
		}
		case T_ETHTYPE_0:
			ok = (f & IF_ETH) && bytes_match(k, prs->l2 + 12, t);
			break;
		case T_ETHTYPE_X:
			ok = (f & (IF_VLAN | IF_VLAN_QINQ)) &&
			     bytes_match(k, prs->l2 + ((f & IF_VLAN_QINQ) ? 20 : 16), t);
			break;
		case T_VLAN_ID_0:
		case T_VLAN_ID_X: {
			uint32_t o;

			if (t->term == T_VLAN_ID_0) {
				ok = (f & IF_ETH) && (f & IF_VLAN);
				o = prs->l2 + 14;
			} else {
				ok = (f & (IF_VLAN | IF_VLAN_QINQ)) != 0;
				o = prs->l2 + ((f & IF_VLAN_QINQ) ? 18 : 14);
			}
			if (ok) {
				uint32_t vid0 = B(k, o) & 0x0f, vid1 = B(k, o + 1);

				ok = ((vid0 & t->mask[0]) == t->value[0]) &&
				     ((vid1 & t->mask[1]) == t->value[1]);
			}
			break;
		}
		case T_VLAN_PCP_0:
			ok = (f & IF_ETH) && (f & IF_VLAN) &&
			     (((B(k, prs->l2 + 14) >> 5) & t->mask[0]) == t->value[0]);
			break;
		case T_DMAC:
			ok = (f & IF_ETH) && bytes_match(k, prs->l2, t);
			break;
		case T_IPPROTO:
			if (f & IF_IPV4)
				ok = (B(k, prs->l3 + 9) & t->mask[0]) == t->value[0];
			else if (f & IF_IPV6)
				ok = (B(k, prs->l3 + 6) & t->mask[0]) == t->value[0];
			else
				ok = 0;
			break;
		case T_IP_DSCP: {
			uint32_t d;

			if (f & IF_IPV4)
				d = (B(k, prs->l3 + 1) & 0xfc) >> 2;
			else if (f & IF_IPV6)
				d = (be32(k, prs->l3) & 0x0fc00000u) >> 22;
			else {
				ok = 0;
				break;
			}
			ok = (d & t->mask[0]) == t->value[0];
			break;
		}
		case T_UDP_DPORT:
			ok = (f & IF_UDP) && bytes_match(k, prs->l4 + 2, t);
			break;
		case T_TCP_DPORT:
			ok = (f & IF_TCP) && bytes_match(k, prs->l4 + 2, t);
			break;
		case T_UDP_SPORT:
			ok = (f & IF_UDP) && bytes_match(k, prs->l4, t);
			break;
		case T_TCP_SPORT:
			ok = (f & IF_TCP) && bytes_match(k, prs->l4, t);
			break;
		case T_SIP_ADDR:
			ok = (f & IF_IPV4) && bytes_match(k, prs->l3 + 12, t);
			break;
		case T_DIP_ADDR:
			ok = (f & IF_IPV4) && bytes_match(k, prs->l3 + 16, t);
			break;
		case T_SIP6_ADDR:
			ok = (f & IF_IPV6) && bytes_match(k, prs->l3 + 8, t);
			break;
		case T_DIP6_ADDR:
			ok = (f & IF_IPV6) && bytes_match(k, prs->l3 + 24, t);
			break;
		case T_IPSEC_SPI:
			if (f & IF_IPSEC_AH)
				ok = bytes_match(k, prs->l4 + 4, t);
			else if (f & IF_IPSEC_ESP)
				ok = bytes_match(k, prs->l4, t);
			else
				ok = 0;
			break;
		case T_LD_VNI:
			ok = 0;
			break;
		case T_CUSTOM_FRAME:
			ok = !(k->len <= t->offset + t->val_sz) && bytes_match(k, t->offset, t);
			break;
		case T_CUSTOM_L3: {
			uint32_t o = (uint32_t)prs->l3 + t->offset;

			ok = (f & IF_L2) && prs->l3 != 0xFFFF &&
			     !(k->len <= o + t->val_sz) && bytes_match(k, o, t);
			break;
		}
		case T_INNER_HDR_OFF:
			ok = 1;
			break;
		default:
			ok = 0;
		}
		if (!ok)
			return 0;
	}
	return 1;
}

/* thash_softrss (include/protocols/thash.h:82-99) with the default key
 * (odp_classification.c:50-58) */
static const uint8_t rss_key[40] = {
	0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2,
	0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3, 0x8f, 0xb0,
	0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4,
	0x77, 0xcb, 0x2d, 0xa3, 0x80, 0x30, 0xf2, 0x0c,
	0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa,
};

static uint32_t key_word(int j)
{
	return ((uint32_t)rss_key[4 * j] << 24) | ((uint32_t)rss_key[4 * j + 1] << 16) |
	       ((uint32_t)rss_key[4 * j + 2] << 8) | rss_key[4 * j + 3];
}

uint32_t orc_softrss(const uint32_t *tuple, uint32_t len)
{
	uint32_t i, j, ret = 0;

	for (j = 0; j < len; j++)
		for (i = 0; i < 32; i++)
			if (tuple[j] & (1u << (31 - i)))
				ret ^= (key_word(j) << i) |
				       (uint32_t)((uint64_t)key_word(j + 1) >> (32 - i));
	return ret;
}

/* packet_rss_hash (:1773-1839).  The uninitialised-word case (L4 hashing
 * without L3 hashing) is undefined in the reference; word 0 reads zero here. */
static uint32_t rss_hash(const pkt_t *k, const orc_parser_t *prs, uint32_t hp)
{
	uint32_t t[9] = { 0 }, n = 0, i;
	uint64_t f = prs->input_flags;

	if (f & IF_IPV4) {
		if (hp & 1) {
			t[0] = raw32(k, prs->l3 + 12);
			t[1] = raw32(k, prs->l3 + 16);
			n += 2;
		}
		if (((f & IF_TCP) && (hp & 8)) || ((f & IF_UDP) && (hp & 4))) {
			t[2] = raw16(k, prs->l4) | (raw16(k, prs->l4 + 2) << 16);
			n += 1;
		}
	} else if (f & IF_IPV6) {
		if (hp & 2) {
			for (i = 0; i < 4; i++) {
				t[i] = be32(k, prs->l3 + 8 + 4 * i);
				t[4 + i] = be32(k, prs->l3 + 24 + 4 * i);
			}
			n += 8;
		}
		if (((f & IF_TCP) && (hp & 8)) || ((f & IF_UDP) && (hp & 4))) {
			t[8] = raw16(k, prs->l4) | (raw16(k, prs->l4 + 2) << 16);
			n += 1;
		}
	}
	return n ? orc_softrss(t, n) : 0;
}

/* match_pmr_cos (:1624-1667), cls_select_cos (:1694-1726),
 * _odp_cls_classify_packet (:1742-1771), get_dest_queue (:395-405).
 * The reference loops forever on a CoS cycle; this restatement stops after
 * max_hops matches and reports OUT_LOOP (the device does the same). */
static void classify(const pkt_t *k, orc_parser_t *prs, orc_result_t *out, uint32_t max_hops)
{
	int cos;
	uint32_t hops = 0;

	out->mark = 0;
	if (prs->err) {
		cos = G.error_cos;
		if (cos >= 0 && G.cos[cos].stats_enable)
			G.cos[cos].stats_packets++;
	} else {
		int def = G.default_cos;

		cos = def;
		if (def >= 0 && G.cos[def].valid) {
			int c = def, matched = -1;

			for (;;) {
				uint32_t i, n = G.cos[c].num_rule;

				for (i = 0; i < n; i++) {
					int pm = G.cos[c].pmr[i], lk = G.cos[c].linked[i];

					if (!G.cos[lk].valid)
						continue;
					if (verify_pmr(&G.pmr[pm], k, prs)) {
						matched = pm;
						c = lk;
						if (G.cos[c].stats_enable)
							G.cos[c].stats_packets++;
						break;
					}
				}
				if (i == n)
					break;
				if (++hops > max_hops)
					break;
			}
			if (hops > max_hops) {
				out->outcome = OUT_LOOP;
				out->cos = 0xFF;
				out->queue = 0;
				out->hops = 0xFF;
				return;
			}
			if (matched >= 0) {
				prs->input_flags &= ~IF_CLS_MARK;
				if (G.pmr[matched].mark) {
					prs->input_flags |= IF_CLS_MARK;
					out->mark = G.pmr[matched].mark;
				}
			}
			if (c != def) {
				cos = c;
				goto have_cos;
			}
		}
		cos = def;
		if (cos >= 0 && G.cos[cos].stats_enable)
			G.cos[cos].stats_packets++;
	}
have_cos:
	out->hops = (uint8_t)hops;
	if (cos < 0) {
		out->outcome = OUT_DISCARD;
		out->cos = 0xFF;
		out->queue = 0;
		return;
	}
	out->cos = G.cos[cos].index;
	out->queue = 0;
	if (G.cos[cos].action == 1) {
		out->outcome = OUT_COS_DROP;
		return;
	}
	out->outcome = OUT_ENQ;
	if (G.cos[cos].num_queue > 1) {
		uint32_t h = rss_hash(k, prs, G.cos[cos].hash_proto) & 31;

		out->queue = (uint16_t)(h % G.cos[cos].num_queue);
	}
}

static void classify_one(const uint8_t *p, uint32_t len, orc_result_t *o, uint32_t max_hops)
{
	orc_parser_t prs;
	pkt_t k = { p, len };
	int r = orc_parse(p, len, &prs);

	o->hops = 0;
	o->mark = 0;
	if (r < 0) {
		o->outcome = OUT_PARSE_DROP;
		o->cos = 0xFF;
		o->queue = 0;
	} else {
		classify(&k, &prs, o, max_hops);
	}
	o->in_flags = (uint32_t)prs.input_flags;
	o->err = (uint8_t)prs.err;
	o->l3_offset = prs.l3;
	o->l4_offset = prs.l4;
}

void orc_classify_batch(const uint8_t *buf, const uint32_t *off, const uint16_t *len,
			uint32_t n, orc_result_t *out, uint32_t max_hops)
{
	uint32_t i;

	for (i = 0; i < n; i++)
		classify_one(buf + off[i], len[i], &out[i], max_hops);
}

/* Parse only, for the parser fixtures: fills input_flags (u64), err, l2/l3/l4. */
int orc_parse_one(const uint8_t *p, uint32_t len, uint64_t *input_flags, uint32_t *err,
		  uint16_t *l2, uint16_t *l3, uint16_t *l4)
{
	orc_parser_t prs;
	int r = orc_parse(p, len, &prs);

	*input_flags = prs.input_flags;
	*err = prs.err;
	*l2 = prs.l2;
	*l3 = prs.l3;
	*l4 = prs.l4;
	return r;
}

uint32_t orc_rss_hash_one(const uint8_t *p, uint32_t len, uint32_t hash_proto_bits)
{
	orc_parser_t prs;
	pkt_t k = { p, len };

	orc_parse(p, len, &prs);
	return rss_hash(&k, &prs, hash_proto_bits);
}

/* Multi-threaded batch run for the CPU baseline: each thread takes a
 * disjoint contiguous slice (stats counters are not thread safe, so the
 * baseline runs with stats disabled, as the benchmark rule sets do). */
typedef struct {
	const uint8_t *buf;
	const uint32_t *off;
	const uint16_t *len;
	orc_result_t *out;
	uint32_t begin, end, max_hops;
} slice_t;

static void *slice_run(void *a)
{
	slice_t *s = a;
	uint32_t i;

	for (i = s->begin; i < s->end; i++)
		classify_one(s->buf + s->off[i], s->len[i], &s->out[i], s->max_hops);
	return NULL;
}

int orc_classify_batch_mt(const uint8_t *buf, const uint32_t *off, const uint16_t *len,
			  uint32_t n, orc_result_t *out, uint32_t max_hops, int threads)
{
	pthread_t tid[256];
	slice_t sl[256];
	int t;

	if (threads < 1)
		threads = 1;
	if (threads > 256)
		threads = 256;
	for (t = 0; t < threads; t++) {
		sl[t] = (slice_t){ buf, off, len, out,
				   (uint32_t)((uint64_t)n * t / threads),
				   (uint32_t)((uint64_t)n * (t + 1) / threads), max_hops };
		if (pthread_create(&tid[t], NULL, slice_run, &sl[t]))
			return -1;
	}
	for (t = 0; t < threads; t++)
		pthread_join(tid[t], NULL);
	return 0;
}
