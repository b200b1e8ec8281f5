// mi_cls.hip -- gfx950 (MI355X / CDNA4) packet parse + PMR classify kernel and
// the C ABI declared in include/mi_cls.h.
//
// What it replaces (reference, platform/linux-generic/):
//   pktio/loop.c:283-339        per-packet parse + classify inside loopback_recv
//   odp_parse.c:23-488          _odp_parse_eth / parse_ipv4 / parse_ipv6 / parse_tcp
//                               / parse_udp / parse_sctp / _odp_packet_parse_common_l3_l4
//   odp_classification.c:931-1515   verify_pmr and the per-term verifiers
//   odp_classification.c:1624-1771  match_pmr_cos / cls_select_cos / _odp_cls_classify_packet
//   odp_classification.c:395-405, 1773-1839 + protocols/thash.h:82-99  hash-queue pick
//
// Design (MI355X-first, not a translation):
//   * one wavefront owns 64 consecutive packets (one packet per lane);
//   * the first 128 B of each packet are staged into LDS with coalesced 16-B
//     loads: lane l of staging round k loads 16-B piece (l & 7) of packet
//     8k + (l >> 3), so a round covers 8 packets x 128 B and adjacent lanes
//     read adjacent bytes; pieces past the frame are not fetched and read 0;
//   * each lane then parses its own packet out of its LDS window (stride 33
//     dwords: conflict-free ds_read_b32 when lanes read the same field);
//     bytes beyond the window come from HBM, bytes beyond frame_len read 0;
//   * the CoS tree is walked as a wavefront "waterfall": the CoS of the first
//     pending lane is made wave-uniform (readlane), every lane sitting on it
//     scans that CoS's rules in order with the rule/term words in SGPRs
//     (scalar loads, all lanes test the same rule), per-lane first match is
//     tracked in an exec-mask and the scan ends as soon as a ballot shows no
//     lane of the group still unmatched.  No MFMA: this is parse-and-compare.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "mi_cls.h"

#define WAVE 64
#define WAVES_PER_BLOCK 4
#define BLOCK (WAVE * WAVES_PER_BLOCK)
#define WIN 128            // staged header window, bytes
#define WSTRIDE 33         // dwords per packet window in LDS (32 + 1 pad)
#define MAX_STATS_COS 256

// ---------------------------------------------------------------- flags
// input_flags bits: include/odp/api/plat/packet_inline_types.h:66-107
#define F_CLS_MARK  (1u << 0)
#define F_L2        (1u << 3)
#define F_L3        (1u << 4)
#define F_L4        (1u << 5)
#define F_ETH       (1u << 6)
#define F_ETH_BCAST (1u << 7)
#define F_ETH_MCAST (1u << 8)
#define F_JUMBO     (1u << 9)
#define F_VLAN      (1u << 10)
#define F_QINQ      (1u << 11)
#define F_ARP       (1u << 12)
#define F_IPV4      (1u << 13)
#define F_IPV6      (1u << 14)
#define F_IP_BCAST  (1u << 15)
#define F_IP_MCAST  (1u << 16)
#define F_IPFRAG    (1u << 17)
#define F_IPOPT     (1u << 18)
#define F_IPSEC     (1u << 19)
#define F_AH        (1u << 20)
#define F_ESP       (1u << 21)
#define F_UDP       (1u << 22)
#define F_TCP       (1u << 23)
#define F_SCTP      (1u << 24)
#define F_ICMP      (1u << 25)
#define F_NO_NEXT   (1u << 26)
// error group bits (flags.all.error, packet_inline_types.h:152-165)
#define E_SNAP 1u
#define E_IP   2u
#define E_TCP  8u
#define E_UDP  16u
#define E_SCTP 32u

// ------------------------------------------------------- packet byte access
struct Pkt {
	const uint32_t *w;      // this lane's LDS window (dwords)
	const uint8_t *g;       // packet start in HBM
	uint32_t len;           // frame_len
};

__device__ __forceinline__ uint32_t rb(const Pkt &k, uint32_t o)
{
	if (o < WIN)
		return (k.w[o >> 2] >> ((o & 3u) * 8u)) & 0xffu;
	return o < k.len ? (uint32_t)k.g[o] : 0u;
}

// 4 bytes starting at byte offset o, little-endian (== the reference's raw load)
__device__ __forceinline__ uint32_t r32(const Pkt &k, uint32_t o)
{
	if (o <= WIN - 4u) {
		uint32_t i = o >> 2;
		return __builtin_amdgcn_alignbyte(k.w[i + 1], k.w[i], o & 3u);
	}
	return rb(k, o) | (rb(k, o + 1) << 8) | (rb(k, o + 2) << 16) | (rb(k, o + 3) << 24);
}

__device__ __forceinline__ uint32_t r16(const Pkt &k, uint32_t o)
{
	return r32(k, o) & 0xffffu;
}

__device__ __forceinline__ uint32_t be16(const Pkt &k, uint32_t o)
{
	uint32_t v = r16(k, o);
	return ((v & 0xffu) << 8) | (v >> 8);
}

__device__ __forceinline__ uint32_t be32(const Pkt &k, uint32_t o)
{
	return __builtin_bswap32(r32(k, o));
}

// ------------------------------------------------------------------ parse
struct Parsed {
	uint32_t flags;
	uint32_t err;
	uint32_t l3, l4;
	int ret;                // 0 ok, 1 error flags, -1 drop
};

// _odp_parse_eth + _odp_packet_parse_common_l3_l4 (layer ALL, checksum opts off),
// odp_parse.c:23-105, 112-354, 362-488; contiguous packet so seg_end == frame_len.
__device__ __forceinline__ Parsed parse_packet(const Pkt &k)
{
	Parsed r;
	const uint32_t len = k.len;
	uint32_t f = F_L2 | F_ETH, err = 0, off = 14, ethtype, ip_proto = 255;
	bool non_first = false;

	r.l4 = 0xFFFFu;
	uint32_t w0 = r32(k, 0), w1 = r32(k, 4);
	if (len > 1514u)
		f |= F_JUMBO;
	if (w0 & 1u)
		f |= F_ETH_MCAST;
	if (w0 == 0xffffffffu && (w1 & 0xffffu) == 0xffffu)
		f |= F_ETH_BCAST;
	ethtype = be16(k, 12);
	bool snap_err = false;
	if (ethtype < 1514u) {
		if (ethtype > len - 14u) {
			err |= E_SNAP;
			ethtype = 0;
			snap_err = true;
		} else {
			ethtype = be16(k, 20);
			off = 22;
		}
	}
	if (!snap_err) {
		if (ethtype == 0x88A8u) {
			f |= F_QINQ | F_VLAN;
			ethtype = be16(k, off + 2);
			off += 4;
		}
		if (ethtype == 0x8100u) {
			f |= F_VLAN;
			ethtype = be16(k, off + 2);
			off += 4;
		}
		if (off > len) {
			f = F_L2;
			ethtype = 0;
		}
	}

	const uint32_t l3 = off;
	r.l3 = l3;
	f |= F_L3;
	if (ethtype == 0x0800u) {
		f |= F_IPV4;
		uint32_t vi = rb(k, l3);
		uint32_t ihl = vi & 0xfu;
		uint32_t tot = be16(k, l3 + 2);
		if (ihl < 5u || (vi >> 4) != 4u || 20u > len - l3 || tot > len - l3) {
			err |= E_IP;
			ip_proto = 0;
		} else {
			uint32_t frag = be16(k, l3 + 6);
			uint32_t dst = be32(k, l3 + 16);
			off = l3 + ihl * 4u;
			if (ihl > 5u)
				f |= F_IPOPT;
			if (frag & 0x3fffu) {
				f |= F_IPFRAG;
				non_first = (frag & 0x1fffu) != 0;
			}
			if (dst == 0xffffffffu)
				f |= F_IP_BCAST;
			if ((dst >> 28) == 0xeu)
				f |= F_IP_MCAST;
			ip_proto = rb(k, l3 + 9);
			r.l4 = off;
		}
	} else if (ethtype == 0x86DDu) {
		f |= F_IPV6;
		uint32_t plen = be16(k, l3 + 4);
		if ((rb(k, l3) >> 4) != 6u || 40u > len - l3 || plen + 40u > len - l3) {
			err |= E_IP;
			ip_proto = 0;
		} else {
			if (rb(k, l3 + 24) == 0xffu)
				f |= F_IP_MCAST;
			off = l3 + 40;
			uint32_t nh = rb(k, l3 + 6);
			if (nh == 0u || nh == 43u) {
				uint32_t nxt;
				f |= F_IPOPT;
				do {
					uint32_t ext = off;
					off += 8u + rb(k, ext + 1) * 8u;
					nxt = rb(k, ext);
				} while ((nxt == 0u || nxt == 43u) && off < len);
				if (off >= l3 + plen) {
					err |= E_IP;
					ip_proto = 0;
				} else {
					if (nxt == 44u)
						f |= F_IPFRAG;
					ip_proto = nxt;
					r.l4 = off;
				}
			} else {
				if (nh == 44u)
					f |= F_IPOPT | F_IPFRAG;
				ip_proto = nh;
				r.l4 = off;
			}
		}
	} else if (ethtype == 0x0806u) {
		f |= F_ARP;
	} else {
		f &= ~F_L3;
	}

	int ret = 0;
	f |= F_L4;
	switch (ip_proto) {
	case 1u:
	case 58u:
		f |= F_ICMP;
		break;
	case 4u:
		break;
	case 6u:
		f |= F_TCP;
		if (!non_first) {
			if (off + 20u > len)
				ret = -1;
			else if ((rb(k, off + 12) >> 4) < 5u)
				err |= E_TCP;
		}
		break;
	case 17u:
		f |= F_UDP;
		if (!non_first) {
			if (off + 8u > len) {
				ret = -1;
			} else {
				uint32_t ports = r32(k, off);
				uint32_t ulen = be16(k, off + 4);
				if (ulen < 8u)
					err |= E_UDP;
				else if ((ports >> 16) == 0x9411u /* be16(4500) raw */ && ulen > 4u &&
					 r32(k, off + 8) != 0u)
					f |= F_IPSEC;
			}
		}
		break;
	case 51u:
		f |= F_IPSEC | F_AH;
		break;
	case 50u:
		f |= F_IPSEC | F_ESP;
		break;
	case 132u:
		f |= F_SCTP;
		if (!non_first) {
			if (off + 12u > len)
				ret = -1;
			else if (((len - r.l4) & 0xffffu) < 12u)
				err |= E_SCTP;
		}
		break;
	case 59u:
		f |= F_NO_NEXT;
		break;
	default:
		f &= ~F_L4;
		break;
	}
	r.flags = f;
	r.err = err;
	r.ret = ret < 0 ? -1 : (err != 0 ? 1 : 0);
	return r;
}

// --------------------------------------------------------- field registers
// Gate bits (presence tests of the verify_pmr_<term> helpers)
#define G_ETH   (1u << 0)
#define G_VLAN0 (1u << 1)   // eth && vlan
#define G_VLANX (1u << 2)   // vlan || qinq
#define G_V4    (1u << 3)
#define G_V6    (1u << 4)
#define G_UDP   (1u << 5)
#define G_TCP   (1u << 6)
#define G_SPI   (1u << 7)   // ah || esp
#define G_L3OK  (1u << 8)   // l2 && l3 valid

struct Fields {
	uint32_t gates;
	uint32_t eth0, ethx, vid0, vidx, pcp0, dmac0, dmac1;
	uint32_t proto, dscp, ports, sip, dip, spi;
	uint32_t s6[4], d6[4];
};

__device__ __forceinline__ void load_fields(const Pkt &k, const Parsed &p, uint32_t used, Fields &x)
{
	const uint32_t f = p.flags;
	uint32_t g = 0;
	if (f & F_ETH) g |= G_ETH;
	if ((f & F_ETH) && (f & F_VLAN)) g |= G_VLAN0;
	if (f & (F_VLAN | F_QINQ)) g |= G_VLANX;
	if (f & F_IPV4) g |= G_V4;
	if (f & F_IPV6) g |= G_V6;
	if (f & F_UDP) g |= G_UDP;
	if (f & F_TCP) g |= G_TCP;
	if (f & (F_AH | F_ESP)) g |= G_SPI;
	if ((f & F_L2) && p.l3 != 0xFFFFu) g |= G_L3OK;
	x.gates = g;
	const bool qinq = (f & F_QINQ) != 0;
	const uint32_t l3 = p.l3, l4 = p.l4;
	if (used & (1u << MI_K_ETH0)) x.eth0 = r16(k, 12);
	if (used & (1u << MI_K_ETHX)) x.ethx = r16(k, qinq ? 20u : 16u);
	if (used & ((1u << MI_K_VID0) | (1u << MI_K_PCP0))) {
		uint32_t t = r16(k, 14);
		x.vid0 = t & 0xff0fu;
		x.pcp0 = (t & 0xffu) >> 5;
	}
	if (used & (1u << MI_K_VIDX)) x.vidx = r16(k, qinq ? 18u : 14u) & 0xff0fu;
	if (used & (1u << MI_K_DMAC)) {
		x.dmac0 = r32(k, 0);
		x.dmac1 = r16(k, 4);
	}
	if (used & (1u << MI_K_PROTO))
		x.proto = (f & F_IPV4) ? rb(k, l3 + 9) : rb(k, l3 + 6);
	if (used & (1u << MI_K_DSCP)) {
		if (f & F_IPV4) {
			x.dscp = rb(k, l3 + 1) >> 2;
		} else {
			uint32_t v = be32(k, l3);
			x.dscp = (v & 0x0fc00000u) >> 22;
		}
	}
	if (used & ((1u << MI_K_UDP_DPORT) | (1u << MI_K_TCP_DPORT) |
		    (1u << MI_K_UDP_SPORT) | (1u << MI_K_TCP_SPORT)))
		x.ports = (f & (F_UDP | F_TCP)) ? r32(k, l4) : 0u;
	if (used & (1u << MI_K_SIP)) x.sip = r32(k, l3 + 12);
	if (used & (1u << MI_K_DIP)) x.dip = r32(k, l3 + 16);
	if (used & (1u << MI_K_SIP6)) {
#pragma unroll
		for (int i = 0; i < 4; ++i)
			x.s6[i] = r32(k, l3 + 8 + 4 * i);
	}
	if (used & (1u << MI_K_DIP6)) {
#pragma unroll
		for (int i = 0; i < 4; ++i)
			x.d6[i] = r32(k, l3 + 24 + 4 * i);
	}
	if (used & (1u << MI_K_SPI))
		x.spi = (f & F_AH) ? r32(k, l4 + 4) : r32(k, l4);
}

// ----------------------------------------------------------- Toeplitz hash
// thash_softrss (protocols/thash.h:82-99) with the default 40-B key
// (odp_classification.c:50-58), key words in big-endian order.
__constant__ uint32_t c_rss_key[10] = {
	0x6d5a56dau, 0x255b0ec2u, 0x4167253du, 0x43a38fb0u, 0xd0ca2bcbu,
	0xae7b30b4u, 0x77cb2da3u, 0x8030f20cu, 0x6a42b73bu, 0xbeac01fau,
};

__device__ __forceinline__ uint32_t thash_word(uint32_t w, uint32_t j)
{
	uint32_t kj = c_rss_key[j], kn = c_rss_key[j + 1], h = 0;
	while (w) {
		uint32_t p = 31u - __builtin_clz(w);   // bit position from LSB
		uint32_t i = 31u - p;                  // reference loop index
		h ^= (kj << i) | (i ? (kn >> (32u - i)) : 0u);
		w &= ~(1u << p);
	}
	return h;
}

// packet_rss_hash, odp_classification.c:1773-1839
__device__ uint32_t rss_hash(const Pkt &k, const Parsed &p, uint32_t hp)
{
	const uint32_t f = p.flags;
	uint32_t h = 0, j = 0;
	bool l4 = ((f & F_TCP) && (hp & 8u)) || ((f & F_UDP) && (hp & 4u));
	if (f & F_IPV4) {
		if (hp & 1u) {
			h ^= thash_word(r32(k, p.l3 + 12), 0);
			h ^= thash_word(r32(k, p.l3 + 16), 1);
			j = 2;
		}
		if (l4) {
			// without L3 hashing the reference hashes an uninitialised word 0;
			// here word 0 is taken as zero (undefined in the reference)
			if (j == 2)
				h ^= thash_word(r32(k, p.l4), 2);
		}
	} else if (f & F_IPV6) {
		if (hp & 2u) {
#pragma unroll
			for (uint32_t i = 0; i < 4; ++i) {
				h ^= thash_word(be32(k, p.l3 + 8 + 4 * i), i);
				h ^= thash_word(be32(k, p.l3 + 24 + 4 * i), 4 + i);
			}
			j = 8;
		}
		if (l4 && j == 8)
			h ^= thash_word(r32(k, p.l4), 8);
	}
	return h;
}

// ----------------------------------------------------------- term verifier
__device__ __forceinline__ bool eq1(uint32_t x, uint32_t m, uint32_t v)
{
	return (x & m) == v;
}

// verify one compiled term (all wave-uniform inputs in SGPRs except the
// packet fields); the kind switch is a scalar branch.
__device__ __forceinline__ bool term_ok(const mi_term_t *__restrict__ t, const Pkt &k,
					const Parsed &p, const Fields &x)
{
	const uint32_t kind = __builtin_amdgcn_readfirstlane(t->kind);
	const uint32_t m0 = __builtin_amdgcn_readfirstlane(t->mask[0]);
	const uint32_t v0 = __builtin_amdgcn_readfirstlane(t->value[0]);
	const uint32_t g = x.gates;
	switch (kind) {
	case MI_K_LEN:
		return eq1(k.len, m0, v0);
	case MI_K_ETH0:
		return (g & G_ETH) && eq1(x.eth0, m0, v0);
	case MI_K_ETHX:
		return (g & G_VLANX) && eq1(x.ethx, m0, v0);
	case MI_K_VID0:
		return (g & G_VLAN0) && eq1(x.vid0, m0, v0);
	case MI_K_VIDX:
		return (g & G_VLANX) && eq1(x.vidx, m0, v0);
	case MI_K_PCP0:
		return (g & G_VLAN0) && eq1(x.pcp0, m0, v0);
	case MI_K_DMAC: {
		const uint32_t m1 = __builtin_amdgcn_readfirstlane(t->mask[1]);
		const uint32_t v1 = __builtin_amdgcn_readfirstlane(t->value[1]);
		return (g & G_ETH) && eq1(x.dmac0, m0, v0) && eq1(x.dmac1, m1, v1);
	}
	case MI_K_PROTO:
		return (g & (G_V4 | G_V6)) && eq1(x.proto, m0, v0);
	case MI_K_DSCP:
		return (g & (G_V4 | G_V6)) && eq1(x.dscp, m0, v0);
	case MI_K_UDP_DPORT:
	case MI_K_UDP_SPORT:
		return (g & G_UDP) && eq1(x.ports, m0, v0);
	case MI_K_TCP_DPORT:
	case MI_K_TCP_SPORT:
		return (g & G_TCP) && eq1(x.ports, m0, v0);
	case MI_K_SIP:
		return (g & G_V4) && eq1(x.sip, m0, v0);
	case MI_K_DIP:
		return (g & G_V4) && eq1(x.dip, m0, v0);
	case MI_K_SIP6:
	case MI_K_DIP6: {
		const uint32_t *a = (kind == MI_K_SIP6) ? x.s6 : x.d6;
		bool ok = (g & G_V6) && eq1(a[0], m0, v0);
#pragma unroll
		for (int i = 1; i < 4; ++i) {
			const uint32_t mi = __builtin_amdgcn_readfirstlane(t->mask[i]);
			const uint32_t vi = __builtin_amdgcn_readfirstlane(t->value[i]);
			ok = ok && eq1(a[i], mi, vi);
		}
		return ok;
	}
	case MI_K_SPI:
		return (g & G_SPI) && eq1(x.spi, m0, v0);
	case MI_K_CUSTOM_FRAME:
	case MI_K_CUSTOM_L3: {
		const uint32_t toff = __builtin_amdgcn_readfirstlane(t->offset);
		const uint32_t sz = __builtin_amdgcn_readfirstlane(t->size);
		uint32_t o = toff;
		bool ok = true;
		if (kind == MI_K_CUSTOM_L3) {
			ok = (g & G_L3OK) != 0;
			o = p.l3 + toff;
		}
		// verify_pmr_custom_*: "packet_len <= offset + val_sz" -> no match (u32 math)
		ok = ok && !(k.len <= o + sz);
		if (ok) {
			ok = eq1(r32(k, o), m0, v0);
#pragma unroll
			for (int i = 1; i < 4; ++i) {
				const uint32_t mi = __builtin_amdgcn_readfirstlane(t->mask[i]);
				const uint32_t vi = __builtin_amdgcn_readfirstlane(t->value[i]);
				if (sz > 4u * i)
					ok = ok && eq1(r32(k, o + 4u * i), mi, vi);
			}
		}
		return ok;
	}
	case MI_K_ALWAYS:
		return true;
	default:   // MI_K_NEVER (LD_VNI) and anything unknown
		return false;
	}
}

// ------------------------------------------------------------------ kernel
struct KArgs {
	const uint8_t *pkts;
	const uint32_t *off;
	const uint16_t *len;
	uint32_t n;
	const uint8_t *tbl;
	mi_cls_result_t *out;
	unsigned long long *stats;   // num_cos counters, or NULL
	uint32_t stats_mask[8];
};

__device__ __forceinline__ bool stats_bit(const KArgs &a, uint32_t c)
{
	return c < MAX_STATS_COS && ((a.stats_mask[c >> 5] >> (c & 31u)) & 1u);
}

__global__ __launch_bounds__(BLOCK) void mi_cls_kernel(KArgs a)
{
	__shared__ uint32_t s_win[WAVES_PER_BLOCK * WAVE * WSTRIDE];
	__shared__ uint32_t s_cnt[MAX_STATS_COS];

	const uint32_t lane = threadIdx.x & (WAVE - 1);
	const uint32_t wave = threadIdx.x >> 6;
	uint32_t *W = s_win + wave * WAVE * WSTRIDE;

	const mi_tbl_hdr_t *hdr = (const mi_tbl_hdr_t *)a.tbl;
	const mi_cos_t *cos_tbl = (const mi_cos_t *)(a.tbl + hdr->cos_off);
	const mi_rule_t *rule_tbl = (const mi_rule_t *)(a.tbl + hdr->rule_off);
	const mi_term_t *term_tbl = (const mi_term_t *)(a.tbl + hdr->term_off);
	const int32_t def_cos = __builtin_amdgcn_readfirstlane(hdr->default_cos);
	const int32_t err_cos = __builtin_amdgcn_readfirstlane(hdr->error_cos);
	const uint32_t def_valid = __builtin_amdgcn_readfirstlane(hdr->default_valid);
	const uint32_t used = __builtin_amdgcn_readfirstlane(hdr->used_kinds);
	const uint32_t max_hops = __builtin_amdgcn_readfirstlane(hdr->max_hops);
	const bool stats_on = a.stats != nullptr;

	if (stats_on) {
		for (uint32_t i = threadIdx.x; i < MAX_STATS_COS; i += BLOCK)
			s_cnt[i] = 0;
	}

	for (uint32_t bt = blockIdx.x; (uint64_t)bt * BLOCK < a.n; bt += gridDim.x) {
		const uint32_t base = bt * BLOCK + wave * WAVE;
		const uint32_t pi = base + lane;
		const bool valid = pi < a.n;
		const uint32_t my_off = valid ? a.off[pi] : 0u;
		const uint32_t my_len = valid ? (uint32_t)a.len[pi] : 0u;

		__syncthreads();   // previous tile's windows fully consumed
		// ---- stage the first WIN bytes of the wave's 64 packets into LDS
#pragma unroll
		for (uint32_t r = 0; r < 8; ++r) {
			const uint32_t q = r * 8u + (lane >> 3);
			const uint32_t c = lane & 7u;
			const uint32_t q_off = __shfl(my_off, (int)q);
			const uint32_t q_len = __shfl(my_len, (int)q);
			const uint32_t b0 = c * 16u;
			uint4 d = make_uint4(0, 0, 0, 0);
			if (b0 < q_len) {
				const uint8_t *src = a.pkts + q_off + b0;
				if ((q_off & 15u) == 0u) {
					d = *(const uint4 *)src;
				} else {
					uint32_t t[4];
#pragma unroll
					for (int i = 0; i < 4; ++i)
						t[i] = (uint32_t)src[4 * i] | ((uint32_t)src[4 * i + 1] << 8) |
						       ((uint32_t)src[4 * i + 2] << 16) | ((uint32_t)src[4 * i + 3] << 24);
					d = make_uint4(t[0], t[1], t[2], t[3]);
				}
				const uint32_t rem = q_len - b0;   // bytes of the piece inside the frame
				if (rem < 16u) {
					uint32_t t[4] = { d.x, d.y, d.z, d.w };
#pragma unroll
					for (uint32_t i = 0; i < 4; ++i) {
						uint32_t lo = 4u * i;
						uint32_t keep = rem <= lo ? 0u : (rem >= lo + 4u ? 0xffffffffu
								: (0xffffffffu >> (8u * (lo + 4u - rem))));
						t[i] &= keep;
					}
					d = make_uint4(t[0], t[1], t[2], t[3]);
				}
			}
			uint32_t *dst = W + q * WSTRIDE + c * 4u;
			dst[0] = d.x;
			dst[1] = d.y;
			dst[2] = d.z;
			dst[3] = d.w;
		}
		W[lane * WSTRIDE + 32] = 0u;
		__syncthreads();

		Pkt k;
		k.w = W + lane * WSTRIDE;
		k.g = a.pkts + my_off;
		k.len = my_len;

		Parsed p = parse_packet(k);

		// ---- select the starting CoS (cls_select_cos, odp_classification.c:1694-1726)
		int32_t cur = -1;
		bool pend = false;
		uint32_t outcome = MI_CLS_OUT_ENQ;
		if (!valid) {
			outcome = MI_CLS_OUT_DISCARD;
		} else if (p.ret < 0) {
			outcome = MI_CLS_OUT_PARSE_DROP;
		} else if (p.err) {
			cur = err_cos;
		} else {
			cur = def_cos;
			pend = def_cos >= 0 && def_valid;
		}

		Fields x;
		if (__ballot(pend))
			load_fields(k, p, used, x);

		// ---- CoS descent as a wavefront waterfall (match_pmr_cos, :1624-1667)
		uint32_t hops = 0, mark = 0;
		bool matched = false, loop = false;
		for (;;) {
			const unsigned long long pm = __ballot(pend);
			if (pm == 0ull)
				break;
			const int32_t c = __builtin_amdgcn_readlane(cur, (int)__builtin_ctzll(pm));
			const bool in_grp = pend && cur == c;
			const mi_cos_t *cd = cos_tbl + c;
			const uint32_t rb0 = __builtin_amdgcn_readfirstlane(cd->rule_begin);
			const uint32_t nr = __builtin_amdgcn_readfirstlane(cd->num_rules);
			bool done = false;
			uint32_t nxt = 0, nmark = 0;
			for (uint32_t r = 0; r < nr; ++r) {
				const bool cand = in_grp && !done;
				if (__ballot(cand) == 0ull)
					break;
				const mi_rule_t *ru = rule_tbl + rb0 + r;
				const uint32_t tb = __builtin_amdgcn_readfirstlane(ru->term_begin);
				const uint32_t nt = __builtin_amdgcn_readfirstlane(ru->num_terms);
				bool ok = cand;
				for (uint32_t t = 0; t < nt; ++t) {
					if (__ballot(ok) == 0ull)
						break;
					ok = ok && term_ok(term_tbl + tb + t, k, p, x);
				}
				if (ok) {
					nxt = __builtin_amdgcn_readfirstlane(ru->dst_cos);
					nmark = __builtin_amdgcn_readfirstlane(ru->mark);
					done = true;
				}
			}
			if (in_grp) {
				if (done) {
					cur = (int32_t)nxt;
					mark = nmark;
					matched = true;
					++hops;
					if (stats_on && stats_bit(a, nxt))
						atomicAdd(&s_cnt[nxt], 1u);
					if (hops > max_hops) {
						loop = true;
						pend = false;
					}
				} else {
					pend = false;
				}
			}
		}

		// ---- final CoS -> outcome / queue (_odp_cls_classify_packet, :1742-1771)
		uint32_t flags = p.flags, out_mark = 0, queue = 0, cos_idx = 0xFFu;
		if (matched && !loop) {
			flags &= ~F_CLS_MARK;
			if (mark) {
				flags |= F_CLS_MARK;
				out_mark = mark;
			}
		}
		if (loop) {
			outcome = MI_CLS_OUT_LOOP;
			hops = 0xFFu;
		} else if (valid && p.ret >= 0) {
			int32_t fc;
			if (p.err) {
				fc = err_cos;
				if (stats_on && fc >= 0 && stats_bit(a, (uint32_t)fc))
					atomicAdd(&s_cnt[fc], 1u);
			} else if (matched && cur != def_cos) {
				fc = cur;
			} else {
				fc = def_cos;
				if (stats_on && fc >= 0 && stats_bit(a, (uint32_t)fc))
					atomicAdd(&s_cnt[fc], 1u);
			}
			if (fc < 0) {
				outcome = MI_CLS_OUT_DISCARD;
			} else {
				const mi_cos_t cdesc = cos_tbl[fc];
				cos_idx = cdesc.index;
				if (cdesc.action == 1u) {
					outcome = MI_CLS_OUT_COS_DROP;
				} else {
					outcome = MI_CLS_OUT_ENQ;
					if (cdesc.num_queue > 1u) {
						uint32_t h = rss_hash(k, p, cdesc.hash_proto) & 31u;
						queue = h % cdesc.num_queue;
					}
				}
			}
		}

		if (valid) {
			uint4 rec;
			rec.x = flags;
			rec.y = (p.err & 0xffu) | ((outcome & 0xffu) << 8) | ((cos_idx & 0xffu) << 16) |
				((hops & 0xffu) << 24);
			rec.z = (queue & 0xffffu) | ((out_mark & 0xffffu) << 16);
			rec.w = (p.l3 & 0xffffu) | ((p.l4 & 0xffffu) << 16);
			*(uint4 *)(a.out + pi) = rec;
		}
	}

	if (stats_on) {
		__syncthreads();
		for (uint32_t i = threadIdx.x; i < MAX_STATS_COS; i += BLOCK)
			if (s_cnt[i])
				atomicAdd(a.stats + i, (unsigned long long)s_cnt[i]);
	}
}

// ------------------------------------------------------------------- host
struct mi_cls_ctx {
	int device;
	uint8_t *d_tbl;
	size_t tbl_cap;
	size_t tbl_bytes;
	int loaded;
	unsigned long long *d_stats;
	int stats_on;
	uint32_t stats_mask[8];
	int num_cu;
};

#define HIP_OK(x) do { if ((x) != hipSuccess) return -EIO; } while (0)

extern "C" int mi_cls_device_count(void)
{
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess)
		return 0;
	return n;
}

extern "C" int mi_cls_ctx_create(int device, mi_cls_ctx_t **out)
{
	if (!out)
		return -EINVAL;
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
		return -ENODEV;
	mi_cls_ctx_t *c = (mi_cls_ctx_t *)calloc(1, sizeof(*c));
	if (!c)
		return -ENOMEM;
	c->device = device;
	int cur = 0;
	(void)hipGetDevice(&cur);
	if (hipSetDevice(device) != hipSuccess) {
		free(c);
		return -EIO;
	}
	hipDeviceProp_t prop;
	if (hipGetDeviceProperties(&prop, device) == hipSuccess)
		c->num_cu = prop.multiProcessorCount;
	else
		c->num_cu = 256;
	if (hipMalloc((void **)&c->d_stats, MAX_STATS_COS * sizeof(unsigned long long)) != hipSuccess ||
	    hipMemset(c->d_stats, 0, MAX_STATS_COS * sizeof(unsigned long long)) != hipSuccess) {
		free(c);
		(void)hipSetDevice(cur);
		return -ENOMEM;
	}
	(void)hipSetDevice(cur);
	*out = c;
	return 0;
}

extern "C" int mi_cls_ctx_destroy(mi_cls_ctx_t *c)
{
	if (!c)
		return -EINVAL;
	(void)hipSetDevice(c->device);
	if (c->d_tbl)
		(void)hipFree(c->d_tbl);
	if (c->d_stats)
		(void)hipFree(c->d_stats);
	free(c);
	return 0;
}

static int validate_tbl(const void *tbl, size_t bytes)
{
	if (!tbl || bytes < sizeof(mi_tbl_hdr_t))
		return -EINVAL;
	const mi_tbl_hdr_t *h = (const mi_tbl_hdr_t *)tbl;
	if (h->magic != MI_CLS_TBL_MAGIC || h->version != MI_CLS_TBL_VERSION || h->total_bytes != bytes)
		return -EINVAL;
	if (h->num_cos > 256 || h->cos_off != sizeof(mi_tbl_hdr_t))
		return -EINVAL;
	if ((uint64_t)h->rule_off != (uint64_t)h->cos_off + (uint64_t)h->num_cos * sizeof(mi_cos_t) ||
	    (uint64_t)h->term_off != (uint64_t)h->rule_off + (uint64_t)h->num_rules * sizeof(mi_rule_t) ||
	    (uint64_t)h->total_bytes != (uint64_t)h->term_off + (uint64_t)h->num_terms * sizeof(mi_term_t))
		return -EINVAL;
	if (h->default_cos >= (int32_t)h->num_cos || h->error_cos >= (int32_t)h->num_cos ||
	    h->default_cos < -1 || h->error_cos < -1)
		return -EINVAL;
	// every index the kernel follows must stay inside the table
	const uint8_t *b = (const uint8_t *)tbl;
	const mi_cos_t *cs = (const mi_cos_t *)(b + h->cos_off);
	const mi_rule_t *rs = (const mi_rule_t *)(b + h->rule_off);
	const mi_term_t *ts = (const mi_term_t *)(b + h->term_off);
	for (uint32_t i = 0; i < h->num_cos; ++i) {
		if ((uint64_t)cs[i].rule_begin + cs[i].num_rules > h->num_rules)
			return -EINVAL;
		if (cs[i].num_queue < 1 || cs[i].num_queue > 32)
			return -EINVAL;
	}
	for (uint32_t i = 0; i < h->num_rules; ++i) {
		if (rs[i].dst_cos >= h->num_cos || rs[i].num_terms > 8 ||
		    (uint64_t)rs[i].term_begin + rs[i].num_terms > h->num_terms)
			return -EINVAL;
	}
	for (uint32_t i = 0; i < h->num_terms; ++i) {
		if (ts[i].kind >= MI_K_COUNT || ts[i].size > 16)
			return -EINVAL;
	}
	return 0;
}

extern "C" int mi_cls_rules_load(mi_cls_ctx_t *c, const void *tbl, size_t bytes, void *stream)
{
	if (!c)
		return -EINVAL;
	int rc = validate_tbl(tbl, bytes);
	if (rc)
		return rc;
	HIP_OK(hipSetDevice(c->device));
	if (bytes > c->tbl_cap) {
		// stream-ordered free of the old table: wait for in-flight work first
		if (c->d_tbl) {
			HIP_OK(hipStreamSynchronize((hipStream_t)stream));
			(void)hipFree(c->d_tbl);
			c->d_tbl = nullptr;
		}
		size_t cap = bytes < 4096 ? 4096 : bytes;
		HIP_OK(hipMalloc((void **)&c->d_tbl, cap));
		c->tbl_cap = cap;
	}
	// the blob lives in caller memory that may be freed right after return
	HIP_OK(hipMemcpyAsync(c->d_tbl, tbl, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
	HIP_OK(hipStreamSynchronize((hipStream_t)stream));
	c->tbl_bytes = bytes;
	c->loaded = 1;
	return 0;
}

extern "C" int mi_cls_classify(mi_cls_ctx_t *c, const uint8_t *pkts, const uint32_t *off,
			       const uint16_t *len, uint32_t n, mi_cls_result_t *out, void *stream)
{
	if (!c || !c->loaded)
		return -EINVAL;
	if (n == 0)
		return 0;
	if (!pkts || !off || !len || !out)
		return -EINVAL;
	if (((uintptr_t)out & 15u) != 0)
		return -EINVAL;
	HIP_OK(hipSetDevice(c->device));
	KArgs a;
	a.pkts = pkts;
	a.off = off;
	a.len = len;
	a.n = n;
	a.tbl = c->d_tbl;
	a.out = out;
	a.stats = c->stats_on ? c->d_stats : nullptr;
	memcpy(a.stats_mask, c->stats_mask, sizeof(a.stats_mask));
	uint32_t tiles = (n + BLOCK - 1) / BLOCK;
	uint32_t max_grid = (uint32_t)c->num_cu * 16u;
	uint32_t grid = tiles < max_grid ? tiles : max_grid;
	hipLaunchKernelGGL(mi_cls_kernel, dim3(grid), dim3(BLOCK), 0, (hipStream_t)stream, a);
	if (hipGetLastError() != hipSuccess)
		return -EIO;
	return 0;
}

extern "C" int mi_cls_stats_enable(mi_cls_ctx_t *c, const uint32_t mask[8])
{
	if (!c)
		return -EINVAL;
	int any = 0;
	for (int i = 0; i < 8; ++i) {
		c->stats_mask[i] = mask ? mask[i] : 0u;
		any |= c->stats_mask[i] != 0;
	}
	c->stats_on = any;
	return 0;
}

extern "C" int mi_cls_stats_read(mi_cls_ctx_t *c, uint64_t *host, uint32_t num)
{
	if (!c || !host || num > MAX_STATS_COS)
		return -EINVAL;
	HIP_OK(hipSetDevice(c->device));
	HIP_OK(hipDeviceSynchronize());
	HIP_OK(hipMemcpy(host, c->d_stats, num * sizeof(uint64_t), hipMemcpyDeviceToHost));
	return 0;
}

extern "C" int mi_cls_stats_reset(mi_cls_ctx_t *c)
{
	if (!c)
		return -EINVAL;
	HIP_OK(hipSetDevice(c->device));
	HIP_OK(hipDeviceSynchronize());
	HIP_OK(hipMemset(c->d_stats, 0, MAX_STATS_COS * sizeof(unsigned long long)));
	return 0;
}

extern "C" const char *mi_cls_strerror(int err)
{
	switch (-err) {
	case 0: return "success";
	case EINVAL: return "invalid argument or malformed rule table";
	case ENODEV: return "no such HIP device";
	case ENOMEM: return "out of device memory";
	case EIO: return "HIP runtime error";
	default: return "unknown error";
	}
}
