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
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mi_cls.h"

#include <algorithm>
#include <array>
#include <map>
#include <vector>

#define WAVE 64
#ifndef WAVES_PER_BLOCK
#define WAVES_PER_BLOCK 4
#endif
#define BLOCK (WAVE * WAVES_PER_BLOCK)
#ifndef WIN
#define WIN 128            // staged header window, bytes (multiple of 16)
#endif
#define WROWS (WIN / 4 + 1)     // LDS dword rows per wave window (+1 zero row)
#define NPIECE (WIN / 16)       // 16-B pieces per window
#ifndef MIN_WAVES_PER_EU
#define MIN_WAVES_PER_EU 1
#endif
#ifndef PREFETCH
#define PREFETCH 1          // software-pipeline the next tile's loads
#endif
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
// The LDS window of a wave is dword-major, lane-minor: dword i of lane l's
// packet lives at W[i * WAVE + l].  Any per-lane byte offset then reads
// conflict-free (lane l always hits bank l mod 32), whatever the packets'
// header layouts.
struct Pkt {
	const uint32_t *w;      // &W[lane]
	const uint8_t *g;       // packet start in HBM
	uint32_t len;           // frame_len
};

__device__ __forceinline__ uint32_t rb(const Pkt &k, uint32_t o)
{
	if (o < WIN)
		return (k.w[(o >> 2) * WAVE] >> ((o & 3u) * 8u)) & 0xffu;
	return o < k.len ? (uint32_t)k.g[o] : 0u;
}

// 4 bytes starting at byte offset o, little-endian (== the reference's raw load)
__device__ __forceinline__ uint32_t r32(const Pkt &k, uint32_t o)
{
	if (o <= WIN - 4u) {
		uint32_t i = o >> 2;
		return __builtin_amdgcn_alignbyte(k.w[(i + 1) * WAVE], k.w[i * WAVE], o & 3u);
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

// Branch-light parse for the common header shapes.  Under _odp_parse_eth's
// rules the L3 offset is one of 14/18/22/26/30 (DIX or SNAP, plus 0-2 tags),
// so l3 and every L4 offset reached from it are 2 (mod 4): the parse becomes
// three batches of independent LDS reads (bytes 0-31, the IP header, the
// L4 header) combined with selects instead of a branch chain.  Lanes it does
// not cover -- IPv6 HBH/routing chains, or a field past the staged window --
// report `slow` and take parse_packet() instead; for every other lane the
// result is identical to parse_packet's.
__device__ __forceinline__ uint32_t bsw16(uint32_t v)   // be16 of the low half
{
	return ((v & 0xffu) << 8) | ((v >> 8) & 0xffu);
}

__device__ __forceinline__ Parsed parse_fast(const Pkt &k, bool &slow)
{
	Parsed r;
	const uint32_t len = k.len;
	uint32_t w[8];
#pragma unroll
	for (int i = 0; i < 8; ++i)
		w[i] = k.w[i * WAVE];

	uint32_t f = F_L2 | F_ETH;
	if (len > 1514u)
		f |= F_JUMBO;
	if (w[0] & 1u)
		f |= F_ETH_MCAST;
	if (w[0] == 0xffffffffu && (w[1] & 0xffffu) == 0xffffu)
		f |= F_ETH_BCAST;
	const uint32_t et0 = bsw16(w[3]);
	const bool snap = et0 < 1514u;
	const bool snap_err = snap && et0 > len - 14u;
	uint32_t e = snap ? bsw16(w[5]) : et0;
	uint32_t off = snap ? 22u : 14u;
	// outer tag: type at off+2 = 16 / 24
	const bool qinq = e == 0x88A8u;
	if (qinq) {
		e = snap ? bsw16(w[6]) : bsw16(w[4]);
		off += 4u;
	}
	// inner tag: type at off+2 = 16 / 20 / 24 / 28
	const bool vlan = e == 0x8100u;
	if (vlan) {
		const uint32_t j = (off + 2u) >> 2;
		const uint32_t wv = j == 4u ? w[4] : (j == 5u ? w[5] : (j == 6u ? w[6] : w[7]));
		e = bsw16(wv);
		off += 4u;
	}
	uint32_t err = 0;
	if (snap_err) {
		err = E_SNAP;
		e = 0;
		off = 14u;
	} else {
		if (qinq)
			f |= F_QINQ | F_VLAN;
		if (vlan)
			f |= F_VLAN;
		if (off > len) {
			f = F_L2;
			e = 0;
		}
	}
	const uint32_t l3 = off;
	r.l3 = l3;

	// IP header bytes l3 .. l3+27 (dwords jb .. jb+7, byte shift 2)
	const uint32_t jb = (l3 - 2u) >> 2;
	uint32_t h[8];
#pragma unroll
	for (int i = 0; i < 8; ++i)
		h[i] = k.w[(jb + i) * WAVE];
	uint32_t hb[7];
#pragma unroll
	for (int i = 0; i < 7; ++i)
		hb[i] = __builtin_amdgcn_alignbyte(h[i + 1], h[i], 2u);   // bytes l3+4i .. +3

	const bool is4 = e == 0x0800u, is6 = e == 0x86DDu, isarp = e == 0x0806u;
	uint32_t ip_proto = 255u, l4 = 0xFFFFu;
	bool non_first = false;
	slow = false;
	if (is4 || is6 || isarp)
		f |= F_L3;
	if (isarp)
		f |= F_ARP;
	if (is4) {
		f |= F_IPV4;
		const uint32_t vi = hb[0] & 0xffu, ihl = vi & 0xfu;
		const uint32_t tot = bsw16(hb[0] >> 16);
		if (ihl < 5u || (vi >> 4) != 4u || 20u > len - l3 || tot > len - l3) {
			err |= E_IP;
			ip_proto = 0;
		} else {
			const uint32_t frag = bsw16(hb[1] >> 16);
			const uint32_t dst = __builtin_bswap32(hb[4]);
			l4 = l3 + ihl * 4u;
			if (ihl > 5u)
				f |= F_IPOPT;
			if (frag & 0x3fffu)
				f |= F_IPFRAG;
			non_first = (frag & 0x1fffu) != 0;
			if (dst == 0xffffffffu)
				f |= F_IP_BCAST;
			if ((dst >> 28) == 0xeu)
				f |= F_IP_MCAST;
			ip_proto = (hb[2] >> 8) & 0xffu;
		}
	} else if (is6) {
		f |= F_IPV6;
		const uint32_t plen = bsw16(hb[1]);
		if (((hb[0] & 0xffu) >> 4) != 6u || 40u > len - l3 || plen + 40u > len - l3) {
			err |= E_IP;
			ip_proto = 0;
		} else {
			if ((hb[6] & 0xffu) == 0xffu)
				f |= F_IP_MCAST;
			const uint32_t nh = (hb[1] >> 16) & 0xffu;
			if (nh == 0u || nh == 43u)
				slow = true;                 // extension chain: general parser
			if (nh == 44u)
				f |= F_IPOPT | F_IPFRAG;
			ip_proto = nh;
			l4 = l3 + 40u;
		}
	}

	const bool l4hdr = (ip_proto == 6u || ip_proto == 17u || ip_proto == 132u) && !non_first;
	// L4 header bytes l4 .. l4+15 (dwords jl .. jl+4, byte shift 2)
	uint32_t lb[4] = { 0, 0, 0, 0 };
	if (l4hdr) {
		if (l4 + 18u > WIN) {
			slow = true;                         // past the staged window
		} else {
			const uint32_t jl = (l4 - 2u) >> 2;
			uint32_t m[5];
#pragma unroll
			for (int i = 0; i < 5; ++i)
				m[i] = k.w[(jl + i) * WAVE];
#pragma unroll
			for (int i = 0; i < 4; ++i)
				lb[i] = __builtin_amdgcn_alignbyte(m[i + 1], m[i], 2u);
		}
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
			if (l4 + 20u > len)
				ret = -1;
			else if (((lb[3] & 0xffu) >> 4) < 5u)
				err |= E_TCP;
		}
		break;
	case 17u:
		f |= F_UDP;
		if (!non_first) {
			if (l4 + 8u > len) {
				ret = -1;
			} else {
				const uint32_t ulen = bsw16(lb[1]);
				if (ulen < 8u)
					err |= E_UDP;
				else if ((lb[0] >> 16) == 0x9411u && ulen > 4u && lb[2] != 0u)
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
			if (l4 + 12u > len)
				ret = -1;
			else if (((len - l4) & 0xffffu) < 12u)
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
	if (!is4 && !is6 && !isarp)
		f &= ~F_L3;
	r.l4 = l4;
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
__device__ __forceinline__ uint32_t rss_hash(const Pkt &k, const Parsed &p, uint32_t hp)
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

// ------------------------------------------------------ device rule program
// mi_cls_rules_load() assembles the mi_cls.h table into this private,
// read-only encoding, read by the kernel through the constant address space
// (scalar loads: every lane of a wave tests the same rule):
//
//   words [0, 16)          header  (DH_* below)
//   words [cos_off, ...)   8 words per CoS slot: rule record index, #rules,
//                          meta = action | num_queue<<8 | hash_proto<<16 | index<<24,
//                          valid, bit-vector block offset (0 = linear scan)
//   words [prog_off, ...)  16-word rule records, CoS rules contiguous in scan order:
//        w0  = inline terms | ext terms<<4 | mark<<16
//        w1  = dst CoS | ext word offset<<8
//        w2.. terms: op word (kind | size<<8 | nw<<16), [offset word for custom
//             kinds], then nw (mask, value) word pairs; terms that do not fit
//             the 14 inline words continue at the ext offset.
typedef const __attribute__((address_space(4))) uint32_t *cword_t;

enum { DH_MAGIC = 0, DH_NCOS, DH_DEFAULT, DH_ERROR, DH_DEFAULT_VALID, DH_USED, DH_MAX_HOPS,
       DH_COS_OFF, DH_PROG_OFF, DH_TOTAL, DH_WORDS = 16 };
#define DEV_MAGIC 0x32564544u   // "DEV2"
#define REC_WORDS 16u
#define COS_WORDS 8u
#define BV_MAX_CLS 8u
#define BV_CLS_WORDS 16u
#define BV_EMPTY 0xFFFFFFFFu

// Bit-vector (BV) block of a CoS, used when its rules fall into at most
// BV_MAX_CLS key classes.  A key class is one (term kind, mask[, offset,
// size]) combination; for every class the block holds a hash table
// key -> bitmap row over the CoS's rules (bit r = rule r's terms of that
// class all equal the key, or rule r has no term of that class), row 0 being
// the "no term of this class" row used when the packet lacks the field.
// A packet's matching rules are the AND of its rows; the lowest set bit is
// the first rule in scan order whose every term matches -- exactly the rule
// match_pmr_cos picks (odp_classification.c:1631-1650).
//   bv[0] = W (32-bit words per row), bv[1] = #classes, bv[2] = alive row offset
//   bv[4 + 16 k ...] class k: kind, nkey, 0, offset, size, mask[4],
//                    table mask, table offset, rows offset
//   table slot: nkey key words + row index (BV_EMPTY = free slot)

__device__ __forceinline__ bool eq1(uint32_t x, uint32_t m, uint32_t v)
{
	return (x & m) == v;
}

// verify_pmr_<term> for one term whose words start at prog[q] (uniform);
// returns the lane's verdict and advances q past the term.
__device__ __forceinline__ bool term_ok(cword_t prog, uint32_t &q, const Pkt &k, const Parsed &p,
					const Fields &x)
{
	const uint32_t op = prog[q];
	const uint32_t kind = op & 0xffu;
	const uint32_t g = x.gates;
	if (kind == MI_K_CUSTOM_FRAME || kind == MI_K_CUSTOM_L3) {
		const uint32_t sz = (op >> 8) & 0xffu;
		const uint32_t nw = (op >> 16) & 0xffu;
		const uint32_t toff = prog[q + 1];
		uint32_t o = toff;
		bool ok = true;
		if (kind == MI_K_CUSTOM_L3) {
			ok = (g & G_L3OK) != 0;
			o = p.l3 + toff;
		}
		// verify_pmr_custom_*: "packet_len <= offset + val_sz" -> no match (u32 math)
		ok = ok && !(k.len <= o + sz);
		if (ok) {
			for (uint32_t i = 0; i < nw; ++i)
				ok = ok && eq1(r32(k, o + 4u * i), prog[q + 2 + 2 * i], prog[q + 3 + 2 * i]);
		}
		q += 2u + 2u * nw;
		return ok;
	}
	const uint32_t m0 = prog[q + 1];
	const uint32_t v0 = prog[q + 2];
	bool ok;
	switch (kind) {
	case MI_K_LEN:
		ok = eq1(k.len, m0, v0);
		break;
	case MI_K_ETH0:
		ok = (g & G_ETH) && eq1(x.eth0, m0, v0);
		break;
	case MI_K_ETHX:
		ok = (g & G_VLANX) && eq1(x.ethx, m0, v0);
		break;
	case MI_K_VID0:
		ok = (g & G_VLAN0) && eq1(x.vid0, m0, v0);
		break;
	case MI_K_VIDX:
		ok = (g & G_VLANX) && eq1(x.vidx, m0, v0);
		break;
	case MI_K_PCP0:
		ok = (g & G_VLAN0) && eq1(x.pcp0, m0, v0);
		break;
	case MI_K_DMAC:
		ok = (g & G_ETH) && eq1(x.dmac0, m0, v0) && eq1(x.dmac1, prog[q + 3], prog[q + 4]);
		q += 2;
		break;
	case MI_K_PROTO:
		ok = (g & (G_V4 | G_V6)) && eq1(x.proto, m0, v0);
		break;
	case MI_K_DSCP:
		ok = (g & (G_V4 | G_V6)) && eq1(x.dscp, m0, v0);
		break;
	case MI_K_UDP_DPORT:
	case MI_K_UDP_SPORT:
		ok = (g & G_UDP) && eq1(x.ports, m0, v0);
		break;
	case MI_K_TCP_DPORT:
	case MI_K_TCP_SPORT:
		ok = (g & G_TCP) && eq1(x.ports, m0, v0);
		break;
	case MI_K_SIP:
		ok = (g & G_V4) && eq1(x.sip, m0, v0);
		break;
	case MI_K_DIP:
		ok = (g & G_V4) && eq1(x.dip, m0, v0);
		break;
	case MI_K_SIP6:
	case MI_K_DIP6: {
		// element-wise select: a pointer select would put the arrays on the stack
		const bool src = kind == MI_K_SIP6;
		ok = (g & G_V6) && eq1(src ? x.s6[0] : x.d6[0], m0, v0) &&
		     eq1(src ? x.s6[1] : x.d6[1], prog[q + 3], prog[q + 4]) &&
		     eq1(src ? x.s6[2] : x.d6[2], prog[q + 5], prog[q + 6]) &&
		     eq1(src ? x.s6[3] : x.d6[3], prog[q + 7], prog[q + 8]);
		q += 6;
		break;
	}
	case MI_K_SPI:
		ok = (g & G_SPI) && eq1(x.spi, m0, v0);
		break;
	case MI_K_ALWAYS:
		ok = true;
		break;
	default:   // MI_K_NEVER (LD_VNI)
		ok = false;
		break;
	}
	q += 3;
	return ok;
}

__device__ __forceinline__ uint32_t bv_hash(const uint32_t k[4])
{
	uint32_t h = k[0] * 0x9E3779B1u ^ k[1] * 0x85EBCA77u ^ k[2] * 0xC2B2AE3Du ^ k[3] * 0x27D4EB2Fu;
	h ^= h >> 15;
	h *= 0x2C1B3C6Du;
	h ^= h >> 12;
	return h;
}

// Key of a packet for one BV class: the masked field the class's terms
// compare, and whether the packet has that field at all (the term's gate).
__device__ __forceinline__ bool bv_key(cword_t cr, const Pkt &k, const Parsed &p, const Fields &x,
				       uint32_t key[4])
{
	const uint32_t kind = cr[0];
	const uint32_t m0 = cr[5], m1 = cr[6], m2 = cr[7], m3 = cr[8];
	const uint32_t g = x.gates;
	key[1] = key[2] = key[3] = 0;
	switch (kind) {
	case MI_K_LEN:
		key[0] = k.len & m0;
		return true;
	case MI_K_ETH0:
		key[0] = x.eth0 & m0;
		return g & G_ETH;
	case MI_K_ETHX:
		key[0] = x.ethx & m0;
		return g & G_VLANX;
	case MI_K_VID0:
		key[0] = x.vid0 & m0;
		return g & G_VLAN0;
	case MI_K_VIDX:
		key[0] = x.vidx & m0;
		return g & G_VLANX;
	case MI_K_PCP0:
		key[0] = x.pcp0 & m0;
		return g & G_VLAN0;
	case MI_K_DMAC:
		key[0] = x.dmac0 & m0;
		key[1] = x.dmac1 & m1;
		return g & G_ETH;
	case MI_K_PROTO:
		key[0] = x.proto & m0;
		return g & (G_V4 | G_V6);
	case MI_K_DSCP:
		key[0] = x.dscp & m0;
		return g & (G_V4 | G_V6);
	case MI_K_UDP_DPORT:
	case MI_K_UDP_SPORT:
		key[0] = x.ports & m0;
		return g & G_UDP;
	case MI_K_TCP_DPORT:
	case MI_K_TCP_SPORT:
		key[0] = x.ports & m0;
		return g & G_TCP;
	case MI_K_SIP:
		key[0] = x.sip & m0;
		return g & G_V4;
	case MI_K_DIP:
		key[0] = x.dip & m0;
		return g & G_V4;
	case MI_K_SIP6:
	case MI_K_DIP6: {
		const bool src = kind == MI_K_SIP6;
		key[0] = (src ? x.s6[0] : x.d6[0]) & m0;
		key[1] = (src ? x.s6[1] : x.d6[1]) & m1;
		key[2] = (src ? x.s6[2] : x.d6[2]) & m2;
		key[3] = (src ? x.s6[3] : x.d6[3]) & m3;
		return g & G_V6;
	}
	case MI_K_SPI:
		key[0] = x.spi & m0;
		return g & G_SPI;
	case MI_K_CUSTOM_FRAME:
	case MI_K_CUSTOM_L3: {
		const uint32_t toff = cr[3], sz = cr[4], nk = cr[1];
		uint32_t o = toff;
		bool ok = true;
		if (kind == MI_K_CUSTOM_L3) {
			ok = (g & G_L3OK) != 0;
			o = p.l3 + toff;
		}
		ok = ok && !(k.len <= o + sz);
		key[0] = 0;
		if (ok) {
			key[0] = r32(k, o) & m0;
			if (nk > 1)
				key[1] = r32(k, o + 4) & m1;
			if (nk > 2) {
				key[2] = r32(k, o + 8) & m2;
				key[3] = r32(k, o + 12) & m3;
			}
		}
		return ok;
	}
	default:
		key[0] = 0;
		return false;
	}
}

// Bit-vector evaluation of one CoS for the lanes in `act`.  `blk` is the
// CoS's BV block and `rec` its first rule record; both may be wave-uniform
// (scalar loads) or per lane (gathers), decided per call site after inlining.
// On return, lanes of `act` with a matching rule have done = true and the
// rule's destination CoS / mark in nxt / nmark.
__device__ __forceinline__ void bv_eval(cword_t blk, const uint32_t *rec, bool act, const Pkt &k,
					const Parsed &p, const Fields &x, const uint32_t *dv,
					bool &done, uint32_t &nxt, uint32_t &nmark)
{
	const uint32_t Wd = blk[0], ncls = blk[1], alive = blk[2];
	uint32_t ridx[BV_MAX_CLS];
#pragma unroll
	for (uint32_t kc = 0; kc < BV_MAX_CLS; ++kc) {
		ridx[kc] = 0;
		if (kc < ncls) {
			const cword_t cr = blk + 4u + BV_CLS_WORDS * kc;
			const uint32_t nk = cr[1], tmask = cr[9], tbl = cr[10], rows = cr[11];
			uint32_t key[4];
			const bool present = bv_key(cr, k, p, x, key);
			uint32_t row = 0;
			if (act && present) {
				uint32_t h = bv_hash(key) & tmask;
				for (uint32_t probe = 0; probe <= tmask; ++probe) {
					const uint32_t *sl = dv + tbl + h * (nk + 1u);
					const uint32_t rw = sl[nk];
					if (rw == BV_EMPTY)
						break;
					bool eq = sl[0] == key[0];
					if (nk > 1)
						eq = eq && sl[1] == key[1];
					if (nk > 2)
						eq = eq && sl[2] == key[2] && sl[3] == key[3];
					if (eq) {
						row = rw;
						break;
					}
					h = (h + 1u) & tmask;
				}
			}
			ridx[kc] = rows + row * Wd;
		}
	}
	uint32_t first = 0;
	bool found = false;
	for (uint32_t w = 0; w < Wd; ++w) {
		if (__ballot(act && !found) == 0ull)
			break;
		if (act && !found) {
			uint32_t acc = dv[alive + w];
#pragma unroll
			for (uint32_t kc = 0; kc < BV_MAX_CLS; ++kc)
				if (kc < ncls)
					acc &= dv[ridx[kc] + w];
			if (acc) {
				found = true;
				first = w * 32u + (uint32_t)__builtin_ctz(acc);
			}
		}
	}
	if (act && found) {
		const uint32_t *r = rec + first * REC_WORDS;
		nxt = r[1] & 0xffu;
		nmark = r[0] >> 16;
		done = true;
	}
}

// Linear scan of one wave-uniform CoS's rule records for the lanes in
// `grp` (verify_pmr over cos->pmr[] in order, first match wins).
__device__ __forceinline__ void linear_scan(cword_t prog, uint32_t rec0, uint32_t nr, bool grp,
					    const Pkt &k, const Parsed &p, const Fields &x,
					    bool &done, uint32_t &nxt, uint32_t &nmark)
{
	for (uint32_t r = 0; r < nr; ++r) {
		const bool cand = grp && !done;
		if (__ballot(cand) == 0ull)
			break;
		const uint32_t base = (rec0 + r) * REC_WORDS;
		const uint32_t w0 = prog[base];
		const uint32_t w1 = prog[base + 1];
		const uint32_t n_in = w0 & 0xfu, n_ext = (w0 >> 8) & 0xfu;
		// AND of the terms; stop as soon as no lane can still match
		bool ok = cand;
		uint32_t q = base + 2;
		for (uint32_t t = 0; t < n_in; ++t) {
			if (__ballot(ok) == 0ull)
				break;
			ok = term_ok(prog, q, k, p, x) && ok;
		}
		if (n_ext && __ballot(ok) != 0ull) {
			q = w1 >> 8;
			for (uint32_t t = 0; t < n_ext; ++t) {
				if (__ballot(ok) == 0ull)
					break;
				ok = term_ok(prog, q, k, p, x) && ok;
			}
		}
		if (ok) {
			nxt = w1 & 0xffu;
			nmark = w0 >> 16;
			done = true;
		}
	}
}

// Diagnostic build only (-DDIAG_STAMPS): per-phase cycle sums per wave,
// written to a debug buffer nobody else reads (cdna_hip_programming.md §7).
#ifdef DIAG_STAMPS
#define NSTAMP 8
#define STAMP(i)                                                                   \
	do {                                                                       \
		__builtin_amdgcn_sched_barrier(0);                                 \
		unsigned long long t_;                                             \
		asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_) :: "memory"); \
		__builtin_amdgcn_sched_barrier(0);                                 \
		st_acc[i] += t_ - st_last;                                         \
		st_last = t_;                                                      \
	} while (0)
#else
#define STAMP(i) do { } while (0)
#endif

// ------------------------------------------------------------------ kernel
struct KArgs {
	const uint8_t *pkts;
	const uint32_t *off;
	const uint16_t *len;
	uint32_t n;
	const uint32_t *dev;         // device rule program (constant address space)
	mi_cls_result_t *out;
	unsigned long long *stats;   // MAX_STATS_COS counters, or NULL
	unsigned long long *diag;    // DIAG_STAMPS builds only
	uint32_t stats_mask[8];
};

__device__ __forceinline__ bool stats_bit(const KArgs &a, uint32_t c)
{
	return c < MAX_STATS_COS && ((a.stats_mask[c >> 5] >> (c & 31u)) & 1u);
}

// Make this wave's LDS writes visible to its own later LDS reads by other
// lanes: LDS ops of one wave complete in order, so a wave-scope fence (which
// keeps the compiler from reordering) is all that is needed -- no block
// barrier, waves run independently.
__device__ __forceinline__ void wave_lds_sync()
{
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(BLOCK, MIN_WAVES_PER_EU) void mi_cls_kernel(KArgs a)
{
	__shared__ uint32_t s_win[WAVES_PER_BLOCK * WAVE * WROWS];
	__shared__ uint32_t s_cnt[MAX_STATS_COS];

	const uint32_t lane = threadIdx.x & (WAVE - 1);
	const uint32_t wave = threadIdx.x >> 6;
	uint32_t *W = s_win + wave * WAVE * WROWS;

	const cword_t dev = (cword_t)a.dev;
	const int32_t def_cos = (int32_t)dev[DH_DEFAULT];
	const int32_t err_cos = (int32_t)dev[DH_ERROR];
	const uint32_t def_valid = dev[DH_DEFAULT_VALID];
	const uint32_t used = dev[DH_USED];
	const uint32_t max_hops = dev[DH_MAX_HOPS];
	const cword_t cos_tbl = dev + dev[DH_COS_OFF];
	const cword_t prog = dev + dev[DH_PROG_OFF];
	const bool stats_on = a.stats != nullptr;

	if (stats_on) {
		for (uint32_t i = threadIdx.x; i < MAX_STATS_COS; i += BLOCK)
			s_cnt[i] = 0;
		__syncthreads();
	}

	// Software pipeline over this wave's tiles (64 packets each): while tile
	// t is parsed and classified, tile t+1's header windows are in flight
	// into registers and tile t+2's descriptors are being fetched.  Each
	// lane loads its own packet's window (NPIECE x 16 B).
	const uint32_t nt = (a.n + WAVE - 1) / WAVE;
	const uint32_t tstride = gridDim.x * WAVES_PER_BLOCK;
	uint32_t tile = blockIdx.x * WAVES_PER_BLOCK + wave;
	uint32_t d_off = 0, d_len = 0, n_off = 0, n_len = 0;
	uint4 d[NPIECE];
	{
		const uint32_t p0 = tile * WAVE + lane, p1 = (tile + tstride) * WAVE + lane;
		if (tile < nt && p0 < a.n) {
			d_off = a.off[p0];
			d_len = a.len[p0];
		}
		if (tile + tstride < nt && p1 < a.n) {
			n_off = a.off[p1];
			n_len = a.len[p1];
		}
#pragma unroll
		for (uint32_t r = 0; r < NPIECE; ++r) {
			d[r] = make_uint4(0, 0, 0, 0);
#ifndef DIAG_NOLOAD
			if (16u * r < d_len)
				__builtin_memcpy(&d[r], a.pkts + d_off + 16u * r, 16);
#endif
		}
	}
#ifdef DIAG_STAMPS
	unsigned long long st_acc[NSTAMP] = { 0 }, st_last;
	asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_last) :: "memory");
#endif
	for (; tile < nt; tile += tstride) {
		const uint32_t pi = tile * WAVE + lane;
		const bool valid = pi < a.n;
		if (!PREFETCH && tile != blockIdx.x * WAVES_PER_BLOCK + wave) {
			d_off = valid ? a.off[pi] : 0u;
			d_len = valid ? (uint32_t)a.len[pi] : 0u;
#pragma unroll
			for (uint32_t r = 0; r < NPIECE; ++r) {
				d[r] = make_uint4(0, 0, 0, 0);
				if (16u * r < d_len)
					__builtin_memcpy(&d[r], a.pkts + d_off + 16u * r, 16);
			}
		}
		const uint32_t my_off = d_off, my_len = d_len;

		wave_lds_sync();   // previous tile's window reads are done
#pragma unroll
		for (uint32_t r = 0; r < NPIECE; ++r) {
			uint32_t t[4] = { d[r].x, d[r].y, d[r].z, d[r].w };
			const uint32_t b0 = 16u * r;
			// zero the bytes past the frame (reads beyond frame_len give 0)
			// only the piece holding the frame's last byte is partial; pieces
			// past the frame were never loaded and are already zero
			const uint32_t rem = my_len - b0;
			if (my_len > b0 && rem < 16u) {
#pragma unroll
				for (uint32_t i = 0; i < 4; ++i) {
					const uint32_t lo = 4u * i;
					const uint32_t keep = rem <= lo ? 0u : (rem >= lo + 4u ? 0xffffffffu
						: (0xffffffffu >> (8u * (lo + 4u - rem))));
					t[i] &= keep;
				}
			}
#pragma unroll
			for (uint32_t i = 0; i < 4; ++i)
				W[(4u * r + i) * WAVE + lane] = t[i];
		}
		W[(WIN / 4) * WAVE + lane] = 0u;

		STAMP(0);   // data of this tile landed in LDS
		// advance the pipeline: data of tile+stride, descriptors of tile+2*stride
		if (PREFETCH) {
			d_off = n_off;
			d_len = n_len;
			const uint32_t t2 = tile + 2u * tstride, p2 = t2 * WAVE + lane;
			n_off = 0;
			n_len = 0;
			if (t2 < nt && p2 < a.n) {
				n_off = a.off[p2];
				n_len = a.len[p2];
			}
#pragma unroll
			for (uint32_t r = 0; r < NPIECE; ++r) {
				d[r] = make_uint4(0, 0, 0, 0);
#ifndef DIAG_NOLOAD
				if (16u * r < d_len)
					__builtin_memcpy(&d[r], a.pkts + d_off + 16u * r, 16);
#endif
			}
		}
		wave_lds_sync();
#ifdef DIAG_STAGEONLY
		if (valid) {
			uint4 rec;
			rec.x = W[3 * WAVE + lane] ^ W[8 * WAVE + lane];
			rec.y = my_len;
			rec.z = 0;
			rec.w = 0;
			*(uint4 *)(a.out + pi) = rec;
		}
		continue;
#endif

		Pkt k;
		k.w = W + lane;
		k.g = a.pkts + my_off;
		k.len = my_len;

		STAMP(1);   // next tile's loads issued
		bool slow;
		Parsed p = parse_fast(k, slow);
		if (__ballot(slow) != 0ull) {
			if (slow)
				p = parse_packet(k);
		}

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

		STAMP(2);   // parsed, start CoS selected, fields loaded
		// ---- CoS descent (match_pmr_cos, :1624-1667).  Each round moves every
		// pending lane one hop: lanes on a bit-vector CoS evaluate it in
		// parallel (uniformly when they all sit on one CoS -- scalar loads --
		// or each on its own CoS); lanes on a linear-scan CoS are served one
		// CoS per round, wave-uniform, with the rule words in SGPRs.
		uint32_t hops = 0, mark = 0;
		bool matched = false, loop = false;
		for (;;) {
			const unsigned long long pm = __ballot(pend);
			if (pm == 0ull)
				break;
			const int32_t c0 = __builtin_amdgcn_readlane(cur, (int)__builtin_ctzll(pm));
			const bool uniform = __ballot(pend && cur != c0) == 0ull;
			bool done = false, proc = false;
			uint32_t nxt = 0, nmark = 0;
			if (uniform) {
				const uint32_t rec0 = cos_tbl[COS_WORDS * (uint32_t)c0];
				const uint32_t nr = cos_tbl[COS_WORDS * (uint32_t)c0 + 1u];
				const uint32_t bv = cos_tbl[COS_WORDS * (uint32_t)c0 + 4u];
				proc = pend;
				if (bv != 0u && nr != 0u)
					bv_eval(dev + bv, a.dev + dev[DH_PROG_OFF] + rec0 * REC_WORDS, pend, k,
						p, x, a.dev, done, nxt, nmark);
				else
					linear_scan(prog, rec0, nr, pend, k, p, x, done, nxt, nmark);
			} else {
				const uint32_t ci = COS_WORDS * (uint32_t)(pend ? cur : c0);
				const uint32_t my_rec0 = a.dev[dev[DH_COS_OFF] + ci];
				const uint32_t my_nr = a.dev[dev[DH_COS_OFF] + ci + 1u];
				const uint32_t my_bv = a.dev[dev[DH_COS_OFF] + ci + 4u];
				const bool empty = pend && my_nr == 0u;
				const bool bvl = pend && my_nr != 0u && my_bv != 0u;
				if (__ballot(bvl))
					bv_eval((cword_t)(a.dev + my_bv),
						a.dev + dev[DH_PROG_OFF] + my_rec0 * REC_WORDS, bvl, k, p, x,
						a.dev, done, nxt, nmark);
				const bool lin = pend && !empty && !bvl;
				bool grp = false;
				const unsigned long long lm = __ballot(lin);
				if (lm) {
					const int32_t c1 = __builtin_amdgcn_readlane(cur, (int)__builtin_ctzll(lm));
					grp = lin && cur == c1;
					const uint32_t rec1 = cos_tbl[COS_WORDS * (uint32_t)c1];
					const uint32_t nr1 = cos_tbl[COS_WORDS * (uint32_t)c1 + 1u];
					bool d1 = false;
					uint32_t n1 = 0, m1 = 0;
					linear_scan(prog, rec1, nr1, grp, k, p, x, d1, n1, m1);
					if (grp) {
						done = d1;
						nxt = n1;
						nmark = m1;
					}
				}
				proc = bvl || empty || grp;
			}
			if (proc) {
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

		STAMP(3);   // descent done
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
				const uint32_t meta = a.dev[dev[DH_COS_OFF] + COS_WORDS * (uint32_t)fc + 2u];
				cos_idx = meta >> 24;
				const uint32_t nq = (meta >> 8) & 0xffu;
				if (meta & 0xffu) {
					outcome = MI_CLS_OUT_COS_DROP;
				} else {
					outcome = MI_CLS_OUT_ENQ;
					if (nq > 1u) {
						uint32_t h = rss_hash(k, p, (meta >> 16) & 0xffu) & 31u;
						queue = h % nq;
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
		STAMP(4);   // outcome computed, record stored
	}
#ifdef DIAG_STAMPS
	if (lane == 0 && a.diag) {
		for (int i = 0; i < NSTAMP; ++i)
			atomicAdd(a.diag + i, st_acc[i]);
		atomicAdd(a.diag + NSTAMP, 1ull);
	}
#endif

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
	uint32_t *d_dev;         // assembled device rule program
	size_t dev_cap;          // bytes
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
	if (c->d_dev)
		(void)hipFree(c->d_dev);
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

// words of one term in the device encoding (see "device rule program")
static uint32_t encode_term(const mi_term_t &t, uint32_t *w)
{
	uint32_t n = 0;
	if (t.kind == MI_K_CUSTOM_FRAME || t.kind == MI_K_CUSTOM_L3) {
		uint32_t nw = (t.size + 3u) / 4u;
		w[n++] = t.kind | ((uint32_t)t.size << 8) | (nw << 16);
		w[n++] = t.offset;
		for (uint32_t i = 0; i < nw; ++i) {
			w[n++] = t.mask[i];
			w[n++] = t.value[i];
		}
		return n;
	}
	uint32_t nw = (t.kind == MI_K_SIP6 || t.kind == MI_K_DIP6) ? 4u : (t.kind == MI_K_DMAC ? 2u : 1u);
	w[n++] = t.kind | ((uint32_t)t.size << 8) | (nw << 16);
	for (uint32_t i = 0; i < nw; ++i) {
		w[n++] = t.mask[i];
		w[n++] = t.value[i];
	}
	return n;
}

// ---- bit-vector block construction (host) ----
struct ClassKey {
	uint32_t kind, nkey, offset, size, mask[4];
	bool operator<(const ClassKey &o) const
	{
		if (kind != o.kind) return kind < o.kind;
		if (offset != o.offset) return offset < o.offset;
		if (size != o.size) return size < o.size;
		for (int i = 0; i < 4; ++i)
			if (mask[i] != o.mask[i]) return mask[i] < o.mask[i];
		return false;
	}
};

typedef std::array<uint32_t, 4> Key4;

static uint32_t host_bv_hash(const Key4 &k)
{
	uint32_t h = k[0] * 0x9E3779B1u ^ k[1] * 0x85EBCA77u ^ k[2] * 0xC2B2AE3Du ^ k[3] * 0x27D4EB2Fu;
	h ^= h >> 15;
	h *= 0x2C1B3C6Du;
	h ^= h >> 12;
	return h;
}

static bool class_of(const mi_term_t &t, ClassKey &ck)
{
	memset(&ck, 0, sizeof(ck));
	ck.kind = t.kind;
	switch (t.kind) {
	case MI_K_NEVER:
	case MI_K_ALWAYS:
		return false;
	case MI_K_CUSTOM_FRAME:
	case MI_K_CUSTOM_L3:
		ck.offset = t.offset;
		ck.size = t.size;
		ck.nkey = t.size > 8 ? 4 : (t.size > 4 ? 2 : 1);
		break;
	case MI_K_SIP6:
	case MI_K_DIP6:
		ck.nkey = 4;
		break;
	case MI_K_DMAC:
		ck.nkey = 2;
		break;
	default:
		ck.nkey = 1;
	}
	for (uint32_t i = 0; i < 4; ++i)
		ck.mask[i] = i < ck.nkey ? t.mask[i] : 0;
	return true;
}

// Build the BV block of one CoS into `blk` (word offsets relative to the
// start of the device program, base = blk's first word index).  Returns false
// when the CoS needs more than BV_MAX_CLS classes (linear scan instead).
static bool build_bv(const mi_rule_t *rs, const mi_term_t *ts, uint32_t nrules, uint32_t base,
		     std::vector<uint32_t> &blk)
{
	std::map<ClassKey, uint32_t> cls;
	std::vector<ClassKey> cls_list;
	for (uint32_t r = 0; r < nrules; ++r)
		for (uint32_t t = 0; t < rs[r].num_terms; ++t) {
			ClassKey ck;
			if (class_of(ts[rs[r].term_begin + t], ck) && !cls.count(ck)) {
				cls[ck] = (uint32_t)cls_list.size();
				cls_list.push_back(ck);
			}
		}
	const uint32_t ncls = (uint32_t)cls_list.size();
	if (ncls > BV_MAX_CLS)
		return false;
	// canonical class order: CoS with the same classes evaluate them in the
	// same order, so lanes on different CoS stay convergent
	std::sort(cls_list.begin(), cls_list.end());
	for (uint32_t i = 0; i < ncls; ++i)
		cls[cls_list[i]] = i;
	const uint32_t W = (nrules + 31u) / 32u;
	// per rule: alive bit, and per class the required key (or none)
	std::vector<uint32_t> alive(W, 0);
	std::vector<std::map<Key4, std::vector<uint32_t>>> rows_of(ncls);   // key -> rule list
	std::vector<std::vector<uint32_t>> dc(ncls, std::vector<uint32_t>(W, 0));
	for (uint32_t r = 0; r < nrules; ++r) {
		bool ok = true;
		std::vector<int> have(ncls, 0);
		std::vector<Key4> want(ncls);
		for (uint32_t t = 0; t < rs[r].num_terms; ++t) {
			const mi_term_t &tm = ts[rs[r].term_begin + t];
			ClassKey ck;
			if (!class_of(tm, ck)) {
				if (tm.kind == MI_K_NEVER)
					ok = false;
				continue;
			}
			uint32_t c = cls[ck];
			Key4 v = { 0, 0, 0, 0 };
			for (uint32_t i = 0; i < ck.nkey; ++i)
				v[i] = tm.value[i];
			if (have[c] && want[c] != v)
				ok = false;   // two terms of one class with different values
			have[c] = 1;
			want[c] = v;
		}
		if (!ok)
			continue;
		alive[r >> 5] |= 1u << (r & 31);
		for (uint32_t c = 0; c < ncls; ++c) {
			if (have[c])
				rows_of[c][want[c]].push_back(r);
			else
				dc[c][r >> 5] |= 1u << (r & 31);
		}
	}
	// layout: header (4) | classes (16 each) | alive row | per class: table, rows
	blk.assign(4 + BV_CLS_WORDS * ncls, 0);
	blk[0] = W;
	blk[1] = ncls;
	blk[2] = base + (uint32_t)blk.size();
	blk.insert(blk.end(), alive.begin(), alive.end());
	for (uint32_t c = 0; c < ncls; ++c) {
		const ClassKey &ck = cls_list[c];
		const uint32_t nvals = (uint32_t)rows_of[c].size();
		uint32_t tsize = 4;
		while (tsize < 2 * (nvals + 1))
			tsize <<= 1;
		uint32_t *cr = &blk[4 + BV_CLS_WORDS * c];
		cr[0] = ck.kind;
		cr[1] = ck.nkey;
		cr[3] = ck.offset;
		cr[4] = ck.size;
		for (int i = 0; i < 4; ++i)
			cr[5 + i] = ck.mask[i];
		cr[9] = tsize - 1;
		const uint32_t tbl_off = (uint32_t)blk.size();
		cr = nullptr;
		blk.resize(blk.size() + (size_t)tsize * (ck.nkey + 1), 0);
		for (uint32_t i = 0; i < tsize; ++i)
			blk[tbl_off + i * (ck.nkey + 1) + ck.nkey] = BV_EMPTY;
		const uint32_t rows_off = (uint32_t)blk.size();
		// row 0: rules without a term of this class
		blk.insert(blk.end(), dc[c].begin(), dc[c].end());
		uint32_t row = 1;
		for (auto &kv : rows_of[c]) {
			std::vector<uint32_t> bits = dc[c];
			for (uint32_t r : kv.second)
				bits[r >> 5] |= 1u << (r & 31);
			blk.insert(blk.end(), bits.begin(), bits.end());
			uint32_t h = host_bv_hash(kv.first) & (tsize - 1);
			while (blk[tbl_off + h * (ck.nkey + 1) + ck.nkey] != BV_EMPTY)
				h = (h + 1) & (tsize - 1);
			for (uint32_t i = 0; i < ck.nkey; ++i)
				blk[tbl_off + h * (ck.nkey + 1) + i] = kv.first[i];
			blk[tbl_off + h * (ck.nkey + 1) + ck.nkey] = row++;
		}
		uint32_t *cw = &blk[4 + BV_CLS_WORDS * c];
		cw[10] = base + tbl_off;
		cw[11] = base + rows_off;
	}
	return true;
}

// Assemble the mi_cls.h table into the private device encoding.
static int assemble(const void *tbl, uint32_t **out, size_t *out_words)
{
	const mi_tbl_hdr_t *h = (const mi_tbl_hdr_t *)tbl;
	const uint8_t *b = (const uint8_t *)tbl;
	const mi_cos_t *cs = (const mi_cos_t *)(b + h->cos_off);
	const mi_rule_t *rs = (const mi_rule_t *)(b + h->rule_off);
	const mi_term_t *ts = (const mi_term_t *)(b + h->term_off);
	const uint32_t cos_off = DH_WORDS, prog_off = cos_off + COS_WORDS * h->num_cos;
	std::vector<uint32_t> w(prog_off + (size_t)h->num_rules * REC_WORDS, 0);
	w[DH_MAGIC] = DEV_MAGIC;
	w[DH_NCOS] = h->num_cos;
	w[DH_DEFAULT] = (uint32_t)h->default_cos;
	w[DH_ERROR] = (uint32_t)h->error_cos;
	w[DH_DEFAULT_VALID] = h->default_valid;
	w[DH_USED] = h->used_kinds;
	w[DH_MAX_HOPS] = h->max_hops;
	w[DH_COS_OFF] = cos_off;
	w[DH_PROG_OFF] = prog_off;
	for (uint32_t s = 0; s < h->num_cos; ++s) {
		uint32_t *c = &w[cos_off + COS_WORDS * s];
		c[0] = cs[s].rule_begin;
		c[1] = cs[s].num_rules;
		c[2] = (uint32_t)cs[s].action | ((uint32_t)cs[s].num_queue << 8) |
		       ((uint32_t)cs[s].hash_proto << 16) | ((uint32_t)cs[s].index << 24);
		c[3] = cs[s].valid;
	}
	// 16-word rule records (+ ext terms appended after them)
	std::vector<uint32_t> ext;
	const size_t ext_base = (size_t)h->num_rules * REC_WORDS;
	for (uint32_t r = 0; r < h->num_rules; ++r) {
		uint32_t *rec = &w[prog_off + (size_t)r * REC_WORDS];
		uint32_t used = 2, n_in = 0, n_ext = 0;
		size_t ext_begin = ext_base + ext.size();
		for (uint32_t t = 0; t < rs[r].num_terms; ++t) {
			uint32_t tw[12];
			uint32_t n = encode_term(ts[rs[r].term_begin + t], tw);
			if (n_ext == 0 && used + n <= REC_WORDS) {
				memcpy(rec + used, tw, n * sizeof(uint32_t));
				used += n;
				n_in++;
			} else {
				ext.insert(ext.end(), tw, tw + n);
				n_ext++;
			}
		}
		if (ext_begin >= (1u << 24))
			return -E2BIG;
		rec[0] = n_in | (n_ext << 8) | ((uint32_t)rs[r].mark << 16);
		rec[1] = rs[r].dst_cos | ((uint32_t)(n_ext ? ext_begin : 0) << 8);
	}
	w.insert(w.end(), ext.begin(), ext.end());
	// bit-vector blocks (absolute word offsets)
	if (!getenv("MI_CLS_NO_BV")) {
		for (uint32_t s = 0; s < h->num_cos; ++s) {
			if (!cs[s].valid || cs[s].num_rules == 0)
				continue;
			std::vector<uint32_t> blk;
			const uint32_t base = (uint32_t)w.size();
			if (build_bv(rs + cs[s].rule_begin, ts, cs[s].num_rules, base, blk)) {
				w[cos_off + COS_WORDS * s + 4] = base;
				w.insert(w.end(), blk.begin(), blk.end());
			}
		}
	}
	w.resize(w.size() + 16, 0);
	w[DH_TOTAL] = (uint32_t)w.size();
	uint32_t *o = (uint32_t *)malloc(w.size() * sizeof(uint32_t));
	if (!o)
		return -ENOMEM;
	memcpy(o, w.data(), w.size() * sizeof(uint32_t));
	*out = o;
	*out_words = w.size();
	return 0;
}

extern "C" int mi_cls_rules_load(mi_cls_ctx_t *c, const void *tbl, size_t bytes, void *stream)
{
	if (!c)
		return -EINVAL;
	int rc = validate_tbl(tbl, bytes);
	if (rc)
		return rc;
	uint32_t *w = nullptr;
	size_t words = 0;
	rc = assemble(tbl, &w, &words);
	if (rc)
		return rc;
	size_t nbytes = words * sizeof(uint32_t);
	if (hipSetDevice(c->device) != hipSuccess)
		return free(w), -EIO;
	if (nbytes > c->dev_cap) {
		// the old program may still be read by in-flight launches
		if (c->d_dev) {
			if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
				return free(w), -EIO;
			(void)hipFree(c->d_dev);
			c->d_dev = nullptr;
		}
		size_t cap = nbytes < 4096 ? 4096 : nbytes;
		if (hipMalloc((void **)&c->d_dev, cap) != hipSuccess)
			return free(w), -ENOMEM;
		c->dev_cap = cap;
	}
	// stream-ordered after earlier launches; synchronous w.r.t. the host
	// buffer, which is freed on return
	hipError_t e = hipMemcpyAsync(c->d_dev, w, nbytes, hipMemcpyHostToDevice, (hipStream_t)stream);
	if (e == hipSuccess)
		e = hipStreamSynchronize((hipStream_t)stream);
	free(w);
	if (e != hipSuccess)
		return -EIO;
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
	a.dev = c->d_dev;
	a.out = out;
	a.stats = c->stats_on ? c->d_stats : nullptr;
	a.diag = nullptr;
#ifdef DIAG_STAMPS
	static unsigned long long *d_diag = nullptr;
	if (!d_diag)
		(void)hipMalloc((void **)&d_diag, 16 * sizeof(unsigned long long));
	(void)hipMemset(d_diag, 0, 16 * sizeof(unsigned long long));
	a.diag = d_diag;
#endif
	memcpy(a.stats_mask, c->stats_mask, sizeof(a.stats_mask));
	// one wave per 64-packet tile in flight; the grid covers the resident
	// capacity (blocks per CU) and each wave loops over its tiles with the
	// load pipeline (MI_CLS_BLOCKS_PER_CU overrides the default of 4)
	static int per_cu = -1;
	if (per_cu < 0) {
		const char *e = getenv("MI_CLS_BLOCKS_PER_CU");
		per_cu = e ? atoi(e) : 4;
		if (per_cu < 1)
			per_cu = 1;
	}
	uint32_t tiles = (n + BLOCK - 1) / BLOCK;
	uint32_t max_grid = (uint32_t)c->num_cu * (uint32_t)per_cu;
	uint32_t grid = tiles < max_grid ? tiles : max_grid;
	hipLaunchKernelGGL(mi_cls_kernel, dim3(grid), dim3(BLOCK), 0, (hipStream_t)stream, a);
	if (hipGetLastError() != hipSuccess)
		return -EIO;
#ifdef DIAG_STAMPS
	{
		unsigned long long h[16];
		(void)hipStreamSynchronize((hipStream_t)stream);
		(void)hipMemcpy(h, d_diag, sizeof(h), hipMemcpyDeviceToHost);
		fprintf(stderr, "DIAG waves=%llu cycles/wave:", h[8]);
		for (int i = 0; i < 5; ++i)
			fprintf(stderr, " p%d=%.0f", i, (double)h[i] / (double)(h[8] ? h[8] : 1));
		fprintf(stderr, "\n");
	}
#endif
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
