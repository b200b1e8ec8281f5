// mi_cls_dev.h -- device side of the gfx950 (MI355X / CDNA4) packet parse +
// PMR classify path: packet byte access, the parsers, the classification
// engines, the device rule-program encoding and the mi_cls_kernel template.
// Included by the kernel translation units (mi_cls_k<NW>.hip, one block
// shape each, compiled in parallel) and by the host code in mi_cls.hip (for
// the encoding constants and fdesc()).
//
// What it replaces (reference, platform/linux-generic/):
//   pktio/loop.c:283-339        per-packet parse + classify inside loopback_recv
//   odp_parse.c:23-488          _odp_parse_eth / parse_ipv4 / parse_ipv6 / parse_tcp
//                               / parse_udp / parse_sctp / _odp_packet_parse_common_l3_l4
//   odp_classification.c:931-1515   verify_pmr and the per-term verifiers
//   odp_classification.c:1624-1771  match_pmr_cos / cls_select_cos / _odp_cls_classify_packet
//   odp_classification.c:395-405, 1773-1839 + protocols/thash.h:82-99  hash-queue pick
//
// Measurement hooks (phase-floor variants built with tools/ab.py and
// `python -m odp_amd._build DIR DIAG_...`; never in a shipped build, their
// records are wrong on purpose): DIAG_NOSTAGE (no window loads after a
// wave's first tile: the compute-only floor), DIAG_STAGEONLY (windows and
// records only), DIAG_PARSEONLY (no classification), DIAG_MAXROUND=n (the
// descent stops after n rounds), DIAG_DESCENTONLY (no final-CoS step),
// DIAG_CK_NOSUM / DIAG_CK_NOSCTP / DIAG_CK_OK (checksum parts left out).
//
// Design (MI355X-first, not a translation; DESIGN.md has the details):
//   * one wavefront owns 64 consecutive packets (a tile, one packet per lane)
//     and loops over its tiles with the next tile's header loads in flight;
//   * the first 64 B (96 B when the frames need them) of every packet are
//     loaded cooperatively (4 lanes per packet, 16-B buffer loads, so one
//     instruction covers 16 back-to-back headers) and stored dword-major,
//     lane-minor into the wave's LDS window, where each lane reads any byte
//     offset of its own frame without bank conflicts; bytes past the window
//     come from HBM, bytes past the frame read 0;
//   * parse_fast (selects, wave-uniform skips) covers the common header
//     shapes, parse_packet restates every branch of odp_parse.c;
//   * classification: per CoS a block of key classes looked up in two-choice
//     cuckoo tables (16-B buckets), combined by the direct / bitmap / wide
//     bitmap / candidate engines; the CoS tree is descended one hop per
//     round, per-lane blocks when lanes sit on different CoS.  No MFMA:
//     this is parse-and-compare.
#pragma once
// Under hipRTC (program-specialised kernels, mi_cls_spec.cpp) only the
// device part is compiled: no host headers.
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#endif
#include <stdint.h>

#include "mi_cls.h"

#include <type_traits>

#define WAVE 64
#define WIN 96             // staged header window, bytes
#define WROWS (WIN / 4 + 1)     // LDS dword rows per wave window (+1 zero row)
#define RS 66                   // LDS row stride of a window, dwords (see load_window)
#define NPIECE (WIN / 16)       // 16-B pieces per window
#define MIN_WAVES_PER_EU 4   // waves per SIMD of the 4-wave block shapes (the VGPR budget)
#define LOAD_AUX 2          // cache policy of the packet-window loads: nt (read once)
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
#define E_L3CK 4u           // l3_chksum_err
#define E_L4CK 64u          // l4_chksum_err
#define F_L3CK_DONE (1u << 30)   // input_flags.l3_chksum_done
#define F_L4CK_DONE (1u << 31)   // input_flags.l4_chksum_done
// pktin options: odp_pktin_config_opt_t.all_bits (include/odp_rt.h)
#define OPT_IPV4_CK (1u << 2)
#define OPT_UDP_CK (1u << 3)
#define OPT_TCP_CK (1u << 4)
#define OPT_SCTP_CK (1u << 5)
#define OPT_DROP_V4 (1u << 6)
#define OPT_DROP_V6 (1u << 7)
#define OPT_DROP_UDP (1u << 8)
#define OPT_DROP_TCP (1u << 9)
#define OPT_DROP_SCTP (1u << 10)
#define OPT_L4_CK (OPT_UDP_CK | OPT_TCP_CK | OPT_SCTP_CK)

// ------------------------------------------------------- packet byte access
// The LDS window of a wave is dword-major, lane-minor: dword i of lane l's
// packet lives at W[i * RS + l] (RS = 66).  Any per-lane byte offset then
// reads conflict-free (lane l of row i hits bank 2i + l mod 32), whatever the
// packets' header layouts.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Pkt {
	const uint32_t *w;      // &W[lane]
	const uint8_t *g;       // packet start in HBM
	uint32_t len;           // frame_len
	uint32_t win;           // bytes of the frame staged in LDS this tile (64 or WIN;
	                        // wave-uniform): bytes [0, min(len, win)) are in
	                        // the window, bytes past the frame read 0
};

// One byte; past the staged window it comes from HBM (the general parser and
// the rare far field), past the frame it is 0.
__device__ __forceinline__ uint32_t rb(const Pkt &k, uint32_t o)
{
	if (o < k.win)
		return (k.w[(o >> 2) * RS] >> ((o & 3u) * 8u)) & 0xffu;
	return o < k.len ? (uint32_t)k.g[o] : 0u;
}

// 4 bytes starting at byte offset o, little-endian (== the reference's raw
// load).  The LDS read is unconditional (row index clamped into the window
// and its zero row: a lane whose 4 bytes lie in the window reads rows <=
// WIN/4), so lanes do not diverge; a wave-uniform branch fixes up
// the lanes whose 4 bytes reach past the staged window (bytes from HBM).
__device__ __forceinline__ uint32_t r32(const Pkt &k, uint32_t o)
{
	const uint32_t i = min(o >> 2, (uint32_t)(WIN / 4 - 1));
	uint32_t v = __builtin_amdgcn_alignbyte(k.w[(i + 1) * RS], k.w[i * RS], o & 3u);
	const bool far = o + 4u > k.win;
	if (__ballot(far) != 0ull) {
		if (far) {
			// two dword loads from HBM (the dwords that start inside the
			// frame: they end inside its 16-B rounding, the batch contract),
			// funnel-shifted, the bytes past the frame zeroed.  Frames may
			// start at any byte: the dword loads are unaligned then, which
			// gfx950 serves.
			const uint32_t a = o & ~3u;
			const uint32_t w0 = a < k.len ? *(const uint32_t *)(k.g + a) : 0u;
			const uint32_t w1 = a + 4u < k.len ? *(const uint32_t *)(k.g + a + 4u) : 0u;
			const uint32_t keep = k.len > o ? min(k.len - o, 4u) : 0u;
			v = __builtin_amdgcn_alignbyte(w1, w0, o & 3u);
			v = keep >= 4u ? v : (v & ((1u << (8u * keep)) - 1u));
		}
	}
	return v;
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
	uint32_t udp_zero;      // input_flags.udp_chksum_zero (bit 32: not stored)
};

// one's-complement fold of a 64-bit partial sum (chksum_finalize,
// include/odp_chksum_internal.h)
__device__ __forceinline__ uint32_t ck_finalize(uint64_t s)
{
	s = (s >> 32) + (s & 0xffffffffull);
	s = (s >> 16) + (s & 0xffffull);
	return (uint32_t)((s >> 16) + s) & 0xffffu;
}

// _odp_parse_eth + _odp_packet_parse_common_l3_l4 (layer ALL) with the pktin
// options `opt` (IPv4 header checksum, drop on IPv4/IPv6/UDP/TCP/SCTP
// errors; the UDP zero-checksum rule of parse_udp), odp_parse.c:23-105,
// 112-354, 362-488; contiguous packet so seg_end == frame_len.  The L4
// checksums themselves are l4_chksum() below.
__device__ __forceinline__ Parsed parse_packet(const Pkt &k, uint32_t opt)
{
	Parsed r;
	const uint32_t len = k.len;
	uint32_t f = F_L2 | F_ETH, err = 0, off = 14, ethtype, ip_proto = 255;
	bool non_first = false;
	r.udp_zero = 0;

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
		bool bad = ihl < 5u || (vi >> 4) != 4u || 20u > len - l3 || tot > len - l3;
		if (!bad && (opt & OPT_IPV4_CK)) {
			// odp_parse.c:134-141: header checksum over ihl * 4 bytes
			f |= F_L3CK_DONE;
			uint64_t s = 0;
			for (uint32_t i = 0; i < ihl; ++i)
				s += r32(k, l3 + 4u * i);
			if (ck_finalize(s) != 0xffffu) {
				err |= E_L3CK;
				bad = true;
			}
		}
		if (bad) {
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
	// drop_ipv4_err / drop_ipv6_err (odp_parse.c:383-387, 392-396): the L4
	// part is never reached
	if ((err & E_IP) && (((f & F_IPV4) && (opt & OPT_DROP_V4)) ||
			     ((f & F_IPV6) && (opt & OPT_DROP_V6)))) {
		r.l4 = 0xFFFFu;
		r.flags = f;
		r.err = err;
		r.ret = -1;
		return r;
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
			if ((err & E_TCP) && (opt & OPT_DROP_TCP))
				ret = -1;
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
				if (ulen < 8u) {
					err |= E_UDP;
					if (opt & OPT_DROP_UDP)
						ret = -1;
				} else {
					// parse_udp, odp_parse.c:298-313
					if ((opt & OPT_UDP_CK) && !(f & F_IPFRAG) && r16(k, off + 6) == 0u) {
						f |= F_L4CK_DONE;
						err |= (f & F_IPV4) ? 0u : E_L4CK;
						r.udp_zero = 1;
					}
					if ((ports >> 16) == 0x9411u /* be16(4500) raw */ && ulen > 4u &&
					    r32(k, off + 8) != 0u)
						f |= F_IPSEC;
				}
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
			if ((err & E_SCTP) && (opt & OPT_DROP_SCTP))
				ret = -1;
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

// ------------------------------------------------------- pktin checksums
// Buffer offset no frame byte reaches: num_records of the packet resource, so
// a load at or past it returns zeros (batches are < 4 GiB: u32 offsets).
#define OOB_OFF 0xFFFFFE00u

// CRC-32C (Castagnoli, reflected polynomial 0x82F63B78), the arithmetic of
// odp_hash_crc32c (arch/default/odp_hash_crc32.c: table-driven,
// caller-supplied init, no final inversion), as slicing-by-4 tables: t[0] is
// the byte table, t[k][i] = t[k-1][i] >> 8 ^ t[0][t[k-1][i] & 0xff], so four
// bytes advance with four independent lookups instead of four dependent ones.
// s128 / s256: the register advanced over 16 / 32 zero bytes, per register
// byte (s[k][b] = advance(b << 8k)), to join the raw CRCs of consecutive
// 16-B / 32-B chunks with four lookups.  z[m] = x^(512 m), yinv[z] =
// x^(-8 z) and y1[r] = ~0 x^(8 r) mod P in the reflected domain (x^0 =
// 0x80000000): the shifts that combine CRCs of separately processed pieces
// (sctp_crc_wave; zlib's crc32_combine arithmetic).  x^-1 exists (P has a
// constant term): (P + 1) / x, i.e. (0x82F63B78 << 1) | 1.
#define CRC_ZN 256          // pieces of 64 B a frame may have on the cooperative path
// word offsets of the tables in the kernel's LDS copy
#define CRC_S128 1024u
#define CRC_S256 2048u
#define CRC_Z 3072u
#define CRC_YINV (CRC_Z + CRC_ZN)
#define CRC_Y1 (CRC_YINV + 65u)
#define CRC_WORDS (CRC_Y1 + 64u)
__host__ __device__ constexpr uint32_t crc_mulmod_c(uint32_t a, uint32_t b)
{
	uint32_t p = 0;
	for (int i = 31; i >= 0; --i) {
		p ^= ((a >> i) & 1u) ? b : 0u;
		b = (b >> 1) ^ ((b & 1u) ? 0x82F63B78u : 0u);
	}
	return p;
}
struct Crc32cTab {
	uint32_t t[4][256];
	uint32_t s128[4][256];
	uint32_t s256[4][256];
	uint32_t z[CRC_ZN];
	uint32_t yinv[65];
	uint32_t y1[64];
	constexpr Crc32cTab() : t(), s128(), s256(), z(), yinv(), y1()
	{
		for (uint32_t i = 0; i < 256; ++i) {
			uint32_t c = i;
			for (int b = 0; b < 8; ++b)
				c = (c & 1u) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
			t[0][i] = c;
		}
		for (int k = 1; k < 4; ++k)
			for (uint32_t i = 0; i < 256; ++i)
				t[k][i] = (t[k - 1][i] >> 8) ^ t[0][t[k - 1][i] & 0xffu];
		for (int k = 0; k < 4; ++k)
			for (uint32_t i = 0; i < 256; ++i) {
				uint32_t r = i << (8 * k);
				for (int j = 0; j < 32; ++j) {
					if (j == 16)
						s128[k][i] = r;
					r = t[0][r & 0xffu] ^ (r >> 8);
				}
				s256[k][i] = r;
			}
		uint32_t r = 0x80000000u;
		for (uint32_t m = 0; m < CRC_ZN; ++m) {
			z[m] = r;
			for (int i = 0; i < 16; ++i)   // 64 zero bytes, four at a time
				r = t[3][r & 0xffu] ^ t[2][(r >> 8) & 0xffu] ^ t[1][(r >> 16) & 0xffu] ^
				    t[0][r >> 24];
		}
		uint32_t xi8 = 0x80000000u;   // x^-8
		for (int i = 0; i < 8; ++i)
			xi8 = crc_mulmod_c(xi8, (0x82F63B78u << 1) | 1u);
		r = 0x80000000u;
		for (uint32_t i = 0; i < 65; ++i) {
			yinv[i] = r;
			r = crc_mulmod_c(r, xi8);
		}
		r = 0xFFFFFFFFu;
		for (uint32_t i = 0; i < 64; ++i) {
			y1[i] = r;
			r = t[0][r & 0xffu] ^ (r >> 8);
		}
	}
};
static __constant__ Crc32cTab c_crc32c;

// Table lookups go to the kernel's LDS copy of c_crc32c (`tab`, 4 x 256
// words): a lane walks its own frame, so the lookups are divergent.
__device__ __forceinline__ uint32_t crc32c_u8(const uint32_t *tab, uint32_t crc, uint32_t b)
{
	return tab[(crc ^ b) & 0xffu] ^ (crc >> 8);
}

// four bytes, little-endian word w (byte 0 first on the wire)
__device__ __forceinline__ uint32_t crc32c_u32(const uint32_t *tab, uint32_t crc, uint32_t w)
{
	const uint32_t c = crc ^ w;
	return tab[768u + (c & 0xffu)] ^ tab[512u + ((c >> 8) & 0xffu)] ^
	       tab[256u + ((c >> 16) & 0xffu)] ^ tab[c >> 24];
}

// Value of lane `src` (every lane of the wave must be active: callers keep
// the control flow uniform around it).
__device__ __forceinline__ uint32_t lane_get(uint32_t v, uint32_t src)
{
	return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}

// Inclusive prefix sum over the 64 lanes of the wave (all lanes active):
// DPP row shifts within each 16-lane row, then the row totals (readlane of
// lanes 15 / 31 / 47) added to the rows after them -- no LDS traffic.
__device__ __forceinline__ uint32_t wave_scan_add(uint32_t v, uint32_t lane)
{
	v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);   // row_shr:1
	v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);   // row_shr:2
	v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);   // row_shr:4
	v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);   // row_shr:8
	const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
	const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
	const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
	const uint32_t row = lane >> 4;
	return v + (row >= 1u ? r0 : 0u) + (row >= 2u ? r1 : 0u) + (row >= 3u ? r2 : 0u);
}

// Wave-cooperative one's-complement sums of the UDP / TCP payloads of a
// tile (all 64 lanes active).  Lane f asks for the sum of frame bytes
// [from, to) of its frame: `cnt` 64-B pieces starting at batch offset `base`
// (the frame-relative 64-B boundary at or below `from`), with
// prm = (from - boundary) | (to - boundary) << 6.  The pieces of all lanes
// are numbered in lane order (a wave prefix sum of cnt) and dealt out 64 per
// round: lane j of a round takes piece g = round base + j, which belongs to
// the last lane whose first piece number is <= g (binary search over the
// lanes' first numbers with ds_bpermute), and reads its 64 bytes with four
// 16-B loads.  Consecutive pieces are consecutive bytes of one frame and a
// tile's frames are consecutive in the batch, so a round reads ~4 KB of
// contiguous bytes, and every lane is busy whatever the frame lengths are
// (a per-lane loop ran every lane for the longest frame of the tile).
// Dwords wholly inside [from, to) are summed as they are; the two partial
// dwords (`from` is even: the upper half of its dword; the bytes of `to`'s
// dword below it) come from two extra dword loads.  Each piece is folded to a
// value congruent to its sum of 16-bit words modulo 0xffff (2^16 == 1), and a
// prefix sum over the round gives each owner its pieces' total as the
// difference of two prefix values.  Returns the lane's own sum (congruent
// mod 0xffff, < 2^32).
#define CK_HALVES 1         // pieces per lane per round of ck_sum_wave (2, 3 measured slower)
__device__ __forceinline__ uint32_t ck_sum_wave(__amdgpu_buffer_rsrc_t rs, uint32_t base,
						uint32_t prm, uint32_t cnt, uint32_t lane)
{
	const uint32_t incl = wave_scan_add(cnt, lane);
	const uint32_t first = incl - cnt;   // number of this lane's first piece
	const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, WAVE - 1);
	uint32_t acc = 0;
	// CK_HALVES pieces per lane per round (lane j takes pieces B + j and B +
	// 64 + j): the loads of both are in flight together, so a round trip to
	// memory serves twice the bytes (the sum phase is latency-bound: one
	// wave's round waits for its loads)
	for (uint32_t B = 0; B < total; B += CK_HALVES * WAVE) {
		uint32_t r[CK_HALVES];
		{
			uint32_t ob[CK_HALVES];
			int32_t lb[CK_HALVES], hb[CK_HALVES];
			bool live[CK_HALVES];
#pragma unroll
			for (uint32_t h = 0; h < CK_HALVES; ++h) {
				const uint32_t g = B + WAVE * h + lane;
				uint32_t lo = 0;
#pragma unroll
				for (uint32_t st = WAVE / 2; st >= 1; st >>= 1) {
					const uint32_t c = lo + st;
					lo = lane_get(first, c) <= g ? c : lo;
				}
				const uint32_t q = g - lane_get(first, lo);
				const uint32_t pr = lane_get(prm, lo);
				ob[h] = lane_get(base, lo) + 64u * q;
				live[h] = g < total;
				// the piece's byte window [lb, hb), relative to its start
				lb[h] = (int32_t)(pr & 63u) - (int32_t)(64u * q);
				hb[h] = (int32_t)(pr >> 6) - (int32_t)(64u * q);
			}
			u32x4 v[CK_HALVES][4];
			uint32_t xh[CK_HALVES], xt[CK_HALVES];
#pragma unroll
			for (uint32_t h = 0; h < CK_HALVES; ++h) {
#pragma unroll
				for (int32_t k = 0; k < 4; ++k)   // only 16-B parts that reach into [from, to)
					v[h][k] = __builtin_amdgcn_raw_buffer_load_b128(
						rs, (live[h] && 16 * k < hb[h] && 16 * k + 16 > lb[h]) ? ob[h] + 16u * k
													: OOB_OFF, 0, 0);
				const bool ph = live[h] && lb[h] > 0 && (lb[h] & 3) != 0;
				const bool pt = live[h] && hb[h] < 64 && (hb[h] & 3) != 0;
				xh[h] = __builtin_amdgcn_raw_buffer_load_b32(
					rs, ph ? ob[h] + (uint32_t)(lb[h] & ~3) : OOB_OFF, 0, 0);
				xt[h] = __builtin_amdgcn_raw_buffer_load_b32(
					rs, pt ? ob[h] + (uint32_t)(hb[h] & ~3) : OOB_OFF, 0, 0);
			}
#pragma unroll
			for (uint32_t h = 0; h < CK_HALVES; ++h) {
				uint64_t sm = (uint64_t)(xh[h] >> 16) +
					      (xt[h] & ((1u << (8u * ((uint32_t)hb[h] & 3u))) - 1u));
				// dword d is wholly inside iff lb <= 4d and 4d + 4 <= hb
				const uint32_t lo4 = (uint32_t)max(lb[h], 0);
				const int32_t sp = hb[h] - 4 - max(lb[h], 0);   // < 0: no whole dword
#pragma unroll
				for (uint32_t d = 0; d < 16; ++d) {
					const bool in = live[h] && sp >= 0 && (4u * d - lo4) <= (uint32_t)sp;
					sm += in ? v[h][d >> 2][d & 3u] : 0u;
				}
				// < 2^20 + 2^16
				r[h] = (uint32_t)(sm & 0xffffu) + (uint32_t)(sm >> 16);
			}
		}
		// prefix sums over the round's pieces (half h continues half h - 1)
		uint32_t P[CK_HALVES], T = 0;
#pragma unroll
		for (uint32_t h = 0; h < CK_HALVES; ++h) {
			P[h] = wave_scan_add(r[h], lane) + T;
			T = (uint32_t)__builtin_amdgcn_readlane((int)P[h], WAVE - 1);
		}
		// this lane's pieces in the round: [a, e) of it
		const uint32_t a = first > B ? first - B : 0u;
		const uint32_t e = min(incl > B ? incl - B : 0u, (uint32_t)(CK_HALVES * WAVE));
		const uint32_t ie = e > 0u ? e - 1u : 0u, ia = a > 0u ? a - 1u : 0u;
		uint32_t pe = 0, pa = 0;
#pragma unroll
		for (uint32_t h = 0; h < CK_HALVES; ++h) {
			const uint32_t xe = lane_get(P[h], ie & (WAVE - 1u));
			const uint32_t xa = lane_get(P[h], ia & (WAVE - 1u));
			pe = ie / WAVE == h ? xe : pe;
			pa = ia / WAVE == h ? xa : pa;
		}
		acc += (e > a) ? pe - (a > 0u ? pa : 0u) : 0u;
	}
	return acc;
}

// CRC-32C part of the SCTP check (odp_packet.c:2112-2131 via
// _odp_packet_sctp_chksum): over [l4, frame_len) with the 4-byte checksum
// field at l4 + 8 taken as zero, init ~0, four bytes per step (slicing-by-4)
// from 16-B loads of the frame (frame-relative 16-B pieces: never past the
// frame's 16-B rounding, the batch contract), the words funnel-shifted when
// l4 is 2 mod 4; the last 0-3 bytes one at a time.  Returns the finished
// (inverted) CRC.
#define CK_AHEAD 4          // 16-B pieces in flight per lane in sctp_crc
__device__ __forceinline__ uint32_t sctp_crc(const Pkt &k, __amdgpu_buffer_rsrc_t rs, uint32_t boff,
					     uint32_t l4, const uint32_t *tab)
{
	const uint32_t len = k.len, sh = l4 & 3u, j0 = l4 >> 2, n4 = (len - l4) >> 2;
	// word i (bytes l4 + 4i ..) = alignbyte(dword j0 + i + 1, dword j0 + i)
	uint32_t crc = 0xffffffffu, prev = 0u;
	const uint32_t jend = j0 + n4;   // last low dword index + 1
	// pieces are loaded CK_AHEAD ahead of the one the CRC steps consume (the
	// steps are a dependent chain of LDS lookups: without the lookahead
	// every piece would wait a full memory latency); a piece starting at or
	// past frame_len is not loaded (at frame_len, l4 = 0 mod 4 and frame_len
	// = 0 mod 16: it only feeds the last word's unused high half)
	const uint32_t q0 = (j0 >> 2) << 2;
	u32x4 nx[CK_AHEAD];
#pragma unroll
	for (uint32_t i = 0; i < CK_AHEAD; ++i) {
		const uint32_t qi = q0 + 4u * i;
		nx[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (qi <= jend && 4u * qi < len)
								      ? boff + 4u * qi : OOB_OFF, 0, 0);
	}
	for (uint32_t q = q0; q <= jend; q += 4u) {
		const u32x4 v = nx[0];
#pragma unroll
		for (uint32_t i = 0; i + 1 < CK_AHEAD; ++i)
			nx[i] = nx[i + 1];
		{
			const uint32_t qn = q + 4u * CK_AHEAD;
			nx[CK_AHEAD - 1] = __builtin_amdgcn_raw_buffer_load_b128(
				rs, (qn <= jend && 4u * qn < len) ? boff + 4u * qn : OOB_OFF, 0, 0);
		}
#pragma unroll
		for (uint32_t t = 0; t < 4; ++t) {
			// word whose low dword is q + t - 1 (its high dword is v[t])
			const uint32_t lo = q + t - 1u;
			const uint32_t w = __builtin_amdgcn_alignbyte(v[t], prev, sh);
			const bool in = q + t >= 1u && lo >= j0 && lo < jend;
			crc = in ? crc32c_u32(tab, crc, lo - j0 == 2u ? 0u : w) : crc;
			prev = v[t];
		}
	}
	for (uint32_t o = l4 + 4u * n4; o < len; ++o)
		crc = crc32c_u8(tab, crc, rb(k, o));
	return ~crc;
}

// a * b mod P in the reflected domain (zlib multmodp), branch-free
// Five VALU operations per bit, one statement per bit: the compiler's
// own lowering took seven and hoisted the 32 bit masks of `a` into 32 live
// registers, which spilled the checksum kernels (v_bitop3_b32 0x78 = S0 ^
// (S1 & S2)).
__device__ __forceinline__ uint32_t crc_mulmod(uint32_t a, uint32_t b)
{
	uint32_t p = 0;
	const uint32_t poly = 0x82F63B78u;
#pragma unroll
	for (int i = 31; i >= 0; --i) {
		uint32_t m, t;
		asm("v_bfe_i32 %[m], %[a], %[i], 1\n\t"
		    "v_bitop3_b32 %[p], %[p], %[m], %[b] bitop3:0x78\n\t"
		    "v_bfe_i32 %[t], %[b], 0, 1\n\t"
		    "v_lshrrev_b32 %[b], 1, %[b]\n\t"
		    "v_bitop3_b32 %[b], %[b], %[t], %[P] bitop3:0x78"
		    : [p] "+v"(p), [b] "+v"(b), [m] "=&v"(m), [t] "=&v"(t)
		    : [a] "v"(a), [i] "i"(i), [P] "s"(poly));
	}
	return p;
}

__device__ __forceinline__ uint32_t wave_scan_xor(uint32_t v, uint32_t lane)
{
	v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
	v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
	v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);
	v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);
	const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
	const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
	const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
	const uint32_t row = lane >> 4;
	return v ^ (row >= 1u ? r0 : 0u) ^ (row >= 2u ? r1 : 0u) ^ (row >= 3u ? r2 : 0u);
}

// The register advanced over 16 / 32 zero bytes (tables s128 / s256 at S).
__device__ __forceinline__ uint32_t crc_shift(const uint32_t *S, uint32_t v)
{
	return S[v & 0xffu] ^ S[256u + ((v >> 8) & 0xffu)] ^ S[512u + ((v >> 16) & 0xffu)] ^
	       S[768u + (v >> 24)];
}

// Raw CRC-32C (init 0) of 64 bytes: four independent chains of four
// slicing-by-4 steps (one per 16-B chunk), joined pairwise -- six dependent
// LDS lookup levels instead of sixteen.
__device__ __forceinline__ uint32_t crc_piece(const uint32_t *tab, const u32x4 v[4])
{
	uint32_t c[4];
#pragma unroll
	for (uint32_t i = 0; i < 4; ++i) {
		uint32_t x = 0;
#pragma unroll
		for (uint32_t d = 0; d < 4; ++d)
			x = crc32c_u32(tab, x, v[i][d]);
		c[i] = x;
	}
	const uint32_t h0 = crc_shift(tab + CRC_S128, c[0]) ^ c[1];
	const uint32_t h1 = crc_shift(tab + CRC_S128, c[2]) ^ c[3];
	return crc_shift(tab + CRC_S256, h0) ^ h1;
}

// Wave-cooperative CRC-32C of the SCTP check (all 64 lanes active): lane f
// asks (ask != 0) for the CRC over frame bytes [l4, len) of its frame (batch
// offset boff) with the checksum field [l4 + 8, l4 + 12) taken as zero, init
// ~0, inverted.  The n = len - l4 bytes are cut into 64-B pieces counted from
// l4: nf = n / 64 full ones and, when rr = n % 64 != 0, a last one of rr
// bytes zero-padded to 64 (its 16-B parts past rr not loaded, the boundary
// word masked).  The pieces of all lanes are numbered in lane order and dealt
// out 64 per round as in ck_sum_wave (16-B loads from l4 on: no byte below l4
// is ever read into a CRC, and the checksum field is dword 2 of piece 0).
// CRC is linear over GF(2): a lane computes the raw CRC (init 0) of its
// piece (crc_piece) and shifts it by the 64-B blocks after it, x^(512 (nf -
// k)) (table z; the padded last piece counts as a block even when rr = 0);
// the frame's register is the XOR of its pieces' (prefix XOR over the round)
// = raw(message) x^(8 (64 - rr)), brought back by x^(-8 (64 - rr)) (table
// yinv), plus the init's contribution ~0 x^(8 n) = y1[rr] z[nf].  One GF(2)
// multiply per piece and two per frame.  (Round 3 had the last piece walked
// by its owner lane, up to 18 dependent table steps after the rounds.)
// Returns the finished CRC for the asking lanes.
__device__ __forceinline__ uint32_t sctp_crc_wave(__amdgpu_buffer_rsrc_t rs, uint32_t boff,
						  uint32_t l4, uint32_t len, uint32_t ask,
						  uint32_t lane, const uint32_t *tab)
{
	const uint32_t *zt = tab + CRC_Z;
	const uint32_t n = ask ? len - l4 : 0u, nf = n >> 6, rr = n & 63u;
	const uint32_t np = nf + (rr != 0u ? 1u : 0u);
	const uint32_t incl = wave_scan_add(np, lane);
	const uint32_t first = incl - np;
	const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, WAVE - 1);
	const uint32_t p0 = boff + l4;   // batch offset of the first L4 byte
	const uint32_t fi = nf | (rr << 16);
	uint32_t acc = 0;
	for (uint32_t B = 0; B < total; B += WAVE) {
		const uint32_t g = B + lane;
		uint32_t lo = 0;
#pragma unroll
		for (uint32_t st = WAVE / 2; st >= 1; st >>= 1) {
			const uint32_t c = lo + st;
			lo = lane_get(first, c) <= g ? c : lo;
		}
		const uint32_t k = g - lane_get(first, lo);   // piece number from l4
		const uint32_t f2 = lane_get(fi, lo), fnf = f2 & 0xffffu;
		const uint32_t ob = lane_get(p0, lo) + 64u * k;
		const bool live = g < total;
		// bytes of the piece: 64, or the last piece's rr
		const uint32_t vb = k < fnf ? 64u : f2 >> 16;
		u32x4 v[4];
#pragma unroll
		for (uint32_t i = 0; i < 4; ++i)
			v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (live && 16u * i < vb) ? ob + 16u * i
									     : OOB_OFF, 0, 0);
		const uint32_t bm = (1u << (8u * (vb & 3u))) - 1u;
#pragma unroll
		for (uint32_t d = 0; d < 16; ++d) {
			const uint32_t w = v[d >> 2][d & 3];
			v[d >> 2][d & 3] = (d == 2u && k == 0u) ? 0u   // the checksum field
				: (4u * d + 4u <= vb ? w : ((4u * d < vb) ? (w & bm) : 0u));
		}
		const uint32_t crc = crc_piece(tab, v);
		const uint32_t r = live ? crc_mulmod(crc, zt[fnf - k]) : 0u;
		const uint32_t P = wave_scan_xor(r, lane);
		const uint32_t a0 = first > B ? first - B : 0u;
		const uint32_t e = min(incl > B ? incl - B : 0u, (uint32_t)WAVE);
		const uint32_t pe = lane_get(P, e > 0u ? e - 1u : 0u);
		const uint32_t pa = lane_get(P, a0 > 0u ? a0 - 1u : 0u);
		acc ^= (e > a0) ? (pe ^ (a0 > 0u ? pa : 0u)) : 0u;
	}
	const uint32_t raw = crc_mulmod(acc, tab[CRC_YINV + 64u - rr]);
	return ~(raw ^ crc_mulmod(tab[CRC_Y1 + rr], zt[nf]));
}

// _odp_packet_l4_chksum (odp_packet.c:2065-2138) for the lanes whose parse
// returned 0, with the partial sums parse_ipv4 / parse_ipv6 / parse_tcp /
// parse_udp / parse_sctp prepare (odp_parse.c:146-148, 212-214, 267-275,
// 298-313, 341-351): UDP / TCP one's-complement sum over the pseudo header
// and [l4, frame_len) (ck_sum_wave, the whole wave cooperating), SCTP
// CRC-32C over [l4, frame_len) with the checksum field taken as zero.
// Fragments are skipped.  A failure sets l4_chksum_err and the protocol's
// error bit, and drops the packet under drop_<proto>_err.  Called with every
// lane of the wave active.
__device__ __forceinline__ void l4_chksum(const Pkt &k, Parsed &p, uint32_t opt,
					  __amdgpu_buffer_rsrc_t rs, uint32_t boff, uint32_t lane,
					  bool valid, const uint32_t *crc_tab)
{
	const uint32_t f = p.flags, len = k.len, l3 = p.l3, l4 = p.l4;
	const bool go = valid && p.ret == 0 && !(f & F_IPFRAG);
	const uint32_t kind = !go ? 0u
		: (((opt & OPT_UDP_CK) && (f & F_UDP) && !p.udp_zero) ? 1u
		: (((opt & OPT_TCP_CK) && (f & F_TCP)) ? 2u
		: (((opt & OPT_SCTP_CK) && (f & F_SCTP)) ? 3u : 0u)));
	const bool sum = kind == 1u || kind == 2u;
	uint64_t s = 0;
	uint32_t cnt = 0, base = 0, prm = 0;
	if (__ballot(sum) != 0ull) {
		if (sum) {
			if (f & F_IPV4) {
				s = (uint64_t)r32(k, l3 + 12u) + r32(k, l3 + 16u);
			} else {
				for (uint32_t i = 0; i < 8u; ++i)
					s += r32(k, l3 + 8u + 4u * i);
			}
			if (kind == 1u)   // udp->length as stored, IPPROTO_UDP << 8
				s += r16(k, l4 + 4u) + (17u << 8);
			else              // odp_cpu_to_be_16(frame_len - l4), IPPROTO_TCP << 8
				s += (((len - l4) & 0xffu) << 8) + (((len - l4) >> 8) & 0xffu) + (6u << 8);
			// the parse guarantees l4 + 8 <= len (UDP) / l4 + 20 <= len (TCP)
			if (l4 >= 32u && l4 < 64u) {
				// bytes [l4, 64) are in the staged window (bytes past the
				// frame read 0 there): summed from LDS, so the wave's
				// pieces start at byte 64 and a frame of at most 64 B
				// reads nothing more (dword rows 8-15, the first one from
				// l4's, its lower half cut when l4 is 2 mod 4: congruent
				// modulo 0xffff either way)
#pragma unroll
				for (uint32_t d = 8; d < 16; ++d) {
					const uint32_t w = k.w[d * RS];
					const uint32_t m = 4u * d + 4u <= l4 ? 0u : (4u * d < l4 ? 0xffff0000u : ~0u);
					s += w & m;
				}
				cnt = len > 64u ? (len - 64u + 63u) >> 6 : 0u;
				base = boff + 64u;
				prm = len > 64u ? (len - 64u) << 6 : 0u;
			} else {
				const uint32_t p0 = l4 & ~63u;
				cnt = (len - p0 + 63u) >> 6;
				base = boff + p0;
				prm = (l4 - p0) | ((len - p0) << 6);
			}
		}
#ifndef DIAG_CK_NOSUM
		s += ck_sum_wave(rs, base, prm, cnt, lane);
#endif
	}
	bool bad = sum && ck_finalize(s) != 0xffffu;   // ~sum != 0
	if (__ballot(kind == 3u) != 0ull) {
		// frames with at most CRC_ZN 64-B pieces: the wave cooperates;
		// longer (jumbo) ones: one lane walks its frame
		const bool wv = kind == 3u && len - l4 < 64u * CRC_ZN;
#ifdef DIAG_CK_NOSCTP
		const uint32_t crc = 0u;
#else
		const uint32_t crc = sctp_crc_wave(rs, boff, l4, len, wv ? 1u : 0u, lane, crc_tab);
#endif
		if (wv)
			bad = crc != r32(k, l4 + 8u);
		if (__ballot(kind == 3u && !wv) != 0ull) {
			if (kind == 3u && !wv)
				bad = sctp_crc(k, rs, boff, l4, crc_tab) != r32(k, l4 + 8u);
		}
	}
#ifdef DIAG_CK_OK
	// diagnostic timing variants: every L4 checksum passes, so variants
	// that skip checksum work classify the same lanes downstream
	bad = false;
#endif
	if (kind != 0u) {
		p.flags |= F_L4CK_DONE;
		if (bad) {
			p.err |= E_L4CK | (kind == 1u ? E_UDP : (kind == 2u ? E_TCP : E_SCTP));
			const uint32_t d = kind == 1u ? OPT_DROP_UDP : (kind == 2u ? OPT_DROP_TCP : OPT_DROP_SCTP);
			p.ret = (opt & d) ? -1 : 1;
		}
	}
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

// L4 protocol table (one LDS word per IP protocol number, copied in at block
// start): the F_L4 / kind flags _odp_packet_parse_common_l3_l4 sets for the
// protocol (odp_parse.c:395-460) in bits 0..26, and in bits 28..29 the L4
// header check the protocol takes (1 TCP, 2 UDP, 3 SCTP).  Protocol 255 is
// "no IP" and 0 a bad IP header: neither sets anything.
#define L4K_TCP 1u
#define L4K_UDP 2u
#define L4K_SCTP 3u
struct L4Tab {
	uint32_t v[256];
	constexpr L4Tab() : v()
	{
		v[1] = v[58] = F_L4 | F_ICMP;
		v[4] = F_L4;
		v[6] = F_L4 | F_TCP | (L4K_TCP << 28);
		v[17] = F_L4 | F_UDP | (L4K_UDP << 28);
		v[51] = F_L4 | F_IPSEC | F_AH;
		v[50] = F_L4 | F_IPSEC | F_ESP;
		v[132] = F_L4 | F_SCTP | (L4K_SCTP << 28);
		v[59] = F_L4 | F_NO_NEXT;
	}
};
static __constant__ L4Tab c_l4tab;

// Branch-light parse of the common frame shapes: DIX or SNAP, 0-2 VLAN tags,
// IPv4 (any IHL / errors), IPv6 without HBH / routing headers, ARP, every L4.
// The reference places L3 at 14/18/22/26/30, so every L3 and L4 offset here is
// 2 (mod 4) and all header words are one alignbyte of two window dwords.
// Per lane it is written as selects (no data-dependent lane branches); the
// only branches are wave-uniform ones that skip a header family no lane of
// the tile has (tags / SNAP, IPv4, IPv6, TCP-UDP-SCTP checks), so a tile of
// untagged IPv4 frames runs just the IPv4 and its L4 code.  Lanes it cannot
// finish (IPv6 extension chain, L4 header past the window) set `slow` and are
// re-parsed by parse_packet.  Results are identical to parse_packet for every
// lane that does not set `slow`.
// The byte-dependent L4 header checks of parse_fast for one lane: TCP data
// offset (l4+12; tcp = a TCP header that is not dropped), UDP length and,
// for destination port 4500, the NAT-T marker (l4..l4+11; udp = a UDP header
// that is not dropped).  Returns the error bits, the IPsec flag and `need`,
// the bytes past l4 the checks read (the caller tests them against the
// staged window).
__device__ __forceinline__ void l4_bytes(const Pkt &k, uint32_t l4, bool tcp, bool udp, uint32_t &err,
					 uint32_t &f, uint32_t &need)
{
	// L4 header bytes l4 .. l4+15 (dwords jl .. jl+4, byte shift 2)
	const uint32_t jl = min((l4 - 2u) >> 2, (uint32_t)(WIN / 4 - 4));
	uint32_t m[5], lb[4];
#pragma unroll
	for (int i = 0; i < 5; ++i)
		m[i] = k.w[(jl + i) * RS];
#pragma unroll
	for (int i = 0; i < 4; ++i)
		lb[i] = __builtin_amdgcn_alignbyte(m[i + 1], m[i], 2u);
	const bool natt = (lb[0] >> 16) == 0x9411u;   // be16(4500) raw
	need = tcp ? 13u : (udp ? (natt ? 12u : 6u) : 0u);
	err = (tcp && ((lb[3] & 0xffu) >> 4) < 5u) ? E_TCP : 0u;
	const uint32_t ulen = bsw16(lb[1]);
	err |= (udp && ulen < 8u) ? E_UDP : 0u;
	f = (udp && ulen >= 8u && natt && ulen > 4u && lb[2] != 0u) ? F_IPSEC : 0u;
}

// dwin != 0 (tree kernels): a lane longer than the staged window whose L4
// check bytes lie in [k.win, dwin) is not sent to the general parser: `dfr`
// is set, its L4 error bits and IPsec flag are left out, and the kernel
// checks them (l4_bytes) once those bytes are staged.
__device__ __forceinline__ Parsed parse_fast(const Pkt &k, const uint32_t *l4tab, bool &slow,
					     uint32_t dwin, bool &dfr)
{
	Parsed r;
	const uint32_t len = k.len;
	const uint32_t w0 = k.w[0], w1 = k.w[RS], w3 = k.w[3 * RS];

	uint32_t f = F_L2 | F_ETH;
	f |= len > 1514u ? F_JUMBO : 0u;
	f |= (w0 & 1u) << 8;   // F_ETH_MCAST
	f |= (w0 == 0xffffffffu && (w1 & 0xffffu) == 0xffffu) ? F_ETH_BCAST : 0u;
	const uint32_t et0 = bsw16(w3);
	uint32_t e = et0, off = 14u, err = 0u;
	bool snap_err = false;
	if (__ballot(et0 < 1514u || et0 == 0x88A8u || et0 == 0x8100u) != 0ull) {
		// some lane has SNAP or a tag
		uint32_t w[8];
#pragma unroll
		for (int i = 0; i < 8; ++i) {
			w[i] = k.w[i * RS];
			// opaque register value: keeps the selects below v_cndmask
			// instead of letting the compiler fold them into an indexed
			// (scratch) load of w[]
			asm("" : "+v"(w[i]));
		}
		const bool snap = et0 < 1514u;
		snap_err = snap && et0 > len - 14u;
		e = snap ? bsw16(w[5]) : et0;
		off = snap ? 22u : 14u;
		// outer tag: type at off+2 = 16 / 24
		const bool qinq = e == 0x88A8u;
		e = qinq ? bsw16(snap ? w[6] : w[4]) : e;
		off += qinq ? 4u : 0u;
		// inner tag: type at off+2 = 16 / 20 / 24 / 28 (off = 14 + 8 snap +
		// 4 qinq); selected by the two booleans, not by an index (an index
		// would make the compiler spill w[] to scratch)
		const bool vlan = e == 0x8100u;
		const uint32_t wv = snap ? (qinq ? w[7] : w[6]) : (qinq ? w[5] : w[4]);
		e = vlan ? bsw16(wv) : e;
		off += vlan ? 4u : 0u;
		err = snap_err ? E_SNAP : 0u;
		e = snap_err ? 0u : e;
		off = snap_err ? 14u : off;
		f |= (!snap_err && qinq) ? (F_QINQ | F_VLAN) : 0u;
		f |= (!snap_err && vlan) ? F_VLAN : 0u;
	}
	const bool short_l2 = !snap_err && off > len;
	f = short_l2 ? F_L2 : f;
	e = short_l2 ? 0u : e;
	const uint32_t l3 = off;
	r.l3 = l3;

	// IP header bytes l3 .. l3+27 (dwords jb .. jb+7, byte shift 2)
	const uint32_t jb = (l3 - 2u) >> 2;
	uint32_t h[8], hb[7];
#pragma unroll
	for (int i = 0; i < 8; ++i)
		h[i] = k.w[(jb + i) * RS];
#pragma unroll
	for (int i = 0; i < 7; ++i)
		hb[i] = __builtin_amdgcn_alignbyte(h[i + 1], h[i], 2u);   // bytes l3+4i .. +3

	const bool is4 = e == 0x0800u, is6 = e == 0x86DDu, isarp = e == 0x0806u;
	f |= (is4 || is6 || isarp) ? F_L3 : 0u;
	f |= isarp ? F_ARP : 0u;
	uint32_t ip_proto = (is4 || is6) ? 0u : 255u;   // bad IP header / no IP
	uint32_t l4 = 0xFFFFu;
	bool non_first = false, sl = false;
	if (__ballot(is4) != 0ull) {
		// IPv4 (parse_ipv4, odp_parse.c:112-167)
		const uint32_t vi = hb[0] & 0xffu, ihl = vi & 0xfu;
		const uint32_t tot = bsw16(hb[0] >> 16);
		const bool bad4 = ihl < 5u || (vi >> 4) != 4u || 20u > len - l3 || tot > len - l3;
		const uint32_t frag = bsw16(hb[1] >> 16);
		const uint32_t dst = __builtin_bswap32(hb[4]);
		uint32_t f4 = F_IPV4;
		f4 |= ihl > 5u ? F_IPOPT : 0u;
		f4 |= (frag & 0x3fffu) ? F_IPFRAG : 0u;
		f4 |= dst == 0xffffffffu ? F_IP_BCAST : 0u;
		f4 |= (dst >> 28) == 0xeu ? F_IP_MCAST : 0u;
		const bool ok4 = is4 && !bad4;
		f |= is4 ? (bad4 ? F_IPV4 : f4) : 0u;
		err |= (is4 && bad4) ? E_IP : 0u;
		ip_proto = ok4 ? ((hb[2] >> 8) & 0xffu) : ip_proto;
		l4 = ok4 ? l3 + ihl * 4u : l4;
		non_first = ok4 && (frag & 0x1fffu) != 0u;
	}
	if (__ballot(is6) != 0ull) {
		// IPv6 (parse_ipv6, :174-246)
		const uint32_t plen = bsw16(hb[1]);
		const bool bad6 = ((hb[0] & 0xffu) >> 4) != 6u || 40u > len - l3 || plen + 40u > len - l3;
		const uint32_t nh = (hb[1] >> 16) & 0xffu;
		uint32_t f6 = F_IPV6;
		f6 |= (hb[6] & 0xffu) == 0xffu ? F_IP_MCAST : 0u;
		f6 |= nh == 44u ? (F_IPOPT | F_IPFRAG) : 0u;
		const bool ok6 = is6 && !bad6;
		f |= is6 ? (bad6 ? F_IPV6 : f6) : 0u;
		err |= (is6 && bad6) ? E_IP : 0u;
		ip_proto = ok6 ? nh : ip_proto;
		l4 = ok6 ? l3 + 40u : l4;
		sl = ok6 && (nh == 0u || nh == 43u);   // extension chain: general parser
	}

	// L4 (_odp_packet_parse_common_l3_l4, :395-460)
	const uint32_t pt = l4tab[ip_proto];
	f |= pt & 0x0fffffffu;
	const uint32_t kc = pt >> 28;
	const bool chk = kc != 0u && !non_first;   // a TCP / UDP / SCTP header to check
	bool drop = false;
	dfr = false;
	if (__ballot(chk) != 0ull) {
		const bool tcp = chk && kc == L4K_TCP, udp = chk && kc == L4K_UDP;
		const bool sctp = chk && kc == L4K_SCTP;
		// TCP (parse_tcp, :299-316), UDP (parse_udp, :321-354), SCTP
		// (parse_sctp, :362-388): the drops depend on the length only
		const bool tcp_drop = tcp && l4 + 20u > len;
		const bool udp_drop = udp && l4 + 8u > len;
		const bool sctp_drop = sctp && l4 + 12u > len;
		uint32_t e4, f4, need;
		l4_bytes(k, l4, tcp && !tcp_drop, udp && !udp_drop, e4, f4, need);
		// a lane whose checked bytes are not all staged takes the general
		// parser -- or, with a deferral window (dwin, tree kernels), has
		// them checked once its bytes past the window are staged (l4_bytes
		// again, mi_cls_kernel)
		const bool far = chk && l4 + need > k.win;
		dfr = far && l4 + need <= dwin && len > k.win;
		sl = sl || (far && !dfr);
		err |= dfr ? 0u : e4;
		f |= dfr ? 0u : f4;
		err |= (sctp && !sctp_drop && ((len - l4) & 0xffffu) < 12u) ? E_SCTP : 0u;
		drop = tcp_drop || udp_drop || sctp_drop;
	}

	slow = sl;
	r.l4 = l4;
	r.flags = f;
	r.err = err;
	r.ret = drop ? -1 : (err != 0u ? 1 : 0);
	return r;
}

// --------------------------------------------------------- field registers
// What the term verifiers compare is read on use from the packet window
// (LDS; HBM past it) rather than cached in registers: the window stays valid
// for the whole tile, and caching every kind the program might use would
// hold ~20 VGPRs through the descent.
struct Fields {
	Pkt k;
	uint32_t l3, l4, f;
};

// Where the key words of a term kind sit (verify_pmr_<term>,
// odp_classification.c:931-1357): 4-byte little-endian words at
// base + add, or base + alt when the lane's flags have `altf`
// (QinQ outer tag, IPv4 vs IPv6 next-header, AH vs ESP SPI); base is the
// frame start, L3 or L4.  The term's mask words cut each word down to the
// field (e.g. 0xffff for a 16-bit field), so every kind but LEN, PCP and
// DSCP is "read words, AND mask".  gate: the packet has the field iff its
// flags share a bit with `gate` (~0: always).  The verifiers' presence tests
// map onto single flag masks: eth && vlan is F_VLAN (both parsers set VLAN
// only on frames that keep F_ETH), vlan || qinq, ipv4 || ipv6, ah || esp;
// "l2 && l3 valid" (custom L3) is F_L2 plus the l3 != invalid test in
// field_off.
enum { FB_FRAME = 0, FB_L3 = 1, FB_L4 = 2 };
// classification-block pseudo kind: UDP and TCP port terms with one mask
// (class_of), the raw port word at l4 tagged with the protocol
#define K_L4PORT 0x40u
struct FDesc {
	uint32_t base, add, alt, altf, gate;
};

__host__ __device__ inline FDesc fdesc(uint32_t kind, uint32_t toff)
{
	FDesc d = { FB_FRAME, 0u, 0u, 0u, 0u };
	switch (kind) {
	case MI_K_ETH0: d = { FB_FRAME, 12u, 12u, 0u, F_ETH }; break;
	case MI_K_ETHX: d = { FB_FRAME, 16u, 20u, F_QINQ, F_VLAN | F_QINQ }; break;
	case MI_K_VID0: d = { FB_FRAME, 14u, 14u, 0u, F_VLAN }; break;
	case MI_K_VIDX: d = { FB_FRAME, 14u, 18u, F_QINQ, F_VLAN | F_QINQ }; break;
	case MI_K_DMAC: d = { FB_FRAME, 0u, 0u, 0u, F_ETH }; break;
	case MI_K_PROTO: d = { FB_L3, 6u, 9u, F_IPV4, F_IPV4 | F_IPV6 }; break;
	case MI_K_UDP_DPORT:
	case MI_K_UDP_SPORT: d = { FB_L4, 0u, 0u, 0u, F_UDP }; break;
	case MI_K_TCP_DPORT:
	case MI_K_TCP_SPORT: d = { FB_L4, 0u, 0u, 0u, F_TCP }; break;
	case K_L4PORT: d = { FB_L4, 0u, 0u, 0u, F_UDP | F_TCP }; break;
	case MI_K_SIP: d = { FB_L3, 12u, 12u, 0u, F_IPV4 }; break;
	case MI_K_DIP: d = { FB_L3, 16u, 16u, 0u, F_IPV4 }; break;
	case MI_K_SIP6: d = { FB_L3, 8u, 8u, 0u, F_IPV6 }; break;
	case MI_K_DIP6: d = { FB_L3, 24u, 24u, 0u, F_IPV6 }; break;
	case MI_K_SPI: d = { FB_L4, 0u, 4u, F_AH, F_AH | F_ESP }; break;
	case MI_K_CUSTOM_FRAME: d = { FB_FRAME, toff, toff, 0u, ~0u }; break;
	case MI_K_CUSTOM_L3: d = { FB_L3, toff, toff, 0u, F_L2 }; break;
	default: break;
	}
	return d;
}

__device__ __forceinline__ bool kind_special(uint32_t kind)
{
	return kind == MI_K_LEN || kind == MI_K_PCP0 || kind == MI_K_DSCP || kind == MI_K_NEVER ||
	       kind == MI_K_ALWAYS;
}

// LEN / PCP / DSCP values and presence (NEVER: absent, ALWAYS: present)
__device__ __forceinline__ bool special_value(uint32_t kind, const Fields &x, uint32_t &v)
{
	if (kind == MI_K_LEN) {
		v = x.k.len;
		return true;
	}
	if (kind == MI_K_PCP0) {
		v = (r16(x.k, 14) & 0xffu) >> 5;
		return (x.f & F_VLAN) != 0u;
	}
	if (kind == MI_K_DSCP) {
		v = (x.f & F_IPV4) ? (rb(x.k, x.l3 + 1) >> 2)
				   : ((be32(x.k, x.l3) & 0x0fc00000u) >> 22);
		return (x.f & (F_IPV4 | F_IPV6)) != 0u;
	}
	v = 0;
	return kind == MI_K_ALWAYS;
}

// Byte offset of a kind's first key word in the lane's frame, and whether the
// packet has the field (custom kinds: the frame must extend past
// offset + size, verify_pmr_custom_*).
__device__ __forceinline__ uint32_t field_off(const FDesc &d, uint32_t kind, uint32_t size,
					      const Fields &x, bool &present)
{
	const uint32_t base = d.base == FB_L3 ? x.l3 : (d.base == FB_L4 ? x.l4 : 0u);
	const uint32_t o = base + ((x.f & d.altf) ? d.alt : d.add);
	present = d.gate == ~0u || (x.f & d.gate) != 0u;
	if (kind == MI_K_CUSTOM_L3)
		present = present && x.l3 != 0xFFFFu;
	if (kind == MI_K_CUSTOM_FRAME || kind == MI_K_CUSTOM_L3)
		present = present && !(x.k.len <= o + size);
	return o;
}

__device__ __forceinline__ Fields fields_of(const Pkt &k, const Parsed &p)
{
	Fields x;
	x.k = k;
	x.l3 = p.l3;
	x.l4 = p.l4;
	x.f = p.flags;
	return x;
}

// ----------------------------------------------------------- Toeplitz hash
// thash_softrss (protocols/thash.h:82-99) with the default 40-B key
// (odp_classification.c:50-58), key words in big-endian order.
static __constant__ uint32_t c_rss_key[10] = {
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
// read-only encoding (32-bit words):
//
//   [0, 16)              header (DH_* below)
//   [hot_off, +hot_words)  HOT region -- everything a lane may look up with its
//                        own (per-lane) index.  All offsets inside it are
//                        relative to hot_off, so the kernel can read it from
//                        HBM or from a copy in LDS with the same indices:
//      CoS table        4 words per CoS slot: #rules, bit-vector block (0 =
//                       linear scan), meta = action | num_queue<<8 |
//                       hash_proto<<16 | index<<24, first rule record
//      BV blocks        see below
//   [prog_off, ...)      COLD region -- 16-word rule records, read only with
//                        wave-uniform (scalar) loads by the linear engine:
//        w0  = inline terms | ext terms<<8 | mark<<16
//        w1  = dst CoS | ext word offset<<8
//        w2.. terms: op word (kind | size<<8 | nw<<16), [offset word for custom
//             kinds], then nw (mask, value) word pairs; terms that do not fit
//             the 14 inline words continue at the ext offset.
typedef const __attribute__((address_space(4))) uint32_t *cword_t;   // scalar loads
typedef const __attribute__((address_space(3))) uint32_t *lword_t;   // LDS
typedef const __attribute__((address_space(1))) uint32_t *gword_t;   // HBM

enum { DH_MAGIC = 0, DH_NCOS, DH_DEFAULT, DH_ERROR, DH_DEFAULT_VALID, DH_USED, DH_MAX_HOPS,
       DH_HOT_OFF, DH_PROG_OFF, DH_TOTAL, DH_HOT_WORDS,
       // furthest byte past L3 / L4 / the frame start any term (or the hash
       // queue tuple) of the program reads: the kernel's window predictor
       DH_L3END, DH_L4END, DH_FREND,
       // hot-region word of the joint groups' directory (0: none)
       DH_JOINT, DH_WORDS = 16 };
#define DEV_MAGIC 0x33564544u   // "DEV3"
#define REC_WORDS 16u
#define COS_WORDS 4u
#define C_NR 0u
#define C_BV 1u
#define C_META 2u
#define C_REC0 3u
#define BV_MAX_CLS 8u
#define BV_CLS_WORDS 16u
#define BV_WIDE_WORDS 8u        // wide bitmap rows: up to 256 rules
// class words 14-15: the field descriptor of the class's kind (fdesc()),
// resolved at rule load so the device decodes it instead of switching on
// kind: w14 = add | alt << 16; w15 = gate (flag mask, bits 0-23) | base << 24
// | alt-flag code << 26 (1 QinQ, 2 IPv4, 3 AH) | BVF_* << 28
#define BVC_AO 14u
#define BVC_DESC 15u
#define BVF_SPECIAL 1u          // LEN / PCP / DSCP: special_value()
#define BVF_CUSTOM 2u           // custom frame / L3: length test
#define BVF_L3 4u               // custom L3: l3 must be valid
#define BVF_TAG 8u              // merged UDP/TCP port class: protocol tag at bit cr(3)
#define BV_EMPTY 0xFFFFFFFFu
#define BV_NONE 0xFFFFFFFEu
// direct blocks: a slot value / miss word is the rule's result word
// (dst | leaf << 8 | mark << 16) with this bit set; 0 / BV_EMPTY: no rule
#define BV_RES_VALID 0x200u
// joint tables (tree programs): direct blocks sharing a class record, and
// bitmap blocks over the same class records, probe one table per class over
// (key, CoS); header word 1 of a direct member block, word 13 of a bitmap
// member's class record (and word 6 of the class's info in the group's
// info) say how the CoS slot enters the key: in 8 bits of a one-word key no
// rule can set (at bit BVJ_SHIFT's value), or appended as the last key word.
// Group info (hc[DH_JOINT + group - 1] = its word): kind (0 direct, 2
// bitmap), #classes, alive rows and result-array words per CoS slot
// (bitmap), then 8 words per class: class record, #buckets, table, m1, m2,
// miss values per CoS slot, BVJ flags
#define BVJ_ONEWORD 0x10000u
#define BVJ_APPEND 0x20000u
#define BVJ_SHIFT 18u
// CoS entry word C_BV: block offset (bits 0-23), joint group + 1 (bits
// 24-30, tree programs), chain of blocks (bit 31, flat programs)
#define C_BV_OFF 0xFFFFFFu

// Classification block of a CoS ("BV" block for historical reasons), used
// when its rules fall into at most BV_MAX_CLS key classes (a key class is one
// (term kind, mask[, offset, size]) combination).  build_bv() explains the
// modes; the layout (word indices into the hot region) is:
//   b[0] mode (0 direct, 1 candidate, 2 bitmap, 3 wide bitmap, 4 single
//   candidate), b[1] #classes, b[2] result words (dst | leaf<<8 | mark<<16
//   per rule; leaf = the destination CoS has no rules, so the descent ends
//   there), b[3] first rule without a classified term (BV_NONE: none), b[4]
//   rule records (bitmap: alive row; wide: block-relative index of the
//   nw-word alive row), b[5] record words, b[6] wide: nw = words per row
//   class record (16 words): kind, nkey, miss value (wide: index of the miss
//                   row), offset (custom) / tag bit (merged ports), size,
//                   mask[4], #buckets, table offset, cuckoo multipliers m1,
//                   m2, list base, field descriptor (BVC_AO, BVC_DESC)
//   modes 1-4: class k's record at b[8 + 16 k]
//   direct blocks (mode 0, split class): the record holds only what the
//                   class is and is shared by every direct block with that
//                   class; the block keeps the 6-word class info in b[2..7]:
//                   shared record index, miss word, #buckets, table offset,
//                   m1, m2 (no results array)
//   table (16-B aligned): one-word keys 2 slots of (key, value) per 16-B
//             bucket; 2-3-word keys one 16-B slot (key words, value);
//             4-word keys one 32-B slot; value 0: empty
//     direct: the result word of the first live rule with this key or
//             without a term of the class, | BV_RES_VALID (BV_EMPTY: none)
//     bitmap: the 32-bit row of rules with this key or without a term
//     wide:   index of the nw-word row of rules with this key or without a
//             term of the class (rows are deduplicated)
//     candidate: key id | list length << 12 | list offset << 20; the list
//             holds the rules filed under this key, in scan order
//     single candidate: key id << 16 | 1 + the rule filed under the key
//   rule record (candidate, 1 + ceil(#classes / 2) words): constrained-
//             class mask (bit 31: never holds), then the required key id of
//             class c in half c & 1 of word 1 + c / 2
//   rule record (single candidate, 4 or 8 words): constrained-class mask,
//             then the required value (key id for longer keys) per class,
//             or (compact, 4 words) of the <= 3 constrained classes in order

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
	const uint32_t sz = (op >> 8) & 0xffu;
	const uint32_t nw = (op >> 16) & 0xffu;
	if (kind_special(kind)) {
		uint32_t v;
		const bool ok = special_value(kind, x, v) &&
				(kind == MI_K_ALWAYS || eq1(v, prog[q + 1], prog[q + 2]));
		q += 1u + 2u * nw;
		return ok;
	}
	const bool custom = kind == MI_K_CUSTOM_FRAME || kind == MI_K_CUSTOM_L3;
	const FDesc d = fdesc(kind, custom ? prog[q + 1] : 0u);
	const uint32_t q0 = q + (custom ? 2u : 1u);
	bool ok;
	const uint32_t o = field_off(d, kind, sz, x, ok);
	for (uint32_t i = 0; i < nw; ++i)
		ok = ok && eq1(r32(k, o + 4u * i), prog[q0 + 2u * i], prog[q0 + 2u * i + 1u]);
	q = q0 + 2u * nw;
	return ok;
}

__device__ __forceinline__ uint32_t bv_fold(const uint32_t k[4])
{
	uint32_t h = k[0] * 0x9E3779B1u ^ k[1] * 0x85EBCA77u ^ k[2] * 0xC2B2AE3Du ^ k[3] * 0x27D4EB2Fu;
	return h ^ (h >> 15);
}

// Cuckoo bucket of a key: x = the key word (one-word keys) or bv_fold (longer
// keys), folded to 24 bits that depend on every key bit, times a 24-bit
// multiplier; bits 8-23 of the product, scaled to [0, nb) (nb <= 65536).
// (The product's top bits stay near zero for small keys -- DSCP, IP
// protocol, small ports -- which then crowd a few buckets; bits 8-23 spread
// any key set.)  Two v_mul_u32_u24 (full rate, unlike a 32-bit multiply).
// host_bucket() is the same arithmetic.
__device__ __forceinline__ uint32_t bv_bucket(uint32_t x, uint32_t m, uint32_t nb)
{
	// (__umul24 returns int: shift the unsigned products)
	const uint32_t h = (uint32_t)__umul24(x ^ (x >> 16), m);
	return (uint32_t)__umul24((h >> 8) & 0xffffu, nb) >> 16;
}

// Word readers of a classification block: wave-uniform blocks are read with
// scalar loads from HBM (DescU), per-lane blocks from the hot region (LDS or
// HBM, DescL).
// A wave-uniform 16-word descriptor (block header, class record) held in
// SGPRs: one s_load_dwordx16, one wait, instead of a scalar load and wait
// per word on use.
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
struct DescV {
	u32x16 v;
	__device__ __forceinline__ uint32_t operator()(uint32_t i) const { return v[i]; }
};
struct DescU {
	cword_t p;
	cword_t h;              // start of the hot region (root())
	static constexpr bool per_lane = false;
	__device__ __forceinline__ uint32_t operator()(uint32_t i) const { return p[i]; }
	__device__ __forceinline__ DescU at(uint32_t o) const { return DescU{ p + o, h }; }
	// 16 words at o, loaded at once
	__device__ __forceinline__ DescV vec(uint32_t o) const
	{
		return DescV{ *(const __attribute__((address_space(4))) u32x16 *)(p + o) };
	}
	__device__ __forceinline__ DescV hdr() const { return vec(0u); }
	__device__ __forceinline__ DescV vec8(uint32_t o) const { return vec(o); }
	// 16 words at hot-region word o (a direct block's shared class record)
	__device__ __forceinline__ DescV root(uint32_t o) const { return DescU{ h + o, h }.vec(0u); }
};
// Engine value of a program-specialised kernel whose default CoS has a chain
// of blocks (flat programs only): the blocks, their offsets and engines are
// the spec's constants (S::nblk, S::boff, S::bmode).
#define FM_CHAIN 5

// A classification block known when the kernel is compiled (program-
// specialised kernels, mi_cls_spec.cpp): S::blk holds the default CoS's block
// words (header and class records, zero-padded by 16 words) and S::root a
// direct block's shared class record.  Every read has a constant index once
// bv_eval's class loop is unrolled, so the block's words fold into the
// instructions as immediates: no scalar loads, no decode of class records at
// run time.
template <typename S> struct DescC {
	uint32_t o;
	cword_t h;              // the hot region (a chain's further blocks, read as DescU)
	static constexpr bool per_lane = false;
	__device__ __forceinline__ uint32_t operator()(uint32_t i) const { return S::blk[o + i]; }
	__device__ __forceinline__ DescC at(uint32_t o2) const { return DescC{ o + o2, h }; }
	__device__ __forceinline__ DescV vec(uint32_t o2) const
	{
		DescV d;
#pragma unroll
		for (uint32_t i = 0; i < 16; ++i)
			d.v[i] = S::blk[o + o2 + i];
		return d;
	}
	__device__ __forceinline__ DescV hdr() const { return vec(0u); }
	__device__ __forceinline__ DescV vec8(uint32_t o2) const { return vec(o2); }
	__device__ __forceinline__ DescV root(uint32_t) const
	{
		DescV d;
#pragma unroll
		for (uint32_t i = 0; i < 16; ++i)
			d.v[i] = S::root[i];
		return d;
	}
};
// 16-byte read of the hot region (LDS: ds_read_b128, HBM: global dwordx4);
// i is a multiple of 4 (hot-region blocks, buckets and rows are 16-B aligned)
__device__ __forceinline__ u32x4 ld4(lword_t H, uint32_t i)
{
	return *(const __attribute__((address_space(3))) u32x4 *)(H + i);
}
__device__ __forceinline__ u32x4 ld4(gword_t H, uint32_t i)
{
	return *(const __attribute__((address_space(1))) u32x4 *)(H + i);
}

// Per-lane descriptor in the hot region: words on demand, or 16 words at
// once with four 16-B reads (vec: block headers and class records are
// 16-B aligned), instead of one dependent read per word used.
template <typename T> struct DescL {
	T p;
	uint32_t b;
	cword_t h;              // the hot region in the constant address space (scalar loads)
	static constexpr bool per_lane = true;
	__device__ __forceinline__ uint32_t operator()(uint32_t i) const { return p[b + i]; }
	__device__ __forceinline__ DescL at(uint32_t o) const { return DescL{ p, b + o, h }; }
	__device__ __forceinline__ DescV vec(uint32_t o) const
	{
		const u32x4 q0 = ld4(p, b + o), q1 = ld4(p, b + o + 4u), q2 = ld4(p, b + o + 8u),
			    q3 = ld4(p, b + o + 12u);
		DescV d;
		d.v = u32x16{ q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3],
			      q2[0], q2[1], q2[2], q2[3], q3[0], q3[1], q3[2], q3[3] };
		return d;
	}
	__device__ __forceinline__ DescV root(uint32_t o) const { return DescL{ p, o, h }.vec(0u); }
	// 8 words at o (the block header, a split class's info)
	__device__ __forceinline__ DescV vec8(uint32_t o) const
	{
		const u32x4 q0 = ld4(p, b + o), q1 = ld4(p, b + o + 4u);
		DescV d;
		d.v = u32x16{ q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3],
			      0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u };
		return d;
	}
	__device__ __forceinline__ DescV hdr() const { return vec8(0u); }
};

// Key of a packet for one class: the masked field the class's terms
// compare, and whether the packet has that field at all (the term's gate).
template <typename D>
__device__ __forceinline__ bool bv_key(const D &cr, const Pkt &k, const Parsed &p, const Fields &x,
				       uint32_t key[4])
{
	const uint32_t nk = cr(1), desc = cr(BVC_DESC), dfl = desc >> 28;
	key[0] = key[1] = key[2] = key[3] = 0;
	if (dfl & BVF_SPECIAL) {
		uint32_t v;
		const bool pr = special_value(cr(0), x, v);
		key[0] = v & cr(5);
		return pr;
	}
	// the class's field descriptor (fdesc() of its kind, resolved at load)
	const uint32_t ao = cr(BVC_AO), fb = (desc >> 24) & 3u, ac = (desc >> 26) & 3u;
	const uint32_t altf = ac == 1u ? F_QINQ : (ac == 2u ? F_IPV4 : (ac == 3u ? F_AH : 0u));
	const uint32_t base = fb == FB_L3 ? x.l3 : (fb == FB_L4 ? x.l4 : 0u);
	const uint32_t o = base + ((x.f & altf) ? (ao >> 16) : (ao & 0xffffu));
	bool present = (x.f & desc & 0xffffffu) != 0u;
	if (dfl & BVF_CUSTOM)   // verify_pmr_custom_*: the frame extends past the field
		present = present && ((dfl & BVF_L3) == 0u || x.l3 != 0xFFFFu) &&
			  !(x.k.len <= o + cr(4));
	key[0] = r32(k, o) & cr(5);
	if (dfl & BVF_TAG)   // merged UDP/TCP port class
		key[0] |= ((x.f & F_UDP) ? 1u : 2u) << cr(3);
	if (nk > 1u) {
		key[1] = r32(k, o + 4u) & cr(6);
		if (nk > 2u) {
			key[2] = r32(k, o + 8u) & cr(7);
			key[3] = r32(k, o + 12u) & cr(8);
		}
	}
	return present;
}

// Two-choice cuckoo lookup (both candidate buckets read at once, no probe
// loop).  One-word keys: buckets of two (key, value) slots, 16 B, read with
// one 16-B load each.  Longer keys: one slot of nk key words + value per
// bucket.  An empty slot has key words 0 and value 0, and a key sits in at
// most one slot, so OR-ing the values of the slots whose key words equal the
// packet's gives the hit's value, or 0 on a miss.
template <typename T>
__device__ __forceinline__ uint32_t bv_probe(T H, const uint32_t key[4], bool act, uint32_t nk,
					     uint32_t ns, uint32_t tbl, uint32_t m1, uint32_t m2)
{
	// ns = bucket count
	uint32_t val = 0;
	if (nk == 1u) {
		// one-word keys (the common case): bv_fold with zero upper words
		const u32x4 b1 = ld4(H, tbl + 4u * bv_bucket(key[0], m1, ns));
		const u32x4 b2 = ld4(H, tbl + 4u * bv_bucket(key[0], m2, ns));
		val = (b1[0] == key[0] ? b1[1] : 0u) | (b1[2] == key[0] ? b1[3] : 0u) |
		      (b2[0] == key[0] ? b2[1] : 0u) | (b2[2] == key[0] ? b2[3] : 0u);
		return act ? val : 0u;
	}
	// longer keys: one slot per bucket, 16 B (2-3 key words, value) or 32 B
	// (4 key words, value): one or two 16-B reads per bucket
	const uint32_t f = bv_fold(key);
#pragma unroll
	for (uint32_t s = 0; s < 2; ++s) {
		const uint32_t b = bv_bucket(f, s ? m2 : m1, ns);
		uint32_t v;
		bool e;
		if (nk <= 3u) {
			const u32x4 q = ld4(H, tbl + 4u * b);
			e = q[0] == key[0] && q[1] == key[1] && (nk < 3u || q[2] == key[2]);
			v = nk < 3u ? q[2] : q[3];
		} else {
			const u32x4 q = ld4(H, tbl + 8u * b), r = ld4(H, tbl + 8u * b + 4u);
			e = q[0] == key[0] && q[1] == key[1] && q[2] == key[2] && q[3] == key[3];
			v = r[0];
		}
		val = (act && e && v != 0u) ? v : val;
	}
	return val;
}

// The key of a joint group's table (BVJ_*): the CoS slot in 8 free bits of
// a one-word key, or appended as the last key word (selects: nk may differ
// per lane).
__device__ __forceinline__ void joint_key(uint32_t flags, uint32_t cos, uint32_t key[4], uint32_t &nk)
{
	if (flags & BVJ_ONEWORD) {
		key[0] |= cos << ((flags >> BVJ_SHIFT) & 31u);
	} else if (flags & BVJ_APPEND) {
		key[1] = nk == 1u ? cos : key[1];
		key[2] = nk == 2u ? cos : key[2];
		key[3] = nk == 3u ? cos : key[3];
		++nk;
	}
}

// the class record's own table
template <typename D, typename T>
__device__ __forceinline__ uint32_t bv_lookup(const D &cr, T H, const uint32_t key[4], bool act)
{
	return bv_probe(H, key, act, cr(1), cr(9), cr(10), cr(11), cr(12));
}

// Key of a packet for a split class (direct and bitmap blocks: the class
// record is shared, at hot-region word `ro`).  Per-lane blocks whose lanes all
// use one record (a tree level of same-class CoS) read it once with scalar
// loads and decode it in SGPRs.  Returns the presence; nk = key words.
template <typename D>
__device__ __forceinline__ bool split_key(const D &blk, uint32_t ro, bool act, const Pkt &k,
					  const Parsed &p, const Fields &x, uint32_t key[4], uint32_t &nk)
{
	if constexpr (D::per_lane) {
		const unsigned long long am = __ballot(act);
		const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane(
			(int)ro, am ? (int)__builtin_ctzll(am) : 0);
		if (__ballot(act && ro != r0) == 0ull) {
			const auto cu = DescU{ blk.h + r0, blk.h }.vec(0u);
			nk = cu(1);
			return bv_key(cu, k, p, x, key);
		}
	}
	const auto cr = blk.root(ro);
	nk = cr(1);
	return bv_key(cr, k, p, x, key);
}

// First holding rule of one non-direct block (modes 1-4) for the lanes in
// `act` (BV_NONE: none); rule numbers index the block's result words.
template <int FM, bool CHAIN, typename D, typename T>
__device__ __forceinline__ uint32_t bv_first(const D &blk, const DescV &hb, T H, bool act,
					     const Pkt &k, const Parsed &p, const Fields &x, uint32_t cos = 0u)
{
	// header word 0: mode | next block of a chain << 8 (CHAIN kernels only)
	const uint32_t mode = FM >= 0 ? (uint32_t)FM : (CHAIN ? (hb(0) & 0xffu) : hb(0)), ncls = hb(1);
	uint32_t first = BV_NONE;
	if (mode == 2u) {
		// bitmap: AND of the classes' 32-bit rows and the alive row
		uint32_t acc = hb(4);
#pragma unroll
		for (uint32_t kc = 0; kc < BV_MAX_CLS; ++kc) {
			if (kc < ncls) {
				const auto cr = blk.vec(8u + BV_CLS_WORDS * kc);
				uint32_t key[4], nk = cr(1);
				const bool present = bv_key(cr, k, p, x, key);
				// a joint group's member (tree programs): the class's table
				// is the group's, keyed on (key, CoS) (record word 13)
				if constexpr (!CHAIN)
					joint_key(cr(13), cos, key, nk);
				const uint32_t val = bv_probe(H, key, act && present, nk, cr(9), cr(10), cr(11),
							      cr(12));
				acc &= val != 0u ? val : cr(2);
			}
		}
		first = acc != 0u ? (uint32_t)__builtin_ctz(acc) : BV_NONE;
	} else if (mode == 3u) {
		// wide bitmap (33..256 rules): AND of the classes' rows (in the hot
		// region, BV_WIDE_WORDS words each, zero past the rule count; a miss
		// takes the class's miss row) and the alive row; the lowest set bit
		// is the first holding rule
		// rows are split in halves: words 0-3 at the value, words 4-7
		// `half` words further (consecutive rows are then 16 B apart, so the
		// 16-lane groups of a 16-B LDS read spread over all 64 banks)
		const uint32_t ar = hb(4), half = hb(7);
		uint32_t acc[BV_WIDE_WORDS];
#pragma unroll
		for (uint32_t i = 0; i < BV_WIDE_WORDS; ++i)
			acc[i] = blk(ar + i);
#pragma unroll
		for (uint32_t kc = 0; kc < BV_MAX_CLS; ++kc) {
			if (kc < ncls) {
				const auto cr = blk.vec(8u + BV_CLS_WORDS * kc);
				uint32_t key[4];
				const bool present = bv_key(cr, k, p, x, key);
				const uint32_t val = bv_lookup(cr, H, key, act && present);
				const uint32_t ro = val != 0u ? val : cr(2);
				const u32x4 r0 = ld4(H, ro), r1 = ld4(H, ro + half);
#pragma unroll
				for (uint32_t i = 0; i < 4; ++i) {
					acc[i] &= r0[i];
					acc[4 + i] &= r1[i];
				}
			}
		}
#pragma unroll
		for (int i = (int)BV_WIDE_WORDS - 1; i >= 0; --i)
			first = acc[i] != 0u ? 32u * (uint32_t)i + (uint32_t)__builtin_ctz(acc[i]) : first;
	} else if (mode == 4u) {
		// single candidate per primary key: lookups only for the classes
		// rules are filed under (and longer-key classes, for their key
		// ids); each hit names the one rule filed under the packet's key,
		// whose record is checked against the packet's keys of every class
		// it constrains; the smallest holding candidate wins
		const uint32_t rec0 = hb(4), rw = hb(5), lk = hb(6), pm = hb(7);
		uint32_t cmpv[BV_MAX_CLS], cand[BV_MAX_CLS], prm = 0;
		first = hb(3);   // the first rule without a classified term
#pragma unroll
		for (uint32_t kc = 0; kc < BV_MAX_CLS; ++kc) {
			cmpv[kc] = 0u;
			cand[kc] = 0u;
			if (kc < ncls) {
				const auto cr = blk.vec(8u + BV_CLS_WORDS * kc);
				uint32_t key[4];
				const bool present = bv_key(cr, k, p, x, key);
				prm |= present ? 1u << kc : 0u;
				cmpv[kc] = key[0];
				if ((lk >> kc) & 1u) {
					const uint32_t v = bv_lookup(cr, H, key, act && present);
					cand[kc] = ((pm >> kc) & 1u) ? (v & 0xffffu) : 0u;
					cmpv[kc] = cr(1) == 1u ? key[0] : (v >> 16);
				}
			}
		}
		// the lane's candidates (1 + rule), compacted: a packet has at most
		// one per primary class, and usually far fewer than the block has
		// primary classes (config4: two of four), so two checks run always
		// and the others only if some lane needs them.  The smallest holding
		// candidate wins, so the order does not matter.
		uint32_t cl[BV_MAX_CLS];
#pragma unroll
		for (uint32_t i = 0; i < BV_MAX_CLS; ++i)
			cl[i] = 0u;
		uint32_t nc = 0;
#pragma unroll
		for (uint32_t kc = 0; kc < BV_MAX_CLS; ++kc) {
			if (kc < ncls && ((pm >> kc) & 1u)) {
				const uint32_t c1 = cand[kc];
#pragma unroll
				for (uint32_t i = 0; i <= kc; ++i)
					cl[i] = (c1 != 0u && nc == i) ? c1 : cl[i];
				nc += c1 != 0u ? 1u : 0u;
			}
		}
		const bool compact = rw == 4u && ncls > 3u;
		auto check = [&](uint32_t c1) {
			const bool tr = act && c1 != 0u && c1 - 1u < first;
			if (__ballot(tr) == 0ull)
				return;
			const uint32_t ra = rec0 + (tr ? c1 - 1u : 0u) * rw;
			const u32x4 q0 = ld4(H, ra);
			const uint32_t tm = q0[0];
			bool ok = (tm >> 31) == 0u;
			if (compact) {
				// compact record: the values of the <= 3 constrained
				// classes in class order; the packet's value of the
				// j-th one is picked by select (no per-class branches)
				uint32_t t = tm & 0xffu;
#pragma unroll
				for (uint32_t j = 0; j < 3; ++j) {
					const uint32_t c = (uint32_t)__builtin_ctz(t | 0x100u);
					t &= t - 1u;
					uint32_t pv = 0u;
#pragma unroll
					for (uint32_t i = 0; i < BV_MAX_CLS; ++i)
						pv = c == i ? cmpv[i] : pv;
					ok = ok && (c >= BV_MAX_CLS || (((prm >> c) & 1u) && pv == q0[1 + j]));
				}
			} else {
				u32x4 q1 = { 0u, 0u, 0u, 0u }, q2 = { 0u, 0u, 0u, 0u };
				if (rw > 4u)
					q1 = ld4(H, ra + 4u);
				if (rw > 8u)
					q2 = ld4(H, ra + 8u);
#pragma unroll
				for (uint32_t c2 = 0; c2 < BV_MAX_CLS; ++c2) {
					if (c2 < ncls) {
						const uint32_t w = c2 < 3u ? q0[1 + c2] : (c2 < 7u ? q1[c2 - 3u] : q2[0]);
						const bool need = (tm >> c2) & 1u;
						ok = ok && (!need || (((prm >> c2) & 1u) && cmpv[c2] == w));
					}
				}
			}
			first = (tr && ok) ? c1 - 1u : first;
		};
		check(cl[0]);
		check(cl[1]);
#pragma unroll
		for (uint32_t i = 2; i < BV_MAX_CLS; ++i)
			if (__ballot(cl[i] != 0u) != 0ull)
				check(cl[i]);
	} else {
		// candidate: key id per class, then the candidates' records
		const uint32_t rec0 = hb(4), rw = hb(5);
		uint32_t v[BV_MAX_CLS], lb[BV_MAX_CLS];
#pragma unroll
		for (uint32_t kc = 0; kc < BV_MAX_CLS; ++kc) {
			v[kc] = 0u;
			lb[kc] = 0u;
			if (kc < ncls) {
				const auto cr = blk.vec(8u + BV_CLS_WORDS * kc);
				uint32_t key[4];
				const bool present = bv_key(cr, k, p, x, key);
				v[kc] = bv_lookup(cr, H, key, act && present);
				lb[kc] = cr(13);
			}
		}
		first = hb(3);   // the first rule without a classified term
#pragma unroll
		for (uint32_t kc = 0; kc < BV_MAX_CLS; ++kc) {
			if (kc < ncls) {
				// value = key id | list length << 12 | list offset << 20
				uint32_t j = 0, n = (v[kc] >> 12) & 0xffu;
				const uint32_t lo = lb[kc] + (v[kc] >> 20);
				for (;;) {
					const bool more = act && j < n;
					if (__ballot(more) == 0ull)
						break;
					if (more) {
						const uint32_t r = H[lo + j];
						bool ok = r < first;
						if (ok) {
							const uint32_t rec = rec0 + r * rw;
							const uint32_t m = H[rec];
							ok = (m >> 31) == 0u;
#pragma unroll
							for (uint32_t c = 0; c < BV_MAX_CLS; c += 2) {
								if (c < ncls && ((m >> c) & 3u)) {
									const uint32_t w = H[rec + 1u + (c >> 1)];
									ok = ok && (!((m >> c) & 1u) ||
										    (v[c] & 0xfffu) == (w & 0xffffu));
									ok = ok && (!((m >> (c + 1)) & 1u) ||
										    (v[c + 1] & 0xfffu) == (w >> 16));
								}
							}
						}
						first = ok ? r : first;
						// lists are in scan order: the first candidate that
						// holds, or reaches `first`, ends this list
						n = (ok || r >= first) ? 0u : n;
						++j;
					}
				}
			}
		}
	}
	return first;
}

template <typename D> struct SpecOf {
	typedef void type;
};
template <typename S> struct SpecOf<DescC<S>> {
	typedef S type;
};

// First holding rule over a compile-time chain (FM_CHAIN): block I and on,
// each with its engine compiled in; the smallest over the chain.
template <typename S, uint32_t I = 0, typename T>
__device__ __forceinline__ uint32_t chain_first(T H, cword_t hc, bool act, const Pkt &k,
						const Parsed &p, const Fields &x)
{
	if constexpr (I >= S::nblk) {
		return BV_NONE;
	} else {
		const DescC<S> b{ S::boff[I], hc };
		const uint32_t f = bv_first<(int)S::bmode[I], false>(b, b.hdr(), H, act, k, p, x);
		return min(f, chain_first<S, I + 1>(H, hc, act, k, p, x));
	}
}

// Classification block evaluation of one CoS for the lanes in `act`
// (see build_bv for the two modes).  `blk` reads the CoS's block (wave-
// uniform or per lane); H is the hot region the block's offsets index.  On
// return, lanes of `act` with a matching rule have hit = 1 and the rule's
// destination CoS / mark / leaf bit in nxt / nmark / nleaf.
// FM >= 0: the block's engine is known at compile time (the flat-program
// kernels); -1: read from the block.
// A CoS whose rules need more than BV_MAX_CLS key classes has a chain of
// blocks (header word 0 = mode | next block << 8), each over a group of its
// rules with at most BV_MAX_CLS classes and the CoS's rule numbering; the
// first holding rule is the smallest over the chain.  Chained CoS are
// evaluated wave-uniformly only (their CoS entry's block word has bit 31
// set), and only by kernels built with CHAIN (the generic kernels of
// programs without CoS trees): the chain loop's live state pushed the tree
// kernels (DIV) into VGPR spills (config5 46.7 -> 51.2 us, 28 B scratch per
// lane), so the host builds no chains for tree programs -- their CoS with
// more key classes than a block holds take the linear scan.
template <int FM = -1, bool CHAIN = false, typename D, typename T>
__device__ __forceinline__ void bv_eval(const D &blk, T H, bool act, const Pkt &k, const Parsed &p,
					const Fields &x, uint32_t &hit, uint32_t &nxt, uint32_t &nmark,
					uint32_t &nleaf, uint32_t cos = 0u)
{
	const auto hb = blk.hdr();   // the block header (words 0-7)
	const uint32_t mode = FM >= 0 ? (uint32_t)FM : (CHAIN ? (hb(0) & 0xffu) : hb(0)), res = hb(2);
	if (mode == 0u) {
		// direct: one class, the slot holds the result word of the first
		// live rule of its key (BV_EMPTY: none); a miss takes the block's
		// "no term" rule (0: none).  The class record is shared by the
		// direct blocks with the same class (header word 2); the header
		// holds the miss word and the table (bucket count, offset, m1, m2)
		uint32_t key[4], nk;
		const bool present = split_key(blk, hb(2), act, k, p, x, key, nk);
		// a joint group's member: its table is the group's, keyed on (key, CoS)
		joint_key(hb(1), cos, key, nk);
		const uint32_t val = bv_probe(H, key, act && present, nk, hb(4), hb(5), hb(6), hb(7));
		const uint32_t rw = val != 0u ? (val == BV_EMPTY ? 0u : val) : hb(3);
		const bool h = act && rw != 0u;
		nxt = h ? (rw & 0xffu) : nxt;
		nleaf = h ? ((rw >> 8) & 1u) : nleaf;
		nmark = h ? (rw >> 16) : nmark;
		hit = h ? 1u : hit;
		return;
	}
	uint32_t first;
	if constexpr (FM == FM_CHAIN) {
		// a chain compiled into a specialised kernel
		first = chain_first<typename SpecOf<D>::type>(H, blk.h, act, k, p, x);
	} else if constexpr (CHAIN && FM < 0 && std::is_same<D, DescU>::value) {
		// a chain (wave-uniform blocks only): one copy of the engines,
		// looping over the blocks
		first = BV_NONE;
		DescU cur = blk;
		DescV ch = hb;
		for (;;) {
			first = min(first, bv_first<-1, true>(cur, ch, H, act, k, p, x));
			const uint32_t nx = ch(0) >> 8;
			if (nx == 0u)
				break;
			cur = DescU{ blk.h + nx, blk.h };
			ch = cur.hdr();
		}
	} else {
		first = bv_first<FM, CHAIN>(blk, hb, H, act, k, p, x, cos);
	}
	const bool h = act && first != BV_NONE;
	const uint32_t rw2 = H[res + (h ? first : 0u)];
	nxt = h ? (rw2 & 0xffu) : nxt;
	nleaf = h ? ((rw2 >> 8) & 1u) : nleaf;
	nmark = h ? (rw2 >> 16) : nmark;
	hit = h ? 1u : hit;
}

// ---------------------------------------------------- tree-plan kernels
// A program-specialised kernel for a CoS tree (tree programs whose levels are
// joint groups, e.g. config 5: default CoS -> 16 VLAN CoS -> 128 prefix CoS
// -> leaves) carries, besides the default CoS's block (round 1, DescC), the
// tree's plan: S::nplan rounds, round i evaluating the lanes that sit on a
// CoS of joint group S::gid[i] with that group's info words (S::ginfo[i], the
// layout of the group info in the hot region) and class records
// (S::grec[i][c]) compiled in -- no scalar loads and no decoding of group or
// class words per tile.  Membership is tested per lane (the CoS entry's
// group bits), so a lane is advanced only by the round of the group it sits
// on: any lane off the plan (or deeper than it) stays pending and is finished
// by the reference's scan (linear_scan) per CoS after the plan.  The host
// builds a plan only when it covers every non-leaf destination of the tree.
template <typename...> struct mi_void { typedef void type; };
template <typename S, typename = void> struct plan_n {
	static constexpr uint32_t v = 0;
};
template <typename S> struct plan_n<S, typename mi_void<decltype(S::nplan)>::type> {
	static constexpr uint32_t v = S::nplan;
};

template <uint32_t V> struct mi_uconst {
	static constexpr uint32_t value = V;
};
// f(mi_uconst<0>{}) .. f(mi_uconst<N - 1>{}), unrolled at compile time
template <uint32_t N, uint32_t I = 0, typename F>
__device__ __forceinline__ void static_for(F &f)
{
	if constexpr (I < N) {
		f(mi_uconst<I>{});
		static_for<N, I + 1>(f);
	}
}

// One plan round's joint-group evaluation for the lanes in `bvl` (CoS slot
// `cs`): the generic kernel's joint path (mi_cls_kernel) with the group's
// words as compile-time constants.
// (a plain function, not a lambda: clang's constant evaluator crashed on the
// implicitly constexpr lambda's vector element stores)
template <typename S, uint32_t I, uint32_t C>
__device__ __forceinline__ DescV plan_rec()
{
	DescV d;
#pragma unroll
	for (uint32_t i = 0; i < 16; ++i)
		d.v[i] = S::grec[I][C][i];
	return d;
}

template <typename S, uint32_t I, typename T>
__device__ __forceinline__ void plan_eval(T H, bool bvl, uint32_t cs, const Pkt &k, const Parsed &p,
					  const Fields &x, uint32_t &hit, uint32_t &nxt, uint32_t &nmark,
					  uint32_t &nleaf)
{
	constexpr const uint32_t *ji = S::ginfo[I];
	uint32_t rw;
	bool hv;
	if constexpr (ji[0] == 0u) {
		// direct: the first live rule's result word, or the CoS's miss word
		const DescV cr = plan_rec<S, I, 0>();
		uint32_t key[4], nk = cr(1);
		const bool present = bv_key(cr, k, p, x, key);
		joint_key(ji[14], cs, key, nk);
		const uint32_t val = bv_probe(H, key, bvl && present, nk, ji[9], ji[10], ji[11], ji[12]);
		const uint32_t miss = H[ji[13] + cs];
		rw = val != 0u ? (val == BV_EMPTY ? 0u : val) : miss;
		hv = rw != 0u;
	} else {
		// bitmap: AND of the classes' rule rows and the CoS's alive row
		uint32_t acc = H[ji[2] + cs];
		auto cls = [&](auto ic) {
			constexpr uint32_t kc = decltype(ic)::value;
			if constexpr (kc < ji[1]) {
				constexpr const uint32_t *ci = ji + 8u + 8u * kc;
				const DescV cr = plan_rec<S, I, kc>();
				uint32_t key[4], nk = cr(1);
				const bool present = bv_key(cr, k, p, x, key);
				joint_key(ci[6], cs, key, nk);
				const uint32_t val = bv_probe(H, key, bvl && present, nk, ci[1], ci[2], ci[3], ci[4]);
				acc &= val != 0u ? val : H[ci[5] + cs];
			}
		};
		static_for<BV_MAX_CLS>(cls);
		const uint32_t res = H[ji[3] + cs];
		rw = H[res + (acc != 0u ? (uint32_t)__builtin_ctz(acc) : 0u)];
		hv = acc != 0u;
	}
	const bool h = bvl && hv;
	nxt = h ? (rw & 0xffu) : nxt;
	nleaf = h ? ((rw >> 8) & 1u) : nleaf;
	nmark = h ? (rw >> 16) : nmark;
	hit = h ? 1u : hit;
}

// Linear scan of one wave-uniform CoS's rule records for the lanes in
// `grp` (verify_pmr over cos->pmr[] in order, first match wins).
__device__ __forceinline__ void linear_scan(cword_t prog, uint32_t rec0, uint32_t nr, bool grp,
					    const Pkt &k, const Parsed &p, const Fields &x,
					    uint32_t &done, uint32_t &nxt, uint32_t &nmark)
{
	for (uint32_t r = 0; r < nr; ++r) {
		const bool cand = grp && done == 0u;
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
		nxt = ok ? (w1 & 0xffu) : nxt;
		nmark = ok ? (w0 >> 16) : nmark;
		done = ok ? 1u : done;
	}
}

// ------------------------------------------------------------------ kernel
struct KArgs {
	const uint8_t *pkts;
	const uint32_t *off;
	const uint16_t *len;
	uint32_t n;
	const uint32_t *dev;         // device rule program (constant address space)
	mi_cls_result_t *out;
	unsigned long long *stats;   // MAX_STATS_COS counters, or NULL
	uint32_t stats_mask[8];
	uint32_t opt;                // pktin options (OPT_*), 0: none
	// window hint across launches of a context: a wave of block 0 whose
	// frames needed bytes 64.. stores this launch's sequence number `seq` in
	// *hint; the next launch (seq + 1) starts its predictor from it.  Only a
	// performance hint -- results never depend on it.
	uint32_t *hint;
	uint32_t seq;
};

__device__ __forceinline__ bool stats_bit(const KArgs &a, uint32_t c)
{
	return c < MAX_STATS_COS && ((a.stats_mask[c >> 5] >> (c & 31u)) & 1u);
}

static_assert(NPIECE == 6, "WIN is 96");
#define NB (NPIECE - 4)         // upper pieces (phase B)

// Issue the loads of a tile's header windows (64 packets, per-lane
// descriptors off/len).  The lanes cooperate so that each load instruction
// covers whole packets' headers: in phase A lane l loads piece l&3 (bytes
// 16(l&3) ..) of packet 16r + (l>>2), r = 0..3 -- for back-to-back frames an
// instruction reads 16 x 64 contiguous bytes instead of 64 scattered pieces,
// a quarter of the cache-line lookups.  Phase B (pieces 4..) is issued only
// when some frame of the tile is longer than 64 B (returns true).  Pieces
// wholly past a frame get an out-of-range offset and read as zero.
__device__ __forceinline__ bool load_window(__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t len,
					    uint32_t lane, u32x4 d[NPIECE], bool want_hi, uint32_t &win)
{
	const uint32_t q = lane & 3u, pp = lane >> 2;
#pragma unroll
	for (uint32_t r = 0; r < 4; ++r) {
		const int src = (int)((16u * r + pp) << 2);
		const uint32_t o = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)off);
		const uint32_t L = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)len);
		const uint32_t vo = 16u * q < L ? o + 16u * q : OOB_OFF;
		d[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 0, LOAD_AUX);
	}
	// phase B only when some frame is longer than 64 B and the window
	// predictor wants bytes 64.. (want_hi); otherwise a tile with long frames
	// stages 64 B per frame and reads the rare bytes past them from HBM
	// (staging only bytes 64..79, one 16-B load per frame -- enough for a
	// QinQ IPv6 frame's ports -- measured slower and fetched more on config 5:
	// 48.0 -> 54.2 us, 4.2 -> 4.7 KiB per tile)
	const bool any_long = __ballot(len > 64u) != 0ull;
	const bool hi = any_long && want_hi;
	win = (any_long && !hi) ? 64u : (uint32_t)WIN;
	if (hi) {
		const uint32_t qb = lane % NB, pb = lane / NB;
#pragma unroll
		for (uint32_t r = 0; r < NB; ++r) {
			const int src = (int)(((64u / NB) * r + pb) << 2);
			const uint32_t o = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)off);
			const uint32_t L = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)len);
			const uint32_t c = 16u * (4u + qb);
			const uint32_t vo = c < L ? o + c : OOB_OFF;
			d[4 + r] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 0, LOAD_AUX);
		}
	}
	return hi;
}

// Write a tile's loaded pieces into the transposed window: lane l holds
// dwords 4q..4q+3 of packet p, which go to rows 4q..4q+3, column p.  With the
// 66-dword row stride the 64 lanes of one ds_write hit distinct banks
// (bank = 8q + 2i + p mod 32 within each 32-lane half).  Rows 16.. are
// rewritten only when this tile has long frames, or zeroed once after a tile
// that had them (hi_rows tracks whether they hold data).
__device__ __forceinline__ void store_window(uint32_t *W, uint32_t lane, const u32x4 d[NPIECE],
					     bool hi, bool &hi_rows)
{
	const uint32_t q = lane & 3u, pp = lane >> 2;
#pragma unroll
	for (uint32_t r = 0; r < 4; ++r) {
		const uint32_t base = 4u * q * RS + 16u * r + pp;
#pragma unroll
		for (uint32_t i = 0; i < 4; ++i)
			W[base + i * RS] = d[r][i];
	}
	if (hi) {
		const uint32_t qb = lane % NB, pb = lane / NB;
#pragma unroll
		for (uint32_t r = 0; r < NB; ++r) {
			const uint32_t base = 4u * (4u + qb) * RS + (64u / NB) * r + pb;
#pragma unroll
			for (uint32_t i = 0; i < 4; ++i)
				W[base + i * RS] = d[4 + r][i];
		}
	} else if (hi_rows) {
#pragma unroll
		for (uint32_t row = 16; row < WIN / 4; ++row)
			W[row * RS + lane] = 0u;
	}
	hi_rows = hi;
}

// Zero the bytes of the last loaded piece that lie past the frame
// (frame_len .. end of its 16-B piece; loaded pieces wholly past the frame
// read as zero already): bytes b..3 of the partial dword with one byte store
// (b odd) and one 16-bit store (b <= 2) -- stores that are not needed go to
// the lane's pad dword, which is zero anyway -- then the next three whole
// dwords (clamped to the zero row WIN/4): rows past the piece are zero
// (pieces past the frame, or the zero row).
__device__ __forceinline__ void zero_tail(uint32_t *W, uint32_t lane, uint32_t len)
{
	const uint32_t pad = (WIN / 4) * RS + lane;
	const uint32_t dw = len >> 2, b = len & 3u;
	const bool part = b != 0u && len < WIN;
	uint8_t *W8 = (uint8_t *)W;
	const uint32_t pb = (dw * RS + lane) * 4u;
	W8[(part && (b & 1u)) ? pb + b : pad * 4u + 1u] = 0;
	*(uint16_t *)(W8 + ((part && b <= 2u) ? pb + 2u : pad * 4u + 2u)) = 0;
	const uint32_t r0 = (len + 3u) >> 2;
	W[min(r0, (uint32_t)(WIN / 4)) * RS + lane] = 0u;
	W[min(r0 + 1u, (uint32_t)(WIN / 4)) * RS + lane] = 0u;
	W[min(r0 + 2u, (uint32_t)(WIN / 4)) * RS + lane] = 0u;
}

// Packet descriptors are read once (nontemporal loads measured within
// noise: plain loads).
template <typename T> __device__ __forceinline__ uint32_t ld_desc(const T *p)
{
	return (uint32_t)*p;
}

// One 16-B result record (a coalesced dwordx4 store per lane), nontemporal:
// the records are not read again by this kernel, and streaming them out
// instead of leaving 16 MB of dirty lines in L2 for the end-of-kernel
// release cut 4-6 % per launch on every config (cached stores measured).
__device__ __forceinline__ void store_rec(mi_cls_result_t *dst, uint4 r)
{
	u32x4 v = { r.x, r.y, r.z, r.w };
	__builtin_nontemporal_store(v, (u32x4 *)dst);
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

// DIV = the program has rules behind rules (a CoS tree), so lanes of a wave
// can sit on different CoS: such rounds evaluate every lane's own bit-vector
// block at once instead of one CoS per round.
// LT = the hot region is copied into LDS at block start (it fits the
// budget): every per-lane table lookup is then an LDS read and the compute
// phase issues no vector memory loads, so nothing it waits for sits behind
// the next tile's prefetch in the (in-order) vmcnt queue.  !LT reads the hot
// region from HBM (large rule sets).
extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];

// NW = waves per block: 4 (each block copies the hot region for itself), or
// 16 = one block per CU whose 16 waves share one LDS copy of a larger hot
// region.  Either way 4 waves per SIMD (the VGPR budget).
// Waves per SIMD a block shape runs at: 4-wave blocks run 4 blocks per CU,
// the one-block-per-CU shapes NW / 4 (8 and 12 waves give each wave a
// bigger register budget and leave LDS for a larger hot region).
constexpr int waves_per_eu(int nw)
{
	return nw == 4 ? MIN_WAVES_PER_EU : nw / 4;
}

// FM >= 0: flat-program kernel -- every pending lane is decided in round 1
// on the default CoS, whose block uses engine FM (all its rules lead to CoS
// without rules), and no pktin option is set: no descent loop, no linear
// scan, no checksum path in the code (fewer registers, straight-line
// engine).  The host picks it only for such programs (mi_cls_classify).
// CK: pktin-option kernel (mi_cls_kc.hip), launched whenever a pktin
// checksum / drop option is set; the other kernels require opt == 0 and carry
// no option code (the checksum path's registers would otherwise be
// allocated, and spilled, in every kernel).
// SPEC (void: none): a program-specialised kernel -- the default CoS's block
// (evaluated in the first descent round) is the compile-time DescC<SPEC>.
template <bool LT, bool DIV, int NW, int FM = -1, bool CK = false, typename SPEC = void>
__global__ __launch_bounds__(NW * WAVE, waves_per_eu(NW)) void mi_cls_kernel(KArgs a)
{
	__shared__ uint32_t s_win[NW * RS * WROWS];
	__shared__ uint32_t s_cnt[MAX_STATS_COS];
	__shared__ uint32_t s_l4[256];
	// CRC-32C slicing tables and piece shifts (pktin options)
	__shared__ uint32_t s_crc[CK ? CRC_WORDS : 1];

	const uint32_t lane = threadIdx.x & (WAVE - 1);
	const uint32_t wave = threadIdx.x >> 6;
	uint32_t *W = s_win + wave * RS * WROWS;

	const cword_t dev = (cword_t)a.dev;
	const int32_t def_cos = (int32_t)dev[DH_DEFAULT];
	const int32_t err_cos = (int32_t)dev[DH_ERROR];
	const uint32_t def_valid = dev[DH_DEFAULT_VALID];
	const uint32_t max_hops = dev[DH_MAX_HOPS];
	const uint32_t hot_off = dev[DH_HOT_OFF];
	const cword_t hc = dev + hot_off;                 // hot region, scalar reads
	const cword_t prog = dev + dev[DH_PROG_OFF];
	// the default CoS's words (the first descent round always evaluates it)
	const cword_t dce = hc + COS_WORDS * (uint32_t)max(def_cos, 0);
	const uint32_t d_nr = def_cos >= 0 ? dce[C_NR] : 0u;
	// bit 31: a chain of blocks (never set in tree programs)
	const uint32_t d_bv = DIV ? dce[C_BV] & C_BV_OFF : dce[C_BV] & 0x7fffffffu, d_rec0 = dce[C_REC0];
	const uint32_t j_off = DIV ? dev[DH_JOINT] : 0u;   // joint groups' directory
	const bool stats_on = a.stats != nullptr;
	typedef typename std::conditional<LT, lword_t, gword_t>::type hot_t;
	hot_t H;
	// first descriptors before the hot-region copy: their latency overlaps it
	const uint32_t nt = (a.n + WAVE - 1) / WAVE;
	const uint32_t tstride = gridDim.x * NW;
	uint32_t tile = blockIdx.x * NW + wave;
	uint32_t d_off = 0, d_len = 0, n_off = 0, n_len = 0;
	{
		const uint32_t p0 = tile * WAVE + lane, p1 = (tile + tstride) * WAVE + lane;
		if (tile < nt && p0 < a.n) {
			d_off = ld_desc(a.off + p0);
			d_len = ld_desc(a.len + p0);
		}
		if (tile + tstride < nt && p1 < a.n) {
			n_off = ld_desc(a.off + p1);
			n_len = ld_desc(a.len + p1);
		}
	}
	// Software pipeline over this wave's tiles (64 packets each): while tile
	// t is parsed and classified, tile t+1's header windows are in flight
	// into registers (load_window) and tile t+2's descriptors are being
	// fetched.  Tile t's result records are stored at the top of iteration
	// t+1, before tile t+2's loads are issued, so waiting for window data
	// never waits behind a younger store (vmcnt retires in order), and the
	// records are not held in registers through parse and classify.
	const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
		(void *)a.pkts, (short)0, (int)OOB_OFF, 0x00020000);
	u32x4 d[NPIECE];
	bool d_hi, hi_rows = true;
	// window predictor: stage bytes 64..WIN-1 of long frames only while the
	// frames of the last parsed tile needed them (the fields of its rule
	// program and its parse reach past byte 64); the first tiles stage them
	bool want_hi = a.hint == nullptr || *(const uint32_t *)a.hint + 1u == a.seq;
	// PLH (tree kernels without pktin options): bytes 64..WIN-1 are staged
	// per lane, for the frames whose parse or program fields reach past byte
	// 64 (a QinQ IPv6 frame's ports, an IPv6 TCP data offset), after the
	// parse, instead of for every long frame of a tile the predictor marks:
	// on config 5 those 96-B windows cost 1.33x the algorithmic HBM bytes.
	// Their L4 checks (parse_fast: dfr) and the rounds after the first wait
	// for them, so the first descent round runs while they are in flight.
	constexpr bool PLH = DIV && !CK;
	if constexpr (PLH)
		want_hi = false;
	bool saw_hi = false;
	uint32_t d_win = WIN, my_win = WIN;
	const uint32_t p_l3end = dev[DH_L3END], p_l4end = dev[DH_L4END], p_frend = dev[DH_FREND];
	// the first tile's windows are in flight during the block setup below
	if (tile < nt)
		d_hi = load_window(rs, d_off, d_len, lane, d, want_hi, d_win);
	if constexpr (LT) {
		// hot region -> LDS in 16-B pieces (the device program and the
		// dynamic LDS size are padded to 16 B)
		const uint32_t hq = (dev[DH_HOT_WORDS] + 3u) >> 2;
		typedef const __attribute__((address_space(1))) u32x4 *gvec_t;
		const gvec_t src = (gvec_t)(a.dev + hot_off);
		u32x4 *dst = (u32x4 *)s_dyn;
		for (uint32_t i = threadIdx.x; i < hq; i += NW * WAVE)
			dst[i] = src[i];
		H = (lword_t)s_dyn;
	} else {
		H = (gword_t)(a.dev + hot_off);
	}

	if (stats_on) {
		for (uint32_t i = threadIdx.x; i < MAX_STATS_COS; i += NW * WAVE)
			s_cnt[i] = 0;
	}
	for (uint32_t i = threadIdx.x; i < 256u; i += NW * WAVE)
		s_l4[i] = c_l4tab.v[i];
	if constexpr (CK) {
		// Crc32cTab's words in order (CRC_* offsets)
		const uint32_t *cw = reinterpret_cast<const uint32_t *>(&c_crc32c);
		for (uint32_t i = threadIdx.x; i < CRC_WORDS; i += NW * WAVE)
			s_crc[i] = cw[i];
	}
	for (uint32_t r = WIN / 4; r < WROWS; ++r)
		W[r * RS + lane] = 0u;   // pad / zero rows: always zero
	__syncthreads();

	uint4 prev_rec = make_uint4(0, 0, 0, 0);
	uint32_t prev_pi = 0;
	bool prev_valid = false;
	for (; tile < nt; tile += tstride) {
		const uint32_t pi = tile * WAVE + lane;
		const bool valid = pi < a.n;
		const uint32_t my_off = d_off, my_len = d_len;
		my_win = d_win;

		wave_lds_sync();   // previous tile's window reads are done
		store_window(W, lane, d, d_hi, hi_rows);
		zero_tail(W, lane, my_len);   // same wave: LDS stores stay in order
		// previous tile's records: issued before this tile's prefetch, so the
		// next wait for window data never waits behind a younger store
		if (prev_valid)
			store_rec(a.out + prev_pi, prev_rec);
		prev_valid = false;

		// advance the pipeline: data of tile+stride, descriptors of tile+2*stride
		// (PLH: after the parse, behind this tile's far loads in the vmcnt
		// queue, so waiting for those never waits for the next tile's window)
		auto prefetch = [&]() {
#ifdef DIAG_NOSTAGE
			// diagnostic: every tile re-parses and re-classifies this wave's
			// first tile (no window loads after it): the compute-only floor
			if (false) {
#else
			{
#endif
				d_off = n_off;
				d_len = n_len;
				const uint32_t t2 = tile + 2u * tstride, p2 = t2 * WAVE + lane;
				n_off = 0;
				n_len = 0;
				if (t2 < nt && p2 < a.n) {
					n_off = ld_desc(a.off + p2);
					n_len = ld_desc(a.len + p2);
				}
				// no loads for a tile past the end (its registers would be
				// waited for before reuse after the loop)
				if (tile + tstride < nt)
					d_hi = load_window(rs, d_off, d_len, lane, d, want_hi, d_win);
			}
		};
		if constexpr (!PLH)
			prefetch();
		wave_lds_sync();
#ifdef DIAG_STAGEONLY
		if constexpr (PLH)
			prefetch();
		if (valid) {
			uint4 rec;
			rec.x = W[3 * RS + lane] ^ W[8 * RS + lane];
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
		k.win = PLH ? 64u : my_win;

		Parsed p;
		bool dfr = false;
		if constexpr (!CK) {
			bool slow;
			p = parse_fast(k, s_l4, slow, PLH ? (uint32_t)WIN : 0u, dfr);
			if (__ballot(slow) != 0ull) {
				if (slow)
					p = parse_packet(k, 0u);
			}
		} else {
			// pktin options.  The fast parse stands for every lane whose
			// result the options do not change; parse_packet(opt) re-parses
			// the others: lanes with a parse error (drop options), a bad IPv4
			// header checksum, or a zero UDP checksum (the parse_udp rule).
			// A good IPv4 header checksum only adds l3_chksum_done.  Then
			// the L4 checksums (whole frames from HBM, the wave cooperating).
			bool slow;
			p = parse_fast(k, s_l4, slow, 0u, dfr);
			p.udp_zero = 0;
			slow = slow || p.err != 0u;
			if (a.opt & OPT_IPV4_CK) {
				// odp_parse.c:134-141: sum over the ihl * 4 header bytes
				const bool v4 = !slow && (p.flags & F_IPV4) != 0u;
				if (__ballot(v4) != 0ull) {
					if (v4) {
						const uint32_t ihl = rb(k, p.l3) & 0xfu;
						uint64_t sum = 0;
						for (uint32_t i = 0; i < ihl; ++i)
							sum += r32(k, p.l3 + 4u * i);
						if (ck_finalize(sum) != 0xffffu)
							slow = true;
						else
							p.flags |= F_L3CK_DONE;
					}
				}
			}
			if (a.opt & OPT_UDP_CK) {
				const bool u = !slow && (p.flags & F_UDP) != 0u && !(p.flags & F_IPFRAG) &&
					       p.ret == 0;
				if (__ballot(u) != 0ull) {
					if (u && r16(k, p.l4 + 6u) == 0u)
						slow = true;
				}
			}
			if (__ballot(slow) != 0ull) {
				if (slow)
					p = parse_packet(k, a.opt);
			}
			if (a.opt & OPT_L4_CK)
				l4_chksum(k, p, a.opt, rs, my_off, lane, valid, s_crc);
		}
		Fields x = fields_of(k, p);
		// the bytes past byte 64 this lane uses: the parse's L3 / L4 headers
		// and the program's fields (conservative: gates ignored)
		uint32_t need;
		{
			const uint32_t l4h = (p.flags & F_TCP) ? 13u : ((p.flags & F_UDP) ? 6u : 0u);
			need = p_frend;
			need = max(need, p.l3 != 0xFFFFu ? p.l3 + max(p_l3end, (p.flags & F_IPV6) ? 40u : 20u) : 0u);
			need = max(need, p.l4 != 0xFFFFu ? p.l4 + max(p_l4end, l4h) : 0u);
		}
		u32x4 hv0 = { 0u, 0u, 0u, 0u }, hv1 = { 0u, 0u, 0u, 0u };
		bool hneed = false, any_h = false;
		if constexpr (PLH) {
			// this tile's far pieces (bytes 64..95) for the lanes that need
			// them, then the next tile's loads
			hneed = valid && my_len > 64u && (need > 64u || dfr);
			any_h = __ballot(hneed) != 0ull;
			if (any_h) {
				hv0 = __builtin_amdgcn_raw_buffer_load_b128(rs, hneed ? my_off + 64u : OOB_OFF, 0,
									     LOAD_AUX);
				hv1 = __builtin_amdgcn_raw_buffer_load_b128(
					rs, hneed && my_len > 80u ? my_off + 80u : OOB_OFF, 0, LOAD_AUX);
			}
			prefetch();
		} else {
			// window predictor: the next tile stages bytes 64.. when this
			// one's frames needed them
			// (reading a TCP data offset past a 64-B window from HBM instead
			// of staging 96-B windows measured 3-6 % slower on configs 3-5)
			want_hi = __ballot(valid && my_len > 64u && need > 64u) != 0ull;
			saw_hi = saw_hi || want_hi;
		}
		// PLH: the far pieces into the window (rows 16..), the lanes' windows
		// widened, and the deferred L4 checks (parse_fast: dfr) on them
		auto far_in = [&]() {
			if constexpr (PLH) {
				if (any_h) {
					if (hneed) {
#pragma unroll
						for (uint32_t i = 0; i < 4; ++i) {
							W[(16u + i) * RS + lane] = hv0[i];
							W[(20u + i) * RS + lane] = hv1[i];
						}
						zero_tail(W, lane, my_len);
					}
					wave_lds_sync();
					k.win = hneed ? (uint32_t)WIN : 64u;
					x.k.win = k.win;
					if (__ballot(dfr) != 0ull) {
						uint32_t e4, f4, nd;
						const bool tcp = dfr && (p.flags & F_TCP) != 0u && p.l4 + 20u <= my_len;
						const bool udp = dfr && (p.flags & F_UDP) != 0u && p.l4 + 8u <= my_len;
						l4_bytes(k, p.l4, tcp, udp, e4, f4, nd);
						if (dfr) {
							p.err |= e4;
							p.flags |= f4;
							p.ret = p.ret < 0 ? p.ret : (p.err != 0u ? 1 : 0);
							x.f = p.flags;
						}
					}
				}
			}
		};
		// per-hop CoS counters count every hop a lane takes: no descent
		// before the deferred checks then
		if (stats_on)
			far_in();
#ifdef DIAG_PARSEONLY
		if (valid) {
			uint4 rec;
			rec.x = p.flags;
			rec.y = p.err;
			rec.z = x.f ^ x.l4;
			rec.w = (p.l3 & 0xffffu) | ((p.l4 & 0xffffu) << 16);
			*(uint4 *)(a.out + pi) = rec;
		}
		continue;
#endif

		// ---- select the starting CoS (cls_select_cos, odp_classification.c:1694-1726)
		// Per-lane state is kept in integers updated by selects: bools live
		// across the descent loop would become lane masks merged at every
		// join (and spill SGPRs).
		bool ok_parse = valid && p.ret >= 0;
		bool perr = p.err != 0u;
		int32_t cur = perr ? err_cos : def_cos;
		uint32_t pend = (ok_parse && !perr && def_cos >= 0 && def_valid) ? 1u : 0u;

		// ---- CoS descent (match_pmr_cos, :1624-1667).  Each round moves
		// pending lanes one hop: the CoS of the first pending lane is
		// evaluated by every lane sitting on it (bit-vector or linear engine,
		// the CoS's words in SGPRs); in tree programs (DIV) lanes on other
		// bit-vector CoS evaluate their own blocks in the same round.
		uint32_t hops = 0, mark = 0, matched = 0, loop = 0;
		// one hop of the lanes in `proc` whose evaluation gave hit / nxt / ..
		auto advance = [&](uint32_t proc, uint32_t hit, uint32_t nxt, uint32_t nmark,
				   uint32_t nleaf) {
			const uint32_t take = proc & hit;
			cur = take ? (int32_t)nxt : cur;
			mark = take ? nmark : mark;
			matched |= take;
			hops += take;
			const uint32_t lp = (take != 0u && hops > max_hops) ? 1u : 0u;
			loop |= lp;
			// still pending: a rule matched, under the hop limit, and the
			// destination CoS has rules
			pend = proc ? ((take != 0u && lp == 0u && nleaf == 0u) ? 1u : 0u) : pend;
			if (stats_on) {
				if (take != 0u && stats_bit(a, nxt))
					atomicAdd(&s_cnt[nxt], 1u);
			}
		};
		// round 1: every pending lane sits on the default CoS, whose words
		// are loop-invariant (d_nr / d_bv / d_rec0, loaded once per wave)
		if (__ballot(pend != 0u) != 0ull) {
			uint32_t hit = 0, nleaf = 0, nxt = 0, nmark = 0;
			const bool g = pend != 0u;
			if constexpr (!std::is_void<SPEC>::value) {
				// the default CoS's block is compiled in (it has one: the
				// host specialises only such programs)
				bv_eval<FM>(DescC<SPEC>{ 0u, hc }, H, g, k, p, x, hit, nxt, nmark, nleaf,
					    (uint32_t)max(def_cos, 0));
			} else if constexpr (FM >= 0) {
				bv_eval<FM>(DescU{ hc + d_bv, hc }, H, g, k, p, x, hit, nxt, nmark, nleaf);
			} else {
				if (d_bv != 0u && d_nr != 0u)
					bv_eval<-1, !DIV>(DescU{ hc + d_bv, hc }, H, g, k, p, x, hit, nxt, nmark,
							  nleaf, (uint32_t)def_cos);
				else
					linear_scan(prog, d_rec0, d_nr, g, k, p, x, hit, nxt, nmark);
			}
			advance(g ? 1u : 0u, hit, nxt, nmark, nleaf);
		}
		if constexpr (PLH) {
			if (!stats_on) {
				far_in();
				// a deferred check found an L4 error: the lane goes to the
				// error CoS (cls_select_cos) -- round 1 is undone
				const bool nerr = p.err != 0u;
				if (nerr && !perr) {
					cur = err_cos;
					pend = 0u;
					hops = 0u;
					mark = 0u;
					matched = 0u;
					loop = 0u;
				}
				perr = nerr;
				ok_parse = valid && p.ret >= 0;
			}
		}
		if constexpr (plan_n<SPEC>::v > 0) {
			// tree-plan kernel: the plan's rounds, each for the lanes on its
			// joint group, then the reference's scan for any lane still
			// pending (off the plan)
			auto round = [&](auto ic) {
				constexpr uint32_t I = decltype(ic)::value;
				if (__ballot(pend != 0u) == 0ull)
					return;
				const uint32_t cw = pend != 0u ? H[COS_WORDS * (uint32_t)cur + C_BV] : 0u;
				const bool bvl = pend != 0u && ((cw >> 24) & 0x7fu) == SPEC::gid[I];
				uint32_t hit = 0, nleaf = 0, nxt = 0, nmark = 0;
				if (__ballot(bvl) != 0ull)
					plan_eval<SPEC, I>(H, bvl, bvl ? (uint32_t)cur : 0u, k, p, x, hit, nxt, nmark,
							   nleaf);
				advance(bvl ? 1u : 0u, hit, nxt, nmark, nleaf);
			};
			static_for<plan_n<SPEC>::v>(round);
			for (;;) {
				const unsigned long long am = __ballot(pend != 0u);
				if (am == 0ull)
					break;
				const int32_t c1 = __builtin_amdgcn_readlane(cur, (int)__builtin_ctzll(am));
				const bool g = pend != 0u && cur == c1;
				const cword_t ce = hc + COS_WORDS * (uint32_t)c1;
				uint32_t hit = 0, nxt = 0, nmark = 0;
				linear_scan(prog, ce[C_REC0], ce[C_NR], g, k, p, x, hit, nxt, nmark);
				advance(g ? 1u : 0u, hit, nxt, nmark, 0u);
			}
		}
#ifdef DIAG_MAXROUND
		uint32_t diag_round = 1;
#endif
		// (the generic descent: not instantiated in tree-plan kernels)
		if constexpr (plan_n<SPEC>::v == 0) for (; FM < 0;) {
			const unsigned long long pm = __ballot(pend != 0u);
			if (pm == 0ull)
				break;
#ifdef DIAG_MAXROUND
			// diagnostic timing variant: the descent stops after DIAG_MAXROUND
			// rounds (records are wrong; never a shipped build)
			if (++diag_round > DIAG_MAXROUND)
				break;
#endif
			uint32_t hit = 0, nleaf = 0, nxt = 0, nmark = 0, handled = 0;
			bool act = pend != 0u;
			if constexpr (DIV) {
				const int32_t c0 = __builtin_amdgcn_readlane(cur, (int)__builtin_ctzll(pm));
				if (__ballot(pend != 0u && cur != c0) != 0ull) {
					const uint32_t ci = COS_WORDS * (uint32_t)(pend != 0u ? cur : c0);
					const uint32_t my_nr = H[ci + C_NR];
					const uint32_t my_bw = H[ci + C_BV];
					const uint32_t my_bv = my_bw & C_BV_OFF;
					const bool empty = pend != 0u && my_nr == 0u;
					const bool bvl = pend != 0u && my_nr != 0u && my_bv != 0u;
					const unsigned long long bm = __ballot(bvl);
					// every lane with a block sits on a CoS of one joint group:
					// the group's words in SGPRs, one probe per lane and class of
					// the group's (key, CoS) tables, no per-lane block reads
					const uint32_t jg = (my_bw >> 24) & 0x7fu;
					const uint32_t g0 = bm ? (uint32_t)__builtin_amdgcn_readlane(
									 (int)jg, (int)__builtin_ctzll(bm)) : 0u;
					if (g0 != 0u && __ballot(bvl && jg != g0) == 0ull) {
						const DescU jd{ hc + hc[j_off + g0 - 1u], hc };
						const auto ji = jd.vec(0u);
						const uint32_t cs = bvl ? (uint32_t)cur : 0u;
						uint32_t rw;
						bool hv;
						if (ji(0) == 0u) {
							// direct: the first live rule's result word
							const auto cr = DescU{ hc + ji(8), hc }.vec(0u);
							uint32_t key[4], nk = cr(1);
							const bool present = bv_key(cr, k, p, x, key);
							joint_key(ji(14), cs, key, nk);
							const uint32_t val = bv_probe(H, key, bvl && present, nk, ji(9),
										      ji(10), ji(11), ji(12));
							const uint32_t miss = H[ji(13) + cs];
							rw = val != 0u ? (val == BV_EMPTY ? 0u : val) : miss;
							hv = rw != 0u;
						} else {
							// bitmap: AND of the classes' rule rows and the
							// CoS's alive row, then its result word
							const uint32_t ncls = ji(1);
							uint32_t acc = H[ji(2) + cs];
#pragma unroll
							for (uint32_t kc = 0; kc < BV_MAX_CLS; ++kc) {
								if (kc < ncls) {
									const auto ci = jd.vec(8u + 8u * kc);
									const auto cr = DescU{ hc + ci(0), hc }.vec(0u);
									uint32_t key[4], nk = cr(1);
									const bool present = bv_key(cr, k, p, x, key);
									joint_key(ci(6), cs, key, nk);
									const uint32_t val = bv_probe(H, key, bvl && present, nk,
												      ci(1), ci(2), ci(3), ci(4));
									acc &= val != 0u ? val : H[ci(5) + cs];
								}
							}
							const uint32_t res = H[ji(3) + cs];
							rw = H[res + (acc != 0u ? (uint32_t)__builtin_ctz(acc) : 0u)];
							hv = acc != 0u;
						}
						const bool h = bvl && hv;
						nxt = h ? (rw & 0xffu) : nxt;
						nleaf = h ? ((rw >> 8) & 1u) : nleaf;
						nmark = h ? (rw >> 16) : nmark;
						hit = h ? 1u : hit;
					} else if (bm) {
						bv_eval(DescL<hot_t>{ H, my_bv, hc }, H, bvl, k, p, x, hit, nxt, nmark,
							nleaf, (uint32_t)cur);
					}
					handled = (bvl || empty) ? 1u : 0u;
					act = pend != 0u && handled == 0u;
				}
			}
			uint32_t grp = 0;
			const unsigned long long am = __ballot(act);
			if (am) {
				const int32_t c1 = __builtin_amdgcn_readlane(cur, (int)__builtin_ctzll(am));
				const bool g = act && cur == c1;
				grp = g ? 1u : 0u;
				const cword_t ce = hc + COS_WORDS * (uint32_t)c1;
				const uint32_t nr = ce[C_NR], bv = DIV ? ce[C_BV] & C_BV_OFF : ce[C_BV] & 0x7fffffffu;
				if (bv != 0u && nr != 0u)
					bv_eval<-1, !DIV>(DescU{ hc + bv, hc }, H, g, k, p, x, hit, nxt, nmark,
							  nleaf, (uint32_t)c1);
				else
					linear_scan(prog, ce[C_REC0], nr, g, k, p, x, hit, nxt, nmark);
			}
			advance(handled | grp, hit, nxt, nmark, nleaf);
		}

#ifdef DIAG_DESCENTONLY
		if (valid) {
			uint4 rec;
			rec.x = (uint32_t)cur;
			rec.y = mark;
			rec.z = hops | (matched << 8) | (loop << 9);
			rec.w = p.flags;
			*(uint4 *)(a.out + pi) = rec;
		}
		continue;
#endif
		// ---- final CoS -> outcome / queue (_odp_cls_classify_packet, :1742-1771)
		const bool mk = matched != 0u && loop == 0u;
		const uint32_t flags = mk ? ((p.flags & ~F_CLS_MARK) | (mark ? F_CLS_MARK : 0u)) : p.flags;
		const uint32_t out_mark = (mk && mark) ? mark : 0u;
		const bool live = ok_parse && loop == 0u;
		// error CoS, the CoS the descent ended on, or the default CoS
		const bool to_cur = !perr && matched != 0u && cur != def_cos;
		const int32_t fc = perr ? err_cos : (to_cur ? cur : def_cos);
		if (stats_on) {
			if (live && !to_cur && fc >= 0 && stats_bit(a, (uint32_t)fc))
				atomicAdd(&s_cnt[fc], 1u);
		}
		const uint32_t meta = H[COS_WORDS * (uint32_t)max(fc, 0) + C_META];
		const bool have = live && fc >= 0;
		const bool drop = (meta & 0xffu) != 0u;
		const uint32_t outcome = !valid ? MI_CLS_OUT_DISCARD
			: (p.ret < 0 ? MI_CLS_OUT_PARSE_DROP
			: (loop ? MI_CLS_OUT_LOOP
			: (fc < 0 ? MI_CLS_OUT_DISCARD
			: (drop ? MI_CLS_OUT_COS_DROP : MI_CLS_OUT_ENQ))));
		const uint32_t cos_idx = have ? (meta >> 24) : 0xFFu;
		const uint32_t nq = (meta >> 8) & 0xffu;
		const bool hq = have && !drop && nq > 1u;
		uint32_t queue = 0;
		if (__ballot(hq) != 0ull) {
			if (hq)
				queue = (rss_hash(k, p, (meta >> 16) & 0xffu) & 31u) % nq;
		}
		hops = loop ? 0xFFu : hops;

		prev_rec.x = flags;
		prev_rec.y = (p.err & 0xffu) | ((outcome & 0xffu) << 8) | ((cos_idx & 0xffu) << 16) |
			     ((hops & 0xffu) << 24);
		prev_rec.z = (queue & 0xffffu) | ((out_mark & 0xffffu) << 16);
		prev_rec.w = (p.l3 & 0xffffu) | ((p.l4 & 0xffffu) << 16);
		prev_pi = pi;
		prev_valid = valid;
	}
	if (prev_valid)
		store_rec(a.out + prev_pi, prev_rec);
	// the waves of block 0 are the sample that sets the hint: stores to one
	// address serialise, so never one per wave
	if (saw_hi && a.hint && lane == 0 && blockIdx.x == 0)
		*a.hint = a.seq;

	if (stats_on) {
		__syncthreads();
		for (uint32_t i = threadIdx.x; i < MAX_STATS_COS; i += NW * WAVE)
			if (s_cnt[i])
				atomicAdd(a.stats + i, (unsigned long long)s_cnt[i]);
	}
}


#ifndef __HIPCC_RTC__
// Launch one instantiation of the kernel for block shape NW (defined in
// mi_cls_k<NW>.hip).
int mi_cls_launch_k4(bool lt, bool div, unsigned grid, size_t dyn, hipStream_t st, const KArgs &a);
int mi_cls_launch_k8(bool lt, bool div, unsigned grid, size_t dyn, hipStream_t st, const KArgs &a);
int mi_cls_launch_k12(bool lt, bool div, unsigned grid, size_t dyn, hipStream_t st, const KArgs &a);
int mi_cls_launch_k16(bool lt, bool div, unsigned grid, size_t dyn, hipStream_t st, const KArgs &a);
// flat-program kernels (FM = engine of the default CoS block; NW 4, 12, 16;
// hot region in LDS): mi_cls_kf.hip
int mi_cls_launch_flat(int nw, int fm, unsigned grid, size_t dyn, hipStream_t st, const KArgs &a);
// pktin-option kernels (CK; NW 4 or 16): mi_cls_kc.hip
int mi_cls_launch_ck(int nw, bool lt, bool div, unsigned grid, size_t dyn, hipStream_t st,
		     const KArgs &a);
// receive delivery (mi_cls_kd.hip); grid 0: preload only
int mi_cls_launch_deliver(unsigned grid, hipStream_t st, const mi_cls_dlv_args_t &h);
// receive chain (mi_cls_kd.hip): the decisions, then the delivery, on `st`
// after the burst's classification; preload: resolve both kernels only.  The chain's device-resident
// per-burst arrays (the context's, one set per ticket slot): the records
// (the classification writes them here; the delivery copies them to
// args.res), the decision words and each enqueued frame's queue handle --
// the decide and delivery kernels read these from HBM, not over the host
// link.
struct mi_cls_rxdev_t {
	mi_cls_result_t *res;
	uint32_t *dec;
	uint64_t *dq;
	uint16_t *len;              // dlen: each frame's length, and
	uint8_t *pp;                //       its packet's pool + 1 (the stage kernel's)
	const mi_cls_rxtab_t *tab;  // the table's copy in HBM
	uint32_t dlen;              // 1: len / pp hold the burst (else args.slen / ppool)
};
int mi_cls_launch_rx_chain(hipStream_t st, const mi_cls_rxc_args_t &a, const mi_cls_rxdev_t &d, bool preload);
// loop receive staging on the device (mi_cls_rxc_args_t.stage)
int mi_cls_launch_rx_stage(hipStream_t st, const mi_cls_rxc_args_t &a, const mi_cls_rxdev_t &d, uint64_t bytes,
			   bool preload);

// Every launcher goes through mi_launch.  grid == 0 launches nothing: it
// resolves the instantiation on the current device (hipFuncGetAttributes
// loads the code object that holds it), so mi_cls_ctx_create can load every
// kernel of the library before the first launch and no code object is ever
// first loaded later in the process's life (e.g. after specialised modules
// were loaded).
static inline const void *mi_kaddr(void (*k)(KArgs))
{
	return reinterpret_cast<const void *>(k);
}

// `lds` caches the kernel's static LDS bytes (one per launch site): a launch
// whose static + dynamic LDS exceeds the CU's 160 KiB fails with -E2BIG
// instead of running with a hot-region copy past the allocation.
#define MI_LDS_BYTES (160u * 1024u)
static inline int mi_launch(const void *k, unsigned grid, unsigned block, size_t dyn, hipStream_t st,
			    const KArgs &a, size_t *lds)
{
	size_t sl = __atomic_load_n(lds, __ATOMIC_RELAXED);
	if (sl == ~(size_t)0) {
		hipFuncAttributes fa;
		if (hipFuncGetAttributes(&fa, k) != hipSuccess)
			return -EIO;
		sl = fa.sharedSizeBytes;
		__atomic_store_n(lds, sl, __ATOMIC_RELAXED);
	}
	if (grid == 0)
		return 0;
	if (sl + dyn > MI_LDS_BYTES)
		return -E2BIG;
	void *args[] = { (void *)&a };
	return hipLaunchKernel(k, dim3(grid), dim3(block), args, dyn, st) == hipSuccess ? 0 : -EIO;
}

// Variant builds for A/B runs (odp_amd/_build.py, MI_CLS_ONLY): translation
// units outside the selected set are compiled with MI_CLS_STUB, so their
// launchers instantiate no kernel and fail with -ENOSYS.
#ifdef MI_CLS_STUB
#define MI_LAUNCH(K, grid, block, dyn, st, a) return -ENOSYS
#else
#define MI_LAUNCH(K, grid, block, dyn, st, a)                                             \
	do {                                                                               \
		static size_t lds_ = ~(size_t)0;                                           \
		const int rc_ = mi_launch(mi_kaddr(K), grid, (unsigned)(block), dyn, st, a, &lds_); \
		if (rc_)                                                                   \
			return rc_;                                                        \
	} while (0)
#endif

#endif   // !__HIPCC_RTC__
