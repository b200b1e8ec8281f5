"""Packet construction and synthetic batch generation.

Two layers:

* ``Pkt`` builders -- byte-exact single frames (Ethernet / 802.1Q / QinQ /
  SNAP, IPv4 with options and fragments, IPv6 with extension headers, UDP /
  TCP / SCTP / ICMP / AH / ESP) used by the parity zoo.  They play the role of
  the reference's test packet factory (test/validation/api/classification/
  odp_classification_common.c:360-606, create_packet).
* vectorised batch builders (numpy) for the BASELINE.json workloads: 1 M
  packets in a contiguous buffer, each frame at a 64-byte aligned offset,
  described by ``off`` (uint32) and ``len`` (uint16) arrays -- the batch
  layout of include/mi_cls.h.

Frame lengths exclude the FCS (a "64 B" packet is a 60 B buffer, as in
example/classifier/udp64.pcap).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import numpy as np

ETH_IPV4 = 0x0800
ETH_IPV6 = 0x86DD
ETH_ARP = 0x0806
ETH_VLAN = 0x8100
ETH_QINQ = 0x88A8

IPPROTO_ICMP = 1
IPPROTO_IPIP = 4
IPPROTO_TCP = 6
IPPROTO_UDP = 17
IPPROTO_HOPOPTS = 0
IPPROTO_ROUTE = 43
IPPROTO_FRAG = 44
IPPROTO_ESP = 50
IPPROTO_AH = 51
IPPROTO_ICMPV6 = 58
IPPROTO_NONE = 59
IPPROTO_SCTP = 132

ALIGN = 64


def ip4(s: str) -> bytes:
    return bytes(int(x) for x in s.split("."))


def ip6(s: str) -> bytes:
    import ipaddress
    return ipaddress.IPv6Address(s).packed


def mac(s: str) -> bytes:
    return bytes(int(x, 16) for x in s.split(":"))


# --------------------------------------------------------------- single frames
def eth(dst=b"\x02\x00\x00\x00\x00\x01", src=b"\x02\x00\x00\x00\x00\x02",
        ethtype=ETH_IPV4, tags=(), tpids=None) -> bytes:
    """Ethernet header; ``tags`` is a sequence of TCI values, outermost first.
    Default TPIDs: one tag -> 0x8100, two tags -> 0x88A8 then 0x8100."""
    hdr = dst + src
    if tpids is None:
        tpids = [ETH_VLAN] if len(tags) == 1 else [ETH_QINQ, ETH_VLAN][: len(tags)]
    for tpid, tci in zip(tpids, tags):
        hdr += struct.pack("!HH", tpid, tci)
    return hdr + struct.pack("!H", ethtype)


def ipv4(src="10.0.0.1", dst="10.0.0.100", proto=IPPROTO_UDP, payload_len=0, tos=0,
         frag=0, ttl=64, options=b"", tot_len=None, ver=4, ihl=None, ident=1) -> bytes:
    if isinstance(src, str):
        src = ip4(src)
    if isinstance(dst, str):
        dst = ip4(dst)
    assert len(options) % 4 == 0
    if ihl is None:
        ihl = 5 + len(options) // 4
    if tot_len is None:
        tot_len = 20 + len(options) + payload_len
    return struct.pack("!BBHHHBBH4s4s", (ver << 4) | ihl, tos, tot_len, ident, frag, ttl,
                       proto, 0, src, dst) + options


def ipv6(src="2001:db8::1", dst="2001:db8::2", next_hdr=IPPROTO_UDP, payload_len=0,
         tc=0, flow=0, hop=64, ver=6) -> bytes:
    if isinstance(src, str):
        src = ip6(src)
    if isinstance(dst, str):
        dst = ip6(dst)
    vtf = (ver << 28) | (tc << 20) | flow
    return struct.pack("!IHBB", vtf, payload_len, next_hdr, hop) + src + dst


def ipv6_ext(next_hdr, ext_len=0, fill=b"") -> bytes:
    """Generic IPv6 extension header (HBH / routing): 8 + 8*ext_len bytes."""
    body = (fill + bytes(6 + 8 * ext_len))[: 6 + 8 * ext_len]
    return struct.pack("!BB", next_hdr, ext_len) + body


def udp(sport=1024, dport=2048, length=None, payload=b"") -> bytes:
    if length is None:
        length = 8 + len(payload)
    return struct.pack("!HHHH", sport, dport, length, 0) + payload


def tcp(sport=1024, dport=2048, hl=5, flags=0x02) -> bytes:
    return struct.pack("!HHIIBBHHH", sport, dport, 1, 0, hl << 4, flags, 0, 0, 0) + bytes(
        max(0, hl * 4 - 20))


def sctp(sport=1024, dport=2048) -> bytes:
    return struct.pack("!HHII", sport, dport, 0, 0)


def icmp(typ=8, code=0) -> bytes:
    return struct.pack("!BBHHH", typ, code, 0, 1, 1)


def ah(spi, next_hdr=IPPROTO_UDP) -> bytes:
    return struct.pack("!BBHII", next_hdr, 4, 0, spi, 1) + bytes(12)


def esp(spi) -> bytes:
    return struct.pack("!II", spi, 1)


def pad_to(frame: bytes, n: int) -> bytes:
    return frame + bytes(max(0, n - len(frame)))


def udp4_frame(src="10.0.0.1", dst="10.0.0.100", sport=1024, dport=2048, size=60,
               tags=(), tos=0, frag=0, dmac=None, tpids=None) -> bytes:
    """Eth[/VLAN]/IPv4/UDP frame of ``size`` bytes (IP and UDP lengths fit the frame)."""
    l2 = eth(tags=tags, tpids=tpids, **({"dst": dmac} if dmac else {}))
    ip_len = size - len(l2)
    return l2 + ipv4(src, dst, IPPROTO_UDP, payload_len=ip_len - 20, tos=tos, frag=frag) + \
        udp(sport, dport, length=ip_len - 20) + bytes(ip_len - 28)


def tcp4_frame(src="10.0.0.1", dst="10.0.0.100", sport=1024, dport=2048, size=60,
               tags=()) -> bytes:
    l2 = eth(tags=tags)
    ip_len = size - len(l2)
    return l2 + ipv4(src, dst, IPPROTO_TCP, payload_len=ip_len - 20) + tcp(sport, dport) + \
        bytes(ip_len - 40)


def udp6_frame(src="2001:db8::1", dst="2001:db8::2", sport=1024, dport=2048, size=78,
               tags=(), tc=0) -> bytes:
    l2 = eth(ethtype=ETH_IPV6, tags=tags)
    pl = size - len(l2) - 40
    return l2 + ipv6(src, dst, IPPROTO_UDP, payload_len=pl, tc=tc) + udp(sport, dport, length=pl) + \
        bytes(pl - 8)


# --------------------------------------------------------------------- batches
@dataclass
class Batch:
    buf: np.ndarray      # uint8, packed frames
    off: np.ndarray      # uint32 byte offset of each frame (64-B aligned)
    len: np.ndarray      # uint16 frame length

    @property
    def n(self) -> int:
        return int(self.off.shape[0])

    def frame(self, i: int) -> bytes:
        o = int(self.off[i])
        return self.buf[o: o + int(self.len[i])].tobytes()

    def header_bytes(self) -> int:
        """Algorithmic bytes of the batch: min(len,128) window + 6-B descriptor + 16-B result."""
        return int(np.minimum(self.len.astype(np.int64), 128).sum()) + 22 * self.n

    def slice(self, begin: int, end: int) -> "Batch":
        """Contiguous sub-batch [begin, end) with its own compact buffer."""
        o0 = int(self.off[begin])
        o1 = int(self.off[end - 1]) + _round_up(int(self.len[end - 1]))
        return Batch(self.buf[o0:o1].copy(), (self.off[begin:end] - o0).astype(np.uint32),
                     self.len[begin:end].copy())


def _round_up(x, a=ALIGN):
    return (x + a - 1) // a * a


def batch_from_frames(frames) -> Batch:
    lens = np.array([len(f) for f in frames], dtype=np.int64)
    slots = (lens + ALIGN - 1) // ALIGN * ALIGN
    slots = np.maximum(slots, ALIGN)
    off = np.zeros(len(frames), dtype=np.int64)
    if len(frames):
        off[1:] = np.cumsum(slots)[:-1]
    total = int(off[-1] + slots[-1]) if len(frames) else ALIGN
    buf = np.zeros(total + ALIGN, dtype=np.uint8)
    for f, o in zip(frames, off):
        buf[o: o + len(f)] = np.frombuffer(f, dtype=np.uint8)
    return Batch(buf, off.astype(np.uint32), lens.astype(np.uint16))


def _layout(lens: np.ndarray):
    slots = (lens.astype(np.int64) + ALIGN - 1) // ALIGN * ALIGN
    off = np.zeros(lens.shape[0], dtype=np.int64)
    off[1:] = np.cumsum(slots)[:-1]
    total = int(off[-1] + slots[-1]) + ALIGN
    return off, total


def _put_be16(h, col, v):
    v = np.asarray(v, dtype=np.uint32)
    h[:, col] = (v >> 8) & 0xFF
    h[:, col + 1] = v & 0xFF


def _put_be32(h, col, v):
    v = np.asarray(v, dtype=np.uint64)
    for i in range(4):
        h[:, col + i] = (v >> np.uint64(24 - 8 * i)) & np.uint64(0xFF)


def build_batch(lens, *, ipver, l4proto, sip4=None, dip4=None, sip6=None, dip6=None,
                sport, dport, ntags=None, vid0=None, vid1=None, tos=None, seed=0) -> Batch:
    """Vectorised Eth[/VLAN/QinQ]/(IPv4|IPv6)/(UDP|TCP|SCTP) batch.

    All arguments are per-packet arrays.  ntags: 0 untagged, 1 802.1Q (vid0),
    2 QinQ (0x88A8 vid0 outer, 0x8100 vid1 inner).  IP/UDP length fields are
    consistent with the frame length; payload bytes are a deterministic
    pseudo-random fill.
    """
    n = lens.shape[0]
    if ntags is None:
        ntags = np.zeros(n, np.int64)
    # never emit a frame shorter than its own headers
    hdr_len = 14 + 4 * np.asarray(ntags) + np.where(np.asarray(ipver) == 6, 40, 20) + \
        np.where(np.asarray(l4proto) == IPPROTO_TCP, 20,
                 np.where(np.asarray(l4proto) == IPPROTO_SCTP, 12, 8))
    lens = np.maximum(lens.astype(np.int64), hdr_len)
    off, total = _layout(lens)
    rng = np.random.default_rng(seed ^ 0x5EED)
    buf = rng.integers(0, 256, total, dtype=np.uint8)
    # zero each frame's slot tail (bytes past frame_len) so that reads past
    # the frame are deterministic zeros, as in the fixtures
    H = 18 + 4 * 2 + 40 + 20 + 2  # max header span we write
    for nt in (0, 1, 2):
        for v in (4, 6):
            for p in (IPPROTO_UDP, IPPROTO_TCP, IPPROTO_SCTP):
                sel = np.nonzero((ntags == nt) & (ipver == v) & (l4proto == p))[0]
                if sel.size == 0:
                    continue
                m = sel.size
                h = np.zeros((m, H), dtype=np.uint8)
                h[:, 0:6] = np.frombuffer(b"\x02\x00\x00\x00\x00\x01", np.uint8)
                h[:, 6:12] = np.frombuffer(b"\x02\x00\x00\x00\x00\x02", np.uint8)
                c = 12
                if nt == 1:
                    _put_be16(h, c, ETH_VLAN)
                    _put_be16(h, c + 2, vid0[sel])
                    c += 4
                elif nt == 2:
                    _put_be16(h, c, ETH_QINQ)
                    _put_be16(h, c + 2, vid0[sel])
                    _put_be16(h, c + 4, ETH_VLAN)
                    _put_be16(h, c + 6, vid1[sel])
                    c += 8
                ln = lens[sel]
                if v == 4:
                    _put_be16(h, c, ETH_IPV4)
                    c += 2
                    l3 = c
                    ip_len = ln - l3
                    h[:, l3] = 0x45
                    h[:, l3 + 1] = 0 if tos is None else tos[sel]
                    _put_be16(h, l3 + 2, ip_len)
                    _put_be16(h, l3 + 4, 1)
                    h[:, l3 + 8] = 64
                    h[:, l3 + 9] = p
                    _put_be32(h, l3 + 12, sip4[sel])
                    _put_be32(h, l3 + 16, dip4[sel])
                    l4 = l3 + 20
                    l4_len = ip_len - 20
                else:
                    _put_be16(h, c, ETH_IPV6)
                    c += 2
                    l3 = c
                    l4_len = ln - l3 - 40
                    vtf = (6 << 28) | ((0 if tos is None else tos[sel].astype(np.int64)) << 20)
                    _put_be32(h, l3, vtf)
                    _put_be16(h, l3 + 4, l4_len)
                    h[:, l3 + 6] = p
                    h[:, l3 + 7] = 64
                    h[:, l3 + 8: l3 + 24] = sip6[sel]
                    h[:, l3 + 24: l3 + 40] = dip6[sel]
                    l4 = l3 + 40
                _put_be16(h, l4, sport[sel])
                _put_be16(h, l4 + 2, dport[sel])
                if p == IPPROTO_UDP:
                    _put_be16(h, l4 + 4, l4_len)
                    hl = l4 + 8
                elif p == IPPROTO_SCTP:
                    _put_be32(h, l4 + 4, 0x5C7F0001)   # verification tag; CRC 0
                    hl = l4 + 12
                else:
                    _put_be32(h, l4 + 4, 1)
                    h[:, l4 + 12] = 0x50
                    h[:, l4 + 13] = 0x10
                    hl = l4 + 20
                idx = off[sel][:, None] + np.arange(hl)[None, :]
                buf[idx] = h[:, :hl]
    # zero the slot tails
    slot_end = np.empty(n, np.int64)
    slot_end[:-1] = off[1:]
    slot_end[-1] = total
    tail = slot_end - (off + lens)
    maxt = int(tail.max())
    if maxt > 0:
        idx = (off + lens)[:, None] + np.arange(maxt)[None, :]
        msk = np.arange(maxt)[None, :] < tail[:, None]
        buf[idx[msk]] = 0
    return Batch(buf, off.astype(np.uint32), lens.astype(np.uint16))


def _crc32c_tables():
    t = np.zeros(256, np.uint32)
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
        t[i] = c
    return t


_CRC32C = _crc32c_tables()


def sctp_crc32c(frames: np.ndarray) -> np.ndarray:
    """CRC-32C (init ~0, final inversion) of each row of a uint8 matrix,
    vectorised over rows: the SCTP checksum of RFC 4960 appendix B."""
    crc = np.full(frames.shape[0], 0xFFFFFFFF, np.uint32)
    for j in range(frames.shape[1]):
        crc = _CRC32C[(crc ^ frames[:, j]) & 0xFF] ^ (crc >> np.uint32(8))
    return ~crc


def set_checksums(b: Batch, l3: int = 14) -> Batch:
    """Write a valid IPv4 header checksum and valid L4 checksums into an
    untagged build_batch() batch (IPv4 IHL 5 or IPv6 without extension
    headers), in place, vectorised: RFC 1071 sums with the RFC 768 / 793 /
    8200 pseudo headers for UDP and TCP, CRC-32C (RFC 4960) for SCTP.  Other
    L4 protocols are left alone."""
    buf = b.buf
    off = b.off.astype(np.int64)
    ln = b.len.astype(np.int64)

    def fold(s):
        s = (s & 0xFFFF) + (s >> 16)
        s = (s & 0xFFFF) + (s >> 16)
        return (s & 0xFFFF) + (s >> 16)

    def words(base, nw):
        idx = base[:, None] + 2 * np.arange(nw)[None, :]
        return ((buf[idx].astype(np.int64) << 8) | buf[idx + 1]).sum(1)

    et = (buf[off + 12].astype(np.int64) << 8) | buf[off + 13]
    v4 = et == ETH_IPV4
    v6 = et == ETH_IPV6
    o4 = off[v4] + l3
    buf[o4 + 10] = 0
    buf[o4 + 11] = 0
    c = ~fold(words(o4, 10)) & 0xFFFF
    buf[o4 + 10] = (c >> 8).astype(np.uint8)
    buf[o4 + 11] = (c & 0xFF).astype(np.uint8)

    proto = np.where(v4, buf[off + l3 + 9], np.where(v6, buf[off + l3 + 6], 0)).astype(np.int64)
    l4 = off + np.where(v4, l3 + 20, l3 + 40)
    end = off + ln

    # UDP / TCP: 16-bit one's-complement sum over pseudo header + segment
    sel = np.nonzero((v4 | v6) & ((proto == IPPROTO_UDP) | (proto == IPPROTO_TCP)))[0]
    if sel.size:
        l4s, ends, pr, v4s = l4[sel], end[sel], proto[sel], v4[sel]
        cko = l4s + np.where(pr == IPPROTO_UDP, 6, 16)
        buf[cko] = 0
        buf[cko + 1] = 0
        o = off[sel]
        pseudo = np.where(v4s, words(o + l3 + 12, 4), words(o + l3 + 8, 16)) if not v4s.all() \
            else words(o + l3 + 12, 4)
        pseudo = pseudo + pr + (ends - l4s)
        # prefix sums of big-endian 16-bit words at even and at odd buffer
        # offsets (frames may start at either parity)
        s = np.zeros(sel.size, np.int64)
        for par in (0, 1):
            m = (l4s % 2) == par
            if not m.any():
                continue
            nw = (buf.size - par) // 2
            wp = (buf[par: par + 2 * nw: 2].astype(np.int64) << 8) | buf[par + 1: par + 2 * nw: 2]
            cs = np.concatenate([[0], np.cumsum(wp)])
            del wp
            a, e = (l4s[m] - par) // 2, (ends[m] - par) // 2
            odd = (ends[m] - l4s[m]) % 2 == 1
            s[m] = cs[e] - cs[a] + np.where(odd, buf[ends[m] - 1].astype(np.int64) << 8, 0)
        c = ~fold(pseudo + s) & 0xFFFF
        c = np.where((pr == IPPROTO_UDP) & (c == 0), 0xFFFF, c)
        buf[cko] = (c >> 8).astype(np.uint8)
        buf[cko + 1] = (c & 0xFF).astype(np.uint8)

    # SCTP: CRC-32C over the common header (checksum field zero) and chunks,
    # stored little-endian (the reference compares the raw 32-bit field)
    sel = np.nonzero((v4 | v6) & (proto == IPPROTO_SCTP))[0]
    for seg_len in np.unique(end[sel] - l4[sel]):
        g = sel[(end[sel] - l4[sel]) == seg_len]
        idx = l4[g][:, None] + np.arange(int(seg_len))[None, :]
        buf[l4[g][:, None] + 8 + np.arange(4)[None, :]] = 0
        crc = sctp_crc32c(buf[idx])
        for i in range(4):
            buf[l4[g] + 8 + i] = ((crc >> np.uint32(8 * i)) & np.uint32(0xFF)).astype(np.uint8)
    return b


IMIX_SIZES = np.array([60, 566, 1514])
IMIX_WEIGHTS = np.array([7, 4, 1])


def imix_lens(rng, n):
    w = IMIX_WEIGHTS / IMIX_WEIGHTS.sum()
    return rng.choice(IMIX_SIZES, size=n, p=w).astype(np.int64)


def seed_for(cfg: int) -> int:
    """Synthetic-input seed per BASELINE config."""
    return 0x0DF0C1A5 + cfg
