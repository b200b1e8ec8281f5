"""Frames with valid and corrupted checksums for the pktin checksum tests.

Test infrastructure: the checksums are computed here from the protocol
definitions (RFC 1071 one's-complement sum, RFC 768 / RFC 793 / RFC 8200
pseudo headers, RFC 4960 / RFC 3309 CRC-32C), independently of the oracle,
so the oracle's verdicts can be cross-checked on frames whose validity is
known by construction.  The reference's own test frames
(test/common/test_packet_ipv4.h etc., tests/golden/parse_frames.json) carry
valid checksums and pin the same verdicts.
"""
import struct

import numpy as np

from odp_amd import pktgen as pg

# odp_pktin_config_opt_t bits (include/odp/api/spec/packet_io.h)
IPV4_CK, UDP_CK, TCP_CK, SCTP_CK = 1 << 2, 1 << 3, 1 << 4, 1 << 5
DROP_V4, DROP_V6, DROP_UDP, DROP_TCP, DROP_SCTP = 1 << 6, 1 << 7, 1 << 8, 1 << 9, 1 << 10
ALL_CK = IPV4_CK | UDP_CK | TCP_CK | SCTP_CK
ALL_DROP = DROP_V4 | DROP_V6 | DROP_UDP | DROP_TCP | DROP_SCTP

L3_DONE, L4_DONE = 1 << 30, 1 << 31       # input_flags bits
E_IP, E_L3CK, E_TCP, E_UDP, E_SCTP, E_L4CK = 2, 4, 8, 16, 32, 64


def ones_sum(data: bytes) -> int:
    """RFC 1071 16-bit one's-complement sum (big-endian words, odd byte
    padded), folded."""
    if len(data) % 2:
        data += b"\x00"
    s = sum(struct.unpack(f"!{len(data) // 2}H", data))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def inet_csum(data: bytes) -> int:
    return (~ones_sum(data)) & 0xFFFF


def crc32c(data: bytes, crc: int = 0xFFFFFFFF) -> int:
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ 0x82F63B78 if crc & 1 else crc >> 1
    return crc


def _put16(b: bytearray, o: int, v: int):
    b[o:o + 2] = struct.pack("!H", v)


def build(rng, ver=4, proto=pg.IPPROTO_UDP, payload=None, vlan=False, ipopt=False,
          udp_zero=False):
    """One Ethernet frame with correct IPv4 header / UDP / TCP / SCTP
    checksums; returns (frame, l3, l4)."""
    if payload is None:
        payload = bytes(rng.integers(0, 256, int(rng.integers(0, 200))).astype(np.uint8))
    ethtype = pg.ETH_IPV4 if ver == 4 else pg.ETH_IPV6
    e = pg.eth(ethtype=ethtype, tags=(100,) if vlan else ())
    l3 = len(e)
    if proto == pg.IPPROTO_UDP:
        l4h = bytearray(pg.udp(int(rng.integers(1, 65535)), int(rng.integers(1, 65535)),
                               payload=payload))
    elif proto == pg.IPPROTO_TCP:
        l4h = bytearray(pg.tcp(int(rng.integers(1, 65535)), int(rng.integers(1, 65535)))) + payload
    else:
        l4h = bytearray(pg.sctp(int(rng.integers(1, 65535)), int(rng.integers(1, 65535)))) + payload
    if ver == 4:
        src, dst = bytes(rng.integers(0, 256, 4).astype(np.uint8)), bytes(
            rng.integers(0, 256, 4).astype(np.uint8))
        opts = b"\x01\x01\x01\x00" if ipopt else b""
        ip = bytearray(pg.ipv4(src=src, dst=dst, proto=proto, payload_len=len(l4h), options=opts))
        _put16(ip, 10, inet_csum(bytes(ip)))
        pseudo = src + dst + struct.pack("!BBH", 0, proto, len(l4h))
    else:
        src, dst = bytes(rng.integers(0, 256, 16).astype(np.uint8)), bytes(
            rng.integers(0, 256, 16).astype(np.uint8))
        ip = bytearray(pg.ipv6(src=src, dst=dst, next_hdr=proto, payload_len=len(l4h)))
        pseudo = src + dst + struct.pack("!IxxxB", len(l4h), proto)
    l4 = l3 + len(ip)
    if proto == pg.IPPROTO_UDP:
        c = 0 if udp_zero else (inet_csum(pseudo + bytes(l4h)) or 0xFFFF)
        _put16(l4h, 6, c)
    elif proto == pg.IPPROTO_TCP:
        _put16(l4h, 16, inet_csum(pseudo + bytes(l4h)))
    else:
        l4h[8:12] = b"\x00\x00\x00\x00"
        crc = (~crc32c(bytes(l4h))) & 0xFFFFFFFF
        l4h[8:12] = struct.pack("<I", crc)
    return bytes(e) + bytes(ip) + bytes(l4h), l3, l4


def corrupt(rng, frame: bytes, lo: int, hi: int) -> bytes:
    """Flip one bit of a byte in [lo, hi)."""
    b = bytearray(frame)
    i = int(rng.integers(lo, hi))
    b[i] ^= 1 << int(rng.integers(0, 8))
    return bytes(b)


def frame_set(seed=7, n=400):
    """Valid frames of every protocol / IP version, and corrupted copies
    (IP header, L4 header, payload), with the expected verdicts:
    [(frame, l3_bad or None, l4_bad or None)]."""
    rng = np.random.default_rng(seed)
    out = []
    kinds = [(4, pg.IPPROTO_UDP), (4, pg.IPPROTO_TCP), (4, pg.IPPROTO_SCTP),
             (6, pg.IPPROTO_UDP), (6, pg.IPPROTO_TCP), (6, pg.IPPROTO_SCTP)]
    for i in range(n):
        ver, proto = kinds[i % len(kinds)]
        fr, l3, l4 = build(rng, ver, proto, vlan=bool(i % 5 == 0), ipopt=(ver == 4 and i % 7 == 0))
        out.append((fr, False if ver == 4 else None, False))
        what = i % 3
        hdr = {pg.IPPROTO_UDP: 8, pg.IPPROTO_TCP: 20}.get(proto, 12)
        if what == 0 and ver == 4:
            # IPv4 header bit (not the version / IHL / length fields)
            out.append((corrupt(rng, fr, l3 + 8, l4), True, None))
        elif what == 1 and len(fr) > l4 + hdr:
            # payload bit
            out.append((corrupt(rng, fr, l4 + hdr, len(fr)), False if ver == 4 else None, True))
        else:
            # port bit
            out.append((corrupt(rng, fr, l4, l4 + 4), False if ver == 4 else None, True))
    # UDP zero checksum: accepted on IPv4, an error on IPv6 (parse_udp)
    for ver in (4, 6):
        fr, _, _ = build(rng, ver, pg.IPPROTO_UDP, udp_zero=True)
        out.append((fr, False if ver == 4 else None, ver == 6))
    return out
