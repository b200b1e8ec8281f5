#!/usr/bin/env python3
"""Generate tests/golden/ fixtures from the reference tree's own test data.

Run HERE (the build container) only: it reads /root/reference, which does
not exist on the GPU box.  The outputs are committed; tests read only the
outputs.

Sources (all data, no code):
  * example/classifier/udp64.pcap -- the CI capture of the classifier
    example; expected split from platform/linux-generic/test/example/
    classifier/pktio_env:21-23 (`-C queue1:100 -C DefaultCos:100` with
    `-p ODP_PMR_SIP_ADDR:10.10.10.0:0xFFFFFF00:queue1`).
  * test/common/test_packet_{ipv4,ipv6,ipsec,custom}.h -- the byte arrays of
    the parser test frames.
  * the has_*() assertions the parser tests make on those frames
    (test/validation/api/packet/packet.c:3745-4541), transcribed below with
    line numbers; every listed frame also parses with return value 0
    (odp_packet_parse() == 0, e.g. packet.c:3767).
"""
import json
import os
import re
import struct
import sys

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


def c_arrays(path):
    txt = open(path).read()
    out = {}
    for m in re.finditer(r"static const uint8_t (\w+)\[\]\s*=\s*\{(.*?)\};", txt, re.S):
        body = re.sub(r"/\*.*?\*/", "", m.group(2), flags=re.S)
        vals = [int(x, 16) for x in re.findall(r"0x([0-9A-Fa-f]{1,2})", body)]
        out[m.group(1)] = bytes(vals).hex()
    return out


def pcapng_frames(path):
    data = open(path, "rb").read()
    frames, off = [], 0
    while off + 12 <= len(data):
        btype, blen = struct.unpack_from("<II", data, off)
        if btype == 6:   # enhanced packet block
            cap = struct.unpack_from("<I", data, off + 20)[0]
            frames.append(data[off + 28: off + 28 + cap].hex())
        elif btype == 3:  # simple packet block
            olen = struct.unpack_from("<I", data, off + 8)[0]
            frames.append(data[off + 12: off + 12 + olen].hex())
        off += blen
    return frames


# frame -> (packet.c line of the assertion block, {flag: expected})
PARSE_EXPECT = {
    "test_packet_ipv4_udp": (3772, dict(eth=1, ipv4=1, udp=1, ipv6=0, tcp=0)),
    "test_packet_snap_ipv4_udp": (3813, dict(eth=1, ipv4=1, udp=1, ipv6=0, tcp=0)),
    "test_packet_ipv4_tcp": (3881, dict(eth=1, ipv4=1, tcp=1, ipv6=0, udp=0)),
    "test_packet_ipv6_udp": (3914, dict(eth=1, ipv6=1, udp=1, ipv4=0, tcp=0)),
    "test_packet_ipv6_tcp": (3944, dict(eth=1, ipv6=1, tcp=1, ipv4=0, udp=0)),
    "test_packet_vlan_ipv4_udp": (3974, dict(eth=1, vlan=1, ipv4=1, udp=1, ipv6=0, tcp=0)),
    "test_packet_vlan_ipv6_udp": (4005, dict(eth=1, vlan=1, ipv6=1, udp=1, ipv4=0, tcp=0)),
    "test_packet_vlan_qinq_ipv4_udp": (4039, dict(eth=1, vlan=1, vlan_qinq=1, ipv4=1, udp=1,
                                                  ipv6=0, tcp=0)),
    "test_packet_arp": (4071, dict(eth=1, eth_bcast=1, arp=1, vlan=0, ipv4=0, ipv6=0, udp=0)),
    "test_packet_ipv4_icmp": (4103, dict(eth=1, ipv4=1, icmp=1, eth_bcast=0, ipv6=0, tcp=0)),
    "test_packet_ipv6_icmp": (4134, dict(eth=1, ipv6=1, icmp=1, eth_bcast=0, ipv4=0, tcp=0)),
    "test_packet_ipv4_sctp": (4165, dict(eth=1, ipv4=1, sctp=1, ipv6=0, tcp=0, udp=0)),
    "test_packet_ipv4_ipsec_ah": (4196, dict(eth=1, ipv4=1, ipsec=1, ipv6=0, tcp=0, udp=0)),
    "test_packet_ipv4_ipsec_esp": (4227, dict(eth=1, ipv4=1, ipsec=1, ipv6=0, tcp=0, udp=0)),
    "test_packet_ipv6_ipsec_ah": (4258, dict(eth=1, ipv6=1, ipsec=1, ipv4=0, tcp=0, udp=0)),
    "test_packet_ipv6_ipsec_esp": (4292, dict(eth=1, ipv6=1, ipsec=1, ipv4=0, tcp=0, udp=0)),
    "test_packet_mcast_eth_ipv4_udp": (4323, dict(eth=1, eth_mcast=1, ipv4=1, ip_mcast=1, udp=1,
                                                  ipv6=0, tcp=0, eth_bcast=0, ip_bcast=0)),
    "test_packet_bcast_eth_ipv4_udp": (4357, dict(eth=1, eth_bcast=1, eth_mcast=1, ipv4=1,
                                                  ip_bcast=1, udp=1, ipv6=0, tcp=0, ip_mcast=0)),
    "test_packet_mcast_eth_ipv6_udp": (4392, dict(eth=1, eth_mcast=1, ipv6=1, ip_mcast=1, udp=1,
                                                  ipv4=0, tcp=0, eth_bcast=0, ip_bcast=0)),
    "test_packet_ipv4_udp_first_frag": (4426, dict(eth=1, ipv4=1, ipfrag=1, udp=1, ipv6=0,
                                                   tcp=0, ipopt=0)),
    "test_packet_ipv4_udp_last_frag": (4458, dict(eth=1, ipv4=1, ipfrag=1, udp=1, ipv6=0,
                                                  tcp=0, ipopt=0)),
    "test_packet_ipv4_rr_nop_icmp": (4490, dict(eth=1, ipv4=1, ipopt=1, icmp=1, ipfrag=0,
                                                ipv6=0, udp=0, tcp=0)),
}


def main():
    os.makedirs(OUT, exist_ok=True)
    frames = {}
    for h in ("test_packet_ipv4.h", "test_packet_ipv6.h", "test_packet_ipsec.h",
              "test_packet_custom.h"):
        frames.update(c_arrays(os.path.join(REF, "test/common", h)))
    missing = [k for k in PARSE_EXPECT if k not in frames]
    if missing:
        sys.exit(f"frames not found: {missing}")
    parse = {k: {"frame": frames[k], "packet_c_line": ln, "ret": 0, "expect": exp}
             for k, (ln, exp) in PARSE_EXPECT.items()}
    extra = {k: {"frame": v} for k, v in frames.items() if k not in PARSE_EXPECT}
    with open(os.path.join(OUT, "parse_frames.json"), "w") as f:
        json.dump({"source": "test/common/test_packet_*.h; expectations "
                             "test/validation/api/packet/packet.c:3745-4541",
                   "frames": parse, "other_frames": extra}, f, indent=1, sort_keys=True)
    udp = pcapng_frames(os.path.join(REF, "example/classifier/udp64.pcap"))
    with open(os.path.join(OUT, "udp64.json"), "w") as f:
        json.dump({"source": "example/classifier/udp64.pcap",
                   "rule": "ODP_PMR_SIP_ADDR:10.10.10.0:0xFFFFFF00:queue1",
                   "expect_min": {"queue1": 100, "DefaultCos": 100},
                   "expect_source": "platform/linux-generic/test/example/classifier/pktio_env:21-23",
                   "frames": udp}, f, indent=0)
    print(f"{len(parse)} parser frames, {len(extra)} extra frames, {len(udp)} pcap frames")


if __name__ == "__main__":
    main()
