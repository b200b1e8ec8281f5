"""Known-answer cases transcribed from the reference's classifier validation
tests (test/validation/api/classification/), rebuilt with our own packet
factory using the same field values as the reference's create_packet()
(odp_classification_common.c:360-606; constants classification.h:13-84).

Each case: (name, rule program, [(frame, expected CoS ref, expected mark)]).
The expected values are what the reference test asserts: a MATCH packet
arrives on the PMR's destination CoS queue, a NO_MATCH packet on the default
CoS queue (test_pmr, odp_classification_test_pmr.c:678-719).
"""
import struct

from odp_amd import pktgen as pg
from odp_amd import rules as R

SMAC = bytes([0x07, 0x08, 0x09, 0x0a, 0x0b, 0x0c])     # CLS_DEFAULT_SMAC
DMAC = bytes([0x01, 0x02, 0x03, 0x04, 0x05, 0x06])     # CLS_DEFAULT_DMAC
SADDR, DADDR = "10.0.0.1", "10.0.0.100"                # CLS_DEFAULT_SADDR / DADDR
SPORT, DPORT = 1024, 2048                              # CLS_DEFAULT_SPORT / DPORT
V6_SRC = bytes(10) + b"\xff\xff" + bytes([10, 0, 0, 1])     # odp_classification_common.c:16
V6_DST = bytes(10) + b"\xff\xff" + bytes([10, 0, 0, 100])   # :21
MAGIC = 0x01020304                                     # DATA_MAGIC


def create_packet(ipv6=False, l4="tcp", vlan=False, qinq=False, dscp=0, extra_len=0, seq=1,
                  dmac=DMAC, tci0=0, tci1=0, sport=SPORT, dport=DPORT, src=None, dst=None,
                  spi=struct.pack("<I", 256)):
    """Same layout and field values as the reference test factory."""
    payload = struct.pack("<II", MAGIC, seq) + bytes(extra_len)
    l4hdr = {"tcp": 20, "udp": 8, "sctp": 12, "icmp": 8, "ah": 24, "esp": 8}[l4]
    proto = {"tcp": 6, "udp": 17, "sctp": 132, "icmp": 1, "ah": 51, "esp": 50}[l4]
    l4_len = l4hdr + len(payload)
    etype = pg.ETH_IPV6 if ipv6 else pg.ETH_IPV4
    hdr = dmac + SMAC
    if vlan and qinq:
        hdr += struct.pack("!HHHH", pg.ETH_QINQ, tci0, pg.ETH_VLAN, tci1) + struct.pack("!H", etype)
    elif vlan:
        hdr += struct.pack("!HH", pg.ETH_VLAN, tci0) + struct.pack("!H", etype)
    else:
        hdr += struct.pack("!H", etype)
    if not ipv6:
        ip = pg.ipv4(src or SADDR, dst or DADDR, proto, payload_len=l4_len, tos=dscp << 2, ttl=128,
                     ident=seq)
    else:
        ip = pg.ipv6(src or V6_SRC, dst or V6_DST, proto, payload_len=l4_len, tc=dscp << 2,
                     flow=seq, hop=128)
    if l4 == "tcp":
        l4b = struct.pack("!HHIIBBHHH", sport, dport, 0, 0, 5 << 4, 0x10, 0, 0, 0)
    elif l4 == "udp":
        l4b = struct.pack("!HHHH", sport, dport, 8 + len(payload), 0)
    elif l4 == "sctp":
        l4b = struct.pack("!HHII", sport, dport, 0, 0)
    elif l4 == "icmp":
        l4b = struct.pack("!BBHHH", 8, 0, 0, 0, 0)
    elif l4 == "ah":
        l4b = struct.pack("<BBH", 4, 24 // 4 - 2, 0) + spi + struct.pack("<I", 1) + bytes(12)
    else:
        l4b = spi + struct.pack("<I", 1)
    return hdr + ip + l4b + payload


def _with(frame, off, data):
    b = bytearray(frame)
    b[off: off + len(data)] = data
    return bytes(b)


def single(term):
    return [R.cos("default", queue=11), R.cos("hit", queue=22), ("default", 0),
            ("pmr", [term], 0, 1, 0)]


MATCH, NO_MATCH = 1, 0


def term_cases():
    """odp_classification_test_pmr.c:721-1544 (terms supported on linux-generic)."""
    C = []
    tcp = create_packet()
    l4 = 34
    # cls_pmr_term_tcp_sport :721-751
    C.append(("tcp_sport", single(R.t_be16(R.PMR_TCP_SPORT, SPORT)),
              [(tcp, MATCH), (_with(tcp, l4, struct.pack("!H", SPORT + 1)), NO_MATCH)]))
    # cls_pmr_term_tcp_dport (cls_pmr_term_tcp_dport_n :231-...)
    C.append(("tcp_dport", single(R.t_be16(R.PMR_TCP_DPORT, DPORT)),
              [(tcp, MATCH), (_with(tcp, l4 + 2, struct.pack("!H", DPORT + 1)), NO_MATCH)]))
    udp = create_packet(l4="udp")
    # :753-786, :788-821
    C.append(("udp_dport", single(R.t_be16(R.PMR_UDP_DPORT, DPORT)),
              [(udp, MATCH), (_with(udp, l4 + 2, struct.pack("!H", DPORT + 1)), NO_MATCH)]))
    C.append(("udp_sport", single(R.t_be16(R.PMR_UDP_SPORT, SPORT)),
              [(udp, MATCH), (_with(udp, l4, struct.pack("!H", SPORT + 1)), NO_MATCH)]))
    # cls_pmr_term_proto_ip :823-863 (v4 and v6)
    for v6 in (False, True):
        C.append((f"ipproto_v{6 if v6 else 4}", single(R.t_u8(R.PMR_IPPROTO, 17)),
                  [(create_packet(ipv6=v6, l4="udp"), MATCH),
                   (create_packet(ipv6=v6, l4="tcp"), NO_MATCH)]))
    # cls_pmr_term_dscp_ip :865-906, DSCP_CLASS4 = 0x20, mask 0x3f
    for v6 in (False, True):
        C.append((f"dscp_v{6 if v6 else 4}", single(R.t_u8(R.PMR_IP_DSCP, 0x20, 0x3f)),
                  [(create_packet(ipv6=v6, l4="udp", dscp=0x20), MATCH),
                   (create_packet(ipv6=v6, l4="udp", dscp=0), NO_MATCH)]))
    # cls_pmr_term_dmac :908-978
    dm = bytes([0x99, 0xaa, 0xbb, 0xcc, 0xdd, 0xee])
    C.append(("dmac", single((R.PMR_DMAC, dm, b"\xff" * 6, 0)),
              [(create_packet(dmac=dm), MATCH), (create_packet(), NO_MATCH)]))
    # cls_pmr_term_packet_len :980-1011 (val 1024, mask 0xff00)
    big = create_packet(l4="udp", extra_len=1024)
    C.append(("packet_len", single(R.t_len(1024, 0xff00)),
              [(big, MATCH), (create_packet(), NO_MATCH)]))
    # cls_pmr_term_vlan_id_0 :1013-1046 (0x123, mask 0xfff)
    C.append(("vlan_id_0", single(R.t_be16(R.PMR_VLAN_ID_0, 0x123, 0xfff)),
              [(create_packet(vlan=True, tci0=0x123), MATCH), (create_packet(), NO_MATCH)]))
    # cls_pmr_term_vlan_id_x :1048-1094 (0x345, mask 0xfff): single tag, qinq inner, none
    C.append(("vlan_id_x", single(R.t_be16(R.PMR_VLAN_ID_X, 0x345, 0xfff)),
              [(create_packet(vlan=True, tci0=0x345), MATCH),
               (create_packet(vlan=True, qinq=True, tci1=0x345), MATCH),
               (create_packet(), NO_MATCH)]))
    # cls_pmr_term_vlan_pcp_0 :1096-1132 (pcp 5, mask 0x7); NO_MATCH packet has tci 0
    C.append(("vlan_pcp_0", single(R.t_u8(R.PMR_VLAN_PCP_0, 5, 0x7)),
              [(create_packet(vlan=True, tci0=(5 << 13) | 0x123), MATCH),
               (create_packet(vlan=True), NO_MATCH)]))
    # cls_pmr_term_eth_type_0 :1134-1162
    C.append(("eth_type_0", single(R.t_be16(R.PMR_ETHTYPE_0, pg.ETH_IPV6)),
              [(create_packet(ipv6=True), MATCH), (create_packet(), NO_MATCH)]))
    # cls_pmr_term_eth_type_x :1164-1210
    C.append(("eth_type_x", single(R.t_be16(R.PMR_ETHTYPE_X, pg.ETH_IPV4)),
              [(create_packet(vlan=True, tci0=0x123), MATCH),
               (create_packet(vlan=True, qinq=True, tci1=0x123), MATCH),
               (create_packet(), NO_MATCH)]))
    # test_pmr_term_ipv4_addr :1351-1395: rule 10.0.0.88/32 (SIP) or
    # 10.0.0.99/32 (DIP); the MATCH packet carries both addresses (src
    # 10.0.0.88, dst 10.0.0.99, :1380-1382), the NO_MATCH packet the defaults
    for dst in (False, True):
        term = R.PMR_DIP_ADDR if dst else R.PMR_SIP_ADDR
        a = "10.0.0.99" if dst else "10.0.0.88"
        pk = create_packet(src="10.0.0.88", dst="10.0.0.99")
        C.append((f"ipv4_{'d' if dst else 's'}addr", single(R.t_ip4(term, a, 32)),
                  [(pk, MATCH), (create_packet(), NO_MATCH)]))
    # cls_pmr_term_ipv6daddr / saddr :1407-1476 (mask: last 6 bytes)
    m6 = bytes(10) + b"\xff" * 6
    d6 = bytes(10) + b"\xff\xff" + bytes([10, 1, 1, 100])
    s6 = bytes(10) + b"\xff\xff" + bytes([10, 1, 1, 1])
    C.append(("ipv6_daddr", single((R.PMR_DIP6_ADDR, d6, m6, 0)),
              [(create_packet(ipv6=True, dst=d6), MATCH), (create_packet(ipv6=True), NO_MATCH)]))
    C.append(("ipv6_saddr", single((R.PMR_SIP6_ADDR, s6, m6, 0)),
              [(create_packet(ipv6=True, src=s6), MATCH), (create_packet(ipv6=True), NO_MATCH)]))
    # test_pmr_term_custom :1488-1544 (FRAME offset 26 SIP 10.0.8.0/24, L3 offset 16 DIP 10.0.9.0/24)
    cm = create_packet(src="10.0.8.88", dst="10.0.9.99")
    C.append(("custom_frame", single(R.t_custom(R.PMR_CUSTOM_FRAME, 26, pg.ip4("10.0.8.0"),
                                                b"\xff\xff\xff\x00")),
              [(cm, MATCH), (create_packet(), NO_MATCH)]))
    C.append(("custom_l3", single(R.t_custom(R.PMR_CUSTOM_L3, 16, pg.ip4("10.0.9.0"),
                                             b"\xff\xff\xff\x00")),
              [(cm, MATCH), (create_packet(), NO_MATCH)]))
    # test_pmr_term_ipsec_spi_ah / _esp :2020-2110: value be32(0x11223344);
    # the NO_MATCH packet carries the raw value + 1
    val = struct.pack("!I", 0x11223344)
    val1 = struct.pack("<I", struct.unpack("<I", val)[0] + 1)
    for v6 in (False, True):
        for kind in ("ah", "esp"):
            C.append((f"ipsec_spi_{kind}_v{6 if v6 else 4}",
                      single((R.PMR_IPSEC_SPI, val, b"\xff" * 4, 0)),
                      [(create_packet(ipv6=v6, l4=kind, spi=val), MATCH),
                       (create_packet(ipv6=v6, l4=kind, spi=val1), NO_MATCH)]))
    return C


def chain_cases():
    """Chains, marks, error and drop CoS."""
    C = []
    # configure_cls_pmr_chain / test_cls_pmr_chain, odp_classification_tests.c:320-458:
    # default -(SIP 10.0.0.5)-> src -(UDP dport 3000)-> dst
    prog = [R.cos("default", queue=1), R.cos("src", queue=2), R.cos("dst", queue=3),
            ("default", 0),
            ("pmr", [R.t_ip4(R.PMR_SIP_ADDR, "10.0.0.5", 32)], 0, 1, 0),
            ("pmr", [R.t_be16(R.PMR_UDP_DPORT, 3000)], 1, 2, 0)]
    C.append(("pmr_chain", prog,
              [(create_packet(l4="udp", src="10.0.0.5", dport=3000), 2),
               (create_packet(l4="udp", src="10.0.0.5", dport=3001), 1),
               (create_packet(l4="udp", dport=3000), 0)]))
    # test_pmr_series, odp_classification_test_pmr.c:1554-1731: default -(DIP)-> ip
    # -(UDP dport i)-> udp[i], with marks
    prog = [R.cos("default", queue=1), R.cos("ip", queue=2)] + \
        [R.cos(f"udp{i}", queue=10 + i) for i in range(4)] + [("default", 0),
         ("pmr", [R.t_ip4(R.PMR_DIP_ADDR, "10.0.0.100", 24)], 0, 1, 0x100)]
    for i in range(4):
        prog.append(("pmr", [R.t_be16(R.PMR_UDP_DPORT, 5000 + i)], 1, 2 + i, 1000 + i))
    C.append(("pmr_series_marks", prog,
              [(create_packet(l4="udp", dport=5000 + i), 2 + i) for i in range(4)] +
              [(create_packet(l4="udp", dport=6000), 1)]))
    # error CoS via bad IPv4 version (odp_classification_tests.c:747-851)
    bad = bytearray(create_packet(l4="udp"))
    bad[14] = 0x55
    prog = [R.cos("default", queue=1), R.cos("err", queue=2), ("default", 0), ("error", 1)]
    C.append(("error_cos", prog, [(bytes(bad), 1), (create_packet(l4="udp"), 0)]))
    # drop CoS (odp_classification_tests.c:600-666, CLS_DROP_PORT 4001)
    prog = [R.cos("default", queue=1), R.cos("drop", action=1), ("default", 0),
            ("pmr", [R.t_be16(R.PMR_UDP_DPORT, 4001)], 0, 1, 0)]
    C.append(("drop_cos", prog, [(create_packet(l4="udp", dport=4001), 1),
                                 (create_packet(l4="udp"), 0)]))
    return C
