"""Pin the CPU oracle to the reference's own fixtures and known answers.

* parser frames of test/common/test_packet_*.h with the has_*() assertions of
  test/validation/api/packet/packet.c:3745-4541 (tests/golden/parse_frames.json)
* example/classifier/udp64.pcap with the example's rule
  (platform/linux-generic/test/example/classifier/pktio_env:21-23)
* per-term MATCH / NO_MATCH, chains, marks, error and drop CoS of
  test/validation/api/classification/ (tests/refcases.py)
* the input_flags words and quirks the survey observed from the reference
  build
* the Toeplitz core against the published RSS verification vectors for the
  default 40-byte key (the key of odp_classification.c:50-58)
"""
import json
import os
import struct

import numpy as np
import pytest

from odp_amd import pktgen as pg
from odp_amd import rules as R
from tests import refcases as RC
from tests import zoo
from tests.helpers import oracle_run

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

FLAG_BITS = {"cls_mark": 0, "l2": 3, "l3": 4, "l4": 5, "eth": 6, "eth_bcast": 7, "eth_mcast": 8,
             "jumbo": 9, "vlan": 10, "vlan_qinq": 11, "arp": 12, "ipv4": 13, "ipv6": 14,
             "ip_bcast": 15, "ip_mcast": 16, "ipfrag": 17, "ipopt": 18, "ipsec": 19,
             "ipsec_ah": 20, "ipsec_esp": 21, "udp": 22, "tcp": 23, "sctp": 24, "icmp": 25,
             "no_next_hdr": 26}


def parse(frame):
    from oracle.oracle import parse as p
    return p(frame)


def _parse_frames():
    with open(os.path.join(GOLDEN, "parse_frames.json")) as f:
        return json.load(f)["frames"]


@pytest.mark.parametrize("name", sorted(_parse_frames()))
def test_parser_frames(built, name):
    d = _parse_frames()[name]
    ret, flags, err, l2, l3, l4 = parse(bytes.fromhex(d["frame"]))
    assert ret == d["ret"], (name, ret)
    assert err == 0
    for flag, want in d["expect"].items():
        have = (flags >> FLAG_BITS[flag]) & 1
        assert have == want, f"{name}: {flag} = {have}, packet.c:{d['packet_c_line']} wants {want}"


def test_udp64_example_split(built):
    with open(os.path.join(GOLDEN, "udp64.json")) as f:
        d = json.load(f)
    b = pg.batch_from_frames([bytes.fromhex(h) for h in d["frames"]])
    prog = [R.cos("DefaultCos", queue=1), R.cos("queue1", queue=2), ("default", 0),
            ("pmr", [R.t_ip4(R.PMR_SIP_ADDR, "10.10.10.0", 24)], 0, 1, 0)]
    r, _ = oracle_run(prog, b, (64, 256, 8))
    c = np.bincount(r["cos"], minlength=2)
    assert c[1] >= d["expect_min"]["queue1"] and c[0] >= d["expect_min"]["DefaultCos"]
    assert c.sum() == 200


def test_observed_input_flag_words(built):
    """words observed from the reference build."""
    assert parse(pg.udp4_frame())[1] == 0x402078
    assert parse(pg.udp4_frame(frag=0x2000))[1] == 0x422078
    assert parse(pg.udp6_frame())[1] == 0x404078
    hbh = pg.eth(ethtype=pg.ETH_IPV6) + pg.ipv6(next_hdr=0, payload_len=64) + \
        pg.ipv6_ext(pg.IPPROTO_UDP) + pg.udp(5, 6, 56)
    assert parse(pg.pad_to(hbh, 120))[1] == 0x444078
    q1 = pg.udp4_frame(tags=(1,), tpids=[pg.ETH_QINQ], size=64)
    assert parse(q1)[1] == 0x402c78
    bad = pg.pad_to(pg.eth() + pg.ipv4(ver=5, payload_len=8) + pg.udp(), 60)
    r, f, e, l2, l3, l4 = parse(bad)
    assert (r, f, e, l4) == (1, 0x2058, 0x02, 0xFFFF)
    # marked match: cls_mark bit set (0x402079)
    b = pg.batch_from_frames([pg.udp4_frame()])
    res, _ = oracle_run([R.cos("d", queue=1), R.cos("m", queue=2), ("default", 0),
                         ("pmr", [R.t_u8(R.PMR_IPPROTO, 17)], 0, 1, 5)], b)
    assert res["in_flags"][0] == 0x402079 and res["mark"][0] == 5


def test_appendix_a_quirks(built):
    one = lambda prog, frame: oracle_run(prog, pg.batch_from_frames([frame]))[0][0]  # noqa: E731
    E = pg.eth()
    # item 6: tot_len = 20 with a UDP header still parses UDP and matches a dport rule
    f = pg.pad_to(E + pg.ipv4(tot_len=20) + pg.udp(1234, 2048), 60)
    r = one(zoo.prog_single(R.t_be16(R.PMR_UDP_DPORT, 2048)), f)
    assert r["cos"] == 1 and r["l4_offset"] == 34
    # item 7: non-first fragment payload bytes 2-3 = 0x0800 match UDP_DPORT 2048
    f = pg.pad_to(E + pg.ipv4(frag=10, payload_len=26) + struct.pack("!HH", 7, 0x0800) +
                  bytes(22), 60)
    assert one(zoo.prog_single(R.t_be16(R.PMR_UDP_DPORT, 2048)), f)["cos"] == 1
    # item 15: single-tag 0x88A8 frame: ETHTYPE_X compares bytes 20-21 (IPv4 header)
    f = pg.udp4_frame(tags=(0x123,), tpids=[pg.ETH_QINQ], size=64)
    assert one(zoo.prog_single(R.t_be16(R.PMR_ETHTYPE_X, pg.ETH_IPV4)), f)["cos"] == 0
    assert one(zoo.prog_single(R.t_be16(R.PMR_ETHTYPE_X, struct.unpack("!H", f[20:22])[0])),
               f)["cos"] == 1
    # item 16: 2-byte CUSTOM_FRAME at offset 58 misses a 60 B frame, hits 61 B
    base = pg.udp4_frame(size=60)
    prog = zoo.prog_single(R.t_custom(R.PMR_CUSTOM_FRAME, 58, base[58:60], b"\xff\xff"))
    assert one(prog, base)["cos"] == 0
    assert one(prog, base + b"\x00")["cos"] == 1
    # item 9: IPv6+HBH(8)+UDP: payload_len 16 -> ip_err -> error CoS; 64 -> l4 = 62
    for plen, want in ((16, "err"), (64, "ok")):
        f = pg.pad_to(pg.eth(ethtype=pg.ETH_IPV6) + pg.ipv6(next_hdr=0, payload_len=plen) +
                      pg.ipv6_ext(pg.IPPROTO_UDP) + pg.udp(5, 6, 8), 120)
        r = one([R.cos("d", queue=1), R.cos("e", queue=2), ("default", 0), ("error", 1)], f)
        if want == "err":
            assert r["cos"] == 1 and r["err"] == 0x02
        else:
            assert r["cos"] == 0 and r["l4_offset"] == 62
    # item 10: tot_len 26 in a 40 B frame -> parse -1 (drop); tot_len too big -> ip_err
    assert parse((E + pg.ipv4(tot_len=26) + bytes(6))[:40])[0] == -1
    assert parse(pg.pad_to(E + pg.ipv4(tot_len=200) + pg.udp(), 60))[2] == 0x02


@pytest.mark.parametrize("case", RC.term_cases() + RC.chain_cases(), ids=lambda c: c[0])
def test_reference_known_answers(built, case):
    name, prog, pkts = case
    b = pg.batch_from_frames([f for f, _ in pkts])
    r, _ = oracle_run(prog, b)
    assert list(r["cos"]) == [e for _, e in pkts], name


def test_pmr_series_marks(built):
    """test_pmr_series (odp_classification_test_pmr.c:1668-1702): the mark of
    the last matched PMR is delivered."""
    name, prog, pkts = [c for c in RC.chain_cases() if c[0] == "pmr_series_marks"][0]
    b = pg.batch_from_frames([f for f, _ in pkts])
    r, _ = oracle_run(prog, b)
    assert list(r["mark"]) == [1000, 1001, 1002, 1003, 0x100]
    assert all(r["in_flags"] & 1)


def test_swap_on_delete_order(built):
    """odp_cls_pmr_destroy moves the last PMR into the freed slot
    (odp_classification.c:782-786): scan order changes."""
    f = pg.udp4_frame(sport=1024, dport=2048)
    prog = [R.cos("d", queue=1), R.cos("a", queue=2), R.cos("b", queue=3), R.cos("c", queue=4),
            ("default", 0),
            ("pmr", [R.t_u8(R.PMR_IPPROTO, 99)], 0, 1, 0),          # never matches
            ("pmr", [R.t_be16(R.PMR_UDP_DPORT, 2048)], 0, 2, 0),
            ("pmr", [R.t_be16(R.PMR_UDP_SPORT, 1024)], 0, 3, 0)]
    b = pg.batch_from_frames([f])
    assert oracle_run(prog, b)[0]["cos"][0] == 2
    # destroying PMR 0 moves the sport rule (last) in front of the dport rule
    assert oracle_run(prog + [("pmr_destroy", 0)], b)[0]["cos"][0] == 3


def test_destroyed_default_cos_still_used(built):
    """cls_select_cos (:1712-1719): an invalid default CoS is not descended
    but is still returned."""
    b = pg.batch_from_frames([pg.udp4_frame()])
    prog = [R.cos("d", queue=1), R.cos("x", queue=2), ("default", 0),
            ("pmr", [R.t_u8(R.PMR_IPPROTO, 17)], 0, 1, 0), ("cos_destroy", 0)]
    r = oracle_run(prog, b)[0][0]
    assert r["cos"] == 0 and r["outcome"] == R.OUT_ENQ and r["hops"] == 0


def test_toeplitz_published_vectors(built):
    """Microsoft RSS verification suite, default key (odp_classification.c:50-58)."""
    import ctypes as C
    from oracle.oracle import lib
    L = lib()

    def h(words):
        arr = (C.c_uint32 * len(words))(*words)
        return L.orc_softrss(arr, len(words))
    v4 = lambda a, b: [struct.unpack("!I", pg.ip4(a))[0], struct.unpack("!I", pg.ip4(b))[0]]  # noqa
    assert h(v4("66.9.149.187", "161.142.100.80")) == 0x323e8fc2
    assert h(v4("199.92.111.2", "65.69.140.83")) == 0xd718262a
    assert h(v4("66.9.149.187", "161.142.100.80") + [(2794 << 16) | 1766]) == 0x51ccc178
    v6 = list(struct.unpack("!8I", pg.ip6("3ffe:2501:200:1fff::7") + pg.ip6("3ffe:2501:200:3::1")))
    assert h(v6) == 0x2cc18cd5
