"""Rule programs and the BASELINE.json workloads.

A *rule program* is a list of control-plane operations, replayed in order
against an ODP classification API implementation (the product in
``odp_amd.cls`` or the CPU oracle in ``oracle/oracle.py``):

    ("cos", name, {"action": 0|1, "queue": int, "num_queue": int,
                   "hash_proto": bits, "stats": 0|1})     -> appends a CoS ref
    ("pmr", [term, ...], src_ref, dst_ref, mark)            -> appends a PMR ref
    ("pmr_destroy", pmr_ref)
    ("cos_destroy", cos_ref)
    ("default", cos_ref | None)
    ("error", cos_ref | None)

A term is ``(odp_cls_pmr_term_t, value: bytes, mask: bytes, offset)``; value
and mask are the bytes the application would point ``match.value`` /
``match.mask`` at (network order for protocol fields, CPU order for
ODP_PMR_LEN -- classification.h:55-137).

Refs are indices into the program's own CoS / PMR lists, so one program
drives both implementations identically (the same sequence of
odp_cls_cos_create / odp_cls_pmr_create calls the example application makes,
example/classifier/odp_classifier.c:570-742).
"""
from __future__ import annotations

import struct

import numpy as np

from . import pktgen as pg

# odp_cls_pmr_term_t (include/odp/api/spec/classification.h:55-137)
PMR_LEN, PMR_ETHTYPE_0, PMR_ETHTYPE_X, PMR_VLAN_ID_0, PMR_VLAN_ID_X, PMR_VLAN_PCP_0, \
    PMR_DMAC, PMR_IPPROTO, PMR_IP_DSCP, PMR_UDP_DPORT, PMR_TCP_DPORT, PMR_UDP_SPORT, \
    PMR_TCP_SPORT, PMR_SIP_ADDR, PMR_DIP_ADDR, PMR_SIP6_ADDR, PMR_DIP6_ADDR, \
    PMR_IPSEC_SPI, PMR_LD_VNI, PMR_CUSTOM_FRAME, PMR_CUSTOM_L3, PMR_IGMP_GRP_ADDR, \
    PMR_ICMP_ID, PMR_ICMP_TYPE, PMR_ICMP_CODE, PMR_SCTP_SPORT, PMR_SCTP_DPORT, \
    PMR_GTPV1_TEID = range(28)
PMR_INNER_HDR_OFF = 32

# odp_pktin_hash_proto_t bits (packet_io_types.h:124-146)
HP_IPV4_UDP, HP_IPV4_TCP, HP_IPV4, HP_IPV6_UDP, HP_IPV6_TCP, HP_IPV6 = (1 << i for i in range(6))

# result outcomes (include/mi_cls.h)
OUT_ENQ, OUT_COS_DROP, OUT_DISCARD, OUT_PARSE_DROP, OUT_LOOP = range(5)

RESULT_DTYPE = np.dtype([("in_flags", "<u4"), ("err", "u1"), ("outcome", "u1"), ("cos", "u1"),
                         ("hops", "u1"), ("queue", "<u2"), ("mark", "<u2"),
                         ("l3_offset", "<u2"), ("l4_offset", "<u2")])
assert RESULT_DTYPE.itemsize == 16


# ----------------------------------------------------------------- term helpers
def t_be16(term, v, m=0xFFFF):
    return (term, struct.pack("!H", v), struct.pack("!H", m), 0)


def t_u8(term, v, m=0xFF):
    return (term, bytes([v]), bytes([m]), 0)


def t_ip4(term, addr, plen):
    if isinstance(addr, str):
        addr = pg.ip4(addr)
    m = (0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF if plen else 0
    return (term, bytes(addr), struct.pack("!I", m), 0)


def t_ip6(term, addr, plen):
    if isinstance(addr, str):
        addr = pg.ip6(addr)
    m = ((1 << 128) - 1) ^ ((1 << (128 - plen)) - 1) if plen else 0
    return (term, bytes(addr), m.to_bytes(16, "big"), 0)


def t_len(v, m=0xFFFFFFFF):
    return (PMR_LEN, struct.pack("<I", v), struct.pack("<I", m), 0)


def t_custom(term, offset, value: bytes, mask: bytes):
    return (term, value, mask, offset)


def cos(name, queue=1, action=0, num_queue=1, hash_proto=0, stats=0):
    return ("cos", name, {"action": action, "queue": queue, "num_queue": num_queue,
                          "hash_proto": hash_proto, "stats": stats})


def cos_count(prog):
    return sum(1 for op in prog if op[0] == "cos")


def rule_count(prog):
    return sum(1 for op in prog if op[0] == "pmr")


# ------------------------------------------------------------------ workloads
def _u32(a, b, c, d):
    return (a << 24) | (b << 16) | (c << 8) | d


def config1(n=10_000):
    """BASELINE config 1: example/classifier over loopback, n x 64 B IPv4/UDP,
    1 SIP_ADDR /24 rule (10.10.10.0/24 -> queue1), SIP 50 % inside the prefix
    (as udp64.pcap: 10.10.10.1 vs 10.1.1.1, pktio_env:21-23)."""
    rng = np.random.default_rng(pg.seed_for(1))
    inside = rng.random(n) < 0.5
    sip = np.where(inside, _u32(10, 10, 10, 0) | rng.integers(1, 255, n),
                   _u32(10, 1, 1, 0) | rng.integers(1, 255, n)).astype(np.uint64)
    lens = np.full(n, 60)
    b = pg.build_batch(lens, ipver=np.full(n, 4), l4proto=np.full(n, pg.IPPROTO_UDP), sip4=sip,
                       dip4=np.full(n, _u32(10, 1, 1, 2), np.uint64),
                       sport=np.full(n, 39996), dport=np.full(n, 39997), seed=1)
    prog = [cos("DefaultCos", queue=1), cos("queue1", queue=2), ("default", 0),
            ("pmr", [t_ip4(PMR_SIP_ADDR, "10.10.10.0", 24)], 0, 1, 0)]
    return b, prog


def config2(n=1_000_000, tree=False, rank=0):
    """BASELINE config 2: n x 64 B IPv4/UDP, SIP uniform over 32 /24 prefixes
    10.0.0.0-10.0.31.0; 16 SIP_ADDR /24 rules (10.0.0.0-10.0.15.0).
    ``tree=False``: flat list of 16 PMRs on the default CoS (raised per-CoS
    limit); ``tree=True``: the stock-limit shape, 8 + 8 under two /21
    aggregates (same CoS for every packet)."""
    rng = np.random.default_rng(pg.seed_for(2) + 7919 * rank)
    sip = (_u32(10, 0, 0, 0) | (rng.integers(0, 32, n) << 8) | rng.integers(1, 255, n)).astype(
        np.uint64)
    dip = (_u32(192, 168, 0, 0) | rng.integers(0, 65536, n)).astype(np.uint64)
    lens = np.full(n, 60)
    b = pg.build_batch(lens, ipver=np.full(n, 4), l4proto=np.full(n, pg.IPPROTO_UDP), sip4=sip,
                       dip4=dip, sport=rng.integers(1024, 65535, n),
                       dport=rng.integers(1024, 65535, n), seed=2 + rank)
    prog = [cos("default", queue=1)]
    for i in range(16):
        prog.append(cos(f"p{i}", queue=100 + i))
    prog.append(("default", 0))
    if not tree:
        for i in range(16):
            prog.append(("pmr", [t_ip4(PMR_SIP_ADDR, _u32(10, 0, i, 0).to_bytes(4, "big"), 24)],
                         0, 1 + i, 0))
    else:
        prog.append(cos("agg0", queue=200))
        prog.append(cos("agg1", queue=201))
        prog.append(("pmr", [t_ip4(PMR_SIP_ADDR, "10.0.0.0", 21)], 0, 17, 0))
        prog.append(("pmr", [t_ip4(PMR_SIP_ADDR, "10.0.8.0", 21)], 0, 18, 0))
        for i in range(16):
            prog.append(("pmr", [t_ip4(PMR_SIP_ADDR, _u32(10, 0, i, 0).to_bytes(4, "big"), 24)],
                         17 + i // 8, 1 + i, 0))
    return b, prog


def _l34_rules(num_rules, num_dst, rng):
    """num_rules 2-3-term IPv4 PMRs over {SIP/DIP /24, IPPROTO, dport}."""
    rules = []
    for i in range(num_rules):
        use_dip = (i % 3) == 2
        net = _u32(10, 1 + (i >> 8), i & 0xFF, 0)
        proto = pg.IPPROTO_TCP if i % 5 == 0 else pg.IPPROTO_UDP
        terms = [t_ip4(PMR_DIP_ADDR if use_dip else PMR_SIP_ADDR, net.to_bytes(4, "big"), 24),
                 t_u8(PMR_IPPROTO, proto)]
        dport = None
        if i % 2 == 0:
            dport = 1000 + i
            terms.append(t_be16(PMR_TCP_DPORT if proto == pg.IPPROTO_TCP else PMR_UDP_DPORT, dport))
        rules.append(dict(terms=terms, dip=use_dip, net=net, proto=proto, dport=dport,
                          dst=1 + (i % num_dst)))
    return rules


def _target_fields(rules, n, rng, hit_frac, sizes):
    """Per-packet IPv4 fields: hit_frac of packets target a random rule."""
    tgt = rng.integers(0, len(rules), n)
    hit = rng.random(n) < hit_frac
    sip = (_u32(172, 16, 0, 0) | rng.integers(0, 65536, n)).astype(np.uint64)
    dip = (_u32(192, 168, 0, 0) | rng.integers(0, 65536, n)).astype(np.uint64)
    proto = np.where(rng.random(n) < 0.8, pg.IPPROTO_UDP, pg.IPPROTO_TCP)
    dport = rng.integers(20000, 65535, n)
    nets = np.array([r["net"] for r in rules], np.uint64)
    isdip = np.array([r["dip"] for r in rules])
    protos = np.array([r["proto"] for r in rules])
    dports = np.array([r["dport"] if r["dport"] is not None else -1 for r in rules])
    host = rng.integers(1, 255, n).astype(np.uint64)
    h = np.nonzero(hit)[0]
    t = tgt[h]
    sip[h] = np.where(isdip[t], sip[h], nets[t] | host[h])
    dip[h] = np.where(isdip[t], nets[t] | host[h], dip[h])
    proto[h] = protos[t]
    dport[h] = np.where(dports[t] >= 0, dports[t], dport[h])
    return sip, dip, proto, dport


def config3(n=1_000_000, num_rules=256, size="imix", rank=0, sctp_frac=0.0):
    """BASELINE config 3: n IMIX (60/566/1514 B, 7:4:1, shuffled) IPv4 packets,
    80 % UDP / 20 % TCP; num_rules 2-3-term PMRs over {SIP/DIP prefix,
    IPPROTO, UDP/TCP dport} on the default CoS; ~30 % match nothing.
    sctp_frac > 0 turns that fraction of the packets into SCTP (the
    checksum-validation bench's SCTP line)."""
    rng = np.random.default_rng(pg.seed_for(3) + 7919 * rank)
    rules = _l34_rules(num_rules, 32, rng)
    lens = pg.imix_lens(rng, n) if size == "imix" else np.full(n, int(size))
    sip, dip, proto, dport = _target_fields(rules, n, rng, 0.7, lens)
    if sctp_frac > 0:
        proto = np.where(rng.random(n) < sctp_frac, pg.IPPROTO_SCTP, proto)
    b = pg.build_batch(lens, ipver=np.full(n, 4), l4proto=proto, sip4=sip, dip4=dip,
                       sport=rng.integers(1024, 65535, n), dport=dport, seed=3 + rank)
    prog = [cos("default", queue=1)] + [cos(f"c{i}", queue=100 + i) for i in range(32)]
    prog.append(("default", 0))
    for r in rules:
        prog.append(("pmr", r["terms"], 0, r["dst"], 0))
    return b, prog


def config4(n=1_000_000, num_rules=1024, rank=0):
    """BASELINE config 4 (one GPU's shard): IMIX, 70 % IPv4 / 30 % IPv6;
    num_rules PMRs: 70 % IPv4 L3+L4 rules, 30 % SIP6/DIP6 /64 (+ dport) rules."""
    rng = np.random.default_rng(pg.seed_for(4) + 7919 * rank)
    rng_rules = np.random.default_rng(pg.seed_for(4))
    n4r = int(num_rules * 0.7)
    rules4 = _l34_rules(n4r, 48, rng_rules)
    rules6 = []
    for i in range(num_rules - n4r):
        pfx = bytes([0x20, 0x01, 0x0d, 0xb8, (i >> 8) & 0xFF, i & 0xFF, 0, 0])
        use_dst = i % 2 == 1
        terms = [t_ip6(PMR_DIP6_ADDR if use_dst else PMR_SIP6_ADDR, pfx + bytes(8), 64)]
        dport = None
        if i % 3 == 0:
            dport = 3000 + i
            terms.append(t_be16(PMR_UDP_DPORT, dport))
        rules6.append(dict(terms=terms, pfx=pfx, dst6=use_dst, dport=dport, dst=49 + (i % 16)))
    lens = pg.imix_lens(rng, n)
    ipver = np.where(rng.random(n) < 0.7, 4, 6)
    sip, dip, proto, dport = _target_fields(rules4, n, rng, 0.7, lens)
    # IPv6 fields
    sip6 = np.zeros((n, 16), np.uint8)
    dip6 = np.zeros((n, 16), np.uint8)
    sip6[:, :4] = [0x20, 0x01, 0x0d, 0xb8]
    dip6[:, :4] = [0x20, 0x01, 0x0d, 0xb8]
    sip6[:, 4:] = rng.integers(0, 256, (n, 12))
    dip6[:, 4:] = rng.integers(0, 256, (n, 12))
    sip6[:, 4] |= 0x80   # background: outside every rule prefix
    dip6[:, 4] |= 0x80
    six = np.nonzero(ipver == 6)[0]
    hit = six[rng.random(six.size) < 0.7]
    tg = rng.integers(0, len(rules6), hit.size)
    for j, (pi, ti) in enumerate(zip(hit, tg)):
        r = rules6[ti]
        arr = dip6 if r["dst6"] else sip6
        arr[pi, :8] = np.frombuffer(r["pfx"], np.uint8)
        if r["dport"] is not None:
            dport[pi] = r["dport"]
    proto6 = np.where(ipver == 6, pg.IPPROTO_UDP, proto)
    lens = np.where((ipver == 6) & (lens < 78), 78, lens)
    b = pg.build_batch(lens, ipver=ipver, l4proto=proto6, sip4=sip, dip4=dip, sip6=sip6,
                       dip6=dip6, sport=rng.integers(1024, 65535, n), dport=dport, seed=4 + rank)
    prog = [cos("default", queue=1)] + [cos(f"c{i}", queue=100 + i) for i in range(64)]
    prog.append(("default", 0))
    for r in rules4 + rules6:
        prog.append(("pmr", r["terms"], 0, r["dst"], 0))
    return b, prog


def config5(n=1_000_000, rank=0):
    """BASELINE config 5: VLAN-tagged IMIX (802.1Q, 10 % QinQ), 3-level CoS
    tree: VLAN_ID_0 (16) -> SIP / SIP6 prefix (16 per VLAN) -> L4 dport
    (3824 rules over 128 prefix CoS); 4096 PMRs in all."""
    rng = np.random.default_rng(pg.seed_for(5) + 7919 * rank)
    prog = [cos("default", queue=1)]
    vl = [len(prog) + i for i in range(16)]
    prog += [cos(f"vlan{i}", queue=200 + i) for i in range(16)]
    pc = [len(prog) + i for i in range(128)]
    prog += [cos(f"pfx{i}", queue=300 + i) for i in range(128)]
    lc = [len(prog) + i for i in range(32)]
    prog += [cos(f"leaf{i}", queue=500 + i, action=1 if i == 31 else 0) for i in range(32)]
    prog.append(("default", 0))
    vids = [100 + 7 * i for i in range(16)]
    for i in range(16):
        prog.append(("pmr", [t_be16(PMR_VLAN_ID_0, vids[i], 0x0FFF)], 0, vl[i], 0))
    pfx_of = {}
    for v in range(16):
        for p in range(16):
            k = v * 16 + p
            if p < 12:
                net = _u32(10, 20 + v, p * 16, 0)
                t = t_ip4(PMR_SIP_ADDR, net.to_bytes(4, "big"), 20)
                pfx_of[(v, p)] = ("v4", net)
            else:
                a = bytes([0x20, 0x01, 0x0d, 0xb8, v, p, 0, 0]) + bytes(8)
                t = t_ip6(PMR_SIP6_ADDR, a, 48)
                pfx_of[(v, p)] = ("v6", a)
            prog.append(("pmr", [t], vl[v], pc[k % 128], 0))
    port_rules = {}
    for c in range(128):
        cnt = 30 if c < 112 else 29
        port_rules[c] = []
        for j in range(cnt):
            dport = 4000 + 37 * j + c
            mark = (c * 64 + j) & 0xFFFF
            prog.append(("pmr", [t_be16(PMR_UDP_DPORT if j % 4 else PMR_TCP_DPORT, dport)],
                         pc[c], lc[(c + j) % 32], mark))
            port_rules[c].append((dport, pg.IPPROTO_TCP if j % 4 == 0 else pg.IPPROTO_UDP))
    # traffic
    lens = pg.imix_lens(rng, n)
    ntags = np.where(rng.random(n) < 0.1, 2, 1)
    hit = rng.random(n) < 0.8
    v = rng.integers(0, 16, n)
    p = rng.integers(0, 16, n)
    vid0 = np.where(hit, np.array(vids)[v], 3000 + rng.integers(0, 64, n))
    vid1 = rng.integers(1, 4095, n)
    ipver = np.where(p < 12, 4, 6)
    ipver = np.where(hit, ipver, np.where(rng.random(n) < 0.8, 4, 6))
    sip4 = (_u32(172, 16, 0, 0) | rng.integers(0, 65536, n)).astype(np.uint64)
    dip4 = (_u32(192, 168, 0, 0) | rng.integers(0, 65536, n)).astype(np.uint64)
    sip6 = rng.integers(0, 256, (n, 16)).astype(np.uint8)
    sip6[:, 0] = 0xfd
    dip6 = rng.integers(0, 256, (n, 16)).astype(np.uint8)
    proto = np.where(rng.random(n) < 0.8, pg.IPPROTO_UDP, pg.IPPROTO_TCP)
    dport = rng.integers(20000, 65535, n)
    hi = np.nonzero(hit)[0]
    pj = rng.integers(0, 30, n)
    for i in hi:
        kind, net = pfx_of[(int(v[i]), int(p[i]))]
        if kind == "v4":
            sip4[i] = net | int(rng.integers(0, 4096))
        else:
            sip6[i, :6] = np.frombuffer(net[:6], np.uint8)
        c = (int(v[i]) * 16 + int(p[i])) % 128
        pr = port_rules[c]
        if rng.random() < 0.9:
            dp, pt = pr[int(pj[i]) % len(pr)]
            dport[i] = dp
            proto[i] = pt
    lens = np.where((ipver == 6) & (lens < 86), 86, lens)
    b = pg.build_batch(lens, ipver=ipver, l4proto=proto, sip4=sip4, dip4=dip4, sip6=sip6,
                       dip6=dip6, sport=rng.integers(1024, 65535, n), dport=dport, ntags=ntags,
                       vid0=vid0, vid1=vid1, seed=5 + rank)
    return b, prog


def _acl_fields(rules, n, rng, hit_frac, lens):
    """Per-packet IPv4 fields for rule sets with arbitrary constraints: each
    rule is a dict of optional constraints sip / dip ((net, plen)), proto,
    dport, sport, dscp, len; hit_frac of the packets are built to satisfy a
    random rule's constraints (the fields it leaves open stay random, so a
    packet may match an earlier rule first -- first-match order decides)."""
    sip = (_u32(172, 16, 0, 0) | rng.integers(0, 65536, n)).astype(np.uint64)
    dip = (_u32(192, 168, 0, 0) | rng.integers(0, 65536, n)).astype(np.uint64)
    proto = np.where(rng.random(n) < 0.8, pg.IPPROTO_UDP, pg.IPPROTO_TCP)
    dport = rng.integers(20000, 65535, n)
    sport = rng.integers(1024, 65535, n)
    dscp = rng.integers(0, 64, n)
    lens = lens.copy()
    hit = np.nonzero(rng.random(n) < hit_frac)[0]
    tgt = rng.integers(0, len(rules), hit.size)
    host = rng.integers(0, 1 << 16, hit.size).astype(np.uint64)
    for i, t, h in zip(hit, tgt, host):
        r = rules[t]
        for key, arr in (("sip", sip), ("dip", dip)):
            if key in r:
                net, plen = r[key]
                arr[i] = net | (int(h) & ((1 << (32 - plen)) - 1))
        if "proto" in r:
            proto[i] = r["proto"]
        for key, arr in (("dport", dport), ("sport", sport), ("dscp", dscp), ("len", lens)):
            if key in r:
                arr[i] = r[key]
    return sip, dip, proto, dport, sport, dscp, lens


def _acl_terms(r):
    terms = []
    for key, kind in (("sip", PMR_SIP_ADDR), ("dip", PMR_DIP_ADDR)):
        if key in r:
            net, plen = r[key]
            terms.append(t_ip4(kind, net.to_bytes(4, "big"), plen))
    if "proto" in r:
        terms.append(t_u8(PMR_IPPROTO, r["proto"]))
    tcp = r.get("proto") == pg.IPPROTO_TCP
    if "dport" in r:
        terms.append(t_be16(PMR_TCP_DPORT if tcp else PMR_UDP_DPORT, r["dport"]))
    if "sport" in r:
        terms.append(t_be16(PMR_TCP_SPORT if tcp else PMR_UDP_SPORT, r["sport"]))
    if "dscp" in r:
        terms.append(t_u8(PMR_IP_DSCP, r["dscp"], 0x3F))
    if "len" in r:
        terms.append(t_len(r["len"]))
    return terms


def _acl_batch(rules, n, rng, rank, seed, num_dst=32):
    lens = pg.imix_lens(rng, n)
    sip, dip, proto, dport, sport, dscp, lens = _acl_fields(rules, n, rng, 0.7, lens)
    b = pg.build_batch(lens, ipver=np.full(n, 4), l4proto=proto, sip4=sip, dip4=dip,
                       sport=sport, dport=dport, tos=dscp << 2, seed=seed + rank)
    prog = [cos("default", queue=1)] + [cos(f"c{i}", queue=100 + i) for i in range(num_dst)]
    prog.append(("default", 0))
    for i, r in enumerate(rules):
        prog.append(("pmr", _acl_terms(r), 0, 1 + i % num_dst, 0))
    return b, prog


def config3_nested(n=1_000_000, rank=0, scale=1):
    """Config 3 traffic (IMIX IPv4, 70 % aimed at a rule) under an ACL with
    overlapping rules: 256 PMRs over nested SIP / DIP prefixes, longest
    first -- 128 /24s (with protocol, half with a destination port), 64 /20s
    over the same space (protocol only: wildcard ports) and 64 /16s (port
    only: wildcard protocol) -- so a packet's key values name several rules
    and first-match order decides (odp_classification.c:1624-1667; the
    overlapping-PMR series of odp_classification_test_pmr.c:1554-1731).
    scale=4: 1024 PMRs of the same shapes (past the 256 rules a wide bitmap
    block holds: candidate lists)."""
    rng = np.random.default_rng(pg.seed_for(3) + 31 + 7919 * rank)
    rules = []
    for k in range(128 * scale):
        r = {"dip" if k % 3 == 2 else "sip": (_u32(10, 1 + k // 256, k % 256, 0), 24),
             "proto": pg.IPPROTO_TCP if k % 5 == 0 else pg.IPPROTO_UDP}
        if k % 2 == 0:
            r["dport"] = 1000 + k
        rules.append(r)
    for j in range(64 * scale):
        rules.append({"sip" if j % 2 else "dip": (_u32(10, 1 + j // 64, 16 * (j % 16), 0), 20),
                      "proto": pg.IPPROTO_UDP if (j // 2) % 2 else pg.IPPROTO_TCP})
    for m in range(64 * scale):
        rules.append({"dip" if m % 2 else "sip": (_u32(10, 1 + m % (4 * scale), 0, 0), 16),
                      "dport": 2000 + m})
    return _acl_batch(rules, n, rng, rank, 31)


def config3_classes(n=1_000_000, rank=0):
    """Config 3 traffic under 256 PMRs spread over 9 key classes (SIP /24,
    DIP /24, SIP /16, DIP /16, IPPROTO, destination port, source port, DSCP,
    frame length) -- one more than a classification block holds, so the
    default CoS falls back to the linear scan."""
    rng = np.random.default_rng(pg.seed_for(3) + 37 + 7919 * rank)
    rules = []
    for i in range(256):
        k = i // 6
        t = i % 6
        if t == 0:
            r = {"sip": (_u32(10, 2, k, 0), 24), "proto": pg.IPPROTO_UDP, "dport": 3000 + k}
        elif t == 1:
            r = {"dip": (_u32(10, 3, k, 0), 24), "sport": 4000 + k}
        elif t == 2:
            r = {"sip": (_u32(10, 4 + k % 8, 0, 0), 16), "dscp": k % 64}
        elif t == 3:
            r = {"dip": (_u32(10, 12 + k % 8, 0, 0), 16), "proto": pg.IPPROTO_TCP,
                 "sport": 5000 + k}
        elif t == 4:
            r = {"dscp": (k * 7) % 64, "dport": 6000 + k}
        else:
            r = {"len": 566, "dport": 7000 + k}
        rules.append(r)
    return _acl_batch(rules, n, rng, rank, 37)


CONFIGS = {1: config1, 2: config2, 3: config3, 4: config4, 5: config5}
