"""Oracle: pktin checksum validation and drop-on-error options
(odp_parse.c:112-173, 183-249, 256-356, 362-488; odp_packet.c:2065-2138).

Pinned by the reference's own test frames: every frame of
test/common/test_packet_{ipv4,ipv6,ipsec}.h carries valid checksums, and the
reference's pktio checksum tests (test/validation/api/pktio/pktio.c:
4569-4690) expect ODP_PACKET_CHKSUM_OK for such packets with
pktin.bit.{ipv4,udp,sctp}_chksum set.  Frames built here with checksums from
the protocol definitions (tests/chksum_frames.py), and bit-flipped copies,
pin the BAD verdicts.
"""
import numpy as np
import pytest

from odp_amd import pktgen as pg
from odp_amd import rules as R
from oracle import oracle as O
from tests import chksum_frames as CK
from tests import zoo


def status(flags, err, done_bit, err_bit):
    if not (flags >> done_bit) & 1:
        return None
    return bool(err & err_bit)


def test_reference_frames_checksums_ok():
    """test_packet_*.h frames: every checksum the options validate is OK,
    and nothing else changes."""
    seen = 0
    for name, fr in zoo.golden_frames():
        r0, f0, e0, _, l30, l40 = O.parse(fr, 0)
        r, f, e, _, l3, l4 = O.parse(fr, CK.ALL_CK)
        assert (r, e, l3, l4) == (r0, e0, l30, l40), name
        assert f & ~(CK.L3_DONE | CK.L4_DONE) == f0, name
        l3s = status(f, e, 30, CK.E_L3CK)
        l4s = status(f, e, 31, CK.E_L4CK)
        assert l3s in (None, False) and l4s in (None, False), name
        if f0 & (1 << 13):   # IPv4: the header checksum is always checked
            assert l3s is False, name
        if (f0 & ((1 << 22) | (1 << 23) | (1 << 24))) and not (f0 & (1 << 17)):
            assert l4s is False, name   # UDP / TCP / SCTP, not a fragment
            seen += 1
    assert seen >= 12


def test_built_frames_verdicts():
    """Valid frames pass, bit-flipped IPv4 headers / L4 bytes fail; the UDP
    zero checksum passes on IPv4 and fails on IPv6."""
    for fr, l3_bad, l4_bad in CK.frame_set(seed=11, n=300):
        r, f, e, _, _, _ = O.parse(fr, CK.ALL_CK)
        assert status(f, e, 30, CK.E_L3CK) == l3_bad, fr.hex()
        assert status(f, e, 31, CK.E_L4CK) == l4_bad, fr.hex()
        if l3_bad:
            assert e & CK.E_IP and r == 1
        if l4_bad:
            assert r == 1


def test_checksum_options_independent():
    """Each option validates only its own protocol."""
    rng = np.random.default_rng(3)
    for proto, bit in ((pg.IPPROTO_UDP, CK.UDP_CK), (pg.IPPROTO_TCP, CK.TCP_CK),
                       (pg.IPPROTO_SCTP, CK.SCTP_CK)):
        fr, _, l4 = CK.build(rng, 4, proto)
        bad = CK.corrupt(rng, fr, l4, l4 + 4)
        for opt in (CK.UDP_CK, CK.TCP_CK, CK.SCTP_CK):
            r, f, e, _, _, _ = O.parse(bad, opt)
            if opt == bit:
                assert (f >> 31) & 1 and e & CK.E_L4CK and r == 1
            else:
                assert not (f >> 31) & 1 and e == 0 and r == 0


@pytest.mark.parametrize("proto,drop,ebit", [(pg.IPPROTO_UDP, CK.DROP_UDP, CK.E_UDP),
                                             (pg.IPPROTO_TCP, CK.DROP_TCP, CK.E_TCP),
                                             (pg.IPPROTO_SCTP, CK.DROP_SCTP, CK.E_SCTP)])
def test_drop_on_l4_checksum_error(proto, drop, ebit):
    rng = np.random.default_rng(5)
    fr, _, l4 = CK.build(rng, 6, proto)
    bad = CK.corrupt(rng, fr, l4, l4 + 4)
    r, _, e, _, _, _ = O.parse(bad, CK.ALL_CK)
    assert r == 1 and e & ebit and e & CK.E_L4CK
    r, _, e, _, _, _ = O.parse(bad, CK.ALL_CK | drop)
    assert r == -1
    assert O.parse(fr, CK.ALL_CK | drop)[0] == 0


def test_drop_on_ip_errors():
    """drop_ipv4_err / drop_ipv6_err drop any IP header error, checksum or
    not (odp_parse.c:383-396); the L4 part is never reached."""
    rng = np.random.default_rng(9)
    fr, l3, l4 = CK.build(rng, 4, pg.IPPROTO_UDP)
    bad = CK.corrupt(rng, fr, l3 + 12, l3 + 20)          # address bit: checksum error
    assert O.parse(bad, CK.IPV4_CK)[0] == 1
    r, f, e, _, _, l4o = O.parse(bad, CK.IPV4_CK | CK.DROP_V4)
    assert r == -1 and e & CK.E_IP and not f & (1 << 5) and l4o == 0xFFFF
    short = bytearray(fr)
    short[l3] = 0x44                                     # IHL 4: ip_err without checksums
    assert O.parse(bytes(short), CK.DROP_V4)[0] == -1
    assert O.parse(bytes(short), CK.DROP_V6)[0] == 1
    fr6, l36, _ = CK.build(rng, 6, pg.IPPROTO_UDP)
    b6 = bytearray(fr6)
    b6[l36] = 0x50                                       # version 5
    assert O.parse(bytes(b6), CK.DROP_V6)[0] == -1
    assert O.parse(bytes(b6), CK.DROP_V4)[0] == 1


def test_udp_length_error_drop():
    fr = pg.pad_to(pg.eth() + pg.ipv4(payload_len=8) + pg.udp(length=4), 60)
    r, _, e, _, _, _ = O.parse(fr, 0)
    assert r == 1 and e & CK.E_UDP
    assert O.parse(fr, CK.DROP_UDP)[0] == -1


def test_fragments_skip_l4_checksum():
    rng = np.random.default_rng(13)
    fr, l3, l4 = CK.build(rng, 4, pg.IPPROTO_UDP)
    b = bytearray(fr)
    b[l3 + 6] = 0x20                                     # MF: first fragment
    b[l3 + 10:l3 + 12] = b"\x00\x00"
    b[l3 + 10:l3 + 12] = CK.inet_csum(bytes(b[l3:l4])).to_bytes(2, "big")
    bad = CK.corrupt(rng, bytes(b), l4 + 8, len(b)) if len(b) > l4 + 8 else bytes(b)
    r, f, e, _, _, _ = O.parse(bad, CK.ALL_CK)
    assert r == 0 and (f >> 30) & 1 and not (f >> 31) & 1 and e == 0


@pytest.mark.parametrize("ipver", [4, 6])
def test_pktgen_set_checksums_all_ok(ipver):
    """pktgen.set_checksums (the checksum bench's input) writes valid IPv4,
    UDP, TCP and SCTP checksums: with every pktin checksum and drop option
    set, the oracle validates every packet and reports no error; the SCTP
    CRC also equals the independent RFC 4960 construction here."""
    rng = np.random.default_rng(5 + ipver)
    n = 600
    lens = pg.imix_lens(rng, n)
    lens[:4] = [61, 567, 1513, 99]              # odd lengths
    proto = rng.choice([pg.IPPROTO_UDP, pg.IPPROTO_TCP, pg.IPPROTO_SCTP], n)
    kw = dict(sip4=rng.integers(0, 2**32, n).astype(np.uint64),
              dip4=rng.integers(0, 2**32, n).astype(np.uint64)) if ipver == 4 else dict(
        sip6=rng.integers(0, 256, (n, 16), dtype=np.uint8),
        dip6=rng.integers(0, 256, (n, 16), dtype=np.uint8))
    b = pg.build_batch(lens, ipver=np.full(n, ipver), l4proto=proto,
                       sport=rng.integers(1, 65535, n), dport=rng.integers(1, 65535, n),
                       seed=9, **kw)
    pg.set_checksums(b)
    o = O.Oracle(pktin_opt=CK.ALL_CK | CK.ALL_DROP)
    o.apply([R.cos("d", queue=1), ("default", 0)])
    r = o.classify(b)
    assert (r["err"] == 0).all()
    assert ((r["in_flags"] >> 31) & 1).all()                  # every L4 checksum validated
    assert ((r["in_flags"] >> 30) & 1).all() == (ipver == 4)  # IPv4 header checksums
    for i in np.nonzero(proto == pg.IPPROTO_SCTP)[0][:20]:
        f = bytearray(b.frame(i))
        l4 = 14 + (20 if ipver == 4 else 40)
        want = int.from_bytes(f[l4 + 8: l4 + 12], "little")
        f[l4 + 8: l4 + 12] = b"\0\0\0\0"
        assert (~CK.crc32c(bytes(f[l4:]))) & 0xFFFFFFFF == want
