"""pktin checksum validation and drop-on-error options on the GPU
(mi_cls_pktin_opt_set / odp_amd_cls_pktin_opt_set) vs the CPU oracle: every
result record bit-identical, for valid and corrupted IPv4 / IPv6 / UDP /
TCP / SCTP frames, the parser zoo and its fuzzed mutations, unaligned frame
offsets and IMIX traffic (whole-frame L4 sums up to 1514 B)."""
import numpy as np
import pytest

from odp_amd import pktgen as pg
from odp_amd import rules as R
from tests import chksum_frames as CK
from tests import zoo
from tests.helpers import assert_same, gpu_run, oracle_run

pytestmark = pytest.mark.gpu

OPTS = {
    "all_ck": CK.ALL_CK,
    "all_ck_drop": CK.ALL_CK | CK.ALL_DROP,
    "ipv4_ck": CK.IPV4_CK,
    "drop_only": CK.ALL_DROP,
    "udp_ck_drop": CK.UDP_CK | CK.DROP_UDP,
    "sctp_tcp_ck": CK.SCTP_CK | CK.TCP_CK,
}


def both(prog, batch, opt, what):
    got = gpu_run(prog, batch, pktin_opt=opt)
    exp, _ = oracle_run(prog, batch, pktin_opt=opt)
    assert_same(got, exp, batch, what)
    return got


def _frames(seed):
    rng = np.random.default_rng(seed)
    base = [f for _, f in zoo.all_frames()]
    fr = [f for f, _, _ in CK.frame_set(seed=seed, n=300)]
    return fr + base + zoo.mutate_frames(rng, base + fr, 1500)


@pytest.mark.parametrize("name", sorted(OPTS))
def test_checksum_options_zoo(built, gpu, name):
    b = pg.batch_from_frames(_frames(21))
    got = both(zoo.prog_everything(), b, OPTS[name], name)
    if OPTS[name] & CK.ALL_CK:
        assert (got["in_flags"] >> 30).any()   # some checksum was validated


@pytest.mark.parametrize("name", ["all_ck", "all_ck_drop"])
def test_checksum_verdicts_vs_construction(built, gpu, name):
    """GPU verdicts equal the verdicts known by construction."""
    fs = CK.frame_set(seed=31, n=200)
    b = pg.batch_from_frames([f for f, _, _ in fs])
    got = both([R.cos("d", queue=1), ("default", 0)], b, OPTS[name], name)
    for i, (_, l3_bad, l4_bad) in enumerate(fs):
        fl, err = int(got["in_flags"][i]), int(got["err"][i])
        l3 = None if not (fl >> 30) & 1 else bool(err & CK.E_L3CK)
        l4 = None if not (fl >> 31) & 1 else bool(err & CK.E_L4CK)
        if int(got["outcome"][i]) == R.OUT_PARSE_DROP:
            continue
        assert l3 == l3_bad and l4 == l4_bad, i


def test_checksum_unaligned_offsets(built, gpu):
    frames = _frames(41)
    rng = np.random.default_rng(8)
    lens = np.array([len(f) for f in frames], np.int64)
    off = np.zeros(len(frames), np.int64)
    pos = 1
    for i, f in enumerate(frames):
        off[i] = pos
        pos += len(f) + int(rng.integers(0, 40))
    buf = np.zeros(pos + 64, np.uint8)
    for o, f in zip(off, frames):
        buf[o: o + len(f)] = np.frombuffer(f, np.uint8)
    b = pg.Batch(buf, off.astype(np.uint32), lens.astype(np.uint16))
    both(zoo.prog_everything(), b, CK.ALL_CK | CK.ALL_DROP, "unaligned")


@pytest.mark.parametrize("cfg", [3, 4, 5])
def test_checksum_imix_configs(built, gpu, cfg):
    """IMIX traffic up to 1514 B (the generator leaves checksums zero, so
    the IPv4 headers fail and UDP zero checksums take the parse_udp rule)."""
    b, prog = R.CONFIGS[cfg](20_000)
    both(prog, b, CK.ALL_CK, f"config {cfg}")
    both(prog, b, CK.UDP_CK | CK.TCP_CK | CK.SCTP_CK | CK.ALL_DROP, f"config {cfg} l4")


@pytest.mark.parametrize("ipver", [4, 6])
def test_checksum_valid_mixed_lengths(built, gpu, ipver):
    """Valid UDP / TCP / SCTP checksums (pktgen.set_checksums) over IMIX,
    odd and jumbo (up to 9000 B: hundreds of 16-B pieces spread over many
    rounds of the wave-cooperative sum) lengths, then a payload byte flipped
    in every 7th frame: GPU == oracle, and the verdicts are the constructed
    ones (only the flipped frames fail)."""
    rng = np.random.default_rng(40 + ipver)
    n = 6000
    lens = pg.imix_lens(rng, n)
    pick = rng.random(n)
    lens = np.where(pick < 0.05, rng.integers(1515, 9001, n), lens)
    lens = np.where((pick > 0.5) & (pick < 0.6), rng.integers(61, 1514, n), lens)
    proto = rng.choice([pg.IPPROTO_UDP, pg.IPPROTO_TCP, pg.IPPROTO_SCTP], n)
    kw = dict(sip4=rng.integers(0, 2**32, n).astype(np.uint64),
              dip4=rng.integers(0, 2**32, n).astype(np.uint64)) if ipver == 4 else dict(
        sip6=rng.integers(0, 256, (n, 16), dtype=np.uint8),
        dip6=rng.integers(0, 256, (n, 16), dtype=np.uint8))
    b = pg.build_batch(lens, ipver=np.full(n, ipver), l4proto=proto,
                       sport=rng.integers(1, 65535, n), dport=rng.integers(1, 65535, n),
                       seed=11, **kw)
    pg.set_checksums(b)
    l4 = 14 + (20 if ipver == 4 else 40)
    bad = np.zeros(n, bool)
    for i in range(0, n, 7):
        o, ln = int(b.off[i]), int(b.len[i])
        if ln > l4 + 20:   # a payload byte (never a checksum field)
            b.buf[o + int(rng.integers(l4 + 20, ln))] ^= 0x5A
            bad[i] = True
    prog = [R.cos("d", queue=1), ("default", 0)]
    got = both(prog, b, CK.ALL_CK, f"valid ipv{ipver}")
    l4_err = (got["err"] & CK.E_L4CK) != 0
    assert ((got["in_flags"] >> 31) & 1).all()
    assert np.array_equal(l4_err, bad)
    both(prog, b, CK.ALL_CK | CK.ALL_DROP, f"valid ipv{ipver} drop")


def test_sctp_crc_long_frames(built, gpu):
    """SCTP CRC-32C on both paths: frames up to 16 KB of L4 bytes (the
    wave-cooperative CRC over 64-B pieces) and longer ones (one lane per
    frame), valid and with one flipped byte, at odd lengths and unaligned
    piece boundaries: GPU == oracle, verdicts as constructed."""
    rng = np.random.default_rng(77)
    lens = np.array([60, 98, 99, 1514, 9001, 16400, 16417, 16418, 20000, 40001, 65535, 131] * 6)
    n = lens.size
    b = pg.build_batch(lens, ipver=np.full(n, 4), l4proto=np.full(n, pg.IPPROTO_SCTP),
                       sip4=rng.integers(0, 2**32, n).astype(np.uint64),
                       dip4=rng.integers(0, 2**32, n).astype(np.uint64),
                       sport=rng.integers(1, 65535, n), dport=rng.integers(1, 65535, n), seed=5)
    pg.set_checksums(b)
    bad = np.zeros(n, bool)
    for i in range(0, n, 2):
        o, ln = int(b.off[i]), int(b.len[i])
        if ln > 34 + 20:
            b.buf[o + int(rng.integers(34 + 12, ln))] ^= 0x81
            bad[i] = True
    got = both([R.cos("d", queue=1), ("default", 0)], b, CK.SCTP_CK, "sctp long")
    assert ((got["in_flags"] >> 31) & 1).all()
    assert np.array_equal((got["err"] & CK.E_L4CK) != 0, bad)


@pytest.mark.parametrize("ipver", [4, 6])
def test_sctp_crc_every_piece_split(built, gpu, ipver):
    """SCTP CRC-32C at every L4 length from 12 to 395 bytes: no full 64-B
    piece (the checksum field in the owner's partial piece), one to six full
    pieces with partial pieces of every size 0..63; valid, and with the
    checksum's last byte flipped in every 3rd frame: GPU == oracle, verdicts
    as constructed."""
    rng = np.random.default_rng(90 + ipver)
    l4 = 14 + (20 if ipver == 4 else 40)
    lens = np.arange(l4 + 12, l4 + 396)
    n = lens.size
    kw = dict(sip4=rng.integers(0, 2**32, n).astype(np.uint64),
              dip4=rng.integers(0, 2**32, n).astype(np.uint64)) if ipver == 4 else dict(
        sip6=rng.integers(0, 256, (n, 16), dtype=np.uint8),
        dip6=rng.integers(0, 256, (n, 16), dtype=np.uint8))
    b = pg.build_batch(lens, ipver=np.full(n, ipver), l4proto=np.full(n, pg.IPPROTO_SCTP),
                       sport=rng.integers(1, 65535, n), dport=rng.integers(1, 65535, n), seed=9,
                       **kw)
    pg.set_checksums(b)
    bad = np.zeros(n, bool)
    for i in range(0, n, 3):
        b.buf[int(b.off[i]) + l4 + 11] ^= 0x01   # the CRC field's last byte
        bad[i] = True
    got = both([R.cos("d", queue=1), ("default", 0)], b, CK.SCTP_CK, f"sctp splits ipv{ipver}")
    assert ((got["in_flags"] >> 31) & 1).all()
    assert np.array_equal((got["err"] & CK.E_L4CK) != 0, bad)


@pytest.mark.parametrize("name", ["all_ck", "all_ck_drop", "ipv4_ck", "sctp_tcp_ck"])
@pytest.mark.parametrize("cfg", [3, 2])
def test_specialised_option_kernel(built, gpu, name, cfg):
    """With pktin options on, a flat program gets the option kernel with its
    block compiled in (spec_setup: the checksum instantiation): the same
    records as the oracle on the zoo, the checksum frames and the config's
    own traffic; turning the options off again specialises the plain kernel."""
    from odp_amd.cls import Classifier
    b0, prog = R.CONFIGS[cfg](3000)
    pg.set_checksums(b0)
    frames = [b0.frame(i) for i in range(b0.n)] + _frames(5)
    b = pg.batch_from_frames(frames)
    exp, _ = oracle_run(prog, b, pktin_opt=OPTS[name])
    c = Classifier(gpu=0)
    try:
        c.apply(prog)
        c.set_pktin_opt(OPTS[name])
        assert c.spec_wait() == 0
        got = c.classify(b)
        ll = c.last_launch()
        assert ll["ck"] and ll["specialised"], ll
        assert_same(got, exp, b, f"config {cfg} {name} (specialised option kernel)")
        c.set_pktin_opt(0)
        assert c.spec_wait() == 0
        got0 = c.classify(b)
        ll = c.last_launch()
        assert not ll["ck"] and ll["specialised"], ll
        exp0, _ = oracle_run(prog, b)
        assert_same(got0, exp0, b, f"config {cfg} options off")
    finally:
        c.close()
