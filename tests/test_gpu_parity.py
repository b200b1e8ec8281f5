"""HIP path (libmi_cls.so via the libodp_cls.so C ABI) vs the CPU oracle.

Bar: every 16-byte result record (input flags, error bits, outcome, CoS,
queue slot, mark, l3/l4 offsets) bit-identical to the oracle on the same
seeded inputs.
"""
import numpy as np
import pytest

from odp_amd import cls
from odp_amd import pktgen as pg
from odp_amd import rules as R
from tests import refcases as RC
from tests import zoo
from tests.helpers import assert_same, gpu_run, oracle_run, summary

pytestmark = pytest.mark.gpu


ENGINE_ENV = {
    "auto": {},
    "linear": {"MI_CLS_NO_BV": "1"},   # linear scan everywhere
    "nodiv": {"MI_CLS_DIV": "0"},      # no per-lane bit-vector rounds (CoS waterfall)
    "div": {"MI_CLS_DIV": "1"},        # per-lane bit-vector rounds even for flat programs
    "wpb4": {"MI_CLS_WPB": "4"},       # 4-wave blocks (own hot-region copy or HBM)
    "wpb16": {"MI_CLS_WPB": "16"},     # one 16-wave block per CU sharing the LDS copy
    "nowide": {"MI_CLS_NO_WIDE": "1"},  # candidate lists instead of wide bitmap rows
    "nocand1": {"MI_CLS_NO_CAND1": "1"},   # no single-candidate engine (wide / lists)
    "noportmerge": {"MI_CLS_NO_PORTMERGE": "1"},   # separate UDP / TCP port classes
    "noflat": {"MI_CLS_NO_FLAT": "1"},   # general kernel for flat programs too
    "spec": {},                          # program-specialised kernel (waited for)
    "nojit": {"MI_CLS_JIT": "0"},        # no specialised kernels
    "nojoint": {"MI_CLS_NO_JOINT": "1"},   # no joint direct tables for tree levels
}


def both(prog, batch, limits=(255, 8192, 4096), what="", engine="auto"):
    """engine "auto": bit-vector blocks where a CoS has <= 8 key classes,
    linear scan otherwise, per-lane rounds for CoS trees; the other engines
    force one of the kernel's paths (ENGINE_ENV)."""
    import os
    keys = ("MI_CLS_NO_BV", "MI_CLS_DIV", "MI_CLS_WPB", "MI_CLS_NO_WIDE", "MI_CLS_NO_CAND1",
            "MI_CLS_NO_PORTMERGE", "MI_CLS_NO_FLAT", "MI_CLS_JIT", "MI_CLS_NO_JOINT")
    old = {k: os.environ.pop(k, None) for k in keys}
    os.environ.update(ENGINE_ENV[engine])
    try:
        got = gpu_run(prog, batch, limits, spec=engine == "spec")
    finally:
        for k in keys:
            os.environ.pop(k, None)
            if old[k] is not None:
                os.environ[k] = old[k]
    exp, _ = oracle_run(prog, batch, limits)
    assert_same(got, exp, batch, f"{what} [{engine}]")
    return got


def test_udp64_example(built, gpu):
    b = pg.batch_from_frames(zoo.udp64_frames())
    prog = [R.cos("DefaultCos", queue=1), R.cos("queue1", queue=2), ("default", 0),
            ("pmr", [R.t_ip4(R.PMR_SIP_ADDR, "10.10.10.0", 24)], 0, 1, 0)]
    got = both(prog, b, (64, 256, 8), "udp64")
    c = np.bincount(got["cos"], minlength=2)
    # platform/linux-generic/test/example/classifier/pktio_env:21-23
    assert c[0] >= 100 and c[1] >= 100


def test_zoo_no_rules(built, gpu):
    b, _ = zoo.zoo_batch()
    both([R.cos("d", queue=1), ("default", 0)], b, what="zoo/no rules")


@pytest.mark.parametrize("engine", ["auto", "linear"])
@pytest.mark.parametrize("name,term", zoo.term_examples(), ids=[n for n, _ in zoo.term_examples()])
def test_zoo_each_term(built, gpu, name, term, engine):
    b, names = zoo.zoo_batch()
    got = both(zoo.prog_single(term, mark=7), b, what=name, engine=engine)
    assert got.shape[0] == len(names)


def test_zoo_everything(built, gpu):
    b, _ = zoo.zoo_batch()
    got = both(zoo.prog_everything(), b, what="everything")
    s = summary(got)
    assert s["enq"] > 0 and s["cos_drop"] > 0 and s["parse_drop"] > 0


def test_zoo_deletes(built, gpu):
    b, _ = zoo.zoo_batch()
    both(zoo.prog_deletes(), b, what="deletes")


def test_zoo_loop(built, gpu):
    b, _ = zoo.zoo_batch()
    got = both(zoo.prog_loop(), b, what="loop")
    assert summary(got)["loop"] > 0


def test_zoo_no_default(built, gpu):
    b, _ = zoo.zoo_batch()
    got = both(zoo.prog_no_default(), b, what="no default")
    s = summary(got)
    assert s["discard"] > 0 and s["cos_drop"] > 0


@pytest.mark.parametrize("engine", ["auto", "linear", "nodiv", "div", "wpb16", "nowide", "nocand1",
                                    "noportmerge", "noflat", "spec", "nojit", "nojoint"])
@pytest.mark.parametrize("seed", range(12))
def test_random_programs_fuzz(built, gpu, seed, engine):
    rng = np.random.default_rng(1000 + seed)
    frames = [f for _, f in zoo.all_frames()]
    fr = frames + zoo.mutate_frames(rng, frames, 3000)
    b = pg.batch_from_frames(fr)
    prog = zoo.random_program(rng, frames, n_cos=int(rng.integers(3, 40)),
                              n_rules=int(rng.integers(5, 200)),
                              max_kinds=None if seed % 2 else 6)
    both(prog, b, what=f"fuzz seed {seed}", engine=engine)


@pytest.mark.parametrize("engine", ["auto", "linear", "nodiv", "wpb4", "wpb16", "nowide", "nocand1",
                                    "noportmerge", "noflat", "spec", "nojit", "nojoint"])
@pytest.mark.parametrize("cfg,n", [(1, 10_000), (2, 100_000), (3, 50_000), (4, 50_000),
                                   (5, 20_000)])
def test_configs_small(built, gpu, cfg, n, engine):
    b, prog = R.CONFIGS[cfg](n)
    got = both(prog, b, what=f"config {cfg}", engine=engine)
    assert summary(got)["enq"] > 0


@pytest.mark.parametrize("engine", ["auto", "nowide", "div", "nocand1", "noflat", "spec"])
@pytest.mark.parametrize("num_rules", [33, 64, 100, 200, 255, 256, 257])
def test_wide_rule_counts(built, gpu, num_rules, engine):
    """Rule counts around the wide-bitmap engine's word boundaries (33..256
    rules on one CoS) and just past it (257: candidate lists)."""
    b, prog = R.config3(20_000, num_rules=num_rules, size=60)
    both(prog, b, what=f"{num_rules} rules", engine=engine)


def _joint_tree(rng, n, leaf_kind):
    """Default CoS -> 6 VLAN_ID_0 rules -> 6 mid CoS; each mid CoS's rules
    share one class (so the mid level is a joint direct group): 12 rules of
    leaf_kind each to 24 leaf CoS (marks); half the traffic hits."""
    prog = [R.cos("default", queue=1)]
    mids = list(range(1, 7))
    prog += [R.cos(f"mid{i}", queue=10 + i) for i in range(6)]
    leaves = list(range(7, 31))
    prog += [R.cos(f"leaf{i}", queue=50 + i, action=1 if i == 23 else 0) for i in range(24)]
    prog.append(("default", 0))
    vids = [200 + 3 * i for i in range(6)]
    for i in range(6):
        prog.append(("pmr", [R.t_be16(R.PMR_VLAN_ID_0, vids[i], 0x0FFF)], 0, mids[i], 0))
    vals = {}
    for i in range(6):
        for j in range(12):
            if leaf_kind == "dport":
                v = 5000 + 11 * j + i
                t = R.t_be16(R.PMR_UDP_DPORT if j % 3 else R.PMR_TCP_DPORT, v)
            elif leaf_kind == "dip":
                v = (10 << 24) | (i << 16) | (j << 8) | 7
                t = R.t_ip4(R.PMR_DIP_ADDR, v.to_bytes(4, "big"), 32)
            else:   # sip6 /64
                v = bytes([0x20, 0x01, 0x0d, 0xb8, 0, i, 0, j]) + bytes(8)
                t = R.t_ip6(R.PMR_SIP6_ADDR, v, 64)
            vals[(i, j)] = v
            prog.append(("pmr", [t], mids[i], leaves[(i * 12 + j) % 24], (i * 16 + j) & 0xFFFF))
    hit = rng.random(n) < 0.5
    i = rng.integers(0, 6, n)
    j = rng.integers(0, 12, n)
    ipver = np.full(n, 6 if leaf_kind == "sip6" else 4)
    proto = np.where(j % 3 == 0, pg.IPPROTO_TCP, pg.IPPROTO_UDP)
    dport = np.where(hit & (leaf_kind == "dport"), 5000 + 11 * j + i, rng.integers(1, 65535, n))
    dip4 = np.where(hit & (leaf_kind == "dip"), (10 << 24) | (i << 16) | (j << 8) | 7,
                    rng.integers(0, 2 ** 32, n)).astype(np.uint64)
    sip6 = rng.integers(0, 256, (n, 16)).astype(np.uint8)
    if leaf_kind == "sip6":
        for k in np.nonzero(hit)[0]:
            sip6[k, :8] = np.frombuffer(vals[(int(i[k]), int(j[k]))][:8], np.uint8)
    vid0 = np.where(rng.random(n) < 0.9, np.array(vids)[i], 999)
    b = pg.build_batch(np.where(rng.random(n) < 0.7, 60, 300), ipver=ipver, l4proto=proto,
                       sip4=rng.integers(0, 2 ** 32, n).astype(np.uint64), dip4=dip4, sip6=sip6,
                       dip6=rng.integers(0, 256, (n, 16)).astype(np.uint8),
                       sport=rng.integers(1, 65535, n), dport=dport,
                       ntags=np.where(rng.random(n) < 0.2, 2, 1), vid0=vid0,
                       vid1=rng.integers(1, 4095, n), seed=7)
    return b, prog


@pytest.mark.parametrize("engine", ["auto", "nojoint", "wpb4", "linear", "spec", "nojit"])
@pytest.mark.parametrize("leaf_kind", ["dport", "dip", "sip6"])
def test_joint_direct_tree_levels(built, gpu, leaf_kind, engine):
    """A tree level whose CoS all key on one class is one joint direct group
    (one-word keys with the CoS slot in free bits for merged ports, the slot
    appended for a /32 DIP and a two-word SIP6 /64 key): every record
    bit-exact against the oracle, with and without joint tables."""
    rng = np.random.default_rng({"dport": 1, "dip": 2, "sip6": 3}[leaf_kind])
    b, prog = _joint_tree(rng, 30_000, leaf_kind)
    got = both(prog, b, what=f"joint {leaf_kind}", engine=engine)
    s = summary(got)
    assert s["enq"] > 0 and s["cos_drop"] > 0


def _joint_bitmap_tree(rng, n, pair):
    """Default CoS -> 6 VLAN_ID_0 rules -> 6 mid CoS; every mid CoS has 10
    rules over the same two key classes (a joint bitmap group): some rules
    constrain one class, some both, in a different order per CoS, with
    repeated values, so first-match order matters.  pair = the second class:
    "dport" (merged UDP/TCP ports, one-word key, CoS slot in free bits) or
    "sip6" (SIP6 /48, a two-word key: the slot appended)."""
    prog = [R.cos("default", queue=1)]
    mids = list(range(1, 7))
    prog += [R.cos(f"mid{i}", queue=10 + i) for i in range(6)]
    leaves = list(range(7, 27))
    prog += [R.cos(f"leaf{i}", queue=50 + i, action=1 if i == 19 else 0) for i in range(20)]
    prog.append(("default", 0))
    vids = [300 + 5 * i for i in range(6)]
    for i in range(6):
        prog.append(("pmr", [R.t_be16(R.PMR_VLAN_ID_0, vids[i], 0x0FFF)], 0, mids[i], 0))
    dips = [(10 << 24) | (k << 8) for k in range(5)]       # /24 prefixes
    seconds = list(range(4))
    rules = {}
    for i in range(6):
        rs = []
        for j in range(10):
            kind = (i + j) % 3   # 0: DIP only, 1: second only, 2: both
            d, q = int(rng.integers(0, 5)), int(rng.integers(0, 4))
            terms = []
            if kind in (0, 2):
                terms.append(R.t_ip4(R.PMR_DIP_ADDR, dips[d].to_bytes(4, "big"), 24))
            if kind in (1, 2):
                if pair == "dport":
                    terms.append(R.t_be16(R.PMR_UDP_DPORT if q % 2 else R.PMR_TCP_DPORT,
                                          7000 + 13 * q + i))
                else:
                    a6 = bytes([0x20, 0x01, 0x0d, 0xb8, i, q]) + bytes(10)
                    terms.append(R.t_ip6(R.PMR_SIP6_ADDR, a6, 48))
            prog.append(("pmr", terms, mids[i], leaves[(7 * i + j) % 20], (i * 32 + j) & 0xFFFF))
            rs.append((kind, d, q))
        rules[i] = rs
    i = rng.integers(0, 6, n)
    d = rng.integers(0, 6, n)          # 5: no DIP rule's prefix
    q = rng.integers(0, 5, n)          # 4: no second-class value
    ipver = np.full(n, 6 if pair == "sip6" else 4)
    proto = np.where(q % 2 == 1, pg.IPPROTO_UDP, pg.IPPROTO_TCP)
    dip4 = ((10 << 24) | (d << 8) | rng.integers(0, 256, n)).astype(np.uint64)
    dport = np.where(q < 4, 7000 + 13 * q + i, rng.integers(1, 65535, n))
    sip6 = rng.integers(0, 256, (n, 16)).astype(np.uint8)
    if pair == "sip6":
        sip6[:, :4] = [0x20, 0x01, 0x0d, 0xb8]
        sip6[:, 4] = i
        sip6[:, 5] = np.where(q < 4, q, 200)
    vid0 = np.where(rng.random(n) < 0.9, np.array(vids)[i], 999)
    b = pg.build_batch(np.where(rng.random(n) < 0.7, 60, 300), ipver=ipver, l4proto=proto,
                       sip4=rng.integers(0, 2 ** 32, n).astype(np.uint64), dip4=dip4, sip6=sip6,
                       dip6=rng.integers(0, 256, (n, 16)).astype(np.uint8),
                       sport=rng.integers(1, 65535, n), dport=dport,
                       ntags=np.where(rng.random(n) < 0.2, 2, 1), vid0=vid0,
                       vid1=rng.integers(1, 4095, n), seed=11)
    return b, prog


@pytest.mark.parametrize("engine", ["auto", "nojoint", "wpb4", "linear", "spec", "nojit"])
@pytest.mark.parametrize("pair", ["dport", "sip6"])
def test_joint_bitmap_tree_levels(built, gpu, pair, engine):
    """A tree level whose CoS have bitmap blocks over the same two classes
    is one joint bitmap group (per class one (key, CoS) table; the group's
    alive rows, miss rows and result arrays per CoS slot): every record
    bit-exact against the oracle, with and without joint tables.  (IPv6
    traffic for the SIP6 pair: the DIP class is then absent, the rules that
    need it never hold.)"""
    rng = np.random.default_rng({"dport": 21, "sip6": 22}[pair])
    b, prog = _joint_bitmap_tree(rng, 30_000, pair)
    c = cls.Classifier(gpu=0)
    try:
        c.apply(prog)
        info = c.program_info()
    finally:
        c.close()
    assert info["tree"] and info["bitmap"] == 6, info
    if engine == "auto":
        assert info["joint_bitmap"] == 6, info
    got = both(prog, b, what=f"joint bitmap {pair}", engine=engine)
    s = summary(got)
    assert s["enq"] > 0


def test_config2_tree_equals_flat(built, gpu):
    b, flat = R.config2(50_000)
    _, tree = R.config2(50_000, tree=True)
    g1 = both(flat, b, what="flat")
    g2 = both(tree, b, what="tree")
    # same terminal CoS per packet up to the CoS renumbering of the two shapes
    assert np.array_equal(g1["cos"] != 0, g2["cos"] != 0)


def test_unaligned_offsets(built, gpu):
    frames = [f for _, f in zoo.all_frames()]
    rng = np.random.default_rng(7)
    lens = np.array([len(f) for f in frames], np.int64)
    gaps = rng.integers(0, 40, len(frames))
    off = np.zeros(len(frames), np.int64)
    pos = 3
    for i, f in enumerate(frames):
        off[i] = pos
        pos += len(f) + int(gaps[i])
    buf = np.zeros(pos + 64, np.uint8)
    for o, f in zip(off, frames):
        buf[o: o + len(f)] = np.frombuffer(f, np.uint8)
    b = pg.Batch(buf, off.astype(np.uint32), lens.astype(np.uint16))
    both(zoo.prog_everything(), b, what="unaligned")


@pytest.mark.parametrize("n", [1, 63, 64, 65, 255, 256, 257, 1000])
def test_ragged_sizes(built, gpu, n):
    b, prog = R.config3(n, num_rules=64)
    both(prog, b, what=f"n={n}")


def test_empty_batch(built, gpu):
    import torch
    from odp_amd.cls import Classifier
    c = Classifier(gpu=0)
    c.apply([R.cos("d", queue=1), ("default", 0)])
    t = torch.zeros(16, dtype=torch.int32, device="cuda:0")
    assert c.classify_device(t.data_ptr(), t.data_ptr(), t.data_ptr(), 0, t.data_ptr()) == 0
    c.close()


def test_stats_per_hop(built, gpu):
    """CoS packet counters follow the reference's per-hop rule
    (odp_classification.c:1646-1647, 1721-1723)."""
    from odp_amd.cls import Classifier
    from oracle.oracle import Oracle
    b, _ = zoo.zoo_batch()
    prog = zoo.prog_everything()
    c = Classifier(gpu=0)
    cos, _ = c.apply(prog)
    c.classify(b)
    c.classify(b)
    o = Oracle()
    ocos, _ = o.apply(prog)
    o.classify(b)
    o.classify(b)
    for h, oh in zip(cos, ocos):
        if h:
            assert c.cos_stats_packets(h) == o.stats_packets(oh)
    c.close()


def test_rule_change_between_batches(built, gpu):
    """A control-plane change bumps the generation; the next batch uses the
    new snapshot."""
    from odp_amd.cls import Classifier
    from oracle.oracle import Oracle
    b, _ = zoo.zoo_batch()
    c = Classifier(gpu=0)
    o = Oracle()
    p1 = [R.cos("d", queue=1), R.cos("x", queue=2), ("default", 0),
          ("pmr", [R.t_u8(R.PMR_IPPROTO, 17)], 0, 1, 0)]
    c.apply(p1)
    o.apply(p1)
    assert_same(c.classify(b), o.classify(b), b, "gen1")
    c.L.odp_cls_pmr_destroy(c.pmr[0])
    o.L.orc_pmr_destroy(o.pmr[0])
    assert_same(c.classify(b), o.classify(b), b, "gen2")
    c.close()


def test_config3_full_size_properties(built, gpu):
    """Full BASELINE size (1 M IMIX, 256 rules): the oracle checks a 100 k
    slice bit-exactly; the whole batch is checked for size-independent
    properties (CoS histogram of a slice scales, every record well formed)."""
    b, prog = R.config3(1_000_000)
    got = gpu_run(prog, b)
    sl = b.slice(0, 100_000)
    exp, _ = oracle_run(prog, sl)
    assert_same(got[:100_000], exp, sl, "config3 slice")
    assert np.all(got["outcome"] == R.OUT_ENQ)
    assert np.all(got["l3_offset"] == 14) and np.all(got["l4_offset"] == 34)
    # determinism: a second run is identical
    assert np.array_equal(got, gpu_run(prog, b))


@pytest.mark.parametrize("spec", [False, True], ids=["generic", "spec"])
@pytest.mark.parametrize("cfg,kw", [(3, {}), (3, {"size": 60}), (4, {}), (5, {}), (2, {})],
                         ids=["config3_imix", "config3_64B", "config4", "config5", "config2"])
def test_configs_full_size(built, gpu, cfg, kw, spec):
    """BASELINE configs at full size (1 M packets: one GPU's shard for
    configs 4 and 5): every record bit-exact vs the multithreaded oracle,
    with the generic kernels (MI_CLS_JIT=0) and with the program-specialised
    kernel (waited for; config 5's is its tree plan)."""
    import os
    from oracle.oracle import Oracle
    b, prog = (R.config3(1_000_000, **kw) if cfg == 3 else R.CONFIGS[cfg](1_000_000))
    if not spec:
        os.environ["MI_CLS_JIT"] = "0"
    try:
        got = gpu_run(prog, b, spec=spec)
    finally:
        os.environ.pop("MI_CLS_JIT", None)
    o = Oracle()
    o.apply(prog)
    exp = o.classify(b, threads=16)
    assert_same(got, exp, b, f"config {cfg} {kw} full size")
    assert summary(got)["enq"] > 0


@pytest.mark.parametrize("case", RC.term_cases() + RC.chain_cases(), ids=lambda c: c[0])
def test_reference_known_answers_gpu(built, gpu, case):
    """The reference validation suite's MATCH / NO_MATCH expectations on the
    HIP path (odp_classification_test_pmr.c, odp_classification_tests.c)."""
    name, prog, pkts = case
    b = pg.batch_from_frames([f for f, _ in pkts])
    got = both(prog, b, what=name)
    assert list(got["cos"]) == [e for _, e in pkts]


def test_parser_frames_gpu(built, gpu):
    """Parser frames of test/common/test_packet_*.h: every flag word, error
    bit and offset equals the oracle's (which test_oracle_golden pins to
    packet.c's assertions)."""
    frames = zoo.golden_frames()
    b = pg.batch_from_frames([f for _, f in frames])
    got = both([R.cos("d", queue=1), ("default", 0)], b, what="parser frames")
    assert np.all(got["outcome"] == R.OUT_ENQ)


@pytest.mark.parametrize("four_terms", [False, True])
def test_single_candidate_record_forms(built, gpu, four_terms):
    """Single-candidate engine records: config 4's 1024 rules constrain at
    most 3 of their 7 key classes (compact 16-B records); one extra rule
    with 4 terms forces the full per-class layout.  Both == oracle."""
    from odp_amd.cls import Classifier
    b, prog = R.config4(30_000)
    if four_terms:
        terms = [R.t_ip4(R.PMR_SIP_ADDR, "10.1.5.0", 24), R.t_u8(R.PMR_IPPROTO, pg.IPPROTO_UDP),
                 R.t_be16(R.PMR_UDP_DPORT, 1010), R.t_ip4(R.PMR_DIP_ADDR, "192.168.0.0", 16)]
        at = next(i for i, op in enumerate(prog) if op[0] == "pmr") + 3
        prog = prog[:at] + [("pmr", terms, 0, 5, 9)] + prog[at:]
    c = Classifier(gpu=0)
    c.apply(prog)
    assert c.program_info()["cand1"] == 1
    c.close()
    both(prog, b, what=f"config4 four_terms={four_terms}")


@pytest.mark.parametrize("engine", ["auto", "spec", "nojit", "linear", "nowide", "nocand1"])
@pytest.mark.parametrize("name,make", [
    ("nested256", lambda n: R.config3_nested(n)),
    ("nested1024", lambda n: R.config3_nested(n, scale=4)),
    ("classes9", lambda n: R.config3_classes(n))], ids=["nested256", "nested1024", "classes9"])
def test_overlapping_acls(built, gpu, name, make, engine):
    """Rule sets with overlapping keys (nested prefixes, wildcard ports: the
    wide-bitmap and candidate-list engines) and with more key classes than a
    block holds (a chain of blocks): first-match order as the oracle."""
    b, prog = make(50_000)
    got = both(prog, b, what=name, engine=engine)
    assert summary(got)["enq"] > 0


def _shadow_prog(variant):
    """Rules that can never be the first holding rule beside rules that can
    (ADVICE r3): exact duplicates with different destinations and marks, a
    superset rule before and after its subset, and a rule without terms in
    the middle of the list; first match in scan order decides."""
    net = lambda a, p: R.t_ip4(R.PMR_SIP_ADDR, a, p)
    port = lambda v: R.t_be16(R.PMR_UDP_DPORT, v)
    prog = [R.cos("d", queue=1)] + [R.cos(f"c{i}", queue=10 + i) for i in range(8)]
    prog.append(("default", 0))
    rules = [
        ([net("10.0.0.0", 24), port(53)], 1, 11),
        ([net("10.0.0.0", 24), port(53)], 2, 12),          # exact duplicate: shadowed
        ([net("10.0.0.0", 24), port(53), R.t_u8(R.PMR_IPPROTO, 17)], 3, 13),   # superset after
        ([net("10.0.1.0", 24), port(80), R.t_u8(R.PMR_IPPROTO, 17)], 4, 14),   # superset before
        ([net("10.0.1.0", 24), port(80)], 5, 15),          # its subset, later
        ([net("10.0.2.0", 24)], 6, 16),
        ([], 7, 17) if variant == "wildcard_mid" else ([net("10.0.3.0", 24)], 7, 17),
        ([net("10.0.2.0", 24), port(443)], 8, 18),         # behind the /24 (shadowed)
        ([net("10.0.4.0", 24), port(8080)], 1, 19),
    ]
    for terms, dst, mark in rules:
        prog.append(("pmr", terms, 0, dst, mark))
    return prog


@pytest.mark.parametrize("engine", ["auto", "spec", "nocand1", "linear"])
@pytest.mark.parametrize("variant", ["plain", "wildcard_mid"])
def test_shadowed_rules_first_match(built, gpu, variant, engine):
    """First-match parity where block build drops shadowed rules (ADVICE r3:
    the engine-selection test alone did not pin which rule wins)."""
    rng = np.random.default_rng(77)
    n = 20_000
    nets = np.array([(10 << 24) | (k << 8) | 5 for k in range(6)], dtype=np.uint64)
    sip = nets[rng.integers(0, 6, n)]
    dport = np.array([53, 80, 443, 8080, 9])[rng.integers(0, 5, n)]
    proto = np.where(rng.random(n) < 0.8, pg.IPPROTO_UDP, pg.IPPROTO_TCP)
    b = pg.build_batch(np.full(n, 60), ipver=np.full(n, 4), l4proto=proto, sip4=sip,
                       dip4=rng.integers(0, 2 ** 32, n).astype(np.uint64), sport=np.full(n, 1000),
                       dport=dport, seed=3)
    got = both(_shadow_prog(variant), b, what=f"shadowed {variant}", engine=engine)
    # the wildcard rule in the middle takes every packet no earlier rule holds
    assert len(np.unique(got["cos"])) >= (4 if variant == "wildcard_mid" else 5)


def _under_root(prog, root_first=False):
    """The program one level down: a new root CoS becomes the default, its one
    rule (IPv4 ethertype) leads to the old default CoS -- a CoS tree whose
    second level holds the program's rules.  root_first: the root CoS's rule
    set also gets the program's rules (a tree whose default CoS has more key
    classes than a block holds)."""
    n = R.cos_count(prog)
    old = next(op[1] for op in prog if op[0] == "default")
    out = [op for op in prog if op[0] == "cos"] + [R.cos("root", queue=9), ("default", n)]
    out.append(("pmr", [R.t_be16(R.PMR_ETHTYPE_0, 0x0800)], n, old, 0))
    for op in prog:
        if op[0] == "pmr":
            out.append(op)
            if root_first and op[2] == old:
                out.append(("pmr", op[1], n, op[3], op[4]))
    return out


@pytest.mark.parametrize("root_first", [False, True], ids=["second_level", "default_cos"])
@pytest.mark.parametrize("engine", ["auto", "linear"])
def test_many_classes_in_tree(built, gpu, root_first, engine):
    """A CoS tree with a CoS whose rules span 9 key classes: tree programs
    build no chains of blocks (the tree kernels scan such a CoS linearly);
    first-match order and marks as the oracle, at the second level and on
    the default CoS."""
    from odp_amd.cls import Classifier
    b, prog = R.config3_classes(40_000)
    tprog = _under_root(prog, root_first)
    c = Classifier(gpu=0)
    c.apply(tprog)
    info = c.program_info()
    c.close()
    assert info["tree"] and info["chained"] == 0
    got = both(tprog, b, what=f"classes9 tree root_first={root_first}", engine=engine)
    assert summary(got)["enq"] > 0


def _far_l4_errors(n, stats):
    """Config 5 traffic (VLAN / QinQ, IPv4 / IPv6, TCP / UDP) with L4 header
    errors planted where their bytes lie past byte 64 -- IPv6 TCP data
    offsets (byte 70 / 74) and QinQ IPv6 UDP lengths (bytes 66-67) -- and on
    IPv4 frames, plus NAT-T destination ports (4500, marker at l4+8), under
    config 5's tree with an error CoS (and per-CoS counters when `stats`)."""
    from odp_amd import pktgen as pg
    b, prog = R.config5(n)
    rng = np.random.default_rng(505)
    buf = b.buf
    for i in range(b.n):
        o = int(b.off[i])
        f = bytes(buf[o:o + 64])
        l3 = 14
        while int.from_bytes(f[l3 - 2:l3], "big") in (0x8100, 0x88A8):
            l3 += 4
        et = int.from_bytes(f[l3 - 2:l3], "big")
        l4 = l3 + (40 if et == 0x86DD else 20)
        proto = f[l3 + 6] if et == 0x86DD else f[l3 + 9]
        u = rng.random()
        if proto == 6 and u < 0.08:
            buf[o + l4 + 12] = 0x40                    # data offset 4 < 5: E_TCP
        elif proto == 17 and u < 0.08:
            buf[o + l4 + 4:o + l4 + 6] = [0, 4]        # UDP length 4 < 8: E_UDP
        elif proto == 17 and u < 0.12:
            buf[o + l4 + 2:o + l4 + 4] = [0x11, 0x94]  # dport 4500 (NAT-T marker test)
    ncos = R.cos_count(prog)
    prog = [(op[0], op[1], dict(op[2], stats=1 if stats and k % 3 == 0 else 0))
            if op[0] == "cos" else op for k, op in enumerate(prog)]
    prog.append(R.cos("l4err", queue=999, stats=1 if stats else 0))
    prog.append(("error", ncos))
    return b, prog


@pytest.mark.parametrize("stats", [False, True], ids=["nostats", "stats"])
@pytest.mark.parametrize("engine", ["spec", "nojit", "wpb4", "nojoint"])
def test_far_l4_checks_deferred(built, gpu, engine, stats):
    """Tree kernels stage bytes 64.. per lane after the parse and check the L4
    headers whose bytes lie there once they land (the first descent round
    runs meanwhile; a lane found in error is moved to the error CoS, as
    cls_select_cos would have, odp_classification.c:1694-1726).  Records
    bit-exact against the oracle, and with per-CoS counters (no deferral
    then) the counters too (:1646-1647, 1721-1723)."""
    from odp_amd.cls import Classifier
    from oracle.oracle import Oracle
    b, prog = _far_l4_errors(40_000, stats)
    got = both(prog, b, what=f"far L4 errors stats={stats}", engine=engine)
    s = summary(got)
    assert s["enq"] > 0
    assert np.count_nonzero(got["err"] & 0x18) > 500   # E_TCP / E_UDP found
    if stats:
        c = Classifier(gpu=0)
        o = Oracle()
        try:
            cos, _ = c.apply(prog)
            ocos, _ = o.apply(prog)
            c.classify(b)
            o.classify(b)
            for h, oh in zip(cos, ocos):
                if h:
                    assert c.cos_stats_packets(h) == o.stats_packets(oh)
        finally:
            c.close()
