"""Host-side checks that need no GPU: the C-ABI libraries load and export
every symbol their headers declare, the ctypes mirrors match the C layouts,
the ODP classification control plane follows linux-generic's API semantics
(odp_classification.c:137-930), and the rule-table compiler emits the
snapshot the kernel expects (order, skips, limits)."""
import ctypes as C
import os
import re
import struct

import pytest

from odp_amd import cls
from odp_amd import rules as R
from tests import zoo

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions(h):
    txt = open(os.path.join(ROOT, "include", h)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\([^;{]*\)\s*;", txt, flags=re.M)
    return sorted(set(n for n in names if not n.startswith("_")))


@pytest.mark.parametrize("hdr,lib", [("mi_cls.h", cls.LIB_MI), ("odp_cls_api.h", cls.LIB_ODP)])
def test_exports_every_declared_symbol(built, hdr, lib):
    fns = header_functions(hdr)
    assert len(fns) > 5
    so = C.CDLL(lib, mode=C.RTLD_GLOBAL)
    missing = [f for f in fns if not hasattr(so, f)]
    assert not missing, missing


def test_abi_layouts(built):
    L = cls.lib()
    L.odp_amd_cls_abi_size.restype = C.c_size_t
    L.odp_amd_cls_abi_size.argtypes = [C.c_int]
    sz = L.odp_amd_cls_abi_size
    assert sz(0) == C.sizeof(cls.PmrParam)
    assert sz(1) == C.sizeof(cls.PmrCreateOpt)
    assert sz(2) == C.sizeof(cls.CosParam)
    assert sz(3) == C.sizeof(cls.Capability)
    assert sz(4) == C.sizeof(cls.CosStats)
    assert sz(5) == 16 == R.RESULT_DTYPE.itemsize
    assert (sz(6), sz(7), sz(8), sz(9)) == (64, 16, 16, 48)
    assert sz(100) == cls.CosParam.pool.offset
    assert sz(101) == cls.CosParam.vector.offset
    assert sz(102) == cls.CosParam.aggr_enq_profile.offset
    assert sz(103) == cls.Capability.max_mark.offset
    assert sz(104) == cls.PmrParam.val_sz.offset
    assert sz(105) == cls.CosParam.u.offset + cls._QU.qp.offset + cls._QP.hash_proto.offset


@pytest.fixture
def c(built):
    k = cls.Classifier(gpu=0)
    yield k
    k.close()


def test_capability(c):
    cap = cls.Capability()
    assert c.L.odp_cls_capability(C.byref(cap)) == 0
    assert (cap.max_cos, cap.max_pmr, cap.max_pmr_per_cos) == (255, 8192, 4096)
    assert cap.max_terms_per_pmr == 8 and cap.max_hash_queues == 32 and cap.max_mark == 0xFFFF
    assert cap.max_pmr_priority == 0 and not cap.pmr_range_supported
    # terms supported on linux-generic (odp_classification.c:163-183): bits 0..20 except ld_vni(18)
    want = sum(1 << b for b in range(21) if b != 18)
    assert cap.supported_terms == want


def test_stock_limits(built):
    k = cls.Classifier(gpu=0, limits=(64, 256, 8))
    cap = cls.Capability()
    k.L.odp_cls_capability(C.byref(cap))
    assert (cap.max_cos, cap.max_pmr, cap.max_pmr_per_cos) == (64, 256, 8)
    src = k.cos_create("s", queue=1)
    dst = k.cos_create("d", queue=2)
    hs = [k.pmr_create([R.t_u8(R.PMR_IPPROTO, i)], src, dst) for i in range(9)]
    assert all(hs[:8]) and hs[8] == 0          # CLS_PMR_PER_COS_MAX (:832)
    cs = [k.cos_create(f"c{i}", queue=3) for i in range(70)]
    assert sum(1 for x in cs if x) == 62       # 64 slots, 2 used above
    k.close()


def test_cos_create_rules(c):
    assert c.cos_create("noq", queue=0) == 0                  # enqueue needs a queue (:248)
    assert c.cos_create("drop", action=1, queue=0) != 0       # drop needs none (:242-246)
    assert c.cos_create("nq0", num_queue=0) == 0              # (:253)
    assert c.cos_create("nq33", num_queue=33, hash_proto=R.HP_IPV4) == 0
    h = c.cos_create("hq", num_queue=4, hash_proto=R.HP_IPV4_UDP)
    assert h
    assert c.L.odp_cls_cos_num_queue(h) == 4
    arr = (C.c_void_p * 8)()
    assert c.L.odp_cls_cos_queues(h, arr, 8) == 4
    assert all(arr[i] for i in range(4)) and len({arr[i] for i in range(4)}) == 4
    assert c.L.odp_cos_queue_set(h, 5) == -1                  # hashing enabled (:534)


def test_handles_lowest_free_slot(c):
    a, b, d = (c.cos_create(n, queue=1) for n in "abd")
    assert (a, b, d) == (1, 2, 3)                             # handle = index + 1
    assert c.L.odp_cos_destroy(b) == 0
    assert c.L.odp_cos_destroy(b) == -1                       # already invalid
    assert c.cos_create("e", queue=1) == 2                    # lowest free slot
    assert c.L.odp_cos_to_u64(a) == 1
    assert c.L.odp_cos_destroy(0) == -1


def test_cos_queue_and_pool(c):
    h = c.cos_create("q", queue=7, pool=9)
    assert c.L.odp_cos_queue(h) == 7
    assert c.L.odp_cos_queue_set(h, 8) == 0 and c.L.odp_cos_queue(h) == 8
    assert c.L.odp_cos_queue_set(h, 0) == -1
    assert c.L.odp_cls_cos_pool(h) == 9
    assert c.L.odp_cls_cos_pool_set(h, 10) == 0 and c.L.odp_cls_cos_pool(h) == 10
    assert c.L.odp_cos_queue(99) is None and c.L.odp_cls_cos_num_queue(99) == 0


def test_pmr_create_rules(c):
    s, d = c.cos_create("s", queue=1), c.cos_create("d", queue=2)
    ok = R.t_u8(R.PMR_IPPROTO, 17)
    assert c.pmr_create([ok], s, 0) == 0                      # invalid dst (:822)
    assert c.pmr_create([ok] * 9, s, d) == 0                  # > CLS_PMRTERM_MAX (:827)
    assert c.pmr_create([(R.PMR_IPPROTO, b"\x11\x00", b"\xff\xff", 0)], s, d) == 0   # val_sz
    assert c.pmr_create([(R.PMR_ICMP_TYPE, b"\x08", b"\xff", 0)], s, d) == 0  # not supported
    assert c.pmr_create([(R.PMR_CUSTOM_FRAME, bytes(17), bytes(17), 0)], s, d) == 0
    assert c.pmr_create([(R.PMR_CUSTOM_FRAME, bytes(3), bytes(3), 10)], s, d) != 0
    assert c.pmr_create([ok], s, d, mark=0x10000) == 0       # > MAX_MARK (:874)
    h = c.pmr_create([ok], s, d, mark=0xFFFF)
    assert h and c.L.odp_pmr_to_u64(h) >= 1
    assert c.pmr_create([], s, d) != 0                        # 0 terms matches all
    # range terms are rejected (:678-681)
    p = cls.PmrParam()
    c.L.odp_cls_pmr_param_init(C.byref(p))
    v = C.c_uint8(17)
    p.term, p.range_term, p.value, p.mask, p.val_sz = R.PMR_IPPROTO, True, \
        C.cast(C.byref(v), C.c_void_p), C.cast(C.byref(v), C.c_void_p), 1
    assert not c.L.odp_cls_pmr_create(C.byref(p), 1, s, d)
    assert c.L.odp_cls_pmr_destroy(h) == 0 and c.L.odp_cls_pmr_destroy(h) == -1


def test_pktio_setters(c):
    h = c.cos_create("x", queue=1)
    assert c.L.odp_pktio_default_cos_set(c.pktio, h) == 0
    assert c.L.odp_pktio_error_cos_set(c.pktio, h) == 0
    assert c.L.odp_pktio_default_cos_set(c.pktio, 77) == -1  # invalid CoS
    assert c.L.odp_pktio_default_cos_set(0, h) == -1         # invalid pktio
    assert c.L.odp_pktio_skip_set(c.pktio, 4) == -95          # -ENOTSUP (:649-656)
    assert c.L.odp_pktio_headroom_set(c.pktio, 64) == 0


def test_generation_counter(c):
    g0 = c.L.odp_amd_cls_generation()
    c.cos_create("x", queue=1)
    assert c.L.odp_amd_cls_generation() > g0


# ------------------------------------------------------------- compiled blob
def parse_blob(b):
    h = struct.unpack_from("<4I2I2i8I", b, 0)
    hdr = dict(zip(["magic", "version", "total", "ncos", "nrules", "nterms", "default", "error",
                    "default_valid", "used", "max_hops", "cos_off", "rule_off", "term_off",
                    "gen", "rsv"], h))
    cos = [struct.unpack_from("<2I4BI", b, hdr["cos_off"] + 16 * i) for i in range(hdr["ncos"])]
    rules = [struct.unpack_from("<IHHII", b, hdr["rule_off"] + 16 * i)
             for i in range(hdr["nrules"])]
    terms = [struct.unpack_from("<BBHI2I4I4I", b, hdr["term_off"] + 48 * i)
             for i in range(hdr["nterms"])]
    return hdr, cos, rules, terms


def test_compile_blob_layout(c):
    c.apply(zoo.prog_everything())
    hdr, cos, rules, terms = parse_blob(c.compile())
    assert hdr["magic"] == 0x534C434D and hdr["version"] == 1 and hdr["total"] == len(c.compile())
    assert hdr["default"] == 0 and hdr["error"] == 1 and hdr["default_valid"] == 1
    assert hdr["cos_off"] == 64
    # every rule of a CoS is contiguous and in creation order here
    assert sum(x[1] for x in cos) == hdr["nrules"]
    assert all(0 <= r[3] < hdr["ncos"] for r in rules)
    assert sum(r[1] for r in rules) == hdr["nterms"]


def test_compile_order_after_deletes(c):
    """The snapshot reproduces swap-on-delete order and drops links to an
    invalid CoS (odp_classification.c:782-786, 1635-1636)."""
    c.apply(zoo.prog_deletes())
    hdr, cos, rules, terms = parse_blob(c.compile())
    r0 = cos[0]
    dsts = [rules[r0[0] + i][3] for i in range(r0[1])]
    marks = [rules[r0[0] + i][2] for i in range(r0[1])]
    # created: m0..m5 -> c1..c6; destroy pmr0 -> [m5,m1,m2,m3,m4]; destroy cos c5 (slot 5, m4
    # link skipped); destroy pmr2 -> [m5,m1,m4,m3]; new CoS takes slot 5; new pmr m42 -> slot 5
    assert marks == [5, 1, 4, 3, 42]
    assert dsts == [6, 2, 5, 4, 5]


def test_compile_empty_and_no_default(c):
    hdr, cos, rules, terms = parse_blob(c.compile())
    assert hdr["default"] == -1 and hdr["ncos"] == 0 and hdr["nrules"] == 0


def test_classify_without_gpu_fails_loudly(c):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    c.apply([R.cos("d", queue=1), ("default", 0)])
    rc = c.classify_device(0, 0, 0, 1, 0)
    assert rc < 0        # -ENODEV: no CPU fallback exists


@pytest.mark.parametrize("cfg,flat,spec", [(2, True, True), (3, True, True), (4, True, True),
                                           ("nested1024", True, True), (5, False, True),
                                           ("5open", False, False),
                                           ("classes", False, True), ("noblock", False, False)])
def test_specialised_kernel_compiles(built, cfg, flat, spec):
    """The embedded kernel sources compile with hipRTC (no GPU needed) into
    the program-specialised kernel of a flat program (every packet decided
    on the default CoS's block in one round; candidate lists included), of a
    flat program whose default CoS has a chain of blocks (9 key classes: no
    generic flat kernel, the chain compiled in) and of a CoS tree whose
    levels are joint groups (config 5: the tree plan compiled in).  A tree
    whose plan does not cover it (config 5 plus a rule from a prefix CoS to
    a CoS outside any joint group) and a default CoS without rules have
    none."""
    L = cls.lib()
    L.mi_cls_spec_compile.restype = C.c_int
    L.mi_cls_spec_compile.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
    if cfg == "classes":
        b, prog = R.config3_classes(100)
    elif cfg == "nested1024":
        b, prog = R.config3_nested(100, scale=4)
    elif cfg == "noblock":
        b, prog = R.config2(100)
        prog = [op for op in prog if op[0] != "pmr"]
    elif cfg == "5open":
        b, prog = R.config5(100)
        ncos = sum(1 for op in prog if op[0] == "cos")
        # a fourth level below one prefix CoS: "deep" has a rule of its own
        # (to leaf 0) but is in no joint group, so the plan stops covering
        prog = prog + [R.cos("deep", queue=900),
                       ("pmr", [R.t_be16(R.PMR_UDP_SPORT, 7)], 17, ncos, 0),
                       ("pmr", [R.t_u8(R.PMR_IPPROTO, 17)], ncos, 161, 0)]
    else:
        b, prog = R.CONFIGS[cfg](100)
    c = cls.Classifier(gpu=0)
    try:
        c.apply(prog)
        blob = c.compile()
        assert (c.program_info()["flat_engine"] >= 0) == flat
        for nw in ((4, 16) if cfg == 3 else (16,)):
            assert L.mi_cls_spec_compile(blob, len(blob), nw) == (0 if spec else 1)
    finally:
        c.close()


def test_block_chain_for_many_classes(built):
    """256 rules over 9 key classes: one block cannot hold them, so the
    default CoS gets a chain of blocks (not the linear scan); 8 classes or
    fewer keep a single block."""
    c = cls.Classifier(gpu=0)
    try:
        c.apply(R.config3_classes(100)[1])
        info = c.program_info()
        assert info["chained"] == 1 and info["blocks"] == 1 and info["flat_engine"] == -1
        c2 = cls.Classifier(gpu=0)
        c2.apply(R.config3_nested(100)[1])
        assert c2.program_info()["chained"] == 0
        c2.close()
        # the same rules in a CoS tree: the tree kernels scan them linearly
        from tests.test_gpu_parity import _under_root
        for root_first in (False, True):
            c3 = cls.Classifier(gpu=0)
            c3.apply(_under_root(R.config3_classes(100)[1], root_first))
            i3 = c3.program_info()
            c3.close()
            assert i3["tree"] and i3["chained"] == 0, i3
    finally:
        c.close()


def test_shadowed_rules_leave_candidate_lists(built):
    """A rule that can hold only when an earlier rule holds is dropped at
    block build (it is never the first holding rule): the nested-prefix ACL
    with 1024 rules, whose /20 lines repeat, then gets the single-candidate
    engine instead of candidate lists (parity: tests/test_gpu_parity.py
    test_overlapping_acls, every engine forcing)."""
    c = cls.Classifier(gpu=0)
    try:
        c.apply(R.config3_nested(100, scale=4)[1])
        info = c.program_info()
        assert info["cand1"] == 1 and info["candidate"] == 0, info
    finally:
        c.close()


def test_joint_groups_host(built):
    """Tree levels keyed on the same classes assemble into joint groups: one
    (key, CoS) table per level and class instead of a table per CoS -- config
    5's direct level (128 CoS) and its bitmap level (16 CoS);
    MI_CLS_NO_JOINT=1: per-CoS tables.  Host only; GPU parity:
    tests/test_gpu_parity.py test_joint_direct_tree_levels and the configs."""
    def hot_words():
        c = cls.Classifier(gpu=0)
        try:
            c.apply(R.config5(100)[1])
            return c.program_info()
        finally:
            c.close()
    with_joint = hot_words()
    os.environ["MI_CLS_NO_JOINT"] = "1"
    try:
        without = hot_words()
    finally:
        del os.environ["MI_CLS_NO_JOINT"]
    assert with_joint["tree"] and with_joint["direct"] == without["direct"]
    assert with_joint["joint_direct"] == 128 and with_joint["joint_bitmap"] == 16, with_joint
    assert without["joint_direct"] == 0 and without["joint_bitmap"] == 0, without
