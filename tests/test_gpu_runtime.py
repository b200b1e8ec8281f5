"""End-to-end receive path on the GPU through the ODP runtime subset: frames
enter a pcap or loop pktio, are parsed + classified in GPU bursts
(odp_amd_cls_classify_host -> mi_cls_kernel) and land in CoS queues; the
packets every queue delivers (order, pool, input flags, error bit, l3/l4
offsets, cls mark, bytes) and the pktio / queue counters must be exactly what
the reference receive path produces, derived from the CPU oracle
(tests/rt_helpers.expected).  Also runs the reference's example/classifier,
compiled unchanged against this build, with its own CI arguments
(example/classifier/odp_classifier_run.sh,
platform/linux-generic/test/example/classifier/pktio_env:21-23).
"""
import os
import subprocess

import numpy as np
import pytest

from odp_amd import rules as R
from tests import rt_helpers as H
from tests import zoo

pytestmark = pytest.mark.gpu

UDP64 = os.path.join(H.ROOT, "tests", "golden", "udp64.pcap")


def _run_case(tmp_path, prog, frames, mode="sched", pktio="pcap", cos_pools=1, layer=4, cls=1,
              burst=None, pktin_opt=0, env_extra=None):
    pc = str(tmp_path / "in.pcap")
    H.write_pcap(pc, frames)
    rules = str(tmp_path / "rules.txt")
    H.write_rules(rules, prog)
    env = {"ODP_AMD_RX_BURST": str(burst)} if burst else {}
    env.update(env_extra or {})
    if pktin_opt:
        env["RX_PKTIN_OPT"] = str(pktin_opt)
    if pktio == "loop":
        got = H.run_driver("loop", rules, mode, layer, cos_pools, cls, src=pc, env=env)
    else:
        got = H.run_driver(f"pcap:in={pc}", rules, mode, layer, cos_pools, cls, env=env)
    exp = H.expected(prog, frames, cos_pools, cls, layer, pktin_opt=pktin_opt)
    H.compare(got, exp)
    return got


def test_example_classifier_udp64(built, gpu):
    """The reference's own acceptance run: 100 packets to queue1, 100 to
    DefaultCos, exit status 0."""
    # the binary is built in the build container and travels with the tree:
    # missing on the GPU box is a failure, not a skip
    assert os.path.exists(H.EXAMPLE), f"{H.EXAMPLE} missing: run __graft_entry__.build()"
    r = subprocess.run([H.EXAMPLE, "-t", "1", "-i", f"pcap:in={UDP64}", "-m", "0", "-p",
                        "ODP_PMR_SIP_ADDR:10.10.10.0:0xFFFFFF00:queue1", "-P", "-C",
                        "queue1:100", "-C", "DefaultCos:100"],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=90,
                       cwd="/tmp")
    assert r.returncode == 0, r.stdout[-3000:]
    # the statistics row: "<queue> <pool>|" per policy, then total
    rows = [ln for ln in r.stdout.splitlines() if ln.count("|") >= 2 and ln[:1].isdigit()]
    assert rows, r.stdout[-3000:]
    cells = [c.split() for c in rows[-1].split("|")[:2]]
    assert [int(x) for x in cells[0]] == [100, 100]   # queue1: queue, pool
    assert [int(x) for x in cells[1]] == [100, 100]   # DefaultCos
    assert "Exit" in r.stdout


def test_example_classifier_two_workers_dmac(built, gpu):
    """Two worker threads, a DMAC rule, no dedicated CoS pools (-d 0)."""
    # the binary is built in the build container and travels with the tree:
    # missing on the GPU box is a failure, not a skip
    assert os.path.exists(H.EXAMPLE), f"{H.EXAMPLE} missing: run __graft_entry__.build()"
    r = subprocess.run([H.EXAMPLE, "-t", "1", "-c", "2", "-d", "0", "-i", f"pcap:in={UDP64}",
                        "-m", "0", "-p", "ODP_PMR_DMAC:02-00-00-00-00-02:ffffffffffff:mac",
                        "-P", "-C", "mac:200"],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=90,
                       cwd="/tmp")
    assert r.returncode == 0, r.stdout[-3000:]


@pytest.mark.parametrize("mode", ["sched", "direct", "queue"])
def test_rx_zoo_everything(built, gpu, tmp_path, mode):
    frames = H.pcap_frames([f for _, f in zoo.all_frames()])
    _run_case(tmp_path, zoo.prog_everything(), frames, mode)


def test_rx_zoo_shared_pool(built, gpu, tmp_path):
    frames = H.pcap_frames([f for _, f in zoo.all_frames()])
    _run_case(tmp_path, zoo.prog_everything(), frames, cos_pools=0)


def test_rx_loop_pktio(built, gpu, tmp_path):
    frames = H.pcap_frames([f for _, f in zoo.all_frames()])
    _run_case(tmp_path, zoo.prog_everything(), frames, pktio="loop")


@pytest.mark.parametrize("cos_pools", [0, 1])
@pytest.mark.parametrize("delivery", ["gpu", "host", "pageable_pools"])
def test_rx_delivery_paths(built, gpu, tmp_path, cos_pools, delivery):
    """The receive delivery after classification on both paths: the GPU
    delivery kernel (page-locked pools: metadata, frame copies and the
    group-by-queue done by mi_cls_deliver_submit; loop packets classified in
    place, copied only on a pool switch) and the host's
    (ODP_AMD_RX_GPU_DELIVER=0, or pools in ordinary memory).  pcap and loop
    pktios, shared pool (in place) and per-CoS pools (pool switch); every
    queue's packets, metadata and counters as the reference's."""
    env = {"gpu": {}, "host": {"ODP_AMD_RX_GPU_DELIVER": "0"},
           "pageable_pools": {"ODP_AMD_PINNED_POOLS": "0"}}[delivery]
    frames = H.pcap_frames([f for _, f in zoo.all_frames()])
    for pktio in ("pcap", "loop"):
        _run_case(tmp_path, zoo.prog_everything(), frames, mode="direct", pktio=pktio,
                  cos_pools=cos_pools, burst=61, env_extra=env)


def test_rx_pktio_pool_held_cos_pools(built, gpu, tmp_path):
    """Every packet of the pktio's pool held by the application while every
    CoS has a pool of its own: the pcap receive keeps moving --
    the frames never need the pktio's pool -- and delivers what the
    reference delivers."""
    frames = H.pcap_frames([f for _, f in zoo.all_frames()])
    prog = [op for op in zoo.prog_everything()]
    _run_case(tmp_path, prog, frames, mode="direct", cos_pools=1,
              env_extra={"RX_HOLD_PKTIO_POOL": "1"})


def test_rx_deletes_and_drops(built, gpu, tmp_path):
    frames = H.pcap_frames([f for _, f in zoo.all_frames()])
    _run_case(tmp_path, zoo.prog_deletes(), frames)
    _run_case(tmp_path, zoo.prog_no_default(), frames)


@pytest.mark.parametrize("layer", [0, 1, 2, 3])
def test_rx_parse_layers_no_classifier(built, gpu, tmp_path, layer):
    """Classifier disabled: packets go to the pktin queue parsed up to the
    configured layer (odp_packet_io.c:675-677, odp_parse.c:372-414)."""
    frames = H.pcap_frames([f for _, f in zoo.all_frames()])
    _run_case(tmp_path, [], frames, cls=0, layer=layer)


def test_rx_random_programs_small_bursts(built, gpu, tmp_path):
    """Random CoS graphs + fuzzed frames, with 37-packet GPU bursts so that
    enqueue runs straddle burst boundaries."""
    rng = np.random.default_rng(1234)
    base = [f for _, f in zoo.all_frames()]
    for it in range(3):
        frames = H.pcap_frames(base + zoo.mutate_frames(rng, base, 300))
        prog = zoo.random_program(rng, base)
        if any(op[0] == "cos" and " " in op[1] for op in prog):
            continue
        _run_case(tmp_path, prog, frames, burst=37)


@pytest.mark.parametrize("layer,opt,cls", [(4, 0x3C, 1), (4, 0x7FC, 1), (4, 0x780, 1),
                                           (2, 0x7FC, 0), (3, 0x7FC, 0), (4, 0x7FC, 0)])
def test_rx_pktin_checksum_options(built, gpu, tmp_path, layer, opt, cls):
    """odp_pktio_config(pktin.bit.*_chksum / drop_*_err) through the runtime:
    checksum statuses (odp_packet_l3/l4_chksum_status), error-CoS routing,
    drops and in_errors as the reference receive path produces them; with the
    classifier off, the parser layer limits which options apply."""
    from tests import chksum_frames as CK
    frames = H.pcap_frames([f for f, _, _ in CK.frame_set(seed=51, n=120)] +
                           [f for _, f in zoo.all_frames()])
    _run_case(tmp_path, zoo.prog_everything(), frames, layer=layer, cls=cls, pktin_opt=opt)


def test_rx_config2_traffic(built, gpu, tmp_path):
    """BASELINE config 2 traffic (16 SIP /24 rules) through the pcap pktio."""
    b, prog = R.config2(20000)
    frames = [b.frame(i) for i in range(b.n)]
    got = _run_case(tmp_path, prog, frames)
    assert sum(len(v) for v in got[0].values()) == 20000


@pytest.mark.parametrize("max_size,burst", [(4, 37), (1, 64), (64, 4096), (7, 1)])
def test_rx_packet_vector_cos(built, gpu, tmp_path, max_size, burst):
    """CoS packet-vector delivery (odp_cls_cos_param_t.vector): the same
    packets, order, metadata and counters as plain delivery, grouped into
    vectors exactly as _odp_cos_vector_enq groups each enqueue run
    (odp_classification_internal.h:83-137)."""
    frames = H.pcap_frames([f for _, f in zoo.all_frames()] * 3)
    prog = zoo.prog_everything()
    pc = str(tmp_path / "in.pcap")
    H.write_pcap(pc, frames)
    rules = str(tmp_path / "rules.txt")
    H.write_rules(rules, prog)
    ev = {}
    got = H.run_driver(f"pcap:in={pc}", rules, "sched", 4, 1, 1, events=ev,
                       env={"RX_PKTV": f"{max_size},100000", "ODP_AMD_RX_BURST": str(burst)})
    H.compare(got, H.expected(prog, frames, 1, 1, 4))
    exp = H.expected_vectors(prog, frames, burst, max_size)
    assert ev == exp


def test_rx_packet_vector_pool_exhausted(built, gpu, tmp_path):
    """A vector pool too small for the traffic: runs that get no vector are
    dropped and counted as queue discards (odp_classification_internal.h:
    104-108); nothing is lost without a count."""
    frames = H.pcap_frames([f for _, f in zoo.all_frames()] * 4)
    prog = zoo.prog_everything()
    pc = str(tmp_path / "in.pcap")
    H.write_pcap(pc, frames)
    rules = str(tmp_path / "rules.txt")
    H.write_rules(rules, prog)
    queues, stats, qstats = H.run_driver(f"pcap:in={pc}", rules, "sched", 4, 1, 1,
                                         env={"RX_PKTV": "8,1", "ODP_AMD_RX_BURST": "4096"})
    _, _, eqs = H.expected(prog, frames, 1, 1, 4)
    delivered = sum(len(v) for v in queues.values())
    discards = sum(d for _, d in qstats.values())
    assert delivered + discards == sum(v[0] for v in eqs.values())
    assert discards > 0


def test_rx_hash_queue_event_aggregators(built, gpu, tmp_path):
    """Hash-queue CoS whose queues have event aggregators
    (queue_param.num_aggr): runs go to odp_queue_aggr(q, 0)
    (odp_classification_internal.h:149-157), so every packet of those queues
    arrives inside an event vector; order, metadata and queue stats as plain
    delivery."""
    frames = H.pcap_frames([f for _, f in zoo.all_frames()] * 3)
    prog = zoo.prog_everything()
    assert any(op[0] == "cos" and op[2]["num_queue"] > 1 for op in prog)
    pc = str(tmp_path / "in.pcap")
    H.write_pcap(pc, frames)
    rules = str(tmp_path / "rules.txt")
    H.write_rules(rules, prog)
    ev = {}
    got = H.run_driver(f"pcap:in={pc}", rules, "sched", 4, 1, 1, events=ev,
                       env={"RX_AGGR": "8", "ODP_AMD_RX_BURST": "41"})
    H.compare(got, H.expected(prog, frames, 1, 1, 4))
    hq = [q for q in got[0] if q.startswith("_odp_cos_hq_")]
    assert hq
    for q in hq:
        assert all(e[0] == "E" and 1 <= e[1] <= 8 for e in ev[q]), ev[q]
        assert sum(e[1] for e in ev[q]) == len(got[0][q])
    for q in got[0]:
        if q not in hq:
            assert all(e == ("P",) for e in ev[q])


def test_rx_small_first_segment(built, gpu, tmp_path):
    """Pools whose pkt.seg_len (64 B) is below the frame sizes: the runtime
    keeps every packet in one segment (seg_len is the minimum first-segment
    length the spec asks for), so the parse sees seg_end = frame_len and the
    reference's segmented-copy path (pktio/loop.c:299-306) has nothing to
    do; rules on bytes deep in 1514-B frames (custom frame offset 1400)
    classify as the oracle says, and every delivered packet is one segment."""
    from odp_amd import pktgen as pg
    frames = [f for _, f in zoo.all_frames()]
    big = [pg.udp4_frame(src=f"10.0.0.{i}", dport=1000 + i, size=1514) for i in range(40)]
    big = [f[:1400] + bytes([i & 0xFF, 0x5A]) + f[1402:] for i, f in enumerate(big)]
    frames = H.pcap_frames(frames + big + frames)
    prog = [R.cos("default", queue=1), R.cos("deep", queue=2), R.cos("v6", queue=3),
            ("default", 0),
            ("pmr", [R.t_custom(R.PMR_CUSTOM_FRAME, 1400, bytes([7, 0x5A]), b"\xff\xff")],
             0, 1, 9),
            ("pmr", [R.t_be16(R.PMR_ETHTYPE_0, pg.ETH_IPV6)], 0, 2, 0)]
    pc = str(tmp_path / "in.pcap")
    H.write_pcap(pc, frames)
    rules = str(tmp_path / "rules.txt")
    H.write_rules(rules, prog)
    for pktio in ("pcap", "loop"):
        env = {"RX_SEG_LEN": "64"}
        got = (H.run_driver(f"pcap:in={pc}", rules, "sched", 4, 1, 1, env=env) if pktio == "pcap"
               else H.run_driver("loop", rules, "sched", 4, 1, 1, src=pc, env=env))
        H.compare(got, H.expected(prog, frames, 1, 1, 4))
        assert len(got[0]["deep"]) == 1


@pytest.mark.parametrize("switch_after", [1, 2, 3])
def test_rx_cos_destroyed_while_burst_in_flight(built, gpu, tmp_path, switch_after):
    """A hash-queue CoS is destroyed (its queues with it, and a new default
    CoS with a new queue created) between two odp_pktin_recv calls while
    earlier bursts are still in flight on the GPU: after call 1 the first
    burst is being classified, after calls 2 and 3 the first bursts are in
    their GPU delivery (queues and pools already settled under the old
    tables).  Those bursts must be delivered under the current
    tables (as the synchronous path would), not to the destroyed CoS's queues
    or a queue that reused their slots: every packet the current rules
    enqueue reaches the new CoS, and in_discards counts only the frames the
    oracle discards (compare() checks the pktio counters)."""
    frames = H.pcap_frames([f for _, f in zoo.all_frames()])
    pc = str(tmp_path / "in.pcap")
    H.write_pcap(pc, frames)
    before = [R.cos("A", num_queue=4, hash_proto=0x7), ("default", 0)]
    after = [R.cos("B"), ("default", 1), ("cos_destroy", 0)]
    r1, r2 = str(tmp_path / "r1.txt"), str(tmp_path / "r2.txt")
    H.write_rules(r1, before)
    H.write_rules(r2, after)
    # loops=3 (two passes over the capture: the reference's loop count
    # starts at 1, pcap.c:257-278) in bursts of 16: the first call's burst
    # stays in flight (more frames are waiting at the driver)
    got = H.run_driver(f"pcap:in={pc}:loops=3", r1, "direct", 4, 1, 1,
                       env={"ODP_AMD_RX_BURST": "16", "RX_SWITCH_RULES": r2,
                            "RX_SWITCH_AFTER": str(switch_after)})
    exp = H.expected(before + after, frames * 2, 1, 1, 4)
    H.compare(got, exp)
    assert got[0].get("B"), "nothing reached the new default CoS"


def test_rx_mixed_delivery_paths_keep_order(built, gpu, tmp_path):
    """Bursts that alternate between the GPU delivery and the host's (the
    error CoS's pool is in ordinary memory, so a burst holding an error frame
    is delivered on the host at once while older bursts may still be in their
    GPU delivery): every queue still receives its packets in
    arrival order, on pcap and loop pktios, as the reference's synchronous
    receive does (pktio/loop.c:253-384)."""
    frames = H.pcap_frames([f for _, f in zoo.all_frames()] * 3)
    for pktio in ("pcap", "loop"):
        _run_case(tmp_path, zoo.prog_everything(), frames, mode="direct", pktio=pktio,
                  cos_pools=1, burst=8, env_extra={"ODP_AMD_PAGEABLE_POOLS": "errPool"})


def test_rx_burst_above_device_grouping(built, gpu, tmp_path):
    """Bursts larger than the delivery kernel's grouping serves
    (MI_CLS_DLV_GROUP_MAX = 8192 entries): the burst is enqueued
    per run instead, nothing is lost and every queue's order and counters are
    the reference's."""
    b, prog = R.config2(20000)
    frames = [b.frame(i) for i in range(b.n)]
    got = _run_case(tmp_path, prog, frames, mode="direct", burst=9000)
    assert sum(len(v) for v in got[0].values()) == 20000


def test_rx_chain_short_pool_redo(built, gpu, tmp_path):
    """The receive chain takes each burst's packets from the CoS pools before
    the GPU decides (as many per pool as the previous bursts needed, plus a
    margin).  Traffic whose CoS mix flips between bursts leaves a pool short:
    that burst is delivered again by the host path, and every queue's packets,
    order, pools and counters stay the reference's."""
    from odp_amd import pktgen as pg
    prog = [R.cos("default", queue=1), R.cos("a", queue=2), R.cos("b", queue=3), ("default", 0),
            ("pmr", [R.t_be16(R.PMR_UDP_DPORT, 1111)], 0, 1, 5),
            ("pmr", [R.t_be16(R.PMR_UDP_DPORT, 2222)], 0, 2, 6)]
    frames = []
    for blk in range(12):
        port = 1111 if blk % 3 == 0 else (2222 if blk % 3 == 1 else 3333)
        frames += [pg.udp4_frame(src=f"10.1.{blk}.{i % 250}", dport=port, size=60 + (i % 5) * 40)
                   for i in range(64)]
    frames = H.pcap_frames(frames)
    _run_case(tmp_path, prog, frames, mode="direct", cos_pools=1, burst=64)


def test_rx_loop_packets_outside_pinned_arena(built, gpu, tmp_path):
    """Loop packets from a pool in ordinary memory: the GPU staging of the
    loop burst finds them outside the page-locked arena (not_in_place) and
    the host stages (copies), classifies and delivers that burst; the result
    is the reference's."""
    frames = H.pcap_frames([f for _, f in zoo.all_frames()])
    _run_case(tmp_path, zoo.prog_everything(), frames, pktio="loop", cos_pools=0, burst=32,
              env_extra={"RX_FEED_POOL": "1", "ODP_AMD_PAGEABLE_POOLS": "feedPool"})
