"""Multi-GPU product path on the GPU box: a host batch
sharded over several contexts by mi_cls_group_classify_host -- here several
contexts on the one visible device, plus every visible device -- must give
exactly the single-context records (and the oracle's); the runtime pktio opens
a multi-GPU endpoint from ODP_AMD_GPUS; and bench.py's multi-rank path runs
with two ranks (gloo rendezvous, both on the device)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from odp_amd import rules as R
from tests import rt_helpers as H
from tests import zoo
from tests.helpers import assert_same, oracle_run

pytestmark = pytest.mark.gpu


def _group_run(prog, batch, gpus):
    from odp_amd.cls import Classifier
    c = Classifier(gpus=gpus)
    try:
        c.apply(prog)
        return c.classify_host(batch)
    finally:
        c.close()


@pytest.mark.parametrize("cfg,n", [(3, 60_000), (4, 40_000), (5, 30_000), (2, 50_000)])
@pytest.mark.parametrize("ngroup", [2, 3, 8])
def test_group_equals_single(built, gpu, cfg, n, ngroup):
    b, prog = R.CONFIGS[cfg](n)
    exp, _ = oracle_run(prog, b)
    one = _group_run(prog, b, [0])
    grp = _group_run(prog, b, [0] * ngroup)
    assert_same(one, exp, b, f"config {cfg} single context")
    assert_same(grp, exp, b, f"config {cfg} {ngroup} contexts")


def test_group_all_devices(built, gpu):
    import torch
    nd = torch.cuda.device_count()
    b, prog = R.config3(20_000)
    exp, _ = oracle_run(prog, b)
    assert_same(_group_run(prog, b, list(range(nd))), exp, b, f"{nd} devices")


def test_group_ragged_and_tiny(built, gpu):
    """More contexts than packets, empty slices, unaligned offsets."""
    frames = [f for _, f in zoo.all_frames()]
    from odp_amd import pktgen as pg
    prog = zoo.prog_everything()
    for k in (1, 5, len(frames) + 3):
        b = pg.batch_from_frames(frames[:k])
        exp, _ = oracle_run(prog, b)
        assert_same(_group_run(prog, b, [0] * 7), exp, b, f"{k} frames over 7 contexts")


def test_runtime_pktio_multi_gpu(built, gpu, tmp_path):
    """The loop / pcap receive path with ODP_AMD_GPUS=0,0,0: every burst is
    sharded over three contexts; queues, order, metadata and counters are the
    reference's."""
    frames = H.pcap_frames([f for _, f in zoo.all_frames()])
    pc = str(tmp_path / "in.pcap")
    H.write_pcap(pc, frames)
    rules = str(tmp_path / "rules.txt")
    prog = zoo.prog_everything()
    H.write_rules(rules, prog)
    got = H.run_driver(f"pcap:in={pc}", rules, "sched", 4, 1, 1,
                       env={"ODP_AMD_GPUS": "0,0,0", "ODP_AMD_RX_BURST": "53"})
    H.compare(got, H.expected(prog, frames, 1, 1, 4))


def test_bench_two_ranks_one_device(built, gpu):
    """bench.py's multi-rank path (one process per rank, barrier, max over
    ranks, whole-job value) with 2 ranks sharing the device over gloo."""
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo", BENCH_SAME_DEVICE="1",
               MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", "29533", os.path.join(H.ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "3", "--warmup", "1", "--packets", "100000",
                        "--config", "3"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240,
                       env=env, cwd=H.ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["config"]["parallelism"] == "shard2"
    assert line["parity_vs_oracle"] is True


def test_bench_gpus_2_self_launch_one_device(built, gpu):
    """`bench.py --gpus 2` without a launcher starts its own two ranks
    (BENCH_SAME_DEVICE rehearses them on one device) and reports n_gpus 2."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(BENCH_DIST_BACKEND="gloo", BENCH_SAME_DEVICE="1")
    r = subprocess.run([sys.executable, os.path.join(H.ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "3", "--warmup", "1", "--packets", "100000", "--config", "2",
                        "--no-parity"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240,
                       env=env, cwd=H.ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "shard2"


@pytest.mark.parametrize("ngroup", [1, 3])
def test_group_host_batch_timing(built, gpu, ngroup):
    """The group path on a pageable host batch (config 3, 200 k IMIX
    packets): each device's slice is staged from its own host thread, so the
    slices' copies do not serialise; records equal the oracle's.  Prints the
    per-call time (1 and 3 contexts on the one device here)."""
    import time
    from odp_amd.cls import Classifier
    b, prog = R.config3(200_000)
    exp, _ = oracle_run(prog, b)
    c = Classifier(gpus=[0] * ngroup)
    try:
        c.apply(prog)
        got = c.classify_host(b)
        t0 = time.perf_counter()
        for _ in range(5):
            got = c.classify_host(b)
        dt = (time.perf_counter() - t0) / 5
    finally:
        c.close()
    assert_same(got, exp, b, f"{ngroup} contexts")
    print(f"group classify_host: {ngroup} context(s), {b.n} packets, {dt * 1e3:.2f} ms per call, "
          f"{b.n / dt / 1e6:.1f} Mpkt/s")


def _rx_rate(pc, rules, env):
    """rx_driver rate mode (pcap pktio, direct): (Mpkt/s, delivered, in_discards)."""
    import subprocess
    e = dict(os.environ, RX_COUNT_ONLY="1", **env)
    r = subprocess.run([H.DRIVER, f"pcap:in={pc}:loops=5", rules, "direct", "4", "0", "1"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240,
                       env=e)
    assert r.returncode == 0, r.stderr[-2000:]
    rl = [ln for ln in r.stdout.splitlines() if ln.startswith("R ")][-1].split()
    sl = [ln for ln in r.stdout.splitlines() if ln.startswith("S ")][-1].split()
    return int(rl[1]) / int(rl[2]) * 1e3, int(rl[1]), int(sl[3])


def test_runtime_pktio_group_pipelined_rate(built, gpu, tmp_path):
    """A pcap pktio over 1 and 3 contexts (ODP_AMD_GPUS=0 / 0,0,0): with the
    page-locked frame store each burst's slices are submitted to every
    context and waited for one burst later (mi_cls_group_classify_host_submit
    / _wait), so the group pktio keeps two bursts in flight like the single
    one.  Every frame is delivered (0 in_discards); prints both rates."""
    b, prog = R.config3(100_000)
    pc = str(tmp_path / "in.pcap")
    H.write_pcap(pc, [b.frame(i) for i in range(b.n)])
    rules = str(tmp_path / "rules.txt")
    H.write_rules(rules, prog)
    res = {}
    for gpus in ("0", "0,0,0"):
        res[gpus] = _rx_rate(pc, rules, {"ODP_AMD_GPUS": gpus})
        # loops=5 replays the capture as the reference's pcap driver does:
        # loop_cnt starts at 1 (pcap.c:214) and the driver stops when
        # ++loop_cnt >= loops (pcap.c:265), so the capture passes 4 times
        assert res[gpus][1] == res["0"][1] == 4 * b.n and res[gpus][2] == 0, res
    print("group pktio receive: " + ", ".join(f"{g}: {v[0]:.1f} Mpkt/s" for g, v in res.items()))


def test_group_submit_tickets(built, gpu):
    """odp_amd_cls_classify_host_submit / _wait on a 3-context pktio with
    page-locked batches: three batches in flight at once, waited in order,
    every record equal to the oracle's."""
    import ctypes as C
    import numpy as np
    from odp_amd import cls
    from odp_amd.cls import Classifier
    L = cls.lib()
    L.odp_amd_cls_classify_host_submit.restype = C.c_int
    L.odp_amd_cls_classify_host_submit.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                                   C.c_void_p, C.c_uint32, C.c_void_p,
                                                   C.POINTER(C.c_uint64)]
    L.odp_amd_cls_classify_host_wait.restype = C.c_int
    L.odp_amd_cls_classify_host_wait.argtypes = [C.c_void_p, C.c_uint64]
    batches = [R.config3(30_000 + 7 * k, rank=k)[0] for k in range(3)]
    _, prog = R.config3(10)
    c = Classifier(gpus=[0, 0, 0])
    keep = []
    try:
        c.apply(prog)
        tickets = []
        for bt in batches:
            pb = cls.PinnedArray(bt.buf.nbytes + 64)
            po = cls.PinnedArray(4 * bt.n)
            pl = cls.PinnedArray(2 * bt.n)
            pr = cls.PinnedArray(16 * bt.n)
            pb.u8[: bt.buf.nbytes] = bt.buf
            po.view(np.uint32)[:] = bt.off
            pl.view(np.uint16)[:] = bt.len
            keep.append((pb, po, pl, pr))
            t = C.c_uint64()
            assert L.odp_amd_cls_classify_host_submit(c.pktio, pb.ptr, bt.buf.nbytes + 64, po.ptr,
                                                      pl.ptr, bt.n, pr.ptr, C.byref(t)) == 0
            tickets.append(t.value)
        assert tickets == sorted(tickets) and tickets[0] > 0, tickets
        for bt, t, (_, _, _, pr) in zip(batches, tickets, keep):
            assert L.odp_amd_cls_classify_host_wait(c.pktio, t) == 0
            got = pr.view(np.uint8, 16 * bt.n).view(R.RESULT_DTYPE).copy()
            assert_same(got, oracle_run(prog, bt)[0], bt, f"ticket {t}")
    finally:
        c.close()
        for arrs in keep:
            for a in arrs:
                a.close()
