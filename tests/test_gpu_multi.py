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
