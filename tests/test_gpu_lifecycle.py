"""Kernel code-object lifetime and the specialised-kernel compiler.

Round 3's driver bench aborted with HSA_STATUS_ERROR_ILLEGAL_INSTRUCTION on
the first launches of the generic CoS-tree kernel (config 5) after three
contexts had loaded program-specialised modules, classified and been
destroyed in the same process.  The library now loads every fat-binary
kernel at the first context creation and never unloads a specialised
module.  These tests replay that order and check every record against the
oracle, and bound the compiler's concurrency (one compile at a
time, a newer request replaces a queued one).

Semantics kept: descent odp_classification.c:1624-1667; rule changes are
control plane (:1373-1374).
"""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

from odp_amd import rules as R
from tests.helpers import assert_same, oracle_run

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _classify(prog, batch, spec_expected):
    from odp_amd.cls import Classifier
    c = Classifier(gpu=0)
    try:
        c.apply(prog)
        rc = c.spec_wait()
        assert rc == (0 if spec_expected else 1), rc
        got = c.classify(batch)
        return got, c.last_launch()
    finally:
        c.close()


def test_bench_order_replay(built, gpu):
    """bench.py's order in one process: a specialised main context kept
    alive, three flat programs specialised -> classified -> destroyed, then
    config 5 at 1 M packets on its tree-plan kernel and on the generic tree
    kernel (MI_CLS_NO_PLAN).  Bit-exact."""
    from odp_amd.cls import Classifier
    mb, mp = R.config3(200_000)
    cm = Classifier(gpu=0)
    try:
        cm.apply(mp)
        assert cm.spec_wait() == 0
        got = cm.classify(mb)
        assert cm.last_launch()["specialised"]
        assert_same(got, oracle_run(mp, mb)[0], mb, "main config3")
        for make in (lambda: R.config3(200_000, size=60), lambda: R.config2(200_000),
                     lambda: R.config4(200_000)):
            b, p = make()
            got, ll = _classify(p, b, True)
            assert ll["specialised"] and not ll["div"], ll
            assert_same(got, oracle_run(p, b)[0], b, "flat extra")
        b5, p5 = R.config5(1_000_000)
        from oracle.oracle import Oracle
        o = Oracle()
        o.apply(p5)
        exp5 = o.classify(b5, threads=16)
        got, ll = _classify(p5, b5, True)
        assert ll["div"] and ll["specialised"] and ll["flat_engine"] < 0, ll
        assert_same(got, exp5, b5, "config5 tree plan after specialised modules")
        os.environ["MI_CLS_NO_PLAN"] = "1"
        try:
            got, ll = _classify(p5, b5, False)
        finally:
            del os.environ["MI_CLS_NO_PLAN"]
        assert ll["div"] and not ll["specialised"] and ll["flat_engine"] < 0, ll
        assert_same(got, exp5, b5, "config5 generic tree kernel after specialised modules")
    finally:
        cm.close()


def test_spec_one_compile_at_a_time(built, gpu):
    """Six different flat programs loaded back to back on one pktio: at most
    one compiler process runs at any time, superseded requests are dropped
    (their loads classify on the generic kernel), and the last program gets
    its specialised kernel.  Records bit-exact throughout."""
    from odp_amd import cls
    from odp_amd.cls import Classifier
    b, _ = R.config2(20_000)
    c = Classifier(gpu=0)
    try:
        peak = 0
        for k in range(6):
            # distinct programs: config 2's 16 SIP /24 rules shifted by k
            prog = [R.cos("d", queue=1), ("default", 0)]
            for j in range(16):
                prog.append(R.cos(f"c{j}", queue=2 + j))
                prog.append(("pmr", [R.t_ip4(R.PMR_SIP_ADDR, f"10.0.{j + k}.0", 24)], 0, j + 1, 0))
            c.cos, c.pmr = [], []
            c.L.odp_amd_cls_reset()
            assert c.L.odp_amd_cls_limits_set(255, 8192, 4096) == 0
            c.apply(prog)
            got = c.classify(b)   # snapshots the rules: starts / queues a compile
            assert_same(got, oracle_run(prog, b)[0], b, f"program {k}")
            st = cls.spec_pending()
            peak = max(peak, st["running"])
            assert st["running"] <= 1 and st["queued"] <= 1, st
        # the last program's kernel is compiled (or already was)
        assert c.spec_wait() == 0
        got = c.classify(b)
        assert c.last_launch()["specialised"]
        assert_same(got, oracle_run(prog, b)[0], b, "last program, specialised")
        t0 = time.time()
        while cls.spec_pending()["active"] and time.time() - t0 < 60:
            time.sleep(0.1)
        st = cls.spec_pending()
        assert st["running"] == 0 and st["queued"] == 0, st
        assert peak <= 1
    finally:
        c.close()


def test_bench_extras_one_gpu(built, gpu):
    """bench.py --gpus 1 with its extras (the path the driver runs; the
    extras run in their own process): rc 0, one JSON line, every extra
    parity-checked and naming its kernel instantiation."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2",
                        "--warmup", "1", "--packets", "100000", "--no-cpu", "--no-runtime"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=400,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["parity_vs_oracle"] is True
    assert "kernel" in line["roofline"] and "name" in line["roofline"]["launch"]
    ex = line["extra"]
    assert "error" not in ex, ex.get("error")
    for name, e in ex.items():
        assert e["parity_vs_oracle"] is True, name
        assert e["launch"]["nw"] in (4, 8, 12, 16), name
    assert ex["config5"]["launch"]["div"] is True
    assert np.isfinite(line["value"])
