"""Shared test helpers: run one rule program + batch through the HIP path and
the CPU oracle and compare every result record bit for bit."""
import numpy as np

from odp_amd import rules as R


def oracle_run(prog, batch, limits=(255, 8192, 4096), pktin_opt=0):
    from oracle.oracle import Oracle
    o = Oracle(limits=limits, pktin_opt=pktin_opt)
    o.apply(prog)
    return o.classify(batch), o


def gpu_run(prog, batch, limits=(255, 8192, 4096), pktin_opt=0, spec=False):
    """spec: wait for the program-specialised kernel before classifying (a
    flat program must get one); otherwise whichever kernel is ready."""
    from odp_amd.cls import Classifier
    c = Classifier(gpu=0, limits=limits)
    try:
        c.apply(prog)
        if pktin_opt:
            c.set_pktin_opt(pktin_opt)
        if spec:
            rc = c.spec_wait()
            # a flat program always has one (trees: when the default CoS has a block)
            assert rc == 0 or (rc == 1 and c.program_info()["flat_engine"] < 0), rc
        return c.classify(batch)
    finally:
        c.close()


def assert_same(got, exp, batch=None, what=""):
    assert got.shape == exp.shape, (got.shape, exp.shape)
    if np.array_equal(got, exp):
        return
    bad = np.nonzero(got != exp)[0]
    i = int(bad[0])
    msg = [f"{what}: {bad.size} of {got.size} records differ; first at {i}:",
           f"  gpu    {got[i]}", f"  oracle {exp[i]}"]
    if batch is not None:
        msg.append(f"  frame  {batch.frame(i).hex()}")
    raise AssertionError("\n".join(msg))


def summary(res):
    out = np.bincount(res["outcome"], minlength=5)
    return {"enq": int(out[R.OUT_ENQ]), "cos_drop": int(out[R.OUT_COS_DROP]),
            "discard": int(out[R.OUT_DISCARD]), "parse_drop": int(out[R.OUT_PARSE_DROP]),
            "loop": int(out[R.OUT_LOOP])}
