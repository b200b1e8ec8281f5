#!/usr/bin/env python3
"""A/B kernel timing on the GPU box: for each library build and config, one
`bench.py --timed-only` run (single stream, HIP events on the launch
stream), printing kernel µs and HBM fraction, plus the DIAG line a
diagnostic build (-DDIAG_STAMPS) writes to stderr.

Usage (repo root, through gpurun):
  python tools/ab.py --libs odp_amd,build/vst --configs 3,33,2 [--n 1000000,4000000]
                     [--steps 20] [--env MI_CLS_WPB=16] [--bench-args "--rotate 1"]
                     [--pmc "SQ_INSTS_VALU SQ_INSTS_SALU ..."]
With --pmc each run is a rocprofv3 counter pass instead (run from /tmp, one
pass per run, at most 8 SQ_ counters) and the counters are printed per
64-packet tile.  Each run has its own time limit; the first failure ends the
script.
"""
import argparse
import collections
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="odp_amd")
    ap.add_argument("--configs", default="3")
    ap.add_argument("--n", default="1000000")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--env", action="append", default=[])
    ap.add_argument("--bench-args", default="")
    ap.add_argument("--timeout", type=int, default=180)
    ap.add_argument("--pmc", default="")
    a = ap.parse_args()
    extra_env = dict(e.split("=", 1) for e in a.env)
    for cfg in a.configs.split(","):
        for n in a.n.split(","):
            for lib in a.libs.split(","):
                env = dict(os.environ, ODP_AMD_LIB_DIR=os.path.join(ROOT, lib), **extra_env)
                cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", cfg,
                       "--packets", n, "--steps", str(a.steps), "--warmup", "5",
                       "--timed-only"] + a.bench_args.split()
                if a.pmc:
                    pmc_run(a, cmd, env, cfg, n, lib)
                    continue
                r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                   text=True, timeout=a.timeout)
                if r.returncode:
                    print(f"FAILED config {cfg} n {n} lib {lib}: rc {r.returncode}\n{r.stderr[-2000:]}")
                    sys.exit(1)
                d = json.loads(r.stdout.strip().splitlines()[-1])
                diag = [ln for ln in r.stderr.splitlines() if ln.startswith("DIAG")]
                print(f"config {cfg:>3} n {n:>8} {lib:<22} kernel_us "
                      f"{d['roofline']['kernel_ms'] * 1e3:8.2f}  frac {d['roofline']['frac']:.4f}"
                      + (f"\n    {diag[-1]}" if diag else ""), flush=True)


def pmc_run(a, cmd, env, cfg, n, lib):
    out = os.path.join(ROOT, "gpurun_out", "ab_pmc", f"c{cfg}_n{n}_{lib.replace('/', '_')}")
    pc = ["rocprofv3", "--pmc"] + a.pmc.split() + ["--output-format", "csv", "-d", out, "-o",
                                                   "p", "--"] + cmd
    r = subprocess.run(["timeout", "-s", "KILL", str(a.timeout)] + pc, env=env, cwd="/tmp",
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode:
        print(f"FAILED pmc config {cfg} lib {lib}: rc {r.returncode}\n{r.stdout[-2000:]}")
        sys.exit(1)
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(out, "**", "p_counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "mi_cls" in row["Kernel_Name"]:
                agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
    tiles = (int(n) + 63) // 64
    print(f"config {cfg:>3} n {n:>8} {lib:<22} per tile: " + " ".join(
        f"{k.replace('SQ_INSTS_', '').replace('SQ_', '')}={sum(v) / len(v) / tiles:.1f}"
        for k, v in sorted(agg.items())), flush=True)


if __name__ == "__main__":
    main()
