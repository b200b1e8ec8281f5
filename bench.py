#!/usr/bin/env python3
"""Benchmark: device-resident packet parse + PMR classification on MI355X.

Metric (BASELINE.json): Mpkts/s classified device-resident.  A "step" is one
pass of the hot path (one mi_cls_kernel launch through the libodp_cls.so C
ABI) over one batch of synthetic packets already resident in HBM.

Default workload: BASELINE config 3 (configs[2]) -- 1 M IMIX packets
(60/566/1514 B, 7:4:1, shuffled) per GPU, 256 PMRs over L3+L4 fields, the
largest configuration that fits one GPU.  The 64 B / 256-rule north-star case
(config "33") and configs 2, 4 and 5 are reported under `extra`.
Multi-GPU: one process per GPU (torchrun), each rank classifies its own 1 M
packet shard (weak scaling, no data-path collective); the timed region is
bracketed by barrier + synchronize and the max over ranks is taken.

`value` comes from ONE HIP stream: K launches back to back, so the kernel's
single-launch time (`roofline.kernel_ms`, HIP events on that same stream over
the same K launches) is never longer than `ms_per_step`.  A two-stream pass
(consecutive batches alternating over two streams, as a receive path with two
bursts in flight runs them) is reported as `pipelined` only.

Extra fields on the JSON line:
  roofline      HBM roofline of the dominant kernel: algorithmic bytes
                (min(len,128) + 6 B descriptor + 16 B result per packet) over
                the average launch duration; `traffic` = HBM bytes per launch
                from the committed rocprofv3 PMC summary (profiles/)
  issue         the kernel's VALU issue fraction (2 cycles per wave64 VALU
                instruction) from the committed PMC summary
  cpu_baseline  the oracle (scalar C restatement) timed on this host, 1 thread
                and one thread per available core (<= 16)
  parity_vs_oracle  every 16-B record of the timed batch == the oracle's
  e2e           end-to-end rate including pinned H2D / D2H (never `value`)
  extra         the other configurations, each timed and parity-checked
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
N_SIMD = 256 * 4           # 256 CUs x 4 SIMDs
SCLK_GHZ = 2.4             # peak engine clock
WORKLOAD = {2: "config2", 3: "config3", 4: "config4", 5: "config5", 33: "config3_64B",
            1: "config1", 20: "config2_norules", 34: "config3_64rules",
            35: "config3_sctp", 36: "config3_nested", 37: "config3_nested1024",
            38: "config3_9classes"}


_T0 = time.perf_counter()


def log(msg):
    """Progress on stderr (a long run keeps writing, so it is not taken to be hung)."""
    print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--n", "--packets", dest="n", type=int, default=1_000_000,
                    help="packets per GPU (spell it --packets under torchrun, which would "
                         "take --n as an abbreviation of its own options)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-runtime", action="store_true",
                    help="skip the ODP runtime receive-rate leg of e2e")
    ap.add_argument("--extras-json", default=None,
                    help="(internal) run only the extra configurations and write them to this "
                         "file: the main process runs them in a child process, so a failure "
                         "there cannot cost the headline line")
    ap.add_argument("--timed-only", action="store_true",
                    help="only the timed single-config pass (profiling runs)")
    ap.add_argument("--pktin-opt", type=lambda x: int(x, 0), default=0,
                    help="pktin checksum/drop option bits for the main line (profiling the "
                         "checksum path: 0x3C); valid checksums are written into the batch")
    ap.add_argument("--streams", type=int, default=1,
                    help="HIP streams the timed launches alternate over (1: back to back)")
    ap.add_argument("--rotate", type=int, default=4,
                    help="distinct device copies of the batch, used round-robin, so the "
                         "working set (R x batch) exceeds the 256 MiB Infinity Cache and every "
                         "step reads its packets from HBM")
    return ap.parse_args()


def make_workload(cfg, n, rank):
    from odp_amd import rules as R
    if cfg == 2:
        return R.config2(n, rank=rank)
    if cfg == 3:
        return R.config3(n, rank=rank)
    if cfg == 4:
        return R.config4(n, rank=rank)
    if cfg == 5:
        return R.config5(n, rank=rank)
    if cfg == 1:
        return R.config1(n)
    if cfg == 33:   # 64 B packets, 256 L3+L4 rules (north-star target case)
        return R.config3(n, size=60, rank=rank)
    if cfg == 20:   # config 2 traffic, default CoS only (parse + stage floor)
        b, p = R.config2(n, rank=rank)
        return b, [op for op in p if op[0] != "pmr"]
    if cfg == 34:   # config 3 IMIX traffic, 64 rules
        return R.config3(n, num_rules=64, rank=rank)
    if cfg == 35:   # config 3 IMIX traffic with a third of the packets SCTP
        return R.config3(n, rank=rank, sctp_frac=1.0 / 3.0)
    if cfg == 36:   # overlapping ACL: nested SIP/DIP prefixes, wildcard ports (256 rules)
        return R.config3_nested(n, rank=rank)
    if cfg == 37:   # the same shapes, 1024 rules (candidate lists)
        return R.config3_nested(n, rank=rank, scale=4)
    if cfg == 38:   # 256 rules over 9 key classes (linear scan)
        return R.config3_classes(n, rank=rank)
    raise ValueError(cfg)


def to_device(batch, dev):
    import numpy as np
    import torch
    t_buf = torch.from_numpy(np.ascontiguousarray(batch.buf)).to(dev)
    t_off = torch.from_numpy(batch.off.view(np.int32)).to(dev)
    t_len = torch.from_numpy(batch.len.view(np.int16)).to(dev)
    t_out = torch.empty((batch.n, 4), dtype=torch.int32, device=dev)
    return t_buf, t_off, t_len, t_out


def time_device(c, batch, dev, steps, warmup, dist_on=False, rotate=1, streams=1):
    """Warmup, then time `steps` launches; returns (wall_s, avg_kernel_ms, out tensor).
    With rotate > 1 the launches cycle over that many device copies of the
    batch (and of the result array), so consecutive steps do not re-read
    the same bytes from the Infinity Cache."""
    import torch
    import torch.distributed as dist
    copies = [to_device(batch, dev)]
    for _ in range(1, max(1, rotate)):
        b0 = copies[0]
        copies.append(tuple(t.clone() for t in b0[:3]) + (torch.empty_like(b0[3]),))
    stream = torch.cuda.current_stream(dev)
    # streams > 1: consecutive batches alternate between streams (copy i
    # always runs on stream i % streams, so no two in-flight launches share
    # buffers)
    strm = [stream] + [torch.cuda.Stream(dev) for _ in range(1, max(1, streams))]
    if len(copies) % len(strm):
        raise ValueError("rotate must be a multiple of streams")
    arglist = [(cb.data_ptr(), co.data_ptr(), cl.data_ptr(), batch.n, cout.data_ptr(),
                strm[i % len(strm)].cuda_stream)
               for i, (cb, co, cl, cout) in enumerate(copies)]
    t_out = copies[0][3]
    for i in range(warmup):
        rc = c.classify_device(*arglist[i % len(arglist)])
        assert rc == 0, rc
    torch.cuda.synchronize(dev)
    # HIP events on the launch stream bracket the timed region (no per-launch
    # events inside it: each record is a host call between launches); the
    # average launch duration is their span / steps
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for s_ in strm[1:]:
        s_.wait_event(ev0)
    for i in range(steps):
        rc = c.classify_device(*arglist[i % len(arglist)])
        if rc:
            raise RuntimeError(f"classify failed: {rc}")
    for s_ in strm[1:]:
        stream.wait_stream(s_)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    wall = time.perf_counter() - t0
    kms = ev0.elapsed_time(ev1) / steps
    # the last launch on copy 0 wrote t_out: rerun it so the returned records
    # belong to copy 0's batch whatever `steps` was
    c.classify_device(*arglist[0])
    torch.cuda.synchronize(dev)
    return wall, kms, t_out


def records(t_out, n):
    import numpy as np
    from odp_amd import rules as R
    return t_out.cpu().numpy().view(np.uint8).reshape(-1)[: 16 * n].view(R.RESULT_DTYPE)


def oracle_parity(prog, batch, got, threads=16, pktin_opt=0):
    """Bit-exact check of every record against the oracle (multi-threaded)."""
    import numpy as np
    from oracle.oracle import Oracle
    o = Oracle(pktin_opt=pktin_opt)
    o.apply(prog)
    exp = o.classify(batch, threads=threads)
    return bool(np.array_equal(got, exp))


def time_e2e(c, batch, dev, steps=5):
    """Pinned host batch -> H2D -> kernel -> D2H results, per step."""
    import numpy as np
    import torch
    h_buf = torch.from_numpy(np.ascontiguousarray(batch.buf)).pin_memory()
    h_off = torch.from_numpy(batch.off.view(np.int32)).pin_memory()
    h_len = torch.from_numpy(batch.len.view(np.int16)).pin_memory()
    h_out = torch.empty((batch.n, 4), dtype=torch.int32).pin_memory()
    d_buf = torch.empty_like(h_buf, device=dev)
    d_off = torch.empty_like(h_off, device=dev)
    d_len = torch.empty_like(h_len, device=dev)
    d_out = torch.empty((batch.n, 4), dtype=torch.int32, device=dev)
    sp = torch.cuda.current_stream(dev).cuda_stream

    def step():
        d_buf.copy_(h_buf, non_blocking=True)
        d_off.copy_(h_off, non_blocking=True)
        d_len.copy_(h_len, non_blocking=True)
        assert c.classify_device(d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), batch.n,
                                 d_out.data_ptr(), sp) == 0
        h_out.copy_(d_out, non_blocking=True)
    step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / steps
    h2d = batch.buf.nbytes + 6 * batch.n
    out = {"copy": {"mpkts_per_s": round(batch.n / dt / 1e6, 2), "ms_per_step": round(dt * 1e3, 4),
                    "h2d_bytes": int(h2d), "d2h_bytes": 16 * batch.n,
                    "note": "pinned H2D of the whole packed batch + descriptors, kernel, "
                            "D2H of the records"}}
    # zero copy: the kernel reads the packets' header windows and the
    # descriptors straight from page-locked host memory over PCIe and writes
    # the records back the same way -- no staging copy, only the bytes the
    # kernel reads cross the link
    from odp_amd import cls
    hb = cls.PinnedArray(batch.buf.nbytes + 64)
    ho = cls.PinnedArray(4 * batch.n)
    hl = cls.PinnedArray(2 * batch.n)
    hr = cls.PinnedArray(16 * batch.n)
    try:
        hb.u8[: batch.buf.nbytes] = batch.buf
        ho.view(np.uint32)[:] = batch.off
        hl.view(np.uint16)[:] = batch.len

        def zstep():
            assert c.classify_device(hb.ptr, ho.ptr, hl.ptr, batch.n, hr.ptr, sp) == 0
        zstep()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            zstep()
        torch.cuda.synchronize(dev)
        dz = (time.perf_counter() - t0) / steps
        same = bool(np.array_equal(hr.view(np.uint8, 16 * batch.n),
                                   h_out.numpy().view(np.uint8).reshape(-1)))
        out["zero_copy"] = {"mpkts_per_s": round(batch.n / dz / 1e6, 2),
                            "ms_per_step": round(dz * 1e3, 4),
                            "link_bytes": int(batch.header_bytes()),
                            "records_equal_copy_path": same,
                            "note": "kernel reads header windows + descriptors from pinned host "
                                    "memory and writes the records there (no staging copy)"}
    finally:
        for a in (hb, ho, hl, hr):
            a.close()
    return out


def time_runtime(batch, prog, n_frames=200_000, loops=10):
    """Packets / s through the ODP runtime's receive path on this batch's
    traffic: a pcap pktio replaying n_frames frames `loops` times, GPU
    classification per burst (odp_amd_cls_classify_host), CoS enqueue and
    the application draining the queues -- through odp_pktin_recv (DIRECT)
    and through the scheduler (SCHED).  tests/_bin/rx_driver in rate mode."""
    import subprocess
    import tempfile
    from tests import rt_helpers as H
    n = min(n_frames, batch.n)
    frames = [batch.frame(i) for i in range(n)]
    out = {}
    with tempfile.TemporaryDirectory() as td:
        pc = os.path.join(td, "in.pcap")
        rules = os.path.join(td, "rules.txt")
        H.write_pcap(pc, frames)
        H.write_rules(rules, prog)
        # the loop interface carries 32 k frames per round (a few bursts in
        # flight on the "wire", as a loopback pktio does), for n x loops packets
        pcl = os.path.join(td, "in_loop.pcap")
        nl = min(n, 32768)
        H.write_pcap(pcl, frames[:nl])
        loop_rounds = max(1, n * loops // nl)
        runs = {"direct": ([f"pcap:in={pc}:loops={loops}", rules, "direct", "4", "0", "1"], {}),
                "sched": ([f"pcap:in={pc}:loops={loops}", rules, "sched", "4", "0", "1"], {}),
                # loop pktio: the capture sent into the loop interface (its
                # packets in page-locked pool memory), received in place;
                # `loops` rounds of send (not timed) + receive (timed)
                "loop_direct": (["loop", rules, "direct", "4", "0", "1", pcl],
                                {"RX_LOOP_ROUNDS": str(loop_rounds), "RX_POOL_NUM": "65536"})}
        for mode, (args, extra_env) in runs.items():
            env = dict(os.environ, RX_COUNT_ONLY="1", **extra_env)
            r = subprocess.run([H.DRIVER] + args, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                               text=True, timeout=300, env=env)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("R ")]
            if r.returncode or not line:
                out[mode] = {"error": (r.stderr or r.stdout)[-300:]}
                continue
            pk, ns = (int(x) for x in line[-1].split()[1:3])
            out[mode] = {"mpkts_per_s": round(pk / ns * 1e3, 3), "packets_delivered": pk}
            st = [ln for ln in r.stdout.splitlines() if ln.startswith("S ")]
            if st:
                v = [int(x) for x in st[-1].split()[1:5]]
                out[mode].update(in_packets=v[0], in_errors=v[1], in_discards=v[2])
    out["note"] = (f"ODP runtime receive path, steady state after odp_pktio_start ({n} "
                   f"frames x {loops} loops of this workload's traffic; 4096-frame bursts "
                   f"pipelined, each a receive chain on the GPU (classify, decide, deliver; "
                   f"four bursts in flight on two streams): per-frame fates, packets and "
                   f"queue groups decided, packet metadata and frame copies written into "
                   f"page-locked pools by the GPU; CoS enqueue; one "
                   f"application thread draining the queues): a pcap pktio whose page-locked "
                   f"frame store the GPU reads in place through odp_pktin_recv (direct) and "
                   f"odp_schedule (sched), and the loop pktio (loop_direct: rounds of 32768 "
                   f"frames sent into the loop interface, classified in place in pool memory; "
                   f"only the receive rounds are timed) -- tools/rx_rate.sh splits the time per phase")
    return out


def cpu_baseline(prog, batch, seconds):
    """The scalar C restatement (oracle) on this host: first 1 thread, then
    one thread per available core (up to 16, the GPU box's CPU share), each
    thread on a disjoint slice, repeated passes over the batch for about
    `seconds` / 2 each."""
    from oracle.oracle import Oracle
    o = Oracle()
    o.apply(prog)

    def timed(threads, budget, sample):
        t0 = time.perf_counter()
        o.classify(sample, threads=threads)
        passes = 1
        while time.perf_counter() - t0 < budget:
            o.classify(sample, threads=threads)
            passes += 1
        return passes, time.perf_counter() - t0

    one = batch.slice(0, min(batch.n, 200_000))
    p1, dt1 = timed(1, seconds / 2, one)
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    pn, dtn = timed(cores, seconds / 2, batch)
    v1 = p1 * one.n / dt1 / 1e6
    vn = pn * batch.n / dtn / 1e6
    return {"value": round(vn, 3), "unit": "Mpkts/s", "cores": cores, "kind": "port",
            "single_core": round(v1, 3),
            "sample": f"{pn} passes over the same {batch.n}-packet batch with {cores} threads "
                      f"({dtn:.1f} s) and {p1} passes over its first {one.n} packets with 1 "
                      f"thread ({dt1:.1f} s); oracle/odp_cls_oracle.c, gcc -O2, disjoint "
                      f"slices per thread"}


def load_pmc(cfg, n, name=None):
    """The committed PMC summary of a workload (profiles/pmc_traffic.json,
    written by tools/pmc_summary.py); name: an extra's own key (e.g.
    config3_generic), else the config's workload name."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if name:
            return d.get(f"{name}_n{n}")
        return d.get(f"{WORKLOAD[cfg]}_n{n}") or d.get(f"config{cfg}_n{n}")
    except (OSError, ValueError, KeyError):
        return None


def issue_roof(kms, pmc):
    """The kernel's VALU issue fraction from the committed PMC summary: a
    wave64 VALU instruction occupies a SIMD-32 for 2 cycles when the SIMD
    runs more than one wave (MI355X_MICROARCH.md, wave scheduling; these
    kernels run 4 waves per SIMD), so issue frac = SQ_INSTS_VALU x 2 /
    (kernel time x 2.4 GHz x 1024 SIMDs).  None without a PMC summary."""
    v = (pmc or {}).get("SQ_INSTS_VALU_per_launch")
    if not v:
        return None
    issue = v * 2.0 / (kms * 1e-3 * SCLK_GHZ * 1e9 * N_SIMD)
    return {"valu_insts_per_launch": v, "valu_issue_frac": round(issue, 4),
            "note": "SQ_INSTS_VALU x 2 cycles / (kernel time x "
                    f"{SCLK_GHZ} GHz x {N_SIMD} SIMDs), PMC from "
                    f"{(pmc or {}).get('source')}"}


def bench_cfg(cls, cfg, a, dev, local, steps, warmup, pktin_opt=0, parity=True, full_bytes=False,
              env=None, name=None):
    """Time one extra configuration (single stream and two streams), check
    its records against the oracle.  env: library knobs set for this entry
    only (e.g. MI_CLS_JIT=0: the generic kernels)."""
    env = env or {}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        e = _bench_cfg(cls, cfg, a, dev, local, steps, warmup, pktin_opt, parity, full_bytes, name)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    if env:
        e["env"] = env
    return e


def _bench_cfg(cls, cfg, a, dev, local, steps, warmup, pktin_opt, parity, full_bytes, name):
    import numpy as np
    from odp_amd import pktgen as pg, rules as R
    log(f"extra {WORKLOAD[cfg]}{' pktin_opt' if pktin_opt else ''}: workload")
    b2, p2 = make_workload(cfg, a.n, 0)
    if pktin_opt:
        pg.set_checksums(b2)
    c2 = cls.Classifier(gpu=local)
    c2.apply(p2)
    if pktin_opt:
        c2.set_pktin_opt(pktin_opt)
    log("  rules loaded, waiting for the specialised kernel")
    spec = c2.spec_wait() == 0
    info = c2.program_info()
    engine = ("linear scan" if info["blocks"] == 0 else
              ["direct", "candidate lists", "bitmap", "wide bitmap", "single candidate"][
                  [info["direct"], info["candidate"], info["bitmap"], info["wide"],
                   info["cand1"]].index(max(info["direct"], info["candidate"], info["bitmap"],
                                            info["wide"], info["cand1"]))])
    # the instantiation the launches take, logged before the first timed
    # launch (a fault record then names it)
    launch = predicted_launch(c2, b2, dev)
    log(f"  specialised={spec}, engine={engine}, kernel {launch['name']}: timing")
    w1, k1, t_out = time_device(c2, b2, dev, steps, warmup, rotate=a.rotate)
    launch = c2.last_launch()
    got = records(t_out, b2.n).copy()
    w2, _, _ = time_device(c2, b2, dev, steps, warmup, rotate=a.rotate, streams=2)
    c2.close()
    nbytes = (int(b2.len.astype(np.int64).sum()) + 22 * b2.n) if full_bytes else b2.header_bytes()
    e = {"workload": WORKLOAD[cfg], "rules": R.rule_count(p2), "engine": engine,
         "specialised": spec, "launch": launch,
         "mpkts_per_s": round(b2.n * steps / w1 / 1e6, 2),
         "mpkts_per_s_2streams": round(b2.n * steps / w2 / 1e6, 2),
         "kernel_ms": round(k1, 5), "bytes_per_launch": nbytes,
         "roofline_frac": round(nbytes / (k1 * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)}
    pmc = load_pmc(cfg, b2.n, name) if not pktin_opt else None
    if pmc:
        e["traffic"] = pmc.get("hbm_bytes_per_launch")
    if pmc:
        e["issue"] = issue_roof(k1, pmc)
    if parity:
        log("  oracle parity")
        o_prog = p2
        if pktin_opt:
            from oracle.oracle import Oracle
            o = Oracle(pktin_opt=pktin_opt)
            o.apply(o_prog)
            e["parity_vs_oracle"] = bool(np.array_equal(got, o.classify(b2, threads=16)))
            e["checksum_ok"] = bool(np.all((got["err"] & 0x44) == 0))
        else:
            e["parity_vs_oracle"] = oracle_parity(o_prog, b2, got)
    return e


def predicted_launch(c, batch, dev):
    """One launch over the batch's first 64 packets (same rules, same
    options: the kernel choice does not depend on n), returning the
    instantiation the timed launches will take."""
    import torch
    small = batch.slice(0, min(64, batch.n))
    tb, to, tl, tout = to_device(small, dev)
    rc = c.classify_device(tb.data_ptr(), to.data_ptr(), tl.data_ptr(), small.n, tout.data_ptr(),
                           torch.cuda.current_stream(dev).cuda_stream)
    if rc:
        raise RuntimeError(f"classify failed: {rc}")
    torch.cuda.synchronize(dev)
    return c.last_launch()


def run_extras(a, dev, local):
    """The extra configurations (this process: --extras-json)."""
    from odp_amd import cls
    extra = {}
    k_steps = max(5, a.steps // 2)
    for cfg in (33, 2, 4, 5, 36, 37, 38):
        if cfg == a.config:
            continue
        extra[WORKLOAD[cfg]] = bench_cfg(cls, cfg, a, dev, local, k_steps, 3,
                                         parity=not a.no_parity)
    # what an application gets on the generic kernels: right after a rule
    # change (the specialised kernel compiles in the background for 1-4 s)
    # or without the compiler (MI_CLS_JIT=0); config 5 on the generic tree
    # kernel instead of its tree plan (MI_CLS_NO_PLAN=1)
    extra["config3_generic"] = bench_cfg(cls, 3, a, dev, local, k_steps, 3, parity=not a.no_parity,
                                         env={"MI_CLS_JIT": "0"}, name="config3_generic")
    extra["config5_generic"] = bench_cfg(cls, 5, a, dev, local, k_steps, 3, parity=not a.no_parity,
                                         env={"MI_CLS_NO_PLAN": "1"}, name="config5_generic")
    # pktin checksum validation (IPv4 header, UDP/TCP sums over the whole
    # frame): config 3 IMIX with valid checksums; the kernel reads every
    # frame byte, so the bytes are frame + 22 B
    extra["config3_checksums"] = bench_cfg(cls, 3, a, dev, local, k_steps, 3, pktin_opt=0x3C,
                                           parity=not a.no_parity, full_bytes=True)
    # the same with a third of the packets SCTP (CRC-32C over the whole frame)
    extra["config3_sctp_checksums"] = bench_cfg(cls, 35, a, dev, local, k_steps, 3,
                                                pktin_opt=0x3C, parity=not a.no_parity,
                                                full_bytes=True)
    return extra


def extras_child(a):
    """Run the extras in a child process (started, not exec'd: this process
    has initialised the GPU) and return their entries, or an error entry
    with the child's exit status -- the headline line is printed either way."""
    import subprocess
    import tempfile
    fd, path = tempfile.mkstemp(prefix="bench_extra_", suffix=".json")
    os.close(fd)
    cmd = [sys.executable, os.path.abspath(__file__), "--extras-json", path,
           "--steps", str(a.steps), "--warmup", str(a.warmup), "--config", str(a.config),
           "--packets", str(a.n), "--rotate", str(a.rotate)]
    if a.no_parity:
        cmd.append("--no-parity")
    try:
        rc = subprocess.call(cmd, timeout=900)   # progress lines go straight to stderr
        if rc != 0:
            return {"error": f"extras process exited with status {rc}"}
        with open(path) as f:
            return json.load(f)
    except subprocess.TimeoutExpired:
        return {"error": "extras process timed out (900 s)"}
    finally:
        os.unlink(path)


def dist_init_kwargs(backend, local):
    """torch.distributed.init_process_group arguments of one rank: RCCL
    ("nccl") binds the rank's process group to its own device (device_id =
    cuda:LOCAL_RANK, so the one reduction per run never lands on another
    rank's GPU); gloo (CPU rehearsal) takes no device."""
    import torch
    if backend == "nccl":
        return {"backend": "nccl", "device_id": torch.device(f"cuda:{local}")}
    return {"backend": backend}


def reduce_ranks(dist, red_dev, wall, n, kms, bytes_launch, parity):
    """The multi-rank reductions of one timed run (no data-path collective:
    these are the only collectives).  Returns the max wall time over ranks,
    the packets all ranks classified per step, every rank's kernel_ms and
    algorithmic bytes per launch (rank order), the aggregate roofline
    achieved = sum of the ranks' bytes / the slowest rank's kernel time
    (GB/s), and parity AND-ed over the ranks (None if no rank checked)."""
    import torch
    world = dist.get_world_size()
    mine = torch.tensor([wall, float(n), kms, float(bytes_launch),
                         -1.0 if parity is None else float(bool(parity))],
                        dtype=torch.float64, device=red_dev)
    allv = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine)
    rows = [[float(x) for x in t.cpu().tolist()] for t in allv]
    walls = [r[0] for r in rows]
    k = [r[2] for r in rows]
    par = [r[4] for r in rows]
    return {"wall": max(walls), "packets": int(sum(r[1] for r in rows)),
            "kernel_ms": [round(x, 5) for x in k],
            "bytes_per_launch": [int(r[3]) for r in rows],
            "achieved_gbs": sum(r[3] for r in rows) / (max(k) * 1e-3) / 1e9,
            "parity": None if all(p < 0 for p in par) else all(p == 1.0 for p in par)}


def launch_ranks(n):
    """`bench.py --gpus N` started without a launcher: start one fresh worker
    process per GPU (torch.distributed.run, rendezvous on 127.0.0.1) and
    return its exit code.  Runs before this process touches the GPU (only
    torch.cuda.device_count(), which does not initialise it); fails loudly
    when fewer than N devices are visible (BENCH_SAME_DEVICE=1 rehearses N
    ranks on one device)."""
    import socket
    import subprocess
    import torch
    have = torch.cuda.device_count()
    if have < n and not os.environ.get("BENCH_SAME_DEVICE"):
        print(f"bench.py: --gpus {n} requested but {have} GPU(s) visible", file=sys.stderr)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
           str(n), "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.call(cmd, env=env)


def main():
    a = parse_args()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if os.environ.get("BENCH_SAME_DEVICE"):   # multi-rank rehearsal on one GPU (tests)
        local = 0
    dist_on = world > 1
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    if dist_on:
        torch.cuda.set_device(local)
        dist.init_process_group(**dist_init_kwargs(backend, local))
    dev = torch.device(f"cuda:{local}")

    from odp_amd import cls, rules as R
    if a.extras_json:
        extra = run_extras(a, dev, local)
        with open(a.extras_json, "w") as f:
            json.dump(extra, f)
        return
    # The node's capture is world x n packets; rank r classifies slice r of
    # it, cut by the product's multi-GPU sharding (mi_cls_shard, the cut
    # mi_cls_group_classify_host makes: contiguous, balanced by header
    # bytes) over the capture's frame lengths (IMIX drawn from one node-wide
    # seed); the slice's packets are generated with the rank's seed.  No
    # collective on the data path (weak scaling: ~n packets per GPU).
    n_rank = a.n
    if world > 1:
        import numpy as np
        from odp_amd import pktgen as pg
        if a.config in (3, 4, 5, 34):
            node_lens = pg.imix_lens(np.random.default_rng(pg.seed_for(a.config) ^ 0x5EED),
                                     a.n * world)
        else:
            node_lens = np.full(a.n * world, 60)
        bnd = cls.shard(node_lens.astype(np.uint16), world)
        n_rank = int(bnd[rank + 1] - bnd[rank])
    log(f"workload {WORKLOAD[a.config]}: {n_rank} packets")
    batch, prog = make_workload(a.config, n_rank, rank)
    log("rules")
    c = cls.Classifier(gpu=local)
    c.apply(prog)
    if a.pktin_opt:
        from odp_amd import pktgen as pg
        pg.set_checksums(batch)
        c.set_pktin_opt(a.pktin_opt)
    # rule load is control plane: the program-specialised kernel (compiled in
    # the background after the rules are loaded) is ready before timing
    spec = c.spec_wait() == 0
    launch = predicted_launch(c, batch, dev)
    log(f"specialised={spec}, kernel {launch['name']}: timing")

    wall, kms, t_out = time_device(c, batch, dev, a.steps, a.warmup, dist_on, a.rotate,
                                   a.streams)
    launch = c.last_launch()
    red_dev = dev if backend == "nccl" else torch.device("cpu")   # where reductions run
    # with checksum options the kernel reads every frame byte
    bytes_launch = batch.header_bytes() if not a.pktin_opt else \
        int(batch.len.astype("int64").sum()) + 22 * batch.n
    out = records(t_out, batch.n).copy()
    parity = None
    if not a.no_parity and not a.timed_only:
        # every rank checks its own shard: all of its records bit-exact vs the oracle
        log("oracle parity")
        parity = oracle_parity(prog, batch, out, pktin_opt=a.pktin_opt)
    ranks = None
    if dist_on:
        ranks = reduce_ranks(dist, red_dev, wall, batch.n, kms, bytes_launch, parity)
        wall = ranks["wall"]
        total_pkts = ranks["packets"] * a.steps
        parity = ranks["parity"]
        achieved = ranks["achieved_gbs"]
    else:
        total_pkts = batch.n * a.steps
        achieved = bytes_launch / (kms * 1e-3) / 1e9
    value = total_pkts / wall / 1e6
    res = None
    if rank == 0:
        pmc = load_pmc(a.config, batch.n)
        line = {
            "metric": "Mpkts/s classified device-resident",
            "value": round(value, 2),
            "unit": "Mpkts/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(wall / a.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": WORKLOAD[a.config], "packets_per_gpu": batch.n,
                       "packets_total": total_pkts // a.steps,
                       "rules": R.rule_count(prog), "cos": R.cos_count(prog),
                       "frame_bytes": "60 (64 B on the wire)" if a.config in (2, 33)
                       else "IMIX 60/566/1514 7:4:1" if a.config == 3 else "mixed",
                       "streams": a.streams, "rotate": a.rotate,
                       "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": (pmc or {}).get("hbm_bytes_per_launch"),
                         "kernel": "mi_cls_kernel" + (" (program-specialised)" if spec and
                                                       not a.pktin_opt else ""),
                         "launch": launch,
                         "kernel_ms": round(max(ranks["kernel_ms"]) if ranks else kms, 5),
                         "bytes_per_launch": bytes_launch,
                         "traffic_source": (pmc or {}).get("source")},
        }
        if ranks:
            # aggregate roofline: every rank's algorithmic bytes over the
            # slowest rank's kernel time, against world x the HBM peak
            line["roofline"].update(
                frac=round(achieved / (HBM_PEAK_GBS * world), 5), peak=HBM_PEAK_GBS * world,
                per_rank_kernel_ms=ranks["kernel_ms"],
                per_rank_bytes_per_launch=ranks["bytes_per_launch"],
                aggregate="sum of the ranks' bytes per launch / the slowest rank's kernel_ms")
        if parity is not None:
            # AND over every rank's shard (each checked against the oracle)
            line["parity_vs_oracle"] = parity
        if world == 1 and not a.timed_only:
            if pmc:
                line["issue"] = issue_roof(kms, pmc)
            w2, _, _ = time_device(c, batch, dev, a.steps, a.warmup, rotate=a.rotate, streams=2)
            line["pipelined"] = {"streams": 2, "mpkts_per_s": round(batch.n * a.steps / w2 / 1e6, 2),
                                 "ms_per_step": round(w2 / a.steps * 1e3, 5)}
            log("e2e")
            try:
                line["e2e"] = time_e2e(c, batch, dev)
            except Exception as e:   # recorded, never fatal
                line["e2e"] = {"error": str(e)}
            if not a.no_runtime:
                log("ODP runtime receive rate")
                try:
                    line["e2e"]["runtime"] = time_runtime(batch, prog)
                except Exception as e:   # recorded, never fatal
                    line["e2e"]["runtime"] = {"error": str(e)}
            if not a.no_cpu:
                log("cpu baseline")
                line["cpu_baseline"] = cpu_baseline(prog, batch, a.cpu_seconds)
            if not a.no_extra:
                log("extras (child process)")
                line["extra"] = extras_child(a)
        res = line
        print(json.dumps(res), flush=True)
    c.close()
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
