#!/usr/bin/env python3
"""Benchmark: device-resident packet parse + PMR classification on MI355X.

Metric (BASELINE.json): Mpkts/s classified device-resident.  A "step" is one
pass of the hot path (one mi_cls_kernel launch through the libodp_cls.so C
ABI) over one batch of synthetic packets already resident in HBM.

Default workload: BASELINE config 2 -- 1 M x 64 B (60 B buffer) IPv4/UDP per
GPU, 16 SIP-prefix PMRs (configs[1], the single-GPU config the metric is
quoted on).  Multi-GPU: one process per GPU (torchrun), each rank classifies
its own 1 M-packet shard (weak scaling, no data-path collective); the timed
region is bracketed by barrier + synchronize and the max over ranks is taken.

Extra fields on the JSON line:
  roofline      HBM roofline of the dominant kernel: algorithmic bytes
                (min(len,128) + 6 B descriptor + 16 B result per packet) over
                the average launch duration, from HIP events on the launch
                stream in a second, single-stream pass (launches back to back,
                no overlap, so it agrees with rocprofv3's per-dispatch
                average); `pipelined_*` are the same bytes over the
                per-step time of the two-stream `value` pass
  cpu_baseline  the oracle (scalar C restatement, 1 thread) timed on this
                host over repeated passes of the same batch
  e2e           end-to-end rate including pinned H2D of the batch and D2H of
                the results (recorded, never `value`)
  extra         config 3 (IMIX, 256 rules) and the 64 B / 256-rule north-star
                case, timed the same way (rank 0, N=1 only)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--n", type=int, default=1_000_000, help="packets per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--streams", type=int, default=2,
                    help="HIP streams the consecutive batches alternate over (the timed "
                         "`value` pass); the roofline pass always uses one stream")
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
    # streams > 1: consecutive batches alternate between streams, so one
    # launch's ramp-up overlaps the previous one's tail (a pipelined receive
    # path keeps several bursts in flight the same way); copy i always runs on
    # stream i % streams, so no two in-flight launches share buffers
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
    # average launch duration is their span / steps (kernels + the gaps
    # between back-to-back launches)
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
        c.classify_device(*arglist[i % len(arglist)])
    for s_ in strm[1:]:
        stream.wait_stream(s_)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    wall = time.perf_counter() - t0
    kms = ev0.elapsed_time(ev1) / steps
    return wall, kms, t_out


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
    return {"mpkts_per_s": batch.n / dt / 1e6, "ms_per_step": dt * 1e3,
            "h2d_bytes": int(h2d), "d2h_bytes": 16 * batch.n,
            "note": "pinned H2D of the whole packed batch + descriptors, kernel, D2H results"}


def cpu_baseline(prog, batch, seconds, out_gpu):
    """The scalar C restatement (oracle) on this host: first 1 thread, then
    one thread per available core (up to 16, the GPU box's CPU share), each
    thread on a disjoint slice, repeated passes over the batch for about
    `seconds` / 2 each; also checks the GPU records of the timed batch bit
    for bit against the single-thread pass."""
    import numpy as np
    from oracle.oracle import Oracle
    o = Oracle()
    o.apply(prog)

    def timed(threads, budget):
        t0 = time.perf_counter()
        res = o.classify(batch, threads=threads)
        passes = 1
        while time.perf_counter() - t0 < budget:
            o.classify(batch, threads=threads)
            passes += 1
        return res, passes, time.perf_counter() - t0

    exp, p1, dt1 = timed(1, seconds / 2)
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    _, pn, dtn = timed(cores, seconds / 2)
    parity = bool(np.array_equal(out_gpu, exp))
    v1 = p1 * batch.n / dt1 / 1e6
    vn = pn * batch.n / dtn / 1e6
    return {"value": round(vn, 3), "unit": "Mpkts/s", "cores": cores, "kind": "port",
            "single_core": round(v1, 3),
            "sample": f"{pn} passes over the same {batch.n}-packet batch with {cores} threads "
                      f"({dtn:.1f} s) and {p1} passes with 1 thread ({dt1:.1f} s); "
                      f"oracle/odp_cls_oracle.c, gcc -O2, disjoint slices per thread"}, parity


def load_traffic(cfg, n):
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        e = d.get(f"config{cfg}_n{n}")
        return None if e is None else e["hbm_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        return None


def main():
    a = parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist_on = world > 1
    if dist_on:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")

    from odp_amd import cls, rules as R
    batch, prog = make_workload(a.config, a.n, rank)
    c = cls.Classifier(gpu=local)
    c.apply(prog)

    wall, kms_pipe, t_out = time_device(c, batch, dev, a.steps, a.warmup, dist_on, a.rotate,
                                        a.streams)
    if a.streams > 1:
        _, kms, _ = time_device(c, batch, dev, a.steps, a.warmup, dist_on, a.rotate, 1)
    else:
        kms = kms_pipe
    if dist_on:
        t = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    total_pkts = batch.n * world * a.steps
    value = total_pkts / wall / 1e6
    bytes_launch = batch.header_bytes()
    achieved = bytes_launch / (kms * 1e-3) / 1e9
    achieved_pipe = bytes_launch / (kms_pipe * 1e-3) / 1e9
    res = None
    if rank == 0:
        out = t_out.cpu().numpy().view(np.uint8).reshape(-1)[: 16 * batch.n].view(R.RESULT_DTYPE)
        line = {
            "metric": "Mpkts/s classified device-resident",
            "value": round(value, 2),
            "unit": "Mpkts/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(wall / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"config{a.config}", "packets_per_gpu": batch.n,
                       "rules": R.rule_count(prog), "cos": R.cos_count(prog),
                       "frame_bytes": "60 (64 B on the wire)" if a.config == 2 else "mixed",
                       "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": load_traffic(a.config, batch.n),
                         "kernel": "mi_cls_kernel", "kernel_ms": round(kms, 5),
                         "bytes_per_launch": bytes_launch,
                         "pipelined_achieved": round(achieved_pipe, 2),
                         "pipelined_frac": round(achieved_pipe / HBM_PEAK_GBS, 5),
                         "streams": a.streams},
        }
        if world == 1:
            try:
                line["e2e"] = time_e2e(c, batch, dev)
            except Exception as e:   # recorded, never fatal
                line["e2e"] = {"error": str(e)}
            if not a.no_cpu:
                cb, parity = cpu_baseline(prog, batch, a.cpu_seconds, out)
                line["cpu_baseline"] = cb
                line["parity_vs_oracle"] = parity
            if not a.no_extra:
                extra = {}
                names = {33: "config3_64B_256rules", 3: "config3_imix_256rules",
                         4: "config4_imix_v4v6_1024rules", 5: "config5_vlan_tree_4096rules"}
                for cfg in (33, 3, 4, 5):
                    b2, p2 = make_workload(cfg, a.n, 0)
                    c2 = cls.Classifier(gpu=local)
                    c2.apply(p2)
                    k_steps = max(5, a.steps // 5)
                    w2, _, _ = time_device(c2, b2, dev, k_steps, 3, rotate=a.rotate,
                                           streams=a.streams)
                    _, k2, _ = time_device(c2, b2, dev, k_steps, 3, rotate=a.rotate)
                    c2.close()
                    ach = b2.header_bytes() / (k2 * 1e-3) / 1e9
                    extra[names[cfg]] = {
                        "mpkts_per_s": round(b2.n * k_steps / w2 / 1e6, 2),
                        "kernel_ms": round(k2, 4), "roofline_frac": round(ach / HBM_PEAK_GBS, 5),
                        "rules": R.rule_count(p2)}
                # pktin checksum validation (IPv4 header, UDP/TCP sums over the
                # whole frame): config 3 IMIX with valid checksums; the kernel
                # reads every frame byte, so the bytes are frame + 22 B
                from odp_amd import pktgen as pg
                b2, p2 = make_workload(3, a.n, 0)
                pg.set_checksums(b2)
                c2 = cls.Classifier(gpu=local)
                c2.apply(p2)
                c2.set_pktin_opt(0x3C)
                k_steps = max(5, a.steps // 5)
                w2, _, _ = time_device(c2, b2, dev, k_steps, 3, rotate=a.rotate,
                                       streams=a.streams)
                _, k2, _ = time_device(c2, b2, dev, k_steps, 3, rotate=a.rotate)
                c2.close()
                fb = int(b2.len.astype(np.int64).sum()) + 22 * b2.n
                extra["config3_imix_256rules_checksums"] = {
                    "mpkts_per_s": round(b2.n * k_steps / w2 / 1e6, 2),
                    "kernel_ms": round(k2, 4),
                    "roofline_frac": round(fb / (k2 * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                    "bytes_per_launch": fb, "pktin_opt": "ipv4/udp/tcp/sctp checksums",
                    "rules": R.rule_count(p2)}
                line["extra"] = extra
        res = line
        print(json.dumps(res), flush=True)
    c.close()
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
