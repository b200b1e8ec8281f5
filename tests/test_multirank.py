"""World-size-2 rehearsal of the multi-GPU path on CPU (gloo): each rank
takes its contiguous shard with the product's cut (mi_cls_shard in
libmi_cls.so, the one mi_cls_group_classify_host and bench.py use) and
classifies it (here with the CPU oracle standing in for the per-GPU kernel,
which needs a device); results gathered in rank order must equal the
single-process run, and the bench's max-over-ranks timing reduction is
exercised with the same collective calls the GPU run makes.  The GPU side
(several contexts, the runtime pktio over ODP_AMD_GPUS, bench.py with two
ranks) is tests/test_gpu_multi.py."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from odp_amd import rules as R
from odp_amd.shard import shard_bounds, shard_bounds_reference


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg, n, q):
    import torch
    import torch.distributed as dist
    from tests.helpers import oracle_run
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    batch, prog = R.CONFIGS[cfg](n)
    b, e = shard_bounds(batch.len, world)[rank]
    res, _ = oracle_run(prog, batch.slice(b, e))
    rec = torch.from_numpy(res.view(np.uint8).copy())
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([rec.numel()]))
    mx = int(max(s.item() for s in sizes))
    pad = torch.zeros(mx, dtype=torch.uint8)
    pad[: rec.numel()] = rec
    bufs = [torch.zeros(mx, dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(bufs, pad)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)          # bench.py's timing reduction
    dist.barrier()
    if rank == 0:
        out = np.concatenate([bufs[r][: int(sizes[r].item())].numpy() for r in range(world)])
        q.put((out.view(R.RESULT_DTYPE), t.item()))
    dist.destroy_process_group()


def _run(cfg, n, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, cfg, n, q)) for r in range(world)]
    for p in ps:
        p.start()
    got, tmax = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got, tmax


def test_shard_bounds_balanced():
    lens = np.array([60] * 700 + [1514] * 100 + [566] * 200)
    rng = np.random.default_rng(0)
    rng.shuffle(lens)
    for world in (1, 2, 3, 8):
        b = shard_bounds(lens, world)
        assert b[0][0] == 0 and b[-1][1] == len(lens)
        assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
        w = np.minimum(lens, 128) + 22
        parts = [w[s:e].sum() for s, e in b]
        assert max(parts) - min(parts) <= 2 * 150   # each cut is within one packet


def test_c_shard_matches_reference(built):
    """mi_cls_shard (C, product) == the numpy restatement, including empty
    batches, more shards than packets and uniform lengths."""
    rng = np.random.default_rng(3)
    for n in (0, 1, 2, 7, 64, 1000, 50_000):
        for world in (1, 2, 3, 5, 8, 64):
            for kind in ("imix", "60", "big"):
                lens = (rng.choice([60, 566, 1514], n) if kind == "imix"
                        else np.full(n, 60 if kind == "60" else 1514))
                assert shard_bounds(lens, world) == shard_bounds_reference(lens, world), \
                    (n, world, kind)


def test_two_rank_shards_equal_single(built):
    from tests.helpers import oracle_run
    for cfg, n in ((3, 3000), (4, 2000)):
        got, tmax = _run(cfg, n)
        batch, prog = R.CONFIGS[cfg](n)
        exp, _ = oracle_run(prog, batch)
        assert np.array_equal(got, exp)
        assert tmax == 2.0


def test_bench_gpus_n_without_launcher_fails_loudly_without_devices():
    """`bench.py --gpus 2` started without torchrun spawns one worker per
    GPU itself; with fewer devices visible (none here) it must exit non-zero
    instead of printing a 1-GPU line for a 2-GPU request."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "BENCH_SAME_DEVICE")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--steps", "1", "--warmup", "0"], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=120, env=env)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "--gpus 2 requested" in r.stderr


def test_bench_world_size_mismatch_fails():
    """Under a launcher, --gpus must equal WORLD_SIZE."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--steps", "1", "--warmup", "0"], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr


def _reduce_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    kw = bench.dist_init_kwargs("gloo", rank)
    dist.init_process_group(rank=rank, world_size=world, **kw)
    # rank r: wall 1 + r s, n = 1000 (r + 1) packets, kernel (r + 1) * 0.01 ms,
    # bytes 1e6 (r + 1); rank 1 fails parity in the second call, in the
    # third nobody checks
    r1 = bench.reduce_ranks(dist, torch.device("cpu"), 1.0 + rank, 1000 * (rank + 1),
                            0.01 * (rank + 1), 1_000_000 * (rank + 1), True)
    r2 = bench.reduce_ranks(dist, torch.device("cpu"), 1.0, 10, 0.01, 1, rank != 1)
    r3 = bench.reduce_ranks(dist, torch.device("cpu"), 1.0, 10, 0.01, 1, None)
    q.put((rank, r1, r2["parity"], r3["parity"]))
    dist.destroy_process_group()


def test_bench_rank_reductions():
    """bench.py's multi-rank reductions over gloo with 3 ranks: max wall,
    packets summed, per-rank kernel_ms and bytes in rank order, the aggregate
    roofline (sum of bytes / slowest kernel) and parity AND-ed over every
    rank's shard (not rank 0's alone)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    ps = [ctx.Process(target=_reduce_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, r1, p2, p3 in res:
        assert r1["wall"] == 3.0
        assert r1["packets"] == 6000
        assert r1["kernel_ms"] == [0.01, 0.02, 0.03]
        assert r1["bytes_per_launch"] == [1_000_000, 2_000_000, 3_000_000]
        assert abs(r1["achieved_gbs"] - 6e6 / 0.03e-3 / 1e9) < 1e-6
        assert r1["parity"] is True and p2 is False and p3 is None


def test_bench_nccl_init_binds_each_rank_to_its_device():
    """The RCCL branch's init arguments for every local rank of an 8-GPU
    node: device_id = cuda:LOCAL_RANK (the branch never runs on CPU; its
    arguments are checked here)."""
    import torch
    import bench
    for local in range(8):
        kw = bench.dist_init_kwargs("nccl", local)
        assert kw["backend"] == "nccl"
        assert kw["device_id"] == torch.device(f"cuda:{local}")
    assert bench.dist_init_kwargs("gloo", 3) == {"backend": "gloo"}
