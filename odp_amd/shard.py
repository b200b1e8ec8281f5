"""Batch sharding across the GPUs of one node.

The receive path shards with no exchange step: the batch is cut into
contiguous slices (balanced by header-window bytes, so IMIX slices carry
equal work), each GPU classifies its own slice against its own replica of the
rule snapshot, and concatenating the per-GPU result arrays in GPU order
reproduces the single-device result -- and therefore the per-queue arrival
order the reference's _odp_cls_enq runs would see
(platform/linux-generic/include/odp_classification_internal.h:208-236).
No collective is needed on the data path.
"""
from __future__ import annotations

import numpy as np


def shard_bounds(lens: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Contiguous [begin, end) slices, one per rank, balanced by the bytes the
    kernel reads per packet (min(len,128) + descriptor + record).  This is
    the product's cut (mi_cls_shard in libmi_cls.so, the one
    mi_cls_group_classify_host uses), so a multi-process run and a
    multi-GPU pktio shard identically."""
    from .cls import shard
    if world <= 1:
        return [(0, int(lens.shape[0]))]
    b = shard(lens, world)
    return [(int(b[r]), int(b[r + 1])) for r in range(world)]


def shard_bounds_reference(lens: np.ndarray, world: int) -> list[tuple[int, int]]:
    """numpy restatement of mi_cls_shard (tests cross-check the two)."""
    n = int(lens.shape[0])
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    w = np.minimum(lens.astype(np.int64), 128) + 22
    cum = np.cumsum(w)
    total = int(cum[-1])
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(cum, total * r / world, side="left")) + 1)
    cuts.append(n)
    cuts = np.maximum.accumulate(np.minimum(cuts, n))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]
