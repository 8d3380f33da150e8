"""One process per GPU for one sharded cluster (include/swimsim.h "shards").

Launched by torch.distributed (torchrun: RANK / WORLD_SIZE / LOCAL_RANK in the environment), rank r
holds observer rows shard_range(n, world_size, r) of the cluster on GPU LOCAL_RANK. The cross-shard
messages move inside libswimsim over RCCL point-to-point (xGMI), not through torch. torch.distributed
is only the launcher's plumbing here: it broadcasts the RCCL id and reduces read-back results.
"""
from __future__ import annotations

import os

import numpy as np

from . import COUNTER_NAMES, Cluster, shard_range, unique_id


def env():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def broadcast_unique_id(uid, group=None) -> bytes:
    """rank 0's RCCL id (bytes) to every rank"""
    import torch.distributed as dist
    box = [uid if dist.get_rank(group) == 0 else None]
    dist.broadcast_object_list(box, src=0, group=group)
    return box[0]


def sharded_cluster(n, group=None, **kw) -> Cluster:
    """this rank's shard of an n-member cluster, attached to the other ranks through RCCL"""
    import torch.distributed as dist
    ws, rank = dist.get_world_size(group), dist.get_rank(group)
    local = env()[2]
    uid = broadcast_unique_id(unique_id() if rank == 0 else None, group)
    kw.setdefault("device", local)
    return Cluster(n, comm=(ws, rank, uid), **kw)


def gather_rows(local: np.ndarray, group=None) -> np.ndarray:
    """per-observer arrays of every shard, concatenated in observer order"""
    import torch.distributed as dist
    parts = [None] * dist.get_world_size(group)
    dist.all_gather_object(parts, np.asarray(local), group=group)
    return np.concatenate(parts)


def reduce_digest(d, group=None):
    """cluster digest = sum of the shard digests mod 2^64 (k_digest is additive over rows)"""
    import torch.distributed as dist
    parts = [None] * dist.get_world_size(group)
    dist.all_gather_object(parts, tuple(int(x) for x in d), group=group)
    return tuple(sum(p[i] for p in parts) % (1 << 64) for i in range(3))


def reduce_counters(c, group=None):
    """protocol counters of the cluster: every event is counted on exactly one shard; rounds is per shard"""
    import torch.distributed as dist
    parts = [None] * dist.get_world_size(group)
    dist.all_gather_object(parts, dict(c), group=group)
    out = {k: sum(p[k] for p in parts) for k in COUNTER_NAMES}
    out["rounds"] = max(p["rounds"] for p in parts)
    return out


def max_over_ranks(x: float, group=None) -> float:
    import torch.distributed as dist
    parts = [None] * dist.get_world_size(group)
    dist.all_gather_object(parts, float(x), group=group)
    return max(parts)


__all__ = ["env", "broadcast_unique_id", "sharded_cluster", "gather_rows", "reduce_digest", "reduce_counters",
           "max_over_ranks", "shard_range"]
