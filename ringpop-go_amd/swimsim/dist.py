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


class GlooTransport:
    """swimsim_host_transport over a torch.distributed process group (e.g. gloo on CPU): lets one
    process per shard run on any machine, e.g. several shards sharing one GPU in a test. Slow
    (pickled all-gathers); the production path between GPUs is RCCL (sharded_cluster)."""

    def __init__(self, group=None):
        import ctypes as C
        import torch.distributed as dist
        from . import ALLTOALL_U64, ALLTOALLV, BCAST, HostTransport
        self.C, self.dist, self.group = C, dist, group
        self.ws, self.rank = dist.get_world_size(group), dist.get_rank(group)
        self._cbs = (ALLTOALL_U64(self._alltoall_u64), ALLTOALLV(self._alltoallv), BCAST(self._bcast))
        self._struct = HostTransport(None, *self._cbs)

    def c_struct(self):
        return self._struct

    def _alltoall_u64(self, ctx, send, recv, k):
        try:
            ws, r = self.ws, self.rank
            mine = np.ctypeslib.as_array(send, (ws * k,)).copy()
            parts = [None] * ws
            self.dist.all_gather_object(parts, mine, group=self.group)
            out = np.ctypeslib.as_array(recv, (ws * k,))
            for s in range(ws):
                out[s * k:(s + 1) * k] = parts[s][r * k:(r + 1) * k]
            return 0
        except Exception:
            return 1

    def _alltoallv(self, ctx, sbuf, soff, sbytes, rbuf, roff, rbytes):
        try:
            C, ws, r = self.C, self.ws, self.rank
            so, sb = np.ctypeslib.as_array(soff, (ws,)), np.ctypeslib.as_array(sbytes, (ws,))
            ro, rb = np.ctypeslib.as_array(roff, (ws,)), np.ctypeslib.as_array(rbytes, (ws,))
            segs = [C.string_at(sbuf + int(so[p]), int(sb[p])) if sb[p] else b"" for p in range(ws)]
            parts = [None] * ws
            self.dist.all_gather_object(parts, segs, group=self.group)
            for s in range(ws):
                data = parts[s][r]
                if len(data) != int(rb[s]):
                    return 1
                if data:
                    C.memmove(rbuf + int(ro[s]), data, len(data))
            return 0
        except Exception:
            return 1

    def _bcast(self, ctx, buf, nbytes, root):
        try:
            C = self.C
            box = [C.string_at(buf, nbytes) if self.rank == root else None]
            self.dist.broadcast_object_list(box, src=int(root), group=self.group)
            C.memmove(buf, box[0], nbytes)
            return 0
        except Exception:
            return 1


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


__all__ = ["env", "broadcast_unique_id", "sharded_cluster", "GlooTransport", "gather_rows", "reduce_digest", "reduce_counters",
           "max_over_ranks", "shard_range"]
