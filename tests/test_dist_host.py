"""CPU (gloo, world_size 2) checks of the one-process-per-GPU launcher logic in swimsim/dist.py: the
RCCL-id broadcast, the shard split and the read-back reductions. The engine itself needs a GPU; its
sharded path is checked bit-exact against the oracle in tests/test_sharded_parity.py."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, ws, port, q):
    sys.path.insert(0, os.path.join(REPO, "ringpop-go_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from swimsim import dist as sd
    from swimsim import COUNTER_NAMES, shard_range
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        uid = sd.broadcast_unique_id(bytes(range(128)) if rank == 0 else None)
        n = 37
        lo, hi = shard_range(n, ws, rank)
        rows = sd.gather_rows(np.arange(lo, hi, dtype=np.uint32) * 3)
        dg = sd.reduce_digest(((1 << 63) + rank, rank, 2 * rank))
        ctr = sd.reduce_counters({k: (7 if k == "rounds" else rank + 1) for k in COUNTER_NAMES})
        t = sd.max_over_ranks(0.5 + rank)
        q.put((rank, uid, rows.tolist(), dg, ctr, t))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_launcher_helpers_gloo_world_size_2():
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, ws, PORT, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in range(ws)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, uid, rows, dg, ctr, t in res:
        assert uid == bytes(range(128))
        assert rows == [3 * i for i in range(37)]
        assert dg == ((1 << 63) * 2 % (1 << 64) + 1, 1, 2)
        assert ctr["rounds"] == 7 and ctr["pings"] == 3
        assert t == 1.5


PORT = _free_port()
