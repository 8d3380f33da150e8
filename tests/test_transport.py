"""Shard-transport conformance: the same parcel sequence through every transport a sharded cluster
can use, checked byte for byte. swimsim_debug_exchange moves caller bytes exactly as a round's parcel exchange
does (the size exchange, then one variable-size segment to and from every shard, own segment included).

* LocalPort: 2 and 3 shards of one process (threads), device-to-device copies.
* HostPort: 2 and 3 processes sharing cuda:0 over gloo.
* RcclPort: one rank (RCCL send/recv to itself: the grouped self-send every exchange does), and 2 ranks on two
  GPUs when two are visible (skipped on a one-GPU machine: RCCL refuses two ranks on one device).

Segment lengths include 0 and lengths that are not multiples of 16 (the transports align segments to 16 bytes)."""
import concurrent.futures as cf
import hashlib
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROUNDS = 4


def segment(src, dst, k):
    """deterministic bytes shard src sends shard dst at exchange k"""
    n = ((src * 7 + dst * 13 + k * 5) % 11) * 37 + (k == 2) * 70000
    if (src + dst + k) % 5 == 0:
        n = 0
    seed = hashlib.sha256(f"{src}/{dst}/{k}".encode()).digest()
    return (seed * (n // 32 + 1))[:n]


def test_segments_cover_edge_lengths():
    lens = {len(segment(s, d, k)) for s in range(3) for d in range(3) for k in range(ROUNDS)}
    assert 0 in lens and any(x % 16 for x in lens) and max(lens) > 65536


@pytest.mark.gpu
@pytest.mark.parametrize("g", [2, 3])
def test_local_port(g):
    import swimsim
    sc = swimsim.ShardedCluster(64, g)
    try:
        with cf.ThreadPoolExecutor(g) as ex:
            for k in range(ROUNDS):
                futs = [ex.submit(sc.shards[r].debug_exchange, [segment(r, p, k) for p in range(g)]) for r in range(g)]
                got = [f.result(timeout=60) for f in futs]
                for r in range(g):
                    assert got[r] == [segment(s, r, k) for s in range(g)], f"exchange {k}, shard {r}"
    finally:
        sc.close()


@pytest.mark.gpu
def test_rccl_port_one_rank():
    import swimsim
    eng = swimsim.Cluster(64, comm=(1, 0, swimsim.unique_id()))
    try:
        for k in range(ROUNDS):
            assert eng.debug_exchange([segment(0, 0, k)]) == [segment(0, 0, k)]
    finally:
        eng.close()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(ws, xport, timeout=180):
    port = _port()
    procs = []
    for r in range(ws):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(ws), LOCAL_RANK=str(r if xport == "rccl" else 0),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), XPORT=xport)
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "xport_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs, codes = [], []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
        codes.append(p.returncode)
    assert codes == [0] * ws, "\n".join(outs)[-4000:]
    assert "intact" in outs[0]


@pytest.mark.gpu
@pytest.mark.parametrize("ws", [2, 3])
def test_host_port(ws):
    _spawn(ws, "host")


@pytest.mark.gpu
def test_rccl_port_two_gpus():
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("RcclPort between ranks needs two GPUs (RCCL refuses two ranks on one device)")
    _spawn(2, "rccl")
