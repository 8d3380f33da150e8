"""One process per shard on the GPU: 2 and 3 processes share cuda:0, each holding one shard of the
observer rows, exchanging cross-shard traffic through the host transport over gloo. This runs the
multi-process collective call sequence of the RCCL path (sizes, parcels, heal broadcasts) for real,
and tests/dist_worker.py checks every round against the oracle, bit for bit."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(ws, name, timeout=240):
    port = _port()
    procs = []
    for r in range(ws):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(ws), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "dist_worker.py"), name], env=env,
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
    assert "bit-exact" in outs[0]


@pytest.mark.parametrize("name", ["config1", "config4"])
def test_two_processes(name):
    _run(2, name)


@pytest.mark.parametrize("name", ["config2", "config5"])
def test_three_processes(name):
    _run(3, name)


def _bench(extra, timeout=300):
    """bench.py as the driver starts it (a child process; --gpus N > 1 starts its own torch.distributed.run)"""
    repo = os.path.dirname(HERE)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--members", "4096", "--warmup", "6",
                          "--steps", "8", "--no-cpu-baseline", "--no-ring"] + extra, env=env, cwd=repo,
                         capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, (out.stdout + out.stderr)[-4000:]
    from test_bench_launch import json_objects

    lines = [l for l in json_objects(out.stdout) if "metric" in l]
    assert len(lines) == 1, out.stdout[-2000:]
    return lines[0]


def test_bench_two_ranks_host_transport_matches_one_gpu_line():
    """The driver's multi-GPU bench line, rehearsed on one GPU: `bench.py --gpus 2 --host-transport` passes the GPU-count
    gate, starts two ranks through torch.distributed.run, each holding half of the observer rows on cuda:0 and
    exchanging every cross-shard parcel through the gloo host transport (the RCCL port's call sequence), times the
    window max over ranks and prints one line with the exchange block. Its protocol counters (summed over the ranks)
    must equal the 1-GPU line's on the same window (ping_sender.go:90: the exchanged requests and responses are the
    RPCs of the reference)."""
    one = _bench(["--gpus", "1"])
    two = _bench(["--gpus", "2", "--host-transport"])
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert "host transport" in two["config"]["parallelism"]
    ex = two["exchange"]
    assert ex["bytes_rank0"] > 0 and ex["exchanges_rank0"] > 0, ex
    assert two["counters"] == one["counters"], (one["counters"], two["counters"])
    assert two["config"]["live_member_rounds"] == one["config"]["live_member_rounds"]
    print("1 GPU", one["value"], "2 ranks (host transport)", two["value"], "exchange", ex)
