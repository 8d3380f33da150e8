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
