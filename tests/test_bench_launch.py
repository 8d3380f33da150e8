"""bench.py's launch contract on CPU (no GPU call): `--gpus N` without a launcher starts N ranks itself
through a child torch.distributed.run, and the workload accounting counts live members only."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def json_objects(text):
    """every JSON object in text, also when two ranks' lines ever share one line of the pipe"""
    dec, objs, i = json.JSONDecoder(), [], 0
    while True:
        i = text.find("{", i)
        if i < 0:
            return objs
        obj, i = dec.raw_decode(text, i)
        objs.append(obj)


def test_json_objects_parses_merged_lines():
    assert json_objects('noise\n{"rank": 0}{"rank": 1}\n\n{"rank": 2}\n') == [{"rank": 0}, {"rank": 1}, {"rank": 2}]


def test_gpus2_spawns_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--launch-check"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = json_objects(out.stdout)
    assert sorted(l["rank"] for l in lines) == [0, 1]
    assert all(l["world_size"] == 2 for l in lines)


def test_live_member_rounds_counts_live_members_only():
    sys.path.insert(0, REPO)
    import bench
    from swimsim import workloads as W

    wl = W.config3(n=1000, rounds=30, kill_round=10)
    # rounds 5-24: 5 rounds of 1000 live members, then 15 rounds of 990
    assert bench.live_member_rounds(wl, 5, 24) == 5 * 1000 + 15 * 990
