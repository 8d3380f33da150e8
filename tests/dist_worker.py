"""One shard of a sharded cluster in its own process (spawned by tests/test_dist_gpu.py).

Ranks attach through swimsim.dist.GlooTransport (torch.distributed gloo), so every collective exchange
between shard processes runs the same call sequence as the RCCL transport, on one GPU. Rank 0 checks
every round against the CPU oracle: all checksums, the canonical state digests, the phase-S targets and
the protocol counters, bit for bit. Exit code 0 = parity held.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "ringpop-go_amd"))


def main():
    import numpy as np
    import torch.distributed as dist
    import swimsim
    from swimsim import dist as sd
    from swimsim import workloads as W

    dist.init_process_group("gloo")
    ws, rank = dist.get_world_size(), dist.get_rank()
    name = sys.argv[1]
    wl = {"config1": lambda: W.config1(), "config2": lambda: W.config2(n=128, rounds=40),
          "config4": lambda: W.config4(n=64, rounds=100, split_until=40, heals=(40, 60)),
          "config5": lambda: W.config5(n=96, rounds=45, every=15)}[name]()
    eng = swimsim.Cluster(wl.n, device=0, comm=(ws, rank, sd.GlooTransport()))
    ora = None
    if rank == 0:
        from oracle_ffi import OracleSim
        ora = OracleSim(wl.n)
    bad = 0
    for r in range(wl.rounds):
        ev = wl.events_for(r)
        eng.step(1, ev)
        cs = sd.gather_rows(eng.checksums())
        tg = sd.gather_rows(eng.last_targets())
        dg = sd.reduce_digest(eng.digest())
        ct = sd.reduce_counters(eng.counters())
        if rank == 0:
            ora.step(ev)
            ok = (cs == ora.checksums()).all() and (tg == ora.last_targets()).all() and dg == ora.digest() \
                and ct == ora.counters()
            if not ok:
                print(f"{name} round {r}: divergence (checksums {(cs != ora.checksums()).sum()} differ)", flush=True)
                bad = 1
        flag = [bad]
        dist.broadcast_object_list(flag, src=0)
        if flag[0]:
            break
    info = eng.shard_info()
    if rank == 0 and not bad:
        print(f"{name}: {wl.rounds} rounds bit-exact over {ws} processes, exchanges {info['exchanges']}", flush=True)
    eng.close()
    dist.destroy_process_group()
    sys.exit(bad)


if __name__ == "__main__":
    main()
