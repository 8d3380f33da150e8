"""One rank of the shard-transport conformance test (spawned by tests/test_transport.py).

XPORT=host: every rank on cuda:0, shards attached through swimsim.dist.GlooTransport (the host transport);
XPORT=rccl: rank r on GPU r, attached through RCCL (swimsim.dist.sharded_cluster). Each rank sends the
deterministic segments of tests/test_transport.py to every shard (itself included) over several exchanges and
checks every received byte. Exit code 0 = every segment arrived intact."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "ringpop-go_amd"))


def main():
    import torch.distributed as dist
    import swimsim
    from swimsim import dist as sd
    from test_transport import segment, ROUNDS

    dist.init_process_group("gloo")
    ws, rank = dist.get_world_size(), dist.get_rank()
    if os.environ["XPORT"] == "rccl":
        eng = sd.sharded_cluster(64, device=rank)
    else:
        eng = swimsim.Cluster(64, device=0, comm=(ws, rank, sd.GlooTransport()))
    bad = 0
    for k in range(ROUNDS):
        got = eng.debug_exchange([segment(rank, p, k) for p in range(ws)])
        for s in range(ws):
            if got[s] != segment(s, rank, k):
                print(f"rank {rank} exchange {k}: segment from {s} differs ({len(got[s])} bytes, "
                      f"expected {len(segment(s, rank, k))})", flush=True)
                bad = 1
    if rank == 0 and not bad:
        print(f"{os.environ['XPORT']}: {ROUNDS} exchanges over {ws} ranks intact", flush=True)
    eng.close()
    dist.destroy_process_group()
    sys.exit(bad)


if __name__ == "__main__":
    main()
