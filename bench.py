"""bench.py — member-rounds/sec of the MI355X SWIM engine on BASELINE.json's 65,536-member config.

Workload (BASELINE.json configs[2], the metric's "64k members"): 65,536 members, converged start,
1 % (655) killed at round 10 (fixed, whatever --warmup is), then the suspect wave and, 25 rounds
after each suspect declaration, the faulty wave. One "step" is one synchronous protocol round of
every live member (docs/ROUND_SEMANTICS.md §4). --warmup W rounds (0..W-1) run untimed; --steps K
rounds (W..W+K-1) are timed between barrier + synchronize brackets. The JSON line names the window.

value = live member-rounds in the timed window / max-over-ranks time. A member killed at round r
executes no protocol period from round r on (SURVEY.md §8(d) counts live members only).

--gpus N > 1: without WORLD_SIZE in the environment, bench.py starts N ranks itself
(`python -m torch.distributed.run --nproc-per-node N bench.py ...` as a child process, before this
process touches the GPU) and exits with its status; the child's rank 0 prints the line. Each rank
holds observer rows [N*r/G, N*(r+1)/G) of the same 65,536-member cluster on GPU LOCAL_RANK, and every
cross-shard message moves over RCCL point-to-point (xGMI) inside libswimsim. Total work is fixed, so
"scaling" is "strong".

The JSON line carries:
  roofline     : the kernel with the most device time (rank 0): its algorithmic bytes per launch
                 (DESIGN.md §8 per-unit figures x the units the launch processed, counted on the device
                 during the timed rounds) / its average launch time (HIP events on the engine's own
                 stream), against the 8 TB/s HBM peak. `traffic` is FETCH_SIZE + WRITE_SIZE per launch from
                 the rocprofv3 PMC passes of THIS command (profiles/r02_pmc_summary.json; null when that
                 summary was taken on another workload). `merge` gives the same figures for the merge
                 kernels (k_recv, k_resp, k_issue); `merge_kernel` repeats k_recv, the north-star kernel.
  cpu_baseline : the C oracle on the GPU box's host cores (rank 0, N=1 only), bounded sample.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ringpop-go_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_PEAK_GINST = 256 * 4 * 2.4 / 2  # wave-instructions/ns: 1024 SIMDs, one wave64 VALU op per 2 cycles at 2.4 GHz
KILL_ROUND = 10
# kernel family (swimsim_kernel_times) -> kernel symbols in the rocprofv3 PMC summary
# (template arguments are ignored: every instantiation of the named kernel counts)
FAMILY_KERNELS = {"checksum": ["swimdev::k_checksum", "swimdev::k_checksum2", "swimdev::k_checksum3", "swimdev::k_checksum_n16",
                               "swimdev::k_checksum_q16"],
                  "recv_merge": ["swimdev::k_recv"], "issue": ["swimdev::k_issue"], "resp_merge": ["swimdev::k_resp"],
                  "timers": ["swimdev::k_timers"]}
FAMILY_SYMBOL = {"checksum": "k_checksum", "recv_merge": "k_recv", "resp_merge": "k_resp", "issue": "k_issue",
                 "timers": "k_timers"}
PMC_SUMMARY = os.path.join(REPO, "profiles", "r02_pmc_summary.json")


def pmc_family(family, workload):
    """Per-launch PMC figures of the family's kernels, launch-weighted over the committed rocprofv3 --pmc
    passes (FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU..., separate runs; tools/pmc_summary.py), or None when the
    summary is missing or was collected on a different workload than this run's."""
    try:
        with open(PMC_SUMMARY) as f:
            t = json.load(f)
        if t.get("_workload") != workload:
            return None
        names = set(FAMILY_KERNELS.get(family, []))
        ks = [v for k, v in t.items() if not k.startswith("_") and k.split("<")[0].strip() in names]
    except (OSError, KeyError, ValueError):
        return None
    n = sum(k["launches"] for k in ks)
    if not n:
        return None
    tot = lambda key: sum(k.get(key, 0.0) * k["launches"] for k in ks) / n
    return {"traffic": round(tot("fetch_bytes_per_launch") + tot("write_bytes_per_launch"), 1),
            "valu_insts": tot("sq_insts_valu_per_launch"), "lds_insts": tot("sq_insts_lds_per_launch")}


def ring_bench(n, replicas=100, nkeys=1 << 20):
    """SURVEY.md §8(f) rank 1, measured beside the headline (not part of `value`): the hash ring of a
    converged n-member cluster (every member a server, `replicas` points each: hashring.go:148-155)
    built on the device in one AddRemoveServers call, then `nkeys` Lookups in one batch. Device
    times are HIP events around the kernels (swimring_last_times)."""
    from swimsim import address_of
    from swimsim.ring import HashRing

    ring = HashRing(replicas, device=0)
    ring.add_remove_servers([address_of(m) for m in range(n)])
    build_ms, _ = ring.last_times()
    keys = [f"key-{k}" for k in range(nkeys)]
    ring.lookup_ids(keys[:1024])                       # warm-up
    ring.lookup_ids(keys)
    _, look_ms = ring.last_times()
    pts = len(ring.points()[0])
    ring.close()
    return {"servers": n, "replica_points": replicas, "points": pts, "build_ms": round(build_ms, 3),
            "build_points_per_s": round(n * replicas / (build_ms * 1e-3), 1) if build_ms > 0 else None,
            "lookups": nkeys, "lookup_ms": round(look_ms, 3),
            "lookups_per_s": round(nkeys / (look_ms * 1e-3), 1) if look_ms > 0 else None}


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def live_member_rounds(wl, first, last):
    """sum over rounds first..last of the members alive in that round (events apply in phase E)"""
    from swimsim import workloads as W

    live = [True] * wl.n
    nlive, total = wl.n, 0
    for r in range(0, last + 1):
        for (_, k, a, _b) in wl.events_for(r):
            if k == W.EV_KILL and live[a]:
                live[a] = False
                nlive -= 1
            elif k == W.EV_REVIVE and not live[a]:
                live[a] = True
                nlive += 1
        if r >= first:
            total += nlive
    return total


def cpu_baseline(gpu_window, seconds_budget=25.0):
    """The CPU oracle on a bounded sample of the same protocol (tools/cpu_baseline.py does the timing in a
    child process so that OpenMP threads do not share this process with the HIP runtime)."""
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "cpu_baseline.py"), "--budget",
                          str(seconds_budget), "--window", gpu_window], capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        return {"error": out.stderr[-400:]}
    return json.loads(out.stdout.strip().splitlines()[-1])


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """--gpus N without a launcher: start N ranks as a child torch.distributed.run, relay its status."""
    if not args.launch_check:
        import torch  # device_count() does not initialise the GPU on this image

        have = torch.cuda.device_count()
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but only {have} GPU(s) visible", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=90)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--members", type=int, default=65536)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ring", action="store_true")
    # diagnostics: every rank on cuda:0, shards exchanging through the gloo host transport instead of
    # RCCL (lets the multi-process path run on a one-GPU machine); never used for reported numbers
    ap.add_argument("--host-transport", action="store_true")
    # test hook: the ranks report (rank, world size) and exit before any GPU call
    ap.add_argument("--launch-check", action="store_true")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    ws, rank, local = dist_env()
    if ws != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}")
    if args.launch_check:
        print(json.dumps({"rank": rank, "world_size": ws, "local_rank": local}), flush=True)
        return

    import torch

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs an MI355X (no GPU visible)")
    if args.host_transport:
        local = 0
    torch.cuda.set_device(local)
    if ws > 1:
        import torch.distributed as dist

        # launcher plumbing only (RCCL id broadcast, barriers, max-over-ranks time); the data path is
        # libswimsim's own RCCL communicator. gloo prints its banner on the C-level stdout: keep stdout
        # for the one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)

    import swimsim
    from swimsim import workloads as W

    n = args.members
    total_rounds = args.warmup + args.steps
    wl = W.config3(n=n, rounds=max(total_rounds, KILL_ROUND + 1), kill_round=KILL_ROUND)
    nkilled = sum(1 for e in wl.events if e[1] == W.EV_KILL)
    if ws > 1:
        from swimsim import dist as sd

        if args.host_transport:
            eng = swimsim.Cluster(n, device=0, comm=(ws, rank, sd.GlooTransport()))
        else:
            eng = sd.sharded_cluster(n, device=local)
    else:
        eng = swimsim.Cluster(n, device=local)

    def barrier():
        if ws > 1:
            import torch.distributed as dist

            dist.barrier()
        torch.cuda.synchronize()

    for r in range(args.warmup):
        eng.step(1, wl.events_for(r))
    eng.enable_timing(True)
    barrier()
    t0 = time.perf_counter()
    ev = [e for e in wl.events if args.warmup <= e[0] < total_rounds]
    eng.step(args.steps, ev)
    barrier()
    dt = time.perf_counter() - t0
    if ws > 1:
        from swimsim import dist as sd

        dt = sd.max_over_ranks(dt)

    kt = eng.kernel_times()
    counters = eng.counters()
    shard = eng.shard_info()
    eng.enable_timing(False)
    if ws > 1:
        counters = sd.reduce_counters(counters)
    workload = {"members": n, "steps": args.steps, "warmup": args.warmup, "gpus": ws}

    def family_roofline(f):
        # algorithmic bytes per launch / HIP-event time of the same launches; PMC traffic of this command
        k = kt.get(f, {})
        if not k.get("avg_ms"):
            return None
        sec = k["avg_ms"] * 1e-3
        per_launch = k["alg_bytes"] / max(1, k["launches"])
        alg = per_launch / sec / 1e9
        p = pmc_family(f, workload)
        out = {"kernel": FAMILY_SYMBOL.get(f, f), "avg_launch_ms": round(k["avg_ms"], 4), "launches": k["launches"],
               "alg_bytes_per_launch": round(per_launch, 1), "achieved": round(alg, 2),
               "frac": round(alg / HBM_PEAK_GBPS, 4), "unit": "GB/s",
               "traffic": p["traffic"] if p else None,
               "traffic_over_alg": round(p["traffic"] / per_launch, 2) if p and per_launch > 0 else None}
        return out

    if rank == 0:
        timed_first, timed_last = args.warmup, total_rounds - 1
        live_mr = live_member_rounds(wl, timed_first, timed_last)
        value = live_mr / dt
        dominant = max(kt.items(), key=lambda kv: kv[1]["avg_ms"] * kv[1]["launches"])[0]
        dom = family_roofline(dominant)
        in_window = timed_first <= KILL_ROUND <= timed_last
        faulty_from = KILL_ROUND + 25       # first suspicions at KILL_ROUND; their timers fire 25 rounds later
        line = {
            "metric": "simulated member-rounds/sec at 64k members" if n == 65536 else f"simulated member-rounds/sec at {n} members",
            "value": round(value, 1),
            "unit": "member-rounds/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": f"synthetic (converged {n}-member cluster; {nkilled} members killed at round {KILL_ROUND}; Philox seed 11)",
            "config": {"workload": f"config3_cascade: {n} members, {nkilled} killed at r={KILL_ROUND}; rounds "
                                   f"{timed_first}-{timed_last} timed (" +
                                   ("steady state, kill, suspect wave" if in_window else "no kill in window") +
                                   ("; faulty wave from r>=%d in window" % faulty_from if timed_last >= faulty_from
                                    else "; faulty wave (r>=%d) outside the window" % faulty_from) + ")",
                       "members": n, "rounds_timed": args.steps, "live_member_rounds": live_mr,
                       "parallelism": (f"observer-row shards x{ws} over " + ("host transport (diagnostic)" if args.host_transport
                                                                              else "RCCL")) if ws > 1 else "1 GPU"},
            "roofline": {"bound": "hbm", **(dom or {}), "peak": HBM_PEAK_GBPS,
                         "traffic_unit": "bytes per launch (FETCH_SIZE + WRITE_SIZE, " + os.path.basename(PMC_SUMMARY) + ")",
                         "merge_kernel": family_roofline("recv_merge"),
                         "merge": {f: family_roofline(f) for f in ("recv_merge", "resp_merge", "issue")}},
            "kernel_ms": {k: round(v["avg_ms"] * v["launches"], 3) for k, v in kt.items()},
            "counters": counters,
        }
        pmc = pmc_family(dominant, workload)
        if dominant == "checksum" and pmc and pmc["valu_insts"] and kt[dominant]["avg_ms"] > 0:
            # the checksum is integer-VALU work: its instruction rate against the chip's VALU issue peak
            rate = pmc["valu_insts"] / (kt[dominant]["avg_ms"] * 1e6)
            line["roofline"]["valu"] = {"achieved": round(rate, 2), "peak": VALU_PEAK_GINST, "unit": "G wave-instr/s",
                                        "frac": round(rate / VALU_PEAK_GINST, 4),
                                        "valu_insts_per_launch": round(pmc["valu_insts"]),
                                        "lds_insts_per_launch": round(pmc["lds_insts"])}
        if ws > 1:
            line["exchange"] = {"bytes_rank0": shard["exchanged_bytes"], "exchanges_rank0": shard["exchanges"],
                                "bytes_per_round_rank0": round(shard["exchanged_bytes"] / max(1, total_rounds), 1)}
        if ws == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(f"{n}:{args.warmup}:{args.steps}")
        if ws == 1 and not args.no_ring:
            line["hashring"] = ring_bench(n)
        print(json.dumps(line), flush=True)
    if ws > 1:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
