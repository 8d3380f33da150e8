"""bench.py — member-rounds/sec of the MI355X SWIM engine on BASELINE.json's 65,536-member config.

Workload (BASELINE.json configs[2], the metric's "64k members"): 65,536 members, converged start,
1 % (655) killed at round 10, then the suspect wave and the faulty wave ~25 rounds later.
One "step" is one synchronous protocol round of every member (docs/ROUND_SEMANTICS.md §4).
--warmup W rounds (default 10: rounds 0-9, steady state) run untimed. --steps K rounds (default
90: rounds 10-99, the kill and both cascades) are timed between barrier+synchronize brackets.

--gpus N > 1 (one process per GPU, launched by torch.distributed.run): the same 65,536-member
cluster's observer rows are sharded over the N GPUs (rank r holds rows [N*r/G, N*(r+1)/G)) and every
cross-shard message moves over RCCL point-to-point on xGMI inside libswimsim. Total work is fixed, so
"scaling" is "strong". value = members x K / max-over-ranks time.

The JSON line carries:
  roofline     : for the kernel family with the most device time (rank 0), its algorithmic bytes per
                 launch / HIP-event-measured average launch time (events on the engine's stream) vs the
                 8 TB/s HBM peak; merge_kernel_GBps is the same figure for the receive-merge family.
  cpu_baseline : the C oracle (single thread) on a bounded sample of the same protocol, rank 0, N=1 only.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ringpop-go_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_PEAK_GINST = 256 * 4 * 2.4 / 2  # wave-instructions/ns: 1024 SIMDs, one wave64 VALU op per 2 cycles at 2.4 GHz
# kernel family (swimsim_kernel_times) -> kernel symbols in the rocprofv3 PMC summary
FAMILY_KERNELS = {"checksum": ["swimdev::k_checksum<19, 11, 9, 0>", "swimdev::k_checksum_n16<19, 11, 9, 0>"],
                  "recv_merge": ["swimdev::k_recv"], "issue": ["swimdev::k_issue"], "resp_merge": ["swimdev::k_resp"],
                  "timers": ["swimdev::k_timers"]}
PMC_SUMMARY = os.path.join(REPO, "profiles", "r01_pmc_summary.json")


def pmc_family(family):
    """Per-launch PMC figures of the family's kernels (launch-weighted over the committed PMC passes of this
    bench: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU..., separate runs; tools/pmc_summary.py),
    or None."""
    try:
        with open(PMC_SUMMARY) as f:
            t = json.load(f)
        ks = [t[k] for k in FAMILY_KERNELS[family] if k in t]
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


def cpu_baseline(seconds_budget=25.0):
    """Oracle (tests/oracle_ffi.py, CPU restatement) on a bounded sample of the config-3 protocol."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_ffi import OracleSim
    from swimsim import workloads as W

    n, rounds = 4096, 40
    wl = W.config3(n=n, rounds=rounds)
    sim = OracleSim(n)
    t0 = time.perf_counter()
    done = 0
    for r in range(rounds):
        sim.step(wl.events_for(r))
        done += 1
        if time.perf_counter() - t0 > seconds_budget:
            break
    dt = time.perf_counter() - t0
    host = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            host = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), host)
    except OSError:
        pass
    return {
        "value": round(n * done / dt, 1),
        "unit": "member-rounds/s",
        "cores": 1,
        "kind": "port",
        "host_cpu": host,
        "sample": f"C oracle (oracle/swim_oracle.c, -O2, 1 thread) on the config-3 protocol at N={n} "
                  f"(1% killed at r=10), rounds 0-{done - 1}, {dt:.1f} s; per-member-round cost grows ~linearly in N",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=90)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--members", type=int, default=65536)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # diagnostics: every rank on cuda:0, shards exchanging through the gloo host transport instead of
    # RCCL (lets the multi-process path run on a one-GPU machine); never used for reported numbers
    ap.add_argument("--host-transport", action="store_true")
    args = ap.parse_args()

    ws, rank, local = dist_env()
    import torch

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs an MI355X (no GPU visible)")
    if args.host_transport:
        local = 0
    torch.cuda.set_device(local)
    if ws > 1:
        import torch.distributed as dist

        # launcher plumbing only (RCCL id broadcast, barriers, max-over-ranks time); the data path is
        # libswimsim's own RCCL communicator
        # gloo prints its connection banner on the C-level stdout; keep stdout for the one JSON line
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
    wl = W.config3(n=n, rounds=total_rounds)
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
    dominant = max(kt.items(), key=lambda kv: kv[1]["avg_ms"] * kv[1]["launches"])
    fam, info = dominant
    per_launch_bytes = info["alg_bytes"] / max(1, info["launches"])
    achieved = per_launch_bytes / (info["avg_ms"] * 1e-3) / 1e9 if info["avg_ms"] > 0 else 0.0
    pmc = pmc_family(fam)
    merge = kt.get("recv_merge", {})
    merge_gbps = (merge.get("alg_bytes", 0) / max(1, merge.get("launches", 1))) / (merge.get("avg_ms", 1) * 1e-3) / 1e9 \
        if merge.get("avg_ms", 0) > 0 else 0.0

    def family_roofline(f):
        # algorithmic bytes per launch / HIP-event time, and the PMC-measured HBM bytes per launch of the
        # same kernels over the same time (the gathers' sector traffic: what actually bounds them)
        k = kt.get(f, {})
        if not k.get("avg_ms"):
            return None
        sec = k["avg_ms"] * 1e-3
        alg = k["alg_bytes"] / max(1, k["launches"]) / sec / 1e9
        p = pmc_family(f)
        out = {"kernel": FAMILY_KERNELS[f][0], "avg_launch_ms": round(k["avg_ms"], 4), "launches": k["launches"],
               "achieved_alg": round(alg, 2), "frac_alg": round(alg / HBM_PEAK_GBPS, 4), "unit": "GB/s"}
        if p:
            hbm = p["traffic"] / sec / 1e9
            out.update({"traffic_per_launch": p["traffic"], "achieved_hbm": round(hbm, 2),
                        "frac_hbm": round(hbm / HBM_PEAK_GBPS, 4)})
        return out

    if rank == 0:
        value = n * args.steps / dt
        line = {
            "metric": "simulated member-rounds/sec at 64k members",
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
            "data": f"synthetic (converged {n}-member cluster; {max(1, n // 100)} members killed at round 10; Philox seed 11)",
            "config": {"workload": f"config3_cascade: {n} members, 1% killed at r={args.warmup}, rounds {args.warmup}-{total_rounds - 1} timed",
                       "members": n, "rounds_timed": args.steps,
                       "parallelism": (f"observer-row shards x{ws} over " + ("host transport (diagnostic)" if args.host_transport
                                                                              else "RCCL")) if ws > 1 else "1 GPU"},
            "roofline": {"bound": "hbm", "kernel": fam, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5),
                         "traffic": pmc["traffic"] if pmc else None,
                         "traffic_unit": "bytes per launch (FETCH_SIZE + WRITE_SIZE, " + os.path.basename(PMC_SUMMARY) + ")",
                         "avg_launch_ms": round(info["avg_ms"], 5), "launches": info["launches"],
                         "merge_kernel_GBps": round(merge_gbps, 2),
                         "merge": {f: family_roofline(f) for f in ("recv_merge", "resp_merge", "issue")}},
            "kernel_ms": {k: round(v["avg_ms"] * v["launches"], 3) for k, v in kt.items()},
            "counters": counters,
        }
        if pmc and pmc["valu_insts"] and info["avg_ms"] > 0:
            # the checksum is integer-VALU work: its instruction rate against the chip's VALU issue peak
            rate = pmc["valu_insts"] / (info["avg_ms"] * 1e6)
            line["roofline"]["valu"] = {"achieved": round(rate, 2), "peak": VALU_PEAK_GINST, "unit": "G wave-instr/s",
                                        "frac": round(rate / VALU_PEAK_GINST, 4),
                                        "valu_insts_per_launch": round(pmc["valu_insts"]),
                                        "lds_insts_per_launch": round(pmc["lds_insts"])}
        if ws > 1:
            line["exchange"] = {"bytes_rank0": shard["exchanged_bytes"], "exchanges_rank0": shard["exchanges"]}
        if ws == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline()
        if ws == 1:
            line["hashring"] = ring_bench(n)
        print(json.dumps(line), flush=True)
    if ws > 1:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
