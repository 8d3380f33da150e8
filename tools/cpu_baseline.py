"""CPU baseline of bench.py: the C oracle on the host cores, bounded sample.

Two variants of the same protocol (config 3 scaled to --members, 1 % killed at r=10), both built from
oracle/swim_oracle.c with OpenMP over observers (oracle/build/libswim_oracle_omp.so; per-observer work of
a phase is independent, so results equal the single-threaded parity oracle's):
  reference_cost : the reference's cost model. Every Update that applied something rebuilds the checksum
                   string with Sprintf + sort and hashes it (memberlist.go:83-128, 367-368), and
                   AdjustMaxPropagations rescans the list for NumPingableMembers (disseminator.go:78,
                   memberlist.go:188-198).
  optimized_port : static-order string, checksums once per round for dirty rows, incremental counts.
Rounds 0..W-1 run untimed; rounds W.. are timed one by one until the window ends or the budget is spent.
value = live member-rounds of the timed rounds / their time. Prints one JSON object (the bench line's
cpu_baseline). TEST INFRASTRUCTURE: bench.py runs it in a child process; the product never loads the oracle.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "ringpop-go_amd"))


def cores():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    # a one-GPU box's CPU share is 16 (OMP_NUM_THREADS is set to it there)
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", "16"))))


def run_variant(n, warmup, steps, budget, reference_cost):
    from oracle_ffi import OracleSim
    from swimsim import workloads as W

    wl = W.config3(n=n, rounds=warmup + steps)
    sim = OracleSim(n, faithful_checksum=reference_cost, reference_cost=reference_cost)
    for r in range(warmup):
        sim.step(wl.events_for(r))
    live = n - sum(1 for e in wl.events if e[1] == W.EV_KILL and e[0] < warmup)
    done, mr, spent, per_round = 0, 0, 0.0, []
    for r in range(warmup, warmup + steps):
        ev = wl.events_for(r)
        live -= sum(1 for e in ev if e[1] == W.EV_KILL)
        t0 = time.perf_counter()
        sim.step(ev)
        dt = time.perf_counter() - t0
        spent += dt
        per_round.append(round(dt, 3))
        mr += live
        done += 1
        if spent > budget:
            break
    return {"value": round(mr / spent, 1), "rounds": [warmup, warmup + done - 1], "seconds": round(spent, 2),
            "round_s": per_round}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--budget", type=float, default=25.0)
    ap.add_argument("--window", default="65536:5:20", help="GPU line's members:warmup:steps")
    ap.add_argument("--members", type=int, default=16384)
    args = ap.parse_args()
    gpu_n, warmup, steps = (int(x) for x in args.window.split(":"))
    nthr = cores()
    os.environ["OMP_NUM_THREADS"] = str(nthr)
    os.environ["ORACLE_LIB"] = os.path.join(REPO, "oracle", "build", "libswim_oracle_omp.so")
    n = min(args.members, gpu_n)
    ref = run_variant(n, warmup, steps, 0.7 * args.budget, True)
    opt = run_variant(n, warmup, steps, 0.3 * args.budget, False)
    host = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            host = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), host)
    except OSError:
        pass
    print(json.dumps({
        "value": ref["value"], "unit": "member-rounds/s", "cores": nthr, "kind": "port", "host_cpu": host,
        "sample": f"C oracle, reference cost model (Sprintf + sort + Fingerprint32 per applying Update, pingable rescan; "
                  f"oracle/swim_oracle.c reference_cost=1), OpenMP over observers on {nthr} threads, config-3 protocol at "
                  f"N={n} (1% killed at r=10), rounds {ref['rounds'][0]}-{ref['rounds'][1]} of the GPU window "
                  f"{warmup}-{warmup + steps - 1} timed ({ref['seconds']} s)",
        "reference_cost": ref,
        "optimized_port": {**opt, "note": "static-order string, checksum once per round per dirty row"},
    }))


if __name__ == "__main__":
    main()
