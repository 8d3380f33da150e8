"""CPU baseline of bench.py: the C oracle on the host cores, bounded sample.

Two variants of the same protocol (config 3 scaled to --members, 1 % killed at r=10), both built from
oracle/swim_oracle.c with OpenMP over observers (oracle/build/libswim_oracle_omp.so; per-observer work of
a phase is independent, so results equal the single-threaded parity oracle's), each on all the process's cores
and on one thread (faithful and optimized, single-thread and OpenMP):
  reference_cost : the reference's cost model. Every Update that applied something rebuilds the checksum
                   string with Sprintf + sort and hashes it (memberlist.go:83-128, 367-368), and
                   AdjustMaxPropagations rescans the list for NumPingableMembers (disseminator.go:78,
                   memberlist.go:188-198).
  optimized_port : static-order string, checksums once per round for dirty rows, incremental counts.
Rounds 0..W-1 run untimed; rounds W.. are timed one by one until the window ends or the variant's budget is
spent (the OpenMP runs cover the whole window; the single-thread runs a stated prefix of it).
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
    """the cores this process may run on (its affinity mask); OMP_NUM_THREADS, when set, caps them (a one-GPU
    box's CPU share: the box sets it to its 16 cores while the affinity mask shows the whole machine)"""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(cap))) if cap and cap.isdigit() else max(1, n)


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


def run_threads(nthr, fn):
    """run fn() in a child process with OMP_NUM_THREADS = nthr (the OpenMP runtime reads it once, at load)"""
    import subprocess
    env = dict(os.environ, OMP_NUM_THREADS=str(nthr))
    out = subprocess.run([sys.executable, os.path.abspath(__file__), "--variant", fn], capture_output=True, text=True,
                         env=env, timeout=1800)
    if out.returncode != 0:
        return {"error": out.stderr[-400:]}
    return json.loads(out.stdout.strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--budget", type=float, default=60.0, help="seconds of CPU-side timing over all four runs")
    ap.add_argument("--window", default="65536:5:20", help="GPU line's members:warmup:steps")
    ap.add_argument("--members", type=int, default=16384)
    ap.add_argument("--variant", default=None, help=argparse.SUPPRESS)   # child: "ref|opt:n:warmup:steps:budget"
    args = ap.parse_args()
    os.environ["ORACLE_LIB"] = os.path.join(REPO, "oracle", "build", "libswim_oracle_omp.so")
    if args.variant:
        kind, n, warmup, steps, budget = args.variant.split(":")
        r = run_variant(int(n), int(warmup), int(steps), float(budget), kind == "ref")
        r["threads"] = int(os.environ.get("OMP_NUM_THREADS", "1"))
        print(json.dumps(r))
        return
    gpu_n, warmup, steps = (int(x) for x in args.window.split(":"))
    nthr = cores()
    n = min(args.members, gpu_n)
    b = args.budget
    spec = lambda kind, share: f"{kind}:{n}:{warmup}:{steps}:{share * b}"
    ref = run_threads(nthr, spec("ref", 0.45))
    opt = run_threads(nthr, spec("opt", 0.15))
    ref1 = run_threads(1, spec("ref", 0.25))
    opt1 = run_threads(1, spec("opt", 0.15))
    host = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            host = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), host)
    except OSError:
        pass
    rr = ref.get("rounds", [0, -1])
    print(json.dumps({
        "value": ref.get("value"), "unit": "member-rounds/s", "cores": nthr, "kind": "port", "host_cpu": host,
        "members": n,
        "sample": f"C oracle, reference cost model (Sprintf + sort + Fingerprint32 per applying Update, pingable rescan; "
                  f"oracle/swim_oracle.c reference_cost=1), OpenMP over observers on {nthr} threads (the process's "
                  f"cores), config-3 protocol at N={n} (1% killed at r=10), rounds {rr[0]}-{rr[1]} of the GPU window "
                  f"{warmup}-{warmup + steps - 1} timed ({ref.get('seconds')} s)",
        "reference_cost": ref,
        "optimized_port": {**opt, "note": "static-order string, checksum once per round per dirty row"},
        "reference_cost_1thread": ref1,
        "optimized_port_1thread": opt1,
    }))


if __name__ == "__main__":
    main()
