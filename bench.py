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
  roofline     : the kernel with the most device time (rank 0): units per launch (rows hashed, changes
                 merged; counted on the device over the timed rounds) x SURVEY.md §8(d)'s bytes per unit
                 = algorithmic bytes per launch, / its average launch time (HIP events on the engine's own
                 stream), against the 8 TB/s HBM peak. `traffic` = HBM bytes per launch from the rocprofv3
                 PMC passes of THIS command cut to the same timed rounds (k_profile_mark dispatches around
                 them; profiles/r05_pmc_summary.json; null when that summary was taken on another workload).
                 `kernels` gives the same figures for the other kernels (the other checksum kernel, k_recv,
                 k_resp, k_issue); `merge_kernel` repeats k_recv, the north-star merge kernel.
  cpu_baseline : the C oracle on the GPU box's host cores (rank 0, N=1 only) at the GPU line's N, bounded sample.

--workload (1 GPU; default config3, the driver's line): the other BASELINE.json configs measured the same way, each a
line of its own (not the headline): config2 (4,096 members, 1 % churn per round), config4 (16,384 members, 2-way
partition then heal_partition; the line adds the rounds from the heal to convergence, from an untimed replay),
selfstart (16,384 members that know only themselves and two seed members: full syncs and reverse full syncs) and
config5 (incarnation bursts, 10 % of 65,536 members every 20 rounds; 262,144 needs 8 GPUs). Their roofline adds the
dense merges (reverse full syncs, k_jobs_merge) against SURVEY.md §8(d)'s streaming bytes.
"""
import glob
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
MARK_BEGIN, MARK_END = 0x5717, 0x5718   # k_profile_mark ids around the timed rounds (tools/pmc_summary.py --window)
# kernel family (swimsim_kernel_times) -> kernel symbol in rocprofv3 output (template arguments ignored)
# (wide launches of at least 1,024 rows run the reference-row chain kernel k_csr3 by default; k_checksum3 takes the rows
# it leaves and the launches with the path off)
FAMILY_KERNEL = {"checksum_wide": "swimdev::k_csr3", "checksum_narrow": "swimdev::k_checksum_q16",
                 "recv_merge": "swimdev::k_recv", "resp_merge": "swimdev::k_resp", "issue": "swimdev::k_issue",
                 "timers": "swimdev::k_timers", "rfs_merge": "swimdev::k_jobs_merge"}
# PMC summaries of bench.py commands (tools/pmc_summary.py); a line uses the one whose _workload is its own
PMC_GLOB = os.path.join(REPO, "profiles", "r0*_pmc_summary*.json")
# --workload: default members, the builder in swimsim.workloads, what the line says about it
WORKLOADS = {
    "config3": (65536, "config3_cascade"),
    "config2": (4096, "config2_churn"),
    "config4": (16384, "config4_partition_heal"),
    "selfstart": (16384, "selfstart_full_syncs"),
    "config5": (65536, "config5_bursts"),
}
FETCH_CALIB = os.path.join(REPO, "profiles", "r03_fetch_calib.json")


def fetch_factor(fam):
    """HBM bytes per FETCH_SIZE byte for the kernel's dominant read pattern, measured by tools/fetch_calib.hip
    (profiles/r03_fetch_calib.json): the checksum kernels stream each lane's own row 16 B at a time
    (k_rowstream16); the merge and issue kernels gather one 4-B or 8-B word per 64-B sector, which FETCH_SIZE
    counts in full (64 B per sector, factor 1; their coalesced record streams are then undercounted by half, so
    the doubled figure is kept as the upper bound)."""
    try:
        with open(FETCH_CALIB) as f:
            c = json.load(f)
    except (OSError, ValueError):
        c = {}
    if fam.startswith("checksum"):
        r = c.get("k_rowstream16", {}).get("fetch_over_read") or c.get("k_stream16", {}).get("fetch_over_read") or 0.5
        return 1.0 / r, "k_rowstream16" if "k_rowstream16" in c else "k_stream16"
    r = c.get("k_gather<unsigned int>", {}).get("fetch_per_sector")
    return (64.0 / r if r else 1.0), "k_gather<unsigned int>"


def pmc_summary_for(workload):
    """the newest committed PMC summary taken on exactly this bench.py command, cut to its timed rounds"""
    for path in sorted(glob.glob(PMC_GLOB), reverse=True):
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        if t.get("_workload") == workload and t.get("_window"):
            return path, t
    return None, None


def pmc_kernel(symbol, workload):
    """Per-launch PMC figures of one kernel over the timed rounds only (rocprofv3 --pmc passes of this command, cut
    between the k_profile_mark dispatches by tools/pmc_summary.py --window), or None when no committed summary was
    taken on this workload with the window cut."""
    path, t = pmc_summary_for(workload)
    if t is None:
        return None
    try:
        ks = [v for k, v in t.items() if not k.startswith("_") and k.split("<")[0].strip() == symbol]
    except (KeyError, ValueError):
        return None
    n = sum(k["launches"] for k in ks)
    if not n:
        return None
    avg = lambda key: sum(k.get(key, 0.0) * k["launches"] for k in ks) / n
    return {"launches": n, "fetch": avg("fetch_bytes_per_launch"), "write": avg("write_bytes_per_launch"),
            "valu_insts": avg("sq_insts_valu_per_launch"), "lds_insts": avg("sq_insts_lds_per_launch"),
            "source": os.path.relpath(path, REPO)}


def roofline_entry(fam, kt, units, n_members):
    """One kernel against the HBM roofline: achieved = algorithmic bytes per launch (SURVEY.md §8(d) bytes per unit
    x the units the launches processed, counted on the device over the timed rounds) / the average launch time
    (HIP events on the engine's stream); frac = achieved / 8 TB/s. traffic = HBM bytes per launch from the PMC
    passes of this command over the same rounds: FETCH_SIZE doubled (gfx950 tallies a 16-B-per-lane read's
    128-B requests at 64 B, MI355X_MICROARCH.md §HBM; tools/fetch_calib.hip checks the factor per access pattern,
    profiles/r03_fetch_calib.json) + WRITE_SIZE."""
    k = kt.get(fam, {})
    if not k.get("avg_ms") or not k.get("launches"):
        return None
    nl, sec = k["launches"], k["avg_ms"] * 1e-3
    out = {"kernel": FAMILY_KERNEL[fam].split("::")[-1], "avg_launch_ms": round(k["avg_ms"], 4), "launches": nl}
    if fam.startswith("checksum"):
        rows = units["cs_rows_wide" if fam == "checksum_wide" else "cs_rows_narrow"]
        per = 5.0 * n_members
        out.update({"work_unit": "hashed row", "units_per_launch": round(rows / nl, 1),
                    "bytes_per_unit": per, "bytes_per_unit_basis": "SURVEY.md §8(d): 5 B (status u8 + incarnation "
                    "u32) per member per dirty row; the kernel reads a 4-B member word (e << 3 | status) per member",
                    "alg_bytes_per_launch": round(rows / nl * per, 1),
                    "alg_bytes_per_launch_4B": round(rows / nl * 4.0 * n_members, 1)})
    elif fam in ("recv_merge", "resp_merge"):
        pre = "recv" if fam == "recv_merge" else "resp"
        merged, applied = units[pre + "_merged"], units[pre + "_applied"]
        merge_b = 22.0 * merged + 23.0 * applied
        if fam == "recv_merge":
            side_b = 36.0 * units["recv_issued"] + 4.0 * units["bitmap_words_per_row"] * units["recv_calls"]
            side = {"issued_per_launch": round(units["recv_issued"] / nl, 1), "calls_per_launch": round(units["recv_calls"] / nl, 1),
                    "hot_slots_at_end": units.get("hot_slots"),
                    "issue_as_receiver_bytes_per_launch": round(side_b / nl, 1),
                    "issue_as_receiver_basis": "36 B per issued record (16-B cell gather + 16-B record write + 4-B "
                    "counter write-back) + the presence bitmap (4 B per 32 members) per call"}
        else:
            side_b = 24.0 * units["resp_bumped"]
            side = {"bumped_per_launch": round(units["resp_bumped"] / nl, 1), "bump_bytes_per_launch": round(side_b / nl, 1),
                    "bump_basis": "24 B per bumped entry (16-B record read + 4-B counter read and write)"}
        out.update({"work_unit": "processed change", "units_per_launch": round(merged / nl, 1),
                    "applied_per_launch": round(applied / nl, 1),
                    "bytes_per_unit_basis": "SURVEY.md §8(d): 17 B change entry + 5 B row read per processed "
                    "change; + 5 B row write + 9 B dissemination entry + 9 B timer per applied change",
                    "alg_bytes_per_launch": round(merge_b / nl, 1), **side,
                    "achieved_incl_side": round((merge_b + side_b) / nl / sec / 1e9, 2),
                    "frac_incl_side": round((merge_b + side_b) / nl / sec / 1e9 / HBM_PEAK_GBPS, 4)})
    elif fam == "issue":
        out.update({"work_unit": "issued record", "units_per_launch": round(units["issued"] / nl, 1), "bytes_per_unit": 32.0,
                    "alg_bytes_per_launch": round(units["issued"] / nl * 32.0, 1)})
    elif fam == "rfs_merge":
        dense, applied = units.get("dense_jobs", 0.0), units.get("jobs_applied", 0.0)
        if not dense:
            out.update({"work_unit": "dense merge", "units_per_launch": 0.0,
                        "note": "no reverse full sync in the window: the launches exit at once"})
            return out
        out.update({"work_unit": "dense merge (reverse full sync)", "units_per_launch": round(dense / nl, 2),
                    "applied_per_launch": round(applied / nl, 1),
                    "bytes_per_unit_basis": "SURVEY.md §8(d): a dense batch streams the row, 5 B x N per merged snapshot; "
                    "+ 23 B per applied change (the kernel reads the 4-B snapshot word and the 4-B row word per member)",
                    "alg_bytes_per_launch": round((dense * 5.0 * n_members + applied * 23.0) / nl, 1),
                    "physical_read_bytes_per_launch": round(dense * 8.0 * n_members / nl, 1)})
    else:
        return out
    alg = out["alg_bytes_per_launch"] / sec / 1e9
    out.update({"achieved": round(alg, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(alg / HBM_PEAK_GBPS, 4)})
    return out


def dom_bound(fam, entry):
    """The bound of the dominant kernel. The FarmHash checksum kernels are bounded by integer VALU issue (a row's chain is
    sequential and every block costs tens of VALU instructions per 20 string bytes), not by HBM: for them
    the line keeps the §8(d) HBM figures (achieved / peak / frac) and names "valu" as the bound, whose fraction is
    entry["valu"]["frac"]. The merge and issue kernels are HBM-gather kernels."""
    if fam.startswith("checksum"):
        return "valu"
    return "hbm"


def add_pmc(entry, fam, workload):
    if not entry:
        return entry
    p = pmc_kernel(FAMILY_KERNEL[fam], workload)
    if not p:
        entry.update({"traffic": None, "traffic_note": "no PMC summary of this workload's timed window"})
        return entry
    ff, pattern = fetch_factor(fam)
    t = ff * p["fetch"] + p["write"]
    entry.update({"traffic": round(t, 1), "traffic_fetch_factor": round(ff, 3), "traffic_fetch_pattern": pattern,
                  "traffic_raw_fetch_plus_write": round(p["fetch"] + p["write"], 1),
                  "traffic_upper_2x_fetch_plus_write": round(2.0 * p["fetch"] + p["write"], 1),
                  "traffic_over_alg": round(t / entry["alg_bytes_per_launch"], 3) if entry.get("alg_bytes_per_launch") else None,
                  "pmc_launches": p["launches"], "pmc_source": p["source"]})
    if fam.startswith("checksum") and p["valu_insts"]:
        rate = p["valu_insts"] / (entry["avg_launch_ms"] * 1e6)
        entry["valu"] = {"achieved": round(rate, 2), "peak": VALU_PEAK_GINST, "unit": "G wave-instr/s",
                         "frac": round(rate / VALU_PEAK_GINST, 4), "valu_insts_per_launch": round(p["valu_insts"]),
                         "lds_insts_per_launch": round(p["lds_insts"])}
    return entry


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


def cpu_baseline(gpu_window, members, seconds_budget=50.0):
    """The CPU oracle on a bounded sample of the same protocol at the GPU line's own N (tools/cpu_baseline.py does the
    timing in a child process so that OpenMP threads do not share this process with the HIP runtime): the reference
    cost model and the optimized port, each on the box's cores and on one thread, over the first rounds
    of the GPU window that fit the budget (at 65,536 members a cascade round of the reference cost model takes tens of
    seconds); the line's window_note says which rounds each covers."""
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "cpu_baseline.py"), "--budget",
                          str(seconds_budget), "--window", gpu_window, "--members", str(members), "--variants",
                          "ref,opt,ref1,opt1"],
                         stdout=subprocess.PIPE, text=True, timeout=1200)   # (its progress lines pass to stderr)
    if out.returncode != 0:
        return {"error": f"tools/cpu_baseline.py exit {out.returncode}"}
    return json.loads(out.stdout.strip().splitlines()[-1])


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpu_count():
    """GPUs this process may use, counted without initialising HIP (a parent that touched the GPU must not
    re-launch under torch.distributed.run): the *_VISIBLE_DEVICES lists when set, else the KFD topology's GPU
    nodes (nodes with SIMDs). None when neither is readable; each rank then checks LOCAL_RANK itself."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() != ""])
    root = "/sys/class/kfd/kfd/topology/nodes"
    try:
        count = 0
        for node in os.listdir(root):
            with open(os.path.join(root, node, "properties")) as f:
                props = dict(l.split()[:2] for l in f if len(l.split()) >= 2)
            count += int(props.get("simd_count", "0")) > 0
        return count
    except (OSError, ValueError):
        return None


def emit(obj):
    """One JSON line in ONE write(2): ranks sharing a pipe never interleave their lines (< PIPE_BUF bytes)."""
    os.write(1, (json.dumps(obj) + "\n").encode())


def launch_ranks(args):
    """--gpus N without a launcher: start N ranks as a child torch.distributed.run, relay its status."""
    if not args.launch_check and not args.host_transport:   # (--host-transport: every rank on GPU 0, by design)
        have = visible_gpu_count()
        if have is not None and have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but only {have} GPU(s) visible", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def make_workload(name, n, total_rounds):
    from swimsim import workloads as W

    if name == "config3":
        return W.config3(n=n, rounds=max(total_rounds, KILL_ROUND + 1), kill_round=KILL_ROUND)
    if name == "config2":
        return W.config2(n=n, rounds=total_rounds)
    if name == "config4":
        return W.config4(n=n, rounds=total_rounds)
    if name == "selfstart":
        return W.selfstart(n=n, seeds=2, rounds=total_rounds)
    return W.config5(n=n, rounds=total_rounds)


def new_cluster(swimsim, wl, device, tuning):
    """the workload's start: converged rows, or (selfstart) rows that know only themselves plus the seed members, which
    every node learns by MakeChange before round 0 (untimed)"""
    eng = swimsim.Cluster(wl.n, device=device, tuning=tuning, init=wl.init)
    for o in range(wl.n):
        for m in wl.seed_members:
            if m != o:
                eng.make_change(o, m, swimsim.T0_MS, swimsim.ALIVE)
    return eng


def rounds_to_heal(swimsim, wl, device, tuning, heal_round):
    """config4: an untimed replay of the workload, one round per call, until the reference's convergence test holds
    (test_utils.go:164-199: every live node has no changes and all checksums are equal); rounds after heal_round"""
    eng = new_cluster(swimsim, wl, device, tuning)
    try:
        for r in range(wl.rounds):
            eng.step(1, wl.events_for(r))
            if r >= heal_round and eng.converged():
                return r + 1 - heal_round
        return None
    finally:
        eng.close()


def workload_line(args, wl, n, dt, value, live_mr, dominant, entries, kt, counters, units, eng):
    """the JSON line of a --workload other than config3 (1 GPU): the same fields as the headline line, the dense merges'
    roofline entry beside the dominant kernel, and (config4) the rounds from the heal to convergence"""
    import swimsim

    dom = entries.get(dominant) or {}
    line = {
        "metric": f"simulated member-rounds/sec, {WORKLOADS[args.workload][1]} at {n} members",
        "value": round(value, 1), "unit": "member-rounds/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt * 1e3 / args.steps, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u32",
        "data": f"synthetic ({wl.description}; Philox seeds as swimsim.workloads)",
        "config": {"workload": f"{WORKLOADS[args.workload][1]}: {wl.name}, rounds {args.warmup}-{args.warmup + args.steps - 1} "
                               "timed", "members": n, "rounds_timed": args.steps, "live_member_rounds": live_mr,
                   "parallelism": "1 GPU"},
        "roofline": {"bound": dom_bound(dominant, dom), **dom, "dominant_family": dominant,
                     "kernels": {f: e for f, e in entries.items() if e and f != dominant},
                     "merge_kernel": entries.get("recv_merge"), "dense_merge_kernel": entries.get("rfs_merge")},
        "kernel_ms": {k: round(v["avg_ms"] * v["launches"], 3) for k, v in kt.items() if v["launches"]},
        "kernel_ms_note": "HIP-event device time over the window of the roofline's families and k_jobs_merge",
        "counters": counters,
        "dense_merges": {k: int(v) for k, v in units.items() if k in ("dense_resp", "dense_jobs", "jobs_applied",
                                                                     "dense_heal")},
        "checksum_paths": eng.checksum_path_stats(),
    }
    if line["roofline"]["bound"] == "valu":
        line["roofline"]["bound_frac"] = (dom.get("valu") or {}).get("frac")
    if args.workload == "config4":
        eng.close()                                                # (the replay allocates a cluster of its own)
        heal_round = min(e[0] for e in wl.events if e[1] == 6)    # EV_HEAL
        line["rounds_to_heal"] = rounds_to_heal(swimsim, wl, 0, None, heal_round)
        line["rounds_to_heal_basis"] = (f"rounds from the first heal (r={heal_round}) until every live node has no changes "
                                        "and all checksums are equal (test_utils.go:164-199), untimed replay")
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=90)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--members", type=int, default=0)        # 0: the workload's default (config3: 65,536)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="config3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ring", action="store_true")
    # diagnostics: every rank on cuda:0, shards exchanging through the gloo host transport instead of
    # RCCL (lets the multi-process path run on a one-GPU machine); never used for reported numbers
    ap.add_argument("--host-transport", action="store_true")
    # the reference-row checksum path (swimsim_tuning.cs_ref: 0 off, 1 wide launches; default: the library's)
    ap.add_argument("--cs-ref", type=int, default=-1)
    ap.add_argument("--cs-async-rows", type=int, default=-1)   # side-stream checksum launches up to this many rows
    ap.add_argument("--time-all", action="store_true")   # HIP events around every kernel family (diagnostics)
    # test hook: the ranks report (rank, world size) and exit before any GPU call
    ap.add_argument("--launch-check", action="store_true")
    args = ap.parse_args()

    if args.members <= 0:
        args.members = WORKLOADS[args.workload][0]
    if args.gpus > 1 and args.workload != "config3":
        raise SystemExit("bench.py: --workload other than config3 is a 1-GPU line")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    ws, rank, local = dist_env()
    if ws != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}")
    if args.launch_check:
        emit({"rank": rank, "world_size": ws, "local_rank": local})
        return

    import torch

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs an MI355X (no GPU visible)")
    if args.host_transport:
        local = 0
    if local >= torch.cuda.device_count():
        raise SystemExit(f"bench.py: rank {rank} needs GPU {local}, but {torch.cuda.device_count()} are visible")
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
    tuning = {k: v for k, v in (("cs_ref", args.cs_ref), ("cs_async_rows", args.cs_async_rows)) if v >= 0} or None
    wl = make_workload(args.workload, n, total_rounds)
    nkilled = sum(1 for e in wl.events if e[1] == W.EV_KILL and e[0] == KILL_ROUND)
    if ws > 1:
        from swimsim import dist as sd

        if args.host_transport:
            eng = swimsim.Cluster(n, device=0, comm=(ws, rank, sd.GlooTransport()), tuning=tuning)
        else:
            eng = sd.sharded_cluster(n, device=local, tuning=tuning)
    else:
        eng = new_cluster(swimsim, wl, local, tuning)

    def barrier():
        if ws > 1:
            import torch.distributed as dist

            dist.barrier()
        torch.cuda.synchronize()

    for r in range(args.warmup):
        eng.step(1, wl.events_for(r))
    # (level 2: HIP events around the roofline's kernels only; every other family's event pair cost the window ~10 us)
    eng.enable_timing(1 if args.time_all else 2 if args.workload == "config3" else 3)
    if rank == 0:
        eng.profile_mark(MARK_BEGIN)    # rocprofv3 counter passes are cut to the launches between the two marks
    barrier()
    t0 = time.perf_counter()
    ev = [e for e in wl.events if args.warmup <= e[0] < total_rounds]
    eng.step(args.steps, ev)
    barrier()
    dt = time.perf_counter() - t0
    if ws > 1:
        from swimsim import dist as sd

        dt = sd.max_over_ranks(dt)

    if rank == 0:
        eng.profile_mark(MARK_END)
    kt = eng.kernel_times()
    units = eng.kernel_units()
    counters = eng.counters()
    shard = eng.shard_info()
    eng.enable_timing(False)
    if ws > 1:
        counters = sd.reduce_counters(counters)
    workload = {"members": n, "steps": args.steps, "warmup": args.warmup, "gpus": ws}
    if args.workload != "config3":
        workload["workload"] = args.workload

    if rank == 0:
        timed_first, timed_last = args.warmup, total_rounds - 1
        live_mr = live_member_rounds(wl, timed_first, timed_last)
        value = live_mr / dt
        dominant = max(kt.items(), key=lambda kv: kv[1]["avg_ms"] * kv[1]["launches"])[0]
        entries = {f: add_pmc(roofline_entry(f, kt, units, n), f, workload) for f in FAMILY_KERNEL}
        dom = entries.get(dominant) or {}
        in_window = timed_first <= KILL_ROUND <= timed_last
        faulty_from = KILL_ROUND + 25       # first suspicions at KILL_ROUND; their timers fire 25 rounds later
        if args.workload != "config3":
            line = workload_line(args, wl, n, dt, value, live_mr, dominant, entries, kt, counters, units, eng)
            sys.stdout.flush()
            emit(line)
            return
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
            "roofline": {"bound": dom_bound(dominant, dom), **dom, "dominant_family": dominant,
                         "kernels": {f: e for f, e in entries.items() if e and f != dominant},
                         "merge_kernel": entries.get("recv_merge")},
            "kernel_ms": {k: round(v["avg_ms"] * v["launches"], 3) for k, v in kt.items() if v["launches"]},
            "kernel_ms_note": ("HIP-event device time over the window of every kernel family" if args.time_all else
                               "HIP-event device time over the window of the families the roofline reports; the others "
                               "are not timed in the window (bench.py --time-all; profiles/ holds rocprofv3 kernel stats)"),
            "counters": counters,
            "checksum_paths": eng.checksum_path_stats(),
            "deferred_decisions": {k: int(units.get(k, 0)) for k in ("defer", "defer_eq", "defer_rep", "defer_undo",
                                                                              "defer_norow")},
        }
        if line["roofline"]["bound"] == "valu":
            line["roofline"]["bound_frac"] = (dom.get("valu") or {}).get("frac")
            line["roofline"]["frac_basis"] = "achieved / peak / frac: HBM bytes of SURVEY.md §8(d); the bound is VALU issue (bound_frac)"
        if ws > 1:
            line["exchange"] = {"bytes_rank0": shard["exchanged_bytes"], "exchanges_rank0": shard["exchanges"],
                                "bytes_per_round_rank0": round(shard["exchanged_bytes"] / max(1, total_rounds), 1),
                                "exchanges_per_round_rank0": round(shard["exchanges"] / max(1, total_rounds), 2),
                                "host_syncs_per_exchange_rank0": round(shard.get("exchange_host_syncs", 0) /
                                                                       max(1, shard["exchanges"]), 2)}
        if ws == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(f"{n}:{args.warmup}:{args.steps}", n)
        if ws == 1 and not args.no_ring:
            line["hashring"] = ring_bench(n)
        sys.stdout.flush()
        emit(line)
    if ws > 1:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
