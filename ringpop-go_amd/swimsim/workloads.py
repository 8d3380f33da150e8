"""Synthetic workloads of BASELINE.json's five configs, as event lists for Cluster.step().

Events are pure inputs. The same list drives the MI355X engine and the CPU oracle. Random picks
use the Philox4x32-10 stream of docs/ROUND_SEMANTICS.md §6, with counter (round, 0, purpose, i>>2),
so every run and every backend sees the same members.
"""
from __future__ import annotations

from dataclasses import dataclass, field

EV_KILL, EV_REVIVE, EV_REINCARNATE, EV_LEAVE, EV_PARTITION, EV_HEAL, EV_REAP = 1, 2, 3, 4, 5, 6, 7
M32 = 0xFFFFFFFF


def philox4x32_10(c0, c1, c2, c3, seed):
    k0, k1 = seed & M32, (seed >> 32) & M32
    for r in range(10):
        if r:
            k0 = (k0 + 0x9E3779B9) & M32
            k1 = (k1 + 0xBB67AE85) & M32
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & M32, p1 & M32, ((p0 >> 32) ^ c3 ^ k1) & M32, p0 & M32
    return c0, c1, c2, c3


def stream(seed, r, purpose, count):
    out, blk = [], None
    for i in range(count):
        if i % 4 == 0:
            blk = philox4x32_10(r, 0, purpose, i >> 2, seed)
        out.append(blk[i & 3])
    return out


def distinct_members(seed, r, purpose, k, n):
    """k distinct members by rejection on the Philox stream (index = floor(u32 * n / 2^32))."""
    chosen, seen, i = [], set(), 0
    while len(chosen) < min(k, n):
        blk = philox4x32_10(r, 0, purpose, i >> 2, seed)
        m = (blk[i & 3] * n) >> 32
        i += 1
        if m not in seen:
            seen.add(m)
            chosen.append(m)
    return chosen


@dataclass
class Workload:
    name: str
    n: int
    rounds: int
    events: list = field(default_factory=list)
    description: str = ""
    until_converged: bool = False
    init: str = "converged"                      # initial rows: "converged" (everyone knows everyone) or "self"
    seed_members: list = field(default_factory=list)   # members every node learns by MakeChange before round 0

    def events_for(self, r):
        return [e for e in self.events if e[0] == r]


def config1(n=16, rounds=300):
    """ringpop-go swim 16-member in-process cluster, 1 member killed, rounds to convergence."""
    return Workload("config1_kill_one", n, rounds, [(0, EV_KILL, 5 % n, 0)],
                    "kill member 5 at r=0; run until converged with member 5 faulty everywhere", until_converged=True)


def config2(n=4096, rounds=200, churn=0.01, seed=7):
    """1% random churn per round: each pick toggles kill <-> revive (revive = Reincarnate)."""
    k = max(1, int(round(n * churn)))
    dead, ev = set(), []
    for r in range(rounds):
        for m in distinct_members(seed, r, 4, k, n):
            if m in dead:
                dead.discard(m)
                ev.append((r, EV_REVIVE, m, 0))
            else:
                dead.add(m)
                ev.append((r, EV_KILL, m, 0))
    return Workload(f"config2_churn_n{n}", n, rounds, ev, f"{k} members toggled kill/revive per round")


def config3(n=65536, rounds=100, frac=0.01, kill_round=10, seed=11):
    """steady-state gossip, then 1% killed at r=10: suspect wave, then faulty wave ~25 rounds later."""
    k = max(1, int(n * frac))
    ev = [(kill_round, EV_KILL, m, 0) for m in distinct_members(seed, kill_round, 5, k, n)]
    return Workload(f"config3_cascade_n{n}", n, rounds, ev, f"{k} members killed at r={kill_round}")


def config4(n=16384, rounds=140, split_until=60, heals=(60, 80), healer=0):
    """2-way partition for rounds [0, split_until), then the mask is cleared and Heal runs on one node."""
    half = n // 2
    ev = [(0, EV_PARTITION, m, 1) for m in range(half, n)]
    ev += [(split_until, EV_PARTITION, m, 0) for m in range(half, n)]
    ev += [(h, EV_HEAL, healer, 0) for h in heals]
    return Workload(f"config4_partition_heal_n{n}", n, rounds, ev,
                    f"halves partitioned r<{split_until}; heal on {healer} at r={list(heals)}", until_converged=True)


def config5(n=262144, rounds=100, frac=0.10, every=20, seed=13):
    """large incarnation bursts: every 20 rounds 10% of members Reincarnate simultaneously."""
    k = max(1, int(n * frac))
    ev = []
    for r in range(0, rounds, every):
        ev += [(r, EV_REINCARNATE, m, 0) for m in distinct_members(seed, r, 6, k, n)]
    return Workload(f"config5_bursts_n{n}", n, rounds, ev, f"{k} members reincarnate every {every} rounds")


def selfstart(n=16384, seeds=2, rounds=40):
    """Every node starts knowing only itself (a swim.Node before Bootstrap) plus members 0..seeds-1, which each node
    learns by MakeChange (memberlist.go:282-307). Gossip spreads the seeded changes; once a sender's filtered
    changes run dry while the two checksums differ, the receiver answers with its whole membership (full sync,
    disseminator.go:156-181) and the sender asks back (reverse full sync, disseminator.go:257-304), so both paths
    run at size."""
    return Workload(f"selfstart_n{n}_s{seeds}", n, rounds, [], f"self-only start, members 0..{seeds - 1} seeded by "
                    f"MakeChange at every node", init="self", seed_members=list(range(seeds)))

