"""ctypes binding to the CPU oracle (oracle/swim_oracle.c). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module. The
product library (libswimsim.so) never loads the oracle.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "build", "libswim_oracle.so")
# OpenMP build of the same source: bench.py's cpu_baseline leg only (ORACLE_LIB selects it)
OMP_LIB_PATH = os.path.join(ORACLE_DIR, "build", "libswim_oracle_omp.so")

ALIVE, SUSPECT, FAULTY, LEAVE, TOMBSTONE, UNKNOWN = 0, 1, 2, 3, 4, 7
SOURCE_NONE = -1
EV_KILL, EV_REVIVE, EV_REINCARNATE, EV_LEAVE, EV_PARTITION, EV_HEAL, EV_REAP = 1, 2, 3, 4, 5, 6, 7
COUNTER_NAMES = [
    "rounds", "pings", "pings_ok", "pingreqs", "helper_calls", "helper_errors", "inconclusive",
    "suspect_decl", "applied", "refutes", "full_syncs", "full_syncs_pingreq", "rfs_done",
    "rfs_omitted", "timers_fired", "msg_changes", "heal_attempts", "heal_failures",
]
T0_MS = 1_500_000_000_000
PERIOD_MS = 200


class OrChange(C.Structure):
    _fields_ = [("member", C.c_int32), ("status", C.c_int32), ("source", C.c_int32), ("_pad", C.c_int32),
                ("inc", C.c_int64), ("source_inc", C.c_int64)]


class OrConfig(C.Structure):
    _fields_ = [("n", C.c_uint32), ("t0_ms", C.c_int64), ("period_ms", C.c_int64),
                ("suspect_ms", C.c_int64), ("faulty_ms", C.c_int64), ("tombstone_ms", C.c_int64),
                ("ping_request_size", C.c_uint32), ("max_rfs_jobs", C.c_uint32), ("p_factor", C.c_uint32),
                ("faithful_checksum", C.c_uint32), ("seed", C.c_uint64), ("addresses", C.c_char_p),
                ("addr_stride", C.c_uint32), ("reference_cost", C.c_uint32)]


class OrEvent(C.Structure):
    _fields_ = [("round", C.c_uint32), ("kind", C.c_uint32), ("a", C.c_int32), ("b", C.c_int32)]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        path = os.environ.get("ORACLE_LIB", LIB_PATH)
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        P = C.c_void_p
        u32, i32, i64, u64 = C.c_uint32, C.c_int32, C.c_int64, C.c_uint64
        sig = {
            "or_create": (P, [C.POINTER(OrConfig)]),
            "or_destroy": (None, [P]),
            "or_init_converged": (None, [P]),
            "or_init_self_only": (None, [P]),
            "or_set_member": (None, [P, u32, u32, i32, i64]),
            "or_set_clock_offset": (None, [P, u32, i64]),
            "or_set_live": (None, [P, u32, i32]),
            "or_set_partition": (None, [P, u32, i32]),
            "or_set_round": (None, [P, u32]),
            "or_set_maxp": (None, [P, u32, i32, i32]),
            "or_make_change": (C.c_int, [P, u32, u32, i64, i32]),
            "or_clear_changes": (None, [P, u32]),
            "or_step": (None, [P, C.POINTER(OrEvent), C.c_size_t]),
            "or_round": (u32, [P]),
            "or_checksum": (u32, [P, u32]),
            "or_row": (None, [P, u32, P, P]),
            "or_maxp": (i32, [P, u32]),
            "or_num_pingable": (i32, [P, u32]),
            "or_count_reachable": (i32, [P, u32]),
            "or_num_members": (i32, [P, u32]),
            "or_changes_count": (i32, [P, u32]),
            "or_dis_entries": (i32, [P, u32, P, P, P, P, i32]),
            "or_timer_entries": (i32, [P, u32, P, P, P, P, P, i32]),
            "or_iter_state": (None, [P, u32, C.POINTER(i64), C.POINTER(u32)]),
            "or_counters": (None, [P, P]),
            "or_last_targets": (i32, [P, P]),
            "or_live": (i32, [P, u32]),
            "or_digest": (None, [P, C.POINTER(u64), C.POINTER(u64), C.POINTER(u64)]),
            "or_watch": (None, [P, u32, i32]),
            "or_drain_applied": (i32, [P, u32, C.POINTER(OrChange), i32, C.POINTER(u32), C.POINTER(u32),
                                       C.POINTER(i32)]),
            "or_drain_events": (i32, [P, u32, C.POINTER(OrChange), P, i32, C.POINTER(u32), C.POINTER(u32),
                                      C.POINTER(i32)]),
            "or_non_local_override": (i32, [i64, i32, i64, i32]),
            "or_local_override": (i32, [i32, i64, i64, i32]),
            "or_update": (i32, [P, u32, C.POINTER(OrChange), i32, C.POINTER(OrChange), i32]),
            "or_add_join_list": (i32, [P, u32, C.POINTER(OrChange), i32]),
            "or_clear_change": (None, [P, u32, u32]),
            "or_issue_as_sender": (i32, [P, u32, C.POINTER(OrChange), i32]),
            "or_issue_as_receiver": (i32, [P, u32, i32, i64, u32, C.POINTER(OrChange), i32, C.POINTER(i32)]),
            "or_bump": (None, [P, u32, C.POINTER(OrChange), i32]),
            "or_membership_as_changes": (i32, [P, u32, C.POINTER(OrChange), i32]),
            "or_next": (i32, [P, u32]),
            "or_random_pingable": (i32, [P, u32, i32, i32, P]),
            "or_fire_timers": (None, [P, u32]),
            "or_heal": (i32, [P, u32, P, i32]),
            "or_schedule": (None, [P, u32, u32, i32, i64]),
            "or_cancel": (None, [P, u32, u32]),
            "or_fingerprint32": (u32, [C.c_char_p, C.c_size_t]),
            "or_philox4x32_10": (None, [P, P, P]),
            "or_perm": (u32, [u64, u32, u32, u32, u32]),
            "or_perm_inv": (u32, [u64, u32, u32, u32, u32]),
            "or_checksum_string": (C.c_size_t, [P, u32, C.c_char_p, C.c_size_t]),
            "or_ring_new": (P, [u32]),
            "or_ring_free": (None, [P]),
            "or_ring_add_remove": (i32, [P, P, C.c_size_t, P, C.c_size_t]),
            "or_ring_checksum": (u32, [P]),
            "or_ring_server_count": (u32, [P]),
            "or_ring_lookup": (C.c_char_p, [P, C.c_char_p, C.c_size_t]),
            "or_ring_lookup_n": (C.c_size_t, [P, C.c_char_p, C.c_size_t, u32, P]),
            "or_ring_points": (C.c_size_t, [P, P, P, C.c_size_t]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def fingerprint32(b: bytes) -> int:
    return lib().or_fingerprint32(b, len(b))


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().or_philox4x32_10(c, k, o)
    return list(o)


def _changes(lst):
    arr = (OrChange * max(1, len(lst)))()
    for i, c in enumerate(lst):
        arr[i].member, arr[i].status, arr[i].inc = c[0], c[1], c[2]
        arr[i].source = c[3] if len(c) > 3 else SOURCE_NONE
        arr[i].source_inc = c[4] if len(c) > 4 else 0
    return arr


def _unpack(arr, n):
    return [(arr[i].member, arr[i].status, arr[i].inc, arr[i].source, arr[i].source_inc) for i in range(n)]


class OracleSim:
    """One simulated cluster. Observer o == member o (a swim.Node)."""

    def __init__(self, n, *, t0_ms=T0_MS, period_ms=PERIOD_MS, suspect_ms=5000, faulty_ms=24 * 3600 * 1000,
                 tombstone_ms=60_000, ping_request_size=3, max_rfs_jobs=5, p_factor=15, seed=1,
                 faithful_checksum=False, reference_cost=False, addresses=None, init="converged"):
        L = lib()
        self.n = n
        self.t0_ms, self.period_ms = t0_ms, period_ms
        cfg = OrConfig(n, t0_ms, period_ms, suspect_ms, faulty_ms, tombstone_ms, ping_request_size, max_rfs_jobs,
                       p_factor, int(bool(faithful_checksum)), seed, None, 0, int(bool(reference_cost)))
        self._addr_buf = None
        if addresses is not None:
            stride = max(len(a) for a in addresses) + 1
            buf = b"".join(a.encode().ljust(stride, b"\0") for a in addresses)
            self._addr_buf = C.create_string_buffer(buf, len(buf))
            cfg.addresses = C.cast(self._addr_buf, C.c_char_p)
            cfg.addr_stride = stride
        self.h = L.or_create(C.byref(cfg))
        if init == "converged":
            L.or_init_converged(self.h)
        elif init == "self":
            L.or_init_self_only(self.h)
        # init=None: every row empty (all UNKNOWN), as a fresh swim.NewNode

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_destroy(self.h)
            self.h = None

    # --- driving ---
    def step(self, events=()):
        ev = (OrEvent * max(1, len(events)))()
        for i, (r, k, a, b) in enumerate(events):
            ev[i].round, ev[i].kind, ev[i].a, ev[i].b = r, k, a, b
        lib().or_step(self.h, ev, len(events))

    def run(self, rounds, events=()):
        for _ in range(rounds):
            r = self.round
            self.step([e for e in events if e[0] == r])

    @property
    def round(self):
        return lib().or_round(self.h)

    # --- setup ---
    def set_member(self, o, m, status, inc):
        lib().or_set_member(self.h, o, m, status, inc)

    def make_change(self, o, m, inc, status):
        return lib().or_make_change(self.h, o, m, inc, status)

    def clear_changes(self, o):
        lib().or_clear_changes(self.h, o)

    def set_clock_offset(self, o, off):
        lib().or_set_clock_offset(self.h, o, off)

    def set_live(self, o, live):
        lib().or_set_live(self.h, o, int(live))

    def set_partition(self, o, label):
        lib().or_set_partition(self.h, o, label)

    def set_round(self, r):
        lib().or_set_round(self.h, r)

    def set_maxp(self, o, maxp, pfactor):
        lib().or_set_maxp(self.h, o, maxp, pfactor)

    # --- readback ---
    def checksum(self, o):
        return lib().or_checksum(self.h, o)

    def checksums(self):
        return np.array([self.checksum(o) for o in range(self.n)], dtype=np.uint32)

    def row(self, o):
        st = np.empty(self.n, np.uint8)
        inc = np.empty(self.n, np.int64)
        lib().or_row(self.h, o, st.ctypes.data, inc.ctypes.data)
        return st, inc

    def rows(self):
        st = np.empty((self.n, self.n), np.uint8)
        inc = np.empty((self.n, self.n), np.int64)
        for o in range(self.n):
            st[o], inc[o] = self.row(o)
        return st, inc

    def member(self, o, m):
        st, inc = self.row(o)
        return int(st[m]), int(inc[m])

    def maxp(self, o):
        return lib().or_maxp(self.h, o)

    def num_pingable(self, o):
        return lib().or_num_pingable(self.h, o)

    def count_reachable(self, o):
        return lib().or_count_reachable(self.h, o)

    def num_members(self, o):
        return lib().or_num_members(self.h, o)

    def changes_count(self, o):
        return lib().or_changes_count(self.h, o)

    def dis_entries(self, o):
        cap = self.n
        m = np.empty(cap, np.int32); p = np.empty(cap, np.int32); s = np.empty(cap, np.int32)
        si = np.empty(cap, np.int64)
        k = lib().or_dis_entries(self.h, o, m.ctypes.data, p.ctypes.data, s.ctypes.data, si.ctypes.data, cap)
        return {int(m[i]): (int(p[i]), int(s[i]), int(si[i])) for i in range(k)}

    def timer_entries(self, o):
        cap = self.n
        m = np.empty(cap, np.int32); st = np.empty(cap, np.int32); f = np.empty(cap, np.int32)
        dl = np.empty(cap, np.int64); sj = np.empty(cap, np.int64)
        k = lib().or_timer_entries(self.h, o, m.ctypes.data, st.ctypes.data, f.ctypes.data, dl.ctypes.data,
                                   sj.ctypes.data, cap)
        return {int(m[i]): (int(st[i]), int(f[i]), int(dl[i]), int(sj[i])) for i in range(k)}

    def iter_state(self, o):
        idx, ep = C.c_int64(), C.c_uint32()
        lib().or_iter_state(self.h, o, C.byref(idx), C.byref(ep))
        return idx.value, ep.value

    def counters(self):
        out = np.zeros(len(COUNTER_NAMES), np.uint64)
        lib().or_counters(self.h, out.ctypes.data)
        return dict(zip(COUNTER_NAMES, (int(x) for x in out)))

    def last_targets(self):
        out = np.empty(self.n, np.int32)
        lib().or_last_targets(self.h, out.ctypes.data)
        return out

    def live(self, o):
        return bool(lib().or_live(self.h, o))

    def digest(self):
        a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        lib().or_digest(self.h, C.byref(a), C.byref(b), C.byref(c))
        return a.value, b.value, c.value

    def checksum_string(self, o):
        n = lib().or_checksum_string(self.h, o, None, 0)
        buf = C.create_string_buffer(n + 1)
        lib().or_checksum_string(self.h, o, buf, n)
        return buf.raw[:n]

    # --- applied-change stream (MemberlistChangesAppliedEvent, swim/events.go:56-61) ---
    def watch(self, o, on=True):
        """on: True = coalesced drains; "events" = also the per-Update stream; False = off"""
        lib().or_watch(self.h, o, 2 if on == "events" else int(bool(on)))

    def drain_events(self, o):
        """per-Update stream of observer o: ([[change, ...] per applying Update in Update order], old checksum,
        new checksum, NumMembers); changes as (member, status, inc, source, source_inc) in apply order"""
        cap = 4 * self.n + 4096
        out = (OrChange * cap)()
        seq = np.empty(cap, np.int32)
        a, b, c = C.c_uint32(), C.c_uint32(), C.c_int32()
        k = lib().or_drain_events(self.h, o, out, seq.ctypes.data, cap, C.byref(a), C.byref(b), C.byref(c))
        if k < 0:
            raise ValueError(f"observer {o} has no per-Update stream")
        ch = _unpack(out, min(k, cap))
        events = []
        for i, x in enumerate(ch):
            if int(seq[i]) == len(events):
                events.append([])
            events[-1].append(x)
        return events, a.value, b.value, c.value

    def drain_applied(self, o):
        """(changes, old checksum, new checksum, NumMembers) since the last drain of watched observer o;
        changes = [(member, status, inc, source, source_inc)] in member order"""
        out = (OrChange * self.n)()
        a, b, c = C.c_uint32(), C.c_uint32(), C.c_int32()
        k = lib().or_drain_applied(self.h, o, out, self.n, C.byref(a), C.byref(b), C.byref(c))
        if k < 0:
            raise ValueError(f"observer {o} is not watched")
        return _unpack(out, k), a.value, b.value, c.value

    # --- unit-level primitives (reference KATs) ---
    def update(self, j, changes):
        arr = _changes(changes)
        out = (OrChange * max(1, len(changes)))()
        k = lib().or_update(self.h, j, arr, len(changes), out, len(changes))
        return _unpack(out, k)

    def add_join_list_changes(self, j, changes):
        """memberlist.AddJoinList of (member, status, inc, source, source_inc) tuples; #applied"""
        return lib().or_add_join_list(self.h, j, _changes(changes), len(changes))

    def issue_as_sender(self, j):
        out = (OrChange * self.n)()
        k = lib().or_issue_as_sender(self.h, j, out, self.n)
        return _unpack(out, k)

    def issue_as_receiver(self, j, sender, sender_inc, sender_cs):
        out = (OrChange * self.n)()
        fs = C.c_int32()
        k = lib().or_issue_as_receiver(self.h, j, sender, sender_inc, sender_cs, out, self.n, C.byref(fs))
        return _unpack(out, k), bool(fs.value)

    def bump(self, j, changes):
        arr = _changes(changes)
        lib().or_bump(self.h, j, arr, len(changes))

    def membership_as_changes(self, j):
        out = (OrChange * self.n)()
        k = lib().or_membership_as_changes(self.h, j, out, self.n)
        return _unpack(out, k)

    def next(self, o):
        return lib().or_next(self.h, o)

    def random_pingable(self, o, k, exclude):
        out = np.empty(max(1, k), np.int32)
        got = lib().or_random_pingable(self.h, o, k, exclude, out.ctypes.data)
        return [int(x) for x in out[:got]]

    def fire_timers(self, o):
        lib().or_fire_timers(self.h, o)

    def heal(self, o):
        out = np.empty(self.n, np.int32)
        k = lib().or_heal(self.h, o, out.ctypes.data, self.n)
        return [int(x) for x in out[:min(k, self.n)]]

    def schedule(self, o, m, state, subj):
        lib().or_schedule(self.h, o, m, state, subj)

    def cancel(self, o, m):
        lib().or_cancel(self.h, o, m)

    def converged(self):
        """test_utils.go:188-198: no live node has changes and all live checksums are equal."""
        live = [o for o in range(self.n) if self.live(o)]
        if any(self.changes_count(o) for o in live):
            return False
        return len({self.checksum(o) for o in live}) <= 1


def perm(seed, o, epoch, n, idx):
    return lib().or_perm(seed, o, epoch, n, idx)


def perm_inv(seed, o, epoch, n, m):
    return lib().or_perm_inv(seed, o, epoch, n, m)


def _cstrs(lst):
    arr = (C.c_char_p * max(1, len(lst)))(*[x.encode() for x in lst])
    return arr, len(lst)


class OracleRing:
    """CPU restatement of hashring.HashRing (oracle/ring_oracle.c); test infrastructure only."""

    def __init__(self, replica_points=100):
        self.h = lib().or_ring_new(replica_points)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_ring_free(self.h)
            self.h = None

    def add_remove_servers(self, add=(), remove=()):
        a, na = _cstrs(list(add))
        r, nr = _cstrs(list(remove))
        return bool(lib().or_ring_add_remove(self.h, a, na, r, nr))

    def checksum(self):
        return lib().or_ring_checksum(self.h)

    def server_count(self):
        return lib().or_ring_server_count(self.h)

    def lookup(self, key):
        k = key.encode() if isinstance(key, str) else key
        v = lib().or_ring_lookup(self.h, k, len(k))
        return (v.decode(), True) if v is not None else ("", False)

    def lookup_n(self, key, n):
        k = key.encode() if isinstance(key, str) else key
        out = (C.c_char_p * max(1, n + self.server_count()))()
        got = lib().or_ring_lookup_n(self.h, k, len(k), n, out)
        return [out[i].decode() for i in range(got)]

    def points(self):
        n = lib().or_ring_points(self.h, None, None, 0)
        hs = (C.c_uint32 * max(1, n))()
        own = (C.c_char_p * max(1, n))()
        lib().or_ring_points(self.h, hs, own, n)
        return [(hs[i], own[i].decode()) for i in range(n)]
