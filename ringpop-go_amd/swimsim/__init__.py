"""swimsim — Python host binding of libswimsim.so, the MI355X SWIM protocol-round engine.

The classes mirror the reference's swim package surface (maniacs-ops/ringpop-go):
  * ``Cluster``: N simulated ``swim.Node`` processes driven in synchronous protocol rounds.
  * ``Node``: ``swim.NodeInterface`` (swim/node.go:137-147): GetChecksum, CountReachableMembers,
    GetReachableMembers, MemberStats, Incarnation, plus ``memberlist`` and ``disseminator`` views.
  * ``Memberlist``: Checksum, Member, NumMembers, NumPingableMembers, MakeChange...
    (swim/memberlist.go).
  * ``Disseminator``: ChangesCount, ChangesByAddress, HasChanges, MaxP, ClearChanges
    (swim/disseminator.go).

Everything runs through the C ABI of include/swimsim.h and its gfx950 HIP kernels. There is no CPU
fallback. If the library is missing or no device is usable, construction raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SWIMSIM_LIB (diagnostics only): load another build of the library, e.g. a kernel variant under test
LIB_PATH = os.environ.get("SWIMSIM_LIB") or os.path.join(_HERE, "libswimsim.so")

ALIVE, SUSPECT, FAULTY, LEAVE, TOMBSTONE, UNKNOWN = 0, 1, 2, 3, 4, 7
STATUS_NAMES = {ALIVE: "alive", SUSPECT: "suspect", FAULTY: "faulty", LEAVE: "leave", TOMBSTONE: "tombstone"}
SOURCE_NONE = -1
EV_KILL, EV_REVIVE, EV_REINCARNATE, EV_LEAVE, EV_PARTITION, EV_HEAL, EV_REAP = 1, 2, 3, 4, 5, 6, 7
COUNTER_NAMES = [
    "rounds", "pings", "pings_ok", "pingreqs", "helper_calls", "helper_errors", "inconclusive",
    "suspect_decl", "applied", "refutes", "full_syncs", "full_syncs_pingreq", "rfs_done",
    "rfs_omitted", "timers_fired", "msg_changes", "heal_attempts", "heal_failures",
]
T0_MS = 1_500_000_000_000
ERRORS = {-1: "EINVAL", -2: "ENOMEM", -3: "EHIP", -4: "ECAPACITY", -5: "ERANGE"}


class SwimsimError(RuntimeError):
    pass


class Config(C.Structure):
    _fields_ = [
        ("num_members", C.c_uint32), ("device", C.c_uint32), ("t0_ms", C.c_int64),
        ("protocol_period_ms", C.c_uint32), ("suspect_timeout_ms", C.c_uint32), ("faulty_timeout_ms", C.c_uint32),
        ("tombstone_timeout_ms", C.c_uint32), ("ping_request_size", C.c_uint32),
        ("max_reverse_full_sync_jobs", C.c_uint32), ("p_factor", C.c_uint32), ("seed", C.c_uint64),
        ("addresses", C.c_char_p), ("addr_stride", C.c_uint32), ("max_rounds", C.c_uint32),
        ("message_pool_bytes", C.c_uint64), ("observer_begin", C.c_uint32), ("observer_end", C.c_uint32),
        ("tuning", C.c_void_p),
    ]


class Tuning(C.Structure):
    """swimsim_tuning (include/swimsim.h): engine variants for tests and diagnostics, -1 = the production default."""
    _fields_ = [("hot_slots", C.c_int32), ("dense_slots", C.c_int32), ("cs_async", C.c_int32),
                ("cs_async_rows", C.c_int32), ("cs_narrow_rows", C.c_int32), ("cs_ref", C.c_int32),
                ("fault_inject", C.c_int32)]


def make_tuning(tuning):
    """a Tuning struct from a dict of its fields (None: the production engine)"""
    if not tuning:
        return None
    t = Tuning(*([-1] * len(Tuning._fields_)))
    for k, v in tuning.items():
        if k not in dict(Tuning._fields_):
            raise ValueError(f"unknown tuning field {k}")
        setattr(t, k, int(v))
    return t


class Event(C.Structure):
    _fields_ = [("round", C.c_uint32), ("kind", C.c_uint32), ("a", C.c_int32), ("b", C.c_int32)]


_U64P = C.POINTER(C.c_uint64)
ALLTOALL_U64 = C.CFUNCTYPE(C.c_int, C.c_void_p, _U64P, _U64P, C.c_int32)
ALLTOALLV = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, _U64P, _U64P, C.c_void_p, _U64P, _U64P)
BCAST = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32)


class ProtocolStatsC(C.Structure):
    """swimsim_protocol_stats_t (include/swimsim.h)"""
    _fields_ = [("count", C.c_int64)] + [(f, C.c_double) for f in (
        "min_ns", "max_ns", "sum_ns", "mean_ns", "variance", "stddev_ns", "median_ns", "p75_ns", "p95_ns", "p99_ns",
        "p999_ns")] + [("protocol_rate_ns", C.c_int64), ("client_rate", C.c_double), ("server_rate", C.c_double),
                       ("total_rate", C.c_double)]


@dataclass
class MemberlistChangesAppliedEvent:
    """swim.MemberlistChangesAppliedEvent (swim/events.go:56-61): changes are swimsim.wire.Change values"""
    changes: list
    old_checksum: int
    new_checksum: int
    num_members: int


class MemoryC(C.Structure):
    """swimsim_memory_t (include/swimsim.h)"""
    _fields_ = [(f, C.c_uint64) for f in ("row_words", "dissemination", "timers", "message_pool", "dense_snapshots",
                                          "total")] + [("dense_cap", C.c_uint32), ("side_cap", C.c_uint32),
                                                       ("lazy_fallbacks", C.c_uint64)]


class HostTransport(C.Structure):
    """swimsim_host_transport (include/swimsim.h): host collectives for one-process-per-shard runs"""
    _fields_ = [("ctx", C.c_void_p), ("alltoall_u64", ALLTOALL_U64), ("alltoallv", ALLTOALLV), ("bcast", BCAST)]


_lib = None


def load_library(path: str = LIB_PATH):
    """Load libswimsim.so. Raises loudly when it is absent: the product has no fallback. SWIMSIM_LIBRARY selects
    another build of the same ABI (tools/: the diagnostics library with the superseded checksum kernels)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("SWIMSIM_LIBRARY", path)
    if not os.path.exists(path):
        raise SwimsimError(f"{path} is missing: build it with `make -C ringpop-go_amd` (hipcc, gfx950)")
    L = C.CDLL(path)
    P, u32, i32, i64, u64, sz = C.c_void_p, C.c_uint32, C.c_int32, C.c_int64, C.c_uint64, C.c_size_t
    sigs = {
        "swimsim_abi_version": (C.c_int, []),
        "swimsim_create": (C.c_int, [C.POINTER(Config), C.POINTER(P)]),
        "swimsim_destroy": (C.c_int, [P]),
        "swimsim_last_error": (C.c_char_p, [P]),
        "swimsim_init_converged": (C.c_int, [P]),
        "swimsim_init_self_only": (C.c_int, [P]),
        "swimsim_set_member": (C.c_int, [P, u32, u32, i32, i64]),
        "swimsim_set_row": (C.c_int, [P, u32, P, P]),
        "swimsim_make_change": (C.c_int, [P, u32, u32, i64, i32]),
        "swimsim_clear_changes": (C.c_int, [P, u32]),
        "swimsim_add_join_list": (C.c_int, [P, u32, P, P, P, P, P, sz, C.POINTER(u32)]),
        "swimsim_set_live": (C.c_int, [P, u32, i32]),
        "swimsim_set_partition": (C.c_int, [P, u32, i32]),
        "swimsim_set_round": (C.c_int, [P, u32]),
        "swimsim_step": (C.c_int, [P, u32, C.POINTER(Event), sz]),
        "swimsim_heal": (C.c_int, [P, u32, P, sz, C.POINTER(sz)]),
        "swimsim_round": (u32, [P]),
        "swimsim_checksums": (C.c_int, [P, P]),
        "swimsim_row": (C.c_int, [P, u32, P, P]),
        "swimsim_count_reachable": (C.c_int, [P, u32, C.POINTER(u32)]),
        "swimsim_reachable": (C.c_int, [P, u32, P, sz, C.POINTER(sz)]),
        "swimsim_node_stats": (C.c_int, [P, u32, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]),
        "swimsim_changes": (C.c_int, [P, u32, P, P, P, P, sz, C.POINTER(sz)]),
        "swimsim_timers": (C.c_int, [P, u32, P, P, P, P, P, sz, C.POINTER(sz)]),
        "swimsim_iter_state": (C.c_int, [P, u32, C.POINTER(i64), C.POINTER(u32)]),
        "swimsim_last_targets": (C.c_int, [P, P]),
        "swimsim_counters": (C.c_int, [P, P]),
        "swimsim_digest": (C.c_int, [P, C.POINTER(u64), C.POINTER(u64), C.POINTER(u64)]),
        "swimsim_converged": (C.c_int, [P, C.POINTER(i32)]),
        "swimsim_kernel_times": (C.c_int, [P, P, P, P, P, sz, C.POINTER(sz)]),
        "swimsim_enable_timing": (C.c_int, [P, i32]),
        "swimsim_bench_checksum": (C.c_int, [P, u32, i32, i32, C.POINTER(C.c_double)]),
        "swimsim_checksum_path_stats": (C.c_int, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), _U64P]),
        "swimsim_kernel_units": (C.c_int, [P, P, P, sz, C.POINTER(sz)]),
        "swimsim_profile_mark": (C.c_int, [P, u32]),
        "swimsim_debug_cs_stream": (C.c_int, [P, u32, P, sz]),
        "swimsim_group_create": (C.c_int, [C.POINTER(Config), u32, P, P]),
        "swimsim_group_step": (C.c_int, [P, u32, u32, C.POINTER(Event), sz]),
        "swimsim_comm_unique_id": (C.c_int, [P, sz]),
        "swimsim_comm_attach": (C.c_int, [P, u32, u32, P, sz]),
        "swimsim_shard_info": (C.c_int, [P, C.POINTER(u32), C.POINTER(u32), C.POINTER(u32), C.POINTER(u32),
                                         C.POINTER(u64), C.POINTER(u64)]),
        "swimsim_exchange_syncs": (C.c_int, [P, C.POINTER(u64)]),
        "swimsim_comm_attach_host": (C.c_int, [P, u32, u32, C.POINTER(HostTransport)]),
        "swimsim_debug_exchange": (C.c_int, [P, P, P, P, sz, P]),
        "swimsim_watch": (C.c_int, [P, u32, i32]),
        "swimsim_applied_changes": (C.c_int, [P, u32, P, P, P, P, P, sz, C.POINTER(sz), C.POINTER(u32),
                                              C.POINTER(u32), C.POINTER(i32)]),
        "swimsim_applied_events": (C.c_int, [P, u32, P, P, P, P, P, P, sz, C.POINTER(sz), C.POINTER(sz),
                                             C.POINTER(u32), C.POINTER(u32), C.POINTER(i32)]),
        "swimsim_protocol_stats": (C.c_int, [P, C.POINTER(ProtocolStatsC)]),
        "swimsim_memory": (C.c_int, [P, C.POINTER(MemoryC)]),
    }
    for name, (res, args) in sigs.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _events(events):
    arr = (Event * max(1, len(events)))()
    for i, (r, k, a, b) in enumerate(events):
        arr[i].round, arr[i].kind, arr[i].a, arr[i].b = int(r), int(k), int(a), int(b)
    return arr


def make_config(n, *, t0_ms=T0_MS, period_ms=200, suspect_ms=5000, faulty_ms=24 * 3600 * 1000, tombstone_ms=60_000,
                ping_request_size=3, max_rfs_jobs=5, p_factor=15, seed=1, device=0, max_rounds=0,
                message_pool_bytes=0, observer_range=None, tuning=None):
    cfg = Config()
    cfg.num_members, cfg.device, cfg.t0_ms, cfg.protocol_period_ms = n, device, t0_ms, period_ms
    cfg.suspect_timeout_ms, cfg.faulty_timeout_ms, cfg.tombstone_timeout_ms = suspect_ms, faulty_ms, tombstone_ms
    cfg.ping_request_size, cfg.max_reverse_full_sync_jobs, cfg.p_factor = ping_request_size, max_rfs_jobs, p_factor
    cfg.seed, cfg.max_rounds, cfg.message_pool_bytes = seed, max_rounds, message_pool_bytes
    if observer_range:
        cfg.observer_begin, cfg.observer_end = observer_range
    cfg._tuning = make_tuning(tuning)               # kept alive with the config
    if cfg._tuning is not None:
        cfg.tuning = C.cast(C.pointer(cfg._tuning), C.c_void_p)
    return cfg


def shard_range(n, nshards, rank):
    """Observer rows of shard `rank` of `nshards` (the canonical split of include/swimsim.h)."""
    return n * rank // nshards, n * (rank + 1) // nshards


def unique_id() -> bytes:
    """A fresh RCCL communicator id (rank 0 makes it; the launcher broadcasts it to the other ranks)."""
    buf = (C.c_uint8 * 128)()
    rc = load_library().swimsim_comm_unique_id(C.cast(buf, C.c_void_p), 128)
    if rc < 0:
        raise SwimsimError(f"swimsim_comm_unique_id failed: {ERRORS.get(rc, rc)}")
    return bytes(buf)


class Cluster:
    """N swim nodes simulated on one MI355X, or one shard of a sharded cluster's observer rows."""

    @classmethod
    def _adopt(cls, h, n, lo, nl, t0_ms=T0_MS, period_ms=200):
        self = cls.__new__(cls)
        self.h, self.n, self.lo, self.nl = h, n, lo, nl
        self.t0_ms, self.period_ms = t0_ms, period_ms
        self._addr_buf = None
        self._listeners = {}
        return self

    def __init__(self, n, *, t0_ms=T0_MS, period_ms=200, suspect_ms=5000, faulty_ms=24 * 3600 * 1000,
                 tombstone_ms=60_000, ping_request_size=3, max_rfs_jobs=5, p_factor=15, seed=1, addresses=None,
                 device=0, init="converged", max_rounds=0, message_pool_bytes=0, observer_range=None, comm=None,
                 tuning=None):
        """comm = (nranks, rank, unique_id): attach this handle as shard `rank` of a cluster spread over
        nranks processes (RCCL); or comm = (nranks, rank, transport) with a swimsim.dist host transport
        object (any process group). observer_range then defaults to the canonical shard.
        tuning = {field: value} of swimsim_tuning (tests and diagnostics: engine variants, identical results)."""
        L = load_library()
        self.n = n
        self.t0_ms, self.period_ms = t0_ms, period_ms
        self._listeners = {}                     # observer -> [listener] (Node.RegisterListener)
        if comm is not None and observer_range is None:
            observer_range = shard_range(n, comm[0], comm[1])
        cfg = Config()
        cfg.num_members, cfg.device, cfg.t0_ms, cfg.protocol_period_ms = n, device, t0_ms, period_ms
        cfg.suspect_timeout_ms, cfg.faulty_timeout_ms, cfg.tombstone_timeout_ms = suspect_ms, faulty_ms, tombstone_ms
        cfg.ping_request_size, cfg.max_reverse_full_sync_jobs, cfg.p_factor = ping_request_size, max_rfs_jobs, p_factor
        cfg.seed, cfg.max_rounds, cfg.message_pool_bytes = seed, max_rounds, message_pool_bytes
        if observer_range:
            cfg.observer_begin, cfg.observer_end = observer_range
        self._tuning = make_tuning(tuning)
        if self._tuning is not None:
            cfg.tuning = C.cast(C.pointer(self._tuning), C.c_void_p)
        self._addr_buf = None
        if addresses is not None:
            stride = max(len(a) for a in addresses)
            buf = b"".join(a.encode().ljust(stride, b"\0") for a in addresses)
            self._addr_buf = C.create_string_buffer(buf, len(buf))
            cfg.addresses = C.cast(self._addr_buf, C.c_char_p)
            cfg.addr_stride = stride
        h = C.c_void_p()
        rc = L.swimsim_create(C.byref(cfg), C.byref(h))
        if rc != 0:
            raise SwimsimError(f"swimsim_create failed: {ERRORS.get(rc, rc)}")
        self.h = h
        self.lo = observer_range[0] if observer_range else 0
        self.nl = (observer_range[1] - observer_range[0]) if observer_range else n
        if comm is not None:
            nranks, rank, uid = comm
            if isinstance(uid, (bytes, bytearray)):
                idb = (C.c_uint8 * len(uid)).from_buffer_copy(uid)
                self._chk(L.swimsim_comm_attach(self.h, nranks, rank, C.cast(idb, C.c_void_p), len(uid)))
            else:                                    # host transport: keep the callbacks alive with the handle
                self._transport = uid
                self._chk(L.swimsim_comm_attach_host(self.h, nranks, rank, C.byref(uid.c_struct())))
        if init == "converged":
            self._chk(L.swimsim_init_converged(self.h))
        elif init == "self":
            self._chk(L.swimsim_init_self_only(self.h))

    def _chk(self, rc):
        if rc < 0:
            msg = load_library().swimsim_last_error(self.h).decode()
            raise SwimsimError(f"{ERRORS.get(rc, rc)}: {msg}")
        return rc

    def close(self):
        if getattr(self, "h", None):
            load_library().swimsim_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    # ---- driving -------------------------------------------------------------------------
    def step(self, rounds=1, events=()):
        ev = _events(events)
        self._chk(load_library().swimsim_step(self.h, rounds, ev, len(events)))
        self._emit()

    def _emit(self):
        """deliver MemberlistChangesAppliedEvent to the listeners of watched observers (node.emit, node.go:266-270):
        one event per Update that applied something, in the node's Update order (the per-Update stream). Old/New
        checksums are per drain: the first event of a drain carries the checksum at the previous drain, every event
        the current one as NewChecksum (and as OldChecksum after the first)"""
        for o, ls in self._listeners.items():
            if not ls:
                continue
            events, old, new, nm = self.applied_events(o)
            for i, changes in enumerate(events):
                evt = MemberlistChangesAppliedEvent(self._wire_changes(changes), old if i == 0 else new, new, nm)
                for l in ls:
                    (l.HandleEvent if hasattr(l, "HandleEvent") else l)(evt)

    @staticmethod
    def _wire_changes(changes):
        from .wire import Change
        return [Change(address_of(s) if s >= 0 else "", si, address_of(m), inc, STATUS_NAMES[st], False)
                for (m, st, inc, s, si) in changes]

    # ---- applied-change stream (MemberlistChangesAppliedEvent, swim/events.go:56-61) ----------
    def watch(self, o, on=True):
        """on: True = the coalesced drain (applied_changes); "events" = also the per-Update stream (applied_events);
        False = off"""
        self._chk(load_library().swimsim_watch(self.h, o, 2 if on == "events" else int(bool(on))))

    def applied_events(self, o):
        """drain the per-Update stream of observer o (watch(o, "events")): ([[(member, status, inc, source,
        source_inc)] per applying Update, in the node's Update order; changes in member order], old checksum,
        new checksum, NumMembers), the checksums and NumMembers per drain"""
        cap = 4 * self.n + 4096
        m = np.empty(cap, np.int32); st = np.empty(cap, np.int32); inc = np.empty(cap, np.int64)
        s = np.empty(cap, np.int32); si = np.empty(cap, np.int64); ev = np.empty(cap, np.uint32)
        n, ne, old, new, nm = C.c_size_t(), C.c_size_t(), C.c_uint32(), C.c_uint32(), C.c_int32()
        self._chk(load_library().swimsim_applied_events(self.h, o, m.ctypes.data, st.ctypes.data, inc.ctypes.data,
                                                        s.ctypes.data, si.ctypes.data, ev.ctypes.data, cap, C.byref(n),
                                                        C.byref(ne), C.byref(old), C.byref(new), C.byref(nm)))
        events = [[] for _ in range(ne.value)]
        for i in range(n.value):
            events[int(ev[i])].append((int(m[i]), int(st[i]), int(inc[i]), int(s[i]), int(si[i])))
        return events, old.value, new.value, nm.value

    def applied_changes(self, o):
        """drain watched observer o: ([(member, status, inc, source, source_inc)] in member order, old checksum,
        new checksum, NumMembers) since the previous drain"""
        cap = self.n
        m = np.empty(cap, np.int32); st = np.empty(cap, np.int32); inc = np.empty(cap, np.int64)
        s = np.empty(cap, np.int32); si = np.empty(cap, np.int64)
        n, old, new, nm = C.c_size_t(), C.c_uint32(), C.c_uint32(), C.c_int32()
        self._chk(load_library().swimsim_applied_changes(self.h, o, m.ctypes.data, st.ctypes.data, inc.ctypes.data,
                                                         s.ctypes.data, si.ctypes.data, cap, C.byref(n), C.byref(old),
                                                         C.byref(new), C.byref(nm)))
        k = n.value
        return ([(int(m[i]), int(st[i]), int(inc[i]), int(s[i]), int(si[i])) for i in range(k)], old.value, new.value,
                nm.value)

    def register_listener(self, o, listener):
        """NodeInterface.RegisterListener (node.go:146) for simulated node o"""
        if o not in self._listeners:
            self.watch(o, "events")
            self._listeners[o] = []
        self._listeners[o].append(listener)

    def memory(self):
        """device memory of the handle (swimsim_memory): bytes per structure, snapshot slots, lazy-C_o fallbacks"""
        m = MemoryC()
        self._chk(load_library().swimsim_memory(self.h, C.byref(m)))
        return {f: getattr(m, f) for f, _ in MemoryC._fields_}

    def protocol_stats(self):
        """NodeInterface.ProtocolStats (stats.go:81-104): Timing over protocol rounds (ns), ProtocolRate (ns),
        ClientRate / ServerRate / TotalRate per node per simulated second"""
        p = ProtocolStatsC()
        self._chk(load_library().swimsim_protocol_stats(self.h, C.byref(p)))
        timing = {k: getattr(p, k) for k in ("count", "min_ns", "max_ns", "sum_ns", "mean_ns", "variance", "stddev_ns",
                                             "median_ns", "p75_ns", "p95_ns", "p99_ns", "p999_ns")}
        return {"timing": timing, "protocol_rate_ns": p.protocol_rate_ns, "client_rate": p.client_rate,
                "server_rate": p.server_rate, "total_rate": p.total_rate}

    def run(self, rounds, events=()):
        self.step(rounds, events)

    def heal(self, o):
        out = np.empty(self.n, np.int32)
        n = C.c_size_t()
        self._chk(load_library().swimsim_heal(self.h, o, out.ctypes.data, self.n, C.byref(n)))
        return [int(x) for x in out[: min(n.value, self.n)]]

    @property
    def round(self):
        return load_library().swimsim_round(self.h)

    # ---- setup -----------------------------------------------------------------------------
    def set_member(self, o, m, status, inc):
        self._chk(load_library().swimsim_set_member(self.h, o, m, status, inc))

    def set_row(self, o, status, inc):
        """raw write of observer o's whole row (swimsim_set_row); UNKNOWN marks a non-member"""
        st = np.ascontiguousarray(status, dtype=np.uint8)
        ic = np.ascontiguousarray(inc, dtype=np.int64)
        if st.shape != (self.n,) or ic.shape != (self.n,):
            raise ValueError(f"set_row needs two length-{self.n} columns")
        self._chk(load_library().swimsim_set_row(self.h, o, st.ctypes.data, ic.ctypes.data))

    def make_change(self, o, m, inc, status):
        return self._chk(load_library().swimsim_make_change(self.h, o, m, inc, status))

    def clear_changes(self, o):
        self._chk(load_library().swimsim_clear_changes(self.h, o))

    def add_join_list(self, o, member, status, inc, source=None, source_inc=None):
        """memberlist.AddJoinList (memberlist.go:398-406) on observer o in one device launch
        (swimsim_add_join_list): Update of the list, then ClearChange of every applied change except o's own.
        Columns as swimsim.wire.changes_to_arrays makes them; returns the number of applied changes."""
        cols = [np.ascontiguousarray(member, np.int32), np.ascontiguousarray(status, np.int32),
                np.ascontiguousarray(inc, np.int64)]
        n = len(cols[0])
        if any(len(c) != n for c in cols):
            raise ValueError("add_join_list: columns of different lengths")
        src = None if source is None else np.ascontiguousarray(source, np.int32)
        sinc = None if source_inc is None else np.ascontiguousarray(source_inc, np.int64)
        ptr = lambda a: None if a is None else a.ctypes.data
        applied = C.c_uint32(0)
        self._chk(load_library().swimsim_add_join_list(self.h, o, ptr(cols[0]), ptr(cols[1]), ptr(cols[2]), ptr(src),
                                                       ptr(sinc), n, C.byref(applied)))
        return int(applied.value)

    def set_live(self, m, live):
        self._chk(load_library().swimsim_set_live(self.h, m, int(live)))

    def set_partition(self, m, label):
        self._chk(load_library().swimsim_set_partition(self.h, m, label))

    def set_round(self, r):
        self._chk(load_library().swimsim_set_round(self.h, r))

    # ---- read-back -------------------------------------------------------------------------
    def checksums(self):
        out = np.empty(self.nl, np.uint32)
        self._chk(load_library().swimsim_checksums(self.h, out.ctypes.data))
        return out

    def checksum(self, o):
        return int(self.checksums()[o - self.lo])

    def row(self, o):
        st = np.empty(self.n, np.uint8)
        inc = np.empty(self.n, np.int64)
        self._chk(load_library().swimsim_row(self.h, o, st.ctypes.data, inc.ctypes.data))
        return st, inc

    def rows(self):
        st = np.empty((self.nl, self.n), np.uint8)
        inc = np.empty((self.nl, self.n), np.int64)
        for i in range(self.nl):
            st[i], inc[i] = self.row(self.lo + i)
        return st, inc

    def member(self, o, m):
        st, inc = self.row(o)
        return int(st[m]), int(inc[m])

    def node_stats(self, o):
        p, mx, ch, mem = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int32()
        self._chk(load_library().swimsim_node_stats(self.h, o, C.byref(p), C.byref(mx), C.byref(ch), C.byref(mem)))
        return {"pingable": p.value, "maxp": mx.value, "changes": ch.value, "members": mem.value}

    def changes(self, o):
        cap = self.n
        m = np.empty(cap, np.int32); p = np.empty(cap, np.int32); s = np.empty(cap, np.int32)
        si = np.empty(cap, np.int64)
        n = C.c_size_t()
        self._chk(load_library().swimsim_changes(self.h, o, m.ctypes.data, p.ctypes.data, s.ctypes.data, si.ctypes.data,
                                                 cap, C.byref(n)))
        return {int(m[i]): (int(p[i]), int(s[i]), int(si[i])) for i in range(n.value)}

    def timers(self, o):
        cap = self.n
        m = np.empty(cap, np.int32); st = np.empty(cap, np.int32); f = np.empty(cap, np.int32)
        dl = np.empty(cap, np.int64); sj = np.empty(cap, np.int64)
        n = C.c_size_t()
        self._chk(load_library().swimsim_timers(self.h, o, m.ctypes.data, st.ctypes.data, f.ctypes.data,
                                                dl.ctypes.data, sj.ctypes.data, cap, C.byref(n)))
        return {int(m[i]): (int(st[i]), int(f[i]), int(dl[i]), int(sj[i])) for i in range(n.value)}

    def iter_state(self, o):
        idx, ep = C.c_int64(), C.c_uint32()
        self._chk(load_library().swimsim_iter_state(self.h, o, C.byref(idx), C.byref(ep)))
        return idx.value, ep.value

    def last_targets(self):
        out = np.empty(self.nl, np.int32)
        self._chk(load_library().swimsim_last_targets(self.h, out.ctypes.data))
        return out

    def counters(self):
        out = np.zeros(len(COUNTER_NAMES), np.uint64)
        self._chk(load_library().swimsim_counters(self.h, out.ctypes.data))
        return dict(zip(COUNTER_NAMES, (int(x) for x in out)))

    def digest(self):
        a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self._chk(load_library().swimsim_digest(self.h, C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value

    def converged(self):
        v = C.c_int32()
        self._chk(load_library().swimsim_converged(self.h, C.byref(v)))
        return bool(v.value)

    def count_reachable(self, o):
        v = C.c_uint32()
        self._chk(load_library().swimsim_count_reachable(self.h, o, C.byref(v)))
        return v.value

    def enable_timing(self, on=True):
        self._chk(load_library().swimsim_enable_timing(self.h, int(on)))

    def kernel_times(self):
        cap = 32
        names = (C.c_char_p * cap)()
        avg = np.zeros(cap, np.float64)
        n_l = np.zeros(cap, np.uint64)
        byt = np.zeros(cap, np.float64)
        n = C.c_size_t()
        self._chk(load_library().swimsim_kernel_times(self.h, names, avg.ctypes.data, n_l.ctypes.data, byt.ctypes.data,
                                                      cap, C.byref(n)))
        return {names[i].decode(): {"avg_ms": float(avg[i]), "launches": int(n_l[i]), "alg_bytes": float(byt[i])}
                for i in range(n.value)}

    def kernel_units(self):
        """unit counts behind kernel_times' bytes since enable_timing: rows hashed per checksum kernel, changes
        processed / applied per merge kernel, records issued, ..."""
        cap = 32
        names = (C.c_char_p * cap)()
        vals = np.zeros(cap, np.float64)
        n = C.c_size_t()
        self._chk(load_library().swimsim_kernel_units(self.h, names, vals.ctypes.data, cap, C.byref(n)))
        return {names[i].decode(): float(vals[i]) for i in range(n.value)}

    def profile_mark(self, mark_id):
        """one k_profile_mark dispatch: rocprofv3 counter passes are cut between two marks (tools/pmc_summary.py)"""
        self._chk(load_library().swimsim_profile_mark(self.h, mark_id))

    def shard_info(self):
        g, r, lo, hi = C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_uint32()
        xb, xc = C.c_uint64(), C.c_uint64()
        self._chk(load_library().swimsim_shard_info(self.h, C.byref(g), C.byref(r), C.byref(lo), C.byref(hi),
                                                    C.byref(xb), C.byref(xc)))
        xs = C.c_uint64()
        self._chk(load_library().swimsim_exchange_syncs(self.h, C.byref(xs)))
        return {"shards": g.value, "rank": r.value, "lo": lo.value, "hi": hi.value, "exchanged_bytes": xb.value,
                "exchanges": xc.value, "exchange_host_syncs": xs.value}

    # (rows the reference-row path left to the production kernels, by reason; the diagnostics library's round-3 path
    # reports its own reasons in the same slots: entry batch in "record_cap", jump slots and window misses in 5 and 6)
    CSD_REASONS = ("short", "entry_cap", "window_plan", "record_cap", "exception_slots", "reserved5", "reserved6",
                   "declined_launches")

    def checksum_path_stats(self):
        dl, fb = C.c_uint64(), C.c_uint64()
        rs = np.zeros(len(self.CSD_REASONS), np.uint64)
        self._chk(load_library().swimsim_checksum_path_stats(self.h, C.byref(dl), C.byref(fb),
                                                             rs.ctypes.data_as(_U64P)))
        return {"delta_launches": dl.value, "fallback_rows": fb.value,
                "reasons": {k: int(v) for k, v in zip(self.CSD_REASONS, rs)}}

    def debug_cs_stream(self, o, nwords):
        """the words of every 20-byte block the checksum kernel hashes for observer o (diagnostics)"""
        out = np.zeros(nwords, dtype=np.uint32)
        self._chk(load_library().swimsim_debug_cs_stream(self.h, o - self.lo, out.ctypes.data, nwords))
        return out

    def bench_checksum(self, nrows, mode=0, reps=3):
        ms = C.c_double()
        self._chk(load_library().swimsim_bench_checksum(self.h, nrows, mode, reps, C.byref(ms)))
        return ms.value

    def node(self, o):
        return Node(self, o)

    def debug_exchange(self, segments):
        """diagnostics (transport conformance): send segments[p] (bytes) to shard p through this handle's shard
        transport, as a round's parcel exchange moves them; returns the segments received from each shard.
        Collective: every shard calls it."""
        G = len(segments)
        sb = np.array([len(x) for x in segments], np.uint64)
        send = np.frombuffer(b"".join(segments) or b"\0", np.uint8).copy()
        cap = 1 << 22
        recv = np.empty(cap, np.uint8)
        rb = np.zeros(G, np.uint64)
        self._chk(load_library().swimsim_debug_exchange(self.h, send.ctypes.data, sb.ctypes.data, recv.ctypes.data, cap,
                                                        rb.ctypes.data))
        out, at = [], 0
        for k in rb.tolist():
            out.append(recv[at:at + int(k)].tobytes())
            at += int(k)
        return out


@dataclass
class ShardedCluster:
    """One cluster whose observer rows are split over `nshards` shards of this process (threads, one
    per shard, exchanging cross-shard messages by device copies; devices[i] places shard i on another
    GPU). Results are bit-identical to an unsharded Cluster; read-back merges the shards."""

    def __init__(self, n, nshards, *, devices=None, init="converged", **kw):
        L = load_library()
        self.n, self.nshards = n, nshards
        cfg = make_config(n, **{k: v for k, v in kw.items() if k != "addresses"})
        arr = (C.c_void_p * nshards)()
        devs = (C.c_int32 * nshards)(*devices) if devices else None
        rc = L.swimsim_group_create(C.byref(cfg), nshards, C.cast(devs, C.c_void_p) if devs else None, arr)
        if rc != 0:
            raise SwimsimError(f"swimsim_group_create failed: {ERRORS.get(rc, rc)}")
        self._arr = arr
        self.live = np.ones(n, bool)
        self.shards = []
        for i in range(nshards):
            lo, hi = shard_range(n, nshards, i)
            self.shards.append(Cluster._adopt(C.c_void_p(arr[i]), n, lo, hi - lo, kw.get("t0_ms", T0_MS),
                                              kw.get("period_ms", 200)))
        for c in self.shards:
            if init == "converged":
                c._chk(L.swimsim_init_converged(c.h))
            elif init == "self":
                c._chk(L.swimsim_init_self_only(c.h))

    def owner(self, o):
        return next(c for c in self.shards if c.lo <= o < c.lo + c.nl)

    def close(self):
        for c in self.shards:
            c.close()

    def step(self, rounds=1, events=()):
        r0 = self.round
        for (r, k, a, b) in events:                      # liveness mirror for converged()
            if r0 <= r < r0 + rounds and k in (EV_KILL, EV_REVIVE):
                self.live[a] = k == EV_REVIVE
        ev = _events(events)
        rc = load_library().swimsim_group_step(self._arr, self.nshards, rounds, ev, len(events))
        if rc < 0:
            msgs = "; ".join(load_library().swimsim_last_error(c.h).decode() for c in self.shards)
            raise SwimsimError(f"{ERRORS.get(rc, rc)}: {msgs}")
        for c in self.shards:
            c._emit()

    def watch(self, o, on=True):
        self.owner(o).watch(o, on)

    def applied_changes(self, o):
        return self.owner(o).applied_changes(o)

    def applied_events(self, o):
        return self.owner(o).applied_events(o)

    def register_listener(self, o, listener):
        self.owner(o).register_listener(o, listener)

    def protocol_stats(self):
        return self.shards[0].protocol_stats()

    @property
    def round(self):
        return self.shards[0].round

    @property
    def t0_ms(self):
        return self.shards[0].t0_ms

    @property
    def period_ms(self):
        return self.shards[0].period_ms

    def checksum(self, o):
        return self.owner(o).checksum(o)

    def member(self, o, m):
        return self.owner(o).member(o, m)

    def checksums(self):
        return np.concatenate([c.checksums() for c in self.shards])

    def last_targets(self):
        return np.concatenate([c.last_targets() for c in self.shards])

    def digest(self):
        ds = [c.digest() for c in self.shards]
        return tuple(sum(d[i] for d in ds) % (1 << 64) for i in range(3))

    def counters(self):
        cs = [c.counters() for c in self.shards]
        out = {k: sum(c[k] for c in cs) for k in COUNTER_NAMES}
        out["rounds"] = cs[0]["rounds"]
        return out

    def rows(self):
        parts = [c.rows() for c in self.shards]
        return np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts])

    def row(self, o):
        return self.owner(o).row(o)

    def changes(self, o):
        return self.owner(o).changes(o)

    def timers(self, o):
        return self.owner(o).timers(o)

    def node_stats(self, o):
        return self.owner(o).node_stats(o)

    def iter_state(self, o):
        return self.owner(o).iter_state(o)

    def converged(self):
        """test_utils.go:188-198 over all shards: no live node has changes, all live checksums equal"""
        cs = self.checksums()
        live = [o for o in range(self.n) if self.live[o]]
        return all(c.converged() for c in self.shards) and len(set(int(cs[o]) for o in live)) <= 1

    def kernel_units(self):
        """unit counts behind kernel_times' bytes since enable_timing, summed over the shards: rows hashed per
        checksum kernel, changes processed / applied per merge kernel, records issued, ..."""
        tot = {}
        for c in self.shards:
            for k, v in c.kernel_units().items():
                tot[k] = tot.get(k, 0.0) + v
        return tot

    def profile_mark(self, mark_id):
        """one k_profile_mark dispatch per shard (rocprofv3 counter passes are cut between marks)"""
        for c in self.shards:
            c.profile_mark(mark_id)

    def shard_info(self):
        return [c.shard_info() for c in self.shards]

    # setup calls act on the owning shard (row writes) or on every shard (topology)
    def set_member(self, o, m, status, inc):
        self.owner(o).set_member(o, m, status, inc)

    def set_row(self, o, status, inc):
        self.owner(o).set_row(o, status, inc)

    def make_change(self, o, m, inc, status):
        return self.owner(o).make_change(o, m, inc, status)

    def clear_changes(self, o):
        self.owner(o).clear_changes(o)

    def add_join_list(self, o, *cols, **kw):
        return self.owner(o).add_join_list(o, *cols, **kw)

    def set_live(self, m, live):
        self.live[m] = bool(live)
        for c in self.shards:
            c.set_live(m, live)

    def set_partition(self, m, label):
        for c in self.shards:
            c.set_partition(m, label)


class MemberView:
    address: str
    status: str
    incarnation: int


def address_of(m: int) -> str:
    return "10.%03d.%03d.%03d:7000" % ((m >> 16) & 255, (m >> 8) & 255, m & 255)


class Memberlist:
    """swim.memberlist view of one observer (swim/memberlist.go)."""

    def __init__(self, cluster: Cluster, o: int):
        self.c, self.o = cluster, o

    def Checksum(self):                                   # memberlist.go:73-80
        return self.c.checksum(self.o)

    def Member(self, m):                                  # memberlist.go:131-138
        st, inc = self.c.member(self.o, m)
        if st == UNKNOWN:
            return None, False
        return MemberView(address_of(m), STATUS_NAMES[st], inc), True

    def NumMembers(self):                                 # memberlist.go:174-179
        return self.c.node_stats(self.o)["members"]

    def NumPingableMembers(self):                         # memberlist.go:188-198
        return self.c.node_stats(self.o)["pingable"]

    def MakeChange(self, m, incarnation, status):         # memberlist.go:282-307
        return self.c.make_change(self.o, m, incarnation, status)

    def MakeAlive(self, m, inc):
        return self.MakeChange(m, inc, ALIVE)

    def MakeSuspect(self, m, inc):
        return self.MakeChange(m, inc, SUSPECT)

    def MakeFaulty(self, m, inc):
        return self.MakeChange(m, inc, FAULTY)

    def MakeLeave(self, m, inc):
        return self.MakeChange(m, inc, LEAVE)

    def MakeTombstone(self, m, inc):
        return self.MakeChange(m, inc, TOMBSTONE)

    def GetReachableMembers(self):                        # memberlist.go:471-483
        st, _ = self.c.row(self.o)
        return [address_of(m) for m in np.nonzero(st <= SUSPECT)[0]]

    def CountReachableMembers(self):                      # memberlist.go:485-497
        return self.c.count_reachable(self.o)


class Disseminator:
    """swim.disseminator view of one observer (swim/disseminator.go)."""

    def __init__(self, cluster: Cluster, o: int):
        self.c, self.o = cluster, o

    def ChangesCount(self):                               # disseminator.go:239-244
        return self.c.node_stats(self.o)["changes"]

    def HasChanges(self):                                 # disseminator.go:100-105
        return self.ChangesCount() > 0

    def ChangesByAddress(self, m):                        # disseminator.go:229-237
        ch = self.c.changes(self.o)
        return (ch[m], True) if m in ch else (None, False)

    def MaxP(self):                                       # disseminator.go:49
        return self.c.node_stats(self.o)["maxp"]

    def ClearChanges(self):                               # disseminator.go:217-221
        self.c.clear_changes(self.o)


class Node:
    """swim.NodeInterface of simulated member o (swim/node.go:137-147)."""

    def __init__(self, cluster: Cluster, o: int):
        self.c, self.o = cluster, o
        self.memberlist = Memberlist(cluster, o)
        self.disseminator = Disseminator(cluster, o)

    def Address(self):
        return address_of(self.o)

    def GetChecksum(self):
        return self.memberlist.Checksum()

    def CountReachableMembers(self):
        return self.memberlist.CountReachableMembers()

    def GetReachableMembers(self):
        return self.memberlist.GetReachableMembers()

    def Incarnation(self):                                # node.go:256-264
        return self.c.member(self.o, self.o)[1]

    def MemberStats(self):                                # stats.go:41-52
        st, inc = self.c.row(self.o)
        members = [MemberView(address_of(m), STATUS_NAMES[int(st[m])], int(inc[m]))
                   for m in range(self.c.n) if st[m] != UNKNOWN]
        return {"checksum": self.GetChecksum(), "members": members}

    def HasChanges(self):
        return self.disseminator.HasChanges()

    def RegisterListener(self, listener):                 # node.go:146; events.EventListener.HandleEvent
        self.c.register_listener(self.o, listener)

    def ProtocolStats(self):                              # stats.go:81-104
        return self.c.protocol_stats()
