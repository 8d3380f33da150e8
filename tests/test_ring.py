"""The consistent-hash ring: hashring.HashRing semantics on the MI355X.

CPU tests pin the oracle (oracle/ring_oracle.c) against the reference's own hashring tests
(hashring/hashring_test.go, cited per test) and against an independent dictionary restatement of
the red-black tree's insert / delete-by-value behaviour, including real Fingerprint32 collisions.
GPU tests compare libswimsim's ring (include/swimring.h) with the oracle, bit-exact: the sorted
points with their owners, the checksum, the server set, Lookup over many keys and LookupN sets.
"""
import ctypes
import os
import random
import re

import numpy as np
import pytest

from oracle_ffi import OracleRing, fingerprint32

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "swimring.h")
LIB = os.path.join(REPO, "ringpop-go_amd", "swimsim", "libswimsim.so")


def gen_addresses(host, lo, hi):   # hashring_test.go:325-331
    return [f"127.0.0.{host}:{3000 + i}" for i in range(lo, hi + 1)]


class DictRing:
    """Independent restatement: the tree as a dict value -> owner, first insert wins, delete by value."""

    def __init__(self, R):
        self.R, self.pts, self.set = R, {}, set()

    def add_remove(self, add, remove):
        changed = False
        for s in add:
            if s in self.set:
                continue
            self.set.add(s)
            changed = True
            for i in range(self.R):
                self.pts.setdefault(fingerprint32(f"{s}{i}".encode()), s)
        for s in remove:
            if s not in self.set:
                continue
            self.set.discard(s)
            changed = True
            for i in range(self.R):
                self.pts.pop(fingerprint32(f"{s}{i}".encode()), None)
        return changed

    def points(self):
        return sorted(self.pts.items())


def random_batches(servers, nbatch, seed):
    rng = random.Random(seed)
    live = set()
    out = []
    for _ in range(nbatch):
        add = rng.sample(servers, rng.randint(1, len(servers) // 3))
        rem = rng.sample(sorted(live), min(len(live), rng.randint(0, len(servers) // 4))) if live else []
        rem += rng.sample(servers, 2)                    # removes of servers that may not be present
        add += add[:2]                                   # duplicate adds inside one call
        out.append((add, rem))
        live |= set(add)
        live -= set(rem)
    return out


# ------------------------------------------------------------------------------------------
# oracle pinned by the reference's hashring tests (CPU)
# ------------------------------------------------------------------------------------------
def test_oracle_add_server_kat():
    """hashring_test.go:55-70: AddServer twice is a no-op the second time; HasServer."""
    r = OracleRing(10)
    assert r.add_remove_servers(["server1"]) and r.add_remove_servers(["server2"])
    assert not r.add_remove_servers(["server1"])
    assert r.server_count() == 2


def test_oracle_remove_server_kat():
    """hashring_test.go:72-95: removing absent servers changes nothing."""
    r = OracleRing(10)
    r.add_remove_servers(["server1", "server2"])
    assert r.add_remove_servers([], ["server1"])
    assert not r.add_remove_servers([], ["server3"])
    assert not r.add_remove_servers([], ["server1"])
    assert r.server_count() == 1


def test_oracle_checksum_changes_kat():
    """hashring_test.go:97-109 (and the zero checksum of a new ring, hashring.go:76-88)."""
    r = OracleRing(10)
    c0 = r.checksum()
    assert c0 == 0
    r.add_remove_servers(["server1"])
    r.add_remove_servers(["server2"])
    c1 = r.checksum()
    assert c1 != c0
    assert c1 == fingerprint32(b"server1;server2")
    r.add_remove_servers([], ["server1"])
    assert r.checksum() != c1 and r.checksum() == fingerprint32(b"server2")


def test_oracle_add_remove_servers_kat():
    """hashring_test.go:143-161: adds apply before removes; the checksum changes."""
    r = OracleRing(10)
    r.add_remove_servers(["server3", "server4"])
    assert r.server_count() == 2
    old = r.checksum()
    assert r.add_remove_servers(["server1", "server2"], ["server3", "server4"])
    assert r.server_count() == 2 and r.checksum() != old


def test_oracle_lookup_kat():
    """hashring_test.go:163-178: empty ring after removing both servers."""
    r = OracleRing(10)
    r.add_remove_servers(["server1", "server2"])
    assert r.lookup("key")[1]
    r.add_remove_servers([], ["server1", "server2"])
    assert r.lookup("key") == ("", False)


def test_oracle_lookup_distribution_kat():
    """hashring_test.go:180-199: keys "0".."39" land on 40 distinct servers of 1000 x 5 replicas."""
    r = OracleRing(5)
    r.add_remove_servers(gen_addresses(1, 1, 1000))
    assert len({r.lookup(str(i))[0] for i in range(40)}) == 40


def test_oracle_lookup_n_no_gaps_kat():
    """hashring_test.go:203-257: LookupN's servers are a contiguous run of the (1-replica) ring."""
    r = OracleRing(1)
    addrs = gen_addresses(1, 1, 100)
    r.add_remove_servers(addrs)
    got = set(r.lookup_n("key with small hash", 20))
    hs = {a: fingerprint32(f"{a}0".encode()) for a in addrs}
    lo, hi = min(hs[s] for s in got), max(hs[s] for s in got)
    assert all(not (lo <= hs[a] <= hi) for a in addrs if a not in got)


def test_oracle_lookup_n_overflow_and_loop_around_kat():
    """hashring_test.go:259-285"""
    r = OracleRing(10)
    r.add_remove_servers(gen_addresses(1, 1, 10))
    assert len(r.lookup_n("a random key", 20)) == 10
    r1 = OracleRing(1)
    r1.add_remove_servers(gen_addresses(1, 1, 10))
    first_in_tree = r1.points()[0][1]
    first = r1.lookup("a random key")[0]
    assert first != first_in_tree
    assert first in r1.lookup_n("a random key", 9)


def test_oracle_lookup_n_kat():
    """hashring_test.go:287-323"""
    r = OracleRing(10)
    assert r.lookup_n("nil", 5) == []
    addrs = gen_addresses(1, 1, 10)
    r.add_remove_servers(addrs)
    assert len(set(r.lookup_n("key", 5))) == 5
    assert len(set(r.lookup_n("another key", 100))) == 10
    r.add_remove_servers([], [addrs[0]])
    assert len(set(r.lookup_n("yet another key", 10))) == 9


def test_oracle_matches_dict_restatement_with_collisions():
    """first-insert-wins and delete-by-value with real Fingerprint32 collisions"""
    servers = gen_addresses(2, 1, 3000)
    o, d = OracleRing(100), DictRing(100)
    for add, rem in random_batches(servers, 6, seed=5):
        assert o.add_remove_servers(add, rem) == d.add_remove(add, rem)
        assert o.points() == d.points()
    # the batches above must have exercised collisions for this test to mean anything
    allh = [fingerprint32(f"{s}{i}".encode()) for s in servers for i in range(100)]
    assert len(allh) - len(set(allh)) > 0


def test_ring_abi_exports_every_header_symbol():
    names = sorted(set(re.findall(r"\b(swimring_[a-z0-9_]+)\s*\(", open(HEADER).read())))
    assert len(names) >= 12
    lib = ctypes.CDLL(LIB)
    assert [n for n in names if not hasattr(lib, n)] == []


# ------------------------------------------------------------------------------------------
# MI355X ring vs oracle (GPU)
# ------------------------------------------------------------------------------------------
def _gpu_ring(R):
    from swimsim.ring import HashRing
    return HashRing(R, device=0)


def _same(g, o):
    hs, ow = g.points()
    op = o.points()
    assert len(hs) == len(op)
    assert [int(h) for h in hs] == [h for h, _ in op]
    assert [g.name(i) for i in ow] == [s for _, s in op]
    assert g.checksum() == o.checksum()
    assert g.server_count() == o.server_count()


@pytest.mark.gpu
def test_gpu_fingerprint32_all_length_paths():
    g = _gpu_ring(1)
    rng = random.Random(3)
    strs = [bytes(rng.randrange(256) for _ in range(n)) for n in list(range(0, 101)) * 3]
    strs += [b"server1;server2", b"10.000.000.001:70000", b"a random key"]
    got = g.fingerprint32(strs)
    assert [int(x) for x in got] == [fingerprint32(s) for s in strs]


@pytest.mark.gpu
def test_gpu_ring_reference_scenarios():
    """hashring_test.go:55-323 on the device ring"""
    g, o = _gpu_ring(10), OracleRing(10)
    assert g.checksum() == 0
    for add, rem in ([["server1"], []], [["server2"], []], [["server1"], []], [[], ["server3"]],
                     [["server3", "server4"], []], [["server1", "server2"], ["server3", "server4"]]):
        assert g.add_remove_servers(add, rem) == o.add_remove_servers(add, rem)
        _same(g, o)
    assert g.lookup("key") == o.lookup("key")
    g.add_remove_servers([], ["server1", "server2"])
    assert g.lookup("key") == ("", False)
    assert g.lookup_n("nil", 5) == []
    addrs = gen_addresses(1, 1, 10)
    g.add_remove_servers(addrs)
    o.add_remove_servers([], ["server1", "server2"])
    o.add_remove_servers(addrs)
    _same(g, o)
    for key, n in (("key", 5), ("another key", 100), ("a random key", 9), ("x", 1)):
        assert set(g.lookup_n(key, n)) == set(o.lookup_n(key, n))


@pytest.mark.gpu
def test_gpu_ring_random_batches_with_collisions():
    servers = gen_addresses(3, 1, 8000)
    g, o = _gpu_ring(100), OracleRing(100)
    for add, rem in random_batches(servers, 5, seed=11):
        assert g.add_remove_servers(add, rem) == o.add_remove_servers(add, rem)
        _same(g, o)
        keys = [f"key-{k}" for k in range(5000)] + ["", "a", "abcd", "x" * 40]
        ids = g.lookup_ids(keys)
        assert [g.name(i) if i >= 0 else "" for i in ids] == [o.lookup(k)[0] for k in keys]
        for k, n in (("k1", 3), ("k2", 17), ("", 50)):
            assert set(g.lookup_n(k, n)) == set(o.lookup_n(k, n))


@pytest.mark.gpu
def test_gpu_ring_from_engine_rows():
    """Ringpop.handleChanges (ringpop.go:550-563) fed from an observer's row after the cascade"""
    import swimsim
    from swimsim import workloads as W
    wl = W.config3(n=512, rounds=40, kill_round=2)
    eng = swimsim.Cluster(wl.n)
    eng.step(wl.rounds, wl.events)
    st, _ = eng.row(0)
    g, o = _gpu_ring(100), OracleRing(100)
    addr = swimsim.address_of
    assert g.add_remove_servers([addr(m) for m in range(wl.n)]) == o.add_remove_servers([addr(m) for m in range(wl.n)])
    g.sync_from_row(st, addr)
    want = (np.asarray(st) == swimsim.ALIVE) | (np.asarray(st) == swimsim.SUSPECT)
    o.add_remove_servers([], [addr(m) for m in np.nonzero(~want)[0]])
    _same(g, o)
    assert g.server_count() == int(want.sum()) < wl.n


@pytest.mark.gpu
def test_gpu_lookup_n_near_server_count_on_a_large_ring():
    """LookupN with n = server count - 1 walks nearly the whole ring: one bit test per point (a seen-bitmap over
    server ids), not a scan of the owners found so far"""
    import time
    servers = gen_addresses(5, 1, 8192)
    g, o = _gpu_ring(100), OracleRing(100)
    assert g.add_remove_servers(servers) == o.add_remove_servers(servers)
    t0 = time.perf_counter()
    got = g.lookup_n("a random key", len(servers) - 1)
    dt = time.perf_counter() - t0
    assert len(got) == len(set(got)) == len(servers) - 1
    assert set(got) == set(o.lookup_n("a random key", len(servers) - 1))
    assert dt < 5.0


@pytest.mark.gpu
def test_gpu_add_remove_bad_name_leaves_the_ring_unchanged():
    """a batch with an over-long name fails before the server set changes (no half-applied batch)"""
    g, o = _gpu_ring(10), OracleRing(10)
    g.add_remove_servers(["server1", "server2"])
    o.add_remove_servers(["server1", "server2"])
    cs = g.checksum()
    with pytest.raises(Exception):
        g.add_remove_servers(["server3", "x" * 300, "server4"])
    assert g.checksum() == cs and g.server_count() == 2
    assert not g.has_server("server3")
    assert g.add_remove_servers(["server3"]) and o.add_remove_servers(["server3"])
    _same(g, o)
