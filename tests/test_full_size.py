"""Parity at BASELINE.json's full sizes through properties that do not need the oracle to run the
whole protocol (it would take minutes at N = 65,536):

* checksum exactness: for sampled observers, the engine's checksum equals Fingerprint32 of the
  reference's checksum string (memberlist.go:106-128) rebuilt on the host from the engine's own
  row. This covers the wide (64-row) and narrow (16-row) FarmHash kernels, the dedup copies and the
  side-stream checksums at full size;
* shard-count independence: the same config-4 (N = 16,384) and config-3 runs split over 1, 2 and 4
  observer-row shards give identical checksums, state digests and counters;
* protocol invariants: each live member pings once per round; the killed members are suspect or
  faulty in the rows of live observers that know about them.
"""
import numpy as np
import pytest

import swimsim
from swimsim import workloads as W
from oracle_ffi import fingerprint32

pytestmark = pytest.mark.gpu

STATUS = ["alive", "suspect", "faulty", "leave"]


def checksum_from_row(st, inc):
    parts = []
    for m in np.nonzero(st < 4)[0]:
        parts.append(f"{swimsim.address_of(int(m))}{STATUS[st[m]]}{int(inc[m])};")
    return fingerprint32("".join(parts).encode())


def test_config3_full_size_checksums_and_invariants():
    n = 65536
    wl = W.config3(n=n, rounds=24, kill_round=2)
    eng = swimsim.Cluster(n)
    killed = sorted({e[2] for e in wl.events})
    eng.step(wl.rounds, wl.events)                    # one call: side-stream checksums overlap rounds
    cs = eng.checksums()
    live = [o for o in (0, 1, 4097, 32768, 65535) if o not in killed]
    for o in live + killed[:2]:
        st, inc = eng.row(o)
        assert checksum_from_row(st, inc) == int(cs[o]), f"observer {o}"
    c = eng.counters()
    assert c["pings"] == (n - 0) * 2 + (n - len(killed)) * (wl.rounds - 2)
    assert c["suspect_decl"] > 0 and c["applied"] > 0
    st0, _ = eng.row(0)
    ks = st0[killed]
    assert ((ks == swimsim.SUSPECT) | (ks == swimsim.FAULTY) | (ks == swimsim.ALIVE)).all()
    assert (ks != swimsim.ALIVE).mean() > 0.5         # the suspect wave reached observer 0


@pytest.mark.parametrize("shards", [2, 4])
def test_config4_full_size_shard_count_independence(shards):
    wl = W.config4(n=16384, rounds=70, split_until=30, heals=(30, 45))
    one = swimsim.Cluster(wl.n)
    one.step(wl.rounds, wl.events)
    cs1, d1, c1 = one.checksums(), one.digest(), one.counters()
    one.close()
    many = swimsim.ShardedCluster(wl.n, shards)
    many.step(wl.rounds, wl.events)
    assert (many.checksums() == cs1).all()
    assert many.digest() == d1
    assert many.counters() == c1
    assert c1["heal_attempts"] > 0
