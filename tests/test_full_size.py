"""Shard-count independence at full size: the same config-4 run (N = 16,384) split over 1, 2, 4 and 8 observer-row
shards gives identical checksums, state digests and counters. (Per-round parity with the oracle at full size,
and the config-3 row-rebuilt checksum property at 65,536 members: tests/test_parity_at_size.py.)
"""
import pytest

import swimsim
from swimsim import workloads as W

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shards", [2, 4, 8])
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
