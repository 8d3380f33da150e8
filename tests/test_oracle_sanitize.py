"""The CPU oracle under AddressSanitizer / UndefinedBehaviorSanitizer: `make -C oracle sanitize`
builds oracle/selftest.c with the oracle sources and runs it. The driver takes every workload kind (cascade
with eviction and reap, churn with reincarnations, partition and heal, self-only start with full syncs), every
read-back, the applied-change stream, AddJoinList and the hash-ring oracle, and checks that the reference cost
model (checksum string rebuilt and sorted at every applying Update, memberlist.go:106-128) gives the same
checksums and state digests as the static-order one, and that each checksum string hashes to its checksum."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None and shutil.which("cc") is None, reason="no C compiler")
def test_oracle_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "selftest ok" in r.stdout
