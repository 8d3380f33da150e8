"""CPU checks of the drop-in boundary: libswimsim.so loads and exports every include/swimsim.h entry
point; the host-side workload generators agree with the oracle's Philox; no compute runs here."""
import ctypes
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "swimsim.h")
LIB = os.path.join(REPO, "ringpop-go_amd", "swimsim", "libswimsim.so")


def header_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(swimsim_[a-z_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "ringpop-go_amd")], check=True)
    return ctypes.CDLL(LIB)


def test_exports_every_header_symbol(lib):
    names = header_functions()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_header(lib):
    import swimsim
    L = swimsim.load_library(LIB)
    for n in header_functions():
        assert getattr(L, n).restype is not None or n in ()


def test_abi_version(lib):
    lib.swimsim_abi_version.restype = ctypes.c_int
    want = int(re.search(r"#define SWIMSIM_ABI_VERSION (\d+)", open(HEADER).read()).group(1))
    assert lib.swimsim_abi_version() == want


def test_shard_entry_points_reject_bad_arguments_without_touching_device(lib):
    import swimsim
    L = swimsim.load_library(LIB)
    cfg = swimsim.make_config(8)
    out = (ctypes.c_void_p * 4)()
    assert L.swimsim_group_create(ctypes.byref(cfg), 0, None, out) == -1        # no shards
    assert L.swimsim_group_create(ctypes.byref(cfg), 9, None, out) == -1        # more shards than rows
    assert L.swimsim_group_step(None, 2, 1, None, 0) == -1
    assert L.swimsim_comm_attach(None, 2, 0, None, 0) == -1
    assert L.swimsim_shard_info(None, None, None, None, None, None, None) == -1


@pytest.mark.parametrize("n,g", [(1, 1), (5, 4), (16, 3), (65536, 8), (65537, 7)])
def test_canonical_shard_split_covers_all_rows(n, g):
    import swimsim
    ranges = [swimsim.shard_range(n, g, r) for r in range(g)]
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    assert all(hi > lo for lo, hi in ranges)


def test_create_rejects_bad_config_without_touching_device(lib):
    import swimsim
    cfg = swimsim.Config()
    cfg.num_members = 0
    h = ctypes.c_void_p()
    L = swimsim.load_library(LIB)
    assert L.swimsim_create(ctypes.byref(cfg), ctypes.byref(h)) == -1


def test_workload_philox_matches_oracle():
    from oracle_ffi import philox
    from swimsim.workloads import philox4x32_10
    for ctr, key in (((0, 0, 0, 0), 0), ((5, 0, 4, 3), 7), ((0xFFFFFFFF,) * 4, 0xFFFFFFFFFFFFFFFF)):
        assert list(philox4x32_10(*ctr, key)) == philox(list(ctr), [key & 0xFFFFFFFF, key >> 32])


def test_workloads_shapes():
    from swimsim import workloads as W
    w2 = W.config2(n=4096, rounds=5)
    assert sum(1 for e in w2.events if e[0] == 0) == 41
    w3 = W.config3()
    assert len(w3.events) == 655 and len({e[2] for e in w3.events}) == 655
    w4 = W.config4()
    assert sum(1 for e in w4.events if e[1] == W.EV_HEAL) == 2
    w5 = W.config5(n=262144, rounds=40)
    assert sum(1 for e in w5.events if e[0] == 0) == 26214
