"""Diagnostic: how far the rows of a cascade round are from one reference row (the column-wise majority of a
sample of rows). Counts, per sampled row, the members whose word differs from the reference, the byte shift of
the row's checksum string against the reference string along the row (min / max), and the spread of that shift
across rows at the same string position. Input to the reference-row (delta) checksum design.
Usage: delta_probe.py N round nrows"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ringpop-go_amd"))
import swimsim  # noqa: E402
from swimsim import workloads as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
rounds = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "12,14,18").split(",")]
nrows = int(sys.argv[3]) if len(sys.argv) > 3 else 512
wl = W.config3(n=n, rounds=max(rounds) + 1, kill_round=10)
c = swimsim.Cluster(n)
r = 0
for R in rounds:
    while r < R:
        c.step(1, wl.events_for(r))
        r += 1
    idx = np.linspace(0, n - 1, nrows).astype(np.int64)
    st = np.empty((nrows, n), np.uint8)
    inc = np.empty((nrows, n), np.int64)
    for i, o in enumerate(idx):
        st[i], inc[i] = c.row(int(o))
    samp = np.linspace(0, nrows - 1, 31).astype(np.int64)
    # column-wise majority of the sample (by (status, inc) pair)
    key = st.astype(np.int64) * (1 << 50) + inc
    ks = key[samp]
    ks_sorted = np.sort(ks, axis=0)
    ref = ks_sorted[15]                     # median of 31 = majority when a value holds > half
    diff = key != ref[None, :]
    ndiff = diff.sum(axis=1)
    # string byte length per record: 19 + status + digits + 1 (tombstones / unknown: 0)
    lut = np.array([5, 7, 6, 5, 0, 0, 0, 0], np.int64)

    def reclen(stt, incc):
        dl = np.floor(np.log10(np.maximum(incc, 1).astype(np.float64))).astype(np.int64) + 1
        return np.where(stt < 4, 19 + lut[stt & 7] + dl + 1, 0)
    ref_st = (ref >> 50).astype(np.uint8)
    ref_inc = ref & ((1 << 50) - 1)
    lref = reclen(ref_st[None, :], ref_inc[None, :])[0]
    shifts = []
    for i in range(nrows):
        li = reclen(st[i][None, :], inc[i][None, :])[0]
        shifts.append(np.cumsum(li - lref))
    S = np.stack(shifts)                    # shift of member m's record end, per row
    spread_at = S.max(axis=0) - S.min(axis=0)
    out = {"n": n, "round": R, "rows": nrows, "diff_mean": float(ndiff.mean()), "diff_max": int(ndiff.max()),
           "diff_p50": float(np.median(ndiff)), "cols_nonuniform": int((diff.any(axis=0)).sum()),
           "shift_min": int(S.min()), "shift_max": int(S.max()), "spread_max_bytes": int(spread_at.max()),
           "spread_p50_bytes": float(np.median(spread_at)), "ref_len": int(lref.sum())}
    print(json.dumps(out), flush=True)
