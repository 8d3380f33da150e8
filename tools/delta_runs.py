"""Diagnostic: emulate k_csd_scan's exception runs on sampled rows of a real cascade round (config 3), and count
exception blocks per 32-block super step (the helper batch holds 8). Usage: delta_runs.py N round nrows"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ringpop-go_amd"))
import swimsim  # noqa: E402
from swimsim import workloads as W  # noqa: E402

n = int(sys.argv[1]); R = int(sys.argv[2]); nrows = int(sys.argv[3])
wl = W.config3(n=n, rounds=R + 1, kill_round=10)
c = swimsim.Cluster(n)
for r in range(R):
    c.step(1, wl.events_for(r))
lut = np.array([5, 7, 6, 5, 0, 0, 0, 0], np.int64)


def reclen(st, inc):
    dl = np.floor(np.log10(np.maximum(inc, 1).astype(np.float64))).astype(np.int64) + 1
    return np.where(st < 4, 19 + lut[st & 7] + dl + 1, 0)


samp = [int(s * n // 31) for s in range(31)]
S = [c.row(o) for o in samp]
key = np.stack([st.astype(np.int64) * (1 << 50) + inc for st, inc in S])
ref = np.sort(key, axis=0)[15]
ref_st = (ref >> 50).astype(np.int64); ref_inc = ref & ((1 << 50) - 1)
LB = reclen(ref_st, ref_inc)
OB = np.concatenate([[0], np.cumsum(LB)])
out = {"round": R, "rows": []}
hist = np.zeros(40, np.int64)
for o in np.linspace(0, n - 1, nrows).astype(int):
    st, inc = c.row(int(o))
    st = st.astype(np.int64)
    k = st * (1 << 50) + inc
    same = (k == ref) | ((st >= 4) & (ref_st >= 4))
    d = np.nonzero(~same)[0]
    Lr = reclen(st, inc)
    L = int(Lr.sum()); kl = (L - 1) // 20 - 1
    s = 0; runs = [[0, 0]]
    for m in d:
        x = OB[m] + s; y = x + Lr[m]
        klo = (x - 32) // 20 + 1 if x >= 32 else 0
        khi = min((y - 1) // 20 if y >= 1 else -1, kl)
        if klo <= kl and khi >= klo:
            if klo <= runs[-1][1] + 1: runs[-1][1] = max(runs[-1][1], khi)
            else: runs.append([klo, khi])
        s += Lr[m] - LB[m]
    if runs[-1][1] + 1 >= kl: runs[-1][1] = kl
    else: runs.append([kl, kl])
    blocks = np.concatenate([np.arange(a, b + 1) for a, b in runs])
    per = np.bincount(blocks // 32)
    hist += np.bincount(np.minimum(per, 39), minlength=40)[:40]
    out["rows"].append({"o": int(o), "diffs": int(len(d)), "runs": len(runs), "entries": int(len(blocks)),
                        "max_per_superstep": int(per.max()), "over8": int((per > 8).sum()),
                        "run_len_max": int(max(b - a + 1 for a, b in runs))})
out["hist_entries_per_superstep"] = hist.tolist()
print(json.dumps(out))
