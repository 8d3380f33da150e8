"""diagnostics: compare the checksum kernel's hashed block stream with the oracle's checksum string"""
import sys
sys.path.insert(0, 'tests'); sys.path.insert(0, 'ringpop-go_amd')
import numpy as np, swimsim
from oracle_ffi import OracleSim
for n in (16, 64, 100):
    e = swimsim.Cluster(n); o = OracleSim(n)
    ec = e.checksums(); oc = o.checksums()
    s = o.checksum_string(0) if hasattr(o, 'checksum_string') else None
    nw = (n * 40) // 4 + 64
    dump = e.debug_cs_stream(0, nw)
    got = dump.tobytes()
    print(n, hex(int(ec[0])), hex(int(oc[0])), (ec == oc).all(), flush=True)
    if s is not None:
        nb = ((len(s) - 1) // 20) * 20
        exp = s[:nb]
        print(' stream eq', got[:nb] == exp, len(exp))
        if got[:nb] != exp:
            for i in range(nb):
                if got[i] != exp[i]:
                    print(' first diff at byte', i, got[max(0, i - 8):i + 24], exp[max(0, i - 8):i + 24]); break
