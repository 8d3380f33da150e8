"""Per-kernel dispatch statistics from a rocprofv3 rocpd database (the default output of --kernel-trace):
name, calls, average ms, total ms, sorted by total. Usage: kstats.py results.db [limit]"""
import sqlite3
import sys

db = sys.argv[1]
lim = int(sys.argv[2]) if len(sys.argv) > 2 else 20
c = sqlite3.connect(db)
q = ("select s.kernel_name, count(*), avg(k.end - k.start) / 1e6, sum(k.end - k.start) / 1e6 from rocpd_kernel_dispatch k "
     "join rocpd_info_kernel_symbol s on k.kernel_id = s.id group by s.kernel_name order by sum(k.end - k.start) desc "
     f"limit {lim}")
for name, n, avg, tot in c.execute(q):
    print(f"{avg:9.3f} ms x {n:5d} = {tot:9.2f} ms  {name[:110]}")
