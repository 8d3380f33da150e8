"""Kernel summary of a rocprofv3 rocpd database (the SQLite file rocprofv3 writes by default): per kernel name the
launch count, average and total duration; or, with --launches PATTERN, every launch of the matching kernels in order.
With --api, the HIP runtime calls (a --hip-trace run) by total duration, and the 30 longest single calls.
usage: rocpd_summary.py DB [--launches PATTERN] [--top N] [--api]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
args = sys.argv[2:]
if args and args[0] == "--api":
    views = [r[0] for r in db.execute("select name from sqlite_master where type in ('view','table')")]
    src = "regions" if "regions" in views else [v for v in views if "region" in v][0]
    for name, n, avg, tot in db.execute(f"select name, count(*), avg(end-start)/1e6, sum(end-start)/1e6 from {src} group by "
                                        "name order by sum(end-start) desc limit 25"):
        print(f"{name[:60]:60s} n={n:7d} avg={avg:9.3f} ms tot={tot:9.2f}")
    print("-- longest calls")
    for name, st, dur in db.execute(f"select name, start, (end-start)/1e6 from {src} order by (end-start) desc limit 30"):
        print(f"{name[:60]:60s} start={st} {dur:9.3f} ms")
    sys.exit(0)
if args and args[0] == "--launches":
    pat = args[1]
    for name, gx, wx, dur in db.execute("select name, grid_x, workgroup_x, (end-start)/1e6 from kernels where name like ? "
                                        "order by start", (f"%{pat}%",)):
        print(f"{name[:60]:60s} grid={gx:9d} wg={wx:4d} {dur:9.3f} ms")
else:
    top = int(args[1]) if args and args[0] == "--top" else 25
    for name, n, avg, tot in db.execute("select name, count(*), avg(end-start)/1e6, sum(end-start)/1e6 from kernels group by "
                                        "name order by sum(end-start) desc limit ?", (top,)):
        print(f"{name[:90]:90s} n={n:5d} avg={avg:9.3f} ms tot={tot:9.2f}")
