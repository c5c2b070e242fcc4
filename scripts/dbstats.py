"""Kernel summary from a rocprofv3 rocpd database: python scripts/dbstats.py <run_results.db> [n] [csv_out]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tabs = [r[0] for r in db.execute("select name from sqlite_master where type in ('table','view')")]
kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
cols = [r[1] for r in db.execute(f"pragma table_info({ks})")]
name = "kernel_name" if "kernel_name" in cols else ("display_name" if "display_name" in cols else "name")
q = (f"select s.{name}, count(*), avg(d.end - d.start), sum(d.end - d.start) from {kd} d "
     f"join {ks} s on d.kernel_id = s.id group by s.{name} order by sum(d.end - d.start) desc")
rows = list(db.execute(q))
tot = sum(r[3] for r in rows)
out = open(sys.argv[3], "w") if len(sys.argv) > 3 else None
if out:
    out.write("Name,Calls,AverageNs,TotalDurationNs,Percentage\n")
for r in rows:
    if out:
        out.write(f"\"{r[0]}\",{r[1]},{r[2]:.1f},{r[3]},{100 * r[3] / tot:.2f}\n")
for r in rows[:n]:
    print(f"{r[0][:70]:70s} calls={r[1]:>5} avg={r[2] / 1e3:9.1f}us total={r[3] / 1e6:8.2f}ms {100 * r[3] / tot:5.1f}%")
