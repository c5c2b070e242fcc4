"""Kernel / copy timeline of the last bench step from a rocprofv3 rocpd database (kernel-trace and
memory-copy trace): python scripts/timeline.py <run_results.db> [t_window_ms]
Prints every dispatch of the final `t_window_ms` of the trace with start offset, duration and the
idle gap before it on the GPU."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
win = float(sys.argv[2]) if len(sys.argv) > 2 else 40.0
tabs = [r[0] for r in db.execute("select name from sqlite_master where type in ('table','view')")]
kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
cols = [r[1] for r in db.execute(f"pragma table_info({ks})")]
name = "kernel_name" if "kernel_name" in cols else ("display_name" if "display_name" in cols else "name")
ev = [(r[0], r[1], r[2]) for r in db.execute(f"select d.start, d.end, s.{name} from {kd} d join {ks} s on d.kernel_id = s.id")]
mc = next((t for t in tabs if t.startswith("rocpd_memory_copy")), None)
if mc:
    for r in db.execute(f"select start, end, size from {mc}"):
        ev.append((r[0], r[1], f"COPY {r[2] / 1e6:.1f} MB"))
ev.sort()
t_end = max(e[1] for e in ev)
t0 = t_end - win * 1e6
last_end = None
for s, e, n in ev:
    if e < t0:
        last_end = e if last_end is None else max(last_end, e)
        continue
    gap = (s - last_end) / 1e3 if last_end is not None else 0.0
    if not n.startswith("COPY"):
        last_end = e if last_end is None else max(last_end, e)
    print(f"{(s - t0) / 1e6:8.3f} ms  dur {(e - s) / 1e3:8.1f} us  gap {gap:7.1f} us  {n[:80]}")
