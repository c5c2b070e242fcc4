"""Per-kernel summary of a rocprofv3 --kernel-trace database (run_results.db): calls, total and
average duration, share of GPU kernel time -- the same table as rocprofv3 --stats' kernel_stats.csv.
Usage: python scripts/rocpd_stats.py <run_results.db> [steps]  (steps: also the per-step ms)"""
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    rows = list(db.execute("select name, count(*), sum(duration), avg(duration) from kernels group by name"))
    total = sum(r[2] for r in rows) or 1
    rows.sort(key=lambda r: -r[2])
    hdr = f"{'kernel':90s} {'calls':>6s} {'total ms':>10s} {'avg us':>10s} {'%':>6s}"
    if steps:
        hdr += f" {'ms/step':>8s}"
    print(hdr)
    for name, n, tot, avg in rows:
        line = f"{name[:90]:90s} {n:6d} {tot / 1e6:10.3f} {avg / 1e3:10.1f} {100 * tot / total:6.2f}"
        if steps:
            line += f" {tot / 1e6 / steps:8.3f}"
        print(line)


if __name__ == "__main__":
    main()
