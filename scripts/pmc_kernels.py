"""Per-kernel PMC counters (per launch) from scripts/pmc*.sh output: python scripts/pmc_kernels.py <dir> [name-substr...]"""
import collections, csv, glob, os, sys

d = sys.argv[1]
want = sys.argv[2:]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
launches = collections.defaultdict(set)
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0]
        agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
        launches[n].add((f, r["Dispatch_Id"]))
for n in sorted(agg):
    if want and not any(w in n for w in want):
        continue
    npass = len({f for f, _ in launches[n]})
    c = max(1, len(launches[n]) // max(1, npass))
    print(f"{n}  ({c} launches)")
    for k in sorted(agg[n]):
        print(f"    {k:24s} {agg[n][k] / c:14.4g}")
