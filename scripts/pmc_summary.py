"""Average PMC counters per kernel over the dispatches of a pmc run:
python scripts/pmc_summary.py gpurun_out/pmc_<tag>"""
import collections
import csv
import glob
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fk::", "")
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
want = sys.argv[2:] or None
for name, cs in sorted(acc.items()):
    if want and not any(w in name for w in want):
        continue
    vals = {c: sum(v) / len(v) for c, v in cs.items()}
    print(name)
    print("   " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))
