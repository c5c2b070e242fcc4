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
want = [a for a in sys.argv[2:] if not a.startswith("--") and not a.endswith(".json")] or None
for name, cs in sorted(acc.items()):
    if want and not any(w in name for w in want):
        continue
    vals = {c: sum(v) / len(v) for c, v in cs.items()}
    print(name)
    print("   " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))

# --json OUT: HBM traffic of the encode+signature stage for bench.py's roofline.traffic.
# FETCH_SIZE / WRITE_SIZE are KiB; per MI355X_MICROARCH.md (HBM section) FETCH_SIZE
# reports half the bytes of 16-B/lane streaming reads on gfx950, so it is doubled.
if "--json" in sys.argv:
    import json
    out = sys.argv[sys.argv.index("--json") + 1]
    # the fused kernel when the run used it, else the two-kernel path
    fused = any(name.startswith("k_map_fused") for name in acc)
    stage = ("k_map_fused",) if fused else ("k_fasta_parse", "k_superkmers")
    per = {}
    for name, cs in acc.items():
        if any(name.startswith(s) for s in stage) and "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024
            w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
            per[name] = {"fetch_size_bytes_raw": f, "write_size_bytes": w, "hbm_bytes_corrected": 2 * f + w}
    json.dump({"source": sys.argv[1], "stage_kernel": "k_map_fused" if fused else "k_fasta_parse + k_superkmers",
               "kernels": per,
               "encode_signature_hbm_bytes_per_launch": sum(v["hbm_bytes_corrected"] for v in per.values()),
               "correction": "2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), MI355X_MICROARCH.md HBM section"},
              open(out, "w"), indent=1)
