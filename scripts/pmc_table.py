"""Per-kernel HBM bytes / VALU / LDS table of one PMC run (scripts/r06_pmc.sh), per launch and per job:
python scripts/pmc_table.py <dir> <fasta_bytes> <launches-per-job> [--json OUT]

HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes; gfx950: FETCH_SIZE reports half the bytes of
16-B/lane streaming reads, MI355X_MICROARCH.md HBM section); ms = GRBM_GUI_ACTIVE / 8 XCDs / 2.4 GHz.
The count stage = every kernel after the map and the partition (expansion, bucket cut, tiers, split)."""
import collections
import csv
import glob
import json
import os
import sys

d, fasta, jobs = sys.argv[1], float(sys.argv[2]), int(sys.argv[3])
acc = collections.defaultdict(lambda: collections.defaultdict(float))
nd = collections.defaultdict(lambda: collections.defaultdict(set))
for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fk::", "")
        acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
        nd[n][r["Counter_Name"]].add((f, r["Dispatch_Id"]))


def per_job(n, c):
    """counter c of kernel n summed over its dispatches of one job (the run counts `jobs` jobs)"""
    return acc[n].get(c, 0.0) / jobs


MAP, PART = ("k_map_fused", "k_fasta_parse", "k_superkmers", "k_tile_totals"), ("k_part_",)
rows, tot = [], collections.defaultdict(float)
for n in sorted(acc, key=lambda n: -(2 * per_job(n, "FETCH_SIZE") + per_job(n, "WRITE_SIZE"))):
    rd, wr = 2 * per_job(n, "FETCH_SIZE") * 1024, per_job(n, "WRITE_SIZE") * 1024
    ms = per_job(n, "GRBM_GUI_ACTIVE") / 8 / 2.4e6
    valu, lds, confl = per_job(n, "SQ_INSTS_VALU"), per_job(n, "SQ_INSTS_LDS"), per_job(n, "SQ_LDS_BANK_CONFLICT")
    launches = len(nd[n].get("FETCH_SIZE", ())) // jobs if nd[n].get("FETCH_SIZE") else 0
    stage = "map" if n.startswith(MAP) else ("partition" if n.startswith(PART) else "count")
    rows.append((n, stage, launches, ms, rd, wr, valu, lds, confl))
    for key, v in (("read", rd), ("write", wr), ("ms", ms)):
        tot[(stage, key)] += v
print(f"{'kernel':52s} {'stage':9s} {'n':>4s} {'ms':>7s} {'read GB':>8s} {'write GB':>8s} {'VALU':>9s} {'LDS':>9s} {'LDS confl':>9s}")
for n, stage, launches, ms, rd, wr, valu, lds, confl in rows:
    if rd + wr < 1e6 and ms < 0.01:
        continue
    print(f"{n[:52]:52s} {stage:9s} {launches:4d} {ms:7.2f} {rd / 1e9:8.3f} {wr / 1e9:8.3f} {valu:9.3g} {lds:9.3g} {confl:9.3g}")
gb = fasta / 1e9
for stage in ("map", "partition", "count"):
    r, w = tot[(stage, "read")], tot[(stage, "write")]
    print(f"{stage:9s}: read {r / 1e9:.2f} GB + write {w / 1e9:.2f} GB = {(r + w) / 1e9:.2f} GB per job, "
          f"{(r + w) / 1e9 / gb:.2f} GB per GB of FASTA, kernels {tot[(stage, 'ms')]:.2f} ms")
if "--json" in sys.argv:
    out = sys.argv[sys.argv.index("--json") + 1]
    per = {}
    for n, stage, launches, ms, rd, wr, valu, lds, confl in rows:
        if stage == "map" and n.startswith("k_map_fused"):
            per[n] = {"fetch_size_bytes_raw": rd / 2 / max(1, launches), "write_size_bytes": wr / max(1, launches),
                      "hbm_bytes_corrected": (rd + wr) / max(1, launches), "valu_per_launch": valu / max(1, launches),
                      "launches_per_job": launches}
    json.dump({"source": d, "stage_kernel": "k_map_fused", "kernels": per,
               "encode_signature_hbm_bytes_per_launch": sum(v["hbm_bytes_corrected"] for v in per.values()),
               "valu_instructions_per_launch": sum(v["valu_per_launch"] for v in per.values()),
               "fasta_bytes_per_launch": fasta / max(1, sum(v["launches_per_job"] for v in per.values())),
               "correction": "2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), MI355X_MICROARCH.md HBM section"},
              open(out, "w"), indent=1)
