"""Cycles per wave64 VALU instruction per SIMD from rocprofv3 PMC output (scripts/r05_valu_pmc.sh):
GRBM_GUI_ACTIVE counts GPU cycles summed over the 8 XCDs, so a dispatch lasted GRBM / 8 cycles;
SQ_INSTS_VALU / 1024 SIMDs = VALU instructions per SIMD.  Prints, per kernel, the counters per dispatch,
the effective clock (cycles / kernel-trace duration where a trace exists) and cycles per VALU per SIMD.
python scripts/valu_table.py <dir>"""
import collections, csv, glob, os, sys

d = sys.argv[1]
ubench_names = {}
log = os.path.join(d, "ubench.log")
if os.path.exists(log):  # op_survey prints one line per kernel k<i>, in order
    lines = [ln for ln in open(log) if ln[:8].strip().replace(".", "").isdigit()]
    for i, ln in enumerate(lines):
        ubench_names[f"k{i}"] = ln.split(None, 1)[1].strip()
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[n][(f, r["Dispatch_Id"])].append((r["Counter_Name"], float(r["Counter_Value"])))
dur = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, "t", "*kernel_trace.csv")):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")
        dur[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
print(f"{'kernel':58s} {'dispatches':>10s} {'GRBM/8 cyc':>11s} {'VALU/SIMD':>10s} {'cyc/VALU/SIMD':>13s} "
      f"{'BUSY/GRBM':>9s} {'WAIT_INST/WAVE':>14s} {'SALU/VALU':>9s} {'clock GHz':>9s}")
for n in sorted(agg):
    per = []
    for key, vals in agg[n].items():
        c = collections.defaultdict(float)
        for name, v in vals:
            c[name] += v
        per.append(c)
    if not per:
        continue
    m = {k: sum(p[k] for p in per) / len(per) for k in per[0]}
    grbm = m.get("GRBM_GUI_ACTIVE", 0.0) / 8
    valu = m.get("SQ_INSTS_VALU", 0.0) / 1024
    if valu < 1000:
        continue
    label = n
    base = n.split("<")[0].strip()
    if base in ubench_names:
        label = f"{base}: {ubench_names[base][:48]}"
    clk = f"{grbm / (sorted(dur[n])[len(dur[n]) // 2]) / 1e9:9.2f}" if dur.get(n) else f"{'-':>9s}"
    print(f"{label[:58]:58s} {len(per):10d} {grbm:11.4g} {valu:10.4g} {grbm / valu:13.2f} "
          f"{m.get('SQ_BUSY_CYCLES', 0) / max(1.0, m.get('GRBM_GUI_ACTIVE', 1)):9.3f} "
          f"{m.get('SQ_WAIT_INST_ANY', 0) / max(1.0, m.get('SQ_WAVE_CYCLES', 1)):14.3f} "
          f"{m.get('SQ_INSTS_SALU', 0) / max(1.0, m.get('SQ_INSTS_VALU', 1)):9.3f} {clk}")
