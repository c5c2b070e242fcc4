"""The kernels of one job after its last map launch (the tail after the last FASTA byte), from a
rocprofv3 --kernel-trace CSV: python scripts/tail_timeline.py <kernel_trace.csv> [job]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
job = int(sys.argv[2]) if len(sys.argv) > 2 else -1
waves = [i for i, r in enumerate(rows) if "k_bucket_count64_wave" in r["Kernel_Name"] or "count128_wave<2" in r["Kernel_Name"]]
w = waves[job]
last_map = max(i for i in range(w) if "k_map_fused" in rows[i]["Kernel_Name"])
end = next((i for i in range(w, len(rows)) if "k_bin_offsets" in rows[i]["Kernel_Name"]), len(rows) - 1)
t0 = int(rows[last_map]["End_Timestamp"])
prev_end = t0
busy = 0
for r in rows[last_map + 1:end + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = max(0, s - prev_end)
    busy += e - s
    print(f"{(s - t0) / 1e6:8.3f} ms  +{(e - s) / 1e6:7.3f}  gap {gap / 1e6:6.3f}  q{r['Queue_Id']:>2}  {r['Kernel_Name'][:70]}")
    prev_end = max(prev_end, e)
print(f"tail {(prev_end - t0) / 1e6:.2f} ms after the last map launch, kernels {busy / 1e6:.2f} ms")
