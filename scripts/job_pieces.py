"""Where a staged job's piece work falls against its map launches (the landed segments), from a
rocprofv3 --kernel-trace CSV: python scripts/job_pieces.py <kernel_trace.csv> [min_ms]
Prints the last job's kernels of at least min_ms (default 0.25) with their start / end relative to the
job's first map launch, and every 8th map launch as a marker of how far the input had landed."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
min_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 0.25
ends = [i for i, r in enumerate(rows) if "k_bin_offsets" in r["Kernel_Name"]]
hi = ends[-1]
lo = ends[-2] + 1 if len(ends) > 1 else 0
job = rows[lo:hi + 1]
maps = [r for r in job if "k_map_fused" in r["Kernel_Name"]]
t0 = int(maps[0]["Start_Timestamp"])
ms = lambda t: (int(t) - t0) / 1e6  # noqa: E731
for i, r in enumerate(job):
    name = r["Kernel_Name"]
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    if "k_map_fused" in name:
        j = maps.index(r)
        if j % 8 == 0 or j == len(maps) - 1:
            print(f"{ms(r['Start_Timestamp']):9.3f} .. {ms(r['End_Timestamp']):9.3f}  map launch {j + 1}/{len(maps)}")
        continue
    if dur >= min_ms:
        print(f"{ms(r['Start_Timestamp']):9.3f} .. {ms(r['End_Timestamp']):9.3f}  {dur:7.3f}  q{r['Queue_Id']:>2}  {name[:60]}")
print(f"job: first map launch .. last kernel end {ms(job[-1]['End_Timestamp']):.2f} ms; "
      f"last map launch ends {ms(maps[-1]['End_Timestamp']):.2f} ms")
