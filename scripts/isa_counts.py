"""Static instruction counts of k_map_fused<512, 28, 10, 0> per phase (the s_memtime stamps of the
-DFK_PROBES build delimit the phases): python scripts/isa_counts.py [-DFK_MAPV=3 ...].  The map kernel
issues one wave64 VALU instruction per 4 cycles per SIMD (profiles/r04b_pmc_split_map.txt), so the
VALU count of the pass body times ~29 passes per tile is its time."""
import collections, os, subprocess, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(ROOT, "fastkmer_amd", "csrc", "fk_kernels.hip")
out = os.path.join(tempfile.gettempdir(), "fk_isa_counts.s")
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-DFK_PROBES", *sys.argv[1:],
                       "--cuda-device-only", "-S", "-o", out, src], stderr=subprocess.DEVNULL)
lines = open(out).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_ZN2fk11k_map_fusedILi512ELi28ELi10ELi0E"))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
names = ["prologue", "loads", "byte classes", "line state", "compaction", "code store", "signature pass",
         "record phase", "after passes", "last barrier", "tail"]
seg, cur = [], collections.Counter()
for l in lines[start:end]:
    t = l.strip()
    if not t or t.startswith((";", ".")) or t.endswith(":"):
        continue
    op = t.split()[0]
    if op == "s_memtime":
        seg.append(cur)
        cur = collections.Counter()
        continue
    cur["valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "lds" if op.startswith("ds_") else "mem"] += 1
seg.append(cur)
for i, c in enumerate(seg):
    print(f"{i:2d} {names[i] if i < len(names) else '':15s} VALU {c['valu']:5d}  SALU {c['salu']:4d}  LDS {c['lds']:3d}  MEM {c['mem']:3d}")
