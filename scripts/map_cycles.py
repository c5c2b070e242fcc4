"""Per-phase wave cycles of the fused map (FASTKMER_LIB = the -DFK_PROBES library, phase stamps):
the bench's 1 GB configs[1] input mapped FK_MAP_REPS times; prints each phase's share of the summed
wave cycles and the kernel time."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa
import numpy as np
import fastkmer_amd as fk
names = ["byte classes", "line state", "compaction", "code store + halo", "signature passes",
         "record phase", "(after passes)", "last barrier", "tile loads in flight"]
kc = fk.KmerCounter(28, 10, 3, 2048)
kc.synth_device(1_000_000_000 // 114, 100, 100_000_000, seed=0x5EED)
kc.map()
out = np.zeros(16, dtype=np.uint64)
fk._check(fk.lib().fk_debug_map_cycles(out.ctypes.data, 1))
reps = int(os.environ.get("FK_MAP_REPS", "3"))
ms = []
for _ in range(reps):
    kc.map()
    ms.append(kc.stats()["ms_signature_kernel"])
fk._check(fk.lib().fk_debug_map_cycles(out.ctypes.data, 1))
tot = float(out[:9].sum())
print(f"map kernel median {sorted(ms)[len(ms) // 2]:.3f} ms; summed wave cycles per launch {tot / reps:.4g}")
for i, n in enumerate(names):
    print(f"  {n:24s} {out[i] / reps:12.4g} cycles  {100 * out[i] / tot:5.1f} %")
