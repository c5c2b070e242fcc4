"""Map side only (fused parse + signature) of the bench workload, repeated (for profilers and probes).
FK_MAP_REPS (default 3) maps; prints the median kernel time."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa
import fastkmer_amd as fk
kc = fk.KmerCounter(28, 10, 3, int(os.environ.get('FK_B', '2048')))
kc.synth_device(1_000_000_000 // 114, 100, 100_000_000, seed=0x5EED)
ms = []
for i in range(int(os.environ.get('FK_MAP_REPS', '3'))):
    kc.map()
    st = kc.stats()
    ms.append(st['ms_signature_kernel'] + st['ms_encode_kernel'])
ms.sort()
print(f"map kernel median {ms[len(ms) // 2]:.3f} ms  min {ms[0]:.3f}  fused {st['fused_map']}  "
      f"records {st['superkmers']}  kmers {st['kmers']}", flush=True)
