"""Map side only (parse + signature) of the bench workload, three times (for profilers)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa
import fastkmer_amd as fk
kc = fk.KmerCounter(28, 10, 3, 2048)
kc.synth_device(1_000_000_000 // 114, 100, 100_000_000, seed=0x5EED)
for i in range(3):
    kc.map()
st = kc.stats()
print(f"parse {st['ms_parse']:.3f} ms  signature {st['ms_signature']:.3f} ms  sigkernel {st['ms_signature_kernel']:.3f} ms  "
      f"records {st['superkmers']}", flush=True)
