"""useHT count at the configs[3] shape (k=55 m=12 B=8192, 150 bp reads of a 3 Gbp genome), 1 GB:
count time, rounds, spills, for the LDS tables and (FASTKMER_LDS_HT=0) the global tables."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

import fastkmer_amd as fk  # noqa: E402

k, m, B, rl = (int(v) for v in (sys.argv[1:] or ["55", "12", "8192", "150"]))
nbytes = int(os.environ.get("FK_BYTES", "1000000000"))
kc = fk.KmerCounter(k, m, 3, B, use_ht=True)
n = kc.synth_device(nbytes // (rl + 14), rl, 3_000_000_000, seed=0x5EED)
for it in range(3):
    kc.synth_device(nbytes // (rl + 14), rl, 3_000_000_000, seed=0x5EED)
    kc.finish()
    st = kc.stats()
    print(f"LDS_HT={os.environ.get('FASTKMER_LDS_HT', '1')} k={k}: count {st['ms_count']:.2f} ms partition "
          f"{st['ms_partition']:.2f} rounds {st.get('ht_rounds', 0)} spilled {st.get('ht_spilled', 0)} distinct {st['distinct']} "
          f"kmers {st['kmers']} big {st.get('ht_big_groups', 0)}", flush=True)
