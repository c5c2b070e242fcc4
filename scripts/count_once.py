"""One counter, three counts of the bench workload; prints the stage split (for profilers)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa
import fastkmer_amd as fk
K, M, RL = int(os.environ.get('FK_K', '28')), int(os.environ.get('FK_M', '10')), int(os.environ.get('FK_RL', '100'))
kc = fk.KmerCounter(K, M, 3, int(os.environ.get('FK_B', '2048')), use_ht=os.environ.get('FK_HT', '0') == '1')
kc.synth_device(int(os.environ.get('FK_BYTES', '1000000000')) // (RL + 14), RL, int(os.environ.get('FK_GENOME', '100000000')), seed=0x5EED)
for i in range(int(os.environ.get('FK_JOBS', '3'))):
    kc.finish()
st = kc.stats()
print(f"count {st['ms_count']:.2f} ms  partition {st['ms_partition']:.2f}  buckets {st['buckets']} F {st['fine_bits']} "
      f"oversize {st['oversize_buckets']} kmers {st['kmers']} distinct {st['distinct']} heavy_keys {st['heavy_keys']} "
      f"block_buckets {st['block_buckets']} big_buckets {st['big_buckets']} split {st['split_buckets']}"
      f"{' ht_spilled %d ht_rounds %d' % (st.get('ht_spilled', 0), st.get('ht_rounds', 0)) if os.environ.get('FK_HT') == '1' else ''}",
      flush=True)
