"""Host-input leg timing split: fk_ingest (H2D + map + piece counts) vs fk_finish (last piece + merge),
for piece sizes given on the command line (0 = no piece counts).  Prints one line per setting."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fastkmer_amd as fk  # noqa: E402

n_reads = 1_000_000_000 // 114
dev = torch.empty(n_reads * 114, dtype=torch.uint8, device="cuda")
fk.synth_fasta_to_device(dev.data_ptr(), n_reads, 100, 100_000_000, seed=0x5EED)
host = torch.empty(dev.numel(), dtype=torch.uint8, pin_memory=True)
host.copy_(dev)
torch.cuda.synchronize()
for arg in sys.argv[1:]:
    pb = int(float(arg) * (1 << 20))
    if pb:
        os.environ["FASTKMER_PIECE_BYTES"] = str(pb)
        os.environ["FASTKMER_PIECE_COUNT"] = "1"
    else:
        os.environ["FASTKMER_PIECE_COUNT"] = "0"
    kc = fk.KmerCounter(28, 10, 3, 2048)
    rows = []
    for it in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        kc.ingest_ptr(host.data_ptr(), host.numel())
        t1 = time.perf_counter()
        kc.finish()
        t2 = time.perf_counter()
        st = kc.stats()
        rows.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3, st["ms_h2d"], st["pieces_counted"], st.get("ms_merge", 0.0),
                     st["ms_count"], st["ms_partition"]))
    r = rows[-1]
    print(f"piece {arg} MB: ingest {r[0]:.2f} ms finish {r[1]:.2f} ms total {r[0] + r[1]:.2f} | h2d {r[2]:.2f} "
          f"pieces {r[3]} merge {r[4]:.2f} count(sum) {r[5]:.2f} partition(sum) {r[6]:.2f}", flush=True)
    kc.close()
