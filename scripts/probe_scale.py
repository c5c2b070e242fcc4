"""Per-GPU count work of the bench's weak-scaling runs on one GPU: N shards of
1 GB (bench.py's per-GPU workload) are mapped as ranks 0..N-1 of n_ranks=N and
rank 0 counts the records all shards send it (its B/N bins, N times larger
than on one GPU).  Prints the reduce's stage times.  Usage: probe_scale.py N [use_ht]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa
import fastkmer_amd as fk

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
ht = len(sys.argv) > 2 and sys.argv[2] == "1"
K, M, X, B = 28, 10, 3, 2048
reads = 1_000_000_000 // 114
mapper = fk.KmerCounter(K, M, X, B, ht, 0, n_ranks=N, rank=0)
parts, total = [], 0
for r in range(N):
    mapper.synth_device(reads, 100, 100_000_000, seed=0x5EED, first_read=r * reads)
    counts = mapper.map()
    send = torch.empty(max(sum(counts), 1) * 16, dtype=torch.uint8, device="cuda")
    mapper.map_emit(send.data_ptr(), max(sum(counts), 1))
    parts.append(send[:counts[0] * 16].clone())
    total += counts[0]
    del send
mapper.close()
recv = torch.cat(parts)
del parts
torch.cuda.empty_cache()
with fk.KmerCounter(K, M, X, B, ht, 0, n_ranks=N, rank=0) as kc:
    for i in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        kc.reduce(recv.data_ptr(), total)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        st = kc.stats()
    print(f"N={N} ht={int(ht)} rank 0: {total} records, {st['distinct']} distinct, reduce {dt:.1f} ms wall, "
          f"partition {st['ms_partition']:.1f} ms, count {st['ms_count']:.1f} ms, F={st['fine_bits']}, "
          f"buckets {st['buckets']}, large {st['oversize_buckets']}", flush=True)
