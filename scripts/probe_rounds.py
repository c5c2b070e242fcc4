"""Cost of counting one rank's bins in R rounds (virtual ranks) vs one reduce, on one GPU."""
import sys, time
import torch
sys.path.insert(0, ".")
import fastkmer_amd as fk

n_reads = 1_000_000_000 // 114
for R in (1, 2, 4):
    a = fk.KmerCounter(28, 10, 3, 2048, n_ranks=R, rank=0)
    grouped = len(sys.argv) > 1 and sys.argv[1] == "grouped"
    if grouped:
        a.set_grouped_emit(True)
    a.synth_device(n_reads, 100, 100_000_000, seed=0x5EED)
    ctxs = [a] + [fk.KmerCounter(28, 10, 3, 2048, n_ranks=R, rank=r) for r in range(1, R)]
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        counts = a.map()
        rb = a.record_bytes
        send = torch.empty(sum(counts) * rb, dtype=torch.uint8, device="cuda")
        a.map_emit(send.data_ptr(), sum(counts))
        if grouped:
            prec, pkm = a.map_part_counts()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        off = 0
        per = []
        for r in range(R):
            s = time.perf_counter()
            if grouped:
                ctxs[r].reduce_grouped(send.data_ptr() + off * rb, counts[r], prec[r:r + 1], pkm[r:r + 1])
            else:
                ctxs[r].reduce(send.data_ptr() + off * rb, counts[r])
            torch.cuda.synchronize()
            per.append((time.perf_counter() - s) * 1e3)
            off += counts[r]
        t2 = time.perf_counter()
        dist = sum(c.stats()["distinct"] for c in ctxs)
        print(f"R={R} rep={rep} map+emit {1e3*(t1-t0):.2f} ms, reduces {1e3*(t2-t1):.2f} ms {['%.2f' % x for x in per]} distinct={dist}", flush=True)
    for c in ctxs:
        c.close()
