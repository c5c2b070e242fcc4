"""Benchmark: exact canonical k-mer counting throughput on MI355X.

Metric (BASELINE.json): input bases/sec for the whole node, k=28 short reads,
1/2/4/8 GPUs, counts bit-exact.  Workload (BASELINE.json configs[1]):
k=28 m=10 x=3 B=2048, 1 GB of synthetic 100 bp reads per GPU (">r%010d"
records, reads drawn from a 100 Mbp virtual genome, 0.2% substitutions,
0.05% N), generated on the device before timing, so the input is resident
in HBM when the timed region starts.

One step = one full pass of the hot path over the resident FASTA: parse +
2-bit encode + signature + super-k-mer records (getSuperKmers) -> bin
shuffle (RCCL all-to-all for N > 1) -> per-bin exact count (extractKXmers,
sorted), counts resident on device (write=0, the reference's own switch).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
        (N > 1: torchrun --nproc-per-node N bench.py --gpus N ...)
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (first: one HIP runtime per process, see fastkmer_amd.lib)
import torch.distributed as dist  # noqa: E402

import fastkmer_amd as fk  # noqa: E402
from fastkmer_amd.exchange import RoundCounters, count_distributed, count_distributed_rounds, default_rounds  # noqa: E402

K, M, X, B = 28, 10, 3, 2048
READ_LEN = 100
GENOME = 100_000_000
SEED = 0x5EED
REC_BYTES = READ_LEN + 14
FASTA_BYTES_PER_GPU = 1_000_000_000
HBM_PEAK = 8.0e12  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def cpu_baseline(sample_bytes: int) -> dict:
    """The C restatement of the reference (oracle/) on a bounded sample of the
    same synthetic workload: one thread, 4 threads (the reference's Spark
    local[4], LocalTestKmerCounter.scala:62) and every core of this process's
    CPU share (at most 16, the GPU box's share).  `value` is the all-core rate."""
    import os
    import oracle
    n_reads = sample_bytes // REC_BYTES
    data = fk.synth_fasta(n_reads, READ_LEN, GENOME, seed=SEED)
    bases = n_reads * READ_LEN
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    rates, secs = {}, {}
    for t in sorted({1, 4, cores}):
        t0 = time.perf_counter()
        r = oracle.OracleResult(data, K, M, B, threads=t)
        secs[t] = time.perf_counter() - t0
        rates[t] = bases / secs[t]
    return {"value": rates[cores], "unit": "bases/s", "cores": cores, "kind": "port",
            "value_1_thread": rates[1], "value_4_threads": rates[4],
            "sample": f"{n_reads} reads x {READ_LEN} bp ({len(data) / 1e6:.0f} MB) of the bench workload, "
                      f"oracle/fk_oracle.c (fko_count_mt: record-aligned input splits, per-thread bins, "
                      f"bins merged and reduced in parallel) at 1/4/{cores} threads: "
                      f"{secs[1]:.1f}/{secs[4]:.1f}/{secs[cores]:.1f} s, {r.total_kmers} k-mers"}


def long_sequence_fasta(n_bases: int, seed: int = 0x5EED) -> bytes:
    """BASELINE configs[4] shape: one '>chrSynthetic' record,
    60-column lines, uniform ACGT with 100 runs of 10 kbp of N and 5% of
    the bases soft-masked (lowercase, invalid for the reference)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    seq = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, n_bases, dtype=np.uint8)].copy()
    for start in rng.integers(0, max(1, n_bases - 10_000), 100):
        seq[start:start + 10_000] = ord("N")
    for start in rng.integers(0, max(1, n_bases - 50_000), max(1, n_bases // 1_000_000)):
        seq[start:start + 50_000] |= 0x20  # lowercase
    n_lines = (n_bases + 59) // 60
    body = np.full(n_lines * 61, ord("\n"), dtype=np.uint8)
    view = body.reshape(n_lines, 61)
    full = np.zeros(n_lines * 60, dtype=np.uint8)
    full[:n_bases] = seq
    view[:, :60] = full.reshape(n_lines, 60)
    out = body.tobytes()
    tail = n_lines * 60 - n_bases  # drop the padding of the last line
    if tail:
        out = out[:len(out) - 1 - tail] + b"\n"
    return b">chrSynthetic\n" + out


def load_traffic():
    """HBM bytes per launch of the encode+signature stage from the committed
    rocprofv3 PMC summary (profiles/), if present."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    return d.get("encode_signature_hbm_bytes_per_launch")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--bytes-per-gpu", type=int, default=FASTA_BYTES_PER_GPU)
    ap.add_argument("--cpu-sample-bytes", type=int, default=64_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-input", action="store_true",
                    help="PCIe-inclusive variant: the FASTA starts in pinned host memory and every step "
                         "ingests it (H2D) before counting; reported as a separate metric, never as the headline")
    ap.add_argument("--rounds", type=int, default=0,
                    help="N > 1: all-to-all rounds overlapped with the count (0 = auto: 4 up to 4 GPUs, else 2)")
    ap.add_argument("--balance", action="store_true",
                    help="size-aware bin placement (reference useCustomPartitioner=1) instead of bin %% N")
    ap.add_argument("--workload", default="c2", choices=["c2", "c4", "c5"],
                    help="c2 = BASELINE configs[1] (the metric's workload, default); c4 = configs[3] shape "
                         "(k=55 m=12 B=8192, 150 bp reads, two-word keys); c5 = configs[4] shape "
                         "(sequenceType=1, one long record, host-generated, ingested before timing)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo stages records through host memory "
                         "(rehearsal of N > 1 with ranks sharing a GPU)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    gpu = local_rank if args.backend == "nccl" else local_rank % torch.cuda.device_count()
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if distributed:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    k, m, x, b, read_len, seq_type = K, M, X, B, READ_LEN, 0
    if args.workload == "c4":
        k, m, b, read_len = 55, 12, 8192, 150
    elif args.workload == "c5":
        seq_type = 1
    rec_bytes = read_len + 14
    n_reads = args.bytes_per_gpu // rec_bytes
    rounds = 1 if (not distributed or args.balance) else (args.rounds or default_rounds(world))
    if rounds > 1:  # exchange in overlapped rounds (fastkmer_amd.exchange.RoundCounters)
        kc = RoundCounters(k, m, x, b, False, seq_type, world=world, rank=rank, rounds=rounds, device=gpu)
    else:
        kc = fk.KmerCounter(k, m, x, b, use_ht=False, sequence_type=seq_type, n_ranks=world, rank=rank,
                            device=gpu)
    if args.workload == "c5":
        # one long record per rank (weak scaling), resident on the device before timing
        n_bases = args.bytes_per_gpu * 60 // 61
        data = long_sequence_fasta(n_bases, seed=SEED + rank)
        kc.ingest(data)
        fasta_bytes, bases_per_rank = len(data), n_bases
        del data
    else:
        # per-rank shard of one synthetic read set (weak scaling: 1 GB per GPU)
        fasta_bytes = kc.synth_device(n_reads, read_len, GENOME, seed=SEED, first_read=rank * n_reads)
        bases_per_rank = n_reads * read_len
    host_buf = None
    if args.host_input and args.workload == "c2":  # the same shard in pinned host memory, prepared outside the timed region
        import numpy as np
        host_buf = torch.empty(fasta_bytes, dtype=torch.uint8).pin_memory()
        host_buf.copy_(torch.from_numpy(np.frombuffer(
            fk.synth_fasta(n_reads, READ_LEN, GENOME, seed=SEED, first_read=rank * n_reads), dtype=np.uint8)))

    def step():
        if host_buf is not None:
            kc.ingest_ptr(host_buf.data_ptr(), fasta_bytes)
        if distributed:
            if rounds > 1:
                count_distributed_rounds(kc, device=dev)
            else:
                count_distributed(kc, device=dev, balance=args.balance)
        else:
            kc.finish()

    def barrier_sync():
        torch.cuda.synchronize(dev)
        if distributed:
            dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        step()
    barrier_sync()
    stage_ms, stats = [], None
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        st = kc.stats()
        stage_ms.append(st["ms_parse"] + st["ms_signature"])
        stats = st
    barrier_sync()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    # size-independent self-check of this rank's result (outside the timed region)
    sizes = kc.bin_sizes()
    assert int(sizes.sum()) == stats["distinct"] > 0

    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        value = world * bases_per_rank * args.steps / elapsed
        # encode+signature stage: algorithmic bytes = FASTA bytes read,
        # time = every launch between FASTA and super-k-mer records (HIP events on the ctx stream)
        t_es = sum(stage_ms) / len(stage_ms) * 1e-3
        achieved = fasta_bytes / t_es
        metric = "input bases/sec (whole node), k=28 short reads, 1/2/4/8 GPUs; counts bit-exact"
        workload = {"c2": "BASELINE configs[1]: k=28 m=10 x=3 B=2048, 1 GB synthetic 100 bp reads per GPU",
                    "c4": "BASELINE configs[3] shape: k=55 m=12 x=3 B=8192, 1 GB synthetic 150 bp reads per GPU",
                    "c5": "BASELINE configs[4] shape: sequenceType=1, one synthetic long record "
                          "(60-col lines, 100 x 10 kbp N runs, 5% soft-masked) of 1 GB per GPU"}[args.workload]
        if args.workload != "c2":
            metric += f" [{args.workload} workload, not the headline configuration]"
        if args.host_input:
            metric += " [PCIe-inclusive variant: FASTA in pinned host memory, H2D inside every step]"
        out = {
            "metric": metric,
            "value": value,
            "unit": "bases/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": ("synthetic (device-generated %d bp reads, 100 Mbp virtual genome, 0.2%% subst, 0.05%% N)" % read_len
                     if args.workload != "c5" else "synthetic long record (host-generated, ingested before timing)"),
            "config": {"workload": workload,
                       "k": k, "m": m, "x": x, "B": b, "useHT": 0, "sequenceType": seq_type,
                       "fasta_bytes_per_gpu": fasta_bytes,
                       "bases_per_gpu": bases_per_rank, "parallelism": (f"bins placed by size (LPT) over {world} GPU(s)" if args.balance and distributed
                                           else f"bins round-robin over {world} GPU(s)"),
                       "exchange_rounds": rounds},
            "roofline": {"bound": "hbm",
                         "kernel": "encode+signature stage: k_fasta_parse + k_superkmers (+ their memsets and "
                                   "the per-tile k-mer count scan)",
                         "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK, "traffic": load_traffic(),
                         "bytes_alg_per_launch": fasta_bytes, "ms_per_launch": t_es * 1e3},
            "stages_ms": {"parse": stats["ms_parse"], "signature": stats["ms_signature"],
                          "partition": stats["ms_partition"], "count": stats["ms_count"]},
            "kmers_per_gpu": stats["kmers"], "distinct_rank0": stats["distinct"],
        }
        if world == 1 and not args.no_cpu_baseline and args.workload == "c2":
            out["cpu_baseline"] = cpu_baseline(args.cpu_sample_bytes)
        print(json.dumps(out), flush=True)
    kc.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
