"""Benchmark: exact canonical k-mer counting throughput on MI355X.

Metric (BASELINE.json): input bases/sec for the whole node, k=28 short reads,
1/2/4/8 GPUs.  Workload (BASELINE.json configs[1], the metric's single-GPU
configuration): k=28 m=10 x=3 B=2048, 1 GB of synthetic 100 bp reads per GPU
(">r%010d" records, reads drawn from a 100 Mbp virtual genome, 0.2%
substitutions, 0.05% N).

One step = one job over the rank's 1 GB shard: parse + 2-bit encode +
signature + super-k-mer records in one fused kernel (the FASTdoop reader and
getSuperKmers, SBKC:62-65, :34-169) -> bin shuffle (RCCL all-to-all for
N > 1, reduceByKey SBKC:1034-1042) -> per-bin exact count (extractKXmers,
sorted, SBKC:428-660; --use-ht: extractKXmersHT, SBKC:664-739), counts
resident on the device (write=0, the reference's own switch).

Two legs over the same shard (generated on the device before timing):
  * `value` (the bench contract): the FASTA is resident in HBM when the timed
    region starts (fk_ingest_device).  The roofline of the fused
    encode+signature kernel comes from this leg (HIP events around each
    launch, on the stream it runs on).
  * `host_input_value` (SURVEY 8d / BASELINE.md 3's timer): the FASTA starts
    in pinned host memory and every step ingests it -- H2D in 32 MB segments
    on a copy stream, the fused kernel mapping every landed tile meanwhile.

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
FASTA_BYTES_PER_GPU = 1_000_000_000
HBM_PEAK = 8.0e12  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def cpu_baseline(sample_bytes: int, read_len: int = READ_LEN) -> dict:
    """The C restatement of the reference (oracle/) on a bounded sample of the
    same synthetic workload: one thread, 4 threads (the reference's Spark
    local[4], LocalTestKmerCounter.scala:62) and every core of this process's
    CPU share (at most 16, the GPU box's share).  `value` is the all-core rate."""
    import oracle
    n_reads = sample_bytes // (read_len + 14)
    data = fk.synth_fasta(n_reads, read_len, GENOME, seed=SEED)
    bases = n_reads * read_len
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    rates, secs = {}, {}
    for t in sorted({1, 4, cores}):
        t0 = time.perf_counter()
        r = oracle.OracleResult(data, K, M, B, threads=t)
        secs[t] = time.perf_counter() - t0
        rates[t] = bases / secs[t]
    return {"value": rates[cores], "unit": "bases/s", "cores": cores, "kind": "port",
            "value_1_thread": rates[1], "value_4_threads": rates[4],
            "sample": f"{n_reads} reads x {read_len} bp ({len(data) / 1e6:.0f} MB) of the bench workload, "
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


def load_traffic(kernel: str):
    """HBM bytes per launch of the encode+signature kernel from the committed
    rocprofv3 PMC summary (profiles/pmc_summary.json), if it holds that kernel."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    if d.get("stage_kernel") != kernel:
        return None
    return d.get("encode_signature_hbm_bytes_per_launch")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--bytes-per-gpu", type=int, default=FASTA_BYTES_PER_GPU)
    ap.add_argument("--cpu-sample-bytes", type=int, default=160_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-leg", action="store_true", help="skip the pinned-host-input leg")
    ap.add_argument("--use-ht", action="store_true", help="hash count (extractKXmersHT, useHT=1)")
    ap.add_argument("--rounds", type=int, default=0,
                    help="N > 1: all-to-all rounds overlapped with the count (0 = auto: 4 up to 4 GPUs, else 2)")
    ap.add_argument("--balance", action="store_true",
                    help="size-aware bin placement (reference useCustomPartitioner=1) instead of bin %% N")
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c4", "c5"],
                    help="c2 = BASELINE configs[1] (the metric's workload, default); c3 = configs[2] shape "
                         "(B=8192, per-GPU 1 GB); c4 = configs[3] shape (k=55 m=12 B=8192, 150 bp reads, two-word "
                         "keys); c5 = configs[4] shape (sequenceType=1, one long record)")
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

    k, m, x, b, read_len, seq_type, genome = K, M, X, B, READ_LEN, 0, GENOME
    if args.workload == "c3":
        b, genome = 8192, 3_000_000_000
    elif args.workload == "c4":
        k, m, b, read_len, genome = 55, 12, 8192, 150, 3_000_000_000
    elif args.workload == "c5":
        seq_type = 1
    rec_bytes = read_len + 14
    n_reads = args.bytes_per_gpu // rec_bytes
    rounds = 1 if (not distributed or args.balance) else (args.rounds or default_rounds(world))
    if rounds > 1:  # exchange in overlapped rounds (fastkmer_amd.exchange.RoundCounters)
        kc = RoundCounters(k, m, x, b, args.use_ht, seq_type, world=world, rank=rank, rounds=rounds, device=gpu)
    else:
        kc = fk.KmerCounter(k, m, x, b, use_ht=args.use_ht, sequence_type=seq_type, n_ranks=world, rank=rank,
                            device=gpu)

    # the rank's shard in pinned host memory (prepared outside the timed region)
    if args.workload == "c5":
        n_bases = args.bytes_per_gpu * 60 // 61
        data = long_sequence_fasta(n_bases, seed=SEED + rank)
        fasta_bytes, bases_per_rank = len(data), n_bases
        host_buf = torch.empty(fasta_bytes, dtype=torch.uint8).pin_memory()
        import numpy as np
        host_buf.numpy()[:] = np.frombuffer(data, dtype=np.uint8)
        del data
        dev_in = host_buf.to(dev)
    else:
        fasta_bytes = n_reads * rec_bytes
        bases_per_rank = n_reads * read_len
        dev_in = torch.empty(fasta_bytes, dtype=torch.uint8, device=dev)
        fk.synth_fasta_to_device(dev_in.data_ptr(), n_reads, read_len, genome, seed=SEED, first_read=rank * n_reads)
        host_buf = torch.empty(fasta_bytes, dtype=torch.uint8).pin_memory()
        host_buf.copy_(dev_in)
    torch.cuda.synchronize(dev)

    def run_job():
        if distributed:
            if rounds > 1:
                count_distributed_rounds(kc, device=dev)
            else:
                count_distributed(kc, device=dev, balance=args.balance)
        else:
            kc.finish()

    def step_host():
        kc.ingest_ptr(host_buf.data_ptr(), fasta_bytes)
        run_job()

    def step_device():
        kc.ingest_device(dev_in.data_ptr(), fasta_bytes)
        run_job()

    def barrier_sync():
        torch.cuda.synchronize(dev)
        if distributed:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def max_over_ranks(v: float) -> float:
        if not distributed:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def timed(step, steps, warmup):
        for _ in range(warmup):
            step()
        barrier_sync()
        per, t0 = [], time.perf_counter()
        for _ in range(steps):
            step()
            per.append(kc.stats())
        barrier_sync()
        return max_over_ranks(time.perf_counter() - t0), per

    # leg 1 (the bench contract's value): FASTA resident in HBM; also the encode+signature roofline
    elapsed, dev_stats = timed(step_device, args.steps, args.warmup)
    exchange = getattr(kc, "last_exchange", None)
    dev_sizes = kc.bin_sizes()
    assert int(dev_sizes.sum()) == dev_stats[-1]["distinct"] > 0
    # leg 2 (SURVEY 8d's timer): FASTA in pinned host memory, H2D inside every step
    host_elapsed, host_stats = None, None
    if not args.no_host_leg:
        host_elapsed, host_stats = timed(step_host, args.steps, args.warmup)
        # size-independent self-check: both legs counted the same shard
        sizes = kc.bin_sizes()
        assert int(sizes.sum()) == host_stats[-1]["distinct"] > 0 and (sizes == dev_sizes).all()
    del dev_in
    stats = dev_stats[-1]

    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        value = world * bases_per_rank * args.steps / elapsed
        metric = "input bases/sec (whole node), k=28 short reads, 1/2/4/8 GPUs"
        workload = {"c2": "BASELINE configs[1]: k=28 m=10 x=3 B=2048, 1 GB synthetic 100 bp reads per GPU",
                    "c3": "BASELINE configs[2] shape: k=28 m=10 x=3 B=8192, 1 GB synthetic 100 bp reads per GPU "
                          "(3 Gbp virtual genome)",
                    "c4": "BASELINE configs[3] shape: k=55 m=12 x=3 B=8192, 1 GB synthetic 150 bp reads per GPU",
                    "c5": "BASELINE configs[4] shape: sequenceType=1, one synthetic long record "
                          "(60-col lines, 100 x 10 kbp N runs, 5% soft-masked) of 1 GB per GPU"}[args.workload]
        if args.workload != "c2":
            metric += f" [{args.workload} workload, not the headline configuration]"
        if args.use_ht:
            metric += " [useHT=1: hash count]"
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
            "data": ("synthetic %d bp reads (100 Mbp virtual genome, 0.2%% subst, 0.05%% N), generated on the "
                     "device and staged to pinned host memory before timing" % read_len
                     if args.workload != "c5" else "synthetic long record (host-generated, pinned host memory)"),
            "timed_region": "FASTA resident in HBM -> records -> exchange (N > 1) -> counts resident on the "
                            "device (write=0); host_input_value adds the H2D from pinned host memory",
            "config": {"workload": workload,
                       "k": k, "m": m, "x": x, "B": b, "useHT": int(args.use_ht), "sequenceType": seq_type,
                       "fasta_bytes_per_gpu": fasta_bytes,
                       "bases_per_gpu": bases_per_rank,
                       "parallelism": (f"bins placed by size (LPT) over {world} GPU(s)" if args.balance and distributed
                                       else f"bins round-robin over {world} GPU(s)"),
                       "exchange_rounds": rounds},
            "stages_ms": {"map": stats["ms_signature"] + stats["ms_parse"], "partition": stats["ms_partition"],
                          "count": stats["ms_count"], "fused_map": bool(stats["fused_map"])},
            "kmers_per_gpu": stats["kmers"], "distinct_rank0": stats["distinct"],
        }
        if host_stats is not None:
            hs = host_stats[-1]
            out["host_input_value"] = world * bases_per_rank * args.steps / host_elapsed
            out["host_input_ms_per_step"] = host_elapsed / args.steps * 1e3
            out["host_input_timed_region"] = ("FASTA in pinned host memory -> H2D (32 MB segments on a copy stream, "
                                              "overlapped with the fused map) -> records -> exchange -> counts")
            out["host_input_stages_ms"] = {"h2d": hs["ms_h2d"], "map_overlapped_with_h2d": hs["ms_signature"],
                                           "partition": hs["ms_partition"], "count": hs["ms_count"]}
            out["pcie_h2d_GBps"] = fasta_bytes / (hs["ms_h2d"] * 1e-3) / 1e9 if hs["ms_h2d"] else None
        fused = all(s["fused_map"] for s in dev_stats)
        # encode+signature stage: algorithmic bytes = FASTA bytes read per launch,
        # time = the fused kernel's HIP-event duration on its stream (two kernels when not fused)
        t_k = sum(s["ms_signature_kernel"] + s["ms_encode_kernel"] for s in dev_stats) / len(dev_stats) * 1e-3
        kname = ("k_map_fused" if fused else "k_fasta_parse + k_superkmers")
        achieved = fasta_bytes / t_k
        out["roofline"] = {"bound": "hbm", "kernel": kname + " (encode + signature: FASTA bytes -> records)",
                           "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                           "frac": achieved / HBM_PEAK, "traffic": load_traffic(kname),
                           "bytes_alg_per_launch": fasta_bytes, "ms_per_launch": t_k * 1e3,
                           "measured": "HIP events around each launch on the context stream"}
        if exchange:
            out["exchange"] = exchange
        if world == 1 and not args.no_cpu_baseline and args.workload == "c2":
            out["cpu_baseline"] = cpu_baseline(args.cpu_sample_bytes)
        print(json.dumps(out), flush=True)
    kc.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
