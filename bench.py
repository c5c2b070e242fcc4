"""Benchmark: exact canonical k-mer counting throughput on MI355X.

Metric (BASELINE.json): input bases/sec for the whole node, k=28 short reads,
1/2/4/8 GPUs, counts bit-exact.  Workloads (synthetic ">r%010d" 100 bp reads,
0.2% substitutions, 0.05% N):
  * N = 1 (default c2): BASELINE configs[1], k=28 m=10 x=3 B=2048, 1 GB of
    FASTA from a 100 Mbp virtual genome;
  * N > 1 (default c3): BASELINE configs[2], k=28 m=10 x=3 B=8192, 6.25 GB of
    FASTA per GPU from a 3 Gbp virtual genome (N = 8: the 50 GB job),
    weak scaling.

One step = one job over the rank's shard (SparkBinKmerCounter.executeJob,
SBKC:989-1046): parse + 2-bit encode + signature + super-k-mer records in one
fused kernel (the FASTdoop reader and getSuperKmers, SBKC:62-65, :34-169) ->
bin shuffle (N > 1: the library's own RCCL all-to-all over xGMI, reduceByKey
SBKC:1034-1042) -> per-bin exact count (extractKXmers, SBKC:428-660;
--use-ht: extractKXmersHT, SBKC:664-739), counts resident on the device
(write=0, the reference's own switch).

`value` / `ms_per_step` follow SURVEY 8d's timer: the FASTA starts in pinned
host memory and every step ingests it (H2D in segments on a copy stream, the
fused kernel mapping every landed tile meanwhile, and with N > 1 every landed
piece exchanged while the next one is copied) and ends with the counts on the
device.  `device_resident_value` is the same job with the FASTA already in HBM;
the roofline of the fused encode+signature kernel comes from that leg (HIP
events around its one launch, on the stream it runs on).  With N > 1, or more
than 2 GB per GPU, that leg runs only with --device-leg (a rank's 6.25 GB shard
would otherwise hold both legs' buffers on its GPU at once).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
        (N > 1: torchrun --nproc-per-node N bench.py --gpus N ...; one process per GPU,
         the RCCL unique id travels over torch.distributed's gloo group)
        python bench.py --rehearse-local N --bytes-per-gpu B   (N ranks as threads of one
         process on one GPU: the whole native N > 1 path with the in-process transport)
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (first: one HIP runtime per process, see fastkmer_amd.lib)
import torch.distributed as dist  # noqa: E402

import fastkmer_amd as fk  # noqa: E402

SEED = 0x5EED
HBM_PEAK = 8.0e12  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
XGMI_LINK_PEAK = 153e9  # per link, both directions (7 links per GPU; prompt / MI355X_MICROARCH.md)

# workload -> (k, m, B, read_len, genome, sequence_type, default FASTA bytes per GPU, description)
WORKLOADS = {
    "c2": (28, 10, 2048, 100, 100_000_000, 0, 1_000_000_000,
           "BASELINE configs[1]: k=28 m=10 x=3 B=2048, {gb} synthetic 100 bp reads per GPU"),
    "c3": (28, 10, 8192, 100, 3_000_000_000, 0, 6_250_000_000,
           "BASELINE configs[2]: k=28 m=10 x=3 B=8192, {gb} synthetic 100 bp reads per GPU "
           "(3 Gbp virtual genome; 8 GPUs x 6.25 GB = the 50 GB job)"),
    "c4": (55, 12, 8192, 150, 3_000_000_000, 0, 6_250_000_000,
           "BASELINE configs[3]: k=55 m=12 x=3 B=8192, {gb} synthetic 150 bp reads per GPU "
           "(3 Gbp virtual genome; 8 GPUs x 6.25 GB = the 50 GB job)"),
    "c5": (28, 10, 2048, 0, 0, 1, 1_000_000_000,
           "BASELINE configs[4] shape: sequenceType=1, one synthetic long record of {gb} per GPU (60-col lines, "
           "100 x 10 kbp N runs, 5% soft-masked)"),
}


def workload_label(wl: str, fasta_bytes: int) -> str:
    """config.workload: the workload's description with the FASTA bytes per GPU actually run (a run
    below the configuration's per-GPU load says so)."""
    desc, default = WORKLOADS[wl][7], WORKLOADS[wl][6]
    label = desc.format(gb=f"{fasta_bytes / 1e9:.3g} GB")
    if fasta_bytes < 0.99 * default:
        label += f" -- REDUCED: the configuration's per-GPU load is {default / 1e9:.3g} GB"
    return label


def cpu_baseline(sample_bytes: int, k: int, m: int, B: int, read_len: int, genome: int) -> dict:
    """The C restatement of the reference (oracle/) on a bounded sample of the
    same synthetic workload: one thread, 4 threads (the reference's Spark
    local[4], LocalTestKmerCounter.scala:62) and every core of this process's
    CPU share (at most 16, the GPU box's share).  `value` is the all-core rate."""
    import oracle
    n_reads = sample_bytes // (read_len + 14)
    data = fk.synth_fasta(n_reads, read_len, genome, seed=SEED)
    bases = n_reads * read_len
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    rates, secs = {}, {}
    for t in sorted({1, 4, cores}):
        t0 = time.perf_counter()
        r = oracle.OracleResult(data, k, m, B, threads=t)
        secs[t] = time.perf_counter() - t0
        rates[t] = bases / secs[t]
    return {"value": rates[cores], "unit": "bases/s", "cores": cores, "kind": "port",
            "value_1_thread": rates[1], "value_4_threads": rates[4],
            "sample": f"{n_reads} reads x {read_len} bp ({len(data) / 1e6:.0f} MB) of the bench workload, "
                      f"oracle/fk_oracle.c (fko_count_mt: record-aligned input splits, per-thread bins, "
                      f"bins merged and reduced in parallel) at 1/4/{cores} threads: "
                      f"{secs[1]:.1f}/{secs[4]:.1f}/{secs[cores]:.1f} s, {r.total_kmers} k-mers"}


def long_sequence_fasta(n_bases: int, seed: int = SEED) -> bytes:
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
    rocprofv3 PMC summary (profiles/pmc_summary.json), if it holds that kernel
    at this FASTA size."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    if d.get("stage_kernel") != kernel:
        return None
    return d.get("encode_signature_hbm_bytes_per_launch")


class Rank:
    """One rank's context and its shard (pinned host copy and device copy)."""

    def __init__(self, args, wl, rank: int, world: int, device: int):
        k, m, B, read_len, genome, seq_type, _, _ = WORKLOADS[wl]
        self.k, self.m, self.B, self.read_len, self.genome, self.seq_type = k, m, B, read_len, genome, seq_type
        self.rank, self.world, self.device = rank, world, device
        self.dev = torch.device("cuda", device)
        self.kc = fk.KmerCounter(k, m, 3, B, use_ht=args.use_ht, sequence_type=seq_type, n_ranks=world, rank=rank,
                                 device=device)
        if seq_type == 1:
            n_bases = args.bytes_per_gpu * 60 // 61
            data = long_sequence_fasta(n_bases, seed=SEED + rank)
            self.fasta_bytes, self.bases = len(data), n_bases
            import numpy as np
            self.host = torch.empty(self.fasta_bytes, dtype=torch.uint8, pin_memory=True)
            self.host.numpy()[:] = np.frombuffer(data, dtype=np.uint8)
            del data
            self.dev_in = self.host.to(self.dev)
        else:
            rec_bytes = read_len + 14
            n_reads = args.bytes_per_gpu // rec_bytes
            self.fasta_bytes, self.bases = n_reads * rec_bytes, n_reads * read_len
            self.dev_in = torch.empty(self.fasta_bytes, dtype=torch.uint8, device=self.dev)
            with torch.cuda.device(self.dev):
                fk.synth_fasta_to_device(self.dev_in.data_ptr(), n_reads, read_len, genome, seed=SEED,
                                         first_read=rank * n_reads)
            self.host = torch.empty(self.fasta_bytes, dtype=torch.uint8, pin_memory=True)
            self.host.copy_(self.dev_in)
        torch.cuda.synchronize(self.dev)
        if args.no_device_leg:  # the HBM-resident copy only feeds that leg
            self.dev_in = None
            torch.cuda.empty_cache()

    def step_host(self):
        self.kc.ingest_ptr(self.host.data_ptr(), self.fasta_bytes)
        self.kc.finish()

    def step_device(self):
        self.kc.ingest_device(self.dev_in.data_ptr(), self.fasta_bytes)
        self.kc.finish()


def exchange_figures(st: dict, world: int) -> dict:
    """Per-rank exchange figures from the context's stats (fk_stats.xch_*)."""
    out = {"steps": st["xch_steps"], "bytes_sent": st["xch_bytes_sent"], "bytes_received": st["xch_bytes_received"],
           "ms_transfers": st["ms_exchange"], "ms_tail": st["ms_exchange_tail"]}
    if st["ms_exchange"] > 0 and world > 1:
        egress = st["xch_bytes_sent"] / (st["ms_exchange"] * 1e-3)
        out["egress_GBps"] = egress / 1e9
        out["per_link_GBps"] = egress / (world - 1) / 1e9
        out["per_link_frac_of_peak_one_direction"] = egress / (world - 1) / (XGMI_LINK_PEAK / 2)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--bytes-per-gpu", type=int, default=0, help="FASTA bytes per GPU (0: the workload's)")
    ap.add_argument("--cpu-sample-bytes", type=int, default=160_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-device-leg", action="store_true", help="skip the HBM-resident leg (no roofline)")
    ap.add_argument("--device-leg", action="store_true",
                    help="run the HBM-resident leg with N > 1 or > 2 GB per GPU too (default: N = 1 at <= 2 GB "
                         "only; a 6.25 GB shard would hold both legs' buffers on its GPU at once)")
    ap.add_argument("--use-ht", action="store_true", help="hash count (extractKXmersHT, useHT=1)")
    ap.add_argument("--workload", default="", choices=["", "c2", "c3", "c4", "c5"],
                    help="c2 = BASELINE configs[1] (default at N = 1); c3 = configs[2] (default at N > 1); "
                         "c4 = configs[3] (k=55 m=12, two-word keys); c5 = configs[4] shape (one long record)")
    ap.add_argument("--rehearse-local", type=int, default=0,
                    help="N ranks as threads of this process on GPU 0 (in-process transport), a rehearsal "
                         "of the N-GPU job on one card")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local = args.rehearse_local
    if local and world > 1:
        raise SystemExit("--rehearse-local runs in one process")
    n_ranks = local or world
    wl = args.workload or ("c2" if n_ranks == 1 else "c3")
    if not args.bytes_per_gpu:
        args.bytes_per_gpu = WORKLOADS[wl][6]
    # the roofline leg is the N = 1 line's, at its 1 GB; a 6.25 GB shard (configs[2] / [3] per GPU)
    # would hold both legs' buffers on its GPU at once (k = 55: ~57 GB per k-mer array)
    if (n_ranks > 1 or args.bytes_per_gpu > 2_000_000_000) and not args.device_leg:
        args.no_device_leg = True
    distributed = world > 1
    torch.cuda.set_device(0 if local else local_rank)
    if distributed:
        dist.init_process_group("gloo")  # bootstrap + host barriers; the records move over RCCL in the library

    if local:
        ranks = [Rank(args, wl, r, local, 0) for r in range(local)]
        fk.comm_init_local([r.kc for r in ranks])
    else:
        ranks = [Rank(args, wl, rank, world, local_rank)]
        if distributed:
            uid = [fk.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            ranks[0].kc.comm_init(uid[0])

    def run(step_name):
        if len(ranks) == 1:
            getattr(ranks[0], step_name)()
            return
        errs = [None] * len(ranks)

        def work(i):
            try:
                getattr(ranks[i], step_name)()
            except Exception as e:  # noqa: BLE001
                errs[i] = e
        th = [threading.Thread(target=work, args=(i,)) for i in range(len(ranks))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for e in errs:
            if e is not None:
                raise e

    def barrier_sync():
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(v: float) -> float:
        if not distributed:
            return v
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def timed(step_name, steps, warmup):
        for _ in range(warmup):
            run(step_name)
        barrier_sync()
        per, t0 = [], time.perf_counter()
        for _ in range(steps):
            run(step_name)
            per.append([r.kc.stats() for r in ranks])
        barrier_sync()
        return max_over_ranks(time.perf_counter() - t0), per

    # leg 1 (SURVEY 8d's timer, the headline): FASTA in pinned host memory -> counts on the device
    elapsed, host_stats = timed("step_host", args.steps, args.warmup)
    if os.environ.get("FASTKMER_BENCH_MEMINFO"):  # device memory left after the host-input leg
        free_b, total_b = torch.cuda.mem_get_info()
        st0 = host_stats[-1][0]
        print(f"meminfo: {free_b / 1e9:.1f} GB free of {total_b / 1e9:.1f} GB after the host-input leg; "
              f"buckets {st0['buckets']}, oversize {st0['oversize_buckets']}, fine bits {st0['fine_bits']}",
              file=sys.stderr, flush=True)
    host_sizes = [r.kc.bin_sizes() for r in ranks]
    for r, s in zip(ranks, host_sizes):
        assert int(s.sum()) == host_stats[-1][ranks.index(r)]["distinct"] > 0
    # leg 2: FASTA resident in HBM; the encode+signature kernel's roofline
    dev_elapsed, dev_stats = None, None
    if not args.no_device_leg:
        dev_elapsed, dev_stats = timed("step_device", args.steps, args.warmup)
        for r, s in zip(ranks, host_sizes):  # size-independent self-check: both legs counted the same shard
            assert (r.kc.bin_sizes() == s).all()

    if rank == 0:
        r0 = ranks[0]
        k, m, B, read_len, genome, seq_type, _, desc = WORKLOADS[wl]
        bases_all = sum(r.bases for r in ranks) * (world if distributed else 1)
        hs = host_stats[-1][0]
        metric = "input bases/sec (whole node), k=28 short reads, 1/2/4/8 GPUs"
        if wl not in ("c2", "c3"):
            metric += f" [{wl} workload, not the headline configuration]"
        if args.use_ht:
            metric += " [useHT=1: hash count]"
        par = (f"bins round-robin (bin % {n_ranks}) over {n_ranks} GPUs, records exchanged by the library "
               f"({r0.kc.comm_transport} transport)" if n_ranks > 1 else "one GPU")
        if local:
            par += f" -- REHEARSAL: {local} ranks as threads on one GPU"
        out = {
            "metric": metric,
            "value": bases_all * args.steps / elapsed,
            "unit": "bases/s",
            "n_gpus": 1 if local else world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64" if k <= 32 else "u128",
            "data": ("synthetic %d bp reads (%d Mbp virtual genome, 0.2%% subst, 0.05%% N), generated on the device "
                     "and staged to pinned host memory before timing" % (read_len, genome // 1_000_000)
                     if seq_type == 0 else "synthetic long record (host-generated, pinned host memory)"),
            "timed_region": "FASTA in pinned host memory -> H2D (segments on a copy stream, the fused map on every "
                            "landed tile; N > 1: every landed piece exchanged over RCCL while the next is copied) -> "
                            "count -> counts resident on the device (write=0)",
            "config": {"workload": workload_label(wl, r0.fasta_bytes), "k": k, "m": m, "x": 3, "B": B, "useHT": int(args.use_ht),
                       "sequenceType": seq_type, "fasta_bytes_per_gpu": r0.fasta_bytes, "bases_per_gpu": r0.bases,
                       "parallelism": par},
            "stages_ms": {"h2d": hs["ms_h2d"], "map_overlapped_with_h2d": hs["ms_signature"],
                          "partition": hs["ms_partition"], "count": hs["ms_count"]},
            "pcie_h2d_GBps": r0.fasta_bytes / (hs["ms_h2d"] * 1e-3) / 1e9 if hs["ms_h2d"] else None,
            "kmers_per_gpu": hs["kmers"], "distinct_rank0": hs["distinct"],
            "buckets_rank0": {"all": hs["buckets"], "above_wave_tier": hs["block_buckets"], "above_2048_keys": hs["big_buckets"],
                              "large_path": hs["oversize_buckets"], "cell_bits": hs["fine_bits"]},
        }
        if n_ranks > 1:
            out["exchange"] = exchange_figures(hs, n_ranks)
        if dev_stats is not None:
            ds = dev_stats[-1][0]
            out["device_resident_value"] = bases_all * args.steps / dev_elapsed
            out["device_resident_ms_per_step"] = dev_elapsed / args.steps * 1e3
            out["device_resident_stages_ms"] = {"map": ds["ms_signature"] + ds["ms_parse"],
                                                "partition": ds["ms_partition"], "count": ds["ms_count"]}
            if n_ranks > 1:
                out["device_resident_exchange"] = exchange_figures(ds, n_ranks)
            fused = all(s[0]["fused_map"] for s in dev_stats)
            # encode+signature stage: algorithmic bytes = FASTA bytes read per launch,
            # time = the fused kernel's HIP-event duration on its stream (two kernels when not fused)
            t_k = sum(s[0]["ms_signature_kernel"] + s[0]["ms_encode_kernel"] for s in dev_stats) / len(dev_stats) * 1e-3
            kname = ("k_map_fused" if fused else "k_fasta_parse + k_superkmers")
            achieved = r0.fasta_bytes / t_k
            out["roofline"] = {"bound": "hbm", "kernel": kname + " (encode + signature: FASTA bytes -> records)",
                               "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                               "frac": achieved / HBM_PEAK,
                               "traffic": load_traffic(kname) if r0.fasta_bytes == 999_999_906 else None,
                               "bytes_alg_per_launch": r0.fasta_bytes, "ms_per_launch": t_k * 1e3,
                               "measured": "HIP events around each launch on the context's map stream "
                                           "(HBM-resident leg)",
                               "note": "priced against HBM for the contract; the measured limiter is VALU "
                                       "issue (about 6.5e8 wave64 VALU instructions per GB at about 3.7 "
                                       "cycles each per SIMD, profiles/r04b_pmc_split_map.txt)"}
        if n_ranks == 1 and not args.no_cpu_baseline and wl == "c2":
            out["cpu_baseline"] = cpu_baseline(args.cpu_sample_bytes, k, m, B, read_len, genome)
        print(json.dumps(out), flush=True)
    for r in ranks:
        r.kc.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
