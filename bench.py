"""Benchmark: exact canonical k-mer counting throughput on MI355X.

Metric (BASELINE.json): input bases/sec for the whole node, k=28 short reads,
1/2/4/8 GPUs, counts bit-exact.  Synthetic ">r%010d" 100 bp reads, 0.2%
substitutions, 0.05% N.

`value` is weak-scaled: every rank runs the same per-GPU job at every N, so
the driver's 1 -> N ratio compares like with like.  The default job is
BASELINE configs[1]'s: k=28 m=10 x=3 B=2048, 1 GB of FASTA per GPU from a
100 Mbp virtual genome (--workload picks another).  Beside it the line carries
`configs2_per_gpu`: configs[2]'s per-GPU load, k=28 m=10 x=3 B=8192, 6.25 GB
per GPU from a 3 Gbp virtual genome (at N = 8: the 50 GB job), also at every N.

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
events around its one launch, on the stream it runs on).  That leg runs at
N = 1 and <= 2 GB per GPU unless --device-leg asks for it.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
          N > 1 without a launcher: bench.py starts N worker processes itself (one per GPU,
          RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 in their environment) before any
          GPU call, and fails if fewer than N GPUs are visible; --dry-run prints that plan.
        torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
          (one process per GPU; --gpus must equal WORLD_SIZE; the RCCL unique id travels over
          torch.distributed's gloo group)
        python bench.py --rehearse-local N [--bytes-per-gpu B]   (N ranks as threads of one
          process on one GPU: the whole native N > 1 path with the in-process transport)
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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
    """One rank's context and its shard (pinned host copy and, for the HBM-resident leg, a device copy)."""

    def __init__(self, wl: str, nbytes: int, use_ht: bool, device_leg: bool, rank: int, world: int, device: int):
        k, m, B, read_len, genome, seq_type, _, _ = WORKLOADS[wl]
        self.k, self.m, self.B, self.read_len, self.genome, self.seq_type = k, m, B, read_len, genome, seq_type
        self.rank, self.world, self.device = rank, world, device
        self.dev = torch.device("cuda", device)
        self.kc = fk.KmerCounter(k, m, 3, B, use_ht=use_ht, sequence_type=seq_type, n_ranks=world, rank=rank,
                                 device=device)
        if seq_type == 1:
            n_bases = nbytes * 60 // 61
            data = long_sequence_fasta(n_bases, seed=SEED + rank)
            self.fasta_bytes, self.bases = len(data), n_bases
            import numpy as np
            self.host = torch.empty(self.fasta_bytes, dtype=torch.uint8, pin_memory=True)
            self.host.numpy()[:] = np.frombuffer(data, dtype=np.uint8)
            del data
            self.dev_in = self.host.to(self.dev)
        else:
            rec_bytes = read_len + 14
            n_reads = nbytes // rec_bytes
            self.fasta_bytes, self.bases = n_reads * rec_bytes, n_reads * read_len
            self.dev_in = torch.empty(self.fasta_bytes, dtype=torch.uint8, device=self.dev)
            with torch.cuda.device(self.dev):
                fk.synth_fasta_to_device(self.dev_in.data_ptr(), n_reads, read_len, genome, seed=SEED,
                                         first_read=rank * n_reads)
            self.host = torch.empty(self.fasta_bytes, dtype=torch.uint8, pin_memory=True)
            self.host.copy_(self.dev_in)
        torch.cuda.synchronize(self.dev)
        if not device_leg:  # the HBM-resident copy only feeds that leg
            self.dev_in = None
            torch.cuda.empty_cache()

    def step_host(self):
        self.kc.ingest_ptr(self.host.data_ptr(), self.fasta_bytes)
        self.kc.finish()

    def step_device(self):
        self.kc.ingest_device(self.dev_in.data_ptr(), self.fasta_bytes)
        self.kc.finish()

    def close(self):
        self.kc.close()
        self.host = self.dev_in = None


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



KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"
VISIBILITY_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


def kfd_gpus(root: str | None = None) -> list[dict]:
    """The GPU nodes of the KFD topology (sysfs; properties with simd_count > 0), in node order.
    Reading sysfs initialises nothing: the launcher counts GPUs this way, never through HIP."""
    root = root or os.environ.get("FASTKMER_KFD_TOPOLOGY", KFD_TOPOLOGY)
    gpus = []
    try:
        nodes = sorted((d for d in os.listdir(root) if d.isdigit()), key=int)
    except OSError:
        return gpus
    for d in nodes:
        try:
            with open(os.path.join(root, d, "properties")) as f:
                props = dict(ln.split()[:2] for ln in f if len(ln.split()) >= 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0")) > 0:
            gpus.append(props)
    return gpus


def count_gpus(root: str | None = None) -> int:
    """GPUs this process may use: the KFD topology's GPU nodes, narrowed by a visibility mask
    (HIP_/ROCR_/CUDA_VISIBLE_DEVICES: its entries, at most the nodes present)."""
    n = len(kfd_gpus(root))
    for var in VISIBILITY_VARS:
        v = os.environ.get(var)
        if v:  # unset or empty: no mask
            n = min(n, len([e for e in v.split(",") if e.strip()]))
    return n


def pin_to_gpu_numa(local_rank: int):
    """Best effort, before any GPU call: restrict this rank's CPUs to the NUMA node of its GPU (KFD
    topology -> PCI address -> numa_node), so that its pinned host buffers -- first touched here --
    sit next to the GPU's PCIe link.  Returns the node, or None (no sysfs, a visibility mask that
    renumbers the devices, or any error: the affinity is left alone)."""
    if any(os.environ.get(v) for v in VISIBILITY_VARS):
        return None
    try:
        p = kfd_gpus()[local_rank]
        loc, dom = int(p["location_id"]), int(p.get("domain", "0"))
        bdf = f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 31:02x}.{loc & 7}"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            node = int(f.read())
        if node < 0:
            return None
        cpus = set()
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            for part in f.read().strip().split(","):
                lo, _, hi = part.partition("-")
                cpus.update(range(int(lo), int(hi or lo) + 1))
        cur = os.sched_getaffinity(0)
        want = cur & cpus
        if want and want != cur:
            os.sched_setaffinity(0, want)
        return node
    except Exception:  # noqa: BLE001 -- best effort
        return None


class Topology:
    """Where this process sits: one rank of a torch.distributed job (one process per GPU, RCCL
    between them), the only rank, or --rehearse-local N ranks as threads on GPU 0."""

    def __init__(self, args):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.local = args.rehearse_local
        self.distributed = self.world > 1
        self.n_ranks = self.local or self.world

    def barrier_sync(self):
        torch.cuda.synchronize()
        if self.distributed:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(self, v: float) -> float:
        if not self.distributed:
            return v
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())


def make_ranks(topo: Topology, wl: str, nbytes: int, use_ht: bool, device_leg: bool) -> list:
    if topo.local:
        ranks = [Rank(wl, nbytes, use_ht, device_leg, r, topo.local, 0) for r in range(topo.local)]
        fk.comm_init_local([r.kc for r in ranks])
        return ranks
    ranks = [Rank(wl, nbytes, use_ht, device_leg, topo.rank, topo.world, topo.local_rank)]
    if topo.distributed:
        uid = [fk.comm_unique_id() if topo.rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ranks[0].kc.comm_init(uid[0])
    return ranks


def run_step(ranks: list, step_name: str) -> None:
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


def timed(topo: Topology, ranks: list, step_name: str, steps: int, warmup: int):
    """W untimed steps, then exactly K steps between barrier + synchronize pairs; the max over ranks."""
    for _ in range(warmup):
        run_step(ranks, step_name)
    topo.barrier_sync()
    per, t0 = [], time.perf_counter()
    for _ in range(steps):
        run_step(ranks, step_name)
        per.append([r.kc.stats() for r in ranks])
    topo.barrier_sync()
    return topo.max_over_ranks(time.perf_counter() - t0), per


def run_leg(args, topo: Topology, wl: str, nbytes: int, device_leg: bool) -> dict:
    """One workload: the headline leg (pinned-host FASTA -> counts on the device) and, if asked, the
    HBM-resident leg with the encode+signature kernel's roofline.  Collective over the ranks."""
    ranks = make_ranks(topo, wl, nbytes, args.use_ht, device_leg)
    elapsed, host_stats = timed(topo, ranks, "step_host", args.steps, args.warmup)
    res = {"wl": wl, "elapsed": elapsed, "hs": host_stats[-1][0], "fasta_bytes": ranks[0].fasta_bytes,
           "bases_per_gpu": ranks[0].bases,
           "bases_all": sum(r.bases for r in ranks) * (topo.world if topo.distributed else 1),
           "transport": ranks[0].kc.comm_transport}
    if os.environ.get("FASTKMER_BENCH_MEMINFO"):  # device memory left after the host-input leg
        free_b, total_b = torch.cuda.mem_get_info()
        st0 = host_stats[-1][0]
        print(f"meminfo [{wl}]: {free_b / 1e9:.1f} GB free of {total_b / 1e9:.1f} GB after the host-input leg; "
              f"buckets {st0['buckets']}, oversize {st0['oversize_buckets']}, fine bits {st0['fine_bits']}",
              file=sys.stderr, flush=True)
    host_sizes = [r.kc.bin_sizes() for r in ranks]
    for i, s in enumerate(host_sizes):
        assert int(s.sum()) == host_stats[-1][i]["distinct"] > 0
    if device_leg:
        dev_elapsed, dev_stats = timed(topo, ranks, "step_device", args.steps, args.warmup)
        for r, s in zip(ranks, host_sizes):  # size-independent self-check: both legs counted the same shard
            assert (r.kc.bin_sizes() == s).all()
        res.update(dev_elapsed=dev_elapsed, dev_stats=dev_stats)
    for r in ranks:
        r.close()
    del ranks
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


def leg_line(args, topo: Topology, res: dict) -> dict:
    """The figures of one leg as they appear in the JSON line."""
    wl, hs = res["wl"], res["hs"]
    k, m, B, read_len, genome, seq_type, _, _ = WORKLOADS[wl]
    n = topo.n_ranks
    par = (f"bins round-robin (bin % {n}) over {n} GPUs, records exchanged by the library "
           f"({res['transport']} transport)" if n > 1 else "one GPU")
    if topo.local:
        par += f" -- REHEARSAL: {topo.local} ranks as threads on one GPU"
    out = {
        "value": res["bases_all"] * args.steps / res["elapsed"],
        "unit": "bases/s",
        "ms_per_step": res["elapsed"] / args.steps * 1e3,
        "config": {"workload": workload_label(wl, res["fasta_bytes"]), "k": k, "m": m, "x": 3, "B": B,
                   "useHT": int(args.use_ht), "sequenceType": seq_type, "fasta_bytes_per_gpu": res["fasta_bytes"],
                   "bases_per_gpu": res["bases_per_gpu"],
                   "parallelism": par},
        "stages_ms": {"h2d": hs["ms_h2d"], "map_overlapped_with_h2d": hs["ms_signature"],
                      "partition": hs["ms_partition"], "count": hs["ms_count"]},
        "pcie_h2d_GBps": res["fasta_bytes"] / (hs["ms_h2d"] * 1e-3) / 1e9 if hs["ms_h2d"] else None,
        "kmers_per_gpu": hs["kmers"], "distinct_rank0": hs["distinct"],
        "buckets_rank0": {"all": hs["buckets"], "above_wave_tier": hs["block_buckets"] + hs["big_buckets"],
                          "above_block_tier": hs["big_buckets"], "kmers_above_wave_tier": hs["heavy_keys"],
                          "split": hs["split_buckets"], "sub_buckets": hs["sub_buckets"],
                          "large_path": hs["oversize_buckets"], "cell_bits": hs["fine_bits"]},
    }
    if n > 1:
        out["exchange"] = exchange_figures(hs, n)
    return out


def roofline(args, topo: Topology, res: dict) -> dict:
    """The encode+signature kernel: algorithmic bytes = FASTA bytes read per launch,
    time = the fused kernel's HIP-event duration on the stream it runs on (HBM-resident leg)."""
    dev_stats = res["dev_stats"]
    fused = all(s[0]["fused_map"] for s in dev_stats)
    t_k = sum(s[0]["ms_signature_kernel"] + s[0]["ms_encode_kernel"] for s in dev_stats) / len(dev_stats) * 1e-3
    kname = "k_map_fused" if fused else "k_fasta_parse + k_superkmers"
    achieved = res["fasta_bytes"] / t_k
    return {"bound": "hbm", "kernel": kname + " (encode + signature: FASTA bytes -> records)",
            "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": achieved / HBM_PEAK,
            "traffic": load_traffic(kname) if res["fasta_bytes"] == 999_999_906 else None,
            "bytes_alg_per_launch": res["fasta_bytes"], "ms_per_launch": t_k * 1e3,
            "measured": "HIP events around each launch on the context's map stream (HBM-resident leg)",
            "note": "priced against HBM for the contract; the measured limiter is VALU issue (DESIGN.md 4)"}


# ---------------------------------------------------------------------------
# --gpus N without a launcher: one worker process per GPU, started before any GPU call
# ---------------------------------------------------------------------------

def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv: list) -> int:
    """`python bench.py --gpus N` (N > 1, no WORLD_SIZE in the environment): starts N copies of this
    script as ranks 0..N-1 of one torch.distributed job on this node (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR=127.0.0.1 / MASTER_PORT), the same environment torchrun gives them.  This process never
    touches the GPU (it only counts the devices); it waits for the workers and exits with the first
    failing worker's code, stopping the others."""
    n = args.gpus
    port = _free_port()
    cmd = [sys.executable, os.path.abspath(__file__)] + argv
    envs = []
    for r in range(n):
        e = dict(os.environ)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                 HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        envs.append(e)
    visible = count_gpus()  # sysfs only: the launcher never initialises HIP (its workers do)
    if args.dry_run:
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                "HSA_ENABLE_IPC_MODE_LEGACY")
        print(json.dumps({"launcher": "bench.py", "world_size": n, "visible_gpus": visible, "argv": cmd,
                          "ranks": [{k: e[k] for k in keys} for e in envs]}), flush=True)
        return 0
    if visible < n:
        print(f"bench.py --gpus {n}: only {visible} GPU(s) visible; an N-GPU run needs N GPUs of one node "
              f"(one rank per GPU)", file=sys.stderr, flush=True)
        return 2
    procs = [subprocess.Popen(cmd, env=e) for e in envs]
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    return rc


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node (one rank each).  Without WORLD_SIZE in the environment, N > 1 "
                         "starts the N ranks itself; under torchrun it must equal WORLD_SIZE")
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
                    help="the `value` workload at every N: c2 = BASELINE configs[1]'s per-GPU job (default); "
                         "c3 = configs[2]'s per-GPU load; c4 = configs[3] (k=55 m=12, two-word keys); "
                         "c5 = configs[4] shape (one long record)")
    ap.add_argument("--c3-leg", default="auto", choices=["auto", "on", "off"],
                    help="also run configs[2]'s per-GPU load (6.25 GB, B=8192; the 8-GPU 50 GB job at N = 8) "
                         "and report it as `configs2_per_gpu` (auto: on unless the value workload is c3 or "
                         "this is a --rehearse-local run)")
    ap.add_argument("--rehearse-local", type=int, default=0,
                    help="N ranks as threads of this process on GPU 0 (in-process transport), a rehearsal "
                         "of the N-GPU job on one card")
    ap.add_argument("--dry-run", action="store_true",
                    help="with --gpus N > 1: print the ranks' launch plan as JSON and exit (no GPU use)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus is not None and args.gpus > 1 and not args.rehearse_local:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    if args.gpus is not None and args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    topo = Topology(args)
    if args.gpus is not None and not args.rehearse_local and args.gpus != topo.world:
        print(f"bench.py --gpus {args.gpus} under a launcher with WORLD_SIZE={topo.world}: the two must agree",
              file=sys.stderr, flush=True)
        sys.exit(2)
    if topo.local and topo.world > 1:
        raise SystemExit("--rehearse-local runs in one process")
    if args.dry_run:
        raise SystemExit("--dry-run needs --gpus N > 1 without a launcher")
    wl = args.workload or "c2"
    nbytes = args.bytes_per_gpu or WORKLOADS[wl][6]
    # the roofline leg is the N = 1 line's, at its 1 GB; a 6.25 GB shard (configs[2] / [3] per GPU)
    # would hold both legs' buffers on its GPU at once (k = 55: ~57 GB per k-mer array)
    device_leg = not args.no_device_leg and (args.device_leg or (topo.n_ranks == 1 and nbytes <= 2_000_000_000))
    c3_leg = args.c3_leg == "on" or (args.c3_leg == "auto" and wl != "c3" and not topo.local)
    numa = pin_to_gpu_numa(topo.local_rank) if topo.distributed else None
    torch.cuda.set_device(0 if topo.local else topo.local_rank)
    if topo.distributed:
        dist.init_process_group("gloo")  # bootstrap + host barriers; the records move over RCCL in the library

    res = run_leg(args, topo, wl, nbytes, device_leg)
    res3 = run_leg(args, topo, "c3", WORKLOADS["c3"][6], False) if c3_leg else None

    if topo.rank == 0:
        k, m, B, read_len, genome, seq_type, _, _ = WORKLOADS[wl]
        metric = "input bases/sec (whole node), k=28 short reads, 1/2/4/8 GPUs"
        if wl not in ("c2", "c3"):
            metric += f" [{wl} workload, not the headline configuration]"
        if args.use_ht:
            metric += " [useHT=1: hash count]"
        line = leg_line(args, topo, res)
        out = {
            "metric": metric,
            "value": line.pop("value"),
            "unit": line.pop("unit"),
            "n_gpus": 1 if topo.local else topo.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": line.pop("ms_per_step"),
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
            "weak_scaling_unit": "the same per-GPU job at every N (config.workload); value = all ranks' bases / "
                                 "the slowest rank's time",
        }
        out.update(line)
        if "dev_stats" in res:
            ds = res["dev_stats"][-1][0]
            out["device_resident_value"] = res["bases_all"] * args.steps / res["dev_elapsed"]
            out["device_resident_ms_per_step"] = res["dev_elapsed"] / args.steps * 1e3
            out["device_resident_stages_ms"] = {"map": ds["ms_signature"] + ds["ms_parse"],
                                                "partition": ds["ms_partition"], "count": ds["ms_count"]}
            if topo.n_ranks > 1:
                out["device_resident_exchange"] = exchange_figures(ds, topo.n_ranks)
            out["roofline"] = roofline(args, topo, res)
        if res3 is not None:
            out["configs2_per_gpu"] = leg_line(args, topo, res3)
        if topo.distributed:
            out["numa_node_rank0"] = numa  # the node rank 0's CPUs were restricted to (None: left alone)
        if topo.n_ranks == 1 and not args.no_cpu_baseline and wl == "c2":
            out["cpu_baseline"] = cpu_baseline(args.cpu_sample_bytes, k, m, B, read_len, genome)
        print(json.dumps(out), flush=True)
    if topo.distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
