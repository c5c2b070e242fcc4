"""Signature->bin shuffle across ranks (replaces Spark's reduceByKey, SBKC:1035).

One process per GPU.  Each rank packs its super-k-mer records grouped by
destination rank (bin % world: bins are owned round-robin) with
``fk_map_emit``; one ``all_to_all_single`` of per-destination record counts
and one ``all_to_all_single`` of the packed records deliver every record to
the rank that owns its bin, which then runs ``fk_reduce``.  With the "nccl"
backend (RCCL over xGMI on MI355X) the records move GPU to GPU; with "gloo"
(CPU-only tests, or ranks sharing one GPU) they are staged through host
memory.  There is no other collective on the data path.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def owner_of_bin(b: int, world: int) -> int:
    """Rank that counts bin b under the default placement (round-robin)."""
    return b % world


def exchange_records(send: torch.Tensor, send_counts: list[int], record_bytes: int, group=None):
    """All-to-all of packed records.

    ``send`` is a uint8 tensor holding sum(send_counts) records grouped by
    destination rank (rank 0 first).  Returns (recv, recv_counts) on the same
    device as ``send``.  Works with "nccl" (device tensors) and "gloo" (host
    tensors; device tensors are staged through host memory).
    """
    world = dist.get_world_size(group)
    if len(send_counts) != world:
        raise ValueError(f"send_counts has {len(send_counts)} entries for {world} ranks")
    if send.numel() != sum(send_counts) * record_bytes:
        raise ValueError("send buffer size does not match send_counts")
    dev = send.device
    host = dist.get_backend(group) == "gloo"
    wire = torch.device("cpu") if host else dev
    payload = send.to(wire) if host else send
    sc = torch.tensor(send_counts, dtype=torch.int64, device=wire)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = [int(v) for v in rc.tolist()]
    recv = torch.empty(sum(recv_counts) * record_bytes, dtype=torch.uint8, device=wire)
    dist.all_to_all_single(recv, payload,
                           output_split_sizes=[c * record_bytes for c in recv_counts],
                           input_split_sizes=[c * record_bytes for c in send_counts], group=group)
    return (recv.to(dev) if host else recv), recv_counts


def balanced_owners(counter, group=None, device=None):
    """Size-aware placement (useCustomPartitioner, SBKC:1023-1025): exact k-mers
    per bin summed over the ranks (one all-reduce of b counts), then LPT
    (fastkmer_amd.lpt_owners).  Call after counter.map(); returns the owner table."""
    import fastkmer_amd as fk
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    host = dist.get_backend(group) == "gloo"
    sizes = torch.from_numpy(counter.map_bin_kmers().astype("int64"))
    sizes = sizes if host else sizes.to(dev)
    dist.all_reduce(sizes, op=dist.ReduceOp.SUM, group=group)
    return fk.lpt_owners(sizes.cpu().numpy().astype("uint64"), dist.get_world_size(group))


def count_distributed(counter, group=None, device=None, balance: bool = False):
    """map -> all-to-all -> reduce for one rank of a multi-GPU job.

    ``counter`` is a fastkmer_amd.KmerCounter created with n_ranks/rank and
    already holding its input shard.  balance=True places bins by size
    (balanced_owners) instead of bin % world.  Returns the number of records
    received.
    """
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    send_counts = counter.map()
    if balance:
        send_counts = counter.set_bin_owners(balanced_owners(counter, group, dev))
    total = sum(send_counts)
    rb = counter.record_bytes
    send = torch.empty(max(total, 1) * rb, dtype=torch.uint8, device=dev)
    counter.map_emit(send.data_ptr(), max(total, 1))
    send = send[: total * rb]
    recv, recv_counts = exchange_records(send, send_counts, rb, group)
    torch.cuda.synchronize(dev)
    counter.reduce(recv.data_ptr(), sum(recv_counts))
    return sum(recv_counts)


def execute_job_distributed(configuration, group=None, device=None):
    """SparkBinKmerCounter.executeJob (SBKC:989-1046) for one rank of a job.

    Every rank reads the dataset, keeps its shard (fastkmer_amd.sharding),
    maps, exchanges records with the other ranks and counts the bins it owns
    (bin % world == rank); with ``configuration.write`` each rank writes its
    own ``bin<b>`` files into the shared output directory, as the Spark
    executors do.  Returns the rank's KmerCounter.
    """
    import fastkmer_amd as fk
    from fastkmer_amd.sharding import shard_fasta

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    with open(configuration.dataset, "rb") as f:
        data = f.read()
    piece = shard_fasta(data, world, rank, configuration.sequenceType, configuration.k)
    del data
    kc = fk.KmerCounter(configuration.k, configuration.m, configuration.x, configuration.max_b,
                        configuration.useHT, configuration.sequenceType, n_ranks=world, rank=rank,
                        device=dev.index if dev.index is not None else -1)
    kc.ingest(piece)
    count_distributed(kc, group=group, device=dev, balance=configuration.useCustomPartitioner)
    if configuration.write:
        kc.write_bins(configuration.outputDir)
    return kc
