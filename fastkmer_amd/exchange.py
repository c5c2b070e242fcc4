"""Signature->bin shuffle across ranks (replaces Spark's reduceByKey, SBKC:1035).

One process per GPU.  Each rank packs its super-k-mer records grouped by
destination rank (bin % world, round-robin bin ownership) with
``fk_map_emit``; one ``all_to_all_single`` of per-destination record counts
and one ``all_to_all_single`` of the packed records (RCCL over xGMI with the
"nccl" backend, gloo on CPU tensors in tests) deliver every record to the rank
that owns its bin, which then runs ``fk_reduce``.  There is no other
collective on the data path.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def exchange_records(send: torch.Tensor, send_counts: list[int], record_bytes: int, group=None):
    """All-to-all of packed records.

    send: uint8 tensor holding sum(send_counts) records, grouped by destination
    rank (rank 0 first).  Returns (recv uint8 tensor, recv_counts list).
    """
    world = dist.get_world_size(group)
    assert len(send_counts) == world
    dev = send.device
    sc = torch.tensor(send_counts, dtype=torch.int64, device=dev)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = [int(v) for v in rc.cpu().tolist()]
    recv = torch.empty(sum(recv_counts) * record_bytes, dtype=torch.uint8, device=dev)
    dist.all_to_all_single(recv, send,
                           output_split_sizes=[c * record_bytes for c in recv_counts],
                           input_split_sizes=[c * record_bytes for c in send_counts], group=group)
    return recv, recv_counts


def count_distributed(counter, group=None, device=None):
    """map -> all-to-all -> reduce for one rank of a multi-GPU job.

    ``counter`` is a fastkmer_amd.KmerCounter created with n_ranks/rank and
    already holding its input shard.  Returns the number of records received.
    """
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    send_counts = counter.map()
    total = sum(send_counts)
    rb = counter.record_bytes
    send = torch.empty(max(total, 1) * rb, dtype=torch.uint8, device=dev)
    counter.map_emit(send.data_ptr(), max(total, 1))
    send = send[: total * rb]
    recv, recv_counts = exchange_records(send, send_counts, rb, group)
    torch.cuda.synchronize(dev)
    counter.reduce(recv.data_ptr(), sum(recv_counts))
    return sum(recv_counts)
