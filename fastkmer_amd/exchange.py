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
    host = dist.get_backend(group) == "gloo"
    ev = None if host else (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    if ev:
        ev[0].record()
    recv, recv_counts = exchange_records(send, send_counts, rb, group)
    if ev:
        ev[1].record()
    torch.cuda.synchronize(dev)
    rank = dist.get_rank(group)
    counter.last_exchange = {"rounds": 1, "bytes_sent": [(total - send_counts[rank]) * rb],
                             "bytes_received": [(sum(recv_counts) - recv_counts[rank]) * rb],
                             "a2a_ms": [ev[0].elapsed_time(ev[1]) if ev else None]}
    counter.reduce(recv.data_ptr(), sum(recv_counts))
    return sum(recv_counts)


def default_rounds(world: int) -> int:
    """Exchange rounds per step: the all-to-all of round r+1 overlaps the count
    of round r.  With few ranks each peer link carries a large share of the
    records (N = 2: half of them over one link), so more rounds hide more of
    the exchange; each extra round costs ~0.3 ms of per-reduce overhead."""
    return 1 if world <= 1 else (4 if world <= 4 else 2)


class RoundCounters:
    """One rank's bins counted in R exchange rounds.

    R KmerCounter contexts act as virtual ranks rank + world * r of
    world * R: virtual rank v owns the bins b with b % (world * R) == v, so
    physical rank (b % world) owns the same bins as the one-round placement
    and the per-bin results are identical.  parts[0] holds the input and
    maps it; its emitted send buffer is grouped by virtual destination
    (round-major), so round r's records for all ranks are one contiguous
    block.  The result accessors merge the parts.
    """

    def __init__(self, k, m, x=3, B=2048, use_ht=False, sequence_type=0, world=1, rank=0, rounds=1, device=-1):
        import fastkmer_amd as fk
        self.world, self.rank, self.rounds = world, rank, rounds
        self.parts = [fk.KmerCounter(k, m, x, B, use_ht, sequence_type, n_ranks=world * rounds,
                                     rank=rank + world * r, device=device) for r in range(rounds)]
        # one HIP stream for all R contexts (their work is sequential): with the
        # RCCL stream and torch's default stream that stays within the 4
        # hardware queues per process, so the count of round r does not
        # share a queue with the all-to-all of round r+1
        self._stream = torch.cuda.Stream(device=device if device >= 0 else None)
        for p in self.parts:
            p.set_stream(self._stream.cuda_stream)
        p0 = self.parts[0]
        # the sender groups its records by (virtual destination, local bin), so
        # the receiving contexts skip their partition pass (fk_reduce_grouped)
        self.parts_per_rank = p0.set_grouped_emit(True)
        self.k, self.num_bins, self.record_bytes, self.use_ht = p0.k, p0.num_bins, p0.record_bytes, p0.use_ht

    def __getattr__(self, name):  # input side (ingest, synth_device, map, ...) is parts[0]'s
        if name in ("ingest", "ingest_ptr", "ingest_device", "synth_device", "map", "map_emit", "set_stream"):
            return getattr(self.parts[0], name)
        raise AttributeError(name)

    def _part_of(self, b: int):
        return self.parts[(b % (self.world * self.rounds)) // self.world]

    def bin_sizes(self):
        out = self.parts[0].bin_sizes()
        for p in self.parts[1:]:
            out = out + p.bin_sizes()
        return out

    def get_bin(self, b: int):
        return self._part_of(b).get_bin(b)

    def bin_dict(self, b: int) -> dict:
        return self._part_of(b).bin_dict(b)

    def bin_text(self, b: int) -> str:
        return self._part_of(b).bin_text(b)

    def write_bins(self, out_dir: str) -> None:
        for p in self.parts:
            p.write_bins(out_dir)

    def stats(self) -> dict:
        st = dict(self.parts[0].stats())
        for p in self.parts[1:]:
            q = p.stats()
            for key in ("records_received", "distinct", "oversize_buckets", "buckets", "ms_partition", "ms_count"):
                st[key] += q[key]
        return st

    def close(self) -> None:
        for p in self.parts:
            p.close()
        self._stream = None


def count_distributed_rounds(rc: RoundCounters, group=None, device=None) -> int:
    """map -> R overlapped all-to-all rounds -> R reduces for one rank.

    All rounds are posted at once (async); the reduce of round r starts as
    soon as its records have arrived, while the later rounds are still on the
    wire.  Returns the number of records received.
    """
    world, R = rc.world, rc.rounds
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    host = dist.get_backend(group) == "gloo"
    wire = torch.device("cpu") if host else dev
    import numpy as np
    p0 = rc.parts[0]
    send_counts = p0.map()  # world * R virtual destinations, round-major
    prec, pkm = p0.map_part_counts()  # [world * R, parts]: records / k-mers per (destination, local bin)
    parts = prec.shape[1]
    total = sum(send_counts)
    rb = p0.record_bytes
    send = torch.empty(max(total, 1) * rb, dtype=torch.uint8, device=dev)
    p0.map_emit(send.data_ptr(), max(total, 1))
    send = send[: total * rb]
    payload = send.cpu() if host else send
    # per-part counts: rank d receives the rows of virtual ranks r * world + d, every round r
    tab = np.stack([prec, pkm], axis=1).astype(np.int64).reshape(R, world, 2, parts).transpose(1, 0, 2, 3)
    sc = torch.from_numpy(np.ascontiguousarray(tab)).reshape(-1).to(wire)
    rcv = torch.empty_like(sc)
    dist.all_to_all_single(rcv, sc, group=group)
    rt = rcv.cpu().numpy().reshape(world, R, 2, parts)  # [source][round][records | k-mers][local bin]
    recv_counts = [[int(rt[src, r, 0].sum()) for src in range(world)] for r in range(R)]  # [round][source]
    me = dist.get_rank(group)
    works, recvs, off = [], [], 0
    t_post = None if host else torch.cuda.Event(enable_timing=True)
    if t_post is not None:
        t_post.record()
    sent, received = [], []
    for r in range(R):
        ins = [send_counts[r * world + d] * rb for d in range(world)]
        outs = [c * rb for c in recv_counts[r]]
        recv = torch.empty(sum(outs), dtype=torch.uint8, device=wire)
        works.append(dist.all_to_all_single(recv, payload[off:off + sum(ins)], output_split_sizes=outs,
                                            input_split_sizes=ins, group=group, async_op=True))
        recvs.append(recv)
        sent.append(sum(ins) - ins[me])
        received.append(sum(outs) - outs[me])
        off += sum(ins)
    n, done = 0, []
    for r in range(R):
        works[r].wait()  # nccl: the current stream waits for round r (the host does not block)
        recv = recvs[r].to(dev) if host else recvs[r]
        if not host:
            # round r's records have landed once the current stream reaches this
            # event; the count stream waits on it on the device, not the host
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            rc._stream.wait_event(ev)
            done.append(ev)
        rc.parts[r].reduce_grouped(recv.data_ptr(), sum(recv_counts[r]), rt[:, r, 0, :], rt[:, r, 1, :])
        n += sum(recv_counts[r])
    rc.last_exchange = {"rounds": R, "bytes_sent": sent, "bytes_received": received,
                        "a2a_ms": [t_post.elapsed_time(e) for e in done] if done else [None] * R}
    return n


def execute_job_distributed(configuration, group=None, device=None, rounds=None):
    """SparkBinKmerCounter.executeJob (SBKC:989-1046) for one rank of a job.

    Every rank reads only its shard of the dataset with positioned reads
    (fastkmer_amd.sharding.read_shard: its ~size/world bytes plus the k - 1
    positions after them, FASTdoop's split, SBKC:1009-1012), maps, exchanges records with the other ranks and counts the bins it owns
    (bin % world == rank); with ``configuration.write`` each rank writes its
    own ``bin<b>`` files into the shared output directory, as the Spark
    executors do.  The exchange runs in ``rounds`` overlapped rounds
    (default_rounds; the size-aware placement uses one).  Returns the rank's
    counter (a KmerCounter, or a RoundCounters for R > 1).
    """
    import fastkmer_amd as fk
    from fastkmer_amd.sharding import read_shard

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    piece = read_shard(configuration.dataset, world, rank, configuration.k).piece
    R = 1 if configuration.useCustomPartitioner else (default_rounds(world) if rounds is None else rounds)
    args = (configuration.k, configuration.m, configuration.x, configuration.max_b, configuration.useHT,
            configuration.sequenceType)
    if R > 1:
        kc = RoundCounters(*args, world=world, rank=rank, rounds=R,
                           device=dev.index if dev.index is not None else -1)
        kc.ingest(piece)
        count_distributed_rounds(kc, group=group, device=dev)
    else:
        kc = fk.KmerCounter(*args, n_ranks=world, rank=rank, device=dev.index if dev.index is not None else -1)
        kc.ingest(piece)
        count_distributed(kc, group=group, device=dev, balance=configuration.useCustomPartitioner)
    if configuration.write:
        kc.write_bins(configuration.outputDir)
    return kc


SIG_DENSE_MAX = (1 << 24) + 1  # m <= 12: the dense signature counts are all-reduced whole


def execute_find_bin_signatures_job_distributed(configuration, group=None, device=None):
    """executeFindBinSignaturesJob (SBKC:956-986) for one rank of a job.

    Each rank counts the signatures of its shard (getBinSignatures, SBKC:772-917),
    one all-reduce of the 4^m + 1 counts merges them (the reduceByKey of
    SBKC:984), and each rank writes the ``bin_signatures<b>.txt`` of the bins it
    owns.  Short reads (sequenceType 0) are dealt as whole records
    (sharding.read_record_shard), so the merged counts are the whole file's; a
    long sequence (sequenceType 1) is cut between ranks with the k - 1 overlap
    (sharding.read_shard), and a super-k-mer over a cut counts once per side, as
    over the reference's input splits: the merged counts then depend on the number
    of ranks (they equal the sum of every rank's own signature counts of its piece,
    tests/test_distributed.py pins that), as the reference's depend on its HDFS
    splits.  Returns the merged counts (device tensor)."""
    import fastkmer_amd as fk
    from fastkmer_amd.sharding import read_record_shard, read_shard

    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    if configuration.sequenceType == 0:
        piece = read_record_shard(configuration.dataset, world, rank)
    else:
        piece = read_shard(configuration.dataset, world, rank, configuration.k).piece
    with fk.KmerCounter(configuration.k, configuration.m, configuration.x, configuration.max_b,
                        configuration.useHT, configuration.sequenceType, n_ranks=world, rank=rank,
                        device=dev.index if dev.index is not None else -1) as kc:
        kc.ingest(piece)
        counts = kc.signature_counts()
        if counts.numel() > SIG_DENSE_MAX:
            # large m (4^m + 1 slots up to 8.6 GB at m = 15): only the signatures that occur travel,
            # as the reference's reduceByKey only ever holds those
            idx = torch.nonzero(counts).flatten()
            mine = (idx.cpu(), counts[idx].cpu())
            parts = [None] * world
            dist.all_gather_object(parts, mine, group=group)
            counts.zero_()
            for i, v in parts:
                counts.index_add_(0, i.to(counts.device), v.to(counts.device))
        elif dist.get_backend(group) == "gloo":
            host = counts.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
            counts.copy_(host)
        else:
            dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
        torch.cuda.synchronize(dev)
        kc.write_bin_signatures(counts, configuration.outputDir)
    return counts
