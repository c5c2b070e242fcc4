"""Multi-rank path: input sharding, the record all-to-all, and a whole
distributed job.

CPU tests (gloo, world_size 2-3) cover the host logic: shards partition the
input so that per-shard counts add up to the whole-input counts (checked
with the oracle), and exchange_records delivers every record to its owner.
The GPU test runs execute_job_distributed as two processes sharing one GPU
(gloo transport, records staged through host memory) and compares the bin
files with the oracle's.  The RCCL transport is the same code with device
tensors; it runs in bench.py --gpus N.
"""
from __future__ import annotations

import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import fastkmer_amd as fk
import oracle
from fastkmer_amd.exchange import exchange_records, owner_of_bin
from fastkmer_amd.sharding import record_shard_bounds, shard_fasta


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank: int, world: int, port: int, backend: str = "gloo") -> None:
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if backend == "nccl":  # RCCL over xGMI: one GPU per rank
        torch.cuda.set_device(rank)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)


def _long_fasta(n_blocks=8, seed=5) -> bytes:
    rng = random.Random(seed)
    seq = []
    for blk in range(n_blocks):
        s = "".join(rng.choice("ACGT") for _ in range(5_000))
        if blk % 3 == 1:
            s = s[:1000] + "N" * 300 + s[1300:]
        if blk % 4 == 2:
            s = s[:2000] + s[2000:2500].lower() + s[2500:]
        seq.append(s)
    seq = "".join(seq)
    return (">chrS\n" + "\n".join(seq[q:q + 60] for q in range(0, len(seq), 60)) + "\n").encode()


def _all_counts(res: "oracle.OracleResult") -> dict:
    out = {}
    for b in range(res.nbins):
        hi, lo, cnt = res.bin_arrays(b)
        for h, l, c in zip(hi.tolist(), lo.tolist(), cnt.tolist()):
            out[(h, l)] = out.get((h, l), 0) + c
    return out


# ---------------------------------------------------------------- sharding (CPU)

@pytest.mark.parametrize("world", [2, 3, 5])
def test_record_shards_partition_input(world):
    data = fk.synth_fasta(3000, 100, 50_000, seed=world)
    b = record_shard_bounds(data, world)
    assert b[0] == 0 and b[-1] == len(data) and b == sorted(b)
    pieces = [shard_fasta(data, world, r) for r in range(world)]
    assert b"".join(pieces) == data
    for p in pieces:
        assert p == b"" or p.startswith(b">")


@pytest.mark.parametrize("world", [2, 3])
def test_short_read_shard_counts_add_up(world):
    data = fk.synth_fasta(2000, 100, 30_000, seed=11)
    whole = _all_counts(oracle.OracleResult(data, 28, 10, 2048))
    summed: dict = {}
    for r in range(world):
        for key, c in _all_counts(oracle.OracleResult(shard_fasta(data, world, r), 28, 10, 2048)).items():
            summed[key] = summed.get(key, 0) + c
    assert summed == whole


@pytest.mark.parametrize("world,k", [(2, 28), (3, 21), (4, 55)])
def test_long_sequence_shard_counts_add_up(world, k):
    data = _long_fasta()
    whole = _all_counts(oracle.OracleResult(data, k, 9, 256, 1))
    summed: dict = {}
    for r in range(world):
        piece = shard_fasta(data, world, r, sequence_type=1, k=k)
        assert piece.startswith(b">chrS\n")
        for key, c in _all_counts(oracle.OracleResult(piece, k, 9, 256, 1)).items():
            summed[key] = summed.get(key, 0) + c
    assert summed == whole


def test_shard_degenerate_inputs():
    assert shard_fasta(b"", 2, 1) == b""
    assert shard_fasta(b">a\n", 2, 0, sequence_type=1) == b""
    assert shard_fasta(b"ACGT\n", 2, 0, sequence_type=1) == b""
    with pytest.raises(ValueError):
        shard_fasta(b">a\nACGT\n", 2, 2)


def test_owner_of_bin_round_robin():
    assert [owner_of_bin(b, 3) for b in range(7)] == [0, 1, 2, 0, 1, 2, 0]


# ---------------------------------------------------------------- exchange (CPU, gloo)

def _exchange_worker(rank, world, port, rb):
    _init(rank, world, port)
    try:
        g = torch.Generator().manual_seed(100 + rank)
        counts = [int(torch.randint(0, 50, (1,), generator=g)) for _ in range(world)]
        counts[(rank + 1) % world] = 0  # an empty split
        send = torch.randint(0, 256, (sum(counts) * rb,), dtype=torch.uint8, generator=g)
        recv, rcounts = exchange_records(send, counts, rb)
        # rebuild every rank's send buffer deterministically and check our slices
        off = 0
        for src in range(world):
            gs = torch.Generator().manual_seed(100 + src)
            sc = [int(torch.randint(0, 50, (1,), generator=gs)) for _ in range(world)]
            sc[(src + 1) % world] = 0
            ssend = torch.randint(0, 256, (sum(sc) * rb,), dtype=torch.uint8, generator=gs)
            assert rcounts[src] == sc[rank]
            lo = sum(sc[:rank]) * rb
            assert torch.equal(recv[off:off + sc[rank] * rb], ssend[lo:lo + sc[rank] * rb])
            off += sc[rank] * rb
        assert off == recv.numel()
        with pytest.raises(ValueError):
            exchange_records(send, counts[:-1], rb)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,rb", [(2, 16), (3, 24)])
def test_exchange_records_gloo(world, rb):
    mp.spawn(_exchange_worker, args=(world, _free_port(), rb), nprocs=world, join=True)


# ---------------------------------------------------------------- whole job (GPU)

def _job_worker(rank, world, port, cfg_kw, rounds=None, backend="gloo"):
    _init(rank, world, port, backend)
    try:
        from fastkmer_amd.exchange import execute_job_distributed
        gpu = rank if backend == "nccl" else 0
        torch.cuda.set_device(gpu)
        kc = execute_job_distributed(fk.TestConfiguration(**cfg_kw), device=torch.device("cuda", gpu), rounds=rounds)
        sizes = kc.bin_sizes()
        if not cfg_kw.get("useCustomPartitioner"):
            assert all(sizes[b] == 0 for b in range(kc.num_bins) if b % world != rank)
        kc.close()
    finally:
        dist.destroy_process_group()


def _read_bins(d: str) -> dict:
    out = {}
    for name in os.listdir(d):
        with open(os.path.join(d, name), "rb") as f:
            out[name] = f.read()
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("use_ht,seq_type,custom,rounds", [(False, 0, False, 1), (False, 0, False, 3),
                                                           (True, 0, False, None), (False, 1, False, None),
                                                           (False, 0, True, None)])
def test_execute_job_distributed_two_ranks(tmp_path, use_ht, seq_type, custom, rounds):
    k, m, B = 28, 10, 512
    data = _long_fasta(40) if seq_type == 1 else fk.synth_fasta(20_000, 100, 200_000, seed=21)
    path = tmp_path / "in.fa"
    path.write_bytes(data)
    cfg = dict(dataset=str(path), outputDirectory=str(tmp_path / "out") + "/", k=k, m=m, x=3, max_b=B,
               sequenceType=seq_type, useHT=use_ht, write=True, useCustomPartitioner=custom)
    mp.spawn(_job_worker, args=(2, _free_port(), cfg, rounds), nprocs=2, join=True)
    got = _read_bins(fk.TestConfiguration(**cfg).outputDir)
    ref_dir = tmp_path / "ref"
    oracle.OracleResult(data, k, m, B, seq_type).write_bins(str(ref_dir), sorted_eof=not use_ht)
    want = _read_bins(str(ref_dir))
    assert sorted(got) == sorted(want)
    for name in want:
        if use_ht:  # table order: compare as multisets of lines
            g = got[name].split(b"\n")
            w = want[name].split(b"\n")
            assert sorted(x for x in g if x) == sorted(x for x in w if x)
        else:
            assert got[name] == want[name]


@pytest.mark.gpu
@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="RCCL all-to-all needs two GPUs")
@pytest.mark.parametrize("use_ht,rounds", [(False, 1), (False, 2), (True, None)])
def test_execute_job_distributed_rccl(tmp_path, use_ht, rounds):
    """The RCCL transport (torch.distributed "nccl" = RCCL over xGMI): device
    tensors all the way, one GPU per rank; bin files byte-compared with the
    oracle's (the reduceByKey shuffle of SBKC:1034-1042)."""
    k, m, B = 28, 10, 2048
    data = fk.synth_fasta(40_000, 100, 400_000, seed=23)
    path = tmp_path / "in.fa"
    path.write_bytes(data)
    cfg = dict(dataset=str(path), outputDirectory=str(tmp_path / "out") + "/", k=k, m=m, x=3, max_b=B,
               sequenceType=0, useHT=use_ht, write=True)
    mp.spawn(_job_worker, args=(2, _free_port(), cfg, rounds, "nccl"), nprocs=2, join=True)
    got = _read_bins(fk.TestConfiguration(**cfg).outputDir)
    ref_dir = tmp_path / "ref"
    oracle.OracleResult(data, k, m, B).write_bins(str(ref_dir), sorted_eof=not use_ht)
    want = _read_bins(str(ref_dir))
    assert sorted(got) == sorted(want)
    for name in want:
        if use_ht:
            assert sorted(x for x in got[name].split(b"\n") if x) == sorted(x for x in want[name].split(b"\n") if x)
        else:
            assert got[name] == want[name]


@pytest.mark.parametrize("world", [1, 2, 3, 7, 50])
def test_record_shards_hold_whole_records(tmp_path, world):
    """sharding.read_record_shard: the ranks' pieces concatenate to the file and
    each holds whole records, so per-rank signature counts add up exactly."""
    from fastkmer_amd.sharding import read_record_shard
    rng = random.Random(world)
    data = b"junk\n" + b"".join(b">r%d\n" % i + bytes(rng.choice(b"ACGTN") for _ in range(rng.randint(0, 300))) + b"\n"
                                for i in range(200))
    path = tmp_path / "in.fa"
    path.write_bytes(data)
    pieces = [read_record_shard(str(path), world, r, window=64) for r in range(world)]
    assert b"".join(pieces) == data
    assert all(p[:1] == b">" for p in pieces[1:] if p)
    total = sum(oracle.bin_signatures(p, 21, 7) for p in pieces)
    assert (total == oracle.bin_signatures(data, 21, 7)).all()


def _binsig_worker(rank, world, port, cfg_kw):
    _init(rank, world, port, "gloo")
    try:
        from fastkmer_amd.exchange import execute_find_bin_signatures_job_distributed
        torch.cuda.set_device(0)
        execute_find_bin_signatures_job_distributed(fk.TestConfiguration(**cfg_kw), device=torch.device("cuda", 0))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_find_bin_signatures_job_distributed(tmp_path, world):
    """executeFindBinSignaturesJob (SBKC:956-986) over `world` ranks sharing one GPU:
    per-shard getBinSignatures, one all-reduce (the reduceByKey of :984), each rank
    writes its bins' bin_signatures<b>.txt; the union equals the oracle's files."""
    k, m, B = 28, 10, 2048
    data = fk.synth_fasta(20_000, 100, 200_000, seed=31)
    path = tmp_path / "in.fa"
    path.write_bytes(data)
    cfg = dict(dataset=str(path), outputDirectory=str(tmp_path / "out") + "/", k=k, m=m, x=3, max_b=B)
    mp.spawn(_binsig_worker, args=(world, _free_port(), cfg), nprocs=world, join=True)
    got = _read_bins(fk.TestConfiguration(**cfg).outputDir)
    ref_dir = tmp_path / "ref"
    oracle.write_bin_signatures(oracle.bin_signatures(data, k, m), m, B, str(ref_dir))
    want = _read_bins(str(ref_dir))
    assert len(want) > 100 and got == want


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_find_bin_signatures_job_distributed_long_sequence(tmp_path, world):
    """sequenceType = 1 with m = 13: one record cut into byte ranges with the k - 1 overlap
    (read_shard, as the reference's input splits cut it); a super-k-mer across a cut counts once
    per side, so the merged files equal the sum of every rank's own getBinSignatures over its
    piece -- the semantics this job pins -- and they differ from a one-rank run.  4^13 + 1 slots
    exceed the dense all-reduce: only the signatures that occur travel (all_gather of pairs)."""
    from fastkmer_amd.sharding import read_shard
    k, m, B = 28, 13, 4096
    data = _long_fasta()
    path = tmp_path / "long.fa"
    path.write_bytes(data)
    cfg = dict(dataset=str(path), outputDirectory=str(tmp_path / "out") + "/", k=k, m=m, x=3, max_b=B,
               sequenceType=1)
    mp.spawn(_binsig_worker, args=(world, _free_port(), cfg), nprocs=world, join=True)
    got = _read_bins(fk.TestConfiguration(**cfg).outputDir)
    want_counts = sum(oracle.bin_signatures(read_shard(str(path), world, r, k).piece, k, m) for r in range(world))
    ref_dir = tmp_path / "ref"
    oracle.write_bin_signatures(want_counts, m, B, str(ref_dir))
    assert got == _read_bins(str(ref_dir)) and len(got) > 10
    one = oracle.bin_signatures(data, k, m)
    assert int(want_counts.sum()) >= int(one.sum())  # the cuts add super-k-mers, never remove any


# ---------------------------------------------------------------- per-rank file reads (CPU)

def _fasta_variants():
    rng = random.Random(77)

    def reads(n, lo, hi, wrap=0, junk=b"", crlf=False, hdr=(5, 30)):
        out = [junk]
        for i in range(n):
            s = "".join(rng.choice("ACGTN" if rng.random() < 0.05 else "ACGT") for _ in range(rng.randint(lo, hi)))
            if wrap and s:
                s = "\n".join(s[q:q + wrap] for q in range(0, len(s), wrap))
            h = ">" + "".join(rng.choice("abcdef0123 ") for _ in range(rng.randint(*hdr)))
            rec = f"{h}\n{s}\n"
            out.append(rec.replace("\n", "\r\n").encode() if crlf else rec.encode())
        return b"".join(out)

    return {
        "short_reads": fk.synth_fasta(1500, 100, 40_000, seed=3),
        "wrapped_reads": reads(300, 20, 400, wrap=61),
        "junk_first": reads(200, 50, 150, junk=b"some text\nmore ACGT text\n"),
        "crlf": reads(200, 30, 120, crlf=True),
        "long_headers": reads(150, 10, 200, hdr=(200, 3000)),
        "one_long_record": _long_fasta(),
        "empty_records": reads(100, 0, 3),
    }


@pytest.mark.parametrize("name", sorted(_fasta_variants()))
@pytest.mark.parametrize("world", [2, 3, 5])
def test_read_shard_counts_add_up(tmp_path, name, world):
    from fastkmer_amd.sharding import read_shard
    data = _fasta_variants()[name]
    path = tmp_path / "in.fa"
    path.write_bytes(data)
    for k, m, st in [(28, 10, 0), (21, 9, 1)]:
        whole = _all_counts(oracle.OracleResult(data, k, m, 256, st))
        summed: dict = {}
        for r in range(world):
            sh = read_shard(str(path), world, r, k)
            for key, c in _all_counts(oracle.OracleResult(sh.piece, k, m, 256, st)).items():
                summed[key] = summed.get(key, 0) + c
        assert summed == whole, (name, world, k)


def _read_shard_worker(rank, world, port, path, k, q):
    from fastkmer_amd.sharding import read_shard
    _init(rank, world, port)
    sh = read_shard(path, world, rank, k)
    res = oracle.OracleResult(sh.piece, k, 10, 2048)
    counts = _all_counts(res)
    gathered = [None] * world
    dist.all_gather_object(gathered, (sh.touched, counts))
    if rank == 0:
        q.put(gathered)
    dist.destroy_process_group()


def test_per_rank_reads_touch_only_their_range(tmp_path):
    """World-size-2 gloo job: every rank reads only its n / world bytes plus one
    record's worth (the k - 1 positions after its range and the scans placing its
    ends), and the ranks' counts add up to the whole file's (the oracle's)."""
    world, k = 2, 28
    data = fk.synth_fasta(20_000, 100, 200_000, seed=9)
    path = tmp_path / "reads.fa"
    path.write_bytes(data)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_read_shard_worker, args=(r, world, port, str(path), k, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # beyond its range a rank reads: the file's first byte, the first byte of the line holding its
    # range start and one 256-byte scan step each way to place that line (a 114-byte record is
    # shorter than one step), and the k - 1 positions after its range in one read of 2 (k - 1) + 64
    one_record = 2 + 2 * 256 + 2 * (k - 1) + 64
    summed: dict = {}
    for touched, counts in got:
        assert touched <= len(data) // world + one_record + 1, touched
        for key, c in counts.items():
            summed[key] = summed.get(key, 0) + c
    assert summed == _all_counts(oracle.OracleResult(data, k, 10, 2048))
