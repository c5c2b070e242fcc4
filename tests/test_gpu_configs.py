"""BASELINE configs[2] (k=28 m=10 x=3 B=8192, 50 GB of 100 bp reads over 8
GPUs) on one MI355X, through the C-ABI (needs a GPU).

* At oracle size: bit-exact vs the CPU oracle in both count modes
  (extractKXmers, SBKC:428-660, and extractKXmersHT, SBKC:664-739) at the
  configuration's bin count.
* At the configuration's real per-GPU load: the job's 50 GB input is mapped
  as 8 shards (ranks 0..7 of n_ranks = 8, one after the other on this GPU),
  the records each shard sends to rank 0 (bin % 8 == 0, the round-robin
  placement of SURVEY 8e / the reduceByKey of SBKC:1034-1035) are gathered
  and rank 0 counts its 1,024 bins.  Checked through size-independent
  properties: every bin's count total equals the k-mers the 8 shards sent for
  it, keys are strictly ascending, sampled k-mers re-hash to their bin, and
  nothing lands in a bin rank 0 does not own.
"""
import os
import random

import numpy as np
import pytest

import fastkmer_amd as fk
import oracle
from test_gpu_parity import assert_same_as_oracle

pytestmark = pytest.mark.gpu

K, M, X, B = 28, 10, 3, 8192
G = 8
REC = 114  # '>r%010d\n' + 100 bases + '\n'


@pytest.mark.parametrize("use_ht", [False, True])
def test_c3_shape_b8192_vs_oracle(use_ht):
    fasta = fk.synth_fasta(60_000, 100, 2_000_000, seed=0xC3)
    with fk.KmerCounter(K, M, X, B, use_ht) as kc:
        assert kc.num_bins == 8192
        kc.ingest(fasta)
        kc.finish()
        ref = oracle.OracleResult(fasta, K, M, B)
        assert kc.stats()["kmers"] == ref.total_kmers
        assert_same_as_oracle(kc, ref, ordered=not use_ht)


@pytest.mark.parametrize("use_ht", [False, True])
def test_c3_shape_multi_rank_in_one_process_vs_oracle(use_ht):
    # 8 ranks of B=8192 in one process: records routed by bin % 8 (no RCCL),
    # each rank's 1,024 bins bit-exact vs the oracle
    fasta = fk.synth_fasta(24_000, 100, 1_000_000, seed=0xC38)
    n = 24_000 // G
    ref = oracle.OracleResult(fasta, K, M, B)
    ref_sizes = ref.bin_sizes()
    import torch
    sends = []
    mapper = fk.KmerCounter(K, M, X, B, use_ht, 0, n_ranks=G, rank=0)
    for r in range(G):
        mapper.ingest(fasta[r * n * REC:(r + 1) * n * REC])
        counts = mapper.map()
        buf = torch.empty(max(sum(counts), 1) * mapper.record_bytes, dtype=torch.uint8, device="cuda")
        mapper.map_emit(buf.data_ptr(), max(sum(counts), 1))
        torch.cuda.synchronize()
        sends.append((buf, counts))
    mapper.close()
    rb = 16
    for dst in range(G):
        parts = []
        for buf, counts in sends:
            off = sum(counts[:dst])
            parts.append(buf[off * rb:(off + counts[dst]) * rb])
        recv = torch.cat(parts)
        with fk.KmerCounter(K, M, X, B, use_ht, 0, n_ranks=G, rank=dst) as kc:
            kc.reduce(recv.data_ptr(), recv.numel() // rb)
            torch.cuda.synchronize()
            sizes = kc.bin_sizes()
            own = np.arange(B) % G == dst
            assert np.all(sizes[~own] == 0)
            assert np.array_equal(sizes[own].astype(np.int64), ref_sizes[own])
            for b in np.nonzero(ref_sizes * own)[0].tolist()[::7]:
                keys, cnt = kc.get_bin(b)
                _, rlo, rcnt = ref.bin_arrays(b)
                if use_ht:
                    order = np.argsort(keys)
                    keys, cnt = keys[order], cnt[order]
                assert np.array_equal(keys, rlo) and np.array_equal(cnt, rcnt), f"bin {b}"


def _signature(kmer: str) -> int:
    return min(oracle.norm(int("".join("%d" % "ACGT".index(ch) for ch in kmer[j:j + M]), 4), M)
               for j in range(K - M + 1))


def test_c3_per_gpu_load_rank0_properties():
    """configs[2] at its real per-GPU load on one GPU: rank 0's share of a
    50 GB job (FASTKMER_C3_GB overrides the job size for a rehearsal)."""
    import torch
    job_bytes = int(float(os.environ.get("FASTKMER_C3_GB", "50")) * 1e9)
    reads_per_rank = job_bytes // G // REC
    mapper = fk.KmerCounter(K, M, X, B, False, 0, n_ranks=G, rank=0)
    sent_kmers = np.zeros(B, dtype=np.uint64)  # k-mers each bin received from the 8 shards
    recv_parts, total_rec = [], 0
    for r in range(G):
        mapper.synth_device(reads_per_rank, 100, 3_000_000_000, seed=0x5EED, first_read=r * reads_per_rank)
        counts = mapper.map()
        sent_kmers += mapper.map_bin_kmers()
        send = torch.empty(sum(counts) * 16, dtype=torch.uint8, device="cuda")
        mapper.map_emit(send.data_ptr(), sum(counts))
        recv_parts.append(send[:counts[0] * 16].clone())  # rank 0's records come first
        total_rec += counts[0]
        del send
        torch.cuda.synchronize()
    mapper.close()
    torch.cuda.empty_cache()
    recv = torch.cat(recv_parts)
    del recv_parts
    torch.cuda.empty_cache()
    own = np.arange(B) % G == 0
    with fk.KmerCounter(K, M, X, B, False, 0, n_ranks=G, rank=0) as kc:
        kc.reduce(recv.data_ptr(), total_rec)
        torch.cuda.synchronize()
        cold = kc.stats()
        kc.reduce(recv.data_ptr(), total_rec)  # again with the context's buffers allocated (steady state)
        torch.cuda.synchronize()
        del recv
        st = kc.stats()
        sizes = kc.bin_sizes()
        assert st["records_received"] == total_rec
        assert np.all(sizes[~own] == 0)
        assert int(sizes.sum()) == st["distinct"] > 0
        assert np.all((sizes[own] > 0) == (sent_kmers[own] > 0))
        # per-GPU load: ~4 G k-mers into 1,024 bins for the 50 GB job
        assert int(sent_kmers[own].sum()) > 0.9 * job_bytes / REC * 73 / G
        rng = random.Random(8)
        for b in rng.sample(np.nonzero(own & (sizes > 0))[0].tolist(), 12):
            keys, counts = kc.get_bin(b)
            assert len(keys) == int(sizes[b])
            assert np.all(keys[1:] > keys[:-1]), f"bin {b} not strictly ascending"
            assert int(counts.sum(dtype=np.uint64)) == int(sent_kmers[b]), f"bin {b}: counts != k-mers sent"
            for kk in rng.sample(fk.decode_keys(keys, K), 8):
                assert oracle.hash_to_bucket(_signature(kk), B) == b
        print(f"configs[2] rank 0: {total_rec} records, {int(sent_kmers[own].sum())} k-mers, "
              f"{st['distinct']} distinct, count stage {st['ms_count']:.1f} ms "
              f"(first call, buffers allocated inside: {cold['ms_count']:.1f} ms), "
              f"partition {st['ms_partition']:.1f} ms, F={st['fine_bits']}, buckets {st['buckets']}, "
              f"large-path buckets {st['oversize_buckets']}")


def test_c4_per_gpu_load_rank0_properties():
    """BASELINE configs[3] (k=55 m=12 x=3 B=8192, 50 GB of 150 bp reads over 8 GPUs, two-word
    keys) at its real per-GPU load on one GPU: the 8 shards of the job mapped as ranks 0..7,
    the records each sends to rank 0 (bin % 8 == 0) counted by rank 0 (1,024 bins).  Checked
    through size-independent properties, as for configs[2] above (FASTKMER_C4_GB scales the job
    for a rehearsal)."""
    import torch
    k, m, b, read_len = 55, 12, 8192, 150
    rec = read_len + 14
    job_bytes = int(float(os.environ.get("FASTKMER_C4_GB", "50")) * 1e9)
    reads_per_rank = job_bytes // G // rec
    mapper = fk.KmerCounter(k, m, X, b, False, 0, n_ranks=G, rank=0)
    sent_kmers = np.zeros(b, dtype=np.uint64)
    recv_parts, total_rec = [], 0
    for r in range(G):
        mapper.synth_device(reads_per_rank, read_len, 3_000_000_000, seed=0x5EED, first_read=r * reads_per_rank)
        counts = mapper.map()
        sent_kmers += mapper.map_bin_kmers()
        send = torch.empty(sum(counts) * 24, dtype=torch.uint8, device="cuda")
        mapper.map_emit(send.data_ptr(), sum(counts))
        recv_parts.append(send[:counts[0] * 24].clone())  # rank 0's records come first
        total_rec += counts[0]
        del send
        torch.cuda.synchronize()
    mapper.close()
    torch.cuda.empty_cache()
    recv = torch.cat(recv_parts)
    del recv_parts
    torch.cuda.empty_cache()
    own = np.arange(b) % G == 0
    with fk.KmerCounter(k, m, X, b, False, 0, n_ranks=G, rank=0) as kc:
        kc.reduce(recv.data_ptr(), total_rec)
        torch.cuda.synchronize()
        cold = kc.stats()
        kc.reduce(recv.data_ptr(), total_rec)  # again with the context's buffers allocated (steady state)
        torch.cuda.synchronize()
        del recv
        torch.cuda.empty_cache()
        st = kc.stats()
        sizes = kc.bin_sizes()
        assert st["records_received"] == total_rec
        assert np.all(sizes[~own] == 0)
        assert int(sizes.sum()) == st["distinct"] > 0
        # per-GPU load: ~3.7 G k-mers (96 per read) into 1,024 bins for the 50 GB job
        assert int(sent_kmers[own].sum()) > 0.9 * job_bytes / rec * 96 / G
        rng = random.Random(55)
        for bb in rng.sample(np.nonzero(own & (sizes > 0))[0].tolist(), 12):
            keys, counts = kc.get_bin(bb)
            assert len(counts) == int(sizes[bb])
            pairs = keys.reshape(-1, 2)
            asc = (pairs[1:, 0] > pairs[:-1, 0]) | ((pairs[1:, 0] == pairs[:-1, 0]) & (pairs[1:, 1] > pairs[:-1, 1]))
            assert np.all(asc), f"bin {bb} not strictly ascending"
            assert int(counts.sum(dtype=np.uint64)) == int(sent_kmers[bb]), f"bin {bb}: counts != k-mers sent"
            for kk in rng.sample(fk.decode_keys(keys, k), 6):
                sig = min(oracle.norm(int("".join("%d" % "ACGT".index(ch) for ch in kk[j:j + m]), 4), m)
                          for j in range(k - m + 1))
                assert oracle.hash_to_bucket(sig, b) == bb
        print(f"configs[3] rank 0: {total_rec} records, {int(sent_kmers[own].sum())} k-mers, {st['distinct']} "
              f"distinct, count stage {st['ms_count']:.1f} ms (first call, buffers allocated inside: "
              f"{cold['ms_count']:.1f} ms), partition {st['ms_partition']:.1f} ms, F={st['fine_bits']}")


def _c5_job(path, world=8):
    """The record at `path` over `world` ranks of one in-process group (the library's own exchange,
    one host thread per rank), each rank reading its byte range plus the k - 1 overlap."""
    import threading
    from fastkmer_amd.sharding import read_shard
    pieces = [read_shard(str(path), world, r, 28).piece for r in range(world)]
    ctxs = [fk.KmerCounter(28, 10, 3, 2048, sequence_type=1, n_ranks=world, rank=r) for r in range(world)]
    fk.comm_init_local(ctxs)
    errs = [None] * world

    def work(r):
        try:
            ctxs[r].ingest(pieces[r])
            ctxs[r].finish()
        except Exception as e:  # noqa: BLE001
            errs[r] = e
    th = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    [t.start() for t in th]
    [t.join(timeout=600) for t in th]
    assert errs == [None] * world, errs
    return ctxs


def test_c5_whole_genome_over_8_ranks(tmp_path):
    """BASELINE configs[4] (sequenceType=1, a ~1.2 Gbp single record: 60-column lines, 100 N runs of
    10 kbp, 5% soft-masked, k=28) at its real size: the file cut into 8 byte ranges with the k - 1
    overlap (sharding.read_shard, FASTdoop's splits), 8 ranks exchanging their records in the library.
    Size-independent checks: the counts add up to the record's valid windows (counted here from the
    sequence's runs of A/C/G/T), every rank holds only its bins, bins ascend; then the first 20 Mbp
    of the same record over the same 8 ranks bit-exact vs the CPU oracle, every bin
    (FASTKMER_C5_BASES scales the record)."""
    import bench
    from test_gpu_comm import assert_union_matches_oracle
    n_bases = int(float(os.environ.get("FASTKMER_C5_BASES", "1.2e9")))
    data = bench.long_sequence_fasta(n_bases, seed=0xC5)
    path = tmp_path / "chr.fa"
    path.write_bytes(data)
    body = np.frombuffer(data, dtype=np.uint8)[data.index(b"\n") + 1:]
    seq = body[body != 10]
    valid = np.isin(seq, np.frombuffer(b"ACGT", dtype=np.uint8))
    edges = np.flatnonzero(np.diff(np.concatenate([[0], valid.view(np.int8), [0]])))
    runs = edges[1::2] - edges[0::2]
    windows = int(np.maximum(runs - 27, 0).sum())
    del body, seq, valid
    ctxs = _c5_job(path)
    assert sum(c.stats()["kmers"] for c in ctxs) == windows > 0.9 * n_bases
    total = 0
    for r, c in enumerate(ctxs):
        sizes = c.bin_sizes()
        assert np.all(sizes[np.arange(2048) % 8 != r] == 0)
        cnt_sum = 0
        for b in np.nonzero(sizes)[0].tolist():
            keys, counts = c.get_bin(b)
            assert np.all(keys[1:] > keys[:-1]), f"bin {b} not ascending"
            cnt_sum += int(counts.sum(dtype=np.uint64))
        assert cnt_sum > 0  # the k-mers of its bins (from every rank's input)
        total += cnt_sum
        c.close()
    assert total == windows
    # the first 20 Mbp (cut at a line end) bit-exact vs the oracle
    cut = data.index(b"\n", 20_000_000) + 1
    prefix = data[:cut]
    del data
    ppath = tmp_path / "prefix.fa"
    ppath.write_bytes(prefix)
    ctxs = _c5_job(ppath)
    assert_union_matches_oracle(ctxs, oracle.OracleResult(prefix, 28, 10, 2048, sequence_type=1))
    print(f"configs[4]: {n_bases} bases, {windows} k-mers over 8 ranks; 20 Mbp prefix bit-exact")
