"""Staged pieces of a job, through the C-ABI.

While the FASTA is still being copied in, every landed piece of it is partitioned
(the bin grouping of reduceByKey, SBKC:1035) and expanded into canonical k-mers in
its own key array; fk_finish expands the last piece and counts the job's buckets
once over all the pieces' keys (the sorted count of extractKXmers, SBKC:540-597).
A bin's multiset is the sum of its pieces' multisets, so the result must be
bit-exact against the CPU oracle over the whole input -- checked here at sizes
the oracle finishes quickly, with the pieces made small (FASTKMER_PIECE_BYTES)
so that inputs of a few MB cross several of them, for key distributions that
differ from piece to piece.  useHT=1 stages the same way (its buckets are
counted in table order); k = 64 counts the whole input after the last byte.
"""
import numpy as np
import pytest

import fastkmer_amd as fk
import oracle
from test_gpu_parity import assert_same_as_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture
def small_pieces(monkeypatch):
    monkeypatch.setenv("FASTKMER_INGEST_SEG", str(256 << 10))
    monkeypatch.setenv("FASTKMER_PIECE_BYTES", str(512 << 10))


def count_pinned(fasta, k, m, B=2048, use_ht=False, seq=0, repeat=1):
    import torch
    host = torch.empty(max(len(fasta), 1), dtype=torch.uint8).pin_memory()
    if fasta:
        host.numpy()[:len(fasta)] = np.frombuffer(fasta, dtype=np.uint8)
    kc = fk.KmerCounter(k, m, 3, B, use_ht, seq)
    for _ in range(repeat):
        kc.ingest_ptr(host.data_ptr(), len(fasta))
        kc.finish()
    return kc


@pytest.mark.parametrize("k,m,read_len,B", [(28, 10, 100, 2048), (28, 10, 100, 8192), (55, 12, 150, 8192)])
def test_piece_counts_merge_vs_oracle(small_pieces, k, m, read_len, B):
    fasta = fk.synth_fasta(40_000 if read_len == 100 else 25_000, read_len, 1_000_000, seed=0xA1 + k)
    kc = count_pinned(fasta, k, m, B, repeat=2)  # twice: the piece buffers are reused by the second job
    st = kc.stats()
    assert st["pieces_counted"] == 4 and st["fused_map"] == 1
    ref = oracle.OracleResult(fasta, k, m, B)
    assert st["kmers"] == ref.total_kmers and st["distinct"] == ref.distinct
    assert_same_as_oracle(kc, ref)


def test_piece_counts_disjoint_and_skewed_pieces(small_pieces):
    # piece key distributions that share nothing: reads of two unrelated genomes one after the
    # other, a stretch of one repeated read (a piece holding few keys, with huge counts), and
    # a low-complexity stretch -- a bucket's keys come from one piece only, or from all of them
    a = fk.synth_fasta(12_000, 100, 300_000, seed=0xA2)
    b = fk.synth_fasta(12_000, 100, 300_000, seed=0xA3, first_read=12_000)
    rep = b"".join(b">r%010d\n" % i + b"ACGTTGCAAGGCTTACCGATCGGATTACAGGCATCGATCGGGCTAGCTAGGCTAGCTTACGAGCTAGCATCGACTAGCATG"
                   b"CATGCATCGACGTAGCATCG\n" for i in range(6_000))
    low = b"".join(b">l%d\n" % i + (b"ACACACACAC" * 10) + b"\n" for i in range(6_000))
    fasta = a + rep + b + low + a[:len(a) // 2]
    kc = count_pinned(fasta, 28, 10)
    assert kc.stats()["pieces_counted"] >= 4
    assert_same_as_oracle(kc, oracle.OracleResult(fasta, 28, 10, 2048))


def test_piece_counts_piece_without_kmers(small_pieces):
    # pieces that hold no k-mer at all (reads of N only) between pieces that do: they are skipped
    # (no key array, no piece)
    a = fk.synth_fasta(8_000, 100, 300_000, seed=0xA7)
    nn = b"".join(b">n%d\n" % i + b"N" * 100 + b"\n" for i in range(20_000))
    b = fk.synth_fasta(8_000, 100, 300_000, seed=0xA8, first_read=8_000)
    fasta = a + nn + b
    kc = count_pinned(fasta, 28, 10)
    assert kc.stats()["pieces_counted"] >= 2
    assert_same_as_oracle(kc, oracle.OracleResult(fasta, 28, 10, 2048))


def test_piece_counts_long_sequence(small_pieces):
    rng = np.random.default_rng(5)
    seq = np.frombuffer(b"ACGTN", dtype=np.uint8)[rng.choice(5, 3_000_000, p=[.245, .245, .245, .245, .02])]
    fasta = b">chr synthetic\n" + b"\n".join(seq[i:i + 60].tobytes() for i in range(0, len(seq), 60)) + b"\n"
    kc = count_pinned(fasta, 28, 10, seq=1)
    assert kc.stats()["pieces_counted"] >= 4
    assert_same_as_oracle(kc, oracle.OracleResult(fasta, 28, 10, 2048, sequence_type=1))


def test_piece_counts_fallback_counts_whole_input(small_pieces):
    # a 40 KB line after several pieces were staged: the fused map hands the input back, the
    # staged pieces are dropped and the whole input is counted by the two-kernel path
    fasta = fk.synth_fasta(30_000, 100, 600_000, seed=0xA4)
    cut = len(fasta) * 3 // 4 // 114 * 114
    fasta = fasta[:cut] + b">" + b"h" * 40_000 + b"\n" + b"ACGT" * 40 + b"\n" + fasta[cut:]
    kc = count_pinned(fasta, 28, 10)
    st = kc.stats()
    assert st["fused_map"] == 0 and st["pieces_counted"] == 0
    assert_same_as_oracle(kc, oracle.OracleResult(fasta, 28, 10, 2048))


@pytest.mark.parametrize("k,m,read_len", [(28, 10, 100), (55, 12, 150)])
def test_piece_counts_hash_mode_staged(small_pieces, k, m, read_len):
    # useHT=1 stages its pieces like the sorted count; the wave tiers emit table order
    fasta = fk.synth_fasta(30_000 if read_len == 100 else 20_000, read_len, 400_000, seed=0xA5 + k)
    kc = count_pinned(fasta, k, m, use_ht=True)
    assert kc.stats()["pieces_counted"] == 4
    assert_same_as_oracle(kc, oracle.OracleResult(fasta, k, m, 2048), ordered=False)


def test_piece_counts_many_small_pieces(monkeypatch):
    # 64 KB pieces of a 3.4 MB job: the first pieces expanded as they land (at most STAGE_MAXP - 1
    # before fk_finish), the rest is the last piece
    monkeypatch.setenv("FASTKMER_INGEST_SEG", str(64 << 10))
    monkeypatch.setenv("FASTKMER_PIECE_BYTES", str(64 << 10))
    fasta = fk.synth_fasta(30_000, 100, 500_000, seed=0xA6)
    kc = count_pinned(fasta, 28, 10, repeat=2)
    assert kc.stats()["pieces_counted"] == 4
    assert_same_as_oracle(kc, oracle.OracleResult(fasta, 28, 10, 2048))


@pytest.mark.parametrize("cuts,chunks", [("0.45,0.7,0.85", 0), ("0.3", 0), ("0.2,0.25,0.97", 0), ("0.4,0.7,0.9", 7),
                                         ("0.3,0.55,0.75,0.9", 0)])
def test_staged_job_cuts_vs_one_count(monkeypatch, cuts, chunks):
    # a 1 GB job in one fk_ingest call (pinned): staged pieces at the job-size cuts (the
    # bench's path) against the same job counted whole from HBM (fk_ingest_device: no pieces),
    # every bin's keys and counts equal; a sampled slice of bins against the oracle is in
    # test_gpu_write; here both GPU paths must agree on all 2048 bins (a piece ends at its cut once it
    # holds >= 128 MB: "0.2,0.25,0.97" cuts at 0.2, ~0.33 and 0.97; four cuts: five pieces, the
    # schedule of 64-bit jobs of >= 4 GB)
    import torch
    n_reads = 1_000_000_000 // 114  # BASELINE configs[1]: pieces of >= 128 MB at every cut below
    dev = torch.empty(n_reads * 114, dtype=torch.uint8, device="cuda")
    fk.synth_fasta_to_device(dev.data_ptr(), n_reads, 100, 100_000_000, seed=0x5EED)
    host = torch.empty(dev.numel(), dtype=torch.uint8).pin_memory()
    host.copy_(dev)
    torch.cuda.synchronize()
    monkeypatch.setenv("FASTKMER_PIECE_CUTS", cuts)
    a = fk.KmerCounter(28, 10, 3, 2048)
    if chunks:  # a streamed job: fk_ingest_reserve announces its size, the cuts follow it
        a.reserve(host.numel())
        bounds = np.linspace(0, host.numel(), chunks + 1).astype(np.int64)
        for i in range(chunks):
            a.ingest_ptr(host.data_ptr() + int(bounds[i]), int(bounds[i + 1] - bounds[i]), last=i == chunks - 1)
    else:
        a.ingest_ptr(host.data_ptr(), host.numel())
    a.finish()
    st = a.stats()
    assert st["pieces_counted"] == cuts.count(",") + 2
    b = fk.KmerCounter(28, 10, 3, 2048)
    b.ingest_device(dev.data_ptr(), dev.numel())
    b.finish()
    assert b.stats()["pieces_counted"] == 0
    assert st["kmers"] == b.stats()["kmers"] and st["distinct"] == b.stats()["distinct"]
    sa, sb = a.bin_sizes(), b.bin_sizes()
    assert np.array_equal(sa, sb)
    for bin_ in range(2048):
        ka, ca = a.get_bin(bin_)
        kb, cb = b.get_bin(bin_)
        assert np.array_equal(ka, kb) and np.array_equal(ca, cb), f"bin {bin_}"
    a.close()
    b.close()


def test_staged_job_cuts_128bit_keys_at_most_four_pieces(monkeypatch):
    # k > 32 keys stage at most four pieces (their kernels' piece loops stop there, stage_npc): four
    # cuts give four pieces, the last one taking the rest; every bin equal to the job counted whole
    # from HBM (fk_ingest_device: no pieces)
    import torch
    n_reads = 700_000_000 // 164  # 150 bp reads: pieces of >= 128 MB at each cut kept
    dev = torch.empty(n_reads * 164, dtype=torch.uint8, device="cuda")
    fk.synth_fasta_to_device(dev.data_ptr(), n_reads, 150, 100_000_000, seed=0x5EED)
    host = torch.empty(dev.numel(), dtype=torch.uint8).pin_memory()
    host.copy_(dev)
    torch.cuda.synchronize()
    monkeypatch.setenv("FASTKMER_PIECE_CUTS", "0.3,0.55,0.75,0.9")
    a = fk.KmerCounter(55, 12, 3, 1024)
    a.ingest_ptr(host.data_ptr(), host.numel())
    a.finish()
    assert a.stats()["pieces_counted"] == 4
    b = fk.KmerCounter(55, 12, 3, 1024)
    b.ingest_device(dev.data_ptr(), dev.numel())
    b.finish()
    assert a.stats()["kmers"] == b.stats()["kmers"] and a.stats()["distinct"] == b.stats()["distinct"]
    assert np.array_equal(a.bin_sizes(), b.bin_sizes())
    for bin_ in range(0, 1024, 7):
        ka, ca = a.get_bin(bin_)
        kb, cb = b.get_bin(bin_)
        assert np.array_equal(ka, kb) and np.array_equal(ca, cb), f"bin {bin_}"
    a.close()
    b.close()
