"""useHT = 1 (extractKXmersHT, SparkBinKmerCounter.scala:664-739) through the C-ABI: the buckets of the
sorted count's cells, the wave tiers' LDS tables emitting their keys in table order (no rank), the
heavier tiers ascending -- one of the orders a hash map may iterate in.  The counts must be exact
(compared with the CPU oracle as sets: the reference's fastutil iteration order is unpinned).  The
(bin, signature hash) group tables of earlier rounds measured 1.3-1.7x slower at every load
(profiles/r05b_ht_paths.txt) and are gone."""
import pytest

import fastkmer_amd as fk
import oracle
from test_gpu_parity import assert_same_as_oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,genome", [(1, 1_000_000_000), (4, 1_000_000_000), (64, 300_000_000)])
def test_ht_large_bins_vs_oracle(B, genome):
    # one to a few bins of millions of distinct k-mers: many cells above the wave tier (split into
    # sub-buckets, or the block / big tiers)
    fasta = fk.synth_fasta(120_000, 100, genome, seed=0xB1 + B)
    with fk.KmerCounter(28, 10, 3, B, use_ht=True) as kc:
        for _ in range(2):  # the second job reuses the first one's buffers
            kc.ingest(fasta)
            kc.finish()
            st = kc.stats()
            ref = oracle.OracleResult(fasta, 28, 10, B)
            assert st["kmers"] == ref.total_kmers and st["distinct"] == ref.distinct
            assert_same_as_oracle(kc, ref, ordered=False)


@pytest.mark.parametrize("k,m,B", [(33, 11, 2048), (55, 12, 8192), (63, 15, 64), (55, 12, 1), (64, 15, 64)])
def test_ht_two_word_keys_vs_oracle(k, m, B):
    # k > 32: 128-bit keys (the 128-bit wave tiers in table order, the mid wave tier and the LDS sort);
    # k = 64: the one-level count, ascending
    fasta = fk.synth_fasta(40_000, 150, 20_000_000, seed=0xB2 + k + B)
    with fk.KmerCounter(k, m, 3, B, use_ht=True) as kc:
        kc.ingest(fasta)
        kc.finish()
        st = kc.stats()
        ref = oracle.OracleResult(fasta, k, m, B)
        assert st["kmers"] == ref.total_kmers and st["distinct"] == ref.distinct
        assert_same_as_oracle(kc, ref, ordered=False)


def test_ht_repeated_reads_vs_oracle():
    # a read repeated thousands of times: k-mers of counts far above a wave's 512 keys (the sub-bucket
    # split keeps such buckets on the block / big tiers)
    rep = b"".join(b">q%d\n" % i + b"ACGTTGCAAGGCTTACCGATCGGATTACAGGCATCGATCGGGCTAGCTAGGCTAGCTTACGAGCTAGCATCGACTAG"
                   b"CATGCATGCATCGACGTAGCATCG\n" for i in range(5_000))
    fasta = fk.synth_fasta(30_000, 100, 50_000_000, seed=0xB4) + rep
    with fk.KmerCounter(28, 10, 3, 16, use_ht=True) as kc:
        kc.ingest(fasta)
        kc.finish()
        ref = oracle.OracleResult(fasta, 28, 10, 16)
        assert kc.stats()["distinct"] == ref.distinct
        assert_same_as_oracle(kc, ref, ordered=False)
