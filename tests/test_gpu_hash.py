"""useHT = 1 (extractKXmersHT, SparkBinKmerCounter.scala:664-739) through the C-ABI, on both hash
counts: the buckets of the sorted count's cells with the wave tiers' LDS tables emitting table order
(the default), and the (bin, signature hash) group tables with exact spill rounds
(FASTKMER_HT_GROUPS=1: inputs that overflow the tables force spill rounds).  The counts must be exact
(compared with the CPU oracle as sets: the reference's fastutil iteration order is unpinned)."""
import pytest

import fastkmer_amd as fk
import oracle
from test_gpu_parity import assert_same_as_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["buckets", "groups"])
def ht_path(monkeypatch, request):
    monkeypatch.setenv("FASTKMER_HT_GROUPS", "1" if request.param == "groups" else "0")
    return request.param


@pytest.mark.parametrize("B,genome", [(1, 1_000_000_000), (4, 1_000_000_000), (64, 300_000_000)])
def test_ht_large_spills_vs_oracle(ht_path, B, genome):
    # one to a few bins of millions of distinct k-mers: every group table overflows, the
    # spilled keys of a group are split over sub-items that share one spill range per parent
    fasta = fk.synth_fasta(120_000, 100, genome, seed=0xB1 + B)
    with fk.KmerCounter(28, 10, 3, B, use_ht=True) as kc:
        for _ in range(2):  # the second job sizes its groups from the first one's distinct ratio
            kc.ingest(fasta)
            kc.finish()
            st = kc.stats()
            ref = oracle.OracleResult(fasta, 28, 10, B)
            assert st["kmers"] == ref.total_kmers and st["distinct"] == ref.distinct
            assert_same_as_oracle(kc, ref, ordered=False)
        if B == 1 and ht_path == "groups":
            assert st["ht_rounds"] > 1 and st["ht_spilled"] > 1_000_000, st


@pytest.mark.parametrize("k,m,B", [(33, 11, 2048), (55, 12, 8192), (63, 15, 64), (55, 12, 1)])
def test_ht_two_word_lds_tables_vs_oracle(ht_path, k, m, B):
    # k > 32: 128-bit keys in the LDS group tables (k_ht_combine128); B = 1 overflows every table
    fasta = fk.synth_fasta(40_000, 150, 20_000_000, seed=0xB2 + k + B)
    with fk.KmerCounter(k, m, 3, B, use_ht=True) as kc:
        kc.ingest(fasta)
        kc.finish()
        st = kc.stats()
        ref = oracle.OracleResult(fasta, k, m, B)
        assert st["kmers"] == ref.total_kmers and st["distinct"] == ref.distinct
        assert_same_as_oracle(kc, ref, ordered=False)
        if B == 1 and ht_path == "groups":
            assert st["ht_rounds"] > 1


@pytest.mark.parametrize("k,m,B,thr", [(55, 12, 64, 600), (63, 15, 64, 1500), (55, 12, 1, 2000), (55, 12, 1, 0),
                                        (55, 12, 64, 400)])
def test_ht_heavy_group_tables_vs_oracle(monkeypatch, k, m, B, thr):
    # k > 32 with FASTKMER_HT_BIG: groups of more than thr k-mers take the 6144-slot tables
    # (k_ht_combine128<false, 1024, 6144> over the device-listed heavy groups), the rest the
    # 2048-slot ones; B = 1 still spills past the big tables; thr = 0: every group in 2048 slots
    monkeypatch.setenv("FASTKMER_HT_GROUPS", "1")
    monkeypatch.setenv("FASTKMER_HT_BIG", str(thr))
    fasta = fk.synth_fasta(40_000, 150, 20_000_000, seed=0xB3 + k + B)
    with fk.KmerCounter(k, m, 3, B, use_ht=True) as kc:
        kc.ingest(fasta)
        kc.finish()
        st = kc.stats()
        ref = oracle.OracleResult(fasta, k, m, B)
        assert st["kmers"] == ref.total_kmers and st["distinct"] == ref.distinct
        assert_same_as_oracle(kc, ref, ordered=False)
        assert (st["ht_big_groups"] > 0) == (thr > 0), st
