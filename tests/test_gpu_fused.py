"""The fused parse + signature kernel (k_map_fused) vs the CPU oracle, through
the C-ABI (needs an MI355X).

k_map_fused replaces the FASTdoop record reader and getSuperKmers
(SBKC:62-65, :34-169) with one kernel per 32 KB (or 16 KB) tile of FASTA
bytes.  Its own edge cases are the tile boundaries: a tile starting inside a
header or sequence line, windows reaching into the next tile's bytes (the
halo), and the inputs it hands to the two-kernel path (lines longer than its
read-back, text before the first header, halos with too few positions).
Every case is bit-exact against the oracle, and the tests check which path
ran (fk_stats.fused_map).
"""
import random

import numpy as np
import pytest

import fastkmer_amd as fk
import oracle
from test_gpu_parity import assert_same_as_oracle

pytestmark = pytest.mark.gpu

CONFIGS = [(28, 10, 3, 2048), (55, 12, 3, 8192)]


def _fasta(rng: random.Random, n_rec: int, min_len: int, max_len: int, width=None, noise=0.002,
           header_len=(1, 40), crlf=False) -> bytes:
    out = []
    for r in range(n_rec):
        L = rng.randint(min_len, max_len)
        seq = [rng.choice("ACGT") for _ in range(L)]
        for i in range(L):
            if rng.random() < noise:
                seq[i] = rng.choice("NacgtRY\r")
        s = "".join(seq)
        hdr = ">" + "".join(rng.choice("abcdefghij0123456789 >ACGT") for _ in range(rng.randint(*header_len)))
        wdt = width if width is not None else rng.choice([60, 70, 80, 1000, 10 ** 9])
        lines = [s[q:q + wdt] for q in range(0, len(s), wdt)] or [""]
        eol = "\r\n" if crlf else "\n"
        out.append(hdr + eol + eol.join(lines) + "\n")
    return "".join(out).encode()


def _run(fasta, k, m, x, B, use_ht=False, nt=None, monkeypatch=None, sequence_type=0):
    if nt is not None:
        monkeypatch.setenv("FASTKMER_FUSED_NT", str(nt))
    kc = fk.KmerCounter(k, m, x, B, use_ht, sequence_type)
    kc.ingest(fasta)
    kc.finish()
    return kc


@pytest.mark.parametrize("nt", [256, 512])
@pytest.mark.parametrize("k,m,x,B", CONFIGS)
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_fused_random_vs_oracle(monkeypatch, nt, k, m, x, B, seed):
    rng = random.Random(1000 * seed + k + nt)
    fasta = _fasta(rng, 3000, 1, 400, noise=0.01)
    kc = _run(fasta, k, m, x, B, nt=nt, monkeypatch=monkeypatch)
    st = kc.stats()
    assert st["fused_map"] == 1, "the fused kernel should place this input"
    ref = oracle.OracleResult(fasta, k, m, B)
    assert st["kmers"] == ref.total_kmers
    assert_same_as_oracle(kc, ref)


@pytest.mark.parametrize("nt", [256, 512])
def test_fused_short_reads_both_modes(monkeypatch, nt):
    fasta = fk.synth_fasta(40_000, 100, 500_000, seed=77)
    ref = oracle.OracleResult(fasta, 28, 10, 2048)
    for use_ht in (False, True):
        kc = _run(fasta, 28, 10, 3, 2048, use_ht, nt=nt, monkeypatch=monkeypatch)
        assert kc.stats()["fused_map"] == 1
        assert_same_as_oracle(kc, ref, ordered=not use_ht)
        kc.close()


def test_fused_matches_two_kernel_path_records(monkeypatch):
    # same input through both map paths: identical counts, identical k-mer totals
    fasta = _fasta(random.Random(5), 5000, 50, 300)
    a = _run(fasta, 28, 10, 3, 2048)
    monkeypatch.setenv("FASTKMER_FUSED", "0")
    b = _run(fasta, 28, 10, 3, 2048)
    assert a.stats()["fused_map"] == 1 and b.stats()["fused_map"] == 0
    assert a.stats()["kmers"] == b.stats()["kmers"]
    assert np.array_equal(a.bin_sizes(), b.bin_sizes())
    for bin_ in np.nonzero(a.bin_sizes())[0].tolist()[::5]:
        ka, ca = a.get_bin(bin_)
        kb, cb = b.get_bin(bin_)
        assert np.array_equal(ka, kb) and np.array_equal(ca, cb)


@pytest.mark.parametrize("case", ["long_header", "long_line", "junk_first", "one_base_lines", "crlf",
                                  "header_across_tiles", "tiny", "empty", "no_newline_end", "blank_lines"])
@pytest.mark.parametrize("nt", [256, 512])
def test_fused_edge_inputs_vs_oracle(monkeypatch, case, nt):
    rng = random.Random(sum(case.encode()))
    expect_fused = True
    if case == "long_header":  # a 10 kB header line over bytes ~59.5k-69.5k: the tiles starting at
        # 64512 (16 KB tiles) and 65024 (32 KB tiles) find no newline in the 4 kB before them
        body = b""
        while len(body) < 59_500:
            body += _fasta(rng, 1, 50, 200)
        fasta = body + b">" + b"h" * 10_000 + b"\n" + _fasta(rng, 300, 50, 200)[1:]
        expect_fused = False
    elif case == "long_line":  # one 200 kbp line: a tile start has no newline within 4 kB before it
        fasta = _fasta(rng, 2, 100_000, 100_000, width=10 ** 9)
        expect_fused = False
    elif case == "junk_first":  # text before the first header is not sequence
        fasta = b"ACGTACGTACGT" * 500 + b"\n" + _fasta(rng, 600, 50, 200)
        expect_fused = False
    elif case == "one_base_lines":  # 2 bytes per base: the 256-byte halo still holds 128 positions
        fasta = _fasta(rng, 30, 2000, 2000, width=1)
    elif case == "blank_lines":  # 16 bytes per base: a 256-byte halo holds < k - 1 positions
        fasta = b"".join(b">r%d\n" % i + b"".join(bytes([ch]) + b"\n" * 15 for ch in
                                                  rng.choices(b"ACGT", k=3000)) for i in range(12))
        expect_fused = False
    elif case == "crlf":
        fasta = _fasta(rng, 800, 50, 300, crlf=True)
    elif case == "header_across_tiles":  # headers of 100-3000 bytes straddle tile boundaries
        fasta = _fasta(rng, 500, 20, 200, header_len=(100, 3000))
    elif case == "tiny":
        fasta = b">r\nACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTAC\n"
    elif case == "empty":
        fasta = b""
        expect_fused = False
    else:  # the last line has no trailing newline
        fasta = _fasta(rng, 500, 50, 300).rstrip(b"\n")
    for k, m, x, B in CONFIGS:
        kc = _run(fasta, k, m, x, B, nt=nt, monkeypatch=monkeypatch)
        ref = oracle.OracleResult(fasta, k, m, B)
        st = kc.stats()
        assert st["kmers"] == ref.total_kmers
        assert_same_as_oracle(kc, ref)
        if case not in ("tiny",):
            assert st["fused_map"] == (1 if expect_fused else 0), case
        kc.close()


def test_fused_long_sequence_type1_vs_oracle(monkeypatch):
    # sequenceType=1: one long record in 60-column lines with N runs and soft-masking
    rng = random.Random(11)
    seq = [rng.choice("ACGT") for _ in range(300_000)]
    for s in range(0, 300_000, 37_000):
        seq[s:s + 500] = "N" * 500
    for s in range(5_000, 300_000, 50_000):
        seq[s:s + 800] = [ch.lower() for ch in seq[s:s + 800]]
    body = "".join(seq)
    fasta = (">chrT\n" + "\n".join(body[q:q + 60] for q in range(0, len(body), 60)) + "\n").encode()
    kc = _run(fasta, 28, 10, 3, 2048, sequence_type=1)
    assert kc.stats()["fused_map"] == 1
    ref = oracle.OracleResult(fasta, 28, 10, 2048, 1)
    assert_same_as_oracle(kc, ref)


def test_fused_full_size_matches_two_kernel_path(monkeypatch):
    # BASELINE configs[1] size (1 GB): both map paths give the same bins
    n_reads = 1_000_000_000 // 114
    a = fk.KmerCounter(28, 10, 3, 2048)
    a.synth_device(n_reads, 100, 100_000_000, seed=0x5EED)
    a.finish()
    monkeypatch.setenv("FASTKMER_FUSED", "0")
    b = fk.KmerCounter(28, 10, 3, 2048)
    b.synth_device(n_reads, 100, 100_000_000, seed=0x5EED)
    b.finish()
    sa, sb = a.stats(), b.stats()
    assert sa["fused_map"] == 1 and sb["fused_map"] == 0
    assert sa["kmers"] == sb["kmers"] and sa["distinct"] == sb["distinct"] and sa["positions"] == sb["positions"]
    assert np.array_equal(a.bin_sizes(), b.bin_sizes())
    rng = random.Random(3)
    for bin_ in rng.sample(range(2048), 24):
        ka, ca = a.get_bin(bin_)
        kb, cb = b.get_bin(bin_)
        assert np.array_equal(ka, kb) and np.array_equal(ca, cb)
