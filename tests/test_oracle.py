"""CPU oracle pinned against the reference's known answers (no GPU).

The reference ships no tests or fixtures, so the oracle
is pinned by (1) the Appendix B known-answer vectors, (2) a step-for-step
Scala transliteration (oracle/literal_ref.py) and (3) an independent naive
counter, and the committed golden fixtures in tests/golden/.
"""
import json
import os
import random

import pytest

import naive_oracle
import oracle
from conftest import GOLDEN, golden_cases
from oracle import literal_ref


def enc(s):
    v = 0
    for ch in s:
        v = v * 4 + "ACGT".index(ch)
    return v


@pytest.mark.parametrize("B,expected", [
    (2048, [362, 1181, 1677, 77, 2011, 1821, 136]),
    (8192, [2410, 3229, 3725, 2125, 4059, 7965, 136]),
])
def test_hash_to_bucket_kat(B, expected):
    sigs = [0, 1, 5, 123456, 1048575, 1048576, 16777216]
    assert [oracle.hash_to_bucket(s, B) for s in sigs] == expected
    assert [literal_ref.hash_to_bucket(s, B) for s in sigs] == expected
    assert [naive_oracle.hash_to_bucket(s, B) for s in sigs] == expected


@pytest.mark.parametrize("mmer,norm,allowed", [
    ("AAAAAAAAAA", 1048575, False), ("TTTTTTTTTT", 1048575, True),
    ("ACCCCCCCCC", 87381, True), ("ACACACACAC", 768955, False),
    ("CACACACACA", 279620, True), ("GTGTGTGTGT", 768955, True),
    ("ACGTACGTAC", 111025, True), ("CCCCCCCCCC", 349525, True),
])
def test_norm_kat(mmer, norm, allowed):
    assert oracle.norm(enc(mmer), 10) == norm
    assert oracle.is_allowed(enc(mmer), 10) == allowed
    assert naive_oracle.norm(mmer) == norm


@pytest.mark.parametrize("m", [1, 2, 3, 4, 5, 6, 7])
def test_is_allowed_exhaustive_vs_literal(m):
    for v in range(4 ** m):
        assert oracle.is_allowed(v, m) == literal_ref.is_allowed(v, m)
        s = "".join("ACGT"[(v >> (2 * (m - 1 - t))) & 3] for t in range(m))
        assert naive_oracle.allowed(s) == literal_ref.is_allowed(v, m)


def test_norm_table_stats_m10():
    # Appendix B: allowed fraction 0.6029 at m=10; 457,085 distinct signatures
    # (including the default 4^m).
    table = literal_ref.fill_norm(8)
    full = [oracle.norm(v, 8) for v in range(4 ** 8)]
    assert table == full
    import numpy as np
    lib = oracle.lib()
    allowed = sum(lib.fko_is_allowed(v, 10) for v in range(0, 4 ** 10, 7))
    assert abs(allowed / len(range(0, 4 ** 10, 7)) - 0.6029) < 0.003


def test_clamp_bins():
    assert oracle.clamp_bins(10, 2048) == 2048
    assert oracle.clamp_bins(3, 2048) == 64
    assert oracle.clamp_bins(12, 8192) == 8192
    assert literal_ref.clamp_bins(3, 2048) == 64


def test_end_to_end_kat_appendix_b():
    fa = (b">r1\nACGTTGCATGCATGCAACGTTAGCCGATCGATCGGATCCATGCANNACGTTGCATGCATGCAACGTTAGCCGATCGAT\n"
          b">r2\nATCGATCGGCTAACGTTGCATGCATGCAACGTACGTTGCA\n>r3\n" + b"G" * 30 + b"\n")
    r = oracle.OracleResult(fa, 28, 10, 2048)
    nonempty = [b for b in range(r.nbins) if r.bin_size(b)]
    assert nonempty == [270, 1195, 1730, 1829]
    assert r.bin_text(270) == "CGTACGTTGCATGCATGCAACGTTAGCC\t1\nEOF"
    assert r.bin_text(1195) == ("AACGTACGTTGCATGCATGCAACGTTAG\t1\nAACGTTGCATGCATGCAACGTACGTTGC\t1\n"
                                "ACGTACGTTGCATGCATGCAACGTTAGC\t1\nACGTTGCATGCATGCAACGTACGTTGCA\t1\n"
                                "CAACGTACGTTGCATGCATGCAACGTTA\t1\nEOF")
    assert r.bin_text(1730) == "CCCCCCCCCCCCCCCCCCCCCCCCCCCC\t3\nEOF"
    lines = r.bin_text(1829).split("\n")
    assert len(lines) == 20 and lines[-1] == "EOF"
    assert lines[0] == "AACGTTAGCCGATCGATCGGATCCATGC\t1"
    assert lines[1] == "ACGTTAGCCGATCGATCGGATCCATGCA\t1"
    assert lines[2] == "ACGTTGCATGCATGCAACGTTAGCCGAT\t3"
    assert lines[-2] == "TGCAACGTTAGCCGATCGATCGGATCCA\t1"


def test_superkmer_trace_matches_literal():
    rng = random.Random(7)
    for _ in range(40):
        k = rng.choice([9, 21, 28, 31, 33, 55])
        m = min(k, rng.choice([3, 5, 7, 8]))
        read = "".join(rng.choice("ACGTN" if rng.random() < 0.3 else "ACGT") for _ in range(rng.randint(0, 200)))
        bc = oracle.clamp_bins(m, 2048)
        tr = []
        lit = literal_ref.get_super_kmers(k, m, bc, [read.encode()], trace=tr)
        c = oracle.trace_read(read.encode(), k, m, 2048)
        assert [b for (_, _, b) in c] == tr
        lens = sorted(km.length for sks in lit.values() for km in sks)
        assert sorted(l for (_, l, _) in c) == lens


@pytest.mark.parametrize("name", sorted(golden_cases()))
def test_golden_fixture(name):
    params = golden_cases()[name]
    with open(os.path.join(GOLDEN, name + ".fa"), "rb") as f:
        fasta = f.read()
    with open(os.path.join(GOLDEN, name + ".expected.json")) as f:
        expected = json.load(f)
    r = oracle.OracleResult(fasta, params["k"], params["m"], params["B"], params.get("sequence_type", 0))
    got = {f"bin{b}": r.bin_text(b) for b in range(r.nbins) if r.bin_size(b)}
    assert got == expected
    assert r.total_kmers == params["total_kmers"]


def test_oracle_matches_literal_and_naive_random():
    rng = random.Random(1234)
    for trial in range(12):
        k = rng.choice([5, 12, 21, 28, 31, 32, 33, 55, 63])
        m = min(k, rng.choice([1, 2, 3, 7, 10]))
        x = rng.choice([1, 2, 3])
        B = rng.choice([1, 7, 64, 2048])
        reads = []
        for i in range(rng.randint(1, 6)):
            s = "".join(rng.choice("ACGTN" if rng.random() < 0.2 else "ACGT") for _ in range(rng.randint(0, 120)))
            reads.append(f">r{i}\n{s}\n")
        fa = "".join(reads).encode()
        r = oracle.OracleResult(fa, k, m, B)
        assert r.all_dict() == naive_oracle.count(fa, k, m, B)
        lit = literal_ref.run_sorted(fa, k, m, x, B)
        assert {b: r.bin_text(b) for b in lit} == lit
        assert sorted(lit) == [b for b in range(r.nbins) if r.bin_size(b)]
        ht = literal_ref.run_ht(fa, k, m, B)
        assert {b: dict(sorted(d.items())) for b, d in ht.items()} == r.all_dict()


def test_oracle_rejects_invalid_params():
    with pytest.raises(ValueError):
        oracle.OracleResult(b">a\nACGT\n", 70, 10, 2048)
    with pytest.raises(ValueError):
        oracle.OracleResult(b">a\nACGT\n", 28, 16, 2048)
    with pytest.raises(ValueError):
        oracle.OracleResult(b">a\nACGT\n", 28, 10, 0)


@pytest.mark.parametrize("threads", [2, 3, 8])
def test_oracle_threads_match_single(threads):
    # the multi-threaded driver (bench.py's CPU baseline) splits at record starts;
    # text before the first header, tiny inputs and more threads than records included
    rng = random.Random(99 + threads)
    reads = [f">r{i} x\n" + "".join(rng.choice("ACGTN" if rng.random() < 0.1 else "ACGT")
                                     for _ in range(rng.randint(0, 300))) + "\n" for i in range(300)]
    for fa in (b"junk\nACGTACGTACGTAC\n" + "".join(reads).encode(), b">a\nACGTACGTACGTACGTACGTACGTACGTAC\n", b""):
        for k, m, B in ((28, 10, 2048), (21, 7, 64), (55, 12, 8192)):
            a = oracle.OracleResult(fa, k, m, B)
            b = oracle.OracleResult(fa, k, m, B, threads=threads)
            assert (a.total_kmers, a.superkmers, a.reads, a.distinct) == (b.total_kmers, b.superkmers, b.reads, b.distinct)
            assert a.all_dict() == b.all_dict()


@pytest.mark.parametrize("mod,rem", [(1, 0), (4, 3), (64, 17)])
def test_oracle_bin_filter_keeps_exactly_its_bins(mod, rem):
    # fko_count_mt_filtered (the checker of the configs[2] per-GPU load): the kept bins are the
    # unfiltered oracle's, every other bin is empty, and every k-mer is still walked and counted
    import ctypes
    import fastkmer_amd as fk
    fa = fk.synth_fasta(4000, 100, 300_000, seed=5)
    full = oracle.OracleResult(fa, 28, 10, 2048)
    buf = ctypes.create_string_buffer(fa, len(fa))
    for threads in (1, 3):
        f = oracle.OracleResult(None, 28, 10, 2048, threads=threads, bin_mod=mod, bin_rem=rem,
                                ptr=ctypes.addressof(buf), nbytes=len(fa))
        assert (f.total_kmers, f.superkmers, f.reads) == (full.total_kmers, full.superkmers, full.reads)
        for b in range(2048):
            if b % mod == rem:
                assert all((x == y).all() for x, y in zip(f.bin_arrays(b), full.bin_arrays(b))), b
            else:
                assert f.bin_size(b) == 0
    with pytest.raises(ValueError):
        oracle.OracleResult(fa, 28, 10, 2048, bin_mod=4, bin_rem=4)


# ---------------------------------------------------------------- bin-signature diagnostics

def _binsig_files(counts, m, B, tmp_path):
    d = tmp_path / f"sig_{m}_{B}"
    d.parent.mkdir(parents=True, exist_ok=True)
    oracle.write_bin_signatures(counts, m, B, str(d))
    return {p.name: p.read_text() for p in d.iterdir()}


def test_long_to_string_is_31_characters():
    # longToString ignores its length argument (package.scala:616-634)
    assert literal_ref.long_to_string(0, 10) == "A" * 31
    assert literal_ref.long_to_string(enc("ACGTACGTAC"), 10) == "A" * 21 + "ACGTACGTAC"
    assert literal_ref.long_to_string(4 ** 10, 10) == "A" * 20 + "C" + "A" * 10


def test_bin_signatures_match_literal_random(tmp_path):
    rng = random.Random(4321)
    for trial in range(14):
        k = rng.choice([5, 12, 21, 28, 31, 33, 55, 64])
        m = min(k, rng.choice([1, 2, 3, 7, 10]))
        B = rng.choice([1, 7, 64, 2048])
        reads = []
        for i in range(rng.randint(1, 6)):
            alpha = rng.choice(["ACGT", "ACGTN", "AAAC", "ACGTT"])
            reads.append(f">r{i}\n" + "".join(rng.choice(alpha) for _ in range(rng.randint(0, 150))) + "\n")
        fa = "".join(reads).encode()
        counts = oracle.bin_signatures(fa, k, m)
        bc = oracle.clamp_bins(m, B)
        lit = literal_ref.get_bin_signatures(k, m, bc, literal_ref.parse_reads(fa))
        want = {f"bin_signatures{b}.txt": literal_ref.save_bin_signatures_text(dict(sorted(d.items())))
                for b, d in lit.items()}
        assert _binsig_files(counts, m, B, tmp_path / str(trial)) == want
        # one count per super-k-mer of getSuperKmers (the same walk, SBKC:59-161)
        assert int(counts.sum()) == oracle.OracleResult(fa, k, m, B).superkmers


@pytest.mark.parametrize("name", sorted(golden_cases()))
def test_bin_signatures_golden_fixture(name, tmp_path):
    params = golden_cases()[name]
    with open(os.path.join(GOLDEN, name + ".fa"), "rb") as f:
        fasta = f.read()
    with open(os.path.join(GOLDEN, name + ".binsig.json")) as f:
        expected = json.load(f)
    counts = oracle.bin_signatures(fasta, params["k"], params["m"])
    assert _binsig_files(counts, params["m"], params["B"], tmp_path) == expected


def test_bin_signatures_rejects_invalid_params():
    with pytest.raises(ValueError):
        oracle.bin_signatures(b">a\nACGT\n", 70, 10)
    with pytest.raises(ValueError):
        oracle.bin_signatures(b">a\nACGT\n", 8, 9)
