"""Bin-signature diagnostics on the GPU: executeFindBinSignaturesJob,
SBKC:956-986 -- getBinSignatures (:772-917) counted by k_bin_signatures
(fk_bin_signatures.inc) and saveBinSignatures (:920-953) written by
fk_write_bin_signatures, through the C-ABI, against the C oracle
(fko_bin_signatures, itself pinned to the literal transliteration and the
committed tests/golden/*.binsig.json fixtures).

The reference writes each bin's signatures in HashMap order (unspecified);
both writers here use ascending signature order, so files compare byte for
byte.
"""
import json
import os

import numpy as np
import pytest
import torch

import fastkmer_amd as fk
import oracle
from conftest import GOLDEN, golden_cases

pytestmark = pytest.mark.gpu


def _files(d):
    if not os.path.isdir(d):
        return {}
    return {f: open(os.path.join(d, f), "rb").read().decode() for f in sorted(os.listdir(d))}


def _gpu_counts(fasta, k, m, B=2048, seq_type=0, chunks=1):
    with fk.KmerCounter(k, m, 3, B, False, seq_type) as kc:
        if chunks == 1:
            kc.ingest(fasta)
        else:
            step = -(-len(fasta) // chunks)
            for i in range(chunks):
                kc.ingest_chunk(fasta[i * step:(i + 1) * step], i == chunks - 1)
        return kc.signature_counts().cpu().numpy()


def _oracle_files(counts, m, B, d):
    oracle.write_bin_signatures(counts, m, B, str(d))
    return _files(str(d))


@pytest.mark.parametrize("name", sorted(golden_cases()))
def test_golden_fixtures(name, tmp_path):
    p = golden_cases()[name]
    with open(os.path.join(GOLDEN, name + ".fa"), "rb") as f:
        fasta = f.read()
    with open(os.path.join(GOLDEN, name + ".binsig.json")) as f:
        expected = json.load(f)
    with fk.KmerCounter(p["k"], p["m"], p["x"], p["B"], False, p.get("sequence_type", 0)) as kc:
        kc.ingest(fasta)
        counts = kc.signature_counts()
        kc.write_bin_signatures(counts, str(tmp_path / "gpu"))
    assert _files(str(tmp_path / "gpu")) == expected


@pytest.mark.parametrize("k,m", [(28, 10), (55, 12), (21, 7), (5, 3), (8, 2), (12, 1), (64, 12), (31, 11)])
def test_counts_vs_oracle_short_reads(k, m):
    fasta = fk.synth_fasta(20_000, 100, 300_000, seed=0x5EED + k + m, err_rate=0.01, n_rate=0.003)
    got = _gpu_counts(fasta, k, m)
    want = oracle.bin_signatures(fasta, k, m)
    assert got.shape == want.shape
    assert np.array_equal(got, want), f"{int((got != want).sum())} signatures differ"
    assert int(got.sum()) == oracle.OracleResult(fasta, k, m, 2048).superkmers


def _long_records(rng, n, length, alphabet, line=70):
    out = []
    for i in range(n):
        s = "".join(rng.choice(alphabet) for _ in range(length))
        out.append(f">chr{i}\n" + "\n".join(s[q:q + line] for q in range(0, len(s), line)) + "\n")
    return "".join(out).encode()


@pytest.mark.parametrize("alphabet", ["ACGT", "AAAACGT", "AC", "ACGTNNN"])
@pytest.mark.parametrize("k,m", [(28, 10), (21, 5), (64, 3)])
def test_counts_vs_oracle_long_records(k, m, alphabet):
    # records of 60K bases span many 4096-window tiles; low-complexity alphabets put
    # equal-valued minimizers (expiries at ties) and the forbidden-only value 4^m
    # across tile edges
    import random
    rng = random.Random(f"{k}-{m}-{alphabet}")
    fasta = _long_records(rng, 5, 60_000, alphabet) + b">poly\n" + b"A" * 9000 + b"T" * 9000 + b"\n"
    got = _gpu_counts(fasta, k, m, seq_type=1)
    want = oracle.bin_signatures(fasta, k, m)
    assert np.array_equal(got, want), f"{int((got != want).sum())} signatures differ"


def test_streamed_ingest_and_input_kept(tmp_path):
    k, m, B = 28, 10, 2048
    fasta = fk.synth_fasta(30_000, 100, 500_000, seed=77)
    want = oracle.bin_signatures(fasta, k, m)
    assert np.array_equal(_gpu_counts(fasta, k, m, chunks=5), want)
    ref = oracle.OracleResult(fasta, k, m, B)
    with fk.KmerCounter(k, m, 3, B) as kc:
        kc.ingest(fasta)
        c1 = kc.signature_counts()
        kc.finish()  # the input is still there for the count
        assert kc.stats()["distinct"] == ref.distinct
        assert np.array_equal(kc.signature_counts().cpu().numpy(), c1.cpu().numpy())


def test_empty_and_invalid_inputs(tmp_path):
    for fasta in (b"", b"ACGTACGTACGTACGTACGTACGTACGTACGT\n", b">a\nACGTNACGTNACGTNACGTNACGTNACGTN\n", b">a\n>b\n"):
        got = _gpu_counts(fasta, 21, 7)
        assert not got.any()
        with fk.KmerCounter(21, 7, 3, 64) as kc:
            kc.ingest(fasta)
            kc.write_bin_signatures(kc.signature_counts(), str(tmp_path / "e"))
        assert _files(str(tmp_path / "e")) == {}
    with fk.KmerCounter(21, 7, 3, 64) as kc:
        kc.ingest(b">a\nACGT\n")
        small = torch.zeros(10, dtype=torch.int64, device="cuda")
        assert fk.lib().fk_signature_counts(kc._h, small.data_ptr(), 10) == -6  # FK_E_RANGE
        with pytest.raises(ValueError):
            kc.signature_counts(small)


def test_ranks_write_only_owned_bins(tmp_path):
    k, m, B, world = 28, 10, 2048, 3
    fasta = fk.synth_fasta(20_000, 100, 300_000, seed=5)
    counts = oracle.bin_signatures(fasta, k, m)
    want = _oracle_files(counts, m, B, tmp_path / "ref")
    dev_counts = torch.from_numpy(counts).cuda()
    got = {}
    for r in range(world):
        with fk.KmerCounter(k, m, 3, B, n_ranks=world, rank=r) as kc:
            d = tmp_path / f"rank{r}"
            kc.write_bin_signatures(dev_counts, str(d))
            files = _files(str(d))
            assert all(int(f[len("bin_signatures"):-4]) % world == r for f in files)
            assert not set(files) & set(got)
            got.update(files)
    assert got == want


def test_configs1_scale_linearity_and_rate():
    """configs[1] size (1 GB of 100 bp reads): counts of the whole input equal the
    sum of the counts of its two halves (cut at a record start), and the first
    20 MB match the oracle; prints the rate of the parse + signature pass."""
    import time
    rec = fk.lib().fk_synth_record_bytes(100)
    n_reads = 1_000_000_000 // rec
    k, m = 28, 10
    with fk.KmerCounter(k, m, 3, 2048) as kc:
        buf = torch.empty(n_reads * rec, dtype=torch.uint8, device="cuda")
        fk.synth_fasta_to_device(buf.data_ptr(), n_reads, 100, 100_000_000, seed=0x5EED)
        kc.ingest_device(buf.data_ptr(), buf.numel())
        full = kc.signature_counts()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            kc.signature_counts(full)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 3
        half = (n_reads // 2) * rec
        kc.ingest_device(buf.data_ptr(), half)
        a = kc.signature_counts()
        kc.ingest_device(buf.data_ptr() + half, buf.numel() - half)
        b = kc.signature_counts()
        assert torch.equal(full, a + b)
        head = (20_000_000 // rec) * rec
        kc.ingest_device(buf.data_ptr(), head)
        got = kc.signature_counts().cpu().numpy()
    want = oracle.bin_signatures(fk.synth_fasta(head // rec, 100, 100_000_000, seed=0x5EED), k, m)
    assert np.array_equal(got, want)
    print(f"\nbin signatures, 1 GB: {dt * 1e3:.2f} ms ({buf.numel() / dt / 1e9:.1f} GB/s), "
          f"{int(full.sum())} super-k-mers, {int((full != 0).sum())} signatures")


def test_execute_find_bin_signatures_job(tmp_path):
    k, m, B = 21, 7, 64
    fasta = fk.synth_fasta(5_000, 100, 100_000, seed=9, n_rate=0.01)
    path = tmp_path / "in.fa"
    path.write_bytes(fasta)
    cfg = fk.TestConfiguration(dataset=str(path), outputDirectory=str(tmp_path / "out") + "/", k=k, m=m, x=3, max_b=B)
    counts = fk.execute_find_bin_signatures_job(cfg)
    want = _oracle_files(oracle.bin_signatures(fasta, k, m), m, B, tmp_path / "ref")
    assert _files(cfg.outputDir) == want and len(want) == 64
    assert int(counts.sum()) == oracle.OracleResult(fasta, k, m, B).superkmers


def test_find_bin_signatures_one_call(tmp_path):
    """fk_find_bin_signatures (the JNI shim's findBinSignatures): counts into a
    library-owned buffer and writes the same files."""
    k, m, B = 28, 10, 2048
    fasta = fk.synth_fasta(8_000, 100, 100_000, seed=13)
    with fk.KmerCounter(k, m, 3, B) as kc:
        kc.ingest(fasta)
        assert fk.lib().fk_find_bin_signatures(kc._h, str(tmp_path / "gpu").encode()) == 0
    want = _oracle_files(oracle.bin_signatures(fasta, k, m), m, B, tmp_path / "ref")
    assert _files(str(tmp_path / "gpu")) == want
