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


def _run(fasta, k, m, x, B, use_ht=False, sequence_type=0):
    kc = fk.KmerCounter(k, m, x, B, use_ht, sequence_type)
    kc.ingest(fasta)
    kc.finish()
    return kc


@pytest.mark.parametrize("k,m,x,B", CONFIGS)
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_fused_random_vs_oracle(k, m, x, B, seed):
    rng = random.Random(1000 * seed + k + 512)
    fasta = _fasta(rng, 3000, 1, 400, noise=0.01)
    kc = _run(fasta, k, m, x, B)
    st = kc.stats()
    assert st["fused_map"] == 1, ("the fused kernel should place this input", st["fused_fallback"])
    ref = oracle.OracleResult(fasta, k, m, B)
    assert st["kmers"] == ref.total_kmers
    assert_same_as_oracle(kc, ref)


def test_fused_short_reads_both_modes():
    fasta = fk.synth_fasta(40_000, 100, 500_000, seed=77)
    ref = oracle.OracleResult(fasta, 28, 10, 2048)
    for use_ht in (False, True):
        kc = _run(fasta, 28, 10, 3, 2048, use_ht)
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
                                  "header_across_tiles", "header_at_chunk_start", "tiny", "empty",
                                  "no_newline_end", "blank_lines"])
def test_fused_edge_inputs_vs_oracle(case):
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
    elif case == "header_at_chunk_start":
        # 256-byte records: every header starts right after a newline at the last byte of a thread's
        # 64-byte chunk and runs through the next chunk (its line state comes from that newline's
        # thread); the headers are A/C/G/T text, so counting them as sequence would show
        fasta = b"".join(b">" + "".join(rng.choice("ACGT") for _ in range(148)).encode() + b"\n" +
                         "".join(rng.choice("ACGT") for _ in range(105)).encode() + b"\n" for _ in range(600))
    elif case == "tiny":
        fasta = b">r\nACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTAC\n"
    elif case == "empty":
        fasta = b""
        expect_fused = False
    else:  # the last line has no trailing newline
        fasta = _fasta(rng, 500, 50, 300).rstrip(b"\n")
    for k, m, x, B in CONFIGS:
        kc = _run(fasta, k, m, x, B)
        ref = oracle.OracleResult(fasta, k, m, B)
        st = kc.stats()
        assert st["kmers"] == ref.total_kmers
        assert_same_as_oracle(kc, ref)
        if case not in ("tiny",):
            assert st["fused_map"] == (1 if expect_fused else 0), (case, st["fused_fallback"])
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
    assert kc.stats()["fused_map"] == 1, kc.stats()["fused_fallback"]
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


# ---------------------------------------------------------------- streamed ingest (fk_ingest segments)

def _stream(kc, data: bytes, sizes, last_flag=True):
    off = 0
    for i, n in enumerate(sizes):
        chunk = data[off:off + n]
        off += n
        kc.ingest_chunk(chunk, last_flag and off >= len(data))
        if off >= len(data):
            break
    if off < len(data):
        kc.ingest_chunk(data[off:], last_flag)


@pytest.mark.parametrize("reserve,last_flag", [(True, True), (False, True), (False, False)])
def test_streamed_ingest_chunks_vs_oracle(reserve, last_flag):
    # chunks of random sizes (1 byte .. 300 kB): tiles are mapped as their bytes and halo land,
    # the input buffer, look-back words and records grow mid-stream without reserve, and without
    # a final last=1 chunk fk_map launches the remaining tiles
    rng = random.Random(31)
    data = _fasta(rng, 6000, 20, 400)
    sizes = [rng.choice([1, 7, 100, 4096, 30_000, 65_536, 300_000]) for _ in range(400)]
    for k, m, x, B in CONFIGS:
        kc = fk.KmerCounter(k, m, x, B)
        if reserve:
            kc.reserve(len(data))
        _stream(kc, data, sizes, last_flag)
        kc.finish()
        assert kc.stats()["fused_map"] == 1
        ref = oracle.OracleResult(data, k, m, B)
        assert kc.stats()["kmers"] == ref.total_kmers
        assert_same_as_oracle(kc, ref)
        # the context is reused for a second job (the previous records are not carried over)
        _stream(kc, data[: len(data) // 3], [50_000] * 100, True)
        kc.finish()
        ref2 = oracle.OracleResult(data[: len(data) // 3], k, m, B)
        assert_same_as_oracle(kc, ref2)
        kc.close()


def test_streamed_ingest_fallback_vs_oracle():
    # a long header line straddling tile starts: the streamed fused map raises the fallback
    # flag and fk_map maps the resident input with the two-kernel path
    rng = random.Random(32)
    body = b""
    while len(body) < 59_500:
        body += _fasta(rng, 1, 50, 200)
    data = body + b">" + b"h" * 10_000 + b"\n" + _fasta(rng, 3000, 50, 200)[1:]
    kc = fk.KmerCounter(28, 10, 3, 2048)
    _stream(kc, data, [20_000] * 100)
    kc.finish()
    assert kc.stats()["fused_map"] == 0
    assert_same_as_oracle(kc, oracle.OracleResult(data, 28, 10, 2048))


def test_streamed_long_record_sequence_type1_vs_oracle():
    rng = random.Random(33)
    seq = "".join(rng.choice("ACGT") for _ in range(400_000))
    seq = seq[:100_000] + "N" * 2000 + seq[102_000:]
    data = (">chrU\n" + "\n".join(seq[q:q + 60] for q in range(0, len(seq), 60)) + "\n").encode()
    kc = fk.KmerCounter(28, 10, 3, 2048, sequence_type=1)
    _stream(kc, data, [33_333] * 100)
    kc.finish()
    assert kc.stats()["fused_map"] == 1, kc.stats()["fused_fallback"]
    assert_same_as_oracle(kc, oracle.OracleResult(data, 28, 10, 2048, 1))


def test_pinned_ingest_overlapped_vs_oracle():
    # 64 MB from pinned host memory: 32 MB DMA segments on the copy stream, the fused map of
    # each landed segment overlapping the next copy
    import torch
    n_reads = 64_000_000 // 114
    data = fk.synth_fasta(n_reads, 100, 2_000_000, seed=34)
    pinned = torch.empty(len(data), dtype=torch.uint8).pin_memory()
    pinned.numpy()[:] = np.frombuffer(data, dtype=np.uint8)
    kc = fk.KmerCounter(28, 10, 3, 2048)
    for _ in range(2):  # the second job reuses the context's buffers
        kc.ingest_ptr(pinned.data_ptr(), len(data))
        kc.finish()
        st = kc.stats()
        assert st["fused_map"] == 1 and st["ms_h2d"] > 0
    ref = oracle.OracleResult(data, 28, 10, 2048, threads=8)
    assert st["kmers"] == ref.total_kmers
    assert_same_as_oracle(kc, ref)
