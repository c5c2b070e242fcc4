"""HIP path vs the CPU oracle, through the C-ABI (needs an MI355X).

Bit-exact: every bin's (canonical k-mer, count) list must equal the
oracle's, in the same (ascending) order for useHT=0 and as a set for
useHT=1, and written bin files must be byte-identical to the reference
format.  Golden fixtures (tests/golden) pin the small cases; seeded synthetic
inputs cover the BASELINE configurations at sizes the oracle finishes in
seconds; size-independent properties cover the full 1 GB configuration.
"""
import json
import os
import random
import subprocess

import numpy as np
import pytest

import fastkmer_amd as fk
import oracle
from conftest import GOLDEN, golden_cases

pytestmark = pytest.mark.gpu


def counter_arrays(kc, b):
    keys, counts = kc.get_bin(b)
    if kc.k > 32:
        keys = keys.reshape(-1, 2)
        return keys[:, 0].copy(), keys[:, 1].copy(), counts
    return np.zeros(len(keys), dtype=np.uint64), keys, counts


def assert_same_as_oracle(kc, ref, ordered=True):
    sizes = kc.bin_sizes()
    assert len(sizes) == ref.nbins
    ref_sizes = ref.bin_sizes()
    bad = np.nonzero(sizes.astype(np.int64) != ref_sizes)[0]
    assert len(bad) == 0, f"bin sizes differ in {len(bad)} bins, e.g. bin {bad[:5]}"
    for b in np.nonzero(ref_sizes)[0].tolist():
        hi, lo, cnt = counter_arrays(kc, b)
        rhi, rlo, rcnt = ref.bin_arrays(b)
        if not ordered:
            order = np.lexsort((lo, hi))
            hi, lo, cnt = hi[order], lo[order], cnt[order]
        assert np.array_equal(hi, rhi) and np.array_equal(lo, rlo), f"keys differ in bin {b}"
        assert np.array_equal(cnt, rcnt), f"counts differ in bin {b}"


def run_counter(fasta, k, m, x=3, B=2048, use_ht=False, sequence_type=0):
    kc = fk.KmerCounter(k, m, x, B, use_ht, sequence_type)
    kc.ingest(fasta)
    kc.finish()
    return kc


def load_golden(name):
    with open(os.path.join(GOLDEN, name + ".fa"), "rb") as f:
        fasta = f.read()
    with open(os.path.join(GOLDEN, name + ".expected.json")) as f:
        expected = json.load(f)
    return fasta, expected


@pytest.mark.parametrize("name", sorted(golden_cases()))
def test_golden_sorted(name):
    p = golden_cases()[name]
    fasta, expected = load_golden(name)
    kc = run_counter(fasta, p["k"], p["m"], p["x"], p["B"], False, p.get("sequence_type", 0))
    sizes = kc.bin_sizes()
    got = {f"bin{b}": kc.bin_text(b) for b in np.nonzero(sizes)[0].tolist()}
    assert got == expected
    assert kc.stats()["kmers"] == p["total_kmers"]


@pytest.mark.parametrize("name", sorted(golden_cases()))
def test_golden_hash(name):
    p = golden_cases()[name]
    fasta, expected = load_golden(name)
    kc = run_counter(fasta, p["k"], p["m"], p["x"], p["B"], True, p.get("sequence_type", 0))
    got = {}
    for b in np.nonzero(kc.bin_sizes())[0].tolist():
        text = kc.bin_text(b)
        assert not text.endswith("EOF")
        got[f"bin{b}"] = sorted(text.splitlines())
    exp = {b: sorted(t[:-3].splitlines()) for b, t in expected.items()}
    assert got == exp


def test_write_bins_byte_identical(tmp_path):
    fasta, expected = load_golden("short_reads_k28")
    kc = run_counter(fasta, 28, 10, 3, 2048)
    out = tmp_path / "out"
    kc.write_bins(str(out))
    files = {f: (out / f).read_text() for f in os.listdir(out)}
    assert files == expected


def test_cli_matches_reference_layout(tmp_path):
    fasta, expected = load_golden("short_reads_k28")
    inp = tmp_path / "in.fa"
    inp.write_bytes(fasta)
    r = subprocess.run([fk.CLI_PATH, "LocalTestKmerCounter", "28", "10", "3", "2048", "0", "0", str(inp),
                        str(tmp_path) + "/", "run_", "1", "0", "0"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    outdir = tmp_path / "run_k28_m10_x3_b2048_s0"
    files = {f: (outdir / f).read_text() for f in os.listdir(outdir)}
    assert files == expected
    # useHT=1 writes the same lines without EOF
    r = subprocess.run([fk.CLI_PATH, "28", "10", "3", "2048", "1", "0", str(inp), str(tmp_path) + "/", "ht_",
                        "1", "0", "1", "4"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    outdir = tmp_path / "ht_k28_m10_x3_b2048_s0"
    files = {f: sorted((outdir / f).read_text().splitlines()) for f in os.listdir(outdir)}
    assert files == {b: sorted(t[:-3].splitlines()) for b, t in expected.items()}


def random_fasta(rng, nreads, lo, hi, alphabet="ACGT", noise="", noise_p=0.0, wrap=0):
    out = []
    for i in range(nreads):
        s = "".join(rng.choice(alphabet) for _ in range(rng.randint(lo, hi)))
        if noise:
            s = "".join(rng.choice(noise) if rng.random() < noise_p else ch for ch in s)
        if wrap and s:
            s = "\n".join(s[q:q + wrap] for q in range(0, len(s), wrap))
        out.append(f">read{i} some header ACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGTACGT\n{s}\n")
    return "".join(out).encode()


@pytest.mark.parametrize("seed", range(24))
def test_random_vs_oracle(seed):
    rng = random.Random(seed)
    k = rng.choice([5, 11, 15, 21, 27, 28, 31, 32, 33, 40, 55, 63, 64])
    m = min(k, rng.choice([1, 2, 3, 5, 7, 9, 10, 12, 15]))
    B = rng.choice([1, 3, 64, 1000, 2048, 8192])
    use_ht = bool(seed % 3 == 0)
    fasta = random_fasta(rng, rng.randint(1, 300), 0, rng.choice([60, 200, 800]),
                         alphabet=rng.choice(["ACGT", "ACGT", "AC", "GT", "ACGTN"]),
                         noise=rng.choice(["", "Nn\r", "acgtRY"]), noise_p=0.01, wrap=rng.choice([0, 0, 7, 61]))
    kc = run_counter(fasta, k, m, 3, B, use_ht)
    ref = oracle.OracleResult(fasta, k, m, B)
    assert kc.stats()["kmers"] == ref.total_kmers
    assert_same_as_oracle(kc, ref, ordered=not use_ht)


@pytest.mark.parametrize("use_ht", [False, True])
def test_baseline_c1_synthetic_vs_oracle(use_ht):
    # BASELINE configs[0]: k=28 m=10 x=3 B=2048, 10 MB synthetic 100 bp reads
    n_reads = 10_000_000 // 114
    fasta = fk.synth_fasta(n_reads, 100, 1_000_000, seed=0x5EED)
    kc = run_counter(fasta, 28, 10, 3, 2048, use_ht)
    ref = oracle.OracleResult(fasta, 28, 10, 2048)
    assert kc.stats()["kmers"] == ref.total_kmers
    assert_same_as_oracle(kc, ref, ordered=not use_ht)


def test_two_word_k55_vs_oracle():
    # BASELINE configs[3] shape (k=55 m=12, 150 bp) at oracle-friendly size
    fasta = fk.synth_fasta(20_000, 150, 200_000, seed=11)
    for use_ht in (False, True):
        kc = run_counter(fasta, 55, 12, 3, 8192, use_ht)
        ref = oracle.OracleResult(fasta, 55, 12, 8192)
        assert_same_as_oracle(kc, ref, ordered=not use_ht)


def test_long_sequence_type1_vs_oracle():
    # BASELINE configs[4] shape: one long record, 60-column lines, N runs, soft-masked lowercase
    rng = random.Random(5)
    seq = []
    for blk in range(40):
        s = "".join(rng.choice("ACGT") for _ in range(50_000))
        if blk % 7 == 3:
            s = s[:1000] + "N" * 3000 + s[4000:]
        if blk % 5 == 1:
            s = s[:20_000] + s[20_000:30_000].lower() + s[30_000:]
        seq.append(s)
    seq = "".join(seq)
    fasta = (">chrSynthetic\n" + "\n".join(seq[q:q + 60] for q in range(0, len(seq), 60)) + "\n").encode()
    kc = run_counter(fasta, 28, 10, 3, 2048, False, sequence_type=1)
    ref = oracle.OracleResult(fasta, 28, 10, 2048, 1)
    assert_same_as_oracle(kc, ref)


@pytest.mark.parametrize("l1", ["512", "1024"])
def test_long_record_level1_kernels_vs_oracle(monkeypatch, l1):
    # one long record, 60 % of it periodic blocks (a minimizer that never changes: records of 16
    # k-mers), so records average > 9 k-mers and a 1024-record level-1 batch of k_expand_sc1024
    # overflows its 8192-key stage and is stored from registers; both level-1 kernels against the
    # oracle (FASTKMER_X2_L1 forces the kernel at any fan-out)
    monkeypatch.setenv("FASTKMER_X2_L1", l1)
    rng = random.Random(11)
    parts = []
    for blk in range(60):
        if blk % 5 < 3:
            unit = "".join(rng.choice("ACGT") for _ in range(rng.randint(5, 9)))
            parts.append((unit * (25_000 // len(unit) + 1))[:25_000])
        else:
            parts.append("".join(rng.choice("ACGT") for _ in range(25_000)))
    seq = "".join(parts)
    fasta = (">chrL\n" + "\n".join(seq[q:q + 80] for q in range(0, len(seq), 80)) + "\n").encode()
    kc = run_counter(fasta, 28, 10, 3, 64, False, sequence_type=1)
    ref = oracle.OracleResult(fasta, 28, 10, 64, 1)
    st = kc.stats()
    assert st["kmers"] == ref.total_kmers and st["kmers"] > 9.0 * st["superkmers"]
    assert_same_as_oracle(kc, ref)


def test_large_bucket_path_vs_oracle(monkeypatch):
    # every bucket through the streaming global-memory sort (k_bucket_sort_large)
    monkeypatch.setenv("FASTKMER_DEBUG_LARGE_BUCKETS", "1")
    fasta = fk.synth_fasta(3000, 100, 20_000, seed=3)
    for k, m in ((28, 10), (41, 9)):
        kc = run_counter(fasta, k, m, 3, 16)
        assert kc.stats()["oversize_buckets"] > 0
        ref = oracle.OracleResult(fasta, k, m, 16)
        assert_same_as_oracle(kc, ref)


@pytest.mark.parametrize("use_ht", [False, True])
def test_many_bins_global_partition_vs_oracle(use_ht):
    # b = 20000 bins > PART_MAX: the record partition takes its global-atomic path
    fasta = fk.synth_fasta(8000, 100, 200_000, seed=31)
    kc = run_counter(fasta, 24, 9, 3, 20000, use_ht)
    ref = oracle.OracleResult(fasta, 24, 9, 20000)
    assert_same_as_oracle(kc, ref, ordered=not use_ht)


def test_skewed_repeats_vs_oracle():
    # one k-mer repeated ~100k times, poly-A/poly-C blocks: single cells far above the LDS capacity
    fasta = (b">a\n" + b"A" * 100_000 + b"\n>b\n" + b"AC" * 60_000 + b"\n>c\n" + b"ACGTTGCA" * 20_000 + b"\n")
    for use_ht in (False, True):
        kc = run_counter(fasta, 21, 7, 3, 64, use_ht)
        ref = oracle.OracleResult(fasta, 21, 7, 64)
        assert_same_as_oracle(kc, ref, ordered=not use_ht)


@pytest.mark.parametrize("data", [b"", b"ACGT\n", b">only\n", b">a\nACG\n>b\n\n>c\nNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNNN\n"])
def test_empty_and_degenerate(data):
    kc = run_counter(data, 21, 7, 3, 64)
    assert int(kc.bin_sizes().sum()) == 0
    assert kc.stats()["kmers"] == 0


def test_multi_rank_in_one_process_matches_single():
    # the exchange path without RCCL: 3 ranks, records routed by bin % 3
    fasta = fk.synth_fasta(20_000, 100, 300_000, seed=9)
    rec = 114
    G = 3
    shards = [fasta[r * rec * 7000:(r + 1) * rec * 7000] for r in range(G)]
    ranks = [fk.KmerCounter(28, 10, 3, 2048, False, 0, n_ranks=G, rank=r) for r in range(G)]
    import torch
    sends = []
    for r in range(G):
        ranks[r].ingest(shards[r])
        counts = ranks[r].map()
        buf = torch.empty(max(sum(counts), 1) * ranks[r].record_bytes, dtype=torch.uint8, device="cuda")
        ranks[r].map_emit(buf.data_ptr(), max(sum(counts), 1))
        torch.cuda.synchronize()
        sends.append((buf, counts))
    rb = ranks[0].record_bytes
    for dst in range(G):
        parts = []
        for src in range(G):
            buf, counts = sends[src]
            off = sum(counts[:dst])
            parts.append(buf[off * rb:(off + counts[dst]) * rb])
        recv = torch.cat(parts) if parts else torch.empty(0, dtype=torch.uint8, device="cuda")
        ranks[dst].reduce(recv.data_ptr(), recv.numel() // rb)
        torch.cuda.synchronize()
    ref = oracle.OracleResult(fasta, 28, 10, 2048)
    ref_sizes = ref.bin_sizes()
    for dst in range(G):
        sizes = ranks[dst].bin_sizes()
        for b in range(ref.nbins):
            if b % G != dst:
                assert sizes[b] == 0
                continue
            assert sizes[b] == ref_sizes[b]
            if ref_sizes[b]:
                hi, lo, cnt = counter_arrays(ranks[dst], b)
                rhi, rlo, rcnt = ref.bin_arrays(b)
                assert np.array_equal(lo, rlo) and np.array_equal(cnt, rcnt)


@pytest.mark.parametrize("use_ht", [False, True])
def test_size_aware_placement_in_one_process(use_ht):
    # useCustomPartitioner: exact per-bin sizes summed over 3 ranks, LPT owners, records routed by the table
    fasta = fk.synth_fasta(20_000, 100, 300_000, seed=19)
    G, rec = 3, 114
    shards = [fasta[r * rec * 7000:(r + 1) * rec * 7000] for r in range(G)]
    ranks = [fk.KmerCounter(28, 10, 3, 2048, use_ht, 0, n_ranks=G, rank=r) for r in range(G)]
    import torch
    sizes = np.zeros(2048, dtype=np.uint64)
    for r in range(G):
        ranks[r].ingest(shards[r])
        ranks[r].map()
        sizes += ranks[r].map_bin_kmers()
    owner = fk.lpt_owners(sizes, G)
    loads = np.bincount(owner, weights=sizes.astype(np.float64), minlength=G)
    assert loads.max() / loads.mean() < 1.01
    sends = []
    for r in range(G):
        counts = ranks[r].set_bin_owners(owner)
        buf = torch.empty(max(sum(counts), 1) * ranks[r].record_bytes, dtype=torch.uint8, device="cuda")
        ranks[r].map_emit(buf.data_ptr(), max(sum(counts), 1))
        torch.cuda.synchronize()
        sends.append((buf, counts))
    rb = ranks[0].record_bytes
    for dst in range(G):
        parts = []
        for src in range(G):
            buf, counts = sends[src]
            off = sum(counts[:dst])
            parts.append(buf[off * rb:(off + counts[dst]) * rb])
        recv = torch.cat(parts)
        ranks[dst].reduce(recv.data_ptr(), recv.numel() // rb)
        torch.cuda.synchronize()
    ref = oracle.OracleResult(fasta, 28, 10, 2048)
    ref_sizes = ref.bin_sizes()
    for dst in range(G):
        got = ranks[dst].bin_sizes()
        for b in range(ref.nbins):
            assert got[b] == (ref_sizes[b] if owner[b] == dst else 0)
            if owner[b] == dst and ref_sizes[b] and b % 97 == 0:
                hi, lo, cnt = counter_arrays(ranks[dst], b)
                rhi, rlo, rcnt = ref.bin_arrays(b)
                if use_ht:
                    order = np.argsort(lo)
                    lo, cnt = lo[order], cnt[order]
                assert np.array_equal(lo, rlo) and np.array_equal(cnt, rcnt)


def test_chunked_and_pinned_ingest():
    # fk_ingest appends: uneven chunks split inside records equal one call; a pinned
    # source (DMA path) equals a pageable one (staged path)
    import torch
    fasta = fk.synth_fasta(20_000, 100, 300_000, seed=37)
    ref = oracle.OracleResult(fasta, 28, 10, 2048)
    kc = fk.KmerCounter(28, 10, 3, 2048)
    cuts = [0, 1, 777_777, 1_500_001, len(fasta)]
    for a, b in zip(cuts[:-1], cuts[1:]):
        kc.ingest(fasta[a:b])
    kc.finish()
    assert_same_as_oracle(kc, ref)
    kc.finish()  # the same input again
    assert_same_as_oracle(kc, ref)
    pinned = torch.frombuffer(bytearray(fasta), dtype=torch.uint8).pin_memory()
    kc.ingest_ptr(pinned.data_ptr(), pinned.numel())  # a new input after finish
    kc.finish()
    assert_same_as_oracle(kc, ref)


def test_large_staged_ingest_matches_device_input():
    # > 2 staging buffers (64 MB each) of pageable input == the same bytes generated on the device
    n_reads = 1_500_000  # 171 MB
    host = fk.synth_fasta(n_reads, 100, 5_000_000, seed=41)
    a = fk.KmerCounter(25, 9, 3, 512)
    a.ingest(host)
    a.finish()
    b = fk.KmerCounter(25, 9, 3, 512)
    assert b.synth_device(n_reads, 100, 5_000_000, seed=41) == len(host)
    b.finish()
    assert np.array_equal(a.bin_sizes(), b.bin_sizes())
    for bin_ in (0, 17, 511):
        ka, ca = a.get_bin(bin_)
        kb, cb = b.get_bin(bin_)
        assert np.array_equal(ka, kb) and np.array_equal(ca, cb)


def test_device_synth_matches_host():
    import torch
    kc = fk.KmerCounter(28, 10, 3, 2048)
    nb = kc.synth_device(5000, 100, 100_000, seed=42)
    host = fk.synth_fasta(5000, 100, 100_000, seed=42)
    assert nb == len(host)
    kc.finish()
    ref = oracle.OracleResult(host, 28, 10, 2048)
    assert_same_as_oracle(kc, ref)


def test_full_size_properties():
    # BASELINE configs[1] (1 GB, k=28 m=10 B=2048) through size-independent properties:
    # counts sum to the k-mer windows, each bin is strictly ascending, and a sample of
    # k-mers re-hashes (oracle norm + hash_to_bucket) to the bin it was filed under.
    n_reads = 1_000_000_000 // 114
    kc = fk.KmerCounter(28, 10, 3, 2048)
    kc.synth_device(n_reads, 100, 100_000_000, seed=0x5EED)
    kc.finish()
    st = kc.stats()
    sizes = kc.bin_sizes()
    total = 0
    rng = random.Random(0)
    sample_bins = rng.sample(np.nonzero(sizes)[0].tolist(), 16)
    for b in sample_bins:
        keys, counts = kc.get_bin(b)
        assert np.all(keys[1:] > keys[:-1])
        for kk in rng.sample(fk.decode_keys(keys, 28), 20):
            sig = min(oracle.norm(int("".join("%d" % "ACGT".index(ch) for ch in kk[j:j + 10]), 4), 10)
                      for j in range(19))
            assert oracle.hash_to_bucket(sig, 2048) == b
    all_counts = 0
    for b in np.nonzero(sizes)[0].tolist():
        _, counts = kc.get_bin(b)
        all_counts += int(counts.sum(dtype=np.uint64))
    assert st["distinct"] == int(sizes.sum())
    assert all_counts == st["kmers"]
    assert st["kmers"] > 0.9 * n_reads * 73


@pytest.mark.parametrize("k,m", [(28, 10), (55, 12)])
def test_max_fine_bits_one_bin_vs_oracle(monkeypatch, k, m):
    # B = 1: every k-mer in one bin (4.4 M at k = 28, 2.8 M at k = 55), past 2^14 cells of 128 keys
    # (FASTKMER_DEBUG_CELL_TARGET; 64-bit keys default to 512 per cell), so the bin is cut into the
    # most cells (F = MAX_FINE_BITS = 15: the histogram, flag and scatter kernels at 128 KB of LDS) --
    # the largest-F path against the oracle
    monkeypatch.setenv("FASTKMER_DEBUG_CELL_TARGET", "128")
    fasta = fk.synth_fasta(60_000, 100, 10_000_000, seed=67)
    kc = run_counter(fasta, k, m, 3, 1)
    st = kc.stats()
    assert st["fine_bits"] == 15
    ref = oracle.OracleResult(fasta, k, m, 1)
    assert st["kmers"] == ref.total_kmers
    assert_same_as_oracle(kc, ref)


def test_big_bins_two_level_vs_oracle():
    # few, large bins (~800K k-mers each): 2^11 cells per bin, 32 super-cells
    # (the two-level expansion with F1 > 0) and all three count tiers
    fasta = fk.synth_fasta(350_000, 100, 3_000_000, seed=53)
    kc = run_counter(fasta, 28, 10, 3, 32)
    st = kc.stats()
    assert st["fine_bits"] >= 9
    ref = oracle.OracleResult(fasta, 28, 10, 32)
    assert st["kmers"] == ref.total_kmers
    assert_same_as_oracle(kc, ref)


def test_block_and_big_tiers_vs_oracle(monkeypatch):
    # few large bins of a mostly distinct input (~1.4 M k-mers per bin) cut into cells of up to ~2600 keys
    # (FASTKMER_DEBUG_CELL_TARGET): buckets of 513..2048 keys (the block kernel) and above (the
    # 6144-slot big-table kernel, the streaming path past 4096 distinct keys) -- at configs[2]'s
    # per-GPU bins, the cells of the k-mers that start with a frequent minimizer
    monkeypatch.setenv("FASTKMER_DEBUG_CELL_TARGET", "2600")
    fasta = fk.synth_fasta(300_000, 100, 3_000_000_000, seed=71)
    kc = run_counter(fasta, 28, 10, 3, 16)
    st = kc.stats()
    assert st["block_buckets"] > 1000 and st["big_buckets"] > 1000, st
    ref = oracle.OracleResult(fasta, 28, 10, 16, threads=4)
    assert st["kmers"] == ref.total_kmers
    assert_same_as_oracle(kc, ref)


@pytest.mark.parametrize("cell_target,staged,use_ht,mode,genome", [
    (700, False, False, 1, 3_000_000_000), (700, True, False, 1, 3_000_000_000), (700, False, True, 1, 3_000_000_000),
    (400, False, False, 1, 3_000_000_000), (700, False, False, 2, 2_000_000), (700, True, False, 2, 2_000_000),
    (700, False, True, 2, 2_000_000), (700, False, False, 2, 3_000_000_000)])
def test_mid_tier_key_ranges_vs_oracle(monkeypatch, cell_target, staged, use_ht, mode, genome):
    # cells of ~700 (~400) keys: many buckets of 513..1024 keys.  mode 1: the 64-bit mid tier counts them
    # as 2 or 3 key ranges on the wave tier's table (k_bucket_count64_parts); 600 copies of a few reads
    # put k-mers repeated 600 times into some of them, a range above 512 keys that the 1024-key kernel
    # takes over.  mode 2: whole on the wave tier's table (k_bucket_count64_mid512) -- reads of a 2 Mbp
    # genome (10x: ~100 distinct keys per bucket), and of a 3 Gbp one, whose buckets hold more than 512
    # distinct keys and give up to the 1024-key kernel
    monkeypatch.setenv("FASTKMER_DEBUG_CELL_TARGET", str(cell_target))
    monkeypatch.setenv("FASTKMER_DEBUG_MID_PARTS", str(mode))  # the product picks by the mid tier's size
    rep = b"".join(b">r%d\n" % i + b"GATTACAGGCATCGATCGGGCTAGCTAGGCTAGCTTACGAGCTAGCATCGACTAGCATGCATGCATCGACGTAGCATCG"
                   b"ACGTTGCAAGGCTTACCGATCGG\n" for i in range(600))
    fasta = fk.synth_fasta(200_000, 100, genome, seed=0x7A + cell_target) + rep
    if staged:
        import torch
        monkeypatch.setenv("FASTKMER_INGEST_SEG", str(1 << 20))
        monkeypatch.setenv("FASTKMER_PIECE_BYTES", str(2 << 20))
        host = torch.frombuffer(bytearray(fasta), dtype=torch.uint8).pin_memory()
        kc = fk.KmerCounter(28, 10, 3, 16, use_ht=use_ht)
        kc.ingest_ptr(host.data_ptr(), host.numel())
        kc.finish()
        assert kc.stats()["pieces_counted"] > 1
    else:
        kc = run_counter(fasta, 28, 10, 3, 16, use_ht=use_ht)
    st = kc.stats()
    assert st["block_buckets"] > (1000 if cell_target >= 700 else 100), st
    ref = oracle.OracleResult(fasta, 28, 10, 16, threads=4)
    assert st["kmers"] == ref.total_kmers
    assert_same_as_oracle(kc, ref, ordered=not use_ht)


@pytest.mark.parametrize("k,m", [(28, 10), (55, 12)])
def test_wave_tables_of_distinct_keys_vs_oracle(k, m):
    # reads of a 3 Gbp virtual genome: nearly every k-mer is distinct, so the
    # wave buckets (512 keys; 256 two-word keys for k > 32) fill their tables
    # with as many distinct keys (2/3 of the 768 / 384 slots: the longest
    # probe runs)
    fasta = fk.synth_fasta(100_000, 100, 3_000_000_000, seed=61)
    kc = run_counter(fasta, k, m, 3, 64)
    ref = oracle.OracleResult(fasta, k, m, 64)
    assert kc.stats()["distinct"] > 0.95 * ref.total_kmers
    assert_same_as_oracle(kc, ref)


@pytest.mark.parametrize("env", [
    {"FASTKMER_DEBUG_LARGE_BUCKETS": "1"},                           # every bucket through the streaming path
    {"FASTKMER_DEBUG_CELL_TARGET": "64"},                            # small cells: many small buckets
    {"FASTKMER_DEBUG_CELL_TARGET": "2600"},                          # large cells: block and big tiers
    {"FASTKMER_X2_L1": "1024"},                                      # 1024-record level-1 batches
    {"FASTKMER_FUSED": "0"},                                         # the two-kernel map
])
def test_count_variants_identical(monkeypatch, env):
    # every count-stage variant gives the default path's result, bit for bit
    fasta = fk.synth_fasta(120_000, 100, 1_000_000, seed=59)
    base = run_counter(fasta, 27, 9, 3, 128)
    for key, val in env.items():
        monkeypatch.setenv(key, val)
    alt = run_counter(fasta, 27, 9, 3, 128)
    assert np.array_equal(base.bin_sizes(), alt.bin_sizes())
    for b in range(0, 128, 7):
        kb, cb = base.get_bin(b)
        ka, ca = alt.get_bin(b)
        assert np.array_equal(kb, ka) and np.array_equal(cb, ca)


@pytest.mark.parametrize("case", ["long_lines", "text_before_header", "wrapped"])
def test_parse_line_lookback_paths_vs_oracle(monkeypatch, case):
    # the parse finds the line holding each tile start by reading back 4 KB;
    # lines longer than that (sequence or header) and text before the first
    # header take the look-back rerun, which must give the same result
    rng = random.Random(77)
    if case == "long_lines":
        big = "".join(rng.choice("ACGT") for _ in range(40_000))
        hdr = "".join(rng.choice("ACGT>x ") for _ in range(30_000))
        fasta = (random_fasta(rng, 200, 50, 150) + f">big\n{big}\n>{hdr}\nACGTTGCAACGTGGCCA\n".encode()
                 + random_fasta(rng, 200, 50, 150))
    elif case == "text_before_header":
        fasta = b"ACGTACGTTTGACCAGGGTACCA\nGGGTTTACCAGT\n" + random_fasta(rng, 500, 50, 300)
    else:  # wrapped lines through the two-kernel path's scan variant
        monkeypatch.setenv("FASTKMER_FUSED", "0")
        fasta = random_fasta(rng, 2000, 50, 300, wrap=61)
    for k, m in ((28, 10), (55, 12)):
        kc = run_counter(fasta, k, m, 3, 512)
        ref = oracle.OracleResult(fasta, k, m, 512)
        assert kc.stats()["kmers"] == ref.total_kmers
        assert_same_as_oracle(kc, ref)


@pytest.mark.parametrize("k,m,B,use_ht", [(28, 10, 2048, False), (28, 10, 2048, True), (55, 12, 8192, False)])
def test_grouped_exchange_in_one_process_matches_oracle(k, m, B, use_ht):
    # fk_set_grouped_emit / fk_reduce_grouped: senders group records by
    # (destination, local bin); receivers count the segments without a partition pass
    fasta = fk.synth_fasta(20_000, 150 if k > 32 else 100, 300_000, seed=13)
    G = 3
    rec = len(fasta) // 20_000
    shards = [fasta[r * rec * 6667:(r + 1) * rec * 6667] if r < G - 1 else fasta[r * rec * 6667:]
              for r in range(G)]
    ranks = [fk.KmerCounter(k, m, 3, B, use_ht, 0, n_ranks=G, rank=r) for r in range(G)]
    import torch
    sends = []
    for r in range(G):
        parts = ranks[r].set_grouped_emit(True)
        ranks[r].ingest(shards[r])
        counts = ranks[r].map()
        prec, pkm = ranks[r].map_part_counts()
        assert prec.shape == (G, parts) and [int(x) for x in prec.sum(axis=1)] == counts
        buf = torch.empty(max(sum(counts), 1) * ranks[r].record_bytes, dtype=torch.uint8, device="cuda")
        ranks[r].map_emit(buf.data_ptr(), max(sum(counts), 1))
        torch.cuda.synchronize()
        sends.append((buf, counts, prec, pkm))
    rb = ranks[0].record_bytes
    for dst in range(G):
        pieces, seg_rec, seg_km = [], [], []
        for src in range(G):
            buf, counts, prec, pkm = sends[src]
            off = sum(counts[:dst])
            pieces.append(buf[off * rb:(off + counts[dst]) * rb])
            seg_rec.append(prec[dst])
            seg_km.append(pkm[dst])
        recv = torch.cat(pieces)
        ranks[dst].reduce_grouped(recv.data_ptr(), recv.numel() // rb, np.stack(seg_rec), np.stack(seg_km))
        torch.cuda.synchronize()
    ref = oracle.OracleResult(fasta, k, m, B)
    total = np.zeros(ref.nbins, dtype=np.int64)
    for dst in range(G):
        sizes = ranks[dst].bin_sizes().astype(np.int64)
        assert all(sizes[b] == 0 for b in range(ref.nbins) if b % G != dst)
        total += sizes
    assert np.array_equal(total, ref.bin_sizes())
    for b in range(0, ref.nbins, 37):
        if ref.bin_size(b):
            hi, lo, cnt = counter_arrays(ranks[b % G], b)
            rhi, rlo, rcnt = ref.bin_arrays(b)
            if use_ht:
                o = np.lexsort((lo, hi))
                hi, lo, cnt = hi[o], lo[o], cnt[o]
            assert np.array_equal(hi, rhi) and np.array_equal(lo, rlo) and np.array_equal(cnt, rcnt)


@pytest.mark.parametrize("k,m,B", [(28, 10, 2048), (55, 12, 8192)])
def test_grouped_emit_with_owners_set_after_map(k, m, B):
    # the caller-driven custom-partitioner flow: fk_set_grouped_emit, fk_map,
    # fk_map_bin_kmers, LPT over the summed sizes, fk_set_bin_owners -- which must keep the mapped
    # records and recompute their (owner, local bin) parts -- then fk_map_emit / fk_reduce_grouped
    fasta = fk.synth_fasta(18_000, 150 if k > 32 else 100, 400_000, seed=83)
    G = 3
    rec = len(fasta) // 18_000
    shards = [fasta[r * rec * 6000:(r + 1) * rec * 6000] for r in range(G)]
    ranks = [fk.KmerCounter(k, m, 3, B, False, 0, n_ranks=G, rank=r) for r in range(G)]
    import torch
    sizes = np.zeros(ranks[0].num_bins, dtype=np.uint64)
    for r in range(G):
        ranks[r].set_grouped_emit(True)
        ranks[r].ingest(shards[r])
        ranks[r].map()
        sizes += ranks[r].map_bin_kmers()
    owner = fk.lpt_owners(sizes, G)
    assert (owner != np.arange(len(owner)) % G).any()  # not the default placement
    sends = []
    for r in range(G):
        counts = ranks[r].set_bin_owners(owner)
        prec, pkm = ranks[r].map_part_counts()
        parts = prec.shape[1]
        assert sum(counts) > 0 and [int(x) for x in prec.sum(axis=1)] == counts
        buf = torch.empty(max(sum(counts), 1) * ranks[r].record_bytes, dtype=torch.uint8, device="cuda")
        ranks[r].map_emit(buf.data_ptr(), max(sum(counts), 1))
        torch.cuda.synchronize()
        sends.append((buf, counts, prec, pkm))
    rb = ranks[0].record_bytes
    for dst in range(G):
        pieces, seg_rec, seg_km = [], [], []
        for src in range(G):
            buf, counts, prec, pkm = sends[src]
            off = sum(counts[:dst])
            pieces.append(buf[off * rb:(off + counts[dst]) * rb])
            seg_rec.append(prec[dst])
            seg_km.append(pkm[dst])
        recv = torch.cat(pieces)
        ranks[dst].reduce_grouped(recv.data_ptr(), recv.numel() // rb, np.stack(seg_rec), np.stack(seg_km))
        torch.cuda.synchronize()
    ref = oracle.OracleResult(fasta[:G * rec * 6000], k, m, B)
    total = np.zeros(ref.nbins, dtype=np.int64)
    for dst in range(G):
        got = ranks[dst].bin_sizes().astype(np.int64)
        assert all(got[b] == 0 for b in range(ref.nbins) if owner[b] != dst)
        total += got
    assert np.array_equal(total, ref.bin_sizes())
    for b in range(0, ref.nbins, 41):
        if ref.bin_size(b):
            hi, lo, cnt = counter_arrays(ranks[owner[b]], b)
            rhi, rlo, rcnt = ref.bin_arrays(b)
            assert np.array_equal(hi, rhi) and np.array_equal(lo, rlo) and np.array_equal(cnt, rcnt)


@pytest.mark.parametrize("k,m,staged,retry", [(28, 10, False, False), (32, 11, False, False), (21, 7, False, False),
                                               (28, 10, True, False), (55, 12, False, False), (40, 9, False, False),
                                               (63, 15, False, False), (55, 12, True, False), (28, 10, False, True),
                                               (28, 10, True, True), (55, 12, False, True)])
def test_heavy_bucket_split_vs_oracle(monkeypatch, k, m, staged, retry):
    # buckets above the wave tier (cells of a few thousand keys, FASTKMER_DEBUG_CELL_TARGET) split into
    # wave-sized sub-buckets by sampled splitters (~256 keys each), counted by the wave tier and
    # joined back in place -- from one key array and from staged pieces (a pinned ingest in 512 KB
    # pieces); k = 32 keys use all 64 bits; repeated reads leave sub-buckets too large for a wave, which
    # keep the block / big-table path (pieces need the fused map: k=28 m=10 or k=55 m=12); k > 32: the
    # 128-bit split (k_bucket_split128 / k_sub_count128_seq), fallbacks to the LDS sort / streaming path;
    # retry (FASTKMER_DEBUG_SPLIT_RETRY): every bucket cut a second time from another sample into twice
    # as many sub-buckets (the path of a bucket whose first cut left a sub-bucket above a wave's keys)
    monkeypatch.setenv("FASTKMER_DEBUG_CELL_TARGET", "2600")
    if retry:
        monkeypatch.setenv("FASTKMER_DEBUG_SPLIT_RETRY", "1")
    if staged:
        monkeypatch.setenv("FASTKMER_INGEST_SEG", str(256 << 10))
        monkeypatch.setenv("FASTKMER_PIECE_BYTES", str(512 << 10))
    rep = b"".join(b">q%d\n" % i + b"ACGTTGCAAGGCTTACCGATCGGATTACAGGCATCGATCGGGCTAGCTAGGCTAGCTTACGAGCTAGCATCGACTAG"
                   b"CATGCATGCATCGACGTAGCATCG\n" for i in range(3_000))
    fasta = fk.synth_fasta(60_000, 100, 3_000_000_000, seed=0xC1 + k) + rep
    if staged:
        import torch
        host = torch.frombuffer(bytearray(fasta), dtype=torch.uint8).pin_memory()
        kc = fk.KmerCounter(k, m, 3, 16)
        kc.ingest_ptr(host.data_ptr(), host.numel())
        kc.finish()
        assert kc.stats()["pieces_counted"] == 4
    else:
        kc = run_counter(fasta, k, m, 3, 16)
    st = kc.stats()
    assert st["split_buckets"] > 100 and st["sub_buckets"] > 3 * st["split_buckets"], st
    assert st["split_buckets"] < st["block_buckets"] + st["big_buckets"], st  # the repeats fall back
    ref = oracle.OracleResult(fasta, k, m, 16, threads=4)
    assert st["kmers"] == ref.total_kmers
    assert_same_as_oracle(kc, ref)


@pytest.mark.parametrize("k,m,bits,use_ht", [(55, 12, 6, False), (55, 12, 16, False), (55, 12, 16, True),
                                              (40, 9, 10, False)])
def test_wave_fingerprint_collisions_counted_exactly(k, m, bits, use_ht):
    # the 128-bit wave tier dedupes on 64-bit fingerprints and checks every key against its slot's
    # claimer; with the fingerprints cut to `bits` bits (fk_debug_fingerprint_bits) distinct keys share
    # them -- on every bucket at 6 bits, on many at 10 / 16 -- and those buckets take the exact count from
    # LDS; the result stays bit-exact (repeated reads: multi-copy keys included)
    rep = b"".join(b">q%d\n" % i + b"ACGTTGCAAGGCTTACCGATCGGATTACAGGCATCGATCGGGCTAGCTAGGCTAGCTTACGAGCTAGCATCGACTAG"
                   b"CATGCATGCATCGACGTAGCATCG\n" for i in range(500))
    fasta = fk.synth_fasta(20_000, 150, 2_000_000, seed=0xF9 + bits) + rep
    L = fk.lib()
    assert L.fk_debug_fingerprint_bits(0, bits) == 0
    try:
        kc = run_counter(fasta, k, m, 3, 64, use_ht)
        ref = oracle.OracleResult(fasta, k, m, 64, threads=4)
        assert kc.stats()["kmers"] == ref.total_kmers
        assert_same_as_oracle(kc, ref, ordered=not use_ht)
    finally:
        L.fk_debug_fingerprint_bits(0, 0)
