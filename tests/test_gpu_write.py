"""write=1 parity at the BASELINE sizes (the bin<b> writers of
SBKC:550-606 (sorted, "EOF" trailer) and SBKC:715-734 (HT, no trailer)),
through the C-ABI (needs a GPU).

* configs[0] (10 MB of 100 bp reads, k=28 m=10 x=3 B=2048): every bin<b> file
  fk_write_bins writes is compared with the oracle's writer -- byte-identical
  for useHT=0; for useHT=1 the same files with the same lines (the line order
  is the reference's hash-table order, fastutil 7.2.0, unpinned; see DESIGN).
* configs[1] (1 GB), ingested from pinned host memory exactly as bench.py's
  timed step: every bin's keys and counts are compared with the oracle's
  (useHT=0 in order, useHT=1 as sets); fk_write_bins is timed (MB/s printed and checked against a
  floor), then a seeded sample of bins is byte-compared with the oracle's
  text for those bins, and sampled files' line counts are checked against
  the device bin sizes.
"""
import os
import random
import time

import numpy as np
import pytest

import fastkmer_amd as fk
import oracle

pytestmark = pytest.mark.gpu

K, M, X, B = 28, 10, 3, 2048


def _files(d):
    return {f: open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d))}


@pytest.mark.parametrize("use_ht", [False, True])
def test_write_bins_configs0_every_file(tmp_path, use_ht):
    fasta = fk.synth_fasta(10_000_000 // 114, 100, 1_000_000, seed=0x5EED)
    ref = oracle.OracleResult(fasta, K, M, B)
    with fk.KmerCounter(K, M, X, B, use_ht) as kc:
        kc.ingest(fasta)
        kc.finish()
        kc.write_bins(str(tmp_path / "gpu"))
    ref.write_bins(str(tmp_path / "ref"), sorted_eof=not use_ht)
    got, exp = _files(tmp_path / "gpu"), _files(tmp_path / "ref")
    assert sorted(got) == sorted(exp) and len(got) > 1000
    if not use_ht:
        bad = [f for f in exp if got[f] != exp[f]]
        assert not bad, f"{len(bad)} files differ, e.g. {bad[:3]}"
    else:
        for f in exp:
            assert not got[f].endswith(b"EOF")
            assert sorted(got[f].splitlines()) == sorted(exp[f].splitlines()), f


@pytest.fixture(scope="module")
def configs1():
    """configs[1]'s 1 GB job (bench.py's input, same seed) in pinned host memory, and the oracle's
    result over it."""
    import torch
    n_reads = 1_000_000_000 // 114
    fasta = fk.synth_fasta(n_reads, 100, 100_000_000, seed=0x5EED)
    ref = oracle.OracleResult(fasta, K, M, B, threads=min(16, os.cpu_count() or 1))
    pinned = torch.empty(len(fasta), dtype=torch.uint8, pin_memory=True)
    pinned.numpy()[:] = np.frombuffer(fasta, dtype=np.uint8)
    del fasta
    return pinned, ref


def _headline_job(kc, pinned):
    # exactly bench.py's timed step (Rank.step_host): the pinned source copied by DMA in segments,
    # every landed tile mapped, pieces staged while the rest lands, then fk_finish
    kc.ingest_ptr(pinned.data_ptr(), pinned.numel())
    kc.finish()


def test_write_bins_configs1_sampled_and_timed(tmp_path, configs1):
    """configs[1] at full size (the headline job, through bench.py's own ingest path): every bin's
    keys and counts vs the oracle's, then the files (timed; a sample byte-compared, every file's line
    count checked)."""
    pinned, ref = configs1
    with fk.KmerCounter(K, M, X, B) as kc:
        _headline_job(kc, pinned)
        assert kc.stats()["pieces_counted"] > 1  # the staged pieces of the bench's step
        sizes = kc.bin_sizes()
        assert np.array_equal(sizes.astype(np.int64), ref.bin_sizes())
        for b in range(B):  # every bin of the headline job, not a sample
            keys, cnt = kc.get_bin(b)
            _, rlo, rcnt = ref.bin_arrays(b)
            assert np.array_equal(keys, rlo) and np.array_equal(cnt, rcnt), f"bin {b} differs from the oracle"
        out = tmp_path / "out"
        t0 = time.perf_counter()
        kc.write_bins(str(out))
        dt = time.perf_counter() - t0
    nbytes = sum(os.path.getsize(out / f) for f in os.listdir(out))
    mbs = nbytes / dt / 1e6
    print(f"\nfk_write_bins configs[1]: {nbytes / 1e6:.0f} MB in {len(os.listdir(out))} files, "
          f"{dt:.2f} s = {mbs:.0f} MB/s")
    assert mbs > 200  # device formatting + D2H + file writes; ~3.8 GB of text
    files = sorted(os.listdir(out))
    assert files == sorted(f"bin{b}" for b in np.nonzero(sizes)[0].tolist())
    rng = random.Random(7)
    for b in rng.sample(np.nonzero(sizes)[0].tolist(), 24):
        assert (out / f"bin{b}").read_text() == ref.bin_text(b), b
    for f in rng.sample(files, 64):  # one line per distinct k-mer, then "EOF"
        text = (out / f).read_bytes()
        assert text.endswith(b"EOF") and text.count(b"\n") == int(sizes[int(f[3:])])


def test_configs1_use_ht_every_bin_as_a_set(configs1):
    """useHT=1 (extractKXmersHT, SBKC:664-739) on the whole 1 GB headline job through the pinned
    ingest: every bin's (k-mer, count) pairs equal the oracle's as a set (the table order is
    fastutil's, unpinned)."""
    pinned, ref = configs1
    with fk.KmerCounter(K, M, X, B, use_ht=True) as kc:
        _headline_job(kc, pinned)
        sizes = kc.bin_sizes()
        assert np.array_equal(sizes.astype(np.int64), ref.bin_sizes())
        for b in range(B):
            keys, cnt = kc.get_bin(b)
            o = np.argsort(keys, kind="stable")
            _, rlo, rcnt = ref.bin_arrays(b)
            assert np.array_equal(keys[o], rlo) and np.array_equal(cnt[o], rcnt), f"bin {b} differs"
