"""The multi-GPU job inside the library (fk_comm_*), through the C-ABI only.

Each rank is one context; the contexts exchange their records themselves
(grouped by owner rank = bin % n_ranks and local bin, one
all-to-all-v per step -- the reduceByKey shuffle of SparkBinKmerCounter.scala
:1034-1042 inside executeJob :989-1046), pieces of the input while later
pieces are still being ingested, then each rank counts the bins it owns.
No torch.distributed anywhere: the in-process transport (one host thread per
context, device-to-device copies) runs the whole native path with many ranks
on one GPU; the RCCL transport runs with one rank here (self send / receive)
and with two where two GPUs exist.  Every result is compared with the CPU
oracle on the whole input: the union of the ranks' bins must be bit-exact.
"""
import os
import threading

import numpy as np
import pytest

import fastkmer_amd as fk
import oracle
from test_gpu_parity import counter_arrays

pytestmark = pytest.mark.gpu

REC = 114


def record_shards(fasta: bytes, world: int, rec_bytes: int = REC):
    n = len(fasta) // rec_bytes
    cuts = [r * n // world * rec_bytes for r in range(world + 1)]
    return [fasta[cuts[r]:cuts[r + 1]] for r in range(world)]


def run_local_job(shards, k, m, x=3, B=2048, use_ht=False, seq=0, feed="bytes", chunks=1):
    """One context per shard joined in an in-process group; one thread per rank
    ingests its shard (feed = bytes: pageable; pinned: a pinned host buffer)
    and calls finish()."""
    G = len(shards)
    ctxs = [fk.KmerCounter(k, m, x, B, use_ht, seq, n_ranks=G, rank=r) for r in range(G)]
    fk.comm_init_local(ctxs)
    assert all(c.comm_transport == "local" for c in ctxs)
    errs = [None] * G
    keep = []
    if feed == "pinned":
        import torch
        for sh in shards:
            t = torch.empty(max(len(sh), 1), dtype=torch.uint8).pin_memory()
            if sh:
                t.numpy()[:len(sh)] = np.frombuffer(sh, dtype=np.uint8)
            keep.append(t)

    def work(r):
        try:
            sh = shards[r]
            if feed == "pinned":
                ctxs[r].ingest_ptr(keep[r].data_ptr(), len(sh))
            elif chunks > 1:
                cut = [len(sh) * i // chunks for i in range(chunks + 1)]
                for i in range(chunks):
                    ctxs[r].ingest_chunk(sh[cut[i]:cut[i + 1]], i == chunks - 1)
            else:
                ctxs[r].ingest(sh)
            ctxs[r].finish()
        except Exception as e:  # noqa: BLE001 -- reported below
            errs[r] = e

    th = [threading.Thread(target=work, args=(r,)) for r in range(G)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank did not finish"
    for e in errs:
        if e is not None:
            raise e
    return ctxs


def assert_union_matches_oracle(ctxs, ref, ordered=True, owner=None):
    """owner: the bin -> rank placement (default bin % G)"""
    G = len(ctxs)
    ref_sizes = ref.bin_sizes()
    total = np.zeros(ref.nbins, dtype=np.int64)
    owner = np.arange(ref.nbins) % G if owner is None else np.asarray(owner)
    for r, kc in enumerate(ctxs):
        sizes = kc.bin_sizes().astype(np.int64)
        own = owner == r
        assert np.all(sizes[~own] == 0), f"rank {r} holds bins it does not own"
        total += sizes
    bad = np.nonzero(total != ref_sizes)[0]
    assert len(bad) == 0, f"bin sizes differ in {len(bad)} bins, e.g. {bad[:5]}"
    for b in np.nonzero(ref_sizes)[0].tolist():
        hi, lo, cnt = counter_arrays(ctxs[int(owner[b])], b)
        rhi, rlo, rcnt = ref.bin_arrays(b)
        if not ordered:
            order = np.lexsort((lo, hi))
            hi, lo, cnt = hi[order], lo[order], cnt[order]
        assert np.array_equal(hi, rhi) and np.array_equal(lo, rlo), f"keys differ in bin {b}"
        assert np.array_equal(cnt, rcnt), f"counts differ in bin {b}"


@pytest.fixture
def small_pieces(monkeypatch):
    # 256 KB H2D segments and 512 KB pieces: a few MB of input crosses several pieces; the
    # received segments are expanded as staged pieces while later steps move, and counted once
    monkeypatch.setenv("FASTKMER_INGEST_SEG", str(256 << 10))
    monkeypatch.setenv("FASTKMER_PIECE_BYTES", str(512 << 10))


@pytest.mark.parametrize("world,use_ht,feed", [(2, False, "pinned"), (3, False, "bytes"), (8, False, "pinned"),
                                              (2, True, "pinned"), (5, True, "bytes")])
def test_local_exchange_vs_oracle(small_pieces, world, use_ht, feed):
    fasta = fk.synth_fasta(40_000, 100, 1_000_000, seed=0xE1 + world)
    ctxs = run_local_job(record_shards(fasta, world), 28, 10, 3, 2048, use_ht, feed=feed)
    ref = oracle.OracleResult(fasta, 28, 10, 2048)
    st = [c.stats() for c in ctxs]
    assert sum(s["kmers"] for s in st) == ref.total_kmers
    if feed == "pinned":  # pieces went out during the ingest, then the last piece (and closing steps)
        assert all(s["xch_steps"] >= (3 if world == 2 else 2) for s in st)
        if world == 2 and not use_ht:  # earlier steps were staged while later ones moved
            assert all(s["pieces_counted"] >= 2 for s in st)
    assert sum(s["xch_bytes_sent"] for s in st) == sum(s["xch_bytes_received"] for s in st) > 0
    assert_union_matches_oracle(ctxs, ref, ordered=not use_ht)


def test_local_exchange_streamed_chunks(small_pieces):
    # several fk_ingest calls per rank (last = 0 ... 1): pieces cut across call boundaries
    fasta = fk.synth_fasta(30_000, 100, 500_000, seed=0xE7)
    ctxs = run_local_job(record_shards(fasta, 3), 28, 10, 3, 2048, chunks=5)
    assert_union_matches_oracle(ctxs, oracle.OracleResult(fasta, 28, 10, 2048))


def test_local_exchange_uneven_and_empty_ranks(small_pieces):
    # ranks with very different inputs (and one with none) take different numbers of
    # steps; the finished ranks answer the others' steps until every rank is done
    fasta = fk.synth_fasta(36_000, 100, 800_000, seed=0xE2)
    n = len(fasta) // REC
    cuts = [0, n * 2 // 3, n * 2 // 3, n * 5 // 6, n]
    shards = [fasta[cuts[i] * REC:cuts[i + 1] * REC] for i in range(4)]
    assert shards[1] == b""
    ctxs = run_local_job(shards, 28, 10, 3, 2048, feed="pinned")
    steps = [c.stats()["xch_steps"] for c in ctxs]
    assert len(set(steps)) == 1  # every rank took part in every step
    assert_union_matches_oracle(ctxs, oracle.OracleResult(fasta, 28, 10, 2048))


def test_local_exchange_retracts_pieces_on_fallback(small_pieces):
    # a 40 KB header line late in rank 0's input (a tile starts more than the 4 KB read-back
    # inside it) makes the fused map hand the input back
    # after pieces were sent: rank 0 maps again from scratch, retracts its earlier
    # pieces and sends everything with its last piece
    fasta = fk.synth_fasta(30_000, 100, 600_000, seed=0xE3)
    shards = record_shards(fasta, 2)
    cut = len(shards[0]) * 7 // 8 // REC * REC
    long_header = b">" + b"h" * 40_000 + b"\n" + b"ACGT" * 30 + b"\n"
    shards[0] = shards[0][:cut] + long_header + shards[0][cut:]
    ctxs = run_local_job(shards, 28, 10, 3, 2048, feed="pinned")
    assert ctxs[0].stats()["fused_map"] == 0
    assert_union_matches_oracle(ctxs, oracle.OracleResult(shards[0] + shards[1], 28, 10, 2048))


def test_local_exchange_configs2_shape(small_pieces):
    # BASELINE configs[2] parameters: k=28 m=10 x=3 B=8192 over 8 ranks
    fasta = fk.synth_fasta(48_000, 100, 2_000_000, seed=0xC3)
    ctxs = run_local_job(record_shards(fasta, 8), 28, 10, 3, 8192, feed="pinned")
    assert all(c.num_bins == 8192 for c in ctxs)
    assert_union_matches_oracle(ctxs, oracle.OracleResult(fasta, 28, 10, 8192))


@pytest.mark.parametrize("use_ht", [False, True])
def test_local_exchange_two_word_k55(small_pieces, use_ht):
    # BASELINE configs[3] parameters: k=55 m=12 x=3 B=8192, 150 bp reads, 24-byte records
    fasta = fk.synth_fasta(12_000, 150, 1_000_000, seed=0xC4)
    ctxs = run_local_job(record_shards(fasta, 4, 164), 55, 12, 3, 8192, use_ht, feed="pinned")
    assert_union_matches_oracle(ctxs, oracle.OracleResult(fasta, 55, 12, 8192), ordered=not use_ht)


def test_local_exchange_long_sequence(small_pieces, tmp_path):
    # sequenceType = 1: one record cut into byte ranges with the k - 1 overlap (sharding.read_shard)
    from fastkmer_amd.sharding import read_shard
    rng = np.random.default_rng(9)
    seq = np.frombuffer(b"ACGTN", dtype=np.uint8)[rng.choice(5, 3_000_000, p=[.245, .245, .245, .245, .02])]
    lines = b"\n".join(seq[i:i + 60].tobytes() for i in range(0, len(seq), 60))
    fasta = b">chr1 synthetic\n" + lines + b"\n"
    path = tmp_path / "long.fa"
    path.write_bytes(fasta)
    shards = [read_shard(str(path), 3, r, 28).piece for r in range(3)]
    ctxs = run_local_job(shards, 28, 10, 3, 2048, seq=1, feed="pinned")
    assert_union_matches_oracle(ctxs, oracle.OracleResult(fasta, 28, 10, 2048, sequence_type=1))


def test_local_exchange_device_input_and_reuse(small_pieces):
    # the same contexts run two jobs: device-resident inputs (one step each), then host inputs
    import torch
    fasta = fk.synth_fasta(20_000, 100, 400_000, seed=0xE4)
    shards = record_shards(fasta, 2)
    ref = oracle.OracleResult(fasta, 28, 10, 2048)
    ctxs = [fk.KmerCounter(28, 10, 3, 2048, n_ranks=2, rank=r) for r in range(2)]
    fk.comm_init_local(ctxs)
    dev = [torch.frombuffer(bytearray(sh), dtype=torch.uint8).cuda() for sh in shards]
    torch.cuda.synchronize()
    for job in range(2):
        errs = [None, None]

        def work(r):
            try:
                if job == 0:
                    ctxs[r].ingest_device(dev[r].data_ptr(), dev[r].numel())
                else:
                    ctxs[r].ingest(shards[r])
                ctxs[r].finish()
            except Exception as e:  # noqa: BLE001
                errs[r] = e
        th = [threading.Thread(target=work, args=(r,)) for r in range(2)]
        [t.start() for t in th]
        [t.join(timeout=300) for t in th]
        assert errs == [None, None], errs
        assert_union_matches_oracle(ctxs, ref)


def test_rccl_single_rank_self_exchange(small_pieces):
    # the RCCL transport end to end with one rank (self send / receive): comm init from a
    # unique id, the pieced ingest, the count
    import torch
    fasta = fk.synth_fasta(30_000, 100, 600_000, seed=0xE5)
    host = torch.empty(len(fasta), dtype=torch.uint8).pin_memory()
    host.numpy()[:] = np.frombuffer(fasta, dtype=np.uint8)
    with fk.KmerCounter(28, 10, 3, 2048, n_ranks=1, rank=0) as kc:
        kc.comm_init(fk.comm_unique_id())
        assert kc.comm_transport == "rccl"
        for _ in range(2):
            kc.ingest_ptr(host.data_ptr(), len(fasta))
            kc.finish()
            st = kc.stats()
            assert st["xch_steps"] >= 3 and st["records_received"] == st["superkmers"]
            ref = oracle.OracleResult(fasta, 28, 10, 2048)
            assert_union_matches_oracle([kc], ref)


def test_rccl_single_rank_counts_on_the_records_communicator(small_pieces, monkeypatch):
    # FASTKMER_COMM_SPLIT=0: the per-step counts on the records' communicator and the comm stream
    # (no ncclCommSplit) -- the switch that rules the two-communicator ordering out on a first N-GPU run
    import torch
    monkeypatch.setenv("FASTKMER_COMM_SPLIT", "0")
    fasta = fk.synth_fasta(30_000, 100, 600_000, seed=0xE7)
    host = torch.empty(len(fasta), dtype=torch.uint8).pin_memory()
    host.numpy()[:] = np.frombuffer(fasta, dtype=np.uint8)
    with fk.KmerCounter(28, 10, 3, 2048, n_ranks=1, rank=0) as kc:
        kc.comm_init(fk.comm_unique_id())
        for _ in range(2):
            kc.ingest_ptr(host.data_ptr(), len(fasta))
            kc.finish()
            assert kc.stats()["xch_steps"] >= 3
            assert_union_matches_oracle([kc], oracle.OracleResult(fasta, 28, 10, 2048))
        assert (kc.comm_allreduce(np.arange(5)) == np.arange(5)).all()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("split", ["1", "0"])
def test_rccl_wait_times_out_and_aborts(monkeypatch, split):
    """A rank whose collective never completes (here: its streams held by a kernel spinning on a
    host-mapped flag, as behind a dead peer) returns FK_E_COMM after FASTKMER_COMM_TIMEOUT_S instead
    of blocking; the communicator is aborted and later collectives fail at once (the reference fails
    the Spark job when a task fails, SBKC:1031-1043)."""
    import time
    monkeypatch.setenv("FASTKMER_COMM_TIMEOUT_S", "3")
    monkeypatch.setenv("FASTKMER_COMM_SPLIT", split)
    L = fk.lib()
    kc = fk.KmerCounter(28, 10, 3, 2048, n_ranks=1, rank=0)
    try:
        kc.comm_init(fk.comm_unique_id())
        assert (kc.comm_allreduce(np.array([3, 4])) == [3, 4]).all()  # healthy first
        assert L.fk_debug_comm_hold(kc._h, 30) == 0
        time.sleep(0.5)
        assert L.fk_debug_comm_held(kc._h) == 1, "the hold kernel did not hold the comm stream"
        # released well after the timeout: the abort may wait for the held kernel to end
        timer = threading.Timer(6.0, lambda: L.fk_debug_comm_release(kc._h))
        timer.start()
        t0 = time.perf_counter()
        err = None
        try:
            kc.comm_allreduce(np.array([1, 2, 3]))
        except fk.FastKmerError as ex:
            err = ex
        dt = time.perf_counter() - t0
        timer.join()
        assert err is not None, f"the collective returned after {dt:.1f} s without an error"
        assert err.code == -7 and "timed out after 3 s" in str(err), err
        assert 3.0 <= dt < 25.0
        t0 = time.perf_counter()
        with pytest.raises(fk.FastKmerError) as e2:  # the communicator is gone: fail fast
            kc.comm_allreduce(np.array([1]))
        assert e2.value.code == -7 and "aborted" in str(e2.value)
        assert time.perf_counter() - t0 < 1.0
    finally:
        L.fk_debug_comm_release(kc._h)
        kc.close()


def _rccl_rank(rank, world, uid, path, out_dir, q):
    try:
        import torch  # noqa: F401  (one HIP runtime per process, see fastkmer_amd.lib)
        import fastkmer_amd as fk_
        from fastkmer_amd.sharding import read_shard
        piece = read_shard(path, world, rank, 28).piece
        with fk_.KmerCounter(28, 10, 3, 2048, n_ranks=world, rank=rank, device=rank) as kc:
            kc.comm_init(uid)
            kc.ingest(piece)
            kc.finish()
            kc.write_bins(out_dir)
            q.put((rank, kc.stats()["xch_bytes_sent"], None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, 0, repr(e)))


@pytest.mark.skipif(__import__("torch").cuda.device_count() < 2, reason="RCCL between ranks needs two GPUs")
def test_rccl_two_ranks_write_bins(tmp_path):
    import multiprocessing as mp
    fasta = fk.synth_fasta(30_000, 100, 600_000, seed=0xE6)
    path = tmp_path / "in.fa"
    path.write_bytes(fasta)
    out = tmp_path / "out"
    uid = fk.comm_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rccl_rank, args=(r, 2, uid, str(path), str(out), q)) for r in range(2)]
    [p.start() for p in ps]
    res = [q.get(timeout=300) for _ in range(2)]
    [p.join(timeout=60) for p in ps]
    assert all(e is None for _, _, e in res), res
    assert all(sent > 0 for _, sent, _ in res)
    ref_dir = tmp_path / "ref"
    oracle.OracleResult(fasta, 28, 10, 2048).write_bins(str(ref_dir))
    files = sorted(os.listdir(ref_dir))
    assert sorted(os.listdir(out)) == files
    for f in files:
        assert (out / f).read_bytes() == (ref_dir / f).read_bytes(), f


@pytest.mark.parametrize("how", ["bad_ingest", "destroyed"])
def test_local_exchange_failing_rank_fails_the_group(small_pieces, how):
    # an error on one rank of a collective entry point (fk_ingest / fk_finish with a
    # communicator) aborts the group -- its peers return an error instead of blocking in a step.
    # Rank 1 either fails its ingest (null source) or is destroyed without finishing.
    fasta = fk.synth_fasta(20_000, 100, 400_000, seed=0xE8)
    shards = record_shards(fasta, 2)
    ctxs = [fk.KmerCounter(28, 10, 3, 2048, n_ranks=2, rank=r) for r in range(2)]
    fk.comm_init_local(ctxs)
    errs = [None, None]

    def work(r):
        try:
            if r == 1:
                if how == "bad_ingest":
                    fk._check(fk.lib().fk_ingest(ctxs[1]._h, None, 100, 1))
                else:
                    ctxs[1].close()
                return
            ctxs[0].ingest(shards[0])
            ctxs[0].finish()
        except Exception as e:  # noqa: BLE001
            errs[r] = e
    th = [threading.Thread(target=work, args=(r,)) for r in range(2)]
    [t.start() for t in th]
    [t.join(timeout=120) for t in th]
    assert not any(t.is_alive() for t in th), "a rank blocked after its peer failed"
    assert errs[0] is not None and "fail" in str(errs[0]), errs
    if how == "bad_ingest":
        assert errs[1] is not None
    for c in ctxs:
        c.close()


def test_two_rank_context_without_comm_counts_no_pieces(monkeypatch):
    # a context of 2 ranks without a communicator (the caller-driven exchange:
    # fk_map / fk_map_emit) maps its input for the caller; it must not count pieces of it (its
    # input holds the other rank's records too)
    monkeypatch.setenv("FASTKMER_INGEST_SEG", str(256 << 10))
    monkeypatch.setenv("FASTKMER_PIECE_BYTES", str(512 << 10))
    fasta = fk.synth_fasta(40_000, 100, 1_000_000, seed=0xE9)
    with fk.KmerCounter(28, 10, 3, 2048, n_ranks=2, rank=0) as kc:
        kc.ingest(fasta)
        counts = kc.map()
        assert kc.stats()["pieces_counted"] == 0
        assert sum(counts) == kc.stats()["superkmers"]


@pytest.mark.parametrize("world,seq", [(1, 0), (3, 0), (4, 1), (2, 1)])
def test_local_exchange_ingest_file_range(small_pieces, tmp_path, world, seq):
    # the rank's split comes from the library (fk_ingest_file_range: FASTdoop-style
    # splits, positioned reads in pinned windows of 1 MB here) -- ranges start inside records and
    # header lines; the union of the ranks' bins is bit-exact vs the oracle on the whole file
    if seq == 0:
        fasta = b"text before the first header\n" + fk.synth_fasta(20_000, 100, 500_000, seed=0xEA + world)
    else:
        import bench
        fasta = bench.long_sequence_fasta(3_000_000, seed=0xEB + world)
    path = tmp_path / "in.fa"
    path.write_bytes(fasta)
    ctxs = [fk.KmerCounter(28, 10, 3, 2048, sequence_type=seq, n_ranks=world, rank=r) for r in range(world)]
    fk.comm_init_local(ctxs)
    errs = [None] * world

    def work(r):
        try:
            ctxs[r].ingest_file_range(str(path), window_bytes=1 << 20)
            ctxs[r].finish()
        except Exception as e:  # noqa: BLE001
            errs[r] = e
    th = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    [t.start() for t in th]
    [t.join(timeout=300) for t in th]
    assert errs == [None] * world, errs
    assert_union_matches_oracle(ctxs, oracle.OracleResult(fasta, 28, 10, 2048, sequence_type=seq))


@pytest.mark.parametrize("use_ht,k,m", [(False, 28, 10), (True, 28, 10), (False, 55, 12)])
def test_local_exchange_size_aware_placement(small_pieces, tmp_path, use_ht, k, m):
    # useCustomPartitioner (SBKC:1023-1026, MultiprocessorSchedulingPartitioner
    # .scala:35-69) on the library's exchange: 4 ranks sample their splits (fk_balance_bins_file),
    # the per-bin k-mer totals are all-reduced and LPT owners installed on every rank, then the job
    # runs through the native exchange.  Skewed input: a third of the reads come from a 30 kbp
    # region (its bins hold far more k-mers).  Bit-exact vs the oracle under the LPT owners.
    G = 4
    rl = 100 if k == 28 else 150
    fasta = fk.synth_fasta(16_000, rl, 2_000_000, seed=0xF2) + \
        fk.synth_fasta(8_000, rl, 30_000, seed=0xF3, first_read=16_000)
    path = tmp_path / "skewed.fa"
    path.write_bytes(fasta)
    ctxs = [fk.KmerCounter(k, m, 3, 2048, use_ht, n_ranks=G, rank=r) for r in range(G)]
    fk.comm_init_local(ctxs)
    owners, errs = [None] * G, [None] * G

    def work(r):
        try:
            owners[r] = ctxs[r].balance_bins_file(str(path), fraction=0.25)
            ctxs[r].ingest_file_range(str(path))
            ctxs[r].finish()
        except Exception as e:  # noqa: BLE001
            errs[r] = e
    th = [threading.Thread(target=work, args=(r,)) for r in range(G)]
    [t.start() for t in th]
    [t.join(timeout=300) for t in th]
    assert errs == [None] * G, errs
    assert all(np.array_equal(o, owners[0]) for o in owners), "ranks disagree on the placement"
    owner = owners[0]
    assert not np.array_equal(owner, np.arange(2048) % G), "LPT placement equals the default"
    ref = oracle.OracleResult(fasta, k, m, 2048)
    assert_union_matches_oracle(ctxs, ref, ordered=not use_ht, owner=owner)
    # the placement balances the ranks' k-mers better than bin % G on this input
    km = np.array([int(ref.bin_arrays(b)[2].sum(dtype=np.uint64)) for b in range(2048)], dtype=np.int64)
    lpt = max(km[owner == r].sum() for r in range(G))
    default = max(km[np.arange(2048) % G == r].sum() for r in range(G))
    assert lpt <= default * 1.02, (lpt, default)


def test_size_aware_placement_single_line_long_record(small_pieces, tmp_path):
    # a long record whose sequence is one unwrapped line (sequenceType=1) -- every 1 MB
    # sample block lies inside that line and is all sequence; the sample must not come back empty
    # (the placement would silently stay bin % n)
    G = 2
    rng = np.random.default_rng(0x5A)
    seq = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, 12_000_000)].tobytes()
    fasta = b">chrOneLine\n" + seq + b"\n"
    path = tmp_path / "one_line.fa"
    path.write_bytes(fasta)
    ctxs = [fk.KmerCounter(28, 10, 3, 2048, sequence_type=1, n_ranks=G, rank=r) for r in range(G)]
    fk.comm_init_local(ctxs)
    owners, errs = [None] * G, [None] * G

    def work(r):
        try:
            owners[r] = ctxs[r].balance_bins_file(str(path), fraction=0.25)
            ctxs[r].ingest_file_range(str(path))
            ctxs[r].finish()
        except Exception as e:  # noqa: BLE001
            errs[r] = e
    th = [threading.Thread(target=work, args=(r,)) for r in range(G)]
    [t.start() for t in th]
    [t.join(timeout=300) for t in th]
    assert errs == [None] * G, errs
    assert np.array_equal(owners[0], owners[1])
    assert not np.array_equal(owners[0], np.arange(2048) % G), "empty sample: the placement stayed bin % n"
    assert_union_matches_oracle(ctxs, oracle.OracleResult(fasta, 28, 10, 2048, sequence_type=1), owner=owners[0])


def test_local_exchange_rank_closed_right_after_finish(small_pieces):
    # a rank destroyed right after fk_finish while its peer may still be in the job's
    # last step (waiting on the closed rank's events, copying out of its send buffer) -- the peer's
    # result stays exact.  Rank 1 holds a fraction of rank 0's input, so rank 0 takes the
    # closing steps; repeated so both arrival orders at the last barrier occur.
    fasta = fk.synth_fasta(30_000, 100, 400_000, seed=0xEC)
    ref = oracle.OracleResult(fasta, 28, 10, 2048)
    cut = 114 * 26_000
    shards = [fasta[:cut], fasta[cut:]]
    for _ in range(4):
        ctxs = [fk.KmerCounter(28, 10, 3, 2048, n_ranks=2, rank=r) for r in range(2)]
        fk.comm_init_local(ctxs)
        errs = [None, None]

        def work(r):
            try:
                ctxs[r].ingest(shards[r])
                ctxs[r].finish()
                if r == 1:
                    ctxs[1].close()
            except Exception as e:  # noqa: BLE001
                errs[r] = e
        th = [threading.Thread(target=work, args=(r,)) for r in range(2)]
        [t.start() for t in th]
        [t.join(timeout=120) for t in th]
        assert not any(t.is_alive() for t in th)
        assert errs == [None, None], errs
        sizes = ctxs[0].bin_sizes()
        for b in range(0, 2048, 2):
            assert sizes[b] == ref.bin_size(b)
            if b % 64 == 0 and sizes[b]:
                _, lo, cnt = counter_arrays(ctxs[0], b)
                _, rlo, rcnt = ref.bin_arrays(b)
                assert np.array_equal(lo, rlo) and np.array_equal(cnt, rcnt)
        ctxs[0].close()


def test_split_of_another_rank_is_refused(tmp_path):
    # with a communicator the file split must be the context's own (world, rank)
    path = tmp_path / "in.fa"
    path.write_bytes(fk.synth_fasta(2_000, 100, 50_000, seed=0xED))
    ctxs = [fk.KmerCounter(28, 10, 3, 2048, n_ranks=2, rank=r) for r in range(2)]
    fk.comm_init_local(ctxs)
    with pytest.raises(fk.FastKmerError) as e:
        ctxs[0].ingest_file_range(str(path), world=2, rank=1)
    assert e.value.code == -1 and "split 1 of 2" in str(e.value)
    with pytest.raises(fk.FastKmerError) as e:
        ctxs[1].balance_bins_file(str(path), world=3, rank=1)
    assert e.value.code == -1
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("world", [1, 2])
def test_full_size_exchange_vs_one_count(world):
    # BASELINE configs[1] (1 GB) through the in-process group at the product's own sizes (no piece
    # knobs): each rank's one fk_ingest call sends steps of a tenth of its share (>= 64 MB) while
    # it ingests, the received segments are expanded on the staging stream as they land, the rest
    # after the last step; the union of the ranks' bins must equal the same job counted whole from HBM (no
    # communicator, no pieces) on all 2048 bins
    import torch
    n_reads = 1_000_000_000 // REC
    dev = torch.empty(n_reads * REC, dtype=torch.uint8, device="cuda")
    fk.synth_fasta_to_device(dev.data_ptr(), n_reads, 100, 100_000_000, seed=0x5EED + world)
    host = torch.empty(dev.numel(), dtype=torch.uint8).pin_memory()
    host.copy_(dev)
    torch.cuda.synchronize()
    ref = fk.KmerCounter(28, 10, 3, 2048)
    ref.ingest_device(dev.data_ptr(), dev.numel())
    ref.finish()
    del dev
    cuts = [r * n_reads // world * REC for r in range(world + 1)]
    ctxs = [fk.KmerCounter(28, 10, 3, 2048, n_ranks=world, rank=r) for r in range(world)]
    fk.comm_init_local(ctxs)
    errs = [None] * world

    def work(r):
        try:
            ctxs[r].ingest_ptr(host.data_ptr() + cuts[r], cuts[r + 1] - cuts[r])
            ctxs[r].finish()
        except Exception as e:  # noqa: BLE001 -- reported below
            errs[r] = e

    th = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank did not finish"
    for e in errs:
        if e is not None:
            raise e
    sts = [c.stats() for c in ctxs]
    # a tenth of the rank's share per step, at least 64 MB: 10 steps for one rank, 7 for two
    assert all(st["xch_steps"] >= (cuts[r + 1] - cuts[r]) // (128 << 20) + 2 for r, st in enumerate(sts)), \
        [st["xch_steps"] for st in sts]
    rst = ref.stats()
    assert sum(st["kmers"] for st in sts) == rst["kmers"]
    assert sum(st["distinct"] for st in sts) == rst["distinct"]
    rsizes = ref.bin_sizes()
    for r, c in enumerate(ctxs):
        sizes = c.bin_sizes()
        own = np.arange(2048) % world == r
        assert np.all(sizes[~own] == 0) and np.array_equal(sizes[own], rsizes[own]), f"rank {r}"
    for b in range(2048):
        ka, ca = ctxs[b % world].get_bin(b)
        kb, cb = ref.get_bin(b)
        assert np.array_equal(ka, kb) and np.array_equal(ca, cb), f"bin {b}"
    for c in ctxs:
        c.close()
    ref.close()
