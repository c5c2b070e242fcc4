"""A rank's input split of a FASTA file in the C-ABI (fk_split_bytes; the file
reads of fk_ingest_file_range), host only (no GPU).

The reference hands its map tasks FASTdoop input splits (SparkBinKmerCounter
.scala:993, 1009-1012): whole records for the short-read format (sequenceType
0), and for the long-sequence format byte ranges overlapped by k - 1 positions
(sequenceType 1).  The library's split must give the same bytes as the Python
restatement (fastkmer_amd/sharding.py: read_record_shard / read_shard) and the
union of the ranks' counts must equal the whole file's (the CPU oracle), for
world 1..8, with ranges starting inside a record and inside a header line, text
before the first header, long headers, CRLF and blank lines.
"""
import random

import pytest

import fastkmer_amd as fk
import oracle
from fastkmer_amd.sharding import read_record_shard, read_shard


def _all_counts(data: bytes, k: int, m: int, seq: int) -> dict:
    res = oracle.OracleResult(data, k, m, 64, sequence_type=seq)
    out = {}
    for b in range(res.nbins):
        hi, lo, cnt = res.bin_arrays(b)
        for h, l, c in zip(hi.tolist(), lo.tolist(), cnt.tolist()):
            out[(h, l)] = out.get((h, l), 0) + c
    return out


def _fasta(seed: int, kind: str) -> bytes:
    rng = random.Random(seed)
    parts = []
    if kind == "junk":
        parts.append(b"some text before the first header\nACGTACGT\n")
    n_rec = 1 if kind == "long" else 60
    for i in range(n_rec):
        hdr = b">r%d" % i + (b" " + b"h" * rng.randint(0, 3000) if rng.random() < 0.3 else b"")
        n = rng.randint(20_000, 40_000) if kind == "long" else rng.randint(0, 400)
        seq = bytes(rng.choice(b"ACGTACGTACGTNa") for _ in range(n))
        width = rng.choice([60, 61, 1000, 10 ** 6])
        nl = b"\r\n" if kind == "crlf" else b"\n"
        lines = [seq[q:q + width] for q in range(0, len(seq), width)]
        if kind == "blank" and lines:
            lines.insert(rng.randrange(len(lines)), b"")
        parts.append(hdr + nl + nl.join(lines) + (nl if lines else b""))
    return b"".join(parts)


@pytest.mark.parametrize("kind", ["plain", "junk", "crlf", "blank", "long"])
@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
def test_split_matches_sharding_and_counts_add_up(tmp_path, kind, world):
    data = _fasta(world * 7 + len(kind), kind)
    path = tmp_path / "in.fa"
    path.write_bytes(data)
    for seq, k, m in ((0, 21, 7), (1, 21, 7), (1, 55, 11)):
        pieces = [fk.split_bytes(str(path), world, r, k, seq) for r in range(world)]
        if seq == 0:
            assert pieces == [read_record_shard(str(path), world, r) for r in range(world)]
            assert b"".join(pieces) == data  # whole records, in order
        else:
            assert pieces == [read_shard(str(path), world, r, k).piece for r in range(world)]
        if seq == 0 or k == 21:
            whole = _all_counts(data, k, m, seq)
            union = {}
            for p in pieces:
                for key, c in _all_counts(p, k, m, seq).items():
                    union[key] = union.get(key, 0) + c
            assert union == whole, f"seq={seq} k={k}: union of the ranks' counts != the file's"


def test_split_ranges_inside_records_and_headers(tmp_path):
    # cuts placed by hand: inside a header line, right after one, inside a sequence line, on a '\n'
    data = b">first header line\nACGTACGTAC\nGTACGTACGT\n>second\nTTTTGGGGCCCCAAAA\n"
    path = tmp_path / "in.fa"
    path.write_bytes(data)
    n = len(data)
    for world in range(1, n + 1):
        for seq, k in ((0, 5), (1, 5), (1, 1)):
            pieces = [fk.split_bytes(str(path), world, r, k, seq) for r in range(world)]
            ref = [read_record_shard(str(path), world, r) if seq == 0 else read_shard(str(path), world, r, k).piece
                   for r in range(world)]
            assert pieces == ref, (world, seq, k)


def test_split_degenerate_and_errors(tmp_path):
    empty = tmp_path / "e.fa"
    empty.write_bytes(b"")
    assert fk.split_bytes(str(empty), 3, 1, 5, 0) == b""
    assert fk.split_bytes(str(empty), 3, 1, 5, 1) == b""
    nohdr = tmp_path / "n.fa"
    nohdr.write_bytes(b"ACGT\nACGT\n")
    assert fk.split_bytes(str(nohdr), 2, 0, 3, 1) == b""
    with pytest.raises(fk.FastKmerError):
        fk.split_bytes(str(nohdr), 2, 2, 3, 0)
    with pytest.raises(fk.FastKmerError):
        fk.split_bytes(str(tmp_path / "missing.fa"), 1, 0, 3, 0)
