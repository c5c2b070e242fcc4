"""Input sharding across ranks (host logic; replaces Spark/FASTdoop input splits).

The reference reads its dataset through FASTdoop input formats
(SBKC:996-1003): FASTAshortInputFileFormat hands every record to the split
holding its '>' and FASTAlongInputFileFormat cuts one long sequence into
splits that overlap by k-1 bases, so that every k-mer window is seen by
exactly one split.  ``shard_fasta`` gives each rank the same kind of piece
of an in-memory FASTA image:

* sequence_type 0 (short reads): byte ranges of ~n/world, each boundary
  moved forward to the next line-initial '>'; whole records only.
* sequence_type 1 (one long sequence): the sequence positions (bytes of the
  record body other than '\\n') split into ~equal ranges, each extended by
  k-1 positions into the next range and prefixed with the record's header
  line.  Files with more than one record fall back to record sharding (each
  record is then a unit of work, as the reference would count it).

Concatenating the per-rank counts of the shards gives the counts of the
whole input, which tests/test_distributed.py checks against the oracle.
"""
from __future__ import annotations

import numpy as np

_CHUNK = 1 << 20


def _record_starts(data: bytes, lo: int) -> int:
    """First index >= lo holding a line-initial '>' (len(data) if none)."""
    p = lo
    n = len(data)
    while p < n:
        q = data.find(b">", p)
        if q < 0:
            return n
        if q == 0 or data[q - 1] == 0x0A:
            return q
        p = q + 1
    return n


def record_shard_bounds(data: bytes, world: int) -> list[int]:
    """world+1 byte offsets; shard r = data[b[r]:b[r+1]] holds whole records."""
    n = len(data)
    bounds = [0]
    for r in range(1, world):
        bounds.append(max(bounds[-1], _record_starts(data, r * n // world)))
    bounds.append(n)
    return bounds


class _PositionIndex:
    """Maps sequence-position ordinals (non-'\\n' bytes) of a body to byte offsets."""

    def __init__(self, body: bytes):
        self.body = body
        a = np.frombuffer(body, dtype=np.uint8)
        starts = np.arange(0, len(a), _CHUNK, dtype=np.int64)
        per = np.add.reduceat((a != 0x0A).astype(np.int64), starts) if len(a) else np.zeros(0, np.int64)
        self.cum = np.concatenate([[0], np.cumsum(per)])  # positions before chunk i
        self.positions = int(self.cum[-1])

    def byte_of(self, t: int) -> int:
        """Byte offset of position t (len(body) for t == positions)."""
        if t >= self.positions:
            return len(self.body)
        c = int(np.searchsorted(self.cum, t, side="right")) - 1
        a = np.frombuffer(self.body, dtype=np.uint8, count=min(_CHUNK, len(self.body) - c * _CHUNK),
                          offset=c * _CHUNK)
        idx = np.flatnonzero(a != 0x0A)
        return c * _CHUNK + int(idx[t - int(self.cum[c])])


def shard_fasta(data: bytes, world: int, rank: int, sequence_type: int = 0, k: int = 1) -> bytes:
    """The piece of ``data`` rank ``rank`` of ``world`` counts."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    if world == 1:
        return bytes(data)
    if sequence_type == 1:
        p0 = _record_starts(data, 0)  # bytes before the first header are not sequence
        hdr_end = data.find(b"\n", p0) + 1
        if p0 == len(data) or hdr_end == 0:
            return b""
        body = data[hdr_end:]
        if _record_starts(body, 0) == len(body):  # a single record: split its positions
            idx = _PositionIndex(body)
            P = idx.positions
            s, e = rank * P // world, (rank + 1) * P // world
            if s >= e:
                return b""
            e_ext = min(P, e + k - 1)
            b0, b1 = idx.byte_of(s), idx.byte_of(e_ext - 1) + 1
            return data[p0:hdr_end] + body[b0:b1] + b"\n"
    b = record_shard_bounds(data, world)
    return bytes(data[b[rank]:b[rank + 1]])
