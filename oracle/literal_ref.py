"""Literal transliteration of the reference's hot path, for small inputs.

TEST INFRASTRUCTURE ONLY -- never imported by the product package.

This is a deliberately slow, step-for-step restatement of maruscia/fastkmer's
Scala code with Java ``long``/``int`` semantics emulated, used to pin the C
oracle (``oracle/fk_oracle.c``) and the golden fixtures to what the reference
actually computes -- including the parts the C oracle replaces by an exact
count (the 31-nucleotides-per-long ``Kmer`` layout, ``readFromKmer``, the
(k,x)-mer run packing and the ``RIndex`` heap merge of ``extractKXmers``).

Followed (paths relative to /root/reference/src/main/scala/skc/):
  package.scala:17-44    nucleotide tables, upper2bitMask
  package.scala:46-100   is_allowed, fillNorm
  package.scala:103-124  reverse_complement, fillRightOnesMask
  package.scala:138-503  class Kmer (_readKmer, readFromKmer, lastM, firstM,
                         getSignature, getSliceOffset, getNumSymbol, compare,
                         toByteArray)
  package.scala:511-560  class Mmer
  package.scala:562-614  RIndex, PointedMinOrder
  package.scala:642-681  priorityQueueWithIndexes
  package.scala:686-695  hash_to_bucket
  package.scala:721-754  getOrientation(Kmer), firstAndLastOccurrenceOfInvalidNucleotide
  SparkBinKmerCounter.scala:34-169   getSuperKmers
  SparkBinKmerCounter.scala:428-660  extractKXmers
  SparkBinKmerCounter.scala:664-739  extractKXmersHT
  SparkBinKmerCounter.scala:772-953  getBinSignatures, saveBinSignatures
  package.scala:616-634  longToString
"""
from __future__ import annotations

import heapq
import math

NPL = 31  # nucleotidesPerLong, package.scala:17
_BITMASK = {ord("A"): 0, ord("C"): 1, ord("G"): 2, ord("T"): 3}
_RC = [3, 2, 1, 0]  # nucleotideRC, package.scala:37-41
_REPR = b"ACGT"
UPPER2 = (1 << (2 * NPL)) - 1  # upper2bitMask, package.scala:44


def _jl(x: int) -> int:
    """Wrap to a Java signed 64-bit long."""
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >> 63 else x


def _ji(x: int) -> int:
    """Wrap to a Java signed 32-bit int."""
    x &= (1 << 32) - 1
    return x - (1 << 32) if x >> 31 else x


def _shl(x: int, n: int) -> int:
    return _jl(x << (n & 63))


def _shr(x: int, n: int) -> int:  # Java >> on long (arithmetic)
    return _jl(x) >> (n & 63)


def _bitmask(c: int) -> int:
    # nucleotideBitmasks is an Array[Long](85) with only A,C,G,T set.
    return _BITMASK.get(c, 0)


def is_allowed(mmer: int, length: int) -> bool:  # package.scala:46-75
    for _ in range(length - 3):
        if (mmer & 0xF) == 0:
            return False
        mmer >>= 2
    if mmer == 0:
        return False
    if mmer == 0x04:
        return False
    if (mmer & 0x3C) == 0:
        return False
    if (mmer & 0xF) == 0:
        return False
    return True


def reverse_complement(seq: int, length: int) -> int:  # package.scala:103-115
    cur, rev, shift = seq, 0, length * 2 - 2
    for _ in range(length):
        rev += (3 - (cur & 3)) << shift
        cur >>= 2
        shift -= 2
    return rev


def fill_norm(sig_len: int) -> list[int]:  # package.scala:77-100
    default = 1 << sig_len * 2
    norm = [0] * default
    for i in range(default):
        rev = reverse_complement(i, sig_len)
        sv = i if is_allowed(i, sig_len) else default
        rv = rev if is_allowed(rev, sig_len) else default
        norm[i] = min(sv, rv)
    return norm


def fill_right_ones_mask(runlength: int) -> int:  # package.scala:118-124
    res = 0
    for i in range(runlength):
        res |= _shl(1, i)
    return _jl(res)


def hash_to_bucket(s: int, b: int) -> int:  # package.scala:686-695
    key = _ji(s)
    c2 = 0x27D4EB2D
    key = _ji((key ^ 61) ^ ((key & 0xFFFFFFFF) >> 16))
    key = _ji(key + _ji(key << 3))
    key = _ji(key ^ ((key & 0xFFFFFFFF) >> 4))
    key = _ji(key * c2)
    key = _ji(key ^ ((key & 0xFFFFFFFF) >> 15))
    return (key & 0x7FFFFFFF) % b


class Kmer:  # package.scala:138-503
    __slots__ = ("length", "_data")

    def __init__(self, length: int):
        self.length = length
        self._data: list[int] = []

    @classmethod
    def from_bytes(cls, length: int, s: bytes, offset: int) -> "Kmer":  # :303-307
        k = cls(length)
        k._data = k._read_kmer(length, s, offset)
        return k

    @classmethod
    def from_kmer(cls, length: int, frm: "Kmer", start: int, end: int, orientation: int) -> "Kmer":  # :299-302
        k = cls(length)
        k._data = k.read_from_kmer(frm, start, end, length, orientation)
        return k

    def _read_kmer(self, length, s, offset):  # :144-172
        data = [0] * int(math.ceil(length / NPL))
        cur, slc, i = 0, 0, 0
        while i < length:
            cur = _shl(cur, 2)
            cur |= _bitmask(s[offset + i])
            i += 1
            if i % NPL == 0 or i == length:
                cur &= UPPER2
                data[slc] = cur
                cur = 0
                slc += 1
        return data

    def read_from_kmer(self, frm, start_pos, end_pos, amt, orientation):  # :174-295
        length = self.length
        data = [0] * int(math.ceil(amt / NPL))
        from_end_slice, from_end_offset = frm.get_slice_offset(end_pos)
        assert (from_end_slice, from_end_offset) != (-1, -1), "endPos is invalid"
        from_start_slice, from_start_offset = frm.get_slice_offset(start_pos)
        assert (from_start_slice, from_start_offset) != (-1, -1), "startPos is invalid"
        excess = frm.length % NPL
        to_excess = amt % NPL
        orig_final_padding = (NPL - excess) * 2 if excess > 0 else 0
        if orientation == 0:
            slc = 0
            if from_start_offset == 0:
                while from_end_slice - from_start_slice >= 0:
                    data[slc] = frm._data[from_start_slice]
                    from_start_slice += 1
                    slc += 1
                data[-1] = _shr(data[-1], 2 * (NPL - 1) - from_end_offset)
            elif from_start_slice == from_end_slice:
                data[0] = _shr(frm._data[from_start_slice], NPL * 2 - from_end_offset - 2) & fill_right_ones_mask(length * 2)
            else:
                cur_offset = from_start_offset
                while slc < len(data) - 1:
                    data[slc] = _shl(frm._data[from_start_slice], cur_offset) & UPPER2
                    from_start_slice += 1
                    cur = frm._data[from_start_slice]
                    if from_start_slice == len(frm._data) - 1:
                        cur = _shr(cur, NPL * 2 - cur_offset - orig_final_padding)
                    else:
                        cur = _shr(cur, NPL * 2 - cur_offset)
                    data[slc] |= cur
                    slc += 1
                if from_start_slice != from_end_slice:
                    sh = from_end_offset + 2 - (orig_final_padding if from_end_slice == len(frm._data) - 1 else 0)
                    data[slc] = _shl(frm._data[from_start_slice] & fill_right_ones_mask(NPL * 2 - cur_offset), sh)
                data[slc] |= _shr(frm._data[from_end_slice], (NPL - 1) * 2 - from_end_offset)
                if to_excess != 0:
                    data[slc] &= fill_right_ones_mask(to_excess * 2)
        else:
            slc = 0
            cur = _shr(frm._data[from_end_slice], (NPL - 1) * 2 - from_end_offset)
            written = 0
            written_this_slice = 0
            if from_end_slice != len(frm._data) - 1:
                last_slice_quantity = from_end_offset // 2 + 1
            else:
                last_slice_quantity = from_end_offset // 2 - orig_final_padding // 2 + 1
            while written < length:
                data[slc] = _shl(data[slc], 2)
                data[slc] = _jl(data[slc] + _RC[cur & 3])
                written += 1
                written_this_slice += 1
                cur = _shr(cur, 2)
                if written == last_slice_quantity or written_this_slice == NPL:
                    from_end_slice -= 1
                    if from_end_slice >= 0:
                        cur = frm._data[from_end_slice]
                    written_this_slice = 0
                if written % NPL == 0:
                    slc += 1
        return data

    def last_m(self, m_mask: int, norm: list[int], m: int) -> int:  # :310-326
        if len(self._data) == 1 or self.length % NPL >= m:
            return norm[self._data[-1] & m_mask]
        res = 0
        for i in range(self.length - m, self.length):
            res = _ji(res << 2)
            res |= self.get_num_symbol(i)
        return norm[res]

    def first_m(self, m: int) -> int:  # :329-334
        if len(self._data) > 1 or self.length == NPL:
            return _shr(self._data[0], (NPL - m) * 2)
        return _shr(self._data[0], ((self.length % NPL) - m) * 2)

    def get_signature(self, sig_len: int, norm: list[int]):  # :337-357
        mmer = Mmer(sig_len, 0, norm)
        pos = 0
        for i in range(sig_len):
            mmer.insert(self.get_num_symbol(i))
        sig = mmer.get()
        for i in range(sig_len, self.length):
            mmer.insert(self.get_num_symbol(i))
            if mmer.get() < sig:
                sig = mmer.get()
                pos = i - sig_len + 1
        return sig, pos

    def get_slice_offset(self, pos: int):  # :360-373
        if pos >= self.length:
            return -1, -1
        slc = pos // NPL
        if slc == len(self._data) - 1:
            offset = (NPL - (self.length - pos)) * 2
        else:
            offset = (pos % NPL) * 2
        return slc, offset

    def get_num_symbol(self, pos: int) -> int:  # :376-386
        slc, offset = self.get_slice_offset(pos)
        if slc == -1:
            return -1
        mask = _shr(UPPER2, offset)
        symbol = self._data[slc] & mask
        symbol = _shr(symbol, NPL * 2 - offset - 2)
        return symbol

    def compare(self, that: "Kmer") -> int:  # :389-404
        assert self.length == that.length
        for a, b in zip(self._data, that._data):
            if a != b:
                return -1 if a < b else 1
        return 0

    def __eq__(self, other):  # :406-410
        return isinstance(other, Kmer) and self.compare(other) == 0

    def __hash__(self):  # only used as a dict key in the HT path (:413)
        return hash(tuple(self._data))

    def __lt__(self, other):
        return self.compare(other) < 0

    def to_string(self) -> str:  # :416-454, 496-500
        result = bytearray(self.length)
        slc = len(self._data) - 1
        excess = self.length % NPL
        i, j = 0, self.length - 1
        amt = excess if excess > 0 else NPL
        cur = self._data[slc]
        while j >= 0:
            result[j] = _REPR[cur & 3]
            cur = _shr(cur, 2)
            j -= 1
            i += 1
            if i == amt:
                slc -= 1
                i = 0
                amt = NPL
                if slc >= 0:
                    cur = self._data[slc]
        return result.decode()


class Mmer:  # package.scala:511-560
    def __init__(self, length: int, seq: int, norm: list[int]):
        self.mask = _ji((1 << length * 2) - 1)
        self._data = seq
        self.norm = norm
        self.current = norm[seq]

    def get(self) -> int:
        return self.current

    def insert(self, symb: int) -> None:
        self._data = _ji(self._data << 2)
        self._data += symb
        self._data &= self.mask
        self.current = self.norm[self._data]


def first_and_last_invalid(s: bytes, start: int, end: int):  # package.scala:739-754
    first = last = -1
    for i in range(start, end):
        if s[i] not in (65, 67, 71, 84):  # notANucleotide, package.scala:697
            if first == -1:
                first = last = i - start
            else:
                last = i - start
    return first, last


def get_orientation(s: Kmer, i: int, j: int) -> int:  # package.scala:721-728
    while True:
        start, end = s.get_num_symbol(i), s.get_num_symbol(j)
        if start < _RC[end]:
            return 0
        if start > _RC[end] or i >= j:
            return 1
        i, j = i + 1, j - 1


def get_super_kmers(k: int, m: int, b: int, reads: list[bytes], trace: list | None = None):
    """SparkBinKmerCounter.scala:34-169. Returns {bin: [Kmer]}."""
    out: dict[int, list[Kmer]] = {}
    norm = fill_norm(m)
    last_m_mask = _ji((1 << m * 2) - 1)

    def emit(sig_value, kmer):
        bn = hash_to_bucket(sig_value, b)
        out.setdefault(bn, []).append(kmer)
        if trace is not None:
            trace.append(bn)

    for cur in reads:
        if len(cur) >= k:
            min_value, min_pos = -1, -1
            sk_start, i = 0, 0
            while i < len(cur) - k + 1:
                nf, nl = first_and_last_invalid(cur, i, i + k)
                if nf != -1:
                    if sk_start < i:
                        emit(min_value, Kmer.from_bytes(i - 1 + k - sk_start, cur, sk_start))
                    sk_start = i + nl + 1
                    i += nl + 1
                else:
                    s = Kmer.from_bytes(k, cur, i)
                    if i > min_pos:
                        if sk_start < i:
                            emit(min_value, Kmer.from_bytes(i - 1 + k - sk_start, cur, sk_start))
                            sk_start = i
                        sv, sp = s.get_signature(m, norm)
                        min_value, min_pos = sv, sp + i
                    else:
                        last = s.last_m(last_m_mask, norm, m)
                        if last < min_value:
                            if sk_start < i:
                                emit(min_value, Kmer.from_bytes(i - 1 + k - sk_start, cur, sk_start))
                                sk_start = i
                            min_value, min_pos = last, i + k - m
                    i += 1
            if len(cur) - sk_start >= k:
                nf, nl = first_and_last_invalid(cur, i, len(cur))
                if nf == -1:
                    emit(min_value, Kmer.from_bytes(len(cur) - sk_start, cur, sk_start))
                elif i + nf >= sk_start + k:
                    emit(min_value, Kmer.from_bytes(i + nf, cur, sk_start))
    return out


def long_to_string(num: int, length: int = 7) -> str:  # package.scala:616-634 (length unused)
    result = [""] * NPL
    cur = _jl(num)
    for j in range(NPL - 1, -1, -1):
        result[j] = "ACGT"[cur & 3]
        cur = _shr(cur, 2)
    return "".join(result)


def get_bin_signatures(k: int, m: int, b: int, reads: list[bytes]) -> dict[int, dict[str, int]]:
    """SparkBinKmerCounter.scala:772-917 (the HashMaps of bins with a signature)."""
    out: dict[int, dict[str, int]] = {}
    norm = fill_norm(m)
    last_m_mask = _ji((1 << m * 2) - 1)

    def update(sig_value):  # :828-830 (and the three copies below)
        d = out.setdefault(hash_to_bucket(sig_value, b), {})
        sig = long_to_string(sig_value, m)
        d[sig] = d.get(sig, 0) + 1

    for cur in reads:
        if len(cur) >= k:
            min_value, min_pos = -1, -1
            sk_start, i = 0, 0
            while i < len(cur) - k + 1:
                nf, nl = first_and_last_invalid(cur, i, i + k)
                if nf != -1:
                    if sk_start < i:
                        update(min_value)
                    sk_start = i + nl + 1
                    i += nl + 1
                else:
                    s = Kmer.from_bytes(k, cur, i)
                    if i > min_pos:
                        if sk_start < i:
                            update(min_value)
                            sk_start = i
                        sv, sp = s.get_signature(m, norm)
                        min_value, min_pos = sv, sp + i
                    else:
                        last = s.last_m(last_m_mask, norm, m)
                        if last < min_value:
                            if sk_start < i:
                                update(min_value)
                                sk_start = i
                            min_value, min_pos = last, i + k - m
                    i += 1
            if len(cur) - sk_start >= k:
                nf, nl = first_and_last_invalid(cur, i, len(cur))
                if nf == -1 or i + nf >= sk_start + k:
                    update(min_value)
    return out


def save_bin_signatures_text(sigs: dict[str, int]) -> str:  # SparkBinKmerCounter.scala:920-953
    """One bin's file; lines in the dict's order (the reference's HashMap order)."""
    return "".join(f"{s}\t{c}\n" for s, c in sigs.items()) + f"Total\t{sum(sigs.values())}\n"


class RIndex:  # package.scala:562-601
    def __init__(self, arr, start_pos, end_pos, shift, kmer_length):
        self.arr, self.cur, self.end = arr, start_pos, end_pos
        self.shift, self.k = shift, kmer_length
        self._read()

    def _read(self):
        nxt = self.arr[self.cur]
        self.pointed = Kmer.from_kmer(self.k, nxt, self.shift, self.shift + self.k - 1, 0)

    def advance(self):
        self.cur += 1
        if not self.exhausted():
            self._read()

    def exhausted(self):
        return self.cur >= self.end


def priority_queue_with_indexes(arr, k):  # package.scala:642-681
    heap = []
    for r_index, a in enumerate(arr):
        if a:
            starts = [0] * r_index
            heap.append(RIndex(a, 0, len(a), 0, k))
            if len(a) > 1:
                for j in range(1, len(a)):
                    for i in range(r_index):
                        if a[j - 1].first_m(i + 1) != a[j].first_m(i + 1):
                            heap.append(RIndex(a, starts[i], j, i + 1, k))
                            starts[i] = j
            for i in range(len(starts)):
                heap.append(RIndex(a, starts[i], len(a), i + 1, k))
    return heap


def extract_kx_mers(k: int, x: int, bins: dict[int, list[Kmer]]) -> dict[int, str]:
    """SparkBinKmerCounter.scala:428-660; returns {bin: file text}."""
    files = {}
    for bin_id in sorted(bins):
        unsorted_r = [[] for _ in range(x + 1)]
        for sk in bins[bin_id]:
            last_orientation, run_length, run_start = -1, 0, 0
            for i in range(0, sk.length - k + 1):
                orientation = get_orientation(sk, i, i + k - 1)
                if orientation == last_orientation:
                    run_length += 1
                    if run_length == x + 1:
                        unsorted_r[run_length - 1].append(
                            Kmer.from_kmer(k + run_length - 1, sk, run_start, run_start + k + run_length - 2, orientation))
                        run_length, run_start, last_orientation = 0, i, -1
                else:
                    if last_orientation != -1:
                        unsorted_r[run_length - 1].append(
                            Kmer.from_kmer(k + run_length - 1, sk, run_start, run_start + k + run_length - 2, last_orientation))
                    run_length, run_start, last_orientation = 1, i, orientation
            if run_length > 0:
                unsorted_r[run_length - 1].append(
                    Kmer.from_kmer(k + run_length - 1, sk, run_start, run_start + k + run_length - 2, last_orientation))
        sorted_r = [sorted(r, key=lambda km: tuple(km._data)) for r in unsorted_r]
        heap_list = priority_queue_with_indexes(sorted_r, k)
        if not heap_list:
            continue
        # PriorityQueue with PointedMinOrder: min-heap on the pointed k-mer.
        counter = 0
        heap = []
        for idx in heap_list:
            heap.append((tuple(idx.pointed._data), counter, idx))
            counter += 1
        heapq.heapify(heap)
        lines = []
        last_kmer, last_cnt = None, 0
        while heap:
            _, _, idx = heapq.heappop(heap)
            if last_kmer is not None and idx.pointed == last_kmer:
                last_cnt += 1
            else:
                if last_kmer is not None:
                    lines.append(f"{last_kmer.to_string()}\t{last_cnt}\n")
                last_kmer, last_cnt = idx.pointed, 1
            idx.advance()
            if not idx.exhausted():
                heapq.heappush(heap, (tuple(idx.pointed._data), counter, idx))
                counter += 1
        lines.append(f"{last_kmer.to_string()}\t{last_cnt}\n")
        lines.append("EOF")
        files[bin_id] = "".join(lines)
    return files


def extract_kx_mers_ht(k: int, bins: dict[int, list[Kmer]]) -> dict[int, dict[str, int]]:
    """SparkBinKmerCounter.scala:664-739 (map iteration order is unspecified,
    so the result is returned as {bin: {kmer: count}})."""
    res = {}
    for bin_id, sks in bins.items():
        counts: dict[Kmer, int] = {}
        for sk in sks:
            for i in range(0, sk.length - k + 1):
                o = get_orientation(sk, i, i + k - 1)
                km = Kmer.from_kmer(k, sk, i, i + k - 1, o)
                counts[km] = counts.get(km, 0) + 1
        if counts:
            res[bin_id] = {km.to_string(): c for km, c in counts.items()}
    return res


def clamp_bins(m: int, b: int) -> int:  # test/package.scala:32
    return int(min(4.0 ** m, float(b)))


def parse_reads(fasta: bytes) -> list[bytes]:
    """Record values with '\\n' removed (SparkBinKmerCounter.scala:62-65)."""
    reads, cur, in_rec = [], None, False
    for line in fasta.split(b"\n"):
        if line.startswith(b">"):
            if in_rec:
                reads.append(bytes(cur))
            cur, in_rec = bytearray(), True
        elif in_rec:
            cur += line
    if in_rec:
        reads.append(bytes(cur))
    return reads


def run_sorted(fasta: bytes, k: int, m: int, x: int, b: int) -> dict[int, str]:
    """executeJob with useHT=0 (SparkBinKmerCounter.scala:1032-1035)."""
    bins = get_super_kmers(k, m, clamp_bins(m, b), parse_reads(fasta))
    return extract_kx_mers(k, x, bins)


def run_ht(fasta: bytes, k: int, m: int, b: int) -> dict[int, dict[str, int]]:
    """executeJob with useHT=1 (SparkBinKmerCounter.scala:1038-1042)."""
    bins = get_super_kmers(k, m, clamp_bins(m, b), parse_reads(fasta))
    return extract_kx_mers_ht(k, bins)
