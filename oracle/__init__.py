"""CPU parity oracle for the fastkmer hot path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package ``fastkmer_amd``.

``oracle/fk_oracle.c`` is a plain-C restatement of the reference algorithm
(see its header for the file:line map); ``oracle/literal_ref.py`` is a
step-for-step Python transliteration of the Scala code used to pin it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libfk_oracle.so")
_lib = None


def build(force: bool = False) -> str:
    """Compile the C oracle with gcc (oracle/Makefile)."""
    src = os.path.join(_HERE, "fk_oracle.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        L.fko_is_allowed.argtypes = [ctypes.c_int32, ctypes.c_int32]
        L.fko_is_allowed.restype = ctypes.c_int
        L.fko_norm.argtypes = [ctypes.c_int32, ctypes.c_int32]
        L.fko_norm.restype = ctypes.c_int32
        L.fko_hash_to_bucket.argtypes = [ctypes.c_int32, ctypes.c_int32]
        L.fko_hash_to_bucket.restype = ctypes.c_int32
        L.fko_clamp_bins.argtypes = [ctypes.c_int32, ctypes.c_int32]
        L.fko_clamp_bins.restype = ctypes.c_int32
        L.fko_count.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_int32,
                                ctypes.c_int32, ctypes.c_int32]
        L.fko_count.restype = ctypes.c_void_p
        L.fko_count_mt.argtypes = L.fko_count.argtypes + [ctypes.c_int32]
        L.fko_count_mt.restype = ctypes.c_void_p
        L.fko_count_mt_filtered.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_int32]
        L.fko_count_mt_filtered.restype = ctypes.c_void_p
        for name in ("fko_total_kmers", "fko_superkmers", "fko_reads", "fko_distinct"):
            getattr(L, name).argtypes = [ctypes.c_void_p]
            getattr(L, name).restype = ctypes.c_int64
        L.fko_nbins.argtypes = [ctypes.c_void_p]
        L.fko_nbins.restype = ctypes.c_int32
        L.fko_bin_size.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        L.fko_bin_size.restype = ctypes.c_int64
        L.fko_bin_get.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_void_p]
        L.fko_bin_get.restype = ctypes.c_int
        L.fko_write_bins.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int32]
        L.fko_write_bins.restype = ctypes.c_int
        L.fko_free.argtypes = [ctypes.c_void_p]
        L.fko_free.restype = None
        L.fko_trace_read.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                     ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_int64]
        L.fko_trace_read.restype = ctypes.c_int64
        L.fko_bin_signatures.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_void_p]
        L.fko_bin_signatures.restype = ctypes.c_int
        L.fko_write_bin_signatures.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p]
        L.fko_write_bin_signatures.restype = ctypes.c_int
        _lib = L
    return _lib


def is_allowed(v: int, m: int) -> bool:
    return bool(lib().fko_is_allowed(v, m))


def norm(v: int, m: int) -> int:
    return lib().fko_norm(v, m)


def hash_to_bucket(s: int, b: int) -> int:
    return lib().fko_hash_to_bucket(s, b)


def clamp_bins(m: int, b: int) -> int:
    return lib().fko_clamp_bins(m, b)


def kmer_to_string(hi: int, lo: int, k: int) -> str:
    v = (int(hi) << 64) | int(lo)
    out = []
    for _ in range(k):
        out.append("ACGT"[v & 3])
        v >>= 2
    return "".join(reversed(out))


class OracleResult:
    """Per-bin sorted (canonical k-mer, count) lists computed on the CPU."""

    def __init__(self, fasta: bytes, k: int, m: int, B: int, sequence_type: int = 0, threads: int = 1,
                 bin_mod: int = 0, bin_rem: int = 0, ptr: int = 0, nbytes: int = 0):
        """fasta: the input bytes, or (fasta=None) `nbytes` bytes at address `ptr` (e.g. a pinned
        multi-GB buffer, read in place).  bin_mod > 0 keeps only the bins b % bin_mod == bin_rem
        (the others are walked and counted in total_kmers, not stored): a memory bound for checks
        at the full per-GPU loads."""
        L = lib()
        self.k, self.m = k, m
        self.bin_mod, self.bin_rem = bin_mod, bin_rem
        if fasta is None:
            self._buf = None
            h = L.fko_count_mt_filtered(ctypes.c_void_p(ptr), nbytes, k, m, B, sequence_type, max(1, threads),
                                        bin_mod, bin_rem)
        elif bin_mod:
            self._buf = bytes(fasta)
            h = L.fko_count_mt_filtered(ctypes.cast(ctypes.c_char_p(self._buf), ctypes.c_void_p), len(self._buf),
                                        k, m, B, sequence_type, max(1, threads), bin_mod, bin_rem)
        elif threads > 1:
            self._buf = bytes(fasta)
            h = L.fko_count_mt(self._buf, len(self._buf), k, m, B, sequence_type, threads)
        else:
            self._buf = bytes(fasta)
            h = L.fko_count(self._buf, len(self._buf), k, m, B, sequence_type)
        if not h:
            raise ValueError(f"invalid oracle parameters k={k} m={m} B={B}")
        self._h = ctypes.c_void_p(h)
        self.nbins = L.fko_nbins(self._h)
        self.total_kmers = L.fko_total_kmers(self._h)
        self.superkmers = L.fko_superkmers(self._h)
        self.reads = L.fko_reads(self._h)
        self.distinct = L.fko_distinct(self._h)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib is not None:
            _lib.fko_free(h)
            self._h = None

    def bin_size(self, b: int) -> int:
        return lib().fko_bin_size(self._h, b)

    def bin_sizes(self):
        import numpy as np
        return np.array([self.bin_size(b) for b in range(self.nbins)], dtype=np.int64)

    def bin_arrays(self, b: int):
        """(hi, lo, counts) numpy arrays in ascending key order."""
        import numpy as np
        n = self.bin_size(b)
        hi = np.zeros(n, dtype=np.uint64)
        lo = np.zeros(n, dtype=np.uint64)
        cnt = np.zeros(n, dtype=np.uint32)
        if n:
            lib().fko_bin_get(self._h, b, hi.ctypes.data, lo.ctypes.data, cnt.ctypes.data)
        return hi, lo, cnt

    def bin_dict(self, b: int) -> dict:
        hi, lo, cnt = self.bin_arrays(b)
        return {kmer_to_string(h, l, self.k): int(c) for h, l, c in zip(hi, lo, cnt)}

    def all_dict(self) -> dict:
        return {b: self.bin_dict(b) for b in range(self.nbins) if self.bin_size(b)}

    def write_bins(self, out_dir: str, sorted_eof: bool = True) -> None:
        rc = lib().fko_write_bins(self._h, out_dir.encode(), 1 if sorted_eof else 0)
        if rc != 0:
            raise OSError(f"fko_write_bins failed ({rc})")

    def bin_text(self, b: int, sorted_eof: bool = True) -> str:
        lines = [f"{s}\t{c}\n" for s, c in self.bin_dict(b).items()]
        return "".join(lines) + ("EOF" if sorted_eof else "")


def trace_read(read: bytes, k: int, m: int, B: int):
    """Super-k-mers (start, length, bin) that getSuperKmers emits for one read."""
    import numpy as np
    cap = max(16, len(read) + 1)
    st = np.zeros(cap, dtype=np.int64)
    ln = np.zeros(cap, dtype=np.int64)
    bn = np.zeros(cap, dtype=np.int32)
    n = lib().fko_trace_read(read, len(read), k, m, B, st.ctypes.data, ln.ctypes.data, bn.ctypes.data, cap)
    if n < 0:
        raise ValueError("invalid parameters")
    return [(int(st[i]), int(ln[i]), int(bn[i])) for i in range(n)]


def bin_signatures(fasta: bytes, k: int, m: int):
    """getBinSignatures (SBKC:772-917) merged over reads: int64 counts[0..4^m],
    super-k-mers per signature value (fko_bin_signatures)."""
    import numpy as np
    counts = np.zeros((1 << (2 * m)) + 1, dtype=np.int64)
    if lib().fko_bin_signatures(fasta, len(fasta), k, m, counts.ctypes.data) != 0:
        raise ValueError(f"invalid parameters k={k} m={m}")
    return counts


def write_bin_signatures(counts, m: int, B: int, out_dir: str) -> None:
    """saveBinSignatures (SBKC:920-953) for every bin: bin_signatures<b>.txt."""
    import numpy as np
    c = np.ascontiguousarray(counts, dtype=np.int64)
    if c.shape != ((1 << (2 * m)) + 1,):
        raise ValueError("counts must hold 4^m + 1 entries")
    if lib().fko_write_bin_signatures(c.ctypes.data, m, B, out_dir.encode()) != 0:
        raise OSError(f"writing bin signatures under {out_dir} failed")
