"""fastkmer_amd -- MI355X-native exact k-mer counter (host-side mirror).

The compute path is the HIP library ``fastkmer_amd/lib/libfastkmer.so``
(C-ABI in ``include/fastkmer.h``); this module binds it with ctypes and
mirrors the reference's driver-side API:

* :class:`TestConfiguration`  -- skc.test.testutil.TestConfiguration
  (src/main/scala/skc/test/package.scala:16-42)
* :func:`execute_job`         -- SparkBinKmerCounter.executeJob
  (src/main/scala/skc/SparkBinKmerCounter.scala:989-1046)
* :class:`KmerCounter`        -- the map / shuffle / reduce hot path as one
  device-resident object (getSuperKmers :34-169, reduceByKey :1035,
  extractKXmers :428-660, extractKXmersHT :664-739)

There is no CPU fallback: without the built library, or without a GPU,
constructing a :class:`KmerCounter` raises.
"""
from __future__ import annotations

import ctypes
import dataclasses
import os
import re

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FASTKMER_LIB") or os.path.join(_PKG, "lib", "libfastkmer.so")
CLI_PATH = os.path.join(_PKG, "bin", "fastkmer-cli")
HEADER_PATH = os.path.join(os.path.dirname(_PKG), "include", "fastkmer.h")

FK_OK = 0
ERRORS = {-1: "FK_E_INVALID", -2: "FK_E_STATE", -3: "FK_E_DEVICE", -4: "FK_E_NOMEM", -5: "FK_E_IO",
          -6: "FK_E_RANGE", -7: "FK_E_COMM"}
ABI_VERSION = 3  # include/fastkmer.h FK_ABI_VERSION this binding mirrors (fk_config / fk_stats layouts)


class FastKmerError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"{ERRORS.get(code, code)}: {message}")
        self.code = code


class fk_config(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("k", "m", "x", "B", "use_ht", "sequence_type", "write", "n_ranks", "rank", "device")]


class fk_stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in
                ("fasta_bytes", "positions", "bases", "kmers", "superkmers", "records_received", "distinct",
                 "oversize_buckets", "buckets", "fine_bits")] + \
               [(n, ctypes.c_double) for n in
                ("ms_parse", "ms_signature", "ms_partition", "ms_count", "ms_total", "ms_encode_kernel",
                 "ms_signature_kernel")] + [("fused_map", ctypes.c_uint64), ("ms_h2d", ctypes.c_double),
                                       ("fused_fallback", ctypes.c_uint64),
                                       ("xch_steps", ctypes.c_uint64), ("xch_bytes_sent", ctypes.c_uint64),
                                       ("xch_bytes_received", ctypes.c_uint64), ("ms_exchange", ctypes.c_double),
                                       ("ms_exchange_tail", ctypes.c_double),
                                       ("pieces_counted", ctypes.c_uint64),
                                       ("heavy_keys", ctypes.c_uint64), ("block_buckets", ctypes.c_uint64), ("big_buckets", ctypes.c_uint64),
                                       ("split_buckets", ctypes.c_uint64),
                                       ("sub_buckets", ctypes.c_uint64)]

COMM_ID_BYTES = 128


_lib = None


def header_functions() -> list[str]:
    """Names of the functions declared in include/fastkmer.h."""
    with open(HEADER_PATH) as f:
        text = f.read()
    return re.findall(r"^[A-Za-z_][\w \*]*?\b(fk_\w+)\s*\(", text, re.M)


def lib():
    """Load the HIP library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m fastkmer_amd.build` "
                           "(there is no CPU fallback)")
    # One HIP runtime per process: torch ships its own libamdhip64 with the
    # same SONAME as /opt/rocm's.  Loading torch first makes the dynamic
    # loader bind libfastkmer.so to that runtime, so device pointers, streams
    # and RCCL (torch.distributed "nccl") are shared with torch.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    P, I32, U64, SZ = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64, ctypes.c_size_t
    sig = {
        "fk_abi_version": (ctypes.c_int, []),
        "fk_config_init": (ctypes.c_int, [ctypes.POINTER(fk_config)]),
        "fk_config_validate": (ctypes.c_int, [ctypes.POINTER(fk_config)]),
        "fk_clamped_bins": (I32, [I32, I32]),
        "fk_output_dir": (ctypes.c_int, [ctypes.POINTER(fk_config), ctypes.c_char_p, ctypes.c_char_p,
                                         ctypes.c_char_p, SZ]),
        "fk_record_bytes_for_k": (SZ, [I32]),
        "fk_synth_record_bytes": (U64, [I32]),
        "fk_synth_fasta_host": (ctypes.c_int, [P, U64, U64, I32, U64, U64, ctypes.c_double, ctypes.c_double]),
        "fk_create": (ctypes.c_int, [ctypes.POINTER(fk_config), ctypes.POINTER(P)]),
        "fk_destroy": (None, [P]),
        "fk_last_error": (ctypes.c_char_p, []),
        "fk_set_stream": (ctypes.c_int, [P, P]),
        "fk_ingest": (ctypes.c_int, [P, ctypes.c_char_p, SZ, ctypes.c_int]),
        "fk_ingest_device": (ctypes.c_int, [P, P, SZ, ctypes.c_int]),
        "fk_ingest_reserve": (ctypes.c_int, [P, U64]),
        "fk_split_bytes": (ctypes.c_int, [ctypes.c_char_p, I32, I32, I32, I32, P, SZ, ctypes.POINTER(SZ)]),
        "fk_ingest_file_range": (ctypes.c_int, [P, ctypes.c_char_p, I32, I32, U64]),
        "fk_synth_fasta_device": (ctypes.c_int, [P, U64, U64, I32, U64, U64, ctypes.c_double, ctypes.c_double]),
        "fk_synth_fasta_to_device": (ctypes.c_int, [P, U64, U64, I32, U64, U64, ctypes.c_double, ctypes.c_double]),
        "fk_map": (ctypes.c_int, [P, P]),
        "fk_record_bytes": (SZ, [P]),
        "fk_map_emit": (ctypes.c_int, [P, P, U64]),
        "fk_reduce": (ctypes.c_int, [P, P, U64]),
        "fk_set_grouped_emit": (ctypes.c_int, [P, ctypes.c_int32]),
        "fk_grouped_parts_per_rank": (ctypes.c_int32, [P]),
        "fk_map_part_counts": (ctypes.c_int, [P, P, P]),
        "fk_reduce_grouped": (ctypes.c_int, [P, P, U64, P, P, ctypes.c_int32, ctypes.c_int32]),
        "fk_finish": (ctypes.c_int, [P]),
        "fk_num_bins": (I32, [P]),
        "fk_bin_sizes": (ctypes.c_int, [P, P]),
        "fk_get_bin": (ctypes.c_int, [P, I32, P, P, SZ, ctypes.POINTER(SZ)]),
        "fk_write_bins": (ctypes.c_int, [P, ctypes.c_char_p]),
        "fk_get_stats": (ctypes.c_int, [P, ctypes.POINTER(fk_stats)]),
        "fk_map_bin_kmers": (ctypes.c_int, [P, P]),
        "fk_lpt_owners": (ctypes.c_int, [P, I32, I32, P]),
        "fk_set_bin_owners": (ctypes.c_int, [P, P, P]),
        "fk_bin_owners": (ctypes.c_int, [P, P]),
        "fk_signature_slots": (U64, [P]),
        "fk_signature_counts": (ctypes.c_int, [P, P, U64]),
        "fk_write_bin_signatures": (ctypes.c_int, [P, P, U64, ctypes.c_char_p]),
        "fk_find_bin_signatures": (ctypes.c_int, [P, ctypes.c_char_p]),
        "fk_comm_unique_id": (ctypes.c_int, [P]),
        "fk_comm_init": (ctypes.c_int, [P, P]),
        "fk_comm_init_local": (ctypes.c_int, [P, I32]),
        "fk_comm_transport": (ctypes.c_char_p, [P]),
        "fk_comm_allreduce_u64": (ctypes.c_int, [P, P, SZ]),
        "fk_balance_bins": (ctypes.c_int, [P, ctypes.c_char_p, SZ]),
        "fk_balance_bins_file": (ctypes.c_int, [P, ctypes.c_char_p, I32, I32, ctypes.c_double]),
        "fk_exchange_plan": (ctypes.c_int, [I32, I32, P, P, U64, P, P, P, P, P]),
        "fk_debug_map_cycles": (ctypes.c_int, [P, I32]),
        "fk_debug_comm_hold": (ctypes.c_int, [P, I32]),
        "fk_debug_comm_release": (ctypes.c_int, [P]),
        "fk_debug_comm_held": (ctypes.c_int, [P]),
        "fk_debug_fingerprint_bits": (ctypes.c_int, [I32, I32]),
        "fk_debug_wave_count": (ctypes.c_int, [I32, I32, I32, ctypes.c_uint32, ctypes.c_uint32, I32, P,
                                               ctypes.c_uint32, P, P, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.fk_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH} has ABI version {L.fk_abi_version()}, this binding mirrors {ABI_VERSION}: "
                           "rebuild it (python -m fastkmer_amd.build)")
    _lib = L
    return L


def _check(rc: int) -> None:
    if rc != FK_OK:
        raise FastKmerError(rc, lib().fk_last_error().decode(errors="replace"))


def make_config(k: int, m: int, x: int = 3, B: int = 2048, use_ht: bool = False, sequence_type: int = 0,
                write: bool = False, n_ranks: int = 1, rank: int = 0, device: int = -1) -> fk_config:
    c = fk_config()
    lib().fk_config_init(ctypes.byref(c))
    c.k, c.m, c.x, c.B = k, m, x, B
    c.use_ht, c.sequence_type, c.write = int(bool(use_ht)), sequence_type, int(bool(write))
    c.n_ranks, c.rank, c.device = n_ranks, rank, device
    return c


def validate(**kw) -> None:
    """Host-only configuration check (no GPU); raises FastKmerError."""
    c = make_config(**kw)
    _check(lib().fk_config_validate(ctypes.byref(c)))


def clamped_bins(m: int, B: int) -> int:
    return lib().fk_clamped_bins(m, B)


def record_bytes_for_k(k: int) -> int:
    return lib().fk_record_bytes_for_k(k)


def synth_fasta(n_reads: int, read_len: int = 100, genome_len: int = 1_000_000, seed: int = 0x5EED,
                err_rate: float = 0.002, n_rate: float = 0.0005, first_read: int = 0) -> bytes:
    """Deterministic synthetic short-read FASTA (byte-identical to the device generator)."""
    L = lib()
    nb = n_reads * L.fk_synth_record_bytes(read_len)
    buf = ctypes.create_string_buffer(max(nb, 1))
    _check(L.fk_synth_fasta_host(buf, first_read, n_reads, read_len, genome_len, seed, err_rate, n_rate))
    return buf.raw[:nb]


def synth_fasta_to_device(ptr: int, n_reads: int, read_len: int = 100, genome_len: int = 1_000_000,
                          seed: int = 0x5EED, err_rate: float = 0.002, n_rate: float = 0.0005,
                          first_read: int = 0) -> int:
    """The bytes of synth_fasta written into a device buffer at ptr (current device); returns the size."""
    L = lib()
    _check(L.fk_synth_fasta_to_device(ctypes.c_void_p(ptr), first_read, n_reads, read_len, genome_len, seed,
                                      err_rate, n_rate))
    return n_reads * L.fk_synth_record_bytes(read_len)


def split_bytes(path: str, world: int, rank: int, k: int, sequence_type: int = 0) -> bytes:
    """The bytes rank `rank` of `world` ingests from the FASTA file at `path` (fk_split_bytes: the
    FASTdoop-style input split of SBKC:993, 1009-1012; host only)."""
    L = lib()
    n = ctypes.c_size_t()
    p = os.fsencode(path)
    _check(L.fk_split_bytes(p, world, rank, k, sequence_type, None, 0, ctypes.byref(n)))
    buf = ctypes.create_string_buffer(max(n.value, 1))
    _check(L.fk_split_bytes(p, world, rank, k, sequence_type, buf, n.value, ctypes.byref(n)))
    return buf.raw[:n.value]


def decode_keys(keys: np.ndarray, k: int) -> list[str]:
    """2-bit keys (one word for k <= 32, (hi, lo) pairs for k > 32) -> strings."""
    out = []
    words = keys.reshape(-1, 2) if k > 32 else keys.reshape(-1, 1)
    for row in words:
        v = (int(row[0]) << 64) | int(row[1]) if k > 32 else int(row[0])
        s = []
        for _ in range(k):
            s.append("ACGT"[v & 3])
            v >>= 2
        out.append("".join(reversed(s)))
    return out


@dataclasses.dataclass
class TestConfiguration:
    """Mirror of skc.test.testutil.TestConfiguration (test/package.scala:16-42)."""
    __test__ = False  # not a pytest class

    dataset: str
    outputDirectory: str
    k: int
    m: int
    x: int
    max_b: int = 2000
    sequenceType: int = 0
    canonical: bool = True
    debug: bool = False
    write: bool = True
    useKryoSerializer: bool = False
    useHT: bool = False
    useCustomPartitioner: bool = False
    numPartitionTasks: int = 0
    prefix: str = ""

    @property
    def b(self) -> int:  # :32
        return int(min(4.0 ** self.m, float(self.max_b)))

    @property
    def outputDir(self) -> str:  # :33
        base = "/tmp/" if self.debug else self.outputDirectory
        tail = f"{self.prefix}k{self.k}_m{self.m}_x{self.x}_b{self.b}"
        return base + tail if self.debug else base + tail + f"_s{self.sequenceType}"


class KmerCounter:
    """Device-resident exact canonical k-mer counter for one rank."""

    def __init__(self, k: int, m: int, x: int = 3, B: int = 2048, use_ht: bool = False, sequence_type: int = 0,
                 n_ranks: int = 1, rank: int = 0, device: int = -1):
        L = lib()
        self.k, self.m, self.x, self.use_ht = k, m, x, bool(use_ht)
        self.n_ranks, self.rank = n_ranks, rank
        self._cfg = make_config(k, m, x, B, use_ht, sequence_type, False, n_ranks, rank, device)
        self._device = device
        h = ctypes.c_void_p()
        _check(L.fk_create(ctypes.byref(self._cfg), ctypes.byref(h)))
        self._h = h
        self.num_bins = L.fk_num_bins(h)
        self.record_bytes = L.fk_record_bytes(h)
        self._keep = None
        self._sizes = None

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().fk_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- input
    def ingest(self, fasta: bytes) -> None:
        self._keep = bytes(fasta)
        _check(lib().fk_ingest(self._h, self._keep, len(self._keep), 1))

    def ingest_ptr(self, ptr: int, n: int, last: bool = True) -> None:
        """Append n host bytes at ptr (pinned memory is copied by DMA directly)."""
        _check(lib().fk_ingest(self._h, ctypes.cast(ptr, ctypes.c_char_p), n, 1 if last else 0))

    def ingest_chunk(self, chunk: bytes, last: bool) -> None:
        """Streamed input: append one chunk (the map of the landed bytes overlaps the copies)."""
        _check(lib().fk_ingest(self._h, chunk, len(chunk), 1 if last else 0))

    def reserve(self, total_bytes: int) -> None:
        """Size the device input for a streamed ingest of about total_bytes."""
        _check(lib().fk_ingest_reserve(self._h, total_bytes))

    def ingest_file_range(self, path: str, world: int | None = None, rank: int | None = None,
                          window_bytes: int = 0) -> None:
        """The job's input from a file: this rank's split (fk_ingest_file_range; world / rank
        default to the context's), read in pinned windows while earlier ones are copied and mapped."""
        _check(lib().fk_ingest_file_range(self._h, os.fsencode(path), self.n_ranks if world is None else world,
                                          self.rank if rank is None else rank, window_bytes))

    def balance_bins(self, sample: bytes) -> np.ndarray:
        """Size-aware placement (useCustomPartitioner) for the library's exchange, collective: the
        ranks' samples mapped, their per-bin k-mers summed, LPT owners installed; returns them."""
        _check(lib().fk_balance_bins(self._h, sample, len(sample)))
        return self.bin_owners()

    def balance_bins_file(self, path: str, fraction: float = 0.01, world: int | None = None,
                          rank: int | None = None) -> np.ndarray:
        """balance_bins from `fraction` of this rank's split of the file (the reference samples 1 %)."""
        _check(lib().fk_balance_bins_file(self._h, os.fsencode(path), self.n_ranks if world is None else world,
                                          self.rank if rank is None else rank, fraction))
        return self.bin_owners()

    def comm_allreduce(self, v) -> np.ndarray:
        """Collective: v summed over the job's ranks."""
        a = np.ascontiguousarray(v, dtype=np.uint64).copy()
        _check(lib().fk_comm_allreduce_u64(self._h, a.ctypes.data, a.size))
        return a

    def ingest_device(self, ptr: int, n: int) -> None:
        _check(lib().fk_ingest_device(self._h, ctypes.c_void_p(ptr), n, 1))

    def synth_device(self, n_reads: int, read_len: int = 100, genome_len: int = 100_000_000, seed: int = 0x5EED,
                     err_rate: float = 0.002, n_rate: float = 0.0005, first_read: int = 0) -> int:
        _check(lib().fk_synth_fasta_device(self._h, first_read, n_reads, read_len, genome_len, seed, err_rate,
                                           n_rate))
        return n_reads * lib().fk_synth_record_bytes(read_len)

    def set_stream(self, stream_ptr: int) -> None:
        _check(lib().fk_set_stream(self._h, ctypes.c_void_p(stream_ptr)))

    # -- map / shuffle / reduce
    def map(self) -> list[int]:
        self._sizes = None
        counts = (ctypes.c_uint64 * self.n_ranks)()
        _check(lib().fk_map(self._h, counts))
        return list(counts)

    def map_bin_kmers(self) -> np.ndarray:
        """After map(): k-mers per bin (all b bins) of this rank's records."""
        out = np.zeros(self.num_bins, dtype=np.uint64)
        _check(lib().fk_map_bin_kmers(self._h, out.ctypes.data))
        return out

    def bin_owners(self) -> np.ndarray:
        """The placement: owner rank of every bin."""
        out = np.zeros(self.num_bins, dtype=np.int32)
        _check(lib().fk_bin_owners(self._h, out.ctypes.data))
        return out

    def set_bin_owners(self, owner) -> list[int]:
        """Install a bin -> rank placement (identical on every rank); returns the
        send counts of the mapped records under it."""
        own = np.ascontiguousarray(owner, dtype=np.int32)
        if own.shape != (self.num_bins,):
            raise ValueError(f"owner table needs {self.num_bins} entries")
        counts = (ctypes.c_uint64 * self.n_ranks)()
        _check(lib().fk_set_bin_owners(self._h, own.ctypes.data, counts))
        self._sizes = None
        return list(counts)

    def map_emit(self, dst_ptr: int, cap_records: int) -> None:
        _check(lib().fk_map_emit(self._h, ctypes.c_void_p(dst_ptr), cap_records))

    def reduce(self, src_ptr: int, n_records: int) -> None:
        self._sizes = None
        _check(lib().fk_reduce(self._h, ctypes.c_void_p(src_ptr), n_records))

    def set_grouped_emit(self, enable: bool = True) -> int:
        """Group the emitted records by (destination, local bin); returns the
        parts per destination (fk_set_grouped_emit)."""
        _check(lib().fk_set_grouped_emit(self._h, 1 if enable else 0))
        return lib().fk_grouped_parts_per_rank(self._h)

    def map_part_counts(self):
        """After map() with grouped emit: (records, k-mers) per part, shape [n_ranks, parts]."""
        parts = lib().fk_grouped_parts_per_rank(self._h)
        rec = np.zeros(self.n_ranks * parts, dtype=np.uint64)
        km = np.zeros(self.n_ranks * parts, dtype=np.uint64)
        _check(lib().fk_map_part_counts(self._h, rec.ctypes.data, km.ctypes.data))
        return rec.reshape(self.n_ranks, parts), km.reshape(self.n_ranks, parts)

    def reduce_grouped(self, src_ptr: int, n_records: int, seg_records, seg_kmers) -> None:
        """Count records grouped by sender and local bin (fk_reduce_grouped);
        seg_records / seg_kmers: [n_senders, parts] arrays."""
        self._sizes = None
        sr = np.ascontiguousarray(seg_records, dtype=np.uint64)
        sk = np.ascontiguousarray(seg_kmers, dtype=np.uint64)
        if sr.shape != sk.shape or sr.ndim != 2:
            raise ValueError("seg_records and seg_kmers must be [n_senders, parts] arrays of one shape")
        _check(lib().fk_reduce_grouped(self._h, ctypes.c_void_p(src_ptr), n_records, sr.ctypes.data, sk.ctypes.data,
                                       sr.shape[0], sr.shape[1]))

    def finish(self) -> None:
        """Single rank: map + count.  With a communicator (comm_init / comm_init_local):
        the last piece, the exchange with the other ranks, and the count of this rank's
        bins -- collective, every rank of the job calls it."""
        self._sizes = None
        _check(lib().fk_finish(self._h))

    # -- multi-GPU inside the library (fk_comm_*)
    def comm_init(self, unique_id: bytes) -> None:
        """Join the job's RCCL communicator (unique_id from comm_unique_id() on one rank)."""
        if len(unique_id) != COMM_ID_BYTES:
            raise ValueError(f"an RCCL unique id has {COMM_ID_BYTES} bytes")
        buf = ctypes.create_string_buffer(bytes(unique_id), COMM_ID_BYTES)
        _check(lib().fk_comm_init(self._h, buf))

    @property
    def comm_transport(self) -> str:
        return lib().fk_comm_transport(self._h).decode()

    # -- results
    def bin_sizes(self) -> np.ndarray:
        out = np.zeros(self.num_bins, dtype=np.uint64)
        _check(lib().fk_bin_sizes(self._h, out.ctypes.data))
        return out

    def get_bin(self, b: int):
        n = ctypes.c_size_t(0)
        if self._sizes is None:
            self._sizes = self.bin_sizes()
        cnt = int(self._sizes[b])
        kw = 2 if self.k > 32 else 1
        keys = np.zeros(max(cnt, 1) * kw, dtype=np.uint64)
        counts = np.zeros(max(cnt, 1), dtype=np.uint32)
        _check(lib().fk_get_bin(self._h, b, keys.ctypes.data, counts.ctypes.data, max(cnt, 1), ctypes.byref(n)))
        return keys[:n.value * kw], counts[:n.value]

    def bin_dict(self, b: int) -> dict:
        keys, counts = self.get_bin(b)
        return dict(zip(decode_keys(keys, self.k), (int(c) for c in counts)))

    def all_dict(self) -> dict:
        sizes = self.bin_sizes()
        return {b: self.bin_dict(b) for b in np.nonzero(sizes)[0].tolist()}

    def bin_text(self, b: int) -> str:
        keys, counts = self.get_bin(b)
        lines = [f"{s}\t{int(c)}\n" for s, c in zip(decode_keys(keys, self.k), counts)]
        return "".join(lines) + ("" if self.use_ht else "EOF")

    def write_bins(self, out_dir: str) -> None:
        _check(lib().fk_write_bins(self._h, out_dir.encode()))

    # -- bin-signature diagnostics (executeFindBinSignaturesJob, SBKC:956-986)
    def signature_counts(self, out=None):
        """getBinSignatures (SBKC:772-917) over the ingested input: a device
        int64 tensor of 4^m + 1 super-k-mer counts indexed by signature value
        (``out``, if given, must hold that many).  The input stays ingested."""
        import torch
        n = lib().fk_signature_slots(self._h)
        if out is None:
            out = torch.empty(n, dtype=torch.int64, device=self._torch_device())
        if out.numel() < n or out.dtype != torch.int64 or not out.is_cuda or not out.is_contiguous():
            raise ValueError(f"signature counts need a contiguous device int64 tensor of {n} entries")
        _check(lib().fk_signature_counts(self._h, ctypes.c_void_p(out.data_ptr()), out.numel()))
        return out

    def write_bin_signatures(self, counts, out_dir: str) -> None:
        """saveBinSignatures (SBKC:920-953) for the bins this rank owns."""
        _check(lib().fk_write_bin_signatures(self._h, ctypes.c_void_p(counts.data_ptr()), counts.numel(),
                                             out_dir.encode()))

    def _torch_device(self):
        import torch
        return torch.device("cuda", self._device if self._device >= 0 else torch.cuda.current_device())

    def stats(self) -> dict:
        st = fk_stats()
        _check(lib().fk_get_stats(self._h, ctypes.byref(st)))
        return {n: getattr(st, n) for n, _ in fk_stats._fields_}


def debug_wave_count(keys: np.ndarray, k: int, F: int, c0: int, c1: int, slots: int, device: int = 0):
    """Test hook (fk_debug_wave_count): one bucket of keys (uint64; (hi, lo) rows
    for k > 32) through the wave-tier count kernel; returns (distinct keys, counts)."""
    kw = 1 if k <= 32 else 2
    keys = np.ascontiguousarray(keys, dtype=np.uint64).reshape(-1, kw)
    n = len(keys)
    ok = np.zeros(n * kw, dtype=np.uint64)
    oc = np.zeros(n, dtype=np.uint32)
    nout = ctypes.c_uint32(0)
    _check(lib().fk_debug_wave_count(device, k, F, c0, c1, slots, keys.ctypes.data, n, ok.ctypes.data,
                                     oc.ctypes.data, ctypes.byref(nout)))
    u = nout.value
    return (ok[:u] if kw == 1 else ok[:2 * u].reshape(-1, 2)), oc[:u]


def comm_unique_id() -> bytes:
    """A fresh RCCL unique id (fk_comm_unique_id): made on one rank, handed to all."""
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    _check(lib().fk_comm_unique_id(buf))
    return buf.raw


def comm_init_local(counters) -> None:
    """Join KmerCounters of this process (ranks 0..n-1) into one in-process group
    (fk_comm_init_local); drive each from its own thread."""
    arr = (ctypes.c_void_p * len(counters))(*[c._h.value for c in counters])
    _check(lib().fk_comm_init_local(arr, len(counters)))


def exchange_plan(sent, received, record_bytes: int):
    """fk_exchange_plan: one exchange step's send / receive byte blocks.
    sent / received: [n_ranks, 2 * parts + 1] u64 messages.  Returns
    (send_off, send_bytes, recv_off, recv_bytes, all_final)."""
    snd = np.ascontiguousarray(sent, dtype=np.uint64)
    rcv = np.ascontiguousarray(received, dtype=np.uint64)
    if snd.ndim != 2 or snd.shape != rcv.shape or snd.shape[1] % 2 != 1:
        raise ValueError("sent / received must be [n_ranks, 2 * parts + 1] arrays of one shape")
    n, parts = snd.shape[0], (snd.shape[1] - 1) // 2
    so, sb, ro, rb = (np.zeros(n, dtype=np.uint64) for _ in range(4))
    fin = ctypes.c_int32(0)
    _check(lib().fk_exchange_plan(n, parts, snd.ctypes.data, rcv.ctypes.data, record_bytes, so.ctypes.data,
                                  sb.ctypes.data, ro.ctypes.data, rb.ctypes.data, ctypes.byref(fin)))
    return so, sb, ro, rb, bool(fin.value)


def lpt_owners(sizes, n_ranks: int) -> np.ndarray:
    """MultiprocessorSchedulingPartitioner.solve (MultiprocessorSchedulingPartitioner.scala:35-69):
    bins largest first onto the least loaded rank; bins of size 0 stay at bin % n_ranks."""
    sz = np.ascontiguousarray(sizes, dtype=np.uint64)
    owner = np.zeros(len(sz), dtype=np.int32)
    _check(lib().fk_lpt_owners(sz.ctypes.data, len(sz), n_ranks, owner.ctypes.data))
    return owner


def execute_job(configuration: TestConfiguration) -> KmerCounter:
    """SparkBinKmerCounter.executeJob (SparkBinKmerCounter.scala:989-1046) on one GPU.

    Reads the dataset, counts, and writes ``configuration.outputDir/bin<b>``
    when ``configuration.write`` is set.  Returns the counter (results stay
    device resident until it is closed).
    """
    with open(configuration.dataset, "rb") as f:
        data = f.read()
    kc = KmerCounter(configuration.k, configuration.m, configuration.x, configuration.max_b,
                     configuration.useHT, configuration.sequenceType)
    kc.ingest(data)
    kc.finish()
    if configuration.write:
        kc.write_bins(configuration.outputDir)
    return kc


def execute_find_bin_signatures_job(configuration: TestConfiguration):
    """SparkBinKmerCounter.executeFindBinSignaturesJob (SBKC:956-986) on one GPU:
    per-signature super-k-mer counts of the dataset, written as
    ``configuration.outputDir/bin_signatures<b>.txt``.  Returns the counts (a
    device int64 tensor indexed by signature value)."""
    with open(configuration.dataset, "rb") as f:
        data = f.read()
    with KmerCounter(configuration.k, configuration.m, configuration.x, configuration.max_b,
                     configuration.useHT, configuration.sequenceType) as kc:
        kc.ingest(data)
        counts = kc.signature_counts()
        kc.write_bin_signatures(counts, configuration.outputDir)
    return counts
