/*
 * fastkmer.h -- C-ABI of the MI355X-native exact k-mer counter.
 *
 * Drop-in boundary for the hot path of maruscia/fastkmer: the body of
 *   SparkBinKmerCounter.executeJob(spark, configuration)
 *     src/main/scala/skc/SparkBinKmerCounter.scala:989-1046
 * i.e. the map closure getSuperKmers / getSuperKmersWithBinSizes (:34-169,
 * :290-426), the signature->bin shuffle reduceByKey (:1035, :1042) and the
 * reduce closures extractKXmers / extractKXmersHT (:428-660, :664-739).
 * INTEGRATION.md shows the JNI binding a Scala maintainer would add and the
 * ctypes binding used by this repository's tests.
 *
 * Plain C types only.  Every call returns FK_OK (0) or a negative FK_E_*
 * code and never aborts; fk_last_error() returns a thread-local message.
 * A context is used by one host thread at a time.  All GPU work runs on the
 * context's HIP stream on the device selected by fk_config.device.
 */
#ifndef FASTKMER_H
#define FASTKMER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version policy: bumped whenever an exported signature, a struct layout
 * (fk_config, fk_stats) or an error code's meaning changes; callers compare
 * fk_abi_version() with the FK_ABI_VERSION they were built against.
 *   3: fk_stats lost four always-zero fields (ht_spilled, ht_rounds, ms_merge,
 *      ht_big_groups); FK_E_COMM; fk_debug_comm_hold / _release / _held;
 *      fk_debug_fingerprint_bits. */
#define FK_ABI_VERSION 3

#define FK_OK 0
#define FK_E_INVALID (-1) /* bad argument or configuration (reference: require / AIOOBE) */
#define FK_E_STATE (-2)   /* call out of order (e.g. fk_get_bin before fk_finish) */
#define FK_E_DEVICE (-3)  /* HIP runtime failure or no usable GPU */
#define FK_E_NOMEM (-4)   /* device or host allocation failed */
#define FK_E_IO (-5)      /* file system error while writing bins */
#define FK_E_RANGE (-6)   /* caller buffer too small / bin out of range */
#define FK_E_COMM (-7)    /* a collective of the job failed or timed out (FASTKMER_COMM_TIMEOUT_S); the
                             communicator is aborted, later collective calls fail fast (reference: a failed
                             task fails the Spark job, SBKC:1031-1043) */

/* Mirrors skc.test.testutil.TestConfiguration (test/package.scala:16-42). */
typedef struct fk_config {
    int32_t k;             /* k-mer length, 1..64 (reference: any; Kmer packs 31 nt/Long) */
    int32_t m;             /* signature length, 1..15 (m >= 16 breaks Int shifts, SBKC:50) */
    int32_t x;             /* (k,x)-mer factor; must be >= 1 when use_ht == 0 (SBKC:435) */
    int32_t B;             /* requested bins; the library uses b = min(4^m, B) (package.scala:32) */
    int32_t use_ht;        /* 0: sorted count (extractKXmers), 1: hash count (extractKXmersHT) */
    int32_t sequence_type; /* 0: FASTA short reads, 1: long sequence (FASTdoop long format) */
    int32_t write;         /* reference "write" flag; only consulted by the CLI */
    int32_t n_ranks;       /* >= 1: bins are owned round-robin, bin % n_ranks == rank */
    int32_t rank;          /* 0..n_ranks-1 */
    int32_t device;        /* HIP device ordinal, -1 = current device */
} fk_config;

typedef struct fk_ctx fk_ctx;

/* Per-context statistics (device times are HIP-event times on the ctx stream). */
typedef struct fk_stats {
    uint64_t fasta_bytes;      /* bytes ingested */
    uint64_t positions;        /* sequence positions after FASTA parsing */
    uint64_t bases;            /* A/C/G/T/N... sequence bytes (input bases) */
    uint64_t kmers;            /* valid k-mer windows counted */
    uint64_t superkmers;       /* super-k-mer records produced by fk_map */
    uint64_t records_received; /* records counted by fk_reduce */
    uint64_t distinct;         /* distinct canonical k-mers owned by this rank */
    uint64_t oversize_buckets; /* buckets that took the large-bucket path */
    uint64_t buckets;          /* LDS count buckets (sorted path) */
    uint64_t fine_bits;        /* cell bits F below the bin (sorted path) */
    double ms_parse;           /* FASTA parse + 2-bit encode kernels */
    double ms_signature;       /* signature / super-k-mer kernel */
    double ms_partition;       /* record partition kernels */
    double ms_count;           /* expand + bucket + sort/hash + compact kernels */
    double ms_total;           /* fk_map + fk_reduce wall time on the host */
    double ms_encode_kernel;   /* last launch of the encode kernel */
    double ms_signature_kernel;/* last launch of the signature kernel (the fused parse + signature kernel when fused_map) */
    uint64_t fused_map;        /* 1: the last fk_map ran the fused kernel (k_map_fused), 0: parse + signature kernels */
    double ms_h2d;             /* last fk_ingest: host-to-device copy, first segment issued to last landed */
    uint64_t fused_fallback;   /* why the fused kernel handed the input back: 1 long line, 2 text before the
                                  first header, 4 halo too short, 8 too many records in a tile (0: none) */
    /* multi-rank exchange inside the context (fk_comm_init*), last fk_finish */
    uint64_t xch_steps;        /* exchange steps (pieces sent during fk_ingest, the last piece, closing steps) */
    uint64_t xch_bytes_sent;   /* record bytes sent to other ranks */
    uint64_t xch_bytes_received; /* record bytes received from other ranks */
    double ms_exchange;        /* sum over the steps of their record transfer time on the comm stream */
    double ms_exchange_tail;   /* fk_finish: the last piece posted -> every rank's records received */
    /* pieces counted while later ones were still being copied in / received (sorted count) */
    uint64_t pieces_counted;   /* staged pieces of the last fk_finish (0: one count of the whole input) */
    uint64_t heavy_keys;       /* sorted count: k-mers in the buckets above the wave tier (split or block / big) */
    uint64_t block_buckets;    /* block tier: buckets above the wave tier of at most 1024 keys (k <= 32: the mid wave
                                  tier) / 2048 keys (k > 32: mid wave tier, LDS sort) */
    uint64_t big_buckets;      /* above the block tier (k <= 32: split into sub-buckets, fallbacks to the block /
                                  big-table kernels; k > 32: the streaming path) */
    uint64_t split_buckets;    /* k <= 32: buckets above the wave tier split into wave-sized sub-buckets */
    uint64_t sub_buckets;      /* ... into this many sub-buckets (the wave tier counted them) */
} fk_stats;

/* ---- host-only helpers (no GPU needed) ---------------------------------- */

int fk_abi_version(void);
/* Defaults of LocalTestKmerCounter.main (LocalTestKmerCounter.scala:20-33). */
int fk_config_init(fk_config *cfg);
/* Validates without touching the GPU; FK_E_INVALID with a message on error. */
int fk_config_validate(const fk_config *cfg);
/* b = min(4^m, B) exactly as TestConfiguration.b (test/package.scala:32). */
int32_t fk_clamped_bins(int32_t m, int32_t B);
/* TestConfiguration.outputDir (test/package.scala:33, debug == false). */
int fk_output_dir(const fk_config *cfg, const char *output_path, const char *prefix, char *out, size_t cap);
/* Bytes of one packed super-k-mer record for k (16 for k <= 32, 24 for k <= 64). */
size_t fk_record_bytes_for_k(int32_t k);
/* Deterministic synthetic short-read FASTA (">r%010d\n" + read + "\n"),
 * identical on host and device; see fk_synth_fasta_device. */
uint64_t fk_synth_record_bytes(int32_t read_len);
int fk_synth_fasta_host(uint8_t *out, uint64_t first_read, uint64_t n_reads, int32_t read_len,
                        uint64_t genome_len, uint64_t seed, double err_rate, double n_rate);

/* ---- context ------------------------------------------------------------ */

int fk_create(const fk_config *cfg, fk_ctx **out);
void fk_destroy(fk_ctx *ctx);
const char *fk_last_error(void);
/* Optional: run on a caller-owned hipStream_t (e.g. torch's current stream). */
int fk_set_stream(fk_ctx *ctx, void *hip_stream);

/* Input.  fk_ingest copies host FASTA bytes to the device (may be called
 * repeatedly: the chunks are concatenated; last = 1 marks the final chunk).
 * The copy runs in segments on the context's copy stream and, for the fused
 * map configurations, every tile whose bytes have landed is mapped while the
 * next segment is in flight; the call returns once the source has been read.
 * fk_ingest_device borrows a device buffer (zero-copy; it must stay valid
 * until fk_map returns, and one borrowed input is mapped once). */
int fk_ingest(fk_ctx *ctx, const uint8_t *fasta, size_t n, int last);
/* Optional, before a streamed fk_ingest sequence: size the device input for
 * about total_bytes, so the copies of later chunks overlap the map without a
 * reallocation (FASTdoop-style streaming ingest).  The size also
 * places the job's piece cuts and sizes its cells, as for a job passed in one
 * fk_ingest call (a wrong size costs time, never results). */
int fk_ingest_reserve(fk_ctx *ctx, uint64_t total_bytes);
int fk_ingest_device(fk_ctx *ctx, const void *d_fasta, size_t n, int last);
/* A rank's input split of a FASTA file, as the reference's FASTdoop input
 * formats cut it for its map tasks (SBKC:993, 1009-1012): the file is cut into
 * byte ranges of ~size/world.  sequence_type 0 (FASTAshortInputFileFormat):
 * the whole records whose '>' lies in the rank's range.  sequence_type 1
 * (FASTAlongInputFileFormat, overlap key "k"): the k-mer windows whose first
 * base lies in the range -- a header line ">s\n", the range's bytes (after a
 * header line it starts inside; nothing before the file's first header), the
 * k - 1 sequence positions after it (stopping at a record boundary), "\n".
 * The union of the ranks' counts is the whole file's.
 *   fk_split_bytes: host only; the bytes rank `rank` ingests into out (cap
 *     bytes; out = NULL: only *n, the split's size).
 *   fk_ingest_file_range: the whole job input of this context from the file
 *     (a fresh job, as one fk_ingest sequence with last = 1 at its end): the
 *     split of (k, sequence_type) of the context's configuration, read with
 *     positioned reads into two pinned windows of window_bytes (0: 256 MB;
 *     the next window is read while the last one is copied and mapped), the
 *     job's size announced first (fk_ingest_reserve).  Collective like
 *     fk_ingest with a communicator.  world / rank: the split (usually the
 *     context's n_ranks / rank; with a communicator they must be, else
 *     FK_E_INVALID). */
int fk_split_bytes(const char *path, int32_t world, int32_t rank, int32_t k, int32_t sequence_type, uint8_t *out,
                   size_t cap, size_t *n);
int fk_ingest_file_range(fk_ctx *ctx, const char *path, int32_t world, int32_t rank, uint64_t window_bytes);
/* Fill a caller's device buffer (current device) with the same bytes as
 * fk_synth_fasta_host (benchmarks: the input is staged to pinned host memory). */
int fk_synth_fasta_to_device(void *d_out, uint64_t first_read, uint64_t n_reads, int32_t read_len,
                             uint64_t genome_len, uint64_t seed, double err_rate, double n_rate);
/* Fill the device input with fk_synth_fasta-compatible data (benchmarks). */
int fk_synth_fasta_device(fk_ctx *ctx, uint64_t first_read, uint64_t n_reads, int32_t read_len,
                          uint64_t genome_len, uint64_t seed, double err_rate, double n_rate);

/* Map side (getSuperKmers, SBKC:34-169): parse, encode, signature,
 * super-k-mer records; send_counts[r] = records destined to rank r. */
int fk_map(fk_ctx *ctx, uint64_t *send_counts);
size_t fk_record_bytes(const fk_ctx *ctx);
/* Write the mapped records into d_send grouped by destination rank
 * (rank 0 first), send_counts as returned by fk_map. */
int fk_map_emit(fk_ctx *ctx, void *d_send, uint64_t cap_records);
/* Reduce side (reduceByKey + extractKXmers[HT]): count the records in
 * d_recv (device memory, fk_record_bytes each, all owned by this rank). */
int fk_reduce(fk_ctx *ctx, const void *d_recv, uint64_t n_records);
/* Grouped exchange (default placement only): with fk_set_grouped_emit(ctx, 1)
 * before fk_map, fk_map_emit groups the records by (destination rank, local
 * bin) -- the reduceByKey grouping of SBKC:1035 done on the sender -- and
 * fk_map_part_counts returns records / k-mers per part ([n_ranks][parts],
 * parts = fk_grouped_parts_per_rank).  A receiver then skips its partition
 * pass: fk_reduce_grouped counts d_recv = n_seg segments (one per sender, in
 * order), each holding seg_records[s * parts + lb] records of local bin lb,
 * bin after bin. */
int fk_set_grouped_emit(fk_ctx *ctx, int32_t enable);
int32_t fk_grouped_parts_per_rank(const fk_ctx *ctx);
int fk_map_part_counts(fk_ctx *ctx, uint64_t *records, uint64_t *kmers);
int fk_reduce_grouped(fk_ctx *ctx, const void *d_recv, uint64_t n_records, const uint64_t *seg_records,
                      const uint64_t *seg_kmers, int32_t n_seg, int32_t parts_per_seg);
/* Single rank: fk_map + fk_reduce on the local records. */
int fk_finish(fk_ctx *ctx);

/* Size-aware bin placement, the MultiprocessorSchedulingPartitioner of the
 * reference (SBKC:1023-1025, MultiprocessorSchedulingPartitioner.scala:35-69)
 * with exact sizes instead of a 1% sample.  Default placement: bin % n_ranks.
 *   fk_map_bin_kmers: after fk_map, the k-mers per bin of this rank's records
 *     (all b bins); sum them over the ranks (e.g. an all-reduce),
 *   fk_lpt_owners: largest bin first onto the least loaded rank (host only;
 *     bins of size 0 keep bin % n_ranks),
 *   fk_set_bin_owners: install owner[b] (the same table on every rank) before
 *     fk_map_emit / fk_reduce, or before a job's first fk_ingest with a
 *     communicator (the exchange then groups records by (owner, the bin's index
 *     among its owner's bins)); when already mapped it recomputes send_counts
 *     (and, with the grouped emit, fk_map_part_counts) under the new owners, so
 *     fk_map_emit may follow directly. */
int fk_map_bin_kmers(fk_ctx *ctx, uint64_t *kmers_per_bin);
int fk_lpt_owners(const uint64_t *sizes, int32_t nbins, int32_t nranks, int32_t *owner);
int fk_set_bin_owners(fk_ctx *ctx, const int32_t *owner, uint64_t *send_counts);
/* The context's placement: owner[b] for all b bins (bin % n_ranks unless set). */
int fk_bin_owners(const fk_ctx *ctx, int32_t *owner);

/* ---- multi-GPU inside the context (one context per GPU) --------
 * The job's contexts (fk_config.n_ranks = n, rank = 0..n-1) join one
 * communicator.  A context then exchanges its records itself: fk_ingest
 * groups every landed piece of its input (FASTKMER_PIECE_BYTES, 1 GB) by
 * (owner rank, local bin) and sends it while the next piece is still being
 * copied in; fk_finish sends the last piece, receives every rank's, and
 * counts the bins this rank owns (bin % n_ranks), as the executors of the
 * reference's reduceByKey shuffle do (SBKC:1034-1042).  fk_finish (and
 * fk_ingest, which may send pieces) are collective: every rank of the job
 * calls them, each from its own host thread or process.  Ranks may hold
 * different amounts of input: a rank that has sent its last piece keeps
 * answering the others' steps inside fk_finish.
 * Failure semantics (the reference fails the whole Spark job when one task
 * fails: require at package.scala:182,185, exceptions out of SBKC:1031-1043):
 * every host wait on RCCL work is bounded -- it polls the stream and
 * ncclCommGetAsyncError, and after FASTKMER_COMM_TIMEOUT_S seconds (default
 * 120) or an asynchronous RCCL error it aborts the communicator
 * (ncclCommAbort) and the call returns FK_E_COMM; any failing collective call
 * aborts it too, so the peers' waits end instead of blocking.
 * FASTKMER_COMM_SPLIT=0 keeps the per-step count exchange on the records'
 * communicator and stream (default: a communicator split off it, with its own
 * stream). */
#define FK_COMM_ID_BYTES 128
/* A fresh RCCL unique id (ncclGetUniqueId): made on one rank, handed to all. */
int fk_comm_unique_id(uint8_t id[FK_COMM_ID_BYTES]);
/* RCCL over xGMI: joins the job's communicator (blocks until every rank has joined). */
int fk_comm_init(fk_ctx *ctx, const uint8_t id[FK_COMM_ID_BYTES]);
/* n contexts of this process as ranks 0..n-1 (created with n_ranks = n): records move
 * by device-to-device copies; drive each context from its own host thread. */
int fk_comm_init_local(fk_ctx **ctxs, int32_t n);
/* "rccl", "local" or "" (no communicator). */
const char *fk_comm_transport(const fk_ctx *ctx);
/* Collective: v[0..n) summed over the job's ranks (in place). */
int fk_comm_allreduce_u64(fk_ctx *ctx, uint64_t *v, size_t n);
/* Size-aware placement for the library's exchange (useCustomPartitioner:
 * SBKC:1023-1026, MultiprocessorSchedulingPartitioner.scala:35-69), collective,
 * before a job's first fk_ingest: every rank maps a sample of its input (never
 * exchanged), the per-bin k-mer totals are summed over the ranks, and the LPT
 * placement (fk_lpt_owners) is installed on every rank (fk_set_bin_owners);
 * the job's records then go to their bin's owner.  Without a communicator the
 * rank's own sample decides.
 *   fk_balance_bins: the caller's sample bytes (FASTA text);
 *   fk_balance_bins_file: `fraction` of the rank's split of the file (evenly
 *     spaced blocks; the reference samples 1 %); world / rank as for
 *     fk_ingest_file_range. */
int fk_balance_bins(fk_ctx *ctx, const uint8_t *sample, size_t n);
int fk_balance_bins_file(fk_ctx *ctx, const char *path, int32_t world, int32_t rank, double fraction);
/* Host-only arithmetic of one exchange step.  sent[d * (2 * parts + 1) + i] is this
 * rank's message to rank d: records of local bin i (i < parts), k-mers of local bin
 * i - parts, then a flag word (bit 0: the sender's last piece, bit 1: the sender
 * retracts its earlier pieces); received[] holds every sender's message to this
 * rank in the same layout.  Fills the byte offsets and sizes of the step's send
 * blocks (records grouped by destination, rank 0 first) and receive blocks (by
 * sender), and *all_final (every sender has sent its last piece). */
int fk_exchange_plan(int32_t n_ranks, int32_t parts, const uint64_t *sent, const uint64_t *received,
                     uint64_t record_bytes, uint64_t *send_off, uint64_t *send_bytes, uint64_t *recv_off,
                     uint64_t *recv_bytes, int32_t *all_final);

/* ---- results (device resident; copied out on request) ------------------ */

int32_t fk_num_bins(const fk_ctx *ctx); /* b = min(4^m, B) */
/* distinct[b] for all b (0 for bins owned by other ranks). */
int fk_bin_sizes(fk_ctx *ctx, uint64_t *distinct_per_bin);
/* Canonical k-mers of bin b and their counts.  useHT=0: ascending
 * lexicographic order (extractKXmers); useHT=1: table order.  keys hold one
 * word per k-mer for k <= 32 and two (first k-32 bases, last 32 bases) for
 * k > 32, 2 bits per base, A=0 C=1 G=2 T=3, most significant base first. */
int fk_get_bin(fk_ctx *ctx, int32_t bin, uint64_t *keys, uint32_t *counts, size_t cap, size_t *n);
/* Reference byte format: <out_dir>/bin<b>, "<kmer>\t<count>\n" lines, plus
 * "EOF" (no newline) when use_ht == 0 (SBKC:550-606, :715-734). */
int fk_write_bins(fk_ctx *ctx, const char *out_dir);
int fk_get_stats(fk_ctx *ctx, fk_stats *out);

/* ---- test hook (no reference counterpart) ----
 * One bucket through the wave-tier count kernel on `device`: the n keys
 * (k <= 32: one word each, n <= 512; 33 <= k <= 63: (hi, lo) pairs, n <= 256)
 * must lie in cells [c0, c1) of F cell bits (cell = top F bits of the 2k-bit
 * key); slots = table slots per bucket, the product's (640, or 384 for k > 32).
 * Writes the distinct keys ascending and their counts, *n_out of them.  Lets
 * tests drive adversarial buckets (every key in one rank group, keys over all
 * groups) that FASTA inputs cannot aim at. */
int fk_debug_wave_count(int32_t device, int32_t k, int32_t F, uint32_t c0, uint32_t c1, int32_t slots,
                        const uint64_t *keys, uint32_t n, uint64_t *out_keys, uint32_t *out_counts,
                        uint32_t *n_out);

/* ---- test hooks of the failure semantics (no reference counterpart) ----
 * fk_debug_comm_hold queues, on every stream the context's collectives run on,
 * a one-thread kernel that spins on a host-mapped flag (it ends by itself after
 * max_seconds), so that the next collective call waits on a stream that does
 * not drain -- what a rank blocked by a dead peer sees.  fk_debug_comm_release
 * sets the flag (callable from another thread while a collective is waiting);
 * fk_destroy releases it too. */
int fk_debug_comm_hold(fk_ctx *ctx, int32_t max_seconds);
int fk_debug_comm_release(fk_ctx *ctx);
/* 1 while the context's comm stream has not drained (e.g. still held), else 0. */
int fk_debug_comm_held(fk_ctx *ctx);

/* Test hook: the 128-bit wave tier (33 <= k <= 63) dedupes on 64-bit key
 * fingerprints and checks every key against its slot's claimer; a shared
 * fingerprint sends the bucket to an exact count from LDS.  This cuts
 * the fingerprints of `device` to their low `bits` bits (0: whole, the
 * product), so that tests drive that path on every bucket. */
int fk_debug_fingerprint_bits(int32_t device, int32_t bits);

/* Measurement hook: per-phase wave cycles of the fused map kernel summed over
 * its launches since the last reset (out[0..16)); only a library built with
 * -DFK_PROBES records them (FK_E_STATE otherwise). */
int fk_debug_map_cycles(uint64_t *out16, int32_t reset);

/* ---- bin-signature diagnostics (executeFindBinSignaturesJob, SBKC:956-986) ----
 * fk_signature_counts: after the final fk_ingest (the input is left in place,
 *   fk_map may follow), d_counts[v] (device memory of the ctx device, uint64)
 *   = super-k-mers with signature v over this rank's input -- getBinSignatures
 *   (SBKC:772-917); v = 4^m when every m-mer of the window is forbidden.  It
 *   needs fk_signature_slots(ctx) = 4^m + 1 entries.  Across ranks, sum the
 *   arrays (an all-reduce: the reduceByKey of SBKC:984) before writing.
 * fk_write_bin_signatures: saveBinSignatures (SBKC:920-953) for the bins this
 *   rank owns: <out_dir>/bin_signatures<b>.txt, "<signature>\t<count>\n" lines
 *   (longToString: 31 characters, PKG:616-634) in ascending signature order,
 *   then "Total\t<sum>\n"; bins without signatures get no file. */
uint64_t fk_signature_slots(const fk_ctx *ctx);
int fk_signature_counts(fk_ctx *ctx, void *d_counts, uint64_t n_counts);
int fk_write_bin_signatures(fk_ctx *ctx, const void *d_counts, uint64_t n_counts, const char *out_dir);
/* The whole job on one rank (n_ranks == 1, or each rank's own input unmerged):
 * fk_signature_counts into a library-owned buffer, then fk_write_bin_signatures. */
int fk_find_bin_signatures(fk_ctx *ctx, const char *out_dir);

#ifdef __cplusplus
}
#endif
#endif /* FASTKMER_H */
