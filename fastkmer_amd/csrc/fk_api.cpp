// fk_api.cpp -- C-ABI of the MI355X k-mer counter (include/fastkmer.h).
//
// Host orchestration of the device pipeline in fk_kernels.hip.  Replaces the
// body of SparkBinKmerCounter.executeJob (SparkBinKmerCounter.scala:989-1046):
// the map closure, the reduceByKey shuffle and the reduce closure.  All device
// memory is owned by the context and reused across calls (grow-only).
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <unistd.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>

#include <algorithm>
#include <unordered_map>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fastkmer.h"
#include "fk_comm.h"
#include "fk_internal.h"
#include "fk_split.h"

#define FK_EXPORT extern "C" __attribute__((visibility("default")))

using namespace fk;

namespace {

thread_local std::string g_err;

int set_err(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                                \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess)                                                                        \
            return set_err(e_ == hipErrorOutOfMemory ? FK_E_NOMEM : FK_E_DEVICE, "%s failed: %s (%s:%d)", \
                           #expr, hipGetErrorString(e_), __FILE__, __LINE__);                        \
    } while (0)

#define FK_TRY(expr)             \
    do {                         \
        int r_ = (expr);         \
        if (r_ != FK_OK) return r_; \
    } while (0)

// Grow-only pinned host memory: small uploads and read-backs on the hot path go
// through it (pageable transfers are staged by the runtime, and block the host).
struct PinBuf {
    void *p = nullptr;
    size_t bytes = 0;
    int ensure(size_t need) {
        if (bytes >= need) return FK_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
        const size_t want = std::max<size_t>(need + need / 4, 4096);
        if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            return FK_E_NOMEM;
        }
        bytes = want;
        return FK_OK;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <typename T>
    T *as() const { return reinterpret_cast<T *>(p); }
};

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    template <typename T>
    T *as() const { return reinterpret_cast<T *>(p); }
};

int ensure(DevBuf &b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return FK_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    // slack for the next job's slightly larger input: an eighth, at most 1 GiB (4 GB of slack on each
    // k-mer array of a 6.25 GB job would cost more HBM than the reallocations it saves)
    const size_t want = bytes + std::min<size_t>(bytes / 8, 1ull << 30) + 256;
    hipError_t e = hipMalloc(&b.p, want);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return set_err(FK_E_NOMEM, "hipMalloc(%zu) failed: %s", want, hipGetErrorString(e));
    }
    b.bytes = want;
    return FK_OK;
}

void release(DevBuf &b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

// Record partition (fk_partition.inc): histogram -> scan -> scatter.
struct PartBufs {
    DevBuf H, K, Hs, Ts, KT;              // per-workgroup histograms and destinations (rows), segment sums
    DevBuf rec, kmer, off, cursor;        // per-part totals / offsets (device), cursor: global path only
    uint32_t nparts = 0;
    RecSrc src{};                         // the records counted (part_scatter reads the same)
    bool global = false;                  // nparts > PART_MAX: global-atomic kernels
    void release_all() {
        for (DevBuf *b : {&H, &K, &Hs, &Ts, &KT, &rec, &kmer, &off, &cursor}) release(*b);
    }
};

// Counts records and k-mers per part into pb.rec / pb.kmer (device) and keeps
// what part_scatter needs.
int part_count(PartBufs &pb, const RecSrc &src, int mode, uint32_t G, const uint32_t *table, uint32_t nparts,
               ScanWorkspace &ws, hipStream_t s) {
    pb.nparts = nparts;
    pb.src = src;
    pb.global = nparts > PART_MAX;
    FK_TRY(ensure(pb.rec, ((uint64_t)nparts + 1) * 8));
    FK_TRY(ensure(pb.kmer, ((uint64_t)nparts + 1) * 8));
    FK_TRY(ensure(pb.off, ((uint64_t)nparts + 1) * 8));
    if (pb.global) {
        HIP_TRY(hipMemsetAsync(pb.rec.p, 0, ((uint64_t)nparts + 1) * 8, s));
        HIP_TRY(hipMemsetAsync(pb.kmer.p, 0, ((uint64_t)nparts + 1) * 8, s));
        HIP_TRY(launch_part_hist_global(src, mode, G, table, nparts, pb.rec.as<uint64_t>(), pb.kmer.as<uint64_t>(), s));
        HIP_TRY(scan_excl_sum_u64(pb.rec.as<uint64_t>(), pb.off.as<uint64_t>(), nparts, pb.off.as<uint64_t>() + nparts,
                                  ws, s));
        return FK_OK;
    }
    const uint32_t nwg = src.nrec ? part_workgroups(src) : 0u;
    const uint64_t n = (uint64_t)nparts * nwg;
    FK_TRY(ensure(pb.H, n * 4));
    FK_TRY(ensure(pb.K, n * 4));
    const uint64_t nt = (uint64_t)nparts * part_segments(nwg);
    FK_TRY(ensure(pb.Hs, n * 8));
    FK_TRY(ensure(pb.Ts, (nt + 1) * 8));
    FK_TRY(ensure(pb.KT, nt * 8));
    if (n) {
        HIP_TRY(launch_part_hist(src, mode, G, table, nparts, pb.H.as<uint32_t>(), pb.K.as<uint32_t>(), s));
        HIP_TRY(launch_part_segsum(pb.H.as<uint32_t>(), pb.K.as<uint32_t>(), nparts, nwg, pb.Ts.as<uint64_t>(),
                                   pb.KT.as<uint64_t>(), s));
        HIP_TRY(scan_excl_sum_u64(pb.Ts.as<uint64_t>(), pb.Ts.as<uint64_t>(), nt, pb.Ts.as<uint64_t>() + nt, ws, s));
        HIP_TRY(launch_part_segfill(pb.H.as<uint32_t>(), pb.Ts.as<uint64_t>(), nparts, nwg, pb.Hs.as<uint64_t>(), s));
        HIP_TRY(launch_part_totals(pb.Ts.as<uint64_t>(), pb.KT.as<uint64_t>(), nparts, nwg, pb.rec.as<uint64_t>(),
                                   pb.kmer.as<uint64_t>(), pb.off.as<uint64_t>(), s));
    } else {
        HIP_TRY(hipMemsetAsync(pb.rec.p, 0, ((uint64_t)nparts + 1) * 8, s));
        HIP_TRY(hipMemsetAsync(pb.kmer.p, 0, ((uint64_t)nparts + 1) * 8, s));
        HIP_TRY(hipMemsetAsync(pb.off.p, 0, ((uint64_t)nparts + 1) * 8, s));
    }
    return FK_OK;
}

// Writes the records grouped by part (parts in order) into out.
int part_scatter(PartBufs &pb, int mode, uint32_t G, const uint32_t *table, uint64_t *out, hipStream_t s) {
    if (!pb.src.nrec) return FK_OK;
    if (pb.global) {
        FK_TRY(ensure(pb.cursor, ((uint64_t)pb.nparts + 1) * 8));
        HIP_TRY(hipMemsetAsync(pb.cursor.p, 0, ((uint64_t)pb.nparts + 1) * 8, s));
        HIP_TRY(launch_part_scatter_global(pb.src, mode, G, table, pb.nparts, pb.off.as<uint64_t>(),
                                           pb.cursor.as<uint64_t>(), out, s));
        return FK_OK;
    }
    HIP_TRY(launch_part_scatter(pb.src, mode, G, table, pb.nparts, pb.Hs.as<uint64_t>(), out, s));
    return FK_OK;
}

int32_t clamp_bins(int32_t m, int32_t B) {
    // test/package.scala:32: Math.min(Math.pow(4, m), max_b).toInt
    double p = 1.0;
    for (int i = 0; i < m; ++i) p *= 4.0;
    const double b = p < (double)B ? p : (double)B;
    return (int32_t)b;
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// -DFK_PROBES library, FASTKMER_HOST_TRACE=1: host timestamps of the count's steps on stderr (where
// the GPU waits on the host)
static void htrace(const char *what) {
#ifdef FK_PROBES
    static const bool on = getenv("FASTKMER_HOST_TRACE") && getenv("FASTKMER_HOST_TRACE")[0] == '1';
    if (on) fprintf(stderr, "htrace %.3f %s\n", now_ms(), what);
#else
    (void)what;
#endif
}

// Every exported call that touches the GPU selects the context's device for
// its duration and restores the caller's current device on return, so one
// thread may drive contexts on several GPUs and a context may move between
// threads (e.g. JNI executor threads).
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) {
            (void)hipGetLastError();
            prev = -1;
        }
        if (dev >= 0 && prev != dev) {
            (void)hipSetDevice(dev);
        } else {
            prev = -1;  // nothing to restore
        }
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};

constexpr int FUSED_NT = 512;  // threads per fused map workgroup (256-thread tiles measured 2.5 vs 1.1 ms per GB)
constexpr uint32_t CHUNK_RECORDS = 16384;  // records per expansion workgroup (never spans two bins)

// The sorted count's shape: cell bits F (super-cells of 2^F2 cells), tiers.
struct SortedPlan {
    int F = 1, F2 = 0, F1 = 1;
    bool tiered = false, two_level = false;
    uint32_t cap = 2048, wave_cap = WAVE_BUCKET_CAP;
    uint64_t max_bin = 0;  // the largest bin's k-mers the plan was made for
};

}  // namespace

#ifndef FK_SIDE_PRIO
#define FK_SIDE_PRIO 1  // A/B builds: -DFK_SIDE_PRIO=0 the heavy tiers' stream at normal priority
#endif

struct fk_ctx {
    fk_config cfg{};
    int32_t Bc = 0;    // b = min(4^m, B)
    uint32_t G = 1;    // ranks
    uint32_t nlb = 0;  // local bins: b = rank + G * lb (default placement) or lbin_bin[lb] (custom)
    // size-aware placement (fk_set_bin_owners): bin -> rank, bin -> local index, local index -> bin
    bool custom_owners = false;
    std::vector<int32_t> h_owner, h_lbin_bin;
    std::vector<uint32_t> h_bin_lbin;
    DevBuf d_owner, d_local;  // REC_BIN_MASK + 1 entries each (~0u: no part), device copies of the above
    int W = 2, KW = 1;
    FastMod fm{};
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // Test hooks (result-preserving; they steer inputs that FASTA data cannot aim at onto a path):
    bool force_large = false;  // FASTKMER_DEBUG_LARGE_BUCKETS=1: route every bucket through the streaming path
    uint32_t cell_target = 0;  // FASTKMER_DEBUG_CELL_TARGET: average keys per cell of the largest bin (0: auto)
    int mid_parts = -1;        // FASTKMER_DEBUG_MID_PARTS: the 64-bit mid tier's key ranges always (1), the whole
                               // buckets on the 512-key table always (2), the 1024-key kernel only (0), by size (-1)
    bool split_retry = false;  // FASTKMER_DEBUG_SPLIT_RETRY: every split bucket cut a second time
    int x2_l1 = 0;             // FASTKMER_X2_L1: level-1 workgroup size (512, 1024; 0 = by fan-out)
    int fused = 1;             // FASTKMER_FUSED=0: two-kernel map (parse, then signature) for every input
    // Measurement-only (a library built with -DFK_PROBES; wrong results by design):
    int dbg_phase = 99;        // FASTKMER_DEBUG_PHASE: stop the bucket kernel early
    int fused_probe = 0;       // FASTKMER_FUSED_PROBE: stop the fused map kernel after a phase
    int split_map = 0;         // FASTKMER_SPLIT_MAP=1: the map as a parse kernel + a signature-pass kernel
    bool last_map_fused = false;  // the last fk_map used the fused kernel (stats, tests)
    // grouped emit (fk_set_grouped_emit): send buffer grouped by (destination, local bin)
    bool grouped = false;
    uint32_t grp_nlb = 0;                    // parts per destination = ceil(Bc / n_ranks)
    DevBuf grp_table;                        // bin -> dest * grp_nlb + bin / n_ranks
    std::vector<uint64_t> grp_rec, grp_kmer; // per part, after fk_map
    const uint64_t *rsrc = nullptr;          // records the count stage reads (precs, or d_recv when grouped)

    // input
    // host ingest: bytes are streamed to fasta_own (appended until the next fk_map)
    bool ingest_fresh = true;        // the next fk_ingest starts a new input
    bool dev_open = false;           // fk_ingest_device(..., last = 0): the borrowed input is unfinished
    void *pinned[2] = {nullptr, nullptr};  // staging for pageable sources
    hipEvent_t pin_ev[2] = {nullptr, nullptr};
    hipStream_t copy_stream = nullptr;     // H2D of fk_ingest (the map runs on `stream` meanwhile)
    hipStream_t tier_side = nullptr;       // the count's heavy tiers beside the wave tier (FK_TIER_SIDE)
    // [0] cut -> wave tier, [1] heavy tiers -> result, [2] last piece's cell offsets -> cut, [3] -> heavy
    hipEvent_t side_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    bool cut_side = false;                 // the last staged piece: the job's bucket cut beside its expansion
    hipEvent_t seg_ev = nullptr;           // "segment landed" (copy stream -> map stream)
    hipEvent_t h2d_ev[2] = {nullptr, nullptr};  // first copy issued / last copy done (timing)
    // streamed map (fused path): fk_ingest maps every tile whose bytes (and halo) have landed
    bool pm_active = false;     // the current input is being mapped while it is copied
    uint64_t pm_tiles = 0;      // tiles [0, pm_tiles) launched
    bool pm_last_seen = false;  // an fk_ingest with last = 1 launched the final tiles
    const uint8_t *d_fasta = nullptr;
    uint64_t n_fasta = 0;
    DevBuf fasta_own;

    // parse + encode
    DevBuf tile_last_nl, tile_off, npos_dev, codes, valid;
    // signature
    DevBuf records, counters, sig_status, sig_kmers;
    DevBuf tcnt;                  // fused map: records per tile (tiled record layout)
    DevBuf rec_hdr;               // fused map: every record's header word, in the record's tile slot
    DevBuf rec_pos;               // fused map: every record's first position in its tile's code stream (u16)
    DevBuf rec_code;              // fused map: per tile, the tile's 2-bit code stream (map_fused_cslot() words)
    DevBuf tstat;                 // fused map: per tile (k-mers, positions)
    DevBuf map_vslots;            // split map: the parse kernel's valid streams for the passes (MAP_VSLOT_TILES tiles)
    bool rec_tiled = false;       // records: the fused map's tiles (else dense, c->nrec)
    uint64_t rec_tiles = 0;       // tiles of the tiled layout
    uint64_t nrec = 0, nkmers = 0;
    bool mapped = false;
    // destination partition (n_ranks > 1)
    std::vector<uint64_t> send_counts;
    // reduce
    PartBufs dest, part, binhist;  // record partition by destination rank (fk_map) / by local bin (fk_reduce)
    DevBuf precs, chunks, bin_chunk_begin;
    std::vector<uint32_t> h_bcb;  // bin_chunk_begin on the host (the last uploaded chunk table)
    DevBuf hpieces, hpiece_first, hpiece_tot;  // k_expand_hist_piece: bins split into pieces of chunks
    DevBuf chunk_nk, chunk_base, lp, cell_total, cell_base, flags, flag_scan, buckets, keys, out_keys, out_counts;
    DevBuf scratch;
    DevBuf bucket_unique, dense_off, dense_keys, dense_counts, bin_off, misc, tier_list, mid, sc_total;
    DevBuf sp_base, sp_keys, sp_subs, sp_par, sp_fb;  // heavy buckets split into sub-buckets
    DevBuf mid_fb;  // mid-tier buckets left to the 1024-key kernel by the ranges kernel
    ScanWorkspace ws;
    // results
    bool have_result = false;
    uint64_t distinct = 0;
    std::vector<uint64_t> h_bin_off;  // [nlb + 1]
    fk_stats stats{};
    // events: 0/1 parse, 2/3 signature, 4/5 partition, 6/7 count, 8/9 encode kernel, 10/11 sig kernel
    hipEvent_t ev[12] = {};
    double ms_h2d = 0.0;  // last fk_ingest: first copy issued -> last copy done
    bool ev_parse = false, ev_sig = false, ev_part = false, ev_count = false;
    std::vector<hipEvent_t> seg_evs;  // fk_ingest, pinned source: one "segment landed" event per segment
    std::vector<hipEvent_t> map_evs;  // ... and one "segment mapped" event (one rank's staged pieces)
    std::vector<uint64_t> seg_tiles;  // ... the tiles mapped once that segment's map is done
    PinBuf pin_up, pin_down;              // staging: chunk tables up, per-bin counts down
    hipEvent_t pin_up_ev = nullptr;       // the last upload out of pin_up (on whichever stream queued it)
    bool pin_up_busy = false;             // ... was queued and not yet waited for
    PinBuf pin_tier;                      // the bucket tiers' sizes, read while the wave tier runs
    PinBuf file_pin[2];                   // fk_ingest_file_range: the split read in pinned windows
    hipEvent_t tier_ev = nullptr;         // ... once this copy has landed
    bool distinct_pending = false;        // the sorted count's distinct total arrives with the bin offsets
    // The sorted count's result is bucket-major ("gapped"): bucket q's distinct keys ascending at its
    // first slot buckets[q].begin of res_keys / out_counts, dense_off[q] = their exclusive offset in the
    // bin-ordered result, bin_off / h_bin_off per bin.  Readers gather a bin's buckets (fk_get_bin) or
    // the whole result (fk_write_bins).
    bool gapped = false, dense_ready = false;
    const uint64_t *res_keys = nullptr;   // okb of the last sorted count (out_keys, or mid)
    const uint64_t *res_fs = nullptr;     // flag_scan of its bucket cut
    uint64_t res_nbuckets = 0;
    int res_F = 0;
    DevBuf gather_keys, gather_counts;    // fk_get_bin's gather of one bin

    // multi-rank exchange inside the context (fk_comm_init / fk_comm_init_local): the input
    // is emitted in pieces grouped by (destination, local bin) and each piece is exchanged
    // while the next one is still being copied in; fk_finish sends the last piece, then
    // counts every received segment (the reduceByKey shuffle of SBKC:1034-1042)
    // staged pieces (one rank, or the received segments with a communicator; sorted count, k <= 63):
    // each piece of the input is partitioned and expanded into its own key array while later pieces
    // land; the job's buckets are counted once over every piece's keys (no per-piece count, no merge)
    bool pieces_void = false;     // a fallback or a retract: the job is counted whole at the end
    uint64_t tiles_counted = 0;   // one rank: tiled records [0, tiles_counted) staged
    uint64_t job_bytes = 0;       // one rank: the job's input size when one fk_ingest call holds it all, or
                                  // announced by fk_ingest_reserve (0: unknown)
    uint64_t reserve_bytes = 0;   // fk_ingest_reserve's size for the next job
    size_t segs_counted = 0;      // with a communicator: received segments [0, segs_counted) staged
    std::vector<double> st_cuts{0.4, 0.7, 0.9};  // piece ends of a staged job (FASTKMER_PIECE_CUTS; 45 / 70 / 85 % measured 22.84 vs 22.77 ms)
    // ... of a 64-bit job of >= 4 GB without FASTKMER_PIECE_CUTS: five pieces, the last 7 % (configs[2]
    // load 146.2 -> 145.4 ms, profiles/r06z_five_pieces.txt; configs[1]'s 1 GB keeps four)
    std::vector<double> st_cuts5{0.38, 0.64, 0.82, 0.93};
    bool cuts_env = false;
    // ... with a communicator: earlier, a received piece lands a step's partition and transfer later
    // (one in-process rank at the configs[2] load: 153.2-153.7 ms against 156.1-159.4 with the local
    // cuts, profiles/r05z_xch_cuts_seg_ab.txt)
    std::vector<double> xst_cuts{0.35, 0.65, 0.84};
    uint32_t st_np = 0;                          // pieces expanded in the current job
    uint32_t st_cut = 0;                         // one rank: st_cuts passed in the current job
    SortedPlan st_plan;                          // the job's cells (fixed by its first piece)
    uint64_t st_kmers = 0;                       // k-mers expanded so far
    DevBuf st_keys[STAGE_MAXP], st_cb[STAGE_MAXP], st_total, piece_starts;
    hipEvent_t st_ev[4 * STAGE_MAXP] = {};       // per piece: partition begin / end, expansion begin / end

    fk::Comm *comm = nullptr;
    hipStream_t comm_stream = nullptr;
    uint32_t *hold_flag = nullptr;               // fk_debug_comm_hold: host-mapped release flag
    // staging of received segments on its own stream (each waits for its step's transfer, so the map
    // stream never does) with its own scan workspace; the count waits for it
    hipStream_t xstage = nullptr;
    hipEvent_t xstage_ev = nullptr;
    ScanWorkspace ws_x;
    hipEvent_t emit_ev = nullptr;                // map stream: a piece's send records are written
    std::vector<hipEvent_t> xev;                 // comm stream: begin / end of every piece's transfer
    uint64_t piece_bytes = 512ull << 20;         // FASTKMER_PIECE_BYTES: FASTA bytes per piece (with a
                                                 // communicator: a tenth of a known job, 128 MB .. 1 GB)
    bool piece_bytes_set = false;
    uint64_t ingest_seg = 32ull << 20;           // FASTKMER_INGEST_SEG: H2D segment of a pinned source
    DevBuf xsend, xrecv;                         // send ring (pieces in flight), received records
    struct XSeg {                                // received records of one (piece, sender)
        uint64_t off;                            // first record in xrecv
        int32_t sender;
        uint64_t step;                           // the exchange step that delivered it
        std::vector<uint64_t> rec, kmer;         // per local bin
    };
    struct Xch {
        bool open = false;           // a job's exchange has started (pieces sent)
        bool sent_final = false;     // this rank has sent its last piece
        bool all_final = false;      // every rank has sent its last piece
        bool stop_pieces = false;    // the fused map fell back: the rest goes in fk_finish, earlier pieces retracted
        uint64_t tiles_sent = 0;     // tiled records [0, tiles_sent) emitted in pieces
        uint64_t send_used = 0, recv_used = 0;  // records
        uint64_t pieces = 0, bytes_sent = 0, bytes_received = 0, expect_bytes = 0;
        std::vector<XSeg> segs;
    } xch;
};

// ---------------------------------------------------------------------------
// host-only helpers
// ---------------------------------------------------------------------------

FK_EXPORT int fk_abi_version(void) { return FK_ABI_VERSION; }

// Host waits on work that may depend on the exchange (the comm stream, the staging stream that waits
// for a step's transfer, events behind them): with a communicator they are bounded (Comm::wait: RCCL
// polls, times out after FASTKMER_COMM_TIMEOUT_S and aborts the communicator) and fail with FK_E_COMM.
static int comm_sync(fk_ctx *c, hipStream_t st) {
    if (!c->comm) {
        HIP_TRY(hipStreamSynchronize(st));
        return FK_OK;
    }
    std::string err;
    if (c->comm->wait(st, err)) return set_err(FK_E_COMM, "%s", err.c_str());
    return FK_OK;
}
static int comm_event_sync(fk_ctx *c, hipEvent_t ev) {
    if (!c->comm) {
        HIP_TRY(hipEventSynchronize(ev));
        return FK_OK;
    }
    std::string err;
    if (c->comm->wait_event(ev, err)) return set_err(FK_E_COMM, "%s", err.c_str());
    return FK_OK;
}

FK_EXPORT const char *fk_last_error(void) { return g_err.c_str(); }

FK_EXPORT int fk_config_init(fk_config *c) {
    if (!c) return set_err(FK_E_INVALID, "null config");
    // LocalTestKmerCounter.scala:20-33 defaults
    c->k = 20;
    c->m = 4;
    c->x = 3;
    c->B = 2000;
    c->use_ht = 0;
    c->sequence_type = 0;
    c->write = 0;
    c->n_ranks = 1;
    c->rank = 0;
    c->device = -1;
    return FK_OK;
}

FK_EXPORT int32_t fk_clamped_bins(int32_t m, int32_t B) { return clamp_bins(m, B); }

FK_EXPORT int fk_config_validate(const fk_config *c) {
    if (!c) return set_err(FK_E_INVALID, "null config");
    if (c->k < 1 || c->k > 64) return set_err(FK_E_INVALID, "k=%d out of range [1, 64]", c->k);
    if (c->m < 1 || c->m > 15)
        return set_err(FK_E_INVALID, "m=%d out of range [1, 15] (m >= 16 overflows Int shifts, SBKC:50)", c->m);
    if (c->m > c->k) return set_err(FK_E_INVALID, "m=%d must not exceed k=%d", c->m, c->k);
    if (c->B < 1) return set_err(FK_E_INVALID, "B=%d must be >= 1 (hash_to_bucket divides by B)", c->B);
    if (c->use_ht != 0 && c->use_ht != 1) return set_err(FK_E_INVALID, "use_ht must be 0 or 1");
    if (c->use_ht == 0 && c->x < 1)
        return set_err(FK_E_INVALID,
                       "x=%d: the sorted path needs x >= 1 (extractKXmers indexes R(runLength-1), SBKC:435/508)",
                       c->x);
    if (c->sequence_type != 0 && c->sequence_type != 1)
        return set_err(FK_E_INVALID, "sequence_type must be 0 (short) or 1 (long)");
    if (c->n_ranks < 1) return set_err(FK_E_INVALID, "n_ranks must be >= 1");
    if (c->rank < 0 || c->rank >= c->n_ranks) return set_err(FK_E_INVALID, "rank %d out of [0, %d)", c->rank, c->n_ranks);
    const int32_t bc = clamp_bins(c->m, c->B);
    if ((uint32_t)bc > REC_BIN_MASK + 1u)
        return set_err(FK_E_INVALID, "b = min(4^m, B) = %d exceeds the record header limit %u", bc, REC_BIN_MASK + 1u);
    return FK_OK;
}

FK_EXPORT int fk_output_dir(const fk_config *c, const char *output_path, const char *prefix, char *out, size_t cap) {
    if (!c || !out) return set_err(FK_E_INVALID, "null argument");
    // test/package.scala:33 (debug == false)
    const int n = snprintf(out, cap, "%s%sk%d_m%d_x%d_b%d_s%d", output_path ? output_path : "", prefix ? prefix : "",
                           c->k, c->m, c->x, clamp_bins(c->m, c->B), c->sequence_type);
    if (n < 0 || (size_t)n >= cap) return set_err(FK_E_RANGE, "output buffer too small (%d bytes needed)", n + 1);
    return FK_OK;
}

FK_EXPORT size_t fk_record_bytes_for_k(int32_t k) { return k <= 32 ? 16 : 24; }

FK_EXPORT uint64_t fk_synth_record_bytes(int32_t read_len) { return (uint64_t)read_len + 14; }

static SynthParams make_synth(uint64_t first_read, uint64_t n_reads, int32_t read_len, uint64_t genome_len,
                              uint64_t seed, double err_rate, double n_rate) {
    SynthParams p;
    p.first_read = first_read;
    p.n_reads = n_reads;
    p.genome_len = genome_len;
    p.seed = seed;
    p.read_len = (uint32_t)read_len;
    p.rec_bytes = (uint32_t)read_len + 14;
    const double two64 = 18446744073709551616.0;
    p.err_thresh = (uint64_t)(err_rate * two64 * 0.999999);
    p.n_thresh = (uint64_t)(n_rate * two64 * 0.999999);
    return p;
}

FK_EXPORT int fk_synth_fasta_host(uint8_t *out, uint64_t first_read, uint64_t n_reads, int32_t read_len,
                                  uint64_t genome_len, uint64_t seed, double err_rate, double n_rate) {
    if (!out || read_len < 1 || genome_len < 1) return set_err(FK_E_INVALID, "bad synth arguments");
    const SynthParams p = make_synth(first_read, n_reads, read_len, genome_len, seed, err_rate, n_rate);
    const uint64_t nb = n_reads * p.rec_bytes;
    for (uint64_t i = 0; i < nb; ++i) out[i] = synth_byte(p, i);
    return FK_OK;
}

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------

FK_EXPORT int fk_create(const fk_config *cfg, fk_ctx **out) {
    if (!out) return set_err(FK_E_INVALID, "null output pointer");
    *out = nullptr;
    FK_TRY(fk_config_validate(cfg));
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        return set_err(FK_E_DEVICE, "no HIP device available (%s): the k-mer counter runs on MI355X only",
                       hipGetErrorString(e));
    }
    fk_ctx *c = new fk_ctx();
    c->cfg = *cfg;
    c->Bc = clamp_bins(cfg->m, cfg->B);
    c->G = (uint32_t)cfg->n_ranks;
    c->nlb = (uint32_t)((c->Bc - cfg->rank + (int)c->G - 1) / (int)c->G);
    if (cfg->rank >= c->Bc) c->nlb = 0;
    c->W = cfg->k <= 32 ? 2 : 3;
    c->KW = cfg->k <= 32 ? 1 : 2;
    c->fm = make_fastmod((uint32_t)c->Bc);
    // The product library reads nine variables: three sizes of the streamed input and six test
    // hooks that steer small inputs onto paths only large or adversarial inputs reach (all
    // result-preserving).  Timing probes that alter results exist only in a library built with
    // -DFK_PROBES (python -m fastkmer_amd.build --probes).
    auto env = [](const char *name) -> const char * {
        const char *v = getenv(name);
        return v && v[0] ? v : nullptr;
    };
    if (const char *v = env("FASTKMER_PIECE_BYTES")) {  // piece size of a streamed job (1 GB with a communicator)
        c->piece_bytes = std::max(1ull << 16, strtoull(v, nullptr, 10));
        c->piece_bytes_set = true;
    }
    if (const char *v = env("FASTKMER_PIECE_CUTS")) {  // staged piece ends as job fractions, e.g. "0.4,0.7,0.9"
        c->st_cuts.clear();
        c->xst_cuts.clear();
        for (const char *q = v; *q;) {
            char *e = nullptr;
            const double f = strtod(q, &e);
            if (e == q) break;
            if (f > 0.0 && f < 1.0 && c->st_cuts.size() < STAGE_MAXP - 1) c->st_cuts.push_back(f), c->xst_cuts.push_back(f);
            c->cuts_env = true;
            q = *e == ',' ? e + 1 : e;
        }
    }
    if (const char *v = env("FASTKMER_INGEST_SEG")) c->ingest_seg = std::max(1ull << 16, strtoull(v, nullptr, 10));
    if (const char *v = env("FASTKMER_DEBUG_LARGE_BUCKETS")) c->force_large = v[0] == '1';
    if (const char *v = env("FASTKMER_DEBUG_CELL_TARGET")) c->cell_target = (uint32_t)atoi(v);
    if (const char *v = env("FASTKMER_DEBUG_MID_PARTS")) c->mid_parts = atoi(v);  // test hook: 1 / 2 / 0
    if (const char *v = env("FASTKMER_DEBUG_SPLIT_RETRY")) c->split_retry = v[0] == '1';  // test hook
    if (const char *v = env("FASTKMER_X2_L1")) c->x2_l1 = atoi(v);
    if (const char *v = env("FASTKMER_FUSED")) c->fused = atoi(v);
#ifdef FK_PROBES
    if (const char *v = env("FASTKMER_DEBUG_PHASE")) c->dbg_phase = atoi(v);
    if (const char *v = env("FASTKMER_FUSED_PROBE")) c->fused_probe = atoi(v);
    if (const char *v = env("FASTKMER_SPLIT_MAP")) c->split_map = atoi(v);
#endif
    if (cfg->device >= 0) {
        if (cfg->device >= ndev) {
            delete c;
            return set_err(FK_E_DEVICE, "device %d out of range (%d devices)", cfg->device, ndev);
        }
        c->device = cfg->device;
    } else {
        (void)hipGetDevice(&c->device);
    }
    DeviceGuard dg_(c->device);  // the caller's current device is restored on return
    {
        int cur = -1;
        if (hipGetDevice(&cur) != hipSuccess || cur != c->device) {
            (void)hipGetLastError();
            delete c;
            return set_err(FK_E_DEVICE, "cannot select device %d", c->device);
        }
    }
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return set_err(FK_E_DEVICE, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    c->own_stream = true;
    e = hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->seg_ev, hipEventDisableTiming);
    // staged pieces are partitioned and expanded on their own stream (one rank: so that the map of
    // later segments never queues behind a piece's expansion; the exchange: the received segments)
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->xstage, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->xstage_ev, hipEventDisableTiming);
    // the heavy tiers' stream at the device's highest priority (FK_SIDE_PRIO): their kernels are few
    // and long chains (split, in-order sub-buckets, fallbacks with large workgroups), and at normal
    // priority they waited for LDS behind the wave tier's millions of one-wave workgroups and ran
    // alone after it (the configs[2] load's split fallbacks: 13.8 ms of a kernel of ~40 workgroups)
    if (e == hipSuccess) {
        int least = 0, greatest = 0;
        if (FK_SIDE_PRIO && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
            e = hipStreamCreateWithPriority(&c->tier_side, hipStreamNonBlocking, greatest);
        else
            e = hipStreamCreateWithFlags(&c->tier_side, hipStreamNonBlocking);
    }
    for (int i = 0; i < 4 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&c->side_ev[i], hipEventDisableTiming);
    for (int i = 0; i < 2 && e == hipSuccess; ++i) e = hipEventCreate(&c->h2d_ev[i]);
    if (e != hipSuccess) {
        fk_destroy(c);
        return set_err(FK_E_DEVICE, "copy stream / events: %s", hipGetErrorString(e));
    }
    for (auto &ev : c->ev) {
        e = hipEventCreate(&ev);
        if (e != hipSuccess) {
            fk_destroy(c);
            return set_err(FK_E_DEVICE, "hipEventCreate: %s", hipGetErrorString(e));
        }
    }
    e = hipEventCreateWithFlags(&c->tier_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->pin_up_ev, hipEventDisableTiming);
    if (e != hipSuccess) {
        fk_destroy(c);
        return set_err(FK_E_DEVICE, "hipEventCreate: %s", hipGetErrorString(e));
    }
    for (auto &ev : c->st_ev) {
        e = hipEventCreate(&ev);
        if (e != hipSuccess) {
            fk_destroy(c);
            return set_err(FK_E_DEVICE, "hipEventCreate: %s", hipGetErrorString(e));
        }
    }
    *out = c;
    return FK_OK;
}

FK_EXPORT void fk_destroy(fk_ctx *c) {
    if (!c) return;
    DeviceGuard dg_(c->device);
    if (c->hold_flag) __atomic_store_n(c->hold_flag, 1u, __ATOMIC_RELEASE);  // a test's held streams drain
    if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    // staged expansions (an ingest without fk_finish) read the buffers released below
    if (c->xstage) (void)hipStreamSynchronize(c->xstage);
    DevBuf *bufs[] = {&c->fasta_own, &c->tile_last_nl, &c->tile_off,
                      &c->npos_dev, &c->codes, &c->valid, &c->records, &c->counters, &c->sig_status, &c->sig_kmers, &c->tcnt, &c->rec_hdr, &c->rec_pos, &c->rec_code, &c->tstat, &c->map_vslots,
                      &c->precs, &c->chunks, &c->bin_chunk_begin, &c->hpieces, &c->hpiece_first, &c->hpiece_tot, &c->chunk_nk, &c->grp_table,
                      &c->chunk_base, &c->lp, &c->scratch,
                      &c->cell_total, &c->cell_base, &c->flags, &c->flag_scan, &c->buckets, &c->keys,
                      &c->out_keys, &c->out_counts, &c->bucket_unique, &c->dense_off, &c->dense_keys,
                      &c->dense_counts, &c->bin_off, &c->misc, &c->tier_list, &c->mid, &c->sc_total, &c->gather_keys, &c->gather_counts,
                      &c->sp_base, &c->sp_keys, &c->sp_subs, &c->sp_par, &c->sp_fb, &c->mid_fb};
    for (DevBuf *b : bufs) release(*b);
    for (int i = 0; i < 2; ++i) {
        if (c->pinned[i]) (void)hipHostFree(c->pinned[i]);
        if (c->pin_ev[i]) (void)hipEventDestroy(c->pin_ev[i]);
    }
    if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
    delete c->comm;
    c->comm = nullptr;
    c->pin_up.release();
    c->pin_down.release();
    c->pin_tier.release();
    c->file_pin[0].release();
    c->file_pin[1].release();
    if (c->tier_ev) (void)hipEventDestroy(c->tier_ev);
    if (c->pin_up_ev) (void)hipEventDestroy(c->pin_up_ev);
    if (c->hold_flag) (void)hipHostFree(c->hold_flag);
    release(c->xsend);
    release(c->xrecv);
    for (auto &e : c->xev)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : c->seg_evs)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : c->map_evs)
        if (e) (void)hipEventDestroy(e);
    if (c->emit_ev) (void)hipEventDestroy(c->emit_ev);
    if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
    if (c->xstage) (void)hipStreamSynchronize(c->xstage), (void)hipStreamDestroy(c->xstage);
    if (c->xstage_ev) (void)hipEventDestroy(c->xstage_ev);
    if (c->ws_x.ptr) (void)hipFree(c->ws_x.ptr);
    c->dest.release_all();
    c->part.release_all();
    c->binhist.release_all();
    release(c->d_owner);
    release(c->d_local);
    if (c->ws.ptr) (void)hipFree(c->ws.ptr);
    for (auto &ev : c->ev)
        if (ev) (void)hipEventDestroy(ev);
    for (auto &ev : c->st_ev)
        if (ev) (void)hipEventDestroy(ev);
    for (int p = 0; p < STAGE_MAXP; ++p) release(c->st_keys[p]), release(c->st_cb[p]);
    release(c->st_total);
    release(c->piece_starts);
    if (c->seg_ev) (void)hipEventDestroy(c->seg_ev);
    for (auto &ev : c->h2d_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (c->tier_side) (void)hipStreamSynchronize(c->tier_side), (void)hipStreamDestroy(c->tier_side);
    for (auto &ev : c->side_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

FK_EXPORT int fk_set_stream(fk_ctx *c, void *s) {
    if (!c) return set_err(FK_E_INVALID, "null ctx");
    DeviceGuard dg_(c->device);
    if (c->own_stream && c->stream) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamDestroy(c->stream);
    }
    c->stream = (hipStream_t)s;
    c->own_stream = false;
    return FK_OK;
}

FK_EXPORT size_t fk_record_bytes(const fk_ctx *c) { return c ? (size_t)c->W * 8 : 0; }
FK_EXPORT int32_t fk_num_bins(const fk_ctx *c) { return c ? c->Bc : 0; }

static void reset_results(fk_ctx *c) {
    c->mapped = false;
    c->have_result = false;
    c->gapped = c->dense_ready = false;
    c->distinct = 0;
    c->h_bin_off.clear();
}

static float ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) {
        (void)hipGetLastError();
        return 0.f;
    }
    return ms;
}

constexpr size_t PIN_CHUNK = 32ull << 20;  // pinned staging buffer (x2) for pageable sources

// Grows b to at least `bytes`, keeping its first `keep` bytes (stream-ordered copy).
static int grow_keep(DevBuf &b, size_t bytes, size_t keep, hipStream_t s) {
    if (b.bytes >= bytes) return FK_OK;
    DevBuf g;
    FK_TRY(ensure(g, std::max<size_t>(bytes, 2 * b.bytes)));
    if (keep && b.p) HIP_TRY(hipMemcpyAsync(g.p, b.p, std::min(keep, b.bytes), hipMemcpyDeviceToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    release(b);
    b = g;
    return FK_OK;
}

static bool premap_eligible(const fk_ctx *c) {
    return c->fused && map_fused_supported(c->cfg.k, c->cfg.m, (uint32_t)c->Bc);
}

// Streamed map: launches the fused map over the tiles whose bytes (and halo)
// lie below `landed`; `final_` = the input ends at `landed` (every remaining
// tile, the last one sets the record total).  Runs on the map stream after
// the copy stream's segment event.
// The map of tiles [t0, t0 + nt) of the input fa[0, n): parse then signature passes in two kernels
// per MAP_VSLOT_TILES tiles (the parse's waves are latency-bound, the passes' VALU-bound; apart, each
// kernel's waves keep the SIMDs busy), or the fused kernel (FASTKMER_SPLIT_MAP=0, the 256-thread
// tiles, probes).  map_vslots is sized by the callers (map_vslots_reserve).
constexpr uint64_t MAP_VSLOT_TILES = 32768;  // ~1.07 GB of FASTA per split launch pair (140 MB of slots)
static bool map_split(const fk_ctx *c) { return c->split_map && !c->fused_probe; }
static int map_vslots_reserve(fk_ctx *c, uint64_t ntiles) {
    if (!map_split(c)) return FK_OK;
    return ensure(c->map_vslots, std::min(ntiles, MAP_VSLOT_TILES) * map_fused_vslot() * 4);
}
static int map_launch(fk_ctx *c, const uint8_t *fa, uint64_t n, int more, uint64_t t0, uint64_t nt, hipStream_t s) {
    const uint64_t cap = map_split(c) ? c->map_vslots.bytes / ((uint64_t)map_fused_vslot() * 4) : 0;
    for (uint64_t b = 0; b < nt;) {
        const uint64_t m = cap ? std::min(cap, nt - b) : nt - b;
        HIP_TRY(launch_map_fused(FUSED_NT, c->cfg.k, c->cfg.m, fa, n, more, t0 + b, m, c->fm,
                                 c->rec_hdr.as<uint32_t>(), c->rec_pos.as<uint16_t>(), c->rec_code.as<uint32_t>(),
                                 c->tcnt.as<uint32_t>(), c->tstat.as<uint32_t>(), c->counters.as<unsigned long long>(),
                                 s, c->fused_probe, cap ? c->map_vslots.as<uint32_t>() : nullptr));
        b += m;
    }
    return FK_OK;
}

static int premap_launch(fk_ctx *c, uint64_t landed, bool final_) {
    const uint64_t tile = fm_tile_bytes(FUSED_NT), span = fm_span_bytes(FUSED_NT);
    const uint64_t end = final_ ? (landed + tile - 1) / tile : (landed >= span ? (landed - span) / tile + 1 : 0);
    if (end <= c->pm_tiles) return FK_OK;
    if (c->tcnt.bytes < end * 4 || c->tstat.bytes < end * 8 || c->rec_hdr.bytes < end * map_fused_tcap() * 4 ||
        c->rec_pos.bytes < end * map_fused_tcap() * 2 || c->rec_code.bytes < end * map_fused_cslot() * 4)
        return set_err(FK_E_STATE, "streamed map: %llu tiles exceed the reserved record slots",
                       (unsigned long long)end);
    hipStream_t s = c->stream;
    if (c->pm_tiles == 0) HIP_TRY(hipEventRecord(c->ev[10], s));
    FK_TRY(map_launch(c, c->d_fasta, landed, final_ ? 0 : 1, c->pm_tiles, end - c->pm_tiles, s));
    c->pm_tiles = end;
    if (final_) HIP_TRY(hipEventRecord(c->ev[11], s));
    return FK_OK;
}

static int xch_maybe_piece(fk_ctx *c);
static int local_maybe_piece(fk_ctx *c, uint64_t tiles, hipEvent_t mapped);
static void xch_reset(fk_ctx *c);
static void pieces_reset(fk_ctx *c);

// Appends host bytes to the device input on the copy stream, in segments.
// Pinned sources are copied by DMA directly; pageable ones through two
// pinned staging buffers (the memcpy of one overlapping the DMA of the
// other).  With the fused map (k_map_fused) every tile whose bytes have
// landed is mapped on the map stream while the next segment is in flight,
// so the PCIe transfer hides the parse + signature work.  Returns once the
// source has been read (the caller's buffer is free); the map of the last
// segment may still be running.
static int comm_fail(fk_ctx *c, int rc);
static int note_held(fk_ctx *c, int rc);

static int ingest_impl(fk_ctx *c, const uint8_t *fasta, size_t n, int last) {
    if (!fasta && n) return set_err(FK_E_INVALID, "null argument");
    DeviceGuard dg_(c->device);
    if (c->d_fasta && c->d_fasta != c->fasta_own.as<uint8_t>()) {
        // a borrowed device input (fk_ingest_device): host chunks cannot be appended
        // to it, but a host ingest that starts a new job replaces it
        if (c->dev_open) return set_err(FK_E_STATE, "fk_ingest appending to an fk_ingest_device input");
        c->d_fasta = nullptr;
    }
    hipStream_t s = c->stream, cs = c->copy_stream;
    const bool fresh = c->ingest_fresh || !c->d_fasta;
    if (fresh) {
        c->n_fasta = 0;
        c->ingest_fresh = false;
        if (c->comm) {
            if (c->xch.open) return set_err(FK_E_STATE, "fk_ingest: the previous job's exchange is unfinished (fk_finish)");
            FK_TRY(comm_sync(c, c->comm_stream));
            xch_reset(c);
        }
        FK_TRY(comm_sync(c, c->xstage));
        HIP_TRY(hipStreamSynchronize(s));  // a previous job's work may still read the buffers
        pieces_reset(c);
        c->pm_active = premap_eligible(c);
        c->pm_tiles = 0;
        c->pm_last_seen = false;
    } else if (c->pm_last_seen) {
        c->pm_active = false;  // appending after the final tiles: fk_map maps the whole input
    }
    const uint64_t have = c->n_fasta, need = have + n;
    if (c->fasta_own.bytes < need) {  // grow, keeping what was ingested (and what the map reads)
        HIP_TRY(hipStreamSynchronize(cs));
        FK_TRY(grow_keep(c->fasta_own, need, have, s));
    }
    c->d_fasta = c->fasta_own.as<uint8_t>();
    if (c->pm_active) {
        // record slots and per-tile counts of every tile this input can hold (kept on growth)
        const uint64_t tiles = (need + fm_tile_bytes(FUSED_NT) - 1) / fm_tile_bytes(FUSED_NT) + 1;
        if (c->tcnt.bytes < tiles * 4) FK_TRY(grow_keep(c->tcnt, tiles * 4, c->tcnt.bytes, s));
        if (c->tstat.bytes < tiles * 8) FK_TRY(grow_keep(c->tstat, tiles * 8, c->tstat.bytes, s));
        const uint64_t hdr_need = tiles * map_fused_tcap() * 4, pos_need = tiles * map_fused_tcap() * 2;
        const uint64_t code_need = tiles * map_fused_cslot() * 4;
        if (c->rec_hdr.bytes < hdr_need) FK_TRY(grow_keep(c->rec_hdr, hdr_need, c->rec_hdr.bytes, s));
        if (c->rec_pos.bytes < pos_need) FK_TRY(grow_keep(c->rec_pos, pos_need, c->rec_pos.bytes, s));
        if (c->rec_code.bytes < code_need) FK_TRY(grow_keep(c->rec_code, code_need, c->rec_code.bytes, s));
        FK_TRY(map_vslots_reserve(c, tiles));
        if (fresh) {
            FK_TRY(ensure(c->counters, 64));
            HIP_TRY(hipMemsetAsync(c->counters.p, 0, 64, s));
        }
    }
    uint8_t *dst = c->fasta_own.as<uint8_t>() + have;
    hipPointerAttribute_t attr{};
    const bool pinned = hipPointerGetAttributes(&attr, fasta) == hipSuccess && attr.type == hipMemoryTypeHost;
    (void)hipGetLastError();
    if (!pinned && n)
        for (int i = 0; i < 2; ++i)
            if (!c->pinned[i]) {
                HIP_TRY(hipHostMalloc(&c->pinned[i], PIN_CHUNK, hipHostMallocDefault));
                HIP_TRY(hipEventCreateWithFlags(&c->pin_ev[i], hipEventDisableTiming));
                HIP_TRY(hipEventRecord(c->pin_ev[i], cs));
            }
    // with a communicator, every piece of mapped tiles is exchanged while later ones land
    const bool pieces = c->comm && c->pm_active;
    // the job's size: this call's when it holds the whole input, else what fk_ingest_reserve announced
    if (pieces && fresh) {
        c->xch.expect_bytes = last ? n : c->reserve_bytes;
        // a job of known size goes out in about XCH_STEPS steps (at most 1 GB, at least XCH_MIN each):
        // every step but the last moves while later bytes are copied in (one 1 GB step for a 1 GB job
        // would leave the whole exchange after the last byte), and the staging cuts (st_cuts) fall on
        // step ends (1 GB steps of a 6.25 GB job staged 5-6 GB after the last byte: 11 ms of expansion
        // in the tail, profiles/r05d_xch1_c3_tail.txt)
        constexpr uint64_t XCH_STEPS = 10;
#ifndef FK_XCH_MIN_MB
#define FK_XCH_MIN_MB 64  // 1 GB job: ten steps (A/B builds: 128, seven steps)
#endif
        constexpr uint64_t XCH_MIN = (uint64_t)FK_XCH_MIN_MB << 20;
        if (!c->piece_bytes_set)
            c->piece_bytes = c->xch.expect_bytes
                                 ? std::min<uint64_t>(1ull << 30, std::max<uint64_t>(XCH_MIN, c->xch.expect_bytes / XCH_STEPS))
                                 : 1ull << 30;
    }
    if (fresh) {
        c->job_bytes = last ? n : c->reserve_bytes;
        c->reserve_bytes = 0;
    }
    HIP_TRY(hipEventRecord(c->h2d_ev[0], cs));
    if (pinned) {
        // every segment's copy is queued first, so the DMA runs back to back even while the
        // host waits on a piece's exchange.  Each copy boundary costs ~11 us of link time
        // (profiles/r05s_h2d_rates.txt): up to the call's last tenth (at least four small
        // segments) the segments grow to a sixteenth of the call in whole ingest_segs, at most four
        // (1 GB: 64 MB, 6.25 GB: 128 MB; configs[1] 22.70 -> 22.56 ms, profiles/r05z_xch_cuts_seg_ab.txt),
        // with a communicator at most a quarter of an exchange step; ingest_seg in that last tenth, so
        // that what follows the last byte (the last segment's map, the last piece) stays short
        const size_t seg = c->ingest_seg;
        size_t big = seg * std::clamp<size_t>((n / 16 + seg / 2) / seg, 1, 4);
        if (pieces) big = std::min(big, std::max(seg, (size_t)c->piece_bytes / 4 / seg * seg));
        const size_t nseg = (n + seg - 1) / seg;
        const size_t small_from = n - std::min(n, std::max<size_t>(n / 10, 4 * seg));
        auto seg_len = [&](size_t off) { return std::min(off < small_from ? big : seg, n - off); };
        while (c->pm_active && c->seg_evs.size() < nseg) {
            hipEvent_t e = nullptr;
            HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            c->seg_evs.push_back(e);
        }
        size_t off = 0;
        for (size_t i = 0; off < n; ++i) {
            const size_t len = seg_len(off);
            HIP_TRY(hipMemcpyAsync(dst + off, fasta + off, len, hipMemcpyHostToDevice, cs));
            if (c->pm_active) HIP_TRY(hipEventRecord(c->seg_evs[i], cs));
            off += len;
        }
        HIP_TRY(hipEventRecord(c->h2d_ev[1], cs));
        // every segment's map is queued too (one rank; the exchange steps wait on the host between
        // them), then the pieces are staged on the staging stream behind the map of their last
        // segment: the host's waits for a piece's partition never hold back a later map launch
        while (!pieces && c->pm_active && c->map_evs.size() < nseg) {
            hipEvent_t e = nullptr;
            HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            c->map_evs.push_back(e);
        }
        c->seg_tiles.clear();
        off = 0;
        for (size_t i = 0; c->pm_active && off < n; ++i) {
            off += seg_len(off);
            HIP_TRY(hipStreamWaitEvent(s, c->seg_evs[i], 0));
            FK_TRY(premap_launch(c, have + off, last && off == n));
            if (pieces) {
                FK_TRY(xch_maybe_piece(c));
            } else {
                HIP_TRY(hipEventRecord(c->map_evs[i], s));
                c->seg_tiles.push_back(c->pm_tiles);
            }
        }
        for (size_t i = 0; !pieces && c->pm_active && i < c->seg_tiles.size(); ++i)
            FK_TRY(local_maybe_piece(c, c->seg_tiles[i], c->map_evs[i]));
    } else {
        size_t off = 0;
        for (int i = 0; off < n; ++i) {
            const size_t len = std::min(PIN_CHUNK, n - off);
            HIP_TRY(hipEventSynchronize(c->pin_ev[i & 1]));  // its previous DMA is done
            memcpy(c->pinned[i & 1], fasta + off, len);
            HIP_TRY(hipMemcpyAsync(dst + off, c->pinned[i & 1], len, hipMemcpyHostToDevice, cs));
            HIP_TRY(hipEventRecord(c->pin_ev[i & 1], cs));
            off += len;
            if (c->pm_active) {
                HIP_TRY(hipEventRecord(c->seg_ev, cs));
                HIP_TRY(hipStreamWaitEvent(s, c->seg_ev, 0));
                FK_TRY(premap_launch(c, have + off, last && off == n));
                if (pieces) {
                    FK_TRY(xch_maybe_piece(c));
                } else {
                    HIP_TRY(hipEventRecord(c->seg_ev, s));  // reused: the staging stream waits on it at once
                    FK_TRY(local_maybe_piece(c, c->pm_tiles, c->seg_ev));
                }
            }
        }
        HIP_TRY(hipEventRecord(c->h2d_ev[1], cs));
    }
    if (c->pm_active && last) {
        c->pm_last_seen = true;
        if (n == 0) FK_TRY(premap_launch(c, need, true));
    }
    HIP_TRY(hipStreamSynchronize(cs));  // the source has been read
    c->ms_h2d = ev_ms(c->h2d_ev[0], c->h2d_ev[1]);
    c->n_fasta = need;
    reset_results(c);
    return FK_OK;
}

// fk_ingest is collective with a communicator (pieces are exchanged while the input lands): any
// error on this rank aborts the group, so peers blocked in a step return instead of waiting.
FK_EXPORT int fk_ingest(fk_ctx *c, const uint8_t *fasta, size_t n, int last) {
    if (!c) return set_err(FK_E_INVALID, "null ctx");
    const int rc = ingest_impl(c, fasta, n, last);
    return rc && c->comm ? comm_fail(c, rc) : note_held(c, rc);
}

static int reserve_impl(fk_ctx *c, uint64_t total_bytes);

FK_EXPORT int fk_ingest_reserve(fk_ctx *c, uint64_t total_bytes) {
    if (!c) return set_err(FK_E_INVALID, "null ctx");
    return reserve_impl(c, total_bytes);
}

static int reserve_impl(fk_ctx *c, uint64_t total_bytes) {
    DeviceGuard dg_(c->device);
    if (!c->ingest_fresh && c->d_fasta) return set_err(FK_E_STATE, "fk_ingest_reserve inside a streamed input");
    FK_TRY(ensure(c->fasta_own, total_bytes));
    c->reserve_bytes = total_bytes;  // the next (streamed) job's size: piece cuts and staged plans follow it
    if (premap_eligible(c)) {
        const uint64_t tiles = (total_bytes + fm_tile_bytes(FUSED_NT) - 1) / fm_tile_bytes(FUSED_NT) + 1;
        FK_TRY(ensure(c->rec_hdr, tiles * map_fused_tcap() * 4));
        FK_TRY(ensure(c->rec_pos, tiles * map_fused_tcap() * 2));
        FK_TRY(ensure(c->rec_code, tiles * map_fused_cslot() * 4));
        FK_TRY(ensure(c->tcnt, tiles * 4));
        FK_TRY(ensure(c->tstat, tiles * 8));
    }
    return FK_OK;
}

// ---- a rank's split of a FASTA file (fk_split.cpp)

namespace {
struct Fd {
    int fd = -1;
    ~Fd() {
        if (fd >= 0) close(fd);
    }
};
int open_split(const char *path, int32_t world, int32_t rank, int32_t k, int32_t seq, Fd &f, uint64_t &size,
               SplitPlan &plan) {
    f.fd = open(path, O_RDONLY | O_CLOEXEC);
    if (f.fd < 0) return set_err(FK_E_IO, "open(%s): %s", path, strerror(errno));
    struct stat st {};
    if (fstat(f.fd, &st) != 0) return set_err(FK_E_IO, "fstat(%s): %s", path, strerror(errno));
    size = (uint64_t)st.st_size;
    std::string err;
    if (seq != 0 && seq != 1) return set_err(FK_E_INVALID, "sequence_type must be 0 or 1");
    if (plan_split(f.fd, size, world, rank, k, seq, plan, err))
        return set_err(world < 1 || rank < 0 || rank >= world || k < 1 ? FK_E_INVALID : FK_E_IO, "%s: %s", path,
                       err.c_str());
    return FK_OK;
}
}  // namespace

FK_EXPORT int fk_split_bytes(const char *path, int32_t world, int32_t rank, int32_t k, int32_t sequence_type,
                             uint8_t *out, size_t cap, size_t *n) {
    if (!path || !n) return set_err(FK_E_INVALID, "null argument");
    Fd f;
    uint64_t size = 0;
    SplitPlan plan;
    FK_TRY(open_split(path, world, rank, k, sequence_type, f, size, plan));
    *n = (size_t)plan.total;
    if (!out) return FK_OK;
    if (cap < plan.total) return set_err(FK_E_RANGE, "split of %llu bytes, buffer holds %zu", (unsigned long long)plan.total, cap);
    std::string err;
    if (read_split(f.fd, size, plan, 0, plan.total, out, err)) return set_err(FK_E_IO, "%s: %s", path, err.c_str());
    return FK_OK;
}

// With a communicator the split is the job's: (world, rank) must be the context's own (a mismatch
// would count some byte ranges twice and skip others while the exchange still completes).
static int check_split_rank(const fk_ctx *c, int32_t world, int32_t rank, const char *what) {
    if (c->comm && (world != (int32_t)c->G || rank != c->cfg.rank))
        return set_err(FK_E_INVALID, "%s: split %d of %d on the context of rank %d of %u", what, rank, world,
                       c->cfg.rank, c->G);
    return FK_OK;
}

static int ingest_file_impl(fk_ctx *c, const char *path, int32_t world, int32_t rank, uint64_t window) {
    if (!path) return set_err(FK_E_INVALID, "null path");
    FK_TRY(check_split_rank(c, world, rank, "fk_ingest_file_range"));
    if (!c->ingest_fresh && c->d_fasta) return set_err(FK_E_STATE, "fk_ingest_file_range inside a streamed input");
    Fd f;
    uint64_t size = 0;
    SplitPlan plan;
    FK_TRY(open_split(path, world, rank, c->cfg.k, c->cfg.sequence_type, f, size, plan));
    const uint64_t total = plan.total;
    if (total == 0) return ingest_impl(c, nullptr, 0, 1);
    if (!window) window = 256ull << 20;
    window = std::max<uint64_t>(window, 1ull << 20);
    const uint64_t win = std::min(window, total);
    for (int i = 0; i < 2 && i * win < total; ++i)
        if (c->file_pin[i].ensure(win)) return set_err(FK_E_NOMEM, "hipHostMalloc(%llu) failed", (unsigned long long)win);
    FK_TRY(reserve_impl(c, total));
    std::string rerr;
    int rrc = read_split(f.fd, size, plan, 0, win, c->file_pin[0].as<uint8_t>(), rerr);
    if (rrc) return set_err(FK_E_IO, "%s: %s", path, rerr.c_str());
    int b = 0;
    for (uint64_t pos = 0; pos < total;) {
        const uint64_t len = std::min(win, total - pos), next = std::min(win, total - pos - len);
        // the next window is read while this one is copied and mapped
        std::thread reader;
        if (next)
            reader = std::thread([&, b, pos, len, next] {
                rrc = read_split(f.fd, size, plan, pos + len, next, c->file_pin[b ^ 1].as<uint8_t>(), rerr);
            });
        const int rc = ingest_impl(c, c->file_pin[b].as<uint8_t>(), len, pos + len == total ? 1 : 0);
        if (reader.joinable()) reader.join();
        if (rc) return rc;
        if (rrc) return set_err(FK_E_IO, "%s: %s", path, rerr.c_str());
        pos += len;
        b ^= 1;
    }
    return FK_OK;
}

FK_EXPORT int fk_ingest_file_range(fk_ctx *c, const char *path, int32_t world, int32_t rank, uint64_t window_bytes) {
    if (!c) return set_err(FK_E_INVALID, "null ctx");
    const int rc = ingest_file_impl(c, path, world, rank, window_bytes);
    return rc && c->comm ? comm_fail(c, rc) : rc;
}

static int ingest_device_impl(fk_ctx *c, const void *d, size_t n, int last);

FK_EXPORT int fk_ingest_device(fk_ctx *c, const void *d, size_t n, int last) {
    if (!c) return set_err(FK_E_INVALID, "null ctx");
    const int rc = ingest_device_impl(c, d, n, last);
    return rc && c->comm ? comm_fail(c, rc) : rc;
}

static int ingest_device_impl(fk_ctx *c, const void *d, size_t n, int last) {
    if (!d && n) return set_err(FK_E_INVALID, "null argument");
    DeviceGuard dg_(c->device);
    if (c->comm && c->xch.open) return set_err(FK_E_STATE, "fk_ingest_device: the previous job's exchange is unfinished");
    if (c->comm) xch_reset(c);
    c->dev_open = last == 0;  // a borrowed input takes no appended host chunks
    c->ingest_fresh = true;
    c->pm_active = false;
    pieces_reset(c);
    reset_results(c);
    if (((uintptr_t)d & 15) != 0) {
        FK_TRY(ensure(c->fasta_own, n));
        HIP_TRY(hipMemcpyAsync(c->fasta_own.p, d, n, hipMemcpyDeviceToDevice, c->stream));
        c->d_fasta = c->fasta_own.as<uint8_t>();
    } else {
        c->d_fasta = (const uint8_t *)d;
    }
    c->n_fasta = n;
    return FK_OK;
}

FK_EXPORT int fk_synth_fasta_to_device(void *d_out, uint64_t first_read, uint64_t n_reads, int32_t read_len,
                                       uint64_t genome_len, uint64_t seed, double err_rate, double n_rate) {
    if ((!d_out && n_reads) || read_len < 1 || genome_len < 1) return set_err(FK_E_INVALID, "bad synth arguments");
    const SynthParams p = make_synth(first_read, n_reads, read_len, genome_len, seed, err_rate, n_rate);
    const uint64_t nb = n_reads * p.rec_bytes;
    if (nb) HIP_TRY(launch_synth((uint8_t *)d_out, nb, p, nullptr));
    HIP_TRY(hipDeviceSynchronize());
    return FK_OK;
}

FK_EXPORT int fk_synth_fasta_device(fk_ctx *c, uint64_t first_read, uint64_t n_reads, int32_t read_len,
                                    uint64_t genome_len, uint64_t seed, double err_rate, double n_rate) {
    if (!c || read_len < 1 || genome_len < 1) return set_err(FK_E_INVALID, "bad synth arguments");
    DeviceGuard dg_(c->device);
    const SynthParams p = make_synth(first_read, n_reads, read_len, genome_len, seed, err_rate, n_rate);
    const uint64_t nb = n_reads * p.rec_bytes;
    FK_TRY(ensure(c->fasta_own, nb));
    if (c->comm && c->xch.open) return set_err(FK_E_STATE, "fk_synth_fasta_device: the previous job's exchange is unfinished");
    if (c->comm) xch_reset(c);
    HIP_TRY(launch_synth(c->fasta_own.as<uint8_t>(), nb, p, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->dev_open = false;
    c->ingest_fresh = true;
    c->pm_active = false;
    pieces_reset(c);
    c->d_fasta = c->fasta_own.as<uint8_t>();
    c->n_fasta = nb;
    reset_results(c);
    return FK_OK;
}

// ---------------------------------------------------------------------------
// map side: parse + encode + signature + records (+ destination histogram)
// ---------------------------------------------------------------------------


static const uint32_t *owner_table(const fk_ctx *c) { return c->custom_owners ? c->d_owner.as<uint32_t>() : nullptr; }
static const uint32_t *local_table(const fk_ctx *c) { return c->custom_owners ? c->d_local.as<uint32_t>() : nullptr; }
static int32_t global_bin(const fk_ctx *c, uint32_t lb) {
    return c->custom_owners ? c->h_lbin_bin[lb] : (int32_t)(c->cfg.rank + lb * c->G);
}

// Fused parse + signature (k_map_fused): FASTA bytes to records in one kernel.
// *ok = false when a tile raised the fallback flag (the caller then maps with
// the two-kernel path, which places every input).
static int map_fused(fk_ctx *c, uint64_t n, bool *ok) {
    hipStream_t s = c->stream;
    *ok = false;
    const uint64_t tile = fm_tile_bytes(FUSED_NT);
    const uint64_t ntiles = (n + tile - 1) / tile;
    FK_TRY(ensure(c->tcnt, ntiles * 4));
    FK_TRY(ensure(c->tstat, ntiles * 8));
    FK_TRY(ensure(c->counters, 64));
    FK_TRY(ensure(c->rec_hdr, ntiles * map_fused_tcap() * 4));
    FK_TRY(ensure(c->rec_pos, ntiles * map_fused_tcap() * 2));
    FK_TRY(ensure(c->rec_code, ntiles * map_fused_cslot() * 4));
    FK_TRY(map_vslots_reserve(c, ntiles));
    HIP_TRY(hipEventRecord(c->ev[2], s));
    HIP_TRY(hipMemsetAsync(c->counters.p, 0, 64, s));
    HIP_TRY(hipEventRecord(c->ev[10], s));
    FK_TRY(map_launch(c, c->d_fasta, n, 0, 0, ntiles, s));
    HIP_TRY(hipEventRecord(c->ev[11], s));
    HIP_TRY(launch_tile_totals(c->tcnt.as<uint32_t>(), c->tstat.as<uint32_t>(), ntiles,
                               c->counters.as<unsigned long long>(), s));
    HIP_TRY(hipEventRecord(c->ev[3], s));
    uint64_t h[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(h, c->counters.p, 32, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    c->stats.fused_fallback = h[2];
    if (h[2]) return FK_OK;  // fallback
    c->nrec = h[0];
    c->nkmers = h[1];
    c->stats.positions = h[3];
    c->rec_tiled = true;
    c->rec_tiles = ntiles;
    *ok = true;
    c->stats.ms_parse = 0.0;
    c->stats.ms_signature = ev_ms(c->ev[2], c->ev[3]);
    c->stats.ms_encode_kernel = 0.0;
    c->stats.ms_signature_kernel = ev_ms(c->ev[10], c->ev[11]);
    return FK_OK;
}

// the fused map's tiles [t0, t0 + nt) as a partition source (nrec: their records, or a bound)
static RecSrc fused_src(const fk_ctx *c, uint64_t t0, uint64_t nt, uint64_t nrec) {
    const uint64_t tcap = map_fused_tcap(), cslot = map_fused_cslot();
    return tiled_src(c->rec_hdr.as<uint32_t>() + t0 * tcap, c->rec_pos.as<uint16_t>() + t0 * tcap,
                     c->rec_code.as<uint32_t>() + t0 * cslot, c->tcnt.as<uint32_t>() + t0, nrec, nt, (uint32_t)tcap,
                     (uint32_t)cslot, c->W, c->cfg.k);
}

// the records of the last fk_map as a partition source
static RecSrc map_src(const fk_ctx *c) {
    if (c->rec_tiled) return fused_src(c, 0, c->rec_tiles, c->nrec);
    return dense_src(c->records.as<uint64_t>(), c->nrec, c->W);
}

// fk_map steps 0-2: the input's super-k-mer records (fused kernel, or parse + signature)
static int map_records(fk_ctx *c) {
    const double t_start = now_ms();
    hipStream_t s = c->stream;
    c->ingest_fresh = true;  // a later fk_ingest starts a new input
    c->dev_open = false;
    const uint64_t n = c->d_fasta ? c->n_fasta : 0;
    reset_results(c);
    c->stats = fk_stats{};
    c->stats.fasta_bytes = n;
    c->nrec = c->nkmers = 0;
    c->rec_tiled = false;

    // 0. fused parse + signature (streamed by fk_ingest, or one launch here); the
    // two-kernel path below maps the inputs the fused kernel hands back
    bool fused_ok = false;
    c->stats.ms_h2d = c->ms_h2d;
    if (c->pm_active && n) {
        // streamed map (fk_ingest launched the tiles as their bytes landed)
        if (!c->pm_last_seen) FK_TRY(premap_launch(c, n, true));  // the input ends here
        HIP_TRY(launch_tile_totals(c->tcnt.as<uint32_t>(), c->tstat.as<uint32_t>(), c->pm_tiles,
                                   c->counters.as<unsigned long long>(), s));
        uint64_t h[4] = {0, 0, 0, 0};
        HIP_TRY(hipMemcpyAsync(h, c->counters.p, 32, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        c->stats.fused_fallback = h[2];
        if (!h[2]) {
            fused_ok = true;
            c->rec_tiled = true;
            c->rec_tiles = c->pm_tiles;
            c->nrec = h[0];
            c->nkmers = h[1];
            c->stats.positions = h[3];
            c->stats.ms_parse = 0.0;
            // map stream from the first to the last launch, waits for the landing segments included
            c->stats.ms_signature = ev_ms(c->ev[10], c->ev[11]);
            c->stats.ms_signature_kernel = c->stats.ms_signature;
        }
        c->pm_active = false;
    } else if (c->fused && n && map_fused_supported(c->cfg.k, c->cfg.m, (uint32_t)c->Bc)) {
        FK_TRY(map_fused(c, n, &fused_ok));
    }
    c->pm_active = false;

    const uint64_t ntiles = (n + ENC_TILE - 1) / ENC_TILE;
    const uint64_t code_words = n / 16 + 2 * POS_PAD_WORDS + 512;
    const uint64_t valid_words = n / 32 + 2 * POS_PAD_WORDS + 512;
    const uint64_t sig_tiles = (n + SIG_TILE - 1) / SIG_TILE + 1;
    if (!fused_ok) {
        FK_TRY(ensure(c->tile_last_nl, ntiles * 8));  // look-back status: newline / header state
        FK_TRY(ensure(c->tile_off, ntiles * 8));      // look-back status: output positions
        FK_TRY(ensure(c->npos_dev, 16));  // [0] positions, [1] "rerun the parse with the look-back"
        FK_TRY(ensure(c->codes, code_words * 4));
        FK_TRY(ensure(c->valid, valid_words * 4));
        FK_TRY(ensure(c->counters, 64));
        FK_TRY(ensure(c->sig_status, sig_tiles * 8));
        FK_TRY(ensure(c->sig_kmers, sig_tiles * 8));
    }

    // 1. FASTA parse + 2-bit encode.  The scan variant flags inputs it cannot
    // place (a line longer than its read-back, text before the first header);
    // the flag is read with the record count below and the parse is redone
    // with the line look-back.
    auto run_parse = [&](bool scan) -> int {
        HIP_TRY(hipEventRecord(c->ev[0], s));
        HIP_TRY(hipMemsetAsync(c->codes.p, 0, code_words * 4, s));
        HIP_TRY(hipMemsetAsync(c->valid.p, 0, valid_words * 4, s));
        HIP_TRY(hipMemsetAsync(c->npos_dev.p, 0, 16, s));
        if (n) {
            if (!scan) HIP_TRY(hipMemsetAsync(c->tile_last_nl.p, 0, ntiles * 8, s));
            HIP_TRY(hipMemsetAsync(c->tile_off.p, 0, ntiles * 8, s));
            HIP_TRY(hipEventRecord(c->ev[8], s));
            HIP_TRY(launch_fasta_parse(scan, c->d_fasta, n, c->tile_last_nl.as<uint64_t>(), c->tile_off.as<uint64_t>(),
                                       c->codes.as<uint32_t>(), c->valid.as<uint32_t>(), c->npos_dev.as<uint64_t>(),
                                       s));
            HIP_TRY(hipEventRecord(c->ev[9], s));
        }
        HIP_TRY(hipEventRecord(c->ev[1], s));
        return FK_OK;
    };
    c->last_map_fused = fused_ok;
    c->stats.fused_map = fused_ok ? 1 : 0;
    bool parse_scan = true;  // the scan variant first; the look-back rerun if it flags the input
    if (!fused_ok) FK_TRY(run_parse(parse_scan));

    // 2. signature + super-k-mer records (retried once if the capacity estimate was short)
    uint64_t rec_cap = std::max<uint64_t>(n / 6, 4096);
    for (int attempt = 0; attempt < 2 && !fused_ok; ++attempt) {
        FK_TRY(ensure(c->records, rec_cap * c->W * 8));
        rec_cap = c->records.bytes / (c->W * 8);
        HIP_TRY(hipMemsetAsync(c->counters.p, 0, 64, s));
        HIP_TRY(hipEventRecord(c->ev[2], s));
        HIP_TRY(hipMemsetAsync(c->sig_status.p, 0, sig_tiles * 8, s));
        HIP_TRY(hipMemsetAsync(c->sig_kmers.p, 0, sig_tiles * 8, s));
        HIP_TRY(hipEventRecord(c->ev[10], s));
        HIP_TRY(launch_superkmers(c->W, c->codes.as<uint32_t>(), c->valid.as<uint32_t>(), n,
                                  c->npos_dev.as<uint64_t>(), c->cfg.k, c->cfg.m, c->fm, c->records.as<uint64_t>(),
                                  rec_cap, c->sig_status.as<uint64_t>(), c->sig_kmers.as<uint64_t>(),
                                  c->counters.as<unsigned long long>(), s));
        HIP_TRY(hipEventRecord(c->ev[11], s));
        // total k-mers = sum of the per-tile counts (into counters[1])
        HIP_TRY(scan_excl_sum_u64(c->sig_kmers.as<uint64_t>(), c->sig_status.as<uint64_t>(), sig_tiles,
                                  c->counters.as<uint64_t>() + 1, c->ws, s));
        HIP_TRY(hipEventRecord(c->ev[3], s));
        uint64_t h[2], redo = 0;
        HIP_TRY(hipMemcpyAsync(h, c->counters.p, 16, hipMemcpyDeviceToHost, s));
        if (parse_scan) HIP_TRY(hipMemcpyAsync(&redo, c->npos_dev.as<uint64_t>() + 1, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (redo) {
            parse_scan = false;
            FK_TRY(run_parse(false));
            --attempt;
            continue;
        }
        c->nrec = h[0];
        c->nkmers = h[1];
        if (c->nrec <= rec_cap) break;
        rec_cap = c->nrec;
    }
    if (!fused_ok) {
        uint64_t npos = 0;
        HIP_TRY(hipMemcpy(&npos, c->npos_dev.p, 8, hipMemcpyDeviceToHost));
        c->stats.positions = npos;
        c->stats.ms_parse = ev_ms(c->ev[0], c->ev[1]);
        c->stats.ms_signature = ev_ms(c->ev[2], c->ev[3]);
        c->stats.ms_encode_kernel = n ? ev_ms(c->ev[8], c->ev[9]) : 0.0;
        c->stats.ms_signature_kernel = ev_ms(c->ev[10], c->ev[11]);
    }
    c->stats.kmers = c->nkmers;
    c->stats.superkmers = c->nrec;
    c->stats.ms_total += now_ms() - t_start;
    return FK_OK;
}

// Grouped emit: records and k-mers of the mapped records per (destination, local bin) part and the
// send counts per destination, under the current group table (the receiver needs no partition pass).
static int grouped_part_counts(fk_ctx *c) {
    hipStream_t s = c->stream;
    const uint32_t nparts = c->G * c->grp_nlb;
    c->grp_rec.assign(nparts, 0);
    c->grp_kmer.assign(nparts, 0);
    c->send_counts.assign(c->G, 0);
    if (c->nrec) {
        FK_TRY(part_count(c->dest, map_src(c), 0, c->G, c->grp_table.as<uint32_t>(), nparts, c->ws, s));
        HIP_TRY(hipMemcpyAsync(c->grp_rec.data(), c->dest.rec.p, (uint64_t)nparts * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(c->grp_kmer.data(), c->dest.kmer.p, (uint64_t)nparts * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    for (uint32_t d = 0; d < c->G; ++d)
        for (uint32_t lb = 0; lb < c->grp_nlb; ++lb) c->send_counts[d] += c->grp_rec[(uint64_t)d * c->grp_nlb + lb];
    return FK_OK;
}

static int build_group_table(fk_ctx *c);

FK_EXPORT int fk_map(fk_ctx *c, uint64_t *send_counts) {
    if (!c) return set_err(FK_E_INVALID, "null ctx");
    DeviceGuard dg_(c->device);
    // one rank: the pieces staged during fk_ingest read the mapped tiles on the staging stream
    if (c->st_np && !c->comm) HIP_TRY(hipStreamWaitEvent(c->stream, c->xstage_ev, 0));
    FK_TRY(map_records(c));
    const double t_start = now_ms();
    hipStream_t s = c->stream;

    // 3a. destination histogram (records per rank)
    c->send_counts.assign(c->G, 0);
    if (c->grouped) {
        FK_TRY(grouped_part_counts(c));
    } else if (c->G == 1) {
        c->send_counts[0] = c->nrec;
    } else if (c->nrec) {
        FK_TRY(part_count(c->dest, map_src(c), 0, c->G, owner_table(c), c->G, c->ws, s));
        HIP_TRY(hipMemcpyAsync(c->send_counts.data(), c->dest.rec.p, c->G * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    if (send_counts)
        for (uint32_t r = 0; r < c->G; ++r) send_counts[r] = c->send_counts[r];
    c->mapped = true;
    c->stats.ms_total += now_ms() - t_start;
    return FK_OK;
}

FK_EXPORT int fk_map_emit(fk_ctx *c, void *d_send, uint64_t cap_records) {
    if (!c) return set_err(FK_E_INVALID, "null ctx");
    DeviceGuard dg_(c->device);
    if (!c->mapped) return set_err(FK_E_STATE, "fk_map_emit before fk_map");
    if (cap_records < c->nrec) return set_err(FK_E_RANGE, "send buffer holds %llu records, need %llu",
                                              (unsigned long long)cap_records, (unsigned long long)c->nrec);
    if (!c->nrec) return FK_OK;
    const double t0 = now_ms();
    hipStream_t s = c->stream;
    if (c->grouped) {
        FK_TRY(part_scatter(c->dest, 0, c->G, c->grp_table.as<uint32_t>(), (uint64_t *)d_send, s));
    } else if (c->G == 1 && !c->rec_tiled) {
        HIP_TRY(hipMemcpyAsync(d_send, c->records.p, c->nrec * c->W * 8, hipMemcpyDeviceToDevice, s));
    } else if (c->G == 1) {  // the fused map's tiles, made dense
        FK_TRY(part_count(c->dest, map_src(c), 0, 1, nullptr, 1, c->ws, s));
        FK_TRY(part_scatter(c->dest, 0, 1, nullptr, (uint64_t *)d_send, s));
    } else {
        FK_TRY(part_scatter(c->dest, 0, c->G, owner_table(c), (uint64_t *)d_send, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    c->stats.ms_total += now_ms() - t0;
    return FK_OK;
}

// ---------------------------------------------------------------------------
// size-aware placement (MultiprocessorSchedulingPartitioner, SBKC:1023-1025)
// ---------------------------------------------------------------------------

FK_EXPORT int fk_map_bin_kmers(fk_ctx *c, uint64_t *kmers_per_bin) {
    if (!c || !kmers_per_bin) return set_err(FK_E_INVALID, "null argument");
    DeviceGuard dg_(c->device);
    if (!c->mapped) return set_err(FK_E_STATE, "fk_map_bin_kmers before fk_map");
    hipStream_t s = c->stream;
    FK_TRY(part_count(c->binhist, map_src(c), 1, 1, nullptr, (uint32_t)c->Bc, c->ws, s));
    HIP_TRY(hipMemcpyAsync(kmers_per_bin, c->binhist.kmer.p, (uint64_t)c->Bc * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return FK_OK;
}

FK_EXPORT int fk_lpt_owners(const uint64_t *sizes, int32_t nbins, int32_t nranks, int32_t *owner) {
    if (!sizes || !owner || nbins < 0 || nranks < 1) return set_err(FK_E_INVALID, "bad argument");
    // largest first onto the least loaded rank (ties: lowest bin, lowest rank); bins of
    // size 0 were not seen by the estimate and keep the hash placement bin % nranks
    std::vector<int32_t> order;
    for (int32_t b = 0; b < nbins; ++b) {
        if (sizes[b])
            order.push_back(b);
        else
            owner[b] = b % nranks;
    }
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return sizes[a] > sizes[b]; });
    std::vector<uint64_t> load(nranks, 0);
    for (int32_t b : order) {
        int32_t r = 0;
        for (int32_t q = 1; q < nranks; ++q)
            if (load[q] < load[r]) r = q;
        owner[b] = r;
        load[r] += sizes[b];
    }
    return FK_OK;
}

FK_EXPORT int fk_set_bin_owners(fk_ctx *c, const int32_t *owner, uint64_t *send_counts) {
    if (!c || !owner) return set_err(FK_E_INVALID, "null argument");
    DeviceGuard dg_(c->device);
    if (c->comm && c->xch.open) return set_err(FK_E_STATE, "fk_set_bin_owners inside a job's exchange");
    for (int32_t b = 0; b < c->Bc; ++b)
        if (owner[b] < 0 || (uint32_t)owner[b] >= c->G)
            return set_err(FK_E_INVALID, "owner[%d] = %d is not a rank of %u", b, owner[b], c->G);
    hipStream_t s = c->stream;
    c->h_owner.assign(owner, owner + c->Bc);
    c->h_bin_lbin.assign(c->Bc, ~0u);
    c->h_lbin_bin.clear();
    for (int32_t b = 0; b < c->Bc; ++b)
        if (owner[b] == c->cfg.rank) {
            c->h_bin_lbin[b] = (uint32_t)c->h_lbin_bin.size();
            c->h_lbin_bin.push_back(b);
        }
    c->nlb = (uint32_t)c->h_lbin_bin.size();
    // device maps over every value the 22-bit record bin field can hold
    const uint64_t ntab = (uint64_t)REC_BIN_MASK + 1;
    FK_TRY(ensure(c->d_owner, ntab * 4));
    FK_TRY(ensure(c->d_local, ntab * 4));
    HIP_TRY(hipMemsetAsync(c->d_owner.p, 0xff, ntab * 4, s));
    HIP_TRY(hipMemsetAsync(c->d_local.p, 0xff, ntab * 4, s));
    HIP_TRY(hipMemcpyAsync(c->d_owner.p, c->h_owner.data(), (uint64_t)c->Bc * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->d_local.p, c->h_bin_lbin.data(), (uint64_t)c->Bc * 4, hipMemcpyHostToDevice, s));
    c->custom_owners = true;
    c->have_result = false;
    if (c->grouped) {  // the (owner, local bin) parts of the grouped emit follow the new owners
        FK_TRY(build_group_table(c));
        if (c->mapped) FK_TRY(grouped_part_counts(c));  // ... and so do the mapped records' parts
    } else if (c->mapped) {  // the destinations of the mapped records changed
        c->send_counts.assign(c->G, 0);
        if (c->G == 1) {
            c->send_counts[0] = c->nrec;
        } else if (c->nrec) {
            FK_TRY(part_count(c->dest, map_src(c), 0, c->G, owner_table(c), c->G, c->ws, s));
            HIP_TRY(hipMemcpyAsync(c->send_counts.data(), c->dest.rec.p, c->G * 8, hipMemcpyDeviceToHost, s));
        }
    }
    HIP_TRY(hipStreamSynchronize(s));
    if (send_counts)
        for (uint32_t r = 0; r < c->G; ++r) send_counts[r] = c->mapped ? c->send_counts[r] : 0;
    return FK_OK;
}

FK_EXPORT int fk_bin_owners(const fk_ctx *c, int32_t *owner) {
    if (!c || !owner) return set_err(FK_E_INVALID, "null argument");
    for (int32_t b = 0; b < c->Bc; ++b) owner[b] = c->custom_owners ? c->h_owner[b] : (int32_t)((uint32_t)b % c->G);
    return FK_OK;
}

// ---------------------------------------------------------------------------
// reduce side
// ---------------------------------------------------------------------------

static SortedPlan sorted_plan(const fk_ctx *c, uint64_t max_bin_kmers) {
    SortedPlan pl;
    const int k = c->cfg.k;
    const uint32_t cap = 2048;  // keys per LDS bucket (k_bucket_count64 / 128-bit k_bucket_sort)
    // cell bits: the largest bin's cells average cap/4 keys (a bucket groups a
    // few cells; runs of one chunk's keys per cell stay long enough to be
    // written as whole lines)
    // (two-level expansion, 64-bit keys: 512 since round 6 -- half the cells of
    // round 2's cap / 8, so the bucket cut and the last piece's level 2 touch
    // half the cell words: configs[2] load 146.9 -> 146.3 ms, configs[1] equal,
    // profiles/r06r_cell_target.txt; 128-bit keys keep 128 per cell)
    // k = 64 (no spare bit in a 128-bit key's hi word): one-level scatter, one workgroup per bucket
    const bool tiered = c->cfg.k <= 63 && c->dbg_phase == 99 && !c->force_large;
    const bool two_level = c->cfg.k <= 63;
#ifndef FK_CELL_TARGET64
#define FK_CELL_TARGET64 512  // A/B builds: keys per cell of the largest bin, 64-bit keys, two levels
#endif
    const uint64_t target = c->cell_target ? c->cell_target
                                           : (c->KW == 2 && tiered ? WAVE128_BUCKET_CAP / 2
                                                                   : two_level ? FK_CELL_TARGET64 : cap / 4);
    int F = 1;
    while (F < MAX_FINE_BITS && ((uint64_t)1 << F) * target < max_bin_kmers) ++F;
    if (!two_level) F = std::min(F, MAX_FINE_BITS - 1);  // one-level scatter: 8 << F bytes of LDS <= 128 KB
    F = std::min(F, 2 * k);
    // k <= 63: two levels (super-cells, then cells; one level measured slower, DESIGN.md §4 "Count" 7);
    // cells per super-cell: 2^5 up to F = 13, 2^6 above (measured at configs[1] and at 8x larger bins)
    const uint32_t wave_cap = c->KW == 1 ? WAVE_BUCKET_CAP : WAVE128_BUCKET_CAP;
    const int F2 = std::min(F, std::max(5, std::min(6, F - 8))), F1 = F - F2;
    pl.F = F, pl.F2 = F2, pl.F1 = F1, pl.tiered = tiered, pl.two_level = two_level, pl.cap = cap, pl.wave_cap = wave_cap;
    pl.max_bin = max_bin_kmers;
    return pl;
}

// 4: expand the records (chunk table at c->chunks, records at c->rsrc) into canonical k-mers laid
// out bin-major by cell in `keys`; c->cell_total = the cell totals, `cell_base` their exclusive
// scan (ncell_all + 1 entries)
static int sorted_expand(fk_ctx *c, const SortedPlan &pl, uint32_t nchunks, uint64_t total_kmers, DevBuf &keys,
                         DevBuf &cell_base_buf) {
    hipStream_t s = c->stream;
    const int k = c->cfg.k;
    const int F = pl.F, F2 = pl.F2, F1 = pl.F1;
    const bool two_level = pl.two_level;
    const uint32_t ncell = 1u << F;
    const uint64_t ncell_all = (uint64_t)c->nlb << F;
    FK_TRY(ensure(keys, total_kmers * 8 * c->KW));
    FK_TRY(ensure(c->cell_total, ncell_all * 8));
    FK_TRY(ensure(cell_base_buf, (ncell_all + 1) * 8));
    uint64_t *const cell_base = cell_base_buf.as<uint64_t>();
    // 4: expand records -> canonical k-mers, laid out bin-major by cell
    if (two_level) {
        // cell totals by atomics, per-chunk counts only per super-cell
        const uint64_t nsc_all = (uint64_t)c->nlb << F1;
        FK_TRY(ensure(c->lp, ((uint64_t)nchunks << F1) * 4));
        FK_TRY(ensure(c->sc_total, nsc_all * 8));
        // bins split into pieces of chunks so that ~HIST_PIECES workgroups balance over the CUs (one
        // workgroup per bin waits for the largest bin when bins are few and large)
        constexpr double HIST_PIECES = 1024.0;
        std::vector<uint32_t> pieces, first;
        bool split = false;
        if (nchunks && c->h_bcb.size() == (size_t)c->nlb + 1) {
            for (uint32_t lb = 0; lb < c->nlb; ++lb) {
                const uint32_t cb = c->h_bcb[lb], ce = c->h_bcb[lb + 1], nc = ce - cb;
                const uint32_t P = std::max(1u, std::min(nc, (uint32_t)(HIST_PIECES * nc / nchunks + 0.5)));
                const uint32_t f = (uint32_t)(pieces.size() / 4);
                for (uint32_t q = 0; q < P; ++q) {
                    pieces.insert(pieces.end(), {lb, cb + nc * q / P, cb + nc * (q + 1) / P, P == 1 ? 1u : 0u});
                    first.push_back(f);
                }
                split |= P > 1;
            }
        }
        if (split) {
            const uint32_t np = (uint32_t)first.size();
            FK_TRY(ensure(c->hpieces, (uint64_t)np * 16));
            FK_TRY(ensure(c->hpiece_first, (uint64_t)np * 4));
            FK_TRY(ensure(c->hpiece_tot, ((uint64_t)np << F1) * 4));
            HIP_TRY(hipMemcpyAsync(c->hpieces.p, pieces.data(), (uint64_t)np * 16, hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemcpyAsync(c->hpiece_first.p, first.data(), (uint64_t)np * 4, hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemsetAsync(c->cell_total.p, 0, ncell_all * 8, s));
            HIP_TRY(launch_expand_hist_pieces(c->KW, c->rsrc, c->chunks.as<Chunk>(), c->hpieces.as<uint4>(),
                                              c->hpiece_first.as<uint32_t>(), np, k, F, F2,
                                              c->cell_total.as<uint64_t>(), c->lp.as<uint32_t>(),
                                              c->hpiece_tot.as<uint32_t>(), s));
            HIP_TRY(hipStreamSynchronize(s));  // the host piece tables are released below
        } else {
            HIP_TRY(launch_expand_hist_bin(c->KW, c->rsrc, c->chunks.as<Chunk>(), c->bin_chunk_begin.as<uint32_t>(),
                                           c->nlb, k, F, F2, c->cell_total.as<uint64_t>(), c->lp.as<uint32_t>(), s));
        }
    } else {
        FK_TRY(ensure(c->lp, (uint64_t)nchunks * ncell * 4));
        HIP_TRY(launch_expand_hist(c->W, c->rsrc, c->chunks.as<Chunk>(), nchunks, k, F,
                                   c->lp.as<uint32_t>(), s));
        HIP_TRY(launch_cell_prefix(c->bin_chunk_begin.as<uint32_t>(), c->nlb, F, c->lp.as<uint32_t>(),
                                   c->cell_total.as<uint64_t>(), s));
    }
    HIP_TRY(scan_excl_sum_u64(c->cell_total.as<uint64_t>(), cell_base, ncell_all, cell_base + ncell_all, c->ws, s));
    if (c->cut_side) HIP_TRY(hipEventRecord(c->side_ev[2], s));  // the cell totals and offsets are ready
    if (two_level) {
        FK_TRY(ensure(c->mid, total_kmers * 8 * c->KW));
        HIP_TRY(launch_expand_two_level(c->KW, c->rsrc, c->chunks.as<Chunk>(), nchunks, c->nlb, k, F,
                                        F2, c->lp.as<uint32_t>(), cell_base, c->mid.as<uint64_t>(),
                                        keys.as<uint64_t>(), s, c->x2_l1, total_kmers));
    } else {
        HIP_TRY(launch_expand_scatter(c->W, c->rsrc, c->chunks.as<Chunk>(), nchunks, k, F,
                                      c->lp.as<uint32_t>(), cell_base, keys.as<uint64_t>(), s));
    }
    return FK_OK;
}

// 4c + 5: buckets over c->cell_total / c->cell_base (the job's cells), their exact counts from
// `src` (one key array, or the staged pieces'), the dense result and its bin offsets
// The buffers of one bucket cut and its counts (the job's, or a staged job's pre-count).
struct CountBufs {
    DevBuf *flags, *flag_scan, *buckets, *bucket_unique, *tier_list, *piece_starts, *out_counts;
};
static CountBufs main_bufs(fk_ctx *c) {
    return CountBufs{&c->flags, &c->flag_scan, &c->buckets, &c->bucket_unique, &c->tier_list, &c->piece_starts,
                     &c->out_counts};
}

// The listed buckets of at most cap keys above skip_le keys (skip_le: counted by a mid wave tier) in one
// workgroup's LDS: the block kernel (64-bit keys) or the LDS radix sort (128-bit keys).
static int block_tier(fk_ctx *c, const BucketSrc &src, CountBufs B, DevBuf &okb, const uint32_t *list, uint32_t n,
                      uint32_t cap, uint32_t skip_le, hipStream_t s) {
    if (c->KW == 1)
        HIP_TRY(launch_bucket_count64(src, B.buckets->as<Bucket>(), n, c->cfg.k, okb.as<uint64_t>(),
                                      B.out_counts->as<uint32_t>(), B.bucket_unique->as<uint64_t>(),
                                      c->misc.as<unsigned long long>() + 1, cap, 99, list, s, skip_le));
    else
        HIP_TRY(launch_bucket_sort(2, src, B.buckets->as<Bucket>(), n, c->cfg.k, okb.as<uint64_t>(),
                                   B.out_counts->as<uint32_t>(), B.bucket_unique->as<uint64_t>(),
                                   c->misc.as<unsigned long long>() + 1, cap, list, s, skip_le));
    return FK_OK;
}

// 4c + 5: buckets over cell_total / cell_base (ncell_all cells), their exact counts from `src` (one
// key array, or the staged pieces') into okb / B.out_counts at each bucket's first slot, the
// distinct keys per bucket in B.bucket_unique; *nb_out = buckets
static int sorted_count_buckets(fk_ctx *c, const SortedPlan &pl, const BucketSrc &src_in, uint64_t total_kmers,
                                const uint64_t *cell_total, const uint64_t *cell_base, CountBufs B, DevBuf &okb,
                                uint64_t *nb_out) {
    hipStream_t s = c->stream;
    // the cut's stream: `s`, or beside the last staged piece's expansion (cut_side)
    const hipStream_t cs = c->cut_side ? c->tier_side : s;
    const int k = c->cfg.k;
    const int F = pl.F;
    const bool tiered = pl.tiered;
    const uint32_t cap = pl.cap, wave_cap = pl.wave_cap;
    const uint64_t ncell_all = (uint64_t)c->nlb << F;
    // useHT=1 (extractKXmersHT, SBKC:664-739): the wave tiers' LDS hash tables emit their keys in
    // table order (the reference writes its hash map's iteration order, SBKC:723-734), no rank; the
    // heavier tiers' outputs stay ascending, which is one such order too
    const bool ordered = !c->cfg.use_ht;
    FK_TRY(ensure(*B.flags, ncell_all * 4));
    FK_TRY(ensure(*B.flag_scan, (ncell_all + 1) * 8));
    FK_TRY(ensure(c->misc, 64));
    // 4c: buckets.  Tiered (k <= 32): cells packed greedily into buckets of
    // <= wave_cap keys for the wave kernel, larger cells to the block kernel
    // (<= cap) or the large path.  Otherwise buckets of <= cap keys.
    if (tiered)
        HIP_TRY(launch_bucket_flags_greedy(cell_total, c->nlb, F, wave_cap, -1, B.flags->as<uint32_t>(), cs));
    else
        HIP_TRY(launch_bucket_flags(cell_base, cell_total, c->nlb, F, cap / 4, cap - cap / 4, B.flags->as<uint32_t>(), cs));
    HIP_TRY(scan_excl_sum_u32_to_u64(B.flags->as<uint32_t>(), B.flag_scan->as<uint64_t>(), ncell_all,
                                     B.flag_scan->as<uint64_t>() + ncell_all, c->ws, cs));
    uint64_t nbuckets = 0;
    HIP_TRY(hipMemcpyAsync(&nbuckets, B.flag_scan->as<uint64_t>() + ncell_all, 8, hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipStreamSynchronize(cs));
    htrace("sorted: nbuckets read");
    FK_TRY(ensure(*B.buckets, nbuckets * sizeof(Bucket)));
    FK_TRY(ensure(okb, total_kmers * 8 * c->KW));
    FK_TRY(ensure(*B.out_counts, total_kmers * 4));
    FK_TRY(ensure(*B.bucket_unique, (nbuckets + 1) * 8));
    HIP_TRY(launch_bucket_write(cell_base, B.flags->as<uint32_t>(), B.flag_scan->as<uint64_t>(), c->nlb, F, nbuckets,
                                total_kmers, B.buckets->as<Bucket>(), cs));
    BucketSrc src = src_in;
    src.F = F;
    if (src.np > 0) FK_TRY(ensure(*B.piece_starts, nbuckets * sizeof(PieceStarts)));
    // the buckets' sizes, and the staged pieces' starts per bucket (read by the wave tier)
    HIP_TRY(launch_bucket_finish(src, B.buckets->as<Bucket>(), nbuckets, c->nlb, total_kmers,
                                 src.np > 0 ? B.piece_starts->as<PieceStarts>() : nullptr, cs));
    if (src.np > 0) src.starts = B.piece_starts->as<PieceStarts>();
    // 5: exact count per bucket in LDS; buckets that do not fit take the streaming path
    const uint32_t small_limit = c->force_large ? 0u : cap;
    HIP_TRY(hipMemsetAsync(c->misc.p, 0, 64, cs));
    c->stats.buckets = nbuckets;
    c->stats.fine_bits = (uint64_t)F;
    c->stats.heavy_keys = 0;
    c->stats.split_buckets = c->stats.sub_buckets = 0;
    if (tiered) {
        FK_TRY(ensure(*B.tier_list, nbuckets * 8));
        uint32_t *lists = B.tier_list->as<uint32_t>();
#ifndef FK_SPLIT_HEAVY
#define FK_SPLIT_HEAVY 1  // A/B builds (build_variant "nosplit", -DFK_SPLIT_HEAVY=0): no heavy-bucket split
#endif
        // the block tier's top: 64-bit keys with the split, the mid wave tier's cap (above it: split)
        // (the 513..1024-key buckets through the split as well, no mid wave tier: configs[2] load
        // 1.1-1.4 ms slower, configs[1] 0.3 ms, profiles/r05zg_mid_split_ab.txt)
        const uint32_t block_top = FK_SPLIT_HEAVY ? (c->KW == 1 ? WAVE_MID_CAP : WAVE128_MID_CAP) : cap;
        HIP_TRY(launch_bucket_tiers(B.buckets->as<Bucket>(), nbuckets, wave_cap, block_top,
                                    B.bucket_unique->as<uint64_t>(), lists, c->misc.as<unsigned int>(),
                                    c->misc.as<unsigned long long>() + 3, cs));
        // the tier sizes (and the listed buckets' keys) go to pinned memory right behind the tier
        // kernel: the host waits for that copy, not for the wave tier queued after it, before it
        // queues the heavier tiers
        if (c->pin_tier.ensure(64)) return set_err(FK_E_NOMEM, "hipHostMalloc failed");
        HIP_TRY(hipMemcpyAsync(c->pin_tier.p, c->misc.p, 32, hipMemcpyDeviceToHost, cs));
        HIP_TRY(hipEventRecord(c->tier_ev, cs));
#ifndef FK_TIER_SIDE
#define FK_TIER_SIDE 1  // A/B builds: -DFK_TIER_SIDE=0 the heavy tiers queued behind the wave tier
#endif
        // the heavier tiers (split, in-order sub-buckets, mid wave tier, fallbacks) run on their own
        // stream beside the wave tier: their buckets, outputs and counters are disjoint from its, and
        // the host's waits for the split's counts no longer wait for the wave tier
        const hipStream_t hs = (FK_TIER_SIDE && c->tier_side) ? c->tier_side : s;
        if (cs != s) {  // the wave tier after the cut (and, in stream order, the last piece's expansion)
            HIP_TRY(hipEventRecord(c->side_ev[0], cs));
            HIP_TRY(hipStreamWaitEvent(s, c->side_ev[0], 0));
        }
        if (hs != s) {  // the heavy tiers after both as well
            HIP_TRY(hipEventRecord(c->side_ev[3], s));
            HIP_TRY(hipStreamWaitEvent(hs, c->side_ev[3], 0));
        }
        // every bucket of <= wave_cap keys
        if (c->KW == 1)
            HIP_TRY(launch_bucket_count64_wave(src, B.buckets->as<Bucket>(), nbuckets, k,
                                               okb.as<uint64_t>(), B.out_counts->as<uint32_t>(),
                                               B.bucket_unique->as<uint64_t>(), nullptr, s, ordered));
        else
            HIP_TRY(launch_bucket_count128_wave(src, B.buckets->as<Bucket>(), nbuckets, k,
                                                okb.as<uint64_t>(), B.out_counts->as<uint32_t>(),
                                                B.bucket_unique->as<uint64_t>(), s, ordered));
        HIP_TRY(hipEventSynchronize(c->tier_ev));
        const uint32_t ntier[2] = {c->pin_tier.as<uint32_t>()[0], c->pin_tier.as<uint32_t>()[1]};
        const uint64_t listed_keys = c->pin_tier.as<uint64_t>()[3];
        c->stats.heavy_keys = listed_keys;
        htrace("sorted: tiers read");
        c->stats.block_buckets = ntier[0];
        c->stats.big_buckets = ntier[1];
        uint64_t nlarge = 0;
        if (ntier[0] || ntier[1]) {
            // Above the wave tier.  The block tier (up to the mid wave tier's cap: 1024 keys for 64-bit
            // keys, 512 for 128-bit ones) is counted by the mid wave tier, one wave per bucket.  The big
            // tier (above it) is split into wave-sized sub-buckets by sampled splitters and counted in
            // order by one wave per bucket; a bucket with a sub-bucket too large for a wave (a k-mer
            // repeated that often) falls back to the block kernel / LDS sort (<= cap keys) or the
            // big-table kernel (64-bit) and the streaming path.  Without the split (-DFK_SPLIT_HEAVY=0,
            // A/B builds) the block tier reaches cap and the block kernel / LDS sort takes its buckets
            // above the mid wave tier's cap.
            const bool w1 = c->KW == 1;
            const uint32_t *l1 = lists + nbuckets;
            uint32_t *fbB = nullptr, *fbG = lists + nbuckets;  // the fallback lists (block / big)
            uint32_t nfbB = 0, nfbG = ntier[1];
#ifndef FK_MID_PARTS
#define FK_MID_PARTS 1  // A/B builds: -DFK_MID_PARTS=0 the 64-bit mid tier's buckets all on the 1024-key kernel
#endif
            constexpr uint32_t MID_PARTS_MIN = 1u << 17;  // mid-tier buckets from which the ranges kernel pays
            // 64-bit mid tier: 2 or 3 key ranges per bucket on the wave tier's table (k_bucket_count64_parts);
            // the buckets it leaves (a range above 512 keys) are listed for the 1024-key kernel.  Only for a
            // large mid tier: the configs[2] load's 278 K mid buckets 146.5 -> 146.2 ms, but configs[1]'s 59 K
            // 21.8 -> 21.95 ms (profiles/r06v_mid_parts_ab.txt).  A smaller mid tier (a job whose k-mers
            // repeat: configs[1]) goes straight on the wave tier's table whole (k_bucket_count64_mid512), the
            // buckets with more than 512 distinct keys listed for the 1024-key kernel.  Both run first on the
            // side stream, ahead of the split.
            const bool mid_wave = FK_MID_PARTS && w1 && ntier[0] && block_top == WAVE_MID_CAP && c->mid_parts != 0;
            const bool parts = mid_wave && (c->mid_parts == 1 || (c->mid_parts != 2 && ntier[0] >= MID_PARTS_MIN));
            uint32_t *mid_fb = nullptr, nmidfb = 0;
            unsigned int *mid_fbc = c->misc.as<unsigned int>() + 11;
            if (mid_wave) {
                FK_TRY(ensure(c->mid_fb, (uint64_t)ntier[0] * 4));
                mid_fb = c->mid_fb.as<uint32_t>();
                if (parts)
                    HIP_TRY(launch_bucket_count64_parts(src, B.buckets->as<Bucket>(), lists, ntier[0], k,
                                                        okb.as<uint64_t>(), B.out_counts->as<uint32_t>(),
                                                        B.bucket_unique->as<uint64_t>(), mid_fb, mid_fbc, hs, ordered));
                else
                    HIP_TRY(launch_bucket_count64_mid512(src, B.buckets->as<Bucket>(), lists, ntier[0], k,
                                                         okb.as<uint64_t>(), B.out_counts->as<uint32_t>(),
                                                         B.bucket_unique->as<uint64_t>(), mid_fb, mid_fbc, hs, ordered));
            }
            if (FK_SPLIT_HEAVY && ntier[1]) {  // nothing to split: no split kernels, no read-back
                const uint32_t nl = ntier[1];
                const uint64_t maxsub = listed_keys / 64 + nl + 64;  // >= ceil(n / SPL_TGT) sub-buckets per bucket
                const size_t sub_bytes = w1 ? sizeof(SubBucket) : sizeof(SubBucket128);
                FK_TRY(ensure(c->sp_base, ((uint64_t)nl + 1) * 8));
                // 64-bit keys: a 512-key region per first-cut sub-bucket (split_room: <= 2 n + 512 per bucket)
                FK_TRY(ensure(c->sp_keys, (w1 ? 2 * listed_keys + 512ull * nl : listed_keys) * 8 * c->KW));
                FK_TRY(ensure(c->sp_subs, maxsub * sub_bytes));
                FK_TRY(ensure(c->sp_par, (uint64_t)nl * sizeof(SplitParent)));
                FK_TRY(ensure(c->sp_fb, (uint64_t)nl * 8));
                uint32_t *fb = c->sp_fb.as<uint32_t>();
                unsigned int *spc = c->misc.as<unsigned int>() + 8;  // [0] sub-buckets, [1] / [2] fallbacks
                HIP_TRY(launch_listed_sizes(B.buckets->as<Bucket>(), lists, 0, l1, nl, c->sp_base.as<uint64_t>(), hs,
                                            w1));
                HIP_TRY(scan_excl_sum_u64(c->sp_base.as<uint64_t>(), c->sp_base.as<uint64_t>(), nl,
                                          c->sp_base.as<uint64_t>() + nl, c->ws, hs));
                if (w1)
                    HIP_TRY(launch_bucket_split64(src, B.buckets->as<Bucket>(), lists, 0, l1, nl,
                                                  c->sp_base.as<uint64_t>(), c->sp_keys.as<uint64_t>(),
                                                  c->sp_subs.as<SubBucket>(), c->sp_par.as<SplitParent>(), spc, fb,
                                                  fb + nl, cap, k, F, hs, c->split_retry));
                else
                    HIP_TRY(launch_bucket_split128(src, B.buckets->as<Bucket>(), l1, nl, c->sp_base.as<uint64_t>(),
                                                   c->sp_keys.as<uint64_t>(), c->sp_subs.as<SubBucket128>(),
                                                   c->sp_par.as<SplitParent>(), spc, fb, fb + nl, cap, k, F, hs,
                                                   c->split_retry));
                HIP_TRY(hipMemcpyAsync(c->pin_tier.as<uint8_t>() + 32, spc, 16, hipMemcpyDeviceToHost, hs));
                HIP_TRY(hipEventRecord(c->tier_ev, hs));
                HIP_TRY(hipEventSynchronize(c->tier_ev));
                const uint32_t *sc = c->pin_tier.as<uint32_t>() + 8;
                const uint32_t nsub = sc[0];
                nmidfb = sc[3];  // misc word 11: the ranges kernel's fallbacks (queued before the copy)
                fbB = fb, nfbB = sc[1], fbG = fb + nl, nfbG = sc[2];
                htrace("sorted: split counts read");
#ifdef FK_PROBES
                if (w1 && getenv("FASTKMER_HOST_TRACE")) {  // the split buckets by size class: buckets, keys, fallbacks
                    std::vector<uint64_t> base((size_t)nl + 1);
                    std::vector<uint32_t> f(2 * (size_t)nl), h_l((size_t)nl);
                    HIP_TRY(hipMemcpy(base.data(), c->sp_base.p, base.size() * 8, hipMemcpyDeviceToHost));
                    HIP_TRY(hipMemcpy(f.data(), fb, f.size() * 4, hipMemcpyDeviceToHost));
                    HIP_TRY(hipMemcpy(h_l.data(), l1, (size_t)nl * 4, hipMemcpyDeviceToHost));
                    std::unordered_map<uint32_t, uint32_t> pos;
                    for (uint32_t j = 0; j < nl; ++j) pos[h_l[j]] = j;
                    uint64_t hb[40] = {}, hk[40] = {}, hf[40] = {}, hfk[40] = {};
                    std::vector<char> isfb(nl, 0);
                    for (uint32_t j = 0; j < sc[1]; ++j) isfb[pos[f[j]]] = 1;
                    for (uint32_t j = 0; j < sc[2]; ++j) isfb[pos[f[nl + j]]] = 1;
                    for (uint32_t j = 0; j < nl; ++j) {
                        const uint64_t n = base[j + 1] - base[j];
                        const int cl = 63 - __builtin_clzll(n | 1);
                        hb[cl] += 1, hk[cl] += n;
                        if (isfb[j]) hf[cl] += 1, hfk[cl] += n;
                    }
                    unsigned long long rk[4];
                    HIP_TRY(hipDeviceSynchronize());
                    HIP_TRY(rank_probe_read(rk, true));
                    fprintf(stderr, "probe_rank (wave tier, before the split): iterations %llu keys %llu buckets %llu "
                            "wall (small groups) %llu\n", rk[0], rk[1], rk[2], rk[3]);
                    fprintf(stderr, "probe_split: split %u keys %llu subs %u fallbacks %u + %u\n", nl,
                            (unsigned long long)base[nl], nsub, sc[1], sc[2]);
                    for (int cl = 0; cl < 40; ++cl)
                        if (hb[cl])
                            fprintf(stderr, "probe_split: n in [2^%d, 2^%d): buckets %llu keys %llu fallback buckets %llu keys %llu\n",
                                    cl, cl + 1, (unsigned long long)hb[cl], (unsigned long long)hk[cl],
                                    (unsigned long long)hf[cl], (unsigned long long)hfk[cl]);
                }
#endif
                if (nsub > maxsub) return set_err(FK_E_DEVICE, "bucket split: %u sub-buckets of at most %llu", nsub,
                                                  (unsigned long long)maxsub);
                if (w1)
                    HIP_TRY(launch_sub_count64_seq(B.buckets->as<Bucket>(), l1, nl, c->sp_par.as<SplitParent>(),
                                                   c->sp_subs.as<SubBucket>(), c->sp_keys.as<uint64_t>(),
                                                   okb.as<uint64_t>(), B.out_counts->as<uint32_t>(),
                                                   B.bucket_unique->as<uint64_t>(), hs, ordered));
                else
                    HIP_TRY(launch_sub_count128_seq(B.buckets->as<Bucket>(), l1, nl, c->sp_par.as<SplitParent>(),
                                                    c->sp_subs.as<SubBucket128>(), c->sp_keys.as<uint64_t>(),
                                                    okb.as<uint64_t>(), B.out_counts->as<uint32_t>(),
                                                    B.bucket_unique->as<uint64_t>(), hs, ordered));
                c->stats.split_buckets = nl - sc[1] - sc[2];
                c->stats.sub_buckets = nsub;
            }
            if (mid_wave && !(FK_SPLIT_HEAVY && ntier[1])) {  // no split read-back: the fallbacks' count alone
                HIP_TRY(hipMemcpyAsync(c->pin_tier.as<uint8_t>() + 44, mid_fbc, 4, hipMemcpyDeviceToHost, hs));
                HIP_TRY(hipEventRecord(c->tier_ev, hs));
                HIP_TRY(hipEventSynchronize(c->tier_ev));
                nmidfb = c->pin_tier.as<uint32_t>()[11];
            }
            const uint32_t mid_cap = w1 ? WAVE_MID_CAP : WAVE128_MID_CAP;
            if (ntier[0]) {
                if (mid_wave) {
                    if (nmidfb)
                        HIP_TRY(launch_bucket_count64_wave_mid(src, B.buckets->as<Bucket>(), mid_fb, nmidfb, k,
                                                               okb.as<uint64_t>(), B.out_counts->as<uint32_t>(),
                                                               B.bucket_unique->as<uint64_t>(), hs, ordered));
                } else if (w1)
                    HIP_TRY(launch_bucket_count64_wave_mid(src, B.buckets->as<Bucket>(), lists, ntier[0], k,
                                                           okb.as<uint64_t>(), B.out_counts->as<uint32_t>(),
                                                           B.bucket_unique->as<uint64_t>(), hs, ordered));
                else
                    HIP_TRY(launch_bucket_count128_wave_mid(src, B.buckets->as<Bucket>(), lists, ntier[0], k,
                                                            okb.as<uint64_t>(), B.out_counts->as<uint32_t>(),
                                                            B.bucket_unique->as<uint64_t>(), hs, ordered));
                if (block_top > mid_cap)  // no split: the block tier's buckets above the mid wave tier
                    FK_TRY(block_tier(c, src, B, okb, lists, ntier[0], cap, mid_cap, hs));
            }
            if (nfbB) FK_TRY(block_tier(c, src, B, okb, fbB, nfbB, cap, 0, hs));
            if (nfbG && w1) {
                // above 2048 keys with at most 4096 distinct in one workgroup's LDS; others stay REDO
                HIP_TRY(launch_bucket_count64_big(src, B.buckets->as<Bucket>(), nfbG, k, okb.as<uint64_t>(),
                                                  B.out_counts->as<uint32_t>(), B.bucket_unique->as<uint64_t>(),
                                                  c->misc.as<unsigned long long>() + 2, fbG, hs));
                HIP_TRY(hipMemcpyAsync(&nlarge, c->misc.as<unsigned long long>() + 2, 8, hipMemcpyDeviceToHost, hs));
                HIP_TRY(hipStreamSynchronize(hs));
            } else if (nfbG) {
                nlarge = nfbG;  // 128-bit keys: no big-table kernel
            }
            if (nlarge) {  // scratch for the listed buckets' keys only, taken by a cursor
                FK_TRY(ensure(c->scratch, listed_keys * 8 * c->KW));
                HIP_TRY(hipMemsetAsync(c->misc.as<unsigned long long>() + 6, 0, 8, hs));
                HIP_TRY(launch_bucket_sort_large(c->KW, src, B.buckets->as<Bucket>(), nfbG, k,
                                                 c->scratch.as<uint64_t>(), okb.as<uint64_t>(),
                                                 B.out_counts->as<uint32_t>(), B.bucket_unique->as<uint64_t>(),
                                                 fbG, hs, c->misc.as<unsigned long long>() + 6));
            }
        }
        if (hs != s) {  // the result's scans follow both streams
            HIP_TRY(hipEventRecord(c->side_ev[1], hs));
            HIP_TRY(hipStreamWaitEvent(s, c->side_ev[1], 0));
        }
        c->stats.oversize_buckets = nlarge;
    } else {
        if (src.np > 0) return set_err(FK_E_INVALID, "staged pieces need the tiered count");
        if (c->KW == 1)
            HIP_TRY(launch_bucket_count64(src, B.buckets->as<Bucket>(), nbuckets, k,
                                          okb.as<uint64_t>(), B.out_counts->as<uint32_t>(),
                                          B.bucket_unique->as<uint64_t>(), c->misc.as<unsigned long long>(),
                                          small_limit, c->dbg_phase, nullptr, s));
        else
            HIP_TRY(launch_bucket_sort(c->KW, src, B.buckets->as<Bucket>(), nbuckets, k,
                                       okb.as<uint64_t>(), B.out_counts->as<uint32_t>(),
                                       B.bucket_unique->as<uint64_t>(), c->misc.as<unsigned long long>(),
                                       small_limit, nullptr, s));
        uint64_t oversize = 0;
        HIP_TRY(hipMemcpyAsync(&oversize, c->misc.p, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        c->stats.oversize_buckets = oversize;
        if (oversize) {
            FK_TRY(ensure(c->scratch, total_kmers * 8 * c->KW));
            HIP_TRY(launch_bucket_sort_large(c->KW, src, B.buckets->as<Bucket>(), nbuckets, k,
                                             c->scratch.as<uint64_t>(), okb.as<uint64_t>(),
                                             B.out_counts->as<uint32_t>(), B.bucket_unique->as<uint64_t>(),
                                             nullptr, s));
        }
    }
    *nb_out = nbuckets;
    return FK_OK;
}

// The count's result from its buckets: dense_off = the exclusive scan of the distinct keys per bucket,
// bin_off per local bin (`flag_scan` of the bucket cut: a bin's first cell starts a bucket).  The
// result stays bucket-major (no compaction pass): readers gather a bin's buckets (fk_get_bin) or the
// whole result (fk_write_bins, materialize_dense).
static int sorted_result(fk_ctx *c, int F, uint64_t nbuckets, DevBuf &okb, CountBufs B) {
    hipStream_t s = c->stream;
    FK_TRY(ensure(c->dense_off, (nbuckets + 1) * 8));
    HIP_TRY(scan_excl_sum_u64(B.bucket_unique->as<uint64_t>(), c->dense_off.as<uint64_t>(), nbuckets,
                              c->dense_off.as<uint64_t>() + nbuckets, c->ws, s));
    FK_TRY(ensure(c->bin_off, ((uint64_t)c->nlb + 1) * 8));
    c->distinct_pending = true;
    HIP_TRY(launch_bin_offsets(B.flag_scan->as<uint64_t>(), c->dense_off.as<uint64_t>(), c->nlb, F, nbuckets,
                               c->bin_off.as<uint64_t>(), s));
    c->gapped = true;
    c->dense_ready = false;
    c->res_keys = okb.as<uint64_t>();
    c->res_nbuckets = nbuckets;
    c->res_F = F;
    c->res_fs = B.flag_scan->as<uint64_t>();
    return FK_OK;
}

static int sorted_count(fk_ctx *c, const SortedPlan &pl, const BucketSrc &src_in, uint64_t total_kmers) {
    // the two-level count writes its buckets' results over the first expansion level (`mid` is dead
    // once level 2 has run, stream order; a staged job's `mid` held one piece and grows to the job
    // here, its contents dead): one k-mer array less on the device (57 GB at configs[3]'s per-GPU
    // load, 128-bit keys; 36 GB at configs[2]'s)
    DevBuf &okb = pl.two_level ? c->mid : c->out_keys;
    uint64_t nb = 0;
    FK_TRY(sorted_count_buckets(c, pl, src_in, total_kmers, c->cell_total.as<uint64_t>(), c->cell_base.as<uint64_t>(),
                                main_bufs(c), okb, &nb));
    return sorted_result(c, pl.F, nb, okb, main_bufs(c));
}

// After the bin offsets are on the host: the sorted count's distinct total is their last entry.
static void resolve_distinct(fk_ctx *c) {
    if (c->distinct_pending && !c->h_bin_off.empty()) c->distinct = c->h_bin_off.back();
    c->distinct_pending = false;
}

static int reduce_sorted(fk_ctx *c, uint32_t nchunks, uint64_t total_kmers, uint64_t max_bin_kmers) {
    const SortedPlan pl = sorted_plan(c, max_bin_kmers);
    FK_TRY(sorted_expand(c, pl, nchunks, total_kmers, c->keys, c->cell_base));
    BucketSrc src{c->keys.as<uint64_t>(), pl.F};
    return sorted_count(c, pl, src, total_kmers);
}

// Chunks of <= CHUNK_RECORDS records per local bin (chunks never span bins;
// a bin's chunks are consecutive).  ranges[lb] = the bin's record ranges.
static void build_chunks(uint32_t nlb, const std::vector<std::vector<std::pair<uint64_t, uint64_t>>> &ranges,
                         std::vector<Chunk> &chunks, std::vector<uint32_t> &bcb) {
    chunks.clear();
    bcb.assign((size_t)nlb + 1, 0);
    for (uint32_t lb = 0; lb < nlb; ++lb) {
        bcb[lb] = (uint32_t)chunks.size();
        for (const auto &rg : ranges[lb]) {
            for (uint64_t r = rg.first; r < rg.second; r += CHUNK_RECORDS) {
                Chunk ch;
                ch.rec_begin = r;
                ch.rec_end = std::min<uint64_t>(r + CHUNK_RECORDS, rg.second);
                ch.lbin = lb;
                ch.pad = 0;
                chunks.push_back(ch);
            }
        }
    }
    bcb[nlb] = (uint32_t)chunks.size();
}

// The count over the chunk table (records at c->rsrc), bin offsets, stats.
static int reduce_tail(fk_ctx *c, uint64_t nrecv, const std::vector<Chunk> &chunks, const std::vector<uint32_t> &bcb,
                       const std::vector<uint64_t> &bkm, double t0) {
    hipStream_t s = c->stream;
    const uint32_t nlb = c->nlb;
    const uint32_t nchunks = (uint32_t)chunks.size();
    uint64_t total_kmers = 0, max_bin = 0;
    for (uint32_t lb = 0; lb < nlb; ++lb) {
        total_kmers += bkm[lb];
        max_bin = std::max(max_bin, bkm[lb]);
    }
    HIP_TRY(hipEventRecord(c->ev[6], s));
    // the sorted count; useHT=1 (extractKXmersHT) the same with the wave tiers in table order
    FK_TRY(reduce_sorted(c, nchunks, total_kmers, max_bin));
    HIP_TRY(hipEventRecord(c->ev[7], s));
    c->h_bin_off.assign((size_t)nlb + 1, 0);
    if (c->pin_down.ensure(((size_t)nlb + 1) * 8)) return set_err(FK_E_NOMEM, "hipHostMalloc failed");
    HIP_TRY(hipMemcpyAsync(c->pin_down.p, c->bin_off.p, ((uint64_t)nlb + 1) * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    memcpy(c->h_bin_off.data(), c->pin_down.p, ((size_t)nlb + 1) * 8);
    resolve_distinct(c);
    htrace("tail: bin offsets read");
    c->stats.records_received = nrecv;
    c->stats.distinct = c->distinct;
    c->stats.ms_partition = ev_ms(c->ev[4], c->ev[5]);
    c->stats.ms_count = ev_ms(c->ev[6], c->ev[7]);
    c->stats.ms_total += now_ms() - t0;
    c->have_result = true;
    return FK_OK;
}

static int upload_chunks(fk_ctx *c, const std::vector<Chunk> &chunks, const std::vector<uint32_t> &bcb) {
    hipStream_t s = c->stream;
    const uint32_t nchunks = (uint32_t)chunks.size();
    FK_TRY(ensure(c->chunks, nchunks * sizeof(Chunk)));
    FK_TRY(ensure(c->bin_chunk_begin, ((uint64_t)c->nlb + 1) * 4));
    // the previous upload out of the staging buffer may still be queued (on the map stream, or on the
    // staging stream behind a step's transfer): wait for it before the host overwrites the buffer
    if (c->pin_up_busy) FK_TRY(comm_event_sync(c, c->pin_up_ev));
    c->pin_up_busy = false;
    const size_t cb = (size_t)nchunks * sizeof(Chunk), bb = ((size_t)c->nlb + 1) * 4;
    if (c->pin_up.ensure(cb + bb)) return set_err(FK_E_NOMEM, "hipHostMalloc(%zu) failed", cb + bb);
    memcpy(c->pin_up.p, chunks.data(), cb);
    memcpy(c->pin_up.as<uint8_t>() + cb, bcb.data(), bb);
    if (nchunks) HIP_TRY(hipMemcpyAsync(c->chunks.p, c->pin_up.p, cb, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->bin_chunk_begin.p, c->pin_up.as<uint8_t>() + cb, bb, hipMemcpyHostToDevice, s));
    HIP_TRY(hipEventRecord(c->pin_up_ev, s));
    c->pin_up_busy = true;
    c->h_bcb = bcb;
    return FK_OK;
}

// partition of the records of `src` (all owned by this rank) by local bin into c->precs (the
// count stage reads them at c->rsrc), the chunk table uploaded; bkm = k-mers per local bin
static int partition_src(fk_ctx *c, const RecSrc &src, uint64_t &nrecv, std::vector<Chunk> &chunks,
                         std::vector<uint32_t> &bcb, std::vector<uint64_t> &bkm, hipEvent_t e0, hipEvent_t e1) {
    nrecv = src.nrec;  // tiled sources: an upper bound, the partition counts them
    hipStream_t s = c->stream;
    const uint32_t nlb = c->nlb;
    HIP_TRY(hipEventRecord(e0, s));
    FK_TRY(part_count(c->part, src, 1, c->G, local_table(c), nlb, c->ws, s));
    htrace("reduce_src: part_count queued");
    // the scatter needs only the device-side offsets: it is queued before the host reads the part
    // totals (the output sized for src.nrec, for tiled sources the slot count: an upper bound), so
    // the GPU scatters while the host builds and uploads the chunk table
    FK_TRY(ensure(c->precs, src.nrec * c->W * 8));
    FK_TRY(part_scatter(c->part, 1, c->G, local_table(c), c->precs.as<uint64_t>(), s));
    htrace("reduce_src: scatter queued");
    std::vector<uint64_t> brec(nlb);
    bkm.assign(nlb, 0);
    if (c->pin_down.ensure((size_t)nlb * 16 + 16)) return set_err(FK_E_NOMEM, "hipHostMalloc failed");
    if (nlb) {
        HIP_TRY(hipMemcpyAsync(c->pin_down.p, c->part.rec.p, nlb * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(c->pin_down.as<uint64_t>() + nlb, c->part.kmer.p, nlb * 8, hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    if (nlb) {
        memcpy(brec.data(), c->pin_down.p, nlb * 8);
        memcpy(bkm.data(), c->pin_down.as<uint64_t>() + nlb, nlb * 8);
    }
    htrace("reduce_src: part counts read");
    // the bins' records are consecutive after the partition: chunks straight from the bin totals (no
    // per-bin range lists: the host is on the critical path between the read-back and the upload)
    uint64_t off = 0, nch = 0;
    for (uint32_t lb = 0; lb < nlb; ++lb) {
        off += brec[lb];
        nch += (brec[lb] + CHUNK_RECORDS - 1) / CHUNK_RECORDS;
    }
    if (src.tcnt) {
        // a tiled source (the fused map's slots) holds this rank's own input, all of it owned only
        // with one rank; its record total is the partition's
        if (c->G != 1) return set_err(FK_E_STATE, "tiled records partitioned on a context of %u ranks", c->G);
        nrecv = off;
    }
    if (off != nrecv)
        return set_err(FK_E_INVALID, "received records belong to bins of another rank (%llu of %llu owned)",
                       (unsigned long long)off, (unsigned long long)nrecv);
    chunks.resize(nch);
    bcb.assign((size_t)nlb + 1, 0);
    off = 0;
    uint32_t ci = 0;
    for (uint32_t lb = 0; lb < nlb; ++lb) {
        bcb[lb] = ci;
        const uint64_t end = off + brec[lb];
        for (uint64_t r = off; r < end; r += CHUNK_RECORDS)
            chunks[ci++] = Chunk{r, std::min<uint64_t>(r + CHUNK_RECORDS, end), lb, 0u};
        off = end;
    }
    bcb[nlb] = ci;
    FK_TRY(upload_chunks(c, chunks, bcb));
    htrace("reduce_src: chunks uploaded");
    HIP_TRY(hipEventRecord(e1, s));
    c->rsrc = c->precs.as<uint64_t>();
    return FK_OK;
}

// reduce of the records of `src` (all owned by this rank): partition by local bin, then count
static int reduce_src(fk_ctx *c, const RecSrc &src) {
    const double t0 = now_ms();
    c->have_result = false;
    uint64_t nrecv = 0;
    std::vector<Chunk> chunks;
    std::vector<uint32_t> bcb;
    std::vector<uint64_t> bkm;
    FK_TRY(partition_src(c, src, nrecv, chunks, bcb, bkm, c->ev[4], c->ev[5]));
    return reduce_tail(c, nrecv, chunks, bcb, bkm, t0);
}

FK_EXPORT int fk_reduce(fk_ctx *c, const void *d_recv, uint64_t nrecv) {
    if (!c) return set_err(FK_E_INVALID, "null ctx");
    DeviceGuard dg_(c->device);
    if (nrecv && !d_recv) return set_err(FK_E_INVALID, "null receive buffer");
    return reduce_src(c, dense_src((const uint64_t *)d_recv, nrecv, c->W));
}

FK_EXPORT int fk_set_grouped_emit(fk_ctx *c, int32_t enable) {
    if (!c) return set_err(FK_E_INVALID, "null ctx");
    DeviceGuard dg_(c->device);
    c->grouped = enable != 0;
    c->mapped = false;
    if (!c->grouped) return FK_OK;
    return build_group_table(c);
}

// The grouped emit's bin -> part table (part = destination * grp_nlb + the bin's local index there).
static int build_group_table(fk_ctx *c) {
    std::vector<uint32_t> table((size_t)c->Bc);
    if (c->custom_owners) {
        // size-aware placement (fk_set_bin_owners, the same table on every rank): part = owner *
        // L + the bin's index among its owner's bins in ascending order (the receiver's local bin)
        std::vector<uint32_t> cnt(c->G, 0);
        for (int32_t b = 0; b < c->Bc; ++b) table[b] = cnt[c->h_owner[b]]++;
        c->grp_nlb = std::max(1u, *std::max_element(cnt.begin(), cnt.end()));
        for (int32_t b = 0; b < c->Bc; ++b) table[b] += (uint32_t)c->h_owner[b] * c->grp_nlb;
    } else {
        c->grp_nlb = (uint32_t)((c->Bc + (int)c->G - 1) / (int)c->G);
        for (int32_t b = 0; b < c->Bc; ++b) table[b] = ((uint32_t)b % c->G) * c->grp_nlb + (uint32_t)b / c->G;
    }
    FK_TRY(ensure(c->grp_table, (uint64_t)c->Bc * 4));
    HIP_TRY(hipMemcpy(c->grp_table.p, table.data(), (uint64_t)c->Bc * 4, hipMemcpyHostToDevice));
    return FK_OK;
}

FK_EXPORT int32_t fk_grouped_parts_per_rank(const fk_ctx *c) { return c && c->grouped ? (int32_t)c->grp_nlb : 0; }

FK_EXPORT int fk_map_part_counts(fk_ctx *c, uint64_t *records, uint64_t *kmers) {
    if (!c || !records || !kmers) return set_err(FK_E_INVALID, "null argument");
    if (!c->grouped || !c->mapped) return set_err(FK_E_STATE, "fk_map_part_counts needs fk_set_grouped_emit and fk_map");
    std::copy(c->grp_rec.begin(), c->grp_rec.end(), records);
    std::copy(c->grp_kmer.begin(), c->grp_kmer.end(), kmers);
    return FK_OK;
}

// Counts records that arrive grouped by local bin: ranges[lb] = the bin's record ranges in d_recv.
static int reduce_ranges(fk_ctx *c, const uint64_t *d_recv, uint64_t nrecv,
                         const std::vector<std::vector<std::pair<uint64_t, uint64_t>>> &ranges,
                         const std::vector<uint64_t> &bkm, double t0) {
    std::vector<Chunk> chunks;
    std::vector<uint32_t> bcb;
    build_chunks(c->nlb, ranges, chunks, bcb);
    FK_TRY(upload_chunks(c, chunks, bcb));
    HIP_TRY(hipEventRecord(c->ev[5], c->stream));
    c->rsrc = d_recv;
    return reduce_tail(c, nrecv, chunks, bcb, bkm, t0);
}

FK_EXPORT int fk_reduce_grouped(fk_ctx *c, const void *d_recv, uint64_t nrecv, const uint64_t *seg_records,
                                const uint64_t *seg_kmers, int32_t nseg, int32_t parts_per_seg) {
    if (!c) return set_err(FK_E_INVALID, "null ctx");
    DeviceGuard dg_(c->device);
    if (nrecv && !d_recv) return set_err(FK_E_INVALID, "null receive buffer");
    if (nseg < 0 || parts_per_seg < 0 || (nseg && (!seg_records || !seg_kmers)))
        return set_err(FK_E_INVALID, "bad segment table");
    const double t0 = now_ms();
    hipStream_t s = c->stream;
    c->have_result = false;
    const uint32_t nlb = c->nlb;
    if ((uint32_t)parts_per_seg < nlb) return set_err(FK_E_INVALID, "%d parts per segment < %u local bins",
                                                      parts_per_seg, nlb);
    HIP_TRY(hipEventRecord(c->ev[4], s));
    // segment s holds, bin after bin, seg_records[s * parts + lb] records of local bin lb
    std::vector<std::vector<std::pair<uint64_t, uint64_t>>> ranges(nlb);
    std::vector<uint64_t> bkm(nlb, 0);
    uint64_t off = 0;
    for (int32_t sg = 0; sg < nseg; ++sg) {
        for (int32_t lb = 0; lb < parts_per_seg; ++lb) {
            const uint64_t n = seg_records[(uint64_t)sg * parts_per_seg + lb];
            if (n && (uint32_t)lb >= nlb) return set_err(FK_E_INVALID, "records for local bin %d of %u", lb, nlb);
            if (n) {
                ranges[lb].push_back({off, off + n});
                bkm[lb] += seg_kmers[(uint64_t)sg * parts_per_seg + lb];
            }
            off += n;
        }
    }
    if (off != nrecv)
        return set_err(FK_E_INVALID, "segment table holds %llu records, buffer %llu", (unsigned long long)off,
                       (unsigned long long)nrecv);
    return reduce_ranges(c, (const uint64_t *)d_recv, nrecv, ranges, bkm, t0);
}

// ---------------------------------------------------------------------------
// staged pieces: a job's input partitioned and expanded piece by piece while later pieces land
// ---------------------------------------------------------------------------

static void pieces_reset(fk_ctx *c) {
    c->st_np = 0;
    c->st_cut = 0;
    c->st_kmers = 0;
    c->pieces_void = false;
    c->tiles_counted = 0;
    c->segs_counted = 0;
}

// Staged pieces per job: 128-bit keys at most STAGE_MAXP128 (their kernels' piece loops stop there)
static uint32_t stage_maxp(const fk_ctx *c) { return c->KW == 2 ? (uint32_t)STAGE_MAXP128 : (uint32_t)STAGE_MAXP; }
// one rank's piece ends: FASTKMER_PIECE_CUTS, five pieces for a 64-bit job of >= 4 GB, else four
static const std::vector<double> &local_cuts(const fk_ctx *c) {
    if (!c->cuts_env && c->KW == 1 && c->job_bytes >= (4ull << 30) && STAGE_MAXP >= 5) return c->st_cuts5;
    return c->st_cuts;
}

// ---- staged pieces (sorted count, k <= 32): one rank's landed pieces, or the received segments
// (k = 64 counts the whole input after the last byte; so do the test hook that routes every bucket
// through the streaming path and the bucket-kernel probes)
static bool staged_ok(const fk_ctx *c) {
    return c->cfg.k <= 63 && c->dbg_phase == 99 && !c->force_large;
}
static bool staged_eligible(const fk_ctx *c) { return staged_ok(c) && c->G == 1 && !c->comm; }

// Partitions one piece and expands it into its own key array (st_keys[p], its cells' exclusive
// scan in st_cb[p]); the job's cell totals accumulate in st_total.  The first piece fixes the
// job's cells: its largest bin scaled by the job's size over the bytes mapped so far.
// Expands one piece's records (the chunk table at c->chunks, records at c->rsrc; bkm = k-mers per
// local bin) into its own key array (st_keys[p], its cells' exclusive scan in st_cb[p]); the job's
// cell totals accumulate in st_total.  `frac` = the piece's estimated fraction of the job (0:
// unknown).  The first piece fixes the job's cells: its largest bin scaled to the job.
static int staged_expand_chunks(fk_ctx *c, uint32_t nchunks, const std::vector<uint64_t> &bkm, double frac) {
    hipStream_t s = c->stream;
    const uint32_t p = c->st_np;
    uint64_t pk = 0, maxb = 0;
    for (uint64_t v : bkm) pk += v, maxb = std::max(maxb, v);
    if (pk == 0) return FK_OK;  // nothing to expand (the piece's records hold no k-mers)
    if (p == 0) {
        const double scale = frac > 0.0 ? std::max(1.0, 1.0 / frac) : 2.0;
        c->st_plan = sorted_plan(c, (uint64_t)((double)maxb * scale));
        if (!c->st_plan.tiered || !c->st_plan.two_level)
            return set_err(FK_E_STATE, "staged pieces need the tiered two-level count");
    }
    // every piece takes both levels (level 2 sizes its workgroups to the keys per super-cell: a 15 %
    // piece 0.75 ms against 1.14 for a one-pass scatter)
    SortedPlan pl = c->st_plan;
    HIP_TRY(hipEventRecord(c->st_ev[4 * p + 2], s));
    FK_TRY(sorted_expand(c, pl, nchunks, pk, c->st_keys[p], c->st_cb[p]));
    const uint64_t ncell_all = (uint64_t)c->nlb << c->st_plan.F;
    FK_TRY(ensure(c->st_total, ncell_all * 8));
    if (c->cut_side) {  // the job's cell totals on the cut's stream, while this piece is expanded
        HIP_TRY(hipStreamWaitEvent(c->tier_side, c->side_ev[2], 0));
        HIP_TRY(launch_add_u64(c->st_total.as<uint64_t>(), c->cell_total.as<uint64_t>(), ncell_all, p == 0,
                               c->tier_side));
    } else {
        HIP_TRY(launch_add_u64(c->st_total.as<uint64_t>(), c->cell_total.as<uint64_t>(), ncell_all, p == 0, s));
    }
    HIP_TRY(hipEventRecord(c->st_ev[4 * p + 3], s));
    c->st_kmers += pk;
    c->st_np = p + 1;
    htrace("staged: piece expanded");
    return FK_OK;
}

// One rank: partitions a piece of the mapped tiles by local bin, then expands it.
static int staged_expand(fk_ctx *c, const RecSrc &src, double frac) {
    const uint32_t p = c->st_np;
    if (p >= stage_maxp(c)) return set_err(FK_E_STATE, "more than %u staged pieces", stage_maxp(c));
    uint64_t nrecv = 0;
    std::vector<Chunk> chunks;
    std::vector<uint32_t> bcb;
    std::vector<uint64_t> bkm;
    FK_TRY(partition_src(c, src, nrecv, chunks, bcb, bkm, c->st_ev[4 * p], c->st_ev[4 * p + 1]));
    return staged_expand_chunks(c, (uint32_t)chunks.size(), bkm, frac);
}

// The job's count over the staged pieces: buckets over the summed cell totals, each bucket's keys
// read from every piece (BucketSrc pieces), the dense result and its bin offsets.
static int staged_count(fk_ctx *c) {
    const double t0 = now_ms();
    hipStream_t s = c->stream;
    const SortedPlan pl = c->st_plan;
    const uint32_t nlb = c->nlb;
    const uint64_t ncell_all = (uint64_t)nlb << pl.F;
    HIP_TRY(hipEventRecord(c->ev[6], s));
    std::swap(c->cell_total, c->st_total);  // the job's cell totals (st_total is rebuilt by the next job)
    FK_TRY(ensure(c->cell_base, (ncell_all + 1) * 8));
    // the bucket cut (this scan, sorted_count_buckets' flags, buckets and tiers) on the cut's stream when
    // the last piece is still being expanded on `s` (cut_side)
    const hipStream_t cs = c->cut_side ? c->tier_side : s;
    if (cs != s) HIP_TRY(hipStreamWaitEvent(cs, c->side_ev[2], 0));
    HIP_TRY(scan_excl_sum_u64(c->cell_total.as<uint64_t>(), c->cell_base.as<uint64_t>(), ncell_all,
                              c->cell_base.as<uint64_t>() + ncell_all, c->ws, cs));
    BucketSrc src{nullptr, pl.F};
    src.np = (int)c->st_np;
    for (uint32_t p = 0; p < c->st_np; ++p) {
        src.pk[p] = c->st_keys[p].as<uint64_t>();
        src.pcb[p] = c->st_cb[p].as<uint64_t>();
    }
    FK_TRY(sorted_count(c, pl, src, c->st_kmers));
    HIP_TRY(hipEventRecord(c->ev[7], s));
    c->h_bin_off.assign((size_t)nlb + 1, 0);
    if (c->pin_down.ensure(((size_t)nlb + 1) * 8)) return set_err(FK_E_NOMEM, "hipHostMalloc failed");
    HIP_TRY(hipMemcpyAsync(c->pin_down.p, c->bin_off.p, ((uint64_t)nlb + 1) * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    memcpy(c->h_bin_off.data(), c->pin_down.p, ((size_t)nlb + 1) * 8);
    resolve_distinct(c);
    htrace("staged: bin offsets read");
    double mp = 0.0, mx = 0.0;
    for (uint32_t p = 0; p < c->st_np; ++p) {
        mp += ev_ms(c->st_ev[4 * p], c->st_ev[4 * p + 1]);
        mx += ev_ms(c->st_ev[4 * p + 2], c->st_ev[4 * p + 3]);
    }
    c->stats.ms_partition = mp;
    c->stats.ms_count = mx + ev_ms(c->ev[6], c->ev[7]);
    c->stats.pieces_counted = c->st_np;
    c->stats.records_received = c->nrec;
    c->stats.distinct = c->distinct;
    c->stats.ms_total += now_ms() - t0;
    c->have_result = true;
    return FK_OK;
}

// One rank: stages the tiles mapped since the last piece once they cover a piece (fk_ingest).
// The fused map's fallback flag is read first: a flagged input is counted whole by fk_finish.
// Piece ends: with the job's size known (one fk_ingest call, or fk_ingest_reserve) and no
// FASTKMER_PIECE_BYTES, at the fractions st_cuts of it (the last piece -- expanded after the last byte
// lands -- is the smallest); jobs under 2 * MIN_PIECE are counted whole.  A streamed job of unknown
// size: every piece_bytes, at most three pieces before fk_finish stages the last one (with cuts: at
// most stage_maxp - 1).
static bool local_piece_due(const fk_ctx *c, uint64_t tiles) {
#ifndef FK_MIN_PIECE_MB
#define FK_MIN_PIECE_MB 256  // A/B builds: a piece holds >= half of it
#endif
    constexpr uint64_t MIN_PIECE = (uint64_t)FK_MIN_PIECE_MB << 20;
    if (c->st_np >= stage_maxp(c) - 1) return false;
    const uint64_t tile = fm_tile_bytes(FUSED_NT);
    if (c->job_bytes && !c->piece_bytes_set) {
        const std::vector<double> &cuts = local_cuts(c);
        if (c->job_bytes < 2 * MIN_PIECE || c->st_cut >= cuts.size()) return false;
        const uint64_t end = (uint64_t)(cuts[c->st_cut] * (double)c->job_bytes);
        return tiles * tile >= end && (tiles - c->tiles_counted) * tile >= MIN_PIECE / 2;
    }
    // every piece_bytes: at most four pieces (three before fk_finish), as the exchange's
    return c->st_np < 3 && (tiles - c->tiles_counted) * tile >= c->piece_bytes;
}

// The context's stream and scan workspace swapped for the staging stream's while a staging step is
// queued (the expansion code queues on c->stream).
struct StageStream {
    fk_ctx *c;
    explicit StageStream(fk_ctx *c_) : c(c_) {
        std::swap(c->stream, c->xstage);
        std::swap(c->ws, c->ws_x);
    }
    ~StageStream() {
        std::swap(c->stream, c->xstage);
        std::swap(c->ws, c->ws_x);
    }
};

// tiles: the tiles mapped once `mapped` (recorded on the map stream) has passed.  The piece is
// partitioned and expanded on the staging stream (StageStream), which fk_finish joins (xstage_ev).
static int local_maybe_piece(fk_ctx *c, uint64_t tiles, hipEvent_t mapped) {
    if (!staged_eligible(c) || c->pieces_void || !local_piece_due(c, tiles)) return FK_OK;
    StageStream ss_(c);
    hipStream_t s = c->stream;  // the staging stream
    HIP_TRY(hipStreamWaitEvent(s, mapped, 0));
    uint64_t h[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(h, c->counters.p, 32, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (h[2]) {
        c->pieces_void = true;
        return FK_OK;
    }
    const uint64_t t0 = c->tiles_counted, nt = tiles - t0;
    const RecSrc src = fused_src(c, t0, nt, nt * map_fused_tcap());
    c->tiles_counted = tiles;
    c->st_cut += 1;
    FK_TRY(staged_expand(c, src, c->job_bytes ? (double)(nt * fm_tile_bytes(FUSED_NT)) / (double)c->job_bytes : 0.0));
    HIP_TRY(hipEventRecord(c->xstage_ev, s));
    return FK_OK;
}

// ---------------------------------------------------------------------------
// multi-rank exchange inside the context (fk_comm_init*)
// ---------------------------------------------------------------------------

enum : uint64_t { XF_FINAL = 1, XF_RETRACT = 2 };

// Host arithmetic of one exchange step (fk_exchange_plan): byte offsets and sizes of the send
// blocks (destination-major, as the grouped emit writes them) and of the receive blocks
// (sender-major), and whether every sender has sent its last piece.
static int plan_step(uint32_t G, uint32_t L, const uint64_t *sent, const uint64_t *got, uint64_t rb, uint64_t *soff,
                     uint64_t *sbytes, uint64_t *roff, uint64_t *rbytes, bool *all_final) {
    const size_t msg = 2 * (size_t)L + 1;
    uint64_t so = 0, ro = 0;
    bool fin = true;
    for (uint32_t d = 0; d < G; ++d) {
        uint64_t ns = 0, nr = 0;
        for (uint32_t lb = 0; lb < L; ++lb) {
            ns += sent[d * msg + lb];
            nr += got[d * msg + lb];
        }
        const uint64_t fs = sent[d * msg + 2 * L], fr = got[d * msg + 2 * L];
        if ((fs | fr) & ~(XF_FINAL | XF_RETRACT)) return set_err(FK_E_INVALID, "exchange step: unknown flag bits");
        if ((fr & XF_RETRACT) && !(fr & XF_FINAL))
            return set_err(FK_E_INVALID, "exchange step: rank %u retracts outside its last piece", d);
        fin = fin && (fr & XF_FINAL);
        soff[d] = so;
        sbytes[d] = ns * rb;
        roff[d] = ro;
        rbytes[d] = nr * rb;
        so += ns * rb;
        ro += nr * rb;
    }
    *all_final = fin;
    return FK_OK;
}

FK_EXPORT int fk_exchange_plan(int32_t n_ranks, int32_t parts, const uint64_t *sent, const uint64_t *received,
                               uint64_t record_bytes, uint64_t *send_off, uint64_t *send_bytes, uint64_t *recv_off,
                               uint64_t *recv_bytes, int32_t *all_final) {
    if (n_ranks < 1 || parts < 0 || !sent || !received || !send_off || !send_bytes || !recv_off || !recv_bytes ||
        !all_final)
        return set_err(FK_E_INVALID, "bad argument");
    bool fin = false;
    FK_TRY(plan_step((uint32_t)n_ranks, (uint32_t)parts, sent, received, record_bytes, send_off, send_bytes, recv_off,
                     recv_bytes, &fin));
    *all_final = fin ? 1 : 0;
    return FK_OK;
}

static void xch_reset(fk_ctx *c) {
    c->xch = fk_ctx::Xch{};
}

// FK_E_NOMEM from an exported call: the message names what the context holds on the device, largest
// first, so an oversized job shows which of its arrays to size (or free) without a re-run.
static int note_held(fk_ctx *c, int rc) {
    if (rc != FK_E_NOMEM || !c) return rc;
    std::vector<std::pair<size_t, std::string>> v;
    auto add = [&](const char *name, const DevBuf &b) {
        if (b.bytes >= (64u << 20)) v.emplace_back(b.bytes, name);
    };
#define FK_HELD(b) add(#b, c->b)
    FK_HELD(fasta_own); FK_HELD(rec_hdr); FK_HELD(rec_pos); FK_HELD(rec_code); FK_HELD(records);
    FK_HELD(codes); FK_HELD(valid); FK_HELD(precs); FK_HELD(chunks); FK_HELD(lp); FK_HELD(mid);
    FK_HELD(scratch); FK_HELD(keys); FK_HELD(out_keys); FK_HELD(out_counts); FK_HELD(buckets);
    FK_HELD(flags); FK_HELD(flag_scan); FK_HELD(cell_total); FK_HELD(cell_base); FK_HELD(dense_keys);
    FK_HELD(dense_counts); FK_HELD(bucket_unique);
    FK_HELD(sp_keys); FK_HELD(sp_subs); FK_HELD(xsend); FK_HELD(xrecv);
    FK_HELD(gather_keys); FK_HELD(part.K); FK_HELD(part.KT); FK_HELD(dest.K); FK_HELD(dest.KT);
#undef FK_HELD
    std::vector<std::string> piece_names(STAGE_MAXP);
    for (int p = 0; p < STAGE_MAXP; ++p) {
        piece_names[p] = "st_keys[" + std::to_string(p) + "]";
        add(piece_names[p].c_str(), c->st_keys[p]);
    }
    std::sort(v.rbegin(), v.rend());
    size_t total = 0;
    for (const auto &e : v) total += e.first;
    std::string msg = g_err + "; held on the device: " + std::to_string(total >> 20) + " MiB in";
    for (size_t i = 0; i < v.size() && i < 12; ++i)
        msg += (i ? ", " : " ") + v[i].second + " " + std::to_string(v[i].first >> 20) + " MiB";
    g_err = msg;
    return rc;
}

static int comm_fail(fk_ctx *c, int rc) {
    note_held(c, rc);
    if (c->comm) c->comm->abort();  // peers blocked in a step return instead of waiting
    return rc;
}

static hipEvent_t xch_event(fk_ctx *c, size_t i) {
    while (c->xev.size() <= i) {
        hipEvent_t e = nullptr;
        if (hipEventCreate(&e) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        c->xev.push_back(e);
    }
    return c->xev[i];
}

// One exchange step; collective (every rank runs its steps in the same sequence, whatever each
// step carries).  src = this rank's records of the step (null: none): grouped by (destination,
// local bin) into the send ring, their per-part counts and `flags` all-to-all'ed, then the
// records posted on the comm stream (they move while the map stream goes on); the received
// blocks become segments of the count.  `expect` = records expected in all (sizes xrecv).
static int xch_step(fk_ctx *c, const RecSrc *src, uint64_t flags) {
    hipStream_t s = c->stream, cs = c->comm_stream;
    const uint32_t G = c->G, L = c->grp_nlb, nparts = G * L;
    const uint64_t rb = (uint64_t)c->W * 8;
    const size_t msg = 2 * (size_t)L + 1;
    std::vector<uint64_t> pr(nparts, 0), pk(nparts, 0);
    uint64_t piece_rec = 0;
    if (src && src->nrec && src->ntiles) {
        FK_TRY(part_count(c->dest, *src, 0, G, c->grp_table.as<uint32_t>(), nparts, c->ws, s));
        HIP_TRY(hipMemcpyAsync(pr.data(), c->dest.rec.p, (uint64_t)nparts * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(pk.data(), c->dest.kmer.p, (uint64_t)nparts * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        for (uint64_t v : pr) piece_rec += v;
    }
    if (piece_rec) {
        // send ring: earlier pieces are read by the comm stream; wrap around once it has drained
        if ((c->xch.send_used + piece_rec) * rb > c->xsend.bytes) {
            FK_TRY(comm_sync(c, cs));
            c->xch.send_used = 0;
            FK_TRY(ensure(c->xsend, piece_rec * rb * 2));
        }
        FK_TRY(part_scatter(c->dest, 0, G, c->grp_table.as<uint32_t>(), c->xsend.as<uint64_t>() + c->xch.send_used * c->W,
                            s));
        HIP_TRY(hipEventRecord(c->emit_ev, s));
    }
    std::vector<uint64_t> out((size_t)G * msg), in((size_t)G * msg);
    for (uint32_t d = 0; d < G; ++d) {
        for (uint32_t lb = 0; lb < L; ++lb) {
            out[d * msg + lb] = pr[(size_t)d * L + lb];
            out[d * msg + L + lb] = pk[(size_t)d * L + lb];
        }
        out[d * msg + 2 * L] = flags;
    }
    std::string err;
    if (c->comm->alltoall_u64(out.data(), in.data(), msg, cs, err))
        return set_err(FK_E_COMM, "exchange step %llu, counts: %s", (unsigned long long)c->xch.pieces, err.c_str());
    std::vector<uint64_t> soff(G), sbytes(G), roff(G), rbytes(G);
    bool all_final = false;
    FK_TRY(plan_step(G, L, out.data(), in.data(), rb, soff.data(), sbytes.data(), roff.data(), rbytes.data(), &all_final));
    uint64_t recv_rec = 0;
    for (uint32_t r = 0; r < G; ++r) recv_rec += rbytes[r] / rb;
    if ((c->xch.recv_used + recv_rec) * rb > c->xrecv.bytes) {
        // the received records stay until the count: grow, keeping them (sized for the whole input
        // once the first pieces show the records per FASTA byte)
        uint64_t want = c->xch.recv_used + recv_rec;
        if (c->xch.expect_bytes && c->xch.tiles_sent) {
            const double covered = (double)c->xch.tiles_sent * (double)fm_tile_bytes(FUSED_NT);
            want = std::max<uint64_t>(want, (uint64_t)((double)want * (double)c->xch.expect_bytes / covered * 1.1));
        }
        FK_TRY(comm_sync(c, cs));
        FK_TRY(comm_sync(c, c->xstage));  // staged expansions may still read the old buffer
        FK_TRY(grow_keep(c->xrecv, want * rb, c->xch.recv_used * rb, s));
    }
    const size_t step = (size_t)c->xch.pieces;
    hipEvent_t e0 = xch_event(c, 2 * step), e1 = xch_event(c, 2 * step + 1);
    if (!e0 || !e1) return set_err(FK_E_DEVICE, "hipEventCreate failed");
    if (piece_rec) HIP_TRY(hipStreamWaitEvent(cs, c->emit_ev, 0));
    HIP_TRY(hipEventRecord(e0, cs));
    if (c->comm->alltoallv(c->xsend.as<uint8_t>() + c->xch.send_used * rb, soff.data(), sbytes.data(),
                           c->xrecv.as<uint8_t>() + c->xch.recv_used * rb, roff.data(), rbytes.data(), cs, err))
        return set_err(FK_E_COMM, "exchange step %llu, records: %s", (unsigned long long)step, err.c_str());
    HIP_TRY(hipEventRecord(e1, cs));
    for (uint32_t r = 0; r < G; ++r) {
        const uint64_t *m = in.data() + (size_t)r * msg;
        if (m[2 * L] & XF_RETRACT) {  // the sender mapped again from scratch: its earlier pieces are void
            c->pieces_void = true;      // (and so are the piece counts that hold them)
            auto &v = c->xch.segs;
            v.erase(std::remove_if(v.begin(), v.end(), [&](const fk_ctx::XSeg &g) { return g.sender == (int32_t)r; }),
                    v.end());
        }
        if (!rbytes[r]) continue;
        fk_ctx::XSeg g;
        g.off = c->xch.recv_used + roff[r] / rb;
        g.sender = (int32_t)r;
        g.step = step;
        g.rec.assign(m, m + L);
        g.kmer.assign(m + L, m + 2 * L);
        c->xch.segs.push_back(std::move(g));
        if (r != (uint32_t)c->cfg.rank) c->xch.bytes_received += rbytes[r];
    }
    for (uint32_t d = 0; d < G; ++d)
        if (d != (uint32_t)c->cfg.rank) c->xch.bytes_sent += sbytes[d];
    c->xch.send_used += piece_rec;
    c->xch.recv_used += recv_rec;
    c->xch.pieces += 1;
    c->xch.open = true;
    c->xch.all_final = all_final;
    if (flags & XF_FINAL) c->xch.sent_final = true;
    return FK_OK;
}

// Ranges of every local bin over the received segments [s0, s1) (each segment holds its
// records bin after bin).
static int segment_ranges(fk_ctx *c, size_t s0, size_t s1, std::vector<std::vector<std::pair<uint64_t, uint64_t>>> &ranges,
                          std::vector<uint64_t> &bkm, uint64_t *nrecv) {
    const uint32_t nlb = c->nlb;
    ranges.assign(nlb, {});
    bkm.assign(nlb, 0);
    *nrecv = 0;
    for (size_t i = s0; i < s1; ++i) {
        const fk_ctx::XSeg &g = c->xch.segs[i];
        uint64_t off = g.off;
        for (uint32_t lb = 0; lb < c->grp_nlb; ++lb) {
            const uint64_t n = g.rec[lb];
            if (n && lb >= nlb) return set_err(FK_E_INVALID, "records for local bin %u of %u", lb, nlb);
            if (n) {
                ranges[lb].push_back({off, off + n});
                bkm[lb] += g.kmer[lb];
                *nrecv += n;
            }
            off += n;
        }
    }
    return FK_OK;
}

// With a communicator and staged pieces: expands the received segments [segs_counted, s1) as one
// staged piece (they arrive grouped by local bin: no partition), once the comm stream has
// delivered them.  `frac` = their estimated fraction of what this rank receives in the job.
static int xch_stage_segments(fk_ctx *c, size_t s1, double frac) {
    if (s1 <= c->segs_counted) return FK_OK;
    const uint32_t p = c->st_np;
    if (p >= stage_maxp(c)) return set_err(FK_E_STATE, "more than %u staged pieces", stage_maxp(c));
    StageStream ss_(c);
    hipStream_t s = c->stream;  // the staging stream
    // its earlier work (behind earlier steps' transfers) is done: bounded with a communicator
    FK_TRY(comm_sync(c, s));
    const uint64_t step = c->xch.segs[s1 - 1].step;
    HIP_TRY(hipStreamWaitEvent(s, c->xev[2 * step + 1], 0));
    std::vector<std::vector<std::pair<uint64_t, uint64_t>>> ranges;
    std::vector<uint64_t> bkm;
    uint64_t nrecv = 0;
    FK_TRY(segment_ranges(c, c->segs_counted, s1, ranges, bkm, &nrecv));
    c->segs_counted = s1;
    std::vector<Chunk> chunks;
    std::vector<uint32_t> bcb;
    build_chunks(c->nlb, ranges, chunks, bcb);
    HIP_TRY(hipEventRecord(c->st_ev[4 * p], s));
    FK_TRY(upload_chunks(c, chunks, bcb));
    HIP_TRY(hipEventRecord(c->st_ev[4 * p + 1], s));
    c->rsrc = c->xrecv.as<uint64_t>();
    return staged_expand_chunks(c, (uint32_t)chunks.size(), bkm, frac);
}

// Received records of this job so far / expected in all (estimated from the share of the input
// sent so far; 0 when the input's size is unknown).
static double xch_recv_frac(const fk_ctx *c, uint64_t recs) {
    if (!c->xch.expect_bytes || !c->xch.tiles_sent || !c->xch.recv_used) return 0.0;
    const double sent = (double)c->xch.tiles_sent * (double)fm_tile_bytes(FUSED_NT);
    const double est = (double)c->xch.recv_used * (double)c->xch.expect_bytes / sent;
    return est > 0.0 ? std::min(1.0, (double)recs / est) : 0.0;
}

// Staged: the segments received before this step are expanded once they hold about 1 / STAGE_MAXP
// of the job (every step when its size is unknown), at most STAGE_MAXP - 1 times before fk_finish.
static int xch_maybe_stage(fk_ctx *c, size_t s1) {
    // (at most four pieces: the exchange's cuts are xst_cuts)
    if (c->st_np >= std::min<uint32_t>(stage_maxp(c), 4) - 1 || s1 <= c->segs_counted) return FK_OK;
    uint64_t recs = 0, before = 0;
    for (size_t i = 0; i < s1; ++i)
        for (uint64_t n : c->xch.segs[i].rec) (i < c->segs_counted ? before : recs) += n;
    const double frac = xch_recv_frac(c, recs);
    // a piece ends once the received records reach the next cut of the job (st_cuts, as the local
    // path's pieces): the last piece -- expanded after the last byte -- is the smallest.  (Staging at
    // every quarter left ~30 % of a 6.25 GB rank for fk_finish: 61.7 ms after it against 47.7 for
    // the local path, profiles/r04c_xch_tail.txt.)
    if (frac > 0.0) {
        if (c->st_np >= (uint32_t)c->xst_cuts.size()) return FK_OK;
        if (xch_recv_frac(c, before + recs) < c->xst_cuts[c->st_np]) return FK_OK;
    }
    return xch_stage_segments(c, s1, frac);
}

// fk_ingest: sends the tiles mapped since the last piece once they cover a piece.  The fused
// map's fallback flag is read first: a flagged input is mapped again in fk_finish and sent
// whole, retracting the pieces sent so far.
static int xch_maybe_piece(fk_ctx *c) {
    if (c->xch.stop_pieces || c->xch.sent_final) return FK_OK;
    const uint64_t tile = fm_tile_bytes(FUSED_NT);
    if ((c->pm_tiles - c->xch.tiles_sent) * tile < c->piece_bytes) return FK_OK;
    uint64_t h[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(h, c->counters.p, 32, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (h[2]) {
        c->xch.stop_pieces = true;
        return FK_OK;
    }
    const uint64_t t0 = c->xch.tiles_sent, nt = c->pm_tiles - t0;
    const RecSrc src = fused_src(c, t0, nt, nt * map_fused_tcap());
    c->xch.tiles_sent = c->pm_tiles;
    const int rc = xch_step(c, &src, 0);
    if (rc) return comm_fail(c, rc);
    // the received segments are expanded (staged) on the staging stream as soon as their transfer
    // ends, this step's included, while the map stream goes on
    if (staged_ok(c) && !c->pieces_void) FK_TRY(xch_maybe_stage(c, c->xch.segs.size()));
    return FK_OK;
}

// fk_finish with a communicator: the last piece, the closing steps, then the count of every
// received segment.
static int finish_exchange(fk_ctx *c) {
    const double t0 = now_ms();
    hipStream_t s = c->stream, cs = c->comm_stream;
    const bool pieced = c->xch.tiles_sent > 0;
    const uint64_t tiles_sent = c->xch.tiles_sent;
    FK_TRY(map_records(c));
    RecSrc src;
    uint64_t flags = XF_FINAL;
    if (c->rec_tiled && pieced && !c->xch.stop_pieces && tiles_sent <= c->rec_tiles) {
        const uint64_t nt = c->rec_tiles - tiles_sent;
        src = fused_src(c, tiles_sent, nt, nt * map_fused_tcap());
    } else {
        src = map_src(c);
        if (pieced) flags |= XF_RETRACT;
    }
    c->mapped = true;
    int rc = xch_step(c, &src, flags);
    const size_t last_step = (size_t)c->xch.pieces - 1;
    while (!rc && !c->xch.all_final) rc = xch_step(c, nullptr, XF_FINAL);
    // every transfer of the job has been posted; the host waits for them here, bounded, so that none
    // of the count's host waits below can block on a peer that died (FK_E_COMM instead)
    if (!rc) rc = comm_sync(c, cs);
    if (rc) return comm_fail(c, rc);
    HIP_TRY(hipEventRecord(c->ev[4], cs));  // every rank's records have landed
    HIP_TRY(hipStreamWaitEvent(s, c->ev[4], 0));
    HIP_TRY(hipEventRecord(c->xstage_ev, c->xstage));  // and the staged expansions queued so far are done
    HIP_TRY(hipStreamWaitEvent(s, c->xstage_ev, 0));
    uint64_t nrecv = 0;
    for (const auto &g : c->xch.segs)
        for (uint64_t n : g.rec) nrecv += n;
    if (c->st_np && !c->pieces_void) {
        // staged: the segments not yet expanded, then one count over every piece
        if (c->segs_counted < c->xch.segs.size()) {
            uint64_t recs = 0;
            for (size_t i = c->segs_counted; i < c->xch.segs.size(); ++i)
                for (uint64_t n : c->xch.segs[i].rec) recs += n;
            FK_TRY(xch_stage_segments(c, c->xch.segs.size(), nrecv ? (double)recs / (double)nrecv : 0.0));
            HIP_TRY(hipEventRecord(c->xstage_ev, c->xstage));
            HIP_TRY(hipStreamWaitEvent(s, c->xstage_ev, 0));
        }
        FK_TRY(staged_count(c));
    } else {
        std::vector<std::vector<std::pair<uint64_t, uint64_t>>> ranges;
        std::vector<uint64_t> bkm;
        FK_TRY(segment_ranges(c, 0, c->xch.segs.size(), ranges, bkm, &nrecv));
        FK_TRY(reduce_ranges(c, c->xrecv.as<uint64_t>(), nrecv, ranges, bkm, t0));
    }
    pieces_reset(c);
    // exchange figures (every transfer has completed: the count waited for them)
    double ms = 0.0;
    for (size_t i = 0; i < (size_t)c->xch.pieces; ++i) ms += ev_ms(c->xev[2 * i], c->xev[2 * i + 1]);
    c->stats.xch_steps = c->xch.pieces;
    c->stats.xch_bytes_sent = c->xch.bytes_sent;
    c->stats.xch_bytes_received = c->xch.bytes_received;
    c->stats.ms_exchange = ms;
    c->stats.ms_exchange_tail = ev_ms(c->xev[2 * last_step], c->xev[2 * ((size_t)c->xch.pieces - 1) + 1]);
    c->stats.records_received = nrecv;
    xch_reset(c);
    return FK_OK;
}

static int finish_local(fk_ctx *c);

FK_EXPORT int fk_finish(fk_ctx *c) {
    htrace("fk_finish: enter");
    if (!c) return set_err(FK_E_INVALID, "null ctx");
    if (c->comm) {
        DeviceGuard dg_(c->device);
        const int rc = finish_exchange(c);
        return rc ? comm_fail(c, rc) : rc;  // collective: a failed rank fails the group
    }
    return note_held(c, finish_local(c));
}

static int finish_local(fk_ctx *c) {
    if (c->G != 1)
        return set_err(FK_E_STATE, "fk_finish over %u ranks needs a communicator (fk_comm_init); or use "
                                   "fk_map/fk_map_emit/fk_reduce", c->G);
    FK_TRY(fk_map(c, nullptr));  // joins the staging stream first
    DeviceGuard dg_(c->device);
    if (c->st_np && c->rec_tiled && !c->pieces_void && c->tiles_counted <= c->rec_tiles) {
        // staged pieces were expanded while the input landed: the last piece, then one count
#ifndef FK_CUT_SIDE
#define FK_CUT_SIDE 1  // A/B builds: -DFK_CUT_SIDE=0 the bucket cut after the last piece's expansion
#endif
        // the job's bucket cut needs the last piece's cell totals, not its keys: it runs on the side
        // stream while the piece's two expansion levels run on `stream`
        int rc = FK_OK;
        c->cut_side = FK_CUT_SIDE && c->tier_side && c->rec_tiles > c->tiles_counted;
        // the cut's stream starts after everything queued so far (re-recorded once the last piece's cell
        // offsets are scanned; a piece without k-mers records nothing more)
        if (c->cut_side) HIP_TRY(hipEventRecord(c->side_ev[2], c->stream));
        if (c->rec_tiles > c->tiles_counted) {
            const uint64_t t0 = c->tiles_counted, nt = c->rec_tiles - t0;
            rc = staged_expand(c, fused_src(c, t0, nt, nt * map_fused_tcap()),
                               c->job_bytes ? (double)(nt * fm_tile_bytes(FUSED_NT)) / (double)c->job_bytes : 0.0);
        }
        if (rc == FK_OK) rc = staged_count(c);
        if (c->cut_side) (void)hipStreamSynchronize(c->tier_side);
        c->cut_side = false;
        FK_TRY(rc);
        pieces_reset(c);
        return FK_OK;
    }
    pieces_reset(c);
    return reduce_src(c, map_src(c));
}

static int attach_comm(fk_ctx *c, fk::Comm *comm) {
    DeviceGuard dg_(c->device);
    if (!c->comm_stream) HIP_TRY(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
    if (!c->xstage) HIP_TRY(hipStreamCreateWithFlags(&c->xstage, hipStreamNonBlocking));
    if (!c->xstage_ev) HIP_TRY(hipEventCreateWithFlags(&c->xstage_ev, hipEventDisableTiming));
    if (!c->emit_ev) HIP_TRY(hipEventCreateWithFlags(&c->emit_ev, hipEventDisableTiming));
    c->comm = comm;
    if (!c->piece_bytes_set) c->piece_bytes = 1ull << 30;
    FK_TRY(fk_set_grouped_emit(c, 1));  // records leave grouped by (owner rank, local bin)
    xch_reset(c);
    return FK_OK;
}

FK_EXPORT int fk_comm_unique_id(uint8_t *id) {
    if (!id) return set_err(FK_E_INVALID, "null argument");
    std::string err;
    if (fk::comm_unique_id(id, err)) return set_err(FK_E_DEVICE, "%s", err.c_str());
    return FK_OK;
}

FK_EXPORT int fk_comm_init(fk_ctx *c, const uint8_t *id) {
    if (!c || !id) return set_err(FK_E_INVALID, "null argument");
    if (c->comm) return set_err(FK_E_STATE, "the context already has a communicator");
    DeviceGuard dg_(c->device);
    std::string err;
    fk::Comm *comm = fk::comm_create_rccl(id, (int)c->G, c->cfg.rank, c->device, err);
    if (!comm) return set_err(FK_E_DEVICE, "%s", err.c_str());
    const int rc = attach_comm(c, comm);
    if (rc) {
        delete comm;
        c->comm = nullptr;
    }
    return rc;
}

FK_EXPORT int fk_comm_init_local(fk_ctx **ctxs, int32_t n) {
    if (!ctxs || n < 1) return set_err(FK_E_INVALID, "bad argument");
    std::vector<int> devs(n);
    for (int32_t r = 0; r < n; ++r) {
        fk_ctx *c = ctxs[r];
        if (!c) return set_err(FK_E_INVALID, "null context %d", r);
        if (c->G != (uint32_t)n || c->cfg.rank != r)
            return set_err(FK_E_INVALID, "context %d has rank %d of %u; expected rank %d of %d", r, c->cfg.rank, c->G,
                           r, n);
        if (c->comm) return set_err(FK_E_STATE, "context %d already has a communicator", r);
        devs[r] = c->device;
    }
    std::vector<fk::Comm *> comms(n, nullptr);
    std::string err;
    if (fk::comm_create_local(n, devs.data(), comms.data(), err)) return set_err(FK_E_DEVICE, "%s", err.c_str());
    for (int32_t r = 0; r < n; ++r) {
        const int rc = attach_comm(ctxs[r], comms[r]);
        if (rc) {
            for (int32_t q = 0; q < n; ++q) {
                if (ctxs[q]->comm == comms[q]) ctxs[q]->comm = nullptr;
                delete comms[q];
            }
            return rc;
        }
    }
    return FK_OK;
}

FK_EXPORT const char *fk_comm_transport(const fk_ctx *c) { return c && c->comm ? c->comm->kind() : ""; }

FK_EXPORT int fk_comm_allreduce_u64(fk_ctx *c, uint64_t *v, size_t n) {
    if (!c || (!v && n)) return set_err(FK_E_INVALID, "null argument");
    if (!c->comm) return set_err(FK_E_STATE, "fk_comm_allreduce_u64 needs a communicator (fk_comm_init*)");
    DeviceGuard dg_(c->device);
    std::string err;
    if (c->comm->allreduce_sum_u64(v, n, c->comm_stream, err)) return comm_fail(c, set_err(FK_E_COMM, "%s", err.c_str()));
    return FK_OK;
}

// ---- size-aware placement on the library's exchange (useCustomPartitioner, SBKC:1023-1026 and
// MultiprocessorSchedulingPartitioner.scala:35-69): every rank maps a sample of its input (no
// exchange), the per-bin k-mer totals are summed over the ranks (the reduceByKey of :1024), the
// LPT placement is computed identically on every rank and installed for the job's exchange.
static int sample_bin_kmers(fk_ctx *c, const uint8_t *sample, size_t n, std::vector<uint64_t> &sizes) {
    if (c->comm && c->xch.open) return set_err(FK_E_STATE, "bin placement inside a job's exchange");
    sizes.assign((size_t)c->Bc, 0);
    fk::Comm *comm = c->comm;
    c->comm = nullptr;  // the sample is mapped here, never exchanged
    int rc = n ? ingest_impl(c, sample, n, 1) : FK_OK;
    if (!rc && n) rc = map_records(c);
    if (!rc && n && c->nrec) {
        rc = part_count(c->binhist, map_src(c), 1, 1, nullptr, (uint32_t)c->Bc, c->ws, c->stream);
        if (!rc) {
            hipError_t e = hipMemcpyAsync(sizes.data(), c->binhist.kmer.p, (uint64_t)c->Bc * 8, hipMemcpyDeviceToHost,
                                          c->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
            if (e != hipSuccess) rc = set_err(FK_E_DEVICE, "sample histogram: %s", hipGetErrorString(e));
        }
    }
    c->comm = comm;
    c->ingest_fresh = true;
    c->mapped = false;
    c->have_result = false;
    return rc;
}

static int balance_from_sample(fk_ctx *c, const uint8_t *sample, size_t n) {
    DeviceGuard dg_(c->device);
    std::vector<uint64_t> sizes;
    FK_TRY(sample_bin_kmers(c, sample, n, sizes));
    if (c->comm) {
        std::string err;
        if (c->comm->allreduce_sum_u64(sizes.data(), sizes.size(), c->comm_stream, err))
            return set_err(FK_E_COMM, "bin size all-reduce: %s", err.c_str());
    }
    std::vector<int32_t> owner((size_t)c->Bc);
    FK_TRY(fk_lpt_owners(sizes.data(), c->Bc, (int32_t)c->G, owner.data()));
    return fk_set_bin_owners(c, owner.data(), nullptr);
}

FK_EXPORT int fk_balance_bins(fk_ctx *c, const uint8_t *sample, size_t n) {
    if (!c || (!sample && n)) return set_err(FK_E_INVALID, "null argument");
    const int rc = balance_from_sample(c, sample, n);
    return rc && c->comm ? comm_fail(c, rc) : rc;
}

// The sample of a file split: `fraction` of the rank's split as evenly spaced blocks of whole
// records (sequenceType 0) or of sequence (1, each block one record), the reference's
// sample(false, 0.01) of SBKC:1024 taken as blocks of the rank's own input.
static int split_sample(const char *path, int32_t world, int32_t rank, int32_t k, int32_t seq, double fraction,
                        std::vector<uint8_t> &out) {
    out.clear();
    Fd f;
    uint64_t size = 0;
    SplitPlan plan;
    FK_TRY(open_split(path, world, rank, k, seq, f, size, plan));
    if (plan.total == 0 || fraction <= 0.0) return FK_OK;
    std::vector<uint8_t> piece;
    std::string err;
    if (fraction >= 1.0) {
        out.resize(plan.total);
        if (read_split(f.fd, size, plan, 0, plan.total, out.data(), err)) return set_err(FK_E_IO, "%s", err.c_str());
        return FK_OK;
    }
    constexpr uint64_t BLOCK = 1ull << 20;
    const uint64_t want = std::max<uint64_t>((uint64_t)((double)plan.total * fraction), 1);
    const uint64_t nblk = std::max<uint64_t>(1, (want + BLOCK - 1) / BLOCK);
    const uint64_t blk = std::min<uint64_t>(plan.total, std::max<uint64_t>(4096, want / nblk));
    std::vector<uint8_t> buf;
    for (uint64_t i = 0; i < nblk; ++i) {
        const uint64_t at = plan.total * i / nblk, len = std::min(blk, plan.total - at);
        buf.resize(len);
        if (read_split(f.fd, size, plan, at, len, buf.data(), err)) return set_err(FK_E_IO, "%s", err.c_str());
        if (seq == 0) {  // whole records: from the first '>' opening a line to the last record start
            size_t a = 0;
            while (a < buf.size() && !(buf[a] == '>' && (a == 0 ? at == 0 : buf[a - 1] == '\n'))) ++a;
            size_t e = buf.size();
            if (at + len < plan.total) {
                while (e > a + 1 && !(buf[e - 1] == '>' && buf[e - 2] == '\n')) --e;
                e = e > a + 1 ? e - 1 : a;
            }
            out.insert(out.end(), buf.begin() + a, buf.begin() + e);
        } else {  // a block of the sequence as one record
            // the block's first line is dropped (it may be the tail of a header line: the block
            // started inside it, or the file's first header), and the block ends at the next
            // header line (a later record's name is not sequence)
            // -- unless the block holds no newline at all: it lies inside one sequence line (an unwrapped
            // record), and the whole block is sequence (a header line of a megabyte is not a FASTA)
            size_t a = 0;
            while (a < buf.size() && buf[a] != '\n') ++a;
            if (a == buf.size())
                a = (at == 0 && !buf.empty() && buf[0] == '>') ? buf.size() : 0;
            else
                a += 1;
            size_t e = a;
            while (e < buf.size() && !(buf[e] == '>' && e > 0 && buf[e - 1] == '\n')) ++e;
            if (e <= a) continue;
            const uint8_t h[3] = {'\n', '>', '\n'};
            out.insert(out.end(), h, h + 3);
            out.insert(out.end(), buf.begin() + a, buf.begin() + e);
        }
    }
    if (seq == 1) out.push_back('\n');
    if (seq == 1 && !out.empty()) out.erase(out.begin());  // the first block's header starts the input
    return FK_OK;
}

FK_EXPORT int fk_balance_bins_file(fk_ctx *c, const char *path, int32_t world, int32_t rank, double fraction) {
    if (!c || !path) return set_err(FK_E_INVALID, "null argument");
    std::vector<uint8_t> sample;
    int rc = check_split_rank(c, world, rank, "fk_balance_bins_file");
    if (!rc) rc = split_sample(path, world, rank, c->cfg.k, c->cfg.sequence_type, fraction, sample);
    if (!rc) rc = balance_from_sample(c, sample.data(), sample.size());
    return rc && c->comm ? comm_fail(c, rc) : rc;
}

// ---------------------------------------------------------------------------
// results
// ---------------------------------------------------------------------------

static bool owns(const fk_ctx *c, int32_t b) {
    if (b < 0 || b >= c->Bc) return false;
    return c->custom_owners ? c->h_owner[b] == c->cfg.rank : (uint32_t)b % c->G == (uint32_t)c->cfg.rank;
}
static uint32_t local_bin(const fk_ctx *c, int32_t b) { return c->custom_owners ? c->h_bin_lbin[b] : (uint32_t)b / c->G; }

FK_EXPORT int fk_bin_sizes(fk_ctx *c, uint64_t *out) {
    if (!c || !out) return set_err(FK_E_INVALID, "null argument");
    if (!c->have_result) return set_err(FK_E_STATE, "no result: call fk_finish or fk_reduce first");
    for (int32_t b = 0; b < c->Bc; ++b) {
        if (owns(c, b)) {
            const uint32_t lb = local_bin(c, b);
            out[b] = c->h_bin_off[lb + 1] - c->h_bin_off[lb];
        } else {
            out[b] = 0;
        }
    }
    return FK_OK;
}

// A bucket-major result made dense (fk_write_bins): the buckets' outputs compacted in bin order.
static int materialize_dense(fk_ctx *c) {
    if (!c->gapped || c->dense_ready) return FK_OK;
    hipStream_t s = c->stream;
    FK_TRY(ensure(c->dense_keys, c->distinct * 8 * c->KW));
    FK_TRY(ensure(c->dense_counts, c->distinct * 4));
    HIP_TRY(launch_bucket_compact(c->KW, c->res_keys, c->out_counts.as<uint32_t>(), c->buckets.as<Bucket>(),
                                  c->res_nbuckets, c->dense_off.as<uint64_t>(), c->dense_keys.as<uint64_t>(),
                                  c->dense_counts.as<uint32_t>(), s));
    HIP_TRY(hipStreamSynchronize(s));
    c->dense_ready = true;
    return FK_OK;
}

// One local bin of a bucket-major result into dst (device): its buckets [q0, q1) -- the bin's first
// cell starts a bucket, so q0 = flag_scan[lb << F] -- compacted at dense_off[q] - dense_off[q0].
static int gather_bin(fk_ctx *c, uint32_t lb, uint64_t *dkeys, uint32_t *dcounts) {
    hipStream_t s = c->stream;
    uint64_t q[2] = {0, c->res_nbuckets};
    const uint64_t *fs = c->res_fs;
    HIP_TRY(hipMemcpyAsync(&q[0], fs + ((uint64_t)lb << c->res_F), 8, hipMemcpyDeviceToHost, s));
    if (lb + 1 < c->nlb) HIP_TRY(hipMemcpyAsync(&q[1], fs + ((uint64_t)(lb + 1) << c->res_F), 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const uint64_t d0 = c->h_bin_off[lb];
    if (q[1] > q[0])
        HIP_TRY(launch_bucket_compact(c->KW, c->res_keys, c->out_counts.as<uint32_t>(), c->buckets.as<Bucket>() + q[0],
                                      q[1] - q[0], c->dense_off.as<uint64_t>() + q[0], dkeys - d0 * c->KW, dcounts - d0, s));
    return FK_OK;
}

FK_EXPORT int fk_get_bin(fk_ctx *c, int32_t bin, uint64_t *keys, uint32_t *counts, size_t cap, size_t *n) {
    if (!c || !n) return set_err(FK_E_INVALID, "null argument");
    DeviceGuard dg_(c->device);
    if (!c->have_result) return set_err(FK_E_STATE, "no result: call fk_finish or fk_reduce first");
    if (bin < 0 || bin >= c->Bc) return set_err(FK_E_RANGE, "bin %d out of [0, %d)", bin, c->Bc);
    if (!owns(c, bin)) {
        *n = 0;
        return FK_OK;
    }
    const uint32_t lb = local_bin(c, bin);
    const uint64_t b0 = c->h_bin_off[lb], cnt = c->h_bin_off[lb + 1] - b0;
    *n = (size_t)cnt;
    if (cnt == 0) return FK_OK;
    if (cap < cnt) return set_err(FK_E_RANGE, "bin %d has %llu k-mers, buffer holds %zu", bin, (unsigned long long)cnt, cap);
    if (c->gapped && !c->dense_ready) {
        FK_TRY(ensure(c->gather_keys, cnt * 8 * c->KW));
        FK_TRY(ensure(c->gather_counts, cnt * 4));
        FK_TRY(gather_bin(c, lb, c->gather_keys.as<uint64_t>(), c->gather_counts.as<uint32_t>()));
        if (keys)
            HIP_TRY(hipMemcpyAsync(keys, c->gather_keys.p, cnt * 8 * c->KW, hipMemcpyDeviceToHost, c->stream));
        if (counts) HIP_TRY(hipMemcpyAsync(counts, c->gather_counts.p, cnt * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        return FK_OK;
    }
    if (keys)
        HIP_TRY(hipMemcpy(keys, c->dense_keys.as<uint64_t>() + b0 * c->KW, cnt * 8 * c->KW, hipMemcpyDeviceToHost));
    if (counts) HIP_TRY(hipMemcpy(counts, c->dense_counts.as<uint32_t>() + b0, cnt * 4, hipMemcpyDeviceToHost));
    return FK_OK;
}

// Test hooks of the failure semantics (fastkmer.h): hold every stream the context's collectives run
// on with a kernel spinning on a host-mapped flag, so the next collective waits on a stream that does
// not drain; release it from any thread.
FK_EXPORT int fk_debug_comm_hold(fk_ctx *c, int32_t max_seconds) {
    if (!c || max_seconds < 1) return set_err(FK_E_INVALID, "bad argument");
    if (!c->comm) return set_err(FK_E_STATE, "fk_debug_comm_hold needs a communicator (fk_comm_init*)");
    DeviceGuard dg_(c->device);
    if (!c->hold_flag) {
        void *p = nullptr;
        HIP_TRY(hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent));
        c->hold_flag = static_cast<uint32_t *>(p);
    }
    __atomic_store_n(c->hold_flag, 0u, __ATOMIC_RELEASE);
    void *dflag = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&dflag, c->hold_flag, 0));
    // wall-clock ticks of max_seconds: the attribute is in kHz (100 MHz on gfx950); a rate reported
    // below that bounds the hold by 100 MHz ticks instead (longer, never shorter, than asked)
    int khz = 0;
    HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
    const uint64_t ticks = (uint64_t)max_seconds * (uint64_t)std::max(khz, 100000) * 1000ull;
    const hipStream_t cs2 = c->comm->counts_stream();
    for (hipStream_t st : {c->comm_stream, cs2})
        if (st) HIP_TRY(launch_hold_stream(static_cast<const uint32_t *>(dflag), ticks, st));
    return FK_OK;
}

FK_EXPORT int fk_debug_fingerprint_bits(int32_t device, int32_t bits) {
    DeviceGuard dg_(device);
    HIP_TRY(set_fingerprint_bits(bits));
    return FK_OK;
}

FK_EXPORT int fk_debug_comm_held(fk_ctx *c) {
    if (!c || !c->comm_stream) return 0;
    DeviceGuard dg_(c->device);
    const hipError_t e = hipStreamQuery(c->comm_stream);
    if (e != hipErrorNotReady) (void)hipGetLastError();
    return e == hipErrorNotReady ? 1 : 0;
}

FK_EXPORT int fk_debug_comm_release(fk_ctx *c) {
    if (!c) return set_err(FK_E_INVALID, "null ctx");
    if (c->hold_flag) __atomic_store_n(c->hold_flag, 1u, __ATOMIC_RELEASE);
    return FK_OK;
}

// ---------------------------------------------------------------------------
// test hook: one bucket through the wave tier (k_bucket_count64_wave / k_bucket_count128_wave)
// ---------------------------------------------------------------------------
FK_EXPORT int fk_debug_wave_count(int32_t device, int32_t k, int32_t F, uint32_t c0, uint32_t c1, int32_t slots,
                                  const uint64_t *keys, uint32_t n, uint64_t *out_keys, uint32_t *out_counts,
                                  uint32_t *n_out) {
    if (!keys || !out_keys || !out_counts || !n_out || k < 1 || k > 63 || F < 1 || F > MAX_FINE_BITS || c1 <= c0 ||
        c1 > (1u << F))
        return set_err(FK_E_INVALID, "bad argument");
    const int KW = k <= 32 ? 1 : 2;
    const uint32_t cap = KW == 1 ? WAVE_BUCKET_CAP : WAVE128_BUCKET_CAP;
    if (n == 0 || n > cap) return set_err(FK_E_RANGE, "a wave bucket holds 1..%u keys", cap);
    if (slots != (int32_t)(KW == 1 ? WAVE_SLOTS : 384))
        return set_err(FK_E_INVALID, "slots: %u (k <= 32) or 384 (k > 32)", WAVE_SLOTS);
    const int sh = 2 * k - F;
    for (uint32_t i = 0; i < n; ++i) {  // every key inside the bucket's cells
        const uint64_t hi = KW == 1 ? 0 : keys[2 * i], lo = KW == 1 ? keys[i] : keys[2 * i + 1];
        const uint64_t cell = sh >= 64 ? (hi >> (sh - 64)) : (sh == 0 ? lo : ((hi << (64 - sh)) | (lo >> sh)));
        if ((KW == 1 && k < 32 && (lo >> (2 * k)) != 0) || cell < c0 || cell >= c1)
            return set_err(FK_E_RANGE, "key %u lies outside cells [%u, %u)", i, c0, c1);
    }
    DeviceGuard dg_(device);
    DevBuf dk, dok, doc, du, db;
    FK_TRY(ensure(dk, (uint64_t)n * 8 * KW));
    FK_TRY(ensure(dok, (uint64_t)n * 8 * KW));
    FK_TRY(ensure(doc, (uint64_t)n * 4));
    FK_TRY(ensure(du, 16));
    FK_TRY(ensure(db, sizeof(Bucket)));
    const Bucket b{0, n, 0, c0, c1};
    int rc = FK_OK;
    hipError_t e = hipMemcpy(dk.p, keys, (uint64_t)n * 8 * KW, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(db.p, &b, sizeof(Bucket), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = KW == 1 ? launch_bucket_count64_wave(BucketSrc{dk.as<uint64_t>(), F}, db.as<Bucket>(), 1, k, dok.as<uint64_t>(),
                                                 doc.as<uint32_t>(), du.as<uint64_t>(), nullptr, nullptr)
                    : launch_bucket_count128_wave(BucketSrc{dk.as<uint64_t>(), F}, db.as<Bucket>(), 1, k, dok.as<uint64_t>(),
                                                  doc.as<uint32_t>(), du.as<uint64_t>(), nullptr);
    uint64_t U = 0;
    if (e == hipSuccess) e = hipMemcpy(&U, du.p, 8, hipMemcpyDeviceToHost);
    if (e == hipSuccess && U <= n) e = hipMemcpy(out_keys, dok.p, U * 8 * KW, hipMemcpyDeviceToHost);
    if (e == hipSuccess && U <= n) e = hipMemcpy(out_counts, doc.p, U * 4, hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = set_err(FK_E_DEVICE, "%s", hipGetErrorString(e));
    else if (U > n) rc = set_err(FK_E_INVALID, "bucket reported %llu distinct keys of %u", (unsigned long long)U, n);
    *n_out = (uint32_t)U;
    release(dk), release(dok), release(doc), release(du), release(db);
    return rc;
}

// measurement hook (a library built with -DFK_PROBES; FK_E_STATE otherwise): the fused map's
// per-phase wave cycles (s_memtime) summed over every launch since the last reset
FK_EXPORT int fk_debug_map_cycles(uint64_t *out16, int32_t reset) {
    if (!out16) return set_err(FK_E_INVALID, "null argument");
    const hipError_t e = map_fused_cycles(reinterpret_cast<unsigned long long *>(out16), reset != 0);
    if (e == hipErrorNotSupported) {
        (void)hipGetLastError();
        return set_err(FK_E_STATE, "phase stamps exist only in a library built with -DFK_PROBES");
    }
    HIP_TRY(e);
    return FK_OK;
}

FK_EXPORT int fk_get_stats(fk_ctx *c, fk_stats *out) {
    if (!c || !out) return set_err(FK_E_INVALID, "null argument");
    *out = c->stats;
    return FK_OK;
}

static int mkdir_p(const std::string &path) {
    std::string cur;
    for (size_t i = 0; i < path.size(); ++i) {
        cur.push_back(path[i]);
        if ((path[i] == '/' && i > 0) || i + 1 == path.size()) {
            if (mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return -1;
        }
    }
    return 0;
}

// Bin files (writers SBKC:550-606 / 715-734): the text is formatted on the
// device (fk_format.inc), copied to the host once and written one file per bin.
FK_EXPORT int fk_write_bins(fk_ctx *c, const char *out_dir) {
    if (!c || !out_dir) return set_err(FK_E_INVALID, "null argument");
    DeviceGuard dg_(c->device);
    if (!c->have_result) return set_err(FK_E_STATE, "no result: call fk_finish or fk_reduce first");
    if (mkdir_p(out_dir) != 0) return set_err(FK_E_IO, "cannot create %s: %s", out_dir, strerror(errno));
    hipStream_t s = c->stream;
    const uint64_t D = c->distinct;
    const uint32_t nlb = c->nlb;
    const int eof = c->cfg.use_ht == 0;
    if (D == 0) return FK_OK;  // no k-mers: no bin files
    FK_TRY(materialize_dense(c));
    DevBuf len, off, bbytes, text;
    struct Free {
        DevBuf *b[4];
        ~Free() {
            for (DevBuf *x : b) release(*x);
        }
    } guard{{&len, &off, &bbytes, &text}};
    FK_TRY(ensure(len, D * 4));
    FK_TRY(ensure(off, (D + 1) * 8));
    FK_TRY(ensure(bbytes, ((uint64_t)nlb + 1) * 8));
    HIP_TRY(launch_format_lens(c->dense_counts.as<uint32_t>(), D, c->cfg.k, c->bin_off.as<uint64_t>(), nlb, eof,
                               len.as<uint32_t>(), s));
    HIP_TRY(scan_excl_sum_u32_to_u64(len.as<uint32_t>(), off.as<uint64_t>(), D, off.as<uint64_t>() + D, c->ws, s));
    HIP_TRY(launch_gather_u64(off.as<uint64_t>(), c->bin_off.as<uint64_t>(), (uint64_t)nlb + 1,
                              bbytes.as<uint64_t>(), s));
    std::vector<uint64_t> bb(nlb + 1, 0);
    HIP_TRY(hipMemcpyAsync(bb.data(), bbytes.p, ((uint64_t)nlb + 1) * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const uint64_t T = bb[nlb];
    FK_TRY(ensure(text, T + 16));
    HIP_TRY(launch_format_lines(c->KW, c->dense_keys.as<uint64_t>(), c->dense_counts.as<uint32_t>(), D, c->cfg.k,
                                off.as<uint64_t>(), text.as<uint8_t>(), s));
    uint8_t *host = nullptr;
    if (T) {
        HIP_TRY(hipHostMalloc((void **)&host, T, hipHostMallocDefault));
        const hipError_t e = hipMemcpyAsync(host, text.p, T, hipMemcpyDeviceToHost, s);
        const hipError_t e2 = e == hipSuccess ? hipStreamSynchronize(s) : e;
        if (e2 != hipSuccess) {
            (void)hipHostFree(host);
            return set_err(FK_E_DEVICE, "copying the bin text to the host: %s", hipGetErrorString(e2));
        }
    }
    const std::string dir(out_dir);
    const unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<int> errs(nth, 0);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nth; ++t) {
        th.emplace_back([&, t]() {
            for (uint32_t lb = t; lb < nlb; lb += nth) {
                if (c->h_bin_off[lb + 1] == c->h_bin_off[lb]) continue;  // empty bins have no file
                const std::string path = dir + "/bin" + std::to_string(global_bin(c, lb));
                FILE *f = fopen(path.c_str(), "wb");
                const size_t nb = (size_t)(bb[lb + 1] - bb[lb]);
                if (!f || fwrite(host + bb[lb], 1, nb, f) != nb) errs[t] = 1;
                if (f && fclose(f) != 0) errs[t] = 1;
            }
        });
    }
    for (auto &x : th) x.join();
    if (host) (void)hipHostFree(host);
    for (int e : errs)
        if (e) return set_err(FK_E_IO, "writing bin files under %s failed", out_dir);
    return FK_OK;
}

// ---------------------------------------------------------------------------
// bin-signature diagnostics (executeFindBinSignaturesJob, SBKC:956-986)
// ---------------------------------------------------------------------------

FK_EXPORT uint64_t fk_signature_slots(const fk_ctx *c) { return c ? (1ull << (2 * c->cfg.m)) + 1ull : 0ull; }

// getBinSignatures (SBKC:772-917) over the ingested input: the FASTA parse
// (fk_parse.inc, look-back variant) and one pass of k_bin_signatures.  The
// input stays as it was, so fk_map may follow.
FK_EXPORT int fk_signature_counts(fk_ctx *c, void *d_counts, uint64_t n_counts) {
    if (!c || !d_counts) return set_err(FK_E_INVALID, "null argument");
    DeviceGuard dg_(c->device);
    const uint64_t slots = fk_signature_slots(c);
    if (n_counts < slots)
        return set_err(FK_E_RANGE, "signature counts hold %llu entries, need 4^m + 1 = %llu",
                       (unsigned long long)n_counts, (unsigned long long)slots);
    if (c->pm_active && !c->pm_last_seen)
        return set_err(FK_E_STATE, "fk_signature_counts inside a streamed input: finish it with fk_ingest(..., last = 1)");
    hipStream_t s = c->stream;
    const uint64_t n = c->d_fasta ? c->n_fasta : 0;
    HIP_TRY(hipMemsetAsync(d_counts, 0, slots * 8, s));
    if (n) {
        const uint64_t ntiles = (n + ENC_TILE - 1) / ENC_TILE;
        const uint64_t code_words = n / 16 + 2 * POS_PAD_WORDS + 512;
        const uint64_t valid_words = n / 32 + 2 * POS_PAD_WORDS + 512;
        FK_TRY(ensure(c->tile_last_nl, ntiles * 8));
        FK_TRY(ensure(c->tile_off, ntiles * 8));
        FK_TRY(ensure(c->npos_dev, 16));
        FK_TRY(ensure(c->codes, code_words * 4));
        FK_TRY(ensure(c->valid, valid_words * 4));
        HIP_TRY(hipMemsetAsync(c->codes.p, 0, code_words * 4, s));
        HIP_TRY(hipMemsetAsync(c->valid.p, 0, valid_words * 4, s));
        HIP_TRY(hipMemsetAsync(c->npos_dev.p, 0, 16, s));
        HIP_TRY(hipMemsetAsync(c->tile_last_nl.p, 0, ntiles * 8, s));
        HIP_TRY(hipMemsetAsync(c->tile_off.p, 0, ntiles * 8, s));
        HIP_TRY(launch_fasta_parse(false, c->d_fasta, n, c->tile_last_nl.as<uint64_t>(), c->tile_off.as<uint64_t>(),
                                   c->codes.as<uint32_t>(), c->valid.as<uint32_t>(), c->npos_dev.as<uint64_t>(), s));
        HIP_TRY(launch_bin_signatures(c->codes.as<uint32_t>(), c->valid.as<uint32_t>(), n, c->npos_dev.as<uint64_t>(),
                                      c->cfg.k, c->cfg.m, (unsigned long long *)d_counts, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    return FK_OK;
}

// longToString (PKG:616-634): always nucleotidesPerLong = 31 characters, the
// signature's base-4 digits right-aligned behind 'A's (its length argument is unused).
static void signature_string(uint64_t v, char out[31]) {
    static const char rep[4] = {'A', 'C', 'G', 'T'};
    for (int j = 30; j >= 0; --j) {
        out[j] = rep[v & 3u];
        v >>= 2;
    }
}

// saveBinSignatures (SBKC:920-953): <out_dir>/bin_signatures<b>.txt for every
// bin this rank owns that holds a signature, "<signature>\t<count>\n" lines
// (ascending signature; the reference iterates a HashMap) and "Total\t<sum>\n".
FK_EXPORT int fk_write_bin_signatures(fk_ctx *c, const void *d_counts, uint64_t n_counts, const char *out_dir) {
    if (!c || !d_counts || !out_dir) return set_err(FK_E_INVALID, "null argument");
    DeviceGuard dg_(c->device);
    const uint64_t slots = fk_signature_slots(c);
    if (n_counts < slots)
        return set_err(FK_E_RANGE, "signature counts hold %llu entries, need 4^m + 1 = %llu",
                       (unsigned long long)n_counts, (unsigned long long)slots);
    hipStream_t s = c->stream;
    const unsigned long long *counts = (const unsigned long long *)d_counts;
    DevBuf nz, pairs;
    struct Free {
        DevBuf *b[2];
        ~Free() {
            for (DevBuf *x : b) release(*x);
        }
    } guard{{&nz, &pairs}};
    FK_TRY(ensure(nz, 8));
    unsigned long long nnz = 0;
    HIP_TRY(hipMemsetAsync(nz.p, 0, 8, s));
    HIP_TRY(launch_sig_compact(counts, slots, nullptr, nz.as<unsigned long long>(), s));
    HIP_TRY(hipMemcpyAsync(&nnz, nz.p, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<uint64_t> h(2 * nnz);
    if (nnz) {
        FK_TRY(ensure(pairs, nnz * 16));
        HIP_TRY(hipMemsetAsync(nz.p, 0, 8, s));
        HIP_TRY(launch_sig_compact(counts, slots, pairs.as<uint64_t>(), nz.as<unsigned long long>(), s));
        HIP_TRY(hipMemcpyAsync(h.data(), pairs.p, nnz * 16, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    // (bin, signature) order; bins owned by other ranks are theirs to write
    std::vector<std::pair<uint64_t, uint64_t>> rows;  // (bin << 32 | signature, count)
    rows.reserve(nnz);
    for (uint64_t i = 0; i < nnz; ++i) {
        const uint32_t sig = (uint32_t)h[2 * i];
        const int32_t b = (int32_t)bin_of_signature(sig, c->fm);
        if (owns(c, b)) rows.emplace_back(((uint64_t)b << 32) | sig, h[2 * i + 1]);
    }
    std::sort(rows.begin(), rows.end());
    if (rows.empty()) return FK_OK;
    if (mkdir_p(out_dir) != 0) return set_err(FK_E_IO, "cannot create %s: %s", out_dir, strerror(errno));
    const std::string dir(out_dir);
    std::string text;
    for (size_t i = 0; i < rows.size();) {
        const uint32_t b = (uint32_t)(rows[i].first >> 32);
        uint64_t tot = 0;
        text.clear();
        for (; i < rows.size() && (uint32_t)(rows[i].first >> 32) == b; ++i) {
            char sig[31];
            signature_string((uint32_t)rows[i].first, sig);
            text.append(sig, 31);
            text.push_back('\t');
            text += std::to_string(rows[i].second);
            text.push_back('\n');
            tot += rows[i].second;
        }
        text += "Total\t" + std::to_string(tot) + "\n";
        const std::string path = dir + "/bin_signatures" + std::to_string(b) + ".txt";
        FILE *f = fopen(path.c_str(), "wb");
        const bool ok = f && fwrite(text.data(), 1, text.size(), f) == text.size();
        if (f && fclose(f) != 0) return set_err(FK_E_IO, "closing %s failed", path.c_str());
        if (!ok) return set_err(FK_E_IO, "writing %s failed", path.c_str());
    }
    return FK_OK;
}

// executeFindBinSignaturesJob (SBKC:956-986) for one rank holding the whole
// input: fk_signature_counts into a context-owned buffer, then the writer.
FK_EXPORT int fk_find_bin_signatures(fk_ctx *c, const char *out_dir) {
    if (!c || !out_dir) return set_err(FK_E_INVALID, "null argument");
    DeviceGuard dg_(c->device);
    const uint64_t slots = fk_signature_slots(c);
    DevBuf counts;
    struct Free {
        DevBuf *b;
        ~Free() { release(*b); }
    } guard{&counts};
    FK_TRY(ensure(counts, slots * 8));
    FK_TRY(fk_signature_counts(c, counts.p, slots));
    return fk_write_bin_signatures(c, counts.p, slots, out_dir);
}
