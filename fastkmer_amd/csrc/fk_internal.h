// fk_internal.h -- device pipeline stages (launch wrappers in fk_kernels.hip).
//
// Data layout in HBM (one rank):
//   fasta      u8[n]                     input bytes (owned or borrowed)
//   codes      u32[npos/16 + pad]        2-bit bases, 16 per word, MSB-first
//   valid      u32[npos/32 + pad]        1 bit per position (1 = A/C/G/T)
//   records    u64[W * nrec]             super-k-mer records, W = 2 (k<=32) or 3
//              (the fused map: per tile, a header word + a u16 position per record and the
//              tile's 2-bit code stream; the partition builds the W-word records from them)
//   keys       u64[KW * nkmers]          canonical k-mers scattered by (bin, cell)
//   out_keys   u64[KW * nkmers]          per-bucket sorted unique keys
//   dense      u64[KW * distinct] + u32 counts, bin_off[nbins_local + 1]
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fk_common.h"

namespace fk {

constexpr int ENC_NT = 512;      // threads per parse/encode workgroup
constexpr int ENC_TILE = ENC_NT * 64;  // FASTA bytes per parse/encode workgroup (64 per thread)
constexpr int SIG_NT = 512;      // threads per signature workgroup
constexpr int SIG_TILE = SIG_NT * 16;  // k-mer start positions per signature workgroup
constexpr int SIG_PPT = 16;      // positions per thread == max k-mers per record
constexpr int POS_PAD_WORDS = 64;  // zero words after the packed stream (halo reads)
constexpr int SORT_CAP = 4096;   // keys per LDS-sorted bucket (u64 keys; half for 128-bit keys)
constexpr int MAX_FINE_BITS = 15;

// record header (low 32 bits of word 0): bin | (n-1) << 22 | fine_of_signature(sig) << 26
constexpr int REC_BIN_BITS = 22;
constexpr int REC_FINE_SHIFT = 26;
constexpr uint32_t REC_BIN_MASK = (1u << REC_BIN_BITS) - 1u;

struct Bucket {
    uint64_t begin;  // output position of the bucket's first key (prefix over (bin, cell))
    uint32_t n;      // keys in the bucket
    uint32_t lbin;   // local bin
    uint32_t c0, c1; // cells [c0, c1) of the bin
};

// A bucket's keys: np == 0, the contiguous range keys[begin, begin + n); np = 1..STAGE_MAXP,
// the staged pieces' key arrays (one job's input expanded piece by piece while it landed, and
// counted once): piece p holds the bucket's keys at pk[p][pcb[p][g0] .. pcb[p][g1]), g0 / g1 =
// (lbin << F) + c0 / c1, pcb[p] the exclusive scan of the piece's cell totals.
#ifndef FK_STAGE_MAXP
#define FK_STAGE_MAXP 5
#endif
constexpr int STAGE_MAXP = FK_STAGE_MAXP;
static_assert(STAGE_MAXP >= 4 && STAGE_MAXP <= 8, "staged pieces per job");
// 128-bit keys (k > 32) stage at most 4 pieces: their kernels' piece loops stop there (a fifth
// piece's bounds cost configs[3] 0.5-0.9 ms per step, profiles/r06z_five_pieces.txt)
constexpr int STAGE_MAXP128 = 4;
template <int KW>
constexpr int stage_npc() { return KW == 2 ? STAGE_MAXP128 : STAGE_MAXP; }
struct BucketSrc {
    const uint64_t *keys;
    int F;  // cell bits: a bucket's keys lie in [c0 << (2k-F), c1 << (2k-F))
    int np = 0;
    const uint64_t *pk[STAGE_MAXP] = {};
    const uint64_t *pcb[STAGE_MAXP] = {};
    const struct PieceStarts *starts = nullptr;  // per bucket (launch_bucket_finish), or null
};
// one bucket's keys in the staged pieces: piece p's first key at s[p] of pk[p], pre[p] keys of
// the bucket in the pieces before p (pre[p] = ~0u for p >= np)
struct PieceStarts {
    uint64_t s[STAGE_MAXP];
    uint32_t pre[STAGE_MAXP];
};
// every bucket's n / c1 (from the next bucket) and, with staged pieces (src.np > 0), its piece starts
hipError_t launch_bucket_finish(const BucketSrc &src, struct Bucket *buckets, uint64_t nb, uint32_t nlbins,
                                uint64_t total_keys, PieceStarts *out, hipStream_t s);

struct Chunk {
    uint64_t rec_begin, rec_end;  // records [begin, end) of one local bin
    uint32_t lbin, pad;
};

// Grow-only scratch space for the scans.
struct ScanWorkspace {
    void *ptr = nullptr;
    size_t bytes = 0;
};

// ---- scans (exclusive); `total` (device, may be null) receives the sum/max
hipError_t scan_excl_sum_u64(const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *total, ScanWorkspace &ws,
                             hipStream_t s);
hipError_t scan_excl_sum_u32_to_u64(const uint32_t *in, uint64_t *out, uint64_t n, uint64_t *total,
                                    ScanWorkspace &ws, hipStream_t s);
hipError_t scan_excl_max_i64(const int64_t *in, int64_t *out, uint64_t n, ScanWorkspace &ws, hipStream_t s);

// ---- FASTA parse + encode (records -> compacted packed positions)
hipError_t launch_fasta_parse(bool scan, const uint8_t *fa, uint64_t n, uint64_t *st_line, uint64_t *st_pos,
                              uint32_t *codes, uint32_t *valid, uint64_t *npos_dev, hipStream_t s);
hipError_t launch_superkmers(int W, const uint32_t *codes, const uint32_t *valid, uint64_t npos_bound,
                             const uint64_t *npos_dev, int k, int m, FastMod fm, uint64_t *records, uint64_t rec_cap,
                             uint64_t *status, uint64_t *tile_kmers, unsigned long long *counters, hipStream_t s);
hipError_t launch_fill_u64(uint64_t *p, uint64_t n, uint64_t v, hipStream_t s);
// ---- bin-signature diagnostics (fk_bin_signatures.inc, getBinSignatures SBKC:772-917)
hipError_t launch_bin_signatures(const uint32_t *codes, const uint32_t *valid, uint64_t npos_bound,
                                 const uint64_t *npos_dev, int k, int m, unsigned long long *counts, hipStream_t s);
hipError_t launch_sig_compact(const unsigned long long *counts, uint64_t n, uint64_t *pairs, unsigned long long *nout,
                              hipStream_t s);

// ---- fused parse + signature (fk_map_fused.inc): FASTA bytes -> compact records in one kernel
// for (k, m) with an instantiation; tiles of fm_tile_bytes(nth) FASTA bytes (nth = 256 or 512
// threads).  Tile t's records are header words at hdrs + t * map_fused_tcap() and their first
// positions at pos + t * map_fused_tcap(), their count in tcnt[t]; the tile's 2-bit code stream
// (MSB-first, 16 bases per word) at codes + t * map_fused_cslot().  counters[4] (zeroed) =
// records, k-mers, fallback flags, positions.
bool map_fused_supported(int k, int m, uint32_t nbins);
uint64_t fm_tile_bytes(int nth);
uint64_t fm_span_bytes(int nth);
uint32_t map_fused_tcap();
// measurement build (-DFK_PROBES): the fused map's per-phase wave cycles summed since the last reset
hipError_t map_fused_cycles(unsigned long long *out16, bool reset);
// measurement build: the sorted wave tiers' rank loop -- [0] iterations, [1] keys ranked, [2] buckets
hipError_t rank_probe_read(unsigned long long *out4, bool reset);
uint32_t map_fused_cslot();
uint32_t map_fused_vslot();  // split map: valid-stream slot words per tile (vslots)
hipError_t launch_map_fused(int nth, int k, int m, const uint8_t *fa, uint64_t n, int more, uint64_t tile_begin,
                            uint64_t ntiles, FastMod fm, uint32_t *hdrs, uint16_t *pos, uint32_t *codes,
                            uint32_t *tcnt, uint32_t *tstat, unsigned long long *counters, hipStream_t s,
                            int probe = 0, uint32_t *vslots = nullptr);
// counters[0] / [1] / [3] = records / k-mers / positions summed over the fused map's tiles [0, ntiles)
hipError_t launch_tile_totals(const uint32_t *tcnt, const uint32_t *tstat, uint64_t ntiles,
                              unsigned long long *counters, hipStream_t s);

// ---- records to partition: dense (tcnt == null: nrec W-word records, cut into PART_TILE tiles)
// or the fused map's compact tiles (tile t holds tcnt[t] records: slot t * tcap + j has the
// header word hdr[.] and the first position pos[.] of its bases in the tile's code stream
// code + t * cslot; the partition builds the W-word record from them).
constexpr uint32_t PART_TILE = 4096;  // dense records per tile
constexpr uint32_t PART_TPC = 4;      // tiles per partition workgroup (dense: 16384 records)
constexpr uint32_t PART_SEG = 64;     // partition workgroups per segment of the histogram scan
inline uint32_t part_segments(uint32_t nwg) { return (nwg + PART_SEG - 1) / PART_SEG; }
struct RecSrc {
    const uint64_t *rec;   // dense records (null for compact tiles)
    const uint32_t *tcnt;  // null: dense
    uint64_t nrec;         // records (the sum of tcnt when tiled)
    uint64_t ntiles;
    uint32_t tcap;         // record slots per tile
    uint32_t W;            // u64 words per record
    const uint32_t *hdr;   // compact tiles: header word per record slot
    const uint16_t *pos;   // compact tiles: first position of the record's bases in its tile's stream
    const uint32_t *code;  // compact tiles: per tile, cslot words of 2-bit codes (MSB-first)
    uint32_t cslot;        // words per tile's code stream
    uint32_t k;            // bases per record = n + k - 1
};
inline RecSrc dense_src(const uint64_t *rec, uint64_t nrec, int W) {
    return RecSrc{rec, nullptr, nrec, (nrec + PART_TILE - 1) / PART_TILE, PART_TILE, (uint32_t)W,
                  nullptr, nullptr, nullptr, 0u, 0u};
}
inline RecSrc tiled_src(const uint32_t *hdr, const uint16_t *pos, const uint32_t *code, const uint32_t *tcnt,
                        uint64_t nrec, uint64_t ntiles, uint32_t tcap, uint32_t cslot, int W, int k) {
    return RecSrc{nullptr, tcnt, nrec, ntiles, tcap, (uint32_t)W, hdr, pos, code, cslot, (uint32_t)k};
}

// ---- partition records by part = (bin % G) [dest] or (bin / G) [local bin]
// H, K: nparts * part_workgroups(src) u32 each; Hs, Ks: their exclusive scans
// (one more entry, the total).
constexpr uint32_t PART_MAX = 12288;    // parts per partition pass (LDS histogram)
uint32_t part_workgroups(const RecSrc &src);
// table: optional bin -> part map (size-aware placement); null: the formula
hipError_t launch_part_hist(const RecSrc &src, int mode, uint32_t G, const uint32_t *table, uint32_t nparts,
                            uint32_t *H, uint32_t *K, hipStream_t s);
// row-major histograms H/K[wg * nparts + p] -> part-major segment sums T/KT[p * nseg + seg]
hipError_t launch_part_segsum(const uint32_t *H, const uint32_t *K, uint32_t nparts, uint32_t nwg, uint64_t *T,
                              uint64_t *KT, hipStream_t s);
// scanned segment sums -> destinations Hs[wg * nparts + p]
hipError_t launch_part_segfill(const uint32_t *H, const uint64_t *Ts, uint32_t nparts, uint32_t nwg, uint64_t *Hs,
                               hipStream_t s);
hipError_t launch_part_totals(const uint64_t *Hs, const uint64_t *Ks, uint32_t nparts, uint32_t nwg,
                              uint64_t *part_rec, uint64_t *part_kmer, uint64_t *part_off, hipStream_t s);
hipError_t launch_part_scatter(const RecSrc &src, int mode, uint32_t G, const uint32_t *table, uint32_t nparts,
                               const uint64_t *Hs, uint64_t *out, hipStream_t s);
// nparts > PART_MAX: totals by global atomics (part_rec/part_kmer zeroed), scatter by per-part cursors
hipError_t launch_part_hist_global(const RecSrc &src, int mode, uint32_t G, const uint32_t *table, uint32_t nparts,
                                   uint64_t *part_rec, uint64_t *part_kmer, hipStream_t s);
hipError_t launch_part_scatter_global(const RecSrc &src, int mode, uint32_t G, const uint32_t *table,
                                      uint32_t nparts, const uint64_t *part_off, uint64_t *part_cursor,
                                      uint64_t *out, hipStream_t s);

// ---- sorted count
hipError_t launch_expand_hist(int W, const uint64_t *rec, const Chunk *chunks, uint32_t nchunks, int k, int F,
                              uint32_t *hist, hipStream_t s);
hipError_t launch_cell_prefix(const uint32_t *bin_chunk_begin, uint32_t nlbins, int F, uint32_t *hist,
                              uint64_t *cell_total, hipStream_t s);
// one-level expansion (k = 64, W = 3 only)
hipError_t launch_expand_scatter(int W, const uint64_t *rec, const Chunk *chunks, uint32_t nchunks, int k, int F,
                                 const uint32_t *hist, const uint64_t *cell_base, uint64_t *keys, hipStream_t s);
hipError_t launch_bucket_flags(const uint64_t *cell_base, const uint64_t *cell_total, uint32_t nlbins, int F,
                               uint32_t small_cap, uint32_t group, uint32_t *flags, hipStream_t s);
hipError_t launch_bucket_write(const uint64_t *cell_base, const uint32_t *flags, const uint64_t *flag_scan,
                               uint32_t nlbins, int F, uint64_t nbuckets, uint64_t total_keys, Bucket *buckets,
                               hipStream_t s);
hipError_t launch_bucket_count64(const BucketSrc &src, const Bucket *buckets, uint64_t nbuckets, int k,
                                 uint64_t *out_keys, uint32_t *out_counts, uint64_t *bucket_unique,
                                 unsigned long long *oversize, uint32_t small_limit, int dbg_phase,
                                 const uint32_t *list, hipStream_t s, uint32_t skip_le = 0);
hipError_t launch_bucket_count64_big(const BucketSrc &src, const Bucket *buckets, uint64_t nlist, int k,
                                     uint64_t *out_keys, uint32_t *out_counts, uint64_t *bucket_unique,
                                     unsigned long long *oversize, const uint32_t *list, hipStream_t s);
constexpr uint32_t WAVE_BUCKET_CAP = 512;
#ifndef FK_WAVE_SL
#define FK_WAVE_SL 640  // table slots of a 512-key wave bucket (7.4 KB of LDS per wave, 6 waves per SIMD; 768:
                        // 5, 1.4 ms slower at the configs[2] load, profiles/r05l_wave_slots_ab.txt)
#endif
constexpr uint32_t WAVE_SLOTS = FK_WAVE_SL;
constexpr uint32_t WAVE_MID_CAP = 1024;  // 64-bit mid wave tier: listed buckets of 513 .. 1024 keys
#ifndef FK_MID_SL
#define FK_MID_SL 1280  // its table slots (14.6 KB per wave; 1536: kernel 2.15 vs 2.03 ms at the configs[2]
                        // load, profiles/r05q_mid_slots_ab.txt)
#endif
constexpr uint32_t WAVE_MID_SLOTS = FK_MID_SL;
constexpr uint32_t WAVE128_BUCKET_CAP = 256;  // keys per wave-tier bucket, 128-bit keys (k_bucket_count128_wave)
hipError_t launch_bucket_count128_wave(const BucketSrc &src, const Bucket *buckets, uint64_t nbuckets, int k,
                                       uint64_t *out_keys, uint32_t *out_counts, uint64_t *bucket_unique,
                                       hipStream_t s, bool ordered = true);
hipError_t launch_expand_two_level(int KW, const uint64_t *rec, const Chunk *chunks, uint32_t nchunks,
                                   uint32_t nlbins, int k, int F, int F2, const uint32_t *sc_pre,
                                   const uint64_t *cell_base, uint64_t *mid, uint64_t *keys, hipStream_t s,
                                   int l1_threads = 0, uint64_t nkeys = 0);
// pieces of bins (x = local bin, y / z = chunk range, w = whole bin): the same per piece, then the
// earlier pieces' super-cell totals added (first_piece[i] = the bin's first piece)
hipError_t launch_expand_hist_pieces(int KW, const uint64_t *rec, const Chunk *chunks, const uint4 *pieces,
                                     const uint32_t *first_piece, uint32_t npieces, int k, int F, int F2,
                                     uint64_t *cell_total, uint32_t *hist_sc, uint32_t *piece_tot, hipStream_t s);
// one workgroup per local bin: cell totals and the per-chunk exclusive super-cell prefix in one pass
hipError_t launch_expand_hist_bin(int KW, const uint64_t *rec, const Chunk *chunks, const uint32_t *bin_chunk_begin,
                                  uint32_t nlbins, int k, int F, int F2, uint64_t *cell_total, uint32_t *hist_sc,
                                  hipStream_t s);
hipError_t launch_bucket_flags_greedy(const uint64_t *cell_total, uint32_t nlbins, int F, uint32_t cap,
                                      int period_bits, uint32_t *flags, hipStream_t s);
// lists[0, nb): buckets of wave_cap < n <= block_cap, lists[nb, 2 nb): above block_cap; counts[0] / [1]
// their lengths; *listed_keys += their keys
hipError_t launch_bucket_tiers(const Bucket *buckets, uint64_t nb, uint32_t wave_cap, uint32_t block_cap,
                               uint64_t *bucket_unique, uint32_t *lists, unsigned int *counts,
                               unsigned long long *listed_keys, hipStream_t s);
// ordered = false (useHT): every bucket's distinct keys in table order, no rank
hipError_t launch_bucket_count64_wave(const BucketSrc &src, const Bucket *buckets, uint64_t nbuckets, int k,
                                      uint64_t *out_keys, uint32_t *out_counts, uint64_t *bucket_unique,
                                      const uint32_t *list, hipStream_t s, bool ordered = true);
// the listed mid-tier buckets (WAVE_BUCKET_CAP .. WAVE_MID_CAP keys) as 2 or 3 key ranges, each counted
// by the wave tier's code in order; buckets with a range above WAVE_BUCKET_CAP go to fb (count in fb_count)
hipError_t launch_bucket_count64_parts(const BucketSrc &src, const Bucket *buckets, const uint32_t *list,
                                       uint64_t nlist, int k, uint64_t *out_keys, uint32_t *out_counts,
                                       uint64_t *bucket_unique, uint32_t *fb, unsigned int *fb_count, hipStream_t s,
                                       bool ordered);
// the mid tier's buckets on the 512-key table when they hold <= 512 distinct keys (the others listed
// in fb for the 1024-key kernel): a job whose k-mers repeat
hipError_t launch_bucket_count64_mid512(const BucketSrc &src, const Bucket *buckets, const uint32_t *list,
                                        uint64_t nlist, int k, uint64_t *out_keys, uint32_t *out_counts,
                                        uint64_t *bucket_unique, uint32_t *fb, unsigned int *fb_count, hipStream_t s,
                                        bool ordered);
// the listed block-tier buckets of at most WAVE_MID_CAP keys, one wave each (k <= 32)
hipError_t launch_bucket_count64_wave_mid(const BucketSrc &src, const Bucket *buckets, const uint32_t *list,
                                          uint64_t nlist, int k, uint64_t *out_keys, uint32_t *out_counts,
                                          uint64_t *bucket_unique, hipStream_t s, bool ordered = true);
// heavy buckets (above the wave tier, k <= 32) split into wave-sized sub-buckets by sampled
// splitters (k_bucket_split64), counted in order by one wave per bucket (k_sub_count64_seq)
struct SubBucket {
    uint64_t src;   // first key in the split copy (skeys)
    uint64_t lo;    // every key lies in [lo, lo + 2^span) (the rank's group cut)
    uint32_t n, span;
};
struct SplitParent {
    uint32_t first, nsub;  // sub-buckets [first, first + nsub) of the list; nsub = 0: not split
};
// sizes[i] = the room of listed bucket i (list0 then list1) in the split copy: its keys, or with slots
// (64-bit keys) split_room: a 512-key region per first-cut sub-bucket
hipError_t launch_listed_sizes(const Bucket *buckets, const uint32_t *list0, uint32_t n0, const uint32_t *list1,
                               uint32_t n1, uint64_t *sizes, hipStream_t s,
                               bool slots = false);
// counts[0] += sub-buckets, counts[1] / [2] += buckets left to the block / big path (fb0 / fb1: their
// indices; a bucket of n <= block_cap goes to fb0).  A bucket whose cut leaves a sub-bucket above a
// wave's keys is cut again from another sample into twice as many (retry: every bucket, a test hook)
hipError_t launch_bucket_split64(const BucketSrc &src, const Bucket *buckets, const uint32_t *list0, uint32_t n0,
                                 const uint32_t *list1, uint32_t n1, const uint64_t *sbase, uint64_t *skeys,
                                 SubBucket *subs, SplitParent *parents, unsigned int *counts, uint32_t *fb0,
                                 uint32_t *fb1, uint32_t block_cap, int k, int F, hipStream_t s, bool retry = false);
hipError_t launch_sub_count64_seq(const Bucket *buckets, const uint32_t *list, uint32_t nl, const SplitParent *parents,
                                  const SubBucket *subs, const uint64_t *skeys, uint64_t *out_keys,
                                  uint32_t *out_counts, uint64_t *bucket_unique, hipStream_t s, bool ordered);
// the same for 128-bit keys (33 <= k <= 63): sub-bucket keys as (hi, lo) word pairs, counted by the mid
// wave tier's 512-key table; fallbacks: fb0 (<= block_cap keys, the LDS sort), fb1 (the streaming path)
struct SubBucket128 {
    uint64_t src;          // first key (pair index) in the split copy
    uint64_t lo_hi, lo_lo; // every key lies in [lo, lo + 2^span)
    uint32_t n, span;
};
hipError_t launch_bucket_split128(const BucketSrc &src, const Bucket *buckets, const uint32_t *list, uint32_t nl,
                                  const uint64_t *sbase, uint64_t *skeys, SubBucket128 *subs, SplitParent *parents,
                                  unsigned int *counts, uint32_t *fb0, uint32_t *fb1, uint32_t block_cap, int k, int F,
                                  hipStream_t s, bool retry = false);
hipError_t launch_sub_count128_seq(const Bucket *buckets, const uint32_t *list, uint32_t nl, const SplitParent *parents,
                                   const SubBucket128 *subs, const uint64_t *skeys, uint64_t *out_keys,
                                   uint32_t *out_counts, uint64_t *bucket_unique, hipStream_t s, bool ordered);
// dst[i] += src[i] (dst = src when `copy`)
hipError_t launch_add_u64(uint64_t *dst, const uint64_t *src, uint64_t n, bool copy, hipStream_t s);
// skip_le: listed buckets of at most this many keys were counted by a wave tier (skipped)
hipError_t launch_bucket_sort(int KW, const BucketSrc &src, const Bucket *buckets, uint64_t nbuckets, int k,
                              uint64_t *out_keys, uint32_t *out_counts, uint64_t *bucket_unique,
                              unsigned long long *oversize, uint32_t small_limit, const uint32_t *list, hipStream_t s,
                              uint32_t skip_le = 0);
// 128-bit keys, the listed buckets of WAVE128_BUCKET_CAP < n <= WAVE128_MID_CAP keys: one wave each,
// a 768-slot table (the others on the list are skipped)
constexpr uint32_t WAVE128_MID_CAP = 512;
hipError_t launch_bucket_count128_wave_mid(const BucketSrc &src, const Bucket *buckets, const uint32_t *list,
                                           uint64_t nlist, int k, uint64_t *out_keys, uint32_t *out_counts,
                                           uint64_t *bucket_unique, hipStream_t s, bool ordered = true);
hipError_t launch_bucket_sort_large(int KW, const BucketSrc &src, const Bucket *buckets, uint64_t nbuckets, int k,
                                    uint64_t *scratch, uint64_t *out_keys, uint32_t *out_counts,
                                    uint64_t *bucket_unique, const uint32_t *list, hipStream_t s,
                                    unsigned long long *scratch_cursor = nullptr);
hipError_t launch_bucket_compact(int KW, const uint64_t *out_keys, const uint32_t *out_counts,
                                 const Bucket *buckets, uint64_t nbuckets, const uint64_t *dense_off,
                                 uint64_t *dense_keys, uint32_t *dense_counts, hipStream_t s);
hipError_t launch_bin_offsets(const uint64_t *flag_scan, const uint64_t *dense_off, uint32_t nlbins, int F,
                              uint64_t nbuckets, uint64_t *bin_off, hipStream_t s);

// ---- test hook: the 128-bit wave tier's fingerprints cut to `bits` low bits (0: whole), current device
hipError_t set_fingerprint_bits(int bits);

// ---- test hook: a one-thread kernel holding stream s until *flag != 0 (host-mapped) or max_ticks
// of the wall clock have passed
hipError_t launch_hold_stream(const uint32_t *flag, uint64_t max_ticks, hipStream_t s);

// ---- synthetic input
hipError_t launch_synth(uint8_t *out, uint64_t nbytes, SynthParams p, hipStream_t s);

// ---- bin-file text (fk_format.inc) and a small gather: out[i] = src[idx[i]]
hipError_t launch_format_lens(const uint32_t *counts, uint64_t n, int k, const uint64_t *bin_off, uint32_t nlb,
                              int eof, uint32_t *len, hipStream_t s);
hipError_t launch_format_lines(int KW, const uint64_t *keys, const uint32_t *counts, uint64_t n, int k,
                               const uint64_t *off, uint8_t *out, hipStream_t s);
hipError_t launch_gather_u64(const uint64_t *src, const uint64_t *idx, uint64_t n, uint64_t *out, hipStream_t s);

}  // namespace fk
