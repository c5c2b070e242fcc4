// fk_kernels.hip -- CDNA4 (gfx950) kernels of the exact k-mer counting path.
//
// Pipeline per rank (see DESIGN.md for the roofline of each stage):
//   1. FASTA parse + 2-bit encode      (FASTAshortInputFileFormat records, SBKC:62-65)
//   2. signature + super-k-mer records  (getSuperKmers, SBKC:34-169)
//   3. partition records by bin         (reduceByKey shuffle, SBKC:1035)
//   4. expand + cell histogram/scatter  (extractKXmers run loop, SBKC:484-524)
//   5. bucket sort + run-length count   (quickSort + RIndex heap merge, SBKC:540-597)
//      or open-addressing hash count    (extractKXmersHT, SBKC:664-739)
// Every kernel is written for 64-wide wavefronts and 256-thread workgroups.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fk_internal.h"

namespace fk {

constexpr int NT = 256;  // threads per workgroup (4 waves)

// ---------------------------------------------------------------------------
// block-level helpers (256 threads)
// ---------------------------------------------------------------------------

template <typename T>
__device__ __forceinline__ T wave_incl_sum(T v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T u = __shfl_up(v, d, 64);
        if (lane >= d) v += u;
    }
    return v;
}

template <typename T>
__device__ __forceinline__ T wave_incl_max(T v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T u = __shfl_up(v, d, 64);
        if (lane >= d) v = u > v ? u : v;
    }
    return v;
}

// exclusive block prefix sum; *total receives the block sum (all threads)
template <typename T>
__device__ __forceinline__ T block_excl_sum(T v, T *s_tmp /*[4]*/, T *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    T inc = wave_incl_sum(v);
    if (lane == 63) s_tmp[wid] = inc;
    __syncthreads();
    T off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        T x = s_tmp[w];
        if (w < wid) off += x;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

// ---- decoupled look-back (single-pass tile prefix without a shared counter)
// status[t] = flag << 62 | value: flag 1 = tile aggregate, 2 = inclusive
// prefix.  Agent-scope atomic loads/stores keep the 8 XCD L2s coherent.
constexpr uint64_t LB_AGG = 1ull << 62, LB_INC = 2ull << 62, LB_VAL = (1ull << 62) - 1ull;

__device__ __forceinline__ uint64_t lb_load(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Called by one whole wave.  Publishes `agg` for `tile`, returns the sum of
// the aggregates of tiles 0..tile-1 and publishes the inclusive prefix.
// Tiles are dispatched in blockIdx order, so every predecessor is resident
// or finished and the spin terminates.
__device__ uint64_t lookback_excl(uint64_t *status, uint64_t tile, uint64_t agg) {
    const int lane = threadIdx.x & 63;
    if (tile == 0) {
        if (lane == 0) lb_store(&status[0], LB_INC | agg);
        return 0;
    }
    if (lane == 0) lb_store(&status[tile], LB_AGG | agg);
    uint64_t excl = 0;
    int64_t pos = (int64_t)tile - 1;
    while (true) {
        const int64_t q = pos - lane;
        const uint64_t st = q >= 0 ? lb_load(&status[q]) : LB_INC;  // before tile 0: inclusive 0
        const uint32_t flag = (uint32_t)(st >> 62);
        const uint64_t inc_mask = __ballot(flag == 2u);
        const uint64_t zero_mask = __ballot(flag == 0u);
        const int first_inc = inc_mask ? __builtin_ctzll(inc_mask) : 64;
        const uint64_t before = first_inc == 64 ? ~0ull : ((1ull << first_inc) - 1ull);
        if (zero_mask & before) {
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        const uint64_t v = lane <= first_inc ? (st & LB_VAL) : 0ull;
        excl += __shfl(wave_incl_sum(v), 63, 64);
        if (first_inc < 64) break;
        pos -= 64;
    }
    if (lane == 0) lb_store(&status[tile], LB_INC | (excl + agg));
    return excl;
}

// exclusive block prefix max (identity `ident`)
template <typename T>
__device__ __forceinline__ T block_excl_max(T v, T ident, T *s_tmp /*[4]*/, T *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    T inc = wave_incl_max(v);
    T exc = __shfl_up(inc, 1, 64);
    if (lane == 0) exc = ident;
    if (lane == 63) s_tmp[wid] = inc;
    __syncthreads();
    T off = ident, tot = ident;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        T x = s_tmp[w];
        if (w < wid) off = x > off ? x : off;
        tot = x > tot ? x : tot;
    }
    __syncthreads();
    *total = tot;
    return exc > off ? exc : off;
}

// ---------------------------------------------------------------------------
// device-wide exclusive scans (reduce -> scan of block sums -> down-sweep)
// ---------------------------------------------------------------------------

constexpr int SCAN_IPT = 8;
constexpr int SCAN_SEG = NT * SCAN_IPT;  // 2048 elements per block

struct OpSum {
    template <typename T>
    __device__ T operator()(T a, T b) const { return a + b; }
};
struct OpMax {
    template <typename T>
    __device__ T operator()(T a, T b) const { return a > b ? a : b; }
};

template <typename TI, typename TO, typename Op>
__global__ __launch_bounds__(NT) void k_scan_reduce(const TI *in, uint64_t n, TO *sums, TO ident, Op op) {
    __shared__ TO s_red[NT];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_SEG;
    TO acc = ident;
#pragma unroll
    for (int i = 0; i < SCAN_IPT; ++i) {
        uint64_t idx = base + (uint64_t)i * NT + threadIdx.x;
        if (idx < n) acc = op(acc, (TO)in[idx]);
    }
    s_red[threadIdx.x] = acc;
    __syncthreads();
    for (int st = NT / 2; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st) s_red[threadIdx.x] = op(s_red[threadIdx.x], s_red[threadIdx.x + st]);
        __syncthreads();
    }
    if (threadIdx.x == 0) sums[blockIdx.x] = s_red[0];
}

// exclusive scan of one segment with a carry-in (carry[blockIdx] or ident)
template <typename TI, typename TO, typename Op, bool IS_MAX>
__global__ __launch_bounds__(NT) void k_scan_down(const TI *in, TO *out, uint64_t n, const TO *carry, TO ident,
                                                  Op op, TO *total) {
    __shared__ TO s_tmp[NT / 64];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_SEG + (uint64_t)threadIdx.x * SCAN_IPT;
    TO v[SCAN_IPT];
    TO acc = ident;
#pragma unroll
    for (int i = 0; i < SCAN_IPT; ++i) {
        uint64_t idx = base + i;
        v[i] = idx < n ? (TO)in[idx] : ident;
        acc = op(acc, v[i]);
    }
    TO tot;
    TO pre;
    if constexpr (IS_MAX) {
        pre = block_excl_max<TO>(acc, ident, s_tmp, &tot);
    } else {
        pre = block_excl_sum<TO>(acc, s_tmp, &tot);
    }
    TO run = op(carry ? carry[blockIdx.x] : ident, pre);
#pragma unroll
    for (int i = 0; i < SCAN_IPT; ++i) {
        uint64_t idx = base + i;
        if (idx < n) out[idx] = run;
        run = op(run, v[i]);
    }
    if (total && threadIdx.x == NT - 1 && blockIdx.x == gridDim.x - 1) *total = run;
}

template <typename TI, typename TO, typename Op, bool IS_MAX>
static hipError_t scan_impl(const TI *in, TO *out, uint64_t n, TO ident, TO *total, char *ws, size_t ws_bytes,
                            hipStream_t s) {
    if (n == 0) {
        if (total) return hipMemsetAsync(total, 0, sizeof(TO), s);  // only sums report totals
        return hipSuccess;
    }
    const uint64_t nb = (n + SCAN_SEG - 1) / SCAN_SEG;
    if (nb == 1) {
        k_scan_down<TI, TO, Op, IS_MAX><<<1, NT, 0, s>>>(in, out, n, (const TO *)nullptr, ident, Op(), total);
        return hipGetLastError();
    }
    if (ws_bytes < 2 * nb * sizeof(TO)) return hipErrorOutOfMemory;
    TO *sums = (TO *)ws;
    TO *sums_scan = sums + nb;
    k_scan_reduce<TI, TO, Op><<<(unsigned)nb, NT, 0, s>>>(in, n, sums, ident, Op());
    hipError_t e = scan_impl<TO, TO, Op, IS_MAX>(sums, sums_scan, nb, ident, (TO *)nullptr,
                                                 (char *)(sums_scan + nb), ws_bytes - 2 * nb * sizeof(TO), s);
    if (e != hipSuccess) return e;
    k_scan_down<TI, TO, Op, IS_MAX><<<(unsigned)nb, NT, 0, s>>>(in, out, n, sums_scan, ident, Op(), total);
    return hipGetLastError();
}

static size_t scan_ws_need(uint64_t n, size_t elem) {
    size_t need = 0;
    while (n > (uint64_t)SCAN_SEG) {
        n = (n + SCAN_SEG - 1) / SCAN_SEG;
        need += 2 * n * elem;
    }
    return need + 256;
}

static hipError_t ensure_ws(ScanWorkspace &ws, size_t need) {
    if (ws.bytes >= need) return hipSuccess;
    if (ws.ptr) (void)hipFree(ws.ptr);
    ws.ptr = nullptr;
    ws.bytes = 0;
    hipError_t e = hipMalloc(&ws.ptr, need);
    if (e == hipSuccess) ws.bytes = need;
    return e;
}

hipError_t scan_excl_sum_u64(const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *total, ScanWorkspace &ws,
                             hipStream_t s) {
    hipError_t e = ensure_ws(ws, scan_ws_need(n, 8));
    if (e != hipSuccess) return e;
    return scan_impl<uint64_t, uint64_t, OpSum, false>(in, out, n, (uint64_t)0, total, (char *)ws.ptr, ws.bytes, s);
}

hipError_t scan_excl_sum_u32_to_u64(const uint32_t *in, uint64_t *out, uint64_t n, uint64_t *total,
                                    ScanWorkspace &ws, hipStream_t s) {
    hipError_t e = ensure_ws(ws, scan_ws_need(n, 8));
    if (e != hipSuccess) return e;
    return scan_impl<uint32_t, uint64_t, OpSum, false>(in, out, n, (uint64_t)0, total, (char *)ws.ptr, ws.bytes, s);
}

hipError_t scan_excl_max_i64(const int64_t *in, int64_t *out, uint64_t n, ScanWorkspace &ws, hipStream_t s) {
    hipError_t e = ensure_ws(ws, scan_ws_need(n, 8));
    if (e != hipSuccess) return e;
    return scan_impl<int64_t, int64_t, OpMax, true>(in, out, n, (int64_t)-1, (int64_t *)nullptr, (char *)ws.ptr,
                                                    ws.bytes, s);
}

// ---------------------------------------------------------------------------
// 1. FASTA parse + encode
//
// A workgroup owns ENC_TILE bytes; each thread 64 consecutive bytes.  A line
// is a header iff its first byte is '>'; lines before the first header are
// ignored; sequence lines are concatenated with '\n' removed; each header
// contributes one invalid position (its '>') so k-mers never span records.
// ---------------------------------------------------------------------------

constexpr int ENC_BPT = ENC_TILE / NT;  // 64 bytes per thread
enum : int { ST_JUNK = 0, ST_HDR = 1, ST_SEQ = 2, ST_LINESTART = 3 };

// 64 bytes of the tile into registers (16 B vector loads when in bounds)
__device__ __forceinline__ void load64(const uint8_t *fa, uint64_t n, uint64_t p0, uint32_t (&w)[16]) {
    if (p0 + 64 <= n && ((reinterpret_cast<uintptr_t>(fa + p0) & 15) == 0)) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 *src = reinterpret_cast<const u32x4 *>(fa + p0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const u32x4 q = __builtin_nontemporal_load(src + i);
            w[4 * i + 0] = q.x;
            w[4 * i + 1] = q.y;
            w[4 * i + 2] = q.z;
            w[4 * i + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            uint32_t x = 0;
            for (int b = 0; b < 4; ++b) {
                uint64_t p = p0 + 4 * i + b;
                if (p < n) x |= (uint32_t)fa[p] << (8 * b);
            }
            w[i] = x;
        }
    }
}

__device__ __forceinline__ uint8_t byte_of(const uint32_t (&w)[16], int j) {
    return (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
}

__global__ __launch_bounds__(NT) void k_fasta_marks(const uint8_t *fa, uint64_t n, int64_t *tile_last_nl,
                                                    int64_t *tile_first_hdr) {
    __shared__ int64_t s_tmp[NT / 64];
    const uint64_t p0 = (uint64_t)blockIdx.x * ENC_TILE + (uint64_t)threadIdx.x * ENC_BPT;
    uint32_t w[16];
    load64(fa, n, p0, w);
    uint8_t prev = (p0 == 0) ? (uint8_t)'\n' : (p0 - 1 < n ? fa[p0 - 1] : 0);
    int64_t last_nl = -1;
    int64_t hdr = INT64_MAX;
#pragma unroll
    for (int j = 0; j < ENC_BPT; ++j) {
        const uint8_t c = byte_of(w, j);
        const uint64_t p = p0 + j;
        if (p < n) {
            if (c == '\n') last_nl = (int64_t)p;
            if (c == '>' && prev == '\n' && hdr == INT64_MAX) hdr = (int64_t)p;
        }
        prev = c;
    }
    int64_t tot;
    (void)block_excl_max<int64_t>(last_nl, (int64_t)-1, s_tmp, &tot);
    // first header of the tile: max over -hdr (one value per tile, no atomics)
    int64_t neg_first;
    (void)block_excl_max<int64_t>(-hdr, -INT64_MAX, s_tmp, &neg_first);
    if (threadIdx.x == 0) {
        tile_last_nl[blockIdx.x] = tot;
        tile_first_hdr[blockIdx.x] = -neg_first;
    }
}

// first header of the whole input = min over tiles (one workgroup)
__global__ __launch_bounds__(1024) void k_first_header(const int64_t *tile_first_hdr, uint64_t ntiles,
                                                       unsigned long long *first_hdr) {
    __shared__ int64_t s_m[1024];
    int64_t m = INT64_MAX;
    for (uint64_t t = threadIdx.x; t < ntiles; t += 1024) m = min(m, tile_first_hdr[t]);
    s_m[threadIdx.x] = m;
    __syncthreads();
    for (int st = 512; st > 0; st >>= 1) {
        if ((int)threadIdx.x < st) s_m[threadIdx.x] = min(s_m[threadIdx.x], s_m[threadIdx.x + st]);
        __syncthreads();
    }
    if (threadIdx.x == 0) *first_hdr = (unsigned long long)s_m[0];
}

// State machine shared by the count and encode passes.  Returns the kept
// mask: bit j set = byte j of this thread is a sequence position.

__device__ __forceinline__ int line_state_at(const uint8_t *fa, uint64_t n, int64_t ls, int64_t fh) {
    // state of the line that starts at ls (ls < n)
    if (fa[ls] == '>') return ST_HDR;
    return ls > fh ? ST_SEQ : ST_JUNK;
}

__device__ __forceinline__ uint64_t classify64(const uint8_t *fa, uint64_t n, uint64_t p0, const uint32_t (&w)[16],
                                               int64_t tile_prev_nl, int64_t fh, int64_t *s_tmp) {
    // last '\n' before this thread's first byte: max over earlier threads of the tile, else the tile's carry
    int64_t my_last = -1;
#pragma unroll
    for (int j = 0; j < ENC_BPT; ++j)
        if (p0 + j < n && byte_of(w, j) == '\n') my_last = (int64_t)(p0 + j);
    int64_t tot;
    int64_t prev_nl = block_excl_max<int64_t>(my_last, (int64_t)-1, s_tmp, &tot);
    if (prev_nl < tile_prev_nl) prev_nl = tile_prev_nl;
    const int64_t ls = prev_nl + 1;  // start of the line holding byte p0
    int st;
    if ((uint64_t)ls == p0) {
        st = ST_LINESTART;
    } else {
        st = ((uint64_t)ls < n) ? line_state_at(fa, n, ls, fh) : ST_JUNK;
    }
    uint64_t kept = 0;
#pragma unroll
    for (int j = 0; j < ENC_BPT; ++j) {
        const uint64_t p = p0 + j;
        const uint8_t c = byte_of(w, j);
        bool keep = false;
        if (p < n) {
            if (st == ST_LINESTART) {
                st = (c == '>') ? ST_HDR : ((int64_t)p > fh ? ST_SEQ : ST_JUNK);
                keep = (st != ST_JUNK);  // a header keeps its '>' as the record separator
            } else {
                keep = (st == ST_SEQ) && c != '\n';
            }
            if (c == '\n') {
                st = ST_LINESTART;
                keep = false;
            }
        }
        if (keep) kept |= 1ull << j;
    }
    return kept;
}

__global__ __launch_bounds__(NT) void k_fasta_count(const uint8_t *fa, uint64_t n, const int64_t *tile_prev_nl,
                                                    const unsigned long long *first_hdr, uint64_t *tile_kept) {
    __shared__ int64_t s_tmp[NT / 64];
    __shared__ uint64_t s_sum[NT / 64];
    const uint64_t p0 = (uint64_t)blockIdx.x * ENC_TILE + (uint64_t)threadIdx.x * ENC_BPT;
    uint32_t w[16];
    load64(fa, n, p0, w);
    const int64_t fh = (int64_t)*first_hdr;
    const uint64_t kept = classify64(fa, n, p0, w, tile_prev_nl[blockIdx.x], fh, s_tmp);
    uint64_t tot;
    (void)block_excl_sum<uint64_t>((uint64_t)__popcll(kept), s_sum, &tot);
    if (threadIdx.x == 0) tile_kept[blockIdx.x] = tot;
}

__global__ __launch_bounds__(NT) void k_fasta_encode(const uint8_t *fa, uint64_t n, const int64_t *tile_prev_nl,
                                                     const unsigned long long *first_hdr, const uint64_t *tile_off,
                                                     uint32_t *codes, uint32_t *valid) {
    __shared__ int64_t s_tmp[NT / 64];
    __shared__ uint64_t s_sum[NT / 64];
    __shared__ uint8_t s_out[ENC_TILE + 64];
    const uint64_t p0 = (uint64_t)blockIdx.x * ENC_TILE + (uint64_t)threadIdx.x * ENC_BPT;
    uint32_t w[16];
    load64(fa, n, p0, w);
    const int64_t fh = (int64_t)*first_hdr;
    const uint64_t kept = classify64(fa, n, p0, w, tile_prev_nl[blockIdx.x], fh, s_tmp);
    uint64_t tot;
    const uint64_t my_off = block_excl_sum<uint64_t>((uint64_t)__popcll(kept), s_sum, &tot);
    // compact this thread's kept codes into LDS
    uint32_t q = (uint32_t)my_off;
#pragma unroll
    for (int j = 0; j < ENC_BPT; ++j)
        if ((kept >> j) & 1) s_out[q++] = (uint8_t)base_code(byte_of(w, j));
    __syncthreads();
    const uint64_t P0 = tile_off[blockIdx.x];
    const uint64_t K = tot;
    if (K == 0) return;
    // code words: 16 positions per word, MSB-first
    {
        const uint64_t wb = P0 >> 4, we = (P0 + K - 1) >> 4;
        for (uint64_t wi = wb + threadIdx.x; wi <= we; wi += NT) {
            uint32_t word = 0;
            bool partial = false;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint64_t gp = (wi << 4) + j;
                if (gp >= P0 && gp < P0 + K) {
                    const uint32_t c = s_out[gp - P0];
                    word |= (c & 3u) << (30 - 2 * j);
                } else {
                    partial = true;
                }
            }
            if (partial)
                atomicOr(&codes[wi], word);
            else
                codes[wi] = word;
        }
    }
    // valid words: 32 positions per word, MSB-first
    {
        const uint64_t wb = P0 >> 5, we = (P0 + K - 1) >> 5;
        for (uint64_t wi = wb + threadIdx.x; wi <= we; wi += NT) {
            uint32_t word = 0;
            bool partial = false;
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                const uint64_t gp = (wi << 5) + j;
                if (gp >= P0 && gp < P0 + K) {
                    if (s_out[gp - P0] < 4) word |= 1u << (31 - j);
                } else {
                    partial = true;
                }
            }
            if (partial)
                atomicOr(&valid[wi], word);
            else
                valid[wi] = word;
        }
    }
}

hipError_t launch_fasta_marks(const uint8_t *fa, uint64_t n, int64_t *tile_last_nl, int64_t *tile_first_hdr,
                              unsigned long long *first_hdr, hipStream_t s) {
    const uint64_t nt = (n + ENC_TILE - 1) / ENC_TILE;
    if (nt == 0) return hipSuccess;
    k_fasta_marks<<<(unsigned)nt, NT, 0, s>>>(fa, n, tile_last_nl, tile_first_hdr);
    k_first_header<<<1, 1024, 0, s>>>(tile_first_hdr, nt, first_hdr);
    return hipGetLastError();
}

hipError_t launch_fasta_count(const uint8_t *fa, uint64_t n, const int64_t *tile_prev_nl,
                              const unsigned long long *first_hdr, uint64_t *tile_kept, hipStream_t s) {
    const uint64_t nt = (n + ENC_TILE - 1) / ENC_TILE;
    if (nt == 0) return hipSuccess;
    k_fasta_count<<<(unsigned)nt, NT, 0, s>>>(fa, n, tile_prev_nl, first_hdr, tile_kept);
    return hipGetLastError();
}

hipError_t launch_fasta_encode(const uint8_t *fa, uint64_t n, const int64_t *tile_prev_nl,
                               const unsigned long long *first_hdr, const uint64_t *tile_off, uint32_t *codes,
                               uint32_t *valid, hipStream_t s) {
    const uint64_t nt = (n + ENC_TILE - 1) / ENC_TILE;
    if (nt == 0) return hipSuccess;
    k_fasta_encode<<<(unsigned)nt, NT, 0, s>>>(fa, n, tile_prev_nl, first_hdr, tile_off, codes, valid);
    return hipGetLastError();
}

#include "fk_signature.inc"
#include "fk_records.inc"
#include "fk_partition.inc"
#include "fk_radix_rank.inc"
#include "fk_count_sorted.inc"
#include "fk_sort_radix.inc"
#include "fk_compact.inc"
#include "fk_count_hash.inc"
#include "fk_synth.inc"
}  // namespace fk
