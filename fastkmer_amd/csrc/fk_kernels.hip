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

#include <limits>
#include <type_traits>

#include "fk_internal.h"

namespace fk {

constexpr int NT = 256;  // threads per workgroup (4 waves)

// ---------------------------------------------------------------------------
// block-level helpers (256 threads)
// ---------------------------------------------------------------------------

// Wave-wide inclusive scans on DPP lane moves (row_shr within 16-lane rows,
// then row_bcast:15 / row_bcast:31 across rows): no LDS round trips.
// Lanes without a source keep `old` (the identity).
template <int CTRL, int ROWM>
__device__ __forceinline__ uint32_t dpp32(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROWM, 0xf, false);
}
template <int CTRL, int ROWM, typename T>
__device__ __forceinline__ T dpp_move(T ident, T v) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32- or 64-bit scan values");
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, dpp32<CTRL, ROWM>(__builtin_bit_cast(uint32_t, ident), __builtin_bit_cast(uint32_t, v)));
    } else {
        const uint64_t i = __builtin_bit_cast(uint64_t, ident), x = __builtin_bit_cast(uint64_t, v);
        const uint32_t lo = dpp32<CTRL, ROWM>((uint32_t)i, (uint32_t)x);
        const uint32_t hi = dpp32<CTRL, ROWM>((uint32_t)(i >> 32), (uint32_t)(x >> 32));
        return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
    }
}
template <typename T, class F>
__device__ __forceinline__ T wave_incl_scan(T v, T ident, F op) {
    v = op(v, dpp_move<0x111, 0xf>(ident, v));  // row_shr:1
    v = op(v, dpp_move<0x112, 0xf>(ident, v));  // row_shr:2
    v = op(v, dpp_move<0x114, 0xf>(ident, v));  // row_shr:4
    v = op(v, dpp_move<0x118, 0xf>(ident, v));  // row_shr:8
    v = op(v, dpp_move<0x142, 0xa>(ident, v));  // row_bcast:15 -> rows 1, 3
    v = op(v, dpp_move<0x143, 0xc>(ident, v));  // row_bcast:31 -> rows 2, 3
    return v;
}

template <typename T>
__device__ __forceinline__ T wave_incl_sum(T v) {
    return wave_incl_scan<T>(v, (T)0, [](T a, T b) { return a + b; });
}

template <typename T>
__device__ __forceinline__ T wave_incl_max(T v) {
    return wave_incl_scan<T>(v, std::numeric_limits<T>::lowest(), [](T a, T b) { return a > b ? a : b; });
}

// exclusive block prefix sum; *total receives the block sum (all threads)
// TRAIL = false drops the closing barrier: only when s_tmp is not written
// again by the workgroup before every thread has read it (its own array)
template <typename T, bool TRAIL = true, int NTH = NT>
__device__ __forceinline__ T block_excl_sum(T v, T *s_tmp /*[NTH / 64]*/, T *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    T inc = wave_incl_sum(v);
    if (lane == 63) s_tmp[wid] = inc;
    __syncthreads();
    T off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NTH / 64; ++w) {
        T x = s_tmp[w];
        if (w < wid) off += x;
        tot += x;
    }
    if constexpr (TRAIL) __syncthreads();
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

struct LbSum {
    static constexpr uint64_t ident = 0;
    __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return a + b; }
};

// Called by one whole wave.  Publishes `agg` for `tile`, returns the
// combination (commutative, associative `op`) of the aggregates of tiles
// 0..tile-1 and publishes the inclusive value.  Values stay below 2^62.
// Tiles are dispatched in blockIdx order, so every predecessor is resident
// or finished and the spin terminates.
// The two halves can be split (lookback_publish early, lookback_resolve once
// the prefix is needed) so the wait overlaps the tile's own work.
__device__ __forceinline__ void lookback_publish(uint64_t *status, uint64_t tile, uint64_t agg) {
    if ((threadIdx.x & 63) == 0) lb_store(&status[tile], (tile == 0 ? LB_INC : LB_AGG) | agg);
}

template <class Op>
__device__ uint64_t lookback_resolve(uint64_t *status, uint64_t tile, uint64_t agg, Op op) {
    const int lane = threadIdx.x & 63;
    if (tile == 0) return Op::ident;
    uint64_t excl = Op::ident;
    int64_t pos = (int64_t)tile - 1;
    while (true) {
        const int64_t q = pos - lane;
        const uint64_t st = q >= 0 ? lb_load(&status[q]) : (LB_INC | Op::ident);  // before tile 0
        const uint32_t flag = (uint32_t)(st >> 62);
        const uint64_t inc_mask = __ballot(flag == 2u);
        const uint64_t zero_mask = __ballot(flag == 0u);
        const int first_inc = inc_mask ? __builtin_ctzll(inc_mask) : 64;
        const uint64_t before = first_inc == 64 ? ~0ull : ((1ull << first_inc) - 1ull);
        if (zero_mask & before) {
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        uint64_t v = lane <= first_inc ? (st & LB_VAL) : Op::ident;
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) v = op(v, (uint64_t)__shfl_xor(v, d, 64));
        excl = op(excl, v);
        if (first_inc < 64) break;
        pos -= 64;
    }
    if (lane == 0) lb_store(&status[tile], LB_INC | op(excl, agg));
    return excl;
}

template <class Op>
__device__ uint64_t lookback_excl(uint64_t *status, uint64_t tile, uint64_t agg, Op op) {
    lookback_publish(status, tile, agg);
    return lookback_resolve(status, tile, agg, op);
}

// exclusive block prefix max (identity `ident`)
template <typename T, bool TRAIL = true, int NTH = NT>
__device__ __forceinline__ T block_excl_max(T v, T ident, T *s_tmp /*[NTH / 64]*/, T *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    T inc = wave_incl_max(v);
    const T exc = dpp_move<0x138, 0xf>(ident, inc);  // wave_shr:1 (lane 0 keeps ident)
    if (lane == 63) s_tmp[wid] = inc;
    __syncthreads();
    T off = ident, tot = ident;
#pragma unroll
    for (int w = 0; w < NTH / 64; ++w) {
        T x = s_tmp[w];
        if (w < wid) off = x > off ? x : off;
        tot = x > tot ? x : tot;
    }
    if constexpr (TRAIL) __syncthreads();
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

template <typename TI, typename TO, typename Op, bool IS_MAX>
__global__ __launch_bounds__(NT) void k_scan_reduce(const TI *in, uint64_t n, TO *sums, TO ident, Op op) {
    __shared__ TO s_tmp[NT / 64];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_SEG;
    TO acc = ident;
#pragma unroll
    for (int i = 0; i < SCAN_IPT; ++i) {
        uint64_t idx = base + (uint64_t)i * NT + threadIdx.x;
        if (idx < n) acc = op(acc, (TO)in[idx]);
    }
    // wave reductions + one barrier (the block scans' totals), not an LDS tree
    TO tot;
    if constexpr (IS_MAX)
        (void)block_excl_max<TO, false>(acc, ident, s_tmp, &tot);
    else
        (void)block_excl_sum<TO, false>(acc, s_tmp, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// exclusive scan of one segment with a carry-in (carry[blockIdx] or ident)
template <typename TI, typename TO, typename Op, bool IS_MAX>
__global__ __launch_bounds__(NT) void k_scan_down(const TI *in, TO *out, uint64_t n, const TO *carry, TO ident,
                                                  Op op, TO *total) {
    __shared__ TO s_tmp[NT / 64];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_SEG + (uint64_t)threadIdx.x * SCAN_IPT;
    static_assert(sizeof(TI) * SCAN_IPT % 16 == 0 && sizeof(TO) * SCAN_IPT % 16 == 0, "16-B segments");
    // a thread owns SCAN_IPT consecutive elements: 16-B loads and stores when
    // its segment is whole and both arrays are 16-B aligned (scalar accesses
    // at a 32-64 B lane stride touch every line SCAN_IPT times)
    const bool vec = base + SCAN_IPT <= n && ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
    TO v[SCAN_IPT];
    TO acc = ident;
    if (vec) {
        union {
            TI t[SCAN_IPT];
            uint4 q[sizeof(TI) * SCAN_IPT / 16];
        } u;
#pragma unroll
        for (int i = 0; i < (int)(sizeof(TI) * SCAN_IPT / 16); ++i) u.q[i] = reinterpret_cast<const uint4 *>(in + base)[i];
#pragma unroll
        for (int i = 0; i < SCAN_IPT; ++i) {
            v[i] = (TO)u.t[i];
            acc = op(acc, v[i]);
        }
    } else {
#pragma unroll
        for (int i = 0; i < SCAN_IPT; ++i) {
            uint64_t idx = base + i;
            v[i] = idx < n ? (TO)in[idx] : ident;
            acc = op(acc, v[i]);
        }
    }
    TO tot;
    TO pre;
    if constexpr (IS_MAX) {
        pre = block_excl_max<TO>(acc, ident, s_tmp, &tot);
    } else {
        pre = block_excl_sum<TO>(acc, s_tmp, &tot);
    }
    TO run = op(carry ? carry[blockIdx.x] : ident, pre);
    if (vec) {
        union {
            TO t[SCAN_IPT];
            uint4 q[sizeof(TO) * SCAN_IPT / 16];
        } u;
#pragma unroll
        for (int i = 0; i < SCAN_IPT; ++i) {
            u.t[i] = run;
            run = op(run, v[i]);
        }
#pragma unroll
        for (int i = 0; i < (int)(sizeof(TO) * SCAN_IPT / 16); ++i) reinterpret_cast<uint4 *>(out + base)[i] = u.q[i];
    } else {
#pragma unroll
        for (int i = 0; i < SCAN_IPT; ++i) {
            uint64_t idx = base + i;
            if (idx < n) out[idx] = run;
            run = op(run, v[i]);
        }
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
    k_scan_reduce<TI, TO, Op, IS_MAX><<<(unsigned)nb, NT, 0, s>>>(in, n, sums, ident, Op());
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

#include "fk_parse.inc"
#include "fk_signature.inc"
#include "fk_map_fused.inc"
#include "fk_records.inc"
#include "fk_partition.inc"
#include "fk_radix_rank.inc"
#include "fk_count_sorted.inc"
#include "fk_expand2.inc"
#include "fk_sort_radix.inc"
#include "fk_compact.inc"
#include "fk_synth.inc"
#include "fk_format.inc"
#include "fk_bin_signatures.inc"

// Test hook of the failure semantics (fk_debug_comm_hold): one thread spins on a host-mapped flag
// with s_sleep between its system-scope loads, and leaves by itself after max_ticks of the 100 MHz
// wall clock, so the stream it holds always drains.
__global__ void __launch_bounds__(64) k_hold_stream(const uint32_t *flag, uint64_t max_ticks) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
        if (wall_clock64() - t0 > max_ticks) break;
        __builtin_amdgcn_s_sleep(127);
    }
}

hipError_t launch_hold_stream(const uint32_t *flag, uint64_t max_ticks, hipStream_t s) {
    hipLaunchKernelGGL(k_hold_stream, dim3(1), dim3(64), 0, s, flag, max_ticks);
    return hipGetLastError();
}
}  // namespace fk
