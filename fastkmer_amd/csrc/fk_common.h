// fk_common.h -- host+device primitives of the k-mer hot path (gfx950).
//
// Each function names the reference code whose result it reproduces; the
// formulations are closed forms chosen for 64-wide wavefronts, not copies of
// the reference's loops (those are restated in oracle/fk_oracle.c).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define FK_HD __host__ __device__ __forceinline__

namespace fk {

typedef unsigned __int128 u128;

// A,C,G,T -> 0..3, anything else -> 4 (package.scala:18-22, :697).
FK_HD uint32_t base_code(uint8_t c) {
    // 'A'=0x41 'C'=0x43 'G'=0x47 'T'=0x54
    return c == 'A' ? 0u : c == 'C' ? 1u : c == 'G' ? 2u : c == 'T' ? 3u : 4u;
}

// is_allowed(mmer, m) (package.scala:46-75).  For m >= 3 the reference's
// loop + four checks reduce to: no two adjacent 'A' anywhere in the m-mer,
// and the m-mer does not start with "ACA".  For m < 3 the loop is empty and
// the four checks apply to the raw value.
FK_HD bool is_allowed(uint32_t v, int m) {
    if (m < 3) return !(v == 0 || v == 4 || (v & 0x3c) == 0 || (v & 0xf) == 0);
    const uint32_t cmask = (m == 16) ? 0xffffffffu : ((1u << (2 * m)) - 1u);
    const uint32_t za = ~(v | (v >> 1)) & 0x55555555u & cmask;  // bit 2j: char j (from LSB) is 'A'
    const bool aa_free = (za & (za >> 2)) == 0u;
    const bool aca = ((v >> (2 * (m - 3))) & 0x3fu) == 0x04u;
    return aa_free && !aca;
}

// reverse complement of a 2m-bit m-mer (package.scala:103-115).
FK_HD uint32_t revcomp_mmer(uint32_t v, int m) {
    uint32_t x = ~v;
#if defined(__HIP_DEVICE_COMPILE__)
    x = __builtin_bitreverse32(x);
#else
    x = ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
    x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
    x = ((x >> 4) & 0x0f0f0f0fu) | ((x & 0x0f0f0f0fu) << 4);
    x = ((x >> 8) & 0x00ff00ffu) | ((x & 0x00ff00ffu) << 8);
    x = (x >> 16) | (x << 16);
#endif
    x = ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);  // restore bit order inside each base
    return x >> (32 - 2 * m);
}

// fillNorm entry (package.scala:77-100): min over the two strands of the
// allowed value, 4^m when neither strand is allowed.
FK_HD uint32_t norm_mmer(uint32_t v, int m) {
    const uint32_t def = 1u << (2 * m);
    const uint32_t r = revcomp_mmer(v, m);
    const uint32_t a = is_allowed(v, m) ? v : def;
    const uint32_t b = is_allowed(r, m) ? r : def;
    return a < b ? a : b;
}

// Division by the runtime bin count without a divide instruction: the
// dividend of hash_to_bucket is < 2^31, so q = (a * mul) >> shift is exact
// with mul = ceil(2^(31+l) / d), l = ceil(log2 d)  (a*e < 2^(31+l)).
struct FastMod {
    uint32_t d, mul, shift;
};

inline FastMod make_fastmod(uint32_t d) {
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    FastMod f;
    f.d = d;
    f.shift = 31 + l;
    f.mul = (uint32_t)(((1ull << (31 + l)) + d - 1) / d);
    return f;
}

FK_HD uint32_t fastmod(uint32_t a, const FastMod &f) {
    const uint32_t q = (uint32_t)(((uint64_t)a * f.mul) >> f.shift);
    return a - q * f.d;
}

// hash_to_bucket (package.scala:686-695) in uint32 arithmetic, >>> = >>.
FK_HD uint32_t hash32(uint32_t key) {
    key = (key ^ 61u) ^ (key >> 16);
    key = key + (key << 3);
    key = key ^ (key >> 4);
    key = key * 0x27d4eb2du;
    key = key ^ (key >> 15);
    return key & 0x7fffffffu;
}

FK_HD uint32_t bin_of_signature(uint32_t sig, const FastMod &f) { return fastmod(hash32(sig), f); }

// 6-bit "fine" hash of a signature, kept in record header bits 26..31: the
// LDS hash count splits a bin's records into groups by it, and every
// occurrence of a canonical k-mer has the same signature (the norm is
// strand-symmetric), so a k-mer's occurrences all land in one group.
// The top six bits of the 31-bit bin hash: no second multiply per record (the bin takes hash32's
// low bits for a power-of-two B, its residue otherwise).
FK_HD uint32_t fine_of_signature(uint32_t sig) { return hash32(sig) >> 25; }

// ---- canonical k-mers (getOrientation + readFromKmer, package.scala:721-728,
// 174-295): canonical = min(forward, reverse complement) as 2k-bit integers,
// A=0..T=3, most significant base first.

FK_HD uint64_t pairswap64(uint64_t x) {
    return ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
}

FK_HD uint64_t bitrev64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bitreverse64(x);
#else
    x = ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
    x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
    x = ((x >> 4) & 0x0f0f0f0f0f0f0f0full) | ((x & 0x0f0f0f0f0f0f0f0full) << 4);
    x = ((x >> 8) & 0x00ff00ff00ff00ffull) | ((x & 0x00ff00ff00ff00ffull) << 8);
    x = ((x >> 16) & 0x0000ffff0000ffffull) | ((x & 0x0000ffff0000ffffull) << 16);
    return (x >> 32) | (x << 32);
#endif
}

// reverse complement of a k-mer held in the low 2k bits (k <= 32)
FK_HD uint64_t revcomp64(uint64_t fwd, int k) { return pairswap64(bitrev64(~fwd)) >> (64 - 2 * k); }

// k in 33..64: 128-bit key (hi = first k-32 bases, lo = last 32 bases)
FK_HD u128 revcomp128(u128 fwd, int k) {
    const uint64_t lo = (uint64_t)fwd, hi = (uint64_t)(fwd >> 64);
    const uint64_t rlo = pairswap64(bitrev64(~hi));  // reversed hi -> low word of the 128-bit reversal
    const uint64_t rhi = pairswap64(bitrev64(~lo));
    const u128 r = ((u128)rhi << 64) | rlo;
    return r >> (128 - 2 * k);
}

// ---- deterministic synthetic reads ----------------

FK_HD uint64_t splitmix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

struct SynthParams {
    uint64_t first_read, n_reads, genome_len, seed;
    uint32_t read_len, rec_bytes;
    uint64_t err_thresh, n_thresh;  // probabilities scaled to 2^64
};

// byte `idx` (relative to first_read's record) of the synthetic FASTA:
// record r = ">r%010d\n" + read_len bases + "\n".  Reads are drawn from a
// virtual uniform i.i.d. genome (base(p) = hash(seed, p) & 3), half of them
// reverse-complemented, with substitution errors and 'N's.
FK_HD uint8_t synth_byte(const SynthParams &p, uint64_t idx) {
    const uint64_t rr = idx / p.rec_bytes;
    const uint32_t off = (uint32_t)(idx - rr * p.rec_bytes);
    const uint64_t r = p.first_read + rr;
    if (off == 0) return '>';
    if (off == 1) return 'r';
    if (off < 12) {
        uint64_t v = r;
        for (uint32_t d = 11; d > off; --d) v /= 10;
        return (uint8_t)('0' + (v % 10));
    }
    if (off == 12 || off == p.rec_bytes - 1) return '\n';
    const uint32_t t = off - 13;
    const uint64_t h = splitmix64(p.seed ^ splitmix64(r * 0x100000001b3ull + 17));
    const uint64_t span = p.genome_len > p.read_len ? p.genome_len - p.read_len + 1 : 1;
    const uint64_t start = h % span;
    const bool rev = (h >> 63) & 1;
    const uint64_t gp = start + (rev ? (p.read_len - 1 - t) : t);
    uint32_t b = (uint32_t)(splitmix64(p.seed * 0x9e3779b97f4a7c15ull + gp) & 3);
    if (rev) b = 3 - b;
    const uint64_t e = splitmix64(h ^ (0xd1b54a32d192ed03ull * (t + 1)));
    if (e < p.n_thresh) return 'N';
    if (e < p.n_thresh + p.err_thresh) b = (b + 1 + (uint32_t)((e >> 32) % 3)) & 3;
    return "ACGT"[b];
}

}  // namespace fk
