/*
 * fk_oracle.c -- CPU restatement of the reference k-mer counting algorithm.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product library (fastkmer_amd/csrc) never links, calls or falls back to it.
 *
 * It restates, in plain C, the hot path of maruscia/fastkmer (Scala/Spark):
 *   - util.is_allowed            src/main/scala/skc/package.scala:46-75
 *   - util.fillNorm              src/main/scala/skc/package.scala:77-100
 *   - util.reverse_complement    src/main/scala/skc/package.scala:103-115
 *   - Kmer.getSignature          src/main/scala/skc/package.scala:337-357
 *   - Kmer.lastM                 src/main/scala/skc/package.scala:310-326
 *   - util.hash_to_bucket        src/main/scala/skc/package.scala:686-695
 *   - util.getOrientation(Kmer)  src/main/scala/skc/package.scala:721-728
 *   - firstAndLastOccurrenceOfInvalidNucleotide  package.scala:739-754
 *   - SparkBinKmerCounter.getSuperKmers          SparkBinKmerCounter.scala:34-169
 *   - extractKXmers (sorted count + "EOF")       SparkBinKmerCounter.scala:428-660
 *   - extractKXmersHT (hash count, no "EOF")     SparkBinKmerCounter.scala:664-739
 *   - TestConfiguration.b = min(4^m, B)          src/main/scala/skc/test/package.scala:32
 *   - read = record value with '\n' removed      SparkBinKmerCounter.scala:62-65
 *   - getBinSignatures / saveBinSignatures       SparkBinKmerCounter.scala:772-953
 *     (bin-signature diagnostics), longToString  package.scala:616-634
 *
 * Control flow of the map side (getSuperKmers) is kept step for step,
 * including the O(k) invalid-byte scan per window, the O(k) signature
 * recomputation when the minimizer expires and the strict "<" slide, so the
 * super-k-mers and bins it produces are the reference's.  The reduce side
 * counts canonical k-mers per bin exactly; the (k,x)-mer packing and heap
 * merge of extractKXmers are a memory layout of the same multiset (the
 * literal transliteration in oracle/literal_ref.py checks that claim).
 *
 * k-mers are held as unsigned __int128, 2 bits per base, MSB-first (A=0, C=1,
 * G=2, T=3; package.scala:18-22), so numeric order == lexicographic order
 * (Kmer.compare, package.scala:389-404).  k <= 64 is supported.
 *
 * FASTA record semantics (FASTdoop 1.0 is not in /root/reference; SURVEY
 * Appendix A): a header line starts with '>' at a line start; the read is the
 * concatenation of the following non-header lines with every '\n' removed;
 * every other byte ('\r', 'N', lowercase, IUPAC) stays in the read and breaks
 * k-mer windows.  Lines before the first header are ignored.  With
 * sequence_type == 1 (FASTAlongInputFileFormat) each record is one long read
 * (the reference's chunks overlap by k-1, SBKC:993, which gives the same
 * counts as counting the whole record).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <errno.h>
#include <sys/stat.h>
#include <pthread.h>

typedef unsigned __int128 u128;

#define FKO_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------ */
/* primitives                                                          */
/* ------------------------------------------------------------------ */

/* package.scala:18-22 -- A,C,G,T -> 0..3; everything else is "not a
 * nucleotide" (package.scala:697). */
static inline int fko_code(uint8_t c) {
    switch (c) {
        case 'A': return 0;
        case 'C': return 1;
        case 'G': return 2;
        case 'T': return 3;
        default: return -1;
    }
}

/* package.scala:46-75, literally: the loop runs length-3 times on the low
 * 4 bits, then four checks on what is left of the m-mer. */
FKO_API int fko_is_allowed(int32_t mmer_in, int32_t length) {
    int32_t mmer = mmer_in;
    for (int j = 0; j < length - 3; ++j) {
        if ((mmer & 0xf) == 0) return 0; /* AA inside */
        mmer >>= 2;
    }
    if (mmer == 0) return 0;          /* AAA prefix */
    if (mmer == 0x04) return 0;       /* ACA prefix */
    if ((mmer & 0x3c) == 0) return 0; /* AA* prefix */
    if ((mmer & 0xf) == 0) return 0;  /* *AA prefix */
    return 1;
}

/* package.scala:103-115 */
FKO_API int64_t fko_reverse_complement(int64_t seq, int32_t length) {
    int64_t cur = seq, rev = 0;
    int shift = length * 2 - 2;
    for (int i = 0; i < length; ++i) {
        rev += (int64_t)(3 - (cur & 3)) << shift;
        cur >>= 2;
        shift -= 2;
    }
    return rev;
}

/* one entry of fillNorm (package.scala:77-100) */
FKO_API int32_t fko_norm(int32_t v, int32_t m) {
    int32_t def = 1 << (m * 2);
    int32_t rev = (int32_t)fko_reverse_complement(v, m);
    int32_t sv = fko_is_allowed(v, m) ? v : def;
    int32_t rv = fko_is_allowed(rev, m) ? rev : def;
    return sv < rv ? sv : rv;
}

/* package.scala:686-695 (Java int arithmetic, >>> = logical shift) */
FKO_API int32_t fko_hash_to_bucket(int32_t s, int32_t B) {
    uint32_t key = (uint32_t)s;
    const uint32_t c2 = 0x27d4eb2du;
    key = (key ^ 61u) ^ (key >> 16);
    key = key + (key << 3);
    key = key ^ (key >> 4);
    key = key * c2;
    key = key ^ (key >> 15);
    return (int32_t)((key & 0x7FFFFFFFu) % (uint32_t)B);
}

/* test/package.scala:32: b = min(4^m, max_b) computed in double */
FKO_API int32_t fko_clamp_bins(int32_t m, int32_t B) {
    double p = 1.0;
    for (int i = 0; i < m; ++i) p *= 4.0;
    double b = p < (double)B ? p : (double)B;
    return (int32_t)b;
}

/* ------------------------------------------------------------------ */
/* result container                                                    */
/* ------------------------------------------------------------------ */

typedef struct {
    u128 *keys;
    uint32_t *counts; /* filled after reduction */
    int64_t n, cap;
} fko_bin;

typedef struct fko_result {
    int32_t k, m, nbins;
    fko_bin *bins;
    int64_t total_kmers;
    int64_t superkmers;
    int64_t reads;
    /* optional super-k-mer trace (fko_trace_read) */
    int64_t *trace_start, *trace_len;
    int32_t *trace_bin;
    int64_t trace_cap;
} fko_result;

static void bin_push(fko_bin *b, u128 key) {
    if (b->n == b->cap) {
        int64_t nc = b->cap ? b->cap * 2 : 64;
        u128 *nk = (u128 *)realloc(b->keys, (size_t)nc * sizeof(u128));
        if (!nk) { fprintf(stderr, "fk_oracle: out of memory\n"); abort(); }
        b->keys = nk;
        b->cap = nc;
    }
    b->keys[b->n++] = key;
}

/* ------------------------------------------------------------------ */
/* map side: getSuperKmers (SparkBinKmerCounter.scala:34-169)          */
/* ------------------------------------------------------------------ */

typedef struct {
    int32_t k, m, B;
    const int32_t *norm; /* fillNorm table, or NULL -> computed per call */
    int32_t bin_mod, bin_rem; /* keep only bins b with b % bin_mod == bin_rem (bin_mod 0: every bin);
                                 a checker's memory bound at large sizes, not part of the reference */
} fko_params;

static inline int32_t norm_of(const fko_params *p, int32_t v) {
    return p->norm ? p->norm[v] : fko_norm(v, p->m);
}

/* value of the m-mer of cur starting at pos (all bytes valid by caller) */
static inline int32_t mmer_at(const uint8_t *cur, int64_t pos, int m) {
    int32_t v = 0;
    for (int t = 0; t < m; ++t) v = (v << 2) | fko_code(cur[pos + t]);
    return v;
}

/* Kmer.getSignature (package.scala:337-357): leftmost strict minimum of
 * norm over the k-m+1 m-mers of the k-mer that starts at read offset i.
 * Returns the value; *pos receives the m-mer's offset inside the k-mer. */
static int32_t get_signature(const fko_params *p, const uint8_t *cur, int64_t i, int32_t *pos) {
    int32_t sig = norm_of(p, mmer_at(cur, i, p->m));
    *pos = 0;
    for (int t = 1; t + p->m <= p->k; ++t) {
        int32_t v = norm_of(p, mmer_at(cur, i + t, p->m));
        if (v < sig) { sig = v; *pos = t; }
    }
    return sig;
}

/* firstAndLastOccurrenceOfInvalidNucleotide (package.scala:739-754):
 * offsets relative to start, (-1,-1) when the range is all ACGT. */
static void first_last_invalid(const uint8_t *s, int64_t start, int64_t end, int64_t *first, int64_t *last) {
    *first = -1;
    *last = -1;
    for (int64_t i = start; i < end; ++i) {
        if (fko_code(s[i]) < 0) {
            if (*first == -1) *first = i - start;
            *last = i - start;
        }
    }
}

/* getOrientation(Kmer, i, j) (package.scala:721-728) on read bytes:
 * 0 = forward strand is lexicographically smaller, 1 = reverse complement
 * (ties -> 1; a palindrome is its own reverse complement). */
static int orientation(const uint8_t *s, int64_t i, int64_t j) {
    for (;;) {
        int a = fko_code(s[i]);
        int b = 3 - fko_code(s[j]);
        if (a < b) return 0;
        if (a > b || i >= j) return 1;
        ++i;
        --j;
    }
}

/* canonical k-mer of read bytes [i, i+k) via the orientation rule and the
 * (orientation==1 => reverse complement) copy of Kmer.readFromKmer
 * (package.scala:256-290). */
static u128 canonical_at(const uint8_t *s, int64_t i, int k) {
    u128 v = 0;
    if (orientation(s, i, i + k - 1) == 0) {
        for (int t = 0; t < k; ++t) v = (v << 2) | (u128)fko_code(s[i + t]);
    } else {
        for (int t = k - 1; t >= 0; --t) v = (v << 2) | (u128)(3 - fko_code(s[i + t]));
    }
    return v;
}

/* Emit one super-k-mer: on the reduce side (extractKXmers/HT) each of its
 * len-k+1 k-mers is canonicalised and counted in bin `bin`. */
static void emit_superkmer(fko_result *r, const fko_params *p, const uint8_t *cur, int64_t start, int64_t len, int32_t sig) {
    int32_t bin = fko_hash_to_bucket(sig, p->B);
    fko_bin *b = &r->bins[bin];
    if (r->trace_start && r->superkmers < r->trace_cap) {
        r->trace_start[r->superkmers] = start;
        r->trace_len[r->superkmers] = len;
        r->trace_bin[r->superkmers] = bin;
    }
    if (p->bin_mod > 0 && bin % p->bin_mod != p->bin_rem) { /* filtered out: counted, not kept */
        r->total_kmers += len - p->k + 1;
        r->superkmers++;
        return;
    }
    for (int64_t i = start; i + p->k <= start + len; ++i) {
        bin_push(b, canonical_at(cur, i, p->k));
        r->total_kmers++;
    }
    r->superkmers++;
}

/* SparkBinKmerCounter.scala:59-161 for one read `cur` of length n. */
static void get_super_kmers_read(fko_result *r, const fko_params *p, const uint8_t *cur, int64_t n) {
    const int k = p->k, m = p->m;
    if (n < k) return; /* :67 */
    int32_t min_value = -1;
    int64_t min_pos = -1; /* Signature(-1,-1), :69 */
    int64_t sk_start = 0;
    int64_t i = 0;
    int64_t nf, nl;
    while (i < n - k + 1) {                           /* :75 */
        first_last_invalid(cur, i, i + k, &nf, &nl); /* :78 */
        if (nf != -1) {
            if (sk_start < i) /* :84-89 */
                emit_superkmer(r, p, cur, sk_start, i - 1 + k - sk_start, min_value);
            sk_start = i + nl + 1; /* :95 */
            i += nl + 1;           /* :96 */
        } else {
            if (i > min_pos) { /* :102 minimizer left the window */
                if (sk_start < i) {
                    emit_superkmer(r, p, cur, sk_start, i - 1 + k - sk_start, min_value); /* :104 */
                    sk_start = i;
                }
                int32_t rel;
                min_value = get_signature(p, cur, i, &rel); /* :112 */
                min_pos = rel + i;
            } else {
                int32_t last = norm_of(p, mmer_at(cur, i + k - m, m)); /* lastM, :117 */
                if (last < min_value) {                                 /* :119 strict */
                    if (sk_start < i) {
                        emit_superkmer(r, p, cur, sk_start, i - 1 + k - sk_start, min_value); /* :124 */
                        sk_start = i;
                    }
                    min_value = last; /* :132 */
                    min_pos = i + k - m;
                }
            }
            i += 1;
        }
    }
    if (n - sk_start >= k) { /* :142 */
        first_last_invalid(cur, i, n, &nf, &nl);
        if (nf == -1) {
            emit_superkmer(r, p, cur, sk_start, n - sk_start, min_value); /* :148 */
        } else if (i + nf >= sk_start + k) {                              /* :152 (unreachable) */
            emit_superkmer(r, p, cur, sk_start, i + nf, min_value);
        }
    }
}

/* ------------------------------------------------------------------ */
/* FASTA records (SBKC:62-65 + FASTdoop semantics, Appendix A)          */
/* ------------------------------------------------------------------ */

typedef void (*read_cb)(void *ctx, const uint8_t *read, int64_t n);

static void for_each_read(const uint8_t *buf, size_t n, read_cb cb, void *ctx) {
    uint8_t *read = NULL;
    int64_t rn = 0, rcap = 0;
    int in_record = 0;
    size_t pos = 0;
    while (pos < n) {
        size_t e = pos;
        while (e < n && buf[e] != '\n') ++e; /* line [pos, e) */
        if (e > pos && buf[pos] == '>') {
            if (in_record) cb(ctx, read, rn);
            in_record = 1;
            rn = 0;
        } else if (in_record) {
            int64_t len = (int64_t)(e - pos);
            if (rn + len > rcap) {
                int64_t nc = rcap ? rcap : 256;
                while (nc < rn + len) nc *= 2;
                uint8_t *nr = (uint8_t *)realloc(read, (size_t)nc);
                if (!nr) { fprintf(stderr, "fk_oracle: out of memory\n"); abort(); }
                read = nr;
                rcap = nc;
            }
            memcpy(read + rn, buf + pos, (size_t)len);
            rn += len;
        }
        pos = e + 1;
    }
    if (in_record) cb(ctx, read, rn);
    free(read);
}

typedef struct {
    fko_result *r;
    fko_params *p;
} map_ctx;

static void map_read(void *vctx, const uint8_t *read, int64_t n) {
    map_ctx *c = (map_ctx *)vctx;
    c->r->reads++;
    get_super_kmers_read(c->r, c->p, read, n);
}

/* ------------------------------------------------------------------ */
/* reduce side: exact multiplicity per canonical k-mer per bin          */
/* ------------------------------------------------------------------ */

static int cmp_u128(const void *a, const void *b) {
    u128 x = *(const u128 *)a, y = *(const u128 *)b;
    return x < y ? -1 : (x > y ? 1 : 0);
}

static void reduce_bin(fko_bin *b) {
    if (b->n == 0) return;
    qsort(b->keys, (size_t)b->n, sizeof(u128), cmp_u128);
    uint32_t *cnt = (uint32_t *)malloc((size_t)b->n * sizeof(uint32_t));
    int64_t u = 0;
    for (int64_t i = 0; i < b->n; ++i) {
        if (u > 0 && b->keys[u - 1] == b->keys[i]) {
            cnt[u - 1]++;
        } else {
            b->keys[u] = b->keys[i];
            cnt[u] = 1;
            ++u;
        }
    }
    b->n = u;
    b->counts = cnt;
}

/* Runs the whole job. B is the requested bin count; it is clamped to
 * min(4^m, B) exactly like TestConfiguration.b.  Returns NULL on invalid
 * parameters (the reference would throw). */
FKO_API fko_result *fko_count(const uint8_t *fasta, size_t n, int32_t k, int32_t m, int32_t B, int32_t sequence_type) {
    (void)sequence_type; /* same counts for both record formats (see header) */
    if (k < 1 || k > 64 || m < 1 || m > 15 || m > k || B < 1) return NULL;
    fko_params p;
    p.k = k;
    p.m = m;
    p.B = fko_clamp_bins(m, B);
    p.bin_mod = 0;
    p.bin_rem = 0;
    int32_t *norm = NULL;
    if (m <= 12) { /* fillNorm table (package.scala:77-100), per task (SBKC:47) */
        int64_t sz = (int64_t)1 << (2 * m);
        norm = (int32_t *)malloc((size_t)sz * sizeof(int32_t));
        for (int64_t v = 0; v < sz; ++v) norm[v] = fko_norm((int32_t)v, m);
    }
    p.norm = norm;
    fko_result *r = (fko_result *)calloc(1, sizeof(fko_result));
    r->k = k;
    r->m = m;
    r->nbins = p.B;
    r->bins = (fko_bin *)calloc((size_t)p.B, sizeof(fko_bin));
    map_ctx c = {r, &p};
    for_each_read(fasta, n, map_read, &c);
    for (int32_t b = 0; b < p.B; ++b) reduce_bin(&r->bins[b]);
    free(norm);
    return r;
}

/* ------------------------------------------------------------------ */
/* multi-threaded driver (the CPU baseline; the reference runs Spark    */
/* local[4], LocalTestKmerCounter.scala:62): the FASTA is cut at record  */
/* starts into one range per thread (map tasks over input splits), each  */
/* thread maps its range into private bins, then the bins are merged and */
/* reduced, bins dealt round-robin over the threads (reduce tasks).      */
/* Results are identical to fko_count.                                   */
/* ------------------------------------------------------------------ */

FKO_API void fko_free(fko_result *r);

typedef struct {
    const uint8_t *buf;
    size_t lo, hi;
    fko_params *p;
    fko_result *part;   /* map: this thread's bins */
    fko_result *out;    /* reduce: merged bins */
    fko_result **parts; /* reduce: all threads' bins */
    int32_t nthreads, tid;
} mt_task;

static void *mt_map(void *arg) {
    mt_task *t = (mt_task *)arg;
    map_ctx c = {t->part, t->p};
    for_each_read(t->buf + t->lo, t->hi - t->lo, map_read, &c);
    return NULL;
}

static void *mt_reduce(void *arg) {
    mt_task *t = (mt_task *)arg;
    for (int32_t b = t->tid; b < t->out->nbins; b += t->nthreads) {
        fko_bin *ob = &t->out->bins[b];
        int64_t n = 0;
        for (int32_t j = 0; j < t->nthreads; ++j) n += t->parts[j]->bins[b].n;
        if (!n) continue;
        ob->keys = (u128 *)malloc((size_t)n * sizeof(u128));
        if (!ob->keys) { fprintf(stderr, "fk_oracle: out of memory\n"); abort(); }
        ob->cap = n;
        for (int32_t j = 0; j < t->nthreads; ++j) {
            fko_bin *pb = &t->parts[j]->bins[b];
            if (pb->n) memcpy(ob->keys + ob->n, pb->keys, (size_t)pb->n * sizeof(u128));
            ob->n += pb->n;
            free(pb->keys);
            pb->keys = NULL;
            pb->n = 0;
        }
        reduce_bin(ob);
    }
    return NULL;
}

/* fko_count_mt keeping only the bins b % bin_mod == bin_rem (bin_mod 0: all): the other bins' k-mers
 * are walked and counted in total_kmers / superkmers but never canonicalised or stored, so a checker
 * holds 1 / bin_mod of a multi-GB job's keys (tests/test_gpu_configs.py, the configs[2] per-GPU load). */
FKO_API fko_result *fko_count_mt_filtered(const uint8_t *fasta, size_t n, int32_t k, int32_t m, int32_t B,
                                          int32_t sequence_type, int32_t nthreads, int32_t bin_mod, int32_t bin_rem) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if (k < 1 || k > 64 || m < 1 || m > 15 || m > k || B < 1) return NULL;
    if (bin_mod < 0 || (bin_mod > 0 && (bin_rem < 0 || bin_rem >= bin_mod))) return NULL;
    fko_params p;
    p.k = k;
    p.m = m;
    p.B = fko_clamp_bins(m, B);
    p.bin_mod = bin_mod;
    p.bin_rem = bin_rem;
    int32_t *norm = NULL;
    if (m <= 12) {
        int64_t sz = (int64_t)1 << (2 * m);
        norm = (int32_t *)malloc((size_t)sz * sizeof(int32_t));
        for (int64_t v = 0; v < sz; ++v) norm[v] = fko_norm((int32_t)v, m);
    }
    p.norm = norm;
    /* range starts: thread 0 at 0 (it also skips text before the first
     * header), the others at the first record start ('>' at a line start)
     * at or after j*n/T */
    size_t cut[257];
    cut[0] = 0;
    for (int32_t j = 1; j < nthreads; ++j) {
        size_t q = (size_t)((unsigned __int128)n * (unsigned)j / (unsigned)nthreads);
        if (q < cut[j - 1]) q = cut[j - 1];
        while (q < n && !(fasta[q] == '>' && q > 0 && fasta[q - 1] == '\n')) ++q;
        cut[j] = q;
    }
    cut[nthreads] = n;
    fko_result **parts = (fko_result **)calloc((size_t)nthreads, sizeof(fko_result *));
    mt_task *tasks = (mt_task *)calloc((size_t)nthreads, sizeof(mt_task));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    fko_result *r = (fko_result *)calloc(1, sizeof(fko_result));
    r->k = k;
    r->m = m;
    r->nbins = p.B;
    r->bins = (fko_bin *)calloc((size_t)p.B, sizeof(fko_bin));
    for (int32_t j = 0; j < nthreads; ++j) {
        parts[j] = (fko_result *)calloc(1, sizeof(fko_result));
        parts[j]->k = k;
        parts[j]->m = m;
        parts[j]->nbins = p.B;
        parts[j]->bins = (fko_bin *)calloc((size_t)p.B, sizeof(fko_bin));
        tasks[j] = (mt_task){fasta, cut[j], cut[j + 1], &p, parts[j], r, parts, nthreads, j};
        pthread_create(&th[j], NULL, mt_map, &tasks[j]);
    }
    for (int32_t j = 0; j < nthreads; ++j) pthread_join(th[j], NULL);
    for (int32_t j = 0; j < nthreads; ++j) {
        r->total_kmers += parts[j]->total_kmers;
        r->superkmers += parts[j]->superkmers;
        r->reads += parts[j]->reads;
    }
    for (int32_t j = 0; j < nthreads; ++j) pthread_create(&th[j], NULL, mt_reduce, &tasks[j]);
    for (int32_t j = 0; j < nthreads; ++j) pthread_join(th[j], NULL);
    for (int32_t j = 0; j < nthreads; ++j) fko_free(parts[j]);
    free(parts);
    free(tasks);
    free(th);
    free(norm);
    (void)sequence_type;
    return r;
}

FKO_API fko_result *fko_count_mt(const uint8_t *fasta, size_t n, int32_t k, int32_t m, int32_t B,
                                 int32_t sequence_type, int32_t nthreads) {
    return fko_count_mt_filtered(fasta, n, k, m, B, sequence_type, nthreads, 0, 0);
}

FKO_API int32_t fko_nbins(const fko_result *r) { return r->nbins; }
FKO_API int64_t fko_total_kmers(const fko_result *r) { return r->total_kmers; }
FKO_API int64_t fko_superkmers(const fko_result *r) { return r->superkmers; }
FKO_API int64_t fko_reads(const fko_result *r) { return r->reads; }

FKO_API int64_t fko_bin_size(const fko_result *r, int32_t b) {
    if (b < 0 || b >= r->nbins) return -1;
    return r->bins[b].n;
}

FKO_API int64_t fko_distinct(const fko_result *r) {
    int64_t s = 0;
    for (int32_t b = 0; b < r->nbins; ++b) s += r->bins[b].n;
    return s;
}

/* keys split as (hi, lo): lo = last 32 bases, hi = the first k-32 bases
 * (0 for k <= 32); counts are the Java Int counts. */
FKO_API int fko_bin_get(const fko_result *r, int32_t b, uint64_t *hi, uint64_t *lo, uint32_t *counts) {
    if (b < 0 || b >= r->nbins) return -1;
    const fko_bin *bb = &r->bins[b];
    for (int64_t i = 0; i < bb->n; ++i) {
        if (hi) hi[i] = (uint64_t)(bb->keys[i] >> 64);
        if (lo) lo[i] = (uint64_t)bb->keys[i];
        if (counts) counts[i] = bb->counts[i];
    }
    return 0;
}

/* Kmer.toString (package.scala:416-454, 496-500) */
static void key_to_string(u128 key, int k, char *out) {
    static const char rep[4] = {'A', 'C', 'G', 'T'};
    for (int t = k - 1; t >= 0; --t) {
        out[t] = rep[(int)(key & 3)];
        key >>= 2;
    }
    out[k] = 0;
}

/* Output files as extractKXmers (SBKC:550-606: sorted lines + "EOF", no
 * trailing newline) or extractKXmersHT (SBKC:715-734: lines only). */
FKO_API int fko_write_bins(const fko_result *r, const char *dir, int32_t sorted_eof) {
    if (mkdir(dir, 0755) != 0 && errno != EEXIST) return -1;
    char path[4096];
    char kmer[80];
    for (int32_t b = 0; b < r->nbins; ++b) {
        const fko_bin *bb = &r->bins[b];
        if (bb->n == 0) continue;
        snprintf(path, sizeof(path), "%s/bin%d", dir, b);
        FILE *f = fopen(path, "wb");
        if (!f) return -2;
        for (int64_t i = 0; i < bb->n; ++i) {
            key_to_string(bb->keys[i], r->k, kmer);
            fprintf(f, "%s\t%u\n", kmer, bb->counts[i]);
        }
        if (sorted_eof) fputs("EOF", f);
        fclose(f);
    }
    return 0;
}

FKO_API void fko_free(fko_result *r) {
    if (!r) return;
    for (int32_t b = 0; b < r->nbins; ++b) {
        free(r->bins[b].keys);
        free(r->bins[b].counts);
    }
    free(r->bins);
    free(r);
}

/* Super-k-mer trace for the literal cross-check: runs getSuperKmers on one
 * read and records (start, length, bin) of every emitted super-k-mer in
 * emission order.  Returns the number emitted (may exceed cap). */
FKO_API int64_t fko_trace_read(const uint8_t *read, int64_t n, int32_t k, int32_t m, int32_t B,
                               int64_t *out_start, int64_t *out_len, int32_t *out_bin, int64_t cap) {
    if (k < 1 || k > 64 || m < 1 || m > 15 || m > k || B < 1) return -1;
    fko_params p;
    p.k = k;
    p.m = m;
    p.B = fko_clamp_bins(m, B);
    p.norm = NULL;
    p.bin_mod = p.bin_rem = 0;
    fko_result r;
    memset(&r, 0, sizeof(r));
    r.k = k;
    r.m = m;
    r.nbins = p.B;
    r.bins = (fko_bin *)calloc((size_t)p.B, sizeof(fko_bin));
    r.trace_start = out_start;
    r.trace_len = out_len;
    r.trace_bin = out_bin;
    r.trace_cap = cap;
    get_super_kmers_read(&r, &p, read, n);
    for (int32_t b = 0; b < p.B; ++b) free(r.bins[b].keys);
    free(r.bins);
    return r.superkmers;
}

/* ------------------------------------------------------------------ */
/* bin-signature diagnostics: executeFindBinSignaturesJob               */
/* (SparkBinKmerCounter.scala:956-986)                                  */
/* ------------------------------------------------------------------ */

/* getBinSignatures (SBKC:772-917) for one read: the getSuperKmers walk
 * (same N jumps, expiry test and strict "<"), but each super-k-mer adds 1 to
 * counts[signature] (the out(bin) HashMap update of :828-830, :844-846,
 * :868-870, :890-899) instead of emitting k-mers.  The bin and the
 * signature string are functions of the value, applied by the writer. */
static void bin_signatures_read(int64_t *counts, const fko_params *p, const uint8_t *cur, int64_t n) {
    const int k = p->k, m = p->m;
    if (n < k) return; /* :810 */
    int32_t min_value = -1;
    int64_t min_pos = -1; /* Signature(-1,-1), :812 */
    int64_t sk_start = 0, i = 0, nf, nl;
    while (i < n - k + 1) {                           /* :818 */
        first_last_invalid(cur, i, i + k, &nf, &nl); /* :820 */
        if (nf != -1) {
            if (sk_start < i) counts[min_value]++; /* :826-830 */
            sk_start = i + nl + 1;                  /* :835 */
            i += nl + 1;                            /* :836 */
        } else {
            if (i > min_pos) { /* :842 */
                if (sk_start < i) {
                    counts[min_value]++; /* :843-846 */
                    sk_start = i;
                }
                int32_t rel;
                min_value = get_signature(p, cur, i, &rel); /* :854 */
                min_pos = rel + i;
            } else {
                int32_t last = norm_of(p, mmer_at(cur, i + k - m, m)); /* :861 */
                if (last < min_value) {                                 /* :863 */
                    if (sk_start < i) {
                        counts[min_value]++; /* :866-870 */
                        sk_start = i;
                    }
                    min_value = last; /* :876 */
                    min_pos = i + k - m;
                }
            }
            i += 1;
        }
    }
    if (n - sk_start >= k) { /* :886 */
        first_last_invalid(cur, i, n, &nf, &nl);
        if (nf == -1 || i + nf >= sk_start + k) counts[min_value]++; /* :892-902 */
    }
}

typedef struct {
    int64_t *counts;
    fko_params *p;
} sig_ctx;

static void sig_read(void *vctx, const uint8_t *read, int64_t n) {
    sig_ctx *c = (sig_ctx *)vctx;
    bin_signatures_read(c->counts, c->p, read, n);
}

/* counts[0 .. 4^m] (zeroed here): super-k-mers per signature value over all
 * reads of the FASTA, i.e. the per-bin HashMaps of getBinSignatures merged by
 * the reduceByKey of SBKC:984.  Returns 0, or -1 on invalid parameters. */
FKO_API int fko_bin_signatures(const uint8_t *fasta, size_t n, int32_t k, int32_t m, int64_t *counts) {
    if (k < 1 || k > 64 || m < 1 || m > 15 || m > k || !counts) return -1;
    fko_params p;
    p.k = k;
    p.m = m;
    p.B = 1;
    p.norm = NULL;
    p.bin_mod = p.bin_rem = 0;
    memset(counts, 0, (((size_t)1 << (2 * m)) + 1) * sizeof(int64_t));
    sig_ctx c = {counts, &p};
    for_each_read(fasta, n, sig_read, &c);
    return 0;
}

/* saveBinSignatures (SBKC:920-953) for every bin with a signature:
 * <dir>/bin_signatures<b>.txt, "<longToString(v)>\t<count>\n" per signature
 * (longToString, PKG:616-634: 31 characters whatever m) and "Total\t<sum>\n".
 * The reference iterates an immutable HashMap (order unspecified); lines are
 * written in ascending signature value.  B is the requested bin count. */
FKO_API int fko_write_bin_signatures(const int64_t *counts, int32_t m, int32_t B, const char *dir) {
    if (m < 1 || m > 15 || B < 1) return -1;
    if (mkdir(dir, 0755) != 0 && errno != EEXIST) return -1;
    const int32_t nb = fko_clamp_bins(m, B);
    const int64_t slots = ((int64_t)1 << (2 * m)) + 1;
    /* signatures grouped by bin(min_s.value) (:777), ascending inside a bin */
    int64_t *start = (int64_t *)calloc((size_t)nb + 1, sizeof(int64_t));
    int64_t nz = 0;
    for (int64_t v = 0; v < slots; ++v)
        if (counts[v]) { start[fko_hash_to_bucket((int32_t)v, nb) + 1]++; ++nz; }
    for (int32_t b = 0; b < nb; ++b) start[b + 1] += start[b];
    int64_t *order = (int64_t *)malloc((size_t)(nz ? nz : 1) * sizeof(int64_t));
    int64_t *fill = (int64_t *)malloc((size_t)nb * sizeof(int64_t));
    memcpy(fill, start, (size_t)nb * sizeof(int64_t));
    for (int64_t v = 0; v < slots; ++v)
        if (counts[v]) order[fill[fko_hash_to_bucket((int32_t)v, nb)]++] = v;
    char path[4096], sig[32];
    int rc = 0;
    for (int32_t b = 0; b < nb && rc == 0; ++b) {
        if (start[b] == start[b + 1]) continue; /* out.filter(map.nonEmpty), :916 */
        snprintf(path, sizeof(path), "%s/bin_signatures%d.txt", dir, b);
        FILE *f = fopen(path, "wb");
        if (!f) { rc = -2; break; }
        int64_t tot = 0;
        for (int64_t e = start[b]; e < start[b + 1]; ++e) {
            int64_t x = order[e];
            for (int j = 30; j >= 0; --j) { sig[j] = "ACGT"[x & 3]; x >>= 2; }
            sig[31] = 0;
            fprintf(f, "%s\t%lld\n", sig, (long long)counts[order[e]]);
            tot += counts[order[e]];
        }
        fprintf(f, "Total\t%lld\n", (long long)tot);
        fclose(f);
    }
    free(start);
    free(order);
    free(fill);
    return rc;
}
