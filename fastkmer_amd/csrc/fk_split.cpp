// fk_split.cpp -- a rank's input split of a FASTA file (host code, no GPU).
//
// Replaces the FASTdoop input splits the reference hands its map tasks
// (SparkBinKmerCounter.scala:993, 1009-1012): the file is cut into byte ranges
// of ~size/world and rank r counts
//
//   * sequenceType 0 (FASTAshortInputFileFormat, whole records per split): the
//     records whose '>' lies in [r*size/world, (r+1)*size/world), the range's
//     ends moved forward to record starts (a '>' opening a line); rank 0 also
//     gets any text before the first header, which the parse ignores;
//   * sequenceType 1 (FASTAlongInputFileFormat, overlap key "k" at :993): the
//     k-mer windows whose first base lies in the range -- its bytes (after a
//     header line it starts inside, and not before the file's first header),
//     prefixed with a header line (">s\n", the range may start inside a
//     record), plus the k - 1 sequence positions after it (the overlap),
//     stopping at a record boundary, then "\n".
//
// Concatenating the ranks' counts gives the counts of the whole file.  The
// same cut is restated in Python by fastkmer_amd/sharding.py (read_shard,
// read_record_shard); tests/test_split.py checks that both give the same bytes.
#include "fk_split.h"

#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>

namespace fk {

namespace {

// Reads [off, off + len) (clipped to the file); returns the bytes read or -1.
int64_t pread_all(int fd, uint64_t size, uint64_t off, uint64_t len, uint8_t *dst) {
    if (off >= size) return 0;
    len = std::min(len, size - off);
    uint64_t got = 0;
    while (got < len) {
        const ssize_t r = pread(fd, dst + got, len - got, (off_t)(off + got));
        if (r < 0) {
            if (errno == EINTR) continue;
            return -1;
        }
        if (r == 0) break;
        got += (uint64_t)r;
    }
    return (int64_t)got;
}

struct Reader {
    int fd;
    uint64_t n;
    std::string err;
    std::vector<uint8_t> buf;

    bool read(uint64_t off, uint64_t len) {
        buf.resize(len);
        const int64_t r = pread_all(fd, n, off, len, buf.data());
        if (r < 0) {
            err = std::string("pread: ") + strerror(errno);
            return false;
        }
        buf.resize((size_t)r);
        return true;
    }
    // first byte of the line holding p (scanning back in doubling windows)
    bool line_start(uint64_t p, uint64_t *out) {
        uint64_t q = p, w = 256;
        while (q > 0) {
            const uint64_t a = q > w ? q - w : 0;
            if (!read(a, q - a)) return false;
            for (size_t j = buf.size(); j-- > 0;)
                if (buf[j] == '\n') {
                    *out = a + j + 1;
                    return true;
                }
            q = a;
            w = std::min<uint64_t>(2 * w, 4096);
        }
        *out = 0;
        return true;
    }
    // index of the '\n' ending the line holding p (n if none)
    bool line_end(uint64_t p, uint64_t *out) {
        uint64_t q = p, w = 256;
        while (q < n) {
            if (!read(q, w)) return false;
            const void *j = memchr(buf.data(), '\n', buf.size());
            if (j) {
                *out = q + (uint64_t)((const uint8_t *)j - buf.data());
                return true;
            }
            if (buf.empty()) break;
            q += buf.size();
            w = std::min<uint64_t>(2 * w, 4096);
        }
        *out = n;
        return true;
    }
    bool byte_at(uint64_t p, int *c) {
        if (!read(p, 1)) return false;
        *c = buf.empty() ? -1 : buf[0];
        return true;
    }
    // first record start (a '>' opening a line) at or after p (p <= 0: 0); n if none
    bool record_start(uint64_t p, uint64_t *out) {
        if (p == 0) {
            *out = 0;
            return true;
        }
        constexpr uint64_t W = 1ull << 16;
        for (uint64_t q = p - 1; q < n; q += W) {
            if (!read(q, W + 1)) return false;
            for (size_t j = 0; j + 1 < buf.size(); ++j)
                if (buf[j] == '\n' && buf[j + 1] == '>') {
                    *out = q + j + 1;
                    return true;
                }
        }
        *out = n;
        return true;
    }
};

}  // namespace

int plan_split(int fd, uint64_t n, int world, int rank, int k, int sequence_type, SplitPlan &plan, std::string &err) {
    plan = SplitPlan{};
    if (world < 1 || rank < 0 || rank >= world) {
        err = "bad rank " + std::to_string(rank) + " of " + std::to_string(world);
        return -1;
    }
    if (k < 1) {
        err = "bad k";
        return -1;
    }
    Reader rd{fd, n, {}, {}};
    auto fail = [&] {
        err = rd.err;
        return -1;
    };
    const uint64_t r0 = (uint64_t)((unsigned __int128)n * (uint64_t)rank / (uint64_t)world);
    const uint64_t r1 = (uint64_t)((unsigned __int128)n * (uint64_t)(rank + 1) / (uint64_t)world);
    if (sequence_type == 0) {
        uint64_t lo = 0, hi = n;
        if (!rd.record_start(r0, &lo)) return fail();
        if (rank + 1 < world && !rd.record_start(r1, &hi)) return fail();
        if (hi > lo) plan.segs.push_back(SplitSeg{false, {}, lo, hi - lo});
        plan.total = hi > lo ? hi - lo : 0;
        plan.lo = lo, plan.hi = hi;
        return 0;
    }
    // the file's first header: lines before it are not sequence
    uint64_t p0 = 0;
    while (p0 < n) {
        int ch = 0;
        if (!rd.byte_at(p0, &ch)) return fail();
        if (ch == '>') break;
        uint64_t e = 0;
        if (!rd.line_end(p0, &e)) return fail();
        p0 = e + 1;
    }
    uint64_t lo = std::max(r0, p0), hi = r1;
    plan.lo = lo, plan.hi = hi;
    if (lo >= hi) return 0;
    if (lo > p0) {
        uint64_t ls = 0;
        int ch = 0;
        if (!rd.line_start(lo, &ls) || !rd.byte_at(ls, &ch)) return fail();
        if (ch == '>') {  // lo inside a header line: the range's sequence starts after it
            uint64_t e = 0;
            if (!rd.line_end(lo, &e)) return fail();
            lo = e + 1;
        }
    }
    plan.lo = lo;
    if (lo >= hi) return 0;
    // the state at hi: inside a header line?  at a line start?
    bool hdr = false, at_line_start = false;
    {
        // the last '\n' of [lo, hi), scanning back from hi
        uint64_t q = hi, last_nl = UINT64_MAX;
        while (q > lo && last_nl == UINT64_MAX) {
            const uint64_t a = q - lo > 4096 ? q - 4096 : lo;
            if (!rd.read(a, q - a)) return fail();
            for (size_t j = rd.buf.size(); j-- > 0;)
                if (rd.buf[j] == '\n') {
                    last_nl = a + j;
                    break;
                }
            q = a;
        }
        int ch = 0;
        if (last_nl != UINT64_MAX) {
            if (last_nl + 1 < hi) {
                if (!rd.byte_at(last_nl + 1, &ch)) return fail();
                hdr = ch == '>';
            }
        } else {  // the line holding hi started at or before lo (lo is never inside a header line)
            uint64_t ls = 0;
            if (!rd.line_start(lo, &ls) || !rd.byte_at(lo, &ch)) return fail();
            hdr = lo == ls && ch == '>';
        }
        if (!rd.byte_at(hi - 1, &ch)) return fail();
        at_line_start = ch == '\n';
    }
    // k - 1 sequence positions after hi (fewer at a record boundary or the end of the file)
    std::string ext;
    int need = k - 1;
    for (uint64_t q = hi; need > 0 && q < n;) {
        if (!rd.read(q, std::min<uint64_t>(4096, 2 * (uint64_t)need + 64))) return fail();
        if (rd.buf.empty()) break;
        size_t j = 0;
        for (; j < rd.buf.size(); ++j) {
            const uint8_t c = rd.buf[j];
            if (at_line_start && c == '>') {
                need = 0;
                break;
            }
            ext.push_back((char)c);
            if (c == '\n') {
                at_line_start = true;
                hdr = false;
                continue;
            }
            at_line_start = false;
            if (!hdr && --need == 0) break;
        }
        q += rd.buf.size();
    }
    plan.segs.push_back(SplitSeg{true, ">s\n", 0, 3});
    plan.segs.push_back(SplitSeg{false, {}, lo, hi - lo});
    if (!ext.empty()) plan.segs.push_back(SplitSeg{true, ext, 0, ext.size()});
    plan.segs.push_back(SplitSeg{true, "\n", 0, 1});
    plan.total = 0;
    for (const SplitSeg &s : plan.segs) plan.total += s.len;
    return 0;
}

int read_split(int fd, uint64_t n, const SplitPlan &plan, uint64_t pos, uint64_t len, uint8_t *dst, std::string &err) {
    uint64_t base = 0;
    for (const SplitSeg &s : plan.segs) {
        if (len == 0) break;
        const uint64_t end = base + s.len;
        if (pos < end) {
            const uint64_t a = pos - base, take = std::min(len, s.len - a);
            if (s.literal) {
                memcpy(dst, s.bytes.data() + a, take);
            } else {
                const int64_t r = pread_all(fd, n, s.off + a, take, dst);
                if (r < 0 || (uint64_t)r != take) {
                    err = r < 0 ? std::string("pread: ") + strerror(errno) : std::string("the file shrank while read");
                    return -1;
                }
            }
            dst += take;
            pos += take;
            len -= take;
        }
        base = end;
    }
    if (len) {
        err = "read past the split";
        return -1;
    }
    return 0;
}

}  // namespace fk
