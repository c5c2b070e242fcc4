// fk_split.h -- a rank's input split of a FASTA file (see fk_split.cpp).
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

namespace fk {

// One piece of a rank's input: literal bytes (a header prefix, the overlap, a final newline) or a
// byte range of the file.
struct SplitSeg {
    bool literal;
    std::string bytes;
    uint64_t off, len;  // file range (literal: off unused, len = bytes.size())
};

struct SplitPlan {
    std::vector<SplitSeg> segs;
    uint64_t total = 0;     // bytes the rank ingests
    uint64_t lo = 0, hi = 0;  // the rank's byte range of the file (its sequence starts at lo)
};

// The split of rank `rank` of `world` of the n-byte file open at fd for (k, sequence_type).
int plan_split(int fd, uint64_t n, int world, int rank, int k, int sequence_type, SplitPlan &plan, std::string &err);
// Bytes [pos, pos + len) of the rank's input into dst.
int read_split(int fd, uint64_t n, const SplitPlan &plan, uint64_t pos, uint64_t len, uint8_t *dst, std::string &err);

}  // namespace fk
