// fk_cli.cpp -- command-line driver with the reference's positional arguments.
//
//   fastkmer-cli [LocalTestKmerCounter|TestKmerCounter] k m x B useHT sequenceType
//                inputPath outputPath prefix write enableKryo useCustomPartitioner [numPartitionTasks]
//
// Argument order and meaning follow skc.test.LocalTestKmerCounter.main
// (LocalTestKmerCounter.scala:35-48) and TestKmerCounter.main
// (TestKmerCounter.scala:34-47); the output directory is
// TestConfiguration.outputDir (test/package.scala:33).  enableKryo selects a
// JVM serializer and useCustomPartitioner a Spark placement: neither changes
// the counts, both are accepted and reported.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "../../include/fastkmer.h"

static int usage(const char *argv0) {
    fprintf(stderr,
            "usage: %s [LocalTestKmerCounter|TestKmerCounter] k m x B useHT sequenceType inputPath outputPath "
            "prefix write enableKryo useCustomPartitioner [numPartitionTasks]\n",
            argv0);
    return 2;
}

static bool parse_int(const char *s, int *out) {
    char *end = nullptr;
    long v = strtol(s, &end, 10);
    if (!s[0] || *end) return false;
    *out = (int)v;
    return true;
}

int main(int argc, char **argv) {
    int a = 1;
    std::string driver = "LocalTestKmerCounter";
    if (argc > 1 && (!strcmp(argv[1], "LocalTestKmerCounter") || !strcmp(argv[1], "TestKmerCounter") ||
                     !strcmp(argv[1], "skc.test.LocalTestKmerCounter") || !strcmp(argv[1], "skc.test.TestKmerCounter"))) {
        driver = argv[1];
        a = 2;
    }
    if (argc - a < 12) return usage(argv[0]);
    fk_config cfg;
    fk_config_init(&cfg);
    int use_ht, write, kryo, part, ntasks = 0;
    if (!parse_int(argv[a + 0], &cfg.k) || !parse_int(argv[a + 1], &cfg.m) || !parse_int(argv[a + 2], &cfg.x) ||
        !parse_int(argv[a + 3], &cfg.B) || !parse_int(argv[a + 4], &use_ht) ||
        !parse_int(argv[a + 5], &cfg.sequence_type) || !parse_int(argv[a + 9], &write) ||
        !parse_int(argv[a + 10], &kryo) || !parse_int(argv[a + 11], &part))
        return usage(argv[0]);
    cfg.use_ht = use_ht == 1 ? 1 : 0;  // args(4).toInt == 1
    cfg.write = write == 1 ? 1 : 0;
    if (part == 1) {
        if (argc - a < 13 || !parse_int(argv[a + 12], &ntasks)) return usage(argv[0]);
    }
    const char *input = argv[a + 6];
    const char *output = argv[a + 7];
    const char *prefix = argv[a + 8];
    if (fk_config_validate(&cfg) != FK_OK) {
        fprintf(stderr, "invalid configuration: %s\n", fk_last_error());
        return 1;
    }
    char outdir[4096];
    fk_output_dir(&cfg, output, prefix, outdir, sizeof(outdir));
    // TestConfiguration.toString (test/package.scala:37-39)
    printf("Kmer counting on MI355X (%s). \nTest parameters:\nDataset: %s\nk: %d\nm: %d\nx: %d\nb: %d\n"
           "Sequence type: %d\nUsing HT:  %s\nWriting: %s\nUsing Kryo Serializer: %s\n"
           "Multiprocessor Scheduliong Partitioning: %s",
           driver.c_str(), input, cfg.k, cfg.m, cfg.x, fk_clamped_bins(cfg.m, cfg.B), cfg.sequence_type,
           cfg.use_ht ? "true" : "false", cfg.write ? "true" : "false", kryo == 1 ? "true (no effect)" : "false",
           part == 1 ? "true (no effect on one GPU)" : "false");
    if (part == 1) printf("\t no. partition tasks: %d", ntasks);
    printf("\n");

    // the input is memory-mapped and streamed to the device in windows (FASTdoop reads its
    // splits the same way, SBKC:1009-1012): fk_ingest appends each window and the fused map
    // runs over the tiles that have landed while the next window is in flight
    const int fd = open(input, O_RDONLY);
    if (fd < 0) {
        fprintf(stderr, "cannot open %s\n", input);
        return 1;
    }
    struct stat sb;
    if (fstat(fd, &sb) != 0) {
        fprintf(stderr, "cannot stat %s\n", input);
        close(fd);
        return 1;
    }
    const size_t size = (size_t)sb.st_size;
    const uint8_t *map = nullptr;
    if (size) {
        void *p = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (p == MAP_FAILED) {
            fprintf(stderr, "cannot map %s\n", input);
            close(fd);
            return 1;
        }
        (void)madvise(p, size, MADV_SEQUENTIAL);
        map = (const uint8_t *)p;
    }
    fk_ctx *ctx = nullptr;
    if (fk_create(&cfg, &ctx) != FK_OK) {
        fprintf(stderr, "fk_create: %s\n", fk_last_error());
        if (map) munmap((void *)map, size);
        close(fd);
        return 1;
    }
    const size_t window = (size_t)256 << 20;
    auto t0 = std::chrono::steady_clock::now();
    int rc = fk_ingest_reserve(ctx, size);
    for (size_t off = 0; rc == FK_OK && (off < size || off == 0);) {
        const size_t len = std::min(window, size - off);
        rc = fk_ingest(ctx, map ? map + off : nullptr, len, off + len >= size ? 1 : 0);
        off += len;
        if (size == 0) break;
    }
    if (rc == FK_OK) rc = fk_finish(ctx);
    auto t1 = std::chrono::steady_clock::now();
    if (map) munmap((void *)map, size);
    close(fd);
    if (rc != FK_OK) {
        fprintf(stderr, "fk_finish: %s\n", fk_last_error());
        fk_destroy(ctx);
        return 1;
    }
    fk_stats st;
    fk_get_stats(ctx, &st);
    printf("Finished getSuperKmers. parse %.3f ms, signature %.3f ms, %llu super-k-mers, %llu k-mers\n", st.ms_parse,
           st.ms_signature, (unsigned long long)st.superkmers, (unsigned long long)st.kmers);
    printf("extractKXmers%s ended. partition %.3f ms, count %.3f ms, %llu distinct k-mers, host wall %.3f ms\n",
           cfg.use_ht ? "HT" : "", st.ms_partition, st.ms_count, (unsigned long long)st.distinct,
           std::chrono::duration<double, std::milli>(t1 - t0).count());
    if (cfg.write) {
        if (fk_write_bins(ctx, outdir) != FK_OK) {
            fprintf(stderr, "fk_write_bins: %s\n", fk_last_error());
            fk_destroy(ctx);
            return 1;
        }
        printf("Output written to %s\n", outdir);
    }
    fk_destroy(ctx);
    return 0;
}
