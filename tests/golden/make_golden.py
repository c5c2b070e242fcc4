"""Regenerate the golden fixtures in tests/golden/ (TEST INFRASTRUCTURE).

Each case is a small FASTA input plus the reference-format output expected
for it: {"bin<b>": file text} for useHT=0 (sorted lines + "EOF",
SparkBinKmerCounter.scala:550-606).  Expected outputs come from the C oracle
(oracle/fk_oracle.c) and are only written when the step-for-step Scala
transliteration (oracle/literal_ref.py) and the independent naive counter
(tests/naive_oracle.py) produce the same files -- the reference itself cannot
run here (no JVM/Spark/FASTdoop), see DESIGN.md "Oracle".

<name>.binsig.json holds the bin-signature diagnostics of the same input
({"bin_signatures<b>.txt": file text}, SparkBinKmerCounter.scala:772-953, lines
in ascending signature order), written by the C oracle only when the literal
transliteration of getBinSignatures gives the same (bin, signature, count) sets.

Usage: python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402
from oracle import literal_ref  # noqa: E402
import naive_oracle  # noqa: E402


def synth_reads(rng, n, lo, hi, alphabet="ACGT", noise="", noise_p=0.0, wrap=0, genome=None):
    out = []
    for i in range(n):
        L = rng.randint(lo, hi)
        if genome is not None and L <= len(genome):
            st = rng.randint(0, len(genome) - L)
            s = genome[st:st + L]
            if rng.random() < 0.5:
                s = naive_oracle.revcomp(s)
        else:
            s = "".join(rng.choice(alphabet) for _ in range(L))
        if noise:
            s = "".join(rng.choice(noise) if rng.random() < noise_p else ch for ch in s)
        if wrap:
            s = "\n".join(s[q:q + wrap] for q in range(0, len(s), wrap)) if s else ""
        out.append(f">r{i:010d}\n{s}\n")
    return "".join(out).encode()


def cases():
    rng = random.Random(0x5EED)
    genome = "".join(rng.choice("ACGT") for _ in range(3000))
    yield "kat_appendix_b", dict(k=28, m=10, x=3, B=2048), (
        b">r1\nACGTTGCATGCATGCAACGTTAGCCGATCGATCGGATCCATGCANNACGTTGCATGCATGCAACGTTAGCCGATCGAT\n"
        b">r2\nATCGATCGGCTAACGTTGCATGCATGCAACGTACGTTGCA\n>r3\n" + b"G" * 30 + b"\n")
    yield "short_reads_k28", dict(k=28, m=10, x=3, B=2048), synth_reads(rng, 120, 100, 100, genome=genome)
    yield "edge_bytes_k21", dict(k=21, m=7, x=2, B=64), synth_reads(
        rng, 60, 0, 120, noise="NnacgtR\r", noise_p=0.03, wrap=17, genome=genome)
    yield "two_word_k55", dict(k=55, m=12, x=3, B=8192), synth_reads(rng, 40, 150, 150, genome=genome)
    yield "k32_boundary", dict(k=32, m=9, x=1, B=512), synth_reads(rng, 40, 30, 90, genome=genome)
    yield "k31_boundary", dict(k=31, m=11, x=4, B=1000), synth_reads(rng, 40, 30, 90, genome=genome)
    long_seq = genome + "N" * 40 + genome[:800].lower() + genome[900:1700]
    yield "long_record_k28", dict(k=28, m=10, x=3, B=2048, sequence_type=1), (
        b">chrSynthetic\n" + "\n".join(long_seq[q:q + 60] for q in range(0, len(long_seq), 60)).encode() + b"\n")
    yield "tiny_k5_m3", dict(k=5, m=3, x=1, B=7), synth_reads(rng, 30, 0, 40, alphabet="ACGTN")
    yield "low_complexity", dict(k=21, m=5, x=3, B=256), (
        b">a\n" + b"A" * 80 + b"\n>c\n" + b"AC" * 60 + b"\n>g\n" + b"GATTACA" * 20 + b"\n>t\n" + b"T" * 50 + b"\n")
    yield "no_records", dict(k=21, m=7, x=1, B=64), b"ACGTACGTACGTACGTACGTACGTACGT\n\n"
    yield "empty", dict(k=21, m=7, x=1, B=64), b""
    yield "crlf_and_junk", dict(k=11, m=4, x=2, B=33), (
        b"junk line before first header ACGTACGTACGT\n>h1 desc\r\nACGTACGTTTGACCA\r\nGGTACCATTGACCAGT\r\n"
        b">h2\nACGTAGGTAC>GTAGCATCGATCAGCATCGACT\n\n\nACGTAGCTAGCTAGGCAT\n>h3\n>h4\nACGTAGCATCGACTAGC")


def expected_files(fasta, k, m, x, B, sequence_type=0):
    r = oracle.OracleResult(fasta, k, m, B, sequence_type)
    files = {f"bin{b}": r.bin_text(b) for b in range(r.nbins) if r.bin_size(b)}
    lit = literal_ref.run_sorted(fasta, k, m, x, B)
    lit_files = {f"bin{b}": t for b, t in lit.items()}
    if lit_files != files:
        raise SystemExit("literal transliteration disagrees with the C oracle")
    nv = naive_oracle.count(fasta, k, m, B)
    if {f"bin{b}": "".join(f"{s}\t{c}\n" for s, c in d.items()) + "EOF" for b, d in nv.items()} != files:
        raise SystemExit("naive counter disagrees with the C oracle")
    return files, r


def expected_binsig(fasta, k, m, B):
    import tempfile
    counts = oracle.bin_signatures(fasta, k, m)
    with tempfile.TemporaryDirectory() as d:
        oracle.write_bin_signatures(counts, m, B, d)
        files = {}
        for name in sorted(os.listdir(d)):
            with open(os.path.join(d, name)) as f:
                files[name] = f.read()
    lit = literal_ref.get_bin_signatures(k, m, oracle.clamp_bins(m, B), literal_ref.parse_reads(fasta))
    lit_files = {f"bin_signatures{b}.txt": literal_ref.save_bin_signatures_text(dict(sorted(d.items())))
                 for b, d in lit.items()}
    if lit_files != files:
        raise SystemExit("literal getBinSignatures disagrees with the C oracle")
    return files


def main():
    index = {}
    for name, params, fasta in cases():
        files, r = expected_files(fasta, **params)
        with open(os.path.join(HERE, name + ".fa"), "wb") as f:
            f.write(fasta)
        with open(os.path.join(HERE, name + ".expected.json"), "w") as f:
            json.dump(files, f, indent=0, sort_keys=True)
        with open(os.path.join(HERE, name + ".binsig.json"), "w") as f:
            json.dump(expected_binsig(fasta, params["k"], params["m"], params["B"]), f, indent=0, sort_keys=True)
        index[name] = dict(params, total_kmers=r.total_kmers, distinct=r.distinct, nonempty_bins=len(files))
        print(f"{name}: {len(fasta)} B, {r.total_kmers} k-mers, {r.distinct} distinct, {len(files)} bins")
    with open(os.path.join(HERE, "index.json"), "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
