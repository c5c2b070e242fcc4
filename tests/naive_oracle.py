"""Independent naive k-mer counter (TEST INFRASTRUCTURE ONLY).

Written from the semantic contract, not from the
reference's control flow: string slicing, min(s, revcomp(s)), a signature
as the minimum "norm" over the k-m+1 m-mers, and collections.Counter.
Used to cross-check the C oracle and the literal transliteration.
"""
from __future__ import annotations

from collections import Counter

_COMP = str.maketrans("ACGT", "TGCA")


def revcomp(s: str) -> str:
    return s.translate(_COMP)[::-1]


def allowed(s: str) -> bool:
    m = len(s)
    if m >= 3:
        return "AA" not in s and not s.startswith("ACA")
    v = 0
    for ch in s:
        v = v * 4 + "ACGT".index(ch)
    return not (v == 0 or v == 4 or (v & 0x3C) == 0 or (v & 0xF) == 0)


def encode(s: str) -> int:
    v = 0
    for ch in s:
        v = v * 4 + "ACGT".index(ch)
    return v


def norm(s: str) -> int:
    m = len(s)
    d = 4 ** m
    a = encode(s) if allowed(s) else d
    r = revcomp(s)
    b = encode(r) if allowed(r) else d
    return min(a, b)


def hash_to_bucket(s: int, b: int) -> int:
    M = 0xFFFFFFFF
    key = s & M
    key = (key ^ 61) ^ (key >> 16)
    key = (key + (key << 3)) & M
    key = key ^ (key >> 4)
    key = (key * 0x27D4EB2D) & M
    key = key ^ (key >> 15)
    return (key & 0x7FFFFFFF) % b


def reads_of(fasta: bytes) -> list[str]:
    out, cur = [], None
    for line in fasta.decode("latin-1").split("\n"):
        if line.startswith(">"):
            if cur is not None:
                out.append(cur)
            cur = ""
        elif cur is not None:
            cur += line
    if cur is not None:
        out.append(cur)
    return out


def count(fasta: bytes, k: int, m: int, B: int) -> dict[int, dict[str, int]]:
    bc = int(min(4.0 ** m, float(B)))
    bins: dict[int, Counter] = {}
    for r in reads_of(fasta):
        for i in range(len(r) - k + 1):
            w = r[i:i + k]
            if any(ch not in "ACGT" for ch in w):
                continue
            canon = min(w, revcomp(w))
            sig = min(norm(w[j:j + m]) for j in range(k - m + 1))
            b = hash_to_bucket(sig, bc)
            bins.setdefault(b, Counter())[canon] += 1
    return {b: dict(sorted(c.items())) for b, c in bins.items()}
