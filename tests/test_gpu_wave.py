"""Wave-tier count kernel on adversarial buckets (the rank's group counts and cursors
live in the dead table above CAP; FASTA inputs cannot aim at a bucket's groups).  Each bucket goes
through fk_debug_wave_count (one bucket, one wave, the production kernel) and is compared with
numpy's sorted unique counts: keys ascending, counts exact.  Covered for k = 31 (64-bit keys,
512-key buckets, 640 slots) and k = 55 (128-bit keys, 256-key buckets, 384 slots):
U == CAP distinct keys in ONE rank group, keys over all groups, duplicates, the narrow (64 / 128
group) and wide (256 group) ranks, multi-cell buckets."""
import numpy as np
import pytest

import fastkmer_amd as fk

pytestmark = pytest.mark.gpu
F = 10


def expected(keys, kw):
    rows = keys.reshape(-1, kw)
    if kw == 1:
        u, c = np.unique(rows[:, 0], return_counts=True)
        return u, c
    order = np.lexsort((rows[:, 1], rows[:, 0]))
    r = rows[order]
    head = np.ones(len(r), dtype=bool)
    head[1:] = (r[1:] != r[:-1]).any(axis=1)
    starts = np.nonzero(head)[0]
    counts = np.diff(np.append(starts, len(r)))
    return r[starts], counts


def make64(kind, rng, c0, c1, k=31):
    sh = 2 * k - F
    lo = np.uint64(c0) << np.uint64(sh)
    if kind == "one_group_full":        # U == CAP = 512 distinct keys, all in group 0
        keys = lo + np.arange(512, dtype=np.uint64) * np.uint64(7)
    elif kind == "all_groups":          # 4 keys in each group inside the cell (wide rank: 256 groups
        span = (32 - 31) + sh           # over 2^(sh + 1), the upper half past the one cell)
        gsh = span - 8
        g = np.repeat(np.arange(128, dtype=np.uint64), 4)
        keys = lo + (g << np.uint64(gsh)) + np.tile(np.array([1, 5, 6, 11], dtype=np.uint64), 128)
    elif kind == "dups_one_group":      # 150 distinct keys (wide), 512 keys in all, one group
        base = lo + rng.choice(1 << 20, 150, replace=False).astype(np.uint64)
        keys = np.concatenate([base, rng.choice(base, 512 - 150)])
    elif kind == "narrow_dups":         # 100 distinct keys (narrow rank: 64 groups)
        base = lo + rng.choice(1 << 40, 100, replace=False).astype(np.uint64)
        keys = np.concatenate([base, rng.choice(base, 300)])
    elif kind == "multi_cell":          # cells c0 .. c1 - 1, 512 distinct keys
        cells = rng.integers(c0, c1, 512).astype(np.uint64)
        keys = np.unique((cells << np.uint64(sh)) + rng.integers(0, 1 << 50, 512).astype(np.uint64))
        keys = keys[:512]
    rng.shuffle(keys)
    return keys.astype(np.uint64)


def make128(kind, rng, c0, c1, k=55):
    hsh = 2 * k - F - 64                # cell = hi >> hsh
    hi0 = np.uint64(c0) << np.uint64(hsh)
    if kind == "one_group_full":        # 256 distinct keys sharing the hi word
        rows = np.stack([np.full(256, hi0), np.arange(256, dtype=np.uint64) * np.uint64(13)], axis=1)
    elif kind == "all_groups":          # keys over every group of the cell's range
        g = np.arange(64, dtype=np.uint64)
        hi = hi0 + (g << np.uint64(hsh - 6))
        rows = np.stack([np.repeat(hi, 4), np.tile(np.array([3, 9, 10, 77], dtype=np.uint64), 64)], axis=1)
    elif kind == "dups_one_group":
        base = np.stack([np.full(90, hi0), rng.choice(1 << 30, 90, replace=False).astype(np.uint64)], axis=1)
        rows = np.concatenate([base, base[rng.integers(0, 90, 256 - 90)]])
    elif kind == "narrow_dups":
        base = np.stack([np.full(50, hi0), rng.choice(1 << 30, 50, replace=False).astype(np.uint64)], axis=1)
        rows = np.concatenate([base, base[rng.integers(0, 50, 150)]])
    elif kind == "multi_cell":
        cells = rng.integers(c0, c1, 256).astype(np.uint64)
        hi = (cells << np.uint64(hsh)) + rng.integers(0, 1 << 20, 256).astype(np.uint64)
        rows = np.unique(np.stack([hi, rng.integers(0, 1 << 62, 256).astype(np.uint64)], axis=1), axis=0)
    rng.shuffle(rows)
    return rows.astype(np.uint64).reshape(-1)


KINDS = ["one_group_full", "all_groups", "dups_one_group", "narrow_dups", "multi_cell"]


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("slots", [640])
def test_wave64_adversarial_buckets(kind, slots):
    rng = np.random.default_rng(sum(kind.encode()) + slots)
    c0, c1 = (3, 9) if kind == "multi_cell" else (5, 6)
    keys = make64(kind, rng, c0, c1)
    got_k, got_c = fk.debug_wave_count(keys, 31, F, c0, c1, slots)
    ek, ec = expected(keys, 1)
    assert np.array_equal(got_k, ek) and np.array_equal(got_c.astype(np.int64), ec.astype(np.int64))


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("slots", [384])
def test_wave128_adversarial_buckets(kind, slots):
    rng = np.random.default_rng(sum(kind.encode()) + slots)
    c0, c1 = (3, 9) if kind == "multi_cell" else (5, 6)
    keys = make128(kind, rng, c0, c1)
    got_k, got_c = fk.debug_wave_count(keys, 55, F, c0, c1, slots)
    ek, ec = expected(keys, 2)
    assert np.array_equal(got_k, ek) and np.array_equal(got_c.astype(np.int64), ec.astype(np.int64))


def test_wave_hook_rejects_keys_outside_the_cells():
    keys = np.array([np.uint64(7) << np.uint64(52)], dtype=np.uint64)
    with pytest.raises(fk.FastKmerError):
        fk.debug_wave_count(keys, 31, F, 5, 6, 640)
