"""Export order on the MI355X: count_select's MSD sort (one onesweep pass on the top 8 bits of the
2k-bit code, then every top-digit segment sorted in LDS; segments over 16384 keys by the global
radix sort) against the oracle's selection (export_kmers, JellyfishOccurrenceReader.cpp:110-135:
ascending code == LC_ALL=C order).  Sizes put s.rows above the MSD threshold (32768)."""
import random

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def genome(n, alphabet, seed):
    rng = random.Random(seed)
    return "".join(rng.choice(alphabet) for _ in range(n)).encode()


def reads_of(g, n, length, seed):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        s = rng.randrange(0, len(g) - length)
        out.append(g[s:s + length])
    return b"\n".join(out)


def check(ctx, streams, k, lower, upper, min_count):
    ctx.count_begin(k, len(streams))
    for f, s in enumerate(streams):
        ctx.count_add(f, s)
    ctx.count_run(min_count)
    assert ctx.count_stats().distinct_rows >= 32768
    sel, flags, nd = ctx.select(lower, upper)
    dumps = [oracle.count_stream(s, k, min_count, threads=8) for s in streams]
    keys, counts = oracle.merge(dumps)
    o_sel, o_nd = oracle.select(keys, counts, lower, upper)
    assert np.array_equal(sel, o_sel)
    assert nd == o_nd
    nz = (counts > 0).sum(1)
    idx = np.searchsorted(keys, sel)
    assert np.array_equal(flags.astype(bool), nz[idx] == 1)
    return len(sel)


@pytest.mark.parametrize("k", [8, 11, 16, 19, 21, 27, 31])
def test_export_sort_random(gpu_ctx, k):
    ga = genome(300_000, "ACGT", k)
    gb = bytearray(ga)
    rng = random.Random(k + 100)
    for i in range(0, len(gb), 50):
        gb[i] = ord(rng.choice("ACGT"))
    streams = [reads_of(ga, 12_000, 150, 2 * k), reads_of(bytes(gb), 12_000, 150, 2 * k + 1)]
    n = check(gpu_ctx, streams, k, 1, 1 << 30, 1)
    assert n >= 32768


def test_export_sort_skewed_segments_fallback(gpu_ctx):
    # A/C-only sequence: every canonical 19-mer starts with A/C, so only 16 of the 256 top digits
    # are used and each holds more than 16384 keys -> the global-radix fallback per segment
    g = genome(600_000, "AC", 7)
    n = check(gpu_ctx, [reads_of(g, 30_000, 150, 8)], 19, 1, 1 << 30, 1)
    assert n > 16 * 16384


def test_export_sort_range_subset(gpu_ctx, hga_mod):
    ga = hga_mod.gen_genome(400_000, 21)
    gb = hga_mod.gen_haplotype(ga, 0.02, 0, 22)
    streams = [hga_mod.gen_art(ga, 60_000, 150, 23).seq, hga_mod.gen_art(gb, 60_000, 150, 24).seq]
    check(gpu_ctx, streams, 19, 10, 25, 2)


@pytest.mark.parametrize("lo,width", [(1 << 35, 1 << 31), (5 << 30, 1 << 24), (0, 1 << 38)])
def test_export_sort_owner_like_ranges(gpu_ctx, lo, width):
    # rows confined to a key range, as on one owner of a multi-GPU run: the MSD digit spans only the
    # occupied range (12-bit bins lo..hi), not the whole code space
    rng = np.random.default_rng(lo % 1000 + width % 997)
    keys = np.unique(rng.integers(lo, lo + width, 120_000, dtype=np.uint64))
    counts = rng.integers(10, 30, len(keys), dtype=np.uint32)
    gpu_ctx.count_begin(19, 1)
    gpu_ctx.count_add_rows(0, keys, counts)
    gpu_ctx.count_run(2)
    sel, flags, nd = gpu_ctx.select(10, 25)
    want = keys[(counts >= 10) & (counts <= 25)]
    assert np.array_equal(sel, want)
    assert nd == len(want) and np.all(flags == 1)


def test_export_sort_few_big_segments(gpu_ctx):
    # 150 K keys spread over the code space plus 60 K inside one top digit: ONE segment passes the
    # LDS capacity (per-segment global sort) while the rest are sorted in LDS
    rng = np.random.default_rng(5)
    spread = rng.integers(0, 1 << 38, 150_000, dtype=np.uint64)
    hot = rng.integers(77 << 30, (77 << 30) + (1 << 29), 60_000, dtype=np.uint64)
    keys = np.unique(np.concatenate([spread, hot]))
    counts = rng.integers(10, 30, len(keys), dtype=np.uint32)
    gpu_ctx.count_begin(19, 1)
    gpu_ctx.count_add_rows(0, keys, counts)
    gpu_ctx.count_run(2)
    sel, flags, nd = gpu_ctx.select(10, 25)
    want = keys[(counts >= 10) & (counts <= 25)]
    assert np.array_equal(sel, want)
    assert nd == len(want) and np.all(flags == 1)


@pytest.mark.parametrize("k,hot,lsd", [(19, 0, False), (19, 30_000, False), (19, 40_000, False), (19, 0, True),
                                       (19, 30_000, True), (21, 25_000, False), (27, 0, False), (27, 15_000, False),
                                       (27, 20_000, False)])
def test_export_sort_workgroup_segments(gpu_ctx, monkeypatch, k, hot, lsd):
    """~4.5 M exported keys spread over the code space (~1.1 K per 12-bit digit, many past one wave's
    BX_MAX = 1024): the bucketed export sort with workgroup LDS sorts of the larger digit segments
    (count.hip kc_bx_lsort, the C4-shard-sized path: u32 keys up to 32768 a segment at k <= 21, u64 up to
    16384 above); `hot` keys packed into one digit — within the cap, or past it (the MSD + global-radix
    path).  At k <= 21 the segments go through the sub-bucket counting sort (kc_bx_csort) unless `lsd`
    (HGA_BX_LSD: the LSD-pass kernels)."""
    if lsd:
        monkeypatch.setenv("HGA_BX_LSD", "1")
    rng = np.random.default_rng(hot + 3 + k)
    lb = 2 * k - 12
    keys = rng.integers(0, 1 << (2 * k), 6_000_000, dtype=np.uint64)
    if hot:
        keys = np.concatenate([keys, rng.integers(901 << lb, (901 << lb) + (1 << lb), hot, dtype=np.uint64)])
    keys = np.unique(keys)
    counts = rng.integers(10, 30, len(keys), dtype=np.uint32)
    if hot:   # the hot digit's keys all selected
        counts[(keys >> np.uint64(lb)) == 901] = 15
    gpu_ctx.count_begin(k, 1)
    gpu_ctx.count_add_rows(0, keys, counts)
    gpu_ctx.count_run(2)
    sel, flags, nd = gpu_ctx.select(10, 25)
    want = keys[(counts >= 10) & (counts <= 25)]
    assert np.array_equal(sel, want)
    assert nd == len(want) and np.all(flags == 1)


def test_export_sort_crowded_sub_buckets(gpu_ctx):
    """A digit segment whose keys crowd into one sub-bucket of kc_bx_csort (20 K keys inside a 2^14-code
    range, i.e. one of its 4096 sub-buckets at k = 19): sorted by the Shell sort path, ascending."""
    rng = np.random.default_rng(11)
    spread = rng.integers(0, 1 << 38, 2_000_000, dtype=np.uint64)
    crowd = rng.integers(333 << 26, (333 << 26) + (1 << 14), 20_000, dtype=np.uint64)
    keys = np.unique(np.concatenate([spread, crowd]))
    counts = np.full(len(keys), 12, np.uint32)
    gpu_ctx.count_begin(19, 1)
    gpu_ctx.count_add_rows(0, keys, counts)
    gpu_ctx.count_run(2)
    sel, flags, nd = gpu_ctx.select(10, 25)
    assert np.array_equal(sel, keys)
    assert nd == len(keys) and np.all(flags == 1)
