"""Connections between reads (get_connections / get_all_connections,
src/clustering/ReadClusteringEngine.cpp:301-339) on the MI355X against the oracle.
Bit-exact on (x, y, score, is_good) in the deterministic order score desc, (x, y) asc."""
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def lookup(ctx, bases, offsets, k, sdk, first_id=1):
    ctx.lookup_load(k, sdk)
    ctx.lookup_set_reads(bases, offsets, first_id)
    ctx.lookup_run()
    return oracle.construct_indices(bases, offsets, k, sdk, first_id)


def same(g, o):
    for a, b, name in zip(g, o, ("x", "y", "score", "is_good")):
        assert np.array_equal(a, b), name


@pytest.fixture(scope="module")
def golden_case(hga_mod):
    g = np.load(os.path.join(GOLD, "lookup_golden.npz"))
    paths = [os.path.join(GOLD, p) for p in ("reads_a.fq", "reads_b.fq", "reads_c.fa")]
    rec = hga_mod.load_records(paths, True)
    return rec, g


@pytest.mark.parametrize("min_score", [1, 2, 5, 40])
def test_connections_golden(gpu_ctx, golden_case, min_score):
    rec, g = golden_case
    idx = lookup(gpu_ctx, rec["bases"], rec["offsets"], 19, g["sdk_keys_id_order"])
    cat = np.asarray(rec["category"], np.int32)
    got = gpu_ctx.connections(min_score=min_score, categories=cat)
    exp = oracle.connections(idx, min_score=min_score, categories=cat)
    assert len(exp[0]) > 0 or min_score == 40
    same(got, exp)


def test_connections_filters_and_pivots(gpu_ctx, golden_case):
    rec, g = golden_case
    idx = lookup(gpu_ctx, rec["bases"], rec["offsets"], 19, g["sdk_keys_id_order"])
    # filter_components(discriminative_kmer_ids.size() >= s) + get_connections(ids, s), :750-751
    for s in (3, 10):
        same(gpu_ctx.connections(min_kmers=s, min_score=s), oracle.connections(idx, min_kmers=s, min_score=s))
    # explicit pivot list, including reads without hits
    n = len(idx["hit_ptr"]) - 1
    piv = np.arange(1, n + 1, 3, dtype=np.uint32)[::-1]
    same(gpu_ctx.connections(pivots=piv), oracle.connections(idx, pivots=piv))
    assert gpu_ctx.connections(pivots=np.zeros(0, np.uint32))[0].size == 0
    # a pivot listed twice (its runs cannot be keyed by the pivot read: the one-pass key sort)
    dup = np.concatenate([piv[:5], piv[:3]]).astype(np.uint32)
    same(gpu_ctx.connections(pivots=dup), oracle.connections(idx, pivots=dup))


def test_connections_fetch_range(gpu_ctx, golden_case):
    """hga_connections_fetch_range: the prefix run_clustering keeps (:754-755) and arbitrary clipped slices."""
    rec, g = golden_case
    idx = lookup(gpu_ctx, rec["bases"], rec["offsets"], 19, g["sdk_keys_id_order"])
    exp = oracle.connections(idx, min_score=1)
    n = gpu_ctx.connections_run(min_score=1)
    assert n == len(exp[0]) > 10
    for first, count in ((0, int(n * 0.15)), (0, n), (3, 7), (n - 2, 100), (n, 5), (n + 9, 1), (0, 0)):
        a = min(first, n)
        b = min(n, a + count)
        same(gpu_ctx.connections_range(first, count), tuple(e[a:b] for e in exp))


@pytest.mark.parametrize("env", [None, "HGA_CN_FORCE_BLOCK", "HGA_CN_FORCE_GLOBAL", "HGA_CN_TWO_STAGE", "HGA_CN_RCAP",
                                 "HGA_CN_FULL_SORT", "HGA_CN_BIG_HITS=0", "HGA_CN_BIG_HITS=60",
                                 "HGA_CN_SEGSORT", "HGA_CN_KEY64"])
def test_connections_random_first_id(gpu_ctx, hga_mod, monkeypatch, env):
    """HGA_CN_BIG_HITS: pivots with more hits than that take cn_wave's workgroup tier first (0: all)."""
    if env:
        name, _, val = env.partition("=")
        monkeypatch.setenv(name, val or "1")
    gnm = hga_mod.gen_genome(60_000, 11)
    r = hga_mod.gen_nanosim(gnm, 300, 12)
    c, _ = oracle.kmer_windows(gnm, 17)
    sdk = np.unique(c)[::5]
    idx = lookup(gpu_ctx, r.bases, r.offsets, 17, sdk, first_id=1000)
    cat = (np.arange(len(r.offsets) - 1) % 3).astype(np.int32)
    got = gpu_ctx.connections(min_score=2, categories=cat)
    exp = oracle.connections(idx, min_score=2, categories=cat, first_read_id=1000)
    assert len(exp[0]) > 1000
    same(got, exp)


def test_connections_overflow_pivot(gpu_ctx, hga_mod):
    """One long read overlapping ~5000 short reads: more distinct candidates than the LDS table."""
    gnm = hga_mod.gen_genome(30_000, 21)
    rng = np.random.default_rng(3)
    reads = [gnm]
    for s in rng.integers(0, 30_000 - 150, 5000):
        reads.append(gnm[s:s + 150])
    bases = b"".join(reads)
    offsets = np.cumsum([0] + [len(x) for x in reads]).astype(np.uint64)
    c, _ = oracle.kmer_windows(gnm, 15)
    sdk = np.unique(c)[::9]
    idx = lookup(gpu_ctx, bases, offsets, 15, sdk)
    got = gpu_ctx.connections(min_score=1)
    exp = oracle.connections(idx, min_score=1)
    assert int((exp[0] == 1).sum()) > 3500   # the long read's row
    same(got, exp)
    # the long read listed for the workgroup tier up front (its table overflows there too)
    os.environ["HGA_CN_BIG_HITS"] = "100"
    try:
        same(gpu_ctx.connections(min_score=1), exp)
    finally:
        del os.environ["HGA_CN_BIG_HITS"]


def test_connections_duplicate_kmers(gpu_ctx):
    """Multiplicities multiply: a KmerID twice in p and three times in c scores 6."""
    reads = [b"A" * 30, b"A" * 21, b"C" * 40, b"AAAAACCCCCGGGGG"]
    bases = b"".join(reads)
    offsets = np.cumsum([0] + [len(x) for x in reads]).astype(np.uint64)
    sdk = np.array([0, (1 << 10) - 1 - 0], np.uint64)   # AAAAA and its partner code
    idx = lookup(gpu_ctx, bases, offsets, 5, sdk)
    same(gpu_ctx.connections(min_score=1), oracle.connections(idx, min_score=1))
    x, y, s, _ = gpu_ctx.connections(min_score=1)
    assert s[0] == 26 * 17


def test_connections_no_hits(gpu_ctx):
    bases = b"ACGTACGTAC"
    lookup(gpu_ctx, bases, np.array([0, 10], np.uint64), 4, np.zeros(0, np.uint64))
    assert gpu_ctx.connections()[0].size == 0


def test_connections_long_kmer_lists(gpu_ctx):
    """KmerIDs shared by ~1000 reads: a pivot's pairs span several owner-map windows (segments
    straddling window starts) while its distinct candidates still fit the LDS table."""
    rng = np.random.default_rng(17)
    rnd = lambda n: bytes(rng.choice(list(b"ACGT"), n).tolist())
    k1, k2, k3 = rnd(17), rnd(17), rnd(17)
    reads = []
    for i in range(1100):
        r = rnd(20) + k1 + rnd(9) + k2 + rnd(9) + k3
        if i % 7 == 0:
            r += rnd(5) + k1          # multiplicity 2
        reads.append(r)
    bases = b"".join(reads)
    offsets = np.cumsum([0] + [len(x) for x in reads]).astype(np.uint64)
    sdk = np.unique(np.concatenate([oracle.kmer_windows(k, 17)[0] for k in (k1, k2, k3)]))
    idx = lookup(gpu_ctx, bases, offsets, 17, sdk)
    for ms in (1, 4):
        same(gpu_ctx.connections(min_score=ms), oracle.connections(idx, min_score=ms))


@pytest.mark.parametrize("env", [{}, {"HGA_ONESWEEP_MAX": "0"}, {"HGA_ONESWEEP_MAX": "0", "HGA_RS_MAX_DIGIT": "8"}])
def test_connections_wide_scores(gpu_ctx, hga_mod, monkeypatch, env):
    """Scores of several hundred (9-10 score bits): with HGA_ONESWEEP_MAX=0 the score order takes the
    classic radix passes, one wide-digit pass (or 8 + 2 bits with HGA_RS_MAX_DIGIT=8)."""
    for kv in env.items():
        monkeypatch.setenv(*kv)
    gnm = hga_mod.gen_genome(6_000, 31)
    rng = np.random.default_rng(5)
    reads = []
    for _ in range(40):
        L = int(rng.integers(1200, 2000))
        s = int(rng.integers(0, 6_000 - L))
        reads.append(gnm[s:s + L])
    bases = b"".join(reads)
    offsets = np.cumsum([0] + [len(x) for x in reads]).astype(np.uint64)
    c, _ = oracle.kmer_windows(gnm, 15)
    sdk = np.unique(c)[::2]
    idx = lookup(gpu_ctx, bases, offsets, 15, sdk)
    got = gpu_ctx.connections(min_score=1)
    exp = oracle.connections(idx, min_score=1)
    assert 256 <= int(exp[2].max()) < 1024
    same(got, exp)


@pytest.mark.parametrize("n_short", [300, 800])
def test_connections_wide_runs(gpu_ctx, hga_mod, n_short):
    """One long read overlapped by n_short short reads: its run (300 / 800 pairs) is sorted by the
    common run kernel or listed for the 16-keys-a-lane one (512 < run <= 1024)."""
    gnm = hga_mod.gen_genome(30_000, 23)
    rng = np.random.default_rng(n_short)
    reads = [gnm]
    for s in rng.integers(0, 30_000 - 150, n_short):
        reads.append(gnm[s:s + 150])
    bases = b"".join(reads)
    offsets = np.cumsum([0] + [len(x) for x in reads]).astype(np.uint64)
    c, _ = oracle.kmer_windows(gnm, 15)
    sdk = np.unique(c)[::9]
    idx = lookup(gpu_ctx, bases, offsets, 15, sdk)
    exp = oracle.connections(idx, min_score=1)
    assert int((exp[0] == 1).sum()) > 0.9 * n_short
    same(gpu_ctx.connections(min_score=1), exp)
