"""SDK lookup / index construction on the MI355X against the oracle and golden fixtures."""
import os
import random

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ["hit_ptr", "hit_kid", "hit_pos", "sorted_kid", "first_ptr", "first_kid", "first_pos", "kci_ptr",
         "kci_read"]


def run_gpu(ctx, bases, offsets, k, sdk, first_id=1):
    ctx.lookup_load(k, sdk)
    ctx.lookup_set_reads(bases, offsets, first_id)
    ctx.lookup_run()
    return ctx.lookup_fetch()


def assert_same(g, o):
    for n in NAMES:
        assert np.array_equal(g[n], o[n]), n


def test_lookup_golden(gpu_ctx, hga_mod):
    g = np.load(os.path.join(GOLD, "lookup_golden.npz"))
    paths = [os.path.join(GOLD, p) for p in ("reads_a.fq", "reads_b.fq", "reads_c.fa")]
    rec = hga_mod.load_records(paths, True)
    r = run_gpu(gpu_ctx, rec["bases"], rec["offsets"], 19, g["sdk_keys_id_order"])
    assert_same(r, g)
    s = gpu_ctx.lookup_sizes()
    assert s.reads_hit == int((np.diff(g["hit_ptr"]) > 0).sum())


def random_case(seed, n_reads, maxlen, k, alphabet, n_sdk):
    rng = random.Random(seed)
    reads = [("".join(rng.choice(alphabet) for _ in range(rng.randint(0, maxlen)))).encode() for _ in range(n_reads)]
    pool = set()
    for r in reads[: max(1, n_reads // 3)]:
        c, _ = oracle.kmer_windows(r, k)
        pool.update(c.tolist())
    sdk = rng.sample(sorted(pool), min(n_sdk, len(pool))) if pool else []
    sdk += [rng.getrandbits(min(2 * k, 62)) for _ in range(20)]
    sdk = np.array(list(dict.fromkeys(sdk)), np.uint64)
    bases = b"".join(reads)
    offsets = np.cumsum([0] + [len(r) for r in reads]).astype(np.uint64)
    return bases, offsets, sdk


@pytest.mark.parametrize("wide", [False, True])
@pytest.mark.parametrize("k", [1, 3, 11, 19, 21, 31, 32])
def test_lookup_random_vs_oracle(gpu_ctx, monkeypatch, k, wide):
    """wide: the 64-B table buckets (HGA_LK_WIDE) where a key and its KmerID would pack into the
    32-B ones (lookup.hip PBucket; k = 32 always takes the 64-B layout)."""
    if wide:
        monkeypatch.setenv("HGA_LK_WIDE", "1")
    bases, offsets, sdk = random_case(k, 700, 200, k, "ACGTACGTACGTNa", 3000)
    assert_same(run_gpu(gpu_ctx, bases, offsets, k, sdk, 7), oracle.construct_indices(bases, offsets, k, sdk, 7))


def test_lookup_long_reads(gpu_ctx, hga_mod):
    g = hga_mod.gen_genome(200_000, 3)
    r = hga_mod.gen_nanosim(g, 120, 4)
    c, _ = oracle.kmer_windows(g[:50_000], 19)
    sdk = np.unique(c)[::7]
    assert_same(run_gpu(gpu_ctx, r.bases, r.offsets, 19, sdk), oracle.construct_indices(r.bases, r.offsets, 19, sdk))


def test_lookup_edges(gpu_ctx):
    cases = [
        ([b"", b"", b"ACGT"], [0, 1, 5]),
        ([b"A" * 100, b"", b"T" * 50], [0]),          # every window hits one id
        ([b"AC", b"G", b"T"], [1, 2, 3]),              # all shorter than k
        ([b"NNNNNNNN", b"acgtacgt"], [0, 27]),
    ]
    for reads, sdk in cases:
        bases = b"".join(reads)
        offsets = np.cumsum([0] + [len(x) for x in reads]).astype(np.uint64)
        sdk = np.array(sdk, np.uint64)
        assert_same(run_gpu(gpu_ctx, bases, offsets, 4, sdk), oracle.construct_indices(bases, offsets, 4, sdk))
    # empty SDK set
    bases, offsets = b"ACGTACGT", np.array([0, 8], np.uint64)
    assert_same(run_gpu(gpu_ctx, bases, offsets, 4, np.zeros(0, np.uint64)),
                oracle.construct_indices(bases, offsets, 4, np.zeros(0, np.uint64)))


def test_lookup_c3_shape_property(gpu_ctx, hga_mod):
    # C3-shaped (Nanosim-like long reads): the hit lists are consistent with each other
    g = hga_mod.gen_genome(1_000_000, 5)
    r = hga_mod.gen_nanosim(g, 2_000, 6)
    c, _ = oracle.kmer_windows(g, 19)
    sdk = np.unique(c)[::40]
    res = run_gpu(gpu_ctx, r.bases, r.offsets, 19, sdk)
    s = gpu_ctx.lookup_sizes()
    assert res["hit_ptr"][-1] == s.hits == res["kci_ptr"][-1]
    assert np.array_equal(np.bincount(res["hit_kid"], minlength=len(sdk)), np.diff(res["kci_ptr"]))
    assert np.array_equal(np.sort(res["kci_read"]), np.sort(np.repeat(
        np.arange(1, r.n + 1, dtype=np.uint32), np.diff(res["hit_ptr"]).astype(np.int64))))
    # spot-check 200 reads against the oracle
    o = oracle.construct_indices(r.bases[: int(r.offsets[200])], r.offsets[:201], 19, sdk)
    h = int(o["hit_ptr"][-1])
    assert np.array_equal(res["hit_kid"][:h], o["hit_kid"]) and np.array_equal(res["hit_pos"][:h], o["hit_pos"])


@pytest.mark.parametrize("sizes", [(300, 5000, 40), (25000, 1500)])
def test_lookup_hit_dense_reads(gpu_ctx, sizes):
    """Reads whose every window is an SDK, with repeats: per-read sorts of 2..16384 hits (LDS
    segment sorts) and of > 16384 hits (global radix path), duplicates kept in window order."""
    rng = random.Random(sum(sizes))
    k = 15
    reads = []
    for L in sizes:
        unit = "".join(rng.choice("ACGT") for _ in range(max(L // 3, k + 1)))
        reads.append((unit * 4)[:L].encode())
    reads.append(b"ACGTN" * 10)
    pool = set()
    for r in reads:
        c, _ = oracle.kmer_windows(r, k)
        pool.update(c.tolist())
    sdk = np.array(rng.sample(sorted(pool), len(pool)), np.uint64)
    bases = b"".join(reads)
    offsets = np.cumsum([0] + [len(r) for r in reads]).astype(np.uint64)
    assert_same(run_gpu(gpu_ctx, bases, offsets, k, sdk, 3), oracle.construct_indices(bases, offsets, k, sdk, 3))


def test_lookup_many_dense_reads(gpu_ctx):
    """Hundreds of reads whose windows are mostly SDKs with repeats: many concurrent per-read
    LDS sorts with cross-wave stages (sizes 50..2500 hits)."""
    rng = random.Random(11)
    k = 13
    base = "".join(rng.choice("ACGT") for _ in range(3000))
    reads = []
    for _ in range(300):
        L = rng.randint(50, 2500)
        s = rng.randint(0, len(base) - L)
        unit = base[s: s + max(L // 2, k)]
        reads.append((unit * 3)[:L].encode())
    pool = set()
    for r in reads[:50]:
        c, _ = oracle.kmer_windows(r, k)
        pool.update(c.tolist())
    sdk = np.array(rng.sample(sorted(pool), len(pool) * 3 // 4), np.uint64)
    bases = b"".join(reads)
    offsets = np.cumsum([0] + [len(r) for r in reads]).astype(np.uint64)
    want = oracle.construct_indices(bases, offsets, k, sdk, 1)
    for _ in range(3):
        assert_same(run_gpu(gpu_ctx, bases, offsets, k, sdk, 1), want)


@pytest.mark.parametrize("n_share", [40, 300, 700, 1500])
def test_lookup_shared_kmer_lists(gpu_ctx, n_share):
    """kmer_component_index lists of many lengths: one k-mer shared by n_share reads."""
    rng = random.Random(n_share)
    k = 15
    rnd = lambda n: "".join(rng.choice("ACGT") for _ in range(n))
    shared = rnd(k)
    reads = [(rnd(rng.randint(0, 30)) + shared + rnd(rng.randint(0, 30))).encode() for _ in range(n_share)]
    rng.shuffle(reads)
    pool = set()
    for r in reads[:20]:
        c, _ = oracle.kmer_windows(r, k)
        pool.update(c.tolist())
    sdk = np.array(sorted(pool), np.uint64)
    bases = b"".join(reads)
    offsets = np.cumsum([0] + [len(r) for r in reads]).astype(np.uint64)
    exp = oracle.construct_indices(bases, offsets, k, sdk, 5)
    assert int(np.diff(exp["kci_ptr"]).max()) >= n_share
    assert_same(run_gpu(gpu_ctx, bases, offsets, k, sdk, 5), exp)



@pytest.mark.parametrize("n_sdk,mode", [(3000, "bucketed"), (3000, "overflow"), (200_000, "bucketed"),
                                        (200_000, "two_pass"), (200_000, "radix")])
def test_kmer_component_index_paths(gpu_ctx, monkeypatch, n_sdk, mode):
    """kmer_component_index (ReadClusteringEngine.cpp:262-267, 282-284) by the bucketed sort (lookup.hip
    lk_msd_* + lk_kci_*: one or two <= 128-way MSD passes on the top KmerID bits, then per bucket a count
    by KmerID and each KmerID's reads sorted) and by the radix path (HGA_KCI_RADIX=1).  3000 SDKs: one MSD
    pass; 200 K SDKs: two passes (256 buckets; "two_pass": 40 K reads, ~2 M hits, 1024 buckets); "overflow"
    gives one KmerID more reads than a bucket's 4 K LDS pairs, so the kernel flags it and the index is
    rebuilt by the radix path.  Every CSR output equals the oracle's."""
    if mode == "radix":
        monkeypatch.setenv("HGA_KCI_RADIX", "1")
    rng = np.random.default_rng(n_sdk)
    k = 17
    g = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), 20_000 if n_sdk < 4096 else 400_000))
    n_reads = {"overflow": 16_000, "two_pass": 40_000}.get(mode, 6000)
    reads = []
    for _ in range(n_reads):
        s = int(rng.integers(0, len(g) - 200))
        r = g[s:s + int(rng.integers(60, 200))]
        reads.append(g[:k] + r if mode == "overflow" else r)   # every read holds the genome's first k-mer
    codes, _ = oracle.kmer_windows(g, k)
    pool = np.unique(codes)
    if mode == "overflow":
        pool = pool[pool != codes[0]]
    sdk = rng.choice(pool, n_sdk, replace=False).astype(np.uint64)
    if mode == "overflow":
        sdk[0] = codes[0]
    bases = b"".join(reads)
    offsets = np.cumsum([0] + [len(r) for r in reads]).astype(np.uint64)
    exp = oracle.construct_indices(bases, offsets, k, sdk, 1)
    assert len(exp["kci_read"]) > (32768 if n_sdk < 4096 else 1_000_000 if mode == "two_pass" else 200_000)
    if mode == "overflow":
        assert int(np.diff(exp["kci_ptr"]).max()) > 15 * 1024
    assert_same(run_gpu(gpu_ctx, bases, offsets, k, sdk, 1), exp)
