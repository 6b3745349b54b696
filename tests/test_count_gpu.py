"""Counting path on the MI355X (through the C ABI) against the oracle and the golden fixtures.
Bit-exact: per-file dumps, merged rows, specificity histogram, export selection."""
import os
import random

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def run_gpu(ctx, streams, k, lower, upper, min_count=2, thr=oracle.THRESHOLDS):
    ctx.count_begin(k, len(streams))
    for f, s in enumerate(streams):
        ctx.count_add(f, s)
    ctx.count_run(min_count)
    keys, counts = ctx.rows()
    hist = ctx.spec_hist(thr) if len(keys) else np.zeros((0, 3), np.int64)
    sel, flags, nd = ctx.select(lower, upper)
    dumps = [ctx.dump(f) for f in range(len(streams))]
    return {"keys": keys, "counts": counts, "hist": hist, "selected": sel, "flags": flags, "n_discr": nd,
            "dumps": dumps, "stats": ctx.count_stats()}


def assert_same(g, o):
    assert np.array_equal(g["keys"], o["keys"])
    assert np.array_equal(g["counts"], o["counts"])
    assert np.array_equal(g["hist"], o["hist"])
    assert np.array_equal(g["selected"], o["selected"])
    assert g["n_discr"] == o["n_discr"]
    for (gk, gc), (ok, oc) in zip(g["dumps"], o["dumps"]):
        assert np.array_equal(gk, ok) and np.array_equal(gc, oc)


def golden_streams(hga_mod):
    return [hga_mod.jf_stream(os.path.join(GOLD, p)) for p in ("reads_a.fq", "reads_b.fq")]


@pytest.mark.parametrize("k", [5, 15, 19, 21, 31, 32])
def test_count_golden(gpu_ctx, hga_mod, k):
    g = np.load(os.path.join(GOLD, "count_golden.npz"))
    r = run_gpu(gpu_ctx, golden_streams(hga_mod), k, 3, 12)
    assert np.array_equal(r["keys"], g[f"k{k}_rows_keys"])
    assert np.array_equal(r["counts"], g[f"k{k}_rows_counts"])
    assert np.array_equal(r["hist"], g[f"k{k}_hist"])
    assert np.array_equal(r["selected"], g[f"k{k}_selected"])
    assert r["n_discr"] == int(g[f"k{k}_n_discr"][0])
    for f in range(2):
        assert np.array_equal(r["dumps"][f][0], g[f"k{k}_dump{f}_keys"])
        assert np.array_equal(r["dumps"][f][1], g[f"k{k}_dump{f}_counts"])
    assert r["stats"].instances == int(g[f"k{k}_instances"][0])
    # discriminative flags agree with the row counts
    nz = (r["counts"] > 0).sum(1)
    idx = np.searchsorted(r["keys"], r["selected"])
    assert np.array_equal(r["flags"].astype(bool), nz[idx] == 1)


def random_streams(seed, n_files, n_reads, rlen, alphabet="ACGT", dup=0.5):
    rng = random.Random(seed)
    out = []
    base = ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, rlen))) for _ in range(n_reads)]
    for f in range(n_files):
        rs = [r for r in base if rng.random() < 0.7] + \
             ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, rlen))) for _ in range(n_reads // 3)]
        rs += rs[: int(len(rs) * dup)]
        rng.shuffle(rs)
        out.append("\n".join(rs).encode())
    return out


@pytest.mark.parametrize("k", [1, 2, 7, 12, 16, 19, 21, 22, 27, 31, 32])
def test_count_random_vs_oracle(gpu_ctx, k):
    streams = random_streams(k, 2, 400, 120, "ACGTACGTACGTNacgt")
    o = oracle.count_pipeline(streams, k, 2, 6)
    assert_same(run_gpu(gpu_ctx, streams, k, 2, 6), o)


@pytest.mark.parametrize("thr", [(100.01,), (50.0, 75.0, 100.01), (33.333333333333336, 50.0, 60.0, 66.66666666666667,
                                                                    75.0, 80.0, 100.0, 100.01),
                                 tuple(range(10, 101, 10)) + (100.01, 200.0)])
def test_spec_hist_thresholds(gpu_ctx, thr):
    """kc_spec_hist's per-total boundary table (n_thr <= 8: integer compares against boundaries computed on
    the host with the same IEEE expression) and its double path (more thresholds, totals >= 1024): the
    histogram equals the oracle's for thresholds that ratios hit exactly (1/2, 3/4, 2/3 ...), three files,
    and a few k-mers repeated past 1024 instances."""
    rng = random.Random(11)
    reads = [[], [], []]
    for _ in range(400):   # a distinct 25-base read repeated (a, b, c) times: ratios like 1/2, 2/3, 3/4
        r = "".join(rng.choice("ACGT") for _ in range(25)).encode()
        for f in range(3):
            reads[f] += [r] * rng.choice([0, 0, 1, 2, 3, 4, 6, 8, 9, 12])
    reads[0] += [b"ACGTTGCAACGTAGGCTAACG"] * 1500
    reads[1] += [b"ACGTTGCAACGTAGGCTAACG"] * 700
    streams = [b"\n".join(x) for x in reads]
    o = oracle.count_pipeline(streams, 19, 2, 9, thresholds=list(thr))
    r = run_gpu(gpu_ctx, streams, 19, 2, 9, thr=list(thr))
    assert int(o["counts"].sum(1).max()) >= 1024
    assert np.array_equal(r["hist"], o["hist"])


@pytest.mark.parametrize("n_files", [1, 3, 5])
@pytest.mark.parametrize("min_count", [1, 2, 3])
def test_count_files_and_min(gpu_ctx, n_files, min_count):
    streams = random_streams(100 + n_files, n_files, 300, 100)
    o = oracle.count_pipeline(streams, 19, 2, 9, min_count=min_count)
    assert_same(run_gpu(gpu_ctx, streams, 19, 2, 9, min_count=min_count), o)


def test_count_edge_inputs(gpu_ctx):
    cases = [
        [b"", b""],                                  # empty files
        [b"\n\n\n", b"NNNN"],                        # no bases at all
        [b"ACG", b"AC"],                             # reads shorter than k
        [b"A" * 5000 + b"\n" + b"T" * 5000, b"A" * 10],   # one heavy k-mer (poly-A)
        [b"ACGTN" * 2000, b"acgtn" * 2000],
    ]
    for streams in cases:
        o = oracle.count_pipeline(streams, 4, 1, 10 ** 9, min_count=1)
        assert_same(run_gpu(gpu_ctx, streams, 4, 1, 10 ** 9, min_count=1), o)


@pytest.mark.parametrize("lazy", ["0", "1"])
def test_count_claim_modes(gpu_ctx, hga_mod, monkeypatch, lazy):
    """kc_count_s with new keys claimed inline (0) or through the miss queue (1), forced either way
    (count_run picks by instances per bucket): random, all-distinct (table splits) and heavy inputs."""
    monkeypatch.setenv("HGA_CS_LAZY", lazy)
    streams = random_streams(19, 2, 400, 120, "ACGTACGTACGTNacgt")
    assert_same(run_gpu(gpu_ctx, streams, 19, 2, 6), oracle.count_pipeline(streams, 19, 2, 6))
    g = hga_mod.gen_genome(3_000_000, 77)
    streams = [g[:1_500_000], g[1_500_000:]]
    r = run_gpu(gpu_ctx, streams, 25, 1, 5, min_count=1)
    assert_same(r, oracle.count_pipeline(streams, 25, 1, 5, min_count=1))
    assert r["stats"].max_split > 1
    streams = [b"A" * 5000 + b"\n" + b"ACGT" * 3000, b"A" * 10]
    assert_same(run_gpu(gpu_ctx, streams, 13, 1, 10 ** 9, min_count=1),
                oracle.count_pipeline(streams, 13, 1, 10 ** 9, min_count=1))


def test_count_split_buckets_all_distinct(gpu_ctx, hga_mod):
    # coverage-1 random reads: every k-mer distinct -> buckets exceed the LDS table and
    # must be split into sub-ranges
    g = hga_mod.gen_genome(3_000_000, 77)
    streams = [g[:1_500_000], g[1_500_000:]]
    o = oracle.count_pipeline(streams, 25, 1, 5, min_count=1)
    r = run_gpu(gpu_ctx, streams, 25, 1, 5, min_count=1)
    assert_same(r, o)
    assert r["stats"].max_split > 1


def test_count_rerun_and_chunked_add(gpu_ctx):
    streams = random_streams(9, 2, 500, 150)
    a = run_gpu(gpu_ctx, streams, 19, 2, 8)
    gpu_ctx.count_run(2)
    b_keys, b_counts = gpu_ctx.rows()
    assert np.array_equal(a["keys"], b_keys) and np.array_equal(a["counts"], b_counts)
    # adding a file in several chunks (split at read boundaries) gives the same result
    gpu_ctx.count_begin(19, 2)
    for f, s in enumerate(streams):
        parts = s.split(b"\n")
        h = len(parts) // 2
        gpu_ctx.count_add(f, b"\n".join(parts[:h]))
        gpu_ctx.count_add(f, b"\n".join(parts[h:]))
    gpu_ctx.count_run(2)
    c_keys, c_counts = gpu_ctx.rows()
    assert np.array_equal(a["keys"], c_keys) and np.array_equal(a["counts"], c_counts)


def test_count_c1_scale_vs_oracle(gpu_ctx, hga_mod):
    # BASELINE config 1 shape: 500 kb random pair, 3 % divergence, ART-like 30x, k=19
    ga = hga_mod.gen_genome(500_000, 1)
    gb = hga_mod.gen_haplotype(ga, 0.03, 0, 2)
    ra = hga_mod.gen_art(ga, 100_000, 150, 3)
    rb = hga_mod.gen_art(gb, 100_000, 150, 4)
    streams = [ra.seq, rb.seq]
    o = {"dumps": [oracle.count_stream(s, 19, 2, threads=8) for s in streams]}
    o["keys"], o["counts"] = oracle.merge(o["dumps"])
    o["hist"] = oracle.specificity(o["counts"], oracle.THRESHOLDS)
    o["selected"], o["n_discr"] = oracle.select(o["keys"], o["counts"], 10, 25)
    r = run_gpu(gpu_ctx, streams, 19, 10, 25)
    assert_same(r, o)
    assert r["stats"].instances == 2 * 100_000 * 132


def test_count_conservation_large(gpu_ctx, hga_mod):
    # size-independent property at a C2-like size: with min_count=1 every window is counted
    # exactly once, so the merged counts sum to the number of windows
    g = hga_mod.gen_genome(4_641_652, 11)
    r = hga_mod.gen_art(g, 900_000, 150, 12)
    gpu_ctx.count_begin(19, 1)
    gpu_ctx.count_add(0, r.seq)
    gpu_ctx.count_run(1)
    st = gpu_ctx.count_stats()
    assert st.instances == 900_000 * 132
    keys, counts = gpu_ctx.rows()
    assert int(counts.sum()) == st.instances
    assert np.all(np.diff(keys.astype(np.int64)) > 0)


def test_count_level1_overflow_retry(gpu_ctx, hga_mod):
    # one k-mer dominating the input overflows its estimated level-1 region; the run must
    # detect it and redo the binning with the exact region sizes
    g = hga_mod.gen_genome(400_000, 5)
    streams = [b"A" * 3_000_000 + b"\n" + g, b"C" * 1_000_000 + b"\n" + g[:200_000]]
    o = oracle.count_pipeline(streams, 21, 1, 10 ** 9, min_count=1)
    assert_same(run_gpu(gpu_ctx, streams, 21, 1, 10 ** 9, min_count=1), o)


@pytest.mark.parametrize("k,F", [(19, 2), (13, 3), (32, 2)])
def test_count_add_rows_merges_dumps_verbatim(gpu_ctx, hga_mod, k, F):
    """hga_count_add_rows: a cached dump's rows are summed in without the per-file drop
    (JellyfishOccurrenceReader.cpp:19-24 reads an existing dump instead of counting)."""
    rng = np.random.default_rng(k * 10 + F)
    streams = golden_streams(hga_mod) + [b""] * (F - 2)
    lim = (1 << (2 * k)) - 1
    extra = []
    for f in range(F):
        n = 400 + 100 * f
        ks = np.unique(rng.integers(0, lim, n, dtype=np.uint64, endpoint=True))
        if f == 0:   # overlap with counted k-mers of file 0 so sums happen
            k0, _ = oracle.count_stream(streams[0], k, 1)
            ks = np.unique(np.concatenate([ks, k0[::7]]))
        extra.append((ks, rng.integers(1, 5, len(ks)).astype(np.uint32)))
    gpu_ctx.count_begin(k, F)
    for f in range(F):
        if streams[f]:
            gpu_ctx.count_add(f, streams[f])
        gpu_ctx.count_add_rows(f, extra[f][0][::-1], extra[f][1][::-1])   # any order
    gpu_ctx.count_run(2)
    keys, counts = gpu_ctx.rows()
    dumps = []
    for f in range(F):
        d = {}
        if streams[f]:
            kk, cc = oracle.count_stream(streams[f], k, 2)
            d = dict(zip(kk.tolist(), cc.tolist()))
        for kk, cc in zip(*extra[f]):
            d[int(kk)] = d.get(int(kk), 0) + int(cc)
        ks = np.array(sorted(d), np.uint64)
        dumps.append((ks, np.array([d[x] for x in ks.tolist()], np.uint32)))
    ok, oc = oracle.merge(dumps)
    assert np.array_equal(keys, ok) and np.array_equal(counts, oc)
    for f in range(F):
        dk, dc = gpu_ctx.dump(f)
        assert np.array_equal(dk, dumps[f][0]) and np.array_equal(dc, dumps[f][1])
    hist = gpu_ctx.spec_hist(oracle.THRESHOLDS)
    assert np.array_equal(hist, oracle.specificity(oc, oracle.THRESHOLDS))


def test_count_add_rows_only(gpu_ctx):
    """All files cached: no reads at all, rows come from the dumps alone."""
    gpu_ctx.count_begin(11, 2)
    gpu_ctx.count_add_rows(0, np.array([5, 1, 9], np.uint64), np.array([3, 1, 0], np.uint32))
    gpu_ctx.count_add_rows(1, np.array([9, 4], np.uint64), np.array([2, 7], np.uint32))
    gpu_ctx.count_run(2)
    keys, counts = gpu_ctx.rows()
    assert keys.tolist() == [1, 4, 5, 9]
    assert counts.tolist() == [[1, 0], [0, 7], [3, 0], [0, 2]]
    with pytest.raises(hga_err()):
        gpu_ctx.count_add_rows(0, np.array([1 << 22], np.uint64), np.array([1], np.uint32))


def hga_err():
    import hga
    return hga.HgaError


@pytest.mark.parametrize("fb3,k,n_files", [(1, 19, 2), (4, 19, 2), (8, 25, 1), (3, 31, 3), (2, 32, 2)])
def test_count_split3_forced_vs_oracle(gpu_ctx, monkeypatch, fb3, k, n_files):
    # the third partition level (kc_split3, normally only for inputs of a C4 rank shard's size)
    # forced onto small inputs: sub-buckets of u32 and u64 remainders, 1-3 files
    monkeypatch.setenv("HGA_SPLIT3_FORCE", str(fb3))
    streams = random_streams(200 + fb3, n_files, 400, 120, "ACGTACGTACGTNacgt")
    o = oracle.count_pipeline(streams, k, 2, 6)
    r = run_gpu(gpu_ctx, streams, k, 2, 6)
    assert_same(r, o)
    assert r["stats"].buckets > 1


def test_count_split3_slab_overflow(gpu_ctx, monkeypatch):
    # kc_split3 gives every sub-bucket a slab of 1.25x its share: one k-mer repeated ~260 K times
    # (poly-A reads) fills its sub-bucket's slab, and that bucket is redone by the exact two-pass layout
    monkeypatch.setenv("HGA_SPLIT3_FORCE", "5")
    streams = random_streams(77, 2, 400, 120, "ACGT")
    streams[0] = streams[0] + b"\n" + b"\n".join([b"A" * 150] * 2000)
    streams[1] = streams[1] + b"\n" + b"\n".join([b"T" * 150] * 300)
    o = oracle.count_pipeline(streams, 19, 2, 6)
    r = run_gpu(gpu_ctx, streams, 19, 2, 6)
    assert_same(r, o)


def test_count_split3_c1_scale(gpu_ctx, hga_mod, monkeypatch):
    monkeypatch.setenv("HGA_SPLIT3_FORCE", "6")
    ga = hga_mod.gen_genome(500_000, 1)
    gb = hga_mod.gen_haplotype(ga, 0.03, 0, 2)
    streams = [hga_mod.gen_art(ga, 100_000, 150, 3).seq, hga_mod.gen_art(gb, 100_000, 150, 4).seq]
    o = {"dumps": [oracle.count_stream(s, 19, 2, threads=8) for s in streams]}
    o["keys"], o["counts"] = oracle.merge(o["dumps"])
    o["hist"] = oracle.specificity(o["counts"], oracle.THRESHOLDS)
    o["selected"], o["n_discr"] = oracle.select(o["keys"], o["counts"], 10, 25)
    r = run_gpu(gpu_ctx, streams, 19, 10, 25)
    assert_same(r, o)
    assert r["stats"].buckets == 64 * r["stats"].buckets // 64 and r["stats"].buckets >= 64


def test_count_split3_auto_large(gpu_ctx, hga_mod):
    # 4x C2 (1.06 G instances): fine buckets far past one LDS table, so count_run adds the third
    # split level by itself; size-independent checks (every window counted once at min 1, rows
    # strictly ascending after rows())
    g = hga_mod.gen_genome(20_000_000, 31)
    h = hga_mod.gen_haplotype(g, 0.005, 0, 32)
    ra = hga_mod.gen_art(g, 4_000_000, 150, 33)
    rb = hga_mod.gen_art(h, 4_000_000, 150, 34)
    gpu_ctx.count_begin(19, 2)
    gpu_ctx.count_add(0, ra.seq)
    gpu_ctx.count_add(1, rb.seq)
    del ra, rb
    gpu_ctx.count_run(1)
    st = gpu_ctx.count_stats()
    assert st.instances == 8_000_000 * 132
    assert st.buckets > 4096 and st.max_split == 1
    keys, counts = gpu_ctx.rows()
    assert int(counts.astype(np.uint64).sum()) == st.instances
    assert np.all(np.diff(keys.astype(np.int64)) > 0)
    hist = gpu_ctx.spec_hist(oracle.THRESHOLDS)
    assert int(hist[:, 2].sum()) == len(keys)
