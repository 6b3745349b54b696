"""The C oracle against the independent Python restatement (tests/pyref.py), and the
multi-threaded baseline variants against the plain ones."""
import random

import numpy as np
import pytest

import oracle
import pyref


def rand_seq(rng, n, alphabet="ACGT"):
    return "".join(rng.choice(alphabet) for _ in range(n))


@pytest.mark.parametrize("k", [1, 2, 5, 13, 19, 21, 31, 32])
def test_kmer_windows_vs_pyref(k):
    rng = random.Random(k)
    for _ in range(20):
        s = rand_seq(rng, rng.randint(0, 80), "ACGTACGTACGTNacgt\r")
        c, p = oracle.kmer_windows(s.encode(), k)
        ref = pyref.kmer_iterator(s, k)
        assert c.tolist() == [x for x, _ in ref]
        assert p.tolist() == [x for _, x in ref]


@pytest.mark.parametrize("k", [1, 3, 7, 15, 19, 31, 32])
def test_count_vs_pyref(k):
    rng = random.Random(100 + k)
    reads = [rand_seq(rng, rng.randint(0, 60), "ACGTACGTACGTNa") for _ in range(40)]
    # repeat some reads so counts exceed 1
    stream = "\n".join(reads + reads[:15] + reads[:5])
    keys, counts = oracle.count_stream(stream.encode(), k, 2)
    assert list(zip(keys.tolist(), counts.tolist())) == pyref.jf_count(stream, k, 2)


def test_count_mt_matches_plain():
    rng = random.Random(7)
    reads = [rand_seq(rng, 150) for _ in range(3000)]
    stream = "\n".join(reads + reads[:1000]).encode()
    a = oracle.count_stream(stream, 19, 2)
    for t in (1, 3, 8):
        b = oracle.count_stream(stream, 19, 2, threads=t)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert oracle.count_instances(stream, 19) == sum(max(0, len(r) - 18) for r in reads + reads[:1000])


def test_specificity_vs_pyref():
    rng = np.random.default_rng(3)
    rows = rng.integers(0, 40, size=(500, 3)).astype(np.uint32)
    rows = rows[rows.sum(1) > 0]
    got = oracle.specificity(rows, oracle.THRESHOLDS).tolist()
    want = pyref.specificity(rows.tolist(), oracle.THRESHOLDS)
    assert [tuple(x) for x in got] == want


def test_construct_indices_vs_pyref():
    rng = random.Random(11)
    k = 7
    reads = [rand_seq(rng, rng.randint(0, 90), "ACGTACGTN") for _ in range(60)]
    # SDK set: canonical codes of some windows (+ some absent keys)
    pool = sorted({c for r in reads for c, _ in pyref.kmer_iterator(r, k)})
    sdk = rng.sample(pool, min(80, len(pool))) + [3, 5, 99999]
    sdk = list(dict.fromkeys(sdk))
    bases = "".join(reads).encode()
    offsets = np.cumsum([0] + [len(r) for r in reads]).astype(np.uint64)
    got = oracle.construct_indices(bases, offsets, k, np.array(sdk, np.uint64), first_read_id=1)
    per_read, kci = pyref.construct_indices(reads, k, sdk, 1)
    for r, pr in enumerate(per_read):
        a, b = int(got["hit_ptr"][r]), int(got["hit_ptr"][r + 1])
        assert list(zip(got["hit_kid"][a:b].tolist(), got["hit_pos"][a:b].tolist())) == pr["hits"]
        assert got["sorted_kid"][a:b].tolist() == pr["sorted"]
        fa, fb = int(got["first_ptr"][r]), int(got["first_ptr"][r + 1])
        assert list(zip(got["first_kid"][fa:fb].tolist(), got["first_pos"][fa:fb].tolist())) == pr["first"]
    for i, lst in enumerate(kci):
        a, b = int(got["kci_ptr"][i]), int(got["kci_ptr"][i + 1])
        assert got["kci_read"][a:b].tolist() == lst


def py_connections(idx, pivots, min_kmers, min_score, categories, first_id):
    """Pure-Python get_connections (ReadClusteringEngine.cpp:301-333) over construct_indices output."""
    hp, sk, kp, kr = idx["hit_ptr"], idx["sorted_kid"], idx["kci_ptr"], idx["kci_read"]
    n = len(hp) - 1
    has = {first_id + r: r for r in range(n) if hp[r + 1] > hp[r]}
    piv = list(range(first_id, first_id + n)) if pivots is None else [int(p) for p in pivots]
    out = []
    for p in piv:
        if p not in has:
            continue
        r = has[p]
        if hp[r + 1] - hp[r] < min_kmers:
            continue
        cnt = {}
        for kid in sk[hp[r]:hp[r + 1]]:
            for c in kr[kp[kid]:kp[kid + 1]]:
                cnt[int(c)] = cnt.get(int(c), 0) + 1
        cnt.pop(p, None)
        for c, s in cnt.items():
            if s >= min_score:
                g = int(categories[r] == categories[has[c]]) if categories is not None else 0
                out.append((p, c, s, g))
    out.sort(key=lambda t: (-t[2], t[0], t[1]))
    return out


@pytest.mark.parametrize("min_kmers,min_score,use_piv", [(1, 1, False), (1, 3, False), (4, 4, False), (1, 1, True)])
def test_oracle_connections_vs_python(min_kmers, min_score, use_piv):
    rng = np.random.default_rng(7)
    gnm = bytes(rng.choice(list(b"ACGT"), 4000).tolist())
    reads = []
    for _ in range(150):
        s = int(rng.integers(0, 3800))
        reads.append(gnm[s:s + int(rng.integers(20, 300))])
    reads.append(b"A" * 40)
    reads.append(b"A" * 25 + b"T" * 30)
    bases = b"".join(reads)
    offs = np.cumsum([0] + [len(r) for r in reads]).astype(np.uint64)
    c, _ = oracle.kmer_windows(gnm, 13)
    sdk = np.concatenate([np.unique(c)[::4], np.array([0], np.uint64)])
    idx = oracle.construct_indices(bases, offs, 13, sdk, 5)
    cat = (np.arange(len(reads)) % 2).astype(np.int32)
    piv = np.arange(5, 5 + len(reads), 2, dtype=np.uint32) if use_piv else None
    x, y, s, g = oracle.connections(idx, piv, min_kmers, min_score, cat, first_read_id=5)
    exp = py_connections(idx, piv, min_kmers, min_score, cat, 5)
    assert len(exp) > 10
    assert list(zip(x.tolist(), y.tolist(), s.tolist(), g.tolist())) == exp


@pytest.mark.parametrize("k,F,min_count", [(1, 2, 1), (4, 1, 2), (11, 3, 2), (19, 2, 2), (19, 2, 1), (27, 2, 3),
                                           (32, 2, 2)])
def test_count_files_mt_matches_plain(k, F, min_count):
    """The partitioned multi-threaded count stage equals per-file count_stream + merge."""
    rng = random.Random(1000 + k * 10 + F)
    streams = []
    for f in range(F):
        reads = [rand_seq(rng, rng.randint(0, 160), "ACGTACGTACGTACGTNa") for _ in range(1500)]
        streams.append("\n".join(reads + reads[: 400 + 100 * f]).encode())
    dumps = [oracle.count_stream(s, k, min_count) for s in streams]
    keys, counts = oracle.merge(dumps)
    for t in (1, 5):
        k2, c2 = oracle.count_files_mt(streams, k, min_count, threads=t)
        assert np.array_equal(keys, k2) and np.array_equal(counts, c2)
    for (dk, dc), (ek, ec) in zip(oracle.dumps_of(keys, counts), dumps):
        assert np.array_equal(dk, ek) and np.array_equal(dc, ec)


def test_count_reference_like_rows():
    rng = random.Random(5)
    reads = [rand_seq(rng, 150) for _ in range(2000)]
    stream = "\n".join(reads + reads[:700]).encode()
    assert oracle.count_reference_like(stream, 19, 2) == len(oracle.count_stream(stream, 19, 2)[0])


@pytest.mark.parametrize("threads", [1, 2, 7])
def test_construct_indices_mt_matches_plain(threads):
    rng = np.random.default_rng(21)
    gnm = bytes(rng.choice(list(b"ACGT"), 6000).tolist())
    reads = []
    for i in range(400):
        s = int(rng.integers(0, 5800))
        r = bytearray(gnm[s:s + int(rng.integers(0, 400))])
        if i % 7 == 0 and len(r) > 10:
            r[5] = ord("N")
        reads.append(bytes(r))
    bases = b"".join(reads)
    offs = np.cumsum([0] + [len(r) for r in reads]).astype(np.uint64)
    c, _ = oracle.kmer_windows(gnm, 15)
    sdk = np.concatenate([np.unique(c)[::3], np.array([0, 7], np.uint64)])
    a = oracle.construct_indices(bases, offs, 15, sdk, 3)
    b = oracle.construct_indices(bases, offs, 15, sdk, 3, threads=threads)
    assert int(a["hit_ptr"][-1]) > 1000
    for name in a:
        assert np.array_equal(a[name], b[name]), name


@pytest.mark.parametrize("threads,use_piv,min_kmers,min_score", [(1, False, 1, 1), (3, False, 1, 2), (8, True, 2, 1),
                                                                 (64, False, 1, 1)])
def test_connections_mt_matches_plain(threads, use_piv, min_kmers, min_score):
    """The pivot-parallel connections oracle (C5 share test) equals the plain one."""
    rng = np.random.default_rng(33)
    gnm = bytes(rng.choice(list(b"ACGT"), 5000).tolist())
    reads = []
    for _ in range(300):
        s = int(rng.integers(0, 4800))
        reads.append(gnm[s:s + int(rng.integers(0, 350))])
    bases = b"".join(reads)
    offs = np.cumsum([0] + [len(r) for r in reads]).astype(np.uint64)
    c, _ = oracle.kmer_windows(gnm, 13)
    sdk = np.unique(c)[::5]
    idx = oracle.construct_indices(bases, offs, 13, sdk, 2)
    piv = np.arange(300, 1, -3, dtype=np.uint32) if use_piv else None
    x, y, s, _ = oracle.connections(idx, piv, min_kmers, min_score, first_read_id=2)
    x2, y2, s2 = oracle.connections_mt(idx, threads, piv, min_kmers, min_score, first_read_id=2)
    assert len(x) > 100
    assert np.array_equal(x, x2) and np.array_equal(y, y2) and np.array_equal(s, s2)


def test_count_pipeline_mt_matches_plain():
    rng = random.Random(77)
    streams = ["\n".join(rand_seq(rng, 150) for _ in range(3000)).encode() for _ in range(2)]
    streams = [s + b"\n" + s[: len(s) // 3] for s in streams]
    a = oracle.count_pipeline(streams, 17, 2, 4)
    b = oracle.count_pipeline_mt(streams, 17, 2, 4, threads=6)
    for name in ("keys", "counts", "hist", "selected", "n_discr"):
        assert np.array_equal(a[name], b[name]), name
