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
