"""Clustering stages after construct_indices (host/clustering.cpp, ReadClusteringEngine.cpp:301-826)
against the independent Python restatement tests/pyref_cluster.py: union-find, the eigensolver,
spectral clustering and the whole run_clustering on synthetic two-haplotype reads (host path)."""
import random

import numpy as np
import pytest

import oracle
import pyref_cluster as pc


def rand_conns(rng, n_nodes, n_edges, max_score=30):
    c = []
    for _ in range(n_edges):
        x, y = rng.sample(range(1, n_nodes + 1), 2)
        c.append((x, y, rng.randint(1, max_score), False))
    return pc.sort_conns(c)


@pytest.mark.parametrize("seed", range(8))
def test_union_find_matches_restatement(hga_mod, seed):
    rng = random.Random(seed)
    conns = rand_conns(rng, 60, 150)
    restricted = set(rng.sample(range(1, 61), 6)) if seed % 2 else set()
    min_size, max_size = [(1, -1), (2, -1), (3, 10), (5, 7)][seed % 4]
    got = hga_mod.union_find(conns, restricted, min_size, max_size)
    want = pc.union_find(conns, restricted, min_size, max_size)
    assert [(g[0], g[1]) for g in got] == [(list(w[0]), list(w[1])) for w in want]


def test_union_find_negative_min_size_keeps_nothing(hga_mod):
    conns = rand_conns(random.Random(1), 10, 20)
    assert hga_mod.union_find(conns, (), -1, -1) == []       # int -> size_t comparison (:484)


@pytest.mark.parametrize("n", [2, 5, 17, 40])
def test_sym_eigen_matches_numpy(hga_mod, n):
    rng = np.random.default_rng(n)
    a = rng.standard_normal((n, n))
    a = a + a.T
    val, vec = hga_mod.sym_eigen(a)
    ref_val, ref_vec = np.linalg.eigh(a)
    assert np.allclose(val, ref_val, atol=1e-10)
    assert np.allclose(a @ vec, vec * val[None, :], atol=1e-9)
    assert np.allclose(np.abs((vec * ref_vec).sum(axis=0)), 1.0, atol=1e-8)


def block_conns(rng, sizes, intra=(40, 60), inter=(1, 4)):
    nodes, base = [], 1
    for s in sizes:
        nodes.append(list(range(base, base + s)))
        base += s
    c = []
    for bi, b in enumerate(nodes):
        for i in b:
            for j in b:
                if i < j:
                    c.append((i, j, rng.randint(*intra), False))
        for b2 in nodes[bi + 1:]:
            c.append((rng.choice(b), rng.choice(b2), rng.randint(*inter), False))
    return pc.sort_conns(c), nodes


@pytest.mark.parametrize("sizes", [(4, 5), (3, 4, 5), (6, 3, 4, 5)])
def test_spectral_clustering_recovers_blocks(hga_mod, sizes):
    conns, nodes = block_conns(random.Random(len(sizes)), sizes)
    got = hga_mod.spectral_clustering(conns, 16)
    want = pc.spectral_clustering(conns, 16)
    as_sets = lambda cs: sorted(sorted(c) for c in cs if c)
    assert as_sets(got) == as_sets(want)
    # every cluster lies inside one block (ClusterRotate prefers more clusters within 0.001 of the
    # best quality, ClusterRotate.cpp:41-45, so a block may come back split)
    block_of = {v: i for i, b in enumerate(nodes) for v in b}
    assert all(len({block_of[v] for v in c}) == 1 for c in got if c)


def haplotype_case(hga_mod, L=40_000, d=0.02, n_reads=180, k=15):
    ga = hga_mod.gen_genome(L, 5)
    gb = hga_mod.gen_haplotype(ga, d, 0, 6)
    ra, rb = hga_mod.gen_nanosim(ga, n_reads, 7), hga_mod.gen_nanosim(gb, n_reads, 8)
    bases = ra.bases + rb.bases
    offsets = np.concatenate([ra.offsets, rb.offsets[1:] + ra.offsets[-1]]).astype(np.uint64)
    cats = np.array([0] * (len(ra.offsets) - 1) + [1] * (len(rb.offsets) - 1), np.int32)
    # SDKs: k-mers specific to one haplotype genome (what jf_occurrences' export selects)
    ka, _ = oracle.kmer_windows(ga, k)
    kb, _ = oracle.kmer_windows(gb, k)
    sdk = np.setxor1d(np.unique(ka), np.unique(kb))
    idx = oracle.construct_indices(bases, offsets, k, sdk)
    return bases, offsets, cats, idx


CFGS = [dict(sc_min=5, sc_max=-1, sc_fraction=0.15, sc_score=0, enrich=8, tail=10, dims=16),
        dict(sc_min=3, sc_max=40, sc_fraction=0.3, sc_score=0, enrich=4, tail=6, dims=4),
        dict(sc_min=5, sc_max=-1, sc_fraction=0.15, sc_score=6, enrich=8, tail=10, dims=16)]


@pytest.mark.parametrize("ci", range(len(CFGS)))
@pytest.mark.parametrize("debug", [False, True])
def test_run_clustering_host_matches_restatement(hga_mod, ci, debug):
    bases, offsets, cats, idx = haplotype_case(hga_mod)
    c = CFGS[ci]
    lengths = np.diff(offsets)
    avg = int(lengths.sum() // len(lengths))
    cat_in = cats if debug else np.zeros_like(cats)
    cfg = hga_mod.cluster_config(c["sc_min"], c["sc_max"], c["sc_fraction"], c["sc_score"], c["enrich"], c["tail"],
                                 1, c["dims"])
    ids, owner, log = hga_mod.cluster_host(bases, offsets, cat_in, idx, avg, cfg, debug)
    eng = pc.Engine(idx, lengths, cat_in, avg, debug, c)
    want = eng.run()
    assert ids.tolist() == want
    want_owner = np.zeros(len(lengths), np.uint32)
    for cid in want:
        for r in eng.comps[cid]["reads"]:
            want_owner[r - 1] = cid
    assert np.array_equal(owner, want_owner)
    assert "Union-find took" in log and "Merging into core components took" in log
