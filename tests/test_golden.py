"""The oracle and the host reader against the committed golden fixtures (CPU only)."""
import os

import numpy as np
import pytest

import oracle
import pyref_reader

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KS = [5, 15, 19, 21, 31, 32]


def streams():
    return [b"\n".join(r["seq"].encode("latin-1") for r in pyref_reader.read_records([os.path.join(GOLD, p)], True))
            for p in ("reads_a.fq", "reads_b.fq")]


def test_host_jf_stream_matches_fixture_records(hga_mod):
    for p, s in zip(("reads_a.fq", "reads_b.fq"), streams()):
        assert hga_mod.jf_stream(os.path.join(GOLD, p)) == s


@pytest.mark.parametrize("k", KS)
def test_oracle_count_matches_golden(k):
    g = np.load(os.path.join(GOLD, "count_golden.npz"))
    res = oracle.count_pipeline(streams(), k, 3, 12)
    for f in range(2):
        assert np.array_equal(res["dumps"][f][0], g[f"k{k}_dump{f}_keys"])
        assert np.array_equal(res["dumps"][f][1], g[f"k{k}_dump{f}_counts"])
    assert np.array_equal(res["keys"], g[f"k{k}_rows_keys"])
    assert np.array_equal(res["hist"], g[f"k{k}_hist"])
    assert np.array_equal(res["selected"], g[f"k{k}_selected"])
    assert res["n_discr"] == int(g[f"k{k}_n_discr"][0])


def test_oracle_lookup_matches_golden(hga_mod):
    g = np.load(os.path.join(GOLD, "lookup_golden.npz"))
    keys, k = oracle.load_sdk_text(open(os.path.join(GOLD, "sdk_19.txt"), "rb").read())
    assert np.array_equal(keys, g["sdk_keys_id_order"])
    paths = [os.path.join(GOLD, p) for p in ("reads_a.fq", "reads_b.fq", "reads_c.fa")]
    rec = hga_mod.load_records(paths, True)          # product reader feeds the oracle
    assert np.array_equal(rec["offsets"], g["offsets"])
    assert np.array_equal(rec["category"], g["category"])
    got = oracle.construct_indices(rec["bases"], rec["offsets"], k, keys, 1)
    for name, arr in got.items():
        assert np.array_equal(arr, g[name]), name


def test_oracle_windows_match_golden():
    g = np.load(os.path.join(GOLD, "windows_golden.npz"))
    edge = open(os.path.join(GOLD, "windows_inputs.txt"), "rb").read().split(b"\n")[:-1]
    for k in (1, 2, 5, 19, 31, 32):
        for i, s in enumerate(edge):
            c, p = oracle.kmer_windows(s, k)
            assert np.array_equal(c, g[f"k{k}_s{i}_codes"]) and np.array_equal(p, g[f"k{k}_s{i}_pos"])
