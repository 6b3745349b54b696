"""BASELINE.json configs[4] ("C5") at one rank share's size, bit-exact against the oracle:
tools/c5_pipeline.py at --scale 0.125 (a chr1/8-sized diploid: 1.69 G short-read instances, 600 K
long reads, 4.66 G windows — the per-GPU size of the chr1-scale 8-GPU run) at k = 15, 17, 19 and 21 (21: 42-bit codes, u64 level-1 elements): histogram +
export, all 9 CSR outputs of construct_indices (ReadClusteringEngine.cpp:234-299) and the whole read
graph (get_all_connections, :301-339; about 115 M connections) against the oracle (multi-threaded
restatements, each checked against the plain one in tests/test_oracle.py)."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
THREADS = max(1, min(16, os.cpu_count() or 1))


def test_c5_share_k15_k21_pipeline_bit_exact():
    """tools/c5_pipeline.py --scale 0.125 --ks 15,21 --check: count + export, lookup CSR and the whole
    read graph of a chr1/8-sized share equal the oracle (c5_pipeline.verify asserts every stage)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import c5_pipeline
    args = c5_pipeline.parse(["--scale", "0.125", "--ks", "15,21", "--warmup", "0", "--check",
                              "--check-threads", str(THREADS)])
    out = c5_pipeline.run(0, 1, args)
    assert out["checked_against_oracle"]
    r = out["per_k"][15]
    assert r["instances"] > 1_500_000_000 and r["windows"] > 4_000_000_000
    assert r["connections"] > 50_000_000


def test_c5_share_k17_k19_pipeline_bit_exact():
    """The same share at k = 17 and 19 (34- and 38-bit codes: u32 level-1 elements, the compile-time
    k paths of kc_bin1 and lk_scan): count + export, lookup CSR and the read graph equal the oracle."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import c5_pipeline
    args = c5_pipeline.parse(["--scale", "0.125", "--ks", "17,19", "--warmup", "0", "--check",
                              "--check-threads", str(THREADS)])
    out = c5_pipeline.run(0, 1, args)
    assert out["checked_against_oracle"]
    for k in (17, 19):   # (longer k: fewer shared SDK k-mers per read pair, 26 M / 17 M connections)
        r = out["per_k"][k]
        assert r["instances"] > 1_500_000_000 and r["windows"] > 4_000_000_000
        assert r["connections"] > 10_000_000
