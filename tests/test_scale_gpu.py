"""BASELINE.json configs[3] at its own per-GPU size, bit-exact against the oracle.

- C4 (configs[3]): one rank's shard of the 8-GPU run — exactly bench.py's `scale_c4_shard` leg
  (bench.make_c4_shard: ART-like 3.75x of a 2 x 500 Mbp diploid, 3.77 Gbases, 3.3 G 19-mer
  instances, 515 M merged rows; the third split level kc_split3 runs).  Every merged row, both
  per-file dumps, the whole specificity histogram, the [10,25] export with its discriminative flags
  and count are compared with the range-partitioned multi-threaded oracle (or_count_files_mt:
  per-file exact counts + --bc drop + merge, run_jellyfish.sh:3-6, JellyfishOccurrenceReader.cpp:
  63-135); at min 1 the conservation identity sum(counts) = instances holds.
C5 at a rank share's size: tests/test_c5_share_gpu.py.
Host memory: about 80 GB at the peak (the box allows about 270 GB)."""
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
THREADS = max(1, min(16, os.cpu_count() or 1))


@pytest.fixture(scope="module")
def c4_shard():
    import bench
    return bench.make_c4_shard(0)


@pytest.fixture(scope="module")
def c4_gpu(hga_mod, c4_shard):
    import bench
    ra, rb = c4_shard
    out = {}
    with hga_mod.Ctx(int(os.environ.get("HGA_DEVICE", "0"))) as ctx:
        ctx.count_begin(bench.K, 2)
        ctx.count_add(0, ra.seq)
        ctx.count_add(1, rb.seq)
        ctx.count_run(1)   # conservation identity at min 1 (nothing dropped)
        st = ctx.count_stats()
        keys, counts = ctx.rows()
        out["min1_rows"] = len(keys)
        out["min1_sum"] = int(counts.sum(dtype=np.uint64))
        out["min1_ascending"] = bool(len(keys) < 2 or (keys[1:] > keys[:-1]).all())
        del keys, counts
        out["instances"] = int(st.instances)
        ctx.count_run(2)   # the bench step: count_run + spec_hist + select[10,25]
        out["stats"] = ctx.count_stats()
        out["hist"] = ctx.spec_hist(oracle.THRESHOLDS)
        out["selected"], out["flags"], out["n_discr"] = ctx.select(bench.LOWER, bench.UPPER)
        out["keys"], out["counts"] = ctx.rows()
        out["dumps"] = [ctx.dump(f) for f in range(2)]
    return out


@pytest.fixture(scope="module")
def c4_oracle(c4_shard):
    import bench
    ra, rb = c4_shard
    keys, counts = oracle.count_files_mt([ra.seq, rb.seq], bench.K, 2, THREADS)
    return keys, counts


def test_c4_shard_conservation_min1(c4_gpu, c4_shard):
    ra, rb = c4_shard
    inst = oracle.count_instances(ra.seq, 19) + oracle.count_instances(rb.seq, 19)
    assert c4_gpu["instances"] == inst == 3_300_000_000
    assert c4_gpu["min1_sum"] == inst
    assert c4_gpu["min1_ascending"]


def test_c4_shard_rows_bit_exact(c4_gpu, c4_oracle):
    keys, counts = c4_oracle
    assert len(keys) > 400_000_000          # 515 M merged rows at min 2
    assert c4_gpu["stats"].distinct_rows == len(keys)
    assert c4_gpu["stats"].max_split >= 1
    assert np.array_equal(c4_gpu["keys"], keys)
    assert np.array_equal(c4_gpu["counts"], counts)


def test_c4_shard_dumps_bit_exact(c4_gpu, c4_oracle):
    keys, counts = c4_oracle
    for f in range(2):
        m = counts[:, f] > 0
        gk, gc = c4_gpu["dumps"][f]
        assert np.array_equal(gk, keys[m]), f"file {f} dump keys"
        assert np.array_equal(gc, counts[m, f]), f"file {f} dump counts"


def test_c4_shard_histogram_and_export_bit_exact(c4_gpu, c4_oracle):
    import bench
    keys, counts = c4_oracle
    assert np.array_equal(c4_gpu["hist"], oracle.specificity(counts, oracle.THRESHOLDS))
    sel, nd = oracle.select(keys, counts, bench.LOWER, bench.UPPER)
    assert len(sel) > 10_000_000
    assert np.array_equal(c4_gpu["selected"], sel)
    assert c4_gpu["n_discr"] == nd
    idx = np.searchsorted(keys, sel)
    nz = (counts[idx] > 0).sum(1)
    assert np.array_equal(c4_gpu["flags"].astype(bool), nz == 1)
