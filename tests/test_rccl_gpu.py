"""The RCCL transport of the C ABI (hga_comm_init, comm.hip RcclComm) on the one GPU a test box has.

RCCL refuses two ranks on one device ("Duplicate GPU detected"), so the multi-rank protocol is
tested over the host transport hook (test_dist_gpu.py) and the 8-GPU RCCL run belongs to the
driver's scaling bench.  Here a one-rank RCCL communicator runs the same C entry points:
ncclGetUniqueId / ncclCommInitRank, the device staging of the host-memory collectives, and — with
HGA_RCCL_SELF — the rank's own slice through grouped ncclSend / ncclRecv on the ctx stream.  Every
result must equal the single-process oracle (run_jellyfish.sh:3-6, JellyfishOccurrenceReader.cpp:
63-135, ReadClusteringEngine.cpp:234-339)."""
import numpy as np
import pytest

import hga
import oracle
from test_dist import lookup_case, make_streams

pytestmark = pytest.mark.gpu
THR = oracle.THRESHOLDS


@pytest.mark.parametrize("emit", [False, True])
@pytest.mark.parametrize("self_p2p", [False, True])
@pytest.mark.parametrize("k", [13, 27])
def test_rccl_one_rank_count_exchange(monkeypatch, self_p2p, k, emit):
    if self_p2p:
        monkeypatch.setenv("HGA_RCCL_SELF", "1")
    if emit:   # buckets fine enough for the count kernel's exchange emission
        monkeypatch.setenv("HGA_FB_MIN", "10")
    streams = make_streams()
    ref = oracle.count_pipeline(streams, k, 3, 40)
    with hga.Ctx(0) as ctx:
        ctx.comm_init(hga.comm_unique_id(), 0, 1)
        assert ctx.comm_info() == (0, 1)
        ctx.count_begin(k, len(streams))
        for f, s in enumerate(streams):
            ctx.count_add(f, s)
        ctx.count_run(1)
        ctx.count_exchange(2)
        assert ctx.count_stats().distinct_rows == len(ref["keys"])   # the enqueued row-count gather
        # (with emission the instances ride the fused exchange head from the device counters)
        assert ctx.count_stats().instances == sum(oracle.count_instances(x, k) for x in streams)
        assert np.array_equal(ctx.spec_hist(THR), ref["hist"])
        keys, flags, nd = ctx.select(3, 40)
        assert np.array_equal(keys, ref["selected"]) and nd == ref["n_discr"]
        rk, rc = ctx.rows()
        assert np.array_equal(rk, ref["keys"]) and np.array_equal(rc, ref["counts"])
        d0 = ctx.dump(0)
        assert np.array_equal(d0[0], ref["dumps"][0][0]) and np.array_equal(d0[1], ref["dumps"][0][1])
        ctx.comm_destroy()


@pytest.mark.parametrize("generic", [False, True])
def test_rccl_fused_exchange_head_reports_count_errors(monkeypatch, generic):
    """A count that failed on the device (row capacity, HGA_ROW_CAP) and was never settled: the
    exchange head (comm.hip DevEngine::xb_pack_gather) decides on the gathered error bits and raises
    the failing rank's error by name; the context stays usable for a new count.  generic: the count
    did not emit exchange pieces (HGA_XB_GENERIC, as a rank holding cached dump rows): that rank
    settles inside the head without throwing and still gathers the same W + 1 words as an emitting
    rank (the gather shape must not depend on a rank's local state)."""
    monkeypatch.setenv("HGA_FB_MIN", "10")
    if generic:
        monkeypatch.setenv("HGA_XB_GENERIC", "1")
    streams = make_streams()
    with hga.Ctx(0) as ctx:
        ctx.comm_init(hga.comm_unique_id(), 0, 1)
        ctx.count_begin(13, len(streams))
        for f, s in enumerate(streams):
            ctx.count_add(f, s)
        monkeypatch.setenv("HGA_ROW_CAP", "64")
        ctx.count_run(1)
        with pytest.raises(hga.HgaError, match="rank 0: row capacity exceeded"):
            ctx.count_exchange(2)
        monkeypatch.delenv("HGA_ROW_CAP")
        ref = oracle.count_pipeline(streams, 13, 3, 40)
        ctx.count_run(1)
        ctx.count_exchange(2)
        assert ctx.count_stats().instances == sum(oracle.count_instances(x, 13) for x in streams)
        keys, flags, nd = ctx.select(3, 40)
        assert np.array_equal(keys, ref["selected"]) and nd == ref["n_discr"]
        ctx.comm_destroy()


@pytest.mark.parametrize("self_p2p", [False, True])
def test_rccl_one_rank_lookup_and_connections_gather(monkeypatch, self_p2p):
    if self_p2p:
        monkeypatch.setenv("HGA_RCCL_SELF", "1")
    reads, sdk = lookup_case()
    offs = np.cumsum([0] + [len(r) for r in reads]).astype(np.uint64)
    ref = oracle.construct_indices(b"".join(reads), offs, 13, sdk, first_read_id=1)
    cat = (np.arange(len(reads)) % 3).astype(np.int32)
    rx, ry, rs, rg = oracle.connections(ref, min_score=2, categories=cat)
    with hga.Ctx(0) as ctx:
        ctx.comm_init(hga.comm_unique_id(), 0, 1)
        ctx.lookup_load(13, sdk)
        ctx.lookup_set_reads(b"".join(reads), offs, 1)
        ctx.lookup_run()
        ctx.lookup_gather()
        got = ctx.lookup_fetch()
        for name in ref:
            assert np.array_equal(got[name], ref[name]), name
        ctx.connections_run(pivots=np.arange(1, 1 + len(reads), dtype=np.uint32), min_score=2, categories=cat)
        n = ctx.connections_gather()
        x, y, s, g = (np.zeros(n, np.uint32), np.zeros(n, np.uint32), np.zeros(n, np.uint64), np.zeros(n, np.uint8))
        hga.lib().hga_connections_fetch(ctx._h, x.ctypes.data_as(hga._u32p), y.ctypes.data_as(hga._u32p),
                                        s.ctypes.data_as(hga._u64p), g.ctypes.data_as(hga._u8p))
        assert np.array_equal(x, rx) and np.array_equal(y, ry)
        assert np.array_equal(s, rs) and np.array_equal(g, rg)


def _heavy_streams():
    """make_streams plus one k-mer repeated past 65536 instances in a file: its bucket goes to the
    generic count kernel (count.hip kc_count), which emits its exchange pieces as kc_count_s does
    (the XbEmit branch), so the exchange still takes the count_xb_pack fast path."""
    a, b = make_streams()
    return [a + b"\n".join([b"A" * 60] * 1800) + b"\n", b]


@pytest.mark.parametrize("heavy,generic", [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize("k", [13, 19])
def test_local_queries_of_an_exchange_count(monkeypatch, k, heavy, generic):
    """With a communicator attached, count_run(ctx, 1) writes exchange pieces instead of dense rows
    (count.hip XbEmit, both count kernels); local queries before the exchange rebuild the rows from them
    (kc_xb_dense).  generic: HGA_XB_GENERIC turns the emission off, so the sender bins its dense rows
    itself (exchange.hip kx_xb_hist / kx_xb_scatter, the path of cached dump rows)."""
    monkeypatch.setenv("HGA_FB_MIN", "10")   # buckets fine enough for the emission
    if generic:
        monkeypatch.setenv("HGA_XB_GENERIC", "1")
    streams = _heavy_streams() if heavy else make_streams()
    ref1 = oracle.count_pipeline(streams, k, 3, 40, min_count=1)
    ref2 = oracle.count_pipeline(streams, k, 3, 40)
    for query_first in (True, False):
        with hga.Ctx(0) as ctx:
            ctx.comm_init(hga.comm_unique_id(), 0, 1)
            ctx.count_begin(k, len(streams))
            for f, s in enumerate(streams):
                ctx.count_add(f, s)
            ctx.count_run(1)
            if query_first:   # the local count at min 1 (no exchange yet)
                assert ctx.count_stats().distinct_rows == len(ref1["keys"])
                assert np.array_equal(ctx.spec_hist(THR), ref1["hist"])
                rk, rc = ctx.rows()
                assert np.array_equal(rk, ref1["keys"]) and np.array_equal(rc, ref1["counts"])
                keys, flags, nd = ctx.select(3, 40)
                assert np.array_equal(keys, ref1["selected"]) and nd == ref1["n_discr"]
            ctx.count_exchange(2)
            assert np.array_equal(ctx.spec_hist(THR), ref2["hist"])
            rk, rc = ctx.rows()
            assert np.array_equal(rk, ref2["keys"]) and np.array_equal(rc, ref2["counts"])
            if heavy:
                assert int(rc.max()) > 65535
            ctx.comm_destroy()
