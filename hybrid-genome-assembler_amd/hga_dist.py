"""Multi-GPU counting from Python: a thin caller of the C ABI's communicator.

SURVEY.md §8(e): every rank counts its contiguous shard of every file with min 1; the rows travel once
(all-to-all over xGMI) to hash-bucket owners — owner o holds a range of the counting hash's top bits,
the pieces come out of the count kernel already grouped by bucket; each owner sums what
it received and applies the per-file `--bc` drop (src/occurrences/run_jellyfish.sh:3-6).  The count
queries of the ctx then answer for the whole input (JellyfishOccurrenceReader.cpp:63-135): the
histogram is the owners' bins summed; the export, rows and dumps are re-partitioned by canonical-code
range (one all-to-all of the export itself) and come out as the ranks' ranges in rank order.  All of
that runs inside libhga (include/hga.h: hga_comm_init / hga_comm_init_host, hga_count_exchange).

This module only sets the communicator up from a torch.distributed process group:
  backend "nccl" (RCCL): the library's own RCCL communicator over xGMI, its unique id broadcast
                         through the process group;
  any other (gloo):      the library's host-staged transport hook, one all_to_all_single per call.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

import hga


def owner_splitters(k: int, n_owners: int):
    """Python mirror of the library's owner ranges (exchange_protocol.hpp owner_splitters), for tests
    that drive hga_count_partition / hga_count_merge by hand: owner o starts at 4^k (1 - sqrt(1 - o/n))."""
    m = 1 << (2 * k)
    out = []
    for o in range(1, n_owners):
        x = int(m * (1.0 - (1.0 - o / n_owners) ** 0.5))
        out.append(min(max(x, out[-1] if out else 0), m - 1))
    return np.array(out, dtype=np.uint64)


def gloo_transport(group=None) -> "hga.Transport":
    """hga_transport whose all-to-all-v is torch.distributed.all_to_all_single over `group` (host
    tensors).  Also used by the CPU test harness of the same protocol (tests/test_dist.py)."""
    world = dist.get_world_size(group)

    def a2a(send, recv):
        ss = [n for _, n in send]
        rs = [n for _, n in recv]
        sbuf = np.empty(max(sum(ss), 1), np.uint8)
        o = 0
        for addr, n in send:
            if n:
                C.memmove(sbuf.ctypes.data + o, addr, n)
            o += n
        rbuf = torch.empty(max(sum(rs), 1), dtype=torch.uint8)
        dist.all_to_all_single(rbuf[: sum(rs)], torch.from_numpy(sbuf[: sum(ss)]), rs, ss, group=group)
        o, rp = 0, rbuf.data_ptr()
        for addr, n in recv:
            if n:
                C.memmove(addr, rp + o, n)
            o += n

    return hga.transport_of(a2a, world)


def attach(ctx: "hga.Ctx", group=None):
    """Give `ctx` this process group's communicator (collective over the group)."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":
        obj = [hga.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group else 0, group=group)
        ctx.comm_init(obj[0], rank, world)
    else:
        ctx.comm_init_host(rank, world, gloo_transport(group))
    return rank, world


class OwnerExchange:
    """Distributed count of one rank, all through the C ABI."""

    def __init__(self, ctx: "hga.Ctx", group=None):
        self.ctx = ctx
        self.rank, self.world = attach(ctx, group)
        self.local_rows = 0

    def count(self, min_per_file: int = 2):
        """Local count of this rank's shard (no drop), owner exchange, owner merge + drop."""
        self.ctx.count_run(1)
        self.local_rows = None   # rows stay on the device; count_stats() is global after the exchange
        self.ctx.count_exchange(min_per_file)

    def spec_hist(self, thresholds):
        return self.ctx.spec_hist(thresholds)          # global, identical on every rank

    def select(self, lower: int, upper: int):
        keys, flags, _ = self.ctx.select(lower, upper)  # the whole export on every rank
        return keys, flags

    def select_counts(self, lower: int, upper: int):
        return self.ctx.select_device(lower, upper)    # keys stay on their owner; global (n, n_discr)


def shard_reads(seq: bytes, rank: int, world: int) -> bytes:
    """Contiguous range of whole reads ('\\n'-separated) for `rank`."""
    n = len(seq)
    if world <= 1:
        return seq

    def cut(i):
        if i <= 0:
            return 0
        if i >= n:
            return n
        j = seq.find(b"\n", n * i // world)
        return n if j < 0 else j + 1

    return seq[cut(rank): cut(rank + 1)]
