"""Multi-GPU counting: owner exchange over torch.distributed (RCCL on MI355X), DESIGN.md §6.

SURVEY.md §8(e): every rank counts its shard of the reads; the merged rows are range-partitioned
by canonical code and exchanged once (all-to-all over xGMI); each owner sums the rows it
received, applies the per-file `--bc` drop (src/occurrences/run_jellyfish.sh:3-6) and then runs
the specificity histogram (JellyfishOccurrenceReader.cpp:88-108) and the export selection
(:110-135) on its own key range.  Histograms are reduced across ranks; exports concatenated in
rank order are ascending (the reference's LC_ALL=C order) because owner ranges are ordered.

The protocol is written against a small engine interface so that the CPU tests (gloo,
world_size 2) drive exactly this code:

    engine.n_files, engine.k, engine.device
    engine.count_local()                 -> rows   (count of this rank's shard, no drop)
    engine.partition(splitters, keys_buf, counts_buf) -> rows per owner (np.uint64)
    engine.merge(keys, counts, n, min_per_file)
    engine.pack_bits()                   -> bits per file count in the packed form (0: wide only)
    engine.partition_packed(splitters, buf, capacity) -> (pieces per owner, total)
    engine.merge_packed(buf, n, min_per_file)
    engine.spec_hist(thresholds)         -> int64 [m, 3] (threshold index, total, count)
    engine.select(lower, upper)          -> (keys np.uint64 ascending, flags np.uint8)
    engine.select_device(lower, upper)   -> (n, n_discriminative)

`HgaEngine` is the product engine (libhga.so on one GPU).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

import hga


def owner_splitters(k: int, n_owners: int):
    """n_owners-1 ascending splitters over canonical codes in [0, 4^k).

    canonical = min(fwd, rc); for uniformly distributed k-mers P(canon < x) = 1 - (1 - x/4^k)^2,
    so equal-mass owner ranges start at 4^k * (1 - sqrt(1 - o/n)).  Any ascending splitters give
    the same results; these only balance the load."""
    m = 1 << (2 * k)
    out = []
    for o in range(1, n_owners):
        x = int(m * (1.0 - (1.0 - o / n_owners) ** 0.5))
        out.append(min(max(x, out[-1] if out else 0), m - 1))
    return np.array(out, dtype=np.uint64)


class HgaEngine:
    """Counting engine on one GPU through the C ABI."""

    def __init__(self, ctx: "hga.Ctx", k: int, n_files: int, device):
        self.ctx, self.k, self.n_files, self.device = ctx, k, n_files, torch.device(device)

    def count_local(self) -> int:
        self.ctx.count_run(1)
        return int(self.ctx.count_stats().distinct_rows)

    def partition(self, splitters, keys_buf: torch.Tensor, counts_buf: torch.Tensor):
        return self.ctx.count_partition(splitters, keys_buf.data_ptr(), counts_buf.data_ptr())

    def merge(self, keys: torch.Tensor, counts: torch.Tensor, n: int, min_per_file: int):
        self.ctx.count_merge(keys.data_ptr(), counts.data_ptr(), n, min_per_file)

    def pack_bits(self) -> int:
        return self.ctx.count_pack_bits()

    def partition_packed(self, splitters, buf: torch.Tensor, capacity: int):
        return self.ctx.count_partition_packed(splitters, buf.data_ptr(), capacity)

    def merge_packed(self, buf: torch.Tensor, n: int, min_per_file: int):
        self.ctx.count_merge_packed(buf.data_ptr(), n, min_per_file)

    def spec_hist(self, thresholds):
        return self.ctx.spec_hist(thresholds)

    def select(self, lower, upper):
        keys, flags, _ = self.ctx.select(lower, upper)
        return keys, flags

    def select_device(self, lower, upper):
        return self.ctx.select_device(lower, upper)

    def sync(self):
        self.ctx.sync()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)


class OwnerExchange:
    """Runs the distributed counting protocol for one rank."""

    def __init__(self, engine, group=None):
        self.e = engine
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        backend = dist.get_backend(group)
        # RCCL moves device memory directly; gloo (CPU tests, shared-GPU tests) stages on the host
        self.comm_dev = engine.device if backend == "nccl" else torch.device("cpu")
        self.splitters = owner_splitters(engine.k, self.world)
        self.local_rows = 0
        self.received_rows = 0

    def _a2a(self, out, inp, out_splits, in_splits):
        dist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits,
                               group=self.group)

    def count(self, min_per_file: int = 2) -> int:
        """Local count, owner exchange, owner merge.  Returns the rows/pieces this owner received."""
        e = self.e
        rows = e.count_local()
        self.local_rows = rows
        if e.pack_bits() > 0:
            return self._count_packed(rows, min_per_file)
        return self._count_wide(rows, min_per_file)

    def _count_packed(self, rows: int, min_per_file: int) -> int:
        """One u64 per row piece: half the all-to-all bytes of the wide form."""
        e = self.e
        cap = rows + rows // 64 + 1024
        buf = torch.empty(cap, dtype=torch.int64, device=e.device)
        per, total = e.partition_packed(self.splitters, buf, cap)
        if total > cap:   # many rows with huge counts: retry with room for every piece
            cap = total
            buf = torch.empty(cap, dtype=torch.int64, device=e.device)
            per, total = e.partition_packed(self.splitters, buf, cap)
        per = np.asarray(per, dtype=np.int64)
        send_n = torch.from_numpy(per).to(self.comm_dev)
        recv_n = torch.empty_like(send_n)
        self._a2a(recv_n, send_n, None, None)
        rn = recv_n.cpu().numpy().astype(np.int64)
        n = int(rn.sum())
        rbuf = torch.empty(n, dtype=torch.int64, device=self.comm_dev)
        self._a2a(rbuf, buf[:total].to(self.comm_dev), rn.tolist(), per.tolist())
        rbuf = rbuf.to(e.device)
        if e.device.type == "cuda":
            torch.cuda.synchronize(e.device)
        e.merge_packed(rbuf, n, min_per_file)
        self.received_rows = n
        return n

    def _count_wide(self, rows: int, min_per_file: int) -> int:
        e, F = self.e, self.e.n_files
        keys = torch.empty(rows, dtype=torch.int64, device=e.device)
        cnts = torch.empty(rows * F, dtype=torch.int32, device=e.device)
        per = np.asarray(e.partition(self.splitters, keys, cnts), dtype=np.int64)
        send_n = torch.from_numpy(per).to(self.comm_dev)
        recv_n = torch.empty_like(send_n)
        self._a2a(recv_n, send_n, None, None)
        rn = recv_n.cpu().numpy().astype(np.int64)
        total = int(rn.sum())
        keys_c, cnts_c = keys.to(self.comm_dev), cnts.to(self.comm_dev)
        rkeys = torch.empty(total, dtype=torch.int64, device=self.comm_dev)
        rcnts = torch.empty(total * F, dtype=torch.int32, device=self.comm_dev)
        self._a2a(rkeys, keys_c, rn.tolist(), per.tolist())
        self._a2a(rcnts, cnts_c, (rn * F).tolist(), (per * F).tolist())
        rkeys, rcnts = rkeys.to(e.device), rcnts.to(e.device)
        if e.device.type == "cuda":
            torch.cuda.synchronize(e.device)
        e.merge(rkeys, rcnts, total, min_per_file)
        self.received_rows = total
        return total

    def spec_hist(self, thresholds):
        """Global specificity histogram (std::map order), identical on every rank."""
        local = np.ascontiguousarray(self.e.spec_hist(thresholds), dtype=np.int64).reshape(-1, 3)
        parts = self._all_gather_var(local.reshape(-1))
        allp = np.concatenate([p.reshape(-1, 3) for p in parts]) if parts else np.zeros((0, 3), np.int64)
        if len(allp) == 0:
            return np.zeros((0, 3), np.int64)
        # sum the counts of equal (threshold, total) bins; np.unique sorts = std::map order
        packed = (allp[:, 0] << 40) | allp[:, 1]
        u, inv = np.unique(packed, return_inverse=True)
        cnt = np.zeros(len(u), np.int64)
        np.add.at(cnt, inv, allp[:, 2])
        return np.stack([u >> 40, u & ((1 << 40) - 1), cnt], axis=1).astype(np.int64)

    def select(self, lower: int, upper: int, root: int = 0):
        """Export keys (ascending) and discriminative flags gathered on `root` (None elsewhere)."""
        keys, flags = self.e.select(lower, upper)
        ks = self._all_gather_var(np.ascontiguousarray(keys, dtype=np.uint64).view(np.int64))
        fs = self._all_gather_var(np.ascontiguousarray(flags, dtype=np.uint8).astype(np.int64))
        if self.rank != root:
            return None, None
        return (np.concatenate(ks).view(np.uint64) if ks else np.zeros(0, np.uint64),
                np.concatenate(fs).astype(np.uint8) if fs else np.zeros(0, np.uint8))

    def select_all(self, lower: int, upper: int):
        """The global export (ascending keys) on every rank, e.g. as the SDK set for the lookup."""
        keys, _ = self.e.select(lower, upper)
        ks = self._all_gather_var(np.ascontiguousarray(keys, dtype=np.uint64).view(np.int64))
        return np.concatenate(ks).view(np.uint64) if ks else np.zeros(0, np.uint64)

    def select_counts(self, lower: int, upper: int):
        """Export selection left on every owner's device; returns the global (n, n_discriminative)."""
        n, d = self.e.select_device(lower, upper)
        t = torch.tensor([n, d], dtype=torch.int64, device=self.comm_dev)
        dist.all_reduce(t, group=self.group)
        return int(t[0]), int(t[1])

    def _all_gather_var(self, arr: np.ndarray):
        """all_gather of a variable-length int64 vector per rank (rank order)."""
        n = torch.tensor([len(arr)], dtype=torch.int64, device=self.comm_dev)
        ns = [torch.empty_like(n) for _ in range(self.world)]
        dist.all_gather(ns, n, group=self.group)
        lens = [int(x.item()) for x in ns]
        m = max(lens + [1])
        buf = torch.zeros(m, dtype=torch.int64, device=self.comm_dev)
        if len(arr):
            buf[: len(arr)] = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int64)).to(self.comm_dev)
        outs = [torch.empty_like(buf) for _ in range(self.world)]
        dist.all_gather(outs, buf, group=self.group)
        return [o[:l].cpu().numpy() for o, l in zip(outs, lens)]


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
