"""Test-only counting engine for hga_dist.OwnerExchange on the CPU (gloo): the oracle does the
counting, numpy does partition/merge with the semantics libhga's kernels implement
(exchange.hip).  Lets the world_size>1 protocol run here without a GPU."""
import numpy as np
import torch

import oracle


class OracleEngine:
    def __init__(self, shards, k, packed=True):
        self.shards, self.k, self.n_files, self.packed = shards, k, len(shards), packed
        self.device = torch.device("cpu")
        self.keys = np.zeros(0, np.uint64)
        self.counts = np.zeros((0, self.n_files), np.uint32)

    def count_local(self):
        dumps = [oracle.count_stream(s, self.k, 1) for s in self.shards]
        self.keys, self.counts = oracle.merge(dumps)
        return len(self.keys)

    def partition(self, splitters, keys_buf, counts_buf):
        own = np.searchsorted(np.asarray(splitters, np.uint64), self.keys, side="right")
        order = np.argsort(own, kind="stable")
        keys_buf.copy_(torch.from_numpy(self.keys[order].view(np.int64)))
        counts_buf.copy_(torch.from_numpy(np.ascontiguousarray(self.counts[order]).reshape(-1).view(np.int32)))
        return np.bincount(own, minlength=len(splitters) + 1).astype(np.uint64)

    def merge(self, keys, counts, n, min_per_file):
        k = keys.numpy()[:n].view(np.uint64)
        c = counts.numpy()[: n * self.n_files].view(np.uint32).reshape(n, self.n_files).astype(np.uint64)
        uk, inv = np.unique(k, return_inverse=True)
        acc = np.zeros((len(uk), self.n_files), np.uint64)
        np.add.at(acc, inv, c)
        acc[acc < min_per_file] = 0
        keep = acc.sum(axis=1) > 0
        self.keys, self.counts = uk[keep], acc[keep].astype(np.uint32)

    # packed form, same layout as exchange.hip: key in the low 2k bits, per-file counts above
    def pack_bits(self):
        if not self.packed:
            return 0
        cb = (64 - 2 * self.k) // self.n_files
        return min(cb, 32) if (self.n_files <= 8 and cb >= 4) else 0

    def _pieces(self):
        cb = self.pack_bits()
        cmax = (1 << cb) - 1
        out = []
        for key, cnt in zip(self.keys.tolist(), self.counts.tolist()):
            left = list(cnt)
            while True:
                v = key
                for f in range(self.n_files):
                    c = min(left[f], cmax)
                    left[f] -= c
                    v |= c << (2 * self.k + f * cb)
                out.append(v)
                if not any(left):
                    break
        return np.array(out, dtype=np.uint64)

    def partition_packed(self, splitters, buf, capacity):
        pcs = self._pieces()
        own = np.searchsorted(np.asarray(splitters, np.uint64), pcs & np.uint64((1 << (2 * self.k)) - 1),
                              side="right")
        order = np.argsort(own, kind="stable")
        per = np.bincount(own, minlength=len(splitters) + 1).astype(np.uint64)
        if len(pcs) <= capacity:
            buf[: len(pcs)].copy_(torch.from_numpy(pcs[order].view(np.int64)))
        return per, len(pcs)

    def merge_packed(self, buf, n, min_per_file):
        cb = self.pack_bits()
        pcs = buf.numpy()[:n].view(np.uint64)
        kmask = np.uint64((1 << (2 * self.k)) - 1)
        keys = pcs & kmask
        counts = np.stack([(pcs >> np.uint64(2 * self.k + f * cb)) & np.uint64((1 << cb) - 1)
                           for f in range(self.n_files)], axis=1) if n else np.zeros((0, self.n_files), np.uint64)
        uk, inv = np.unique(keys, return_inverse=True)
        acc = np.zeros((len(uk), self.n_files), np.uint64)
        np.add.at(acc, inv, counts)
        acc[acc < min_per_file] = 0
        keep = acc.sum(axis=1) > 0
        self.keys, self.counts = uk[keep], acc[keep].astype(np.uint32)

    def spec_hist(self, thresholds):
        if not len(self.keys):
            return np.zeros((0, 3), np.int64)
        return oracle.specificity(self.counts, thresholds)

    def _sel(self, lower, upper):
        tot = self.counts.astype(np.int64).sum(axis=1)
        m = (tot >= lower) & (tot <= upper)
        return self.keys[m], ((self.counts[m] > 0).sum(axis=1) == 1).astype(np.uint8)

    def select(self, lower, upper):
        return self._sel(lower, upper)

    def select_device(self, lower, upper):
        k, f = self._sel(lower, upper)
        return len(k), int(f.sum())
