"""ctypes binding of oracle/_build/liboracle.so — the CPU restatement (oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product.  Parity status: see the header of oracle.cpp
("parity unpinned" — the reference cannot be built here and ships no fixtures).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_build", "liboracle.so")

_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)
_i64p = C.POINTER(C.c_int64)
_i32p = C.POINTER(C.c_int32)
_u8p = C.POINTER(C.c_uint8)
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            build()
        L = C.CDLL(SO)
        L.or_free.argtypes = [C.c_void_p]
        L.or_kmer_windows.restype = C.c_int64
        L.or_kmer_windows.argtypes = [C.c_char_p, C.c_uint64, C.c_int, _u64p, _u32p]
        L.or_count_stream.restype = C.c_int64
        L.or_count_stream.argtypes = [C.c_char_p, C.c_uint64, C.c_int, C.c_uint32, C.POINTER(_u64p),
                                      C.POINTER(_u32p)]
        L.or_count_stream_mt.restype = C.c_int64
        L.or_count_stream_mt.argtypes = [C.c_char_p, C.c_uint64, C.c_int, C.c_uint32, C.c_int,
                                         C.POINTER(_u64p), C.POINTER(_u32p)]
        L.or_count_files_mt.restype = C.c_int64
        L.or_count_files_mt.argtypes = [C.c_int, C.POINTER(C.c_char_p), _u64p, C.c_int, C.c_uint32, C.c_int,
                                        C.POINTER(_u64p), C.POINTER(_u32p)]
        L.or_count_reference_like.restype = C.c_int64
        L.or_count_reference_like.argtypes = [C.c_char_p, C.c_uint64, C.c_int, C.c_uint32]
        L.or_construct_indices_mt.restype = C.c_int64
        L.or_construct_indices_mt.argtypes = [C.c_char_p, _u64p, C.c_uint64, _u32p, C.c_int, _u64p, C.c_uint32,
                                              C.c_int] + \
            [C.POINTER(_u64p), C.POINTER(_u32p), C.POINTER(_u32p), C.POINTER(_u32p), C.POINTER(_u64p),
             C.POINTER(_u32p), C.POINTER(_u32p), C.POINTER(_u64p), C.POINTER(_u32p), _u64p]
        L.or_count_instances.restype = C.c_uint64
        L.or_count_instances.argtypes = [C.c_char_p, C.c_uint64, C.c_int]
        L.or_merge.restype = C.c_int64
        L.or_merge.argtypes = [C.c_int, C.POINTER(_u64p), C.POINTER(_u32p), _u64p, C.POINTER(_u64p),
                               C.POINTER(_u32p)]
        L.or_specificity.restype = C.c_int64
        L.or_specificity.argtypes = [C.c_int, C.c_uint64, _u32p, C.POINTER(C.c_double), C.c_int,
                                     C.POINTER(_i64p)]
        L.or_select.restype = C.c_int64
        L.or_select.argtypes = [C.c_int, C.c_uint64, _u64p, _u32p, C.c_int64, C.c_int64, C.POINTER(_u64p),
                                _u64p]
        L.or_load_sdk_text.restype = C.c_int64
        L.or_load_sdk_text.argtypes = [C.c_char_p, C.c_uint64, C.POINTER(_u64p), C.POINTER(C.c_int)]
        L.or_construct_indices.restype = C.c_int64
        L.or_construct_indices.argtypes = [C.c_char_p, _u64p, C.c_uint64, _u32p, C.c_int, _u64p, C.c_uint32] + \
            [C.POINTER(_u64p), C.POINTER(_u32p), C.POINTER(_u32p), C.POINTER(_u32p), C.POINTER(_u64p),
             C.POINTER(_u32p), C.POINTER(_u32p), C.POINTER(_u64p), C.POINTER(_u32p), _u64p]
        L.or_connections.restype = C.c_int64
        L.or_connections.argtypes = [C.c_uint64, _u64p, _u32p, _u64p, _u32p, _u32p, _u32p, C.c_uint64, C.c_uint32,
                                     C.c_uint64, _i32p, C.POINTER(_u32p), C.POINTER(_u32p), C.POINTER(_u64p),
                                     C.POINTER(_u8p)]
        L.or_connections_mt.restype = C.c_int64
        L.or_connections_mt.argtypes = [C.c_uint64, _u64p, _u32p, _u64p, _u32p, _u32p, _u32p, C.c_uint64,
                                        C.c_uint32, C.c_uint64, C.c_int, C.POINTER(_u32p), C.POINTER(_u32p),
                                        C.POINTER(_u64p)]
        L.or_lookup_hits_mt.restype = C.c_uint64
        L.or_lookup_hits_mt.argtypes = [C.c_char_p, _u64p, C.c_uint64, C.c_int, _u64p, C.c_uint32, C.c_int]
        L.or_murmur3_x86_32.restype = C.c_uint32
        L.or_murmur3_x86_32.argtypes = [C.c_char_p, C.c_int, C.c_uint32]
        L.or_hll_registers.restype = C.c_int
        L.or_hll_registers.argtypes = [C.c_char_p, _u64p, C.c_uint64, C.c_int, C.c_int, _u8p]
        L.or_hll_estimate.restype = C.c_double
        L.or_hll_estimate.argtypes = [_u8p, C.c_int]
        _lib = L
    return _lib


def _take(ptr, n, dtype):
    try:
        if n == 0:
            return np.zeros(0, dtype=dtype)
        addr = C.cast(ptr, C.c_void_p).value
        buf = (C.c_char * (n * np.dtype(dtype).itemsize)).from_address(addr)
        return np.frombuffer(buf, dtype=dtype).copy()
    finally:
        lib().or_free(ptr)


def _p(a, ct):
    return a.ctypes.data_as(C.POINTER(ct))


def kmer_windows(seq: bytes, k: int):
    """KmerIterator over one read: (canonical codes, end-exclusive positions)."""
    n = max(len(seq) - k + 1, 0)
    codes = np.zeros(max(n, 1), np.uint64)
    pos = np.zeros(max(n, 1), np.uint32)
    w = lib().or_kmer_windows(seq, len(seq), k, _p(codes, C.c_uint64), _p(pos, C.c_uint32))
    if w < 0:
        raise ValueError("k out of range")
    return codes[:w], pos[:w]


def count_stream(seq: bytes, k: int, min_count: int = 2, threads: int = 0):
    kp, cp = _u64p(), _u32p()
    if threads:
        n = lib().or_count_stream_mt(seq, len(seq), k, min_count, threads, C.byref(kp), C.byref(cp))
    else:
        n = lib().or_count_stream(seq, len(seq), k, min_count, C.byref(kp), C.byref(cp))
    if n < 0:
        raise ValueError("k out of range")
    return _take(kp, n, np.uint64), _take(cp, n, np.uint32)


def count_files_mt(streams, k: int, min_count: int = 2, threads: int = 8):
    """Merged rows of the whole count stage (per-file exact counts, drop, merge), multi-threaded:
    (keys ascending, counts[rows, F])."""
    F = len(streams)
    arr = (C.c_char_p * F)(*streams)
    lens = np.array([len(x) for x in streams], np.uint64)
    kp, cp = _u64p(), _u32p()
    n = lib().or_count_files_mt(F, arr, _p(lens, C.c_uint64), k, min_count, threads, C.byref(kp), C.byref(cp))
    if n < 0:
        raise ValueError("k out of range")
    return _take(kp, n, np.uint64), _take(cp, n * F, np.uint32).reshape(-1, F)


def count_reference_like(seq: bytes, k: int, min_count: int = 2) -> int:
    """Single-thread count with the reference's map-based KmerIterator loop; returns rows (timing leg)."""
    return int(lib().or_count_reference_like(seq, len(seq), k, min_count))


def dumps_of(keys, counts):
    """Per-file dumps (rows with a nonzero count in that file) of merged rows."""
    return [(keys[counts[:, f] > 0], counts[counts[:, f] > 0, f]) for f in range(counts.shape[1])]


def count_instances(seq: bytes, k: int) -> int:
    return int(lib().or_count_instances(seq, len(seq), k))


def merge(dumps):
    """dumps: list of (keys, counts) per file -> (keys, counts[rows, F])."""
    F = len(dumps)
    ks = [np.ascontiguousarray(d[0], np.uint64) for d in dumps]
    cs = [np.ascontiguousarray(d[1], np.uint32) for d in dumps]
    kpa = (_u64p * F)(*[_p(a, C.c_uint64) for a in ks])
    cpa = (_u32p * F)(*[_p(a, C.c_uint32) for a in cs])
    lens = np.array([len(a) for a in ks], np.uint64)
    okp, ocp = _u64p(), _u32p()
    n = lib().or_merge(F, kpa, cpa, _p(lens, C.c_uint64), C.byref(okp), C.byref(ocp))
    return _take(okp, n, np.uint64), _take(ocp, n * F, np.uint32).reshape(-1, F)


def specificity(counts, thresholds):
    counts = np.ascontiguousarray(counts, np.uint32)
    F = counts.shape[1] if counts.ndim == 2 else 1
    thr = np.ascontiguousarray(thresholds, np.float64)
    p = _i64p()
    n = lib().or_specificity(F, counts.shape[0], _p(counts, C.c_uint32), _p(thr, C.c_double), len(thr),
                             C.byref(p))
    if n < 0:
        raise ValueError("row above the last threshold")
    return _take(p, 3 * n, np.int64).reshape(-1, 3)


def select(keys, counts, lower, upper):
    keys = np.ascontiguousarray(keys, np.uint64)
    counts = np.ascontiguousarray(counts, np.uint32)
    p = _u64p()
    d = C.c_uint64()
    n = lib().or_select(counts.shape[1], len(keys), _p(keys, C.c_uint64), _p(counts, C.c_uint32), lower, upper,
                        C.byref(p), C.byref(d))
    return _take(p, n, np.uint64), d.value


def load_sdk_text(text: bytes):
    p = _u64p()
    k = C.c_int()
    n = lib().or_load_sdk_text(text, len(text), C.byref(p), C.byref(k))
    if n < 0:
        raise ValueError("line longer than 32")
    return _take(p, n, np.uint64), k.value


def construct_indices(bases: bytes, offsets, k: int, sdk_keys, first_read_id: int = 1, threads: int = 0):
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = len(offsets) - 1
    ids = np.arange(first_read_id, first_read_id + n, dtype=np.uint32)
    sdk = np.ascontiguousarray(sdk_keys, np.uint64)
    ptrs = [_u64p(), _u32p(), _u32p(), _u32p(), _u64p(), _u32p(), _u32p(), _u64p(), _u32p()]
    nf = C.c_uint64()
    if threads:
        H = lib().or_construct_indices_mt(bases, _p(offsets, C.c_uint64), n, _p(ids, C.c_uint32), k,
                                          _p(sdk, C.c_uint64), len(sdk), threads, *[C.byref(x) for x in ptrs],
                                          C.byref(nf))
    else:
        H = lib().or_construct_indices(bases, _p(offsets, C.c_uint64), n, _p(ids, C.c_uint32), k,
                                       _p(sdk, C.c_uint64), len(sdk), *[C.byref(x) for x in ptrs], C.byref(nf))
    if H < 0:
        raise ValueError("k out of range")
    U = nf.value
    K = len(sdk)
    return {
        "hit_ptr": _take(ptrs[0], n + 1, np.uint64), "hit_kid": _take(ptrs[1], H, np.uint32),
        "hit_pos": _take(ptrs[2], H, np.uint32), "sorted_kid": _take(ptrs[3], H, np.uint32),
        "first_ptr": _take(ptrs[4], n + 1, np.uint64), "first_kid": _take(ptrs[5], U, np.uint32),
        "first_pos": _take(ptrs[6], U, np.uint32), "kci_ptr": _take(ptrs[7], K + 1, np.uint64),
        "kci_read": _take(ptrs[8], H, np.uint32),
    }


def connections(idx, pivots=None, min_kmers: int = 1, min_score: int = 1, categories=None,
                first_read_id: int = 1):
    """get_connections on construct_indices output `idx` (dict of construct_indices()).
    Returns (x, y, score, is_good), score descending then (x, y) ascending."""
    hp = np.ascontiguousarray(idx["hit_ptr"], np.uint64)
    n = len(hp) - 1
    sk = np.ascontiguousarray(idx["sorted_kid"], np.uint32)
    kp = np.ascontiguousarray(idx["kci_ptr"], np.uint64)
    kr = np.ascontiguousarray(idx["kci_read"], np.uint32)
    ids = np.arange(first_read_id, first_read_id + n, dtype=np.uint32)
    pv = None if pivots is None else np.ascontiguousarray(pivots, np.uint32)
    cat = None if categories is None else np.ascontiguousarray(categories, np.int32)
    px, py, ps, pg = _u32p(), _u32p(), _u64p(), _u8p()
    m = lib().or_connections(n, _p(hp, C.c_uint64), _p(sk, C.c_uint32), _p(kp, C.c_uint64), _p(kr, C.c_uint32),
                             _p(ids, C.c_uint32), None if pv is None else _p(pv, C.c_uint32),
                             0 if pv is None else len(pv), min_kmers, min_score,
                             None if cat is None else _p(cat, C.c_int32),
                             C.byref(px), C.byref(py), C.byref(ps), C.byref(pg))
    return _take(px, m, np.uint32), _take(py, m, np.uint32), _take(ps, m, np.uint64), _take(pg, m, np.uint8)


def connections_mt(idx, threads: int, pivots=None, min_kmers: int = 1, min_score: int = 1,
                   first_read_id: int = 1):
    """connections() (no categories) with the pivots split over `threads` threads: (x, y, score)."""
    hp = np.ascontiguousarray(idx["hit_ptr"], np.uint64)
    n = len(hp) - 1
    sk = np.ascontiguousarray(idx["sorted_kid"], np.uint32)
    kp = np.ascontiguousarray(idx["kci_ptr"], np.uint64)
    kr = np.ascontiguousarray(idx["kci_read"], np.uint32)
    ids = np.arange(first_read_id, first_read_id + n, dtype=np.uint32)
    pv = None if pivots is None else np.ascontiguousarray(pivots, np.uint32)
    px, py, ps = _u32p(), _u32p(), _u64p()
    m = lib().or_connections_mt(n, _p(hp, C.c_uint64), _p(sk, C.c_uint32), _p(kp, C.c_uint64),
                                _p(kr, C.c_uint32), _p(ids, C.c_uint32), None if pv is None else _p(pv, C.c_uint32),
                                0 if pv is None else len(pv), min_kmers, min_score, threads,
                                C.byref(px), C.byref(py), C.byref(ps))
    return _take(px, m, np.uint32), _take(py, m, np.uint32), _take(ps, m, np.uint64)


def lookup_hits_mt(bases: bytes, offsets, k: int, sdk_keys, threads: int) -> int:
    offsets = np.ascontiguousarray(offsets, np.uint64)
    sdk = np.ascontiguousarray(sdk_keys, np.uint64)
    return int(lib().or_lookup_hits_mt(bases, _p(offsets, C.c_uint64), len(offsets) - 1, k,
                                       _p(sdk, C.c_uint64), len(sdk), threads))


# The specificity thresholds of the jf_occurrences CLI (src/jellyfish_occurrences.cpp:47).
THRESHOLDS = [70.0, 85.0, 90.0, 95.0, 99.0, 100.0, 100.01]


def count_pipeline(streams, k, lower, upper, thresholds=THRESHOLDS, min_count=2):
    """Whole jf_occurrences counting path on the CPU: per-file dumps, merge, histogram, export."""
    dumps = [count_stream(s, k, min_count) for s in streams]
    keys, counts = merge(dumps)
    hist = specificity(counts, thresholds) if len(keys) else np.zeros((0, 3), np.int64)
    sel, disc = select(keys, counts, lower, upper)
    return {"dumps": dumps, "keys": keys, "counts": counts, "hist": hist, "selected": sel, "n_discr": disc}


def count_pipeline_mt(streams, k, lower, upper, threads, thresholds=THRESHOLDS, min_count=2):
    """count_pipeline's outputs from the multi-threaded count stage (or_count_files_mt)."""
    keys, counts = count_files_mt(streams, k, min_count, threads)
    hist = specificity(counts, thresholds) if len(keys) else np.zeros((0, 3), np.int64)
    sel, disc = select(keys, counts, lower, upper)
    return {"keys": keys, "counts": counts, "hist": hist, "selected": sel, "n_discr": disc}


def murmur3_x86_32(data: bytes, seed: int) -> int:
    """MurmurHash3_x86_32 (src/lib/MurmurHash3.cpp:94-140)."""
    return int(lib().or_murmur3_x86_32(data, len(data), seed))


def hll_registers(bases: bytes, offsets, k: int, b: int = 10):
    """HyperLogLog(b) registers over every KmerIterator window (KmerAnalysis.cpp:15-23)."""
    offs = np.ascontiguousarray(offsets, np.uint64)
    regs = np.zeros(1 << b, np.uint8)
    if lib().or_hll_registers(bases, _p(offs, C.c_uint64), len(offs) - 1, k, b, _p(regs, C.c_uint8)) < 0:
        raise ValueError("Kmer size is too big")
    return regs


def hll_estimate(regs, b: int = 10) -> float:
    """hll::HyperLogLog::estimate (src/lib/HyperLogLog.hpp:113-132)."""
    r = np.ascontiguousarray(regs, np.uint8)
    return float(lib().or_hll_estimate(_p(r, C.c_uint8), b))


def unique_k_length(bases: bytes, offsets, registers=None):
    """get_unique_k_length (KmerAnalysis.cpp:41-56): ((k, count), printed lines).
    `registers(k)` may supply the registers (e.g. from the GPU); default = the oracle's."""
    reg = registers or (lambda kk: hll_registers(bases, offsets, kk))
    count_of = lambda kk: int(hll_estimate(reg(kk)))   # double -> uint64_t, truncation
    lines = []
    k = 11
    prev = count_of(k)
    lines.append(f"k=11 : ~{prev} kmers")
    while k < 33:
        cnt = count_of(k + 2)
        lines.append(f"k={k + 2} : ~{cnt} kmers")
        if cnt + prev and abs(cnt - prev) / ((cnt + prev) / 2.0) < 0.1:
            return (k, prev), lines
        k += 2
        prev = cnt
    return (k, prev), lines
