"""Pins against the reference's OWN code (oracle/_ref/libref_hll.so: src/lib/HyperLogLog.hpp and
src/lib/MurmurHash3.cpp compiled unmodified by `make -C oracle ref`): the oracle's MurmurHash3_x86_32
and HyperLogLog restatements must agree with them bit for bit, registers and estimate, for every
k on edge-case reads (the codes fed exactly as KmerAnalysis.cpp:15-23 feeds them)."""
import random

import numpy as np
import pytest

import oracle
import pyref
import refimpl

pytestmark = pytest.mark.skipif(not refimpl.available(),
                                reason="oracle/_ref/libref_hll.so not built (needs /root/reference at build time)")


def test_murmur3_reference_vs_oracle_vs_pyref():
    rng = random.Random(11)
    for _ in range(3000):
        n = rng.randint(0, 40)
        data = bytes(rng.getrandbits(8) for _ in range(n))
        seed = rng.choice([0, 1, 313, 0xFFFFFFFF, rng.getrandbits(32)])
        h = refimpl.murmur3_x86_32(data, seed)
        assert oracle.murmur3_x86_32(data, seed) == h
        if n <= 16:
            assert pyref.murmur3_x86_32(data, seed) == h


def reads_case(seed, n, maxlen, alphabet):
    rng = random.Random(seed)
    reads = [("".join(rng.choice(alphabet) for _ in range(rng.randint(0, maxlen)))).encode() for _ in range(n)]
    return reads, b"".join(reads), np.cumsum([0] + [len(r) for r in reads]).astype(np.uint64)


def ref_codes(reads, k):
    parts = [oracle.kmer_windows(r, k)[0] for r in reads]
    return np.concatenate(parts) if parts else np.zeros(0, np.uint64)


@pytest.mark.parametrize("k", [1, 5, 11, 13, 15, 17, 19, 21, 23, 25, 27, 29, 31, 32])
@pytest.mark.parametrize("b", [4, 10, 14])
def test_hll_registers_and_estimate_vs_reference(k, b):
    reads, bases, offsets = reads_case(100 * k + b, 120, 200, "ACGTACGTACGTNacgt\r")
    regs_ref, est_ref = refimpl.hll(ref_codes(reads, k), b)
    regs = oracle.hll_registers(bases, offsets, k, b)
    assert np.array_equal(regs, regs_ref)
    assert oracle.hll_estimate(regs, b) == est_ref


def test_hll_estimate_ranges_vs_reference():
    # small-range (linear counting), raw and large-range branches of estimate() (:113-132)
    rng = np.random.default_rng(3)
    for n in (0, 1, 10, 300, 5000, 200000):
        codes = rng.integers(0, 1 << 62, n, dtype=np.uint64)
        regs_ref, est_ref = refimpl.hll(codes, 10)
        assert oracle.hll_estimate(regs_ref, 10) == est_ref
