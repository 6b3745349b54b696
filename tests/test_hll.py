"""HyperLogLog auto-k (src/occurrences/KmerAnalysis.cpp:15-56) — CPU side: the oracle against
published MurmurHash3 vectors and the independent Python restatement, the host estimate against
both, and the k-selection loop."""
import random

import numpy as np
import pytest

import oracle
import pyref

# Published MurmurHash3_x86_32 test vectors (data, seed, hash).
MURMUR_KAT = [(b"", 0, 0), (b"", 1, 0x514E28B7), (b"", 0xFFFFFFFF, 0x81F16F39),
              (b"\x00\x00\x00\x00", 0, 0x2362F9DE), (b"aaaa", 0x9747B28C, 0x5A97808A),
              (b"abc", 0, 0xB3DD93FA), (b"Hello, world!", 1234, 0xFAF6CDB3),
              (b"The quick brown fox jumps over the lazy dog", 0x9747B28C, 0x2FA826CD)]


@pytest.mark.parametrize("data,seed,h", MURMUR_KAT)
def test_murmur3_known_answers(data, seed, h):
    assert oracle.murmur3_x86_32(data, seed) == h
    assert pyref.murmur3_x86_32(data, seed) == h


def test_murmur3_u64_keys_agree():
    rng = random.Random(5)
    for _ in range(2000):
        x = rng.getrandbits(64)
        d = x.to_bytes(8, "little")
        assert oracle.murmur3_x86_32(d, 313) == pyref.murmur3_x86_32(d, 313)


def reads_case(seed, n, maxlen, alphabet="ACGT"):
    rng = random.Random(seed)
    reads = ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, maxlen))) for _ in range(n)]
    bases = "".join(reads).encode()
    offsets = np.cumsum([0] + [len(r) for r in reads]).astype(np.uint64)
    return reads, bases, offsets


@pytest.mark.parametrize("k,b", [(1, 4), (5, 10), (11, 10), (19, 8), (32, 12)])
def test_hll_registers_oracle_vs_pyref(k, b):
    reads, bases, offsets = reads_case(k * 7 + b, 60, 120, "ACGTACGTNacgt\r")
    assert oracle.hll_registers(bases, offsets, k, b).tolist() == pyref.hll_registers(reads, k, b)


def test_hll_k_too_big():
    _, bases, offsets = reads_case(1, 3, 50)
    with pytest.raises(ValueError):
        oracle.hll_registers(bases, offsets, 33)


@pytest.mark.parametrize("seed", range(6))
def test_hll_estimate_host_vs_oracle_vs_pyref(hga_mod, seed):
    rng = random.Random(seed)
    b = rng.choice([4, 5, 6, 10, 14])
    top = rng.choice([1, 3, 8, 23])       # sparse (linear counting) .. saturated registers
    regs = np.array([rng.randint(0, top) for _ in range(1 << b)], np.uint8)
    e = oracle.hll_estimate(regs, b)
    assert hga_mod.hll_estimate(regs, b) == e
    assert pyref.hll_estimate(regs.tolist(), b) == e


def test_hll_estimate_edge_registers(hga_mod):
    for b in (4, 10):
        for regs in (np.zeros(1 << b, np.uint8), np.full(1 << b, 23, np.uint8), np.full(1 << b, 1, np.uint8)):
            a, o = hga_mod.hll_estimate(regs, b), oracle.hll_estimate(regs, b)
            assert a == o or (np.isnan(a) and np.isnan(o))   # saturated b=4: log of a negative


def test_unique_k_length_loop():
    """A random 30 kb genome: the estimates grow with k until 4^k >> genome, then flatten."""
    rng = random.Random(9)
    g = "".join(rng.choice("ACGT") for _ in range(30000))
    reads = [g[i:i + 150] for i in range(0, 29850, 50)]
    bases = "".join(reads).encode()
    offsets = np.cumsum([0] + [len(r) for r in reads]).astype(np.uint64)
    (k, cnt), lines = oracle.unique_k_length(bases, offsets)
    assert lines[0].startswith("k=11 : ~") and 11 <= k <= 31 and len(lines) == (k - 11) // 2 + 2
    assert cnt == int(oracle.hll_estimate(oracle.hll_registers(bases, offsets, k)))
