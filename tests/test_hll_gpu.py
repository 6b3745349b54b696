"""HyperLogLog registers on the MI355X (hga_hll_registers) against the oracle: bit-exact registers
for every k, edge-case reads, register widths; the k-selection loop and the CLI without -k."""
import os
import random
import subprocess

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "hybrid-genome-assembler_amd", "bin")
GOLD = os.path.join(ROOT, "tests", "golden")


def case(seed, n, maxlen, alphabet):
    rng = random.Random(seed)
    reads = [("".join(rng.choice(alphabet) for _ in range(rng.randint(0, maxlen)))).encode() for _ in range(n)]
    return b"".join(reads), np.cumsum([0] + [len(r) for r in reads]).astype(np.uint64)


@pytest.mark.parametrize("k", list(range(1, 33)))
def test_hll_registers_every_k(gpu_ctx, k):
    bases, offsets = case(k, 400, 300, "ACGTACGTACGTNacg\r")
    gpu_ctx.lookup_set_reads(bases, offsets, 1)
    assert np.array_equal(gpu_ctx.hll_registers(k, 10), oracle.hll_registers(bases, offsets, k, 10))


@pytest.mark.parametrize("b", [4, 7, 10, 14])
def test_hll_register_widths(gpu_ctx, b):
    bases, offsets = case(100 + b, 300, 500, "ACGT")
    gpu_ctx.lookup_set_reads(bases, offsets, 1)
    assert np.array_equal(gpu_ctx.hll_registers(19, b), oracle.hll_registers(bases, offsets, 19, b))


def test_hll_edge_reads(gpu_ctx, hga_mod):
    reads = [b"", b"A", b"ACGTACGTACGTACGTACG", b"N" * 40, b"acgtacgtacgtacgtacgtacgt", b"", b"ACGT\rACGT" * 7,
             b"T" * 33, b"G" * 64, b"C" * 65, b"A" * 31]
    bases = b"".join(reads)
    offsets = np.cumsum([0] + [len(r) for r in reads]).astype(np.uint64)
    gpu_ctx.lookup_set_reads(bases, offsets, 1)
    for k in (1, 2, 19, 31, 32):
        assert np.array_equal(gpu_ctx.hll_registers(k, 10), oracle.hll_registers(bases, offsets, k, 10)), k
    with pytest.raises(hga_mod.HgaError):
        gpu_ctx.hll_registers(33, 10)          # KmerIterator: "Kmer size is too big"
    with pytest.raises(hga_mod.HgaError):
        gpu_ctx.hll_registers(19, 3)           # HyperLogLog: b out of range


def test_hll_large_genome_reads(gpu_ctx, hga_mod):
    g = hga_mod.gen_genome(400_000, 11)
    r = hga_mod.gen_art(g, 40_000, 150, 12)
    gpu_ctx.lookup_set_reads(r.bases, r.offsets, 1)
    for k in (11, 19):
        assert np.array_equal(gpu_ctx.hll_registers(k, 10), oracle.hll_registers(r.bases, r.offsets, k, 10))


def test_unique_k_length_gpu_vs_oracle(gpu_ctx, hga_mod):
    g = hga_mod.gen_genome(60_000, 21)
    r = hga_mod.gen_art(g, 6000, 150, 22)
    gpu_ctx.lookup_set_reads(r.bases, r.offsets, 1)
    assert gpu_ctx.unique_k_length() == oracle.unique_k_length(r.bases, r.offsets)


def test_jf_occurrences_without_k(tmp_path, hga_mod):
    """No -k: the HyperLogLog lines, then the count at the chosen k (jellyfish_occurrences.cpp:40-44)."""
    paths = []
    for i, name in enumerate(("a.fq", "b.fq")):
        g = hga_mod.gen_genome(30_000, 31 + i)
        hga_mod.write_art_fastq(g, name[0], 3000, 150, 41 + i, str(tmp_path / name))
        paths.append(str(tmp_path / name))
    rec = hga_mod.load_records(paths, True)
    (k, _), lines = oracle.unique_k_length(rec["bases"], rec["offsets"])
    env = dict(os.environ, HGA_PLOT_CMD="cat > /dev/null", HGA_DUMP_CACHE="0")
    out = subprocess.run([os.path.join(BIN, "jf_occurrences"), *paths], input="2 40 1", text=True,
                         capture_output=True, cwd=tmp_path, env=env, timeout=300)
    assert out.returncode == 0, out.stderr
    o = oracle.count_pipeline([hga_mod.jf_stream(p) for p in paths], k, 2, 40)
    assert out.stdout == ("\n".join(lines) + "\n0\nEnter lower and upper bounds for exported kmers as well as "
                          f"percentage\n{o['n_discr']} out of {len(o['selected'])} exported kmers are discriminative")
    assert os.path.exists(tmp_path / f"{k}-mers_2_40_100%.txt")


@pytest.mark.parametrize("k", [11, 15, 19, 23, 27, 31])
def test_hll_registers_vs_reference_code(gpu_ctx, k):
    """GPU registers against the reference's own hll::HyperLogLog (oracle/_ref, tests/test_ref_pin.py)."""
    import refimpl
    if not refimpl.available():
        pytest.skip("oracle/_ref/libref_hll.so not built")
    bases, offsets = case(1000 + k, 300, 400, "ACGTACGTACGTNacg\r")
    gpu_ctx.lookup_set_reads(bases, offsets, 1)
    codes = [oracle.kmer_windows(bases[int(a):int(b)], k)[0] for a, b in zip(offsets[:-1], offsets[1:])]
    regs_ref, est_ref = refimpl.hll(np.concatenate(codes), 10)
    regs = gpu_ctx.hll_registers(k, 10)
    assert np.array_equal(regs, regs_ref)
    assert oracle.hll_estimate(regs, 10) == est_ref
