"""End-to-end runs of the drop-in CLIs (bin/jf_occurrences, bin/categorization) on the GPU."""
import os
import subprocess

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "hybrid-genome-assembler_amd", "bin")
GOLD = os.path.join(ROOT, "tests", "golden")


def kmer_str(code, k):
    return "".join("ACGT"[(int(code) >> (2 * (k - 1 - i))) & 3] for i in range(k))


def expected_wire(hist, k):
    # plot_kmer_specificity (src/common/Plotting.cpp:20-37), fmt formatting of the thresholds
    names = ["70", "85", "90", "95", "99", "100", "100.01"]
    bounds = []
    for ti, name in enumerate(names):
        counts = [f"({t}, {c})" for i, t, c in hist.tolist() if i == ti and c >= 50]
        bounds.append(f"({name}, [{', '.join(counts)}])")
    return f"1 200\n({k}, [{', '.join(bounds)}])"


@pytest.mark.parametrize("k,stdin,fname", [(19, "3 12 1\n", "19-mers_3_12_100%.txt"),
                                           (15, "2 40 1.0\n", "15-mers_2_40_100%.txt")])
def test_jf_occurrences_end_to_end(tmp_path, hga_mod, k, stdin, fname):
    lower, upper = int(stdin.split()[0]), int(stdin.split()[1])
    paths = [os.path.join(GOLD, p) for p in ("reads_a.fq", "reads_b.fq")]
    env = dict(os.environ, HGA_PLOT_CMD=f"cat > {tmp_path}/wire.txt")
    out = subprocess.run([os.path.join(BIN, "jf_occurrences"), *paths, "-k", str(k)], input=stdin, text=True,
                         capture_output=True, cwd=tmp_path, env=env, timeout=300)
    assert out.returncode == 0, out.stderr
    streams = [hga_mod.jf_stream(p) for p in paths]
    o = oracle.count_pipeline(streams, k, lower, upper)
    assert out.stdout == ("0\nEnter lower and upper bounds for exported kmers as well as percentage\n"
                          f"{o['n_discr']} out of {len(o['selected'])} exported kmers are discriminative")
    assert open(tmp_path / "wire.txt").read() == expected_wire(o["hist"], k)
    lines = open(tmp_path / fname).read()
    assert lines == "".join(kmer_str(c, k) + "\n" for c in o["selected"])


def test_jf_occurrences_output_option_and_sampling(tmp_path, hga_mod):
    paths = [os.path.join(GOLD, p) for p in ("reads_a.fq", "reads_b.fq")]
    env = dict(os.environ, HGA_PLOT_CMD="cat > /dev/null")
    out = subprocess.run([os.path.join(BIN, "jf_occurrences"), *paths, "--k-size=19", "-o", "sel.txt"],
                         input="3 12 0.5", text=True, capture_output=True, cwd=tmp_path, env=env, timeout=300)
    assert out.returncode == 0, out.stderr
    full = oracle.count_pipeline([hga_mod.jf_stream(p) for p in paths], 19, 3, 12)
    got = open(tmp_path / "sel.txt").read().split()
    allk = {kmer_str(c, 19) for c in full["selected"]}
    assert set(got) <= allk and got == sorted(got)
    assert 0 < len(got) < len(allk)


def test_categorization_end_to_end(tmp_path):
    g = np.load(os.path.join(GOLD, "lookup_golden.npz"))
    paths = [os.path.join(GOLD, p) for p in ("reads_a.fq", "reads_b.fq", "reads_c.fa")]
    out = subprocess.run([os.path.join(BIN, "categorization"), *paths, "-k", os.path.join(GOLD, "sdk_19.txt"),
                          "-d", "--index-out", str(tmp_path / "idx.bin")], capture_output=True, text=True,
                         cwd=tmp_path, timeout=300)
    assert out.returncode == 0, out.stderr
    assert "reads_a.fq:\n- " in out.stdout and "Index construction took " in out.stdout
    # the debug discriminative line (ReadClusteringEngine.cpp:285-297)
    cat = g["category"]
    disc = tot = 0
    for i in range(len(g["kci_ptr"]) - 1):
        cs = {int(cat[r - 1]) for r in g["kci_read"][g["kci_ptr"][i]:g["kci_ptr"][i + 1]]}
        disc += len(cs) == 1
        tot += len(cs) > 0
    assert f"{disc} out of {tot} kmers are discriminative \n" in out.stdout
    raw = open(tmp_path / "idx.bin", "rb").read()
    n, H, U, K, k = np.frombuffer(raw[:40], np.uint64)
    assert (n, H, U, K, k) == (len(g["hit_ptr"]) - 1, len(g["hit_kid"]), len(g["first_kid"]), len(g["kci_ptr"]) - 1, 19)
    off = 40
    for name, cnt, dt in [("hit_ptr", n + 1, np.uint64), ("sorted_kid", H, np.uint32), ("first_ptr", n + 1, np.uint64),
                          ("first_kid", U, np.uint32), ("first_pos", U, np.uint32), ("kci_ptr", K + 1, np.uint64),
                          ("kci_read", H, np.uint32)]:
        arr = np.frombuffer(raw[off:off + int(cnt) * np.dtype(dt).itemsize], dt)
        off += int(cnt) * np.dtype(dt).itemsize
        assert np.array_equal(arr, g[name]), name
