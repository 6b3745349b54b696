"""End-to-end runs of the drop-in CLIs (bin/jf_occurrences, bin/categorization) on the GPU."""
import os
import shutil
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


def stage_reads(tmp_path, names=("reads_a.fq", "reads_b.fq")):
    """Copies of the golden reads: jf_occurrences writes its dump caches next to them."""
    out = []
    for n in names:
        shutil.copy(os.path.join(GOLD, n), tmp_path / n)
        out.append(str(tmp_path / n))
    return out


def dump_text(keys, counts, k):
    return "".join(f"{kmer_str(c, k)} {int(n)}\n" for c, n in zip(keys, counts))


@pytest.mark.parametrize("k,stdin,fname", [(19, "3 12 1\n", "19-mers_3_12_100%.txt"),
                                           (15, "2 40 1.0\n", "15-mers_2_40_100%.txt")])
def test_jf_occurrences_end_to_end(tmp_path, hga_mod, k, stdin, fname):
    lower, upper = int(stdin.split()[0]), int(stdin.split()[1])
    paths = stage_reads(tmp_path)
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
    paths = stage_reads(tmp_path)
    env = dict(os.environ, HGA_PLOT_CMD="cat > /dev/null")
    out = subprocess.run([os.path.join(BIN, "jf_occurrences"), *paths, "--k-size=19", "-o", "sel.txt"],
                         input="3 12 0.5", text=True, capture_output=True, cwd=tmp_path, env=env, timeout=300)
    assert out.returncode == 0, out.stderr
    full = oracle.count_pipeline([hga_mod.jf_stream(p) for p in paths], 19, 3, 12)
    got = open(tmp_path / "sel.txt").read().split()
    allk = {kmer_str(c, 19) for c in full["selected"]}
    assert set(got) <= allk and got == sorted(got)
    assert 0 < len(got) < len(allk)


def test_jf_occurrences_writes_dump_cache(tmp_path, hga_mod):
    """Every counted file leaves "<reads>_<k>-mers_sorted" as run_jellyfish.sh:5-6 would."""
    paths = stage_reads(tmp_path)
    env = dict(os.environ, HGA_PLOT_CMD="cat > /dev/null")
    out = subprocess.run([os.path.join(BIN, "jf_occurrences"), *paths, "-k", "17"], input="3 12 1",
                         text=True, capture_output=True, cwd=tmp_path, env=env, timeout=300)
    assert out.returncode == 0, out.stderr
    for p in paths:
        keys, counts = oracle.count_stream(hga_mod.jf_stream(p), 17, 2)
        assert open(p + "_17-mers_sorted").read() == dump_text(keys, counts, 17)


def test_jf_occurrences_reads_dump_cache(tmp_path, hga_mod):
    """A file with an existing dump is not read; its rows (even count 1) are merged verbatim
    (JellyfishOccurrenceReader.cpp:19-24, 63-86)."""
    k = 19
    paths = stage_reads(tmp_path)
    stream_b = hga_mod.jf_stream(paths[1])
    ka, ca = oracle.count_stream(hga_mod.jf_stream(paths[0]), k, 2)
    rng = np.random.default_rng(5)
    ca = ca.copy()
    ca[rng.integers(0, len(ca), 200)] = 1                      # counts the GPU drop would remove
    extra = rng.integers(0, 1 << (2 * k), 300, dtype=np.uint64)  # k-mers absent from the reads
    ka2 = np.concatenate([ka, extra])
    ca2 = np.concatenate([ca, rng.integers(1, 40, 300).astype(np.uint32)])
    keep = np.unique(ka2, return_index=True)[1]
    ka2, ca2 = ka2[keep], ca2[keep]
    open(paths[0] + f"_{k}-mers_sorted", "w").write(dump_text(ka2, ca2, k))
    open(paths[0], "w").write("not a read file\n")          # must not be opened
    env = dict(os.environ, HGA_PLOT_CMD=f"cat > {tmp_path}/wire.txt")
    out = subprocess.run([os.path.join(BIN, "jf_occurrences"), *paths, "-k", str(k)], input="2 30 1",
                         text=True, capture_output=True, cwd=tmp_path, env=env, timeout=300)
    assert out.returncode == 0, out.stderr
    kb, cb = oracle.count_stream(stream_b, k, 2)
    keys, counts = oracle.merge([(ka2, ca2), (kb, cb)])
    hist = oracle.specificity(counts, oracle.THRESHOLDS)
    sel, disc = oracle.select(keys, counts, 2, 30)
    assert out.stdout.endswith(f"{disc} out of {len(sel)} exported kmers are discriminative")
    assert open(tmp_path / "wire.txt").read() == expected_wire(hist, k)
    assert open(tmp_path / "19-mers_2_30_100%.txt").read() == "".join(kmer_str(c, k) + "\n" for c in sel)
    assert open(paths[1] + f"_{k}-mers_sorted").read() == dump_text(kb, cb, k)


@pytest.mark.parametrize("tool", ["bin", "script"])
def test_run_jellyfish_dump(tmp_path, hga_mod, tool):
    """run_jellyfish(.sh) <reads> <k> <sorted>: the dump contract of run_jellyfish.sh:3-6."""
    reads = stage_reads(tmp_path, ("reads_c.fa",))[0]
    exe = (os.path.join(BIN, "run_jellyfish") if tool == "bin" else
           os.path.join(ROOT, "hybrid-genome-assembler_amd", "scripts", "run_jellyfish.sh"))
    out = subprocess.run([exe, reads, "15", str(tmp_path / "sorted")], capture_output=True, text=True,
                         cwd=tmp_path, timeout=300)
    assert out.returncode == 0, out.stderr
    keys, counts = oracle.count_stream(hga_mod.jf_stream(reads), 15, 2)
    assert len(keys) > 0
    assert open(tmp_path / "sorted").read() == dump_text(keys, counts, 15)


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


@pytest.mark.parametrize("args,cfg", [
    (["--sc_min_size", "5", "--core_enrichment", "8", "--tail_amplification", "10"],
     dict(sc_min=5, sc_max=-1, sc_fraction=0.15, sc_score=0, enrich=8, tail=10, dims=16)),
    (["--sc_min_size", "3", "--sc_max_size", "40", "--sc_fraction", "0.3", "--core_enrichment", "4",
      "--tail_amplification", "6", "--spectral_dims", "4"],
     dict(sc_min=3, sc_max=40, sc_fraction=0.3, sc_score=0, enrich=4, tail=6, dims=4))])
def test_categorization_clusters_and_export(tmp_path, hga_mod, args, cfg):
    """The whole categorization run (first connection pass on the GPU, the rest on the host) against
    the Python restatement of run_clustering + export_components (ReadClusteringEngine.cpp:699-826)."""
    import pyref_cluster as pc
    k = 15
    ga = hga_mod.gen_genome(40_000, 5)
    gb = hga_mod.gen_haplotype(ga, 0.02, 0, 6)
    paths = [str(tmp_path / "hapA.fa"), str(tmp_path / "hapB.fa")]
    hga_mod.write_nanosim_fasta(ga, "hapA", 180, 7, paths[0])
    hga_mod.write_nanosim_fasta(gb, "hapB", 180, 8, paths[1])
    ka, _ = oracle.kmer_windows(ga, k)
    kb, _ = oracle.kmer_windows(gb, k)
    sdk = np.setxor1d(np.unique(ka), np.unique(kb))
    (tmp_path / "sdk.txt").write_text("".join(kmer_str(c, k) + "\n" for c in sdk))
    out = subprocess.run([os.path.join(BIN, "categorization"), *paths, "-k", str(tmp_path / "sdk.txt"), "-d",
                          "-o", str(tmp_path / "clusters"), *args], capture_output=True, text=True, cwd=tmp_path,
                         timeout=300)
    assert out.returncode == 0, out.stderr
    for line in ("Index construction took", "Calculation of connections between reads took", "Union-find took",
                 "Merging into core components took"):
        assert line in out.stdout
    rec = hga_mod.load_records(paths, True)
    idx = oracle.construct_indices(rec["bases"], rec["offsets"], k, sdk)
    lengths = np.diff(rec["offsets"])
    eng = pc.Engine(idx, lengths, rec["category"], int(rec["meta"][-1][4]), True, cfg, start=rec["start"],
                    end=rec["end"])
    want = eng.run()
    assert f"Exported {len(want)} components\n" in out.stdout
    # -d: print_components after each merge (ReadClusteringEngine.cpp:189-198 at :766, :781, :797)
    assert [ln for ln in out.stdout.splitlines() if ln.startswith("#")] == eng.printed
    assert out.stdout.count("### Printing") >= 2
    files = sorted(os.listdir(tmp_path / "clusters"))
    assert files == sorted(f"#{c}.fa" for c in want)
    headers = [l.split("\n")[0] for p in paths for l in open(p).read().split(">")[1:]]
    for c in want:
        text = open(tmp_path / "clusters" / f"#{c}.fa").read()
        members = sorted(eng.comps[c]["reads"])
        exp = "".join(f">{headers[r - 1]}\n{rec['bases'][rec['offsets'][r - 1]:rec['offsets'][r]].decode()}\n"
                      for r in members)
        assert text == exp


@pytest.mark.parametrize("gpus,cache", [(2, False), (3, False), (2, True)])
def test_jf_occurrences_multi_rank(tmp_path, hga_mod, gpus, cache):
    """--gpus N: N ranks in one process (on a one-GPU box they share it through the library's host
    transport; one rank per GPU over RCCL otherwise), each counting a share of every file, then
    hga_count_exchange.  Export file, stdout, plot wire and the dump caches equal the oracle's, and
    an existing cache (read on rank 0 only) is merged exactly as with one GPU."""
    k, lower, upper = 17, 3, 12
    paths = stage_reads(tmp_path)
    streams = [hga_mod.jf_stream(p) for p in paths]
    o = oracle.count_pipeline(streams, k, lower, upper)
    if cache:   # file 0 comes from its dump cache (JellyfishOccurrenceReader.cpp:19-24)
        open(f"{paths[0]}_{k}-mers_sorted", "w").write(dump_text(*o["dumps"][0], k))
    env = dict(os.environ, HGA_PLOT_CMD=f"cat > {tmp_path}/wire.txt")
    out = subprocess.run([os.path.join(BIN, "jf_occurrences"), *paths, "-k", str(k), "--gpus", str(gpus)],
                         input=f"{lower} {upper} 1\n", text=True, capture_output=True, cwd=tmp_path, env=env,
                         timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout == ("0\nEnter lower and upper bounds for exported kmers as well as percentage\n"
                          f"{o['n_discr']} out of {len(o['selected'])} exported kmers are discriminative")
    assert open(tmp_path / "wire.txt").read() == expected_wire(o["hist"], k)
    assert open(tmp_path / f"{k}-mers_{lower}_{upper}_100%.txt").read() == \
        "".join(kmer_str(c, k) + "\n" for c in o["selected"])
    for f in range(2):
        assert open(f"{paths[f]}_{k}-mers_sorted").read() == dump_text(*o["dumps"][f], k)


@pytest.mark.parametrize("gpus", [2, 3])
def test_categorization_multi_rank_equals_one(tmp_path, hga_mod, gpus):
    """categorization --gpus N (sharded lookup + hga_lookup_gather, the device connection pass split
    over the ranks + hga_connections_gather): the index file, the printed lines (timings aside) and the
    exported clusters equal the one-GPU run's."""
    k = 15
    ga = hga_mod.gen_genome(40_000, 5)
    gb = hga_mod.gen_haplotype(ga, 0.02, 0, 6)
    paths = [str(tmp_path / "hapA.fa"), str(tmp_path / "hapB.fa")]
    hga_mod.write_nanosim_fasta(ga, "hapA", 180, 7, paths[0])
    hga_mod.write_nanosim_fasta(gb, "hapB", 180, 8, paths[1])
    ka, _ = oracle.kmer_windows(ga, k)
    kb, _ = oracle.kmer_windows(gb, k)
    sdk = np.setxor1d(np.unique(ka), np.unique(kb))
    (tmp_path / "sdk.txt").write_text("".join(kmer_str(c, k) + "\n" for c in sdk))
    res = {}
    for g in (1, gpus):
        out = subprocess.run([os.path.join(BIN, "categorization"), *paths, "-k", str(tmp_path / "sdk.txt"), "-d",
                              "-o", str(tmp_path / f"cl{g}"), "--index-out", str(tmp_path / f"idx{g}.bin"),
                              "--sc_min_size", "5", "--core_enrichment", "8", "--tail_amplification", "10",
                              "--gpus", str(g)], capture_output=True, text=True, cwd=tmp_path, timeout=300)
        assert out.returncode == 0, out.stderr
        lines = [l for l in out.stdout.splitlines() if " took " not in l]
        files = {f: open(tmp_path / f"cl{g}" / f).read() for f in sorted(os.listdir(tmp_path / f"cl{g}"))}
        res[g] = (lines, files, open(tmp_path / f"idx{g}.bin", "rb").read())
    assert res[1][2] == res[gpus][2]
    assert res[1][0] == res[gpus][0]
    assert res[1][1] == res[gpus][1] and len(res[1][1]) > 1
