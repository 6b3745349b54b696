"""Host-side C++ (libhga_host.so, the CLIs' argv handling) — no GPU needed."""
import os
import subprocess

import numpy as np
import pytest

import oracle
import pyref_reader

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "hybrid-genome-assembler_amd", "bin")
GOLD = os.path.join(ROOT, "tests", "golden")


def write(path, text):
    with open(path, "wb") as f:
        f.write(text.encode() if isinstance(text, str) else text)
    return str(path)


def check_reader(hga_mod, paths, annotate):
    got = hga_mod.load_records(paths, annotate)
    want = pyref_reader.read_records(paths, annotate)
    assert len(got["offsets"]) - 1 == len(want)
    for i, r in enumerate(want):
        a, b = int(got["offsets"][i]), int(got["offsets"][i + 1])
        assert got["bases"][a:b].decode("latin-1") == r["seq"]
        assert int(got["category"][i]) == r["cat"]
        assert (int(got["start"][i]), int(got["end"][i])) == (r["start"], r["end"])
    return got, want


def test_reader_fastq_fasta_mix(tmp_path, hga_mod):
    a = write(tmp_path / "a.fq", "@r1\nACGTN\n+\nIIIII\n@r2\nacgtACGT\n+\nIIIIIIII\n")
    b = write(tmp_path / "b.fa", ">s1\nTTTT\n>s2\nGATTACA\n")
    got, want = check_reader(hga_mod, [a, b], True)
    # FASTQ -> FASTA: the first record of the FASTA file is read with the FASTQ layout
    # (the reader switches layout only when it opens the next file) — reference quirk.
    assert [r["seq"] for r in want] == ["ACGTN", "acgtACGT", "TTTT"]
    assert got["filename"] == "a.fq__b.fa"
    meta = got["meta"]
    assert meta[0].tolist() == [2, 13, 5, 8, 6]
    # all-files meta never updates max_read_length (SequenceRecordIterator.cpp:45-48)
    assert meta[2][3] == 0


def test_reader_crlf_and_ids(tmp_path, hga_mod):
    a = write(tmp_path / "c.fq", "@x\r\nACGT\r\n+\r\nIIII\r\n@y\r\nGG\r\n+\r\nII\r\n")
    b = write(tmp_path / "d.fq", "@z\nCCCC\n+\nIIII\n")
    got, want = check_reader(hga_mod, [a, b], False)
    assert [r["seq"] for r in want] == ["ACGT\r", "GG\r", "CCCC"]   # no CR stripping
    assert got["category"].tolist() == [0, 0, 0]


def test_reader_nanosim_and_simlord_headers(tmp_path, hga_mod):
    a = write(tmp_path / "n.fa", ">hapA_1200_aligned_0_F_0_350_0\nACGT\n>hapA_77_aligned_1_R_0_90_0\nAC\n")
    b = write(tmp_path / "s.fq", "@read;length=120bp;startpos=5;x\nAAAA\n+\nIIII\n")
    got, want = check_reader(hga_mod, [a], True)
    assert (got["start"].tolist(), got["end"].tolist()) == ([1200, 77], [1550, 167])
    got, want = check_reader(hga_mod, [b], True)
    assert (got["start"].tolist(), got["end"].tolist()) == ([5], [125])


def test_reader_errors(tmp_path, hga_mod):
    bad = write(tmp_path / "bad.txt", "hello\nworld\n")
    with pytest.raises(hga_mod.HgaError, match="Unrecognized file format"):
        hga_mod.load_records([bad], True)
    with pytest.raises(hga_mod.HgaError, match="does not exist"):
        hga_mod.load_records([str(tmp_path / "nope.fq")], True)


def test_jf_stream_multiline(tmp_path, hga_mod):
    p = write(tmp_path / "m.fa", ">a\nACGT\nTTGA\n>b\nCC\n\n>c\nG\n")
    assert hga_mod.jf_stream(p) == b"ACGTTTGA\nCC\nG"
    q = write(tmp_path / "m.fq", "@a\nACGT\nAC\n+\nIIII\nII\n@b\nGG\n+a\n@I\n")
    assert hga_mod.jf_stream(q) == b"ACGTAC\nGG"


@pytest.mark.parametrize("v,s", [(100.0, "100"), (70.0, "70"), (100.01, "100.01"), (12.5, "12.5"),
                                 (0.07 * 100, "7.000000000000001"), (0.57 * 100, "56.99999999999999"), (40.0, "40"), (1e-5, "1e-05"),
                                 (1e16, "1e+16"), (1e15, "1000000000000000"), (0.0001, "0.0001"),
                                 (0.0, "0"), (99.5, "99.5")])
def test_fmt_double(hga_mod, v, s):
    assert hga_mod.fmt_double(v) == s


def test_generators_deterministic(hga_mod):
    g = hga_mod.gen_genome(10000, 5)
    assert len(g) == 10000 and set(g) <= set(b"ACGT")
    assert g == hga_mod.gen_genome(10000, 5)
    h = hga_mod.gen_haplotype(g, 0.03, 500, 9)
    assert len(h) == 10500
    r1 = hga_mod.gen_art(g, 5000, 150, 1)
    r2 = hga_mod.gen_art(g, 5000, 150, 1)
    assert r1.seq == r2.seq and r1.n == 5000
    assert r1.seq.count(b"\n") == 4999 and len(r1.bases) == 5000 * 150
    ns = hga_mod.gen_nanosim(g, 50, 3)
    lens = np.diff(ns.offsets)
    assert ns.n == 50 and lens.min() >= 1


def test_cli_help_needs_no_gpu():
    for tool in ("jf_occurrences", "categorization"):
        out = subprocess.run([os.path.join(BIN, tool), "--help"], capture_output=True, text=True, timeout=60)
        assert out.returncode == 0
        assert "Options" in out.stdout


def test_cli_argument_errors():
    out = subprocess.run([os.path.join(BIN, "jf_occurrences")], capture_output=True, text=True, timeout=60)
    assert out.returncode != 0 and "You need to specify paths to read files" in out.stderr
    out = subprocess.run([os.path.join(BIN, "categorization"), "x.fq"], capture_output=True, text=True, timeout=60)
    assert out.returncode != 0 and "You need to specify path to kmers" in out.stderr
    out = subprocess.run([os.path.join(BIN, "jf_occurrences"), "--bogus", "x"], capture_output=True, text=True,
                         timeout=60)
    assert out.returncode != 0 and "unrecognised option" in out.stderr


@pytest.mark.parametrize("n,threads", [(0, 1), (7, 1), (300_000, 1), (300_000, 5), (1_100_000, 16)])
def test_dump_writer_matches_restatement(tmp_path, n, threads):
    """write_kmer_dump (the dump cache of run_jellyfish.sh:5-6: "KMER COUNT" lines, LC_ALL=C order as
    given) formats chunks on several threads and writes them in order: byte-identical to a plain
    restatement for any thread count, including several chunks of 2^18 rows."""
    rng = np.random.default_rng(n + threads)
    k = 19
    keys = np.sort(rng.integers(0, 4 ** k, n, dtype=np.uint64))
    counts = rng.integers(1, 1 << 20, n, dtype=np.uint64).astype(np.uint32)
    import hga as hga_mod
    hga_mod.set_host_threads(threads)
    try:
        p = tmp_path / "d.txt"
        hga_mod.write_kmer_dump(str(p), k, keys, counts)
    finally:
        hga_mod.set_host_threads(0)
    got = p.read_text()
    lines = got.splitlines(keepends=True)
    assert len(lines) == n
    # written to d.txt.tmp and renamed once complete (an interrupted run leaves no truncated cache)
    assert sorted(x.name for x in tmp_path.iterdir()) == ["d.txt"]

    def kstr(c):
        return "".join("ACGT"[(int(c) >> (2 * (k - 1 - i))) & 3] for i in range(k))
    want = "".join(f"{kstr(c)} {int(v)}\n" for c, v in zip(keys[:2000], counts[:2000]))
    assert "".join(lines[:2000]) == want
    idx = rng.integers(0, max(n, 1), 200) if n else []
    for i in idx:
        kstr = "".join("ACGT"[(int(keys[i]) >> (2 * (k - 1 - j))) & 3] for j in range(k))
        assert lines[i] == f"{kstr} {int(counts[i])}\n"


@pytest.mark.parametrize("n,dup_frac,eol", [(0, 0.0, "\n"), (1, 0.0, "\n"), (12, 0.3, "\n"), (13, 0.0, ""),
                                            (1000, 0.2, "\n"), (29_000, 0.1, "\r\n"), (300_000, 0.05, "\n")])
def test_kmer_text_loader_matches_unordered_set(tmp_path, n, dup_frac, eol):
    """categorization's SDK loader (host/fastio.cpp load_kmer_text: lines encoded in parallel, the KmerID
    order computed by unordered_set_order instead of filling a std::unordered_set) against the oracle's
    load_text_file_kmers (read_clustering.cpp:18-33 with a real std::unordered_set<uint64_t>): same codes
    in the same iteration order (KmerIDs, ReadClusteringEngine.cpp:237-241), same k; sizes cross the
    set's rehash points, lines repeat (also as reverse complements: the same canonical code), CRLF lines
    (the CR is part of the line there), a last line without a newline."""
    import hga as hga_mod
    rng = np.random.default_rng(n)
    k = 19 if eol != "\r\n" else 18   # (with the CR a line is k + 1 long)
    comp = {"A": "T", "C": "G", "G": "C", "T": "A"}
    lines = ["".join(rng.choice(list("ACGT"), k)) for _ in range(n)]
    for i in range(n):
        if i and rng.random() < dup_frac:
            src = lines[int(rng.integers(0, i))]
            lines[i] = src if rng.random() < 0.5 else "".join(comp[c] for c in reversed(src))
    text = "".join(ln + (eol if eol else "\n") for ln in lines)
    if not eol and text:
        text = text[:-1]
    p = tmp_path / "sdk.txt"
    p.write_bytes(text.encode())
    got, gk = hga_mod.load_kmer_text(str(p))
    want, wk = oracle.load_sdk_text(text.encode())
    assert np.array_equal(got, want) and gk == wk


@pytest.mark.parametrize("n", [0, 1, 2, 11, 12, 13, 24, 100, 5000, 200_000])
def test_unordered_set_order_matches_libstdcxx(n):
    """unordered_set_order (libstdc++'s node list regrouped epoch by epoch between its rehashes) against a real
    std::unordered_set<uint64_t>: the oracle's load_text_file_kmers fills one from lines written so that
    each line's canonical code is the key itself (31-mers, the smaller strand), duplicates included."""
    import hga as hga_mod
    rng = np.random.default_rng(1000 + n)
    k = 31
    keys = rng.integers(0, 4 ** k, n, dtype=np.uint64)
    # make every key its own canonical form (the smaller of it and its reverse complement)
    lines, canon = [], []
    for v in keys.tolist():
        s = "".join("ACGT"[(v >> (2 * (k - 1 - j))) & 3] for j in range(k))
        rc = "".join({"A": "T", "C": "G", "G": "C", "T": "A"}[c] for c in reversed(s))
        lines.append(min(s, rc))
    text = ("\n".join(lines) + "\n").encode() if lines else b""
    want, _ = oracle.load_sdk_text(text)
    codes = [int("".join(str("ACGT".index(c)) for c in ln), 4) for ln in lines]
    got = hga_mod.unordered_set_order(np.array(codes, np.uint64))
    assert np.array_equal(got, want)
