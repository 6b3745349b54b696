"""Multi-threaded readers (host/fastio.cpp) against the sequential restatements (seqio.cpp):
identical jf_stream bytes and load_records outputs on regular, irregular and edge-case files."""
import os
import random

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture
def threads(hga_mod):
    yield hga_mod
    hga_mod.set_host_threads(0)


def both(hga_mod, fn):
    hga_mod.set_host_threads(1)
    a = fn()
    hga_mod.set_host_threads(4)
    b = fn()
    return a, b


def same_records(a, b):
    for k in ("bases", "filename"):
        assert a[k] == b[k], k
    for k in ("offsets", "category", "start", "end", "meta"):
        assert np.array_equal(a[k], b[k]), k


def rnd_seq(rng, n, alphabet="ACGT"):
    return "".join(rng.choice(alphabet) for _ in range(n))


def write(tmp_path, name, text):
    p = tmp_path / name
    p.write_bytes(text.encode() if isinstance(text, str) else text)
    return str(p)


def fastq(rng, n, maxlen=90, crlf=False, blank_seq=False):
    e = "\r\n" if crlf else "\n"
    out = []
    for i in range(n):
        s = "" if blank_seq and i % 5 == 0 else rnd_seq(rng, rng.randint(1, maxlen), "ACGTNacgt")
        q = "".join(rng.choice("@+!ABCGT#") for _ in s)
        out.append(f"@r{i}_A{e}{s}{e}+{e}{q}{e}")
    return "".join(out)


def fasta(rng, n, multiline=False, nanosim=False):
    out = []
    for i in range(n):
        s = rnd_seq(rng, rng.randint(0, 200))
        h = f">ref_{rng.randint(1, 9999)}_aligned_{i}_F_0_{len(s)}_0" if nanosim else f">read{i} ACGT"
        if multiline and len(s) > 60:
            s = "\n".join(s[j:j + 60] for j in range(0, len(s), 60))
        out.append(f"{h}\n{s}\n")
    return "".join(out)


CASES = {
    "fastq": lambda r: fastq(r, 500),
    "fastq_crlf": lambda r: fastq(r, 300, crlf=True),
    "fastq_empty_seqs": lambda r: fastq(r, 300, blank_seq=True),
    "fastq_no_final_newline": lambda r: fastq(r, 200).rstrip("\n"),
    "fasta": lambda r: fasta(r, 400),
    "fasta_multiline": lambda r: fasta(r, 300, multiline=True),
    "fasta_nanosim": lambda r: fasta(r, 300, nanosim=True),
    "fasta_leading_blank": lambda r: "\n\n" + fasta(r, 50),
    "fastq_multiline_seq": lambda r: "@a\nACGT\nACGT\n+\nIIII\nIIII\n@b\nGG\n+\n!!\n",
    "fastq_plus_seq": lambda r: "@a\n+ACGT\n+\nIIIII\n@b\nGGT\n+\n!!!\n",
    "fastq_short_qual": lambda r: "@a\nACGTACGT\n+\nIIII\nIIII\n@b\nGG\n+\n!!\n",
    "empty": lambda r: "",
    "blank_lines": lambda r: "\n\n\n",
    "stray_then_fasta": lambda r: "junk\n>h\nACGT\n>g\nTTTT\n",
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_jf_stream_parallel_equals_sequential(tmp_path, threads, name):
    p = write(tmp_path, name, CASES[name](random.Random(name)))
    a, b = both(threads, lambda: threads.jf_stream(p))
    assert a == b


def test_jf_stream_golden_files(threads):
    for n in ("reads_a.fq", "reads_b.fq", "reads_c.fa"):
        p = os.path.join(GOLD, n)
        a, b = both(threads, lambda: threads.jf_stream(p))
        assert a == b


@pytest.mark.parametrize("names", [("fastq",), ("fastq", "fasta"), ("fasta_nanosim", "fastq_crlf"),
                                   ("fastq_empty_seqs", "fasta_nanosim", "fasta"), ("fasta_multiline",),
                                   ("fastq_no_final_newline", "fasta")])
@pytest.mark.parametrize("annotate", [False, True])
def test_load_records_parallel_equals_sequential(tmp_path, threads, names, annotate):
    paths = [write(tmp_path, f"{i}_{n}", CASES[n](random.Random(n))) for i, n in enumerate(names)]
    a, b = both(threads, lambda: threads.load_records(paths, annotate))
    same_records(a, b)


def test_load_records_golden(threads):
    paths = [os.path.join(GOLD, n) for n in ("reads_a.fq", "reads_b.fq", "reads_c.fa")]
    a, b = both(threads, lambda: threads.load_records(paths, True))
    same_records(a, b)


def test_load_records_missing_file(threads, tmp_path):
    for t in (1, 4):
        threads.set_host_threads(t)
        with pytest.raises(threads.HgaError, match="does not exist"):
            threads.load_records([str(tmp_path / "nope.fq")], True)
        with pytest.raises(threads.HgaError, match="does not exist"):
            threads.jf_stream(str(tmp_path / "nope.fq"))


def test_large_generated_fastq(tmp_path, threads):
    g = threads.gen_genome(200_000, 5)
    p = str(tmp_path / "big.fq")
    threads.write_art_fastq(g, "big", 20_000, 150, 6, p)
    a, b = both(threads, lambda: threads.jf_stream(p))
    assert a == b
    a, b = both(threads, lambda: threads.load_records([p, p], True))
    same_records(a, b)
