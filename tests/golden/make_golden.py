"""Generates the committed golden fixtures under tests/golden/.

Inputs are small seeded read files plus hand-written edge-case records; expected outputs
come from the CPU oracle (oracle/oracle.cpp) and the Python reader restatement
(tests/pyref_reader.py).  The reference itself cannot be built or run here (Boost and
jellyfish are absent; see oracle/oracle.cpp), so these fixtures pin the restatement and
every later change against it — they are regression anchors, not reference outputs.

    python tests/golden/make_golden.py        # rewrites the fixtures
"""
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle  # noqa: E402
import pyref_reader  # noqa: E402

KS = [5, 15, 19, 21, 31, 32]
LOWER, UPPER = 3, 12


def genome(rng, n):
    return "".join(rng.choice("ACGT") for _ in range(n))


def mutate(rng, g, d):
    out = []
    for c in g:
        if rng.random() < d:
            out.append(rng.choice([b for b in "ACGT" if b != c]))
        else:
            out.append(c)
    return "".join(out)


def revcomp(s):
    return s.translate(str.maketrans("ACGT", "TGCA"))[::-1]


def reads(rng, g, n, length, err=0.01):
    out = []
    for _ in range(n):
        st = rng.randrange(0, len(g) - length + 1)
        r = g[st:st + length]
        if rng.random() < 0.5:
            r = revcomp(r)
        r = "".join(rng.choice("ACGT") if rng.random() < err else c for c in r)
        out.append(r)
    return out


def edge_reads():
    return ["ACGTNACGTACGTACGTACGTACGTACGTAC",      # N inside
            "acgtacgtacgtacgtacgtacgtACGTACGT",     # lower case
            "ACG",                                  # shorter than every k
            "A" * 32,                               # poly-A, len == 32
            "T" * 40,                               # poly-T (canonical poly-A)
            "GATTACA" * 6,
            "ACGTRYKMACGTACGTACGTACGTACGTACGTACGT"]  # IUPAC codes


def write_fastq(path, rs, prefix):
    with open(path, "w") as f:
        for i, r in enumerate(rs):
            f.write(f"@{prefix}-{i + 1}\n{r}\n+\n{'I' * len(r)}\n")


def write_fasta(path, rs, prefix):
    with open(path, "w") as f:
        for i, r in enumerate(rs):
            f.write(f">{prefix}_{1000 + i}_aligned_{i}_F_0_{len(r)}_0\n{r}\n")


def main():
    rng = random.Random(20261015)
    ga = genome(rng, 3000)
    gb = mutate(rng, ga, 0.03)
    ra = reads(rng, ga, 220, 70) + edge_reads()
    rb = reads(rng, gb, 200, 70) + edge_reads()[:3]
    write_fastq(os.path.join(HERE, "reads_a.fq"), ra, "hapA")
    write_fastq(os.path.join(HERE, "reads_b.fq"), rb, "hapB")
    rc = reads(rng, gb, 40, 300, err=0.05) + ["NNNNACGTACGTACGTACGTACGT", ""]
    write_fasta(os.path.join(HERE, "reads_c.fa"), rc, "hapB")

    # counting path: the jellyfish sequence stream of each file ('\n'-joined sequences)
    streams = ["\n".join(ra).encode(), "\n".join(rb).encode()]
    out = {}
    for k in KS:
        res = oracle.count_pipeline(streams, k, LOWER, UPPER)
        for f, (dk, dc) in enumerate(res["dumps"]):
            out[f"k{k}_dump{f}_keys"] = dk
            out[f"k{k}_dump{f}_counts"] = dc
        out[f"k{k}_rows_keys"] = res["keys"]
        out[f"k{k}_rows_counts"] = res["counts"]
        out[f"k{k}_hist"] = res["hist"]
        out[f"k{k}_selected"] = res["selected"]
        out[f"k{k}_n_discr"] = np.array([res["n_discr"]], np.int64)
        out[f"k{k}_instances"] = np.array([sum(oracle.count_instances(s, k) for s in streams)], np.int64)
    np.savez_compressed(os.path.join(HERE, "count_golden.npz"), **out)

    # SDK file = the k=19 export as text (jf_occurrences output format)
    k = 19
    sel = out[f"k{k}_selected"]
    B = "ACGT"
    lines = ["".join(B[(int(c) >> (2 * (k - 1 - i))) & 3] for i in range(k)) for c in sel]
    sdk_text = ("\n".join(lines) + "\n").encode()
    with open(os.path.join(HERE, "sdk_19.txt"), "wb") as f:
        f.write(sdk_text)
    sdk_keys, k2 = oracle.load_sdk_text(sdk_text)
    assert k2 == k
    lk = {"sdk_keys_id_order": sdk_keys}
    paths = [os.path.join(HERE, p) for p in ("reads_a.fq", "reads_b.fq", "reads_c.fa")]
    recs = pyref_reader.read_records(paths, True)
    bases = "".join(r["seq"] for r in recs).encode("latin-1")
    offsets = np.cumsum([0] + [len(r["seq"].encode("latin-1")) for r in recs]).astype(np.uint64)
    lk["offsets"] = offsets
    lk["category"] = np.array([r["cat"] for r in recs], np.int32)
    got = oracle.construct_indices(bases, offsets, k, sdk_keys, 1)
    for name, arr in got.items():
        lk[name] = arr
    np.savez_compressed(os.path.join(HERE, "lookup_golden.npz"), **lk)

    # KmerIterator windows of edge strings
    kw = {}
    edge = edge_reads() + ["", "N", "TNT", "aC", "ACGT\r"]
    for k in (1, 2, 5, 19, 31, 32):
        for i, s in enumerate(edge):
            c, p = oracle.kmer_windows(s.encode(), k)
            kw[f"k{k}_s{i}_codes"] = c
            kw[f"k{k}_s{i}_pos"] = p
    np.savez_compressed(os.path.join(HERE, "windows_golden.npz"), **kw)
    with open(os.path.join(HERE, "windows_inputs.txt"), "w") as f:
        f.write("\n".join(edge) + "\n")
    print("golden fixtures written")


if __name__ == "__main__":
    main()
