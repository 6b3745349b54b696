"""Copies the reference's own C1 inputs (data files, not source) into this fixture directory.

BASELINE.json configs[0] is "jf_occurrences -k 19 on ART 30x reads of a 500 kb random sequence";
the reference ships exactly that random pair as data/sequences/artificial_size=500000_{A,B}.fasta
(a 60-column multi-line FASTA each).  They are stored gzip-compressed, byte-identical after
decompression; /root/reference is read only in this container (the GPU box never sees it).
"""
import gzip
import os
import shutil

SRC = "/root/reference/data/sequences"
HERE = os.path.dirname(os.path.abspath(__file__))

if __name__ == "__main__":
    for h in "AB":
        name = f"artificial_size=500000_{h}.fasta"
        with open(os.path.join(SRC, name), "rb") as fi, gzip.GzipFile(os.path.join(HERE, name + ".gz"), "wb",
                                                                        mtime=0) as fo:
            shutil.copyfileobj(fi, fo)
