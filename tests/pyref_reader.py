"""Plain-Python restatement of SequenceRecordIterator (src/common/SequenceRecordIterator.cpp)
for small, non-empty files: one std::getline stream across the files; opening a file sniffs
its first lines (FASTQ needs a '+' third line, FASTA a '>' header) and may switch the record
layout / header parser; a record's layout is the one in force when its first line is
requested, its header parser and category the ones in force after its last line (:155-173)."""
import re

SIMLORD = re.compile(r";length=([0-9]+)bp;startpos=([0-9]+);")
NANOSIM = re.compile(r"_([0-9]+)_[^_]+_[^_]+_[^_]+_[^_]+_([0-9]+)_")
PASS = re.compile(r"([0-9]+)_([0-9]+)\|([0-9]+)\|")


def _parse(kind, h):
    m = {"simlord": SIMLORD, "nanosim": NANOSIM, "pass": PASS}.get(kind)
    m = m.search(h) if m else None
    if not m:
        return (0, 0)
    if kind == "simlord":
        return (int(m.group(2)), int(m.group(1)))
    if kind == "nanosim":
        return (int(m.group(1)), int(m.group(2)))
    return (int(m.group(3)), int(m.group(2)) - int(m.group(1)))


def getlines(data: bytes):
    if not data:
        return []
    parts = data.split(b"\n")
    if data.endswith(b"\n"):
        parts = parts[:-1]
    return [p.decode("latin-1") for p in parts]


def read_records(paths, annotate):
    files = [getlines(open(p, "rb").read()) for p in paths]
    states = []
    rec, hdr = "fastq", None
    for lines in files:
        h = lines[0] if lines else ""
        if h.startswith("@"):
            if len(lines) > 2 and lines[2].startswith("+"):
                rec = "fastq"
        elif h.startswith(">"):
            rec = "fasta"
        else:
            raise ValueError("Unrecognized file format")
        for kind in ("simlord", "nanosim", "pass"):
            if _parse(kind, h)[1] != 0:
                hdr = kind
        states.append((rec, hdr))
    lines = [(fi, ln) for fi, ls in enumerate(files) for ln in ls]
    out, i, loaded = [], 0, 0
    while True:
        need = 4 if states[loaded][0] == "fastq" else 2
        if i + need > len(lines):
            break
        chunk = lines[i:i + need]
        i += need
        loaded = chunk[-1][0]
        header = chunk[0][1][1:]
        st, ln = _parse(states[loaded][1], header)
        out.append({"id": len(out) + 1, "header": header, "seq": chunk[1][1],
                    "cat": loaded if annotate else 0, "start": st if st else 0, "end": st + ln if st else 0})
    return out
