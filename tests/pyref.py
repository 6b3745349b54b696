"""Second, independent restatement of the reference semantics in plain Python loops.

Used only on small inputs to cross-check the C oracle (oracle/oracle.cpp).  Written from
the reference text directly, not from the oracle:
  KmerIterator            src/common/KmerIterator.cpp:7-76
  jellyfish count -C/--bc  src/occurrences/run_jellyfish.sh:3-6
  get_specificity          src/occurrences/JellyfishOccurrenceReader.cpp:88-108
  export_kmers             src/occurrences/JellyfishOccurrenceReader.cpp:110-135
  construct_indices        src/clustering/ReadClusteringEngine.cpp:234-299
"""
import bisect

FWD = {"A": 0, "C": 1, "G": 2, "T": 3}      # BASE_TO_NUM; anything else -> 0 (operator[])
RC = {"A": 3, "C": 2, "G": 1, "T": 0}       # COMPLEMENT; anything else -> 0


def kmer_iterator(seq: str, k: int):
    if k > 32:
        raise ValueError("Kmer size is too big")
    if len(seq) < k:
        return []
    mask = (1 << (2 * k)) - 1
    fwd = rc = 0
    out = []
    for i, ch in enumerate(seq):
        fwd = ((fwd << 2) | FWD.get(ch, 0)) & mask
        rc = (rc >> 2) | (RC.get(ch, 0) << (2 * (k - 1)))
        if i >= k - 1:
            out.append((min(fwd, rc), i + 1))
    return out


def canonical_string_min(s: str) -> str:
    comp = {"A": "T", "C": "G", "G": "C", "T": "A"}
    r = "".join(comp[c] for c in reversed(s))
    return min(s, r)


def encode(s: str) -> int:
    v = 0
    for c in s:
        v = (v << 2) | FWD[c]
    return v


def jf_count(stream: str, k: int, min_count: int = 2):
    counts = {}
    run = ""
    for ch in stream + "\n":
        u = ch.upper()
        if u in FWD:
            run += u
            continue
        for i in range(len(run) - k + 1):
            key = encode(canonical_string_min(run[i:i + k]))
            counts[key] = counts.get(key, 0) + 1
        run = ""
    return sorted((key, c) for key, c in counts.items() if c >= min_count)


def specificity(rows, thresholds):
    thr = sorted(set(thresholds))
    result = {t: {} for t in thr}
    for counts in rows:
        prevalent, total = max(counts), sum(counts)
        x = (prevalent / total) * 100
        t = thr[bisect.bisect_right(thr, x)]
        result[t][total] = result[t].get(total, 0) + 1
    out = []
    for ti, t in enumerate(thr):
        for total in sorted(result[t]):
            out.append((ti, total, result[t][total]))
    return out


def construct_indices(reads, k, sdk_keys_in_id_order, first_id=1):
    kmer_index = {key: i for i, key in enumerate(sdk_keys_in_id_order)}
    kci = [[] for _ in sdk_keys_in_id_order]
    per_read = []
    for r, seq in enumerate(reads):
        hits = [(kmer_index[c], p) for c, p in kmer_iterator(seq, k) if c in kmer_index]
        first = {}
        for kid, p in hits:
            kci[kid].append(first_id + r)
            first.setdefault(kid, p)
        per_read.append({"hits": hits, "sorted": sorted(kid for kid, _ in hits),
                         "first": sorted(first.items())})
    return per_read, [sorted(x) for x in kci]
