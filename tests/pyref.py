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


# --- HyperLogLog auto-k: src/lib/MurmurHash3.cpp:94-140, src/lib/HyperLogLog.hpp:96-132,
#     src/occurrences/KmerAnalysis.cpp:15-56
def murmur3_x86_32(data: bytes, seed: int) -> int:
    M = 0xFFFFFFFF
    rotl = lambda x, r: ((x << r) | (x >> (32 - r))) & M
    h = seed & M
    n = len(data) // 4
    for i in range(n):
        k1 = int.from_bytes(data[4 * i:4 * i + 4], "little")
        k1 = rotl((k1 * 0xcc9e2d51) & M, 15) * 0x1b873593 & M
        h = (rotl(h ^ k1, 13) * 5 + 0xe6546b64) & M
    tail = data[4 * n:]
    k1 = 0
    for j in reversed(range(len(tail))):
        k1 ^= tail[j] << (8 * j)
    if tail:
        k1 = rotl((k1 * 0xcc9e2d51) & M, 15) * 0x1b873593 & M
        h ^= k1
    h ^= len(data)
    h ^= h >> 16
    h = (h * 0x85ebca6b) & M
    h ^= h >> 13
    h = (h * 0xc2b2ae35) & M
    return h ^ (h >> 16)


def hll_registers(reads, k: int, b: int = 10):
    regs = [0] * (1 << b)
    for seq in reads:
        for code, _ in kmer_iterator(seq, k):
            h = murmur3_x86_32(code.to_bytes(8, "little"), 313)
            x = (h << b) & 0xFFFFFFFF
            clz = 32 - x.bit_length()          # clz(0) = 32
            rank = min(32 - b, clz) + 1
            idx = h >> (32 - b)
            regs[idx] = max(regs[idx], rank)
    return regs


def hll_estimate(regs, b: int = 10) -> float:
    import math
    m = 1 << b
    alpha = {16: 0.673, 32: 0.697, 64: 0.709}.get(m, 0.7213 / (1.0 + 1.079 / m))
    e = alpha * m * m / sum(1.0 / (1 << r) for r in regs)
    if e <= 2.5 * m:
        z = regs.count(0)
        if z:
            e = m * math.log(m / z)
    elif e > (1.0 / 30.0) * 4294967296.0:
        e = -4294967296.0 * math.log(1.0 - e / 4294967296.0)
    return e
