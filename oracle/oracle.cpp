// oracle/oracle.cpp — CPU restatement of the reference hot path.
//
// TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load this library, and only as the checker / the timed CPU
// baseline.  The product (libhga.so, the CLIs) never links or calls it.
//
// PARITY STATUS: "parity unpinned" in the strict sense of the task rules.  The
// reference has no tests, fixtures or golden vectors for this path,
// and it cannot be compiled here without stand-ins: every translation unit on the
// path includes Boost headers (common/KmerIterator.h:3 <boost/optional.hpp>,
// occurrences/JellyfishOccurrenceReader.h:7 <boost/function.hpp>,
// common/SequenceRecordIterator.h:9 <boost/regex.hpp>) and Boost is not installed.
// The counting stage itself is the external `jellyfish` binary, which is absent.
// Each function below cites the reference lines it restates; hand-derived
// known-answer tests (tests/test_oracle_kat.py) check the restatement.
//
// Written as plain, obviously-correct code (std::unordered_map, std::map,
// std::sort).  The multi-threaded *_mt variants exist for bench.py's cpu_baseline
// and are checked against the plain ones in tests/test_oracle.py.

#include <cmath>
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <memory>
#include <vector>

namespace {

// src/common/KmerIterator.cpp:7-19.  BASE_TO_NUM / COMPLEMENT are
// std::unordered_map<char,Kmer> read with operator[]: any byte that is not one of
// the four upper-case bases default-inserts 0, so it contributes code 0 to BOTH the
// forward and the reverse-complement register.
inline uint64_t ref_fwd_code(char c) {
    switch (c) {
        case 'A': return 0; case 'C': return 1; case 'G': return 2; case 'T': return 3;
        default: return 0;
    }
}
inline uint64_t ref_rc_code(char c) {
    switch (c) {
        case 'A': return 3; case 'C': return 2; case 'G': return 1; case 'T': return 0;
        default: return 0;
    }
}

// Jellyfish counting semantics (src/occurrences/run_jellyfish.sh:3-6, `-C`):
// bases are ACGT case-insensitively; any other byte ends the current k-mer run.
inline int jf_code(unsigned char c) {
    switch (c) {
        case 'A': case 'a': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': return 3;
        default: return -1;
    }
}

inline uint64_t kmask(int k) { return k >= 32 ? ~0ull : ((1ull << (2 * k)) - 1); }

// Canonical k-mers of every window of every ACGT run of a byte stream, in order.
template <class F>
void for_each_jf_kmer(const char* s, uint64_t n, int k, F&& f) {
    const uint64_t mask = kmask(k);
    const int sh = 2 * (k - 1);
    uint64_t fwd = 0, rc = 0;
    int run = 0;
    for (uint64_t i = 0; i < n; ++i) {
        int c = jf_code((unsigned char)s[i]);
        if (c < 0) { run = 0; fwd = rc = 0; continue; }
        fwd = ((fwd << 2) | (uint64_t)c) & mask;
        rc = (rc >> 2) | ((uint64_t)(3 - c) << sh);
        if (++run >= k) f(fwd < rc ? fwd : rc, i);
    }
}

struct Buf { void* p; };

template <class T>
T* dup_vec(const std::vector<T>& v) {
    T* p = (T*)std::malloc(std::max<size_t>(1, v.size() * sizeof(T)));
    if (!v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
    return p;
}

}  // namespace

extern "C" {

void or_free(void* p) { std::free(p); }

// --- A1/A2: KmerIterator (src/common/KmerIterator.cpp:23-76) ------------------------
// Writes the canonical k-mer and the end-exclusive position_in_sequence of every
// window of `seq`.  Returns the number of windows: 0 when len < k
// (KmerIterator.cpp:33-34), len-k+1 otherwise; -1 when k > 32 (KmerIterator.cpp:24-26)
// or k < 1.  Output pointers may be null (count only).
int64_t or_kmer_windows(const char* seq, uint64_t len, int k, uint64_t* out_kmer,
                        uint32_t* out_pos) {
    if (k > 32 || k < 1) return -1;
    if (len < (uint64_t)k) return 0;
    const uint64_t mask = kmask(k);             // KmerIterator.cpp:30 clearing_mask
    const int sh = 2 * (k - 1);                 // KmerIterator.cpp:31 complement_shift_by
    uint64_t fwd = 0, rc = 0;
    int64_t w = 0;
    for (uint64_t i = 0; i < len; ++i) {
        fwd = ((fwd << 2) | ref_fwd_code(seq[i])) & mask;   // roll_forward_strand :54-58
        rc = (rc >> 2) | (ref_rc_code(seq[i]) << sh);       // roll_complementary_strand :60-63
        if (i + 1 >= (uint64_t)k) {                         // next_kmer :65-76
            if (out_kmer) out_kmer[w] = fwd < rc ? fwd : rc;
            if (out_pos) out_pos[w] = (uint32_t)(i + 1);
            ++w;
        }
    }
    return w;
}

// --- A3: jellyfish count of one read file (run_jellyfish.sh:3-6) -------------------
// `s` is the file's sequences joined by any non-ACGT separator byte.  Exact count of
// canonical k-mers, k-mers with count < min_count dropped (`--bc` drops singletons),
// output ascending by 2-bit code == LC_ALL=C order of the dump (run_jellyfish.sh:6).
// Returns the number of (key,count) rows; *keys/*counts are malloc'ed (or_free).
int64_t or_count_stream(const char* s, uint64_t n, int k, uint32_t min_count,
                        uint64_t** keys, uint32_t** counts) {
    if (k > 32 || k < 1) return -1;
    std::unordered_map<uint64_t, uint32_t> m;
    for_each_jf_kmer(s, n, k, [&](uint64_t c, uint64_t) { ++m[c]; });
    std::vector<std::pair<uint64_t, uint32_t>> v;
    v.reserve(m.size());
    for (auto& kv : m)
        if (kv.second >= min_count) v.push_back(kv);
    std::sort(v.begin(), v.end());
    std::vector<uint64_t> ks(v.size());
    std::vector<uint32_t> cs(v.size());
    for (size_t i = 0; i < v.size(); ++i) { ks[i] = v[i].first; cs[i] = v[i].second; }
    *keys = dup_vec(ks);
    *counts = dup_vec(cs);
    return (int64_t)v.size();
}

// Number of k-mer windows the jellyfish semantics count in a stream.
uint64_t or_count_instances(const char* s, uint64_t n, int k) {
    uint64_t c = 0;
    for_each_jf_kmer(s, n, k, [&](uint64_t, uint64_t) { ++c; });
    return c;
}

// Multi-threaded exact count (cpu_baseline leg).  Threads take contiguous slices of
// the stream (cut at separator bytes so no window is split), count into private
// hash maps partitioned by key hash, then each partition is merged by one thread.
int64_t or_count_stream_mt(const char* s, uint64_t n, int k, uint32_t min_count,
                           int threads, uint64_t** keys, uint32_t** counts) {
    if (k > 32 || k < 1) return -1;
    if (threads < 1) threads = 1;
    const int P = threads;
    std::vector<uint64_t> cut(threads + 1, 0);
    cut[threads] = n;
    for (int t = 1; t < threads; ++t) {
        uint64_t c = n * (uint64_t)t / threads;
        if (c < cut[t - 1]) c = cut[t - 1];
        while (c < n && jf_code((unsigned char)s[c]) >= 0) ++c;
        cut[t] = c;
    }
    auto part_of = [P](uint64_t key) {
        uint64_t h = key * 0x9E3779B97F4A7C15ull;
        return (int)((h >> 40) % (uint64_t)P);
    };
    std::vector<std::vector<std::unordered_map<uint64_t, uint32_t>>> local(
        threads, std::vector<std::unordered_map<uint64_t, uint32_t>>(P));
    {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t] {
                auto& L = local[t];
                for_each_jf_kmer(s + cut[t], cut[t + 1] - cut[t], k,
                                 [&](uint64_t c, uint64_t) { ++L[part_of(c)][c]; });
            });
        for (auto& x : th) x.join();
    }
    std::vector<std::vector<std::pair<uint64_t, uint32_t>>> out(P);
    {
        std::vector<std::thread> th;
        for (int p = 0; p < P; ++p)
            th.emplace_back([&, p] {
                std::unordered_map<uint64_t, uint32_t> m;
                for (int t = 0; t < threads; ++t)
                    for (auto& kv : local[t][p]) m[kv.first] += kv.second;
                for (int t = 0; t < threads; ++t) std::unordered_map<uint64_t, uint32_t>().swap(local[t][p]);
                auto& o = out[p];
                for (auto& kv : m)
                    if (kv.second >= min_count) o.push_back(kv);
                std::sort(o.begin(), o.end());
            });
        for (auto& x : th) x.join();
    }
    // k-way merge of the P sorted partitions
    size_t total = 0;
    for (auto& o : out) total += o.size();
    std::vector<uint64_t> ks;
    std::vector<uint32_t> cs;
    ks.reserve(total);
    cs.reserve(total);
    std::vector<size_t> idx(P, 0);
    using QE = std::pair<uint64_t, int>;
    std::vector<QE> heap;
    for (int p = 0; p < P; ++p)
        if (!out[p].empty()) heap.push_back({out[p][0].first, p});
    auto cmp = [](const QE& a, const QE& b) { return a.first > b.first; };
    std::make_heap(heap.begin(), heap.end(), cmp);
    while (!heap.empty()) {
        std::pop_heap(heap.begin(), heap.end(), cmp);
        int p = heap.back().second;
        heap.pop_back();
        ks.push_back(out[p][idx[p]].first);
        cs.push_back(out[p][idx[p]].second);
        if (++idx[p] < out[p].size()) {
            heap.push_back({out[p][idx[p]].first, p});
            std::push_heap(heap.begin(), heap.end(), cmp);
        }
    }
    *keys = dup_vec(ks);
    *counts = dup_vec(cs);
    return (int64_t)ks.size();
}

// --- A3 + A4, multi-threaded over all files: merged rows of the whole count stage ----------
// The same result as or_count_stream per file followed by or_merge, computed by range
// partitioning (so no heap merge is needed): threads extract every canonical k-mer of their
// slice of a file (cut at separator bytes) and count them per code-range partition; a prefix sum
// gives every (partition, thread) its place in one array per file, and a second extraction pass
// scatters the codes there (no per-thread bins: threads x partitions vectors did not scale to 256
// threads).  Then, one partition at a time (threads take partitions from a shared counter), each
// file's codes are sorted and run-length counted (count < min_count dropped: `--bc`,
// run_jellyfish.sh:3-6) and the F sorted per-file lists are merged into rows (counts[f] = 0 where
// file f lacks the k-mer, JellyfishOccurrenceReader.cpp:63-86).  Partitions are ascending code
// ranges, so their rows concatenate in ascending order.  Output: keys[rows], counts[rows * F]
// row-major.
int64_t or_count_files_mt(int F, const char* const* s, const uint64_t* n, int k, uint32_t min_count,
                          int threads, uint64_t** keys, uint32_t** counts) {
    if (k > 32 || k < 1 || F < 1) return -1;
    if (threads < 1) threads = 1;
    const int nb = 2 * k;
    const int tb = nb < 16 ? nb : 16;              // top bits that pick the partition
    const int P = nb <= 8 ? 1 : (nb <= 12 ? 64 : 4096);
    // canonical = min(fwd, rc) of uniform codes has mass 1 - (1 - x)^2 below x: equal-mass
    // ranges, aligned to the top tb bits (any ascending ranges give the same rows)
    std::vector<uint16_t> part_of(1u << tb);
    for (uint32_t t = 0; t < (1u << tb); ++t) {
        const double x = (double)t / (double)(1u << tb);
        const int p = (int)((1.0 - (1.0 - x) * (1.0 - x)) * P);
        part_of[t] = (uint16_t)std::min(p, P - 1);
    }
    const int shift = nb - tb;
    // codes[f]: file f's codes grouped by partition; start[f][p] = partition p's first
    std::vector<std::unique_ptr<uint64_t[]>> codes(F);
    std::vector<std::vector<uint64_t>> start(F, std::vector<uint64_t>(P + 1, 0));
    for (int f = 0; f < F; ++f) {
        std::vector<uint64_t> cut(threads + 1, 0);
        cut[threads] = n[f];
        for (int t = 1; t < threads; ++t) {
            uint64_t c = n[f] * (uint64_t)t / threads;
            if (c < cut[t - 1]) c = cut[t - 1];
            while (c < n[f] && jf_code((unsigned char)s[f][c]) >= 0) ++c;
            cut[t] = c;
        }
        std::vector<uint64_t> cnt((size_t)threads * P, 0);   // [t][p]
        {
            std::vector<std::thread> th;
            for (int t = 0; t < threads; ++t)
                th.emplace_back([&, f, t] {
                    uint64_t* C = cnt.data() + (size_t)t * P;
                    for_each_jf_kmer(s[f] + cut[t], cut[t + 1] - cut[t], k,
                                     [&](uint64_t c, uint64_t) { ++C[part_of[c >> shift]]; });
                });
            for (auto& x : th) x.join();
        }
        uint64_t run = 0;   // partition-major, threads in order
        for (int p = 0; p < P; ++p) {
            start[f][p] = run;
            for (int t = 0; t < threads; ++t) {
                const uint64_t c = cnt[(size_t)t * P + p];
                cnt[(size_t)t * P + p] = run;
                run += c;
            }
        }
        start[f][P] = run;
        codes[f].reset(new uint64_t[std::max<uint64_t>(run, 1)]);
        uint64_t* out = codes[f].get();
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, f, t] {
                uint64_t* O = cnt.data() + (size_t)t * P;
                for_each_jf_kmer(s[f] + cut[t], cut[t + 1] - cut[t], k,
                                 [&](uint64_t c, uint64_t) { out[O[part_of[c >> shift]]++] = c; });
            });
        for (auto& x : th) x.join();
    }
    std::vector<std::vector<uint64_t>> pk(P);
    std::vector<std::vector<uint32_t>> pc(P);
    std::atomic<int> next{0};
    {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&] {
                std::vector<std::vector<std::pair<uint64_t, uint32_t>>> runs(F);
                for (int p; (p = next.fetch_add(1)) < P;) {
                    for (int f = 0; f < F; ++f) {
                        uint64_t* v = codes[f].get() + start[f][p];
                        const size_t m = start[f][p + 1] - start[f][p];
                        std::sort(v, v + m);
                        auto& r = runs[f];
                        r.clear();
                        for (size_t i = 0; i < m;) {
                            size_t j = i + 1;
                            while (j < m && v[j] == v[i]) ++j;
                            if (j - i >= min_count) r.push_back({v[i], (uint32_t)(j - i)});
                            i = j;
                        }
                    }
                    std::vector<size_t> idx(F, 0);
                    auto& K = pk[p];
                    auto& C = pc[p];
                    while (true) {
                        uint64_t m = ~0ull;
                        bool any = false;
                        for (int f = 0; f < F; ++f)
                            if (idx[f] < runs[f].size()) {
                                m = std::min(m, runs[f][idx[f]].first);
                                any = true;
                            }
                        if (!any) break;
                        K.push_back(m);
                        for (int f = 0; f < F; ++f) {
                            uint32_t c = 0;
                            if (idx[f] < runs[f].size() && runs[f][idx[f]].first == m) c = runs[f][idx[f]++].second;
                            C.push_back(c);
                        }
                    }
                }
            });
        for (auto& x : th) x.join();
    }
    codes.clear();
    size_t total = 0;
    for (auto& x : pk) total += x.size();
    uint64_t* ok = (uint64_t*)std::malloc(std::max<size_t>(1, total * 8));
    uint32_t* oc = (uint32_t*)std::malloc(std::max<size_t>(1, total * 4 * F));
    size_t o = 0;
    for (int p = 0; p < P; ++p) {
        if (!pk[p].empty()) {
            std::memcpy(ok + o, pk[p].data(), pk[p].size() * 8);
            std::memcpy(oc + o * F, pc[p].data(), pc[p].size() * 4);
        }
        o += pk[p].size();
    }
    *keys = ok;
    *counts = oc;
    return (int64_t)total;
}

// Reference-like single-thread count (cpu_baseline "reference_like" figure):
// per read (the stream split at '\n'), the reference's KmerIterator inner loop with its
// std::unordered_map<char, Kmer> BASE_TO_NUM / COMPLEMENT lookups (KmerIterator.cpp:7-19, 54-63;
// operator[] as in the reference), counted into a std::unordered_map, then the per-file drop and
// the sort of the dump.  For ACGT-only reads (the synthetic ones) the rows equal
// or_count_stream's; returns the number of rows.
int64_t or_count_reference_like(const char* s, uint64_t n, int k, uint32_t min_count) {
    if (k > 32 || k < 1) return -1;
    static std::unordered_map<char, uint64_t> base_to_num = {{'A', 0}, {'C', 1}, {'G', 2}, {'T', 3}};
    static std::unordered_map<char, uint64_t> complement = {{'A', 3}, {'C', 2}, {'G', 1}, {'T', 0}};
    const uint64_t mask = kmask(k);
    const int sh = 2 * (k - 1);
    std::unordered_map<uint64_t, uint32_t> m;
    uint64_t i = 0;
    while (i < n) {
        uint64_t j = i;
        while (j < n && s[j] != '\n') ++j;
        const std::string read(s + i, s + j);   // GenomeReadData::sequence
        if (read.size() >= (uint64_t)k) {
            uint64_t fwd = 0, rc = 0;
            for (size_t p = 0; p < read.size(); ++p) {
                fwd = ((fwd << 2) | base_to_num[read[p]]) & mask;
                rc = (rc >> 2) | (complement[read[p]] << sh);
                if (p + 1 >= (size_t)k) ++m[fwd < rc ? fwd : rc];
            }
        }
        i = j + 1;
    }
    std::vector<std::pair<uint64_t, uint32_t>> v;
    for (auto& kv : m)
        if (kv.second >= min_count) v.push_back(kv);
    std::sort(v.begin(), v.end());
    return (int64_t)v.size();
}

// --- A4: k-way merge of the per-file sorted dumps -------------------------------------
// JellyfishOccurrenceReader::get_next_kmer (JellyfishOccurrenceReader.cpp:63-86): one
// merged row per distinct k-mer, counts[f] = 0 where file f's dump lacks it.
// For a fixed k the string order of the dump lines equals ascending 2-bit code.
// Inputs: F sorted key arrays with counts.  Output: merged keys (ascending) and a
// row-major [rows][F] count matrix.  Returns rows.
int64_t or_merge(int F, const uint64_t* const* keys, const uint32_t* const* counts,
                 const uint64_t* lens, uint64_t** out_keys, uint32_t** out_counts) {
    std::map<uint64_t, std::vector<uint32_t>> m;
    for (int f = 0; f < F; ++f)
        for (uint64_t i = 0; i < lens[f]; ++i) {
            auto it = m.find(keys[f][i]);
            if (it == m.end()) it = m.emplace(keys[f][i], std::vector<uint32_t>(F, 0)).first;
            it->second[f] = counts[f][i];
        }
    std::vector<uint64_t> ks;
    std::vector<uint32_t> cs;
    ks.reserve(m.size());
    cs.reserve(m.size() * F);
    for (auto& kv : m) {
        ks.push_back(kv.first);
        for (int f = 0; f < F; ++f) cs.push_back(kv.second[f]);
    }
    *out_keys = dup_vec(ks);
    *out_counts = dup_vec(cs);
    return (int64_t)ks.size();
}

// --- A5: get_specificity (JellyfishOccurrenceReader.cpp:88-108) ----------------------
// For every merged row: total = Σcounts, prevalent = max counts,
// spec = *thresholds.upper_bound(((double)prevalent / (double)total) * 100)
// and result[spec][total] += 1.  Output: flattened (threshold_index, total, n) triples
// in std::map order (threshold ascending, total ascending).  Returns the triple count;
// *out is malloc'ed [3*count] int64.  (upper_bound past the largest threshold is
// undefined in the reference; it cannot happen with the CLI's 100.01 sentinel.)
int64_t or_specificity(int F, uint64_t rows, const uint32_t* counts, const double* thr,
                       int n_thr, int64_t** out) {
    std::set<double> T(thr, thr + n_thr);
    std::vector<double> tv(T.begin(), T.end());
    std::map<double, std::map<int, int>> result;
    for (double t : tv) result.insert({t, {}});
    for (uint64_t r = 0; r < rows; ++r) {
        int prevalent = 0, total = 0;
        for (int f = 0; f < F; ++f) {
            int c = (int)counts[r * F + f];
            prevalent = std::max(c, prevalent);
            total += c;
        }
        auto it = T.upper_bound(((double)prevalent / (double)total) * 100);
        if (it == T.end()) return -1;
        result[*it].insert(std::pair<int, int>(total, 0)).first->second += 1;
    }
    std::vector<int64_t> v;
    for (auto& tk : result) {
        int ti = (int)(std::lower_bound(tv.begin(), tv.end(), tk.first) - tv.begin());
        for (auto& oc : tk.second) {
            v.push_back(ti);
            v.push_back(oc.first);
            v.push_back(oc.second);
        }
    }
    *out = dup_vec(v);
    return (int64_t)(v.size() / 3);
}

// --- A7: export_kmers selection (JellyfishOccurrenceReader.cpp:110-135) -------------
// Deterministic part (percent >= 1): every merged row with lower <= total <= upper is
// exported in merge order; `discriminative` counts exported rows with exactly one
// nonzero file count (:128-130).  Returns the number exported; keys malloc'ed.
int64_t or_select(int F, uint64_t rows, const uint64_t* keys, const uint32_t* counts,
                  int64_t lower, int64_t upper, uint64_t** out_keys, uint64_t* n_discr) {
    std::vector<uint64_t> ks;
    uint64_t d = 0;
    for (uint64_t r = 0; r < rows; ++r) {
        int64_t total = 0;
        int nz = 0;
        for (int f = 0; f < F; ++f) {
            total += counts[r * F + f];
            nz += counts[r * F + f] > 0;
        }
        if (lower <= total && total <= upper) {
            ks.push_back(keys[r]);
            if (nz == 1) ++d;
        }
    }
    *n_discr = d;
    *out_keys = dup_vec(ks);
    return (int64_t)ks.size();
}

// --- A8: load_text_file_kmers (src/read_clustering.cpp:18-33) ------------------------
// Per line (std::getline, so no trailing-newline line): k = line length, the line's
// canonical code via KmerIterator, inserted into a std::unordered_set<uint64_t>.
// KmerIDs are the set's iteration order (ReadClusteringEngine.cpp:237-241), so the
// output is the keys in that order.  *k_out = the last line's length.  Returns the
// number of keys, -1 if a line is longer than 32 (KmerIterator throws).
int64_t or_load_sdk_text(const char* text, uint64_t n, uint64_t** keys_in_id_order,
                         int* k_out) {
    std::unordered_set<uint64_t> s;
    int k = 0;
    uint64_t i = 0;
    while (i < n) {
        uint64_t j = i;
        while (j < n && text[j] != '\n') ++j;
        const char* line = text + i;
        uint64_t len = j - i;
        k = (int)len;
        if (k > 32) return -1;
        uint64_t code = 0;  // current_kmer stays 0 when next_kmer() returns false
        if (k >= 1) or_kmer_windows(line, len, k, &code, nullptr);
        s.insert(code);
        i = j + 1;
    }
    std::vector<uint64_t> v(s.begin(), s.end());
    *keys_in_id_order = dup_vec(v);
    *k_out = k;
    return (int64_t)v.size();
}

// --- A9: construct_indices (src/clustering/ReadClusteringEngine.cpp:234-299) ---------
// Reads are given as a CSR (bases, offsets[n+1]) in reader order; read_ids[i] is the
// reader's 1-based ReadID.  SDK keys are given in KmerID order.
// Outputs (all malloc'ed, or_free):
//  hit_ptr[n+1], hit_kid[H], hit_pos[H]  - per read, every window whose canonical code
//        is in the set, in window order (:248-254), with the end-exclusive position;
//  sorted_kid[H]                         - per read, the KmerIDs sorted ascending with
//        duplicates (ReadComponent::discriminative_kmer_ids, :262-272);
//  first_ptr[n+1], first_kid[U], first_pos[U] - per read, kmer_positions (:267):
//        the FIRST position of each distinct KmerID, listed by ascending KmerID;
//  kci_ptr[K+1], kci_read[H]             - kmer_component_index: per KmerID the
//        ReadIDs (one per occurrence) sorted ascending (:262-263, 282-284).
// Returns H.
int64_t or_construct_indices(const char* bases, const uint64_t* offsets, uint64_t n,
                             const uint32_t* read_ids, int k, const uint64_t* sdk_keys,
                             uint32_t n_sdk, uint64_t** hit_ptr, uint32_t** hit_kid,
                             uint32_t** hit_pos, uint32_t** sorted_kid, uint64_t** first_ptr,
                             uint32_t** first_kid, uint32_t** first_pos, uint64_t** kci_ptr,
                             uint32_t** kci_read, uint64_t* n_first) {
    if (k > 32 || k < 1) return -1;
    std::unordered_map<uint64_t, uint32_t> kmer_index;  // KmerIndex, :237-241
    for (uint32_t i = 0; i < n_sdk; ++i) kmer_index[sdk_keys[i]] = i;
    std::vector<std::vector<uint32_t>> kci(n_sdk);
    std::vector<uint64_t> hp(n + 1, 0), fp(n + 1, 0);
    std::vector<uint32_t> hk, hpos, sk, fk, fpos;
    std::vector<uint64_t> wk;
    std::vector<uint32_t> wp;
    for (uint64_t r = 0; r < n; ++r) {
        uint64_t len = offsets[r + 1] - offsets[r];
        wk.resize(len + 1);
        wp.resize(len + 1);
        int64_t w = or_kmer_windows(bases + offsets[r], len, k, wk.data(), wp.data());
        std::vector<uint32_t> ids;
        std::map<uint32_t, uint32_t> firstpos;  // robin_map insert: first wins
        for (int64_t i = 0; i < w; ++i) {
            auto it = kmer_index.find(wk[i]);
            if (it == kmer_index.end()) continue;
            hk.push_back(it->second);
            hpos.push_back(wp[i]);
            ids.push_back(it->second);
            kci[it->second].push_back(read_ids[r]);
            firstpos.insert({it->second, wp[i]});
        }
        std::sort(ids.begin(), ids.end());
        sk.insert(sk.end(), ids.begin(), ids.end());
        for (auto& kv : firstpos) {
            fk.push_back(kv.first);
            fpos.push_back(kv.second);
        }
        hp[r + 1] = hk.size();
        fp[r + 1] = fk.size();
    }
    std::vector<uint64_t> kp(n_sdk + 1, 0);
    std::vector<uint32_t> kr;
    for (uint32_t i = 0; i < n_sdk; ++i) {
        std::sort(kci[i].begin(), kci[i].end());
        kr.insert(kr.end(), kci[i].begin(), kci[i].end());
        kp[i + 1] = kr.size();
    }
    *hit_ptr = dup_vec(hp);
    *hit_kid = dup_vec(hk);
    *hit_pos = dup_vec(hpos);
    *sorted_kid = dup_vec(sk);
    *first_ptr = dup_vec(fp);
    *first_kid = dup_vec(fk);
    *first_pos = dup_vec(fpos);
    *kci_ptr = dup_vec(kp);
    *kci_read = dup_vec(kr);
    *n_first = fk.size();
    return (int64_t)hk.size();
}

// Multi-threaded construct_indices with exactly or_construct_indices' outputs: threads take
// contiguous read ranges (so per-thread hit lists concatenate in read order), each with the
// same per-read steps; kmer_component_index lists are concatenated in thread order and sorted
// per KmerID (:282-284).  For the C3-size parity test and the lookup cpu_baseline leg.
int64_t or_construct_indices_mt(const char* bases, const uint64_t* offsets, uint64_t n,
                                const uint32_t* read_ids, int k, const uint64_t* sdk_keys,
                                uint32_t n_sdk, int threads, uint64_t** hit_ptr, uint32_t** hit_kid,
                                uint32_t** hit_pos, uint32_t** sorted_kid, uint64_t** first_ptr,
                                uint32_t** first_kid, uint32_t** first_pos, uint64_t** kci_ptr,
                                uint32_t** kci_read, uint64_t* n_first) {
    if (k > 32 || k < 1) return -1;
    if (threads < 1) threads = 1;
    std::unordered_map<uint64_t, uint32_t> kmer_index;  // KmerIndex, :237-241
    kmer_index.reserve(n_sdk * 2);
    for (uint32_t i = 0; i < n_sdk; ++i) kmer_index[sdk_keys[i]] = i;
    struct Part {
        std::vector<uint32_t> hk, hpos, sk, fk, fpos;
        std::vector<uint64_t> hcnt, fcnt;   // per read of the range
        std::vector<std::pair<uint32_t, uint32_t>> kci;   // (KmerID, ReadID) in hit order
    };
    std::vector<Part> parts(threads);
    std::vector<uint64_t> r0(threads + 1);
    for (int t = 0; t <= threads; ++t) r0[t] = n * (uint64_t)t / threads;
    {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t] {
                Part& P = parts[t];
                std::vector<uint64_t> wk;
                std::vector<uint32_t> wp, ids;
                std::vector<std::pair<uint32_t, uint32_t>> fp;
                for (uint64_t r = r0[t]; r < r0[t + 1]; ++r) {
                    const uint64_t len = offsets[r + 1] - offsets[r];
                    wk.resize(len + 1);
                    wp.resize(len + 1);
                    const int64_t w = or_kmer_windows(bases + offsets[r], len, k, wk.data(), wp.data());
                    ids.clear();
                    fp.clear();
                    for (int64_t i = 0; i < w; ++i) {
                        auto it = kmer_index.find(wk[i]);
                        if (it == kmer_index.end()) continue;
                        P.hk.push_back(it->second);
                        P.hpos.push_back(wp[i]);
                        ids.push_back(it->second);
                        P.kci.push_back({it->second, read_ids[r]});
                        fp.push_back({it->second, wp[i]});
                    }
                    std::sort(ids.begin(), ids.end());
                    P.sk.insert(P.sk.end(), ids.begin(), ids.end());
                    // first occurrence per KmerID (positions ascend in window order: stable sort)
                    std::stable_sort(fp.begin(), fp.end(),
                                     [](const auto& a, const auto& b) { return a.first < b.first; });
                    uint64_t nf = 0;
                    for (size_t i = 0; i < fp.size(); ++i)
                        if (i == 0 || fp[i].first != fp[i - 1].first) {
                            P.fk.push_back(fp[i].first);
                            P.fpos.push_back(fp[i].second);
                            ++nf;
                        }
                    P.hcnt.push_back(ids.size());
                    P.fcnt.push_back(nf);
                }
            });
        for (auto& x : th) x.join();
    }
    std::vector<uint64_t> hp(n + 1, 0), fpp(n + 1, 0);
    std::vector<uint32_t> hk, hpos, sk, fk, fpos;
    for (int t = 0; t < threads; ++t) {
        const Part& P = parts[t];
        for (uint64_t i = 0; i < P.hcnt.size(); ++i) {
            const uint64_t r = r0[t] + i;
            hp[r + 1] = hp[r] + P.hcnt[i];
            fpp[r + 1] = fpp[r] + P.fcnt[i];
        }
        hk.insert(hk.end(), P.hk.begin(), P.hk.end());
        hpos.insert(hpos.end(), P.hpos.begin(), P.hpos.end());
        sk.insert(sk.end(), P.sk.begin(), P.sk.end());
        fk.insert(fk.end(), P.fk.begin(), P.fk.end());
        fpos.insert(fpos.end(), P.fpos.begin(), P.fpos.end());
    }
    // kmer_component_index: counting sort by KmerID, then each list sorted
    std::vector<uint64_t> kp(n_sdk + 1, 0);
    for (auto& P : parts)
        for (auto& e : P.kci) ++kp[e.first + 1];
    for (uint32_t i = 0; i < n_sdk; ++i) kp[i + 1] += kp[i];
    std::vector<uint32_t> kr(kp[n_sdk]);
    {
        std::vector<uint64_t> cur(kp.begin(), kp.end() - 1);
        for (auto& P : parts)
            for (auto& e : P.kci) kr[cur[e.first]++] = e.second;
    }
    {
        std::atomic<uint32_t> next{0};
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&] {
                for (uint32_t b; (b = next.fetch_add(4096)) < n_sdk;)
                    for (uint32_t i = b; i < std::min<uint32_t>(n_sdk, b + 4096); ++i)
                        std::sort(kr.begin() + kp[i], kr.begin() + kp[i + 1]);
            });
        for (auto& x : th) x.join();
    }
    *hit_ptr = dup_vec(hp);
    *hit_kid = dup_vec(hk);
    *hit_pos = dup_vec(hpos);
    *sorted_kid = dup_vec(sk);
    *first_ptr = dup_vec(fpp);
    *first_kid = dup_vec(fk);
    *first_pos = dup_vec(fpos);
    *kci_ptr = dup_vec(kp);
    *kci_read = dup_vec(kr);
    *n_first = fk.size();
    return (int64_t)hk.size();
}

// get_connections (src/clustering/ReadClusteringEngine.cpp:301-333) on the state that
// construct_indices leaves: component r = read r (ReadID read_ids[r]) with
// discriminative_kmer_ids = its sorted KmerIDs with duplicates, kmer_component_index =
// kci_ptr/kci_read (ReadIDs).  Per pivot: count every candidate over the KmerID lists
// (:311-315, robin_map -> unordered_map), erase the pivot (:316), keep count >= min_score
// (:318-325); is_good = equal categories when given (debug, :319).  pivots == nullptr means
// every read with >= min_kmers hits (get_all_connections :335-339 for min_kmers = 1, the
// filter_components call site :750-751 otherwise); an explicit pivot list is also filtered by
// min_kmers.  Order: score descending (:331), ties by (x, y) ascending (unordered in the
// reference).  Returns the number of connections; arrays malloc'ed.
int64_t or_connections(uint64_t n, const uint64_t* hit_ptr, const uint32_t* sorted_kid,
                       const uint64_t* kci_ptr, const uint32_t* kci_read, const uint32_t* read_ids,
                       const uint32_t* pivots, uint64_t n_piv, uint32_t min_kmers, uint64_t min_score,
                       const int32_t* categories, uint32_t** ox, uint32_t** oy, uint64_t** os,
                       uint8_t** og) {
    std::unordered_map<uint32_t, uint64_t> row_of;   // ReadID -> read index (component_index)
    for (uint64_t r = 0; r < n; ++r)
        if (hit_ptr[r + 1] > hit_ptr[r]) row_of[read_ids[r]] = r;
    std::vector<uint32_t> piv;
    if (pivots) {
        piv.assign(pivots, pivots + n_piv);
    } else {
        for (uint64_t r = 0; r < n; ++r) piv.push_back(read_ids[r]);
    }
    struct Conn { uint32_t x, y; uint64_t s; uint8_t g; };
    std::vector<Conn> conns;
    for (uint32_t p : piv) {
        auto it = row_of.find(p);
        if (it == row_of.end()) continue;
        const uint64_t r = it->second;
        if (hit_ptr[r + 1] - hit_ptr[r] < min_kmers) continue;
        std::unordered_map<uint32_t, uint64_t> shared;
        for (uint64_t i = hit_ptr[r]; i < hit_ptr[r + 1]; ++i) {
            const uint32_t kid = sorted_kid[i];
            for (uint64_t j = kci_ptr[kid]; j < kci_ptr[kid + 1]; ++j) shared[kci_read[j]]++;
        }
        shared.erase(p);
        for (auto& kv : shared) {
            if (kv.second < min_score) continue;
            uint8_t g = 0;
            if (categories) g = categories[r] == categories[row_of.at(kv.first)];
            conns.push_back({p, kv.first, kv.second, g});
        }
    }
    std::sort(conns.begin(), conns.end(), [](const Conn& a, const Conn& b) {
        if (a.s != b.s) return a.s > b.s;
        if (a.x != b.x) return a.x < b.x;
        return a.y < b.y;
    });
    std::vector<uint32_t> x, y;
    std::vector<uint64_t> sc;
    std::vector<uint8_t> g;
    for (auto& c : conns) {
        x.push_back(c.x);
        y.push_back(c.y);
        sc.push_back(c.s);
        g.push_back(c.g);
    }
    *ox = dup_vec(x);
    *oy = dup_vec(y);
    *os = dup_vec(sc);
    *og = dup_vec(g);
    return (int64_t)conns.size();
}

// or_connections with the pivots split over `threads` threads (contiguous pivot ranges, the same
// per-pivot count as above), each thread's list sorted in the same order and the sorted lists
// merged pairwise.  Identical output; for the config-size parity tests (C5 share: 600 K pivots,
// 115 M connections) where one thread would take minutes.
int64_t or_connections_mt(uint64_t n, const uint64_t* hit_ptr, const uint32_t* sorted_kid,
                          const uint64_t* kci_ptr, const uint32_t* kci_read, const uint32_t* read_ids,
                          const uint32_t* pivots, uint64_t n_piv, uint32_t min_kmers, uint64_t min_score,
                          int threads, uint32_t** ox, uint32_t** oy, uint64_t** os) {
    if (threads < 1) threads = 1;
    std::unordered_map<uint32_t, uint64_t> row_of;
    for (uint64_t r = 0; r < n; ++r)
        if (hit_ptr[r + 1] > hit_ptr[r]) row_of[read_ids[r]] = r;
    std::vector<uint32_t> piv;
    if (pivots) piv.assign(pivots, pivots + n_piv);
    else for (uint64_t r = 0; r < n; ++r) piv.push_back(read_ids[r]);
    struct Conn { uint32_t x, y; uint64_t s; };
    auto less = [](const Conn& a, const Conn& b) {
        if (a.s != b.s) return a.s > b.s;
        if (a.x != b.x) return a.x < b.x;
        return a.y < b.y;
    };
    std::vector<std::vector<Conn>> part(threads);
    {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t] {
                const size_t p0 = piv.size() * t / threads, p1 = piv.size() * (t + 1) / threads;
                auto& out = part[t];
                std::unordered_map<uint32_t, uint64_t> shared;
                for (size_t q = p0; q < p1; ++q) {
                    const uint32_t p = piv[q];
                    auto it = row_of.find(p);
                    if (it == row_of.end()) continue;
                    const uint64_t r = it->second;
                    if (hit_ptr[r + 1] - hit_ptr[r] < min_kmers) continue;
                    shared.clear();
                    for (uint64_t i = hit_ptr[r]; i < hit_ptr[r + 1]; ++i) {
                        const uint32_t kid = sorted_kid[i];
                        for (uint64_t j = kci_ptr[kid]; j < kci_ptr[kid + 1]; ++j) shared[kci_read[j]]++;
                    }
                    shared.erase(p);
                    for (auto& kv : shared)
                        if (kv.second >= min_score) out.push_back({p, kv.first, kv.second});
                }
                std::sort(out.begin(), out.end(), less);
            });
        for (auto& x : th) x.join();
    }
    // pairwise merges, independent pairs in parallel
    while (part.size() > 1) {
        std::vector<std::vector<Conn>> next((part.size() + 1) / 2);
        std::vector<std::thread> th;
        for (size_t i = 0; i < next.size(); ++i)
            th.emplace_back([&, i] {
                if (2 * i + 1 >= part.size()) {
                    next[i].swap(part[2 * i]);
                    return;
                }
                auto& a = part[2 * i];
                auto& b = part[2 * i + 1];
                next[i].resize(a.size() + b.size());
                std::merge(a.begin(), a.end(), b.begin(), b.end(), next[i].begin(), less);
                std::vector<Conn>().swap(a);
                std::vector<Conn>().swap(b);
            });
        for (auto& x : th) x.join();
        part.swap(next);
    }
    const auto& c = part[0];
    uint32_t* X = (uint32_t*)std::malloc(std::max<size_t>(1, c.size() * 4));
    uint32_t* Y = (uint32_t*)std::malloc(std::max<size_t>(1, c.size() * 4));
    uint64_t* S = (uint64_t*)std::malloc(std::max<size_t>(1, c.size() * 8));
    for (size_t i = 0; i < c.size(); ++i) {
        X[i] = c[i].x;
        Y[i] = c[i].y;
        S[i] = c[i].s;
    }
    *ox = X;
    *oy = Y;
    *os = S;
    return (int64_t)c.size();
}

// Multi-threaded lookup-only timing kernel for the cpu_baseline leg: counts SDK hits
// over all windows of all reads with a std::unordered_set, reads split over threads.
uint64_t or_lookup_hits_mt(const char* bases, const uint64_t* offsets, uint64_t n, int k,
                           const uint64_t* sdk_keys, uint32_t n_sdk, int threads) {
    std::unordered_set<uint64_t> s(sdk_keys, sdk_keys + n_sdk);
    if (threads < 1) threads = 1;
    std::atomic<uint64_t> hits{0};
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            uint64_t h = 0;
            std::vector<uint64_t> wk;
            for (uint64_t r = (uint64_t)t; r < n; r += threads) {
                uint64_t len = offsets[r + 1] - offsets[r];
                wk.resize(len + 1);
                int64_t w = or_kmer_windows(bases + offsets[r], len, k, wk.data(), nullptr);
                for (int64_t i = 0; i < w; ++i) h += s.count(wk[i]);
            }
            hits += h;
        });
    for (auto& x : th) x.join();
    return hits.load();
}

// --- HLL auto-k (src/occurrences/KmerAnalysis.cpp:15-56, src/lib/HyperLogLog.hpp) ------
// MurmurHash3_x86_32 (src/lib/MurmurHash3.cpp:94-140), any length, byte-wise tail.
uint32_t or_murmur3_x86_32(const void* key, int len, uint32_t seed) {
    const uint8_t* data = (const uint8_t*)key;
    const int nblocks = len / 4;
    uint32_t h1 = seed;
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    auto rotl = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
    for (int i = 0; i < nblocks; ++i) {
        uint32_t k1;
        std::memcpy(&k1, data + 4 * i, 4);
        k1 *= c1; k1 = rotl(k1, 15); k1 *= c2;
        h1 ^= k1; h1 = rotl(h1, 13); h1 = h1 * 5 + 0xe6546b64u;
    }
    const uint8_t* tail = data + nblocks * 4;
    uint32_t k1 = 0;
    switch (len & 3) {
        case 3: k1 ^= (uint32_t)tail[2] << 16; [[fallthrough]];
        case 2: k1 ^= (uint32_t)tail[1] << 8; [[fallthrough]];
        case 1: k1 ^= tail[0]; k1 *= c1; k1 = rotl(k1, 15); k1 *= c2; h1 ^= k1;
    }
    h1 ^= (uint32_t)len;
    h1 ^= h1 >> 16; h1 *= 0x85ebca6bu; h1 ^= h1 >> 13; h1 *= 0xc2b2ae35u; h1 ^= h1 >> 16;
    return h1;
}

// HyperLogLog(b)::add of every KmerIterator window's canonical code (8 bytes, seed 313) of
// every read (KmerAnalysis.cpp:15-23; HyperLogLog.hpp:96-106).  clz(0) is taken as 32.
// Returns 0, or -1 when k is outside [1, 32] (KmerIterator.cpp:24-26) and reads exist.
int or_hll_registers(const char* bases, const uint64_t* offsets, uint64_t n, int k, int b, uint8_t* regs) {
    const uint32_t m = 1u << b;
    std::memset(regs, 0, m);
    std::vector<uint64_t> wk;
    for (uint64_t r = 0; r < n; ++r) {
        const uint64_t len = offsets[r + 1] - offsets[r];
        wk.resize(len + 1);
        const int64_t w = or_kmer_windows(bases + offsets[r], len, k, wk.data(), nullptr);
        if (w < 0) return -1;
        for (int64_t i = 0; i < w; ++i) {
            const uint64_t kmer = wk[i];   // little-endian bytes of the u64 (x86)
            const uint32_t h = or_murmur3_x86_32(&kmer, 8, 313);
            const uint32_t idx = h >> (32 - b);
            const uint32_t x = h << b;
            const int clz = x ? __builtin_clz(x) : 32;
            const uint8_t rank = (uint8_t)(std::min(32 - b, clz) + 1);
            if (rank > regs[idx]) regs[idx] = rank;
        }
    }
    return 0;
}

// hll::HyperLogLog::estimate (HyperLogLog.hpp:66-87 alpha, :113-132).
double or_hll_estimate(const uint8_t* regs, int b) {
    const uint32_t m = 1u << b;
    double alpha;
    switch (m) {
        case 16: alpha = 0.673; break;
        case 32: alpha = 0.697; break;
        case 64: alpha = 0.709; break;
        default: alpha = 0.7213 / (1.0 + 1.079 / m); break;
    }
    const double alphaMM = alpha * m * m;
    double sum = 0.0;
    for (uint32_t i = 0; i < m; i++) sum += 1.0 / (1 << regs[i]);
    double estimate = alphaMM / sum;
    if (estimate <= 2.5 * m) {
        uint32_t zeros = 0;
        for (uint32_t i = 0; i < m; i++) zeros += regs[i] == 0;
        if (zeros != 0) estimate = m * std::log(static_cast<double>(m) / zeros);
    } else if (estimate > (1.0 / 30.0) * 4294967296.0) {
        estimate = -4294967296.0 * std::log(1.0 - (estimate / 4294967296.0));
    }
    return estimate;
}

}  // extern "C"
