// fastio.cpp — multi-threaded ingest for the two readers of seqio.h.
//
// Both readers have a sequential definition in seqio.cpp (jf_stream_seq / load_records_seq) that
// restates the reference line by line.  Here the same results are produced in parallel for the
// layouts that make records line-local:
//   * whole files are mapped read-only (populated), line starts found by a chunked SSE2 newline
//     scan, outputs written in parallel into never-zeroed huge-page buffers (Bytes);
//   * jf_stream: FASTA whose first non-empty line is a header is line-local (a header line
//     closes the previous record, every other line is sequence); FASTQ is taken when every
//     record is exactly 4 lines ('@' header, a sequence line not starting with '+', a '+' line,
//     a quality line as long as the sequence) — otherwise the sequential parser runs;
//   * load_records (SequenceRecordIterator.cpp:73-173): every file must hold a whole number of
//     4-line (FASTQ) / 2-line (FASTA) records, sniff cleanly and share one layout, so no record
//     straddles a file switch; the header regex parser is chosen per file with the reference's
//     carry-over.
// Anything else falls back to the sequential reader, so the outputs are identical by
// construction; tests/test_fastio.py compares the two on edge-case and random inputs.
#include <emmintrin.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <memory>
#include <thread>
#include <unordered_set>
#include <vector>

#include "seqio.h"
#include "seqio_internal.h"

namespace hgah {

// ---- Bytes
namespace {
constexpr size_t HUGE_PG = 2u << 20;
char* map_anon(size_t cap) {
    void* p = ::mmap(nullptr, cap, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) throw std::bad_alloc();
    if (cap >= HUGE_PG) (void)::madvise(p, cap, MADV_HUGEPAGE);
    return static_cast<char*>(p);
}
}  // namespace

Bytes::~Bytes() {
    if (p_) ::munmap(p_, cap_);
}
Bytes& Bytes::operator=(Bytes&& o) noexcept {
    if (this != &o) {
        if (p_) ::munmap(p_, cap_);
        p_ = o.p_;
        n_ = o.n_;
        cap_ = o.cap_;
        o.p_ = nullptr;
        o.n_ = o.cap_ = 0;
    }
    return *this;
}
void Bytes::reserve(size_t n) {
    if (n <= cap_) return;
    size_t cap = std::max<size_t>(n, cap_ * 2);
    cap = (cap + HUGE_PG - 1) / HUGE_PG * HUGE_PG;
    char* q = map_anon(cap);
    if (n_) std::memcpy(q, p_, n_);
    if (p_) ::munmap(p_, cap_);
    p_ = q;
    cap_ = cap;
}
void Bytes::resize(size_t n) {
    reserve(n);
    n_ = n;
}
void Bytes::append(const char* s, size_t n) {
    if (!n) return;
    reserve(n_ + n);
    std::memcpy(p_ + n_, s, n);
    n_ += n;
}

namespace {
std::atomic<int> g_threads{0};

template <class F>
void par_for(size_t n, int T, F&& f) {
    if (T <= 1 || n <= 1) {
        for (size_t i = 0; i < n; ++i) f(i);
        return;
    }
    std::atomic<size_t> next{0};
    std::vector<std::thread> th;
    const int nt = (int)std::min<size_t>((size_t)T, n);
    th.reserve(nt);
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&] {
            size_t i;
            while ((i = next.fetch_add(1)) < n) f(i);
        });
    for (auto& x : th) x.join();
}

// A read-only private mapping of a whole file, pages populated up front (page-cache speed, no
// copy).  Empty files map nothing.
struct MappedFile {
    const char* p = nullptr;
    size_t n = 0;
    explicit MappedFile(const std::string& path) {
        const int fd = ::open(path.c_str(), O_RDONLY);
        if (fd < 0) throw std::invalid_argument("File with path \"" + path + "\" does not exist");
        const off_t sz = ::lseek(fd, 0, SEEK_END);
        if (sz > 0) {
            void* m = ::mmap(nullptr, (size_t)sz, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
            if (m == MAP_FAILED) {
                ::close(fd);
                throw std::runtime_error("cannot map " + path);
            }
            (void)::madvise(m, (size_t)sz, MADV_SEQUENTIAL);
            p = static_cast<const char*>(m);
            n = (size_t)sz;
        }
        ::close(fd);
    }
    ~MappedFile() {
        if (p) ::munmap(const_cast<char*>(p), n);
    }
    MappedFile(const MappedFile&) = delete;
    MappedFile& operator=(const MappedFile&) = delete;
};

// Calls f(position) for every '\n' in [b, e), in order (16 bytes per SSE2 compare).
template <class F>
inline void each_newline(const char* base, size_t b, size_t e, F&& f) {
    size_t i = b;
    const __m128i nl = _mm_set1_epi8('\n');
    for (; i + 16 <= e; i += 16) {
        unsigned m = (unsigned)_mm_movemask_epi8(
            _mm_cmpeq_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(base + i)), nl));
        while (m) {
            f(i + (size_t)__builtin_ctz(m));
            m &= m - 1;
        }
    }
    for (; i < e; ++i)
        if (base[i] == '\n') f(i);
}

// Line starts of `d` as std::getline sees lines: line i = [st[i], st[i+1] - 1); st has
// n_lines + 1 entries, the last one size + 1 when the data does not end with '\n'.
std::vector<uint64_t> line_starts(const char* d, size_t n, int T) {
    std::vector<uint64_t> st;
    if (!n) {
        st.push_back(0);
        return st;
    }
    constexpr size_t CH = 4u << 20;
    const size_t nch = (n + CH - 1) / CH;
    std::vector<uint64_t> cnt(nch + 1, 0);
    par_for(nch, T, [&](size_t c) {
        uint64_t k = 0;
        each_newline(d, c * CH, std::min(n, (c + 1) * CH), [&](size_t) { ++k; });
        cnt[c + 1] = k;
    });
    for (size_t c = 0; c < nch; ++c) cnt[c + 1] += cnt[c];
    const uint64_t nl = cnt[nch];
    const bool tail = d[n - 1] != '\n';
    st.resize(nl + (tail ? 1 : 0) + 1);
    st[0] = 0;
    par_for(nch, T, [&](size_t c) {
        uint64_t k = cnt[c];
        each_newline(d, c * CH, std::min(n, (c + 1) * CH), [&](size_t i) { st[++k] = (uint64_t)i + 1; });
    });
    if (tail) st[nl + 1] = n + 1;
    return st;
}

struct LineView {
    const char* d;
    const std::vector<uint64_t>& st;
    uint64_t n() const { return st.size() - 1; }
    uint64_t b(uint64_t i) const { return st[i]; }
    uint64_t len(uint64_t i) const { return st[i + 1] - 1 - st[i]; }
    char c0(uint64_t i) const { return len(i) ? d[st[i]] : '\0'; }
};

// Chunked exclusive prefix sum of f(i), i < n (in parallel).
template <class F>
std::vector<uint64_t> prefix(uint64_t n, int T, F&& f) {
    std::vector<uint64_t> out(n + 1, 0);
    constexpr uint64_t CH = 1u << 16;
    const uint64_t nch = (n + CH - 1) / CH;
    std::vector<uint64_t> part(nch + 1, 0);
    par_for(nch, T, [&](size_t c) {
        uint64_t s = 0;
        for (uint64_t i = c * CH, e = std::min(n, (c + 1) * CH); i < e; ++i) {
            out[i + 1] = s += f(i);
        }
        part[c + 1] = s;
    });
    for (uint64_t c = 0; c < nch; ++c) part[c + 1] += part[c];
    par_for(nch, T, [&](size_t c) {
        for (uint64_t i = c * CH, e = std::min(n, (c + 1) * CH); i < e; ++i) out[i + 1] += part[c];
    });
    return out;
}

bool jf_stream_fast(const char* d, size_t n, int T, Bytes& out, uint64_t* n_records) {
    const std::vector<uint64_t> st = line_starts(d, n, T);
    const LineView L{d, st};
    const uint64_t nl = L.n();
    uint64_t first = 0;
    while (first < nl && L.len(first) == 0) ++first;
    if (first == nl) {   // only empty lines
        out.clear();
        if (n_records) *n_records = 0;
        return true;
    }
    const char h = L.c0(first);
    if (h == '>') {
        // per line: header -> one separator (none for the first), sequence line -> its bytes
        const std::vector<uint64_t> pre = prefix(nl - first, T, [&](uint64_t j) -> uint64_t {
            const uint64_t i = first + j;
            if (L.c0(i) == '>') return j == 0 ? 0 : 1;
            return L.len(i);
        });
        out.resize(pre.back());
        std::atomic<uint64_t> recs{0};
        constexpr uint64_t CH = 1u << 16;
        par_for((nl - first + CH - 1) / CH, T, [&](size_t c) {
            uint64_t r = 0;
            for (uint64_t j = c * CH, e = std::min(nl - first, (c + 1) * CH); j < e; ++j) {
                const uint64_t i = first + j;
                if (L.c0(i) == '>') {
                    ++r;
                    if (j) out[pre[j]] = '\n';
                } else if (L.len(i)) {
                    std::memcpy(&out[pre[j]], d + L.b(i), L.len(i));
                }
            }
            recs += r;
        });
        if (n_records) *n_records = recs;
        return true;
    }
    if (h != '@' || first != 0 || nl % 4 != 0) return false;
    const uint64_t R = nl / 4;
    std::atomic<bool> ok{true};
    constexpr uint64_t CH = 1u << 14;
    par_for((R + CH - 1) / CH, T, [&](size_t c) {
        for (uint64_t r = c * CH, e = std::min(R, (c + 1) * CH); r < e && ok; ++r) {
            const uint64_t l = 4 * r;
            if (L.c0(l) != '@' || L.c0(l + 1) == '+' || L.c0(l + 2) != '+' || L.len(l + 1) != L.len(l + 3))
                ok = false;
        }
    });
    if (!ok) return false;
    const std::vector<uint64_t> pre = prefix(R, T, [&](uint64_t r) { return L.len(4 * r + 1) + (r ? 1 : 0); });
    out.resize(pre.back());
    par_for((R + CH - 1) / CH, T, [&](size_t c) {
        for (uint64_t r = c * CH, e = std::min(R, (c + 1) * CH); r < e; ++r) {
            uint64_t o = pre[r];
            if (r) out[o++] = '\n';
            std::memcpy(&out[o], d + L.b(4 * r + 1), L.len(4 * r + 1));
        }
    });
    if (n_records) *n_records = R;
    return true;
}

}  // namespace

int host_threads() {
    int t = g_threads.load();
    if (t > 0) return t;
    if (const char* e = std::getenv("HGA_HOST_THREADS")) t = std::atoi(e);
    if (t <= 0) t = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    return t;
}
void set_host_threads(int n) { g_threads = n; }

Bytes jf_stream(const std::string& path, uint64_t* n_records) {
    const int T = host_threads();
    if (T <= 1) return jf_stream_seq(path, n_records);
    Bytes out;
    {
        const MappedFile m(path);
        if (jf_stream_fast(m.p, m.n, T, out, n_records)) return out;
    }
    return jf_stream_seq(path, n_records);
}

RecordSet load_records(const std::vector<std::string>& paths, bool annotate, bool keep_text) {
    const int T = host_threads();
    if (T <= 1 || paths.empty()) return load_records_seq(paths, annotate, keep_text);
    const HeaderParsers& hp = header_parsers();
    const size_t F = paths.size();
    std::vector<std::unique_ptr<MappedFile>> mf(F);
    std::vector<const char*> data(F);
    std::vector<std::vector<uint64_t>> st(F);
    for (size_t f = 0; f < F; ++f) {
        mf[f] = std::make_unique<MappedFile>(paths[f]);
        data[f] = mf[f]->p;
        st[f] = line_starts(mf[f]->p, mf[f]->n, T);
    }
    // sniff every file as LineStream::open does; anything unusual -> the sequential reader
    std::vector<int> rsz(F), ftype(F);
    std::vector<Hdr> hdr(F);
    Hdr carry = Hdr::UNKNOWN;
    for (size_t f = 0; f < F; ++f) {
        const LineView L{data[f], st[f]};
        if (L.n() < 2) return load_records_seq(paths, annotate, keep_text);
        const char h0 = L.c0(0);
        if (h0 == '@') {
            if (L.n() < 3 || L.c0(2) != '+') return load_records_seq(paths, annotate, keep_text);
            rsz[f] = 4;
            ftype[f] = 1;
        } else if (h0 == '>') {
            rsz[f] = 2;
            ftype[f] = 0;
        } else {
            return load_records_seq(paths, annotate, keep_text);
        }
        if (L.n() % (uint64_t)rsz[f]) return load_records_seq(paths, annotate, keep_text);
        // the layout is checked before a record's first line is read, so the first record after
        // a FASTQ <-> FASTA switch is read with the previous file's layout: sequential reader
        if (f && rsz[f] != rsz[f - 1]) return load_records_seq(paths, annotate, keep_text);
        const std::string header(data[f] + L.b(0), L.len(0));
        if (hp.parse(Hdr::SIMLORD, header).second != 0) carry = Hdr::SIMLORD;
        if (hp.parse(Hdr::NANOSIM, header).second != 0) carry = Hdr::NANOSIM;
        if (hp.parse(Hdr::PASS, header).second != 0) carry = Hdr::PASS;
        hdr[f] = carry;
    }
    std::vector<uint64_t> fr(F + 1, 0);   // first record of each file
    for (size_t f = 0; f < F; ++f) fr[f + 1] = fr[f] + (st[f].size() - 1) / rsz[f];
    const uint64_t R = fr[F];
    auto file_of = [&](uint64_t r) { return (size_t)(std::upper_bound(fr.begin(), fr.end(), r) - fr.begin() - 1); };
    auto seq_len = [&](uint64_t r) {
        const size_t f = file_of(r);
        const LineView L{data[f], st[f]};
        return L.len((r - fr[f]) * rsz[f] + 1);
    };
    RecordSet rs;
    rs.offsets = prefix(R, T, seq_len);
    rs.bases.resize(rs.offsets.back());
    rs.category.resize(R);
    rs.start.resize(R);
    rs.end.resize(R);
    if (keep_text) {
        rs.headers.resize(R);
        rs.qualities.resize(R);
    }
    constexpr uint64_t CH = 1u << 12;
    par_for((R + CH - 1) / CH, T, [&](size_t c) {
        for (uint64_t r = c * CH, e = std::min(R, (c + 1) * CH); r < e; ++r) {
            const size_t f = file_of(r);
            const LineView L{data[f], st[f]};
            const uint64_t l = (r - fr[f]) * rsz[f];
            std::memcpy(rs.bases.data() + rs.offsets[r], data[f] + L.b(l + 1), L.len(l + 1));
            rs.category[r] = annotate ? (int32_t)f : 0;
            const uint64_t hl = L.len(l);
            std::pair<uint32_t, uint32_t> se{0, 0};
            if (hdr[f] != Hdr::UNKNOWN || keep_text) {
                const std::string h = hl ? std::string(data[f] + L.b(l) + 1, hl - 1) : std::string();
                se = hp.parse(hdr[f], h);
                if (keep_text) {
                    rs.headers[r] = h;
                    if (rsz[f] == 4) rs.qualities[r] = std::string(data[f] + L.b(l + 3), L.len(l + 3));
                }
            }
            rs.start[r] = se.first != 0 ? se.first : 0;
            rs.end[r] = se.first != 0 ? se.first + se.second : 0;
        }
    });
    // load_meta_data (SequenceRecordIterator.cpp:31-71)
    rs.file_meta.resize(F);
    uint64_t sum_all = 0;
    std::vector<std::string> names;
    for (size_t f = 0; f < F; ++f) {
        FileMeta& m = rs.file_meta[f];
        m.filename = basename_of(paths[f]);
        m.file_type = ftype[f];
        names.push_back(m.filename);
        uint64_t mn = UINT64_MAX, mx = 0;
        for (uint64_t r = fr[f]; r < fr[f + 1]; ++r) {
            const uint64_t len = rs.offsets[r + 1] - rs.offsets[r];
            mn = std::min(mn, len);
            mx = std::max(mx, len);
        }
        m.records = fr[f + 1] - fr[f];
        m.total_bases = rs.offsets[fr[f + 1]] - rs.offsets[fr[f]];
        m.min_read_length = mn;
        m.max_read_length = mx;
        m.avg_read_length = m.total_bases / m.records;
        rs.meta.total_bases += m.total_bases;
        rs.meta.min_read_length = std::min(rs.meta.min_read_length, mn);
        rs.meta.records += m.records;
        sum_all += m.total_bases;
    }
    rs.meta.avg_read_length = sum_all / rs.meta.records;
    for (size_t i = 0; i < names.size(); ++i) rs.meta.filename += (i ? "__" : "") + names[i];
    rs.categories = annotate ? (uint32_t)F : 1u;
    return rs;
}

}  // namespace hgah

namespace hgah {

// The iteration order of a std::unordered_set<uint64_t> (libstdc++) after inserting `keys` in order,
// without building it.  std::hash<uint64_t> is the identity, bucket = key % bucket_count, and the node
// list only ever changes in two ways, both "a node goes to the front of its bucket's run, a node of an
// empty bucket to the front of the whole list": _Hashtable::_M_insert_bucket_begin for an insert, and
// _M_rehash_aux(unique) walking the old list in order for a rehash.  So after a rehash to n buckets
// followed by inserts, the list is the sequence S = (old list, then the new keys) regrouped: buckets in
// decreasing order of their first element's position in S, each bucket's keys in decreasing position.
// Rehash points depend only on the element count (the library's own _Prime_rehash_policy, asked once
// per new key as the table asks it), so the order is built epoch by epoch with counting passes over
// flat arrays (no per-key pointer chase), and a key already present changes nothing (insert() of a
// duplicate).  tests/test_host.py checks it against a real std::unordered_set (the oracle's
// or_load_sdk_text) on random key sets with and without duplicates.
namespace {
// a % d for any 64-bit a and d >= 1 (M = 2^128 / d rounded up; 128 fraction bits are exact for 64-bit
// operands), a multiply-only replacement for the library's 64-bit division
inline uint64_t fastmod_u64(uint64_t a, unsigned __int128 M, uint64_t d) {
    const unsigned __int128 low = M * a;
    const unsigned __int128 bot = ((unsigned __int128)(uint64_t)low * d) >> 64;
    const unsigned __int128 top = (unsigned __int128)(uint64_t)(low >> 64) * d;
    return (uint64_t)((bot + top) >> 64);
}

// the list order after inserting the distinct keys u in order; *nb_out = the final bucket count
std::vector<uint64_t> order_of_distinct(const std::vector<uint64_t>& u, size_t* nb_out) {
    const size_t U = u.size();
    std::__detail::_Prime_rehash_policy pol;
    std::vector<size_t> start, nbs;   // epoch e: keys [start[e], start[e+1]) inserted with nbs[e] buckets
    size_t nb = 1;                    // _M_single_bucket
    for (size_t m = 0; m < U; ++m) {
        const auto r = pol._M_need_rehash(nb, m, 1);
        if (r.first) {
            nb = r.second;
            start.push_back(m);
            nbs.push_back(nb);
        }
    }
    if (U && (start.empty() || start[0] != 0)) {
        start.insert(start.begin(), 0);
        nbs.insert(nbs.begin(), 1);
    }
    *nb_out = nb;
    std::vector<uint64_t> cur, seq;
    std::vector<uint32_t> bk, cnt, firsts;
    for (size_t e = 0; e < start.size(); ++e) {
        const size_t a = start[e], b = e + 1 < start.size() ? start[e + 1] : U, nbe = nbs[e];
        seq.assign(cur.begin(), cur.end());
        seq.insert(seq.end(), u.begin() + (int64_t)a, u.begin() + (int64_t)b);
        const size_t L = seq.size();
        const unsigned __int128 M = ~(unsigned __int128)0 / nbe + 1;
        bk.resize(L);
        cnt.assign(nbe, 0);
        firsts.clear();
        for (size_t j = 0; j < L; ++j) {
            const uint32_t bj = (uint32_t)fastmod_u64(seq[j], M, nbe);
            bk[j] = bj;
            if (cnt[bj]++ == 0) firsts.push_back(bj);
        }
        uint32_t pos = 0;   // buckets by decreasing first position: cnt becomes each bucket's cursor
        for (size_t t = firsts.size(); t-- > 0;) {
            const uint32_t c = cnt[firsts[t]];
            cnt[firsts[t]] = pos;
            pos += c;
        }
        cur.resize(L);
        for (size_t j = L; j-- > 0;) cur[cnt[bk[j]]++] = seq[j];   // decreasing position inside a bucket
    }
    return cur;
}
}  // namespace

std::vector<uint64_t> unordered_set_order(const uint64_t* keys, size_t n) {
    if (n >= (1ull << 32)) throw std::invalid_argument("too many k-mers");
    size_t nb = 1;
    // SDK lines are almost always distinct: order them as such, then look for a repeat inside the final
    // bucket runs (equal keys share a bucket); only then take the distinct keys in first-occurrence order
    std::vector<uint64_t> u(keys, keys + n);
    std::vector<uint64_t> out = order_of_distinct(u, &nb);
    bool dup = false;
    {
        const unsigned __int128 M = ~(unsigned __int128)0 / nb + 1;
        size_t r0 = 0;
        uint64_t b0 = n ? fastmod_u64(out[0], M, nb) : 0;
        std::vector<uint64_t> run;
        for (size_t j = 1; j <= n && !dup; ++j) {
            const uint64_t bj = j < n ? fastmod_u64(out[j], M, nb) : ~0ull;
            if (bj == b0) continue;
            if (j - r0 > 1) {   // the bucket run [r0, j)
                run.assign(out.begin() + (int64_t)r0, out.begin() + (int64_t)j);
                std::sort(run.begin(), run.end());
                dup = std::adjacent_find(run.begin(), run.end()) != run.end();
            }
            r0 = j;
            b0 = bj;
        }
    }
    if (!dup) return out;
    u.clear();
    int lg = 4;
    while ((1ull << lg) < 2 * n) ++lg;
    const size_t cap = 1ull << lg, msk = cap - 1;
    std::vector<uint64_t> slot(cap);
    std::vector<uint8_t> used(cap, 0);
    for (size_t i = 0; i < n; ++i) {
        const uint64_t key = keys[i];
        size_t h = (size_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - lg));
        while (used[h] && slot[h] != key) h = (h + 1) & msk;
        if (!used[h]) {
            used[h] = 1;
            slot[h] = key;
            u.push_back(key);
        }
    }
    return order_of_distinct(u, &nb);
}

// load_text_file_kmers (src/read_clustering.cpp:18-33) without its per-line cost: the file mapped, its
// lines ('\n'-split as std::getline, a CR kept in the line, no line after a final '\n') encoded on
// host_threads() threads (line_canonical = KmerIterator(line, len).next_kmer()), then the KmerID order
// of inserting them into a std::unordered_set in file order (unordered_set_order).  k = the last line's
// length; a line longer than 32 throws, the first such line in file order deciding, as the reference's.
std::vector<uint64_t> load_kmer_text(const std::string& path, int* k_out) {
    MappedFile f(path);
    std::vector<size_t> ends;   // line i = [ends[i-1] + 1, ends[i])
    each_newline(f.p, 0, f.n, [&](size_t pos) { ends.push_back(pos); });
    if (f.n && (ends.empty() || ends.back() != f.n - 1)) ends.push_back(f.n);   // last line without '\n'
    const size_t L = ends.size();
    std::vector<uint64_t> codes(L);
    std::atomic<size_t> bad{SIZE_MAX};
    const size_t CH = 1 << 16;
    par_for((L + CH - 1) / CH, host_threads(), [&](size_t c) {
        for (size_t i = c * CH; i < std::min(L, (c + 1) * CH); ++i) {
            const size_t b = i ? ends[i - 1] + 1 : 0, e = ends[i];
            if (e - b > 32) {
                size_t cur = bad.load();
                while (i < cur && !bad.compare_exchange_weak(cur, i)) {}
                continue;
            }
            codes[i] = line_canonical(f.p + b, e - b);
        }
    });
    if (bad.load() != SIZE_MAX) throw std::invalid_argument("Kmer size is too big");
    *k_out = L ? (int)(ends[L - 1] - (L > 1 ? ends[L - 2] + 1 : 0)) : 0;
    return unordered_set_order(codes.data(), codes.size());
}

}  // namespace hgah
