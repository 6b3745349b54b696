// TEST HARNESS (not product code): the multi-GPU counting protocol of libhga
// (hybrid-genome-assembler_amd/csrc/exchange_protocol.hpp, the same source the product compiles)
// driven on the CPU: a host engine stands in for the device rows (plain std::map counting, the packed
// piece format of exchange.hip restated), and the transport is the caller's hga_transport hook, as
// with hga_comm_init_host.  tests/test_dist.py runs it with gloo at world size 2 and 3 and compares
// with the single-process oracle.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/hga.h"
#include "../../hybrid-genome-assembler_amd/csrc/exchange_protocol.hpp"

namespace {

using hga::proto::Xport;

struct HostXport : Xport {
    hga_transport t;
    void a2a(const void* const* s, const uint64_t* sb, void* const* r, const uint64_t* rb) {
        if (t.alltoallv(t.user, s, sb, r, rb) != 0) throw std::runtime_error("transport failed");
    }
    void allgather(const void* mine, uint64_t bytes, void* all) override {
        std::vector<const void*> s(nranks, mine);
        std::vector<void*> r(nranks);
        std::vector<uint64_t> sz(nranks, bytes);
        for (int p = 0; p < nranks; ++p) r[p] = static_cast<char*>(all) + p * bytes;
        a2a(s.data(), sz.data(), r.data(), sz.data());
    }
    std::vector<std::vector<char>> allgatherv(const void* mine, uint64_t bytes) override {
        std::vector<uint64_t> sz(nranks);
        allgather(&bytes, 8, sz.data());
        std::vector<std::vector<char>> out(nranks);
        std::vector<const void*> s(nranks, mine);
        std::vector<void*> r(nranks);
        std::vector<uint64_t> sb(nranks, bytes);
        for (int p = 0; p < nranks; ++p) {
            out[p].resize(sz[p]);
            r[p] = out[p].data();
        }
        a2a(s.data(), sb.data(), r.data(), sz.data());
        return out;
    }
    void alltoallv_eng(const void* send, const uint64_t* sb, void* recv, const uint64_t* rb, bool keep_self) override {
        std::vector<const void*> s(nranks);
        std::vector<void*> r(nranks);
        std::vector<uint64_t> ss(sb, sb + nranks), rr(rb, rb + nranks);
        uint64_t so = 0, ro = 0;
        for (int p = 0; p < nranks; ++p) {
            s[p] = static_cast<const char*>(send) + so;
            r[p] = static_cast<char*>(recv) + ro;
            so += sb[p];
            ro += rb[p];
        }
        if (!keep_self) ss[rank] = rr[rank] = 0;
        a2a(s.data(), ss.data(), r.data(), rr.data());
    }
    std::vector<std::vector<char>> gatherv_root(const void* mine, uint64_t bytes, int root) override {
        std::vector<uint64_t> sz(nranks);
        allgather(&bytes, 8, sz.data());
        std::vector<std::vector<char>> out(nranks);
        std::vector<const void*> s(nranks, mine);
        std::vector<void*> r(nranks, nullptr);
        std::vector<uint64_t> sb(nranks, 0), rb(nranks, 0);
        sb[root] = bytes;
        if (rank == root)
            for (int p = 0; p < nranks; ++p) {
                out[p].resize(sz[p]);
                r[p] = out[p].data();
                rb[p] = sz[p];
            }
        a2a(s.data(), sb.data(), r.data(), rb.data());
        return out;
    }
};

int jf_code(unsigned char c) {
    switch (c) {
        case 'A': case 'a': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': return 3;
        default: return -1;
    }
}

// the device's bucket hash (kmer_dev.hpp Mix), restated: multiply by an odd constant mod 4^k, then
// xor the top half into the bottom half
uint64_t mix_host(uint64_t x, int k) {
    const int n = 2 * k;
    const uint64_t mask = n >= 64 ? ~0ull : (1ull << n) - 1;
    x = (x * 0x9E3779C07F4A7C15ull) & mask;
    return x ^ (x >> ((n + 1) / 2));
}

struct HostEngine {
    int k_ = 0;
    uint32_t F = 0;
    int rank_ = 0;
    bool allow_pack = true;
    std::vector<uint64_t> keys;                 // ascending
    std::vector<std::vector<uint32_t>> counts;  // per row, F counts
    std::vector<char> sbuf, rbuf;
    std::vector<uint64_t> xbp, xbd;             // pieces in bucket order, per-bucket counts

    int k() const { return k_; }
    uint32_t n_files() const { return F; }
    uint64_t rows() const { return keys.size(); }
    int pack_bits() const {
        if (!allow_pack) return 0;
        const int cb = (64 - 2 * k_) / (int)F;
        return (F <= 8 && cb >= 4) ? std::min(cb, 32) : 0;
    }
    void* send_buf(uint64_t b) { sbuf.assign(b + 64, 0); return sbuf.data(); }
    void* recv_buf(uint64_t b) { rbuf.assign(b + 64, 0); return rbuf.data(); }
    void sync() {}
    static uint32_t owner(const uint64_t* spl, uint32_t P, uint64_t key) {
        return (uint32_t)(std::upper_bound(spl, spl + (P - 1), key) - spl);
    }
    void set_rows(std::map<uint64_t, std::vector<uint64_t>>& m, uint32_t min) {
        keys.clear();
        counts.clear();
        for (auto& kv : m) {
            std::vector<uint32_t> c(F);
            bool any = false;
            for (uint32_t f = 0; f < F; ++f) {
                const uint64_t v = std::min<uint64_t>(kv.second[f], 0xFFFFFFFFull);
                c[f] = v >= min ? (uint32_t)v : 0u;
                any |= c[f] != 0;
            }
            if (!any) continue;
            keys.push_back(kv.first);
            counts.push_back(c);
        }
    }
    // pieces of every row, by hash bucket at resolution R; R differs between ranks on purpose (the
    // owners merge at the coarsest one)
    bool xb_pack_gather(uint32_t, std::vector<uint64_t>&, std::vector<uint64_t>&, int&) { return false; }
    int xb_pack(uint32_t P, uint64_t* per) {
        const int eb0 = hga::proto::xb_base_bits(k_);
        const int R = std::min(2 * k_, eb0 + rank_ % 3);
        const int cb = pack_bits();
        const uint64_t cmax = (1ull << cb) - 1;
        std::vector<std::pair<uint64_t, uint64_t>> t;   // (bucket, piece)
        for (size_t i = 0; i < keys.size(); ++i) {
            const uint64_t b = mix_host(keys[i], k_) >> (2 * k_ - R);
            std::vector<uint64_t> left(counts[i].begin(), counts[i].end());
            while (true) {
                uint64_t v = keys[i];
                bool more = false;
                for (uint32_t f = 0; f < F; ++f) {
                    const uint64_t c = std::min(left[f], cmax);
                    left[f] -= c;
                    more |= left[f] != 0;
                    v |= c << (2 * k_ + f * cb);
                }
                t.push_back({b, v});
                if (!more) break;
            }
        }
        std::stable_sort(t.begin(), t.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
        xbd.assign(1ull << R, 0);
        xbp.clear();
        for (auto& e : t) {
            xbd[e.first]++;
            xbp.push_back(e.second);
        }
        xbp.push_back(0);   // never empty
        for (uint32_t o = 0; o < P; ++o) {
            per[o] = 0;
            for (uint64_t j = hga::proto::xb_first(o, P, eb0, R); j < hga::proto::xb_first(o + 1, P, eb0, R); ++j)
                per[o] += xbd[j];
        }
        return R;
    }
    const void* xb_pieces() const { return xbp.data(); }
    const void* xb_dir() const { return xbd.data(); }
    // every bucket of the coarsest resolution from all senders' runs; checks that each run holds only
    // keys of its bucket and that the runs cover every received piece
    void xb_merge(const uint64_t* in, const uint64_t* self, const uint64_t* n_from, const uint64_t* dir_in,
                  const int* r_from, uint32_t P, uint32_t me, uint32_t min) {
        const int eb0 = hga::proto::xb_base_bits(k_);
        const int cb = pack_bits();
        const uint64_t kmask = 2 * k_ >= 64 ? ~0ull : (1ull << (2 * k_)) - 1, cmax = (1ull << cb) - 1;
        int rmin = 64;
        for (uint32_t p = 0; p < P; ++p) rmin = std::min(rmin, r_from[p]);
        std::vector<std::vector<uint64_t>> pre(P);   // per sender: piece offset of each of its buckets
        std::vector<const uint64_t*> src(P);
        uint64_t po = 0, dof = 0;
        for (uint32_t p = 0; p < P; ++p) {
            const uint64_t ne = hga::proto::xb_first(me + 1, P, eb0, r_from[p]) - hga::proto::xb_first(me, P, eb0, r_from[p]);
            pre[p].assign(ne + 1, 0);
            for (uint64_t j = 0; j < ne; ++j) pre[p][j + 1] = pre[p][j] + dir_in[dof + j];
            if (pre[p][ne] != n_from[p]) throw std::runtime_error("directory does not cover the pieces");
            src[p] = p == me ? self : in + po;   // the own slice stays in the send buffer
            if (p != me) po += n_from[p];
            dof += ne;
        }
        const uint64_t u0 = hga::proto::xb_first(me, P, eb0, rmin), u1 = hga::proto::xb_first(me + 1, P, eb0, rmin);
        std::map<uint64_t, std::vector<uint64_t>> m;
        uint64_t seen = 0;
        for (uint64_t u = 0; u < u1 - u0; ++u)
            for (uint32_t p = 0; p < P; ++p) {
                const int d = r_from[p] - rmin;
                for (uint64_t i = pre[p][u << d]; i < pre[p][(u + 1) << d]; ++i, ++seen) {
                    const uint64_t key = src[p][i] & kmask;
                    if ((mix_host(key, k_) >> (2 * k_ - rmin)) != u0 + u) throw std::runtime_error("piece in a foreign bucket");
                    auto& c = m.try_emplace(key, std::vector<uint64_t>(F, 0)).first->second;
                    for (uint32_t f = 0; f < F; ++f) c[f] += (src[p][i] >> (2 * k_ + f * cb)) & cmax;
                }
            }
        if (seen != po + n_from[me]) throw std::runtime_error("pieces outside every bucket");
        set_rows(m, min);
    }
    void partition(const uint64_t* spl, uint32_t P, uint64_t* ko, uint32_t* co, uint64_t* per) {
        std::vector<std::vector<size_t>> by(P);
        for (size_t i = 0; i < keys.size(); ++i) by[owner(spl, P, keys[i])].push_back(i);
        for (uint32_t p = 0; p < P; ++p) {
            per[p] = by[p].size();
            for (size_t i : by[p]) {
                *ko++ = keys[i];
                for (uint32_t f = 0; f < F; ++f) *co++ = counts[i][f];
            }
        }
    }
    void merge(const uint64_t* ki, const uint32_t* ci, uint64_t n, uint32_t min) {
        std::map<uint64_t, std::vector<uint64_t>> m;
        for (uint64_t i = 0; i < n; ++i) {
            auto& c = m.try_emplace(ki[i], std::vector<uint64_t>(F, 0)).first->second;
            for (uint32_t f = 0; f < F; ++f) c[f] += ci[i * F + f];
        }
        set_rows(m, min);
    }
};

// An ascending host list for proto::repartition (vw u32 payload words per entry); checks that every
// received run is ascending and inside this rank's code range
struct HostList {
    int bits = 0;
    uint32_t vw = 0;
    std::vector<uint64_t> k;
    std::vector<uint32_t> v;
    std::vector<char> buf;
    std::vector<uint64_t> spl;
    int me = 0;
    uint64_t cm() const { return bits >= 64 ? ~0ull : (1ull << bits) - 1; }
    uint32_t vbytes() const { return 4 * vw; }
    const void* keys() const { return k.data(); }
    const void* vals() const { return v.data(); }
    void split(const uint64_t* s, uint32_t P, uint64_t* per) {
        spl.assign(s, s + (P - 1));
        uint64_t prev = 0;
        for (uint32_t o = 0; o < P; ++o) {
            const uint64_t e = o + 1 < P ? (uint64_t)(std::lower_bound(k.begin(), k.end(), s[o],
                                                                       [&](uint64_t a, uint64_t b) { return (a & cm()) < b; }) - k.begin())
                                         : k.size();
            per[o] = e - prev;
            prev = e;
        }
    }
    void* recv(uint64_t n) { buf.assign(n * (8 + 4ull * vw) + 64, 0); return buf.data(); }
    void finish(const uint64_t* n_from, uint32_t P, uint64_t n) {
        const uint64_t* rk = reinterpret_cast<const uint64_t*>(buf.data());
        const uint32_t* rv = reinterpret_cast<const uint32_t*>(rk + n);
        const uint64_t lo = me ? spl[me - 1] : 0, hi = me + 1 < (int)P ? spl[me] : ~0ull;
        uint64_t at = 0;
        for (uint32_t p = 0; p < P; ++p)
            for (uint64_t i = 0; i < n_from[p]; ++i, ++at) {
                const uint64_t c = rk[at] & cm();
                if (c < lo || (me + 1 < (int)P && c >= hi)) throw std::runtime_error("entry outside the code range");
                if (i && (rk[at - 1] & cm()) >= c) throw std::runtime_error("received run not ascending");
            }
        std::vector<uint64_t> idx(n);
        for (uint64_t i = 0; i < n; ++i) idx[i] = i;
        std::sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return (rk[a] & cm()) < (rk[b] & cm()); });
        std::vector<uint64_t> nk(n);
        std::vector<uint32_t> nv(n * vw);
        for (uint64_t i = 0; i < n; ++i) {
            nk[i] = rk[idx[i]];
            for (uint32_t q = 0; q < vw; ++q) nv[i * vw + q] = rv[idx[i] * vw + q];
        }
        k.swap(nk);
        v.swap(nv);
    }
};

struct Rank {
    HostEngine e;
    HostXport x;
    std::vector<std::string> shard;
    int root = -1;   // hga_comm_set_root: gathered lists on this rank only
};

template <class T>
T* dup(const std::vector<T>& v) {
    T* p = (T*)std::malloc(std::max<size_t>(1, v.size() * sizeof(T)));
    if (!v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
    return p;
}

}  // namespace

extern "C" {

void xt_free(void* p) { std::free(p); }

void* xt_create(int k, int n_files, int rank, int nranks, const hga_transport* t, int allow_pack) {
    auto* r = new Rank();
    r->e.k_ = k;
    r->e.F = (uint32_t)n_files;
    r->e.allow_pack = allow_pack != 0;
    r->e.rank_ = rank;
    r->x.rank = rank;
    r->x.nranks = nranks;
    r->x.t = *t;
    r->shard.resize(n_files);
    return r;
}

void xt_destroy(void* h) { delete static_cast<Rank*>(h); }

void xt_add(void* h, int file, const char* seq, uint64_t n) { static_cast<Rank*>(h)->shard[file].append(seq, n); }

// local count with min 1 (every canonical window of every ACGT run), then the protocol's exchange
int xt_count_exchange(void* h, uint32_t min) {
    auto* r = static_cast<Rank*>(h);
    const int k = r->e.k_;
    const uint64_t mask = k >= 32 ? ~0ull : (1ull << (2 * k)) - 1;
    std::map<uint64_t, std::vector<uint64_t>> m;
    for (uint32_t f = 0; f < r->e.F; ++f) {
        uint64_t fwd = 0, rc = 0;
        int run = 0;
        for (unsigned char ch : r->shard[f]) {
            const int c = jf_code(ch);
            if (c < 0) { run = 0; fwd = rc = 0; continue; }
            fwd = ((fwd << 2) | (uint64_t)c) & mask;
            rc = (rc >> 2) | ((uint64_t)(3 - c) << (2 * (k - 1)));
            if (++run >= k) m.try_emplace(std::min(fwd, rc), std::vector<uint64_t>(r->e.F, 0)).first->second[f]++;
        }
    }
    r->e.set_rows(m, 1);
    try {
        hga::proto::count_exchange(r->e, r->x, min);
    } catch (...) {
        return -1;
    }
    return 0;
}

// global histogram: (threshold index, total, count) triples, (threshold, total) order
int64_t xt_spec_hist(void* h, const double* thr, int n_thr, int64_t** out) {
    auto* r = static_cast<Rank*>(h);
    std::set<double> T(thr, thr + n_thr);
    std::vector<double> tv(T.begin(), T.end());
    std::map<std::pair<int64_t, int64_t>, int64_t> bins;
    for (auto& c : r->e.counts) {
        int64_t tot = 0, prev = 0;
        for (auto v : c) { tot += v; prev = std::max<int64_t>(prev, v); }
        const double x = ((double)prev / (double)tot) * 100;
        const int64_t ti = std::upper_bound(tv.begin(), tv.end(), x) - tv.begin();
        bins[{ti, tot}] += 1;
    }
    std::vector<int64_t> local;
    for (auto& b : bins) { local.push_back(b.first.first); local.push_back(b.first.second); local.push_back(b.second); }
    const std::vector<int64_t> g = hga::proto::spec_hist_global(r->x, local);
    *out = dup(g);
    return (int64_t)g.size() / 3;
}

// the protocol's histogram merge on given triples (both the one-gather path and the variable-size
// fallback for more than proto::HIST_CAP triples on a rank)
int64_t xt_hist_merge(void* h, const int64_t* local, int64_t n_triples, int64_t** out) {
    auto* r = static_cast<Rank*>(h);
    const std::vector<int64_t> v(local, local + 3 * n_triples);
    const std::vector<int64_t> g = hga::proto::spec_hist_global(r->x, v);
    *out = dup(g);
    return (int64_t)g.size() / 3;
}

// the product's hga_comm_set_root
void xt_set_root(void* h, int root) { static_cast<Rank*>(h)->root = root; }

// global export: keys ascending (the owners' slices merged), flags; *n_discr over all owners
int64_t xt_select(void* h, int64_t lower, int64_t upper, uint64_t** keys, uint8_t** flags, uint64_t* n_discr) {
    auto* r = static_cast<Rank*>(h);
    std::vector<uint64_t> k;
    std::vector<uint8_t> f;
    uint64_t d = 0;
    for (size_t i = 0; i < r->e.keys.size(); ++i) {
        int64_t tot = 0;
        int nz = 0;
        for (auto v : r->e.counts[i]) { tot += v; nz += v > 0; }
        if (lower <= tot && tot <= upper) {
            k.push_back(r->e.keys[i]);
            f.push_back(nz == 1);
            d += nz == 1;
        }
    }
    // the owners' ascending selections re-partitioned by code range (one all-to-all of the export),
    // the ranks' ranges concatenated — the product's count_fetch_selected_global
    HostList l;
    l.bits = 2 * r->e.k_;
    l.vw = 1;
    l.me = r->x.rank;
    l.k = k;
    l.v.assign(f.begin(), f.end());
    hga::proto::repartition(l, r->x, r->e.k_);
    std::vector<uint8_t> lf(l.v.begin(), l.v.end());
    const std::vector<uint64_t> gk = hga::proto::concat_root(r->x, l.k, r->root);
    const std::vector<uint8_t> gf = hga::proto::concat_root(r->x, lf, r->root);
    *n_discr = hga::proto::sum_u64(r->x, {d})[0];
    *keys = dup(gk);
    *flags = dup(gf);
    return (int64_t)gk.size();
}

// global rows: keys ascending, counts row-major
int64_t xt_rows(void* h, uint64_t** keys, uint32_t** counts) {
    auto* r = static_cast<Rank*>(h);
    std::vector<uint32_t> c;
    for (auto& v : r->e.counts) c.insert(c.end(), v.begin(), v.end());
    HostList l;   // code-range re-partition of the rows, as count_rows_global
    l.bits = 2 * r->e.k_;
    l.vw = r->e.F;
    l.me = r->x.rank;
    l.k = r->e.keys;
    l.v = c;
    hga::proto::repartition(l, r->x, r->e.k_);
    const std::vector<uint64_t> gk = hga::proto::concat_root(r->x, l.k, r->root);
    const std::vector<uint32_t> gc = hga::proto::concat_root(r->x, l.v, r->root);
    *keys = dup(gk);
    *counts = dup(gc);
    return (int64_t)gk.size();
}

// ---- errors and the one-shot histogram gather of the device path, every rank deciding alike ----
// The general histogram gather with this rank's error bits: returns the triples (0 on an error),
// *qe_rank / *qe_bits = the lowest failing rank and its bits (-1 / 0: none).
int64_t xt_spec_hist_err(void* h, const int64_t* local, int64_t n_triples, uint64_t err, int64_t** out,
                         int* qe_rank, uint64_t* qe_bits) {
    auto* r = static_cast<Rank*>(h);
    hga::proto::QueryError qe;
    const std::vector<int64_t> g =
        hga::proto::spec_hist_global(r->x, std::vector<int64_t>(local, local + 3 * n_triples), err, &qe);
    *qe_rank = qe.rank;
    *qe_bits = qe.bits;
    *out = dup(g);
    return (int64_t)g.size() / 3;
}

// The device path's slot gather (comm.hip count_spec_hist_global) on the host: this rank's slot
// [err, overflow rows, pairs, (ti << 56 | total, count) pairs], an all-gather of the slots, then
// proto::merge_hist_slots; a fallback takes the general gather of the same triples.  Returns
// 0 ok / 1 fallback / 2 error with the triples in *out and the error in *qe_rank / *qe_bits.
int xt_hist_slots(void* h, uint64_t err, uint64_t n_over, const int64_t* local, int64_t n_triples, int64_t** out,
                  int64_t* n_out, int* qe_rank, uint64_t* qe_bits) {
    auto* r = static_cast<Rank*>(h);
    using namespace hga::proto;
    std::vector<uint64_t> slot(HS_WORDS, 0), all((size_t)r->x.nranks * HS_WORDS);
    slot[0] = err;
    slot[1] = n_over;
    slot[2] = (uint64_t)n_triples;
    for (int64_t i = 0; i < n_triples && (uint64_t)i < HS_CAP; ++i) {
        slot[HS_HDR + 2 * i] = (uint64_t)local[3 * i] << 56 | (uint64_t)local[3 * i + 1];
        slot[HS_HDR + 2 * i + 1] = (uint64_t)local[3 * i + 2];
    }
    r->x.allgather(slot.data(), HS_WORDS * 8, all.data());
    std::vector<int64_t> g;
    QueryError qe;
    const SlotMerge m = merge_hist_slots(all.data(), r->x.nranks, g, &qe);
    int rc = m == SlotMerge::ok ? 0 : m == SlotMerge::fallback ? 1 : 2;
    if (m == SlotMerge::fallback) g = spec_hist_global(r->x, std::vector<int64_t>(local, local + 3 * n_triples), 0, &qe);
    *qe_rank = qe.rank;
    *qe_bits = qe.bits;
    *out = dup(g);
    *n_out = (int64_t)g.size() / 3;
    return rc;
}

// ---- sharded categorization: construct_indices output of this rank's reads -> the whole input's
struct XIndex {   // flat C view of proto::CsrIndex (host arrays)
    uint64_t n, windows, reads_hit, H, U;
    uint32_t first_read_id, n_sdk;
    uint64_t *hit_ptr, *first_ptr, *kci_ptr;
    uint32_t *hit_kid, *hit_pos, *sorted_kid, *first_kid, *first_pos, *kci_read;
};

int xt_index_gather(void* h, const XIndex* in, XIndex* out) {
    auto* r = static_cast<Rank*>(h);
    hga::proto::CsrIndex a, g;
    a.n = in->n;
    a.windows = in->windows;
    a.reads_hit = in->reads_hit;
    a.first_read_id = in->first_read_id;
    a.n_sdk = in->n_sdk;
    a.hit_ptr.assign(in->hit_ptr, in->hit_ptr + in->n + 1);
    a.first_ptr.assign(in->first_ptr, in->first_ptr + in->n + 1);
    a.kci_ptr.assign(in->kci_ptr, in->kci_ptr + in->n_sdk + 1);
    a.hit_kid.assign(in->hit_kid, in->hit_kid + in->H);
    a.hit_pos.assign(in->hit_pos, in->hit_pos + in->H);
    a.sorted_kid.assign(in->sorted_kid, in->sorted_kid + in->H);
    a.kci_read.assign(in->kci_read, in->kci_read + in->H);
    a.first_kid.assign(in->first_kid, in->first_kid + in->U);
    a.first_pos.assign(in->first_pos, in->first_pos + in->U);
    if (!hga::proto::gather_index(r->x, a, g)) return -1;
    *out = XIndex{g.n, g.windows, g.reads_hit, g.hit_kid.size(), g.first_kid.size(), g.first_read_id, g.n_sdk,
                  dup(g.hit_ptr), dup(g.first_ptr), dup(g.kci_ptr), dup(g.hit_kid), dup(g.hit_pos),
                  dup(g.sorted_kid), dup(g.first_kid), dup(g.first_pos), dup(g.kci_read)};
    return 0;
}

// this rank's connections (reference order) -> the global list
int64_t xt_merge_connections(void* h, uint64_t n, const uint32_t* x, const uint32_t* y, const uint64_t* s,
                             const uint8_t* g, uint32_t** ox, uint32_t** oy, uint64_t** os, uint8_t** og) {
    auto* r = static_cast<Rank*>(h);
    hga::proto::ConnList in;
    in.x.assign(x, x + n);
    in.y.assign(y, y + n);
    in.s.assign(s, s + n);
    in.g.assign(g, g + n);
    const hga::proto::ConnList m = hga::proto::merge_connections(r->x, in);
    *ox = dup(m.x);
    *oy = dup(m.y);
    *os = dup(m.s);
    *og = dup(m.g);
    return (int64_t)m.x.size();
}

// splitters of the protocol (for the test of owner ranges)
void xt_splitters(int k, int P, uint64_t* out) {
    const auto s = hga::proto::owner_splitters(k, P);
    std::copy(s.begin(), s.end(), out);
}

}  // extern "C"
