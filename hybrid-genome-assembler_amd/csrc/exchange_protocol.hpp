// exchange_protocol.hpp — the multi-GPU counting protocol, written once over two
// small interfaces so that the product (comm.hip: device engine, RCCL or host-staged transport) and
// the CPU test harness (tests/native/xproto_host.cpp: host engine, the caller's transport hook)
// run the same code.  Plain C++17, no HIP.
//
//   every rank has counted its shard with min 1 (no per-file drop before the global sum);
//   packed rows (one u64 piece per row, the default): owners hold HASH ranges — the engine orders
//   its pieces by a bijective hash of the key (the same on every rank) and counts them per hash
//   bucket at a resolution of R bits (R may differ between ranks); bucket cells of the top EB0
//   bits are split evenly over the owners; one all-to-all-v moves the pieces, a second the
//   per-bucket counts (the owner's directory of every sender's runs), and the owner sums each of
//   its buckets from all senders' runs without re-binning;
//   wide rows ((key, counts[F]) when rows do not pack): owner o holds canonical codes
//   [spl[o-1], spl[o]) on equal-mass splitters;
//   the owner sums equal keys and drops counts < min per file (jellyfish --bc, run_jellyfish.sh:3-6);
//   histogram triples of all owners are summed per (threshold, total) bin in std::map order
//   (JellyfishOccurrenceReader.cpp:88-108); exports and rows are the owners' sorted slices merged by
//   key, i.e. ascending code order (:63-86, :110-135).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <queue>
#include <utility>
#include <vector>

namespace hga {
namespace proto {

// Collectives of one rank.  Host-memory forms take host pointers; `alltoallv_eng` moves engine
// memory (device memory in the product) with per-peer slices contiguous in rank order; with
// keep_self false the rank's own slice stays where it is (it keeps its place in the send buffer,
// none in the receive buffer).
struct Xport {
    int rank = 0, nranks = 1;
    virtual ~Xport() = default;
    virtual void allgather(const void* mine, uint64_t bytes, void* all) = 0;
    virtual std::vector<std::vector<char>> allgatherv(const void* mine, uint64_t bytes) = 0;
    virtual void alltoallv_eng(const void* send, const uint64_t* send_bytes, void* recv, const uint64_t* recv_bytes,
                               bool keep_self = true) = 0;
    // Every rank's bytes, in rank order, on `root` only (the other ranks get an empty list): one copy of
    // a gathered result crosses the ranks instead of P (the export to one writer).
    virtual std::vector<std::vector<char>> gatherv_root(const void* mine, uint64_t bytes, int root) = 0;
};

// Owner ranges over canonical codes in [0, 4^k): canonical = min(fwd, rc) of uniform codes has mass
// 1 - (1 - x/4^k)^2 below x, so owner o starts at 4^k (1 - sqrt(1 - o/P)).  Any ascending splitters
// give the same global result; these balance the load.
inline std::vector<uint64_t> owner_splitters(int k, int P) {
    const long double m = std::ldexp(1.0L, 2 * k);
    std::vector<uint64_t> out;
    for (int o = 1; o < P; ++o) {
        const long double x = m * (1.0L - std::sqrt(1.0L - (long double)o / P));
        uint64_t v = x >= m ? (uint64_t)(m - 1) : (uint64_t)x;
        if (!out.empty() && v < out.back()) v = out.back();
        out.push_back(v);
    }
    return out;
}

// Hash-bucket ownership of the packed exchange.  A rank's directory resolution R (bits of the hash,
// R >= EB0) is its own choice; cell c of the top EB0 bits belongs to owner floor(c P / 2^EB0), so a
// bucket at any resolution lies in one owner, and owner o's buckets at resolution R are the
// contiguous range [cell_lo(o) << (R - EB0), cell_lo(o + 1) << (R - EB0)).  EB0 = 10 covers up to
// 1024 owners (KX_MAX_OWN).
inline int xb_base_bits(int k) { return std::min(10, 2 * k); }
inline uint64_t xb_cell_lo(int o, int P, int eb0) {   // smallest cell c with floor(c P / 2^eb0) >= o
    return (((uint64_t)o << eb0) + (uint64_t)P - 1) / (uint64_t)P;
}
inline uint64_t xb_first(int o, int P, int eb0, int R) { return xb_cell_lo(o, P, eb0) << (R - eb0); }
inline uint32_t xb_owner_of_cell(uint64_t c, int P, int eb0) { return (uint32_t)((c * (uint64_t)P) >> eb0); }

// Engine E (the rank's rows after a local count with min 1):
//   int k(); uint32_t n_files(); uint64_t rows(); int pack_bits();
//   void* send_buf(uint64_t bytes); void* recv_buf(uint64_t bytes);     (engine memory, kept by E)
//   packed (hash-bucket owners):
//     int xb_pack(uint32_t P, uint64_t* per_owner);
//         orders the pieces by bucket (owner-major) in engine memory xb_pieces() and counts them per
//         bucket in xb_dir() (u64, 2^R entries); returns R; per_owner[o] = pieces for owner o
//     bool xb_pack_gather(uint32_t P, std::vector<uint64_t>& per, std::vector<uint64_t>& all, int& R);
//         optional fused form of xb_pack + the piece-count all-gather below (an engine whose transport
//         gathers its device words directly): per = this rank's W words with the extras filled, out:
//         per[0, P] and `all` (P x W, rank-major) as recv_counts leaves them; false: not taken (the
//         engine did nothing), xb_pack + allgather follow
//     const void* xb_pieces(); const void* xb_dir();
//     void xb_merge(const uint64_t* in, const uint64_t* self, const uint64_t* n_from, const uint64_t* dir_in,
//                   const int* r_from, uint32_t P, uint32_t me, uint32_t min);
//         in = the other senders' pieces for this owner (sender order, n_from[p] each), self = this
//         rank's own slice of its send buffer (it does not move); dir_in = every sender's counts of
//         this owner's buckets at its resolution r_from[p] (sender order)
//   wide (code-range owners):
//     void partition(const uint64_t* spl, uint32_t P, uint64_t* keys, uint32_t* counts, uint64_t* per);
//     void merge(const uint64_t* keys, const uint32_t* counts, uint64_t n, uint32_t min);
//   void sync();
// Returns the pieces / rows this owner received.  `extra` (same length on every rank) rides in the
// piece-count all-gather; *extra_sum receives its element-wise sums over the ranks (one collective
// less per exchange).
template <class E>
uint64_t count_exchange(E& e, Xport& x, uint32_t min_per_file, const std::vector<uint64_t>& extra = {},
                        std::vector<uint64_t>* extra_sum = nullptr) {
    const int P = x.nranks, me = x.rank;
    const size_t X = extra.size(), W = (size_t)P + 1 + X;
    std::vector<uint64_t> per(W), all((size_t)P * W), rn(P), sb(P), rb(P);
    for (size_t i = 0; i < X; ++i) per[P + 1 + i] = extra[i];
    auto digest = [&] {   // `all` gathered: pieces per sender for this owner, the extras' sums
        uint64_t n = 0;
        for (int p = 0; p < P; ++p) n += (rn[p] = all[(size_t)p * W + me]);
        if (extra_sum) {
            extra_sum->assign(X, 0);
            for (int p = 0; p < P; ++p)
                for (size_t i = 0; i < X; ++i) (*extra_sum)[i] += all[(size_t)p * W + P + 1 + i];
        }
        return n;
    };
    auto recv_counts = [&] {
        x.allgather(per.data(), 8 * (uint64_t)W, all.data());
        return digest();
    };
    if (e.pack_bits() > 0) {   // one u64 piece per row (a count past the piece width: several pieces)
        const int eb0 = xb_base_bits(e.k());
        int R = 0;
        uint64_t n;
        if (e.xb_pack_gather((uint32_t)P, per, all, R)) {
            n = digest();
        } else {
            R = e.xb_pack((uint32_t)P, per.data());
            per[P] = (uint64_t)R;
            n = recv_counts();
        }
        std::vector<int> rf(P);
        uint64_t nd = 0;   // directory entries this owner receives
        for (int p = 0; p < P; ++p) {
            rf[p] = (int)all[(size_t)p * W + P];
            nd += xb_first(me + 1, P, eb0, rf[p]) - xb_first(me, P, eb0, rf[p]);
        }
        // engine receive memory: the other senders' pieces, then the directories (8-byte aligned);
        // this rank's own slice is merged from its send buffer
        const uint64_t n_in = n - rn[me];
        uint64_t self_off = 0;
        for (int p = 0; p < me; ++p) self_off += per[p];
        char* in = static_cast<char*>(e.recv_buf((n_in + nd + 1) * 8));
        uint64_t* dir_in = reinterpret_cast<uint64_t*>(in + n_in * 8);
        for (int p = 0; p < P; ++p) {
            sb[p] = per[p] * 8;
            rb[p] = p == me ? 0 : rn[p] * 8;
        }
        x.alltoallv_eng(e.xb_pieces(), sb.data(), in, rb.data(), false);
        for (int p = 0; p < P; ++p) {
            sb[p] = 8 * (xb_first(p + 1, P, eb0, R) - xb_first(p, P, eb0, R));
            rb[p] = 8 * (xb_first(me + 1, P, eb0, rf[p]) - xb_first(me, P, eb0, rf[p]));
        }
        x.alltoallv_eng(e.xb_dir(), sb.data(), dir_in, rb.data());
        e.xb_merge(reinterpret_cast<const uint64_t*>(in), static_cast<const uint64_t*>(e.xb_pieces()) + self_off,
                   rn.data(), dir_in, rf.data(), (uint32_t)P, (uint32_t)me, min_per_file);
        return n;
    }
    const std::vector<uint64_t> spl = owner_splitters(e.k(), P);
    // wide rows: keys u64 then counts u32[F] row-major, one all-to-all each
    const uint32_t F = e.n_files();
    const uint64_t rows = e.rows(), rcap = rows ? rows : 1;
    char* w = static_cast<char*>(e.send_buf(rcap * (8 + 4ull * F)));
    uint64_t* keys = reinterpret_cast<uint64_t*>(w);
    uint32_t* cnts = reinterpret_cast<uint32_t*>(w + rcap * 8);
    e.partition(spl.data(), (uint32_t)P, keys, cnts, per.data());
    const uint64_t n = recv_counts(), ncap = n ? n : 1;
    char* r = static_cast<char*>(e.recv_buf(ncap * (8 + 4ull * F)));
    uint64_t* rk = reinterpret_cast<uint64_t*>(r);
    uint32_t* rc = reinterpret_cast<uint32_t*>(r + ncap * 8);
    for (int p = 0; p < P; ++p) {
        sb[p] = per[p] * 8;
        rb[p] = rn[p] * 8;
    }
    x.alltoallv_eng(keys, sb.data(), rk, rb.data());
    for (int p = 0; p < P; ++p) {
        sb[p] = per[p] * 4 * F;
        rb[p] = rn[p] * 4 * F;
    }
    x.alltoallv_eng(cnts, sb.data(), rc, rb.data());
    e.sync();
    e.merge(rk, rc, n, min_per_file);
    return n;
}

// ---- errors of the global count queries ------------------------------------------------------
// Every rank reports its error bits in the words the query gathers anyway, and every rank decides
// on the gathered words: all ranks raise the same error, and none enters a collective (a fallback
// gather) that a failed rank skips.  Bits: the settle bits of an unconsumed count run (1 a bucket
// could not be split, 2 row capacity, 4 level-1 pool) and the histogram's own (8 a specificity above
// the last threshold, 16 overflow list full, 32 compaction buffer full).
// 64: any other local failure before the rank's gather (state, allocation): it still takes part in the
// gather with this bit set.
enum : uint64_t { QE_UNSPLIT = 1, QE_ROWCAP = 2, QE_POOL = 4, QE_SPEC_THR = 8, QE_OVER = 16, QE_COMPACT = 32,
                  QE_LOCAL = 64 };
struct QueryError {
    int rank = -1;   // the lowest failing rank, -1: none
    uint64_t bits = 0;
};
inline QueryError first_error(const uint64_t* words, int P, size_t stride) {
    QueryError e;
    for (int p = 0; p < P && e.rank < 0; ++p)
        if (words[(size_t)p * stride]) {
            e.rank = p;
            e.bits = words[(size_t)p * stride];
        }
    return e;
}

// Owners' (threshold index, total, count) triples -> the global histogram, (threshold, total) order.
// One fixed-size all-gather of [n, up to HIST_CAP triples] per rank; only when some rank has more
// triples (very wide count ranges) a variable-size all-gather follows.
// `err` (this rank's error bits, see QueryError) rides in the slot; when any rank reports one, every
// rank returns an empty histogram with *qe naming the lowest failing rank (no further collective).
constexpr size_t HIST_CAP = 1024;
inline std::vector<int64_t> spec_hist_global(Xport& x, const std::vector<int64_t>& local, uint64_t err = 0,
                                             QueryError* qe = nullptr) {
    const size_t P = (size_t)x.nranks, slot = 2 + 3 * HIST_CAP;
    std::vector<int64_t> mine(slot, 0), all(P * slot);
    const size_t n = err ? 0 : local.size() / 3;
    mine[0] = (int64_t)err;
    mine[1] = (int64_t)n;
    for (size_t i = 0; i < 3 * n && i < 3 * HIST_CAP; ++i) mine[2 + i] = local[i];
    x.allgather(mine.data(), slot * 8, all.data());
    const QueryError e = first_error(reinterpret_cast<const uint64_t*>(all.data()), (int)P, slot);
    if (qe) *qe = e;
    if (e.rank >= 0) return {};
    bool fits = true;
    for (size_t p = 0; p < P; ++p) fits = fits && (size_t)all[p * slot + 1] <= HIST_CAP;
    std::vector<std::vector<char>> parts;
    if (fits) {
        parts.resize(P);
        for (size_t p = 0; p < P; ++p) {
            const size_t np = (size_t)all[p * slot + 1];
            parts[p].resize(np * 24);
            if (np) std::memcpy(parts[p].data(), &all[p * slot + 2], np * 24);
        }
    } else {
        parts = x.allgatherv(local.data(), local.size() * 8);
    }
    std::map<std::pair<int64_t, int64_t>, int64_t> bins;
    for (const auto& pt : parts) {
        const int64_t* t = reinterpret_cast<const int64_t*>(pt.data());
        for (size_t i = 0; i + 3 <= pt.size() / 8; i += 3) bins[{t[i], t[i + 1]}] += t[i + 2];
    }
    std::vector<int64_t> out;
    out.reserve(bins.size() * 3);
    for (const auto& b : bins) {
        out.push_back(b.first.first);
        out.push_back(b.first.second);
        out.push_back(b.second);
    }
    return out;
}

// Element-wise sums of a small u64 vector over all ranks.
inline std::vector<uint64_t> sum_u64(Xport& x, const std::vector<uint64_t>& mine) {
    std::vector<uint64_t> all(mine.size() * x.nranks), out(mine.size(), 0);
    x.allgather(mine.data(), mine.size() * 8, all.data());
    for (int p = 0; p < x.nranks; ++p)
        for (size_t i = 0; i < mine.size(); ++i) out[i] += all[p * mine.size() + i];
    return out;
}

// Every rank's vector of T, concatenated in rank order (owner order = ascending codes).
template <class T>
std::vector<T> concat(Xport& x, const std::vector<T>& mine) {
    const auto parts = x.allgatherv(mine.data(), mine.size() * sizeof(T));
    std::vector<T> out;
    for (const auto& pt : parts) {
        const T* v = reinterpret_cast<const T*>(pt.data());
        out.insert(out.end(), v, v + pt.size() / sizeof(T));
    }
    return out;
}

// concat on `root` only (root >= 0; the other ranks get an empty vector), or on every rank (root < 0).
template <class T>
std::vector<T> concat_root(Xport& x, const std::vector<T>& mine, int root) {
    if (root < 0) return concat(x, mine);
    const auto parts = x.gatherv_root(mine.data(), mine.size() * sizeof(T), root);
    std::vector<T> out;
    for (const auto& pt : parts) {
        const T* v = reinterpret_cast<const T*>(pt.data());
        out.insert(out.end(), v, v + pt.size() / sizeof(T));
    }
    return out;
}

// Every rank's ascending keys (with vw values of type V per key) merged into one ascending list:
// the owners' slices of exports and rows (hash-bucket owners interleave in code order; code-range
// owners come out concatenated in rank order).  Equal keys keep rank order.
template <class V>
void merge_sorted(Xport& x, const std::vector<uint64_t>& keys, const std::vector<V>& vals, size_t vw,
                  std::vector<uint64_t>& out_keys, std::vector<V>& out_vals) {
    const auto pk = x.allgatherv(keys.data(), keys.size() * 8);
    const auto pv = x.allgatherv(vals.data(), vals.size() * sizeof(V));
    const int P = x.nranks;
    std::vector<const uint64_t*> k(P);
    std::vector<const V*> v(P);
    std::vector<size_t> n(P), at(P, 0);
    size_t tot = 0;
    for (int p = 0; p < P; ++p) {
        k[p] = reinterpret_cast<const uint64_t*>(pk[p].data());
        v[p] = reinterpret_cast<const V*>(pv[p].data());
        tot += (n[p] = pk[p].size() / 8);
    }
    out_keys.clear();
    out_vals.clear();
    out_keys.reserve(tot);
    out_vals.reserve(tot * vw);
    using Head = std::pair<uint64_t, int>;   // (key, rank): smallest key first, ties by rank
    std::priority_queue<Head, std::vector<Head>, std::greater<Head>> q;
    for (int p = 0; p < P; ++p)
        if (n[p]) q.push({k[p][0], p});
    while (!q.empty()) {
        const int p = q.top().second;
        q.pop();
        const size_t i = at[p]++;
        out_keys.push_back(k[p][i]);
        out_vals.insert(out_vals.end(), v[p] + i * vw, v[p] + (i + 1) * vw);
        if (at[p] < n[p]) q.push({k[p][at[p]], p});
    }
}

// Code-range re-partition of per-rank ascending lists.  With hash-bucket owners
// every owner's export and rows span the whole code space; instead of every rank merging every
// owner's slice (merge_sorted), the ranks cut their ascending lists at the code-range splitters
// (owner_splitters: rank o takes the codes [spl[o-1], spl[o])) and swap the pieces in one all-to-all
// of the list itself — the export, not the rows behind it; each rank orders the P runs it received.
// The global list is then the ranks' ranges concatenated in rank order (concat), the reference's
// single ascending pass (JellyfishOccurrenceReader.cpp:110-135).
// Engine L (engine memory: device memory in the product):
//   uint32_t vbytes();                            payload bytes per entry (0: keys only)
//   void split(const uint64_t* spl, uint32_t P, uint64_t* per);   entries per code range (list ascending)
//   const void* keys(); const void* vals();
//   void* recv(uint64_t n);                       room for n keys (u64) followed by n payloads
//   void finish(const uint64_t* n_from, uint32_t P, uint64_t n);  the runs in recv (sender order) ->
//                                                 the rank's ascending list of n entries
// Returns the entries of this rank's code range.
template <class L>
uint64_t repartition(L& l, Xport& x, int k) {
    const int P = x.nranks, me = x.rank;
    const std::vector<uint64_t> spl = owner_splitters(k, P);
    std::vector<uint64_t> per(P), all((size_t)P * P), rn(P), sb(P), rb(P);
    l.split(spl.data(), (uint32_t)P, per.data());
    x.allgather(per.data(), 8ull * (uint64_t)P, all.data());
    uint64_t n = 0;
    for (int p = 0; p < P; ++p) n += (rn[p] = all[(size_t)p * P + me]);
    char* r = static_cast<char*>(l.recv(n));
    const uint32_t vb = l.vbytes();
    for (int p = 0; p < P; ++p) {
        sb[p] = per[p] * 8;
        rb[p] = rn[p] * 8;
    }
    x.alltoallv_eng(l.keys(), sb.data(), r, rb.data());
    if (vb) {
        for (int p = 0; p < P; ++p) {
            sb[p] = per[p] * vb;
            rb[p] = rn[p] * vb;
        }
        x.alltoallv_eng(l.vals(), sb.data(), r + n * 8, rb.data());
    }
    l.finish(rn.data(), (uint32_t)P, n);
    return n;
}

// The one-shot histogram gather of the device path: rank p's slot holds [error bits, overflow rows,
// n pairs, the first HS_CAP (threshold << 56 | total, count) pairs].  ok: `out` holds the global
// (threshold, total, count) triples in (threshold, total) order; fallback: some rank has an overflow
// list or more than HS_CAP pairs (every rank then takes the general gather); error: *err names it.
constexpr uint64_t HS_CAP = 1024, HS_HDR = 3, HS_WORDS = HS_HDR + 2 * HS_CAP;
enum class SlotMerge { ok, fallback, error };
inline SlotMerge merge_hist_slots(const uint64_t* hs, int P, std::vector<int64_t>& out, QueryError* err) {
    *err = first_error(hs, P, HS_WORDS);
    if (err->rank >= 0) return SlotMerge::error;
    for (int p = 0; p < P; ++p)
        if (hs[(size_t)p * HS_WORDS + 1] != 0 || hs[(size_t)p * HS_WORDS + 2] > HS_CAP) return SlotMerge::fallback;
    std::map<std::pair<int64_t, int64_t>, int64_t> bins;
    for (int p = 0; p < P; ++p) {
        const uint64_t* sl = hs + (size_t)p * HS_WORDS;
        for (uint64_t i = 0; i < sl[2]; ++i) {
            const uint64_t key = sl[HS_HDR + 2 * i];
            bins[{(int64_t)(key >> 56), (int64_t)(key & ((1ull << 56) - 1))}] += (int64_t)sl[HS_HDR + 2 * i + 1];
        }
    }
    out.clear();
    out.reserve(3 * bins.size());
    for (const auto& b : bins) {
        out.push_back(b.first.first);
        out.push_back(b.first.second);
        out.push_back(b.second);
    }
    return SlotMerge::ok;
}

// ---- sharded categorization -------------------------------------------
// construct_indices output of one rank (ReadClusteringEngine.cpp:234-299) over its contiguous ReadID
// range: per-read CSRs (hit_ptr[n+1] with hit_kid/hit_pos/sorted_kid[H], first_ptr[n+1] with
// first_kid/first_pos[U]) and kmer_component_index kci_ptr[K+1] / kci_read[H] holding read
// indices relative to first_read_id.
struct CsrIndex {
    uint64_t n = 0, windows = 0, reads_hit = 0;
    uint32_t first_read_id = 1, n_sdk = 0;
    std::vector<uint64_t> hit_ptr, first_ptr, kci_ptr;
    std::vector<uint32_t> hit_kid, hit_pos, sorted_kid, first_kid, first_pos, kci_read;
};

// The whole input's index from every rank's shard, identical on every rank: reads concatenated in
// rank order (ReadIDs must be contiguous across ranks), kmer_component_index per KmerID the ranks'
// lists concatenated in rank order — ascending ReadIDs, as the reference's sort leaves them
// (:282-284).  Returns false when the shards are not contiguous or use different SDK sets.
inline bool gather_index(Xport& x, const CsrIndex& in, CsrIndex& out) {
    const int P = x.nranks;
    const std::vector<uint64_t> mine{in.n, in.hit_kid.size(), in.first_kid.size(), in.first_read_id, in.n_sdk,
                                     in.windows, in.reads_hit};
    std::vector<uint64_t> all(mine.size() * P);
    x.allgather(mine.data(), mine.size() * 8, all.data());
    auto at = [&](int r, int i) { return all[(size_t)r * mine.size() + i]; };
    std::vector<uint64_t> read_off(P + 1, 0), hit_off(P + 1, 0), first_off(P + 1, 0);
    bool ok = true;
    for (int r = 0; r < P; ++r) {
        read_off[r + 1] = read_off[r] + at(r, 0);
        hit_off[r + 1] = hit_off[r] + at(r, 1);
        first_off[r + 1] = first_off[r] + at(r, 2);
        ok = ok && at(r, 4) == at(0, 4) && at(r, 3) == at(0, 3) + read_off[r];
    }
    if (!ok) return false;
    const int me = x.rank;
    std::vector<uint64_t> hp(in.n), fp(in.n);
    for (uint64_t i = 0; i < in.n; ++i) {
        hp[i] = in.hit_ptr[i + 1] + hit_off[me];
        fp[i] = in.first_ptr[i + 1] + first_off[me];
    }
    std::vector<uint32_t> kr(in.kci_read);
    for (auto& v : kr) v += (uint32_t)read_off[me];
    out = CsrIndex();
    out.n = read_off[P];
    out.first_read_id = (uint32_t)at(0, 3);
    out.n_sdk = (uint32_t)at(0, 4);
    for (int r = 0; r < P; ++r) {
        out.windows += at(r, 5);
        out.reads_hit += at(r, 6);
    }
    out.hit_ptr = concat(x, hp);
    out.hit_ptr.insert(out.hit_ptr.begin(), 0);
    out.first_ptr = concat(x, fp);
    out.first_ptr.insert(out.first_ptr.begin(), 0);
    out.hit_kid = concat(x, in.hit_kid);
    out.hit_pos = concat(x, in.hit_pos);
    out.sorted_kid = concat(x, in.sorted_kid);
    out.first_kid = concat(x, in.first_kid);
    out.first_pos = concat(x, in.first_pos);
    const std::vector<uint64_t> kps = concat(x, in.kci_ptr);   // P blocks of K+1
    const std::vector<uint32_t> krs = concat(x, kr);           // P blocks of H_r
    const uint64_t K = out.n_sdk;
    out.kci_ptr.assign(K + 1, 0);
    for (int r = 0; r < P; ++r)
        for (uint64_t i = 0; i < K; ++i) out.kci_ptr[i + 1] += kps[r * (K + 1) + i + 1] - kps[r * (K + 1) + i];
    for (uint64_t i = 0; i < K; ++i) out.kci_ptr[i + 1] += out.kci_ptr[i];
    out.kci_read.resize(out.kci_ptr[K]);
    for (uint64_t i = 0; i < K; ++i) {
        uint64_t o = out.kci_ptr[i];
        for (int r = 0; r < P; ++r) {
            const uint64_t a = kps[r * (K + 1) + i], b = kps[r * (K + 1) + i + 1];
            for (uint64_t j = a; j < b; ++j) out.kci_read[o++] = krs[hit_off[r] + j];
        }
    }
    return true;
}

// Connections of every rank's own pivots (each rank's list already in the reference order: score
// descending, ties by (pivot, candidate), ReadClusteringEngine.cpp:331) merged into the global list.
struct ConnList {
    std::vector<uint32_t> x, y;
    std::vector<uint64_t> s;
    std::vector<uint8_t> g;
};
inline ConnList merge_connections(Xport& xp, const ConnList& in) {
    const std::vector<uint64_t> cnt = concat(xp, std::vector<uint64_t>{in.x.size()});
    const std::vector<uint32_t> X = concat(xp, in.x), Y = concat(xp, in.y);
    const std::vector<uint64_t> S = concat(xp, in.s);
    const std::vector<uint8_t> G = concat(xp, in.g);
    const int P = xp.nranks;
    std::vector<uint64_t> pos(P, 0), end(P, 0);
    for (int r = 0; r < P; ++r) {
        pos[r] = r ? end[r - 1] : 0;
        end[r] = pos[r] + cnt[r];
    }
    auto before = [&](uint64_t a, uint64_t b) {   // (score desc, x, y)
        if (S[a] != S[b]) return S[a] > S[b];
        if (X[a] != X[b]) return X[a] < X[b];
        return Y[a] < Y[b];
    };
    ConnList out;
    const uint64_t N = X.size();
    out.x.reserve(N);
    out.y.reserve(N);
    out.s.reserve(N);
    out.g.reserve(N);
    while (true) {
        int best = -1;
        for (int r = 0; r < P; ++r)
            if (pos[r] < end[r] && (best < 0 || before(pos[r], pos[best]))) best = r;
        if (best < 0) break;
        const uint64_t i = pos[best]++;
        out.x.push_back(X[i]);
        out.y.push_back(Y[i]);
        out.s.push_back(S[i]);
        out.g.push_back(G[i]);
    }
    return out;
}

}  // namespace proto
}  // namespace hga
