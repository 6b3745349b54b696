// lookup.hip — MI355X replacement for the per-read SDK lookup loop of
// ReadClusteringEngine::construct_indices (src/clustering/ReadClusteringEngine.cpp:234-299).
//
//   lk_pack (pack_kernel<REF>)  reads -> 2-bit codes with KmerIterator semantics (non-ACGT
//                 contributes 0 to both strands, KmerIterator.cpp:7-19,54-63) + valid bits.
//   lk_starts     read-start bitmap (1 bit per base): a window is in one read iff no read
//                 starts inside (start, end].
//   lk_build      bucketised read-only table {canonical code -> KmerID} (8 keys per 64-B
//                 line) and a blocked Bloom filter (one u64 per key, ~11 bits/key) small
//                 enough to stay in every XCD's L2.  KmerIDs come from the host
//                 (std::unordered_set order, ReadClusteringEngine.cpp:237-241).
//   lk_scan<0>    32 window ends per thread from packed frames: closed-form canonical
//                 codes, filter, table probe on filter pass; per-thread hit mask + tile counts.
//   lk_scan<1>    threads with hits re-probe only their hits and write (read, KmerID,
//                 end-exclusive position) at block-scanned offsets: read / window order.
//   post          CSR pointers, stable radix sorts for the per-read sorted KmerID lists
//                 (:272) and first positions (:267), and kmer_component_index (:282-284).
#include <algorithm>

#include "hga_internal.hpp"
#include "kmer_dev.hpp"

namespace hga {
namespace {

constexpr int LK_T = 256;
constexpr int LK_P = 32;                  // window ends per thread (frame of 4 words)
constexpr uint64_t EMPTY_KEY = ~0ull;     // never canonical: min(fwd, rc) of all-T is 0
constexpr int BKT = 8;                    // keys per table bucket (one 64-B line)
constexpr int SB_PAD = 1;                 // leading zero words of the read-start bitmap

__device__ __forceinline__ uint64_t tab_hash(uint64_t x) {
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 32;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}
__device__ __forceinline__ uint64_t bloom_bits(uint64_t h) {
    return (1ull << ((h >> 40) & 63)) | (1ull << ((h >> 46) & 63)) | (1ull << ((h >> 52) & 63)) |
           (1ull << ((h >> 58) & 63));
}

__global__ void lk_fill(uint64_t* __restrict__ k, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) k[i] = EMPTY_KEY;
}

__global__ void lk_build(const uint64_t* __restrict__ keys, uint32_t n, uint64_t* __restrict__ tk,
                         uint32_t* __restrict__ tid, uint64_t bmask, unsigned long long* __restrict__ filt,
                         uint64_t fmask) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t key = keys[i];
    const uint64_t h = tab_hash(key);
    atomicOr(&filt[h & fmask], (unsigned long long)bloom_bits(h));
    uint64_t b = (h >> 20) & bmask;
    while (true) {
        for (int s = 0; s < BKT; ++s) {
            const unsigned long long old = atomicCAS((unsigned long long*)&tk[b * BKT + s],
                                                     (unsigned long long)EMPTY_KEY, (unsigned long long)key);
            if (old == EMPTY_KEY || old == key) {
                tid[b * BKT + s] = i;
                return;
            }
        }
        b = (b + 1) & bmask;
    }
}

// Table probe: KmerID or -1.
__device__ __forceinline__ int64_t lk_probe(const uint64_t* __restrict__ tk, const uint32_t* __restrict__ tids,
                                            uint64_t bmask, uint64_t key, uint64_t h) {
    uint64_t b = (h >> 20) & bmask;
    while (true) {
        const uint4* line = reinterpret_cast<const uint4*>(tk + b * BKT);
        bool any_empty = false;
#pragma unroll
        for (int q = 0; q < BKT / 2; ++q) {
            const uint4 v = line[q];
            const uint64_t k0 = ((uint64_t)v.y << 32) | v.x, k1 = ((uint64_t)v.w << 32) | v.z;
            if (k0 == key) return tids[b * BKT + 2 * q];
            if (k1 == key) return tids[b * BKT + 2 * q + 1];
            any_empty |= (k0 == EMPTY_KEY) | (k1 == EMPTY_KEY);
        }
        if (any_empty) return -1;
        b = (b + 1) & bmask;
    }
}

__global__ void lk_starts(const uint64_t* __restrict__ offs, uint64_t nreads, uint64_t nbases,
                          unsigned int* __restrict__ sb) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nreads) return;
    const uint64_t p = offs[r];
    if (p < nbases) atomicOr(&sb[SB_PAD + p / 32], 1u << (p & 31));
}

struct LkTab {
    const uint64_t* tk;
    const uint32_t* tid;
    const unsigned long long* filt;
    uint64_t bmask, fmask;
};

// Canonical code of the window ending at p0+j (j compile-time after unrolling).
__device__ __forceinline__ uint64_t lk_canon(const Frame<LK_P>& f, int j, uint64_t mask) {
    constexpr int NW = Frame<LK_P>::NW;
    const uint64_t fwd = field64<NW>(f.x, 2 * (16 * NW - 33 - j)) & mask;
    const uint64_t rc = field64<NW>(f.r, 2 * j) & mask;
    return fwd < rc ? fwd : rc;
}

// Same for a runtime j: word selects by compare chains (no dynamic register indexing).
__device__ __forceinline__ uint32_t lk_sel(const uint32_t (&x)[Frame<LK_P>::NW], int i) {
    uint32_t v = 0;
#pragma unroll
    for (int t = 0; t < Frame<LK_P>::NW; ++t) v = i == t ? x[t] : v;
    return v;
}
__device__ __forceinline__ uint64_t lk_field_rt(const uint32_t (&x)[Frame<LK_P>::NW], int sh) {
    constexpr int NW = Frame<LK_P>::NW;
    const int wb = sh >> 5, b = sh & 31;
    const uint32_t a0 = lk_sel(x, NW - 1 - wb), a1 = lk_sel(x, NW - 2 - wb), a2 = lk_sel(x, NW - 3 - wb);
    return ((uint64_t)__builtin_amdgcn_alignbit(a2, a1, b) << 32) | __builtin_amdgcn_alignbit(a1, a0, b);
}
__device__ __forceinline__ uint64_t lk_canon_rt(const Frame<LK_P>& f, int j, uint64_t mask) {
    constexpr int NW = Frame<LK_P>::NW;
    const uint64_t fwd = lk_field_rt(f.x, 2 * (16 * NW - 33 - j)) & mask;
    const uint64_t rc = lk_field_rt(f.r, 2 * j) & mask;
    return fwd < rc ? fwd : rc;
}

constexpr int LK_FB = 16;   // filter words in flight per thread
constexpr int LK_PB = 4;    // table lines in flight per thread

// Up to LK_PB table probes with their first bucket line loaded together; a line without the
// key but with an empty slot ends the probe, a full line (rare) falls back to lk_probe.
__device__ __forceinline__ void lk_probe_batch(const LkTab& tab, const uint64_t (&key)[LK_PB], uint32_t live,
                                               int64_t (&id)[LK_PB]) {
    uint64_t b[LK_PB];
    uint4 ln[LK_PB][BKT / 2];
#pragma unroll
    for (int q = 0; q < LK_PB; ++q) {
        b[q] = (tab_hash(key[q]) >> 20) & tab.bmask;
        if ((live >> q) & 1u) {
            const uint4* line = reinterpret_cast<const uint4*>(tab.tk + b[q] * BKT);
#pragma unroll
            for (int t = 0; t < BKT / 2; ++t) ln[q][t] = line[t];
        }
    }
#pragma unroll
    for (int q = 0; q < LK_PB; ++q) {
        id[q] = -1;
        if (!((live >> q) & 1u)) continue;
        bool any_empty = false;
        int slot = -1;
#pragma unroll
        for (int t = 0; t < BKT / 2; ++t) {
            const uint64_t k0 = ((uint64_t)ln[q][t].y << 32) | ln[q][t].x;
            const uint64_t k1 = ((uint64_t)ln[q][t].w << 32) | ln[q][t].z;
            slot = k0 == key[q] ? 2 * t : slot;
            slot = k1 == key[q] ? 2 * t + 1 : slot;
            any_empty |= (k0 == EMPTY_KEY) | (k1 == EMPTY_KEY);
        }
        if (slot >= 0) id[q] = tab.tid[b[q] * BKT + slot];
        else if (!any_empty) id[q] = lk_probe(tab.tk, tab.tid, tab.bmask, key[q], tab_hash(key[q]));
    }
}

template <bool EMIT>
__global__ void __launch_bounds__(LK_T) lk_scan(const uint32_t* __restrict__ pk, const uint16_t* __restrict__ vd,
                                                const unsigned int* __restrict__ sb, uint64_t nbases,
                                                const uint64_t* __restrict__ offs, uint64_t nreads, int k,
                                                LkTab tab, uint32_t* __restrict__ hmask,
                                                unsigned long long* __restrict__ tile_cnt,
                                                uint32_t* __restrict__ h_read, uint32_t* __restrict__ h_kid,
                                                uint32_t* __restrict__ h_pos) {
    __shared__ uint32_t ws[LK_T / 64 + 1];
    const uint64_t gt = (uint64_t)blockIdx.x * LK_T + threadIdx.x;
    const uint64_t p0 = gt * LK_P;
    const uint64_t mask = k >= 32 ? ~0ull : ((1ull << (2 * k)) - 1);
    if (!EMIT) {
        uint32_t hits = 0;
        if (p0 < nbases) {
            Frame<LK_P> f;
            (void)load_frame<LK_P, true>(pk, vd, PAD_WORDS + p0 / 16 - 2, k, f);
            const uint64_t s64 = (uint64_t)sb[SB_PAD + p0 / 32 - 1] | ((uint64_t)sb[SB_PAD + p0 / 32] << 32);
            uint32_t wm = (uint32_t)(runs_of(~s64, k - 1) >> 32);   // no read start in (s, e]
            const uint64_t left = nbases - p0;
            if (left < 32) wm &= (1u << left) - 1u;
            // 1) filter words, LK_FB in flight
            uint32_t cand = 0;
#pragma unroll
            for (int j0 = 0; j0 < LK_P; j0 += LK_FB) {
                uint32_t bits[LK_FB];
                uint64_t fw[LK_FB];
#pragma unroll
                for (int j = 0; j < LK_FB; ++j) {
                    const uint64_t h = tab_hash(lk_canon(f, j0 + j, mask));
                    bits[j] = (uint32_t)(h >> 40);
                    fw[j] = ((wm >> (j0 + j)) & 1u) ? tab.filt[h & tab.fmask] : 0ull;
                }
#pragma unroll
                for (int j = 0; j < LK_FB; ++j) {
                    const uint32_t x = bits[j];
                    const uint64_t bb = (1ull << (x & 63)) | (1ull << ((x >> 6) & 63)) |
                                        (1ull << ((x >> 12) & 63)) | (1ull << ((x >> 18) & 63));
                    if ((fw[j] & bb) == bb && ((wm >> (j0 + j)) & 1u)) cand |= 1u << (j0 + j);
                }
            }
            // 2) table probes for the filter passes, LK_PB lines in flight
            while (cand) {
                uint64_t key[LK_PB];
                int jj[LK_PB];
                uint32_t live = 0;
#pragma unroll
                for (int q = 0; q < LK_PB; ++q) {
                    jj[q] = cand ? __builtin_ctz(cand) : 0;
                    if (cand) { live |= 1u << q; cand &= cand - 1u; }
                    key[q] = lk_canon_rt(f, jj[q], mask);
                }
                int64_t id[LK_PB];
                lk_probe_batch(tab, key, live, id);
#pragma unroll
                for (int q = 0; q < LK_PB; ++q)
                    if (((live >> q) & 1u) && id[q] >= 0) hits |= 1u << jj[q];
            }
            hmask[gt] = hits;
        }
        uint32_t tot;
        (void)block_excl_scan<LK_T>((uint32_t)__popc(hits), ws, &tot);
        if (threadIdx.x == 0) tile_cnt[blockIdx.x] = tot;
        return;
    }
    uint32_t hits = p0 < nbases ? hmask[gt] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan<LK_T>((uint32_t)__popc(hits), ws, &tot);
    if (!hits) return;
    uint64_t o = tile_cnt[blockIdx.x] + ex;
    Frame<LK_P> f;
    (void)load_frame<LK_P, true>(pk, vd, PAD_WORDS + p0 / 16 - 2, k, f);
    // read containing p0: last r with offs[r] <= p0
    uint64_t lo = 0, hi = nreads;
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (offs[mid] <= p0) lo = mid; else hi = mid;
    }
    uint64_t r = lo, re = offs[r + 1];
    while (hits) {
        uint64_t key[LK_PB];
        int jj[LK_PB];
        uint32_t live = 0;
#pragma unroll
        for (int q = 0; q < LK_PB; ++q) {
            jj[q] = hits ? __builtin_ctz(hits) : 0;
            if (hits) { live |= 1u << q; hits &= hits - 1u; }
            key[q] = lk_canon_rt(f, jj[q], mask);
        }
        int64_t id[LK_PB];
        lk_probe_batch(tab, key, live, id);
#pragma unroll
        for (int q = 0; q < LK_PB; ++q) {
            if (!((live >> q) & 1u)) continue;
            const uint64_t e = p0 + jj[q];
            while (re <= e) re = offs[++r + 1];
            h_read[o] = (uint32_t)r;
            h_kid[o] = (uint32_t)id[q];
            h_pos[o] = (uint32_t)(e + 1 - offs[r]);
            ++o;
        }
    }
}

// ptr[s] = first index i with idx[i] >= s (CSR over a sorted segment-id array), ptr[nseg] = H.
__global__ void lk_ptr(const uint32_t* __restrict__ idx, uint64_t H, uint64_t nseg,
                       uint64_t* __restrict__ ptr) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > H) return;
    const uint64_t lo = i == 0 ? 0 : (uint64_t)idx[i - 1] + 1;
    const uint64_t hi = i == H ? nseg : (uint64_t)idx[i];
    for (uint64_t s = lo; s <= hi; ++s) ptr[s] = i;
}

// Number of non-empty CSR segments (one atomic per 1024 segments).
__global__ void __launch_bounds__(1024) lk_nonempty(const uint64_t* __restrict__ ptr, uint64_t nseg,
                                                    unsigned long long* __restrict__ out) {
    __shared__ uint32_t ws[1024 / 64 + 1];
    const uint64_t s = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    const uint32_t v = s < nseg && ptr[s + 1] > ptr[s] ? 1u : 0u;
    uint32_t tot;
    (void)block_excl_scan<1024>(v, ws, &tot);
    if (threadIdx.x == 0 && tot) atomicAdd(out, (unsigned long long)tot);
}

__global__ void lk_compose(const uint32_t* __restrict__ rd, const uint32_t* __restrict__ kid,
                           const uint32_t* __restrict__ pos, uint64_t H, int kbits,
                           uint64_t* __restrict__ key, uint32_t* __restrict__ val) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= H) return;
    key[i] = ((uint64_t)rd[i] << kbits) | kid[i];
    val[i] = pos[i];
}

__global__ void lk_first_flags(const uint64_t* __restrict__ key, uint64_t H, uint64_t* __restrict__ flag,
                               uint32_t* __restrict__ sorted_kid, uint64_t kmask) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= H) return;
    flag[i] = (i == 0 || key[i] != key[i - 1]) ? 1ull : 0ull;
    sorted_kid[i] = (uint32_t)(key[i] & kmask);
}

__global__ void lk_first_scatter(const uint64_t* __restrict__ key, const uint32_t* __restrict__ pos,
                                 const uint64_t* __restrict__ off, uint64_t H, int kbits,
                                 uint64_t kmask, uint32_t* __restrict__ fk, uint32_t* __restrict__ fp,
                                 uint32_t* __restrict__ fr) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= H) return;
    if (i == 0 || key[i] != key[i - 1]) {
        const uint64_t o = off[i];
        fk[o] = (uint32_t)(key[i] & kmask);
        fp[o] = pos[i];
        fr[o] = (uint32_t)(key[i] >> kbits);
    }
}

inline unsigned blocks_for(uint64_t n, int t) { return (unsigned)((n + t - 1) / t); }
inline int bits_for(uint64_t n) {   // bits to hold values in [0, n)
    int b = 0;
    while (b < 64 && (n - 1) >> b) ++b;
    return b < 1 ? 1 : b;
}

}  // namespace

void lookup_load(hga_ctx* c, int k, const uint64_t* keys, uint32_t n) {
    HGA_REQUIRE(k >= 1 && k <= 32, HGA_ERR_INVALID, "k must be in [1,32]");
    auto& L = c->lookup;
    uint64_t nbk = 128;
    while (nbk * BKT < 2ull * n) nbk <<= 1;            // <= 50 % slot load
    uint64_t fw = 1024;
    while (fw * 64 < 11ull * n) fw <<= 1;               // >= 11 filter bits per key
    L.slots = nbk * BKT;
    L.fwords = fw;
    L.k = k;
    L.n_sdk = n;
    uint64_t* tk = static_cast<uint64_t*>(L.tab_key.ensure(L.slots * 8));
    uint32_t* ti = static_cast<uint32_t*>(L.tab_id.ensure(L.slots * 4));
    auto* filt = static_cast<unsigned long long*>(L.filter.ensure(fw * 8));
    DevBuf tmp;
    uint64_t* dk = static_cast<uint64_t*>(tmp.ensure(std::max<uint64_t>(n, 1) * 8));
    if (n) HGA_HIP(hipMemcpyAsync(dk, keys, (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(lk_fill, dim3(blocks_for(L.slots, 256)), dim3(256), 0, c->stream, tk, L.slots);
    c->check_launch("lk_fill");
    HGA_HIP(hipMemsetAsync(filt, 0, fw * 8, c->stream));
    if (n) {
        c->launch("lk_build", [&] {
            hipLaunchKernelGGL(lk_build, dim3(blocks_for(n, 256)), dim3(256), 0, c->stream, dk, n, tk, ti, nbk - 1,
                               filt, fw - 1);
        });
        c->check_launch("lk_build");
    }
    c->sync();
    L.loaded = true;
    L.ran = false;
}

void lookup_set_reads(hga_ctx* c, const char* bases, const uint64_t* offsets, uint64_t n,
                      uint32_t first_id) {
    auto& L = c->lookup;
    HGA_REQUIRE(n < (1ull << 32), HGA_ERR_INVALID, "too many reads");
    HGA_REQUIRE(offsets[0] == 0 || n == 0, HGA_ERR_INVALID, "offsets[0] must be 0");
    for (uint64_t i = 0; i < n; ++i)
        HGA_REQUIRE(offsets[i + 1] >= offsets[i], HGA_ERR_INVALID, "offsets must be non-decreasing");
    const uint64_t nb = n ? offsets[n] - offsets[0] : 0;
    L.n_reads = n;
    L.n_bases = nb;
    L.first_read_id = first_id;
    void* db = L.bases.ensure(nb + 16);
    void* dof = L.offsets.ensure((n + 1) * 8);
    if (nb) HGA_HIP(hipMemcpyAsync(db, bases, nb, hipMemcpyHostToDevice, c->stream));
    HGA_HIP(hipMemcpyAsync(dof, offsets, (n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    // packed codes (KmerIterator semantics), valid bits, read-start bitmap
    const uint64_t nw = (nb + 15) / 16, tail = 64;
    L.pk_words = PAD_WORDS + nw + tail;
    uint32_t* pk = static_cast<uint32_t*>(L.packed.ensure(L.pk_words * 4));
    uint16_t* vd = static_cast<uint16_t*>(L.valid.ensure(L.pk_words * 2));
    HGA_HIP(hipMemsetAsync(pk, 0, L.pk_words * 4, c->stream));
    HGA_HIP(hipMemsetAsync(vd, 0, L.pk_words * 2, c->stream));
    const uint64_t sbw = SB_PAD + (nb + 31) / 32 + tail;
    unsigned int* sb = static_cast<unsigned int*>(L.starts.ensure(sbw * 4));
    HGA_HIP(hipMemsetAsync(sb, 0, sbw * 4, c->stream));
    if (nw)
        hipLaunchKernelGGL(pack_kernel<true>, dim3(blocks_for(nw, 256)), dim3(256), 0, c->stream,
                           static_cast<const uint8_t*>(db), nb, pk, vd, nw);
    if (n)
        hipLaunchKernelGGL(lk_starts, dim3(blocks_for(n, 256)), dim3(256), 0, c->stream,
                           static_cast<const uint64_t*>(dof), n, nb, sb);
    c->check_launch("lk_pack");
    c->sync();
    L.h_offsets.assign(offsets, offsets + n + 1);
    L.have_reads = true;
    L.ran = false;
}

void lookup_run(hga_ctx* c) {
    auto& L = c->lookup;
    HGA_REQUIRE(L.loaded, HGA_ERR_STATE, "hga_lookup_load not called");
    HGA_REQUIRE(L.have_reads, HGA_ERR_STATE, "hga_lookup_set_reads not called");
    const uint64_t n = L.n_reads, nb = L.n_bases;
    const int k = L.k;
    uint64_t w = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t len = L.h_offsets[i + 1] - L.h_offsets[i];
        if (len >= (uint64_t)k) w += len - k + 1;
    }
    L.windows = w;
    L.hits = L.firsts = L.reads_hit = 0;
    const uint64_t n_threads = (nb + LK_P - 1) / LK_P;
    const uint64_t n_tiles = (n_threads + LK_T - 1) / LK_T;
    uint32_t* hm = static_cast<uint32_t*>(L.scratch.ensure(std::max<uint64_t>(n_threads, 1) * 4 + 256));
    auto* tile = static_cast<unsigned long long*>(L.tile_cnt.ensure((n_tiles + 1) * 8));
    const uint32_t* pk = L.packed.as<uint32_t>();
    const uint16_t* vd = L.valid.as<uint16_t>();
    const unsigned int* sb = L.starts.as<unsigned int>();
    const uint64_t* offs = L.offsets.as<uint64_t>();
    LkTab tab{L.tab_key.as<uint64_t>(), L.tab_id.as<uint32_t>(), L.filter.as<unsigned long long>(),
              L.slots / BKT - 1, L.fwords - 1};
    uint64_t H = 0;
    if (n_tiles) {
        c->launch("lk_count", [&] {
            hipLaunchKernelGGL(lk_scan<false>, dim3((unsigned)n_tiles), dim3(LK_T), 0, c->stream, pk, vd, sb, nb,
                               offs, n, k, tab, hm, tile, (uint32_t*)nullptr, (uint32_t*)nullptr,
                               (uint32_t*)nullptr);
        });
        c->check_launch("lk_count");
        HGA_HIP(hipMemsetAsync(tile + n_tiles, 0, 8, c->stream));
        exclusive_scan_u64(c, reinterpret_cast<uint64_t*>(tile), n_tiles + 1, L.scratch3);
        HGA_HIP(hipMemcpyAsync(&H, tile + n_tiles, 8, hipMemcpyDeviceToHost, c->stream));
        c->sync();
    }
    L.hits = H;
    uint32_t* hr = static_cast<uint32_t*>(L.hit_read.ensure(std::max<uint64_t>(H, 1) * 4));
    uint32_t* hk = static_cast<uint32_t*>(L.hit_kid.ensure(std::max<uint64_t>(H, 1) * 4));
    uint32_t* hp = static_cast<uint32_t*>(L.hit_pos.ensure(std::max<uint64_t>(H, 1) * 4));
    if (H) {
        c->launch("lk_emit", [&] {
            hipLaunchKernelGGL(lk_scan<true>, dim3((unsigned)n_tiles), dim3(LK_T), 0, c->stream, pk, vd, sb, nb,
                               offs, n, k, tab, hm, tile, hr, hk, hp);
        });
        c->check_launch("lk_emit");
    }
    // hit_ptr over reads
    auto* ctr = static_cast<unsigned long long*>(L.first_flag.ensure(64));
    HGA_HIP(hipMemsetAsync(ctr, 0, 32, c->stream));
    uint64_t* hptr = static_cast<uint64_t*>(L.hit_ptr.ensure((n + 1) * 8));
    c->launch("lk_post", [&] {
        hipLaunchKernelGGL(lk_ptr, dim3(blocks_for(H + 1, 256)), dim3(256), 0, c->stream, hr, H, n, hptr);
        if (n)
            hipLaunchKernelGGL(lk_nonempty, dim3(blocks_for(n, 1024)), dim3(1024), 0, c->stream, hptr, n, ctr);
    });
    c->check_launch("lk_ptr");
    const int kbits = bits_for(std::max<uint32_t>(L.n_sdk, 1));
    const int rbits = bits_for(std::max<uint64_t>(n, 1));
    const uint64_t kmask = (1ull << kbits) - 1;
    uint64_t U = 0;
    if (H) {
        // per-read (read, KmerID) sort, positions as payload (stable: window order kept)
        uint64_t* sk = static_cast<uint64_t*>(L.s_key.ensure(H * 8));
        uint32_t* sv = static_cast<uint32_t*>(L.s_val.ensure(H * 4));
        c->launch("lk_post", [&] {
            hipLaunchKernelGGL(lk_compose, dim3(blocks_for(H, 256)), dim3(256), 0, c->stream, hr, hk, hp, H,
                               kbits, sk, sv);
        });
        radix_sort_u64(c, sk, sv, H, kbits + rbits, L.scratch2);
        uint64_t* flag = static_cast<uint64_t*>(L.s_key2.ensure((H + 1) * 8));
        uint32_t* skid = static_cast<uint32_t*>(L.s_val2.ensure(H * 4));
        c->launch("lk_post", [&] {
            hipLaunchKernelGGL(lk_first_flags, dim3(blocks_for(H, 256)), dim3(256), 0, c->stream, sk, H, flag,
                               skid, kmask);
        });
        HGA_HIP(hipMemsetAsync(flag + H, 0, 8, c->stream));
        exclusive_scan_u64(c, flag, H + 1, L.scratch3);
        HGA_HIP(hipMemcpyAsync(&U, flag + H, 8, hipMemcpyDeviceToHost, c->stream));
        c->sync();
        uint32_t* fk = static_cast<uint32_t*>(L.first_kid.ensure(U * 4));
        uint32_t* fp = static_cast<uint32_t*>(L.first_pos.ensure(U * 4));
        uint32_t* fr = static_cast<uint32_t*>(L.first_read.ensure(U * 4));
        c->launch("lk_post", [&] {
            hipLaunchKernelGGL(lk_first_scatter, dim3(blocks_for(H, 256)), dim3(256), 0, c->stream, sk, sv, flag,
                               H, kbits, kmask, fk, fp, fr);
        });
        // kmer_component_index: stable sort of the read-ordered hits by KmerID
        uint32_t* kk = static_cast<uint32_t*>(L.kci_key.ensure(H * 4));
        uint32_t* kv = static_cast<uint32_t*>(L.kci_val.ensure(H * 4));
        HGA_HIP(hipMemcpyAsync(kk, hk, H * 4, hipMemcpyDeviceToDevice, c->stream));
        HGA_HIP(hipMemcpyAsync(kv, hr, H * 4, hipMemcpyDeviceToDevice, c->stream));
        radix_sort_u32(c, kk, kv, H, kbits, L.scratch2);
    }
    L.firsts = U;
    uint64_t* fptr = static_cast<uint64_t*>(L.first_ptr.ensure((n + 1) * 8));
    uint64_t* kptr = static_cast<uint64_t*>(L.kci_ptr.ensure(((uint64_t)L.n_sdk + 1) * 8));
    c->launch("lk_post", [&] {
        hipLaunchKernelGGL(lk_ptr, dim3(blocks_for(U + 1, 256)), dim3(256), 0, c->stream,
                           U ? L.first_read.as<uint32_t>() : (const uint32_t*)nullptr, U, n, fptr);
        hipLaunchKernelGGL(lk_ptr, dim3(blocks_for(H + 1, 256)), dim3(256), 0, c->stream,
                           H ? L.kci_key.as<uint32_t>() : (const uint32_t*)nullptr, H, (uint64_t)L.n_sdk, kptr);
    });
    c->check_launch("lk_ptr");
    unsigned long long hc[4];
    HGA_HIP(hipMemcpyAsync(hc, ctr, 32, hipMemcpyDeviceToHost, c->stream));
    c->sync();
    L.reads_hit = hc[0];
    L.ran = true;
}

void lookup_sizes(hga_ctx* c, hga_lookup_sizes* out) {
    auto& L = c->lookup;
    out->n_reads = L.n_reads;
    out->windows = L.windows;
    out->hits = L.ran ? L.hits : 0;
    out->firsts = L.ran ? L.firsts : 0;
    out->reads_hit = L.ran ? L.reads_hit : 0;
    out->n_sdk = L.n_sdk;
}

void lookup_fetch(hga_ctx* c, const hga_lookup_result* o) {
    auto& L = c->lookup;
    HGA_REQUIRE(L.ran, HGA_ERR_STATE, "hga_lookup_run not called");
    const uint64_t n = L.n_reads, H = L.hits, U = L.firsts, K = L.n_sdk;
    auto cp = [&](void* dst, const DevBuf& src, size_t bytes) {
        if (dst && bytes) HGA_HIP(hipMemcpyAsync(dst, src.p, bytes, hipMemcpyDeviceToHost, c->stream));
    };
    cp(o->hit_ptr, L.hit_ptr, (n + 1) * 8);
    cp(o->hit_kid, L.hit_kid, H * 4);
    cp(o->hit_pos, L.hit_pos, H * 4);
    cp(o->sorted_kid, L.s_val2, H * 4);
    cp(o->first_ptr, L.first_ptr, (n + 1) * 8);
    cp(o->first_kid, L.first_kid, U * 4);
    cp(o->first_pos, L.first_pos, U * 4);
    cp(o->kci_ptr, L.kci_ptr, (K + 1) * 8);
    cp(o->kci_read, L.kci_val, H * 4);
    c->sync();
    if (o->kci_read)
        for (uint64_t i = 0; i < H; ++i) o->kci_read[i] += L.first_read_id;
}

}  // namespace hga
