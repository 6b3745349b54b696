// connect.hip — shared-k-mer connections between reads, the stage after construct_indices
// (SURVEY.md §8(f) rank 1): ReadClusteringEngine::get_connections / get_all_connections
// (src/clustering/ReadClusteringEngine.cpp:301-339) on the state construct_indices leaves,
// where every read with >= 1 hit is a one-read component whose discriminative_kmer_ids are
// its sorted KmerIDs WITH duplicates (:262-273) and kmer_component_index[id] lists the ReadIDs
// once per occurrence, sorted (:264-266, 282-284).
//
// For a pivot read p the reference counts, in a robin_map, every candidate c met while walking
// kmer_component_index[id] for every id of p (:311-315), erases p (:316) and keeps pairs with
// count >= min_score (:318-325): score(p, c) = sum over KmerIDs of mult_p(id) * mult_c(id), a
// sparse A·Aᵀ with multiplicities.  Output ordering: std::sort(rbegin, rend) by score (:331),
// i.e. descending; ties are unordered there (threads + unstable sort) and ordered here by
// (pivot, candidate) ascending, so the result is deterministic.
//
// Device work, one workgroup per pivot:
//   cn_local    LDS open-addressing table (CAP candidates); the pivot's hit list is walked in
//               chunks of 256 KmerIDs whose kmer_component_index lists are flattened with a
//               block scan, so every lane handles one (id, candidate) pair; survivors are
//               compacted with one global atomic per workgroup.  A pivot whose distinct
//               candidates pass 3/4 of CAP goes to the overflow list;
//   cn_global   the same walk over a per-pivot table in HBM for the overflow list;
//   cn_keys / radix sort / cn_decode
//               composite sort key (CAP-free): (max - score, pivot, candidate).
#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <vector>

#include "hga_internal.hpp"
#include "kmer_dev.hpp"

namespace hga {
namespace {

constexpr int CN_T = 256;
constexpr uint32_t CN_EMPTY = 0xFFFFFFFFu;

inline unsigned cn_blocks(uint64_t n, uint64_t t) { return (unsigned)((n + t - 1) / t); }

__device__ __forceinline__ uint32_t cn_hash(uint32_t x) { return (x * 0x9E3779B1u) ^ (x >> 15); }

// Table reads go through relaxed atomics: LDS reads either way, and for the HBM tables of
// cn_global they bypass non-coherent cached copies of lines other workgroup lanes update.
__device__ __forceinline__ uint32_t cn_ld(const uint32_t* p) { return __atomic_load_n(p, __ATOMIC_RELAXED); }

// Adds one occurrence of `cand` to the table; false when the table is full.
__device__ __forceinline__ bool cn_insert(uint32_t* tk, uint32_t* tv, uint32_t mask, uint32_t cand,
                                          uint32_t* fill, uint32_t limit, uint32_t* ovf) {
    uint32_t s = cn_hash(cand) & mask;
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        uint32_t k = cn_ld(&tk[s]);
        if (k == CN_EMPTY) {
            k = atomicCAS(&tk[s], CN_EMPTY, cand);
            if (k == CN_EMPTY) {
                if (atomicAdd(fill, 1u) + 1 >= limit) __atomic_store_n(ovf, 1u, __ATOMIC_RELAXED);
                atomicAdd(&tv[s], 1u);
                return true;
            }
        }
        if (k == cand) {
            atomicAdd(&tv[s], 1u);
            return true;
        }
        s = (s + 1) & mask;
    }
    __atomic_store_n(ovf, 1u, __ATOMIC_RELAXED);
    return false;
}

struct CnIn {
    const uint64_t* hit_ptr;   // per read, into skid
    const uint32_t* skid;      // sorted KmerIDs per read, with duplicates
    const uint64_t* kci_ptr;   // per KmerID, into kci
    const uint32_t* kci;       // read indices per KmerID, sorted, with duplicates
    uint32_t min_kmers, min_score;
    const uint32_t* slots;     // cn_wave: per KmerID one 128-B slot (cn_slots), or null
};

// kmer_component_index as one 128-B slot (one L2 line) per KmerID for cn_wave: word 0 = the list's
// length when it fits (<= SLOT_W - 1 read indices, in words 1..), else SLOT_LONG with the length in
// word 1 and the list's kci offset in words 2-3.  A hit's list then costs one aligned line fetch with
// no kci_ptr read before it (the pointer read and the list's line straddles made cn_wave fetch ~2x
// its model bytes), and the slot header arrives with the entries.
constexpr uint32_t SLOT_W = 32, SLOT_LONG = 0xFFFFFFFFu;
__global__ void __launch_bounds__(256) cn_slots(const uint64_t* __restrict__ kci_ptr, const uint32_t* __restrict__ kci,
                                                uint64_t K, uint32_t* __restrict__ slots) {
    const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= K) return;
    const uint64_t l0 = kci_ptr[k], len = kci_ptr[k + 1] - l0;
    uint32_t w[SLOT_W];
#pragma unroll
    for (uint32_t i = 0; i < SLOT_W; ++i) w[i] = 0;
    if (len < SLOT_W) {
        w[0] = (uint32_t)len;
#pragma unroll
        for (uint32_t i = 1; i < SLOT_W; ++i)
            if (i <= len) w[i] = kci[l0 + i - 1];
    } else {
        w[0] = SLOT_LONG;
        w[1] = (uint32_t)len;
        w[2] = (uint32_t)l0;
        w[3] = (uint32_t)(l0 >> 32);
    }
    uint4* dst = reinterpret_cast<uint4*>(slots + k * SLOT_W);
#pragma unroll
    for (uint32_t i = 0; i < SLOT_W / 4; ++i) dst[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

// Output: CN_R regions of rcap entries, each with its own cursor in its own 128-B line, so the
// per-pivot reservations spread over CN_R addresses instead of serialising on one.  Pivot p
// writes to region p % CN_R, so the region sizes do not depend on scheduling (an overflowing
// first attempt gives the exact size for the retry).
constexpr int CN_R = 64;
constexpr int CN_RSTRIDE = 16;             // u64 words between region cursors
struct CnOut {
    uint32_t *x, *y, *s;
    uint64_t rcap;                 // entries per region
    unsigned long long* ctr;       // [1] max score, [2] / [3] tier-2 / tier-3 pivots, [5] work
    unsigned long long* rcur;      // region cursors, stride CN_RSTRIDE
    uint64_t *pst, *pcnt;          // per pivot read: first output slot and pair count (null: unused)
};

// Reserves n entries in region r; returns the region-local offset (entries past rcap are
// counted but not written, and the host retries with the exact size).
__device__ __forceinline__ uint64_t cn_reserve(const CnOut& out, uint32_t r, uint32_t n) {
    return atomicAdd(&out.rcur[(uint64_t)r * CN_RSTRIDE], (unsigned long long)n);
}
// Records pivot p's output run (one reservation per pivot in every tier).
__device__ __forceinline__ void cn_note(const CnOut& out, uint32_t p, uint32_t r, uint64_t base, uint32_t n) {
    if (out.pcnt) {
        out.pst[p] = (uint64_t)r * out.rcap + base;
        out.pcnt[p] = n;
    }
}
__device__ __forceinline__ void cn_put(const CnOut& out, uint32_t r, uint64_t w, uint32_t x, uint32_t y, uint32_t sc) {
    if (w < out.rcap) {
        const uint64_t g = (uint64_t)r * out.rcap + w;
        out.x[g] = x;
        out.y[g] = y;
        out.s[g] = sc;
    }
}

// Walks pivot p's hit list into the table.  Returns false (uniformly) on overflow.
__device__ bool cn_walk(const CnIn& in, uint32_t p, uint64_t b, uint64_t e, uint32_t* tk, uint32_t* tv,
                        uint32_t mask, uint32_t limit, uint32_t* sh) {
    // sh: [0] fill, [1] ovf, [2..7] scan scratch, then lo[256] (u64 as 2 words) and off[257]
    uint32_t* ws = sh + 2;
    uint64_t* lo = reinterpret_cast<uint64_t*>(sh + 8);
    uint32_t* off = sh + 8 + 2 * CN_T;
    const uint32_t t = threadIdx.x;
    for (uint64_t cb = b; cb < e; cb += CN_T) {
        const uint64_t i = cb + t;
        uint32_t len = 0;
        uint64_t l0 = 0;
        if (i < e) {
            const uint32_t kid = in.skid[i];
            l0 = in.kci_ptr[kid];
            len = (uint32_t)(in.kci_ptr[kid + 1] - l0);
        }
        uint32_t T;
        const uint32_t o = block_excl_scan<CN_T>(len, ws, &T);
        lo[t] = l0;
        off[t] = o;
        if (t == 0) off[CN_T] = T;
        __syncthreads();
        for (uint32_t j = t; j < T; j += CN_T) {
            uint32_t a = 0, z = CN_T;   // last h with off[h] <= j
            while (z - a > 1) {
                const uint32_t m = (a + z) >> 1;
                if (off[m] <= j) a = m; else z = m;
            }
            const uint32_t cand = in.kci[lo[a] + (j - off[a])];
            if (cand != p && !cn_insert(tk, tv, mask, cand, &sh[0], limit, &sh[1])) break;
        }
        __syncthreads();
        if (__atomic_load_n(&sh[1], __ATOMIC_RELAXED)) return false;
    }
    return true;
}

// Compacts the table's surviving pairs into the output (one global atomic per workgroup).
__device__ void cn_emit(const CnIn& in, const CnOut& out, uint32_t p, const uint32_t* tk, const uint32_t* tv,
                        uint32_t size, uint32_t* ws) {
    const uint32_t per = size / CN_T;
    const uint32_t s0 = threadIdx.x * per;
    uint32_t cnt = 0, mx = 0;
    for (uint32_t s = s0; s < s0 + per; ++s) {
        const uint32_t v = cn_ld(&tv[s]);
        if (cn_ld(&tk[s]) != CN_EMPTY && v >= in.min_score) {
            ++cnt;
            mx = max(mx, v);
        }
    }
#pragma unroll
    for (int o = 32; o; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, o, 64));
    uint32_t total;
    const uint32_t pre = block_excl_scan<CN_T>(cnt, ws, &total);
    if (total == 0) return;
    __shared__ unsigned long long base_s;
    const uint32_t reg = p % CN_R;
    if (threadIdx.x == 0) {
        base_s = cn_reserve(out, reg, total);
        cn_note(out, p, reg, base_s, total);
    }
    if ((threadIdx.x & 63) == 0 && mx) atomicMax(&out.ctr[1], (unsigned long long)mx);
    __syncthreads();
    uint64_t w = base_s + pre;
    for (uint32_t s = s0; s < s0 + per && cnt; ++s) {
        const uint32_t v = cn_ld(&tv[s]);
        const uint32_t key = cn_ld(&tk[s]);
        if (key != CN_EMPTY && v >= in.min_score) {
            cn_put(out, reg, w, p, key, v);
            ++w;
            --cnt;
        }
    }
}

// ---- cn_local: the LDS path (every pivot whose distinct candidates fit 3/4 of CN_CAP).
// Table entries are one u64 (candidate in the low word, count in the high word), so a repeat
// is one ds_add_u64 and a new candidate one ds_cmpst_b64.  The table is sized per pivot from
// its (id, candidate) pair count (an upper bound of its distinct candidates), so short pivots
// clear and scan a small table.  Pairs of a chunk of 256 KmerIDs are assigned lane-strided
// (neighbouring lanes read neighbouring kmer_component_index words); the owner KmerID of each
// pair comes from an LDS owner map (segment starts + a block max-scan) instead of a per-pair
// binary search, and every lane issues its CN_U candidate loads before its inserts.
constexpr uint32_t CN_CAP = 2048;          // LDS table entries (16 KB)
constexpr uint32_t CN_W = 2048;            // pairs per owner-map window
constexpr int CN_U = CN_W / CN_T;          // pairs per lane per window
constexpr uint64_t CN_EMPTY64 = 0x00000000FFFFFFFFull;

__device__ __forceinline__ bool cn_insert64(uint64_t* t, uint32_t mask, uint32_t cand, uint32_t* fill, uint32_t limit,
                                            uint32_t* ovf) {
    uint32_t s = cn_hash(cand) & mask;
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        uint64_t v = __atomic_load_n(&t[s], __ATOMIC_RELAXED);
        if ((uint32_t)v == CN_EMPTY) {
            v = atomicCAS((unsigned long long*)&t[s], (unsigned long long)CN_EMPTY64,
                          (unsigned long long)((1ull << 32) | cand));
            if (v == CN_EMPTY64) {
                if (atomicAdd(fill, 1u) + 1 >= limit) __atomic_store_n(ovf, 1u, __ATOMIC_RELAXED);
                return true;
            }
        }
        if ((uint32_t)v == cand) {
            atomicAdd((unsigned long long*)&t[s], 1ull << 32);
            return true;
        }
        s = (s + 1) & mask;
    }
    __atomic_store_n(ovf, 1u, __ATOMIC_RELAXED);
    return false;
}

// ---- Candidate order of a pivot's run.  Every tier emits its pairs sorted by candidate, so the
// final order (score desc, pivot, candidate) is one stable pass over the score bits of the
// pivot-ordered runs.  Sort keys are candidate << 32 | score (candidates < 2^32 - 1), ~0 pads.
constexpr uint64_t CN_PAD = ~0ull;
constexpr uint32_t CN_SORT_W = 1024;   // runs up to this long are sorted by cn_runs_keys (one wave, 16 keys a lane)
constexpr uint32_t CN_SORT_N = 512;    // ... up to this long by its common launch (8 keys a lane)
__device__ __forceinline__ uint64_t cn_key(uint64_t ent) { return (ent << 32) | (ent >> 32); }

// Bitonic sort of tab[0, n) in LDS by the whole workgroup (n a power of two, <= CN_CAP).
__device__ void block_bitonic_sort(uint64_t* tab, uint32_t n) {
    for (uint32_t k = 2; k <= n; k <<= 1) {
        for (uint32_t j = k >> 1; j; j >>= 1) {
            for (uint32_t x = threadIdx.x; x < n / 2; x += CN_T) {
                const uint32_t i = 2 * x - (x & (j - 1)), q = i + j;
                const uint64_t a = tab[i], b = tab[q];
                const bool asc = (i & k) == 0;
                if (asc ? a > b : a < b) {
                    tab[i] = b;
                    tab[q] = a;
                }
            }
            __syncthreads();
        }
    }
}

// Inclusive max-scan of own[0..CN_W) in place (CN_U = 8 consecutive bytes per thread, one u64).
static_assert(CN_U == 8, "owner map: eight pairs (one u64 of bytes) per thread");
__device__ __forceinline__ void cn_owner_scan(uint8_t* own, uint32_t* ws) {
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    uint64_t* own64 = reinterpret_cast<uint64_t*>(own);
    const uint64_t ov = own64[t];
    uint32_t v[CN_U];
    uint32_t m = 0;
#pragma unroll
    for (int u = 0; u < CN_U; ++u) {
        m = max(m, (uint32_t)(ov >> (8 * u)) & 0xFFu);
        v[u] = m;
    }
    const uint32_t x = wave_scan_max_dpp(m);
    if (lane == 63) ws[wave] = x;
    __syncthreads();
    uint32_t pre = dpp_take<0x138, 0xf>(x);   // wave_shr:1: the max over earlier lanes
    for (uint32_t w = 0; w < wave; ++w) pre = max(pre, ws[w]);
    uint64_t nv = 0;
#pragma unroll
    for (int u = 0; u < CN_U; ++u) nv |= (uint64_t)max(pre, v[u]) << (8 * u);
    own64[t] = nv;
    __syncthreads();
}

struct CnBlockLds {
    uint64_t tab[CN_CAP];
    uint64_t lo[CN_T];   // per hit of the chunk: kci offset of its list minus its first pair index
    uint32_t sh[12];   // [0] fill, [1] ovf, [2..] scan scratch, [11] next listed pivot
    alignas(8) uint8_t own[CN_W];
    unsigned long long base_s;
};

// Pivot p by the whole workgroup (every thread calls it; the return is uniform).  False when its
// distinct candidates passed `limit`: nothing was emitted and the caller lists p for the next tier.
__device__ bool cn_block_pivot(const CnIn& in, const CnOut& out, uint32_t p, uint32_t limit, CnBlockLds& L) {
    const uint32_t t = threadIdx.x;
    __syncthreads();   // the previous pivot's table reads are done
    const uint64_t b = in.hit_ptr[p], e = in.hit_ptr[p + 1];
    if (e - b < (uint64_t)in.min_kmers || e == b) return true;
    // pair count -> table size (>= 2 x distinct candidates when it fits)
    uint64_t acc = 0;
    for (uint64_t i = b + t; i < e; i += CN_T) {
        const uint32_t kid = in.skid[i];
        acc += in.kci_ptr[kid + 1] - in.kci_ptr[kid];
    }
#pragma unroll
    for (int o = 32; o; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((t & 63) == 0) L.sh[4 + (t >> 6)] = (uint32_t)min<uint64_t>(acc, 1u << 30);
    if (t < 2) L.sh[t] = 0;
    __syncthreads();
    const uint64_t pairs = (uint64_t)L.sh[4] + L.sh[5] + L.sh[6] + L.sh[7];
    uint32_t size = 256;
    while (size < CN_CAP && size < 2 * pairs) size <<= 1;
    const uint32_t mask = size - 1;
    const uint32_t lim = min(limit, size * 3 / 4 + (size < CN_CAP ? size : 0u));   // small tables cannot fill
    for (uint32_t s2 = t; s2 < size; s2 += CN_T) L.tab[s2] = CN_EMPTY64;
    __syncthreads();
    bool ok = true;
    for (uint64_t cb = b; cb < e && ok; cb += CN_T) {
        const uint64_t i = cb + t;
        uint32_t len = 0;
        uint64_t l0 = 0;
        if (i < e) {
            const uint32_t kid = in.skid[i];
            l0 = in.kci_ptr[kid];
            len = (uint32_t)(in.kci_ptr[kid + 1] - l0);
        }
        uint32_t T;
        const uint32_t o = block_excl_scan<CN_T>(len, L.sh + 2, &T);
        L.lo[t] = l0 - o;   // pair j of this hit reads kci[l0 + j - o]
        for (uint32_t w0 = 0; w0 < T && ok; w0 += CN_W) {
            // owner map of pairs [w0, w0 + CN_W): segment starts, then a max-scan
            reinterpret_cast<uint64_t*>(L.own)[t] = 0;
            __syncthreads();
            if (len && o >= w0 && o < w0 + CN_W) L.own[o - w0] = (uint8_t)t;
            if (w0 && o < w0 && o + len > w0) L.own[0] = (uint8_t)t;   // segment straddling the window start
            __syncthreads();
            cn_owner_scan(L.own, L.sh + 2);
            uint32_t cand[CN_U];
            uint32_t ob[CN_U];
#pragma unroll
            for (int u = 0; u < CN_U; ++u) ob[u] = L.own[t + CN_T * u];   // (j - w0 < CN_W) all LDS reads first
            decltype(+L.lo[0]) lb[CN_U];
#pragma unroll
            for (int u = 0; u < CN_U; ++u) lb[u] = L.lo[ob[u]];
#pragma unroll
            for (int u = 0; u < CN_U; ++u) {
                const uint32_t j = w0 + t + CN_T * u;
                cand[u] = CN_EMPTY;
                if (j < T) cand[u] = in.kci[lb[u] + j];
            }
#pragma unroll
            for (int u = 0; u < CN_U; ++u)
                if (cand[u] != CN_EMPTY && cand[u] != p) (void)cn_insert64(L.tab, mask, cand[u], &L.sh[0], lim, &L.sh[1]);
            __syncthreads();
            ok = __atomic_load_n(&L.sh[1], __ATOMIC_RELAXED) == 0;
        }
        __syncthreads();
    }
    if (!ok) return false;
    // emit: survivors compacted to tab[0, total), sorted by candidate, one global atomic per workgroup
    // slots read thread-strided (slot u * CN_T + t): consecutive lanes on consecutive entries, no
    // bank conflicts (a thread-contiguous block of 8 entries put 16 lanes on one bank)
    uint64_t ent[CN_CAP / CN_T];
    uint32_t cnt = 0, mx = 0;
#pragma unroll
    for (uint32_t u = 0; u < CN_CAP / CN_T; ++u) {
        ent[u] = CN_PAD;
        if (u * CN_T + t < size) {
            const uint64_t v = L.tab[u * CN_T + t];
            const uint32_t c = (uint32_t)(v >> 32);
            if ((uint32_t)v != CN_EMPTY && c >= in.min_score) {
                ent[u] = cn_key(v);
                ++cnt;
                mx = max(mx, c);
            }
        }
    }
#pragma unroll
    for (int o2 = 32; o2; o2 >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, o2, 64));
    uint32_t total;
    const uint32_t pre = block_excl_scan<CN_T>(cnt, L.sh + 2, &total);   // its barriers end the table reads
    if (total == 0) return true;
    uint32_t n2 = 2;
    while (n2 < total) n2 <<= 1;
    uint32_t w0 = pre;
#pragma unroll
    for (uint32_t u = 0; u < CN_CAP / CN_T; ++u)
        if (ent[u] != CN_PAD) L.tab[w0++] = ent[u];
    for (uint32_t i = total + t; i < n2; i += CN_T) L.tab[i] = CN_PAD;
    const uint32_t reg = p % CN_R;
    if (t == 0) {
        L.base_s = cn_reserve(out, reg, total);
        cn_note(out, p, reg, L.base_s, total);
    }
    if ((t & 63) == 0 && mx) atomicMax(&out.ctr[1], (unsigned long long)mx);
    __syncthreads();
    if (total > CN_SORT_W) block_bitonic_sort(L.tab, n2);   // shorter runs: cn_runs_keys
    const uint64_t base = L.base_s;
    for (uint32_t i = t; i < total; i += CN_T) {
        const uint64_t k = L.tab[i];
        cn_put(out, reg, base + i, p, (uint32_t)(k >> 32), (uint32_t)k);
    }
    return true;
}

// Pivots listed in piv[0, *n_piv) (the wave tier's overflow list, final when this launch starts),
// one workgroup each over a fixed grid: launched without reading the count back.
__global__ void __launch_bounds__(CN_T) cn_local(CnIn in, CnOut out, const uint32_t* __restrict__ piv,
                                                 const unsigned long long* __restrict__ n_piv,
                                                 uint32_t* __restrict__ ovf_list, unsigned long long* __restrict__ ovf_n,
                                                 uint32_t limit) {
    __shared__ CnBlockLds L;
    const unsigned long long n = *n_piv;
    for (unsigned long long q = blockIdx.x; q < n; q += gridDim.x) {
        const uint32_t p = piv[q];
        if (!cn_block_pivot(in, out, p, limit, L) && threadIdx.x == 0) ovf_list[atomicAdd(ovf_n, 1ull)] = p;
    }
}

// ---- cn_wave: the first tier — one wave per pivot, pivots taken from a work counter.
// Every wave owns a CNW_CAP-entry LDS table (u64 entries as in cn_local) and its own chunk /
// owner-map state, so a workgroup walks four pivots at once without workgroup barriers (a
// wave's LDS accesses are ordered) and a CU keeps 16 pivots' dependent load chains in flight.
// A pivot whose distinct candidates pass 3/4 of the table goes to the cn_local list.  1024 entries
// (4 workgroups a CU) against 512 (7 a CU): on C3 almost no pivot overflows to cn_local any more
// (cn_wave + cn_local 1.50 -> 1.41 ms, profiles/r04cn_variants_3.txt).
#ifndef HGA_CNW_CAP
#define HGA_CNW_CAP 1024
#endif
#ifndef HGA_CNW_WAVES
#define HGA_CNW_WAVES 4
#endif
constexpr uint32_t CNW_CAP = HGA_CNW_CAP;
constexpr uint32_t CNW_W = 512;            // pairs per owner-map window
constexpr int CNW_U = CNW_W / 64;
constexpr int CNW_WAVES = HGA_CNW_WAVES;
#ifndef HGA_CN_HOME
#define HGA_CN_HOME 1   // cn_wave: home-slot hits first, the rest through a per-wave queue (0: per-lane inserts)
#endif
#ifndef HGA_CNW_GRAB
#define HGA_CNW_GRAB 4
#endif
#ifndef HGA_CNW_MINW
#define HGA_CNW_MINW 4
#endif
#ifndef HGA_CN_BIG_HITS
#define HGA_CN_BIG_HITS 896
#endif
constexpr uint32_t CNW_GRAB = HGA_CNW_GRAB;   // pivots per work-counter atomic

constexpr uint32_t CNW_Q = 128;   // per-wave queue of a window's candidates not found at their home slot
struct CnWaveLds {
    uint64_t tab[CNW_CAP];
    uint64_t base[64];             // per hit of the chunk: byte address of its list minus 4 x its first pair index
    uint64_t own[CNW_W / 8];       // owner map, one byte per pair of the window
    uint32_t q[CNW_Q];
    uint32_t fill, ovf;
};
static_assert(CNW_U == 8, "owner map: eight pairs (one u64 of bytes) per lane");
static_assert(CNW_CAP * 3 / 4 <= CN_SORT_W, "wave-tier runs are sorted by cn_runs_keys");

// Tiers 1 and 2 in one launch: every workgroup first takes listed pivots (more than `big_hits`
// hits, from cn_big_list) one at a time as a workgroup (cn_block_pivot), then its waves take the
// other pivots one wave each.  The long pivots start first and the short ones fill in behind
// them, with no host round trip between the tiers; a listed pivot that overflows the workgroup
// table goes to ovf2 (the HBM tier), a wave pivot that overflows its wave table to ovf_list.
union CnFusedLds {
    CnBlockLds B;
    CnWaveLds W[CNW_WAVES];
};

__global__ void __launch_bounds__(64 * CNW_WAVES, HGA_CNW_MINW) cn_wave(CnIn in, CnOut out, const uint32_t* __restrict__ piv,
                                                          uint64_t n_piv, uint32_t* __restrict__ ovf_list,
                                                          uint32_t limit, const uint32_t* __restrict__ big,
                                                          uint64_t big_hits, uint32_t limit_b,
                                                          uint32_t* __restrict__ ovf2) {
    static_assert(64 * CNW_WAVES == CN_T, "the workgroup tier runs on the wave tier's workgroups");
    __shared__ CnFusedLds U;
    {
        const unsigned long long n_big = out.ctr[0];
        while (true) {
            __syncthreads();
            if (threadIdx.x == 0) U.B.sh[11] = (uint32_t)atomicAdd(out.ctr + 7, 1ull);
            __syncthreads();
            const uint32_t idx = U.B.sh[11];
            if (idx >= n_big) break;
            const uint32_t p = big[idx];
            if (!cn_block_pivot(in, out, p, limit_b, U.B) && threadIdx.x == 0) ovf2[atomicAdd(out.ctr + 3, 1ull)] = p;
        }
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    CnWaveLds& W = U.W[wave];
    uint8_t* own8 = reinterpret_cast<uint8_t*>(W.own);
    for (uint32_t s2 = lane; s2 < CNW_CAP; s2 += 64) W.tab[s2] = CN_EMPTY64;
    // pivots are taken CNW_GRAB at a time (device-wide same-address atomics serialise) and the
    // largest score is kept per wave until the end
    unsigned long long* work = out.ctr + 5;
    uint32_t wmax = 0;
    unsigned long long q = 0, q_end = 0;
    while (true) {
        if (q == q_end) {
            if (lane == 0) q = atomicAdd(work, (unsigned long long)CNW_GRAB);
            q = __shfl(q, 0, 64);
            q_end = q + CNW_GRAB;
        }
        if (q >= n_piv) break;
        const uint32_t p = piv ? piv[q] : (uint32_t)q;
        ++q;
        const uint64_t b = in.hit_ptr[p], e = in.hit_ptr[p + 1];
        if (e - b < (uint64_t)in.min_kmers || e == b || e - b > big_hits) continue;   // listed: done above
        if (lane == 0) {
            W.fill = 0;
            W.ovf = 0;
        }
        wave_lds_sync();
        bool ok = true;
        // the chunk's KmerIDs were requested one chunk ahead (their latency behind the previous chunk's walk)
        uint32_t nkid = b + lane < e ? in.skid[b + lane] : 0u;
        for (uint64_t cb = b; cb < e && ok; cb += 64) {
            const uint64_t i = cb + lane;
            uint32_t len = 0;
            uint64_t first = 0;   // byte address of the hit's first read index
            const uint32_t ckid = nkid;
            if (cb + 64 < e) nkid = cb + 64 + lane < e ? in.skid[cb + 64 + lane] : 0u;
            if (i < e) {
                const uint32_t kid = ckid;
                if (in.slots) {   // one 128-B slot: header and (short) list in the same line
                    const uint32_t* sl = in.slots + (uint64_t)kid * SLOT_W;
                    const uint4 h = *reinterpret_cast<const uint4*>(sl);
                    if (h.x != SLOT_LONG) {
                        len = h.x;
                        first = reinterpret_cast<uint64_t>(sl + 1);
                    } else {
                        len = h.y;
                        first = reinterpret_cast<uint64_t>(in.kci + ((uint64_t)h.z | ((uint64_t)h.w << 32)));
                    }
                } else {
                    const uint64_t l0 = in.kci_ptr[kid];
                    len = (uint32_t)(in.kci_ptr[kid + 1] - l0);
                    first = reinterpret_cast<uint64_t>(in.kci + l0);
                }
            }
            // pairs of the chunk numbered 0..T: hit h owns [o, o + len); pair j of h reads the word at
            // first + 4 (j - o)
            const uint32_t inc = wave_scan_add_dpp(len);
            const uint32_t o = inc - len;
            const uint32_t T = wave_lane(inc, 63);
            W.base[lane] = first - 4ull * o;
            for (uint32_t w0 = 0; w0 < T && ok; w0 += CNW_W) {
                // owner map of pairs [w0, w0 + CNW_W): segment starts, then a max-scan (bytes within a
                // lane's u64, then across lanes)
                W.own[lane] = 0;
                wave_lds_sync();
                if (len && o >= w0 && o < w0 + CNW_W) own8[o - w0] = (uint8_t)lane;
                if (w0 && o < w0 && o + len > w0) own8[0] = (uint8_t)lane;
                wave_lds_sync();
                const uint64_t ov = W.own[lane];
                uint32_t v[CNW_U];
                uint32_t m = 0;
#pragma unroll
                for (int u = 0; u < CNW_U; ++u) {
                    m = max(m, (uint32_t)(ov >> (8 * u)) & 0xFFu);
                    v[u] = m;
                }
                // the largest owner over earlier lanes: the inclusive max-scan moved up one lane (wave_shr:1)
                const uint32_t before = dpp_take<0x138, 0xf>(wave_scan_max_dpp(m));
                uint64_t nv = 0;
#pragma unroll
                for (int u = 0; u < CNW_U; ++u) nv |= (uint64_t)max(before, v[u]) << (8 * u);
                wave_lds_sync();
                W.own[lane] = nv;
                wave_lds_sync();
                // the owners and their list bases read for all eight pairs first (unpredicated: j - w0 <
                // CNW_W, an owner < 64), so the LDS reads wait twice per window instead of twice per pair
                // before its candidate load can issue
                uint32_t cand[CNW_U];
                uint32_t ob[CNW_U];
                uint64_t cb[CNW_U];
#pragma unroll
                for (int u = 0; u < CNW_U; ++u) ob[u] = own8[lane + 64 * u];
#pragma unroll
                for (int u = 0; u < CNW_U; ++u) cb[u] = W.base[ob[u]];
#pragma unroll
                for (int u = 0; u < CNW_U; ++u) {
                    const uint32_t j = w0 + lane + 64 * u;
                    cand[u] = CN_EMPTY;
                    // a global (not flat) load: flat loads count in lgkmcnt with the LDS reads, so each
                    // LDS wait would also wait for the candidate loads issued before it
                    if (j < T) cand[u] = *reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(cb[u] + 4ull * j);
                }
                // a candidate already at its home slot (most walks repeat a candidate) is one count add;
                // the rest go through the wave's queue and are inserted with every lane busy (a lane's own
                // probe loops would run with most lanes idle)
                uint32_t miss = 0;
                if (HGA_CN_HOME) {
                    uint32_t hs[CNW_U];
                    uint64_t hv[CNW_U];
#pragma unroll
                    for (int u = 0; u < CNW_U; ++u) {
                        hs[u] = cn_hash(cand[u]) & (CNW_CAP - 1);
                        hv[u] = (cand[u] != CN_EMPTY && cand[u] != p) ? __atomic_load_n(&W.tab[hs[u]], __ATOMIC_RELAXED)
                                                                       : CN_EMPTY64;
                    }
#pragma unroll
                    for (int u = 0; u < CNW_U; ++u) {
                        if (cand[u] == CN_EMPTY || cand[u] == p) continue;
                        if ((uint32_t)hv[u] == cand[u]) atomicAdd((unsigned long long*)&W.tab[hs[u]], 1ull << 32);
                        else miss |= 1u << u;
                    }
                } else {
#pragma unroll
                    for (int u = 0; u < CNW_U; ++u)
                        if (cand[u] != CN_EMPTY && cand[u] != p) miss |= 1u << u;
                }
                const uint32_t nm = (uint32_t)__popc(miss);
                const uint32_t qinc = wave_scan_add_dpp(nm);
                const uint32_t qtot = wave_lane(qinc, 63);
                if (HGA_CN_HOME && qtot <= CNW_Q) {
                    uint32_t pos = qinc - nm;
#pragma unroll
                    for (int u = 0; u < CNW_U; ++u)
                        if ((miss >> u) & 1u) W.q[pos++] = cand[u];
                    wave_lds_sync();
                    for (uint32_t i = lane; i < qtot; i += 64)
                        (void)cn_insert64(W.tab, CNW_CAP - 1, W.q[i], &W.fill, limit, &W.ovf);
                } else {
#pragma unroll
                    for (int u = 0; u < CNW_U; ++u)
                        if ((miss >> u) & 1u) (void)cn_insert64(W.tab, CNW_CAP - 1, cand[u], &W.fill, limit, &W.ovf);
                }
                wave_lds_sync();
                ok = __atomic_load_n(&W.ovf, __ATOMIC_RELAXED) == 0;
            }
            wave_lds_sync();
        }
        if (!ok) {
            if (lane == 0) ovf_list[atomicAdd(&out.ctr[2], 1ull)] = p;
            for (uint32_t s2 = lane; s2 < CNW_CAP; s2 += 64) W.tab[s2] = CN_EMPTY64;
            wave_lds_sync();
            continue;
        }
        // emit (and reset the table for the next pivot); cn_runs_keys sorts the run by candidate
        constexpr int PER = CNW_CAP / 64;
        uint64_t ent[PER];
        uint32_t cnt = 0, mx = 0;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            ent[u] = W.tab[u * 64 + lane];   // lane-strided: no bank conflicts
            W.tab[u * 64 + lane] = CN_EMPTY64;
            const uint32_t c = (uint32_t)(ent[u] >> 32);
            if ((uint32_t)ent[u] != CN_EMPTY && c >= in.min_score) {
                ++cnt;
                mx = max(mx, c);
            } else {
                ent[u] = CN_EMPTY64;
            }
        }
        wave_lds_sync();
        const uint32_t inc = wave_scan_add_dpp(cnt);
        const uint32_t tot = wave_lane(inc, 63);
        if (!tot) continue;
#pragma unroll
        for (int o2 = 32; o2; o2 >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, o2, 64));
        wmax = max(wmax, mx);
        unsigned long long base = 0;
        const uint32_t reg = p % CN_R;
        if (lane == 0) {
            base = cn_reserve(out, reg, tot);
            cn_note(out, p, reg, base, tot);
        }
        base = __shfl(base, 0, 64);
        uint64_t w = base + inc - cnt;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            if ((uint32_t)ent[u] != CN_EMPTY) {
                cn_put(out, reg, w, p, (uint32_t)ent[u], (uint32_t)(ent[u] >> 32));
                ++w;
            }
        }
    }
    if (lane == 0 && wmax) atomicMax(&out.ctr[1], (unsigned long long)wmax);
}

// Pivots with more than big_hits hits (and at least min_kmers), for cn_wave's workgroup tier.
__global__ void cn_big_list(const uint64_t* __restrict__ hit_ptr, const uint32_t* __restrict__ piv, uint64_t n_piv,
                            uint32_t min_kmers, uint64_t big_hits, uint32_t* __restrict__ big,
                            unsigned long long* __restrict__ n_big) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t p = 0;
    bool take = false;
    if (q < n_piv) {
        p = piv ? piv[q] : (uint32_t)q;
        const uint64_t h = hit_ptr[p + 1] - hit_ptr[p];
        take = h > big_hits && h >= min_kmers;
    }
    // one counter atomic per wave (same-address device atomics serialise)
    const uint64_t m = __ballot(take);
    if (!m) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t first = (uint32_t)__builtin_ctzll(m);
    unsigned long long base = 0;
    if (lane == first) base = atomicAdd(n_big, (unsigned long long)__popcll(m));
    base = __shfl(base, (int)first, 64);
    if (take) big[base + (uint64_t)__popcll(m & ((1ull << lane) - 1))] = p;
}

// Upper bound of a pivot's distinct candidates: its (id, candidate) pair count.
__global__ void __launch_bounds__(CN_T) cn_contrib(CnIn in, const uint32_t* __restrict__ list,
                                                   unsigned long long* __restrict__ mx) {
    __shared__ uint32_t ws[8];
    const uint32_t p = list[blockIdx.x];
    const uint64_t b = in.hit_ptr[p], e = in.hit_ptr[p + 1];
    uint64_t acc = 0;
    for (uint64_t i = b + threadIdx.x; i < e; i += CN_T) {
        const uint32_t kid = in.skid[i];
        acc += in.kci_ptr[kid + 1] - in.kci_ptr[kid];
    }
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 32; o; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) ws[threadIdx.x >> 6] = (uint32_t)min<uint64_t>(acc, 0xFFFFFFFFull);
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(mx, (unsigned long long)ws[0] + ws[1] + ws[2] + ws[3]);
}

// Overflow pivots: table of `size` entries per pivot in HBM (keys preset to EMPTY, values 0).
__global__ void __launch_bounds__(CN_T) cn_global(CnIn in, CnOut out, const uint32_t* __restrict__ list,
                                                  uint32_t* __restrict__ gk, uint32_t* __restrict__ gv,
                                                  uint32_t size) {
    __shared__ uint64_t sh64[(8 + 2 * CN_T + CN_T + 2) / 2];
    uint32_t* sh = reinterpret_cast<uint32_t*>(sh64);
    const uint32_t p = list[blockIdx.x];
    uint32_t* tk = gk + (uint64_t)blockIdx.x * size;
    uint32_t* tv = gv + (uint64_t)blockIdx.x * size;
    const uint64_t b = in.hit_ptr[p], e = in.hit_ptr[p + 1];
    if (threadIdx.x < 2) sh[threadIdx.x] = 0;
    __syncthreads();
    // size >= 2 * (pair count), so the walk cannot overflow; limit = size keeps the flag off
    if (!cn_walk(in, p, b, e, tk, tv, size - 1, size, sh)) return;
    __threadfence_block();
    __syncthreads();
    cn_emit(in, out, p, tk, tv, size, sh + 2);
}

// Dense index i -> output slot: region r with rpre[r] <= i < rpre[r + 1] (rpre: CN_R + 1 prefix
// counts of the regions), slot r * rcap + (i - rpre[r]).
__device__ __forceinline__ uint64_t cn_slot(const uint64_t* __restrict__ rpre, uint64_t rcap, uint64_t i) {
    uint32_t a = 0, z = CN_R;
    while (z - a > 1) {
        const uint32_t m = (a + z) >> 1;
        if (rpre[m] <= i) a = m; else z = m;
    }
    return (uint64_t)a * rcap + (i - rpre[a]);
}

// key = (max - score) << 2*ib | pivot << ib | candidate  (ascending = score desc, then ids)
__global__ void cn_keys(const uint32_t* __restrict__ x, const uint32_t* __restrict__ y, const uint32_t* __restrict__ s,
                        const uint64_t* __restrict__ rpre, uint64_t rcap, uint64_t n, uint32_t mxs, int ib,
                        uint64_t* __restrict__ key) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t g = cn_slot(rpre, rcap, i);
    key[i] = ((uint64_t)(mxs - s[g]) << (2 * ib)) | ((uint64_t)x[g] << ib) | y[g];
}

__global__ void cn_decode(const uint64_t* __restrict__ key, uint64_t n, uint32_t mxs, int ib,
                          const int32_t* __restrict__ cat, uint32_t first_id, uint32_t* __restrict__ ox,
                          uint32_t* __restrict__ oy, uint64_t* __restrict__ os, uint8_t* __restrict__ og) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = key[i];
    const uint64_t m = (1ull << ib) - 1;
    const uint32_t y = (uint32_t)(k & m), x = (uint32_t)((k >> ib) & m);
    ox[i] = x + first_id;
    oy[i] = y + first_id;
    os[i] = mxs - (uint32_t)(k >> (2 * ib));
    og[i] = cat ? (uint8_t)(cat[x] == cat[y]) : (uint8_t)0;
}

// Two-stage order when the composite key does not fit 64 bits: sort (pivot, candidate) first,
// then stably by (max - score).
__global__ void cn_pair_keys(const uint32_t* __restrict__ x, const uint32_t* __restrict__ y,
                             const uint64_t* __restrict__ rpre, uint64_t rcap, uint64_t n, int ib,
                             uint64_t* __restrict__ key, uint32_t* __restrict__ idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t g = cn_slot(rpre, rcap, i);
    key[i] = ((uint64_t)x[g] << ib) | y[g];
    idx[i] = (uint32_t)g;   // slots < 2^32 (checked on the host)
}

__global__ void cn_score_keys(const uint32_t* __restrict__ s, const uint32_t* __restrict__ idx, uint64_t n,
                              uint32_t mxs, uint32_t* __restrict__ key, uint32_t* __restrict__ pos) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    key[i] = mxs - s[idx[i]];
    pos[i] = (uint32_t)i;
}

__global__ void cn_decode2(const uint64_t* __restrict__ pkey, const uint32_t* __restrict__ skey,
                           const uint32_t* __restrict__ pos, uint64_t n, uint32_t mxs, int ib,
                           const int32_t* __restrict__ cat, uint32_t first_id, uint32_t* __restrict__ ox,
                           uint32_t* __restrict__ oy, uint64_t* __restrict__ os, uint8_t* __restrict__ og) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint64_t k = pkey[pos[j]];
    const uint64_t m = ib >= 64 ? ~0ull : (1ull << ib) - 1;
    const uint32_t y = (uint32_t)(k & m), x = (uint32_t)(k >> ib);
    ox[j] = x + first_id;
    oy[j] = y + first_id;
    os[j] = mxs - skey[j];
    og[j] = cat ? (uint8_t)(cat[x] == cat[y]) : (uint8_t)0;
}

// Pivot-ordered pairs: pivot p's run (candidate, score) copied to its scanned offset, one wave
// per pivot; the per-pivot sort by candidate then the stable score pass give the final order.
__global__ void __launch_bounds__(256) cn_gather(const uint64_t* __restrict__ pst, const uint64_t* __restrict__ poff,
                                                 uint64_t nr, int ib, const uint32_t* __restrict__ y,
                                                 const uint32_t* __restrict__ s, uint64_t* __restrict__ sk,
                                                 uint32_t* __restrict__ sv) {
    const uint64_t p = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= nr) return;
    const uint64_t o = poff[p], m = poff[p + 1] - o;
    if (!m) return;
    const uint64_t g = pst[p];
    for (uint64_t i = threadIdx.x & 63; i < m; i += 64) {
        sk[o + i] = (p << ib) | y[g + i];   // composed: runs of one pair are left as they are
        sv[o + i] = s[g + i];
    }
}
// Pivot p's run copied to its scanned offset as the final sort key
// (pivot << ib | candidate) << sb | (max - score), in candidate order: one wave per pivot; runs of
// up to CN_SORT_W pairs are sorted here in registers (64 x R keys, R the smallest power of two
// that holds the run), longer ones come sorted from the workgroup tier.
// Sort keys: candidate << sbits | score in a u32 when they fit (sbits = 0: u64 keys, candidate << 32).
template <int R, class T>
__device__ __forceinline__ void cn_run_sort_put(uint64_t p, uint64_t o, uint64_t m, uint64_t g, uint32_t lane, int ib,
                                                int sb, uint32_t mxs, int sbits, const uint32_t* __restrict__ y,
                                                const uint32_t* __restrict__ s, uint64_t* __restrict__ key) {
    constexpr int SH = sizeof(T) == 8 ? 32 : 0;
    const int sh = SH ? SH : sbits;
    const T smask = (T)(((uint64_t)1 << sh) - 1);
    T v[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
        const uint32_t i = lane * R + u;
        v[u] = i < m ? (T)(((T)y[g + i] << sh) | s[g + i]) : (T)~(T)0;
    }
    bitonic_stage<R, 2>(v, lane);
#pragma unroll
    for (int u = 0; u < R; ++u) {
        const uint32_t i = lane * R + u;
        if (i < m)
            key[o + i] = (((p << ib) | (uint64_t)(v[u] >> sh)) << sb) | (uint64_t)(mxs - (uint32_t)(v[u] & smask));
    }
}
template <class T, bool WIDE>
__device__ __forceinline__ void cn_run_sort_any(uint64_t p, uint64_t o, uint64_t m, uint64_t g, uint32_t lane, int ib,
                                                int sb, uint32_t mxs, int sbits, const uint32_t* __restrict__ y,
                                                const uint32_t* __restrict__ s, uint64_t* __restrict__ key) {
    if constexpr (WIDE) {
        cn_run_sort_put<16, T>(p, o, m, g, lane, ib, sb, mxs, sbits, y, s, key);
    } else {
        if (m <= 64) cn_run_sort_put<1, T>(p, o, m, g, lane, ib, sb, mxs, sbits, y, s, key);
        else if (m <= 128) cn_run_sort_put<2, T>(p, o, m, g, lane, ib, sb, mxs, sbits, y, s, key);
        else if (m <= 256) cn_run_sort_put<4, T>(p, o, m, g, lane, ib, sb, mxs, sbits, y, s, key);
        else cn_run_sort_put<8, T>(p, o, m, g, lane, ib, sb, mxs, sbits, y, s, key);
    }
}
#ifndef HGA_CN_RK_PPW
#define HGA_CN_RK_PPW 4
#endif
constexpr int CN_RK_PPW = HGA_CN_RK_PPW;   // pivots per wave (their offsets loaded by one coalesced load)
// Runs of up to CN_SORT_N pairs sorted here, runs over CN_SORT_W copied (they come sorted from the
// workgroup tier); the pivots of the runs in between are listed for cn_runs_keys_wide.
__global__ void __launch_bounds__(256) cn_runs_keys(const uint64_t* __restrict__ pst, const uint64_t* __restrict__ poff,
                                                    uint64_t nr, int ib, int sb, uint32_t mxs, int sbits,
                                                    const uint32_t* __restrict__ y, const uint32_t* __restrict__ s,
                                                    uint64_t* __restrict__ key, uint32_t* __restrict__ wide,
                                                    unsigned long long* __restrict__ n_wide) {
    const uint64_t p0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * CN_RK_PPW;
    if (p0 >= nr) return;
    const uint32_t lane = threadIdx.x & 63;
    uint64_t lo = 0, lm = 0, lg = 0;
    if (lane < CN_RK_PPW && p0 + lane < nr) {
        lo = poff[p0 + lane];
        lm = poff[p0 + lane + 1] - lo;
        lg = pst[p0 + lane];
    }
    for (int j = 0; j < CN_RK_PPW; ++j) {
        const uint64_t p = p0 + j;
        const uint64_t m = __shfl(lm, j, 64);
        if (p >= nr) break;
        if (!m) continue;
        const uint64_t o = __shfl(lo, j, 64), g = __shfl(lg, j, 64);
        if (m <= CN_SORT_N) {
            if (sbits) cn_run_sort_any<uint32_t, false>(p, o, m, g, lane, ib, sb, mxs, sbits, y, s, key);
            else cn_run_sort_any<uint64_t, false>(p, o, m, g, lane, ib, sb, mxs, 0, y, s, key);
        } else if (m <= CN_SORT_W) {
            if (lane == 0) wide[atomicAdd(n_wide, 1ull)] = (uint32_t)p;
        } else {
            for (uint64_t i = lane; i < m; i += 64)
                key[o + i] = ((((uint64_t)p << ib) | y[g + i]) << sb) | (uint64_t)(mxs - s[g + i]);
        }
    }
}
// The listed runs (CN_SORT_N + 1 .. CN_SORT_W pairs, 16 keys a lane): a separate kernel so that its
// registers do not cost the common runs occupancy; a fixed grid reading the count on the device.
__global__ void __launch_bounds__(256) cn_runs_keys_wide(const uint64_t* __restrict__ pst, const uint64_t* __restrict__ poff,
                                                         int ib, int sb, uint32_t mxs, int sbits,
                                                         const uint32_t* __restrict__ y, const uint32_t* __restrict__ s,
                                                         uint64_t* __restrict__ key, const uint32_t* __restrict__ wide,
                                                         const unsigned long long* __restrict__ n_wide) {
    const unsigned long long n = *n_wide;
    const uint32_t lane = threadIdx.x & 63;
    for (unsigned long long q = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); q < n; q += (uint64_t)gridDim.x * 4) {
        const uint64_t p = wide[q], o = poff[p], m = poff[p + 1] - o, g = pst[p];
        if (sbits) cn_run_sort_any<uint32_t, true>(p, o, m, g, lane, ib, sb, mxs, sbits, y, s, key);
        else cn_run_sort_any<uint64_t, true>(p, o, m, g, lane, ib, sb, mxs, 0, y, s, key);
    }
}
// key = (pivot << ib | candidate) << sb | (max - score): a stable sort by the low sb bits of keys
// already in (pivot, candidate) order gives (score desc, pivot, candidate)
__global__ void cn_keys3(const uint64_t* __restrict__ sk, const uint32_t* __restrict__ sv, uint64_t n, uint32_t mxs,
                         int sb, uint64_t* __restrict__ key) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) key[i] = (sk[i] << sb) | (uint64_t)(mxs - sv[i]);
}
__global__ void cn_decode3(const uint64_t* __restrict__ key, uint64_t n, uint32_t mxs, int ib, int sb,
                           const int32_t* __restrict__ cat, uint32_t first_id, uint32_t* __restrict__ ox,
                           uint32_t* __restrict__ oy, uint64_t* __restrict__ os, uint8_t* __restrict__ og) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = key[i];
    const uint64_t m = (1ull << ib) - 1, sm = sb ? (1ull << sb) - 1 : 0ull;
    const uint32_t y = (uint32_t)((k >> sb) & m), x = (uint32_t)((k >> (sb + ib)) & m);
    ox[i] = x + first_id;
    oy[i] = y + first_id;
    os[i] = mxs - (uint32_t)(k & sm);
    og[i] = cat ? (uint8_t)(cat[x] == cat[y]) : (uint8_t)0;
}

int bits_for(uint64_t v) {
    int b = 0;
    while (b < 64 && (v >> b)) ++b;
    return b;
}

}  // namespace

void connections_run(hga_ctx* c, const uint32_t* pivots, uint64_t n_piv, uint32_t min_kmers, uint64_t min_score,
                     const int32_t* categories, uint64_t* n_out) {
    auto& L = c->lookup;
    auto& S = c->conn;
    HGA_REQUIRE(L.ran, HGA_ERR_STATE, "hga_lookup_run not called");
    HGA_REQUIRE(min_kmers >= 1, HGA_ERR_INVALID, "min_kmers must be >= 1");
    S.n = 0;
    S.ready = false;
    const uint64_t nr = L.n_reads;
    *n_out = 0;
    if (min_score > 0xFFFFFFFFull || nr == 0 || L.hits == 0) {
        S.ready = true;
        return;
    }
    HGA_REQUIRE(nr < (1ull << 32), HGA_ERR_INVALID, "too many reads");
    const uint32_t ms = min_score ? (uint32_t)min_score : 0u;
    // pivots: ReadIDs -> read indices
    const uint32_t* d_piv = nullptr;
    uint64_t P = nr;
    bool dup_piv = false;   // a pivot listed twice: its runs cannot be keyed by the pivot read
    if (pivots) {
        std::vector<uint32_t> idx(n_piv);
        for (uint64_t i = 0; i < n_piv; ++i) {
            HGA_REQUIRE(pivots[i] >= L.first_read_id && (uint64_t)(pivots[i] - L.first_read_id) < nr,
                        HGA_ERR_INVALID, "pivot ReadID outside the lookup's reads");
            idx[i] = pivots[i] - L.first_read_id;
        }
        std::vector<uint32_t> srt(idx);
        std::sort(srt.begin(), srt.end());
        dup_piv = std::adjacent_find(srt.begin(), srt.end()) != srt.end();
        P = n_piv;
        if (!P) {
            S.ready = true;
            return;
        }
        HGA_HIP(hipMemcpyAsync(S.piv.ensure(P * 4), idx.data(), P * 4, hipMemcpyHostToDevice, c->stream));
        d_piv = S.piv.as<uint32_t>();
        c->sync();
    }
#ifdef HGA_CN_DIAG_LPT
    if (!pivots) {   // experiment: pivots in descending hit count (host order)
        std::vector<uint64_t> hp(nr + 1);
        HGA_HIP(hipMemcpyAsync(hp.data(), L.hit_ptr.p, (nr + 1) * 8, hipMemcpyDeviceToHost, c->stream));
        c->sync();
        std::vector<uint32_t> idx(nr);
        for (uint64_t i = 0; i < nr; ++i) idx[i] = (uint32_t)i;
        std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b2) {
            return hp[a + 1] - hp[a] > hp[b2 + 1] - hp[b2];
        });
        HGA_HIP(hipMemcpyAsync(S.piv.ensure(nr * 4), idx.data(), nr * 4, hipMemcpyHostToDevice, c->stream));
        d_piv = S.piv.as<uint32_t>();
        c->sync();
    }
#endif
    HGA_REQUIRE(P < (1u << 31), HGA_ERR_INVALID, "too many pivots");
    const int32_t* d_cat = nullptr;
    if (categories) {
        HGA_HIP(hipMemcpyAsync(S.cat.ensure(nr * 4), categories, nr * 4, hipMemcpyHostToDevice, c->stream));
        d_cat = S.cat.as<int32_t>();
    }
    const uint32_t* slots = nullptr;
    if (!std::getenv("HGA_CN_NO_SLOTS") && L.n_sdk) {   // cn_wave's list slots, once per index
        if (S.slots_epoch != L.kci_epoch) {
            uint32_t* sl = static_cast<uint32_t*>(S.slots.ensure((uint64_t)L.n_sdk * SLOT_W * 4));
            c->launch("cn_slots", [&] {
                hipLaunchKernelGGL(cn_slots, dim3(cn_blocks(L.n_sdk, 256)), dim3(256), 0, c->stream,
                                   L.kci_ptr.as<uint64_t>(), L.kci_val.as<uint32_t>(), (uint64_t)L.n_sdk, sl);
            });
            c->check_launch("cn_slots");
            S.slots_epoch = L.kci_epoch;
        }
        slots = S.slots.as<uint32_t>();
    }
    CnIn in{L.hit_ptr.as<uint64_t>(), L.s_val2.as<uint32_t>(), L.kci_ptr.as<uint64_t>(), L.kci_val.as<uint32_t>(),
            min_kmers, ms, slots};
    const size_t ctr_bytes = 64 + (size_t)CN_R * CN_RSTRIDE * 8;
    auto* ctr = static_cast<unsigned long long*>(S.ctr.ensure(ctr_bytes));
    unsigned long long* rcur = ctr + 8;
    uint32_t* ovf = static_cast<uint32_t*>(S.ovf.ensure(P * 4));
    uint32_t* ovf2 = static_cast<uint32_t*>(S.ovf2.ensure(P * 4));
    uint64_t rcap = (std::max<uint64_t>(S.cap_hint, 2 * L.hits + (1u << 20)) + CN_R - 1) / CN_R;
    // test hooks: every pivot through the workgroup tier / the HBM-table tier / the two-stage sort
    const bool force_global = std::getenv("HGA_CN_FORCE_GLOBAL") != nullptr;
    const bool force_block = force_global || std::getenv("HGA_CN_FORCE_BLOCK") != nullptr;
    const bool force_two = std::getenv("HGA_CN_TWO_STAGE") != nullptr;
    const bool force_full = std::getenv("HGA_CN_FULL_SORT") != nullptr;   // test hook: the one-pass key sort
    const bool runs = !dup_piv && !force_two && !force_full;
    uint64_t* pst = runs ? static_cast<uint64_t*>(S.pst.ensure(nr * 8)) : nullptr;
    uint64_t* pcnt = runs ? static_cast<uint64_t*>(S.pcnt.ensure((nr + 1) * 8)) : nullptr;
    if (const char* rc = std::getenv("HGA_CN_RCAP")) rcap = std::max<uint64_t>(1, std::strtoull(rc, nullptr, 10));
    unsigned long long h[4];
    std::vector<unsigned long long> hc(ctr_bytes / 8);
    // every synchronisation reads all counters (tier counts and the 64 region cursors) at once
    auto readback = [&] {
        HGA_HIP(hipMemcpyAsync(hc.data(), ctr, ctr_bytes, hipMemcpyDeviceToHost, c->stream));
        c->sync();
        std::memcpy(h, hc.data(), sizeof(h));
    };
    // pivots with more hits than this start first, one workgroup each (inside cn_wave); ~0: none.
    // The wave tables hold 3/4 x CNW_CAP distinct candidates: on C3, 2.3 % of the reads pass
    // that, nearly all of them long reads (tools/cnstats.py).
    uint64_t big_hits = force_block ? ~0ull : HGA_CN_BIG_HITS;
    if (const char* bh = std::getenv("HGA_CN_BIG_HITS")) big_hits = std::strtoull(bh, nullptr, 10);
    uint32_t* big = static_cast<uint32_t*>(S.big.ensure(P * 4));
    std::vector<uint64_t> rpre(CN_R + 1, 0);
    for (int attempt = 0; attempt < 2; ++attempt) {
        const uint64_t cap = rcap * CN_R;
        CnOut out{static_cast<uint32_t*>(S.x.ensure(cap * 4)), static_cast<uint32_t*>(S.y.ensure(cap * 4)),
                  static_cast<uint32_t*>(S.s.ensure(cap * 4)), rcap, ctr, rcur, pst, pcnt};
        HGA_HIP(hipMemsetAsync(ctr, 0, ctr_bytes, c->stream));
        if (pcnt) HGA_HIP(hipMemsetAsync(pcnt, 0, (nr + 1) * 8, c->stream));
        static const int wres = [] {   // resident cn_wave workgroups per CU: one round of the grid
            int nb = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, cn_wave, 64 * CNW_WAVES, 0) != hipSuccess || nb < 1) nb = 4;
            return nb;
        }();
        const uint64_t wblk = std::min<uint64_t>((P + CNW_WAVES - 1) / CNW_WAVES, (uint64_t)c->num_cu * wres);
        c->launch("cn_wave", [&] {
            if (big_hits != ~0ull)
                hipLaunchKernelGGL(cn_big_list, dim3(cn_blocks(P, 256)), dim3(256), 0, c->stream, in.hit_ptr, d_piv, P,
                                   min_kmers, big_hits, big, ctr);
            hipLaunchKernelGGL(cn_wave, dim3((unsigned)wblk), dim3(64 * CNW_WAVES), 0, c->stream, in, out, d_piv, P,
                               ovf, force_block ? 1u : CNW_CAP * 3 / 4, big, big_hits,
                               force_global ? 1u : CN_CAP * 3 / 4, ovf2);
        });
        c->check_launch("cn_wave");
        // pivots with more distinct candidates than a wave table: one workgroup each
        c->launch("cn_local", [&] {
            hipLaunchKernelGGL(cn_local, dim3((unsigned)std::min<uint64_t>(P, (uint64_t)c->num_cu * 4)), dim3(CN_T), 0,
                               c->stream, in, out, ovf, ctr + 2, ovf2, ctr + 3, force_global ? 1u : CN_CAP * 3 / 4);
        });
        c->check_launch("cn_local");
        readback();
        if (h[3]) {   // overflow pivots: HBM tables of 2 x (largest pair count), in batches of <= 1 GiB
            auto* mx = ctr + 4;
            c->launch("cn_global", [&] {
                hipLaunchKernelGGL(cn_contrib, dim3((unsigned)h[3]), dim3(CN_T), 0, c->stream, in, ovf2, mx);
            });
            c->check_launch("cn_contrib");
            unsigned long long mc = 0;
            HGA_HIP(hipMemcpyAsync(&mc, mx, 8, hipMemcpyDeviceToHost, c->stream));
            c->sync();
            const uint64_t distinct = std::min<uint64_t>(mc, nr);
            uint64_t size = 1024;
            while (size < 2 * distinct) size <<= 1;
            HGA_REQUIRE(size <= (1ull << 31), HGA_ERR_OOM, "connection table too large");
            const uint64_t batch = std::max<uint64_t>(1, (1ull << 27) / size);
            for (uint64_t b0 = 0; b0 < h[3]; b0 += batch) {
                const uint64_t nb = std::min<uint64_t>(batch, h[3] - b0);
                uint32_t* gk = static_cast<uint32_t*>(S.gk.ensure(nb * size * 4));
                uint32_t* gv = static_cast<uint32_t*>(S.gv.ensure(nb * size * 4));
                HGA_HIP(hipMemsetAsync(gk, 0xFF, nb * size * 4, c->stream));
                HGA_HIP(hipMemsetAsync(gv, 0, nb * size * 4, c->stream));
                c->launch("cn_global", [&] {
                    hipLaunchKernelGGL(cn_global, dim3((unsigned)nb), dim3(CN_T), 0, c->stream, in, out, ovf2 + b0,
                                       gk, gv, (uint32_t)size);
                });
                c->check_launch("cn_global");
            }
            readback();
        }
        uint64_t mx_region = 0;
        for (int r = 0; r < CN_R; ++r) {
            const uint64_t cnt = hc[8 + (size_t)r * CN_RSTRIDE];
            rpre[r + 1] = rpre[r] + cnt;
            mx_region = std::max<uint64_t>(mx_region, cnt);
        }
        if (mx_region <= rcap) break;
        HGA_REQUIRE(attempt == 0, HGA_ERR_OOM, "connection output grew between attempts");
        rcap = mx_region;   // exact now: run again with room for every pair
    }
    const uint64_t n = rpre[CN_R];
    HGA_REQUIRE(n < (1ull << 32), HGA_ERR_OOM, "too many connections for one sort");
    S.cap_hint = rcap * CN_R;
    uint64_t* d_rpre = static_cast<uint64_t*>(S.rpre.ensure((CN_R + 1) * 8));
    HGA_HIP(hipMemcpyAsync(d_rpre, rpre.data(), (CN_R + 1) * 8, hipMemcpyHostToDevice, c->stream));
    const uint32_t mxs = (uint32_t)h[1];
    const int ib = std::max(1, bits_for(nr - 1));
    const int sb = bits_for(mxs - ms);
    uint32_t* ox = static_cast<uint32_t*>(S.ox.ensure(std::max<uint64_t>(n, 1) * 4));
    uint32_t* oy = static_cast<uint32_t*>(S.oy.ensure(std::max<uint64_t>(n, 1) * 4));
    uint64_t* os = static_cast<uint64_t*>(S.os.ensure(std::max<uint64_t>(n, 1) * 8));
    uint8_t* og = static_cast<uint8_t*>(S.og.ensure(std::max<uint64_t>(n, 1)));
    bool done = false;
    if (n && runs && sb + 2 * ib <= 64) {
        // pivot-ordered runs, each sorted by candidate, then one stable pass over the score bits
        exclusive_scan_u64(c, pcnt, nr + 1, L.scratch);
        if (!h[3] && !std::getenv("HGA_CN_SEGSORT")) {   // no HBM-tier run: sorted in cn_runs_keys
            // u32 sort keys (candidate << sbits | score) when they fit, u64 otherwise
            const int sbits = (bits_for(mxs) + ib <= 32 && !std::getenv("HGA_CN_KEY64")) ? std::max(1, bits_for(mxs)) : 0;
            uint32_t* wide = static_cast<uint32_t*>(S.big.ensure(std::max<uint64_t>(nr, P) * 4));   // the long-pivot list is done
            HGA_HIP(hipMemsetAsync(ctr, 0, 8, c->stream));
            uint64_t* key = static_cast<uint64_t*>(S.key.ensure(n * 8));
            c->launch("cn_sort", [&] {
                hipLaunchKernelGGL(cn_runs_keys, dim3(cn_blocks(nr, 4 * CN_RK_PPW)), dim3(256), 0, c->stream, pst, pcnt, nr,
                                   ib, sb, mxs, sbits, S.y.as<uint32_t>(), S.s.as<uint32_t>(), key, wide, ctr);
                hipLaunchKernelGGL(cn_runs_keys_wide, dim3((unsigned)c->num_cu), dim3(256), 0, c->stream, pst, pcnt, ib, sb,
                                   mxs, sbits, S.y.as<uint32_t>(), S.s.as<uint32_t>(), key, wide, ctr);
            });
            c->check_launch("cn_runs_keys");
            uint64_t* sorted = static_cast<uint64_t*>(S.sk2.ensure(n * 8));
            radix_sort_u64_from(c, key, sorted, n, sb, L.scratch);
            c->launch("cn_sort", [&] {
                hipLaunchKernelGGL(cn_decode3, dim3(cn_blocks(n, 256)), dim3(256), 0, c->stream, sorted, n, mxs, ib, sb,
                                   d_cat, L.first_read_id, ox, oy, os, og);
            });
            c->check_launch("cn_decode3");
            done = true;
        }
    }
    if (n && runs && !done && sb + 2 * ib <= 64) {   // an HBM-tier pivot's run is in table order
        uint64_t* sk = static_cast<uint64_t*>(S.sk2.ensure(n * 8));
        uint32_t* sv = static_cast<uint32_t*>(S.sv2.ensure(n * 4));
        c->launch("cn_sort", [&] {
            hipLaunchKernelGGL(cn_gather, dim3(cn_blocks(nr, 4)), dim3(256), 0, c->stream, pst, pcnt, nr, ib,
                               S.y.as<uint32_t>(), S.s.as<uint32_t>(), sk, sv);
        });
        c->check_launch("cn_gather");
        if (segment_sort(c, pcnt, nr, ~0ull, ib, sk, sv, S.lst, ctr + 6, "cn_sort")) {
            uint64_t* key = static_cast<uint64_t*>(S.key.ensure(n * 8));
            c->launch("cn_sort", [&] {
                hipLaunchKernelGGL(cn_keys3, dim3(cn_blocks(n, 256)), dim3(256), 0, c->stream, sk, sv, n, mxs, sb,
                                   key);
            });
            c->check_launch("cn_keys3");
            radix_sort_u64(c, key, nullptr, n, sb, L.scratch);
            c->launch("cn_sort", [&] {
                hipLaunchKernelGGL(cn_decode3, dim3(cn_blocks(n, 256)), dim3(256), 0, c->stream, key, n, mxs, ib, sb,
                                   d_cat, L.first_read_id, ox, oy, os, og);
            });
            c->check_launch("cn_decode3");
            done = true;
        }
    }
    if (n && !done) {
        uint64_t* key = static_cast<uint64_t*>(S.key.ensure(n * 8));
        if (sb + 2 * ib <= 64 && !force_two) {
            c->launch("cn_sort", [&] {
                hipLaunchKernelGGL(cn_keys, dim3(cn_blocks(n, 256)), dim3(256), 0, c->stream, S.x.as<uint32_t>(),
                                   S.y.as<uint32_t>(), S.s.as<uint32_t>(), d_rpre, rcap, n, mxs, ib, key);
            });
            c->check_launch("cn_keys");
            radix_sort_u64(c, key, nullptr, n, sb + 2 * ib, L.scratch);
            c->launch("cn_sort", [&] {
                hipLaunchKernelGGL(cn_decode, dim3(cn_blocks(n, 256)), dim3(256), 0, c->stream, key, n, mxs, ib,
                                   d_cat, L.first_read_id, ox, oy, os, og);
            });
            c->check_launch("cn_decode");
        } else {
            HGA_REQUIRE(rcap * CN_R < (1ull << 32), HGA_ERR_OOM, "too many connection slots for one sort");
            uint32_t* idx = static_cast<uint32_t*>(S.idx.ensure(n * 4));
            uint32_t* sk = static_cast<uint32_t*>(S.skey.ensure(n * 4));
            uint32_t* pos = static_cast<uint32_t*>(S.pos.ensure(n * 4));
            c->launch("cn_sort", [&] {
                hipLaunchKernelGGL(cn_pair_keys, dim3(cn_blocks(n, 256)), dim3(256), 0, c->stream, S.x.as<uint32_t>(),
                                   S.y.as<uint32_t>(), d_rpre, rcap, n, ib, key, idx);
            });
            radix_sort_u64(c, key, idx, n, 2 * ib, L.scratch);
            c->launch("cn_sort", [&] {
                hipLaunchKernelGGL(cn_score_keys, dim3(cn_blocks(n, 256)), dim3(256), 0, c->stream,
                                   S.s.as<uint32_t>(), idx, n, mxs, sk, pos);
            });
            radix_sort_u32(c, sk, pos, n, sb, L.scratch);
            c->launch("cn_sort", [&] {
                hipLaunchKernelGGL(cn_decode2, dim3(cn_blocks(n, 256)), dim3(256), 0, c->stream, key, sk, pos, n, mxs,
                                   ib, d_cat, L.first_read_id, ox, oy, os, og);
            });
            c->check_launch("cn_decode2");
        }
    }
    c->sync();
    S.n = n;
    S.ready = true;
    *n_out = n;
}

void connections_fetch(hga_ctx* c, uint32_t* x, uint32_t* y, uint64_t* score, uint8_t* is_good, uint64_t first,
                       uint64_t count) {
    auto& S = c->conn;
    HGA_REQUIRE(S.ready, HGA_ERR_STATE, "hga_connections_run not called");
    const uint64_t a = std::min<uint64_t>(first, S.n), n = std::min<uint64_t>(count, S.n - a);
    if (n) {
        if (x) HGA_HIP(hipMemcpyAsync(x, static_cast<const uint32_t*>(S.ox.p) + a, n * 4, hipMemcpyDeviceToHost, c->stream));
        if (y) HGA_HIP(hipMemcpyAsync(y, static_cast<const uint32_t*>(S.oy.p) + a, n * 4, hipMemcpyDeviceToHost, c->stream));
        if (score)
            HGA_HIP(hipMemcpyAsync(score, static_cast<const uint64_t*>(S.os.p) + a, n * 8, hipMemcpyDeviceToHost, c->stream));
        if (is_good)
            HGA_HIP(hipMemcpyAsync(is_good, static_cast<const uint8_t*>(S.og.p) + a, n, hipMemcpyDeviceToHost, c->stream));
    }
    c->sync();
}

}  // namespace hga
