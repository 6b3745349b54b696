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
#include <cstdlib>

#include "hga_internal.hpp"
#include "kmer_dev.hpp"

namespace hga {
namespace {

constexpr int CN_T = 256;
constexpr uint32_t CN_CAP = 4096;          // LDS table entries (32 KB)
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
};

struct CnOut {
    uint32_t *x, *y, *s;
    uint64_t cap;
    unsigned long long* ctr;   // [0] cursor, [1] max score, [2] overflow pivots
};

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
    if (threadIdx.x == 0) base_s = atomicAdd(&out.ctr[0], (unsigned long long)total);
    if ((threadIdx.x & 63) == 0 && mx) atomicMax(&out.ctr[1], (unsigned long long)mx);
    __syncthreads();
    uint64_t w = base_s + pre;
    for (uint32_t s = s0; s < s0 + per && cnt; ++s) {
        const uint32_t v = cn_ld(&tv[s]);
        const uint32_t key = cn_ld(&tk[s]);
        if (key != CN_EMPTY && v >= in.min_score) {
            if (w < out.cap) {
                out.x[w] = p;
                out.y[w] = key;
                out.s[w] = v;
            }
            ++w;
            --cnt;
        }
    }
}

__global__ void __launch_bounds__(CN_T) cn_local(CnIn in, CnOut out, const uint32_t* __restrict__ piv,
                                                 uint32_t* __restrict__ ovf_list, uint32_t limit) {
    __shared__ uint32_t tk[CN_CAP], tv[CN_CAP];
    __shared__ uint64_t sh64[(8 + 2 * CN_T + CN_T + 2) / 2];
    uint32_t* sh = reinterpret_cast<uint32_t*>(sh64);
    const uint32_t p = piv ? piv[blockIdx.x] : blockIdx.x;
    const uint64_t b = in.hit_ptr[p], e = in.hit_ptr[p + 1];
    if (e - b < (uint64_t)in.min_kmers || e == b) return;
    for (uint32_t s = threadIdx.x; s < CN_CAP; s += CN_T) {
        tk[s] = CN_EMPTY;
        tv[s] = 0;
    }
    if (threadIdx.x < 2) sh[threadIdx.x] = 0;
    __syncthreads();
    if (!cn_walk(in, p, b, e, tk, tv, CN_CAP - 1, limit, sh)) {
        if (threadIdx.x == 0) ovf_list[atomicAdd(&out.ctr[2], 1ull)] = p;
        return;
    }
    cn_emit(in, out, p, tk, tv, CN_CAP, sh + 2);
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

// key = (max - score) << 2*ib | pivot << ib | candidate  (ascending = score desc, then ids)
__global__ void cn_keys(const uint32_t* __restrict__ x, const uint32_t* __restrict__ y, const uint32_t* __restrict__ s,
                        uint64_t n, uint32_t mxs, int ib, uint64_t* __restrict__ key) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    key[i] = ((uint64_t)(mxs - s[i]) << (2 * ib)) | ((uint64_t)x[i] << ib) | y[i];
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
__global__ void cn_pair_keys(const uint32_t* __restrict__ x, const uint32_t* __restrict__ y, uint64_t n, int ib,
                             uint64_t* __restrict__ key, uint32_t* __restrict__ idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    key[i] = ((uint64_t)x[i] << ib) | y[i];
    idx[i] = (uint32_t)i;
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
    if (pivots) {
        std::vector<uint32_t> idx(n_piv);
        for (uint64_t i = 0; i < n_piv; ++i) {
            HGA_REQUIRE(pivots[i] >= L.first_read_id && (uint64_t)(pivots[i] - L.first_read_id) < nr,
                        HGA_ERR_INVALID, "pivot ReadID outside the lookup's reads");
            idx[i] = pivots[i] - L.first_read_id;
        }
        P = n_piv;
        if (!P) {
            S.ready = true;
            return;
        }
        HGA_HIP(hipMemcpyAsync(S.piv.ensure(P * 4), idx.data(), P * 4, hipMemcpyHostToDevice, c->stream));
        d_piv = S.piv.as<uint32_t>();
        c->sync();
    }
    HGA_REQUIRE(P < (1u << 31), HGA_ERR_INVALID, "too many pivots");
    const int32_t* d_cat = nullptr;
    if (categories) {
        HGA_HIP(hipMemcpyAsync(S.cat.ensure(nr * 4), categories, nr * 4, hipMemcpyHostToDevice, c->stream));
        d_cat = S.cat.as<int32_t>();
    }
    CnIn in{L.hit_ptr.as<uint64_t>(), L.s_val2.as<uint32_t>(), L.kci_ptr.as<uint64_t>(), L.kci_val.as<uint32_t>(),
            min_kmers, ms};
    auto* ctr = static_cast<unsigned long long*>(S.ctr.ensure(64));
    uint32_t* ovf = static_cast<uint32_t*>(S.ovf.ensure(P * 4));
    uint64_t cap = std::max<uint64_t>(S.cap_hint, 2 * L.hits + (1u << 20));
    // test hooks: every pivot through the HBM-table path / the two-stage sort
    const bool force_global = std::getenv("HGA_CN_FORCE_GLOBAL") != nullptr;
    const bool force_two = std::getenv("HGA_CN_TWO_STAGE") != nullptr;
    unsigned long long h[3];
    for (int attempt = 0; attempt < 2; ++attempt) {
        CnOut out{static_cast<uint32_t*>(S.x.ensure(cap * 4)), static_cast<uint32_t*>(S.y.ensure(cap * 4)),
                  static_cast<uint32_t*>(S.s.ensure(cap * 4)), cap, ctr};
        HGA_HIP(hipMemsetAsync(ctr, 0, 64, c->stream));
        c->launch("cn_local", [&] {
            hipLaunchKernelGGL(cn_local, dim3((unsigned)P), dim3(CN_T), 0, c->stream, in, out, d_piv, ovf,
                               force_global ? 1u : CN_CAP * 3 / 4);
        });
        c->check_launch("cn_local");
        HGA_HIP(hipMemcpyAsync(h, ctr, 24, hipMemcpyDeviceToHost, c->stream));
        c->sync();
        if (h[2]) {   // overflow pivots: HBM tables of 2 x (largest pair count), in batches of <= 1 GiB
            auto* mx = ctr + 4;
            c->launch("cn_global", [&] {
                hipLaunchKernelGGL(cn_contrib, dim3((unsigned)h[2]), dim3(CN_T), 0, c->stream, in, ovf, mx);
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
            for (uint64_t b0 = 0; b0 < h[2]; b0 += batch) {
                const uint64_t nb = std::min<uint64_t>(batch, h[2] - b0);
                uint32_t* gk = static_cast<uint32_t*>(S.gk.ensure(nb * size * 4));
                uint32_t* gv = static_cast<uint32_t*>(S.gv.ensure(nb * size * 4));
                HGA_HIP(hipMemsetAsync(gk, 0xFF, nb * size * 4, c->stream));
                HGA_HIP(hipMemsetAsync(gv, 0, nb * size * 4, c->stream));
                c->launch("cn_global", [&] {
                    hipLaunchKernelGGL(cn_global, dim3((unsigned)nb), dim3(CN_T), 0, c->stream, in, out, ovf + b0, gk,
                                       gv, (uint32_t)size);
                });
                c->check_launch("cn_global");
            }
            HGA_HIP(hipMemcpyAsync(h, ctr, 24, hipMemcpyDeviceToHost, c->stream));
            c->sync();
        }
        if (h[0] <= cap) break;
        cap = h[0];   // exact now: run again with room for every pair
    }
    const uint64_t n = h[0];
    HGA_REQUIRE(n <= cap, HGA_ERR_OOM, "connection output grew between attempts");
    HGA_REQUIRE(n < (1ull << 32), HGA_ERR_OOM, "too many connections for one sort");
    S.cap_hint = cap;
    const uint32_t mxs = (uint32_t)h[1];
    const int ib = std::max(1, bits_for(nr - 1));
    const int sb = bits_for(mxs - ms);
    uint32_t* ox = static_cast<uint32_t*>(S.ox.ensure(std::max<uint64_t>(n, 1) * 4));
    uint32_t* oy = static_cast<uint32_t*>(S.oy.ensure(std::max<uint64_t>(n, 1) * 4));
    uint64_t* os = static_cast<uint64_t*>(S.os.ensure(std::max<uint64_t>(n, 1) * 8));
    uint8_t* og = static_cast<uint8_t*>(S.og.ensure(std::max<uint64_t>(n, 1)));
    if (n) {
        uint64_t* key = static_cast<uint64_t*>(S.key.ensure(n * 8));
        if (sb + 2 * ib <= 64 && !force_two) {
            c->launch("cn_sort", [&] {
                hipLaunchKernelGGL(cn_keys, dim3(cn_blocks(n, 256)), dim3(256), 0, c->stream, S.x.as<uint32_t>(),
                                   S.y.as<uint32_t>(), S.s.as<uint32_t>(), n, mxs, ib, key);
            });
            c->check_launch("cn_keys");
            radix_sort_u64(c, key, nullptr, n, sb + 2 * ib, L.scratch);
            c->launch("cn_sort", [&] {
                hipLaunchKernelGGL(cn_decode, dim3(cn_blocks(n, 256)), dim3(256), 0, c->stream, key, n, mxs, ib,
                                   d_cat, L.first_read_id, ox, oy, os, og);
            });
            c->check_launch("cn_decode");
        } else {
            uint32_t* idx = static_cast<uint32_t*>(S.idx.ensure(n * 4));
            uint32_t* sk = static_cast<uint32_t*>(S.skey.ensure(n * 4));
            uint32_t* pos = static_cast<uint32_t*>(S.pos.ensure(n * 4));
            c->launch("cn_sort", [&] {
                hipLaunchKernelGGL(cn_pair_keys, dim3(cn_blocks(n, 256)), dim3(256), 0, c->stream, S.x.as<uint32_t>(),
                                   S.y.as<uint32_t>(), n, ib, key, idx);
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

void connections_fetch(hga_ctx* c, uint32_t* x, uint32_t* y, uint64_t* score, uint8_t* is_good) {
    auto& S = c->conn;
    HGA_REQUIRE(S.ready, HGA_ERR_STATE, "hga_connections_run not called");
    const uint64_t n = S.n;
    if (n) {
        if (x) HGA_HIP(hipMemcpyAsync(x, S.ox.p, n * 4, hipMemcpyDeviceToHost, c->stream));
        if (y) HGA_HIP(hipMemcpyAsync(y, S.oy.p, n * 4, hipMemcpyDeviceToHost, c->stream));
        if (score) HGA_HIP(hipMemcpyAsync(score, S.os.p, n * 8, hipMemcpyDeviceToHost, c->stream));
        if (is_good) HGA_HIP(hipMemcpyAsync(is_good, S.og.p, n, hipMemcpyDeviceToHost, c->stream));
    }
    c->sync();
}

}  // namespace hga
