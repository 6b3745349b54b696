// exchange.hip — device side of the multi-GPU owner exchange.
//
// Every rank counts its shard of reads with hga_count_run(ctx, 1) (no per-file drop yet: a
// k-mer seen once on each of two ranks has a global count of 2).  Then
//   kx_owner_hist / kx_scatter   partition the merged rows by owner = #splitters <= key, into
//                                caller-owned device buffers (keys u64, counts u32[F] row-major) so
//                                one all_to_all per array moves each owner's slice (RCCL, caller);
//   kx_merge_flags / kx_merge_emit
//                                on the owner: radix-sort the received keys, sum the counts of equal
//                                keys (one row per source rank at most), apply the per-file
//                                `--bc` drop (run_jellyfish.sh:3-6, count >= min), and rebuild the
//                                ctx rows so spec_hist / select / rows / dump run unchanged.
// Owners hold disjoint ascending code ranges, so per-owner exports concatenated in rank order
// are the reference's LC_ALL=C export order (JellyfishOccurrenceReader.cpp:110-135).
#include "hga_internal.hpp"
#include "kmer_dev.hpp"

namespace hga {
namespace {

constexpr int KX_T = 256;
constexpr int KX_R = 16;                 // rows per thread
constexpr int KX_TILE = KX_T * KX_R;
constexpr uint32_t KX_MAX_OWN = 1024;

inline unsigned kx_blocks(uint64_t n, uint64_t t) { return (unsigned)((n + t - 1) / t); }

__device__ __forceinline__ uint32_t kx_owner(uint64_t key, const uint64_t* __restrict__ spl, uint32_t n_spl) {
    uint32_t lo = 0, hi = n_spl;   // first splitter > key
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (spl[mid] <= key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// Per-tile owner histogram, owner-major: hist[own * n_tiles + tile].
__global__ void __launch_bounds__(KX_T) kx_owner_hist(const uint64_t* __restrict__ keys, uint64_t rows,
                                                      const uint64_t* __restrict__ spl, uint32_t n_own,
                                                      uint64_t* __restrict__ hist, uint64_t n_tiles) {
    __shared__ uint32_t h[KX_MAX_OWN];
    for (uint32_t o = threadIdx.x; o < n_own; o += KX_T) h[o] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * KX_TILE;
#pragma unroll
    for (int r = 0; r < KX_R; ++r) {
        const uint64_t i = base + (uint64_t)r * KX_T + threadIdx.x;
        if (i < rows) atomicAdd(&h[kx_owner(keys[i], spl, n_own - 1)], 1u);
    }
    __syncthreads();
    for (uint32_t o = threadIdx.x; o < n_own; o += KX_T) hist[(uint64_t)o * n_tiles + blockIdx.x] = h[o];
}

// Scatter rows to their owner's slice; counts go row-major so every slice is contiguous.
__global__ void __launch_bounds__(KX_T) kx_scatter(const uint64_t* __restrict__ keys,
                                                   const uint32_t* __restrict__ cnt, uint64_t cap, uint32_t F,
                                                   uint64_t rows, const uint64_t* __restrict__ spl,
                                                   uint32_t n_own, const uint64_t* __restrict__ base,
                                                   uint64_t n_tiles, uint64_t* __restrict__ okeys,
                                                   uint32_t* __restrict__ ocnt) {
    __shared__ uint32_t cur[KX_MAX_OWN];
    for (uint32_t o = threadIdx.x; o < n_own; o += KX_T) cur[o] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * KX_TILE;
#pragma unroll 4
    for (int r = 0; r < KX_R; ++r) {
        const uint64_t i = t0 + (uint64_t)r * KX_T + threadIdx.x;
        if (i >= rows) continue;
        const uint64_t key = keys[i];
        const uint32_t o = kx_owner(key, spl, n_own - 1);
        const uint64_t pos = base[(uint64_t)o * n_tiles + blockIdx.x] + atomicAdd(&cur[o], 1u);
        okeys[pos] = key;
        for (uint32_t f = 0; f < F; ++f) ocnt[pos * F + f] = cnt[(uint64_t)f * cap + i];
    }
}

__global__ void kx_owner_totals(const uint64_t* __restrict__ base, uint64_t n_tiles, uint32_t n_own,
                                uint64_t rows, uint64_t* __restrict__ out) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= n_own) return;
    const uint64_t b = base[(uint64_t)o * n_tiles];
    const uint64_t e = o + 1 < n_own ? base[(uint64_t)(o + 1) * n_tiles] : rows;
    out[o] = e - b;
}

// Per-owner totals from an owner-major exclusive scan of nh + 1 entries (the last = total).
__global__ void kx_owner_totals2(const uint64_t* __restrict__ base, uint64_t n_tiles, uint32_t n_own,
                                 uint64_t* __restrict__ out) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= n_own) return;
    out[o] = base[(uint64_t)(o + 1) * n_tiles] - base[(uint64_t)o * n_tiles];
}

__global__ void kx_iota(uint32_t* v, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}

// Sum of the equal-key run starting at sorted position i (caller: i is a run head).
__device__ __forceinline__ uint32_t kx_run_sum(const uint64_t* __restrict__ sk, const uint32_t* __restrict__ sv,
                                               const uint32_t* __restrict__ cnt, uint64_t n, uint32_t F,
                                               uint64_t i, uint32_t f) {
    const uint64_t key = sk[i];
    uint64_t c = 0;
    for (uint64_t j = i; j < n && sk[j] == key; ++j) c += cnt[(uint64_t)sv[j] * F + f];
    return c > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)c;
}

// keep[i] = 1 iff i heads a run and some file's summed count passes the drop; keep[n] = 0.
__global__ void kx_merge_flags(const uint64_t* __restrict__ sk, const uint32_t* __restrict__ sv,
                               const uint32_t* __restrict__ cnt, uint64_t n, uint32_t F, uint32_t min_c,
                               uint64_t* __restrict__ keep) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    uint64_t k = 0;
    if (i < n && (i == 0 || sk[i] != sk[i - 1]))
        for (uint32_t f = 0; f < F && !k; ++f) k = kx_run_sum(sk, sv, cnt, n, F, i, f) >= min_c;
    keep[i] = k;
}

__global__ void kx_merge_emit(const uint64_t* __restrict__ sk, const uint32_t* __restrict__ sv,
                              const uint32_t* __restrict__ cnt, uint64_t n, uint32_t F, uint32_t min_c,
                              const uint64_t* __restrict__ pos, uint64_t* __restrict__ rkey,
                              uint32_t* __restrict__ rcnt, uint64_t cap) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || pos[i + 1] == pos[i]) return;
    const uint64_t p = pos[i];
    rkey[p] = sk[i];
    for (uint32_t f = 0; f < F; ++f) {
        const uint32_t c = kx_run_sum(sk, sv, cnt, n, F, i, f);
        rcnt[(uint64_t)f * cap + p] = c >= min_c ? c : 0u;
    }
}

}  // namespace

void count_partition(hga_ctx* c, const uint64_t* splitters, uint32_t n_own, uint64_t* keys_out,
                     uint32_t* counts_out, uint64_t* rows_per_owner) {
    auto& s = c->count;
    count_settle(c);
    HGA_REQUIRE(s.ran, HGA_ERR_STATE, "hga_count_run not called");
    HGA_REQUIRE(n_own >= 1 && n_own <= KX_MAX_OWN, HGA_ERR_INVALID, "n_owners must be in [1, 1024]");
    for (uint32_t o = 1; o + 1 < n_own; ++o)
        HGA_REQUIRE(splitters[o - 1] <= splitters[o], HGA_ERR_INVALID, "splitters must be ascending");
    const uint64_t rows = s.rows;
    const uint64_t n_tiles = std::max<uint64_t>(1, kx_blocks(rows, KX_TILE));
    const uint64_t nh = n_tiles * n_own;
    char* w = static_cast<char*>(s.xch.ensure(8 * (n_own + nh + n_own) + 64));
    uint64_t* spl = reinterpret_cast<uint64_t*>(w);
    uint64_t* hist = spl + n_own;
    uint64_t* tot = hist + nh;
    if (n_own > 1)
        HGA_HIP(hipMemcpyAsync(spl, splitters, 8 * (n_own - 1), hipMemcpyHostToDevice, c->stream));
    if (rows) {
        HGA_REQUIRE(keys_out && counts_out, HGA_ERR_INVALID, "output buffers required");
        c->launch("kx_partition", [&] {
            hipLaunchKernelGGL(kx_owner_hist, dim3(n_tiles), dim3(KX_T), 0, c->stream, s.rows_key.as<uint64_t>(),
                               rows, spl, n_own, hist, n_tiles);
        });
        c->check_launch("kx_owner_hist");
        exclusive_scan_u64(c, hist, nh, s.scratch);
        c->launch("kx_partition", [&] {
            hipLaunchKernelGGL(kx_scatter, dim3(n_tiles), dim3(KX_T), 0, c->stream, s.rows_key.as<uint64_t>(),
                               s.rows_cnt.as<uint32_t>(), s.rows_cap, s.n_files, rows, spl, n_own, hist, n_tiles,
                               keys_out, counts_out);
            hipLaunchKernelGGL(kx_owner_totals, dim3(kx_blocks(n_own, 256)), dim3(256), 0, c->stream, hist,
                               n_tiles, n_own, rows, tot);
        });
        c->check_launch("kx_scatter");
        HGA_HIP(hipMemcpyAsync(rows_per_owner, tot, 8 * n_own, hipMemcpyDeviceToHost, c->stream));
    } else {
        for (uint32_t o = 0; o < n_own; ++o) rows_per_owner[o] = 0;
    }
    c->sync();
}

void count_merge(hga_ctx* c, const uint64_t* keys, const uint32_t* counts, uint64_t n, uint32_t min_c) {
    auto& s = c->count;
    count_settle(c);
    HGA_REQUIRE(s.begun, HGA_ERR_STATE, "hga_count_begin not called");
    HGA_REQUIRE(n < (1ull << 32), HGA_ERR_INVALID, "at most 2^32-1 rows per merge");
    HGA_REQUIRE(min_c >= 1, HGA_ERR_INVALID, "min_per_file must be >= 1");
    const uint32_t F = s.n_files;
    const uint64_t cap = (std::max<uint64_t>(n, 1) + 3) & ~3ull;   // x4: 16-B row groups (kc_spec_hist)
    s.rows_key.ensure(cap * 8);
    s.rows_cnt.ensure(cap * 4 * F);
    s.rows = 0;
    s.rows_cap = cap;
    if (n) {
        HGA_REQUIRE(keys && counts, HGA_ERR_INVALID, "input buffers required");
        char* w = static_cast<char*>(s.xch2.ensure(n * 8 + n * 4 + (n + 1) * 8 + 64));
        uint64_t* sk = reinterpret_cast<uint64_t*>(w);
        uint32_t* sv = reinterpret_cast<uint32_t*>(w + n * 8);
        uint64_t* keep = reinterpret_cast<uint64_t*>(w + n * 12 + (8 - (n * 12) % 8) % 8);
        HGA_HIP(hipMemcpyAsync(sk, keys, n * 8, hipMemcpyDeviceToDevice, c->stream));
        c->launch("kx_merge", [&] {
            hipLaunchKernelGGL(kx_iota, dim3(kx_blocks(n, 256)), dim3(256), 0, c->stream, sv, n);
        });
        radix_sort_u64(c, sk, sv, n, 2 * s.k, s.scratch);
        c->launch("kx_merge", [&] {
            hipLaunchKernelGGL(kx_merge_flags, dim3(kx_blocks(n + 1, 256)), dim3(256), 0, c->stream, sk, sv, counts,
                               n, F, min_c, keep);
        });
        c->check_launch("kx_merge_flags");
        exclusive_scan_u64(c, keep, n + 1, s.scratch);
        c->launch("kx_merge", [&] {
            hipLaunchKernelGGL(kx_merge_emit, dim3(kx_blocks(n, 256)), dim3(256), 0, c->stream, sk, sv, counts, n, F,
                               min_c, keep, s.rows_key.as<uint64_t>(), s.rows_cnt.as<uint32_t>(), cap);
        });
        c->check_launch("kx_merge_emit");
        uint64_t rows = 0;
        HGA_HIP(hipMemcpyAsync(&rows, keep + n, 8, hipMemcpyDeviceToHost, c->stream));
        c->sync();
        s.rows = rows;
    }
    s.min_per_file = min_c;
    s.ran = true;
    s.n_sel = 0;
}

}  // namespace hga

// ================================================================ packed rows
// One u64 per row piece: key in the low 2k bits, file f's count in bits [2k + f*cb, 2k+(f+1)*cb)
// with cb = (64 - 2k) / F.  A row whose count exceeds 2^cb - 1 in some file is split into
// several pieces with the same key; the owner's run-sum joins them again.
namespace hga {
namespace {

struct PackFmt {
    int kb;          // key bits = 2k
    int cb;          // bits per file count
    uint32_t F;
    uint64_t cmax;   // 2^cb - 1
};

__device__ __forceinline__ uint64_t pieces_of(const uint32_t* __restrict__ cnt, uint64_t cap, uint64_t i,
                                              const PackFmt& pf) {
    uint64_t p = 1;
    for (uint32_t f = 0; f < pf.F; ++f) {
        const uint64_t c = cnt[(uint64_t)f * cap + i];
        const uint64_t q = (c + pf.cmax - 1) / pf.cmax;
        p = q > p ? q : p;
    }
    return p;
}

__global__ void __launch_bounds__(KX_T) kx_piece_hist(const uint64_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ cnt, uint64_t cap,
                                                      uint64_t rows, const uint64_t* __restrict__ spl,
                                                      uint32_t n_own, PackFmt pf, uint64_t* __restrict__ hist,
                                                      uint64_t n_tiles) {
    __shared__ unsigned long long h[KX_MAX_OWN];
    for (uint32_t o = threadIdx.x; o < n_own; o += KX_T) h[o] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * KX_TILE;
#pragma unroll 4
    for (int r = 0; r < KX_R; ++r) {
        const uint64_t i = base + (uint64_t)r * KX_T + threadIdx.x;
        if (i < rows)
            atomicAdd(&h[kx_owner(keys[i], spl, n_own - 1)], (unsigned long long)pieces_of(cnt, cap, i, pf));
    }
    __syncthreads();
    for (uint32_t o = threadIdx.x; o < n_own; o += KX_T) hist[(uint64_t)o * n_tiles + blockIdx.x] = h[o];
}

__global__ void __launch_bounds__(KX_T) kx_pack_scatter(const uint64_t* __restrict__ keys,
                                                        const uint32_t* __restrict__ cnt, uint64_t cap,
                                                        uint64_t rows, const uint64_t* __restrict__ spl,
                                                        uint32_t n_own, PackFmt pf,
                                                        const uint64_t* __restrict__ base,
                                                        uint64_t n_tiles, uint64_t* __restrict__ out) {
    __shared__ unsigned long long cur[KX_MAX_OWN];
    for (uint32_t o = threadIdx.x; o < n_own; o += KX_T) cur[o] = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * KX_TILE;
#pragma unroll 4
    for (int r = 0; r < KX_R; ++r) {
        const uint64_t i = t0 + (uint64_t)r * KX_T + threadIdx.x;
        if (i >= rows) continue;
        const uint64_t key = keys[i];
        const uint32_t o = kx_owner(key, spl, n_own - 1);
        const uint64_t np = pieces_of(cnt, cap, i, pf);
        uint64_t pos = base[(uint64_t)o * n_tiles + blockIdx.x] + atomicAdd(&cur[o], (unsigned long long)np);
        uint64_t left[8];   // F <= 8 on this path
        for (uint32_t f = 0; f < pf.F; ++f) left[f] = cnt[(uint64_t)f * cap + i];
        for (uint64_t p = 0; p < np; ++p) {
            uint64_t v = key;
            for (uint32_t f = 0; f < pf.F; ++f) {
                const uint64_t c = left[f] < pf.cmax ? left[f] : pf.cmax;
                left[f] -= c;
                v |= c << (pf.kb + (int)f * pf.cb);
            }
            out[pos++] = v;
        }
    }
}

// keep[i] = 1 iff piece i heads a key run and some file's summed count passes the drop.
__global__ void kx_pk_flags(const uint64_t* __restrict__ sk, uint64_t n, PackFmt pf, uint64_t kmask, uint32_t min_c,
                            uint64_t* __restrict__ keep) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    uint64_t k = 0;
    if (i < n && (i == 0 || ((sk[i] ^ sk[i - 1]) & kmask) != 0)) {
        const uint64_t key = sk[i] & kmask;
        for (uint32_t f = 0; f < pf.F && !k; ++f) {
            uint64_t c = 0;
            for (uint64_t j = i; j < n && (sk[j] & kmask) == key; ++j) c += (sk[j] >> (pf.kb + (int)f * pf.cb)) & pf.cmax;
            k = c >= min_c;
        }
    }
    keep[i] = k;
}

__global__ void kx_pk_emit(const uint64_t* __restrict__ sk, uint64_t n, PackFmt pf, uint64_t kmask, uint32_t min_c,
                           const uint64_t* __restrict__ pos, uint64_t* __restrict__ rkey,
                           uint32_t* __restrict__ rcnt, uint64_t cap) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || pos[i + 1] == pos[i]) return;
    const uint64_t p = pos[i], key = sk[i] & kmask;
    rkey[p] = key;
    for (uint32_t f = 0; f < pf.F; ++f) {
        uint64_t c = 0;
        for (uint64_t j = i; j < n && (sk[j] & kmask) == key; ++j) c += (sk[j] >> (pf.kb + (int)f * pf.cb)) & pf.cmax;
        const uint32_t cc = c > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)c;
        rcnt[(uint64_t)f * cap + p] = cc >= min_c ? cc : 0u;
    }
}

}  // namespace

// Bits per file count in the packed form (0 = not packable: use the wide exchange).
int count_pack_bits(hga_ctx* c) {
    auto& s = c->count;
    count_settle(c);
    const int kb = 2 * s.k;
    const int cb = s.n_files ? (64 - kb) / (int)s.n_files : 0;
    return (s.n_files <= 8 && cb >= 4) ? (cb > 32 ? 32 : cb) : 0;
}

// Packs this rank's rows by owner into `out` (capacity cap_out pieces).  Returns the number of
// pieces; if it exceeds cap_out nothing is written (the caller retries with more room).
uint64_t count_partition_packed(hga_ctx* c, const uint64_t* splitters, uint32_t n_own, uint64_t* out,
                                uint64_t cap_out, uint64_t* pieces_per_owner) {
    auto& s = c->count;
    count_settle(c);
    HGA_REQUIRE(s.ran, HGA_ERR_STATE, "hga_count_run not called");
    HGA_REQUIRE(n_own >= 1 && n_own <= KX_MAX_OWN, HGA_ERR_INVALID, "n_owners must be in [1, 1024]");
    const int cb = count_pack_bits(c);
    HGA_REQUIRE(cb > 0, HGA_ERR_INVALID, "rows of this k / file count do not pack into 64 bits");
    for (uint32_t o = 1; o + 1 < n_own; ++o)
        HGA_REQUIRE(splitters[o - 1] <= splitters[o], HGA_ERR_INVALID, "splitters must be ascending");
    const PackFmt pf{2 * s.k, cb, s.n_files, (1ull << cb) - 1};
    const uint64_t rows = s.rows;
    const uint64_t n_tiles = std::max<uint64_t>(1, kx_blocks(rows, KX_TILE));
    const uint64_t nh = n_tiles * n_own;
    char* w = static_cast<char*>(s.xch.ensure(8 * (n_own + nh + 1 + n_own) + 64));
    uint64_t* spl = reinterpret_cast<uint64_t*>(w);
    uint64_t* hist = spl + n_own;          // nh + 1 entries: the last one ends as the total
    uint64_t* tot = hist + nh + 1;
    if (n_own > 1)
        HGA_HIP(hipMemcpyAsync(spl, splitters, 8 * (n_own - 1), hipMemcpyHostToDevice, c->stream));
    if (!rows) {
        for (uint32_t o = 0; o < n_own; ++o) pieces_per_owner[o] = 0;
        return 0;
    }
    HGA_HIP(hipMemsetAsync(hist + nh, 0, 8, c->stream));
    c->launch("kx_partition", [&] {
        hipLaunchKernelGGL(kx_piece_hist, dim3(n_tiles), dim3(KX_T), 0, c->stream, s.rows_key.as<uint64_t>(),
                           s.rows_cnt.as<uint32_t>(), s.rows_cap, rows, spl, n_own, pf, hist, n_tiles);
    });
    c->check_launch("kx_piece_hist");
    exclusive_scan_u64(c, hist, nh + 1, s.scratch);
    c->launch("kx_partition", [&] {
        hipLaunchKernelGGL(kx_owner_totals2, dim3(kx_blocks(n_own, 256)), dim3(256), 0, c->stream, hist, n_tiles,
                           n_own, tot);
    });
    HGA_HIP(hipMemcpyAsync(pieces_per_owner, tot, 8 * n_own, hipMemcpyDeviceToHost, c->stream));
    c->sync();
    uint64_t total = 0;
    for (uint32_t o = 0; o < n_own; ++o) total += pieces_per_owner[o];
    if (total > cap_out) return total;
    HGA_REQUIRE(out, HGA_ERR_INVALID, "output buffer required");
    c->launch("kx_partition", [&] {
        hipLaunchKernelGGL(kx_pack_scatter, dim3(n_tiles), dim3(KX_T), 0, c->stream, s.rows_key.as<uint64_t>(),
                           s.rows_cnt.as<uint32_t>(), s.rows_cap, rows, spl, n_own, pf, hist, n_tiles, out);
    });
    c->check_launch("kx_pack_scatter");
    c->sync();
    return total;
}

// Owner side: pieces from every rank (device pointer, any order) -> merged ctx rows.
void count_merge_packed(hga_ctx* c, const uint64_t* pieces, uint64_t n, uint32_t min_c) {
    auto& s = c->count;
    count_settle(c);
    HGA_REQUIRE(s.begun, HGA_ERR_STATE, "hga_count_begin not called");
    HGA_REQUIRE(min_c >= 1, HGA_ERR_INVALID, "min_per_file must be >= 1");
    const int cb = count_pack_bits(c);
    HGA_REQUIRE(cb > 0, HGA_ERR_INVALID, "rows of this k / file count do not pack into 64 bits");
    const PackFmt pf{2 * s.k, cb, s.n_files, (1ull << cb) - 1};
    const uint64_t kmask = pf.kb >= 64 ? ~0ull : ((1ull << pf.kb) - 1);
    const uint32_t F = s.n_files;
    const uint64_t cap = (std::max<uint64_t>(n, 1) + 3) & ~3ull;   // x4: 16-B row groups (kc_spec_hist)
    s.rows_key.ensure(cap * 8);
    s.rows_cnt.ensure(cap * 4 * F);
    s.rows = 0;
    s.rows_cap = cap;
    if (n) {
        HGA_REQUIRE(pieces, HGA_ERR_INVALID, "input buffer required");
        char* w = static_cast<char*>(s.xch2.ensure(n * 8 + (n + 1) * 8 + 64));
        uint64_t* sk = reinterpret_cast<uint64_t*>(w);
        uint64_t* keep = reinterpret_cast<uint64_t*>(w + n * 8);
        HGA_HIP(hipMemcpyAsync(sk, pieces, n * 8, hipMemcpyDeviceToDevice, c->stream));
        radix_sort_u64(c, sk, nullptr, n, pf.kb, s.scratch);   // by the key bits only; counts ride along
        c->launch("kx_merge", [&] {
            hipLaunchKernelGGL(kx_pk_flags, dim3(kx_blocks(n + 1, 256)), dim3(256), 0, c->stream, sk, n, pf, kmask,
                               min_c, keep);
        });
        c->check_launch("kx_pk_flags");
        exclusive_scan_u64(c, keep, n + 1, s.scratch);
        c->launch("kx_merge", [&] {
            hipLaunchKernelGGL(kx_pk_emit, dim3(kx_blocks(n, 256)), dim3(256), 0, c->stream, sk, n, pf, kmask, min_c,
                               keep, s.rows_key.as<uint64_t>(), s.rows_cnt.as<uint32_t>(), cap);
        });
        c->check_launch("kx_pk_emit");
        uint64_t rows = 0;
        HGA_HIP(hipMemcpyAsync(&rows, keep + n, 8, hipMemcpyDeviceToHost, c->stream));
        c->sync();
        s.rows = rows;
    }
    s.min_per_file = min_c;
    s.ran = true;
    s.n_sel = 0;
}

}  // namespace hga
