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
// The caller-driven packed form (hga_count_partition_packed / hga_count_merge_packed: one u64
// piece per row, code-range owners) partitions with one LDS atomic per owner per wave
// (kx_piece_hist / kx_pack_scatter) and merges without a sort: pieces are binned by a hash of the
// key and every bin is summed in an LDS table (kx_mb_*).
// hga_count_exchange uses hash-bucket owners instead (kx_xb_*, below): the count kernels write the
// pieces (count.hip XbEmit), the sender groups them by bucket (kx_xb_gather; kx_xb_hist /
// kx_xb_scatter when it has to bin dense rows), the owner sums each bucket from every sender's run
// (kx_xb_merge).  Exports and rows are then the owners' sorted slices merged by key
// (exchange_protocol.hpp merge_sorted) = the reference's LC_ALL=C order (:110-135).
#include <cstdlib>

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
    count_dense(c);
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
    s.xb_on = false;
    s.dense_pending = false;
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
    s.dist = false;
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
    uint32_t big = 0;   // the largest count; one piece unless it passes 2^cb - 1 (cb <= 32)
    for (uint32_t f = 0; f < pf.F; ++f) {
        const uint32_t c = cnt[(uint64_t)f * cap + i];
        big = c > big ? c : big;
    }
    if (big <= pf.cmax) return 1;
    return ((uint64_t)big + pf.cmax - 1) / pf.cmax;
}

// Wave-aggregated owner counters (kmer_dev.hpp wave_key_add): rows go to random owners, per-lane
// adds on n_own <= 64 counters would serialise.
__device__ __forceinline__ unsigned long long wave_owner_add(unsigned long long* ctr, uint32_t o, bool live,
                                                             uint32_t n_own, int nbits) {
    return wave_key_add<unsigned long long>(ctr, o, live, n_own, nbits);
}
__device__ __forceinline__ int owner_bits(uint32_t n_own) {
    int b = 0;
    while ((1u << b) < n_own) ++b;
    return b;
}

// A tile's rows, loads issued together: keys, their packed single piece (valid when every
// count <= 2^cb - 1) and the largest count; splitters staged in LDS for the owner search.
struct RowTile {
    uint64_t key[KX_R], pk[KX_R];
    uint32_t big[KX_R];
};
__device__ __forceinline__ void load_row_tile(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ cnt,
                                              uint64_t cap, uint64_t rows, uint64_t t0, const PackFmt& pf,
                                              RowTile& rt) {
#pragma unroll
    for (int r = 0; r < KX_R; ++r) {
        const uint64_t i = t0 + (uint64_t)r * KX_T + threadIdx.x;
        rt.key[r] = i < rows ? keys[i] : 0ull;
        rt.big[r] = 0;
    }
#pragma unroll
    for (int r = 0; r < KX_R; ++r) rt.pk[r] = rt.key[r];
    for (uint32_t f = 0; f < pf.F; ++f) {
        uint32_t c[KX_R];
#pragma unroll
        for (int r = 0; r < KX_R; ++r) {
            const uint64_t i = t0 + (uint64_t)r * KX_T + threadIdx.x;
            c[r] = i < rows ? cnt[(uint64_t)f * cap + i] : 0u;
        }
#pragma unroll
        for (int r = 0; r < KX_R; ++r) {
            rt.big[r] = c[r] > rt.big[r] ? c[r] : rt.big[r];
            rt.pk[r] |= (uint64_t)c[r] << (pf.kb + (int)f * pf.cb);
        }
    }
}
__device__ __forceinline__ void stage_splitters(const uint64_t* __restrict__ spl, uint32_t n_own, uint64_t* ls) {
    for (uint32_t o = threadIdx.x; o + 1 < n_own; o += KX_T) ls[o] = spl[o];
}

__global__ void __launch_bounds__(KX_T) kx_piece_hist(const uint64_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ cnt, uint64_t cap,
                                                      uint64_t rows, const uint64_t* __restrict__ spl,
                                                      uint32_t n_own, PackFmt pf, uint64_t* __restrict__ hist,
                                                      uint64_t n_tiles) {
    __shared__ unsigned long long h[KX_MAX_OWN];
    __shared__ uint64_t ls[KX_MAX_OWN];
    for (uint32_t o = threadIdx.x; o < n_own; o += KX_T) h[o] = 0;
    stage_splitters(spl, n_own, ls);
    const uint64_t t0 = (uint64_t)blockIdx.x * KX_TILE;
    const int nbits = owner_bits(n_own);
    RowTile rt;
    load_row_tile(keys, cnt, cap, rows, t0, pf, rt);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < KX_R; ++r) {
        const bool live = t0 + (uint64_t)r * KX_T + threadIdx.x < rows;
        const uint32_t o = kx_owner(rt.key[r], ls, n_own - 1);
        if (nbits > 6 || __ballot(live && rt.big[r] > pf.cmax)) {   // split rows / many owners: per-lane adds
            if (live) atomicAdd(&h[o], (unsigned long long)(rt.big[r] <= pf.cmax ? 1ull
                                                             : ((uint64_t)rt.big[r] + pf.cmax - 1) / pf.cmax));
        } else {
            (void)wave_owner_add(h, o, live, n_own, nbits);
        }
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
    __shared__ uint64_t ls[KX_MAX_OWN];
    for (uint32_t o = threadIdx.x; o < n_own; o += KX_T) cur[o] = base[(uint64_t)o * n_tiles + blockIdx.x];
    stage_splitters(spl, n_own, ls);
    const uint64_t t0 = (uint64_t)blockIdx.x * KX_TILE;
    const int nbits = owner_bits(n_own);
    RowTile rt;
    load_row_tile(keys, cnt, cap, rows, t0, pf, rt);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < KX_R; ++r) {
        const uint64_t i = t0 + (uint64_t)r * KX_T + threadIdx.x;
        const bool live = i < rows;
        const uint32_t o = kx_owner(rt.key[r], ls, n_own - 1);
        if (nbits > 6 || __ballot(live && rt.big[r] > pf.cmax)) {   // per-lane reservation, pieces one by one
            if (!live) continue;
            const uint64_t np = pieces_of(cnt, cap, i, pf);
            uint64_t pos = atomicAdd(&cur[o], (unsigned long long)np);
            uint64_t left[8];   // F <= 8 on this path
            for (uint32_t f = 0; f < pf.F; ++f) left[f] = cnt[(uint64_t)f * cap + i];
            for (uint64_t p = 0; p < np; ++p) {
                uint64_t v = rt.key[r];
                for (uint32_t f = 0; f < pf.F; ++f) {
                    const uint64_t c = left[f] < pf.cmax ? left[f] : pf.cmax;
                    left[f] -= c;
                    v |= c << (pf.kb + (int)f * pf.cb);
                }
                out[pos++] = v;
            }
        } else {
            const unsigned long long at = wave_owner_add(cur, o, live, n_own, nbits);
            if (live) out[at] = rt.pk[r];
        }
    }
}

// ---------------------------------------------------------------- owner merge by hash buckets
// The owner's pieces (any order; a key has up to one piece per sender, more when a count passes
// the piece width) are binned by the top mb bits of the counting mix (kmer_dev.hpp Mix: the
// senders' rows come out of kc_count_s in runs of one fine bucket, so the bins arrive in runs):
// kx_mb_hist adds every tile's per-bin counts to the bin totals (one device atomic per nonzero
// bin), a scan of the totals gives the bin starts, kx_mb_scatter reserves each tile's run per bin
// with one device atomic and writes it; kx_mb_merge sums each bin (about T/2 pieces) in an LDS
// hash table, applies the per-file drop and writes the kept rows into the bin's own range, and
// kx_mb_compact packs them after a scan of the per-bin row counts.  No sort: spec_hist is
// order-free and the export sort (kc_select + sort_export_u64) orders the keys.
constexpr int MB_NT = 1024;
constexpr int MB_R = 16;                       // pieces per thread per tile
constexpr uint64_t MB_TILE = (uint64_t)MB_NT * MB_R;
constexpr int MB_MAXB = 14;                    // <= 16384 buckets
#ifndef HGA_MG_NT
#define HGA_MG_NT 256   // 256-thread merge workgroups: 0.208 -> 0.157 ms at C2 (more of them resident)
#endif
#ifndef HGA_MG_R
#define HGA_MG_R 4
#endif
constexpr int MG_NT = HGA_MG_NT;
constexpr int MG_R = HGA_MG_R;                 // pieces per thread in flight

__device__ __forceinline__ uint64_t fmix64(uint64_t k) {   // MurmurHash3's 64-bit finaliser
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}
__device__ __forceinline__ uint32_t mb_bucket(uint64_t key, const Mix& mx, int mb) {
    return mb ? (uint32_t)(mix_fwd(key, mx) >> (mx.n - mb)) : 0u;
}

// LDS counter add for pieces that arrive in runs of one bucket (the senders' fine-bucket
// runs): the buckets of lane 0 and lane 63 take one add each for all their lanes, the rest
// (a third bucket inside one wave is rare) add per lane.  Returns the lane's position.
__device__ __forceinline__ uint32_t run_add(uint32_t* ctr, uint32_t b, bool live) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t pos = 0;
    bool done = !live;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const uint32_t lb = __shfl(b, e ? 63 : 0, 64);
        const uint64_t m = __ballot(!done && b == lb);
        if (!m) continue;
        const int first = __builtin_ctzll(m);
        uint32_t base = 0;
        if ((int)lane == first) base = atomicAdd(&ctr[lb], (uint32_t)__popcll(m));
        base = __shfl(base, first, 64);
        if (!done && b == lb) {
            pos = base + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            done = true;
        }
    }
    if (!done) pos = atomicAdd(&ctr[b], 1u);
    return pos;
}

// tot[b] += pieces of this tile in bucket b (one device atomic per nonzero bucket: the pieces
// arrive in runs, so a tile touches few buckets).
__global__ void __launch_bounds__(MB_NT) kx_mb_hist(const uint64_t* __restrict__ pieces, uint64_t n, uint64_t kmask,
                                                    Mix mx, int mb, unsigned long long* __restrict__ tot) {
    __shared__ uint32_t h[1 << MB_MAXB];
    const uint32_t nb = 1u << mb;
    for (uint32_t b = threadIdx.x; b < nb; b += MB_NT) h[b] = 0;
    const uint64_t t0 = (uint64_t)blockIdx.x * MB_TILE;
    uint64_t v[MB_R];
#pragma unroll
    for (int r = 0; r < MB_R; ++r) {
        const uint64_t i = t0 + (uint64_t)r * MB_NT + threadIdx.x;
        v[r] = i < n ? pieces[i] : 0ull;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MB_R; ++r) {
        const bool live = t0 + (uint64_t)r * MB_NT + threadIdx.x < n;
        (void)run_add(h, live ? mb_bucket(v[r] & kmask, mx, mb) : 0u, live);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += MB_NT)
        if (h[b]) atomicAdd(&tot[b], (unsigned long long)h[b]);
}

// Pieces to their buckets: ranks within the tile in LDS, one device atomic per nonzero bucket on
// `cursor` (initialised to the bucket starts) reserves the tile's run, then the run is written.
__global__ void __launch_bounds__(MB_NT) kx_mb_scatter(const uint64_t* __restrict__ pieces, uint64_t n,
                                                       uint64_t kmask, Mix mx, int mb,
                                                       unsigned long long* __restrict__ cursor,
                                                       uint64_t* __restrict__ out) {
    __shared__ uint32_t cnt[1 << MB_MAXB];
    __shared__ uint32_t start[1 << MB_MAXB];   // n < 2^32 (count_merge_packed)
    const uint32_t nb = 1u << mb;
    for (uint32_t b = threadIdx.x; b < nb; b += MB_NT) cnt[b] = 0;
    const uint64_t t0 = (uint64_t)blockIdx.x * MB_TILE;
    uint64_t v[MB_R];
#pragma unroll
    for (int r = 0; r < MB_R; ++r) {
        const uint64_t i = t0 + (uint64_t)r * MB_NT + threadIdx.x;
        v[r] = i < n ? pieces[i] : 0ull;
    }
    __syncthreads();
    uint32_t bk[MB_R], at[MB_R];
#pragma unroll
    for (int r = 0; r < MB_R; ++r) {
        const bool live = t0 + (uint64_t)r * MB_NT + threadIdx.x < n;
        bk[r] = live ? mb_bucket(v[r] & kmask, mx, mb) : 0u;
        at[r] = run_add(cnt, bk[r], live);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += MB_NT)
        if (cnt[b]) start[b] = (uint32_t)atomicAdd(&cursor[b], (unsigned long long)cnt[b]);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MB_R; ++r)
        if (t0 + (uint64_t)r * MB_NT + threadIdx.x < n) out[(uint64_t)start[bk[r]] + at[r]] = v[r];
}

// One workgroup per bucket: pieces summed per key in an LDS table of T slots (u64 key + FMAX u32
// counts), P passes over the bucket when it holds more than 3T/4 pieces (pass p takes the keys
// whose top 8 bits of fmix64(key) fall in its share; slots from its low bits), per-file drop,
// kept rows staged in LDS and written coalesced into the bucket's own piece range of wkey /
// wcnt (rows <= pieces), kept[b] = its rows.  No device-wide cursor: same-address device atomics
// serialise, one per workgroup would bound the kernel.  gstat[1] |= 1 when a table filled (the
// host reruns with pmul doubled).  `ld(i)` returns the bucket's i-th piece, i < m; `a` is the
// bucket's first slot in wkey / wcnt.  HASHED: the pieces carry the counting mix h of the key (the
// hash-bucket exchange), whose low bits are the slot; the table holds h & kmask (KT = u32 when the
// bucket's own bits leave <= 31 others: hbase holds the rest) and the rows get the key back
// (mix_inv(hbase | key)).
template <int T, int FMAX, class KT = unsigned long long>
struct MergeLds {
    KT tkey[T];
    uint32_t tcnt[FMAX * T];
    uint32_t tsat[(FMAX * T + 31) / 32];   // bit f * T + slot: that sum passed 2^32 - 1
    uint32_t ws[MG_NT / 64 + 1];
    uint32_t s_ovf;
};
template <int T, int FMAX, bool HASHED, class KT, class Load>
__device__ __forceinline__ void merge_bucket(MergeLds<T, FMAX, KT>& L, const Load& ld, uint64_t m, uint64_t a, uint32_t b,
                                             const PackFmt& pf, const Mix& mx, uint64_t kmask, uint64_t hbase,
                                             uint32_t min_c, uint32_t pmul,
                                             uint64_t* __restrict__ wkey, uint32_t* __restrict__ wcnt, uint64_t n,
                                             uint64_t* __restrict__ kept, unsigned long long* __restrict__ gstat) {
    static_assert(T % MG_NT == 0 && T / MG_NT <= 32, "each thread owns T / MG_NT <= 32 slots");
    constexpr KT EMPTY = (KT)~(KT)0;
    const int tid = threadIdx.x;
    uint64_t rb = 0;   // rows written so far (uniform)
    const uint32_t F = pf.F;
    const bool can_wrap = (m * pf.cmax) >> 32 != 0;          // m pieces of <= cmax each
    uint32_t P = (uint32_t)((m * 4 + 3 * T - 1) / (3 * T));   // <= 3/4 load per pass
    P = pmul ? (P ? P : 1u) * pmul : 1u;   // pmul 0: one pass whatever the size (test hook)
    P = P < 256u ? P : 256u;
    if (tid == 0) L.s_ovf = 0;
    for (uint32_t p = 0; p < P; ++p) {
        for (uint32_t j = tid; j < T; j += MG_NT) L.tkey[j] = EMPTY;
        for (uint32_t j = tid; j < F * T; j += MG_NT) L.tcnt[j] = 0;
        for (uint32_t j = tid; j < (FMAX * T + 31) / 32; j += MG_NT) L.tsat[j] = 0;
        __syncthreads();
        for (uint64_t i0 = 0; i0 < m; i0 += (uint64_t)MG_NT * MG_R) {
            uint64_t v[MG_R];
#pragma unroll
            for (int q = 0; q < MG_R; ++q) {   // all loads issued before the table work
                const uint64_t i = i0 + (uint64_t)q * MG_NT + tid;
                v[q] = i < m ? ld(i) : 0ull;
            }
#pragma unroll
            for (int q = 0; q < MG_R; ++q) {
                if (i0 + (uint64_t)q * MG_NT + tid >= m) continue;
                const KT key = (KT)(v[q] & kmask);
                if (P > 1 && (((uint32_t)(fmix64(key) >> 56) * P) >> 8) != p) continue;   // this pass's share
                uint32_t slot = (uint32_t)(HASHED ? (uint64_t)key : fmix64(key)) & (T - 1);
                uint32_t t = 0;
                for (; t < T; ++t) {
                    const KT old = atomicCAS(&L.tkey[slot], EMPTY, key);
                    if (old == EMPTY || old == key) break;
                    slot = (slot + 1) & (T - 1);
                }
                if (t == T) {
                    L.s_ovf = 1;
                    continue;
                }
                for (uint32_t f = 0; f < F; ++f) {
                    const uint32_t c = (uint32_t)((v[q] >> (pf.kb + (int)f * pf.cb)) & pf.cmax);
                    if (!c) continue;
                    if (!can_wrap) {   // no sum of this bucket can pass 2^32 - 1: a plain add, no return
                        atomicAdd(&L.tcnt[f * T + slot], c);
                        continue;
                    }
                    // counts saturate at 2^32 - 1 like count_merge's (a wrapping add is flagged)
                    const uint32_t old = atomicAdd(&L.tcnt[f * T + slot], c);
                    if (old + c < old) atomicOr(&L.tsat[(f * T + slot) >> 5], 1u << ((f * T + slot) & 31));
                }
            }
        }
        __syncthreads();
        if (L.s_ovf) {
            if (tid == 0) {
                atomicOr(&gstat[1], 1ull);
                kept[b] = 0;   // the compaction that follows this attempt stays in bounds
            }
            return;   // uniform: every thread read s_ovf after the barrier
        }
        // each thread reads slots j * MG_NT + tid (lanes on consecutive banks) and writes its kept
        // rows straight to a range of its own (one block scan, no LDS round trip; rows in any order)
        constexpr int ES = T / MG_NT;
        KT kk[ES];
        uint32_t cc[ES * FMAX];
        uint32_t keep = 0;
#pragma unroll
        for (int j = 0; j < ES; ++j) {
            const uint32_t s = j * MG_NT + tid;
            kk[j] = L.tkey[s];
            bool any = false;
#pragma unroll
            for (int f = 0; f < FMAX; ++f) {
                if (f >= (int)F) break;
                uint32_t c = L.tcnt[f * T + s];
                if ((L.tsat[(f * T + s) >> 5] >> ((f * T + s) & 31)) & 1u) c = 0xFFFFFFFFu;
                c = c >= min_c ? c : 0u;
                cc[j * FMAX + f] = c;
                any |= c != 0u;
            }
            if (kk[j] != EMPTY && any) keep |= 1u << j;
        }
        uint32_t tot;
        const uint32_t ex = block_excl_scan<MG_NT>((uint32_t)__popc(keep), L.ws, &tot);
        uint64_t o = a + rb + ex;
#pragma unroll
        for (int j = 0; j < ES; ++j)
            if ((keep >> j) & 1u) {
                wkey[o] = HASHED ? mix_inv(hbase | (uint64_t)kk[j], mx) : (uint64_t)kk[j];
#pragma unroll
                for (int f = 0; f < FMAX; ++f)
                    if (f < (int)F) wcnt[(uint64_t)f * n + o] = cc[j * FMAX + f];
                ++o;
            }
        rb += tot;
        __syncthreads();   // the next pass clears the table
    }
    if (tid == 0) kept[b] = rb;
}

template <int T, int FMAX>
__global__ void __launch_bounds__(MG_NT) kx_mb_merge(const uint64_t* __restrict__ sk, const uint64_t* __restrict__ bstart,
                                                     PackFmt pf, uint64_t kmask, int mb,
                                                     uint32_t min_c, uint32_t pmul, uint64_t* __restrict__ wkey,
                                                     uint32_t* __restrict__ wcnt, uint64_t n,
                                                     uint64_t* __restrict__ kept, unsigned long long* __restrict__ gstat) {
    __shared__ MergeLds<T, FMAX> L;
    (void)mb;
    const uint32_t b = blockIdx.x;
    const uint64_t a = bstart[b], e = bstart[b + 1];
    merge_bucket<T, FMAX, false>(L, [&](uint64_t i) { return sk[a + i]; }, e - a, a, b, pf, Mix{}, kmask, 0ull, min_c,
                                 pmul, wkey, wcnt, n, kept, gstat);
}

// Rows of bucket b from its piece range to the scanned row offset off[b] (one workgroup per bucket).
__global__ void __launch_bounds__(256) kx_mb_compact(const uint64_t* __restrict__ wkey, const uint32_t* __restrict__ wcnt,
                                                     uint64_t n, uint32_t F, const uint64_t* __restrict__ bstart,
                                                     const uint64_t* __restrict__ off, uint64_t* __restrict__ rkey,
                                                     uint32_t* __restrict__ rcnt, uint64_t cap) {
    const uint32_t b = blockIdx.x;
    const uint64_t a = bstart[b], o = off[b], m = off[b + 1] - o;
    for (uint64_t j = threadIdx.x; j < m; j += 256) {
        rkey[o + j] = wkey[a + j];
        for (uint32_t f = 0; f < F; ++f) rcnt[(uint64_t)f * cap + o + j] = wcnt[(uint64_t)f * n + a + j];
    }
}

// ---------------------------------------------------------------- hash-bucket exchange
// hga_count_exchange's packed form (exchange_protocol.hpp): owners hold ranges of the counting mix's
// top bits (kmer_dev.hpp Mix, the same on every rank).  The sender bins its pieces by the top R bits
// (kx_xb_hist: per-bucket totals, one device atomic per tile and nonzero bucket; a scan;
// kx_xb_scatter: ranks in LDS, one device atomic per tile and bucket reserves the tile's run), so
// every owner's pieces leave as one bucket-ordered range and its directory as its slice of the
// per-bucket counts.  The owner sums each of its buckets, at the coarsest resolution any sender
// used, straight from the senders' runs (kx_xb_units sizes them, kx_xb_merge sums them): no
// re-binning on the owner.
constexpr int XB_MAXR = 14;        // sender resolution: LDS counters per tile
constexpr int XB_NT = 1024;
constexpr int XB_R = 8;            // rows per thread per tile
constexpr uint64_t XB_TILE = (uint64_t)XB_NT * XB_R;
constexpr uint32_t XB_MAXP = 1024; // senders (= KX_MAX_OWN)

// A tile's rows: the counting mix of each key (the pieces carry it: the owner's buckets and table
// slots are its bits), the packed single piece and the largest count.
struct XbRows {
    uint64_t h[XB_R], pk[XB_R];
    uint32_t big[XB_R];
};
__device__ __forceinline__ void xb_load(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ cnt,
                                        uint64_t cap, uint64_t rows, uint64_t t0, const PackFmt& pf, const Mix& mx,
                                        XbRows& x) {
#pragma unroll
    for (int r = 0; r < XB_R; ++r) {
        const uint64_t i = t0 + (uint64_t)r * XB_NT + threadIdx.x;
        x.h[r] = i < rows ? keys[i] : 0ull;
        x.big[r] = 0;
    }
#pragma unroll
    for (int r = 0; r < XB_R; ++r) x.h[r] = mix_fwd(x.h[r], mx);
#pragma unroll
    for (int r = 0; r < XB_R; ++r) x.pk[r] = x.h[r];
    for (uint32_t f = 0; f < pf.F; ++f) {
        uint32_t c[XB_R];
#pragma unroll
        for (int r = 0; r < XB_R; ++r) {
            const uint64_t i = t0 + (uint64_t)r * XB_NT + threadIdx.x;
            c[r] = i < rows ? cnt[(uint64_t)f * cap + i] : 0u;
        }
#pragma unroll
        for (int r = 0; r < XB_R; ++r) {
            x.big[r] = c[r] > x.big[r] ? c[r] : x.big[r];
            x.pk[r] |= (uint64_t)c[r] << (pf.kb + (int)f * pf.cb);   // the single piece (valid when big <= cmax)
        }
    }
}
__device__ __forceinline__ uint32_t xb_pieces_of(uint32_t big, const PackFmt& pf) {
    return big <= pf.cmax ? 1u : (uint32_t)(((uint64_t)big + pf.cmax - 1) / pf.cmax);
}
__device__ __forceinline__ uint32_t xb_bucket(uint64_t h, const Mix& mx, int R) {
    return (uint32_t)(h >> (mx.n - (uint32_t)R));
}

__global__ void __launch_bounds__(XB_NT) kx_xb_hist(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ cnt,
                                                    uint64_t cap, uint64_t rows, PackFmt pf, Mix mx, int R,
                                                    unsigned long long* __restrict__ tot) {
    __shared__ uint32_t h[1 << XB_MAXR];
    const uint32_t nb = 1u << R;
    for (uint32_t b = threadIdx.x; b < nb; b += XB_NT) h[b] = 0;
    const uint64_t t0 = (uint64_t)blockIdx.x * XB_TILE;
    XbRows x;
    xb_load(keys, cnt, cap, rows, t0, pf, mx, x);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < XB_R; ++r)
        if (t0 + (uint64_t)r * XB_NT + threadIdx.x < rows)
            atomicAdd(&h[xb_bucket(x.h[r], mx, R)], xb_pieces_of(x.big[r], pf));
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += XB_NT)
        if (h[b]) atomicAdd(&tot[b], (unsigned long long)h[b]);
}

// Pieces to their buckets: ranks within the tile in LDS, one device atomic per nonzero bucket on
// `cursor` (initialised to the bucket starts) reserves the tile's run; a row whose count passes the
// piece width writes its pieces one after the other.
__global__ void __launch_bounds__(XB_NT) kx_xb_scatter(const uint64_t* __restrict__ keys,
                                                       const uint32_t* __restrict__ cnt, uint64_t cap, uint64_t rows,
                                                       PackFmt pf, Mix mx, int R,
                                                       unsigned long long* __restrict__ cursor,
                                                       uint64_t* __restrict__ out) {
    __shared__ uint32_t c[1 << XB_MAXR];
    __shared__ uint32_t st[1 << XB_MAXR];   // pieces < 2^32 per rank (count_xb_pack)
    const uint32_t nb = 1u << R;
    for (uint32_t b = threadIdx.x; b < nb; b += XB_NT) c[b] = 0;
    const uint64_t t0 = (uint64_t)blockIdx.x * XB_TILE;
    XbRows x;
    xb_load(keys, cnt, cap, rows, t0, pf, mx, x);
    __syncthreads();
    uint32_t bk[XB_R], at[XB_R];
#pragma unroll
    for (int r = 0; r < XB_R; ++r) {
        const bool live = t0 + (uint64_t)r * XB_NT + threadIdx.x < rows;
        bk[r] = live ? xb_bucket(x.h[r], mx, R) : 0u;
        at[r] = live ? atomicAdd(&c[bk[r]], xb_pieces_of(x.big[r], pf)) : 0u;
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += XB_NT)
        if (c[b]) st[b] = (uint32_t)atomicAdd(&cursor[b], (unsigned long long)c[b]);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < XB_R; ++r) {
        const uint64_t i = t0 + (uint64_t)r * XB_NT + threadIdx.x;
        if (i >= rows) continue;
        uint64_t pos = (uint64_t)st[bk[r]] + at[r];
        if (x.big[r] <= pf.cmax) {
            out[pos] = x.pk[r];
            continue;
        }
        uint64_t left[8];   // F <= 8 on this path
        for (uint32_t f = 0; f < pf.F; ++f) left[f] = cnt[(uint64_t)f * cap + i];
        for (uint32_t p = 0, np = xb_pieces_of(x.big[r], pf); p < np; ++p) {
            uint64_t v = x.h[r];
            for (uint32_t f = 0; f < pf.F; ++f) {
                const uint64_t q = left[f] < pf.cmax ? left[f] : pf.cmax;
                left[f] -= q;
                v |= q << (pf.kb + (int)f * pf.cb);
            }
            out[pos++] = v;
        }
    }
}

// Pieces of the count kernel's exchange emission (count.hip XbEmit) from each count bucket's slab
// run to its place in the send buffer (S = scanned per-bucket counts), grouped by the next x bits
// of the hash on the way (wave-aggregated LDS ranks; any order inside a group), and the bucket's
// 2^x group counts into the directory at resolution fb + x.
__global__ void __launch_bounds__(256) kx_xb_gather(const uint64_t* __restrict__ slab, const uint64_t* __restrict__ fs,
                                                    uint32_t F, uint32_t x, int sub_shift,
                                                    const uint64_t* __restrict__ S, uint64_t* __restrict__ out,
                                                    uint64_t* __restrict__ dir) {
    __shared__ uint32_t cnt[64];
    const uint64_t b = blockIdx.x;
    const uint64_t a = S[b], m = S[b + 1] - a;
    const uint64_t* __restrict__ src = slab + fs[b * (F + 1)];
    const uint32_t nsub = 1u << x, tid = threadIdx.x;
    if (tid < 64) cnt[tid] = 0;
    __syncthreads();
    for (uint64_t i0 = 0; i0 < m; i0 += 256) {   // uniform trip count
        const uint64_t i = i0 + tid;
        const bool live = i < m;
        const uint32_t sb = live ? (uint32_t)(src[i] >> sub_shift) & (nsub - 1) : 0u;
        (void)wave_key_add<uint32_t>(cnt, sb, live, nsub, (int)x);
    }
    __syncthreads();
    if (tid < 64) {   // group starts; the directory entries
        const uint32_t v = tid < nsub ? cnt[tid] : 0u;
        const uint32_t inc = wave_incl_scan(v, (int)tid);
        if (tid < nsub) {
            cnt[tid] = inc - v;
            dir[(b << x) + tid] = v;
        }
    }
    __syncthreads();
    for (uint64_t i0 = 0; i0 < m; i0 += 256) {
        const uint64_t i = i0 + tid;
        const bool live = i < m;
        const uint64_t v = live ? src[i] : 0ull;
        const uint32_t sb = (uint32_t)(v >> sub_shift) & (nsub - 1);
        const uint32_t pos = wave_key_add<uint32_t>(cnt, sb, live, nsub, (int)x);
        if (live) out[a + pos] = v;
    }
}

// Per-owner piece totals from the scanned bucket starts S (2^R + 1 entries).
__global__ void kx_xb_owner_tot(const uint64_t* __restrict__ S, uint32_t P, int eb0, int R, uint64_t* __restrict__ per) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= P) return;
    auto first = [&](uint32_t q) { return ((((uint64_t)q << eb0) + P - 1) / P) << (R - eb0); };
    per[o] = S[first(o + 1)] - S[first(o)];
}

// Owner side.  S = exclusive scan of the received directories (sender-major, sender p's buckets
// from entry src[p].off at resolution rmin + src[p].d): bucket u of this owner at the coarsest
// resolution rmin is sender p's entries [u << d, (u + 1) << d), its pieces base + S[off + (u << d)]
// - S[off] .. base + S[off + ((u + 1) << d)] - S[off] (base: the received buffer's segment of p,
// or this rank's own slice of its send buffer).
struct XbSrc {
    uint64_t off;
    uint32_t d, pad;
    const uint64_t* base;
};
// ut[u] = the pieces of this owner's buckets before u, over all senders (no scan: each sender's
// share is a difference of S).
__global__ void kx_xb_units(const uint64_t* __restrict__ S, const XbSrc* __restrict__ src, uint32_t P, uint64_t units,
                            uint64_t* __restrict__ ut) {
    const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u > units) return;
    uint64_t t = 0;
    for (uint32_t p = 0; p < P; ++p) {
        const XbSrc s = src[p];
        t += S[s.off + (u << s.d)] - S[s.off];
    }
    ut[u] = t;
}

// KT u32: the table keeps the low `lowbits` (<= 31) bits of h, the unit index the rest; MAXP: senders
// whose runs fit the LDS run table.
template <int T, int FMAX, class KT, uint32_t MAXP>
__global__ void __launch_bounds__(MG_NT) kx_xb_merge(const uint64_t* __restrict__ in, const uint64_t* __restrict__ S,
                                                     const XbSrc* __restrict__ src, uint32_t P,
                                                     const uint64_t* __restrict__ ubase, PackFmt pf, Mix mx, uint64_t kmask,
                                                     uint64_t u_first, uint32_t lowbits,
                                                     uint32_t min_c, uint32_t pmul, uint64_t* __restrict__ wkey,
                                                     uint32_t* __restrict__ wcnt, uint64_t n,
                                                     uint64_t* __restrict__ kept, unsigned long long* __restrict__ gstat) {
    __shared__ MergeLds<T, FMAX, KT> L;
    __shared__ uint64_t rst[MAXP];        // address of sender p's run
    __shared__ uint32_t rpre[MAXP + 1];   // run lengths, exclusive prefix (a bucket holds < 2^32 pieces)
    const uint32_t u = blockIdx.x;
    const int tid = threadIdx.x;
    for (uint32_t p = tid; p < P; p += MG_NT) {
        const XbSrc s = src[p];
        const uint64_t a = S[s.off + ((uint64_t)u << s.d)];
        rst[p] = reinterpret_cast<uint64_t>(s.base + (a - S[s.off]));
        rpre[p + 1] = (uint32_t)(S[s.off + ((uint64_t)(u + 1) << s.d)] - a);
    }
    __syncthreads();
    if (tid < 64) {   // prefix over the senders, 64 at a time
        uint32_t carry = 0;
        for (uint32_t p0 = 0; p0 < P; p0 += 64) {
            const uint32_t p = p0 + tid;
            const uint32_t v = p < P ? rpre[p + 1] : 0u;
            const uint32_t inc = wave_incl_scan(v, tid);
            if (p < P) rpre[p + 1] = carry + inc;
            carry += __shfl(inc, 63, 64);
        }
        if (tid == 0) rpre[0] = 0;
    }
    __syncthreads();
    const uint64_t m = rpre[P];
    auto ld = [&](uint64_t i) {   // i-th piece of the bucket: sender run by binary search
        uint32_t lo = 0, hi = P;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (rpre[mid] <= i) lo = mid; else hi = mid;
        }
        // a global (not flat) load: flat loads count in lgkmcnt, so the next piece's binary search in
        // LDS would wait for this load
        return reinterpret_cast<const __attribute__((address_space(1))) uint64_t*>(rst[lo])[i - rpre[lo]];
    };
    const uint64_t hbase = sizeof(KT) == 4 ? (u_first + u) << lowbits : 0ull;
    merge_bucket<T, FMAX, true>(L, ld, m, ubase[u], u, pf, mx, sizeof(KT) == 4 ? (1ull << lowbits) - 1 : kmask, hbase,
                                min_c, pmul, wkey, wcnt, n, kept, gstat);
}

}  // namespace

// Bits per file count in the packed form (0 = not packable: use the wide exchange).
// (k and the file count only: no settle, so the exchange's fused head can still take an unsettled count)
int count_pack_bits(hga_ctx* c) {
    auto& s = c->count;
    const int kb = 2 * s.k;
    const int cb = s.n_files ? (64 - kb) / (int)s.n_files : 0;
    return (s.n_files <= 8 && cb >= 4) ? (cb > 32 ? 32 : cb) : 0;
}

// Packs this rank's rows by owner into `out` (capacity cap_out pieces).  Returns the number of
// pieces; if it exceeds cap_out nothing is written (the caller retries with more room).
uint64_t count_partition_packed(hga_ctx* c, const uint64_t* splitters, uint32_t n_own, uint64_t* out,
                                uint64_t cap_out, uint64_t* pieces_per_owner, bool sync_out) {
    auto& s = c->count;
    count_settle(c);
    HGA_REQUIRE(s.ran, HGA_ERR_STATE, "hga_count_run not called");
    count_dense(c);
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
    c->launch("kx_piece_hist", [&] {
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
    c->launch("kx_pack_scatter", [&] {
        hipLaunchKernelGGL(kx_pack_scatter, dim3(n_tiles), dim3(KX_T), 0, c->stream, s.rows_key.as<uint64_t>(),
                           s.rows_cnt.as<uint32_t>(), s.rows_cap, rows, spl, n_own, pf, hist, n_tiles, out);
    });
    c->check_launch("kx_pack_scatter");
    // the C entry point hands `out` to the caller; the exchange protocol's next use of it is ordered
    // on this stream (RCCL) or behind a synchronising copy (host transport)
    if (sync_out) c->sync();
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
    s.xb_on = false;
    s.dense_pending = false;
    if (n) {
        HGA_REQUIRE(pieces, HGA_ERR_INVALID, "input buffer required");
        // table slots per bucket (u64 key + F u32 counts): 32 KB for F <= 2, so four workgroups share a CU
        HGA_REQUIRE(n < (1ull << 32), HGA_ERR_INVALID, "at most 2^32-1 pieces per merge");
        const uint32_t T = F <= 2 ? 2048u : 1024u;
        const Mix mx = make_mix(s.k);
        int mb = 0;   // about T/2 pieces per bucket
        while (mb < MB_MAXB && mb < (int)mx.n && ((uint64_t)T / 2 << mb) < n) ++mb;
        const uint64_t nb = 1ull << mb;
        const uint64_t n_tiles = kx_blocks(n, MB_TILE);
        char* w = static_cast<char*>(s.xch2.ensure(n * (16 + 4 * F) + (3 * nb + 2) * 8 + 16 + 64));
        uint64_t* sk = reinterpret_cast<uint64_t*>(w);
        uint64_t* wkey = sk + n;                                     // rows per bucket range
        auto* tot = reinterpret_cast<unsigned long long*>(wkey + n);   // nb + 1: scanned = bucket starts
        auto* cursor = tot + nb + 1;
        auto* gstat = cursor + nb;
        uint64_t* kept = reinterpret_cast<uint64_t*>(gstat + 2);     // nb + 1: scanned = row offsets
        uint32_t* wcnt = reinterpret_cast<uint32_t*>(kept + nb + 1);
        HGA_HIP(hipMemsetAsync(tot, 0, (nb + 1) * 8, c->stream));
        c->launch("kx_mb_hist", [&] {
            hipLaunchKernelGGL(kx_mb_hist, dim3(n_tiles), dim3(MB_NT), 0, c->stream, pieces, n, kmask, mx, mb, tot);
        });
        c->check_launch("kx_mb_hist");
        exclusive_scan_u64(c, reinterpret_cast<uint64_t*>(tot), nb + 1, s.scratch);
        HGA_HIP(hipMemcpyAsync(cursor, tot, nb * 8, hipMemcpyDeviceToDevice, c->stream));
        c->launch("kx_mb_scatter", [&] {
            hipLaunchKernelGGL(kx_mb_scatter, dim3(n_tiles), dim3(MB_NT), 0, c->stream, pieces, n, kmask, mx, mb,
                               cursor, sk);
        });
        c->check_launch("kx_mb_scatter");
        const uint64_t* hist = reinterpret_cast<const uint64_t*>(tot);
        // one host round trip per attempt: the overflow flag and the row total come back together
        unsigned long long* hs = static_cast<unsigned long long*>(c->pinned.ensure(16));
        // HGA_MB_ONE_PASS: the first attempt sums every bucket in one pass, so a large one
        // overflows its table and the retry path runs (tests)
        for (uint32_t pmul = std::getenv("HGA_MB_ONE_PASS") ? 0u : 1u;; pmul = pmul ? pmul * 2 : 1u) {
            HGA_REQUIRE(pmul <= 256, HGA_ERR_OOM, "owner merge: a bucket does not fit its LDS table");
            HGA_HIP(hipMemsetAsync(gstat, 0, 16, c->stream));
            c->launch("kx_mb_merge", [&] {
                if (F <= 2)
                    hipLaunchKernelGGL((kx_mb_merge<2048, 2>), dim3(nb), dim3(MG_NT), 0, c->stream, sk, hist,
                                       pf, kmask, mb, min_c, pmul, wkey, wcnt, n, kept, gstat);
                else if (F <= 4)
                    hipLaunchKernelGGL((kx_mb_merge<1024, 4>), dim3(nb), dim3(MG_NT), 0, c->stream, sk, hist,
                                       pf, kmask, mb, min_c, pmul, wkey, wcnt, n, kept, gstat);
                else
                    hipLaunchKernelGGL((kx_mb_merge<1024, 8>), dim3(nb), dim3(MG_NT), 0, c->stream, sk, hist,
                                       pf, kmask, mb, min_c, pmul, wkey, wcnt, n, kept, gstat);
            });
            c->check_launch("kx_mb_merge");
            HGA_HIP(hipMemsetAsync(kept + nb, 0, 8, c->stream));
            exclusive_scan_u64(c, kept, nb + 1, s.scratch);
            c->launch("kx_mb_compact", [&] {
                hipLaunchKernelGGL(kx_mb_compact, dim3(nb), dim3(256), 0, c->stream, wkey, wcnt, n, F, hist, kept,
                                   s.rows_key.as<uint64_t>(), s.rows_cnt.as<uint32_t>(), cap);
            });
            c->check_launch("kx_mb_compact");
            HGA_HIP(hipMemcpyAsync(hs, kept + nb, 8, hipMemcpyDeviceToHost, c->stream));
            HGA_HIP(hipMemcpyAsync(hs + 1, gstat + 1, 8, hipMemcpyDeviceToHost, c->stream));
            c->sync();
            if (!hs[1]) break;
        }
        s.rows = hs[0];
    }
    s.min_per_file = min_c;
    s.ran = true;
    s.dist = false;
    s.n_sel = 0;
}

// ---- hash-bucket exchange (hga_count_exchange, exchange_protocol.hpp) ---------------------------
// Sender: this rank's rows as pieces in bucket order in `xsend`, the per-bucket counts in `xdir`,
// pieces per owner in per_owner[P]; returns the bucket resolution R (about 1024 pieces per owner
// bucket if every rank holds as many rows as this one, within [EB0, min(2k, XB_MAXR)]).
// Fast path, first half (enqueued, no host round trip): the count kernels' per-bucket piece counts
// scanned into the gather offsets and the per-owner totals written to d_per (P words, device or
// mapped memory).  False (nothing enqueued): the count kernels did not write the pieces.
// Owners hold whole count buckets (count_run checked fb >= EB0).
bool count_xb_pack_begin(hga_ctx* c, uint32_t P, uint64_t* d_per) {
    auto& s = c->count;
    HGA_REQUIRE(P >= 1 && P <= XB_MAXP, HGA_ERR_INVALID, "at most 1024 ranks");
    if (!(s.xb_on && s.xb_P == P)) return false;
    const int eb0 = std::min(10, 2 * s.k);
    const int fbc = s.xb_R - (int)s.xb_x;
    const uint64_t nbc = s.xb_nbc;
    uint64_t* S = static_cast<uint64_t*>(s.xch.ensure((nbc + 1) * 8 + 64));
    HGA_HIP(hipMemcpyAsync(S, s.xdir_b.p, nbc * 8, hipMemcpyDeviceToDevice, c->stream));
    HGA_HIP(hipMemsetAsync(S + nbc, 0, 8, c->stream));
    exclusive_scan_u64(c, S, nbc + 1, s.scratch);
    c->launch("kx_xb_pack", [&] {
        hipLaunchKernelGGL(kx_xb_owner_tot, dim3(kx_blocks(P, 256)), dim3(256), 0, c->stream, S, P, eb0, fbc, d_per);
    });
    c->check_launch("kx_xb_owner_tot");
    return true;
}

// Second half, once the count is settled and this rank's per-owner totals are on the host: the
// pieces gathered into owner order (xb_pieces) with their directory (xb_dir).  Returns R.
int count_xb_pack_finish(hga_ctx* c, uint32_t P, const uint64_t* per_owner) {
    auto& s = c->count;
    HGA_REQUIRE(s.ran, HGA_ERR_STATE, "hga_count_run not called");
    HGA_REQUIRE(s.xb_on && s.xb_P == P, HGA_ERR_STATE, "the count did not emit exchange pieces");
    const int R = s.xb_R;
    uint64_t total = 0;
    for (uint32_t o = 0; o < P; ++o) total += per_owner[o];
    HGA_REQUIRE(total < (1ull << 32), HGA_ERR_INVALID, "at most 2^32-1 pieces per rank");
    uint64_t* out = static_cast<uint64_t*>(s.xsend.ensure(std::max<uint64_t>(total, 1) * 8 + 64));
    uint64_t* dir = static_cast<uint64_t*>(s.xdir.ensure((8ull << R) + 64));
    c->launch("kx_xb_gather", [&] {
        hipLaunchKernelGGL(kx_xb_gather, dim3((unsigned)s.xb_nbc), dim3(256), 0, c->stream, s.xslab.as<uint64_t>(),
                           s.xb_fs, s.n_files, s.xb_x, 2 * s.k - R, s.xch.as<uint64_t>(), out, dir);
    });
    c->check_launch("kx_xb_gather");
    return R;
}

int count_xb_pack(hga_ctx* c, uint32_t P, uint64_t* per_owner) {
    auto& s = c->count;
    HGA_REQUIRE(P >= 1 && P <= XB_MAXP, HGA_ERR_INVALID, "at most 1024 ranks");
    const int eb0 = std::min(10, 2 * s.k);
    // the count kernels wrote the pieces: one host round trip, the count's counters and the
    // per-owner totals come back together
    auto* hp = static_cast<unsigned long long*>(s.xpack_h.ensure(8 * (8 + (uint64_t)P)));
    if (count_xb_pack_begin(c, P, reinterpret_cast<uint64_t*>(s.xpack_h.dev(hp + 8)))) {
        const bool pend = s.pending;
        if (pend) HGA_HIP(hipMemcpyAsync(hp, s.cursor.p, 64, hipMemcpyDeviceToHost, c->stream));
        c->sync();
        if (pend) count_settle(c, hp);
        for (uint32_t o = 0; o < P; ++o) per_owner[o] = hp[8 + o];
        return count_xb_pack_finish(c, P, per_owner);
    }
    count_settle(c);
    HGA_REQUIRE(s.ran, HGA_ERR_STATE, "hga_count_run not called");
    count_dense(c);
    const int cb = count_pack_bits(c);
    HGA_REQUIRE(cb > 0, HGA_ERR_INVALID, "rows of this k / file count do not pack into 64 bits");
    const PackFmt pf{2 * s.k, cb, s.n_files, (1ull << cb) - 1};
    const Mix mx = make_mix(s.k);
    const int rmax = std::min(2 * s.k, XB_MAXR);
    const uint64_t rows = s.rows;
    int R = eb0;
    while (R < rmax && ((uint64_t)1024 << R) < rows * P) ++R;
    if (const char* e = std::getenv("HGA_XB_R")) R = std::max(eb0, std::min(rmax, std::atoi(e)));   // test hook
    const uint64_t nb = 1ull << R;
    char* w = static_cast<char*>(s.xch.ensure((3 * nb + 2) * 8 + 8 * (uint64_t)P + 64));
    auto* tot = reinterpret_cast<unsigned long long*>(w);   // nb + 1: scanned = bucket starts
    auto* cursor = tot + nb + 1;
    uint64_t* per_d = reinterpret_cast<uint64_t*>(cursor + nb);
    uint64_t* dir = static_cast<uint64_t*>(s.xdir.ensure(nb * 8 + 64));
    HGA_HIP(hipMemsetAsync(tot, 0, (nb + 1) * 8, c->stream));
    const uint64_t n_tiles = kx_blocks(rows, XB_TILE);
    if (rows)
        c->launch("kx_xb_hist", [&] {
            hipLaunchKernelGGL(kx_xb_hist, dim3(n_tiles), dim3(XB_NT), 0, c->stream, s.rows_key.as<uint64_t>(),
                               s.rows_cnt.as<uint32_t>(), s.rows_cap, rows, pf, mx, R, tot);
        });
    c->check_launch("kx_xb_hist");
    HGA_HIP(hipMemcpyAsync(dir, tot, nb * 8, hipMemcpyDeviceToDevice, c->stream));
    exclusive_scan_u64(c, reinterpret_cast<uint64_t*>(tot), nb + 1, s.scratch);
    c->launch("kx_xb_pack", [&] {
        hipLaunchKernelGGL(kx_xb_owner_tot, dim3(kx_blocks(P, 256)), dim3(256), 0, c->stream,
                           reinterpret_cast<const uint64_t*>(tot), P, eb0, R, per_d);
    });
    c->check_launch("kx_xb_owner_tot");
    HGA_HIP(hipMemcpyAsync(per_owner, per_d, 8 * (uint64_t)P, hipMemcpyDeviceToHost, c->stream));
    c->sync();
    uint64_t total = 0;
    for (uint32_t o = 0; o < P; ++o) total += per_owner[o];
    HGA_REQUIRE(total < (1ull << 32), HGA_ERR_INVALID, "at most 2^32-1 pieces per rank");
    uint64_t* out = static_cast<uint64_t*>(s.xsend.ensure(std::max<uint64_t>(total, 1) * 8 + 64));
    if (rows) {
        HGA_HIP(hipMemcpyAsync(cursor, tot, nb * 8, hipMemcpyDeviceToDevice, c->stream));
        c->launch("kx_xb_scatter", [&] {
            hipLaunchKernelGGL(kx_xb_scatter, dim3(n_tiles), dim3(XB_NT), 0, c->stream, s.rows_key.as<uint64_t>(),
                               s.rows_cnt.as<uint32_t>(), s.rows_cap, rows, pf, mx, R, cursor, out);
        });
        c->check_launch("kx_xb_scatter");
    }
    return R;
}

// Owner: every sender's runs of this owner's buckets -> merged ctx rows (drop at min_c per file).
void count_xb_merge(hga_ctx* c, const uint64_t* in, const uint64_t* self, const uint64_t* n_from,
                    const uint64_t* dir_in, const int* r_from, uint32_t P, uint32_t me, uint32_t min_c) {
    auto& s = c->count;
    count_settle(c);
    HGA_REQUIRE(min_c >= 1, HGA_ERR_INVALID, "min_per_file must be >= 1");
    const int cb = count_pack_bits(c);
    const PackFmt pf{2 * s.k, cb, s.n_files, (1ull << cb) - 1};
    const uint64_t kmask = pf.kb >= 64 ? ~0ull : ((1ull << pf.kb) - 1);
    const uint32_t F = s.n_files;
    const Mix mx = make_mix(s.k);
    const int eb0 = std::min(10, 2 * s.k);
    auto first = [&](uint32_t o, int R) { return ((((uint64_t)o << eb0) + P - 1) / P) << (R - eb0); };
    int rmin = 64;
    for (uint32_t p = 0; p < P; ++p) {
        HGA_REQUIRE(r_from[p] >= eb0 && r_from[p] <= 2 * s.k, HGA_ERR_COMM, "exchange: bad bucket resolution");
        rmin = std::min(rmin, r_from[p]);
    }
    // the senders' run tables go up through mapped pinned memory (no pageable copy)
    XbSrc* src = static_cast<XbSrc*>(s.xsrc_h.ensure(sizeof(XbSrc) * P + 64));
    uint64_t n = 0, nd = 0, po = 0;
    for (uint32_t p = 0; p < P; ++p) {
        src[p] = XbSrc{nd, (uint32_t)(r_from[p] - rmin), 0, p == me ? self : in + po};
        nd += first(me + 1, r_from[p]) - first(me, r_from[p]);
        n += n_from[p];
        if (p != me) po += n_from[p];
    }
    HGA_REQUIRE(n < (1ull << 32), HGA_ERR_INVALID, "at most 2^32-1 pieces per merge");
    const uint64_t units = first(me + 1, rmin) - first(me, rmin);
    const uint64_t u_first = first(me, rmin);
    const uint32_t lowbits = 2u * (uint32_t)s.k - (uint32_t)rmin;
    const bool small = lowbits <= 31 && !std::getenv("HGA_XB_WIDE");   // u32 table keys (HGA_XB_WIDE: test hook)
    const bool big_units = units && n / units > 1100;   // about 2 K pieces per unit: a 4096-slot table
    const uint64_t cap = (std::max<uint64_t>(n, 1) + 3) & ~3ull;   // x4: 16-B row groups (kc_spec_hist)
    s.rows_key.ensure(cap * 8);
    s.rows_cnt.ensure(cap * 4 * F);
    s.rows = 0;
    s.rows_cap = cap;
    s.xb_on = false;
    s.dense_pending = false;
    // S (nd + 1) | ut = unit starts (units + 1) | kept (units + 1) | gstat 2 | wkey n | wcnt F n
    char* w = static_cast<char*>(s.xch2.ensure((nd + 1 + 2 * (units + 1) + 2 + n) * 8 + 4ull * F * n + 64));
    uint64_t* S = reinterpret_cast<uint64_t*>(w);
    uint64_t* ut = S + nd + 1;
    uint64_t* kept = ut + units + 1;
    auto* gstat = reinterpret_cast<unsigned long long*>(kept + units + 1);
    uint64_t* wkey = reinterpret_cast<uint64_t*>(gstat + 2);
    uint32_t* wcnt = reinterpret_cast<uint32_t*>(wkey + n);
    XbSrc* d_src = static_cast<XbSrc*>(s.xsrc.ensure(sizeof(XbSrc) * P + 64));
    HGA_HIP(hipMemcpyAsync(d_src, src, sizeof(XbSrc) * P, hipMemcpyHostToDevice, c->stream));
    if (nd) HGA_HIP(hipMemcpyAsync(S, dir_in, nd * 8, hipMemcpyDeviceToDevice, c->stream));
    HGA_HIP(hipMemsetAsync(S + nd, 0, 8, c->stream));
    exclusive_scan_u64(c, S, nd + 1, s.scratch);
    c->launch("kx_xb_units", [&] {
        hipLaunchKernelGGL(kx_xb_units, dim3(kx_blocks(units + 1, 256)), dim3(256), 0, c->stream, S, d_src, P, units,
                           ut);
    });
    c->check_launch("kx_xb_units");
    unsigned long long* hs = static_cast<unsigned long long*>(c->pinned.ensure(16));
    if (n) {
        // one host round trip per attempt: the overflow flag and the row total come back together
        for (uint32_t pmul = std::getenv("HGA_MB_ONE_PASS") ? 0u : 1u;; pmul = pmul ? pmul * 2 : 1u) {
            HGA_REQUIRE(pmul <= 256, HGA_ERR_OOM, "owner merge: a bucket does not fit its LDS table");
            HGA_HIP(hipMemsetAsync(gstat, 0, 16, c->stream));
            c->launch("kx_xb_merge", [&] {
#define HGA_XBM(TT, FM, KT, MP)                                                                             \
    hipLaunchKernelGGL((kx_xb_merge<TT, FM, KT, MP>), dim3(units), dim3(MG_NT), 0, c->stream, in, S, d_src, P, ut, pf, mx, \
                       kmask, u_first, lowbits, min_c, pmul, wkey, wcnt, n, kept, gstat)
                if (F <= 2 && small && P <= 64 && big_units) HGA_XBM(4096, 2, uint32_t, 64);
                else if (F <= 2 && small && P <= 64) HGA_XBM(2048, 2, uint32_t, 64);
                else if (F <= 2 && small) HGA_XBM(2048, 2, uint32_t, XB_MAXP);
                else if (F <= 2 && P <= 64) HGA_XBM(2048, 2, unsigned long long, 64);
                else if (F <= 2) HGA_XBM(2048, 2, unsigned long long, XB_MAXP);
                else if (F <= 4) HGA_XBM(1024, 4, unsigned long long, XB_MAXP);
                else HGA_XBM(1024, 8, unsigned long long, XB_MAXP);
#undef HGA_XBM
            });
            c->check_launch("kx_xb_merge");
            HGA_HIP(hipMemsetAsync(kept + units, 0, 8, c->stream));
            exclusive_scan_u64(c, kept, units + 1, s.scratch);
            c->launch("kx_mb_compact", [&] {
                hipLaunchKernelGGL(kx_mb_compact, dim3(units), dim3(256), 0, c->stream, wkey, wcnt, n, F, ut, kept,
                                   s.rows_key.as<uint64_t>(), s.rows_cnt.as<uint32_t>(), cap);
            });
            c->check_launch("kx_mb_compact");
            HGA_HIP(hipMemcpyAsync(hs, kept + units, 8, hipMemcpyDeviceToHost, c->stream));
            HGA_HIP(hipMemcpyAsync(hs + 1, gstat + 1, 8, hipMemcpyDeviceToHost, c->stream));
            c->sync();
            if (!hs[1]) break;
        }
        s.rows = hs[0];
    } else {
        c->sync();
    }
    s.min_per_file = min_c;
    s.ran = true;
    s.dist = false;
    s.n_sel = 0;
}

}  // namespace hga
