// lookup.hip — MI355X replacement for the per-read SDK lookup loop of
// ReadClusteringEngine::construct_indices (src/clustering/ReadClusteringEngine.cpp:234-299).
//
//   lk_build      read-only open-addressing table {canonical code -> KmerID}
//                 (the host assigns KmerIDs in std::unordered_set order, :237-241).
//   lk_scan<false> per thread 32 consecutive window ends of the concatenated reads:
//                 KmerIterator-exact rolling code (non-ACGT -> 0 on both strands),
//                 window never crosses a read, probe; per-thread hit counts (u8) and
//                 per-tile totals.
//   lk_scan<true> same walk, writes (read, KmerID, end-exclusive position) in read /
//                 window order at block-scanned offsets (no sort needed for hit order).
//   post          CSR pointers, stable radix sorts for the per-read sorted KmerID lists
//                 (:272) and first positions (:267), and kmer_component_index (:282-284).
#include <algorithm>

#include "hga_internal.hpp"
#include "kmer_dev.hpp"

namespace hga {
namespace {

constexpr int LK_T = 256;
constexpr int LK_P = 32;
constexpr uint64_t LK_TILE = (uint64_t)LK_T * LK_P;
constexpr uint64_t EMPTY_KEY = ~0ull;   // never canonical: min(fwd, rc) of all-T is 0

__device__ __forceinline__ uint64_t tab_hash(uint64_t x) {
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 32;
    return x;
}

__global__ void lk_fill(uint64_t* __restrict__ k, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) k[i] = EMPTY_KEY;
}

__global__ void lk_build(const uint64_t* __restrict__ keys, uint32_t n, uint64_t* __restrict__ tk,
                         uint32_t* __restrict__ tid, uint64_t smask) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t key = keys[i];
    uint64_t slot = tab_hash(key) & smask;
    while (true) {
        const unsigned long long old = atomicCAS((unsigned long long*)&tk[slot],
                                                 (unsigned long long)EMPTY_KEY,
                                                 (unsigned long long)key);
        if (old == EMPTY_KEY || old == key) { tid[slot] = i; return; }
        slot = (slot + 1) & smask;
    }
}

__device__ __forceinline__ int lk_probe(const uint64_t* __restrict__ tk, uint64_t smask, uint64_t key,
                                        uint64_t& slot_out) {
    uint64_t slot = tab_hash(key) & smask;
    while (true) {
        const uint64_t t = tk[slot];
        if (t == key) { slot_out = slot; return 1; }
        if (t == EMPTY_KEY) return 0;
        slot = (slot + 1) & smask;
    }
}

template <bool EMIT>
__global__ void __launch_bounds__(LK_T) lk_scan(const uint8_t* __restrict__ bases, uint64_t nbases,
                                                const uint64_t* __restrict__ offs, uint64_t nreads,
                                                int k, const uint64_t* __restrict__ tk,
                                                const uint32_t* __restrict__ tids, uint64_t smask,
                                                uint8_t* __restrict__ tcnt,
                                                unsigned long long* __restrict__ tile_cnt,
                                                uint32_t* __restrict__ h_read,
                                                uint32_t* __restrict__ h_kid,
                                                uint32_t* __restrict__ h_pos) {
    __shared__ uint32_t ws[LK_T / 64 + 1];
    const uint64_t gt = (uint64_t)blockIdx.x * LK_T + threadIdx.x;
    const uint64_t p0 = gt * LK_P;
    uint32_t mycnt = 0;
    uint64_t obase = 0;
    if (EMIT) {
        mycnt = p0 < nbases ? tcnt[gt] : 0u;
        uint32_t tot;
        const uint32_t ex = block_excl_scan<LK_T>(mycnt, ws, &tot);
        obase = tile_cnt[blockIdx.x] + ex;
        if (mycnt == 0) return;
    }
    uint32_t found = 0;
    if (p0 < nbases) {
        // read containing p0: last r with offs[r] <= p0
        uint64_t lo = 0, hi = nreads;   // offs[lo] <= p0 < offs[hi]
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) >> 1;
            if (offs[mid] <= p0) lo = mid; else hi = mid;
        }
        uint64_t r = lo;
        uint64_t rs = offs[r], re = offs[r + 1];
        const uint64_t pe = p0 + LK_P < nbases ? p0 + LK_P : nbases;
        uint64_t q = p0 >= (uint64_t)(k - 1) ? p0 - (uint64_t)(k - 1) : 0;
        if (q < rs) q = rs;
        const uint64_t mask = k >= 32 ? ~0ull : ((1ull << (2 * k)) - 1);
        const int sh = 2 * (k - 1);
        uint64_t fwd = 0, rc = 0;
        int run = 0;
        for (uint64_t cb = q & ~15ull; cb < pe; cb += 16) {
            const uint4 v = load16(bases, (int64_t)cb, nbases);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint64_t e = cb + j;
                if (e < q || e >= pe) continue;
                if (e >= re) {   // entering the next non-empty read
                    do { ++r; } while (offs[r + 1] <= e);
                    rs = offs[r];
                    re = offs[r + 1];
                    run = 0;
                }
                uint32_t fc, rcc;
                ref_codes((w[j >> 2] >> (8 * (j & 3))) & 0xFFu, fc, rcc);
                fwd = ((fwd << 2) | fc) & mask;
                rc = (rc >> 2) | ((uint64_t)rcc << sh);
                ++run;
                if (e >= p0 && run >= k) {
                    const uint64_t canon = fwd < rc ? fwd : rc;
                    uint64_t slot;
                    if (lk_probe(tk, smask, canon, slot)) {
                        if (EMIT) {
                            const uint64_t o = obase + found;
                            h_read[o] = (uint32_t)r;
                            h_kid[o] = tids[slot];
                            h_pos[o] = (uint32_t)(e + 1 - rs);
                        }
                        ++found;
                    }
                }
            }
        }
    }
    if (!EMIT) {
        if (p0 < nbases) tcnt[gt] = (uint8_t)found;
        uint32_t tot;
        (void)block_excl_scan<LK_T>(found, ws, &tot);
        if (threadIdx.x == 0) tile_cnt[blockIdx.x] = tot;
    }
}

// ptr[s] = first index i with idx[i] >= s (CSR over a sorted segment-id array),
// ptr[nseg] = H.  *nonempty += number of distinct segment ids.
__global__ void lk_ptr(const uint32_t* __restrict__ idx, uint64_t H, uint64_t nseg,
                       uint64_t* __restrict__ ptr, unsigned long long* __restrict__ nonempty) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > H) return;
    const uint64_t lo = i == 0 ? 0 : (uint64_t)idx[i - 1] + 1;
    const uint64_t hi = i == H ? nseg : (uint64_t)idx[i];
    for (uint64_t s = lo; s <= hi; ++s) ptr[s] = i;
    if (i < H && (i == 0 || idx[i] != idx[i - 1])) atomicAdd(nonempty, 1ull);
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
    uint64_t slots = 1024;
    while (slots < 2ull * n) slots <<= 1;
    L.slots = slots;
    L.k = k;
    L.n_sdk = n;
    uint64_t* tk = static_cast<uint64_t*>(L.tab_key.ensure(slots * 8));
    uint32_t* ti = static_cast<uint32_t*>(L.tab_id.ensure(slots * 4));
    DevBuf tmp;
    uint64_t* dk = static_cast<uint64_t*>(tmp.ensure(std::max<uint64_t>(n, 1) * 8));
    if (n) HGA_HIP(hipMemcpyAsync(dk, keys, (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(lk_fill, dim3(blocks_for(slots, 256)), dim3(256), 0, c->stream, tk, slots);
    c->check_launch("lk_fill");
    if (n) {
        c->launch("lk_build", [&] {
            hipLaunchKernelGGL(lk_build, dim3(blocks_for(n, 256)), dim3(256), 0, c->stream, dk, n, tk,
                               ti, slots - 1);
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
    const uint64_t nb = n ? offsets[n] - offsets[0] : 0;
    HGA_REQUIRE(offsets[0] == 0 || n == 0, HGA_ERR_INVALID, "offsets[0] must be 0");
    for (uint64_t i = 0; i < n; ++i)
        HGA_REQUIRE(offsets[i + 1] >= offsets[i], HGA_ERR_INVALID, "offsets must be non-decreasing");
    L.n_reads = n;
    L.n_bases = nb;
    L.first_read_id = first_id;
    void* db = L.bases.ensure(nb + 16);
    void* dof = L.offsets.ensure((n + 1) * 8);
    if (nb) HGA_HIP(hipMemcpyAsync(db, bases, nb, hipMemcpyHostToDevice, c->stream));
    HGA_HIP(hipMemcpyAsync(dof, offsets, (n + 1) * 8, hipMemcpyHostToDevice, c->stream));
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
    uint8_t* tcnt = static_cast<uint8_t*>(L.scratch.ensure(std::max<uint64_t>(n_threads, 1) + 256));
    auto* tile = static_cast<unsigned long long*>(L.tile_cnt.ensure((n_tiles + 1) * 8));
    const uint8_t* bases = L.bases.as<uint8_t>();
    const uint64_t* offs = L.offsets.as<uint64_t>();
    const uint64_t smask = L.slots - 1;
    uint64_t H = 0;
    if (n_tiles) {
        c->launch("lk_count", [&] {
            hipLaunchKernelGGL(lk_scan<false>, dim3((unsigned)n_tiles), dim3(LK_T), 0, c->stream, bases,
                               nb, offs, n, k, L.tab_key.as<uint64_t>(), L.tab_id.as<uint32_t>(), smask,
                               tcnt, tile, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr);
        });
        c->check_launch("lk_count");
        HGA_HIP(hipMemsetAsync(tile + n_tiles, 0, 8, c->stream));
        DevBuf sc;
        exclusive_scan_u64(c, reinterpret_cast<uint64_t*>(tile), n_tiles + 1, sc);
        HGA_HIP(hipMemcpyAsync(&H, tile + n_tiles, 8, hipMemcpyDeviceToHost, c->stream));
        c->sync();
    }
    L.hits = H;
    uint32_t* hr = static_cast<uint32_t*>(L.hit_read.ensure(std::max<uint64_t>(H, 1) * 4));
    uint32_t* hk = static_cast<uint32_t*>(L.hit_kid.ensure(std::max<uint64_t>(H, 1) * 4));
    uint32_t* hp = static_cast<uint32_t*>(L.hit_pos.ensure(std::max<uint64_t>(H, 1) * 4));
    if (H) {
        c->launch("lk_emit", [&] {
            hipLaunchKernelGGL(lk_scan<true>, dim3((unsigned)n_tiles), dim3(LK_T), 0, c->stream, bases, nb,
                               offs, n, k, L.tab_key.as<uint64_t>(), L.tab_id.as<uint32_t>(), smask, tcnt,
                               tile, hr, hk, hp);
        });
        c->check_launch("lk_emit");
    }
    // hit_ptr over reads
    auto* ctr = static_cast<unsigned long long*>(L.first_flag.ensure(64));
    HGA_HIP(hipMemsetAsync(ctr, 0, 16, c->stream));
    uint64_t* hptr = static_cast<uint64_t*>(L.hit_ptr.ensure((n + 1) * 8));
    c->launch("lk_post", [&] {
        hipLaunchKernelGGL(lk_ptr, dim3(blocks_for(H + 1, 256)), dim3(256), 0, c->stream, hr, H, n, hptr,
                           ctr);
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
        DevBuf sc;
        exclusive_scan_u64(c, flag, H + 1, sc);
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
                           U ? L.first_read.as<uint32_t>() : (const uint32_t*)nullptr, U, n, fptr, ctr + 2);
        hipLaunchKernelGGL(lk_ptr, dim3(blocks_for(H + 1, 256)), dim3(256), 0, c->stream,
                           H ? L.kci_key.as<uint32_t>() : (const uint32_t*)nullptr, H, (uint64_t)L.n_sdk,
                           kptr, ctr + 3);
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
