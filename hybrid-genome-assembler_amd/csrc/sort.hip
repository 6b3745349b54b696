// sort.hip — stable LSD radix sort and exclusive scans (gfx950, wave64).
//
// Used for everything that needs the reference's orders: the exported k-mers
// ascending (== LC_ALL=C order, run_jellyfish.sh:6), per-read sorted KmerID lists
// (ReadClusteringEngine.cpp:272) and kmer_component_index (:282-284).
//
// Per 8-bit digit pass: upsweep (per-tile digit histogram, digit-major so one
// linear exclusive scan gives every (digit, tile) output offset), scan, downsweep
// (stable in-tile rank via 64-lane ballot matching, staged through LDS so the global
// writes leave in digit runs).
#include <algorithm>
#include <cstdlib>

#include "hga_internal.hpp"
#include "kmer_dev.hpp"

namespace hga {
namespace {

constexpr int RS_T = 256;              // threads per tile
#ifndef HGA_RS_I
#define HGA_RS_I 16
#endif
constexpr int RS_I = HGA_RS_I;         // items per thread
constexpr int RS_TILE = RS_T * RS_I;   // 4096 keys per tile
constexpr int SC_T = 1024, SC_I = 4, SC_TILE = SC_T * SC_I;
#ifndef HGA_RS_MAX_DIGIT
#define HGA_RS_MAX_DIGIT 10
#endif
#ifndef HGA_LBW
#define HGA_LBW 8   // predecessor tiles read per look-back step (independent loads per digit thread)
#endif

// dmask: the pass's digit mask (the last pass may cover fewer than 8 bits: bits above the sort
// width are payload and must not order the keys).
template <class K, int DB>
__global__ void __launch_bounds__(RS_T) rs_upsweep(const K* __restrict__ keys, uint64_t n,
                                                   int shift, uint32_t dmask, uint32_t* __restrict__ counts,
                                                   uint32_t n_tiles) {
    constexpr int NB = 1 << DB;
    __shared__ uint32_t h[NB];
    for (int d = threadIdx.x; d < NB; d += RS_T) h[d] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
#pragma unroll
    for (int j = 0; j < RS_I; ++j) {
        uint64_t i = base + (uint64_t)j * RS_T + threadIdx.x;
        if (i < n) atomicAdd(&h[(uint32_t)(keys[i] >> shift) & dmask], 1u);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < NB; d += RS_T) counts[(uint64_t)d * n_tiles + blockIdx.x] = h[d];
}

// DB-bit digits (DB = 8 .. 11): NB = 2^DB bins, each thread owns NB / RS_T consecutive digits in
// the tile's digit scan.
template <class K, bool HAS_V, int DB>
__global__ void __launch_bounds__(RS_T) rs_downsweep(const K* __restrict__ kin,
                                                     const uint32_t* __restrict__ vin,
                                                     K* __restrict__ kout,
                                                     uint32_t* __restrict__ vout, uint64_t n,
                                                     int shift, uint32_t dmask,
                                                     const uint32_t* __restrict__ offs,
                                                     uint32_t n_tiles) {
    constexpr uint32_t NB = 1u << DB;
    constexpr int DPT = (int)NB / RS_T;
    static_assert(DPT >= 1, "at least one digit per thread");
    __shared__ uint32_t wcnt[4][NB];
    __shared__ uint32_t dstart[NB];
    __shared__ uint32_t ws[8];
    __shared__ K sk[RS_TILE];
    __shared__ uint32_t sv[HAS_V ? RS_TILE : 1];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (uint32_t i = tid; i < 4 * NB; i += RS_T) (&wcnt[0][0])[i] = 0;
    __syncthreads();

    const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
    const uint64_t lt = (1ull << lane) - 1ull;
    K key[RS_I];
    uint32_t val[RS_I];
    uint32_t dig[RS_I];
    uint32_t rank[RS_I];
#pragma unroll
    for (int j = 0; j < RS_I; ++j) {
        const uint64_t i = base + (uint64_t)wave * (RS_I * 64) + (uint64_t)j * 64 + lane;
        const bool ok = i < n;
        key[j] = ok ? kin[i] : K(0);
        if (HAS_V) val[j] = ok ? vin[i] : 0u;
        dig[j] = ok ? ((uint32_t)(key[j] >> shift) & dmask) : NB;
    }
    // Stable rank inside the wave: items in (j, lane) order.
#pragma unroll
    for (int j = 0; j < RS_I; ++j) {
        const uint32_t d = dig[j];
        const bool ok = d < NB;
        uint64_t m = __ballot(ok);
#pragma unroll
        for (int b = 0; b < DB; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            m &= bit ? bb : ~bb;
        }
        uint32_t before = 0;
        if (ok) before = wcnt[wave][d];
        rank[j] = before + (uint32_t)__popcll(m & lt);
        if (ok && (m & lt) == 0ull) wcnt[wave][d] = before + (uint32_t)__popcll(m);
        wave_lds_sync();
    }
    __syncthreads();
    // digit starts inside the tile, then per-wave starts
    {
        uint32_t c[DPT][4];
        uint32_t sum = 0;
#pragma unroll
        for (int q = 0; q < DPT; ++q) {
            const uint32_t d = tid * DPT + q;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                c[q][w] = wcnt[w][d];
                sum += c[q][w];
            }
        }
        uint32_t tot;
        uint32_t run = block_excl_scan<RS_T>(sum, ws, &tot);
#pragma unroll
        for (int q = 0; q < DPT; ++q) {
            const uint32_t d = tid * DPT + q;
            dstart[d] = run;
            wcnt[0][d] = run;
            wcnt[1][d] = run + c[q][0];
            wcnt[2][d] = run + c[q][0] + c[q][1];
            wcnt[3][d] = run + c[q][0] + c[q][1] + c[q][2];
            run += c[q][0] + c[q][1] + c[q][2] + c[q][3];
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RS_I; ++j) {
        if (dig[j] < NB) {
            const uint32_t lp = wcnt[wave][dig[j]] + rank[j];
            sk[lp] = key[j];
            if (HAS_V) sv[lp] = val[j];
        }
    }
    __syncthreads();
    const uint32_t cnt = (uint32_t)((n - base) < (uint64_t)RS_TILE ? (n - base) : RS_TILE);
    for (uint32_t i = tid; i < cnt; i += RS_T) {
        const K kk = sk[i];
        const uint32_t d = (uint32_t)(kk >> shift) & dmask;
        const uint64_t g = (uint64_t)offs[(uint64_t)d * n_tiles + blockIdx.x] + (i - dstart[d]);
        kout[g] = kk;
        if (HAS_V) vout[g] = sv[i];
    }
}

// ---- onesweep: one histogram kernel for all passes, then ONE kernel per pass ----------------
// Each tile takes the next tile id (atomic), ranks its keys stably in LDS as above, publishes
// its per-digit count, and looks back over earlier tiles (decoupled look-back) for its
// exclusive prefix per digit.  Status words carry flag + value in one 32-bit granule: agent-
// scope relaxed atomic stores/loads (sc1), the hand-off MI355X_MICROARCH.md lists for a flag
// that is its own payload.  A tile only waits on tiles with smaller ids, which are running.
constexpr uint32_t LB_A = 1u << 30, LB_P = 2u << 30, LB_M = (1u << 30) - 1;

template <class K>
__global__ void __launch_bounds__(RS_T) rs_hist_all(const K* __restrict__ keys, uint64_t n, int passes, int bits,
                                                    uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[8][256];
    for (int i = threadIdx.x; i < 8 * 256; i += RS_T) (&h[0][0])[i] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * RS_T + threadIdx.x; i < n; i += (uint64_t)gridDim.x * RS_T) {
        const K k = keys[i];
        for (int p = 0; p < passes; ++p) {
            const int w = bits - 8 * p < 8 ? bits - 8 * p : 8;
            atomicAdd(&h[p][(uint32_t)(k >> (8 * p)) & ((1u << w) - 1u)], 1u);
        }
    }
    __syncthreads();
    for (int p = 0; p < passes; ++p) {
        const uint32_t v = h[p][threadIdx.x];
        if (v) atomicAdd(&hist[p * 256 + threadIdx.x], v);
    }
}

template <class K, bool HAS_V>
__global__ void __launch_bounds__(RS_T) rs_onesweep(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                    K* __restrict__ kout, uint32_t* __restrict__ vout, uint64_t n,
                                                    int shift, uint32_t dmask, const uint32_t* __restrict__ ghist,
                                                    uint32_t* __restrict__ status, uint32_t* __restrict__ tile_ctr,
                                                    uint32_t dbase = 0u) {
    __shared__ uint32_t wcnt[4][256];
    __shared__ uint32_t gofs[256];
    __shared__ uint32_t ws[8];
    __shared__ uint32_t s_tile;
    __shared__ K sk[RS_TILE];
    __shared__ uint32_t sv[HAS_V ? RS_TILE : 1];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(tile_ctr, 1u);
    for (int i = tid; i < 4 * 256; i += RS_T) (&wcnt[0][0])[i] = 0;
    uint32_t gtot;
    const uint32_t gstart = block_excl_scan<RS_T>(ghist[tid], ws, &gtot);   // digit tid's global start
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t base = (uint64_t)tile * RS_TILE;
    const uint64_t lt = (1ull << lane) - 1ull;
    K key[RS_I];
    uint32_t val[RS_I];
    uint32_t dig[RS_I];
    uint32_t rank[RS_I];
#pragma unroll
    for (int j = 0; j < RS_I; ++j) {
        const uint64_t i = base + (uint64_t)wave * (RS_I * 64) + (uint64_t)j * 64 + lane;
        const bool ok = i < n;
        key[j] = ok ? kin[i] : K(0);
        if (HAS_V) val[j] = ok ? vin[i] : 0u;
        dig[j] = ok ? (((uint32_t)(key[j] >> shift) - dbase) & dmask) : 256u;
    }
#pragma unroll
    for (int j = 0; j < RS_I; ++j) {
        const uint32_t d = dig[j];
        const bool ok = d < 256u;
        uint64_t m = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            m &= bit ? bb : ~bb;
        }
        uint32_t before = 0;
        if (ok) before = wcnt[wave][d];
        rank[j] = before + (uint32_t)__popcll(m & lt);
        if (ok && (m & lt) == 0ull) wcnt[wave][d] = before + (uint32_t)__popcll(m);
        wave_lds_sync();
    }
    __syncthreads();
    {
        const int d = tid;
        const uint32_t c0 = wcnt[0][d], c1 = wcnt[1][d], c2 = wcnt[2][d], c3 = wcnt[3][d];
        const uint32_t c = c0 + c1 + c2 + c3;
        uint32_t tot;
        const uint32_t ex = block_excl_scan<RS_T>(c, ws, &tot);
        wcnt[0][d] = ex;
        wcnt[1][d] = ex + c0;
        wcnt[2][d] = ex + c0 + c1;
        wcnt[3][d] = ex + c0 + c1 + c2;
        uint32_t* st = status + (uint64_t)tile * 256 + d;
        uint32_t excl = 0;
        if (tile == 0) {
            __hip_atomic_store(st, LB_P | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(st, LB_A | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // look back LBW tiles per step (independent loads), newest first; restart at the
            // first tile that has not published yet
            constexpr int LBW = HGA_LBW;
            int64_t t = (int64_t)tile - 1;
            while (true) {
                uint32_t v[LBW];
#pragma unroll
                for (int i = 0; i < LBW; ++i)
                    v[i] = t - i >= 0 ? __hip_atomic_load(status + (uint64_t)(t - i) * 256 + d, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT)
                                      : LB_P;   // before tile 0: an empty inclusive prefix
                int stop = LBW;   // 0..LBW-1: index of a P (done) or an unpublished tile (wait)
                bool done = false;
#pragma unroll
                for (int i = LBW - 1; i >= 0; --i) {
                    const uint32_t f = v[i] & ~LB_M;
                    if (f == 0u || f == LB_P) { stop = i; done = f == LB_P; }
                }
                for (int i = 0; i < stop; ++i) excl += v[i] & LB_M;   // all A
                if (stop < LBW && done) {
                    excl += v[stop] & LB_M;
                    break;
                }
                t -= stop;   // stop == LBW: all A, continue further back; else wait on tile t - stop
            }
            __hip_atomic_store(st, LB_P | (excl + c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        gofs[d] = gstart + excl - ex;   // element at in-tile sorted index i, digit d -> gofs[d] + i
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RS_I; ++j) {
        if (dig[j] < 256u) {
            const uint32_t lp = wcnt[wave][dig[j]] + rank[j];
            sk[lp] = key[j];
            if (HAS_V) sv[lp] = val[j];
        }
    }
    __syncthreads();
    const uint32_t cnt = (uint32_t)((n - base) < (uint64_t)RS_TILE ? (n - base) : RS_TILE);
    for (uint32_t i = tid; i < cnt; i += RS_T) {
        const K kk = sk[i];
        const uint64_t g = (uint64_t)gofs[((uint32_t)(kk >> shift) - dbase) & dmask] + i;
        kout[g] = kk;
        if (HAS_V) vout[g] = sv[i];
    }
}

// ---- export sort: one MSD digit pass, then every digit's segment sorted in LDS --------------
// The exported k-mers (count_select) are ~10^6-10^7 keys of 2k <= 62 bits: one onesweep pass on
// the top 8 bits of the sort width scatters them into 256 segments, each of which one workgroup
// sorts in LDS by the remaining bits (stable LSD passes over 8-bit digits: ballot-matched ranks
// inside each wave, waves in order), instead of ceil(2k/8) global passes.  Segments larger than
// the LDS (rare: a prefix holding > 16384 keys) are sorted by the global radix sort.
// (SS_T / SS_I / SS_CAP and lds_lsd_sort live in kmer_dev.hpp: count.hip sorts export segments with them too)

__global__ void __launch_bounds__(SS_T) ss_segsort(const uint64_t* __restrict__ kin, uint64_t* __restrict__ kout,
                                                   const uint32_t* __restrict__ ghist, int bits_low) {
    __shared__ uint64_t sk[SS_CAP];
    __shared__ uint32_t wcnt[SS_T / 64][256];
    __shared__ uint32_t ws[SS_T / 64 + 1];
    __shared__ uint32_t s_start, s_cnt;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t seg = blockIdx.x;
    {   // this segment's start: exclusive prefix of the digit totals
        uint32_t tot;
        const uint32_t h = tid < 256 ? ghist[tid] : 0u;
        const uint32_t ex = block_excl_scan<SS_T>(h, ws, &tot);
        if (tid == (int)seg) {
            s_start = ex;
            s_cnt = h;
        }
        __syncthreads();
    }
    const uint32_t start = s_start, cnt = s_cnt;
    if (cnt == 0 || cnt > (uint32_t)SS_CAP) return;   // empty, or left to the global fallback
    uint64_t key[SS_I];
#pragma unroll
    for (int j = 0; j < SS_I; ++j) {
        const uint32_t i = (uint32_t)wave * (SS_I * 64) + (uint32_t)j * 64 + lane;
        key[j] = i < cnt ? kin[(uint64_t)start + i] : 0ull;
    }
    lds_lsd_sort(key, cnt, bits_low, sk, wcnt, ws);
#pragma unroll
    for (int j = 0; j < SS_I; ++j) {
        const uint32_t i = (uint32_t)wave * (SS_I * 64) + (uint32_t)j * 64 + lane;
        if (i < cnt) kout[(uint64_t)start + i] = key[j];
    }
}

// ---- exclusive scans --------------------------------------------------------------
// Single-pass exclusive scan (chained scan with decoupled look-back, one launch, kmer_dev.hpp
// chained_lookback): each workgroup takes the next tile id from a counter that only grows (tile =
// counter - the value at launch), scans its SC_TILE elements, publishes its aggregate and then its
// inclusive prefix.
template <class T>
__global__ void __launch_bounds__(SC_T) sc_onepass(T* data, uint64_t n, unsigned long long* __restrict__ status,
                                                   unsigned long long* __restrict__ ctr, uint64_t tbase,
                                                   uint32_t epoch) {
    __shared__ uint64_t ws[SC_T / 64];
    __shared__ uint64_t s_tile, s_pre;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_tile = atomicAdd(ctr, 1ull) - tbase;
    __syncthreads();
    const uint64_t tile = s_tile;
    const uint64_t base = tile * SC_TILE + (uint64_t)threadIdx.x * SC_I;
    uint64_t v[SC_I];
    uint64_t sum = 0;
#pragma unroll
    for (int j = 0; j < SC_I; ++j) {
        v[j] = base + j < n ? (uint64_t)data[base + j] : 0ull;
        sum += v[j];
    }
    const uint64_t inc = wave_incl_scan64(sum, lane);
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t agg = 0;
        for (int w = 0; w < SC_T / 64; ++w) {
            const uint64_t x = ws[w];
            ws[w] = agg;
            agg += x;
        }
        s_pre = chained_lookback(status, tile, agg, epoch);
    }
    __syncthreads();
    uint64_t run = s_pre + ws[wave] + inc - sum;
#pragma unroll
    for (int j = 0; j < SC_I; ++j) {
        if (base + j < n) data[base + j] = (T)run;
        run += v[j];
    }
}

}  // namespace

// Status words and tile ids for nt tiles of one chained scan (chained_lookback): a fresh epoch, the
// tile counter's value at launch.
ScanTicket scan_ticket(hga_ctx* c, uint64_t nt) {
    const size_t need = 256 + nt * 8;
    const bool fresh = need > c->scan_state.cap;
    auto* st = static_cast<unsigned long long*>(c->scan_state.ensure(std::max<size_t>(need, 1 << 16)));
    if (fresh) {   // a new allocation: zero words are unpublished under every epoch; the counter restarts
        HGA_HIP(hipMemsetAsync(st, 0, c->scan_state.cap, c->stream));
        c->scan_tiles = 0;
    }
    if (++c->scan_epoch == SCS_EPOCHS) {   // wrap: clear the words of old scans
        HGA_HIP(hipMemsetAsync(st + 32, 0, c->scan_state.cap - 256, c->stream));
        c->scan_epoch = 1;
    }
    ScanTicket t{st + 32, st, c->scan_tiles, c->scan_epoch};   // first 256 B: the tile counter
    c->scan_tiles += nt;
    return t;
}

namespace {

template <class T>
void excl_scan_impl(hga_ctx* c, T* data, uint64_t n) {
    if (n == 0) return;
    const uint64_t nt = (n + SC_TILE - 1) / SC_TILE;
    const ScanTicket t = scan_ticket(c, nt);
    c->launch("scan", [&] {
        hipLaunchKernelGGL(sc_onepass<T>, dim3((unsigned)nt), dim3(SC_T), 0, c->stream, data, n, t.status, t.ctr,
                           t.tbase, t.epoch);
    });
    c->check_launch("sc_onepass");
}

// n below which the onesweep path is used (env HGA_ONESWEEP_MAX overrides per call; 0 disables).
// Widest radix digit of the classic (upsweep / scan / downsweep) passes: HGA_RS_MAX_DIGIT, 8..11.
inline int rs_max_digit() {
    const char* e = std::getenv("HGA_RS_MAX_DIGIT");
    const int v = e ? std::atoi(e) : HGA_RS_MAX_DIGIT;
    return v < 8 ? 8 : (v > 11 ? 11 : v);
}
inline uint64_t hga_onesweep_max() {
    const char* e = std::getenv("HGA_ONESWEEP_MAX");
    return e ? (uint64_t)std::strtoull(e, nullptr, 10) : (uint64_t)(4ull << 20);
}

// src_k / src_v (optional): read the first pass from these instead of keys / vals (saves the copy
// of an input that must stay intact); the result always ends in keys / vals.
template <class K>
void radix_sort_impl(hga_ctx* c, K* keys, uint32_t* vals, uint64_t n, int bits, DevBuf& scratch,
                     const K* src_k = nullptr, const uint32_t* src_v = nullptr) {
    if (src_k && (n <= 1 || bits <= 0)) {
        if (n) {
            HGA_HIP(hipMemcpyAsync(keys, src_k, n * sizeof(K), hipMemcpyDeviceToDevice, c->stream));
            if (vals) HGA_HIP(hipMemcpyAsync(vals, src_v, n * 4, hipMemcpyDeviceToDevice, c->stream));
        }
        return;
    }
    if (n <= 1 || bits <= 0) return;
    HGA_REQUIRE(n < (1ull << 32), HGA_ERR_INVALID, "radix sort: n >= 2^32");
    const uint32_t n_tiles = (uint32_t)((n + RS_TILE - 1) / RS_TILE);
    const int npass = (bits + 7) / 8;
    const bool one = n < (uint64_t)hga_onesweep_max() && npass <= 8;
    // classic passes: 8-bit digits, or one pass of up to rs_max_digit() bits
    // (9..10 bits: one wide pass instead of 8 + 1-2; wider keys keep 8-bit digits — 10-bit passes
    // measured slower per key, C4's 27-bit export sort 2.67 -> 3.16 ms in three of them)
    int db = 8;
    if (!one && bits > 8 && bits <= rs_max_digit()) db = bits;
    const uint64_t n_cnt = ((uint64_t)1 << db) * n_tiles;
    const size_t kb = ((n * sizeof(K) + 255) & ~255ull);
    const size_t vb = vals ? ((n * 4 + 255) & ~255ull) : 0;
    const size_t cb = ((n_cnt * 4 + 255) & ~255ull);
    char* base = static_cast<char*>(scratch.ensure(kb + vb + cb));
    K* k2 = reinterpret_cast<K*>(base);
    uint32_t* v2 = vals ? reinterpret_cast<uint32_t*>(base + kb) : nullptr;
    uint32_t* cnt = reinterpret_cast<uint32_t*>(base + kb + vb);
    K* ka = keys;
    K* kbuf = k2;
    uint32_t* va = vals;
    uint32_t* vbuf = v2;
    // onesweep where launch count dominates (small n); the classic pass is faster per byte
    if (one) {
        const size_t hb = (size_t)npass * 256 * 4, stb = (size_t)npass * n_tiles * 256 * 4, tcb = 64;
        char* ob = static_cast<char*>(scratch.ensure(kb + vb + hb + stb + tcb));
        K* k2o = reinterpret_cast<K*>(ob);
        uint32_t* v2o = vals ? reinterpret_cast<uint32_t*>(ob + kb) : nullptr;
        uint32_t* hist = reinterpret_cast<uint32_t*>(ob + kb + vb);
        uint32_t* status = reinterpret_cast<uint32_t*>(ob + kb + vb + hb);
        uint32_t* tctr = reinterpret_cast<uint32_t*>(ob + kb + vb + hb + stb);
        HGA_HIP(hipMemsetAsync(hist, 0, hb + stb + tcb, c->stream));
        const unsigned hgrid = (unsigned)std::min<uint64_t>(n_tiles, (uint64_t)c->num_cu * 2);
        c->launch("radix_upsweep", [&] {
            hipLaunchKernelGGL(rs_hist_all<K>, dim3(hgrid), dim3(RS_T), 0, c->stream, src_k ? src_k : keys, n, npass,
                               bits, hist);
        });
        c->check_launch("rs_hist_all");
        // buffers by pass: [src,] then alternating so that the last pass writes keys when possible
        K* ka2 = keys;
        K* kb2 = k2o;
        uint32_t* va2 = vals;
        uint32_t* vb2 = v2o;
        if (src_k) {
            ka2 = const_cast<K*>(src_k);
            va2 = const_cast<uint32_t*>(src_v);
            kb2 = (npass & 1) ? keys : k2o;
            vb2 = (npass & 1) ? vals : v2o;
        }
        for (int p = 0; p < npass; ++p) {
            const uint32_t dm = bits - 8 * p >= 8 ? 255u : ((1u << (bits - 8 * p)) - 1u);
            c->launch("radix_downsweep", [&] {
                if (vals)
                    hipLaunchKernelGGL((rs_onesweep<K, true>), dim3(n_tiles), dim3(RS_T), 0, c->stream, ka2, va2, kb2,
                                       vb2, n, 8 * p, dm, hist + p * 256, status + (size_t)p * n_tiles * 256, tctr + p);
                else
                    hipLaunchKernelGGL((rs_onesweep<K, false>), dim3(n_tiles), dim3(RS_T), 0, c->stream, ka2,
                                       (const uint32_t*)nullptr, kb2, (uint32_t*)nullptr, n, 8 * p, dm, hist + p * 256,
                                       status + (size_t)p * n_tiles * 256, tctr + p);
            });
            c->check_launch("rs_onesweep");
            if (src_k && p == 0) {   // the source is never written: continue between keys and k2o
                ka2 = kb2;
                va2 = vb2;
                kb2 = ka2 == keys ? k2o : keys;
                vb2 = va2 == vals ? v2o : vals;
                continue;
            }
            std::swap(ka2, kb2);
            std::swap(va2, vb2);
        }
        if (ka2 != keys) {
            HGA_HIP(hipMemcpyAsync(keys, ka2, n * sizeof(K), hipMemcpyDeviceToDevice, c->stream));
            if (vals) HGA_HIP(hipMemcpyAsync(vals, va2, n * 4, hipMemcpyDeviceToDevice, c->stream));
        }
        return;
    }
    if (src_k) {
        const int np = (bits + db - 1) / db;
        ka = const_cast<K*>(src_k);
        va = const_cast<uint32_t*>(src_v);
        kbuf = (np & 1) ? keys : k2;
        vbuf = (np & 1) ? vals : v2;
    }
    for (int shift = 0; shift < bits; shift += db) {
        const uint32_t dm = bits - shift >= db ? (1u << db) - 1u : ((1u << (bits - shift)) - 1u);
        c->launch("radix_upsweep", [&] {
            switch (db) {
            case 8: hipLaunchKernelGGL((rs_upsweep<K, 8>), dim3(n_tiles), dim3(RS_T), 0, c->stream, ka, n, shift, dm, cnt, n_tiles); break;
            case 9: hipLaunchKernelGGL((rs_upsweep<K, 9>), dim3(n_tiles), dim3(RS_T), 0, c->stream, ka, n, shift, dm, cnt, n_tiles); break;
            case 10: hipLaunchKernelGGL((rs_upsweep<K, 10>), dim3(n_tiles), dim3(RS_T), 0, c->stream, ka, n, shift, dm, cnt, n_tiles); break;
            default: hipLaunchKernelGGL((rs_upsweep<K, 11>), dim3(n_tiles), dim3(RS_T), 0, c->stream, ka, n, shift, dm, cnt, n_tiles); break;
            }
        });
        c->check_launch("rs_upsweep");
        excl_scan_impl<uint32_t>(c, cnt, n_cnt);
        c->launch("radix_downsweep", [&] {
            if (vals) {
                switch (db) {
                case 8: hipLaunchKernelGGL((rs_downsweep<K, true, 8>), dim3(n_tiles), dim3(RS_T), 0, c->stream, ka, va, kbuf, vbuf, n, shift, dm, cnt, n_tiles); break;
                case 9: hipLaunchKernelGGL((rs_downsweep<K, true, 9>), dim3(n_tiles), dim3(RS_T), 0, c->stream, ka, va, kbuf, vbuf, n, shift, dm, cnt, n_tiles); break;
                case 10: hipLaunchKernelGGL((rs_downsweep<K, true, 10>), dim3(n_tiles), dim3(RS_T), 0, c->stream, ka, va, kbuf, vbuf, n, shift, dm, cnt, n_tiles); break;
                default: hipLaunchKernelGGL((rs_downsweep<K, true, 11>), dim3(n_tiles), dim3(RS_T), 0, c->stream, ka, va, kbuf, vbuf, n, shift, dm, cnt, n_tiles); break;
                }
            } else {
                const uint32_t* nv = nullptr;
                uint32_t* nvo = nullptr;
                switch (db) {
                case 8: hipLaunchKernelGGL((rs_downsweep<K, false, 8>), dim3(n_tiles), dim3(RS_T), 0, c->stream, ka, nv, kbuf, nvo, n, shift, dm, cnt, n_tiles); break;
                case 9: hipLaunchKernelGGL((rs_downsweep<K, false, 9>), dim3(n_tiles), dim3(RS_T), 0, c->stream, ka, nv, kbuf, nvo, n, shift, dm, cnt, n_tiles); break;
                case 10: hipLaunchKernelGGL((rs_downsweep<K, false, 10>), dim3(n_tiles), dim3(RS_T), 0, c->stream, ka, nv, kbuf, nvo, n, shift, dm, cnt, n_tiles); break;
                default: hipLaunchKernelGGL((rs_downsweep<K, false, 11>), dim3(n_tiles), dim3(RS_T), 0, c->stream, ka, nv, kbuf, nvo, n, shift, dm, cnt, n_tiles); break;
                }
            }
        });
        c->check_launch("rs_downsweep");
        if (src_k && shift == 0) {   // the source is never written: continue between keys and k2
            ka = kbuf;
            va = vbuf;
            kbuf = ka == keys ? k2 : keys;
            vbuf = va == vals ? v2 : vals;
            continue;
        }
        std::swap(ka, kbuf);
        std::swap(va, vbuf);
    }
    if (ka != keys) {
        HGA_HIP(hipMemcpyAsync(keys, ka, n * sizeof(K), hipMemcpyDeviceToDevice, c->stream));
        if (vals) HGA_HIP(hipMemcpyAsync(vals, va, n * 4, hipMemcpyDeviceToDevice, c->stream));
    }
}

}  // namespace

void radix_sort_u64(hga_ctx* c, uint64_t* keys, uint32_t* vals, uint64_t n, int bits,
                    DevBuf& scratch) {
    radix_sort_impl<uint64_t>(c, keys, vals, n, bits, scratch);
}
// keys: n keys, all with ((key >> shift) - dbase) in [0, 256) (the MSD digit; bits of key above the
// sort width are payload and vanish in the 8-bit difference), d_hist / h_hist: the device / host
// copies of the 256 digit counts.  Sorted in place by the digit, then by the low `shift` bits.
void sort_export_u64(hga_ctx* c, uint64_t* keys, uint64_t n, int shift, uint32_t dbase, const uint32_t* d_hist,
                     const uint32_t* h_hist, DevBuf& scratch) {
    if (n <= 1) return;
    HGA_REQUIRE(shift >= 0 && shift <= 54 && n < (1ull << 32), HGA_ERR_INVALID, "export sort: bad width");
    uint32_t n_big = 0;
    for (int d = 0; d < 256; ++d) n_big += h_hist[d] > (uint32_t)SS_CAP;
    // Many segments past the LDS (a large export, e.g. a C4 rank shard's): one global LSD sort of
    // the low `shift` bits first, then the stable digit pass below finishes the order.
    const bool global_low = n_big > 8;
    if (global_low && shift > 0) radix_sort_u64(c, keys, nullptr, n, shift, scratch);
    const uint32_t n_tiles = (uint32_t)((n + RS_TILE - 1) / RS_TILE);
    const size_t kb = ((n * 8 + 255) & ~255ull), stb = (size_t)n_tiles * 256 * 4, tcb = 64;
    char* base = static_cast<char*>(scratch.ensure(kb + stb + tcb));
    uint64_t* k2 = reinterpret_cast<uint64_t*>(base);
    uint32_t* status = reinterpret_cast<uint32_t*>(base + kb);
    uint32_t* tctr = reinterpret_cast<uint32_t*>(base + kb + stb);
    HGA_HIP(hipMemsetAsync(status, 0, stb + tcb, c->stream));
    c->launch("radix_downsweep", [&] {
        hipLaunchKernelGGL((rs_onesweep<uint64_t, false>), dim3(n_tiles), dim3(RS_T), 0, c->stream, keys,
                           (const uint32_t*)nullptr, k2, (uint32_t*)nullptr, n, shift, 255u, d_hist, status, tctr,
                           dbase);
    });
    c->check_launch("rs_onesweep");
    if (global_low) {
        HGA_HIP(hipMemcpyAsync(keys, k2, n * 8, hipMemcpyDeviceToDevice, c->stream));
        return;
    }
    c->launch("radix_segsort", [&] {
        hipLaunchKernelGGL(ss_segsort, dim3(256), dim3(SS_T), 0, c->stream, k2, keys, d_hist, shift);
    });
    c->check_launch("ss_segsort");
    uint64_t st = 0;
    for (int d = 0; d < 256; ++d) {   // segments too large for one workgroup's LDS
        if (h_hist[d] > (uint32_t)SS_CAP) {
            DevBuf tmp;
            if (shift > 0) radix_sort_u64(c, k2 + st, nullptr, h_hist[d], shift, tmp);
            HGA_HIP(hipMemcpyAsync(keys + st, k2 + st, (size_t)h_hist[d] * 8, hipMemcpyDeviceToDevice, c->stream));
            c->sync();   // tmp is freed on return
        }
        st += h_hist[d];
    }
}
void radix_sort_u64_from(hga_ctx* c, const uint64_t* src_k, uint64_t* keys, uint64_t n, int bits, DevBuf& scratch) {
    radix_sort_impl<uint64_t>(c, keys, nullptr, n, bits, scratch, src_k, nullptr);
}
void radix_sort_u32(hga_ctx* c, uint32_t* keys, uint32_t* vals, uint64_t n, int bits,
                    DevBuf& scratch) {
    radix_sort_impl<uint32_t>(c, keys, vals, n, bits > 32 ? 32 : bits, scratch);
}
void radix_sort_u32_from(hga_ctx* c, const uint32_t* src_k, const uint32_t* src_v, uint32_t* keys, uint32_t* vals,
                         uint64_t n, int bits, DevBuf& scratch) {
    radix_sort_impl<uint32_t>(c, keys, vals, n, bits > 32 ? 32 : bits, scratch, src_k, src_v);
}
// Exclusive scan in place.  Contract: the total stays below 2^40 (the look-back status words carry
// 40-bit values; a larger total wraps, it never hangs).  Every caller scans counts of elements of
// HBM-resident arrays (at most a few 10^9).
void exclusive_scan_u64(hga_ctx* c, uint64_t* data, uint64_t n, DevBuf& scratch) {
    (void)scratch;   // the single-pass scan keeps its state in the ctx
    excl_scan_impl<uint64_t>(c, data, n);
}

}  // namespace hga
