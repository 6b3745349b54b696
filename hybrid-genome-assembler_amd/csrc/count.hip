// count.hip — MI355X k-mer counting: the replacement for `jellyfish count -C --bc`
// + `dump` + `sort` (src/occurrences/run_jellyfish.sh:3-6) and for the two string
// k-way merge passes of JellyfishOccurrenceReader (JellyfishOccurrenceReader.cpp:63-135).
//
// Pipeline (all HBM-bound integer work, no MFMA):
//   A  kc_hist   per super-tile: scan the resident sequence bytes, canonical k-mer of
//                every valid window, bijective 2k-bit mix, LDS histogram of the top
//                fb bits (bucket) -> one row of st_hist[super-tile][bucket].
//   S  kc_scan_cols / kc_bucket_scan / kc_file_start: column prefix sums -> every
//                (super-tile, bucket) output offset; bucket-major, file-minor layout.
//   B  kc_bin    recompute the windows, rank them inside a tile by bucket through
//                LDS, write each bucket's run contiguously (coalesced) as the mixed
//                value's low bits (u32 when 2k - fb <= 31).
//   C  kc_count  one workgroup per bucket: LDS open-addressing table keyed by the
//                remainder with one u32 counter per file; adaptive sub-range splitting
//                if a bucket holds more distinct k-mers than the table; per-file drop
//                of counts < min (jellyfish --bc); emit merged rows (key, counts[F]).
//   H  kc_spec_hist   specificity x total histogram (get_specificity, :88-108).
//   X  kc_select      rows with lower <= total <= upper, + radix sort ascending
//                     (export_kmers, :110-135; numeric order == LC_ALL=C order).
#include <algorithm>
#include <map>

#include "hga_internal.hpp"
#include "kmer_dev.hpp"

namespace hga {
namespace {

constexpr int NT_AB = 1024;   // threads of pass A / B workgroups
constexpr int P_AB = 16;      // window ends per thread per tile (u32 elements)
constexpr int NT_B64 = 512;   // pass B workgroup for u64 elements (LDS budget)
constexpr uint64_t TILE_POS = (uint64_t)NT_AB * P_AB;  // 16384
constexpr int MAX_FB = 12;
constexpr int MAX_NB = 1 << MAX_FB;
constexpr int NT_C = 512;     // threads of the per-bucket count workgroup
constexpr uint32_t LDS_TAB = 128 * 1024;

struct KP {
    int k, sh;
    uint64_t mask;
    Mix mix;
    uint32_t fb, rbits, nb;
    uint64_t rmask;
};

__device__ __forceinline__ uint32_t bucket_of(uint64_t h, const KP& kp) {
    return kp.fb ? (uint32_t)(h >> kp.rbits) : 0u;
}

// ---------------------------------------------------------------- pass A
__global__ void __launch_bounds__(NT_AB) kc_hist(const uint8_t* __restrict__ s, uint64_t n,
                                                 uint64_t st_pos, uint32_t st0, KP kp,
                                                 uint32_t* __restrict__ st_hist,
                                                 unsigned long long* __restrict__ instances) {
    __shared__ uint32_t hist[MAX_NB];
    __shared__ uint32_t ws[NT_AB / 64 + 1];
    const int tid = threadIdx.x;
    for (uint32_t b = tid; b < kp.nb; b += NT_AB) hist[b] = 0;
    __syncthreads();
    const uint64_t start = (uint64_t)blockIdx.x * st_pos;
    const uint64_t end = start + st_pos < n ? start + st_pos : n;
    uint32_t cnt = 0;
    for (uint64_t t0 = start; t0 < end; t0 += TILE_POS) {
        const uint64_t p0 = t0 + (uint64_t)tid * P_AB;
        scan_count_windows<P_AB>(s, n, p0, kp.k, kp.mask, kp.sh, [&](uint64_t canon, int) {
            const uint64_t h = mix_fwd(canon, kp.mix);
            atomicAdd(&hist[bucket_of(h, kp)], 1u);
            ++cnt;
        });
    }
    uint32_t tot;
    (void)block_excl_scan<NT_AB>(cnt, ws, &tot);
    if (tid == 0 && tot) atomicAdd(instances, (unsigned long long)tot);
    uint32_t* row = st_hist + (uint64_t)(st0 + blockIdx.x) * kp.nb;
    for (uint32_t b = tid; b < kp.nb; b += NT_AB) row[b] = hist[b];
}

// ---------------------------------------------------------------- scans
// In place: st_hist[st][b] -> exclusive prefix over st; row n_st receives the totals.
__global__ void kc_scan_cols(uint32_t* __restrict__ st, uint32_t n_st, uint32_t nb) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    uint32_t run = 0;
    uint32_t i = 0;
    for (; i + 4 <= n_st; i += 4) {
        const uint32_t v0 = st[(uint64_t)(i + 0) * nb + b], v1 = st[(uint64_t)(i + 1) * nb + b];
        const uint32_t v2 = st[(uint64_t)(i + 2) * nb + b], v3 = st[(uint64_t)(i + 3) * nb + b];
        st[(uint64_t)(i + 0) * nb + b] = run; run += v0;
        st[(uint64_t)(i + 1) * nb + b] = run; run += v1;
        st[(uint64_t)(i + 2) * nb + b] = run; run += v2;
        st[(uint64_t)(i + 3) * nb + b] = run; run += v3;
    }
    for (; i < n_st; ++i) {
        const uint32_t v = st[(uint64_t)i * nb + b];
        st[(uint64_t)i * nb + b] = run;
        run += v;
    }
    st[(uint64_t)n_st * nb + b] = run;
}

// bucket_base[b] = Σ_{b'<b} totals[b'] (u64), bucket_base[nb] = grand total.
__global__ void __launch_bounds__(1024) kc_bucket_scan(const uint32_t* __restrict__ totals,
                                                       uint32_t nb, uint64_t* __restrict__ base) {
    __shared__ uint64_t ws[17];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint64_t v[4], s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t b = tid * 4 + i;
        v[i] = b < nb ? totals[b] : 0ull;
        s += v[i];
    }
    const uint64_t inc = wave_incl_scan64(s, lane);
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    if (tid == 0) {
        uint64_t t = 0;
        for (int w = 0; w < 16; ++w) { uint64_t x = ws[w]; ws[w] = t; t += x; }
        ws[16] = t;
    }
    __syncthreads();
    uint64_t run = ws[wave] + inc - s;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t b = tid * 4 + i;
        if (b < nb) base[b] = run;
        run += v[i];
    }
    if (tid == 0) base[nb] = ws[16];
}

// fs[b*(F+1)+f] = start of file f's run inside bucket b; fs[b*(F+1)+F] = bucket end.
__global__ void kc_file_start(const uint32_t* __restrict__ st_off, const uint64_t* __restrict__ base,
                              const uint32_t* __restrict__ st_first, uint32_t F, uint32_t nb,
                              uint64_t* __restrict__ fs) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    for (uint32_t f = 0; f < F; ++f)
        fs[(uint64_t)b * (F + 1) + f] = base[b] + st_off[(uint64_t)st_first[f] * nb + b];
    fs[(uint64_t)b * (F + 1) + F] = base[b + 1];
}

// ---------------------------------------------------------------- pass B
template <class E, int P, int NT>
__global__ void __launch_bounds__(NT) kc_bin(const uint8_t* __restrict__ s, uint64_t n,
                                                uint64_t st_pos, uint32_t st0, KP kp,
                                                const uint64_t* __restrict__ bucket_base,
                                                const uint32_t* __restrict__ st_off,
                                                E* __restrict__ out) {
    __shared__ uint64_t run[MAX_NB];
    __shared__ uint32_t off[MAX_NB + 1];
    __shared__ E stage[P * NT];
    __shared__ uint16_t sbk[P * NT];
    __shared__ uint32_t ws[NT / 64 + 1];
    const int tid = threadIdx.x;
    const uint32_t nb = kp.nb;
    const uint32_t* row = st_off + (uint64_t)(st0 + blockIdx.x) * nb;
    for (uint32_t b = tid; b < nb; b += NT) {
        run[b] = bucket_base[b] + row[b];
        off[b] = 0;
    }
    __syncthreads();
    const uint64_t start = (uint64_t)blockIdx.x * st_pos;
    const uint64_t end = start + st_pos < n ? start + st_pos : n;
    constexpr uint64_t TP = (uint64_t)P * NT;
    constexpr int BPT = MAX_NB / NT;   // bins per thread in the scan
    for (uint64_t t0 = start; t0 < end; t0 += TP) {
        const uint64_t p0 = t0 + (uint64_t)tid * P;
        uint32_t bk[P], rk[P];
        E rr[P];
        uint32_t vm = 0;
#pragma unroll
        for (int j = 0; j < P; ++j) { bk[j] = 0; rr[j] = 0; rk[j] = 0; }
        scan_count_windows<P>(s, n, p0, kp.k, kp.mask, kp.sh, [&](uint64_t canon, int j) {
            const uint64_t h = mix_fwd(canon, kp.mix);
            bk[j] = bucket_of(h, kp);
            rr[j] = (E)(h & kp.rmask);
            vm |= 1u << j;
        });
#pragma unroll
        for (int j = 0; j < P; ++j)
            if ((vm >> j) & 1u) rk[j] = atomicAdd(&off[bk[j]], 1u);
        __syncthreads();
        {   // exclusive scan of off[0..nb) in place, off[nb] = tile total
            uint32_t v[BPT], sm = 0;
#pragma unroll
            for (int i = 0; i < BPT; ++i) {
                const uint32_t b = tid * BPT + i;
                v[i] = b < nb ? off[b] : 0u;
                sm += v[i];
            }
            uint32_t tot;
            uint32_t ex = block_excl_scan<NT>(sm, ws, &tot);
#pragma unroll
            for (int i = 0; i < BPT; ++i) {
                const uint32_t b = tid * BPT + i;
                if (b < nb) off[b] = ex;
                ex += v[i];
            }
            if (tid == 0) off[nb] = tot;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < P; ++j)
            if ((vm >> j) & 1u) {
                const uint32_t pos = off[bk[j]] + rk[j];
                stage[pos] = rr[j];
                sbk[pos] = (uint16_t)bk[j];
            }
        __syncthreads();
        const uint32_t tot = off[nb];
        for (uint32_t i = tid; i < tot; i += NT) {
            const uint32_t b = sbk[i];
            out[run[b] + (i - off[b])] = stage[i];
        }
        __syncthreads();
        for (uint32_t b = tid; b < nb; b += NT) run[b] += off[b + 1] - off[b];
        __syncthreads();
        for (uint32_t b = tid; b < nb; b += NT) off[b] = 0;
        __syncthreads();
    }
}

// ---------------------------------------------------------------- pass C
// gstat: [0] output cursor, [1] max sub-ranges any bucket needed, [2] error bits
// (1 = unsplittable overflow, 2 = output capacity exceeded).
template <class E>
__global__ void __launch_bounds__(NT_C) kc_count(const E* __restrict__ binned,
                                                 const uint64_t* __restrict__ fs, uint32_t F,
                                                 uint32_t T, uint32_t maxload, uint32_t min_count,
                                                 KP kp, uint64_t* __restrict__ out_key,
                                                 uint32_t* __restrict__ out_cnt, uint64_t cap,
                                                 unsigned long long* __restrict__ gstat) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_TAB];
    __shared__ uint32_t s_occ, s_ovf, s_sp, s_ranges;
    __shared__ uint32_t stk_lo[40], stk_hi[40];
    __shared__ uint32_t ws[NT_C / 64 + 1];
    __shared__ unsigned long long s_base;
    E* keys = reinterpret_cast<E*>(smem);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(smem + (size_t)T * sizeof(E));
    const int tid = threadIdx.x;
    const uint32_t b = blockIdx.x;
    const uint64_t* f = fs + (uint64_t)b * (F + 1);
    const E EMPTY = ~E(0);
    const uint32_t rbits = kp.rbits;
    const uint32_t SUBB = rbits < 16 ? rbits : 16;
    const uint32_t full_hi = 1u << SUBB;
    const uint32_t mc = min_count ? min_count : 1u;
    if (tid == 0) {
        stk_lo[0] = 0;
        stk_hi[0] = full_hi;
        s_sp = 1;
        s_ranges = 0;
    }
    __syncthreads();
    while (true) {
        const uint32_t sp = s_sp;
        if (sp == 0) break;
        const uint32_t lo = stk_lo[sp - 1], hi = stk_hi[sp - 1];
        __syncthreads();
        if (tid == 0) {
            s_sp = sp - 1;
            s_occ = 0;
            s_ovf = 0;
        }
        for (uint32_t i = tid; i < T; i += NT_C) keys[i] = EMPTY;
        for (uint32_t i = tid; i < F * T; i += NT_C) cnt[i] = 0;
        __syncthreads();
        const bool filt = !(lo == 0 && hi == full_hi);
        for (uint32_t ff = 0; ff < F; ++ff) {
            const uint64_t a = f[ff], e = f[ff + 1];
            uint32_t* cf = cnt + (size_t)ff * T;
            for (uint64_t i = a + tid; i < e; i += NT_C) {
                if (*(volatile uint32_t*)&s_ovf) break;
                const E r = binned[i];
                if (filt) {
                    const uint32_t sk = SUBB ? (uint32_t)(r >> (rbits - SUBB)) : 0u;
                    if (sk < lo || sk >= hi) continue;
                }
                uint32_t slot = (uint32_t)r & (T - 1);
                while (true) {
                    const E cur = keys[slot];
                    if (cur == r) { atomicAdd(&cf[slot], 1u); break; }
                    if (cur == EMPTY) {
                        const E old = atomicCAS(&keys[slot], EMPTY, r);
                        if (old == EMPTY) {
                            const uint32_t o = atomicAdd(&s_occ, 1u);
                            if (o + 1 >= maxload) s_ovf = 1;
                            atomicAdd(&cf[slot], 1u);
                            break;
                        }
                        if (old == r) { atomicAdd(&cf[slot], 1u); break; }
                    }
                    slot = (slot + 1) & (T - 1);
                }
            }
        }
        __syncthreads();
        if (s_ovf) {
            __syncthreads();
            if (tid == 0) {
                if (hi - lo <= 1 || s_sp + 2 > 40) {
                    atomicOr(&gstat[2], 1ull);
                    s_sp = 0;
                } else {
                    const uint32_t mid = lo + (hi - lo) / 2;
                    stk_lo[s_sp] = mid; stk_hi[s_sp] = hi;
                    stk_lo[s_sp + 1] = lo; stk_hi[s_sp + 1] = mid;
                    s_sp += 2;
                }
            }
            __syncthreads();
            continue;
        }
        // emit the rows of this sub-range
        uint32_t mine = 0;
        for (uint32_t i = tid; i < T; i += NT_C) {
            if (keys[i] == EMPTY) continue;
            bool any = false;
            for (uint32_t ff = 0; ff < F; ++ff) any |= cnt[(size_t)ff * T + i] >= mc;
            mine += any;
        }
        uint32_t tot;
        const uint32_t ex = block_excl_scan<NT_C>(mine, ws, &tot);
        if (tid == 0) {
            s_base = tot ? atomicAdd(&gstat[0], (unsigned long long)tot) : 0ull;
            ++s_ranges;
        }
        __syncthreads();
        uint64_t o = s_base + ex;
        if (o + mine > cap) {
            if (mine) atomicOr(&gstat[2], 2ull);
        } else {
            for (uint32_t i = tid; i < T; i += NT_C) {
                const E r = keys[i];
                if (r == EMPTY) continue;
                bool any = false;
                for (uint32_t ff = 0; ff < F; ++ff) any |= cnt[(size_t)ff * T + i] >= mc;
                if (!any) continue;
                const uint64_t h = (kp.fb ? ((uint64_t)b << rbits) : 0ull) | (uint64_t)r;
                out_key[o] = mix_inv(h, kp.mix);
                for (uint32_t ff = 0; ff < F; ++ff) {
                    const uint32_t c = cnt[(size_t)ff * T + i];
                    out_cnt[(size_t)ff * cap + o] = c >= mc ? c : 0u;
                }
                ++o;
            }
        }
        __syncthreads();
    }
    if (tid == 0) atomicMax(&gstat[1], (unsigned long long)s_ranges);
}

// ---------------------------------------------------------------- histogram / select
constexpr int NT_H = 256;
constexpr uint32_t TL = 1024;         // LDS-privatised totals
constexpr uint32_t TD = 1u << 16;     // dense global totals; beyond -> overflow list
constexpr uint32_t MAX_THR = 16;

__global__ void __launch_bounds__(NT_H) kc_spec_hist(const uint32_t* __restrict__ cnt, uint64_t rows,
                                                     uint64_t cap, uint32_t F,
                                                     const double* __restrict__ thr, uint32_t n_thr,
                                                     unsigned long long* __restrict__ hist,
                                                     unsigned long long* __restrict__ over,
                                                     unsigned long long* __restrict__ over_cur,
                                                     uint64_t over_cap,
                                                     unsigned long long* __restrict__ err) {
    __shared__ uint32_t lh[MAX_THR * TL];
    __shared__ double sthr[MAX_THR];
    for (uint32_t i = threadIdx.x; i < n_thr * TL; i += NT_H) lh[i] = 0;
    if (threadIdx.x < n_thr) sthr[threadIdx.x] = thr[threadIdx.x];
    __syncthreads();
    for (uint64_t r = (uint64_t)blockIdx.x * NT_H + threadIdx.x; r < rows;
         r += (uint64_t)gridDim.x * NT_H) {
        uint64_t total = 0;
        uint32_t prev = 0;
        for (uint32_t f = 0; f < F; ++f) {
            const uint32_t c = cnt[(size_t)f * cap + r];
            total += c;
            prev = c > prev ? c : prev;
        }
        // ((double)prevalent / (double)total) * 100, IEEE round-to-nearest, no FMA
        const double x = __dmul_rn(__ddiv_rn((double)prev, (double)total), 100.0);
        uint32_t ti = 0;
        while (ti < n_thr && !(sthr[ti] > x)) ++ti;   // std::set::upper_bound
        if (ti >= n_thr) { atomicOr(err, 1ull); continue; }
        if (total < TL) atomicAdd(&lh[ti * TL + (uint32_t)total], 1u);
        else if (total < TD) atomicAdd(&hist[(uint64_t)ti * TD + total], 1ull);
        else {
            const unsigned long long o = atomicAdd(over_cur, 1ull);
            if (o < over_cap) over[o] = ((unsigned long long)ti << 56) | total;
            else atomicOr(err, 2ull);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n_thr * TL; i += NT_H) {
        const uint32_t v = lh[i];
        if (v) atomicAdd(&hist[(uint64_t)(i / TL) * TD + (i % TL)], (unsigned long long)v);
    }
}

__global__ void __launch_bounds__(NT_H) kc_select(const uint64_t* __restrict__ keys,
                                                  const uint32_t* __restrict__ cnt, uint64_t rows,
                                                  uint64_t cap, uint32_t F, int64_t lower,
                                                  int64_t upper, uint64_t* __restrict__ out,
                                                  uint32_t* __restrict__ out_flag,
                                                  unsigned long long* __restrict__ stat) {
    __shared__ uint32_t ws[NT_H / 64 + 1];
    __shared__ unsigned long long s_base;
    const uint64_t r = (uint64_t)blockIdx.x * NT_H + threadIdx.x;
    bool take = false, disc = false;
    uint64_t key = 0;
    if (r < rows) {
        int64_t total = 0;
        uint32_t nz = 0;
        for (uint32_t f = 0; f < F; ++f) {
            const uint32_t c = cnt[(size_t)f * cap + r];
            total += c;
            nz += c > 0;
        }
        take = lower <= total && total <= upper;
        disc = take && nz == 1;
        key = keys[r];
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan<NT_H>(take ? 1u : 0u, ws, &tot);
    const uint64_t dm = __ballot(disc);
    if ((threadIdx.x & 63) == 0 && dm) atomicAdd(&stat[1], (unsigned long long)__popcll(dm));
    if (threadIdx.x == 0) s_base = tot ? atomicAdd(&stat[0], (unsigned long long)tot) : 0ull;
    __syncthreads();
    if (take) {
        out[s_base + ex] = key;
        out_flag[s_base + ex] = disc ? 1u : 0u;
    }
}

__global__ void kc_iota(uint32_t* v, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}

__global__ void kc_gather_rows(const uint32_t* __restrict__ idx, const uint32_t* __restrict__ cnt,
                               uint64_t rows, uint64_t cap, uint32_t F, uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows) return;
    const uint32_t src = idx[i];
    for (uint32_t f = 0; f < F; ++f) out[i * F + f] = cnt[(size_t)f * cap + src];
}

inline unsigned blocks_for(uint64_t n, int t) { return (unsigned)((n + t - 1) / t); }

}  // namespace

// ================================================================ host side

void count_begin(hga_ctx* c, int k, uint32_t n_files) {
    HGA_REQUIRE(k >= 1 && k <= 32, HGA_ERR_INVALID, "k must be in [1,32]");
    HGA_REQUIRE(n_files >= 1 && n_files <= 64, HGA_ERR_INVALID, "n_files must be in [1,64]");
    auto& s = c->count;
    for (auto* b : s.seq) delete b;
    s.seq.clear();
    s.seq_len.assign(n_files, 0);
    for (uint32_t i = 0; i < n_files; ++i) s.seq.push_back(new DevBuf());
    s.k = k;
    s.n_files = n_files;
    s.begun = true;
    s.ran = false;
    s.rows = s.instances = s.n_sel = 0;
}

void count_add(hga_ctx* c, uint32_t file, const char* seq, uint64_t n) {
    auto& s = c->count;
    HGA_REQUIRE(s.begun, HGA_ERR_STATE, "hga_count_begin not called");
    HGA_REQUIRE(file < s.n_files, HGA_ERR_INVALID, "file index out of range");
    if (n == 0) return;
    // A separator byte between calls keeps windows from spanning two calls.
    const uint64_t old = s.seq_len[file];
    const uint64_t need = old + (old ? 1 : 0) + n;
    DevBuf* b = s.seq[file];
    if (need > b->cap) {
        size_t cap = std::max<size_t>(need + 64, b->cap ? b->cap * 2 : 0);
        DevBuf* nb = new DevBuf();
        nb->ensure(cap);
        if (old) HGA_HIP(hipMemcpyAsync(nb->p, b->p, old, hipMemcpyDeviceToDevice, c->stream));
        c->sync();
        delete b;
        s.seq[file] = b = nb;
    }
    char* d = b->as<char>();
    if (old) HGA_HIP(hipMemsetAsync(d + old, '\n', 1, c->stream));
    HGA_HIP(hipMemcpyAsync(d + need - n, seq, n, hipMemcpyHostToDevice, c->stream));
    c->sync();
    s.seq_len[file] = need;
    s.ran = false;
}

void count_run(hga_ctx* c, uint32_t min_per_file) {
    auto& s = c->count;
    HGA_REQUIRE(s.begun, HGA_ERR_STATE, "hga_count_begin not called");
    const uint32_t F = s.n_files;
    s.min_per_file = min_per_file;
    uint64_t total_bytes = 0;
    for (auto l : s.seq_len) total_bytes += l;

    KP kp{};
    kp.k = s.k;
    kp.sh = 2 * (s.k - 1);
    kp.mask = s.k >= 32 ? ~0ull : ((1ull << (2 * s.k)) - 1);
    kp.mix = make_mix(s.k);
    const uint32_t nbits = 2u * (uint32_t)s.k;
    // fan-out: ~16K windows per bucket, at most 4096 buckets, never more bits than the key
    uint32_t fb = 0;
    while (fb < (uint32_t)MAX_FB && fb < nbits && (total_bytes >> fb) > 16384) ++fb;
    kp.fb = fb;
    kp.nb = 1u << fb;
    kp.rbits = nbits - fb;
    kp.rmask = kp.rbits >= 64 ? ~0ull : ((1ull << kp.rbits) - 1);
    const bool e32 = kp.rbits <= 31;
    s.fb = fb;
    s.buckets = kp.nb;

    // super-tiles: ~4 per CU over all files, a multiple of the tile
    uint64_t st_pos = total_bytes / ((uint64_t)c->num_cu * 4) + 1;
    st_pos = std::max<uint64_t>(TILE_POS, (st_pos + TILE_POS - 1) / TILE_POS * TILE_POS);
    std::vector<uint32_t> st_first(F + 1, 0), n_st(F, 0);
    for (uint32_t f = 0; f < F; ++f) {
        n_st[f] = (uint32_t)((s.seq_len[f] + st_pos - 1) / st_pos);
        st_first[f + 1] = st_first[f] + n_st[f];
    }
    const uint32_t n_st_tot = st_first[F];
    const uint32_t nb = kp.nb;

    uint32_t* st_hist = static_cast<uint32_t*>(s.st_hist.ensure((size_t)(n_st_tot + 1) * nb * 4));
    uint64_t* bucket_base = static_cast<uint64_t*>(s.bucket_base.ensure((size_t)(nb + 1) * 8));
    uint64_t* fs = static_cast<uint64_t*>(s.file_start.ensure((size_t)nb * (F + 1) * 8));
    uint32_t* d_st_first = static_cast<uint32_t*>(s.misc.ensure((F + 1) * 4 + 256));
    auto* gstat = static_cast<unsigned long long*>(s.cursor.ensure(8 * 8));
    HGA_HIP(hipMemcpyAsync(d_st_first, st_first.data(), (F + 1) * 4, hipMemcpyHostToDevice, c->stream));
    HGA_HIP(hipMemsetAsync(gstat, 0, 8 * 8, c->stream));
    if (n_st_tot == 0) HGA_HIP(hipMemsetAsync(st_hist, 0, (size_t)nb * 4, c->stream));

    // A: per-super-tile bucket histograms + instance count (gstat[4])
    for (uint32_t f = 0; f < F; ++f) {
        if (!n_st[f]) continue;
        const uint8_t* sp = s.seq[f]->as<uint8_t>();
        const uint64_t n = s.seq_len[f];
        c->launch("kc_hist", [&] {
            hipLaunchKernelGGL(kc_hist, dim3(n_st[f]), dim3(NT_AB), 0, c->stream, sp, n, st_pos,
                               st_first[f], kp, st_hist, gstat + 4);
        });
        c->check_launch("kc_hist");
    }
    // S: offsets
    c->launch("kc_scan", [&] {
        hipLaunchKernelGGL(kc_scan_cols, dim3(blocks_for(nb, 256)), dim3(256), 0, c->stream,
                           st_hist, n_st_tot, nb);
        hipLaunchKernelGGL(kc_bucket_scan, dim3(1), dim3(1024), 0, c->stream,
                           st_hist + (size_t)n_st_tot * nb, nb, bucket_base);
        hipLaunchKernelGGL(kc_file_start, dim3(blocks_for(nb, 256)), dim3(256), 0, c->stream,
                           st_hist, bucket_base, d_st_first, F, nb, fs);
    });
    c->check_launch("kc_scan");

    // B: bin (capacity bound = bytes; instances <= bytes)
    const size_t esz = e32 ? 4 : 8;
    void* binned = s.binned.ensure(std::max<size_t>(total_bytes, 1) * esz);
    for (uint32_t f = 0; f < F; ++f) {
        if (!n_st[f]) continue;
        const uint8_t* sp = s.seq[f]->as<uint8_t>();
        const uint64_t n = s.seq_len[f];
        c->launch("kc_bin", [&] {
            if (e32)
                hipLaunchKernelGGL((kc_bin<uint32_t, P_AB, NT_AB>), dim3(n_st[f]), dim3(NT_AB), 0, c->stream,
                                   sp, n, st_pos, st_first[f], kp, bucket_base, st_hist,
                                   static_cast<uint32_t*>(binned));
            else
                hipLaunchKernelGGL((kc_bin<uint64_t, P_AB, NT_B64>), dim3(n_st[f]), dim3(NT_B64), 0,
                                   c->stream, sp, n, st_pos, st_first[f], kp, bucket_base, st_hist,
                                   static_cast<uint64_t*>(binned));
        });
        c->check_launch("kc_bin");
    }

    // C: per-bucket count
    const uint64_t cap = total_bytes / std::max<uint32_t>(1, min_per_file) + 1;
    s.rows_key.ensure(cap * 8);
    s.rows_cnt.ensure(cap * 4 * F);
    const uint32_t slot_b = (uint32_t)esz + 4u * F;
    uint32_t T = 1;
    while ((uint64_t)T * 2 * slot_b <= LDS_TAB) T *= 2;
    HGA_REQUIRE(T >= 2 * NT_C, HGA_ERR_INVALID, "too many files for the LDS table");
    uint32_t maxload = std::min<uint32_t>((uint32_t)(T * 0.8), T - NT_C - 8);
    c->launch("kc_count", [&] {
        if (e32)
            hipLaunchKernelGGL(kc_count<uint32_t>, dim3(nb), dim3(NT_C), 0, c->stream,
                               static_cast<const uint32_t*>(binned), fs, F, T, maxload, min_per_file,
                               kp, s.rows_key.as<uint64_t>(), s.rows_cnt.as<uint32_t>(), cap, gstat);
        else
            hipLaunchKernelGGL(kc_count<uint64_t>, dim3(nb), dim3(NT_C), 0, c->stream,
                               static_cast<const uint64_t*>(binned), fs, F, T, maxload, min_per_file,
                               kp, s.rows_key.as<uint64_t>(), s.rows_cnt.as<uint32_t>(), cap, gstat);
    });
    c->check_launch("kc_count");
    unsigned long long h_stat[8];
    HGA_HIP(hipMemcpyAsync(h_stat, gstat, sizeof(h_stat), hipMemcpyDeviceToHost, c->stream));
    c->sync();
    HGA_REQUIRE(!(h_stat[2] & 1ull), HGA_ERR_INVALID, "a bucket could not be split to fit the LDS table");
    HGA_REQUIRE(!(h_stat[2] & 2ull), HGA_ERR_OOM, "row capacity exceeded");
    s.rows = h_stat[0];
    s.max_split = (uint32_t)h_stat[1];
    s.instances = h_stat[4];
    s.rows_cap = cap;
    s.ran = true;
    s.n_sel = 0;
}

void count_spec_hist(hga_ctx* c, const double* thr_in, uint32_t n_thr_in, std::vector<int64_t>& out) {
    auto& s = c->count;
    HGA_REQUIRE(s.ran, HGA_ERR_STATE, "hga_count_run not called");
    std::vector<double> thr(thr_in, thr_in + n_thr_in);   // std::set<double> semantics
    std::sort(thr.begin(), thr.end());
    thr.erase(std::unique(thr.begin(), thr.end()), thr.end());
    const uint32_t n_thr = (uint32_t)thr.size();
    HGA_REQUIRE(n_thr >= 1 && n_thr <= MAX_THR, HGA_ERR_INVALID, "1..16 thresholds supported");
    const uint64_t over_cap = 1u << 20;
    const size_t hbytes = (size_t)n_thr * TD * 8;
    char* base = static_cast<char*>(s.hist_dense.ensure(hbytes + over_cap * 8 + 256 + 64));
    auto* hist = reinterpret_cast<unsigned long long*>(base);
    auto* over = reinterpret_cast<unsigned long long*>(base + hbytes);
    auto* ctrl = reinterpret_cast<unsigned long long*>(base + hbytes + over_cap * 8);
    double* dthr = reinterpret_cast<double*>(ctrl + 4);
    HGA_HIP(hipMemsetAsync(base, 0, hbytes, c->stream));
    HGA_HIP(hipMemsetAsync(ctrl, 0, 32, c->stream));
    HGA_HIP(hipMemcpyAsync(dthr, thr.data(), n_thr * 8, hipMemcpyHostToDevice, c->stream));
    const unsigned grid = (unsigned)std::min<uint64_t>(blocks_for(std::max<uint64_t>(s.rows, 1), NT_H),
                                                       (uint64_t)c->num_cu * 2);
    c->launch("kc_spec_hist", [&] {
        hipLaunchKernelGGL(kc_spec_hist, dim3(grid), dim3(NT_H), 0, c->stream,
                           s.rows_cnt.as<uint32_t>(), s.rows, s.rows_cap, s.n_files, dthr, n_thr,
                           hist, over, ctrl, over_cap, ctrl + 1);
    });
    c->check_launch("kc_spec_hist");
    std::vector<unsigned long long> h((size_t)n_thr * TD);
    unsigned long long hc[2];
    HGA_HIP(hipMemcpyAsync(h.data(), hist, hbytes, hipMemcpyDeviceToHost, c->stream));
    HGA_HIP(hipMemcpyAsync(hc, ctrl, 16, hipMemcpyDeviceToHost, c->stream));
    c->sync();
    HGA_REQUIRE(!(hc[1] & 1ull), HGA_ERR_INVALID, "a row's specificity is above the last threshold");
    HGA_REQUIRE(!(hc[1] & 2ull), HGA_ERR_OOM, "histogram overflow list full");
    std::map<std::pair<uint32_t, uint64_t>, uint64_t> sparse;
    if (hc[0]) {
        std::vector<unsigned long long> ov(hc[0]);
        HGA_HIP(hipMemcpy(ov.data(), over, hc[0] * 8, hipMemcpyDeviceToHost));
        for (auto v : ov) sparse[{(uint32_t)(v >> 56), v & ((1ull << 56) - 1)}] += 1;
    }
    out.clear();
    for (uint32_t t = 0; t < n_thr; ++t) {
        for (uint32_t tot = 0; tot < TD; ++tot) {
            const auto v = h[(size_t)t * TD + tot];
            if (v) { out.push_back(t); out.push_back(tot); out.push_back((int64_t)v); }
        }
        for (auto it = sparse.lower_bound({t, 0}); it != sparse.end() && it->first.first == t; ++it) {
            out.push_back(t);
            out.push_back((int64_t)it->first.second);
            out.push_back((int64_t)it->second);
        }
    }
}

void count_select(hga_ctx* c, int64_t lower, int64_t upper, uint64_t* n_out, uint64_t* n_discr) {
    auto& s = c->count;
    HGA_REQUIRE(s.ran, HGA_ERR_STATE, "hga_count_run not called");
    const uint64_t cap = std::max<uint64_t>(s.rows, 1);
    char* sb = static_cast<char*>(s.sel_keys.ensure(cap * 12 + 256));
    uint64_t* out = reinterpret_cast<uint64_t*>(sb);
    uint32_t* flag = reinterpret_cast<uint32_t*>(sb + cap * 8);
    auto* stat = static_cast<unsigned long long*>(s.sel_tmp.ensure(64));
    HGA_HIP(hipMemsetAsync(stat, 0, 16, c->stream));
    if (s.rows) {
        c->launch("kc_select", [&] {
            hipLaunchKernelGGL(kc_select, dim3(blocks_for(s.rows, NT_H)), dim3(NT_H), 0, c->stream,
                               s.rows_key.as<uint64_t>(), s.rows_cnt.as<uint32_t>(), s.rows,
                               s.rows_cap, s.n_files, lower, upper, out, flag, stat);
        });
        c->check_launch("kc_select");
    }
    unsigned long long hs[2];
    HGA_HIP(hipMemcpyAsync(hs, stat, 16, hipMemcpyDeviceToHost, c->stream));
    c->sync();
    radix_sort_u64(c, out, flag, hs[0], 2 * s.k, s.scratch);
    s.n_sel = hs[0];
    *n_out = hs[0];
    *n_discr = hs[1];
}

void count_fetch_selected(hga_ctx* c, uint64_t* dst, uint8_t* flags) {
    auto& s = c->count;
    const uint64_t cap = std::max<uint64_t>(s.rows, 1);
    if (s.n_sel && dst)
        HGA_HIP(hipMemcpyAsync(dst, s.sel_keys.p, s.n_sel * 8, hipMemcpyDeviceToHost, c->stream));
    std::vector<uint32_t> f;
    if (s.n_sel && flags) {
        f.resize(s.n_sel);
        HGA_HIP(hipMemcpyAsync(f.data(), static_cast<char*>(s.sel_keys.p) + cap * 8, s.n_sel * 4,
                               hipMemcpyDeviceToHost, c->stream));
    }
    c->sync();
    if (flags)
        for (uint64_t i = 0; i < s.n_sel; ++i) flags[i] = (uint8_t)f[i];
}

// All merged rows ascending (file < 0), or one file's dump rows (file >= 0).
void count_rows(hga_ctx* c, int file, std::vector<uint64_t>& keys, std::vector<uint32_t>& counts) {
    auto& s = c->count;
    HGA_REQUIRE(s.ran, HGA_ERR_STATE, "hga_count_run not called");
    HGA_REQUIRE(file < (int)s.n_files, HGA_ERR_INVALID, "file index out of range");
    const uint64_t rows = s.rows;
    const uint32_t F = s.n_files;
    keys.clear();
    counts.clear();
    if (!rows) return;
    DevBuf tk, tv, tc;
    uint64_t* k = static_cast<uint64_t*>(tk.ensure(rows * 8));
    uint32_t* v = static_cast<uint32_t*>(tv.ensure(rows * 4));
    uint32_t* cc = static_cast<uint32_t*>(tc.ensure(rows * 4 * F));
    HGA_HIP(hipMemcpyAsync(k, s.rows_key.p, rows * 8, hipMemcpyDeviceToDevice, c->stream));
    hipLaunchKernelGGL(kc_iota, dim3(blocks_for(rows, 256)), dim3(256), 0, c->stream, v, rows);
    c->check_launch("kc_iota");
    radix_sort_u64(c, k, v, rows, 2 * s.k, s.scratch);
    hipLaunchKernelGGL(kc_gather_rows, dim3(blocks_for(rows, 256)), dim3(256), 0, c->stream, v,
                       s.rows_cnt.as<uint32_t>(), rows, s.rows_cap, F, cc);
    c->check_launch("kc_gather_rows");
    std::vector<uint64_t> hk(rows);
    std::vector<uint32_t> hc(rows * F);
    HGA_HIP(hipMemcpyAsync(hk.data(), k, rows * 8, hipMemcpyDeviceToHost, c->stream));
    HGA_HIP(hipMemcpyAsync(hc.data(), cc, rows * 4 * F, hipMemcpyDeviceToHost, c->stream));
    c->sync();
    if (file < 0) {
        keys.swap(hk);
        counts.swap(hc);
        return;
    }
    for (uint64_t i = 0; i < rows; ++i) {
        const uint32_t cnt = hc[i * F + (uint32_t)file];
        if (cnt) {
            keys.push_back(hk[i]);
            counts.push_back(cnt);
        }
    }
}

}  // namespace hga
