// Device-side k-mer primitives shared by the counting and lookup kernels (gfx950).
//
// Encoding follows src/common/KmerIterator.cpp: 2 bits per base, A0 C1 G2 T3, the
// first base of a window in the highest bits; canonical = min(forward, reverse
// complement).  Two base-mapping semantics exist on the hot path:
//  * counting (jellyfish, run_jellyfish.sh:3-6): A/C/G/T in either case are bases,
//    any other byte breaks the window run;
//  * lookup (KmerIterator, KmerIterator.cpp:7-19,54-63): only upper-case A/C/G/T map
//    to their codes; every other byte contributes code 0 to BOTH strands (the
//    unordered_map operator[] default), so rc != revcomp(fwd) at such positions.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace hga {

// Bijective mix on n = 2k bits (all arithmetic mod 2^n).  The xor-shift uses
// s = ceil(n/2) so it is its own inverse; the multipliers are odd so they invert
// mod 2^n.  Buckets take the top bits of the mixed value, LDS slots the low bits.
struct Mix {
    uint64_t mask, c1, c2, c1i, c2i;
    uint32_t n, s;
};

__host__ __device__ inline uint64_t mix_fwd(uint64_t x, const Mix& m) {
    x = (x * m.c1) & m.mask;
    x ^= x >> m.s;
    x = (x * m.c2) & m.mask;
    x ^= x >> m.s;
    return x;
}
__host__ __device__ inline uint64_t mix_inv(uint64_t h, const Mix& m) {
    h ^= h >> m.s;
    h = (h * m.c2i) & m.mask;
    h ^= h >> m.s;
    h = (h * m.c1i) & m.mask;
    return h;
}

inline uint64_t inv_odd_u64(uint64_t a) {  // a * x == 1 mod 2^64 (Newton)
    uint64_t x = a;
    for (int i = 0; i < 6; ++i) x *= 2 - a * x;
    return x;
}
inline Mix make_mix(int k) {
    Mix m;
    m.n = 2u * (uint32_t)k;
    m.mask = m.n >= 64 ? ~0ull : ((1ull << m.n) - 1);
    m.s = (m.n + 1) / 2;
    m.c1 = 0x9E3779B97F4A7C15ull;
    m.c2 = 0xC2B2AE3D27D4EB4Full;
    m.c1i = inv_odd_u64(m.c1);
    m.c2i = inv_odd_u64(m.c2);
    return m;
}

// 0x41 'A' -> 0, 'C' -> 2, 'G' -> 6, 'T' -> 19 : bit mask of the valid offsets.
constexpr uint32_t kBaseBits = (1u << 0) | (1u << 2) | (1u << 6) | (1u << 19);

// Counting semantics: case-insensitive ACGT.  Returns code in [0,3]; *ok = base?
__device__ __forceinline__ uint32_t jf_code(uint32_t b, bool& ok) {
    const uint32_t u = b & 0xDFu;
    const uint32_t d = u - 0x41u;
    ok = d < 20u && ((kBaseBits >> d) & 1u);
    return ((u >> 1) ^ (u >> 2)) & 3u;
}

// Lookup semantics (KmerIterator): forward and reverse-complement contributions.
__device__ __forceinline__ void ref_codes(uint32_t b, uint32_t& fc, uint32_t& rcc) {
    const uint32_t d = b - 0x41u;
    const bool ok = d < 20u && ((kBaseBits >> d) & 1u);
    const uint32_t c = ((b >> 1) ^ (b >> 2)) & 3u;
    fc = ok ? c : 0u;
    rcc = ok ? 3u - c : 0u;
}

// 16 bytes starting at byte index `base` (a multiple of 16) of a stream of length n;
// bytes outside [0, n) read as 0 (not a base in either semantics).
__device__ __forceinline__ uint4 load16(const uint8_t* s, int64_t base, uint64_t n) {
    if (base >= 0 && (uint64_t)base + 16 <= n) return *reinterpret_cast<const uint4*>(s + base);
    uint32_t w[4] = {0, 0, 0, 0};
    for (int j = 0; j < 16; ++j) {
        int64_t i = base + j;
        if (i >= 0 && (uint64_t)i < n) w[j >> 2] |= (uint32_t)s[i] << (8 * (j & 3));
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Counting-semantics scan of the P window-ends [p0, p0+P) (p0 % 16 == 0, P % 16 == 0).
// Rolls the 32 preceding bytes as halo (k <= 32), then calls f(canonical, j) for
// every j in [0,P) whose window [p0+j-k+1, p0+j] consists of bases only.  Fully
// unrolled so per-position state stays in registers.
template <int P, class F>
__device__ __forceinline__ void scan_count_windows(const uint8_t* s, uint64_t n, uint64_t p0,
                                                   int k, uint64_t mask, int sh, F&& f) {
    static_assert(P % 16 == 0 && P > 0, "P must be a positive multiple of 16");
    uint64_t fwd = 0, rc = 0;
    int run = 0;
#pragma unroll
    for (int c = -2; c < P / 16; ++c) {
        const uint4 v = load16(s, (int64_t)p0 + 16 * c, n);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            bool ok;
            const uint32_t code = jf_code((w[j >> 2] >> (8 * (j & 3))) & 0xFFu, ok);
            fwd = ((fwd << 2) | code) & mask;
            rc = (rc >> 2) | ((uint64_t)(3u - code) << sh);
            run = ok ? run + 1 : 0;
            if (c >= 0 && run >= k) f(fwd < rc ? fwd : rc, 16 * c + j);
        }
    }
}

// Wave / block scans (wave64).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// Block-wide exclusive scan of one value per thread; NT threads (multiple of 64,
// <= 1024).  `ws` is LDS scratch of >= NT/64 + 1 words.  Returns the exclusive
// prefix; *total receives the block sum.  Contains __syncthreads().
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* ws, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int NW = NT / 64;
    uint32_t inc = wave_incl_scan(v, lane);
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    if (wave == 0) {
        uint32_t t = lane < NW ? ws[lane] : 0u;
        uint32_t ti = wave_incl_scan(t, lane);
        if (lane < NW) ws[lane] = ti - t;
        if (lane == NW - 1) ws[NW] = ti;
    }
    __syncthreads();
    uint32_t r = ws[wave] + inc - v;
    *total = ws[NW];
    __syncthreads();
    return r;
}

}  // namespace hga
