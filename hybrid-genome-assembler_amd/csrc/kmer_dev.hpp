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

// Bijective mix on n = 2k bits (arithmetic mod 2^n): multiply by an odd constant (the
// top bits then depend on every key bit), then xor the top half into the bottom half
// (s = ceil(n/2), so the xor-shift is its own inverse).  Buckets take the top bits of
// the mixed value, LDS table slots the low bits.
struct Mix {
    uint64_t mask, c1, c2, c1i, c2i;
    uint32_t n, s;
};

__host__ __device__ inline uint64_t mix_fwd(uint64_t x, const Mix& m) {
    x = (x * m.c1) & m.mask;
    return x ^ (x >> m.s);
}
__host__ __device__ inline uint64_t mix_inv(uint64_t h, const Mix& m) {
    h ^= h >> m.s;
    return (h * m.c1i) & m.mask;
}

inline uint64_t inv_odd_u64(uint64_t a) {  // a * x == 1 mod 2^64 (Newton)
    uint64_t x = a;
    for (int i = 0; i < 6; ++i) x *= 2 - a * x;
    return x;
}
// The multiplier's high word is a multiple of 64: for 2k <= 38 bits (k <= 19) the product mod 4^k
// then needs one 32x32->64 multiply-add and one low multiply instead of three quarter-rate
// multiplies (x_lo * c_hi vanishes mod 2^38).  Any odd constant gives a bijection.
constexpr uint64_t kMixC1 = 0x9E3779C07F4A7C15ull;
// mix_fwd for a compile-time 16 < K <= 19 with kMixC1 (what make_mix(K) gives): x * c1 mod 2^(2K) as the
// low words' 32x32->64 product plus the high word's contribution, of which only the low 2K - 32 bits
// count — a small multiply by c1 mod 64 (c1's high word, a multiple of 64, contributes nothing below
// 2^38) — one 64-bit multiply-add instead of two.  Equal to mix_fwd.
#ifndef HGA_MIX_K
#define HGA_MIX_K 1
#endif
template <int K>
__device__ __forceinline__ uint64_t mix_fwd_k(uint64_t x, const Mix& m) {
    if constexpr (HGA_MIX_K && K > 16 && K <= 19) {
        static_assert((kMixC1 >> 32) % 64 == 0, "c1's high word must vanish below 2^38");
        constexpr uint32_t CL = (uint32_t)kMixC1;
        const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
        // one v_mad_u64_u32 with the small product as the high word of its addend (written out: the
        // compiler otherwise re-derives the 64-bit product and issues two)
        const uint64_t add = (uint64_t)(xh * (CL & 63u)) << 32;
        uint64_t p;
        uint64_t carry;
        asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(p), "=s"(carry) : "v"(xl), "s"(CL), "v"(add));
        (void)carry;
        const uint64_t y = p & ((1ull << (2 * K)) - 1);
        return y ^ (y >> ((2 * K + 1) / 2));
    } else {
        return mix_fwd(x, m);
    }
}

inline Mix make_mix(int k) {
    Mix m;
    m.n = 2u * (uint32_t)k;
    m.mask = m.n >= 64 ? ~0ull : ((1ull << m.n) - 1);
    m.s = (m.n + 1) / 2;
    m.c1 = kMixC1;
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

// Load through the global address space.  A pointer the compiler cannot prove global (one read
// from a struct in memory) is accessed with flat instructions, which count against lgkmcnt as
// well as vmcnt: every `s_waitcnt lgkmcnt(0)` of an LDS phase would then also drain such a
// load, so a prefetch would not stay in flight across LDS barriers.
// (A native vector type: HIP's uint4 is a struct whose copy goes through a generic pointer.)
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
#ifndef HGA_GLOBAL_LOADS
#define HGA_GLOBAL_LOADS 1   // 0: generic-pointer loads (timing comparison only)
#endif
__device__ __forceinline__ uint4 load_global16(const void* p) {
    if (!HGA_GLOBAL_LOADS) return *reinterpret_cast<const uint4*>(p);
    const u32x4_t v = *(const __attribute__((address_space(1))) u32x4_t*)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

// 16 bytes starting at byte index `base` (a multiple of 16) of a stream of length n;
// bytes outside [0, n) read as 0 (not a base in either semantics).
__device__ __forceinline__ uint4 load16(const uint8_t* s, int64_t base, uint64_t n) {
    if (base >= 0 && (uint64_t)base + 16 <= n) return load_global16(s + base);
    uint32_t w[4] = {0, 0, 0, 0};
    for (int j = 0; j < 16; ++j) {
        int64_t i = base + j;
        if (i >= 0 && (uint64_t)i < n)
            w[j >> 2] |= (uint32_t)*(const __attribute__((address_space(1))) uint8_t*)(s + i) << (8 * (j & 3));
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// ---------------------------------------------------------------- packed frames (K1/K2)
// The sequence stream is packed once (lk_pack; kc_bin1 per tile into LDS): per 16 bases one u32 of 2-bit
// codes (first base in the top bits) and one u16 of base-valid bits (bit b = base b).
// Two leading pad words (all invalid) let every frame read two words before its start.
constexpr int PAD_WORDS = 2;

// Reverse the order of the 16 2-bit groups of a word.
__device__ __forceinline__ uint32_t rev2(uint32_t x) {
    const uint32_t y = __builtin_bitreverse32(x);
    return ((y >> 1) & 0x55555555u) | ((y & 0x55555555u) << 1);
}

// Base-valid bits of one word expanded to the 2-bit code positions (base b -> bits 31-2b, 30-2b).
__device__ __forceinline__ uint32_t expand2(uint32_t v16) {
    uint32_t x = __builtin_bitreverse32(v16) >> 16;   // base b -> bit 15-b
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x | (x << 1);
}

// Bit e of the result is set iff bits [e-len+1, e] of v are all set (len in [1, 64]).
__device__ __forceinline__ uint64_t runs_of(uint64_t v, int len) {
    uint64_t p[7];
    p[0] = v;
#pragma unroll
    for (int b = 1; b < 7; ++b) p[b] = p[b - 1] & (p[b - 1] << (1 << (b - 1)));
    uint64_t w = ~0ull;
    int off = 0;
#pragma unroll
    for (int b = 6; b >= 0; --b)
        if (len & (1 << b)) {
            w &= p[b] << off;
            off += 1 << b;
        }
    return w;
}

// 64-bit field of an NW-word big-endian bit string starting at bit `sh` from the bottom
// (sh a compile-time constant after unrolling -> two alignbit instructions).
template <int NW>
__device__ __forceinline__ uint64_t field64(const uint32_t (&x)[NW], int sh) {
    const int wb = sh >> 5, b = sh & 31;
    const int i0 = NW - 1 - wb, i1 = NW - 2 - wb, i2 = NW - 3 - wb;
    const uint32_t a0 = i0 >= 0 ? x[i0] : 0u, a1 = i1 >= 0 ? x[i1] : 0u, a2 = i2 >= 0 ? x[i2] : 0u;
    const uint32_t lo = __builtin_amdgcn_alignbit(a1, a0, b);
    const uint32_t hi = __builtin_amdgcn_alignbit(a2, a1, b);
    return ((uint64_t)hi << 32) | lo;
}

// Per-thread frame of P window ends [p0, p0+P): bases [p0-32, p0+P) as NW words of the
// forward codes, the matching reverse-complement string pre-shifted so that the rc code of
// the window ending at p0+j is field64(r, 2j), and the valid-window bits.
template <int P>
struct Frame {
    static constexpr int NW = 2 + P / 16;
    uint32_t x[NW];
    uint32_t r[NW];
};

// The raw words of a frame (what load_frame reads, or what a kernel packs from ASCII itself).
template <int P>
struct FrameRaw {
    static constexpr int NW = Frame<P>::NW;
    uint32_t x[NW];
    uint32_t v[NW];
};

// REF = KmerIterator semantics (non-bases contribute 0 to both strands); otherwise the
// counting semantics (a window with a non-base is never used, so rc = revcomp(fwd)).
// Returns the frame's valid bits.
template <int P, bool REF>
__device__ __forceinline__ uint64_t build_frame(const FrameRaw<P>& raw, int k, Frame<P>& f) {
    constexpr int NW = Frame<P>::NW;
    uint64_t v64 = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        f.x[i] = raw.x[i];
        v64 |= (uint64_t)raw.v[i] << (16 * i);
    }
    uint32_t R[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        uint32_t c = ~f.x[NW - 1 - i];
        if (REF) c &= expand2(raw.v[NW - 1 - i]);
        R[i] = rev2(c);
    }
    // f.r = R >> (66 - 2k)   (v in [2, 64]; a and b are uniform across the wave)
    const int v = 66 - 2 * k;
    const int a = v >> 5, b = v & 31;
#pragma unroll
    for (int i = 0; i < NW; ++i) {        // i counts words from the bottom
        const uint32_t c0 = i < NW ? R[NW - 1 - i] : 0u;
        const uint32_t c1 = i + 1 < NW ? R[NW - 2 - i] : 0u;
        const uint32_t c2 = i + 2 < NW ? R[NW - 3 - i] : 0u;
        const uint32_t c3 = i + 3 < NW ? R[NW - 4 - i] : 0u;
        const uint32_t lo = a == 0 ? c0 : (a == 1 ? c1 : c2);
        const uint32_t hi = a == 0 ? c1 : (a == 1 ? c2 : c3);
        f.r[NW - 1 - i] = __builtin_amdgcn_alignbit(hi, lo, b);
    }
    return v64;
}

// w0 = index (with padding) of the frame's first word in the packed stream.
template <int P, bool REF>
__device__ __forceinline__ uint64_t load_frame(const uint32_t* __restrict__ pk,
                                               const uint16_t* __restrict__ vd, uint64_t w0, int k,
                                               Frame<P>& f) {
    FrameRaw<P> r;
#pragma unroll
    for (int i = 0; i < FrameRaw<P>::NW; ++i) {
        r.x[i] = pk[w0 + i];
        r.v[i] = vd[w0 + i];
    }
    return build_frame<P, REF>(r, k, f);
}

// ASCII -> packed frames (lk_pack, kc_bin1).  REF = KmerIterator semantics (upper-case
// ACGT only), otherwise jellyfish semantics (either case).
// One thread per 16 bases: packed codes (first base in bits 31:30) and valid bits.
// 16 bases starting at 16w -> 2-bit codes (MSB-first) + valid bits.
template <bool REF>
__device__ __forceinline__ void pack_bytes(const uint4 v, uint32_t& code, uint32_t& valid) {
    // four bytes per 32-bit word at a time (SWAR): a byte is a base iff it equals one of 'A' 'C'
    // 'G' 'T' (after the case fold of the counting semantics) — exact per-byte zero tests of the
    // xor with each; codes ((u >> 1) ^ (u >> 2)) & 3, forced to 0 for non-bases
    const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
    code = 0;
    valid = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t u = REF ? ws[i] : (ws[i] & 0xDFDFDFDFu);
        uint32_t c4 = ((u >> 1) ^ (u >> 2)) & 0x03030303u;
        // the base letter each byte's code stands for ('A' 'C' 'G' 'T' as bytes 0..3 of the table,
        // one v_perm_b32 picks them by code): a byte is a base iff it equals its own letter, since
        // every other byte value differs from all four
        const uint32_t want = __builtin_amdgcn_perm(0u, 0x54474341u, c4);
        const uint32_t d = u ^ want;
        const uint32_t f = ~(((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;   // bit 7: byte is a base
        const uint32_t m = f >> 7;                        // bits 0, 8, 16, 24
        if (REF) c4 &= m * 3u;   // KmerIterator: a non-base contributes code 0 (counting ignores it)
        const uint32_t r = __builtin_bswap32(c4);         // first base in the top byte
        const uint32_t t = (r | (r >> 6)) & 0x000F000Fu;
        code |= ((t | (t >> 12)) & 0xFFu) << (24 - 8 * i);
        valid |= ((m * 0x01020408u) >> 24) << (4 * i);    // byte b -> bit b
    }
}

template <bool REF>
__device__ __forceinline__ void pack_word(const uint8_t* __restrict__ s, uint64_t n, uint64_t w, uint32_t& code,
                                          uint32_t& valid) {
    pack_bytes<REF>(load16(s, (int64_t)(w * 16), n), code, valid);
}

template <bool REF>
__global__ void pack_kernel(const uint8_t* __restrict__ s, uint64_t n, uint32_t* __restrict__ pk,
                            uint16_t* __restrict__ vd, uint64_t nw) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nw) return;
    uint32_t code, valid;
    pack_word<REF>(s, n, w, code, valid);
    pk[PAD_WORDS + w] = code;
    vd[PAD_WORDS + w] = (uint16_t)valid;
}

// Hand-off of LDS data between lanes of ONE wave: a wave's LDS instructions execute in order,
// so only the compiler must be kept from reordering or caching across this point.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// Inclusive wave64 scans through DPP row shifts and row broadcasts: VALU only, no LDS-pipe
// traffic (a shuffle scan issues one ds_bpermute per step).  Lanes whose DPP source is outside
// the row, and the rows a broadcast step leaves out, read the identity 0, so the operation must
// have 0 as its identity (unsigned add / max).  All 64 lanes must be active.
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_take(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_scan_add_dpp(uint32_t x) {
    x += dpp_take<0x111, 0xf>(x);   // row_shr:1
    x += dpp_take<0x112, 0xf>(x);   // row_shr:2
    x += dpp_take<0x114, 0xf>(x);   // row_shr:4
    x += dpp_take<0x118, 0xf>(x);   // row_shr:8
    x += dpp_take<0x142, 0xa>(x);   // row_bcast:15 into rows 1, 3
    x += dpp_take<0x143, 0xc>(x);   // row_bcast:31 into rows 2, 3
    return x;
}
__device__ __forceinline__ uint32_t wave_scan_max_dpp(uint32_t x) {
    x = max(x, dpp_take<0x111, 0xf>(x));
    x = max(x, dpp_take<0x112, 0xf>(x));
    x = max(x, dpp_take<0x114, 0xf>(x));
    x = max(x, dpp_take<0x118, 0xf>(x));
    x = max(x, dpp_take<0x142, 0xa>(x));
    x = max(x, dpp_take<0x143, 0xc>(x));
    return x;
}
// Value of lane L (uniform result, no LDS).
__device__ __forceinline__ uint32_t wave_lane(uint32_t x, int L) { return (uint32_t)__builtin_amdgcn_readlane((int)x, L); }

// Value of lane ^ X, on the VALU: DPP quad permutes (X = 1, 2), row shifts (4), a row rotate (8),
// the gfx950 permlane swaps (16, 32).  A swap of a register with itself leaves one of its two
// results equal to the lane's own value and the other the partner's, whichever half the
// instruction moves, so the partner is the result that differs (equal values: either).
template <int X>
__device__ __forceinline__ uint32_t lane_xor32(uint32_t v) {
    if constexpr (X == 1) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, true);   // quad_perm [1,0,3,2]
    } else if constexpr (X == 2) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, true);   // quad_perm [2,3,0,1]
    } else if constexpr (X == 4) {
        const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x104, 0xf, 0xf, true);   // row_shl:4
        const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);   // row_shr:4
        return (__lane_id() & 4) ? dn : up;
    } else if constexpr (X == 8) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, true);   // row_ror:8
    } else if constexpr (X == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return r[0] == v ? r[1] : r[0];
    } else {
        static_assert(X == 32, "lane_xor32: X in {1, 2, 4, 8, 16, 32}");
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return r[0] == v ? r[1] : r[0];
    }
}
template <int X>
__device__ __forceinline__ uint64_t lane_xor(uint64_t v) {
    return ((uint64_t)lane_xor32<X>((uint32_t)(v >> 32)) << 32) | lane_xor32<X>((uint32_t)v);
}
template <int X>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) { return lane_xor32<X>(v); }

// Ascending bitonic sort of 64 x R keys held blocked by one wave (key index lane * R + u).
template <int R, int K, int J, class T>
__device__ __forceinline__ void bitonic_step(T (&v)[R], uint32_t lane) {
    if constexpr (J < R) {   // partners in the same lane
#pragma unroll
        for (int u = 0; u < R; ++u) {
            if ((u & J) == 0) {
                const bool asc = ((lane * R + u) & K) == 0;
                const T a = v[u], b = v[u ^ J];
                const bool sw = asc ? (a > b) : (a < b);
                v[u] = sw ? b : a;
                v[u ^ J] = sw ? a : b;
            }
        }
    } else {   // partner lane ^ (J / R), same register
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const T o = lane_xor<J / R>(v[u]);
            const uint32_t i = lane * R + u;
            const bool keep_min = ((i & J) == 0) == ((i & K) == 0);
            v[u] = keep_min ? min(v[u], o) : max(v[u], o);
        }
    }
    if constexpr (J > 1) bitonic_step<R, K, J / 2>(v, lane);
}
template <int R, int K, class T>
__device__ __forceinline__ void bitonic_stage(T (&v)[R], uint32_t lane) {
    bitonic_step<R, K, K / 2>(v, lane);
    if constexpr (K < 64 * R) bitonic_stage<R, K * 2>(v, lane);
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

// Wave-wide exclusive scan of small values (v < 2^B) through ballots of the bit planes:
// no LDS-pipe traffic (a shuffle scan issues ds_bpermute).  *total = the wave sum.
template <int B>
__device__ __forceinline__ uint32_t wave_excl_scan_small(uint32_t v, uint32_t* total) {
    uint32_t ex = 0, tot = 0;
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const uint64_t m = __ballot((v >> b) & 1u);
        ex += (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << b;
        tot += (uint32_t)__popcll(m) << b;
    }
    *total = tot;
    return ex;
}

// Wave-aggregated counter add for keys with few distinct values (o < n_own <= 64, nbits =
// ceil(log2 n_own) <= 6): the key's bit planes are balloted once, lane j builds key j's lane mask
// and makes that key's one LDS add, every live lane gets its position (in lane order) from its
// key's mask.  Per-lane adds on so few counters would serialise on the same LDS addresses.
template <class C>
__device__ __forceinline__ C wave_key_add(C* ctr, uint32_t o, bool live, uint32_t n_own, int nbits) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t L = __ballot(live);
    uint64_t m = L, mo = L;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
        if (b >= nbits) break;
        const uint64_t B = __ballot(live && ((o >> b) & 1u));
        m &= ((o >> b) & 1u) ? B : ~B;
        mo &= ((lane >> b) & 1u) ? B : ~B;
    }
    C base = 0;
    if (lane < n_own && mo) base = atomicAdd(&ctr[lane], (C)__popcll(mo));
    base = __shfl(base, (int)(o & 63u), 64);
    return base + (C)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Chained scan with decoupled look-back over "tiles" that take their ids in start order (a
// counter that only grows): 64-bit status words [flag 2 | epoch 22 | value 40] published with
// agent-scope relaxed stores; words of other scans carry another epoch and count as unpublished,
// so the status array is never cleared between scans.  A tile only waits on tiles with smaller
// ids, which have started.  Called by one thread: publishes `agg`, returns the tile's exclusive
// prefix (values < 2^40).
constexpr uint64_t SCS_A = 1ull << 62, SCS_P = 2ull << 62, SCS_F = 3ull << 62;
constexpr uint64_t SCS_V = (1ull << 40) - 1;
constexpr uint32_t SCS_EPOCHS = 1u << 22;
__device__ __forceinline__ uint64_t chained_lookback(unsigned long long* __restrict__ status, uint64_t tile,
                                                     uint64_t agg, uint32_t epoch) {
    const uint64_t tag = (uint64_t)epoch << 40;
    unsigned long long* st = status + tile;
    uint64_t excl = 0;
    if (tile == 0) {
        __hip_atomic_store(st, SCS_P | tag | (agg & SCS_V), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    __hip_atomic_store(st, SCS_A | tag | (agg & SCS_V), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int64_t t = (int64_t)tile - 1;
    while (true) {
        const uint64_t w = __hip_atomic_load(status + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t f = (((w >> 40) & (SCS_EPOCHS - 1)) == epoch) ? (w & SCS_F) : 0ull;
        if (f == SCS_P) {
            excl += w & SCS_V;
            break;
        }
        if (f == SCS_A) {
            excl += w & SCS_V;
            --t;
        }   // else: tile t has not published yet, read it again
    }
    // the value field is 40 bits: a prefix of 2^40 or more wraps in the published word (its flag and
    // epoch stay intact, so successors never spin on it); callers scan counts far below 2^40
    __hip_atomic_store(st, SCS_P | tag | ((excl + agg) & SCS_V), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
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

// ---- LDS segment sort (the export sort: sort.hip ss_segsort, count.hip kc_bx_lsort) ----
constexpr int SS_T = 1024, SS_I = 16, SS_CAP = SS_T * SS_I;

// One segment of cnt <= NT * I keys (loaded by the caller into key[], items in (wave, j, lane) order)
// sorted in LDS by bits [lo, lo + nbits) of the key by NT threads: stable LSD passes over DB-bit digits
// (DB <= 9, 2^DB <= NT), ballot-matched ranks inside each wave, waves in order.  T = uint64_t or
// uint32_t (u32 keys: the same LDS holds twice as many); wcnt holds [NT / 64][2^DB] counters.
template <class T, int I, int NT = SS_T, int DB = 8>
__device__ __forceinline__ void lds_lsd_sort_t(T (&key)[I], uint32_t cnt, int lo, int nbits, T* sk,
                                               uint32_t (*wcnt)[1 << DB], uint32_t* ws) {
    static_assert(DB <= 9 && (1 << DB) <= NT, "digit counters: one per thread in the scan");
    constexpr uint32_t ND = 1u << DB, NONE = ND;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int sh = lo; sh < lo + nbits; sh += DB) {
        const uint32_t dm = lo + nbits - sh >= DB ? ND - 1 : ((1u << (lo + nbits - sh)) - 1u);
        for (int i = tid; i < (NT / 64) * (int)ND; i += NT) (&wcnt[0][0])[i] = 0;
        __syncthreads();
        uint32_t dr[I];   // rank << 10 | digit (ND: no item) — one register per item
#pragma unroll
        for (int j = 0; j < I; ++j) {   // stable rank inside the wave, items in (j, lane) order
            const uint32_t i0 = (uint32_t)wave * (I * 64) + (uint32_t)j * 64;   // wave-uniform
            const uint32_t i = i0 + lane;
            const bool ok = i < cnt;
            const uint32_t d = ok ? ((uint32_t)(key[j] >> sh) & dm) : NONE;
            dr[j] = d;
            if (i0 >= cnt) continue;   // no item of this row: skip its ballots
            uint64_t m = __ballot(ok);
#pragma unroll
            for (int b = 0; b < DB; ++b) {
                const bool bit = (d >> b) & 1u;
                const uint64_t bb = __ballot(bit);
                m &= bit ? bb : ~bb;
            }
            uint32_t before = 0;
            if (ok) before = wcnt[wave][d];
            dr[j] = d | (before + (uint32_t)__popcll(m & lt)) << 10;
            if (ok && (m & lt) == 0ull) wcnt[wave][d] = before + (uint32_t)__popcll(m);
            wave_lds_sync();
        }
        __syncthreads();
        {   // digit starts, then each wave's start inside its digit (waves in order: stable)
            const uint32_t d = (uint32_t)tid & (ND - 1);
            uint32_t tot_d = 0;
            if (tid < (int)ND)
                for (int w = 0; w < NT / 64; ++w) tot_d += wcnt[w][d];
            uint32_t tt;
            const uint32_t exd = block_excl_scan<NT>(tid < (int)ND ? tot_d : 0u, ws, &tt);
            if (tid < (int)ND) {
                uint32_t o = exd;
                for (int w = 0; w < NT / 64; ++w) {
                    const uint32_t c = wcnt[w][d];
                    wcnt[w][d] = o;
                    o += c;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < I; ++j)
            if ((dr[j] & 1023u) < ND) sk[wcnt[wave][dr[j] & 1023u] + (dr[j] >> 10)] = key[j];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < I; ++j) {
            const uint32_t i = (uint32_t)wave * (I * 64) + (uint32_t)j * 64 + lane;
            if (i < cnt) key[j] = sk[i];
        }
        __syncthreads();
    }
}
// The u64 form over the low bits_low bits (sort.hip ss_segsort).
__device__ __forceinline__ void lds_lsd_sort(uint64_t (&key)[SS_I], uint32_t cnt, int bits_low, uint64_t* sk,
                                             uint32_t (*wcnt)[256], uint32_t* ws) {
    lds_lsd_sort_t<uint64_t, SS_I>(key, cnt, 0, bits_low, sk, wcnt, ws);
}

}  // namespace hga
