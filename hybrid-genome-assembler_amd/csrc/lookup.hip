// lookup.hip — MI355X replacement for the per-read SDK lookup loop of
// ReadClusteringEngine::construct_indices (src/clustering/ReadClusteringEngine.cpp:234-299).
//
//   lk_pack       the read-start bitmap and word -> read map (the 2-bit codes with KmerIterator
//                 semantics — non-ACGT contributes 0 to both strands, KmerIterator.cpp:7-19,54-63 — are
//                 packed by lk_scan from the ASCII reads; pack_kernel<REF> only for hll_scan).
//   lk_starts     read-start bitmap (1 bit per base): a window is in one read iff no read
//                 starts inside (start, end].
//   lk_build      read-only table {canonical code -> KmerID}, 5 keys + 5 ids per 64-B bucket,
//                 and a minimizer-blocked Bloom filter (16-B block per minimizer, one bit per
//                 key in each of its 4 words; a power of two of >= 11 bits per key: 4 MiB at C3, mostly L2/MALL-resident).
//                 KmerIDs come from the host (std::unordered_set order,
//                 ReadClusteringEngine.cpp:237-241).
//   lk_scan<0>    32 window ends per thread from packed frames: closed-form canonical codes,
//                 minimizers, one filter block per minimizer run; passing windows are queued
//                 per wave and probed with all lanes busy; KmerIDs kept per window slot.
//   lk_scan<1>    threads with hits copy their KmerIDs to (read, KmerID, end-exclusive
//                 position) at block-scanned offsets: read / window order.
//   post          CSR pointers, per-read LDS sorts for the sorted KmerID lists (:272) and
//                 first positions (:267), stable radix sort for kmer_component_index (:282-284).
#include <algorithm>

#include "hga_internal.hpp"
#include "kmer_dev.hpp"

namespace hga {
namespace {

#ifndef HGA_FBITS2
#define HGA_FBITS2 22
#endif
#ifndef HGA_LK_SLOTS10
// table slots per 10 keys: 40 = <= 25 % slot load (a probe rarely passes its home line; C3 lk_scan<0>
// 1.80 ms at 50 % load, 1.72 at 33 %, 1.70 at 25 %, 1.72 at 17 %; 2.23 at 71 %)
#define HGA_LK_SLOTS10 40
#endif
#ifndef HGA_LK_T
#define HGA_LK_T 256
#endif
#ifndef HGA_LK_MINW
#define HGA_LK_MINW 6   // lk_scan's count pass (compile-time k): 6 waves per SIMD, i.e. <= 80 VGPRs
#endif
#ifndef HGA_LK_ASCII
// lk_scan packs its frames from the ASCII reads itself (four 16-B loads + the SWAR packer per thread),
// so lookup_run has no codes pass: C3 lk_pack 0.23 -> 0.03 ms (the read-start bits and word -> read map
// stay), lk_count 1.59 -> 1.72 ms, lookup 2.98 -> 2.92 ms (round 6); hll_scan packs for itself
#define HGA_LK_ASCII 1
#endif
constexpr int LK_T = HGA_LK_T;   // lookup scan workgroup
constexpr int LK_P = 32;                  // window ends per thread (frame of 4 words)
static_assert(LK_P % 32 == 0, "a thread's windows start on a 32-base word (word_read, lk_scan's emit)");
constexpr int LK_QN = 256;                // filter-pass queue entries per wave
constexpr int LK_ST = 2048;               // emit pass: hits per tile staged in LDS (more: direct stores)
constexpr uint64_t EMPTY_KEY = ~0ull;     // never canonical: min(fwd, rc) of all-T is 0
constexpr int SB_PAD = 1;                 // leading zero words of the read-start bitmap

// Table: buckets of one 64-B line = 5 keys + their 5 KmerIDs, so a probe is one line read
// (no dependent id load).  Bucket = multiply-shift of 32 hash bits (any bucket count).
constexpr int BKT = 5;
struct alignas(64) Bucket {
    uint64_t key[BKT];
    uint32_t id[BKT];
    uint32_t pad;
};
static_assert(sizeof(Bucket) == 64, "one line per bucket");

// One 64-bit multiply + xorshift: filter bits from bits 40..58, table bucket from bits 24..55.
__device__ __forceinline__ uint64_t tab_hash(uint64_t x) {
    const uint64_t m = x * 0x9E3779B97F4A7C15ull;
    return m ^ (m >> 31);
}
__device__ __forceinline__ uint64_t bucket_of(uint64_t h, uint64_t nbk) {
    return (((h >> 24) & 0xFFFFFFFFull) * nbk) >> 32;
}
// Blocked Bloom filter bits: three bits of one 32-bit word.
__device__ __forceinline__ uint32_t bloom_bits(uint64_t h) {
    const uint32_t x = (uint32_t)(h >> 40);
    return (1u << (x & 31)) | (1u << ((x >> 5) & 31)) | (1u << ((x >> 10) & 31));
}

// Minimizer-blocked filter: a key's 16-B block (4 words) is picked by the smallest hash of its
// canonical m-mers (m = k - KM), the word inside it and the three bits by the k-mer hash.  The
// canonical m-mer set of a k-mer equals that of its reverse complement, so the block is a
// function of the canonical k-mer; consecutive windows of a read share minimizers, so a
// thread's 32 windows load a few filter blocks instead of 32 (the scan is bound by the L2
// request rate, not by bytes).  Only used for ACGT-only windows (see lk_scan).
// Minimizer width: m = k - km m-mers, km + 1 of them per window.  km = 7 (eight m-mers per window)
// for k >= 18; for 15 <= k <= 17 km shrinks so that m stays 11: with fewer distinct m-mers (4^m) the
// filter's blocks would not spread (k = 15 with m = 8: 65 K minimizer blocks for the whole SDK set,
// filter words saturate and most windows pass); k < 15: plain per-window hashing (km = 0).
constexpr int LK_KM = 7;
inline int lk_km_for(int k) { return k >= 18 ? LK_KM : (k >= 15 ? k - 11 : 0); }
__device__ __forceinline__ uint64_t revcomp_code(uint64_t x, int m) {
    uint64_t y = ~x;                                           // complement: c -> 3 - c
    y = __builtin_bitreverse64(y);                             // reverse bits (and each pair)
    y = ((y >> 1) & 0x5555555555555555ull) | ((y & 0x5555555555555555ull) << 1);   // fix pairs
    return y >> (64 - 2 * m);
}
// Hash of a canonical m-mer: high half of one 64-bit product.  A multiplicative hash keeps
// the hashes of overlapping m-mers correlated, which lengthens minimizer runs (fewer filter
// blocks per thread); murmur-style mixing measured fewer false positives but 2x the scan time.
__device__ __forceinline__ uint32_t mmer_hash(uint64_t canon_m) {
    return (uint32_t)((canon_m * 0x9E3779B97F4A7C15ull) >> 32);
}
__device__ __forceinline__ uint64_t filter_word(uint32_t minh, uint64_t h, uint64_t fmask) {
    return ((((uint64_t)minh) << 2) | ((h >> 56) & 3u)) & fmask;
}
// Build side: the minimizer hash of canonical k-mer x (and the xor of its first and last
// m-mer hashes, see end_mix).
__device__ __forceinline__ uint32_t key_minimizer(uint64_t x, int k, int km, uint32_t* ends = nullptr) {
    const int m = k - km;
    const uint64_t mm = m >= 32 ? ~0ull : ((1ull << (2 * m)) - 1);
    uint32_t best = 0xFFFFFFFFu, e = 0;
    for (int i = 0; i <= km; ++i) {
        const uint64_t fm = (x >> (2 * (km - i))) & mm;
        const uint64_t rm = revcomp_code(fm, m);
        const uint32_t hh = mmer_hash(fm < rm ? fm : rm);
        best = hh < best ? hh : best;
        if (i == 0 || i == km) e ^= hh;
    }
    if (ends) *ends = e;
    return best;
}

// Filter word and bits of a k-mer inside its minimizer block (km > 0): from the hashes
// of the k-mer's first and last canonical m-mers, which a strand flip swaps, so their xor is a
// function of the canonical k-mer — the scan has both in registers already (the minimizer pass), so
// a window costs one 32-bit multiply instead of the 64-bit k-mer hash (lk_scan<0> 1.87 -> 1.81 ms at
// C3); the canonical code is formed only for the windows that pass.
__device__ __forceinline__ uint32_t end_mix(uint32_t e) {
    return (e ^ (e >> 16)) * 0x9E3779B1u;
}
// Partitioned block (km > 0): a key sets ONE bit in EACH of its block's four 32-bit words (5-bit
// fields of x from bit 27 down), a window passes when all four are set.  The lane loads the whole
// 16-B block per minimizer run anyway, so the four words cost nothing extra; against the former three
// bits of one word picked by two hash bits, the same 16-B request and ~12 VALU a window, filter false
// positives fall by ~40 % (tools/lk_filter_sim: 0.54 -> 0.32 per hit on a 1/8-scale C2/C3; each is a
// table-line probe in lk_scan).
__device__ __forceinline__ uint32_t part_bit(uint32_t x, int w) { return (x >> (27 - 5 * w)) & 31u; }
__device__ __forceinline__ uint64_t block_of(uint32_t minh, uint64_t fmask) { return (((uint64_t)minh) << 2) & fmask; }
__device__ __forceinline__ bool part_pass(const uint4& b, uint32_t x) {
    return ((b.x >> part_bit(x, 0)) & (b.y >> part_bit(x, 1)) & (b.z >> part_bit(x, 2)) & (b.w >> part_bit(x, 3)) & 1u) != 0;
}

// Packed layout (2k bits of key + the KmerID bits fit 64: the SDK sets of C3-C5): 32-B buckets of
// four u64 entries key << idb | KmerID, so a probe reads half a 64-B line instead of a whole one.
// An empty entry is ~0 (its key field, all ones, is the all-T code, which is never canonical).
constexpr int PBKT = 4;
struct alignas(32) PBucket {
    uint64_t e[PBKT];
};
static_assert(sizeof(PBucket) == 32, "half a line per packed bucket");
#ifndef HGA_LK_PACKED
#define HGA_LK_PACKED 1   // 0: always the 64-B layout
#endif

__global__ void lk_fill(Bucket* __restrict__ t, uint64_t nbk) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nbk * BKT) return;
    t[i / BKT].key[i % BKT] = EMPTY_KEY;
}

__global__ void lk_build(const uint64_t* __restrict__ keys, uint32_t n, Bucket* __restrict__ t, uint64_t nbk,
                         uint32_t* __restrict__ filt, uint64_t fmask, int k, int km, uint32_t idb) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t key = keys[i];
    const uint64_t h = tab_hash(key);
    if (km > 0) {
        uint32_t e;
        const uint32_t mz = key_minimizer(key, k, km, &e);
        const uint32_t x = end_mix(e);
        const uint64_t w0 = block_of(mz, fmask);
#pragma unroll
        for (int w = 0; w < 4; ++w) atomicOr(&filt[w0 + (uint64_t)w], 1u << part_bit(x, w));
    } else {
        atomicOr(&filt[filter_word(key_minimizer(key, k, km), h, fmask)], bloom_bits(h));
    }
    uint64_t b = bucket_of(h, nbk);
    if (idb) {   // packed buckets
        PBucket* pt = reinterpret_cast<PBucket*>(t);
        const unsigned long long ent = (key << idb) | i;
        while (true) {
            for (int s = 0; s < PBKT; ++s) {
                const unsigned long long old = atomicCAS((unsigned long long*)&pt[b].e[s], ~0ull, ent);
                if (old == ~0ull || (old >> idb) == key) return;
            }
            b = b + 1 == nbk ? 0 : b + 1;
        }
    }
    while (true) {
        for (int s = 0; s < BKT; ++s) {
            const unsigned long long old = atomicCAS((unsigned long long*)&t[b].key[s],
                                                     (unsigned long long)EMPTY_KEY, (unsigned long long)key);
            if (old == EMPTY_KEY || old == key) {
                t[b].id[s] = i;
                return;
            }
        }
        b = b + 1 == nbk ? 0 : b + 1;
    }
}

// Keys and ids of one bucket line.
struct Line {
    uint4 v[4];
    __device__ __forceinline__ uint64_t key(int s) const {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(v);
        return ((uint64_t)w[2 * s + 1] << 32) | w[2 * s];
    }
    __device__ __forceinline__ uint32_t id(int s) const {
        return reinterpret_cast<const uint32_t*>(v)[2 * BKT + s];
    }
};
__device__ __forceinline__ Line load_line(const Bucket* __restrict__ t, uint64_t b) {
    const uint4* p = reinterpret_cast<const uint4*>(t + b);
    Line l;
#pragma unroll
    for (int q = 0; q < 4; ++q) l.v[q] = p[q];
    return l;
}
// Looks key up in a loaded line: 1 = found (id set), 0 = absent (the line has an empty slot),
// -1 = line full without the key (continue with the next bucket).
__device__ __forceinline__ int line_find(const Line& l, uint64_t key, uint32_t& id) {
    bool found = false, empty = false;
    uint32_t v = 0;
#pragma unroll
    for (int s = 0; s < BKT; ++s) {   // compile-time slots: no dynamic register indexing
        const uint64_t kk = l.key(s);
        v = kk == key ? l.id(s) : v;
        found |= kk == key;
        empty |= kk == EMPTY_KEY;
    }
    id = v;
    return found ? 1 : (empty ? 0 : -1);
}
// Packed bucket: two 16-B loads, four entries.
struct PLine {
    uint4 v[2];
};
__device__ __forceinline__ PLine load_pline(const PBucket* __restrict__ t, uint64_t b) {
    const uint4* p = reinterpret_cast<const uint4*>(t + b);
    PLine l;
    l.v[0] = p[0];
    l.v[1] = p[1];
    return l;
}
__device__ __forceinline__ int pline_find(const PLine& l, uint64_t key, uint32_t idb, uint32_t& id) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(l.v);
    bool found = false, empty = false;
    uint32_t v = 0;
#pragma unroll
    for (int s = 0; s < PBKT; ++s) {
        const uint64_t e = ((uint64_t)w[2 * s + 1] << 32) | w[2 * s];
        const bool hit = (e >> idb) == key;
        v = hit ? (uint32_t)(idb >= 32 ? e : (e & ((1ull << idb) - 1))) : v;   // KmerIDs < 2^32
        found |= hit;
        empty |= e == ~0ull;
    }
    id = v;
    return found ? 1 : (empty ? 0 : -1);
}
// One bucket of either layout: 1 found (id set), 0 absent, -1 full without the key.
template <bool PK>
__device__ __forceinline__ int bucket_find(const void* __restrict__ t, uint64_t b, uint64_t key, uint32_t idb,
                                           uint32_t& id) {
    if constexpr (PK) return pline_find(load_pline(static_cast<const PBucket*>(t), b), key, idb, id);
    else return line_find(load_line(static_cast<const Bucket*>(t), b), key, id);
}
// Full probe from bucket b: KmerID or -1.
template <bool PK>
__device__ __forceinline__ int64_t lk_probe(const void* __restrict__ t, uint64_t nbk, uint32_t idb, uint64_t key,
                                            uint64_t b) {
    while (true) {
        uint32_t id;
        const int r = bucket_find<PK>(t, b, key, idb, id);
        if (r > 0) return id;
        if (r == 0) return -1;
        b = b + 1 == nbk ? 0 : b + 1;
    }
}

// Per read r (one wave): its start bit in the read-start bitmap, and word_read[w] = r for every
// 32-base word w with offs[r] <= 32w < offs[r+1] — the last read starting at or before base 32w
// (reads are whole CSR ranges; an empty read owns no word).  Coalesced runs of stores instead of a
// binary search per word (0.217 ms at C3 with 17 dependent offset loads per word).
__global__ void __launch_bounds__(256) lk_read_map(const uint64_t* __restrict__ offs, uint64_t nreads,
                                                   uint64_t nbases, unsigned int* __restrict__ sb,
                                                   uint32_t* __restrict__ word_read) {
    const uint64_t r = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (r >= nreads) return;
    const uint64_t p = offs[r], e = offs[r + 1];
    if (lane == 0 && p < nbases) atomicOr(&sb[SB_PAD + p / 32], 1u << (p & 31));
    for (uint64_t w = (p + 31) / 32 + lane; w < (e + 31) / 32; w += 64) word_read[w] = (uint32_t)r;
}

struct LkTab {
    const void* t;          // Bucket[nbk], or PBucket[nbk] when idb > 0
    const uint32_t* filt;
    uint64_t nbk, fmask;
    uint32_t idb;           // packed layout: KmerID bits of an entry (0: the 64-B layout)
    const uint8_t* asc;     // the ASCII reads when lk_scan packs its frames itself (HGA_LK_ASCII), else null
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

// K > 0: k known at compile time (masks and the m-mer / k-mer widths fold, narrowing the 64-bit
// hash multiplies); K == 0: any k.
template <bool EMIT, int KM, int K = 0, bool PK = false>
__global__ void __launch_bounds__(LK_T, (!EMIT && K != 0) ? HGA_LK_MINW : 1) lk_scan(const uint32_t* __restrict__ pk, const uint16_t* __restrict__ vd,
                                                const unsigned int* __restrict__ sb, uint64_t nbases,
                                                const uint64_t* __restrict__ offs, uint64_t nreads, int k_rt,
                                                const uint32_t* __restrict__ word_read,
                                                LkTab tab, uint32_t* __restrict__ hmask,
                                                uint32_t* __restrict__ win_kid,
                                                unsigned long long* __restrict__ tile_cnt,
                                                uint32_t* __restrict__ h_read, uint32_t* __restrict__ h_kid,
                                                uint32_t* __restrict__ h_pos, uint64_t* __restrict__ h_skey = nullptr,
                                                uint32_t* __restrict__ h_sval = nullptr, int kbits = 0) {
    __shared__ uint32_t ws[LK_T / 64 + 1];
    const int k = K ? K : k_rt;
    const uint64_t gt = (uint64_t)blockIdx.x * LK_T + threadIdx.x;
    const uint64_t p0 = gt * LK_P;
    const uint64_t mask = k >= 32 ? ~0ull : ((1ull << (2 * k)) - 1);
    if (!EMIT) {
        __shared__ uint64_t qkey[LK_T / 64][LK_QN];
        __shared__ uint16_t qorg[LK_T / 64][LK_QN];
        __shared__ uint32_t qcnt[LK_T / 64];
        __shared__ uint32_t lhit[LK_T];
        const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        if (lane == 0) qcnt[wave] = 0;
        lhit[threadIdx.x] = 0;
        wave_lds_sync();
        uint32_t hits = 0, ovf = 0;
        Frame<LK_P> f;
        if (p0 < nbases) {
            uint64_t v64;
            if (HGA_LK_ASCII && tab.asc) {   // the frame's four 16-base words packed from the ASCII reads
                FrameRaw<LK_P> raw;
#pragma unroll
                for (int i = 0; i < FrameRaw<LK_P>::NW; ++i)
                    pack_bytes<true>(load16(tab.asc, (int64_t)p0 - 32 + 16 * i, nbases), raw.x[i], raw.v[i]);
                v64 = build_frame<LK_P, true>(raw, k, f);
            } else {
                v64 = load_frame<LK_P, true>(pk, vd, PAD_WORDS + p0 / 16 - 2, k, f);
            }
            const uint32_t acgt = (uint32_t)(runs_of(v64, k) >> 32);   // window has only ACGT
            const uint64_t s64 = (uint64_t)sb[SB_PAD + p0 / 32 - 1] | ((uint64_t)sb[SB_PAD + p0 / 32] << 32);
            uint32_t wm = (uint32_t)(runs_of(~s64, k - 1) >> 32);   // no read start in (s, e]
            const uint64_t left = nbases - p0;
            if (left < 32) wm &= (1u << left) - 1u;
            // 1) minimizer of every window: hashes of the canonical m-mers ending at p0-KM..p0+31,
            //    then a sliding minimum of width KM+1 (van Herk / Gil-Werman, blocks of KM+1)
            constexpr int NM = LK_P + KM;
            constexpr int NWF = Frame<LK_P>::NW;
            const int m = k - KM;
            const uint64_t mm = m >= 32 ? ~0ull : ((1ull << (2 * m)) - 1);
            uint32_t mh[NM];
#pragma unroll
            for (int t = 0; t < NM; ++t) {
                const int pj = t - KM;   // m-mer ending at p0 + pj
                // fwd: the last m bases of the window frame; rc: the rc frame is pre-shifted so the
                // k-window ending at p0+j is field64(r, 2j); its m-mer ending at the same base sits
                // 2(k-m) bits higher, i.e. at field64(r, 2(pj + KM)) — both compile-time offsets
                const uint64_t fm = field64<NWF>(f.x, 2 * (16 * NWF - 33 - pj)) & mm;
                const uint64_t rm = field64<NWF>(f.r, 2 * (pj + KM)) & mm;
                mh[t] = mmer_hash(fm < rm ? fm : rm);
            }
            uint32_t wmin[LK_P];
            if constexpr (KM == 0) {
#pragma unroll
                for (int j = 0; j < LK_P; ++j) wmin[j] = mh[j];
            } else {
                constexpr int B = KM + 1;
                uint32_t pre[NM], suf[NM];
#pragma unroll
                for (int t = 0; t < NM; ++t) pre[t] = (t % B == 0) ? mh[t] : min(pre[t - 1], mh[t]);
#pragma unroll
                for (int t = NM - 1; t >= 0; --t)
                    suf[t] = (t % B == B - 1 || t == NM - 1) ? mh[t] : min(suf[t + 1], mh[t]);
#pragma unroll
                for (int j = 0; j < LK_P; ++j) wmin[j] = min(suf[j], pre[j + KM]);
            }
            // 2) filter blocks: a lane loads the 16-B block once per minimizer run (only the lanes
            //    whose run changes issue the load, so L2 sees one request per run) and serves
            //    the run's windows from registers.  Windows with a non-ACGT byte (REF codes are
            //    not strand-consistent there, so their minimizer block is undefined) always pass.
            //    Passing windows go to this wave's queue as (key, origin lane, window).
            const uint4* __restrict__ filt4 = reinterpret_cast<const uint4*>(tab.filt);
            const uint64_t bmask4 = tab.fmask >> 2;
            const uint32_t force = ~acgt;
            uint4 blk = make_uint4(0u, 0u, 0u, 0u);
            uint32_t cur = 0;
#pragma unroll
            for (int j = 0; j < LK_P; ++j) {
                const uint32_t bi = (uint32_t)(wmin[j] & bmask4);
                if (j == 0 || bi != cur) {
                    blk = filt4[bi];
                    cur = bi;
                }
                bool fp;   // the filter lets the window through
                if constexpr (KM > 0) {
                    fp = part_pass(blk, end_mix(mh[j] ^ mh[j + KM]));
                } else {
                    const uint64_t h = tab_hash(lk_canon(f, j, mask));
                    const uint32_t sel = (uint32_t)(h >> 56) & 3u, bb = bloom_bits(h);
                    const uint32_t wv = sel == 0 ? blk.x : sel == 1 ? blk.y : sel == 2 ? blk.z : blk.w;
                    fp = (wv & bb) == bb;
                }
                const bool pass = (fp || ((force >> j) & 1u)) && ((wm >> j) & 1u);
                if (pass) {
                    const uint64_t key = lk_canon(f, j, mask);
                    const uint32_t pos = atomicAdd(&qcnt[wave], 1u);
                    if (pos < LK_QN) {
                        qkey[wave][pos] = key;
                        qorg[wave][pos] = (uint16_t)((lane << 5) | j);
                    } else {
                        ovf |= 1u << j;
                    }
                }
            }
        }
        // 3) the wave's queue with every lane busy, two probes in flight per lane
        wave_lds_sync();
        const uint32_t nq = min(qcnt[wave], (uint32_t)LK_QN);
        const uint64_t gbase = (uint64_t)blockIdx.x * LK_T + (uint64_t)wave * 64;
        for (uint32_t q0 = 0; q0 < nq; q0 += 128) {
            const uint32_t i0 = q0 + lane, i1 = q0 + 64 + lane;
            const bool l0 = i0 < nq, l1 = i1 < nq;
            const uint64_t k0 = l0 ? qkey[wave][i0] : 0ull, k1 = l1 ? qkey[wave][i1] : 0ull;
            const uint64_t b0 = bucket_of(tab_hash(k0), tab.nbk), b1 = bucket_of(tab_hash(k1), tab.nbk);
            using LineK = std::conditional_t<PK, PLine, Line>;
            LineK L0, L1;
            auto load_k = [&](uint64_t b) {
                if constexpr (PK) return load_pline(static_cast<const PBucket*>(tab.t), b);
                else return load_line(static_cast<const Bucket*>(tab.t), b);
            };
            auto find_k = [&](const LineK& l, uint64_t key, uint32_t& id) {
                if constexpr (PK) return pline_find(l, key, tab.idb, id);
                else return line_find(l, key, id);
            };
            if (l0) L0 = load_k(b0);
            if (l1) L1 = load_k(b1);
            if (l0) {
                uint32_t id;
                int r = find_k(L0, k0, id);
                if (r < 0) {
                    const int64_t x = lk_probe<PK>(tab.t, tab.nbk, tab.idb, k0, b0 + 1 == tab.nbk ? 0 : b0 + 1);
                    r = x >= 0;
                    id = (uint32_t)x;
                }
                if (r > 0) {
                    const uint32_t o = qorg[wave][i0];
                    atomicOr(&lhit[wave * 64 + (o >> 5)], 1u << (o & 31));
                    win_kid[(gbase + (o >> 5)) * LK_P + (o & 31)] = id;
                }
            }
            if (l1) {
                uint32_t id;
                int r = find_k(L1, k1, id);
                if (r < 0) {
                    const int64_t x = lk_probe<PK>(tab.t, tab.nbk, tab.idb, k1, b1 + 1 == tab.nbk ? 0 : b1 + 1);
                    r = x >= 0;
                    id = (uint32_t)x;
                }
                if (r > 0) {
                    const uint32_t o = qorg[wave][i1];
                    atomicOr(&lhit[wave * 64 + (o >> 5)], 1u << (o & 31));
                    win_kid[(gbase + (o >> 5)) * LK_P + (o & 31)] = id;
                }
            }
        }
        wave_lds_sync();
        hits = lhit[threadIdx.x];
        // 4) queue overflow (rare): this lane probes its own leftovers
        while (ovf) {
            const int j = __builtin_ctz(ovf);
            ovf &= ovf - 1u;
            const uint64_t key = lk_canon_rt(f, j, mask);
            const int64_t x = lk_probe<PK>(tab.t, tab.nbk, tab.idb, key, bucket_of(tab_hash(key), tab.nbk));
            if (x >= 0) {
                hits |= 1u << j;
                win_kid[gt * LK_P + j] = (uint32_t)x;
            }
        }
        if (p0 < nbases) hmask[gt] = hits;
        uint32_t tot;
        (void)block_excl_scan<LK_T>((uint32_t)__popc(hits), ws, &tot);
        if (threadIdx.x == 0) tile_cnt[blockIdx.x] = tot;
        return;
    }
    // independent loads first (hit mask, tile offset, the read containing p0 — p0 is 32-aligned,
    // so it is precomputed per word), so their latencies overlap instead of chaining
    uint32_t hits = p0 < nbases ? hmask[gt] : 0u;
    const uint64_t tb = tile_cnt[blockIdx.x];
    uint64_t r = p0 < nbases ? word_read[p0 / 32] : 0u, re = 0;
    uint32_t tot;
    const uint32_t ex = block_excl_scan<LK_T>((uint32_t)__popc(hits), ws, &tot);
    if (tot == 0) return;   // uniform
    if (tot <= (uint32_t)LK_ST) {
        // the tile's hit windows listed in LDS at their tile offsets, then every thread takes hits
        // i, i + LK_T, ...: uniform work per lane (hits cluster at SNPs, so per-lane loops diverged:
        // 0.39 -> 0.245 ms at C3 against staging each lane's own hits), stores coalesced
        __shared__ uint32_t s_w[LK_ST];
        {
            uint32_t o = ex, h = hits;
            while (h) {
                const uint32_t j = (uint32_t)__builtin_ctz(h);
                h &= h - 1u;
                s_w[o++] = ((uint32_t)threadIdx.x << 5) | j;
            }
        }
        __syncthreads();
        const uint64_t gt0 = (uint64_t)blockIdx.x * LK_T;
        for (uint32_t i = threadIdx.x; i < tot; i += LK_T) {
            const uint32_t w = s_w[i];
            const uint64_t gtt = gt0 + (w >> 5);
            const uint64_t e = gtt * LK_P + (w & 31u);
            const uint32_t kk = win_kid[e];
            uint64_t rr = word_read[(gtt * LK_P) >> 5];   // word_read is per 32 bases
            uint64_t nx = offs[rr + 1];
            while (nx <= e) nx = offs[++rr + 1];
            const uint32_t pp = (uint32_t)(e + 1 - offs[rr]);
            h_read[tb + i] = (uint32_t)rr;
            h_kid[tb + i] = kk;
            h_pos[tb + i] = pp;
            h_skey[tb + i] = (rr << kbits) | kk;
            h_sval[tb + i] = pp;
        }
        return;
    }
    // more hits than the LDS list holds (rare): each lane writes its own
    if (hits) re = offs[r + 1];
    const uint32_t* __restrict__ wk = win_kid + gt * LK_P;
    uint64_t o = tb + ex;
    while (hits) {
        const int j = __builtin_ctz(hits);
        hits &= hits - 1u;
        const uint64_t e = p0 + j;
        while (re <= e) re = offs[++r + 1];
        const uint32_t kk = wk[j], pp = (uint32_t)(e + 1 - offs[r]);
        h_read[o] = (uint32_t)r;
        h_kid[o] = kk;
        h_pos[o] = pp;
        h_skey[o] = (r << kbits) | kk;
        h_sval[o] = pp;
        ++o;
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

// ---- kmer_component_index without LSD radix passes (ReadClusteringEngine.cpp:262-267, 282-284) ----
// The hits arrive in read order; kmer_component_index is, per KmerID, its reads ascending (with
// duplicates).  The top D KmerID bits (D <= 14) pick a bucket of ~2.5 K hits: one or two MSD passes of
// <= 7 bits each move (KmerID, read) pairs there — per tile a 128-way LDS counting sort, so every digit's
// run leaves the tile as one contiguous write (a single 4096-way pass writes 8-B runs: 0.51 ms at C3,
// the pattern of profiles/r05_slab_probe.txt); deterministic offsets from per-tile digit counts, no
// global atomics.  Then one workgroup per bucket counts its pairs into 2^S sub-buckets = single KmerIDs
// (S = kbits - D <= 10), which gives kci_ptr directly, places the reads by sub-bucket in LDS and each
// thread sorts its KmerIDs' reads (insertion sort of ~10 at C3; Shell sort for a crowded one) — the
// order a stable sort by KmerID leaves them in.  Replaces three 8-bit LSD passes and lk_ptr.
constexpr int KC_T = 512, KC_I = 16;
constexpr uint32_t KC_TILE = KC_T * KC_I;   // pairs per MSD tile (64 KB of LDS stage)
constexpr int KC_DMAX = 14, KC_SMAX = 10, KC_PASS_BITS = 7;
constexpr int KC_CT = 256, KC_PT = 16;      // bucket-sort workgroup, pairs a thread holds in registers
constexpr uint32_t KC_CAP = KC_CT * KC_PT;  // pairs per bucket (16 KB of u32 reads + 4 KB of counters in LDS: 8 workgroups a CU)
static_assert((1 << KC_SMAX) <= 4 * KC_CT, "lk_kci_bsort scans four sub-bucket counts a thread");

// An MSD tile: SEG = false, tile t of the hit arrays; SEG = true, tile t - tstart[s] of segment s
// (the previous pass's digit s at [sbase[s], sbase[s] + stot[s])).  Returns false past the last tile.
template <bool SEG>
__device__ __forceinline__ bool msd_tile(uint32_t t, uint64_t H, const uint32_t* tstart, const uint32_t* sbase,
                                         const uint32_t* stot, uint32_t& seg, uint64_t& lo, uint32_t& n) {
    if constexpr (!SEG) {
        seg = 0;
        lo = (uint64_t)t * KC_TILE;
        if (lo >= H) return false;
        n = (uint32_t)min<uint64_t>(H - lo, KC_TILE);
        return true;
    } else {
        if (t >= tstart[1u << KC_PASS_BITS]) return false;
        uint32_t a = 0, b = 1u << KC_PASS_BITS;   // the last segment with tstart <= t
        while (b - a > 1) {
            const uint32_t m = (a + b) / 2;
            if (tstart[m] <= t) a = m; else b = m;
        }
        seg = a;
        const uint32_t j = t - tstart[a];
        lo = (uint64_t)sbase[a] + (uint64_t)j * KC_TILE;
        n = min(stot[a] - j * KC_TILE, KC_TILE);
        return true;
    }
}
template <bool SEG>
__device__ __forceinline__ uint64_t msd_item(const uint32_t* hk, const uint32_t* hr, const uint64_t* pin, uint64_t i) {
    if constexpr (SEG) return pin[i];
    else return ((uint64_t)hk[i] << 32) | hr[i];
}
// per tile: counts of its digits (KmerID >> sh, nd of them), stored digit-major (rows[d][tile])
template <bool SEG>
__global__ void __launch_bounds__(KC_T) lk_msd_hist(const uint32_t* __restrict__ hk, const uint64_t* __restrict__ pin,
                                                    uint64_t H, int sh, uint32_t nd, const uint32_t* __restrict__ tstart,
                                                    const uint32_t* __restrict__ sbase, const uint32_t* __restrict__ stot,
                                                    uint32_t tiles, uint32_t* __restrict__ rows) {
    __shared__ uint32_t h[1 << KC_PASS_BITS];
    uint32_t seg, n;
    uint64_t lo;
    if (!msd_tile<SEG>(blockIdx.x, H, tstart, sbase, stot, seg, lo, n)) return;
    if (threadIdx.x < nd) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t dm = nd - 1;
#pragma unroll
    for (int q = 0; q < KC_I; ++q) {
        const uint32_t i = threadIdx.x + (uint32_t)q * KC_T;
        if (i < n) {
            const uint32_t k = SEG ? (uint32_t)(pin[lo + i] >> 32) : hk[lo + i];
            atomicAdd(&h[(k >> sh) & dm], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x < nd) rows[(uint64_t)threadIdx.x * tiles + blockIdx.x] = h[threadIdx.x];
}
// One wave per (segment s, digit d): the tiles tstart[s] .. tstart[s+1] of row d -> exclusive offsets
// inside (s, d) (in place), tot[s * nd + d] = its size.  tstart == nullptr: one segment of all tiles.
__global__ void __launch_bounds__(256) lk_msd_bscan(uint32_t* __restrict__ rows, uint32_t tiles, uint32_t nd,
                                                    uint32_t nseg, const uint32_t* __restrict__ tstart,
                                                    uint32_t* __restrict__ tot) {
    const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w >= nseg * nd) return;
    const uint32_t sg = w / nd, d = w % nd;
    const uint32_t t0 = tstart ? tstart[sg] : 0u, t1 = tstart ? tstart[sg + 1] : tiles;
    uint32_t* __restrict__ r = rows + (uint64_t)d * tiles;
    uint32_t run = 0;
    for (uint32_t tb = t0; tb < t1; tb += 64) {
        const uint32_t t = tb + lane;
        const uint32_t c = t < t1 ? r[t] : 0u;
        const uint32_t inc = wave_incl_scan(c, (int)lane);
        if (t < t1) r[t] = run + inc - c;
        run += __shfl(inc, 63, 64);
    }
    if (lane == 0) tot[w] = run;
}
// Tiles of the second pass: tstart[s] = sum of ceil(tot[s'] / KC_TILE) over s' < s (<= 128 segments;
// past nseg the total)
__global__ void lk_msd_tiles(const uint32_t* __restrict__ tot, uint32_t nseg, uint32_t* __restrict__ tstart) {
    if (threadIdx.x != 0) return;
    uint32_t o = 0;
    for (uint32_t sg = 0; sg <= (1u << KC_PASS_BITS); ++sg) {
        tstart[sg] = o;
        if (sg < nseg) o += (tot[sg] + KC_TILE - 1) / KC_TILE;
    }
}
// Per tile: a 64-way counting sort of its pairs in LDS by digit, then each digit's run written
// contiguously at obase[seg * nd + d] + the tile's offset inside (seg, d) (lk_msd_bscan)
template <bool SEG>
__global__ void __launch_bounds__(KC_T) lk_msd_scatter(const uint32_t* __restrict__ hk, const uint32_t* __restrict__ hr,
                                                       const uint64_t* __restrict__ pin, uint64_t H, int sh, uint32_t nd,
                                                       const uint32_t* __restrict__ tstart, const uint32_t* __restrict__ sbase,
                                                       const uint32_t* __restrict__ stot, uint32_t tiles,
                                                       const uint32_t* __restrict__ rows, const uint32_t* __restrict__ obase,
                                                       uint64_t* __restrict__ out) {
    __shared__ uint64_t st[KC_TILE];
    __shared__ uint32_t cnt[1 << KC_PASS_BITS], lst[1 << KC_PASS_BITS];
    __shared__ unsigned long long gof[1 << KC_PASS_BITS];
    uint32_t seg, n;
    uint64_t lo;
    if (!msd_tile<SEG>(blockIdx.x, H, tstart, sbase, stot, seg, lo, n)) return;
    const uint32_t tid = threadIdx.x, dm = nd - 1;
    if (tid < nd) cnt[tid] = 0;   // (nd <= 128 < KC_T)
    __syncthreads();
    uint64_t it[KC_I];
    uint32_t rk[KC_I];
#pragma unroll
    for (int q = 0; q < KC_I; ++q) {
        const uint32_t i = tid + (uint32_t)q * KC_T;
        it[q] = i < n ? msd_item<SEG>(hk, hr, pin, lo + i) : 0ull;
    }
#pragma unroll
    for (int q = 0; q < KC_I; ++q)
        if (tid + (uint32_t)q * KC_T < n) rk[q] = atomicAdd(&cnt[((uint32_t)(it[q] >> 32) >> sh) & dm], 1u);
    __syncthreads();
    if (tid < 64) {   // one wave scans the <= 128 digit counts, two a lane
        const uint32_t c0 = 2 * tid < nd ? cnt[2 * tid] : 0u, c1 = 2 * tid + 1 < nd ? cnt[2 * tid + 1] : 0u;
        const uint32_t inc = wave_incl_scan(c0 + c1, (int)tid);
        if (2 * tid < nd) {
            lst[2 * tid] = inc - c0 - c1;
            gof[2 * tid] = (unsigned long long)obase[seg * nd + 2 * tid] + rows[(uint64_t)(2 * tid) * tiles + blockIdx.x];
        }
        if (2 * tid + 1 < nd) {
            lst[2 * tid + 1] = inc - c1;
            gof[2 * tid + 1] = (unsigned long long)obase[seg * nd + 2 * tid + 1] +
                               rows[(uint64_t)(2 * tid + 1) * tiles + blockIdx.x];
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < KC_I; ++q)
        if (tid + (uint32_t)q * KC_T < n) st[lst[((uint32_t)(it[q] >> 32) >> sh) & dm] + rk[q]] = it[q];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < KC_I; ++q) {
        const uint32_t i = tid + (uint32_t)q * KC_T;
        if (i < n) {
            const uint64_t v = st[i];
            const uint32_t d = ((uint32_t)(v >> 32) >> sh) & dm;
            out[gof[d] + (i - lst[d])] = v;
        }
    }
}
// bbase[b] = exclusive scan of tot (nb <= 16384: one 1024-thread workgroup, sixteen a thread); stat[0] =
// the largest bucket
__global__ void __launch_bounds__(1024) lk_kci_scan(const uint32_t* __restrict__ tot, uint32_t nb,
                                                    uint32_t* __restrict__ bbase, unsigned long long* __restrict__ stat) {
    constexpr int V = (1 << KC_DMAX) / 1024;
    __shared__ uint32_t ws[1024 / 64 + 1];
    __shared__ uint32_t mx;
    const uint32_t t = threadIdx.x;
    if (t == 0) mx = 0;
    uint32_t v[V], sum = 0, m = 0;
#pragma unroll
    for (int q = 0; q < V; ++q) {
        const uint32_t i = V * t + (uint32_t)q;
        v[q] = i < nb ? tot[i] : 0u;
        sum += v[q];
        m = max(m, v[q]);
    }
    uint32_t total;
    uint32_t o = block_excl_scan<1024>(sum, ws, &total);
#pragma unroll
    for (int q = 0; q < V; ++q) {
        const uint32_t i = V * t + (uint32_t)q;
        if (i < nb) bbase[i] = o;
        o += v[q];
    }
    atomicMax(&mx, m);
    __syncthreads();
    if (t == 0) stat[0] = mx;
}
// One workgroup per bucket: sub-bucket counts -> kci_ptr of its KmerIDs, reads placed by KmerID in LDS,
// each KmerID's reads sorted ascending, written to kci_val.  A bucket past KC_CAP sets *flag (the host
// redoes the index by the radix path).
__global__ void __launch_bounds__(KC_CT) lk_kci_bsort(const uint64_t* __restrict__ pairs, const uint32_t* __restrict__ tot,
                                                      const uint32_t* __restrict__ bbase, int S, uint64_t n_sdk,
                                                      uint64_t H, uint64_t* __restrict__ kptr, uint32_t* __restrict__ kv,
                                                      unsigned long long* __restrict__ flag) {
    __shared__ uint32_t sk[KC_CAP];
    __shared__ uint32_t cnt[1 << KC_SMAX];
    __shared__ uint32_t ws[KC_CT / 64 + 1];
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    const uint32_t n = tot[b], st = bbase[b];
    const uint32_t ns = 1u << S;
    if (b == 0 && tid == 0) kptr[n_sdk] = H;
    if (n > KC_CAP) {
        if (tid == 0) atomicOr(flag, 1ull);
        return;
    }
    for (uint32_t i = tid; i < ns; i += KC_CT) cnt[i] = 0;
    __syncthreads();
    const uint64_t* __restrict__ src = pairs + st;
    uint64_t pr[KC_PT];   // the bucket is read once: all loads in flight, then the ranks by LDS atomics
    const uint64_t smask = ((1ull << S) - 1ull) << 32;
#pragma unroll
    for (int q = 0; q < KC_PT; ++q) {   // (KmerID, read) -> (its low S bits, read)
        const uint32_t i = tid + (uint32_t)q * KC_CT;
        const uint64_t v = i < n ? src[i] : 0ull;
        pr[q] = (v & smask) | (uint32_t)v;
    }
#pragma unroll
    for (int q = 0; q < KC_PT; ++q)   // the rank inside the sub-bucket joins the high word (sub < 2^12, rank < 2^14)
        if (tid + (uint32_t)q * KC_CT < n) {
            const uint32_t sb = (uint32_t)(pr[q] >> 32);
            pr[q] += (uint64_t)atomicAdd(&cnt[sb], 1u) << 44;
        }
    __syncthreads();
    {   // exclusive scan of the sub-bucket counts (<= 4096: four a thread); kci_ptr of the bucket's KmerIDs
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = 4 * tid + (uint32_t)q;
            v[q] = i < ns ? cnt[i] : 0u;
            sum += v[q];
        }
        uint32_t total;
        uint32_t o = block_excl_scan<KC_CT>(sum, ws, &total);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = 4 * tid + (uint32_t)q;
            if (i < ns) {
                cnt[i] = o;
                const uint64_t kid = ((uint64_t)b << S) | i;
                if (kid < n_sdk) kptr[kid] = (uint64_t)st + o;
            }
            o += v[q];
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < KC_PT; ++q)
        if (tid + (uint32_t)q * KC_CT < n)
            sk[cnt[(uint32_t)(pr[q] >> 32) & 0xfffu] + (uint32_t)(pr[q] >> 44)] = (uint32_t)pr[q];
    __syncthreads();
    constexpr uint32_t gaps[8] = {701, 301, 132, 57, 23, 10, 4, 1};
    for (uint32_t s2 = tid; s2 < ns; s2 += KC_CT) {
        const uint32_t lo = cnt[s2], hi = s2 + 1 < ns ? cnt[s2 + 1] : n;
        for (int gi = 0; gi < 8; ++gi) {   // Shell sort (gap 1 = insertion sort of a KmerID's ~11 reads)
            const uint32_t g = gaps[gi];
            if (g >= hi - lo) continue;
            for (uint32_t i = lo + g; i < hi; ++i) {
                const uint32_t v = sk[i];
                uint32_t j = i;
                for (; j >= lo + g && sk[j - g] > v; j -= g) sk[j] = sk[j - g];
                sk[j] = v;
            }
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < n; i += KC_CT) kv[(uint64_t)st + i] = sk[i];
}

// Number of non-empty CSR segments, the largest one, and the segments with more than 512 / 2048 entries
// listed for the per-segment sort tiers (order irrelevant; one list atomic per workgroup): out[0] non-empty
// segments, out[1] largest, out[2] / out[3]
// the two list lengths — all read back with one synchronisation.
__global__ void __launch_bounds__(1024) lk_seg_stats(const uint64_t* __restrict__ ptr, uint64_t nseg,
                                                     unsigned long long* __restrict__ out, uint32_t* __restrict__ mid,
                                                     uint32_t* __restrict__ big, uint32_t lo_mid, uint32_t lo_big) {
    __shared__ uint32_t ws[1024 / 64 + 1];
    __shared__ unsigned long long smax, s_mid, s_big;
    const uint64_t s = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    const uint64_t len = s < nseg ? ptr[s + 1] - ptr[s] : 0;
    if (threadIdx.x == 0) smax = 0;
    __syncthreads();
    if (len) atomicMax(&smax, (unsigned long long)len);
    uint32_t tot, nm, nbg;
    (void)block_excl_scan<1024>(len ? 1u : 0u, ws, &tot);
    const uint32_t em = block_excl_scan<1024>(len > lo_mid ? 1u : 0u, ws, &nm);
    const uint32_t eb = block_excl_scan<1024>(len > lo_big ? 1u : 0u, ws, &nbg);
    if (threadIdx.x == 0) {
        if (tot) atomicAdd(&out[0], (unsigned long long)tot);
        if (smax) atomicMax(&out[1], smax);
        s_mid = nm ? atomicAdd(&out[2], (unsigned long long)nm) : 0ull;
        s_big = nbg ? atomicAdd(&out[3], (unsigned long long)nbg) : 0ull;
    }
    __syncthreads();
    if (len > lo_mid) mid[s_mid + em] = (uint32_t)s;
    if (len > lo_big) big[s_big + eb] = (uint32_t)s;
}

// Reads with more than `lo` hits (order irrelevant).
__global__ void lk_big_reads(const uint64_t* __restrict__ hptr, uint64_t n, uint64_t lo,
                             uint32_t* __restrict__ list, unsigned long long* __restrict__ cnt) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n && hptr[r + 1] - hptr[r] > lo) list[atomicAdd(cnt, 1ull)] = (uint32_t)r;
}

// Per-read sort of the (read << kbits | KmerID, position) pairs: one workgroup per read with
// 2 <= hits <= NT * IPT.  The hits of a read arrive in window order (positions ascending), so a
// STABLE sort by KmerID alone gives the (KmerID, position) order of the stable (read, KmerID)
// sort (ReadClusteringEngine.cpp:262-272: sorted ids; :267 first occurrence): LSD passes over
// 8-bit digits of the KmerID in LDS, ranks by ballot-matched digits inside each wave (items in
// (row, lane) order, waves in order).  `list` (optional) names the reads to sort.
template <int NT, int IPT>
__global__ void __launch_bounds__(NT) lk_segsort(const uint64_t* __restrict__ hptr, uint64_t nreads, int kbits,
                                                 uint64_t* __restrict__ sk, uint32_t* __restrict__ sv,
                                                 uint32_t lo_excl, const uint32_t* __restrict__ list) {
    static_assert(NT >= 256 && NT % 64 == 0, "digit scan: one thread per digit");
    constexpr int NW = NT / 64, CAP = NT * IPT;
    __shared__ uint64_t buf[CAP];
    __shared__ uint32_t wcnt[NW][256];
    __shared__ uint32_t ws[NW + 1];
    const uint64_t r = list ? list[blockIdx.x] : blockIdx.x;
    if (r >= nreads) return;
    const uint64_t b = hptr[r], cnt64 = hptr[r + 1] - b;
    if (cnt64 <= lo_excl || cnt64 > (uint64_t)CAP) return;
    const uint32_t cnt = (uint32_t)cnt64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t kmask = (1ull << kbits) - 1;
    const uint64_t lt = (1ull << lane) - 1ull;
    uint64_t key[IPT];   // position << 32 | KmerID
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint32_t i = (uint32_t)wave * (IPT * 64) + (uint32_t)j * 64 + lane;
        key[j] = i < cnt ? ((uint64_t)sv[b + i] << 32) | (sk[b + i] & kmask) : 0ull;
    }
    for (int sh = 0; sh < kbits; sh += 8) {
        const uint32_t dm = kbits - sh >= 8 ? 255u : ((1u << (kbits - sh)) - 1u);
        for (int i = tid; i < NW * 256; i += NT) (&wcnt[0][0])[i] = 0;
        __syncthreads();
        uint32_t dig[IPT], rank[IPT];
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const uint32_t i0 = (uint32_t)wave * (IPT * 64) + (uint32_t)j * 64;   // wave-uniform
            const bool ok = i0 + lane < cnt;
            const uint32_t d = ok ? ((uint32_t)(key[j] >> sh) & dm) : 256u;
            dig[j] = d;
            rank[j] = 0;
            if (i0 >= cnt) continue;
            uint64_t m = __ballot(ok);
#pragma unroll
            for (int bb = 0; bb < 8; ++bb) {
                const bool bit = (d >> bb) & 1u;
                const uint64_t mb = __ballot(bit);
                m &= bit ? mb : ~mb;
            }
            uint32_t before = 0;
            if (ok) before = wcnt[wave][d];
            rank[j] = before + (uint32_t)__popcll(m & lt);
            if (ok && (m & lt) == 0ull) wcnt[wave][d] = before + (uint32_t)__popcll(m);
            wave_lds_sync();
        }
        __syncthreads();
        {   // digit starts, then each wave's start inside its digit (waves in order: stable)
            const uint32_t d = (uint32_t)tid & 255u;
            uint32_t tot_d = 0;
            if (tid < 256)
                for (int w = 0; w < NW; ++w) tot_d += wcnt[w][d];
            uint32_t tt;
            const uint32_t exd = block_excl_scan<NT>(tid < 256 ? tot_d : 0u, ws, &tt);
            if (tid < 256) {
                uint32_t o = exd;
                for (int w = 0; w < NW; ++w) {
                    const uint32_t c = wcnt[w][d];
                    wcnt[w][d] = o;
                    o += c;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IPT; ++j)
            if (dig[j] < 256u) buf[wcnt[wave][dig[j]] + rank[j]] = key[j];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const uint32_t i = (uint32_t)wave * (IPT * 64) + (uint32_t)j * 64 + lane;
            if (i < cnt) key[j] = buf[i];
        }
        __syncthreads();
    }
    const uint64_t rk = r << kbits;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint32_t i = (uint32_t)wave * (IPT * 64) + (uint32_t)j * 64 + lane;
        if (i < cnt) {
            sk[b + i] = rk | (key[j] & kmask);
            sv[b + i] = (uint32_t)(key[j] >> 32);
        }
    }
}

// The same sort for reads of at most 64 * WIPT hits, one wave per read and no workgroup barrier:
// the 256 digit counts live four per lane and are scanned with shuffles (most reads, ~220 hits
// at C3, fit; a 256-thread workgroup would leave three waves idle behind its barriers).
constexpr int WIPT = 8;
__global__ void __launch_bounds__(64) lk_wsort(const uint64_t* __restrict__ hptr, uint64_t nreads, int kbits,
                                               uint64_t* __restrict__ sk, uint32_t* __restrict__ sv) {
    __shared__ uint64_t buf[64 * WIPT];
    __shared__ uint32_t wcnt[256];
    const uint64_t r = blockIdx.x;
    if (r >= nreads) return;
    const uint64_t b = hptr[r], cnt64 = hptr[r + 1] - b;
    if (cnt64 < 2 || cnt64 > 64u * WIPT) return;
    const uint32_t cnt = (uint32_t)cnt64;
    const int lane = threadIdx.x;
    const uint64_t kmask = (1ull << kbits) - 1;
    const uint64_t lt = (1ull << lane) - 1ull;
    uint64_t key[WIPT];   // position << 32 | KmerID, item i = j * 64 + lane
#pragma unroll
    for (int j = 0; j < WIPT; ++j) {
        const uint32_t i = (uint32_t)j * 64 + lane;
        key[j] = i < cnt ? ((uint64_t)sv[b + i] << 32) | (sk[b + i] & kmask) : 0ull;
    }
    for (int sh = 0; sh < kbits; sh += 8) {
        const uint32_t dm = kbits - sh >= 8 ? 255u : ((1u << (kbits - sh)) - 1u);
#pragma unroll
        for (int q = 0; q < 4; ++q) wcnt[q * 64 + lane] = 0;
        wave_lds_sync();
        uint32_t dig[WIPT], rank[WIPT];
#pragma unroll
        for (int j = 0; j < WIPT; ++j) {
            const bool ok = (uint32_t)j * 64 + lane < cnt;
            const uint32_t d = ok ? ((uint32_t)(key[j] >> sh) & dm) : 256u;
            dig[j] = d;
            rank[j] = 0;
            if ((uint32_t)j * 64 >= cnt) continue;   // wave-uniform
            uint64_t m = __ballot(ok);
#pragma unroll
            for (int bb = 0; bb < 8; ++bb) {
                const bool bit = (d >> bb) & 1u;
                const uint64_t mb = __ballot(bit);
                m &= bit ? mb : ~mb;
            }
            uint32_t before = 0;
            if (ok) before = wcnt[d];
            rank[j] = before + (uint32_t)__popcll(m & lt);
            if (ok && (m & lt) == 0ull) wcnt[d] = before + (uint32_t)__popcll(m);
            wave_lds_sync();
        }
        {   // exclusive scan of the 256 digit counts: lane l holds digits 4l..4l+3
            const uint32_t c0 = wcnt[4 * lane], c1 = wcnt[4 * lane + 1], c2 = wcnt[4 * lane + 2],
                           c3 = wcnt[4 * lane + 3];
            const uint32_t s4 = c0 + c1 + c2 + c3;
            const uint32_t ex = wave_incl_scan(s4, lane) - s4;
            wave_lds_sync();
            wcnt[4 * lane] = ex;
            wcnt[4 * lane + 1] = ex + c0;
            wcnt[4 * lane + 2] = ex + c0 + c1;
            wcnt[4 * lane + 3] = ex + c0 + c1 + c2;
            wave_lds_sync();
        }
#pragma unroll
        for (int j = 0; j < WIPT; ++j)
            if (dig[j] < 256u) buf[wcnt[dig[j]] + rank[j]] = key[j];
        wave_lds_sync();
#pragma unroll
        for (int j = 0; j < WIPT; ++j) {
            const uint32_t i = (uint32_t)j * 64 + lane;
            if (i < cnt) key[j] = buf[i];
        }
        wave_lds_sync();
    }
    const uint64_t rk = r << kbits;
#pragma unroll
    for (int j = 0; j < WIPT; ++j) {
        const uint32_t i = (uint32_t)j * 64 + lane;
        if (i < cnt) {
            sk[b + i] = rk | (key[j] & kmask);
            sv[b + i] = (uint32_t)(key[j] >> 32);
        }
    }
}


constexpr int FC = 4;   // chunks of 64 hits per round in the first-occurrence passes
// First occurrences per (read, KmerID) from the per-read sorted hits, one wave per read (no
// H-sized flag array or scan): pass A writes the sorted KmerIDs and counts each read's distinct
// ids into cnt[r]; after an exclusive scan over the reads (= the first-occurrence CSR pointers)
// pass B writes each read's heads at its offset, in sorted order (ReadClusteringEngine.cpp:267).
__global__ void __launch_bounds__(256) lk_first_count(const uint64_t* __restrict__ hptr, uint64_t n,
                                                      const uint64_t* __restrict__ key, uint64_t kmask,
                                                      uint32_t* __restrict__ sorted_kid, uint64_t* __restrict__ cnt) {
    const uint64_t r = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= n) return;
    const uint64_t b = hptr[r], e = hptr[r + 1];
    uint64_t prev = ~0ull;   // last key of the previous chunk
    uint32_t u = 0;
    for (uint64_t i00 = b; i00 < e; i00 += 64 * FC) {   // FC chunks' loads in flight together
        uint64_t kk[FC];
#pragma unroll
        for (int t = 0; t < FC; ++t) {
            const uint64_t i = i00 + 64 * t + lane;
            kk[t] = i < e ? key[i] : 0ull;
        }
#pragma unroll
        for (int t = 0; t < FC; ++t) {
            const uint64_t i = i00 + 64 * t + lane;
            if (i00 + 64 * t >= e) break;   // wave-uniform
            const bool ok = i < e;
            const uint64_t k = kk[t];
            uint64_t kp = __shfl_up(k, 1, 64);
            if (lane == 0) kp = prev;
            const bool head = ok && k != kp;
            if (ok) sorted_kid[i] = (uint32_t)(k & kmask);
            u += (uint32_t)__popcll(__ballot(head));
            prev = __shfl(k, 63, 64);
        }
    }
    if (lane == 0) cnt[r] = u;
}
__global__ void __launch_bounds__(256) lk_first_write(const uint64_t* __restrict__ hptr, uint64_t n,
                                                      const uint64_t* __restrict__ key,
                                                      const uint32_t* __restrict__ pos,
                                                      const uint64_t* __restrict__ foff, uint64_t kmask,
                                                      uint32_t* __restrict__ fk, uint32_t* __restrict__ fp,
                                                      uint32_t* __restrict__ fr) {
    const uint64_t r = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= n) return;
    const uint64_t b = hptr[r], e = hptr[r + 1];
    const uint64_t lt = (1ull << lane) - 1ull;
    uint64_t prev = ~0ull, o = foff[r];
    for (uint64_t i00 = b; i00 < e; i00 += 64 * FC) {   // FC chunks' loads in flight together
        uint64_t kk[FC];
        uint32_t pp[FC];
#pragma unroll
        for (int t = 0; t < FC; ++t) {
            const uint64_t i = i00 + 64 * t + lane;
            kk[t] = i < e ? key[i] : 0ull;
            pp[t] = i < e ? pos[i] : 0u;   // with the key: no dependent load per head
        }
#pragma unroll
        for (int t = 0; t < FC; ++t) {
            if (i00 + 64 * t >= e) break;   // wave-uniform
            const uint64_t i = i00 + 64 * t + lane;
            const bool ok = i < e;
            const uint64_t k = kk[t];
            const uint32_t ps = pp[t];
            uint64_t kp = __shfl_up(k, 1, 64);
            if (lane == 0) kp = prev;
            const bool head = ok && k != kp;
            const uint64_t m = __ballot(head);
            if (head) {
                const uint64_t at = o + (uint64_t)__popcll(m & lt);
                fk[at] = (uint32_t)(k & kmask);
                fp[at] = ps;
                fr[at] = (uint32_t)r;
            }
            o += (uint64_t)__popcll(m);
            prev = __shfl(k, 63, 64);
        }
    }
}


inline unsigned blocks_for(uint64_t n, int t) { return (unsigned)((n + t - 1) / t); }
inline int bits_for(uint64_t n) {   // bits to hold values in [0, n)
    int b = 0;
    while (b < 64 && (n - 1) >> b) ++b;
    return b < 1 ? 1 : b;
}

}  // namespace

// Stable per-segment sort of (sk low kbits, sv) by the key, segments hptr[s]..hptr[s+1] of at
// most maxlen <= 16384 entries (returns false, doing nothing, above that): one wave per segment
// up to 512 entries, listed segments on 256- and 1024-thread workgroups above.  Leaves
// sk = s << kbits | key (segments of one entry are not touched: sk must arrive composed).  maxlen ~0: measured here (with the tier lists).  `ctr2`: two device counters of scratch.
bool segment_sort(hga_ctx* c, const uint64_t* hptr, uint64_t nseg, uint64_t maxlen, int kbits, uint64_t* sk,
                  uint32_t* sv, DevBuf& list_buf, unsigned long long* ctr2, const char* label, uint32_t* lists,
                  const unsigned long long* lists_n) {
    unsigned long long h4[4] = {0, 0, 0, 0};
    if (maxlen == ~0ull && !lists) {   // unknown: the longest segment and the tier lists, one read-back
        const size_t lb = (2 * nseg * 4 + 7) & ~(size_t)7;
        char* lp = static_cast<char*>(list_buf.ensure(lb + 64));
        lists = reinterpret_cast<uint32_t*>(lp);
        auto* cnt = reinterpret_cast<unsigned long long*>(lp + lb);
        HGA_HIP(hipMemsetAsync(cnt, 0, 32, c->stream));
        if (nseg)
            hipLaunchKernelGGL(lk_seg_stats, dim3(blocks_for(nseg, 1024)), dim3(1024), 0, c->stream, hptr, nseg, cnt,
                               lists, lists + nseg, (uint32_t)(64 * WIPT), 2048u);
        HGA_HIP(hipMemcpyAsync(h4, cnt, 32, hipMemcpyDeviceToHost, c->stream));
        c->sync();
        maxlen = h4[1];
        lists_n = h4 + 2;
    }
    if (maxlen > 16384 || nseg >= (1ull << 31)) return false;
    uint32_t* mid = nullptr;
    uint32_t* big = nullptr;
    unsigned long long nl[2] = {0, 0};
    if (maxlen > 64u * WIPT && lists) {   // listed by the caller (lk_seg_stats)
        mid = lists;
        big = lists + nseg;
        nl[0] = lists_n[0];
        nl[1] = lists_n[1];
    } else if (maxlen > 64u * WIPT) {
        mid = static_cast<uint32_t*>(list_buf.ensure(2 * nseg * 4 + 64));
        big = mid + nseg;
        HGA_HIP(hipMemsetAsync(ctr2, 0, 16, c->stream));
        hipLaunchKernelGGL(lk_big_reads, dim3(blocks_for(nseg, 256)), dim3(256), 0, c->stream, hptr, nseg,
                           (unsigned long long)(64 * WIPT), mid, ctr2);
        if (maxlen > 2048)
            hipLaunchKernelGGL(lk_big_reads, dim3(blocks_for(nseg, 256)), dim3(256), 0, c->stream, hptr, nseg,
                               2048ull, big, ctr2 + 1);
        HGA_HIP(hipMemcpyAsync(nl, ctr2, 16, hipMemcpyDeviceToHost, c->stream));
        c->sync();
        HGA_HIP(hipMemsetAsync(ctr2, 0, 16, c->stream));
    }
    c->launch(label, [&] {
        hipLaunchKernelGGL(lk_wsort, dim3((unsigned)nseg), dim3(64), 0, c->stream, hptr, nseg, kbits, sk, sv);
        if (nl[0])
            hipLaunchKernelGGL((lk_segsort<256, 8>), dim3((unsigned)nl[0]), dim3(256), 0, c->stream, hptr, nseg,
                               kbits, sk, sv, (uint32_t)(64 * WIPT), (const uint32_t*)mid);
        if (nl[1])
            hipLaunchKernelGGL((lk_segsort<1024, 16>), dim3((unsigned)nl[1]), dim3(1024), 0, c->stream, hptr, nseg,
                               kbits, sk, sv, 2048u, (const uint32_t*)big);
    });
    c->check_launch("segment_sort");
    return true;
}

void lookup_load(hga_ctx* c, int k, const uint64_t* keys, uint32_t n) {
    HGA_REQUIRE(k >= 1 && k <= 32, HGA_ERR_INVALID, "k must be in [1,32]");
    auto& L = c->lookup;
    // packed 32-B buckets when a key and its KmerID fit one u64 (HGA_LK_WIDE: test hook for the 64-B layout)
    const int nbits_id = bits_for(std::max<uint32_t>(n, 1));
    const uint32_t idb = HGA_LK_PACKED && 2 * k + nbits_id <= 64 && !std::getenv("HGA_LK_WIDE") ? 64u - 2u * (uint32_t)k
                                                                                                   : 0u;
    const int bkt = idb ? PBKT : BKT;
    const uint64_t nbk = std::max<uint64_t>(64, ((uint64_t)HGA_LK_SLOTS10 * n / 10 + bkt - 1) / bkt);   // slot load 10 / HGA_LK_SLOTS10
    uint64_t fw = 1024;
    while (fw * 64 < (uint64_t)HGA_FBITS2 * n) fw <<= 1;   // >= HGA_FBITS2/2 filter bits per key
    L.slots = nbk;   // buckets
    L.idb = idb;
    L.fwords = fw;
    L.k = k;
    L.km = lk_km_for(k);
    L.n_sdk = n;
    Bucket* tb = static_cast<Bucket*>(L.tab_key.ensure(nbk * (idb ? sizeof(PBucket) : sizeof(Bucket))));
    auto* filt = static_cast<uint32_t*>(L.filter.ensure(fw * 4));
    DevBuf tmp;
    uint64_t* dk = static_cast<uint64_t*>(tmp.ensure(std::max<uint64_t>(n, 1) * 8));
    if (n) HGA_HIP(hipMemcpyAsync(dk, keys, (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
    if (idb) {
        HGA_HIP(hipMemsetAsync(tb, 0xFF, nbk * sizeof(PBucket), c->stream));
    } else {
        hipLaunchKernelGGL(lk_fill, dim3(blocks_for(nbk * BKT, 256)), dim3(256), 0, c->stream, tb, nbk);
        c->check_launch("lk_fill");
    }
    HGA_HIP(hipMemsetAsync(filt, 0, fw * 4, c->stream));
    if (n) {
        c->launch("lk_build", [&] {
            hipLaunchKernelGGL(lk_build, dim3(blocks_for(n, 256)), dim3(256), 0, c->stream, dk, n, tb, nbk, filt,
                               fw - 1, k, L.km, idb);
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
    L.gathered = false;
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
    L.packed_ok = false;
    L.ran = false;
}

// The per-base encode of KmerIterator (KmerIterator.cpp:54-76) over the resident ASCII reads:
// packed 2-bit codes + valid bits (pack_kernel<REF>), the read-start bitmap and the per-word read
// index.  Part of every hga_lookup_run (the reference encodes inside construct_indices,
// ReadClusteringEngine.cpp:248-254); hga_hll_registers packs when the reads changed since.
void lookup_pack(hga_ctx* c, bool skip_codes) {
    auto& L = c->lookup;
    const uint64_t n = L.n_reads, nb = L.n_bases;
    const uint64_t nw = (nb + 15) / 16, tail = 64;
    L.pk_words = PAD_WORDS + nw + tail;
    uint32_t* pk = static_cast<uint32_t*>(L.packed.ensure(L.pk_words * 4));
    uint16_t* vd = static_cast<uint16_t*>(L.valid.ensure(L.pk_words * 2));
    // only the pads are not written by pack_kernel
    HGA_HIP(hipMemsetAsync(pk, 0, PAD_WORDS * 4, c->stream));
    HGA_HIP(hipMemsetAsync(vd, 0, PAD_WORDS * 2, c->stream));
    HGA_HIP(hipMemsetAsync(pk + PAD_WORDS + nw, 0, tail * 4, c->stream));
    HGA_HIP(hipMemsetAsync(vd + PAD_WORDS + nw, 0, tail * 2, c->stream));
    const uint64_t sbw = SB_PAD + (nb + 31) / 32 + tail;
    unsigned int* sb = static_cast<unsigned int*>(L.starts.ensure(sbw * 4));
    HGA_HIP(hipMemsetAsync(sb, 0, sbw * 4, c->stream));
    const uint64_t nwr = (nb + 31) / 32;
    uint32_t* wr = static_cast<uint32_t*>(L.word_read.ensure(std::max<uint64_t>(nwr, 1) * 4));
    c->launch("lk_pack", [&] {
        if (nw && !skip_codes)
            hipLaunchKernelGGL(pack_kernel<true>, dim3(blocks_for(nw, 256)), dim3(256), 0, c->stream,
                               L.bases.as<uint8_t>(), nb, pk, vd, nw);
        if (n)
            hipLaunchKernelGGL(lk_read_map, dim3(blocks_for(n, 4)), dim3(256), 0, c->stream, L.offsets.as<uint64_t>(),
                               n, nb, sb, wr);
    });
    c->check_launch("lk_pack");
    L.packed_ok = !skip_codes;
}

void lookup_run(hga_ctx* c) {
    auto& L = c->lookup;
    if (L.gathered) {   // back to this rank's own reads (hga_lookup_gather replaced the results)
        L.n_reads = L.loc_n_reads;
        L.first_read_id = L.loc_first_read_id;
        L.gathered = false;
    }
    HGA_REQUIRE(L.loaded, HGA_ERR_STATE, "hga_lookup_load not called");
    HGA_REQUIRE(L.have_reads, HGA_ERR_STATE, "hga_lookup_set_reads not called");
    c->conn.ready = false;
    lookup_pack(c, HGA_LK_ASCII != 0);
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
    uint32_t* wkid = static_cast<uint32_t*>(L.win_kid.ensure(std::max<uint64_t>(n_threads, 1) * LK_P * 4));
    auto* tile = static_cast<unsigned long long*>(L.tile_cnt.ensure((n_tiles + 1) * 8));
    const uint32_t* pk = L.packed.as<uint32_t>();
    const uint16_t* vd = L.valid.as<uint16_t>();
    const unsigned int* sb = L.starts.as<unsigned int>();
    const uint64_t* offs = L.offsets.as<uint64_t>();
    LkTab tab{L.tab_key.p, L.filter.as<uint32_t>(), L.slots, L.fwords - 1, L.idb,
              HGA_LK_ASCII ? L.bases.as<uint8_t>() : nullptr};
    uint64_t H = 0;
    if (n_tiles) {
        c->launch("lk_count", [&] {
#define HGA_LK_SCAN2(KMV, KK, PKV)                                                                           \
    hipLaunchKernelGGL((lk_scan<false, KMV, KK, PKV>), dim3((unsigned)n_tiles), dim3(LK_T), 0, c->stream, pk, vd, \
                       sb, nb, offs, n, k, L.word_read.as<uint32_t>(), tab, hm, wkid, tile, (uint32_t*)nullptr,  \
                       (uint32_t*)nullptr, (uint32_t*)nullptr)
#define HGA_LK_SCAN(KMV, KK)                       \
    do {                                           \
        if (L.idb) HGA_LK_SCAN2(KMV, KK, true);    \
        else HGA_LK_SCAN2(KMV, KK, false);         \
    } while (0)
            if (L.km == LK_KM && k == 19) HGA_LK_SCAN(LK_KM, 19);   // compile-time k for the usual SDK k
            else if (L.km == LK_KM && k == 21) HGA_LK_SCAN(LK_KM, 21);
            else if (L.km == LK_KM) HGA_LK_SCAN(LK_KM, 0);
            else if (L.km == 6) HGA_LK_SCAN(6, 17);   // k = 17
            else if (L.km == 5) HGA_LK_SCAN(5, 16);
            else if (L.km == 4) HGA_LK_SCAN(4, 15);
            else HGA_LK_SCAN(0, 0);
#undef HGA_LK_SCAN
#undef HGA_LK_SCAN2
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
    const int kbits = bits_for(std::max<uint32_t>(L.n_sdk, 1));
    uint64_t* sk = static_cast<uint64_t*>(L.s_key.ensure(std::max<uint64_t>(H, 1) * 8));
    uint32_t* sv = static_cast<uint32_t*>(L.s_val.ensure(std::max<uint64_t>(H, 1) * 4));
    if (H) {
        c->launch("lk_emit", [&] {
            hipLaunchKernelGGL((lk_scan<true, 0>), dim3((unsigned)n_tiles), dim3(LK_T), 0, c->stream, pk, vd, sb, nb,
                               offs, n, k, L.word_read.as<uint32_t>(), tab, hm, wkid, tile, hr, hk, hp, sk, sv,
                               kbits);
        });
        c->check_launch("lk_emit");
    }
    // kmer_component_index (ReadClusteringEngine.cpp:262-267, 282-284), from the read-ordered hits
    bool kjoin = false;
    uint64_t* kptr = static_cast<uint64_t*>(L.kci_ptr.ensure(((uint64_t)L.n_sdk + 1) * 8));
    uint32_t* kv = static_cast<uint32_t*>(L.kci_val.ensure(std::max<uint64_t>(H, 1) * 4));
    ++L.kci_epoch;
    // kmer_component_index: the bucketed sort (lk_msd_* + lk_kci_*) when every bucket fits a workgroup's
    // LDS, else (or with HGA_KCI_RADIX) a stable radix sort of the read-ordered hits by KmerID + lk_ptr
    // D top KmerID bits pick the bucket: at least kbits - KC_SMAX (sub-buckets = KmerIDs fit the LDS
    // counters) and enough buckets for ~2.5 K hits each (KC_CAP = 4 K a bucket), at most KC_DMAX
    int kD = kbits > KC_SMAX ? kbits - KC_SMAX : 0;
    while (kD < KC_DMAX && kD < kbits && (H >> kD) > 2500) ++kD;
    const int kS = kbits - kD;
    const bool bucketed = H && kD <= KC_DMAX && !std::getenv("HGA_KCI_RADIX");
    auto radix_kci = [&] {
        uint32_t* kk = static_cast<uint32_t*>(L.kci_key.ensure(H * 4));
        radix_sort_u32_from(c, hk, hr, kk, kv, H, kbits, L.scratch2);
        c->launch("lk_post", [&] {
            hipLaunchKernelGGL(lk_ptr, dim3(blocks_for(H + 1, 256)), dim3(256), 0, c->stream, (const uint32_t*)kk, H,
                               (uint64_t)L.n_sdk, kptr);
        });
        c->check_launch("lk_ptr");
    };
    unsigned long long* kflag = nullptr;
    if (bucketed) {
        // pass A on the top D1 bucket bits, pass B (if D2 > 0) on the next D2 inside each A digit
        const int D1 = kD > KC_PASS_BITS ? kD - KC_PASS_BITS : kD, D2 = kD - D1;
        const uint32_t ndA = 1u << D1, ndB = 1u << D2, nbk = 1u << kD;
        const uint32_t tilesA = (uint32_t)((H + KC_TILE - 1) / KC_TILE), tilesB = D2 ? tilesA + ndA : 0u;
        const size_t rowsA_b = (size_t)tilesA * ndA * 4, rowsB_b = (size_t)tilesB * ndB * 4;
        const size_t small_b = 64 + rowsA_b + rowsB_b + (128 + 128 + 256) * 4 + 2 * (size_t)nbk * 4;
        const size_t pairs_off = (small_b + 255) & ~(size_t)255;
        char* kt = static_cast<char*>(L.kci_tmp.ensure(pairs_off + 2 * H * 8));
        kflag = reinterpret_cast<unsigned long long*>(kt);
        uint32_t* rowsA = reinterpret_cast<uint32_t*>(kt + 64);
        uint32_t* rowsB = reinterpret_cast<uint32_t*>(kt + 64 + rowsA_b);
        uint32_t* totA = reinterpret_cast<uint32_t*>(kt + 64 + rowsA_b + rowsB_b);
        uint32_t* baseA = totA + 128;
        uint32_t* tstart = baseA + 128;
        uint32_t* tot = tstart + 256;
        uint32_t* bbase = tot + nbk;
        uint64_t* pairsA = reinterpret_cast<uint64_t*>(kt + pairs_off);
        uint64_t* pairsB = pairsA + H;
        const int shA = kS + D2, shB = kS;
        // on the ctx's side stream, forked here: it overlaps the per-read sort and first-occurrence
        // kernels below (independent: they read sk / sv, this reads hk / hr); joined before the read-back
        hipStream_t ks = c->side_stream();
        HGA_HIP(hipEventRecord(c->ev_fork, c->stream));
        HGA_HIP(hipStreamWaitEvent(ks, c->ev_fork, 0));
        HGA_HIP(hipMemsetAsync(kflag, 0, 64, ks));
        c->launch_on("lk_kci", ks, [&] {
            hipLaunchKernelGGL(lk_msd_hist<false>, dim3(tilesA), dim3(KC_T), 0, ks, hk, (const uint64_t*)nullptr, H,
                               shA, ndA, (const uint32_t*)nullptr, (const uint32_t*)nullptr, (const uint32_t*)nullptr,
                               tilesA, rowsA);
            hipLaunchKernelGGL(lk_msd_bscan, dim3(blocks_for(ndA, 4)), dim3(256), 0, ks, rowsA, tilesA, ndA, 1u,
                               (const uint32_t*)nullptr, totA);
            hipLaunchKernelGGL(lk_kci_scan, dim3(1), dim3(1024), 0, ks, (const uint32_t*)totA, ndA, baseA, kflag + 1);
            hipLaunchKernelGGL(lk_msd_scatter<false>, dim3(tilesA), dim3(KC_T), 0, ks, hk, hr,
                               (const uint64_t*)nullptr, H, shA, ndA, (const uint32_t*)nullptr, (const uint32_t*)nullptr,
                               (const uint32_t*)nullptr, tilesA, (const uint32_t*)rowsA, (const uint32_t*)baseA,
                               D2 ? pairsA : pairsB);
            if (D2) {
                hipLaunchKernelGGL(lk_msd_tiles, dim3(1), dim3(64), 0, ks, (const uint32_t*)totA, ndA, tstart);
                hipLaunchKernelGGL(lk_msd_hist<true>, dim3(tilesB), dim3(KC_T), 0, ks, (const uint32_t*)nullptr,
                                   (const uint64_t*)pairsA, H, shB, ndB, (const uint32_t*)tstart, (const uint32_t*)baseA,
                                   (const uint32_t*)totA, tilesB, rowsB);
                hipLaunchKernelGGL(lk_msd_bscan, dim3(blocks_for(nbk, 4)), dim3(256), 0, ks, rowsB, tilesB, ndB,
                                   ndA, (const uint32_t*)tstart, tot);
                hipLaunchKernelGGL(lk_kci_scan, dim3(1), dim3(1024), 0, ks, (const uint32_t*)tot, nbk, bbase,
                                   kflag + 1);
                hipLaunchKernelGGL(lk_msd_scatter<true>, dim3(tilesB), dim3(KC_T), 0, ks, (const uint32_t*)nullptr,
                                   (const uint32_t*)nullptr, (const uint64_t*)pairsA, H, shB, ndB, (const uint32_t*)tstart,
                                   (const uint32_t*)baseA, (const uint32_t*)totA, tilesB, (const uint32_t*)rowsB,
                                   (const uint32_t*)bbase, pairsB);
            }
            hipLaunchKernelGGL(lk_kci_bsort, dim3(nbk), dim3(KC_CT), 0, ks, (const uint64_t*)pairsB,
                               (const uint32_t*)(D2 ? tot : totA), (const uint32_t*)(D2 ? bbase : baseA), kS,
                               (uint64_t)L.n_sdk, H, kptr, kv, kflag);
        });
        c->check_launch("lk_kci");
        HGA_HIP(hipEventRecord(c->ev_join, ks));
        kjoin = true;
    } else if (H) {
        radix_kci();
    }
    // hit_ptr over reads
    auto* ctr = static_cast<unsigned long long*>(L.first_flag.ensure(64));
    HGA_HIP(hipMemsetAsync(ctr, 0, 32, c->stream));
    uint64_t* hptr = static_cast<uint64_t*>(L.hit_ptr.ensure((n + 1) * 8));
    // reads listed for the per-read sort tiers: mid (> 64 * WIPT hits) then big (> 2048), n entries each
    uint32_t* lists = static_cast<uint32_t*>(L.big_list.ensure(2 * std::max<uint64_t>(n, 1) * 4 + 64));
    c->launch("lk_post", [&] {
        hipLaunchKernelGGL(lk_ptr, dim3(blocks_for(H + 1, 256)), dim3(256), 0, c->stream, hr, H, n, hptr);
        if (n)
            hipLaunchKernelGGL(lk_seg_stats, dim3(blocks_for(n, 1024)), dim3(1024), 0, c->stream, hptr, n, ctr, lists,
                               lists + n, (uint32_t)(64 * WIPT), 2048u);
    });
    c->check_launch("lk_ptr");
    const int rbits = bits_for(std::max<uint64_t>(n, 1));
    const uint64_t kmask = (1ull << kbits) - 1;
    uint64_t U = 0;
    if (H) {
        // per-read (read, KmerID) sort of the emitted (read << kbits | KmerID, position) pairs
        unsigned long long mx[4];   // non-empty reads, most hits, the two tier lists' lengths: one sync
        HGA_HIP(hipMemcpyAsync(mx, ctr, 32, hipMemcpyDeviceToHost, c->stream));
        c->sync();
        if (!segment_sort(c, hptr, n, mx[1], kbits, sk, sv, L.big_list, ctr + 4, "lk_sort", lists, mx + 2))
            radix_sort_u64(c, sk, sv, H, kbits + rbits, L.scratch2);   // a read with > 16384 hits
        uint32_t* skid = static_cast<uint32_t*>(L.s_val2.ensure(H * 4));
        uint64_t* fptr0 = static_cast<uint64_t*>(L.first_ptr.ensure((n + 1) * 8));
        c->launch("lk_post", [&] {
            hipLaunchKernelGGL(lk_first_count, dim3(blocks_for(n, 4)), dim3(256), 0, c->stream, hptr, n, sk, kmask,
                               skid, fptr0);
        });
        c->check_launch("lk_first_count");
        HGA_HIP(hipMemsetAsync(fptr0 + n, 0, 8, c->stream));
        exclusive_scan_u64(c, fptr0, n + 1, L.scratch3);
        // U <= H first occurrences: the arrays are sized by H, U itself comes with the final counters
        uint32_t* fk = static_cast<uint32_t*>(L.first_kid.ensure(H * 4));
        uint32_t* fp = static_cast<uint32_t*>(L.first_pos.ensure(H * 4));
        uint32_t* fr = static_cast<uint32_t*>(L.first_read.ensure(H * 4));
        c->launch("lk_post", [&] {
            hipLaunchKernelGGL(lk_first_write, dim3(blocks_for(n, 4)), dim3(256), 0, c->stream, hptr, n, sk, sv,
                               fptr0, kmask, fk, fp, fr);
        });
        c->check_launch("lk_first_write");
    }
    uint64_t* fptr = static_cast<uint64_t*>(L.first_ptr.ensure((n + 1) * 8));
    c->launch("lk_post", [&] {
        if (!H)   // with hits the first-occurrence scan above already left the CSR pointers in fptr
            hipLaunchKernelGGL(lk_ptr, dim3(blocks_for(U + 1, 256)), dim3(256), 0, c->stream,
                               (const uint32_t*)nullptr, U, n, fptr);
        if (!H)
            hipLaunchKernelGGL(lk_ptr, dim3(blocks_for(H + 1, 256)), dim3(256), 0, c->stream, (const uint32_t*)nullptr,
                               H, (uint64_t)L.n_sdk, kptr);
    });
    c->check_launch("lk_ptr");
    if (kjoin) HGA_HIP(hipStreamWaitEvent(c->stream, c->ev_join, 0));
    unsigned long long hc[4], kf = 0;
    HGA_HIP(hipMemcpyAsync(hc, ctr, 32, hipMemcpyDeviceToHost, c->stream));
    if (H) HGA_HIP(hipMemcpyAsync(&U, fptr + n, 8, hipMemcpyDeviceToHost, c->stream));
    if (kflag) HGA_HIP(hipMemcpyAsync(&kf, kflag, 8, hipMemcpyDeviceToHost, c->stream));
    c->sync();
    if (kf) {   // a bucket past the LDS: the radix path (reads hk / hr, still intact)
        radix_kci();
        c->sync();
    }
    L.firsts = U;
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
