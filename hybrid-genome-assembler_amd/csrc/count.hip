// count.hip — MI355X k-mer counting: the replacement for `jellyfish count -C --bc`
// + `dump` + `sort` (src/occurrences/run_jellyfish.sh:3-6) and for the two string
// k-way merge passes of JellyfishOccurrenceReader (JellyfishOccurrenceReader.cpp:63-135).
//
// Pipeline (integer / byte work, no MFMA; DESIGN.md §4 has each kernel's bound):
//   B1 kc_bin1   per tile of 8K window ends: the tile's ASCII bases packed once into LDS
//                (2-bit codes + base-valid bits, 16 bases per thread, the next tile's bytes
//                in flight meanwhile), closed-form canonical k-mer of every valid window
//                from packed frames, bijective 2k-bit mix; the top fb1 (<= 6) bits
//                pick a level-1 region, ranked through LDS so every region's run leaves as
//                one coalesced segment (>= 512 B); space reserved with one returning atomic
//                per (tile, region); per-fine-bucket histogram kept in LDS, flushed once.
//   L  kc_layout one workgroup: fine-bucket bases (bucket-major, file-minor) and the
//                chunk table of the level-1 regions.
//   B2 kc_rebin  per 8K-element chunk of a level-1 region: the next fb2 bits pick the fine
//                bucket (again <= 64-way, coalesced); writes the remainder (u32 when <= 31 bits).
//   B3 kc_split3 (inputs far above C2 only) per fine bucket: the next fb3 bits pick one of
//                2^fb3 sub-buckets, staged in LDS and written in runs; the count kernels then
//                run on the sub-buckets.
//   C  kc_count  one workgroup per fine bucket: LDS open-addressing table keyed by the
//                remainder with one u32 counter per file; adaptive sub-range splitting
//                if a bucket holds more distinct k-mers than the table; per-file drop
//                of counts < min (jellyfish --bc); emit merged rows (key, counts[F]).
//   H  kc_spec_hist   specificity x total histogram (get_specificity, :88-108).
//   X  kc_select      rows with lower <= total <= upper, + the export sort ascending
//                     (export_kmers, :110-135; numeric order == LC_ALL=C order).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <type_traits>

#include "hga_internal.hpp"
#include "kmer_dev.hpp"

#ifndef HGA_B1_NOFB
#define HGA_B1_NOFB 0   // timing comparison: kc_bin1 without the compile-time fine-bucket bits
#endif
#ifndef HGA_B1_BRANCHFREE
#define HGA_B1_BRANCHFREE 0   // 1: kc_bin1 ranks every window (invalid ones into per-lane dummy counters)
#endif

namespace hga {
namespace {

constexpr int NT_B = 512;     // level-1 binning workgroup
constexpr int P_B = 16;       // window ends per thread
constexpr int TP_B = NT_B * P_B;       // 8192 window ends per tile
constexpr uint64_t ST_ALIGN = TP_B;    // super-tiles are whole tiles
#ifndef HGA_MAX_FB
#define HGA_MAX_FB 12
#endif
#ifndef HGA_NT_C
#define HGA_NT_C 1024
#endif
#ifndef HGA_LDS_TAB_KB
#define HGA_LDS_TAB_KB 128
#endif
#ifndef HGA_PB_P
#define HGA_PB_P 65536
#endif
constexpr int MAX_FB = HGA_MAX_FB;
constexpr int MAX_NB = 1 << MAX_FB;
#ifndef HGA_MAX_FB1
#define HGA_MAX_FB1 6
#endif
constexpr int MAX_FB1 = HGA_MAX_FB1;    // level-1 fan-out <= 64
constexpr int NB1_MAX = 1 << MAX_FB1;
constexpr int NB2_MAX = 1 << (MAX_FB - MAX_FB1 > 6 ? MAX_FB - MAX_FB1 : 6);   // level-2 fan-out
static_assert(NB1_MAX <= 64 && NB2_MAX <= 128, "bin1 scans <= 64 regions with one wave, rebin <= 128 digits with two");
#ifndef HGA_NT_R
#define HGA_NT_R 256
#endif
#ifndef HGA_NT_R64
#define HGA_NT_R64 512
#endif
constexpr int CH_R = 8192;       // elements per re-bin chunk (one level-1 block)
// re-bin workgroup: 256 threads for u32 remainders (4 workgroups per CU on 33 KB of stage:
// 0.456 vs 0.472 ms at C2 with 512), 512 for u64 ones (two per CU on 66 KB)
template <class E>
constexpr int rebin_nt() { return sizeof(E) == 4 ? HGA_NT_R : HGA_NT_R64; }
constexpr int NT_R_MAX = HGA_NT_R > HGA_NT_R64 ? HGA_NT_R : HGA_NT_R64;
static_assert(HGA_NT_R >= 128 && HGA_NT_R64 >= 128 && CH_R % HGA_NT_R == 0 && CH_R % HGA_NT_R64 == 0,
              "rebin scans 128 digits with two waves");
constexpr int NT_C = HGA_NT_C;   // threads of the per-bucket count workgroup
#ifndef HGA_PF_C
#define HGA_PF_C 8
#endif
constexpr int PF_C = HGA_PF_C;   // binned elements each count thread has in flight
constexpr uint32_t LDS_TAB = HGA_LDS_TAB_KB * 1024;

struct KP {
    int k, sh;
    uint64_t mask;
    Mix mix;
    uint32_t fb, rbits, nb;      // fine buckets: top fb bits; remainder = low rbits bits
    uint64_t rmask;
    uint32_t fb1, r1bits, nb1;   // level-1 regions: top fb1 bits; element = low r1bits bits
    uint64_t r1mask;
    uint32_t fb2, nb2;           // level-2 digit: the next fb2 bits
};

__device__ __forceinline__ uint32_t bucket_of(uint64_t h, const KP& kp) {
    return kp.fb ? (uint32_t)(h >> kp.rbits) : 0u;
}
__device__ __forceinline__ uint32_t region_of(uint64_t h, const KP& kp) {
    return kp.fb1 ? (uint32_t)(h >> kp.r1bits) : 0u;
}

// Canonical code of the window ending at p0+j, from a loaded frame.
template <int P>
__device__ __forceinline__ uint64_t frame_canon(const Frame<P>& f, int j, uint64_t mask) {
    constexpr int NW = Frame<P>::NW;
    const uint64_t fwd = field64<NW>(f.x, 2 * (16 * NW - 33 - j)) & mask;
    const uint64_t rc = field64<NW>(f.r, 2 * j) & mask;
    return fwd < rc ? fwd : rc;
}

// ---------------------------------------------------------------- pass B1
// LDS-only barrier: waits for this wave's LDS traffic, not for its global loads, so a
// prefetch issued before it stays in flight (a __syncthreads() would drain vmcnt too).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// (the builtin returns int: each half is widened as uint32_t, never sign-extended)
__device__ __forceinline__ uint64_t readfirstlane64(uint64_t v) {
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    return ((uint64_t)hi << 32) | lo;
}

// dst[i] through a wave-uniform base and a 32-bit lane byte offset (one global_store with an SGPR
// base, no 64-bit address arithmetic per element); i * sizeof(T) < 2^32.
template <class T>
__device__ __forceinline__ void store_at(T* dst, uint32_t i, T v) {
    *reinterpret_cast<T*>(reinterpret_cast<char*>(dst) + (uint32_t)(i * (uint32_t)sizeof(T))) = v;
}

#ifndef HGA_B1_BUFST
#define HGA_B1_BUFST 1   // kc_bin1's flush through buffer stores (0: global stores, 64-bit lane addresses)
#endif
// dst[0, n) = src[0, n) by one wave (dst wave-uniform): buffer stores off a descriptor built from the
// run's uniform base, so each store takes a 32-bit lane offset instead of 64-bit address arithmetic
// (the descriptor's record count is the run's length: a lane past it stores nothing)
template <class T>
__device__ __forceinline__ void store_run(T* dst, uint32_t n, const T* src, uint32_t lane) {
    if (!HGA_B1_BUFST) {
        for (uint32_t jj = lane; jj < n; jj += 64) store_at(dst, jj, src[jj]);
        return;
    }
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)(n * (uint32_t)sizeof(T)), 0x00020000);
    // four elements per lane and round, read and stored unpredicated: src has 256 readable elements past
    // any run (the caller's padding) and the descriptor drops the stores past n
    for (uint32_t j0 = 0; j0 < n; j0 += 256) {
        T v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = src[j0 + 64u * (uint32_t)u + lane];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t jj = j0 + 64u * (uint32_t)u + lane;
            if constexpr (sizeof(T) == 4) {
                __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v[u], rs, (int)(jj * 4u), 0, 0);
            } else {
                typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
                __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{(uint32_t)v[u], (uint32_t)((uint64_t)v[u] >> 32)}, rs,
                                                      (int)(jj * 8u), 0, 0);
            }
        }
    }
}

// Level-1 blocks: every workgroup takes BLK-element blocks per region from one pool with a
// single atomic (and a new one only when a block fills), so a tile's region runs are
// written without any global atomic.  block table entry: start, used, file<<8 | region.
struct Blk {
    unsigned long long start;
    uint32_t used;
    uint32_t tag;
};
constexpr uint32_t BLK = TP_B;   // >= a tile, so a tile's run spans at most two blocks
static_assert(BLK < 65536, "kc_bin1 packs a block count and a run offset in 16 bits each");

// gstat: [0] row cursor, [1] max split, [2] error bits (1 unsplittable, 2 row capacity,
// 4 level-1 pool exhausted), [3] blocks used, [4] instances.
// Block e always starts at e * BLK in the pool.  Workgroup w's first block of region r is
// entry w * nb1 + r (no atomic); spill blocks are numbered from W * nb1 up (gstat[3]).
// Block e (reserved from gstat[3] by the caller) for the run tagged `tag`.
__device__ __forceinline__ uint32_t claim_block(unsigned long long e, unsigned long long* gstat, Blk* table,
                                                uint64_t table_cap, uint32_t tag, unsigned long long& start) {
    if (e >= table_cap) {
        atomicOr(&gstat[2], 4ull);
        start = table_cap * (unsigned long long)BLK;   // writes into this block are dropped
        return 0xFFFFFFFFu;
    }
    start = e * (unsigned long long)BLK;
    table[e].start = start;
    table[e].used = 0;
    table[e].tag = tag;
    return (uint32_t)e;
}

// One level-1 binning launch covers every file: workgroup w belongs to file f when
// files[f].w0 <= w < files[f+1].w0 (file-major, so per-file runs stay contiguous).
struct BinFile {
    uint64_t n;      // bases
    uint32_t w0, pad;
    const uint8_t* seq;   // the file's ASCII bases
};

#ifndef HGA_B1_PER_CU
#define HGA_B1_PER_CU 2   // bin1 super-tiles per CU
#endif
#ifndef HGA_B1_WAVES
#define HGA_B1_WAVES 1
#endif
// K > 0: k known at compile time (the usual k of a run): the window mask, the run-of-k validity
// doubling and the mix's mask and shift fold to constants — with a runtime k those uniform values
// spill out of the SGPR file (v_readlane per use) and runs_of is a chain of uniform selects.
// FB > 0 (with K): the fine-bucket bits known at compile time too (C2-sized inputs: 12), so region and
// bucket are constant shifts of the mixed key (no 64-bit shift by a uniform register per window).
template <class E1, int K = 0, int FB = 0>
__global__ void __launch_bounds__(NT_B, HGA_B1_WAVES) kc_bin1(const BinFile* __restrict__ files, uint32_t F,
                                                uint64_t st_pos, KP kp,
                                                Blk* __restrict__ table, uint64_t table_cap,
                                                uint64_t pool_cap, E1* __restrict__ out1,
                                                uint32_t* __restrict__ wcnt, uint32_t* __restrict__ nblk,
                                                unsigned long long* __restrict__ gstat) {
    __shared__ uint32_t cnt1[NB1_MAX + (HGA_B1_BRANCHFREE ? 64 : 0)];
    __shared__ uint32_t off1[NB1_MAX + 1];
    __shared__ uint32_t offb[NB1_MAX];               // the same run offsets in bytes of the stage
    __shared__ unsigned long long bstart[NB1_MAX];   // current block of each region
    __shared__ uint32_t bfill[NB1_MAX];              // elements already in it
    __shared__ uint32_t bent[NB1_MAX];               // its table entry
    __shared__ uint32_t nchain[NB1_MAX];             // blocks this workgroup used per region
    __shared__ unsigned long long base_a[NB1_MAX], base_b[NB1_MAX];
    __shared__ uint2 fl_n[NB1_MAX];                  // flush: elements into the current / the fresh block
    __shared__ uint32_t fhist[MAX_NB + (HGA_B1_BRANCHFREE ? 64 : 0)];
    // + one dummy slot per lane for invalid windows, + 256 readable past any run (store_run's rounds)
    __shared__ E1 stage[TP_B + 64 + 256];
    __shared__ uint32_t ws[NT_B / 64 + 1];
    // packed words [t0/16 - 2, t0/16 + 512) of this tile and the next (code | valid << 32)
    __shared__ uint64_t lpw[2][TP_B / 16 + 2];
    const int tid = threadIdx.x;
    const uint32_t nb1 = kp.nb1, nb = kp.nb;
    const uint32_t w = blockIdx.x;
    uint32_t file = 0;
    while (file + 1 < F && files[file + 1].w0 <= w) ++file;
    const uint64_t n = files[file].n;
    const uint32_t tag0 = w << 8;
    for (uint32_t b = tid; b < nb; b += NT_B) fhist[b] = 0;
    if (tid < (int)nb1) {
        cnt1[tid] = 0;
        const unsigned long long e = (unsigned long long)w * nb1 + tid;
        table[e].start = e * BLK;
        table[e].used = 0;
        table[e].tag = tag0 | tid;
        bent[tid] = (uint32_t)e;
        bstart[tid] = e * BLK;
        bfill[tid] = 0;
        nchain[tid] = 1;
    }
    __syncthreads();
    const uint64_t start = (uint64_t)(w - files[file].w0) * st_pos;
    const uint64_t end = start + st_pos < n ? start + st_pos : n;
    uint32_t inst = 0;
    static_assert(P_B == 16 && Frame<P_B>::NW == 3, "one packed word per thread, frames of three");
    const uint8_t* __restrict__ seq = files[file].seq;
    const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
    // tile t's words are packed into lpw[t & 1] while tile t-1 is binned, so the tile's own
    // barriers publish them; the raw bytes of tile t+1 are in flight meanwhile
    auto pack_into = [&](uint64_t* dst, const uint4 a, const uint4 h) {
        uint32_t cw, vw;
        pack_bytes<false>(a, cw, vw);
        dst[tid + 2] = cw | ((uint64_t)vw << 32);
        if (tid < 2) {
            pack_bytes<false>(h, cw, vw);
            dst[tid] = cw | ((uint64_t)vw << 32);
        }
    };
    auto load_raw = [&](uint64_t t, uint4& a, uint4& h) {
        a = z4;
        h = z4;
        if (t < end) {
            a = load16(seq, (int64_t)(t + 16 * (uint64_t)tid), n);
            if (tid < 2) h = load16(seq, (int64_t)t - 32 + 16 * tid, n);
        }
    };
    uint4 nraw, nhalo;
    load_raw(start, nraw, nhalo);
    pack_into(lpw[0], nraw, nhalo);
    load_raw(start + TP_B, nraw, nhalo);
    lds_barrier();
    uint32_t buf = 0;
    for (uint64_t t0 = start; t0 < end; t0 += TP_B) {
        Frame<P_B> f;
        FrameRaw<P_B> fr;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const uint64_t wv = lpw[buf][tid + i];
            fr.x[i] = (uint32_t)wv;
            fr.v[i] = (uint32_t)(wv >> 32);
        }
        if (t0 + TP_B < end) {
            pack_into(lpw[buf ^ 1], nraw, nhalo);
            load_raw(t0 + 2 * TP_B, nraw, nhalo);
        }
        buf ^= 1;
        const int kk = K ? K : kp.k;
        const uint64_t v64 = build_frame<P_B, false>(fr, kk, f);
        const uint32_t wm = (uint32_t)(runs_of(v64, kk) >> 32);   // bit j: window at p0+j valid
        uint32_t dd[P_B], rk[P_B];
        E1 ee[P_B];
        const uint64_t wmask = K ? (K >= 32 ? ~0ull : ((1ull << (2 * K)) - 1)) : kp.mask;
        Mix mx = kp.mix;
        if (K) {
            mx.mask = wmask;
            mx.s = (uint32_t)(2 * K + 1) / 2;
            mx.c1 = kMixC1;   // make_mix's constant
        }
#pragma unroll
        for (int j = 0; j < P_B; ++j) {
            const uint64_t h = mix_fwd_k<K>(frame_canon<P_B>(f, j, wmask), mx);
            // (k < 32: h < 4^k, so a shift by the full width 2k already gives region / bucket 0)
            constexpr int R1B = 2 * K - (FB < MAX_FB1 ? FB : MAX_FB1), RB = 2 * K - FB;
            const uint32_t r1s = K && FB ? (uint32_t)R1B : kp.r1bits, rbs = K && FB ? (uint32_t)RB : kp.rbits;
            // Byte units: the region counters count sizeof(E1) per element, so a rank is the element's
            // byte offset in its stage run and dd the region's byte offset in the counter / run-offset
            // arrays (the stage needs no index scaling).  An invalid window is staged into this lane's
            // dummy slot TP_B + lane: "region" 0 (whose run offset is 0) with that rank.
            const bool ok = (wm >> j) & 1u;
            const uint32_t reg = K && K < 32 ? (uint32_t)(h >> r1s) : region_of(h, kp);
            dd[j] = ok ? reg * 4u : 0u;
            // (u32 elements of a k with 2k - MAX_FB1 >= 32: r1bits == 32, the truncation is the mask)
            constexpr bool trunc = K && sizeof(E1) == 4 && 2 * K - MAX_FB1 >= 32;
            ee[j] = trunc ? (E1)h : (E1)(h & kp.r1mask);
            rk[j] = ((uint32_t)TP_B + (uint32_t)(tid & 63)) * (uint32_t)sizeof(E1);
            if (HGA_B1_BRANCHFREE) {   // invalid windows count into this lane's dummy counters
                const uint32_t r = atomicAdd(&cnt1[ok ? reg : NB1_MAX + (uint32_t)(tid & 63)], (uint32_t)sizeof(E1));
                atomicAdd(&fhist[ok ? (K && K < 32 ? (uint32_t)(h >> kp.rbits) : bucket_of(h, kp))
                                    : MAX_NB + (uint32_t)(tid & 63)], 1u);
                if (ok) rk[j] = r;
            } else if (ok) {
                rk[j] = atomicAdd(&cnt1[reg], (uint32_t)sizeof(E1));
                atomicAdd(&fhist[K && K < 32 ? (uint32_t)(h >> rbs) : bucket_of(h, kp)], 1u);
            }
        }
        inst += __popc(wm);
        lds_barrier();
        if (tid < 64) {   // one wave: scan the <= 64 region counts, place them in the blocks
            const uint32_t c = tid < (int)nb1 ? cnt1[tid] / (uint32_t)sizeof(E1) : 0u;   // (byte units)
            const uint32_t inc = wave_scan_add_dpp(c);   // wave 0, all lanes active
            const uint32_t room = tid < (int)nb1 ? BLK - bfill[tid] : 0u;
            const bool spill = tid < (int)nb1 && c > room;   // the run spills into a fresh block
            if (tid < (int)nb1) {
                off1[tid] = inc - c;
                offb[tid] = (inc - c) * (uint32_t)sizeof(E1);
                cnt1[tid] = 0;
                base_a[tid] = bstart[tid] + bfill[tid];
                if (!spill) bfill[tid] += c;
            }
            // ONE returning atomic per workgroup and tile for all spilling runs: regions fill in
            // lockstep, so at a C4 shard every lane of every workgroup spills in the same tiles (one
            // atomic per lane queued 32 K same-address atomics, ~0.37 ms at ~88/us, per round)
            const uint64_t sm = __ballot(spill);
            if (sm) {
                const int l0 = __builtin_ctzll(sm);
                unsigned long long e0 = 0;
                if (tid == l0) e0 = atomicAdd(&gstat[3], (unsigned long long)__popcll(sm));
                e0 = __shfl(e0, l0, 64);
                if (spill) {
                    if (bent[tid] != 0xFFFFFFFFu) table[bent[tid]].used = BLK;
                    unsigned long long st;
                    bent[tid] = claim_block(e0 + (unsigned long long)__popcll(sm & ((1ull << tid) - 1ull)), gstat,
                                            table, table_cap, tag0 | tid, st);
                    ++nchain[tid];
                    bstart[tid] = st;
                    base_b[tid] = st;
                    bfill[tid] = c - room;
                }
            }
            if (tid == 63) off1[nb1] = inc;
            if (tid < (int)nb1) {   // the flush's two pieces per region, clipped to the pool here once
                const uint32_t na = spill ? room : c, nb = c - na;
                const uint64_t ba = base_a[tid], bb = spill ? base_b[tid] : 0ull;
                // y: the fresh block's count | its first element's run offset << 16 (both <= BLK < 2^16)
                fl_n[tid] = make_uint2(ba < pool_cap ? (uint32_t)min<uint64_t>(pool_cap - ba, na) : 0u,
                                       (nb && bb < pool_cap ? (uint32_t)min<uint64_t>(pool_cap - bb, nb) : 0u) | na << 16);
            }
        }
        lds_barrier();
        {   // all 16 run offsets read first (no wait per element), then the writes
            uint32_t o1[P_B];
#pragma unroll
            for (int j = 0; j < P_B; ++j) o1[j] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(offb) + dd[j]);
#pragma unroll
            for (int j = 0; j < P_B; ++j)   // (offb[0] == 0)
                *reinterpret_cast<E1*>(reinterpret_cast<char*>(stage) + o1[j] + rk[j]) = ee[j];
        }
        lds_barrier();
        // flush: one wave per region run (region-uniform bases, lanes on consecutive elements)
        // (run values made wave-uniform: scalar base addresses, 32-bit lane offsets, no per-element
        // 64-bit select / bound check)
        const uint32_t lane = (uint32_t)(tid & 63);
        // (a piece past the pool — table exhausted, error bit set — was clipped to nothing by wave 0)
        for (uint32_t d = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6); d < nb1; d += NT_B / 64) {
            const uint32_t o = __builtin_amdgcn_readfirstlane(off1[d]);
            const uint2 n2 = fl_n[d];
            const uint32_t na = __builtin_amdgcn_readfirstlane(n2.x), y = __builtin_amdgcn_readfirstlane(n2.y);
            if (na) store_run(out1 + readfirstlane64(base_a[d]), na, stage + o, lane);
            if (y & 0xFFFFu) store_run(out1 + readfirstlane64(base_b[d]), y & 0xFFFFu, stage + o + (y >> 16), lane);
        }
        lds_barrier();
    }
    __syncthreads();
    if (tid < (int)nb1) {
        if (bent[tid] != 0xFFFFFFFFu) table[bent[tid]].used = bfill[tid];
        nblk[(uint64_t)w * nb1 + tid] = nchain[tid];
    }
    for (uint32_t b = tid; b < nb; b += NT_B) wcnt[(uint64_t)w * nb + b] = fhist[b];
    uint32_t tot;
    (void)block_excl_scan<NT_B>(inst, ws, &tot);
    if (tid == 0 && tot) atomicAdd(&gstat[4], (unsigned long long)tot);
}

// Pipeline counters: gstat[3] = the first spill block, the rest 0.
__global__ void kc_init_stat(unsigned long long* __restrict__ gstat, uint64_t n_first) {
    if (threadIdx.x < 8) gstat[threadIdx.x] = threadIdx.x == 3 ? (unsigned long long)n_first : 0ull;
}
// ---------------------------------------------------------------- layout
// off[b * W + w] = wcnt[w * nb + b] (64 x 64 LDS tiles), off[nb * W] = 0.  One exclusive scan
// of off then gives every (fine bucket, workgroup) its first output slot: buckets in order,
// inside a bucket the workgroups in order (files are workgroup ranges, so file runs are
// contiguous) — the re-bin needs no cursor atomics.
__global__ void __launch_bounds__(256) kc_transpose(const uint32_t* __restrict__ wcnt, uint32_t W, uint32_t nb,
                                                    uint64_t* __restrict__ off) {
    __shared__ uint32_t t[64][65];
    const uint32_t b0 = blockIdx.x * 64, w0 = blockIdx.y * 64;
    const uint32_t tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (uint32_t r = ty; r < 64; r += 4) {
        const uint32_t w = w0 + r, b = b0 + tx;
        t[r][tx] = (w < W && b < nb) ? wcnt[(uint64_t)w * nb + b] : 0u;
    }
    __syncthreads();
    for (uint32_t r = ty; r < 64; r += 4) {
        const uint32_t b = b0 + r, w = w0 + tx;
        if (b < nb && w < W) off[(uint64_t)b * W + w] = t[tx][r];
    }
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) off[(uint64_t)nb * W] = 0;
}

// fs[b*(F+1)+f] = start of file f's run in fine bucket b, fs[b*(F+1)+F] = bucket end.
__global__ void kc_fs(const uint64_t* __restrict__ off, const BinFile* __restrict__ files, uint32_t W,
                      uint32_t nb, uint32_t F, uint64_t* __restrict__ fs) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)nb * (F + 1)) return;
    const uint64_t b = i / (F + 1), f = i % (F + 1);
    fs[i] = f == F ? off[(b + 1) * W] : off[b * W + files[f].w0];
}

// ---------------------------------------------------------------- pass B3 (large inputs)
// Inputs with far more than 2^MAX_FB x 65536 instances (a C4 rank shard: ~800 K per fine bucket)
// would make every count workgroup re-read its bucket once per LDS-sized sub-range.  One more
// level instead: one workgroup per fine bucket b splits each file's run by the top fb3 bits of
// the remainder into S = 2^fb3 sub-buckets and strips those bits, so the count kernels run
// unchanged on nb * S buckets of rbits - fb3 bit remainders
// (((b << fb3 | s) << (rbits - fb3)) | rem == (b << rbits) | v).
// One read of the bucket: sub-bucket sizes of a hashed key are near-uniform, so each gets a slab of
// cap = 1.25x its share + 64 in the bucket's output region [R(b), R(b+1)), R(b) = a + a/4 + b*S*64
// for the bucket's input start a; files are written one after the other into every slab, so fs3
// keeps its (sub-bucket, file) start + sub-bucket end form (sub-buckets need not be adjacent).  A
// slab that would overflow (a key repeated far more often than the rest) makes the workgroup redo
// its bucket exactly: a histogram pass, then the scatter, packed from R(b).
constexpr int NT_3 = 1024;
constexpr int R_3 = 8;   // elements per thread in flight
constexpr uint32_t MAX_SF3 = 4096;
constexpr uint32_t SLACK_3 = 64;   // extra slots per sub-bucket slab
template <class E>
__global__ void __launch_bounds__(NT_3) kc_split3(const E* __restrict__ in, const uint64_t* __restrict__ fs,
                                                  uint32_t F, uint32_t fb3, uint32_t rbits, E* __restrict__ out,
                                                  uint64_t* __restrict__ fs3) {
    constexpr uint32_t BT = (uint32_t)NT_3 * R_3;   // batch: staged in LDS, written in sub-bucket runs
    __shared__ uint32_t h[MAX_SF3];                   // per (sub-bucket, file): counts, then cursors
    __shared__ uint32_t bc[256], bo[256];             // per-batch sub-bucket counts / offsets
    __shared__ E stage[BT];
    __shared__ uint32_t ws[NT_3 / 64 + 1];
    __shared__ uint32_t s_ovf;
    const uint32_t tid = threadIdx.x, b = blockIdx.x, S = 1u << fb3, SF = S * F;
    const uint64_t* f = fs + (uint64_t)b * (F + 1);
    const uint32_t sh = rbits - fb3;
    const E rm = (E)(((E)1 << sh) - 1);
    const uint64_t a0 = f[0], e0 = f[F];
    const uint64_t R0 = a0 + (a0 >> 2) + (uint64_t)b * S * SLACK_3;
    const uint64_t R1 = e0 + (e0 >> 2) + (uint64_t)(b + 1) * S * SLACK_3;
    const uint64_t cap = (R1 - R0) / S;
    // one batch of file ff's run [a, e) from i0: ranked by sub-bucket, staged, written in runs to
    // dst(t) + h[t * hs] + rank; returns nothing, sets s_ovf if a run would pass lim (0: no limit)
    auto load_batch = [&](uint64_t i0, uint64_t e, E (&v)[R_3]) {
#pragma unroll
        for (int q = 0; q < R_3; ++q) {
            const uint64_t i = i0 + (uint64_t)q * NT_3 + tid;
            v[q] = i < e ? in[i] : (E)0;
        }
    };
    // the next batch's elements are loaded before this one is ranked, so they are in flight meanwhile
    auto scatter_batch = [&](uint64_t i0, uint64_t e, uint32_t hs, uint32_t hoff, uint64_t lim, auto dst,
                             E (&nx)[R_3]) {
        E v[R_3];
        uint32_t sb[R_3], rk[R_3];
#pragma unroll
        for (int q = 0; q < R_3; ++q) v[q] = nx[q];
        if (i0 + BT < e) load_batch(i0 + BT, e, nx);
        for (uint32_t j = tid; j < S; j += NT_3) bc[j] = 0;
        lds_barrier();   // LDS only: the next batch's loads stay in flight
#pragma unroll
        for (int q = 0; q < R_3; ++q) {
            sb[q] = (uint32_t)(v[q] >> sh);
            rk[q] = i0 + (uint64_t)q * NT_3 + tid < e ? atomicAdd(&bc[sb[q]], 1u) : 0u;
        }
        lds_barrier();   // LDS only: the next batch's loads stay in flight
        if (tid < 64) {   // batch offsets per sub-bucket (S <= 256): one wave, four per lane
            uint32_t c[4], t4 = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                c[q] = tid * 4 + q < S ? bc[tid * 4 + q] : 0u;
                t4 += c[q];
            }
            uint32_t o = wave_incl_scan(t4, (int)tid) - t4;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (tid * 4 + q < S) bo[tid * 4 + q] = o;
                o += c[q];
            }
        }
        lds_barrier();   // LDS only: the next batch's loads stay in flight
#pragma unroll
        for (int q = 0; q < R_3; ++q)
            if (i0 + (uint64_t)q * NT_3 + tid < e) stage[bo[sb[q]] + rk[q]] = v[q];
        lds_barrier();   // LDS only: the next batch's loads stay in flight
        const uint32_t m = (uint32_t)((e - i0) < (uint64_t)BT ? (e - i0) : BT);
        for (uint32_t j = tid; j < m; j += NT_3) {   // staged order: one run per sub-bucket
            const E x = stage[j];
            const uint32_t t = (uint32_t)(x >> sh);
            const uint64_t pos = (uint64_t)h[t * hs + hoff] + (j - bo[t]);
            if (lim && pos >= lim) {
                s_ovf = 1u;
                continue;
            }
            out[dst(t) + pos] = x & rm;
        }
        lds_barrier();   // LDS only: the next batch's loads stay in flight
        for (uint32_t t = tid; t < S; t += NT_3) h[t * hs + hoff] += bc[t];
        lds_barrier();   // LDS only: the next batch's loads stay in flight
    };
    // 1) optimistic: one read, every sub-bucket in its slab (h[t] = the slab's fill)
    for (uint32_t j = tid; j < S; j += NT_3) h[j] = 0;
    if (tid == 0) s_ovf = 0;
    __syncthreads();
    for (uint32_t ff = 0; ff < F; ++ff) {
        for (uint32_t t = tid; t < S; t += NT_3) fs3[((uint64_t)b * S + t) * (F + 1) + ff] = R0 + t * cap + h[t];
        const uint64_t a = f[ff], e = f[ff + 1];
        E nx[R_3];
        if (a < e) load_batch(a, e, nx);
        for (uint64_t i0 = a; i0 < e; i0 += BT)
            scatter_batch(i0, e, 1u, 0u, cap, [&](uint32_t t) { return R0 + (uint64_t)t * cap; }, nx);
    }
    if (!s_ovf) {
        for (uint32_t t = tid; t < S; t += NT_3) fs3[((uint64_t)b * S + t) * (F + 1) + F] = R0 + t * cap + h[t];
        return;
    }
    // 2) a slab overflowed: exact two-pass layout, packed from R0
    __syncthreads();
    for (uint32_t j = tid; j < SF; j += NT_3) h[j] = 0;
    __syncthreads();
    for (uint32_t ff = 0; ff < F; ++ff) {
        const uint64_t a = f[ff], e = f[ff + 1];
        for (uint64_t i0 = a; i0 < e; i0 += BT) {
#pragma unroll
            for (int q = 0; q < R_3; ++q) {
                const uint64_t i = i0 + (uint64_t)q * NT_3 + tid;
                if (i < e) atomicAdd(&h[(uint32_t)(in[i] >> sh) * F + ff], 1u);
            }
        }
    }
    __syncthreads();
    // exclusive scan in (sub-bucket, file) order: 4 consecutive entries per thread (SF <= 4096)
    uint32_t loc[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t j = tid * 4 + q;
        loc[q] = j < SF ? h[j] : 0u;
        sum += loc[q];
    }
    uint32_t tot;
    uint32_t run = block_excl_scan<NT_3>(sum, ws, &tot);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t j = tid * 4 + q;
        if (j < SF) {
            h[j] = run;
            fs3[((uint64_t)b * S + j / F) * (F + 1) + j % F] = R0 + run;
            run += loc[q];
        }
    }
    __syncthreads();
    for (uint32_t sb = tid; sb < S; sb += NT_3)
        fs3[((uint64_t)b * S + sb) * (F + 1) + F] = sb + 1 < S ? R0 + h[(sb + 1) * F] : R0 + (e0 - a0);
    __syncthreads();
    for (uint32_t ff = 0; ff < F; ++ff) {
        const uint64_t a = f[ff], e = f[ff + 1];
        E nx[R_3];
        if (a < e) load_batch(a, e, nx);
        for (uint64_t i0 = a; i0 < e; i0 += BT)
            scatter_batch(i0, e, F, ff, 0ull, [&](uint32_t) { return R0; }, nx);
    }
}

// ---------------------------------------------------------------- pass B2
// One workgroup per level-1 block: the next fb2 bits pick the fine bucket (<= 64-way,
// ranked through LDS so each bucket's run is one coalesced segment).
#ifndef HGA_NT_REBIN_LD
#define HGA_NT_REBIN_LD 0   // timing variants: nontemporal element loads / stores in kc_rebin
#endif
#ifndef HGA_NT_REBIN_ST
#define HGA_NT_REBIN_ST 0
#endif
#ifndef HGA_SPILL_GRID
#define HGA_SPILL_GRID 1024   // workgroups of the spill-block launch (grid-stride over gstat[3])
#endif
template <class E1, class E>
__device__ __forceinline__ void rebin_block(const uint64_t blk, const E1* __restrict__ in1,
                                            const Blk* __restrict__ table, uint32_t W, const KP& kp,
                                            const uint32_t* __restrict__ nblk, unsigned long long* __restrict__ off,
                                            E* __restrict__ out) {
    constexpr int NT_R = rebin_nt<E>();
    constexpr int IT = CH_R / NT_R;
    static_assert(CH_R >= (int)BLK, "a block must fit one re-bin pass");
    __shared__ uint32_t cnt2[NB2_MAX];
    __shared__ uint32_t off2[NB2_MAX + 1];
    __shared__ unsigned long long base2[NB2_MAX];
    __shared__ uint32_t s_w0;
    __shared__ E stage[CH_R];
    const int tid = threadIdx.x;
    const uint32_t nb2 = kp.nb2;
    const uint64_t n_first = (uint64_t)W * kp.nb1;
    // first blocks: everything is known from the index, so the element, size and offset loads
    // all go out together; spill blocks (rare) look themselves up
    const E1* __restrict__ src = in1 + blk * BLK;
    E1 v[IT];
#pragma unroll
    for (int j = 0; j < IT; ++j)
        v[j] = HGA_NT_REBIN_LD ? __builtin_nontemporal_load(&src[(uint32_t)j * NT_R + tid]) : src[(uint32_t)j * NT_R + tid];
    uint32_t w, d1;
    if (blk < n_first) {
        w = (uint32_t)(blk / kp.nb1);
        d1 = (uint32_t)(blk % kp.nb1);
    } else {
        const uint32_t tag = table[blk].tag;
        w = tag >> 8;
        d1 = tag & 0xFFu;
    }
    const uint32_t used = table[blk].used;
    // a workgroup's only block of a region owns the whole (bucket, workgroup) slot range;
    // chained blocks (spills) share it atomically
    const bool sole = nblk[(uint64_t)w * kp.nb1 + d1] == 1u;
    const uint64_t oidx = ((((uint64_t)d1 << kp.fb2) | (uint64_t)(tid & (NB2_MAX - 1))) * W) + w;
    const unsigned long long pre = (tid < (int)nb2 && sole) ? off[oidx] : 0ull;
    if (tid < (int)nb2) cnt2[tid] = 0;
    __syncthreads();
    uint32_t dd[IT], rk[IT];
    E ee[IT];
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const uint32_t i = (uint32_t)j * NT_R + tid;
        dd[j] = kp.fb2 ? (uint32_t)((uint64_t)v[j] >> kp.rbits) : 0u;
        ee[j] = (E)((uint64_t)v[j] & kp.rmask);
        rk[j] = i < used ? atomicAdd(&cnt2[dd[j]], 1u) : 0u;
    }
    __syncthreads();
    uint32_t c2 = 0, inc2 = 0;
    if (tid < NB2_MAX) {   // two waves scan the <= 128 digit counts
        c2 = tid < (int)nb2 ? cnt2[tid] : 0u;
        inc2 = wave_scan_add_dpp(c2);   // whole waves (NB2_MAX is a multiple of 64)
        if (tid == 63) s_w0 = inc2;
    }
    __syncthreads();
    if (tid < NB2_MAX) {
        if (tid >= 64) inc2 += s_w0;
        if (tid < (int)nb2) {
            off2[tid] = inc2 - c2;
            base2[tid] = sole ? pre : (c2 ? atomicAdd(&off[oidx], (unsigned long long)c2) : 0ull);
        }
        if (tid == NB2_MAX - 1) off2[nb2] = inc2;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const uint32_t i = (uint32_t)j * NT_R + tid;
        if (i < used) stage[off2[dd[j]] + rk[j]] = ee[j];
    }
    __syncthreads();
    // flush: one wave per digit run (digit-uniform base, lanes on consecutive elements)
    for (uint32_t d = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6); d < nb2; d += NT_R / 64) {
        const uint32_t o = off2[d], len = off2[d + 1] - o;
        E* __restrict__ dst = out + base2[d];
        for (uint32_t jj = (uint32_t)(tid & 63); jj < len; jj += 64) {
            if (HGA_NT_REBIN_ST) __builtin_nontemporal_store(stage[o + jj], &dst[jj]);
            else dst[jj] = stage[o + jj];
        }
    }
}

// first = true: one workgroup per first block (block blockIdx.x < W * nb1); first = false: the spill
// blocks [W * nb1, gstat[3]) grid-stride over a small grid (at C2 there are none, and a grid of every
// possible spill block retired ~36 K empty workgroups)
template <class E1, class E>
__global__ void __launch_bounds__(NT_R_MAX) kc_rebin(const E1* __restrict__ in1, const Blk* __restrict__ table,
                                                 const unsigned long long* __restrict__ gstat, uint32_t W,
                                                 KP kp, const uint32_t* __restrict__ nblk,
                                                 unsigned long long* __restrict__ off,
                                                 E* __restrict__ out, bool first) {
    if (first) {
        rebin_block<E1, E>(blockIdx.x, in1, table, W, kp, nblk, off, out);
        return;
    }
    const uint64_t n_first = (uint64_t)W * kp.nb1, used = gstat[3];
    for (uint64_t blk = n_first + blockIdx.x; blk < used; blk += gridDim.x) {
        rebin_block<E1, E>(blk, in1, table, W, kp, nblk, off, out);
        __syncthreads();   // the block's LDS is reused by the next one
    }
}

// ---------------------------------------------------------------- pass C
// LDS table: T slots in T/4 groups of 4 (one ds_read_b128 per probe for u32 keys), keys
// SoA with one u32 counter per file per slot.  A key's home group is its low bits.
#ifndef HGA_GROUP
#define HGA_GROUP 4
#endif
constexpr int GRP = HGA_GROUP;   // slots per probe group (4: one ds_read_b128 of u32 keys)
template <class E>
__device__ __forceinline__ void read_group(const E* keys, uint32_t g, E (&k)[GRP]) {
    if constexpr (sizeof(E) == 4) {
#pragma unroll
        for (int t = 0; t < GRP / 4; ++t) {
            const uint4 v = reinterpret_cast<const uint4*>(keys)[g * (GRP / 4) + t];
            k[4 * t] = v.x; k[4 * t + 1] = v.y; k[4 * t + 2] = v.z; k[4 * t + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int t = 0; t < GRP / 2; ++t) {
            const ulonglong2 a = reinterpret_cast<const ulonglong2*>(keys)[g * (GRP / 2) + t];
            k[2 * t] = a.x; k[2 * t + 1] = a.y;
        }
    }
}

// One probe step for key r at group g: count it if present, claim an empty slot if the group
// has one, else move to the next group.  r becomes EMPTY once settled (or dropped because the
// table is over its load limit, in which case the whole sub-range is redone after a split).
template <class E>
__device__ __forceinline__ bool count_step(E* keys, uint32_t* cf, uint32_t G, uint32_t& s_ovf, E& r,
                                           uint32_t& g) {
    const E EMPTY = ~E(0);
    E kg[GRP];
    read_group(keys, g, kg);
    int w = -1, e0 = -1;
#pragma unroll
    for (int t = GRP - 1; t >= 0; --t) {
        w = kg[t] == r ? t : w;
        e0 = kg[t] == EMPTY ? t : e0;
    }
    if (w >= 0) {
        atomicAdd(&cf[GRP * g + w], 1u);
        r = EMPTY;
    } else if (e0 >= 0) {
        if (__atomic_load_n(&s_ovf, __ATOMIC_RELAXED)) {
            r = EMPTY;
        } else {
            const uint32_t sl = GRP * g + (uint32_t)e0;
            const E old = atomicCAS(&keys[sl], EMPTY, r);
            if (old == EMPTY || old == r) {
                atomicAdd(&cf[sl], 1u);
                r = EMPTY;
                return old == EMPTY;
            }   // else: lost the slot to another key, re-read the group
        }
    } else {
        g = (g + 1) & (G - 1);
    }
    return false;
}

// Occupancy is accounted once per wave and probe iteration (at most 64 new keys), so the
// table can exceed maxload by at most (waves x 64) before s_ovf stops insertions; the host
// keeps maxload + NT_C below T, so a probe always finds an empty slot.
__device__ __forceinline__ void count_occupancy(bool ins, uint32_t& s_occ, uint32_t& s_ovf, uint32_t maxload) {
    const uint64_t bal = __ballot(ins);
    if (bal && (threadIdx.x & 63) == 0) {
        const uint32_t n = (uint32_t)__popcll(bal);
        const uint32_t o = atomicAdd(&s_occ, n);
        if (o + n >= maxload) __atomic_store_n(&s_ovf, 1u, __ATOMIC_RELAXED);
    }
}

__device__ __forceinline__ uint64_t lanemask_lt() {
    return (1ull << (threadIdx.x & 63)) - 1ull;
}

constexpr uint32_t QN_C = 128;   // miss-queue entries per wave
// Exchange emission (hga_count_exchange's hash buckets, exchange.hip count_xb_pack): with a
// communicator attached, count_run(ctx, 1) writes every bucket's rows as packed pieces that carry
// the mix h of the key (h in the low 2k bits, file f's count in bits [2k + f cb, ...), a count past
// 2^cb - 1 split over several adjacent pieces) into `slab` from the bucket's first binned position
// (pieces <= instances), and the bucket's piece count into dir[b]; the sender's gather groups them
// by the next hash bits.  The dense rows are not written then: each bucket reserves its row range
// once (rbase[b]) and kc_xb_dense fills it from the pieces if a local query needs them.  kc_count
// (the buckets kc_count_s leaves to it) emits the same way.
struct XbEmit {
    uint64_t* slab;   // nullptr: off
    uint64_t* dir;
    uint64_t* rbase;
    uint32_t cb, kb, cmax;
};
static_assert(sizeof(XbEmit) <= 64, "CountState::xemit_host holds one XbEmit");

#ifndef HGA_EMIT_STAGE
#define HGA_EMIT_STAGE 1
#endif
constexpr int EMIT_F = 4;        // files handled by the LDS-staged emit
constexpr int EMIT_S = 8;        // slots per thread in it (T == NT_C * EMIT_S)

// gstat: [0] output cursor, [1] max sub-ranges any bucket needed, [2] error bits
// (1 = unsplittable overflow, 2 = output capacity exceeded, 4 = level-1 overflow).
template <class E>
__global__ void __launch_bounds__(NT_C) kc_count(const E* __restrict__ binned,
                                                 const uint64_t* __restrict__ fs, uint32_t F,
                                                 uint32_t T, uint32_t maxload, uint32_t min_count,
                                                 KP kp, uint64_t* __restrict__ out_key,
                                                 uint32_t* __restrict__ out_cnt, uint64_t cap,
                                                 unsigned long long* __restrict__ gstat,
                                                 const uint32_t* __restrict__ blist,
                                                 const XbEmit* __restrict__ xep = nullptr) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_TAB];
    __shared__ uint32_t s_occ, s_ovf, s_sp, s_ranges, s_xw, s_xrows;
    __shared__ uint32_t stk_lo[40], stk_hi[40];
    __shared__ uint32_t ws[NT_C / 64 + 1];
    __shared__ unsigned long long s_base;
    __shared__ E qbuf[NT_C / 64][QN_C];
    E* keys = reinterpret_cast<E*>(smem);
    const uint32_t lane = threadIdx.x & 63;
    E* myq = qbuf[threadIdx.x >> 6];
    uint32_t* cnt = reinterpret_cast<uint32_t*>(smem + (size_t)T * sizeof(E));
    const int tid = threadIdx.x;
    const E EMPTY = ~E(0);
    const uint32_t rbits = kp.rbits;
    const uint32_t SUBB = rbits < 16 ? rbits : 16;
    const uint32_t full_hi = 1u << SUBB;
    const uint32_t mc = min_count ? min_count : 1u;
    const uint32_t G = T / GRP;
    // every bucket (blist null), or the buckets listed by kc_count_s (count in gstat[5])
    const uint32_t n_b = blist ? (uint32_t)gstat[5] : gridDim.x;
    for (uint32_t it = blockIdx.x; it < n_b; it += gridDim.x) {
    const uint32_t b = blist ? blist[it] : it;
    const uint64_t* f = fs + (uint64_t)b * (F + 1);
    __syncthreads();
    if (tid == 0) {
        stk_lo[0] = 0;
        stk_hi[0] = full_hi;
        s_sp = 1;
        s_ranges = 0;
        s_xw = 0;
        s_xrows = 0;
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
            constexpr uint64_t STEP = (uint64_t)NT_C * PF_C;
            if (a == e) continue;
            // full batches load from a uniform base (scalar address + lane offset, no bounds);
            // only the last, partial batch checks bounds.  The next batch is in flight while
            // this one is counted.
            const uint64_t nfull = (e - a) / STEP;
            E nx[PF_C];
            auto load = [&](uint64_t i0, uint64_t bi) {
                if (bi < nfull) {
                    const E* __restrict__ bp = binned + i0;
#pragma unroll
                    for (int q = 0; q < PF_C; ++q) nx[q] = bp[q * NT_C + tid];
                } else {
#pragma unroll
                    for (int q = 0; q < PF_C; ++q) {
                        const uint64_t i = i0 + (uint64_t)q * NT_C + tid;
                        nx[q] = i < e ? binned[i] : EMPTY;
                    }
                }
            };
            load(a, 0);
            uint64_t bi = 0;
            for (uint64_t i0 = a; i0 < e; i0 += STEP, ++bi) {
                E rv[PF_C];
#pragma unroll
                for (int q = 0; q < PF_C; ++q) rv[q] = nx[q];
                if (i0 + STEP < e) load(i0 + STEP, bi + 1);
                if (filt) {
#pragma unroll
                    for (int q = 0; q < PF_C; ++q) {
                        const uint32_t sk = SUBB ? (uint32_t)(rv[q] >> (rbits - SUBB)) : 0u;
                        rv[q] = (sk >= lo && sk < hi) ? rv[q] : EMPTY;
                    }
                }
                // 1) every home group read before any counter is touched (the counters share
                //    the LDS array, so an atomic in between would serialise the reads): one LDS
                //    round trip settles every element whose key already sits in its home group
                E kg[PF_C][GRP];
#pragma unroll
                for (int q = 0; q < PF_C; ++q) read_group(keys, (uint32_t)rv[q] & (G - 1), kg[q]);
                uint32_t miss = 0;
#pragma unroll
                for (int q = 0; q < PF_C; ++q) {
                    const uint32_t g = (uint32_t)rv[q] & (G - 1);
                    int w = -1;
#pragma unroll
                    for (int t = GRP - 1; t >= 0; --t) w = kg[q][t] == rv[q] ? t : w;
                    const bool live = rv[q] != EMPTY;   // EMPTY would match an empty slot
                    if (live && w >= 0) atomicAdd(&cf[GRP * g + w], 1u);
                    else if (live) miss |= 1u << q;
                }
                // the misses (new keys, keys displaced from home) are compacted into this
                // wave's queue once per batch
                const uint32_t nm = (uint32_t)__popc(miss);
                const uint32_t incl = wave_incl_scan(nm, (int)lane);
                const uint32_t qn = __shfl(incl, 63);
                uint32_t pos = incl - nm;
                while (miss && pos < QN_C) {
                    const int q = __builtin_ctz(miss);
                    miss &= miss - 1u;
                    E pick = rv[0];
#pragma unroll
                    for (int t = 1; t < PF_C; ++t) pick = q == t ? rv[t] : pick;
                    myq[pos++] = pick;
                }
                wave_lds_sync();
                // 2) the queue, 64 misses at a time with every lane busy, one probe step per
                //    iteration; then the (rare) queue overflow, lane by lane
                const uint32_t nq = qn < QN_C ? qn : QN_C;
                for (uint32_t q0 = 0; q0 < nq; q0 += 64) {
                    E r = q0 + lane < nq ? myq[q0 + lane] : EMPTY;
                    uint32_t g = (uint32_t)r & (G - 1);
                    while (__any(r != EMPTY)) {
                        const bool ins = r != EMPTY && count_step(keys, cf, G, s_ovf, r, g);
                        count_occupancy(ins, s_occ, s_ovf, maxload);
                    }
                }
                wave_lds_sync();
                E r = EMPTY;
                uint32_t g = 0;
                while (__any(miss != 0u || r != EMPTY)) {
                    if (r == EMPTY && miss) {
                        const int q = __builtin_ctz(miss);
                        miss &= miss - 1u;
                        E pick = rv[0];
#pragma unroll
                        for (int t = 1; t < PF_C; ++t) pick = q == t ? rv[t] : pick;
                        r = pick;
                        g = (uint32_t)r & (G - 1);
                    }
                    const bool ins = r != EMPTY && count_step(keys, cf, G, s_ovf, r, g);
                    count_occupancy(ins, s_occ, s_ovf, maxload);
                }
                if (__atomic_load_n(&s_ovf, __ATOMIC_RELAXED)) break;
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
        if (HGA_EMIT_STAGE && !xep && F <= EMIT_F && T == (uint32_t)NT_C * EMIT_S) {
            // each thread owns EMIT_S consecutive slots: rows are compacted through LDS (in
            // place, after everyone has read its slots) and then written out coalesced
            E rk[EMIT_S];
            uint32_t rc[EMIT_S][EMIT_F];
            uint32_t keep = 0;
#pragma unroll
            for (int j = 0; j < EMIT_S; ++j) {
                const uint32_t i = (uint32_t)tid * EMIT_S + j;
                rk[j] = keys[i];
                bool any = false;
#pragma unroll
                for (int ff = 0; ff < EMIT_F; ++ff) {
                    const uint32_t c = ff < (int)F ? cnt[(size_t)ff * T + i] : 0u;
                    rc[j][ff] = c >= mc ? c : 0u;
                    any |= c >= mc;
                }
                if (rk[j] != EMPTY && any) keep |= 1u << j;
            }
            uint32_t tot;
            const uint32_t ex = block_excl_scan<NT_C>((uint32_t)__popc(keep), ws, &tot);
            if (tid == 0) {
                s_base = tot ? atomicAdd(&gstat[0], (unsigned long long)tot) : 0ull;
                ++s_ranges;
            }
            __syncthreads();   // every slot read: the table space becomes the staging area
            E* sk = keys;
            uint32_t* sc = reinterpret_cast<uint32_t*>(smem + (size_t)T * sizeof(E));
            uint32_t o = ex;
#pragma unroll
            for (int j = 0; j < EMIT_S; ++j)
                if ((keep >> j) & 1u) {
                    sk[o] = rk[j];
#pragma unroll
                    for (int ff = 0; ff < EMIT_F; ++ff)
                        if (ff < (int)F) sc[(size_t)ff * T + o] = rc[j][ff];
                    ++o;
                }
            __syncthreads();
            const uint64_t base = s_base;
            if (base + tot > cap) {
                if (tid == 0 && tot) atomicOr(&gstat[2], 2ull);
            } else {
                const uint64_t hb = kp.fb ? ((uint64_t)b << rbits) : 0ull;
                for (uint32_t j = tid; j < tot; j += NT_C) {
                    out_key[base + j] = mix_inv(hb | (uint64_t)sk[j], kp.mix);
                    for (uint32_t ff = 0; ff < F; ++ff) out_cnt[(size_t)ff * cap + base + j] = sc[(size_t)ff * T + j];
                }
            }
            __syncthreads();
            continue;
        }
        if (xep) {   // exchange emission (F <= 2): pieces appended to the bucket's slab run, no dense rows
            const XbEmit xe = *xep;
            uint64_t* __restrict__ slab = xe.slab + f[0];
            uint32_t rows = 0;
            for (uint32_t i0 = 0; i0 < T; i0 += NT_C) {   // uniform trip count
                const uint32_t i = i0 + tid;
                const E r = keys[i];
                uint32_t c0 = 0, c1 = 0;
                if (r != EMPTY) {
                    c0 = cnt[i] >= mc ? cnt[i] : 0u;
                    if (F > 1) c1 = cnt[(size_t)T + i] >= mc ? cnt[(size_t)T + i] : 0u;
                }
                const uint32_t big = max(c0, c1);
                const uint32_t np = big == 0u ? 0u : big <= xe.cmax ? 1u : (uint32_t)(((uint64_t)big + xe.cmax - 1) / xe.cmax);
                rows += np != 0u;
                const uint32_t inc = wave_incl_scan(np, (int)lane);
                uint32_t base = 0;
                if (lane == 63 && inc) base = atomicAdd(&s_xw, inc);
                base = __shfl(base, 63, 64);
                if (!np) continue;
                uint64_t at = (uint64_t)base + inc - np;
                const uint64_t h = (kp.fb ? ((uint64_t)b << rbits) : 0ull) | (uint64_t)r;
                while (c0 | c1) {   // one piece, or several adjacent ones past the piece width
                    const uint32_t q0 = min(c0, xe.cmax), q1 = min(c1, xe.cmax);
                    slab[at++] = h | ((uint64_t)q0 << xe.kb) | ((uint64_t)q1 << (xe.kb + xe.cb));
                    c0 -= q0;
                    c1 -= q1;
                }
            }
            if (rows) atomicAdd(&s_xrows, rows);
            if (tid == 0) ++s_ranges;
            __syncthreads();
            continue;
        }
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
    if (xep && tid == 0) {   // the bucket's piece count and its dense row range, reserved once
        xep->dir[b] = s_xw;
        const uint64_t base = s_xrows ? atomicAdd(&gstat[0], (unsigned long long)s_xrows) : 0ull;
        if (base + s_xrows > cap) atomicOr(&gstat[2], 2ull);
        xep->rbase[b] = base;
    }
    if (tid == 0) atomicMax(&gstat[1], (unsigned long long)s_ranges);
    }
}

#ifndef HGA_NT_P
#define HGA_NT_P 512
#endif
#ifndef HGA_PF_P
#define HGA_PF_P 6
#endif
#ifndef HGA_NT_COUNT_LD
#define HGA_NT_COUNT_LD 0   // timing variant: nontemporal element loads in kc_count_s
#endif
constexpr int NT_P = HGA_NT_P;
constexpr int PF_P = HGA_PF_P;          // binned elements per thread per batch
static_assert(PF_P <= 15, "miss counts are scanned as 4-bit values");
constexpr uint32_t QN_P = 128;          // per-wave queue of unsettled keys
constexpr uint32_t MAXPROBE_P = 64;     // groups probed before the table counts as over-full

// ---------------------------------------------------------------- pass C (packed counts, SoA)
// F <= 2 files, u32 remainders, every per-file run of the bucket < 65536 instances (so no
// count can pass 16 bits).  Keys and the packed counts (16 bits per file) in two u32 arrays: a probe
// reads 4 keys with one ds_read_b128, a hit is one ds_add_u32 on the count word (32 banks
// for the count array instead of the odd half of 64), a claim is ds_cmpst_b32 on the key then
// the add.
#ifndef HGA_T_S
#define HGA_T_S 8192
#endif
#ifndef HGA_CS_WAVES
#define HGA_CS_WAVES 4
#endif
constexpr uint32_t T_S = HGA_T_S;       // slots (32 KB keys + 32 KB counts)
#ifndef HGA_GS_S
#define HGA_GS_S 4
#endif
#ifndef HGA_GS_LAZY
#define HGA_GS_LAZY 4
#endif
// keys per probe group, per kernel mode: 4 (one ds_read_b128) or 2 (one ds_read_b64).  A random
// ds_read_b64 is serviced in 2 lane groups of 32 over 64 banks, a ds_read_b128 in 4 groups of 16
// (MI355X_MICROARCH.md §LDS), but 2-key groups displace more keys from their home group (load ~0.48:
// ~10 % vs ~3 %), and in the lazy kernel every instance of a displaced key goes through the miss
// queue: measured at C2, lazy kc_count_s 0.381 ms with 4-key groups, 0.406 with 2 (round 6).
template <int GS>
using KGrpT = std::conditional_t<GS == 4, uint4, uint2>;
static_assert(HGA_GS_S == 2 || HGA_GS_S == 4, "probe groups of 2 or 4 keys");
static_assert(HGA_GS_LAZY == 2 || HGA_GS_LAZY == 4, "probe groups of 2 or 4 keys");

template <int GS>
__device__ __forceinline__ void group_keys(const KGrpT<GS> kg, uint32_t (&k)[GS]) {
    if constexpr (GS == 4) {
        k[0] = kg.x; k[1] = kg.y; k[2] = kg.z; k[3] = kg.w;
    } else {
        k[0] = kg.x; k[1] = kg.y;
    }
}
template <int GS>
__device__ __forceinline__ KGrpT<GS> read_keys_s(const uint32_t* tkey, uint32_t g) {
    return reinterpret_cast<const KGrpT<GS>*>(tkey)[g];
}
template <int GS>
__device__ __forceinline__ void match_s(const KGrpT<GS> kg, uint32_t r, int& w, int& e0) {
    uint32_t k[GS];
    group_keys<GS>(kg, k);
    w = -1;
    e0 = -1;
#pragma unroll
    for (int t = GS - 1; t >= 0; --t) {
        w = k[t] == r ? t : w;
        e0 = k[t] == 0xFFFFFFFFu ? t : e0;
    }
}

// The byte offset of r in a loaded group (4 x its slot), -1 if absent (keys are unique in the table:
// at most one match).
template <int GS>
__device__ __forceinline__ int match_hit4_s(const KGrpT<GS> kg, uint32_t r) {
    uint32_t k[GS];
    group_keys<GS>(kg, k);
    int w = k[0] == r ? 0 : -1;
#pragma unroll
    for (int t = 1; t < GS; ++t) w = k[t] == r ? 4 * t : w;
    return w;
}

// Settle key r (+inc) from its home group; false if MAXPROBE_P groups were full.
template <int GS>
__device__ __forceinline__ bool probe_s(uint32_t* tkey, uint32_t* tcnt, uint32_t r, uint32_t inc) {
    constexpr uint32_t G = T_S / GS;
    uint32_t g = r & (G - 1);
    for (uint32_t steps = 0; steps < MAXPROBE_P * (4 / GS);) {
        int w, e0;
        match_s<GS>(read_keys_s<GS>(tkey, g), r, w, e0);
        if (w >= 0) {
            atomicAdd(&tcnt[g * GS + w], inc);
            return true;
        }
        if (e0 >= 0) {
            const uint32_t sl = g * GS + (uint32_t)e0;
            const uint32_t old = atomicCAS(&tkey[sl], 0xFFFFFFFFu, r);
            if (old == 0xFFFFFFFFu || old == r) {
                atomicAdd(&tcnt[sl], inc);
                return true;
            }
            continue;   // lost the slot to another key: re-read the same group
        }
        g = (g + 1) & (G - 1);
        ++steps;
    }
    return false;
}


// LAZY: the batch only finds existing keys (a hit is one add); a key not in its home group goes
// through the miss queue, which claims new keys with all lanes busy — cheaper where most instances
// repeat a key (C2: ~12 instances per distinct key and bucket, kc_count_s 0.47 -> 0.39 ms); otherwise
// the home group's first empty slot is claimed inline (C4 rank shard: ~5 per key, 9.7 vs 10.0 ms).
template <bool LAZY>
__global__ void __launch_bounds__(NT_P, HGA_CS_WAVES) kc_count_s(const uint32_t* __restrict__ binned,
                                                      const uint64_t* __restrict__ fs, uint32_t F,
                                                      uint32_t min_count, KP kp, uint64_t* __restrict__ out_key,
                                                      uint32_t* __restrict__ out_cnt, uint64_t cap,
                                                      unsigned long long* __restrict__ gstat,
                                                      uint32_t* __restrict__ blist, const XbEmit* __restrict__ xep) {
    __shared__ __attribute__((aligned(16))) uint32_t tkey[T_S];
    __shared__ __attribute__((aligned(16))) uint32_t tcnt[T_S + 64];   // + per-lane dummies (branch-free hits)
    __shared__ uint32_t qbuf[NT_P / 64][QN_P];
    __shared__ uint32_t s_ovf, s_sp, s_ranges;
    __shared__ uint32_t stk_lo[40], stk_hi[40];
    __shared__ uint32_t ws[NT_P / 64 + 1];
    __shared__ unsigned long long s_base;
    __shared__ uint32_t s_xw, s_xrows;   // exchange emission: pieces and rows so far
    constexpr int GS = LAZY ? HGA_GS_LAZY : HGA_GS_S;
    constexpr uint32_t G_S = T_S / GS;
    using KGrp = KGrpT<GS>;
    const int tid = threadIdx.x;
    const uint32_t lane = tid & 63;
    uint32_t* myq = qbuf[tid >> 6];
    const uint32_t b = blockIdx.x;
    const uint64_t* f = fs + (uint64_t)b * (F + 1);
    for (uint32_t ff = 0; ff < F; ++ff)
        if (f[ff + 1] - f[ff] >= 65536u && F > 1) {   // a count could pass 16 bits: kc_count takes it
            if (tid == 0) blist[atomicAdd(&gstat[5], 1ull)] = b;
            if (xep && tid == 0) xep->dir[b] = 0;   // no pieces here
            return;
        }
    const uint32_t rbits = kp.rbits;
    const uint32_t SUBB = rbits < 16 ? rbits : 16;
    const uint32_t full_hi = 1u << SUBB;
    const uint32_t mc = min_count ? min_count : 1u;
    if (tid == 0) {
        stk_lo[0] = 0;
        stk_hi[0] = full_hi;
        s_sp = 1;
        s_ranges = 0;
        s_xw = 0;
        s_xrows = 0;
    }
    __syncthreads();
    while (true) {
        const uint32_t sp = s_sp;
        if (sp == 0) break;
        const uint32_t lo = stk_lo[sp - 1], hi = stk_hi[sp - 1];
        __syncthreads();
        if (tid == 0) {
            s_sp = sp - 1;
            s_ovf = 0;
        }
        for (uint32_t i = tid; i < T_S; i += NT_P) {
            tkey[i] = 0xFFFFFFFFu;
            tcnt[i] = 0;
        }
        __syncthreads();
        const bool filt = !(lo == 0 && hi == full_hi);
        uint32_t qn = 0;   // this wave's queued keys (uniform)
        for (uint32_t ff = 0; ff < F; ++ff) {
            const uint64_t a = f[ff], e = f[ff + 1];
            const uint32_t inc = F == 1 ? 1u : (1u << (16 * ff));
            constexpr uint64_t STEP = (uint64_t)NT_P * PF_P;
            if (a == e) continue;
            const uint64_t nfull = (e - a) / STEP;
            uint32_t nx[PF_P];
            auto load = [&](uint64_t i0, uint64_t bi) {
                if (bi < nfull) {
                    const uint32_t* __restrict__ bp = binned + i0;
#pragma unroll
                    for (int q = 0; q < PF_P; ++q)
                        nx[q] = HGA_NT_COUNT_LD ? __builtin_nontemporal_load(&bp[q * NT_P + tid]) : bp[q * NT_P + tid];
                } else {
#pragma unroll
                    for (int q = 0; q < PF_P; ++q) {
                        const uint64_t i = i0 + (uint64_t)q * NT_P + tid;
                        nx[q] = i < e ? binned[i] : 0xFFFFFFFFu;
                    }
                }
            };
            auto drain = [&](uint32_t min_take) {   // while at least min_take (>= 1) are queued
                while (qn >= min_take && qn > 0) {
                    const uint32_t take = qn < 64 ? qn : 64;
                    const uint32_t q0 = qn - take;
                    bool ok = true;
                    if (lane < take) ok = probe_s<GS>(tkey, tcnt, myq[q0 + lane], inc);
                    if (!ok) s_ovf = 1u;
                    qn = q0;
                    wave_lds_sync();
                }
            };
            load(a, 0);
            uint64_t bi = 0;
            for (uint64_t i0 = a; i0 < e; i0 += STEP, ++bi) {
                uint32_t rv[PF_P];
#pragma unroll
                for (int q = 0; q < PF_P; ++q) rv[q] = nx[q];
                if (i0 + STEP < e) load(i0 + STEP, bi + 1);
                if (filt) {
#pragma unroll
                    for (int q = 0; q < PF_P; ++q) {
                        const uint32_t sk = SUBB ? rv[q] >> (rbits - SUBB) : 0u;
                        rv[q] = (sk >= lo && sk < hi) ? rv[q] : 0xFFFFFFFFu;
                    }
                }
                KGrp kg[PF_P];
                uint32_t ga[PF_P];   // byte offset of each home group (keys; counts at the same offset)
#pragma unroll
                for (int q = 0; q < PF_P; ++q) {
                    ga[q] = (rv[q] & (G_S - 1)) * (GS * 4u);
                    kg[q] = *reinterpret_cast<const KGrp*>(reinterpret_cast<const char*>(tkey) + ga[q]);
                }
                uint32_t claim = 0, miss = 0, slot[PF_P];
                if constexpr (LAZY) {   // new keys go through the miss queue (claimed there, all lanes busy)
                    // byte addresses: the group's key offset, + the match's byte offset = its count word
                    // (tkey and tcnt share the layout); a lane without a hit adds to its dummy word
#pragma unroll
                    for (int q = 0; q < PF_P; ++q) {
                        const int w4 = match_hit4_s<GS>(kg[q], rv[q]);
                        const bool live = rv[q] != 0xFFFFFFFFu;
                        const bool hit = live && w4 >= 0;
                        atomicAdd(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(tcnt) +
                                                              (hit ? ga[q] + (uint32_t)w4 : (T_S + lane) * 4u)),
                                  inc);
                        miss |= (live && !hit) ? 1u << q : 0u;
                    }
                }
#pragma unroll
                for (int q = 0; q < PF_P && !LAZY; ++q) {
                    int w, e0;
                    match_s<GS>(kg[q], rv[q], w, e0);
                    const bool live = rv[q] != 0xFFFFFFFFu;
                    slot[q] = (rv[q] & (G_S - 1)) * GS + (uint32_t)(w >= 0 ? w : e0);
                    {   // every lane adds: a hit to its slot, anything else to its own dummy word
                        const bool hit = live && w >= 0;
                        atomicAdd(&tcnt[hit ? slot[q] : T_S + lane], inc);
                        claim |= (live && !hit && e0 >= 0) ? 1u << q : 0u;
                        miss |= (live && !hit && e0 < 0) ? 1u << q : 0u;
                    }
                }
#pragma unroll
                for (int q = 0; q < PF_P; ++q)
                    if ((claim >> q) & 1u) {
                        const uint32_t old = atomicCAS(&tkey[slot[q]], 0xFFFFFFFFu, rv[q]);
                        if (old == 0xFFFFFFFFu || old == rv[q]) atomicAdd(&tcnt[slot[q]], inc);
                        else miss |= 1u << q;
                    }
                const uint32_t nm = (uint32_t)__popc(miss);
                const uint64_t any = __ballot(nm != 0u);
                if (any) {
                    uint32_t tot;
                    const uint32_t incl = wave_excl_scan_small<4>(nm, &tot) + nm;   // nm <= PF_P = 8
                    if (qn + tot > QN_P) {   // no room: settle the queue first, then these in place
                        drain(1);
                        bool ok = true;
                        while (__any(miss != 0u)) {
                            if (miss) {
                                const int q = __builtin_ctz(miss);
                                miss &= miss - 1u;
                                uint32_t pick = rv[0];
#pragma unroll
                                for (int t = 1; t < PF_P; ++t) pick = q == t ? rv[t] : pick;
                                ok = probe_s<GS>(tkey, tcnt, pick, inc) && ok;
                            }
                        }
                        if (!ok) s_ovf = 1u;
                    } else {
                        uint32_t pos = qn + incl - nm;
#pragma unroll
                        for (int q = 0; q < PF_P; ++q)   // predicated stores, no per-lane loop
                            if ((miss >> q) & 1u) myq[pos++] = rv[q];
                        qn += tot;
                        wave_lds_sync();
                        drain(64);
                    }
                }
                if ((bi & 3u) == 0 && __atomic_load_n(&s_ovf, __ATOMIC_RELAXED)) break;
            }
            drain(1);
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
        // emit: each thread owns ES slots, four consecutive ones per 16-B read, the reads thread-strided
        // (quad (j / 4) * NT_P + tid: lanes on consecutive 16-B groups, no bank conflicts; a
        // thread-contiguous block of 16 slots put every fourth lane on the same banks); kept rows are
        // compacted in place (rows leave a bucket in any order)
        constexpr int ES = T_S / NT_P;
        uint32_t kk[ES], cc[ES];
#pragma unroll
        for (int j = 0; j < ES; j += 4) {
            const uint4 k4 = reinterpret_cast<const uint4*>(tkey)[(j / 4) * NT_P + tid];
            const uint4 c4 = reinterpret_cast<const uint4*>(tcnt)[(j / 4) * NT_P + tid];
            kk[j] = k4.x; kk[j + 1] = k4.y; kk[j + 2] = k4.z; kk[j + 3] = k4.w;
            cc[j] = c4.x; cc[j + 1] = c4.y; cc[j + 2] = c4.z; cc[j + 3] = c4.w;
        }
        uint32_t keep = 0;
#pragma unroll
        for (int j = 0; j < ES; ++j) {
            uint32_t c = cc[j];
            if (F == 1) {
                c = c >= mc ? c : 0u;
            } else {
                const uint32_t c0 = c & 0xFFFFu, c1 = c >> 16;
                c = (c0 >= mc ? c0 : 0u) | ((c1 >= mc ? c1 : 0u) << 16);
            }
            cc[j] = c;
            if (kk[j] != 0xFFFFFFFFu && c) keep |= 1u << j;
        }
        uint32_t tot;
        const uint32_t ex = block_excl_scan<NT_P>((uint32_t)__popc(keep), ws, &tot);
        if (tid == 0) {
            s_base = tot && !xep ? atomicAdd(&gstat[0], (unsigned long long)tot) : 0ull;   // emission: once, at the end
            s_xrows += tot;
            ++s_ranges;
        }
        __syncthreads();   // every slot read: the table becomes the staging area
        uint32_t o = ex;
#pragma unroll
        for (int j = 0; j < ES; ++j)
            if ((keep >> j) & 1u) {
                tkey[o] = kk[j];
                tcnt[o] = cc[j];
                ++o;
            }
        __syncthreads();
        const uint64_t base = s_base;
        const uint64_t hb = kp.fb ? ((uint64_t)b << rbits) : 0ull;
        if (xep) {   // no dense rows: kc_xb_dense writes them from the pieces if a local query needs them
        } else if (base + tot > cap) {
            if (tid == 0 && tot) atomicOr(&gstat[2], 2ull);
        } else {
            for (uint32_t j = tid; j < tot; j += NT_P) {
                const uint32_t c = tcnt[j];
                out_key[base + j] = mix_inv(hb | tkey[j], kp.mix);
                if (F == 1) {
                    out_cnt[base + j] = c;
                } else {
                    out_cnt[base + j] = c & 0xFFFFu;
                    out_cnt[cap + base + j] = c >> 16;
                }
            }
        }
        if (xep) {   // uniform: the exchange pieces of these rows after the earlier ranges' (any order)
            const XbEmit xe = *xep;
            uint64_t* __restrict__ slab = xe.slab + f[0];
            for (uint32_t j0 = 0; j0 < tot; j0 += NT_P) {
                const uint32_t j = j0 + tid;
                const bool live = j < tot;
                const uint32_t c = live ? tcnt[j] : 0u;
                uint32_t c0 = F == 1 ? c : c & 0xFFFFu, c1 = F == 1 ? 0u : c >> 16;
                const uint32_t big = max(c0, c1);
                const uint32_t np = !live ? 0u : big <= xe.cmax ? 1u : (big + xe.cmax - 1) / xe.cmax;
                // wave-aggregated slots: one LDS add per wave
                const uint32_t inc = wave_incl_scan(np, (int)lane);
                uint32_t base = 0;
                if (lane == 63 && inc) base = atomicAdd(&s_xw, inc);
                base = __shfl(base, 63, 64);
                if (!live) continue;
                uint64_t at = (uint64_t)base + inc - np;
                const uint64_t h = hb | tkey[j];
                if (np == 1) {
                    slab[at] = h | ((uint64_t)c0 << xe.kb) | ((uint64_t)c1 << (xe.kb + xe.cb));
                    continue;
                }
                while (c0 | c1) {   // a count past the piece width: several adjacent pieces of one row
                    const uint32_t q0 = min(c0, xe.cmax), q1 = min(c1, xe.cmax);
                    slab[at++] = h | ((uint64_t)q0 << xe.kb) | ((uint64_t)q1 << (xe.kb + xe.cb));
                    c0 -= q0;
                    c1 -= q1;
                }
            }
        }
        __syncthreads();
    }
    __syncthreads();
    if (xep && tid == 0) {   // the bucket's piece count and its dense row range, reserved once
        xep->dir[b] = s_xw;
        const uint64_t base = s_xrows ? atomicAdd(&gstat[0], (unsigned long long)s_xrows) : 0ull;
        if (base + s_xrows > cap) atomicOr(&gstat[2], 2ull);
        xep->rbase[b] = base;
    }
    if (tid == 0) atomicMax(&gstat[1], (unsigned long long)s_ranges);
}

// Dense rows of the buckets kc_count_s emitted as exchange pieces only (XbEmit): one workgroup per
// bucket walks its slab run (pieces of one row are adjacent: a count past the piece width), sums
// each row's pieces and writes the row into the bucket's reserved range rbase[b].
__global__ void __launch_bounds__(256) kc_xb_dense(const uint64_t* __restrict__ slab, const uint64_t* __restrict__ fs,
                                                   uint32_t F, const XbEmit* __restrict__ xep, Mix mx,
                                                   uint64_t* __restrict__ out_key, uint32_t* __restrict__ out_cnt,
                                                   uint64_t cap) {
    __shared__ uint32_t ws[256 / 64 + 1];
    const XbEmit xe = *xep;
    const uint64_t b = blockIdx.x;
    const uint64_t m = xe.dir[b];
    const uint64_t* __restrict__ src = slab + fs[b * (F + 1)];
    const uint64_t kmask = xe.kb >= 64 ? ~0ull : (1ull << xe.kb) - 1, cmax = xe.cmax;
    uint64_t o = xe.rbase[b];
    for (uint64_t i0 = 0; i0 < m; i0 += 256) {   // uniform trip count
        const uint64_t i = i0 + threadIdx.x;
        const uint64_t h = i < m ? src[i] & kmask : 0ull;
        const bool head = i < m && (i == 0 || (src[i - 1] & kmask) != h);
        uint32_t tot;
        const uint32_t ex = block_excl_scan<256>(head ? 1u : 0u, ws, &tot);
        if (head) {
            uint64_t c0 = 0, c1 = 0;
            for (uint64_t q = i; q < m && (src[q] & kmask) == h; ++q) {
                const uint64_t v = src[q];
                c0 += (v >> xe.kb) & cmax;
                if (F > 1) c1 += (v >> (xe.kb + xe.cb)) & cmax;
            }
            out_key[o + ex] = mix_inv(h, mx);
            out_cnt[o + ex] = (uint32_t)c0;
            if (F > 1) out_cnt[cap + o + ex] = (uint32_t)c1;
        }
        o += tot;
    }
}

// ---------------------------------------------------------------- histogram / select
constexpr int NT_H = 256;
constexpr int NT_S = 1024;            // spec_hist workgroup
constexpr int SG_S = 4;               // 4-row groups per thread per step (16-B loads, all issued together)
constexpr uint32_t TL = 1024;         // LDS-privatised totals
constexpr uint32_t TD = 1u << 16;     // dense global totals; beyond -> overflow list
constexpr uint32_t MAX_THR = 16;

// Threshold index of a row: std::set<double>::upper_bound of ((double)prev / total) * 100
// (JellyfishOccurrenceReader.cpp:103), IEEE round-to-nearest, no FMA; thresholds ascending
// and unique (a std::set), so upper_bound = the number of thresholds <= x.  Branch-free over
// the uniform threshold array (scalar loads).
__device__ __forceinline__ uint32_t spec_index(uint32_t prev, uint32_t total, const double* __restrict__ thr,
                                               uint32_t n_thr) {
    const double x = __dmul_rn(__ddiv_rn((double)prev, (double)total), 100.0);
    uint32_t ti = 0;
#pragma unroll
    for (uint32_t t = 0; t < MAX_THR; ++t)
        if (t < n_thr) ti += thr[t] <= x ? 1u : 0u;
    return ti;
}

// Per row: total and prevalent count -> threshold index -> one LDS increment (total < TL).
// Rows are taken four at a time with 16-B loads per file (rows_cap is a multiple of 4) and
// SG_S groups in flight per thread; one workgroup per CU, whose LDS histogram is flushed with
// one global atomic per nonzero bin.  Totals in [TL, TD) (rare) go to the dense global
// histogram directly (ctrl[3] counts them), >= TD to an overflow list.
// bnd (n_thr <= 8, else null): per total t < TL the eight u16 boundaries b_i = the smallest prev with
// thr[i] <= spec(prev, t) (spec_index's expression, evaluated on the host; 0xFFFF: none, and for the
// unused entries) — spec is monotone in prev, so spec_index(prev, t) = #{i : prev >= b_i}: eight integer
// compares instead of a double division per row (C4 shard: 1.47 -> 0.8 ms)
__global__ void __launch_bounds__(NT_S) kc_spec_hist(const uint32_t* __restrict__ cnt, uint64_t rows,
                                                     const unsigned long long* __restrict__ rows_dev,
                                                     uint64_t cap, uint32_t F,
                                                     const double* __restrict__ thr, uint32_t n_thr,
                                                     const uint4* __restrict__ bnd,
                                                     unsigned long long* __restrict__ hist,
                                                     unsigned long long* __restrict__ over,
                                                     unsigned long long* __restrict__ ctrl,
                                                     uint64_t over_cap) {
    extern __shared__ uint32_t lh[];   // n_thr * TL counters (sized at launch)
    __shared__ uint4 sb[TL];
    for (uint32_t i = threadIdx.x; i < n_thr * TL; i += NT_S) lh[i] = 0;
    if (bnd)
        for (uint32_t i = threadIdx.x; i < TL; i += NT_S) sb[i] = bnd[i];
    if (rows_dev) {   // count_run not settled yet: the row cursor it left on the device (<= cap)
        const uint64_t r = *rows_dev;
        rows = r < cap ? r : cap;
    }
    __syncthreads();
    const uint64_t groups = (rows + 3) / 4;
    const uint64_t stride = (uint64_t)gridDim.x * NT_S;
    const uint4* __restrict__ c4 = reinterpret_cast<const uint4*>(cnt);
    for (uint64_t g0 = (uint64_t)blockIdx.x * NT_S + threadIdx.x; g0 < groups; g0 += stride * SG_S) {
        uint32_t tot[SG_S][4], prv[SG_S][4];
#pragma unroll
        for (int u = 0; u < SG_S; ++u) {
            const uint64_t g = g0 + (uint64_t)u * stride;
#pragma unroll
            for (int j = 0; j < 4; ++j) tot[u][j] = prv[u][j] = 0;
#pragma unroll
            for (uint32_t f = 0; f < 4; ++f)
                if (f < F && g < groups) {
                    const uint4 v = c4[(f * cap) / 4 + g];
                    const uint32_t c[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        tot[u][j] += c[j];
                        prv[u][j] = c[j] > prv[u][j] ? c[j] : prv[u][j];
                    }
                }
            for (uint32_t f = 4; f < F && g < groups; ++f) {
                const uint4 v = c4[(f * cap) / 4 + g];
                const uint32_t c[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    tot[u][j] += c[j];
                    prv[u][j] = c[j] > prv[u][j] ? c[j] : prv[u][j];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < SG_S; ++u) {
            const uint64_t g = g0 + (uint64_t)u * stride;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (g * 4 + j >= rows) continue;
                const uint32_t total = tot[u][j];
                uint32_t ti;
                if (bnd && total < TL) {
                    const uint4 b = sb[total];
                    const uint32_t pv = prv[u][j];
                    const uint32_t w[4] = {b.x, b.y, b.z, b.w};
                    ti = 0;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        ti += (pv >= (w[q] & 0xFFFFu) ? 1u : 0u) + (pv >= (w[q] >> 16) ? 1u : 0u);
                } else {
                    ti = spec_index(prv[u][j], total, thr, n_thr);
                }
                if (ti >= n_thr) { atomicOr(&ctrl[1], 1ull); continue; }
                if (total < TL) {
                    atomicAdd(&lh[ti * TL + total], 1u);
                } else if (total < TD) {
                    atomicAdd(&hist[(uint64_t)ti * TD + total], 1ull);
                    atomicAdd(&ctrl[3], 1ull);
                } else {
                    const unsigned long long o = atomicAdd(&ctrl[0], 1ull);
                    if (o < over_cap) over[o] = ((unsigned long long)ti << 56) | total;
                    else atomicOr(&ctrl[1], 2ull);
                }
            }
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n_thr * TL; i += NT_S) {
        const uint32_t v = lh[i];
        if (v) atomicAdd(&hist[(uint64_t)(i / TL) * TD + (i % TL)], (unsigned long long)v);
    }
}

// Nonzero dense bins -> (threshold index << 56 | total, count) pairs, one cursor atomic per
// workgroup; bins are zeroed as they are read (the histogram is cleared once, at allocation).
// Totals >= TL are scanned only when kc_spec_hist put rows there (ctrl[3]).
constexpr int NT_HC = 256;
__global__ void __launch_bounds__(NT_HC) kc_hist_compact(unsigned long long* __restrict__ hist, uint32_t n_thr,
                                                         unsigned long long* __restrict__ out,
                                                         unsigned long long* __restrict__ ctrl, uint64_t cap,
                                                         unsigned long long* __restrict__ hout, uint64_t hcap) {
    __shared__ uint32_t ws[NT_HC / 64 + 1];
    __shared__ unsigned long long s_base;
    const uint64_t i = (uint64_t)blockIdx.x * NT_HC + threadIdx.x;
    const uint32_t ti = (uint32_t)(i / TD), tot = (uint32_t)(i % TD);
    const uint32_t bt = (uint32_t)(((uint64_t)blockIdx.x * NT_HC) % TD);
    if (bt >= TL && ctrl[3] == 0) return;   // uniform per workgroup (TL is a multiple of NT_HC)
    unsigned long long v = 0;
    if (ti < n_thr) {
        v = hist[i];
        if (v) hist[i] = 0;
    }
    uint32_t n;
    const uint32_t ex = block_excl_scan<NT_HC>(v ? 1u : 0u, ws, &n);
    if (threadIdx.x == 0) s_base = n ? atomicAdd(&ctrl[2], (unsigned long long)n) : 0ull;
    __syncthreads();
    const uint64_t o = s_base + ex;
    if (v && o < cap) {
        out[2 * o] = ((unsigned long long)ti << 56) | tot;
        out[2 * o + 1] = v;
    }
    if (v && o < hcap) {   // the first triples also straight into the host's mapped staging
        hout[2 * o] = ((unsigned long long)ti << 56) | tot;
        hout[2 * o + 1] = v;
    }
}

// The spec_hist counters (and an unsettled count_run's) into the host's mapped staging, then ctrl
// cleared for the next call: no copy or fill operations in the step.
__global__ void kc_spec_publish(unsigned long long* __restrict__ ctrl, const unsigned long long* __restrict__ run,
                                unsigned long long* __restrict__ hctrl, unsigned long long* __restrict__ hrun) {
    const uint32_t t = threadIdx.x;
    if (t < 4) {
        hctrl[t] = ctrl[t];
        ctrl[t] = 0;
    }
    if (run && t < 8) hrun[t] = run[t];
}

#ifndef HGA_SEL_GRID
#define HGA_SEL_GRID 1024u   // kc_select workgroups at most (each takes a contiguous range of chunks)
#endif
constexpr int SEL_R = 16;   // rows per thread: chunks of NT_H * SEL_R = 4096 rows
constexpr uint32_t SEL_HB = 4096;   // top-12-bit histogram of the kept keys (the export sort's MSD pass)

// block_excl_scan with LDS-only barriers (global loads issued before it stay in flight)
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan_lb(uint32_t v, uint32_t* ws, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int NW = NT / 64;
    const uint32_t inc = wave_incl_scan(v, lane);
    if (lane == 63) ws[wave] = inc;
    lds_barrier();
    if (wave == 0) {
        const uint32_t t = lane < NW ? ws[lane] : 0u;
        const uint32_t ti = wave_incl_scan(t, lane);
        if (lane < NW) ws[lane] = ti - t;
        if (lane == NW - 1) ws[NW] = ti;
    }
    lds_barrier();
    const uint32_t r = ws[wave] + inc - v;
    *total = ws[NW];
    lds_barrier();
    return r;
}

// Each workgroup takes `cpw` consecutive chunks of 4096 rows and writes its kept keys, in row order,
// to its own region of wkeys (region = cpw * 4096 slots): no device-wide cursor (one same-address
// atomic per chunk serialised at ≈88/µs: 3 ms at a C4 shard's 126 K chunks); kc_sel_compact then
// moves the regions together.  The next chunk's counts are loaded while this one is selected
// (LDS-only barriers keep them in flight).  With dhist_rows the workgroup also counts its kept keys
// by the top 12 bits of the sort width (hshift = 2k - 12), one row of SEL_HB counts per workgroup.
__global__ void __launch_bounds__(NT_H) kc_select(const uint64_t* __restrict__ keys,
                                                  const uint32_t* __restrict__ cnt, uint64_t rows,
                                                  uint64_t cap, uint32_t F, int64_t lower,
                                                  int64_t upper, uint64_t* __restrict__ wkeys,
                                                  uint32_t* __restrict__ wflag, bool flag_bit, uint32_t cpw,
                                                  unsigned long long* __restrict__ wcnt,
                                                  uint32_t* __restrict__ dhist_rows, int hshift,
                                                  unsigned long long* __restrict__ zstat, uint32_t* __restrict__ zdh) {
    __shared__ uint32_t ws[NT_H / 64 + 1];
    // clear what the next kernels of the select accumulate into (kc_sel_compact: stat; kc_dhist_reduce:
    // the 12-bit histogram) — nothing here reads them
    if (blockIdx.x == 0 && threadIdx.x < 8) zstat[threadIdx.x] = 0;
    if (zdh)
        for (uint32_t i = blockIdx.x * NT_H + threadIdx.x; i < SEL_HB; i += gridDim.x * NT_H) zdh[i] = 0;
    __shared__ uint64_t stage[NT_H * SEL_R];
    __shared__ uint8_t sflag[NT_H * SEL_R];
    __shared__ uint32_t dh[SEL_HB];
    if (dhist_rows)
        for (uint32_t i = threadIdx.x; i < SEL_HB; i += NT_H) dh[i] = 0;
    const uint64_t chunks = (rows + NT_H * SEL_R - 1) / (NT_H * SEL_R);
    const uint64_t ch0 = (uint64_t)blockIdx.x * cpw;
    const uint64_t ch1 = ch0 + cpw < chunks ? ch0 + cpw : chunks;
    const uint64_t region = (uint64_t)cpw * NT_H * SEL_R;
    uint64_t* __restrict__ wk = wkeys + blockIdx.x * region;
    uint32_t* __restrict__ wf = flag_bit ? nullptr : wflag + blockIdx.x * region;
    uint64_t wo = 0, wd = 0;   // this workgroup's kept / discriminative rows so far (uniform)
    // the first two files' counts of a chunk's SEL_R rows per thread (rows < cap are allocated)
    uint32_t n0[SEL_R], n1[SEL_R];
    auto load_counts = [&](uint64_t ch) {
        const uint64_t bn = ch * NT_H * SEL_R;
#pragma unroll
        for (int q = 0; q < SEL_R; ++q) {
            const uint64_t r = bn + (uint64_t)q * NT_H + threadIdx.x;
            n0[q] = r < cap ? cnt[r] : 0u;
            n1[q] = (F > 1 && r < cap) ? cnt[cap + r] : 0u;
        }
    };
    if (ch0 < ch1) load_counts(ch0);
    for (uint64_t ch = ch0; ch < ch1; ++ch) {
        const uint64_t base = ch * NT_H * SEL_R;
        uint64_t take = 0, disc = 0;   // bit q: row base + q*NT_H + tid
        uint32_t c0[SEL_R], c1[SEL_R];
#pragma unroll
        for (int q = 0; q < SEL_R; ++q) {
            c0[q] = n0[q];
            c1[q] = n1[q];
        }
        if (ch + 1 < ch1) load_counts(ch + 1);
#pragma unroll
        for (int q = 0; q < SEL_R; ++q) {
            const uint64_t r = base + (uint64_t)q * NT_H + threadIdx.x;
            if (r >= rows) continue;
            int64_t total = (int64_t)c0[q] + c1[q];
            uint32_t nz = (c0[q] > 0) + (c1[q] > 0);
            for (uint32_t f = 2; f < F; ++f) {
                const uint32_t c = cnt[(size_t)f * cap + r];
                total += c;
                nz += c > 0;
            }
            if (lower <= total && total <= upper) {
                take |= 1ull << q;
                if (nz == 1) disc |= 1ull << q;
            }
        }
        // the kept rows' keys requested now: their latency overlaps the scans
        uint64_t kv[SEL_R];
#pragma unroll
        for (int q = 0; q < SEL_R; ++q)
            kv[q] = ((take >> q) & 1ull) ? keys[base + (uint64_t)q * NT_H + threadIdx.x] : 0ull;
        uint32_t tot, dtot;
        const uint32_t ex = block_excl_scan_lb<NT_H>((uint32_t)__popcll(take), ws, &tot);
        (void)block_excl_scan_lb<NT_H>((uint32_t)__popcll(disc), ws, &dtot);
        // kept keys staged in LDS (row order), then written out coalesced
        uint32_t o = ex;
#pragma unroll
        for (int q = 0; q < SEL_R; ++q)
            if ((take >> q) & 1ull) {
                stage[o++] = kv[q] | (flag_bit ? (((disc >> q) & 1ull) << 63) : 0ull);
                if (!flag_bit) sflag[o - 1] = (uint8_t)((disc >> q) & 1ull);
                if (dhist_rows) atomicAdd(&dh[(uint32_t)(kv[q] >> hshift) & (SEL_HB - 1)], 1u);
            }
        lds_barrier();
        for (uint32_t j = threadIdx.x; j < tot; j += NT_H) {
            wk[wo + j] = stage[j];
            if (!flag_bit) wf[wo + j] = sflag[j];
        }
        wo += tot;
        wd += dtot;
        lds_barrier();   // stage is reused by the next chunk
    }
    if (threadIdx.x == 0) {
        wcnt[2 * blockIdx.x] = wo;
        wcnt[2 * blockIdx.x + 1] = wd;
    }
    if (dhist_rows) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < SEL_HB; i += NT_H) dhist_rows[(uint64_t)blockIdx.x * SEL_HB + i] = dh[i];
    }
}

// Workgroup w of kc_select's grid: its kept keys (and flags) to out[sum of the kept counts of
// workgroups < w ...]; workgroup 0 also leaves the totals in stat[0] (kept) and stat[1]
// (discriminative).  The grid's counts are summed by every workgroup (<= HGA_SEL_GRID of them).
__global__ void __launch_bounds__(256) kc_sel_compact(const uint64_t* __restrict__ wkeys,
                                                      const uint32_t* __restrict__ wflag, uint64_t region,
                                                      const unsigned long long* __restrict__ wcnt, uint32_t grid,
                                                      uint64_t* __restrict__ out, uint32_t* __restrict__ out_flag,
                                                      bool flag_bit, unsigned long long* __restrict__ stat) {
    __shared__ unsigned long long red[3][4];
    const uint32_t w = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    unsigned long long pre = 0, tk = 0, td = 0;
    for (uint32_t i = tid; i < grid; i += 256) {
        const unsigned long long k = wcnt[2 * i], d = wcnt[2 * i + 1];
        pre += i < w ? k : 0ull;
        tk += k;
        td += d;
    }
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        pre += __shfl_xor(pre, o, 64);
        tk += __shfl_xor(tk, o, 64);
        td += __shfl_xor(td, o, 64);
    }
    if (lane == 0) {
        red[0][wave] = pre;
        red[1][wave] = tk;
        red[2][wave] = td;
    }
    __syncthreads();
    pre = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    if (w == 0 && tid == 0) {
        stat[0] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
        stat[1] = red[2][0] + red[2][1] + red[2][2] + red[2][3];
    }
    const uint64_t n = wcnt[2 * w];
    const uint64_t* __restrict__ src = wkeys + (uint64_t)w * region;
    for (uint64_t j = tid; j < n; j += 256) {
        out[pre + j] = src[j];
        if (!flag_bit) out_flag[pre + j] = wflag[(uint64_t)w * region + j];
    }
}

// hist[b] += sum over a group of 32 kc_select workgroups' top-12-bit counts (rows x SEL_HB,
// row-major); grid (SEL_HB / 256, row groups), hist zeroed beforehand.
__global__ void __launch_bounds__(256) kc_dhist_reduce(const uint32_t* __restrict__ rows, uint32_t n_rows,
                                                       uint32_t* __restrict__ hist) {
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    const uint32_t r0 = blockIdx.y * 32, r1 = r0 + 32 < n_rows ? r0 + 32 : n_rows;
    uint32_t s = 0;
#pragma unroll 8
    for (uint32_t r = r0; r < r1; ++r) s += rows[(uint64_t)r * SEL_HB + b];
    if (s) atomicAdd(&hist[b], s);
}

// The export sort's MSD digit from the 12-bit histogram, on the device (so only 1 KB comes back):
// the occupied bins [lo, hi], the smallest lg with (hi >> lg) - (lo >> lg) < 256, dbase = lo >> lg,
// and the 256 digit counts dig[d] = sum of bins b in [lo, hi] with (b >> lg) - dbase == d.
// span = {lo, hi, lg, dbase}; all zero when no key was kept.  One 256-thread workgroup.
__global__ void __launch_bounds__(256) kc_sel_span(const uint32_t* __restrict__ hist, uint32_t* __restrict__ span,
                                                   uint32_t* __restrict__ dig, const unsigned long long* __restrict__ stat,
                                                   unsigned long long* __restrict__ hstat, uint32_t* __restrict__ hdig) {
    __shared__ uint32_t s_lo[4], s_hi[4];
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
    for (uint32_t b = t; b < SEL_HB; b += 256)
        if (hist[b]) {
            lo = min(lo, b);
            hi = max(hi, b);
        }
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor(lo, o, 64));
        hi = max(hi, (uint32_t)__shfl_xor(hi, o, 64));
    }
    if (lane == 0) {
        s_lo[wave] = lo;
        s_hi[wave] = hi;
    }
    __syncthreads();
    lo = min(min(s_lo[0], s_lo[1]), min(s_lo[2], s_lo[3]));
    hi = max(max(s_hi[0], s_hi[1]), max(s_hi[2], s_hi[3]));
    // the counts (stat[0..1], from kc_sel_compact), span (stat + 4) and digit counts also go straight
    // into the host's mapped staging
    auto publish = [&](uint32_t d) {
        dig[t] = d;
        hdig[t] = d;
        __syncthreads();   // span (thread 0) before the copy of stat
        if (t < 8) hstat[t] = stat[t];
    };
    if (lo > hi) {   // nothing kept
        if (t < 4) span[t] = 0;
        publish(0u);
        return;
    }
    uint32_t lg = 0;
    while ((hi >> lg) - (lo >> lg) + 1 > 256) ++lg;
    const uint32_t dbase = lo >> lg;
    uint32_t sum = 0;
    const uint32_t b0 = (dbase + t) << lg;
    for (uint32_t b = b0; b < b0 + (1u << lg); ++b)
        if (b >= lo && b <= hi) sum += hist[b];
    if (t == 0) {
        span[0] = lo;
        span[1] = hi;
        span[2] = lg;
        span[3] = dbase;
    }
    publish(sum);
}

// ---- bucketed export sort (moderate exports, flag in key bit 63): the kept keys go straight from
// kc_select's per-workgroup regions to their 12-bit digit segments — deterministic offsets from the
// per-workgroup digit counts (column scan), LDS-ranked inside a workgroup — and every segment of at
// most BX_MAX keys is sorted by one wave in registers (bitonic, 64 x R keys).  Replaces the compaction,
// the MSD onesweep pass and the 256 one-workgroup LDS segment sorts (C2: 0.16 -> ~0.09 ms); exports
// with a larger segment keep that path (sort_export_u64).
constexpr uint32_t BX_MAX = 1024;
// One 1024-thread workgroup: dbase[d] = exclusive scan of the digit totals hist[d]; stat[0] / [1] =
// kept / discriminative keys (the per-workgroup counts wcnt), stat[2] = the largest digit total;
// stat[0..3] also into the host's mapped staging hstat.
__global__ void __launch_bounds__(1024) kc_bx_prep(const uint32_t* __restrict__ hist, const unsigned long long* __restrict__ wcnt,
                                                   uint32_t grid, uint32_t* __restrict__ dbase,
                                                   unsigned long long* __restrict__ stat,
                                                   unsigned long long* __restrict__ hstat) {
    __shared__ uint32_t ws[1024 / 64 + 1];
    __shared__ unsigned long long red[3][16];
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    uint32_t h[4], sum = 0, mx = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        h[q] = hist[4 * t + q];
        sum += h[q];
        mx = max(mx, h[q]);
    }
    uint32_t tot;
    uint32_t o = block_excl_scan<1024>(sum, ws, &tot);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        dbase[4 * t + q] = o;
        o += h[q];
    }
    unsigned long long k = 0, d = 0, m = mx;
    for (uint32_t i = t; i < grid; i += 1024) {
        k += wcnt[2 * i];
        d += wcnt[2 * i + 1];
    }
#pragma unroll
    for (int s2 = 32; s2; s2 >>= 1) {
        k += __shfl_xor(k, s2, 64);
        d += __shfl_xor(d, s2, 64);
        m = max(m, (unsigned long long)__shfl_xor(m, s2, 64));
    }
    if (lane == 0) {
        red[0][wave] = k;
        red[1][wave] = d;
        red[2][wave] = m;
    }
    __syncthreads();
    if (t < 4) {
        unsigned long long v = 0;
        for (int w = 0; w < 16; ++w) v = t == 2 ? max(v, red[2][w]) : v + (t < 2 ? red[t][w] : 0ull);
        stat[t] = v;
        hstat[t] = v;
    }
}
// off[w][d] = dbase[d] + sum over workgroups w' < w of their digit-d counts (rows[w'][d]); one
// workgroup per 16 digits, 16 row groups of threads.
__global__ void __launch_bounds__(256) kc_bx_colscan(const uint32_t* __restrict__ rows, uint32_t n_rows,
                                                     const uint32_t* __restrict__ dbase, uint32_t* __restrict__ off) {
    __shared__ uint32_t part[16][17];
    const uint32_t dl = threadIdx.x & 15, rg = threadIdx.x >> 4, d = blockIdx.x * 16 + dl;
    const uint32_t per = (n_rows + 15) / 16, r0 = rg * per, r1 = min(n_rows, r0 + per);
    uint32_t s2 = 0;
    for (uint32_t r = r0; r < r1; ++r) s2 += rows[(uint64_t)r * SEL_HB + d];
    part[rg][dl] = s2;
    __syncthreads();
    uint32_t base = dbase[d];
    for (uint32_t g = 0; g < rg; ++g) base += part[g][dl];
    for (uint32_t r = r0; r < r1; ++r) {
        off[(uint64_t)r * SEL_HB + d] = base;
        base += rows[(uint64_t)r * SEL_HB + d];
    }
}
// Workgroup w of kc_select's grid: its kept keys from its region to their digit segments (ranks
// inside the workgroup by LDS atomics; a segment is fully sorted afterwards and keys are unique, so
// the order inside it does not matter).
__global__ void __launch_bounds__(256) kc_bx_scatter(const uint64_t* __restrict__ wkeys, uint64_t region,
                                                     const unsigned long long* __restrict__ wcnt,
                                                     const uint32_t* __restrict__ off, int hshift,
                                                     uint64_t* __restrict__ out) {
    __shared__ uint32_t cur[SEL_HB];
    const uint32_t w = blockIdx.x;
    for (uint32_t i = threadIdx.x; i < SEL_HB; i += 256) cur[i] = off[(uint64_t)w * SEL_HB + i];
    __syncthreads();
    const uint64_t n = wcnt[2 * w];
    const uint64_t* __restrict__ src = wkeys + (uint64_t)w * region;
    for (uint64_t j = threadIdx.x; j < n; j += 256) {
        const uint64_t key = src[j];
        const uint32_t pos = atomicAdd(&cur[(uint32_t)(key >> hshift) & (SEL_HB - 1)], 1u);
        out[pos] = key;
    }
}
// One wave per digit segment of at most BX_MAX keys: bitonic sort in registers by the code (the flag
// in bit 63 moved below it: codes are unique, the flag never decides), padding sorts last.
template <int R>
__device__ __forceinline__ void bx_sort_seg(uint64_t* __restrict__ keys, uint32_t start, uint32_t len, uint32_t lane,
                                            int bits) {
    const uint64_t cm = bits >= 63 ? ~0ull >> 1 : (1ull << bits) - 1;
    uint64_t v[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
        const uint32_t i = lane * R + u;
        const uint64_t k = i < len ? keys[start + i] : 0ull;
        v[u] = i < len ? ((k & cm) << 1) | (k >> 63) : ~0ull;
    }
    bitonic_stage<R, 2>(v, lane);
#pragma unroll
    for (int u = 0; u < R; ++u) {
        const uint32_t i = lane * R + u;
        if (i < len) keys[start + i] = (v[u] >> 1) | ((v[u] & 1ull) << 63);
    }
}
// The same with u32 sort keys when the code bits below the digit and the flag fit (2k - 12 + 1 <= 32,
// k <= 21): (low code bits << 1 | flag), the digit restored on the way out — half the registers and
// compare-exchange work of the u64 form.
template <int R>
__device__ __forceinline__ void bx_sort_seg32(uint64_t* __restrict__ keys, uint32_t start, uint32_t len, uint32_t lane,
                                              int bits, uint64_t dig) {
    const int lb = bits - 12;   // code bits below the digit
    const uint64_t lm = (1ull << lb) - 1;
    uint32_t v[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
        const uint32_t i = lane * R + u;
        const uint64_t k = i < len ? keys[start + i] : 0ull;
        v[u] = i < len ? (uint32_t)(((k & lm) << 1) | (k >> 63)) : ~0u;
    }
    bitonic_stage<R, 2>(v, lane);
    const uint64_t hi = dig << lb;
#pragma unroll
    for (int u = 0; u < R; ++u) {
        const uint32_t i = lane * R + u;
        if (i < len) keys[start + i] = hi | (uint64_t)(v[u] >> 1) | ((uint64_t)(v[u] & 1u) << 63);
    }
}
__global__ void __launch_bounds__(256) kc_bx_wsort(uint64_t* __restrict__ keys, const uint32_t* __restrict__ hist,
                                                   const uint32_t* __restrict__ dbase, int bits) {
    const uint32_t d = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t len = hist[d], st = dbase[d];
    if (len <= 1 || len > BX_MAX) return;   // (larger segments: kc_bx_lsort)
    if (bits - 12 + 1 <= 32) {
        if (len <= 64) bx_sort_seg32<1>(keys, st, len, lane, bits, d);
        else if (len <= 256) bx_sort_seg32<4>(keys, st, len, lane, bits, d);
        else if (len <= 512) bx_sort_seg32<8>(keys, st, len, lane, bits, d);
        else bx_sort_seg32<16>(keys, st, len, lane, bits, d);   // len <= BX_MAX (checked by the host)
        return;
    }
    if (len <= 64) bx_sort_seg<1>(keys, st, len, lane, bits);
    else if (len <= 256) bx_sort_seg<4>(keys, st, len, lane, bits);
    else if (len <= 512) bx_sort_seg<8>(keys, st, len, lane, bits);
    else bx_sort_seg<16>(keys, st, len, lane, bits);   // len <= BX_MAX (checked by the host)
}

// Large exports (a C4 rank shard's ~50 M keys: ~12 K a digit, ~25 K in the lowest digits, canonical
// codes being twice as dense there): every digit segment of more than BX_MAX keys is sorted by one
// workgroup in LDS (stable LSD passes, kmer_dev.hpp lds_lsd_sort_t).  With the code bits below the digit
// and the flag in 32 bits (k <= 21) the keys are sorted as u32 (low code bits << 1 | flag, by bits 1..,
// the digit restored on the way out): segments up to 16 K keys by 512 threads over 9-bit digits (80 KB
// of LDS: two workgroups a CU; 3 passes for k = 19), up to 32 K by 1024 threads over 8-bit digits;
// else as u64 by the low code bits (the flag in bit 63 lies above them; codes are unique), 16 K.  With
// kc_bx_scatter this replaces the global LSD radix sort of the low bits + the MSD pass (5-6 global
// passes over the export) by one scatter and one LDS pass.
constexpr uint32_t BX_CAP32 = SS_T * 2 * SS_I;   // 32 K u32 keys
template <bool U32, int NT, int I, int DB>
__global__ void __launch_bounds__(NT) kc_bx_lsort(uint64_t* __restrict__ keys, const uint32_t* __restrict__ hist,
                                                  const uint32_t* __restrict__ dbase, int bits, uint32_t min_len) {
    using T = std::conditional_t<U32, uint32_t, uint64_t>;
    __shared__ T sk[NT * I];
    __shared__ uint32_t wcnt[NT / 64][1 << DB];
    __shared__ uint32_t ws[NT / 64 + 1];
    const uint32_t d = blockIdx.x;
    const uint32_t cnt = hist[d], start = dbase[d];
    if (cnt <= min_len || cnt > (uint32_t)(NT * I)) return;   // (another launch has it)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lb = bits - 12;   // code bits below the digit
    const uint64_t lm = (1ull << lb) - 1;
    T key[I];
#pragma unroll
    for (int j = 0; j < I; ++j) {
        const uint32_t i = (uint32_t)wave * (I * 64) + (uint32_t)j * 64 + lane;
        const uint64_t k = i < cnt ? keys[(uint64_t)start + i] : 0ull;
        if constexpr (U32) key[j] = (uint32_t)(((k & lm) << 1) | (k >> 63));
        else key[j] = k;
    }
    if constexpr (U32) lds_lsd_sort_t<uint32_t, I, NT, DB>(key, cnt, 1, lb, sk, wcnt, ws);
    else lds_lsd_sort_t<uint64_t, I, NT, DB>(key, cnt, 0, lb, sk, wcnt, ws);
    const uint64_t hi = (uint64_t)d << lb;
#pragma unroll
    for (int j = 0; j < I; ++j) {
        const uint32_t i = (uint32_t)wave * (I * 64) + (uint32_t)j * 64 + lane;
        if (i < cnt) {
            if constexpr (U32) keys[(uint64_t)start + i] = hi | (uint64_t)(key[j] >> 1) | ((uint64_t)(key[j] & 1u) << 63);
            else keys[(uint64_t)start + i] = key[j];
        }
    }
}

// The u32 case (k <= 21) of the large-segment sort without LSD passes: the segment's keys (unique
// codes, spread evenly below their digit) are counted into 4096 sub-buckets by the next 12 code bits (LDS
// atomics), the counts scanned, the keys scattered into LDS by sub-bucket (an L2-hot second read of the
// segment), and each thread then sorts its sub-buckets (~3 keys each at a C4 shard's 12 K-key segments,
// ~6 at its 25 K ones: insertion sort; a crowded one by Shell sort) in LDS and writes them out in order —
// about one LDS atomic, write and read per key instead of three stable 9-bit passes with ten ballots a key.
constexpr int CS_T = 1024, CS_B = 12;
__global__ void __launch_bounds__(CS_T) kc_bx_csort(uint64_t* __restrict__ keys, const uint32_t* __restrict__ hist,
                                                    const uint32_t* __restrict__ dbase, int bits, uint32_t min_len) {
    __shared__ uint32_t sk[BX_CAP32];
    __shared__ uint32_t cnt[1 << CS_B];
    __shared__ uint32_t ws[CS_T / 64 + 1];
    const uint32_t d = blockIdx.x;
    const uint32_t n = hist[d], st = dbase[d];
    if (n <= min_len || n > BX_CAP32) return;   // (the host checked the cap for every digit)
    const uint32_t tid = threadIdx.x;
    const int lb = bits - 12;                    // code bits below the digit (<= 30: u32 keys)
    const int sb = lb < CS_B ? lb : CS_B;        // sub-bucket bits
    const int sh = lb - sb;
    const uint64_t lm = (1ull << lb) - 1;
    const uint32_t nsb = 1u << sb;
    for (uint32_t i = tid; i < nsb; i += CS_T) cnt[i] = 0;
    __syncthreads();
    const uint64_t* __restrict__ src = keys + st;
    for (uint32_t i = tid; i < n; i += CS_T) atomicAdd(&cnt[(uint32_t)((src[i] & lm) >> sh)], 1u);
    __syncthreads();
    {   // exclusive scan of the sub-bucket counts, four per thread
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = 4 * tid + (uint32_t)q;
            v[q] = i < nsb ? cnt[i] : 0u;
            sum += v[q];
        }
        uint32_t tot;
        uint32_t o = block_excl_scan<CS_T>(sum, ws, &tot);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = 4 * tid + (uint32_t)q;
            if (i < nsb) cnt[i] = o;
            o += v[q];
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < n; i += CS_T) {
        const uint64_t k = src[i];
        const uint32_t pos = atomicAdd(&cnt[(uint32_t)((k & lm) >> sh)], 1u);   // cnt[c] ends at c's end
        sk[pos] = (uint32_t)(((k & lm) << 1) | (k >> 63));
    }
    __syncthreads();
    const uint64_t hi = (uint64_t)d << lb;
    for (uint32_t c = tid; c < nsb; c += CS_T) {
        const uint32_t b = c ? cnt[c - 1] : 0u, e = cnt[c];
        // Shell sort (Ciura's gaps; gap 1 = insertion sort, all a sub-bucket of a few keys needs): a
        // skewed segment — keys crowded into a few sub-buckets, e.g. a narrow code range — stays
        // O(n^1.3) per thread instead of insertion sort's O(n^2)
        constexpr uint32_t gaps[8] = {701, 301, 132, 57, 23, 10, 4, 1};
        for (int gi = 0; gi < 8; ++gi) {
            const uint32_t g = gaps[gi];
            if (g >= e - b) continue;
            for (uint32_t i = b + g; i < e; ++i) {
                const uint32_t v = sk[i];
                uint32_t j = i;
                for (; j >= b + g && sk[j - g] > v; j -= g) sk[j] = sk[j - g];
                sk[j] = v;
            }
        }
        for (uint32_t i = b; i < e; ++i) {
            const uint32_t v = sk[i];
            keys[(uint64_t)st + i] = hi | (uint64_t)(v >> 1) | ((uint64_t)(v & 1u) << 63);
        }
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

void merge_dump_rows(hga_ctx* c);

void count_begin(hga_ctx* c, int k, uint32_t n_files) {
    HGA_REQUIRE(k >= 1 && k <= 32, HGA_ERR_INVALID, "k must be in [1,32]");
    HGA_REQUIRE(n_files >= 1 && n_files <= 64, HGA_ERR_INVALID, "n_files must be in [1,64]");
    auto& s = c->count;
    for (auto* b : s.seq) delete b;
    s.seq.clear();
    s.seq_len.assign(n_files, 0);
    for (uint32_t i = 0; i < n_files; ++i) s.seq.push_back(new DevBuf());
    s.dump_keys.assign(n_files, {});
    s.dump_cnt.assign(n_files, {});
    s.k = k;
    s.n_files = n_files;
    s.begun = true;
    s.ran = false;
    s.dist = false;
    s.rows = s.instances = s.n_sel = 0;
    s.pending = false;
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
    s.dist = false;
}

void count_run(hga_ctx* c, uint32_t min_per_file) {
    auto& s = c->count;
    HGA_REQUIRE(s.begun, HGA_ERR_STATE, "hga_count_begin not called");
    // A previous run nobody consumed is discarded, errors included: this run replaces its rows
    // (the stream is in order, and kc_init_stat re-initialises the counters it would have read).
    s.pending = false;
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
    // fan-out: ~16K windows per fine bucket, at most 8192 buckets, never more bits than the key
    // packed-count counting (kc_count_s): F <= 2 and u32 remainders; ~64K windows per bucket
    const bool legacy = std::getenv("HGA_COUNT_LEGACY") != nullptr;   // test hook: generic kc_count for F <= 2
    const bool packed = F <= 2 && nbits - std::min<uint32_t>(MAX_FB, nbits) <= 31 && !legacy;
    const uint64_t per_bucket = packed ? HGA_PB_P : 16384;
    uint32_t fb = 0, fb_max = MAX_FB;
    if (const char* e = std::getenv("HGA_FB_MAX")) fb_max = std::min<uint32_t>(MAX_FB, (uint32_t)std::atoi(e));
    // HGA_FB_MIN (test hook): at least that many bucket bits, so small inputs take the paths of large
    // ones (the exchange emission needs fb >= 10)
    const uint32_t fb_min = std::getenv("HGA_FB_MIN") ? (uint32_t)std::atoi(std::getenv("HGA_FB_MIN")) : 0u;
    while (fb < fb_max && fb < nbits && ((total_bytes >> fb) > per_bucket || fb < fb_min)) ++fb;
    kp.fb = fb;
    kp.nb = 1u << fb;
    kp.rbits = nbits - fb;
    kp.rmask = kp.rbits >= 64 ? ~0ull : ((1ull << kp.rbits) - 1);
    kp.fb1 = std::min<uint32_t>(fb, MAX_FB1);
    kp.nb1 = 1u << kp.fb1;
    kp.r1bits = nbits - kp.fb1;
    kp.r1mask = kp.r1bits >= 64 ? ~0ull : ((1ull << kp.r1bits) - 1);
    kp.fb2 = fb - kp.fb1;
    kp.nb2 = 1u << kp.fb2;
    const bool e1_32 = kp.r1bits <= 32;
    const bool e32 = kp.rbits <= 31;
    s.fb = fb;
    s.buckets = kp.nb;
    const uint32_t nb = kp.nb, nb1 = kp.nb1;

    // super-tiles: ~2 per CU over all files (one resident wave of bin1 workgroups, so each
    // (workgroup, region) fills about one level-1 block), whole tiles
    uint64_t st_pos = total_bytes / ((uint64_t)c->num_cu * HGA_B1_PER_CU) + 1;
    // far larger inputs (a C4 rank shard: 7.4 M bases per super-tile, each region's run a chain of
    // ~12 blocks) take more, smaller super-tiles instead, sized so that each (workgroup, region) still
    // fits one block: every re-bin block then writes to precomputed offsets (a chained block reserves
    // its digit runs with a returning device atomic per digit) and bin1 spills almost never
    const uint64_t st_cap = (uint64_t)BLK * nb1 * 15 / 16;   // bases; instances <= bases
    const char* sole_env = std::getenv("HGA_B1_SOLE");
    if ((!sole_env || std::atoi(sole_env) != 0) && st_pos > st_cap + st_cap / 2) st_pos = st_cap;
    st_pos = std::max<uint64_t>(ST_ALIGN, (st_pos + ST_ALIGN - 1) / ST_ALIGN * ST_ALIGN);
    std::vector<uint32_t> n_st(F, 0);
    std::vector<BinFile> bf(F);
    uint32_t W = 0;
    for (uint32_t f = 0; f < F; ++f) {
        n_st[f] = (uint32_t)((s.seq_len[f] + st_pos - 1) / st_pos);
        bf[f].n = s.seq_len[f];
        bf[f].w0 = W;
        W += n_st[f];
    }

    auto* gstat = static_cast<unsigned long long*>(s.cursor.ensure(8 * 8));
    uint64_t* fs = static_cast<uint64_t*>(s.file_start.ensure((size_t)nb * (F + 1) * 8));
    uint32_t* wcnt = static_cast<uint32_t*>(s.fine_hist.ensure((size_t)std::max<uint32_t>(W, 1) * nb * 4));
    auto* off = static_cast<unsigned long long*>(s.cursor2.ensure(((size_t)W * nb + 1) * 8));
    uint32_t* nblk = static_cast<uint32_t*>(s.nblk.ensure((size_t)std::max<uint32_t>(W, 1) * nb1 * 4));
    for (uint32_t f = 0; f < F; ++f) bf[f].seq = s.seq[f]->as<uint8_t>();
    // per-file tables: uploaded only when they change (they are fixed for repeated runs)
    const size_t tb = sizeof(BinFile) * F;
    std::vector<char> tab(tb);
    std::memcpy(tab.data(), bf.data(), tb);
    char* d_tab = static_cast<char*>(s.bin_files.ensure(tb));
    if (s.tab_host != tab) {
        HGA_HIP(hipMemcpy(d_tab, tab.data(), tb, hipMemcpyHostToDevice));
        s.tab_host = tab;
    }
    BinFile* d_bf = reinterpret_cast<BinFile*>(d_tab);

    const size_t esz1 = e1_32 ? 4 : 8, esz = e32 ? 4 : 8;
    uint64_t cap = (total_bytes / std::max<uint32_t>(1, min_per_file) + 4) & ~3ull;   // x4: 16-B row groups
    if (const char* e = std::getenv("HGA_ROW_CAP")) cap = std::max<uint64_t>(4, std::strtoull(e, nullptr, 10) & ~3ull);   // test hook
    const uint32_t slot_b = (uint32_t)esz + 4u * F;
    uint32_t T = 1;
    while ((uint64_t)T * 2 * slot_b <= LDS_TAB) T *= 2;
    HGA_REQUIRE(T >= 2 * NT_C, HGA_ERR_INVALID, "too many files for the LDS table");
    const uint32_t maxload = std::min<uint32_t>((uint32_t)(T * 0.85), T - NT_C - 8);
    void* binned = s.binned.ensure(std::max<size_t>(total_bytes, 1) * esz);

    // level-1 pool: one first block per (workgroup, region) + spill blocks for the worst case
    const uint64_t n_first = (uint64_t)W * nb1;
    const uint64_t table_cap = n_first + total_bytes / BLK + 2;
    const uint64_t pool_cap = table_cap * BLK;
    void* binned1 = s.binned1.ensure(pool_cap * esz1);
    Blk* table = static_cast<Blk*>(s.regions.ensure(table_cap * sizeof(Blk)));
    // pipeline counters (the ASCII bases are packed inside kc_bin1)
    c->launch("kc_init", [&] { hipLaunchKernelGGL(kc_init_stat, dim3(1), dim3(64), 0, c->stream, gstat, n_first); });
    c->check_launch("kc_init");

    // B1: level-1 binning of every file into pool blocks + per-workgroup fine histograms
    if (W) {
        c->launch("kc_bin1", [&] {
#define HGA_BIN1(E1T, KK, FBB)                                                                              \
    hipLaunchKernelGGL((kc_bin1<E1T, KK, FBB>), dim3(W), dim3(NT_B), 0, c->stream, d_bf, F, st_pos, kp, table, table_cap, \
                       pool_cap, static_cast<E1T*>(binned1), wcnt, nblk, gstat)
            // compile-time k for the k of the configs (C1-C4: 19; C5: 15, 17, 19, 21)
            if (e1_32 && kp.k == 19 && kp.fb == MAX_FB && !HGA_B1_NOFB) HGA_BIN1(uint32_t, 19, MAX_FB);
            else if (e1_32 && kp.k == 19) HGA_BIN1(uint32_t, 19, 0);
            else if (e1_32 && kp.k == 17) HGA_BIN1(uint32_t, 17, 0);
            else if (e1_32 && kp.k == 15) HGA_BIN1(uint32_t, 15, 0);
            else if (e1_32) HGA_BIN1(uint32_t, 0, 0);
            else if (kp.k == 21) HGA_BIN1(uint64_t, 21, 0);
            else HGA_BIN1(uint64_t, 0, 0);
#undef HGA_BIN1
        });
        c->check_launch("kc_bin1");
    }
    // L: (bucket, workgroup) output offsets and per-file bucket runs
    c->launch("kc_layout", [&] {
        hipLaunchKernelGGL(kc_transpose, dim3(blocks_for(nb, 64), blocks_for(std::max<uint32_t>(W, 1), 64)), dim3(256),
                           0, c->stream, wcnt, W, nb, reinterpret_cast<uint64_t*>(off));
    });
    c->check_launch("kc_transpose");
    exclusive_scan_u64(c, reinterpret_cast<uint64_t*>(off), (uint64_t)W * nb + 1, s.scratch);
    c->launch("kc_layout", [&] {
        hipLaunchKernelGGL(kc_fs, dim3(blocks_for((uint64_t)nb * (F + 1), 256)), dim3(256), 0, c->stream,
                           reinterpret_cast<const uint64_t*>(off), d_bf, W, nb, F, fs);
    });
    c->check_launch("kc_fs");
    // B2: re-bin every level-1 block into the fine buckets: the first blocks, then the spill blocks
    const unsigned spill_grid = (unsigned)std::min<uint64_t>(table_cap - n_first, HGA_SPILL_GRID);
    c->launch("kc_rebin", [&] {
#define HGA_REBIN(E1T, ET)                                                                                 \
    do {                                                                                                   \
        if (n_first)                                                                                       \
            hipLaunchKernelGGL((kc_rebin<E1T, ET>), dim3((unsigned)n_first), dim3(rebin_nt<ET>()), 0, c->stream, \
                               static_cast<const E1T*>(binned1), table, gstat, W, kp, nblk, off,            \
                               static_cast<ET*>(binned), true);                                              \
        if (spill_grid)                                                                                    \
            hipLaunchKernelGGL((kc_rebin<E1T, ET>), dim3(spill_grid), dim3(rebin_nt<ET>()), 0, c->stream,  \
                               static_cast<const E1T*>(binned1), table, gstat, W, kp, nblk, off,            \
                               static_cast<ET*>(binned), false);                                             \
    } while (0)
        if (e1_32 && e32) HGA_REBIN(uint32_t, uint32_t);
        else if (e32) HGA_REBIN(uint64_t, uint32_t);
        else if (e1_32) HGA_REBIN(uint32_t, uint64_t);
        else HGA_REBIN(uint64_t, uint64_t);
#undef HGA_REBIN
    });
    c->check_launch("kc_rebin");
    // B3: one more split level for inputs whose fine buckets hold far more than one LDS table
    // (the per-bucket estimate, total bytes >> fb, passes 2 x per_bucket only with fb at MAX_FB)
    uint32_t fb3 = 0;
    {
        const uint64_t avg = total_bytes >> fb;
        const char* te = std::getenv("HGA_SPLIT3_TARGET");
        const char* fe = std::getenv("HGA_SPLIT3_FORCE");   // tests: split small inputs too
        const uint64_t target = te ? std::strtoull(te, nullptr, 10) : 32768;
        if (fe) {
            const uint32_t want = (uint32_t)std::atoi(fe);
            while (fb3 < want && fb3 < 8 && ((2u << fb3) * F) <= MAX_SF3 && kp.rbits - fb3 > 1) ++fb3;
        } else if (avg > 2 * per_bucket && fb == MAX_FB) {
            while (fb3 < 8 && (avg >> fb3) > target && ((2u << fb3) * F) <= MAX_SF3 && kp.rbits - fb3 > 10) ++fb3;
        }
    }
    if (fb3) {
        const uint32_t S = 1u << fb3;
        // output regions: 1.25x every bucket + SLACK_3 per sub-bucket (kc_split3's slabs)
        void* binned3 = s.binned3.ensure((total_bytes + total_bytes / 4 + (uint64_t)nb * S * SLACK_3 + 64) * esz);
        uint64_t* fs3 = static_cast<uint64_t*>(s.file_start3.ensure((size_t)nb * S * (F + 1) * 8));
        c->launch("kc_split3", [&] {
            if (e32)
                hipLaunchKernelGGL(kc_split3<uint32_t>, dim3(nb), dim3(NT_3), 0, c->stream,
                                   static_cast<const uint32_t*>(binned), fs, F, fb3, kp.rbits,
                                   static_cast<uint32_t*>(binned3), fs3);
            else
                hipLaunchKernelGGL(kc_split3<uint64_t>, dim3(nb), dim3(NT_3), 0, c->stream,
                                   static_cast<const uint64_t*>(binned), fs, F, fb3, kp.rbits,
                                   static_cast<uint64_t*>(binned3), fs3);
        });
        c->check_launch("kc_split3");
        kp.fb += fb3;
        kp.nb <<= fb3;
        kp.rbits -= fb3;
        kp.rmask = kp.rbits >= 64 ? ~0ull : ((1ull << kp.rbits) - 1);
        binned = binned3;
        fs = fs3;
        s.buckets = kp.nb;
    }
    const uint32_t nbc = kp.nb;   // count buckets
    // exchange emission (kc_count_s XbEmit): a communicator is attached and this is the exchange's
    // local count (min 1) of packable rows; sub-bins x = ceil(log2 P) + 2 bits below the count bucket
    // (about 1024 pieces per owner bucket at C2-sized shards), at least the owners' EB0 bits in all
    XbEmit xe{};
    const XbEmit* d_xe = nullptr;   // the emission parameters in device memory (kernel SGPRs are full)
    s.xb_on = false;
    bool dumps = false;
    for (auto& v : s.dump_keys) dumps = dumps || !v.empty();
    s.dense_pending = false;
    if (c->comm && min_per_file == 1 && packed && e32 && !dumps && !std::getenv("HGA_XB_GENERIC")) {
        const uint32_t P = (uint32_t)c->comm->nranks;
        const int cbits = F <= 8 ? std::min<int>(32, (64 - (int)nbits) / (int)F) : 0;
        const uint32_t eb0 = std::min<uint32_t>(10, nbits);
        const int xoff = std::getenv("HGA_XB_XOFF") ? std::atoi(std::getenv("HGA_XB_XOFF")) : 2;   // tuning
        uint32_t x = (uint32_t)std::max(0, xoff);   // 2: C2 units of ~1024 pieces (1: 0.21 ms merge, 3: 0.19, 2: 0.14)
        for (uint32_t q = 1; q < P; q <<= 1) ++x;
        x = std::min<uint32_t>(x, 6u);
        // owners' cells (EB0 bits) must be whole count buckets: the per-owner sizes come from the
        // per-bucket counts before the gather sub-bins them
        if (cbits >= 4 && kp.fb >= eb0 && x <= kp.rbits) {
            const uint64_t slab_n = fb3 ? (total_bytes + total_bytes / 4 + (uint64_t)nbc * SLACK_3 + 64) : total_bytes;
            xe.slab = static_cast<uint64_t*>(s.xslab.ensure(std::max<uint64_t>(slab_n, 1) * 8));
            xe.dir = static_cast<uint64_t*>(s.xdir_b.ensure((uint64_t)nbc * 8 + 64));
            xe.rbase = static_cast<uint64_t*>(s.xrbase.ensure((uint64_t)nbc * 8 + 64));
            xe.cb = (uint32_t)cbits;
            xe.kb = nbits;
            xe.cmax = (uint32_t)((1ull << cbits) - 1);
            s.xb_on = true;
            s.xb_P = P;
            s.xb_x = x;
            s.xb_R = (int)(kp.fb + x);
            s.xb_nbc = nbc;
            s.xb_fs = fs;
            XbEmit* d = static_cast<XbEmit*>(s.xemit.ensure(sizeof(XbEmit)));
            if (std::memcmp(&s.xemit_host, &xe, sizeof(XbEmit)) != 0) {   // uploaded when it changes
                HGA_HIP(hipMemcpy(d, &xe, sizeof(XbEmit), hipMemcpyHostToDevice));
                std::memcpy(&s.xemit_host, &xe, sizeof(XbEmit));
            }
            d_xe = d;
            s.dense_pending = true;
            s.xb_dev = d;
            s.xb_cap = cap;
        }
    }
    // the dense rows (an emitting count writes none: count_dense allocates them if a query needs them;
    // at a C4 rank shard's min-1 capacity they would be 60 GB)
    if (!d_xe) {
        s.rows_key.ensure(cap * 8);
        s.rows_cnt.ensure(cap * 4 * F);
    }
    // C: per-bucket count
    if (packed && e32) {
        uint32_t* blist = static_cast<uint32_t*>(s.blist.ensure((size_t)nbc * 4));
        c->launch("kc_count", [&] {
            // instances per count bucket: >= 32 K (C2-sized) -> the lazy claim (HGA_CS_LAZY=0/1 forces)
            const char* le = std::getenv("HGA_CS_LAZY");
            const bool lazy = le ? std::atoi(le) != 0 : (total_bytes >> kp.fb) >= 32768;
            if (lazy)
                hipLaunchKernelGGL(kc_count_s<true>, dim3(nbc), dim3(NT_P), 0, c->stream,
                                   static_cast<const uint32_t*>(binned), fs, F, min_per_file, kp,
                                   s.rows_key.as<uint64_t>(), s.rows_cnt.as<uint32_t>(), cap, gstat, blist, d_xe);
            else
                hipLaunchKernelGGL(kc_count_s<false>, dim3(nbc), dim3(NT_P), 0, c->stream,
                                   static_cast<const uint32_t*>(binned), fs, F, min_per_file, kp,
                                   s.rows_key.as<uint64_t>(), s.rows_cnt.as<uint32_t>(), cap, gstat, blist, d_xe);
            // buckets with a per-file run >= 65536 (listed in blist, count in gstat[5])
            hipLaunchKernelGGL(kc_count<uint32_t>, dim3(std::min<uint32_t>(nbc, (uint32_t)c->num_cu)), dim3(NT_C), 0,
                               c->stream, static_cast<const uint32_t*>(binned), fs, F, T, maxload, min_per_file, kp,
                               s.rows_key.as<uint64_t>(), s.rows_cnt.as<uint32_t>(), cap, gstat,
                               (const uint32_t*)blist, d_xe);
        });
        c->check_launch("kc_count");
    } else
    c->launch("kc_count", [&] {
        if (e32)
            hipLaunchKernelGGL(kc_count<uint32_t>, dim3(nbc), dim3(NT_C), 0, c->stream,
                               static_cast<const uint32_t*>(binned), fs, F, T, maxload, min_per_file, kp,
                               s.rows_key.as<uint64_t>(), s.rows_cnt.as<uint32_t>(), cap, gstat, (const uint32_t*)nullptr);
        else
            hipLaunchKernelGGL(kc_count<uint64_t>, dim3(nbc), dim3(NT_C), 0, c->stream,
                               static_cast<const uint64_t*>(binned), fs, F, T, maxload, min_per_file, kp,
                               s.rows_key.as<uint64_t>(), s.rows_cnt.as<uint32_t>(), cap, gstat, (const uint32_t*)nullptr);
    });
    c->check_launch("kc_count");
    // No synchronisation here: the counters stay on the device until the next call that needs
    // them (count_settle), so the following spec_hist queues behind the count without a gap.
    s.rows_cap = cap;
    s.ran = true;
    s.dist = false;
    s.n_sel = 0;
    s.sel_rep_n = ~0ull;
    s.pending = true;
    if (dumps) count_settle(c);   // the cached rows are merged on the host side now
}

// Read back the counters of a count_run that has not been settled yet (one D2H + sync, or the
// caller's copy `h` of them), report its errors, publish rows / instances and merge dump rows.
void count_settle(hga_ctx* c, const unsigned long long* h) {
    auto& s = c->count;
    if (!s.pending) return;
    unsigned long long h_stat[8];
    if (!h) {
        HGA_HIP(hipMemcpyAsync(h_stat, s.cursor.p, sizeof(h_stat), hipMemcpyDeviceToHost, c->stream));
        c->sync();
        h = h_stat;
    }
    s.pending = false;
    if (h[2] & 7ull) s.ran = false;   // a failed run has no rows to consume
    s.last_err = h[2] & 7ull;         // proto::QE_UNSPLIT / QE_ROWCAP / QE_POOL
    HGA_REQUIRE(!(h[2] & 4ull), HGA_ERR_OOM, "level-1 block pool exhausted");
    HGA_REQUIRE(!(h[2] & 1ull), HGA_ERR_INVALID, "a bucket could not be split to fit the LDS table");
    HGA_REQUIRE(!(h[2] & 2ull), HGA_ERR_OOM, "row capacity exceeded");
    s.rows = h[0];
    s.max_split = (uint32_t)h[1];
    s.instances = h[4];
    s.listed = h[5];
    merge_dump_rows(c);
}

// The dense rows of an exchange-emitting count (kc_count_s XbEmit writes pieces only), for the
// local queries; enqueued on the stream, no host round trip.
void count_dense(hga_ctx* c) {
    auto& s = c->count;
    if (!s.dense_pending) return;
    s.dense_pending = false;
    if (!s.xb_nbc) return;
    s.rows_key.ensure(s.xb_cap * 8);
    s.rows_cnt.ensure(s.xb_cap * 4 * s.n_files);
    c->launch("kc_xb_dense", [&] {
        hipLaunchKernelGGL(kc_xb_dense, dim3(s.xb_nbc), dim3(256), 0, c->stream, s.xslab.as<uint64_t>(), s.xb_fs,
                           s.n_files, static_cast<const XbEmit*>(s.xb_dev), make_mix(s.k), s.rows_key.as<uint64_t>(),
                           s.rows_cnt.as<uint32_t>(), s.xb_cap);
    });
    c->check_launch("kc_xb_dense");
}

// Pre-counted rows of a file whose `<reads>_<k>-mers_sorted` cache exists
// (JellyfishOccurrenceReader.cpp:19-24 skips jellyfish for it and reads the dump verbatim).
void count_add_rows(hga_ctx* c, uint32_t file, const uint64_t* keys, const uint32_t* counts, uint64_t n) {
    auto& s = c->count;
    s.pending = false;   // an unconsumed run is discarded: its rows are out of date from here on
    HGA_REQUIRE(s.begun, HGA_ERR_STATE, "hga_count_begin not called");
    HGA_REQUIRE(file < s.n_files, HGA_ERR_INVALID, "file index out of range");
    HGA_REQUIRE(n == 0 || (keys && counts), HGA_ERR_INVALID, "null rows pointer");
    const uint64_t lim = s.k >= 32 ? ~0ull : (1ull << (2 * s.k)) - 1;
    auto& dk = s.dump_keys[file];
    auto& dc = s.dump_cnt[file];
    for (uint64_t i = 0; i < n; ++i) {
        HGA_REQUIRE(keys[i] <= lim, HGA_ERR_INVALID, "dump key exceeds 4^k - 1");
        if (!counts[i]) continue;
        dk.push_back(keys[i]);
        dc.push_back(counts[i]);
    }
    s.ran = false;
    s.dist = false;
}

// Folds the staged dump rows into the counted rows: one merge (sum per key, no drop: the
// reference reads cached dumps as they are), leaving the rows ascending.
void merge_dump_rows(hga_ctx* c) {
    auto& s = c->count;
    const uint32_t F = s.n_files;
    uint64_t nd = 0;
    for (auto& v : s.dump_keys) nd += v.size();
    if (!nd) return;
    const uint64_t n = s.rows + nd;
    std::vector<uint64_t> hk;
    std::vector<uint32_t> hc;
    hk.reserve(nd);
    hc.assign(nd * F, 0);
    for (uint32_t f = 0; f < F; ++f)
        for (uint64_t i = 0; i < s.dump_keys[f].size(); ++i) {
            hc[hk.size() * F + f] = s.dump_cnt[f][i];
            hk.push_back(s.dump_keys[f][i]);
        }
    DevBuf tk, tc, ti;
    uint64_t* k = static_cast<uint64_t*>(tk.ensure(n * 8));
    uint32_t* cc = static_cast<uint32_t*>(tc.ensure(n * 4 * F));
    if (s.rows) {
        uint32_t* v = static_cast<uint32_t*>(ti.ensure(s.rows * 4));
        HGA_HIP(hipMemcpyAsync(k, s.rows_key.p, s.rows * 8, hipMemcpyDeviceToDevice, c->stream));
        hipLaunchKernelGGL(kc_iota, dim3(blocks_for(s.rows, 256)), dim3(256), 0, c->stream, v, s.rows);
        c->check_launch("kc_iota");
        hipLaunchKernelGGL(kc_gather_rows, dim3(blocks_for(s.rows, 256)), dim3(256), 0, c->stream, v,
                           s.rows_cnt.as<uint32_t>(), s.rows, s.rows_cap, F, cc);
        c->check_launch("kc_gather_rows");
    }
    HGA_HIP(hipMemcpyAsync(k + s.rows, hk.data(), nd * 8, hipMemcpyHostToDevice, c->stream));
    HGA_HIP(hipMemcpyAsync(cc + s.rows * F, hc.data(), nd * 4 * F, hipMemcpyHostToDevice, c->stream));
    const uint32_t min_c = s.min_per_file;
    count_merge(c, k, cc, n, 1);   // synchronises before the host staging goes out of scope
    s.min_per_file = min_c;
}

void count_spec_hist(hga_ctx* c, const double* thr_in, uint32_t n_thr_in, std::vector<int64_t>& out,
                     const SpecHook* before_publish) {
    auto& s = c->count;
    HGA_REQUIRE(s.ran, HGA_ERR_STATE, "hga_count_run not called");
    count_dense(c);
    std::vector<double> thr(thr_in, thr_in + n_thr_in);   // std::set<double> semantics
    std::sort(thr.begin(), thr.end());
    thr.erase(std::unique(thr.begin(), thr.end()), thr.end());
    const uint32_t n_thr = (uint32_t)thr.size();
    HGA_REQUIRE(n_thr >= 1 && n_thr <= MAX_THR, HGA_ERR_INVALID, "1..16 thresholds supported");
    const uint64_t over_cap = 1u << 20;
    const size_t hbytes = (size_t)MAX_THR * TD * 8;
    const bool fresh = s.hist_dense.cap == 0;
    char* base = static_cast<char*>(s.hist_dense.ensure(hbytes + over_cap * 8 + 256 + 64 + (size_t)TL * 16));
    auto* hist = reinterpret_cast<unsigned long long*>(base);
    auto* over = reinterpret_cast<unsigned long long*>(base + hbytes);
    auto* ctrl = reinterpret_cast<unsigned long long*>(base + hbytes + over_cap * 8);
    double* dthr = reinterpret_cast<double*>(ctrl + 4);
    // pinned staging: [thresholds | ctrl readback (4 u64) | first SPEC_CHUNK compacted triples]
    // 1024 triples (16 KB) cover a C2-sized histogram; the speculative read-back of 4096 (64 KB)
    // cost ~20 us per call in the bench step
    constexpr uint64_t SPEC_CHUNK = 1u << 10;
    char* hp = static_cast<char*>(c->pinned.ensure(MAX_THR * 8 + 32 + SPEC_CHUNK * 16 + 64));
    double* hthr = reinterpret_cast<double*>(hp);
    auto* hc = reinterpret_cast<unsigned long long*>(hp + MAX_THR * 8);
    auto* hcomp = reinterpret_cast<unsigned long long*>(hp + MAX_THR * 8 + 32);
    auto* hrun = reinterpret_cast<unsigned long long*>(hp + MAX_THR * 8 + 32 + SPEC_CHUNK * 16);
    std::memcpy(hthr, thr.data(), n_thr * 8);
    // hist is kept clear by kc_hist_compact, ctrl by kc_spec_publish
    if (fresh) HGA_HIP(hipMemsetAsync(base, 0, hbytes + over_cap * 8 + 256, c->stream));
    auto* dbnd = reinterpret_cast<uint4*>(base + hbytes + over_cap * 8 + 256 + 64);
    const bool use_bnd = n_thr <= 8 && !std::getenv("HGA_SPEC_FP64");
    if (fresh || s.thr_dev != thr) {   // the same thresholds as last time are already there
        HGA_HIP(hipMemcpyAsync(dthr, hthr, n_thr * 8, hipMemcpyHostToDevice, c->stream));
        if (n_thr <= 8) {   // the per-total boundaries of kc_spec_hist (its comment), same IEEE expression
            std::vector<uint16_t> b((size_t)TL * 8, 0xFFFF);
            for (uint32_t t = 1; t < TL; ++t)
                for (uint32_t i = 0; i < n_thr; ++i) {
                    uint32_t lo = 0, hi = t + 1;   // smallest prev in [0, t] passing, t + 1 = none
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi) / 2;
                        const volatile double x = (double)mid / (double)t;
                        if (thr[i] <= x * 100.0) hi = mid; else lo = mid + 1;
                    }
                    b[(size_t)t * 8 + i] = lo > t ? 0xFFFF : (uint16_t)lo;
                }
            HGA_HIP(hipMemcpy(dbnd, b.data(), b.size() * 2, hipMemcpyHostToDevice));
        }
        s.thr_dev = thr;
    }
    // an unsettled count_run: rows come from its device cursor, the counters ride in this readback
    const bool pend = s.pending;
    const uint64_t rows_hint = pend ? s.rows_cap : s.rows;
    const unsigned grid = (unsigned)std::min<uint64_t>(blocks_for(std::max<uint64_t>((rows_hint + 3) / 4, 1), NT_S * SG_S),
                                                       (uint64_t)c->num_cu);
    c->launch("kc_spec_hist", [&] {
        hipLaunchKernelGGL(kc_spec_hist, dim3(grid), dim3(NT_S), (size_t)n_thr * TL * 4, c->stream,
                           s.rows_cnt.as<uint32_t>(), rows_hint,
                           pend ? static_cast<const unsigned long long*>(s.cursor.p) : nullptr, s.rows_cap, s.n_files,
                           dthr, n_thr, use_bnd ? (const uint4*)dbnd : nullptr,
                           hist, over, ctrl, over_cap);
    });
    c->check_launch("kc_spec_hist");
    // compact the dense bins on the device: only (threshold, total, count) triples cross PCIe
    const uint64_t ncap = 1u << 20;
    auto* comp = static_cast<unsigned long long*>(s.hist_comp.ensure(ncap * 16 + 64));
    const uint64_t nd = (uint64_t)n_thr * TD;
    c->launch("kc_spec_hist", [&] {
        hipLaunchKernelGGL(kc_hist_compact, dim3(blocks_for(nd, NT_HC)), dim3(NT_HC), 0, c->stream, hist, n_thr, comp,
                           ctrl, ncap, c->pinned.dev(hcomp), SPEC_CHUNK);
        if (before_publish) (*before_publish)(ctrl, comp);
        // one synchronisation: counters and (speculatively) the first chunk of triples together,
        // written into the mapped staging by the kernels themselves
        hipLaunchKernelGGL(kc_spec_publish, dim3(1), dim3(64), 0, c->stream, ctrl,
                           pend ? static_cast<const unsigned long long*>(s.cursor.p) : nullptr, c->pinned.dev(hc),
                           c->pinned.dev(hrun));
    });
    c->check_launch("kc_hist_compact");
    c->sync();
    s.last_err = 0;
    if (pend) count_settle(c, hrun);
    s.last_err = ((hc[1] & 1ull) ? 8ull : 0ull) | ((hc[1] & 2ull) ? 16ull : 0ull) | (hc[2] > ncap ? 32ull : 0ull);
    HGA_REQUIRE(!(hc[1] & 1ull), HGA_ERR_INVALID, "a row's specificity is above the last threshold");
    HGA_REQUIRE(!(hc[1] & 2ull), HGA_ERR_OOM, "histogram overflow list full");
    HGA_REQUIRE(hc[2] <= ncap, HGA_ERR_OOM, "histogram compaction buffer full");
    // (threshold << 56 | total, count) pairs: the dense bins are unique, overflow rows add 1 each;
    // sorted by the packed key = std::map<double, std::map<int, int>> order (threshold, then total)
    std::vector<std::pair<uint64_t, uint64_t>> bins;
    bins.reserve(hc[2] + std::min<uint64_t>(hc[0], over_cap));
    if (hc[2]) {
        const unsigned long long* cv = hcomp;
        std::vector<unsigned long long> rest;
        if (hc[2] > SPEC_CHUNK) {
            rest.resize(2 * hc[2]);
            HGA_HIP(hipMemcpy(rest.data(), comp, hc[2] * 16, hipMemcpyDeviceToHost));
            cv = rest.data();
        }
        for (uint64_t i = 0; i < hc[2]; ++i) bins.emplace_back(cv[2 * i], cv[2 * i + 1]);
    }
    if (hc[0]) {
        std::vector<unsigned long long> ov(std::min<uint64_t>(hc[0], over_cap));
        HGA_HIP(hipMemcpy(ov.data(), over, ov.size() * 8, hipMemcpyDeviceToHost));
        for (auto v : ov) bins.emplace_back(v, 1ull);
    }
    std::sort(bins.begin(), bins.end());
    out.clear();
    out.reserve(3 * bins.size());
    for (size_t i = 0; i < bins.size();) {
        const uint64_t key = bins[i].first;
        uint64_t cnt = 0;
        for (; i < bins.size() && bins[i].first == key; ++i) cnt += bins[i].second;
        out.push_back((int64_t)(key >> 56));
        out.push_back((int64_t)(key & ((1ull << 56) - 1)));
        out.push_back((int64_t)cnt);
    }
}

void count_select(hga_ctx* c, int64_t lower, int64_t upper, uint64_t* n_out, uint64_t* n_discr,
                  const SelHook* before_sync) {
    auto& s = c->count;
    count_settle(c);
    HGA_REQUIRE(s.ran, HGA_ERR_STATE, "hga_count_run not called");
    count_dense(c);
    const uint64_t cap = std::max<uint64_t>(s.rows, 1);
    char* sb = static_cast<char*>(s.sel_keys.ensure(cap * 12 + 256));
    uint64_t* out = reinterpret_cast<uint64_t*>(sb);
    uint32_t* flag = reinterpret_cast<uint32_t*>(sb + cap * 8);
    const bool flag_bit = s.k <= 31;   // the discriminative flag rides in key bit 63
    const int bits = 2 * s.k;
    // export sort: one MSD pass over the span the kept keys actually occupy (the whole code space:
    // hash-bucket owners' keys also cover every code; the re-partition by code range comes after,
    // comm.hip count_export_repartition) + per-segment LDS sorts (sort_export_u64) when the flag rides
    // in the key; kc_select counts the kept keys by the top 12 bits of the code
    const bool msd = flag_bit && bits >= 16 && s.rows >= (1u << 15);
    const uint64_t chunks = blocks_for(std::max<uint64_t>(s.rows, 1), NT_H * SEL_R);
    if (!s.sel_grid) {   // one resident round of workgroups: a second, partial round would run alone
        int nb = 0;      // (C4 shard: 1024 workgroups at 3 per CU took two rounds)
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kc_select, NT_H, 0) != hipSuccess || nb < 1) nb = 1;
        s.sel_grid = (uint32_t)std::min<uint64_t>((uint64_t)nb * c->num_cu, HGA_SEL_GRID);
        if (const char* e = std::getenv("HGA_SEL_GRID_X")) s.sel_grid = std::max(1, std::atoi(e));   // tuning
    }
    // below 32 M rows half the grid: the export sort's column scan runs over every workgroup's digit
    // histogram (C2: -0.005 ms; a C4 shard's 515 M rows keep the whole grid, 1.65 vs 1.93 ms)
    const uint32_t sel_grid = s.rows < (1ull << 25) && !std::getenv("HGA_SEL_GRID_X") ? std::min(s.sel_grid, 512u)
                                                                                        : s.sel_grid;
    const uint32_t cpw = (uint32_t)blocks_for(chunks, sel_grid);   // chunks per workgroup
    const unsigned grid = (unsigned)blocks_for(chunks, cpw);
    const uint64_t region = (uint64_t)cpw * NT_H * SEL_R;
    const size_t hb = (size_t)SEL_HB * 4;
    // [stat 64 | dhist | dig256 1 KB | dhist_rows (msd) | wcnt | dbase (msd) | off (msd)]
    const size_t rows_b = msd ? (size_t)grid * hb : 0;
    char* tb = static_cast<char*>(s.sel_tmp.ensure(64 + hb + 1024 + rows_b + (size_t)grid * 16 + (msd ? hb + rows_b : 0)));
    auto* wcnt = reinterpret_cast<unsigned long long*>(tb + 64 + hb + 1024 + rows_b);
    uint32_t* bx_dbase = msd ? reinterpret_cast<uint32_t*>(tb + 64 + hb + 1024 + rows_b + (size_t)grid * 16) : nullptr;
    uint32_t* bx_off = msd ? bx_dbase + SEL_HB : nullptr;
    char* wt = static_cast<char*>(s.sel_wtmp.ensure((size_t)grid * region * (flag_bit ? 8 : 12) + 64));
    uint64_t* wkeys = reinterpret_cast<uint64_t*>(wt);
    uint32_t* wflag = reinterpret_cast<uint32_t*>(wt + (size_t)grid * region * 8);
    auto* stat = reinterpret_cast<unsigned long long*>(tb);
    uint32_t* dhist = reinterpret_cast<uint32_t*>(tb + 64);                // SEL_HB top-12-bit counts
    uint32_t* dig256 = reinterpret_cast<uint32_t*>(tb + 64 + hb);          // the MSD digit counts
    uint32_t* dhist_rows = msd ? reinterpret_cast<uint32_t*>(tb + 64 + hb + 1024) : nullptr;
    char* hp = static_cast<char*>(c->pinned_sel.ensure(64 + 1024));
    auto* hs = reinterpret_cast<unsigned long long*>(hp);
    uint32_t* h256 = reinterpret_cast<uint32_t*>(hp + 64);
    if (!s.rows) HGA_HIP(hipMemsetAsync(stat, 0, 64, c->stream));   // else kc_select clears stat and dhist
    if (s.rows) {
        c->launch("kc_select", [&] {
            hipLaunchKernelGGL(kc_select, dim3(grid), dim3(NT_H), 0, c->stream, s.rows_key.as<uint64_t>(),
                               s.rows_cnt.as<uint32_t>(), s.rows, s.rows_cap, s.n_files, lower, upper, wkeys, wflag,
                               flag_bit, cpw, wcnt, dhist_rows, bits - 12, stat, msd ? dhist : nullptr);
            if (msd) {   // the digit totals, their scan, the counts and the largest digit (kc_bx_prep)
                hipLaunchKernelGGL(kc_dhist_reduce, dim3(SEL_HB / 256, (grid + 31) / 32), dim3(256), 0, c->stream,
                                   dhist_rows, grid, dhist);
                hipLaunchKernelGGL(kc_bx_prep, dim3(1), dim3(1024), 0, c->stream, (const uint32_t*)dhist,
                                   (const unsigned long long*)wcnt, grid, bx_dbase, stat, c->pinned_sel.dev(hs));
            } else {
                hipLaunchKernelGGL(kc_sel_compact, dim3(grid), dim3(256), 0, c->stream, (const uint64_t*)wkeys,
                                   (const uint32_t*)wflag, region, (const unsigned long long*)wcnt, grid, out, flag,
                                   flag_bit, stat);
            }
        });
        c->check_launch("kc_select");
    }
    // one synchronisation for the counts (kc_bx_prep writes them into the mapped staging; else a copy)
    if (!(s.rows && msd)) HGA_HIP(hipMemcpyAsync(hs, stat, 64, hipMemcpyDeviceToHost, c->stream));
    if (before_sync) (*before_sync)(stat);
    c->sync();
    const uint64_t n = hs[0];
    // bucketed export sort while every 12-bit digit segment fits one workgroup's LDS sort (C2: all of them
    // fit one wave's registers; a C4 rank shard's ~12 K-key segments take kc_bx_lsort)
    const bool u32seg = bits - 12 + 1 <= 32;
    const bool bx = msd && n > 1 && hs[2] <= (u32seg ? (uint64_t)BX_CAP32 : (uint64_t)SS_CAP) && !std::getenv("HGA_BX_OFF");
    if (bx) {   // bucketed export sort: digit segments straight from the workgroup regions
        c->launch("bx_colscan", [&] {
            hipLaunchKernelGGL(kc_bx_colscan, dim3(SEL_HB / 16), dim3(256), 0, c->stream, (const uint32_t*)dhist_rows,
                               grid, (const uint32_t*)bx_dbase, bx_off);
        });
        c->launch("bx_scatter", [&] {
            hipLaunchKernelGGL(kc_bx_scatter, dim3(grid), dim3(256), 0, c->stream, (const uint64_t*)wkeys, region,
                               (const unsigned long long*)wcnt, (const uint32_t*)bx_off, bits - 12, out);
        });
        c->launch("radix_segsort", [&] {
            hipLaunchKernelGGL(kc_bx_wsort, dim3(SEL_HB / 4), dim3(256), 0, c->stream, out, (const uint32_t*)dhist,
                               (const uint32_t*)bx_dbase, bits);
        });
        c->check_launch("kc_bx_wsort");
        if (hs[2] > BX_MAX) {
            c->launch("radix_segsort", [&] {
                if (u32seg && !std::getenv("HGA_BX_LSD")) {   // (HGA_BX_LSD: the LSD-pass kernels, tests)
                    hipLaunchKernelGGL(kc_bx_csort, dim3(SEL_HB), dim3(CS_T), 0, c->stream, out, (const uint32_t*)dhist,
                                       (const uint32_t*)bx_dbase, bits, BX_MAX);
                } else if (u32seg) {
                    hipLaunchKernelGGL((kc_bx_lsort<true, 512, 32, 9>), dim3(SEL_HB), dim3(512), 0, c->stream, out,
                                       (const uint32_t*)dhist, (const uint32_t*)bx_dbase, bits, BX_MAX);
                    if (hs[2] > 16384u)
                        hipLaunchKernelGGL((kc_bx_lsort<true, 1024, 32, 8>), dim3(SEL_HB), dim3(1024), 0, c->stream,
                                           out, (const uint32_t*)dhist, (const uint32_t*)bx_dbase, bits, 16384u);
                } else {
                    hipLaunchKernelGGL((kc_bx_lsort<false, SS_T, SS_I, 8>), dim3(SEL_HB), dim3(SS_T), 0, c->stream,
                                       out, (const uint32_t*)dhist, (const uint32_t*)bx_dbase, bits, BX_MAX);
                }
            });
            c->check_launch("kc_bx_lsort");
        }
    } else if (msd && n > 1) {
        // compaction, then the MSD pass: digit = (code >> shift) - dbase over the occupied 12-bit bins
        // [lo, hi], <= 256 digits (kc_sel_span: span into stat + 4, the 256 digit counts into dig256)
        c->launch("kc_select", [&] {
            hipLaunchKernelGGL(kc_sel_compact, dim3(grid), dim3(256), 0, c->stream, (const uint64_t*)wkeys,
                               (const uint32_t*)wflag, region, (const unsigned long long*)wcnt, grid, out, flag,
                               flag_bit, stat);
            hipLaunchKernelGGL(kc_sel_span, dim3(1), dim3(256), 0, c->stream, (const uint32_t*)dhist,
                               reinterpret_cast<uint32_t*>(stat + 4), dig256, (const unsigned long long*)stat,
                               c->pinned_sel.dev(hs), c->pinned_sel.dev(h256));
        });
        c->check_launch("kc_sel_span");
        c->sync();
        const uint32_t* span = reinterpret_cast<const uint32_t*>(hs + 4);   // written at stat + 4
        const int shift = bits - 12 + (int)span[2];
        sort_export_u64(c, out, n, shift, span[3], dig256, h256, s.scratch);
    } else if (msd && n == 1) {
        c->launch("kc_select", [&] {
            hipLaunchKernelGGL(kc_sel_compact, dim3(grid), dim3(256), 0, c->stream, (const uint64_t*)wkeys,
                               (const uint32_t*)wflag, region, (const unsigned long long*)wcnt, grid, out, flag,
                               flag_bit, stat);
        });
        c->check_launch("kc_sel_compact");
    } else {
        radix_sort_u64(c, out, flag_bit ? nullptr : flag, n, bits, s.scratch);
    }
    s.n_sel = n;
    s.sel_rep_n = ~0ull;   // a new selection: its code-range re-partition is stale
    *n_out = n;
    *n_discr = hs[1];
}

void count_fetch_selected(hga_ctx* c, uint64_t* dst, uint8_t* flags) {
    auto& s = c->count;
    count_settle(c);
    const uint64_t cap = std::max<uint64_t>(s.rows, 1);
    const bool flag_bit = s.k <= 31;
    if (flag_bit) {   // flag in bit 63 of each key
        std::vector<uint64_t> tmp;
        uint64_t* kd = dst;
        if (!kd && flags && s.n_sel) {
            tmp.resize(s.n_sel);
            kd = tmp.data();
        }
        if (s.n_sel && kd) HGA_HIP(hipMemcpyAsync(kd, s.sel_keys.p, s.n_sel * 8, hipMemcpyDeviceToHost, c->stream));
        c->sync();
        for (uint64_t i = 0; kd && i < s.n_sel; ++i) {
            if (flags) flags[i] = (uint8_t)(kd[i] >> 63);
            kd[i] &= ~(1ull << 63);
        }
        return;
    }
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

// The merged rows ascending on the device: keys[rows], counts row-major [rows][F] (enqueued).
void count_rows_device(hga_ctx* c, DevBuf& keys, DevBuf& counts) {
    auto& s = c->count;
    const uint64_t rows = s.rows;
    const uint32_t F = s.n_files;
    uint64_t* k = static_cast<uint64_t*>(keys.ensure(std::max<uint64_t>(rows, 1) * 8));
    uint32_t* cc = static_cast<uint32_t*>(counts.ensure(std::max<uint64_t>(rows, 1) * 4 * F));
    if (!rows) return;
    DevBuf tv;
    uint32_t* v = static_cast<uint32_t*>(tv.ensure(rows * 4));
    HGA_HIP(hipMemcpyAsync(k, s.rows_key.p, rows * 8, hipMemcpyDeviceToDevice, c->stream));
    hipLaunchKernelGGL(kc_iota, dim3(blocks_for(rows, 256)), dim3(256), 0, c->stream, v, rows);
    c->check_launch("kc_iota");
    radix_sort_u64(c, k, v, rows, 2 * s.k, s.scratch);
    hipLaunchKernelGGL(kc_gather_rows, dim3(blocks_for(rows, 256)), dim3(256), 0, c->stream, v,
                       s.rows_cnt.as<uint32_t>(), rows, s.rows_cap, F, cc);
    c->check_launch("kc_gather_rows");
    c->sync();   // tv is freed on return
}

// All merged rows ascending into malloc'ed buffers (hga_count_rows): keys[rows], counts[rows][F].
void count_rows_to(hga_ctx* c, uint64_t** keys, uint32_t** counts, uint64_t* n_rows) {
    auto& s = c->count;
    count_settle(c);
    HGA_REQUIRE(s.ran, HGA_ERR_STATE, "hga_count_run not called");
    count_dense(c);
    const uint64_t rows = s.rows;
    const uint32_t F = s.n_files;
    auto* hk = static_cast<uint64_t*>(std::malloc(std::max<uint64_t>(rows, 1) * 8));
    auto* hc = static_cast<uint32_t*>(std::malloc(std::max<uint64_t>(rows, 1) * 4ull * F));
    if (!hk || !hc) {
        std::free(hk);
        std::free(hc);
        throw std::bad_alloc();
    }
    try {
        if (rows) {
            DevBuf tk, tc;
            count_rows_device(c, tk, tc);
            HGA_HIP(hipMemcpyAsync(hk, tk.p, rows * 8, hipMemcpyDeviceToHost, c->stream));
            HGA_HIP(hipMemcpyAsync(hc, tc.p, rows * 4ull * F, hipMemcpyDeviceToHost, c->stream));
            c->sync();
        }
    } catch (...) {
        std::free(hk);
        std::free(hc);
        throw;
    }
    *keys = hk;
    *counts = hc;
    *n_rows = rows;
}

// All merged rows ascending (file < 0), or one file's dump rows (file >= 0).
void count_rows(hga_ctx* c, int file, std::vector<uint64_t>& keys, std::vector<uint32_t>& counts) {
    auto& s = c->count;
    count_settle(c);
    HGA_REQUIRE(s.ran, HGA_ERR_STATE, "hga_count_run not called");
    count_dense(c);
    HGA_REQUIRE(file < (int)s.n_files, HGA_ERR_INVALID, "file index out of range");
    const uint64_t rows = s.rows;
    const uint32_t F = s.n_files;
    keys.clear();
    counts.clear();
    if (!rows) return;
    DevBuf tk, tc;
    count_rows_device(c, tk, tc);
    const uint64_t* k = tk.as<uint64_t>();
    const uint32_t* cc = tc.as<uint32_t>();
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
