// hll.hip — MI355X replacement for the HyperLogLog k-mer cardinality estimate behind
// jf_occurrences' automatic k selection (src/jellyfish_occurrences.cpp:40-44 ->
// get_unique_k_length / get_approximate_kmer_count, src/occurrences/KmerAnalysis.cpp:15-56).
//
// The reference feeds every KmerIterator window of every record (canonical code, KmerIterator
// semantics: non-ACGT bytes contribute code 0 to both strands) as its 8 little-endian bytes to
// hll::HyperLogLog(b = 10)::add (src/lib/HyperLogLog.hpp:96-106):
//     h = MurmurHash3_x86_32(&kmer, 8, seed 313)        (src/lib/MurmurHash3.cpp:94-140)
//     index = h >> (32 - b);  rank = min(32 - b, clz(h << b)) + 1;  M[index] = max(M[index], rank)
// Registers are a max over a set, so they are independent of thread and window order: the
// device result equals the reference's bit for bit.  clz(0) (h << b == 0, undefined for
// __builtin_clz) is taken as 32, i.e. rank = 32 - b + 1.
//
//   hll_scan    32 window ends per thread from the lookup's packed frames (lk_pack output:
//               hga_lookup_set_reads); canonical code, murmur3, rank; registers privatised in
//               LDS (a window only touches LDS when it raises its register, which after the
//               first few thousand windows almost never happens); every workgroup loops over
//               tiles and writes its registers once.
//   hll_reduce  max over the workgroups' register rows (row groups in parallel + atomicMax).
// Algorithmic bytes: 0.375 B per base (packed codes + valid bits) + 0.125 B (read-start bits).
#include <algorithm>

#include "hga_internal.hpp"
#include "kmer_dev.hpp"

namespace hga {
namespace {

constexpr int HL_T = 256;       // threads per workgroup
constexpr int HL_P = 32;        // window ends per thread (one read-start word)
constexpr int HL_MAXB = 14;     // 2^14 u32 registers = 64 KB of LDS
constexpr int SB_PAD = 1;       // leading zero words of the read-start bitmap (lookup.hip)
constexpr uint32_t HLL_SEED = 313;   // HLL_HASH_SEED, src/lib/HyperLogLog.hpp:17

// MurmurHash3_x86_32 of the 8 bytes of a little-endian u64 (two 4-byte blocks, no tail).
__device__ __forceinline__ uint32_t murmur3_u64(uint64_t key, uint32_t seed) {
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    uint32_t h = seed;
    const uint32_t blk[2] = {(uint32_t)key, (uint32_t)(key >> 32)};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        uint32_t k1 = blk[i] * c1;
        k1 = (k1 << 15) | (k1 >> 17);
        k1 *= c2;
        h ^= k1;
        h = (h << 13) | (h >> 19);
        h = h * 5u + 0xe6546b64u;
    }
    h ^= 8u;
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

// K > 0: k known at compile time (frame offsets and masks fold; for K <= 16 the high 4-byte block
// of the key is zero and its murmur round folds to constants); K == 0: any k.
template <int K>
__global__ void __launch_bounds__(HL_T) hll_scan(const uint32_t* __restrict__ pk, const uint16_t* __restrict__ vd,
                                                 const unsigned int* __restrict__ sb, uint64_t nbases, int k_rt,
                                                 int b, uint64_t n_threads, uint8_t* __restrict__ part) {
    extern __shared__ uint32_t reg[];
    const int k = K ? K : k_rt;
    const uint32_t m = 1u << b;
    for (uint32_t i = threadIdx.x; i < m; i += HL_T) reg[i] = 0;
    __syncthreads();
    const uint64_t mask = k >= 32 ? ~0ull : ((1ull << (2 * k)) - 1);
    const uint32_t rb = 32u - (uint32_t)b;
    for (uint64_t gt = (uint64_t)blockIdx.x * HL_T + threadIdx.x; gt < n_threads;
         gt += (uint64_t)gridDim.x * HL_T) {
        const uint64_t p0 = gt * HL_P;
        Frame<HL_P> f;
        (void)load_frame<HL_P, true>(pk, vd, PAD_WORDS + p0 / 16 - 2, k, f);
        const uint64_t s64 = (uint64_t)sb[SB_PAD + p0 / 32 - 1] | ((uint64_t)sb[SB_PAD + p0 / 32] << 32);
        uint32_t wm = (uint32_t)(runs_of(~s64, k - 1) >> 32);   // window inside one read
        const uint64_t left = nbases - p0;
        if (left < 32) wm &= (1u << left) - 1u;
        constexpr int NW = Frame<HL_P>::NW;
#pragma unroll
        for (int j = 0; j < HL_P; ++j) {
            const uint64_t fwd = field64<NW>(f.x, 2 * (16 * NW - 33 - j)) & mask;
            const uint64_t rc = field64<NW>(f.r, 2 * j) & mask;
            const uint32_t h = murmur3_u64(fwd < rc ? fwd : rc, HLL_SEED);
            const uint32_t idx = h >> rb;
            // rank = min(32 - b, clz(h << b)) + 1, with clz(0) = 32 (see the header)
            const uint32_t rank = min(rb, (uint32_t)__clz((int)(h << b))) + 1u;
            if (((wm >> j) & 1u) && rank > reg[idx]) atomicMax(&reg[idx], rank);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < m; i += HL_T) part[(uint64_t)blockIdx.x * m + i] = (uint8_t)reg[i];
}

// Max over the workgroups' register rows: block (x, y) takes 256 registers of rows
// [y * HL_RG, (y + 1) * HL_RG) (independent loads, unrolled), then one atomicMax per register
// and block (HL_RG = 64: 32 atomics per register at 2048 rows).
constexpr uint32_t HL_RG = 64;
__global__ void __launch_bounds__(256) hll_reduce(const uint8_t* __restrict__ part, uint32_t nblk, uint32_t m,
                                                  uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const uint32_t r0 = blockIdx.y * HL_RG, r1 = min(nblk, r0 + HL_RG);
    uint32_t v = 0;
#pragma unroll 8
    for (uint32_t w = r0; w < r1; ++w) v = max(v, (uint32_t)part[(uint64_t)w * m + i]);
    if (v) atomicMax(&out[i], v);
}

}  // namespace

void hll_registers(hga_ctx* c, int k, int b, uint8_t* regs) {
    auto& L = c->lookup;
    HGA_REQUIRE(L.have_reads, HGA_ERR_STATE, "hga_lookup_set_reads not called");
    HGA_REQUIRE(k >= 1, HGA_ERR_INVALID, "k must be >= 1");
    HGA_REQUIRE(k <= 32, HGA_ERR_INVALID, "Kmer size is too big");   // KmerIterator.cpp:24-26
    HGA_REQUIRE(b >= 4 && b <= HL_MAXB, HGA_ERR_INVALID, "bit width must be in the range [4,14]");
    if (!L.packed_ok) lookup_pack(c);
    const uint32_t m = 1u << b;
    const uint64_t nb = L.n_bases;
    const uint64_t n_threads = (nb + HL_P - 1) / HL_P;
    if (n_threads == 0) {
        std::fill(regs, regs + m, (uint8_t)0);
        return;
    }
    const uint64_t want = (n_threads + HL_T - 1) / HL_T;
    const uint32_t nblk = (uint32_t)std::min<uint64_t>(want, (uint64_t)c->num_cu * 8);
    uint8_t* part = static_cast<uint8_t*>(L.hll_part.ensure((uint64_t)nblk * m + 4ull * m));
    uint32_t* dout = reinterpret_cast<uint32_t*>(part + (uint64_t)nblk * m);
    HGA_HIP(hipMemsetAsync(dout, 0, 4ull * m, c->stream));
    c->launch("hll_scan", [&] {
        // compile-time k for the auto-k sweep (k = 11, 13, ..., 31: KmerAnalysis.cpp:41-56)
#define HGA_HLL(KK)                                                                                           \
    hipLaunchKernelGGL(hll_scan<KK>, dim3(nblk), dim3(HL_T), m * 4, c->stream, L.packed.as<uint32_t>(),        \
                       L.valid.as<uint16_t>(), L.starts.as<unsigned int>(), nb, k, b, n_threads, part)
        switch (k) {
            case 11: HGA_HLL(11); break;
            case 13: HGA_HLL(13); break;
            case 15: HGA_HLL(15); break;
            case 17: HGA_HLL(17); break;
            case 19: HGA_HLL(19); break;
            case 21: HGA_HLL(21); break;
            case 23: HGA_HLL(23); break;
            case 25: HGA_HLL(25); break;
            case 27: HGA_HLL(27); break;
            case 29: HGA_HLL(29); break;
            case 31: HGA_HLL(31); break;
            default: HGA_HLL(0); break;
        }
#undef HGA_HLL
    });
    c->check_launch("hll_scan");
    c->launch("hll_reduce", [&] {
        hipLaunchKernelGGL(hll_reduce, dim3((m + 255) / 256, (nblk + HL_RG - 1) / HL_RG), dim3(256), 0, c->stream,
                           part, nblk, m, dout);
    });
    c->check_launch("hll_reduce");
    std::vector<uint32_t> r32(m);
    HGA_HIP(hipMemcpyAsync(r32.data(), dout, 4ull * m, hipMemcpyDeviceToHost, c->stream));
    c->sync();
    for (uint32_t i = 0; i < m; ++i) regs[i] = (uint8_t)r32[i];
}

}  // namespace hga
