// Feasibility probe (not product code): level-1 binning of super-k-mer records (windows that share
// their minimizer, cut to <= R windows) instead of one element per window.  Times the kernel on a
// C2-sized synthetic input; compare with kc_bin1's 0.63 ms for the same 256 M windows.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include "../../hybrid-genome-assembler_amd/csrc/kmer_dev.hpp"
using namespace hga;

constexpr int K = 19, KM = 8, M = K - KM, P = 16, NT = NT_SK, TP = NT * P;
constexpr int NB1 = 64, FB2 = 7, NB2 = 1 << FB2, NB = NB1 * NB2, R = RMAX;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1);} } while (0)

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__global__ void __launch_bounds__(NT) sk_bin1(const uint32_t* __restrict__ pk, const uint16_t* __restrict__ vd,
                                              uint64_t nb, uint64_t st_pos, uint64_t* __restrict__ out, uint64_t capr,
                                              uint32_t* __restrict__ wcnt, unsigned long long* __restrict__ gstat) {
    __shared__ uint32_t cnt1[NB1], off1[NB1 + 1], fill[NB1];
    __shared__ uint32_t fh[NB];
    __shared__ uint64_t stage[TP];
    const int tid = threadIdx.x;
    for (int b = tid; b < NB; b += NT) fh[b] = 0;
    if (tid < NB1) { cnt1[tid] = 0; fill[tid] = 0; }
    __syncthreads();
    const uint64_t start = (uint64_t)blockIdx.x * st_pos, end = start + st_pos < nb ? start + st_pos : nb;
    uint32_t nrec = 0, nwin = 0;
    constexpr uint64_t mm = (1ull << (2 * M)) - 1;
    for (uint64_t t0 = start; t0 < end; t0 += TP) {
        const uint64_t p0 = t0 + (uint64_t)tid * P;
        Frame<P> f;
        const uint64_t v64 = load_frame<P, false>(pk, vd, PAD_WORDS + p0 / 16 - 2, K, f);
        const uint32_t wm = (uint32_t)(runs_of(v64, K) >> 32) & 0xFFFFu;
        constexpr int NM = P + KM, NWF = Frame<P>::NW;
        uint32_t mh[NM];
#pragma unroll
        for (int t = 0; t < NM; ++t) {
            const int pj = t - KM;
            const uint32_t fm = (uint32_t)(field64<NWF>(f.x, 2 * (16 * NWF - 33 - pj)) & mm);
            const uint32_t rm = (uint32_t)(field64<NWF>(f.r, 2 * (pj + KM)) & mm);
            mh[t] = (fm < rm ? fm : rm) * 0x9E3779B1u;
        }
        uint32_t wmin[P];
        {
            constexpr int B = KM + 1;
            uint32_t pre[NM], suf[NM];
#pragma unroll
            for (int t = 0; t < NM; ++t) pre[t] = (t % B == 0) ? mh[t] : min(pre[t - 1], mh[t]);
#pragma unroll
            for (int t = NM - 1; t >= 0; --t) suf[t] = (t % B == B - 1 || t == NM - 1) ? mh[t] : min(suf[t + 1], mh[t]);
#pragma unroll
            for (int j = 0; j < P; ++j) wmin[j] = min(suf[j], pre[j + KM]);
        }
        // records: runs of valid windows with one minimizer, <= R long; closed at window j
        uint64_t rec[P];
        uint32_t dd[P], rk[P], close = 0;
        uint32_t len = 0;
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const bool v = (wm >> j) & 1u;
            len = v ? len + 1 : 0;
            const bool nxt = j + 1 < P && ((wm >> (j + 1)) & 1u) && wmin[j + 1 < P ? j + 1 : j] == wmin[j] && len < R;
            rk[j] = 0; dd[j] = 0; rec[j] = 0;
            if (v && !nxt) {
                close |= 1u << j;
                const uint32_t h = wmin[j];
                const uint32_t rh = (h ^ (h >> 15)) * 0x85EBCA6Bu;
                const uint32_t d = rh >> 26, d2 = (rh >> 19) & (NB2 - 1);
                const int B = K - 1 + (int)len;
                const uint64_t bases = field64<NWF>(f.x, 2 * (16 * NWF - 33 - j)) & ((1ull << (2 * B)) - 1);
                rec[j] = bases | ((uint64_t)(len - 1) << 54) | ((uint64_t)d2 << 57);
                dd[j] = d;
                rk[j] = atomicAdd(&cnt1[d], 1u);
                atomicAdd(&fh[(d << FB2) | d2], 1u);
                len = 0;
            }
        }
        nrec += __popc(close);
        nwin += __popc(wm);
        lds_barrier();
        if (tid < 64) {
            const uint32_t c = cnt1[tid];
            const uint32_t inc = wave_incl_scan(c, tid);
            off1[tid] = inc - c;
            cnt1[tid] = 0;
            if (tid == 63) off1[NB1] = inc;
        }
        lds_barrier();
#pragma unroll
        for (int j = 0; j < P; ++j)
            if ((close >> j) & 1u) stage[off1[dd[j]] + rk[j]] = rec[j];
        lds_barrier();
        for (uint32_t d = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6); d < NB1; d += NT / 64) {
            const uint32_t o = off1[d], n = off1[d + 1] - o, fo = fill[d];
            uint64_t* dst = out + ((uint64_t)blockIdx.x * NB1 + d) * capr + fo;
            for (uint32_t jj = (uint32_t)(tid & 63); jj < n; jj += 64) if (fo + jj < capr) dst[jj] = stage[o + jj];
            if ((tid & 63) == 0) fill[d] = fo + n;
        }
        lds_barrier();
    }
    __syncthreads();
    for (int b = tid; b < NB; b += NT) wcnt[(uint64_t)blockIdx.x * NB + b] = fh[b];
    atomicAdd(&gstat[0], (unsigned long long)nrec);
    atomicAdd(&gstat[1], (unsigned long long)nwin);
}

int main() {
    const uint64_t G = 10000000, nreads = 1940000, L = 150;
    std::mt19937_64 rng(1);
    std::vector<char> g(G);
    const char* A = "ACGT";
    for (auto& c : g) c = A[rng() & 3];
    std::vector<uint8_t> s;
    s.reserve(nreads * (L + 1));
    for (uint64_t r = 0; r < nreads; ++r) {
        const uint64_t st = rng() % (G - L);
        for (uint64_t i = 0; i < L; ++i) {
            char c = g[st + i];
            if ((rng() % 1000) < 5) c = A[rng() & 3];
            s.push_back((uint8_t)c);
        }
        s.push_back('\n');
    }
    const uint64_t n = s.size(), nw = (n + 15) / 16, words = PAD_WORDS + nw + 1024;
    uint8_t* ds; uint32_t* pk; uint16_t* vd;
    CK(hipMalloc(&ds, n)); CK(hipMalloc(&pk, words * 4)); CK(hipMalloc(&vd, words * 2));
    CK(hipMemset(pk, 0, words * 4)); CK(hipMemset(vd, 0, words * 2));
    CK(hipMemcpy(ds, s.data(), n, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(pack_kernel<false>, dim3((nw + 255) / 256), dim3(256), 0, 0, ds, n, pk, vd, nw);
    int cu = 256;
    const uint64_t W = cu * PER_CU;
    uint64_t st_pos = (n + W - 1) / W;
    st_pos = (st_pos + TP - 1) / TP * TP;
    const uint64_t nwg = (n + st_pos - 1) / st_pos;
    const uint64_t capr = st_pos / NB1 * 2 + 4096;
    uint64_t* out; uint32_t* wcnt; unsigned long long* gs;
    CK(hipMalloc(&out, nwg * NB1 * capr * 8)); CK(hipMalloc(&wcnt, nwg * NB * 4)); CK(hipMalloc(&gs, 64));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float best = 1e9, sum = 0;
    for (int it = 0; it < 12; ++it) {
        CK(hipMemset(gs, 0, 64));
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(sk_bin1, dim3(nwg), dim3(NT), 0, 0, pk, vd, n, st_pos, out, capr, wcnt, gs);
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        if (it >= 2) { best = ms < best ? ms : best; sum += ms; }
    }
    unsigned long long h[2]; CK(hipMemcpy(h, gs, 16, hipMemcpyDeviceToHost));
    printf("NT=%d R=%d PER_CU=%d: sk_bin1 best %.4f ms avg %.4f ms; windows %llu records %llu (%.2f windows/record)\n",
           NT, R, PER_CU, best, sum / 10, h[1], h[0], (double)h[1] / h[0]);
    return 0;
}
