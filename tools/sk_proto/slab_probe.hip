// Write-pattern probe for a two-pass count (DESIGN §3 "two-pass prototype"): can one pass scatter
// every instance straight into 4096 fine buckets fast enough to replace kc_bin1's region write plus
// kc_rebin's round trip?  Each workgroup owns a slab of S u32 per fine bucket and appends, per tile,
// the tile's run for every bucket (TILE / 4096 elements on average).  Timed against a plain
// contiguous write of the same bytes.  Stand-alone: hipcc --offload-arch=gfx950 -O3 slab_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int NB = 4096;

// tile of TILE elements: run length c = TILE / NB per bucket; element j of the tile goes to bucket
// j / c, position fill[b] + j % c of the workgroup's slab (lanes on consecutive elements)
template <int NT, bool NTS>
__global__ void __launch_bounds__(NT) slab_write(uint32_t* __restrict__ out, uint64_t per_wg, uint32_t tile,
                                                 uint32_t S) {
    __shared__ uint16_t fill[NB];
    const uint32_t w = blockIdx.x;
    for (int b = threadIdx.x; b < NB; b += NT) fill[b] = 0;
    __syncthreads();
    const uint32_t c = tile / NB;
    uint32_t* __restrict__ slab = out + (uint64_t)w * NB * S;
    for (uint64_t t0 = 0; t0 < per_wg; t0 += tile) {
        for (uint32_t j = threadIdx.x; j < tile; j += NT) {
            const uint32_t b = j / c, p = j - b * c;
            const uint32_t f = fill[b] + p;
            if (f < S) {
                if (NTS) __builtin_nontemporal_store((uint32_t)(t0 + j), &slab[(uint64_t)b * S + f]);
                else slab[(uint64_t)b * S + f] = (uint32_t)(t0 + j);
            }
        }
        __syncthreads();
        for (int b = threadIdx.x; b < NB; b += NT) fill[b] = (uint16_t)(fill[b] + c);
        __syncthreads();
    }
}

__global__ void __launch_bounds__(256) flat_write(uint32_t* __restrict__ out, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        out[i] = (uint32_t)i;
}

int main() {
    const uint64_t N = 256ull << 20;   // C2: ~256 M instances
    const uint32_t W = 512;
    const uint64_t per_wg = N / W;
    const uint32_t S = 320;            // slab capacity per (workgroup, bucket): 2.6x the mean of 128
    uint32_t* out;
    CK(hipMalloc(&out, (uint64_t)2 * W * NB * S * 4));   // the 2W-workgroup variant too
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto launch) -> float {
        for (int i = 0; i < 3; ++i) launch();
        (void)hipEventRecord(e0);
        for (int i = 0; i < 10; ++i) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return ms / 10;
    };
    printf("flat write %.3f ms (%.2f GB)\n", timeit([&] { hipLaunchKernelGGL(flat_write, dim3(4096), dim3(256), 0, 0, out, N); }),
           N * 4 / 1e9);
    for (uint32_t tile : {8192u, 16384u, 32768u, 65536u}) {
        const float ms = timeit([&] { hipLaunchKernelGGL((slab_write<512, false>), dim3(W), dim3(512), 0, 0, out, per_wg, tile, S); });
        const float ms2 = timeit([&] { hipLaunchKernelGGL((slab_write<1024, false>), dim3(W), dim3(1024), 0, 0, out, per_wg, tile, S); });
        const float ms3 = timeit([&] { hipLaunchKernelGGL((slab_write<512, true>), dim3(W), dim3(512), 0, 0, out, per_wg, tile, S); });
        const float ms4 = timeit([&] { hipLaunchKernelGGL((slab_write<512, false>), dim3(2 * W), dim3(512), 0, 0, out, per_wg / 2, tile, S); });
        printf("slab tile %6u run %3u B: %.3f ms (512 thr)  %.3f (1024 thr)  %.3f (nt stores)  %.3f (1024 wg)\n", tile, tile / NB * 4, ms, ms2, ms3, ms4);
    }
    CK(hipFree(out));
    return 0;
}
