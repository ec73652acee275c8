// mfma_dep_ubench.hip -- issue cost of v_mfma_scale_f32_32x32x64_f8f6f4 (fp4) in a dependent chain
// (every MFMA accumulates into the previous one's result, as the adder chain's tiles do) versus
// NACC independent accumulators interleaved, at 1..8 waves per SIMD.  Prints SIMD-clocks per MFMA
// (s_memtime ticks are the 100 MHz constant clock; the kernel also reports the launch time, from
// which the per-MFMA time in ns follows).
// build: hipcc --offload-arch=gfx950 -O3 tools/mfma_dep_ubench.hip -o tools/mfma_dep_ubench
#include <hip/hip_runtime.h>

#include <cstdio>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ v16f mf(const v8i &a, const v8i &b, const v16f &c) {
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 4, 4, 0, 127, 0, 127);
}

template <int NACC>
__global__ void __launch_bounds__(512) chain(float *out, int iters, int seed) {
    const int l = threadIdx.x & 63;
    v8i a = {l * seed, l + seed, l ^ seed, l, 0, 0, 0, 0};
    v8i b = {l + 1, l * 3, l ^ 5, seed, 0, 0, 0, 0};
    v16f acc[NACC];
#pragma unroll
    for (int k = 0; k < NACC; ++k)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[k][j] = (float)(j + k);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < 12; c += NACC)
#pragma unroll
            for (int k = 0; k < NACC; ++k) acc[k] = mf(a, b, acc[k]);
        asm volatile("" : "+v"(a));
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NACC; ++k)
#pragma unroll
        for (int j = 0; j < 16; ++j) s += acc[k][j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
static void run(int wps, float *d) {
    // one block per CU of wps*4 waves: wps waves per SIMD, 256 CUs
    const int iters = 2000, blocks = 256, threads = 64 * 4 * wps;
    hipEvent_t e0, e1;
    hipEventCreate(&e0), hipEventCreate(&e1);
    chain<NACC><<<blocks, threads>>>(d, 10, 3);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    chain<NACC><<<blocks, threads>>>(d, iters, 3);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double mfma_per_simd = 12.0 * iters * wps;
    printf("NACC=%d waves/SIMD=%d: %.3f ms, %.2f ns per MFMA per SIMD (%.1f clk at 2.4 GHz)\n", NACC, wps,
           ms, ms * 1e6 / mfma_per_simd, ms * 1e6 / mfma_per_simd * 2.4);
}

int main() {
    float *d;
    hipMalloc(&d, 256 * 512 * 4);
    for (int w : {1, 2, 4}) {
        run<1>(w, d);
        run<2>(w, d);
        run<4>(w, d);
    }
    hipFree(d);
    return 0;
}
