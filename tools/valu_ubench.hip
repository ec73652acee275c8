// Micro-benchmark: VALU/SALU issue throughput of the integer ops the engine is built from (gfx950).
// 8 independent chains per lane of one inline-asm instruction each; reports wave-instr per CU per ns.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#define ITERS 2048
#define CHAINS 8
template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t *out, uint32_t seed) {
    uint32_t a[CHAINS], b = seed ^ threadIdx.x, c = seed * 3u + threadIdx.x;
    uint32_t s = seed;
#pragma unroll
    for (int j = 0; j < CHAINS; ++j) a[j] = seed + j * 77u + threadIdx.x;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int j = 0; j < CHAINS; ++j) {
            if (OP == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
            if (OP == 1) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[j]) : "v"(c));
            if (OP == 2) asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0x6c" : "+v"(a[j]) : "v"(b), "v"(c));
            if (OP == 3) asm volatile("v_bfe_i32 %0, %0, 7, 1" : "+v"(a[j]));
            if (OP == 4) asm volatile("s_bitcmp1_b32 %0, 3\n\ts_cbranch_scc1 1f\n\ts_nop 0\n1:" :: "s"(s));
            if (OP == 5) asm volatile("v_xor_b32 %0, %0, %1\n\ts_bitcmp1_b32 %2, 3\n\ts_cbranch_scc0 1f\n1:" : "+v"(a[j]) : "v"(b), "s"(s));
        }
    }
    uint32_t r = s;
#pragma unroll
    for (int j = 0; j < CHAINS; ++j) r ^= a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int OP>
void run(const char *name, int waves_per_simd) {
    uint32_t *out;
    int blocks = 256 * waves_per_simd; // 256 threads = 4 waves = one per SIMD of one CU
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 1u);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0), (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 2u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    double winstr = (double)blocks * 4 * ITERS * CHAINS;
    printf("%-12s waves/SIMD=%d  %.3f ms  %.3f wave-ops per CU per ns (per-op groups)\n", name,
           waves_per_simd, ms, winstr / ms / 1e6 / 256);
    (void)hipFree(out);
}
int main() {
    for (int w : {1, 2, 4, 8}) {
        run<0>("xor", w);
        run<1>("alignbit", w);
        run<2>("bitop3", w);
        run<3>("bfe", w);
        run<4>("bitcmp+br", w);
        run<5>("xor+cmp+br", w);
    }
    return 0;
}
