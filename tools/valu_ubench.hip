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
    uint64_t aa[CHAINS];
    uint32_t k31 = 31u + (seed >> 30), k7 = 7u + (seed >> 30), k1 = 1u + (seed >> 30);
#pragma unroll
    for (int j = 0; j < CHAINS; ++j) aa[j] = seed + j * 7ull + threadIdx.x;
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
            if (OP == 6) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a[j]) : "s"(s));
            if (OP == 7) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x6c" : "+v"(a[j]) : "v"(b), "s"(s));
            if (OP == 8) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[j]) : "v"(b), "v"(c));
            if (OP == 9) asm volatile("v_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(a[j]) :: "vcc");
            if (OP == 10) asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(a[j]) : "v"(b));
            if (OP == 11) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(a[j]));
            if (OP == 12) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
            if (OP == 13) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(aa[j]));
            if (OP == 16) asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(c), "v"(k31));
            if (OP == 17) asm volatile("v_bfe_i32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(k7), "v"(k1));
            if (OP == 18) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a[j]) : "v"(k1));
            if (OP == 19) asm volatile("v_xor_b32 %0, 1, %0" : "+v"(a[j]));
            if (OP == 20) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[j]) : "v"(a[(j + 1) % CHAINS]));
            if (OP == 21) asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(a[(j + 1) % CHAINS]), "v"(k31));
            if (OP == 22) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(aa[j]) : "v"(a[j]), "v"(b) : "vcc");
            if (OP == 23) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
            if (OP == 24) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
            if (OP == 25) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[j]) : "v"(b));
            if (OP == 26) asm volatile("v_and_b32 %0, 0x11111111, %0" : "+v"(a[j]));
            if (OP == 27) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(aa[j]) : "v"(a[j]), "v"(b) : "vcc");
            if (OP == 15) asm volatile("v_xor_b32 %0, %0, %1 row_shr:1 bound_ctrl:0" : "+v"(a[j]) : "v"(b));
            if (OP == 14) asm volatile("v_pk_mov_b32 %0, %1, %0 op_sel:[1,0]" : "+v"(aa[j]) : "v"(aa[(j + 1) % CHAINS]));
            if (OP == 28) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
            if (OP == 29) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
            if (OP == 32) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "s"(s));
            if (OP == 30) asm volatile("v_lshlrev_b32 %0, 1, %0\n\tv_xor_b32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
            if (OP == 31) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a[j]), "+v"(c));
        }
    }
    uint32_t r = s;
#pragma unroll
    for (int j = 0; j < CHAINS; ++j) r ^= a[j] ^ (uint32_t)aa[j];
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
    for (int w : {4, 8}) {
        run<22>("mad_u64", w);
        run<27>("mad_u64_acc", w);
        run<23>("mul_lo", w);
        run<24>("mul_hi", w);
        run<25>("mul_u24", w);
        run<26>("and_lit", w);
        run<16>("alignbit_vvv", w);
        run<17>("bfe_vvv", w);
        run<18>("lshl_vv", w);
        run<19>("xor_const", w);
        run<20>("xor_vv_dep", w);
        run<21>("alignbit_vvv_dep", w);
        run<0>("xor", w);
        run<1>("alignbit", w);
        run<2>("bitop3", w);
        run<3>("bfe", w);
        run<4>("bitcmp+br", w);
        run<5>("xor+cmp+br", w);
        run<6>("xor_vs", w);
        run<7>("bitop3_vvs", w);
        run<8>("bitop3_xor3", w);
        run<9>("addc", w);
        run<10>("lshl_or", w);
        run<11>("lshl", w);
        run<12>("and", w);
        run<13>("lshl_b64", w);
        run<14>("pk_mov", w);
        run<15>("xor_dpp", w);
        run<28>("perm", w);
        run<32>("perm_vvs", w);
        run<29>("and_or", w);
        run<30>("lshl+xor", w);
        run<31>("permlane32_swap", w);
    }
    return 0;
}
