// fp4_mfma_probe.hip -- checks the gfx950 fp4 (e2m1) block-scaled MFMA
// v_mfma_scale_f32_32x32x64_f8f6f4 as a {0,1} matrix product, which the MFMA carry chain relies on:
//   (1) lane l holds A row l%32 and B column l%32; the K elements of lane l are the same set for
//       A and B, element e of lane half h pairing with element e of lane half h:
//         C[m][n] = sum_{h,e} A[m+32h][e] * B[n+32h][e]
//   (2) C/D: col = l&31, row = (reg&3) + 8(reg>>2) + 4(l>>5)
//   (3) fp4 reads only the low 4 VGPRs of each operand (garbage in the upper 4)
//   (4) throughput: cycles per MFMA with 1/2/4 independent accumulators, and with one
//       ds_read_b128 B operand per MFMA.
// build: hipcc --offload-arch=gfx950 -O3 tools/fp4_mfma_probe.hip -o tools/fp4_mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void layout_kernel(const uint32_t *a, const uint32_t *b, float *out) {
    v8i A, B;
    v16f C = {};
    for (int i = 0; i < 8; ++i) {
        A[i] = (int)a[threadIdx.x * 8 + i];
        B[i] = (int)b[threadIdx.x * 8 + i];
    }
    C = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, C, 4, 4, 0, 127, 0, 127);
    for (int i = 0; i < 16; ++i) out[threadIdx.x * 16 + i] = C[i];
}

template <int NACC, bool LDSB>
__global__ void rate_kernel(const uint32_t *a, float *out, int iters, long long *clk) {
    __shared__ uint32_t lds[64 * 4 * 16];
    v8i A, B;
    for (int i = 0; i < 8; ++i) A[i] = (int)a[threadIdx.x % 64 * 8 + i], B[i] = A[i] ^ 0x22222222;
    for (int i = threadIdx.x; i < 64 * 4 * 16; i += blockDim.x) lds[i] = a[i % 512];
    __syncthreads();
    v16f C[NACC];
    for (int j = 0; j < NACC; ++j) C[j] = (v16f){};
    long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < NACC; ++j) {
            if (LDSB) {
                const uint4 v = *(const uint4 *)&lds[((threadIdx.x & 63) * 4 + ((it * NACC + j) & 15) * 256) & 4095];
                B[0] = v.x, B[1] = v.y, B[2] = v.z, B[3] = v.w;
            }
            C[j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, C[j], 4, 4, 0, 127, 0, 127);
        }
    }
    long long t1 = clock64();
    float s = 0;
    for (int j = 0; j < NACC; ++j)
        for (int i = 0; i < 16; ++i) s += C[j][i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) *clk = t1 - t0;
}

int main() {
    srand(7);
    const int n = 64 * 8;
    std::vector<uint32_t> ha(n), hb(n);
    // random bits -> fp4 1.0 (0b0010) or 0 in the low 4 VGPRs; garbage in VGPRs 4..7
    for (int l = 0; l < 64; ++l)
        for (int v = 0; v < 8; ++v) {
            uint32_t wa = 0, wb = 0;
            for (int e = 0; e < 8; ++e) {
                if (rand() & 1) wa |= 2u << (4 * e);
                if (rand() & 1) wb |= 2u << (4 * e);
            }
            ha[l * 8 + v] = v < 4 ? wa : (uint32_t)rand();
            hb[l * 8 + v] = v < 4 ? wb : (uint32_t)rand();
        }
    uint32_t *da, *db;
    float *dout;
    long long *dclk;
    hipMalloc(&da, n * 4);
    hipMalloc(&db, n * 4);
    hipMalloc(&dout, 1 << 22);
    hipMalloc(&dclk, 8);
    hipMemcpy(da, ha.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, hb.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(layout_kernel, dim3(1), dim3(64), 0, 0, da, db, dout);
    std::vector<float> hc(64 * 16);
    hipMemcpy(hc.data(), dout, 64 * 16 * 4, hipMemcpyDeviceToHost);
    auto elem = [](const std::vector<uint32_t> &x, int lane, int e) { return (x[lane * 8 + e / 8] >> (4 * (e % 8))) & 0xF ? 1 : 0; };
    int bad = 0, nz = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r) {
            const int col = l & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
            int ref = 0;
            for (int h = 0; h < 2; ++h)
                for (int e = 0; e < 32; ++e) ref += elem(ha, row + 32 * h, e) * elem(hb, col + 32 * h, e);
            if ((float)ref != hc[l * 16 + r]) ++bad;
            nz += ref != 0;
        }
    printf("layout: mismatches %d of 1024 (nonzero refs %d)\n", bad, nz);

    int dev_clk_khz = 0;
    hipDeviceGetAttribute(&dev_clk_khz, hipDeviceAttributeClockRate, 0);
    const int iters = 2000;
    auto run = [&](auto kern, const char *name, int nacc, int waves_per_simd) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        const int blocks = 256 * waves_per_simd; // one 256-thread block = 4 waves = one per SIMD
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, da, dout, iters, dclk);
        hipEventRecord(e0);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, da, dout, iters, dclk);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        long long clk;
        hipMemcpy(&clk, dclk, 8, hipMemcpyDeviceToHost);
        const double mfma_per_simd = (double)iters * nacc * waves_per_simd;
        printf("%-10s nacc=%d waves/SIMD=%d  %.3f ms  wave0 %.1f clk/mfma  chip %.1f ns per mfma per SIMD  %.2f PF(MAC*2)\n", name,
               nacc, waves_per_simd, ms, (double)clk / (iters * nacc), ms * 1e6 / mfma_per_simd,
               2.0 * 65536 * mfma_per_simd * 1024 / (ms * 1e-3) / 1e15);
    };
    run(rate_kernel<1, false>, "reg", 1, 1);
    run(rate_kernel<2, false>, "reg", 2, 1);
    run(rate_kernel<4, false>, "reg", 4, 1);
    run(rate_kernel<1, false>, "reg", 1, 2);
    run(rate_kernel<2, false>, "reg", 2, 2);
    run(rate_kernel<1, true>, "ldsB", 1, 1);
    run(rate_kernel<2, true>, "ldsB", 2, 1);
    run(rate_kernel<4, true>, "ldsB", 4, 1);
    run(rate_kernel<2, true>, "ldsB", 2, 2);
    run(rate_kernel<2, true>, "ldsB", 2, 4);
    printf("clock attr %d kHz\n", dev_clk_khz);
    return bad ? 1 : 0;
}
