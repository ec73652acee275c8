// chain_check.hip -- standalone check of the MFMA carry chain (homomorph-rust_amd/csrc/adder_mfma.hip)
// against a CPU carry-less chain on a synthetic prep workspace:
//   carry_0 = 0;  s_i = x_i ^ carry_i;  carry_{i+1} = ab_i ^ P_i * carry_i
// Modes: random words, or single set bits (localises index errors).  Prints the first mismatching
// output words.  build: hipcc --offload-arch=gfx950 -O3 -I homomorph-rust_amd/csrc \
//   tools/chain_check.hip -o tools/chain_check
#ifndef HM_NO_PROFILE // -DHM_NO_PROFILE: the library's kernel exactly (no phase timers)
#define HM_MFMA_PROFILE 1
#endif
#include "../homomorph-rust_amd/csrc/adder_mfma.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

using namespace hm;

static std::vector<uint32_t> clmul(const std::vector<uint32_t> &a, const std::vector<uint32_t> &b) {
    std::vector<uint32_t> r(a.size() + b.size() + 1, 0u);
    for (size_t i = 0; i < a.size() * 32; ++i)
        if ((a[i / 32] >> (i % 32)) & 1u)
            for (size_t j = 0; j < b.size() * 32; ++j)
                if ((b[j / 32] >> (j % 32)) & 1u) r[(i + j) / 32] ^= 1u << ((i + j) % 32);
    return r;
}
static int degp1(const uint32_t *w, int n) {
    for (int k = n - 1; k >= 0; --k)
        if (w[k]) return k * 32 + 32 - __builtin_clz(w[k]);
    return 0;
}

static int run_case(int L, int npw, int abw, int mode, int pbit, int cbit, bool quiet);

static int timing(int nvals, bool wide);

int main(int argc, char **argv) {
    if (argc > 1 && !strcmp(argv[1], "time")) return timing(argc > 2 ? atoi(argv[2]) : 4096, false);
    if (argc > 1 && !strcmp(argv[1], "time25")) return timing(argc > 2 ? atoi(argv[2]) : 131072, true);
    if (argc > 1 && (!strcmp(argv[1], "sweep") || !strcmp(argv[1], "sweep25"))) {
        // single set bits of P_1 and carry_1 at chosen positions (NC = 13: P of 24 words;
        // sweep25: NC = 25, P of 49 words, ab of 33)
        const bool w = !strcmp(argv[1], "sweep25");
        const int ps13[] = {0, 5, 31, 32, 100, 400, 650, 700, 736, 767};
        const int ps25[] = {0, 5, 31, 32, 100, 700, 800, 1100, 1500, 1567};
        const int cs[] = {0, 7, 31, 32, 100, 300, 480, 511};
        const int *ps = w ? ps25 : ps13;
        int nbad = 0;
        for (int q = 0; q < 10; ++q)
            for (int cb : cs)
                if (const int pb = ps[q]; run_case(3, w ? 49 : 24, w ? 33 : 16, 1, pb, cb, true)) {
                    const int o = pb + cb;
                    printf("FAIL p=%d c=%d -> out bit %d (W=%d m=%d, cword=%d, pword=%d)\n", pb, cb, o, o / 32, o % 32, cb / 32, pb / 32);
                    ++nbad;
                }
        printf("sweep: %d failing cases\n", nbad);
        return 0;
    }
    const int L = argc > 1 ? atoi(argv[1]) : 4;          // bits
    const int npw = argc > 2 ? atoi(argv[2]) : 24;       // P words
    const int abw = argc > 3 ? atoi(argv[3]) : 16;       // ab words
    const int mode = argc > 4 ? atoi(argv[4]) : 0;       // 0 random, 1 single bits
    const int pbit = argc > 5 ? atoi(argv[5]) : 0, cbit = argc > 6 ? atoi(argv[6]) : 0;
    return run_case(L, npw, abw, mode, pbit, cbit, false) ? 1 : 0;
}

static int run_case(int L, int npw, int abw, int mode, int pbit, int cbit, bool quiet) {
    std::mt19937_64 rng(5);
    const uint32_t cntAB = abw, cntP = npw, cntX = 9;
    std::vector<std::vector<uint32_t>> P(L), AB(L), X(L);
    for (int i = 0; i < L; ++i) {
        P[i].assign(cntP, 0u), AB[i].assign(cntAB, 0u), X[i].assign(cntX, 0u);
        if (mode == 0) {
            for (auto &w : P[i]) w = (uint32_t)rng();
            for (auto &w : AB[i]) w = (uint32_t)rng();
            for (auto &w : X[i]) w = (uint32_t)rng();
        } else {
            P[i][pbit / 32] = 1u << (pbit % 32);
            if (i == 0) AB[i][cbit / 32] = 1u << (cbit % 32);
        }
    }
    // CPU chain
    std::vector<std::vector<uint32_t>> S(L);
    std::vector<uint32_t> carry;
    size_t maxw = 0;
    for (int i = 0; i < L; ++i) {
        S[i] = carry;
        if (S[i].size() < cntX) S[i].resize(cntX, 0u);
        for (uint32_t k = 0; k < cntX; ++k) S[i][k] ^= X[i][k];
        maxw = std::max(maxw, S[i].size());
        auto pr = clmul(P[i], carry);
        pr.resize(std::max(pr.size(), (size_t)cntAB), 0u);
        for (uint32_t k = 0; k < cntAB; ++k) pr[k] ^= AB[i][k];
        carry = pr;
    }
    // workspace
    AddArgs A{};
    A.n = 1, A.nbits = L, A.cntAB = cntAB, A.cntP = cntP, A.cntX = cntX;
    A.ws_stride = (uint64_t)L * (cntAB + cntP + 2 + cntX);
    std::vector<uint32_t> ws(A.ws_stride, 0u);
    for (int i = 0; i < L; ++i) {
        memcpy(&ws[i * cntAB], AB[i].data(), cntAB * 4);
        memcpy(&ws[L * cntAB + i * cntP], P[i].data(), cntP * 4);
        ws[L * (cntAB + cntP) + i] = degp1(AB[i].data(), cntAB);
        ws[L * (cntAB + cntP) + L + i] = degp1(P[i].data(), cntP);
        memcpy(&ws[L * (cntAB + cntP + 2) + i * cntX], X[i].data(), cntX * 4);
    }
    uint32_t outcap = (uint32_t)((maxw * 32 + 63) / 64 + 1);
    for (int i = 0; i < L; ++i) A.ob.b[i] = outcap * 64 - 1;
    A.out.stride = (uint64_t)outcap * L;
    const uint32_t tiles = (uint32_t)((maxw + 31) / 32) + 1;
    A.mf_cw = 32 * tiles + 64;
    A.mfma = npw <= 25 ? 13 : 25;
    A.chain_lds = (A.mfma == 13 ? MfmaCfg<13>::kHalo + MfmaCfg<13>::kRsWords + MfmaCfg<13>::kRingWords
                                : MfmaCfg<25>::kHalo + MfmaCfg<25>::kRsWords + MfmaCfg<25>::kRingWords) +
                  A.mf_cw;
    uint32_t *dws;
    uint64_t *dout;
    uint32_t *ddeg;
    int *dst;
    hipMalloc(&dws, ws.size() * 4);
    hipMalloc(&dout, A.out.stride * 8);
    hipMalloc(&ddeg, L * 4);
    hipMalloc(&dst, 4);
    hipMemcpy(dws, ws.data(), ws.size() * 4, hipMemcpyHostToDevice);
    hipMemset(dout, 0xA5, A.out.stride * 8); // every output word must be written
    hipMemset(dst, 0, 4);
    A.ws = dws, A.out.limbs = dout, A.out.degree = ddeg, A.status = dst;
#ifdef HM_MFMA_PROFILE
    static unsigned long long *dprof1 = nullptr;
    if (!dprof1) {
        hipMalloc(&dprof1, 64);
        hipMemcpyToSymbol(HIP_SYMBOL(g_mfma_prof), &dprof1, sizeof dprof1);
    }
#endif
    if (launch_add_chain_mfma(A, nullptr)) { printf("launch failed\n"); return 2; }
    hipDeviceSynchronize();
    std::vector<uint64_t> out(A.out.stride);
    hipMemcpy(out.data(), dout, out.size() * 8, hipMemcpyDeviceToHost);
    int st;
    hipMemcpy(&st, dst, 4, hipMemcpyDeviceToHost);
    std::vector<uint32_t> gdeg(L);
    hipMemcpy(gdeg.data(), ddeg, L * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < L; ++i) {
        const int dp1 = degp1(S[i].data(), (int)S[i].size());
        const uint32_t want = dp1 ? (uint32_t)(dp1 - 1) : 0u;
        if (gdeg[i] != want) {
            ++bad;
            if (!quiet) printf("bit %d degree: gpu %u ref %u\n", i, gdeg[i], want);
        }
        const uint32_t *g = (const uint32_t *)&out[(size_t)i * outcap];
        int shown = 0;
        for (size_t k = 0; k < 2 * outcap; ++k) {
            const uint32_t ref = k < S[i].size() ? S[i][k] : 0u;
            if (g[k] != ref) {
                ++bad;
                if (!quiet && shown++ < 6) printf("bit %d word %zu: gpu %08x ref %08x\n", i, k, g[k], ref);
            }
        }
    }
    if (!quiet)
        printf("L=%d np=%d ab=%d mode=%d pbit=%d cbit=%d: %d mismatching words, status %d\n", L, npw,
               abw, mode, pbit, cbit, bad, st);
    hipFree(dws), hipFree(dout), hipFree(ddeg), hipFree(dst);
    return bad;
}

// configs[1]-shaped chain (32 bits, P 25 words, ab 17 words, x 9 words; wide: configs[4]'s,
// P 49, ab 33, x 17) replicated over nvals values: kernel time and per-phase s_memtime sums
// (cycles summed over waves)
static int timing(int nvals, bool wide) {
    const int L = 32;
    const uint32_t cntAB = wide ? 33 : 17, cntP = wide ? 49 : 25, cntX = wide ? 17 : 9;
    const uint32_t D = wide ? 512 : 256;
    std::mt19937_64 rng(11);
    AddArgs A{};
    A.n = (uint64_t)nvals, A.nbits = L, A.cntAB = cntAB, A.cntP = cntP, A.cntX = cntX;
    A.ws_stride = ((uint64_t)L * (cntAB + cntP + 2 + cntX) + 63) & ~(uint64_t)63;
    std::vector<uint32_t> ws(A.ws_stride * nvals, 0u);
    for (int v = 0; v < nvals; ++v) {
        uint32_t *w = &ws[(size_t)v * A.ws_stride];
        for (int i = 0; i < L; ++i) {
            for (uint32_t k = 0; k < cntAB; ++k) w[i * cntAB + k] = (uint32_t)rng();
            w[i * cntAB + cntAB - 1] &= 0x7FFFFFFFu;
            for (uint32_t k = 0; k < cntP; ++k) w[L * cntAB + i * cntP + k] = k + 1 < cntP ? (uint32_t)rng() : 1u;
            w[L * (cntAB + cntP) + i] = degp1(&w[i * cntAB], cntAB);
            w[L * (cntAB + cntP) + L + i] = degp1(&w[L * cntAB + i * cntP], cntP);
            for (uint32_t k = 0; k < cntX; ++k) w[L * (cntAB + cntP + 2) + i * cntX + k] = (uint32_t)rng() & (k + 1 < cntX ? ~0u : 1u);
        }
    }
    const uint32_t maxw = (cntP - 1) * (L - 1) + cntP; // the host plan's SC (carry_31 + P words)
    // the add's output bounds (hm_add_out_bounds): s_0 <= D, s_i <= (3i-1) D
    uint64_t stride = 0;
    for (int i = 0; i < L; ++i) {
        A.ob.b[i] = i == 0 ? D : (uint32_t)(3 * i - 1) * D;
        stride += A.ob.b[i] / 64 + 1;
    }
    A.out.stride = stride;
    const uint32_t tiles = (maxw + 31) / 32;
    A.mf_cw = 32 * tiles + 64;
    A.mfma = wide ? 25 : 13;
    A.chain_lds = (wide ? MfmaCfg<25>::kHalo + MfmaCfg<25>::kRsWords + MfmaCfg<25>::kRingWords
                        : MfmaCfg<13>::kHalo + MfmaCfg<13>::kRsWords + MfmaCfg<13>::kRingWords) +
                  A.mf_cw;
    uint32_t *dws, *ddeg;
    uint64_t *dout;
    int *dst;
    hipMalloc(&dws, ws.size() * 4);
    hipMalloc(&dout, A.out.stride * 8 * nvals);
    hipMalloc(&ddeg, (size_t)L * 4 * nvals);
    hipMalloc(&dst, 4);
    hipMemcpy(dws, ws.data(), ws.size() * 4, hipMemcpyHostToDevice);
    hipMemset(dst, 0, 4);
    A.ws = dws, A.out.limbs = dout, A.out.degree = ddeg, A.status = dst;
    hipEvent_t e0, e1;
    hipEventCreate(&e0), hipEventCreate(&e1);
#ifdef HM_MFMA_PROFILE
    unsigned long long *dprof;
    hipMalloc(&dprof, (size_t)nvals * 4 * 8);
    hipMemcpyToSymbol(HIP_SYMBOL(g_mfma_prof), &dprof, sizeof dprof);
#endif
    // ~0.3 s of launches first: the clock ramps up under load (MI355X_MICROARCH.md DVFS)
    for (int r = 0; r < (wide ? 20 : 300); ++r) launch_add_chain_mfma(A, nullptr);
    hipDeviceSynchronize();
    const int reps = wide ? 5 : 50;
    float ms = 0.f;
    if (getenv("HM_CC_HOT")) {
        // as in the engine, where add_prep_kernel writes the workspace right before the chain:
        // the workspace is rewritten (device copy) before each launch, chain launches timed alone
        uint32_t *dws2;
        hipMalloc(&dws2, ws.size() * 4);
        hipMemcpy(dws2, dws, ws.size() * 4, hipMemcpyDeviceToDevice);
        std::vector<hipEvent_t> ev(2 * reps);
        for (auto &x : ev) hipEventCreate(&x);
        for (int r = 0; r < reps; ++r) {
            hipMemcpyAsync(dws, dws2, ws.size() * 4, hipMemcpyDeviceToDevice, nullptr);
            hipEventRecord(ev[2 * r]);
            launch_add_chain_mfma(A, nullptr);
            hipEventRecord(ev[2 * r + 1]);
        }
        hipDeviceSynchronize();
        for (int r = 0; r < reps; ++r) {
            float t;
            hipEventElapsedTime(&t, ev[2 * r], ev[2 * r + 1]);
            ms += t;
        }
        printf("(workspace rewritten before each launch) ");
    } else {
        hipEventRecord(e0);
        for (int r = 0; r < reps; ++r) launch_add_chain_mfma(A, nullptr);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
    }
#ifdef HM_MFMA_PROFILE
    std::vector<unsigned long long> hp((size_t)nvals * 4);
    hipMemcpy(hp.data(), dprof, hp.size() * 8, hipMemcpyDeviceToHost);
    double z[4] = {0, 0, 0, 0};
    for (int v = 0; v < nvals; ++v)
        for (int k = 0; k < 4; ++k) z[k] += (double)hp[(size_t)v * 4 + k];
    const double waves = (double)nvals; // the last launch's per-wave sums
    printf("chain %d values: %.1f us per launch; per wave (s_memtime ticks): sum-store %.0f, RS+A build %.0f, tiles %.0f, vmcnt wait %.0f\n",
           nvals, ms * 1e3 / reps, z[0] / waves, z[1] / waves, z[2] / waves, z[3] / waves);
#else
    printf("chain %d values: %.1f us per launch\n", nvals, ms * 1e3 / reps);
#endif
    return 0;
}
