// Probe: event-record nodes inside a stream capture (timing kernels inside a replayed graph).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void spin(float *x, int n) {
    float v = x[threadIdx.x];
    for (int i = 0; i < n; ++i) v = v * 1.0000001f + 1e-7f;
    x[threadIdx.x] = v;
}
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s -> %d %s\n", #x, (int)e_, hipGetErrorString(e_)); } } while (0)
int main() {
    float *x; CK(hipMalloc(&x, 4096));
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e[4]; for (auto &v : e) CK(hipEventCreate(&v));
    for (int mode = 0; mode < 3; ++mode) {
        printf("capture mode %d\n", mode);
        hipGraph_t g = nullptr; hipGraphExec_t ge = nullptr;
        CK(hipStreamBeginCapture(s, (hipStreamCaptureMode)mode));
        spin<<<1, 64, 0, s>>>(x, 1000);
        CK(hipEventRecordWithFlags(e[0], s, hipEventRecordExternal));
        spin<<<1, 64, 0, s>>>(x, 200000);
        CK(hipEventRecordWithFlags(e[1], s, hipEventRecordExternal));
        spin<<<1, 64, 0, s>>>(x, 1000);
        CK(hipStreamEndCapture(s, &g));
        if (!g) continue;
        size_t nn = 0; CK(hipGraphGetNodes(g, nullptr, &nn)); printf(" nodes %zu\n", nn);
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int r = 0; r < 3; ++r) {
            CK(hipGraphLaunch(ge, s)); CK(hipStreamSynchronize(s));
            float ms = -1; CK(hipEventElapsedTime(&ms, e[0], e[1])); printf(" replay %d: %.4f ms\n", r, ms);
        }
        CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
    // manual node: capture info + add node + update deps
    {
        printf("manual node\n");
        hipGraph_t g = nullptr; hipGraphExec_t ge = nullptr;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        spin<<<1, 64, 0, s>>>(x, 1000);
        for (int k = 0; k < 2; ++k) {
            hipStreamCaptureStatus st; unsigned long long id; hipGraph_t cg; const hipGraphNode_t *deps; size_t nd;
            CK(hipStreamGetCaptureInfo_v2(s, &st, &id, &cg, &deps, &nd));
            hipGraphNode_t node;
            CK(hipGraphAddEventRecordNode(&node, cg, deps, nd, e[2 + k]));
            CK(hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies));
            if (k == 0) spin<<<1, 64, 0, s>>>(x, 200000);
        }
        spin<<<1, 64, 0, s>>>(x, 1000);
        CK(hipStreamEndCapture(s, &g));
        size_t nn = 0; CK(hipGraphGetNodes(g, nullptr, &nn)); printf(" nodes %zu\n", nn);
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int r = 0; r < 3; ++r) {
            CK(hipGraphLaunch(ge, s)); CK(hipStreamSynchronize(s));
            float ms = -1; CK(hipEventElapsedTime(&ms, e[2], e[3])); printf(" replay %d: %.4f ms\n", r, ms);
        }
    }
    // direct reference
    spin<<<1, 64, 0, s>>>(x, 1000);
    CK(hipEventRecord(e[0], s)); spin<<<1, 64, 0, s>>>(x, 200000); CK(hipEventRecord(e[1], s));
    CK(hipStreamSynchronize(s)); float ms; CK(hipEventElapsedTime(&ms, e[0], e[1])); printf("direct: %.4f ms\n", ms);
    return 0;
}
