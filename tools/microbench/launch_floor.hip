// Per-kernel cost floor on this GPU: a chain of K dependent empty/tiny kernels,
// eager and HIP-graph replayed, 1 and 256 workgroups.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
__global__ void tiny(int* p) { if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1; }
#define CK(x) do { hipError_t e = (x); if (e) { printf("err %d line %d\n", e, __LINE__); return 1; } } while (0)
int main() {
    int* d; CK(hipMalloc(&d, 4));
    hipStream_t s; CK(hipStreamCreate(&s));
    const int K = 200;
    for (int blocks : {1, 256, 2048}) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipStreamSynchronize(s));
            auto t0 = std::chrono::high_resolution_clock::now();
            for (int i = 0; i < K; ++i) hipLaunchKernelGGL(tiny, dim3(blocks), dim3(256), 0, s, d);
            CK(hipStreamSynchronize(s));
            auto t1 = std::chrono::high_resolution_clock::now();
            if (rep) printf("eager  blocks=%5d  %.2f us/kernel\n", blocks, std::chrono::duration<double, std::micro>(t1 - t0).count() / K);
        }
        hipGraph_t g; hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int i = 0; i < K; ++i) hipLaunchKernelGGL(tiny, dim3(blocks), dim3(256), 0, s, d);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipStreamSynchronize(s));
            auto t0 = std::chrono::high_resolution_clock::now();
            CK(hipGraphLaunch(ge, s));
            CK(hipStreamSynchronize(s));
            auto t1 = std::chrono::high_resolution_clock::now();
            if (rep) printf("graph  blocks=%5d  %.2f us/kernel\n", blocks, std::chrono::duration<double, std::micro>(t1 - t0).count() / K);
        }
        CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
    return 0;
}
