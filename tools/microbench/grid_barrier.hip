// Phase boundary cost on gfx950: what a persistent "one kernel per inner
// step" engine would pay per phase (a grid-wide barrier) against what the
// captured window pays now (a dependent kernel launch inside a HIP graph).
//
//   graph:   K dependent launches of a G-block kernel, replayed from one graph;
//   barrier: one cooperative launch of G blocks crossing K grid barriers
//            (arrive = one device-scope atomic add per block, release = the
//            last arriver bumps a generation word the others poll; every poll
//            loop is bounded, so a wave always exits).
// Each phase does the same dependent work: every block writes one word and,
// after the boundary, reads the word another block wrote (the data hand-off
// the engine's phases make through HBM / L2).
// Build: hipcc --offload-arch=gfx950 -O3 grid_barrier.hip -o grid_barrier
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e) { printf("hip error %d (%s) line %d\n", e, hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kSpinLimit = 1 << 20;

__global__ __launch_bounds__(256) void phase_kernel(int* data, int phase, int* sink) {
    const int b = blockIdx.x, g = gridDim.x;
    if (threadIdx.x == 0) {
        const int v = data[(b * 7 + 3) % g];  // another block's word from the previous phase
        data[b] = v + phase;
        if (v == -12345) sink[0] = v;
    }
}

__device__ __forceinline__ bool grid_barrier(unsigned* count, unsigned* gen, unsigned nblocks, unsigned& mygen,
                                             int* timeout) {
    bool ok = true;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned g = mygen;
        __threadfence();
        const unsigned arrived = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (arrived == nblocks * (g + 1) - 1) {
            __hip_atomic_store(gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            int spins = 0;
            while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
                if (++spins > kSpinLimit) {
                    ok = false;
                    __hip_atomic_store(timeout, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
        mygen = g + 1;
    }
    __syncthreads();
    return ok;
}

__global__ __launch_bounds__(256) void persistent_kernel(int* data, int phases, unsigned* count, unsigned* gen,
                                                         int* timeout, int* sink) {
    const int b = blockIdx.x, g = gridDim.x;
    unsigned mygen = 0;
    __shared__ int stop;
    for (int p = 0; p < phases; ++p) {
        if (threadIdx.x == 0) {
            const int v = __hip_atomic_load(&data[(b * 7 + 3) % g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&data[b], v + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (v == -12345) sink[0] = v;
            stop = 0;
        }
        if (!grid_barrier(count, gen, (unsigned)g, mygen, timeout)) stop = 1;
        __syncthreads();
        if (stop) return;
    }
}

int main() {
    const int K = 200;
    int dev = 0, cus = 0, coop = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
    int per_cu = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, persistent_kernel, 256, 0));
    printf("{\"cus\": %d, \"cooperative\": %d, \"max_blocks_per_cu\": %d}\n", cus, coop, per_cu);
    int *data, *sink, *timeout;
    unsigned *count, *gen;
    CK(hipMalloc(&data, 1 << 20));
    CK(hipMalloc(&sink, 4));
    CK(hipMalloc(&timeout, 4));
    CK(hipMalloc(&count, 4));
    CK(hipMalloc(&gen, 4));
    CK(hipMemset(data, 0, 1 << 20));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int blocks : {256, 512, 1024}) {
        if (blocks > cus * per_cu) continue;
        // graph of K dependent launches
        hipGraph_t gr;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int p = 0; p < K; ++p) hipLaunchKernelGGL(phase_kernel, dim3(blocks), dim3(256), 0, s, data, p, sink);
        CK(hipStreamEndCapture(s, &gr));
        CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        float best_graph = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(a, s));
            CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            best_graph = ms < best_graph ? ms : best_graph;
        }
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(gr));
        // one cooperative kernel crossing K grid barriers
        float best_bar = 1e30f;
        int to = 0;
        for (int rep = 0; rep < 6 && !to; ++rep) {
            CK(hipMemsetAsync(count, 0, 4, s));
            CK(hipMemsetAsync(gen, 0, 4, s));
            CK(hipMemsetAsync(timeout, 0, 4, s));
            int phases = K;
            void* args[] = {&data, &phases, &count, &gen, &timeout, &sink};
            CK(hipEventRecord(a, s));
            CK(hipLaunchCooperativeKernel((const void*)persistent_kernel, dim3(blocks), dim3(256), args, 0, s));
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            CK(hipMemcpy(&to, timeout, 4, hipMemcpyDeviceToHost));
            if (rep > 0) best_bar = ms < best_bar ? ms : best_bar;
        }
        printf("{\"blocks\": %d, \"phases\": %d, \"graph_launch_us\": %.3f, \"grid_barrier_us\": %.3f, \"timeout\": %d}\n",
               blocks, K, 1000.0 * best_graph / K, 1000.0 * best_bar / K, to);
    }
    return 0;
}
