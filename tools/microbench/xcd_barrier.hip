// The phase boundary of a persistent inner step confined to ONE XCD
// (round-5 VERDICT item 3): what a barrier among the 32 workgroups of one
// XCD costs, against a dependent launch of a 32- and a 256-workgroup kernel
// in a HIP graph and against the flat 256-workgroup barrier of
// grid_barrier.hip (15.2 µs).
//
// Geometry: a 256-workgroup grid, one 256-thread workgroup per CU (the LDS
// request keeps two from sharing a CU).  Workgroup b belongs to group
// b % 8 — under the round-robin dispatch of gfx950 that is one XCD per
// group, which is the speed assumption being measured; correctness never
// depends on it (every barrier counts its own group's arrivals, every spin
// is bounded).  Modes:
//   groups = 1: group 0's 32 workgroups cross K barriers, the other 224
//               workgroups exit at once (one replica's chain on one XCD);
//   groups = 8: all eight groups cross K barriers each, independently
//               (one replica chain per XCD, BASELINE config 4 at 8 per GPU).
// Each phase makes the engine's kind of hand-off: every workgroup stores one
// word, and after the barrier loads the word another workgroup of its group
// stored (agent-scope relaxed atomics, ordered by the barrier's release /
// acquire fences).
// Barrier: one arrival counter and one generation word per group on lines of
// their own; lane 0 of each workgroup: release fence -> relaxed add; the
// last arriver stores the next generation; the others poll it with relaxed
// loads and s_sleep, then an acquire fence.
// Build: hipcc --offload-arch=gfx950 -O3 xcd_barrier.hip -o xcd_barrier
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e) { printf("hip error %d (%s) line %d\n", e, hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kSpinLimit = 1 << 22;
constexpr int kGroups = 8;
constexpr int kLine = 32;  // ints per 128-byte line

__global__ __launch_bounds__(256) void launch_phase(int* data, int phase, int* sink) {
    // the dependent-launch form of one phase: the same store / load hand-off
    const int b = blockIdx.x, g = gridDim.x;
    if (threadIdx.x == 0) {
        const int v = data[(b * 7 + 3) % g];
        data[b] = v + phase;
        if (v == -12345) sink[0] = v;
    }
}

__global__ __launch_bounds__(256) void xcd_persistent(int* data, int phases, int groups, unsigned* count,
                                                      unsigned* gen, int* timeout, int* sink) {
    __shared__ int pad[24 * 1024];  // 96 KB: one workgroup per CU
    __shared__ int stop;
    const int grp = blockIdx.x % kGroups;
    if (grp >= groups) return;
    const int per = gridDim.x / kGroups;
    const int me = blockIdx.x / kGroups;
    unsigned* cnt = count + grp * kLine;
    unsigned* gw = gen + grp * kLine;
    int* d = data + grp * 1024;
    unsigned mygen = 0;
    if (threadIdx.x == 0) pad[0] = 0;
    for (int p = 0; p < phases; ++p) {
        if (threadIdx.x == 0) {
            const int v = __hip_atomic_load(&d[(me * 7 + 3) % per], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&d[me], v + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (v == -12345) sink[0] = v + pad[0];
            stop = 0;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            __atomic_thread_fence(__ATOMIC_RELEASE);  // (agent scope by default in HIP)
            const unsigned arrived = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (arrived == (unsigned)per * (mygen + 1) - 1) {
                __hip_atomic_store(gw, mygen + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                int spins = 0;
                while (__hip_atomic_load(gw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == mygen) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > kSpinLimit) {
                        stop = 1;
                        __hip_atomic_store(timeout, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
            __atomic_thread_fence(__ATOMIC_ACQUIRE);
            mygen += 1;
        }
        __syncthreads();
        if (stop) return;
    }
}

int main() {
    const int K = 400;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    int per_cu = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, xcd_persistent, 256, 0));
    printf("{\"cus\": %d, \"persistent_blocks_per_cu\": %d}\n", cus, per_cu);
    if (per_cu < 1 || cus < 256) {
        printf("{\"error\": \"needs 256 CUs with one resident workgroup each\"}\n");
        return 1;
    }
    int *data, *sink, *timeout;
    unsigned *count, *gen;
    CK(hipMalloc(&data, 1 << 20));
    CK(hipMalloc(&sink, 4));
    CK(hipMalloc(&timeout, 4));
    CK(hipMalloc(&count, 4 * kLine * kGroups));
    CK(hipMalloc(&gen, 4 * kLine * kGroups));
    CK(hipMemset(data, 0, 1 << 20));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    // dependent launches replayed from one graph, 32- and 256-workgroup grids
    for (int blocks : {32, 256}) {
        hipGraph_t gr;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int p = 0; p < K; ++p) hipLaunchKernelGGL(launch_phase, dim3(blocks), dim3(256), 0, s, data, p, sink);
        CK(hipStreamEndCapture(s, &gr));
        CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(a, s));
            CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
        }
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(gr));
        printf("{\"form\": \"graph-launch\", \"blocks\": %d, \"phases\": %d, \"us_per_phase\": %.3f}\n", blocks, K,
               1000.0 * best / K);
    }
    // persistent: one group (one XCD) and all eight groups, K barriers each;
    // a plain launch (the grid is one workgroup per CU, all resident)
    for (int groups : {1, 8}) {
        float best = 1e30f, base = 1e30f;
        int to = 0;
        for (int phases : {0, K}) {
            for (int rep = 0; rep < 6 && !to; ++rep) {
                CK(hipMemsetAsync(count, 0, 4 * kLine * kGroups, s));
                CK(hipMemsetAsync(gen, 0, 4 * kLine * kGroups, s));
                CK(hipMemsetAsync(timeout, 0, 4, s));
                CK(hipEventRecord(a, s));
                hipLaunchKernelGGL(xcd_persistent, dim3(256), dim3(256), 0, s, data, phases, groups, count, gen,
                                   timeout, sink);
                CK(hipGetLastError());
                CK(hipEventRecord(b, s));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                CK(hipMemcpy(&to, timeout, 4, hipMemcpyDeviceToHost));
                if (rep > 0) {
                    if (phases) best = ms < best ? ms : best;
                    else base = ms < base ? ms : base;
                }
            }
        }
        printf("{\"form\": \"xcd-barrier\", \"groups\": %d, \"blocks_per_group\": 32, \"phases\": %d, "
               "\"launch_us\": %.3f, \"us_per_phase\": %.3f, \"timeout\": %d}\n",
               groups, K, 1000.0 * base, 1000.0 * (best - base) / K, to);
        if (to) return 1;
    }
    return 0;
}
