// Philox4x32-10 throughput on gfx950: the 32x32->64 products as
// v_mul_hi_u32 + v_mul_lo_u32 (compiler default) vs one v_mad_u64_u32
// (mode 1), and that with each round's three-way xor as one v_bitop3_b32 (XOR3 table 0x96; gfx950 has no v_xor3_b32) whose
// key operand is the SGPR round key (mode 2; the compiler emits two
// v_xor_b32 for `hi ^ c ^ k`).  Keys are kernel arguments (run-time SGPRs).
// Build: hipcc --offload-arch=gfx950 -O3 philox_rate.hip -o philox_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

struct Q { uint32_t x, y, z, w; };

__device__ __forceinline__ void mul_split(uint32_t m, uint32_t a, uint32_t& hi, uint32_t& lo) {
    hi = __umulhi(m, a);
    lo = m * a;
}

__device__ __forceinline__ void mul_mad(uint32_t m, uint32_t a, uint32_t& hi, uint32_t& lo) {
    uint64_t r, cc;
    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(cc) : "v"(m), "v"(a));
    hi = (uint32_t)(r >> 32);
    lo = (uint32_t)r;
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t k) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
}

template <int kMode>
__device__ __forceinline__ Q philox(Q c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0, lo0, hi1, lo1;
        if (kMode == 0) {
            mul_split(0xD2511F53u, c.x, hi0, lo0);
            mul_split(0xCD9E8D57u, c.z, hi1, lo1);
        } else {
            mul_mad(0xD2511F53u, c.x, hi0, lo0);
            mul_mad(0xCD9E8D57u, c.z, hi1, lo1);
        }
        if (kMode == 2)
            c = Q{xor3(hi1, c.y, k0), lo1, xor3(hi0, c.w, k1), lo0};
        else
            c = Q{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
        asm volatile("" : "+s"(k0), "+s"(k1));
    }
    return c;
}

template <int kMode>
__global__ __launch_bounds__(256) void bench(uint32_t* out, int iters, uint32_t k0, uint32_t k1) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    uint32_t acc = 0;
    for (int i = 0; i < iters; ++i) {
        const Q o = philox<kMode>(Q{t, (uint32_t)i, 7u, acc & 1u}, k0, k1);
        acc ^= o.x ^ o.y ^ o.z ^ o.w;
    }
    out[t] = acc;
}

int main() {
    const int blocks = 256 * 8 * 4, iters = 64;
    uint32_t* d;
    hipMalloc(&d, (size_t)blocks * 256 * 4);
    uint32_t* h[3] = {new uint32_t[blocks * 256], new uint32_t[blocks * 256], new uint32_t[blocks * 256]};
    const char* names[3] = {"mul_hi+mul_lo", "v_mad_u64_u32", "v_mad_u64_u32 + v_bitop3_b32"};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int mode = 0; mode < 3; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a);
            if (mode == 0) hipLaunchKernelGGL(bench<0>, dim3(blocks), dim3(256), 0, 0, d, iters, 0x1234u, 0x5678u);
            else if (mode == 1) hipLaunchKernelGGL(bench<1>, dim3(blocks), dim3(256), 0, 0, d, iters, 0x1234u, 0x5678u);
            else hipLaunchKernelGGL(bench<2>, dim3(blocks), dim3(256), 0, 0, d, iters, 0x1234u, 0x5678u);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double calls = (double)blocks * 256 * iters;
            if (rep == 2) printf("mode %d (%s): %.3f ms, %.2f G philox/s\n", mode, names[mode], ms,
                                 calls / (ms * 1e-3) / 1e9);
        }
        hipMemcpy(h[mode], d, (size_t)blocks * 256 * 4, hipMemcpyDeviceToHost);
    }
    int diff1 = 0, diff2 = 0;
    for (int i = 0; i < blocks * 256; ++i) {
        diff1 += h[0][i] != h[1][i];
        diff2 += h[0][i] != h[2][i];
    }
    printf("outputs differ from mode 0: mode 1 %d, mode 2 %d\n", diff1, diff2);
    return 0;
}
