// Shared device helpers for the LDS hot-path kernels (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define LDS_CHECK_ARG(cond)                                   \
    do {                                                      \
        if (!(cond)) return (int)hipErrorInvalidValue;        \
    } while (0)

#define LDS_RETURN_LAST_ERROR() return (int)hipGetLastError()

namespace lds {

constexpr int kWave = 64;
constexpr int kEllWidth = 64;  // neighbours per row in a graph's ELL head ({j, s_j} pairs): one wave's step
// The j field of an ELL entry: node index in the low 24 bits, the node's flag
// byte (e.g. train / opt mask bits, include/ldsgnn.h) above them.
constexpr int kEllIndex = 0x00FFFFFF;
constexpr int kEllFlagShift = 24;

// Packed upper-triangle index of (i, j), i <= j, of an n×n matrix in
// torch.triu_indices(n, n) row-major order (src/utils/graph.py:41-45).
__host__ __device__ __forceinline__ int64_t tri_index(int64_t i, int64_t j, int64_t n) {
    return i * (2 * n - i + 1) / 2 + (j - i);
}

// Linear tile id -> (row block a, col block b) with b <= a, enumerating the
// lower triangle of an nb×nb block grid row by row; callers use (bi, bj) =
// (b, a) so bi <= bj covers the upper triangle.
__device__ __forceinline__ void tri_tile(int t, int& a, int& b) {
    int r = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
    while ((int64_t)r * (r + 1) / 2 > t) --r;
    while ((int64_t)(r + 1) * (r + 2) / 2 <= t) ++r;
    a = r;
    b = t - r * (r + 1) / 2;
}

struct U32x4 {
    uint32_t x, y, z, w;
};

// Philox4x32-10 (Salmon et al., SC'11).  Counter (c0..c3), key (k0, k1).
__device__ __forceinline__ U32x4 philox4x32_10(U32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // (a v_mad_u64_u32 form was 1.31x faster in isolation,
        // tools/microbench/philox_rate.hip, but slower inside the sampler)
        const uint32_t lo0 = 0xD2511F53u * c.x;
        const uint32_t hi0 = __umulhi(0xD2511F53u, c.x);
        const uint32_t lo1 = 0xCD9E8D57u * c.z;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z);
        c = U32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// 24-bit uniform in [0, 1), exactly representable in fp32.
__device__ __forceinline__ float u01(uint32_t x) {
    return (float)(x >> 8) * (1.0f / 16777216.0f);
}

// The four uniforms u(row, col) for rows 4*(row>>2) .. +3 at one column.
__device__ __forceinline__ void philox_quad(uint32_t k0, uint32_t k1, uint32_t tag,
                                            uint32_t counter, uint32_t col, uint32_t row_quad,
                                            float u[4]) {
    const U32x4 o = philox4x32_10(U32x4{col, row_quad, tag, counter}, k0, k1);
    u[0] = u01(o.x);
    u[1] = u01(o.y);
    u[2] = u01(o.z);
    u[3] = u01(o.w);
}

// fl32(1 / fl32(sqrt(d))) with IEEE round-to-nearest at both steps: the
// correctly rounded value of `1.0 / degree.sqrt()` (src/utils/graph.py:148),
// as a GPU (and numpy) computes it.  (torch CPU routes `1.0 / t` through a
// vectorised reciprocal whose last bit depends on the host ISA.)  Evaluated
// in fp64 and rounded to fp32: for sqrt and division a 53-bit intermediate
// rounds to the correctly rounded 24-bit result (53 >= 2·24+2).
__device__ __forceinline__ float inv_sqrt_degree(int d) {
    const float sq = (float)__dsqrt_rn((double)d);
    return (float)__ddiv_rn(1.0, (double)sq);
}

__device__ __forceinline__ int wave_lane() { return threadIdx.x & (kWave - 1); }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

}  // namespace lds
