// Aggregation-kernel variants for the latency-bound Cora chain: Y = Â·Z,
// F = 16, CSR + ELL head (the engine's graph layout), one launch = one
// aggregation.  Built as its own library (tools/microbench/aggbench.py) and
// timed in a replayed chain of K launches per variant.
//   0  16 lanes per row, ELL head + chunks of 16 (the engine's agg_row)
//   1  one wave per row: the row's entries in 64-wide steps, 4 groups of 16
//      lanes, xor-shuffle reduction across groups (no ELL)
//   2  one wave per row: group 0 takes the ELL head, groups 1-3 the first 48
//      entries past it, then 64-wide steps over all groups
//   3  variant 1 with up to 4 of its 64-wide steps loaded at once
//   4  variant 1 with rows of more than 64 entries on a whole 4-wave block
//   8  floor: a trivial kernel with variant 0's grid
//   9  one dependent load round trip per lane, variant 0's grid
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {
constexpr int HID = 16;

__global__ __launch_bounds__(256) void agg_v0(const int* __restrict__ rp, const int* __restrict__ col,
                                              const float* __restrict__ s, const int2* __restrict__ ell, int n,
                                              const float* __restrict__ z, float* __restrict__ y) {
    const int lane = threadIdx.x & (HID - 1);
    const int row = (blockIdx.x * 256 + threadIdx.x) / HID;
    if (row >= n) return;
    float acc = 0.f;
    const int end = rp[row + 1];
    const int2 e = ell[row * HID + lane];
    int p0 = rp[row] + HID;
    const float sl = __int_as_float(e.y);
    float zk[HID];
#pragma unroll
    for (int k = 0; k < HID; ++k) zk[k] = z[__shfl(e.x, k, HID) * HID + lane];
#pragma unroll
    for (int k = 0; k < HID; ++k) acc = fmaf(__shfl(sl, k, HID), zk[k], acc);
    for (; p0 < end; p0 += HID) {
        const int p = p0 + lane;
        const int jl = p < end ? col[p] : row;
        const float s2 = p < end ? s[jl] : 0.f;
#pragma unroll
        for (int k = 0; k < HID; ++k) zk[k] = z[__shfl(jl, k, HID) * HID + lane];
#pragma unroll
        for (int k = 0; k < HID; ++k) acc = fmaf(__shfl(s2, k, HID), zk[k], acc);
    }
    y[row * HID + lane] = s[row] * acc;
}

// one wave per row, 64 entries per step: group g of step t takes entries
// beg + 64t + 16g .. +15; lane h of a group gathers feature h of each.
__global__ __launch_bounds__(256) void agg_v1(const int* __restrict__ rp, const int* __restrict__ col,
                                              const float* __restrict__ s, const int2* __restrict__ ell, int n,
                                              const float* __restrict__ z, float* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int h = lane & (HID - 1);
    const int g = lane >> 4;
    const int row = (blockIdx.x * 256 + threadIdx.x) >> 6;
    if (row >= n) return;
    const int beg = rp[row], end = rp[row + 1];
    float acc = 0.f;
    for (int p0 = beg; p0 < end; p0 += 64) {
        const int p = p0 + lane;
        const int jl = p < end ? col[p] : row;
        const float sl = p < end ? s[jl] : 0.f;
        float zk[HID];
#pragma unroll
        for (int k = 0; k < HID; ++k) zk[k] = z[__shfl(jl, g * HID + k) * HID + h];
#pragma unroll
        for (int k = 0; k < HID; ++k) acc = fmaf(__shfl(sl, g * HID + k), zk[k], acc);
    }
    acc += __shfl_xor(acc, 16);
    acc += __shfl_xor(acc, 32);
    if (lane < HID) y[row * HID + h] = s[row] * acc;
}

// one wave per row with the ELL head in group 0 and entries 16..63 in groups
// 1..3 at the same time (their col loads need rp, loaded beside the ELL)
__global__ __launch_bounds__(256) void agg_v2(const int* __restrict__ rp, const int* __restrict__ col,
                                              const float* __restrict__ s, const int2* __restrict__ ell, int n,
                                              const float* __restrict__ z, float* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int h = lane & (HID - 1);
    const int g = lane >> 4;
    const int row = (blockIdx.x * 256 + threadIdx.x) >> 6;
    if (row >= n) return;
    const int beg = rp[row], end = rp[row + 1];
    float acc = 0.f;
    int jl;
    float sl;
    if (g == 0) {
        const int2 e = ell[row * HID + h];
        jl = e.x;
        sl = __int_as_float(e.y);
    } else {
        const int p = beg + lane;  // entries 16..63
        jl = p < end ? col[p] : row;
        sl = p < end ? s[jl] : 0.f;
    }
    {
        float zk[HID];
#pragma unroll
        for (int k = 0; k < HID; ++k) zk[k] = z[__shfl(jl, g * HID + k) * HID + h];
#pragma unroll
        for (int k = 0; k < HID; ++k) acc = fmaf(__shfl(sl, g * HID + k), zk[k], acc);
    }
    for (int p0 = beg + 64; p0 < end; p0 += 64) {
        const int p = p0 + lane;
        const int j2 = p < end ? col[p] : row;
        const float s2 = p < end ? s[j2] : 0.f;
        float zk[HID];
#pragma unroll
        for (int k = 0; k < HID; ++k) zk[k] = z[__shfl(j2, g * HID + k) * HID + h];
#pragma unroll
        for (int k = 0; k < HID; ++k) acc = fmaf(__shfl(s2, g * HID + k), zk[k], acc);
    }
    acc += __shfl_xor(acc, 16);
    acc += __shfl_xor(acc, 32);
    if (lane < HID) y[row * HID + h] = s[row] * acc;
}

// one wave per row, the wave-uniform iteration count taken up to 4 steps at a
// time: every step's col loads, then every step's s / Z gathers
__global__ __launch_bounds__(256) void agg_v3(const int* __restrict__ rp, const int* __restrict__ col,
                                              const float* __restrict__ s, const int2* __restrict__ ell, int n,
                                              const float* __restrict__ z, float* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int h = lane & (HID - 1);
    const int g = lane >> 4;
    const int row = (blockIdx.x * 256 + threadIdx.x) >> 6;
    if (row >= n) return;
    const int beg = rp[row], end = rp[row + 1];
    const int nit = (end - beg + 63) >> 6;
    float acc = 0.f;
    for (int i0 = 0; i0 < nit; i0 += 4) {
        const int m = min(4, nit - i0);
        int jl[4];
        float sl[4];
        float zk[4][HID];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (c < m) {
                const int p = beg + (i0 + c) * 64 + lane;
                jl[c] = p < end ? col[p] : row;
            }
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (c < m) {
                const int p = beg + (i0 + c) * 64 + lane;
                sl[c] = p < end ? s[jl[c]] : 0.f;
#pragma unroll
                for (int k = 0; k < HID; ++k) zk[c][k] = z[__shfl(jl[c], g * HID + k) * HID + h];
            }
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (c < m) {
#pragma unroll
                for (int k = 0; k < HID; ++k) acc = fmaf(__shfl(sl[c], g * HID + k), zk[c][k], acc);
            }
        }
    }
    acc += __shfl_xor(acc, 16);
    acc += __shfl_xor(acc, 32);
    if (lane < HID) y[row * HID + h] = s[row] * acc;
}

// variant 1 plus a row plan: the `nh` rows with more than 64 entries first,
// each taking a whole 4-wave block (256 entries per step, the four wave sums
// combined through LDS in wave order), then the other rows one wave each
__global__ __launch_bounds__(256) void agg_v4(const int* __restrict__ rp, const int* __restrict__ col,
                                              const float* __restrict__ s, const int* __restrict__ plan, int nh,
                                              int n, const float* __restrict__ z, float* __restrict__ y) {
    __shared__ float part[4][HID];
    const int lane = threadIdx.x & 63;
    const int h = lane & (HID - 1);
    const int g = lane >> 4;
    const int wave = threadIdx.x >> 6;
    const bool heavy = (int)blockIdx.x < nh;
    int row;
    if (heavy) {
        row = plan[blockIdx.x];
    } else {
        const int i = nh + ((int)blockIdx.x - nh) * 4 + wave;
        if (i >= n) return;
        row = plan[i];
    }
    const int beg = rp[row], end = rp[row + 1];
    const int step = heavy ? 256 : 64;
    float acc = 0.f;
    for (int p0 = beg + (heavy ? wave * 64 : 0); p0 < end; p0 += step) {
        const int p = p0 + lane;
        const int jl = p < end ? col[p] : row;
        const float sl = p < end ? s[jl] : 0.f;
        float zk[HID];
#pragma unroll
        for (int k = 0; k < HID; ++k) zk[k] = z[__shfl(jl, g * HID + k) * HID + h];
#pragma unroll
        for (int k = 0; k < HID; ++k) acc = fmaf(__shfl(sl, g * HID + k), zk[k], acc);
    }
    acc += __shfl_xor(acc, 16);
    acc += __shfl_xor(acc, 32);
    if (heavy) {
        if (lane < HID) part[wave][lane] = acc;
        __syncthreads();
        if (wave != 0) return;
        acc = ((part[0][h] + part[1][h]) + part[2][h]) + part[3][h];
    }
    if (lane < HID) y[row * HID + h] = s[row] * acc;
}

// trivial kernel with the same grid as v0: the launch / boundary floor
__global__ __launch_bounds__(256) void agg_floor(const int* __restrict__ rp, int n, float* __restrict__ y) {
    const int row = (blockIdx.x * 256 + threadIdx.x) / HID;
    if (row >= n) return;
    y[row * HID + (threadIdx.x & 15)] = (float)rp[row];
}

// one load round trip through the previous launch's output (z), same grid
__global__ __launch_bounds__(256) void agg_one_hop(const int* __restrict__ rp, int n, const float* __restrict__ z,
                                                   float* __restrict__ y) {
    const int row = (blockIdx.x * 256 + threadIdx.x) / HID;
    if (row >= n) return;
    const int i = row * HID + (threadIdx.x & 15);
    y[i] = z[i] * 0.5f + 1.0f;
}
}  // namespace

extern "C" int aggbench_launch_plan(const int* rp, const int* col, const float* s, const int* plan, int nh, int n,
                                    const float* z, float* y, void* stream) {
    hipLaunchKernelGGL(agg_v4, dim3(nh + (n - nh + 3) / 4), dim3(256), 0, (hipStream_t)stream, rp, col, s, plan, nh,
                       n, z, y);
    return (int)hipGetLastError();
}

extern "C" int aggbench_launch(int variant, const int* rp, const int* col, const float* s, const int2* ell, int n,
                               const float* z, float* y, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    switch (variant) {
        case 0: hipLaunchKernelGGL(agg_v0, dim3((n * HID + 255) / 256), dim3(256), 0, st, rp, col, s, ell, n, z, y); break;
        case 1: hipLaunchKernelGGL(agg_v1, dim3((n * 64 + 255) / 256), dim3(256), 0, st, rp, col, s, ell, n, z, y); break;
        case 2: hipLaunchKernelGGL(agg_v2, dim3((n * 64 + 255) / 256), dim3(256), 0, st, rp, col, s, ell, n, z, y); break;
        case 3: hipLaunchKernelGGL(agg_v3, dim3((n * 64 + 255) / 256), dim3(256), 0, st, rp, col, s, ell, n, z, y); break;
        case 8: hipLaunchKernelGGL(agg_floor, dim3((n * HID + 255) / 256), dim3(256), 0, st, rp, n, y); break;
        case 9: hipLaunchKernelGGL(agg_one_hop, dim3((n * HID + 255) / 256), dim3(256), 0, st, rp, n, z, y); break;
        default: return 1;
    }
    return (int)hipGetLastError();
}
