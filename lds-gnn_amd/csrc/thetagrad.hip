// θ-gradient assembly: the hypergradient of one (or several) sampled graphs.
//
// Replaces the reverse pass the reference gets from autograd through
//   normalize_adjacency_matrix  (src/utils/graph.py:136-153)
//   straight_through_estimator  (src/models/sampling.py:82-85)
//   triu_values_to_symmetric_matrix (src/utils/graph.py:166-181, clamp at 180)
// which materialises dense N×N gradients (plus the N³ normalisation backward).
// For a cotangent dL/dÂ = Σ_c G_c Z_cᵀ the gradient on θ is
//   dθ_ij = s_i s_j Σ_c (G_c,i·Z_c,j + G_c,j·Z_c,i) + r_i + r_j   (i < j)
//   dθ_ii = 0                                                    (fill_diagonal_)
// with r_i = -½ s_i² Σ_c (G_c,i·Y_c,i + Z_c,i·(ÂG_c)_i) — derivation in DESIGN.md.
// With U = s⊙[G_c], V = s⊙[Z_c] this is a rank-2k symmetric update written
// straight into the packed upper triangle: 4·N(N+1)/2 bytes out, 2·4·N·k in.
#include "common.hpp"
#include "../../include/ldsgnn.h"

namespace lds {

constexpr int kTile = 64;
constexpr int kKC = 16;  // k-chunk staged in LDS

// One 256-thread block per 64×64 tile (bi <= bj) of the upper triangle.  Thread
// (ty, tx) owns rows 4ty..4ty+3 and columns 4tx..4tx+3 of the tile.
__global__ __launch_bounds__(256) void theta_grad_kernel(
    const float* __restrict__ u, const float* __restrict__ v, int ld, int k,
    const float* __restrict__ r, int ldr, int nr, const float* __restrict__ theta, int n,
    float* __restrict__ grad, int accumulate) {
    __shared__ __attribute__((aligned(16))) float Ui[kKC][kTile];
    __shared__ __attribute__((aligned(16))) float Vi[kKC][kTile];
    __shared__ __attribute__((aligned(16))) float Uj[kKC][kTile];
    __shared__ __attribute__((aligned(16))) float Vj[kKC][kTile];
    __shared__ float Ri[kTile], Rj[kTile];

    int a, b;
    tri_tile(blockIdx.x, a, b);
    const int bi = b, bj = a;
    const int i0 = bi * kTile, j0 = bj * kTile;
    const int t = threadIdx.x;
    const int tx = t & 15, ty = t >> 4;

    if (t < 2 * kTile) {
        const int rr = t & (kTile - 1);
        const int row = (t < kTile ? i0 : j0) + rr;
        float acc = 0.f;
        if (row < n)
            for (int c = 0; c < nr; ++c) acc += r[(int64_t)row * ldr + c];
        (t < kTile ? Ri : Rj)[rr] = acc;
    }

    float acc[4][4];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[m][q] = 0.f;

    for (int k0 = 0; k0 < k; k0 += kKC) {
        __syncthreads();
        // stage 64 rows × 16 k of U_i, V_i, U_j, V_j, transposed to [k][row]
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int idx = t + 256 * e;  // 0..1023
            const int rr = idx >> 4, kk = idx & 15;
            const int gi = i0 + rr, gj = j0 + rr, gk = k0 + kk;
            const bool kin = gk < k;
            Ui[kk][rr] = (kin && gi < n) ? u[(int64_t)gi * ld + gk] : 0.f;
            Vi[kk][rr] = (kin && gi < n) ? v[(int64_t)gi * ld + gk] : 0.f;
            Uj[kk][rr] = (kin && gj < n) ? u[(int64_t)gj * ld + gk] : 0.f;
            Vj[kk][rr] = (kin && gj < n) ? v[(int64_t)gj * ld + gk] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < kKC; ++kk) {
            const float4 ui = *reinterpret_cast<const float4*>(&Ui[kk][4 * ty]);
            const float4 vi = *reinterpret_cast<const float4*>(&Vi[kk][4 * ty]);
            const float4 uj = *reinterpret_cast<const float4*>(&Uj[kk][4 * tx]);
            const float4 vj = *reinterpret_cast<const float4*>(&Vj[kk][4 * tx]);
            const float uia[4] = {ui.x, ui.y, ui.z, ui.w};
            const float via[4] = {vi.x, vi.y, vi.z, vi.w};
            const float uja[4] = {uj.x, uj.y, uj.z, uj.w};
            const float vja[4] = {vj.x, vj.y, vj.z, vj.w};
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    acc[m][q] = fmaf(uia[m], vja[q], acc[m][q]);
                    acc[m][q] = fmaf(via[m], uja[q], acc[m][q]);
                }
        }
    }

    const int64_t nn = n;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int li = 4 * ty + m;
        const int i = i0 + li;
        if (i >= n) continue;
        const int64_t rowbase = tri_index(i, i, nn);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int lj = 4 * tx + q;
            const int j = j0 + lj;
            if (j >= n || j < i) continue;
            const int64_t idx = rowbase + (j - i);
            float g = 0.f;
            if (j > i) {
                g = acc[m][q] + Ri[li] + Rj[lj];
                if (theta != nullptr) {
                    const float th = theta[idx];
                    if (!(th >= 0.f && th <= 1.f)) g = 0.f;  // clamp backward
                }
            }
            if (accumulate) grad[idx] += g;
            else grad[idx] = g;
        }
    }
}

// ---------------------------------------------------------------------------
// MFMA form: C_IJ = U_I V_Jᵀ + V_I U_Jᵀ on fp32-in v_mfma_f32_32x32x2_f32
// (exact f32 FMA chains, 64 FLOP/clk/SIMD = the fp32 peak with one VGPR per
// operand).  One 256-thread block per 64×64 tile of the upper triangle, each
// wave a 32×32 sub-tile; k staged through LDS in chunks of 16, transposed to
// [k][row] with a +1 row pad (conflict-free transposed writes and b32 reads).
// Epilogue per mode: 0 grad = g, 1 grad += g, 2 θ = clamp(θ - lr·g, 0, 1)
// with lr read from device memory (and grad = g when grad != NULL), 3 as 2
// with g += grad (the partial sum of earlier column chunks) and grad = g.
// ---------------------------------------------------------------------------
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kLdsRow = kTile + 1;
constexpr int kMC = 32;  // k-chunk of the MFMA form

// Global -> register stage of one k-chunk: thread t holds rows (t >> 2) of the
// i- and j-blocks, k quads (t & 3)·4 and 16 + (t & 3)·4, of U and V.
struct ChunkRegs {
    float4 ui[2], vi[2], uj[2], vj[2];
};

__device__ __forceinline__ void load_chunk(const float* __restrict__ u, const float* __restrict__ v, int ld,
                                           int k, int n, int gi, int gj, int k0, int fq, int vec4,
                                           ChunkRegs& c) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int gk = k0 + fq + 16 * h;
        float4 z = {0.f, 0.f, 0.f, 0.f};
        c.ui[h] = z; c.vi[h] = z; c.uj[h] = z; c.vj[h] = z;
        if (vec4 && gk + 3 < k) {
            if (gi < n) {
                c.ui[h] = *reinterpret_cast<const float4*>(u + (int64_t)gi * ld + gk);
                c.vi[h] = *reinterpret_cast<const float4*>(v + (int64_t)gi * ld + gk);
            }
            if (gj < n) {
                c.uj[h] = *reinterpret_cast<const float4*>(u + (int64_t)gj * ld + gk);
                c.vj[h] = *reinterpret_cast<const float4*>(v + (int64_t)gj * ld + gk);
            }
        } else {
            float* pui = &c.ui[h].x;
            float* pvi = &c.vi[h].x;
            float* puj = &c.uj[h].x;
            float* pvj = &c.vj[h].x;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (gk + e < k) {
                    if (gi < n) {
                        pui[e] = u[(int64_t)gi * ld + gk + e];
                        pvi[e] = v[(int64_t)gi * ld + gk + e];
                    }
                    if (gj < n) {
                        puj[e] = u[(int64_t)gj * ld + gk + e];
                        pvj[e] = v[(int64_t)gj * ld + gk + e];
                    }
                }
            }
        }
    }
}

__device__ __forceinline__ void store4(float (*dst)[kLdsRow], int kq, int row, const float4& x) {
    dst[kq + 0][row] = x.x;
    dst[kq + 1][row] = x.y;
    dst[kq + 2][row] = x.z;
    dst[kq + 3][row] = x.w;
}

// ---------------------------------------------------------------------------
// MFMA form: C_IJ = U_I V_Jᵀ + V_I U_Jᵀ on fp32-in v_mfma_f32_32x32x2_f32
// (exact f32 FMA chains, 64 FLOP/clk/SIMD = the fp32 peak with one VGPR per
// operand).  One 256-thread block per 64×64 tile of the upper triangle, each
// wave a 32×32 sub-tile; k staged through LDS in chunks of 32, transposed to
// [k][row] with a +1 row pad (conflict-free transposed writes and b32 reads).
// Software-pipelined: chunk c+1's global loads are in flight during chunk c's
// MFMAs, and the tile's θ values are loaded before the k loop.
// Epilogue per mode: 0 grad = g, 1 grad += g, 2 θ = clamp(θ - lr·g, 0, 1)
// with lr read from device memory (and grad = g when grad != NULL), 3 as 2
// with g += grad (the partial sum of earlier column chunks) and grad = g.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void theta_grad_mfma_kernel(
    const float* __restrict__ u, const float* __restrict__ v, int ld, int k,
    const float* __restrict__ r, int ldr, int nr, float* __restrict__ theta, int n,
    float* __restrict__ grad, int mode, const double* __restrict__ lr_dev, int vec4, int ldrc,
    float gscale) {
    __shared__ float Ui[kMC][kLdsRow];
    __shared__ float Vi[kMC][kLdsRow];
    __shared__ float Uj[kMC][kLdsRow];
    __shared__ float Vj[kMC][kLdsRow];
    __shared__ float Ri[kTile], Rj[kTile];

    int a, b;
    tri_tile(blockIdx.x, a, b);
    const int bi = b, bj = a;
    const int i0 = bi * kTile, j0 = bj * kTile;
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    const int wr = wave >> 1, wc = wave & 1;  // 32×32 sub-tile of this wave
    const int64_t nn = n;
    const int lj = wc * 32 + (lane & 31);
    const int j = j0 + lj;

    // fill mapping: thread -> (row fr, k quads fq and fq + 16)
    const int fr = t >> 2, fq = (t & 3) * 4;
    const int gi = i0 + fr, gj = j0 + fr;
    ChunkRegs cr;
    if (k > 0) load_chunk(u, v, ld, k, n, gi, gj, 0, fq, vec4, cr);

    // the epilogue's θ / partial-grad operands: issued now, used after the k loop
    float th[16], part[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int i = i0 + wr * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        const bool in = i < n && j < n && j >= i;
        const int64_t idx = in ? tri_index(i, i, nn) + (j - i) : 0;
        th[e] = (in && theta != nullptr) ? theta[idx] : 0.f;
        part[e] = (in && (mode == 1 || mode == 3)) ? grad[idx] : 0.f;
    }

    if (t < 2 * kTile) {
        const int rr = t & (kTile - 1);
        const int row = (t < kTile ? i0 : j0) + rr;
        float acc = 0.f;
        if (row < n)
            for (int c = 0; c < nr; ++c) acc += r[(int64_t)row * ldr + (int64_t)c * ldrc];
        (t < kTile ? Ri : Rj)[rr] = acc;
    }

    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;

    const int ar = wr * 32 + (lane & 31), bc = wc * 32 + (lane & 31), kh = lane >> 5;
    for (int k0 = 0; k0 < k; k0 += kMC) {
        __syncthreads();  // previous chunk's MFMAs are done with the LDS stage
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            store4(Ui, fq + 16 * h, fr, cr.ui[h]);
            store4(Vi, fq + 16 * h, fr, cr.vi[h]);
            store4(Uj, fq + 16 * h, fr, cr.uj[h]);
            store4(Vj, fq + 16 * h, fr, cr.vj[h]);
        }
        __syncthreads();
        if (k0 + kMC < k) load_chunk(u, v, ld, k, n, gi, gj, k0 + kMC, fq, vec4, cr);
        const int kc = min(kMC, k - k0);  // trailing chunk: zero-filled past k, skip whole pairs
#pragma unroll
        for (int kk = 0; kk < kMC; kk += 2) {
            if (kk < kc) {
                // A[i][k] (lane: i = lane&31, k = lane>>5), B[k][j] (k = lane>>5, j = lane&31)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Ui[kk + kh][ar], Vj[kk + kh][bc], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Vi[kk + kh][ar], Uj[kk + kh][bc], acc, 0, 0, 0);
            }
        }
    }
    __syncthreads();  // Ri / Rj written by other waves

    const float lr = mode >= 2 ? (float)(*lr_dev) : 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int li = wr * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        const int i = i0 + li;
        if (i >= n || j >= n || j < i) continue;
        const int64_t idx = tri_index(i, i, nn) + (j - i);
        float g = 0.f;
        if (j > i) {
            // gscale: 1/S for the mean over S replica samples (exactly 1 otherwise)
            const float gs = gscale * (acc[e] + Ri[li] + Rj[lj]);
            g = mode == 3 ? part[e] + gs : gs;
            if (theta != nullptr && !(th[e] >= 0.f && th[e] <= 1.f)) g = 0.f;  // clamp backward
        }
        if (mode == 3) {
            grad[idx] = g;
            theta[idx] = fminf(fmaxf(fmaf(-lr, g, th[e]), 0.f), 1.f);
        } else if (mode == 2) {
            if (grad != nullptr) grad[idx] = g;
            theta[idx] = fminf(fmaxf(fmaf(-lr, g, th[e]), 0.f), 1.f);
        } else if (mode == 1) {
            grad[idx] = part[e] + g;
        } else {
            grad[idx] = g;
        }
    }
}

// Slot factors: G lanes per row (fpad <= G), one feature per lane.
template <int G>
__global__ __launch_bounds__(256) void slot_factors_kernel(
    const float* __restrict__ g, int ldg, const float* __restrict__ z, int ldz,
    const float* __restrict__ y, int ldy, const float* __restrict__ dz, int lddz,
    const float* __restrict__ s, int n, int f, int fpad, float* __restrict__ u, int ldu,
    float* __restrict__ v, int ldv, float* __restrict__ r, int ldr) {
    const int lane = threadIdx.x & (G - 1);
    const int row = (blockIdx.x * 256 + threadIdx.x) / G;
    if (row >= n) return;
    const float si = s[row];
    float gv = 0.f, zv = 0.f, yv = 0.f, dzv = 0.f;
    if (lane < f) {
        gv = g[(int64_t)row * ldg + lane];
        zv = z[(int64_t)row * ldz + lane];
        yv = y[(int64_t)row * ldy + lane];
        dzv = dz[(int64_t)row * lddz + lane];
    }
    float d = gv * yv + zv * dzv;
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) d += __shfl_xor(d, o, G);
    if (lane < fpad) {
        u[(int64_t)row * ldu + lane] = si * gv;
        v[(int64_t)row * ldv + lane] = si * zv;
    }
    if (lane == 0) r[(int64_t)row * ldr] = -0.5f * si * si * d;
}

template <int G>
static void launch_slot(const float* g, int ldg, const float* z, int ldz, const float* y,
                        int ldy, const float* dz, int lddz, const float* s, int n, int f,
                        int fpad, float* u, int ldu, float* v, int ldv, float* r, int ldr,
                        hipStream_t st) {
    const int rows_per_block = 256 / G;
    hipLaunchKernelGGL(slot_factors_kernel<G>, dim3((n + rows_per_block - 1) / rows_per_block),
                       dim3(256), 0, st, g, ldg, z, ldz, y, ldy, dz, lddz, s, n, f, fpad, u, ldu,
                       v, ldv, r, ldr);
}

__global__ void sgd_clamp_kernel(float* __restrict__ theta, const float* __restrict__ grad,
                                 float lr, int64_t count) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n4 = count / 4;
    float4* t4 = reinterpret_cast<float4*>(theta);
    const float4* g4 = reinterpret_cast<const float4*>(grad);
    for (int64_t e = i; e < n4; e += stride) {
        float4 tv = t4[e];
        const float4 gv = g4[e];
        // p.add_(grad, alpha=-lr) (fused multiply-add, as ATen's vectorised add) then clamp_(0, 1)
        tv.x = fminf(fmaxf(fmaf(-lr, gv.x, tv.x), 0.f), 1.f);
        tv.y = fminf(fmaxf(fmaf(-lr, gv.y, tv.y), 0.f), 1.f);
        tv.z = fminf(fmaxf(fmaf(-lr, gv.z, tv.z), 0.f), 1.f);
        tv.w = fminf(fmaxf(fmaf(-lr, gv.w, tv.w), 0.f), 1.f);
        t4[e] = tv;
    }
    for (int64_t e = 4 * n4 + i; e < count; e += stride)
        theta[e] = fminf(fmaxf(fmaf(-lr, grad[e], theta[e]), 0.f), 1.f);
}

__global__ void sgd_clamp_scalar_kernel(float* __restrict__ theta, const float* __restrict__ grad,
                                        float lr, int64_t count) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < count; e += stride)
        theta[e] = fminf(fmaxf(fmaf(-lr, grad[e], theta[e]), 0.f), 1.f);
}

}  // namespace lds

using namespace lds;

extern "C" int lds_theta_grad(const float* u, const float* v, int ld, int k, const float* r,
                              int ldr, int nr, const float* theta, int n, float* grad,
                              int accumulate, void* stream) {
    LDS_CHECK_ARG(grad != nullptr && n > 0 && k >= 0 && nr >= 0);
    LDS_CHECK_ARG(k == 0 || (u != nullptr && v != nullptr && ld >= k));
    LDS_CHECK_ARG(nr == 0 || (r != nullptr && ldr >= nr));
    const int nb = (n + kTile - 1) / kTile;
    const int ntiles = nb * (nb + 1) / 2;
    const int vec4 = ((ld & 3) == 0 && ((((uintptr_t)u) | ((uintptr_t)v)) & 15) == 0) ? 1 : 0;
    hipLaunchKernelGGL(theta_grad_mfma_kernel, dim3(ntiles), dim3(256), 0, (hipStream_t)stream, u,
                       v, ld, k, r, ldr, nr, const_cast<float*>(theta), n, grad, accumulate ? 1 : 0,
                       (const double*)nullptr, vec4, 1, 1.0f);
    LDS_RETURN_LAST_ERROR();
}

// VALU reference form of lds_theta_grad (kept for A/B timing and testing).
extern "C" int lds_theta_grad_valu(const float* u, const float* v, int ld, int k, const float* r,
                                   int ldr, int nr, const float* theta, int n, float* grad,
                                   int accumulate, void* stream) {
    LDS_CHECK_ARG(grad != nullptr && n > 0 && k >= 0 && nr >= 0);
    LDS_CHECK_ARG(k == 0 || (u != nullptr && v != nullptr && ld >= k));
    LDS_CHECK_ARG(nr == 0 || (r != nullptr && ldr >= nr));
    const int nb = (n + kTile - 1) / kTile;
    const int ntiles = nb * (nb + 1) / 2;
    hipLaunchKernelGGL(theta_grad_kernel, dim3(ntiles), dim3(256), 0, (hipStream_t)stream, u, v,
                       ld, k, r, ldr, nr, theta, n, grad, accumulate);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_theta_grad_sgd(const float* u, const float* v, int ld, int k, const float* r,
                                  int ldr, int nr, float* theta, int n, float* grad,
                                  const void* scalars, void* stream) {
    LDS_CHECK_ARG(theta != nullptr && scalars != nullptr && n > 0 && k >= 0 && nr >= 0);
    LDS_CHECK_ARG(k == 0 || (u != nullptr && v != nullptr && ld >= k));
    LDS_CHECK_ARG(nr == 0 || (r != nullptr && ldr >= nr));
    const int nb = (n + kTile - 1) / kTile;
    const int ntiles = nb * (nb + 1) / 2;
    const int vec4 = ((ld & 3) == 0 && ((((uintptr_t)u) | ((uintptr_t)v)) & 15) == 0) ? 1 : 0;
    // EngineScalars: f64 outer_lr at byte offset 16
    const double* lr = reinterpret_cast<const double*>((const char*)scalars + 16);
    hipLaunchKernelGGL(theta_grad_mfma_kernel, dim3(ntiles), dim3(256), 0, (hipStream_t)stream, u,
                       v, ld, k, r, ldr, nr, theta, n, grad, 2, lr, vec4, 1, 1.0f);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_theta_grad_sgd_accum(const float* u, const float* v, int ld, int k, const float* r,
                                        int ldr, int nr, float* theta, int n, float* grad,
                                        const void* scalars, void* stream) {
    LDS_CHECK_ARG(theta != nullptr && grad != nullptr && scalars != nullptr && n > 0 && k >= 0 && nr >= 0);
    LDS_CHECK_ARG(k == 0 || (u != nullptr && v != nullptr && ld >= k));
    LDS_CHECK_ARG(nr == 0 || (r != nullptr && ldr >= nr));
    const int nb = (n + kTile - 1) / kTile;
    const int ntiles = nb * (nb + 1) / 2;
    const int vec4 = ((ld & 3) == 0 && ((((uintptr_t)u) | ((uintptr_t)v)) & 15) == 0) ? 1 : 0;
    const double* lr = reinterpret_cast<const double*>((const char*)scalars + 16);
    hipLaunchKernelGGL(theta_grad_mfma_kernel, dim3(ntiles), dim3(256), 0, (hipStream_t)stream, u,
                       v, ld, k, r, ldr, nr, theta, n, grad, 3, lr, vec4, 1, 1.0f);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_theta_grad_ex(const float* u, const float* v, int ld, int k, const float* r,
                                 int ldr_row, int ldr_col, int nr, float* theta, int n, float* grad,
                                 int mode, const void* scalars, float gscale, void* stream) {
    LDS_CHECK_ARG(n > 0 && k >= 0 && nr >= 0 && mode >= 0 && mode <= 3);
    LDS_CHECK_ARG(k == 0 || (u != nullptr && v != nullptr && ld >= k));
    LDS_CHECK_ARG(nr == 0 || (r != nullptr && ldr_row >= 0 && ldr_col >= 0));
    LDS_CHECK_ARG(mode < 2 ? grad != nullptr : (theta != nullptr && scalars != nullptr));
    LDS_CHECK_ARG(mode != 3 || grad != nullptr);
    const int nb = (n + kTile - 1) / kTile;
    const int ntiles = nb * (nb + 1) / 2;
    const int vec4 = ((ld & 3) == 0 && ((((uintptr_t)u) | ((uintptr_t)v)) & 15) == 0) ? 1 : 0;
    const double* lr = mode >= 2 ? reinterpret_cast<const double*>((const char*)scalars + 16) : nullptr;
    // (a 128×128-tile variant — 8 MFMAs per 8 LDS reads, 4 accumulators per
    //  wave — measured slower at both ends: at n = 2708 it has 253 tiles, one
    //  4-wave block per CU; at n = 20 000 (12 k tiles) 3.12 ms against 2.27 ms,
    //  196 VGPRs and 66 KB LDS leave 2 waves per SIMD.  MFMA busy of this form
    //  at S = 16 is 63 % of the cycles at a 2.26 GHz DVFS clock, r01 PMC)
    hipLaunchKernelGGL(theta_grad_mfma_kernel, dim3(ntiles), dim3(256), 0, (hipStream_t)stream, u, v, ld, k, r,
                       ldr_row, nr, theta, n, grad, mode, lr, vec4, ldr_col, gscale);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_slot_factors(const float* g, int ldg, const float* z, int ldz, const float* y,
                                int ldy, const float* dz, int lddz, const float* s, int n, int f,
                                int fpad, float* u, int ldu, float* v, int ldv, float* r, int ldr,
                                void* stream) {
    LDS_CHECK_ARG(g && z && y && dz && s && u && v && r && n > 0);
    LDS_CHECK_ARG(f > 0 && fpad >= f && fpad <= 64 && ldu >= fpad && ldv >= fpad);
    LDS_CHECK_ARG(ldg >= f && ldz >= f && ldy >= f && lddz >= f && ldr >= 1);
    hipStream_t st = (hipStream_t)stream;
    if (fpad <= 8) launch_slot<8>(g, ldg, z, ldz, y, ldy, dz, lddz, s, n, f, fpad, u, ldu, v, ldv, r, ldr, st);
    else if (fpad <= 16) launch_slot<16>(g, ldg, z, ldz, y, ldy, dz, lddz, s, n, f, fpad, u, ldu, v, ldv, r, ldr, st);
    else if (fpad <= 32) launch_slot<32>(g, ldg, z, ldz, y, ldy, dz, lddz, s, n, f, fpad, u, ldu, v, ldv, r, ldr, st);
    else launch_slot<64>(g, ldg, z, ldz, y, ldy, dz, lddz, s, n, f, fpad, u, ldu, v, ldv, r, ldr, st);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_sgd_clamp(float* theta, const float* grad, float lr, int64_t count,
                             void* stream) {
    LDS_CHECK_ARG(theta != nullptr && grad != nullptr && count >= 0);
    if (count == 0) return 0;
    const int64_t blocks64 = (count / 4 + 255) / 256 + 1;
    const int blocks = (int)(blocks64 < 8192 ? blocks64 : 8192);
    const bool aligned = ((((uintptr_t)theta) | ((uintptr_t)grad)) & 15) == 0;
    if (aligned)
        hipLaunchKernelGGL(sgd_clamp_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                           theta, grad, lr, count);
    else
        hipLaunchKernelGGL(sgd_clamp_scalar_kernel, dim3(blocks), dim3(256), 0,
                           (hipStream_t)stream, theta, grad, lr, count);
    LDS_RETURN_LAST_ERROR();
}
