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

// R_i = Σ_c r[i·ldr + c·ldrc], summed in c order; the loads of four terms are
// issued together (one wait per four, not one per term: nr = S at S samples).
__device__ __forceinline__ float row_r_sum(const float* __restrict__ r, int64_t base, int ldrc, int nr) {
    float acc = 0.f;
    int c = 0;
    for (; c + 4 <= nr; c += 4) {
        const float a0 = r[base + (int64_t)c * ldrc], a1 = r[base + (int64_t)(c + 1) * ldrc];
        const float a2 = r[base + (int64_t)(c + 2) * ldrc], a3 = r[base + (int64_t)(c + 3) * ldrc];
        acc += a0;
        acc += a1;
        acc += a2;
        acc += a3;
    }
    for (; c < nr; ++c) acc += r[base + (int64_t)c * ldrc];
    return acc;
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
            acc = row_r_sum(r, (int64_t)row * ldr, ldrc, nr);
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

// ---------------------------------------------------------------------------
// Split-bf16 MFMA form of the same assembly (the default).  Every fp32
// operand x is cut at staging time into three bf16 words x = x0 + x1 + x2
// (truncations: x0 = top 8 significand bits, x1 = the next 8 of the exact
// remainder, x2 = the next 8 of what is left), so x0 + x1 + x2 carries all
// 24 bits to within one truncation of x2 (≤ 2⁻²³|x|).  A product keeps the
// six terms down to order 2⁻¹⁶: a0b0 + a0b1 + a1b0 + a0b2 + a1b1 + a2b0; the
// dropped three are ≤ 2⁻²⁴|ab| — fp32 accuracy at fp32 accumulation.  Six
// v_mfma_f32_32x32x16_bf16 (32 cycles each) replace eight
// v_mfma_f32_32x32x2_f32 (64 cycles each) per 16-wide k-step: 2.67× fewer
// MFMA cycles.
// LDS: 12 planes (U_I, V_I, U_J, V_J × three splits) of [64 rows][KC bf16].
// A lane's fragment (row r, 8 consecutive k) is one ds_read_b128.  KC = 16:
// rows of 8 dwords, unpadded, the two 16-byte halves of row r swapped when
// bit 3 of r is set (swz16).  That keeps both the fragment reads (ds_read_b128
// lane groups {0-3,12-15,20-27}, ... : 16 rows of one half) and the staging
// stores (ds_write_b64 groups of 16 lanes: 4 rows × 4 k-quarters, banks mod 32;
// ds_write_b128 groups of 8: 4 rows × 2 halves) on distinct banks.  The
// previous 12-dword rows (4 × odd) read conflict-free but stored 2-way
// conflicted: 12.8 M extra LDS cycles per 128-tile launch at Cora S = 8.  KC =
// 32: rows of KC/2 + 4 dwords, no swap.  Global loads of chunk c+1 are in
// flight during chunk c's MFMAs, as in the fp32 form.
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Upper halves of two dwords packed (b0 -> low half, b1 -> high half).
__device__ __forceinline__ uint32_t pack_hi16(uint32_t b0, uint32_t b1) {
    return __builtin_amdgcn_perm(b1, b0, 0x07060302u);
}

// Split a pair of fp32 values into three packed bf16 pairs.
__device__ __forceinline__ void split3_pair(float x0, float x1, uint32_t& h, uint32_t& m, uint32_t& l) {
    const uint32_t b0 = __float_as_uint(x0), b1 = __float_as_uint(x1);
    const float r0 = x0 - __uint_as_float(b0 & 0xffff0000u);
    const float r1 = x1 - __uint_as_float(b1 & 0xffff0000u);
    const uint32_t c0 = __float_as_uint(r0), c1 = __float_as_uint(r1);
    const float q0 = r0 - __uint_as_float(c0 & 0xffff0000u);
    const float q1 = r1 - __uint_as_float(c1 & 0xffff0000u);
    h = pack_hi16(b0, b1);
    m = pack_hi16(c0, c1);
    l = pack_hi16(__float_as_uint(q0), __float_as_uint(q1));
}

// Zero block that out-of-range lanes load from (rows past n, k past the end).
__device__ __attribute__((aligned(16))) float g_zero8[8];

template <int KC>
struct Bf3Stage {
    // thread t stages row t >> 2 of each block, k = (t & 3)·(KC/4) … + KC/4 - 1
    static constexpr int kPer = KC / 4;       // fp32 values per thread per array
    static constexpr bool kSwz = KC == 16;    // unpadded rows, halves swapped by row bit 3
    static constexpr int kStr = kSwz ? 8 : KC / 2 + 4;   // dwords per LDS row
    static constexpr int kPlane = 64 * kStr;  // dwords per plane
    float x[4][kPer];                         // U_I, V_I, U_J, V_J
};

template <int KC, bool VEC>
__device__ __forceinline__ void bf3_load(const float* __restrict__ u, const float* __restrict__ v, int ld,
                                         int k, int n, int gi, int gj, int k0, Bf3Stage<KC>& st) {
    constexpr int P = Bf3Stage<KC>::kPer;
    const int gk = k0 + (threadIdx.x & 3) * P;
    const float* src[4] = {u + (int64_t)gi * ld, v + (int64_t)gi * ld, u + (int64_t)gj * ld,
                           v + (int64_t)gj * ld};
    const bool rowok[4] = {gi < n, gi < n, gj < n, gj < n};
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        if constexpr (VEC) {  // branch-free, as in the 128-tile kernel below
            const float* p = (rowok[a] && gk < k) ? src[a] + gk : g_zero8;
#pragma unroll
            for (int q = 0; q < P; q += 4) {
                const float4 f = *reinterpret_cast<const float4*>(p + q);
                st.x[a][q] = f.x; st.x[a][q + 1] = f.y; st.x[a][q + 2] = f.z; st.x[a][q + 3] = f.w;
            }
        } else {
#pragma unroll
            for (int q = 0; q < P; ++q) st.x[a][q] = (rowok[a] && gk + q < k) ? src[a][gk + q] : 0.f;
        }
    }
}

// Pre-split operands (lds_theta_grad_planes): U and V carry the split3
// words of every fp32 value (split once by whoever writes a column; staging
// here is a plain copy instead of the ~14 VALU per MFMA of the split),
// chunk-major: the 16-column chunk c of row i is [hi ×16 | mid ×16 | lo ×16]
// (96 bytes) at uint16 offset (c·rows + i)·48, so the chunk of 64 (128)
// consecutive rows a tile stages is one contiguous 6 (12) KB block that a wave
// copies with fully coalesced 1 KB load instructions.  Measured at Cora S = 1
// (k = 264, engine factors written pre-split): 42.8-45 µs per launch against
// 40.7 for the fp32-operand staging, so the engine keeps fp32 factors.  The
// 64-tile kernel is bound by LDS bandwidth, not by the split VALU: per
// 16-wide chunk a block writes 24 KB and reads 48 KB of LDS for 48 MFMAs
// (1.5 KB per 32-cycle MFMA against 128 B per cycle per CU; SQ_WAIT_INST_LDS
// 15-23 % of wave cycles, MFMA busy ~22 %), the same in both forms.
struct Planes {
    const uint16_t* u;
    const uint16_t* v;
};

// 16-byte half of row r that holds logical half h in the unpadded 8-dword
// layout (see the split-bf16 comment above).
__device__ __forceinline__ int swz16(int r) { return (r >> 3) & 1; }

__host__ __device__ __forceinline__ int64_t ci_at(int64_t i, int c, int p, int64_t rows) {
    return ((int64_t)(c >> 4) * rows + i) * 48 + p * 16 + (c & 15);
}

// One wave copies NQ KB of chunk k0/16 starting at row r0 of an operand into
// LDS planes 3a..3a+2 (rows of S dwords, planes of PL dwords): lane l holds
// bytes 16m + 1024q of the block, m = 15l mod 64 — each load instruction
// still reads one contiguous KB, and with planes 4 dwords past a multiple of
// 64 banks every 16-lane group of the b128 LDS writes hits 64 distinct banks
// (with m = l the writes were 3-way conflicted: 5·10^6 conflict cycles per
// Cora launch); rows past n and half-chunks at or past k (k a multiple of 8)
// load zeros.
template <int NQ>
struct CiCopy {
    u32x4 x[NQ];
};
template <int NQ>
__device__ __forceinline__ void ci_load(const uint16_t* __restrict__ op, int rows, int r0, int k, int k0,
                                        CiCopy<NQ>& c) {
    const int m = (15 * (threadIdx.x & 63)) & 63;
    const uint16_t* blk = op + ((int64_t)(k0 >> 4) * rows + r0) * 48;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int o = 16 * m + 1024 * q;  // byte offset in the block
        const int row = o / 96, half = (o % 32) >> 4;
        const bool ok = r0 + row < rows && k0 + 8 * half < k;
        c.x[q] = ok ? *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(blk) + o)
                    : *reinterpret_cast<const u32x4*>(g_zero8);
    }
}
template <int NQ, int S, int PL>
__device__ __forceinline__ void ci_store(uint32_t* lds, int a, const CiCopy<NQ>& c) {
    const int m = (15 * (threadIdx.x & 63)) & 63;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int o = 16 * m + 1024 * q;
        const int row = o / 96, w = o % 96;
        const int half = ((w % 32) >> 4) ^ (S == 8 ? swz16(row) : 0);
        *reinterpret_cast<u32x4*>(lds + (3 * a + w / 32) * PL + row * S + 4 * half) = c.x[q];
    }
}

template <int KC>
__device__ __forceinline__ void bf3_store(uint32_t* lds, const Bf3Stage<KC>& st) {
    constexpr int P = Bf3Stage<KC>::kPer;
    constexpr int S = Bf3Stage<KC>::kStr, PL = Bf3Stage<KC>::kPlane;
    const int row = threadIdx.x >> 2, kq = threadIdx.x & 3;
    const int off = Bf3Stage<KC>::kSwz ? row * S + 4 * ((kq >> 1) ^ swz16(row)) + 2 * (kq & 1)
                                       : row * S + kq * (P / 2);
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        uint32_t h[P / 2], m[P / 2], l[P / 2];
#pragma unroll
        for (int q = 0; q < P / 2; ++q) split3_pair(st.x[a][2 * q], st.x[a][2 * q + 1], h[q], m[q], l[q]);
        uint32_t* p0 = lds + (3 * a + 0) * PL + off;
        uint32_t* p1 = lds + (3 * a + 1) * PL + off;
        uint32_t* p2 = lds + (3 * a + 2) * PL + off;
        if constexpr (P == 8) {
            *reinterpret_cast<u32x4*>(p0) = u32x4{h[0], h[1], h[2], h[3]};
            *reinterpret_cast<u32x4*>(p1) = u32x4{m[0], m[1], m[2], m[3]};
            *reinterpret_cast<u32x4*>(p2) = u32x4{l[0], l[1], l[2], l[3]};
        } else {
            *reinterpret_cast<uint2*>(p0) = uint2{h[0], h[1]};
            *reinterpret_cast<uint2*>(p1) = uint2{m[0], m[1]};
            *reinterpret_cast<uint2*>(p2) = uint2{l[0], l[1]};
        }
    }
}

// Linear id L of the XCD-grouped order -> upper-triangle block (bi <= bj):
// the nb block columns are cut into strips of G, a strip enumerated row block
// by row block (G tiles per row above its diagonal block, fewer on it).
__device__ __forceinline__ void grouped_tile(int L, int nb, int G, int& bi, int& bj) {
    // strips s of columns [sG, sG + g), g = min(G, nb - sG); tiles before strip s: T(sG)
    int s = 0;
    while (true) {
        const int c1 = min((s + 1) * G, nb);
        const int before_next = c1 * (c1 + 1) / 2;
        if (L < before_next) break;
        ++s;
    }
    const int c0 = s * G, g = min(G, nb - c0);
    int rem = L - c0 * (c0 + 1) / 2;
    if (rem < c0 * g) {  // rows above the strip's diagonal: g tiles each
        bi = rem / g;
        bj = c0 + rem % g;
        return;
    }
    rem -= c0 * g;
    int i = c0;          // diagonal part: row c0 + q has g - q tiles
    while (rem >= c0 + g - i) {
        rem -= c0 + g - i;
        ++i;
    }
    bi = i;
    bj = i + rem;
}

// The next window's graph draw, fused into the θ-grad epilogue (form 6, mode
// 2): each block draws `graphs` Bernoulli graphs from the θ values its tile
// just wrote (still in registers) — the sampler's tile draw (sampler.hip
// sample_tiles_kernel<false, true, true>) with the same Philox words per
// (row quad, column), the same bit rows / columns and degree atomics, so the
// bits are identical to lds_sample_graphs_multi on the updated θ.
struct DrawArgs {
    uint64_t* bits;   // [graphs][n][words]
    int words;
    int* dacc;        // degree accumulators, wsi ints per graph, zero on entry
    int wsi;
    uint32_t k0, k1, tag, counter;
    const uint32_t* counter_base;  // device draw counter (EngineScalars) or NULL
    int graphs;
};

template <int KC, bool VEC, bool PRE = false, bool PART = true, bool DRAW = false>
__global__ __launch_bounds__(256) void theta_grad_bf3_kernel(
    const float* __restrict__ u, const float* __restrict__ v, int ld, int k,
    const float* __restrict__ r, int ldr, int nr, float* __restrict__ theta, int n,
    float* __restrict__ grad, int mode, const double* __restrict__ lr_dev, int vec4, int ldrc,
    float gscale, int group, int per_xcd, Planes pl, DrawArgs dr = DrawArgs{}) {
    // (pre-split copies: planes 4 dwords past a multiple of 64 banks, ci_store)
    constexpr int S = Bf3Stage<KC>::kStr, PL = Bf3Stage<KC>::kPlane + (PRE ? 4 : 0);
    __shared__ __attribute__((aligned(16))) uint32_t lds[12 * PL];
    __shared__ float Ri[kTile], Rj[kTile];

    int a, b;
    if (group > 0) {  // XCD-grouped order, as in the 128-tile kernel below
        const int nb = (n + kTile - 1) / kTile;
        const int L = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
        if (L >= nb * (nb + 1) / 2) return;  // whole block: no barrier reached
        grouped_tile(L, nb, group, b, a);
    } else {
        tri_tile(blockIdx.x, a, b);
    }
    const int i0 = b * kTile, j0 = a * kTile;
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int64_t nn = n;
    const int lj = wc * 32 + (lane & 31);
    const int j = j0 + lj;

    const int gi = i0 + (t >> 2), gj = j0 + (t >> 2);
    Bf3Stage<KC> st;
    // pre-split: wave w copies operand w (U_I, V_I, U_J, V_J) of the chunk
    // (one chunk in flight: two measured slower — more registers, and the
    // kernel is bound by LDS bandwidth, ~1.5 KB of LDS traffic per MFMA)
    CiCopy<6> cc;
    const int cop = t >> 6;
    const uint16_t* cbase = (cop & 1) ? pl.v : pl.u;
    const int crow0 = cop < 2 ? i0 : j0;
    const int nch = (k + KC - 1) / KC;
    if (k > 0) {
        if constexpr (PRE) {
            ci_load<6>(cbase, n, crow0, k, 0, cc);
        } else {
            bf3_load<KC, VEC>(u, v, ld, k, n, gi, gj, 0, st);
        }
    }

    // PART (modes 1, 3): the partial grad is read too — a template flag so
    // the SGD-only launch (mode 2) keeps its 16 registers for the staging
    float th[16], part[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int i = i0 + wr * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        const bool in = i < n && j < n && j >= i;
        const int64_t idx = in ? tri_index(i, i, nn) + (j - i) : 0;
        th[e] = (in && theta != nullptr) ? theta[idx] : 0.f;
        part[e] = (PART && in && (mode == 1 || mode == 3)) ? grad[idx] : 0.f;
    }

    if (t < 2 * kTile) {
        const int rr = t & (kTile - 1);
        const int row = (t < kTile ? i0 : j0) + rr;
        float acc = 0.f;
        if (row < n)
            acc = row_r_sum(r, (int64_t)row * ldr, ldrc, nr);
        (t < kTile ? Ri : Rj)[rr] = acc;
    }

    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;

    // fragment offsets (dwords): row (wave's 32-row half + lane & 31), k-half 8·(lane >> 5)
    // (row bit 3 = lane bit 3: the rows of a fragment read are wr·32 + lane & 31)
    const int fh = Bf3Stage<KC>::kSwz ? 4 * ((lane >> 5) ^ ((lane >> 3) & 1)) : 4 * (lane >> 5);
    const int ra = (wr * 32 + (lane & 31)) * S + fh;
    const int rb = (wc * 32 + (lane & 31)) * S + fh;
    auto compute = [&](int k0) {
#pragma unroll
        for (int kk = 0; kk < KC; kk += 16) {
            if (k0 + kk < k) {  // zero-filled past k: whole k-steps beyond it are skipped
                const int o = kk / 2;
                bf16x8 fa[3], fb[3];
                // U_I × V_J
#pragma unroll
                for (int s = 0; s < 3; ++s) {
                    fa[s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(lds + (0 + s) * PL + ra + o));
                    fb[s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(lds + (9 + s) * PL + rb + o));
                }
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[1], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[2], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[0], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[1], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[0], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0], acc, 0, 0, 0);
                // V_I × U_J
#pragma unroll
                for (int s = 0; s < 3; ++s) {
                    fa[s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(lds + (3 + s) * PL + ra + o));
                    fb[s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(lds + (6 + s) * PL + rb + o));
                }
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[1], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[2], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[0], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[1], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[0], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0], acc, 0, 0, 0);
            }
        }
    };
    if constexpr (PRE) {
        static_assert(!PRE || KC == 16, "pre-split staging: 16-wide k chunks");
        for (int c = 0; c < nch; ++c) {
            __syncthreads();
            ci_store<6, S, PL>(lds, cop, cc);
            __syncthreads();
            if (c + 1 < nch) ci_load<6>(cbase, n, crow0, k, KC * (c + 1), cc);
            compute(KC * c);
        }
    } else {
        for (int k0 = 0; k0 < k; k0 += KC) {
            __syncthreads();
            bf3_store<KC>(lds, st);
            __syncthreads();
            if (k0 + KC < k) bf3_load<KC, VEC>(u, v, ld, k, n, gi, gj, k0 + KC, st);
            compute(k0);
        }
    }
    __syncthreads();

    const float lr = mode >= 2 ? (float)(*lr_dev) : 0.f;
    uint32_t thr[16];  // DRAW: the next draw's integer thresholds (sampler.hip)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int li = wr * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        const int i = i0 + li;
        thr[e] = 0u;
        if (i >= n || j >= n || j < i) continue;
        const int64_t idx = tri_index(i, i, nn) + (j - i);
        float g = 0.f;
        if (j > i) {
            const float gs = gscale * (acc[e] + Ri[li] + Rj[lj]);
            g = mode == 3 ? part[e] + gs : gs;
            if (theta != nullptr && !(th[e] >= 0.f && th[e] <= 1.f)) g = 0.f;  // clamp backward
        }
        if (mode == 3) {
            grad[idx] = g;
            theta[idx] = fminf(fmaxf(fmaf(-lr, g, th[e]), 0.f), 1.f);
        } else if (mode == 2) {
            if (grad != nullptr) grad[idx] = g;
            const float tn = fminf(fmaxf(fmaf(-lr, g, th[e]), 0.f), 1.f);
            theta[idx] = tn;
            if (DRAW && j > i) thr[e] = (uint32_t)ceilf(tn * 16777216.0f);
        } else if (mode == 1) {
            grad[idx] = part[e] + g;
        } else {
            grad[idx] = g;
        }
    }
    if constexpr (DRAW) {
        // rows of this lane: quad m = e >> 2 covers rows r4(m) .. r4(m) + 3 of column j
        // graphs in groups of four: each leaves its row words / column words
        // in LDS, then threads 64q .. 64q + 63 store graph q's (one barrier
        // pair per group)
        constexpr int kGrp = 4;
        __shared__ uint32_t rw[kGrp][64][2];   // row words: [graph][row][column half]
        __shared__ uint64_t cwp[kGrp][2][64];  // column words: [graph][wave row half][column]
        const bool diag = i0 == j0;
        const uint32_t cb = dr.counter_base != nullptr ? *dr.counter_base : 0u;
        const int rq0 = (i0 + wr * 32 + 4 * (lane >> 5)) >> 2;  // row quad of e = 0
#pragma unroll 1
        for (int base = 0; base < dr.graphs; base += kGrp) {
            const int gn = min(kGrp, dr.graphs - base);
#pragma unroll 1
            for (int q = 0; q < gn; ++q) {
                const uint32_t ctr = dr.counter + cb + (uint32_t)(base + q);
                uint32_t x[16];
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const U32x4 o = philox4x32_10(U32x4{(uint32_t)j, (uint32_t)(rq0 + 2 * m), dr.tag, ctr}, dr.k0,
                                                  dr.k1);
                    x[4 * m] = o.x;
                    x[4 * m + 1] = o.y;
                    x[4 * m + 2] = o.z;
                    x[4 * m + 3] = o.w;
                }
                uint64_t colw = 0;
                uint32_t mylo = 0, myhi = 0;  // lane e (< 16) keeps the ballot of element e
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const bool bit = (x[e] >> 8) < thr[e];
                    const uint64_t w = __ballot(bit);
                    mylo = lane == e ? (uint32_t)w : mylo;
                    myhi = lane == e ? (uint32_t)(w >> 32) : myhi;
                    colw |= (uint64_t)bit << ((e & 3) + 8 * (e >> 2) + 4 * (lane >> 5) + wr * 32);
                }
                colw |= __shfl_xor(colw, 32);  // the other row interleave of this column
                if (lane < 16) {  // element e = lane: rows r (h = 0) and r + 4 (h = 1), columns wc·32 …
                    const int r = wr * 32 + (lane & 3) + 8 * (lane >> 2);
                    rw[q][r][wc] = mylo;
                    rw[q][r + 4][wc] = myhi;
                }
                if (lane < 32) cwp[q][wr][wc * 32 + lane] = colw;
            }
            __syncthreads();
            const int q = t >> 6, tt = t & 63;
            if (q < gn) {
                uint64_t* __restrict__ gb = dr.bits + (int64_t)(base + q) * n * dr.words;
                int* __restrict__ da = dr.dacc + (int64_t)(base + q) * dr.wsi;
                const uint64_t roww = (uint64_t)rw[q][tt][0] | ((uint64_t)rw[q][tt][1] << 32);
                const int jj = j0 + tt, ii = i0 + tt;
                uint64_t out = cwp[q][0][tt] | cwp[q][1][tt];
                if (!diag) {
                    if (ii < n) {
                        gb[(int64_t)ii * dr.words + (j0 >> 6)] = roww;
                        const int pc = __popcll(roww);
                        if (pc != 0) atomicAdd(&da[ii], pc);
                    }
                } else {
                    out |= roww | (1ull << tt);  // self-loop: diagonal set to 1
                }
                if (jj < n) {
                    gb[(int64_t)jj * dr.words + (i0 >> 6)] = out;
                    const int pc = __popcll(out);
                    if (pc != 0) atomicAdd(&da[jj], pc);
                }
            }
            if (base + kGrp < dr.graphs) __syncthreads();  // rw / cwp reused by the next group
        }
    }
}

// ---------------------------------------------------------------------------
// Split-bf16, 128 × 128 tiles: the 64 × 64 forms above re-read U and V once
// per 64 output columns, 16 fp32-equivalent flop per staged byte, and at
// n = 20 000 (42 MB of U, V against a 4 MB L2 per XCD) that stream from the
// Infinity Cache, not the MFMAs, sets the time.  Here a 256-thread block owns
// a 128 × 128 tile (each wave a 64 × 64 quarter: 2 × 2 accumulators of
// 32 × 32), staging 16-wide k chunks of the 12 bf16 planes (48 KB of LDS;
// 2 blocks per CU, VGPR-bound): 32 flop per byte, 48 MFMAs per wave between barriers.
// Tile order (`group` > 0): the triangle's block columns are cut into strips
// of `group` columns, a strip enumerated row block by row block, and each XCD
// (blocks b, b + 8, … share one) takes a contiguous range of that order, so
// the ≈64 tiles an XCD runs at once span ≈8 row blocks × `group` column
// blocks and share their U, V rows in its L2.
// ---------------------------------------------------------------------------
constexpr int kT2 = 128;
constexpr int kS2 = 8;              // dwords per LDS row, unpadded, halves swapped by row bit 3 (swz16)
constexpr int kPL2 = kT2 * kS2;     // dwords per plane (pre-split copies: + 4, see ci_store)

// Packed index of (i, j), i <= j, in 32-bit arithmetic (the epilogue's 64
// index computations per lane are 64-bit multiplies otherwise).  i(2n - i + 1)
// peaks at (n-1)(n+2) < 2^32 for n <= 65 535; the launch uses it for
// n <= 46 340, where n(n+1) < 2^31 (so the packed index itself also fits an
// int32), and the 64-bit path above that (form 7 forces it for testing).
template <bool SMALL>
__device__ __forceinline__ int64_t tri_at_t(int i, int j, int64_t n) {
    if constexpr (SMALL) {
        const uint32_t ui = (uint32_t)i, un = (uint32_t)n;
        return (int64_t)((ui * (2u * un - ui + 1u)) >> 1) + (j - i);
    } else {
        return tri_index(i, i, n) + (j - i);
    }
}

// Epilogue of the 128-tile kernels (wave (wr, wc) owns outputs wr·64 … + 63 ×
// wc·64 … + 63 of the tile): dθ = gscale·(acc + R_i + R_j) on the strict upper
// triangle, clamp-backward mask, then the mode's stores.
template <bool SMALL, bool DRAW = false>
__device__ __forceinline__ void t128_epilogue(const f32x16 (&acc)[2][2], const float* Ri, const float* Rj,
                                              float* __restrict__ theta, float* __restrict__ grad, int n,
                                              int mode, const double* __restrict__ lr_dev, float gscale,
                                              int i0, int j0, int wr, int wc, int lane,
                                              uint32_t (*thr)[2][16] = nullptr) {
    if constexpr (DRAW) mode = 2;  // (every DRAW launch is mode 2: the mode branches fold)
    const int64_t nn = n;
    auto tri_at = [](int i, int j, int64_t nn_) { return tri_at_t<SMALL>(i, j, nn_); };
    // Epilogue: every θ (and partial-grad) operand of the wave's 64 outputs is
    // loaded before the first store — a load after a store to the same array
    // cannot be hoisted above it, and per-element load → store chains cost one
    // memory latency each (1.1 ms of 2.5 at n = 20 000 before this).
    const bool need_part = mode == 1 || mode == 3;
    float th[2][2][16], part[2][2][16];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int j = j0 + wc * 64 + q * 32 + (lane & 31);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int i = i0 + wr * 64 + m * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
                const bool in = i < n && j < n && j >= i;
                const int64_t id = in ? tri_at(i, j, nn) : 0;
                th[m][q][e] = (in && theta != nullptr) ? theta[id] : 0.f;
                part[m][q][e] = (in && need_part) ? grad[id] : 0.f;
            }
        }
    __syncthreads();  // Ri / Rj written by other waves

    const float lr = mode >= 2 ? (float)(*lr_dev) : 0.f;
    // R sums read outside the per-element branches: the column's two once,
    // the rows' as one 16-byte read per run of four consecutive rows (shared
    // by both column halves) — inside the branches every element paid an LDS
    // round trip of its own
    const float rj[2] = {Rj[wc * 64 + (lane & 31)], Rj[wc * 64 + 32 + (lane & 31)]};
    // an off-diagonal tile inside the triangle takes the loop without bounds
    // and diagonal tests (kIn); here in every launch — the lambda form, which
    // the register allocator fits in 256 VGPRs without spilling (a function
    // template spilled)
    auto elements = [&](auto in_c) {
        constexpr bool kIn = decltype(in_c)::value;
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) {
                const float4 r4 = *reinterpret_cast<const float4*>(Ri + wr * 64 + m * 32 + 8 * qd + 4 * (lane >> 5));
                const float ri4[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int j = j0 + wc * 64 + q * 32 + (lane & 31);
#pragma unroll
                    for (int e4 = 0; e4 < 4; ++e4) {
                        const int e = 4 * qd + e4;
                        const int i = i0 + wr * 64 + m * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
                        if constexpr (DRAW) thr[m][q][e] = 0u;
                        if (!kIn && (i >= n || j >= n || j < i)) continue;
                        const int64_t id = tri_at(i, j, nn);
                        const float t0 = th[m][q][e];
                        float g = 0.f;
                        if (kIn || j > i) {
                            const float gs = gscale * (acc[m][q][e] + ri4[e4] + rj[q]);
                            g = mode == 3 ? part[m][q][e] + gs : gs;
                            if (theta != nullptr && !(t0 >= 0.f && t0 <= 1.f)) g = 0.f;  // clamp backward
                        }
                        if (mode == 3) {
                            grad[id] = g;
                            theta[id] = fminf(fmaxf(fmaf(-lr, g, t0), 0.f), 1.f);
                        } else if (mode == 2) {
                            if (grad != nullptr) grad[id] = g;
                            const float tn = fminf(fmaxf(fmaf(-lr, g, t0), 0.f), 1.f);
                            theta[id] = tn;
                            // the next draw's integer threshold (sampler.hip): bit iff (x >> 8) < ceil(θ·2^24)
                            if constexpr (DRAW) thr[m][q][e] = (kIn || j > i) ? (uint32_t)ceilf(tn * 16777216.0f) : 0u;
                        } else if (mode == 1) {
                            grad[id] = part[m][q][e] + g;
                        } else {
                            grad[id] = g;
                        }
                    }
                }
            }
    };
    if (i0 != j0 && j0 + kT2 <= n) elements(BoolC<true>{});
    else elements(BoolC<false>{});
}

// The next window's draw from the θ a 128-tile epilogue just wrote (mode 2;
// lds_theta_grad_sgd_draw at 128-tile shapes, config 5): the sampler's Philox
// words per (row quad, column) — each lane's 16 outputs of a 32 × 32
// accumulator are 4 row quads of one column, the sampler tile kernel's counter
// shape — the same integer compare, bit rows by ballot (32-column segments,
// four per 128-column row, joined in LDS), column words from each lane's own
// bits, then one 16-byte store per (graph, row) of the tile's two words and one
// degree atomic: the bits and degrees of lds_sample_graphs_multi on the
// updated θ.  `lds` is the dead staging buffer (>= 32 KB).
constexpr int kT128Grp = 8;  // graphs per draw group (4 KB of LDS each)

__device__ __forceinline__ void t128_draw(const uint32_t (&thr)[2][2][16], uint32_t* lds, const DrawArgs& dr, int n,
                                          int i0, int j0, int wr, int wc, int lane, int t) {
    uint32_t* const rwb = lds;                                                 // [grp][128 rows][4 segs]
    uint64_t* const cwb = reinterpret_cast<uint64_t*>(lds + kT128Grp * 512);  // [grp][2 halves][128 cols]
    const bool diag = i0 == j0;
    const uint32_t cb = dr.counter_base != nullptr ? *dr.counter_base : 0u;
#pragma unroll 1
    for (int base = 0; base < dr.graphs; base += kT128Grp) {
        const int gn = min(kT128Grp, dr.graphs - base);
        __syncthreads();  // the stage buffer (first group) / the previous group's words are consumed
#pragma unroll 1
        for (int q = 0; q < gn; ++q) {
            const uint32_t ctr = dr.counter + cb + (uint32_t)(base + q);
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                const uint32_t j = (uint32_t)(j0 + wc * 64 + qq * 32 + (lane & 31));
                uint64_t colw = 0;  // rows wr·64 … + 63 of column j
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    const int rq0 = (i0 + wr * 64 + m * 32 + 4 * (lane >> 5)) >> 2;  // row quad of e = 0
                    uint32_t x[16];
#pragma unroll
                    for (int qd = 0; qd < 4; ++qd) {
                        const U32x4 o = philox4x32_10(U32x4{j, (uint32_t)(rq0 + 2 * qd), dr.tag, ctr}, dr.k0, dr.k1);
                        x[4 * qd] = o.x;
                        x[4 * qd + 1] = o.y;
                        x[4 * qd + 2] = o.z;
                        x[4 * qd + 3] = o.w;
                    }
                    uint32_t cbits = 0;  // bit e: this lane's element e (as in w8_epilogue)
#pragma unroll
                    for (int e = 15; e >= 0; --e) {
                        const bool bit = (x[e] >> 8) < thr[m][qq][e];
                        const uint64_t w = __ballot(bit);
                        cbits = (cbits << 1) + (uint32_t)bit;
                        if (lane == 0) {  // the ballot's words: rows rr and rr + 4, column segment wc·2 + qq
                            const int rr = wr * 64 + m * 32 + (e & 3) + 8 * (e >> 2);
                            rwb[(q * 128 + rr) * 4 + wc * 2 + qq] = (uint32_t)w;
                            rwb[(q * 128 + rr + 4) * 4 + wc * 2 + qq] = (uint32_t)(w >> 32);
                        }
                    }
                    cbits = (cbits | (cbits << 8)) & 0x00FF00FFu;
                    cbits = (cbits | (cbits << 4)) & 0x0F0F0F0Fu;
                    colw |= (uint64_t)(cbits << (4 * (lane >> 5))) << (32 * m);
                }
                colw |= __shfl_xor(colw, 32);  // the other row interleave of this column
                if (lane < 32) cwb[(q * 2 + wr) * 128 + wc * 64 + qq * 32 + lane] = colw;
            }
        }
        __syncthreads();
        // one (row, two words) pair per work item: rows of I (part 0), rows of J (part 1)
        for (int it = t; it < gn * 256; it += 256) {
            const int q = it >> 8, part1 = (it >> 7) & 1, x = it & 127;
            if (diag && part1) continue;
            const int row = (part1 ? j0 : i0) + x;
            if (row >= n) continue;
            uint64_t* __restrict__ gb = dr.bits + (int64_t)(base + q) * n * dr.words;
            int* __restrict__ da = dr.dacc + (int64_t)(base + q) * dr.wsi;
            const uint32_t* rws = rwb + (q * 128 + x) * 4;
            uint64_t w0, w1;
            int wbase;
            if (part1) {  // column x of J: its rows of I (the mirrored entries)
                w0 = cwb[(q * 2 + 0) * 128 + x];
                w1 = cwb[(q * 2 + 1) * 128 + x];
                wbase = i0 >> 6;
            } else {
                w0 = (uint64_t)rws[0] | ((uint64_t)rws[1] << 32);
                w1 = (uint64_t)rws[2] | ((uint64_t)rws[3] << 32);
                wbase = j0 >> 6;
                if (diag) {  // strict upper (row words) | strict lower (column words) | self-loop
                    w0 |= cwb[(q * 2 + 0) * 128 + x];
                    w1 |= cwb[(q * 2 + 1) * 128 + x];
                    if (x < 64) w0 |= 1ull << x;
                    else w1 |= 1ull << (x - 64);
                }
            }
            *reinterpret_cast<ulonglong2*>(gb + (int64_t)row * dr.words + wbase) = ulonglong2{w0, w1};
            const int pc = __popcll(w0) + __popcll(w1);
            if (pc != 0) atomicAdd(&da[row], pc);
        }
    }
}

template <bool VEC, bool SMALL = false, bool PRE = false, bool DRAW = false>
__global__ __launch_bounds__(256, 2) void theta_grad_bf3_t128_kernel(
    const float* __restrict__ u, const float* __restrict__ v, int ld, int k,
    const float* __restrict__ r, int ldr, int nr, float* __restrict__ theta, int n,
    float* __restrict__ grad, int mode, const double* __restrict__ lr_dev, int vec4, int ldrc,
    float gscale, int group, int per_xcd, Planes pl, DrawArgs dr = DrawArgs{}) {
    constexpr int kPL = kPL2 + (PRE ? 4 : 0);
    __shared__ __attribute__((aligned(16))) uint32_t lds[12 * kPL];
    __shared__ __attribute__((aligned(16))) float Ri[kT2], Rj[kT2];

    const int nb = (n + kT2 - 1) / kT2;
    const int ntiles = nb * (nb + 1) / 2;
    int bi, bj;
    if (group > 0) {
        const int L = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
        if (L >= ntiles) return;  // whole block: no barrier reached
        grouped_tile(L, nb, group, bi, bj);
    } else if (group < 0) {  // a row band's tiles: block rows -group - 1 … (the grid is the band's tile count)
        band_tile((int)blockIdx.x, nb, -group - 1, bi, bj);
    } else {
        int a, b;
        tri_tile(blockIdx.x, a, b);
        bi = b;
        bj = a;
    }
    const int i0 = bi * kT2, j0 = bj * kT2;
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    const int wr = wave >> 1, wc = wave & 1;

    // staging: thread t owns row t >> 1 of both blocks, k = 8·(t & 1) … + 7 of the chunk
    const int srow = t >> 1, sk = (t & 1) * 8;
    const int gi = i0 + srow, gj = j0 + srow;
    const float* src[4] = {u + (int64_t)gi * ld, v + (int64_t)gi * ld, u + (int64_t)gj * ld,
                           v + (int64_t)gj * ld};
    const bool rowok[4] = {gi < n, gi < n, gj < n, gj < n};
    // two register sets: chunk c + 2 loads while chunk c is staged and computed
    float xa[4][8], xb[4][8];
    // VEC (k % 8 == 0, 16-byte aligned rows): branch-free — rows past n and k
    // past the end load from a zero block instead, so nothing consumes the
    // loaded values before the next barrier and the next chunk's loads stay in
    // flight through this chunk's MFMAs (divergent load paths, or a select on
    // the loaded value, made the compiler wait on them right away).
    auto load = [&](float (&x)[4][8], int k0) {
        const int gk = k0 + sk;
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            if constexpr (VEC) {
                const float* p = (rowok[a] && gk < k) ? src[a] + gk : g_zero8;
                const float4 f0 = *reinterpret_cast<const float4*>(p);
                const float4 f1 = *reinterpret_cast<const float4*>(p + 4);
                x[a][0] = f0.x; x[a][1] = f0.y; x[a][2] = f0.z; x[a][3] = f0.w;
                x[a][4] = f1.x; x[a][5] = f1.y; x[a][6] = f1.z; x[a][7] = f1.w;
            } else {
#pragma unroll
                for (int q = 0; q < 8; ++q) x[a][q] = (rowok[a] && gk + q < k) ? src[a][gk + q] : 0.f;
            }
        }
    };
    // pre-split: wave w copies operand w (U_I, V_I, U_J, V_J) of the chunk: 12 KB
    CiCopy<12> pa_, pb_;
    const int cop = t >> 6;
    const uint16_t* cbase = (cop & 1) ? pl.v : pl.u;
    const int crow0 = cop < 2 ? i0 : j0;
    auto pload = [&](CiCopy<12>& x, int k0) { ci_load<12>(cbase, n, crow0, k, k0, x); };
    auto pstage = [&](const CiCopy<12>& x) { ci_store<12, kS2, kPL>(lds, cop, x); };
    if constexpr (PRE) {
        if (k > 0) pload(pa_, 0);
        if (k > 16) pload(pb_, 16);
    } else {
        if (k > 0) load(xa, 0);
        if (k > 16) load(xb, 16);
    }

    if (t < 2 * kT2) {
        const int rr = t & (kT2 - 1);
        const int row = (t < kT2 ? i0 : j0) + rr;
        float acc = 0.f;
        if (row < n)
            acc = row_r_sum(r, (int64_t)row * ldr, ldrc, nr);
        (t < kT2 ? Ri : Rj)[rr] = acc;
    }

    f32x16 acc[2][2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[m][q][e] = 0.f;

    const int soff = srow * kS2 + 4 * ((t & 1) ^ swz16(srow));
    const int fo = 4 * ((lane >> 5) ^ ((lane >> 3) & 1));  // rows wr·64 (+32) + lane & 31: bit 3 = lane bit 3
    const int ra0 = (wr * 64 + (lane & 31)) * kS2 + fo, ra1 = ra0 + 32 * kS2;
    const int rb0 = (wc * 64 + (lane & 31)) * kS2 + fo, rb1 = rb0 + 32 * kS2;
    auto stage = [&](const float (&x)[4][8]) {
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            uint32_t h[4], m[4], l[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) split3_pair(x[a][2 * q], x[a][2 * q + 1], h[q], m[q], l[q]);
            *reinterpret_cast<u32x4*>(lds + (3 * a + 0) * kPL + soff) = u32x4{h[0], h[1], h[2], h[3]};
            *reinterpret_cast<u32x4*>(lds + (3 * a + 1) * kPL + soff) = u32x4{m[0], m[1], m[2], m[3]};
            *reinterpret_cast<u32x4*>(lds + (3 * a + 2) * kPL + soff) = u32x4{l[0], l[1], l[2], l[3]};
        }
    };
    auto compute = [&]() {
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {  // pr 0: U_I × V_J (planes 0-2, 9-11); pr 1: V_I × U_J (3-5, 6-8)
            const int pa = pr == 0 ? 0 : 3, pb = pr == 0 ? 9 : 6;
            bf16x8 fa[2][3], fb[2][3];
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                fa[0][s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(lds + (pa + s) * kPL + ra0));
                fa[1][s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(lds + (pa + s) * kPL + ra1));
                fb[0][s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(lds + (pb + s) * kPL + rb0));
                fb[1][s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(lds + (pb + s) * kPL + rb1));
            }
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    f32x16 c = acc[m][q];
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][1], fb[q][1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][0], fb[q][2], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][2], fb[q][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][0], fb[q][1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][1], fb[q][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][0], fb[q][0], c, 0, 0, 0);
                    acc[m][q] = c;
                }
        }
    };
    for (int k0 = 0; k0 < k; k0 += 32) {
        __syncthreads();  // the previous chunk's fragment reads are done
        if constexpr (PRE) pstage(pa_);
        else stage(xa);
        __syncthreads();
        if (k0 + 32 < k) {
            if constexpr (PRE) pload(pa_, k0 + 32);
            else load(xa, k0 + 32);
        }
        compute();
        if (k0 + 16 >= k) break;
        __syncthreads();
        if constexpr (PRE) pstage(pb_);
        else stage(xb);
        __syncthreads();
        if (k0 + 48 < k) {
            if constexpr (PRE) pload(pb_, k0 + 48);
            else load(xb, k0 + 48);
        }
        compute();
    }
    if constexpr (DRAW) {
        uint32_t thr[2][2][16];
        t128_epilogue<SMALL, true>(acc, Ri, Rj, theta, grad, n, mode, lr_dev, gscale, i0, j0, wr, wc, lane, thr);
        t128_draw(thr, lds, dr, n, i0, j0, wr, wc, lane, t);
    } else {
        t128_epilogue<SMALL>(acc, Ri, Rj, theta, grad, n, mode, lr_dev, gscale, i0, j0, wr, wc, lane);
    }
}

// ---------------------------------------------------------------------------
// Software-pipelined 128 × 128 form (form 8).  Ablations of the 64-tile
// kernel at Cora S = 16 (k = 4224) put half its time in the staging phase: with
// the LDS stores skipped 546 -> 281 µs, with the bf16 split skipped (stores
// kept) 509 µs, with the MFMAs skipped 396 µs.  Between its two barriers a
// chunk's split + LDS stores run while no MFMA of the block can issue, and the
// resident blocks reach those phases together.  Here the LDS stage is double
// buffered (2 × 48 KB, dynamic LDS, one block per CU): while a wave reads
// buffer c & 1 and runs chunk c's 48 MFMAs, it splits chunk c + 1 (loaded two
// chunks earlier) and stores it into the other buffer; one barrier per chunk.
// Chunk c + 3's loads are issued after that store, into the registers it
// freed.  Same chunks, same LDS rows, same MFMA order as form 5: identical bits.
// ---------------------------------------------------------------------------
constexpr int kPipeLds = 2 * 12 * kPL2 * 4;  // bytes of the two stage buffers

template <bool SMALL>
__global__ __launch_bounds__(256, 1) void theta_grad_bf3_pipe_kernel(
    const float* __restrict__ u, const float* __restrict__ v, int ld, int k,
    const float* __restrict__ r, int ldr, int nr, float* __restrict__ theta, int n,
    float* __restrict__ grad, int mode, const double* __restrict__ lr_dev, int ldrc,
    float gscale, int group, int per_xcd) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_dyn[];
    __shared__ __attribute__((aligned(16))) float Ri[kT2], Rj[kT2];

    const int nb = (n + kT2 - 1) / kT2;
    const int ntiles = nb * (nb + 1) / 2;
    int bi, bj;
    {
        const int L = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
        if (L >= ntiles) return;  // whole block: no barrier reached
        grouped_tile(L, nb, group, bi, bj);
    }
    const int i0 = bi * kT2, j0 = bj * kT2;
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    const int wr = wave >> 1, wc = wave & 1;

    // staging: thread t owns row t >> 1 of both blocks, k = 8·(t & 1) … + 7 of
    // the chunk; branch-free loads (rows past n and k past the end read zeros)
    const int srow = t >> 1, sk = (t & 1) * 8;
    const int gi = i0 + srow, gj = j0 + srow;
    const float* src[4] = {u + (int64_t)gi * ld, v + (int64_t)gi * ld, u + (int64_t)gj * ld,
                           v + (int64_t)gj * ld};
    const bool rowok[4] = {gi < n, gi < n, gj < n, gj < n};
    auto load = [&](float (&x)[4][8], int k0) {
        const int gk = k0 + sk;
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const float* p = (rowok[a] && gk < k) ? src[a] + gk : g_zero8;
            const float4 f0 = *reinterpret_cast<const float4*>(p);
            const float4 f1 = *reinterpret_cast<const float4*>(p + 4);
            x[a][0] = f0.x; x[a][1] = f0.y; x[a][2] = f0.z; x[a][3] = f0.w;
            x[a][4] = f1.x; x[a][5] = f1.y; x[a][6] = f1.z; x[a][7] = f1.w;
        }
    };
    const int soff = srow * kS2 + 4 * ((t & 1) ^ swz16(srow));
    auto stage = [&](uint32_t* buf, const float (&x)[4][8]) {
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            uint32_t h[4], m[4], l[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) split3_pair(x[a][2 * q], x[a][2 * q + 1], h[q], m[q], l[q]);
            *reinterpret_cast<u32x4*>(buf + (3 * a + 0) * kPL2 + soff) = u32x4{h[0], h[1], h[2], h[3]};
            *reinterpret_cast<u32x4*>(buf + (3 * a + 1) * kPL2 + soff) = u32x4{m[0], m[1], m[2], m[3]};
            *reinterpret_cast<u32x4*>(buf + (3 * a + 2) * kPL2 + soff) = u32x4{l[0], l[1], l[2], l[3]};
        }
    };
    const int fo = 4 * ((lane >> 5) ^ ((lane >> 3) & 1));
    const int ra0 = (wr * 64 + (lane & 31)) * kS2 + fo, ra1 = ra0 + 32 * kS2;
    const int rb0 = (wc * 64 + (lane & 31)) * kS2 + fo, rb1 = rb0 + 32 * kS2;
    f32x16 acc[2][2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[m][q][e] = 0.f;
    // chunk c from `cur`, overlapped with the stage of the next chunk into `nxt`
    auto step = [&](const uint32_t* cur, uint32_t* nxt, const float (&x)[4][8]) {
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {  // pr 0: U_I × V_J (planes 0-2, 9-11); pr 1: V_I × U_J (3-5, 6-8)
            const int pa = pr == 0 ? 0 : 3, pb = pr == 0 ? 9 : 6;
            bf16x8 fa[2][3], fb[2][3];
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                fa[0][s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(cur + (pa + s) * kPL2 + ra0));
                fa[1][s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(cur + (pa + s) * kPL2 + ra1));
                fb[0][s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(cur + (pb + s) * kPL2 + rb0));
                fb[1][s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(cur + (pb + s) * kPL2 + rb1));
            }
            // half of the next chunk's stage (operands 2pr, 2pr + 1) beside these MFMAs
#pragma unroll
            for (int a = 2 * pr; a < 2 * pr + 2; ++a) {
                uint32_t h[4], m[4], l[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) split3_pair(x[a][2 * q], x[a][2 * q + 1], h[q], m[q], l[q]);
                *reinterpret_cast<u32x4*>(nxt + (3 * a + 0) * kPL2 + soff) = u32x4{h[0], h[1], h[2], h[3]};
                *reinterpret_cast<u32x4*>(nxt + (3 * a + 1) * kPL2 + soff) = u32x4{m[0], m[1], m[2], m[3]};
                *reinterpret_cast<u32x4*>(nxt + (3 * a + 2) * kPL2 + soff) = u32x4{l[0], l[1], l[2], l[3]};
            }
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    f32x16 c = acc[m][q];
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][1], fb[q][1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][0], fb[q][2], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][2], fb[q][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][0], fb[q][1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][1], fb[q][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][0], fb[q][0], c, 0, 0, 0);
                    acc[m][q] = c;
                }
        }
    };

    uint32_t* const b0 = lds_dyn;
    uint32_t* const b1 = lds_dyn + 12 * kPL2;
    float xa[4][8], xb[4][8];
    const int nch = (k + 15) / 16;
    if (nch > 0) {
        load(xa, 0);
        load(xb, 16);
    }
    if (t < 2 * kT2) {
        const int rr = t & (kT2 - 1);
        const int row = (t < kT2 ? i0 : j0) + rr;
        float racc = 0.f;
        if (row < n) racc = row_r_sum(r, (int64_t)row * ldr, ldrc, nr);
        (t < kT2 ? Ri : Rj)[rr] = racc;
    }
    if (nch > 0) {
        stage(b0, xa);
        load(xa, 32);
    }
    __syncthreads();
    // chunk c: buffer c & 1 holds it; registers xb (c even) / xa (c odd) hold c + 1
    for (int c = 0; c < nch; c += 2) {
        step(b0, b1, xb);
        load(xb, 16 * (c + 3));
        __syncthreads();
        if (c + 1 >= nch) break;
        step(b1, b0, xa);
        load(xa, 16 * (c + 4));
        __syncthreads();
    }
    t128_epilogue<SMALL>(acc, Ri, Rj, theta, grad, n, mode, lr_dev, gscale, i0, j0, wr, wc, lane);
}

constexpr int kW8Lds = 2 * 12 * kPL2 * 4;  // bytes of the two stage buffers (96 KB)
constexpr int kW8Grp = 8;                  // graphs per draw group (4 KB of LDS each)

// w8_epilogue's element loop: dθ = gscale·(acc + R_i + R_j) on the strict
// upper triangle, clamp-backward mask, the mode's stores and (DRAW) the
// next draw's thresholds.  IN: an off-diagonal tile inside the triangle, no
// bounds or diagonal tests.
template <bool SMALL, bool DRAW, bool IN>
__device__ __forceinline__ void w8_elements(const f32x16 (&acc)[2], const float (&th)[2][16],
                                            const float (&part)[2][16], const float (&ri)[2][16], float rj,
                                            float* __restrict__ theta, float* __restrict__ grad, int n, int mode,
                                            float lr, float gscale, int i0, int j, int wr, int lane,
                                            uint32_t (&thr)[2][16]) {
    const int64_t nn = n;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int i = i0 + wr * 64 + m * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
            thr[m][e] = 0u;
            if (!IN && (i >= n || j >= n || j < i)) continue;
            const int64_t id = tri_at_t<SMALL>(i, j, nn);
            const float t0 = th[m][e];
            float g = 0.f;
            if (IN || j > i) {
                const float gs = gscale * (acc[m][e] + ri[m][e] + rj);
                g = mode == 3 ? part[m][e] + gs : gs;
                if (theta != nullptr && !(t0 >= 0.f && t0 <= 1.f)) g = 0.f;  // clamp backward
            }
            if (mode == 3) {
                grad[id] = g;
                theta[id] = fminf(fmaxf(fmaf(-lr, g, t0), 0.f), 1.f);
            } else if (mode == 2) {
                if (grad != nullptr) grad[id] = g;
                const float tn = fminf(fmaxf(fmaf(-lr, g, t0), 0.f), 1.f);
                theta[id] = tn;
                if (DRAW && (IN || j > i)) thr[m][e] = (uint32_t)ceilf(tn * 16777216.0f);
            } else if (mode == 1) {
                grad[id] = part[m][e] + g;
            } else {
                grad[id] = g;
            }
        }
}

// Epilogue of the eight-wave 128-tile kernels (forms 9 and 10; wave (wr, wc)
// owns outputs wr·64 … + 63 × wc·32 … + 31 of the tile, lane column j): dθ =
// gscale·(acc + R_i + R_j) on the strict upper triangle, clamp-backward mask,
// the mode's stores and, with DRAW (mode 2), the next window's draw from the
// θ just written, its words joined in the dead stage buffers (`lds_dyn`).
template <bool SMALL, bool DRAW>
__device__ __forceinline__ void w8_epilogue(const f32x16 (&acc)[2], const float (&th)[2][16],
                                            const float (&part)[2][16], const float* Ri, const float* Rj,
                                            float* __restrict__ theta, float* __restrict__ grad, int n, int mode,
                                            const double* __restrict__ lr_dev, float gscale, int i0, int j0, int wr,
                                            int wc, int lane, int t, uint32_t* lds_dyn, const DrawArgs& dr) {
    if constexpr (DRAW) mode = 2;  // (every DRAW launch is mode 2: the mode branches fold)
    const int jl = wc * 32 + (lane & 31);
    const int j = j0 + jl;
    auto row_of = [&](int m, int e) { return wr * 64 + m * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5); };
    const float lr = mode >= 2 ? (float)(*lr_dev) : 0.f;
    // the R sums of this lane's 32 rows (four runs of four consecutive rows
    // per accumulator: 16-byte reads) and of its column, read together ahead
    // of the element loop — inside it each element's two dependent reads sat
    // behind its own branch, an LDS round trip per element
    float ri[2][16];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 r4 = *reinterpret_cast<const float4*>(Ri + row_of(m, 4 * q));
            ri[m][4 * q] = r4.x;
            ri[m][4 * q + 1] = r4.y;
            ri[m][4 * q + 2] = r4.z;
            ri[m][4 * q + 3] = r4.w;
        }
    const float rj = Rj[jl];
    uint32_t thr[2][16];  // DRAW: the next draw's integer thresholds (sampler.hip)
    // an off-diagonal tile inside the triangle (every i < j < n: all but the
    // diagonal and the last column of tiles) takes the loop without bounds
    // and diagonal tests — in draw launches only, where the mode is folded
    if constexpr (DRAW) {
        if (i0 != j0 && j0 + kT2 <= n)
            w8_elements<SMALL, DRAW, true>(acc, th, part, ri, rj, theta, grad, n, mode, lr, gscale, i0, j, wr, lane, thr);
        else
            w8_elements<SMALL, DRAW, false>(acc, th, part, ri, rj, theta, grad, n, mode, lr, gscale, i0, j, wr, lane, thr);
    } else {
        w8_elements<SMALL, DRAW, false>(acc, th, part, ri, rj, theta, grad, n, mode, lr, gscale, i0, j, wr, lane, thr);
    }
    if constexpr (DRAW) {
        // LDS (the dead stage buffers): per graph of a group, row segments
        // rw[row][wc] (uint32: 32 columns) and column words cw[h][col] (uint64:
        // 64 rows of half h)
        uint32_t* const rwb = lds_dyn;                                              // kW8Grp × 128 × 4
        uint64_t* const cwb = reinterpret_cast<uint64_t*>(lds_dyn + kW8Grp * 512);  // kW8Grp × 2 × 128
        const bool diag = i0 == j0;
        const uint32_t cb = dr.counter_base != nullptr ? *dr.counter_base : 0u;
#pragma unroll 1
        for (int base = 0; base < dr.graphs; base += kW8Grp) {
            const int gn = min(kW8Grp, dr.graphs - base);
            __syncthreads();  // the stage buffers (first group) / the previous group's words are consumed
            // two graphs per pass: both accumulators' eight Philox calls of
            // each graph (sixteen chains per lane) issued together — at two
            // waves per SIMD the rounds' multiply latency needs the ILP
#pragma unroll 1
            for (int q = 0; q < gn; q += 2) {
                const int gq = min(2, gn - q);  // wave-uniform
                uint32_t x[2][2][16];
#pragma unroll
                for (int gg = 0; gg < 2; ++gg) {
                    if (gg >= gq) break;
                    const uint32_t ctr = dr.counter + cb + (uint32_t)(base + q + gg);
#pragma unroll
                    for (int m = 0; m < 2; ++m) {
                        const int rq0 = (i0 + wr * 64 + m * 32 + 4 * (lane >> 5)) >> 2;  // row quad of e = 0
#pragma unroll
                        for (int qd = 0; qd < 4; ++qd) {
                            const U32x4 o = philox4x32_10(
                                U32x4{(uint32_t)j, (uint32_t)(rq0 + 2 * qd), dr.tag, ctr}, dr.k0, dr.k1);
                            x[gg][m][4 * qd] = o.x;
                            x[gg][m][4 * qd + 1] = o.y;
                            x[gg][m][4 * qd + 2] = o.z;
                            x[gg][m][4 * qd + 3] = o.w;
                        }
                    }
                }
#pragma unroll
                for (int gg = 0; gg < 2; ++gg) {
                    if (gg >= gq) break;
                    const int qg = q + gg;
                    uint64_t colw = 0;
#pragma unroll
                    for (int m = 0; m < 2; ++m) {
                        uint32_t cb = 0;  // bit e: this lane's element e (shift-and-add chain)
#pragma unroll
                        for (int e = 15; e >= 0; --e) {
                            const bool bit = (x[gg][m][e] >> 8) < thr[m][e];
                            const uint64_t w = __ballot(bit);
                            cb = (cb << 1) + (uint32_t)bit;
                            if (lane == 0) {  // the ballot's words: rows rr and rr + 4 of columns wc·32 …
                                const int rr = wr * 64 + m * 32 + (e & 3) + 8 * (e >> 2);
                                rwb[(qg * 128 + rr) * 4 + wc] = (uint32_t)w;
                                rwb[(qg * 128 + rr + 4) * 4 + wc] = (uint32_t)(w >> 32);
                            }
                        }
                        // element e is row (e & 3) + 8·(e >> 2) + 4·(lane >> 5) of the
                        // accumulator: nibble t of cb to bits 8t … 8t + 3, then the
                        // lane half's 4-row offset.  With the ballots stored by lane 0
                        // as they come (no lane-select masks, no per-word v_mov +
                        // v_cndmask) the draw's bit assembly is ≈ 1 µs shorter at Cora
                        // (tools/microbench/tg_fixed_cost.py; bits unchanged)
                        cb = (cb | (cb << 8)) & 0x00FF00FFu;
                        cb = (cb | (cb << 4)) & 0x0F0F0F0Fu;
                        colw |= (uint64_t)(cb << (4 * (lane >> 5))) << (32 * m);
                    }
                    colw |= __shfl_xor(colw, 32);  // the other row interleave of this column
                    if (lane < 32) cwb[(qg * 2 + wr) * 128 + wc * 32 + lane] = colw;
                }
            }
            __syncthreads();
            // one (row, two words) pair per work item: rows of I (part 0), rows of J (part 1)
            for (int it = t; it < gn * 256; it += 512) {
                const int q = it >> 8, part1 = (it >> 7) & 1, x = it & 127;
                if (diag && part1) continue;
                const int row = (part1 ? j0 : i0) + x;
                if (row >= n) continue;
                uint64_t* __restrict__ gb = dr.bits + (int64_t)(base + q) * n * dr.words;
                int* __restrict__ da = dr.dacc + (int64_t)(base + q) * dr.wsi;
                const uint32_t* rws = rwb + (q * 128 + x) * 4;
                uint64_t w0, w1;
                int wbase;
                if (part1) {  // column x of J: its rows of I (the mirrored entries)
                    w0 = cwb[(q * 2 + 0) * 128 + x];
                    w1 = cwb[(q * 2 + 1) * 128 + x];
                    wbase = i0 >> 6;
                } else {
                    w0 = (uint64_t)rws[0] | ((uint64_t)rws[1] << 32);
                    w1 = (uint64_t)rws[2] | ((uint64_t)rws[3] << 32);
                    wbase = j0 >> 6;
                    if (diag) {  // strict upper (row words) | strict lower (column words) | self-loop
                        w0 |= cwb[(q * 2 + 0) * 128 + x];
                        w1 |= cwb[(q * 2 + 1) * 128 + x];
                        if (x < 64) w0 |= 1ull << x;
                        else w1 |= 1ull << (x - 64);
                    }
                }
                *reinterpret_cast<ulonglong2*>(gb + (int64_t)row * dr.words + wbase) = ulonglong2{w0, w1};
                const int pc = __popcll(w0) + __popcll(w1);
                if (pc != 0) atomicAdd(&da[row], pc);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Eight-wave pipelined 128 × 128 form (form 9).  Form 8 runs one wave per
// SIMD: its 176 split VALU, 12 ds_write and 24 ds_read_b128 per chunk issue
// from the same single instruction stream as its 48 MFMAs, and every LDS read
// latency and load wait is exposed (1.87 µs per chunk against a 0.64 µs MFMA
// floor at Cora S = 16).  Here a 512-thread block owns the 128 × 128 tile:
// wave (wr, wc) = (w >> 2, w & 3) a 64 × 32 sub-tile (two 32 × 32
// accumulators sharing each staged V_J / U_J fragment), two waves per SIMD, so
// one wave's staging and reads issue beside its partner's MFMAs.  Per chunk a
// wave reads 18 fragments for 24 MFMAs (0.75 KB per MFMA; the 64-tile form
// reads 1 KB and writes 0.5 KB more per MFMA) and stages a quarter row of
// each of the four operands; the stage is double-buffered (2 × 48 KB dynamic
// LDS, one barrier per chunk) as in form 8.  Same chunks, same LDS rows, same
// MFMA sequence per accumulator as forms 2-8: identical bits.
//
// DRAW (mode 2): the next window's graphs are drawn from the θ the epilogue
// writes, as in the 64-tile lds_theta_grad_sgd_draw: each lane's 2 × 16
// outputs are 2 × 4 row quads of one column, exactly the Philox counters of
// the sampler's tile draw (sampler.hip).  Bit rows come from ballots (row
// segments of 32 columns, joined across the wc pairs in LDS) and column words
// from each lane's own bits; the dead stage buffers hold them, and a second
// pass stores each (row, 2-word) pair once with 16-byte stores and one degree
// atomic per row and graph (half the 64-tile form's atomics).  All eight waves
// run the Philox work, two per SIMD: the VALU issues at its full rate.
// ---------------------------------------------------------------------------

template <bool SMALL, bool PART, bool DRAW>
__global__ __launch_bounds__(512, 1) void theta_grad_w8_kernel(
    const float* __restrict__ u, const float* __restrict__ v, int ld, int k,
    const float* __restrict__ r, int ldr, int nr, float* __restrict__ theta, int n,
    float* __restrict__ grad, int mode, const double* __restrict__ lr_dev, int ldrc,
    float gscale, int group, int per_xcd, DrawArgs dr) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_dyn[];
    __shared__ __attribute__((aligned(16))) float Ri[kT2], Rj[kT2];

    const int nb = (n + kT2 - 1) / kT2;
    const int ntiles = nb * (nb + 1) / 2;
    int bi, bj;
    {
        const int L = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
        if (L >= ntiles) return;  // whole block: no barrier reached
        grouped_tile(L, nb, group, bi, bj);
    }
    const int i0 = bi * kT2, j0 = bj * kT2;
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    const int64_t nn = n;

    // staging: thread t owns row t >> 2 of both blocks, k = 4·(t & 3) … + 3 of
    // the chunk; branch-free loads (rows past n and k past the end read zeros)
    const int srow = t >> 2, kq = t & 3;
    const int gi = i0 + srow, gj = j0 + srow;
    const float* src[4] = {u + (int64_t)gi * ld, v + (int64_t)gi * ld, u + (int64_t)gj * ld,
                           v + (int64_t)gj * ld};
    const bool rowok[4] = {gi < n, gi < n, gj < n, gj < n};
    auto load = [&](float (&x)[4][4], int k0) {
        const int gk = k0 + 4 * kq;
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const float* p = (rowok[a] && gk < k) ? src[a] + gk : g_zero8;
            const float4 f = *reinterpret_cast<const float4*>(p);
            x[a][0] = f.x; x[a][1] = f.y; x[a][2] = f.z; x[a][3] = f.w;
        }
    };
    // the 16-wide-chunk LDS rows of forms 2-8: 8 dwords, 16-byte halves
    // swapped by row bit 3; this thread's quarter is dwords 2·(kq & 1) … + 1
    // of half kq >> 1 (ds_write_b64 lane groups: 4 rows × 4 quarters, 32
    // distinct banks)
    const int soff = srow * kS2 + 4 * ((kq >> 1) ^ swz16(srow)) + 2 * (kq & 1);
    auto stage_arr = [&](uint32_t* buf, const float (&x)[4], int a) {
        uint32_t h0, m0, l0, h1, m1, l1;
        split3_pair(x[0], x[1], h0, m0, l0);
        split3_pair(x[2], x[3], h1, m1, l1);
        *reinterpret_cast<uint2*>(buf + (3 * a + 0) * kPL2 + soff) = uint2{h0, h1};
        *reinterpret_cast<uint2*>(buf + (3 * a + 1) * kPL2 + soff) = uint2{m0, m1};
        *reinterpret_cast<uint2*>(buf + (3 * a + 2) * kPL2 + soff) = uint2{l0, l1};
    };

    // the epilogue's θ (and partial-grad) operands, issued before the k loop
    const int jl = wc * 32 + (lane & 31);
    const int j = j0 + jl;
    auto row_of = [&](int m, int e) { return wr * 64 + m * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5); };
    float th[2][16], part[2][16];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int i = i0 + row_of(m, e);
            const bool in = i < n && j < n && j >= i;
            const int64_t id = in ? tri_at_t<SMALL>(i, j, nn) : 0;
            th[m][e] = (in && theta != nullptr) ? theta[id] : 0.f;
            part[m][e] = (PART && in) ? grad[id] : 0.f;
        }

    if (t < 2 * kT2) {
        const int rr = t & (kT2 - 1);
        const int row = (t < kT2 ? i0 : j0) + rr;
        float racc = 0.f;
        if (row < n) racc = row_r_sum(r, (int64_t)row * ldr, ldrc, nr);
        (t < kT2 ? Ri : Rj)[rr] = racc;
    }

    const int fo = 4 * ((lane >> 5) ^ ((lane >> 3) & 1));  // fragment rows: bit 3 = lane bit 3
    const int ra0 = (wr * 64 + (lane & 31)) * kS2 + fo, ra1 = ra0 + 32 * kS2;
    const int rb = (wc * 32 + (lane & 31)) * kS2 + fo;
    f32x16 acc[2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[m][e] = 0.f;
    // chunk c from `cur`, beside the stage of the next chunk into `nxt`
    auto step = [&](const uint32_t* cur, uint32_t* nxt, const float (&x)[4][4]) {
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {  // pr 0: U_I × V_J (planes 0-2, 9-11); pr 1: V_I × U_J (3-5, 6-8)
            const int pa = pr == 0 ? 0 : 3, pb = pr == 0 ? 9 : 6;
            bf16x8 fa[2][3], fb[3];
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                fa[0][s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(cur + (pa + s) * kPL2 + ra0));
                fa[1][s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(cur + (pa + s) * kPL2 + ra1));
                fb[s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(cur + (pb + s) * kPL2 + rb));
            }
            stage_arr(nxt, x[2 * pr], 2 * pr);
            stage_arr(nxt, x[2 * pr + 1], 2 * pr + 1);
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                f32x16 c = acc[m];
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][1], fb[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][0], fb[2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][2], fb[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][0], fb[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][1], fb[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[m][0], fb[0], c, 0, 0, 0);
                acc[m] = c;
            }
        }
    };

    uint32_t* const b0 = lds_dyn;
    uint32_t* const b1 = lds_dyn + 12 * kPL2;
    float xa[4][4], xb[4][4];
    const int nch = (k + 15) / 16;
    if (nch > 0) {
        load(xa, 0);
        load(xb, 16);
#pragma unroll
        for (int a = 0; a < 4; ++a) stage_arr(b0, xa[a], a);
        load(xa, 32);
    }
    __syncthreads();
    // chunk c: buffer c & 1 holds it; registers xb (c even) / xa (c odd) hold c + 1
    for (int c = 0; c < nch; c += 2) {
        step(b0, b1, xb);
        load(xb, 16 * (c + 3));
        __syncthreads();
        if (c + 1 >= nch) break;
        step(b1, b0, xa);
        load(xa, 16 * (c + 4));
        __syncthreads();
    }

    w8_epilogue<SMALL, DRAW>(acc, th, part, Ri, Rj, theta, grad, n, mode, lr_dev, gscale, i0, j0, wr, wc, lane, t,
                             lds_dyn, dr);
}

// ---------------------------------------------------------------------------
// Direct-staged eight-wave 128 × 128 form (form 10, round 3).  Form 9's chunk
// is bound by its staging phase, not by its 24 MFMAs per wave: every thread
// splits its quarter rows (≈60 VALU per wave and chunk) and writes them with
// 12 ds_write_b64, and the barrier that publishes them drains every load in
// flight (__syncthreads() waits vmcnt(0)), so the next chunk's loads are
// exposed once per chunk.  Here the operands arrive pre-split (U and V as
// three bf16 planes in the tile layout below, written by
// lds_split_planes_t128 or by whoever produces the factors) and the stage is
// a verbatim copy: each (16-wide chunk, 128-row tile) block of an operand is
// 12 KB, laid out exactly as form 9's LDS planes (rows of 8 dwords, halves
// swapped by row bit 3), so every wave moves 6 of the chunk's 48 KB with
// direct global -> LDS loads (global_load_lds_dwordx4: no VGPR round trip, no
// ds_write, no split).  The stage is a ring of three buffers (144 KB):
// chunk c + 2 streams in while chunk c is multiplied, and a chunk's barrier
// waits only for the loads of chunk c itself (counted vmcnt, raw s_barrier;
// the loads are issued from inline asm, which keeps the compiler from
// draining them before every LDS read).  Same chunks, same LDS planes, same
// MFMA sequence per accumulator as forms 2-9: identical bits.
//
// Plane layout (uint16 offsets; nt = ceil(rows / 128) row tiles, rows and
// k zero-padded to whole tiles / 16-wide chunks): value x(i, kk), split word
// s (0 = high, 1 = middle, 2 = low) at
//   (((c·nt + T)·3 + s)·128 + r)·16 + 8·(h ^ ((r >> 3) & 1)) + (kk & 7),
//   c = kk >> 4, T = i >> 7, r = i & 127, h = (kk >> 3) & 1.
// ---------------------------------------------------------------------------
constexpr int kDmaStages = 3;
constexpr int kDmaStageBytes = 12 * kPL2 * 4;                 // 48 KB: U_I, V_I, U_J, V_J × 3 planes
constexpr int kDmaLds = kDmaStages * kDmaStageBytes;           // 144 KB
constexpr int kTileBlk = 3 * kT2 * 16;                         // uint16 per (chunk, row tile) block of one operand



template <bool SMALL, bool PART, bool DRAW>
__global__ __launch_bounds__(512, 1) void theta_grad_dma_kernel(
    const uint16_t* __restrict__ up, const uint16_t* __restrict__ vp, int nt, int k,
    const float* __restrict__ r, int ldr, int nr, float* __restrict__ theta, int n,
    float* __restrict__ grad, int mode, const double* __restrict__ lr_dev, int ldrc,
    float gscale, int group, int per_xcd, DrawArgs dr) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_dyn[];
    __shared__ __attribute__((aligned(16))) float Ri[kT2], Rj[kT2];

    const int nb = (n + kT2 - 1) / kT2;
    const int ntiles = nb * (nb + 1) / 2;
    int bi, bj;
    {
        const int L = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
        if (L >= ntiles) return;  // whole block: no barrier reached
        grouped_tile(L, nb, group, bi, bj);
    }
    const int i0 = bi * kT2, j0 = bj * kT2;
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    const int nch = (k + 15) / 16;

    // stage fill: wave w copies the 1-KB blocks w, w + 8, …, w + 40 of a chunk
    // (block b: operand b / 12 = U_I, V_I, U_J, V_J, its bytes 1024·(b % 12) …)
    const uint32_t lds_base =
        (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint32_t*)lds_dyn);
    const int64_t cstride = (int64_t)nt * kTileBlk;  // uint16 per chunk of one operand
    const uint16_t* const opb[4] = {up + (int64_t)bi * kTileBlk, vp + (int64_t)bi * kTileBlk,
                                    up + (int64_t)bj * kTileBlk, vp + (int64_t)bj * kTileBlk};
    auto fill = [&](int c, int buf) {
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            const int b = wave + 8 * q;
            const int a = b / 12, p = b - 12 * a;
            const uint16_t* src = (a == 0 ? opb[0] : a == 1 ? opb[1] : a == 2 ? opb[2] : opb[3]) + c * cstride +
                                  512 * p + 8 * lane;
            lds_dma16(src, lds_base + (uint32_t)(buf * kDmaStageBytes + 1024 * b));
        }
    };
    if (nch > 0) fill(0, 0);
    if (nch > 1) fill(1, 1);
    if (nch > 2) fill(2, 2);

    // the epilogue's θ (and partial-grad) operands, issued before the k loop
    const int jl = wc * 32 + (lane & 31);
    const int j = j0 + jl;
    auto row_of = [&](int m, int e) { return wr * 64 + m * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5); };
    // n in a VGPR, and the loads branch-free (entries outside the triangle
    // read element 0; the epilogue skips them): under this kernel's SGPR
    // pressure the compiler otherwise re-read n from the kernel arguments,
    // with a wait, for each of the 32 loads behind an exec branch
    int nv = n;
    asm volatile("" : "+v"(nv));
    float th[2][16], part[2][16];
    const bool has_theta = theta != nullptr;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int i = i0 + row_of(m, e);
            const bool in = i < nv && j < nv && j >= i;
            const int64_t id0 = tri_at_t<SMALL>(i, j, (int64_t)nv);  // (any value outside the triangle)
            const int64_t id = in ? id0 : 0;
            th[m][e] = has_theta ? theta[id] : 0.f;
            part[m][e] = PART ? grad[id] : 0.f;
        }

    if (t < 2 * kT2) {
        const int rr = t & (kT2 - 1);
        const int row = (t < kT2 ? i0 : j0) + rr;
        float racc = 0.f;
        if (row < n) racc = row_r_sum(r, (int64_t)row * ldr, ldrc, nr);
        (t < kT2 ? Ri : Rj)[rr] = racc;
    }
    // the first three chunks staged: the compiler does not count the asm loads, so
    // its barrier would not wait for them (nor for the θ loads, issued after)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __syncthreads();                     // R sums and the stage visible to every wave

    const int fo = 4 * ((lane >> 5) ^ ((lane >> 3) & 1));  // fragment rows: bit 3 = lane bit 3
    const int ra0 = (wr * 64 + (lane & 31)) * kS2 + fo, ra1 = ra0 + 32 * kS2;
    const int rb = (wc * 32 + (lane & 31)) * kS2 + fo;
    f32x16 acc[2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[m][e] = 0.f;

    // Half-chunk software pipeline: the fragments of one product pair (pr 0:
    // U_I × V_J, planes 0-2 and 9-11; pr 1: V_I × U_J, planes 3-5 and 6-8) are
    // read while the other pair's MFMAs run — pr 1 of chunk c during pr 0 of
    // c, pr 0 of chunk c + 1 (after the chunk barrier) during pr 1 of c — so
    // the LDS read latency and the barrier hide behind MFMAs in flight.  The
    // ring holds chunk c + 1 (read next), c + 2 (in flight) and c + 3 (filled
    // into chunk c's buffer once every wave has read it).
    typedef bf16x8 Half[2][3 + 3];  // [m][s] A fragments of rows m·32 …, [0][3 + s] the B fragments
    auto read_half = [&](int c, int pr, Half& f) {
        const uint32_t* cur = lds_dyn + (c % kDmaStages) * (kDmaStageBytes / 4);
        const int pa = pr == 0 ? 0 : 3, pb = pr == 0 ? 9 : 6;
#pragma unroll
        for (int s = 0; s < 3; ++s) {
            f[0][s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(cur + (pa + s) * kPL2 + ra0));
            f[1][s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(cur + (pa + s) * kPL2 + ra1));
            f[0][3 + s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(cur + (pb + s) * kPL2 + rb));
        }
    };
    auto mfmas = [&](const Half& f) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const bf16x8* a = f[m];
            const bf16x8* b = f[0] + 3;
            f32x16 cc = acc[m];
            cc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], cc, 0, 0, 0);
            cc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], cc, 0, 0, 0);
            cc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], cc, 0, 0, 0);
            cc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], cc, 0, 0, 0);
            cc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], cc, 0, 0, 0);
            cc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], cc, 0, 0, 0);
            acc[m] = cc;
        }
    };
    Half h0, h1;
    if (nch > 0) read_half(0, 0, h0);
    for (int c = 0; c < nch; ++c) {
        read_half(c, 1, h1);
        mfmas(h0);
        if (c + 1 < nch) {
            // this wave's loads of chunk c + 1 done (those of c + 2 may be in
            // flight) and its reads of chunk c returned; the barrier makes both
            // hold for every wave
            if (c + 2 < nch) __builtin_amdgcn_s_waitcnt(0x0076);  // vmcnt(6) expcnt(7) lgkmcnt(0)
            else __builtin_amdgcn_s_waitcnt(0x0070);              // vmcnt(0) lgkmcnt(0)
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");  // no LDS access of the next chunk above the barrier
            if (c + 3 < nch) fill(c + 3, c % kDmaStages);
            read_half(c + 1, 0, h0);
        }
        mfmas(h1);
    }
    __syncthreads();  // every wave done with the stage (the draw reuses it)

    w8_epilogue<SMALL, DRAW>(acc, th, part, Ri, Rj, theta, grad, n, mode, lr_dev, gscale, i0, j0, wr, wc, lane, t,
                             lds_dyn, dr);
}

// x (rows × ld fp32, its first k columns) -> the split3 planes of form 10
// (t128_plane_at; rows padded to whole 128-row tiles and k to whole 16-wide
// chunks with zeros).  One thread per (row, 8-wide half chunk): 32 bytes read,
// three 16-byte stores, consecutive threads on consecutive rows' halves.
__global__ __launch_bounds__(256) void split_planes_t128_kernel(const float* __restrict__ x, int rows, int ld, int k,
                                                                int nt, int nch, uint16_t* __restrict__ planes) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;  // ((c·nt + T)·128 + r)·2 + h
    if (e >= (int64_t)nch * nt * kT2 * 2) return;
    const int h = (int)(e & 1);
    const int64_t ct = e >> 1;  // (c·nt + T)·128 + r
    const int r = (int)(ct & (kT2 - 1));
    const int64_t cT = ct >> 7;
    const int c = (int)(cT / nt);
    const int64_t i = (cT - (int64_t)c * nt) * kT2 + r;
    const int kk0 = 16 * c + 8 * h;
    float xv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) xv[q] = (i < rows && kk0 + q < k) ? x[i * ld + kk0 + q] : 0.f;
    uint32_t hw[4], mw[4], lw[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) split3_pair(xv[2 * q], xv[2 * q + 1], hw[q], mw[q], lw[q]);
    *reinterpret_cast<u32x4*>(planes + t128_plane_at(i, kk0, 0, nt)) = u32x4{hw[0], hw[1], hw[2], hw[3]};
    *reinterpret_cast<u32x4*>(planes + t128_plane_at(i, kk0, 1, nt)) = u32x4{mw[0], mw[1], mw[2], mw[3]};
    *reinterpret_cast<u32x4*>(planes + t128_plane_at(i, kk0, 2, nt)) = u32x4{lw[0], lw[1], lw[2], lw[3]};
}

template <bool SMALL, bool PART, bool DRAW>
static void launch_dma_inst(int grid, hipStream_t st, const uint16_t* up, const uint16_t* vp, int nt, int k,
                            const float* r, int ldr, int nr, float* theta, int n, float* grad, int mode,
                            const double* lr, int ldrc, float gscale, int per, const DrawArgs& dr) {
    // > 64 KB of dynamic LDS must be enabled per kernel and device: set on every
    // launch (a cheap host call); a refusal surfaces as the launch's error
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&theta_grad_dma_kernel<SMALL, PART, DRAW>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kDmaLds);
    hipLaunchKernelGGL((theta_grad_dma_kernel<SMALL, PART, DRAW>), dim3(grid), dim3(512), kDmaLds, st, up, vp, nt, k,
                       r, ldr, nr, theta, n, grad, mode, lr, ldrc, gscale, 8, per, dr);
}

static void launch_dma(hipStream_t st, const uint16_t* up, const uint16_t* vp, int nt, int k, const float* r, int ldr,
                       int nr, float* theta, int n, float* grad, int mode, const double* lr, int ldrc, float gscale,
                       const DrawArgs* dr) {
    const int nb2 = (n + kT2 - 1) / kT2;
    const int nt2 = nb2 * (nb2 + 1) / 2;
    const int per = (nt2 + 7) / 8;
    const int grid = 8 * per;
    const bool small = n <= 46340;
    const bool part = mode == 1 || mode == 3;
#define LDS_DMA_ARGS grid, st, up, vp, nt, k, r, ldr, nr, theta, n, grad, mode, lr, ldrc, gscale, per
    if (dr != nullptr) {  // mode 2 only (checked by the caller)
        if (small) launch_dma_inst<true, false, true>(LDS_DMA_ARGS, *dr);
        else launch_dma_inst<false, false, true>(LDS_DMA_ARGS, *dr);
        return;
    }
    const DrawArgs none{};
    if (small && part) launch_dma_inst<true, true, false>(LDS_DMA_ARGS, none);
    else if (small) launch_dma_inst<true, false, false>(LDS_DMA_ARGS, none);
    else if (part) launch_dma_inst<false, true, false>(LDS_DMA_ARGS, none);
    else launch_dma_inst<false, false, false>(LDS_DMA_ARGS, none);
#undef LDS_DMA_ARGS
}

// Assembly form: 0 = fp32 MFMA (v_mfma_f32_32x32x2_f32); split-bf16: 1 = by
// shape (below), 2 = 64-tile with 16-wide k chunks, 3 = 64-tile with 32-wide
// k chunks, 4 = 128-tile in plain triangle order, 5 = 128-tile in XCD-grouped
// order, 6 = form 2 in XCD-grouped order, 7 = form 5 with 64-bit index
// arithmetic at every n (the n > 46 340 path; for testing), 8 = the
// software-pipelined 128-tile (double-buffered stage, XCD-grouped order),
// 9 = the eight-wave pipelined 128-tile.  Chosen per call (the `form`
// argument of every entry point).
constexpr int kGroup = 8;

template <bool SMALL, bool PART, bool DRAW>
static void launch_w8_inst(int grid, hipStream_t st, const float* u, const float* v, int ld, int k, const float* r,
                           int ldr, int nr, float* theta, int n, float* grad, int mode, const double* lr, int ldrc,
                           float gscale, int per, const DrawArgs& dr) {
    // > 64 KB of dynamic LDS, enabled per kernel and device on every launch
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&theta_grad_w8_kernel<SMALL, PART, DRAW>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kW8Lds);
    hipLaunchKernelGGL((theta_grad_w8_kernel<SMALL, PART, DRAW>), dim3(grid), dim3(512), kW8Lds, st, u, v, ld, k, r,
                       ldr, nr, theta, n, grad, mode, lr, ldrc, gscale, kGroup, per, dr);
}

// Form 9 (needs 16-byte aligned rows and k % 8 == 0, the `fast` condition).
static void launch_w8(hipStream_t st, const float* u, const float* v, int ld, int k, const float* r, int ldr, int nr,
                      float* theta, int n, float* grad, int mode, const double* lr, int ldrc, float gscale,
                      const DrawArgs* dr) {
    const int nb2 = (n + kT2 - 1) / kT2;
    const int nt2 = nb2 * (nb2 + 1) / 2;
    const int per = (nt2 + 7) / 8;
    const int grid = 8 * per;
    const bool small = n <= 46340;
    const bool part = mode == 1 || mode == 3;
#define LDS_W8_ARGS grid, st, u, v, ld, k, r, ldr, nr, theta, n, grad, mode, lr, ldrc, gscale, per
    if (dr != nullptr) {  // mode 2 only (checked by the caller)
        if (small) launch_w8_inst<true, false, true>(LDS_W8_ARGS, *dr);
        else launch_w8_inst<false, false, true>(LDS_W8_ARGS, *dr);
        return;
    }
    const DrawArgs none{};
    if (small && part) launch_w8_inst<true, true, false>(LDS_W8_ARGS, none);
    else if (small) launch_w8_inst<true, false, false>(LDS_W8_ARGS, none);
    else if (part) launch_w8_inst<false, true, false>(LDS_W8_ARGS, none);
    else launch_w8_inst<false, false, false>(LDS_W8_ARGS, none);
#undef LDS_W8_ARGS
}

static void launch_theta_grad(int ntiles, hipStream_t st, const float* u, const float* v, int ld, int k,
                              const float* r, int ldr, int nr, float* theta, int n, float* grad, int mode,
                              const double* lr, int vec4, int ldrc, float gscale, int form,
                              Planes pl = Planes{nullptr, nullptr}) {
    const bool pre = pl.u != nullptr;
    if (pre && (form == 0 || form == 3)) form = 6;  // pre-split: the 16-wide-chunk 64-tile or the 128-tile forms
    const int nb2 = (n + kT2 - 1) / kT2;
    const int nt2 = nb2 * (nb2 + 1) / 2;
    // by shape (tools/thetagrad_forms.py, MI355X): 64-tiles in XCD-grouped
    // order while the 128-tile grid cannot fill the chip with short k (Cora
    // S = 1: 44.7 vs 65 µs; 46.8 in plain order);
    // 128-tiles in XCD-grouped order for long k (Cora / Citeseer S = 16:
    // 577 / 695 vs 604 / 895 µs) or large n (n = 20 000: 2.01 vs 2.27 ms)
    // and the pipelined 128-tile (form 8) where its one block per CU still runs
    // every tile in one round and k is long (Cora S = 16: 494 vs 546 µs; at
    // Citeseer S = 16, 351 tiles, 847 vs 674; at n = 20 000, 2.29 vs 1.93 ms)
    // round 3 (tools/microbench/tg_draw_ab.py, profiles/r03_theta_forms.jsonl):
    // the eight-wave 128-tile (form 9) wherever its one block per CU runs every
    // tile in one round (Cora S = 1: 41.8 µs against 47.4 pipelined, 49.0
    // 64-tile; S = 16: 399 against 422), else the 128-tile form in XCD-grouped
    // order (Citeseer S = 1: 59.9 against 63.6; S = 16: 577 against 728;
    // n = 20 000: 1.77 against 1.93 ms)
    if (form == 1) form = nt2 <= 256 ? 9 : 5;
    // the branch-free staging needs whole 8-wide k groups in 16-byte aligned rows
    const bool fast = vec4 && (k & 7) == 0;
    if (form == 9 && !pre && fast) {
        launch_w8(st, u, v, ld, k, r, ldr, nr, theta, n, grad, mode, lr, ldrc, gscale, nullptr);
        return;
    }
    if (form == 9) form = 5;  // pre-split operands or unaligned rows: the plain 128-tile form
#define LDS_TG_ARGS u, v, ld, k, r, ldr, nr, theta, n, grad, mode, lr, vec4, ldrc, gscale
    if (form == 8 && !pre && fast) {
        const int per = (nt2 + 7) / 8;
        const bool small = n <= 46340;
        // > 64 KB of dynamic LDS, enabled per kernel and device on every launch
        if (small)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&theta_grad_bf3_pipe_kernel<true>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, kPipeLds);
        else
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&theta_grad_bf3_pipe_kernel<false>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, kPipeLds);
        if (small)
            hipLaunchKernelGGL((theta_grad_bf3_pipe_kernel<true>), dim3(8 * per), dim3(256), kPipeLds, st, u, v, ld, k,
                               r, ldr, nr, theta, n, grad, mode, lr, ldrc, gscale, kGroup, per);
        else
            hipLaunchKernelGGL((theta_grad_bf3_pipe_kernel<false>), dim3(8 * per), dim3(256), kPipeLds, st, u, v, ld,
                               k, r, ldr, nr, theta, n, grad, mode, lr, ldrc, gscale, kGroup, per);
        return;
    }
    if (form == 8) form = 5;  // pre-split operands or unaligned rows: the plain 128-tile form
    if (form == 4 || form == 5 || form == 7) {
        const int per = (nt2 + 7) / 8;
        const int grid = form != 4 ? 8 * per : nt2;
        const int grp = form != 4 ? kGroup : 0;
        const bool small = n <= 46340 && form != 7;
        if (pre && small)
            hipLaunchKernelGGL((theta_grad_bf3_t128_kernel<true, true, true>), dim3(grid), dim3(256), 0, st, LDS_TG_ARGS,
                               grp, per, pl);
        else if (pre)
            hipLaunchKernelGGL((theta_grad_bf3_t128_kernel<true, false, true>), dim3(grid), dim3(256), 0, st,
                               LDS_TG_ARGS, grp, per, pl);
        else if (fast && small)
            hipLaunchKernelGGL((theta_grad_bf3_t128_kernel<true, true>), dim3(grid), dim3(256), 0, st, LDS_TG_ARGS, grp,
                               per, pl);
        else if (fast)
            hipLaunchKernelGGL((theta_grad_bf3_t128_kernel<true, false>), dim3(grid), dim3(256), 0, st, LDS_TG_ARGS,
                               grp, per, pl);
        else
            hipLaunchKernelGGL((theta_grad_bf3_t128_kernel<false, false>), dim3(grid), dim3(256), 0, st, LDS_TG_ARGS,
                               grp, per, pl);
    } else if (form == 3) {
        if (fast)
            hipLaunchKernelGGL((theta_grad_bf3_kernel<32, true>), dim3(ntiles), dim3(256), 0, st, LDS_TG_ARGS, 0, 0, pl);
        else
            hipLaunchKernelGGL((theta_grad_bf3_kernel<32, false>), dim3(ntiles), dim3(256), 0, st, LDS_TG_ARGS, 0, 0, pl);
    } else if (form == 2 || form == 6) {
        const int per = (ntiles + 7) / 8;
        const int grid = form == 6 ? 8 * per : ntiles;
        const int grp = form == 6 ? kGroup : 0;
        if (pre && (mode == 1 || mode == 3))
            hipLaunchKernelGGL((theta_grad_bf3_kernel<16, true, true, true>), dim3(grid), dim3(256), 0, st, LDS_TG_ARGS,
                               grp, per, pl);
        else if (pre)
            hipLaunchKernelGGL((theta_grad_bf3_kernel<16, true, true, false>), dim3(grid), dim3(256), 0, st,
                               LDS_TG_ARGS, grp, per, pl);
        else if (fast)
            hipLaunchKernelGGL((theta_grad_bf3_kernel<16, true>), dim3(grid), dim3(256), 0, st, LDS_TG_ARGS, grp, per, pl);
        else
            hipLaunchKernelGGL((theta_grad_bf3_kernel<16, false>), dim3(grid), dim3(256), 0, st, LDS_TG_ARGS, grp, per, pl);
#undef LDS_TG_ARGS
    } else {
        hipLaunchKernelGGL(theta_grad_mfma_kernel, dim3(ntiles), dim3(256), 0, st, u, v, ld, k, r, ldr, nr,
                           theta, n, grad, mode, lr, vec4, ldrc, gscale);
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
                              int accumulate, int form, void* stream) {
    LDS_CHECK_ARG(form >= 0 && form <= 10);
    if (form == 10) form = 1;  // the direct-staged form needs planes (lds_theta_grad_direct): by shape here
    LDS_CHECK_ARG(grad != nullptr && n > 0 && k >= 0 && nr >= 0);
    LDS_CHECK_ARG(k == 0 || (u != nullptr && v != nullptr && ld >= k));
    LDS_CHECK_ARG(nr == 0 || (r != nullptr && ldr >= nr));
    const int nb = (n + kTile - 1) / kTile;
    const int ntiles = nb * (nb + 1) / 2;
    const int vec4 = ((ld & 3) == 0 && ((((uintptr_t)u) | ((uintptr_t)v)) & 15) == 0) ? 1 : 0;
    launch_theta_grad(ntiles, (hipStream_t)stream, u, v, ld, k, r, ldr, nr, const_cast<float*>(theta), n, grad, accumulate ? 1 : 0, (const double*)nullptr, vec4, 1, 1.0f, form);
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
                                  const void* scalars, int form, void* stream) {
    LDS_CHECK_ARG(form >= 0 && form <= 10);
    if (form == 10) form = 1;  // the direct-staged form needs planes (lds_theta_grad_direct): by shape here
    LDS_CHECK_ARG(theta != nullptr && scalars != nullptr && n > 0 && k >= 0 && nr >= 0);
    LDS_CHECK_ARG(k == 0 || (u != nullptr && v != nullptr && ld >= k));
    LDS_CHECK_ARG(nr == 0 || (r != nullptr && ldr >= nr));
    const int nb = (n + kTile - 1) / kTile;
    const int ntiles = nb * (nb + 1) / 2;
    const int vec4 = ((ld & 3) == 0 && ((((uintptr_t)u) | ((uintptr_t)v)) & 15) == 0) ? 1 : 0;
    // EngineScalars: f64 outer_lr at byte offset 16
    const double* lr = reinterpret_cast<const double*>((const char*)scalars + 16);
    launch_theta_grad(ntiles, (hipStream_t)stream, u, v, ld, k, r, ldr, nr, theta, n, grad, 2, lr, vec4, 1, 1.0f, form);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_theta_grad_sgd_accum(const float* u, const float* v, int ld, int k, const float* r,
                                        int ldr, int nr, float* theta, int n, float* grad,
                                        const void* scalars, int form, void* stream) {
    LDS_CHECK_ARG(form >= 0 && form <= 10);
    if (form == 10) form = 1;  // the direct-staged form needs planes (lds_theta_grad_direct): by shape here
    LDS_CHECK_ARG(theta != nullptr && grad != nullptr && scalars != nullptr && n > 0 && k >= 0 && nr >= 0);
    LDS_CHECK_ARG(k == 0 || (u != nullptr && v != nullptr && ld >= k));
    LDS_CHECK_ARG(nr == 0 || (r != nullptr && ldr >= nr));
    const int nb = (n + kTile - 1) / kTile;
    const int ntiles = nb * (nb + 1) / 2;
    const int vec4 = ((ld & 3) == 0 && ((((uintptr_t)u) | ((uintptr_t)v)) & 15) == 0) ? 1 : 0;
    const double* lr = reinterpret_cast<const double*>((const char*)scalars + 16);
    launch_theta_grad(ntiles, (hipStream_t)stream, u, v, ld, k, r, ldr, nr, theta, n, grad, 3, lr, vec4, 1, 1.0f, form);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_theta_grad_ex(const float* u, const float* v, int ld, int k, const float* r,
                                 int ldr_row, int ldr_col, int nr, float* theta, int n, float* grad,
                                 int mode, const void* scalars, float gscale, int form, void* stream) {
    LDS_CHECK_ARG(form >= 0 && form <= 10);
    if (form == 10) form = 1;  // the direct-staged form needs planes (lds_theta_grad_direct): by shape here
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
    launch_theta_grad(ntiles, (hipStream_t)stream, u, v, ld, k, r, ldr_row, nr, theta, n, grad, mode, lr, vec4, ldr_col, gscale, form);
    LDS_RETURN_LAST_ERROR();
}

// lds_theta_grad_ex over the rows [row0, row1) of the packed triangle only
// (their 128-row block tiles, every column block from the diagonal on; the
// plain split-bf16 128-tile form): the band-sharded exchange of BASELINE
// config 5, where rank b assembles, updates and draws from its
// own row band of θ with every rank's factors.  row0 a multiple of 128, row1
// too or n; mode 0 (dθ of the band into grad) or 2 (fused SGD + clamp of the
// band of θ, grad optional).  Same result bits per entry as the full launch.
extern "C" int lds_theta_grad_band(const float* u, const float* v, int ld, int k, const float* r, int ldr_row,
                                   int ldr_col, int nr, float* theta, int n, float* grad, int mode,
                                   const void* scalars, float gscale, int row0, int row1, void* stream) {
    LDS_CHECK_ARG(n > 0 && k > 0 && nr >= 0 && (mode == 0 || mode == 2));
    LDS_CHECK_ARG(u != nullptr && v != nullptr && ld >= k);
    LDS_CHECK_ARG(nr == 0 || (r != nullptr && ldr_row >= 0 && ldr_col >= 0));
    LDS_CHECK_ARG(mode == 0 ? grad != nullptr : (theta != nullptr && scalars != nullptr));
    LDS_CHECK_ARG(0 <= row0 && row0 < row1 && row1 <= n && row0 % kT2 == 0 && (row1 % kT2 == 0 || row1 == n));
    const int nb = (n + kT2 - 1) / kT2;
    const int b0 = row0 / kT2, b1 = (row1 + kT2 - 1) / kT2;
    int64_t tiles = 0;
    for (int b = b0; b < b1; ++b) tiles += nb - b;
    LDS_CHECK_ARG(tiles > 0 && tiles < (1 << 30));
    const int vec4 = ((ld & 3) == 0 && ((((uintptr_t)u) | ((uintptr_t)v)) & 15) == 0) ? 1 : 0;
    const bool fast = vec4 && (k & 7) == 0, small = n <= 46340;
    const double* lr = mode == 2 ? reinterpret_cast<const double*>((const char*)scalars + 16) : nullptr;
    hipStream_t st = (hipStream_t)stream;
    const Planes none{nullptr, nullptr};
#define LDS_TGB_ARGS u, v, ld, k, r, ldr_row, nr, theta, n, grad, mode, lr, vec4, ldr_col, gscale, -b0 - 1, 0, none
    if (fast && small)
        hipLaunchKernelGGL((theta_grad_bf3_t128_kernel<true, true>), dim3((unsigned)tiles), dim3(256), 0, st, LDS_TGB_ARGS);
    else if (fast)
        hipLaunchKernelGGL((theta_grad_bf3_t128_kernel<true, false>), dim3((unsigned)tiles), dim3(256), 0, st, LDS_TGB_ARGS);
    else
        hipLaunchKernelGGL((theta_grad_bf3_t128_kernel<false, false>), dim3((unsigned)tiles), dim3(256), 0, st, LDS_TGB_ARGS);
#undef LDS_TGB_ARGS
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_theta_grad_planes(const uint16_t* up, const uint16_t* vp, int ld, int k, const float* r,
                                     int ldr_row, int ldr_col, int nr, float* theta, int n, float* grad, int mode,
                                     const void* scalars, float gscale, int form, void* stream) {
    LDS_CHECK_ARG(form >= 0 && form <= 10);
    if (form == 10) form = 1;  // the direct-staged form needs planes (lds_theta_grad_direct): by shape here
    LDS_CHECK_ARG(n > 0 && k >= 0 && nr >= 0 && mode >= 0 && mode <= 3);
    LDS_CHECK_ARG(k == 0 || (up != nullptr && vp != nullptr && ld >= k));
    LDS_CHECK_ARG((k & 7) == 0);
    LDS_CHECK_ARG(((((uintptr_t)up) | ((uintptr_t)vp)) & 15) == 0);
    LDS_CHECK_ARG(nr == 0 || (r != nullptr && ldr_row >= 0 && ldr_col >= 0));
    LDS_CHECK_ARG(mode < 2 ? grad != nullptr : (theta != nullptr && scalars != nullptr));
    LDS_CHECK_ARG(mode != 3 || grad != nullptr);
    const int nb = (n + kTile - 1) / kTile;
    const int ntiles = nb * (nb + 1) / 2;
    const double* lr = mode >= 2 ? reinterpret_cast<const double*>((const char*)scalars + 16) : nullptr;
    launch_theta_grad(ntiles, (hipStream_t)stream, nullptr, nullptr, ld, k, r, ldr_row, nr, theta, n, grad, mode, lr,
                      1, ldr_col, gscale, form, Planes{up, vp});
    LDS_RETURN_LAST_ERROR();
}

// x (rows × ld fp32, the first k columns) -> its chunk-major split3 words
// (ci_at; ceil(k/16) chunks of rows × 48 uint16).
__global__ __launch_bounds__(256) void split_planes_kernel(const float* __restrict__ x, int rows, int ld, int k,
                                                           uint16_t* __restrict__ planes) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= (int64_t)rows * k) return;
    const int64_t i = e / k;
    const int c = (int)(e - i * k);
    uint16_t h, m, l;
    split3_one(x[i * ld + c], h, m, l);
    planes[ci_at(i, c, 0, rows)] = h;
    planes[ci_at(i, c, 1, rows)] = m;
    planes[ci_at(i, c, 2, rows)] = l;
}

extern "C" int lds_split_planes(const float* x, int rows, int ld, int k, uint16_t* planes, void* stream) {
    LDS_CHECK_ARG(x && planes && rows > 0 && k > 0 && ld >= k);
    const int64_t tot = (int64_t)rows * k;
    hipLaunchKernelGGL(split_planes_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x,
                       rows, ld, k, planes);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_theta_grad_sgd_draw(const float* u, const float* v, int ld, int k, const float* r,
                                       int ldr, int nr, float* theta, int n, float* grad, const void* scalars,
                                       uint64_t seed, uint32_t tag, const uint32_t* counter_base,
                                       uint32_t counter_offset, int graphs, uint64_t* bits, int words,
                                       int* deg_ws, int form, void* stream) {
    LDS_CHECK_ARG(form >= 0 && form <= 10);
    if (form == 10) form = 1;  // the direct-staged form needs planes (lds_theta_grad_direct): by shape here
    LDS_CHECK_ARG(u && v && theta && scalars && bits && deg_ws && n > 0 && k >= 0 && ld >= k);
    // the 128-tile draws store two words per (graph, row): whole 128-column word pairs
    LDS_CHECK_ARG(graphs > 0 && graphs <= 65535 && (words & 1) == 0 && words >= 2 * ((n + 127) / 128) && nr >= 0);
    LDS_CHECK_ARG(nr == 0 || (r != nullptr && ldr >= nr));
    LDS_CHECK_ARG((ld & 3) == 0 && (k & 7) == 0 && ((uintptr_t)u & 15) == 0 && ((uintptr_t)v & 15) == 0);
    const int nb = (n + kTile - 1) / kTile;
    const int ntiles = nb * (nb + 1) / 2;
    const int per = (ntiles + 7) / 8;
    const double* lr = reinterpret_cast<const double*>(reinterpret_cast<const char*>(scalars) + 16);
    DrawArgs dr{bits, words, deg_ws, lds_sample_ws_ints(n), (uint32_t)seed, (uint32_t)(seed >> 32), tag,
                counter_offset, counter_base, graphs};
    // by shape (form 1): the 64-tile form (6) while the 128-tile grid cannot
    // fill the chip (as launch_theta_grad's rule), else the 128-tile form in
    // XCD-grouped order (5); 9 the eight-wave 128-tile form; every form gives
    // identical θ, bits and degrees.  MI355X (tools/microbench/tg_draw_ab.py,
    // six graphs, k = 264): 64-tile 61.8 vs eight-wave 63.6 µs at Cora, 86 vs
    // 114 at Citeseer, 2.61 vs 2.91 ms at n = 20 000.
    const int nb2 = (n + kT2 - 1) / kT2;
    const int nt2 = nb2 * (nb2 + 1) / 2;
    // by shape, with the draw (same tool): the eight-wave form at Cora-sized
    // grids (62.2 µs against 63.2 for the 64-tile), the 64-tile form in between
    // (Citeseer: 82.8 against 97.4 for the 128-tile, 112 eight-wave), the
    // 128-tile form at large n (2.49 against 2.63 ms at n = 20 000)
    if (form == 1) form = nt2 <= 256 ? 9 : nt2 >= 1024 ? 5 : 6;
    if (form == 4 || form == 5 || form == 7 || form == 8) {
        const int per2 = (nt2 + 7) / 8;
        if (n <= 46340 && form != 7)
            hipLaunchKernelGGL((theta_grad_bf3_t128_kernel<true, true, false, true>), dim3(8 * per2), dim3(256), 0,
                               (hipStream_t)stream, u, v, ld, k, r, ldr, nr, theta, n, grad, 2, lr, 1, 1, 1.0f, kGroup,
                               per2, Planes{nullptr, nullptr}, dr);
        else
            hipLaunchKernelGGL((theta_grad_bf3_t128_kernel<true, false, false, true>), dim3(8 * per2), dim3(256), 0,
                               (hipStream_t)stream, u, v, ld, k, r, ldr, nr, theta, n, grad, 2, lr, 1, 1, 1.0f, kGroup,
                               per2, Planes{nullptr, nullptr}, dr);
    } else if (form == 9) {
        launch_w8((hipStream_t)stream, u, v, ld, k, r, ldr, nr, theta, n, grad, 2, lr, 1, 1.0f, &dr);
    } else {
        hipLaunchKernelGGL((theta_grad_bf3_kernel<16, true, false, true, true>), dim3(8 * per), dim3(256), 0,
                           (hipStream_t)stream, u, v, ld, k, r, ldr, nr, theta, n, grad, 2, lr, 1, 1, 1.0f, kGroup,
                           per, Planes{nullptr, nullptr}, dr);
    }
    LDS_RETURN_LAST_ERROR();
}

// Form 10's operands: the split3 planes of U / V in the 128-row-tile layout
// (t128_plane_at), uint16 count for `rows` rows and k columns.
extern "C" int64_t lds_planes_t128_elems(int rows, int k) {
    if (rows <= 0 || k <= 0) return 0;
    return (int64_t)((k + 15) / 16) * ((rows + kT2 - 1) / kT2) * kTileBlk;
}

extern "C" int lds_split_planes_t128(const float* x, int rows, int ld, int k, uint16_t* planes, void* stream) {
    LDS_CHECK_ARG(x && planes && rows > 0 && k > 0 && ld >= k && ((uintptr_t)planes & 15) == 0);
    const int nt = (rows + kT2 - 1) / kT2, nch = (k + 15) / 16;
    const int64_t tot = (int64_t)nch * nt * kT2 * 2;
    hipLaunchKernelGGL(split_planes_t128_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, x, rows, ld, k, nt, nch, planes);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_theta_grad_direct(const uint16_t* up, const uint16_t* vp, int k, const float* r, int ldr_row,
                                     int ldr_col, int nr, float* theta, int n, float* grad, int mode,
                                     const void* scalars, float gscale, uint64_t seed, uint32_t tag,
                                     const uint32_t* counter_base, uint32_t counter_offset, int graphs, uint64_t* bits,
                                     int words, int* deg_ws, void* stream) {
    LDS_CHECK_ARG(n > 0 && k >= 0 && nr >= 0 && mode >= 0 && mode <= 3 && graphs >= 0 && graphs <= 65535);
    LDS_CHECK_ARG(k == 0 || (up != nullptr && vp != nullptr && ((((uintptr_t)up) | ((uintptr_t)vp)) & 15) == 0));
    LDS_CHECK_ARG(nr == 0 || (r != nullptr && ldr_row >= 0 && ldr_col >= 0));
    LDS_CHECK_ARG(mode < 2 ? grad != nullptr : (theta != nullptr && scalars != nullptr));
    LDS_CHECK_ARG(mode != 3 || grad != nullptr);
    LDS_CHECK_ARG(graphs == 0 || (mode == 2 && bits && deg_ws && (words & 1) == 0 && words >= 2 * ((n + 127) / 128)));
    const double* lr = mode >= 2 ? reinterpret_cast<const double*>((const char*)scalars + 16) : nullptr;
    const int nt = (n + kT2 - 1) / kT2;
    const DrawArgs dr{bits, words, deg_ws, lds_sample_ws_ints(n), (uint32_t)seed, (uint32_t)(seed >> 32), tag,
                      counter_offset, counter_base, graphs};
    launch_dma((hipStream_t)stream, up, vp, nt, k, r, ldr_row, nr, theta, n, grad, mode, lr, ldr_col, gscale,
               graphs > 0 ? &dr : nullptr);
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
