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
// Device error word bits (include/ldsgnn.h LDS_DEVERR_*).
constexpr uint32_t kDevErrFillDegree = 1u;
constexpr uint32_t kDevErrCsrColumns = 2u;
constexpr uint32_t kDevErrSgdTileCounter = 4u;

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

// Linear id L of a row band's tiles -> upper-triangle block (bi <= bj): the
// block rows b0, b0 + 1, … of the band in order, each from its diagonal block
// to the last column block (lds_theta_grad_band, lds_sample_band_bits: the band-sharded exchange
// of BASELINE config 5).
__device__ __forceinline__ void band_tile(int L, int nb, int b0, int& bi, int& bj) {
    int i = b0;
    while (L >= nb - i) {
        L -= nb - i;
        ++i;
    }
    bi = i;
    bj = i + L;
}

// A compile-time bool as a value (for generic lambdas instantiated per case).
template <bool B>
struct BoolC {
    static constexpr bool value = B;
};

struct U32x4 {
    uint32_t x, y, z, w;
};

// Philox4x32-10 (Salmon et al., SC'11).  Counter (c0..c3), key (k0, k1).
// REQUIREMENT: the key must be the same in every lane (it is a kernel argument
// at every call site): the rounds take it as the SGPR operand ("s") of
// v_bitop3_b32, so a per-lane key would silently use one lane's.  (Forcing it
// with readfirstlane here costs 17 more SGPR spills in the θ-grad draw
// epilogues; the equality tests against the host Philox are the guard.)
__device__ __forceinline__ U32x4 philox4x32_10(U32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // one v_mad_u64_u32 per 32x32->64 product instead of v_mul_lo_u32 +
        // v_mul_hi_u32 (both quarter rate); non-volatile asm so the four quads
        // of a thread still interleave
        uint64_t p0, p1, cc0, cc1;
        asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(p0), "=s"(cc0) : "s"(0xD2511F53u), "v"(c.x));
        asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(p1), "=s"(cc1) : "s"(0xCD9E8D57u), "v"(c.z));
        (void)cc0;
        (void)cc1;
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        // hi ^ c ^ k as one v_bitop3_b32 (XOR3 truth table 0x96, the round key
        // as its SGPR operand; gfx950 has no v_xor3_b32 and the compiler emits
        // two v_xor_b32): 626 -> 758 G Philox calls/s on MI355X, same words
        // (tools/microbench/philox_rate.hip)
        uint32_t x0, x2;
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(x0) : "v"(hi1), "v"(c.y), "s"(k0));
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(x2) : "v"(hi0), "v"(c.w), "s"(k1));
        c = U32x4{x0, lo1, x2, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
        // the round keys advance in place: without this the compiler hoists
        // all twenty into SGPRs, which the θ-grad draw epilogues then spill
        // (84 → 66 spills in the eight-wave form, 19 → 2 in the 64-tile one)
        asm volatile("" : "+s"(k0), "+s"(k1));
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

// x = x0 + x1 + x2 as three bf16 words by truncation: x0 = the top 16 bits of
// x, x1 those of the exact remainder x - x0, x2 those of what is left (the
// split-bf16 θ-grad assembly, thetagrad.hip; pre-split planes hold these).
__device__ __forceinline__ void split3_one(float x, uint16_t& h, uint16_t& m, uint16_t& l) {
    const uint32_t b = __float_as_uint(x);
    const float r = x - __uint_as_float(b & 0xffff0000u);
    const uint32_t c = __float_as_uint(r);
    const float q = r - __uint_as_float(c & 0xffff0000u);
    h = (uint16_t)(b >> 16);
    m = (uint16_t)(c >> 16);
    l = (uint16_t)(__float_as_uint(q) >> 16);
}

__device__ __forceinline__ int wave_lane() { return threadIdx.x & (kWave - 1); }
// The wave's index in its block, as a wave-uniform (SGPR) value: the compiler
// cannot prove threadIdx.x >> 6 uniform, and everything derived from it (row
// indices, row offsets, 64-bit addresses, branches) would otherwise run
// per lane on the VALU under exec masks.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// 64-lane integer sum and inclusive scan on the VALU: DPP within 16-lane rows
// (row_ror / row_shr), row_bcast15/31 or v_permlane16/32_swap across rows —
// no LDS-crossbar round trips (the __shfl forms cost ~100 cycles per hop).
template <int CTRL>
__device__ __forceinline__ int dpp_int(int v) { return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true); }
__device__ __forceinline__ int wave_sum_int(int v) {
    v += dpp_int<0x128>(v);  // row_ror:8, 4, 2, 1: every lane of a row holds the row's sum
    v += dpp_int<0x124>(v);
    v += dpp_int<0x122>(v);
    v += dpp_int<0x121>(v);
    auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    v += (int)((threadIdx.x & 16) ? r[0] : r[1]);
    r = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
    v += (int)((threadIdx.x & 32) ? r[0] : r[1]);
    return v;
}
__device__ __forceinline__ int wave_incl_scan_int(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1, 2, 4, 8 (0 past the row start)
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 into rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 into rows 2, 3
    return v;
}

// Inclusive scan within each 16-lane row (DPP row_shr), and lane 15's value
// of the row broadcast to the row (row_newbcast:15).
__device__ __forceinline__ int row16_incl_scan_int(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
    return v;
}
__device__ __forceinline__ int row16_last_int(int v) { return dpp_int<0x15F>(v); }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// 16 bytes per lane from global address p to LDS byte address m0 + 16·lane
// (m0 wave-uniform).  Issued from asm: the compiler does not see an LDS DMA
// in flight, so it inserts no vmcnt(0) before the kernel's LDS reads; the
// kernel counts these loads itself (s_waitcnt vmcnt).  Vector-memory
// operations count in issue order, so loads the compiler adds only make such
// a count stricter.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // m0 is reserved; the asm sets it before its one use
// s_waitcnt vmcnt(n) for a wave-uniform run-time n (0..15; larger counts
// wait for 15, which is stricter, never looser).  Kernels that count their own
// inline-asm loads and stores use it to wait for exactly the op they need.
__device__ __forceinline__ void wait_vmcnt(int n) {
    n = __builtin_amdgcn_readfirstlane(n);  // uniform: a scalar branch, not every case under exec masks
    switch (n < 0 ? 0 : n > 15 ? 15 : n) {
#define LDS_VMW(N) \
    case N: __builtin_amdgcn_s_waitcnt(0x0F70 | N); break;
        LDS_VMW(0) LDS_VMW(1) LDS_VMW(2) LDS_VMW(3) LDS_VMW(4) LDS_VMW(5) LDS_VMW(6) LDS_VMW(7)
        LDS_VMW(8) LDS_VMW(9) LDS_VMW(10) LDS_VMW(11) LDS_VMW(12) LDS_VMW(13) LDS_VMW(14) LDS_VMW(15)
#undef LDS_VMW
    }
}

__device__ __forceinline__ void lds_dma16(const void* p, uint32_t m0) {
    m0 = __builtin_amdgcn_readfirstlane(m0);  // wave-uniform by contract; free when already in an SGPR
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(p), "s"(m0) : "memory", "m0");
}
#pragma clang diagnostic pop

// The split-bf16 planes of a factor matrix in the 128-row-tile layout of the
// direct-staged θ-grad form (thetagrad.hip form 10, include/ldsgnn.h
// lds_split_planes_t128): value x(i, kk), word s (0 hi, 1 mid, 2 lo) at this
// uint16 offset (nt = row tiles).
__host__ __device__ __forceinline__ int64_t t128_plane_at(int64_t i, int kk, int s, int nt) {
    const int r = (int)(i & 127);
    const int h = ((kk >> 3) & 1) ^ ((r >> 3) & 1);
    return ((((int64_t)(kk >> 4) * nt + (i >> 7)) * 3 + s) * 128 + r) * 16 + 8 * h + (kk & 7);
}

// One (U, V) factor entry: fp32 at row·ld + col (ld > 0), or, with ld = -nt,
// U / V as the split planes above (uint16) — what the factor producers write
// when the window's θ-grad runs the direct-staged form.
__device__ __forceinline__ void put_uv(float* __restrict__ U, float* __restrict__ V, int ld, int row, int col,
                                       float u, float v) {
    if (ld > 0) {
        U[(int64_t)row * ld + col] = u;
        V[(int64_t)row * ld + col] = v;
        return;
    }
    const int64_t o = t128_plane_at(row, col, 0, -ld);
    uint16_t* up = reinterpret_cast<uint16_t*>(U);
    uint16_t* vp = reinterpret_cast<uint16_t*>(V);
    uint16_t h, m, l;
    split3_one(u, h, m, l);
    up[o] = h;
    up[o + 2048] = m;
    up[o + 4096] = l;
    split3_one(v, h, m, l);
    vp[o] = h;
    vp[o + 2048] = m;
    vp[o + 4096] = l;
}

}  // namespace lds
