// Bitmask aggregation Y = diag(s)·Ã·diag(s)·Z for dense sampled graphs
// (BASELINE config 5: θ ~ U(0,1), ~N/2 neighbours per row).
//
// Same operator as lds_spmm_norm / lds_spmm_norm_blocked — torch.mm of
// normalize_adjacency_matrix(A) (src/utils/graph.py:136-153) with the
// embeddings (src/models/layers.py:44) — but Ã is read as the sampler's
// bitmask (1 bit per entry, self-loops set) instead of as CSR (32 bits per
// entry).  At 50 % density that is 50 MB instead of 0.8 GB per call at
// N = 20 000, and the aggregation becomes a dense 0/1 × s⊙Z product that
// the integer matrix cores run exactly:
//
//   t_kf   = fl32(s_k · z_kf)
//   q_kf   = rint(t_kf · 2^e_f)      (e_f: max_k |t_kf| · 2^e_f < 2^30)
//   q_kf   = Σ_L d_kfL · 2^(8L)      (four signed base-256 digits, int8)
//   acc_ifL = Σ_k Ã_ik · d_kfL       (v_mfma_i32_16x16x64_i8, exact int32)
//   y_if   = s_i · 2^-e_f · Σ_L acc_ifL · 2^(8L)
//
// The integer sums are exact and order-independent; the only roundings are
// t's product, the 2^-31-relative quantisation of t against its column's
// maximum and the final combination.  (Exactness w.r.t. the fp32 CSR sum is
// not a goal: both are within a few fp32 ulps of the real-valued result.)
//
// A operand (mask): lane l = 16g + r holds row r of the tile and, for one
// 512-column chunk, the 128 bits [128g, 128g+128) of that row as four 32-bit
// words.  The 16 int8 A values of k-step q (0..7) are bytes of
//   (word[q>>1] >> (4(q&1) + dd)) & 0x01010101,   dd = 0..3,
// i.e. byte b of dword dd is column 128g + 32(q>>1) + 4(q&1) + dd + 8b.  The
// B operand (digits of s⊙Z) is stored pre-permuted in that same k order by
// bitagg_quant_kernel, so the MFMA's k index is a permutation of the columns
// that A and B share; which (lane group, byte) the hardware pairs does not
// matter as long as it is the same map for A and B.
#include "common.hpp"
#include "../../include/ldsgnn.h"

namespace lds {

namespace {

constexpr int kF = 16;            // features (the GCN hidden width)
constexpr int kChunk = 512;       // columns per staged B chunk
constexpr int kSteps = kChunk / 64;   // MFMA k-steps per chunk
constexpr int kLimbs = 4;         // base-256 digits of the fixed-point s⊙Z
constexpr int kChunkBytes = kChunk * kF * kLimbs;   // 32 KB
constexpr int kMaxBlocks = 256;   // column-max partial blocks
constexpr int kWaves = 8;         // waves per workgroup (share one LDS stage)
constexpr int kTiles = 2;         // 16-row tiles per wave
constexpr int kThreads = 64 * kWaves;
constexpr int kRowsPerWg = kWaves * 16 * kTiles;   // 256
constexpr int kResidentWgs = 512;  // 2 workgroups per CU (64 KB LDS, <= 256 VGPRs each)

typedef int v4i __attribute__((ext_vector_type(4)));

int chunks_of(int n) { return (n + kChunk - 1) / kChunk; }
int row_groups_of(int n) { return (n + kRowsPerWg - 1) / kRowsPerWg; }
int splits_of(int n) {
    const int nc = chunks_of(n), rg = row_groups_of(n);
    int ks = kResidentWgs / rg;   // every workgroup resident at once
    if (ks > nc) ks = nc;
    return ks < 1 ? 1 : ks;
}

struct Ws {
    uint32_t* colmax;   // [kMaxBlocks][kF] float bits of max |t|
    int8_t* zq;         // [chunks][kChunkBytes]
    float* part;        // [splits][n][kF]
};

Ws carve(void* ws, int n) {
    char* p = (char*)ws;
    Ws w;
    w.colmax = (uint32_t*)p;
    p += kMaxBlocks * kF * 4;
    w.zq = (int8_t*)p;
    p += (size_t)chunks_of(n) * kChunkBytes;
    w.part = (float*)p;
    return w;
}

}  // namespace

// Per-block column maxima of |s_k z_kf| (non-negative floats compare as
// their bit patterns).  grid = kMaxBlocks, 256 threads = 16 rows × 16 features.
__global__ __launch_bounds__(256) void bitagg_colmax_kernel(const float* __restrict__ s, int n,
                                                            const float* __restrict__ z, int ldz,
                                                            uint32_t* __restrict__ colmax) {
    const int f = threadIdx.x & 15;
    uint32_t m = 0;
#pragma unroll 4
    for (int k = blockIdx.x * 16 + (threadIdx.x >> 4); k < n; k += kMaxBlocks * 16)
        m = max(m, __float_as_uint(fabsf(s[k] * z[(int64_t)k * ldz + f])));
    // 4 rows per wave share a feature: lanes f, f+16, f+32, f+48
    m = max(m, (uint32_t)__shfl_xor((int)m, 16));
    m = max(m, (uint32_t)__shfl_xor((int)m, 32));
    __shared__ uint32_t red[4][16];
    if ((threadIdx.x & 63) < 16) red[threadIdx.x >> 6][f] = m;
    __syncthreads();
    if (threadIdx.x < 16)
        colmax[blockIdx.x * kF + threadIdx.x] =
            max(max(red[0][threadIdx.x], red[1][threadIdx.x]), max(red[2][threadIdx.x], red[3][threadIdx.x]));
}

__device__ __forceinline__ int col_exponent(uint32_t maxbits) {
    // e such that max · 2^e < 2^30 (max = m·2^E, m in [0.5, 1) -> e = 30 - E)
    if (maxbits == 0) return 0;
    int E;
    frexpf(__uint_as_float(maxbits), &E);
    return 30 - E;
}

// max over the kMaxBlocks partials of feature lane & 15 (lanes f, f+16,
// f+32, f+48 all end with feature f's value)
__device__ __forceinline__ uint32_t colmax_of(const uint32_t* __restrict__ colmax, int lane) {
    const int f = lane & 15;
    uint32_t m = 0;
    for (int b = lane >> 4; b < kMaxBlocks; b += 4) m = max(m, colmax[b * kF + f]);
    m = max(m, (uint32_t)__shfl_xor((int)m, 16));
    m = max(m, (uint32_t)__shfl_xor((int)m, 32));
    return m;
}

// Fixed-point digits of s⊙Z in the chunk layout [chunk][q][limb][g][f][16 B]:
// one thread per lane fragment (chunk c, k-step q, lane group g, feature f)
// = 16 columns, written as one 16-byte store per limb.  Columns past n are 0.
__global__ __launch_bounds__(256) void bitagg_quant_kernel(const float* __restrict__ s, int n,
                                                           const float* __restrict__ z, int ldz,
                                                           const uint32_t* __restrict__ colmax,
                                                           int8_t* __restrict__ zq, int chunks) {
    __shared__ int e_sh[kF];
    if (threadIdx.x < 64) {
        const uint32_t m = colmax_of(colmax, threadIdx.x);
        if (threadIdx.x < kF) e_sh[threadIdx.x] = col_exponent(m);
    }
    __syncthreads();
    const int idx = blockIdx.x * 256 + threadIdx.x;   // ((c·8 + q)·4 + g)·16 + f
    if (idx >= chunks * kSteps * 4 * kF) return;
    const int f = idx & 15, g = (idx >> 4) & 3, q = (idx >> 6) & 7, c = idx >> 9;
    const int e = e_sh[f];
    const int kb = c * kChunk + 128 * g + 32 * (q >> 1) + 4 * (q & 1);
    uint32_t out[kLimbs][4];
#pragma unroll
    for (int dd = 0; dd < 4; ++dd) {
#pragma unroll
        for (int L = 0; L < kLimbs; ++L) out[L][dd] = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int k = kb + dd + 8 * b;
            int v = 0;
            if (k < n) v = (int)rintf(ldexpf(s[k] * z[(int64_t)k * ldz + f], e));
#pragma unroll
            for (int L = 0; L < kLimbs; ++L) {
                const int d = ((v + 128) & 255) - 128;   // balanced digit in [-128, 127]
                out[L][dd] |= (uint32_t)(d & 255) << (8 * b);
                v = (v - d) >> 8;
            }
        }
    }
#pragma unroll
    for (int L = 0; L < kLimbs; ++L)
        *(uint4*)(zq + (int64_t)c * kChunkBytes + (q * kLimbs + L) * 1024 + g * 256 + f * 16) =
            uint4{out[L][0], out[L][1], out[L][2], out[L][3]};
}

// This lane's mask bits for chunk c: row r of each tile, words 8c + 2g, +1.
__device__ __forceinline__ void load_mask(const uint64_t* __restrict__ bits, int words, int n, int row0, int r,
                                          int g, int c, uint32_t (&mw)[kTiles][4]) {
    const int wi = 8 * c + 2 * g;
#pragma unroll
    for (int t = 0; t < kTiles; ++t) {
        const int row = row0 + t * 16 + r;
        uint64_t a = 0, b = 0;
        if (row < n && wi + 1 < words) {
            const uint64_t* p = bits + (int64_t)row * words + wi;
            a = p[0];
            b = p[1];
        }
        mw[t][0] = (uint32_t)a;
        mw[t][1] = (uint32_t)(a >> 32);
        mw[t][2] = (uint32_t)b;
        mw[t][3] = (uint32_t)(b >> 32);
    }
}

// Grid (row groups of 256, column splits); 8 waves, each 2 tiles of 16 rows
// (the 64 KB LDS stage allows 2 workgroups per CU: 8-wave groups at ~116
// VGPRs give 4 waves per SIMD, against 2 for 4 waves × 4 tiles at 212 VGPRs;
// 28.5 vs 30.2 µs at N = 20 000).  Measured and not kept:
//  - the 32×32×32 i8 form (A = 32 rows × 32 columns, B = two limbs × 16
//    features; a quarter of the issue slots held instead of half): 33 µs;
//  - the mask prefetched two chunks deep in registers with counted vmcnt
//    waits: hipcc drains vmcnt to 0 at the use of an ordinary load while a
//    direct-to-LDS load is in flight (loop head, .s);
//  - mask and digits both through direct-to-LDS loads from inline asm (the
//    builtin makes hipcc wait vmcnt(0) before every ds_read), 3-deep mask
//    ring, counted waits, 112 KB LDS, 1 workgroup per CU: 27.9 µs — 2 %, not
//    worth hand-counted vmcnt.
// PMC at N = 20 000 (r01): MFMA busy 42 % of the cycles, 40 % of the wave
// time waiting; per chunk and wave 64 MFMAs, ~130 VALU, 34 LDS reads.
// Per 512-column chunk the workgroup stages the chunk's digits (32 KB) in
// LDS by direct global->LDS loads, double-buffered (chunk c+1 streams in
// while chunk c is multiplied); every wave reads its B fragments from there
// and its mask bits from HBM into registers, also one chunk ahead (64
// contiguous bytes per row per chunk).  Partials per split in fp32.
__global__ __launch_bounds__(kThreads) void bitagg_main_kernel(const uint64_t* __restrict__ bits, int words, int n,
                                                          const int8_t* __restrict__ zq, int chunks, int splits,
                                                          float* __restrict__ part, const uint32_t* __restrict__ colmax,
                                                          const float* __restrict__ s, float* __restrict__ y, int ldy,
                                                          int beta, int partials_only) {
    __shared__ __attribute__((aligned(16))) int8_t bsh[2 * kChunkBytes];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int c0 = (int)((int64_t)blockIdx.y * chunks / splits);
    const int c1 = (int)((int64_t)(blockIdx.y + 1) * chunks / splits);
    const int row0 = blockIdx.x * kRowsPerWg + wave * 16 * kTiles;

    v4i acc[kTiles][kLimbs];
#pragma unroll
    for (int t = 0; t < kTiles; ++t)
#pragma unroll
        for (int L = 0; L < kLimbs; ++L) acc[t][L] = v4i{0, 0, 0, 0};

    // wave w stages the 1-KB blocks kWaves·i + w of a chunk (64 lanes x 16 B each)
    auto stage = [&](int c, int buf) {
#pragma unroll
        for (int i = 0; i < kChunkBytes / 1024 / kWaves; ++i) {
            const int kb = kWaves * i + wave;
            __builtin_amdgcn_global_load_lds(
                (const void*)(zq + (int64_t)c * kChunkBytes + kb * 1024 + lane * 16),
                (__attribute__((address_space(3))) void*)(bsh + buf * kChunkBytes + kb * 1024), 16, 0, 0);
        }
    };
    uint32_t mw[kTiles][4], mn[kTiles][4];
    if (c0 < c1) {
        stage(c0, 0);
        load_mask(bits, words, n, row0, r, g, c0, mn);
    }
    for (int c = c0; c < c1; ++c) {
        const int buf = (c - c0) & 1;
        __syncthreads();   // chunk c staged (vmcnt 0) and chunk c-1's readers done
#pragma unroll
        for (int t = 0; t < kTiles; ++t)
#pragma unroll
            for (int j = 0; j < 4; ++j) mw[t][j] = mn[t][j];
        if (c + 1 < c1) {
            stage(c + 1, buf ^ 1);
            load_mask(bits, words, n, row0, r, g, c + 1, mn);
        }
        const v4i* bs = (const v4i*)(bsh + buf * kChunkBytes);
        v4i bfr[2][kLimbs];   // k-step q+1's fragments load during step q's MFMAs
#pragma unroll
        for (int L = 0; L < kLimbs; ++L) bfr[0][L] = bs[L * 64 + lane];
#pragma unroll
        for (int q = 0; q < kSteps; ++q) {
            if (q + 1 < kSteps) {
#pragma unroll
                for (int L = 0; L < kLimbs; ++L) bfr[(q + 1) & 1][L] = bs[((q + 1) * kLimbs + L) * 64 + lane];
            }
            const v4i* bf = bfr[q & 1];
#pragma unroll
            for (int t = 0; t < kTiles; ++t) {
                const uint32_t wsel = mw[t][q >> 1];
                const int sh = 4 * (q & 1);
                v4i a;
                a.x = (int)((wsel >> sh) & 0x01010101u);
                a.y = (int)((wsel >> (sh + 1)) & 0x01010101u);
                a.z = (int)((wsel >> (sh + 2)) & 0x01010101u);
                a.w = (int)((wsel >> (sh + 3)) & 0x01010101u);
#pragma unroll
                for (int L = 0; L < kLimbs; ++L)
                    acc[t][L] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bf[L], acc[t][L], 0, 0, 0);
            }
        }
    }
    // C/D: col = lane & 15 (feature), row = 4(lane >> 4) + i
    const int f = lane & 15;
    const int e = col_exponent(colmax_of(colmax, lane));
    float* out = part + (int64_t)blockIdx.y * n * kF;
#pragma unroll
    for (int t = 0; t < kTiles; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = row0 + t * 16 + 4 * g + i;
            if (row < n) {
                const int64_t v = (int64_t)acc[t][0][i] + ((int64_t)acc[t][1][i] << 8) +
                                  ((int64_t)acc[t][2][i] << 16) + ((int64_t)acc[t][3][i] << 24);
                const float pv = (float)ldexp((double)v, -e);
                if (splits == 1 && !partials_only) {  // one split: y = s_i · part here (bitagg_final_kernel's arithmetic)
                    float* o = y + (int64_t)row * ldy + f;
                    const float r = s[row] * pv;
                    *o = beta ? *o + r : r;
                } else {
                    out[(int64_t)row * kF + f] = pv;
                }
            }
        }
}

// y = s_i · Σ_split part (split order fixed), beta: y += instead of y =.
// One thread per 4 features of a row.
__global__ __launch_bounds__(256) void bitagg_final_kernel(const float* __restrict__ part, int splits, int n,
                                                           const float* __restrict__ s, float* __restrict__ y,
                                                           int ldy, int beta) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;   // row·4 + quarter
    if (idx >= (int64_t)n * 4) return;
    const int row = (int)(idx >> 2), f0 = 4 * (int)(idx & 3);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4* p4 = (const float4*)part + idx;
#pragma unroll 4
    for (int p = 0; p < splits; ++p) {
        const float4 v = p4[(int64_t)p * n * 4];
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
    }
    const float si = s[row];
    float* o = y + (int64_t)row * ldy + f0;
    const float r[4] = {si * acc.x, si * acc.y, si * acc.z, si * acc.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = beta ? o[j] + r[j] : r[j];
}

}  // namespace lds

using namespace lds;

extern "C" int64_t lds_bitmask_agg_ws_bytes(int n) {
    if (n <= 0) return 0;
    return (int64_t)kMaxBlocks * kF * 4 + (int64_t)chunks_of(n) * kChunkBytes + (int64_t)splits_of(n) * n * kF * 4;
}

extern "C" int lds_aggregate_bitmask(const uint64_t* bits, int words, const float* s, int n, const float* z,
                                     int ldz, float* y, int ldy, int beta, void* ws, void* stream) {
    LDS_CHECK_ARG(bits && s && z && y && ws && n > 0 && n <= (1 << 20));
    LDS_CHECK_ARG(words >= (n + 63) / 64 && (words & 1) == 0 && ldz >= kF && ldy >= kF);
    LDS_CHECK_ARG(((uintptr_t)ws & 15) == 0);
    hipStream_t st = (hipStream_t)stream;
    const Ws w = carve(ws, n);
    const int nc = chunks_of(n), ks = splits_of(n);
    hipLaunchKernelGGL(bitagg_colmax_kernel, dim3(kMaxBlocks), dim3(256), 0, st, s, n, z, ldz, w.colmax);
    hipLaunchKernelGGL(bitagg_quant_kernel, dim3((nc * kSteps * 4 * kF + 255) / 256), dim3(256), 0, st,
                       s, n, z, ldz, (const uint32_t*)w.colmax, w.zq, nc);
    hipLaunchKernelGGL(bitagg_main_kernel, dim3(row_groups_of(n), ks), dim3(kThreads), 0, st, bits, words, n,
                       (const int8_t*)w.zq, nc, ks, w.part, (const uint32_t*)w.colmax, s, y, ldy, beta, 0);
    // several splits: their partials are summed by a separate launch.  A
    // last-block-per-row-group reduction in the main kernel (ticket counter,
    // device-scope fences around it) was measured at 151 vs 28.5 µs per call
    // at N = 20 000: on this GPU each block's release / acquire fence writes
    // back and invalidates its XCD's L2 under the other blocks' operands.
    if (ks > 1)
        hipLaunchKernelGGL(bitagg_final_kernel, dim3((unsigned)(((int64_t)n * 4 + 255) / 256)), dim3(256), 0, st,
                       (const float*)w.part, ks, n, s, y, ldy, beta);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_bitmask_agg_splits(int n) { return n > 0 ? splits_of(n) : 0; }

extern "C" int64_t lds_bitmask_agg_part_offset(int n) {
    if (n <= 0) return 0;
    return (int64_t)kMaxBlocks * kF * 4 + (int64_t)chunks_of(n) * kChunkBytes;
}

extern "C" int lds_aggregate_bitmask_partials(const uint64_t* bits, int words, const float* s, int n, const float* z,
                                              int ldz, void* ws, void* stream) {
    LDS_CHECK_ARG(bits && s && z && ws && n > 0 && n <= (1 << 20));
    LDS_CHECK_ARG(words >= (n + 63) / 64 && (words & 1) == 0 && ldz >= kF);
    LDS_CHECK_ARG(((uintptr_t)ws & 15) == 0);
    hipStream_t st = (hipStream_t)stream;
    const Ws w = carve(ws, n);
    const int nc = chunks_of(n), ks = splits_of(n);
    hipLaunchKernelGGL(bitagg_colmax_kernel, dim3(kMaxBlocks), dim3(256), 0, st, s, n, z, ldz, w.colmax);
    hipLaunchKernelGGL(bitagg_quant_kernel, dim3((nc * kSteps * 4 * kF + 255) / 256), dim3(256), 0, st,
                       s, n, z, ldz, (const uint32_t*)w.colmax, w.zq, nc);
    hipLaunchKernelGGL(bitagg_main_kernel, dim3(row_groups_of(n), ks), dim3(kThreads), 0, st, bits, words, n,
                       (const int8_t*)w.zq, nc, ks, w.part, (const uint32_t*)w.colmax, s, (float*)nullptr, 0, 0,
                       1);
    LDS_RETURN_LAST_ERROR();
}
