// Shared pieces of the dense-graph aggregations (bitagg.hip): the fixed-point
// digit layout of s⊙Z that every int8 matrix-core product reads, the
// workspace carve, and small device / host helpers.  Included by the product
// library (bitagg.hip) and by the tools-only variants library
// (tools/variants/spmm_variants.hip), which must read the same workspace.
#pragma once

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
constexpr int kColBlocks = 64;    // column-max partials written (of the kMaxBlocks slots)

typedef int v4i __attribute__((ext_vector_type(4)));

inline int chunks_of(int n) { return (n + kChunk - 1) / kChunk; }
inline int row_groups_of(int n) { return (n + kRowsPerWg - 1) / kRowsPerWg; }
inline int splits_of(int n) {
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

inline Ws carve(void* ws, int n) {
    char* p = (char*)ws;
    Ws w;
    w.colmax = (uint32_t*)p;
    p += kMaxBlocks * kF * 4;
    w.zq = (int8_t*)p;
    p += (size_t)chunks_of(n) * kChunkBytes;
    w.part = (float*)p;
    return w;
}

// The CSR-SpMM for dense graphs (lds_spmm_norm_dense): n limit and the
// workspace after the column maxima and digits (the tile kernel's partials).
constexpr int kDnMaxChunks = 47;      // n <= 24 064: the tile kernel's two bit tiles + rings <= 160 KB
constexpr int kDnStep = 512;          // entries per streaming step of the tile kernel
constexpr int kDnMaxGrid = 512;       // workgroups (partials scratch in ws)
constexpr int kDnMma = 8;             // the tile kernel's MFMA waves
constexpr int kDnPartBytes = 2 * kDnMma * 256 * 8;  // per workgroup: a tile's int64 partials, double-buffered

inline int64_t dense_scratch_off(int n) { return (int64_t)kMaxBlocks * kF * 4 + (int64_t)chunks_of(n) * kChunkBytes; }

}  // namespace

__device__ __forceinline__ int col_exponent(uint32_t maxbits) {
    // e such that max · 2^e < 2^30 (max = m·2^E, m in [0.5, 1) -> e = 30 - E)
    if (maxbits == 0) return 0;
    int E;
    frexpf(__uint_as_float(maxbits), &E);
    return 30 - E;
}

// max over the kColBlocks partials of feature lane & 15 (lanes f, f+16,
// f+32, f+48 all end with feature f's value)
__device__ __forceinline__ uint32_t colmax_of(const uint32_t* __restrict__ colmax, int lane) {
    const int f = lane & 15;
    uint32_t m = 0;
#pragma unroll
    for (int b = lane >> 4; b < kColBlocks; b += 4) m = max(m, colmax[b * kF + f]);
    m = max(m, (uint32_t)__shfl_xor((int)m, 16));
    m = max(m, (uint32_t)__shfl_xor((int)m, 32));
    return m;
}

__device__ __forceinline__ void dn_or(uint32_t* p, uint32_t m) {
    if (m != 0u) atomicOr(p, m);
}

// Loads issued from asm: the compiler's own waits for loads carried around a
// loop in a register ring come out as vmcnt(0) at the loop head (no prefetch
// at all); kernels count these loads themselves (s_waitcnt vmcnt) and rb_bind
// ties the registers to that wait, so nothing reads or copies them earlier.
__device__ __forceinline__ void rb_gload(v4i& v, const v4i* p) {
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
}
// the same with the non-temporal cache policy (a once-read stream)
__device__ __forceinline__ void rb_gload_nt(v4i& v, const v4i* p) {
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
}
__device__ __forceinline__ void rb_bind(v4i& a, v4i& b) { asm volatile("" : "+v"(a), "+v"(b)); }

inline int device_cus() {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus > 0 ? cus : 256;
}

// > 64 KB of dynamic LDS must be enabled per kernel (and device): set on
// every launch, it is a cheap host call.
template <typename K>
inline hipError_t allow_lds(K kernel, int bytes) {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               bytes);
}

}  // namespace lds
