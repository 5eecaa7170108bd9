// Side work of an engine launch (round 3): blocks appended to the grid of a
// latency-bound aggregation kernel that draw one graph of the window from θ
// (the sampler's tile draw for one item) or fill one drawn graph's CSR / s /
// ELL head (fill.hpp).  The engine moves the window's later draws and fills
// there — graph t + 1 drawn beside inner step t's first aggregation, filled
// beside its second — instead of drawing all τ + 1 graphs in the hyper
// step's θ-grad epilogue, where the Philox VALU is on the critical path.
#pragma once
#include "common.hpp"
#include "fill.hpp"
#include "../../include/ldsgnn.h"

namespace lds {

struct SideWork {
    // draw (theta != NULL): one graph, draw counter *ctr_base + ctr_off
    const float* theta;
    uint32_t k0, k1, tag, ctr_off;
    const uint32_t* ctr_base;
    uint64_t* bits;
    int words;
    int* deg;
    int draw_blocks;  // 64 × 64 tiles of the triangle (set by the launch)
    // fill (fbits != NULL): one graph's CSR / s / ELL head
    const uint64_t* fbits;
    const int* fdeg;
    int wsi;
    int* row_ptr;
    int* col;
    int64_t capacity;
    float* s;
    int2* ell;
    const uint8_t* flags;
    int fill_blocks;  // 16-row blocks (set by the launch)
};

// One 64 × 64 tile of one graph: exactly sample_tiles_kernel's item (sampler.hip:
// the same Philox words per (row quad, column), integer-threshold compare, bit
// rows by ballot, column words assembled by wave 0, degree atomics), so the
// bits and counts equal lds_sample_graphs_multi's for this counter.
__device__ __forceinline__ void draw_one_tile(int tile, const float* __restrict__ theta, int n, uint32_t k0,
                                              uint32_t k1, uint32_t tag, uint32_t ctr, uint64_t* __restrict__ bits,
                                              int words, int* __restrict__ dacc) {
    __shared__ uint32_t colpart[4][64];
    __shared__ uint64_t rowword[64];
    const int lane = wave_lane();
    const int wave = wave_id();
    int a, b;
    tri_tile(tile, a, b);
    const int bi = b, bj = a;  // bi <= bj
    const int j = bj * 64 + lane;
    const bool diag_tile = (bi == bj);
    const int64_t nn = n;
    const int r0 = bi * 64 + wave * 16;
    uint32_t thr[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int i = r0 + r;
        const float th = (i < j && j < n) ? theta[tri_index(i, j, nn)] : -1.0f;
        thr[r] = th >= 0.0f ? (uint32_t)ceilf(fminf(th, 1.0f) * 16777216.0f) : 0u;
    }
    uint32_t x[16];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const U32x4 o = philox4x32_10(U32x4{(uint32_t)j, (uint32_t)((r0 >> 2) + m), tag, ctr}, k0, k1);
        x[4 * m] = o.x;
        x[4 * m + 1] = o.y;
        x[4 * m + 2] = o.z;
        x[4 * m + 3] = o.w;
    }
    uint32_t row_lo = 0, row_hi = 0, cw = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const bool e = (x[r] >> 8) < thr[r];
        const uint64_t w = __ballot(e);
        row_lo = lane == r ? (uint32_t)w : row_lo;
        row_hi = lane == r ? (uint32_t)(w >> 32) : row_hi;
        cw |= (uint32_t)e << r;
    }
    const uint64_t myrow = ((uint64_t)row_hi << 32) | row_lo;
    const bool rvalid = lane < 16 && r0 + lane < n;
    if (!diag_tile) {
        if (rvalid) {
            bits[(int64_t)(r0 + lane) * words + bj] = myrow;
            const int pc = __popcll(myrow);
            if (pc != 0) atomicAdd(&dacc[r0 + lane], pc);
        }
    } else if (rvalid) {
        rowword[wave * 16 + lane] = myrow;
    }
    colpart[wave][lane] = cw;
    __syncthreads();
    if (wave == 0 && j < n) {
        uint64_t out = (uint64_t)colpart[0][lane] | ((uint64_t)colpart[1][lane] << 16) |
                       ((uint64_t)colpart[2][lane] << 32) | ((uint64_t)colpart[3][lane] << 48);
        if (diag_tile) out |= rowword[lane] | (1ull << lane);  // self-loop: diagonal set to 1
        bits[(int64_t)j * words + bi] = out;
        const int pc = __popcll(out);
        if (pc != 0) atomicAdd(&dacc[j], pc);
    }
}

// Run this block's side work if it is one of the appended blocks (block-
// uniform: every thread of the block takes the same branch).  True if it was.
__device__ __forceinline__ bool side_block(const SideWork& sw, int n) {
    const int extra = sw.draw_blocks + sw.fill_blocks;
    if (extra == 0) return false;
    const int b = (int)blockIdx.x - ((int)gridDim.x - extra);
    if (b < 0) return false;
    if (b < sw.draw_blocks)
        draw_one_tile(b, sw.theta, n, sw.k0, sw.k1, sw.tag, sw.ctr_off + (sw.ctr_base ? *sw.ctr_base : 0u), sw.bits,
                      sw.words, sw.deg);
    else
        fill_csr_block(b - sw.draw_blocks, 0, sw.fbits, n, sw.words, sw.fdeg, sw.wsi, sw.row_ptr, sw.col,
                       sw.capacity, sw.s, sw.ell, sw.flags);
    return true;
}

// Host: the device copy of an LdsSideWork and its block counts for n nodes.
inline SideWork side_of(const LdsSideWork* h, int n) {
    SideWork w{};
    if (h == nullptr) return w;
    if (h->theta != nullptr) {
        w.theta = h->theta;
        w.k0 = (uint32_t)h->seed;
        w.k1 = (uint32_t)(h->seed >> 32);
        w.tag = h->tag;
        w.ctr_off = h->counter_offset;
        w.ctr_base = h->counter_base;
        w.bits = h->bits;
        w.deg = h->deg;
        const int nb = (n + 63) / 64;
        w.draw_blocks = nb * (nb + 1) / 2;
    }
    w.words = h->words;
    if (h->fill_bits != nullptr) {
        w.fbits = h->fill_bits;
        w.fdeg = h->fill_deg;
        w.wsi = n;  // lds_sample_ws_ints(n)
        w.row_ptr = h->row_ptr;
        w.col = h->col;
        w.capacity = h->col_capacity;
        w.s = h->s;
        w.ell = reinterpret_cast<int2*>(h->ell);
        w.flags = h->node_flags;
        w.fill_blocks = (n + 15) / 16;
    }
    return w;
}

}  // namespace lds
