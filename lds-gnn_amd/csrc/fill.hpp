// The CSR / s / ELL fill of drawn graphs (one 256-thread block per 16 rows of
// one graph), shared by the sampler's fill launch (sampler.hip) and the
// engine's window-start launch that runs the fill beside the first X product
// (engine.hip, lds_engine_fill_x_linear).
#pragma once

#include "common.hpp"

namespace lds {

// ELL j field: index | node flags (common.hpp kEllIndex); no flags: the index.
__device__ __forceinline__ int ell_index(int j, const uint8_t* __restrict__ flags) {
    return flags != nullptr ? (j | ((int)flags[j] << kEllFlagShift)) : j;
}

// Rows with at least this many entries use the word-at-a-time compaction.
constexpr int kDenseRowFill = 1024;

// One row of the fused fill with a whole wave (rows of kDenseRowFill or more
// entries, or a wave that holds one): ascending columns into col from
// position pre, the first 64 into head.
// Returns the entries the row's bits hold (written from pre on, below `capacity`:
// callers pass min(col capacity, pre + the row's degree count), so a row whose
// bits hold more entries than its count never writes into the next row's slots).
__device__ __forceinline__ int64_t fill_row_wave(const uint64_t* __restrict__ rb_bits, int nbw, int64_t pre, int deg,
                                                 int* __restrict__ col, int64_t capacity, int* __restrict__ head) {
    const int lane = wave_lane();
    int64_t base = pre;
    if (deg < kDenseRowFill) {  // each lane pops its own word's bits
        for (int w0 = 0; w0 < nbw; w0 += 64) {
            const int w = w0 + lane;
            uint64_t word = w < nbw ? rb_bits[w] : 0ull;
            const int cnt = __popcll(word);
            const int incl = wave_incl_scan_int(cnt);
            int64_t pos = base + (incl - cnt);
            while (word) {
                const int bit = __ffsll((unsigned long long)word) - 1;
                const int j = w * 64 + bit;
                if (pos < capacity) col[pos] = j;
                if (pos - pre < kEllWidth) head[pos - pre] = j;
                ++pos;
                word &= word - 1;
            }
            base += __builtin_amdgcn_readlane(incl, 63);
        }
        return base - pre;
    }
    // dense rows: for every non-zero word (uniform loop over a ballot) lane l
    // tests bit l; the word's entries go out as one contiguous store
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int w0 = 0; w0 < nbw; w0 += 64) {
        const int w = w0 + lane;
        const uint64_t word = w < nbw ? rb_bits[w] : 0ull;
        uint64_t nz = __ballot(word != 0ull);
        while (nz) {
            const int src = __ffsll((unsigned long long)nz) - 1;
            nz &= nz - 1;
            const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)word, src);
            const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(word >> 32), src);
            const uint64_t wd = ((uint64_t)hi << 32) | lo;
            const bool set = (wd >> lane) & 1ull;
            const int64_t pos = base + __popcll(wd & below);
            if (set) {
                const int j = (w0 + src) * 64 + lane;
                if (pos < capacity) col[pos] = j;
                if (pos - pre < kEllWidth) head[pos - pre] = j;
            }
            base += __popcll(wd);
        }
    }
    return base - pre;
}

// A row whose bits hold `got` entries where its degree count says `deg`
// (a degree workspace that was not zero on entry, or counts from another
// draw): row_ptr came from the counts, so slots [pre + got, pre + deg) would
// keep whatever col held before — stale or never-written indices that the
// aggregations gather through.  They are written with the row itself (a
// valid index: wrong weights, never an address outside the graph) and the
// device error word gets kDevErrFillDegree, which the host reads and raises
// (include/ldsgnn.h "Device error word").  got > deg (counts short of the
// bits) is flagged too; the fill wrote only the row's own [pre, pre + deg)
// slots, so the next row's columns stay intact.  lane / lanes: this row's
// threads (16 or 64).
__device__ __forceinline__ void fill_degree_guard(int64_t pre, int64_t got, int deg, int row, int* __restrict__ col,
                                                  int64_t capacity, int lane, int lanes, uint32_t* __restrict__ err) {
    if (got == (int64_t)deg) return;
    for (int64_t q = pre + got + lane; q < pre + deg && q < capacity; q += lanes) col[q] = row;
    if (lane == 0 && err != nullptr) atomicOr(err, kDevErrFillDegree);
}

// The CSR fill of the fused sampler: the tile kernel's degree counts give
// each row its CSR offset directly — the block's 256 threads sum the degrees
// of all rows before its first row (one coalesced pass, a block reduction),
// the block's own 16 degrees are scanned in one 16-lane row — so no scan
// launch runs between the draw and the fill.  A 16-lane group per row: lane
// h pops the bits of words h, h+16, ... (positions from a 16-lane scan of
// their counts), keeping the first 64 columns in LDS; the ELL head is
// written last, four entries per lane, whose s_j = deg_j^-1/2
// (inv_sqrt_degree) and flag byte are parallel loads.  A wave holding a row
// of kDenseRowFill or more entries fills its four rows one at a time with the
// whole wave instead.  (One wave per row: 11.2 µs per Cora window of 6
// graphs; four rows per wave: see DESIGN.)
__device__ __forceinline__ void fill_csr_block(int bx, int by, const uint64_t* __restrict__ bits, int n, int words,
                                               const int* __restrict__ dacc, int wsi, int* __restrict__ row_ptr,
                                               int* __restrict__ col, int64_t capacity, float* __restrict__ s,
                                               int2* __restrict__ ell, const uint8_t* __restrict__ flags,
                                               uint32_t* __restrict__ err) {
    __shared__ int red[4];
    __shared__ int dblk[16];  // exclusive scan of the block's 16 row degrees
    __shared__ int head[16][kEllWidth];
    const int wave = wave_id();
    const int lane = wave_lane();
    const int h = lane & 15, k = wave * 4 + (lane >> 4);  // row k of the block (this lane's group)
    const int row0 = bx * 16;
    const int row = row0 + k;
    const int g = by;
    bits += (int64_t)g * n * words;
    dacc += (int64_t)g * wsi;
    row_ptr += (int64_t)g * (n + 1);
    col += (int64_t)g * capacity;
    s += (int64_t)g * n;
    const int nbw = (n + 63) / 64;
    const bool live = row < n;
    const uint64_t* rb_bits = bits + (int64_t)row * words;
    // the row's own operands first (independent of the block prefix): its
    // degree and its first 64 bit words (four per lane), so that rows of up
    // to 4 096 columns walk their words without a load per 16-word step
    const int deg = live ? dacc[row] : 0;
    uint64_t wpre[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) wpre[q] = (live && 16 * q + h < nbw) ? rb_bits[16 * q + h] : 0ull;
    // head entries past the row's drawn count read as the row itself: a degree
    // workspace that was not zero on entry (deg above the bits' count) then
    // yields wrong weights, never an index outside the graph
#pragma unroll
    for (int m = 0; m < 4; ++m) head[k][h + 16 * m] = live ? row : 0;
    if (wave == 0 && lane < 16) {
        const int d = row0 + lane < n ? dacc[row0 + lane] : 0;
        dblk[lane] = row16_incl_scan_int(d) - d;
    }
    // degrees of the rows before the block: 16 independent loads per thread
    // per round (one round up to 4 096 rows)
    int acc = 0;
    for (int r0b = 0; r0b < row0; r0b += 16 * 256) {
        int v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int r = r0b + q * 256 + (int)threadIdx.x;
            v[q] = r < row0 ? dacc[r] : 0;
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) acc += v[q];
    }
    acc = wave_sum_int(acc);
    if (lane == 0) red[wave] = acc;
    __syncthreads();
    const int bpre = red[0] + red[1] + red[2] + red[3];
    const int pre = bpre + dblk[k];
    if (live && h == 0) {  // (clamped: a workspace that was not zero on entry cannot send readers past col)
        row_ptr[row] = (int)min((int64_t)pre, capacity);
        if (row == n - 1) row_ptr[n] = (int)min((int64_t)pre + deg, capacity);
        s[row] = inv_sqrt_degree(deg);
    }
    if (__ballot(live && deg >= kDenseRowFill) == 0) {
        int64_t base = pre;
        const int64_t lim = min(capacity, (int64_t)pre + deg);  // this row's slots only
        auto step = [&](int w0, uint64_t word) {  // 16 words of the row, one per lane
            const int w = w0 + h;
            const int cnt = __popcll(word);
            const int incl = row16_incl_scan_int(cnt);
            int64_t pos = base + (incl - cnt);
            while (word) {
                const int bit = __ffsll((unsigned long long)word) - 1;
                const int j = w * 64 + bit;
                if (pos < lim) col[pos] = j;
                if (pos - pre < kEllWidth) head[k][pos - pre] = j;
                ++pos;
                word &= word - 1;
            }
            base += row16_last_int(incl);
        };
        // uniform: every group walks the same word count
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (16 * q < nbw) step(16 * q, wpre[q]);
        for (int w0 = 64; w0 < nbw; w0 += 16) step(w0, (live && w0 + h < nbw) ? rb_bits[w0 + h] : 0ull);
        if (live) fill_degree_guard(pre, base - pre, deg, row, col, capacity, h, 16, err);
    } else {
#pragma unroll 1
        for (int q = 0; q < 4; ++q) {  // the wave's four rows, one at a time
            const int kq = wave * 4 + q, rq = row0 + kq;
            if (rq >= n) break;
            const int64_t pq = (int64_t)bpre + dblk[kq];
            const int dq = dacc[rq];
            const int64_t got = fill_row_wave(bits + (int64_t)rq * words, nbw, pq, dq, col,
                                              min(capacity, pq + dq), head[kq]);
            fill_degree_guard(pq, got, dq, rq, col, capacity, lane, 64, err);
        }
    }
    if (ell == nullptr || !live) return;
    // the head columns of this wave's rows are in LDS (written by this wave only)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int2* __restrict__ er = ell + ((int64_t)g * n + row) * kEllWidth;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int e = h + 16 * m;
        int2 v = make_int2(row, 0);  // padding: a valid index with weight 0
        if (e < deg) {
            const int j = head[k][e];
            v = make_int2(ell_index(j, flags), __float_as_int(inv_sqrt_degree(dacc[j])));
        }
        er[e] = v;
    }
}

}  // namespace lds
