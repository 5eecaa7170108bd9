// Graph sampling: θ (packed triu) -> symmetric bitmask -> degree / s -> CSR.
//
// Replaces, for the LDS configuration (undirected=True, sparsification NONE,
// dense=False), the dense chain
//   triu_values_to_symmetric_matrix   src/utils/graph.py:166-181
//   Bernoulli(probs=P).sample()       src/models/sampling.py:68
//   to_undirected(from_triu_only)     src/utils/graph.py:35-37
//   add_self_loops + degree           src/utils/graph.py:123-149
// which the reference runs over all N² entries with four dense temporaries.
// Here θ is read once, the graph is born as a 1-bit-per-pair symmetric mask
// (N²/8 bytes) and compacted into CSR; P is never materialised.
#include "common.hpp"
#include "fill.hpp"
#include "../../include/ldsgnn.h"

namespace lds {

// One 4-wave block per 64×64 tile (bi <= bj) of the upper triangle.  Lane l
// owns column j = 64*bj + l; wave w owns the tile's rows 16w .. 16w+15 and
// issues all 16 of its θ loads (each a coalesced 256-B row segment) before any
// compute, then draws four Philox quads (one call = four rows' uniforms of a
// column; the four chains interleave) and compares them as integers.  Row
// words come out of __ballot (lane r keeps row r's word: one store per wave);
// the transposed (lower-triangle) words collect one bit per row in each lane
// and are OR-combined across the four waves in LDS.  Every word of `bits` has exactly one writer: no atomics,
// no memset.
// Batched launches: grid.y = graph (counter + y), grid.z = replica sample (tag +
// z·tag_step); bit matrix (y·samples + z) of the batch.  kLoop: the block loops
// over the (graph, sample) items of the launch on ONE θ tile load (θ read once
// per window instead of once per graph; always on since round 3).  r01's form
// of that loop took 157 VGPRs and lost to one block per graph; with the
// integer-threshold compare and the single row-word store below it takes 69
// and the loop is the faster form (31.0 µs, 21.9 MB fetched per Cora window of
// 6 graphs, against 30.8 µs, 113.9 MB).  Philox-bound: 4 calls × 10 rounds of
// two v_mad_u64_u32 per lane per item.
//
// kDeg: the tile also counts what it stores into the row degrees dacc[graph]
// (integer atomics, no-return, one per non-zero word: about a dozen per row
// at Cora density), so the CSR fill needs no degree pass.  dacc must be zero
// on entry.  (Per-64-row-block totals kept the same way cost 2x the kernel's
// time: ~10^4 atomics per graph on three cache lines serialise at the memory
// side.)
// kSgd (lds_sgd_sample_graphs, kLoop): the tile computes the outer SGD step
// θ <- clamp(θ - lr·g, 0, 1) (lr = the engine's device f64 at lr_dev; the
// arithmetic of lds_engine_sgd_clamp) of every packed entry it owns (i <= j)
// and draws from the new θ.  With the samples split over grid.z, every block
// of the tile reads the OLD θ, so the new one is written by the tile's last
// block to finish (tile_ctr[tile] counts them; that block recomputes the
// update from θ and g — nobody else writes them — and resets the counter):
// a block counts itself only after its draws, i.e. after its θ loads
// returned, so no block can read a θ already updated.  grid.z = 1: the one
// block writes at its end.
template <bool kInj, bool kLoop, bool kDeg, bool kSgd = false>
__global__ __launch_bounds__(256) void sample_tiles_kernel(
    const float* __restrict__ theta, int n, uint32_t k0, uint32_t k1, uint32_t tag,
    uint32_t counter, const uint32_t* __restrict__ counter_base, const float* __restrict__ u_inj,
    uint64_t* __restrict__ bits, int words, int ntiles, uint32_t tag_step, int samples, int graphs,
    int* __restrict__ dacc, int wsi, float* __restrict__ theta_w = nullptr,
    const float* __restrict__ grad = nullptr, const double* __restrict__ lr_dev = nullptr,
    int* __restrict__ tile_ctr = nullptr, int band0 = -1, int mirror = 1) {
    // items are drawn in groups of kGrp: per item wave w leaves its column bits
    // (rows 16w .. 16w+15 of the tile) here, then wave q assembles item q's
    // column words — one barrier pair per group instead of per item
    constexpr int kGrp = 4;
    __shared__ uint32_t colpart[kGrp][4][64];
    __shared__ uint64_t rowword[kGrp][64];
    const int tile = blockIdx.x;
    // batched launches: graph blockIdx.y draws counter + blockIdx.y; replica
    // samples either come from grid.z (one per block) or, with `samples` > 1,
    // from the loop below over ONE θ tile load (the θ re-read per sample was
    // the sampler's dominant traffic at 16 samples per GPU)
    counter += blockIdx.y;
    if (counter_base != nullptr) counter += *counter_base;  // device-resident draw counter
    const int nsamp = kLoop ? samples : (int)gridDim.z;
    (void)ntiles;
    const int lane = wave_lane();
    const int wave = wave_id();
    // band0 >= 0 (lds_sample_band_bits): the tiles of 64-row blocks band0, …
    // in band order; mirror = 0: an off-diagonal tile writes its rows' words
    // only, not the transposed words of the rows below the band
    int bi, bj;  // bi <= bj
    if (band0 >= 0) {
        band_tile(tile, (n + 63) / 64, band0, bi, bj);
    } else {
        int a, b;
        tri_tile(tile, a, b);
        bi = b;
        bj = a;
    }
    const int j = bj * 64 + lane;
    const bool diag_tile = (bi == bj);
    const int64_t nn = n;
    const int r0 = bi * 64 + wave * 16;  // first row of this wave

    float th[16];
    if constexpr (kSgd) {
        const float lr = (float)*lr_dev;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int i = r0 + r;
            th[r] = -1.0f;
            if (i <= j && j < n) {
                const int64_t idx = tri_index(i, j, nn);
                const float t = fminf(fmaxf(fmaf(-lr, grad[idx], theta_w[idx]), 0.f), 1.f);  // θ via theta_w only
                if (i < j) th[r] = t;
            }
        }
    } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int i = r0 + r;
            th[r] = (i < j && j < n) ? theta[tri_index(i, j, nn)] : -1.0f;  // i < n follows
        }
    }
    // Edge (i, j) iff u < clamp(θ, 0, 1) (triu_values_to_symmetric_matrix,
    // src/utils/graph.py:180; θ = -1 marks pairs outside the strict upper
    // triangle).  With u = m·2^-24 (m = the Philox word >> 8, an integer) that
    // is m < ceil(clamp(θ)·2^24) exactly (scaling by 2^24 is exact; m < T iff
    // m < ceil T for an integer m and T >= 0): one integer compare per draw.
    uint32_t thr[16];
#pragma unroll
    for (int r = 0; r < 16; ++r)
        thr[r] = th[r] >= 0.0f ? (uint32_t)ceilf(fminf(th[r], 1.0f) * 16777216.0f) : 0u;
    // kLoop: items (graph blockIdx.y + g, sample z), g < graphs, g-major, over
    // this one θ tile load (graph blockIdx.y + g draws counter + g); with
    // grid.z > 1 the samples are split into grid.z consecutive ranges, one per
    // block (more waves per SIMD to hide the Philox chains and the stores; the
    // tile's θ is then loaded once per range — the same draws either way).
    // The ranges are of the flattened (graph, sample) items, g-major, so the
    // blocks of a tile get equal shares (±1) whatever divides what.
    const int fper = kLoop ? (samples * graphs + (int)gridDim.z - 1) / (int)gridDim.z : 1;  // items per block
    const int f0 = kLoop ? (int)blockIdx.z * fper : 0;
    const int z0 = kLoop ? 0 : (int)blockIdx.z;
    const int z1 = kLoop ? max(0, min(samples * graphs, f0 + fper) - f0) : z0 + 1;
    const bool rvalid = lane < 16 && r0 + lane < n;  // lane r stores row r0 + r's word
    // item -> (graph index, sample, counter, tag, its bits / degree slices)
    auto item = [&](int it, int& gidx, int& z) {
        int gl = 0;
        if constexpr (kLoop) {
            const int ig = f0 + it;
            gl = ig / samples;
            z = ig - gl * samples;
        } else {
            z = it;
        }
        gidx = (int)blockIdx.y + gl;
        return gl;
    };
#pragma unroll 1
    for (int base = z0; base < z1; base += kGrp) {
        const int gn = min(kGrp, z1 - base);
        // one item's words out of its draws e[16]: row words (lane r keeps row
        // r's, from ballots), column bits per lane
        auto emit = [&](int q, const bool (&e)[16]) {
            int gidx, z;
            item(base + q, gidx, z);
            uint64_t* __restrict__ gb = bits + ((int64_t)gidx * nsamp + z) * n * words;
            int* __restrict__ da = kDeg ? dacc + ((int64_t)gidx * nsamp + z) * wsi : nullptr;
            uint32_t row_lo = 0, row_hi = 0, cw = 0;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const uint64_t w = __ballot(e[r]);
                row_lo = lane == r ? (uint32_t)w : row_lo;
                row_hi = lane == r ? (uint32_t)(w >> 32) : row_hi;
                cw |= (uint32_t)e[r] << r;
            }
            const uint64_t myrow = ((uint64_t)row_hi << 32) | row_lo;
            if (!diag_tile) {
                if (rvalid) {
                    gb[(int64_t)(r0 + lane) * words + bj] = myrow;
                    if constexpr (kDeg) {  // row part of an off-diagonal tile (diagonal tiles: column part only)
                        const int pc = __popcll(myrow);
                        if (pc != 0) atomicAdd(&da[r0 + lane], pc);
                    }
                }
            } else if (rvalid) {
                rowword[q][wave * 16 + lane] = myrow;
            }
            colpart[q][wave][lane] = cw;
        };
        if constexpr (kInj) {
#pragma unroll 1
            for (int q = 0; q < gn; ++q) {
                bool e[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int i = r0 + r;
                    const float u = (i < n && j < n) ? u_inj[(int64_t)i * nn + j] : 1.0f;
                    e[r] = th[r] >= 0.0f && u < fminf(th[r], 1.0f);
                }
                emit(q, e);
            }
        } else {
            // the draws of kPar items at a time: 4·kPar independent Philox chains
            // per lane (a short group's last pass redraws its last item, unused;
            // one item per block without kLoop draws it alone)
            constexpr int kPar = kLoop ? 2 : 1;
#pragma unroll 1
            for (int q = 0; q < gn; q += kPar) {
                bool e[kPar][16];
#pragma unroll
                for (int h = 0; h < kPar; ++h) {
                    int gidx, z;
                    const int gl = item(base + min(q + h, gn - 1), gidx, z);
                    const uint32_t ctr = counter + (uint32_t)gl;
                    const uint32_t tg = tag + (uint32_t)z * tag_step;
#pragma unroll
                    for (int m = 0; m < 4; ++m) {
                        const U32x4 o = philox4x32_10(U32x4{(uint32_t)j, (uint32_t)((r0 >> 2) + m), tg, ctr}, k0, k1);
                        e[h][4 * m] = (o.x >> 8) < thr[4 * m];
                        e[h][4 * m + 1] = (o.y >> 8) < thr[4 * m + 1];
                        e[h][4 * m + 2] = (o.z >> 8) < thr[4 * m + 2];
                        e[h][4 * m + 3] = (o.w >> 8) < thr[4 * m + 3];
                    }
                }
#pragma unroll
                for (int h = 0; h < kPar; ++h)
                    if (q + h < gn) emit(q + h, e[h]);
            }
        }
        __syncthreads();
        if (wave < gn) {  // wave q: the column words of item base + q
            int gidx, z;
            item(base + wave, gidx, z);
            uint64_t* __restrict__ gb = bits + ((int64_t)gidx * nsamp + z) * n * words;
            int* __restrict__ da = kDeg ? dacc + ((int64_t)gidx * nsamp + z) * wsi : nullptr;
            int pc = 0;
            if (j < n) {
                uint64_t out = (uint64_t)colpart[wave][0][lane] | ((uint64_t)colpart[wave][1][lane] << 16) |
                               ((uint64_t)colpart[wave][2][lane] << 32) | ((uint64_t)colpart[wave][3][lane] << 48);
                if (diag_tile) out |= rowword[wave][lane] | (1ull << lane);  // self-loop: diagonal set to 1
                if (mirror || diag_tile) gb[(int64_t)j * words + bi] = out;
                pc = __popcll(out);
            }
            if constexpr (kDeg) {
                if (pc != 0) atomicAdd(&da[j], pc);
            }
        }
        if (base + kGrp < z1) __syncthreads();  // colpart / rowword are reused by the next group
    }
    if constexpr (kSgd) {
        __shared__ int last_sh;
        bool last = true;
        if (gridDim.z > 1) {
            __syncthreads();  // every thread's θ loads have returned (their draws are done)
            if (threadIdx.x == 0) {
                const int prev = atomicAdd(tile_ctr + tile, 1);
                last_sh = prev == (int)gridDim.z - 1;
                if (last_sh) tile_ctr[tile] = 0;
                // a counter that was not zero on entry (stale or shared workspace):
                // some block counts past the tile's blocks; report it (the engine's
                // error word, EngineScalars.error at byte 32 of `counter_base`)
                if (prev >= (int)gridDim.z && counter_base != nullptr)
                    atomicOr(const_cast<uint32_t*>(counter_base) + 8, kDevErrSgdTileCounter);
            }
            __syncthreads();
            last = last_sh != 0;
        }
        if (last) {
            const float lr = (float)*lr_dev;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int i = r0 + r;
                if (i <= j && j < n) {
                    const int64_t idx = tri_index(i, j, nn);
                    theta_w[idx] = fminf(fmaxf(fmaf(-lr, grad[idx], theta_w[idx]), 0.f), 1.f);
                }
            }
        }
    }
}

// The strict lower triangle of `graphs` bitmasks from their upper triangle
// (lds_bitmask_mirror_degree).  A workgroup takes an 8 × 8 super-block of
// 64 × 64 bit blocks — source row blocks 8R … 8R + 7, words 8C … 8C + 7,
// C >= R — loads its 512 rows × 64 bytes coalesced into LDS, transposes each
// block (rb, w) with w > rb in registers (lane l holds row 64·rb + l's word
// w; six butterfly stages, bit64_transpose, leave lane c with the word rb of
// row 64·w + c), and stores the 512 transposed rows × 64 bytes coalesced.
// (One wave per block with row-strided 8-byte accesses and 64 ballots: 270
// µs for six config-5 graphs; super-blocks with the ballots: 230.)  Graph
// blockIdx.y.
// 64 × 64 bit transpose across a wave: lane l holds row l (bit c = column c);
// afterwards lane l holds column l.  Stage s swaps, between lanes l and l ^ s,
// the s × s sub-blocks off the diagonal of every 2s × 2s block.
__device__ __forceinline__ uint64_t bit64_transpose(uint64_t v, int lane) {
    const uint64_t masks[6] = {0xFFFFFFFF00000000ull, 0xFFFF0000FFFF0000ull, 0xFF00FF00FF00FF00ull,
                               0xF0F0F0F0F0F0F0F0ull, 0xCCCCCCCCCCCCCCCCull, 0xAAAAAAAAAAAAAAAAull};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int s = 32 >> k;
        const uint64_t m = masks[k];  // columns with bit s set
        const uint32_t lo = __shfl_xor((uint32_t)v, s), hi = __shfl_xor((uint32_t)(v >> 32), s);
        const uint64_t x = ((uint64_t)hi << 32) | lo;
        // lanes without bit s keep their columns without bit s and take the
        // partner's such columns, shifted up; lanes with bit s the converse
        v = (lane & s) ? ((v & m) | ((x >> s) & ~m)) : ((v & ~m) | ((x << s) & m));
    }
    return v;
}

constexpr int kMirSb = 8;                 // blocks per super-block side
constexpr int kMirRows = 64 * kMirSb;     // 512 rows
__global__ __launch_bounds__(256) void mirror_kernel(uint64_t* __restrict__ bits, int n, int words) {
    // 2 × 32 KB; entry (r, q) at column q ^ (r & 7): the per-block column reads
    // and writes (lanes on consecutive rows) spread over the banks
    __shared__ uint64_t src[kMirRows][kMirSb];
    __shared__ uint64_t dst[kMirRows][kMirSb];
    int C, R;
    tri_tile((int)blockIdx.x, C, R);  // R <= C
    const int nbw = (n + 63) / 64;
    bits += (int64_t)blockIdx.y * n * words;
    const int t = threadIdx.x;
    // source: rows 512·R + r (r < 512), words 8·C + q (q < 8)
    for (int idx = t; idx < kMirRows * kMirSb; idx += 256) {
        const int r = idx >> 3, q = idx & 7;
        const int row = kMirRows * R + r, w = kMirSb * C + q;
        src[r][q ^ (r & 7)] = (row < n && w < nbw) ? bits[(int64_t)row * words + w] : 0ull;
    }
    __syncthreads();
    const int lane = wave_lane(), wave = wave_id();
    for (int blk = wave; blk < kMirSb * kMirSb; blk += 4) {
        const int rbl = blk >> 3, wl = blk & 7;  // block (row block 8R + rbl, word 8C + wl)
        if (kMirSb * C + wl <= kMirSb * R + rbl) continue;  // (uniform) not strictly upper
        const uint64_t v = src[64 * rbl + lane][wl ^ (lane & 7)];
        dst[64 * wl + lane][rbl ^ (lane & 7)] = bit64_transpose(v, lane);
    }
    __syncthreads();
    // destination: rows 512·C + r, words 8·R + q, where the block was transposed
    for (int idx = t; idx < kMirRows * kMirSb; idx += 256) {
        const int r = idx >> 3, q = idx & 7;
        const int row = kMirRows * C + r, w = kMirSb * R + q;
        if (kMirSb * C + (r >> 6) > w && row < n && w < nbw) bits[(int64_t)row * words + w] = dst[r][q ^ (r & 7)];
    }
}

// One wave per row: popcount of the row's words.
__global__ __launch_bounds__(256) void degree_kernel(const uint64_t* __restrict__ bits, int n,
                                                      int words, int* __restrict__ deg,
                                                      float* __restrict__ s, int deg_stride) {
    const int row = blockIdx.x * 4 + wave_id();
    if (row >= n) return;
    bits += (int64_t)blockIdx.y * n * words;  // batched: graph blockIdx.y
    deg += (int64_t)blockIdx.y * deg_stride;
    s += (int64_t)blockIdx.y * n;
    const int lane = wave_lane();
    const int nbw = (n + 63) / 64;
    const uint64_t* rb = bits + (int64_t)row * words;
    int c = 0;
    for (int w = lane; w < nbw; w += 64) c += __popcll(rb[w]);
    c = wave_sum(c);
    if (lane == 0) {
        deg[row] = c;
        s[row] = inv_sqrt_degree(c);
    }
}

// Single-workgroup exclusive scan of n ints into n+1 row pointers.
__global__ __launch_bounds__(1024) void scan_kernel(const int* __restrict__ deg, int n,
                                                     int* __restrict__ row_ptr) {
    __shared__ int partial[1024];
    deg += (int64_t)blockIdx.y * n;  // batched: graph blockIdx.y
    row_ptr += (int64_t)blockIdx.y * (n + 1);
    const int t = threadIdx.x;
    const int per = (n + 1023) / 1024;
    const int beg = min(n, t * per), end = min(n, beg + per);
    int sum = 0;
    for (int i = beg; i < end; ++i) sum += deg[i];
    partial[t] = sum;
    __syncthreads();
    // Hillis-Steele inclusive scan over the 1024 thread totals.
    for (int o = 1; o < 1024; o <<= 1) {
        const int v = t >= o ? partial[t - o] : 0;
        __syncthreads();
        partial[t] += v;
        __syncthreads();
    }
    int run = t > 0 ? partial[t - 1] : 0;
    for (int i = beg; i < end; ++i) {
        row_ptr[i] = run;
        run += deg[i];
    }
    if (t == 1023) row_ptr[n] = partial[1023];
}


// One wave per row: ascending column indices of the set bits.  Short rows
// (the Cora-sized graphs): each lane pops the bits of its own word after a
// wave scan of the counts.  Dense rows: the row's
// words are scanned 64 at a time; for every NON-ZERO word (uniform loop over
// a ballot) lane l tests bit l, a second ballot + mbcnt gives each set bit its
// position, and the word's entries go out as one contiguous store (128 B for
// a half-dense word) — the earlier per-lane bit-popping form wrote 64
// scattered 4-B addresses per store and ran at ~1 TB/s on config 5's
// 2·10^8-entry graphs.  Same output: columns ascending.
__global__ __launch_bounds__(256) void fill_csr_kernel(const uint64_t* __restrict__ bits, int n,
                                                        int words, const int* __restrict__ row_ptr,
                                                        int* __restrict__ col, int64_t capacity,
                                                        int* __restrict__ overflow,
                                                        const float* __restrict__ s,
                                                        int2* __restrict__ ell,
                                                        const uint8_t* __restrict__ flags) {
    const int row = blockIdx.x * 4 + wave_id();
    if (row >= n) return;
    bits += (int64_t)blockIdx.y * n * words;  // batched: graph blockIdx.y, col stride = capacity
    row_ptr += (int64_t)blockIdx.y * (n + 1);
    col += (int64_t)blockIdx.y * capacity;
    const int lane = wave_lane();
    const int nbw = (n + 63) / 64;
    const uint64_t* rb = bits + (int64_t)row * words;
    const int64_t row_beg = row_ptr[row];
    int64_t base = row_beg;
    bool over = false;
    if (ell != nullptr) {
        s += (int64_t)blockIdx.y * n;
        ell += ((int64_t)blockIdx.y * n + row) * kEllWidth;
        // padding of the ELL head ({row, 0}: a valid index with weight 0)
        const int64_t deg = row_ptr[row + 1] - row_beg;
        if (lane < kEllWidth && lane >= deg) ell[lane] = make_int2(row, 0);
    }
    const int64_t row_deg = row_ptr[row + 1] - row_beg;
    if (row_deg < kDenseRowFill) {  // short rows: each lane pops its own word's bits
        for (int w0 = 0; w0 < nbw; w0 += 64) {
            const int w = w0 + lane;
            uint64_t word = w < nbw ? rb[w] : 0ull;
            const int cnt = __popcll(word);
            int incl = cnt;  // inclusive wave scan of cnt
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int v = __shfl_up(incl, o);
                if (lane >= o) incl += v;
            }
            int64_t pos = base + (incl - cnt);
            while (word) {
                const int bit = __ffsll((unsigned long long)word) - 1;
                const int j = w * 64 + bit;
                if (pos < capacity) col[pos] = j;
                else over = true;
                if (ell != nullptr && pos - row_beg < kEllWidth)
                    ell[pos - row_beg] = make_int2(ell_index(j, flags), __float_as_int(s[j]));
                ++pos;
                word &= word - 1;
            }
            base += __shfl(incl, 63);
        }
        if (over && overflow != nullptr) *overflow = 1;
        return;
    }
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));  // lanes < this lane
    for (int w0 = 0; w0 < nbw; w0 += 64) {
        const int w = w0 + lane;
        const uint64_t word = w < nbw ? rb[w] : 0ull;
        uint64_t nz = __ballot(word != 0ull);
        while (nz) {
            const int src = __ffsll((unsigned long long)nz) - 1;
            nz &= nz - 1;
            const uint32_t lo = __shfl((uint32_t)word, src), hi = __shfl((uint32_t)(word >> 32), src);
            const uint64_t wd = ((uint64_t)hi << 32) | lo;
            const bool set = (wd >> lane) & 1ull;
            const int64_t pos = base + __popcll(wd & below);
            if (set) {
                const int j = (w0 + src) * 64 + lane;
                if (pos < capacity) col[pos] = j;
                else over = true;
                if (ell != nullptr && pos - row_beg < kEllWidth)
                    ell[pos - row_beg] = make_int2(ell_index(j, flags), __float_as_int(s[j]));
            }
            base += __popcll(wd);
        }
    }
    if (over && overflow != nullptr) *overflow = 1;
}

// The CSR fill of the fused sampler (fill.hpp fill_csr_block).
__global__ __launch_bounds__(256) void fill_csr_fused_kernel(const uint64_t* __restrict__ bits, int n, int words,
                                                              const int* __restrict__ dacc, int wsi,
                                                              int* __restrict__ row_ptr, int* __restrict__ col,
                                                              int64_t capacity, float* __restrict__ s,
                                                              int2* __restrict__ ell,
                                                              const uint8_t* __restrict__ flags,
                                                              uint32_t* __restrict__ err) {
    fill_csr_block(blockIdx.x, blockIdx.y, bits, n, words, dacc, wsi, row_ptr, col, capacity, s, ell, flags, err);
}

__global__ void csr_degree_scale_kernel(const int* __restrict__ row_ptr, int n,
                                        int* __restrict__ deg, float* __restrict__ s) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int d = row_ptr[i + 1] - row_ptr[i];
    if (deg != nullptr) deg[i] = d;
    s[i] = inv_sqrt_degree(d);
}

__global__ void philox_uniform_kernel(uint32_t k0, uint32_t k1, uint32_t tag, uint32_t counter,
                                      int rows, int cols, float* __restrict__ out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int rq = blockIdx.y;
    if (j >= cols) return;
    float u[4];
    philox_quad(k0, k1, tag, counter, (uint32_t)j, (uint32_t)rq, u);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = rq * 4 + r;
        if (i < rows) out[(int64_t)i * cols + j] = u[r];
    }
}

}  // namespace lds

using namespace lds;

extern "C" int lds_bitmask_words(int n) {
    int w = (n + 63) / 64;
    return (w + 1) & ~1;
}

extern "C" int lds_philox_uniform(uint64_t seed, uint32_t tag, uint32_t counter, int rows,
                                  int cols, float* out, void* stream) {
    LDS_CHECK_ARG(rows > 0 && cols > 0 && out != nullptr && rows <= 4 * 65535);
    dim3 grid((cols + 255) / 256, (rows + 3) / 4);
    hipLaunchKernelGGL(philox_uniform_kernel, grid, dim3(256), 0, (hipStream_t)stream,
                       (uint32_t)seed, (uint32_t)(seed >> 32), tag, counter, rows, cols, out);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_sample_bitmask(const float* theta, int n, uint64_t seed, uint32_t tag,
                                  uint32_t counter, const float* u_inject, uint64_t* bits,
                                  int words, void* stream) {
    LDS_CHECK_ARG(theta != nullptr && bits != nullptr && n > 0 && n <= (1 << 20));
    LDS_CHECK_ARG(words >= (n + 63) / 64);
    const int nb = (n + 63) / 64;
    const int ntiles = nb * (nb + 1) / 2;
    if (u_inject != nullptr)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(sample_tiles_kernel<true, false, false>), dim3(ntiles), dim3(256), 0,
                           (hipStream_t)stream, theta, n, (uint32_t)seed, (uint32_t)(seed >> 32), tag,
                           counter, (const uint32_t*)nullptr, u_inject, bits, words, ntiles, 0u, 1, 1,
                           (int*)nullptr, 0);
    else
        hipLaunchKernelGGL(HIP_KERNEL_NAME(sample_tiles_kernel<false, false, false>), dim3(ntiles), dim3(256), 0,
                           (hipStream_t)stream, theta, n, (uint32_t)seed, (uint32_t)(seed >> 32), tag,
                           counter, (const uint32_t*)nullptr, u_inject, bits, words, ntiles, 0u, 1, 1,
                           (int*)nullptr, 0);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_sample_bitmask_dev(const float* theta, int n, uint64_t seed, uint32_t tag,
                                      const uint32_t* counter_base, uint32_t counter_offset,
                                      uint64_t* bits, int words, void* stream) {
    LDS_CHECK_ARG(theta != nullptr && bits != nullptr && counter_base != nullptr);
    LDS_CHECK_ARG(n > 0 && n <= (1 << 20) && words >= (n + 63) / 64);
    const int nb = (n + 63) / 64;
    const int ntiles = nb * (nb + 1) / 2;
    hipLaunchKernelGGL(HIP_KERNEL_NAME(sample_tiles_kernel<false, false, false>), dim3(ntiles), dim3(256), 0,
                       (hipStream_t)stream, theta, n, (uint32_t)seed, (uint32_t)(seed >> 32), tag,
                       counter_offset, counter_base, (const float*)nullptr, bits, words, ntiles, 0u, 1, 1,
                       (int*)nullptr, 0);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_bitmask_degree(const uint64_t* bits, int n, int words, int* deg, float* s,
                                  void* stream) {
    LDS_CHECK_ARG(bits != nullptr && deg != nullptr && s != nullptr && n > 0);
    LDS_CHECK_ARG(words >= (n + 63) / 64);
    hipLaunchKernelGGL(degree_kernel, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, bits,
                       n, words, deg, s, n);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_exclusive_scan(const int* deg, int n, int* row_ptr, void* stream) {
    LDS_CHECK_ARG(deg != nullptr && row_ptr != nullptr && n > 0 && n <= (1 << 24));
    hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, deg, n, row_ptr);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_bitmask_fill_csr(const uint64_t* bits, int n, int words, const int* row_ptr,
                                    int* col, int64_t col_capacity, int* overflow,
                                    void* stream) {
    LDS_CHECK_ARG(bits != nullptr && row_ptr != nullptr && col != nullptr && n > 0);
    LDS_CHECK_ARG(words >= (n + 63) / 64 && col_capacity >= 0);
    hipLaunchKernelGGL(fill_csr_kernel, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                       bits, n, words, row_ptr, col, col_capacity, overflow, (const float*)nullptr,
                       (int2*)nullptr, (const uint8_t*)nullptr);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_bitmask_fill_csr_ell(const uint64_t* bits, int n, int words, const int* row_ptr,
                                        int* col, int64_t col_capacity, int* overflow, const float* s,
                                        int* ell, void* stream) {
    LDS_CHECK_ARG(bits != nullptr && row_ptr != nullptr && col != nullptr && n > 0);
    LDS_CHECK_ARG(words >= (n + 63) / 64 && col_capacity >= 0 && s != nullptr && ell != nullptr);
    hipLaunchKernelGGL(fill_csr_kernel, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                       bits, n, words, row_ptr, col, col_capacity, overflow, s, (int2*)ell,
                       (const uint8_t*)nullptr);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_csr_degree_scale(const int* row_ptr, int n, int* deg, float* s,
                                    void* stream) {
    LDS_CHECK_ARG(row_ptr != nullptr && s != nullptr && n > 0);
    hipLaunchKernelGGL(csr_degree_scale_kernel, dim3((n + 255) / 256), dim3(256), 0,
                       (hipStream_t)stream, row_ptr, n, deg, s);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_sample_ws_ints(int n) { return n; }

// Clears the degree workspace of a draw that does not find it zeroed.  A
// kernel rather than hipMemsetAsync, so that a captured step holds kernel
// nodes only (the per-step graphs of the fused runner replay this call).
__global__ void __launch_bounds__(256) zero_ints_kernel(int* __restrict__ p, int64_t count) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) p[i] = 0;
}

// the batched draw's target block count (16 waves per SIMD-slot's worth on
// 256 CUs at 4 waves per block).  MI355X, window draw per call (sample
// splits): Cora S = 16 358 µs unsplit, 317 at 2048 blocks, 310 at 4096, 314
// at 8192; Citeseer S = 16 475 / 429 / 423 / 415; Cora S = 8 189 / 177 /
// 175 / 180 (profiles/r03_draw_split.jsonl)
constexpr int kDrawBlocks = 4096;

// The outer SGD step + clamp (lds_engine_sgd_clamp) and the NEXT window's
// draw of `count` graphs × `samples` replicas from the θ it writes, in one
// pass over the triangle: graph g, sample b takes counter counter_offset + g
// + the scalars' graph counter and tag + b·tag_step, as lds_sample_graphs_multi;
// bits and degree counts as its tile kernel (deg_ws zero on entry); the fill
// is left to the caller (lds_sample_fill_csr).  `scalars`: the engine's
// EngineScalars (graph counter at byte 0, f64 lr at byte 16).  tile_ctr
// (optional): lds_sgd_tile_ints(n) ints, zero on entry and left zero — the
// per-tile counters that let the samples split over grid.z (see the kernel).
extern "C" int lds_sgd_tile_ints(int n) {
    const int nb = (n + 63) / 64;
    return nb * (nb + 1) / 2;
}

extern "C" int lds_sgd_sample_graphs(float* theta, const float* grad, const void* scalars, int n, uint64_t seed,
                                     uint32_t tag, uint32_t tag_step, uint32_t counter_offset, int count,
                                     int samples, uint64_t* bits, int words, int* deg_ws, int* tile_ctr,
                                     void* stream) {
    LDS_CHECK_ARG(theta && grad && scalars && bits && deg_ws && n > 0 && n <= (1 << 20));
    LDS_CHECK_ARG(count > 0 && samples > 0 && (int64_t)count * samples <= 65535 && words >= (n + 63) / 64);
    const int nb = (n + 63) / 64;
    const int ntiles = nb * (nb + 1) / 2;
    const double* lr = reinterpret_cast<const double*>(reinterpret_cast<const char*>(scalars) + 16);
    // with replica samples and the per-tile counters: the (graph, sample)
    // items split over grid.z towards kDrawBlocks blocks, at most one block per
    // sample, as lds_sample_graphs_multi's draw splits its samples (same
    // draws); one block per tile otherwise.  Measured at Cora (no-op exchange
    // captured): S = 8 0.2748 / 0.2745 ms per step unsplit, 0.2716 / 0.2712
    // with five blocks of ten items; S = 1 split into three blocks of two
    // graphs LOST (13.5k against 13.9k steps/s: the extra θ and dθ reads and
    // the counters cost more than the parallelism gains at six items a tile)
    int zsplit = 1;
    if (tile_ctr != nullptr) {
        const int total = count * samples;
        const int want = std::max(1, std::min(samples, (kDrawBlocks + ntiles - 1) / ntiles));
        const int per = (total + want - 1) / want;
        zsplit = (total + per - 1) / per;  // no empty block
    }
    hipLaunchKernelGGL(HIP_KERNEL_NAME(sample_tiles_kernel<false, true, true, true>), dim3(ntiles, 1, zsplit),
                       dim3(256), 0, (hipStream_t)stream, theta, n, (uint32_t)seed, (uint32_t)(seed >> 32), tag,
                       counter_offset, (const uint32_t*)scalars, (const float*)nullptr, bits, words, ntiles, tag_step,
                       samples, count, deg_ws, lds_sample_ws_ints(n), theta, grad, lr, tile_ctr);
    LDS_RETURN_LAST_ERROR();
}

// s = deg^-1/2 of `graphs` graphs from their accumulated degree counts (the
// bitmask form of the fill: dense graphs aggregated from their bits need no CSR).
__global__ __launch_bounds__(256) void degree_scale_kernel(const int* __restrict__ dacc, int wsi, int n,
                                                           float* __restrict__ s) {
    const int row = blockIdx.x * 256 + threadIdx.x;
    if (row >= n) return;
    s[(int64_t)blockIdx.y * n + row] = inv_sqrt_degree(dacc[(int64_t)blockIdx.y * wsi + row]);
}

// The fill launch of lds_sample_graphs_multi alone, for graphs whose bits and
// degree counts were drawn elsewhere (lds_theta_grad_sgd_draw); col == NULL:
// s only (row_ptr, ell unused, may be NULL).
extern "C" int lds_sample_fill_csr(const uint64_t* bits, int n, int words, const int* deg_ws, int graphs,
                                   int* row_ptr, int* col, int64_t col_stride, float* s, int* ell,
                                   const uint8_t* node_flags, uint32_t* err, void* stream) {
    LDS_CHECK_ARG(bits && deg_ws && s && n > 0 && n <= kEllIndex + 1);
    LDS_CHECK_ARG(col == nullptr || (row_ptr != nullptr && col_stride > 0));
    LDS_CHECK_ARG(graphs > 0 && graphs <= 65535 && words >= (n + 63) / 64);
    if (col == nullptr) {
        hipLaunchKernelGGL(degree_scale_kernel, dim3((n + 255) / 256, graphs), dim3(256), 0, (hipStream_t)stream,
                           deg_ws, lds_sample_ws_ints(n), n, s);
        LDS_RETURN_LAST_ERROR();
    }
    hipLaunchKernelGGL(fill_csr_fused_kernel, dim3((n + 15) / 16, graphs), dim3(256), 0, (hipStream_t)stream, bits,
                       n, words, deg_ws, lds_sample_ws_ints(n), row_ptr, col, col_stride, s, (int2*)ell, node_flags,
                       err);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_sample_graphs_multi(const float* theta, int n, uint64_t seed, uint32_t tag,
                                       uint32_t tag_step, const uint32_t* counter_base,
                                       uint32_t counter_offset, int count, int samples, uint64_t* bits,
                                       int words, int* deg_ws, int* row_ptr, int* col, int64_t col_stride,
                                       float* s, int* ell, const uint8_t* node_flags, int ws_zeroed,
                                       uint32_t* err, void* stream) {
    // col == NULL: bitmask, degrees and s only (the bitmask aggregation of
    // dense graphs reads no CSR); row_ptr / ell are then not written.
    // deg_ws: lds_sample_ws_ints(n) ints per graph (degrees first); with CSR
    // the tile kernel accumulates into it, so it must be zero on entry —
    // ws_zeroed = 1 promises that (the engine zeroes it at the end of every
    // window, lds_engine_end_window), 0 lets this call clear it first.
    LDS_CHECK_ARG(theta && bits && deg_ws && s && n > 0 && n <= (1 << 20));
    LDS_CHECK_ARG(col == nullptr || (row_ptr != nullptr && col_stride > 0));
    LDS_CHECK_ARG(count > 0 && samples > 0 && samples <= 65535 && (int64_t)count * samples <= 65535);
    LDS_CHECK_ARG(words >= (n + 63) / 64 && n <= kEllIndex + 1);
    const int nb = (n + 63) / 64;
    const int ntiles = nb * (nb + 1) / 2;
    const int graphs = count * samples;
    const int wsi = lds_sample_ws_ints(n);
    hipStream_t st = (hipStream_t)stream;
    const bool fused = col != nullptr;  // degrees counted by the tiles, scan folded into the fill
    if (fused && !ws_zeroed) {
        const int64_t cnt = (int64_t)graphs * wsi;
        const int blocks = (int)std::min<int64_t>((cnt + 255) / 256, 1024);
        hipLaunchKernelGGL(zero_ints_kernel, dim3(blocks), dim3(256), 0, st, deg_ws, cnt);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return (int)e;
    }
    int* dacc = fused ? deg_ws : nullptr;
    // replica samples and the window's graphs loop inside the block over one
    // θ tile load (θ read once per window)
    const int loop_graphs = count;
    // with replica samples, the (graph, sample) items split over grid.z so the
    // launch has >= kDrawBlocks blocks, at most one block per sample and none
    // empty (one item range per block; same draws)
    int zsplit = 1;
    {
        const int total = count * samples;
        const int want = std::max(1, std::min(samples, (kDrawBlocks + ntiles - 1) / ntiles));
        const int per = (total + want - 1) / want;
        zsplit = (total + per - 1) / per;
    }
    if (samples > 1 || (loop_graphs > 1 && count > 1)) {
        if (fused)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(sample_tiles_kernel<false, true, true>), dim3(ntiles, count / loop_graphs, zsplit),
                               dim3(256), 0, st, theta, n, (uint32_t)seed, (uint32_t)(seed >> 32), tag, counter_offset,
                               counter_base, (const float*)nullptr, bits, words, ntiles, tag_step, samples, loop_graphs,
                               dacc, wsi);
        else
            hipLaunchKernelGGL(HIP_KERNEL_NAME(sample_tiles_kernel<false, true, false>), dim3(ntiles, count / loop_graphs, zsplit),
                               dim3(256), 0, st, theta, n, (uint32_t)seed, (uint32_t)(seed >> 32), tag, counter_offset,
                               counter_base, (const float*)nullptr, bits, words, ntiles, tag_step, samples, loop_graphs,
                               dacc, wsi);
    } else {
        if (fused)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(sample_tiles_kernel<false, false, true>), dim3(ntiles, count, 1), dim3(256), 0,
                               st, theta, n, (uint32_t)seed, (uint32_t)(seed >> 32), tag, counter_offset, counter_base,
                               (const float*)nullptr, bits, words, ntiles, tag_step, 1, 1, dacc, wsi);
        else
            hipLaunchKernelGGL(HIP_KERNEL_NAME(sample_tiles_kernel<false, false, false>), dim3(ntiles, count, 1), dim3(256), 0,
                               st, theta, n, (uint32_t)seed, (uint32_t)(seed >> 32), tag, counter_offset, counter_base,
                               (const float*)nullptr, bits, words, ntiles, tag_step, 1, 1, dacc, wsi);
    }
    if (!fused) {
        hipLaunchKernelGGL(degree_kernel, dim3((n + 3) / 4, graphs), dim3(256), 0, st, bits, n, words,
                           deg_ws, s, wsi);
        LDS_RETURN_LAST_ERROR();
    }
    hipLaunchKernelGGL(fill_csr_fused_kernel, dim3((n + 15) / 16, graphs), dim3(256), 0, st, bits, n, words,
                       (const int*)deg_ws, wsi, row_ptr, col, col_stride, s, (int2*)ell, node_flags, err);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_sample_graphs(const float* theta, int n, uint64_t seed, uint32_t tag,
                                 const uint32_t* counter_base, uint32_t counter_offset, int count,
                                 uint64_t* bits, int words, int* deg_ws, int* row_ptr, int* col,
                                 int64_t col_stride, float* s, int* ell, void* stream) {
    return lds_sample_graphs_multi(theta, n, seed, tag, 0u, counter_base, counter_offset, count, 1, bits,
                                   words, deg_ws, row_ptr, col, col_stride, s, ell, nullptr, 0, nullptr, stream);
}

extern "C" int lds_sample_graph(const float* theta, int n, uint64_t seed, uint32_t tag,
                                uint32_t counter, const float* u_inject, uint64_t* bits, int words,
                                int* deg_ws, int* row_ptr, int* col, int64_t col_capacity,
                                int* overflow, float* s, void* stream) {
    int e = lds_sample_bitmask(theta, n, seed, tag, counter, u_inject, bits, words, stream);
    if (e) return e;
    e = lds_bitmask_degree(bits, n, words, deg_ws, s, stream);
    if (e) return e;
    e = lds_exclusive_scan(deg_ws, n, row_ptr, stream);
    if (e) return e;
    return lds_bitmask_fill_csr(bits, n, words, row_ptr, col, col_capacity, overflow, stream);
}

// The band draw of the band-sharded exchange (BASELINE config 5 at N > 1,
// DESIGN §5b): the Bernoulli draws of the upper-triangle tiles of the rows
// [row0, row1) only — the tiles of 64-row blocks row0 / 64 … — for `count`
// graphs × `samples` replicas (graph g, replica b: counter *counter_base +
// counter_offset + g, tag + b·tag_step, stored as graph g·samples + b, as
// lds_sample_graphs_multi), writing those rows' words and nothing below the
// band (no transposed words, no degree counts).  Every (i, j), i < j, of the
// band gets the bit lds_sample_graphs_multi gives it.  row0 a multiple of 64,
// row1 too or n.
extern "C" int lds_sample_band_bits(const float* theta, int n, uint64_t seed, uint32_t tag, uint32_t tag_step,
                                    const uint32_t* counter_base, uint32_t counter_offset, int count, int samples,
                                    int row0, int row1, uint64_t* bits, int words, void* stream) {
    LDS_CHECK_ARG(theta && bits && n > 0 && n <= (1 << 20) && words >= (n + 63) / 64);
    LDS_CHECK_ARG(count > 0 && samples > 0 && (int64_t)count * samples <= 65535);
    LDS_CHECK_ARG(0 <= row0 && row0 < row1 && row1 <= n && row0 % 64 == 0 && (row1 % 64 == 0 || row1 == n));
    const int nb = (n + 63) / 64, b0 = row0 / 64, b1 = (row1 + 63) / 64;
    int64_t tiles = 0;
    for (int b = b0; b < b1; ++b) tiles += nb - b;
    LDS_CHECK_ARG(tiles > 0 && tiles < (1 << 30));
    int zsplit = 1;  // as lds_sample_graphs_multi: the (graph, sample) items over grid.z
    {
        const int total = count * samples;
        const int want = std::max(1, std::min(samples, (int)((kDrawBlocks + tiles - 1) / tiles)));
        const int per = (total + want - 1) / want;
        zsplit = (total + per - 1) / per;
    }
    hipLaunchKernelGGL(HIP_KERNEL_NAME(sample_tiles_kernel<false, true, false>), dim3((unsigned)tiles, 1, zsplit),
                       dim3(256), 0, (hipStream_t)stream, theta, n, (uint32_t)seed, (uint32_t)(seed >> 32), tag,
                       counter_offset, counter_base, (const float*)nullptr, bits, words, (int)tiles, tag_step,
                       samples, count, (int*)nullptr, 0, (float*)nullptr, (const float*)nullptr,
                       (const double*)nullptr, (int*)nullptr, b0, 0);
    LDS_RETURN_LAST_ERROR();
}

// Complete `graphs` bitmasks whose upper triangle (diagonal words included)
// is drawn — e.g. assembled from the row bands of lds_sample_band_bits —
// with their strict lower triangle (the transposed words), then their
// degrees into deg_ws (lds_sample_ws_ints(n) ints per graph) and s = deg^-1/2
// ([graphs][n]), as lds_sample_graphs_multi leaves them with col = NULL.
extern "C" int lds_bitmask_mirror_degree(uint64_t* bits, int n, int words, int graphs, int* deg_ws, float* s,
                                         void* stream) {
    LDS_CHECK_ARG(bits && deg_ws && s && n > 0 && n <= (1 << 20) && words >= (n + 63) / 64 && graphs > 0 &&
                  graphs <= 65535);
    hipStream_t st = (hipStream_t)stream;
    const int nsb = ((n + 63) / 64 + kMirSb - 1) / kMirSb;  // super-blocks per side
    if (n > 64)
        hipLaunchKernelGGL(mirror_kernel, dim3(nsb * (nsb + 1) / 2, graphs), dim3(256), 0, st, bits, n, words);
    hipLaunchKernelGGL(degree_kernel, dim3((n + 3) / 4, graphs), dim3(256), 0, st, (const uint64_t*)bits, n, words,
                       deg_ws, s, lds_sample_ws_ints(n));
    LDS_RETURN_LAST_ERROR();
}
