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
#include "bitagg.hpp"
#include "spill.hpp"

namespace lds {

// Per-block column maxima of |s_k z_kf| (non-negative floats compare as
// their bit patterns), kColBlocks partials.  1024 threads = 256 rows × four
// feature quads per pass (one float4 of Z per thread when Z is 16-byte
// aligned), so at N = 20 000 every thread has its loads in flight at once:
// one round trip, where 256 blocks of 16 rows × 16 features took five.  The
// launch itself did not get faster (4.93 vs 4.95 µs at N = 20 000: the floor
// of a dependent launch there), but a quarter of the partials makes the
// readers' reductions (colmax_of) one round of loads.  The maximum is
// order-independent: the same values as any other partition.
template <bool kVec>
__global__ __launch_bounds__(1024) void bitagg_colmax_kernel(const float* __restrict__ s, int n,
                                                             const float* __restrict__ z, int ldz,
                                                             uint32_t* __restrict__ colmax) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int fq = t & 3;  // features 4fq .. 4fq + 3
    uint32_t m[4] = {0u, 0u, 0u, 0u};
#pragma unroll 2
    for (int k = blockIdx.x * 256 + (t >> 2); k < n; k += kColBlocks * 256) {
        const float sk = s[k];
        const float* zr = z + (int64_t)k * ldz + 4 * fq;
        float v[4];
        if constexpr (kVec) {
            const float4 w = *reinterpret_cast<const float4*>(zr);
            v[0] = w.x, v[1] = w.y, v[2] = w.z, v[3] = w.w;
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = zr[i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) m[i] = max(m[i], __float_as_uint(fabsf(sk * v[i])));
    }
    // the 16 lanes of a wave holding quad fq: xor over lane bits 2..5
#pragma unroll
    for (int sh = 4; sh < 64; sh <<= 1)
#pragma unroll
        for (int i = 0; i < 4; ++i) m[i] = max(m[i], (uint32_t)__shfl_xor((int)m[i], sh));
    __shared__ uint32_t red[16][kF];
    if (lane < 4)
#pragma unroll
        for (int i = 0; i < 4; ++i) red[wave][4 * lane + i] = m[i];
    __syncthreads();
    if (t < kF) {
        uint32_t r = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) r = max(r, red[w][t]);
        colmax[blockIdx.x * kF + t] = r;
    }
}

// Fixed-point digits of s⊙Z in the chunk layout [chunk][q][limb][g][f][16 B]:
// one thread per dword of a lane fragment (chunk c, k-step q, lane group g,
// feature f, dword dd) = 4 columns, one 4-byte store per limb (a wave's 64
// threads: one 256-byte run per limb).  The thread's s·z products are loaded
// before the column maxima are reduced (every thread of the block reads a
// quarter of the partials), so the block pays one round trip, not three.
// Columns past n are 0.
__global__ __launch_bounds__(256) void bitagg_quant_kernel(const float* __restrict__ s, int n,
                                                           const float* __restrict__ z, int ldz,
                                                           const uint32_t* __restrict__ colmax,
                                                           int8_t* __restrict__ zq, int chunks) {
    __shared__ uint32_t red[4][kF];
    __shared__ int e_sh[kF];
    const int t = threadIdx.x, lane = t & 63;
    const int idx = blockIdx.x * 256 + t;   // (((c·8 + q)·4 + g)·16 + f)·4 + dd
    const bool live = idx < chunks * kSteps * 4 * kF * 4;
    const int dd = idx & 3, f = (idx >> 2) & 15, g = (idx >> 6) & 3, q = (idx >> 8) & 7, c = idx >> 11;
    const int kb = c * kChunk + 128 * g + 32 * (q >> 1) + 4 * (q & 1) + dd;
    float tv[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int k = kb + 8 * b;
        tv[b] = (live && k < n) ? s[k] * z[(int64_t)k * ldz + f] : 0.f;
    }
    uint32_t m = 0;
#pragma unroll
    for (int b = t >> 4; b < kColBlocks; b += 16) m = max(m, colmax[b * kF + (t & 15)]);
    m = max(m, (uint32_t)__shfl_xor((int)m, 16));
    m = max(m, (uint32_t)__shfl_xor((int)m, 32));
    if (lane < kF) red[t >> 6][lane] = m;
    __syncthreads();
    if (t < kF) e_sh[t] = col_exponent(max(max(red[0][t], red[1][t]), max(red[2][t], red[3][t])));
    __syncthreads();
    if (!live) return;
    const int e = e_sh[f];
    uint32_t out[kLimbs] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        int v = kb + 8 * b < n ? (int)rintf(ldexpf(tv[b], e)) : 0;
#pragma unroll
        for (int L = 0; L < kLimbs; ++L) {
            const int d = ((v + 128) & 255) - 128;   // balanced digit in [-128, 127]
            out[L] |= (uint32_t)(d & 255) << (8 * b);
            v = (v - d) >> 8;
        }
    }
#pragma unroll
    for (int L = 0; L < kLimbs; ++L)
        *(uint32_t*)(zq + (int64_t)c * kChunkBytes + (q * kLimbs + L) * 1024 + g * 256 + f * 16 + dd * 4) = out[L];
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

// ---------------------------------------------------------------------------
// CSR-SpMM for dense sampled graphs (BASELINE config 5: N = 20 000, ~N/2
// entries per row; lds_spmm_norm_dense).  The operator of lds_spmm_norm —
// torch.mm(normalize_adjacency_matrix(A), Z) (src/models/layers.py:44,
// src/utils/graph.py:136-153) on the sampled graph's CSR — with the column
// index stream (4 bytes per entry, 0.8 GB per call at config 5) read once
// from HBM and nothing else of size nnz touched:
//  - per 16-row tile, 8 streaming waves read the tile's CSR rows (each lane
//    16 consecutive entries per step, four 16-byte loads, two steps in
//    flight) and set the entries' bits in a 16-row bit tile in LDS (OR in
//    registers, then one or two LDS ORs per lane and step);
//  - 4 MFMA waves multiply the previous tile's bits with the fixed-point
//    digits of s⊙Z on the int8 matrix cores, exactly as lds_aggregate_bitmask
//    does from the sampler's bitmask (same digits and k order, exact int32
//    sums), while the streaming waves fill the next tile: two bit-tile
//    buffers, one barrier per tile.  MFMA wave m owns k-steps 2m, 2m + 1 of
//    every 512-column chunk, i.e. dwords ≡ m (mod 4) of each bit row, and
//    clears exactly those after its last read, so no other wave waits on it.
//  - Why not gathers: one 64-byte row of s⊙Z per entry is 12.8 GB of LDS
//    reads per call at this density, more than the LDS delivers in the time
//    the index stream takes; here each tile reads s⊙Z as 1.3 MB of digits
//    from L2.
// Workgroups are persistent (one per CU; tiles b, b + grid, …).  Columns
// must be distinct within a row (a CSR of a 0/1 matrix); their order is free.
// ---------------------------------------------------------------------------
constexpr int kDnStream = 8;                       // streaming waves (rows 2w, 2w + 1 of each tile)
// (kDnMma = 8 MFMA waves: k-steps 2·(m >> 1), + 1 of the chunks of parity m & 1; kDnStep = 512 entries
// per step, lane l: entries p + 8l … + 7; kDnMaxChunks, kDnMaxGrid, kDnPartBytes: bitagg.hpp)
constexpr int kDnThreads = 64 * (kDnStream + kDnMma);
constexpr int kDnUnits = 8;                        // 1-KB ring units per streaming wave (a step takes two)

int dense_lds_bytes(int chunks) { return 2 * 16 * 16 * chunks * 4 + kDnStream * kDnUnits * 1024; }

// A streaming wave's position (wave-uniform): tile `it` of this workgroup,
// row slot rr (row 2·wave + rr of the tile), the entries [p, p + 512) of that
// row's [beg, end), p ≡ 0 mod 4.
struct Step {
    int it, rr, beg, end, p;
};
// The next step: the row's next 512 entries, else the next non-empty row
// slot, else the next tile (it == my_tiles: past the last).
__device__ __forceinline__ void dn_advance(Step& s, const int* __restrict__ rp, int n, int my_tiles, int wave) {
    if (s.rr >= 0) {
        s.p += kDnStep;
        if (s.p < s.end) return;
    }
    while (true) {
        if (++s.rr == 2) {
            s.rr = 0;
            ++s.it;
        }
        if (s.it >= my_tiles) return;
        const int row = ((int)blockIdx.x + s.it * (int)gridDim.x) * 16 + 2 * wave + s.rr;
        if (row >= n) continue;
        s.beg = __builtin_amdgcn_readfirstlane(rp[row]);
        s.end = __builtin_amdgcn_readfirstlane(rp[row + 1]);
        s.p = s.beg & ~3;
        if (s.beg < s.end) return;
    }
}

// (Round 3's timing ablations of this kernel — no MFMA waves, no bit setting,
// no streaming, constant digits — are in r03_spmm_dense_ablations.txt.)
__global__ __launch_bounds__(kDnThreads, 1) void csr_dense_agg_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, int n, const int8_t* __restrict__ zq, int chunks,
    const uint32_t* __restrict__ colmax, const float* __restrict__ s, float* __restrict__ y, int ldy, int beta,
    int64_t* __restrict__ parts) {
    extern __shared__ __attribute__((aligned(16))) uint32_t dn_lds[];
    __shared__ int e_sh[kF];
    const int rs = 16 * chunks;                          // dwords per bit-tile row
    uint32_t* const tiles = dn_lds;                      // [2][16][rs]
    uint32_t* const ring = dn_lds + 2 * 16 * rs;         // [kDnStream][kDnUnits][256]
    // [2][kDnMma][16 rows][16 f] int64 partials of this workgroup (global scratch, L2)
    int64_t* const red = parts + (size_t)blockIdx.x * (kDnPartBytes / 8);
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int ntile = (n + 15) / 16;
    const int my_tiles = ntile > (int)blockIdx.x ? (ntile - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    const int nnz = rp[n];

    for (int d = 4 * t; d < 2 * 16 * rs; d += 4 * kDnThreads)
        *reinterpret_cast<uint4*>(tiles + d) = make_uint4(0u, 0u, 0u, 0u);
    if (t < 64) {  // per-feature exponents (lds_aggregate_bitmask's quantisation)
        const uint32_t m = colmax_of(colmax, t);
        if (t < kF) e_sh[t] = col_exponent(m);
    }

    // Streaming waves: their index stream through a ring of 1-KB LDS units
    // filled by direct loads three steps ahead, across rows and tiles (the next
    // tile's entries land before the tile barrier; their bits are set after it).
    Step is{0, -1, 0, 0, 0}, ps{0, -1, 0, 0, 0};
    int kis = 0, kps = 0;  // steps issued / processed
    const uint32_t ring_lds = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint32_t*)ring) +
                              (uint32_t)(wave * kDnUnits * 1024);
    const uint32_t* myring = ring + wave * kDnUnits * 256;
    auto issue = [&]() {
        const uint32_t unit = (uint32_t)((2 * kis) % kDnUnits);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int a = is.p + 256 * h + 4 * lane;
            const int* src = a + 4 <= nnz ? col + a : col;  // past the array: a dummy block (reloaded below)
            lds_dma16(src, ring_lds + (unit + h) * 1024u);
        }
        ++kis;
        dn_advance(is, rp, n, my_tiles, wave);
    };
    if (wave < kDnStream) {
        dn_advance(is, rp, n, my_tiles, wave);
        ps = is;
        for (int d = 0; d < 3 && is.it < my_tiles; ++d) issue();
    }
    __syncthreads();

    const int mw = wave - kDnStream;  // MFMA wave index
    const int r16 = lane & 15, g = lane >> 4;
    for (int it = 0; it <= my_tiles; ++it) {
        const int buf = it & 1;
        if (wave < kDnStream) {
            while (ps.it == it && it < my_tiles) {
                if (is.it < my_tiles) issue();
                // step kps landed: at most the three younger steps (two loads each) in flight
                if (kis - kps == 4) __builtin_amdgcn_s_waitcnt(0x0F76);  // vmcnt(6)
                else __builtin_amdgcn_s_waitcnt(0x0F70);                 // vmcnt(0)
                asm volatile("" ::: "memory");
                const uint32_t* sl = myring + ((2 * kps) % kDnUnits) * 256 + 8 * lane;
                const int4 c0 = *reinterpret_cast<const int4*>(sl);
                const int4 c1 = *reinterpret_cast<const int4*>(sl + 4);
                int c[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
                uint32_t* rb = tiles + buf * 16 * rs + (2 * wave + ps.rr) * rs;
                const int p = ps.p + 8 * lane;
                // interior step (every entry of it is the row's, none from a dummy block): the fast path
                const bool interior = ps.p >= ps.beg && ps.p + kDnStep <= ps.end && ps.p + kDnStep + 4 <= nnz;
                bool done = false;
                if (interior) {
                    // the eight columns within the 64 from the first one's word (the
                    // dense, ascending case): one 64-bit mask, two LDS ORs
                    const uint32_t wf = (uint32_t)c[0] >> 5;
                    const int base = (int)(wf << 5);
                    uint32_t out = 0u;
                    uint64_t m = 0;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const uint32_t r = (uint32_t)(c[e] - base);
                        out |= r >> 6;  // nonzero: outside [base, base + 64)
                        m |= 1ull << (r & 63);
                    }
                    if (out == 0u) {
                        dn_or(rb + wf, (uint32_t)m);
                        dn_or(rb + wf + 1, (uint32_t)(m >> 32));
                        done = true;
                    }
                }
                if (!done) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const int idx = p + e;
                        if (idx >= ps.beg && idx < ps.end) {
                            const int v = (idx & ~3) + 4 > nnz ? col[idx] : c[e];
                            atomicOr(rb + (v >> 5), 1u << (v & 31));
                        }
                    }
                }
                ++kps;
                dn_advance(ps, rp, n, my_tiles, wave);
            }
        } else if (it >= 1) {
            // multiply tile it - 1 (its bits in buffer buf ^ 1): k-steps 2·pm, 2·pm + 1
            // of the chunks of parity cp, the digits from L2 through a ring of
            // register sets three k-steps ahead; then clear the dwords of the buffer
            // this wave read (dword pm of every group of its chunks: no other wave
            // reads them)
            const int pm = mw >> 1, cp = mw & 1;
            uint32_t* tb = tiles + (buf ^ 1) * 16 * rs;
            const uint32_t* ta = tb + r16 * rs + 4 * g + pm;  // + 16·c
            v4i acc[kLimbs];
#pragma unroll
            for (int L = 0; L < kLimbs; ++L) acc[L] = v4i{0, 0, 0, 0};
            const v4i* zv = reinterpret_cast<const v4i*>(zq) + (2 * pm * kLimbs) * 64 + lane;
            constexpr int kRing = 4;
            const int ncp = (chunks - cp + 1) / 2;  // this wave's chunks cp, cp + 2, …
            const int nj = 2 * ncp;                 // j = 2i + h: chunk cp + 2i, k-step 2·pm + h
            v4i bq[kRing][kLimbs];
            auto bload = [&](int j, v4i (&b)[kLimbs]) {
                const int c = cp + 2 * (j >> 1), h = j & 1;
#pragma unroll
                for (int L = 0; L < kLimbs; ++L)
                    b[L] = j < nj ? zv[(int64_t)c * (kChunkBytes / 16) + (h * kLimbs + L) * 64] : v4i{0, 0, 0, 0};
            };
#pragma unroll
            for (int d = 0; d < kRing - 1; ++d) bload(d, bq[d]);
            uint32_t w = 0u;
#pragma unroll 1
            for (int j0 = 0; j0 < nj; j0 += kRing) {
#pragma unroll
                for (int d = 0; d < kRing; ++d) {
                    const int j = j0 + d;
                    if (j < nj) {
                        bload(j + kRing - 1, bq[(d + kRing - 1) % kRing]);
                        const int h = d & 1;  // kRing even: j & 1 == d & 1
                        if (h == 0) w = ta[16 * (cp + 2 * (j >> 1))];
                        const int sh = 4 * h;  // k-step 2·pm + h: dword pm, shift 4·(q & 1)
                        v4i a;
                        a.x = (int)((w >> sh) & 0x01010101u);
                        a.y = (int)((w >> (sh + 1)) & 0x01010101u);
                        a.z = (int)((w >> (sh + 2)) & 0x01010101u);
                        a.w = (int)((w >> (sh + 3)) & 0x01010101u);
#pragma unroll
                        for (int L = 0; L < kLimbs; ++L)
                            acc[L] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bq[d][L], acc[L], 0, 0, 0);
                    }
                }
            }
            int64_t* rd = red + ((it - 1) & 1) * (kDnMma * 256) + mw * 256;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                rd[(4 * g + i) * 16 + r16] = (int64_t)acc[0][i] + ((int64_t)acc[1][i] << 8) +
                                             ((int64_t)acc[2][i] << 16) + ((int64_t)acc[3][i] << 24);
            // dwords 16c + 4g' + pm of every row, c ≡ cp (mod 2): lane = (row, g')
            for (int e = lane; e < 16 * 4 * ncp; e += 64) {
                const int row = e & 15, gg = (e >> 4) & 3, c = cp + 2 * (e >> 6);
                tb[row * rs + 16 * c + 4 * gg + pm] = 0u;
            }
        }
        __syncthreads();
        if (it >= 1 && wave >= kDnStream && t < 64 * kDnStream + 256) {  // tile it - 1: partials summed, scaled, stored
            const int tile = (int)blockIdx.x + (it - 1) * (int)gridDim.x;
            const int64_t* rdb = red + ((it - 1) & 1) * (kDnMma * 256);
            {
                const int o = t - 64 * kDnStream;  // output lr·16 + f
                const int lr = o >> 4, f = o & 15;
                const int row = tile * 16 + lr;
                if (row < n) {
                    int64_t v = 0;
#pragma unroll
                    for (int m = 0; m < kDnMma; ++m) v += rdb[m * 256 + o];
                    const float r = s[row] * (float)ldexp((double)v, -e_sh[f]);
                    float* out = y + (int64_t)row * ldy + f;
                    *out = beta ? *out + r : r;
                }
            }
        }
    }
}

}  // namespace lds

using namespace lds;

static void launch_colmax(const float* s, int n, const float* z, int ldz, uint32_t* colmax, hipStream_t st) {
    if ((ldz & 3) == 0 && ((uintptr_t)z & 15) == 0)
        hipLaunchKernelGGL(bitagg_colmax_kernel<true>, dim3(kColBlocks), dim3(1024), 0, st, s, n, z, ldz, colmax);
    else
        hipLaunchKernelGGL(bitagg_colmax_kernel<false>, dim3(kColBlocks), dim3(1024), 0, st, s, n, z, ldz, colmax);
}

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
    launch_colmax(s, n, z, ldz, w.colmax, st);
    hipLaunchKernelGGL(bitagg_quant_kernel, dim3(nc * kSteps * 4 * kF * 4 / 256), dim3(256), 0, st,
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
    launch_colmax(s, n, z, ldz, w.colmax, st);
    hipLaunchKernelGGL(bitagg_quant_kernel, dim3(nc * kSteps * 4 * kF * 4 / 256), dim3(256), 0, st,
                       s, n, z, ldz, (const uint32_t*)w.colmax, w.zq, nc);
    hipLaunchKernelGGL(bitagg_main_kernel, dim3(row_groups_of(n), ks), dim3(kThreads), 0, st, bits, words, n,
                       (const int8_t*)w.zq, nc, ks, w.part, (const uint32_t*)w.colmax, s, (float*)nullptr, 0, 0,
                       1);
    LDS_RETURN_LAST_ERROR();
}

// Workspace of lds_spmm_norm_dense: lds_aggregate_bitmask's column maxima and
// digit chunks, then (grid < 0) the tile kernel's partials.
extern "C" int64_t lds_spmm_dense_ws_bytes(int n) {
    if (n <= 0) return 0;
    return dense_scratch_off(n) + (int64_t)kDnMaxGrid * kDnPartBytes;
}

extern "C" int lds_spmm_dense_max_n(void) { return kDnMaxChunks * kChunk; }

// grid >= 0: the spill-pass kernel on `grid` workgroups (0: one per CU; rows
// split evenly, at most kSpMaxRows per workgroup); grid < 0: the round-3 tile
// kernel (csr_dense_agg_kernel, any column order) on -grid persistent
// workgroups.  MI355X, config 5 (n = 20 000, 2·10⁸ entries): spill-pass
// 164-168 µs per launch, tile kernel 230-243.
extern "C" int lds_spmm_norm_dense(const int* row_ptr, const int* col, const float* s, int n, const float* z,
                                   int ldz, float* y, int ldy, int beta, void* ws, int grid, int quantize,
                                   uint32_t* err, void* stream) {
    LDS_CHECK_ARG(row_ptr && col && s && z && y && ws && n > 0 && n <= kDnMaxChunks * kChunk);
    LDS_CHECK_ARG(ldz >= kF && ldy >= kF);
    LDS_CHECK_ARG((((uintptr_t)col) & 15) == 0 && (((uintptr_t)ws) & 15) == 0);
    hipStream_t st = (hipStream_t)stream;
    const Ws w = carve(ws, n);
    const int nc = chunks_of(n);
    if (quantize) {
        launch_colmax(s, n, z, ldz, w.colmax, st);
        hipLaunchKernelGGL(bitagg_quant_kernel, dim3(nc * kSteps * 4 * kF * 4 / 256), dim3(256), 0, st, s, n, z,
                           ldz, (const uint32_t*)w.colmax, w.zq, nc);
    }
    if (grid < 0) {  // the tile kernel
        const int ntile = (n + 15) / 16;
        int g = -grid;
        if (g > kDnMaxGrid) g = kDnMaxGrid;
        if (g > ntile) g = ntile;
        const int lds = dense_lds_bytes(nc);
        const hipError_t e = allow_lds(&csr_dense_agg_kernel, lds);
        if (e != hipSuccess) return (int)e;
        hipLaunchKernelGGL(csr_dense_agg_kernel, dim3(g), dim3(kDnThreads), lds, st, row_ptr, col, n,
                           (const int8_t*)w.zq, nc, (const uint32_t*)w.colmax, s, y, ldy, beta,
                           reinterpret_cast<int64_t*>(reinterpret_cast<char*>(ws) + dense_scratch_off(n)));
        LDS_RETURN_LAST_ERROR();
    }
    return spill::sp_launch<0>(row_ptr, col, s, n, w, y, ldy, beta, grid, err, st);
}
