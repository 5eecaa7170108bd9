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

// ---------------------------------------------------------------------------
// CSR-SpMM for dense sampled graphs, spill-pass form (the product of
// lds_spmm_norm_dense since round 4).  Each workgroup owns one
// contiguous block of rows (R <= 96) and sweeps its columns in P passes of
// cpp 512-column chunks, with three LDS bit buffers (R rows × cpp·64 B each):
//  * streaming waves 0-11 (wave w: local rows w, w + 12, …) load 2-KB steps
//    of col (512 entries, 8 per lane as two 16-byte loads) into a register
//    ring four steps deep (three in flight; asm loads with counted waits, so
//    the compiler never waits early) and set each entry's bit in pass p's
//    buffer; entries of pass p + 1 that a step holds (a row's boundary step,
//    or steps streamed past a row's predicted pass end) go to pass p + 1's
//    buffer at once ("spill"), so no step is read twice.  A row's stream in
//    pass p ends at its predicted end (the row's remaining entries × the
//    pass's share of the remaining columns + kSpMargin); a row whose boundary
//    lies beyond it is finished with blocking loads (rare: dense rows are
//    binomial).  Entries past pass p + 1 (sparse rows only) are left for a
//    later pass to re-read.
//  * multiply waves 12-15 (limb m, both k-halves of every chunk) run pass
//    p − 1's buffer against the digits of its chunks while pass p streams
//    (lds_aggregate_bitmask's digits, k order and exact int32 sums); the last
//    of them to finish a buffer clears it for pass p + 2's spills.  One
//    barrier per pass.
// Bit setting, per lane and step: the fast path ORs the lane's eight columns
// into one 64-bit window (two LDS ORs) when the step is interior to its row
// and every column lies in the window and inside the pass; two more windowed
// paths take lanes wholly in pass p + 1 and lanes straddling the boundary;
// everything else goes entry by entry (sp_put).  The sums of the multiply
// waves meet in LDS as int64 adds (exact, order free), then y = s_i · 2^-e_f · Σ.
//
// Columns must ascend within each row (canonical CSR, as every sampler and
// fill of this package writes it): a pass's stream of a row starts where the
// row's previous pass ended.  The windowed paths test every column they place
// (not just a lane's first and last), so a column out of order is either
// placed exactly or reaches sp_put below the pass's first column — an entry
// whose pass has already been multiplied.  That, and a column outside [0, n),
// sets LDS_DEVERR_CSR_COLUMNS in the caller's error word instead of being
// dropped silently; a single-pass geometry (small n) places every column
// exactly, in any order.
// ---------------------------------------------------------------------------
constexpr int kSpStream = 12;         // streaming waves 0-11; multiply waves 12-15
constexpr int kSpMul = 16 - kSpStream;
constexpr int kSpThreads = 1024;
constexpr int kSpE = 8;               // entries per lane and step
constexpr int kSpStepEntries = 64 * kSpE;  // 512 entries (2 KB) per step
constexpr int kSpDepth = 4;           // register ring slots per streaming wave (three steps in flight)
constexpr int kSpMaxTiles = 6;
constexpr int kSpMaxRows = 16 * kSpMaxTiles;  // rows per workgroup
constexpr int kSpMaxGrid = 512;
constexpr int kSpMargin = 192;        // entries streamed past a row's predicted pass end
constexpr int kSpStateInts = 3 * kSpMaxRows + 16 + 4;  // pos, rend, fin per row; the exponents; done counters
constexpr int kSpNone = 0x7FFFFFFF;

struct SpGeom {
    int cpp, passes, rowdw;  // chunks per pass, passes, dwords per buffer row (16·cpp + 2: bank spread)
};
inline SpGeom sp_geom(int chunks, int tiles) {
    const int rows = 16 * tiles;
    int cpp = ((163840 - 4 * kSpStateInts) / (3 * rows * 4) - 2) / 16;
    if (cpp > chunks) cpp = chunks;
    if (cpp < 1) cpp = 1;
    const int passes = (chunks + cpp - 1) / cpp;
    cpp = (chunks + passes - 1) / passes;
    return SpGeom{cpp, passes, 16 * cpp + 2};
}
inline int sp_lds_bytes(int tiles, const SpGeom& g) { return 3 * 16 * tiles * g.rowdw * 4 + 4 * kSpStateInts; }

// Entry c (column) of a row in pass p: its bit in pass p's buffer row bp
// (c < hi), pass p + 1's row bq (c < hq), or past both (returns true).  A
// column below the pass (out of order: its pass is gone) sets `bad`.
__device__ __forceinline__ bool sp_put(int c, int lo, int hi, int hq, uint32_t* bp, uint32_t* bq, bool& spill,
                                       bool& bad) {
    if (c < lo) {
        bad = true;
        return false;
    }
    if (c < hi) {
        atomicOr(bp + ((c - lo) >> 5), 1u << ((c - lo) & 31));
        return false;
    }
    spill = true;
    if (c < hq) {
        atomicOr(bq + ((c - hi) >> 5), 1u << ((c - hi) & 31));
        return false;
    }
    return true;
}

// A rare path's column load (the array's last step, rows finished with
// blocking loads), issued from asm with its own vmcnt(0): a plain load there
// leaves the compiler's wait analysis believing some ring register may still
// be waiting on it, and it then waits vmcnt(1-2) in the hot path of every step
// (measured: 192 against 164 µs at config 5 with the plain loads).
__device__ __forceinline__ int sp_ld(const int* p) {
    int v;
    asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}

// OR of a lane's eight window offsets c_e - base (as unsigned: a column below
// the base is huge): < 64 iff every column lies in [base, base + 64), and
// base + it bounds the largest column from above.
__device__ __forceinline__ uint32_t sp_offsets(const int (&c)[kSpE], int base, uint32_t (&r)[kSpE]) {
    uint32_t o = 0u;
#pragma unroll
    for (int e = 0; e < kSpE; ++e) {
        r[e] = (uint32_t)(c[e] - base);
        o |= r[e];
    }
    return o;
}

// kCheck (err != NULL): the windowed paths test every column and the error
// word is set as described above; without it (the caller guarantees
// ascending columns in [0, n), as for every CSR this library builds) they test
// a lane's first and last column only, as the round-4 product did.
template <int kTiles, bool kCheck>
__global__ __launch_bounds__(kSpThreads, 1) void csr_spill_agg_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, int n, int rows_per_wg, const int8_t* __restrict__ zq,
    int chunks, int cpp, int passes, int rowdw, const uint32_t* __restrict__ colmax, const float* __restrict__ s,
    float* __restrict__ y, int ldy, int beta, uint32_t* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint32_t sp_lds[];
    constexpr int D = kSpDepth, kStep = kSpStepEntries;
    static_assert((D - 1) * (kSpE / 4) <= 15, "vmcnt field");
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int r0 = (int)blockIdx.x * rows_per_wg;
    const int nrows = min(rows_per_wg, n - r0);
    if (nrows <= 0) return;  // (uniform: the whole workgroup)
    const int rowsL = 16 * ((rows_per_wg + 15) / 16);  // buffer rows (the host sized LDS for these)
    const int bufdw = rowsL * rowdw;
    int* const pos = reinterpret_cast<int*>(sp_lds + 3 * bufdw);
    int* const rend = pos + kSpMaxRows;
    int* const fin = rend + kSpMaxRows;
    int* const e_sh = fin + kSpMaxRows;
    int* const done = e_sh + 16;  // per buffer: multiply waves finished with it
    const int nnz = rp[n];
    const int span = cpp * kChunk;  // columns per pass
    for (int i = t; i < 3 * bufdw; i += kSpThreads) sp_lds[i] = 0u;
    for (int i = t; i < nrows; i += kSpThreads) {
        pos[i] = rp[r0 + i];
        rend[i] = rp[r0 + i + 1];
        fin[i] = -1;
    }
    if (t < 64) {  // per-feature exponents (lds_aggregate_bitmask's quantisation)
        const uint32_t m = colmax_of(colmax, t);
        if (t < kF) e_sh[t] = col_exponent(m);
        if (t < 3) done[t] = 0;
    }
    __syncthreads();

    v4i acc[kTiles];
#pragma unroll
    for (int T = 0; T < kTiles; ++T) acc[T] = v4i{0, 0, 0, 0};

    if (wave < kSpStream) {
        // ---- streaming waves -------------------------------------------------
        const int nrw = nrows > wave ? (nrows - 1 - wave) / kSpStream + 1 : 0;  // this wave's rows
        const int* const dummy = reinterpret_cast<const int*>(zq) + 4 * lane;    // null steps load here
        // issue side: pass ip, row ordinal iq, next step ia, the row's stream end
        int ip = 0, iq = 0, ia = 0, iend = 0, ilow = 0, iup = 0;
        bool irow = false, ifirst = false;
        int pending = 0;  // non-null steps in the ring
        // the ring: a step's start, row bounds and packed (row | pass << 8 |
        // first << 16 | last << 17), -1 for a null step; its columns in registers
        int ma[D], mlo[D], mup[D], mk[D];
        v4i rg[D][2];
        // process side: the pass the multiply waves wait for; (row, pass) of the
        // last step and its bounds / bit rows; the row's spill flag and first
        // entry past pass p + 1
        int cp = 0, estar = kSpNone;
        int pk = -1, plo = 0, phi = 0, phq = 0;
        uint32_t *pbp = sp_lds, *pbq = sp_lds;
        bool bnd = false, bad = false;
#define LDS_SP_ISSUE(J)                                                                                      \
    do {                                                                                                     \
        int a_ = -1, lo_ = 0, up_ = 0, k_ = -1;                                                              \
        while (ip < passes) {                                                                                \
            if (!irow) {                                                                                     \
                if (iq >= nrw) {                                                                             \
                    ++ip;                                                                                    \
                    iq = 0;                                                                                  \
                    continue;                                                                                \
                }                                                                                            \
                const int lr_ = wave + kSpStream * iq;                                                       \
                /* this row's previous pass not yet processed (the process side runs D - 1 steps behind): */ \
                /* a null step */                                                                            \
                if (__builtin_amdgcn_readfirstlane(fin[lr_]) < ip - 1) break;                                \
                ilow = __builtin_amdgcn_readfirstlane(pos[lr_]);                                             \
                iup = __builtin_amdgcn_readfirstlane(rend[lr_]);                                             \
                if (ilow >= iup) { /* the row is done: closed for this pass too */                          \
                    fin[lr_] = ip;                                                                           \
                    ++iq;                                                                                    \
                    continue;                                                                                \
                }                                                                                            \
                ia = ilow & ~3;                                                                              \
                if (ip == passes - 1) {                                                                      \
                    iend = iup;                                                                              \
                } else {                                                                                     \
                    const int lo0_ = ip * span, hi0_ = min(lo0_ + span, n);                                  \
                    const float fr_ = (float)(hi0_ - lo0_) / (float)(n - lo0_);                              \
                    iend = min(iup, ilow + (int)((float)(iup - ilow) * fr_) + kSpMargin);                    \
                }                                                                                            \
                irow = true;                                                                                 \
                ifirst = true;                                                                               \
            }                                                                                                \
            const bool last_ = ia + kStep >= iend;                                                           \
            a_ = ia;                                                                                         \
            lo_ = ilow;                                                                                      \
            up_ = iup;                                                                                       \
            k_ = (wave + kSpStream * iq) | (ip << 8) | (ifirst ? 1 << 16 : 0) | (last_ ? 1 << 17 : 0);      \
            ia += kStep;                                                                                     \
            ifirst = false;                                                                                  \
            if (last_) {                                                                                     \
                irow = false;                                                                                \
                ++iq;                                                                                        \
            }                                                                                                \
            break;                                                                                           \
        }                                                                                                    \
        ma[J] = a_;                                                                                          \
        mlo[J] = lo_;                                                                                        \
        mup[J] = up_;                                                                                        \
        mk[J] = k_;                                                                                          \
        pending += k_ >= 0 ? 1 : 0;                                                                          \
        _Pragma("unroll") for (int h_ = 0; h_ < 2; ++h_) {                                                   \
            const int aa_ = a_ + kSpE * lane + 4 * h_;                                                       \
            const int* src_ = (a_ >= 0 && aa_ + 4 <= nnz) ? col + aa_ : dummy;                               \
            rb_gload(rg[J][h_], reinterpret_cast<const v4i*>(src_));                                         \
        }                                                                                                    \
    } while (0)
#define LDS_SP_PROCESS(J)                                                                                    \
    do {                                                                                                     \
        /* slot J's step landed: every iteration issues exactly two loads, so D - 1 younger steps stay */    \
        /* in flight (the rare paths' plain loads are waited for where they are used: stricter) */           \
        __builtin_amdgcn_s_waitcnt(0x0F70 | ((D - 1) * 2));                                                  \
        asm volatile("" ::: "memory");                                                                       \
        const int k_ = mk[J];                                                                                \
        if (k_ >= 0) {                                                                                       \
            --pending;                                                                                       \
            const int lr_ = k_ & 0xFF, p_ = (k_ >> 8) & 0xFF;                                                \
            for (; cp < p_; ++cp) { /* pass cp streamed: the multiply waves take it */                      \
                __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0): this wave's bit ORs are done */           \
                __builtin_amdgcn_s_barrier();                                                                \
            }                                                                                                \
            if (k_ & (1 << 16)) {                                                                            \
                bnd = false;                                                                                 \
                estar = kSpNone;                                                                             \
            }                                                                                                \
            if ((k_ & 0xFFFF) != pk) { /* a new (row, pass): its bounds and bit rows */                     \
                pk = k_ & 0xFFFF;                                                                            \
                plo = p_ * span;                                                                             \
                phi = min(plo + span, n);                                                                    \
                phq = min(phi + span, n);                                                                    \
                pbp = sp_lds + (p_ % 3) * bufdw + lr_ * rowdw;                                               \
                pbq = sp_lds + ((p_ + 1) % 3) * bufdw + lr_ * rowdw;                                         \
            }                                                                                                \
            const int lo_ = plo, hi_ = phi, hq_ = phq;                                                       \
            uint32_t* const bp_ = pbp;                                                                       \
            uint32_t* const bq_ = pbq;                                                                       \
            const int a_ = ma[J], rlo_ = mlo[J], rup_ = mup[J];                                              \
            rb_bind(rg[J][0], rg[J][1]);                                                                     \
            const int c_[kSpE] = {rg[J][0][0], rg[J][0][1], rg[J][0][2], rg[J][0][3],                        \
                                  rg[J][1][0], rg[J][1][1], rg[J][1][2], rg[J][1][3]};                       \
            const int i0_ = a_ + kSpE * lane;                                                                \
            bool spill_ = false, fast_ = false;                                                              \
            int myx_ = kSpNone;                                                                              \
            if (a_ >= rlo_ && a_ + kStep <= rup_) { /* interior (uniform): every entry is the row's */       \
                const uint32_t w0_ = (uint32_t)(c_[0] - lo_) >> 5;                                           \
                const int base_ = lo_ + (int)(w0_ << 5);                                                     \
                uint32_t r_[kSpE];                                                                           \
                if constexpr (kCheck) { /* all eight in [base, base + 64) and below the pass end */         \
                    const uint32_t o_ = sp_offsets(c_, base_, r_);                                           \
                    fast_ = c_[0] >= lo_ && o_ < 64u && base_ + (int)o_ < hi_;                               \
                } else { /* ascending: the first and the last bound the lane */                              \
                    _Pragma("unroll") for (int e = 0; e < kSpE; ++e) r_[e] = (uint32_t)(c_[e] - base_);      \
                    fast_ = c_[0] >= lo_ && c_[kSpE - 1] < hi_ && r_[kSpE - 1] < 64u;                        \
                }                                                                                            \
                if (fast_) {                                                                                 \
                    uint64_t m_ = 0;                                                                         \
                    _Pragma("unroll") for (int e = 0; e < kSpE; ++e) m_ |= 1ull << r_[e];                    \
                    dn_or(bp_ + w0_, (uint32_t)m_);                                                          \
                    dn_or(bp_ + w0_ + 1, (uint32_t)(m_ >> 32));                                              \
                }                                                                                            \
                /* (two ifs, not if / else: the compiler then keeps the fast path first and */              \
                /* waits for the ring as it did in round 4; with an else it laid the slow paths */           \
                /* first and waited vmcnt(1) on the fast path, 192 against 164 µs at config 5) */            \
                if (!fast_) {                                                                                \
                    /* all of pass p + 1 (steps streamed past the boundary) */                               \
                    const uint32_t q0_ = (uint32_t)(c_[0] - hi_) >> 5;                                       \
                    const int qbase_ = hi_ + (int)(q0_ << 5);                                                \
                    uint32_t rq_[kSpE];                                                                      \
                    bool pq_;                                                                                \
                    if constexpr (kCheck) {                                                                  \
                        const uint32_t oq_ = sp_offsets(c_, qbase_, rq_);                                    \
                        pq_ = c_[0] >= hi_ && oq_ < 64u && qbase_ + (int)oq_ < hq_;                          \
                    } else {                                                                                 \
                        _Pragma("unroll") for (int e = 0; e < kSpE; ++e) rq_[e] = (uint32_t)(c_[e] - qbase_); \
                        pq_ = c_[0] >= hi_ && c_[kSpE - 1] < hq_ && rq_[kSpE - 1] < 64u;                     \
                    }                                                                                        \
                    if (pq_) {                                                                               \
                        uint64_t m_ = 0;                                                                     \
                        _Pragma("unroll") for (int e = 0; e < kSpE; ++e) m_ |= 1ull << rq_[e];               \
                        dn_or(bq_ + q0_, (uint32_t)m_);                                                      \
                        dn_or(bq_ + q0_ + 1, (uint32_t)(m_ >> 32));                                          \
                        spill_ = true;                                                                       \
                        fast_ = true;                                                                        \
                    } else if (c_[0] >= lo_ && c_[0] < hi_ && c_[kSpE - 1] >= hi_ && c_[kSpE - 1] < hq_ &&    \
                               (uint32_t)(c_[kSpE - 1] - hi_) < 64u) { /* straddles the boundary */          \
                        uint64_t mp_ = 0, mq_ = 0;                                                           \
                        bool ok_ = true;                                                                     \
                        _Pragma("unroll") for (int e = 0; e < kSpE; ++e) {                                   \
                            /* every entry checked: pass p's in this lane's window, pass p + 1's in */       \
                            /* its first 64 columns */                                                       \
                            const bool in_ = c_[e] < hi_;                                                    \
                            const uint32_t rr_ = in_ ? (uint32_t)(c_[e] - lo_) - (w0_ << 5) : (uint32_t)(c_[e] - hi_); \
                            ok_ = ok_ && rr_ < 64u;                                                          \
                            const uint64_t b_ = 1ull << (rr_ & 63u);                                         \
                            mp_ |= in_ ? b_ : 0ull;                                                          \
                            mq_ |= in_ ? 0ull : b_;                                                          \
                        }                                                                                    \
                        if (ok_) {                                                                           \
                            dn_or(bp_ + w0_, (uint32_t)mp_);                                                 \
                            dn_or(bp_ + w0_ + 1, (uint32_t)(mp_ >> 32));                                     \
                            dn_or(bq_, (uint32_t)mq_);                                                       \
                            dn_or(bq_ + 1, (uint32_t)(mq_ >> 32));                                           \
                            spill_ = true;                                                                   \
                            fast_ = true;                                                                    \
                        }                                                                                    \
                    }                                                                                        \
                }                                                                                            \
            }                                                                                                \
            if (!fast_) {                                                                                    \
                /* per entry; two copies under a uniform branch: only the array's last step reloads the */   \
                /* lanes that read the dummy (a lane-conditional load costs vmcnt(0) on every path) */       \
                if (a_ + kStep > nnz) {                                                                      \
                    _Pragma("unroll") for (int e = 0; e < kSpE; ++e) {                                       \
                        const int idx_ = i0_ + e;                                                            \
                        if (idx_ >= rlo_ && idx_ < rup_ &&                                                   \
                            sp_put((idx_ & ~3) + 4 > nnz ? sp_ld(col + idx_) : c_[e], lo_, hi_, hq_, bp_, bq_, spill_, bad)) \
                            myx_ = min(myx_, idx_);                                                          \
                    }                                                                                        \
                } else {                                                                                     \
                    _Pragma("unroll") for (int e = 0; e < kSpE; ++e) {                                       \
                        const int idx_ = i0_ + e;                                                            \
                        if (idx_ >= rlo_ && idx_ < rup_ && sp_put(c_[e], lo_, hi_, hq_, bp_, bq_, spill_, bad)) \
                            myx_ = min(myx_, idx_);                                                          \
                    }                                                                                        \
                }                                                                                            \
            }                                                                                                \
            if (__ballot(spill_) != 0ull) bnd = true;                                                        \
            const uint64_t xm_ = __ballot(myx_ != kSpNone);                                                  \
            if (xm_ != 0ull) estar = min(estar, __builtin_amdgcn_readlane(myx_, __builtin_ctzll(xm_)));      \
            if (k_ & (1 << 17)) { /* the row's last issued step: where pass p + 1 starts */                 \
                int np_ = min(a_ + kStep, rup_);                                                             \
                if (estar == kSpNone && !bnd && np_ < rup_) {                                                \
                    /* the boundary lies past the predicted end: finish the row with blocking loads */       \
                    while (np_ < rup_) {                                                                     \
                        const int b_ = (np_ & ~3) + 4 * lane;                                                \
                        bool sp2_ = false;                                                                   \
                        int mx2_ = kSpNone;                                                                  \
                        _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                      \
                            const int idx_ = b_ + e;                                                         \
                            if (idx_ >= np_ && idx_ < rup_ && sp_put(sp_ld(col + idx_), lo_, hi_, hq_, bp_, bq_, sp2_, bad)) \
                                mx2_ = min(mx2_, idx_);                                                      \
                        }                                                                                    \
                        np_ = min((np_ & ~3) + 256, rup_);                                                   \
                        const uint64_t xm2_ = __ballot(mx2_ != kSpNone);                                     \
                        if (xm2_ != 0ull) estar = min(estar, __builtin_amdgcn_readlane(mx2_, __builtin_ctzll(xm2_))); \
                        if (__ballot(sp2_) != 0ull) break;                                                   \
                    }                                                                                        \
                }                                                                                            \
                if (estar != kSpNone) {                                                                      \
                    np_ = estar;                                                                             \
                    if (p_ == passes - 1) bad = true; /* a column at or past n */                            \
                }                                                                                            \
                if (lane == 0) {                                                                             \
                    pos[lr_] = np_;                                                                          \
                    fin[lr_] = p_;                                                                           \
                }                                                                                            \
            }                                                                                                \
        }                                                                                                    \
    } while (0)
        // every plain load of the prologue has landed before the ring starts: the
        // compiler's wait analysis does not see the ring's asm loads, so a
        // prologue load still counted as outstanding would make it wait (vmcnt
        // 1-2) wherever the ring later reuses that load's registers
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#pragma unroll
        for (int j = 0; j < D - 1; ++j) LDS_SP_ISSUE(j);
        while (true) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                LDS_SP_ISSUE((j + D - 1) % D);
                LDS_SP_PROCESS(j);
                if (ip >= passes && pending == 0) goto streamed;
            }
        }
#undef LDS_SP_PROCESS
#undef LDS_SP_ISSUE
    streamed:
        for (; cp < passes; ++cp) {  // the last pass (and passes without steps of this wave)
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_s_barrier();
        }
        if constexpr (kCheck)
            if (__ballot(bad) != 0ull && lane == 0) atomicOr(err, kDevErrCsrColumns);
    } else {
        // ---- multiply waves --------------------------------------------------
        // wave 12 + m: limb m, both k-halves of every chunk of the pass
        const int L = wave - kSpStream;
        const int r16 = lane & 15, g = lane >> 4;
        const v4i* const zv = reinterpret_cast<const v4i*>(zq) + L * 64 + lane;
        const int ntiles = (nrows + 15) / 16;
#define LDS_SP_DIG(CH, HH, DQ)                                                                 \
    do {                                                                                       \
        const v4i* z_ = zv + (int64_t)(CH) * (kChunkBytes / 16) + 4 * (HH) * kLimbs * 64;      \
        _Pragma("unroll") for (int i = 0; i < 4; ++i) DQ[i] = z_[i * kLimbs * 64];             \
    } while (0)
#define LDS_SP_MUL(CC, HH, DQ)                                                                                  \
    do {                                                                                                      \
        _Pragma("unroll") for (int T = 0; T < kTiles; ++T) {                                                  \
            if (T < ntiles) {                                                                                 \
                const uint2 w_ = *reinterpret_cast<const uint2*>(bp + (16 * T + r16) * rowdw + (CC) * 16 + 4 * g + 2 * (HH)); \
                _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                               \
                    const uint32_t w = (i >> 1) ? w_.y : w_.x;                                                \
                    const int sh = 4 * (i & 1);                                                               \
                    v4i a;                                                                                    \
                    a.x = (int)((w >> sh) & 0x01010101u);                                                     \
                    a.y = (int)((w >> (sh + 1)) & 0x01010101u);                                               \
                    a.z = (int)((w >> (sh + 2)) & 0x01010101u);                                               \
                    a.w = (int)((w >> (sh + 3)) & 0x01010101u);                                               \
                    acc[T] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, DQ[i], acc[T], 0, 0, 0);                \
                }                                                                                             \
            }                                                                                                 \
        }                                                                                                     \
    } while (0)
        for (int p = 0; p < passes; ++p) {
            const int c0 = p * cpp, cn = min(cpp, chunks - c0);
            v4i da[4], db[4];
            // units u = (chunk u / 2, half u % 2)
            const int un = cn * 2;
            LDS_SP_DIG(c0, 0, da);  // before the barrier: in flight while pass p finishes streaming
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_s_barrier();  // pass p streamed
            const uint32_t* const bp = sp_lds + (p % 3) * bufdw;
            for (int u = 0; u < un; u += 2) {
                if (u + 1 < un) LDS_SP_DIG(c0 + (u + 1) / 2, (u + 1) % 2, db);
                LDS_SP_MUL(u / 2, u % 2, da);
                if (u + 1 >= un) break;
                if (u + 2 < un) LDS_SP_DIG(c0 + (u + 2) / 2, (u + 2) % 2, da);
                LDS_SP_MUL((u + 1) / 2, (u + 1) % 2, db);
            }
            // pass p done: the last multiply wave to finish with its buffer clears it
            // for pass p + 3 (whose spills start in pass p + 2, after the next barrier);
            // clearing it from every wave raced with the slower waves' reads
            __builtin_amdgcn_s_waitcnt(0xC07F);  // this wave's fragment reads of the buffer returned
            const int order = __builtin_amdgcn_readfirstlane(lane == 0 ? atomicAdd(done + p % 3, 1) : 0);
            if (order == kSpMul - 1) {
                uint4* const bz = reinterpret_cast<uint4*>(sp_lds + (p % 3) * bufdw);
                for (int i = lane; i < bufdw / 4; i += 64) bz[i] = make_uint4(0u, 0u, 0u, 0u);
                if (lane == 0) done[p % 3] = 0;
            }
        }
#undef LDS_SP_MUL
#undef LDS_SP_DIG
    }
    __syncthreads();  // every pass multiplied
    unsigned long long* const sums = reinterpret_cast<unsigned long long*>(sp_lds);  // [rowsL][16]
    for (int i = t; i < rowsL * kF; i += kSpThreads) sums[i] = 0ull;
    __syncthreads();
    if (wave >= kSpStream) {
        const int L = wave - kSpStream;
        const int r16 = lane & 15, g = lane >> 4;
#pragma unroll
        for (int T = 0; T < kTiles; ++T)
            if (16 * T < nrows)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    atomicAdd(sums + (T * 16 + 4 * g + i) * kF + r16,
                              (unsigned long long)((int64_t)acc[T][i] * ((int64_t)1 << (8 * L))));
    }
    __syncthreads();
    for (int o = t; o < nrows * kF; o += kSpThreads) {
        const int lr = o >> 4, f = o & 15;
        const int row = r0 + lr;
        const float r = s[row] * (float)ldexp((double)(int64_t)sums[o], -e_sh[f]);
        float* out = y + (int64_t)row * ldy + f;
        *out = beta ? *out + r : r;
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
    int g = grid > 0 ? grid : device_cus();
    const int gmin = (n + kSpMaxRows - 1) / kSpMaxRows;  // at most kSpMaxRows rows per workgroup
    if (g < gmin) g = gmin;
    if (g > kSpMaxGrid) g = kSpMaxGrid;
    const int R = (n + g - 1) / g;
    LDS_CHECK_ARG(R <= kSpMaxRows);
    g = (n + R - 1) / R;  // every workgroup has rows
    const int tiles = (R + 15) / 16;
    const SpGeom sg = sp_geom(nc, tiles);
    const int lds = sp_lds_bytes(tiles, sg);
    LDS_CHECK_ARG(lds <= 163840 && sg.passes <= 255);  // (the pass is an 8-bit field of a ring record)
#define LDS_SP_LAUNCH1(TT, CK)                                                                                 \
    do {                                                                                                       \
        const hipError_t e = allow_lds(&csr_spill_agg_kernel<TT, CK>, lds);                                    \
        if (e != hipSuccess) return (int)e;                                                                    \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(csr_spill_agg_kernel<TT, CK>), dim3(g), dim3(kSpThreads), lds, st, row_ptr, \
                           col, n, R, (const int8_t*)w.zq, nc, sg.cpp, sg.passes, sg.rowdw,                    \
                           (const uint32_t*)w.colmax, s, y, ldy, beta, err);                                   \
    } while (0)
    // (5 tiles run the 6-tile build: 170-171 µs at config 5 against 175-178 for a 5-tile build of the same code)
#define LDS_SP_LAUNCH(TT)                    \
    do {                                     \
        if (err != nullptr)                  \
            LDS_SP_LAUNCH1(TT, true);        \
        else                                 \
            LDS_SP_LAUNCH1(TT, false);       \
    } while (0)
    if (tiles <= 2) LDS_SP_LAUNCH(2);
    else if (tiles <= 4) LDS_SP_LAUNCH(4);
    else LDS_SP_LAUNCH(6);
#undef LDS_SP_LAUNCH
#undef LDS_SP_LAUNCH1
    LDS_RETURN_LAST_ERROR();
}
