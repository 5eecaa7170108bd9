// Tools-only library: every non-product form of the dense-graph CSR-SpMM
// (lds_spmm_norm_dense) that rounds 3-4 measured, kept for the ablation and
// diagnosis tools (tools/spmm_config5.py, tools/diag/spill_diag.py) and the
// variants test (tests/test_spmm_variants_gpu.py).  NOT part of the product
// library: several codes are timing-only ablations that return wrong results.
//
// The forms: the row-block kernel (bit rows through a
// global slab, any column order), the column-pass kernel (ascending columns),
// and the spill-pass kernel in every configuration that led to the product
// (the product itself, mode 17, lives in lds-gnn_amd/csrc/bitagg.hip).  The
// code is the round-4 source, unchanged, in its own namespace; it reads the
// digits of s⊙Z an earlier lds_spmm_norm_dense call left in the workspace.
//
// Build: make -C tools/variants  ->  tools/variants/libldsgnn_variants.so
#include "../../lds-gnn_amd/csrc/bitagg.hpp"
#include "../../lds-gnn_amd/csrc/spill.hpp"  // the product kernel, for its delayed test build

namespace lds_variants {
using namespace lds;

// ---------------------------------------------------------------------------
// CSR-SpMM for dense sampled graphs, row-block form (round 4; the product
// of lds_spmm_norm_dense until the spill-pass kernel replaced it).  csr_dense_agg_kernel above multiplies each
// 16-row bit tile as soon as it is streamed, so every tile reads all of s⊙Z's
// digits (1.3 MB at N = 20 000) from L2: 1.6 GB per call, twice the index
// stream, on the same CUs — and the two streams serialise (its ablations:
// 140 µs streaming alone, 71 µs MFMA alone, 230 µs together).  Here each
// workgroup owns ONE contiguous block of rows (R = ceil(n / grid), at most
// kRbMaxTiles·16) and runs two phases:
//  A. all 16 waves stream the block's CSR rows (wave w: local rows w, w + 16,
//     …) through per-wave rings of 1-KB LDS-DMA units (512-entry steps, two
//     in flight behind the one being read, across rows), set each entry's bit
//     in a per-wave LDS row buffer (one 64-bit mask and two LDS ORs per lane
//     for 8 entries within 64 columns, a per-entry path otherwise) and, at the
//     row's end, write the bit row to a workgroup-private scratch slab
//     (global, L2-resident: R rows × n bits) and clear the buffer;
//  B. the block's rows multiply s⊙Z's digits once: per 512-column chunk the
//     digits (32 KB) and the block's bit rows of the chunk (64 B per row) are
//     staged in LDS by direct global -> LDS loads, three chunks in flight;
//     wave w runs limb w & 3, k-steps 2(w >> 2), +1 of the chunk for every
//     row tile (lds_aggregate_bitmask's digits, k order and exact int32
//     sums); the 16 waves' sums meet in LDS as int64 adds (exact, order-free),
//     then y = s_i · 2^-e_f · Σ.
// Per CU the digits are read once per call (1.3 MB from L2), not once per
// 16-row tile.  Columns must be distinct within a row; order is free.
// ---------------------------------------------------------------------------
constexpr int kRbWaves = 16;
constexpr int kRbThreads = 64 * kRbWaves;
constexpr int kRbUnits = 6;                  // 1-KB ring units per wave: three 512-entry steps
constexpr int kRbRing = kRbUnits / 2;        // steps in a wave's ring
constexpr int kRbMaxTiles = 6;               // 16-row tiles per workgroup (R <= 96)
constexpr int kRbStages = 3;                 // phase-B chunk stages in flight
constexpr int kRbAhead = 4;                  // column-pass multiply waves: digit chunks in flight (registers)
constexpr int kRbMaxGrid = 512;

// Scratch rows of the bit slabs for any grid <= kRbMaxGrid: G·T·16 <= n + 17·G.
int64_t rb_scratch_rows(int n) { return (int64_t)n + 17 * kRbMaxGrid; }
__host__ __device__ constexpr int rb_stage_bytes(int tiles) { return kChunkBytes + tiles * 1024; }
int rb_lds_bytes(int chunks, int tiles) {
    const int a = kRbWaves * kRbUnits * 1024 + kRbWaves * 64 * chunks;      // phase A: rings + row buffers
    const int b = kRbStages * rb_stage_bytes(tiles) + tiles * 16 * kF * 8;  // phase B: stages + int64 sums
    return a > b ? a : b;
}

// Phase B's digit loads, issued from asm: the compiler's own waits for loads
// carried around the chunk loop came out as vmcnt(0) on the chunk just issued
// (no prefetch at all); the kernel counts these with its bit DMAs and waits
// itself, and rb_bind ties the registers to that wait (nothing reads them
// earlier).
__device__ __forceinline__ void rb_gload(v4i& v, const v4i* p) {
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
}
__device__ __forceinline__ void rb_bind(v4i& a, v4i& b) { asm volatile("" : "+v"(a), "+v"(b)); }

// A wave's position in its CSR stream (wave-uniform): its k-th row (local row
// wave + 16k of the block), entries [p, p + 512) of [beg, end), p ≡ 0 mod 4;
// k == kend: past the last.
struct RbStep {
    int k, beg, end, p;
};
__device__ __forceinline__ void rb_advance(RbStep& s, const int* __restrict__ rp, int r0, int nrows, int kend,
                                           int wave) {
    if (s.k >= 0) {
        s.p += kDnStep;
        if (s.p < s.end) return;
    }
    while (true) {
        if (++s.k >= kend) {
            s.k = kend;
            return;
        }
        const int row = r0 + wave + 16 * s.k;
        s.beg = __builtin_amdgcn_readfirstlane(rp[row]);
        s.end = __builtin_amdgcn_readfirstlane(rp[row + 1]);
        s.p = s.beg & ~3;
        if (s.beg < s.end) return;
    }
}

// DBG (timing-only ablations, wrong results): 1 phase A only, 2 phase A without
// the slab stores, 3 phase B only, 4 phase B without the bit-row loads.  The
// product path is DBG = 0.
template <int kTiles, int DBG = 0>
__global__ __launch_bounds__(kRbThreads, 1) void csr_rowblock_agg_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, int n, int rows_per_wg, const int8_t* __restrict__ zq,
    int chunks, const uint32_t* __restrict__ colmax, const float* __restrict__ s, float* __restrict__ y, int ldy,
    int beta, uint32_t* __restrict__ slab_all) {
    extern __shared__ __attribute__((aligned(16))) uint32_t rb_lds[];
    __shared__ int e_sh[kF];
    const int rs = 16 * chunks;  // dwords per bit row
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int r0 = (int)blockIdx.x * rows_per_wg;
    const int nrows = min(rows_per_wg, n - r0);
    if (nrows <= 0) return;  // (uniform: the whole workgroup)
    const int nnz = rp[n];
    const int tiles = (rows_per_wg + 15) / 16;  // (the last block may use fewer)
    uint32_t* const slab = slab_all + (int64_t)blockIdx.x * (tiles * 16) * rs;  // this block's bit rows
    if (t < 64) {  // per-feature exponents (lds_aggregate_bitmask's quantisation)
        const uint32_t m = colmax_of(colmax, t);
        if (t < kF) e_sh[t] = col_exponent(m);
    }

    // ---- phase A: stream the block's rows into bit rows --------------------
    uint32_t* const rowbuf = rb_lds + kRbWaves * kRbUnits * 256 + wave * rs;
    for (int d = 4 * lane; d < rs; d += 256) *reinterpret_cast<uint4*>(rowbuf + d) = make_uint4(0u, 0u, 0u, 0u);
    const int kend = nrows > wave ? (nrows - 1 - wave) / 16 + 1 : 0;  // this wave's rows
    const uint32_t ring_lds = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint32_t*)rb_lds) +
                              (uint32_t)(wave * kRbUnits * 1024);
    const uint32_t* myring = rb_lds + wave * kRbUnits * 256;
    RbStep is{-1, 0, 0, 0}, ps{-1, 0, 0, 0};
    int kis = 0, kps = 0, cur = 0;  // steps issued / processed; next row to write out
    // vector-memory ops this wave issued (loads and stores count together, in
    // order) and the count after each in-flight step's loads, oldest first:
    // waiting for the oldest step is vmcnt(ops - q0), so the bit-row stores of
    // a flush do not hold up the next step's wait
    int ops = 0, q0 = 0, q1 = 0, q2 = 0;
    const int row_stores = DBG == 2 || DBG == 5 ? 0 : (rs + 255) / 256;  // store instructions per bit row
    rb_advance(is, rp, r0, nrows, kend, wave);
    ps = is;
    while (DBG != 3 && DBG != 4 && DBG != 7 && DBG != 8) {
        // fill the ring: up to kRbRing steps in flight, the one read next included
        while (is.k < kend && kis - kps < kRbRing) {
            const uint32_t unit = (uint32_t)(2 * (kis % kRbRing));
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int a = is.p + 256 * h + 4 * lane;
                const int* src = a + 4 <= nnz ? col + a : col;  // past the array: a dummy block (reloaded below)
                lds_dma16(src, ring_lds + (unit + h) * 1024u);
            }
            ops += 2;
            const int inflight = kis - kps;
            q0 = inflight == 0 ? ops : q0;
            q1 = inflight == 1 ? ops : q1;
            q2 = inflight == 2 ? ops : q2;
            ++kis;
            rb_advance(is, rp, r0, nrows, kend, wave);
        }
        if (ps.k >= kend) break;
        wait_vmcnt(ops - q0);  // step kps landed; every op issued after its loads may stay in flight
        asm volatile("" ::: "memory");
        // a new row: write the wave's bit rows cur .. ps.k - 1 to the slab (the
        // buffer holds row cur's bits, the rows between are empty) and clear it
        for (; cur < ps.k; ++cur) {
            uint32_t* dst = slab + (int64_t)(wave + 16 * cur) * rs;
            for (int d = 4 * lane; d < rs; d += 256) {
                uint4* b = reinterpret_cast<uint4*>(rowbuf + d);
                // plain stores: the multiply phase reads the slab back through L2
                // (nontemporal stores measured 291 against 223 µs per call)
                if (DBG != 2 && DBG != 5) *reinterpret_cast<uint4*>(dst + d) = *b;
                *b = make_uint4(0u, 0u, 0u, 0u);
            }
            ops += row_stores;
        }
        const uint32_t* sl = myring + (2 * (kps % kRbRing)) * 256 + 8 * lane;
        const int4 c0 = *reinterpret_cast<const int4*>(sl);
        const int4 c1 = *reinterpret_cast<const int4*>(sl + 4);
        const int c[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        const int p = ps.p + 8 * lane;
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
                dn_or(rowbuf + wf, (uint32_t)m);
                dn_or(rowbuf + wf + 1, (uint32_t)(m >> 32));
                done = true;
            }
        }
        if (!done) {
            // the per-entry path (row ends, sparse rows, unsorted columns); entries
            // in a dummy block past the array's end are reloaded — only in the
            // array's last step (wave-uniform), so no other step waits on a load
            // (two copies of the loop: a load under a lane condition makes the
            // compiler wait vmcnt(0) at the join whether or not it was taken)
            if (ps.p + kDnStep + 4 > nnz) {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const int idx = p + e;
                    if (idx >= ps.beg && idx < ps.end) {
                        const int v = (idx & ~3) + 4 > nnz ? col[idx] : c[e];
                        atomicOr(rowbuf + (v >> 5), 1u << (v & 31));
                    }
                }
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const int idx = p + e;
                    if (idx >= ps.beg && idx < ps.end) atomicOr(rowbuf + (c[e] >> 5), 1u << (c[e] & 31));
                }
            }
        }
        if constexpr (DBG == 5) {  // ablation: the column-pass kernel's per-step bookkeeping, no effect
            __shared__ int dbg_state[16];
            int myx = 0x7FFFFFFF;
#pragma unroll
            for (int e = 7; e >= 0; --e)
                if (p + e >= ps.beg && p + e < ps.end && c[e] >= n) myx = p + e;
            const int st = __builtin_amdgcn_readfirstlane(dbg_state[wave]);
            const uint64_t hit = __ballot(myx != 0x7FFFFFFF);
            const int nx = hit != 0ull ? __builtin_amdgcn_readlane(myx, __builtin_ctzll(hit)) : st + 1;
            if (lane == 0) dbg_state[wave] = nx;
        }
        ++kps;
        q0 = q1;
        q1 = q2;
        rb_advance(ps, rp, r0, nrows, kend, wave);
    }
    if (DBG != 3 && DBG != 4 && DBG != 7 && DBG != 8) {  // the wave's last bit row(s)
        for (; cur < kend; ++cur) {
            uint32_t* dst = slab + (int64_t)(wave + 16 * cur) * rs;
            for (int d = 4 * lane; d < rs; d += 256) {
                uint4* b = reinterpret_cast<uint4*>(rowbuf + d);
                if (DBG != 2 && DBG != 5) *reinterpret_cast<uint4*>(dst + d) = *b;
                *b = make_uint4(0u, 0u, 0u, 0u);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the slab rows are written before any wave stages them
    __syncthreads();
    if constexpr (DBG == 1 || DBG == 2 || DBG == 5) return;

    if constexpr (DBG == 6 || DBG == 7 || DBG == 8) {
        // ---- phase B, hybrid staging (DBG 6; 7: phase B alone) ---------------
        // digits straight into registers, S chunks ahead (each wave its limb's
        // two k-steps: register loads from L2 run ~3.5x the LDS-DMA rate per
        // CU here); the block's bit-row segments of a chunk (64 B per row) by
        // LDS-DMA, wave T < tiles one 1-KB block (row tile T) per chunk, S
        // chunks in flight; one barrier per chunk.  Same chunks, k order and
        // exact sums as the staged form.
        constexpr int S = 4;
        const int L = wave & 3, pm = wave >> 2;
        const int r16 = lane & 15, g = lane >> 4;
        const int rot = (int)(blockIdx.x % (unsigned)chunks);
        unsigned long long* const sums = reinterpret_cast<unsigned long long*>(rb_lds + S * kTiles * 256);
        for (int i = t; i < kTiles * 16 * kF; i += kRbThreads) sums[i] = 0ull;
        const uint32_t stage_lds = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint32_t*)rb_lds);
        const v4i* const zv = reinterpret_cast<const v4i*>(zq) + (2 * pm * kLimbs + L) * 64 + lane;
        const bool loader = wave < tiles;
        const uint32_t* const sseg = slab + (int64_t)(16 * (loader ? wave : 0) + (lane >> 2)) * rs + 4 * (lane & 3);
        int ops = 0;  // this wave's vector-memory operations, in issue order
        int qa[S];    // ops right after the loads of the chunk in slot s (its bit DMA, then its digits)
        v4i bq[S][2];
        v4i acc[kTiles];
#pragma unroll
        for (int T = 0; T < kTiles; ++T) acc[T] = v4i{0, 0, 0, 0};
#define LDS_RB_ISSUE(CH, SL)                                                                      \
    do {                                                                                          \
        const int cc_ = (CH) + rot < chunks ? (CH) + rot : (CH) + rot - chunks;                   \
        if (loader) {                                                                             \
            lds_dma16(sseg + 16 * cc_, stage_lds + (uint32_t)(((SL) * kTiles + wave) * 1024));    \
            ++ops;                                                                                \
        }                                                                                         \
        const v4i* z_ = zv + (int64_t)cc_ * (kChunkBytes / 16);                                   \
        rb_gload(bq[SL][0], z_);                                                                  \
        rb_gload(bq[SL][1], z_ + kLimbs * 64);                                                    \
        ops += 2;                                                                                 \
        qa[SL] = ops;                                                                             \
    } while (0)
#pragma unroll
        for (int c = 0; c < S - 1; ++c)
            if (c < chunks) LDS_RB_ISSUE(c, c);
        for (int c0 = 0; c0 < chunks; c0 += S) {
#pragma unroll
            for (int d = 0; d < S; ++d) {
                const int c = c0 + d;
                if (c < chunks) {  // (uniform)
                    // this wave's loads of chunk c landed (its digits, and its bit
                    // block, issued before them), then every wave's bit blocks
                    // (barrier), and every wave is done with chunk c - 1's slot
                    wait_vmcnt(ops - qa[d]);
                    rb_bind(bq[d][0], bq[d][1]);
                    asm volatile("" ::: "memory");
                    if (DBG != 8) __builtin_amdgcn_s_barrier();  // (8: timing only, no barrier)
                    asm volatile("" ::: "memory");
                    if (c + S - 1 < chunks) LDS_RB_ISSUE(c + S - 1, (d + S - 1) % S);
                    // every tile slot is read and multiplied (no per-tile guard, so the
                    // reads issue together); slots past `tiles` hold stale bits whose
                    // sums are never stored
                    const uint32_t* const tb = rb_lds + d * kTiles * 256;
                    uint32_t wv[kTiles];
#pragma unroll
                    for (int T = 0; T < kTiles; ++T) wv[T] = tb[T * 256 + r16 * 16 + 4 * g + pm];
#pragma unroll
                    for (int T = 0; T < kTiles; ++T) {
                        const uint32_t w = wv[T];
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const int sh = 4 * h;
                            v4i a;
                            a.x = (int)((w >> sh) & 0x01010101u);
                            a.y = (int)((w >> (sh + 1)) & 0x01010101u);
                            a.z = (int)((w >> (sh + 2)) & 0x01010101u);
                            a.w = (int)((w >> (sh + 3)) & 0x01010101u);
                            acc[T] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bq[d][h], acc[T], 0, 0, 0);
                        }
                    }
                }
            }
        }
#undef LDS_RB_ISSUE
#pragma unroll
        for (int T = 0; T < kTiles; ++T)
            if (T < tiles)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    atomicAdd(sums + (T * 16 + 4 * g + i) * kF + r16,
                              (unsigned long long)((int64_t)acc[T][i] * ((int64_t)1 << (8 * L))));
        __syncthreads();
        for (int o = t; o < nrows * kF; o += kRbThreads) {
            const int lr = o >> 4, f = o & 15;
            const int row = r0 + lr;
            const float r = s[row] * (float)ldexp((double)(int64_t)sums[o], -e_sh[f]);
            float* out = y + (int64_t)row * ldy + f;
            *out = beta ? *out + r : r;
        }
        return;
    }

    // ---- phase B: the block's bit rows × the digits, chunk by chunk --------
    // Per chunk the digits (32 KB) and the block's bit-row segments (64 B per
    // row) are staged by LDS-DMA, three chunks in flight, one barrier per chunk.
    // (Register loads of the slab's A dwords, one 4-byte load per row tile and
    // lane, measured 287-290 against 223 µs per call: 16 lines per load.)
    int8_t* const stage0 = reinterpret_cast<int8_t*>(rb_lds);
    const int sbytes = rb_stage_bytes(kTiles);
    unsigned long long* const sums =
        reinterpret_cast<unsigned long long*>(stage0 + kRbStages * sbytes);  // [kTiles·16][16] int64
    for (int i = t; i < kTiles * 16 * kF; i += kRbThreads) sums[i] = 0ull;
    const uint32_t stage_lds = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint32_t*)rb_lds);
    // chunk c's stage: 32 digit blocks of 1 KB, then `tiles` blocks of the bit
    // rows' 64-byte chunk segments (lane l: row 16T + (l >> 2), 16 bytes l & 3)
    const int nblk = 32 + tiles;
    auto stage = [&](int c, int buf) {
        for (int i = wave; i < nblk; i += kRbWaves) {
            const uint32_t dst = stage_lds + (uint32_t)(buf * sbytes + i * 1024);
            if (i < 32) {
                lds_dma16(zq + (int64_t)c * kChunkBytes + i * 1024 + lane * 16, dst);
            } else {
                const int T = i - 32;
                lds_dma16(slab + (int64_t)(16 * T + (lane >> 2)) * rs + 16 * c + 4 * (lane & 3), dst);
            }
        }
    };
    const int mine = (nblk - 1 - wave) / kRbWaves + 1;  // stage loads this wave issues per chunk (>= 2)
    const int L = wave & 3, pm = wave >> 2;              // limb; k-steps 2pm, 2pm + 1 (dword pm of each group)
    const int r16 = lane & 15, g = lane >> 4;
    v4i acc[kTiles];
#pragma unroll
    for (int T = 0; T < kTiles; ++T) acc[T] = v4i{0, 0, 0, 0};
    for (int c = 0; c < kRbStages - 1 && c < chunks; ++c) stage(c, c);
    for (int c = 0; c < chunks; ++c) {
        // chunk c landed (the younger chunk's loads may stay in flight), and every
        // wave is past chunk c - 1 (whose buffer the next stage call refills)
        if (c + 1 < chunks) {
            if (mine >= 3) __builtin_amdgcn_s_waitcnt(0x0F73);  // vmcnt(3)
            else __builtin_amdgcn_s_waitcnt(0x0F72);            // vmcnt(2)
        } else {
            __builtin_amdgcn_s_waitcnt(0x0F70);
        }
        __syncthreads();
        if (c + kRbStages - 1 < chunks) stage(c + kRbStages - 1, (c + kRbStages - 1) % kRbStages);
        const int8_t* sb = stage0 + (c % kRbStages) * sbytes;
        const v4i* bs = reinterpret_cast<const v4i*>(sb);
        const v4i b0 = bs[((2 * pm) * kLimbs + L) * 64 + lane];
        const v4i b1 = bs[((2 * pm + 1) * kLimbs + L) * 64 + lane];
        const uint32_t* tb = reinterpret_cast<const uint32_t*>(sb + kChunkBytes);
#pragma unroll
        for (int T = 0; T < kTiles; ++T) {
            if (T < tiles) {
                const uint32_t w = DBG == 4 ? 0x01010101u : tb[T * 256 + r16 * 16 + 4 * g + pm];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int sh = 4 * h;
                    v4i a;
                    a.x = (int)((w >> sh) & 0x01010101u);
                    a.y = (int)((w >> (sh + 1)) & 0x01010101u);
                    a.z = (int)((w >> (sh + 2)) & 0x01010101u);
                    a.w = (int)((w >> (sh + 3)) & 0x01010101u);
                    acc[T] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, h ? b1 : b0, acc[T], 0, 0, 0);
                }
            }
        }
    }
    // C/D: col = lane & 15 (feature), row = 4(lane >> 4) + i; limb L weighs 2^(8L)
#pragma unroll
    for (int T = 0; T < kTiles; ++T)
        if (T < tiles)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                atomicAdd(sums + (T * 16 + 4 * g + i) * kF + r16,
                          (unsigned long long)((int64_t)acc[T][i] * ((int64_t)1 << (8 * L))));
    __syncthreads();
    for (int o = t; o < nrows * kF; o += kRbThreads) {
        const int lr = o >> 4, f = o & 15;
        const int row = r0 + lr;
        const float r = s[row] * (float)ldexp((double)(int64_t)sums[o], -e_sh[f]);
        float* out = y + (int64_t)row * ldy + f;
        *out = beta ? *out + r : r;
    }
}

// ---------------------------------------------------------------------------
// CSR-SpMM for dense sampled graphs, column-pass form (round 4, a candidate
// for lds_spmm_norm_dense, never the product).  Each workgroup owns one contiguous block of
// rows (R <= kTiles·16) and sweeps the columns in P passes of cpp 512-column
// chunks, so that the block's bit rows of ONE pass fit in LDS (R × cpp·64 B):
// nothing of size nnz leaves the CU, and each CU reads s⊙Z's digits once.
//  - streaming waves stream the block's CSR rows through per-wave rings of
//    1-KB LDS-DMA units (512-entry steps, three in flight) and set each
//    entry of the pass's column range in the pass's bit buffer.  A row's
//    entries are ascending, so a pass ends for a row at its first entry past
//    the range (the row's position is kept for the next pass; the one step
//    that straddles the boundary is read again there).  A wave interleaves its
//    rows round robin, a step of one row in flight at a time, so every load it
//    issues is one the pass needs;
//  - multiply waves run the pass's chunks: digits straight from L2 into
//    registers kRbAhead chunks ahead, the A operand from the bit buffer
//    (lds_aggregate_bitmask's digits, k order and exact int32 sums).
// kConc: 8 streaming + 8 multiply waves and two bit buffers (pass p is
// multiplied while pass p + 1 streams; one barrier per pass); otherwise all 16
// waves stream, then all 16 multiply (one buffer, two barriers per pass).
// The waves' int32 sums meet as int64 adds in LDS; y = s_i · 2^-e_f · Σ.
// Columns must be ascending within each row (the sampler's CSR).
// ---------------------------------------------------------------------------
constexpr int kCpUnits = 6;                 // 1-KB ring units per streaming wave (three steps)
constexpr int kCpRing = kCpUnits / 2;

__host__ __device__ constexpr int cp_stream_waves(bool conc) { return conc ? 8 : 16; }
int cp_fixed_lds(bool conc) { return cp_stream_waves(conc) * kCpUnits * 1024; }
// LDS bytes of the pass buffers for tiles row tiles and cpp chunks per pass
int cp_buf_lds(bool conc, int tiles, int cpp) { return (conc ? 2 : 1) * tiles * 16 * cpp * 64; }

// DBG (timing-only, wrong results): 1 no multiply, 2 no streaming.
template <int kTiles, bool kConc, int DBG = 0>
__global__ __launch_bounds__(1024, 1) void csr_colpass_agg_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, int n, int rows_per_wg, const int8_t* __restrict__ zq,
    int chunks, int cpp, const uint32_t* __restrict__ colmax, const float* __restrict__ s, float* __restrict__ y,
    int ldy, int beta) {
    constexpr int NS = cp_stream_waves(kConc);  // streaming waves
    constexpr int MW0 = kConc ? NS : 0;         // first multiply wave
    constexpr int NM = 16 - MW0;                // multiply waves
    constexpr int KP = NM == 16 ? 1 : 2;        // dwords (k-step pairs) per multiply wave and chunk
    constexpr int NBUF = kConc ? 2 : 1;
    extern __shared__ __attribute__((aligned(16))) uint32_t cp_lds[];
    __shared__ int e_sh[kF];
    __shared__ int rpos[kTiles * 16], rend[kTiles * 16];  // per local row: next entry, row end
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int r0 = (int)blockIdx.x * rows_per_wg;
    const int nrows = min(rows_per_wg, n - r0);
    if (nrows <= 0) return;  // (uniform: the whole workgroup)
    const int nnz = rp[n];
    const int tiles = (nrows + 15) / 16;
    const int rsp = 16 * cpp;               // dwords per bit row of a pass buffer
    const int bufdw = kTiles * 16 * rsp;    // dwords per pass buffer
    uint32_t* const bufs = cp_lds + NS * kCpUnits * 256;
    if (t < 64) {
        const uint32_t m = colmax_of(colmax, t);
        if (t < kF) e_sh[t] = col_exponent(m);
    }
    for (int i = t; i < kTiles * 16; i += 1024) {
        rpos[i] = i < nrows ? rp[r0 + i] : 0;
        rend[i] = i < nrows ? rp[r0 + i + 1] : 0;
    }
    for (int d = 4 * t; d < NBUF * bufdw; d += 4096)
        *reinterpret_cast<uint4*>(bufs + d) = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    const int npass = (chunks + cpp - 1) / cpp;

    // ---- streaming waves' state
    const int kcnt = wave < NS && nrows > wave ? (nrows - 1 - wave) / NS + 1 : 0;  // rows of this wave (<= 12)
    const uint32_t ring_lds = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint32_t*)cp_lds) +
                              (uint32_t)(wave * kCpUnits * 1024);
    const uint32_t* const myring = cp_lds + wave * kCpUnits * 256;
    int kis = 0;  // steps issued (ring slot = kis % kCpRing)

    // ---- multiply waves' state
    const int mw = wave - MW0;
    const int L = mw & 3, pm0 = (mw >> 2) * KP;  // limb; dwords pm0 .. pm0 + KP - 1 (k-steps 2pm, 2pm + 1)
    const int r16 = lane & 15, g = lane >> 4;
    v4i acc[kTiles];
#pragma unroll
    for (int T = 0; T < kTiles; ++T) acc[T] = v4i{0, 0, 0, 0};

    for (int pass = 0; pass < npass; ++pass) {
        const int c0 = pass * cpp, cn = min(cpp, chunks - c0);
        uint32_t* const buf = bufs + (kConc ? (pass & 1) : 0) * bufdw;
        if (wave < NS && DBG != 2) {
            // stream pass `pass`: columns [lo, hi) of this wave's rows into buf
            const int lo = c0 * kChunk, hi = min(n, (c0 + cn) * kChunk);
            uint32_t act = 0u;  // rows that may still hold entries of this pass
            for (int k = 0; k < kcnt; ++k) {
                const int i = wave + NS * k;
                if (__builtin_amdgcn_readfirstlane(rpos[i]) < __builtin_amdgcn_readfirstlane(rend[i])) act |= 1u << k;
            }
            uint32_t fl = 0u;  // rows with a step in flight
            int cursor = 0, nf = 0;
            int fk0 = 0, fa0 = 0, fp0 = 0, fk1 = 0, fa1 = 0, fp1 = 0, fk2 = 0, fa2 = 0, fp2 = 0;  // FIFO, oldest first
            while (true) {
                while (nf < kCpRing) {  // issue: the next row (round robin) with no step in flight
                    const uint32_t elig = act & ~fl;
                    if (elig == 0u) break;
                    const uint32_t up = elig & (~0u << cursor);
                    const int k = __builtin_ctz(up != 0u ? up : elig);
                    cursor = k + 1 >= kcnt ? 0 : k + 1;
                    const int i = wave + NS * k;
                    const int p0 = __builtin_amdgcn_readfirstlane(rpos[i]);
                    const int a = p0 & ~3;
                    const uint32_t unit = (uint32_t)(2 * (kis % kCpRing));
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int e = a + 256 * h + 4 * lane;
                        const int* src = e + 4 <= nnz ? col + e : col;  // past the array: a dummy block
                        lds_dma16(src, ring_lds + (unit + h) * 1024u);
                    }
                    ++kis;
                    fl |= 1u << k;
                    if (nf == 0) { fk0 = k; fa0 = a; fp0 = p0; }
                    else if (nf == 1) { fk1 = k; fa1 = a; fp1 = p0; }
                    else { fk2 = k; fa2 = a; fp2 = p0; }
                    ++nf;
                }
                if (nf == 0) break;  // the pass is done for this wave
                wait_vmcnt(2 * (nf - 1));  // the oldest step landed
                asm volatile("" ::: "memory");
                const int k = fk0, a = fa0, p0 = fp0;
                const int i = wave + NS * k;
                const int end = __builtin_amdgcn_readfirstlane(rend[i]);
                const uint32_t* sl = myring + (2 * ((kis - nf) % kCpRing)) * 256 + 8 * lane;
                const int4 q0 = *reinterpret_cast<const int4*>(sl);
                const int4 q1 = *reinterpret_cast<const int4*>(sl + 4);
                int c[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
                const int p = a + 8 * lane;
                const bool tail = a + kDnStep + 4 > nnz;  // (wave-uniform) entries past the array reloaded
                if (tail) {
#pragma unroll
                    for (int e = 0; e < 8; ++e)
                        if (p + e < end && (((p + e) & ~3) + 4 > nnz)) c[e] = col[p + e];
                }
                uint32_t* const rowb = buf + i * rsp;
                // first entry of this lane at or past hi (sorted: the row's crossing is the first such entry)
                int myx = 0x7FFFFFFF;
#pragma unroll
                for (int e = 7; e >= 0; --e)
                    if (p + e >= p0 && p + e < end && c[e] >= hi) myx = p + e;
                const bool full = a >= p0 && a + kDnStep <= end;  // every entry of the step is the row's
                bool done = false;
                if (full && c[7] < hi) {  // (c[7] < hi: all eight are in the pass; ascending)
                    const uint32_t wf = (uint32_t)(c[0] - lo) >> 5;
                    const int base = lo + (int)(wf << 5);
                    uint32_t out = 0u;
                    uint64_t m = 0;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const uint32_t r = (uint32_t)(c[e] - base);
                        out |= r >> 6;
                        m |= 1ull << (r & 63);
                    }
                    if (out == 0u) {
                        dn_or(rowb + wf, (uint32_t)m);
                        dn_or(rowb + wf + 1, (uint32_t)(m >> 32));
                        done = true;
                    }
                }
                if (!done) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const int v = c[e];
                        if (p + e >= p0 && p + e < end && v < hi) atomicOr(rowb + ((v - lo) >> 5), 1u << ((v - lo) & 31));
                    }
                }
                // the row goes on in this pass iff no entry reached hi and the step
                // did not reach the row's end
                const uint64_t hit = __ballot(myx != 0x7FFFFFFF);
                int nextpos;
                bool more;
                if (hit != 0ull) {
                    nextpos = __builtin_amdgcn_readlane(myx, __builtin_ctzll(hit));
                    more = false;
                } else if (a + kDnStep < end) {
                    nextpos = a + kDnStep;
                    more = true;
                } else {
                    nextpos = end;
                    more = false;
                }
                if (lane == 0) rpos[i] = nextpos;
                fl &= ~(1u << k);
                if (!more) act &= ~(1u << k);
                fk0 = fk1; fa0 = fa1; fp0 = fp1;
                fk1 = fk2; fa1 = fa2; fp1 = fp2;
                --nf;
            }
        }
        __syncthreads();  // pass `pass` is in buf (and, kConc, the multiply waves are done with pass - 1)
        if (kConc && wave < NS && pass + 1 < npass) {
            // clear the rows this wave owns in the other buffer (multiplied up to the barrier) for the next pass
            uint32_t* const nb = bufs + ((pass + 1) & 1) * bufdw;
            for (int k = 0; k < kcnt; ++k)
                for (int d = 4 * lane; d < rsp; d += 256)
                    *reinterpret_cast<uint4*>(nb + (wave + NS * k) * rsp + d) = make_uint4(0u, 0u, 0u, 0u);
        }
        if (wave >= MW0 && DBG != 1) {
            // multiply pass `pass`: chunks c0 .. c0 + cn - 1, starting at a block-dependent one
            const int rot = (int)(blockIdx.x % (unsigned)cn);
            const v4i* const zv = reinterpret_cast<const v4i*>(zq) + (2 * pm0 * kLimbs + L) * 64 + lane;
            constexpr int D = kRbAhead;
            v4i bq[D][2 * KP];
#define LDS_CP_LOAD(cc, BQ)                                                                   \
    do {                                                                                      \
        const int u_ = (cc) < cn ? ((cc) + rot < cn ? (cc) + rot : (cc) + rot - cn) : 0;      \
        const v4i* z_ = zv + (int64_t)(c0 + u_) * (kChunkBytes / 16);                         \
        _Pragma("unroll") for (int x = 0; x < 2 * KP; ++x) BQ[x] = z_[x * kLimbs * 64];       \
    } while (0)
#pragma unroll
            for (int d = 0; d < D - 1; ++d) LDS_CP_LOAD(d, bq[d]);
            for (int cb = 0; cb < cn; cb += D) {
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    const int cc = cb + d;
                    if (cc < cn) {
                        LDS_CP_LOAD(cc + D - 1, bq[(d + D - 1) % D]);
                        const int u = cc + rot < cn ? cc + rot : cc + rot - cn;
                        const uint32_t* ab = buf + r16 * rsp + u * 16 + 4 * g + pm0;
#pragma unroll
                        for (int T = 0; T < kTiles; ++T) {
                            if (T < tiles) {
                                uint32_t w[KP];
                                if constexpr (KP == 2) {
                                    const uint2 ww = *reinterpret_cast<const uint2*>(ab + T * 16 * rsp);
                                    w[0] = ww.x;
                                    w[1] = ww.y;
                                } else {
                                    w[0] = ab[T * 16 * rsp];
                                }
#pragma unroll
                                for (int x = 0; x < 2 * KP; ++x) {
                                    const uint32_t wsel = w[x >> 1];
                                    const int sh = 4 * (x & 1);
                                    v4i av;
                                    av.x = (int)((wsel >> sh) & 0x01010101u);
                                    av.y = (int)((wsel >> (sh + 1)) & 0x01010101u);
                                    av.z = (int)((wsel >> (sh + 2)) & 0x01010101u);
                                    av.w = (int)((wsel >> (sh + 3)) & 0x01010101u);
                                    acc[T] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bq[d][x], acc[T], 0, 0, 0);
                                }
                            }
                        }
                    }
                }
            }
#undef LDS_CP_LOAD
        }
        if constexpr (!kConc) {
            __syncthreads();  // every wave's reads of the buffer are done
            if (pass + 1 < npass)
                for (int d = 4 * t; d < bufdw; d += 4096)
                    *reinterpret_cast<uint4*>(bufs + d) = make_uint4(0u, 0u, 0u, 0u);
            __syncthreads();
        }
    }
    // the int64 sums in the (idle) ring memory
    unsigned long long* const sums = reinterpret_cast<unsigned long long*>(cp_lds);  // [kTiles·16][16]
    __syncthreads();
    for (int i = t; i < kTiles * 16 * kF; i += 1024) sums[i] = 0ull;
    __syncthreads();
    if (wave >= MW0) {
#pragma unroll
        for (int T = 0; T < kTiles; ++T)
            if (T < tiles)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    atomicAdd(sums + (T * 16 + 4 * g + i) * kF + r16,
                              (unsigned long long)((int64_t)acc[T][i] * ((int64_t)1 << (8 * L))));
    }
    __syncthreads();
    for (int o = t; o < nrows * kF; o += 1024) {
        const int lr = o >> 4, f = o & 15;
        const int row = r0 + lr;
        const float r = s[row] * (float)ldexp((double)(int64_t)sums[o], -e_sh[f]);
        float* out = y + (int64_t)row * ldy + f;
        *out = beta ? *out + r : r;
    }
}

// ---------------------------------------------------------------------------
// CSR-SpMM for dense sampled graphs, spill-pass form (round 4; its frozen
// configurations, the product's ancestors).  The row-block kernel above writes every bit
// row to a global slab and reads it back (51 MB each way at config 5, and its
// multiply phase runs after the stream instead of beside it); the column-pass
// kernel keeps the bits on chip but re-reads the step that straddles each
// pass boundary and feeds its streaming waves through LDS rings that leave
// no room for deep prefetch.  Here each workgroup owns one contiguous block
// of rows (R <= 96) and sweeps its columns in P passes of cpp 512-column
// chunks, with three LDS bit buffers (R rows × cpp·64 B each):
//  * streaming waves 0-7 (wave w: local rows w, w + 8, …) load 1-KB steps
//    of col (256 entries, one 16-byte load per lane) into a register ring D
//    steps deep — no LDS ring, so 8·(D − 1) KB stay in flight per CU — and
//    set each entry's bit in pass p's buffer; entries of pass p + 1 that a
//    step holds (a row's boundary step, or steps streamed past a row's
//    predicted pass end) go to pass p + 1's buffer at once ("spill"), so no
//    step is read twice.  A row's stream in pass p ends at its predicted end
//    (the row's remaining entries × the pass's share of the remaining
//    columns + kSpMargin); a row whose boundary lies beyond it is finished
//    with blocking loads (rare: dense rows are binomial).  Entries past pass
//    p + 1 (sparse rows only) are left for a later pass to re-read.
//  * multiply waves 8-15 (limb m & 3, k-steps 4(m >> 2) … + 3 of each chunk)
//    run pass p − 1's buffer against the digits of its chunks while pass p
//    streams (lds_aggregate_bitmask's digits, k order and exact int32 sums),
//    then zero the buffer for pass p + 2's spills.  One barrier per pass.
// The sums of the multiply waves meet in LDS as int64 adds (exact, order
// free), then y = s_i · 2^-e_f · Σ.  Columns must ascend within each row
// (canonical CSR, as every sampler and fill of this package writes it).
// ---------------------------------------------------------------------------
constexpr int kSpStream = 8;         // streaming waves 0-7; multiply waves 8-15
constexpr int kSpThreads = 1024;
constexpr int kSpStep = 256;         // entries per step: lane l loads p + 4l … + 3
constexpr int kSpMaxRows = 96;       // rows per workgroup (six 16-row tiles)
constexpr int kSpMaxGrid = 512;
constexpr int kSpMargin = 192;       // entries streamed past a row's predicted pass end
constexpr int kSpStateInts = 3 * kSpMaxRows + 20 + 12 * 12 * 4;  // pos, rend, fin per row; the exponents;
                                                                         // done counters; (DBG 8) ring slot records
constexpr int kSpDepth = 8;          // 1-KB ring slots per streaming wave (D - 1 steps in flight)

struct SpGeom {
    int cpp, passes, rowdw;  // chunks per pass, passes, dwords per buffer row (16·cpp + 2: bank spread)
};
SpGeom sp_geom(int chunks, int tiles, int depth, int ns = kSpStream, int slot = 1024) {
    const int rows = 16 * tiles;
    int cpp = ((163840 - ns * depth * slot - 4 * kSpStateInts) / (3 * rows * 4) - 2) / 16;
    if (cpp > chunks) cpp = chunks;
    if (cpp < 1) cpp = 1;
    const int passes = (chunks + cpp - 1) / cpp;
    cpp = (chunks + passes - 1) / passes;
    return SpGeom{cpp, passes, 16 * cpp + 2};
}
int sp_lds_bytes(int tiles, const SpGeom& g, int depth, int ns = kSpStream, int slot = 1024) {
    return ns * depth * slot + 3 * 16 * tiles * g.rowdw * 4 + 4 * kSpStateInts;
}

// The product configuration of the spill-pass kernel: 12 streaming + 4
// multiply waves, 2-KB steps (8 entries per lane, the fast paths for pass
// p + 1 and for boundary lanes), the ring in registers, four steps deep (asm
// loads with counted waits; no LDS ring, so the whole LDS holds the pass
// buffers: 4 passes at config 5), and a step's pass bounds and bit-row
// pointers reused while its (row, pass) repeats (mode 17).  Config 5: 165 µs,
// against 171 without the reuse (mode 15), 178 with a 2-slot LDS ring (mode
// 12, 6 passes) and 375 for round 4's first form (8 + 8 waves, 1-KB steps, an
// LDS ring 8 deep): the streaming waves are bound by the instructions they
// issue per step, not by HBM.
constexpr int kSpProdMode = 17, kSpProdWaves = 12, kSpProdDepth = 4;
struct SpCfg {
    int depth, ns, slot;  // ring slots per streaming wave, streaming waves, bytes per slot
};
// the spill-pass configurations by dbg code (tools/spmm_config5.py; 64 = the round-4 product form)
SpCfg sp_cfg(int dbg) {
    if (dbg == 0) return SpCfg{kSpProdDepth, kSpProdWaves, 0};  // (the register ring takes no LDS)
    if (dbg == 58 || dbg == 59) return SpCfg{2, 12, 2048};
    if (dbg >= 60 && dbg <= 69) return SpCfg{dbg == 60 || dbg == 68 ? 3 : dbg == 62 ? 6 : 4, dbg == 67 ? 14 : 12, 0};  // register ring: no LDS
    const int depth = dbg == 33 || dbg == 38 || dbg == 44 ? 6 : dbg == 34 || dbg == 42 ? 12
                    : dbg == 43 || dbg == 46 ? 5 : dbg == 45 || dbg == 48 || (dbg >= 50 && dbg <= 52) ? 4
                    : dbg == 47 || dbg == 49 || dbg == 53 || dbg == 54 ? 3 : dbg >= 55 && dbg <= 57 ? 2 : kSpDepth;
    const int ns = (dbg >= 43 && dbg <= 47) || dbg == 50 || (dbg >= 52 && dbg <= 55) ? 12
                 : dbg == 48 || dbg == 49 || dbg == 51 || dbg == 57 ? 14 : kSpStream;
    return SpCfg{depth, ns, dbg >= 54 && dbg <= 57 ? 2048 : 1024};
}

// Entry c (column) of a row in pass p: its bit in pass p's buffer row bp
// (c < hi), pass p + 1's row bq (c < hq), or past both (returns true).
__device__ __forceinline__ bool sp_put(int c, int lo, int hi, int hq, uint32_t* bp, uint32_t* bq, bool& spill) {
    if (c < lo) return false;  // (columns out of order: never written outside the row's buffer)
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

// A streaming wave's bit setting for one step (lane: entries i0 … i0 + 3 of
// its row, columns c; the row's entries [rlo, rup); pass p's columns [lo, hi),
// pass p + 1's [hi, hq)).  Each quad of lanes (16 entries, ~32 columns of a
// dense row) ORs its pass-p entries into one 64-bit window from its first
// valid column's word: one pair of LDS ORs per quad instead of per lane (four
// lanes on one word serialise).  Entries outside the window — sparse rows,
// the next pass's (spill), later passes' (their first index: myx) — take the
// per-entry path.
__device__ __forceinline__ void sp_set_bits(const int (&c)[4], int i0, int rlo, int rup, int lo, int hi, int hq,
                                            uint32_t* bp, uint32_t* bq, int lane, bool& spill, int& myx) {
    bool v[4];
    int cm = 0x7FFFFFFF;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        v[e] = i0 + e >= rlo && i0 + e < rup;
        if (v[e] && c[e] >= lo && c[e] < hi) cm = min(cm, c[e]);
    }
    cm = min(cm, __builtin_amdgcn_mov_dpp(cm, 0xB1, 0xF, 0xF, false));  // quad_perm 1,0,3,2
    cm = min(cm, __builtin_amdgcn_mov_dpp(cm, 0x4E, 0xF, 0xF, false));  // quad_perm 2,3,0,1
    const int wb = cm == 0x7FFFFFFF ? 0 : (cm - lo) >> 5;
    uint32_t mlo = 0u, mhi = 0u;
    bool left = false;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        if (!v[e]) continue;
        const uint32_t r = (uint32_t)(c[e] - lo) - (uint32_t)(wb << 5);
        if (c[e] >= lo && c[e] < hi && r < 64u) {
            if (r < 32u) mlo |= 1u << r;
            else mhi |= 1u << (r - 32u);
        } else {
            left = true;
        }
    }
    mlo |= (uint32_t)__builtin_amdgcn_mov_dpp((int)mlo, 0xB1, 0xF, 0xF, false);
    mhi |= (uint32_t)__builtin_amdgcn_mov_dpp((int)mhi, 0xB1, 0xF, 0xF, false);
    mlo |= (uint32_t)__builtin_amdgcn_mov_dpp((int)mlo, 0x4E, 0xF, 0xF, false);
    mhi |= (uint32_t)__builtin_amdgcn_mov_dpp((int)mhi, 0x4E, 0xF, 0xF, false);
    if ((lane & 3) == 0) {
        dn_or(bp + wb, mlo);
        dn_or(bp + wb + 1, mhi);
    }
    if (__ballot(left) != 0ull && left) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (!v[e]) continue;
            const uint32_t r = (uint32_t)(c[e] - lo) - (uint32_t)(wb << 5);
            if (c[e] >= lo && c[e] < hi && r < 64u) continue;
            if (sp_put(c[e], lo, hi, hq, bp, bq, spill)) myx = min(myx, i0 + e);
        }
    }
}

// A streaming wave's bit setting for one step without per-entry branches
// (DBG 5): each lane ORs its entries of pass p into one 64-bit window from
// its first such entry's word and its entries of pass p + 1 into another, so
// a row's boundary steps (about a third of all steps at 8 passes) cost about
// what an interior step costs.  Entries that fit neither window (sparse rows)
// take single-bit ORs under a wave-uniform guard; entries past pass p + 1
// only report their first index (myx).  Same bits as sp_put entry by entry.
__device__ __forceinline__ void sp_set_bits_win(const int (&c)[4], int i0, int rlo, int rup, int lo, int hi, int hq,
                                                uint32_t* bp, uint32_t* bq, bool& spill, int& myx) {
    constexpr int kNone = 0x7FFFFFFF;
    bool vp[4], vq[4];
    int fp = kNone, fq = kNone;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const bool v = i0 + e >= rlo && i0 + e < rup;
        vp[e] = v && c[e] >= lo && c[e] < hi;
        vq[e] = v && c[e] >= hi && c[e] < hq;
        spill = spill || (v && c[e] >= hi);
        myx = v && c[e] >= hq ? min(myx, i0 + e) : myx;
        fp = vp[e] ? min(fp, c[e]) : fp;
        fq = vq[e] ? min(fq, c[e]) : fq;
    }
    // window starts (a lane without entries of a pass: the row's first word, empty mask)
    const int bp0 = fp == kNone ? lo : lo + ((fp - lo) & ~31);
    const int bq0 = fq == kNone ? hi : hi + ((fq - hi) & ~31);
    uint64_t mp = 0, mq = 0;
    bool misfit = false;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const uint32_t rp = (uint32_t)(c[e] - bp0), rq = (uint32_t)(c[e] - bq0);
        mp |= vp[e] && rp < 64u ? 1ull << (rp & 63u) : 0ull;
        mq |= vq[e] && rq < 64u ? 1ull << (rq & 63u) : 0ull;
        misfit = misfit || (vp[e] && rp >= 64u) || (vq[e] && rq >= 64u);
    }
    uint32_t* const wp = bp + ((bp0 - lo) >> 5);
    dn_or(wp, (uint32_t)mp);
    dn_or(wp + 1, (uint32_t)(mp >> 32));
    if (__ballot(mq != 0ull) != 0ull) {
        uint32_t* const wq = bq + ((bq0 - hi) >> 5);
        dn_or(wq, (uint32_t)mq);
        dn_or(wq + 1, (uint32_t)(mq >> 32));
    }
    if (__ballot(misfit) != 0ull) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if (vp[e] && (uint32_t)(c[e] - bp0) >= 64u) atomicOr(bp + ((c[e] - lo) >> 5), 1u << ((c[e] - lo) & 31));
            if (vq[e] && (uint32_t)(c[e] - bq0) >= 64u) atomicOr(bq + ((c[e] - hi) >> 5), 1u << ((c[e] - hi) & 31));
        }
    }
}

// DBG (timing-only ablations, wrong results): 1 no MFMAs, 2 streaming waves
// load and count but set no bits.  The product path is DBG = 0.  Same
// results: 3 drains the ring before every read, 4 quad-reduced bit setting
// (sp_set_bits), 5 windowed bit setting on every step (sp_set_bits_win), 6 each
// step's columns read from the ring one step ahead of its bit ORs.  Timing
// only: 7 the interior steps' ORs as plain stores.  8 (same results): the
// ring loop not unrolled (the slot a runtime index, its records in LDS); 9
// the interior fast path, sp_set_bits_win for every other step; 10 a second
// fast path for lanes whose four entries all belong to pass p + 1; 11 as 10
// and a third for lanes that straddle the pass boundary; 12 as 11 with 2-KB
// steps (8 entries per lane, two DMAs per step).
template <int kTiles, int D, int DBG = 0, int NS = kSpStream>
__global__ __launch_bounds__(kSpThreads, 1) void csr_spill_agg_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, int n, int rows_per_wg, const int8_t* __restrict__ zq,
    int chunks, int cpp, int passes, int rowdw, const uint32_t* __restrict__ colmax, const float* __restrict__ s,
    float* __restrict__ y, int ldy, int beta) {
    extern __shared__ __attribute__((aligned(16))) uint32_t sp_lds_all[];
    // entries per lane and step: 4 (1-KB steps) or, DBG 12, 8 (2-KB steps, two DMAs)
    constexpr int kE = DBG == 20 ? 12 : DBG >= 12 ? 8 : 4;  // (20: 3-KB steps)
    constexpr bool kNoBits = DBG == 2 || DBG == 13;  // timing only: no bit setting
    constexpr bool kRegRing = DBG >= 15 && DBG <= 20;  // the ring in registers (asm loads, counted waits): no LDS ring
    constexpr bool kDynRows = DBG == 16;  // rows taken per pass from an LDS counter, not wave + NS·i
    constexpr bool kKeyCache = DBG >= 17 && DBG <= 20;  // a step's pass bounds and bit rows reused while (row, pass) repeats
    constexpr bool kOneBallot = DBG == 19;  // one ballot for the spill and past-pass flags of a step
    constexpr bool kLean = DBG == 18;  // fast-path ORs without the zero test; one wave-wide skip of the other paths
    constexpr bool kNoMfma = DBG == 1 || DBG == 14;  // timing only: no matrix-core products
    constexpr int kStep = 64 * kE;
    static_assert((D - 1) * (kE / 4) <= 15, "vmcnt field");
    uint32_t* const sp_lds = sp_lds_all + (kRegRing ? 0 : NS * D * kStep);  // after the rings: pass buffers, row state
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
    int4* const meta = reinterpret_cast<int4*>(done + 4);  // (DBG 8) per wave and slot: start, row bounds, key
    int* const nxt = done + 4;  // (kDynRows) per pass: rows taken so far (the meta area: passes <= 576)
    const int nnz = rp[n];
    const int span = cpp * kChunk;  // columns per pass
    for (int i = t; i < 3 * bufdw; i += kSpThreads) sp_lds[i] = 0u;
    if constexpr (kDynRows)
        for (int i = t; i < passes; i += kSpThreads) nxt[i] = 0;
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

    // multiply waves: kMW; each runs kLW limbs over kHalves halves of every chunk
    constexpr int kMW = 16 - NS;
    constexpr int kLW = kMW == 2 ? 2 : 1;
    constexpr int kHalves = kMW <= 4 ? 2 : 1;
    static_assert(kMW == 2 || kMW == 4 || kMW == 8, "8, 4 or 2 multiply waves");
    v4i acc[kLW][kTiles];
#pragma unroll
    for (int l = 0; l < kLW; ++l)
#pragma unroll
        for (int T = 0; T < kTiles; ++T) acc[l][T] = v4i{0, 0, 0, 0};

    if (wave < NS) {
        // ---- streaming waves -------------------------------------------------
        const int nrw = nrows > wave ? (nrows - 1 - wave) / NS + 1 : 0;  // this wave's rows
        const int* const dummy = reinterpret_cast<const int*>(zq) + 4 * lane;    // null steps load here
        // issue side: pass ip, row ordinal iq, next step ia, the row's stream end
        int ip = 0, iq = 0, ia = 0, iend = 0, ilow = 0, iup = 0;
        int ilr = -1, spins = 0;  // (kDynRows) the row taken for pass ip, -1 none; wait steps so far
        int pk = -1, plo = 0, phi = 0, phq = 0;  // (kKeyCache) (row | pass << 8) of the last step, its bounds
        uint32_t *pbp = sp_lds, *pbq = sp_lds;  // and bit rows
        bool irow = false, ifirst = false;
        int pending = 0;  // non-null steps in the ring
        // the ring: a step's data, start, row bounds and packed (row | pass << 8 |
        // first << 16 | last << 17), -1 for a null step
        int ma[D], mlo[D], mup[D], mk[D];
        v4i rg[D][kE / 4];  // (kRegRing) the ring's columns
        const uint32_t ring_lds = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint32_t*)sp_lds_all) +
                                  (uint32_t)(wave * D * kStep * 4);
        const uint32_t* const myring = sp_lds_all + wave * D * kStep;
        // process side: the pass the multiply waves wait for; the row's flags
        int cp = 0, estar = 0x7FFFFFFF;
        int4 nxt_ = int4{0, 0, 0, 0};  // (DBG 6) the next step's columns
        bool bnd = false;
#define LDS_SP_ISSUE(J)                                                                                      \
    do {                                                                                                     \
        int a_ = -1, lo_ = 0, up_ = 0, k_ = -1;                                                              \
        while (ip < passes) {                                                                                \
            if (!irow) {                                                                                     \
                if constexpr (kDynRows) {                                                                    \
                    if (ilr < 0) { /* take the next row of pass ip */                                        \
                        int g_ = 0;                                                                          \
                        if (lane == 0) g_ = atomicAdd(nxt + ip, 1);                                          \
                        g_ = __builtin_amdgcn_readfirstlane(g_);                                             \
                        if (g_ >= nrows) {                                                                   \
                            ++ip;                                                                            \
                            continue;                                                                        \
                        }                                                                                    \
                        ilr = g_;                                                                            \
                    }                                                                                        \
                } else if (iq >= nrw) {                                                                      \
                    ++ip;                                                                                    \
                    iq = 0;                                                                                  \
                    continue;                                                                                \
                }                                                                                            \
                const int lr_ = kDynRows ? ilr : wave + NS * iq;                                             \
                /* previous pass not closed (kDynRows: a bound on the wait, so that no logic error can */   \
                /* leave waves spinning on the GPU; never reached when the barriers below are right) */       \
                if (__builtin_amdgcn_readfirstlane(fin[lr_]) < ip - 1 && (!kDynRows || ++spins < (1 << 20))) {  \
                    if constexpr (kDynRows) k_ = -2 - ip; /* a wait step: passes < ip are this wave's past */  \
                    break;                                                                                   \
                }                                                                                            \
                ilow = __builtin_amdgcn_readfirstlane(pos[lr_]);                                             \
                iup = __builtin_amdgcn_readfirstlane(rend[lr_]);                                             \
                if (ilow >= iup) { /* the row is done: closed for this pass too */                          \
                    fin[lr_] = ip;                                                                           \
                    ++iq;                                                                                    \
                    ilr = -1;                                                                                \
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
            k_ = (kDynRows ? ilr : wave + NS * iq) | (ip << 8) | (ifirst ? 1 << 16 : 0) | (last_ ? 1 << 17 : 0); \
            ia += kStep;                                                                                     \
            ifirst = false;                                                                                  \
            if (last_) {                                                                                     \
                irow = false;                                                                                \
                ++iq;                                                                                        \
                ilr = -1;                                                                                    \
            }                                                                                                \
            break;                                                                                           \
        }                                                                                                    \
        if constexpr (DBG == 8) {                                                                            \
            if (lane == 0) meta[wave * D + (J)] = int4{a_, lo_, up_, k_};                                    \
        } else {                                                                                             \
            ma[J] = a_;                                                                                      \
            mlo[J] = lo_;                                                                                    \
            mup[J] = up_;                                                                                    \
            mk[J] = k_;                                                                                      \
        }                                                                                                    \
        pending += k_ >= 0 ? 1 : 0;                                                                          \
        _Pragma("unroll") for (int h_ = 0; h_ < kE / 4; ++h_) {                                              \
            const int aa_ = a_ + (kRegRing ? kE * lane + 4 * h_ : 256 * h_ + 4 * lane);                       \
            const int* src_ = (a_ >= 0 && aa_ + 4 <= nnz) ? col + aa_ : dummy;                               \
            if constexpr (kRegRing) rb_gload(rg[J][h_], reinterpret_cast<const v4i*>(src_));                  \
            else lds_dma16(src_, ring_lds + (uint32_t)(J) * (uint32_t)(4 * kStep) + 1024u * h_);             \
        }                                                                                                    \
    } while (0)
#define LDS_SP_PROCESS(J)                                                                                    \
    do {                                                                                                     \
        /* slot J's step landed: every iteration issues exactly one DMA, so D - 1 younger ones stay in */    \
        /* flight (the rare paths' plain loads are waited for where they are used: stricter, never looser) */ \
        if (DBG == 3) __builtin_amdgcn_s_waitcnt(0x0F70);                                                     \
        else if (DBG == 6) __builtin_amdgcn_s_waitcnt(0x0F70 | (D - 2)); /* slots J and J + 1 landed */       \
        else __builtin_amdgcn_s_waitcnt(0x0F70 | ((D - 1) * (kE / 4)));                                                 \
        asm volatile("" ::: "memory");                                                                       \
        const int4 cur_ = nxt_; /* DBG 6: slot J, read one step ahead of its bit ORs */                      \
        if (DBG == 6) nxt_ = *reinterpret_cast<const int4*>(myring + (((J) + 1) % D) * 256 + 4 * lane);      \
        int k_, ma_, mlo_, mup_;                                                                             \
        if constexpr (DBG == 8) {                                                                            \
            const int4 mt_ = meta[wave * D + (J)];                                                           \
            k_ = __builtin_amdgcn_readfirstlane(mt_.w);                                                      \
            ma_ = __builtin_amdgcn_readfirstlane(mt_.x);                                                     \
            mlo_ = __builtin_amdgcn_readfirstlane(mt_.y);                                                    \
            mup_ = __builtin_amdgcn_readfirstlane(mt_.z);                                                    \
        } else {                                                                                             \
            k_ = mk[J];                                                                                      \
            ma_ = ma[J];                                                                                     \
            mlo_ = mlo[J];                                                                                   \
            mup_ = mup[J];                                                                                   \
        }                                                                                                    \
        if (kDynRows && k_ <= -2) {                                                                          \
            /* a wait step issued at pass -2 - k_: every step of the earlier passes is processed, so arrive */ \
            /* at their barriers (the row's previous pass may belong to a wave waiting at one of them) */    \
            for (; cp < -2 - k_; ++cp) {                                                                     \
                __builtin_amdgcn_s_waitcnt(0xC07F);                                                          \
                __builtin_amdgcn_s_barrier();                                                                \
            }                                                                                                \
        }                                                                                                    \
        if (k_ >= 0) {                                                                                       \
            --pending;                                                                                       \
            const int lr_ = k_ & 0xFF, p_ = (k_ >> 8) & 0xFF;                                                \
            for (; cp < p_; ++cp) { /* pass cp streamed: the multiply waves take it */                      \
                __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0): this wave's bit ORs are done */           \
                __builtin_amdgcn_s_barrier();                                                                \
            }                                                                                                \
            if (k_ & (1 << 16)) {                                                                            \
                bnd = false;                                                                                 \
                estar = 0x7FFFFFFF;                                                                          \
            }                                                                                                \
            if (!kKeyCache || (k_ & 0xFFFF) != pk) {                                                         \
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
            const int a_ = ma_, rlo_ = mlo_, rup_ = mup_;                                                    \
            int c_[kE];                                                                                      \
            if constexpr (kRegRing) {                                                                        \
                if constexpr (kE == 8) rb_bind(rg[J][0], rg[J][1]);                                          \
                if constexpr (kE == 12) asm volatile("" : "+v"(rg[J][0]), "+v"(rg[J][1]), "+v"(rg[J][2]));   \
            }                                                                                                \
            _Pragma("unroll") for (int h_ = 0; h_ < kE / 4; ++h_) {                                          \
                const int4 v_ = kRegRing ? int4{rg[J][h_][0], rg[J][h_][1], rg[J][h_][2], rg[J][h_][3]}      \
                              : DBG == 6 ? cur_ : *reinterpret_cast<const int4*>(myring + (J) * kStep + kE * lane + 4 * h_); \
                c_[4 * h_] = v_.x;                                                                           \
                c_[4 * h_ + 1] = v_.y;                                                                       \
                c_[4 * h_ + 2] = v_.z;                                                                       \
                c_[4 * h_ + 3] = v_.w;                                                                       \
            }                                                                                                \
            const int i0_ = a_ + kE * lane;                                                                  \
            bool spill_ = false;                                                                        \
            int myx_ = 0x7FFFFFFF;                                                                      \
            if constexpr (DBG == 4) { /* the quad-reduced bit setting (sp_set_bits) */                  \
                if (a_ + kStep > nnz) {                                                                 \
                    _Pragma("unroll") for (int e = 0; e < 4; ++e)                                       \
                        if (i0_ + 4 > nnz) c_[e] = i0_ + e < nnz ? col[i0_ + e] : 0;                    \
                    sp_set_bits(c_, i0_, rlo_, rup_, lo_, hi_, hq_, bp_, bq_, lane, spill_, myx_);      \
                } else {                                                                                \
                    sp_set_bits(c_, i0_, rlo_, rup_, lo_, hi_, hq_, bp_, bq_, lane, spill_, myx_);      \
                }                                                                                       \
            } else {                                                                                    \
            bool fast_ = false;                                                                              \
            if (DBG != 5 && a_ >= rlo_ && a_ + kStep <= rup_) { /* interior (uniform): all the row's */   \
                const uint32_t w0_ = (uint32_t)(c_[0] - lo_) >> 5;                                           \
                fast_ = c_[0] >= lo_ && c_[kE - 1] < hi_ && (uint32_t)(c_[kE - 1] - lo_) - (w0_ << 5) < 64u; \
                if (fast_ && !kNoBits) {                                                                    \
                    uint64_t m_ = 0;                                                                         \
                    _Pragma("unroll") for (int e = 0; e < kE; ++e) m_ |= 1ull << ((uint32_t)(c_[e] - lo_) - (w0_ << 5)); \
                    if (DBG == 7) { /* timing only: plain stores instead of ORs */                           \
                        bp_[w0_] = (uint32_t)m_;                                                             \
                        bp_[w0_ + 1] = (uint32_t)(m_ >> 32);                                                 \
                    } else {                                                                                 \
                        if (kLean) { /* m_ is never 0 here: the low word holds c_[0]'s bit */                \
                            atomicOr(bp_ + w0_, (uint32_t)m_);                                               \
                            atomicOr(bp_ + w0_ + 1, (uint32_t)(m_ >> 32));                                   \
                        } else {                                                                             \
                            dn_or(bp_ + w0_, (uint32_t)m_);                                                  \
                            dn_or(bp_ + w0_ + 1, (uint32_t)(m_ >> 32));                                      \
                        }                                                                                    \
                    }                                                                                        \
                }                                                                                            \
                if (!kLean || __ballot(!fast_) != 0ull) { /* (kLean: every lane fast: skip both below) */    \
                if ((DBG == 10 || DBG >= 11) && !kNoBits && !fast_) { /* all of pass p + 1 (past the boundary) */       \
                    const uint32_t q0_ = (uint32_t)(c_[0] - hi_) >> 5;                                       \
                    if (c_[0] >= hi_ && c_[kE - 1] < hq_ && (uint32_t)(c_[kE - 1] - hi_) - (q0_ << 5) < 64u) { \
                        uint64_t m_ = 0;                                                                     \
                        _Pragma("unroll") for (int e = 0; e < kE; ++e) m_ |= 1ull << ((uint32_t)(c_[e] - hi_) - (q0_ << 5)); \
                        dn_or(bq_ + q0_, (uint32_t)m_);                                                      \
                        dn_or(bq_ + q0_ + 1, (uint32_t)(m_ >> 32));                                          \
                        spill_ = true;                                                                       \
                        fast_ = true;                                                                        \
                    }                                                                                        \
                }                                                                                            \
                if (DBG >= 11 && !kNoBits && !fast_ && c_[0] >= lo_ && c_[0] < hi_ && c_[kE - 1] >= hi_ &&               \
                    c_[kE - 1] < hq_ && (uint32_t)(c_[kE - 1] - hi_) < 64u) { /* straddles the boundary */   \
                    uint64_t mp_ = 0, mq_ = 0;                                                               \
                    bool ok_ = true;                                                                         \
                    _Pragma("unroll") for (int e = 0; e < kE; ++e) {                                         \
                        const bool in_ = c_[e] < hi_;                                                        \
                        const uint32_t r_ = in_ ? (uint32_t)(c_[e] - lo_) - (w0_ << 5) : (uint32_t)(c_[e] - hi_); \
                        ok_ = ok_ && r_ < 64u;                                                               \
                        const uint64_t b_ = 1ull << (r_ & 63u);                                              \
                        mp_ |= in_ ? b_ : 0ull;                                                              \
                        mq_ |= in_ ? 0ull : b_;                                                              \
                    }                                                                                        \
                    if (ok_) {                                                                               \
                        dn_or(bp_ + w0_, (uint32_t)mp_);                                                     \
                        dn_or(bp_ + w0_ + 1, (uint32_t)(mp_ >> 32));                                         \
                        dn_or(bq_, (uint32_t)mq_);                                                           \
                        dn_or(bq_ + 1, (uint32_t)(mq_ >> 32));                                               \
                        spill_ = true;                                                                       \
                        fast_ = true;                                                                        \
                    }                                                                                        \
                }                                                                                            \
                }                                                                                            \
            }                                                                                                \
            if (!fast_ && !kNoBits) {                                                                       \
                /* per entry; two copies under a uniform branch: only the array's last step reloads the */\
                /* lanes that read the dummy (a lane-conditional load costs vmcnt(0) on every path) */  \
                if (a_ + kStep > nnz) {                                                                 \
                    _Pragma("unroll") for (int e = 0; e < kE; ++e) {                                    \
                        const int idx_ = i0_ + e;                                                       \
                        if (idx_ >= rlo_ && idx_ < rup_ &&                                              \
                            sp_put((idx_ & ~3) + 4 > nnz ? col[idx_] : c_[e], lo_, hi_, hq_, bp_, bq_, spill_)) \
                            myx_ = min(myx_, idx_);                                                     \
                    }                                                                                   \
                } else if constexpr (DBG == 5 || DBG == 9) {                                            \
                    sp_set_bits_win(c_, i0_, rlo_, rup_, lo_, hi_, hq_, bp_, bq_, spill_, myx_);        \
                } else {                                                                                \
                    _Pragma("unroll") for (int e = 0; e < kE; ++e) {                                    \
                        const int idx_ = i0_ + e;                                                       \
                        if (idx_ >= rlo_ && idx_ < rup_ && sp_put(c_[e], lo_, hi_, hq_, bp_, bq_, spill_))\
                            myx_ = min(myx_, idx_);                                                     \
                    }                                                                                   \
                }                                                                                       \
            }                                                                                                \
            }                                                                                           \
            if (!kOneBallot || __ballot(spill_ || myx_ != 0x7FFFFFFF) != 0ull) { /* (most steps: neither) */ \
                if (__ballot(spill_) != 0ull) bnd = true;                                                    \
                const uint64_t xm_ = __ballot(myx_ != 0x7FFFFFFF);                                           \
                if (xm_ != 0ull) estar = min(estar, __builtin_amdgcn_readlane(myx_, __builtin_ctzll(xm_)));  \
            }                                                                                                \
            if (k_ & (1 << 17)) { /* the row's last issued step: where pass p + 1 starts */                 \
                int np_ = min(a_ + kStep, rup_);                                                             \
                if (estar == 0x7FFFFFFF && !bnd && np_ < rup_ && !kNoBits) {                               \
                    /* the boundary lies past the predicted end: finish the row with blocking loads */       \
                    while (np_ < rup_) {                                                                     \
                        const int b_ = (np_ & ~3) + 4 * lane;                                                \
                        bool sp2_ = false;                                                                   \
                        int mx2_ = 0x7FFFFFFF;                                                               \
                        _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                      \
                            const int idx_ = b_ + e;                                                         \
                            if (idx_ >= np_ && idx_ < rup_ &&                                                \
                                sp_put(col[idx_], lo_, hi_, hq_, bp_, bq_, sp2_))             \
                                mx2_ = min(mx2_, idx_);                                                      \
                        }                                                                                    \
                        np_ = min((np_ & ~3) + kSpStep, rup_);                                               \
                        const uint64_t xm_ = __ballot(mx2_ != 0x7FFFFFFF);                                   \
                        if (xm_ != 0ull) estar = min(estar, __builtin_amdgcn_readlane(mx2_, __builtin_ctzll(xm_))); \
                        if (__ballot(sp2_) != 0ull) break;                                                   \
                    }                                                                                        \
                }                                                                                            \
                if (estar != 0x7FFFFFFF) np_ = estar;                                                        \
                if (lane == 0) {                                                                             \
                    pos[lr_] = np_;                                                                          \
                    fin[lr_] = p_;                                                                           \
                }                                                                                            \
            }                                                                                                \
        }                                                                                                    \
    } while (0)
        if constexpr (DBG == 8) {  // one copy of the loop body, the slot a runtime index
            for (int j = 0; j < D - 1; ++j) LDS_SP_ISSUE(j);
            for (int j = 0;; j = j + 1 == D ? 0 : j + 1) {
                LDS_SP_ISSUE(j == 0 ? D - 1 : j - 1);
                LDS_SP_PROCESS(j);
                if (ip >= passes && pending == 0) goto streamed;
            }
        }
#pragma unroll
        for (int j = 0; j < D - 1; ++j) LDS_SP_ISSUE(j);
        if (DBG == 6) {  // slot 0 landed: read it ahead
            __builtin_amdgcn_s_waitcnt(0x0F70 | (D - 2));
            asm volatile("" ::: "memory");
            nxt_ = *reinterpret_cast<const int4*>(myring + 4 * lane);
        }
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
    } else {
        // ---- multiply waves --------------------------------------------------
        // 8 multiply waves: limb m & 3, k-steps 4(m >> 2) … + 3 of each chunk; 4
        // (NS = 12): limb m, both halves of each chunk in turn
        const int m = wave - NS, L = kLW * (m & 3), hh0 = kHalves == 2 ? 0 : m >> 2;
        const int r16 = lane & 15, g = lane >> 4;
        const v4i* const zv = reinterpret_cast<const v4i*>(zq) + L * 64 + lane;
        const int ntiles = (nrows + 15) / 16;
#define LDS_SP_DIG(CH, HH, DQ)                                                                 \
    do {                                                                                       \
        const v4i* z_ = zv + (int64_t)(CH) * (kChunkBytes / 16) + 4 * (HH) * kLimbs * 64;      \
        _Pragma("unroll") for (int l = 0; l < kLW; ++l)                                      \
            _Pragma("unroll") for (int i = 0; i < 4; ++i) DQ[l][i] = z_[i * kLimbs * 64 + l * 64]; \
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
                    _Pragma("unroll") for (int l = 0; l < kLW; ++l) {                                         \
                        if (!kNoMfma) acc[l][T] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, DQ[l][i], acc[l][T], 0, 0, 0); \
                        else acc[l][T] += a;                                                                  \
                    }                                                                                         \
                }                                                                                             \
            }                                                                                                 \
        }                                                                                                     \
    } while (0)
        for (int p = 0; p < passes; ++p) {
            const int c0 = p * cpp, cn = min(cpp, chunks - c0);
            v4i da[kLW][4], db[kLW][4];
            // units u = (chunk, half): chunk u / kHalves, half hh0 + u % kHalves
            const int un = cn * kHalves;
            LDS_SP_DIG(c0, hh0, da);  // before the barrier: in flight while pass p finishes streaming
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_s_barrier();  // pass p streamed
            const uint32_t* const bp = sp_lds + (p % 3) * bufdw;
            for (int u = 0; u < un; u += 2) {
                if (u + 1 < un) LDS_SP_DIG(c0 + (u + 1) / kHalves, hh0 + (u + 1) % kHalves, db);
                LDS_SP_MUL(u / kHalves, hh0 + u % kHalves, da);
                if (u + 1 >= un) break;
                if (u + 2 < un) LDS_SP_DIG(c0 + (u + 2) / kHalves, hh0 + (u + 2) % kHalves, da);
                LDS_SP_MUL((u + 1) / kHalves, hh0 + (u + 1) % kHalves, db);
            }
            // pass p done: the last multiply wave to finish with its buffer clears it
            // for pass p + 3 (whose spills start in pass p + 2, after the next barrier);
            // clearing it from every wave raced with the slower waves' reads
            __builtin_amdgcn_s_waitcnt(0xC07F);  // this wave's fragment reads of the buffer returned
            const int order = __builtin_amdgcn_readfirstlane(lane == 0 ? atomicAdd(done + p % 3, 1) : 0);
            if (order == 16 - NS - 1) {
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
    if (wave >= NS) {
        const int m = wave - NS, L0 = kLW * (m & 3);
        const int r16 = lane & 15, g = lane >> 4;
#pragma unroll
        for (int l = 0; l < kLW; ++l)
#pragma unroll
            for (int T = 0; T < kTiles; ++T)
                if (16 * T < nrows)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        atomicAdd(sums + (T * 16 + 4 * g + i) * kF + r16,
                                  (unsigned long long)((int64_t)acc[l][T][i] * ((int64_t)1 << (8 * (L0 + l)))));
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

}  // namespace lds_variants

using namespace lds_variants;

#define LDS_VAR_EXPORT extern "C" __attribute__((visibility("default")))

// Workspace of lds_variants_spmm_dense: lds_spmm_norm_dense's column maxima and
// digits (same carve), then the row-block kernel's bit slabs.
LDS_VAR_EXPORT int64_t lds_variants_ws_bytes(int n) {
    if (n <= 0) return 0;
    return dense_scratch_off(n) + rb_scratch_rows(n) * 64 * chunks_of(n);
}

static int variants_launch(const int* row_ptr, const int* col, const float* s, int n, const float* z, int ldz,
                           float* y, int ldy, int beta, void* ws, int grid, int quantize, int dbg, hipStream_t st);

// dbg: the variant codes of DESIGN.md §4g-4h (the round-4 lds_spmm_dense_ablation
// codes).  Same results as the product: 6 / 22 the row-block kernel (digits by
// register loads / LDS-DMA; any column order), 20 / 21 the column-pass kernel
// (concurrent / sequential), the spill-pass forms 23, 33-39, 41-57, 60-69
// (64 = the product's mode 17).  Timing-only ablations (wrong results): 1-5, 7,
// 8 (row-block phases), 11-13 (column-pass halves), 31 / 32 / 40 / 58 / 59
// (spill-pass without MFMAs / without bit setting / plain-store ORs).  The
// digits of s, z must be in ws (an lds_spmm_norm_dense call with the same
// s, z and a workspace of lds_variants_ws_bytes(n) bytes).
LDS_VAR_EXPORT int lds_variants_spmm_dense(const int* row_ptr, const int* col, const float* s, int n,
                                           const float* z, int ldz, float* y, int ldy, void* ws, int dbg,
                                           void* stream) {
    LDS_CHECK_ARG((dbg >= 1 && dbg <= 8) || (dbg >= 11 && dbg <= 13) || (dbg >= 20 && dbg <= 23) || (dbg >= 31 && dbg <= 69));
    return variants_launch(row_ptr, col, s, n, z, ldz, y, ldy, 0, ws, 0, 0, dbg, (hipStream_t)stream);
}

// The PRODUCT spill-pass kernel (lds-gnn_amd/csrc/spill.hpp, the code
// lds_spmm_norm_dense runs), built with a test delay: multiply wave 12 sleeps
// `delay` × 127 × 64 cycles after every pass barrier (delay 1 or 4), so it
// finishes each pass buffer last and the buffer clear must wait for it.  Exact
// sums (equal to the undelayed product) whatever the delay is the
// timing-independent check of the last-finisher clear.  err as in
// lds_spmm_norm_dense; the digits of s, z must be in ws.
LDS_VAR_EXPORT int lds_variants_spmm_dense_delayed(const int* row_ptr, const int* col, const float* s, int n,
                                                   float* y, int ldy, void* ws, int grid, int delay, uint32_t* err,
                                                   void* stream) {
    LDS_CHECK_ARG(row_ptr && col && s && y && ws && n > 0 && n <= kDnMaxChunks * kChunk && ldy >= kF);
    LDS_CHECK_ARG((((uintptr_t)col) & 15) == 0 && (((uintptr_t)ws) & 15) == 0);
    LDS_CHECK_ARG(delay == 1 || delay == 4);
    const Ws w = carve(ws, n);
    if (delay == 1) return lds::spill::sp_launch<1>(row_ptr, col, s, n, w, y, ldy, 0, grid, err, (hipStream_t)stream);
    return lds::spill::sp_launch<4>(row_ptr, col, s, n, w, y, ldy, 0, grid, err, (hipStream_t)stream);
}

static int variants_launch(const int* row_ptr, const int* col, const float* s, int n, const float* z, int ldz,
                             float* y, int ldy, int beta, void* ws, int grid, int quantize, int dbg, hipStream_t st) {
    LDS_CHECK_ARG(row_ptr && col && s && z && y && ws && n > 0 && n <= kDnMaxChunks * kChunk);
    LDS_CHECK_ARG(ldz >= kF && ldy >= kF);
    LDS_CHECK_ARG((((uintptr_t)col) & 15) == 0 && (((uintptr_t)ws) & 15) == 0);
    const Ws w = carve(ws, n);
    const int nc = chunks_of(n);
    (void)quantize;
    char* scratch = reinterpret_cast<char*>(ws) + dense_scratch_off(n);
    const int cus = device_cus();
    int g = grid > 0 ? grid : cus;
    const int gmin = (n + 16 * kRbMaxTiles - 1) / (16 * kRbMaxTiles);  // at most kRbMaxTiles tiles per block
    if (g < gmin) g = gmin;
    if (g > kRbMaxGrid) g = kRbMaxGrid;
    const int R = (n + g - 1) / g;
    LDS_CHECK_ARG(R <= 16 * kRbMaxTiles);
    g = (n + R - 1) / R;  // every block has rows
    const int tiles = (R + 15) / 16;
    // variant: 0 the column-pass kernel, 8 + 8 waves (a round-4 candidate); 1 the
    // same, 16 waves streaming then multiplying; 2 the row-block kernel with
    // bit slabs in global scratch.  dbg (ablations): rowblock 1-4, column-pass
    // (concurrent) 11 no multiply, 12 no streaming
    const int variant = dbg >= 30 ? 3 : dbg >= 20 ? dbg - 20 : dbg == 13 ? 1 : dbg >= 10 ? 0 : dbg > 0 ? 2
                                                                                                : 3;
    if (variant == 3) {  // the round-4 spill-pass kernels (dbg 64 = the round-4 product form) (sp_cfg)
        LDS_CHECK_ARG(R <= kSpMaxRows && g <= kSpMaxGrid);
        const SpCfg cfg = sp_cfg(dbg);
        const int depth = cfg.depth, ns = cfg.ns, slot = cfg.slot;
        const SpGeom sg = sp_geom(nc, tiles, depth, ns, slot);
        const int lds = sp_lds_bytes(tiles, sg, depth, ns, slot);
        LDS_CHECK_ARG(lds <= 163840 && sg.passes <= 576);  // (the row counters of mode 16 share the 576-int meta area)
#define LDS_SP_LAUNCH(TT, DP, DD) LDS_SP_LAUNCH_NS(TT, DP, DD, kSpStream)
#define LDS_SP_LAUNCH_NS(TT, DP, DD, NS)                                                                           \
    do {                                                                                                           \
        const hipError_t e = allow_lds(&csr_spill_agg_kernel<TT, DP, DD, NS>, lds);                                \
        if (e != hipSuccess) return (int)e;                                                                        \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(csr_spill_agg_kernel<TT, DP, DD, NS>), dim3(g), dim3(kSpThreads), lds,  \
                           st,                                                                                     \
                           row_ptr, col, n, R, (const int8_t*)w.zq, nc, sg.cpp, sg.passes, sg.rowdw,              \
                           (const uint32_t*)w.colmax, s, y, ldy, beta);                                           \
    } while (0)
        if (dbg == 0 && tiles <= 2) LDS_SP_LAUNCH_NS(2, kSpProdDepth, kSpProdMode, kSpProdWaves);
        else if (dbg == 0 && tiles <= 4) LDS_SP_LAUNCH_NS(4, kSpProdDepth, kSpProdMode, kSpProdWaves);
        else if (dbg == 0) LDS_SP_LAUNCH_NS(6, kSpProdDepth, kSpProdMode, kSpProdWaves);  // (5 tiles too: the
        // 6-tile build measured 170-171 µs at config 5 against 175-178 for a 5-tile build of the same code)
        else if (dbg == 31) LDS_SP_LAUNCH(6, kSpDepth, 1);
        else if (dbg == 32) LDS_SP_LAUNCH(6, kSpDepth, 2);
        else if (dbg == 35) LDS_SP_LAUNCH(6, kSpDepth, 3);
        else if (dbg == 36) LDS_SP_LAUNCH(6, kSpDepth, 4);
        else if (dbg == 37) LDS_SP_LAUNCH(6, kSpDepth, 5);
        else if (dbg == 38) LDS_SP_LAUNCH(6, 6, 5);
        else if (dbg == 39) LDS_SP_LAUNCH(6, kSpDepth, 6);
        else if (dbg == 40) LDS_SP_LAUNCH(6, kSpDepth, 7);
        else if (dbg == 41) LDS_SP_LAUNCH(6, kSpDepth, 8);
        else if (dbg == 42) LDS_SP_LAUNCH(6, 12, 8);
        else if (dbg == 43) LDS_SP_LAUNCH_NS(6, 5, 0, 12);
        else if (dbg == 44) LDS_SP_LAUNCH_NS(6, 6, 0, 12);
        else if (dbg == 45) LDS_SP_LAUNCH_NS(6, 4, 0, 12);
        else if (dbg == 46) LDS_SP_LAUNCH_NS(6, 5, 9, 12);
        else if (dbg == 47) LDS_SP_LAUNCH_NS(6, 3, 0, 12);
        else if (dbg == 48 && tiles <= 5) LDS_SP_LAUNCH_NS(5, 4, 0, 14);
        else if (dbg == 48) LDS_SP_LAUNCH_NS(6, 4, 0, 14);
        else if (dbg == 49 && tiles <= 5) LDS_SP_LAUNCH_NS(5, 3, 0, 14);
        else if (dbg == 49) LDS_SP_LAUNCH_NS(6, 3, 0, 14);
        else if (dbg == 50) LDS_SP_LAUNCH_NS(6, 4, 10, 12);
        else if (dbg == 51 && tiles <= 5) LDS_SP_LAUNCH_NS(5, 4, 10, 14);
        else if (dbg == 51) LDS_SP_LAUNCH_NS(6, 4, 10, 14);
        else if (dbg == 52) LDS_SP_LAUNCH_NS(6, 4, 11, 12);
        else if (dbg == 53) LDS_SP_LAUNCH_NS(6, 3, 11, 12);
        else if (dbg == 54) LDS_SP_LAUNCH_NS(6, 3, 12, 12);
        else if (dbg == 55) LDS_SP_LAUNCH_NS(6, 2, 12, 12);
        else if (dbg == 56) LDS_SP_LAUNCH_NS(6, 2, 12, 8);
        else if (dbg == 57 && tiles <= 5) LDS_SP_LAUNCH_NS(5, 2, 12, 14);
        else if (dbg == 57) LDS_SP_LAUNCH_NS(6, 2, 12, 14);
        else if (dbg == 58) LDS_SP_LAUNCH_NS(6, 2, 13, 12);
        else if (dbg == 59) LDS_SP_LAUNCH_NS(6, 2, 14, 12);
        else if (dbg == 60) LDS_SP_LAUNCH_NS(6, 3, 15, 12);
        else if (dbg == 61) LDS_SP_LAUNCH_NS(6, 4, 15, 12);
        else if (dbg == 62) LDS_SP_LAUNCH_NS(6, 6, 15, 12);
        else if (dbg == 63 && tiles <= 5) LDS_SP_LAUNCH_NS(5, 4, 16, 12);
        else if (dbg == 63) LDS_SP_LAUNCH_NS(6, 4, 16, 12);
        else if (dbg == 64) LDS_SP_LAUNCH_NS(6, 4, 17, 12);
        else if (dbg == 65) LDS_SP_LAUNCH_NS(6, 4, 18, 12);
        else if (dbg == 66) LDS_SP_LAUNCH_NS(6, 4, 19, 12);
        else if (dbg == 67 && tiles <= 5) LDS_SP_LAUNCH_NS(5, 4, 17, 14);
        else if (dbg == 67) LDS_SP_LAUNCH_NS(6, 4, 17, 14);
        else if (dbg == 68) LDS_SP_LAUNCH_NS(6, 3, 20, 12);
        else if (dbg == 69) LDS_SP_LAUNCH_NS(6, 4, 20, 12);
        else if (dbg == 33) LDS_SP_LAUNCH(6, 6, 0);
        else if (dbg == 34) LDS_SP_LAUNCH(6, 12, 0);
        else if (tiles <= 2) LDS_SP_LAUNCH(2, kSpDepth, 0);
        else if (tiles <= 4) LDS_SP_LAUNCH(4, kSpDepth, 0);
        else if (tiles <= 5) LDS_SP_LAUNCH(5, kSpDepth, 0);
        else LDS_SP_LAUNCH(6, kSpDepth, 0);
#undef LDS_SP_LAUNCH
#undef LDS_SP_LAUNCH_NS
        LDS_RETURN_LAST_ERROR();
    }
    if (variant == 2) {
        LDS_CHECK_ARG((int64_t)g * tiles * 16 <= rb_scratch_rows(n));
        uint32_t* slabs = reinterpret_cast<uint32_t*>(scratch);
#define LDS_RB_LAUNCH(TT, DD)                                                                                    \
    do {                                                                                                         \
        const int lds = rb_lds_bytes(nc, TT);                                                                    \
        const hipError_t e = allow_lds(&csr_rowblock_agg_kernel<TT, DD>, lds);                                   \
        if (e != hipSuccess) return (int)e;                                                                      \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(csr_rowblock_agg_kernel<TT, DD>), dim3(g), dim3(kRbThreads), lds, st,  \
                           row_ptr, col, n, R, (const int8_t*)w.zq, nc, (const uint32_t*)w.colmax, s, y, ldy,    \
                           beta, slabs);                                                                         \
    } while (0)
        if (dbg == 1) LDS_RB_LAUNCH(6, 1);
        else if (dbg == 2) LDS_RB_LAUNCH(6, 2);
        else if (dbg == 3) LDS_RB_LAUNCH(6, 3);
        else if (dbg == 4) LDS_RB_LAUNCH(6, 4);
        else if (dbg == 5) LDS_RB_LAUNCH(6, 5);
        else if (dbg == 6 && tiles <= 2) LDS_RB_LAUNCH(2, 6);
        else if (dbg == 6 && tiles <= 4) LDS_RB_LAUNCH(4, 6);
        else if (dbg == 6) LDS_RB_LAUNCH(6, 6);
        else if (dbg == 7) LDS_RB_LAUNCH(6, 7);
        else if (dbg == 8) LDS_RB_LAUNCH(6, 8);
        else if (dbg == 22 && tiles <= 2) LDS_RB_LAUNCH(2, 0);  // the LDS-staged multiply phase
        else if (dbg == 22 && tiles <= 4) LDS_RB_LAUNCH(4, 0);
        else if (dbg == 22) LDS_RB_LAUNCH(6, 0);
        else if (tiles <= 2) LDS_RB_LAUNCH(2, 6);  // dbg 6: digits by register loads (the round-4 row-block product)
        else if (tiles <= 4) LDS_RB_LAUNCH(4, 6);
        else LDS_RB_LAUNCH(6, 6);
#undef LDS_RB_LAUNCH
        LDS_RETURN_LAST_ERROR();
    }
    const bool conc = variant == 0;
    const int cd = dbg == 11 || dbg == 13 ? 1 : dbg == 12 ? 2 : 0;
    // chunks per pass: as many as the pass buffers hold next to the rings (LDS
    // 160 KB, ~2 KB of static arrays), evened out over the passes
    const int kt = tiles <= 2 ? 2 : tiles <= 3 ? 3 : tiles <= 4 ? 4 : tiles <= 5 ? 5 : 6;
    const int room = 163840 - 2048 - cp_fixed_lds(conc);
    int cmax = room / cp_buf_lds(conc, kt, 1);
    LDS_CHECK_ARG(cmax >= 1);
    const int passes = (nc + cmax - 1) / cmax;
    const int cpp = (nc + passes - 1) / passes;
    const int lds = cp_fixed_lds(conc) + cp_buf_lds(conc, kt, cpp);
#define LDS_CP_LAUNCH(TT, CC, DD)                                                                                 \
    do {                                                                                                          \
        const hipError_t e = allow_lds(&csr_colpass_agg_kernel<TT, CC, DD>, lds);                                 \
        if (e != hipSuccess) return (int)e;                                                                       \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(csr_colpass_agg_kernel<TT, CC, DD>), dim3(g), dim3(1024), lds, st,      \
                           row_ptr, col, n, R, (const int8_t*)w.zq, nc, cpp, (const uint32_t*)w.colmax, s, y, ldy, \
                           beta);                                                                                 \
    } while (0)
#define LDS_CP_TILES(CC, DD)                     \
    do {                                         \
        if (kt == 2) LDS_CP_LAUNCH(2, CC, DD);   \
        else if (kt == 3) LDS_CP_LAUNCH(3, CC, DD); \
        else if (kt == 4) LDS_CP_LAUNCH(4, CC, DD); \
        else if (kt == 5) LDS_CP_LAUNCH(5, CC, DD); \
        else LDS_CP_LAUNCH(6, CC, DD);           \
    } while (0)
    if (!conc && cd == 1) LDS_CP_LAUNCH(5, false, 1);
    else if (!conc) LDS_CP_TILES(false, 0);
    else if (cd == 1) LDS_CP_LAUNCH(5, true, 1);
    else if (cd == 2) LDS_CP_LAUNCH(5, true, 2);
    else LDS_CP_TILES(true, 0);
#undef LDS_CP_TILES
#undef LDS_CP_LAUNCH
    LDS_RETURN_LAST_ERROR();
}

// The product spill-pass kernel with its column stream loaded non-temporally
// (global_load_dwordx4 ... nt; round 6 A/B, tools/microbench/spmm_nt_ab.py).
// Operands as lds_spmm_norm_dense after its quantisation (ws holds the digits).
LDS_VAR_EXPORT int lds_variants_spmm_dense_nt(const int* row_ptr, const int* col, const float* s, int n, float* y,
                                              int ldy, void* ws, int grid, uint32_t* err, void* stream) {
    LDS_CHECK_ARG(row_ptr && col && s && y && ws && n > 0 && n <= kDnMaxChunks * kChunk && ldy >= kF);
    LDS_CHECK_ARG((((uintptr_t)col) & 15) == 0 && (((uintptr_t)ws) & 15) == 0);
    const Ws w = carve(ws, n);
    return lds::spill::sp_launch<0, true>(row_ptr, col, s, n, w, y, ldy, 0, grid, err, (hipStream_t)stream);
}
