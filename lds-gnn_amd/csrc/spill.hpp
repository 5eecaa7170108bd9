// The spill-pass CSR-SpMM for dense sampled graphs (the product of
// lds_spmm_norm_dense, bitagg.hip) and its launch: a header so that the
// tools-only variants library can build the same kernel with a test delay
// (kDelay) for the timing-independent buffer-clear test.
#pragma once

#include "bitagg.hpp"

// (own namespace: the tools-only variants library keeps the round-4 forms,
// with the same constant names, in lds_variants)
namespace lds {
namespace spill {

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

// kDelay (tests only, tools/variants: lds_variants_spmm_dense_delayed): multiply
// wave 12 sleeps kDelay × 127 × 64 cycles after each pass barrier, so it is
// the last to finish every buffer — the buffer-clear protocol (the last
// finisher clears) must still give exact sums, whatever the timing.
// kCheck (err != NULL): the windowed paths test every column and the error
// word is set as described above; without it (the caller guarantees
// ascending columns in [0, n), as for every CSR this library builds) they test
// a lane's first and last column only, as the round-4 product did.
// kNt (tools only): the column stream loaded with the non-temporal policy
template <int kTiles, bool kCheck, int kDelay = 0, bool kNt = false>
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
            if constexpr (kNt) rb_gload_nt(rg[J][h_], reinterpret_cast<const v4i*>(src_));                   \
            else rb_gload(rg[J][h_], reinterpret_cast<const v4i*>(src_));                                    \
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
            if (kCheck && a_ >= rlo_ && a_ + kStep <= rup_) { /* interior (uniform): every entry is the row's */       \
                const uint32_t w0_ = (uint32_t)(c_[0] - lo_) >> 5;                                           \
                const int base_ = lo_ + (int)(w0_ << 5);                                                     \
                uint32_t r_[kSpE];                                                                           \
                { /* all eight in [base, base + 64) and below the pass end */                                \
                    const uint32_t o_ = sp_offsets(c_, base_, r_);                                           \
                    fast_ = c_[0] >= lo_ && o_ < 64u && base_ + (int)o_ < hi_;                               \
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
                    {                                                                                        \
                        const uint32_t oq_ = sp_offsets(c_, qbase_, rq_);                                    \
                        pq_ = c_[0] >= hi_ && oq_ < 64u && qbase_ + (int)oq_ < hq_;                          \
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
            /* unchecked (ascending columns vouched for by the caller): the round-4 product's */            \
            /* expressions, verbatim — the same code the compiler scheduled at 164.8 µs (config 5) */        \
            if (!kCheck && a_ >= rlo_ && a_ + kStep <= rup_) {                                               \
                const uint32_t w0_ = (uint32_t)(c_[0] - lo_) >> 5;                                           \
                fast_ = c_[0] >= lo_ && c_[kSpE - 1] < hi_ && (uint32_t)(c_[kSpE - 1] - lo_) - (w0_ << 5) < 64u; \
                if (fast_) {                                                                                 \
                    uint64_t m_ = 0;                                                                         \
                    _Pragma("unroll") for (int e = 0; e < kSpE; ++e) m_ |= 1ull << ((uint32_t)(c_[e] - lo_) - (w0_ << 5)); \
                    dn_or(bp_ + w0_, (uint32_t)m_);                                                          \
                    dn_or(bp_ + w0_ + 1, (uint32_t)(m_ >> 32));                                              \
                }                                                                                            \
                if (!fast_) {                                                                                \
                    const uint32_t q0_ = (uint32_t)(c_[0] - hi_) >> 5;                                       \
                    if (c_[0] >= hi_ && c_[kSpE - 1] < hq_ && (uint32_t)(c_[kSpE - 1] - hi_) - (q0_ << 5) < 64u) { \
                        uint64_t m_ = 0;                                                                     \
                        _Pragma("unroll") for (int e = 0; e < kSpE; ++e) m_ |= 1ull << ((uint32_t)(c_[e] - hi_) - (q0_ << 5)); \
                        dn_or(bq_ + q0_, (uint32_t)m_);                                                      \
                        dn_or(bq_ + q0_ + 1, (uint32_t)(m_ >> 32));                                          \
                        spill_ = true;                                                                       \
                        fast_ = true;                                                                        \
                    }                                                                                        \
                }                                                                                            \
                if (!fast_ && c_[0] >= lo_ && c_[0] < hi_ && c_[kSpE - 1] >= hi_ && c_[kSpE - 1] < hq_ &&    \
                    (uint32_t)(c_[kSpE - 1] - hi_) < 64u) { /* straddles the boundary */                     \
                    uint64_t mp_ = 0, mq_ = 0;                                                               \
                    bool ok_ = true;                                                                         \
                    _Pragma("unroll") for (int e = 0; e < kSpE; ++e) {                                       \
                        const bool in_ = c_[e] < hi_;                                                        \
                        const uint32_t rr_ = in_ ? (uint32_t)(c_[e] - lo_) - (w0_ << 5) : (uint32_t)(c_[e] - hi_); \
                        ok_ = ok_ && rr_ < 64u;                                                              \
                        const uint64_t b_ = 1ull << (rr_ & 63u);                                             \
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
            }                                                                                                \
            if (!fast_) {                                                                                    \
                /* per entry; two copies under a uniform branch: only the array's last step reloads the */   \
                /* lanes that read the dummy (a lane-conditional load costs vmcnt(0) on every path) */       \
                if (a_ + kStep > nnz) {                                                                      \
                    _Pragma("unroll") for (int e = 0; e < kSpE; ++e) {                                       \
                        const int idx_ = i0_ + e;                                                            \
                        if (idx_ >= rlo_ && idx_ < rup_ &&                                                   \
                            sp_put((idx_ & ~3) + 4 > nnz ? (kCheck ? sp_ld(col + idx_) : col[idx_]) : c_[e], lo_, hi_, hq_, bp_, bq_, spill_, bad)) \
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
                            if (idx_ >= np_ && idx_ < rup_ && sp_put(kCheck ? sp_ld(col + idx_) : col[idx_], lo_, hi_, hq_, bp_, bq_, sp2_, bad)) \
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
        // checked build: every plain load of the prologue has landed before the
        // ring starts (the compiler's wait analysis does not see the ring's asm
        // loads, so a prologue load still counted as outstanding made it wait
        // vmcnt 1-2 wherever the ring later reused that load's registers); the
        // unchecked build keeps the round-4 product's code, which the compiler
        // schedules without those waits
        if constexpr (kCheck) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
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
            if constexpr (kDelay > 0) {  // test build only: limb 0 starts every pass last
                if (L == 0)
                    for (int d = 0; d < kDelay; ++d) __builtin_amdgcn_s_sleep(127);
            }
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

// Launch on grid g (0: one workgroup per CU; rows split evenly, at most
// kSpMaxRows per workgroup).  err != NULL: the checked form.
template <int kDelay, bool kNt = false>
inline int sp_launch(const int* row_ptr, const int* col, const float* s, int n, const Ws& w, float* y, int ldy,
                     int beta, int grid, uint32_t* err, hipStream_t st) {
    const int nc = chunks_of(n);
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
        const hipError_t e = allow_lds(&csr_spill_agg_kernel<TT, CK, kDelay, kNt>, lds);                       \
        if (e != hipSuccess) return (int)e;                                                                    \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(csr_spill_agg_kernel<TT, CK, kDelay, kNt>), dim3(g), dim3(kSpThreads), lds, st, \
                           row_ptr, col, n, R, (const int8_t*)w.zq, nc, sg.cpp, sg.passes, sg.rowdw,          \
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

}  // namespace spill
}  // namespace lds
