// Fused LDS bilevel engine: forward / backward / differentiable-Adam / reverse
// (hypergradient) kernels for the 2-layer GCN of src/models/gcn.py:23-34 on a
// sampled graph, written for 16-lane row groups (hidden width H = 16; class
// count C <= 16 padded to 16 columns).  Every per-node array is N × 16 fp32.
//
// Replaces, for the LDS configuration, the autograd machinery the reference
// runs per inner step (src/trainers/inner.py:55-74 with higher's
// DifferentiableAdam, create_graph=True) and per hyper step
// (src/trainers/outer.py:57-87: loss.backward through <= τ unrolled steps).
// The reverse pass is derived by hand; each aggregation's
// θ-gradient factor pair (s⊙G, s⊙Z) and r term is emitted by the epilogue of
// the kernel that has the pair in registers, so one rank-K update
// (lds_theta_grad) assembles the whole window's dθ.
//
// RNG counters, the Adam step and the outer learning rate are read from device
// memory (EngineScalars) so a whole τ-window is capturable as one HIP graph and
// replays advance them.
#include "common.hpp"
#include "fill.hpp"
#include "../../include/ldsgnn.h"

namespace lds {

constexpr int HID = 16;   // hidden width / row-group width
constexpr int RG = 256 / HID;  // row groups per 256-thread block

// Cross-lane moves on the VALU instead of the LDS crossbar (ds_bpermute, the
// lowering of __shfl / __shfl_xor: ~100 cycles per dependent hop).  A 16-lane
// row group is one DPP row: row_newbcast:K broadcasts lane K of the row,
// row_ror:R rotates it.  Sums / maxima over a row by rotations 8, 4, 2, 1 pair
// exactly the lanes the xor butterfly 8, 4, 2, 1 pairs (the partial sums are
// periodic), so results are bit-identical to the __shfl_xor form, in every
// lane.  Lanes L and L^16 / L^32 swap through v_permlane16/32_swap (gfx950).
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) { return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true); }
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) { return __int_as_float(dpp_i<CTRL>(__float_as_int(v))); }
template <int K>
__device__ __forceinline__ int rbc_i(int v) { return dpp_i<0x150 + K>(v); }  // row_newbcast:K
template <int K>
__device__ __forceinline__ float rbc_f(float v) { return dpp_f<0x150 + K>(v); }
#define LDS_R16(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)

__device__ __forceinline__ float gsum16(float v) {
    v += dpp_f<0x128>(v);  // row_ror:8
    v += dpp_f<0x124>(v);
    v += dpp_f<0x122>(v);
    v += dpp_f<0x121>(v);
    return v;
}
__device__ __forceinline__ float gmax16(float v) {
    v = fmaxf(v, dpp_f<0x128>(v));
    v = fmaxf(v, dpp_f<0x124>(v));
    v = fmaxf(v, dpp_f<0x122>(v));
    v = fmaxf(v, dpp_f<0x121>(v));
    return v;
}
// v + v of lane L^16, then + v of lane L^32 (the wave's four row groups summed,
// bit-identical to v += __shfl_xor(v, 16); v += __shfl_xor(v, 32))
__device__ __forceinline__ float xor16_add(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return v + __uint_as_float((threadIdx.x & 16) ? r[0] : r[1]);
}
__device__ __forceinline__ float xor32_add(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return v + __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
}
__device__ __forceinline__ float groups_sum(float v) { return xor32_add(xor16_add(v)); }
// argmax over the row's lanes (largest value, lowest lane on ties: torch.argmax)
__device__ __forceinline__ void argmax16_step(float& best, int& bi, float ob, int oi) {
    if (ob > best || (ob == best && oi < bi)) {
        best = ob;
        bi = oi;
    }
}
__device__ __forceinline__ int argmax16(float best, int bi) {
    argmax16_step(best, bi, dpp_f<0x128>(best), dpp_i<0x128>(bi));
    argmax16_step(best, bi, dpp_f<0x124>(best), dpp_i<0x124>(bi));
    argmax16_step(best, bi, dpp_f<0x122>(best), dpp_i<0x122>(bi));
    argmax16_step(best, bi, dpp_f<0x121>(best), dpp_i<0x121>(bi));
    return bi;
}
__device__ __forceinline__ float bcast16(float v, int src) { return __shfl(v, src, HID); }

// Device-resident scalars of an engine (one per replica).
struct EngineScalars {
    uint32_t graph_ctr;   // next graph draw counter
    uint32_t fwd_ctr;     // next training-forward counter
    int32_t adam_step;    // Adam steps taken so far (state['step'])
    int32_t hyper_steps;  // hyper steps taken so far
    double outer_lr;      // current SGD lr on θ (StepLR applied after each hyper step)
    double lr_decay;      // StepLR gamma (1.0 = none)
    uint32_t error;       // device error word (include/ldsgnn.h LDS_DEVERR_*): set by kernels, read by the host
    uint32_t pad;
};

struct Keys {
    uint32_t k0, k1, tag_x, tag_h;
};

// Per-sample element strides of a batched launch (include/ldsgnn.h LdsBatch):
// sample = blockIdx.y owns every per-sample array at base + sample·stride, its
// replica tags at tag + sample·tag.  A single-sample launch passes all zeros.
struct Batch {
    int64_t act, row, rp, col, ell2, par, xval, xd, uv, part, met;
    uint32_t tag;
    const int* heavy;       // row plan (include/ldsgnn.h LdsBatch)
    const uint8_t* hflag;
    int nh;
    int asplit;             // > 0: `agg` holds asplit partial n × 16 arrays (LdsBatch.agg_splits)
};

// kB = false (single-sample launch): no offset code at all.
template <bool kB, typename T>
__device__ __forceinline__ T* boff(T* p, int64_t stride) {
    if constexpr (!kB) return p;
    return p == nullptr ? p : p + (int64_t)blockIdx.y * stride;
}

template <bool kB>
__device__ __forceinline__ void bkeys(Keys& k, const Batch& bt) {
    if constexpr (kB) {
        k.tag_x += blockIdx.y * bt.tag;
        k.tag_h += blockIdx.y * bt.tag;
    }
}

// The same with the sample given (the row-plan kernels: plan_pos).
template <bool kB, typename T>
__device__ __forceinline__ T* boffs(int smp, T* p, int64_t stride) {
    if constexpr (!kB) return p;
    return p == nullptr ? p : p + (int64_t)smp * stride;
}
template <bool kB>
__device__ __forceinline__ void bkeys_s(int smp, Keys& k, const Batch& bt) {
    if constexpr (kB) {
        k.tag_x += smp * bt.tag;
        k.tag_h += smp * bt.tag;
    }
}

__device__ __forceinline__ float u_at(const Keys& k, uint32_t tag, uint32_t ctr, int row, int col) {
    const U32x4 o = philox4x32_10(U32x4{(uint32_t)col, (uint32_t)(row >> 2), tag, ctr}, k.k0, k.k1);
    const uint32_t w = (row & 3) == 0 ? o.x : (row & 3) == 1 ? o.y : (row & 3) == 2 ? o.z : o.w;
    return u01(w);
}

// Normalised aggregation of one 16-wide row, one wave per row:
// s_row Σ_j s_j Z[j][h].  The row's CSR entries are taken 64 at a time: lane
// t of a step loads entry beg + 64·step + t and its s_j, then 16-lane group g
// gathers the Z rows of the step's entries 16g..16g+15 (lane h: feature h);
// the four group partials combine by two xor-shuffles (fixed order), so every
// lane ends with feature h of the row.  A row of degree d costs 1 + 2·⌈d/64⌉
// dependent memory round trips.  A launch takes as long as its slowest row:
// with 16 lanes per row and chunks of 16 the kNN-initialised Cora θ₀ (degree
// up to 175) cost 8.8 µs per aggregation launch, one wave per row 4.2 µs, a
// trivial launch 1.75 µs (tools/microbench/aggbench.py; batching several steps'
// loads measured slower, 4.7 µs).  `ell` (the head {j, s_j} pairs) is unused
// on this path.
__device__ __forceinline__ float agg_row(const int* __restrict__ rp, const int* __restrict__ col,
                                         const float* __restrict__ s, const int2* __restrict__ ell,
                                         const float* __restrict__ z, int row, int lane) {
    (void)ell;
    (void)lane;
    const int t = threadIdx.x & 63;
    const int h = t & (HID - 1);
    const int beg = rp[row], end = rp[row + 1];
    float acc = 0.f;
    for (int p0 = beg; p0 < end; p0 += 64) {
        const int p = p0 + t;
        const int jl = p < end ? col[p] : row;
        const float sl = p < end ? s[jl] : 0.f;
        float zk[HID];
#define LDS_G(K) zk[K] = z[rbc_i<K>(jl) * HID + h];
        LDS_R16(LDS_G)
#undef LDS_G
#define LDS_F(K) acc = fmaf(rbc_f<K>(sl), zk[K], acc);
        LDS_R16(LDS_F)
#undef LDS_F
    }
    acc = groups_sum(acc);
    return s[row] * acc;
}

// ---------------------------------------------------------------------------
// Row plan of the aggregating kernels (include/ldsgnn.h LdsBatch): the first
// ceil(n / W) blocks give each row one wave (W waves per block); a row the
// plan marks heavy is skipped there and runs on a block of its own (logical
// blocks ceil(n / W) …), its W waves taking the row's entries 64 at a time,
// W·64 apart, their sums combined through LDS in wave order (every wave of the
// block ends with the row's value; wave 0 stores).  On the kNN-initialised
// Cora θ₀ the 17 rows of more than 64 entries (up to 175) otherwise set every
// launch's time: 4.3 -> 3.4 µs per aggregation launch
// (tools/microbench/aggbench.py).  The heavy blocks are the grid's FIRST
// physical blocks (plan_block): dispatched first, their longer walks start
// while the light blocks are still being dispatched.  Everything a block
// writes is indexed by its logical number, so the order changes no result.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int plan_block(int nlight, int nh) {
    const int p = (int)blockIdx.x;
    return p < nh ? nlight + p : p - nh;
}

// (sample, logical block) of a row-plan launch (grid nlight + nh by samples):
// sample blockIdx.y, heavy blocks first within it.  (Dispatching the heavy
// blocks of every sample ahead of all light blocks measured slower at S = 8:
// 0.279 against 0.271 ms per step.)
struct PlanPos {
    int smp, blk;
};
template <bool kB, int W>
__device__ __forceinline__ PlanPos plan_pos(int n, const Batch& bt) {
    return PlanPos{kB ? (int)blockIdx.y : 0, plan_block((n + W - 1) / W, bt.nh)};
}

struct RowSel {
    int row;          // -1: no row for this wave
    int first, end;   // this wave's first CSR entry, the row's end
    int step;         // entry stride between this wave's steps
    bool heavy;       // a heavy-row block (all its waves share the row)
    bool lead;        // this wave stores the row's results
    int blk;          // the logical block (plan_block)
    int2 e;           // light rows: this lane's ELL head entry {j, s_j}
};

// The ELL head, row_ptr and the plan flag of a light row load together (the
// head's address must not wait for the flag).
template <int W, bool kAgg>
__device__ __forceinline__ RowSel select_row(int blk, int n, const int* __restrict__ rp, const int2* __restrict__ ell,
                                             const Batch& bt) {
    RowSel r;
    r.e = make_int2(0, 0);
    const int wave = wave_id();
    const int nlight = (n + W - 1) / W;
    r.blk = blk;
    r.heavy = blk >= nlight;
    r.step = r.heavy ? 64 * W : 64;
    int row;
    if (r.heavy) {
        row = bt.heavy[blk - nlight];
    } else {
        row = blk * W + wave;
        if (row >= n) {
            r.row = -1;
            r.lead = false;
            r.first = r.end = 0;
            return r;
        }
    }
    if constexpr (!kAgg) {
        if (!r.heavy && ell != nullptr) r.e = ell[(int64_t)row * kEllWidth + (threadIdx.x & 63)];
        const int beg = rp[row];
        r.end = rp[row + 1];
        r.first = beg + (r.heavy ? wave * 64 : 0);
    } else {
        r.first = r.end = 0;
    }
    if (!r.heavy && bt.nh > 0 && bt.hflag[row]) row = -1;  // its own block aggregates it
    r.row = row;
    r.lead = row >= 0 && (!r.heavy || wave == 0);
    return r;
}

// s_row Σ_j s_j Z[j][h] of the selected row (feature h = lane % 16 in every
// lane), the heavy-block combine included; 0 for waves without a row.
// Light rows take their first 64 entries from the graph's ELL head ({j, s_j}
// pairs, padded with {row, 0}: a zero weight on a finite row), which needs no
// row_ptr: the head's load and the Z gathers are the row's only dependent
// round trips up to degree 64 (one fewer than through row_ptr -> col -> s / Z).
template <int W, bool kAgg>
__device__ __forceinline__ float agg_value(const RowSel& r, const int* __restrict__ col,
                                           const float* __restrict__ s, const int2* __restrict__ ell,
                                           const float* __restrict__ z, const float* __restrict__ agg,
                                           const Batch& bt, int n) {
    const int t = threadIdx.x & 63;
    const int h = t & (HID - 1);
    if constexpr (kAgg) {
        if (r.row < 0) return 0.f;
        if (bt.asplit > 0) {  // the bitmask aggregation's split partials: s_i · Σ_p part_p (p in order)
            float v[8];
            const int m = min(bt.asplit, 8);
#pragma unroll
            for (int p = 0; p < 8; ++p) v[p] = p < m ? agg[(int64_t)p * n * HID + r.row * HID + h] : 0.f;
            float a = 0.f;
#pragma unroll
            for (int p = 0; p < 8; ++p)
                if (p < m) a += v[p];
            for (int p = 8; p < bt.asplit; ++p) a += agg[(int64_t)p * n * HID + r.row * HID + h];
            return s[r.row] * a;
        }
        return agg[r.row * HID + h];
    } else {
        __shared__ float part[W][HID];
        float acc = 0.f;
        if (r.row >= 0) {
            int p0 = r.first;
            if (!r.heavy && ell != nullptr) {
                const int2 e = r.e;
                const float sl = __int_as_float(e.y);
                float zk[HID];
#define LDS_G(K) zk[K] = z[(rbc_i<K>(e.x) & kEllIndex) * HID + h];
                LDS_R16(LDS_G)
#undef LDS_G
#define LDS_F(K) acc = fmaf(rbc_f<K>(sl), zk[K], acc);
                LDS_R16(LDS_F)
#undef LDS_F
                p0 += kEllWidth;
            }
            for (; p0 < r.end; p0 += r.step) {
                const int p = p0 + t;
                const int jl = p < r.end ? col[p] : r.row;
                const float sl = p < r.end ? s[jl] : 0.f;
                float zk[HID];
#define LDS_G(K) zk[K] = z[rbc_i<K>(jl) * HID + h];
                LDS_R16(LDS_G)
#undef LDS_G
#define LDS_F(K) acc = fmaf(rbc_f<K>(sl), zk[K], acc);
                LDS_R16(LDS_F)
#undef LDS_F
            }
            acc = groups_sum(acc);
        }
        if (r.heavy) {  // block-uniform: every wave of the block reaches the barrier
            if (t < HID) part[threadIdx.x >> 6][t] = acc;
            __syncthreads();
            acc = part[0][h];
#pragma unroll
            for (int w = 1; w < W; ++w) acc += part[w][h];
        }
        return r.row >= 0 ? s[r.row] * acc : 0.f;
    }
}

// Write one factor pair (U = s⊙G, V = s⊙Z) into columns [off, off+width) of the
// window's factor matrices and add r = -½ s² (G·Y + Z·ÂG) into R[row].
__device__ __forceinline__ void emit_factor(float* __restrict__ U, float* __restrict__ V, int ldk,
                                            float* __restrict__ R, int off, int width, int row,
                                            int lane, float si, float g, float z, float y, float ag,
                                            bool assign = false) {
    const float d = gsum16(g * y + z * ag);
    if (lane < width) {
        put_uv(U, V, ldk, row, off + lane, si * g, si * z);
    }
    if (lane == 0) {
        const float r = -0.5f * si * si * d;
        R[row] = assign ? r : R[row] + r;
    }
}

// emit_factor with R[row] loaded beforehand (ahead of the aggregation)
__device__ __forceinline__ void emit_factor_pre(float* __restrict__ U, float* __restrict__ V, int ldk,
                                                float* __restrict__ R, float rprev, int off, int width, int row,
                                                int lane, float si, float g, float z, float y, float ag) {
    const float d = gsum16(g * y + z * ag);
    if (lane < width) {
        put_uv(U, V, ldk, row, off + lane, si * g, si * z);
    }
    if (lane == 0) R[row] = rprev + (-0.5f * si * si * d);
}

// ---------------------------------------------------------------------------
// X-side products (X is CSR / CSC, dropout keyed per (node, feature))
// ---------------------------------------------------------------------------

// One wave per X row (CSR) or X column (CSC): its entries are split over the
// wave's four 16-lane groups in chunks of 16 (group q takes chunks q, q+4, ...);
// per chunk one coalesced index/value load, dropout keyed per (node, feature)
// (optionally stored: xd_out in this order, xd_perm_out[perm[p]] in the other),
// then 16 independent row gathers of `src`; the groups' partials are combined
// by two xor-shuffles (fixed order).  Returns the full sum in every lane.
// x_wave_dot_range: the same over the entry range [beg, end) of row / column r.
template <bool kCsc>
__device__ __forceinline__ float x_wave_dot_range(int beg, int end, const int* __restrict__ idx,
                                                  const float* __restrict__ val, int r,
                                                  const float* __restrict__ src, const Keys& keys,
                                                  uint32_t ctr, int train, float keep, float scale,
                                                  float* __restrict__ xd_out = nullptr,
                                                  float* __restrict__ xd_perm_out = nullptr,
                                                  const int* __restrict__ perm = nullptr) {
    const int lane = threadIdx.x & (HID - 1);
    const int q = (threadIdx.x >> 4) & 3;
    float acc = 0.f;
    for (int p0 = beg + q * HID; p0 < end; p0 += 4 * HID) {
        const int p = p0 + lane;
        int j = 0;
        float x = 0.f;
        if (p < end) {
            j = idx[p];
            x = val[p];
            if (train) {
                const int node = kCsc ? j : r, feat = kCsc ? r : j;
                x = u_at(keys, keys.tag_x, ctr, node, feat) < keep ? x * scale : 0.f;
            }
            // keep Xd for the later products of this step (no redraw there)
            if (xd_out != nullptr) xd_out[p] = x;
            if (xd_perm_out != nullptr) xd_perm_out[perm[p]] = x;
        }
        float sk[HID];
#define LDS_G(K) sk[K] = src[rbc_i<K>(j) * HID + lane];
        LDS_R16(LDS_G)
#undef LDS_G
#define LDS_F(K) acc = fmaf(rbc_f<K>(x), sk[K], acc);
        LDS_R16(LDS_F)
#undef LDS_F
    }
    return groups_sum(acc);
}

// The same over a row / column described by its HEAD (the engine builds one
// per X, LdsEngine._x_heads): {p0, nnz} and the first 64 entries.  kHead 0:
// {index, value bits} pairs, X's own values used; 1: the same pairs, values
// from val[p0 + e] (e.g. the dropped Xd a training forward stored); 2: indices
// only (int), values from val.  The head replaces the
// dependent row-pointer load: entries and the gathers they index are the
// only round trips up to 64 entries; entries past 64 come from the CSR /
// CSC arrays as in x_wave_dot_range.
// kPre (kHead 2): the lane's head indices (entries e and 64 + e) were loaded by
// the caller (jpre, jpre2), ahead of the loads that give p0 / nnz; kPreP
// (kHead 0 / 1): the lane's head pair {index, value bits} likewise (jpre, jpre2).
template <bool kCsc, int kHead, bool kPre = false, bool kPreP = false>
__device__ __forceinline__ float x_wave_dot_head(int r, int p0, int nnz, const int* __restrict__ head,
                                                 const int* __restrict__ idx, const float* __restrict__ val,
                                                 const float* __restrict__ src, const Keys& keys, uint32_t ctr,
                                                 int train, float keep, float scale,
                                                 float* __restrict__ xd_out = nullptr,
                                                 float* __restrict__ xd_perm_out = nullptr,
                                                 const int* __restrict__ perm = nullptr, int jpre = 0, int jpre2 = 0) {
    static_assert(!kPre || kHead == 2, "a preloaded head index is an index-only head");
    static_assert(!kPreP || kHead != 2, "a preloaded head pair is a pair head");
    const int lane = threadIdx.x & (HID - 1);
    const int q = (threadIdx.x >> 4) & 3;
    float acc = 0.f;
    {
        const int e = 16 * q + lane;  // group q: head entries 16q .. 16q+15
        const bool v = e < nnz;
        int j;
        float x;
        if constexpr (kHead == 0) {
            const int2 hv = kPreP ? make_int2(jpre, jpre2) : reinterpret_cast<const int2*>(head)[e];
            j = hv.x;
            x = __int_as_float(hv.y);  // 0 past nnz
        } else if constexpr (kPreP) {
            j = jpre;
            x = v ? val[p0 + e] : 0.f;
        } else {
            j = kPre ? jpre : kHead == 1 ? reinterpret_cast<const int2*>(head)[e].x : head[e];
            x = v ? val[p0 + e] : 0.f;
        }
        if (v) {
            if (train) {
                const int node = kCsc ? j : r, feat = kCsc ? r : j;
                x = u_at(keys, keys.tag_x, ctr, node, feat) < keep ? x * scale : 0.f;
            }
            if (xd_out != nullptr) xd_out[p0 + e] = x;
            if (xd_perm_out != nullptr) xd_perm_out[perm[p0 + e]] = x;
        }
        if (16 * q < nnz) {  // group-uniform: chunks past the row's end are skipped
            float sk[HID];
#define LDS_G(K) sk[K] = src[rbc_i<K>(j) * HID + lane];
            LDS_R16(LDS_G)
#undef LDS_G
#define LDS_F(K) acc = fmaf(rbc_f<K>(x), sk[K], acc);
            LDS_R16(LDS_F)
#undef LDS_F
        }
    }
    const int end = p0 + nnz;
    int pstart = p0 + 64;
    if constexpr (kPre) {  // head entries 64..127 (jpre2): the same chunk order as the loop below
        const int e = 64 + 16 * q + lane;
        const bool v = e < nnz;
        float x = v ? val[p0 + e] : 0.f;
        if (v && train) x = u_at(keys, keys.tag_x, ctr, kCsc ? jpre2 : r, kCsc ? r : jpre2) < keep ? x * scale : 0.f;
        if (64 + 16 * q < nnz) {
            const int j = jpre2;
            float sk[HID];
#define LDS_G(K) sk[K] = src[rbc_i<K>(j) * HID + lane];
            LDS_R16(LDS_G)
#undef LDS_G
#define LDS_F(K) acc = fmaf(rbc_f<K>(x), sk[K], acc);
            LDS_R16(LDS_F)
#undef LDS_F
        }
        pstart = p0 + 128;
    }
    for (int pb = pstart + q * HID; pb < end; pb += 4 * HID) {
        const int p = pb + lane;
        int j = 0;
        float x = 0.f;
        if (p < end) {
            j = idx[p];
            x = val[p];
            if (train) {
                const int node = kCsc ? j : r, feat = kCsc ? r : j;
                x = u_at(keys, keys.tag_x, ctr, node, feat) < keep ? x * scale : 0.f;
            }
            if (xd_out != nullptr) xd_out[p] = x;
            if (xd_perm_out != nullptr) xd_perm_out[perm[p]] = x;
        }
        float sk[HID];
#define LDS_G(K) sk[K] = src[rbc_i<K>(j) * HID + lane];
        LDS_R16(LDS_G)
#undef LDS_G
#define LDS_F(K) acc = fmaf(rbc_f<K>(x), sk[K], acc);
        LDS_R16(LDS_F)
#undef LDS_F
    }
    return groups_sum(acc);
}

// x_wave_dot_head<true, 2> (train = 0) for TWO samples that share the
// column's indices: lanes 0-31 sample a, 32-63 sample b.  Group h (0 / 1) of
// a sample runs the chunk streams h and h + 2 of the one-sample walk, each in
// an accumulator of its own in the same entry order, and the streams are
// combined as groups_sum combines the four groups: (s0 + s1) + (s2 + s3) —
// the same bits as two one-sample walks.  The index loads of a and b are the
// same addresses in one instruction (one access), the value and row loads
// are the samples' own.
__device__ __forceinline__ float x_wave_dot_head_pair(int p0, int nnz, const int* __restrict__ head,
                                                      const int* __restrict__ idx, const float* __restrict__ val_a,
                                                      const float* __restrict__ val_b, const float* __restrict__ src_a,
                                                      const float* __restrict__ src_b) {
    const int lane = threadIdx.x & (HID - 1);
    const int grp = (threadIdx.x >> 4) & 3;
    const int h = grp & 1;
    const float* __restrict__ val = grp >= 2 ? val_b : val_a;
    const float* __restrict__ src = grp >= 2 ? src_b : src_a;
    float acc[2] = {0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int q = h + 2 * u;
        const int e = 16 * q + lane;
        const int j = head[e];
        const float x = e < nnz ? val[p0 + e] : 0.f;
        if (16 * q < nnz) {  // group-uniform, as in the one-sample walk
            float sk[HID];
#define LDS_G(K) sk[K] = src[rbc_i<K>(j) * HID + lane];
            LDS_R16(LDS_G)
#undef LDS_G
#define LDS_F(K) acc[u] = fmaf(rbc_f<K>(x), sk[K], acc[u]);
            LDS_R16(LDS_F)
#undef LDS_F
        }
    }
    const int end = p0 + nnz;
    for (int pb = p0 + 64 + h * HID; pb < end; pb += 4 * HID) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int pu = pb + 2 * HID * u;  // stream h + 2u: its chunk of this round
            if (pu < end) {
                const int p = pu + lane;
                int j = 0;
                float x = 0.f;
                if (p < end) {
                    j = idx[p];
                    x = val[p];
                }
                float sk[HID];
#define LDS_G(K) sk[K] = src[rbc_i<K>(j) * HID + lane];
                LDS_R16(LDS_G)
#undef LDS_G
#define LDS_F(K) acc[u] = fmaf(rbc_f<K>(x), sk[K], acc[u]);
                LDS_R16(LDS_F)
#undef LDS_F
            }
        }
    }
    return xor16_add(acc[0]) + xor16_add(acc[1]);
}

// A SHORT X column (at most 32 entries) on part of a wave: the column's
// 16-lane groups take its head entries 16·qc … 16·qc + 15 (qc = the group's
// place in the column: 0 for a column of a group, 0 / 1 for a column of two
// groups), exactly as groups qc of x_wave_dot_head<true, 2> do; the caller
// adds the groups of a two-group column with xor16_add.  Groups past a
// column's entries contribute nothing there either, so the sums are the same
// bits (up to the sign of a zero sum).  train = 0 (the stored Xd).
__device__ __forceinline__ float x_group_dot_head(int qc, int p0, int nnz, int j,
                                                  const float* __restrict__ val, const float* __restrict__ src) {
    const int lane = threadIdx.x & (HID - 1);
    float acc = 0.f;
    const int e = 16 * qc + lane;
    const float x = e < nnz ? val[p0 + e] : 0.f;
    if (16 * qc < nnz) {  // group-uniform
        float sk[HID];
#define LDS_G(K) sk[K] = src[rbc_i<K>(j) * HID + lane];
        LDS_R16(LDS_G)
#undef LDS_G
#define LDS_F(K) acc = fmaf(rbc_f<K>(x), sk[K], acc);
        LDS_R16(LDS_F)
#undef LDS_F
    }
    return acc;
}

template <bool kCsc>
__device__ __forceinline__ float x_wave_dot(const int* __restrict__ ptr, const int* __restrict__ idx,
                                            const float* __restrict__ val, int r,
                                            const float* __restrict__ src, const Keys& keys,
                                            uint32_t ctr, int train, float keep, float scale,
                                            float* __restrict__ xd_out = nullptr,
                                            float* __restrict__ xd_perm_out = nullptr,
                                            const int* __restrict__ perm = nullptr) {
    return x_wave_dot_range<kCsc>(ptr[r], ptr[r + 1], idx, val, r, src, keys, ctr, train, keep, scale, xd_out,
                                  xd_perm_out, perm);
}

// out[i][h] = bias[h] + Σ_f Xd[i][f] · Wt[f][h]      (H0 = Xd W0ᵀ + b0)
// Xd = dropout(X) with key (tag_x, fwd counter) when `train`, else X.
// (row block bx of replica sample smp)
template <bool kB>
__device__ __forceinline__ void x_linear_rows(int bx, int smp,
    const int* __restrict__ xrp, const int* __restrict__ xcol, const float* __restrict__ xval, int n,
    const float* __restrict__ wt, const float* __restrict__ bias, float* __restrict__ out, Keys keys,
    const EngineScalars* __restrict__ sc, int fwd_off, int train, float keep, float scale,
    float* __restrict__ xd_csr, float* __restrict__ xd_csc, const int* __restrict__ csr2csc,
    const int* __restrict__ xhead, const int2* __restrict__ xinfo, int head_vals, Batch bt) {
    const int row = bx * 4 + wave_id();
    if (row >= n) return;
    xval = boffs<kB>(smp, xval, bt.xval);
    wt = boffs<kB>(smp, wt, bt.par);
    bias = boffs<kB>(smp, bias, bt.par);
    out = boffs<kB>(smp, out, bt.act);
    xd_csr = boffs<kB>(smp, xd_csr, bt.xd);
    xd_csc = boffs<kB>(smp, xd_csc, bt.xd);
    bkeys_s<kB>(smp, keys, bt);
    const int lane = threadIdx.x & 63;
    const float bl = (bias != nullptr && lane < HID) ? bias[lane] : 0.f;
    const uint32_t ctr = sc->fwd_ctr + fwd_off;
    float acc;
    if (xhead != nullptr) {
        // the lane's head pair first: it does not wait for the row's info
        // (a scalar load the compiler waited for before issuing the head's)
        const int2 hv = reinterpret_cast<const int2*>(xhead + (int64_t)row * 128)[16 * ((threadIdx.x >> 4) & 3) + (threadIdx.x & (HID - 1))];
        const int2 inf = xinfo[row];  // {p0, nnz}
        if (head_vals)  // X's own values from the head (forward)
            acc = x_wave_dot_head<false, 0, false, true>(row, inf.x, inf.y, xhead + (int64_t)row * 128, xcol, xval,
                                                         wt, keys, ctr, train, keep, scale, xd_csr, xd_csc, csr2csc,
                                                         hv.x, hv.y);
        else            // values from xval (the Xd a training forward stored)
            acc = x_wave_dot_head<false, 1, false, true>(row, inf.x, inf.y, xhead + (int64_t)row * 128, xcol, xval,
                                                         wt, keys, ctr, train, keep, scale, xd_csr, xd_csc, csr2csc,
                                                         hv.x, hv.y);
    } else {
        acc = x_wave_dot<false>(xrp, xcol, xval, row, wt, keys, ctr, train, keep, scale, xd_csr, xd_csc, csr2csc);
    }
    if (lane < HID) out[row * HID + lane] = bl + acc;
}

template <bool kB>
__global__ __launch_bounds__(256) void x_linear_kernel(
    const int* __restrict__ xrp, const int* __restrict__ xcol, const float* __restrict__ xval, int n,
    const float* __restrict__ wt, const float* __restrict__ bias, float* __restrict__ out, Keys keys,
    const EngineScalars* __restrict__ sc, int fwd_off, int train, float keep, float scale,
    float* __restrict__ xd_csr, float* __restrict__ xd_csc, const int* __restrict__ csr2csc,
    const int* __restrict__ xhead, const int2* __restrict__ xinfo, int head_vals, Batch bt) {
    x_linear_rows<kB>(blockIdx.x, blockIdx.y, xrp, xcol, xval, n, wt, bias, out, keys, sc, fwd_off, train, keep,
                      scale, xd_csr, xd_csc, csr2csc, xhead, xinfo, head_vals, bt);
}

// A window's first launch with prefetched draws: the CSR / s / ELL fill of its
// graphs (fill.hpp; blocks [0, fill_blocks)) and the first inner step's
// dropout(X)·W0ᵀ (the rest), which does not read the graphs — one launch and
// one dependent boundary instead of two.  kB: the X product of every replica
// sample, sample-major after the fill blocks (one grid dimension, so no fill
// block is repeated per sample).
template <bool kB>
__global__ __launch_bounds__(256) void fill_x_linear_kernel(
    const uint64_t* __restrict__ bits, int words, const int* __restrict__ dacc, int wsi, int graphs,
    int* __restrict__ row_ptr, int* __restrict__ gcol, int64_t capacity, float* __restrict__ gs,
    int2* __restrict__ ell, const uint8_t* __restrict__ flags,
    const int* __restrict__ xrp, const int* __restrict__ xcol, const float* __restrict__ xval, int n,
    const float* __restrict__ wt, const float* __restrict__ bias, float* __restrict__ out, Keys keys,
    const EngineScalars* __restrict__ sc, int fwd_off, int train, float keep, float scale,
    float* __restrict__ xd_csr, float* __restrict__ xd_csc, const int* __restrict__ csr2csc,
    const int* __restrict__ xhead, const int2* __restrict__ xinfo, int head_vals, Batch bt,
    uint32_t* __restrict__ err) {
    const int fb = (n + 15) / 16;
    const int b = blockIdx.x;
    if (b < fb * graphs) {
        fill_csr_block(b % fb, b / fb, bits, n, words, dacc, wsi, row_ptr, gcol, capacity, gs, ell, flags, err);
        return;
    }
    const int xb = (n + 3) / 4, bx = b - fb * graphs;
    const int smp = kB ? bx / xb : 0;
    x_linear_rows<kB>(bx - smp * xb, smp, xrp, xcol, xval, n, wt, bias, out, keys, sc, fwd_off, train, keep, scale,
                      xd_csr, xd_csc, csr2csc, xhead, xinfo, head_vals, bt);
}

// out[f][h] (= or +=) Σ_i Xd[i][f] · D[i][h]  (+ wd · w[f][h])   via CSC of X.
__global__ __launch_bounds__(256) void xt_linear_kernel(
    const int* __restrict__ xcp, const int* __restrict__ xrow, const float* __restrict__ xval, int fin,
    const float* __restrict__ d, float* __restrict__ out, const float* __restrict__ w, float wd,
    int accumulate, Keys keys, const EngineScalars* __restrict__ sc, int fwd_off, int train, float keep,
    float scale) {
    const int lane = threadIdx.x & (HID - 1);
    const int f = (blockIdx.x * 256 + threadIdx.x) / HID;
    if (f >= fin) return;
    const uint32_t ctr = sc->fwd_ctr + fwd_off;
    float acc = 0.f;
    const int beg = xcp[f], end = xcp[f + 1];
    for (int p0 = beg; p0 < end; p0 += HID) {
        const int p = p0 + lane;
        int i = 0;
        float x = 0.f;
        if (p < end) {
            i = xrow[p];
            x = xval[p];
            if (train) x = u_at(keys, keys.tag_x, ctr, i, f) < keep ? x * scale : 0.f;
        }
        float dk[HID];
#define LDS_G(K) dk[K] = d[rbc_i<K>(i) * HID + lane];
        LDS_R16(LDS_G)
#undef LDS_G
#define LDS_F(K) acc = fmaf(rbc_f<K>(x), dk[K], acc);
        LDS_R16(LDS_F)
#undef LDS_F
    }
    float* o = out + f * HID + lane;
    if (w != nullptr) acc = acc + wd * w[f * HID + lane];
    *o = accumulate ? *o + acc : acc;
}

// ---------------------------------------------------------------------------
// Forward
// ---------------------------------------------------------------------------

struct GcnW {  // pointers into a flat parameter vector (layout in engine.py)
    const float* w0t;  // [fin][16]
    const float* b0;   // [16]
    const float* w1;   // [C][16]
    const float* b1;   // [C]
};

// Y0 = Â H0;  H1d = relu(Y0) ⊙ D1;  H2 = H1d W1ᵀ + b1  (16-padded, zeros past C)
template <bool kB, bool kAgg>
__global__ __launch_bounds__(256) void fwd_layer1_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, const float* __restrict__ s,
    const int2* __restrict__ ell, int n,
    const float* __restrict__ h0, float* __restrict__ y0, float* __restrict__ h1d, float* __restrict__ h2,
    GcnW w, int c, Keys keys, const EngineScalars* __restrict__ sc, int fwd_off, int train, float keep,
    float scale, float* __restrict__ dmask, const float* __restrict__ agg, Batch bt) {
    const PlanPos pp = plan_pos<kB, 4>(n, bt);
    const int lane = threadIdx.x & (HID - 1);
    const bool g0 = (threadIdx.x & 63) < HID;  // group 0 stores; groups 1-3 hold copies
    if constexpr (kAgg) agg = boffs<kB>(pp.smp, agg, bt.act);
    rp = boffs<kB>(pp.smp, rp, bt.rp);
    col = boffs<kB>(pp.smp, col, bt.col);
    s = boffs<kB>(pp.smp, s, bt.row);
    ell = boffs<kB>(pp.smp, ell, bt.ell2);
    h0 = boffs<kB>(pp.smp, h0, bt.act);
    y0 = boffs<kB>(pp.smp, y0, bt.act);
    h1d = boffs<kB>(pp.smp, h1d, bt.act);
    h2 = boffs<kB>(pp.smp, h2, bt.act);
    dmask = boffs<kB>(pp.smp, dmask, bt.act);
    w.w1 = boffs<kB>(pp.smp, w.w1, bt.par);
    w.b1 = boffs<kB>(pp.smp, w.b1, bt.par);
    bkeys_s<kB>(pp.smp, keys, bt);
    const RowSel rsel = select_row<4, kAgg>(pp.blk, n, rp, ell, bt);
    // the row's own operands (dropout draw, W1, b1) ahead of the aggregation
    float dk = 1.f, b1l = 0.f, w1v[HID];
    if (rsel.lead) {
        if (train) dk = u_at(keys, keys.tag_h, sc->fwd_ctr + fwd_off, rsel.row, lane) < keep ? scale : 0.f;
        b1l = lane < c ? w.b1[lane] : 0.f;
#pragma unroll
        for (int k = 0; k < HID; ++k) w1v[k] = k < c ? w.w1[k * HID + lane] : 0.f;
    }
    const float y = agg_value<4, kAgg>(rsel, col, s, ell, h0, agg, bt, n);
    if (!rsel.lead) return;
    const int row = rsel.row;
    float hd = fmaxf(y, 0.f);
    if (train) hd = dk != 0.f ? hd * scale : 0.f;
    if (g0) {
        y0[row * HID + lane] = y;
        h1d[row * HID + lane] = hd;
    }
    // D1 ⊙ [Y0 > 0] (× 1/keep): the mask every later product with this layer's
    // ReLU + dropout Jacobian reads instead of redrawing it
    if (dmask != nullptr && g0) dmask[row * HID + lane] = y > 0.f ? dk : 0.f;
    float out = 0.f;
#define LDS_W(K) if (K < c) { const float t = gsum16(hd * w1v[K]); if (lane == K) out = t + b1l; }
    LDS_R16(LDS_W)
#undef LDS_W
    if (g0) h2[row * HID + lane] = out;
}

// O = Â H2; P = softmax(O) (over c classes); dO = (P - onehot(y)) ⊙ m / |m|;
// per-row loss -log P[y] and correctness (argmax == y) where m.
template <bool kB, bool kAgg>
__global__ __launch_bounds__(256) void fwd_layer2_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, const float* __restrict__ s,
    const int2* __restrict__ ell, int n,
    const float* __restrict__ h2, float* __restrict__ o_out, float* __restrict__ p_out,
    float* __restrict__ d_o, const int* __restrict__ label, const uint8_t* __restrict__ mask,
    float inv_count, float* __restrict__ lossrow, float* __restrict__ corrrow, int c, const float* __restrict__ agg, Batch bt) {
    const PlanPos pp = plan_pos<kB, 4>(n, bt);
    const int lane = threadIdx.x & (HID - 1);
    const bool g0 = (threadIdx.x & 63) < HID;  // group 0 stores; groups 1-3 hold copies
    if constexpr (kAgg) agg = boffs<kB>(pp.smp, agg, bt.act);
    rp = boffs<kB>(pp.smp, rp, bt.rp);
    col = boffs<kB>(pp.smp, col, bt.col);
    s = boffs<kB>(pp.smp, s, bt.row);
    ell = boffs<kB>(pp.smp, ell, bt.ell2);
    h2 = boffs<kB>(pp.smp, h2, bt.act);
    o_out = boffs<kB>(pp.smp, o_out, bt.act);
    p_out = boffs<kB>(pp.smp, p_out, bt.act);
    d_o = boffs<kB>(pp.smp, d_o, bt.act);
    lossrow = boffs<kB>(pp.smp, lossrow, bt.row);
    corrrow = boffs<kB>(pp.smp, corrrow, bt.row);
    const RowSel rsel = select_row<4, kAgg>(pp.blk, n, rp, ell, bt);
    const float o = agg_value<4, kAgg>(rsel, col, s, ell, h2, agg, bt, n);
    if (!rsel.lead) return;
    const int row = rsel.row;
    const bool act = lane < c;
    const float m = gmax16(act ? o : -INFINITY);
    const float e = act ? expf(o - m) : 0.f;
    const float sum = gsum16(e);
    const float lse = logf(sum);
    const float logp = o - m - lse;
    const float p = act ? expf(logp) : 0.f;
    const int y = label[row];
    const bool sel = mask != nullptr && mask[row];
    if (o_out && g0) o_out[row * HID + lane] = act ? o : 0.f;
    if (p_out && g0) p_out[row * HID + lane] = p;
    if (d_o && g0) d_o[row * HID + lane] = (sel && act) ? (p - (lane == y ? 1.f : 0.f)) * inv_count : 0.f;
    // argmax with first-index tie-break (torch.argmax)
    const int bi = argmax16(act ? o : -INFINITY, lane);
    const float logpy = bcast16(logp, y);
    if (lane == 0 && g0) {
        lossrow[row] = sel ? -logpy : 0.f;
        corrrow[row] = (sel && bi == y) ? 1.f : 0.f;
    }
}

// ---------------------------------------------------------------------------
// Backward (first order)
// ---------------------------------------------------------------------------

// dH2 = Â dO;  dY0 = (dH2 W1) ⊙ D1 ⊙ [Y0 > 0].  Outer mode: emit factor (dO, H2).
template <bool kB, bool kAgg>
__global__ __launch_bounds__(256) void bwd_layer2_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, const float* __restrict__ s,
    const int2* __restrict__ ell, int n,
    const float* __restrict__ d_o, const float* __restrict__ y0, float* __restrict__ dh2,
    float* __restrict__ dy0, GcnW w, int c, Keys keys, const EngineScalars* __restrict__ sc, int fwd_off,
    int train, float keep, float scale, const float* __restrict__ o_in, const float* __restrict__ h2,
    float* __restrict__ U, float* __restrict__ V, int ldk, float* __restrict__ R, int foff, int fwidth,
    int r_assign, const float* __restrict__ dmask, const float* __restrict__ agg, Batch bt) {
    const PlanPos pp = plan_pos<kB, 4>(n, bt);
    const int lane = threadIdx.x & (HID - 1);
    const bool g0 = (threadIdx.x & 63) < HID;  // group 0 stores; groups 1-3 hold copies
    if constexpr (kAgg) agg = boffs<kB>(pp.smp, agg, bt.act);
    rp = boffs<kB>(pp.smp, rp, bt.rp);
    col = boffs<kB>(pp.smp, col, bt.col);
    s = boffs<kB>(pp.smp, s, bt.row);
    ell = boffs<kB>(pp.smp, ell, bt.ell2);
    d_o = boffs<kB>(pp.smp, d_o, bt.act);
    y0 = boffs<kB>(pp.smp, y0, bt.act);
    dh2 = boffs<kB>(pp.smp, dh2, bt.act);
    dy0 = boffs<kB>(pp.smp, dy0, bt.act);
    o_in = boffs<kB>(pp.smp, o_in, bt.act);
    h2 = boffs<kB>(pp.smp, h2, bt.act);
    dmask = boffs<kB>(pp.smp, dmask, bt.act);
    U = boffs<kB>(pp.smp, U, bt.uv);
    V = boffs<kB>(pp.smp, V, bt.uv);
    R = boffs<kB>(pp.smp, R, bt.row);
    w.w1 = boffs<kB>(pp.smp, w.w1, bt.par);
    bkeys_s<kB>(pp.smp, keys, bt);
    const RowSel rsel = select_row<4, kAgg>(pp.blk, n, rp, ell, bt);
    const float g2 = agg_value<4, kAgg>(rsel, col, s, ell, d_o, agg, bt, n);  // zero past c (dO is)
    if (!rsel.lead) return;
    const int row = rsel.row;
    if (g0) dh2[row * HID + lane] = g2;
    float dh1d = 0.f;
#define LDS_W(K) if (K < c) dh1d = fmaf(rbc_f<K>(g2), w.w1[K * HID + lane], dh1d);
    LDS_R16(LDS_W)
#undef LDS_W
    float mask;
    if (dmask != nullptr) {
        mask = dmask[row * HID + lane];
    } else {
        mask = y0[row * HID + lane] > 0.f ? 1.f : 0.f;
        if (train) mask = u_at(keys, keys.tag_h, sc->fwd_ctr + fwd_off, row, lane) < keep ? mask * scale : 0.f;
    }
    if (g0) dy0[row * HID + lane] = dh1d * mask;
    if (U != nullptr && g0)  // outer graph, use 2: G = dO, Z = H2, Y = O, ÂG = dH2
        emit_factor(U, V, ldk, R, foff, fwidth, row, lane, s[row], d_o[row * HID + lane],
                    h2[row * HID + lane], o_in[row * HID + lane], g2, r_assign != 0);
}

// dH0 = Â dY0.  Outer mode: emit factor (dY0, H0).
__global__ __launch_bounds__(256) void bwd_layer1_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, const float* __restrict__ s,
    const int2* __restrict__ ell, int n,
    const float* __restrict__ dy0, float* __restrict__ dh0, const float* __restrict__ y0,
    const float* __restrict__ h0, float* __restrict__ U, float* __restrict__ V, int ldk,
    float* __restrict__ R, int foff) {
    const int lane = threadIdx.x & (HID - 1);
    const int row = blockIdx.x * 4 + wave_id();  // one wave per row (agg_row)
    if (row >= n) return;
    const bool g0 = (threadIdx.x & 63) < HID;  // group 0 stores; groups 1-3 hold copies
    const float g = agg_row(rp, col, s, ell, dy0, row, lane);
    if (g0) dh0[row * HID + lane] = g;
    if (U != nullptr && g0)  // outer graph, use 1: G = dY0, Z = H0, Y = Y0, ÂG = dH0
        emit_factor(U, V, ldk, R, foff, HID, row, lane, s[row], dy0[row * HID + lane],
                    h0[row * HID + lane], y0[row * HID + lane], g);
}

// ---------------------------------------------------------------------------
// Column reductions over nodes (deterministic two-stage): per block partials of
//   A[c][h] = Σ_i (a1[i][c] b1[i][h] + a2[i][c] b2[i][h])   (c < c_n, h < 16)
//   v1[h]   = Σ_i x1[i][h],  v2[h] = Σ_i x2[i][h]
//   l0 = Σ_i l[i], l1 = Σ_i q[i]
// Layout of a partial: [A (16×16) | v1 (16) | v2 (16) | l0 | l1 | pad to 304].
// ---------------------------------------------------------------------------
constexpr int kRedLen = 16 * 16 + 16 + 16 + 16;  // 304 floats per partial
constexpr int kRedBlocks = 64;                      // max first-stage blocks

__global__ __launch_bounds__(256) void colreduce_kernel(
    int n, int c_n, const float* __restrict__ a1, const float* __restrict__ b1,
    const float* __restrict__ a2, const float* __restrict__ b2, const float* __restrict__ x1,
    const float* __restrict__ x2, const float* __restrict__ l, const float* __restrict__ q,
    float* __restrict__ partials, int rows_per_block) {
    __shared__ float red[RG][kRedLen];
    const int lane = threadIdx.x & (HID - 1);
    const int grp = threadIdx.x / HID;
    const int r0 = blockIdx.x * rows_per_block;
    const int r1 = min(n, r0 + rows_per_block);
    float acc[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = 0.f;
    float s1 = 0.f, s2 = 0.f, sl = 0.f, sq = 0.f;
    for (int i = r0 + grp; i < r1; i += RG) {
        const float bh1 = b1 ? b1[i * HID + lane] : 0.f;
        const float bh2 = b2 ? b2[i * HID + lane] : 0.f;
        const float av1 = a1 ? a1[i * HID + lane] : 0.f;
        const float av2 = a2 ? a2[i * HID + lane] : 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (k < c_n) {
                acc[k] = fmaf(bcast16(av1, k), bh1, acc[k]);
                acc[k] = fmaf(bcast16(av2, k), bh2, acc[k]);
            }
        }
        if (x1) s1 += x1[i * HID + lane];
        if (x2) s2 += x2[i * HID + lane];
        if (lane == 0) {
            if (l) sl += l[i];
            if (q) sq += q[i];
        }
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) red[grp][k * 16 + lane] = acc[k];
    red[grp][256 + lane] = s1;
    red[grp][272 + lane] = s2;
    if (lane >= 2) red[grp][288 + lane] = 0.f;
    if (lane == 0) {
        red[grp][288] = sl;
        red[grp][289] = sq;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < kRedLen; e += 256) {
        float t = 0.f;
        for (int g = 0; g < RG; ++g) t += red[g][e];
        partials[(int64_t)blockIdx.x * kRedLen + e] = t;
    }
}

// Sum the partials in block order; scatter into destinations (+= or =).
//   A -> dst_a[c][h] (c < c_n), v1 -> dst_v1[h], v2 -> dst_v2[c] (c < c_n
//   when v2_is_class else 16), l0 -> dst_l[0], l1 -> dst_l[1].
__global__ __launch_bounds__(320) void colreduce_final_kernel(
    const float* __restrict__ partials, int nblocks, int c_n, float* __restrict__ dst_a,
    float* __restrict__ dst_v1, int v1_width, float* __restrict__ dst_v2, int v2_width,
    float* __restrict__ dst_l, int accumulate) {
    const int e = threadIdx.x;
    if (e >= kRedLen) return;
    // all partial loads issued at once, then a fixed-shape tree sum (deterministic)
    float v[kRedBlocks];
#pragma unroll
    for (int b = 0; b < kRedBlocks; ++b) v[b] = b < nblocks ? partials[(int64_t)b * kRedLen + e] : 0.f;
#pragma unroll
    for (int w = kRedBlocks / 2; w > 0; w >>= 1)
#pragma unroll
        for (int b = 0; b < w; ++b) v[b] += v[b + w];
    const float t = v[0];
    float* dst = nullptr;
    if (e < 256) {
        const int k = e / 16;
        if (dst_a && k < c_n) dst = dst_a + e;
    } else if (e < 272) {
        if (dst_v1 && e - 256 < v1_width) dst = dst_v1 + (e - 256);
    } else if (e < 288) {
        if (dst_v2 && e - 272 < v2_width) dst = dst_v2 + (e - 272);
    } else if (e < 290) {
        if (dst_l) dst = dst_l + (e - 288);
    }
    if (dst) *dst = accumulate ? *dst + t : t;
}

// ---------------------------------------------------------------------------
// Differentiable Adam (higher's rule) forward and reverse, per parameter.
//   g' = g + wd·w (first n_wd entries);  m1 = β1 m0 + (1-β1) g';
//   v1 = β2 v0 + (1-β2) g'²;  w1 = w0 - (lr/bc1) m1 / (sqrt(v1)/sqrt(bc2) + eps)
// ---------------------------------------------------------------------------
struct AdamHyper {
    float lr, beta1, beta2, eps, wd;
    float omb1, omb2;  // float(1 - β) computed in double, as Python evaluates `1 - beta`
    int n_wd;          // parameters [0, n_wd) carry weight decay (group 0)
};

// bias corrections in double from the double β's, as Python computes them
__device__ __forceinline__ void adam_consts(const EngineScalars* sc, int step_off, const AdamHyper& hp,
                                            const double* betas, float& step_size, float& c2, int& step) {
    step = sc->adam_step + step_off + 1;
    const double bc1 = 1.0 - pow(betas[0], (double)step);
    const double bc2 = 1.0 - pow(betas[1], (double)step);
    step_size = (float)(betas[2] / bc1);
    c2 = (float)sqrt(bc2);
}

__global__ __launch_bounds__(256) void adam_fwd_kernel(
    int np, const float* __restrict__ w0, const float* __restrict__ g, const float* __restrict__ m0,
    const float* __restrict__ v0, float* __restrict__ w1, float* __restrict__ m1, float* __restrict__ v1,
    float* __restrict__ gp_out, AdamHyper hp, const double* __restrict__ betas,
    const EngineScalars* __restrict__ sc, int step_off) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= np) return;
    float step_size, c2;
    int step;
    adam_consts(sc, step_off, hp, betas, step_size, c2, step);
    const float w = w0[e];
    float gp = g[e];
    if (e < hp.n_wd && hp.wd != 0.f) gp = gp + hp.wd * w;
    const float m = m0[e] * hp.beta1 + hp.omb1 * gp;
    const float v = v0[e] * hp.beta2 + (hp.omb2 * gp) * gp;
    const float denom = sqrtf(v) / c2 + hp.eps;
    // torch CPU addcdiv: self + (value * t1) / t2
    w1[e] = w + ((-step_size) * m) / denom;
    m1[e] = m;
    v1[e] = v;
    if (gp_out) gp_out[e] = gp;
}

// Reverse of one Adam step.  In: wbar (adjoint of w1, updated in place to the
// adjoint of w0's direct + weight-decay paths), mbar/vbar (adjoints of m1/v1,
// updated in place to those of m0/v0), m1, v1, g' of the step.  Out: gbar
// (adjoint of the data gradient g — fed to the Hessian-vector reverse).
__global__ __launch_bounds__(256) void adam_rev_kernel(
    int np, float* __restrict__ wbar, float* __restrict__ mbar, float* __restrict__ vbar,
    const float* __restrict__ m1, const float* __restrict__ v1, const float* __restrict__ gp,
    float* __restrict__ gbar, AdamHyper hp, const double* __restrict__ betas,
    const EngineScalars* __restrict__ sc, int step_off) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= np) return;
    float step_size, c2;
    int step;
    adam_consts(sc, step_off, hp, betas, step_size, c2, step);
    const float wb = wbar[e];
    const float m = m1[e], v = v1[e], g = gp[e];
    const float sq = sqrtf(v);
    const float denom = sq / c2 + hp.eps;
    // w1 = w0 + (α m) / denom,  α = -step_size  (torch's addcdiv backward formulas)
    const float alpha = -step_size;
    const float mb = mbar[e] + wb * alpha / denom;            // total adjoint of m1
    const float db = -wb * alpha * m / (denom * denom);       // adjoint of denom
    float vb = vbar[e] + (db / c2) / (2.f * sq);               // sqrt backward: grad / (2 result)
    if (v == 0.f) vb = 0.f;  // higher's _maybe_mask hook on exp_avg_sq
    const float gb = hp.omb1 * mb + 2.f * (hp.omb2 * g) * vb;
    gbar[e] = gb;
    mbar[e] = hp.beta1 * mb;
    vbar[e] = hp.beta2 * vb;
    if (e < hp.n_wd && hp.wd != 0.f) wbar[e] = wb + hp.wd * gb;
}

// ---------------------------------------------------------------------------
// Reverse of the inner backward (Hessian-vector part), three aggregation
// kernels; see DESIGN.md §4 for the adjoint equations.
// ---------------------------------------------------------------------------

// dY0bar = Â dH0bar.  Factor use 4 (G = dH0bar, Z = dY0, Y = dH0, ÂG = dY0bar).
// dH1dbar = dY0bar ⊙ D1 ⊙ [Y0 > 0]
// dH2bar  = dH1dbar W1ᵀ + H1d ḡW1ᵀ + ḡb1
// H1dbar_part = dH2 ḡW1
template <bool kB, bool kAgg>
__global__ __launch_bounds__(256) void rev_a_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, const float* __restrict__ s,
    const int2* __restrict__ ell, int n,
    const float* __restrict__ dh0bar, const float* __restrict__ dy0, const float* __restrict__ dh0,
    const float* __restrict__ y0, const float* __restrict__ h1d, const float* __restrict__ dh2,
    GcnW w, const float* __restrict__ gw1bar, const float* __restrict__ gb1bar, int c,
    float* __restrict__ dh1dbar, float* __restrict__ dh2bar, float* __restrict__ h1dbar,
    Keys keys, const EngineScalars* __restrict__ sc, int fwd_off, int train, float keep, float scale,
    float* __restrict__ U, float* __restrict__ V, int ldk, float* __restrict__ R, int foff,
    const float* __restrict__ dmask, const float* __restrict__ agg, Batch bt) {
    const PlanPos pp = plan_pos<kB, 4>(n, bt);
    const int lane = threadIdx.x & (HID - 1);
    const bool g0 = (threadIdx.x & 63) < HID;  // group 0 stores; groups 1-3 hold copies
    if constexpr (kAgg) agg = boffs<kB>(pp.smp, agg, bt.act);
    rp = boffs<kB>(pp.smp, rp, bt.rp);
    col = boffs<kB>(pp.smp, col, bt.col);
    s = boffs<kB>(pp.smp, s, bt.row);
    ell = boffs<kB>(pp.smp, ell, bt.ell2);
    dh0bar = boffs<kB>(pp.smp, dh0bar, bt.act);
    dy0 = boffs<kB>(pp.smp, dy0, bt.act);
    dh0 = boffs<kB>(pp.smp, dh0, bt.act);
    y0 = boffs<kB>(pp.smp, y0, bt.act);
    h1d = boffs<kB>(pp.smp, h1d, bt.act);
    dh2 = boffs<kB>(pp.smp, dh2, bt.act);
    dh1dbar = boffs<kB>(pp.smp, dh1dbar, bt.act);
    dh2bar = boffs<kB>(pp.smp, dh2bar, bt.act);
    h1dbar = boffs<kB>(pp.smp, h1dbar, bt.act);
    dmask = boffs<kB>(pp.smp, dmask, bt.act);
    w.w1 = boffs<kB>(pp.smp, w.w1, bt.par);
    gw1bar = boffs<kB>(pp.smp, gw1bar, bt.par);
    gb1bar = boffs<kB>(pp.smp, gb1bar, bt.par);
    U = boffs<kB>(pp.smp, U, bt.uv);
    V = boffs<kB>(pp.smp, V, bt.uv);
    R = boffs<kB>(pp.smp, R, bt.row);
    bkeys_s<kB>(pp.smp, keys, bt);
    const RowSel rsel = select_row<4, kAgg>(pp.blk, n, rp, ell, bt);
    // the row's own operands ahead of the aggregation (their loads overlap it)
    const int row = rsel.row;
    const int ix = row * HID + lane;
    float si = 0.f, rprev = 0.f, o_dh0bar = 0.f, o_dy0 = 0.f, o_dh0 = 0.f, mask = 0.f, hd = 0.f, g2 = 0.f, gb1l = 0.f;
    float w1v[HID], gwv[HID];
    if (rsel.lead) {
        si = s[row];
        rprev = R[row];
        o_dh0bar = dh0bar[ix];
        o_dy0 = dy0[ix];
        o_dh0 = dh0[ix];
        if (dmask != nullptr) {
            mask = dmask[ix];
        } else {
            mask = y0[ix] > 0.f ? 1.f : 0.f;
            if (train) mask = u_at(keys, keys.tag_h, sc->fwd_ctr + fwd_off, row, lane) < keep ? mask * scale : 0.f;
        }
        hd = h1d[ix];
        g2 = dh2[ix];
        gb1l = lane < c ? gb1bar[lane] : 0.f;
#pragma unroll
        for (int k = 0; k < HID; ++k) {
            w1v[k] = k < c ? w.w1[k * HID + lane] : 0.f;
            gwv[k] = k < c ? gw1bar[k * HID + lane] : 0.f;
        }
    }
    const float ag = agg_value<4, kAgg>(rsel, col, s, ell, dh0bar, agg, bt, n);  // dY0bar
    if (!rsel.lead) return;
    if (g0) emit_factor_pre(U, V, ldk, R, rprev, foff, HID, row, lane, si, o_dh0bar, o_dy0, o_dh0, ag);
    const float a = ag * mask;  // dH1dbar
    if (g0) dh1dbar[ix] = a;
    float out = 0.f;
#define LDS_W(K) if (K < c) { const float t = gsum16(a * w1v[K] + hd * gwv[K]); if (lane == K) out = t + gb1l; }
    LDS_R16(LDS_W)
#undef LDS_W
    if (g0) dh2bar[ix] = out;
    float hb = 0.f;
#define LDS_W(K) if (K < c) hb = fmaf(rbc_f<K>(g2), gwv[K], hb);
    LDS_R16(LDS_W)
#undef LDS_W
    if (g0) h1dbar[ix] = hb;
}

// dObar = Â dH2bar.  Factor use 3 (G = dH2bar, Z = dO, Y = dH2, ÂG = dObar).
// Obar = P ⊙ (ū - P·ū), ū = dObar ⊙ m / |m|   (softmax Jacobian of dO = (P - E) m/|m|)
template <bool kB, bool kAgg>
__global__ __launch_bounds__(256) void rev_b_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, const float* __restrict__ s,
    const int2* __restrict__ ell, int n,
    const float* __restrict__ dh2bar, const float* __restrict__ d_o, const float* __restrict__ dh2,
    const float* __restrict__ p, const uint8_t* __restrict__ mask, float inv_count, int c,
    float* __restrict__ obar, float* __restrict__ U, float* __restrict__ V, int ldk,
    float* __restrict__ R, int foff, int cw, const float* __restrict__ agg, Batch bt) {
    const PlanPos pp = plan_pos<kB, 4>(n, bt);
    const int lane = threadIdx.x & (HID - 1);
    const bool g0 = (threadIdx.x & 63) < HID;  // group 0 stores; groups 1-3 hold copies
    if constexpr (kAgg) agg = boffs<kB>(pp.smp, agg, bt.act);
    rp = boffs<kB>(pp.smp, rp, bt.rp);
    col = boffs<kB>(pp.smp, col, bt.col);
    s = boffs<kB>(pp.smp, s, bt.row);
    ell = boffs<kB>(pp.smp, ell, bt.ell2);
    dh2bar = boffs<kB>(pp.smp, dh2bar, bt.act);
    d_o = boffs<kB>(pp.smp, d_o, bt.act);
    dh2 = boffs<kB>(pp.smp, dh2, bt.act);
    p = boffs<kB>(pp.smp, p, bt.act);
    obar = boffs<kB>(pp.smp, obar, bt.act);
    U = boffs<kB>(pp.smp, U, bt.uv);
    V = boffs<kB>(pp.smp, V, bt.uv);
    R = boffs<kB>(pp.smp, R, bt.row);
    const RowSel rsel = select_row<4, kAgg>(pp.blk, n, rp, ell, bt);
    const float ag = agg_value<4, kAgg>(rsel, col, s, ell, dh2bar, agg, bt, n);  // dObar
    if (!rsel.lead) return;
    const int row = rsel.row;
    const int ix = row * HID + lane;
    if (g0) emit_factor(U, V, ldk, R, foff, cw, row, lane, s[row], dh2bar[ix], d_o[ix], dh2[ix], ag);
    const bool sel = mask[row] != 0;
    const float ub = (sel && lane < c) ? ag * inv_count : 0.f;
    const float pv = p[ix];
    const float dot = gsum16(ub * pv);
    if (g0) obar[ix] = (lane < c) ? pv * (ub - dot) : 0.f;
}

// H2bar = Â Obar.  Factor use 2 (G = Obar, Z = H2, Y = O, ÂG = H2bar).
// H1dbar = H1dbar_part + H2bar W1;  Y0bar = H1dbar ⊙ D1 ⊙ [Y0 > 0]
template <bool kB, bool kAgg>
__global__ __launch_bounds__(256) void rev_c_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, const float* __restrict__ s,
    const int2* __restrict__ ell, int n,
    const float* __restrict__ obar, const float* __restrict__ h2, const float* __restrict__ o,
    const float* __restrict__ h1dbar_part, const float* __restrict__ y0, GcnW w, int c,
    float* __restrict__ h2bar, float* __restrict__ y0bar, Keys keys, const EngineScalars* __restrict__ sc,
    int fwd_off, int train, float keep, float scale, float* __restrict__ U, float* __restrict__ V,
    int ldk, float* __restrict__ R, int foff, int cw, const float* __restrict__ dmask, const float* __restrict__ agg, Batch bt) {
    const PlanPos pp = plan_pos<kB, 4>(n, bt);
    const int lane = threadIdx.x & (HID - 1);
    const bool g0 = (threadIdx.x & 63) < HID;  // group 0 stores; groups 1-3 hold copies
    if constexpr (kAgg) agg = boffs<kB>(pp.smp, agg, bt.act);
    rp = boffs<kB>(pp.smp, rp, bt.rp);
    col = boffs<kB>(pp.smp, col, bt.col);
    s = boffs<kB>(pp.smp, s, bt.row);
    ell = boffs<kB>(pp.smp, ell, bt.ell2);
    obar = boffs<kB>(pp.smp, obar, bt.act);
    h2 = boffs<kB>(pp.smp, h2, bt.act);
    o = boffs<kB>(pp.smp, o, bt.act);
    h1dbar_part = boffs<kB>(pp.smp, h1dbar_part, bt.act);
    y0 = boffs<kB>(pp.smp, y0, bt.act);
    h2bar = boffs<kB>(pp.smp, h2bar, bt.act);
    y0bar = boffs<kB>(pp.smp, y0bar, bt.act);
    dmask = boffs<kB>(pp.smp, dmask, bt.act);
    w.w1 = boffs<kB>(pp.smp, w.w1, bt.par);
    U = boffs<kB>(pp.smp, U, bt.uv);
    V = boffs<kB>(pp.smp, V, bt.uv);
    R = boffs<kB>(pp.smp, R, bt.row);
    bkeys_s<kB>(pp.smp, keys, bt);
    const RowSel rsel = select_row<4, kAgg>(pp.blk, n, rp, ell, bt);
    const float ag = agg_value<4, kAgg>(rsel, col, s, ell, obar, agg, bt, n);  // H2bar (zero past c)
    if (!rsel.lead) return;
    const int row = rsel.row;
    const int ix = row * HID + lane;
    if (g0) {
        emit_factor(U, V, ldk, R, foff, cw, row, lane, s[row], obar[ix], h2[ix], o[ix], ag);
        h2bar[ix] = ag;
    }
    float hb = h1dbar_part[ix];
#define LDS_W(K) if (K < c) hb = fmaf(rbc_f<K>(ag), w.w1[K * HID + lane], hb);
    LDS_R16(LDS_W)
#undef LDS_W
    float mask;
    if (dmask != nullptr) {
        mask = dmask[ix];
    } else {
        mask = y0[ix] > 0.f ? 1.f : 0.f;
        if (train) mask = u_at(keys, keys.tag_h, sc->fwd_ctr + fwd_off, row, lane) < keep ? mask * scale : 0.f;
    }
    if (g0) y0bar[ix] = hb * mask;
}

// H0bar = Â Y0bar.  Factor use 1 (G = Y0bar, Z = H0, Y = Y0, ÂG = H0bar).
__global__ __launch_bounds__(256) void rev_d_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, const float* __restrict__ s,
    const int2* __restrict__ ell, int n,
    const float* __restrict__ y0bar, const float* __restrict__ h0, const float* __restrict__ y0,
    float* __restrict__ h0bar, float* __restrict__ U, float* __restrict__ V, int ldk,
    float* __restrict__ R, int foff) {
    const int lane = threadIdx.x & (HID - 1);
    const int row = blockIdx.x * 4 + wave_id();  // one wave per row (agg_row)
    if (row >= n) return;
    const bool g0 = (threadIdx.x & 63) < HID;  // group 0 stores; groups 1-3 hold copies
    const int ix = row * HID + lane;
    const float ag = agg_row(rp, col, s, ell, y0bar, row, lane);
    if (g0) {
        emit_factor(U, V, ldk, R, foff, HID, row, lane, s[row], y0bar[ix], h0[ix], y0[ix], ag);
        h0bar[ix] = ag;
    }
}

// ---------------------------------------------------------------------------
// Two-hop forms: the loss layer and the aggregation of its gradient in one
// launch.  dO (and, in the reverse, Ōbar) is non-zero only on the rows of the
// loss mask M (train: 140 of Cora's 2708 nodes; opt: ~250), so
//   Â dO at row i = s_i Σ_{j ∈ N(i) ∩ M} s_j dO_j
// needs dO_j only at the few masked neighbours — and dO_j is a function of
// row j's own aggregation O_j = s_j Σ_{k ∈ N(j)} s_k H2_k.  Each wave walks
// its row's entries (ELL head: the neighbour's mask bits ride in the j field),
// ballots the masked ones and hands them out four at a time, one per 16-lane
// group; the group recomputes O_j (or dŌ_j) from row j's ELL head / CSR tail,
// applies the softmax (Jacobian) epilogue and accumulates s_j·(result).  The
// group that meets j = i itself stores row i's own outputs.  O_j is computed
// by one routine (group_agg, entries in CSR order) wherever it is needed, so
// every wave that recomputes it gets the bits row j stored.  This replaces
// the fwd_layer2 -> bwd_layer2 and rev_b -> rev_c launch pairs (one dependent
// boundary and one memory level each).
// ---------------------------------------------------------------------------

// s-weighted sum over row j's entries of z (16-lane group, lane h = feature h),
// in CSR order: the ELL head (all four 16-entry chunks' gathers issued before
// the first use: one memory level for degree <= 64), then the CSR tail 64
// entries at a time (indices, then s and the gathers: two levels per 64).
// The caller multiplies by s_j.
__device__ __forceinline__ float group_agg(int j, const int* __restrict__ rp, const int* __restrict__ col,
                                           const float* __restrict__ s, const int2* __restrict__ ell,
                                           const float* __restrict__ z) {
    const int t = threadIdx.x & 63;
    const int h = t & (HID - 1);
    const int beg = rp[j], end = rp[j + 1];
    const int2* __restrict__ eh = ell + (int64_t)j * kEllWidth;
    int2 e[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) e[q] = eh[16 * q + h];
    const int deg = end - beg;
    float acc = 0.f;
    {
        float zk[4][HID];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (16 * q < deg) {  // group-uniform; entries past deg are the head's {j, 0} padding
#define LDS_G(K) zk[q][K] = z[(rbc_i<K>(e[q].x) & kEllIndex) * HID + h];
                LDS_R16(LDS_G)
#undef LDS_G
            }
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (16 * q < deg) {
#define LDS_F(K) acc = fmaf(__int_as_float(rbc_i<K>(e[q].y)), zk[q][K], acc);
                LDS_R16(LDS_F)
#undef LDS_F
            }
    }
    for (int p0 = beg + kEllWidth; p0 < end; p0 += 4 * HID) {
        int kk[4];
        float sk[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int p = p0 + 16 * q + h;
            kk[q] = p < end ? col[p] : j;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) sk[q] = p0 + 16 * q + h < end ? s[kk[q]] : 0.f;
        float zk[4][HID];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (p0 + 16 * q < end) {
#define LDS_G(K) zk[q][K] = z[rbc_i<K>(kk[q]) * HID + h];
                LDS_R16(LDS_G)
#undef LDS_G
            }
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (p0 + 16 * q < end) {
#define LDS_F(K) acc = fmaf(rbc_f<K>(sk[q]), zk[q][K], acc);
                LDS_R16(LDS_F)
#undef LDS_F
            }
    }
    return acc;
}

// Walk the selected row's entries; for every masked neighbour j call f(j, s_j)
// in the 16-lane group it is handed to.  Picks go out in entry order, one per
// group per round: a light row's wave takes four per round; the W waves of a
// heavy-row block all walk the whole row (same ballots) and wave w's group g
// takes pick 4w + g of each round of 4W — the plan gives a block to rows with
// many masked neighbours, not only to long rows.  Uniform control flow: a
// group without a pick calls f with j = -1.
template <int W, class F>
__device__ __forceinline__ void for_masked(const RowSel& r, const int* __restrict__ col, const float* __restrict__ s,
                                           const uint8_t* __restrict__ nflag, int mbit, F&& f) {
    if (r.row < 0) return;
    const int t = threadIdx.x & 63;
    const int g = t >> 4;
    const int wave = wave_id();
    const int nw = r.heavy ? W : 1;                  // waves sharing the row
    const int slot = (r.heavy ? wave : 0) * 4 + g;   // this group's pick in each round
    const int beg = r.heavy ? r.first - 64 * wave : r.first;
    bool head = !r.heavy;
    int p0 = beg;
    for (;;) {
        int jl;
        float sl;
        bool ml;
        if (head) {
            jl = r.e.x & kEllIndex;
            sl = __int_as_float(r.e.y);
            ml = ((r.e.x >> kEllFlagShift) & mbit) != 0;
        } else {
            if (p0 >= r.end) break;
            const int p = p0 + t;
            const bool v = p < r.end;
            jl = v ? col[p] : 0;
            sl = v ? s[jl] : 0.f;
            ml = v && (nflag[jl] & mbit) != 0;
        }
        uint64_t ball = __ballot(ml);
        while (ball) {
            int mine = -1;
            for (int q = 0; q < 4 * nw; ++q) {
                if (ball) {
                    const int b = __ffsll((unsigned long long)ball) - 1;
                    ball &= ball - 1;
                    if (q == slot) mine = b;
                }
            }
            const int src = mine >= 0 ? mine : 0;
            const int j = __shfl(jl, src);
            const float sj = __shfl(sl, src);
            f(mine >= 0 ? j : -1, sj);
        }
        p0 += kEllWidth;
        head = false;
    }
}

// Sum a per-lane 16-vector over the four groups (fixed order), then over the
// W waves of a heavy-row block (LDS, wave order): every lane ends with the
// row's total for feature h.
template <int W, int NV>
__device__ __forceinline__ void combine_groups(const RowSel& r, float (&v)[NV]) {
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = groups_sum(v[k]);
    if (r.heavy) {  // block-uniform
        __shared__ float part[W][NV][HID];
        const int t = threadIdx.x & 63;
        if (t < HID)
#pragma unroll
            for (int k = 0; k < NV; ++k) part[threadIdx.x >> 6][k][t] = v[k];
        __syncthreads();
        const int h = t & (HID - 1);
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            float a = part[0][k][h];
#pragma unroll
            for (int w = 1; w < W; ++w) a += part[w][k][h];
            v[k] = a;
        }
    }
}

// U/V columns of one factor pair (emit_factor without the R update); returns
// this pair's r = -½ s² (G·Y + Z·ÂG) (every lane of the group).
__device__ __forceinline__ float emit_uv(float* __restrict__ U, float* __restrict__ V, int ldk, int off, int width,
                                         int row, int lane, float si, float g, float z, float y, float ag) {
    const float d = gsum16(g * y + z * ag);
    if (lane < width) {
        put_uv(U, V, ldk, row, off + lane, si * g, si * z);
    }
    return -0.5f * si * si * d;
}

// Softmax NLL epilogue of one row of O (16-lane group, lane h < c active):
// p, dO = (p - onehot(y)) / |M|, -log p_y, argmax == y.
struct LossRow {
    float p, d_o, nll, corr;
};
__device__ __forceinline__ LossRow loss_row(float o, int y, int c, float inv_count) {
    const int lane = threadIdx.x & (HID - 1);
    const bool act = lane < c;
    const float m = gmax16(act ? o : -INFINITY);
    const float e = act ? expf(o - m) : 0.f;
    const float sum = gsum16(e);
    const float lse = logf(sum);
    const float logp = o - m - lse;
    LossRow r;
    r.p = act ? expf(logp) : 0.f;
    r.d_o = act ? (r.p - (lane == y ? 1.f : 0.f)) * inv_count : 0.f;
    const int bi = argmax16(act ? o : -INFINITY, lane);
    r.nll = -bcast16(logp, y);
    r.corr = bi == y ? 1.f : 0.f;
    return r;
}

// fwd_layer2 + bwd_layer2 for a loss over the rows flagged `mbit`:
//   O = Â H2 (rows of M: o, p, dO, loss, correct stored; other rows zeros),
//   dH2 = Â dO;  dY0 = (dH2 W1) ⊙ D1 ⊙ [Y0 > 0];  outer mode: factor (dO, H2).
template <bool kB>
__global__ __launch_bounds__(256) void fwd2_bwd2_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, const float* __restrict__ s,
    const int2* __restrict__ ell, int n, const uint8_t* __restrict__ nflag, int mbit,
    const float* __restrict__ h2, float* __restrict__ o_out, float* __restrict__ p_out, float* __restrict__ d_o,
    const int* __restrict__ label, float inv_count, float* __restrict__ lossrow, float* __restrict__ corrrow,
    int c, const float* __restrict__ y0, float* __restrict__ dh2, float* __restrict__ dy0, GcnW w, Keys keys,
    const EngineScalars* __restrict__ sc, int fwd_off, int train, float keep, float scale,
    float* __restrict__ U, float* __restrict__ V, int ldk, float* __restrict__ R, int foff, int fwidth, int r_assign,
    const float* __restrict__ dmask, Batch bt) {
    const PlanPos pp = plan_pos<kB, 4>(n, bt);
    const int lane = threadIdx.x & (HID - 1);
    const bool g0 = (threadIdx.x & 63) < HID;
    rp = boffs<kB>(pp.smp, rp, bt.rp);
    col = boffs<kB>(pp.smp, col, bt.col);
    s = boffs<kB>(pp.smp, s, bt.row);
    ell = boffs<kB>(pp.smp, ell, bt.ell2);
    h2 = boffs<kB>(pp.smp, h2, bt.act);
    o_out = boffs<kB>(pp.smp, o_out, bt.act);
    p_out = boffs<kB>(pp.smp, p_out, bt.act);
    d_o = boffs<kB>(pp.smp, d_o, bt.act);
    lossrow = boffs<kB>(pp.smp, lossrow, bt.row);
    corrrow = boffs<kB>(pp.smp, corrrow, bt.row);
    y0 = boffs<kB>(pp.smp, y0, bt.act);
    dh2 = boffs<kB>(pp.smp, dh2, bt.act);
    dy0 = boffs<kB>(pp.smp, dy0, bt.act);
    dmask = boffs<kB>(pp.smp, dmask, bt.act);
    U = boffs<kB>(pp.smp, U, bt.uv);
    V = boffs<kB>(pp.smp, V, bt.uv);
    R = boffs<kB>(pp.smp, R, bt.row);
    w.w1 = boffs<kB>(pp.smp, w.w1, bt.par);
    bkeys_s<kB>(pp.smp, keys, bt);
    const RowSel rsel = select_row<4, false>(pp.blk, n, rp, ell, bt);
    const int row = rsel.row;
    // the lead's own-row operands, loaded ahead of the two-hop walk
    const int ix = row * HID + lane;
    float si = 0.f, mk = 0.f, h2i = 0.f, w1v[HID];
    bool in_mask = false;
    if (rsel.lead) {
        si = s[row];
        in_mask = (nflag[row] & mbit) != 0;
        mk = dmask != nullptr ? dmask[ix] : 0.f;
        h2i = U != nullptr ? h2[ix] : 0.f;
#pragma unroll
        for (int k = 0; k < HID; ++k) w1v[k] = k < c ? w.w1[k * HID + lane] : 0.f;
    }
    // v[0]: Σ s_j dO_j;  v[1], v[2]: row i's own dO_i, O_i (one contributor)
    float v[3] = {0.f, 0.f, 0.f};
    for_masked<4>(rsel, col, s, nflag, mbit, [&](int j, float sj) {
        if (j < 0) return;
        const int y = label[j];
        const float o = sj * group_agg(j, rp, col, s, ell, h2);
        const LossRow lr = loss_row(o, y, c, inv_count);
        v[0] = fmaf(sj, lr.d_o, v[0]);
        if (j == row) {
            const float ov = lane < c ? o : 0.f;
            v[1] = lr.d_o;
            v[2] = ov;
            o_out[j * HID + lane] = ov;
            p_out[j * HID + lane] = lr.p;
            d_o[j * HID + lane] = lr.d_o;
            if (lane == 0) {
                lossrow[j] = lr.nll;
                corrrow[j] = lr.corr;
            }
        }
    });
    combine_groups<4, 3>(rsel, v);
    if (!rsel.lead) return;
    if (g0 && !in_mask) {  // rows outside the mask: no loss, dO = 0
        o_out[ix] = 0.f;
        p_out[ix] = 0.f;
        d_o[ix] = 0.f;
        if (lane == 0) {
            lossrow[row] = 0.f;
            corrrow[row] = 0.f;
        }
    }
    const float g2 = si * v[0];
    if (g0) dh2[ix] = g2;
    float dh1d = 0.f;
#define LDS_W(K) if (K < c) dh1d = fmaf(rbc_f<K>(g2), w1v[K], dh1d);
    LDS_R16(LDS_W)
#undef LDS_W
    float mask;
    if (dmask != nullptr) {
        mask = mk;
    } else {
        mask = y0[ix] > 0.f ? 1.f : 0.f;
        if (train) mask = u_at(keys, keys.tag_h, sc->fwd_ctr + fwd_off, row, lane) < keep ? mask * scale : 0.f;
    }
    if (g0) dy0[ix] = dh1d * mask;
    if (U != nullptr && g0) {  // outer graph, use 2: G = dO, Z = H2, Y = O, ÂG = dH2
        const float r = emit_uv(U, V, ldk, foff, fwidth, row, lane, si, v[1], h2i, v[2], g2);
        if (lane == 0) R[row] = r_assign ? r : R[row] + r;
    }
}

// rev_b + rev_c (train mask):
//   dŌ = Â dH2bar (rows of M only), Ōbar = P ⊙ (ū - P·ū), ū = dŌ / |M|;
//   H2bar = Â Ōbar;  factor uses 3 (dH2bar, dO, dH2, dŌ) and 2 (Ōbar, H2, O, H2bar);
//   H1dbar = H1dbar_part + H2bar W1;  Y0bar = H1dbar ⊙ D1 ⊙ [Y0 > 0].
template <bool kB>
__global__ __launch_bounds__(256) void rev_bc_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, const float* __restrict__ s,
    const int2* __restrict__ ell, int n, const uint8_t* __restrict__ nflag, int mbit,
    const float* __restrict__ dh2bar, const float* __restrict__ d_o, const float* __restrict__ dh2,
    const float* __restrict__ p, const float* __restrict__ h2, const float* __restrict__ o, float inv_count, int c,
    const float* __restrict__ h1dbar_part, const float* __restrict__ y0, GcnW w, float* __restrict__ h2bar,
    float* __restrict__ y0bar, Keys keys, const EngineScalars* __restrict__ sc, int fwd_off, int train, float keep,
    float scale, float* __restrict__ U, float* __restrict__ V, int ldk, float* __restrict__ R, int foff_b,
    int foff_c, int cw, const float* __restrict__ dmask, Batch bt) {
    const PlanPos pp = plan_pos<kB, 4>(n, bt);
    const int lane = threadIdx.x & (HID - 1);
    const bool g0 = (threadIdx.x & 63) < HID;
    rp = boffs<kB>(pp.smp, rp, bt.rp);
    col = boffs<kB>(pp.smp, col, bt.col);
    s = boffs<kB>(pp.smp, s, bt.row);
    ell = boffs<kB>(pp.smp, ell, bt.ell2);
    dh2bar = boffs<kB>(pp.smp, dh2bar, bt.act);
    d_o = boffs<kB>(pp.smp, d_o, bt.act);
    dh2 = boffs<kB>(pp.smp, dh2, bt.act);
    p = boffs<kB>(pp.smp, p, bt.act);
    h2 = boffs<kB>(pp.smp, h2, bt.act);
    o = boffs<kB>(pp.smp, o, bt.act);
    h1dbar_part = boffs<kB>(pp.smp, h1dbar_part, bt.act);
    y0 = boffs<kB>(pp.smp, y0, bt.act);
    h2bar = boffs<kB>(pp.smp, h2bar, bt.act);
    y0bar = boffs<kB>(pp.smp, y0bar, bt.act);
    dmask = boffs<kB>(pp.smp, dmask, bt.act);
    U = boffs<kB>(pp.smp, U, bt.uv);
    V = boffs<kB>(pp.smp, V, bt.uv);
    R = boffs<kB>(pp.smp, R, bt.row);
    w.w1 = boffs<kB>(pp.smp, w.w1, bt.par);
    bkeys_s<kB>(pp.smp, keys, bt);
    const RowSel rsel = select_row<4, false>(pp.blk, n, rp, ell, bt);
    const int row = rsel.row;
    // the lead's own-row operands, loaded ahead of the two-hop walk
    const int ix = row * HID + lane;
    float si = 0.f, a_dh2bar = 0.f, a_do = 0.f, a_dh2 = 0.f, a_h2 = 0.f, a_o = 0.f, a_hb = 0.f, mk = 0.f;
    float w1v[HID];
    if (rsel.lead) {
        si = s[row];
        a_dh2bar = dh2bar[ix];
        a_do = d_o[ix];
        a_dh2 = dh2[ix];
        a_h2 = h2[ix];
        a_o = o[ix];
        a_hb = h1dbar_part[ix];
        mk = dmask != nullptr ? dmask[ix] : 0.f;
#pragma unroll
        for (int k = 0; k < HID; ++k) w1v[k] = k < c ? w.w1[k * HID + lane] : 0.f;
    }
    // v[0]: Σ s_j Ōbar_j;  v[1], v[2]: row i's own dŌ_i, Ōbar_i
    float v[3] = {0.f, 0.f, 0.f};
    for_masked<4>(rsel, col, s, nflag, mbit, [&](int j, float sj) {
        if (j < 0) return;
        const float pv = p[j * HID + lane];
        const float dob = sj * group_agg(j, rp, col, s, ell, dh2bar);
        const float ub = lane < c ? dob * inv_count : 0.f;
        const float dot = gsum16(ub * pv);
        const float ob = lane < c ? pv * (ub - dot) : 0.f;
        v[0] = fmaf(sj, ob, v[0]);
        if (j == row) {
            v[1] = dob;
            v[2] = ob;
        }
    });
    combine_groups<4, 3>(rsel, v);
    if (!rsel.lead) return;
    const float ag = si * v[0];  // H2bar (zero past c)
    if (g0) {
        // use 3: G = dH2bar, Z = dO, Y = dH2, ÂG = dŌ (dO = 0 off the mask);
        // use 2: G = Ōbar, Z = H2, Y = O, ÂG = H2bar — R += r3, then += r2 (rev_b, rev_c order)
        const float r3 = emit_uv(U, V, ldk, foff_b, cw, row, lane, si, a_dh2bar, a_do, a_dh2, v[1]);
        const float r2 = emit_uv(U, V, ldk, foff_c, cw, row, lane, si, v[2], a_h2, a_o, ag);
        if (lane == 0) R[row] = (R[row] + r3) + r2;
        h2bar[ix] = ag;
    }
    float hb = a_hb;
#define LDS_W(K) if (K < c) hb = fmaf(rbc_f<K>(ag), w1v[K], hb);
    LDS_R16(LDS_W)
#undef LDS_W
    float mask;
    if (dmask != nullptr) {
        mask = mk;
    } else {
        mask = y0[ix] > 0.f ? 1.f : 0.f;
        if (train) mask = u_at(keys, keys.tag_h, sc->fwd_ctr + fwd_off, row, lane) < keep ? mask * scale : 0.f;
    }
    if (g0) y0bar[ix] = hb * mask;
}

// ---------------------------------------------------------------------------
// Fused forms (fewer launches per window).
//   * the column reductions run in the epilogue of the aggregation that
//     produces their last input, one row per 16-lane group in 1024-thread
//     blocks (64 rows), reduced in-wave by xor-shuffles and across waves in
//     LDS into one partial per block (fixed order: deterministic);
//   * the final reduction applies the differentiable-Adam forward (inner
//     step) or reverse (hyper step) to b0 / W1 / b1, and xt_adam applies it
//     to W0 right where each W0 gradient / adjoint is completed.
// ---------------------------------------------------------------------------
// timing-only builds of the W0 products (tools/microbench/xt_parts.py); 0 in the product
#ifndef LDS_XT_EXPT
#define LDS_XT_EXPT 0
#endif

struct AdamArgs {
    // mode 1 (forward): w0, m0, v0 -> w1, m1, v1, gp
    // mode 2 (reverse of the step whose post-state is m1, v1 and whose g' is
    //         gp): wbar (in: complete adjoint of w1; out: + wd·ḡ), mbar, vbar
    //         (in/out; read as 0 when `first`), gbar (out)
    const float* w0;
    const float* m0;
    const float* v0;
    float* w1;
    float* m1;
    float* v1;
    float* gp;
    float* wbar;
    float* mbar;
    float* vbar;
    float* gbar;
    AdamHyper hp;
    const float* tab;  // Adam step table (refresh_adam_table): {step_size, c2} per step offset
    int step_off;
    int mode;
    int first;
};

// Operands of one parameter's Adam step, loaded ahead of the value they wait
// for (so their latency overlaps the reduction / product that completes it).
struct AdamOps {
    float p0, p1, p2, p3, p4;
};

__device__ __forceinline__ AdamOps adam_load(const AdamArgs& a, int idx) {
    AdamOps o{0.f, 0.f, 0.f, 0.f, 0.f};
    if (LDS_XT_EXPT == 9) return AdamOps{1.f, 1.f, 1.f, 0.5f, 0.5f};  // timing only: no operand loads
    if (a.mode == 1) {
        o.p0 = a.w0[idx];
        o.p1 = a.m0[idx];
        o.p2 = a.v0[idx];
    } else if (a.mode == 2) {
        o.p0 = a.m1[idx];
        o.p1 = a.v1[idx];
        o.p2 = a.gp[idx];
        if (!a.first) {
            o.p3 = a.mbar[idx];
            o.p4 = a.vbar[idx];
        }
    }
    return o;
}

// x: mode 1 the data gradient g; mode 2 the complete adjoint of w1.
__device__ __forceinline__ void adam_apply(const AdamArgs& a, int idx, float x, const AdamOps& o,
                                           float step_size, float c2) {
    if (LDS_XT_EXPT == 10) {  // timing only: the operands loaded, no update computed or stored
        float z = o.p0 + o.p1 + o.p2 + o.p3 + o.p4 + x * step_size * c2;
        asm volatile("" : "+v"(z));
        return;
    }
    if (a.mode == 1) {
        const float w = o.p0;
        float gp = x;
        if (idx < a.hp.n_wd && a.hp.wd != 0.f) gp = gp + a.hp.wd * w;
        const float m = o.p1 * a.hp.beta1 + a.hp.omb1 * gp;
        const float v = o.p2 * a.hp.beta2 + (a.hp.omb2 * gp) * gp;
        const float denom = sqrtf(v) / c2 + a.hp.eps;
        a.w1[idx] = w + ((-step_size) * m) / denom;
        if (LDS_XT_EXPT != 8) {  // (timing-only build 8: no m / v / g' stores)
            a.m1[idx] = m;
            a.v1[idx] = v;
            a.gp[idx] = gp;
        }
    } else if (a.mode == 2) {
        const float wb = x;
        const float m = o.p0, v = o.p1, g = o.p2;
        const float sq = sqrtf(v);
        const float denom = sq / c2 + a.hp.eps;
        const float alpha = -step_size;
        const float mb = o.p3 + wb * alpha / denom;
        const float db = -wb * alpha * m / (denom * denom);
        float vb = o.p4 + (db / c2) / (2.f * sq);
        if (v == 0.f) vb = 0.f;  // higher's _maybe_mask hook on exp_avg_sq
        const float gb = a.hp.omb1 * mb + 2.f * (a.hp.omb2 * g) * vb;
        a.gbar[idx] = gb;
        a.mbar[idx] = a.hp.beta1 * mb;
        a.vbar[idx] = a.hp.beta2 * vb;
        a.wbar[idx] = (idx < a.hp.n_wd && a.hp.wd != 0.f) ? wb + a.hp.wd * gb : wb;
    }
}

// {step_size, c2} = {0, 1} without an Adam step (mode 0: no table)
__device__ const float kAdamNoStep[2] = {0.f, 1.f};

// The step constants, loaded without a branch: with the load under `if
// (a.mode)` the compiler waited for it (lgkmcnt(0)) at the branch merge, right
// where it was issued — one more dependent round trip in front of every
// wave's product loads (xt_adam: 4.95 -> ... us per launch, tools/microbench/xt_parts.py).
__device__ __forceinline__ void adam_step_consts(const AdamArgs& a, const EngineScalars* __restrict__ sc,
                                                 float& step_size, float& c2) {
    (void)sc;
    const float* t = a.mode ? a.tab + 2 * a.step_off : kAdamNoStep;
    step_size = t[0];
    c2 = t[1];
}

// {step_size, c2} of the Adam steps adam_step + 1 + k, k < count (one thread
// each): the fp64 pow of the bias corrections runs once per window here
// instead of in every wave of every Adam-fused kernel.
__device__ __forceinline__ void refresh_adam_table(int adam_step, const double* __restrict__ betas,
                                                   float* __restrict__ tab, int count, int k) {
    if (k < count) {
        const int step = adam_step + k + 1;
        const double bc1 = 1.0 - pow(betas[0], (double)step);
        const double bc2 = 1.0 - pow(betas[1], (double)step);
        tab[2 * k] = (float)(betas[2] / bc1);
        tab[2 * k + 1] = (float)sqrt(bc2);
    }
}

constexpr int kRowsPer1K = 1024 / 64;  // rows per 1024-thread block, one wave per row
constexpr int kAdamTabMax = 256;  // step offsets covered by one Adam table

// One row per wave (its 16-vectors in lanes 0-15; `valid` false for waves
// without a row): the block's partial of
//   A[c][h] = Σ_rows av1[c] bh1[h] + av2[c] bh2[h]   (c < c_n)
//   v1[h] = Σ x1[h],  v2[h] = Σ x2[h],  l0 = Σ l,  l1 = Σ q
// (layout of colreduce_kernel).  The rows stage their vectors in LDS and
// thread e < kRedLen sums element e over the 16 rows in row order — no
// cross-lane broadcasts (the 16-lane-row form needed 64 shuffles per row).
__device__ __forceinline__ void block_reduce_1024(int c_n, bool valid, float av1, float bh1, float av2,
                                                  float bh2, float x1, float x2, float l, float q,
                                                  float* __restrict__ partials, int blk) {
    __shared__ float vec[16][6][HID];
    __shared__ float sca[16][2];
    const int lane = threadIdx.x & 63;
    const int wave = wave_id();
    if (lane < HID) {
        vec[wave][0][lane] = valid ? av1 : 0.f;
        vec[wave][1][lane] = valid ? bh1 : 0.f;
        vec[wave][2][lane] = valid ? av2 : 0.f;
        vec[wave][3][lane] = valid ? bh2 : 0.f;
        vec[wave][4][lane] = valid ? x1 : 0.f;
        vec[wave][5][lane] = valid ? x2 : 0.f;
        if (lane == 0) {
            sca[wave][0] = valid ? l : 0.f;
            sca[wave][1] = valid ? q : 0.f;
        }
    }
    __syncthreads();
    const int e = threadIdx.x;
    if (e >= kRedLen) return;
    float t = 0.f;
    if (e < 256) {
        const int c = e >> 4, h = e & (HID - 1);
        if (c < c_n) {
#pragma unroll
            for (int r = 0; r < 16; ++r) t += fmaf(vec[r][2][c], vec[r][3][h], vec[r][0][c] * vec[r][1][h]);
        }
    } else if (e < 288) {
        const int k = e < 272 ? 4 : 5, h = (e - 256) & (HID - 1);
#pragma unroll
        for (int r = 0; r < 16; ++r) t += vec[r][k][h];
    } else if (e < 290) {
#pragma unroll
        for (int r = 0; r < 16; ++r) t += sca[r][e - 288];
    }
    partials[(int64_t)blk * kRedLen + e] = t;
}

// dH0 = Â dY0 (+ outer factor (dY0, H0)); block partials of
// {gW1 = dH2ᵀ H1d, gb0 = Σ dH0, gb1 = Σ dH2, Σ loss, Σ correct}.
template <bool kB, bool kAgg>
__global__ __launch_bounds__(1024) void bwd1_reduce_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, const float* __restrict__ s,
    const int2* __restrict__ ell, int n,
    const float* __restrict__ dy0, float* __restrict__ dh0, const float* __restrict__ y0,
    const float* __restrict__ h0, float* __restrict__ U, float* __restrict__ V, int ldk,
    float* __restrict__ R, int foff, const float* __restrict__ dh2, const float* __restrict__ h1d,
    const float* __restrict__ lossrow, const float* __restrict__ corrrow, int c, float* __restrict__ partials,
    const float* __restrict__ agg, Batch bt) {
    const PlanPos pp = plan_pos<kB, 16>(n, bt);
    const int lane = threadIdx.x & (HID - 1);
    const bool g0 = (threadIdx.x & 63) < HID;  // group 0 stores and reduces; groups 1-3 hold copies
    if constexpr (kAgg) agg = boffs<kB>(pp.smp, agg, bt.act);
    rp = boffs<kB>(pp.smp, rp, bt.rp);
    col = boffs<kB>(pp.smp, col, bt.col);
    s = boffs<kB>(pp.smp, s, bt.row);
    ell = boffs<kB>(pp.smp, ell, bt.ell2);
    dy0 = boffs<kB>(pp.smp, dy0, bt.act);
    dh0 = boffs<kB>(pp.smp, dh0, bt.act);
    y0 = boffs<kB>(pp.smp, y0, bt.act);
    h0 = boffs<kB>(pp.smp, h0, bt.act);
    dh2 = boffs<kB>(pp.smp, dh2, bt.act);
    h1d = boffs<kB>(pp.smp, h1d, bt.act);
    lossrow = boffs<kB>(pp.smp, lossrow, bt.row);
    corrrow = boffs<kB>(pp.smp, corrrow, bt.row);
    partials = boffs<kB>(pp.smp, partials, bt.part);
    U = boffs<kB>(pp.smp, U, bt.uv);
    V = boffs<kB>(pp.smp, V, bt.uv);
    R = boffs<kB>(pp.smp, R, bt.row);
    const RowSel rsel = select_row<16, kAgg>(pp.blk, n, rp, ell, bt);
    const bool valid = rsel.lead;
    const int row = rsel.row;
    const int ix = row * HID + lane;
    // the row's own operands ahead of the aggregation
    float a1 = 0.f, b1 = 0.f, lr = 0.f, qr = 0.f, si = 0.f, rprev = 0.f, o_dy0 = 0.f, o_h0 = 0.f, o_y0 = 0.f;
    if (valid) {
        a1 = dh2[ix];
        b1 = h1d[ix];
        lr = lossrow[row];
        qr = corrrow[row];
        if (U != nullptr) {
            si = s[row];
            rprev = R[row];
            o_dy0 = dy0[ix];
            o_h0 = h0[ix];
            o_y0 = y0[ix];
        }
    }
    float g = agg_value<16, kAgg>(rsel, col, s, ell, dy0, agg, bt, n);
    if (valid && g0) dh0[ix] = g;
    if (U != nullptr && valid && g0)  // outer graph, use 1: G = dY0, Z = H0, Y = Y0, ÂG = dH0
        emit_factor_pre(U, V, ldk, R, rprev, foff, HID, row, lane, si, o_dy0, o_h0, o_y0, g);
    block_reduce_1024(c, valid && g0, a1, b1, 0.f, 0.f, g, a1, lr, qr, partials, rsel.blk);
}

// H0bar = Â Y0bar (+ factor use 1); block partials of
// {W̄1 += dH2ᵀ dH1dbar + H2barᵀ H1d, b̄0 += Σ H0bar, b̄1 += Σ H2bar}.
template <bool kB, bool kAgg>
__global__ __launch_bounds__(1024) void rev_d_reduce_kernel(
    const int* __restrict__ rp, const int* __restrict__ col, const float* __restrict__ s,
    const int2* __restrict__ ell, int n,
    const float* __restrict__ y0bar, const float* __restrict__ h0, const float* __restrict__ y0,
    float* __restrict__ h0bar, float* __restrict__ U, float* __restrict__ V, int ldk,
    float* __restrict__ R, int foff, const float* __restrict__ dh2, const float* __restrict__ dh1dbar,
    const float* __restrict__ h2bar, const float* __restrict__ h1d, int c, float* __restrict__ partials,
    const float* __restrict__ agg, Batch bt) {
    const PlanPos pp = plan_pos<kB, 16>(n, bt);
    const int lane = threadIdx.x & (HID - 1);
    const bool g0 = (threadIdx.x & 63) < HID;  // group 0 stores and reduces; groups 1-3 hold copies
    if constexpr (kAgg) agg = boffs<kB>(pp.smp, agg, bt.act);
    rp = boffs<kB>(pp.smp, rp, bt.rp);
    col = boffs<kB>(pp.smp, col, bt.col);
    s = boffs<kB>(pp.smp, s, bt.row);
    ell = boffs<kB>(pp.smp, ell, bt.ell2);
    y0bar = boffs<kB>(pp.smp, y0bar, bt.act);
    h0 = boffs<kB>(pp.smp, h0, bt.act);
    y0 = boffs<kB>(pp.smp, y0, bt.act);
    h0bar = boffs<kB>(pp.smp, h0bar, bt.act);
    dh2 = boffs<kB>(pp.smp, dh2, bt.act);
    dh1dbar = boffs<kB>(pp.smp, dh1dbar, bt.act);
    h2bar = boffs<kB>(pp.smp, h2bar, bt.act);
    h1d = boffs<kB>(pp.smp, h1d, bt.act);
    partials = boffs<kB>(pp.smp, partials, bt.part);
    U = boffs<kB>(pp.smp, U, bt.uv);
    V = boffs<kB>(pp.smp, V, bt.uv);
    R = boffs<kB>(pp.smp, R, bt.row);
    const RowSel rsel = select_row<16, kAgg>(pp.blk, n, rp, ell, bt);
    const bool valid = rsel.lead;
    const int row = rsel.row;
    const int ix = row * HID + lane;
    // the row's own operands ahead of the aggregation
    float a1 = 0.f, b1 = 0.f, a2 = 0.f, b2 = 0.f, si = 0.f, rprev = 0.f, o_y0bar = 0.f, o_h0 = 0.f, o_y0 = 0.f;
    if (valid) {
        a1 = dh2[ix];
        b1 = dh1dbar[ix];
        a2 = h2bar[ix];
        b2 = h1d[ix];
        si = s[row];
        rprev = R[row];
        o_y0bar = y0bar[ix];
        o_h0 = h0[ix];
        o_y0 = y0[ix];
    }
    const float ag = agg_value<16, kAgg>(rsel, col, s, ell, y0bar, agg, bt, n);
    if (valid && g0) {
        emit_factor_pre(U, V, ldk, R, rprev, foff, HID, row, lane, si, o_y0bar, o_h0, o_y0, ag);
        h0bar[ix] = ag;
    }
    block_reduce_1024(c, valid && g0, a1, b1, a2, b2, ag, a2, 0.f, 0.f, partials, rsel.blk);
}

// Sum the block partials (fixed order) into the flat parameter-shaped buffer
// `dst` (W1 at off_w1, b0 at off_b0, b1 at off_b1; = or +=), Σ loss / Σ correct
// into metrics[0..1], then Adam (mode 1 forward / mode 2 reverse) on those
// parameters.  Element e of a partial (layout of colreduce_kernel).
struct FinalArgs {
    const float* partials;
    int nblocks, c, off_b0, off_w1, off_b1, accumulate;
    float* dst;
    float* metrics;
};

// Parameter index of partial element e (-1: none; -2 / -3: Σ loss / Σ correct).
__device__ __forceinline__ int final_index(const FinalArgs& f, int e) {
    if (e < 256) return (e >> 4) < f.c ? f.off_w1 + e : -1;
    if (e < 272) return f.off_b0 + (e - 256);
    if (e < 288) return e - 272 < f.c ? f.off_b1 + (e - 272) : -1;
    if (e < 290) return -2 - (e - 288);
    return -1;
}

__device__ __forceinline__ float final_sum(const FinalArgs& f, int e) {
    float t = 0.f;
    for (int b0 = 0; b0 < f.nblocks; b0 += kRedBlocks) {
        float v[kRedBlocks];
#pragma unroll
        for (int b = 0; b < kRedBlocks; ++b)
            v[b] = b0 + b < f.nblocks ? f.partials[(int64_t)(b0 + b) * kRedLen + e] : 0.f;
#pragma unroll
        for (int w = kRedBlocks / 2; w > 0; w >>= 1)
#pragma unroll
            for (int b = 0; b < w; ++b) v[b] += v[b + w];
        t += v[0];
    }
    return t;
}

// Final stage for up to two partial elements per thread (e1 < 0: none): all
// loads (Adam operands, dst, partials) are issued before the sums complete.
__device__ __forceinline__ void final_pair(const FinalArgs& f, int e0, int e1, const AdamArgs& adam,
                                           const EngineScalars* __restrict__ sc) {
    const int i0 = final_index(f, e0);
    const int i1 = e1 >= 0 ? final_index(f, e1) : -1;
    AdamOps o0{0.f, 0.f, 0.f, 0.f, 0.f}, o1{0.f, 0.f, 0.f, 0.f, 0.f};
    float d0 = 0.f, d1 = 0.f;
    if (i0 >= 0) {
        o0 = adam_load(adam, i0);
        if (f.accumulate) d0 = f.dst[i0];
    }
    if (i1 >= 0) {
        o1 = adam_load(adam, i1);
        if (f.accumulate) d1 = f.dst[i1];
    }
    float step_size, c2;
    adam_step_consts(adam, sc, step_size, c2);
    const float t0 = final_sum(f, e0);
    const float t1 = e1 >= 0 ? final_sum(f, e1) : 0.f;
    if (i0 >= 0) {
        const float val = f.accumulate ? d0 + t0 : t0;
        f.dst[i0] = val;
        adam_apply(adam, i0, val, o0, step_size, c2);
    } else if (i0 <= -2 && f.metrics) {
        f.metrics[-2 - i0] = t0;
    }
    if (i1 >= 0) {
        const float val = f.accumulate ? d1 + t1 : t1;
        f.dst[i1] = val;
        adam_apply(adam, i1, val, o1, step_size, c2);
    } else if (i1 <= -2 && f.metrics) {
        f.metrics[-2 - i1] = t1;
    }
}

// The final stage in a 1024-thread block: three threads per partial element,
// each summing a third of the first-stage blocks (in order), the thirds then
// added in order through LDS; thread e < kRedLen completes element e (as
// final_pair: dst, metrics, Adam).  With one wave per row the fused
// reductions write ⌈n/16⌉ (+ heavy rows) partials, 187 at Cora.  A third is
// summed as consecutive groups of 16 partials (a fixed pairwise tree each),
// accumulated in order; kBatch (16 or 64) is how many are loaded per round
// trip — the same sums either way.  The single-sample launch loads 64 at once
// (its final block is on the critical path); the batched one 16, which keeps
// xt_adam at 40 VGPRs instead of 86 (two 1024-thread blocks per CU, not one).
//
// The final stage runs as kFinParts such blocks, part p completing elements
// [p·kFinPer, (p + 1)·kFinPer): the same sums per element, an eighth of the
// 63-partial loads per block (one block issued ≈900 wave loads of 256 B, a
// TA-bound ≈1.4 µs on one CU; 4 parts 4.57, 8 parts 4.50, 16 parts 4.55-4.59
// µs per xt_adam launch).
constexpr int kFinParts = 8;
constexpr int kFinPer = (kRedLen + kFinParts - 1) / kFinParts;
template <int kBatch>
__device__ __forceinline__ void final_block_1024(const FinalArgs& f, const AdamArgs& adam,
                                                 const EngineScalars* __restrict__ sc, int part) {
    static_assert(kBatch % 16 == 0 && kBatch <= kRedBlocks, "groups of 16");
    static_assert(3 * kFinPer <= 1024, "three thirds per element in one block");
    __shared__ float third[3][kFinPer];
    const int t = threadIdx.x;
    const int q = t / kFinPer, el = t - q * kFinPer;
    const int e0 = part * kFinPer, e1 = min(kRedLen, e0 + kFinPer);
    const int e = e0 + el;
    float step_size, c2;
    adam_step_consts(adam, sc, step_size, c2);
    // the completing thread's Adam operands first (they overlap the sums)
    const int idx = t < kFinPer && e0 + t < e1 ? final_index(f, e0 + t) : -1;
    AdamOps o{0.f, 0.f, 0.f, 0.f, 0.f};
    float prev = 0.f;
    if (idx >= 0) {
        o = adam_load(adam, idx);
        if (f.accumulate) prev = f.dst[idx];
    }
    if (q < 3 && e < e1) {
        const int per = (f.nblocks + 2) / 3;
        const int b0 = q * per, b1 = min(f.nblocks, b0 + per);
        float v = 0.f;
        for (int c0 = b0; c0 < b1; c0 += kBatch) {
            float x[kBatch];
#pragma unroll
            for (int b = 0; b < kBatch; ++b)
                x[b] = c0 + b < b1 ? f.partials[(int64_t)(c0 + b) * kRedLen + e] : 0.f;
#pragma unroll
            for (int g = 0; g < kBatch / 16; ++g) {
                float* y = x + 16 * g;
#pragma unroll
                for (int w = 8; w > 0; w >>= 1)
#pragma unroll
                    for (int b = 0; b < w; ++b) y[b] += y[b + w];
                v += y[0];
            }
        }
        third[q][el] = v;
    }
    __syncthreads();
    if (t >= kFinPer || e0 + t >= e1) return;
    const float tot = (third[0][t] + third[1][t]) + third[2][t];
    if (idx >= 0) {
        const float val = f.accumulate ? prev + tot : tot;
        f.dst[idx] = val;
        adam_apply(adam, idx, val, o, step_size, c2);
    } else if (idx <= -2 && f.metrics) {
        f.metrics[-2 - idx] = tot;
    }
}

__global__ __launch_bounds__(320) void final_kernel(FinalArgs f, AdamArgs adam,
                                                    const EngineScalars* __restrict__ sc) {
    if (threadIdx.x < kRedLen) final_pair(f, threadIdx.x, -1, adam, sc);
}

// out[W0 part] (= or +=) Xdᵀ d (one wave per feature) + Adam on the W0 entry it
// completes (param index f·16 + h).  With f.partials != NULL the grid carries
// one extra block that runs the final reduction of b0 / W1 / b1 (+ their Adam)
// concurrently: both only need the kernel that produced d and the partials.
// Long X columns (dense X, config 5): Xdᵀ d in `splits` entry ranges per
// column, one wave per (column, range), partial p of column f in
// part[(p·fin + f)·16 + h] (per sample: + sample·splits·fin·16); xt_adam then
// sums the partials in range order instead of running the column dot itself.
template <bool kB>
__global__ __launch_bounds__(256) void xt_partials_kernel(
    const int* __restrict__ xcp, const int* __restrict__ xrow, const float* __restrict__ xval, int fin,
    const float* __restrict__ d, Keys keys, const EngineScalars* __restrict__ sc, int fwd_off, int train,
    float keep, float scale, int splits, float* __restrict__ part, Batch bt) {
    xval = boff<kB>(xval, bt.xval);
    d = boff<kB>(d, bt.act);
    bkeys<kB>(keys, bt);
    if (kB) part += (int64_t)blockIdx.y * splits * fin * HID;
    const int w = blockIdx.x * 4 + wave_id();   // f·splits + p
    if (w >= fin * splits) return;
    const int f = w / splits, p = w - f * splits;
    const int beg = xcp[f], end = xcp[f + 1];
    const int seg = ((end - beg + splits - 1) / splits + 4 * HID - 1) / (4 * HID) * (4 * HID);
    const int b = min(end, beg + p * seg), e = min(end, b + seg);
    const float acc = x_wave_dot_range<true>(b, e, xrow, xval, f, d, keys, sc->fwd_ctr + fwd_off, train, keep, scale);
    const int lane = threadIdx.x & 63;
    if (lane < HID) part[((int64_t)p * fin + f) * HID + lane] = acc;
}

// Columns of X are very uneven (Cora: 34 entries on average, up to 1083), and
// one wave walking a long column one 64-entry step per round trip set the
// launch's time.  The column plan (built once per X by the host,
// LdsEngine._xt_plan) lists the `n_heavy` columns longer than 128 entries first:
// each gets a 1024-thread block whose 16 waves take consecutive 64-aligned
// entry ranges, their partial sums combined through LDS in wave order; then
// n_single columns one wave each, n_pair columns of 17-32 entries two per
// wave (32 lanes each) and the rest, columns of at most 16 entries, four per
// wave (a 16-lane group each): fewer waves for the same sums (Cora: 68 heavy,
// 329 / 255 / 781 columns; 1,741 waves instead of 2,453 per sample).

// Column heads of the W0 products (xthead, ABI 18): the first kXtHead row
// indices of every plan slot, so a one-wave column (at most 128 entries) needs
// no index loads past its head.
constexpr int kXtHead = 128;

template <bool kB>
__global__ __launch_bounds__(1024) void xt_adam_kernel(
    const int* __restrict__ xcp, const int* __restrict__ xrow, const float* __restrict__ xval, int fin,
    const float* __restrict__ d, Keys keys, const EngineScalars* __restrict__ sc, int fwd_off, int train,
    float keep, float scale, FinalArgs fin_args, AdamArgs adam, const float* __restrict__ xt_part,
    int xt_splits, const int* __restrict__ order, int n_heavy, const int4* __restrict__ xtinfo,
    const int* __restrict__ xthead, int n_single, int n_pair, Batch bt) {
    fin_args.partials = boff<kB>(fin_args.partials, bt.part);
    fin_args.dst = boff<kB>(fin_args.dst, bt.par);
    fin_args.metrics = boff<kB>(fin_args.metrics, bt.met);
    adam.w0 = boff<kB>(adam.w0, bt.par);
    adam.m0 = boff<kB>(adam.m0, bt.par);
    adam.v0 = boff<kB>(adam.v0, bt.par);
    adam.w1 = boff<kB>(adam.w1, bt.par);
    adam.m1 = boff<kB>(adam.m1, bt.par);
    adam.v1 = boff<kB>(adam.v1, bt.par);
    adam.gp = boff<kB>(adam.gp, bt.par);
    adam.wbar = boff<kB>(adam.wbar, bt.par);
    adam.mbar = boff<kB>(adam.mbar, bt.par);
    adam.vbar = boff<kB>(adam.vbar, bt.par);
    adam.gbar = boff<kB>(adam.gbar, bt.par);
    xval = boff<kB>(xval, bt.xval);
    d = boff<kB>(d, bt.act);
    bkeys<kB>(keys, bt);
    // the final reduction is block 0: dispatched first, so its chain of
    // partial-sum round trips overlaps the column blocks (as the last block it
    // started after every other block of its sample had been dispatched)
    if (LDS_XT_EXPT == 5) return;
    if (LDS_XT_EXPT == 6) adam.mode = 0;  // no Adam loads or updates (the products and stores only)
    const int fb = fin_args.partials != nullptr ? kFinParts : 0;
    if ((int)blockIdx.x < fb) {
        if (LDS_XT_EXPT == 4) return;  // timing-only builds (tools/microbench/xt_parts.py)
        final_block_1024<kB ? 16 : 64>(fin_args, adam, sc, (int)blockIdx.x);
        return;
    }
    float step_size, c2;
    adam_step_consts(adam, sc, step_size, c2);
    const int bx = (int)blockIdx.x - fb;
    const int wave = wave_id();
    const int lane = threadIdx.x & 63;
    const bool heavy = bx < n_heavy;
    if (LDS_XT_EXPT == 1 && heavy) return;
    if (LDS_XT_EXPT == 2 && !heavy && (bx - n_heavy) * 16 + wave < n_single) return;
    if (LDS_XT_EXPT == 3 && !heavy && (bx - n_heavy) * 16 + wave >= n_single) return;
    {
        // light waves past the single-column ones: two or four short columns
        const int lw = (bx - n_heavy) * 16 + wave;  // light wave number
        const int w2 = n_single + (n_pair + 1) / 2;  // first four-column wave
        if (!heavy && lw >= n_single) {
            const int base = n_heavy + n_single;
            const bool four = lw >= w2;
            const int qc = four ? 0 : (lane >> 4) & 1;
            const int slot = four ? base + n_pair + 4 * (lw - w2) + (lane >> 4)
                                  : base + 2 * (lw - n_single) + (lane >> 5);
            const int send = four ? fin : base + n_pair;
            if (__ballot(slot < send) == 0ull) return;  // light waves never reach a barrier
            const bool live = slot < send;
            const int hs = live ? slot : base;
            // the head entry first: it does not wait for the column's info,
            // so the gathers need one round trip after it, not two
            const int jh = xthead[(int64_t)hs * kXtHead + 16 * qc + (lane & (HID - 1))];
            const int4 inf = xtinfo[hs];
            const int idx = inf.x * HID + (lane & (HID - 1));
            const bool owner = live && qc == 0;
            AdamOps o{0.f, 0.f, 0.f, 0.f, 0.f};
            float prev = 0.f;
            if (owner) {
                if (LDS_XT_EXPT != 7) o = adam_load(adam, idx);
                if (fin_args.accumulate) prev = fin_args.dst[idx];
            }
            float acc = x_group_dot_head(qc, inf.y, live ? inf.z : 0, jh, xval, d);
            if (!four) acc = xor16_add(acc);  // the column's two groups, as groups_sum adds them
            if (LDS_XT_EXPT == 7 && owner) o = adam_load(adam, idx);
            if (owner) {
                const float val = fin_args.accumulate ? prev + acc : acc;
                fin_args.dst[idx] = val;
                adam_apply(adam, idx, val, o, step_size, c2);
            }
            return;
        }
    }
    // with the column heads (xtinfo[slot] = {f, p0, nnz}, slot = position in
    // `order`) one load gives the column, its range and its first 64 rows;
    // without them: order[slot] -> xcp[f] -> entries, two dependent loads first
    int f, beg, end, slot, jh = 0, jh2 = 0;
    if (heavy) {
        slot = bx;
        int cb, ce;
        if (xtinfo != nullptr) {
            const int4 inf = xtinfo[slot];
            f = inf.x;
            cb = inf.y;
            ce = inf.y + inf.z;
        } else {
            f = order[slot];
            cb = xcp[f];
            ce = xcp[f + 1];
        }
        const int seg = ((ce - cb + 15) / 16 + 63) / 64 * 64;
        beg = min(ce, cb + wave * seg);
        end = min(ce, beg + seg);
    } else {
        slot = n_heavy + (bx - n_heavy) * 16 + wave;
        if (slot >= fin) return;  // light blocks never reach a barrier
        // the lane's head entry ahead of the column's info (the gathers then
        // wait one round trip, not two)
        if (xthead != nullptr && xt_part == nullptr) {
            const int* hp = xthead + (int64_t)slot * kXtHead + 16 * ((threadIdx.x >> 4) & 3) + (lane & (HID - 1));
            jh = hp[0];
            jh2 = hp[64];
        }
        if (xtinfo != nullptr) {
            const int4 inf = xtinfo[slot];
            f = inf.x;
            beg = inf.y;
            end = inf.y + inf.z;
        } else {
            f = order[slot];
            beg = xcp[f];
            end = xcp[f + 1];
        }
    }
    // A block of sixteen one-column waves completes its columns' Adam steps on
    // four waves, four columns (64 lanes) each, after one barrier: the Adam
    // tail (a correctly rounded square root and two or more divisions per
    // element) then costs each SIMD one wave's issue instead of four, where
    // every wave used 16 of its 64 lanes.  The same operands and arithmetic.
    const bool batched = !heavy && xthead != nullptr && xt_part == nullptr && (bx - n_heavy + 1) * 16 <= n_single;
    int idx = f * HID + (lane & (HID - 1));
    bool owner = lane < HID && (!heavy || wave == 0);
    if (batched) {
        owner = wave < 4;
        if (owner) {  // column 4·wave + lane / 16 of the block, feature lane % 16
            const int4 ainf = xtinfo[n_heavy + (bx - n_heavy) * 16 + 4 * wave + (lane >> 4)];
            idx = ainf.x * HID + (lane & (HID - 1));
        }
    }
    // Adam operands and constants first: they overlap the product's loads
    AdamOps o{0.f, 0.f, 0.f, 0.f, 0.f};
    float prev = 0.f;
    if (owner) {
        if (LDS_XT_EXPT != 7) o = adam_load(adam, idx);
        if (fin_args.accumulate) prev = fin_args.dst[idx];
    }
    float acc = 0.f;
    if (xt_part != nullptr) {   // partials of xt_partials_kernel, summed in range order (n_heavy = 0)
        if (kB) xt_part += (int64_t)blockIdx.y * xt_splits * fin * HID;
        if (lane < HID)
            for (int p = 0; p < xt_splits; ++p) acc += xt_part[((int64_t)p * fin + f) * HID + lane];
    } else if (xthead != nullptr && !heavy) {
        acc = x_wave_dot_head<true, 2, true>(f, beg, end - beg, xthead + (int64_t)slot * kXtHead, xrow, xval, d,
                                             keys, sc->fwd_ctr + fwd_off, train, keep, scale, nullptr, nullptr,
                                             nullptr, jh, jh2);
    } else {
        acc = x_wave_dot_range<true>(beg, end, xrow, xval, f, d, keys, sc->fwd_ctr + fwd_off, train, keep, scale);
    }
    __shared__ float part[16][HID];
    if (heavy) {
        if (lane < HID) part[wave][lane] = acc;
        __syncthreads();
        if (wave == 0 && lane < HID) {
            acc = 0.f;
#pragma unroll
            for (int w = 0; w < 16; ++w) acc += part[w][lane];
        }
    } else if (batched) {  // block-uniform: all sixteen waves have a column
        if (lane < HID) part[wave][lane] = acc;
        __syncthreads();
        if (owner) acc = part[4 * wave + (lane >> 4)][lane & (HID - 1)];
    }
    if (LDS_XT_EXPT == 7 && owner) o = adam_load(adam, idx);
    if (owner) {
        const float val = fin_args.accumulate ? prev + acc : acc;
        fin_args.dst[idx] = val;
        adam_apply(adam, idx, val, o, step_size, c2);
    }
}

// Per-sample views of a batched launch's arrays (sample smp; the one-sample
// kernels take it from blockIdx.y through boff).
template <typename T>
__device__ __forceinline__ T* soff(T* p, int64_t stride, int smp) {
    return p == nullptr ? p : p + (int64_t)smp * stride;
}
__device__ __forceinline__ void sample_views(FinalArgs& f, AdamArgs& a, const Batch& bt, int smp) {
    f.partials = soff(f.partials, bt.part, smp);
    f.dst = soff(f.dst, bt.par, smp);
    f.metrics = soff(f.metrics, bt.met, smp);
    a.w0 = soff(a.w0, bt.par, smp);
    a.m0 = soff(a.m0, bt.par, smp);
    a.v0 = soff(a.v0, bt.par, smp);
    a.w1 = soff(a.w1, bt.par, smp);
    a.m1 = soff(a.m1, bt.par, smp);
    a.v1 = soff(a.v1, bt.par, smp);
    a.gp = soff(a.gp, bt.par, smp);
    a.wbar = soff(a.wbar, bt.par, smp);
    a.mbar = soff(a.mbar, bt.par, smp);
    a.vbar = soff(a.vbar, bt.par, smp);
    a.gbar = soff(a.gbar, bt.par, smp);
}

// xt_adam_kernel<true> over pairs of samples (LdsBatch.xt_pair): grid.y =
// samples / 2, a wave takes one column for samples 2y and 2y + 1
// (x_wave_dot_head_pair: one index walk, the same sums), lanes 0-15 and 32-47
// complete the two W0 entries' Adam; the first two blocks run the samples'
// final reductions.  Light columns only (no heavy-column plan), column heads,
// no split partials, train = 0 (the stored Xd).
__global__ __launch_bounds__(1024) void xt_adam_pair_kernel(
    const int* __restrict__ xrow, const float* __restrict__ xval, int fin, const float* __restrict__ d,
    const EngineScalars* __restrict__ sc, FinalArgs fin_args, AdamArgs adam, const int4* __restrict__ xtinfo,
    const int* __restrict__ xthead, Batch bt) {
    const int s0 = 2 * (int)blockIdx.y;
    const int fb = fin_args.partials != nullptr ? 2 * kFinParts : 0;  // the final blocks first (as xt_adam_kernel)
    if ((int)blockIdx.x < fb) {
        sample_views(fin_args, adam, bt, s0 + (int)blockIdx.x / kFinParts);
        final_block_1024<16>(fin_args, adam, sc, (int)blockIdx.x % kFinParts);
        return;
    }
    const int wave = wave_id();
    const int lane = threadIdx.x & 63;
    const int slot = ((int)blockIdx.x - fb) * 16 + wave;
    if (slot >= fin) return;  // light blocks never reach a barrier
    sample_views(fin_args, adam, bt, s0 + (lane >> 5));
    float step_size, c2;
    adam_step_consts(adam, sc, step_size, c2);
    const int4 inf = xtinfo[slot];
    const int f = inf.x;
    const int idx = f * HID + (lane & (HID - 1));
    const bool owner = (lane & 31) < HID;
    AdamOps o{0.f, 0.f, 0.f, 0.f, 0.f};
    float prev = 0.f;
    if (owner) {
        o = adam_load(adam, idx);
        if (fin_args.accumulate) prev = fin_args.dst[idx];
    }
    const float acc = x_wave_dot_head_pair(inf.y, inf.z, xthead + (int64_t)slot * kXtHead, xrow,
                                           soff(xval, bt.xval, s0), soff(xval, bt.xval, s0 + 1),
                                           soff(d, bt.act, s0), soff(d, bt.act, s0 + 1));
    if (owner) {
        const float val = fin_args.accumulate ? prev + acc : acc;
        fin_args.dst[idx] = val;
        adam_apply(adam, idx, val, o, step_size, c2);
    }
}

// End of a window: slot T -> slot 0 for w, m, v, and advance the scalars.
__global__ __launch_bounds__(256) void end_window_kernel(int np, const float* __restrict__ wT,
                                                         const float* __restrict__ mT,
                                                         const float* __restrict__ vT,
                                                         float* __restrict__ w0, float* __restrict__ m0,
                                                         float* __restrict__ v0, EngineScalars* sc,
                                                         int graphs, int forwards, int adam_steps,
                                                         int hypers, const double* __restrict__ betas,
                                                         float* __restrict__ tab, int tab_count, int64_t par,
                                                         int* __restrict__ ws, int* __restrict__ ws_src,
                                                         int64_t ws_count) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (ws != nullptr) {  // the next window's sampler workspace (lds_sample_graphs_multi, ws_zeroed)
        const int64_t stride = (int64_t)gridDim.x * gridDim.y * 256;
        // ws_src (a prefetched draw's degrees, lds_theta_grad_sgd_draw): moved
        // into ws for the next window's fill, and cleared for the next draw
        for (int64_t k = ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x; k < ws_count; k += stride) {
            if (ws_src != nullptr) {
                ws[k] = ws_src[k];
                ws_src[k] = 0;
            } else {
                ws[k] = 0;
            }
        }
    }
    if (wT != nullptr && e < np) {
        const int64_t o = (int64_t)blockIdx.y * par;
        w0[o + e] = wT[o + e];
        m0[o + e] = mT[o + e];
        v0[o + e] = vT[o + e];
    }
    if (blockIdx.x == 0 && blockIdx.y == 0) {  // the scalars are shared by all samples
        __shared__ int new_step;
        if (threadIdx.x == 0) {
            sc->graph_ctr += graphs;
            sc->fwd_ctr += forwards;
            const int st = sc->adam_step + adam_steps;
            sc->adam_step = st;
            new_step = st;
            for (int h = 0; h < hypers; ++h) {
                sc->hyper_steps += 1;
                sc->outer_lr = sc->outer_lr * sc->lr_decay;
            }
        }
        __syncthreads();
        if (tab != nullptr) refresh_adam_table(new_step, betas, tab, tab_count, threadIdx.x);
    }
}

__global__ __launch_bounds__(256) void adam_table_kernel(const EngineScalars* __restrict__ sc,
                                                         const double* __restrict__ betas,
                                                         float* __restrict__ tab, int count) {
    refresh_adam_table(sc->adam_step, betas, tab, count, threadIdx.x);
}

// θ <- clamp(θ - lr·g, 0, 1) with lr from the scalars, then StepLR: lr *= γ.
__global__ void sgd_clamp_dev_kernel(float* __restrict__ theta, const float* __restrict__ grad,
                                     int64_t count, const EngineScalars* __restrict__ sc) {
    const float lr = (float)sc->outer_lr;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < count; e += stride)
        theta[e] = fminf(fmaxf(fmaf(-lr, grad[e], theta[e]), 0.f), 1.f);
}

// Advance the device scalars after a window: graph/forward counters, Adam
// step, hyper step count and the StepLR learning rate.
__global__ void advance_kernel(EngineScalars* sc, int graphs, int forwards, int adam_steps, int hypers) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        sc->graph_ctr += graphs;
        sc->fwd_ctr += forwards;
        sc->adam_step += adam_steps;
        for (int h = 0; h < hypers; ++h) {
            sc->hyper_steps += 1;
            sc->outer_lr = sc->outer_lr * sc->lr_decay;
        }
    }
}

}  // namespace lds

using namespace lds;

// ---------------------------------------------------------------------------
// C-ABI (see include/ldsgnn.h, "Fused engine")
// ---------------------------------------------------------------------------
static inline int rows_blocks(int n) { return (n + RG - 1) / RG; }
// one wave per row (agg_row): 4 rows per 256-thread block, 16 per 1024-thread block
static inline int wave_blocks(int n) { return (n + 3) / 4; }

// Kernel-side strides of a host LdsBatch (NULL: one sample); returns grid.y.
static inline int mk_batch(const LdsBatch* b, Batch& bt) {
    bt = Batch{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0u, nullptr, nullptr, 0, 0};
    if (b == nullptr) return 1;
    bt.asplit = b->agg_splits > 0 ? b->agg_splits : 0;
    bt.heavy = b->heavy_rows;  // the row plan applies to single-sample launches too
    bt.hflag = b->heavy_flag;
    bt.nh = b->n_heavy > 0 && b->heavy_rows && b->heavy_flag ? b->n_heavy : 0;
    if (b->samples <= 1) return 1;
    bt.act = b->act; bt.row = b->row; bt.rp = b->rp; bt.col = b->col; bt.ell2 = b->ell / 2; bt.par = b->par;
    bt.xval = b->xval; bt.xd = b->xd; bt.uv = b->uv; bt.part = b->part; bt.met = b->met; bt.tag = b->tag_step;
    return b->samples;
}
// lds_engine_xt_adam pairs samples per wave by shape from this many samples
// on (MI355X, profiles/r03_xt_pair_ab.jsonl: Citeseer S = 16 56.6 -> 41.6 µs
// per call, Cora S = 16 30.9 -> 28.8; at Cora S = 8 the doubled walk per wave
// costs more than the shared index loads save, 15.7 -> 19.2)
constexpr int kXtPairMinSamples = 16;
static inline int plan_heavy(const LdsBatch* b) {
    return b != nullptr && b->n_heavy > 0 && b->heavy_rows && b->heavy_flag ? b->n_heavy : 0;
}
// Launch the batched (kB = true) instantiation only for more than one sample.
#define LDS_LAUNCH_B(kern, ns, ...)                          \
    do {                                                      \
        if ((ns) > 1) hipLaunchKernelGGL(kern<true>, __VA_ARGS__);  \
        else hipLaunchKernelGGL(kern<false>, __VA_ARGS__);          \
    } while (0)

// ... and the precomputed-aggregation (kAgg) instantiation only when agg != NULL.
#define LDS_LAUNCH_BA(kern, ns, agg, ...)                                                       \
    do {                                                                                       \
        if ((agg) != nullptr) {                                                                \
            if ((ns) > 1) hipLaunchKernelGGL(HIP_KERNEL_NAME(kern<true, true>), __VA_ARGS__);   \
            else hipLaunchKernelGGL(HIP_KERNEL_NAME(kern<false, true>), __VA_ARGS__);           \
        } else {                                                                               \
            if ((ns) > 1) hipLaunchKernelGGL(HIP_KERNEL_NAME(kern<true, false>), __VA_ARGS__);  \
            else hipLaunchKernelGGL(HIP_KERNEL_NAME(kern<false, false>), __VA_ARGS__);          \
        }                                                                                      \
    } while (0)

static inline bool batch_ok(const LdsBatch* b) {
    return b == nullptr || (b->samples >= 1 && b->samples <= 65535 && (b->ell & 1) == 0);
}
// The error word of an engine's scalars (fill kernels report into it).
static inline uint32_t* engine_error_word(const void* scalars) {
    return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(const_cast<void*>(scalars)) +
                                       offsetof(EngineScalars, error));
}
static inline Keys mk_keys(uint64_t seed, uint32_t tag_x, uint32_t tag_h) {
    return Keys{(uint32_t)seed, (uint32_t)(seed >> 32), tag_x, tag_h};
}

extern "C" int lds_engine_x_linear(const int* xrp, const int* xcol, const float* xval, int n,
                                   const float* wt, const float* bias, float* out, uint64_t seed,
                                   uint32_t tag_x, const void* scalars, int fwd_off, int train,
                                   float keep, float scale, float* xd_csr, float* xd_csc,
                                   const int* csr2csc, const int* xhead, const int* xinfo, int head_vals,
                                   const LdsBatch* batch, void* stream) {
    LDS_CHECK_ARG(xrp && xcol && xval && wt && out && scalars && n > 0 && batch_ok(batch));
    LDS_CHECK_ARG(xd_csc == nullptr || (xd_csr && csr2csc));
    LDS_CHECK_ARG(xhead == nullptr || xinfo != nullptr);
    Batch bt;
    const int ns = mk_batch(batch, bt);
    LDS_LAUNCH_B(x_linear_kernel, ns, dim3((n + 3) / 4, ns), dim3(256), 0, (hipStream_t)stream, xrp,
                       xcol, xval, n, wt, bias, out, mk_keys(seed, tag_x, 0),
                       (const EngineScalars*)scalars, fwd_off, train, keep, scale, xd_csr, xd_csc, csr2csc, xhead,
                       (const int2*)xinfo, head_vals, bt);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_fill_x_linear(const uint64_t* bits, int words, const int* deg_ws, int graphs,
                                        int* row_ptr, int* col, int64_t col_stride, float* s, int* ell,
                                        const uint8_t* node_flags, const int* xrp, const int* xcol,
                                        const float* xval, int n, const float* wt, const float* bias, float* out,
                                        uint64_t seed, uint32_t tag_x, const void* scalars, int fwd_off, int train,
                                        float keep, float scale, float* xd_csr, float* xd_csc, const int* csr2csc,
                                        const int* xhead, const int* xinfo, int head_vals, const LdsBatch* batch,
                                        void* stream) {
    LDS_CHECK_ARG(bits && deg_ws && row_ptr && col && s && n > 0 && n <= kEllIndex + 1 && col_stride > 0);
    LDS_CHECK_ARG(graphs > 0 && graphs <= 65535 && words >= (n + 63) / 64);
    LDS_CHECK_ARG(xrp && xcol && xval && wt && out && scalars && batch_ok(batch));
    LDS_CHECK_ARG(xd_csc == nullptr || (xd_csr && csr2csc));
    LDS_CHECK_ARG(xhead == nullptr || xinfo != nullptr);
    Batch bt;
    const int ns = mk_batch(batch, bt);
    const int64_t blocks = (int64_t)((n + 15) / 16) * graphs + (int64_t)((n + 3) / 4) * ns;
    LDS_CHECK_ARG(blocks < (1ll << 31));
    LDS_LAUNCH_B(fill_x_linear_kernel, ns, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, bits, words,
                       deg_ws, lds_sample_ws_ints(n), graphs, row_ptr, col, col_stride, s, (int2*)ell, node_flags,
                       xrp, xcol, xval, n, wt, bias, out, mk_keys(seed, tag_x, 0), (const EngineScalars*)scalars,
                       fwd_off, train, keep, scale, xd_csr, xd_csc, csr2csc, xhead, (const int2*)xinfo, head_vals,
                       bt, engine_error_word(scalars));
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_xt_linear(const int* xcp, const int* xrow, const float* xval, int fin,
                                    const float* d, float* out, const float* w, float wd,
                                    int accumulate, uint64_t seed, uint32_t tag_x, const void* scalars,
                                    int fwd_off, int train, float keep, float scale, void* stream) {
    LDS_CHECK_ARG(xcp && xrow && xval && d && out && scalars && fin > 0);
    hipLaunchKernelGGL(xt_linear_kernel, dim3(rows_blocks(fin)), dim3(256), 0, (hipStream_t)stream,
                       xcp, xrow, xval, fin, d, out, w, wd, accumulate, mk_keys(seed, tag_x, 0),
                       (const EngineScalars*)scalars, fwd_off, train, keep, scale);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_fwd_layer1(const int* rp, const int* col, const float* s, const int* ell, int n,
                                     const float* h0, float* y0, float* h1d, float* h2,
                                     const float* w1, const float* b1, int c, uint64_t seed,
                                     uint32_t tag_h, const void* scalars, int fwd_off, int train,
                                     float keep, float scale, float* dmask, const float* agg, const LdsBatch* batch,
                                     void* stream) {
    LDS_CHECK_ARG(rp && col && s && h0 && y0 && h1d && h2 && w1 && b1 && scalars && n > 0);
    LDS_CHECK_ARG(c > 0 && c <= HID && batch_ok(batch));
    GcnW w{nullptr, nullptr, w1, b1};
    Batch bt;
    const int ns = mk_batch(batch, bt);
    LDS_LAUNCH_BA(fwd_layer1_kernel, ns, agg, dim3(wave_blocks(n) + plan_heavy(batch), ns), dim3(256), 0, (hipStream_t)stream, rp,
                       col, s, (const int2*)ell, n, h0, y0, h1d, h2, w, c, mk_keys(seed, 0, tag_h),
                       (const EngineScalars*)scalars, fwd_off, train, keep, scale, dmask, agg, bt);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_fwd_layer2(const int* rp, const int* col, const float* s, const int* ell, int n,
                                     const float* h2, float* o, float* p, float* d_o,
                                     const int* label, const uint8_t* mask, float inv_count,
                                     float* lossrow, float* corrrow, int c, const float* agg, const LdsBatch* batch,
                                     void* stream) {
    LDS_CHECK_ARG(rp && col && s && h2 && label && lossrow && corrrow && n > 0 && c > 0 && c <= HID);
    LDS_CHECK_ARG(batch_ok(batch));
    Batch bt;
    const int ns = mk_batch(batch, bt);
    LDS_LAUNCH_BA(fwd_layer2_kernel, ns, agg, dim3(wave_blocks(n) + plan_heavy(batch), ns), dim3(256), 0, (hipStream_t)stream, rp,
                       col, s, (const int2*)ell, n, h2, o, p, d_o, label, mask, inv_count, lossrow, corrrow, c,
                       agg, bt);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_bwd_layer2(const int* rp, const int* col, const float* s, const int* ell, int n,
                                     const float* d_o, const float* y0, float* dh2, float* dy0,
                                     const float* w1, int c, uint64_t seed, uint32_t tag_h,
                                     const void* scalars, int fwd_off, int train, float keep,
                                     float scale, const float* o, const float* h2, float* U, float* V,
                                     int ldk, float* R, int foff, int fwidth, int r_assign,
                                     const float* dmask, const float* agg, const LdsBatch* batch, void* stream) {
    LDS_CHECK_ARG(rp && col && s && d_o && y0 && dh2 && dy0 && w1 && scalars && n > 0 && batch_ok(batch));
    LDS_CHECK_ARG(c > 0 && c <= HID && (U == nullptr || (V && R && o && h2 && fwidth <= HID)));
    GcnW w{nullptr, nullptr, w1, nullptr};
    Batch bt;
    const int ns = mk_batch(batch, bt);
    LDS_LAUNCH_BA(bwd_layer2_kernel, ns, agg, dim3(wave_blocks(n) + plan_heavy(batch), ns), dim3(256), 0, (hipStream_t)stream, rp,
                       col, s, (const int2*)ell, n, d_o, y0, dh2, dy0, w, c, mk_keys(seed, 0, tag_h),
                       (const EngineScalars*)scalars, fwd_off, train, keep, scale, o, h2, U, V, ldk, R,
                       foff, fwidth, r_assign, dmask, agg, bt);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_bwd_layer1(const int* rp, const int* col, const float* s, const int* ell, int n,
                                     const float* dy0, float* dh0, const float* y0, const float* h0,
                                     float* U, float* V, int ldk, float* R, int foff, void* stream) {
    LDS_CHECK_ARG(rp && col && s && dy0 && dh0 && n > 0);
    LDS_CHECK_ARG(U == nullptr || (V && R && y0 && h0));
    hipLaunchKernelGGL(bwd_layer1_kernel, dim3(wave_blocks(n)), dim3(256), 0, (hipStream_t)stream, rp,
                       col, s, (const int2*)ell, n, dy0, dh0, y0, h0, U, V, ldk, R, foff);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_colreduce(int n, int c_n, const float* a1, const float* b1, const float* a2,
                                    const float* b2, const float* x1, const float* x2, const float* l,
                                    const float* q, float* partials, int nblocks, float* dst_a,
                                    float* dst_v1, int v1_width, float* dst_v2, int v2_width,
                                    float* dst_l, int accumulate, void* stream) {
    LDS_CHECK_ARG(partials && n > 0 && nblocks > 0 && nblocks <= kRedBlocks && c_n >= 0 && c_n <= HID);
    const int rpb = (n + nblocks - 1) / nblocks;
    hipLaunchKernelGGL(colreduce_kernel, dim3(nblocks), dim3(256), 0, (hipStream_t)stream, n, c_n, a1,
                       b1, a2, b2, x1, x2, l, q, partials, rpb);
    hipLaunchKernelGGL(colreduce_final_kernel, dim3(1), dim3(320), 0, (hipStream_t)stream, partials,
                       nblocks, c_n, dst_a, dst_v1, v1_width, dst_v2, v2_width, dst_l, accumulate);
    LDS_RETURN_LAST_ERROR();
}

// `hyper` = {lr, beta1, beta2, eps, weight_decay} as doubles (Python floats); the
// kernels use float(x) of each, float(1 - beta) and the double bias corrections.
static AdamHyper mk_adam(const double* h, int n_wd) {
    return AdamHyper{(float)h[0], (float)h[1], (float)h[2], (float)h[3], (float)h[4],
                     (float)(1.0 - h[1]), (float)(1.0 - h[2]), n_wd};
}

extern "C" int lds_engine_adam(int np, const float* w0, const float* g, const float* m0,
                               const float* v0, float* w1, float* m1, float* v1, float* gp_out,
                               const double* hyper, const double* betas_dev, int n_wd,
                               const void* scalars, int step_off, void* stream) {
    LDS_CHECK_ARG(np > 0 && w0 && g && m0 && v0 && w1 && m1 && v1 && scalars && hyper && betas_dev);
    hipLaunchKernelGGL(adam_fwd_kernel, dim3((np + 255) / 256), dim3(256), 0, (hipStream_t)stream, np,
                       w0, g, m0, v0, w1, m1, v1, gp_out, mk_adam(hyper, n_wd), betas_dev,
                       (const EngineScalars*)scalars, step_off);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_adam_reverse(int np, float* wbar, float* mbar, float* vbar, const float* m1,
                                       const float* v1, const float* gp, float* gbar,
                                       const double* hyper, const double* betas_dev, int n_wd,
                                       const void* scalars, int step_off, void* stream) {
    LDS_CHECK_ARG(np > 0 && wbar && mbar && vbar && m1 && v1 && gp && gbar && scalars && hyper);
    LDS_CHECK_ARG(betas_dev != nullptr);
    hipLaunchKernelGGL(adam_rev_kernel, dim3((np + 255) / 256), dim3(256), 0, (hipStream_t)stream, np,
                       wbar, mbar, vbar, m1, v1, gp, gbar, mk_adam(hyper, n_wd), betas_dev,
                       (const EngineScalars*)scalars, step_off);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_rev_a(const int* rp, const int* col, const float* s, const int* ell, int n,
                                const float* dh0bar, const float* dy0, const float* dh0,
                                const float* y0, const float* h1d, const float* dh2, const float* w1,
                                const float* gw1bar, const float* gb1bar, int c, float* dh1dbar,
                                float* dh2bar, float* h1dbar, uint64_t seed, uint32_t tag_h,
                                const void* scalars, int fwd_off, int train, float keep, float scale,
                                float* U, float* V, int ldk, float* R, int foff, const float* dmask,
                                const float* agg, const LdsBatch* batch, void* stream) {
    LDS_CHECK_ARG(rp && col && s && dh0bar && dy0 && dh0 && y0 && h1d && dh2 && w1 && gw1bar && gb1bar);
    LDS_CHECK_ARG(dh1dbar && dh2bar && h1dbar && scalars && U && V && R && n > 0 && c > 0 && c <= HID);
    LDS_CHECK_ARG(batch_ok(batch));
    GcnW w{nullptr, nullptr, w1, nullptr};
    Batch bt;
    const int ns = mk_batch(batch, bt);
    LDS_LAUNCH_BA(rev_a_kernel, ns, agg, dim3(wave_blocks(n) + plan_heavy(batch), ns), dim3(256), 0, (hipStream_t)stream, rp, col, s,
                       (const int2*)ell, n, dh0bar, dy0, dh0, y0, h1d, dh2, w, gw1bar, gb1bar, c, dh1dbar, dh2bar,
                       h1dbar, mk_keys(seed, 0, tag_h), (const EngineScalars*)scalars, fwd_off, train, keep,
                       scale, U, V, ldk, R, foff, dmask, agg, bt);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_rev_b(const int* rp, const int* col, const float* s, const int* ell, int n,
                                const float* dh2bar, const float* d_o, const float* dh2, const float* p,
                                const uint8_t* mask, float inv_count, int c, float* obar, float* U,
                                float* V, int ldk, float* R, int foff, int cw, const float* agg, const LdsBatch* batch,
                                void* stream) {
    LDS_CHECK_ARG(rp && col && s && dh2bar && d_o && dh2 && p && mask && obar && U && V && R && n > 0);
    LDS_CHECK_ARG(c > 0 && c <= HID && cw >= c && cw <= HID && batch_ok(batch));
    Batch bt;
    const int ns = mk_batch(batch, bt);
    LDS_LAUNCH_BA(rev_b_kernel, ns, agg, dim3(wave_blocks(n) + plan_heavy(batch), ns), dim3(256), 0, (hipStream_t)stream, rp, col, s,
                       (const int2*)ell, n, dh2bar, d_o, dh2, p, mask, inv_count, c, obar, U, V, ldk, R, foff, cw,
                       agg, bt);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_rev_c(const int* rp, const int* col, const float* s, const int* ell, int n,
                                const float* obar, const float* h2, const float* o,
                                const float* h1dbar_part, const float* y0, const float* w1, int c,
                                float* h2bar, float* y0bar, uint64_t seed, uint32_t tag_h,
                                const void* scalars, int fwd_off, int train, float keep, float scale,
                                float* U, float* V, int ldk, float* R, int foff, int cw,
                                const float* dmask, const float* agg, const LdsBatch* batch, void* stream) {
    LDS_CHECK_ARG(rp && col && s && obar && h2 && o && h1dbar_part && y0 && w1 && h2bar && y0bar);
    LDS_CHECK_ARG(scalars && U && V && R && n > 0 && c > 0 && c <= HID && cw >= c && cw <= HID);
    LDS_CHECK_ARG(batch_ok(batch));
    GcnW w{nullptr, nullptr, w1, nullptr};
    Batch bt;
    const int ns = mk_batch(batch, bt);
    LDS_LAUNCH_BA(rev_c_kernel, ns, agg, dim3(wave_blocks(n) + plan_heavy(batch), ns), dim3(256), 0, (hipStream_t)stream, rp, col, s,
                       (const int2*)ell, n, obar, h2, o, h1dbar_part, y0, w, c, h2bar, y0bar,
                       mk_keys(seed, 0, tag_h), (const EngineScalars*)scalars, fwd_off, train, keep, scale, U, V,
                       ldk, R, foff, cw, dmask, agg, bt);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_rev_d(const int* rp, const int* col, const float* s, const int* ell, int n,
                                const float* y0bar, const float* h0, const float* y0, float* h0bar,
                                float* U, float* V, int ldk, float* R, int foff, void* stream) {
    LDS_CHECK_ARG(rp && col && s && y0bar && h0 && y0 && h0bar && U && V && R && n > 0);
    hipLaunchKernelGGL(rev_d_kernel, dim3(wave_blocks(n)), dim3(256), 0, (hipStream_t)stream, rp, col, s, (const int2*)ell,
                       n, y0bar, h0, y0, h0bar, U, V, ldk, R, foff);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_fwd2_bwd2(const int* rp, const int* col, const float* s, const int* ell, int n,
                                     const uint8_t* node_flags, int mask_bit, const float* h2, float* o, float* p,
                                     float* d_o, const int* label, float inv_count, float* lossrow, float* corrrow,
                                     int c, const float* y0, float* dh2, float* dy0, const float* w1, uint64_t seed,
                                     uint32_t tag_h, const void* scalars, int fwd_off, int train, float keep,
                                     float scale, float* U, float* V, int ldk, float* R, int foff, int fwidth,
                                     int r_assign, const float* dmask, const LdsBatch* batch, void* stream) {
    LDS_CHECK_ARG(rp && col && s && ell && node_flags && h2 && o && p && d_o && label && lossrow && corrrow);
    LDS_CHECK_ARG(y0 && dh2 && dy0 && w1 && scalars && n > 0 && n <= kEllIndex + 1 && mask_bit > 0 && mask_bit < 256);
    LDS_CHECK_ARG(c > 0 && c <= HID && batch_ok(batch) && (U == nullptr || (V && R && fwidth <= HID)));
    GcnW w{nullptr, nullptr, w1, nullptr};
    Batch bt;
    const int ns = mk_batch(batch, bt);
    LDS_LAUNCH_B(fwd2_bwd2_kernel, ns, dim3(wave_blocks(n) + plan_heavy(batch), ns), dim3(256), 0,
                 (hipStream_t)stream, rp, col, s, (const int2*)ell, n, node_flags, mask_bit, h2, o, p, d_o, label,
                 inv_count, lossrow, corrrow, c, y0, dh2, dy0, w, mk_keys(seed, 0, tag_h),
                 (const EngineScalars*)scalars, fwd_off, train, keep, scale, U, V, ldk, R, foff, fwidth, r_assign,
                 dmask, bt);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_rev_bc(const int* rp, const int* col, const float* s, const int* ell, int n,
                                 const uint8_t* node_flags, int mask_bit, const float* dh2bar, const float* d_o,
                                 const float* dh2, const float* p, const float* h2, const float* o,
                                 float inv_count, int c, const float* h1dbar_part, const float* y0,
                                 const float* w1, float* h2bar, float* y0bar, uint64_t seed, uint32_t tag_h,
                                 const void* scalars, int fwd_off, int train, float keep, float scale, float* U,
                                 float* V, int ldk, float* R, int foff_b, int foff_c, int cw, const float* dmask,
                                 const LdsBatch* batch, void* stream) {
    LDS_CHECK_ARG(rp && col && s && ell && node_flags && dh2bar && d_o && dh2 && p && h2 && o && h1dbar_part);
    LDS_CHECK_ARG(y0 && w1 && h2bar && y0bar && scalars && U && V && R && n > 0 && n <= kEllIndex + 1);
    LDS_CHECK_ARG(mask_bit > 0 && mask_bit < 256 && c > 0 && c <= HID && cw >= c && cw <= HID && batch_ok(batch));
    GcnW w{nullptr, nullptr, w1, nullptr};
    Batch bt;
    const int ns = mk_batch(batch, bt);
    LDS_LAUNCH_B(rev_bc_kernel, ns, dim3(wave_blocks(n) + plan_heavy(batch), ns), dim3(256), 0,
                 (hipStream_t)stream, rp, col, s, (const int2*)ell, n, node_flags, mask_bit, dh2bar, d_o, dh2, p, h2,
                 o, inv_count, c, h1dbar_part, y0, w, h2bar, y0bar, mk_keys(seed, 0, tag_h),
                 (const EngineScalars*)scalars, fwd_off, train, keep, scale, U, V, ldk, R, foff_b, foff_c, cw, dmask,
                 bt);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_sgd_clamp(float* theta, const float* grad, int64_t count, const void* scalars,
                                    void* stream) {
    LDS_CHECK_ARG(theta && grad && scalars && count >= 0);
    if (count == 0) return 0;
    const int64_t b = (count + 255) / 256;
    hipLaunchKernelGGL(sgd_clamp_dev_kernel, dim3((unsigned)(b < 8192 ? b : 8192)), dim3(256), 0,
                       (hipStream_t)stream, theta, grad, count, (const EngineScalars*)scalars);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_advance(void* scalars, int graphs, int forwards, int adam_steps, int hypers,
                                  void* stream) {
    LDS_CHECK_ARG(scalars != nullptr);
    hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                       (EngineScalars*)scalars, graphs, forwards, adam_steps, hypers);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_scalars_size(void) { return (int)sizeof(EngineScalars); }

// ----- fused entry points -----
static AdamArgs mk_adam_args(int mode, int first, const float* w0, const float* m0, const float* v0,
                             float* w1, float* m1, float* v1, float* gp, float* wbar, float* mbar,
                             float* vbar, float* gbar, const double* hyper, const float* tab,
                             int n_wd, int step_off) {
    AdamArgs a;
    a.w0 = w0; a.m0 = m0; a.v0 = v0; a.w1 = w1; a.m1 = m1; a.v1 = v1; a.gp = gp;
    a.wbar = wbar; a.mbar = mbar; a.vbar = vbar; a.gbar = gbar;
    a.hp = hyper ? mk_adam(hyper, n_wd) : AdamHyper{};
    a.tab = tab; a.step_off = step_off; a.mode = mode; a.first = first;
    return a;
}

static bool adam_ok(int mode, const float* w0, const float* m0, const float* v0, const float* w1,
                    const float* m1, const float* v1, const float* gp, const float* wbar,
                    const float* mbar, const float* vbar, const float* gbar, const double* hyper,
                    const float* tab, int step_off) {
    if (mode == 0) return true;
    if (!hyper || !tab || step_off < 0 || step_off >= kAdamTabMax) return false;
    if (mode == 1) return w0 && m0 && v0 && w1 && m1 && v1 && gp;
    if (mode == 2) return m1 && v1 && gp && wbar && mbar && vbar && gbar;
    return false;
}

extern "C" int lds_engine_bwd1_reduce(const int* rp, const int* col, const float* s, const int* ell, int n,
                                      const float* dy0, float* dh0, const float* y0, const float* h0,
                                      float* U, float* V, int ldk, float* R, int foff, const float* dh2,
                                      const float* h1d, const float* lossrow, const float* corrrow, int c,
                                      float* partials, const float* agg, const LdsBatch* batch, void* stream) {
    LDS_CHECK_ARG(rp && col && s && dy0 && dh0 && dh2 && h1d && lossrow && corrrow && partials && n > 0);
    LDS_CHECK_ARG(c > 0 && c <= HID && (U == nullptr || (V && R && y0 && h0)) && batch_ok(batch));
    Batch bt;
    const int ns = mk_batch(batch, bt);
    LDS_LAUNCH_BA(bwd1_reduce_kernel, ns, agg, dim3((n + kRowsPer1K - 1) / kRowsPer1K + plan_heavy(batch), ns), dim3(1024), 0, (hipStream_t)stream,
                       rp, col, s, (const int2*)ell, n, dy0, dh0, y0, h0, U, V, ldk, R, foff, dh2, h1d, lossrow,
                       corrrow, c, partials, agg, bt);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_rev_d_reduce(const int* rp, const int* col, const float* s, const int* ell, int n,
                                       const float* y0bar, const float* h0, const float* y0, float* h0bar,
                                       float* U, float* V, int ldk, float* R, int foff, const float* dh2,
                                       const float* dh1dbar, const float* h2bar, const float* h1d, int c,
                                       float* partials, const float* agg, const LdsBatch* batch, void* stream) {
    LDS_CHECK_ARG(rp && col && s && y0bar && h0 && y0 && h0bar && U && V && R && dh2 && dh1dbar && h2bar);
    LDS_CHECK_ARG(h1d && partials && n > 0 && c > 0 && c <= HID && batch_ok(batch));
    Batch bt;
    const int ns = mk_batch(batch, bt);
    LDS_LAUNCH_BA(rev_d_reduce_kernel, ns, agg, dim3((n + kRowsPer1K - 1) / kRowsPer1K + plan_heavy(batch), ns), dim3(1024), 0,
                       (hipStream_t)stream, rp, col, s, (const int2*)ell, n, y0bar, h0, y0, h0bar, U, V, ldk, R,
                       foff, dh2, dh1dbar, h2bar, h1d, c, partials, agg, bt);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_final(const float* partials, int nblocks, int c, float* dst, int off_b0,
                                int off_w1, int off_b1, int accumulate, float* metrics, int adam_mode,
                                int first, const float* w0, const float* m0, const float* v0, float* w1,
                                float* m1, float* v1, float* gp, float* wbar, float* mbar, float* vbar,
                                float* gbar, const double* hyper, const float* adam_tab, int n_wd,
                                const void* scalars, int step_off, void* stream) {
    LDS_CHECK_ARG(partials && dst && scalars && nblocks > 0 && c > 0 && c <= HID);
    LDS_CHECK_ARG(adam_ok(adam_mode, w0, m0, v0, w1, m1, v1, gp, wbar, mbar, vbar, gbar, hyper, adam_tab,
                          step_off));
    AdamArgs a = mk_adam_args(adam_mode, first, w0, m0, v0, w1, m1, v1, gp, wbar, mbar, vbar, gbar, hyper,
                              adam_tab, n_wd, step_off);
    FinalArgs f{partials, nblocks, c, off_b0, off_w1, off_b1, accumulate, dst, metrics};
    hipLaunchKernelGGL(final_kernel, dim3(1), dim3(320), 0, (hipStream_t)stream, f, a,
                       (const EngineScalars*)scalars);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_xt_adam(const int* xcp, const int* xrow, const float* xval, int fin,
                                  const float* d, float* out, int accumulate, uint64_t seed, uint32_t tag_x,
                                  const void* scalars, int fwd_off, int train, float keep, float scale,
                                  const float* partials, int nblocks, int c, int off_b0, int off_w1,
                                  int off_b1, float* metrics, int adam_mode, int first, const float* w0,
                                  const float* m0, const float* v0, float* w1, float* m1, float* v1,
                                  float* gp, float* wbar, float* mbar, float* vbar, float* gbar,
                                  const double* hyper, const float* adam_tab, int n_wd, int step_off,
                                  const float* xt_part, int xt_splits, const int* order, int n_heavy,
                                  const int* xtinfo, const int* xthead, int n_single, int n_pair,
                                  const LdsBatch* batch, void* stream) {
    LDS_CHECK_ARG(xcp && xrow && xval && d && out && scalars && order && fin > 0 && batch_ok(batch));
    LDS_CHECK_ARG(xthead == nullptr || xtinfo != nullptr);
    LDS_CHECK_ARG(n_heavy >= 0 && n_heavy <= fin && (xt_part == nullptr || n_heavy == 0));
    LDS_CHECK_ARG(partials == nullptr || (nblocks > 0 && c > 0 && c <= HID));
    LDS_CHECK_ARG(xt_part == nullptr || xt_splits > 0);
    LDS_CHECK_ARG(adam_ok(adam_mode, w0, m0, v0, w1, m1, v1, gp, wbar, mbar, vbar, gbar, hyper, adam_tab,
                          step_off));
    AdamArgs a = mk_adam_args(adam_mode, first, w0, m0, v0, w1, m1, v1, gp, wbar, mbar, vbar, gbar, hyper,
                              adam_tab, n_wd, step_off);
    FinalArgs f{partials, nblocks, c, off_b0, off_w1, off_b1, accumulate, out, metrics};
    Batch bt;
    const int ns = mk_batch(batch, bt);
    // pairs of samples per wave (LdsBatch.xt_pair): by shape from
    // kXtPairMinSamples samples on
    const int mode = batch != nullptr ? batch->xt_pair : 1;
    LDS_CHECK_ARG(mode >= 0 && mode <= 2);
    const bool can_pair = ns >= 2 && ns % 2 == 0 && n_heavy == 0 && xt_part == nullptr && xthead != nullptr &&
                          train == 0;
    LDS_CHECK_ARG(mode != 2 || can_pair);
    if (can_pair && (mode == 2 || (mode == 0 && ns >= kXtPairMinSamples))) {
        const int pblocks = (fin + 15) / 16 + (partials != nullptr ? 2 * kFinParts : 0);
        hipLaunchKernelGGL(xt_adam_pair_kernel, dim3(pblocks, ns / 2), dim3(1024), 0, (hipStream_t)stream, xrow,
                           xval, fin, d, (const EngineScalars*)scalars, f, a, (const int4*)xtinfo, xthead, bt);
        LDS_RETURN_LAST_ERROR();
    }
    // light waves: n_single one-column waves, then n_pair columns two per
    // wave, then the rest four per wave (these need the heads, train = 0)
    LDS_CHECK_ARG(n_single >= 0 && n_pair >= 0 && n_heavy + n_single + n_pair <= fin);
    LDS_CHECK_ARG(n_heavy + n_single == fin || (xthead != nullptr && xt_part == nullptr && train == 0));
    const int n_four = fin - n_heavy - n_single - n_pair;
    const int lwaves = n_single + (n_pair + 1) / 2 + (n_four + 3) / 4;
    const int blocks = n_heavy + (lwaves + 15) / 16 + (partials != nullptr ? kFinParts : 0);
    LDS_LAUNCH_B(xt_adam_kernel, ns, dim3(blocks, ns), dim3(1024), 0, (hipStream_t)stream, xcp, xrow, xval, fin,
                       d, mk_keys(seed, tag_x, 0), (const EngineScalars*)scalars, fwd_off, train, keep, scale, f,
                       a, xt_part, xt_splits, order, n_heavy, (const int4*)xtinfo, xthead, n_single, n_pair, bt);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_xt_partials(const int* xcp, const int* xrow, const float* xval, int fin,
                                      const float* d, uint64_t seed, uint32_t tag_x, const void* scalars,
                                      int fwd_off, int train, float keep, float scale, int splits, float* part,
                                      const LdsBatch* batch, void* stream) {
    LDS_CHECK_ARG(xcp && xrow && xval && d && part && scalars && fin > 0 && splits > 0 && batch_ok(batch));
    LDS_CHECK_ARG((int64_t)fin * splits * 64 <= ((int64_t)1 << 31) - 256);
    Batch bt;
    const int ns = mk_batch(batch, bt);
    const int blocks = (fin * splits + 3) / 4;
    LDS_LAUNCH_B(xt_partials_kernel, ns, dim3(blocks, ns), dim3(256), 0, (hipStream_t)stream, xcp, xrow, xval, fin,
                 d, mk_keys(seed, tag_x, 0), (const EngineScalars*)scalars, fwd_off, train, keep, scale, splits,
                 part, bt);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_end_window(int np, const float* wT, const float* mT, const float* vT, float* w0,
                                     float* m0, float* v0, void* scalars, int graphs, int forwards,
                                     int adam_steps, int hypers, const double* betas_dev, float* adam_tab,
                                     int tab_count, int* ws, int* ws_src, int64_t ws_count,
                                     const LdsBatch* batch, void* stream) {
    LDS_CHECK_ARG(scalars && np > 0 && (wT == nullptr || (mT && vT && w0 && m0 && v0)) && batch_ok(batch));
    LDS_CHECK_ARG(ws_count >= 0 && (ws != nullptr || ws_count == 0) && (ws_src == nullptr || ws != nullptr));
    LDS_CHECK_ARG(adam_tab == nullptr || (betas_dev && tab_count > 0 && tab_count <= kAdamTabMax));
    Batch bt;
    const int ns = mk_batch(batch, bt);
    hipLaunchKernelGGL(end_window_kernel, dim3((np + 255) / 256, ns), dim3(256), 0, (hipStream_t)stream, np, wT,
                       mT, vT, w0, m0, v0, (EngineScalars*)scalars, graphs, forwards, adam_steps, hypers,
                       betas_dev, adam_tab, tab_count, bt.par, ws, ws_src, ws_count);
    LDS_RETURN_LAST_ERROR();
}

extern "C" int lds_engine_adam_table(const void* scalars, const double* betas_dev, float* adam_tab,
                                     int tab_count, void* stream) {
    LDS_CHECK_ARG(scalars && betas_dev && adam_tab && tab_count > 0 && tab_count <= kAdamTabMax);
    hipLaunchKernelGGL(adam_table_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream,
                       (const EngineScalars*)scalars, betas_dev, adam_tab, tab_count);
    LDS_RETURN_LAST_ERROR();
}
