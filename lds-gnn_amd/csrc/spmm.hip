// Normalised CSR aggregation Y = diag(s)·Ã·diag(s)·Z — the GCN's Â·(XW + b).
//
// Replaces torch.mm(dense_adj, embeddings) (src/models/layers.py:44) after
// normalize_adjacency_matrix (src/utils/graph.py:136-153): the reference
// builds Â with two dense N³ matmuls and aggregates with a dense N²·F GEMM.
// Here Â is never formed: its values are s_i·s_j, implied by the CSR pattern
// of the sampled graph (self-loops included) and the vector s = deg^-1/2.
//
// Memory-bound: per call the algorithmic bytes are
//   4(N+1) row_ptr + 4·nnz col + 4N s + 4·N·F (Z, read once) + 4·N·F (Y).
// Z rows are gathered (coalesced 4·F-byte segments); Z of an N≤50k graph is
// L2/Infinity-Cache resident, so HBM sees the index stream and Y.
#include "common.hpp"
#include "../../include/ldsgnn.h"

namespace lds {

// G lanes per row, one feature per lane (F <= G), 256/G rows per block.
// Accumulation order is the CSR (ascending column) order, deterministic.
template <int G>
__global__ __launch_bounds__(256) void spmm_norm_group_kernel(
    const int* __restrict__ row_ptr, const int* __restrict__ col, const float* __restrict__ s,
    int n, const float* __restrict__ z, int f, int ldz, float* __restrict__ y, int ldy, int beta) {
    const int lane = threadIdx.x & (G - 1);
    const int row = (blockIdx.x * 256 + threadIdx.x) / G;
    if (row >= n) return;
    const bool act = lane < f;
    const int beg = row_ptr[row], end = row_ptr[row + 1];
    float acc = 0.0f;
    int p = beg;
    for (; p + 4 <= end; p += 4) {
        const int j0 = col[p], j1 = col[p + 1], j2 = col[p + 2], j3 = col[p + 3];
        const float s0 = s[j0], s1 = s[j1], s2 = s[j2], s3 = s[j3];
        float z0 = 0.f, z1 = 0.f, z2 = 0.f, z3 = 0.f;
        if (act) {
            z0 = z[(int64_t)j0 * ldz + lane];
            z1 = z[(int64_t)j1 * ldz + lane];
            z2 = z[(int64_t)j2 * ldz + lane];
            z3 = z[(int64_t)j3 * ldz + lane];
        }
        acc = fmaf(s0, z0, acc);
        acc = fmaf(s1, z1, acc);
        acc = fmaf(s2, z2, acc);
        acc = fmaf(s3, z3, acc);
    }
    for (; p < end; ++p) {
        const int j = col[p];
        const float zj = act ? z[(int64_t)j * ldz + lane] : 0.f;
        acc = fmaf(s[j], zj, acc);
    }
    if (act) {
        float* out = y + (int64_t)row * ldy + lane;
        const float v = s[row] * acc;
        *out = beta ? *out + v : v;
    }
}

template <int G>
static void launch_group(const int* row_ptr, const int* col, const float* s, int n,
                         const float* z, int f, int ldz, float* y, int ldy, int beta,
                         hipStream_t stream) {
    const int rows_per_block = 256 / G;
    const int blocks = (n + rows_per_block - 1) / rows_per_block;
    hipLaunchKernelGGL(spmm_norm_group_kernel<G>, dim3(blocks), dim3(256), 0, stream, row_ptr,
                       col, s, n, z, f, ldz, y, ldy, beta);
}

}  // namespace lds

using namespace lds;

extern "C" int lds_spmm_norm(const int* row_ptr, const int* col, const float* s, int n,
                             const float* z, int f, int ldz, float* y, int ldy, int beta,
                             void* stream) {
    LDS_CHECK_ARG(row_ptr != nullptr && col != nullptr && s != nullptr && z != nullptr &&
                  y != nullptr);
    LDS_CHECK_ARG(n > 0 && f > 0 && f <= 64 && ldz >= f && ldy >= f);
    hipStream_t st = (hipStream_t)stream;
    if (f <= 4) launch_group<4>(row_ptr, col, s, n, z, f, ldz, y, ldy, beta, st);
    else if (f <= 8) launch_group<8>(row_ptr, col, s, n, z, f, ldz, y, ldy, beta, st);
    else if (f <= 16) launch_group<16>(row_ptr, col, s, n, z, f, ldz, y, ldy, beta, st);
    else if (f <= 32) launch_group<32>(row_ptr, col, s, n, z, f, ldz, y, ldy, beta, st);
    else launch_group<64>(row_ptr, col, s, n, z, f, ldz, y, ldy, beta, st);
    LDS_RETURN_LAST_ERROR();
}
