// Keyed dropout and library-level entry points (ABI version, error text).
//
// lds_dropout replaces F.dropout (src/models/gcn.py:27,29).  The mask of
// element (i, j) is a pure function of (seed, tag, counter, i, j) through the
// Philox map of common.hpp, so the backward (and the CPU oracle) regenerate it
// instead of storing it.
#include "common.hpp"
#include "../../include/ldsgnn.h"

namespace lds {

// One thread per (column j, row quad): one Philox call covers four rows.
__global__ __launch_bounds__(256) void dropout_kernel(const float* __restrict__ x, int ldx,
                                                       float* __restrict__ y, int ldy, int rows,
                                                       int cols, float keep_prob, float scale,
                                                       uint32_t k0, uint32_t k1, uint32_t tag,
                                                       uint32_t counter, int quads) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)quads * cols;
    if (t >= total) return;
    const int rq = (int)(t / cols);
    const int j = (int)(t - (int64_t)rq * cols);
    float u[4];
    philox_quad(k0, k1, tag, counter, (uint32_t)j, (uint32_t)rq, u);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = rq * 4 + r;
        if (i < rows) {
            const float xv = x[(int64_t)i * ldx + j];
            y[(int64_t)i * ldy + j] = u[r] < keep_prob ? xv * scale : 0.0f;
        }
    }
}

}  // namespace lds

using namespace lds;

extern "C" int lds_abi_version(void) { return LDS_ABI_VERSION; }

extern "C" const char* lds_error_string(int err) {
    const char* s = hipGetErrorString((hipError_t)err);
    return s ? s : "unknown hip error";
}

extern "C" int lds_dropout(const float* x, int ldx, float* y, int ldy, int rows, int cols,
                           float keep_prob, float scale, uint64_t seed, uint32_t tag,
                           uint32_t counter, void* stream) {
    LDS_CHECK_ARG(x != nullptr && y != nullptr && rows >= 0 && cols >= 0);
    LDS_CHECK_ARG(ldx >= cols && ldy >= cols);
    if (rows == 0 || cols == 0) return 0;
    const int quads = (rows + 3) / 4;
    const int64_t total = (int64_t)quads * cols;
    const int64_t blocks = (total + 255) / 256;
    LDS_CHECK_ARG(blocks < (int64_t)1 << 31);
    hipLaunchKernelGGL(dropout_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       x, ldx, y, ldy, rows, cols, keep_prob, scale, (uint32_t)seed,
                       (uint32_t)(seed >> 32), tag, counter, quads);
    LDS_RETURN_LAST_ERROR();
}
