// θ pre-training step (Pretrainer.train_step, src/trainers/pretrainer.py:68-81):
//   P = triu_values_to_symmetric_matrix(θ)            (src/utils/graph.py:166-181)
//   loss = F.binary_cross_entropy(P, T, weight=W),     W = 1 + T·(pos_weight - 1)
//   loss.backward(); Adam.step()                       (torch.optim.Adam, no decay)
// on the packed upper triangle, one pass: P, the weighted-BCE gradient, the
// clamp and symmetrisation backward and the Adam update are fused, so the
// dense N×N P / W / grad tensors of the reference never exist.  HBM-bound:
// 4·3 B read + 4·3 B written per θ entry (θ, m, v) + N²/8 B of the T bitmask.
//
// Gradient per entry (torch's binary_cross_entropy_backward with mean
// reduction, EPSILON = 1e-12):  g(p, t) = (1/N²)·(p - t)/max(p(1-p), ε)·w.
// θ_ij, i < j, feeds P_ij and P_ji: dθ_ij = 2·g (if 0 <= θ_ij <= 1, the clamp's
// pass-through range); the diagonal feeds P_ii once.  Loss terms use torch's
// log clamp at -100.  Row partial losses (fixed-order block sums) go to
// loss_rows[i] for the host's Σ / N².
#include "common.hpp"
#include "../../include/ldsgnn.h"

namespace lds {

__global__ __launch_bounds__(256) void pretrain_step_kernel(
    float* __restrict__ theta, int n, const uint64_t* __restrict__ tbits, int words, float pos_weight,
    float inv_count, float* __restrict__ m, float* __restrict__ v, float beta1, float beta2, float omb1,
    float omb2, float eps, float step_size, float c2, float* __restrict__ loss_rows) {
    __shared__ float red[4];
    const int i = blockIdx.x;
    const int64_t base = tri_index(i, i, n);
    const uint64_t* trow = tbits + (int64_t)i * words;
    float lsum = 0.f;
    for (int j = i + threadIdx.x; j < n; j += 256) {
        const int64_t e = base + (j - i);
        const float th = theta[e];
        const float t = ((trow[j >> 6] >> (j & 63)) & 1ull) ? 1.f : 0.f;
        const float p = fminf(fmaxf(th, 0.f), 1.f);
        const float w = t * (pos_weight - 1.f) + 1.f;
        const float mult = (j == i) ? 1.f : 2.f;
        // loss (log clamped at -100 as torch's binary_cross_entropy)
        const float lp = fmaxf(logf(p), -100.f), l1p = fmaxf(logf(1.f - p), -100.f);
        lsum += mult * (w * -(t * lp + (1.f - t) * l1p));
        // gradient through BCE, clamp (pass-through on [0, 1]) and symmetrisation
        float g = (inv_count * (p - t)) / fmaxf((1.f - p) * p, 1e-12f) * w;
        g = (th >= 0.f && th <= 1.f) ? mult * g : 0.f;
        // Adam (torch.optim.Adam): exp_avg, exp_avg_sq, denom, addcdiv
        const float mm = m[e] * beta1 + omb1 * g;
        const float vv = v[e] * beta2 + (omb2 * g) * g;
        const float denom = sqrtf(vv) / c2 + eps;
        theta[e] = th + ((-step_size) * mm) / denom;
        m[e] = mm;
        v[e] = vv;
    }
    lsum = wave_sum(lsum);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = lsum;
    __syncthreads();
    if (threadIdx.x == 0) loss_rows[i] = (red[0] + red[1]) + (red[2] + red[3]);
}

}  // namespace lds

using namespace lds;

extern "C" int lds_pretrain_step(float* theta, int n, const uint64_t* train_bits, int words, float pos_weight,
                                 float* exp_avg, float* exp_avg_sq, int step, double lr, double beta1,
                                 double beta2, double eps, float* loss_rows, void* stream) {
    LDS_CHECK_ARG(theta && train_bits && exp_avg && exp_avg_sq && loss_rows && n > 0 && step >= 1);
    LDS_CHECK_ARG(words >= (n + 63) / 64);
    // bias corrections in double, as torch.optim.Adam computes them in Python
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    const float inv_count = (float)(1.0 / ((double)n * (double)n));
    hipLaunchKernelGGL(pretrain_step_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream, theta, n, train_bits,
                       words, pos_weight, inv_count, exp_avg, exp_avg_sq, (float)beta1, (float)beta2,
                       (float)(1.0 - beta1), (float)(1.0 - beta2), (float)eps, (float)(lr / bc1),
                       (float)sqrt(bc2), loss_rows);
    LDS_RETURN_LAST_ERROR();
}
