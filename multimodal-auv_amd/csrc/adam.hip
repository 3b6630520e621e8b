// Fused multi-tensor Adam for the Bayesian parameter set.
//
// The reference builds torch.optim.Adam over the model's ~700 parameter tensors
// (train/loop_utils.py:45-61; lr 5e-5, weight_decay 1e-5 when retraining) and steps it after
// every batch (train/multimodal.py:141-143).  This is the same update — torch's Adam with
// amsgrad=False, maximize=False, L2 weight decay folded into the gradient — for every tensor of
// a table in ONE launch (grid.y = table entry), one read and one write of p, m, v and one read
// of g per element:
//   g' = g + wd * p;  m = m + (1 - b1) * (g' - m);  v = b2 * v + (1 - b2) * g'^2
//   p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
#include "mauv_common.h"

using namespace mauv;

namespace mauv {

__global__ __launch_bounds__(256) void adam_kernel(const MauvAdamEntry* __restrict__ tab,
                                                   float lr, float beta1, float beta2, float eps,
                                                   float wd, float step_size, float bc2_sqrt) {
  const MauvAdamEntry t = tab[blockIdx.y];
  // 16-byte vector path only when all four tensors are 16-byte aligned (a parameter may be
  // a view at any offset); otherwise every element takes the scalar loop below
  const bool aligned = ((reinterpret_cast<uintptr_t>(t.param) | reinterpret_cast<uintptr_t>(t.grad) |
                         reinterpret_cast<uintptr_t>(t.exp_avg) |
                         reinterpret_cast<uintptr_t>(t.exp_avg_sq)) & 15) == 0;
  const long long n4 = aligned ? t.numel / 4 : 0;
  const float omb1 = 1.0f - beta1, omb2 = 1.0f - beta2;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    floatx4 p = ((const floatx4*)t.param)[i];
    floatx4 g = ((const floatx4*)t.grad)[i];
    floatx4 m = ((const floatx4*)t.exp_avg)[i];
    floatx4 v = ((const floatx4*)t.exp_avg_sq)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float ge = wd != 0.f ? g[e] + wd * p[e] : g[e];
      m[e] = m[e] + omb1 * (ge - m[e]);
      v[e] = v[e] * beta2 + omb2 * ge * ge;
      p[e] = p[e] - step_size * (m[e] / (sqrtf(v[e]) / bc2_sqrt + eps));
    }
    ((floatx4*)t.param)[i] = p;
    ((floatx4*)t.exp_avg)[i] = m;
    ((floatx4*)t.exp_avg_sq)[i] = v;
  }
  // scalar tail
  const long long base = n4 * 4;
  for (long long i = base + blockIdx.x * 256LL + threadIdx.x; i < t.numel;
       i += (long long)gridDim.x * 256) {
    float p = t.param[i], g = t.grad[i], m = t.exp_avg[i], v = t.exp_avg_sq[i];
    const float ge = wd != 0.f ? g + wd * p : g;
    m = m + omb1 * (ge - m);
    v = v * beta2 + omb2 * ge * ge;
    p = p - step_size * (m / (sqrtf(v) / bc2_sqrt + eps));
    t.param[i] = p;
    t.exp_avg[i] = m;
    t.exp_avg_sq[i] = v;
  }
}

}  // namespace mauv

// One Adam step (bias-correction step index `step` >= 1, shared by the table) for n tensors.
// Entries whose pointers are all 16-byte aligned take 16-byte vector loads, others scalar ones.
MAUV_API int mauv_adam_step(const MauvAdamEntry* table, int n, float lr, float beta1,
                            float beta2, float eps, float weight_decay, long long step,
                            hipStream_t stream) {
  if (n <= 0 || n > 65535 || step < 1) { set_error("adam_step: bad table size / step"); return kErrArg; }
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  hipLaunchKernelGGL(adam_kernel, dim3(64, n), dim3(256), 0, stream, table, lr, beta1, beta2, eps,
                     weight_decay, (float)(lr / bc1), (float)sqrt(bc2));
  return check_launch("adam_step");
}
