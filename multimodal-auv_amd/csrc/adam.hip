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

// One element of torch's Adam update (m, v, p updated in place).
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float omb1,
                                          float beta2, float omb2, float eps, float wd,
                                          float step_size, float bc2_sqrt) {
  const float ge = wd != 0.f ? g + wd * p : g;
  m = m + omb1 * (ge - m);
  v = v * beta2 + omb2 * ge * ge;
  p = p - step_size * (m / (sqrtf(v) / bc2_sqrt + eps));
}

// MODE 1: Adam update; MODE 3: Adam update, then the gradient is zeroed (the reference's
// optimizer.zero_grad() after a successful step, multimodal.py:141-143); MODE 2: zero the
// gradient only.  The gated launch reads the mode and constants from the device gate.
template <bool GATED>
__global__ __launch_bounds__(256) void adam_kernel(const MauvAdamEntry* __restrict__ tab,
                                                   float lr, float beta1, float beta2, float eps,
                                                   float wd, float step_size, float bc2_sqrt,
                                                   const MauvStepGate* __restrict__ gate) {
  int mode = 1;
  if (GATED) {
    mode = gate->mode;
    if (mode == 0) return;
    step_size = gate->step_size;
    bc2_sqrt = gate->bc2_sqrt;
  }
  const MauvAdamEntry t = tab[blockIdx.y];
  float* grad = const_cast<float*>(t.grad);
  const bool upd = mode & 1, zero = mode & 2;
  // 16-byte vector path only when all four tensors are 16-byte aligned (a parameter may be
  // a view at any offset); otherwise every element takes the scalar loop below
  const bool aligned = ((reinterpret_cast<uintptr_t>(t.param) | reinterpret_cast<uintptr_t>(t.grad) |
                         reinterpret_cast<uintptr_t>(t.exp_avg) |
                         reinterpret_cast<uintptr_t>(t.exp_avg_sq)) & 15) == 0;
  const long long n4 = aligned ? t.numel / 4 : 0;
  const float omb1 = 1.0f - beta1, omb2 = 1.0f - beta2;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    if (upd) {
      floatx4 p = ((const floatx4*)t.param)[i];
      floatx4 g = ((const floatx4*)t.grad)[i];
      floatx4 m = ((const floatx4*)t.exp_avg)[i];
      floatx4 v = ((const floatx4*)t.exp_avg_sq)[i];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float pe = p[e], me = m[e], ve = v[e];
        adam_elem(pe, g[e], me, ve, omb1, beta2, omb2, eps, wd, step_size, bc2_sqrt);
        p[e] = pe; m[e] = me; v[e] = ve;
      }
      ((floatx4*)t.param)[i] = p;
      ((floatx4*)t.exp_avg)[i] = m;
      ((floatx4*)t.exp_avg_sq)[i] = v;
    }
    if (zero) ((floatx4*)grad)[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  // scalar tail
  const long long base = n4 * 4;
  for (long long i = base + blockIdx.x * 256LL + threadIdx.x; i < t.numel;
       i += (long long)gridDim.x * 256) {
    if (upd) {
      float p = t.param[i], m = t.exp_avg[i], v = t.exp_avg_sq[i];
      adam_elem(p, t.grad[i], m, v, omb1, beta2, omb2, eps, wd, step_size, bc2_sqrt);
      t.param[i] = p;
      t.exp_avg[i] = m;
      t.exp_avg_sq[i] = v;
    }
    if (zero) grad[i] = 0.f;
  }
}

// The step decision of train/multimodal.py:133-145 taken on the device (one thread):
//   loss non-finite  -> no step; the batch's gradients are taken back out of the arena
//                       (mode 2 zeroes it when it was clean before; a poisoned arena stays)
//   grads non-finite -> no step, no zero_grad: the arena keeps them ("poisoned")
//   otherwise        -> Adam at step count t+1, then zero_grad (mode 3)
// and the non-finite counter is reset for the next scan.
__global__ void step_gate_kernel(MauvStepGate* g, float lr, float beta1, float beta2) {
  const int ok_loss = g->ok_loss != 0, ok_grad = g->nonfinite == 0;
  if (ok_loss && ok_grad) {
    const int t = g->step + 1;
    const double bc1 = 1.0 - pow((double)beta1, (double)t);
    const double bc2 = 1.0 - pow((double)beta2, (double)t);
    g->step = t;
    g->step_size = (float)((double)lr / bc1);
    g->bc2_sqrt = (float)sqrt(bc2);
    g->mode = 3;
    g->poisoned = 0;
    g->stepped = 1;
  } else {
    g->stepped = 0;
    if (!ok_loss) {
      g->mode = g->poisoned ? 0 : 2;
      g->skipped_loss += 1;
    } else {
      g->mode = 0;
      g->poisoned = 1;
      g->skipped_grad += 1;
    }
  }
  g->nonfinite = 0;
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
  hipLaunchKernelGGL(adam_kernel<false>, dim3(64, n), dim3(256), 0, stream, table, lr, beta1,
                     beta2, eps, weight_decay, (float)(lr / bc1), (float)sqrt(bc2), nullptr);
  return check_launch("adam_step");
}

// The same step gated on the device (no host round trip): the caller has written
// gate->ok_loss before the backward and counted the arena's non-finite elements into
// gate->nonfinite after it (mauv_nonfinite_count); the step count lives in gate->step.
MAUV_API int mauv_adam_step_gated(const MauvAdamEntry* table, int n, float lr, float beta1,
                                  float beta2, float eps, float weight_decay, MauvStepGate* gate,
                                  hipStream_t stream) {
  if (n <= 0 || n > 65535 || !gate) { set_error("adam_step_gated: bad table size / gate"); return kErrArg; }
  hipLaunchKernelGGL(step_gate_kernel, dim3(1), dim3(1), 0, stream, gate, lr, beta1, beta2);
  hipLaunchKernelGGL(adam_kernel<true>, dim3(64, n), dim3(256), 0, stream, table, lr, beta1,
                     beta2, eps, weight_decay, 0.f, 1.f, (const MauvStepGate*)gate);
  return check_launch("adam_step_gated");
}
