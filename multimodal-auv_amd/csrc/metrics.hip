// Evaluation metrics on the device.
//
// The reference's evaluation pulls every batch's predictions, labels and uncertainties to the
// host (train/multimodal.py:312-321 `.cpu().numpy()` per batch) and runs sklearn once per
// epoch: confusion_matrix (:322-347), and in the noise scripts
// (Examples/"Example training with image noise.py":530-634) roc_auc_score of the
// uncertainty against the error indicator, macro F1 and a 15-bin expected / maximum
// calibration error of the MC-mean softmax.  Here the per-sample work stays on the GPU:
//  * mauv_confusion_update  — C x C counts (int32 atomics), labels outside [0, C) counted in
//                             slot C*C so the host can refuse them;
//  * mauv_calibration_update — per bin (count, sum of confidences, correct count) with the
//                             reference's bin rule conf in (b_i, b_i+1] on float64 edges
//                             (np.linspace) and its argmax (first maximum);
//  * mauv_auroc_pairs       — the Mann-Whitney count over (positive, negative) pairs,
//                             s_pos > s_neg counts 2, ties 1 (exact integers), which equals
//                             sklearn's trapezoidal ROC area times 2 * n_pos * n_neg.
#include "mauv_common.h"

using namespace mauv;

namespace mauv {

__global__ __launch_bounds__(256) void confusion_kernel(const long long* __restrict__ labels,
                                                        const long long* __restrict__ pred,
                                                        int n, int C, int* __restrict__ counts) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const long long y = labels[i], p = pred[i];
    const bool ok = y >= 0 && y < C && p >= 0 && p < C;
    atomicAdd(counts + (ok ? (int)(y * C + p) : C * C), 1);
  }
}

// (v2, i2) replaces (v1, i1) in np.argmax order: a NaN wins, then the larger value, then the
// smaller index
__device__ __forceinline__ bool argmax_better(float v1, int i1, float v2, int i2) {
  const bool n1 = v1 != v1, n2 = v2 != v2;
  if (n1 != n2) return n2;
  if (n1 || v1 == v2) return i2 < i1;
  return v2 > v1;
}

// one wave per sample row (lanes stride the classes)
__global__ __launch_bounds__(256) void calibration_kernel(const float* __restrict__ probs,
                                                          const long long* __restrict__ labels,
                                                          int n, int C, int nbins,
                                                          const double* __restrict__ edges,
                                                          double* __restrict__ bins) {
  const int lane = threadIdx.x & 63;
  for (int r = blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += gridDim.x * 4) {
    const float* p = probs + (long long)r * C;
    float best = -INFINITY;
    int arg = C;   // sentinel index: loses every tie
    for (int c = lane; c < C; c += 64) {
      const float v = p[c];
      if (argmax_better(best, arg, v, c)) { best = v; arg = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oa = __shfl_xor(arg, o, 64);
      if (argmax_better(best, arg, ob, oa)) { best = ob; arg = oa; }
    }
    if (lane == 0) {
      const double conf = (double)best;
      int bi = -1;
      for (int b = 0; b < nbins; ++b)
        if (conf > edges[b] && conf <= edges[b + 1]) { bi = b; break; }
      if (bi >= 0) {
        atomicAdd(bins + 3 * bi, 1.0);
        atomicAdd(bins + 3 * bi + 1, conf);
        atomicAdd(bins + 3 * bi + 2, (long long)arg == labels[r] ? 1.0 : 0.0);
      }
    }
  }
}

// pairs (i positive, j negative); each block takes 256 i's and sweeps all j through LDS
__global__ __launch_bounds__(256) void auroc_kernel(const float* __restrict__ score,
                                                    const unsigned char* __restrict__ pos, int n,
                                                    unsigned long long* __restrict__ out) {
  __shared__ float s_s[256];
  __shared__ unsigned char s_p[256];
  const int i = blockIdx.x * 256 + threadIdx.x;
  const bool mine = i < n && pos[i];
  const float si = i < n ? score[i] : 0.f;
  unsigned long long acc = 0;
  for (int j0 = 0; j0 < n; j0 += 256) {
    const int j = j0 + threadIdx.x;
    s_s[threadIdx.x] = j < n ? score[j] : 0.f;
    s_p[threadIdx.x] = j < n ? pos[j] : 1;   // padding counts as positive: never paired
    __syncthreads();
    if (mine) {
      const int m = min(256, n - j0);
      for (int k = 0; k < m; ++k)
        if (!s_p[k]) acc += si > s_s[k] ? 2u : (si == s_s[k] ? 1u : 0u);
    }
    __syncthreads();
  }
  // block reduction, one 64-bit atomic per wave
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

static int grid_n(long long n, int per, int cap) {
  long long b = (n + per - 1) / per;
  if (b > cap) b = cap;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace mauv

MAUV_API int mauv_confusion_update(const long long* labels, const long long* pred, int n, int C,
                                   int* counts, hipStream_t stream) {
  if (n < 0 || C < 1 || C > 4096) { set_error("confusion_update: bad n / C"); return kErrArg; }
  if (n == 0) return 0;
  hipLaunchKernelGGL(confusion_kernel, dim3(grid_n(n, 256, 1024)), dim3(256), 0, stream, labels,
                     pred, n, C, counts);
  return check_launch("confusion_update");
}

MAUV_API int mauv_calibration_update(const float* probs, const long long* labels, int n, int C,
                                     int nbins, const double* edges, double* bins,
                                     hipStream_t stream) {
  if (n < 0 || C < 1 || nbins < 1) { set_error("calibration_update: bad n / C / bins"); return kErrArg; }
  if (n == 0) return 0;
  hipLaunchKernelGGL(calibration_kernel, dim3(grid_n(n, 4, 4096)), dim3(256), 0, stream, probs,
                     labels, n, C, nbins, edges, bins);
  return check_launch("calibration_update");
}

MAUV_API int mauv_auroc_pairs(const float* score, const unsigned char* positive, int n,
                              unsigned long long* count2, hipStream_t stream) {
  if (n < 0) { set_error("auroc_pairs: bad n"); return kErrArg; }
  if (n == 0) return 0;
  hipLaunchKernelGGL(auroc_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, score, positive, n,
                     count2);
  return check_launch("auroc_pairs");
}
