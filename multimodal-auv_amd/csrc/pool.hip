// ResNet-50 stem max-pool (3x3 / 2, pad 1) and the adaptive average pool to 1x1, NHWC,
// forward + backward (torchvision resnet50 as used at models/base_models.py:15 and
// models/model_utils.py:57).  N = G*B images (the MC groups are just more images here).
#include "mauv_common.h"

using namespace mauv;

namespace mauv {

// Tie-break as torch's max_pool2d: first maximum in (kh, kw) scan order; NaN wins.
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const float* __restrict__ x, int N,
                                                          int H, int W, int C, int Ho, int Wo,
                                                          float* __restrict__ y,
                                                          unsigned char* __restrict__ idx) {
  const long long total = (long long)N * Ho * Wo * C;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    long long p = i / C;
    const int ow = (int)(p % Wo); p /= Wo;
    const int oh = (int)(p % Ho);
    const int n = (int)(p / Ho);
    float best = -INFINITY;
    int bi = 0;
    for (int r = 0; r < 3; ++r) {
      const int ih = oh * 2 - 1 + r;
      if (ih < 0 || ih >= H) continue;
      for (int s = 0; s < 3; ++s) {
        const int iw = ow * 2 - 1 + s;
        if (iw < 0 || iw >= W) continue;
        const float v = x[(((long long)n * H + ih) * W + iw) * C + c];
        if (v > best || isnan(v)) { best = v; bi = r * 3 + s; }
      }
    }
    y[i] = best;
    idx[i] = (unsigned char)bi;
  }
}

__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const float* __restrict__ dy,
                                                          const unsigned char* __restrict__ idx,
                                                          int N, int H, int W, int C, int Ho,
                                                          int Wo, float* __restrict__ dx) {
  const long long total = (long long)N * H * W * C;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    long long p = i / C;
    const int iw = (int)(p % W); p /= W;
    const int ih = (int)(p % H);
    const int n = (int)(p / H);
    float acc = 0.f;
    const int oh_lo = max(0, ih / 2), oh_hi = min(Ho - 1, (ih + 1) / 2);
    const int ow_lo = max(0, iw / 2), ow_hi = min(Wo - 1, (iw + 1) / 2);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int r = ih - (oh * 2 - 1);
      if (r < 0 || r > 2) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int s = iw - (ow * 2 - 1);
        if (s < 0 || s > 2) continue;
        const long long o = (((long long)n * Ho + oh) * Wo + ow) * C + c;
        if (idx[o] == r * 3 + s) acc += dy[o];
      }
    }
    dx[i] = acc;
  }
}

__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const float* __restrict__ x, int N,
                                                          int HW, int C, float* __restrict__ y) {
  const long long total = (long long)N * C;
  const float inv = 1.0f / (float)HW;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long long n = i / C;
    const float* src = x + n * HW * C + c;
    float acc = 0.f;
    for (int p = 0; p < HW; ++p) acc += src[(long long)p * C];
    y[i] = acc * inv;
  }
}

__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const float* __restrict__ dy, int N,
                                                          int HW, int C, float* __restrict__ dx) {
  const long long total = (long long)N * HW * C;
  const float inv = 1.0f / (float)HW;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long long n = i / ((long long)HW * C);
    dx[i] = dy[n * C + c] * inv;
  }
}

static int grid1(long long n) {
  long long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace mauv

MAUV_API int mauv_maxpool_fwd(const float* x, int N, int H, int W, int C, float* y,
                              unsigned char* idx, hipStream_t stream) {
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid1((long long)N * Ho * Wo * C)), dim3(256), 0,
                     stream, x, N, H, W, C, Ho, Wo, y, idx);
  return check_launch("maxpool_fwd");
}

MAUV_API int mauv_maxpool_bwd(const float* dy, const unsigned char* idx, int N, int H, int W,
                              int C, float* dx, hipStream_t stream) {
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid1((long long)N * H * W * C)), dim3(256), 0,
                     stream, dy, idx, N, H, W, C, Ho, Wo, dx);
  return check_launch("maxpool_bwd");
}

MAUV_API int mauv_avgpool_fwd(const float* x, int N, int HW, int C, float* y, hipStream_t stream) {
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(grid1((long long)N * C)), dim3(256), 0, stream, x,
                     N, HW, C, y);
  return check_launch("avgpool_fwd");
}

MAUV_API int mauv_avgpool_bwd(const float* dy, int N, int HW, int C, float* dx,
                              hipStream_t stream) {
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid1((long long)N * HW * C)), dim3(256), 0,
                     stream, dy, N, HW, C, dx);
  return check_launch("avgpool_bwd");
}
