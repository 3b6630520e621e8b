// The ResNet-50 stems (conv1: 7x7 / 2 over the 3-channel optical / bathy and 1-channel SSS
// tiles, models/base_models.py:18, models/model_utils.py:58-59) as a GEMM over im2col rows.
//
// Every MC sample of a batch convolves the SAME images with its own sampled weights
// (train/multimodal.py:107-112: the loop re-runs the model on identical inputs).  The
// per-sample implicit GEMM (G launches of M x 64 x 147 on 3 zero-padded channels per tap)
// wastes 25-75 % of its K on padding and re-reads the image G times with only 64 output
// columns per read.  Here the image is unrolled ONCE into rows cols[m][k], k = c*R*S + r*S + s
// (the OIHW parameter order: the sampled weights need no transpose), zero-padded to Kp (a
// multiple of the GEMM's K slice: 32 fp32 / 64 16-bit), and the G weight sets are stacked
// along N: one GEMM M x (G*64) x Kp whose epilogue writes each group's output and BN
// statistics (mauv_stem_fwd_f32 / _h16, ConvArgs::cpg).  The weight gradient is the per-group
// 1x1 weight-gradient GEMM over the same rows (group stride 0).
#include "h16.h"

using namespace mauv;

namespace mauv {

// one thread per (row m, 8 consecutive k): gathers the taps from the NCHW fp32 images
template <int DT>
__global__ __launch_bounds__(256) void im2col_kernel(const float* __restrict__ x, int C, int H,
                                                     int W, int R, int S, int stride, int pad,
                                                     int Ho, int Wo, int K, int Kp, long long M,
                                                     void* __restrict__ out) {
  const int kc = Kp / 8;
  const long long total = M * kc;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long m = i / kc;
    const int k0 = 8 * (int)(i - m * kc);
    const int HW = Ho * Wo;
    const int b = (int)(m / HW), rem = (int)(m - (long long)b * HW);
    const int oh = rem / Wo, ow = rem - oh * Wo;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = k0 + e;
      float t = 0.f;
      if (k < K) {
        const int c = k / (R * S), rs = k - c * (R * S), r = rs / S, s = rs - r * S;
        const int ih = oh * stride - pad + r, iw = ow * stride - pad + s;
        if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
          t = x[(((long long)b * C + c) * H + ih) * W + iw];
      }
      v[e] = t;
    }
    if constexpr (DT < 0) {
      float* o = (float*)out + m * Kp + k0;
      *(floatx4*)o = floatx4{v[0], v[1], v[2], v[3]};
      *(floatx4*)(o + 4) = floatx4{v[4], v[5], v[6], v[7]};
    } else {
      const floatx8 f = {v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]};
      *(u32x4*)((u16*)out + m * Kp + k0) = pack8<DT>(f);   // RNE, as every 16-bit store
    }
  }
}

}  // namespace mauv

// dtype -1 = fp32, 0 = bf16, 1 = f16 rows; Kp % 8 == 0 and Kp >= C*R*S.
MAUV_API int mauv_stem_im2col(int dtype, const float* x, int B, int C, int H, int W, int R, int S,
                              int stride, int pad, int Kp, void* out, hipStream_t stream) {
  const int K = C * R * S;
  if (B <= 0 || C <= 0 || R <= 0 || S <= 0 || stride <= 0 || Kp < K || Kp % 8 ||
      dtype < -1 || dtype > 1) {
    set_error("stem_im2col: bad shape / dtype (Kp % 8 == 0, Kp >= C*R*S)");
    return kErrArg;
  }
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  const long long M = (long long)B * Ho * Wo;
  if (Ho <= 0 || Wo <= 0) { set_error("stem_im2col: empty output"); return kErrArg; }
  const long long n = M * (Kp / 8);
  long long nb = (n + 255) / 256;
  if (nb > 16384) nb = 16384;
  const dim3 grid((unsigned)nb);
  if (dtype < 0)
    hipLaunchKernelGGL(im2col_kernel<-1>, grid, dim3(256), 0, stream, x, C, H, W, R, S, stride, pad, Ho, Wo, K, Kp, M, out);
  else if (dtype == DT_BF16)
    hipLaunchKernelGGL(im2col_kernel<DT_BF16>, grid, dim3(256), 0, stream, x, C, H, W, R, S, stride, pad, Ho, Wo, K, Kp, M, out);
  else
    hipLaunchKernelGGL(im2col_kernel<DT_F16>, grid, dim3(256), 0, stream, x, C, H, W, R, S, stride, pad, Ho, Wo, K, Kp, M, out);
  return check_launch("stem_im2col");
}
