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

// one thread per (row m, 8 consecutive k): gathers the taps from the NCHW fp32 images.  The
// k -> (c, r, s) decomposition is a per-block LDS table of input offsets (c*H*W + r*W + s) and
// taps; the row index is split with 32-bit arithmetic (host-checked M * Kp/8 < 2^31): the 64-bit
// divisions per element of the first version made this a 1 TB/s integer-bound pass
constexpr int kMaxStemK = 2048;  // C*R*S of a stem (7x7: up to 41 input channels)
template <int DT>
__global__ __launch_bounds__(256) void im2col_kernel(const float* __restrict__ x, int C, int H,
                                                     int W, int R, int S, int stride, int pad,
                                                     int Ho, int Wo, int K, int Kp, long long M,
                                                     void* __restrict__ out) {
  __shared__ int tab_off[kMaxStemK], tab_rs[kMaxStemK];
  const int RS = R * S;
  for (int k = threadIdx.x; k < Kp; k += 256) {
    if (k < K) {
      const int c = k / RS, rs = k - c * RS, r = rs / S, q = rs - r * S;
      tab_off[k] = (c * H + r) * W + q;
      tab_rs[k] = (r << 16) | q;
    } else {
      tab_off[k] = 0;
      tab_rs[k] = -1;   // zero padding of K
    }
  }
  __syncthreads();
  const int kc = Kp / 8;
  const unsigned total = (unsigned)(M * kc);
  const unsigned HW = (unsigned)(Ho * Wo);
  const long long CHW = (long long)C * H * W;
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const unsigned m = i / (unsigned)kc;
    const int k0 = 8 * (int)(i - m * (unsigned)kc);
    const unsigned b = m / HW, rem = m - b * HW;
    const int oh = (int)(rem / (unsigned)Wo), ow = (int)rem - oh * Wo;
    const int ih0 = oh * stride - pad, iw0 = ow * stride - pad;
    const float* xb = x + (long long)b * CHW + (long long)ih0 * W + iw0;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int rs = tab_rs[k0 + e];
      const int ih = ih0 + (rs >> 16), iw = iw0 + (rs & 0xffff);
      v[e] = (rs >= 0 && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
                 ? xb[tab_off[k0 + e]] : 0.f;
    }
    if constexpr (DT < 0) {
      float* o = (float*)out + (long long)m * Kp + k0;
      *(floatx4*)o = floatx4{v[0], v[1], v[2], v[3]};
      *(floatx4*)(o + 4) = floatx4{v[4], v[5], v[6], v[7]};
    } else {
      const floatx8 f = {v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]};
      *(u32x4*)((u16*)out + (long long)m * Kp + k0) = pack8<DT>(f);   // RNE, as every 16-bit store
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
  if (n >= (1LL << 31) || Kp > kMaxStemK || S > 0xffff) {
    set_error("stem_im2col: more than 2^31 row chunks or Kp > 2048");
    return kErrArg;
  }
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
