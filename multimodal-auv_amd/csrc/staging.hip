// Input staging on the device.
//
//  * data/datasets.py:239-250 (CustomImageDataset.__getitem__, :343-352): every tile is
//    decoded by PIL and turned into fp32 on CPU workers — ToTensor (x / 255, HWC -> CHW) and,
//    for the optical tile, Normalize((x - mean) / std) — and train/multimodal.py:87-94 copies
//    the fp32 tensors (and every patch size) to the GPU.  mauv_stage_u8 takes the decoded
//    uint8 HWC tiles instead (4x fewer bytes over PCIe) and does ToTensor + Normalize on the
//    device, with the same fp32 operations in the same order (bit-exact).
//  * Example training with image noise.py:55-93 (simulate_underwater_degradation, applied to
//    the normalised optical batch at :237-262): the underwater image formation model
//        t = exp(-beta_c * turbidity * d * depth);  I = clamp(J * t + B_inf,c * (1 - t), 0, 1)
//    with beta = (0.8, 0.5, 0.3), B_inf = (0.1, 0.3, 0.5) and d a [B][1][H][W] distance map
//    (the script passes a map of ones).  mauv_uifm applies it to fp32 NCHW tiles;
//    mauv_stage_u8 can apply it in the same pass as the normalisation (one read of the uint8
//    tile, one fp32 write).
// Both kernels are HBM-bound element-wise passes: 4 consecutive pixels of one (b, c, h) row
// per thread, 16-byte output stores.
#include "mauv_common.h"

using namespace mauv;

namespace mauv {

struct StageArgs {
  const unsigned char* x;  // uint8 [B][H][W][C] (mauv_stage_u8) or null
  const float* xf;         // fp32 [B][C][H][W] (mauv_uifm) or null
  int B, C, H, W;
  const float* mean;       // [C] or null
  const float* stdv;       // [C] or null
  const float* bt;         // [C]: beta_c * turbidity (fp32, as the reference computes it) or null
  const float* binf;       // [C]
  const float* dist;       // [B][1][H][W] or null (uniform distance 1)
  float depth;
  float* out;              // fp32 [B][C][H][W]
};

__device__ __forceinline__ float uifm1(float j, float bt, float binf, float d, float depth) {
  // reference order: d = map * depth; t = exp(-beta * d); J * t + B_inf * (1 - t); clamp
  // separate roundings as the reference's tensor ops (no fma contraction)
  const float t = expf(__fmul_rn(-bt, __fmul_rn(d, depth)));
  const float v = __fadd_rn(__fmul_rn(j, t), __fmul_rn(binf, __fadd_rn(1.0f, -t)));
  return fminf(fmaxf(v, 0.0f), 1.0f);
}

__global__ __launch_bounds__(256) void stage_kernel(const StageArgs a) {
  const int W4 = (a.W + 3) >> 2;
  const long long total = (long long)a.B * a.C * a.H * W4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int w4 = (int)(i % W4);
    long long r = i / W4;
    const int h = (int)(r % a.H);
    r /= a.H;
    const int c = (int)(r % a.C);
    const int b = (int)(r / a.C);
    const int w0 = 4 * w4;
    const int nw = min(4, a.W - w0);
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int w = w0 + (e < nw ? e : 0);
      float x;
      if (a.x) {
        // ToTensor: img.float().div(255) (torchvision functional.to_tensor)
        x = (float)a.x[(((long long)b * a.H + h) * a.W + w) * a.C + c] / 255.0f;
        // Normalize: tensor.sub_(mean).div_(std)
        if (a.mean) x = (x - a.mean[c]) / a.stdv[c];
      } else {
        x = a.xf[(((long long)b * a.C + c) * a.H + h) * a.W + w];
      }
      if (a.bt) {
        const float d = a.dist ? a.dist[((long long)b * a.H + h) * a.W + w] : 1.0f;
        x = uifm1(x, a.bt[c], a.binf[c], d, a.depth);
      }
      v[e] = x;
    }
    float* o = a.out + (((long long)b * a.C + c) * a.H + h) * a.W + w0;
    if (nw == 4 && (a.W & 3) == 0) {
      *(floatx4*)o = floatx4{v[0], v[1], v[2], v[3]};
    } else {
      for (int e = 0; e < nw; ++e) o[e] = v[e];
    }
  }
}

static int stage_grid(long long n) {
  long long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  return (int)(b < 1 ? 1 : b);
}

static int stage_launch(const StageArgs& a, hipStream_t stream, const char* what) {
  if (a.B < 0 || a.C < 1 || a.H < 0 || a.W < 0) {
    set_error(std::string(what) + ": bad shape or null output");
    return kErrArg;
  }
  if ((a.mean == nullptr) != (a.stdv == nullptr) || (a.bt && !a.binf)) {
    set_error(std::string(what) + ": mean/std and bt/binf come in pairs");
    return kErrArg;
  }
  const long long n = (long long)a.B * a.C * a.H * ((a.W + 3) / 4);
  if (n == 0) return 0;
  if ((!a.x && !a.xf) || !a.out) { set_error(std::string(what) + ": null input / output"); return kErrArg; }
  hipLaunchKernelGGL(stage_kernel, dim3(stage_grid(n)), dim3(256), 0, stream, a);
  return check_launch(what);
}

}  // namespace mauv

MAUV_API int mauv_stage_u8(const unsigned char* x, int B, int H, int W, int C, const float* mean,
                           const float* stdv, const float* uifm_bt, const float* uifm_binf,
                           const float* dist, float depth, float* out, hipStream_t stream) {
  StageArgs a{x, nullptr, B, C, H, W, mean, stdv, uifm_bt, uifm_binf, dist, depth, out};
  return stage_launch(a, stream, "stage_u8");
}

MAUV_API int mauv_uifm(const float* x, int B, int C, int H, int W, const float* bt,
                       const float* binf, const float* dist, float depth, float* out,
                       hipStream_t stream) {
  StageArgs a{nullptr, x, B, C, H, W, nullptr, nullptr, bt, binf, dist, depth, out};
  if (!bt) { set_error("uifm: null bt"); return kErrArg; }
  return stage_launch(a, stream, "uifm");
}
