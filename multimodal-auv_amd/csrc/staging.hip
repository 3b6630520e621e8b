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

// ToTensor (+ Normalize) (+ UIFM) of one uint8 sample of channel c at (b, h, w)
__device__ __forceinline__ float stage_u8_val(const StageArgs& a, unsigned v, int b, int c, int h,
                                              int w) {
  // ToTensor: img.float().div(255) (torchvision functional.to_tensor)
  float x = (float)v / 255.0f;
  // Normalize: tensor.sub_(mean).div_(std)
  if (a.mean) x = (x - a.mean[c]) / a.stdv[c];
  if (a.bt) {
    const float d = a.dist ? a.dist[((long long)b * a.H + h) * a.W + w] : 1.0f;
    x = uifm1(x, a.bt[c], a.binf[c], d, a.depth);
  }
  return x;
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
        x = stage_u8_val(a, a.x[(((long long)b * a.H + h) * a.W + w) * a.C + c], b, c, h, w);
      } else {
        x = a.xf[(((long long)b * a.C + c) * a.H + h) * a.W + w];
        if (a.bt) {
          const float d = a.dist ? a.dist[((long long)b * a.H + h) * a.W + w] : 1.0f;
          x = uifm1(x, a.bt[c], a.binf[c], d, a.depth);
        }
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

// ---------------------------------------------------------------------------------- Resize
// data/datasets.py:240-246: transforms.Resize((256, 256)) of every PIL tile before ToTensor /
// Normalize = PIL's Image.resize(size, BILINEAR) (PIL always antialiases).  Pillow's 8-bit
// separable resampler (libImaging/Resample.c; the reference pins pillow 11.0.0), restated:
//  * coefficients per output position o of a pass (in -> out): scale = in / out, filterscale =
//    max(scale, 1), support = filterscale (triangle filter of radius 1, widened when
//    downscaling), center = (o + 0.5) * scale, taps xmin = max((int)(center - support + 0.5), 0)
//    .. min((int)(center + support + 0.5), in) - 1, w_x = tri((x - center + 0.5) / filterscale)
//    normalised by their double sum, then (int)(0.5 + w * 2^22) — all in double, no FMA
//    contraction (PIL's x86-64 build issues separate multiplies and adds);
//  * a pass: acc = 2^21 + sum_x v_x * k_x (int32), out = clamp(acc >> 22, 0, 255) — the
//    horizontal pass into an 8-bit intermediate [B][H][Wo][C], then the vertical pass (each
//    only when its size changes, as ImagingResample does).
// The vertical pass optionally ends in the staging maths above (ToTensor, Normalize, UIFM):
// one fp32 NCHW write instead of an 8-bit image and a second pass.
constexpr int kResizeBits = 22;

__device__ __forceinline__ double tri_filter(double x) {
  if (x < 0.0) x = -x;
  return x < 1.0 ? 1.0 - x : 0.0;
}

// one thread per output position: bounds[o] = (xmin, n), kk[o][0..ksize) fixed point
__global__ __launch_bounds__(256) void resize_coeffs_kernel(int in, int out, int ksize,
                                                            int* bounds, int* kk) {
#pragma clang fp contract(off)
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= out) return;
  const double scale = (double)in / (double)out;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale, ss = 1.0 / filterscale;
  const double center = 0.0 + ((double)o + 0.5) * scale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in) xmax = in;
  xmax -= xmin;
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) ww += tri_filter(((double)(x + xmin) - center + 0.5) * ss);
  for (int x = 0; x < ksize; ++x) {
    int k = 0;
    if (x < xmax) {
      double w = tri_filter(((double)(x + xmin) - center + 0.5) * ss);
      if (ww != 0.0) w /= ww;
      k = w < 0.0 ? (int)(-0.5 + w * (double)(1 << kResizeBits))
                  : (int)(0.5 + w * (double)(1 << kResizeBits));
    }
    kk[(long long)o * ksize + x] = k;
  }
  bounds[2 * o] = xmin;
  bounds[2 * o + 1] = xmax;
}

__device__ __forceinline__ unsigned clip8_acc(int acc) {
  const int v = acc >> kResizeBits;
  return (unsigned)(v < 0 ? 0 : v > 255 ? 255 : v);
}

struct ResizeArgs {
  const unsigned char* x;  // [B][H][W][C]
  int B, H, W, C, Ho, Wo;
  const int *hb, *hk, *vb, *vk;  // horizontal / vertical bounds + coefficients (null: no pass)
  int hks, vks;
  unsigned char* tmp;      // [B][H][Wo][C] (both passes) or null
  unsigned char* out8;     // [B][Ho][Wo][C] or null
  StageArgs st;            // out8 null: fused staging into st.out [B][C][Ho][Wo]
};

// horizontal pass: one thread per (b, h, output column), all C channels
__global__ __launch_bounds__(256) void resize_h_kernel(const ResizeArgs a) {
  const long long n = (long long)a.B * a.H * a.Wo;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int xo = (int)(i % a.Wo);
    const long long bh = i / a.Wo;
    const int xmin = a.hb[2 * xo], nx = a.hb[2 * xo + 1];
    const int* k = a.hk + (long long)xo * a.hks;
    const unsigned char* src = a.x + (bh * a.W + xmin) * a.C;
    int acc[4] = {1 << (kResizeBits - 1), 1 << (kResizeBits - 1), 1 << (kResizeBits - 1),
                  1 << (kResizeBits - 1)};
    for (int t = 0; t < nx; ++t) {
      const int kt = k[t];
      for (int c = 0; c < a.C; ++c) acc[c] += (int)src[t * a.C + c] * kt;
    }
    unsigned char* dst = a.tmp + (bh * a.Wo + xo) * a.C;
    for (int c = 0; c < a.C; ++c) dst[c] = (unsigned char)clip8_acc(acc[c]);
  }
}

// vertical pass (or the only pass): one thread per (b, output row, output column); the source
// is tmp [B][H][Wo][C] after a horizontal pass, else x (W == Wo)
__global__ __launch_bounds__(256) void resize_v_kernel(const ResizeArgs a) {
  const long long n = (long long)a.B * a.Ho * a.Wo;
  const unsigned char* src = a.tmp ? a.tmp : a.x;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int xo = (int)(i % a.Wo);
    const long long r = i / a.Wo;
    const int yo = (int)(r % a.Ho), b = (int)(r / a.Ho);
    unsigned v[4];
    if (a.vb) {
      const int ymin = a.vb[2 * yo], ny = a.vb[2 * yo + 1];
      const int* k = a.vk + (long long)yo * a.vks;
      int acc[4] = {1 << (kResizeBits - 1), 1 << (kResizeBits - 1), 1 << (kResizeBits - 1),
                    1 << (kResizeBits - 1)};
      for (int t = 0; t < ny; ++t) {
        const unsigned char* p = src + (((long long)b * a.H + ymin + t) * a.Wo + xo) * a.C;
        const int kt = k[t];
        for (int c = 0; c < a.C; ++c) acc[c] += (int)p[c] * kt;
      }
      for (int c = 0; c < a.C; ++c) v[c] = clip8_acc(acc[c]);
    } else {  // height unchanged: the horizontal result (or the input) as it is
      const unsigned char* p = src + (((long long)b * a.H + yo) * a.Wo + xo) * a.C;
      for (int c = 0; c < a.C; ++c) v[c] = p[c];
    }
    if (a.out8) {
      unsigned char* d = a.out8 + (((long long)b * a.Ho + yo) * a.Wo + xo) * a.C;
      for (int c = 0; c < a.C; ++c) d[c] = (unsigned char)v[c];
    } else {
      for (int c = 0; c < a.C; ++c)
        a.st.out[(((long long)b * a.C + c) * a.Ho + yo) * a.Wo + xo] =
            stage_u8_val(a.st, v[c], b, c, yo, xo);
    }
  }
}

static int resize_ksize(int in, int out) {
  const double scale = (double)in / (double)out;
  const double support = scale < 1.0 ? 1.0 : scale;
  return (int)ceil(support) * 2 + 1;
}

// workspace layout: hb [2 Wo] | hk [Wo * hks] | vb [2 Ho] | vk [Ho * vks] (int32), then the
// 8-bit horizontal result [B][H][Wo][C] (16-byte aligned; when the width changes)
static long long resize_ws(int B, int H, int W, int C, int Ho, int Wo, long long* tmp_off) {
  long long ints = 0;
  if (Wo != W) ints += 2LL * Wo + (long long)Wo * resize_ksize(W, Wo);
  if (Ho != H) ints += 2LL * Ho + (long long)Ho * resize_ksize(H, Ho);
  const long long off = (ints * 4 + 15) / 16 * 16;
  if (tmp_off) *tmp_off = off;
  return off + (Wo != W ? (long long)B * H * Wo * C : 0);
}

}  // namespace mauv

MAUV_API long long mauv_resize_workspace_bytes(int B, int H, int W, int C, int Ho, int Wo) {
  if (B < 0 || H < 1 || W < 1 || C < 1 || C > 4 || Ho < 1 || Wo < 1) return -1;
  return resize_ws(B, H, W, C, Ho, Wo, nullptr);
}

MAUV_API int mauv_resize_u8(const unsigned char* x, int B, int H, int W, int C, int Ho, int Wo,
                            void* workspace, unsigned char* out_u8, const float* mean,
                            const float* stdv, const float* uifm_bt, const float* uifm_binf,
                            const float* dist, float depth, float* out_f32, hipStream_t stream) {
  if (B < 0 || H < 1 || W < 1 || C < 1 || C > 4 || Ho < 1 || Wo < 1) {
    set_error("resize_u8: bad shape (1 <= C <= 4)");
    return kErrArg;
  }
  if ((out_u8 == nullptr) == (out_f32 == nullptr)) {
    set_error("resize_u8: exactly one of out_u8 / out_f32");
    return kErrArg;
  }
  if ((mean == nullptr) != (stdv == nullptr) || (uifm_bt && !uifm_binf)) {
    set_error("resize_u8: mean/std and bt/binf come in pairs");
    return kErrArg;
  }
  if (B == 0) return 0;
  if (!x) { set_error("resize_u8: null input"); return kErrArg; }
  long long tmp_off = 0;
  resize_ws(B, H, W, C, Ho, Wo, &tmp_off);
  if ((Wo != W || Ho != H) && !workspace) { set_error("resize_u8: null workspace"); return kErrArg; }
  int* ws = (int*)workspace;
  ResizeArgs a{};
  a.x = x; a.B = B; a.H = H; a.W = W; a.C = C; a.Ho = Ho; a.Wo = Wo;
  a.out8 = out_u8;
  a.st = StageArgs{nullptr, nullptr, B, C, Ho, Wo, mean, stdv, uifm_bt, uifm_binf, dist, depth,
                   out_f32};
  int* p = ws;
  if (Wo != W) {
    a.hks = resize_ksize(W, Wo);
    a.hb = p; a.hk = p + 2 * Wo; p += 2 * Wo + (long long)Wo * a.hks;
    hipLaunchKernelGGL(resize_coeffs_kernel, dim3(ceil_div(Wo, 256)), dim3(256), 0, stream, W, Wo,
                       a.hks, (int*)a.hb, (int*)a.hk);
  }
  if (Ho != H) {
    a.vks = resize_ksize(H, Ho);
    a.vb = p; a.vk = p + 2 * Ho;
    hipLaunchKernelGGL(resize_coeffs_kernel, dim3(ceil_div(Ho, 256)), dim3(256), 0, stream, H, Ho,
                       a.vks, (int*)a.vb, (int*)a.vk);
  }
  if (Wo != W) {
    // the intermediate: the vertical pass's source; with the height unchanged the horizontal
    // pass writes straight into the 8-bit output, or into the workspace before the staging
    const bool direct = Ho == H && out_u8;
    a.tmp = direct ? out_u8 : (unsigned char*)workspace + tmp_off;
    const long long n = (long long)B * H * Wo;
    hipLaunchKernelGGL(resize_h_kernel, dim3(stage_grid(n)), dim3(256), 0, stream, a);
    if (direct) return check_launch("resize_u8");
  }
  const long long n = (long long)B * Ho * Wo;
  hipLaunchKernelGGL(resize_v_kernel, dim3(stage_grid(n)), dim3(256), 0, stream, a);
  return check_launch("resize_u8");
}

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
