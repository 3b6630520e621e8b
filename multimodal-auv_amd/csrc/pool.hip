// ResNet-50 stem max-pool (3x3 / 2, pad 1) and the adaptive average pool to 1x1, NHWC,
// forward + backward (torchvision resnet50 as used at models/base_models.py:15 and
// models/model_utils.py:57).  N = G*B images (the MC groups are just more images here).
// Templated on the activation storage (fp32 or 16-bit, h16.h); arithmetic in fp32.  The
// average pool's pooled features are always fp32 (the fusion head runs in fp32).
#include "h16.h"

using namespace mauv;

namespace mauv {

// Tie-break as torch's max_pool2d: first maximum in (kh, kw) scan order; NaN wins.
// One thread per 8 channels of one output pixel (C % 8 == 0, the stem has C = 64; one 16-B
// load per tap for 16-bit storage); pixel decomposition in 32-bit when the output fits.
// Branch-free taps: the nine loads are issued together from clamped in-image addresses and the
// taps outside the image (padding) become -inf after the load, which never wins the scan —
// the same maxima and indices as skipping them.  Block order: with gridDim.x % 8 == 0 each XCD
// (blocks are dealt round-robin to the 8 XCDs) walks a contiguous eighth of every grid-stride
// sweep, so the input row shared by two neighbouring output rows is read through one L2.
template <class S, class I>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const typename S::T* __restrict__ x,
                                                          int N, int H, int W, int C, int Ho,
                                                          int Wo, typename S::T* __restrict__ y,
                                                          unsigned char* __restrict__ idx,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift,
                                                          int npg) {
  const I C8 = (I)(C / 8);
  const I total = (I)N * Ho * Wo * C8;
  const unsigned nb = gridDim.x, b = blockIdx.x;
  const unsigned bid = (nb % 8 == 0) ? (b % 8) * (nb / 8) + b / 8 : b;
  for (I i = (I)bid * 256 + threadIdx.x; i < total; i += (I)nb * 256) {
    const int c = 8 * (int)(i % C8);
    I p = i / C8;
    const int ow = (int)(p % (I)Wo); p /= (I)Wo;
    const int oh = (int)(p % (I)Ho);
    const int n = (int)(p / (I)Ho);
    floatx8 v[9];
    unsigned ok = 0;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int ih = oh * 2 - 1 + r;
      const bool vr = (unsigned)ih < (unsigned)H;
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int iw = ow * 2 - 1 + s;
        const bool vt = vr & ((unsigned)iw < (unsigned)W);
        ok |= (vt ? 1u : 0u) << (r * 3 + s);
        const int ihc = vr ? ih : 0, iwc = ((unsigned)iw < (unsigned)W) ? iw : 0;
        v[r * 3 + s] = S::ld8(x + (((long long)n * H + ihc) * W + iwc) * C + c);
      }
    }
    floatx8 sc, sh;
    if (scale) {  // pending BN + ReLU of the stem, applied on load (group g = n / npg)
      const int gc = (n / npg) * C + c;
      sc = ldf8(scale + gc);
      sh = ldf8(shift + gc);
    }
    if (scale && !idx) {
      // no argmax wanted (inference): f(y) = round(relu(y*sc + sh)) is monotone in y for one
      // channel (non-decreasing for sc >= 0, non-increasing for sc < 0), so the window maximum
      // of f is f of the window's largest (sc >= 0) or smallest (sc < 0) raw value — one
      // transform per output instead of nine.  NaN taps: f(NaN) = 0 <= every f, and
      // fmaxf / fminf skip them.  The centre tap (2oh, 2ow) is always inside the image.
      floatx8 hi = v[4], lo = v[4], out;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (t == 4 || !((ok >> t) & 1u)) continue;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          hi[e] = fmaxf(hi[e], v[t][e]);
          lo[e] = fminf(lo[e], v[t][e]);
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float u = __builtin_fmaf(sc[e] >= 0.f ? hi[e] : lo[e], sc[e], sh[e]);
        out[e] = u > 0.f ? u : 0.f;
      }
      S::st8(y + 8 * (long long)i, out);
      continue;
    }
    floatx8 best;
    int bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      floatx8 u = v[t];
      if (scale) {
        // exactly what bn_apply would have stored: relu(y*scale + shift) in fp32, rounded to
        // the storage type — so maxima and tie-breaks match the materialised path
        u = u * sc + sh;
#pragma unroll
        for (int e = 0; e < 8; ++e) u[e] = u[e] > 0.f ? u[e] : 0.f;
        alignas(16) typename S::T tmp[8];
        S::st8(tmp, u);
        u = S::ld8(tmp);
      }
      const bool vt = (ok >> t) & 1u;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float q = vt ? u[e] : -INFINITY;
        if (q > best[e] || isnan(q)) { best[e] = q; bi[e] = t; }
      }
    }
    S::st8(y + 8 * (long long)i, best);
    if (idx) {
      uint2 bb;
      bb.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
      bb.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
      *(uint2*)(idx + 8 * (long long)i) = bb;
    }
  }
}

template <class S>
static void launch_maxpool_fwd(const typename S::T* x, int N, int H, int W, int C, int Ho, int Wo,
                               typename S::T* y, unsigned char* idx, const float* scale,
                               const float* shift, int npg, hipStream_t stream);

// dx of the 3x3 / stride-2 / pad-1 max-pool as a gather: input pixel (ih, iw) collects dy of the
// (at most 2 x 2) windows whose stored argmax tap is it.  V channels per thread (8 for 16-bit
// storage: 16-byte dx stores, 8-byte argmax loads; 4 for fp32), index arithmetic in I (32-bit
// whenever the element count allows: the 64-bit divisions had held this pass to ~2 TB/s).
// The per-channel sum order over windows (oh, then ow, ascending) is the same for every V.
template <class S, int V, typename I>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const typename S::T* __restrict__ dy,
                                                          const unsigned char* __restrict__ idx,
                                                          int N, int H, int W, int C, int Ho,
                                                          int Wo, typename S::T* __restrict__ dx) {
  typedef float vf __attribute__((ext_vector_type(V)));
  const I CV = (I)(C / V);
  const I total = (I)N * (I)H * (I)W * CV;
  for (I i = (I)blockIdx.x * 256 + threadIdx.x; i < total; i += (I)gridDim.x * 256) {
    I p = i / CV;
    const int c = V * (int)(i - p * CV);
    I q = p / (I)W;
    const int iw = (int)(p - q * (I)W);
    const I n = q / (I)H;
    const int ih = (int)(q - n * (I)H);
    vf acc = (vf)(0.f);
    const int oh_lo = max(0, ih / 2), oh_hi = min(Ho - 1, (ih + 1) / 2);
    const int ow_lo = max(0, iw / 2), ow_hi = min(Wo - 1, (iw + 1) / 2);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int r = ih - (oh * 2 - 1);
      if (r < 0 || r > 2) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int s = iw - (ow * 2 - 1);
        if (s < 0 || s > 2) continue;
        const I o = ((n * (I)Ho + (I)oh) * (I)Wo + (I)ow) * (I)C + (I)c;
        const unsigned char t = (unsigned char)(r * 3 + s);
        if constexpr (V == 8) {
          const uint2 kk = *(const uint2*)(idx + o);
          const floatx8 g = S::ld8(dy + o);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const unsigned char k = (unsigned char)(((e < 4 ? kk.x : kk.y) >> (8 * (e & 3))) & 0xff);
            if (k == t) acc[e] += g[e];
          }
        } else {
          const uchar4 k = *(const uchar4*)(idx + o);
          const floatx4 g = S::ld4(dy + o);
          if (k.x == t) acc[0] += g[0];
          if (k.y == t) acc[1] += g[1];
          if (k.z == t) acc[2] += g[2];
          if (k.w == t) acc[3] += g[3];
        }
      }
    }
    if constexpr (V == 8) S::st8(dx + (I)V * i, acc);
    else S::st4(dx + (I)V * i, acc);
  }
}

template <class S>
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const typename S::T* __restrict__ x,
                                                          int N, int HW, int C,
                                                          float* __restrict__ y) {
  const long long total = (long long)N * C;
  const float inv = 1.0f / (float)HW;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long long n = i / C;
    const typename S::T* src = x + n * HW * C + c;
    float acc = 0.f;
    for (int p = 0; p < HW; ++p) acc += S::ld(src + (long long)p * C);
    y[i] = acc * inv;
  }
}

template <class S>
__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const float* __restrict__ dy, int N,
                                                          int HW, int C,
                                                          typename S::T* __restrict__ dx) {
  const long long total = (long long)N * HW * C;
  const float inv = 1.0f / (float)HW;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long long n = i / ((long long)HW * C);
    S::st(dx + i, dy[n * C + c] * inv);
  }
}

// Stem input: the caller's fp32 NCHW images -> NHWC with the channels zero-padded to Cp (8 for
// the 16-bit path, 4 for fp32), so the stem conv runs on 16-byte channel chunks.
template <class S>
__global__ __launch_bounds__(256) void pack_nchw_kernel(const float* __restrict__ x, int B, int C,
                                                        int HW, int Cp, typename S::T* __restrict__ y) {
  const long long total = (long long)B * HW * Cp;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % Cp);
    const long long p = i / Cp;
    const long long b = p / HW, hw = p - b * HW;
    S::st(y + i, c < C ? x[(b * C + c) * HW + hw] : 0.f);
  }
}

static int grid1(long long n) {
  long long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  return (int)(b < 1 ? 1 : b);
}

template <class S, int V>
static void launch_maxpool_bwd(const typename S::T* dy, const unsigned char* idx, int N, int H,
                               int W, int C, int Ho, int Wo, typename S::T* dx, hipStream_t stream) {
  const long long total = (long long)N * H * W * (C / V);
  if (total + (long long)8192 * 256 < (1LL << 31))
    hipLaunchKernelGGL((maxpool_bwd_kernel<S, V, unsigned>), dim3(grid1(total)), dim3(256), 0, stream,
                       dy, idx, N, H, W, C, Ho, Wo, dx);
  else
    hipLaunchKernelGGL((maxpool_bwd_kernel<S, V, long long>), dim3(grid1(total)), dim3(256), 0,
                       stream, dy, idx, N, H, W, C, Ho, Wo, dx);
}

template <class S>
static void launch_maxpool_fwd(const typename S::T* x, int N, int H, int W, int C, int Ho, int Wo,
                               typename S::T* y, unsigned char* idx, const float* scale,
                               const float* shift, int npg, hipStream_t stream) {
  const long long total = (long long)N * Ho * Wo * (C / 8);
  if (total + (long long)8192 * 256 < (1LL << 31))
    hipLaunchKernelGGL((maxpool_fwd_kernel<S, int>), dim3(grid1(total)), dim3(256), 0, stream, x, N,
                       H, W, C, Ho, Wo, y, idx, scale, shift, npg);
  else
    hipLaunchKernelGGL((maxpool_fwd_kernel<S, long long>), dim3(grid1(total)), dim3(256), 0, stream,
                       x, N, H, W, C, Ho, Wo, y, idx, scale, shift, npg);
}

}  // namespace mauv

MAUV_API int mauv_maxpool_fwd(const float* x, int N, int H, int W, int C, float* y,
                              unsigned char* idx, hipStream_t stream) {
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  if (C % 8) { set_error("maxpool_fwd: C % 8 != 0"); return kErrArg; }
  launch_maxpool_fwd<SF32>(x, N, H, W, C, Ho, Wo, y, idx, nullptr, nullptr, 1, stream);
  return check_launch("maxpool_fwd");
}

MAUV_API int mauv_maxpool_bn_fwd(const float* y, const float* scale, const float* shift, int G,
                                 int N, int H, int W, int C, float* out, unsigned char* idx,
                                 hipStream_t stream) {
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  if (C % 8 || G <= 0 || N % G) { set_error("maxpool_bn_fwd: C % 8 != 0 or N % G != 0"); return kErrArg; }
  launch_maxpool_fwd<SF32>(y, N, H, W, C, Ho, Wo, out, idx, scale, shift, N / G, stream);
  return check_launch("maxpool_bn_fwd");
}

MAUV_API int mauv_maxpool_bwd(const float* dy, const unsigned char* idx, int N, int H, int W,
                              int C, float* dx, hipStream_t stream) {
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  if (C % 4) { set_error("maxpool_bwd: C % 4 != 0"); return kErrArg; }
  launch_maxpool_bwd<SF32, 4>(dy, idx, N, H, W, C, Ho, Wo, dx, stream);
  return check_launch("maxpool_bwd");
}

MAUV_API int mauv_avgpool_fwd(const float* x, int N, int HW, int C, float* y, hipStream_t stream) {
  hipLaunchKernelGGL(avgpool_fwd_kernel<SF32>, dim3(grid1((long long)N * C)), dim3(256), 0,
                     stream, x, N, HW, C, y);
  return check_launch("avgpool_fwd");
}

MAUV_API int mauv_avgpool_bwd(const float* dy, int N, int HW, int C, float* dx,
                              hipStream_t stream) {
  hipLaunchKernelGGL(avgpool_bwd_kernel<SF32>, dim3(grid1((long long)N * HW * C)), dim3(256), 0,
                     stream, dy, N, HW, C, dx);
  return check_launch("avgpool_bwd");
}

// ---- 16-bit activations (dtype 0 = bf16, 1 = f16) ----

MAUV_API int mauv_maxpool_fwd_h16(int dtype, const void* x, int N, int H, int W, int C, void* y,
                                  unsigned char* idx, hipStream_t stream) {
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  if (C % 8) { set_error("maxpool_fwd_h16: C % 8 != 0"); return kErrArg; }
#define L(D) launch_maxpool_fwd<S16<D>>((const u16*)x, N, H, W, C, Ho, Wo, (u16*)y, idx, nullptr, \
                                        nullptr, 1, stream);
  MAUV_DT_DISPATCH(dtype, "maxpool_fwd_h16", L)
#undef L
  return check_launch("maxpool_fwd_h16");
}

MAUV_API int mauv_maxpool_bn_fwd_h16(int dtype, const void* y, const float* scale,
                                     const float* shift, int G, int N, int H, int W, int C,
                                     void* out, unsigned char* idx, hipStream_t stream) {
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  if (C % 8 || G <= 0 || N % G) { set_error("maxpool_bn_fwd_h16: C % 8 != 0 or N % G != 0"); return kErrArg; }
#define L(D) launch_maxpool_fwd<S16<D>>((const u16*)y, N, H, W, C, Ho, Wo, (u16*)out, idx, scale, \
                                        shift, N / G, stream);
  MAUV_DT_DISPATCH(dtype, "maxpool_bn_fwd_h16", L)
#undef L
  return check_launch("maxpool_bn_fwd_h16");
}

MAUV_API int mauv_maxpool_bwd_h16(int dtype, const void* dy, const unsigned char* idx, int N,
                                  int H, int W, int C, void* dx, hipStream_t stream) {
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  if (C % 4) { set_error("maxpool_bwd_h16: C % 4 != 0"); return kErrArg; }
#define L(D) if (C % 8 == 0) launch_maxpool_bwd<S16<D>, 8>((const u16*)dy, idx, N, H, W, C, Ho, Wo, \
                                                          (u16*)dx, stream);                     \
             else launch_maxpool_bwd<S16<D>, 4>((const u16*)dy, idx, N, H, W, C, Ho, Wo, (u16*)dx, \
                                                stream);
  MAUV_DT_DISPATCH(dtype, "maxpool_bwd_h16", L)
#undef L
  return check_launch("maxpool_bwd_h16");
}

MAUV_API int mauv_avgpool_fwd_h16(int dtype, const void* x, int N, int HW, int C, float* y,
                                  hipStream_t stream) {
#define L(D) hipLaunchKernelGGL(avgpool_fwd_kernel<S16<D>>, dim3(grid1((long long)N * C)), dim3(256), \
                                0, stream, (const u16*)x, N, HW, C, y);
  MAUV_DT_DISPATCH(dtype, "avgpool_fwd_h16", L)
#undef L
  return check_launch("avgpool_fwd_h16");
}

MAUV_API int mauv_avgpool_bwd_h16(int dtype, const float* dy, int N, int HW, int C, void* dx,
                                  hipStream_t stream) {
#define L(D) hipLaunchKernelGGL(avgpool_bwd_kernel<S16<D>>, dim3(grid1((long long)N * HW * C)), \
                                dim3(256), 0, stream, dy, N, HW, C, (u16*)dx);
  MAUV_DT_DISPATCH(dtype, "avgpool_bwd_h16", L)
#undef L
  return check_launch("avgpool_bwd_h16");
}

MAUV_API int mauv_pack_nchw_h16(int dtype, const float* x, int B, int C, int H, int W, int Cp,
                                void* y, hipStream_t stream) {
  if (Cp < C) { set_error("pack_nchw_h16: Cp < C"); return kErrArg; }
#define L(D) hipLaunchKernelGGL(pack_nchw_kernel<S16<D>>, dim3(grid1((long long)B * H * W * Cp)), \
                                dim3(256), 0, stream, x, B, C, H * W, Cp, (u16*)y);
  MAUV_DT_DISPATCH(dtype, "pack_nchw_h16", L)
#undef L
  return check_launch("pack_nchw_h16");
}

MAUV_API int mauv_pack_nchw_f32(const float* x, int B, int C, int H, int W, int Cp, float* y,
                                hipStream_t stream) {
  if (Cp < C) { set_error("pack_nchw_f32: Cp < C"); return kErrArg; }
  hipLaunchKernelGGL(pack_nchw_kernel<SF32>, dim3(grid1((long long)B * H * W * Cp)), dim3(256), 0,
                     stream, x, B, C, H * W, Cp, y);
  return check_launch("pack_nchw_f32");
}
