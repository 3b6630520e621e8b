// Variational weight sampling, its backward, and the KL divergence (bayesian-torch 0.5.0
// Conv2dReparameterization / LinearReparameterization semantics).
//
//   forward  (per MC sample g):  w_g = mu + softplus(rho) * eps_g     eps_g ~ N(0,1)
//   backward:                    dmu  += sum_g dW_g
//                                drho += sum_g dW_g * eps_g * sigmoid(rho)
//   KL       (per tensor):       mean(log s_p - log s + (s^2 + (mu - m_p)^2) / (2 s_p^2) - 1/2)
//
// eps_g is never stored: it is regenerated from (seed, sample, layer, element quad) with
// Philox4x32-10 in both passes, so the MC-batched launch (G samples at once) draws exactly
// the stream G sequential single-sample forwards would.  An explicit eps pointer
// ([G][numel], parameter (OIHW) order) replaces the generator for parity tests.
// Sampled weights are written in the GEMM layout [G][Cout][R][S][Cin] (KRSC) consumed by
// conv_gemm.hip; parameters / gradients stay in the reference's OIHW layout so state_dicts
// keep bayesian-torch's shapes.
#include "h16.h"

using namespace mauv;

namespace mauv {

template <class S>
__global__ __launch_bounds__(256) void reparam_sample_kernel(
    const float* __restrict__ mu, const float* __restrict__ rho, const float* __restrict__ eps,
    uint64_t seed, uint64_t sample0, uint32_t layer, int G, int Cout, int Cin, int RS, int cin_pad,
    typename S::T* __restrict__ out, long long out_gs,
    const unsigned long long* __restrict__ base = nullptr) {
  // base (nullable): a device counter added to sample0 — a captured HIP graph replays the
  // same launch with fresh MC samples by updating it (mauv_reparam_sample_ex)
  if (base) sample0 += *base;
  const long long numel = (long long)Cout * Cin * RS;
  const long long nq = (numel + 3) / 4;
  for (long long q = blockIdx.x * 256LL + threadIdx.x; q < nq; q += (long long)gridDim.x * 256) {
    float m[4], s[4];
    long long dst[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long long i = 4 * q + e;
      if (i < numel) {
        m[e] = mu[i];
        s[e] = softplus(rho[i]);
        const long long o = i / ((long long)Cin * RS);
        const long long rem = i - o * Cin * RS;
        const int c = (int)(rem / RS), rs = (int)(rem - (long long)c * RS);
        dst[e] = (o * RS + rs) * cin_pad + c;
      } else {
        m[e] = 0.f; s[e] = 0.f; dst[e] = -1;
      }
    }
    // blockIdx.y takes groups g = blockIdx.y, blockIdx.y + gridDim.y, ... (the Philox counter
    // is (sample, layer, quad): the same normals whichever block draws them)
    for (int g = blockIdx.y; g < G; g += gridDim.y) {
      floatx4 ep;
      if (eps) {
#pragma unroll
        for (int e = 0; e < 4; ++e) ep[e] = dst[e] >= 0 ? eps[(long long)g * numel + 4 * q + e] : 0.f;
      } else {
        ep = normal4(seed, sample0 + g, layer, (uint32_t)q);
      }
      typename S::T* og = out + (long long)g * out_gs;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (dst[e] >= 0) S::st(og + dst[e], m[e] + s[e] * ep[e]);
    }
  }
}

// Block form of the sampling (round 3): the kernel above computes a KRSC destination per element
// with 64-bit divisions and stores 2-4 B scattered by cin_pad across the taps (bf16 step: 189
// launches, 2.3 ms, 0.4-1.2 TB/s).  Here a block owns one output channel o and CB input channels
// — ONE contiguous OIHW interval, read once (mu, softplus(rho) kept in registers) — and per sample
// g draws the interval's Philox quads into an LDS image, then writes it in KRSC order as 4-channel
// vector stores (8 B 16-bit, 16 B fp32).  Same normals (counter = (sample, layer, OIHW quad)),
// same fp32 arithmetic: bit-identical output.  CB * RS <= 1024 (one quad or two per thread).
// Needs Cin, cin_pad, out_gs % 4 == 0 and an aligned out (host checks).
template <class S>
__global__ __launch_bounds__(256) void reparam_sample_blk(
    const float* __restrict__ mu, const float* __restrict__ rho, const float* __restrict__ eps,
    uint64_t seed, uint64_t sample0, uint32_t layer, int G, int Cout, int Cin, int RS, int cin_pad,
    typename S::T* __restrict__ out, long long out_gs, const unsigned long long* __restrict__ base,
    int CB) {
  __shared__ float sv[1024];
  if (base) sample0 += *base;
  const int o = blockIdx.x, tid = threadIdx.x;
  const int c0 = blockIdx.y * CB, cb = min(CB, Cin - c0), len = cb * RS;
  const long long numel = (long long)Cout * Cin * RS;
  const long long i0 = ((long long)o * Cin + c0) * RS;
  const long long q0 = i0 >> 2;
  const int nq = (int)(((i0 + len - 1) >> 2) - q0 + 1);   // <= 257
  float m[2][4], sg[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int qi = tid + 256 * j;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long long i = 4 * (q0 + qi) + e;
      const bool in = qi < nq && i >= i0 && i < i0 + len;
      m[j][e] = in ? mu[i] : 0.f;
      sg[j][e] = in ? softplus(rho[i]) : 0.f;
    }
  }
  for (int g = blockIdx.z; g < G; g += gridDim.z) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int qi = tid + 256 * j;
      if (qi < nq) {
        const long long q = q0 + qi;
        floatx4 ep;
        if (eps) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const long long i = 4 * q + e;
            ep[e] = (i >= i0 && i < i0 + len) ? eps[(long long)g * numel + i] : 0.f;
          }
        } else {
          ep = normal4(seed, sample0 + g, layer, (uint32_t)q);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const long long i = 4 * q + e;
          if (i >= i0 && i < i0 + len) sv[(int)(i - i0)] = m[j][e] + sg[j][e] * ep[e];
        }
      }
    }
    __syncthreads();
    typename S::T* og = out + (long long)g * out_gs + (long long)o * RS * cin_pad + c0;
    for (int k = 4 * tid; k < len; k += 1024) {   // KRSC order inside the block: rs-major
      const int rs = k / cb, c = k - rs * cb;
      const floatx4 v = {sv[c * RS + rs], sv[(c + 1) * RS + rs], sv[(c + 2) * RS + rs],
                         sv[(c + 3) * RS + rs]};
      S::st4(og + (long long)rs * cin_pad + c, v);
    }
    __syncthreads();
  }
}

// One block per (output channel o, range of CB input channels): that range's parameters are
// ONE contiguous OIHW interval [(o*Cin + c0)*RS, (o*Cin + c0 + cb)*RS) and, per tap rs, a
// contiguous KRSC run of cb channels — so the block
//   (A) streams the slab runs coalesced (KRSC order), summing split-K partials (and, in
//       reference mode, the G samples) with 4 independent accumulators, into an LDS image in
//       OIHW order, then
//   (B) walks the interval's OIHW quads (the Philox counter unit) and applies the chain rule:
//       dmu += sum,  drho += sum_g d_g * eps_g' * sigmoid(rho).
// Reference mode (fixed >= 0): one epsilon for every g, so drho += (sum_g d_g) * eps * sig —
// one pass.  Exact mode: one pass per g.
// input channels per block: 64 for 1x1 (RS = 1) and for the 3x3 layers whose Cout x Cin/64
// blocks still number >= 1024 (then each (o, tap) run of the slab is one 256-B line instead of
// four 64-B pieces), 16 otherwise (<= 16*49 parameters; a small layer keeps its block count).
// The per-element sum order does not depend on it.
inline int rb_cb(int Cout, int Cin, int RS) {
  if (RS == 1) return 64;
  if (RS * 64 <= 16 * 49 && (long long)Cout * ((Cin + 63) / 64) >= 1024) return 64;
  return 16;
}

__global__ __launch_bounds__(256) void reparam_bwd_kernel(
    const float* __restrict__ dw, int splits, long long dw_gs, long long dw_ss,
    const float* __restrict__ mu, const float* __restrict__ rho, const float* __restrict__ eps,
    uint64_t seed, uint64_t sample0, uint32_t layer, int G, int Cout, int Cin, int RS, int cin_pad,
    float* __restrict__ dmu, float* __restrict__ drho, long long fixed, int CB) {
  __shared__ float sd[16 * 49];   // [cb][RS]
  __shared__ float red[4][64];
  const int o = blockIdx.x, tid = threadIdx.x;
  const int c0 = blockIdx.y * CB, cb = min(CB, Cin - c0);
  const int len = cb * RS;
  const long long numel = (long long)Cout * Cin * RS;
  const long long i0 = ((long long)o * Cin + c0) * RS;
  const long long q0 = i0 >> 2, q1 = (i0 + len - 1) >> 2;  // quads touching the interval
  const int npass = fixed >= 0 ? 1 : G;
  const int lane = tid & 63, tg = tid >> 6;  // 64 elements x 4 term groups per round
  for (int pass = 0; pass < npass; ++pass) {
    const int g0 = fixed >= 0 ? 0 : pass, ng = fixed >= 0 ? G : 1;
    const int nt = ng * splits;  // terms per element: t -> (g = g0 + t / splits, s = t % splits)
    for (int kb = 0; kb < len; kb += 64) {
      const int k = kb + lane;  // k = rs*cb + cc (coalesced in cc)
      float d0 = 0.f, d1 = 0.f;
      if (k < len) {
        const int rs = k / cb, cc = k - rs * cb;
        const float* src = dw + ((long long)o * RS + rs) * cin_pad + c0 + cc + g0 * dw_gs;
        int t = tg;
        for (; t + 4 < nt; t += 8) {
          const int ga = t / splits, gb = (t + 4) / splits;
          d0 += src[(t - ga * splits) * dw_ss + ga * dw_gs];
          d1 += src[(t + 4 - gb * splits) * dw_ss + gb * dw_gs];
        }
        if (t < nt) {
          const int ga = t / splits;
          d0 += src[(t - ga * splits) * dw_ss + ga * dw_gs];
        }
      }
      red[tg][lane] = d0 + d1;
      __syncthreads();
      if (tg == 0 && k < len) {
        const int rs = k / cb, cc = k - rs * cb;
        sd[cc * RS + rs] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
      }
      __syncthreads();
    }
    __syncthreads();
    const long long esample = fixed >= 0 ? fixed : pass;
    for (long long q = q0 + tid; q <= q1; q += 256) {
      floatx4 ep;
      if (eps) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const long long i = 4 * q + e;
          ep[e] = (i < numel) ? eps[esample * numel + i] : 0.f;
        }
      } else {
        ep = normal4(seed, sample0 + esample, layer, (uint32_t)q);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long long i = 4 * q + e;
        if (i < i0 || i >= i0 + len) continue;
        const float d = sd[(int)(i - i0)];
        dmu[i] += d;
        drho[i] += d * ep[e] * sigmoidf_(rho[i]);
      }
    }
    __syncthreads();
  }
}

// The same reduction with 16-byte slab loads (round 3).  The kernel above moves 4 B per lane per
// load with one division per term and ran at 0.7-2.8 TB/s (bf16 step: 189 launches, 4.5 ms).
// Here a lane owns a QUAD of consecutive KRSC channels (float4 loads); the block's NT threads are
// QW quad lanes x NG term groups (QW = the quads of one pass, up to 64, so a small 1x1 layer with
// 16 quads per block still keeps every lane busy); the term offsets s*dw_ss + g*dw_gs are tabled
// once per block in LDS; each lane keeps four loads in flight.  Per element the terms are summed
// in a fixed order (group grp takes t = grp + j*NG, four interleaved accumulators, then the
// groups in order), so the result is deterministic (not bit-equal to the kernel above).
// Phase B (chain rule over OIHW quads) is the same.  Needs cin_pad, c0, both strides % 4 == 0,
// a 16-B aligned slab, G*splits <= RB4_TERMS and int32 term offsets (host checks).
constexpr int RB4_TERMS = 2048;

template <int NT>
__global__ __launch_bounds__(NT) void reparam_bwd4_kernel(
    const float* __restrict__ dw, int splits, long long dw_gs, long long dw_ss,
    const float* __restrict__ mu, const float* __restrict__ rho, const float* __restrict__ eps,
    uint64_t seed, uint64_t sample0, uint32_t layer, int G, int Cout, int Cin, int RS, int cin_pad,
    float* __restrict__ dmu, float* __restrict__ drho, long long fixed, int CB, int QW) {
  __shared__ int toff[RB4_TERMS];
  __shared__ floatx4 red[NT];
  __shared__ float sd[16 * 49];   // [cb][RS]
  const int o = blockIdx.x, tid = threadIdx.x;
  const int c0 = blockIdx.y * CB, cb = min(CB, Cin - c0);
  const int len = cb * RS;
  const int cq = cb >> 2, lenq = RS * cq;
  const int NG = NT / QW, lq = tid & (QW - 1), grp = tid / QW;
  const long long numel = (long long)Cout * Cin * RS;
  const long long i0 = ((long long)o * Cin + c0) * RS;
  const long long q0 = i0 >> 2, q1 = (i0 + len - 1) >> 2;
  const int npass = fixed >= 0 ? 1 : G;
  const int ng = fixed >= 0 ? G : 1;
  const int nt = ng * splits;
  for (int t = tid; t < nt; t += NT) {
    const int g = t / splits;
    toff[t] = (int)((t - g * splits) * dw_ss + g * dw_gs);
  }
  __syncthreads();
  for (int pass = 0; pass < npass; ++pass) {
    const int g0 = fixed >= 0 ? 0 : pass;
    for (int kb = 0; kb < lenq; kb += QW) {
      const int kq = kb + lq;
      floatx4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
      int rs = 0, c4 = 0;
      if (kq < lenq) {
        rs = kq / cq;
        c4 = kq - rs * cq;
        const float* src = dw + ((long long)o * RS + rs) * cin_pad + c0 + 4 * c4 + g0 * dw_gs;
        int t = grp;
        for (; t + 3 * NG < nt; t += 4 * NG) {
          a0 += *(const floatx4*)(src + toff[t]);
          a1 += *(const floatx4*)(src + toff[t + NG]);
          a2 += *(const floatx4*)(src + toff[t + 2 * NG]);
          a3 += *(const floatx4*)(src + toff[t + 3 * NG]);
        }
        for (; t < nt; t += NG) a0 += *(const floatx4*)(src + toff[t]);
      }
      red[tid] = (a0 + a1) + (a2 + a3);
      __syncthreads();
      if (grp == 0 && kq < lenq) {
        floatx4 r = red[lq];
        for (int j = 1; j < NG; ++j) r += red[j * QW + lq];
#pragma unroll
        for (int e = 0; e < 4; ++e) sd[(4 * c4 + e) * RS + rs] = r[e];
      }
      __syncthreads();
    }
    const long long esample = fixed >= 0 ? fixed : pass;
    for (long long q = q0 + tid; q <= q1; q += NT) {
      floatx4 ep;
      if (eps) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const long long i = 4 * q + e;
          ep[e] = (i < numel) ? eps[esample * numel + i] : 0.f;
        }
      } else {
        ep = normal4(seed, sample0 + esample, layer, (uint32_t)q);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long long i = 4 * q + e;
        if (i < i0 || i >= i0 + len) continue;
        const float d = sd[(int)(i - i0)];
        dmu[i] += d;
        drho[i] += d * ep[e] * sigmoidf_(rho[i]);
      }
    }
    __syncthreads();
  }
}

// KL: one block-row of partials per table entry (deterministic, fixed-order finalize).
constexpr int KL_BLOCKS = 32;

__global__ __launch_bounds__(256) void kl_partial_kernel(const MauvKlEntry* __restrict__ tab,
                                                         double* __restrict__ partial) {
  const MauvKlEntry t = tab[blockIdx.y];
  const float lsp = logf(t.prior_sigma), inv2 = 1.0f / (2.0f * t.prior_sigma * t.prior_sigma);
  double acc = 0.0;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < t.numel; i += (long long)KL_BLOCKS * 256) {
    const float s = softplus(t.rho[i]);
    const float d = t.mu[i] - t.prior_mu;
    acc += (double)(lsp - logf(s) + (s * s + d * d) * inv2 - 0.5f);
  }
  __shared__ double red[4];
  acc = wave_sum_d(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0)
    partial[(long long)blockIdx.y * KL_BLOCKS + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void kl_finalize_kernel(const MauvKlEntry* __restrict__ tab, int n,
                                   const double* __restrict__ partial, float scale,
                                   float* __restrict__ out) {
  // one wave: lane-strided over entries, then fixed-order wave reduction
  double acc = 0.0;
  for (int e = threadIdx.x; e < n; e += 64) {
    double s = 0.0;
    for (int b = 0; b < KL_BLOCKS; ++b) s += partial[(long long)e * KL_BLOCKS + b];
    acc += s / (double)tab[e].numel;
  }
  acc = wave_sum_d(acc);
  if (threadIdx.x == 0) out[0] = (float)(acc * scale);
}

__global__ __launch_bounds__(256) void kl_bwd_kernel(const MauvKlEntry* __restrict__ tab,
                                                     const float* __restrict__ coef_dev,
                                                     float scale) {
  const MauvKlEntry t = tab[blockIdx.y];
  const float coef = (coef_dev ? coef_dev[0] : 1.0f) * scale / (float)t.numel;
  const float inv_sp2 = 1.0f / (t.prior_sigma * t.prior_sigma);
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < t.numel; i += (long long)gridDim.x * 256) {
    const float r = t.rho[i];
    const float s = softplus(r);
    t.dmu[i] += coef * (t.mu[i] - t.prior_mu) * inv_sp2;
    t.drho[i] += coef * (-1.0f / s + s * inv_sp2) * sigmoidf_(r);
  }
}

__global__ void philox_raw_kernel(uint64_t seed, uint64_t sample, uint32_t layer, int nq,
                                  uint4* out, floatx4* nrm) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  out[q] = philox4x32_10(make_uint4(q, (uint32_t)sample, layer, (uint32_t)(sample >> 32)),
                         make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  nrm[q] = normal4(seed, sample, layer, q);
}

static int grid_for(long long nq) {
  long long b = (nq + 255) / 256;
  if (b > 65536) b = 65536;
  return (int)(b < 1 ? 1 : b);
}
// reparam_sample grid: quads along x; the MC groups split along y until ~2048 blocks (eight
// per CU) — a small layer's few quad blocks otherwise walk all G groups one after another
static dim3 sample_grid(long long nq, int G) {
  const int bx = grid_for(nq);
  long long gy = (2048 + bx - 1) / bx;
  if (gy > G) gy = G;
  return dim3(bx, (unsigned)(gy < 1 ? 1 : gy));
}

// Kernel forms (MauvRoute.reparam_kernels, default 3): bit 0 = block-form sampling, bit 1 =
// 16-byte reparam_bwd.

// The block form when its layout conditions hold, else the element kernel.
template <class S>
static void launch_sample(const float* mu, const float* rho, const float* eps,
                          unsigned long long seed, unsigned long long sample0,
                          const unsigned long long* base, unsigned int layer, int G, int Cout,
                          int Cin, int RS, int cin_pad, typename S::T* out, long long gs,
                          hipStream_t stream) {
  const int blk = g_route.reparam_kernels & 1;
  const int align = (int)sizeof(typename S::T) * 4;
  if (blk && Cin % 4 == 0 && cin_pad % 4 == 0 && gs % 4 == 0 && RS <= 256 &&
      ((uintptr_t)out % align) == 0) {
    const int CB = RS == 1 ? 1024 : (1024 / RS) / 4 * 4;
    const long long nb = (long long)Cout * ceil_div(Cin, CB);
    long long gz = (1024 + nb - 1) / nb;
    if (gz > G) gz = G;
    hipLaunchKernelGGL(reparam_sample_blk<S>, dim3(Cout, ceil_div(Cin, CB), (unsigned)gz),
                       dim3(256), 0, stream, mu, rho, eps, seed, sample0, layer, G, Cout, Cin, RS,
                       cin_pad, out, gs, base, CB);
    return;
  }
  const long long nq = ((long long)Cout * Cin * RS + 3) / 4;
  hipLaunchKernelGGL(reparam_sample_kernel<S>, sample_grid(nq, G), dim3(256), 0, stream, mu, rho,
                     eps, seed, sample0, layer, G, Cout, Cin, RS, cin_pad, out, gs, base);
}

}  // namespace mauv

// Sample G weight sets: out[g] (KRSC) = mu + softplus(rho) * eps_g.  mu/rho in OIHW
// [Cout][Cin][R*S] (linear: [out][in], R*S = 1; bias: Cout = n, Cin = RS = 1).
// out_gstride: element stride between groups (0 = numel; lets several layers share one
// concatenated weight buffer, e.g. the attention q|k|v projection).
MAUV_API int mauv_reparam_sample(const float* mu, const float* rho, const float* eps,
                                 unsigned long long seed, unsigned long long sample0,
                                 unsigned int layer, int G, int Cout, int Cin, int RS,
                                 float* out, long long out_gstride, hipStream_t stream) {
  const long long numel = (long long)Cout * Cin * RS;
  const long long nq = (numel + 3) / 4;
  (void)nq;
  launch_sample<SF32>(mu, rho, eps, seed, sample0, nullptr, layer, G, Cout, Cin, RS, Cin, out,
                      out_gstride ? out_gstride : numel, stream);
  return check_launch("reparam_sample");
}

// mauv_reparam_sample into a KRSC layout with the input channels padded to cin_pad (the fp32
// stems' 4-channel layout; pad channels are left untouched: the caller zero-fills them once).
MAUV_API int mauv_reparam_sample_padded(const float* mu, const float* rho, const float* eps,
                                        unsigned long long seed, unsigned long long sample0,
                                        unsigned int layer, int G, int Cout, int Cin, int RS,
                                        int cin_pad, float* out, long long out_gstride,
                                        hipStream_t stream) {
  if (cin_pad < Cin) { set_error("reparam_sample_padded: cin_pad < Cin"); return kErrArg; }
  const long long numel = (long long)Cout * Cin * RS;
  const long long nq = (numel + 3) / 4;
  (void)nq;
  launch_sample<SF32>(mu, rho, eps, seed, sample0, nullptr, layer, G, Cout, Cin, RS, cin_pad, out,
                      out_gstride ? out_gstride : (long long)Cout * RS * cin_pad, stream);
  return check_launch("reparam_sample_padded");
}

// 16-bit sampled weights (dtype 0 = bf16, 1 = f16) for the 16-bit convs, KRSC with the input
// channels padded to cin_pad (pad channels are left untouched: the caller zero-fills them
// once).  Sampling arithmetic is fp32; only the stored weight is rounded.
MAUV_API int mauv_reparam_sample_h16(int dtype, const float* mu, const float* rho,
                                     const float* eps, unsigned long long seed,
                                     unsigned long long sample0, unsigned int layer, int G,
                                     int Cout, int Cin, int RS, int cin_pad, void* out,
                                     long long out_gstride, hipStream_t stream) {
  if (cin_pad < Cin) { set_error("reparam_sample_h16: cin_pad < Cin"); return kErrArg; }
  const long long numel = (long long)Cout * Cin * RS;
  const long long nq = (numel + 3) / 4;
  const long long gs = out_gstride ? out_gstride : (long long)Cout * RS * cin_pad;
  (void)nq;
#define L(D) launch_sample<S16<D>>(mu, rho, eps, seed, sample0, nullptr, layer, G, Cout, Cin, RS, \
                                   cin_pad, (u16*)out, gs, stream);
  MAUV_DT_DISPATCH(dtype, "reparam_sample_h16", L)
#undef L
  return check_launch("reparam_sample_h16");
}

// All three sampling forms in one entry (dtype -1 = fp32, 0 = bf16, 1 = f16; cin_pad >= Cin,
// pad channels untouched) with the MC sample index sample0 + *sample_base + g when sample_base
// (a device counter) is given: a captured HIP graph of a forward replays with fresh samples.
MAUV_API int mauv_reparam_sample_ex(int dtype, const float* mu, const float* rho,
                                    const float* eps, unsigned long long seed,
                                    unsigned long long sample0,
                                    const unsigned long long* sample_base, unsigned int layer,
                                    int G, int Cout, int Cin, int RS, int cin_pad, void* out,
                                    long long out_gstride, hipStream_t stream) {
  if (cin_pad < Cin) { set_error("reparam_sample_ex: cin_pad < Cin"); return kErrArg; }
  const long long numel = (long long)Cout * Cin * RS;
  const long long nq = (numel + 3) / 4;
  const long long gs = out_gstride ? out_gstride : (long long)Cout * RS * cin_pad;
  if (dtype < 0) {
    launch_sample<SF32>(mu, rho, eps, seed, sample0, sample_base, layer, G, Cout, Cin, RS, cin_pad,
                        (float*)out, gs, stream);
    return check_launch("reparam_sample_ex");
  }
  (void)nq;
#define L(D) launch_sample<S16<D>>(mu, rho, eps, seed, sample0, sample_base, layer, G, Cout, Cin, \
                                   RS, cin_pad, (u16*)out, gs, stream);
  MAUV_DT_DISPATCH(dtype, "reparam_sample_ex", L)
#undef L
  return check_launch("reparam_sample_ex");
}

// dmu += sum_g sum_s dw[s][g];  drho += sum_g (sum_s dw[s][g]) * eps_g' * sigmoid(rho), where
// g' = g (exact reparameterisation gradient, fixed_sample < 0) or g' = fixed_sample - sample0
// for every g (fixed_sample >= 0: bayesian-torch 0.5.0 semantics — its forward does
// `eps = self.eps_kernel.data.normal_()`, so when several MC forwards precede one backward
// autograd's saved eps aliases the buffer and every pass's rho-gradient sees the LAST draw).
// dw element (s, g, i) at dw[s*dw_sstride + g*dw_gstride + i] (strides 0 = dense
// [splits][G][Cout*RS*dw_cin]); i in the KRSC weight layout with dw_cin (>= Cin) channels
// (the 16-bit stems' zero-padded input channels are skipped).
MAUV_API int mauv_reparam_bwd(const float* dw, int splits, long long dw_gstride,
                              long long dw_sstride, const float* mu, const float* rho,
                              const float* eps, unsigned long long seed,
                              unsigned long long sample0, unsigned int layer, int G, int Cout,
                              int Cin, int RS, int dw_cin, float* dmu, float* drho,
                              long long fixed_sample, hipStream_t stream) {
  if (dw_cin < Cin) { set_error("reparam_bwd: dw_cin < Cin"); return kErrArg; }
  const long long numel = (long long)Cout * Cin * RS;
  const long long nq = (numel + 3) / 4;
  const long long gs = dw_gstride ? dw_gstride : (long long)Cout * RS * dw_cin;
  const long long ss = dw_sstride ? dw_sstride : gs * G;
  if (RS > 49) { set_error("reparam_bwd: R*S > 49"); return kErrArg; }
  (void)nq;
  const int nt = (fixed_sample >= 0 ? G : 1) * splits;
  const int v4 = (mauv::g_route.reparam_kernels >> 1) & 1;
  if (v4 && Cin % 4 == 0 && dw_cin % 4 == 0 && gs % 4 == 0 && ss % 4 == 0 &&
      ((uintptr_t)dw & 15) == 0 && nt <= RB4_TERMS &&
      (long long)(splits - 1) * ss + (long long)(G - 1) * gs + (long long)Cout * RS * dw_cin <
          (1LL << 31)) {
    // 1x1: up to 256 channels per block (64 quads: one full pass of QW = 64 lanes); 3x3: the
    // rule above (16 or 64 channels, <= 16*49 parameters per block)
    const int cb = RS == 1 ? (Cin >= 256 ? 256 : (Cin + 3) / 4 * 4) : rb_cb(Cout, Cin, RS);
    const int lenq = RS * (cb / 4);
    int qw = 1;
    while (qw < lenq && qw < 64) qw *= 2;
    const long long xs = fixed_sample >= 0 ? (long long)(fixed_sample - (long long)sample0) : -1LL;
    if (nt >= 32)
      hipLaunchKernelGGL(reparam_bwd4_kernel<1024>, dim3(Cout, ceil_div(Cin, cb)), dim3(1024), 0,
                         stream, dw, splits, gs, ss, mu, rho, eps, seed, sample0, layer, G, Cout,
                         Cin, RS, dw_cin, dmu, drho, xs, cb, qw);
    else
      hipLaunchKernelGGL(reparam_bwd4_kernel<256>, dim3(Cout, ceil_div(Cin, cb)), dim3(256), 0,
                         stream, dw, splits, gs, ss, mu, rho, eps, seed, sample0, layer, G, Cout,
                         Cin, RS, dw_cin, dmu, drho, xs, cb, qw);
    return check_launch("reparam_bwd");
  }
  const int cb = rb_cb(Cout, Cin, RS);
  hipLaunchKernelGGL(reparam_bwd_kernel, dim3(Cout, ceil_div(Cin, cb)), dim3(256), 0, stream, dw, splits,
                     gs, ss, mu, rho, eps, seed, sample0, layer, G, Cout, Cin, RS, dw_cin, dmu, drho,
                     fixed_sample >= 0 ? (long long)(fixed_sample - (long long)sample0) : -1LL, cb);
  return check_launch("reparam_bwd");
}

MAUV_API int mauv_kl_workspace_bytes(int n_entries) { return n_entries * KL_BLOCKS * 8; }

// out[0] = scale * sum_entries mean(KL elementwise) — get_kl_loss over a table of tensors.
MAUV_API int mauv_kl_fwd(const MauvKlEntry* table, int n, double* workspace, float scale,
                         float* out, hipStream_t stream) {
  if (n <= 0 || n > 65535) { set_error("kl_fwd: bad table size"); return kErrArg; }
  hipLaunchKernelGGL(kl_partial_kernel, dim3(KL_BLOCKS, n), dim3(256), 0, stream, table, workspace);
  hipLaunchKernelGGL(kl_finalize_kernel, dim3(1), dim3(64), 0, stream, table, n, workspace, scale, out);
  return check_launch("kl_fwd");
}

// dmu/drho += (coef_dev ? *coef_dev : 1) * scale * dKL/d(mu,rho) for every table entry.
MAUV_API int mauv_kl_bwd(const MauvKlEntry* table, int n, const float* coef_dev, float scale,
                         hipStream_t stream) {
  if (n <= 0 || n > 65535) { set_error("kl_bwd: bad table size"); return kErrArg; }
  hipLaunchKernelGGL(kl_bwd_kernel, dim3(64, n), dim3(256), 0, stream, table, coef_dev, scale);
  return check_launch("kl_bwd");
}

// Debug/test: raw Philox4x32-10 words and the derived normals for quads [0, nq).
MAUV_API int mauv_philox_raw(unsigned long long seed, unsigned long long sample,
                             unsigned int layer, int nq, unsigned int* out_u32x4,
                             float* out_normal4, hipStream_t stream) {
  hipLaunchKernelGGL(philox_raw_kernel, dim3((nq + 255) / 256), dim3(256), 0, stream, seed,
                     sample, layer, nq, (uint4*)out_u32x4, (floatx4*)out_normal4);
  return check_launch("philox_raw");
}
