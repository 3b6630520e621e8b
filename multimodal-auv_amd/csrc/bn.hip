// Training-mode BatchNorm (+ residual add + ReLU), forward and backward, per MC group.
//
// The reference keeps every model in .train() for training, evaluation AND prediction
// (train/multimodal.py:60,232; inference/predictors.py:27), so every MC pass normalises with
// the batch statistics of THAT pass (torchvision BatchNorm2d, eps 1e-5, momentum 0.1).  With
// the MC loop collapsed into G groups the statistics are taken per group g over its own
// (B,H,W) rows, and the running statistics are updated G times in sample order —
// bit-for-bit the sequence of G sequential forward calls.
//
// Layout: y/out/dout [G][M][C] (NHWC rows, M = B*H*W), per-group stats [G][C].
// Statistics: per-thread Welford over a row slab, Chan merges across threads and blocks
// (double in the final merge) — no E[x^2]-E[x]^2 cancellation.
#include <cstdlib>
#include <type_traits>

#include "h16.h"

using namespace mauv;

namespace mauv {

struct RowMap {
  int tpr, rp, cpt;  // threads per row (float4 each), rows in parallel, float4 per thread
};
static inline RowMap row_map(int C) {
  RowMap r;
  const int c4 = C / 4;
  r.tpr = c4 < 256 ? c4 : 256;
  r.rp = 256 / r.tpr;
  r.cpt = c4 / r.tpr;
  return r;
}

constexpr int MAXCPT = 2;  // C <= 2048

// Stage 1: per (group, block) partial (count, mean, M2) per channel.
__global__ __launch_bounds__(256) void bn_stats_partial(const float* __restrict__ y, long long M,
                                                        int C, int rpb, RowMap rm,
                                                        float* __restrict__ pmean,
                                                        float* __restrict__ pm2,
                                                        float* __restrict__ pcnt) {
  const int g = blockIdx.y, blk = blockIdx.x, nblk = gridDim.x;
  const int tid = threadIdx.x;
  const int t_c = tid % rm.tpr, t_r = tid / rm.tpr;
  const long long r0 = (long long)blk * rpb;
  const long long r1 = min(M, r0 + rpb);
  const float* yg = y + (long long)g * M * C;
  float mean[MAXCPT][4], m2[MAXCPT][4];
#pragma unroll
  for (int j = 0; j < MAXCPT; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) { mean[j][e] = 0.f; m2[j][e] = 0.f; }
  float n = 0.f;
  for (long long r = r0 + t_r; r < r1; r += rm.rp) {
    n += 1.f;
    const float inv = 1.0f / n;
#pragma unroll
    for (int j = 0; j < MAXCPT; ++j) {
      if (j >= rm.cpt) break;
      const floatx4 v = *(const floatx4*)(yg + r * C + 4 * (t_c + j * rm.tpr));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[e] - mean[j][e];
        mean[j][e] += d * inv;
        m2[j][e] += d * (v[e] - mean[j][e]);
      }
    }
  }
  // merge the rp row-threads of every channel through LDS
  __shared__ float s_mean[2048 * 2], s_m2[2048 * 2];  // rp * C <= 4096
  __shared__ float s_n[256];
  if (t_c == 0) s_n[t_r] = n;
#pragma unroll
  for (int j = 0; j < MAXCPT; ++j) {
    if (j >= rm.cpt) break;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = 4 * (t_c + j * rm.tpr) + e;
      s_mean[t_r * C + c] = mean[j][e];
      s_m2[t_r * C + c] = m2[j][e];
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float nn = 0.f, mu = 0.f, mm = 0.f;
    for (int r = 0; r < rm.rp; ++r) {
      const float nb = s_n[r];
      if (nb == 0.f) continue;
      const float mb = s_mean[r * C + c], m2b = s_m2[r * C + c];
      const float nt = nn + nb;
      const float d = mb - mu;
      mu += d * (nb / nt);
      mm += m2b + d * d * (nn * nb / nt);
      nn = nt;
    }
    const long long o = ((long long)g * nblk + blk) * C + c;
    pmean[o] = mu;
    pm2[o] = mm;
    if (c == 0) pcnt[(long long)g * nblk + blk] = nn;
  }
}

__device__ __forceinline__ void chan_merge(double& nn, double& mu, double& mm, double nb,
                                           double mb, double m2b) {
  if (nb == 0.0) return;
  const double nt = nn + nb, d = mb - mu;
  mu += d * (nb / nt);
  mm += m2b + d * d * (nn * nb / nt);
  nn = nt;
}

// Stage 2: grid (C/64, G), 1024 threads = 64 channels x 16 lanes.  Exact two-pass merge of
// the (count, mean, M2) partials: N = sum n_b, mean = sum n_b*mean_b / N,
// M2 = sum [M2_b + n_b*(mean_b - mean)^2] (double; no divisions in the loops).
constexpr int FIN_L = 16;

// The finalized statistics of channel c of group g from partials of the STORED values: with ysh
// (the centre a 16-bit forward stored y around, ConvArgs::ysh) they are those of y - ysh, which
// every consumer (BN on load, the BN backward's xhat) reads — mean / shift describe them as they
// are; the running statistics take the true mean mu + ysh (ws[G*C + ...], bn_running_kernel).
__device__ __forceinline__ void stats_out(int G, int g, int c, int C, double nn, double mu,
                                          double mm,
                                          const float* gamma, const float* beta, float eps,
                                          const float* ysh, float* mean_out, float* invstd_out,
                                          float* scale_out, float* shift_out, float* ws) {
  const double var = mm / nn;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float sc = gamma[c] * invstd;
  mean_out[g * C + c] = (float)mu;
  invstd_out[g * C + c] = invstd;
  scale_out[g * C + c] = sc;
  shift_out[g * C + c] = beta[c] - (float)mu * sc;
  ws[g * C + c] = (float)(nn > 1.0 ? mm / (nn - 1.0) : var);            // unbiased variance
  ws[(long long)G * C + g * C + c] = (float)(ysh ? mu + (double)ysh[c] : mu);  // true mean
}

__device__ __forceinline__ double lane_sum16(double v, double (*red)[64], int tx, int ty) {
  red[ty][tx] = v;
  __syncthreads();
  double s = 0.0;
  for (int k = 0; k < FIN_L; ++k) s += red[k][tx];
  __syncthreads();
  return s;
}

__global__ __launch_bounds__(1024) void bn_stats_final(
    int G, int nblk, int C, const float* __restrict__ pmean, const float* __restrict__ pm2,
    const float* __restrict__ pcnt, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, const float* __restrict__ ysh,
    float* __restrict__ mean_out, float* __restrict__ invstd_out, float* __restrict__ scale_out,
    float* __restrict__ shift_out, float* __restrict__ uvar_out) {
  const int g = blockIdx.y, tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  __shared__ double red[FIN_L][64];
  double n = 0.0, s = 0.0;
  if (c < C) {
    for (int b = ty; b < nblk; b += FIN_L) {
      const double nb = pcnt[(long long)g * nblk + b];
      n += nb;
      s += nb * (double)pmean[((long long)g * nblk + b) * C + c];
    }
  }
  const double nn = lane_sum16(n, red, tx, ty);
  const double mu = lane_sum16(s, red, tx, ty) / nn;
  double q = 0.0;
  if (c < C) {
    for (int b = ty; b < nblk; b += FIN_L) {
      const long long o = ((long long)g * nblk + b) * C + c;
      const double d = (double)pmean[o] - mu;
      q += (double)pm2[o] + pcnt[(long long)g * nblk + b] * d * d;
    }
  }
  const double mm = lane_sum16(q, red, tx, ty);
  if (ty != 0 || c >= C) return;
  stats_out(G, g, c, C, nn, mu, mm, gamma, beta, eps, ysh, mean_out, invstd_out, scale_out,
            shift_out, uvar_out);
}

// Large partial counts (an MC-batched inference chunk: tens of thousands of 128-row partials per
// channel) are merged in two launches: stage 2a reduces segments of SEG partials per channel
// exactly as above (two passes, double) into (count, mean, M2), stage 2b Chan-merges the
// segments in order.  One segment keeps the single-launch path above.  Segment length: 128
// partials up to 64 segments (a training step's layers: 4x more finalize blocks and 4x shorter
// chains than 512 — bn_stats_final + seg + merge 3.14 -> 2.09 ms per bf16 step,
// profiles/round3/bn_finalize_geometry_ab.txt), 512 beyond (an inference chunk's hundreds of
// thousands of partials: the in-order merge walks one segment list per channel).
static inline int stat_seg_len(int nblk) { return nblk <= 128 * 64 ? 128 : 512; }
static inline int stat_segs(int nblk) {
  const int L = stat_seg_len(nblk);
  return (nblk + L - 1) / L;
}

__global__ __launch_bounds__(1024) void bn_stats_seg(int nblk, int C, int SEG,
                                                     const float* __restrict__ pmean,
                                                     const float* __restrict__ pm2,
                                                     const float* __restrict__ pcnt,
                                                     double* __restrict__ seg) {
  const int g = blockIdx.y, sg = blockIdx.z, S = gridDim.z;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  const int b0 = sg * SEG, b1 = min(nblk, b0 + SEG);
  __shared__ double red[FIN_L][64];
  double n = 0.0, s = 0.0;
  if (c < C) {
    for (int b = b0 + ty; b < b1; b += FIN_L) {
      const double nb = pcnt[(long long)g * nblk + b];
      n += nb;
      s += nb * (double)pmean[((long long)g * nblk + b) * C + c];
    }
  }
  const double nn = lane_sum16(n, red, tx, ty);
  const double mu = nn > 0.0 ? lane_sum16(s, red, tx, ty) / nn : lane_sum16(s, red, tx, ty);
  double q = 0.0;
  if (c < C) {
    for (int b = b0 + ty; b < b1; b += FIN_L) {
      const long long o = ((long long)g * nblk + b) * C + c;
      const double d = (double)pmean[o] - mu;
      q += (double)pm2[o] + pcnt[(long long)g * nblk + b] * d * d;
    }
  }
  const double mm = lane_sum16(q, red, tx, ty);
  if (ty != 0 || c >= C) return;
  double* o = seg + (((long long)g * S + sg) * C + c) * 3;
  o[0] = nn;
  o[1] = mu;
  o[2] = mm;
}

__global__ __launch_bounds__(256) void bn_stats_merge(int G, int S, int C,
                                                      const double* __restrict__ seg,
                                                      const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, float eps,
                                                      const float* __restrict__ ysh,
                                                      float* __restrict__ mean_out,
                                                      float* __restrict__ invstd_out,
                                                      float* __restrict__ scale_out,
                                                      float* __restrict__ shift_out,
                                                      float* __restrict__ uvar_out) {
  const int g = blockIdx.y, c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  double nn = 0.0, mu = 0.0, mm = 0.0;
  for (int s = 0; s < S; ++s) {
    const double* o = seg + (((long long)g * S + s) * C + c) * 3;
    chan_merge(nn, mu, mm, o[0], o[1], o[2]);
  }
  stats_out(G, g, c, C, nn, mu, mm, gamma, beta, eps, ysh, mean_out, invstd_out, scale_out,
            shift_out, uvar_out);
}

// stage 2 dispatch: ws holds uvar [G][C] and the true means [G][C] (stats_out), then
// (segmented path) the segment triples
static void stats_final(int G, int nblk, int C, const float* pmean, const float* pm2,
                        const float* pcnt, const float* gamma, const float* beta, float eps,
                        const float* ysh, float* mean, float* invstd, float* scale, float* shift,
                        float* ws, hipStream_t stream) {
  const int S = stat_segs(nblk);
  if (S == 1) {
    hipLaunchKernelGGL(bn_stats_final, dim3((C + 63) / 64, G), dim3(1024), 0, stream, G, nblk, C,
                       pmean, pm2, pcnt, gamma, beta, eps, ysh, mean, invstd, scale, shift, ws);
    return;
  }
  double* seg = (double*)(((uintptr_t)(ws + 2LL * G * C) + 7) & ~(uintptr_t)7);
  hipLaunchKernelGGL(bn_stats_seg, dim3((C + 63) / 64, G, S), dim3(1024), 0, stream, nblk, C,
                     stat_seg_len(nblk), pmean, pm2, pcnt, seg);
  hipLaunchKernelGGL(bn_stats_merge, dim3((C + 255) / 256, G), dim3(256), 0, stream, G, S, C, seg,
                     gamma, beta, eps, ysh, mean, invstd, scale, shift, ws);
}
static long long stats_ws_floats(int G, int nblk, int C) {
  const int S = stat_segs(nblk);
  return 2LL * G * C + (S > 1 ? 6LL * G * S * C + 2 : 0);
}

// Stage 3: the G running-stat updates, in MC-sample order (= G sequential forward calls), from
// stage 2's workspace: uvar [G][C], then the true means [G][C].
__global__ void bn_running_kernel(int G, int C, const float* __restrict__ ws,
                                  float* __restrict__ run_mean, float* __restrict__ run_var,
                                  float momentum) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float* uvar = ws;
  const float* mean = ws + (long long)G * C;
  float rm = run_mean[c], rv = run_var[c];
  for (int g = 0; g < G; ++g) {
    rm = (1.f - momentum) * rm + momentum * mean[g * C + c];
    rv = (1.f - momentum) * rv + momentum * uvar[g * C + c];
  }
  run_mean[c] = rm;
  run_var[c] = rv;
}

// out = [relu]( y * scale[g][c] + shift[g][c] (+ res') ),  res' = res, or — when the residual
// is itself a pending BatchNorm (the bottleneck's downsample branch, never materialised) —
// res' = res * res_scale[g][c] + res_shift[g][c]
template <class S>
__global__ __launch_bounds__(256) void bn_apply_kernel(const typename S::T* __restrict__ y,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift,
                                                       const typename S::T* __restrict__ res,
                                                       const float* __restrict__ res_scale,
                                                       const float* __restrict__ res_shift,
                                                       int relu, typename S::T* __restrict__ out,
                                                       long long M, int C) {
  const int c8n = C / 8;  // 8 channels per thread-iteration: 16-B (16-bit) / 2x16-B (fp32)
  const long long per_g = M * c8n;
  const int g = blockIdx.y;
  const typename S::T* yg = y + (long long)g * M * C;
  typename S::T* og = out + (long long)g * M * C;
  const typename S::T* rg = res ? res + (long long)g * M * C : nullptr;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < per_g; i += (long long)gridDim.x * 256) {
    const int c = 8 * (int)(i % c8n);
    floatx8 v = S::ld8(yg + 8 * i);
    v = v * ldf8(scale + g * C + c) + ldf8(shift + g * C + c);
    if (rg) {
      floatx8 rv = S::ld8(rg + 8 * i);
      if (res_scale) rv = rv * ldf8(res_scale + g * C + c) + ldf8(res_shift + g * C + c);
      v += rv;
    }
    if (relu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
    }
    S::st8(og + 8 * i, v);
  }
}

// ReLU mask of the BN output: from the stored output when there is one (residual blocks),
// else recomputed from y (lazily-applied BN: out = relu(y*scale + shift) was never stored).
template <class S>
__device__ __forceinline__ floatx4 relu_mask(floatx4 dz, const typename S::T* out, long long o,
                                             floatx4 yv, const float* scale,
                                             const float* shift, int gc) {
  floatx4 pre;
  if (out) pre = S::ld4(out + o);
  else pre = yv * *(const floatx4*)(scale + gc) + *(const floatx4*)(shift + gc);
#pragma unroll
  for (int e = 0; e < 4; ++e) dz[e] = pre[e] > 0.f ? dz[e] : 0.f;
  return dz;
}

// Backward stage 1: per (g, block) partial sums of dz and dz*xhat per channel,
// dz = dout * (relu ? out > 0 : 1), xhat = (y - mean) * invstd.
template <class S>
__global__ __launch_bounds__(256) void bn_bwd_partial(const typename S::T* __restrict__ y,
                                                      const typename S::T* __restrict__ out,
                                                      const typename S::T* __restrict__ dout,
                                                      int relu,
                                                      const float* __restrict__ mean,
                                                      const float* __restrict__ invstd,
                                                      const float* __restrict__ scale,
                                                      const float* __restrict__ shift,
                                                      long long M, int C, int rpb, RowMap rm,
                                                      float* __restrict__ p1,
                                                      float* __restrict__ p2,
                                                      const unsigned char* __restrict__ mask) {
  // one 8-channel group per thread (C % 8 == 0, C <= 2048): tpr threads span a row, rp rows
  // are walked in parallel
  const int tpr = C / 8, rp = 256 / tpr;
  const int g = blockIdx.y, blk = blockIdx.x, nblk = gridDim.x;
  const int tid = threadIdx.x;
  const int t_c = tid % tpr, t_r = tid / tpr;
  const long long r0 = (long long)blk * rpb;
  const long long r1 = min(M, r0 + rpb);
  const long long go = (long long)g * M * C;
  const int c0 = 8 * t_c, gc = g * C + c0;
  floatx8 s1 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, s2 = s1;
  if (t_r < rp) {
    const floatx8 mu = ldf8(mean + gc), is = ldf8(invstd + gc);
    floatx8 sc = s1, sh = s1;
    if (relu && !out && !mask) { sc = ldf8(scale + gc); sh = ldf8(shift + gc); }
    // RU rows per thread per step: every row's loads issued before the first is consumed (one
    // row at a time, with the ReLU-source branches inside the loop, left two 16-byte loads in
    // flight per lane: latency-bound); rows past r1 add zeros, so the sums keep their row order.
    // The ReLU source is chosen once, outside the row loop.
    constexpr int RU = 4;
    const floatx8 z8 = s1;
    auto rows = [&](auto src) {
      constexpr int SRC = decltype(src)::value;  // 0 none, 1 mask bits, 2 out, 3 y*scale+shift
      for (long long r = r0 + t_r; r < r1; r += RU * rp) {
        typename S::R8 yr[RU], dr[RU], pr[RU];
        unsigned m[RU];
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          // rows past r1 re-read row r (unconditional loads, no branch to wait inside)
          const long long rr = r + (long long)u * rp;
          const long long o = go + (rr < r1 ? rr : r) * C + c0;
          yr[u] = S::raw8(y + o);
          dr[u] = S::raw8(dout + o);
          if constexpr (SRC == 1) m[u] = mask[o >> 3];
          if constexpr (SRC == 2) pr[u] = S::raw8(out + o);
        }
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const floatx8 yv = S::cvt8(yr[u]);
          floatx8 dz = r + (long long)u * rp < r1 ? S::cvt8(dr[u]) : z8;
          if constexpr (SRC == 1) {
#pragma unroll
            for (int e = 0; e < 8; ++e) dz[e] = (m[u] >> e) & 1u ? dz[e] : 0.f;
          } else if constexpr (SRC >= 2) {
            const floatx8 p = SRC == 2 ? S::cvt8(pr[u]) : yv * sc + sh;
#pragma unroll
            for (int e = 0; e < 8; ++e) dz[e] = p[e] > 0.f ? dz[e] : 0.f;
          }
          s1 += dz;
          s2 += dz * (yv - mu) * is;
        }
      }
    };
    if (mask) rows(std::integral_constant<int, 1>());
    else if (!relu) rows(std::integral_constant<int, 0>());
    else if (out) rows(std::integral_constant<int, 2>());
    else rows(std::integral_constant<int, 3>());
  }
  __shared__ float sh1[2048], sh2[2048];  // [rp][C], rp * C = 8 * 256
  if (t_r < rp) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sh1[t_r * C + c0 + e] = s1[e];
      sh2[t_r * C + c0 + e] = s2[e];
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < rp; ++r) { a += sh1[r * C + c]; b += sh2[r * C + c]; }
    const long long o = ((long long)g * nblk + blk) * C + c;
    p1[o] = a;
    p2[o] = b;
  }
}

// Backward stage 2: grid (C/64, G), 64 channels x 4 lanes: k1 = sum dz / M, k2 = sum
// dz*xhat / M per (g,c) (double sums, fixed order).
__global__ __launch_bounds__(1024) void bn_bwd_final(int G, int nblk, int C, long long M,
                                                     const float* __restrict__ p1,
                                                     const float* __restrict__ p2,
                                                     float* __restrict__ k1,
                                                     float* __restrict__ k2) {
  const int g = blockIdx.y, tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  __shared__ double red[FIN_L][64];
  double a = 0.0, b = 0.0;
  if (c < C) {
    for (int k = ty; k < nblk; k += FIN_L) {
      const long long o = ((long long)g * nblk + k) * C + c;
      a += p1[o];
      b += p2[o];
    }
  }
  a = lane_sum16(a, red, tx, ty);
  b = lane_sum16(b, red, tx, ty);
  if (ty != 0 || c >= C) return;
  k1[g * C + c] = (float)(a / (double)M);
  k2[g * C + c] = (float)(b / (double)M);
}

// Many partials per channel (the data-gradient epilogue's one per 128-row tile: thousands at the
// layer-1 shapes) are reduced in segments of SEGB by (C/64, G, S) blocks into double pairs, then
// one thread per channel sums the segments in order, forms k1 / k2 for every group and the
// parameter gradients (stage 3 below, fused) — the single-block-per-(group, 64 channels) stage
// 2 above walks every partial of a layer with G * C / 64 blocks.
// (Only above 1024 partials — the epilogue's — : for the standalone pass's <= 1024 the extra
// launch ate the gain, bf16 step 3.55 vs 3.55 ms of finalize kernels, tools/gpubatch_r3i.sh.)
constexpr int SEGB = 128, kSegAbove = 1024;
static inline int bwd_segs(int nblk) { return (nblk + SEGB - 1) / SEGB; }

__global__ __launch_bounds__(1024) void bn_bwd_seg(int nblk, int C, const float* __restrict__ p1,
                                                   const float* __restrict__ p2,
                                                   double* __restrict__ seg) {
  const int g = blockIdx.y, sg = blockIdx.z, S = gridDim.z;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  const int b0 = sg * SEGB, b1 = min(nblk, b0 + SEGB);
  __shared__ double red[FIN_L][64];
  double a = 0.0, b = 0.0;
  if (c < C) {
    for (int k = b0 + ty; k < b1; k += FIN_L) {
      const long long o = ((long long)g * nblk + k) * C + c;
      a += p1[o];
      b += p2[o];
    }
  }
  a = lane_sum16(a, red, tx, ty);
  b = lane_sum16(b, red, tx, ty);
  if (ty != 0 || c >= C) return;
  double* o = seg + (((long long)g * S + sg) * C + c) * 2;
  o[0] = a;
  o[1] = b;
}

__global__ void bn_bwd_merge(int G, int S, int C, long long M, const double* __restrict__ seg,
                             float* __restrict__ k1, float* __restrict__ k2,
                             float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double tg = 0.0, tb = 0.0;
  for (int g = 0; g < G; ++g) {
    double a = 0.0, b = 0.0;
    for (int s = 0; s < S; ++s) {
      const double* o = seg + (((long long)g * S + s) * C + c) * 2;
      a += o[0];
      b += o[1];
    }
    const float f1 = (float)(a / (double)M), f2 = (float)(b / (double)M);
    k1[g * C + c] = f1;
    k2[g * C + c] = f2;
    tb += f1;
    tg += f2;
  }
  if (dgamma) dgamma[c] += (float)(tg * (double)M);
  if (dbeta) dbeta[c] += (float)(tb * (double)M);
}

// Backward stage 3: dgamma += M * sum_g k2, dbeta += M * sum_g k1 (sample order).
__global__ void bn_bwd_param_kernel(int G, int C, long long M, const float* __restrict__ k1,
                                    const float* __restrict__ k2, float* __restrict__ dgamma,
                                    float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double tg = 0.0, tb = 0.0;
  for (int g = 0; g < G; ++g) { tb += k1[g * C + c]; tg += k2[g * C + c]; }
  if (dgamma) dgamma[c] += (float)(tg * (double)M);
  if (dbeta) dbeta[c] += (float)(tb * (double)M);
}

// dy = gamma*invstd * (dz - k1 - xhat*k2); dres = dz (optional).  8 channels per iteration.
template <class S>
__global__ __launch_bounds__(256) void bn_bwd_apply(const typename S::T* __restrict__ y,
                                                    const typename S::T* __restrict__ out,
                                                    const typename S::T* __restrict__ dout,
                                                    int relu,
                                                    const float* __restrict__ mean,
                                                    const float* __restrict__ invstd,
                                                    const float* __restrict__ scale,
                                                    const float* __restrict__ shift,
                                                    const float* __restrict__ k1,
                                                    const float* __restrict__ k2,
                                                    typename S::T* __restrict__ dy,
                                                    typename S::T* __restrict__ dres, long long M,
                                                    int C) {
  const int c8n = C / 8;
  const long long per_g = M * c8n;
  const int g = blockIdx.y;
  const long long go = (long long)g * M * C;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < per_g; i += (long long)gridDim.x * 256) {
    const int c = 8 * (int)(i % c8n);
    const long long o = go + 8 * i;
    floatx8 dz = S::ld8(dout + o);
    const floatx8 yv = S::ld8(y + o);
    const int gc = g * C + c;
    if (relu) {
      const floatx8 pre = out ? S::ld8(out + o) : yv * ldf8(scale + gc) + ldf8(shift + gc);
#pragma unroll
      for (int e = 0; e < 8; ++e) dz[e] = pre[e] > 0.f ? dz[e] : 0.f;
    }
    const floatx8 xh = (yv - ldf8(mean + gc)) * ldf8(invstd + gc);
    S::st8(dy + o, ldf8(scale + gc) * (dz - ldf8(k1 + gc) - xh * ldf8(k2 + gc)));
    if (dres) S::st8(dres + o, dz);
  }
}

// bn_bwd_partial geometry: C/8 threads span a row, so a 256-thread block walks 256/(C/8)
// rows at once; at most 32 rows per thread keeps G*nblk in the hundreds for the deep,
// narrow-M layers (layer4: M = B*49 rows of 2048 channels) that one-block-per-256-rows left at
// ~13 blocks per group, at the cost of <= 1/32 extra partial traffic per element (32 vs 16 vs
// 8 rows per thread with the ReLU masks: 234.5-235.5 vs 231.8-232.5 vs 230.9-232.0 fp32
// triplets/s, 574-575 vs 562-565 vs 554 bf16 on one box, tools/gpubatch_rpt2.sh).
static int ew_grid(long long n4);

// Row-walk forms of the two elementwise passes (the default): C/8 threads span a row, 256/(C/8)
// rows are walked in parallel and each block takes rpb consecutive rows, so a thread keeps its
// 8 channels' per-group parameters in registers for the whole slab and its offsets need no
// 64-bit modulo — the grid-stride forms above reload scale/shift (L1 hits, but issue slots) and
// divide per element group, which is what held the 16-bit passes (48 B of HBM traffic per
// iteration) well below the fp32 ones' bandwidth.  C <= 2048.
template <class S>
__global__ __launch_bounds__(256) void bn_apply_rows(const typename S::T* __restrict__ y,
                                                     const float* __restrict__ scale,
                                                     const float* __restrict__ shift,
                                                     const typename S::T* __restrict__ res,
                                                     const float* __restrict__ res_scale,
                                                     const float* __restrict__ res_shift,
                                                     int relu, typename S::T* __restrict__ out,
                                                     long long M, int C, int rpb,
                                                     unsigned char* __restrict__ mask) {
  const int tpr = C / 8, rp = 256 / tpr;
  const int tid = threadIdx.x, t_c = tid % tpr, t_r = tid / tpr;
  if (t_r >= rp) return;
  const int g = blockIdx.y;
  const long long r0 = (long long)blockIdx.x * rpb;
  const long long r1 = min(M, r0 + rpb);
  const int c0 = 8 * t_c, gc = g * C + c0;
  const floatx8 sc = ldf8(scale + gc), sh = ldf8(shift + gc);
  floatx8 rsc, rsh;
  if (res_scale) { rsc = ldf8(res_scale + gc); rsh = ldf8(res_shift + gc); }
  const long long base = (long long)g * M * C + c0;
  // RU rows per step, every row's loads (y, the residual) issued before the first is used, the
  // residual's form chosen outside the loop (bn_bwd_apply_rows' reasoning)
  constexpr int RU = 2;
  auto rows = [&](auto rk) {
    constexpr int RES = decltype(rk)::value;  // 0 none, 1 res, 2 res * res_scale + res_shift
    for (long long r = r0 + t_r; r < r1; r += RU * rp) {
      typename S::R8 yr[RU], rr_[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const long long rr = r + (long long)u * rp;
        const long long o = base + (rr < r1 ? rr : r) * C;   // past r1: row r again, not stored
        yr[u] = S::raw8(y + o);
        if constexpr (RES != 0) rr_[u] = S::raw8(res + o);
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const long long rr = r + (long long)u * rp;
        floatx8 v = S::cvt8(yr[u]) * sc + sh;
        if constexpr (RES != 0) {
          floatx8 rv = S::cvt8(rr_[u]);
          if constexpr (RES == 2) rv = rv * rsc + rsh;
          v += rv;
        }
        if (relu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
        }
        if (rr >= r1) continue;
        const long long o = base + rr * C;
        S::st8(out + o, v);
        if (mask) {  // bit e = (stored out > 0): the value as rounded to the storage type
          alignas(16) typename S::T tmp[8];
          S::st8(tmp, v);
          const floatx8 q = S::ld8(tmp);
          unsigned m = 0;
#pragma unroll
          for (int e = 0; e < 8; ++e) m |= (q[e] > 0.f ? 1u : 0u) << e;
          mask[o >> 3] = (unsigned char)m;
        }
      }
    }
  };
  if (!res) rows(std::integral_constant<int, 0>());
  else if (!res_scale) rows(std::integral_constant<int, 1>());
  else rows(std::integral_constant<int, 2>());
}

template <class S>
__global__ __launch_bounds__(256) void bn_bwd_apply_rows(const typename S::T* __restrict__ y,
                                                         const typename S::T* __restrict__ out,
                                                         const typename S::T* __restrict__ dout,
                                                         int relu,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ invstd,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift,
                                                         const float* __restrict__ k1,
                                                         const float* __restrict__ k2,
                                                         typename S::T* __restrict__ dy,
                                                         typename S::T* __restrict__ dres,
                                                         long long M, int C, int rpb,
                                                         const unsigned char* __restrict__ mask) {
  const int tpr = C / 8, rp = 256 / tpr;
  const int tid = threadIdx.x, t_c = tid % tpr, t_r = tid / tpr;
  if (t_r >= rp) return;
  const int g = blockIdx.y;
  const long long r0 = (long long)blockIdx.x * rpb;
  const long long r1 = min(M, r0 + rpb);
  const int c0 = 8 * t_c, gc = g * C + c0;
  const floatx8 sc = ldf8(scale + gc), mu = ldf8(mean + gc), is = ldf8(invstd + gc);
  const floatx8 a1 = ldf8(k1 + gc), a2 = ldf8(k2 + gc);
  floatx8 sh = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (relu && !out && !mask) sh = ldf8(shift + gc);
  const long long base = (long long)g * M * C + c0;
  // RU rows per step with every load (dz, y, the mask byte / out) issued before the first use
  // and the ReLU source chosen outside the loop: in one loop body with the branches inside,
  // each row waited for dz and y, then for its mask byte, then stored — three latencies a row
  constexpr int RU = 2;
  auto rows = [&](auto src) {
    constexpr int SRC = decltype(src)::value;  // 0 none, 1 mask bits, 2 out, 3 y*scale+shift
    for (long long r = r0 + t_r; r < r1; r += RU * rp) {
      typename S::R8 yr[RU], dr[RU], pr[RU];
      unsigned m[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const long long rr = r + (long long)u * rp;
        const long long o = base + (rr < r1 ? rr : r) * C;   // past r1: row r again, not stored
        dr[u] = S::raw8(dout + o);
        yr[u] = S::raw8(y + o);
        if constexpr (SRC == 1) m[u] = mask[o >> 3];
        if constexpr (SRC == 2) pr[u] = S::raw8(out + o);
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const long long rr = r + (long long)u * rp;
        const floatx8 yv = S::cvt8(yr[u]);
        floatx8 dz = S::cvt8(dr[u]);
        if constexpr (SRC == 1) {
#pragma unroll
          for (int e = 0; e < 8; ++e) dz[e] = (m[u] >> e) & 1u ? dz[e] : 0.f;
        } else if constexpr (SRC >= 2) {
          const floatx8 p = SRC == 2 ? S::cvt8(pr[u]) : yv * sc + sh;
#pragma unroll
          for (int e = 0; e < 8; ++e) dz[e] = p[e] > 0.f ? dz[e] : 0.f;
        }
        if (rr < r1) {
          const long long o = base + rr * C;
          const floatx8 xh = (yv - mu) * is;
          S::st8(dy + o, sc * (dz - a1 - xh * a2));
          if (dres) S::st8(dres + o, dz);
        }
      }
    }
  };
  if (mask) rows(std::integral_constant<int, 1>());
  else if (!relu) rows(std::integral_constant<int, 0>());
  else if (out) rows(std::integral_constant<int, 2>());
  else rows(std::integral_constant<int, 3>());
}

// Row-walk geometry: <= 2 rows per thread (measured 2 vs 4 vs 8 vs 16: inference 10.40-10.43k vs 10.32-10.35k vs 10.16-10.19k vs 10.12k
// MC-samples/s on one box; training flat).
static void rows_geometry(long long M, int C, int& nblk, int& rpb) {
  constexpr int rpt = 2;
  const int rp = 256 / (C / 8);
  const long long r = (long long)rp * rpt;
  rpb = (int)r;
  nblk = (int)((M + r - 1) / r);
}

static bool use_rows(int C) { return C % 8 == 0 && C <= 2048; }

template <class S>
static void launch_apply(const typename S::T* y, const float* scale, const float* shift,
                         const typename S::T* res, const float* res_scale, const float* res_shift,
                         int relu, typename S::T* out, int G, long long M, int C,
                         hipStream_t stream, unsigned char* mask = nullptr) {
  if (mask || use_rows(C)) {
    int nblk, rpb;
    rows_geometry(M, C, nblk, rpb);
    hipLaunchKernelGGL(bn_apply_rows<S>, dim3(nblk, G), dim3(256), 0, stream, y, scale, shift,
                       res, res_scale, res_shift, relu, out, M, C, rpb, mask);
  } else {
    hipLaunchKernelGGL(bn_apply_kernel<S>, dim3(ew_grid(M * C / 8), G), dim3(256), 0, stream, y,
                       scale, shift, res, res_scale, res_shift, relu, out, M, C);
  }
}

static void bwd_geometry(long long M, int C, int& nblk, int& rpb) {
  constexpr int rpt = 32;  // rows per thread of the backward partial pass
  const int rp = 256 / (C / 8);
  long long r = (long long)rp * rpt;
  long long n = (M + r - 1) / r;
  // at most 256 partial blocks per group (was 1024: bn_bwd_final walks 4x fewer partials,
  // 1.53 -> 1.01 ms per bf16 step, and the partial pass itself 11.35 -> 11.23 ms)
  if (n > 256) { n = 256; r = (M + n - 1) / n; }
  if (r < rp) r = rp;
  rpb = (int)r;
  nblk = (int)((M + r - 1) / r);
}

static void reduce_geometry(long long M, int C, int& nblk, int& rpb) {
  const RowMap rm = row_map(C);
  long long target = (M + 255) / 256;  // ~256 rows per block
  if (target > 1024) target = 1024;
  if (target < 1) target = 1;
  rpb = (int)((M + target - 1) / target);
  if (rpb < rm.rp) rpb = rm.rp;
  nblk = (int)((M + rpb - 1) / rpb);
}

static int ew_grid(long long n4) {
  long long b = (n4 + 255) / 256;
  if (b > 4096) b = 4096;
  return (int)(b < 1 ? 1 : b);
}

// eval-mode BN (running statistics): per-group copies of scale/shift
__global__ void bn_eval_params_kernel(int G, int C, const float* __restrict__ gamma,
                                      const float* __restrict__ beta,
                                      const float* __restrict__ rm, const float* __restrict__ rv,
                                      float eps, float* __restrict__ scale,
                                      float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float sc = gamma[c] / sqrtf(rv[c] + eps);
  const float sh = beta[c] - rm[c] * sc;
  for (int g = 0; g < G; ++g) { scale[g * C + c] = sc; shift[g * C + c] = sh; }
}

}  // namespace mauv

// Eval-mode BN parameters (module.eval()): scale = gamma/sqrt(rv+eps), shift = beta - rm*scale.
MAUV_API int mauv_bn_eval_params(int G, int C, const float* gamma, const float* beta,
                                 const float* run_mean, const float* run_var, float eps,
                                 float* scale, float* shift, hipStream_t stream) {
  hipLaunchKernelGGL(bn_eval_params_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, G, C,
                     gamma, beta, run_mean, run_var, eps, scale, shift);
  return check_launch("bn_eval_params");
}

// Workspace floats needed by mauv_bn_fwd_train / mauv_bn_bwd for (G, M, C).
MAUV_API long long mauv_bn_workspace_floats(int G, long long M, int C) {
  int nblk, rpb, bnblk, brpb;
  reduce_geometry(M, C, nblk, rpb);
  const long long fwd = (long long)G * nblk * (2LL * C + 1) + 2LL * G * C + stats_ws_floats(G, nblk, C);
  if (C <= 0 || C % 8 != 0 || C > 2048) return fwd;
  bwd_geometry(M, C, bnblk, brpb);
  // + the segment pairs of bn_bwd_seg for the most partials either source gives (the
  // standalone pass's bnblk, or a data-gradient epilogue's one per >= 64 rows), 8-B aligned
  const long long pre = (M + 63) / 64;
  const long long nseg = (((pre > bnblk ? pre : bnblk) + SEGB - 1) / SEGB);
  const long long bwd = 2LL * G * bnblk * C + 2LL * G * C + 4LL * G * nseg * C + 2;
  return fwd > bwd ? fwd : bwd;
}

// Workspace floats of mauv_bn_stats_finalize for nblk partials per channel.
MAUV_API long long mauv_bn_stats_workspace_floats(int G, int nblk, int C) {
  return stats_ws_floats(G, nblk, C);
}

// Training-mode BN forward for G groups: statistics (mean/invstd/scale/shift out, [G][C]),
// sequential running-stat updates (run_* nullable), then out = [relu](bn(y) (+ res)).
MAUV_API int mauv_bn_fwd_train(const float* y, int G, long long M, int C, const float* gamma,
                               const float* beta, float* run_mean, float* run_var,
                               float momentum, float eps, float* workspace, float* mean,
                               float* invstd, float* scale, float* shift, const float* res,
                               int relu, float* out, hipStream_t stream) {
  if (C % 8 != 0 || C > 2048 || G <= 0 || M <= 0) { set_error("bn_fwd: unsupported C/G/M"); return kErrArg; }
  int nblk, rpb;
  reduce_geometry(M, C, nblk, rpb);
  const RowMap rm = row_map(C);
  float* pmean = workspace;
  float* pm2 = pmean + (long long)G * nblk * C;
  float* pcnt = pm2 + (long long)G * nblk * C;
  hipLaunchKernelGGL(bn_stats_partial, dim3(nblk, G), dim3(256), 0, stream, y, M, C, rpb, rm,
                     pmean, pm2, pcnt);
  float* uvar = pcnt + (long long)G * nblk;
  stats_final(G, nblk, C, pmean, pm2, pcnt, gamma, beta, eps, nullptr, mean, invstd, scale, shift,
              uvar, stream);
  if (run_mean && run_var)
    hipLaunchKernelGGL(bn_running_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, G, C, uvar,
                       run_mean, run_var, momentum);
  if (out) {
    launch_apply<SF32>(y, scale, shift, res, nullptr, nullptr, relu, out, G, M, C, stream);
  }
  return check_launch("bn_fwd_train");
}

// Statistics from per-m-tile partials of the fused conv epilogue (conv_gemm.hip).
MAUV_API int mauv_bn_stats_finalize(int G, int nblk, int C, const float* pmean, const float* pm2,
                                    const float* pcnt, const float* gamma, const float* beta,
                                    float* run_mean, float* run_var, float momentum, float eps,
                                    float* workspace, float* mean, float* invstd, float* scale,
                                    float* shift, const float* y_shift, hipStream_t stream) {
  if (G <= 0 || nblk <= 0 || C <= 0) { set_error("bn_stats_finalize: bad shape"); return kErrArg; }
  stats_final(G, nblk, C, pmean, pm2, pcnt, gamma, beta, eps, y_shift, mean, invstd, scale, shift,
              workspace, stream);
  if (run_mean && run_var)
    hipLaunchKernelGGL(bn_running_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, G, C,
                       workspace, run_mean, run_var, momentum);
  return check_launch("bn_stats_finalize");
}

// out = [relu](y * scale + shift (+ res')) with precomputed per-group scale/shift;
// res' = res * res_scale + res_shift when res_scale is given (pending BN on the residual).
MAUV_API int mauv_bn_apply(const float* y, const float* scale, const float* shift,
                           const float* res, const float* res_scale, const float* res_shift,
                           int relu, float* out, int G, long long M, int C, hipStream_t stream) {
  if (C % 8 != 0) { set_error("bn_apply: C % 8 != 0"); return kErrArg; }
  launch_apply<SF32>(y, scale, shift, res, res_scale, res_shift, relu, out, G, M, C, stream);
  return check_launch("bn_apply");
}

template <class S>
static int bn_bwd_impl(const typename S::T* y, const typename S::T* out,
                       const typename S::T* dout, int relu, const float* mean,
                       const float* invstd, const float* scale, const float* shift, int G,
                       long long M, int C, float* workspace, typename S::T* dy,
                       typename S::T* dres, float* dgamma, float* dbeta, const float* pre_p1,
                       const float* pre_p2, int pre_nblk, hipStream_t stream,
                       const unsigned char* mask = nullptr) {
  if (C % 8 != 0 || C > 2048) { set_error("bn_bwd: unsupported C (C % 8 != 0 or > 2048)"); return kErrArg; }
  if (relu && !out && !shift && !mask) { set_error("bn_bwd: relu mask needs out or scale/shift"); return kErrArg; }
  int nblk, rpb;
  bwd_geometry(M, C, nblk, rpb);
  const RowMap rm = row_map(C);
  float* p1 = workspace;
  float* p2 = p1 + (long long)G * nblk * C;
  float* k1 = p2 + (long long)G * nblk * C;
  float* k2 = k1 + (long long)G * C;
  const float* q1 = p1;
  const float* q2 = p2;
  int qn = nblk;
  if (pre_p1) {  // partial sums already produced by a data-gradient epilogue
    q1 = pre_p1; q2 = pre_p2; qn = pre_nblk;
  } else {
    hipLaunchKernelGGL(bn_bwd_partial<S>, dim3(nblk, G), dim3(256), 0, stream, y, out, dout,
                       relu, mean, invstd, scale, shift, M, C, rpb, rm, p1, p2, mask);
  }
  const int nseg = qn > kSegAbove ? bwd_segs(qn) : 1;
  if (nseg > 1) {
    double* seg = (double*)(((uintptr_t)(k2 + (long long)G * C) + 7) & ~(uintptr_t)7);
    hipLaunchKernelGGL(bn_bwd_seg, dim3((C + 63) / 64, G, nseg), dim3(1024), 0, stream, qn, C,
                       q1, q2, seg);
    hipLaunchKernelGGL(bn_bwd_merge, dim3((C + 255) / 256), dim3(256), 0, stream, G, nseg, C, M,
                       seg, k1, k2, dgamma, dbeta);
  } else {
    hipLaunchKernelGGL(bn_bwd_final, dim3((C + 63) / 64, G), dim3(1024), 0, stream, G, qn, C, M,
                       q1, q2, k1, k2);
    if (dgamma || dbeta)
      hipLaunchKernelGGL(bn_bwd_param_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, G, C,
                         M, k1, k2, dgamma, dbeta);
  }
  if (!dy && !dres) return check_launch("bn_bwd");   // partial sums / parameter grads only
  if (mask || use_rows(C)) {
    int anblk, arpb;
    rows_geometry(M, C, anblk, arpb);
    hipLaunchKernelGGL(bn_bwd_apply_rows<S>, dim3(anblk, G), dim3(256), 0, stream, y, out, dout,
                       relu, mean, invstd, scale, shift, k1, k2, dy, dres, M, C, arpb, mask);
  } else {
    hipLaunchKernelGGL(bn_bwd_apply<S>, dim3(ew_grid(M * C / 8), G), dim3(256), 0, stream, y, out,
                       dout, relu, mean, invstd, scale, shift, k1, k2, dy, dres, M, C);
  }
  return check_launch("bn_bwd");
}

// Training-mode BN backward (+ReLU mask from `out`, + residual split):
//   dy = gamma*invstd*(dz - mean(dz) - xhat*mean(dz*xhat)),  dres = dz (nullable),
//   dgamma += sum dz*xhat, dbeta += sum dz (over all groups; nullable).
MAUV_API int mauv_bn_bwd(const float* y, const float* out, const float* dout, int relu,
                         const float* mean, const float* invstd, const float* scale,
                         const float* shift, int G, long long M, int C, float* workspace,
                         float* dy, float* dres, float* dgamma, float* dbeta,
                         const float* pre_p1, const float* pre_p2, int pre_nblk,
                         hipStream_t stream) {
  return bn_bwd_impl<SF32>(y, out, dout, relu, mean, invstd, scale, shift, G, M, C, workspace,
                           dy, dres, dgamma, dbeta, pre_p1, pre_p2, pre_nblk, stream);
}

// 16-bit activations (dtype 0 = bf16, 1 = f16): y/out/dout/dy/dres are 16-bit, statistics,
// scale/shift, workspace and parameter gradients fp32.
MAUV_API int mauv_bn_apply_h16(int dtype, const void* y, const float* scale, const float* shift,
                               const void* res, const float* res_scale, const float* res_shift,
                               int relu, void* out, int G, long long M, int C,
                               hipStream_t stream) {
  if (C % 8 != 0) { set_error("bn_apply_h16: C % 8 != 0"); return kErrArg; }
#define L(D) launch_apply<S16<D>>((const u16*)y, scale, shift, (const u16*)res, res_scale,  \
                                  res_shift, relu, (u16*)out, G, M, C, stream);
  MAUV_DT_DISPATCH(dtype, "bn_apply_h16", L)
#undef L
  return check_launch("bn_apply_h16");
}

MAUV_API int mauv_bn_bwd_h16(int dtype, const void* y, const void* out, const void* dout,
                             int relu, const float* mean, const float* invstd, const float* scale,
                             const float* shift, int G, long long M, int C, float* workspace,
                             void* dy, void* dres, float* dgamma, float* dbeta,
                             hipStream_t stream) {
#define L(D) return bn_bwd_impl<S16<D>>((const u16*)y, (const u16*)out, (const u16*)dout, relu, mean, \
                                        invstd, scale, shift, G, M, C, workspace, (u16*)dy,       \
                                        (u16*)dres, dgamma, dbeta, nullptr, nullptr, 0, stream);
  MAUV_DT_DISPATCH(dtype, "bn_bwd_h16", L)
#undef L
}

// Block-output BN apply that also writes the ReLU mask bits of the stored output (training):
// mask[G][M][C/8], bit e of byte j = out[8j + e] > 0.  The backward then reads 1 bit per
// element instead of the 2-4 B output (mauv_bn_bwd_mask).  dtype -1 = fp32, 0 = bf16, 1 = f16.
MAUV_API int mauv_bn_apply_mask(int dtype, const void* y, const float* scale, const float* shift,
                                const void* res, const float* res_scale, const float* res_shift,
                                void* out, unsigned char* mask, int G, long long M, int C,
                                hipStream_t stream) {
  if (C % 8 != 0 || C > 2048 || !mask) { set_error("bn_apply_mask: C % 8 != 0, C > 2048 or no mask"); return kErrArg; }
  if (dtype < 0) {
    launch_apply<SF32>((const float*)y, scale, shift, (const float*)res, res_scale, res_shift, 1,
                       (float*)out, G, M, C, stream, mask);
    return check_launch("bn_apply_mask");
  }
#define L(D) launch_apply<S16<D>>((const u16*)y, scale, shift, (const u16*)res, res_scale,  \
                                  res_shift, 1, (u16*)out, G, M, C, stream, mask);
  MAUV_DT_DISPATCH(dtype, "bn_apply_mask", L)
#undef L
  return check_launch("bn_apply_mask");
}

// BN + ReLU backward with the ReLU mask from mauv_bn_apply_mask (instead of the output).
MAUV_API int mauv_bn_bwd_mask(int dtype, const void* y, const unsigned char* mask,
                              const void* dout, const float* mean, const float* invstd,
                              const float* scale, int G, long long M, int C, float* workspace,
                              void* dy, void* dres, float* dgamma, float* dbeta,
                              hipStream_t stream) {
  if (!mask) { set_error("bn_bwd_mask: no mask"); return kErrArg; }
  if (dtype < 0)
    return bn_bwd_impl<SF32>((const float*)y, nullptr, (const float*)dout, 1, mean, invstd, scale,
                             nullptr, G, M, C, workspace, (float*)dy, (float*)dres, dgamma, dbeta,
                             nullptr, nullptr, 0, stream, mask);
#define L(D) return bn_bwd_impl<S16<D>>((const u16*)y, nullptr, (const u16*)dout, 1, mean, invstd,  \
                                        scale, nullptr, G, M, C, workspace, (u16*)dy, (u16*)dres, \
                                        dgamma, dbeta, nullptr, nullptr, 0, stream, mask);
  MAUV_DT_DISPATCH(dtype, "bn_bwd_mask", L)
#undef L
}

MAUV_API int mauv_bn_bwd_ex(int dtype, const void* y, const void* out, const unsigned char* mask,
                            const void* dout, int relu, const float* mean, const float* invstd,
                            const float* scale, const float* shift, int G, long long M, int C,
                            float* workspace, void* dy, void* dres, float* dgamma, float* dbeta,
                            const float* pre_p1, const float* pre_p2, int pre_nblk,
                            hipStream_t stream) {
  if (pre_p1 && (!pre_p2 || pre_nblk <= 0)) { set_error("bn_bwd_ex: pre_p1 needs pre_p2 and pre_nblk > 0"); return kErrArg; }
  if (mask) relu = 1, out = nullptr;
  if (dtype < 0)
    return bn_bwd_impl<SF32>((const float*)y, (const float*)out, (const float*)dout, relu, mean,
                             invstd, scale, shift, G, M, C, workspace, (float*)dy, (float*)dres,
                             dgamma, dbeta, pre_p1, pre_p2, pre_nblk, stream, mask);
#define L(D) return bn_bwd_impl<S16<D>>((const u16*)y, (const u16*)out, (const u16*)dout, relu, mean, \
                                        invstd, scale, shift, G, M, C, workspace, (u16*)dy,       \
                                        (u16*)dres, dgamma, dbeta, pre_p1, pre_p2, pre_nblk,      \
                                        stream, mask);
  MAUV_DT_DISPATCH(dtype, "bn_bwd_ex", L)
#undef L
}
