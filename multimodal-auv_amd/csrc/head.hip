// Fusion-head epilogues, the fused MC-head reductions, and small reductions.
//
//  * AdditiveAttention (models/base_models.py:43-52): with q|k|v produced by ONE linear over
//    the concatenated [Wq;Wk;Wv] sample (N = 384), the epilogues are
//       t = tanh(q + k)                        (attn_t)
//       s = Wm t + bm                          (linear, conv_gemm.hip 1x1 path)
//       a = softmax(s, dim=1);  o = v * a      (attn_out; o written into the concat slot)
//  * MC head (train/multimodal.py:121-127, :287-310; inference/predictors.py:65-84):
//       mean over MC of logits + cross-entropy (+ backward), and the sufficient statistics
//       sum_g p, sum_g p^2, sum_g H[p_g] -> mean prob, unbiased variance, aleatoric
//       entropy, predictive entropy, argmax.  Partial sums are shardable across GPUs
//       (MC-sharded inference: one all-reduce of [B,2C+1] doubles).
#include "mauv_common.h"

using namespace mauv;

namespace mauv {

// qkv rows are [q | k | v], each `hid` wide (the reference model: hid = 128, d_model 2048)
__global__ __launch_bounds__(256) void attn_t_kernel(const float* __restrict__ qkv, int rows,
                                                     int hid, float* __restrict__ t) {
  const long long total = (long long)rows * hid;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long r = i / hid;
    const int j = (int)(i - r * hid);
    t[i] = tanhf(qkv[r * 3 * hid + j] + qkv[r * 3 * hid + hid + j]);
  }
}

__global__ __launch_bounds__(256) void attn_t_bwd_kernel(const float* __restrict__ dt,
                                                         const float* __restrict__ t, int rows,
                                                         int hid, float* __restrict__ dqkv) {
  const long long total = (long long)rows * hid;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long r = i / hid;
    const int j = (int)(i - r * hid);
    const float tv = t[i];
    const float d = dt[i] * (1.0f - tv * tv);
    dqkv[r * 3 * hid + j] = d;
    dqkv[r * 3 * hid + hid + j] = d;
  }
}

// softmax over the hidden dim of one row, one wave per row (lane j covers j, j+64, ...):
// returns the row max and 1 / sum exp(s - max)
__device__ __forceinline__ void row_softmax_norm(const float* __restrict__ s, int hid, int lane,
                                                 float& m, float& inv) {
  m = -INFINITY;
  for (int j = lane; j < hid; j += 64) m = fmaxf(m, s[j]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  float e = 0.f;
  for (int j = lane; j < hid; j += 64) e += expf(s[j] - m);
  inv = 1.0f / wave_sum(e);
}

__global__ __launch_bounds__(256) void attn_out_kernel(const float* __restrict__ qkv,
                                                       const float* __restrict__ s, int rows,
                                                       int hid, float* __restrict__ comb,
                                                       int comb_ld, int comb_off) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float* sr = s + (long long)r * hid;
  float m, inv;
  row_softmax_norm(sr, hid, lane, m, inv);
  const float* v = qkv + (long long)r * 3 * hid + 2 * hid;
  float* o = comb + (long long)r * comb_ld + comb_off;
  for (int j = lane; j < hid; j += 64) o[j] = v[j] * (expf(sr[j] - m) * inv);
}

__global__ __launch_bounds__(256) void attn_out_bwd_kernel(const float* __restrict__ dcomb,
                                                           int comb_ld, int comb_off,
                                                           const float* __restrict__ qkv,
                                                           const float* __restrict__ s, int rows,
                                                           int hid, float* __restrict__ dqkv,
                                                           float* __restrict__ ds) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float* sr = s + (long long)r * hid;
  float m, inv;
  row_softmax_norm(sr, hid, lane, m, inv);
  const float* v = qkv + (long long)r * 3 * hid + 2 * hid;
  const float* d = dcomb + (long long)r * comb_ld + comb_off;
  float* dv = dqkv + (long long)r * 3 * hid + 2 * hid;
  float dot = 0.f;
  for (int j = lane; j < hid; j += 64) {
    const float a = expf(sr[j] - m) * inv;
    dv[j] = d[j] * a;
    dot += a * d[j] * v[j];
  }
  dot = wave_sum(dot);
  for (int j = lane; j < hid; j += 64) {
    const float a = expf(sr[j] - m) * inv;
    ds[(long long)r * hid + j] = a * (d[j] * v[j] - dot);
  }
}

// out[g][n] (+)= sum_rows dy[g][row][n]
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ dy, int G,
                                                     int rows, int N, float* __restrict__ out,
                                                     int accumulate) {
  const long long total = (long long)G * N;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long g = i / N;
    const int n = (int)(i - g * N);
    const float* src = dy + g * rows * (long long)N + n;
    float acc = 0.f;
    for (int r = 0; r < rows; ++r) acc += src[(long long)r * N];
    out[i] = accumulate ? out[i] + acc : acc;
  }
}

// mean over G of logits [G][B][C] -> [B][C]; optional cross-entropy with int64 labels.
__global__ __launch_bounds__(256) void mc_mean_ce_kernel(const float* __restrict__ logits,
                                                         const long long* __restrict__ labels,
                                                         int G, int B, int C,
                                                         float* __restrict__ mean,
                                                         float* __restrict__ loss,
                                                         long long* __restrict__ pred) {
  __shared__ float red[256];
  float acc = 0.f;
  for (int b = threadIdx.x; b < B; b += 256) {
    float m = -INFINITY;
    int arg = 0;
    for (int c = 0; c < C; ++c) {
      float s = 0.f;
      for (int g = 0; g < G; ++g) s += logits[((long long)g * B + b) * C + c];
      s = s / (float)G;
      mean[(long long)b * C + c] = s;
      if (s > m) { m = s; arg = c; }
    }
    if (pred) pred[b] = arg;
    if (labels) {
      float se = 0.f;
      for (int c = 0; c < C; ++c) se += expf(mean[(long long)b * C + c] - m);
      acc += (logf(se) + m) - mean[(long long)b * C + labels[b]];
    }
  }
  if (!labels) return;
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = red[0] / (float)B;
}

// dlogits[g][b][c] = (dmean[b][c] or g_loss*(softmax(mean)-onehot)/B) / G
__global__ __launch_bounds__(256) void mc_mean_bwd_kernel(const float* __restrict__ dmean,
                                                          const float* __restrict__ gloss,
                                                          const float* __restrict__ mean,
                                                          const long long* __restrict__ labels,
                                                          int G, int B, int C,
                                                          float* __restrict__ dlogits) {
  for (int b = blockIdx.x * 256 + threadIdx.x; b < B; b += gridDim.x * 256) {
    float d[32];
    if (labels) {
      float m = -INFINITY;
      for (int c = 0; c < C; ++c) m = fmaxf(m, mean[(long long)b * C + c]);
      float se = 0.f;
      for (int c = 0; c < C; ++c) se += expf(mean[(long long)b * C + c] - m);
      const float gl = gloss ? gloss[0] : 1.0f;
      for (int c = 0; c < C; ++c) {
        const float p = expf(mean[(long long)b * C + c] - m) / se;
        d[c] = gl * (p - (labels[b] == c ? 1.f : 0.f)) / (float)B;
      }
    } else {
      for (int c = 0; c < C; ++c) d[c] = dmean[(long long)b * C + c];
    }
    for (int g = 0; g < G; ++g)
      for (int c = 0; c < C; ++c) dlogits[((long long)g * B + b) * C + c] = d[c] / (float)G;
  }
}

// sums layout per item b: [sum_p (C)][sum_p2 (C)][sum_H] doubles, stride 2C+1.
__global__ __launch_bounds__(256) void mc_stats_kernel(const float* __restrict__ logits, int G,
                                                       int B, int C, float eps_h,
                                                       double* __restrict__ sums,
                                                       int accumulate) {
  for (int b = blockIdx.x * 256 + threadIdx.x; b < B; b += gridDim.x * 256) {
    double sp[32], sp2[32], sh = 0.0;
    for (int c = 0; c < C; ++c) { sp[c] = 0.0; sp2[c] = 0.0; }
    for (int g = 0; g < G; ++g) {
      const float* l = logits + ((long long)g * B + b) * C;
      float m = -INFINITY;
      for (int c = 0; c < C; ++c) m = fmaxf(m, l[c]);
      float se = 0.f;
      for (int c = 0; c < C; ++c) se += expf(l[c] - m);
      float h = 0.f;
      for (int c = 0; c < C; ++c) {
        const float p = expf(l[c] - m) / se;
        sp[c] += p;
        sp2[c] += (double)p * p;
        h -= p * logf(p + eps_h);
      }
      sh += h;
    }
    double* o = sums + (long long)b * (2 * C + 1);
    for (int c = 0; c < C; ++c) {
      o[c] = (accumulate ? o[c] : 0.0) + sp[c];
      o[C + c] = (accumulate ? o[C + c] : 0.0) + sp2[c];
    }
    o[2 * C] = (accumulate ? o[2 * C] : 0.0) + sh;
  }
}

__global__ __launch_bounds__(256) void mc_finalize_kernel(const double* __restrict__ sums, int N,
                                                          int B, int C, float eps_pred,
                                                          float* __restrict__ mean_prob,
                                                          float* __restrict__ var_unc,
                                                          float* __restrict__ alea,
                                                          float* __restrict__ pred_entropy,
                                                          long long* __restrict__ pred) {
  for (int b = blockIdx.x * 256 + threadIdx.x; b < B; b += gridDim.x * 256) {
    const double* s = sums + (long long)b * (2 * C + 1);
    double vsum = 0.0, H = 0.0;
    int arg = 0;
    float best = -INFINITY;
    for (int c = 0; c < C; ++c) {
      const double pm = s[c] / N;
      const float pmf = (float)pm;
      if (mean_prob) mean_prob[(long long)b * C + c] = pmf;
      vsum += (s[C + c] - N * pm * pm) / (double)(N - 1);
      H -= (double)pmf * log((double)pmf + (double)eps_pred);
      if (pmf > best) { best = pmf; arg = c; }
    }
    if (var_unc) var_unc[b] = (float)(vsum / C);
    if (alea) alea[b] = (float)(s[2 * C] / N);
    if (pred_entropy) pred_entropy[b] = (float)H;
    if (pred) pred[b] = arg;
  }
}

__global__ __launch_bounds__(256) void nonfinite_kernel(const float* __restrict__ p, long long n,
                                                        int* __restrict__ out) {
  int bad = 0;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    bad |= !isfinite(p[i]);
  bad = __syncthreads_or(bad);
  if (threadIdx.x == 0 && bad) atomicAdd(out, 1);
}

static int grid1(long long n, int cap = 4096) {
  long long b = (n + 255) / 256;
  if (b > cap) b = cap;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace mauv

static bool attn_args_ok(int rows, int hid) {
  if (rows < 0 || hid < 1) {
    set_error("attn: rows must be >= 0 and hid >= 1");
    return false;
  }
  return true;
}
MAUV_API int mauv_attn_t(const float* qkv, int rows, int hid, float* t, hipStream_t stream) {
  if (!attn_args_ok(rows, hid)) return -1;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(attn_t_kernel, dim3(grid1((long long)rows * hid)), dim3(256), 0, stream, qkv, rows, hid, t);
  return check_launch("attn_t");
}
MAUV_API int mauv_attn_t_bwd(const float* dt, const float* t, int rows, int hid, float* dqkv,
                             hipStream_t stream) {
  if (!attn_args_ok(rows, hid)) return -1;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(attn_t_bwd_kernel, dim3(grid1((long long)rows * hid)), dim3(256), 0, stream, dt, t, rows, hid, dqkv);
  return check_launch("attn_t_bwd");
}
MAUV_API int mauv_attn_out(const float* qkv, const float* s, int rows, int hid, float* comb,
                           int comb_ld, int comb_off, hipStream_t stream) {
  if (!attn_args_ok(rows, hid)) return -1;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(attn_out_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, qkv, s, rows, hid, comb, comb_ld, comb_off);
  return check_launch("attn_out");
}
MAUV_API int mauv_attn_out_bwd(const float* dcomb, int comb_ld, int comb_off, const float* qkv,
                               const float* s, int rows, int hid, float* dqkv, float* ds,
                               hipStream_t stream) {
  if (!attn_args_ok(rows, hid)) return -1;
  if (rows == 0) return 0;
  hipLaunchKernelGGL(attn_out_bwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, dcomb, comb_ld, comb_off, qkv, s, rows, hid, dqkv, ds);
  return check_launch("attn_out_bwd");
}
MAUV_API int mauv_colsum(const float* dy, int G, int rows, int N, float* out, int accumulate,
                         hipStream_t stream) {
  hipLaunchKernelGGL(colsum_kernel, dim3(grid1((long long)G * N)), dim3(256), 0, stream, dy, G, rows, N, out, accumulate);
  return check_launch("colsum");
}
// mean over MC samples of logits (train/multimodal.py:121), cross-entropy against int64
// labels (:127, nullable) and argmax of the mean (torch.max(output, 1), :151; nullable).
MAUV_API int mauv_mc_mean_ce(const float* logits, const long long* labels, int G, int B, int C,
                             float* mean, float* loss, long long* pred, hipStream_t stream) {
  if (C > 32) { set_error("mc_mean_ce: C > 32"); return kErrArg; }
  hipLaunchKernelGGL(mc_mean_ce_kernel, dim3(1), dim3(256), 0, stream, logits, labels, G, B, C, mean, loss, pred);
  return check_launch("mc_mean_ce");
}
MAUV_API int mauv_mc_mean_bwd(const float* dmean, const float* gloss, const float* mean,
                              const long long* labels, int G, int B, int C, float* dlogits,
                              hipStream_t stream) {
  if (C > 32) { set_error("mc_mean_bwd: C > 32"); return kErrArg; }
  hipLaunchKernelGGL(mc_mean_bwd_kernel, dim3(grid1(B)), dim3(256), 0, stream, dmean, gloss, mean, labels, G, B, C, dlogits);
  return check_launch("mc_mean_bwd");
}
MAUV_API int mauv_mc_stats(const float* logits, int G, int B, int C, float eps_h, double* sums,
                           int accumulate, hipStream_t stream) {
  if (C > 32) { set_error("mc_stats: C > 32"); return kErrArg; }
  hipLaunchKernelGGL(mc_stats_kernel, dim3(grid1(B)), dim3(256), 0, stream, logits, G, B, C, eps_h, sums, accumulate);
  return check_launch("mc_stats");
}
MAUV_API int mauv_mc_finalize(const double* sums, int N, int B, int C, float eps_pred,
                              float* mean_prob, float* var_unc, float* alea,
                              float* pred_entropy, long long* pred, hipStream_t stream) {
  hipLaunchKernelGGL(mc_finalize_kernel, dim3(grid1(B)), dim3(256), 0, stream, sums, N, B, C, eps_pred, mean_prob, var_unc, alea, pred_entropy, pred);
  return check_launch("mc_finalize");
}
MAUV_API int mauv_nonfinite_count(const float* p, long long n, int* out, hipStream_t stream) {
  hipLaunchKernelGGL(nonfinite_kernel, dim3(grid1(n, 2048)), dim3(256), 0, stream, p, n, out);
  return check_launch("nonfinite_count");
}
