// Implicit-GEMM convolution on CDNA4 16-bit MFMA (bf16 / f16 operands, fp32 accumulation).
//
// The reduced-precision counterpart of conv_gemm.hip for BASELINE configs[2] (bf16 training)
// and the reference predictor's autocast inference (inference/predictors.py:55): the same three
// GEMM views of every Bayesian conv of the three trunks (models/base_models.py:15-18,
// models/model_utils.py:57-61), one launch for all G MC samples (blockIdx.y = sample).
//
//   FWD   y [B*Ho*Wo][Cout]  = im2col(x)[.][R*S*Cin] . W_g^T            (16-bit out, fp32 BN
//                                                                        statistics partials)
//   DGRAD dx[B*H*W][Cin]     = gather(dy)[.][R*S*Cout] . W_g[(r,s,n)][c]  (per output-parity
//                                                                        class, as conv_gemm.hip)
//   WGRAD dW[Cout][R*S*Cin]  = dy^T[Cout][pixels] . im2col(x)[pixels][.]  (fp32 split-K slabs)
//
// MFMA v_mfma_f32_32x32x16_{bf16,f16}: lane l holds A[row l&31][k = 8(l>>5) + j] and
// B[k = 8(l>>5) + j][col l&31], j = 0..7.  Operands are staged global -> registers -> LDS in
// 16-byte chunks (8 channels; every conv of the path has Cin, Cout % 8 == 0 — the stems' 1/3
// input channels are zero-padded to 8 by the caller), double buffered, BK = 32 per stage, in
// one of two LDS images:
//   row image [rows][BK+8]   k-contiguous (80-B rows): an operand fragment is ONE
//                            ds_read_b128, conflict-free (FWD A and B, DGRAD A);
//   col image [BK][rows+32]  rows-contiguous, i.e. the natural layout of a k-strided operand
//                            (DGRAD B = KRSC weights along Cin, WGRAD A = dy, WGRAD B = x):
//                            an operand fragment is two ds_read_b64_tr_b16 hardware-transposed
//                            reads; the 64-B pad makes a 32-lane half's 4 rows x 64 B cover
//                            the 64 banks once (conflict-free).
// 256 threads = 4 waves (2x2), wave tile (BM/2)x(BN/2) = 2x2 MFMA tiles of 32x32.
#include <stdlib.h>

#include "conv_common.h"

namespace mauv {

enum { H_FWD = 0, H_DGRAD = 1, H_WGRAD = 2 };

struct ConvArgs16 {
  int B, H, W, Cin, Ho, Wo, Cout, R, S, stride, pad;
  long long xs_g, xs_b, xs_h, xs_w;  // x element strides (channel stride 1)
  const u16* x;
  const u16* w;  // [G][Cout][R][S][Cin]
  long long ws_g;
  const u16* dy;  // [G][B*Ho*Wo][Cout]
  void* out;      // FWD/DGRAD: 16-bit [G][M][N]; WGRAD: fp32 slabs [splits][G][M][N]
  long long out_sg;
  const u16* addend;
  int accumulate;
  int G, splits, kchunk;
  int M, N, K;
  int ph, pw, Hc, Wc, r0, s0, nr, ns;  // DGRAD output-parity class
  const float* xsc;                    // lazy BN(+ReLU) of x on load (FWD A, WGRAD B)
  const float* xsh;
  int xrelu;
  float *st_mean, *st_m2, *st_cnt;  // FWD epilogue BN statistics partials
  int st_nblk;
  const float* ysh;                 // FWD: centred storage (conv_common.h ConvArgs::ysh)
};

constexpr int HBK = 32;
constexpr int RLD = HBK + 8;
__host__ __device__ constexpr int cld(int rows) { return rows + 32; }

template <int DT>
__device__ __forceinline__ u32x4 bn_chunk(u32x4 v, const float* sc, const float* sh, int relu) {
  floatx8 f = unpack8<DT>(v);
  const floatx4 s0 = *(const floatx4*)sc, s1 = *(const floatx4*)(sc + 4);
  const floatx4 h0 = *(const floatx4*)sh, h1 = *(const floatx4*)(sh + 4);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[e] = f[e] * s0[e] + h0[e];
    f[4 + e] = f[4 + e] * s1[e] + h1[e];
  }
  if (relu) {
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = f[e] > 0.f ? f[e] : 0.f;
  }
  return pack8<DT>(f);
}

// operand fragment of 32 rows (R0..R0+31) for k-step s from a row image
__device__ __forceinline__ u32x4 row_frag(const u16* img, int R0, int s, int li, int lh) {
  return *(const u32x4*)(img + (R0 + li) * RLD + 16 * s + 8 * lh);
}
// ... and from a col image with leading dimension LD: col_frag (h16.h)

template <int MODE, int DT, int BM, int BN, bool TAPU>
__global__ __launch_bounds__(256) void conv_gemm_h16(const ConvArgs16 a) {
  constexpr bool A_COL = (MODE == H_WGRAD);
  constexpr bool B_COL = (MODE != H_FWD);
  constexpr int A_SZ = A_COL ? HBK * cld(BM) : BM * RLD;
  constexpr int B_SZ = B_COL ? HBK * cld(BN) : BN * RLD;
  constexpr int STG = A_SZ + B_SZ;
  constexpr int WM = BM / 2, WN = BN / 2, MI = WM / 32, NI = WN / 32;
  constexpr int NA = BM / 64, NB = BN / 64;  // 16-B chunks per thread per stage
  __shared__ __attribute__((aligned(16))) u16 smem[2 * STG];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
  int m0, n0;
  {  // XCD-aware tile order (as conv_gemm.hip): n-fastest logical tiles kept on one XCD
    const int nN = (a.N + BN - 1) / BN;
    const int b = blockIdx.x, nwg = gridDim.x, xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
    m0 = (L / nN) * BM;
    n0 = (L - (L / nN) * nN) * BN;
  }
  int g, sp = 0;
  if constexpr (MODE == H_WGRAD) { g = blockIdx.y / a.splits; sp = blockIdx.y % a.splits; }
  else g = blockIdx.y;
  int kbeg = 0, kend = a.K;
  if constexpr (MODE == H_WGRAD) { kbeg = sp * a.kchunk; kend = min(a.K, kbeg + a.kchunk); }

  const u16* xg = a.x + (long long)g * a.xs_g;
  const u16* wg = a.w + (long long)g * a.ws_g;
  const u16* dyg = a.dy + (long long)g * ((long long)a.B * a.Ho * a.Wo * a.Cout);

  // ---------------- per-thread loader state ----------------
  long long a_base[NA];
  int a_p0[NA], a_p1[NA];
  bool a_ok[NA];
  int b_r[NB], b_s[NB], b_c[NB];
  bool b_ok[NB];
  int px_b[NB], px_h[NB], px_w[NB];  // WGRAD B: pixel of this thread's chunk row
  const int kc = tid & 3;           // row images: chunk within the 32-deep k slice
  // A
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    if constexpr (MODE == H_FWD || MODE == H_DGRAD) {
      const int m = m0 + (tid >> 2) + 64 * j;
      a_ok[j] = m < a.M;
      const int mm = a_ok[j] ? m : 0;
      const int HW = (MODE == H_FWD) ? a.Ho * a.Wo : a.Hc * a.Wc;
      const int WW = (MODE == H_FWD) ? a.Wo : a.Wc;
      const int b = mm / HW, rem = mm - b * HW, oh = rem / WW, ow = rem - oh * WW;
      if constexpr (MODE == H_FWD) {
        a_base[j] = (long long)b * a.xs_b;
        a_p0[j] = oh * a.stride - a.pad;
        a_p1[j] = ow * a.stride - a.pad;
      } else {
        a_base[j] = (long long)b * a.Ho * a.Wo * a.Cout;
        a_p0[j] = oh * a.stride + a.ph + a.pad;
        a_p1[j] = ow * a.stride + a.pw + a.pad;
      }
    } else {  // WGRAD A (col image [pixel][cout])
      const int idx = tid + 256 * j;
      a_p0[j] = idx / (BM / 8);        // k row
      a_p1[j] = m0 + 8 * (idx % (BM / 8));  // cout
      a_ok[j] = a_p1[j] < a.M;
      a_base[j] = 0;
    }
  }
  // B
  floatx8 bsc[NB], bsh[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int idx = tid + 256 * j;
    if constexpr (MODE == H_FWD) {
      const int n = n0 + (tid >> 2) + 64 * j;
      b_ok[j] = n < a.N;
      b_r[j] = b_ok[j] ? n : 0;
    } else if constexpr (MODE == H_DGRAD) {
      b_r[j] = idx / (BN / 8);              // k row within the stage
      b_c[j] = n0 + 8 * (idx % (BN / 8));   // cin
      b_ok[j] = b_c[j] < a.N;
    } else {  // WGRAD B: fixed column chunk (r,s,c..c+7), moving pixel row
      const int col = n0 + 8 * (idx % (BN / 8));
      b_ok[j] = col < a.N;
      const int cc = b_ok[j] ? col : 0;
      const int rs = cc / a.Cin;
      b_c[j] = cc - rs * a.Cin;
      b_r[j] = rs / a.S;
      b_s[j] = rs - b_r[j] * a.S;
      const int p = kbeg + idx / (BN / 8);
      const int HW = a.Ho * a.Wo;
      px_b[j] = p / HW;
      const int rem = p - px_b[j] * HW;
      px_h[j] = rem / a.Wo;
      px_w[j] = rem - px_h[j] * a.Wo;
      if (a.xsc && b_ok[j]) {
        const float* s = a.xsc + g * a.Cin + b_c[j];
        const float* h = a.xsh + g * a.Cin + b_c[j];
#pragma unroll
        for (int e = 0; e < 8; ++e) { bsc[j][e] = s[e]; bsh[j][e] = h[e]; }
      }
    }
  }

  // tile-uniform tap counters (FWD with Cin % 32 == 0; DGRAD: Cout % 32 == 0 always)
  int t_r = 0, t_s = 0, t_c = 0;  // FWD: (r, s, c0)   DGRAD: (tr, ts, n0)

  u32x4 ra[NA], rb[NB];
  const u32x4 zero = {0u, 0u, 0u, 0u};

  auto load = [&](int k0) {
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      u32x4 v = zero;
      if constexpr (MODE == H_FWD) {
        int r, s, c;
        bool kok = true;
        if constexpr (TAPU) {
          r = t_r; s = t_s; c = t_c + 8 * kc;
        } else {
          const int k = k0 + 8 * kc;
          kok = k < kend;
          const int tap = k / a.Cin;
          c = k - tap * a.Cin;
          r = tap / a.S;
          s = tap - r * a.S;
        }
        const int ih = a_p0[j] + r, iw = a_p1[j] + s;
        if (a_ok[j] && kok && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) {
          v = *(const u32x4*)(xg + a_base[j] + (long long)ih * a.xs_h + (long long)iw * a.xs_w + c);
          if (a.xsc) v = bn_chunk<DT>(v, a.xsc + g * a.Cin + c, a.xsh + g * a.Cin + c, a.xrelu);
        }
      } else if constexpr (MODE == H_DGRAD) {
        const int ohn = a_p0[j] - a.r0 - a.stride * t_r, own = a_p1[j] - a.s0 - a.stride * t_s;
        if (a_ok[j] && ohn >= 0 && own >= 0) {
          const int oh = a.stride == 1 ? ohn : ohn / a.stride;
          const int ow = a.stride == 1 ? own : own / a.stride;
          if (oh < a.Ho && ow < a.Wo)
            v = *(const u32x4*)(dyg + a_base[j] + ((long long)oh * a.Wo + ow) * a.Cout + t_c + 8 * kc);
        }
      } else {  // WGRAD A
        const int p = k0 + a_p0[j];
        if (a_ok[j] && p < kend) v = *(const u32x4*)(dyg + (long long)p * a.Cout + a_p1[j]);
      }
      ra[j] = v;
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      u32x4 v = zero;
      if constexpr (MODE == H_FWD) {
        const int k = k0 + 8 * kc;
        if (b_ok[j] && k < kend) v = *(const u32x4*)(wg + (long long)b_r[j] * a.K + k);
      } else if constexpr (MODE == H_DGRAD) {
        const int n = t_c + b_r[j];
        const int r = a.r0 + a.stride * t_r, s = a.s0 + a.stride * t_s;
        if (b_ok[j]) v = *(const u32x4*)(wg + (((long long)n * a.R + r) * a.S + s) * a.Cin + b_c[j]);
      } else {  // WGRAD B
        const int p = k0 + (tid + 256 * j) / (BN / 8);
        if (b_ok[j] && p < kend) {
          const int ih = px_h[j] * a.stride - a.pad + b_r[j];
          const int iw = px_w[j] * a.stride - a.pad + b_s[j];
          if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) {
            v = *(const u32x4*)(xg + (long long)px_b[j] * a.xs_b + (long long)ih * a.xs_h +
                                (long long)iw * a.xs_w + b_c[j]);
            if (a.xsc) {
              floatx8 f = unpack8<DT>(v);
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                f[e] = f[e] * bsc[j][e] + bsh[j][e];
                if (a.xrelu) f[e] = f[e] > 0.f ? f[e] : 0.f;
              }
              v = pack8<DT>(f);
            }
          }
        }
        // advance this chunk's pixel by one stage
        px_w[j] += HBK;
        while (px_w[j] >= a.Wo) { px_w[j] -= a.Wo; ++px_h[j]; }
        while (px_h[j] >= a.Ho) { px_h[j] -= a.Ho; ++px_b[j]; }
      }
      rb[j] = v;
    }
    // advance the tile-uniform tap counters by one stage
    if constexpr ((MODE == H_FWD && TAPU)) {
      t_c += HBK;
      if (t_c >= a.Cin) { t_c = 0; if (++t_s == a.S) { t_s = 0; ++t_r; } }
    } else if constexpr (MODE == H_DGRAD) {
      t_c += HBK;
      if (t_c >= a.Cout) { t_c = 0; if (++t_s == a.ns) { t_s = 0; ++t_r; } }
    }
  };

  auto store = [&](int buf) {
    u16* A = smem + buf * STG;
    u16* Bm = A + A_SZ;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      if constexpr (A_COL) {
        const int idx = tid + 256 * j;
        *(u32x4*)(A + (idx / (BM / 8)) * cld(BM) + 8 * (idx % (BM / 8))) = ra[j];
      } else {
        *(u32x4*)(A + ((tid >> 2) + 64 * j) * RLD + 8 * kc) = ra[j];
      }
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if constexpr (B_COL) {
        const int idx = tid + 256 * j;
        *(u32x4*)(Bm + (idx / (BN / 8)) * cld(BN) + 8 * (idx % (BN / 8))) = rb[j];
      } else {
        *(u32x4*)(Bm + ((tid >> 2) + 64 * j) * RLD + 8 * kc) = rb[j];
      }
    }
  };

  floatx16 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  const int ntiles = (kend - kbeg + HBK - 1) / HBK;
  if (ntiles > 0) {
    load(kbeg);
    store(0);
  }
  __syncthreads();
  int cur = 0;
  for (int t = 0; t < ntiles; ++t) {
    const bool more = t + 1 < ntiles;
    if (more) load(kbeg + (t + 1) * HBK);
    const u16* A = smem + cur * STG;
    const u16* Bm = A + A_SZ;
#pragma unroll
    for (int s = 0; s < HBK / 16; ++s) {
      u32x4 af[MI], bfr[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
        af[mi] = A_COL ? col_frag(A, cld(BM), wm * WM + mi * 32, s, lane)
                       : row_frag(A, wm * WM + mi * 32, s, li, lh);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        bfr[ni] = B_COL ? col_frag(Bm, cld(BN), wn * WN + ni * 32, s, lane)
                        : row_frag(Bm, wn * WN + ni * 32, s, li, lh);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = H16<DT>::mfma(af[mi], bfr[ni], acc[mi][ni]);
    }
    if (more) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // ---------------- epilogue ----------------
  if ((MODE == H_FWD) && a.ysh) {  // centred storage (conv_epi16.h acc_start16's semantics)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int col = n0 + wn * WN + ni * 32 + li;
      const float c = col < a.N ? a.ysh[col] : 0.f;
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mi][ni][r] -= c;
    }
  }
  // FWD statistics (from the fp32 accumulators, before any rounding)
  if ((MODE == H_FWD) && a.st_mean) {
    const int nvalid = min(BM, a.M - m0);
    float s1[NI], s2[NI], mean[NI];
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) { s1[ni] = 0.f; s2[ni] = 0.f; }
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * WM + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (row < a.M) s1[ni] += acc[mi][ni][r];
        }
    float* red = (float*)smem;  // LDS is free: the main loop ended with a barrier
    const int tcol = wn * WN + li;
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) s1[ni] += __shfl_xor(s1[ni], 32, 64);
    if (lh == 0) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) red[wm * BN + tcol + ni * 32] = s1[ni];
    }
    __syncthreads();
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
      mean[ni] = (red[tcol + ni * 32] + red[BN + tcol + ni * 32]) / (float)nvalid;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * WM + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (row < a.M) {
            const float d = acc[mi][ni][r] - mean[ni];
            s2[ni] += d * d;
          }
        }
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) s2[ni] += __shfl_xor(s2[ni], 32, 64);
    if (lh == 0) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) red[2 * BN + wm * BN + tcol + ni * 32] = s2[ni];
    }
    __syncthreads();
    if (tid < BN && n0 + tid < a.N) {
      const float t1 = red[tid] + red[BN + tid], t2 = red[2 * BN + tid] + red[3 * BN + tid];
      const int mt = m0 / BM;
      const long long so = ((long long)g * a.st_nblk + mt) * a.N + n0 + tid;
      a.st_mean[so] = t1 / (float)nvalid;
      a.st_m2[so] = t2;
      if (n0 + tid == 0) a.st_cnt[(long long)g * a.st_nblk + mt] = (float)nvalid;
    }
    __syncthreads();  // red is overwritten by the staged store below
  }

  if constexpr (MODE == H_WGRAD) {  // fp32 split-K slabs: 32 lanes x 4 B contiguous per store
    float* outg = (float*)a.out + ((long long)sp * a.G + g) * ((long long)a.M * a.N);
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int col = n0 + wn * WN + ni * 32 + li;
        if (col >= a.N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * WM + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (row < a.M) outg[(long long)row * a.N + col] = acc[mi][ni][r];
        }
      }
  } else {
    // 16-bit output through LDS: each wave row (wm = 0, 1) in turn parks its fp32 accumulators
    // as a [WM][BN+4] tile, then all 256 threads write it out as 16-byte rows of 8 channels
    // (adding the residual addend / previous dx in fp32, one rounding).
    constexpr int SLD = BN + 4;
    static_assert(WM * SLD * 4 <= 2 * STG * 2, "staging tile exceeds LDS");
    float* stile = (float*)smem;
    constexpr int CPR = BN / 8, NCH = WM * CPR;
    u16* outp = (u16*)a.out;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      if (wm == pass) {
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              stile[(mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * SLD + wn * WN + ni * 32 + li] =
                  acc[mi][ni][r];
      }
      __syncthreads();
      for (int c = tid; c < NCH; c += 256) {
        const int rl = c / CPR, cc = c - rl * CPR;
        const int row = m0 + pass * WM + rl, col = n0 + 8 * cc;
        if (row >= a.M || col >= a.N) continue;
        floatx4 v0 = *(const floatx4*)(stile + rl * SLD + 8 * cc);
        floatx4 v1 = *(const floatx4*)(stile + rl * SLD + 8 * cc + 4);
        floatx8 f;
#pragma unroll
        for (int e = 0; e < 4; ++e) { f[e] = v0[e]; f[4 + e] = v1[e]; }
        long long orow = row;
        if constexpr (MODE == H_DGRAD) {
          if (a.stride != 1) {
            const int HW = a.Hc * a.Wc, b = row / HW, rem = row - b * HW;
            const int i = rem / a.Wc, jj = rem - i * a.Wc;
            orow = ((long long)b * a.H + a.stride * i + a.ph) * a.W + a.stride * jj + a.pw;
          }
        }
        const long long o = (long long)g * a.out_sg + orow * a.N + col;
        if constexpr (MODE == H_DGRAD) {
          if (a.addend) f += unpack8<DT>(*(const u32x4*)(a.addend + o));
          if (a.accumulate) f += unpack8<DT>(*(const u32x4*)(outp + o));
        }
        *(u32x4*)(outp + o) = pack8<DT>(f);
      }
      __syncthreads();
    }
  }
}

template <int MODE, int DT, int BM, int BN, bool TAPU>
static void launch16(const ConvArgs16& a, hipStream_t st) {
  dim3 grid(ceil_div(a.M, BM) * ceil_div(a.N, BN), MODE == H_WGRAD ? a.G * a.splits : a.G);
  hipLaunchKernelGGL((conv_gemm_h16<MODE, DT, BM, BN, TAPU>), grid, dim3(256), 0, st, a);
}

template <int MODE, int DT, bool TAPU>
static void tiles16(const ConvArgs16& a, hipStream_t st) {
  const int bm = conv_tile_rows(a.M), bn = conv_tile_rows(a.N);
  if (bm == 64 && bn == 64) launch16<MODE, DT, 64, 64, TAPU>(a, st);
  else if (bm == 64) launch16<MODE, DT, 64, 128, TAPU>(a, st);
  else if (bn == 64) launch16<MODE, DT, 128, 64, TAPU>(a, st);
  else launch16<MODE, DT, 128, 128, TAPU>(a, st);
}

template <int MODE, bool TAPU>
static void dispatch16(int dt, const ConvArgs16& a, hipStream_t st) {
  if (dt == DT_BF16) tiles16<MODE, DT_BF16, TAPU>(a, st);
  else tiles16<MODE, DT_F16, TAPU>(a, st);
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static ConvArgs16 make_args16(int G, int B, int H, int W, int Cin, int Cout, int R, int S,
                              int stride, int pad, const long long* xs) {
  ConvArgs16 a{};
  a.G = G; a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.R = R; a.S = S;
  a.stride = stride; a.pad = pad;
  a.Ho = (H + 2 * pad - R) / stride + 1;
  a.Wo = (W + 2 * pad - S) / stride + 1;
  if (xs) { a.xs_g = xs[0]; a.xs_b = xs[1]; a.xs_h = xs[2]; a.xs_w = xs[3]; }
  else {
    a.xs_w = Cin; a.xs_h = (long long)W * Cin; a.xs_b = (long long)H * W * Cin;
    a.xs_g = (long long)B * H * W * Cin;
  }
  a.ws_g = (long long)Cout * R * S * Cin;
  a.splits = 1;
  return a;
}

// the pipelined kernels (conv_pipe16.hip) take the fp32 argument block with 16-bit pointers
static ConvArgs pipe_args(const ConvArgs16& h) {
  ConvArgs a{};
  a.B = h.B; a.H = h.H; a.W = h.W; a.Cin = h.Cin; a.Ho = h.Ho; a.Wo = h.Wo; a.Cout = h.Cout;
  a.R = h.R; a.S = h.S; a.stride = h.stride; a.pad = h.pad;
  a.xs_g = h.xs_g; a.xs_b = h.xs_b; a.xs_h = h.xs_h; a.xs_w = h.xs_w; a.xs_c = 1;
  a.x = (const float*)h.x; a.w = (const float*)h.w; a.ws_g = h.ws_g; a.dy = (const float*)h.dy;
  a.out = (float*)h.out; a.out_sg = h.out_sg; a.addend = (const float*)h.addend;
  a.accumulate = h.accumulate; a.G = h.G; a.splits = h.splits; a.kchunk = h.kchunk;
  a.M = h.M; a.N = h.N; a.K = h.K;
  a.ph = h.ph; a.pw = h.pw; a.Hc = h.Hc; a.Wc = h.Wc; a.r0 = h.r0; a.s0 = h.s0; a.nr = h.nr;
  a.ns = h.ns; a.xsc = h.xsc; a.xsh = h.xsh; a.xrelu = h.xrelu;
  a.st_mean = h.st_mean; a.st_m2 = h.st_m2; a.st_cnt = h.st_cnt; a.st_nblk = h.st_nblk;
  a.ysh = h.ysh;
  return a;
}

static int check_shape16(const char* what, int dt, int G, int B, int Cin, int Cout,
                         const long long* xs) {
  if (dt != DT_BF16 && dt != DT_F16) { set_error(std::string(what) + ": dtype must be 0 (bf16) or 1 (f16)"); return kErrArg; }
  if (G <= 0 || B <= 0 || Cin <= 0 || Cout <= 0) { set_error(std::string(what) + ": bad shape"); return kErrArg; }
  if (Cin % 8 || Cout % 8) { set_error(std::string(what) + ": 16-bit path needs Cin, Cout % 8 == 0 (pad the stem input)"); return kErrArg; }
  if (xs && (xs[4] != 1 || xs[0] % 8 || xs[1] % 8 || xs[2] % 8 || xs[3] % 8)) {
    set_error(std::string(what) + ": x strides must be channel-contiguous multiples of 8");
    return kErrArg;
  }
  return 0;
}

}  // namespace mauv

using namespace mauv;

MAUV_API int mauv_conv2d_fwd_h16(int dtype, const void* x, const long long* x_strides,
                                 const float* x_scale, const float* x_shift, int x_relu,
                                 const void* w, void* y, int G, int B, int H, int W, int Cin,
                                 int Cout, int R, int S, int stride, int pad, float* st_mean,
                                 float* st_m2, float* st_cnt, const float* y_shift,
                                 hipStream_t stream) {
  if (int e = check_shape16("conv2d_fwd_h16", dtype, G, B, Cin, Cout, x_strides)) return e;
  if (!aligned16(x) || !aligned16(w)) { set_error("conv2d_fwd_h16: x, w must be 16-B aligned"); return kErrArg; }
  ConvArgs16 a = make_args16(G, B, H, W, Cin, Cout, R, S, stride, pad, x_strides);
  a.x = (const u16*)x; a.w = (const u16*)w; a.out = y;
  a.xsc = x_scale; a.xsh = x_shift; a.xrelu = x_relu;
  a.M = B * a.Ho * a.Wo; a.N = Cout; a.K = R * S * Cin;
  a.out_sg = (long long)a.M * a.N;
  a.st_mean = st_mean; a.st_m2 = st_m2; a.st_cnt = st_cnt;
  a.st_nblk = ceil_div(a.M, conv_tile_rows(a.M));
  a.ysh = y_shift;
  if (conv_pipe16_launch(FWD, dtype, pipe_args(a), stream)) {}
  else if (Cin % HBK == 0) dispatch16<H_FWD, true>(dtype, a, stream);
  else dispatch16<H_FWD, false>(dtype, a, stream);
  return check_launch("conv2d_fwd_h16");
}

// A bottleneck's conv1 (1x1, stride 1) whose input is the previous block's output, formed while
// its tiles are loaded: out = relu(y*scale + shift + r), r = res or res*res_scale + res_shift
// (conv_big16.hip's fold; bn_apply's arithmetic), written through once (with out_mask non-null
// also its ReLU-mask bits, mauv_bn_apply_mask's) and fed to the GEMM.
// 0: launched; 1: shape outside the kernel (nothing launched: the caller runs mauv_bn_apply,
// then mauv_conv2d_fwd_h16 on its output); < 0: argument error.
MAUV_API int mauv_conv2d_fwd_fold_h16(int dtype, const void* y, const float* scale,
                                      const float* shift, const void* res, const float* res_scale,
                                      const float* res_shift, void* out, unsigned char* out_mask,
                                      const void* w, void* y1, int G, int B, int H, int W,
                                      int Cin, int Cout,
                                      float* st_mean, float* st_m2, float* st_cnt,
                                      const float* y1_shift, hipStream_t stream) {
  if (int e = check_shape16("conv2d_fwd_fold_h16", dtype, G, B, Cin, Cout, nullptr)) return e;
  if (!y || !scale || !shift || !res || !out || !w || !y1 || !res_scale != !res_shift) {
    set_error("conv2d_fwd_fold_h16: y, scale, shift, res, out, w, y1 required; res_scale and "
              "res_shift together");
    return kErrArg;
  }
  if (!aligned16(y) || !aligned16(res) || !aligned16(out) || !aligned16(w)) {
    set_error("conv2d_fwd_fold_h16: y, res, out, w must be 16-B aligned");
    return kErrArg;
  }
  ConvArgs16 h = make_args16(G, B, H, W, Cin, Cout, 1, 1, 1, 0, nullptr);
  h.x = (const u16*)y; h.w = (const u16*)w; h.out = y1;
  h.xsc = scale; h.xsh = shift; h.xrelu = 1;
  h.M = B * H * W; h.N = Cout; h.K = Cin;
  h.out_sg = (long long)h.M * h.N;
  h.st_mean = st_mean; h.st_m2 = st_m2; h.st_cnt = st_cnt;
  h.st_nblk = ceil_div(h.M, conv_tile_rows(h.M));
  h.ysh = y1_shift;
  ConvArgs a = pipe_args(h);
  a.rs = res; a.rs_sc = res_scale; a.rs_sh = res_shift; a.fout = out; a.fmask = out_mask;
  if (!conv_big16_fold_launch(dtype, a, stream)) return 1;
  return check_launch("conv2d_fwd_fold_h16");
}

// 16-bit counterpart of mauv_stem_fwd_f32 (conv_gemm.hip): the pipelined kernel over the
// shared im2col rows with the G weight sets stacked along N; Kp % 64 == 0.
MAUV_API int mauv_stem_fwd_h16(int dtype, const void* cols, const void* w, void* y, int G,
                               int M, int Kp, int Cout, float* st_mean, float* st_m2,
                               float* st_cnt, const float* y_shift, hipStream_t stream) {
  if (int e = check_shape16("stem_fwd_h16", dtype, G, 1, Kp, Cout, nullptr)) return e;
  if (M <= 0 || Kp % 64) { set_error("stem_fwd_h16: needs M > 0 and Kp % 64 == 0"); return kErrArg; }
  if (!aligned16(cols) || !aligned16(w)) { set_error("stem_fwd_h16: cols, w must be 16-B aligned"); return kErrArg; }
  ConvArgs16 h = make_args16(1, 1, 1, M, Kp, G * Cout, 1, 1, 1, 0, nullptr);
  h.x = (const u16*)cols; h.w = (const u16*)w; h.out = y;
  h.M = M; h.N = G * Cout; h.K = Kp;
  h.out_sg = (long long)M * Cout;
  h.st_mean = st_mean; h.st_m2 = st_m2; h.st_cnt = st_cnt;
  h.st_nblk = ceil_div(M, conv_tile_rows(M));
  h.ysh = y_shift;
  ConvArgs a = pipe_args(h);
  a.cpg = Cout;
  // the pipelined kernel reads cols by a buffer descriptor (31-bit byte offsets): rows beyond
  // that (configs[4]'s 512 px sonar at B = 256: 16.8 M rows) go in chunks of whole 128-row
  // tiles, each writing its rows of y and its statistics blocks (st_base)
  const long long lim_rows = (0x7fff0000LL / 2 / Kp) / 128 * 128;
  for (long long r0 = 0; r0 < M; r0 += lim_rows) {
    ConvArgs c = a;
    c.M = (int)(M - r0 < lim_rows ? M - r0 : lim_rows);
    // cols as one 1 x M "image" of Kp channels (make_args16 above): the chunk is 1 x c.M
    c.W = c.Wo = c.M;
    c.xs_h = c.xs_b = (long long)c.M * Kp;
    c.x = (const float*)((const u16*)cols + r0 * Kp);
    c.out = (float*)((u16*)y + r0 * Cout);
    c.st_base = (int)(r0 / 128);
    if (!conv_pipe16_launch(FWD, dtype, c, stream)) { set_error("stem_fwd_h16: shape outside the pipelined kernel"); return kErrArg; }
  }
  return check_launch("stem_fwd_h16");
}

MAUV_API int mauv_conv2d_bwd_data_h16(int dtype, const void* dy, const void* w, void* dx,
                                      const void* addend, int accumulate, int G, int B, int H,
                                      int W, int Cin, int Cout, int R, int S, int stride, int pad,
                                      hipStream_t stream) {
  return mauv_conv2d_bwd_data_bn_h16(dtype, dy, w, dx, addend, accumulate, G, B, H, W, Cin, Cout,
                                     R, S, stride, pad, nullptr, nullptr, nullptr, nullptr,
                                     nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr,
                                     stream);
}

// The data gradient with the BN-backward partial sums of the BatchNorm whose output gradient dx
// is (bn_bwd_partial's sum dz, sum dz*xhat per [G][nblk][Cin], nblk =
// mauv_conv2d_bwd_data_stat_blocks) written by the epilogue (conv_epi16.h).  ReLU mask source:
// bn_mask bits (mauv_bn_apply_mask), else bn_out > 0, else bn_y*bn_scale + bn_shift > 0.  The
// partials need the pipelined kernel (Cout % 64 == 0) and every dx row written by this call
// (accumulate without addend over a tapless parity class is refused).  addend_mask (nullable):
// the addend counts only where these ReLU-mask bits ([G][B*H*W][Cin] / 8, mauv_bn_apply_mask)
// are set — the residual gradient of a block output's BN without a dres tensor.
MAUV_API int mauv_conv2d_bwd_data_bn_h16(int dtype, const void* dy, const void* w, void* dx,
                                         const void* addend, int accumulate, int G, int B, int H,
                                         int W, int Cin, int Cout, int R, int S, int stride,
                                         int pad, const unsigned char* addend_mask,
                                         const void* bn_y, const void* bn_out,
                                         const unsigned char* bn_mask, const float* bn_scale,
                                         const float* bn_shift, const float* bn_mean,
                                         const float* bn_invstd, int bn_relu, float* bn_p1,
                                         float* bn_p2, hipStream_t stream) {
  if (int e = check_shape16("conv2d_bwd_data_h16", dtype, G, B, Cin, Cout, nullptr)) return e;
  if (Cout % HBK) { set_error("conv2d_bwd_data_h16: needs Cout % 32 == 0"); return kErrArg; }
  const bool bst = bn_p1 != nullptr;
  if (addend_mask && (!addend || Cout % 64)) { set_error("conv2d_bwd_data_bn_h16: addend_mask needs an addend and Cout % 64 == 0"); return kErrArg; }
  if (bst) {
    if (!bn_p2 || !bn_y || !bn_mean || !bn_invstd || Cout % 64) { set_error("conv2d_bwd_data_bn_h16: partials need p1, p2, y, mean, invstd and Cout % 64 == 0"); return kErrArg; }
    if (bn_relu && !bn_mask && !bn_out && (!bn_scale || !bn_shift)) { set_error("conv2d_bwd_data_bn_h16: relu mask needs mask, out or scale/shift"); return kErrArg; }
    if (!aligned16(bn_y) || !aligned16(bn_out)) { set_error("conv2d_bwd_data_bn_h16: y, out must be 16-B aligned"); return kErrArg; }
  }
  ConvArgs16 a = make_args16(G, B, H, W, Cin, Cout, R, S, stride, pad, nullptr);
  a.dy = (const u16*)dy; a.w = (const u16*)w; a.out = dx;
  a.addend = (const u16*)addend; a.accumulate = accumulate;
  a.N = Cin;
  a.out_sg = (long long)B * H * W * Cin;
  int bp_base = 0;
  const int bp_nblk = bst ? mauv_conv2d_bwd_data_stat_blocks(G, B, H, W, Cin, Cout, R, S, stride, pad) : 0;
  for (int ph = 0; ph < stride; ++ph)
    for (int pw = 0; pw < stride; ++pw) {
      a.ph = ph; a.pw = pw;
      a.Hc = (H - ph + stride - 1) / stride;
      a.Wc = (W - pw + stride - 1) / stride;
      a.r0 = (ph + pad) % stride;
      a.s0 = (pw + pad) % stride;
      a.nr = a.r0 < R ? (R - a.r0 + stride - 1) / stride : 0;
      a.ns = a.s0 < S ? (S - a.s0 + stride - 1) / stride : 0;
      a.M = B * a.Hc * a.Wc;
      a.K = a.nr * a.ns * Cout;
      if (a.M <= 0) continue;
      // a tapless class accumulating into dx adds nothing (stride-2 1x1 downsample: 3 of 4)
      if (a.K == 0 && accumulate && !addend) {
        if (bst) { set_error("conv2d_bwd_data_bn_h16: partials over a tapless accumulate class"); return kErrArg; }
        continue;
      }
      ConvArgs p = pipe_args(a);
      p.add_mask = addend_mask;
      if (bst) {
        p.bp_y = (const float*)bn_y; p.bp_out = (const float*)bn_out; p.bp_mask = bn_mask;
        p.bp_sc = bn_scale; p.bp_sh = bn_shift; p.bp_mean = bn_mean; p.bp_invstd = bn_invstd;
        p.bp_relu = bn_relu; p.bp_p1 = bn_p1; p.bp_p2 = bn_p2;
        p.bp_nblk = bp_nblk; p.bp_base = bp_base;
        bp_base += ceil_div(a.M, conv_tile_rows(a.M));
        if (!conv_pipe16_launch(DGRAD, dtype, p, stream)) { set_error("conv2d_bwd_data_bn_h16: shape outside the pipelined kernel"); return kErrArg; }
      } else if (!conv_pipe16_launch(DGRAD, dtype, p, stream)) {
        if (addend_mask) { set_error("conv2d_bwd_data_bn_h16: addend_mask outside the pipelined kernel"); return kErrArg; }
        dispatch16<H_DGRAD, true>(dtype, a, stream);
      }
    }
  return check_launch("conv2d_bwd_data_h16");
}

MAUV_API int mauv_conv2d_bwd_weight_h16(int dtype, const void* x, const long long* x_strides,
                                        const float* x_scale, const float* x_shift, int x_relu,
                                        const void* dy, float* ws, int splits, int G, int B,
                                        int H, int W, int Cin, int Cout, int R, int S, int stride,
                                        int pad, hipStream_t stream) {
  if (int e = check_shape16("conv2d_bwd_weight_h16", dtype, G, B, Cin, Cout, x_strides)) return e;
  ConvArgs16 a = make_args16(G, B, H, W, Cin, Cout, R, S, stride, pad, x_strides);
  a.x = (const u16*)x; a.dy = (const u16*)dy; a.out = ws;
  a.xsc = x_scale; a.xsh = x_shift; a.xrelu = x_relu;
  a.M = Cout; a.N = R * S * Cin; a.K = B * a.Ho * a.Wo;
  a.splits = splits;
  ConvArgs p = pipe_args(a);
  p.kchunk = ((a.K + splits - 1) / splits + 63) / 64 * 64;  // the pipelined kernel's BK
  a.kchunk = ((a.K + splits - 1) / splits + HBK - 1) / HBK * HBK;
  if (!conv_pipe16_launch(WGRAD, dtype, p, stream)) dispatch16<H_WGRAD, false>(dtype, a, stream);
  return check_launch("conv2d_bwd_weight_h16");
}

