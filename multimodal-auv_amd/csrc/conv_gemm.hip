// Implicit-GEMM convolution (forward, data-gradient, weight-gradient) on CDNA4 MFMA, fp32.
//
// Replaces F.conv2d inside bayesian-torch Conv2dReparameterization.forward (called for every
// ResNet-50 conv of the three trunks, reference models/base_models.py:15-18 and
// models/model_utils.py:57-61) and its cuDNN backward (train/multimodal.py:138).  The MC
// loop of train/multimodal.py:107-112 is collapsed into the grid: blockIdx.z = MC sample g,
// each with its own sampled weight set W_g and its own activations.
//
// Layouts (all NHWC, channel-last, per MC group g):
//   x   [G][B][H][W][Cin]   (arbitrary element strides; group stride 0 = shared input,
//                            used by the stems which read the caller's NCHW images directly)
//   W_g [G][Cout][R][S][Cin]  sampled weights (written by mauv_reparam_sample_conv)
//   y   [G][B][Ho][Wo][Cout]
// GEMM views:
//   FWD   y [B*Ho*Wo][Cout]   = im2col(x)[B*Ho*Wo][R*S*Cin] . W_g^T
//   DGRAD dx[B*H*W][Cin]      = gather(dy)[B*H*W][R*S*Cout] . W_g[(r,s,n)][c]
//   WGRAD dW[Cout][R*S*Cin]   = dy^T[Cout][B*Ho*Wo] . im2col(x)[B*Ho*Wo][R*S*Cin]
//                               (split-K over pixels; fp32 partial slabs, reduced
//                                deterministically by mauv_reparam_bwd)
// Tiles: 256 threads = 4 waves (2x2), block tile BM x BN x 16, double-buffered LDS stored
// k-major ([k][row], rows contiguous) so each MFMA operand is one conflict-free ds_read_b32;
// MFMA v_mfma_f32_32x32x2_f32 (exact fp32, fmaf-chain numerics).
//
// Arithmetic of the fp32 products (MauvRoute.f32_math; template parameter SPL):
//   SPL = 0  exact  — v_mfma_f32_32x32x2_f32 (f32 MFMA = the f32 vector rate, 157 TF/s);
//   SPL = 6  split  (default) — every staged fp32 operand element is written to LDS as three
//            bf16 planes, x = h + m + l exactly (h16.h split_bf16), and each 32x32x16 k-step
//            issues the six plane products h.h | h.m, m.h, h.l, l.h, m.m on
//            v_mfma_f32_32x32x16_bf16 (products exact in fp32, fp32 accumulation).  The
//            dropped m.l, l.m, l.l total <= 2^-24 |a.b| (one fp32 rounding), and h.h
//            accumulates in its own register tile so the large terms see one rounding per
//            k as in an fmaf chain: fp32-grade results at 16/6 = 2.67x the f32 MFMA rate;
//   SPL = 3  split3 (opt-in) — planes (h, m), products h.h | h.m, m.h: |error| <= ~2^-16
//            |a.b| (finer than TF32's 2^-11), 5.3x the f32 MFMA rate.
// Split tiles use the 16-bit kernel's LDS images (conv_gemm16.hip): k-contiguous operands
// (FWD A/B, DGRAD A) as row images [rows][BKT+8] read with one ds_read_b128 per fragment,
// k-strided operands (DGRAD B, WGRAD A/B) as col images [BKT][rows+32] read with two
// ds_read_b64_tr_b16.  The accumulator layout of the two MFMA shapes is the same, so the
// epilogues are shared.
#include <stdlib.h>
#include <string.h>

#include "conv_common.h"

namespace mauv {

constexpr int BK = 16;  // host-side alignment granule (both tile depths are multiples)
constexpr int PAD = 4;

// ROW: operands that are k-contiguous in HBM (FWD A and B, DGRAD A) are staged as row images
// [rows][BKT+4] with one ds_write_b128 per float4, and each lane reads its whole k-slice of a
// tile with ds_read_b128s up front (k order permuted: instruction kk of lane half lh takes
// k = (BKT/2)*lh + kk, the same for A and B); k-strided operands keep the k-major image
// [BKT][rows+4] read with one ds_read_b32 per MFMA.
// split tiles: 2 accumulator sets (128 AGPRs at 128x128) — held to <= 256 registers so two
// blocks (2 waves per SIMD) share a CU, as their LDS (<= 72 KB per block) allows
template <int MODE, int BM, int BN, int BKT, bool VA, bool VB, bool ROW, int SPL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SPL == 6 || SPL == 3 ? 2 : 1)))
void conv_gemm_f32(const ConvArgs a) {
  constexpr int KQ = BKT / 4;  // float4 per k-row of a k-contiguous tile row
  constexpr int WM = BM / 2, WN = BN / 2, MI = WM / 32, NI = WN / 32;
  constexpr int NVA = BM * BKT / 4 / 256, NVB = BN * BKT / 4 / 256;
  constexpr bool RA = ROW && (MODE != WGRAD), RB = ROW && (MODE == FWD);
  constexpr int RLDF = BKT + 4;
  constexpr int A_SZ = RA ? BM * RLDF : BKT * (BM + PAD);
  constexpr int B_SZ = RB ? BN * RLDF : BKT * (BN + PAD);
  // SPL > 0: NPL bf16 planes per operand (sizes in 16-bit words)
  constexpr int NPL = SPL == 3 ? 2 : 3;
  constexpr bool SA_COL = (MODE == WGRAD), SB_COL = (MODE != FWD);
  constexpr int SRLD = BKT + 8;
  constexpr int SA_PL = SA_COL ? BKT * (BM + 32) : BM * SRLD;
  constexpr int SB_PL = SB_COL ? BKT * (BN + 32) : BN * SRLD;
  constexpr int S_STG = NPL * (SA_PL + SB_PL);
  constexpr int STG_F = SPL ? S_STG / 2 : A_SZ + B_SZ;  // floats per pipeline stage
  static_assert(2 * STG_F >= 4 * BN, "epilogue reduction scratch exceeds LDS");
  __shared__ __attribute__((aligned(16))) float smem[2 * STG_F];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
  // XCD-aware tile order (1-D grid over tiles): blocks are dealt round-robin to the 8 XCDs,
  // so consecutive logical tiles are remapped onto one XCD (bijective for any grid size);
  // logical tiles run n-fastest, so the N/BN blocks that share an A (activation) tile sit on
  // the same XCD at the same time and hit its L2.
  int m0, n0;
  {
    const int nN = (a.N + BN - 1) / BN;
    const int b = blockIdx.x, nwg = gridDim.x, xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
    m0 = (L / nN) * BM;
    n0 = (L - (L / nN) * nN) * BN;
  }
  int g, sp = 0;
  if constexpr (MODE == WGRAD) { g = blockIdx.y / a.splits; sp = blockIdx.y % a.splits; }
  else g = blockIdx.y;
  int kbeg = 0, kend = a.K;
  if constexpr (MODE == WGRAD) { kbeg = sp * a.kchunk; kend = min(a.K, kbeg + a.kchunk); }

  // ---------------- per-thread loader state ----------------
  // A (FWD/DGRAD: k-contiguous rows; WGRAD: row-contiguous, rows = Cout)
  long long a_off[NVA];
  int a_p0[NVA], a_p1[NVA];
  bool a_ok[NVA];
  // B (FWD: k-contiguous rows = Cout; DGRAD: rows = Cin contiguous; WGRAD: rows=(r,s,c))
  int b_r[NVB], b_s[NVB], b_c[NVB];
  bool b_ok[NVB];
  const float* xg = a.x + (long long)g * a.xs_g;
  const float* dyg = a.dy + (long long)g * ((long long)a.B * a.Ho * a.Wo * a.Cout);
  const float* wg = a.w + (long long)g * a.ws_g;

#pragma unroll
  for (int j = 0; j < NVA; ++j) {
    const int idx = tid + 256 * j;
    if constexpr (MODE == FWD || MODE == DGRAD) {
      const int m = m0 + idx / KQ;
      a_ok[j] = m < a.M;
      const int mm = a_ok[j] ? m : 0;
      const int HW = (MODE == FWD) ? a.Ho * a.Wo : a.Hc * a.Wc;
      const int WW = (MODE == FWD) ? a.Wo : a.Wc;
      const int b = mm / HW, rem = mm - b * HW, oh = rem / WW, ow = rem - oh * WW;
      if constexpr (MODE == FWD) {
        a_off[j] = (long long)b * a.xs_b;
        a_p0[j] = oh * a.stride - a.pad;
        a_p1[j] = ow * a.stride - a.pad;
      } else {  // (oh, ow) = class-local (i, j); ih = stride*i + ph
        a_off[j] = (long long)b * a.Ho * a.Wo * a.Cout;
        a_p0[j] = oh * a.stride + a.ph + a.pad;  // ih + pad
        a_p1[j] = ow * a.stride + a.pw + a.pad;
      }
    } else {  // WGRAD: row4 fixed
      const int row = m0 + 4 * (idx % (BM / 4));
      a_p0[j] = row;
      a_p1[j] = idx / (BM / 4);  // k offset within tile
      a_ok[j] = true;
      a_off[j] = 0;
    }
  }
#pragma unroll
  for (int j = 0; j < NVB; ++j) {
    const int idx = tid + 256 * j;
    if constexpr (MODE == FWD) {
      const int n = n0 + idx / KQ;
      b_ok[j] = n < a.N;
      b_r[j] = n;
    } else if constexpr (MODE == DGRAD) {
      b_c[j] = n0 + 4 * (idx % (BN / 4));
      b_r[j] = idx / (BN / 4);
      b_ok[j] = true;
    } else {  // WGRAD: col=(r,s,c) of 4 consecutive columns
      const int col = n0 + 4 * (idx % (BN / 4));
      b_ok[j] = col < a.N;
      const int cc = b_ok[j] ? col : 0;
      const int rs = cc / a.Cin;
      b_c[j] = cc - rs * a.Cin;
      b_r[j] = rs / a.S;
      b_s[j] = rs - b_r[j] * a.S;
    }
  }

  floatx4 ra[NVA], rb[NVB];
  floatx4 bsc[NVB], bsh[NVB];  // WGRAD: per-thread channel transform (fixed columns)
  // tile-uniform tap counters: FWD (r, s, c0), DGRAD (tr, ts, n0) — advanced by load_b
  int t_r = 0, t_s = 0, t_c = 0;
  // WGRAD B: (b, oh, ow) of each loader row's pixel, advanced by BKT per tile
  int px_b[NVB], px_h[NVB], px_w[NVB];
  if constexpr (MODE == WGRAD) {
#pragma unroll
    for (int j = 0; j < NVB; ++j) {
      const int p = kbeg + (tid + 256 * j) / (BN / 4);
      const int HW = a.Ho * a.Wo;
      px_b[j] = p / HW;
      const int rem = p - px_b[j] * HW;
      px_h[j] = rem / a.Wo;
      px_w[j] = rem - px_h[j] * a.Wo;
    }
  }
  if constexpr (MODE == WGRAD && VB) {
#pragma unroll
    for (int j = 0; j < NVB; ++j) {
      if (a.xsc && b_ok[j]) {
        bsc[j] = *(const floatx4*)(a.xsc + g * a.Cin + b_c[j]);
        bsh[j] = *(const floatx4*)(a.xsh + g * a.Cin + b_c[j]);
      }
    }
  }

  auto load_a = [&](int k0) {
#pragma unroll
    for (int j = 0; j < NVA; ++j) {
      const int idx = tid + 256 * j;
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if constexpr (MODE == FWD) {
        const int kq = idx % KQ;
        if constexpr (VA) {  // Cin % 32 == 0: the tile's k slice is one (r, s) tap
          const int r = t_r, s = t_s, c = t_c + 4 * kq;
          const int ih = a_p0[j] + r, iw = a_p1[j] + s;
          if (a_ok[j] && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) {
            v = *(const floatx4*)(xg + a_off[j] + (long long)ih * a.xs_h + (long long)iw * a.xs_w + c);
            if (a.xsc)
              v = bn_act(v, *(const floatx4*)(a.xsc + g * a.Cin + c),
                         *(const floatx4*)(a.xsh + g * a.Cin + c), a.xrelu);
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int k = k0 + 4 * kq + e;
            if (a_ok[j] && k < kend) {
              const int rs = k / a.Cin, c = k - rs * a.Cin, r = rs / a.S, s = rs - r * a.S;
              const int ih = a_p0[j] + r, iw = a_p1[j] + s;
              if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
                v[e] = xg[a_off[j] + (long long)ih * a.xs_h + (long long)iw * a.xs_w +
                          (long long)c * a.xs_c];
            }
          }
        }
      } else if constexpr (MODE == DGRAD) {
        const int kq = idx % KQ;
        // k = (tap t = (tr, ts), n); tap (tr, ts) -> (r0 + stride*tr, s0 + stride*ts), so
        // ih + pad - r is a multiple of the stride by construction
        if constexpr (VA) {  // Cout % 32 == 0: the tile's k slice is one tap (tr, ts)
          const int n = t_c + 4 * kq, tr = t_r, ts = t_s;
          const int ohn = a_p0[j] - a.r0 - a.stride * tr, own = a_p1[j] - a.s0 - a.stride * ts;
          if (a_ok[j] && ohn >= 0 && own >= 0) {
            const int oh = a.stride == 1 ? ohn : ohn / a.stride;
            const int ow = a.stride == 1 ? own : own / a.stride;
            if (oh < a.Ho && ow < a.Wo)
              v = *(const floatx4*)(dyg + a_off[j] + ((long long)oh * a.Wo + ow) * a.Cout + n);
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int k = k0 + 4 * kq + e;
            if (a_ok[j] && k < kend) {
              const int t = k / a.Cout, n = k - t * a.Cout, tr = t / a.ns, ts = t - tr * a.ns;
              const int ohn = a_p0[j] - a.r0 - a.stride * tr;
              const int own = a_p1[j] - a.s0 - a.stride * ts;
              if (ohn >= 0 && own >= 0) {
                const int oh = ohn / a.stride, ow = own / a.stride;
                if (oh < a.Ho && ow < a.Wo)
                  v[e] = dyg[a_off[j] + ((long long)oh * a.Wo + ow) * a.Cout + n];
              }
            }
          }
        }
      } else {  // WGRAD A: dy^T, rows = cout, k = pixel
        const int p = k0 + a_p1[j], co = a_p0[j];
        if (p < kend) {
          const float* src = dyg + (long long)p * a.Cout;
          if constexpr (VA) {
            if (co < a.Cout) v = *(const floatx4*)(src + co);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (co + e < a.Cout) v[e] = src[co + e];
          }
        }
      }
      ra[j] = v;
    }
  };

  auto load_b = [&](int k0) {
#pragma unroll
    for (int j = 0; j < NVB; ++j) {
      const int idx = tid + 256 * j;
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
      if constexpr (MODE == FWD) {
        const int kq = idx % KQ;
        const int k = k0 + 4 * kq;
        const float* src = wg + (long long)b_r[j] * a.K;
        if constexpr (VB) {
          if (b_ok[j] && k < kend) v = *(const floatx4*)(src + k);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (b_ok[j] && k + e < kend) v[e] = src[k + e];
        }
      } else if constexpr (MODE == DGRAD) {
        const int k = k0 + b_r[j];
        const int c = b_c[j];
        if (k < kend) {
          int n, tr, ts;
          if constexpr (VA) {  // tile-uniform tap (Cout % 32 == 0)
            n = t_c + b_r[j]; tr = t_r; ts = t_s;
          } else {
            const int t = k / a.Cout;
            n = k - t * a.Cout; tr = t / a.ns; ts = t - tr * a.ns;
          }
          const int r = a.r0 + a.stride * tr, s = a.s0 + a.stride * ts;
          const float* src = wg + (((long long)n * a.R + r) * a.S + s) * a.Cin;
          if constexpr (VB) {
            if (c < a.N) v = *(const floatx4*)(src + c);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (c + e < a.N) v[e] = src[c + e];
          }
        }
      } else {  // WGRAD B: im2col(x), rows=(r,s,c), k = pixel
        const int p = k0 + (idx / (BN / 4));
        if (p < kend && b_ok[j]) {
          const int b = px_b[j], oh = px_h[j], ow = px_w[j];
          if constexpr (VB) {
            const int ih = oh * a.stride - a.pad + b_r[j], iw = ow * a.stride - a.pad + b_s[j];
            if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) {
              v = *(const floatx4*)(xg + (long long)b * a.xs_b + (long long)ih * a.xs_h +
                                    (long long)iw * a.xs_w + b_c[j]);
              if (a.xsc) v = bn_act(v, bsc[j], bsh[j], a.xrelu);
            }
          } else {
            const int col0 = n0 + 4 * (idx % (BN / 4));
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int col = col0 + e;
              if (col < a.N) {
                const int rs = col / a.Cin, c = col - rs * a.Cin, r = rs / a.S, s = rs - r * a.S;
                const int ih = oh * a.stride - a.pad + r, iw = ow * a.stride - a.pad + s;
                if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
                  v[e] = xg[(long long)b * a.xs_b + (long long)ih * a.xs_h +
                            (long long)iw * a.xs_w + (long long)c * a.xs_c];
              }
            }
          }
        }
      }
      rb[j] = v;
      if constexpr (MODE == WGRAD) {  // advance this row's pixel by one tile
        px_w[j] += BKT;
        while (px_w[j] >= a.Wo) { px_w[j] -= a.Wo; ++px_h[j]; }
        while (px_h[j] >= a.Ho) { px_h[j] -= a.Ho; ++px_b[j]; }
      }
    }
    // advance the tile-uniform tap counters (FWD / DGRAD vector paths)
    if constexpr (MODE == FWD && VA) {
      t_c += BKT;
      if (t_c >= a.Cin) { t_c = 0; if (++t_s == a.S) { t_s = 0; ++t_r; } }
    } else if constexpr (MODE == DGRAD && VA) {
      t_c += BKT;
      if (t_c >= a.Cout) { t_c = 0; if (++t_s == a.ns) { t_s = 0; ++t_r; } }
    }
  };

  auto store_tiles = [&](int buf) {
    if constexpr (SPL != 0) {  // split planes (h16.h split_bf16) into the 16-bit images
      u16* As = (u16*)smem + buf * S_STG;
      u16* Bs = As + NPL * SA_PL;
#pragma unroll
      for (int j = 0; j < NVA; ++j) {
        const int idx = tid + 256 * j;
        const int off = SA_COL ? (idx / (BM / 4)) * (BM + 32) + 4 * (idx % (BM / 4))
                               : (idx / KQ) * SRLD + 4 * (idx % KQ);
        uint2 pl[3];
        split_bf16<NPL>(ra[j], pl);
#pragma unroll
        for (int p = 0; p < NPL; ++p) *(uint2*)(As + p * SA_PL + off) = pl[p];
      }
#pragma unroll
      for (int j = 0; j < NVB; ++j) {
        const int idx = tid + 256 * j;
        const int off = SB_COL ? (idx / (BN / 4)) * (BN + 32) + 4 * (idx % (BN / 4))
                               : (idx / KQ) * SRLD + 4 * (idx % KQ);
        uint2 pl[3];
        split_bf16<NPL>(rb[j], pl);
#pragma unroll
        for (int p = 0; p < NPL; ++p) *(uint2*)(Bs + p * SB_PL + off) = pl[p];
      }
      return;
    }
    float* Ab = smem + buf * (A_SZ + B_SZ);
    float* Bb = Ab + A_SZ;
#pragma unroll
    for (int j = 0; j < NVA; ++j) {
      const int idx = tid + 256 * j;
      if constexpr (MODE == WGRAD) {
        const int kr = idx / (BM / 4), r4 = idx % (BM / 4);
        *(floatx4*)(Ab + kr * (BM + PAD) + 4 * r4) = ra[j];
      } else if constexpr (RA) {
        const int row = idx / KQ, kq = idx % KQ;
        *(floatx4*)(Ab + row * RLDF + 4 * kq) = ra[j];
      } else {
        const int row = idx / KQ, kq = idx % KQ;
#pragma unroll
        for (int e = 0; e < 4; ++e) Ab[(4 * kq + e) * (BM + PAD) + row] = ra[j][e];
      }
    }
#pragma unroll
    for (int j = 0; j < NVB; ++j) {
      const int idx = tid + 256 * j;
      if constexpr (MODE == FWD) {
        const int row = idx / KQ, kq = idx % KQ;
        if constexpr (RB) {
          *(floatx4*)(Bb + row * RLDF + 4 * kq) = rb[j];
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) Bb[(4 * kq + e) * (BN + PAD) + row] = rb[j][e];
        }
      } else {
        const int kr = idx / (BN / 4), r4 = idx % (BN / 4);
        *(floatx4*)(Bb + kr * (BN + PAD) + 4 * r4) = rb[j];
      }
    }
  };

  floatx16 acc[MI][NI], acl[MI][NI];  // acl: the split modes' small plane products
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) { acc[mi][ni][r] = 0.f; acl[mi][ni][r] = 0.f; }

  const int ntiles = (kend - kbeg + BKT - 1) / BKT;
  if (ntiles > 0) {
    load_a(kbeg);
    load_b(kbeg);
    store_tiles(0);
  }
  __syncthreads();
  int cur = 0;
  for (int t = 0; t < ntiles; ++t) {
    const bool more = t + 1 < ntiles;
    if (more) {
      load_a(kbeg + (t + 1) * BKT);
      load_b(kbeg + (t + 1) * BKT);
    }
    const float* Ab = smem + cur * (A_SZ + B_SZ);
    const float* Bb = Ab + A_SZ;
    if constexpr (SPL != 0) {
      const u16* As = (const u16*)smem + cur * S_STG;
      const u16* Bs = As + NPL * SA_PL;
#pragma unroll
      for (int s = 0; s < BKT / 16; ++s) {
        u32x4 af[NPL][MI], bq[NPL][NI];
#pragma unroll
        for (int p = 0; p < NPL; ++p) {
#pragma unroll
          for (int mi = 0; mi < MI; ++mi) {
            if constexpr (SA_COL)
              af[p][mi] = col_frag(As + p * SA_PL, BM + 32, wm * WM + mi * 32, s, lane);
            else
              af[p][mi] = row_frag_ld<SRLD>(As + p * SA_PL, wm * WM + mi * 32, s, li, lh);
          }
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) {
            if constexpr (SB_COL)
              bq[p][ni] = col_frag(Bs + p * SB_PL, BN + 32, wn * WN + ni * 32, s, lane);
            else
              bq[p][ni] = row_frag_ld<SRLD>(Bs + p * SB_PL, wn * WN + ni * 32, s, li, lh);
          }
        }
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) {
            if constexpr (SPL == 5) {  // one accumulator for all six products
              floatx16 c = acc[mi][ni];
              c = H16<DT_BF16>::mfma(af[0][mi], bq[2][ni], c);
              c = H16<DT_BF16>::mfma(af[2][mi], bq[0][ni], c);
              c = H16<DT_BF16>::mfma(af[1][mi], bq[1][ni], c);
              c = H16<DT_BF16>::mfma(af[0][mi], bq[1][ni], c);
              c = H16<DT_BF16>::mfma(af[1][mi], bq[0][ni], c);
              acc[mi][ni] = H16<DT_BF16>::mfma(af[0][mi], bq[0][ni], c);
              continue;
            }
            floatx16 c = acl[mi][ni];
            if constexpr (SPL == 6) {
              c = H16<DT_BF16>::mfma(af[0][mi], bq[2][ni], c);
              c = H16<DT_BF16>::mfma(af[2][mi], bq[0][ni], c);
              c = H16<DT_BF16>::mfma(af[1][mi], bq[1][ni], c);
            }
            c = H16<DT_BF16>::mfma(af[0][mi], bq[1][ni], c);
            acl[mi][ni] = H16<DT_BF16>::mfma(af[1][mi], bq[0][ni], c);
            acc[mi][ni] = H16<DT_BF16>::mfma(af[0][mi], bq[0][ni], acc[mi][ni]);
          }
      }
    } else if constexpr (RA || RB) {
      constexpr int KH = BKT / 2;
      float a8[MI][KH], b8[NI][KH];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        if constexpr (RA) {
#pragma unroll
          for (int q = 0; q < KH / 4; ++q) {
            const floatx4 v = *(const floatx4*)(Ab + (wm * WM + mi * 32 + li) * RLDF + KH * lh + 4 * q);
#pragma unroll
            for (int e = 0; e < 4; ++e) a8[mi][4 * q + e] = v[e];
          }
        } else {
#pragma unroll
          for (int kk = 0; kk < KH; ++kk)
            a8[mi][kk] = Ab[(KH * lh + kk) * (BM + PAD) + wm * WM + mi * 32 + li];
        }
      }
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        if constexpr (RB) {
#pragma unroll
          for (int q = 0; q < KH / 4; ++q) {
            const floatx4 v = *(const floatx4*)(Bb + (wn * WN + ni * 32 + li) * RLDF + KH * lh + 4 * q);
#pragma unroll
            for (int e = 0; e < 4; ++e) b8[ni][4 * q + e] = v[e];
          }
        } else {
#pragma unroll
          for (int kk = 0; kk < KH; ++kk)
            b8[ni][kk] = Bb[(KH * lh + kk) * (BN + PAD) + wn * WN + ni * 32 + li];
        }
      }
#pragma unroll
      for (int kk = 0; kk < KH; ++kk)
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a8[mi][kk], b8[ni][kk], acc[mi][ni], 0, 0, 0);
    } else {
#pragma unroll
      for (int kk = 0; kk < BKT / 2; ++kk) {
        float av[MI], bv[NI];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) av[mi] = Ab[(2 * kk + lh) * (BM + PAD) + wm * WM + mi * 32 + li];
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) bv[ni] = Bb[(2 * kk + lh) * (BN + PAD) + wn * WN + ni * 32 + li];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mi], bv[ni], acc[mi][ni], 0, 0, 0);
      }
    }
    if (more) store_tiles(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // ---------------- epilogue ----------------
  if constexpr (SPL == 6 || SPL == 3) {
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) acc[mi][ni] += acl[mi][ni];
  }
  conv_epilogue<MODE, BM, BN>(a, acc, smem, tid, m0, n0, g, sp);
}

// exact mode: DGRAD uses row images + b128 operand reads (measured on the bench workload:
// DGRAD +3.5 %, FWD -2 %); a 32-deep tile measured slower (2 vs 3 blocks per CU) and was removed

// fp32 product arithmetic (file header): 6 = split (default), 5 = split1, 3 = split3, 0 = exact
// (MauvRoute.f32_math; initial value from MAUV_F32_MATH, capi.cpp)
static int f32_math() { return g_route.f32_math; }

template <int MODE, int BM, int BN, bool VA, bool VB>
static void launch(const ConvArgs& a, hipStream_t st) {
  dim3 grid(ceil_div(a.M, BM) * ceil_div(a.N, BN), MODE == WGRAD ? a.G * a.splits : a.G);
  const int fm = f32_math();
  if (fm == 6) {
    hipLaunchKernelGGL((conv_gemm_f32<MODE, BM, BN, 16, VA, VB, false, 6>), grid, dim3(256), 0, st, a);
  } else if (fm == 5) {
    hipLaunchKernelGGL((conv_gemm_f32<MODE, BM, BN, 16, VA, VB, false, 5>), grid, dim3(256), 0, st, a);
  } else if (fm == 3) {
    hipLaunchKernelGGL((conv_gemm_f32<MODE, BM, BN, 16, VA, VB, false, 3>), grid, dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL((conv_gemm_f32<MODE, BM, BN, 16, VA, VB, MODE == DGRAD, 0>), grid, dim3(256), 0, st, a);
  }
}

template <int MODE, bool VA, bool VB>
static void launch_tiles(const ConvArgs& a, hipStream_t st) {
  // measured: halving the row tile for launches with fewer blocks than resident slots does
  // not pay (co-resident blocks share the MFMA pipes, so a partial last wave runs faster)
  const int bm = conv_tile_rows(a.M), bn = conv_tile_rows(a.N);
  if (bm == 64 && bn == 64) launch<MODE, 64, 64, VA, VB>(a, st);
  else if (bm == 64) launch<MODE, 64, 128, VA, VB>(a, st);
  else if (bn == 64) launch<MODE, 128, 64, VA, VB>(a, st);
  else launch<MODE, 128, 128, VA, VB>(a, st);
}

}  // namespace mauv

using namespace mauv;

// m-tiles of a launch (BM = conv_tile_rows(M)), = per-m-tile BN statistic partials
static int stat_blocks(int M, int N, int G) { return ceil_div(M, conv_tile_rows(M)); }
static int dgrad_stat_blocks(int G, int B, int H, int W, int N, int stride) {
  int n = 0;
  for (int ph = 0; ph < stride; ++ph)
    for (int pw = 0; pw < stride; ++pw) {
      const int M = B * ((H - ph + stride - 1) / stride) * ((W - pw + stride - 1) / stride);
      if (M > 0) n += stat_blocks(M, N, G);
    }
  return n;
}

static ConvArgs make_args(int G, int B, int H, int W, int Cin, int Cout, int R, int S,
                          int stride, int pad, const long long* xs) {
  ConvArgs a{};
  a.G = G; a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.R = R; a.S = S;
  a.stride = stride; a.pad = pad;
  a.Ho = (H + 2 * pad - R) / stride + 1;
  a.Wo = (W + 2 * pad - S) / stride + 1;
  if (xs) { a.xs_g = xs[0]; a.xs_b = xs[1]; a.xs_h = xs[2]; a.xs_w = xs[3]; a.xs_c = xs[4]; }
  else {
    a.xs_c = 1; a.xs_w = Cin; a.xs_h = (long long)W * Cin; a.xs_b = (long long)H * W * Cin;
    a.xs_g = (long long)B * H * W * Cin;
  }
  a.ws_g = (long long)Cout * R * S * Cin;
  a.splits = 1;
  return a;
}

// Forward: y[g] = conv(x[g], W_g) (+ bias[g]) — NHWC, fp32.
// x_strides (nullable): element strides {group, batch, h, w, c} of x; NULL = dense NHWC.
// Replaces F.conv2d in bayesian-torch Conv2dReparameterization.forward / F.linear in
// LinearReparameterization.forward (a linear is the 1x1 case with H=W=1).
MAUV_API int mauv_conv2d_fwd_f32(const float* x, const long long* x_strides,
                                 const float* x_scale, const float* x_shift, int x_relu,
                                 const float* w, const float* bias, float* y, int G, int B,
                                 int H, int W, int Cin, int Cout, int R, int S, int stride,
                                 int pad, float* st_mean, float* st_m2, float* st_cnt,
                                 hipStream_t stream) {
  if (G <= 0 || B <= 0 || Cin <= 0 || Cout <= 0) { set_error("conv2d_fwd: bad shape"); return kErrArg; }
  ConvArgs a = make_args(G, B, H, W, Cin, Cout, R, S, stride, pad, x_strides);
  a.x = x; a.w = w; a.out = y; a.bias = bias; a.bias_sg = Cout;
  a.xsc = x_scale; a.xsh = x_shift; a.xrelu = x_relu;
  a.M = B * a.Ho * a.Wo; a.N = Cout; a.K = R * S * Cin;
  a.out_sg = (long long)a.M * a.N;
  a.st_mean = st_mean; a.st_m2 = st_m2; a.st_cnt = st_cnt;
  a.st_nblk = stat_blocks(a.M, a.N, G); a.st_base = 0;
  const bool va = (Cin % 32 == 0) && a.xs_c == 1 && (a.xs_w % 4 == 0) && (a.xs_h % 4 == 0) &&
                  (a.xs_b % 4 == 0) && (a.xs_g % 4 == 0);
  const bool vb = (a.K % 4 == 0);
  if (x_scale && !(va && vb)) { set_error("conv2d_fwd: x transform needs the vector path"); return kErrArg; }
  const int fm = f32_math();
  if ((fm == 6 || fm == 5) && conv_split_launch(FWD, a, fm == 5, stream)) return check_launch("conv2d_fwd");
  if (va && vb) launch_tiles<FWD, true, true>(a, stream);
  else if (vb) launch_tiles<FWD, false, true>(a, stream);
  else launch_tiles<FWD, false, false>(a, stream);
  return check_launch("conv2d_fwd");
}

// The stems as ONE GEMM over im2col rows shared by the G MC samples (stem.hip):
// y[g][m][c] = sum_k cols[m][k] * w[g][c][k] with the G weight sets stacked along N
// (N = G * Cout, ConvArgs::cpg = Cout): every row of the images is read once for all samples.
MAUV_API int mauv_stem_fwd_f32(const float* cols, const float* w, float* y, int G, int M,
                               int Kp, int Cout, float* st_mean, float* st_m2, float* st_cnt,
                               hipStream_t stream) {
  if (G <= 0 || M <= 0 || Kp <= 0 || Cout <= 0 || Kp % 4) { set_error("stem_fwd_f32: bad shape"); return kErrArg; }
  ConvArgs a = make_args(1, 1, 1, M, Kp, G * Cout, 1, 1, 1, 0, nullptr);
  a.x = cols; a.w = w; a.out = y;
  a.M = M; a.N = G * Cout; a.K = Kp;
  a.out_sg = (long long)M * Cout;
  a.cpg = Cout;
  a.st_mean = st_mean; a.st_m2 = st_m2; a.st_cnt = st_cnt;
  a.st_nblk = stat_blocks(M, Cout, G); a.st_base = 0;
  const int fm = f32_math();
  if (fm == 6 || fm == 5) {
    // the split kernel reads cols by a buffer descriptor (31-bit byte offsets): more rows
    // (configs[4]'s 512 px sonar at B = 256) go in chunks of whole 128-row tiles, each writing
    // its rows of y and its statistics blocks (st_base)
    const long long lim_rows = (0x7fff0000LL / 4 / Kp) / 128 * 128;
    bool ok = true;
    for (long long r0 = 0; r0 < M && ok; r0 += lim_rows) {
      ConvArgs c = a;
      c.M = (int)(M - r0 < lim_rows ? M - r0 : lim_rows);
      c.W = c.Wo = c.M;                        // cols as one 1 x M image of Kp channels
      c.xs_h = c.xs_b = (long long)c.M * Kp;
      c.x = cols + r0 * Kp;
      c.out = y + r0 * Cout;
      c.st_base = (int)(r0 / 128);
      ok = conv_split_launch(FWD, c, fm == 5, stream);
      if (!ok && r0 > 0) { set_error("stem_fwd_f32: chunk outside the split kernel"); return kErrArg; }
    }
    if (ok) return check_launch("stem_fwd_f32");
  }
  if (Kp % 32 == 0) launch_tiles<FWD, true, true>(a, stream);
  else launch_tiles<FWD, false, true>(a, stream);
  return check_launch("stem_fwd_f32");
}

// Data gradient: dx[g] = conv_transpose(dy[g], W_g) (+ addend) (+ dx if accumulate).
MAUV_API int mauv_conv2d_bwd_data_f32(const float* dy, const float* w, float* dx,
                                      const float* addend, const unsigned char* addend_mask,
                                      int accumulate, int G, int B, int H,
                                      int W, int Cin, int Cout, int R, int S, int stride,
                                      int pad, const float* bn_y, const float* bn_out,
                                      const unsigned char* bn_mask,
                                      const float* bn_scale, const float* bn_shift,
                                      const float* bn_mean, const float* bn_invstd, int bn_relu,
                                      float* bn_p1, float* bn_p2, hipStream_t stream) {
  ConvArgs a = make_args(G, B, H, W, Cin, Cout, R, S, stride, pad, nullptr);
  a.dy = dy; a.w = w; a.out = dx; a.addend = addend; a.accumulate = accumulate;
  a.add_mask = addend ? addend_mask : nullptr;
  a.N = Cin;
  a.out_sg = (long long)B * H * W * Cin;
  a.bp_y = bn_y; a.bp_out = bn_out; a.bp_mask = bn_mask; a.bp_sc = bn_scale; a.bp_sh = bn_shift;
  a.bp_mean = bn_mean; a.bp_invstd = bn_invstd; a.bp_relu = bn_relu;
  a.bp_p1 = bn_p1; a.bp_p2 = bn_p2;
  a.bp_nblk = dgrad_stat_blocks(G, B, H, W, Cin, stride);
  a.bp_base = 0;
  if (bn_p1 && bn_relu && !bn_out && !bn_mask && !bn_shift) { set_error("conv2d_bwd_data: mask source"); return kErrArg; }
  const bool va = (Cout % 32 == 0), vb = (Cin % 4 == 0);
  // one launch per output-parity class (stride^2 of them; 1 for stride 1)
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
      a.K = a.nr * a.ns * Cout;  // 0 -> the class only receives the addend / zeros
      if (a.M <= 0) continue;
      // a tapless class accumulating into dx adds nothing (stride-2 1x1 downsample: 3 of 4)
      if (a.K == 0 && accumulate && !addend && !bn_p1) continue;
      const int fm = f32_math();
      if ((fm == 6 || fm == 5) && conv_split_launch(DGRAD, a, fm == 5, stream)) {}
      else if (va && vb) launch_tiles<DGRAD, true, true>(a, stream);
      else if (vb) launch_tiles<DGRAD, false, true>(a, stream);
      else launch_tiles<DGRAD, false, false>(a, stream);
      a.bp_base += stat_blocks(a.M, a.N, G);
    }
  return check_launch("conv2d_bwd_data");
}


// Number of per-m-tile BN statistic partials the fused epilogues write (host sizing helpers).
MAUV_API int mauv_conv2d_fwd_stat_blocks(int G, int B, int H, int W, int Cin, int Cout, int R,
                                         int S, int stride, int pad) {
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  return stat_blocks(B * Ho * Wo, Cout, G);
}
MAUV_API int mauv_conv2d_bwd_data_stat_blocks(int G, int B, int H, int W, int Cin, int Cout,
                                              int R, int S, int stride, int pad) {
  return dgrad_stat_blocks(G, B, H, W, Cin, stride);
}

// Split count used by mauv_conv2d_bwd_weight for a given problem (host helper so the caller
// can size the partial-slab workspace: splits * G * Cout * R*S*Cin floats).
MAUV_API int mauv_conv2d_wgrad_splits(int G, int B, int H, int W, int Cin, int Cout, int R,
                                      int S, int stride, int pad) {
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  const long long P = (long long)B * Ho * Wo;
  const int N = R * S * Cin;
  const long long tiles = (long long)ceil_div(Cout, Cout <= 64 ? 64 : 128) *
                          ceil_div(N, N <= 64 ? 64 : 128) * G;
  // keep >= 256 pixels per split; at most 256 splits
  long long maxs = (P + 255) / 256;
  if (maxs > 256) maxs = 256;
  if (maxs < 1) maxs = 1;
  // The weight-gradient kernels run two blocks per CU: 512 resident blocks on the 256 CUs.  The
  // round-1 rule (the fewest splits giving >= 1024 blocks) landed every trunk launch at
  // 1025-1440 blocks, i.e. a third block round holding 0.2-40 % of a round.  Take, among the
  // split counts giving one to three rounds (>= one full round where the pixels allow it), the
  // fewest splits whose last round is filled within 5 % of the best fill (fewer splits: fewer
  // fp32 slab bytes).  MAUV_WGRAD_SPLITS=0 restores the round-1 rule.
  static int mode = -1;
  if (mode < 0) { const char* e = getenv("MAUV_WGRAD_SPLITS"); mode = e ? atoi(e) : 2; }
  if (mode == 0) {
    long long splits = (1024 + tiles - 1) / tiles;
    if (splits > maxs) splits = maxs;
    return (int)(splits < 1 ? 1 : splits);
  }
  if (mode == 2) {
    // Every split writes a full fp32 slab of its tiles that mauv_reparam_bwd reads back: at the
    // layer-3/4 shapes the fill rule below chose 19 splits (1520 blocks, 11 GB of slabs per bf16
    // step).  Price both: block rounds x the per-block MFMA time of its pixel chunk, plus the
    // slab bytes (written and read back) at HBM rate, and take the cheapest split count.
    const double tile_m = Cout <= 64 ? 64.0 : 128.0, tile_n = N <= 64 ? 64.0 : 128.0;
    const double blk_flops = 480e12 / 512.0;       // sustained 16-bit MFMA rate per resident block
    const double hbm = 5.0e12;                     // bytes/s a streaming pass sustains
    const double ovh = 2.0e-6;                     // per-block prologue / epilogue (s)
    long long best = 1;
    double tbest = 1e30;
    for (long long s = 1; s <= maxs; ++s) {
      const long long nb = tiles * s, rounds = (nb + 511) / 512;
      const long long kch = ((P + s - 1) / s + 31) / 32 * 32;
      const double t = (double)rounds * ((double)kch * 2.0 * tile_m * tile_n / blk_flops + ovh) +
                       (double)nb * tile_m * tile_n * 4.0 * 2.0 / hbm;
      if (t < tbest * 0.995) { tbest = t; best = s; }
    }
    return (int)best;
  }
  const long long slots = 512;
  const long long lo = tiles * maxs < slots ? maxs : (slots + tiles - 1) / tiles;
  auto fill = [&](long long s) {
    const long long nb = tiles * s, rounds = (nb + slots - 1) / slots;
    return (double)nb / (double)(rounds * slots);
  };
  double top = 0.0;
  for (long long s = lo; s <= maxs && (s == lo || tiles * s <= 3 * slots); ++s) top = fmax(top, fill(s));
  long long best = lo;
  for (long long s = lo; s <= maxs && (s == lo || tiles * s <= 3 * slots); ++s)
    if (fill(s) >= top - 0.05) { best = s; break; }
  return (int)best;
}

// Weight gradient partial slabs: ws[split][g][Cout][R*S*Cin] (reduced by mauv_reparam_bwd).
MAUV_API int mauv_conv2d_bwd_weight_f32(const float* x, const long long* x_strides,
                                        const float* x_scale, const float* x_shift, int x_relu,
                                        const float* dy, float* ws, int splits, int G, int B,
                                        int H, int W, int Cin, int Cout, int R, int S,
                                        int stride, int pad, hipStream_t stream) {
  ConvArgs a = make_args(G, B, H, W, Cin, Cout, R, S, stride, pad, x_strides);
  a.x = x; a.dy = dy; a.out = ws;
  a.xsc = x_scale; a.xsh = x_shift; a.xrelu = x_relu;
  a.M = Cout; a.N = R * S * Cin; a.K = B * a.Ho * a.Wo;
  a.splits = splits;
  a.kchunk = ((a.K + splits - 1) / splits + 31) / 32 * 32;  // multiple of both tile depths
  const bool va = (Cout % 4 == 0);
  const bool vb = (Cin % 4 == 0) && a.xs_c == 1 && (a.xs_w % 4 == 0) && (a.xs_h % 4 == 0) &&
                  (a.xs_b % 4 == 0) && (a.xs_g % 4 == 0);
  if (x_scale && !(va && vb)) { set_error("conv2d_bwd_weight: x transform needs the vector path"); return kErrArg; }
  const int fm = f32_math();
  if ((fm == 6 || fm == 5) && conv_split_launch(WGRAD, a, fm == 5, stream)) return check_launch("conv2d_bwd_weight");
  if (va && vb) launch_tiles<WGRAD, true, true>(a, stream);
  else if (va) launch_tiles<WGRAD, true, false>(a, stream);
  else launch_tiles<WGRAD, false, false>(a, stream);
  return check_launch("conv2d_bwd_weight");
}
