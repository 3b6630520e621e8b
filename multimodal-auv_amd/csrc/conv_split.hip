// Pipelined split-fp32 implicit-GEMM convolution: the default arithmetic of every fp32 conv of
// the three ResNet-50 trunks (models/base_models.py:15-18, models/model_utils.py:57-61) and of
// the fusion head's linears, forward / data gradient / weight gradient, on the vector paths
// (every conv of the path; the 1- and 3-channel stems through their STEM mode over images packed
// to 4 zero-padded NHWC channels — other channel counts fall back to conv_gemm.hip).
//
// Arithmetic (conv_gemm.hip header, include/mauv.h MauvRoute.f32_math): each fp32 operand
// element is split exactly into bf16 planes x = h + m + l and the product a.b is accumulated in
// fp32 from h.h, h.m, m.h, h.l, l.h, m.m on v_mfma_f32_32x32x16_bf16 (dropped terms <= 2^-24
// |a.b|).  With the MFMAs 2.67x cheaper than f32 MFMA, the staging becomes the bottleneck of a
// load -> wait -> split -> LDS -> barrier loop; this kernel restructures it:
//  * two tiles in flight: stage t issues the global loads of tile t+2, runs the MFMAs of tile t
//    from one LDS buffer and splits + writes tile t+1 (loaded a stage earlier) into the other —
//    one branch-free basic block per stage, so the split VALU and ds_writes interleave with the
//    MFMAs and HBM latency hides behind a whole stage;
//  * raw buffer loads: 32-bit offsets = per-thread constant + tile-uniform scalar; an offset past
//    the descriptor's range returns 0, which implements spatial padding, ragged tiles and the
//    tiles past the end of K without branches;
//  * the producing layer's pending BatchNorm(+ReLU) is applied at split time (FWD: scale/shift
//    of the input channels staged in LDS once per block; WGRAD: per-thread channel constants).
// LDS images are conv_gemm16.hip's: k-contiguous operands (FWD A/B, DGRAD A) as row images
// [rows][BK+8] (one ds_read_b128 per fragment), k-strided ones (DGRAD B, WGRAD A/B) as col images
// [BK][rows+32] (two ds_read_b64_tr_b16).  Epilogue: conv_common.h (shared with conv_gemm.hip).
#include <stdlib.h>

#include "conv_common.h"

namespace mauv {

namespace {

constexpr unsigned kOOB = 0x7ffffff0u;  // beyond every descriptor range: the load returns 0
constexpr int kMaxXbn = 512;            // FWD pending-BN input channels staged in LDS

__device__ __forceinline__ floatx4 bload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p, long long nfloats) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(nfloats * 4), 0x00020000);
}
__device__ __forceinline__ unsigned mdiv(unsigned n, unsigned long long m, int s) {
  return (unsigned)(((unsigned long long)n * m) >> s);
}
__device__ __forceinline__ floatx4 bn_relu(floatx4 v, floatx4 sc, floatx4 sh, int relu, bool ok) {
  v = v * sc + sh;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = (!ok || (relu && !(v[e] > 0.f))) ? 0.f : v[e];
  return v;
}

template <int NVA, int NVB>
struct Stage {
  floatx4 a[NVA], b[NVB];
  unsigned ok;  // validity bits (pending-BN operands): a j -> bit j, b j -> bit 8 + j
  int tc;       // FWD: input-channel offset of this stage's k slice
};

}  // namespace

// Waves: 2 x 2 for tiles up to 128 x 128 (256 threads, two blocks per CU); the launcher
// instantiates 64 x 64 with these.
// WV = 8 on a 128 x 128 tile: 4 x 2 waves of 32 x 64 (one accumulator set, <= 128 VGPRs, two
// blocks = four waves per SIMD for latency hiding)
// (128 x 64 / 64 x 128 with WV = 8: waves of 32 x 32; the 64-wide operand is then loaded by
// half the threads)
template <int BM, int BN, int WV>
struct SplitWaves {
  static constexpr bool W8 = (WV == 8 && BM <= 128 && BN <= 128 && BM + BN >= 192);
  static constexpr int M = W8 ? (BM == 128 ? 4 : 2) : (BM == 256 ? 4 : 2);
  static constexpr int N = W8 ? (BM == 128 ? 2 : 4) : (BN == 256 ? 4 : 2);
  static constexpr int T = 64 * M * N, EU = W8 ? 4 : 2;
};
// loader row of index idx for the row images: wave-local permutation so that each 16-lane
// ds_write_b64 group stores rows r, r+2, r+4, r+6 (row stride 12 dwords: conflict-free)
__device__ __forceinline__ int row_of(int idx) {
  const int l = idx & 63;
  return (idx >> 6) * 16 + 8 * (l >> 5) + 2 * ((l >> 2) & 3) + ((l >> 4) & 1);
}

// SEQ: short K (the 1x1 forwards over <= 256 channels): one register stage and one LDS buffer,
// stages one after another, a register budget for three blocks per CU instead of two (the
// 16-bit kernel's short-K variant, conv_pipe16.hip)
template <int MODE, int BM, int BN, bool XBN, bool ONEACC, int WV, bool STEM = false,
          bool SEQ = false, bool BP = false>
__global__ __launch_bounds__((SplitWaves<BM, BN, WV>::T))
__attribute__((amdgpu_waves_per_eu(SEQ && !BP ? 6 : SplitWaves<BM, BN, WV>::EU)))
void conv_split_f32(const ConvArgs a) {
  constexpr int BK = 16;
  constexpr int WGM = SplitWaves<BM, BN, WV>::M, WGN = SplitWaves<BM, BN, WV>::N;
  constexpr int NT = SplitWaves<BM, BN, WV>::T;
  constexpr int WM = BM / WGM, WN = BN / WGN, MI = WM / 32, NI = WN / 32;
  // float4 per stage per operand (LA, LB) and per thread (NVA, NVB); with LB < NT the threads
  // tid >= LB load nothing (offset past the descriptor) and park their split planes in a dummy
  // LDS slot, keeping the stage branch-free
  constexpr int LA = 4 * BM, LB = 4 * BN;
  constexpr int NVA = (LA + NT - 1) / NT, NVB = (LB + NT - 1) / NT;
  constexpr bool PA = LA % NT != 0, PB = LB % NT != 0;
  constexpr bool A_COL = (MODE == WGRAD), B_COL = (MODE != FWD);
  constexpr int RLD = BK + 8;
  constexpr int A_PL = A_COL ? BK * (BM + 32) : BM * RLD;  // 16-bit words per plane
  constexpr int B_PL = B_COL ? BK * (BN + 32) : BN * RLD;
  constexpr int STG = 3 * (A_PL + B_PL);
  constexpr int XS = (XBN && MODE == FWD) ? 2 * kMaxXbn : 0;  // floats
  constexpr int DUM = (PA || PB) ? 12 * NT : 0;                // dummy plane slots (16-bit)
  constexpr int NBUF = SEQ ? 1 : 2;
  static_assert(NBUF * STG >= 8 * BN, "epilogue scratch");
  __shared__ __attribute__((aligned(16))) u16 smem[NBUF * STG + 2 * XS + DUM];
  float* xbn = (float*)(smem + NBUF * STG);
  u16* dum = smem + NBUF * STG + 2 * XS + 12 * threadIdx.x;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN, li = lane & 31, lh = lane >> 5;
  int m0, n0, by;
  conv_block_tile<BM, BN>(a, m0, n0, by);  // XCD-aware order over the whole grid
  int g, sp = 0;
  if constexpr (MODE == WGRAD) { g = by / a.splits; sp = by % a.splits; }
  else g = by;
  int kbeg = 0, kend = a.K;
  if constexpr (MODE == WGRAD) { kbeg = sp * a.kchunk; kend = min(a.K, kbeg + a.kchunk); }
  // STEM (FWD, Cin = 4 zero-padded channels, xs_w = 4): the taps of one filter row as pixel
  // quads, s = 4h .. 4h+3 in stage h of the row (S <= 8: two stages per row; S <= 4: one)
  const int nt = STEM ? a.R * ((a.S + 3) / 4) : kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  const long long ny = (long long)a.B * a.Ho * a.Wo * a.Cout;  // dy floats per group
  const float* xg = a.x + (long long)g * a.xs_g;
  const float* wg = a.w + (long long)g * a.ws_g;
  const float* dyg = a.dy + (long long)g * ny;
  __amdgpu_buffer_rsrc_t ra, rb;
  if constexpr (MODE == FWD) { ra = rsrc(xg, a.B * a.xs_b); rb = rsrc(wg, a.ws_g); }
  else if constexpr (MODE == DGRAD) { ra = rsrc(dyg, ny); rb = rsrc(wg, a.ws_g); }
  else { ra = rsrc(dyg, ny); rb = rsrc(xg, a.B * a.xs_b); }
  const int xs_h = (int)a.xs_h, xs_w = (int)a.xs_w, xs_b = (int)a.xs_b;

  // ---- per-thread loader constants ----
  unsigned abase[NVA], bbase[NVB];
  int aq0[NVA], aq1[NVA];
  int bq0[NVB], bq1[NVB], bq2[NVB];
  floatx4 wsc = {1.f, 1.f, 1.f, 1.f}, wsh = {0.f, 0.f, 0.f, 0.f};  // WGRAD pending BN of x
  const int kq = tid & 3;
#pragma unroll
  for (int j = 0; j < NVA; ++j) {
    const int idx = tid + NT * j;
    if constexpr (MODE == FWD || MODE == DGRAD) {
      const int m = m0 + row_of(idx);
      const bool ok = m < a.M;
      const int mm = ok ? m : 0;
      if constexpr (MODE == FWD) {
        const int HW = a.Ho * a.Wo, b = mm / HW, rem = mm - b * HW;
        const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
        const int p0 = oh * a.stride - a.pad, p1 = ow * a.stride - a.pad;
        abase[j] = (unsigned)((b * xs_b + p0 * xs_h + p1 * xs_w + 4 * kq) * 4);
        aq0[j] = ok ? p0 : -(1 << 28);
        aq1[j] = STEM ? p1 + kq : p1;  // STEM: quad kq is the pixel of tap t_s + kq
      } else {
        const int HW = a.Hc * a.Wc, b = mm / HW, rem = mm - b * HW;
        const int i = rem / a.Wc, jj = rem - i * a.Wc;
        const int q0 = i + (a.ph + a.pad - a.r0) / a.stride;
        const int q1 = jj + (a.pw + a.pad - a.s0) / a.stride;
        abase[j] = (unsigned)(((b * a.Ho * a.Wo + q0 * a.Wo + q1) * a.Cout + 4 * kq) * 4);
        aq0[j] = ok ? q0 : (1 << 28);
        aq1[j] = q1;
      }
    } else {  // WGRAD A: 4 consecutive couts at k row idx / (BM/4)
      const int co = m0 + 4 * (idx % (BM / 4)), kr = idx / (BM / 4);
      abase[j] = co < a.M ? (unsigned)((kr * a.Cout + co) * 4) : kOOB;
      aq0[j] = kr;
      aq1[j] = 0;
    }
  }
#pragma unroll
  for (int j = 0; j < NVB; ++j) {
    const int idx = tid + NT * j;
    if constexpr (MODE == FWD) {
      const int n = n0 + row_of(idx);
      bbase[j] = n < a.N ? (unsigned)((n * a.K + 4 * kq) * 4) : kOOB;
    } else if constexpr (MODE == DGRAD) {
      const int c = n0 + 4 * (idx % (BN / 4)), kr = idx / (BN / 4);
      bbase[j] = c < a.N ? (unsigned)((kr * a.R * a.S * a.Cin + c) * 4) : kOOB;
    } else {  // WGRAD B: fixed column quad (r, s, c..c+3), pixel row idx / (BN/4)
      const int col = n0 + 4 * (idx % (BN / 4));
      const bool ok = col < a.N;
      const int cc = ok ? col : 0, rs = cc / a.Cin, c = cc - rs * a.Cin;
      const int r = rs / a.S, s = rs - r * a.S;
      bq0[j] = idx / (BN / 4);        // pixel row within the stage
      bq1[j] = ok ? r - a.pad : -(1 << 28);
      bq2[j] = s - a.pad;
      bbase[j] = (unsigned)(c * 4);
      if constexpr (XBN) {
        if (j == 0) {
          wsc = *(const floatx4*)(a.xsc + g * a.Cin + c);
          wsh = *(const floatx4*)(a.xsh + g * a.Cin + c);
        }
      }
    }
  }
  if constexpr (XBN && MODE == FWD) {
    for (int i = tid; i < a.Cin; i += NT) {
      xbn[i] = a.xsc[g * a.Cin + i];
      xbn[kMaxXbn + i] = a.xsh[g * a.Cin + i];
    }
  }

  // ---- tile-uniform k position (FWD: tap r, s + channel; DGRAD: tap tr, ts + cout) ----
  int t_r = 0, t_s = 0, t_c = 0;
  typedef Stage<NVA, NVB> St;

  auto load = [&](St& S, int t) {
    const int k0 = kbeg + t * BK;
    const bool sok = STEM ? t < nt : k0 < kend;  // stage-uniform (FWD / DGRAD: K % 16 == 0)
    if constexpr (MODE == FWD) {
      const unsigned soff = (unsigned)((t_r * xs_h + t_s * xs_w + t_c) * 4);
      const bool tap = !STEM || kq + t_s < a.S;  // STEM: quad kq is tap s = t_s + kq
      S.ok = 0;
      S.tc = t_c;
#pragma unroll
      for (int j = 0; j < NVA; ++j) {
        const bool ok = sok & tap & ((unsigned)(aq0[j] + t_r) < (unsigned)a.H) &
                        ((unsigned)(aq1[j] + t_s) < (unsigned)a.W);
        const bool act = !PA || tid + NT * j < LA;
        S.a[j] = bload(ra, sel_off(ok & act, abase[j] + soff, kOOB));
        S.ok |= (unsigned)ok << j;
      }
#pragma unroll
      for (int j = 0; j < NVB; ++j) {
        const bool act = !PB || tid + NT * j < LB;
        S.b[j] = bload(rb, sok && act && tap ? bbase[j] + (unsigned)(STEM ? (t_r * a.S + t_s) * 16
                                                                         : k0 * 4)
                                             : kOOB);
      }
      if constexpr (STEM) {
        t_s += 4;
        if (t_s >= a.S) { t_s = 0; ++t_r; }
      } else {
        t_c += BK;
        if (t_c >= a.Cin) { t_c = 0; if (++t_s == a.S) { t_s = 0; ++t_r; } }
      }
    } else if constexpr (MODE == DGRAD) {
      const unsigned soff = (unsigned)((t_c - (t_r * a.Wo + t_s) * a.Cout) * 4);
#pragma unroll
      for (int j = 0; j < NVA; ++j) {
        const bool ok = sok & ((unsigned)(aq0[j] - t_r) < (unsigned)a.Ho) &
                        ((unsigned)(aq1[j] - t_s) < (unsigned)a.Wo) & (!PA || tid + NT * j < LA);
        S.a[j] = bload(ra, sel_off(ok, abase[j] + soff, kOOB));
      }
      const int r = a.r0 + a.stride * t_r, s = a.s0 + a.stride * t_s;
      const unsigned woff = (unsigned)(((t_c * a.R + r) * a.S + s) * a.Cin * 4);
#pragma unroll
      for (int j = 0; j < NVB; ++j)
        S.b[j] = bload(rb, sok && (!PB || tid + NT * j < LB) ? bbase[j] + woff : kOOB);
      t_c += BK;
      if (t_c >= a.Cout) { t_c = 0; if (++t_s == a.ns) { t_s = 0; ++t_r; } }
    } else {
#pragma unroll
      for (int j = 0; j < NVA; ++j) {
        const bool ok = k0 + aq0[j] < kend && (!PA || tid + NT * j < LA);
        S.a[j] = bload(ra, ok ? abase[j] + (unsigned)(k0 * a.Cout * 4) : kOOB);
      }
      // pixel k0 + d (d = the float4's pixel row < 16): conv_pipe16.hip's branch-free form
      const unsigned HW = (unsigned)(a.Ho * a.Wo);
      const unsigned b0 = mdiv((unsigned)k0, a.mg_hw, a.sh_hw), p0 = (unsigned)k0 - b0 * HW;
      const unsigned oh0 = mdiv(p0, a.mg_w, a.sh_w), ow0 = p0 - oh0 * (unsigned)a.Wo;
      const int lim = kend - k0;
      S.ok = 0;
#pragma unroll
      for (int j = 0; j < NVB; ++j) {
        const unsigned tw = ow0 + (unsigned)bq0[j], q1 = udiv16(tw, a.m16_w);
        const unsigned th = oh0 + q1, q2 = udiv16(th, a.m16_h);
        const int ow = (int)(tw - q1 * (unsigned)a.Wo), oh = (int)(th - q2 * (unsigned)a.Ho);
        const int b = (int)(b0 + q2);
        const int ih = oh * a.stride + bq1[j], iw = ow * a.stride + bq2[j];
        const bool ok = (bq0[j] < lim) & ((unsigned)ih < (unsigned)a.H) &
                        ((unsigned)iw < (unsigned)a.W) & (!PB || tid + NT * j < LB);
        S.b[j] = bload(rb, sel_off(ok, bbase[j] + (unsigned)((b * xs_b + ih * xs_h + iw * xs_w) * 4),
                                   kOOB));
        S.ok |= (unsigned)ok << (8 + j);
      }
    }
  };

  auto split_store = [&](const St& S, int buf) {
    u16* As = smem + buf * STG;
    u16* Bs = As + 3 * A_PL;
#pragma unroll
    for (int j = 0; j < NVA; ++j) {
      const int idx = tid + NT * j;
      floatx4 v = S.a[j];
      if constexpr (XBN && MODE == FWD) {
        const int c = S.tc + 4 * kq;
        v = bn_relu(v, *(const floatx4*)(xbn + c), *(const floatx4*)(xbn + kMaxXbn + c), a.xrelu,
                    (S.ok >> j) & 1);
      }
      const int off = A_COL ? (idx / (BM / 4)) * (BM + 32) + 4 * (idx % (BM / 4))
                            : row_of(idx) * RLD + 4 * (idx & 3);
      const bool act = !PA || idx < LA;
      u16* dst = act ? As + off : dum;
      const int pst = act ? A_PL : 4;
      uint2 pl[3];
      split_bf16<3>(v, pl);
#pragma unroll
      for (int p = 0; p < 3; ++p) *(uint2*)(dst + p * pst) = pl[p];
    }
#pragma unroll
    for (int j = 0; j < NVB; ++j) {
      const int idx = tid + NT * j;
      floatx4 v = S.b[j];
      if constexpr (XBN && MODE == WGRAD) v = bn_relu(v, wsc, wsh, a.xrelu, (S.ok >> (8 + j)) & 1);
      const int off = B_COL ? (idx / (BN / 4)) * (BN + 32) + 4 * (idx % (BN / 4))
                            : row_of(idx) * RLD + 4 * (idx & 3);
      const bool act = !PB || idx < LB;
      u16* dst = act ? Bs + off : dum;
      const int pst = act ? B_PL : 4;
      uint2 pl[3];
      split_bf16<3>(v, pl);
#pragma unroll
      for (int p = 0; p < 3; ++p) *(uint2*)(dst + p * pst) = pl[p];
    }
  };

  floatx16 acc[MI][NI], acl[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) { acc[mi][ni][r] = 0.f; acl[mi][ni][r] = 0.f; }

  auto compute = [&](int buf) {
    const u16* As = smem + buf * STG;
    const u16* Bs = As + 3 * A_PL;
    u32x4 af[3][MI], bq[3][NI];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        if constexpr (A_COL) af[p][mi] = col_frag(As + p * A_PL, BM + 32, wm * WM + mi * 32, 0, lane);
        else af[p][mi] = row_frag_ld<RLD>(As + p * A_PL, wm * WM + mi * 32, 0, li, lh);
      }
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        if constexpr (B_COL) bq[p][ni] = col_frag(Bs + p * B_PL, BN + 32, wn * WN + ni * 32, 0, lane);
        else bq[p][ni] = row_frag_ld<RLD>(Bs + p * B_PL, wn * WN + ni * 32, 0, li, lh);
      }
    }
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        floatx16 c = ONEACC ? acc[mi][ni] : acl[mi][ni];
        c = H16<DT_BF16>::mfma(af[0][mi], bq[2][ni], c);
        c = H16<DT_BF16>::mfma(af[2][mi], bq[0][ni], c);
        c = H16<DT_BF16>::mfma(af[1][mi], bq[1][ni], c);
        c = H16<DT_BF16>::mfma(af[0][mi], bq[1][ni], c);
        c = H16<DT_BF16>::mfma(af[1][mi], bq[0][ni], c);
        if constexpr (ONEACC) {
          acc[mi][ni] = H16<DT_BF16>::mfma(af[0][mi], bq[0][ni], c);
        } else {
          acl[mi][ni] = c;
          acc[mi][ni] = H16<DT_BF16>::mfma(af[0][mi], bq[0][ni], acc[mi][ni]);
        }
      }
  };

  // SEQ with the BN-partials epilogue (BP): its register budget is the pipelined kernel's (four
  // waves per SIMD), so the next stage's loads go out before this stage's MFMAs — one LDS buffer,
  // two register stages — instead of each stage waiting for its own loads
  constexpr bool SEQ_PF = SEQ && BP;
  if constexpr (SEQ_PF) {
    St S0, S1;
    load(S0, 0);
    for (int t = 0; t < nt; t += 2) {
      split_store(S0, 0);
      __syncthreads();
      if (t + 1 < nt) load(S1, t + 1);
      compute(0);
      __syncthreads();  // the next stage / the epilogue scratch reuses the buffer
      if (t + 1 >= nt) break;
      split_store(S1, 0);
      __syncthreads();
      if (t + 2 < nt) load(S0, t + 2);
      compute(0);
      __syncthreads();
    }
  } else if constexpr (SEQ) {
    St S0;
    if constexpr (XBN && MODE == FWD) __syncthreads();  // xbn staged
    for (int t = 0; t < nt; ++t) {
      load(S0, t);
      split_store(S0, 0);
      __syncthreads();
      compute(0);
      __syncthreads();  // the next stage / the epilogue scratch reuses the buffer
    }
  } else {
  // ---- pipeline: buffer 0 <- tile 0, registers S1 <- tile 1 ----
  St S0, S1;
  load(S0, 0);
  load(S1, 1);
  if constexpr (XBN && MODE == FWD) __syncthreads();  // xbn staged
  split_store(S0, 0);
  __syncthreads();
  for (int t = 0; t < nt; t += 2) {
    load(S0, t + 2);
    compute(0);
    split_store(S1, 1);
    __syncthreads();
    // (an odd nt — only the ragged last split-K chunk of a WGRAD — computes one all-zero tile
    // here rather than branching out of the stage pair)
    load(S1, t + 3);
    compute(1);
    split_store(S0, 0);
    __syncthreads();
  }
  }

  if constexpr (!ONEACC) {
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) acc[mi][ni] += acl[mi][ni];
  }
  // fp32 outputs through LDS as 16-byte rows (staged_epilogue_f32): data gradients with a
  // residual addend / accumulation, and forwards (statistics from the registers first); the
  // per-element stores of conv_epilogue stay for the rest (plain data gradients, N % 4 != 0)
  if constexpr (MODE == DGRAD) {
    if (BP || a.addend || a.accumulate) {
      staged_epilogue_f32<DGRAD, BM, BN, MI, NI, WGM, WGN, NBUF * STG * 2, BP>(
          a, acc, (float*)smem, m0, n0, g);
      return;
    }
  }
  if constexpr (MODE == FWD) {
    if (a.N % 4 == 0 && a.out_sg % 4 == 0 && a.cpg % 4 == 0 && a.bias_sg % 4 == 0) {
      if (a.st_mean) fwd_stats_f32<BM, BN, MI, NI, WGM, WGN>(a, acc, (float*)smem, tid, m0, n0, g);
      staged_epilogue_f32<FWD, BM, BN, MI, NI, WGM, WGN, NBUF * STG * 2>(a, acc, (float*)smem,
                                                                        m0, n0, g);
      return;
    }
  }
  conv_epilogue<MODE, BM, BN, MI, NI, WGM, WGN, BP>(a, acc, (float*)smem, tid, m0, n0, g, sp);
}

template <int MODE, int BM, int BN, bool XBN, int WV = 4, bool STEM = false, bool SEQ = false,
          bool BP = false>
static void launch_split(const ConvArgs& a, int oneacc, hipStream_t st) {
  dim3 grid(ceil_div(a.M, BM) * ceil_div(a.N, BN), MODE == WGRAD ? a.G * a.splits : a.G);
  const dim3 block(SplitWaves<BM, BN, WV>::T);
  if constexpr (WV == 8) {  // one accumulator set (128-VGPR budget)
    hipLaunchKernelGGL((conv_split_f32<MODE, BM, BN, XBN, true, WV, STEM, SEQ, BP>), grid, block, 0, st,
                       a);
  } else {
    if (oneacc)
      hipLaunchKernelGGL((conv_split_f32<MODE, BM, BN, XBN, true, WV, STEM, false, BP>), grid, block,
                         0, st, a);
    else
      hipLaunchKernelGGL((conv_split_f32<MODE, BM, BN, XBN, false, WV, STEM, false, BP>), grid,
                         block, 0, st, a);
  }
}

// forward launches with K <= 256 take the SEQ kernel
constexpr int kSplitShortK = 256;

template <int MODE, bool XBN>
static void split_tiles(const ConvArgs& a, int oneacc, hipStream_t st) {
  const int bm = conv_tile_rows(a.M), bn = conv_tile_rows(a.N);
  if constexpr (MODE == DGRAD) {
    if (a.bp_p1) {  // BN-backward partials from the epilogue (the bn_p1 arguments of the C-ABI)
      if (bm == 128 && bn == 128 && a.K > 0 && a.K <= kSplitShortK)
        launch_split<MODE, 128, 128, XBN, 8, false, true, true>(a, oneacc, st);
      else if (bm == 128 && bn == 128) launch_split<MODE, 128, 128, XBN, 8, false, false, true>(a, oneacc, st);
      else if (bm == 128 && bn == 64) launch_split<MODE, 128, 64, XBN, 8, false, false, true>(a, oneacc, st);
      else if (bm == 64 && bn == 128) launch_split<MODE, 64, 128, XBN, 8, false, false, true>(a, oneacc, st);
      else launch_split<MODE, 64, 64, XBN, 4, false, false, true>(a, oneacc, st);
      return;
    }
  }
  // eight-wave blocks (four waves per SIMD): 128 x 128 tiles as waves of 32 x 64, 128 x 64 and
  // 64 x 128 as waves of 32 x 32 — measured 200 vs 235 ms of convs per bench step over four
  // waves.  256-wide tiles (225 vs 229 ms of convs per step against two co-resident 128 x 128
  // blocks) were measured and removed.  The short-K (SEQ) kernel serves the forwards and the
  // data gradients without the BN-partials epilogue.
  if constexpr (MODE == FWD || MODE == DGRAD) {
    if (bm == 128 && bn == 128 && a.K > 0 && a.K <= kSplitShortK) {
      launch_split<MODE, 128, 128, XBN, 8, false, true>(a, oneacc, st);
      return;
    }
  }
  if (bm == 128 && bn == 128) launch_split<MODE, 128, 128, XBN, 8>(a, oneacc, st);
  else if (bm == 128 && bn == 64) launch_split<MODE, 128, 64, XBN, 8>(a, oneacc, st);
  else if (bm == 64 && bn == 128) launch_split<MODE, 64, 128, XBN, 8>(a, oneacc, st);
  else launch_split<MODE, 64, 64, XBN>(a, oneacc, st);
}

bool conv_split_launch(int mode, const ConvArgs& a0, int oneacc, hipStream_t st) {
  const long long lim = 0x7fff0000LL / 4;  // floats addressable by a 31-bit byte offset
  const long long nx = (long long)a0.B * a0.xs_b, ny = (long long)a0.B * a0.Ho * a0.Wo * a0.Cout;
  if (mode == FWD && nx > lim && !a0.cpg && a0.xs_g != 0)
    return conv_fwd_batch_chunks(a0, lim, 4, [&](const ConvArgs& c) {
      return conv_split_launch(FWD, c, oneacc, st);
    });
  // (the FWD output is stored through plain pointers: only dgrad / wgrad read y by rsrc)
  if (nx > lim || (mode != FWD && ny > lim) || a0.ws_g > lim) return false;
  ConvArgs a = a0;
  a.xcd_grid = 1;
  if (mode == FWD && a.Cin == 4 && a.S <= 8 && a.xs_c == 1 && a.xs_w == 4 && !a.xsc &&
      a.xs_h % 4 == 0 && a.xs_b % 4 == 0 && a.xs_g % 4 == 0 && a.N == 64) {
    // the stems over 4 zero-padded input channels (mauv_pack_nchw_f32)
    if (a.M > 64) launch_split<FWD, 128, 64, false, 8, true>(a, oneacc, st);
    else launch_split<FWD, 64, 64, false, 4, true>(a, oneacc, st);
    return true;
  }
  if (mode == FWD) {
    const bool va = (a.Cin % 32 == 0) && a.xs_c == 1 && a.xs_w % 4 == 0 && a.xs_h % 4 == 0 &&
                    a.xs_b % 4 == 0 && a.xs_g % 4 == 0 && a.xs_g != 0;
    if (!va || (a.xsc && a.Cin > kMaxXbn)) return false;
    if (a.xsc) split_tiles<FWD, true>(a, oneacc, st);
    else split_tiles<FWD, false>(a, oneacc, st);
  } else if (mode == DGRAD) {
    if (a.Cout % 32 || a.Cin % 4) return false;
    split_tiles<DGRAD, false>(a, oneacc, st);
  } else {
    const bool vb = (a.Cin % 4 == 0) && a.xs_c == 1 && a.xs_w % 4 == 0 && a.xs_h % 4 == 0 &&
                    a.xs_b % 4 == 0 && a.xs_g % 4 == 0;
    if (a.Cout % 4 || !vb) return false;
    if (a.Wo > 4096 || a.Ho > 4096) return false;
    magic_div((unsigned)(a.Ho * a.Wo), a.mg_hw, a.sh_hw);
    magic_div((unsigned)a.Wo, a.mg_w, a.sh_w);
    a.m16_w = m16_div((unsigned)a.Wo);
    a.m16_h = m16_div((unsigned)a.Ho);
    if (a.xsc) split_tiles<WGRAD, true>(a, oneacc, st);
    else split_tiles<WGRAD, false>(a, oneacc, st);
  }
  return true;
}

}  // namespace mauv
