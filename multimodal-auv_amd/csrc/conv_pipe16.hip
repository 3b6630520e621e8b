// Pipelined 16-bit implicit-GEMM convolution (bf16 training, BASELINE configs[2]; f16 MC
// inference under the reference predictor's torch.amp.autocast, inference/predictors.py:55):
// the three GEMM views of conv_gemm16.hip with the staging structure of the split-fp32 kernel
// (conv_split.hip):
//  * tiles BM x BN x 64 (one (r, s) tap per stage), eight waves per 128-wide block;
//  * two tiles in flight: stage t issues the 16-byte buffer loads of tile t+2, runs the MFMAs of
//    tile t (four v_mfma_f32_32x32x16 k-steps) from one LDS buffer and writes tile t+1 into the
//    other — one branch-free basic block per stage;
//  * raw buffer loads with 32-bit offsets (an offset past the descriptor range returns 0:
//    padding, ragged tiles and tiles past K need no branches);
//  * the producing layer's pending BN(+ReLU) applied when the staged chunk is written to LDS
//    (forward: scale/shift of the input channels staged in LDS once per block).
// LDS images as conv_gemm16.hip: k-contiguous operands (FWD A/B, DGRAD A) as row images
// [rows][72] (ds_read_b128 fragments, conflict-free 144-B rows), k-strided operands (DGRAD B,
// WGRAD A/B) as col images [64][rows+32] (ds_read_b64_tr_b16).  Epilogues: FWD statistics from
// the fp32 accumulators and 16-bit rows staged through LDS (DGRAD: + addend / accumulate, parity
// class row remap); WGRAD fp32 split-K slabs (conv_common.h).

#include <stdlib.h>

#include "conv_common.h"
#include "conv_epi16.h"

namespace mauv {

namespace {

constexpr unsigned kOOB16 = 0x7ffffff0u;  // beyond every descriptor range: the load returns 0
constexpr int kMaxXbn16 = 512;             // FWD pending-BN input channels staged in LDS

__device__ __forceinline__ u32x4 bload16(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc16(const void* p, long long nelem) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(nelem * 2), 0x00020000);
}
__device__ __forceinline__ unsigned mdiv16(unsigned n, unsigned long long m, int s) {
  return (unsigned)(((unsigned long long)n * m) >> s);
}
template <int NVA, int NVB>
struct Stage16 {
  u32x4 a[NVA], b[NVB];
  unsigned ok;  // validity bits of pending-BN chunks: a j -> bit j, b j -> bit 8 + j
  int tc;       // FWD: input-channel offset of this stage's k slice
};

}  // namespace

// 2 x 2 waves (32 x 32 each) for 64 x 64 tiles; 4 x 2 / 2 x 4 waves of 32 x 64 / 64 x 32 for
// 128 x 128, 4 x 2 / 2 x 4 of 32 x 32 for 128 x 64 / 64 x 128 (eight waves, four per SIMD:
// two blocks per CU).  Measured and dropped: 128 x 256 tiles as 2 x 4 waves of 64 x 64 (one
// block per CU: 5-25 % slower per shape) and 128 x 128 as 2 x 2 waves of 64 x 64 (neutral to
// -2 %), DESIGN.md §2.7.
template <int BM, int BN>
struct Waves16 {
  static constexpr bool W8 = BM + BN >= 192;
  static constexpr int M = W8 ? (BM == 128 ? 4 : 2) : 2;
  static constexpr int N = W8 ? (BM == 128 ? 2 : 4) : 2;
  static constexpr int T = 64 * M * N, EU = 4;
};

// ONE: short K (a few 64-deep stages, the 1x1 convs over 64-128 channels): one LDS buffer, one
// register stage, stages run one after another, and a register budget low enough for three to
// four blocks per CU instead of two — with one or two stages there is little of a next tile to
// overlap inside a block, so more resident blocks are the cover for load and store latency
// SHORT: 0 = the two-stage pipeline; 1 = exactly one stage (nt == 1, straight-line: 62 VGPRs,
// up to four blocks per CU); 2 = short K through one buffer, stages one after another.
template <int MODE, int DT, int BM, int BN, bool XBN, bool STEM, int SHORT = 0, bool BP = false>
__global__ __launch_bounds__((Waves16<BM, BN>::T))
__attribute__((amdgpu_waves_per_eu(SHORT ? 6 : Waves16<BM, BN>::EU)))
void conv_pipe16(const ConvArgs a) {
  constexpr int BK = 64, EPC = 8, KQ = BK / EPC;
  constexpr int WGM = Waves16<BM, BN>::M, WGN = Waves16<BM, BN>::N, NT = Waves16<BM, BN>::T;
  constexpr int WM = BM / WGM, WN = BN / WGN, MI = WM / 32, NI = WN / 32;
  // 16-byte chunks per stage per operand (LA, LB) and per thread; with LB < NT the threads
  // tid >= LB load nothing and park their chunk in a dummy LDS slot (branch-free stage)
  constexpr int LA = BM * KQ, LB = BN * KQ;
  constexpr int NVA = (LA + NT - 1) / NT, NVB = (LB + NT - 1) / NT;
  constexpr bool PA = LA % NT != 0, PB = LB % NT != 0;
  constexpr bool A_COL = (MODE == WGRAD), B_COL = (MODE != FWD);
  constexpr int RLD = BK + 8;
  constexpr int A_SZ = A_COL ? BK * (BM + 32) : BM * RLD;  // 16-bit words
  constexpr int B_SZ = B_COL ? BK * (BN + 32) : BN * RLD;
  constexpr int STG = A_SZ + B_SZ;
  constexpr int XS = (XBN && MODE == FWD) ? 2 * kMaxXbn16 : 0;  // floats
  constexpr int DUM = (PA || PB) ? 8 * NT : 0;                 // dummy chunk slots (16-bit)
  constexpr bool ONE = SHORT != 0;
  constexpr int NBUF = ONE ? 1 : 2;
  static_assert(NBUF * STG >= 2 * WM * (BN + 4) && NBUF * STG >= 8 * WGM * BN, "epilogue scratch");
  __shared__ __attribute__((aligned(16))) u16 smem[NBUF * STG + 2 * XS + DUM];
  float* xbn = (float*)(smem + NBUF * STG);
  u16* dum = smem + NBUF * STG + 2 * XS + 8 * threadIdx.x;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN, li = lane & 31, lh = lane >> 5;
  int m0, n0, by;
  conv_block_tile<BM, BN>(a, m0, n0, by);  // XCD-aware order over the whole grid
  int g, sp = 0;
  if constexpr (MODE == WGRAD) { g = by / a.splits; sp = by % a.splits; }
  else g = by;
  int kbeg = 0, kend = a.K;
  if constexpr (MODE == WGRAD) { kbeg = sp * a.kchunk; kend = min(a.K, kbeg + a.kchunk); }
  // STEM (FWD, Cin = 8, S <= 8): stage r holds the S taps of filter row r as 8 pixel chunks
  const int nt = STEM ? a.R : kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  const long long ny = (long long)a.B * a.Ho * a.Wo * a.Cout;  // dy elements per group
  const u16* xg = (const u16*)a.x + (long long)g * a.xs_g;
  const u16* wg = (const u16*)a.w + (long long)g * a.ws_g;
  const u16* dyg = (const u16*)a.dy + (long long)g * ny;
  __amdgpu_buffer_rsrc_t ra, rb;
  if constexpr (MODE == FWD) { ra = rsrc16(xg, a.B * a.xs_b); rb = rsrc16(wg, a.ws_g); }
  else if constexpr (MODE == DGRAD) { ra = rsrc16(dyg, ny); rb = rsrc16(wg, a.ws_g); }
  else { ra = rsrc16(dyg, ny); rb = rsrc16(xg, a.B * a.xs_b); }
  const int xs_h = (int)a.xs_h, xs_w = (int)a.xs_w, xs_b = (int)a.xs_b;

  // ---- per-thread loader constants ----
  unsigned abase[NVA], bbase[NVB];
  int aq0[NVA], aq1[NVA];
  int bq0[NVB], bq1[NVB], bq2[NVB];
  floatx8 wsc, wsh;  // WGRAD pending BN of x (per-thread channel chunk)
#pragma unroll
  for (int e = 0; e < 8; ++e) { wsc[e] = 1.f; wsh[e] = 0.f; }
  const int kq = tid % KQ;
#pragma unroll
  for (int j = 0; j < NVA; ++j) {
    const int idx = tid + NT * j;
    if constexpr (MODE == FWD || MODE == DGRAD) {
      const int m = m0 + idx / KQ;
      const bool ok = m < a.M && (!PA || idx < LA);
      const int mm = m < a.M ? m : 0;
      if constexpr (MODE == FWD) {
        const int HW = a.Ho * a.Wo, b = mm / HW, rem = mm - b * HW;
        const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
        const int p0 = oh * a.stride - a.pad, p1 = ow * a.stride - a.pad;
        abase[j] = (unsigned)((b * xs_b + p0 * xs_h + p1 * xs_w + EPC * kq) * 2);
        aq0[j] = ok ? p0 : -(1 << 28);
        aq1[j] = STEM ? (kq < a.S ? p1 + kq : -(1 << 28)) : p1;  // STEM: chunk kq = tap s
      } else {
        const int HW = a.Hc * a.Wc, b = mm / HW, rem = mm - b * HW;
        const int i = rem / a.Wc, jj = rem - i * a.Wc;
        const int q0 = i + (a.ph + a.pad - a.r0) / a.stride;
        const int q1 = jj + (a.pw + a.pad - a.s0) / a.stride;
        abase[j] = (unsigned)(((b * a.Ho * a.Wo + q0 * a.Wo + q1) * a.Cout + EPC * kq) * 2);
        aq0[j] = ok ? q0 : (1 << 28);
        aq1[j] = q1;
      }
    } else {  // WGRAD A: 8 consecutive couts at k row idx / (BM/8)
      const int co = m0 + EPC * (idx % (BM / EPC)), kr = idx / (BM / EPC);
      abase[j] = (co < a.M && (!PA || idx < LA)) ? (unsigned)((kr * a.Cout + co) * 2) : kOOB16;
      aq0[j] = kr;
      aq1[j] = 0;
    }
  }
#pragma unroll
  for (int j = 0; j < NVB; ++j) {
    const int idx = tid + NT * j;
    if constexpr (MODE == FWD) {
      const int n = n0 + idx / KQ;
      bbase[j] = (n < a.N && (!PB || idx < LB) && (!STEM || kq < a.S))
                     ? (unsigned)((n * a.K + EPC * kq) * 2) : kOOB16;
    } else if constexpr (MODE == DGRAD) {
      const int c = n0 + EPC * (idx % (BN / EPC)), kr = idx / (BN / EPC);
      bbase[j] = (c < a.N && (!PB || idx < LB)) ? (unsigned)((kr * a.R * a.S * a.Cin + c) * 2)
                                                 : kOOB16;
    } else {  // WGRAD B: fixed column chunk (r, s, c..c+7), pixel row idx / (BN/8)
      const int col = n0 + EPC * (idx % (BN / EPC));
      const bool ok = col < a.N && (!PB || idx < LB);
      const int cc = ok ? col : 0, rs = cc / a.Cin, c = cc - rs * a.Cin;
      const int r = rs / a.S, s = rs - r * a.S;
      bq0[j] = idx / (BN / EPC);
      bq1[j] = ok ? r - a.pad : -(1 << 28);
      bq2[j] = s - a.pad;
      bbase[j] = (unsigned)(c * 2);
      if constexpr (XBN) {
        if (j == 0) {
          wsc = ldf8(a.xsc + g * a.Cin + c);
          wsh = ldf8(a.xsh + g * a.Cin + c);
        }
      }
    }
  }
  // FWD pending BN: fetched here, put into LDS once the first tile loads are issued
  constexpr int XJ = (XBN && MODE == FWD) ? (kMaxXbn16 + NT - 1) / NT : 1;
  float xv[XJ][2];
  if constexpr (XBN && MODE == FWD) xbn_fetch(xv, a.xsc + g * a.Cin, a.xsh + g * a.Cin, a.Cin, tid, NT);
  auto xbn_stage = [&]() {
    if constexpr (XBN && MODE == FWD) xbn_put(xbn, xbn + kMaxXbn16, xv, a.Cin, tid, NT);
  };

  int t_r = 0, t_s = 0, t_c = 0;  // tile-uniform k position (FWD: r, s, cin; DGRAD: tr, ts, cout)
  typedef Stage16<NVA, NVB> St;

  auto load = [&](St& S, int t) {
    const int k0 = kbeg + t * BK;
    const bool sok = STEM ? t < a.R : k0 < kend;  // stage-uniform (FWD / DGRAD: K % 64 == 0)
    if constexpr (MODE == FWD) {
      const unsigned soff = (unsigned)((t_r * xs_h + t_s * xs_w + t_c) * 2);
      S.ok = 0;
      S.tc = t_c;
#pragma unroll
      for (int j = 0; j < NVA; ++j) {
        const bool ok = sok & ((unsigned)(aq0[j] + t_r) < (unsigned)a.H) &
                        ((unsigned)(aq1[j] + t_s) < (unsigned)a.W);
        S.a[j] = bload16(ra, sel_off(ok, abase[j] + soff, kOOB16));
        S.ok |= (unsigned)ok << j;
      }
#pragma unroll
      for (int j = 0; j < NVB; ++j)
        S.b[j] = bload16(rb, sok ? bbase[j] + (unsigned)(STEM ? t_r * a.S * 16 : k0 * 2) : kOOB16);
      if constexpr (STEM) {
        ++t_r;
      } else {
        t_c += BK;
        if (t_c >= a.Cin) { t_c = 0; if (++t_s == a.S) { t_s = 0; ++t_r; } }
      }
    } else if constexpr (MODE == DGRAD) {
      const unsigned soff = (unsigned)((t_c - (t_r * a.Wo + t_s) * a.Cout) * 2);
#pragma unroll
      for (int j = 0; j < NVA; ++j) {
        const bool ok = sok & ((unsigned)(aq0[j] - t_r) < (unsigned)a.Ho) &
                        ((unsigned)(aq1[j] - t_s) < (unsigned)a.Wo);
        S.a[j] = bload16(ra, sel_off(ok, abase[j] + soff, kOOB16));
      }
      const int r = a.r0 + a.stride * t_r, s = a.s0 + a.stride * t_s;
      const unsigned woff = (unsigned)(((t_c * a.R + r) * a.S + s) * a.Cin * 2);
#pragma unroll
      for (int j = 0; j < NVB; ++j) S.b[j] = bload16(rb, sok ? bbase[j] + woff : kOOB16);
      t_c += BK;
      if (t_c >= a.Cout) { t_c = 0; if (++t_s == a.ns) { t_s = 0; ++t_r; } }
    } else {
#pragma unroll
      for (int j = 0; j < NVA; ++j) {
        const bool ok = k0 + aq0[j] < kend;
        S.a[j] = bload16(ra, ok ? abase[j] + (unsigned)(k0 * a.Cout * 2) : kOOB16);
      }
      // pixel k0 + d of this stage (d = the chunk's pixel row < 64): k0 decomposed once per
      // stage (uniform), then d carried through the row and image with two 32-bit magic
      // divisions; branch-free (one select per load)
      const unsigned HW = (unsigned)(a.Ho * a.Wo);
      const unsigned b0 = mdiv16((unsigned)k0, a.mg_hw, a.sh_hw), p0 = (unsigned)k0 - b0 * HW;
      const unsigned oh0 = mdiv16(p0, a.mg_w, a.sh_w), ow0 = p0 - oh0 * (unsigned)a.Wo;
      const int lim = kend - k0;
      S.ok = 0;
#pragma unroll
      for (int j = 0; j < NVB; ++j) {
        const unsigned tw = ow0 + (unsigned)bq0[j], q1 = udiv16(tw, a.m16_w);
        const unsigned th = oh0 + q1, q2 = udiv16(th, a.m16_h);
        const int ow = (int)(tw - q1 * (unsigned)a.Wo), oh = (int)(th - q2 * (unsigned)a.Ho);
        const int b = (int)(b0 + q2);
        const int ih = oh * a.stride + bq1[j], iw = ow * a.stride + bq2[j];
        const bool ok = (bq0[j] < lim) & ((unsigned)ih < (unsigned)a.H) & ((unsigned)iw < (unsigned)a.W);
        S.b[j] = bload16(rb, sel_off(ok, bbase[j] + (unsigned)((b * xs_b + ih * xs_h + iw * xs_w) * 2),
                                     kOOB16));
        S.ok |= (unsigned)ok << (8 + j);
      }
    }
  };

  const unsigned rfloor = a.xrelu ? 0u : 0x80008000u;
  auto store = [&](const St& S, int buf) {
    u16* As = smem + buf * STG;
    u16* Bs = As + A_SZ;
    floatx8 fsc, fsh;  // FWD: every A chunk of this thread holds the same 8 input channels
    if constexpr (XBN && MODE == FWD) {
      fsc = ldf8(xbn + S.tc + EPC * kq);
      fsh = ldf8(xbn + kMaxXbn16 + S.tc + EPC * kq);
    }
#pragma unroll
    for (int j = 0; j < NVA; ++j) {
      const int idx = tid + NT * j;
      u32x4 v = S.a[j];
      if constexpr (XBN && MODE == FWD) v = bn_relu8<DT>(v, fsc, fsh, rfloor, (S.ok >> j) & 1);
      const int off = A_COL ? (idx / (BM / EPC)) * (BM + 32) + EPC * (idx % (BM / EPC))
                            : (idx / KQ) * RLD + EPC * (idx % KQ);
      *(u32x4*)((!PA || idx < LA) ? As + off : dum) = v;
    }
#pragma unroll
    for (int j = 0; j < NVB; ++j) {
      const int idx = tid + NT * j;
      u32x4 v = S.b[j];
      if constexpr (XBN && MODE == WGRAD) v = bn_relu8<DT>(v, wsc, wsh, rfloor, (S.ok >> (8 + j)) & 1);
      const int off = B_COL ? (idx / (BN / EPC)) * (BN + 32) + EPC * (idx % (BN / EPC))
                            : (idx / KQ) * RLD + EPC * (idx % KQ);
      *(u32x4*)((!PB || idx < LB) ? Bs + off : dum) = v;
    }
  };

  floatx16 acc[MI][NI];
  float cs[NI];  // the accumulators' start, loaded here and filled after the first tile loads
  acc_shift16(cs, a, n0 + wn * WN, MODE == FWD);

  auto compute = [&](int buf) {
    const u16* As = smem + buf * STG;
    const u16* Bs = As + A_SZ;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      u32x4 af[MI], bq[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        if constexpr (A_COL) af[mi] = col_frag(As, BM + 32, wm * WM + mi * 32, s, lane);
        else af[mi] = row_frag_ld<RLD>(As, wm * WM + mi * 32, s, li, lh);
      }
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        if constexpr (B_COL) bq[ni] = col_frag(Bs, BN + 32, wn * WN + ni * 32, s, lane);
        else bq[ni] = row_frag_ld<RLD>(Bs, wn * WN + ni * 32, s, li, lh);
      }
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = H16<DT>::mfma(af[mi], bq[ni], acc[mi][ni]);
    }
  };

  if constexpr (SHORT == 1) {  // nt == 1 (host-checked)
    St S0;
    load(S0, 0);
    acc_start16(acc, cs);
    xbn_stage();
    if constexpr (XBN && MODE == FWD) __syncthreads();  // xbn staged
    store(S0, 0);
    __syncthreads();
    compute(0);
    __syncthreads();  // the epilogue reuses the operand buffer
  } else if constexpr (SHORT == 2) {  // short K: stages one after another through one buffer
    St S0;
    auto stage = [&]() {
      store(S0, 0);
      __syncthreads();
      compute(0);
      __syncthreads();  // the next stage / the epilogue reuses the operand buffer
    };
    // (two loop shapes, each the one that fits the 80-VGPR budget of waves_per_eu(6) without a
    // spill or a lower occupancy: checked with -Rpass-analysis=kernel-resource-usage)
    if constexpr (XBN && MODE == FWD) {
      // the pending BN staged before the first tile load: no room to hold it across the load
      xbn_stage();
      __syncthreads();  // xbn staged
      for (int t = 0; t < nt; ++t) {
        load(S0, t);
        if (t == 0) acc_start16(acc, cs);
        stage();
      }
    } else {
      load(S0, 0);
      acc_start16(acc, cs);
      for (int t = 0;;) {
        stage();
        if (++t == nt) break;
        load(S0, t);
      }
    }
  } else {
  // ---- pipeline: buffer 0 <- tile 0, registers S1 <- tile 1 ----
  St S0, S1;
  load(S0, 0);
  load(S1, 1);
  acc_start16(acc, cs);
  xbn_stage();
  if constexpr (XBN && MODE == FWD) __syncthreads();  // xbn staged
  store(S0, 0);
  __syncthreads();
  for (int t = 0; t + 1 < nt; t += 2) {
    load(S0, t + 2);
    compute(0);
    store(S1, 1);
    __syncthreads();
    load(S1, t + 3);
    compute(1);
    store(S0, 0);
    __syncthreads();
  }
  // odd nt (1x1 over 64 channels, 3x3 over 64: 9 taps, the stems' 7 rows): the last tile sits
  // in buffer 0 — computed here, outside the branch-free loop body
  if (nt & 1) {
    compute(0);
    __syncthreads();  // the epilogue reuses the operand buffers
  }
  }

  // ---------------- epilogue ----------------
  if constexpr (MODE == WGRAD) {
    conv_epilogue<WGRAD, BM, BN, MI, NI, WGM, WGN>(a, acc, (float*)smem, tid, m0, n0, g, sp);
    return;
  }
  epilogue16<MODE, DT, BM, BN, MI, NI, WGM, WGN, NBUF * STG * 2, BP>(a, acc, smem, m0, n0, g);
}

template <int MODE, int DT, int BM, int BN, bool XBN, bool STEM = false, int SHORT = 0,
          bool BP = false>
static void launch_pipe16(const ConvArgs& a, hipStream_t st) {
  dim3 grid(ceil_div(a.M, BM) * ceil_div(a.N, BN), MODE == WGRAD ? a.G * a.splits : a.G);
  hipLaunchKernelGGL((conv_pipe16<MODE, DT, BM, BN, XBN, STEM, SHORT, BP>), grid,
                     dim3(Waves16<BM, BN>::T), 0, st, a);
}

// forward and data-gradient launches with K <= 256 take the short-K kernels (DESIGN.md §2.8b,
// §2.15: f16 inference 11.03k -> 11.52k MC-samples/s, bf16 training 563 -> 582 triplets/s)
constexpr int kShortK = 256;

template <int MODE, int DT, bool XBN, bool STEM>
static void pipe16_tiles(const ConvArgs& a, hipStream_t st) {
  const int bm = conv_tile_rows(a.M), bn = conv_tile_rows(a.N);
  if constexpr (MODE == DGRAD) {
    if (a.bp_p1) {  // BN-backward partials from the epilogue (mauv_conv2d_bwd_data_bn_h16)
      if (bm == 64 && bn == 64) launch_pipe16<MODE, DT, 64, 64, XBN, STEM, 0, true>(a, st);
      else if (bm == 64) launch_pipe16<MODE, DT, 64, 128, XBN, STEM, 0, true>(a, st);
      else if (bn == 64) launch_pipe16<MODE, DT, 128, 64, XBN, STEM, 0, true>(a, st);
      else launch_pipe16<MODE, DT, 128, 128, XBN, STEM, 0, true>(a, st);
      return;
    }
  }
  // short-K kernels: forwards, and data gradients without the BN-partials epilogue (K = the
  // parity class's taps x Cout)
  constexpr bool SHORT_OK = (MODE == FWD || MODE == DGRAD) && !STEM;
  constexpr bool use = true;
  if (bm == 64 && bn == 64) launch_pipe16<MODE, DT, 64, 64, XBN, STEM>(a, st);
  else if (bm == 64) launch_pipe16<MODE, DT, 64, 128, XBN, STEM>(a, st);
  else if (bn == 64) launch_pipe16<MODE, DT, 128, 64, XBN, STEM>(a, st);
  else if (SHORT_OK && use && a.K == 64)
    launch_pipe16<MODE, DT, 128, 128, XBN, STEM, SHORT_OK ? 1 : 0>(a, st);
  else if (SHORT_OK && use && a.K > 0 && a.K <= kShortK)
    launch_pipe16<MODE, DT, 128, 128, XBN, STEM, SHORT_OK ? 2 : 0>(a, st);
  else launch_pipe16<MODE, DT, 128, 128, XBN, STEM>(a, st);
}

template <int MODE, bool XBN, bool STEM = false>
static void pipe16_dt(int dt, const ConvArgs& a, hipStream_t st) {
  if (dt == DT_BF16) pipe16_tiles<MODE, DT_BF16, XBN, STEM>(a, st);
  else pipe16_tiles<MODE, DT_F16, XBN, STEM>(a, st);
}

// MauvRoute.big16: 1 (default) = the forwards where the 256-row LDS-DMA kernel (conv_big16.hip)
// measured faster take it; 2 = every forward it covers with K >= big16_min_k; 0 = none
static int big16() { return g_route.big16; }
static int big16_min_k() { return g_route.big16_min_k; }
// measured (tools/fwd_ab.py): faster only on 1x1 forwards without a pending
// BN over K >= 512 input channels into N >= 256 outputs with enough 256 x 256 tiles for two
// rounds of the chip; the 3x3s and the 128-column / few-tile shapes of the training slice ran
// 5-70 % slower than the implicit GEMM
static bool big16_wins(const ConvArgs& a) {
  const long long tiles = (long long)ceil_div(a.M, 256) * ceil_div(a.N, 256) * a.G;
  return a.R == 1 && a.S == 1 && !a.xsc && a.K >= 512 && a.N >= 256 && tiles >= 512;
}

bool conv_pipe16_launch(int mode, int dt, const ConvArgs& a0, hipStream_t st) {
  const long long lim = 0x7fff0000LL / 2;  // elements addressable by a 31-bit byte offset
  const long long nx = (long long)a0.B * a0.xs_b, ny = (long long)a0.B * a0.Ho * a0.Wo * a0.Cout;
  if (mode == FWD && nx > lim && !a0.cpg)
    return conv_fwd_batch_chunks(a0, lim, 2, [&](const ConvArgs& c) {
      return conv_pipe16_launch(FWD, dt, c, st);
    });
  // (the FWD output is stored through plain pointers: only dgrad / wgrad read y by rsrc)
  if (nx > lim || (mode != FWD && ny > lim) || a0.ws_g > lim) return false;
  const bool xs8 = a0.xs_w % 8 == 0 && a0.xs_h % 8 == 0 && a0.xs_b % 8 == 0 && a0.xs_g % 8 == 0;
  ConvArgs a = a0;
  a.xcd_grid = 1;
  if (mode == FWD) {
    if (a.Cin == 8 && a.S <= 8 && a.xs_w == 8 && !a.xsc && a.xs_h % 8 == 0 && a.xs_b % 8 == 0 &&
        a.xs_g % 8 == 0) {  // the stems: 7x7 taps over 8 zero-padded input channels
      pipe16_dt<FWD, false, true>(dt, a, st);
      return true;
    }
    if (a.Cin % 64 || !xs8 || (a.xsc && a.Cin > kMaxXbn16)) return false;
    if (conv_halo16_launch(FWD, dt, a, st)) return true;
    if (conv_haloc16_launch(FWD, dt, a, st)) return true;
    if (conv_expand16_launch(dt, a, st)) return true;
    if (big16() && a.K >= big16_min_k() && (big16() == 2 || big16_wins(a)) &&
        conv_big16_launch(dt, a, st))
      return true;
    if (a.xsc) pipe16_dt<FWD, true>(dt, a, st);
    else pipe16_dt<FWD, false>(dt, a, st);
  } else if (mode == DGRAD) {
    if (a.Cout % 64 || a.Cin % 8) return false;
    if (conv_halo16_launch(DGRAD, dt, a, st)) return true;
    if (conv_haloc16_launch(DGRAD, dt, a, st)) return true;
    pipe16_dt<DGRAD, false>(dt, a, st);
  } else {
    if (a.Cout % 8 || a.Cin % 8 || !xs8 || a.kchunk % 64) return false;
    if (a.Wo > 4096 || a.Ho > 4096) return false;
    magic_div((unsigned)(a.Ho * a.Wo), a.mg_hw, a.sh_hw);
    magic_div((unsigned)a.Wo, a.mg_w, a.sh_w);
    a.m16_w = m16_div((unsigned)a.Wo);
    a.m16_h = m16_div((unsigned)a.Ho);
    if (a.xsc) pipe16_dt<WGRAD, true>(dt, a, st);
    else pipe16_dt<WGRAD, false>(dt, a, st);
  }
  return true;
}

}  // namespace mauv
