// 16-bit 3x3 / stride-1 / pad-1 forward over 64 input and 64 output channels (the layer-1
// conv2 of every bottleneck: BASELINE configs[2]'s bf16 training, the f16 MC inference under
// the reference predictor's torch.amp.autocast, inference/predictors.py:55) through an LDS
// image of the input rows the block's output pixels touch.
//
// The implicit GEMM (conv_pipe16.hip) stages a tap-shifted A tile per (r, s) tap: every input
// pixel crosses L2 -> LDS nine times, and with 64 output channels a 128 x 64 tile does only
// 32 MFMAs per 24 KB staged — these convs ran at 0.18 of their roofline, bound by L2 -> CU
// bytes, not by HBM or the matrix cores.  Here a block of BM consecutive
// output pixels (one m tile of the GEMM view, so the BN statistics partials and the epilogue
// are the implicit GEMM's) stages, once:
//  * the input rows its pixels read — rows R0-1 .. R1+1 of the group's B*H image rows, each
//    with a zero column on either side — as [row][W+2] pixels of 64 channels, the producing
//    layer's pending BN(+ReLU) applied on the way in (bn_relu8, as the implicit GEMM's loader:
//    identical operands);
//  * then, tap by tap (double-buffered), the 64 x 64 weight slice of tap (r, s).
// The A fragment of output pixel (oh, ow) for tap (r, s) is the LDS pixel
// (row - R0 + r, ow + s); a tap that leaves the image vertically (padding, or a neighbouring
// image's row in the flattened row space) reads the zero pixel (row 0, column 0).  Taps, and
// k inside a tap, are accumulated in the implicit GEMM's order: outputs are bit-identical to it.
#include <stdlib.h>

#include "conv_common.h"
#include "conv_epi16.h"

namespace mauv {

namespace {

// LDS pixel slots, (rows + 2) * (W + 2): two blocks per CU with the weight double buffer (FWD
// row images 2 x 9.2 KB, DGRAD column images 2 x 12.3 KB)
template <int MODE>
constexpr int halo_px() { return MODE == FWD ? 472 : 400; }
constexpr int kHp = 72;          // LDS pitch of a weight row, 16-bit words (144 B)
// LDS pixels are 128 B (64 channels, no padding); 16-byte chunk c of pixel p sits in slot
// c ^ ((p >> 1) & 7), which keeps every ds_read_b128 fragment conflict-free for any first pixel
// of its 32-pixel run (each 16-lane group of the b128 read covers all 64 banks once)
__device__ __forceinline__ int hslot(int p, int c) { return p * 64 + 8 * (c ^ ((p >> 1) & 7)); }
constexpr unsigned kOOBh = 0x7ffffff0u;

__device__ __forceinline__ u32x4 hload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}

}  // namespace

// BM = 256: 8 waves of 32 x 64; BM = 128: 4 x 2 waves of 32 x 32 (two blocks per CU either way).
// MODE = DGRAD: dx = the same 3x3 / stride-1 correlation of dy with the taps mirrored
// (dx(ih, iw) += dy(ih + 1 - r, iw + 1 - s) . w[.][r][s][.]), B = w[co][r][s][ci] staged as a
// column image (k = co strided) and read with ds_read_b64_tr_b16, as the implicit GEMM does
template <int MODE, int DT, int BM, bool XBN>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
void conv_halo16(const ConvArgs a) {
  constexpr int NT = 512, BN = 64, C = 64, WGM = BM / 32, WGN = 8 / WGM;
  constexpr int WN = BN / WGN, NI = WN / 32;
  constexpr int WLD = MODE == FWD ? kHp : BN + 32;     // weight image: rows / columns
  constexpr int HALO = halo_px<MODE>() * 64, WB = 64 * WLD;  // 16-bit words
  constexpr int NCH = (halo_px<MODE>() * 8 + NT - 1) / NT;  // 16-byte halo chunks per thread
  __shared__ __attribute__((aligned(16))) u16 smem[HALO + 2 * WB];
  __shared__ float xbn[2 * C];
  u16* halo = smem;
  u16* wbuf = smem + HALO;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN, li = lane & 31, lh = lane >> 5;
  int m0, n0, g;
  conv_block_tile<BM, BN>(a, m0, n0, g);
  const int W = a.W, H = a.H, W2 = W + 2, BH = a.B * H;
  // image rows (flattened over the batch) this tile's pixels lie in: R0 .. R1
  const int R0 = __builtin_amdgcn_readfirstlane(m0 / W);
  const int R1 = __builtin_amdgcn_readfirstlane((min(a.M, m0 + BM) - 1) / W);
  const int nhr = R1 - R0 + 3;                         // LDS rows incl. the two halo rows

  const long long nin = MODE == FWD ? a.B * a.xs_b : (long long)BH * W * C;  // input elements
  const u16* xg = MODE == FWD ? (const u16*)a.x + (long long)g * a.xs_g
                              : (const u16*)a.dy + (long long)g * nin;
  const u16* wg = (const u16*)a.w + (long long)g * a.ws_g;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)xg, (short)0, (int)(nin * 2), 0x00020000);
  // the pending BN: fetched here, put into LDS once the input rows' loads are issued
  float xv[1][2];
  if constexpr (XBN) xbn_fetch(xv, a.xsc + g * C, a.xsh + g * C, C, tid, NT);

  // ---- the input rows: chunk q = (LDS row hr, column iw, channel chunk cq), 8 per pixel ----
  float cs[NI];  // the accumulators' start, loaded here and filled after the weight loads
  acc_shift16(cs, a, n0 + wn * WN, MODE == FWD);
  const unsigned nch = (unsigned)(nhr * W * 8);
  u32x4 v[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const unsigned q = (unsigned)(tid + NT * j);
    const unsigned hr = udiv16(q, a.m16_w), rem = q - hr * (unsigned)(W * 8);
    const int iw = (int)(rem >> 3), cq = (int)(rem & 7);
    const int gr = R0 - 1 + (int)hr;                   // flattened image row b * H + ih
    const unsigned b = udiv16((unsigned)gr, a.m16_h);
    const int ih = gr - (int)b * H;
    const bool ok = (q < nch) & ((unsigned)gr < (unsigned)BH);
    const unsigned off = MODE == FWD
        ? (unsigned)((b * a.xs_b + ih * a.xs_h + iw * a.xs_w + 8 * cq) * 2)
        : (unsigned)(((gr * W + iw) * C + 8 * cq) * 2);
    v[j] = hload(rx, sel_off(ok, off, kOOBh));
  }
  // first weight slice (tap 0): thread -> (row wn_ = tid / 8 of w[.][r][s][.], chunk tid % 8);
  // FWD: row = output channel n (a row image over k = input channels); DGRAD: row = k = output
  // channel co, its 64 input channels n in place (a column image)
  const int wn_ = tid >> 3, wq = tid & 7;
  const u16* wrow = wg + (long long)wn_ * 9 * C + 8 * wq;
  // all nine taps' slices are fetched here, beside the input rows: the tap loop then issues no
  // global loads (an L2 round trip per tap had sat in front of every tap's barrier)
  u32x4 wv[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) wv[t] = *(const u32x4*)(wrow + t * C);
  floatx16 acc[NI];
  {
    floatx16 a0[1][NI];
    acc_start16(a0, cs);
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) acc[ni] = a0[0][ni];
  }
  if constexpr (XBN) {
    xbn_put(xbn, xbn + C, xv, C, tid, NT);
    __syncthreads();  // xbn staged
  }
  const unsigned rfloor = a.xrelu ? 0u : 0x80008000u;
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const unsigned q = (unsigned)(tid + NT * j);
    if (q < nch) {
      const unsigned hr = udiv16(q, a.m16_w), rem = q - hr * (unsigned)(W * 8);
      const int iw = (int)(rem >> 3), cq = (int)(rem & 7);
      u32x4 t = v[j];
      if constexpr (XBN) {
        const int gr = R0 - 1 + (int)hr;
        t = bn_relu8<DT>(t, ldf8(xbn + 8 * cq), ldf8(xbn + C + 8 * cq), rfloor,
                         (unsigned)gr < (unsigned)BH);
      }
      *(u32x4*)(halo + hslot((int)hr * W2 + iw + 1, cq)) = t;
    }
  }
  // the zero columns 0 and W+1 of every LDS row
  for (int q = tid; q < nhr * 16; q += NT) {
    const int hr = q >> 4, side = (q >> 3) & 1, cq = q & 7;
    *(u32x4*)(halo + hslot(hr * W2 + side * (W + 1), cq)) = u32x4{0u, 0u, 0u, 0u};
  }
  *(u32x4*)(wbuf + wn_ * WLD + 8 * wq) = wv[0];

  // ---- this lane's output pixel (row li of its wave's 32-pixel fragment) ----
  const int m = m0 + wm * 32 + li;
  const bool mok = m < a.M;
  const int gr_m = mok ? m / W : R0;
  const int ow = mok ? m - gr_m * W : 0;
  const int oh = gr_m - (gr_m / H) * H;
  const int hb = (gr_m - R0) * W2 + ow;                // LDS pixel of tap (0, 0)
  __syncthreads();

#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int r = MODE == FWD ? t / 3 : 2 - t / 3, s = MODE == FWD ? t % 3 : 2 - t % 3;
    const u16* wb = wbuf + (t & 1) * WB;
    const int pix = (mok & ((unsigned)(oh + r - 1) < (unsigned)H)) ? hb + r * W2 + s : 0;
    const u16* ap = halo + pix * 64;
    const int sw = (pix >> 1) & 7;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const u32x4 af = *(const u32x4*)(ap + 8 * ((2 * ks + lh) ^ sw));
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        u32x4 bq;
        if constexpr (MODE == FWD) bq = row_frag_ld<kHp>(wb, wn * WN + ni * 32, ks, li, lh);
        else bq = col_frag(wb, WLD, wn * WN + ni * 32, ks, lane);
        acc[ni] = H16<DT>::mfma(af, bq, acc[ni]);
      }
    }
    if (t < 8) *(u32x4*)(wbuf + ((t + 1) & 1) * WB + wn_ * WLD + 8 * wq) = wv[t + 1];
    __syncthreads();
  }

  floatx16 acc2[1][NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) acc2[0][ni] = acc[ni];
  epilogue16<MODE, DT, BM, BN, 1, NI, WGM, WGN, (HALO + 2 * WB) * 2>(a, acc2, smem, m0, n0, g);
}

// MauvRoute.halo3 (default on): the 3x3 C = 64 forwards and data gradients take this kernel
static int halo3() { return g_route.halo3; }

// rows of the flattened B*H image rows a BM-pixel tile touches, at most
static int halo_rows(int BM, int W) { return BM % W == 0 ? BM / W : BM / W + 2; }

// true: launched (a = the pipelined kernels' prepared arguments; DGRAD: the stride-1 parity
// class, without the BN-partials epilogue)
bool conv_halo16_launch(int mode, int dt, const ConvArgs& a0, hipStream_t st) {
  if (!halo3()) return false;
  if (a0.R != 3 || a0.S != 3 || a0.stride != 1 || a0.pad != 1 || a0.Cin != 64 || a0.Cout != 64 ||
      a0.N != 64 || a0.cpg || a0.W > 512 || a0.H > 4096 || a0.Ho != a0.H || a0.Wo != a0.W ||
      (long long)a0.B * a0.H >= (1 << 17))
    return false;
  if (mode == FWD) {
    if (a0.xs_c != 1 || a0.xs_w % 8 || a0.xs_h % 8 || a0.xs_b % 8 || a0.xs_g % 8) return false;
    if ((long long)a0.B * a0.xs_b * 2 > 0x7fff0000LL) return false;  // 31-bit buffer offsets
  } else {
    if (mode != DGRAD || a0.bp_p1 || a0.xsc) return false;
    if ((long long)a0.B * a0.H * a0.W * 64 * 2 > 0x7fff0000LL) return false;
  }
  const int cap = mode == FWD ? halo_px<FWD>() : halo_px<DGRAD>();
  int BM = 0;
  if ((halo_rows(256, a0.W) + 2) * (a0.W + 2) <= cap) BM = 256;
  else if ((halo_rows(128, a0.W) + 2) * (a0.W + 2) <= cap) BM = 128;
  if (!BM) return false;
  ConvArgs a = a0;
  a.m16_w = m16_div((unsigned)(a.W * 8));
  a.m16_h = m16_div((unsigned)a.H);
  const dim3 grid(ceil_div(a.M, BM), a.G);
  const bool xb = a.xsc != nullptr;
#define MAUV_HALO_LAUNCH(MD, D, M_, X)                                                       \
  hipLaunchKernelGGL((conv_halo16<MD, D, M_, X>), grid, dim3(512), 0, st, a)
#define MAUV_HALO_DT(MD, D)                                                                   \
  do {                                                                                        \
    if (BM == 256) { if (xb) MAUV_HALO_LAUNCH(MD, D, 256, true); else MAUV_HALO_LAUNCH(MD, D, 256, false); } \
    else { if (xb) MAUV_HALO_LAUNCH(MD, D, 128, true); else MAUV_HALO_LAUNCH(MD, D, 128, false); }          \
  } while (0)
  if (mode == FWD) {
    if (dt == DT_BF16) MAUV_HALO_DT(FWD, DT_BF16);
    else MAUV_HALO_DT(FWD, DT_F16);
  } else {  // no pending BN on a data gradient's input
    if (dt == DT_BF16) {
      if (BM == 256) MAUV_HALO_LAUNCH(DGRAD, DT_BF16, 256, false);
      else MAUV_HALO_LAUNCH(DGRAD, DT_BF16, 128, false);
    } else {
      if (BM == 256) MAUV_HALO_LAUNCH(DGRAD, DT_F16, 256, false);
      else MAUV_HALO_LAUNCH(DGRAD, DT_F16, 128, false);
    }
  }
#undef MAUV_HALO_DT
#undef MAUV_HALO_LAUNCH
  return true;
}

}  // namespace mauv
