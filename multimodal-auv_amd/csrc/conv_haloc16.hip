// 16-bit 3x3 / stride-1 / pad-1 forwards over C = 128 / 256 / 512 channels (the conv2 of the
// layer-2..4 bottlenecks, pending bn1 + ReLU on load) through an LDS image of the input rows,
// one 64-channel chunk at a time — conv_halo16.hip (C = 64) generalised.
//
// The implicit GEMM stages a tap-shifted A tile per (tap, channel chunk): every input pixel is
// loaded and BN-transformed nine times.  Here a block of 128 consecutive output pixels x 128
// output channels walks the input channels in chunks of 64: per chunk it stages, once, the
// input rows its pixels read (+ one halo row each side, a zero column at either end; the
// pending BN applied by bn_relu8 on the way in), then the nine taps' 128 x 64 weight slices
// (double-buffered, the next slice in registers one tap ahead); the next chunk's rows are in
// registers while the current chunk's taps run.  Accumulation order is (chunk, tap, k): it is
// not the implicit GEMM's (tap, chunk, k), so outputs agree with it to fp32 summation order
// (routing is by shape only, MauvRoute.haloc16); the statistics epilogue is epilogue16's.
#include "conv_common.h"
#include "conv_epi16.h"

namespace mauv {

namespace {

constexpr int kHc = 72;        // LDS pitch of a weight row, 16-bit words (144 B)
constexpr int kHcPx = 256;     // LDS pixel slots of one 64-channel image chunk (32 KB)
constexpr int kMaxHcC = 512;   // channels
constexpr unsigned kOOBc = 0x7ffffff0u;
// 128-B pixels (64 channels), 16-byte chunk c of pixel p in slot c ^ ((p >> 1) & 7): every
// ds_read_b128 fragment conflict-free for any first pixel (conv_halo16.hip's layout)
__device__ __forceinline__ int cslot(int p, int c) { return p * 64 + 8 * (c ^ ((p >> 1) & 7)); }
__device__ __forceinline__ u32x4 cload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}

}  // namespace

// MI = 1: 4 x 2 waves of 32 x 64 over a 128-pixel x 128-channel tile (512 threads, the default);
// MI = 2: 2 x 2 waves of 64 x 64 (256 threads: one A and one B fragment read per MFMA instead of
// 1.5, but half the waves to cover LDS and barrier latency: 1-3 % slower over the routed shapes,
// profiles/round5/haloc16_unroll_ab_*.txt).  Two blocks per CU either way.  The per-thread
// global offsets are fixed over the chunks and taps (the chunk / tap part is a scalar offset),
// which keeps the nine unrolled taps within 128 VGPRs (MI = 1).
// MODE = DGRAD: dx = the same 3x3 / stride-1 correlation of dy (C = Cout channels, the image)
// with the taps mirrored; the weight slice of a tap is w[co][r][s][ci] for 64 co (k) x 128 ci
// (n), staged as a column image and read with col_frag (conv_halo16.hip's data gradient).
template <int MODE, int DT, bool XBN, int MI>
__global__ __launch_bounds__(256 * (3 - MI)) __attribute__((amdgpu_waves_per_eu(6 - 2 * MI)))
void conv_haloc16(const ConvArgs a) {
  constexpr int WGM = 4 / MI, WGN = 2, NT = 64 * WGM * WGN, BM = 128, BN = 128, WN = 64, NI = 2;
  constexpr int WM = 32 * MI;
  constexpr int WLD = MODE == FWD ? kHc : BN + 32;  // weight image: rows (FWD) / columns
  constexpr int IMG = kHcPx * 64, WB = (MODE == FWD ? BN : 64) * WLD;  // 16-bit words
  constexpr int NCH = kHcPx * 8 / NT;               // 16-byte image chunks per thread
  constexpr int NWJ = BN * 8 / NT;                  // 16-byte weight chunks per thread and tap
  __shared__ __attribute__((aligned(16))) u16 smem[IMG + 2 * WB];
  __shared__ float xbn[XBN ? 2 * kMaxHcC : 1];
  u16* img = smem;
  u16* wbuf = smem + IMG;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN, li = lane & 31, lh = lane >> 5;
  int m0, n0, g;
  conv_block_tile<BM, BN>(a, m0, n0, g);
  const int C = MODE == FWD ? a.Cin : a.Cout, W = a.W, H = a.H, W2 = W + 2, BH = a.B * H;
  const int R0 = __builtin_amdgcn_readfirstlane(m0 / W);
  const int R1 = __builtin_amdgcn_readfirstlane((min(a.M, m0 + BM) - 1) / W);
  const int nhr = R1 - R0 + 3;  // LDS rows incl. the two halo rows (host-checked: fits kHcPx)

  // the image's source: x (FWD, strided NHWC) or dy (DGRAD, dense [B*H*W][Cout])
  const long long nin = MODE == FWD ? (long long)a.B * a.xs_b : (long long)BH * W * C;
  const u16* xg = MODE == FWD ? (const u16*)a.x + (long long)g * a.xs_g
                              : (const u16*)a.dy + (long long)g * nin;
  const u16* wg = (const u16*)a.w + (long long)g * a.ws_g;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)xg, (short)0, (int)(nin * 2), 0x00020000);
  // the pending BN: fetched here, put into LDS once the first chunk's loads are issued
  constexpr int XJ = XBN ? (kMaxHcC + NT - 1) / NT : 1;
  float xv[XJ][2];
  if constexpr (XBN) xbn_fetch(xv, a.xsc + g * C, a.xsh + g * C, C, tid, NT);
  const unsigned rfloor = a.xrelu ? 0u : 0x80008000u;

  // ---- one 64-channel chunk of the input rows: chunk q = (LDS row hr, column iw, cq) ----
  // Per thread, fixed over the chunks: its NCH 16-byte pieces' input offsets (the chunk's 128 B
  // come as the scalar offset; out-of-image rows and pieces past the image get an offset past
  // the buffer: zeros), LDS slots (-1: no piece) and in-image bits.  cq = tid & 7 for every j.
  const unsigned nch = (unsigned)(nhr * W * 8);
  const int cq = tid & 7;
  unsigned goff[NCH];
  int lslot[NCH];
  unsigned rowok = 0;
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const unsigned q = (unsigned)(tid + NT * j);
    const unsigned hr = udiv16(q, a.m16_w), rem = q - hr * (unsigned)(W * 8);
    const int iw = (int)(rem >> 3);
    const int gr = R0 - 1 + (int)hr;  // flattened image row b * H + ih
    const unsigned b = udiv16((unsigned)gr, a.m16_h);
    const int ih = gr - (int)b * H;
    const bool in = (unsigned)gr < (unsigned)BH;
    const bool ok = (q < nch) & in;
    const unsigned off = MODE == FWD
        ? (unsigned)((b * a.xs_b + ih * a.xs_h + iw * a.xs_w + 8 * cq) * 2)
        : (unsigned)(((gr * W + iw) * C + 8 * cq) * 2);
    goff[j] = sel_off(ok, off, kOOBc);
    lslot[j] = q < nch ? cslot((int)hr * W2 + iw + 1, cq) : -1;
    rowok |= (unsigned)in << j;
  }
  u32x4 v[NCH];
  auto load_img = [&](int cc) {
#pragma unroll
    for (int j = 0; j < NCH; ++j)
      v[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)goff[j],
                                                                             128 * cc, 0));
  };
  auto store_img = [&](int cc) {
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      if (lslot[j] >= 0) {
        u32x4 t = v[j];
        if constexpr (XBN) {
          const int ch = 64 * cc + 8 * cq;
          t = bn_relu8<DT>(t, ldf8(xbn + ch), ldf8(xbn + kMaxHcC + ch), rfloor, (rowok >> j) & 1);
        }
        *(u32x4*)(img + lslot[j]) = t;
      }
    }
  };
  // weight slice of (chunk cc, tap t), (tap, chunk) as the scalar offset.  FWD: rows
  // n0 + (tid >> 3) + NT / 8 j of w[n][r][s][c], channels 64 cc + 8 (tid & 7) .. + 7, as a row
  // image [128][kHc].  DGRAD: rows co = 64 cc + (idx >> 4) of w[co][r][s][ci], input channels
  // n0 + 8 (idx & 15) .. + 7 (idx = tid + NT j), as a column image [64 k][BN + 32].
  const int wr = MODE == FWD ? tid >> 3 : tid >> 4, wq = MODE == FWD ? tid & 7 : tid & 15;
  constexpr int WRS = MODE == FWD ? NT / 8 : NT / 16;  // rows per j
  const int wstride = MODE == FWD ? 9 * C : 9 * a.N;  // elements between weight rows
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)wg, (short)0, (int)((long long)a.N * 9 * (MODE == FWD ? C : a.Cout) * 2),
      0x00020000);
  unsigned woff[NWJ];
#pragma unroll
  for (int j = 0; j < NWJ; ++j) {
    const int row = wr + WRS * j;
    if constexpr (MODE == FWD)
      woff[j] = sel_off(n0 + row < a.N, (unsigned)(((n0 + row) * wstride + 8 * wq) * 2), kOOBc);
    else
      woff[j] = (unsigned)((row * wstride + n0 + 8 * wq) * 2);
  }
  u32x4 wv[NWJ];
  auto load_w = [&](int cc, int t) {
    const int so = MODE == FWD ? (t * C + 64 * cc) * 2 : (64 * cc * 9 * a.N + t * a.N) * 2;
#pragma unroll
    for (int j = 0; j < NWJ; ++j)
      wv[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            rw, (int)woff[j], so, 0));
  };
  auto store_w = [&](int buf) {
#pragma unroll
    for (int j = 0; j < NWJ; ++j)
      *(u32x4*)(wbuf + buf * WB + (wr + WRS * j) * WLD + 8 * wq) = wv[j];
  };

  // the zero columns 0 and W + 1 of every LDS row (no chunk writes them)
  for (int q = tid; q < nhr * 16; q += NT) {
    const int hr = q >> 4, side = (q >> 3) & 1, cq = q & 7;
    *(u32x4*)(img + cslot(hr * W2 + side * (W + 1), cq)) = u32x4{0u, 0u, 0u, 0u};
  }
  float cs[NI];  // the accumulators' start, loaded first and filled after the first tile loads
  acc_shift16(cs, a, n0 + wn * WN, MODE == FWD);
  load_img(0);
  load_w(0, 0);
  floatx16 acc[MI][NI];
  acc_start16(acc, cs);
  if constexpr (XBN) {
    xbn_put(xbn, xbn + kMaxHcC, xv, C, tid, NT);
    __syncthreads();  // xbn staged
  }
  store_img(0);
  store_w(0);
  const int nchunk = C / 64;
  if (nchunk > 1) load_img(1);
  load_w(0, 1);

  // ---- this lane's output pixels (row li of each of its wave's 32-pixel fragments) ----
  int hb[MI], ohs[MI];
  bool mok[MI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
    const int m = m0 + wm * WM + mi * 32 + li;
    mok[mi] = m < a.M;
    const int gr_m = mok[mi] ? m / W : R0;
    const int ow = mok[mi] ? m - gr_m * W : 0;
    ohs[mi] = gr_m - (gr_m / H) * H;
    hb[mi] = (gr_m - R0) * W2 + ow;  // LDS pixel of tap (0, 0)
  }
  __syncthreads();

  int wb = 0;  // weight buffer of the current tap
  for (int cc = 0; cc < nchunk; ++cc) {
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      // the image pixel of tap t (DGRAD: mirrored; the weight slice is tap t's)
      const int r = MODE == FWD ? t / 3 : 2 - t / 3, s = MODE == FWD ? t % 3 : 2 - t % 3;
      const u16* wcur = wbuf + wb * WB;
      const u16* ap[MI];
      int sw[MI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int pix = (mok[mi] & ((unsigned)(ohs[mi] + r - 1) < (unsigned)H)) ? hb[mi] + r * W2 + s
                                                                                : 0;
        ap[mi] = img + pix * 64;
        sw[mi] = (pix >> 1) & 7;
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        u32x4 af[MI], bq[NI];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) af[mi] = *(const u32x4*)(ap[mi] + 8 * ((2 * ks + lh) ^ sw[mi]));
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          if constexpr (MODE == FWD) bq[ni] = row_frag_ld<kHc>(wcur, wn * WN + ni * 32, ks, li, lh);
          else bq[ni] = col_frag(wcur, WLD, wn * WN + ni * 32, ks, lane);
        }
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = H16<DT>::mfma(af[mi], bq[ni], acc[mi][ni]);
      }
      // the next tap's slice (chunk cc, tap t + 1; or chunk cc + 1, tap 0) into the other buffer
      const bool more = t < 8 || cc + 1 < nchunk;
      if (more) store_w(wb ^ 1);
      if (t < 8) {
        if (t + 2 < 9) load_w(cc, t + 2);
        else if (cc + 1 < nchunk) load_w(cc + 1, 0);
      } else if (cc + 1 < nchunk) {
        load_w(cc + 1, 1);
      }
      if (t == 8 && cc + 1 < nchunk) {
        __syncthreads();  // every wave is done with this chunk's image
        store_img(cc + 1);
        if (cc + 2 < nchunk) load_img(cc + 2);
      }
      __syncthreads();
      wb ^= 1;
    }
  }

  epilogue16<MODE, DT, BM, BN, MI, NI, WGM, WGN, (IMG + 2 * WB) * 2>(a, acc, smem, m0, n0, g);
}

// rows of the flattened B*H image rows a 128-pixel tile touches, at most
static int haloc_rows(int W) { return 128 % W == 0 ? 128 / W : 128 / W + 2; }

// MauvRoute.haloc16: 1 (default) routes the covered forwards and data gradients here (32 x 64
// wave tiles, 512 threads), 2 the same with 64 x 64 wave tiles (256 threads; measured 1-3 %
// slower), 3 the forwards only (32 x 64), 0 neither (the implicit GEMM)

// true: launched.  FWD: the pending BN (xsc) on load; DGRAD: the stride-1 data gradient
// without the BN-partials epilogue (addend / accumulate / mask forms through epilogue16)
bool conv_haloc16_launch(int mode, int dt, const ConvArgs& a0, hipStream_t st) {
  const int route = g_route.haloc16;
  if (!route || (mode == DGRAD && route == 3)) return false;
  const int C = mode == FWD ? a0.Cin : a0.Cout;  // the image's channels
  if (a0.R != 3 || a0.S != 3 || a0.stride != 1 || a0.pad != 1 || a0.cpg || a0.Ho != a0.H ||
      a0.Wo != a0.W || C % 64 || C < 128 || C > kMaxHcC || a0.N % 128 || a0.W > 512 ||
      a0.H > 4096 || (long long)a0.B * a0.H >= (1 << 17))
    return false;
  if (mode == FWD) {
    if (a0.xs_c != 1 || a0.xs_w % 8 || a0.xs_h % 8 || a0.xs_b % 8 || a0.xs_g % 8) return false;
    if ((long long)a0.B * a0.xs_b * 2 > 0x7fff0000LL) return false;  // 31-bit buffer offsets
  } else {
    // the torchvision bottleneck's stride-1 3x3 maps C -> C (the only form the tests cover)
    if (mode != DGRAD || a0.bp_p1 || a0.xsc || a0.Cin != a0.Cout) return false;
    if ((long long)a0.B * a0.H * a0.W * C * 2 > 0x7fff0000LL) return false;
  }
  if ((long long)a0.N * 9 * C * 2 > 0x7fff0000LL) return false;
  if ((haloc_rows(a0.W) + 2) * (a0.W + 2) > kHcPx) return false;
  ConvArgs a = a0;
  a.m16_w = m16_div((unsigned)(a.W * 8));
  a.m16_h = m16_div((unsigned)a.H);
  const dim3 grid(ceil_div(a.M, 128) * (a.N / 128), a.G);
  const bool xb = a.xsc != nullptr;
#define HC_GO(MD, D, X, MI_) \
  hipLaunchKernelGGL((conv_haloc16<MD, D, X, MI_>), grid, dim3(256 * (3 - MI_)), 0, st, a)
#define HC_MI(MD, D, X) \
  if (route == 2) HC_GO(MD, D, X, 2); \
  else HC_GO(MD, D, X, 1)
  if (mode == FWD) {
    if (dt == DT_BF16) {
      if (xb) HC_MI(FWD, DT_BF16, true);
      else HC_MI(FWD, DT_BF16, false);
    } else {
      if (xb) HC_MI(FWD, DT_F16, true);
      else HC_MI(FWD, DT_F16, false);
    }
  } else {  // no pending BN on a data gradient's input
    if (dt == DT_BF16) HC_MI(DGRAD, DT_BF16, false);
    else HC_MI(DGRAD, DT_F16, false);
  }
#undef HC_MI
#undef HC_GO
  return true;
}

}  // namespace mauv
