// LDS-DMA 16-bit implicit-GEMM convolution for the convs whose operands need no transform on
// the way to the matrix cores: the data gradient of every Bayesian conv (A = the gathered dy
// rows, B = the sampled weights transposed to [R][S][Cin][Cout] so both operands are
// k-contiguous rows) and the forwards over materialised inputs (conv1 / downsample of every
// bottleneck: A = im2col rows of x, B = the KRSC weights).
//
// Why a second kernel beside conv_pipe16.hip: with register staging (global -> VGPR ->
// ds_write) the 16-bit data gradient is LDS-bound — per CU and block stage the ds_write
// transfer (13 cycles per 1 KiB wave-instruction) plus the 32 x 64 wave tiles' fragment reads
// exceed the MFMA time.  Here:
//  * operands move global -> LDS by buffer_load ... lds (LDS-DMA: no VGPR round trip, no
//    ds_write transfer, no staging registers); one wave-instruction lands 1 KiB = 8 rows of one
//    64-deep k slice; out-of-range offsets return 0 (padding, ragged tiles);
//  * the LDS image is the row image [rows][64] with 16-byte k-chunk c of row r in slot
//    c ^ ((r >> 1) & 7) — the swizzle is put on the SOURCE address (the DMA destination is
//    lane-linear), and every ds_read_b128 fragment read is conflict-free;
//  * four waves of 64 x 64 (2 x 2 MFMA 32x32x16 tiles): one fragment read per MFMA (the
//    eight-wave 32 x 64 layout needs 1.5);
//  * two LDS stages (64 KiB, two blocks per CU): the DMA of stage t+1 is in flight while the
//    MFMAs of stage t run; one vmcnt(0) + barrier per stage.
// Epilogue: conv_epi16.h (shared with conv_pipe16.hip).
#include <stdlib.h>

#include "conv_common.h"
#include "conv_epi16.h"

namespace mauv {

namespace {

constexpr unsigned kOOBd = 0x7ffffff0u;  // beyond every descriptor range: the load returns 0

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_d(const void* p, long long nelem) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(nelem * 2), 0x00020000);
}
// one 16-byte LDS-DMA piece per lane: LDS destination = wave-uniform base + 16 * lane
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, unsigned char* lds, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16,
                                           (int)voff, 0, 0, 0);
}

}  // namespace

constexpr int kMaxXbnD = 512;  // ABN: input channels whose pending-BN scale/shift sit in LDS

// ABN (FWD only): x carries the producing layer's pending BN(+ReLU) (conv2 / conv3 of every
// bottleneck): A is register-staged — 16-byte global loads of stage t+1 issued before the MFMAs
// of stage t, the BN applied and the swizzled row image written after them — while B still
// lands by DMA.
template <int MODE, int DT, bool ABN = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
void conv_dma16(const ConvArgs a) {
  constexpr int BM = 128, BN = 128, BK = 64;
  constexpr int WGM = 2, WGN = 2, WM = 64, WN = 64, MI = WM / 32, NI = WN / 32;
  constexpr int ROWB = BK * 2;                        // bytes per LDS row
  constexpr int A_B = BM * ROWB, B_B = BN * ROWB, STG = A_B + B_B;
  constexpr int NBUF = 2, PIECES = BM / 8 / 4;        // DMA pieces per wave per operand (4)
  constexpr int NVA = BM * 8 / 256;                   // ABN: 16-byte A chunks per thread (4)
  static_assert(BM == BN, "one piece schedule for both operands");
  static_assert(!ABN || MODE == FWD, "pending BN on the forward input only");
  __shared__ __attribute__((aligned(16))) unsigned char smem[NBUF * STG + (ABN ? 8 * kMaxXbnD : 0)];
  float* xbn = (float*)(smem + NBUF * STG);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN, li = lane & 31, lh = lane >> 5;
  int m0, n0, g;
  conv_block_tile<BM, BN>(a, m0, n0, g);  // XCD-aware order over the whole grid
  const int nt = a.K / BK;                // host-checked: K % 64 == 0

  const long long ny = (long long)a.B * a.Ho * a.Wo * a.Cout;  // dy elements per group
  const u16* wg = (const u16*)a.w + (long long)g * a.ws_g;
  __amdgpu_buffer_rsrc_t ra;
  if constexpr (MODE == FWD) ra = rsrc_d((const u16*)a.x + (long long)g * a.xs_g, a.B * a.xs_b);
  else ra = rsrc_d((const u16*)a.dy + (long long)g * ny, ny);
  const __amdgpu_buffer_rsrc_t rb = rsrc_d(wg, a.ws_g);
  const int xs_h = (int)a.xs_h, xs_w = (int)a.xs_w, xs_b = (int)a.xs_b;

  // ---- per-lane DMA constants: wave w lands pieces p = w * PIECES + i of each operand; piece
  // p = rows 8p .. 8p+7, lane l -> row 8p + (l >> 3), LDS slot l & 7, which holds k-chunk
  // c = slot ^ ((row >> 1) & 7) of that row ----
  unsigned abase[PIECES], bbase[PIECES];
  int aq0[PIECES], aq1[PIECES];
#pragma unroll
  for (int i = 0; i < PIECES; ++i) {
    const int row = (wave * PIECES + i) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    const int m = m0 + row;
    const bool ok = m < a.M;
    const int mm = ok ? m : 0;
    if constexpr (MODE == FWD) {
      const int HW = a.Ho * a.Wo, b = mm / HW, rem = mm - b * HW;
      const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
      const int p0 = oh * a.stride - a.pad, p1 = ow * a.stride - a.pad;
      abase[i] = (unsigned)((b * xs_b + p0 * xs_h + p1 * xs_w + 8 * c) * 2);
      aq0[i] = ok ? p0 : -(1 << 28);
      aq1[i] = p1;
    } else {
      const int HW = a.Hc * a.Wc, b = mm / HW, rem = mm - b * HW;
      const int i0 = rem / a.Wc, j0 = rem - i0 * a.Wc;
      const int q0 = i0 + (a.ph + a.pad - a.r0) / a.stride;
      const int q1 = j0 + (a.pw + a.pad - a.s0) / a.stride;
      abase[i] = (unsigned)(((b * a.Ho * a.Wo + q0 * a.Wo + q1) * a.Cout + 8 * c) * 2);
      aq0[i] = ok ? q0 : (1 << 28);
      aq1[i] = q1;
    }
    const int n = n0 + row;
    // FWD: weight row n = [R][S][Cin] (k-contiguous); DGRAD: transposed weights, row n = input
    // channel n of tap (r, s): [Cout] contiguous
    bbase[i] = n < a.N ? (unsigned)((MODE == FWD ? n * a.K + 8 * c : n * a.Cout + 8 * c) * 2) : kOOBd;
  }

  // ---- ABN: register-staged A (thread chunk j = row (tid + 256 j) >> 3, k-chunk tid & 7) ----
  unsigned rbase[ABN ? NVA : 1];
  int rq0[ABN ? NVA : 1], rq1[ABN ? NVA : 1];
  const int rc = tid & 7;
  if constexpr (ABN) {
#pragma unroll
    for (int j = 0; j < NVA; ++j) {
      const int row = (tid + 256 * j) >> 3;
      const int m = m0 + row;
      const bool ok = m < a.M;
      const int mm = ok ? m : 0;
      const int HW = a.Ho * a.Wo, b = mm / HW, rem = mm - b * HW;
      const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
      const int p0 = oh * a.stride - a.pad, p1 = ow * a.stride - a.pad;
      rbase[j] = (unsigned)((b * xs_b + p0 * xs_h + p1 * xs_w + 8 * rc) * 2);
      rq0[j] = ok ? p0 : -(1 << 28);
      rq1[j] = p1;
    }
    for (int i = tid; i < a.Cin; i += 256) {
      xbn[i] = a.xsc[g * a.Cin + i];
      xbn[kMaxXbnD + i] = a.xsh[g * a.Cin + i];
    }
  }
  u32x4 areg[ABN ? NVA : 1];
  unsigned aok = 0;
  int a_c = 0;   // input-channel offset of the staged A registers' k slice

  int t_r = 0, t_s = 0, t_c = 0;  // tile-uniform k position (FWD: r, s, cin; DGRAD: tr, ts, cout)
  auto load = [&](int t, int buf) {
    unsigned char* As = smem + buf * STG;
    unsigned char* Bs = As + A_B;
    unsigned soff, boff;
    if constexpr (MODE == FWD) {
      soff = (unsigned)((t_r * xs_h + t_s * xs_w + t_c) * 2);
      boff = (unsigned)(t * BK * 2);
    } else {
      soff = (unsigned)((t_c - (t_r * a.Wo + t_s) * a.Cout) * 2);
      const int r = a.r0 + a.stride * t_r, s = a.s0 + a.stride * t_s;
      boff = (unsigned)(((r * a.S + s) * a.Cin * a.Cout + t_c) * 2);
    }
    if constexpr (ABN) {   // A into registers (BN + the LDS write after the stage's MFMAs)
      aok = 0;
      a_c = t_c;
#pragma unroll
      for (int j = 0; j < NVA; ++j) {
        const bool ok = ((unsigned)(rq0[j] + t_r) < (unsigned)a.H) &
                        ((unsigned)(rq1[j] + t_s) < (unsigned)a.W);
        areg[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                      ra, (int)sel_off(ok, rbase[j] + soff, kOOBd), 0, 0));
        aok |= (unsigned)ok << j;
      }
    } else {
#pragma unroll
      for (int i = 0; i < PIECES; ++i) {
        bool ok;
        if constexpr (MODE == FWD)
          ok = ((unsigned)(aq0[i] + t_r) < (unsigned)a.H) & ((unsigned)(aq1[i] + t_s) < (unsigned)a.W);
        else
          ok = ((unsigned)(aq0[i] - t_r) < (unsigned)a.Ho) & ((unsigned)(aq1[i] - t_s) < (unsigned)a.Wo);
        dma16(ra, As + (wave * PIECES + i) * 1024, sel_off(ok, abase[i] + soff, kOOBd));
      }
    }
#pragma unroll
    for (int i = 0; i < PIECES; ++i)
      dma16(rb, Bs + (wave * PIECES + i) * 1024,
            sel_off(bbase[i] != kOOBd, bbase[i] + boff, kOOBd));
    if constexpr (MODE == FWD) {
      t_c += BK;
      if (t_c >= a.Cin) { t_c = 0; if (++t_s == a.S) { t_s = 0; ++t_r; } }
    } else {
      t_c += BK;
      if (t_c >= a.Cout) { t_c = 0; if (++t_s == a.ns) { t_s = 0; ++t_r; } }
    }
  };

  floatx16 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  // fragment rows wm*64 + mi*32 + li: the swizzle term ((row >> 1) & 7) is (li >> 1) & 7
  const int sw = (li >> 1) & 7;
  auto compute = [&](int buf) {
    const unsigned char* As = smem + buf * STG;
    const unsigned char* Bs = As + A_B;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const int slot = ((2 * s + lh) ^ sw) * 16;
      u32x4 af[MI], bq[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
        af[mi] = *(const u32x4*)(As + (wm * WM + mi * 32 + li) * ROWB + slot);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        bq[ni] = *(const u32x4*)(Bs + (wn * WN + ni * 32 + li) * ROWB + slot);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = H16<DT>::mfma(af[mi], bq[ni], acc[mi][ni]);
    }
  };

  // ABN: the staged A registers -> BN(+ReLU) -> swizzled row image of buffer buf
  const unsigned rfloor = a.xrelu ? 0u : 0x80008000u;
  auto store_a = [&](int buf) {
    if constexpr (ABN) {
      unsigned char* As = smem + buf * STG;
      const floatx8 fsc = ldf8(xbn + a_c + 8 * rc), fsh = ldf8(xbn + kMaxXbnD + a_c + 8 * rc);
#pragma unroll
      for (int j = 0; j < NVA; ++j) {
        const int row = (tid + 256 * j) >> 3;
        *(u32x4*)(As + row * ROWB + ((rc ^ ((row >> 1) & 7)) << 4)) =
            bn_relu8<DT>(areg[j], fsc, fsh, rfloor, (aok >> j) & 1);
      }
    }
  };

  if constexpr (ABN) __syncthreads();   // xbn staged
  load(0, 0);
  store_a(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    if (t + 1 < nt) load(t + 1, (t + 1) & 1);
    compute(t & 1);
    if (t + 1 < nt) store_a((t + 1) & 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of stage t+1 landed
    __syncthreads();                                  // ... and every wave's; stage t read
  }
  epilogue16<MODE, DT, BM, BN, MI, NI, WGM, WGN, NBUF * STG>(a, acc, smem, m0, n0, g);
}

// MAUV_DMA16 (default 1) / mauv_set_dma16: 0 sends these convs to conv_pipe16.hip (A/B); 2 also
// runs the forwards with a pending BN on x (ABN) here
static int g_dma16 = -1;
static int dma16_on() {
  if (g_dma16 < 0) { const char* e = getenv("MAUV_DMA16"); g_dma16 = e ? atoi(e) : 1; }
  return g_dma16;
}

// FWD (no pending BN on x) and DGRAD (w = the RSCK-transposed weights) on 128 x 128 tiles;
// false: the caller takes conv_pipe16.hip
bool conv_dma16_launch(int mode, int dt, const ConvArgs& a0, hipStream_t st) {
  if (!dma16_on() || (mode != FWD && mode != DGRAD)) return false;
  const long long lim = 0x7fff0000LL / 2;
  const long long nx = (long long)a0.B * a0.xs_b, ny = (long long)a0.B * a0.Ho * a0.Wo * a0.Cout;
  if ((mode == FWD ? nx : ny) > lim || a0.ws_g > lim) return false;
  if (conv_tile_rows(a0.M) != 128 || conv_tile_rows(a0.N) != 128 || a0.K <= 0 || a0.K % 64)
    return false;
  if (a0.N % 8) return false;  // the epilogue stores 8-channel rows
  if (mode == FWD) {
    const bool xs8 = a0.xs_w % 8 == 0 && a0.xs_h % 8 == 0 && a0.xs_b % 8 == 0 && a0.xs_g % 8 == 0;
    if (a0.cpg || a0.Cin % 64 || !xs8 || (a0.xsc && (a0.Cin > kMaxXbnD || dma16_on() < 2)))
      return false;
  } else {
    if (a0.Cout % 64 || a0.Cin % 8) return false;
  }
  ConvArgs a = a0;
  a.xcd_grid = conv_xcd_grid();
  dim3 grid(ceil_div(a.M, 128) * ceil_div(a.N, 128), a.G);
  if (mode == FWD && a.xsc) {
    if (dt == DT_BF16) hipLaunchKernelGGL((conv_dma16<FWD, DT_BF16, true>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((conv_dma16<FWD, DT_F16, true>), grid, dim3(256), 0, st, a);
  } else if (mode == FWD) {
    if (dt == DT_BF16) hipLaunchKernelGGL((conv_dma16<FWD, DT_BF16>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((conv_dma16<FWD, DT_F16>), grid, dim3(256), 0, st, a);
  } else {
    if (dt == DT_BF16) hipLaunchKernelGGL((conv_dma16<DGRAD, DT_BF16>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((conv_dma16<DGRAD, DT_F16>), grid, dim3(256), 0, st, a);
  }
  return true;
}

}  // namespace mauv

MAUV_API int mauv_set_dma16(int on) {
  const int prev = mauv::dma16_on();
  if (on >= 0) mauv::g_dma16 = on;
  return prev;
}
