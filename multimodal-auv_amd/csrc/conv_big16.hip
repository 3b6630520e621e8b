// 16-bit implicit-GEMM forward on 256-row block tiles whose operands reach LDS by LDS-DMA
// (buffer_load ... lds): the long-K forwards of the trunks (layer-2..4 3x3 convs, the 1x1 convs
// over >= 512 channels) in bf16 training (BASELINE configs[2]) and in the f16 MC inference the
// reference predictor runs under torch.amp.autocast (inference/predictors.py:55).
//
// conv_pipe16's 128 x 128 tiles stage operands through registers (load, BN-on-load VALU,
// ds_write) and give each wave 8 MFMAs per barrier (latency-bound, MFMA busy
// <= 0.33).  Here one block of 8 waves owns a 256 x BN tile (BN = 256: waves of 128 x 64, 32
// MFMAs per 64-deep stage; BN = 128: 64 x 64), the DMA of stage t+1 is in flight while stage t
// computes, and the operands never pass through VGPRs:
//  * LDS images of 64-k rows (128 B), chunk c of row r in slot c ^ ((r >> 1) & 7) (every
//    ds_read_b128 fragment of v_mfma_f32_32x32x16 conflict-free); the DMA writes each wave
//    instruction's 1 KiB linearly, so each lane fetches the chunk its slot holds;
//  * A = the im2col rows of x for tap (r, s), channels c0..c0+63 (zero outside the image and
//    past M: the buffer offset is past the descriptor), B = the KRSC weight rows;
//  * the producing layer's pending BN(+ReLU) (XBN) is applied to the landed A tile in place
//    (bn_relu8, the implicit GEMM's transform: identical operands), one extra barrier;
//  * the epilogue is conv_pipe16's (epilogue16: BN statistics from the fp32 accumulators in
//    128-row partials, 16-bit rows through LDS).
// Accumulation order over k is the implicit GEMM's; outputs match it to accumulation order.
#include "conv_common.h"
#include "conv_epi16.h"

namespace mauv {

namespace {

constexpr int BK = 64;
constexpr unsigned kOOBb = 0x7ffffff0u;
constexpr int kMaxXbnB = 512;   // pending-BN input channels staged in LDS
constexpr int kMaxFold = 2048;  // fold: block-output channels whose BN parameters sit in LDS

__device__ __forceinline__ u32x4 bload16(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}

// The block output relu(y*sc + sh + r) of one 8-channel chunk, r = res or res*rsc + rsh (the
// downsample branch's pending BN): bn_apply_rows' fp32 operations (bn.hip: two fmas, one add,
// ReLU, one rounding to the 16-bit format), so the value written through and fed to the MFMAs
// is the one that pass would have stored.  tab = [sc | sh | rsc | rsh] x kMaxFold in LDS.
template <int DT, bool RBN>
__device__ __forceinline__ u32x4 fold8(u32x4 y, u32x4 r, const float* tab, int ch, bool ok) {
  const floatx8 yf = unpack8<DT>(y), rf = unpack8<DT>(r);
  const floatx8 sc = ldf8(tab + ch), sh = ldf8(tab + kMaxFold + ch);
  floatx8 rsc, rsh;
  if constexpr (RBN) {
    rsc = ldf8(tab + 2 * kMaxFold + ch);
    rsh = ldf8(tab + 3 * kMaxFold + ch);
  }
  u32x4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float f[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int k = 2 * i + e;
      float v = __builtin_fmaf(yf[k], sc[k], sh[k]);
      float rv = rf[k];
      if constexpr (RBN) rv = __builtin_fmaf(rv, rsc[k], rsh[k]);
      asm("" : "+v"(v), "+v"(rv));  // no contraction across the add (bn_apply_rows rounds here)
      v = v + rv;
      f[e] = v > 0.f ? v : 0.f;
    }
    const unsigned p = pk2<DT>(f[0], f[1]);
    o[i] = ok ? p : 0u;
  }
  return o;
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16,
                                           voff, 0, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void block_sync() {  // LDS-only barrier: DMAs stay in flight
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrcb(const void* p, long long nelem) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)(nelem * 2), 0x00020000);
}

// 8 waves on 256-row tiles: BN = 256 as 2 x 4 waves of 128 x 64, BN <= 128 as 4 x 2 waves
template <int BN>
struct WavesB {
  static constexpr int M = BN == 256 ? 2 : 4, N = 8 / M;
};

}  // namespace

// RES (fold, 1x1 stride-1 only): 0 = off; 1 = A is relu(x*xsc + xsh + rs) (identity residual),
// 2 = relu(x*xsc + xsh + rs*rs_sc + rs_sh); the column-tile-0 blocks write A through to fout
template <int DT, int BM, int BN, bool XBN, int RES = 0>
__global__ __launch_bounds__(512, 2) void conv_big16(const ConvArgs a) {
  constexpr int NW = 8, NT = 64 * NW;
  constexpr int WGM = WavesB<BN>::M, WGN = WavesB<BN>::N;
  constexpr int WM = BM / WGM, WN = BN / WGN, MI = WM / 32, NI = WN / 32;
  constexpr int A_B = BM * 128, B_B = BN * 128, STG = A_B + B_B;  // bytes
  constexpr int RA = BM / NW, RB = BN / NW, JA = RA / 8, JB = RB / 8, J = JA + JB;
  constexpr bool XF = XBN || RES != 0;  // a transform of the landed A tile
  constexpr int XS = RES ? kMaxFold : kMaxXbnB;  // stride of the parameter tables
  constexpr int XOFF = 2 * STG;
  constexpr int XB = RES ? (RES == 2 ? 4 : 2) * kMaxFold * 4 : (XBN ? 2 * kMaxXbnB * 4 : 0);
  // epilogue16's staging: per wave row (PR rows a pass)
  constexpr int PR = BM / WGM, EPI = PR * (BN + 4) * 4;
  constexpr int LDSB = XOFF + XB > EPI ? XOFF + XB : EPI;
  static_assert(LDSB <= 160 * 1024, "LDS");
  constexpr int TCH = BM * 8 / NT;  // A chunks each thread transforms per stage (XBN)
  // ONE shared array (a second __shared__ object makes hipcc wait vmcnt(0) before ds_reads)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[LDSB];
  float* xbn = (float*)(smem + XOFF);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN, li = lane & 31, lh = lane >> 5;
  int m0, n0, g;
  conv_block_tile<BM, BN>(a, m0, n0, g);
  const u16* xg = (const u16*)a.x + (long long)g * a.xs_g;
  const u16* wg = (const u16*)a.w + (long long)g * a.ws_g;
  const __amdgpu_buffer_rsrc_t ra = rsrcb(xg, (long long)a.B * a.xs_b);
  const __amdgpu_buffer_rsrc_t rb = rsrcb(wg, a.ws_g);
  const int xs_h = (int)a.xs_h, xs_w = (int)a.xs_w, xs_b = (int)a.xs_b;
  const int HW = a.Ho * a.Wo;

  // DMA lanes: row r = wave * R + 8 j + (lane >> 3) of the tile, slot lane & 7 holds chunk
  // c = (lane & 7) ^ ((r >> 1) & 7)
  unsigned abase[JA];
  int ap0[JA], ap1[JA];
#pragma unroll
  for (int j = 0; j < JA; ++j) {
    const int r = wave * RA + 8 * j + (lane >> 3), c = (lane & 7) ^ ((r >> 1) & 7);
    const int m = m0 + r, mm = m < a.M ? m : 0;
    const int b = mm / HW, rem = mm - b * HW, oh = rem / a.Wo, ow = rem - oh * a.Wo;
    const int p0 = oh * a.stride - a.pad, p1 = ow * a.stride - a.pad;
    abase[j] = (unsigned)((b * xs_b + p0 * xs_h + p1 * xs_w + 8 * c) * 2);
    ap0[j] = m < a.M ? p0 : -(1 << 28);
    ap1[j] = p1;
  }
  unsigned bbase[JB];
#pragma unroll
  for (int j = 0; j < JB; ++j) {
    const int r = wave * RB + 8 * j + (lane >> 3), c = (lane & 7) ^ ((r >> 1) & 7);
    bbase[j] = n0 + r < a.N ? (unsigned)(((n0 + r) * a.K + 8 * c) * 2) : kOOBb;
  }
  // XBN transform: this thread's rows (tid >> 3) + 64 i and their input pixel origins
  int tp0[XF ? TCH : 1], tp1[XF ? TCH : 1];
  if constexpr (XF) {
#pragma unroll
    for (int i = 0; i < TCH; ++i) {
      const int m = m0 + (tid >> 3) + (NT / 8) * i, mm = m < a.M ? m : 0;
      const int b = mm / HW, rem = mm - b * HW, oh = rem / a.Wo, ow = rem - oh * a.Wo;
      tp0[i] = m < a.M ? oh * a.stride - a.pad : -(1 << 28);
      tp1[i] = ow * a.stride - a.pad;
    }
  }
  // the parameter tables: fetched here, put into LDS once the first tile's DMAs are issued
  constexpr int XJ = XF ? (XS + NT - 1) / NT : 1;
  float xv[XJ][2], rv[RES == 2 ? XJ : 1][2];
  if constexpr (XF) xbn_fetch(xv, a.xsc + g * a.Cin, a.xsh + g * a.Cin, a.Cin, tid, NT);
  if constexpr (RES == 2) xbn_fetch(rv, a.rs_sc + g * a.Cin, a.rs_sh + g * a.Cin, a.Cin, tid, NT);
  // fold: this thread's residual chunks (the rows / slots it transforms, 1x1: pixel = row) reach
  // registers one stage ahead, issued after the transform that frees them
  u32x4 rres[RES ? TCH : 1];
  unsigned roff[RES ? TCH : 1];
  __amdgpu_buffer_rsrc_t rr = ra;
  if constexpr (RES) {
    rr = rsrcb((const u16*)a.rs + (long long)g * a.xs_g, (long long)a.B * a.xs_b);
#pragma unroll
    for (int i = 0; i < TCH; ++i) {
      const int row = (tid >> 3) + (NT / 8) * i, c = (tid & 7) ^ ((row >> 1) & 7);
      roff[i] = m0 + row < a.M ? (unsigned)(((m0 + row) * a.Cin + 8 * c) * 2) : kOOBb;
    }
  }
  auto load_res = [&](int kc) {
#pragma unroll
    for (int i = 0; i < TCH; ++i) rres[i] = bload16(rr, roff[i] + (unsigned)(kc * 2));
  };

  const int nt = a.K / BK;
  int t_r = 0, t_s = 0, t_c = 0;  // k position of the next stage to issue
  auto issue = [&](int t) {
    unsigned char* As = smem + (t & 1) * STG;
    unsigned char* Bs = As + A_B;
    const unsigned soff = (unsigned)((t_r * xs_h + t_s * xs_w + t_c) * 2);
#pragma unroll
    for (int j = 0; j < JA; ++j) {
      const bool ok = ((unsigned)(ap0[j] + t_r) < (unsigned)a.H) &
                      ((unsigned)(ap1[j] + t_s) < (unsigned)a.W);
      dma16(ra, As + (wave * RA + 8 * j) * 128, sel_off(ok, abase[j] + soff, kOOBb));
    }
    const unsigned koff = (unsigned)(t * BK * 2);
#pragma unroll
    for (int j = 0; j < JB; ++j) dma16(rb, Bs + (wave * RB + 8 * j) * 128, bbase[j] + koff);
    t_c += BK;
    if (t_c >= a.Cin) { t_c = 0; if (++t_s == a.S) { t_s = 0; ++t_r; } }
  };

  floatx16 acc[MI][NI];
  float cs[NI];  // the accumulators' start, loaded here and filled after the first DMAs
  acc_shift16(cs, a, n0 + wn * WN, true);

  auto frag = [&](const unsigned char* img, int row, int chunk) -> u32x4 {
    return *(const u32x4*)(img + row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4));
  };
  // fragments of k-step s + 1 are read while the MFMAs of k-step s run
  auto compute = [&](int t) {
    const unsigned char* As = smem + (t & 1) * STG;
    const unsigned char* Bs = As + A_B;
    u32x4 af[2][MI], bq[2][NI];
    auto rd = [&](int s, int q) {
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) af[q][mi] = frag(As, wm * WM + mi * 32 + li, 2 * s + lh);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) bq[q][ni] = frag(Bs, wn * WN + ni * 32 + li, 2 * s + lh);
    };
    rd(0, 0);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      if (s + 1 < BK / 16) rd(s + 1, (s + 1) & 1);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = H16<DT>::mfma(af[s & 1][mi], bq[s & 1][ni], acc[mi][ni]);
    }
  };

  const unsigned rfloor = a.xrelu ? 0u : 0x80008000u;
  int x_r = 0, x_s = 0, x_c = 0;  // k position of the stage being transformed
  issue(0);
  if constexpr (RES != 0) load_res(0);
  acc_start16(acc, cs);
  if constexpr (XF) xbn_put(xbn, xbn + XS, xv, a.Cin, tid, NT);
  if constexpr (RES == 2) xbn_put(xbn + 2 * XS, xbn + 3 * XS, rv, a.Cin, tid, NT);
  if constexpr (XF) block_sync();  // xbn staged
  for (int t = 0; t < nt; ++t) {
    // tile t + 1 goes to the buffer tile t - 1 was read from (free since the barrier ending t - 1).
    // Fold: issued unconditionally (past the last stage the descriptors return zeros into the
    // idle buffer), so hipcc's own wait for the residual registers counts these DMAs on every
    // path instead of draining them (vmcnt(0)) before the transform
    if (RES != 0 || t + 1 < nt) {
      issue(t + 1);
      wait_vm<J>();   // this wave's DMAs of tile t (and the residual chunks issued before) landed
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();  // every wave's DMAs of tile t have landed
    asm volatile("" ::: "memory");
    if constexpr (XF) {
      unsigned char* As = smem + (t & 1) * STG;
#pragma unroll
      for (int i = 0; i < TCH; ++i) {
        const int idx = tid + NT * i, row = idx >> 3;
        const int c = (idx & 7) ^ ((row >> 1) & 7), ch = x_c + 8 * c;
        const bool ok = ((unsigned)(tp0[i] + x_r) < (unsigned)a.H) &
                        ((unsigned)(tp1[i] + x_s) < (unsigned)a.W);
        u32x4* p = (u32x4*)(As + idx * 16);
        if constexpr (RES != 0) {
          const u32x4 v = fold8<DT, RES == 2>(*p, rres[i], xbn, ch, ok);
          *p = v;
          if (n0 == 0 && m0 + row < a.M) {
            const long long o = (long long)g * a.xs_g + (long long)(m0 + row) * a.Cin + ch;
            *(u32x4*)((u16*)a.fout + o) = v;
            if (a.fmask) {  // ReLU output: a stored value is > 0 exactly when its bits are not 0
              unsigned mb = 0;
#pragma unroll
              for (int e = 0; e < 4; ++e)
                mb |= ((v[e] & 0xffffu) ? 1u : 0u) << (2 * e) | ((v[e] >> 16) ? 1u : 0u) << (2 * e + 1);
              a.fmask[o >> 3] = (unsigned char)mb;
            }
          }
        } else {
          *p = bn_relu8<DT>(*p, ldf8(xbn + ch), ldf8(xbn + kMaxXbnB + ch), rfloor, ok);
        }
      }
      // 1x1: stage t + 1 covers the next 64 channels (past the last: zeros or unused values)
      if constexpr (RES != 0) load_res(x_c + BK);
      x_c += BK;
      if (x_c >= a.Cin) { x_c = 0; if (++x_s == a.S) { x_s = 0; ++x_r; } }
      block_sync();
    }
    compute(t);
    block_sync();  // tile t's buffer is free for the DMA issued next
  }
  if constexpr (RES != 0) {  // the DMAs past the last stage land before the epilogue reuses LDS
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  epilogue16<FWD, DT, BM, BN, MI, NI, WGM, WGN, 2 * STG>(a, acc, smem, m0, n0, g);
}

// true: launched (a = conv_pipe16_launch's prepared FWD arguments)
bool conv_big16_launch(int dt, const ConvArgs& a, hipStream_t st) {
  if (a.cpg || a.Cin % 64 || a.K != a.R * a.S * a.Cin || a.xs_c != 1 || a.xs_w % 8 ||
      a.xs_h % 8 || a.xs_b % 8 || a.xs_g % 8 || (a.xsc && a.Cin > kMaxXbnB))
    return false;
  if ((long long)a.B * a.xs_b * 2 > 0x7fff0000LL || a.ws_g * 2 > 0x7fff0000LL) return false;
  if (a.M <= 64) return false;  // the statistics partials are 128-row (conv_tile_rows)
  const bool xb = a.xsc != nullptr;
  const int BN = a.N >= 256 ? 256 : 128;
  const dim3 grid(ceil_div(a.M, 256) * ceil_div(a.N, BN), a.G);
#define MAUV_BIG_LAUNCH(D, N_, X) \
  hipLaunchKernelGGL((conv_big16<D, 256, N_, X>), grid, dim3(512), 0, st, a)
#define MAUV_BIG_DT(D)                                                             \
  do {                                                                             \
    if (BN == 256) { if (xb) MAUV_BIG_LAUNCH(D, 256, true); else MAUV_BIG_LAUNCH(D, 256, false); } \
    else { if (xb) MAUV_BIG_LAUNCH(D, 128, true); else MAUV_BIG_LAUNCH(D, 128, false); }          \
  } while (0)
  if (dt == DT_BF16) MAUV_BIG_DT(DT_BF16);
  else MAUV_BIG_DT(DT_F16);
#undef MAUV_BIG_DT
#undef MAUV_BIG_LAUNCH
  return true;
}

// true: launched.  a: conv_pipe16_launch-style FWD arguments of a 1x1 / stride-1 conv over a
// contiguous [G][B][H][W][Cin] input, plus xsc / xsh (the block output's BN) and rs (the
// residual, same layout as x), rs_sc / rs_sh (nullable), fout (the block output, same layout).
bool conv_big16_fold_launch(int dt, const ConvArgs& a, hipStream_t st) {
  if (a.cpg || a.R != 1 || a.S != 1 || a.stride != 1 || a.pad != 0 || a.Cin % 64 ||
      a.Cin > kMaxFold || a.K != a.Cin || !a.xsc || !a.xsh || !a.rs || !a.fout)
    return false;
  if (a.xs_c != 1 || a.xs_w != a.Cin || a.xs_h != (long long)a.W * a.Cin ||
      a.xs_b != (long long)a.H * a.W * a.Cin || a.xs_g % 8)
    return false;
  if ((long long)a.B * a.xs_b * 2 > 0x7fff0000LL || a.ws_g * 2 > 0x7fff0000LL) return false;
  if (a.M <= 64) return false;  // the statistics partials are 128-row (conv_tile_rows)
  ConvArgs c = a;
  c.xrelu = 1;
  c.xcd_grid = 1;
  const bool rbn = a.rs_sc != nullptr;
  // 64 output channels (layer 1's conv1): 256 x 64 tiles of 4 x 2 waves (64 x 32), no half-empty
  // B tile or MFMAs on padding columns
  const int BN = a.N >= 256 ? 256 : (a.N > 64 ? 128 : 64);
  const dim3 grid(ceil_div(a.M, 256) * ceil_div(a.N, BN), a.G);
#define MAUV_FOLD_LAUNCH(D, N_, R_) \
  hipLaunchKernelGGL((conv_big16<D, 256, N_, false, R_>), grid, dim3(512), 0, st, c)
#define MAUV_FOLD_DT(D)                                                                  \
  do {                                                                                   \
    if (BN == 256) { if (rbn) MAUV_FOLD_LAUNCH(D, 256, 2); else MAUV_FOLD_LAUNCH(D, 256, 1); } \
    else if (BN == 128) { if (rbn) MAUV_FOLD_LAUNCH(D, 128, 2); else MAUV_FOLD_LAUNCH(D, 128, 1); } \
    else { if (rbn) MAUV_FOLD_LAUNCH(D, 64, 2); else MAUV_FOLD_LAUNCH(D, 64, 1); }            \
  } while (0)
  if (dt == DT_BF16) MAUV_FOLD_DT(DT_BF16);
  else MAUV_FOLD_DT(DT_F16);
#undef MAUV_FOLD_DT
#undef MAUV_FOLD_LAUNCH
  return true;
}

}  // namespace mauv
