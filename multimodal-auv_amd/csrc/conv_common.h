// Shared pieces of the fp32 implicit-GEMM convs (conv_gemm.hip: exact f32 MFMA and the
// register-staged split path; conv_split.hip: the pipelined split-fp32 kernels): the argument
// block, the BN-on-load transform and the fused epilogue (bias, residual addend / accumulate,
// BN statistics partials of the forward, BN-backward partials of the data gradient).
#pragma once
#include "h16.h"

namespace mauv {

enum { FWD = 0, DGRAD = 1, WGRAD = 2 };

struct ConvArgs {
  int B, H, W, Cin, Ho, Wo, Cout, R, S, stride, pad;
  long long xs_g, xs_b, xs_h, xs_w, xs_c;  // x element strides
  const float* x;
  const float* w;
  long long ws_g;
  const float* dy;  // [G][B*Ho*Wo][Cout]
  float* out;
  long long out_sg;
  const float* bias;
  long long bias_sg;
  const float* addend;
  int accumulate;
  int G, splits, kchunk;
  int M, N, K;  // GEMM dims (per group)
  // DGRAD output-parity class (sub-pixel decomposition): this launch computes dx for the
  // input pixels (stride*i + ph, stride*j + pw) only, whose contributing taps are
  // r = r0 + stride*tr (tr < nr), s = s0 + stride*ts (ts < ns) — no structurally-zero MACs.
  int ph, pw, Hc, Wc, r0, s0, nr, ns;
  // optional per-(group, channel) transform of x on load: x' = [relu](x*xsc + xsh) — the
  // pending BatchNorm(+ReLU) of the producing layer, applied lazily so that layer's
  // normalised activation is never written to HBM (FWD A-loader, WGRAD B-loader)
  const float* xsc;
  const float* xsh;
  int xrelu;
  // FWD with the previous bottleneck's output formed on load (conv_big16 fold, 1x1 only): the
  // A operand is relu(x*xsc + xsh + r), r = rs or rs*rs_sc + rs_sh (rs_sc non-null: the
  // downsample branch's pending BN); the blocks of column tile 0 write it through to fout and,
  // with fmask, its ReLU-mask bits (bn_apply_mask's: bit e of byte o / 8 = stored value > 0)
  const void* rs;
  const float *rs_sc, *rs_sh;
  void* fout;
  unsigned char* fmask;
  // FWD epilogue BN statistics partials [G][st_nblk][N] (+ counts [G][st_nblk])
  float *st_mean, *st_m2, *st_cnt;
  int st_nblk, st_base;
  // 16-bit FWD: the accumulators start at -ysh[channel] (nullable, [N] or [cpg]; the consuming
  // BatchNorm's centre, conv_epi16.h acc_start16), so the stored output and its statistics
  // partials are those of y - ysh: the 16-bit rounding error then scales with |y - ysh| (the
  // batch spread) instead of |y|, which the BN's 1/std amplifies when a channel's mean is
  // large (mauv_bn_stats_finalize takes the same ysh to add it back for the running mean)
  const float* ysh;
  // DGRAD epilogue BN-backward partials [G][bp_nblk][N]: sum dz, sum dz*xhat
  const float *bp_y, *bp_out, *bp_sc, *bp_sh, *bp_mean, *bp_invstd;
  int bp_relu;
  float *bp_p1, *bp_p2;
  int bp_nblk, bp_base;
  const unsigned char* bp_mask;  // DGRAD: the ReLU mask as bn_apply_mask's bits
  // DGRAD: the residual addend is taken where this ReLU mask (bn_apply_mask's bits over the
  // [G][M][N] output) is set, 0 elsewhere: the residual branch's gradient dres = dout * mask
  // of a block output's BN is added without being written as a tensor
  const unsigned char* add_mask;
  // WGRAD pixel -> (b, oh, ow) by multiply-shift division (conv_split.hip): n / d =
  // (n * mg) >> sh for n < 2^31 (mauv::magic_div)
  unsigned long long mg_hw, mg_w;
  int sh_hw, sh_w;
  // WGRAD: n / Wo and n / Ho for n < 2^17 as umulhi(n, m16) (m16 = 0: divisor 1; m16_div)
  unsigned m16_w, m16_h;
  // FWD with the MC groups stacked along N (the stems over shared im2col rows, stem.hip):
  // column n belongs to group n / cpg, channel n % cpg; outputs and BN statistics go to that
  // group's tensors ([G][M][cpg], [G][nblk][cpg]).  0 = off.
  int cpg;
  // block order over the whole grid (1, what every launch sets) or over blockIdx.x only (0): see
// conv_block_tile
  int xcd_grid;
};

// XCD-aware block -> (tile, group / split-K slice) map.  Blocks are dealt round-robin over the 8
// XCDs by their LINEAR id (blockIdx.x + gridDim.x * blockIdx.y; MI355X_MICROARCH.md, workgroup
// dispatch), so blocks l and l + 8 share an L2.  The linear ids of one XCD are given one
// contiguous range of the logical order (tiles m-major within a group / split-K slice, then the
// next slice): the column tiles of one row tile, and all tiles of one weight-gradient slice,
// share an XCD and its L2 instead of being dealt to eight.  xcd_grid = 0 restores the round-1
// order over blockIdx.x only (which puts every group's / slice's tiles on all eight XCDs
// whenever gridDim.x is a multiple of 8, and scatters them when it is not).
template <int BM, int BN>
__device__ __forceinline__ void conv_block_tile(const ConvArgs& a, int& m0, int& n0, int& by) {
  const int nN = (a.N + BN - 1) / BN;
  int L;
  if (a.xcd_grid) {
    const int nx = gridDim.x, tot = nx * gridDim.y;
    const int lin = blockIdx.x + nx * blockIdx.y, xcd = lin & 7, q = tot >> 3, r = tot & 7;
    const int Lg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (lin >> 3);
    by = Lg / nx;
    L = Lg - by * nx;
  } else {
    const int b = blockIdx.x, nwg = gridDim.x, xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
    by = blockIdx.y;
  }
  // block-uniform: keep them in SGPRs (the divisions above expand to VALU code, and a buffer
  // descriptor derived from a VGPR value costs a waterfall loop at every load)
  by = __builtin_amdgcn_readfirstlane(by);
  m0 = __builtin_amdgcn_readfirstlane((L / nN) * BM);
  n0 = __builtin_amdgcn_readfirstlane((L - (L / nN) * nN) * BN);
}


// output element (row, col) of a FWD/DGRAD epilogue, relative to the block's group base
__device__ __forceinline__ long long conv_out_index(const ConvArgs& a, long long orow, int col) {
  if (a.cpg) return (long long)(col / a.cpg) * a.out_sg + orow * a.cpg + col % a.cpg;
  return orow * a.N + col;
}

// q = n / d as (n * m) >> s for every n < 2^31: s = 31 + ceil(log2 d), m = floor(2^s / d) + 1
// (m*d - 2^s lies in (0, d], so the error term n*(m*d - 2^s)/(d*2^s) < 1/d never crosses an
// integer).
inline void magic_div(unsigned d, unsigned long long& m, int& s) {
  int l = 0;
  while ((1ull << l) < d) ++l;
  s = 31 + l;
  m = (unsigned long long)(((unsigned __int128)1 << s) / d) + 1;
}

// q = n / d as umulhi(n, m) with m = floor((2^32 - 1) / d) + 1, exact for n < 2^17 and
// 2 <= d <= 4096 (checked exhaustively, tests/test_abi_host.py); d = 1 -> m = 0 (q = n)
inline unsigned m16_div(unsigned d) { return d <= 1 ? 0u : (unsigned)(0xFFFFFFFFull / d + 1); }
// buffer offset `off` when `ok`, else `oob` (past the descriptor: the load returns 0), as one
// v_cndmask: the empty asm pins `off` to a VGPR computed before the select, so the compiler
// does not move the offset arithmetic under a branch around the load
__device__ __forceinline__ unsigned sel_off(bool ok, unsigned off, unsigned oob) {
  asm("" : "+v"(off));
  return ok ? off : oob;
}
__device__ __forceinline__ unsigned udiv16(unsigned n, unsigned m) {
  return m ? __umulhi(n, m) : n;
}

// A forward whose input exceeds the pipelined kernels' 31-bit buffer offsets (configs[4]'s
// 512 px sonar at B = 256: 2^31 bytes of layer-1 activations per MC group) runs as launches
// over batch chunks: images are independent in a forward, every chunk covers whole 128-row
// tiles (its statistics blocks start at st_base), y rows are written through plain pointers.
// esz: bytes per element.  false: no chunking possible (the caller falls back).
template <class F>
bool conv_fwd_batch_chunks(const ConvArgs& a0, long long lim, int esz, F launch) {
  const long long hw = (long long)a0.Ho * a0.Wo;
  int bc = (int)(lim / a0.xs_b);
  while (bc > 0 && (bc * hw) % 128) --bc;
  if (bc <= 0 || a0.xs_b <= 0) return false;
  for (int b0 = 0; b0 < a0.B; b0 += bc) {
    ConvArgs c = a0;
    c.B = a0.B - b0 < bc ? a0.B - b0 : bc;
    c.M = (int)(c.B * hw);
    c.x = (const float*)((const char*)a0.x + (long long)b0 * a0.xs_b * esz);
    c.out = (float*)((char*)a0.out + (long long)b0 * hw * a0.N * esz);
    c.st_base = a0.st_base + (int)(b0 * hw / 128);
    if (!launch(c)) return false;
  }
  return true;
}

// Launch the pipelined split-fp32 kernel (conv_split.hip) for an fp32 conv; false when the
// problem is outside its vector paths (the caller then runs conv_gemm.hip's kernels).
bool conv_split_launch(int mode, const ConvArgs& a, int oneacc, hipStream_t st);
// pipelined 16-bit kernels (conv_pipe16.hip); x/w/dy/out/addend hold 16-bit data of type dt
// (DT_BF16 / DT_F16), WGRAD out stays fp32 slabs; false: shape not covered
bool conv_pipe16_launch(int mode, int dt, const ConvArgs& a, hipStream_t st);
// 16-bit forwards on 256-row tiles with LDS-DMA operands (conv_big16.hip); false: not covered
bool conv_big16_launch(int dt, const ConvArgs& a, hipStream_t st);
// the same kernel on 128 x 128 tiles of four waves; false: not covered
// the same kernel forming the previous block's output on load (ConvArgs::rs / fout); false:
// shape not covered (nothing launched)
bool conv_big16_fold_launch(int dt, const ConvArgs& a, hipStream_t st);
// 1x1 / stride-1 forwards over K = 64 / 128 / 256 channels into N >= 256 outputs, weight-
// stationary (conv_expand16.hip); false: shape not covered (or MauvRoute.expand16 = 0)
bool conv_expand16_launch(int dt, const ConvArgs& a, hipStream_t st);
// 3x3 / stride-1 forwards and data gradients over 128-512 channels through an LDS image of the
// input (dy) rows, 64 channels at a time (conv_haloc16.hip); false: shape not covered (or
// switched off, MauvRoute.haloc16)
bool conv_haloc16_launch(int mode, int dt, const ConvArgs& a, hipStream_t st);
// 3x3 / stride-1 forwards and data gradients over 64 -> 64 channels through an LDS image of the
// input rows (conv_halo16.hip); false: shape not covered (or MauvRoute.halo3 = 0)
bool conv_halo16_launch(int mode, int dt, const ConvArgs& a, hipStream_t st);

__device__ __forceinline__ floatx4 bn_act(floatx4 v, floatx4 sc, floatx4 sh, int relu) {
  v = v * sc + sh;
  if (relu) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
  }
  return v;
}


// FWD BatchNorm statistics partials of the block tile from the fp32 accumulators (+ bias): the
// statistics half of conv_epilogue (same operations, same partial layout), for the staged
// store of staged_epilogue_f32.  Ends with a barrier (the LDS is free again).
template <int BM, int BN, int MI, int NI, int WGM, int WGN>
__device__ __forceinline__ void fwd_stats_f32(const ConvArgs& a, floatx16 (&acc)[MI][NI],
                                              float* red, int tid, int m0, int n0, int g) {
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int SR = BM > 128 ? 128 : BM, SUB = BM / SR, WPS = WGM / SUB;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN, li = lane & 31, lh = lane >> 5;
  const int sub = wm / WPS;
  float s1[NI], s2[NI];
  const int nvalid = min(SR, a.M - (m0 + sub * SR));
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    s1[ni] = 0.f;
    s2[ni] = 0.f;
    const int col = n0 + wn * WN + ni * 32 + li;
    if (col >= a.N) continue;
    const float bias = a.bias ? a.bias[(long long)g * a.bias_sg + col] : 0.f;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * WM + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row < a.M) s1[ni] += acc[mi][ni][r] + bias;
      }
  }
  const int tcol = wn * WN + li;
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) s1[ni] += __shfl_xor(s1[ni], 32, 64);
  if (lh == 0) {
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) red[wm * BN + tcol + ni * 32] = s1[ni];
  }
  __syncthreads();
  float mean[NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < WPS; ++w) t += red[(sub * WPS + w) * BN + tcol + ni * 32];
    mean[ni] = t / (float)nvalid;
  }
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int col = n0 + wn * WN + ni * 32 + li;
      const float bias = (a.bias && col < a.N) ? a.bias[(long long)g * a.bias_sg + col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * WM + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row < a.M) {
          const float d = acc[mi][ni][r] + bias - mean[ni];
          s2[ni] += d * d;
        }
      }
    }
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) s2[ni] += __shfl_xor(s2[ni], 32, 64);
  if (lh == 0) {
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) red[WGM * BN + wm * BN + tcol + ni * 32] = s2[ni];
  }
  __syncthreads();
  const int col = tid % BN, sb = tid / BN, nv = min(SR, a.M - (m0 + sb * SR));
  if (tid < SUB * BN && n0 + col < a.N && nv > 0) {
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int w = 0; w < WPS; ++w) {
      t1 += red[(sb * WPS + w) * BN + col];
      t2 += red[WGM * BN + (sb * WPS + w) * BN + col];
    }
    const int mt = m0 / SR + sb;
    const int gc = a.cpg ? (n0 + col) / a.cpg : g, cc = a.cpg ? (n0 + col) % a.cpg : n0 + col;
    const int nc = a.cpg ? a.cpg : a.N;
    const long long so = ((long long)gc * a.st_nblk + a.st_base + mt) * nc + cc;
    a.st_mean[so] = t1 / (float)nv;
    a.st_m2[so] = t2;
    if (cc == 0) a.st_cnt[(long long)gc * a.st_nblk + a.st_base + mt] = (float)nv;
  }
  __syncthreads();
}

// fp32 data-gradient epilogue with a residual addend (optionally counted under ReLU-mask bits)
// and / or accumulation into dx: the accumulators are parked in LDS ([rows][BN + 4] floats, the
// whole tile when it fits SCRATCH bytes, else one wave row band per pass) and every thread then
// moves 16-byte row chunks: the addend, its 4 mask bits and the previous dx are fetched into
// registers BEFORE the accumulators are parked (their HBM latency hides behind the LDS round
// trip), added in fp32 and stored as float4.  The direct per-element form (conv_epilogue: one
// 4-byte addend load behind each 1-byte mask load, per element) ran the bench's masked-addend
// data gradients at 1.6-2.3 TB/s.  Requires N % 4 == 0 (host-checked Cin % 4).
// FWD (after fwd_stats_f32): the same 16-byte stores of the output rows (+ bias), for the
// output-heavy short-K forwards (fp32 training step 267.6-267.9 -> 269.8-270.3 triplets/s
// over the data-gradient change alone, same box).
// DGRAD + BP (bp_p1): dx is the output gradient of a BatchNorm (+ReLU); the store loop also
// sums dz = dx * relu-mask and dz * xhat per column (bn_bwd_partial's two sums), with y (and the
// mask bits / the BN's output) fetched beside the addend — one partial per block tile (the
// conv_tile_rows m-tile) instead of a pass over (y, dout).
template <int MODE, int BM, int BN, int MI, int NI, int WGM, int WGN, int SCRATCH, bool BP = false>
__device__ __forceinline__ void staged_epilogue_f32(const ConvArgs& a, floatx16 (&acc)[MI][NI],
                                                    float* stile, int m0, int n0, int g) {
  constexpr int NT = 64 * WGM * WGN, WM = BM / WGM, WN = BN / WGN;
  constexpr int SLD = BN + 4, CPR = BN / 4;
  constexpr int PASSES = BM * SLD * 4 <= SCRATCH ? 1
                         : ((WGM % 2 == 0 && (BM / 2) * SLD * 4 <= SCRATCH) ? 2 : WGM);
  static_assert((BM / PASSES) * SLD * 4 <= SCRATCH && WGM % PASSES == 0, "staged epilogue scratch");
  constexpr int PR = BM / PASSES, NCH = PR * CPR, CPT = (NCH + NT - 1) / NT;
  constexpr int WPP = WGM / PASSES;  // wave rows per pass
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN, li = lane & 31, lh = lane >> 5;
  float* outp = a.out;
  auto chunk = [&](int pass, int c, long long& o) -> bool {
    const int rl = c / CPR, cc = c - rl * CPR;
    const int row = m0 + pass * PR + rl, col = n0 + 4 * cc;
    if (c >= NCH || row >= a.M || col >= a.N) return false;
    long long orow = row;
    if constexpr (MODE == DGRAD) {
      if (a.stride != 1) {  // class-local row -> input pixel
        const int HW = a.Hc * a.Wc, b = row / HW, rem = row - b * HW;
        const int i = rem / a.Wc, jj = rem - i * a.Wc;
        orow = ((long long)b * a.H + a.stride * i + a.ph) * a.W + a.stride * jj + a.pw;
      }
      o = (long long)g * a.out_sg + orow * a.N + col;
    } else {
      o = (long long)g * a.out_sg + conv_out_index(a, orow, col);
    }
    return true;
  };
  // two chunks in flight (a deeper prefetch spills the 128-VGPR budget of the eight-wave tiles)
  constexpr int PFD = 2;
  floatx4 pa[PFD], pd[PFD], py[PFD];
  unsigned pm[PFD], pr[PFD];
  static_assert(!BP || NT % CPR == 0, "BP: each thread keeps one column chunk");
  const bool bst = MODE == DGRAD && BP && a.bp_p1;
  // BP: this thread's column chunk (fixed: NT % CPR == 0) and its BN parameters
  const int bcol = n0 + 4 * (tid % CPR);
  floatx4 b1 = {0.f, 0.f, 0.f, 0.f}, b2 = b1, bmu = b1, bis = b1, bsc = b1, bsh = b1;
  if (bst && bcol < a.N) {
    bmu = *(const floatx4*)(a.bp_mean + (long long)g * a.N + bcol);
    bis = *(const floatx4*)(a.bp_invstd + (long long)g * a.N + bcol);
    if (a.bp_relu && !a.bp_out && !a.bp_mask) {
      bsc = *(const floatx4*)(a.bp_sc + (long long)g * a.N + bcol);
      bsh = *(const floatx4*)(a.bp_sh + (long long)g * a.N + bcol);
    }
  }
  // The prefetch only issues loads: the mask bytes are kept as loaded (shifted at the chunk's
  // use) and the ReLU test on y*scale + shift is made there too — an operation on a loaded value
  // inside the prefetch made every prefetch wait for its own loads (one chunk in flight, not two)
  auto prefetch = [&](int pass, int k) {
    const int q = k % PFD;
    long long o = 0;
    pa[q] = pd[q] = py[q] = floatx4{0.f, 0.f, 0.f, 0.f};
    pm[q] = 0xfffu;   // (all four bits set after any in-byte shift)
    pr[q] = 0xfffu;
    if (MODE == DGRAD && k < CPT && chunk(pass, tid + k * NT, o)) {
      if (a.addend) {
        pa[q] = *(const floatx4*)(a.addend + o);
        if (a.add_mask) pm[q] = a.add_mask[o >> 3];
      }
      if (a.accumulate) pd[q] = *(const floatx4*)(outp + o);
      if (bst) {
        py[q] = *(const floatx4*)(a.bp_y + o);
        if (a.bp_relu) {
          if (a.bp_mask) {
            pr[q] = a.bp_mask[o >> 3];
          } else if (a.bp_out) {  // (the BN's materialised output: rare) tested here
            const floatx4 pre = *(const floatx4*)(a.bp_out + o);
            pr[q] = 0u;
#pragma unroll
            for (int e = 0; e < 4; ++e) pr[q] |= (pre[e] > 0.f ? 1u : 0u) << (e + (o & 7));
          }
        }
      }
    }
  };
#pragma unroll
  for (int pass = 0; pass < PASSES; ++pass) {
#pragma unroll
    for (int k = 0; k < PFD; ++k) prefetch(pass, k);
    if (wm / WPP == pass) {
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            stile[(wm * WM - pass * PR + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * SLD +
                  wn * WN + ni * 32 + li] = acc[mi][ni][r];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int c = tid + k * NT, q = k % PFD;
      long long o;
      if (chunk(pass, c, o)) {
        const int rl = c / CPR, cc = c - rl * CPR;
        floatx4 v = *(const floatx4*)(stile + rl * SLD + 4 * cc);
        if constexpr (MODE == DGRAD) {
          const unsigned sh = (unsigned)(o & 7);   // this chunk's first bit in its mask byte
          const unsigned am = pm[q] >> sh;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if ((am >> e) & 1u) v[e] += pa[q][e];
            v[e] += pd[q][e];
          }
          if (bst) {
            unsigned rm = pr[q] >> sh;
            if (a.bp_relu && !a.bp_mask && !a.bp_out) {
              const floatx4 pre = py[q] * bsc + bsh;
              rm = 0u;
#pragma unroll
              for (int e = 0; e < 4; ++e) rm |= (pre[e] > 0.f ? 1u : 0u) << e;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float dz = (rm >> e) & 1u ? v[e] : 0.f;
              b1[e] += dz;
              b2[e] += dz * (py[q][e] - bmu[e]) * bis[e];
            }
          }
        } else if (a.bias) {
          v += *(const floatx4*)(a.bias + (long long)g * a.bias_sg + n0 + 4 * cc);
        }
        *(floatx4*)(outp + o) = v;
      }
      prefetch(pass, k + PFD);   // (slot q is this chunk's: free)
    }
    if (pass + 1 < PASSES) __syncthreads();
  }
  if (bst) {
    // the NT / CPR threads of a column chunk, through LDS (after the last pass's stile reads)
    constexpr int TPC = NT / CPR;
    float* red = stile;
    __syncthreads();
    *(floatx4*)(red + (tid / CPR) * BN + 4 * (tid % CPR)) = b1;
    *(floatx4*)(red + (TPC + tid / CPR) * BN + 4 * (tid % CPR)) = b2;
    __syncthreads();
    if (tid < 2 * BN) {
      const int col = tid % BN, which = tid / BN;
      if (n0 + col < a.N) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < TPC; ++w) t += red[(which * TPC + w) * BN + col];
        const long long so = ((long long)g * a.bp_nblk + a.bp_base + m0 / BM) * a.N + n0 + col;
        (which ? a.bp_p2 : a.bp_p1)[so] = t;
      }
    }
  }
}

// Epilogue of one BM x BN block tile: acc[mi][ni] holds the fp32 32x32 accumulator tiles of
// this wave (the C/D layout of both v_mfma_f32_32x32x2_f32 and v_mfma_f32_32x32x16_bf16:
// lane l = column l&31, register r = row (r&3) + 8(r>>2) + 4(l>>5)).
// WGM x WGN waves (wave = wm * WGN + wn).  BN statistics partials are per SR = min(BM, 128)
// rows (the conv_tile_rows granularity the host sizes them with), so a 256-row tile writes two.
template <int MODE, int BM, int BN, int MI, int NI, int WGM = 2, int WGN = 2, bool BP = true>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, floatx16 (&acc)[MI][NI],
                                              float* smem, int tid, int m0, int n0, int g,
                                              int sp) {
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int SR = BM > 128 ? 128 : BM, SUB = BM / SR, WPS = WGM / SUB;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int li = lane & 31, lh = lane >> 5;
  const int sub = wm / WPS;
  float* outg;
  if constexpr (MODE == WGRAD)
    outg = a.out + ((long long)sp * a.G + g) * ((long long)a.M * a.N);
  else
    outg = a.out + (long long)g * a.out_sg;
  // Fused BatchNorm reductions (per block tile, per column = channel), written as per-m-tile
  // partials that bn.hip's finalize kernels merge — the standalone statistics passes over y
  // (forward) and over dx (backward) disappear:
  //   FWD   + st_mean: tile-local (count, mean, M2) of y (two register passes, Welford-exact)
  //   DGRAD + bp_p1  : sum dz and sum dz*xhat of the BN whose output gradient this dx is
  //                    (dz = dx * relu-mask; mask/xhat from that BN's y and statistics)
  const bool fst = (MODE == FWD) && a.st_mean;
  const bool bst = (MODE == DGRAD) && BP && a.bp_p1;  // BP = false: compiled out
  float s1[NI], s2[NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) { s1[ni] = 0.f; s2[ni] = 0.f; }
  const int nvalid = min(SR, a.M - (m0 + sub * SR));  // rows of this wave's partial
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int col = n0 + wn * WN + ni * 32 + li;
      if (col >= a.N) continue;
      float bias = 0.f;
      if constexpr (MODE == FWD)
        if (a.bias) bias = a.bias[(long long)g * a.bias_sg + col];
      float bmu = 0.f, bis = 0.f, bsc = 0.f, bsh = 0.f;
      if constexpr (MODE == DGRAD) {
        if (bst) {
          bmu = a.bp_mean[g * a.N + col];
          bis = a.bp_invstd[g * a.N + col];
          if (!a.bp_out && !a.bp_mask) { bsc = a.bp_sc[g * a.N + col]; bsh = a.bp_sh[g * a.N + col]; }
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * WM + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row >= a.M) continue;
        long long orow = row;
        if constexpr (MODE == DGRAD) {  // class-local row -> input pixel
          if (a.stride != 1) {
            const int HW = a.Hc * a.Wc, b = row / HW, rem = row - b * HW;
            const int i = rem / a.Wc, jj = rem - i * a.Wc;
            orow = ((long long)b * a.H + a.stride * i + a.ph) * a.W + a.stride * jj + a.pw;
          }
        }
        const long long o = MODE == FWD ? conv_out_index(a, orow, col) : orow * a.N + col;
        float v = acc[mi][ni][r] + bias;
        if constexpr (MODE == DGRAD) {
          if (a.addend) {
            const long long ao = (long long)g * a.out_sg + o;
            if (!a.add_mask || ((a.add_mask[ao >> 3] >> (ao & 7)) & 1u)) v += a.addend[ao];
          }
          if (a.accumulate) v += outg[o];
          if (bst) {
            const long long go = (long long)g * a.out_sg + o;
            const float yv = a.bp_y[go];
            bool on = true;
            if (a.bp_relu) {
              if (a.bp_mask) on = (a.bp_mask[go >> 3] >> (go & 7)) & 1u;
              else on = (a.bp_out ? a.bp_out[go] : yv * bsc + bsh) > 0.f;
            }
            const float dz = on ? v : 0.f;
            s1[ni] += dz;
            s2[ni] += dz * (yv - bmu) * bis;
          }
        }
        if constexpr (MODE == FWD) s1[ni] += v;
        outg[o] = v;
      }
    }
  if (fst || bst) {
    float* red = smem;  // LDS is free: the main loop ended with a barrier
    const int tcol = wn * WN + li;  // + ni*32
    // column totals of s1 over the block tile: lane halves, then the two wm waves
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) s1[ni] += __shfl_xor(s1[ni], 32, 64);
    if (lh == 0) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) red[wm * BN + tcol + ni * 32] = s1[ni];
    }
    __syncthreads();
    if (fst) {
      // pass 2: M2 around the tile mean
      float mean[NI];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < WPS; ++w) t += red[(sub * WPS + w) * BN + tcol + ni * 32];
        mean[ni] = t / (float)nvalid;
      }
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) s2[ni] = 0.f;
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          const int col = n0 + wn * WN + ni * 32 + li;
          const float bias = (a.bias && col < a.N) ? a.bias[(long long)g * a.bias_sg + col] : 0.f;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = m0 + wm * WM + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            if (row < a.M) {
              const float d = acc[mi][ni][r] + bias - mean[ni];
              s2[ni] += d * d;
            }
          }
        }
    }
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) s2[ni] += __shfl_xor(s2[ni], 32, 64);
    if (lh == 0) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) red[WGM * BN + wm * BN + tcol + ni * 32] = s2[ni];
    }
    __syncthreads();
    const int col = tid % BN, sb = tid / BN, nv = min(SR, a.M - (m0 + sb * SR));
    if (tid < SUB * BN && n0 + col < a.N && nv > 0) {
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int w = 0; w < WPS; ++w) {
        t1 += red[(sb * WPS + w) * BN + col];
        t2 += red[WGM * BN + (sb * WPS + w) * BN + col];
      }
      const int mt = m0 / SR + sb;
      if (fst) {
        const int gc = a.cpg ? (n0 + col) / a.cpg : g, cc = a.cpg ? (n0 + col) % a.cpg : n0 + col;
        const int nc = a.cpg ? a.cpg : a.N;
        const long long so = ((long long)gc * a.st_nblk + a.st_base + mt) * nc + cc;
        a.st_mean[so] = t1 / (float)nv;
        a.st_m2[so] = t2;
        if (cc == 0) a.st_cnt[(long long)gc * a.st_nblk + a.st_base + mt] = (float)nv;
      } else {
        const long long so = ((long long)g * a.bp_nblk + a.bp_base + mt) * a.N + n0 + col;
        a.bp_p1[so] = t1;
        a.bp_p2[so] = t2;
      }
    }
  }
}

// A pending BatchNorm's per-channel scale / shift staged into LDS without stalling the block
// (a staging loop at the top of the kernel waited for its global loads before the first tile
// load was issued: one exposed load latency per block).  xbn_fetch issues branch-free buffer
// loads of channels tid + NT j (beyond n: out of range, 0) into registers; xbn_put writes them to
// LDS once the tile loads are in flight (before the barrier that publishes the staged values).
template <int J>
__device__ __forceinline__ void xbn_fetch(float (&v)[J][2], const float* sc, const float* sh,
                                          int n, int tid, int nt) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)sc, (short)0, 4 * n,
                                                                      0x00020000);
  const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc((void*)sh, (short)0, 4 * n,
                                                                      0x00020000);
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int i = tid + nt * j;
    const int off = i < n ? 4 * i : 0x7ffffff0;
    v[j][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
    v[j][1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rh, off, 0, 0));
  }
}
template <int J>
__device__ __forceinline__ void xbn_put(float* dsc, float* dsh, const float (&v)[J][2], int n,
                                        int tid, int nt) {
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int i = tid + nt * j;
    if (i < n) {
      dsc[i] = v[j][0];
      dsh[i] = v[j][1];
    }
  }
}

}  // namespace mauv
