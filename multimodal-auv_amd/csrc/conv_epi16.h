// Epilogue of the 16-bit implicit-GEMM convs (conv_pipe16.hip) for FWD and
// DGRAD: BN statistics partials of y from the fp32 accumulators (tile mean, then M2 around it;
// FWD with st_mean), then the 16-bit output through LDS as 16-byte row chunks (DGRAD: residual
// addend / previous dx added in fp32, one rounding; parity-class row remap).  acc[MI][NI] are
// this wave's 32 x 32 accumulator tiles (C/D layout of v_mfma_f32_32x32x16: lane l = column
// l & 31, register r = row (r & 3) + 8 (r >> 2) + 4 (l >> 5)); waves wave = wm * WGN + wn.
// The caller's main loop ended with a barrier: the LDS (SCRATCH bytes) is free.
#pragma once
#include "conv_common.h"

namespace mauv {

template <int DT>
__device__ __forceinline__ unsigned pk2(float a, float b) {
  if constexpr (DT == DT_BF16) {
    return pk_bf16(a, b);
  } else {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 v = {(_Float16)a, (_Float16)b};
    return __builtin_bit_cast(unsigned, v);
  }
}

// The producing layer's pending BN(+ReLU) on one 8-channel chunk: fp32 fma per element, one
// round-to-nearest-even, then ReLU on the packed words as a signed-int16 max against `floor`
// (0 with ReLU: both formats keep the sign in bit 15, so exactly the negative values and -0
// become +0; 0x80008000 without).  Chunks outside the image (padding, ragged rows) become 0.
template <int DT>
__device__ __forceinline__ u32x4 bn_relu8(u32x4 v, const floatx8& sc, const floatx8& sh,
                                          unsigned floor, bool ok) {
  typedef short s2 __attribute__((ext_vector_type(2)));
  u32x4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float lo, hi;
    if constexpr (DT == DT_BF16) {
      lo = bf_lo(v[i]);
      hi = bf_hi(v[i]);
    } else {
      lo = (float)__builtin_bit_cast(_Float16, (u16)(v[i] & 0xffffu));
      hi = (float)__builtin_bit_cast(_Float16, (u16)(v[i] >> 16));
    }
    unsigned p = pk2<DT>(__builtin_fmaf(lo, sc[2 * i], sh[2 * i]),
                         __builtin_fmaf(hi, sc[2 * i + 1], sh[2 * i + 1]));
    asm("" : "+v"(p));  // keeps one v_cvt_pk per pair (else: two single conversions + v_perm)
    const s2 m = __builtin_elementwise_max(__builtin_bit_cast(s2, p), __builtin_bit_cast(s2, floor));
    o[i] = ok ? __builtin_bit_cast(unsigned, m) : 0u;
  }
  return o;
}

template <int MODE, int DT, int BM, int BN, int MI, int NI, int WGM, int WGN, int SCRATCH>
__device__ __forceinline__ void epilogue16(const ConvArgs& a, floatx16 (&acc)[MI][NI], void* smem,
                                           int m0, int n0, int g) {
  constexpr int NT = 64 * WGM * WGN, WM = BM / WGM, WN = BN / WGN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN, li = lane & 31, lh = lane >> 5;
  float* red = (float*)smem;  // LDS is free: the main loop ended with a barrier
  if (MODE == FWD && a.st_mean) {
    // per-tile BN statistics of y from the fp32 accumulators (tile mean, then M2 around it)
    const int nvalid = min(BM, a.M - m0);
    const int tcol = wn * WN + li;
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
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) s1[ni] += __shfl_xor(s1[ni], 32, 64);
    if (lh == 0) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) red[wm * BN + tcol + ni * 32] = s1[ni];
    }
    __syncthreads();
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < WGM; ++w) t += red[w * BN + tcol + ni * 32];
      mean[ni] = t / (float)nvalid;
    }
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
      for (int ni = 0; ni < NI; ++ni) red[WGM * BN + wm * BN + tcol + ni * 32] = s2[ni];
    }
    __syncthreads();
    if (tid < BN && n0 + tid < a.N) {
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int w = 0; w < WGM; ++w) { t1 += red[w * BN + tid]; t2 += red[WGM * BN + w * BN + tid]; }
      const int mt = m0 / BM;
      const int col = n0 + tid;
      const int gc = a.cpg ? col / a.cpg : g, cc = a.cpg ? col % a.cpg : col;
      const long long so = ((long long)gc * a.st_nblk + a.st_base + mt) * (a.cpg ? a.cpg : a.N) + cc;
      a.st_mean[so] = t1 / (float)nvalid;
      a.st_m2[so] = t2;
      if (cc == 0) a.st_cnt[(long long)gc * a.st_nblk + a.st_base + mt] = (float)nvalid;
    }
    __syncthreads();  // red is overwritten by the staged store below
  }
  // 16-bit output through LDS: the fp32 accumulators are parked as a row-major [rows][BN+4]
  // tile — the whole block tile at once when it fits the operand buffers (one barrier), else
  // one wave row wm per pass — then every thread writes 16-byte rows of 8 channels (residual
  // addend / previous dx added in fp32, one rounding)
  constexpr int SLD = BN + 4, CPR = BN / 8;
  constexpr int PASSES = BM * SLD * 4 <= SCRATCH ? 1 : WGM, PR = BM / PASSES;
  constexpr int NCH = PR * CPR;
  float* stile = (float*)smem;
  u16* outp = (u16*)a.out;
  const u16* addp = (const u16*)a.addend;
#pragma unroll
  for (int pass = 0; pass < PASSES; ++pass) {
    if (PASSES == 1 || wm == pass) {
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
    for (int c = tid; c < NCH; c += NT) {
      const int rl = c / CPR, cc = c - rl * CPR;
      const int row = m0 + pass * PR + rl, col = n0 + 8 * cc;
      if (row >= a.M || col >= a.N) continue;
      const floatx4 v0 = *(const floatx4*)(stile + rl * SLD + 8 * cc);
      const floatx4 v1 = *(const floatx4*)(stile + rl * SLD + 8 * cc + 4);
      floatx8 f;
#pragma unroll
      for (int e = 0; e < 4; ++e) { f[e] = v0[e]; f[4 + e] = v1[e]; }
      long long orow = row;
      if constexpr (MODE == DGRAD) {
        if (a.stride != 1) {
          const int HW = a.Hc * a.Wc, b = row / HW, rem = row - b * HW;
          const int i = rem / a.Wc, jj = rem - i * a.Wc;
          orow = ((long long)b * a.H + a.stride * i + a.ph) * a.W + a.stride * jj + a.pw;
        }
      }
      const long long o = (long long)g * a.out_sg +
                          (MODE == FWD ? conv_out_index(a, orow, col) : orow * a.N + col);
      if constexpr (MODE == DGRAD) {
        if (addp) f += unpack8<DT>(*(const u32x4*)(addp + o));
        if (a.accumulate) f += unpack8<DT>(*(const u32x4*)(outp + o));
      }
      u32x4 pk;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pk[e] = pk2<DT>(f[2 * e], f[2 * e + 1]);
        asm("" : "+v"(pk[e]));
      }
      *(u32x4*)(outp + o) = pk;
    }
    if (pass + 1 < PASSES) __syncthreads();
  }
}

}  // namespace mauv
