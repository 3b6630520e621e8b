// Epilogue of the 16-bit implicit-GEMM convs (conv_pipe16.hip) for FWD and
// DGRAD: BN statistics partials of y from the fp32 accumulators (tile mean, then M2 around it;
// FWD with st_mean), then the 16-bit output through LDS as 16-byte row chunks (DGRAD: residual
// addend / previous dx added in fp32, one rounding; parity-class row remap; with bp_p1 the
// BN-backward partial sums of the BatchNorm whose output gradient dx is).  acc[MI][NI] are
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
    // the fp32 result is pinned before the conversion: one fp32 fma, then one rounding to the
    // 16-bit format (the reference's fp32 BN output cast by autocast) — without the pin hipcc
    // may contract f16 paths into v_fma_mix (one rounding straight to f16), kernel by kernel
    float f0 = __builtin_fmaf(lo, sc[2 * i], sh[2 * i]);
    float f1 = __builtin_fmaf(hi, sc[2 * i + 1], sh[2 * i + 1]);
    asm("" : "+v"(f0), "+v"(f1));
    unsigned p = pk2<DT>(f0, f1);
    asm("" : "+v"(p));  // keeps one v_cvt_pk per pair (else: two single conversions + v_perm)
    const s2 m = __builtin_elementwise_max(__builtin_bit_cast(s2, p), __builtin_bit_cast(s2, floor));
    o[i] = ok ? __builtin_bit_cast(unsigned, m) : 0u;
  }
  return o;
}

// The accumulators' starting value: 0, or - a FWD with centred storage (ConvArgs::ysh) - minus
// the column's centre, so that they hold y - ysh[channel] from the first MFMA on: the stored
// output AND the statistics partials are those of the centred values (mauv_bn_stats_finalize
// adds the centre back for the running mean).  Every 16-bit forward kernel starts its
// accumulators this way with the same C/D column map (lane l -> column col0 + 32 ni + (l & 31)),
// so the kernels stay bit-identical to each other.  col0 = the wave's first output column.
// Two halves, so that the centre's load overlaps the tile loads instead of stalling the block
// (measured: a load-and-wait at the top cost 5-18 % on short-K forwards): acc_shift16 issues one
// branch-free buffer load per column fragment at the top of the kernel (no centre, or a column
// >= N: a zero-length / out-of-range descriptor access, which returns 0); acc_start16 fills the
// accumulators after the prologue's tile loads are issued, where the wait for the centre (the
// oldest load) costs nothing.  0 - c keeps +0 without a centre (the uncentred bits).
template <int NI>
__device__ __forceinline__ void acc_shift16(float (&c)[NI], const ConvArgs& a, int col0, bool fwd) {
  const int li = threadIdx.x & 31;
  const bool on = fwd && a.ysh;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.ysh, (short)0, on ? 4 * (a.cpg ? a.cpg : a.N) : 0, 0x00020000);
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const int col = col0 + ni * 32 + li;
    const int off = col < a.N ? 4 * (a.cpg ? col % a.cpg : col) : 0x7ffffff0;
    c[ni] = on ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0)) : 0.f;
  }
}
template <int MI, int NI>
__device__ __forceinline__ void acc_start16(floatx16 (&acc)[MI][NI], const float (&c)[NI]) {
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const float v = 0.f - c[ni];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = v;
  }
}

// Chan et al.'s merge of two row sets' (count, mean, M2) into the first: the 16-bit forwards'
// statistics partials combine their 64-row halves with exactly these operations
__device__ __forceinline__ void stats_merge(float na, float ma, float qa, float nb, float mb,
                                            float qb, float& mean, float& m2) {
  if (nb > 0.f) {
    const float n = na + nb, d = mb - ma;
    mean = __builtin_fmaf(d, nb / n, ma);
    m2 = __builtin_fmaf(d * d, na * nb / n, qa + qb);
  } else {
    mean = ma;
    m2 = qa;
  }
}

template <int MODE, int DT, int BM, int BN, int MI, int NI, int WGM, int WGN, int SCRATCH,
          bool BP = false>
__device__ __forceinline__ void epilogue16(const ConvArgs& a, floatx16 (&acc)[MI][NI], void* smem,
                                           int m0, int n0, int g) {
  constexpr int NT = 64 * WGM * WGN, WM = BM / WGM, WN = BN / WGN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN, li = lane & 31, lh = lane >> 5;
  float* red = (float*)smem;  // LDS is free: the main loop ended with a barrier
  if (MODE == FWD && a.st_mean) {
    // BN statistics of y from the fp32 accumulators, one partial per SR = min(BM, 128) rows (the
    // granularity the host sizes them with), in the canonical form every 16-bit forward kernel
    // writes (conv_expand16 included, so a shape's statistics do not depend on the kernel that
    // ran it): each 32-row group summed on its own (lane order, then across the wave halves),
    // per 64-row half the mean of its two group sums and M2 around that mean (fma per row),
    // the halves of a partial merged by Chan's formula (stats_merge)
    constexpr int SR = BM > 128 ? 128 : BM, SUB = BM / SR;
    constexpr int VW = WGM * MI, VPS = VW / SUB;  // 32-row groups: of the tile, of a partial
    static_assert(VW % SUB == 0 && VPS % 2 == 0, "whole 64-row halves per statistics partial");
    const int tcol = wn * WN + li;
    float s1[MI][NI], s2[MI][NI], mean[MI][NI];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        s1[mi][ni] = 0.f;
        s2[mi][ni] = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * WM + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (row < a.M) s1[mi][ni] += acc[mi][ni][r];
        }
        s1[mi][ni] += __shfl_xor(s1[mi][ni], 32, 64);
      }
    if (lh == 0) {
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) red[(wm * MI + mi) * BN + tcol + ni * 32] = s1[mi][ni];
    }
    __syncthreads();
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int g0 = (wm * MI + mi) & ~1;  // the first group of this group's 64-row half
      const int nh = max(0, min(64, a.M - (m0 + 32 * g0)));
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        mean[mi][ni] = (red[g0 * BN + tcol + ni * 32] + red[(g0 + 1) * BN + tcol + ni * 32]) /
                       (float)(nh > 0 ? nh : 1);
    }
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * WM + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (row < a.M) {
            const float d = acc[mi][ni][r] - mean[mi][ni];
            s2[mi][ni] = __builtin_fmaf(d, d, s2[mi][ni]);
          }
        }
        s2[mi][ni] += __shfl_xor(s2[mi][ni], 32, 64);
      }
    if (lh == 0) {
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          red[VW * BN + (wm * MI + mi) * BN + tcol + ni * 32] = s2[mi][ni];
    }
    __syncthreads();
    const int col = tid % BN, sb = tid / BN, nv = min(SR, a.M - (m0 + sb * SR));
    if (tid < SUB * BN && n0 + col < a.N && nv > 0) {
      float hn[2], hm[2], hq[2];
#pragma unroll
      for (int h = 0; h < VPS / 2; ++h) {
        const int gA = sb * VPS + 2 * h;
        const int nh = max(0, min(64, a.M - (m0 + 32 * gA)));
        hn[h] = (float)nh;
        hm[h] = (red[gA * BN + col] + red[(gA + 1) * BN + col]) / (float)(nh > 0 ? nh : 1);
        hq[h] = red[VW * BN + gA * BN + col] + red[VW * BN + (gA + 1) * BN + col];
      }
      float mu = hm[0], m2 = hq[0];
      if constexpr (VPS / 2 == 2) stats_merge(hn[0], hm[0], hq[0], hn[1], hm[1], hq[1], mu, m2);
      const int mt = m0 / SR + sb;
      const int cn = n0 + col;
      const int gc = a.cpg ? cn / a.cpg : g, cc = a.cpg ? cn % a.cpg : cn;
      const long long so = ((long long)gc * a.st_nblk + a.st_base + mt) * (a.cpg ? a.cpg : a.N) + cc;
      a.st_mean[so] = mu;
      a.st_m2[so] = m2;
      if (cc == 0) a.st_cnt[(long long)gc * a.st_nblk + a.st_base + mt] = (float)nv;
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
  static_assert(NT % CPR == 0 && 64 % CPR == 0, "a thread keeps one 8-column chunk");
  float* stile = (float*)smem;
  u16* outp = (u16*)a.out;
  const u16* addp = (const u16*)a.addend;
  // DGRAD + bp_p1: this dx is the output gradient of a BatchNorm (+ReLU); the store loop also
  // sums dz = dx * relu-mask and dz * xhat per column (bn_bwd_partial's two sums, bn.hip), from
  // the ROUNDED 16-bit dx the apply pass will read, with y / the mask read as 16-byte chunks
  // beside the store — one per-(m-tile, column) partial instead of a pass over y and dx
  // (BP: the instantiation that carries this path; the plain data gradients compile it out,
  // which keeps them within the short-K kernels' register budget)
  const bool bst = MODE == DGRAD && BP && a.bp_p1;
  const int bcol = n0 + 8 * (tid % CPR);
  floatx8 b1 = {}, b2 = {}, bmu = {}, bis = {}, bsc = {}, bsh = {};
  if (bst && bcol < a.N) {
    bmu = ldf8(a.bp_mean + (long long)g * a.N + bcol);
    bis = ldf8(a.bp_invstd + (long long)g * a.N + bcol);
    if (a.bp_relu && !a.bp_out && !a.bp_mask) {
      bsc = ldf8(a.bp_sc + (long long)g * a.N + bcol);
      bsh = ldf8(a.bp_sh + (long long)g * a.N + bcol);
    }
  }
  // chunk c of pass `pass` -> its output element offset (false: outside the tile)
  auto chunk = [&](int pass, int c, long long& o) -> bool {
    const int rl = c / CPR, cc = c - rl * CPR;
    const int row = m0 + pass * PR + rl, col = n0 + 8 * cc;
    if (row >= a.M || col >= a.N) return false;
    long long orow = row;
    if constexpr (MODE == DGRAD) {
      if (a.stride != 1) {
        const int HW = a.Hc * a.Wc, b = row / HW, rem = row - b * HW;
        const int i = rem / a.Wc, jj = rem - i * a.Wc;
        orow = ((long long)b * a.H + a.stride * i + a.ph) * a.W + a.stride * jj + a.pw;
      }
    }
    o = (long long)g * a.out_sg + (MODE == FWD ? conv_out_index(a, orow, col) : orow * a.N + col);
    return true;
  };
  // DGRAD, one pass: the residual addend, the BN's y and its mask bits are fetched into
  // registers two chunks ahead — the first two BEFORE the accumulators are parked, so their
  // latency hides behind the LDS round trip instead of serialising each chunk's store (a
  // previous dx / the BN's stored output, the rarer forms, are read in the loop; deeper
  // prefetch spills the 128-VGPR budget)
  constexpr bool PF = MODE == DGRAD && PASSES == 1;
  constexpr int CPT = (NCH + NT - 1) / NT, PFD = 2;
  u32x4 pa[PFD], py[PFD];
  unsigned pm[PFD], pam[PFD];
  auto prefetch = [&](int k) {
    long long o;
    const int q = k % PFD;
    pa[q] = py[q] = u32x4{0u, 0u, 0u, 0u};
    pm[q] = pam[q] = 0u;
    if (k < CPT && tid + k * NT < NCH && chunk(0, tid + k * NT, o)) {
      if (addp) pa[q] = *(const u32x4*)(addp + o);
      if (addp && a.add_mask) pam[q] = a.add_mask[o >> 3];
      if (bst) {
        py[q] = *(const u32x4*)((const u16*)a.bp_y + o);
        if (a.bp_mask) pm[q] = a.bp_mask[o >> 3];
      }
    }
  };
  if constexpr (PF) {
#pragma unroll
    for (int k = 0; k < PFD; ++k) prefetch(k);
  }
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
    for (int k = 0; k * NT < NCH; ++k) {
      const int c = tid + k * NT;
      long long o;
      if (c >= NCH || !chunk(pass, c, o)) {
        if constexpr (PF) prefetch(k + PFD);  // (slot k % PFD is this chunk's: free)
        continue;
      }
      const int rl = c / CPR, cc = c - rl * CPR;
      const floatx4 v0 = *(const floatx4*)(stile + rl * SLD + 8 * cc);
      const floatx4 v1 = *(const floatx4*)(stile + rl * SLD + 8 * cc + 4);
      floatx8 f;
#pragma unroll
      for (int e = 0; e < 4; ++e) { f[e] = v0[e]; f[4 + e] = v1[e]; }
      const int kk = k % PFD;
      if constexpr (MODE == DGRAD) {
        if (addp) {
          floatx8 av = unpack8<DT>(PF ? pa[kk] : *(const u32x4*)(addp + o));
          if (a.add_mask) {  // dres = dout * mask of the block output's BN, never stored
            const unsigned m = PF ? pam[kk] : a.add_mask[o >> 3];
#pragma unroll
            for (int e = 0; e < 8; ++e) av[e] = (m >> e) & 1u ? av[e] : 0.f;
          }
          f += av;
        }
        if (a.accumulate) f += unpack8<DT>(*(const u32x4*)(outp + o));
      }
      u32x4 pk;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pk[e] = pk2<DT>(f[2 * e], f[2 * e + 1]);
        asm("" : "+v"(pk[e]));
      }
      *(u32x4*)(outp + o) = pk;
      if (bst) {
        floatx8 dz = unpack8<DT>(pk);
        const floatx8 yv = unpack8<DT>(PF ? py[kk] : *(const u32x4*)((const u16*)a.bp_y + o));
        if (a.bp_relu) {
          if (a.bp_mask) {  // bn_apply_mask's bits: one byte per 8 channels
            const unsigned m = PF ? pm[kk] : a.bp_mask[o >> 3];
#pragma unroll
            for (int e = 0; e < 8; ++e) dz[e] = (m >> e) & 1u ? dz[e] : 0.f;
          } else {
            const floatx8 pre =
                a.bp_out ? unpack8<DT>(*(const u32x4*)((const u16*)a.bp_out + o))
                         : yv * bsc + bsh;
#pragma unroll
            for (int e = 0; e < 8; ++e) dz[e] = pre[e] > 0.f ? dz[e] : 0.f;
          }
        }
        b1 += dz;
        b2 += dz * (yv - bmu) * bis;
      }
      if constexpr (PF) prefetch(k + PFD);
    }
    if (pass + 1 < PASSES) __syncthreads();
  }
  if (bst) {
    // the lanes of a wave that share a column chunk, then the waves, through LDS
#pragma unroll
    for (int off = CPR; off < 64; off *= 2)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        b1[e] += __shfl_xor(b1[e], off, 64);
        b2[e] += __shfl_xor(b2[e], off, 64);
      }
    constexpr int NW = NT / 64;
    static_assert(2 * NW * BN * 4 <= SCRATCH, "bn-backward partials scratch");
    float* red = (float*)smem;
    __syncthreads();  // the last pass's reads of stile are done
    if (lane < CPR) {
      *(floatx4*)(red + wave * BN + 8 * lane) = __builtin_shufflevector(b1, b1, 0, 1, 2, 3);
      *(floatx4*)(red + wave * BN + 8 * lane + 4) = __builtin_shufflevector(b1, b1, 4, 5, 6, 7);
      *(floatx4*)(red + (NW + wave) * BN + 8 * lane) = __builtin_shufflevector(b2, b2, 0, 1, 2, 3);
      *(floatx4*)(red + (NW + wave) * BN + 8 * lane + 4) = __builtin_shufflevector(b2, b2, 4, 5, 6, 7);
    }
    __syncthreads();
    if (tid < 2 * BN) {
      const int col = tid % BN, which = tid / BN;
      if (n0 + col < a.N) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) t += red[(which * NW + w) * BN + col];
        const long long so = ((long long)g * a.bp_nblk + a.bp_base + m0 / BM) * a.N + n0 + col;
        (which ? a.bp_p2 : a.bp_p1)[so] = t;
      }
    }
  }
}

}  // namespace mauv
