// 16-bit 1x1 / stride-1 forwards over K = 64..256 input channels into N >= 256 outputs: the
// bottleneck expansions (conv3 of layers 1-3, with the pending bn2 + ReLU applied on load; the
// layer-1 downsample) — weight-stationary.
//
// The short-K implicit GEMM (conv_pipe16 SHORT) runs these at 2.0-2.8 TB/s: a 128 x 128 tile of
// eight 32 x 64 waves reads 1.5 ds_read_b128 per MFMA and re-loads + re-transforms its A rows for
// every 128-column tile.  Here a block owns NB = 8 * WN output columns of one
// MC group for its whole life: every wave keeps the MFMA B fragments of its WN columns over the
// full K in registers (K/16 x WN/32 x 16 B per lane, loaded once), and the block walks 64-row
// tiles of the image rows (pairs of them, grid-stride): per tile the A rows are loaded once,
// the pending BN is applied once in registers, written to one of two LDS row images while the
// other is multiplied, each wave reads 2 A fragments per 16-deep k-step for 2 x WN/32 MFMAs
// (0.5-1 read per MFMA), and the epilogue parks the wave's 64 x WN tile as 16-bit words in a
// wave-private LDS region and stores 16-byte rows.  Outputs are bit-identical to conv_pipe16
// (same MFMA chain over k, same rounding), and so are the BN statistics: one partial per 128
// rows as the host sizes them (mauv_conv2d_fwd_stat_blocks), in epilogue16's canonical form —
// each 64-row tile's half partial (32-row group sums, the half's mean, M2 around it) merged
// with the pair's other half by stats_merge.
#include "conv_common.h"
#include "conv_epi16.h"

namespace mauv {

namespace {

constexpr unsigned kOOBx = 0x7ffffff0u;  // past every descriptor range: the load returns 0

__device__ __forceinline__ u32x4 xload16(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}

}  // namespace

// K: input channels (= GEMM K); WN: output columns per wave (eight waves: NB = 8 * WN columns
// per block).  grid (slots, G * N / NB); block (slot, g * ncg + cg) walks row pairs slot,
// slot + slots, ... < npairs.
template <int DT, int K, int WN, bool XBN>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(WN == 32 && K <= 128 ? 4 : 2)))
void conv_expand16(const ConvArgs a, int npairs, int ncg) {
  constexpr int BM = 64, NW = 8, NT = 64 * NW, NI = WN / 32, MI = BM / 32;
  constexpr int KS = K / 16, KQ = K / 8, NVA = BM * KQ / NT;
  constexpr int RLD = K + 8, A_SZ = BM * RLD;  // A row image [64][K + 8] (u16), two of them
  constexpr int PLD = WN + 8, P_SZ = BM * PLD;  // a wave's parked output tile [64][WN + 8]
  constexpr int CPW = BM * WN / 8 / 64;         // 16-byte output chunks per lane per tile
  static_assert(NVA >= 1 && NT % KQ == 0 && CPW >= 1 && MI == 2, "tile geometry");
  constexpr int XS = XBN ? 2 * K : 0;  // the pending BN's scale / shift (floats)
  // + the accumulators' starting values of the block's NW * WN columns (acc_start16's: minus
  // the centre of centred storage, else 0), staged once: the weight fragments leave no
  // registers to hold them across the tile loop
  __shared__ __attribute__((aligned(16))) u16 smem[2 * A_SZ + NW * P_SZ + 2 * XS + 2 * NW * WN];
  float* xbn = (float*)(smem + 2 * A_SZ + NW * P_SZ);
  float* acc0 = (float*)(smem + 2 * A_SZ + NW * P_SZ + 2 * XS);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 31, lh = lane >> 5;
  const int g = blockIdx.y / ncg, cg = blockIdx.y - g * ncg;
  const int nw0 = cg * NW * WN + wave * WN;  // this wave's first output column
  const u16* xg = (const u16*)a.x + (long long)g * a.xs_g;
  const u16* wg = (const u16*)a.w + (long long)g * a.ws_g;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)xg, (short)0, (int)((long long)a.M * K * 2), 0x00020000);

  // B fragments (v_mfma_f32_32x32x16 operand: lane l = column l & 31, k = 16 s + 8 (l >> 5) + j)
  u32x4 bw[KS][NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const u16* wr = wg + (long long)(nw0 + ni * 32 + li) * K + 8 * lh;
#pragma unroll
    for (int s = 0; s < KS; ++s) bw[s][ni] = *(const u32x4*)(wr + 16 * s);
  }
  // this thread's A chunks: rows (tid + NT j) / KQ of a tile, channels 8 kq .. 8 kq + 7
  const int kq = tid % KQ;
  if constexpr (XBN) {  // staged in LDS (read once per tile) rather than held in 16 VGPRs
    for (int c = tid; c < K; c += NT) {
      xbn[c] = a.xsc[g * a.Cin + c];
      xbn[K + c] = a.xsh[g * a.Cin + c];
    }
  }
  for (int c = tid; c < NW * WN; c += NT) {
    const int col = cg * NW * WN + c;
    acc0[c] = a.ysh && col < a.N ? -a.ysh[col] : 0.f;
  }
  __syncthreads();
  const unsigned rfloor = a.xrelu ? 0u : 0x80008000u;

  // tile i of this block: row pair blockIdx.x + (i / 2) * gridDim.x, half i % 2
  const int ntl = 2 * ((npairs - 1 - (int)blockIdx.x) / (int)gridDim.x + 1);
  auto tile_of = [&](int i) { return 2 * ((int)blockIdx.x + (i >> 1) * (int)gridDim.x) + (i & 1); };
  u32x4 va[NVA];
  auto load_a = [&](int t) {
#pragma unroll
    for (int j = 0; j < NVA; ++j) {
      const int row = t * BM + (tid + NT * j) / KQ;
      va[j] = xload16(ra, row < a.M ? (unsigned)((row * K + 8 * kq) * 2) : kOOBx);
    }
  };
  auto store_a = [&](int buf, int t) {
    u16* As = smem + buf * A_SZ;
    floatx8 fsc, fsh;
    if constexpr (XBN) {
      fsc = ldf8(xbn + 8 * kq);
      fsh = ldf8(xbn + K + 8 * kq);
    }
#pragma unroll
    for (int j = 0; j < NVA; ++j) {
      const int r = (tid + NT * j) / KQ;
      u32x4 v = va[j];
      if constexpr (XBN) v = bn_relu8<DT>(v, fsc, fsh, rfloor, t * BM + r < a.M);
      *(u32x4*)(As + r * RLD + 8 * kq) = v;
    }
  };

  load_a(tile_of(0));
  store_a(0, tile_of(0));
  load_a(tile_of(1));
  __syncthreads();

  u16* park = smem + 2 * A_SZ + wave * P_SZ;
  float hn = 0.f, hmean[NI], hm2[NI];  // the pair's first 64-row half: count, mean, M2
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) hmean[ni] = hm2[ni] = 0.f;

  for (int i = 0; i < ntl; ++i) {
    const int t = tile_of(i), buf = i & 1;
    floatx16 acc[MI][NI];
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const float v = acc0[((int)threadIdx.x >> 6) * WN + ni * 32 + ((int)threadIdx.x & 31)];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mi][ni][r] = v;
    }
    const u16* As = smem + buf * A_SZ;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      u32x4 af[MI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) af[mi] = row_frag_ld<RLD>(As, mi * 32, s, li, lh);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = H16<DT>::mfma(af[mi], bw[s][ni], acc[mi][ni]);
    }
    // the next tile's rows into the other image (its last readers passed the previous
    // iteration's barrier), the one after into registers
    if (i + 1 < ntl) {
      store_a(buf ^ 1, tile_of(i + 1));
      if (i + 2 < ntl) load_a(tile_of(i + 2));
    }

    // ---- BN statistics: the 64-row half's partial (epilogue16's canonical form: 32-row group
    // sums, the half's mean, M2 per group around it), merged with the pair's other half ----
    const int nval = min(BM, a.M - t * BM);  // may be <= 0: the second half past M
    if (a.st_mean) {
      float s1[NI], m2[NI];
      if constexpr (K <= 128) {
        // rows past M hold exact zeros (their A rows were loaded and transformed as 0): the
        // sums need no mask; on a partial tile those rows are set to the mean before the M2
        // pass (each then adds an exact 0)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          float sg[MI];
#pragma unroll
          for (int mi = 0; mi < MI; ++mi) {
            float p = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) p += acc[mi][ni][r];
            sg[mi] = p + __shfl_xor(p, 32, 64);
          }
          s1[ni] = (sg[0] + sg[1]) / (float)(nval > 0 ? nval : 1);
        }
        if (nval < BM) {  // block-uniform
          const int lim = nval - 4 * lh;
#pragma unroll
          for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < NI; ++ni)
#pragma unroll
              for (int r = 0; r < 16; ++r)
                if ((r & 3) + 8 * (r >> 2) >= lim - 32 * mi) acc[mi][ni][r] = s1[ni];
        }
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          float qg[MI];
#pragma unroll
          for (int mi = 0; mi < MI; ++mi) {
            float q = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float d = acc[mi][ni][r] - s1[ni];
              q = __builtin_fmaf(d, d, q);
            }
            qg[mi] = q + __shfl_xor(q, 32, 64);
          }
          m2[ni] = qg[0] + qg[1];
        }
      } else {  // measured: the masked form runs the K = 256 kernel (255 VGPRs) 1.5x faster
        const bool full = nval >= BM;
        const int lim = nval - 4 * lh;
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          float sg[MI], qg[MI];
#pragma unroll
          for (int mi = 0; mi < MI; ++mi) {
            float p = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r)
              p += (full || (r & 3) + 8 * (r >> 2) < lim - 32 * mi) ? acc[mi][ni][r] : 0.f;
            sg[mi] = p + __shfl_xor(p, 32, 64);
          }
          s1[ni] = (sg[0] + sg[1]) / (float)(nval > 0 ? nval : 1);
#pragma unroll
          for (int mi = 0; mi < MI; ++mi) {
            float q = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float d = acc[mi][ni][r] - s1[ni];
              q = (full || (r & 3) + 8 * (r >> 2) < lim - 32 * mi) ? __builtin_fmaf(d, d, q) : q;
            }
            qg[mi] = q + __shfl_xor(q, 32, 64);
          }
          m2[ni] = qg[0] + qg[1];
        }
      }
      const float n1 = (float)(nval > 0 ? nval : 0);
      if ((i & 1) == 0) {
        hn = n1;
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) { hmean[ni] = s1[ni]; hm2[ni] = m2[ni]; }
      } else {
        const int pr = t >> 1;
        if (lh == 0) {
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) {
            float mean, M2;
            stats_merge(hn, hmean[ni], hm2[ni], n1, s1[ni], m2[ni], mean, M2);
            const long long so = ((long long)g * a.st_nblk + a.st_base + pr) * a.N + nw0 + ni * 32 + li;
            a.st_mean[so] = mean;
            a.st_m2[so] = M2;
          }
        }
        if (tid == 0 && cg == 0) a.st_cnt[(long long)g * a.st_nblk + a.st_base + pr] = hn + n1;
      }
    }

    // ---- 16-bit output: park the wave's 64 x WN tile, store 16-byte rows ----
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          park[(mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * PLD + ni * 32 + li] =
              H16<DT>::from_f(acc[mi][ni][r]);
    __syncthreads();  // parked tiles and the next A image visible; every wave done with `buf`
    u16* outp = (u16*)a.out + (long long)g * a.out_sg;
#pragma unroll
    for (int q = 0; q < CPW; ++q) {
      const int c = lane + 64 * q, row = c / (WN / 8), cc = c % (WN / 8);
      const int grow = t * BM + row;
      const u32x4 v = *(const u32x4*)(park + row * PLD + 8 * cc);
      if (grow < a.M) *(u32x4*)(outp + (long long)grow * a.N + nw0 + 8 * cc) = v;
    }
  }
}

// MauvRoute.expand16: 1 (default) = the shapes where it measured faster (expand_wins), 2 = every
// shape the kernel covers, 3 = as 2 with 32-column waves for K = 128 (the A/B of §2.28's wave
// width), 0 = none (conv_pipe16's short-K form)

template <int DT, int K, int WN>
static void launch_expand(const ConvArgs& a, hipStream_t st) {
  const int ncg = a.N / (8 * WN), npairs = (a.M + 127) / 128;
  const int units = a.G * ncg;
  int slots = (2 * 256 + units - 1) / units;  // ~two blocks per CU over the grid
  if (slots > npairs) slots = npairs;
  if (slots < 1) slots = 1;
  const dim3 grid(slots, units);
  if (a.xsc) hipLaunchKernelGGL((conv_expand16<DT, K, WN, true>), grid, dim3(512), 0, st, a, npairs, ncg);
  else hipLaunchKernelGGL((conv_expand16<DT, K, WN, false>), grid, dim3(512), 0, st, a, npairs, ncg);
}

template <int DT>
static bool expand_dt(const ConvArgs& a, hipStream_t st) {
  switch (a.K) {
    case 64: launch_expand<DT, 64, 32>(a, st); return true;
    case 128:
      if (g_route.expand16 == 3) launch_expand<DT, 128, 32>(a, st);
      else launch_expand<DT, 128, 64>(a, st);
      return true;
    case 256: launch_expand<DT, 256, 64>(a, st); return true;
  }
  return false;
}

// where it measured faster than the implicit GEMM (tools/expand_ab.py): K = 128
// (1.22-1.32x); K = 256 with >= 8 row pairs per block (1.19-1.20x at the inference chunk; the
// training slice's 2-3 pairs per block do not amortise the 128-register weight fragments:
// 0.84-0.95x); K = 64 never (0.86-0.96x).  Outputs AND statistics are bit-identical to the
// implicit GEMM's (epilogue16's canonical statistics), so a rule that depends on the MC group
// count cannot change a sample's result with the chunk size
static bool expand_wins(const ConvArgs& a) {
  if (a.K == 128) return true;
  if (a.K != 256) return false;
  const int ncg = a.N / 512, units = a.G * ncg, npairs = (a.M + 127) / 128;
  const int slots = (2 * 256 + units - 1) / units;
  return npairs >= 8 * slots;
}

bool conv_expand16_launch(int dt, const ConvArgs& a, hipStream_t st) {
  const int route = g_route.expand16;
  if (!route) return false;
  if (a.R != 1 || a.S != 1 || a.stride != 1 || a.pad != 0 || a.cpg || a.Ho != a.H || a.Wo != a.W)
    return false;
  const int K = a.Cin;
  if (a.K != K || (K != 64 && K != 128 && K != 256)) return false;
  const int NB = 8 * (K == 64 ? 32 : 64);
  if (a.N % NB || a.M <= 0 || a.G > 65535 / (a.N / NB)) return false;
  // dense NHWC rows (a row's K channels contiguous, rows back to back) within 31-bit offsets
  if (a.xs_c != 1 || a.xs_w != K || a.xs_h != (long long)a.W * K ||
      a.xs_b != (long long)a.H * a.W * K || (long long)a.M * K * 2 > 0x7fff0000LL)
    return false;
  if (a.st_mean && (!a.st_m2 || !a.st_cnt)) return false;
  if (route == 1 && !expand_wins(a)) return false;
  return dt == DT_BF16 ? expand_dt<DT_BF16>(a, st) : expand_dt<DT_F16>(a, st);
}

}  // namespace mauv
