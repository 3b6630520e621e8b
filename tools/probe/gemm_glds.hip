// Probe (not product code): a 16-bit grouped GEMM  C[g] = A[g] . B[g]^T  (A [M][K], B [N][K],
// k contiguous: the 1x1-conv forward's operands) on 256-row block tiles whose operands reach LDS
// by LDS-DMA (buffer_load ... lds), to measure what the big-tile structure of
// cdna_hip_programming.md §5 is worth on the trunks' shapes against conv_pipe16 and hipBLASLt.
// LDS images: rows of 64 k (128 B), chunk c of row r in slot c ^ ((r >> 1) & 7) (conflict-free
// ds_read_b128 fragments of v_mfma_f32_32x32x16); the DMA source addresses are permuted so each
// wave-instruction's 1 KiB lands linearly.  The epilogue is conv_pipe16's (epilogue16).
#include "conv_epi16.h"

using namespace mauv;

namespace {

constexpr int BK = 64;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16,
                                           voff, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// NBUF LDS stages; STAGES_AHEAD tiles in flight while computing
template <int BM, int BN, int WGM, int WGN, int DT, int NBUF, bool XT = false>
__global__ __launch_bounds__(64 * WGM * WGN, (WGM * WGN + 3) / 4) void gemm_glds(const ConvArgs a) {
  constexpr int NT = 64 * WGM * WGN, NW = NT / 64;
  constexpr int WM = BM / WGM, WN = BN / WGN, MI = WM / 32, NI = WN / 32;
  constexpr int A_B = BM * 128, B_B = BN * 128, STG = A_B + B_B;
  constexpr int RA = BM / NW, RB = BN / NW;  // rows each wave stages per tile
  constexpr int JA = RA / 8, JB = RB / 8;    // DMA wave-instructions per tile per operand
  static_assert(RA % 8 == 0 && RB % 8 == 0, "8 rows per DMA instruction");
  constexpr int PR = BM / WGM, EPI = PR * (BN + 4) * 4;
  constexpr int LDSB = NBUF * STG > EPI ? NBUF * STG : EPI;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[LDSB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN, li = lane & 31, lh = lane >> 5;
  int m0, n0, g;
  conv_block_tile<BM, BN>(a, m0, n0, g);
  const int M = a.M, N = a.N, K = a.K;
  const u16* Ag = (const u16*)a.x + (long long)g * a.xs_g;
  const u16* Bg = (const u16*)a.w + (long long)g * a.ws_g;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)Ag, (short)0, M * K * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)Bg, (short)0, N * K * 2, 0x00020000);
  // per-lane DMA source offsets (tile k0 = 0): row r = this wave's row (l >> 3) of instruction
  // j, slot l & 7 holds chunk (l & 7) ^ ((r >> 1) & 7)
  unsigned aoff[JA], boff[JB];
#pragma unroll
  for (int j = 0; j < JA; ++j) {
    const int r = wave * RA + 8 * j + (lane >> 3), c = (lane & 7) ^ ((r >> 1) & 7);
    aoff[j] = (m0 + r < M) ? (unsigned)(((m0 + r) * K + 8 * c) * 2) : 0x7ffffff0u;
  }
#pragma unroll
  for (int j = 0; j < JB; ++j) {
    const int r = wave * RB + 8 * j + (lane >> 3), c = (lane & 7) ^ ((r >> 1) & 7);
    boff[j] = (n0 + r < N) ? (unsigned)(((n0 + r) * K + 8 * c) * 2) : 0x7ffffff0u;
  }
  auto issue = [&](int t) {
    unsigned char* As = smem + (t % NBUF) * STG;
    unsigned char* Bs = As + A_B;
    const unsigned kb = (unsigned)(t * BK * 2);
#pragma unroll
    for (int j = 0; j < JA; ++j) dma16(ra, As + (wave * RA + 8 * j) * 128, aoff[j] + kb);
#pragma unroll
    for (int j = 0; j < JB; ++j) dma16(rb, Bs + (wave * RB + 8 * j) * 128, boff[j] + kb);
  };

  floatx16 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  auto frag = [&](const unsigned char* img, int row, int chunk) -> u32x4 {
    return *(const u32x4*)(img + row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4));
  };
  // fragments of k-step s + 1 are read while the MFMAs of k-step s run (two register sets)
  auto compute = [&](int t) {
    const unsigned char* As = smem + (t % NBUF) * STG;
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

  const int nt = K / BK;
  constexpr int J = JA + JB;
#pragma unroll
  for (int t = 0; t < NBUF - 1; ++t)
    if (t < nt) issue(t);
  for (int t = 0; t < nt; ++t) {
    // the buffer tile t + NBUF - 1 goes to was read at t - 1 (a barrier ago)
    if (t + NBUF - 1 < nt) {
      issue(t + NBUF - 1);
      wait_vm<J * (NBUF - 1)>();   // own DMAs of tile t have landed
    } else if (NBUF == 3 && t + 1 < nt) {
      wait_vm<J>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();  // every wave's DMAs of tile t have landed
    asm volatile("" ::: "memory");
    if constexpr (XT) {
      // the producing layer's pending BN + ReLU on the landed A tile, in place in LDS
      unsigned char* As = smem + (t % NBUF) * STG;
#pragma unroll
      for (int j = 0; j < BM * 8 / NT; ++j) {
        const int idx = tid + NT * j, row = idx >> 3, slot = idx & 7;
        const int c = slot ^ ((row >> 1) & 7), ch = t * BK + 8 * c;
        u32x4* p = (u32x4*)(As + idx * 16);
        const floatx8 sc = ldf8(a.xsc + (long long)g * K + ch), sh = ldf8(a.xsh + (long long)g * K + ch);
        *p = bn_relu8<DT>(*p, sc, sh, 0u, m0 + row < M);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    compute(t);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // tile t's buffer is free for the DMA issued next
    asm volatile("" ::: "memory");
  }
  epilogue16<FWD, DT, BM, BN, MI, NI, WGM, WGN, NBUF * STG>(a, acc, smem, m0, n0, g);
}

template <int BM, int BN, int WGM, int WGN, int NBUF, bool XT = false>
void launch(const ConvArgs& a, hipStream_t st) {
  dim3 grid(((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN), a.G);
  hipLaunchKernelGGL((gemm_glds<BM, BN, WGM, WGN, DT_BF16, NBUF, XT>), grid, dim3(64 * WGM * WGN),
                     0, st, a);
}

}  // namespace

// variant: 0 = 256x256 (2x4 waves of 128x64), 2 LDS stages; 1 = 256x128 (4x2 waves of 64x64),
// 2 stages; 2 = 256x128, 3 stages; 3 = 128x128 (4 waves of 64x64), 2 stages; 4 / 5 = 1 / 0 with
// the pending BN + ReLU applied to the landed A tile in LDS (xsc / xsh [G][K])
extern "C" int probe_gemm_glds(int variant, const void* A, const void* B, void* C, int M, int N,
                               int K, int G, const float* xsc, const float* xsh, hipStream_t st) {
  ConvArgs a = {};
  a.xsc = xsc; a.xsh = xsh; a.xrelu = 1;
  a.x = (const float*)A;
  a.w = (const float*)B;
  a.out = (float*)C;
  a.M = M; a.N = N; a.K = K; a.G = G;
  a.xs_g = (long long)M * K;
  a.ws_g = (long long)N * K;
  a.out_sg = (long long)M * N;
  a.xcd_grid = 1;
  if (K % BK || M <= 0 || N <= 0) return -1;
  switch (variant) {
    case 0: launch<256, 256, 2, 4, 2>(a, st); break;
    case 1: launch<256, 128, 4, 2, 2>(a, st); break;
    case 2: launch<256, 128, 4, 2, 3>(a, st); break;
    case 3: launch<128, 128, 2, 2, 2>(a, st); break;
    case 4: launch<256, 128, 4, 2, 2, true>(a, st); break;   // + pending BN + ReLU on A
    case 5: launch<256, 256, 2, 4, 2, true>(a, st); break;
    default: return -2;
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
