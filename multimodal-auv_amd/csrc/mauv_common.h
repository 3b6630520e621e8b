// Common device/host helpers for libmauv_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "mauv.h"  // the C-ABI (include/mauv.h): definitions below must match it

#define MAUV_API extern "C" __attribute__((visibility("default")))

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace mauv {

// Thread-local last error (mauv_last_error()).
void set_error(const std::string& s);

// Launch-status check used by every C-ABI entry point: returns 0 or a negative code.
int check_launch(const char* what);

// Process-wide kernel routing (include/mauv.h MauvRoute): written only by mauv_set_route, read
// by the launchers; the defaults are the measured-fastest routes (capi.cpp).
extern MauvRoute g_route;

constexpr int kErrArg = -1;      // invalid argument / unsupported shape
constexpr int kErrLaunch = -2;   // hipGetLastError() after launch

inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

// Block-tile extent along a GEMM dimension of the implicit-GEMM convs (fp32 and 16-bit):
// 64 when the extent is 64 or less, else 128.  The per-m-tile BN statistics partials the FWD
// epilogues write are counted with the same rule (mauv_conv2d_fwd_stat_blocks).
inline int conv_tile_rows(int extent) { return extent <= 64 ? 64 : 128; }

// ---------------- Philox4x32-10 + Box-Muller (counter-based, recomputable) --------------
// Standard constants (Salmon et al. 2011).  ctr = (quad index, sample lo, layer id,
// sample hi), key = seed.  The oracle restates this bit-exactly in numpy
// (oracle/philox_ref.py) so epsilon streams can be checked integer-exactly.
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = c.x * 0xD2511F53u, hi0 = __umulhi(c.x, 0xD2511F53u);
    const uint32_t lo1 = c.z * 0xCD9E8D57u, hi1 = __umulhi(c.z, 0xCD9E8D57u);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

// Four N(0,1) samples for quad `q` of layer `layer` in MC sample `sample`.
__device__ __forceinline__ floatx4 normal4(uint64_t seed, uint64_t sample, uint32_t layer,
                                           uint32_t q) {
  const uint4 r = philox4x32_10(
      make_uint4(q, (uint32_t)sample, layer, (uint32_t)(sample >> 32)),
      make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  const float k = 2.3283064365386963e-10f;  // 2^-32
  const float u0 = ((float)r.x + 0.5f) * k, u1 = ((float)r.y + 0.5f) * k;
  const float u2 = ((float)r.z + 0.5f) * k, u3 = ((float)r.w + 0.5f) * k;
  const float m0 = sqrtf(-2.0f * logf(u0)), m1 = sqrtf(-2.0f * logf(u2));
  float s0, c0, s1, c1;
  sincospif(2.0f * u1, &s0, &c0);
  sincospif(2.0f * u3, &s1, &c1);
  floatx4 o;
  o.x = m0 * c0; o.y = m0 * s0; o.z = m1 * c1; o.w = m1 * s1;
  return o;
}

__device__ __forceinline__ float softplus(float r) { return log1pf(expf(r)); }
__device__ __forceinline__ float sigmoidf_(float r) { return 1.0f / (1.0f + expf(-r)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace mauv
