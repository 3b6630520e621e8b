// 16-bit storage helpers (bf16 / f16) for the reduced-precision path.
//
// Activations, activation gradients and sampled weights are stored as 16-bit words; every
// reduction (GEMM accumulation, BatchNorm statistics, weight gradients) runs in fp32.  DT
// selects the format: 0 = bf16 (training, BASELINE configs[2]), 1 = f16 (what the reference's
// predictor computes in under torch.amp.autocast on a GPU, inference/predictors.py:55).
#pragma once
#include "mauv_common.h"

typedef unsigned short u16;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float floatx8 __attribute__((ext_vector_type(8)));

namespace mauv {

enum { DT_BF16 = 0, DT_F16 = 1 };

template <int DT>
struct H16;

template <>
struct H16<DT_BF16> {
  typedef bf16x8 V8;
  static __device__ __forceinline__ float to_f(u16 v) { return __uint_as_float((unsigned)v << 16); }
  static __device__ __forceinline__ u16 from_f(float f) {
    return __builtin_bit_cast(u16, (__bf16)f);  // round-to-nearest-even (v_cvt_pk_bf16_f32)
  }
  static __device__ __forceinline__ floatx16 mfma(u32x4 a, u32x4 b, floatx16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(V8, a),
                                                   __builtin_bit_cast(V8, b), c, 0, 0, 0);
  }
};

template <>
struct H16<DT_F16> {
  typedef f16x8 V8;
  static __device__ __forceinline__ float to_f(u16 v) { return (float)__builtin_bit_cast(_Float16, v); }
  static __device__ __forceinline__ u16 from_f(float f) { return __builtin_bit_cast(u16, (_Float16)f); }
  static __device__ __forceinline__ floatx16 mfma(u32x4 a, u32x4 b, floatx16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(V8, a),
                                                  __builtin_bit_cast(V8, b), c, 0, 0, 0);
  }
};

// 8 packed 16-bit values <-> 8 floats
template <int DT>
__device__ __forceinline__ floatx8 unpack8(u32x4 v) {
  floatx8 f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = H16<DT>::to_f((u16)(v[i] & 0xffffu));
    f[2 * i + 1] = H16<DT>::to_f((u16)(v[i] >> 16));
  }
  return f;
}
template <int DT>
__device__ __forceinline__ u32x4 pack8(floatx8 f) {
  u32x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    v[i] = (unsigned)H16<DT>::from_f(f[2 * i]) | ((unsigned)H16<DT>::from_f(f[2 * i + 1]) << 16);
  return v;
}

// ---- MFMA operand fragments (v_mfma_f32_32x32x16_{bf16,f16}: lane l holds row l&31,
// k = 8(l>>5) + j, j = 0..7) from the two LDS operand images of the implicit-GEMM convs ----
// row image [rows][LD] (k-contiguous rows): one ds_read_b128 for k-step s
template <int LD>
__device__ __forceinline__ u32x4 row_frag_ld(const u16* img, int R0, int s, int li, int lh) {
  return *(const u32x4*)(img + (R0 + li) * LD + 16 * s + 8 * lh);
}
// col image [k][LD] (rows-contiguous, k-strided operand): two hardware-transposed
// ds_read_b64_tr_b16 reads; LD = rows + 32 makes a 32-lane half cover the 64 banks once
__device__ __forceinline__ u32x4 col_frag(const u16* img, int LD, int R0, int s, int lane) {
  const int gq = (lane >> 4) & 3, i = lane & 15, q = i >> 2, p = i & 3, h = lane >> 5;
  const int col = R0 + 16 * (gq & 1) + 4 * p;
  const int kr = 16 * s + 8 * h + q;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + kr * LD + col));
  const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + (kr + 4) * LD + col));
  const uint2 u0 = __builtin_bit_cast(uint2, t0), u1 = __builtin_bit_cast(uint2, t1);
  u32x4 r;
  r[0] = u0.x; r[1] = u0.y; r[2] = u1.x; r[3] = u1.y;
  return r;
}

// ---- exact split of fp32 into bf16 planes (the split-fp32 conv arithmetic) ----
// x = h + m + l exactly: h = RNE_bf16(x) keeps 8 significant bits, r = x - h is exact in
// fp32 and spans at most x's low 16 bit positions, m = RNE_bf16(r), and r - m spans at most
// 8 bit positions, so l = r - m is itself a bf16.  |m| <= 2^-8 |x|, |l| <= 2^-16 |x|.
__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  const bf16x2_t v = {(__bf16)a, (__bf16)b};  // v_cvt_pk_bf16_f32 (round to nearest even)
  return __builtin_bit_cast(unsigned, v);
}
__device__ __forceinline__ float bf_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }
// NPL = 3: (h, m, l) exact; NPL = 2: (h, m), x - h - m <= 2^-16 |x| dropped
template <int NPL>
__device__ __forceinline__ void split_bf16(floatx4 v, uint2* pl) {
  pl[0].x = pk_bf16(v[0], v[1]);
  pl[0].y = pk_bf16(v[2], v[3]);
  // opaque to the optimiser: it would otherwise re-convert each element alone to extract the
  // low half instead of shifting the packed word
  asm("" : "+v"(pl[0].x), "+v"(pl[0].y));
  const float r0 = v[0] - bf_lo(pl[0].x), r1 = v[1] - bf_hi(pl[0].x);
  const float r2 = v[2] - bf_lo(pl[0].y), r3 = v[3] - bf_hi(pl[0].y);
  pl[1].x = pk_bf16(r0, r1);
  pl[1].y = pk_bf16(r2, r3);
  if constexpr (NPL == 3) {
    asm("" : "+v"(pl[1].x), "+v"(pl[1].y));
    pl[2].x = pk_bf16(r0 - bf_lo(pl[1].x), r1 - bf_hi(pl[1].x));
    pl[2].y = pk_bf16(r2 - bf_lo(pl[1].y), r3 - bf_hi(pl[1].y));
  }
}

}  // namespace mauv

namespace mauv {

// Storage policies for kernels shared by the fp32 and 16-bit paths: values are always
// computed in fp32; S::T is what sits in HBM.
struct SF32 {
  typedef float T;
  static __device__ __forceinline__ float ld(const T* p) { return *p; }
  static __device__ __forceinline__ void st(T* p, float v) { *p = v; }
  static __device__ __forceinline__ floatx4 ld4(const T* p) { return *(const floatx4*)p; }
  static __device__ __forceinline__ void st4(T* p, floatx4 v) { *(floatx4*)p = v; }
  static __device__ __forceinline__ floatx8 ld8(const T* p) {
    const floatx4 a = *(const floatx4*)p, b = *(const floatx4*)(p + 4);
    floatx8 f;
#pragma unroll
    for (int e = 0; e < 4; ++e) { f[e] = a[e]; f[4 + e] = b[e]; }
    return f;
  }
  static __device__ __forceinline__ void st8(T* p, floatx8 v) {
    floatx4 a, b;
#pragma unroll
    for (int e = 0; e < 4; ++e) { a[e] = v[e]; b[e] = v[4 + e]; }
    *(floatx4*)p = a;
    *(floatx4*)(p + 4) = b;
  }
  // 8 elements as loaded (R8) and converted at their use (cvt8): keeps a batch of rows in
  // flight in as few registers as the storage format needs
  typedef floatx8 R8;
  static __device__ __forceinline__ R8 raw8(const T* p) { return ld8(p); }
  static __device__ __forceinline__ floatx8 cvt8(const R8& r) { return r; }
};

template <int DT>
struct S16 {
  typedef u16 T;
  static __device__ __forceinline__ float ld(const T* p) { return H16<DT>::to_f(*p); }
  static __device__ __forceinline__ void st(T* p, float v) { *p = H16<DT>::from_f(v); }
  static __device__ __forceinline__ floatx4 ld4(const T* p) {
    const uint2 u = *(const uint2*)p;
    floatx4 f;
    f[0] = H16<DT>::to_f((u16)(u.x & 0xffffu));
    f[1] = H16<DT>::to_f((u16)(u.x >> 16));
    f[2] = H16<DT>::to_f((u16)(u.y & 0xffffu));
    f[3] = H16<DT>::to_f((u16)(u.y >> 16));
    return f;
  }
  static __device__ __forceinline__ void st4(T* p, floatx4 v) {
    uint2 u;
    u.x = (unsigned)H16<DT>::from_f(v[0]) | ((unsigned)H16<DT>::from_f(v[1]) << 16);
    u.y = (unsigned)H16<DT>::from_f(v[2]) | ((unsigned)H16<DT>::from_f(v[3]) << 16);
    *(uint2*)p = u;
  }
  static __device__ __forceinline__ floatx8 ld8(const T* p) { return unpack8<DT>(*(const u32x4*)p); }
  static __device__ __forceinline__ void st8(T* p, floatx8 v) { *(u32x4*)p = pack8<DT>(v); }
  typedef u32x4 R8;
  static __device__ __forceinline__ R8 raw8(const T* p) { return *(const u32x4*)p; }
  static __device__ __forceinline__ floatx8 cvt8(const R8& r) { return unpack8<DT>(r); }
};

}  // namespace mauv

namespace mauv {
__device__ __forceinline__ floatx8 ldf8(const float* p) { return SF32::ld8(p); }
}  // namespace mauv

// Dispatch a C-ABI dtype code to a launch macro L(DT) (returns kErrArg on a bad code).
#define MAUV_DT_DISPATCH(dtype, what, L)                                      \
  if (dtype == mauv::DT_BF16) { L(mauv::DT_BF16) }                            \
  else if (dtype == mauv::DT_F16) { L(mauv::DT_F16) }                         \
  else { mauv::set_error(std::string(what) + ": dtype must be 0 (bf16) or 1 (f16)"); return mauv::kErrArg; }
