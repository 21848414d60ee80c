// f32-accurate products on the bf16 matrix pipe (gfx950).
//
// Every f32 operand x is split EXACTLY into three bf16 terms x = hi + mid + lo:
// hi = the top 8 significant bits (truncation of the f32 to its upper half),
// mid = the top 8 of the exact remainder x - hi, lo = the last 8 (x - hi - mid,
// exact): 24 bits, the whole f32 significand.  A product a*b is accumulated as
// the six terms down to 2^-16 of it -- hi*hi, hi*mid, mid*hi, hi*lo, lo*hi,
// mid*mid -- each exact in f32; the dropped mid*lo, lo*mid, lo*lo are below
// 2^-23 of |a*b|, the size of one f32 rounding.  On v_mfma_f32_32x32x16_bf16
// (32 cycles) / v_mfma_f32_16x16x32_bf16 (16 cycles) that is 6 MFMAs per 16 / 32
// k against 8 x v_mfma_f32_32x32x2_f32 (64 cycles) / 8 x v_mfma_f32_16x16x4_f32
// (32 cycles) for the f32 forms: 2.7x the f32 matrix rate at f32 accuracy,
// paid with ~5.5 VALU operations per split element.  Sums run in another order
// than the f32 forms' k-ordered fma chains: results agree to f32 rounding, not
// bitwise.  Users: k_dw_x3s, k_rowgemm_x3 (cheb_stream.hip), k_lstm_bstep's
// D_k contraction (lstm_seq.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace cg {
namespace x3 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Split3 {
  bf16x8 hi, mid, lo;
};

// the three terms of 8 values, packed as MFMA fragments (element j = v[j])
__device__ __forceinline__ Split3 split3(const float (&v)[8]) {
  float r[8], s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    r[j] = v[j] - __uint_as_float(__float_as_uint(v[j]) & 0xffff0000u);  // exact
    s[j] = r[j] - __uint_as_float(__float_as_uint(r[j]) & 0xffff0000u);  // exact, <= 8 bits
  }
  u32x4 h, m, l;
  // the upper halves of elements 2i (low half) and 2i+1 (high half)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    h[i] = __builtin_amdgcn_perm(__float_as_uint(v[2 * i + 1]), __float_as_uint(v[2 * i]), 0x07060302u);
    m[i] = __builtin_amdgcn_perm(__float_as_uint(r[2 * i + 1]), __float_as_uint(r[2 * i]), 0x07060302u);
    l[i] = __builtin_amdgcn_perm(__float_as_uint(s[2 * i + 1]), __float_as_uint(s[2 * i]), 0x07060302u);
  }
  Split3 x;
  x.hi = __builtin_bit_cast(bf16x8, h);
  x.mid = __builtin_bit_cast(bf16x8, m);
  x.lo = __builtin_bit_cast(bf16x8, l);
  return x;
}

// c += a * b over one 16-deep k-block of a 32x32 tile (smallest terms first)
__device__ __forceinline__ f32x16 mfma32_x3(const Split3& a, const Split3& b, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.mid, b.mid, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.lo, b.hi, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, b.lo, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.mid, b.hi, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, b.mid, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, b.hi, c, 0, 0, 0);
}

// c += a * b with b given as 8 raw f32 values, split one term at a time (a
// tighter register peak than split3(b): one B fragment live at once); the same
// six products, in the order lo*hi, mid*hi, hi*hi, mid*mid, hi*mid, hi*lo
__device__ __forceinline__ f32x16 mfma32_x3b(const Split3& a, const float (&b)[8], f32x16 c) {
  float r[8];
  u32x4 w;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    w[i] = __builtin_amdgcn_perm(__float_as_uint(b[2 * i + 1]), __float_as_uint(b[2 * i]), 0x07060302u);
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = b[j] - __uint_as_float(__float_as_uint(b[j]) & 0xffff0000u);
  bf16x8 f = __builtin_bit_cast(bf16x8, w);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.lo, f, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.mid, f, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, f, c, 0, 0, 0);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    w[i] = __builtin_amdgcn_perm(__float_as_uint(r[2 * i + 1]), __float_as_uint(r[2 * i]), 0x07060302u);
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = r[j] - __uint_as_float(__float_as_uint(r[j]) & 0xffff0000u);
  f = __builtin_bit_cast(bf16x8, w);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.mid, f, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, f, c, 0, 0, 0);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    w[i] = __builtin_amdgcn_perm(__float_as_uint(r[2 * i + 1]), __float_as_uint(r[2 * i]), 0x07060302u);
  f = __builtin_bit_cast(bf16x8, w);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.hi, f, c, 0, 0, 0);
}

// c += a * b over one 32-deep k-block of a 16x16 tile
__device__ __forceinline__ f32x4 mfma16_x3(const Split3& a, const Split3& b, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.mid, b.mid, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.lo, b.hi, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.lo, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.mid, b.hi, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.mid, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.hi, b.hi, c, 0, 0, 0);
}

}  // namespace x3
}  // namespace cg
