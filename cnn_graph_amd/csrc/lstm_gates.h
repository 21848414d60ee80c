// Gate nonlinearities of the gconv-LSTM cell (lib/gconv_lstm.py:188-218:
// z = tan, i = f = sigmoid, o = tanh in the reference; tanh / sigmoid for the
// standard gates; h' = o tanh(c')), shared by EVERY LSTM kernel (the pointwise
// cell kernels, the one-launch h-step, the sequence forward and the BPTT
// steps) so that all paths agree bitwise on the same pre-activations.
//
// The device library's tanf / tanhf / expf + IEEE division cost ~350 VALU
// instructions per unit in the sequence kernel's gate epilogue (mostly range
// reduction for arguments no gate ever sees).  These forms keep a few ulp of
// accuracy (the parity bar is 1e-5 normwise against float64) in ~60:
//   tan:     Cody-Waite reduction by pi/2 (three-part constant, fused
//            multiply-adds: exact for |x| < 8192) + the Cephes minimax
//            polynomial on [-pi/4, pi/4] (relative error <= 4e-7), -1/tan
//            in odd quadrants; |x| >= 8192 or non-finite: the library tanf
//   sigmoid: 1 / (1 + exp(-a)) with the hardware 2^x and reciprocal (1 ulp each)
//   tanh:    |x| < 0.625: the Cephes odd polynomial (<= 2 ulp); else
//            1 - 2 / (exp(2|x|) + 1) with the sign restored (exp overflow
//            gives exactly +-1)
#pragma once
#include <hip/hip_runtime.h>

namespace cg {

__device__ __forceinline__ float gate_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// e^x as the hardware 2^x of x log2(e): the product's rounding (|x| 2^-24
// relative in the exponent) is <= 1.2e-6 relative for the |x| <= 20 that
// leave a sigmoid or tanh short of saturation; out of range it saturates to
// 0 / +inf like expf
__device__ __forceinline__ float gate_exp(float x) {
#pragma clang fp contract(off)
  return __builtin_amdgcn_exp2f(x * 1.44269504088896341f);
}

__device__ __forceinline__ float gate_sigmoid(float a) {
#pragma clang fp contract(off)
  return gate_rcp(1.f + gate_exp(-a));
}

__device__ __forceinline__ float gate_tanh(float x) {
#pragma clang fp contract(off)
  const float ax = fabsf(x);
  const float z = x * x;
  float p = -5.70498872745e-3f;
  p = __builtin_fmaf(p, z, 2.06390887954e-2f);
  p = __builtin_fmaf(p, z, -5.37397155531e-2f);
  p = __builtin_fmaf(p, z, 1.33314422036e-1f);
  p = __builtin_fmaf(p, z, -3.33332819422e-1f);
  const float small = __builtin_fmaf(p * z, x, x);
  const float e = gate_exp(2.f * ax);
  const float big = 1.f - 2.f * gate_rcp(e + 1.f);
  const float r = ax < 0.625f ? small : __builtin_copysignf(big, x);
  return x != x ? x : r;
}

__device__ __forceinline__ float gate_tan(float x) {
#pragma clang fp contract(off)
  if (!(fabsf(x) < 8192.f)) return tanf(x);  // huge or non-finite: the library routine
  const float k = __builtin_rintf(x * 0.636619772367581343f);  // x * 2/pi
  float r = __builtin_fmaf(-k, 1.57079637050628662109375f, x);
  r = __builtin_fmaf(-k, -4.37113900018624283e-8f, r);
  r = __builtin_fmaf(-k, -1.71512451438203e-15f, r);
  const float z = r * r;
  float p = 9.38540185543e-3f;
  p = __builtin_fmaf(p, z, 3.11992232697e-3f);
  p = __builtin_fmaf(p, z, 2.44301354525e-2f);
  p = __builtin_fmaf(p, z, 5.34112807005e-2f);
  p = __builtin_fmaf(p, z, 1.33387994085e-1f);
  p = __builtin_fmaf(p, z, 3.33331568548e-1f);
  const float t = __builtin_fmaf(p * z, r, r);
  const bool odd = (int(k) & 1) != 0;
  return odd ? -gate_rcp(t) : t;
}

}  // namespace cg
