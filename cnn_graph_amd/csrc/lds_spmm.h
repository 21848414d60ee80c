// One lane's piece of a CSR row product out of an LDS-resident operand, for
// the resident kernels that keep both the sparse matrix (16-bit columns +
// values) and the dense operand X ([rows][stride] floats) in LDS:
//
//   out[c0 .. c0+3] = sum_{j in row, CSR order} val[j] * X[col[j]][c0 .. c0+3]
//
// accumulated from +0 with one rounding per product and per add (the caller
// compiles with fp contraction off) -- the order of lib/graph.py::chebyshev's
// scipy csr_matvecs, so the result is bit-exact to it.  With a wave-uniform
// bound L on the row length the entry loads and the gathers are unrolled and
// issued together (the dynamic loop serialises one LDS round trip per entry);
// entries past the row end read the zero row `zrow` with value 0, which adds
// +0 to the sum.
#pragma once
#include <hip/hip_runtime.h>

namespace cg {

template <int L>
__device__ __forceinline__ float4 lds_row_spmm(const float* X, int stride, int c0,
                                               const unsigned short* col, const float* val,
                                               int rb, int re, int zrow) {
#pragma clang fp contract(off)
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (L == 0) {  // any length
    for (int jj = rb; jj < re; ++jj) {
      const float w = val[jj];
      const float4 g = *reinterpret_cast<const float4*>(X + int(col[jj]) * stride + c0);
      s.x = s.x + w * g.x;
      s.y = s.y + w * g.y;
      s.z = s.z + w * g.z;
      s.w = s.w + w * g.w;
    }
    return s;
  }
  int c[L > 0 ? L : 1];
  float w[L > 0 ? L : 1];
#pragma unroll
  for (int e = 0; e < L; ++e) {
    const bool ok = rb + e < re;
    const int jj = ok ? rb + e : 0;
    c[e] = ok ? int(col[jj]) : zrow;
    w[e] = ok ? val[jj] : 0.f;
  }
  float4 g[L > 0 ? L : 1];
#pragma unroll
  for (int e = 0; e < L; ++e) g[e] = *reinterpret_cast<const float4*>(X + c[e] * stride + c0);
#pragma unroll
  for (int e = 0; e < L; ++e) {
    s.x = s.x + w[e] * g[e].x;
    s.y = s.y + w[e] * g[e].y;
    s.z = s.z + w[e] * g[e].z;
    s.w = s.w + w[e] * g[e].w;
  }
  return s;
}

// bytes of LDS kept past the end of the 16-bit column array by a kernel using
// lds_row_spmm_w: a padded row at the CSR's end reads up to L + 1 - len <= 13
// columns past it (and its values read on into the column array)
constexpr int kSpmmSlack = 32;

// lds_row_spmm with the row's CSR metadata read two entries per LDS access:
// the 16-bit columns as 32-bit words and the values as 64-bit pairs from the
// even-aligned entry at or below rb, so a row of L entries takes
// 2 ceil((L + 1) / 2) metadata reads + L gathers instead of 3L LDS accesses.
// Entry e sits at word / pair (e + a) >> 1, half (e + a) & 1, a = rb & 1 (per
// lane: a select); entries past the row end gather the zero row with value 0,
// exactly as lds_row_spmm (the words read past the CSR's end feed only those).
// col must be 4-byte and val 8-byte aligned; the sum is lds_row_spmm's.  A
// kernel using it keeps kSpmmSlack bytes of LDS past its column array.

template <int L>
__device__ __forceinline__ float4 lds_row_spmm_w(const float* X, int stride, int c0,
                                                 const unsigned short* col, const float* val,
                                                 int rb, int re, int zrow) {
#pragma clang fp contract(off)
  if constexpr (L == 0) {
    return lds_row_spmm<0>(X, stride, c0, col, val, rb, re, zrow);
  } else {
    constexpr int NW = (L + 2) / 2;  // words / pairs covering entries 0 .. L-1 at either parity
    const int a = rb & 1, r0 = rb - a;
    unsigned cw[NW];
    float2 vw[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      cw[i] = *reinterpret_cast<const unsigned*>(col + r0 + 2 * i);
      vw[i] = *reinterpret_cast<const float2*>(val + r0 + 2 * i);
    }
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    int c[L];
    float w[L];
#pragma unroll
    for (int e = 0; e < L; ++e) {
      const bool ok = rb + e < re;
      // entry e: word (e + a) >> 1, half (e + a) & 1
      const unsigned wlo = cw[e >> 1], whi = cw[(e + 1) >> 1];
      const float2 plo = vw[e >> 1], phi = vw[(e + 1) >> 1];
      unsigned cword;
      float v;
      if (e & 1) {  // (e + a) >> 1 = e/2 + a: the word changes with a, the half is 1 - a
        cword = a ? (whi & 0xffffu) : (wlo >> 16);
        v = a ? phi.x : plo.y;
      } else {      // (e + a) >> 1 = e/2: the same word, half a
        cword = a ? (wlo >> 16) : (wlo & 0xffffu);
        v = a ? plo.y : plo.x;
      }
      c[e] = ok ? int(cword) : zrow;
      w[e] = ok ? v : 0.f;
    }
    float4 g[L];
#pragma unroll
    for (int e = 0; e < L; ++e) g[e] = *reinterpret_cast<const float4*>(X + c[e] * stride + c0);
#pragma unroll
    for (int e = 0; e < L; ++e) {
      s.x = s.x + w[e] * g[e].x;
      s.y = s.y + w[e] * g[e].y;
      s.z = s.z + w[e] * g[e].z;
      s.w = s.w + w[e] * g[e].w;
    }
    return s;
  }
}

// The same product with the row's columns already in registers: pk holds the
// row's (up to 2*NP) column indices packed two per word (entry e in bits
// 16*(e & 1) of pk[e / 2]; entries past the row hold zrow).  The gathers no
// longer wait on an LDS read of the column, and the row takes L LDS gathers +
// L value reads instead of 3L reads; sum order and padding (+0 for w = 0)
// exactly lds_row_spmm's.  SH = log2(stride).
template <int L, int NP, int SH>
__device__ __forceinline__ float4 lds_row_spmm_pc(const float* X, int c0, const unsigned (&pk)[NP],
                                                  const float* val, int rb, int re) {
#pragma clang fp contract(off)
  static_assert(L <= 2 * NP, "row longer than the packed columns");
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  float w[L];
  float4 g[L];
#pragma unroll
  for (int e = 0; e < L; ++e) {
    const bool ok = rb + e < re;
    w[e] = ok ? val[rb + e] : 0.f;
    const int c = int((pk[e >> 1] >> (16 * (e & 1))) & 0xffffu);
    g[e] = *reinterpret_cast<const float4*>(X + (c << SH) + c0);
  }
#pragma unroll
  for (int e = 0; e < L; ++e) {
    s.x = s.x + w[e] * g[e].x;
    s.y = s.y + w[e] * g[e].y;
    s.z = s.z + w[e] * g[e].z;
    s.w = s.w + w[e] * g[e].w;
  }
  return s;
}

// pk for lds_row_spmm_pc: the columns of CSR row entries [rb, re), padded with zrow
template <int NP>
__device__ __forceinline__ void pack_row_cols(unsigned (&pk)[NP], const unsigned short* col, int rb,
                                              int re, int zrow) {
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int e0 = rb + 2 * p, e1 = e0 + 1;
    const unsigned lo = e0 < re ? unsigned(col[e0]) : unsigned(zrow);
    const unsigned hi = e1 < re ? unsigned(col[e1]) : unsigned(zrow);
    pk[p] = lo | (hi << 16);
  }
}

template <int V>
struct IntC {
  static constexpr int value = V;
};

// f(IntC<L>{}) with L the smallest supported unrolled bound >= len (0 = the
// dynamic loop beyond 12); len must be wave-uniform
template <typename F>
__device__ __forceinline__ void with_row_len(int len, F&& f) {
  if (len <= 4) f(IntC<4>{});
  else if (len <= 6) f(IntC<6>{});
  else if (len <= 8) f(IntC<8>{});
  else if (len <= 10) f(IntC<10>{});
  else if (len <= 12) f(IntC<12>{});
  else f(IntC<0>{});
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const int u = __shfl_xor(v, o);
    v = u > v ? u : v;
  }
  return v;
}

}  // namespace cg
