// Fast resident path of the Chebyshev graph convolution for gfx950
// (graphs with M <= 1024 vertices and rows of at most 16 nonzeros; Fin in
// {1, 2, 4}): configs A, B and E of SURVEY.md §8.
//
// Kernel templates only: each (direction, Fin, Fout-tiles / fused-dW)
// instantiation is compiled in its own translation unit from
// cheb_fast_inst.hip (the Makefile builds them in parallel: the 17-way
// row-length switch makes one TU of all of them take ~5 minutes), and
// cheb_fast.hip holds the geometry and the dispatch.
//
// One 1024-thread workgroup (16 waves) per sample n, one row of the sparse
// operand per thread, the whole K-step recurrence
//   T_0 = X, T_1 = L~X, T_k = 2 L~ T_{k-1} - T_{k-2}      (lib/graph_conv.py:163-169)
// on chip.  What distinguishes it from cheb_resident.hip:
//   * the 3-slot ring T_{k-2}, T_{k-1}, T_k sits at LDS address 0 as one
//     12*FV-byte record per vertex ([pos][slot][fin]); record positions are
//     chosen by the host (cheb_abi.cpp::build_fast_image) and every gather
//     address is a register holding pos*12*FV, so a gather is ONE ds_read with
//     the ring slot as its immediate offset -- no address arithmetic per step;
//   * rows are dealt to threads in decreasing-length order, so a wave's rows
//     have (nearly) one length; the kernel switches ONCE on the wave's maximum
//     length L and runs a main loop compiled for exactly L gathers and L
//     multiply-adds per step (no per-slot selects, no dead slots);
//   * idle lanes write to a dummy record and padding entries gather a record
//     that stays zero, so the step has no divergent branch;
//   * Fin in {2, 4} is carried in the record (ds_read_b64 / _b128 gathers).
// The weight contraction y = basis @ W (lib/graph_conv.py:175) runs on MFMA
// between steps, fed from the ring; the basis is staged in LDS in the layout
// of lib/graph_conv.py:172 and leaves after the recurrence with coalesced
// 16-byte stores.  (Storing each wave's finished orders during the
// recurrence instead -- partial 8..48-byte row pieces -- was measured
// 1.4-2.7x SLOWER on config B, profiles/r02b/flush.json: partial-line stores
// are what the memory system handles worst.)
//
// The backward kernel does dBasis = dy W^T on MFMA into LDS, the reverse
// (Clenshaw) recurrence over L~^T with the same machinery, writes dx = G_0,
// and -- when FinK <= 32 and Fout <= 32 -- the per-sample dW partial
// basis^T dy on MFMA interleaved with the recurrence (operands streamed from
// HBM three steps ahead), reduced across waves in a fixed order into one
// [FinK][Fout] slab per sample (summed over samples by k_reduce_slabs).
//
// Numerics: each row accumulates sequentially from +0 in CSR order with one
// rounding per product and per add (fp contraction OFF): the order of scipy
// csr_matvecs / TF SparseTensorDenseMatMul, so the basis is bit-exact to
// lib/graph.py::chebyshev.  Padding adds 0*0 = +0 after the real entries and
// before none of them, which leaves every partial sum unchanged.
#pragma once
#include <algorithm>
#include <type_traits>

#include "cg_internal.h"
#include "split_bf16.h"

namespace cg {
namespace fastk {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kT = 1024;
constexpr int kW = kT / 64;  // waves per workgroup
template <int V>
using I = std::integral_constant<int, V>;

template <int FV>
struct VecT;
template <>
struct VecT<1> { typedef float type; };
template <>
struct VecT<2> { typedef float2 type; };
template <>
struct VecT<4> { typedef float4 type; };

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int imin(int a, int b) { return a < b ? a : b; }

template <int FV>
__device__ __forceinline__ typename VecT<FV>::type lds_v(const char* p) {
  return *reinterpret_cast<const typename VecT<FV>::type*>(p);
}
template <int FV>
__device__ __forceinline__ void lds_stv(char* p, typename VecT<FV>::type v) {
  *reinterpret_cast<typename VecT<FV>::type*>(p) = v;
}
__device__ __forceinline__ float lds_f(const char* p) { return *reinterpret_cast<const float*>(p); }

// fp32 vector helpers that keep one rounding per operation (contract off)
#pragma clang fp contract(off)
__device__ __forceinline__ float vzero1() { return 0.f; }
__device__ __forceinline__ float madd(float a, float v, float g) { return a + v * g; }
__device__ __forceinline__ float2 madd(float2 a, float v, float2 g) {
  return make_float2(a.x + v * g.x, a.y + v * g.y);
}
__device__ __forceinline__ float4 madd(float4 a, float v, float4 g) {
  return make_float4(a.x + v * g.x, a.y + v * g.y, a.z + v * g.z, a.w + v * g.w);
}
__device__ __forceinline__ float rec2(float a, float p) { return 2.f * a - p; }
__device__ __forceinline__ float2 rec2(float2 a, float2 p) {
  return make_float2(2.f * a.x - p.x, 2.f * a.y - p.y);
}
__device__ __forceinline__ float4 rec2(float4 a, float4 p) {
  return make_float4(2.f * a.x - p.x, 2.f * a.y - p.y, 2.f * a.z - p.z, 2.f * a.w - p.w);
}
// Clenshaw: d + c*a - p (p optional)
__device__ __forceinline__ float clen(float d, float c, float a) { return d + c * a; }
template <typename V>
__device__ __forceinline__ V vzero();
template <>
__device__ __forceinline__ float vzero<float>() { return 0.f; }
template <>
__device__ __forceinline__ float2 vzero<float2>() { return make_float2(0.f, 0.f); }
template <>
__device__ __forceinline__ float4 vzero<float4>() { return make_float4(0.f, 0.f, 0.f, 0.f); }
// order-only dependence: x is "rewritten" by an empty asm that reads a
__device__ __forceinline__ void pin(float& a, float& x) { asm volatile("" : "+v"(a), "+v"(x)); }
__device__ __forceinline__ void pin(float2& a, float& x) {
  asm volatile("" : "+v"(a.x), "+v"(a.y), "+v"(x));
}
__device__ __forceinline__ void pin(float4& a, float& x) {
  asm volatile("" : "+v"(a.x), "+v"(a.y), "+v"(a.z), "+v"(a.w), "+v"(x));
}
__device__ __forceinline__ float comp(float v, int) { return v; }
__device__ __forceinline__ float comp(float2 v, int i) { return i == 0 ? v.x : v.y; }
__device__ __forceinline__ float comp(float4 v, int i) {
  return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}
__device__ __forceinline__ void setc(float& v, int, float x) { v = x; }
__device__ __forceinline__ void setc(float2& v, int i, float x) {
  if (i == 0) v.x = x; else v.y = x;
}
__device__ __forceinline__ void setc(float4& v, int i, float x) {
  if (i == 0) v.x = x; else if (i == 1) v.y = x; else if (i == 2) v.z = x; else v.w = x;
}

// Registers of the one row a thread owns.
struct Row {
  int row;          // vertex, or -1 (idle)
  int rb, rb1;      // byte offsets of the row's two own records (dummy when idle)
  int rr;           // byte offset of the own-record copy read as T_{k-2}
  int ca[kFastWidth];  // byte offsets of the gathered records (zero record = padding)
  float v[kFastWidth];

  // NL: slots loaded -- kFastWidth, or the wave's row length when the caller
  // is already specialised on it (no per-slot branches: loading the first wl
  // slots under runtime conditions was measured SLOWER, the branches
  // serialise the loads; a compile-time count does not branch at all)
  template <int FV, int NL = kFastWidth>
  __device__ __forceinline__ void load(const FastImage& E, int tid) {
    constexpr int REC = 12 * FV;
    row = E.row[tid];
    rb = E.rpos[tid] * REC;
    rb1 = E.rpos1[tid] * REC;
    rr = E.rposr[tid] * REC;
#pragma unroll
    for (int j2 = 0; j2 < (NL + 1) / 2; ++j2) {
      const uint32_t pk = uint32_t(E.cpos[j2 * kT + tid]);
      ca[2 * j2] = int(pk & 0xffffu) * REC;
      ca[2 * j2 + 1] = int(pk >> 16) * REC;
    }
#pragma unroll
    for (int j = 0; j < NL; ++j) v[j] = E.val[j * kT + tid];
  }

  // the L gathers T[c_j][SLOT] of a step, issued together
  template <int FV, int L, int SLOT>
  __device__ __forceinline__ void gather(const char* ring, typename VecT<FV>::type* g) const {
#pragma unroll
    for (int j = 0; j < L; ++j) g[j] = lds_v<FV>(ring + ca[j] + SLOT * 4 * FV);
  }
  // sum_{j < L, CSR order} v_j * g_j  (sequential, one rounding each)
  template <int FV, int L>
  __device__ __forceinline__ typename VecT<FV>::type reduce(const typename VecT<FV>::type* g) const {
    typedef typename VecT<FV>::type V;
    V a = vzero<V>();
#pragma unroll
    for (int j = 0; j < L; ++j) a = madd(a, v[j], g[j]);
    return a;
  }
  template <int FV, int L, int SLOT>
  __device__ __forceinline__ typename VecT<FV>::type dot(const char* ring) const {
    typename VecT<FV>::type g[L > 0 ? L : 1];
    gather<FV, L, SLOT>(ring, g);
    return reduce<FV, L>(g);
  }
};

// ---------------------------------------------------------------------------
// Forward
// ---------------------------------------------------------------------------
// OB: the basis goes out in the orders layout during the recurrence (no LDS staging)
template <int FV, int NT, bool OB>
struct Fwd {
  typedef typename VecT<FV>::type V;
  static constexpr int REC = 12 * FV;
  static constexpr int MT = 2;  // 32-vertex tiles per wave (ntiles <= 32)

  const FastFwdArgs& A;
  char* ring;
  float* s_W;
  float* s_B;
  float* gB;  // orders layout: this sample's [FinK][bord] basis planes in HBM
  int K, M, Fout, FinK, wave, lane, li, h, ntiles, bord;
  int mb[MT];  // byte offsets of the records of this lane's MFMA tile rows
  bool keep_basis;
  Row r;
  V t1, t2;  // T_{k-1}, T_{k-2} of the own row
  f32x16 acc[MT][NT];

  __device__ __forceinline__ Fwd(const FastFwdArgs& a, char* smem, int tid) : A(a) {
    K = a.K;
    M = a.M;
    Fout = a.Fout;
    FinK = FV * K;
    lane = tid & 63;
    wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    li = lane & 31;
    h = lane >> 5;
    ntiles = (M + 31) >> 5;
    ring = smem;
    size_t off = align16(size_t(a.E.P) * REC);
    s_W = reinterpret_cast<float*>(smem + off);
    off = align16(off + size_t(FinK) * Fout * 4);
    s_B = reinterpret_cast<float*>(smem + off);
    keep_basis = a.basis != nullptr && !CG_DBG(a.dbg, 2);
    bord = a.bord;
    gB = a.basis ? a.basis + size_t(blockIdx.x) * FinK * bord : nullptr;
  }

  // Contraction of the pair (T_{2s}, T_{2s+1}) on MFMA; stage the basis
  // (rows layout) or store it (orders layout: a half-wave's 32 rows of one
  // order are 128 contiguous bytes, so each store is two whole lines and the
  // basis leaves during the recurrence instead of after it).
  __device__ __forceinline__ void pair(int s) {
    const int kk = 2 * s + h;
    const bool kv = kk < K;
    const int soff = (kk % 3) * 4 * FV;
#pragma unroll
    for (int fin = 0; fin < FV; ++fin) {
      float b[NT];
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        const int f = q * 32 + li;
        b[q] = (kv && f < Fout) ? s_W[(fin * K + kk) * Fout + f] : 0.f;
      }
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int tile = wave + t * kW;
        if (tile < ntiles) {
          const int m = tile * 32 + li;
          float a = 0.f;
          if (kv) {
            a = lds_f(ring + mb[t] + soff + fin * 4);
            if (keep_basis) {
              if (OB) gB[(fin * K + kk) * bord + m] = a;  // rows >= M: the zero record
              else if (m < M) s_B[m * FinK + fin * K + kk] = a;
            }
          }
          if (!CG_DBG(A.dbg, 4)) {
#pragma unroll
            for (int q = 0; q < NT; ++q) acc[t][q] = mfma32(a, b[q], acc[t][q]);
          }
        }
      }
    }
  }

  template <int L, int CUR, int PRV, int PRV2>
  __device__ __forceinline__ void step(int k) {
#pragma clang fp contract(off)
    // ablation build: 64 skips the gathers, 128 the own-record writes (LDS attribution)
    const V a = CG_DBG(A.dbg, 64) ? r.v[0] * t1 : r.template dot<FV, L, PRV>(ring);
    V o;
    if (CG_DBG(A.dbg, 32)) {  // A/B switch: T_{k-2} of the own row re-read from the ring
      const V p = lds_v<FV>(ring + r.rr + PRV2 * 4 * FV);
      o = (k == 1) ? a : rec2(a, p);
    } else {           // T_{k-2} of the own row kept in registers (this thread wrote it)
      o = (k == 1) ? a : rec2(a, t2);
    }
    if (!CG_DBG(A.dbg, 128)) {
      lds_stv<FV>(ring + r.rb + CUR * 4 * FV, o);
      lds_stv<FV>(ring + r.rb1 + CUR * 4 * FV, o);
    }
    t2 = t1;
    t1 = o;
    __syncthreads();
  }

  template <int L>
  __device__ __forceinline__ void go() {
    constexpr int REC_ = REC;
    const int tid = threadIdx.x;
    const int n = blockIdx.x;
    r.template load<FV, L>(A.E, tid);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int tile = imin(wave + t * kW, ntiles - 1);
      mb[t] = A.E.mpos[tile * 32 + li] * REC_;
    }
    char* smem = ring;
    if (A.ad_grad) {  // W' = ApplyAdam(W, grad), identical in every workgroup
      for (int i = tid; i < FinK * Fout; i += kT) {
        const AdamElem e = adam_math(A.W[i], A.ad_m[i], A.ad_v[i], A.ad_grad[i], A.ad_scale,
                                     A.ad_lr_t, A.ad_b1, A.ad_b2, A.ad_eps);
        s_W[i] = e.p;
        if (blockIdx.x == 0) {
          A.ad_W[i] = e.p;
          A.ad_mo[i] = e.m;
          A.ad_vo[i] = e.v;
        }
      }
    } else {
      for (int i = tid; i < FinK * Fout; i += kT) s_W[i] = A.W ? A.W[i] : 0.f;
    }
    // T_0 = x into ring slot 0 ([pos][0][fin]); zero record kept at 0
    const float* xn = A.x + size_t(n) * M * FV;
    for (int i = tid; i < M * FV; i += kT) {
      const int m = i / FV, fin = i - m * FV;
      const float xv = xn[i];
      reinterpret_cast<float*>(smem + A.E.pos0[m] * REC_)[fin] = xv;
      reinterpret_cast<float*>(smem + A.E.pos1[m] * REC_)[fin] = xv;
    }
    for (int i = tid; i < 32 * 3 * FV; i += kT)  // the 32 zero records
      reinterpret_cast<float*>(smem + A.E.zpos * REC_)[i] = 0.f;
    // T_0 of the own row for the register-held T_{k-2}
    t1 = vzero<V>();
    if (r.row >= 0) {
#pragma unroll
      for (int fin = 0; fin < FV; ++fin) setc(t1, fin, xn[r.row * FV + fin]);
    }
    t2 = t1;
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int q = 0; q < NT; ++q)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[t][q][e] = 0.f;
    __syncthreads();
    CG_TS(A.ts, 1);
    if (CG_DBG(A.dbg, 16)) return;
    run<L>();
  }

  template <int L>
  __device__ __forceinline__ void run() {
    for (int k = 1; k < K; k += 6) {  // k = 1 (mod 6): slots cur/prv/prv2 = 1/0/2
      step<L, 1, 0, 2>(k);
      if (k + 1 < K) { pair((k - 1) >> 1); step<L, 2, 1, 0>(k + 1); }
      if (k + 2 < K) step<L, 0, 2, 1>(k + 2);
      if (k + 3 < K) { pair((k + 1) >> 1); step<L, 1, 0, 2>(k + 3); }
      if (k + 4 < K) step<L, 2, 1, 0>(k + 4);
      if (k + 5 < K) { pair((k + 3) >> 1); step<L, 0, 2, 1>(k + 5); }
    }
    pair((K - 1) >> 1);  // the last (possibly half-empty) pair
  }
};

template <int FV, int NT, bool OB>
__global__ __launch_bounds__(kT) void cheb_fwd_fast(FastFwdArgs A) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef Fwd<FV, NT, OB> F;
  const int tid = threadIdx.x;
  const int n = blockIdx.x;
  CG_TS(A.ts, 0);
  F c(A, smem, tid);
  const int M = c.M, Fout = c.Fout, FinK = c.FinK;

  // the whole prologue is specialised on the wave's row length, so each
  // thread loads exactly the L gather slots its run<L> uses
  const int wl = __builtin_amdgcn_readfirstlane(A.E.wlen[c.wave]);
  switch (wl) {
#define CG_L(L_) case L_: c.template go<L_>(); break;
    CG_L(0) CG_L(1) CG_L(2) CG_L(3) CG_L(4) CG_L(5) CG_L(6) CG_L(7) CG_L(8)
    CG_L(9) CG_L(10) CG_L(11) CG_L(12) CG_L(13) CG_L(14) CG_L(15) CG_L(16)
#undef CG_L
    default: break;  // unreachable: the host only selects this kernel for rows <= 16
  }
  if (CG_DBG(A.dbg, 16)) return;
  CG_TS(A.ts, 2);

  // y first: its stores leave from registers while the other waves finish
  // the last pair; then the block-wide barrier for the basis staged in LDS
  if (A.y && !CG_DBG(A.dbg, 8)) {
    float* yn = A.y + size_t(n) * M * Fout;
#pragma unroll
    for (int t = 0; t < F::MT; ++t) {
      const int tile = c.wave + t * kW;
      if (tile < c.ntiles) {
#pragma unroll
        for (int q = 0; q < NT; ++q) {
          const int f = q * 32 + c.li;
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int m = tile * 32 + (e & 3) + 8 * (e >> 2) + 4 * c.h;
            if (m < M && f < Fout) {
              float v = c.acc[t][q][e];
              if (A.res) v = v + A.res[size_t(n) * M * Fout + size_t(m) * Fout + f];
              if (A.act) v = v > 0.f ? v : 0.f;
              yn[size_t(m) * Fout + f] = v;
            }
          }
        }
      }
    }
  }

  CG_TS(A.ts, 3);
  if (!OB && c.keep_basis) {
    __syncthreads();
    float* basis_n = A.basis + size_t(n) * M * FinK;
    const int total = M * FinK;
    if ((reinterpret_cast<uintptr_t>(basis_n) & 15) == 0) {
      const int n4 = total >> 2;
      const float4* src = reinterpret_cast<const float4*>(c.s_B);
      float4* dst = reinterpret_cast<float4*>(basis_n);
      for (int i = tid; i < n4; i += kT) dst[i] = src[i];
      for (int i = (n4 << 2) + tid; i < total; i += kT) basis_n[i] = c.s_B[i];
    } else {
      for (int i = tid; i < total; i += kT) basis_n[i] = c.s_B[i];
    }
  }
  CG_TS(A.ts, 4);
}

// ---------------------------------------------------------------------------
// Backward: dBasis (phase A), Clenshaw over L~^T -> dx, fused dW partial
// ---------------------------------------------------------------------------
// DW: 0 no fused dW, 1 fused dW from the rows-layout basis, 2 from the orders
// layout, 3 from the orders layout on the split-bf16 matrix pipe (dw_x3_*)
template <int FV, int DW>
struct Bwd {
  typedef typename VecT<FV>::type V;
  static constexpr int REC = 12 * FV;
  static constexpr int NU = 2;  // dW MFMAs per recurrence step
  static constexpr int PF = 6;  // dW operand buffers: loads run PF steps ahead
  static constexpr bool OB = DW >= 2;
  static constexpr bool X3 = DW == 3;
  static_assert(NU == 2 && PF % 2 == 0, "the orders-layout dW loads one row octet per two steps");

  const FastBwdArgs& A;
  char* ring;
  float* s_D;  // [FinK][Mp]
  int K, M, Fout, FinK, Mp, wave, li, h, n, bord;
  Row r;
  // fused dW: this wave's basis rows [dm0, dm1), 2 per MFMA
  int dm0, dm1, npair, nexti;
  V g1, g2;  // G_{k+1}, G_{k+2} of the own row
  f32x16 dacc;
  float da[X3 ? 1 : PF][NU], db[X3 ? 1 : PF][NU];
  // X3: 16-row groups, group g = octets w + 16 (2g + h) of this wave (lane
  // half h takes 8 contiguous rows, element e = row 8 oct + e): the basis
  // plane's 32 contiguous bytes and 8 dy rows per lane, one group in flight;
  // consumed every 6 recurrence steps (BUF == 5)
  float xr[8], yr[8];
  int ngrp, oct_lim;

  __device__ __forceinline__ Bwd(const FastBwdArgs& a, char* smem, int tid) : A(a) {
    K = a.K;
    M = a.M;
    Fout = a.Fout;
    FinK = FV * K;
    Mp = a.Mp;
    n = blockIdx.x;
    const int lane = tid & 63;
    wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    li = lane & 31;
    h = lane >> 5;
    ring = smem;
    s_D = reinterpret_cast<float*>(smem + align16(size_t(a.E.P) * REC));
    bord = a.bord;
  }

  // Basis row of the wave's MFMA i in lane half h.  Rows layout: rows
  // dm0 + 2i + h of the wave's chunk.  Orders layout: row octets dealt
  // round-robin (octet w + 16g to wave w); step s = i / 2 of octet g = s / 2
  // takes rows 8(w + 16g) + 4h + 2(s % 2) + i % 2, so ONE 16-byte load per
  // lane (rows 4h .. 4h+3 of the octet in one plane) feeds the four MFMAs of
  // two steps: half the load instructions of a per-step 8-byte load, each
  // still touching the 32 planes
  __device__ __forceinline__ int dw_row(int i) const {
    return OB ? 8 * (wave + kW * (i >> 2)) + 4 * h + 2 * ((i >> 1) & 1) + (i & 1) : dm0 + 2 * i + h;
  }
  // orders layout: the operands of steps s (even) and s + 1 into buffers b0, b1
  __device__ __forceinline__ void dw_load_oct(int b0, int b1, int s) {
    const float* dyn = A.dy + size_t(n) * M * Fout;
    const int jc = imin(li, FinK - 1), fc = imin(li, Fout - 1);
    const float* bn = A.basis + size_t(n) * FinK * bord;
    const int m = dw_row(s * NU);  // octet base + 4h (rows < bord: bord is a multiple of 32)
    const float4 bv = *reinterpret_cast<const float4*>(bn + size_t(jc) * bord + m);
    da[b0][0] = bv.x;
    da[b0][1] = bv.y;
    da[b1][0] = bv.z;
    da[b1][1] = bv.w;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      db[b0][u] = dyn[size_t(imin(m + u, M - 1)) * Fout + fc];
      db[b1][u] = dyn[size_t(imin(m + 2 + u, M - 1)) * Fout + fc];
    }
  }

  // ---- fused dW: acc[j][f] += sum over row pairs of basis[m][j] * dy[m][f]
  __device__ __forceinline__ void dw_load(int buf, int i0) {
    const float* dyn = A.dy + size_t(n) * M * Fout;
    const int jc = imin(li, FinK - 1), fc = imin(li, Fout - 1);
    if (OB) {  // i0 even: rows dw_row(i0) + {0, 1} (the tail after the recurrence)
      const float* bn = A.basis + size_t(n) * FinK * bord;
      const int m = dw_row(i0);
      const float2 bv = *reinterpret_cast<const float2*>(bn + size_t(jc) * bord + m);
      da[buf][0] = bv.x;
      da[buf][1] = bv.y;
#pragma unroll
      for (int u = 0; u < NU; ++u) db[buf][u] = dyn[size_t(imin(m + u, M - 1)) * Fout + fc];
      return;
    }
    const float* bn = A.basis + size_t(n) * M * FinK;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int m = imin(dm0 + 2 * (i0 + u) + h, M - 1);
      da[buf][u] = bn[size_t(m) * FinK + jc];
      db[buf][u] = dyn[size_t(m) * Fout + fc];
    }
  }
  // MFMA u of the NU held in buffer buf (the u-th row pair from i0).  With
  // `after` given, the MFMA is pinned behind the computation of *after: its
  // operand passes through an empty asm that also consumes *after (the
  // compiler otherwise hoists it next to MFMA 0, ahead of the reduction)
  template <typename T = float>
  __device__ __forceinline__ void dw_mfma1(int buf, int i0, int u, T* after = nullptr) {
    const int i = i0 + u;
    if (i < npair) {
      const bool rv = dw_row(i) < dm1;
      float x = da[buf][u];
      if (after) pin(*after, x);
      dacc = mfma32((rv && li < FinK) ? x : 0.f, (rv && li < Fout) ? db[buf][u] : 0.f, dacc);
    }
  }
  __device__ __forceinline__ void dw_mfma(int buf, int i0) {
#pragma unroll
    for (int u = 0; u < NU; ++u) dw_mfma1(buf, i0, u);
  }
  // X3: group g's operands into xr / yr (a group past the wave's octets loads
  // octet 0: its values are masked in dw_x3_mfma)
  // (buffer loads over the sample's slabs: 32-bit offsets, the bases in
  // SGPRs; a dy row past M reads 0 -- its basis entries are 0 anyway)
  __device__ __forceinline__ void dw_x3_load(int g) {
    const int oct0 = wave + kW * (2 * g + h);
    const int oct = oct0 < oct_lim ? oct0 : 0;
    int lq = threadIdx.x;  // the lane's column re-derived here (a hoisted copy is spilled)
    asm volatile("" : "+v"(lq));
    const int jc = imin(lq & 31, FinK - 1), fc = imin(lq & 31, Fout - 1);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(A.basis + size_t(n) * FinK * bord), 0, FinK * bord * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(A.dy + size_t(n) * M * Fout), 0, M * Fout * 4, 0x00020000);
    const int bo = (jc * bord + 8 * oct) * 4;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rb, bo + 16 * q, 0, 0);
      xr[4 * q] = __uint_as_float(v[0]);
      xr[4 * q + 1] = __uint_as_float(v[1]);
      xr[4 * q + 2] = __uint_as_float(v[2]);
      xr[4 * q + 3] = __uint_as_float(v[3]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e)
      yr[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ry, ((8 * oct + e) * Fout + fc) * 4, 0, 0));
  }
  // X3: the group's six bf16 MFMAs (rows >= M: the basis planes hold zeros there)
  __device__ __forceinline__ void dw_x3_mfma(int g) {
    const bool v = wave + kW * (2 * g + h) < oct_lim;
    float x[8], y[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      x[e] = (v && li < FinK) ? xr[e] : 0.f;
      y[e] = (v && li < Fout) ? yr[e] : 0.f;
    }
    dacc = x3::mfma32_x3b(x3::split3(x), y, dacc);
  }

  template <int L, int CUR, int NX1, int NX2, int BUF>
  __device__ __forceinline__ void step(int i) {
#pragma clang fp contract(off)
    const int k = K - 1 - i;
    // The step's gathers go out first, then the step's two dW MFMAs
    // (operands loaded PF steps ago) one on each side of the reduction: the
    // matrix pipe works while the wave waits for LDS, and a wave never stalls
    // in order behind its own dependent MFMA.  (Both MFMAs ahead of the
    // gathers queued the SIMD's four waves behind 8 MFMAs -- 512 cycles --
    // every step: measured +4.5 us over the recurrence.)
    V gth[L > 0 ? L : 1];
    if (i >= 1) r.template gather<FV, L, NX1>(ring, gth);
    // (ablation build: bit 64 skips the dW MFMAs, bit 128 the dW loads)
    if constexpr (X3) {
      if (BUF == 5 && i / 6 < ngrp) {  // every sixth step: one group's MFMAs, the next group's loads
        dw_x3_mfma(i / 6);
        if (i / 6 + 1 < ngrp) dw_x3_load(i / 6 + 1);
      }
    } else if (DW && !CG_DBG(A.dbg, 64)) {
      dw_mfma1(BUF, i * NU, 0);
    }
    const float c = (k >= 1) ? 2.f : 1.f;
    V a = vzero<V>();
    if (i >= 1) a = r.template reduce<FV, L>(gth);
    if (!X3 && DW && !CG_DBG(A.dbg, 64)) dw_mfma1(BUF, i * NU, 1, &a);
    if (!X3 && DW && !CG_DBG(A.dbg, 128)) {
      if (!OB) {
        dw_load(BUF, (i + PF) * NU);  // refill for step i + PF
      } else if (BUF & 1) {
        // odd step: refill steps i + PF - 1 and i + PF (buffers of steps i - 1 and i)
        dw_load_oct(BUF - 1, BUF, i + PF - 1);
      }
    }
    // G_{k+2} of the own row: kept in registers (this thread wrote it two
    // steps ago); debug bit 32 re-reads it from the ring (A/B switch)
    const V p = CG_DBG(A.dbg, 32) ? lds_v<FV>(ring + r.rr + NX2 * 4 * FV) : g2;
    const int rr = r.row < 0 ? 0 : r.row;
    V g;
#pragma unroll
    for (int fin = 0; fin < FV; ++fin) {
      float gv = s_D[(fin * K + k) * Mp + rr] + c * comp(a, fin);
      if (i >= 2) gv = gv - comp(p, fin);
      setc(g, fin, gv);
    }
    if (k == 0) {
      if (A.dx && r.row >= 0) {
        float* d = A.dx + (size_t(n) * M + r.row) * FV;
#pragma unroll
        for (int fin = 0; fin < FV; ++fin) d[fin] = A.dx_acc ? d[fin] + comp(g, fin) : comp(g, fin);
      }
    } else {
      lds_stv<FV>(ring + r.rb + CUR * 4 * FV, g);
      lds_stv<FV>(ring + r.rb1 + CUR * 4 * FV, g);
      g2 = g1;
      g1 = g;
      __syncthreads();
    }
  }

  template <int L>
  __device__ __forceinline__ void go() {
    r.template load<FV, L>(A.E, threadIdx.x);
    g1 = vzero<V>();
    g2 = g1;
    if (X3) {
      oct_lim = (M + 7) >> 3;
      const int no = oct_lim > wave ? (oct_lim - wave + kW - 1) / kW : 0;  // this wave's octets
      ngrp = (no + 1) >> 1;
      npair = 0;
#pragma unroll
      for (int e = 0; e < 16; ++e) dacc[e] = 0.f;
      if (ngrp > 0) dw_x3_load(0);
    } else if (DW) {
      if (OB) {  // row octets wave, wave + 16, ... (dw_row)
        const int no = (M + 7) >> 3;
        dm0 = 0;
        dm1 = M;
        npair = wave < no ? 4 * ((no - wave + kW - 1) / kW) : 0;
      } else {  // rows of this wave: 16 near-equal even-sized chunks of [0, M)
        const int q = ((M + 2 * kW - 1) / (2 * kW)) * 2;
        dm0 = imin(wave * q, M);
        dm1 = imin(dm0 + q, M);
        npair = (dm1 - dm0 + 1) >> 1;
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) dacc[e] = 0.f;
      if (OB) {
#pragma unroll
        for (int b = 0; b < PF; b += 2) dw_load_oct(b, b + 1, b);
      } else {
#pragma unroll
        for (int b = 0; b < PF; ++b) dw_load(b, b * NU);
      }
    }
    __syncthreads();
    CG_TS(A.ts, 3);
    run<L>();
  }

  template <int L>
  __device__ __forceinline__ void run() {
    static_assert(PF == 6, "the loop below cycles the ring (3) and the dW buffers (6)");
    for (int i = 0; i < K; i += 6) {
      step<L, 0, 2, 1, 0>(i);
      if (i + 1 < K) step<L, 1, 0, 2, 1>(i + 1);
      if (i + 2 < K) step<L, 2, 1, 0, 2>(i + 2);
      if (i + 3 < K) step<L, 0, 2, 1, 3>(i + 3);
      if (i + 4 < K) step<L, 1, 0, 2, 4>(i + 4);
      if (i + 5 < K) step<L, 2, 1, 0, 5>(i + 5);
    }
  }
};

template <int FV, int DW>
__global__ __launch_bounds__(kT) void cheb_bwd_fast(FastBwdArgs A) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef Bwd<FV, DW> B;
  constexpr int REC = B::REC;
  const int tid = threadIdx.x;
  CG_TS(A.ts, 0);
  B c(A, smem, tid);
  const int M = c.M, Fout = c.Fout, FinK = c.FinK, Mp = c.Mp, n = c.n;
  const int li = c.li, h = c.h, wave = c.wave;
  const int ws = Fout + 1;  // padded W row: the transposed B-operand read is conflict-free
  float* s_W = reinterpret_cast<float*>(reinterpret_cast<char*>(c.s_D) +
                                        align16(size_t(A.dscratch_bytes)));
  const float* dyn = A.dy + size_t(n) * M * Fout;
  const int mtiles = (M + 31) >> 5, jtiles = (FinK + 31) >> 5;
  const int ns = (Fout + 1) >> 1;  // lane half h owns f in [h*ns, h*ns + ns)
  // W first: its LDS copy (needed before the barrier) then waits only for
  // this load, not for the dy tiles queued behind it (vmcnt is in order)
  const int nW = FinK * Fout;
  const float wv = tid < nW ? A.W[tid] : 0.f;
  // Fast Phase-A operand path (config B/E shapes): each wave's <= 2 dy tiles
  // are loaded as float4 at kernel entry; tile 0's MFMAs start while tile 1
  // is still in flight.  (Always taken by the fused-dW variants: the host
  // requires FinK <= 32, Fout <= 32, Fout % 8 == 0 for them, so the loads are
  // unconditional and the waits below count them exactly.)
  const bool fastA = DW != 0 || (mtiles <= 2 * kW && jtiles == 1 && Fout <= 32 && (Fout & 7) == 0);
  float4 av[2][4];
  if (fastA) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int m = imin((wave + t * kW) * 32 + li, M - 1);
      const float4* rowp = reinterpret_cast<const float4*>(dyn + size_t(m) * Fout + h * ns);
#pragma unroll
      for (int q = 0; q < 4; ++q) av[t][q] = rowp[imin(q, (ns >> 2) - 1)];
    }
  }
  if (tid < nW) s_W[(tid / Fout) * ws + (tid % Fout)] = wv;
  for (int i = tid + kT; i < nW; i += kT) s_W[(i / Fout) * ws + (i % Fout)] = A.W[i];
  for (int i = tid; i < 32 * 3 * FV; i += kT)  // the 32 zero records
    reinterpret_cast<float*>(smem + A.E.zpos * REC)[i] = 0.f;
  __syncthreads();
  CG_TS(A.ts, 1);
  if (CG_DBG(A.dbg, 16)) return;

  // A. dBasis = dy W^T  (rows m, cols j = fin*K + k, inner f) on MFMA into LDS
  auto store_D = [&](const f32x16& acc, int mt, int j) {
    if (j < FinK) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int mm = mt * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (mm < M) c.s_D[j * Mp + mm] = acc[e];
      }
    }
  };
  if (!CG_DBG(A.dbg, 2)) {
    if (fastA && A.x3) {
      // the split-bf16 form (split_bf16.h): 16-deep k-blocks of f, element e
      // of lane half h in block kb is f = h*ns + 8kb + e -- the lane's own dy
      // registers for A, W[j][f] from LDS for B (split once, both tiles)
      const int j = li;
      const bool jv = j < FinK;
      const float* wrow = s_W + imin(j, FinK - 1) * ws + h * ns;
      const int nkb = (ns + 7) >> 3;
      x3::Split3 wb[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (jv && 8 * kb + e < ns) ? wrow[8 * kb + e] : 0.f;
        wb[kb] = x3::split3(v);
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int mt = wave + t * kW;
        if (mt < mtiles) {
          const bool mv = mt * 32 + li < M;
          f32x16 acc;
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) {
            if (kb < nkb) {
              float v[8];
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const int f = 8 * kb + e;
                v[e] = (mv && f < ns) ? comp(av[t][f >> 2], f & 3) : 0.f;
              }
              acc = x3::mfma32_x3(x3::split3(v), wb[kb], acc);
            }
          }
          store_D(acc, mt, j);
        }
      }
    } else if (fastA) {
      const int j = li;
      const bool jv = j < FinK;
      const float* wrow = s_W + imin(j, FinK - 1) * ws + h * ns;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int mt = wave + t * kW;
        if (mt < mtiles) {
          const bool mv = mt * 32 + li < M;
          f32x16 acc;
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
          for (int s = 0; s < 16; ++s) {
            if (s < ns) acc = mfma32(mv ? comp(av[t][s >> 2], s & 3) : 0.f, jv ? wrow[s] : 0.f, acc);
          }
          store_D(acc, mt, j);
        }
      }
    } else {
      for (int task = wave; task < mtiles * jtiles; task += kW) {
        const int mt = task / jtiles, jt = task - mt * jtiles;
        const int m = mt * 32 + li, j = jt * 32 + li;
        const bool mv = m < M, jv = j < FinK;
        const float* dyrow = dyn + size_t(imin(m, M - 1)) * Fout;
        const float* wrow = s_W + imin(j, FinK - 1) * ws;
        f32x16 acc;
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[e] = 0.f;
        for (int s0 = 0; s0 < ns; s0 += 8) {
          float a[8], b[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int fc = imin(h * ns + s0 + u, Fout - 1);
            a[u] = dyrow[fc];
            b[u] = wrow[fc];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const bool fv = (s0 + u) < ns && (h * ns + s0 + u) < Fout;
            acc = mfma32((mv && fv) ? a[u] : 0.f, (jv && fv) ? b[u] : 0.f, acc);
          }
        }
        store_D(acc, mt, j);
      }
    }
  }
  CG_TS(A.ts, 2);
  // B. reverse recurrence over L~^T (+ dW MFMAs between steps); the row
  // registers (exactly the wave's row length of them) and the first dW
  // operands are loaded after phase A, whose dy tiles occupy 32 registers
  // per lane until then
  const int wl = __builtin_amdgcn_readfirstlane(A.E.wlen[wave]);
  switch (wl) {
#define CG_L(L_) case L_: c.template go<L_>(); break;
    CG_L(0) CG_L(1) CG_L(2) CG_L(3) CG_L(4) CG_L(5) CG_L(6) CG_L(7) CG_L(8)
    CG_L(9) CG_L(10) CG_L(11) CG_L(12) CG_L(13) CG_L(14) CG_L(15) CG_L(16)
#undef CG_L
    default: break;
  }
  CG_TS(A.ts, 4);

  if (DW) {
    // remaining row pairs / groups (K small relative to M/32), then the cross-wave sum
    if constexpr (B::X3) {
      for (int g = c.K / 6; g < c.ngrp; ++g) {
        // (group K / 6 was loaded by the last in-loop group, or by go())
        c.dw_x3_mfma(g);
        if (g + 1 < c.ngrp) c.dw_x3_load(g + 1);
      }
    }
    for (int i0 = c.K * B::NU; i0 < c.npair; i0 += B::NU) {
      c.dw_load(0, i0);
      c.dw_mfma(0, i0);
    }
    __syncthreads();  // every wave is past its last read of s_D
    float* part = c.s_D;  // [16 waves][32][32]
#pragma unroll
    for (int e = 0; e < 16; ++e)
      part[(wave * 32 + (e & 3) + 8 * (e >> 2) + 4 * h) * 32 + li] = c.dacc[e];
    __syncthreads();
    {
      const int j = tid >> 5, f = tid & 31;
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < kW; ++w) s = s + part[(w * 32 + j) * 32 + f];
      if (j < FinK && f < Fout) A.dw_slab[(size_t(n) * FinK + j) * Fout + f] = s;
    }
  }
  CG_TS(A.ts, 5);
}

template <typename Kern>
hipError_t allow_big_lds(Kern k) {
  return hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                             hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
}

template <int FV, int NT, bool OB>
hipError_t launch_fwd_fast_t(size_t lds, int N, const FastFwdArgs& a, hipStream_t s) {
  static hipError_t attr = allow_big_lds(&cheb_fwd_fast<FV, NT, OB>);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((cheb_fwd_fast<FV, NT, OB>), dim3(N), dim3(kT), lds, s, a);
  return hipGetLastError();
}

template <int FV, int DW>
hipError_t launch_bwd_fast_t(size_t lds, int N, const FastBwdArgs& a, hipStream_t s) {
  static hipError_t attr = allow_big_lds(&cheb_bwd_fast<FV, DW>);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((cheb_bwd_fast<FV, DW>), dim3(N), dim3(kT), lds, s, a);
  return hipGetLastError();
}

}  // namespace fastk
}  // namespace cg
