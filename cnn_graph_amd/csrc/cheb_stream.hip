// Streaming path of the Chebyshev graph convolution for gfx950: any graph
// size (the dense right-hand side lives in HBM, one launch per Chebyshev step),
// sample-major layout ([N][M][Fin], the layout of x); small Fin (< 8) runs on
// the wide-column layout of cheb_wide.hip instead.
//
//   k_cheb_step / k_cheb_last
//                 T_k = 2 L~ T_{k-1} - T_{k-2} (T_1 = L~ T_0, T_0 IS x), LPR =
//                 Fin/VEC lanes per (sample, row), sample-per-XCD block mapping
//                 for slabs <= 2 MB; the last step assembles the basis rows
//                 [fin][k] of lib/graph_conv.py:172 (staged in LDS)
//   k_clenshaw_step
//                 G_k = D_k + c L~^T G_{k+1} - G_{k+2}, D_k a plane of the
//                 k-major dBasis, G_k written in place of it; k = 0 writes dx
//   k_rowgemm     persistent skinny MFMA GEMM (32x32x2 f32, small operand in
//                 LDS): y = basis W (+ residual / ReLU epilogue) and the k-major
//                 dBasis planes (all planes in one pass over dy)
//   k_gemm_f32    LDS-tiled MFMA GEMM for the other shapes
//   k_dw_slabs / k_reduce_slabs
//                 dW = basis^T dy as per-chunk slabs, fixed-order reduction
//
// The SpMM accumulates sequentially in CSR order with fp contraction off, so
// the basis is bit-identical to the resident path and to lib/graph.py::chebyshev.
#include "cg_internal.h"
#include "occupancy_cache.h"
#include "split_bf16.h"

#include <algorithm>
#include <type_traits>

namespace cg {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

inline int grid_for(int64_t total, int block) {
  int64_t g = (total + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return int(g);
}

// ---- Chebyshev steps in the sample-major layout ---------------------------------
// T_k is stored like x: [N][M][Fin] (T_0 IS x, no transpose).  A work item is
// one (sample n, vertex row r): LPR lanes own its Fin columns (VEC floats per
// lane), a wave holds 64/LPR rows.  Gathers of T_{k-1}[n][c][:] read Fin*4
// contiguous bytes of the SAME sample, so a sample's slab (M*Fin*4 bytes) is
// the gathered working set; blocks are mapped so that each XCD works through
// its own samples (n = xcd, xcd+8, ...) and that slab stays in its L2.
// The last step assembles the basis row (n, r) = [fin][k] (lib/graph_conv.py:172)
// from the own-row T_0..T_{K-2} and the fresh T_{K-1}: every basis byte is
// written once, by one lane, contiguously.
struct StepGeom {
  int lpr;      // lanes per row
  int rpw;      // rows per wave (64 / lpr)
  int rb;       // row blocks (of 4 waves) per sample
  int xcd_map;  // 1: sample-per-XCD block mapping
  int N;        // samples; with xcd_map the grid covers 8 * ceil(N / 8) of
                // them and the blocks of samples n >= N exit at once
  unsigned grid;  // blocks to launch
};

// Block -> (sample, row block).  Returns false for the padding blocks of the
// sample-per-XCD mapping (N not a multiple of 8), which exit immediately.
__device__ __forceinline__ bool block_coords(const StepGeom g, int* n, int* rb) {
  const int i = blockIdx.x;
  if (g.xcd_map) {
    const int x = i & 7, q = i >> 3;
    *n = x + 8 * (q / g.rb);
    *rb = q % g.rb;
  } else {
    *n = i / g.rb;
    *rb = i % g.rb;
  }
  return *n < g.N;
}

template <int VEC>
struct Vec;
template <>
struct Vec<1> {
  typedef float T;
  static __device__ __forceinline__ T ld(const float* p) { return *p; }
  static __device__ __forceinline__ void st(float* p, T v) { *p = v; }
  static __device__ __forceinline__ T zero() { return 0.f; }
  static __device__ __forceinline__ float get(const T& v, int) { return v; }
  static __device__ __forceinline__ T fma_seq(T a, float w, T t) {
#pragma clang fp contract(off)
    return a + w * t;
  }
  static __device__ __forceinline__ T two_minus(T a, T p) {
#pragma clang fp contract(off)
    return 2.f * a - p;
  }
  static __device__ __forceinline__ T add_c_sub(T d, float c, T a) {
#pragma clang fp contract(off)
    return d + c * a;
  }
  static __device__ __forceinline__ T sub(T a, T b) { return a - b; }
  static __device__ __forceinline__ T add(T a, T b) { return a + b; }
};
template <>
struct Vec<4> {
  typedef float4 T;
  static __device__ __forceinline__ T ld(const float* p) { return *reinterpret_cast<const float4*>(p); }
  static __device__ __forceinline__ void st(float* p, T v) { *reinterpret_cast<float4*>(p) = v; }
  static __device__ __forceinline__ T zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
  static __device__ __forceinline__ float get(const T& v, int i) {
    return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
  }
  static __device__ __forceinline__ T fma_seq(T a, float w, T t) {
#pragma clang fp contract(off)
    return make_float4(a.x + w * t.x, a.y + w * t.y, a.z + w * t.z, a.w + w * t.w);
  }
  static __device__ __forceinline__ T two_minus(T a, T p) {
#pragma clang fp contract(off)
    return make_float4(2.f * a.x - p.x, 2.f * a.y - p.y, 2.f * a.z - p.z, 2.f * a.w - p.w);
  }
  static __device__ __forceinline__ T add_c_sub(T d, float c, T a) {
#pragma clang fp contract(off)
    return make_float4(d.x + c * a.x, d.y + c * a.y, d.z + c * a.z, d.w + c * a.w);
  }
  static __device__ __forceinline__ T sub(T a, T b) {
#pragma clang fp contract(off)
    return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
  }
  static __device__ __forceinline__ T add(T a, T b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  }
};

// sum_{j in row r, CSR order} val[j] * S[col[j]*Fin + f0 .. +VEC), sequential
// from +0 with one rounding per product and per add (the order of scipy
// csr_matvecs / TF's SparseTensorDenseMatMul).  Four entries' loads are issued
// before their (in-order) accumulation (eight were measured 1-2 % slower on
// configs R and C2, profiles/r02_planes/gather8_ab).
template <int VEC>
__device__ __forceinline__ typename Vec<VEC>::T row_spmm(const int* __restrict__ col,
                                                         const float* __restrict__ val, int j0,
                                                         int j1, const float* __restrict__ S,
                                                         int Fin, int f0) {
#pragma clang fp contract(off)
  typedef Vec<VEC> V;
  typename V::T acc = V::zero();
  int j = j0;
  for (; j + 4 <= j1; j += 4) {
    const int c0 = col[j], c1 = col[j + 1], c2 = col[j + 2], c3 = col[j + 3];
    const float v0 = val[j], v1 = val[j + 1], v2 = val[j + 2], v3 = val[j + 3];
    const typename V::T t0 = V::ld(S + int64_t(c0) * Fin + f0);
    const typename V::T t1 = V::ld(S + int64_t(c1) * Fin + f0);
    const typename V::T t2 = V::ld(S + int64_t(c2) * Fin + f0);
    const typename V::T t3 = V::ld(S + int64_t(c3) * Fin + f0);
    acc = V::fma_seq(acc, v0, t0);
    acc = V::fma_seq(acc, v1, t1);
    acc = V::fma_seq(acc, v2, t2);
    acc = V::fma_seq(acc, v3, t3);
  }
  for (; j < j1; ++j) acc = V::fma_seq(acc, val[j], V::ld(S + int64_t(col[j]) * Fin + f0));
  return acc;
}

struct ChebStepArgs {
  const int* rowptr;
  const int* col;
  const float* val;
  const int* rperm;   // row visiting order (degree-sorted) or NULL
  const float* Tp;    // T_{k-1}
  const float* Tpp;   // T_{k-2} (k >= 2)
  float* Tout;        // T_k (not last step)
  const float* x;     // T_0 (last step)
  const float* slots; // T_1 .. T_{K-2}, slot_elems apart (last step)
  int64_t slot_elems; // N*M*Fin
  float* basis;       // (last step)
  int M, Fin, K, k;
};

template <int VEC, bool LAST>
__global__ __launch_bounds__(256) void k_cheb_step(ChebStepArgs a, StepGeom g) {
#pragma clang fp contract(off)
  typedef Vec<VEC> V;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int n, rb;
  if (!block_coords(g, &n, &rb)) return;
  const int rsub = lane / g.lpr, lc = lane - rsub * g.lpr;
  if (rsub >= g.rpw) return;
  const int ri = (rb * 4 + wave) * g.rpw + rsub;
  if (ri >= a.M) return;
  const int r = a.rperm ? a.rperm[ri] : ri;
  const int j0 = a.rowptr[r], j1 = a.rowptr[r + 1];
  const int64_t sbase = int64_t(n) * a.M * a.Fin;
  const int64_t rbase = sbase + int64_t(r) * a.Fin;
  const float* S = a.Tp + sbase;
  for (int f0 = lc * VEC; f0 < a.Fin; f0 += g.lpr * VEC) {
    const typename V::T acc = row_spmm<VEC>(a.col, a.val, j0, j1, S, a.Fin, f0);
    const typename V::T o = (a.k >= 2) ? V::two_minus(acc, V::ld(a.Tpp + rbase + f0)) : acc;
    if (!LAST) {
      V::st(a.Tout + rbase + f0, o);
    } else {
      float* brow = a.basis + (int64_t(n) * a.M + r) * int64_t(a.Fin) * a.K;
      for (int kk = 0; kk < a.K - 1; ++kk) {
        const float* Tk = (kk == 0) ? a.x : a.slots + int64_t(kk - 1) * a.slot_elems;
        const typename V::T tv = V::ld(Tk + rbase + f0);
#pragma unroll
        for (int v = 0; v < VEC; ++v) brow[(f0 + v) * a.K + kk] = V::get(tv, v);
      }
#pragma unroll
      for (int v = 0; v < VEC; ++v) brow[(f0 + v) * a.K + a.K - 1] = V::get(o, v);
    }
  }
}

// Last forward step with the basis assembly staged through LDS: each wave
// writes its rows' [fin][k] basis rows into LDS, then stores them with
// coalesced 4-B lane stores (consecutive rows are one contiguous span in the
// natural row order; with rperm each row's Fin*K floats are).  LDS rows are
// Fin*K + 1 floats apart (odd): with Fin*K a multiple of 32 (the ResGNN hidden
// layers, 32 x 20) an unpadded stride put every row of a wave in one bank.
template <int VEC>
__global__ __launch_bounds__(256) void k_cheb_last(ChebStepArgs a, StepGeom g) {
#pragma clang fp contract(off)
  typedef Vec<VEC> V;
  extern __shared__ float stage[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int n, rb;
  if (!block_coords(g, &n, &rb)) return;
  const int FinK = a.Fin * a.K;
  const int ls = FinK + 1;  // LDS row stride
  float* ws = stage + wave * g.rpw * ls;
  const int rsub = lane / g.lpr, lc = lane - rsub * g.lpr;
  const int ri0 = (rb * 4 + wave) * g.rpw;
  const int ri = ri0 + rsub;
  if (rsub < g.rpw && ri < a.M) {
    const int r = a.rperm ? a.rperm[ri] : ri;
    const int j0 = a.rowptr[r], j1 = a.rowptr[r + 1];
    const int64_t sbase = int64_t(n) * a.M * a.Fin;
    const int64_t rbase = sbase + int64_t(r) * a.Fin;
    float* srow = ws + rsub * ls;
    for (int f0 = lc * VEC; f0 < a.Fin; f0 += g.lpr * VEC) {
      const typename V::T acc = row_spmm<VEC>(a.col, a.val, j0, j1, a.Tp + sbase, a.Fin, f0);
      const typename V::T o = (a.k >= 2) ? V::two_minus(acc, V::ld(a.Tpp + rbase + f0)) : acc;
      for (int kk = 0; kk < a.K - 1; ++kk) {
        const float* Tk = (kk == 0) ? a.x : a.slots + int64_t(kk - 1) * a.slot_elems;
        const typename V::T tv = V::ld(Tk + rbase + f0);
#pragma unroll
        for (int v = 0; v < VEC; ++v) srow[(f0 + v) * a.K + kk] = V::get(tv, v);
      }
#pragma unroll
      for (int v = 0; v < VEC; ++v) srow[(f0 + v) * a.K + a.K - 1] = V::get(o, v);
    }
  }
  __syncthreads();
  if (ri0 >= a.M) return;
  const int nrows = (a.M - ri0 < g.rpw) ? a.M - ri0 : g.rpw;
  if (!a.rperm) {
    float* dst = a.basis + (int64_t(n) * a.M + ri0) * FinK;
    const int count = nrows * FinK;
    for (int e = lane; e < count; e += 64) {
      const int q = e / FinK;
      dst[e] = ws[e + q];  // row q at q * (FinK + 1)
    }
  } else {
    for (int q = 0; q < nrows; ++q) {
      float* dst = a.basis + (int64_t(n) * a.M + a.rperm[ri0 + q]) * FinK;
      for (int e = lane; e < FinK; e += 64) dst[e] = ws[q * ls + e];
    }
  }
}

// ---- skinny row GEMM on MFMA --------------------------------------------------------
// C[p][r][j] = sum_k A[r][k] * B_p[k][j] for R (huge) rows, Kc, Nc <= 256:
// the contraction y = basis W (lib/graph_conv.py:175), and dBasis = dy W^T
// written one k-plane at a time (p = k, B_p[f][fin] = W[fin*K + k][f]) so the
// streaming backward reads D_k contiguously.  B_p is staged once per block in
// LDS; blocks are persistent over 128-row tiles (a 32-row tile per wave).
// MFMA 32x32x2 f32 with the k index split in halves: lane (i, h) feeds
// A[r0+i][h*KC2 + s] at step s, read straight from HBM as contiguous
// 64-byte chunks of its half-row (no LDS for A), B[h*KC2 + s][j] from LDS.
struct RowGemmArgs {
  const float* A;
  int64_t R;
  int Kc, lda, KC2;        // KC2 = half of Kc (rounded up to a multiple of 16 when Kc >= 32)
  const float* B;          // B_p[k][j] = B[p*bs_p + k*bs_k + j*bs_j]
  int64_t bs_k, bs_j, bs_p;
  int Nc;
  float* C;
  int ldc;
  int64_t c_plane;
  const float* res;  // epilogue: C = act(C + res)
  int act;
  int pfin;          // > 0: ONE pass computes every plane -- column jj is
                     // (plane jj / pfin, column jj % pfin) of B and of C
  int vecA;          // A rows are 16-byte aligned (lda % 4 == 0): float4 loads
  // A in the planes basis layout (apl_fin > 0): A[r][kk] =
  // A[(kk / apl_fin) * apl_stride + r * apl_fin + kk % apl_fin] (order k =
  // kk / apl_fin, channel kk % apl_fin; lda unused), and B row kk is row
  // (kk % apl_fin) * bmapK + kk / apl_fin of the [Fin*K][Nc] weight
  int apl_fin;
  int64_t apl_stride;
  int bmapK;
};

// PF: the A-chunk prefetch variant (its register ring costs occupancy, so the
// host picks it only for >= 3 full chunks per half: measured D's y GEMM
// -12 %, while the single-chunk dBasis GEMMs of C2 / R lost 6 % with it)
template <int NT, bool PF>
__global__ __launch_bounds__(256) void k_rowgemm(RowGemmArgs a) {
  extern __shared__ float Bs[];  // [2*KC2][NT*32]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int p = blockIdx.y;
  const int KP = 2 * a.KC2, NP = NT * 32;
  for (int e = tid; e < KP * NP; e += 256) {
    const int kk = e / NP, j = e - kk * NP;
    // row kk of the padded operand: half 0 holds k < KC2, half 1 holds KC2 + (kk - KC2)
    const int k = a.apl_fin > 0 ? (kk % a.apl_fin) * a.bmapK + kk / a.apl_fin : kk;
    float v = 0.f;
    if (kk < a.Kc && j < a.Nc) {
      const int pp = a.pfin > 0 ? j / a.pfin : p;
      const int jj = a.pfin > 0 ? j - pp * a.pfin : j;
      v = a.B[pp * a.bs_p + int64_t(k) * a.bs_k + int64_t(jj) * a.bs_j];
    }
    Bs[e] = v;
  }
  __syncthreads();
  float* C = a.C + p * a.c_plane;
  const int64_t ntiles = (a.R + 127) / 128;
  const int kbeg = h * a.KC2;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t r0 = tile * 128 + wave * 32;
    if (r0 >= a.R) continue;
    const int64_t row = (r0 + i < a.R) ? r0 + i : a.R - 1;
    const float* arow = a.A + row * (a.apl_fin > 0 ? a.apl_fin : a.lda);
    // element kk of this row (planes layout: order kk / apl_fin's plane)
    auto aptr = [&](int kk) -> const float* {
      return a.apl_fin > 0 ? arow + (kk / a.apl_fin) * a.apl_stride + kk % a.apl_fin : arow + kk;
    };
    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
    auto mm = [&](const float (&av)[16], int c0, int nq) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (q < nq) {
          const float* brow = Bs + (kbeg + c0 + q) * NP + i;
#pragma unroll
          for (int t = 0; t < NT; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], brow[t * 32], acc[t], 0, 0, 0);
        }
      }
    };
    if constexpr (PF) {
      // every chunk is 16 contiguous in-range floats: loaded two chunks ahead
      // of their MFMAs through a 3-buffer register ring (one wave per SIMD
      // when B fills the LDS, so nothing else hides a chunk's HBM latency)
      auto ld = [&](float (&av)[16], int c0) {
        const float* ap = aptr(kbeg + c0);  // (host: apl_fin % 16 == 0)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 v = *reinterpret_cast<const float4*>(ap + 4 * q);
          av[4 * q] = v.x;
          av[4 * q + 1] = v.y;
          av[4 * q + 2] = v.z;
          av[4 * q + 3] = v.w;
        }
      };
      const int nch = a.KC2 / 16;
      float b0[16], b1[16], b2[16];
      ld(b0, 0);
      if (nch > 1) ld(b1, 16);
      for (int ci = 0; ci < nch; ci += 3) {
        if (ci + 2 < nch) ld(b2, (ci + 2) * 16);
        mm(b0, ci * 16, 16);
        if (ci + 1 < nch) {
          if (ci + 3 < nch) ld(b0, (ci + 3) * 16);
          mm(b1, (ci + 1) * 16, 16);
        }
        if (ci + 2 < nch) {
          if (ci + 4 < nch) ld(b1, (ci + 4) * 16);
          mm(b2, (ci + 2) * 16, 16);
        }
      }
    } else {
      for (int c0 = 0; c0 < a.KC2; c0 += 16) {
        float av[16];
        const int k0 = kbeg + c0;
        const int nq = (a.KC2 - c0 < 16) ? a.KC2 - c0 : 16;  // (small Kc: no padded MFMAs)
        if (a.vecA && nq == 16 && k0 + 16 <= a.Kc) {
          const float* ap = aptr(k0);  // 16 contiguous floats (host: apl_fin % 16 == 0)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 v = *reinterpret_cast<const float4*>(ap + 4 * q);
            av[4 * q] = v.x;
            av[4 * q + 1] = v.y;
            av[4 * q + 2] = v.z;
            av[4 * q + 3] = v.w;
          }
        } else {
#pragma unroll
          for (int q = 0; q < 16; ++q) av[q] = (q < nq && k0 + q < a.Kc) ? *aptr(k0 + q) : 0.f;
        }
        mm(av, c0, nq);
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int jcol = t * 32 + i;
      if (jcol >= a.Nc) continue;
      const int pp = a.pfin > 0 ? jcol / a.pfin : 0;
      const int col = a.pfin > 0 ? jcol - pp * a.pfin : jcol;
      float* Cp = C + pp * a.c_plane;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t rr = r0 + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (rr < a.R) {
          float v = acc[t][q];
          if (a.res) v = v + a.res[rr * a.ldc + col];
          if (a.act) v = v > 0.f ? v : 0.f;
          Cp[rr * a.ldc + col] = v;
        }
      }
    }
  }
}

// ---- the skinny row GEMM on the bf16 matrix pipe, f32-accurate ----------------
// k_rowgemm's job (same arguments, same persistent 128-row tiles, same
// epilogue) with every f32 operand split exactly into three bf16 terms and six
// v_mfma_f32_32x32x16_bf16 per 16-deep k-block (split3 / mfma_x3 below: 2.7x
// the f32 matrix rate at f32 accuracy).  B_p is split ONCE per block into LDS
// in the B-fragment layout [k-block][tile][term][lane] x 16 B (lane (i, h)
// holds B[16 kb + 8h + j][32 t + i], j = 0..7: one ds_read_b128 per fragment);
// lane (i, h) of a wave streams A[r0 + i][16 kb + 8h .. + 7] -- 32 contiguous
// bytes -- from HBM, one k-block ahead of its MFMAs, and splits it in registers.
using x3::bf16x8;
using x3::Split3;
using x3::split3;

template <int NT>
__global__ __launch_bounds__(256) void k_rowgemm_x3(RowGemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char Bx[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int p = blockIdx.y;
  const int KB = (a.Kc + 15) / 16;
  bf16x8* bf = reinterpret_cast<bf16x8*>(Bx);
  for (int e = tid; e < KB * NT * 64; e += 256) {
    const int l = e & 63, t = (e >> 6) % NT, kb = (e >> 6) / NT;
    const int j = t * 32 + (l & 31);
    float v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int kk = kb * 16 + 8 * (l >> 5) + q;
      const int k = a.apl_fin > 0 ? (kk % a.apl_fin) * a.bmapK + kk / a.apl_fin : kk;
      float x = 0.f;
      if (kk < a.Kc && j < a.Nc) {
        const int pp = a.pfin > 0 ? j / a.pfin : p;
        const int jj = a.pfin > 0 ? j - pp * a.pfin : j;
        x = a.B[pp * a.bs_p + int64_t(k) * a.bs_k + int64_t(jj) * a.bs_j];
      }
      v[q] = x;
    }
    const Split3 sp = split3(v);
    bf16x8* d = bf + ((kb * NT + t) * 3) * 64 + l;
    d[0] = sp.hi;
    d[64] = sp.mid;
    d[128] = sp.lo;
  }
  __syncthreads();
  float* C = a.C + p * a.c_plane;
  const int64_t ntiles = (a.R + 127) / 128;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t r0 = tile * 128 + wave * 32;
    if (r0 >= a.R) continue;
    const int64_t row = (r0 + i < a.R) ? r0 + i : a.R - 1;
    const float* arow = a.A + row * (a.apl_fin > 0 ? a.apl_fin : a.lda);
    // elements 16 kb + 8h .. + 7 of this row (planes layout: apl_fin % 16 == 0,
    // so the eight sit in one plane)
    auto ld = [&](float (&v)[8], int kb) {
      const int k0 = kb * 16 + 8 * h;
      const float* ap = a.apl_fin > 0 ? arow + (k0 / a.apl_fin) * a.apl_stride + k0 % a.apl_fin : arow + k0;
      if (a.vecA && k0 + 8 <= a.Kc) {
        const float4 x0 = *reinterpret_cast<const float4*>(ap);
        const float4 x1 = *reinterpret_cast<const float4*>(ap + 4);
        v[0] = x0.x, v[1] = x0.y, v[2] = x0.z, v[3] = x0.w;
        v[4] = x1.x, v[5] = x1.y, v[6] = x1.z, v[7] = x1.w;
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = k0 + q < a.Kc ? ap[q] : 0.f;
      }
    };
    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[t][q] = 0.f;
    float va[8];
    ld(va, 0);
    for (int kb = 0; kb < KB; ++kb) {
      const Split3 xa = split3(va);
      if (kb + 1 < KB) ld(va, kb + 1);  // the next k-block in flight during the MFMAs
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const bf16x8* f = bf + ((kb * NT + t) * 3) * 64 + lane;
        Split3 yb;
        yb.hi = f[0];
        yb.mid = f[64];
        yb.lo = f[128];
        acc[t] = x3::mfma32_x3(xa, yb, acc[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int jcol = t * 32 + i;
      if (jcol >= a.Nc) continue;
      const int pp = a.pfin > 0 ? jcol / a.pfin : 0;
      const int col = a.pfin > 0 ? jcol - pp * a.pfin : jcol;
      float* Cp = C + pp * a.c_plane;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t rr = r0 + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (rr < a.R) {
          float v = acc[t][q];
          if (a.res) v = v + a.res[rr * a.ldc + col];
          if (a.act) v = v > 0.f ? v : 0.f;
          Cp[rr * a.ldc + col] = v;
        }
      }
    }
  }
}

// Reverse (Clenshaw) step over L~^T in the sample-major layout:
//   G_k = D_k + c * (L~^T G_{k+1}) - G_{k+2},  c = 2 (k >= 1) or 1 (k = 0),
// D_k = plane k of dBasis in the k-major layout [K][N][M][Fin] (written so by
// the dy W^T GEMM); k = 0 writes dx [N][M][Fin] directly.
struct ClenArgs {
  const int* rowptr;
  const int* col;
  const float* val;
  const int* rperm;
  const float* Gn1;  // G_{k+1}
  const float* Gn2;  // G_{k+2}
  float* Gout;       // G_k (or dx when k == 0)
  const float* Dk;   // D_k plane
  int M, Fin, K, k;
  int dx_acc;        // k == 0: dx += G_0
};

template <int VEC>
__global__ __launch_bounds__(256) void k_clenshaw_step(ClenArgs a, StepGeom g) {
#pragma clang fp contract(off)
  typedef Vec<VEC> V;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int n, rb;
  if (!block_coords(g, &n, &rb)) return;
  const int rsub = lane / g.lpr, lc = lane - rsub * g.lpr;
  if (rsub >= g.rpw) return;
  const int ri = (rb * 4 + wave) * g.rpw + rsub;
  if (ri >= a.M) return;
  const int r = a.rperm ? a.rperm[ri] : ri;
  const int j0 = a.rowptr[r], j1 = a.rowptr[r + 1];
  const int64_t sbase = int64_t(n) * a.M * a.Fin;
  const int64_t rbase = sbase + int64_t(r) * a.Fin;
  const bool has1 = (a.k + 1) <= (a.K - 1), has2 = (a.k + 2) <= (a.K - 1);
  const float c = (a.k >= 1) ? 2.f : 1.f;
  for (int f0 = lc * VEC; f0 < a.Fin; f0 += g.lpr * VEC) {
    typename V::T acc = V::zero();
    if (has1) acc = row_spmm<VEC>(a.col, a.val, j0, j1, a.Gn1 + sbase, a.Fin, f0);
    typename V::T o = V::add_c_sub(V::ld(a.Dk + rbase + f0), c, acc);
    if (has2) o = V::sub(o, V::ld(a.Gn2 + rbase + f0));
    if (a.dx_acc && a.k == 0) o = V::add(V::ld(a.Gout + rbase + f0), o);
    V::st(a.Gout + rbase + f0, o);
  }
}

StepGeom step_geom(int N, int M, int Fin, int vec) {
  StepGeom g;
  const int lanes = (Fin + vec - 1) / vec;
  g.lpr = lanes < 64 ? lanes : 64;
  g.rpw = 64 / g.lpr;
  g.rb = (M + 4 * g.rpw - 1) / (4 * g.rpw);
  // sample-per-XCD mapping keeps each XCD's gathers inside one sample slab in
  // its own 4 MB L2; slabs larger than that are better shared by all XCDs at
  // once (all blocks of sample n before sample n+1) so the one slab being
  // gathered stays in the 256 MB Infinity Cache.  N not a multiple of 8 (the
  // humanflow ResGNN's batch of 100) pads the grid to 8 * ceil(N / 8) samples
  // rather than falling back to the sample-major order, which spreads every
  // sample's blocks over all 8 XCDs (each L2 then holds all N slabs)
  const int64_t slab = int64_t(M) * Fin * 4;
  g.xcd_map = (slab <= (int64_t(2) << 20)) ? 1 : 0;
  g.N = N;
  const int64_t ns = g.xcd_map ? (int64_t(N) + 7) / 8 * 8 : int64_t(N);
  g.grid = unsigned(ns * g.rb);
  return g;
}

// C = op(A) op(B), 64x64 output tile per 256-thread block, each wave a 32x32
// MFMA tile; BK = 16 staged through LDS ([k][row] images so an MFMA operand
// read is 32 consecutive floats).
template <bool TA, bool TB>
__global__ __launch_bounds__(256) void k_gemm_f32(int Mg, int Ng, int Kg, const float* __restrict__ A,
                                                  int lda, const float* __restrict__ B, int ldb,
                                                  float* __restrict__ C, int ldc, int kchunk,
                                                  int remapK) {
  __shared__ float As[16][68];
  __shared__ float Bs[16][68];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int h = lane >> 5, li = lane & 31;
  const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  const int kbeg = blockIdx.z * kchunk;
  const int kend = (kbeg + kchunk < Kg) ? (kbeg + kchunk) : Kg;
  C += size_t(blockIdx.z) * size_t(Mg) * ldc;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int k0 = kbeg; k0 < kend; k0 += 16) {
#pragma unroll
    for (int e0 = 0; e0 < 1024; e0 += 256) {
      const int e = e0 + tid;
      int row, kk;
      if (!TA) { row = e >> 4; kk = e & 15; } else { kk = e >> 6; row = e & 63; }
      const int gm = m0 + row, gk = k0 + kk;
      float v = 0.f;
      if (gm < Mg && gk < kend) v = TA ? A[size_t(gk) * lda + gm] : A[size_t(gm) * lda + gk];
      As[kk][row] = v;
    }
#pragma unroll
    for (int e0 = 0; e0 < 1024; e0 += 256) {
      const int e = e0 + tid;
      int cc, kk;
      if (!TB) { kk = e >> 6; cc = e & 63; } else { cc = e >> 4; kk = e & 15; }
      const int gn = n0 + cc, gk = k0 + kk;
      float v = 0.f;
      if (gn < Ng && gk < kend) v = TB ? B[size_t(gn) * ldb + gk] : B[size_t(gk) * ldb + gn];
      Bs[kk][cc] = v;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const float a = As[2 * s + h][wr * 32 + li];
      const float b = Bs[2 * s + h][wc * 32 + li];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  const int col = n0 + wc * 32 + li;
  // remapK > 0: column col = fin*K + k of row `row` goes to plane k of a
  // [K][Mg][Ng/K] tensor (dBasis in the streaming backward's k-major layout)
  const int rk = remapK > 0 ? remapK : 1;
  const int64_t cidx = remapK > 0 ? int64_t(col % rk) * Mg * (Ng / rk) + col / rk : col;
  const int64_t rstride = remapK > 0 ? int64_t(Ng / rk) : int64_t(ldc);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (row < Mg && col < Ng) C[int64_t(row) * rstride + cidx] = acc[r];
  }
}

// dW partial slabs: slab[z][j][f] = sum_{r in chunk z} basis[r][j] * dy[r][f]
// over the R = N*M basis rows (j < FinK, f < Fout): a skinny TN GEMM whose
// inner dimension is the whole batch.  Block (z, g) = 4 waves owns chunk z and
// a group of up to 16 of the 32x32 (j, f) output tiles (all of them when
// FinK/32 * Fout/32 <= 16), so every basis and dy row of the chunk is read
// from HBM ONCE per group (the earlier one-tile-per-block grid read the basis
// Fout/32 times and dy FinK/32 times: 3x the compulsory bytes on config D,
// r03 PMC).  The chunk's rows stream through LDS in batches of 16 (the next
// batch's 16-B loads are in flight in registers while the 4 waves run the
// current one); wave w accumulates tiles w, w+4, .. of the group on
// v_mfma_f32_32x32x2_f32 (K = 2 rows per MFMA: lane half h takes the odd
// rows), one tile per accumulator, rows in order -- bitwise reproducible.
// pl_fin > 0: the basis is in the planes layout (column jj = k*pl_fin + fin of
// row r at basis[k*pl_stride + r*pl_fin + fin]); the slab keeps the rows
// layout's column order fin*K + k.
// xb != NULL (the gconv-LSTM weight gradients in one pass over dpre): FinKh
// planes columns from `basis`, then x_fin*K planes columns from xb (plane
// stride x_stride, slab column FinKh + fin*K + k) and one column of ones
// (slab column FinK - 1: the bias gradient); FinK counts all of them.
constexpr int kDwRB = 16;     // rows per LDS batch (4 per wave)
constexpr int kDwTiles = 16;  // output tiles per block at most (4 per wave)
constexpr int kDwNA = 2;      // basis pieces per lane and staged row (64 lanes x VW floats each)
// dy pieces per lane and staged row: Fout <= 256 either way
template <int VW> constexpr int dw_nb() { return VW == 4 ? 1 : 4; }

// NW waves per block (4 or 8): wave w stages rows w*(16/NW) .. of a batch and
// accumulates tiles w, w+NW, ..; a tile's MFMA sequence over the rows is the
// same whatever NW, so the slabs are bitwise independent of it.
template <int VW, int NW>  // VW 4: float4 pieces (FinK, Fout, pl_fin multiples of 4), 1: floats
__global__ __launch_bounds__(64 * NW) void k_dw_slabs(const float* __restrict__ basis,
                                                  const float* __restrict__ dy, int64_t R,
                                                  int FinK, int Fout, int64_t rows_per_chunk,
                                                  float* __restrict__ slab, int pl_fin,
                                                  int64_t pl_stride, int K, int tpb,
                                                  const float* __restrict__ xb, int x_fin,
                                                  int64_t x_stride, int FinKh, int ldd) {
  typedef typename std::conditional<VW == 4, float4, float>::type V;
  constexpr int kDwNB = dw_nb<VW>();
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int ftl = (Fout + 31) >> 5;
  const int ntiles = ((FinK + 31) >> 5) * ftl;
  const int t0 = blockIdx.y * tpb;
  const int t1 = (t0 + tpb < ntiles) ? t0 + tpb : ntiles;
  // the group's basis columns [jlo, jhi) (tiles are jt-major) and all of dy
  const int jlo = (t0 / ftl) * 32;
  const int jhi0 = ((t1 - 1) / ftl + 1) * 32;
  const int jhi = jhi0 < FinK ? jhi0 : FinK;
  const int SA = ((jhi0 - jlo) | 1);         // LDS row strides (odd: the two half-wave
  const int SB = (((Fout + 31) & ~31) | 1);  // rows of an operand read hit other banks)
  float* s_a = sm;               // [kDwRB][SA]
  float* s_b = sm + kDwRB * SA;  // [kDwRB][SB]
  const int64_t c0 = int64_t(blockIdx.x) * rows_per_chunk;
  const int64_t c1 = (c0 + rows_per_chunk < R) ? c0 + rows_per_chunk : R;
  for (int e = threadIdx.x; e < kDwRB * SA; e += 64 * NW) s_a[e] = 0.f;  // padding columns
  for (int e = threadIdx.x; e < kDwRB * SB; e += 64 * NW) s_b[e] = 0.f;
  // this lane's pieces of a staged row: basis columns jlo + VW*(lane + 64 i),
  // dy columns VW*(lane + 64 i); their offsets from the row's base
  int64_t aoff[kDwNA];
  bool av[kDwNA], bv[kDwNB];
  const int jhb = jhi < FinKh ? jhi : FinKh;  // the group's columns from `basis`
#pragma unroll
  for (int i = 0; i < kDwNA; ++i) {
    const int cc = jlo + VW * (lane + 64 * i);
    av[i] = cc < jhb;
    aoff[i] = pl_fin > 0 ? int64_t(cc / pl_fin) * pl_stride + cc % pl_fin : cc;
  }
#pragma unroll
  for (int i = 0; i < kDwNB; ++i) bv[i] = VW * (lane + 64 * i) < Fout;
  const int64_t ald = pl_fin > 0 ? pl_fin : FinKh;  // basis row stride
  // the extra columns (xb): lane e stages column FinKh + e of each row
  const int nxc = xb ? x_fin * K : 0;
  const int xcol = FinKh + lane;
  const bool xv = xb && lane <= nxc && xcol >= jlo && xcol < jhi;
  const int64_t xoff = lane < nxc ? int64_t(lane / x_fin) * x_stride + lane % x_fin : 0;
  constexpr int NR = kDwRB / NW;  // rows per wave and batch
  V ra[NR][kDwNA], rbv[NR][kDwNB];
  float rx[NR];
  auto fetch = [&](int64_t rb) {  // rows rb + NR w .. rb + NR w + NR - 1 into registers
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      const int64_t rr = rb + NR * w + q;
      const bool rv = rr < c1;
      if (xv) rx[q] = lane == nxc ? 1.f : rv ? xb[xoff + rr * x_fin] : 0.f;
#pragma unroll
      for (int i = 0; i < kDwNA; ++i)
        if (av[i]) ra[q][i] = rv ? *reinterpret_cast<const V*>(basis + rr * ald + aoff[i]) : V{};
#pragma unroll
      for (int i = 0; i < kDwNB; ++i)
        if (bv[i]) rbv[q][i] = rv ? *reinterpret_cast<const V*>(dy + rr * ldd + VW * (lane + 64 * i)) : V{};
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      float* da = s_a + (NR * w + q) * SA;
      float* db = s_b + (NR * w + q) * SB;
      if (xv) da[xcol - jlo] = rx[q];
#pragma unroll
      for (int i = 0; i < kDwNA; ++i)
        if (av[i]) {
          const float* v = reinterpret_cast<const float*>(&ra[q][i]);
#pragma unroll
          for (int c = 0; c < VW; ++c) da[VW * (lane + 64 * i) + c] = v[c];
        }
#pragma unroll
      for (int i = 0; i < kDwNB; ++i)
        if (bv[i]) {
          const float* v = reinterpret_cast<const float*>(&rbv[q][i]);
#pragma unroll
          for (int c = 0; c < VW; ++c) db[VW * (lane + 64 * i) + c] = v[c];
        }
    }
  };
  constexpr int NT = kDwTiles / NW;  // tiles per wave
  f32x16 acc[NT];
#pragma unroll
  for (int a = 0; a < NT; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;
  __syncthreads();  // padding zeroed before the first stage
  if (c0 < c1) fetch(c0);
  for (int64_t rb = c0; rb < c1; rb += kDwRB) {
    stage();
    __syncthreads();
    if (rb + kDwRB < c1) fetch(rb + kDwRB);  // in flight during the MFMAs
#pragma unroll
    for (int a = 0; a < NT; ++a) {
      const int t = t0 + w + NW * a;
      if (t < t1) {
        const int jt = t / ftl, ft = t - jt * ftl;
        const float* pa = s_a + h * SA + (jt * 32 - jlo) + li;
        const float* pb = s_b + h * SB + ft * 32 + li;
#pragma unroll
        for (int u = 0; u < kDwRB / 2; ++u)
          acc[a] = __builtin_amdgcn_mfma_f32_32x32x2f32(pa[2 * u * SA], pb[2 * u * SB], acc[a], 0, 0, 0);
      }
    }
    __syncthreads();  // the batch buffers are restaged next
  }
#pragma unroll
  for (int a = 0; a < NT; ++a) {
    const int t = t0 + w + NW * a;
    if (t >= t1) continue;
    const int jt = t / ftl, ft = t - jt * ftl;
    const int ff = ft * 32 + li;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int jj = jt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      const int jx = jj - FinKh;
      const int jo = jj >= FinKh ? (jx < nxc ? FinKh + (jx % x_fin) * K + jx / x_fin : jj)
                                 : pl_fin > 0 ? (jj % pl_fin) * K + jj / pl_fin : jj;
      if (jj < FinK && ff < Fout) slab[(int64_t(blockIdx.x) * FinK + jo) * ldd + ff] = acc[a][r];
    }
  }
}

// ---- dW on registers only: k_dw_direct -----------------------------------
// The slabs of k_dw_slabs, bitwise -- the same chunks, the same row pairs in
// the same order for every output element, the same v_mfma_f32_32x32x2_f32 --
// without LDS or barriers: each wave owns one chunk and NA x NB output tiles of
// it (a column group grp of the basis, all of dy) and streams the chunk's rows
// straight from HBM into the MFMA operand registers, PD row pairs in flight.
// Lane (i, h) of an MFMA needs column i of row r + h of each operand; a
// V-float load gives a lane V consecutive columns V*i .. V*i + V-1 of one row,
// i.e. its operand for V "virtual tiles" (tile e holds the columns V*i + e):
// a permutation of where an output element sits in the accumulators, not of
// the products summed into it.  For large row counts (config D: 65 536 rows
// per chunk) this replaces k_dw_slabs' 16-row LDS batches and their two
// barriers per batch.
struct DwDirectArgs {
  const float* basis;
  const float* dy;
  int64_t R, rpc;
  int chunks, G;         // chunks x column groups = waves
  int FinKh, Fout, ldd;  // basis columns, dy columns (this slice), dy / slab row stride
  float* slab;
  int pl_fin;            // > 0: planes layout (column jj = k*pl_fin + fin)
  int64_t pl_stride;
  int K;
  // the gconv-LSTM's extra columns (VA == 1 only), as k_dw_slabs' xb: x planes
  // (x column e = plane e / x_fin, fin e % x_fin at xb + plane*x_stride + r*x_fin
  // + fin, slab column FinKh + fin*K + plane) then one column of ones
  const float* xb;
  int x_fin, nxc, FinK;  // nxc = x_fin*K; FinK = FinKh (+ nxc + 1 with xb)
  int64_t x_stride;
};

template <int V> struct DwVec { typedef float T; };
template <> struct DwVec<2> { typedef float2 T; };
template <> struct DwVec<4> { typedef float4 T; };
template <int V> __device__ __forceinline__ float dw_el(const typename DwVec<V>::T& v, int e) {
  return reinterpret_cast<const float*>(&v)[e];
}

template <int VA, int NLA, int VB, int NLB, int PD>
__device__ __forceinline__ void dw_direct_body(const DwDirectArgs& A) {
  typedef typename DwVec<VA>::T TA;
  typedef typename DwVec<VB>::T TB;
  constexpr int NA = VA * NLA, NB = VB * NLB;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int gw = blockIdx.x * 4 + w;
  const int chunk = gw / A.G, grp = gw - chunk * A.G;
  if (chunk >= A.chunks) return;
  const int64_t c0 = int64_t(chunk) * A.rpc;
  const int64_t c1 = (c0 + A.rpc < A.R) ? c0 + A.rpc : A.R;
  const int cg0 = grp * 32 * NA;  // the group's first basis column
  const int64_t ald = A.pl_fin > 0 ? A.pl_fin : A.FinKh;
  const float* pa[NLA];
  int lst[NLA];  // the load's row stride (floats): basis rows or x-plane rows
  bool av[NLA], aone[NLA];
#pragma unroll
  for (int q = 0; q < NLA; ++q) {
    const int c = cg0 + 32 * VA * q + VA * li;
    av[q] = c < A.FinKh;
    aone[q] = false;
    const int64_t off = A.pl_fin > 0 ? int64_t(c / A.pl_fin) * A.pl_stride + c % A.pl_fin : c;
    pa[q] = A.basis + (av[q] ? off : 0) + (c0 + h) * ald;
    lst[q] = int(ald);
    if (VA == 1 && A.xb && !av[q]) {
      const int e = c - A.FinKh;
      if (e < A.nxc) {
        av[q] = true;
        pa[q] = A.xb + int64_t(e / A.x_fin) * A.x_stride + e % A.x_fin + (c0 + h) * A.x_fin;
        lst[q] = A.x_fin;
      } else if (e == A.nxc) {
        aone[q] = true;  // the bias gradient's column of ones
      }
    }
  }
  const float* pb[NLB];
  bool bv[NLB];
#pragma unroll
  for (int q = 0; q < NLB; ++q) {
    const int f = 32 * VB * q + VB * li;
    bv[q] = f < A.Fout;
    pb[q] = A.dy + (bv[q] ? f : 0) + (c0 + h) * int64_t(A.ldd);
  }
  const int64_t npairs = (c1 - c0 + 1) >> 1;
  TA ra[PD][NLA];
  TB rb[PD][NLB];
  bool rvs[PD];
  // row pair p into ring slot s, RAW: the loads are unconditional (a row past
  // the chunk reads the chunk's first row, an idle column column 0) and the
  // zeros are selected in consume(), one loop iteration later.  A select next
  // to its load lets the compiler sink the load into a branch on the row's
  // validity with a vmcnt(0) wait behind it -- which serialises the ring.
  auto fetch = [&](int s, int64_t p) {
    const bool rv = c0 + 2 * p + h < c1;
    rvs[s] = rv;
    const int64_t ro = rv ? 2 * p : -int64_t(h);  // row c0 + h + ro (row c0 when idle)
#pragma unroll
    for (int q = 0; q < NLA; ++q) ra[s][q] = *reinterpret_cast<const TA*>(pa[q] + ro * lst[q]);
#pragma unroll
    for (int q = 0; q < NLB; ++q)
      rb[s][q] = *reinterpret_cast<const TB*>(pb[q] + ro * int64_t(A.ldd));
  };
  f32x16 acc[NA][NB];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
#pragma unroll
  for (int s = 0; s < PD; ++s) fetch(s, s);
  // full rounds of PD pairs with no control flow (the compiler then counts the
  // ring's loads: each MFMA group waits only for its own slot), then the tail;
  // a pair past the chunk (p >= npairs) is never consumed; the missing row of
  // an odd chunk's last pair and idle columns enter as zeros
  auto consume = [&](int s) {
    const bool rv = rvs[s];
    float y[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const float v = dw_el<VB>(rb[s][b / VB], b % VB);
      y[b] = (rv && bv[b / VB]) ? v : 0.f;
    }
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      float x = dw_el<VA>(ra[s][a / VA], a % VA);
      x = (rv && av[a / VA]) ? x : 0.f;
      if constexpr (VA == 1) x = aone[a] ? (rv ? 1.f : 0.f) : x;
#pragma unroll
      for (int b = 0; b < NB; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y[b], acc[a][b], 0, 0, 0);
    }
  };
  const int64_t nfull = npairs / PD * PD;
  for (int64_t p0 = 0; p0 < nfull; p0 += PD) {
#pragma unroll
    for (int s = 0; s < PD; ++s) {
      consume(s);
      fetch(s, p0 + s + PD);
      // keep slot s's loads right behind its MFMAs (a rolling ring); the
      // scheduler otherwise hoists every MFMA of the round ahead of all the
      // round's loads, and the next round waits out a whole memory latency
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int s = 0; s < PD; ++s)
    if (nfull + s < npairs) consume(s);
  // tile (a, b), accumulator r: A lane i = (r & 3) + 8 (r >> 2) + 4 h, B lane li
  const int FinK = A.FinK;
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int f = 32 * VB * (b / VB) + VB * li + b % VB;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int c = cg0 + 32 * VA * (a / VA) + VA * i + a % VA;
        const int jx = c - A.FinKh;
        const int jo = c >= A.FinKh ? (jx < A.nxc ? A.FinKh + (jx % A.x_fin) * A.K + jx / A.x_fin : c)
                                    : A.pl_fin > 0 ? (c % A.pl_fin) * A.K + c / A.pl_fin : c;
        if (c < FinK && f < A.Fout)
          A.slab[(int64_t(chunk) * FinK + jo) * A.ldd + f] = acc[a][b][r];
      }
    }
}

// one wave per SIMD (up to 512 registers: the deep rings / wide tile sets)
template <int VA, int NLA, int VB, int NLB, int PD>
__global__ __launch_bounds__(256) void k_dw_direct(DwDirectArgs A) {
  dw_direct_body<VA, NLA, VB, NLB, PD>(A);
}
// two waves per SIMD (<= 256 registers): one wave's loads run under the
// other's MFMAs, for the instantiations that fit without spills
template <int VA, int NLA, int VB, int NLB, int PD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_dw_direct2(DwDirectArgs A) {
  dw_direct_body<VA, NLA, VB, NLB, PD>(A);
}

// ---- dW on the bf16 matrix pipe, f32-accurate: k_dw_x3s ------------------
// The split arithmetic of split_bf16.h on v_mfma_f32_32x32x16_bf16.  Sums run
// in another order than k_dw_slabs', so dW agrees to f32 rounding, not bitwise
// (tests/test_gpu_dw_x3.py bounds both against float64).  (A register-only
// form -- k_dw_direct's layout, two basis-column groups so dy was read twice
// -- took 470 us on config E's pass against this kernel's 407-425 and was
// dropped: profiles/r06_x3.)  Lane (i, h) of the MFMA holds rows 8h .. 8h+7 of
// a 16-row block for column i of each operand (the bf16 A/B lane map).
// k_dw_x3s: dy read ONCE per chunk however
// many basis tiles there are.  One workgroup per chunk, one wave per 32-column
// basis tile (FinK <= 256); the chunk's rows go in batches of 32: every wave
// loads its own basis tile straight into registers, while the dy batch (NBT
// tiles of 32 columns) is loaded once by the workgroup, split, and written to
// LDS already in the MFMA's B-fragment layout ([piece][k-block][tile][lane]
// x 16 B: a lane's fragment is one conflict-free ds_read_b128), double
// buffered with one barrier per batch.  The staging is spread over every
// thread of the workgroup: a task is one float4 (4 columns) of RPT consecutive
// rows, i.e. RPT elements of the fragments of 4 lanes, split in registers and
// written as RPT bf16 per piece (the barrier waits for the slowest wave, so a
// stage done by a few waves stalls all of them).
constexpr int kX3Rows = 32;  // rows per batch (two 16-row k-blocks)
template <int RPT>
__device__ __forceinline__ void x3_put(char* p, const float (&v)[RPT]) {
  // the upper halves of v (hi terms: truncation), RPT bf16 at p (2 * RPT bytes)
  if constexpr (RPT == 1) {
    *reinterpret_cast<unsigned short*>(p) = static_cast<unsigned short>(__float_as_uint(v[0]) >> 16);
  } else {
    unsigned wv[RPT / 2];
#pragma unroll
    for (int i = 0; i < RPT / 2; ++i)
      wv[i] = __builtin_amdgcn_perm(__float_as_uint(v[2 * i + 1]), __float_as_uint(v[2 * i]), 0x07060302u);
    if constexpr (RPT == 2) {
      *reinterpret_cast<unsigned*>(p) = wv[0];
    } else if constexpr (RPT == 4) {
      *reinterpret_cast<uint2*>(p) = make_uint2(wv[0], wv[1]);
    } else {
      *reinterpret_cast<uint4*>(p) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
    }
  }
}
template <int NBT, int RPT>
__global__ __launch_bounds__(512) void k_dw_x3s(DwDirectArgs A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int FRAG = 2 * NBT * 64;      // fragments per piece per batch (2 k-blocks)
  constexpr int BUF = 3 * FRAG * 16;      // bytes per batch buffer
  constexpr int NCQ = 8 * NBT;            // float4 column groups of the dy batch
  constexpr int TASKS = (32 / RPT) * NCQ;  // (column group, RPT-row group) staging tasks
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int chunk = blockIdx.x;
  const int64_t c0 = int64_t(chunk) * A.rpc;
  const int64_t c1 = (c0 + A.rpc < A.R) ? c0 + A.rpc : A.R;
  const int64_t nb = (c1 - c0 + kX3Rows - 1) / kX3Rows;
  // this wave's basis column (tile w), VA = 1 (x planes / ones as k_dw_direct)
  const int c = 32 * w + li;
  const int64_t ald = A.pl_fin > 0 ? A.pl_fin : A.FinKh;
  bool av = c < A.FinKh, aone = false;
  const float* pa = A.basis + (av ? (A.pl_fin > 0 ? int64_t(c / A.pl_fin) * A.pl_stride + c % A.pl_fin : c) : 0) +
                    (c0 + 8 * h) * ald;
  int64_t lst = ald;
  if (A.xb && !av) {
    const int e = c - A.FinKh;
    if (e < A.nxc) {
      av = true;
      pa = A.xb + int64_t(e / A.x_fin) * A.x_stride + e % A.x_fin + (c0 + 8 * h) * A.x_fin;
      lst = A.x_fin;
    } else if (e == A.nxc) {
      aone = true;
    }
  }
  // staging task of this thread (if any): column group cq, batch rows
  // RPT rg .. RPT rg + RPT - 1 = k-block kr >> 4, lane half (kr >> 3) & 1,
  // fragment elements kr & 7 ..
  const bool stg = tid < TASKS;
  const int cq = tid % NCQ, rg = tid / NCQ, kr = RPT * rg;
  const bool bvq = stg && 4 * cq < A.Fout;  // Fout % 4 == 0: a group is all in or all out
  const float* pb = A.dy + (bvq ? 4 * cq : 0) + (c0 + kr) * int64_t(A.ldd);
  const int sfr = ((kr >> 4) * NBT + (cq >> 3)) * 64 + 4 * (cq & 7) + 32 * ((kr >> 3) & 1);
  const int sby = 2 * (kr & 7);  // byte offset of the task's elements in a fragment
  float ra[2][8];     // this lane's basis rows of the batch: k-block kb, element j
  float4 rb[RPT];     // the staging task's dy rows
  int nva[2], nvb;
  auto fetch = [&](int64_t bi) {
    const int64_t r0 = 32 * bi;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const int64_t left = c1 - (c0 + r0 + 16 * kb + 8 * h);
      nva[kb] = left <= 0 ? 0 : left >= 8 ? 8 : int(left);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t ro = j < nva[kb] ? r0 + 16 * kb + j : -8 * int64_t(h);
        ra[kb][j] = pa[ro * lst];
      }
    }
    const int64_t left = c1 - (c0 + r0 + kr);
    nvb = left <= 0 ? 0 : left >= RPT ? RPT : int(left);
    if (stg) {
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const int64_t ro = j < nvb ? r0 + j : -int64_t(kr);
        rb[j] = *reinterpret_cast<const float4*>(pb + ro * int64_t(A.ldd));
      }
    }
  };
  f32x16 acc[NBT];
#pragma unroll
  for (int b = 0; b < NBT; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;
  if (nb > 0) fetch(0);
  for (int64_t bi = 0; bi < nb; ++bi) {
    char* buf = smem + (bi & 1) * BUF;
    if (stg) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float y[RPT], r[RPT], q[RPT];
#pragma unroll
        for (int j = 0; j < RPT; ++j) {
          const float v = reinterpret_cast<const float*>(&rb[j])[e];
          y[j] = (j < nvb && bvq) ? v : 0.f;
          r[j] = y[j] - __uint_as_float(__float_as_uint(y[j]) & 0xffff0000u);  // exact
          q[j] = r[j] - __uint_as_float(__float_as_uint(r[j]) & 0xffff0000u);  // exact
        }
        char* f = buf + (sfr + e) * 16 + sby;
        x3_put<RPT>(f, y);
        x3_put<RPT>(f + FRAG * 16, r);
        x3_put<RPT>(f + 2 * FRAG * 16, q);
      }
    }
    Split3 xa[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = (j < nva[kb] && av) ? ra[kb][j] : 0.f;
        x[j] = aone ? (j < nva[kb] ? 1.f : 0.f) : v;
      }
      xa[kb] = split3(x);
    }
    __syncthreads();  // the batch's fragments are in; the other buffer is free
    if (bi + 1 < nb) fetch(bi + 1);  // in flight during the MFMAs
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int b = 0; b < NBT; ++b) {
        const int fr = (kb * NBT + b) * 64 + lane;
        Split3 yb;
        yb.hi = *reinterpret_cast<const bf16x8*>(buf + (0 * FRAG + fr) * 16);
        yb.mid = *reinterpret_cast<const bf16x8*>(buf + (1 * FRAG + fr) * 16);
        yb.lo = *reinterpret_cast<const bf16x8*>(buf + (2 * FRAG + fr) * 16);
        acc[b] = x3::mfma32_x3(xa[kb], yb, acc[b]);
      }
  }
  // tile (w, b): k_dw_direct's store layout
  const int FinK = A.FinK;
#pragma unroll
  for (int b = 0; b < NBT; ++b) {
    const int f = 32 * b + li;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int cc = 32 * w + (r & 3) + 8 * (r >> 2) + 4 * h;
      const int jx = cc - A.FinKh;
      const int jo = cc >= A.FinKh ? (jx < A.nxc ? A.FinKh + (jx % A.x_fin) * A.K + jx / A.x_fin : cc)
                                   : A.pl_fin > 0 ? (cc % A.pl_fin) * A.K + cc / A.pl_fin : cc;
      if (cc < FinK && f < A.Fout) A.slab[(int64_t(chunk) * FinK + jo) * A.ldd + f] = acc[b][r];
    }
  }
}

// out[i] = sum_z slab[z][i] in a FIXED order (bitwise reproducible): wave w of
// a block sums the slabs z = w, w+16, ... for 64 consecutive outputs (one
// 256-B coalesced load per slab, 8 in flight), then the 16 partial sums are
// added in wave order through LDS.
template <class OUT>
__device__ __forceinline__ void reduce_slabs_body(const float* __restrict__ slab, int nslab,
                                                  int64_t count, OUT&& out) {
#pragma clang fp contract(off)
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i = int64_t(blockIdx.x) * 64 + lane;
  float s = 0.f;
  if (i < count) {
    // this lane's slabs z = w, w + 16, ..: up to 16 loads in flight at once,
    // then added in order (the same order as one load per add)
    for (int z0 = w; z0 < nslab; z0 += 256) {
      float vz[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int z = z0 + 16 * q;
        vz[q] = z < nslab ? slab[int64_t(z) * count + i] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (z0 + 16 * q < nslab) s = s + vz[q];
    }
  }
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && i < count) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t = t + part[q][lane];
    out(i, t);
  }
}

__global__ __launch_bounds__(1024) void k_reduce_slabs(const float* __restrict__ slab, int nslab,
                                                       int64_t count, float* __restrict__ out,
                                                       int accumulate) {
#pragma clang fp contract(off)
  reduce_slabs_body(slab, nslab, count, [&](int64_t i, float t) {
    out[i] = accumulate ? out[i] + t : t;
  });
}

// the same sums, elements [0, n0) into out0, [n0, n01) into out1, the rest
// into out2 (the gconv-LSTM's dWh | dWx | db of one slab row block)
__global__ __launch_bounds__(1024) void k_reduce_slabs3(const float* __restrict__ slab, int nslab,
                                                        int64_t count, float* __restrict__ out0,
                                                        int64_t n0, float* __restrict__ out1,
                                                        int64_t n01, float* __restrict__ out2) {
  reduce_slabs_body(slab, nslab, count, [&](int64_t i, float t) {
    if (i < n0)
      out0[i] = t;
    else if (i < n01)
      out1[i - n0] = t;
    else
      out2[i - n01] = t;
  });
}

// dW = basis^T dy of a small problem in one block (config A: N*M = 3 200 rows,
// FinK = 5, Fout = 4).  One CU's vector-memory pipeline is the limit of a
// one-block kernel, so the rows reach it as whole 16-byte vectors: each chunk
// of rows (its basis and dy spans are contiguous in the rows layout) is copied
// into LDS with coalesced float4 loads, then thread t takes rows t, t + 512,
// .. of the chunk from LDS and accumulates ALL outputs (acc[j][f] in
// registers); the 512 partials of each output are summed in LDS in a fixed
// two-level order (32 segments of 16 threads in thread order, then the
// segments in order), so dW is bitwise reproducible (another grouping than
// the slabs': it agrees with them to fp32 rounding).  (Per-lane scalar global
// loads -- an output per thread, or a row per thread -- took 8.6-13 us on
// config A, and so did this staging while each lane had one load in flight:
// the time was memory round trips in series; profiles/r06_A.)
// Rows layout only (basis[r*FinK + j]): the planes layout needs Fin % 16 == 0.
constexpr int kDwsT = 512, kDwsFK = 8, kDwsFO = 8, kDwsSeg = kDwsT / 16;
constexpr int kDwsStage = 96 * 1024;  // LDS bytes for a chunk's basis + dy spans (+ 32 B slack)
__device__ __forceinline__ void dws_stage(const float* __restrict__ src, int64_t lo, int64_t hi,
                                          float* dst, int64_t* base) {
  // [lo, hi) floats of src (16-byte aligned: the host checks) into dst from the
  // aligned floor of lo, as float4 up to the last whole vector and the <= 3
  // trailing floats one by one (no read past hi's vector); the element at
  // index e lands at dst[e - *base]
  const int64_t b = lo & ~int64_t(3), e4 = hi >> 2;
  *base = b;
  const float4* s4 = reinterpret_cast<const float4*>(src);
  // 8 vectors per lane in flight before their LDS stores (one at a time, each
  // load waited out its own memory round trip: ~10 us for config A's spans)
  for (int64_t q0 = (b >> 2) + threadIdx.x; q0 < e4; q0 += 8 * kDwsT) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t q = q0 + int64_t(u) * kDwsT;
      v[u] = s4[q < e4 ? q : e4 - 1];  // unconditional (clamped) loads
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t q = q0 + int64_t(u) * kDwsT;
      if (q < e4) reinterpret_cast<float4*>(dst)[q - (b >> 2)] = v[u];
    }
  }
  const int64_t tail = (e4 << 2) + threadIdx.x;
  if (tail < hi && tail >= lo) dst[tail - b] = src[tail];
}
__global__ __launch_bounds__(kDwsT) void k_dw_small(const float* __restrict__ basis,
                                                    const float* __restrict__ dy, int64_t R,
                                                    int FinK, int Fout, int rows_per_chunk,
                                                    float* __restrict__ out) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) float dws_sm[];
  const int t = threadIdx.x;
  const int nout = FinK * Fout;
  float acc[kDwsFK][kDwsFO];
#pragma unroll
  for (int j = 0; j < kDwsFK; ++j)
#pragma unroll
    for (int f = 0; f < kDwsFO; ++f) acc[j][f] = 0.f;
  float* s_a = dws_sm;
  float* s_b = dws_sm + ((int64_t(rows_per_chunk) * FinK + 8 + 3) & ~int64_t(3));
  for (int64_t r0 = 0; r0 < R; r0 += rows_per_chunk) {
    const int64_t r1 = r0 + rows_per_chunk < R ? r0 + rows_per_chunk : R;
    int64_t ba, bb;
    dws_stage(basis, r0 * FinK, r1 * FinK, s_a, &ba);
    dws_stage(dy, r0 * Fout, r1 * Fout, s_b, &bb);
    __syncthreads();
    for (int64_t r = r0 + t; r < r1; r += kDwsT) {
      float a[kDwsFK], b[kDwsFO];
#pragma unroll
      for (int j = 0; j < kDwsFK; ++j) a[j] = j < FinK ? s_a[r * FinK + j - ba] : 0.f;
#pragma unroll
      for (int f = 0; f < kDwsFO; ++f) b[f] = f < Fout ? s_b[r * Fout + f - bb] : 0.f;
#pragma unroll
      for (int j = 0; j < kDwsFK; ++j)
#pragma unroll
        for (int f = 0; f < kDwsFO; ++f) acc[j][f] = acc[j][f] + a[j] * b[f];
    }
    __syncthreads();  // the chunk's spans are overwritten next
  }
  float* part = dws_sm;                         // [nout][kDwsT + 1]
  float* seg = dws_sm + nout * (kDwsT + 1);     // [kDwsSeg][nout]
#pragma unroll
  for (int j = 0; j < kDwsFK; ++j)
#pragma unroll
    for (int f = 0; f < kDwsFO; ++f)
      if (j < FinK && f < Fout) part[(j * Fout + f) * (kDwsT + 1) + t] = acc[j][f];
  __syncthreads();
  // level 1: (output o, segment sg) sums threads 16 sg .. 16 sg + 15 in order;
  // consecutive lanes take consecutive outputs (row stride kDwsT + 1: a bank
  // apart, so the reads are conflict-free; lanes over segments were 16-way)
  for (int e = t; e < nout * kDwsSeg; e += kDwsT) {
    const int sg = e / nout, o = e - sg * nout;
    float v = 0.f;
#pragma unroll
    for (int u = 0; u < 16; ++u) v = v + part[o * (kDwsT + 1) + 16 * sg + u];
    seg[sg * nout + o] = v;
  }
  __syncthreads();
  if (t < nout) {
    float v = 0.f;
#pragma unroll
    for (int sg = 0; sg < kDwsSeg; ++sg) v = v + seg[sg * nout + t];
    out[t] = v;
  }
}

}  // namespace

bool dw_small_ok(int64_t R, int FinK, int Fout) {
  return FinK >= 1 && FinK <= kDwsFK && Fout >= 1 && Fout <= kDwsFO && R >= 1 && R <= 16384;
}
bool dw_small_aligned(const float* basis, const float* dy) {
  return ((reinterpret_cast<uintptr_t>(basis) | reinterpret_cast<uintptr_t>(dy)) & 15) == 0;
}

hipError_t launch_dw_small(const float* basis, const float* dy, int64_t R, int FinK, int Fout,
                           float* out, hipStream_t s) {
  if (!dw_small_ok(R, FinK, Fout) || !dw_small_aligned(basis, dy)) return hipErrorInvalidValue;
  // rows per chunk: both spans (+ alignment slack) within kDwsStage bytes
  const int rpc = (kDwsStage - 64) / ((FinK + Fout) * 4);
  const size_t red = size_t(FinK) * Fout * (kDwsT + 1 + kDwsSeg) * 4;  // <= 64 x 545 x 4 = 140 KB
  const size_t lds = red > size_t(kDwsStage) ? red : size_t(kDwsStage);
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dw_small),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     kLdsBytes);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL(k_dw_small, dim3(1), dim3(kDwsT), lds, s, basis, dy, R, FinK, Fout, rpc, out);
  return hipGetLastError();
}

hipError_t launch_cheb_step(const int* rowptr, const int* col, const float* val, const int* rperm,
                            const float* Tp, const float* Tpp, float* Tout, const float* x,
                            const float* slots, float* basis, int N, int M, int Fin, int K, int k,
                            bool last, hipStream_t s) {
  ChebStepArgs a{rowptr, col, val, rperm, Tp, Tpp, Tout, x, slots,
                 int64_t(N) * M * Fin, basis, M, Fin, K, k};
  const int vec = (Fin % 4 == 0) ? 4 : 1;
  const StepGeom g = step_geom(N, M, Fin, vec);
  const dim3 grid(g.grid), block(256);
  const size_t stage = size_t(4) * g.rpw * (size_t(Fin) * K + 1) * sizeof(float);
  // up to the CU's whole LDS: the per-lane scattered basis stores of
  // k_cheb_step<., true> are ~10x slower (config R's 32 x 20 hidden layers:
  // 835 us per call, profiles/r02_resgnn)
  static const hipError_t attr4 = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&k_cheb_last<4>), hipFuncAttributeMaxDynamicSharedMemorySize,
      kLdsBytes);
  static const hipError_t attr1 = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&k_cheb_last<1>), hipFuncAttributeMaxDynamicSharedMemorySize,
      kLdsBytes);
  if (last && stage <= size_t(kLdsBytes) && attr4 == hipSuccess && attr1 == hipSuccess) {
    if (vec == 4) hipLaunchKernelGGL((k_cheb_last<4>), grid, block, stage, s, a, g);
    else hipLaunchKernelGGL((k_cheb_last<1>), grid, block, stage, s, a, g);
  } else if (vec == 4) {
    if (last) hipLaunchKernelGGL((k_cheb_step<4, true>), grid, block, 0, s, a, g);
    else hipLaunchKernelGGL((k_cheb_step<4, false>), grid, block, 0, s, a, g);
  } else {
    if (last) hipLaunchKernelGGL((k_cheb_step<1, true>), grid, block, 0, s, a, g);
    else hipLaunchKernelGGL((k_cheb_step<1, false>), grid, block, 0, s, a, g);
  }
  return hipGetLastError();
}

hipError_t launch_clenshaw(const int* trowptr, const int* tcol, const float* tval, const int* rperm,
                           const float* Gn1, const float* Gn2, float* Gout, const float* Dk, int N,
                           int M, int Fin, int K, int k, int dx_acc, hipStream_t s) {
  ClenArgs a{trowptr, tcol, tval, rperm, Gn1, Gn2, Gout, Dk, M, Fin, K, k, dx_acc};
  const int vec = (Fin % 4 == 0) ? 4 : 1;
  const StepGeom g = step_geom(N, M, Fin, vec);
  const dim3 grid(g.grid), block(256);
  if (vec == 4) hipLaunchKernelGGL((k_clenshaw_step<4>), grid, block, 0, s, a, g);
  else hipLaunchKernelGGL((k_clenshaw_step<1>), grid, block, 0, s, a, g);
  return hipGetLastError();
}

static int rowgemm_kc2(int Kc) {
  return Kc < 32 ? (Kc + 1) / 2 : ((Kc + 1) / 2 + 15) / 16 * 16;
}

bool rowgemm_ok(int Kc, int lda, int Nc) {
  const int KC2 = rowgemm_kc2(Kc);
  const int NT = (Nc + 31) / 32;
  // (B staged whole in LDS: up to the CU's 160 KB, e.g. the ResGNN hidden
  // layers' y = basis W with Kc = 32 x 20 = 640, 80 KB)
  return Kc >= 2 && Kc <= 1024 && Nc >= 1 && NT <= 8 && lda >= Kc &&
         size_t(2) * KC2 * NT * 32 * 4 <= size_t(kLdsBytes);
}

hipError_t launch_rowgemm(const float* A, int64_t R, int Kc, int lda, const float* B, int64_t bs_k,
                          int64_t bs_j, int64_t bs_p, int planes, int Nc, float* C, int ldc,
                          int64_t c_plane, hipStream_t s, const float* res, int act, int pfin,
                          int apl_fin, int64_t apl_stride, int bmapK) {
  if (pfin > 0 && (planes != 1 || res || act)) return hipErrorInvalidValue;
  if (apl_fin > 0 && (apl_fin % 16 != 0 || apl_stride % 4 != 0 || Kc < 32 || planes != 1 ||
                      pfin > 0 || bmapK < 1))
    return hipErrorInvalidValue;
  const int arow_elems = apl_fin > 0 ? apl_fin : lda;
  RowGemmArgs a{A, R, Kc, lda, rowgemm_kc2(Kc), B, bs_k, bs_j, bs_p, Nc, C, ldc, c_plane,
                res, act, pfin,
                int(arow_elems % 4 == 0 && (reinterpret_cast<uintptr_t>(A) & 15) == 0),
                apl_fin, apl_stride, bmapK};
  const int NT = (Nc + 31) / 32;
  const int64_t ntiles = (R + 127) / 128;
  if (option(kOptGemmX3) != 0 && NT <= 8) {
    // the split-bf16 form: B_p's three terms in LDS, [k-block][tile][term][lane] x 16 B
    const size_t lx = size_t((Kc + 15) / 16) * NT * 3 * 64 * 16;
    if (lx <= size_t(kLdsBytes)) {
      const void* k = nullptr;
      switch (NT) {
#define CG_RGX(n) \
  case n: k = reinterpret_cast<const void*>(&k_rowgemm_x3<n>); break;
        CG_RGX(1) CG_RGX(2) CG_RGX(3) CG_RGX(4) CG_RGX(5) CG_RGX(6) CG_RGX(7) default: CG_RGX(8)
#undef CG_RGX
      }
      int dev = 0;
      (void)hipGetDevice(&dev);
      static ResidentCache xcache;
      const int res_blocks = xcache.get(dev, k, 256, lx, [&](const void* kf, int thr, size_t l, int* per_cu,
                                                             int* cus) {
        (void)hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, kf, thr, l) == hipSuccess &&
               hipDeviceGetAttribute(cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess;
      });
      const dim3 grid(persistent_grid(ntiles, res_blocks, planes), unsigned(planes)), block(256);
      void* args[] = {&a};
      return hipLaunchKernel(k, grid, block, args, lx, s);
    }
  }
  const size_t lds = size_t(2) * a.KC2 * NT * 32 * 4;
  // every chunk 16 contiguous in-range floats, at least 3 of them per half
  const bool pf = a.vecA && a.KC2 % 16 == 0 && 2 * a.KC2 <= Kc && a.KC2 / 16 >= 3;
  // the persistent blocks: as many as are resident at once (a grid beyond that
  // runs its last blocks as a tail at a fraction of the chip: config D's y GEMM
  // had 1 024 blocks for 768 resident slots), at most 1 024
  unsigned gx;
  {
    const int nt = NT < 8 ? NT : 8;
    const void* k = nullptr;
#define CG_RGK(n)                                                                              \
  case n:                                                                                      \
    k = pf ? reinterpret_cast<const void*>(&k_rowgemm<n, true>)                                \
           : reinterpret_cast<const void*>(&k_rowgemm<n, false>);                              \
    break;
    switch (nt) { CG_RGK(1) CG_RGK(2) CG_RGK(3) CG_RGK(4) CG_RGK(5) CG_RGK(6) CG_RGK(7) default: CG_RGK(8) }
#undef CG_RGK
    int dev = 0;
    (void)hipGetDevice(&dev);
    // keyed on (device, kernel, threads, dynamic LDS): the LDS follows Kc
    static ResidentCache cache;
    const int res_blocks = cache.get(dev, k, 256, lds, [&](const void* kf, int thr, size_t l, int* per_cu,
                                                           int* cus) {
      if (l > size_t(64) * 1024)
        (void)hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
      return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, kf, thr, l) == hipSuccess &&
             hipDeviceGetAttribute(cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess;
    });
    gx = persistent_grid(ntiles, res_blocks, planes);
  }
  const dim3 grid(gx, unsigned(planes)), block(256);
  if (lds > size_t(64) * 1024) {
    // once per process, thread-safe (a function-local static's initialiser)
    static const hipError_t attr = [] {
      const void* ks[16] = {reinterpret_cast<const void*>(&k_rowgemm<1, false>),
                            reinterpret_cast<const void*>(&k_rowgemm<2, false>),
                            reinterpret_cast<const void*>(&k_rowgemm<3, false>),
                            reinterpret_cast<const void*>(&k_rowgemm<4, false>),
                            reinterpret_cast<const void*>(&k_rowgemm<5, false>),
                            reinterpret_cast<const void*>(&k_rowgemm<6, false>),
                            reinterpret_cast<const void*>(&k_rowgemm<7, false>),
                            reinterpret_cast<const void*>(&k_rowgemm<8, false>),
                            reinterpret_cast<const void*>(&k_rowgemm<1, true>),
                            reinterpret_cast<const void*>(&k_rowgemm<2, true>),
                            reinterpret_cast<const void*>(&k_rowgemm<3, true>),
                            reinterpret_cast<const void*>(&k_rowgemm<4, true>),
                            reinterpret_cast<const void*>(&k_rowgemm<5, true>),
                            reinterpret_cast<const void*>(&k_rowgemm<6, true>),
                            reinterpret_cast<const void*>(&k_rowgemm<7, true>),
                            reinterpret_cast<const void*>(&k_rowgemm<8, true>)};
      for (const void* k : ks) {
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
        if (e != hipSuccess) return e;
      }
      return hipSuccess;
    }();
    if (attr != hipSuccess) return attr;
  }
#define CG_RG(nt)                                                                 \
  case nt:                                                                        \
    if (pf) hipLaunchKernelGGL((k_rowgemm<nt, true>), grid, block, lds, s, a);    \
    else hipLaunchKernelGGL((k_rowgemm<nt, false>), grid, block, lds, s, a);      \
    break;
  switch (NT < 8 ? NT : 8) {
    CG_RG(1) CG_RG(2) CG_RG(3) CG_RG(4) CG_RG(5) CG_RG(6) CG_RG(7)
    default: CG_RG(8)
  }
#undef CG_RG
  return hipGetLastError();
}

static int gemm_kchunk(int Kg, int splits) {
  if (splits < 1) splits = 1;
  const int kchunk = (Kg + splits - 1) / splits;
  return ((kchunk + 15) / 16) * 16;
}

int gemm_effective_splits(int Kg, int splits) {
  const int kchunk = gemm_kchunk(Kg, splits);
  return kchunk > 0 ? (Kg + kchunk - 1) / kchunk : 1;
}

hipError_t launch_gemm_f32(bool trans_a, bool trans_b, int Mg, int Ng, int Kg, const float* A,
                           int lda, const float* B, int ldb, float* C, int ldc, int splits,
                           hipStream_t s, int remapK) {
  const int kchunk = gemm_kchunk(Kg, splits);
  const int nsplit = gemm_effective_splits(Kg, splits);
  const dim3 grid((Mg + 63) / 64, (Ng + 63) / 64, nsplit > 0 ? nsplit : 1);
  if (!trans_a && !trans_b)
    hipLaunchKernelGGL((k_gemm_f32<false, false>), grid, dim3(256), 0, s, Mg, Ng, Kg, A, lda, B,
                       ldb, C, ldc, kchunk, remapK);
  else if (!trans_a && trans_b)
    hipLaunchKernelGGL((k_gemm_f32<false, true>), grid, dim3(256), 0, s, Mg, Ng, Kg, A, lda, B,
                       ldb, C, ldc, kchunk, remapK);
  else if (trans_a && !trans_b)
    hipLaunchKernelGGL((k_gemm_f32<true, false>), grid, dim3(256), 0, s, Mg, Ng, Kg, A, lda, B,
                       ldb, C, ldc, kchunk, remapK);
  else
    hipLaunchKernelGGL((k_gemm_f32<true, true>), grid, dim3(256), 0, s, Mg, Ng, Kg, A, lda, B, ldb,
                       C, ldc, kchunk, remapK);
  return hipGetLastError();
}

int dw_chunks(int64_t R) {
  // ~512 rows per chunk, at most 1024 chunks (slab bytes stay <= 1024*FinK*Fout*4).
  // (Small problems with few columns take k_dw_small instead -- config A's 3 200
  // rows in 7 serial chunks took 29.8 us, profiles/r06_A.  Smaller chunks for
  // every small R changed the summation order of config R's dW at N = 3, where
  // the end-to-end test sits near its ReLU-flip-bound 5e-5 bar: kept as it was.)
  int64_t c = (R + 511) / 512;
  if (c > 1024) c = 1024;
  return int(c < 1 ? 1 : c);
}

// the two-waves-per-SIMD build of the instantiations that fit in 256
// registers: config C2's dW 223 -> 215 us, config E's weight-gradient pass
// 584 -> 551 us (profiles/r04_j).  CG_OPT_DW_W2 = 0 keeps the one-wave build
// (ablation build only: the release library does not compile the one-wave
// alternatives of the two-wave builds)
#ifdef CG_DEBUG
static bool dw_two_waves() { return option(kOptDwW2) != 0; }
#else
static constexpr bool dw_two_waves() { return true; }
#endif

// k_dw_direct for this shape, if one of its instantiations serves it: the dy
// columns of the slice decide the B loads (VB, NLB), the basis columns (with
// the LSTM's x-plane and ones columns) are cut into G groups of NA = VA*NLA
// virtual tiles, NA chosen for the fewest MFMAs per row pair (G*NA*NB);
// CG_OPT_DW_DIRECT = 0 keeps k_dw_slabs (A/B runs); 2 forces k_dw_direct
// whatever the wave count, 3 too but with one-float basis loads only (tests)
static bool launch_dw_direct(const float* basis, const float* dy, int64_t R, int FinKh, int Fout,
                             int ldd, float* slab, hipStream_t s, int pl_fin, int64_t pl_stride,
                             int K, int chunks, int64_t rpc, const float* xb, int x_fin,
                             int64_t x_stride, hipError_t* err) {
  const int mode = option(kOptDwDirect);
  if (mode == 0 || rpc < 256) return false;
  const bool a8 = (reinterpret_cast<uintptr_t>(basis) & 7) == 0;
  const bool b8 = (reinterpret_cast<uintptr_t>(dy) & 7) == 0;
  const bool a2 = !xb && a8 && FinKh % 2 == 0 && (pl_fin == 0 || (pl_fin % 2 == 0 && pl_stride % 2 == 0));
  const bool b2 = b8 && Fout % 2 == 0 && ldd % 2 == 0;
  const int nxc = xb ? x_fin * K : 0;
  const int FinK = FinKh + (xb ? nxc + 1 : 0);
  DwDirectArgs a{basis, dy, R, rpc, chunks, 1, FinKh, Fout, ldd, slab, pl_fin, pl_stride, K,
                 xb, x_fin > 0 ? x_fin : 1, nxc, FinK, x_stride};
  auto go = [&](auto kern, int na) {
    a.G = (FinK + 32 * na - 1) / (32 * na);
    const int64_t waves = int64_t(chunks) * a.G;
    // one wave per SIMD at least (its ~300-500 VGPRs allow no second one):
    // below that k_dw_slabs' LDS-batched waves win (config R: 800 waves,
    // 4.87 vs 5.10 ms per step, profiles/r04_ab)
    if (mode == 1 && waves < 1024) return false;
    hipLaunchKernelGGL(kern, dim3(unsigned((waves + 3) / 4)), dim3(256), 0, s, a);
    *err = hipGetLastError();
    return true;
  };
  auto mfmas = [&](int na) { return (FinK + 32 * na - 1) / (32 * na) * na; };  // per B tile
  // the two-wave build, or (ablation build, CG_OPT_DW_W2 = 0) the one-wave one
#ifdef CG_DEBUG
  const bool w2 = dw_two_waves();
#define CG_W2(two, one, na) (w2 ? go(two, na) : go(one, na))
#else
#define CG_W2(two, one, na) go(two, na)
#endif
  if (Fout <= 32) return CG_W2((k_dw_direct2<1, 5, 1, 1, 12>), (k_dw_direct<1, 5, 1, 1, 12>), 5);
  if (!b2) return false;
  if (Fout <= 64) {
    // two-float basis loads, six virtual tiles: FinK <= 192 in ONE column
    // group, so dy is read once (config D: 17.5 ms per call against 19.7 for
    // <1, 3, ...> and 20.6 for k_dw_slabs, profiles/r04_d)
    // (two waves per SIMD measured slower on config D at N = 256, 19.8 ms per
    // call for both <1, 3, 2, 1, 12> and two-float <2, 1, 2, 1, 12> in three
    // groups of two tiles: profiles/r05_b)
    if (a2 && mode != 3) return go(k_dw_direct<2, 3, 2, 1, 8>, 6);
    return CG_W2((k_dw_direct2<1, 3, 2, 1, 12>), (k_dw_direct<1, 3, 2, 1, 12>), 3);
  }
  if (Fout <= 128) {
    if (mfmas(2) < mfmas(3)) return CG_W2((k_dw_direct2<1, 2, 2, 2, 10>), (k_dw_direct<1, 2, 2, 2, 10>), 2);
    return go(k_dw_direct<1, 3, 2, 2, 8>, 3);
  }
  return CG_W2((k_dw_direct2<1, 1, 2, 4, 8>), (k_dw_direct<1, 1, 2, 4, 8>), 1);
#undef CG_W2
}

// k_dw_x3s (CG_OPT_DW_X3 = 1, the default) where it measured faster than the
// f32 kernels: dy of 65-128 columns (three or four 32-column tiles, e.g. the
// gconv-LSTM's 4H = 128 gate columns: config E's weight-gradient pass 564 ->
// 407-425 us, profiles/r06_x3), 8 or fewer basis tiles and >= 256 chunks.
// With one or two dy tiles the split's VALU and LDS work per MFMA is not
// hidden and k_dw_direct stays faster (config D 2.32 vs 2.29-2.51 ms per
// N = 32 call, config C2 0.24 vs 0.29 ms).
static bool launch_dw_x3(const float* basis, const float* dy, int64_t R, int FinKh, int Fout,
                         int ldd, float* slab, hipStream_t s, int pl_fin, int64_t pl_stride, int K,
                         int chunks, int64_t rpc, const float* xb, int x_fin, int64_t x_stride,
                         hipError_t* err) {
  if (option(kOptDwX3) == 0 || option(kOptDwDirect) == 0 || rpc < 256 || chunks < 256) return false;
  const int nxc = xb ? x_fin * K : 0;
  const int FinK = FinKh + (xb ? nxc + 1 : 0);
  const int nat = (FinK + 31) / 32, nbt = (Fout + 31) / 32;
  const bool b16 = (reinterpret_cast<uintptr_t>(dy) & 15) == 0 && Fout % 4 == 0 && ldd % 4 == 0;
  if (!b16 || nat > 8 || nbt < 3 || nbt > 4 || 32 * nbt > 64 * nat) return false;
  DwDirectArgs a{basis, dy, R, rpc, chunks, 1, FinKh, Fout, ldd, slab, pl_fin, pl_stride, K,
                 xb, x_fin > 0 ? x_fin : 1, nxc, FinK, x_stride};
  const size_t lds = size_t(2) * 3 * 2 * nbt * 64 * 16;
  // rows per staging task: the fewest with every task on its own thread
  int rpt = 8;
  while (rpt > 1 && 8 * nbt * (32 / (rpt / 2)) <= 64 * nat) rpt /= 2;
  const void* kf = nullptr;
#define CG_X3S(NB_)                                                                   \
  kf = rpt == 1   ? reinterpret_cast<const void*>(&k_dw_x3s<NB_, 1>)                  \
       : rpt == 2 ? reinterpret_cast<const void*>(&k_dw_x3s<NB_, 2>)                  \
       : rpt == 4 ? reinterpret_cast<const void*>(&k_dw_x3s<NB_, 4>)                  \
                  : reinterpret_cast<const void*>(&k_dw_x3s<NB_, 8>);
  if (nbt == 3) {
    CG_X3S(3)
  } else {
    CG_X3S(4)
  }
#undef CG_X3S
  void* args[] = {&a};
  *err = hipLaunchKernel(kf, dim3(unsigned(chunks)), dim3(unsigned(64 * nat)), args, lds, s);
  return true;
}

static hipError_t launch_dw_slabs_cols(const float* basis, const float* dy, int64_t R, int FinKh,
                                       int Fout, int ldd, float* slab, hipStream_t s, int pl_fin,
                                       int64_t pl_stride, int K, const float* xb, int x_fin,
                                       int64_t x_stride) {
  const int chunks = dw_chunks(R);
  const int64_t rpc = (R + chunks - 1) / chunks;
  hipError_t derr = hipSuccess;
  if (launch_dw_x3(basis, dy, R, FinKh, Fout, ldd, slab, s, pl_fin, pl_stride, K, chunks, rpc, xb,
                   x_fin, x_stride, &derr))
    return derr;
  if (launch_dw_direct(basis, dy, R, FinKh, Fout, ldd, slab, s, pl_fin, pl_stride, K, chunks, rpc,
                       xb, x_fin, x_stride, &derr))
    return derr;
  const int FinK = FinKh + (xb ? x_fin * K + 1 : 0);
  const int jtl = (FinK + 31) / 32, ftl = (Fout + 31) / 32;
  const int ntiles = jtl * ftl;
  // float4 pieces only where every piece is a whole aligned float4: column
  // counts, row strides, plane stride and both base pointers
  const bool a16 = (reinterpret_cast<uintptr_t>(basis) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(dy) & 15) == 0;
  const int vw = (a16 && FinKh % 4 == 0 && Fout % 4 == 0 && ldd % 4 == 0 &&
                  (pl_fin == 0 || (pl_fin % 4 == 0 && pl_stride % 4 == 0))) ? 4 : 1;
  // tiles per block: as many as the staging pieces allow (every group
  // re-reads the chunk's dy rows and its own basis columns)
  int tpb = kDwTiles, groups = 0, span = 0;
  for (;; tpb /= 2) {
    groups = (ntiles + tpb - 1) / tpb;
    span = 0;
    bool ok = true;
    for (int g = 0; g < groups; ++g) {
      const int t0 = g * tpb, t1 = std::min(t0 + tpb, ntiles);
      const int jlo = (t0 / ftl) * 32, jhi0 = ((t1 - 1) / ftl + 1) * 32, jhi = std::min(jhi0, FinKh);
      span = std::max(span, jhi0 - jlo);
      if (jhi - jlo > kDwNA * 64 * vw) ok = false;
    }
    if (ok) break;
    if (tpb == 1) return hipErrorInvalidValue;
  }
  const size_t lds = size_t(kDwRB) * ((span | 1) + (((Fout + 31) & ~31) | 1)) * 4;
  const dim3 grid(chunks, groups);
  // 8 waves per block unless CG_OPT_DW_WAVES = 4 (A/B runs; the slabs are the same)
  const int nw = option(kOptDwWaves);
  if (vw == 4 && nw == 8)
    hipLaunchKernelGGL((k_dw_slabs<4, 8>), grid, dim3(512), lds, s, basis, dy, R, FinK, Fout, rpc,
                       slab, pl_fin, pl_stride, K, tpb, xb, x_fin, x_stride, FinKh, ldd);
  else if (vw == 4)
    hipLaunchKernelGGL((k_dw_slabs<4, 4>), grid, dim3(256), lds, s, basis, dy, R, FinK, Fout, rpc,
                       slab, pl_fin, pl_stride, K, tpb, xb, x_fin, x_stride, FinKh, ldd);
  else if (nw == 8)
    hipLaunchKernelGGL((k_dw_slabs<1, 8>), grid, dim3(512), lds, s, basis, dy, R, FinK, Fout, rpc,
                       slab, pl_fin, pl_stride, K, tpb, xb, x_fin, x_stride, FinKh, ldd);
  else
    hipLaunchKernelGGL((k_dw_slabs<1, 4>), grid, dim3(256), lds, s, basis, dy, R, FinK, Fout, rpc,
                       slab, pl_fin, pl_stride, K, tpb, xb, x_fin, x_stride, FinKh, ldd);
  return hipGetLastError();
}

hipError_t launch_dw_slabs(const float* basis, const float* dy, int64_t R, int FinKh, int Fout,
                           float* slab, hipStream_t s, int pl_fin, int64_t pl_stride, int K,
                           const float* xb, int x_fin, int64_t x_stride) {
  if (xb && (x_fin < 1 || x_fin * K + 1 > 64)) return hipErrorInvalidValue;
  // the kernel stages at most 256 dy columns per row: wider outputs run as
  // column slices of 256 (each slice its own launch over the same rows, slab
  // columns f0 .. f0 + 255 of the same [chunk][FinK][Fout] slabs)
  for (int f0 = 0; f0 < Fout; f0 += 256) {
    const int fw = Fout - f0 < 256 ? Fout - f0 : 256;
    const hipError_t e = launch_dw_slabs_cols(basis, dy + f0, R, FinKh, fw, Fout, slab + f0, s,
                                              pl_fin, pl_stride, K, xb, x_fin, x_stride);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_reduce_slabs(const float* slab, int nslab, int64_t count, float* out,
                               hipStream_t s) {
  return launch_reduce_slabs_acc(slab, nslab, count, out, 0, s);
}

hipError_t launch_reduce_slabs3(const float* slab, int nslab, int64_t count, float* out0,
                                int64_t n0, float* out1, int64_t n01, float* out2, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce_slabs3, dim3(unsigned((count + 63) / 64)), dim3(1024), 0, s, slab,
                     nslab, count, out0, n0, out1, n01, out2);
  return hipGetLastError();
}

hipError_t launch_reduce_slabs_acc(const float* slab, int nslab, int64_t count, float* out,
                                   int accumulate, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce_slabs, dim3(unsigned((count + 63) / 64)), dim3(1024), 0, s, slab,
                     nslab, count, out, accumulate);
  return hipGetLastError();
}

}  // namespace cg
