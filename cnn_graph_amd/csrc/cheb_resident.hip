// Resident (LDS) path of the Chebyshev graph convolution for gfx950.
//
// One 512-thread workgroup per sample n.  The whole K-step recurrence
//   T_0 = X, T_1 = L~X, T_k = 2 L~ T_{k-1} - T_{k-2}      (lib/graph_conv.py:163-169)
// runs out of LDS: the CSR of L~ (uint16 columns) and a 3-slot ring of
// vertex vectors stay on chip, so HBM sees only x in, the basis out (layout of
// lib/graph_conv.py:172) and y out.  The weight contraction
//   y = basis @ W                                          (lib/graph_conv.py:175)
// is folded into the recurrence: every two steps each wave feeds the pair
// (T_{2s}, T_{2s+1}) of its 32-vertex tiles to v_mfma_f32_32x32x2_f32, whose
// K=2 is exactly one Chebyshev pair, accumulating y in registers.
//
// The backward kernel does, per sample:
//   A. dBasis = dy W^T on MFMA into LDS (D[j][m], j = fin*K + k);
//   B. the reverse (Clenshaw) recurrence over L~^T in LDS
//        G_{K-1} = D_{K-1};  G_k = D_k + 2 L~^T G_{k+1} - G_{k+2};  G_0 = D_0 + L~^T G_1 - G_2
//      writing dx = G_0 straight to HBM;
//   C. the per-sample dW partial basis^T dy on MFMA (waves split the vertex
//      range, summed across waves through LDS in a fixed order -> deterministic),
//      written to a slab reduced over samples by a second tiny kernel.
//
// Numerics: the SpMM accumulates each row sequentially from 0 in CSR order,
// one rounding per product and per add (fp contraction OFF) -- the order of
// scipy csr_matvecs / TF SparseTensorDenseMatMul -- so the basis is bit-exact
// to lib/graph.py::chebyshev.  MFMA f32 is an exact fp32 fma chain.
#include "cg_internal.h"

namespace cg {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// Forward
// ---------------------------------------------------------------------------
template <int MT, int NT>
__global__ __launch_bounds__(kResidentThreads) void cheb_fwd_resident(
    int M, int Fin, int K, int Fout, int nnz, int Mp, const int* __restrict__ rowptr,
    const uint16_t* __restrict__ col16, const float* __restrict__ val, const float* __restrict__ x,
    const float* __restrict__ W, float* __restrict__ basis, float* __restrict__ y) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, li = lane & 31;
  const int FinK = Fin * K;

  int* s_rp = reinterpret_cast<int*>(smem);
  size_t off = align16(size_t(M + 1) * 4);
  uint16_t* s_col = reinterpret_cast<uint16_t*>(smem + off);
  off = align16(off + size_t(nnz) * 2);
  float* s_val = reinterpret_cast<float*>(smem + off);
  off = align16(off + size_t(nnz) * 4);
  float* s_W = reinterpret_cast<float*>(smem + off);
  off = align16(off + size_t(FinK) * Fout * 4);
  float* s_T = reinterpret_cast<float*>(smem + off);  // [3][Fin][Mp]

  for (int i = tid; i <= M; i += kResidentThreads) s_rp[i] = rowptr[i];
  for (int i = tid; i < nnz; i += kResidentThreads) {
    s_col[i] = col16[i];
    s_val[i] = val[i];
  }
  for (int i = tid; i < FinK * Fout; i += kResidentThreads) s_W[i] = W ? W[i] : 0.f;
  const float* xn = x + size_t(n) * M * Fin;
  for (int i = tid; i < M * Fin; i += kResidentThreads) {
    const int m = i / Fin, fin = i - m * Fin;
    s_T[fin * Mp + m] = xn[i];  // slot 0 = T_0
  }
  __syncthreads();

  const int ntiles = (M + 31) >> 5;
  f32x16 acc[MT][NT];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int q = 0; q < NT; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][q][r] = 0.f;

  float* basis_n = basis ? basis + size_t(n) * M * FinK : nullptr;

  // Contraction of the Chebyshev pair (T_{2s}, T_{2s+1}) on MFMA; also stores
  // those basis entries (both already in registers as the A operand).
  auto mfma_pair = [&](int s) {
    const int kk = 2 * s + h;
    const bool kv = kk < K;
    const int slot = kk % 3;
    for (int fin = 0; fin < Fin; ++fin) {
      float b[NT];
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        const int f = q * 32 + li;
        b[q] = (kv && f < Fout) ? s_W[(fin * K + kk) * Fout + f] : 0.f;
      }
      const float* Ts = s_T + (slot * Fin + fin) * Mp;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int tile = wave + t * 8;
        if (tile < ntiles) {
          const int m = tile * 32 + li;
          float a = 0.f;
          if (kv && m < M) {
            a = Ts[m];
            if (basis_n) basis_n[size_t(m) * FinK + fin * K + kk] = a;
          }
#pragma unroll
          for (int q = 0; q < NT; ++q) acc[t][q] = mfma32(a, b[q], acc[t][q]);
        }
      }
    }
  };

  for (int k = 1; k < K; ++k) {
    if ((k & 1) == 0) mfma_pair((k - 2) >> 1);
    const int cur = k % 3, prv = (k - 1) % 3, prv2 = (k + 1) % 3;  // (k-2) mod 3 == (k+1) mod 3
    for (int fin = 0; fin < Fin; ++fin) {
      const float* Tp = s_T + (prv * Fin + fin) * Mp;
      const float* Tp2 = s_T + (prv2 * Fin + fin) * Mp;
      float* To = s_T + (cur * Fin + fin) * Mp;
      for (int r = tid; r < M; r += kResidentThreads) {
        const int j0 = s_rp[r], j1 = s_rp[r + 1];
        float a = 0.f;
        for (int j = j0; j < j1; ++j) a = a + s_val[j] * Tp[s_col[j]];
        To[r] = (k == 1) ? a : (2.f * a - Tp2[r]);
      }
    }
    __syncthreads();
  }
  mfma_pair((K - 1) >> 1);  // the last (possibly half-empty) pair

  if (y) {
    float* yn = y + size_t(n) * M * Fout;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int tile = wave + t * 8;
      if (tile < ntiles) {
#pragma unroll
        for (int q = 0; q < NT; ++q) {
          const int f = q * 32 + li;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = tile * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (m < M && f < Fout) yn[size_t(m) * Fout + f] = acc[t][q][r];
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Backward
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kResidentThreads) void cheb_bwd_resident(
    int M, int Fin, int K, int Fout, int nnzT, int Mp, const int* __restrict__ trowptr,
    const uint16_t* __restrict__ tcol16, const float* __restrict__ tval,
    const float* __restrict__ dy, const float* __restrict__ basis, const float* __restrict__ W,
    float* __restrict__ dx, float* __restrict__ dw_slab) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, li = lane & 31;
  const int FinK = Fin * K;

  int* s_rp = reinterpret_cast<int*>(smem);
  size_t off = align16(size_t(M + 1) * 4);
  uint16_t* s_col = reinterpret_cast<uint16_t*>(smem + off);
  off = align16(off + size_t(nnzT) * 2);
  float* s_val = reinterpret_cast<float*>(smem + off);
  off = align16(off + size_t(nnzT) * 4);
  float* s_D = reinterpret_cast<float*>(smem + off);  // [FinK][Mp], later dW scratch
  const size_t dbytes = size_t(FinK) * Mp * 4;
  off = align16(off + (dbytes > 32768 ? dbytes : 32768));
  float* s_G = reinterpret_cast<float*>(smem + off);  // [3][Fin][Mp]

  for (int i = tid; i <= M; i += kResidentThreads) s_rp[i] = trowptr[i];
  for (int i = tid; i < nnzT; i += kResidentThreads) {
    s_col[i] = tcol16[i];
    s_val[i] = tval[i];
  }

  const float* dyn = dy + size_t(n) * M * Fout;
  const float* bn = basis + size_t(n) * M * FinK;

  // A. dBasis = dy W^T  (rows m, cols j, inner f; lane half h owns f in [h*ns, h*ns+ns))
  {
    const int mtiles = (M + 31) >> 5, jtiles = (FinK + 31) >> 5;
    const int ns = (Fout + 1) >> 1;
    for (int task = wave; task < mtiles * jtiles; task += 8) {
      const int mt = task / jtiles, jt = task - mt * jtiles;
      const int m = mt * 32 + li, j = jt * 32 + li;
      const float* dyrow = dyn + size_t(m) * Fout;
      const float* wrow = W + size_t(j) * Fout;
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll 4
      for (int s = 0; s < ns; ++s) {
        const int f = h * ns + s;
        const float a = (m < M && f < Fout) ? dyrow[f] : 0.f;
        const float b = (j < FinK && f < Fout) ? wrow[f] : 0.f;
        acc = mfma32(a, b, acc);
      }
      if (j < FinK) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int mm = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (mm < M) s_D[j * Mp + mm] = acc[r];
        }
      }
    }
  }
  __syncthreads();

  // B. reverse recurrence over L~^T
  for (int k = K - 1; k >= 0; --k) {
    const int cur = k % 3, nx1 = (k + 1) % 3, nx2 = (k + 2) % 3;
    const bool has1 = (k + 1) <= (K - 1), has2 = (k + 2) <= (K - 1);
    const float c = (k >= 1) ? 2.f : 1.f;
    for (int fin = 0; fin < Fin; ++fin) {
      const float* G1 = s_G + (nx1 * Fin + fin) * Mp;
      const float* G2 = s_G + (nx2 * Fin + fin) * Mp;
      float* Go = s_G + (cur * Fin + fin) * Mp;
      const float* Dk = s_D + (fin * K + k) * Mp;
      for (int r = tid; r < M; r += kResidentThreads) {
        float a = 0.f;
        if (has1) {
          const int j0 = s_rp[r], j1 = s_rp[r + 1];
          for (int j = j0; j < j1; ++j) a = a + s_val[j] * G1[s_col[j]];
        }
        float g = Dk[r] + c * a;
        if (has2) g = g - G2[r];
        if (k == 0) {
          if (dx) dx[(size_t(n) * M + r) * Fin + fin] = g;
        } else {
          Go[r] = g;
        }
      }
    }
    if (k > 0) __syncthreads();
  }

  // C. dW partial = basis^T dy (rows j, cols f, inner m split over the 8 waves)
  {
    const int jtl = (FinK + 31) >> 5, ftl = (Fout + 31) >> 5;
    const int chunk = (((M + 7) >> 3) + 1) & ~1;
    const int mbeg = wave * chunk;
    const int mend = (mbeg + chunk < M) ? (mbeg + chunk) : M;
    float* scratch = s_D;  // [8][32][32]
    for (int task = 0; task < jtl * ftl; ++task) {
      const int jt = task / ftl, ft = task - jt * ftl;
      const int j = jt * 32 + li, f = ft * 32 + li;
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll 8
      for (int mm = mbeg; mm < mend; mm += 2) {
        const int m = mm + h;
        const float a = (m < mend && j < FinK) ? bn[size_t(m) * FinK + j] : 0.f;
        const float b = (m < mend && f < Fout) ? dyn[size_t(m) * Fout + f] : 0.f;
        acc = mfma32(a, b, acc);
      }
      __syncthreads();  // s_D free (phase B done) / previous task's readers done
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        scratch[(wave * 32 + row) * 32 + li] = acc[r];
      }
      __syncthreads();
      for (int e = tid; e < 1024; e += kResidentThreads) {
        const int row = e >> 5, col = e & 31;
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < 8; ++w) s = s + scratch[(w * 32 + row) * 32 + col];
        const int jj = jt * 32 + row, ff = ft * 32 + col;
        if (jj < FinK && ff < Fout) dw_slab[(size_t(n) * FinK + jj) * Fout + ff] = s;
      }
    }
  }
}

template <int MT, int NT>
hipError_t launch_fwd_t(size_t lds, int N, int M, int Fin, int K, int Fout, int nnz,
                        const int* rowptr, const uint16_t* col16, const float* val,
                        const float* x, const float* W, float* basis, float* y, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&cheb_fwd_resident<MT, NT>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL((cheb_fwd_resident<MT, NT>), dim3(N), dim3(kResidentThreads), lds, s, M, Fin,
                     K, Fout, nnz, lds_vertex_stride(M), rowptr, col16, val, x, W, basis, y);
  return hipGetLastError();
}

}  // namespace

ResidentGeom resident_geometry(int M, int64_t nnz, int64_t nnzT, int Fin, int K, int Fout) {
  ResidentGeom g{};
  const int Mp = lds_vertex_stride(M);
  const int ntiles = (M + 31) / 32;
  const int need_mt = (ntiles + 7) / 8;
  int mt = 1;
  while (mt < need_mt) mt <<= 1;
  const int nt = (Fout + 31) / 32;
  g.mt = mt;
  g.nt = nt;
  const size_t FinK = size_t(Fin) * K;
  g.fwd_lds = align16(size_t(M + 1) * 4) + align16(size_t(nnz) * 2) + align16(size_t(nnz) * 4) +
              align16(FinK * Fout * 4) + size_t(3) * Fin * Mp * 4;
  const size_t dbytes = FinK * Mp * 4;
  g.bwd_lds = align16(size_t(M + 1) * 4) + align16(size_t(nnzT) * 2) + align16(size_t(nnzT) * 4) +
              align16(dbytes > 32768 ? dbytes : 32768) + size_t(3) * Fin * Mp * 4;
  const bool small = M >= 1 && M <= 65535 && Fin >= 1 && K >= 1 && Fout >= 1;
  g.fwd_ok = small && need_mt <= 8 && nt <= 2 && mt * nt <= 8 && g.fwd_lds <= size_t(kLdsBytes);
  g.bwd_ok = small && g.bwd_lds <= size_t(kLdsBytes);
  return g;
}

hipError_t launch_resident_forward(const ResidentGeom& g, int N, int M, int Fin, int K, int Fout,
                                   int nnz, const int* rowptr, const uint16_t* col16,
                                   const float* val, const float* x, const float* W, float* basis,
                                   float* y, hipStream_t s) {
#define CG_FWD(MT_, NT_)                                                                       \
  if (g.mt == MT_ && g.nt == NT_)                                                              \
    return launch_fwd_t<MT_, NT_>(g.fwd_lds, N, M, Fin, K, Fout, nnz, rowptr, col16, val, x, W, \
                                  basis, y, s);
  CG_FWD(1, 1) CG_FWD(2, 1) CG_FWD(4, 1) CG_FWD(8, 1) CG_FWD(1, 2) CG_FWD(2, 2) CG_FWD(4, 2)
#undef CG_FWD
  return hipErrorInvalidValue;
}

hipError_t launch_resident_backward(const ResidentGeom& g, int N, int M, int Fin, int K, int Fout,
                                    int nnzT, const int* trowptr, const uint16_t* tcol16,
                                    const float* tval, const float* dy, const float* basis,
                                    const float* W, float* dx, float* dw_slab, hipStream_t s) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&cheb_bwd_resident),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(cheb_bwd_resident, dim3(N), dim3(kResidentThreads), g.bwd_lds, s, M, Fin, K,
                     Fout, nnzT, lds_vertex_stride(M), trowptr, tcol16, tval, dy, basis, W, dx,
                     dw_slab);
  return hipGetLastError();
}

}  // namespace cg
