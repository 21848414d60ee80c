// Streaming path of the Chebyshev graph convolution for gfx950: any graph
// size (the dense right-hand side lives in HBM, one launch per Chebyshev step).
//
//   x_to_cols   : x [N][M][Fin] -> T_0 [M][B] (column b = n*Fin + fin) and basis k=0
//   spmm_step   : T_k = 2 L~ T_{k-1} - T_{k-2} (T_1 = L~ T_0), one wave per CSR row,
//                 lanes over dense columns (16 B per lane when B % 4 == 0), with
//                 the recurrence fused into the epilogue and the basis column
//                 fin*K + k of lib/graph_conv.py:172 written in the same pass.
//   clenshaw    : G_k = D_k + c L~^T G_{k+1} - G_{k+2}, D_k gathered from dBasis,
//                 k = 0 writes dx directly.
//   gemm_f32    : LDS-tiled v_mfma_f32_32x32x2_f32 GEMM (64x64 tile, 4 waves),
//                 optional split-K partial slabs; contraction y = basis W,
//                 dBasis = dy W^T and dW = basis^T dy.
//
// The SpMM accumulates sequentially in CSR order with fp contraction off, so
// the basis is bit-identical to the resident path and to lib/graph.py::chebyshev.
#include "cg_internal.h"

namespace cg {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

inline int grid_for(int64_t total, int block) {
  int64_t g = (total + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return int(g);
}

__global__ __launch_bounds__(256) void k_x_to_cols(const float* __restrict__ x,
                                                   float* __restrict__ T0,
                                                   float* __restrict__ basis, int N, int M,
                                                   int Fin, int K) {
  const int64_t B = int64_t(N) * Fin;
  const int64_t total = int64_t(M) * B;
  const int64_t FinK = int64_t(Fin) * K;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t m = i / B, b = i - m * B;
    const int64_t n = b / Fin, fin = b - n * Fin;
    const float v = x[(n * M + m) * Fin + fin];
    T0[i] = v;
    if (basis) basis[(n * M + m) * FinK + fin * K] = v;
  }
}

// (n*M + r)*Fin*K + fin*K for dense column b = n*Fin + fin
__device__ __forceinline__ int64_t row_base(int64_t r, int64_t b, int M, int Fin, int K) {
  const int64_t n = b / Fin, fin = b - n * Fin;
  return (n * M + r) * (int64_t(Fin) * K) + fin * K;
}

template <bool VEC4>
__global__ __launch_bounds__(256) void k_spmm_cheb(
    const int* __restrict__ rowptr, const int* __restrict__ col, const float* __restrict__ val,
    const float* __restrict__ Tprev, const float* __restrict__ Tprev2, float* __restrict__ Tout,
    float* __restrict__ basis, int N, int M, int Fin, int K, int k) {
#pragma clang fp contract(off)
  const int64_t B = int64_t(N) * Fin;
  const int r = __builtin_amdgcn_readfirstlane(int(blockIdx.x) * 4 + int(threadIdx.x >> 6));
  if (r >= M) return;
  const int lane = threadIdx.x & 63;
  const int j0 = rowptr[r], j1 = rowptr[r + 1];
  if (VEC4) {
    for (int64_t b = int64_t(lane) * 4; b < B; b += 256) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int j = j0; j < j1; ++j) {
        const float v = val[j];
        const float4 t = *reinterpret_cast<const float4*>(Tprev + int64_t(col[j]) * B + b);
        a.x = a.x + v * t.x;
        a.y = a.y + v * t.y;
        a.z = a.z + v * t.z;
        a.w = a.w + v * t.w;
      }
      float4 o = a;
      if (k >= 2) {
        const float4 p = *reinterpret_cast<const float4*>(Tprev2 + int64_t(r) * B + b);
        o.x = 2.f * a.x - p.x;
        o.y = 2.f * a.y - p.y;
        o.z = 2.f * a.z - p.z;
        o.w = 2.f * a.w - p.w;
      }
      if (Tout) *reinterpret_cast<float4*>(Tout + int64_t(r) * B + b) = o;
      if (basis) {
        basis[row_base(r, b + 0, M, Fin, K) + k] = o.x;
        basis[row_base(r, b + 1, M, Fin, K) + k] = o.y;
        basis[row_base(r, b + 2, M, Fin, K) + k] = o.z;
        basis[row_base(r, b + 3, M, Fin, K) + k] = o.w;
      }
    }
  } else {
    for (int64_t b = lane; b < B; b += 64) {
      float a = 0.f;
      for (int j = j0; j < j1; ++j) a = a + val[j] * Tprev[int64_t(col[j]) * B + b];
      const float o = (k >= 2) ? (2.f * a - Tprev2[int64_t(r) * B + b]) : a;
      if (Tout) Tout[int64_t(r) * B + b] = o;
      if (basis) basis[row_base(r, b, M, Fin, K) + k] = o;
    }
  }
}

__global__ __launch_bounds__(256) void k_clenshaw(
    const int* __restrict__ rowptr, const int* __restrict__ col, const float* __restrict__ val,
    const float* __restrict__ Gn1, const float* __restrict__ Gn2, float* __restrict__ Gout,
    const float* __restrict__ dA, float* __restrict__ dx, int N, int M, int Fin, int K, int k) {
#pragma clang fp contract(off)
  const int64_t B = int64_t(N) * Fin;
  const int r = __builtin_amdgcn_readfirstlane(int(blockIdx.x) * 4 + int(threadIdx.x >> 6));
  if (r >= M) return;
  const int lane = threadIdx.x & 63;
  const int j0 = rowptr[r], j1 = rowptr[r + 1];
  const bool has1 = (k + 1) <= (K - 1), has2 = (k + 2) <= (K - 1);
  const float c = (k >= 1) ? 2.f : 1.f;
  for (int64_t b = lane; b < B; b += 64) {
    float a = 0.f;
    if (has1)
      for (int j = j0; j < j1; ++j) a = a + val[j] * Gn1[int64_t(col[j]) * B + b];
    float g = dA[row_base(r, b, M, Fin, K) + k] + c * a;
    if (has2) g = g - Gn2[int64_t(r) * B + b];
    if (k == 0) {
      if (dx) {
        const int64_t n = b / Fin, fin = b - n * Fin;
        dx[(n * M + r) * Fin + fin] = g;
      }
    } else {
      Gout[int64_t(r) * B + b] = g;
    }
  }
}

// C = op(A) op(B), 64x64 output tile per 256-thread block, each wave a 32x32
// MFMA tile; BK = 16 staged through LDS ([k][row] images so an MFMA operand
// read is 32 consecutive floats).
template <bool TA, bool TB>
__global__ __launch_bounds__(256) void k_gemm_f32(int Mg, int Ng, int Kg, const float* __restrict__ A,
                                                  int lda, const float* __restrict__ B, int ldb,
                                                  float* __restrict__ C, int ldc, int kchunk) {
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
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (row < Mg && col < Ng) C[size_t(row) * ldc + col] = acc[r];
  }
}

// dW partial slabs: slab[z][j][f] = sum_{r in chunk z} basis[r][j] * dy[r][f]
// over the R = N*M basis rows (j < FinK, f < Fout): a skinny TN GEMM whose
// inner dimension is the whole batch.  Block (z, tile) = 4 waves; wave w
// streams rows r0 + 2u + h of its quarter of chunk z (lane half h takes the
// odd rows) straight into v_mfma_f32_32x32x2_f32 (K = 2 rows per MFMA):
// A lane (j, h) = basis[r][j], B lane (f, h) = dy[r][f] -- each wave load
// instruction reads two whole 4*FinK / 4*Fout-byte rows.  16 loads per lane
// are in flight per batch; the 4 wave partials are added in a fixed order
// through LDS, so the result is bitwise reproducible.  HBM-bound: it reads
// basis + dy once (4*R*(FinK + Fout) bytes) and is meant to run on a side
// stream concurrently with the latency-bound backward recurrence.
__global__ __launch_bounds__(256) void k_dw_slabs(const float* __restrict__ basis,
                                                  const float* __restrict__ dy, int64_t R,
                                                  int FinK, int Fout, int64_t rows_per_chunk,
                                                  float* __restrict__ slab) {
  __shared__ float part[4][32][33];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int ftl = (Fout + 31) >> 5;
  const int jt = blockIdx.y / ftl, ft = blockIdx.y - jt * ftl;
  const int j = jt * 32 + li, f = ft * 32 + li;
  const bool jv = j < FinK, fv = f < Fout;
  const int jc = jv ? j : FinK - 1, fc = fv ? f : Fout - 1;
  const int64_t c0 = int64_t(blockIdx.x) * rows_per_chunk;
  const int64_t c1 = (c0 + rows_per_chunk < R) ? c0 + rows_per_chunk : R;
  const int64_t q = (((c1 - c0) + 3) / 4 + 1) & ~int64_t(1);  // even rows per wave
  const int64_t r0 = c0 + w * q;
  const int64_t r1 = (r0 + q < c1) ? r0 + q : c1;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int64_t rb = r0; rb < r1; rb += 16) {
    float a[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      int64_t rr = rb + 2 * u + h;
      rr = rr < R ? rr : R - 1;
      a[u] = basis[rr * FinK + jc];
      b[u] = dy[rr * Fout + fc];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool rv = (rb + 2 * u + h) < r1;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32((rv && jv) ? a[u] : 0.f, (rv && fv) ? b[u] : 0.f,
                                                 acc, 0, 0, 0);
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) part[w][(r & 3) + 8 * (r >> 2) + 4 * h][li] = acc[r];
  __syncthreads();
  for (int e = threadIdx.x; e < 1024; e += 256) {
    const int row = e >> 5, col = e & 31;
    const float s = ((part[0][row][col] + part[1][row][col]) + part[2][row][col]) + part[3][row][col];
    const int jj = jt * 32 + row, ff = ft * 32 + col;
    if (jj < FinK && ff < Fout) slab[(int64_t(blockIdx.x) * FinK + jj) * Fout + ff] = s;
  }
}

// out[i] = sum_z slab[z][i] in a FIXED order (bitwise reproducible): wave w of
// a block sums the slabs z = w, w+16, ... for 64 consecutive outputs (one
// 256-B coalesced load per slab, 8 in flight), then the 16 partial sums are
// added in wave order through LDS.
__global__ __launch_bounds__(1024) void k_reduce_slabs(const float* __restrict__ slab, int nslab,
                                                       int64_t count, float* __restrict__ out,
                                                       int accumulate) {
#pragma clang fp contract(off)
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i = int64_t(blockIdx.x) * 64 + lane;
  float s = 0.f;
  if (i < count) {
#pragma unroll 8
    for (int z = w; z < nslab; z += 16) s = s + slab[int64_t(z) * count + i];
  }
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && i < count) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t = t + part[q][lane];
    out[i] = accumulate ? out[i] + t : t;
  }
}

}  // namespace

hipError_t launch_x_to_cols(const float* x, float* T0, float* basis, int N, int M, int Fin, int K,
                            hipStream_t s) {
  const int64_t total = int64_t(M) * N * Fin;
  hipLaunchKernelGGL(k_x_to_cols, dim3(grid_for(total, 256)), dim3(256), 0, s, x, T0, basis, N, M,
                     Fin, K);
  return hipGetLastError();
}

hipError_t launch_spmm_cheb_step(const int* rowptr, const int* col, const float* val,
                                 const float* Tprev, const float* Tprev2, float* Tout, float* basis,
                                 int N, int M, int Fin, int K, int k, hipStream_t s) {
  const int64_t B = int64_t(N) * Fin;
  const dim3 grid((M + 3) / 4);
  const bool vec4 = (B % 4 == 0) && (reinterpret_cast<uintptr_t>(Tprev) % 16 == 0) &&
                    (!Tout || reinterpret_cast<uintptr_t>(Tout) % 16 == 0) &&
                    (!Tprev2 || reinterpret_cast<uintptr_t>(Tprev2) % 16 == 0);
  if (vec4)
    hipLaunchKernelGGL(k_spmm_cheb<true>, grid, dim3(256), 0, s, rowptr, col, val, Tprev, Tprev2,
                       Tout, basis, N, M, Fin, K, k);
  else
    hipLaunchKernelGGL(k_spmm_cheb<false>, grid, dim3(256), 0, s, rowptr, col, val, Tprev, Tprev2,
                       Tout, basis, N, M, Fin, K, k);
  return hipGetLastError();
}

hipError_t launch_clenshaw_step(const int* trowptr, const int* tcol, const float* tval,
                                const float* Gn1, const float* Gn2, float* Gout, const float* dA,
                                float* dx, int N, int M, int Fin, int K, int k, hipStream_t s) {
  hipLaunchKernelGGL(k_clenshaw, dim3((M + 3) / 4), dim3(256), 0, s, trowptr, tcol, tval, Gn1, Gn2,
                     Gout, dA, dx, N, M, Fin, K, k);
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
                           hipStream_t s) {
  const int kchunk = gemm_kchunk(Kg, splits);
  const int nsplit = gemm_effective_splits(Kg, splits);
  const dim3 grid((Mg + 63) / 64, (Ng + 63) / 64, nsplit > 0 ? nsplit : 1);
  if (!trans_a && !trans_b)
    hipLaunchKernelGGL((k_gemm_f32<false, false>), grid, dim3(256), 0, s, Mg, Ng, Kg, A, lda, B,
                       ldb, C, ldc, kchunk);
  else if (!trans_a && trans_b)
    hipLaunchKernelGGL((k_gemm_f32<false, true>), grid, dim3(256), 0, s, Mg, Ng, Kg, A, lda, B,
                       ldb, C, ldc, kchunk);
  else if (trans_a && !trans_b)
    hipLaunchKernelGGL((k_gemm_f32<true, false>), grid, dim3(256), 0, s, Mg, Ng, Kg, A, lda, B,
                       ldb, C, ldc, kchunk);
  else
    hipLaunchKernelGGL((k_gemm_f32<true, true>), grid, dim3(256), 0, s, Mg, Ng, Kg, A, lda, B, ldb,
                       C, ldc, kchunk);
  return hipGetLastError();
}

int dw_chunks(int64_t R) {
  // ~512 rows per chunk, at most 1024 chunks (slab bytes stay <= 1024*FinK*Fout*4)
  int64_t c = (R + 511) / 512;
  if (c > 1024) c = 1024;
  return int(c < 1 ? 1 : c);
}

hipError_t launch_dw_slabs(const float* basis, const float* dy, int64_t R, int FinK, int Fout,
                           float* slab, hipStream_t s) {
  const int chunks = dw_chunks(R);
  const int64_t rpc = (R + chunks - 1) / chunks;
  const dim3 grid(chunks, ((FinK + 31) / 32) * ((Fout + 31) / 32));
  hipLaunchKernelGGL(k_dw_slabs, grid, dim3(256), 0, s, basis, dy, R, FinK, Fout, rpc, slab);
  return hipGetLastError();
}

hipError_t launch_reduce_slabs(const float* slab, int nslab, int64_t count, float* out,
                               hipStream_t s) {
  return launch_reduce_slabs_acc(slab, nslab, count, out, 0, s);
}

hipError_t launch_reduce_slabs_acc(const float* slab, int nslab, int64_t count, float* out,
                                   int accumulate, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce_slabs, dim3(unsigned((count + 63) / 64)), dim3(1024), 0, s, slab,
                     nslab, count, out, accumulate);
  return hipGetLastError();
}

}  // namespace cg
