// Spectral (Fourier) graph filter, lib/graph_conv.py:83-111 (filter_in_fourier /
// fourier; dupes lib/models.py:129-159, lib/filter.py fourier_conv):
//
//   Xh = U^T x      (graph Fourier transform, U = eigenvectors of L, lib/graph.py:148)
//   Yh[m] = W[m] Xh[m]     per frequency m: W [M][Fout][Fin]
//   y  = U Yh       (inverse transform)
//
// Layout here keeps the sample-major tensors of the Chebyshev path: with
// Xh [N][Fin][M] both transforms are plain row-major GEMMs over all N*Fin
// (resp. N*Fout) signals against the resident M x M basis U (on MFMA, the
// shared k_gemm_f32), and the per-frequency filter below is an HBM-streaming
// kernel with m on consecutive lanes (every load and store coalesced).
// The [N][M][F] <-> [N][F][M] re-layouts are LDS-tiled transposes, skipped
// when F == 1.
#include "cg_internal.h"

namespace cg {
namespace {

inline int grid_1d(int64_t n, int per_block) {
  int64_t g = (n + per_block - 1) / per_block;
  return int(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

// 32x32 tile per block of 256 threads (32 x 8), +1 padding against LDS bank
// conflicts on the transposed read.
__global__ __launch_bounds__(256) void k_transpose_batched(const float* __restrict__ in, int R, int C,
                                                           float* __restrict__ out) {
  __shared__ float tile[32][33];
  const int64_t b = blockIdx.z;
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const float* src = in + b * int64_t(R) * C;
  float* dst = out + b * int64_t(R) * C;
#pragma unroll
  for (int j = 0; j < 32; j += 8) {
    const int r = r0 + ty + j, c = c0 + tx;
    tile[ty + j][tx] = (r < R && c < C) ? src[int64_t(r) * C + c] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 32; j += 8) {
    const int c = c0 + ty + j, r = r0 + tx;
    if (r < R && c < C) dst[int64_t(c) * R + r] = tile[tx][ty + j];
  }
}

__global__ __launch_bounds__(256) void k_fourier_mix(const float* __restrict__ Xh,
                                                     const float* __restrict__ W, int N, int M,
                                                     int Fin, int Fout, float* __restrict__ Yh) {
#pragma clang fp contract(off)
  const int64_t total = int64_t(N) * Fout * M;
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * 256) {
    const int m = int(i % M);
    const int64_t t = i / M;
    const int fo = int(t % Fout);
    const int64_t n = t / Fout;
    const float* w = W + (int64_t(m) * Fout + fo) * Fin;
    const float* xh = Xh + n * Fin * M + m;
    float acc = 0.f;
    for (int f = 0; f < Fin; ++f) acc = acc + w[f] * xh[int64_t(f) * M];
    Yh[i] = acc;
  }
}

__global__ __launch_bounds__(256) void k_fourier_mix_t(const float* __restrict__ dYh,
                                                       const float* __restrict__ W, int N, int M,
                                                       int Fin, int Fout, float* __restrict__ dXh) {
#pragma clang fp contract(off)
  const int64_t total = int64_t(N) * Fin * M;
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * 256) {
    const int m = int(i % M);
    const int64_t t = i / M;
    const int fi = int(t % Fin);
    const int64_t n = t / Fin;
    const float* w = W + int64_t(m) * Fout * Fin + fi;
    const float* dy = dYh + n * Fout * M + m;
    float acc = 0.f;
    for (int o = 0; o < Fout; ++o) acc = acc + w[int64_t(o) * Fin] * dy[int64_t(o) * M];
    dXh[i] = acc;
  }
}

// one thread per (fo, fin, m), m fastest: each step of the n loop is a
// coalesced row read of dYh and Xh; the sum over n runs in fixed order.
__global__ __launch_bounds__(256) void k_fourier_dw(const float* __restrict__ dYh,
                                                    const float* __restrict__ Xh, int N, int M,
                                                    int Fin, int Fout, float* __restrict__ dW) {
#pragma clang fp contract(off)
  const int64_t total = int64_t(Fout) * Fin * M;
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * 256) {
    const int m = int(i % M);
    const int64_t t = i / M;
    const int fi = int(t % Fin);
    const int fo = int(t / Fin);
    const float* dy = dYh + int64_t(fo) * M + m;
    const float* xh = Xh + int64_t(fi) * M + m;
    const int64_t sy = int64_t(Fout) * M, sx = int64_t(Fin) * M;
    float acc = 0.f;
    for (int n = 0; n < N; ++n) acc = acc + dy[n * sy] * xh[n * sx];
    dW[(int64_t(m) * Fout + fo) * Fin + fi] = acc;
  }
}

}  // namespace

hipError_t launch_transpose_batched(const float* in, int64_t B, int R, int C, float* out,
                                    hipStream_t s) {
  if (B > 65535) return hipErrorInvalidValue;
  const dim3 grid((C + 31) / 32, (R + 31) / 32, unsigned(B));
  hipLaunchKernelGGL(k_transpose_batched, grid, dim3(256), 0, s, in, R, C, out);
  return hipGetLastError();
}

hipError_t launch_fourier_mix(const float* Xh, const float* W, int N, int M, int Fin, int Fout,
                              float* Yh, hipStream_t s) {
  const int64_t total = int64_t(N) * Fout * M;
  hipLaunchKernelGGL(k_fourier_mix, dim3(grid_1d(total, 256)), dim3(256), 0, s, Xh, W, N, M, Fin,
                     Fout, Yh);
  return hipGetLastError();
}

hipError_t launch_fourier_mix_t(const float* dYh, const float* W, int N, int M, int Fin, int Fout,
                                float* dXh, hipStream_t s) {
  const int64_t total = int64_t(N) * Fin * M;
  hipLaunchKernelGGL(k_fourier_mix_t, dim3(grid_1d(total, 256)), dim3(256), 0, s, dYh, W, N, M,
                     Fin, Fout, dXh);
  return hipGetLastError();
}

hipError_t launch_fourier_dw(const float* dYh, const float* Xh, int N, int M, int Fin, int Fout,
                             float* dW, hipStream_t s) {
  const int64_t total = int64_t(Fout) * Fin * M;
  hipLaunchKernelGGL(k_fourier_dw, dim3(grid_1d(total, 256)), dim3(256), 0, s, dYh, Xh, N, M, Fin,
                     Fout, dW);
  return hipGetLastError();
}

}  // namespace cg
