// gconv-LSTM cell pointwise kernels and the deterministic column reductions
// the cell's backward needs (lib/gconv_lstm.py:77-221, GConvLSTMCell.__call__).
//
// The graph-convolution parts of the cell are chebyshev5 calls (the x-conv of
// every time step batched into ONE call, the h-conv one call per step, both
// with the four gate weights concatenated into one [K*F, 4H] matrix, so the
// Chebyshev basis of x and of h is built once per step instead of four times,
// SURVEY.md §8f item 2).  What remains per step is pointwise and HBM-bound:
//
//   gates  [R][4H] = gx + gh + bias (blocks z | i | f | o, each H wide)
//   reference gate functions (lib/gconv_lstm.py:188-209):
//     z = tan, i = sigmoid, f = sigmoid, o = tanh      (CG_LSTM_GATES_REFERENCE)
//   standard LSTM: z = tanh, o = sigmoid               (CG_LSTM_GATES_STANDARD)
//   c' = f*c + i*z ;  h' = o * tanh(c')                (:215, :218)
//
// R = N*M rows (sample-major, vertex-minor: the [N][M][.] tensors of the
// reference).  forget_bias is accepted by the reference cell but never used
// (lib/gconv_lstm.py:49), so it is not applied here either.
//
// Bytes per row: forward reads 8H (gx, gh) + H (c) and writes 4H (saved
// activations) + 2H (c', h'); backward reads 4H + 3H (+H dc) and writes 4H + H.
#include "cg_internal.h"
#include "lstm_gates.h"

namespace cg {
namespace {

__device__ __forceinline__ float sigmoidf_(float a) { return gate_sigmoid(a); }

struct GateVals {
  float z, i, f, o;
};

template <bool REF>
__device__ __forceinline__ GateVals activate(float az, float ai, float af, float ao) {
  GateVals g;
  g.z = REF ? gate_tan(az) : gate_tanh(az);
  g.i = sigmoidf_(ai);
  g.f = sigmoidf_(af);
  g.o = REF ? gate_tanh(ao) : sigmoidf_(ao);
  return g;
}

// One thread per (row r, unit j).  Gate block q of row r lives at
// r*4H + q*H + j, so the 64 lanes of a wave read 4 coalesced 256-B runs
// per operand when H >= 64 (and whole rows when H < 64).
template <bool REF>
__global__ __launch_bounds__(256) void k_lstm_fwd(int total, int H, const float* __restrict__ gx,
                                                  const float* __restrict__ gh,
                                                  const float* __restrict__ bias,
                                                  const float* __restrict__ c,
                                                  float* __restrict__ c_out,
                                                  float* __restrict__ h_out,
                                                  float* __restrict__ act) {
#pragma clang fp contract(off)
  for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
    const int r = e / H, j = e - r * H;
    const int64_t g0 = int64_t(r) * 4 * H + j;
    float az = gx[g0], ai = gx[g0 + H], af = gx[g0 + 2 * H], ao = gx[g0 + 3 * H];
    if (gh) {  // zxt + zht (:186)
      az = az + gh[g0];
      ai = ai + gh[g0 + H];
      af = af + gh[g0 + 2 * H];
      ao = ao + gh[g0 + 3 * H];
    }
    if (bias) {  // ... + bzt
      az = az + bias[j];
      ai = ai + bias[H + j];
      af = af + bias[2 * H + j];
      ao = ao + bias[3 * H + j];
    }
    const GateVals g = activate<REF>(az, ai, af, ao);
    const float cp = c ? c[e] : 0.f;
    const float cn = g.f * cp + g.i * g.z;  // ft * c + it * zt (:215)
    const float hn = g.o * gate_tanh(cn);   // ot * tanh(new_c) (:218)
    c_out[e] = cn;
    h_out[e] = hn;
    if (act) {
      act[g0] = g.z;
      act[g0 + H] = g.i;
      act[g0 + 2 * H] = g.f;
      act[g0 + 3 * H] = g.o;
    }
  }
}

// Reverse of k_lstm_fwd (TF autodiff of the same expressions).  dh + dh_rec
// and dc are the gradients w.r.t. this step's h' and c' (NULL = 0); writes
// the pre-activation gradients dpre [R][4H] (the dy of the x- and h-conv
// contractions and of the bias) and dc_prev = dL/dc.
template <bool REF>
__global__ __launch_bounds__(256) void k_lstm_bwd(int total, int H, int act_um, const float* __restrict__ dh,
                                                  const float* __restrict__ dh_rec,
                                                  const float* __restrict__ dc,
                                                  const float* __restrict__ act,
                                                  const float* __restrict__ c,
                                                  const float* __restrict__ c_out,
                                                  float* __restrict__ dpre,
                                                  float* __restrict__ dc_prev) {
#pragma clang fp contract(off)
  for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
    const int r = e / H, j = e - r * H;
    const int64_t g0 = int64_t(r) * 4 * H + j;
    // act gate-major [R][4][H] or unit-major [R][H][4] (the sequence kernel's records)
    const int64_t a0 = act_um ? int64_t(r) * 4 * H + 4 * j : g0;
    const int as = act_um ? 1 : H;
    const float z = act[a0], i = act[a0 + as], f = act[a0 + 2 * as], o = act[a0 + 3 * as];
    const float cp = c ? c[e] : 0.f;
    const float tc = gate_tanh(c_out[e]);
    float dhv = dh ? dh[e] : 0.f;
    if (dh_rec) dhv = dhv + dh_rec[e];
    float dcn = dhv * o * (1.f - tc * tc);
    if (dc) dcn = dcn + dc[e];
    const float d_o = dhv * tc;
    const float d_i = dcn * z, d_z = dcn * i, d_f = dcn * cp;
    dpre[g0] = REF ? d_z * (1.f + z * z) : d_z * (1.f - z * z);  // tan' = 1 + tan^2
    dpre[g0 + H] = d_i * (i * (1.f - i));
    dpre[g0 + 2 * H] = d_f * (f * (1.f - f));
    dpre[g0 + 3 * H] = REF ? d_o * (1.f - o * o) : d_o * (o * (1.f - o));
    if (dc_prev) dc_prev[e] = dcn * f;
  }
}

// k_lstm_bwd on unit-major act records (the sequence kernel's), four units
// per lane: every operand moves in 16-byte accesses (H % 4 == 0, 16-byte
// aligned operands); per element the expressions of k_lstm_bwd, bitwise
template <bool REF>
__global__ __launch_bounds__(256) void k_lstm_bwd_um4(int total4, int H, const float* __restrict__ dh,
                                                      const float* __restrict__ dh_rec,
                                                      const float* __restrict__ dc,
                                                      const float* __restrict__ act,
                                                      const float* __restrict__ c,
                                                      const float* __restrict__ c_out,
                                                      float* __restrict__ dpre,
                                                      float* __restrict__ dc_prev) {
#pragma clang fp contract(off)
  const int H4 = H >> 2;
  for (int e4 = blockIdx.x * 256 + threadIdx.x; e4 < total4; e4 += gridDim.x * 256) {
    const int r = e4 / H4, j0 = (e4 - r * H4) * 4;
    const int64_t e = int64_t(r) * H + j0;  // element (r, j0)
    auto ld4 = [&](const float* p) {
      return p ? *reinterpret_cast<const float4*>(p + e) : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    const float4 cp4 = ld4(c), co4 = ld4(c_out), dh4 = ld4(dh), dr4 = ld4(dh_rec), dc4 = ld4(dc);
    float dp[4][4], dcp[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float4 a = *reinterpret_cast<const float4*>(act + int64_t(r) * 4 * H + 4 * (j0 + u));
      const float z = a.x, i = a.y, f = a.z, o = a.w;
      const float cp = (&cp4.x)[u];
      const float tc = gate_tanh((&co4.x)[u]);
      float dhv = dh ? (&dh4.x)[u] : 0.f;
      if (dh_rec) dhv = dhv + (&dr4.x)[u];
      float dcn = dhv * o * (1.f - tc * tc);
      if (dc) dcn = dcn + (&dc4.x)[u];
      const float d_o = dhv * tc;
      const float d_i = dcn * z, d_z = dcn * i, d_f = dcn * cp;
      dp[0][u] = REF ? d_z * (1.f + z * z) : d_z * (1.f - z * z);
      dp[1][u] = d_i * (i * (1.f - i));
      dp[2][u] = d_f * (f * (1.f - f));
      dp[3][u] = REF ? d_o * (1.f - o * o) : d_o * (o * (1.f - o));
      dcp[u] = dcn * f;
    }
    const int64_t g0 = int64_t(r) * 4 * H + j0;
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<float4*>(dpre + g0 + g * H) = make_float4(dp[g][0], dp[g][1], dp[g][2], dp[g][3]);
    if (dc_prev) *reinterpret_cast<float4*>(dc_prev + e) = make_float4(dcp[0], dcp[1], dcp[2], dcp[3]);
  }
}

// Column sums of A [R][C] as per-chunk partial slabs slab[chunk][C]: block
// (chunk, 64-column tile) = 4 waves; wave w sums rows c0 + w, c0 + w + 4, ...
// of the chunk for its 64 columns (one coalesced 256-B load per row), then the
// four partials are added in wave order -- bitwise reproducible.
__global__ __launch_bounds__(256) void k_colsum_slabs(const float* __restrict__ A, int64_t R, int C,
                                                      int64_t rows_per_chunk,
                                                      float* __restrict__ slab) {
#pragma clang fp contract(off)
  __shared__ float part[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.y * 64 + lane;
  const int64_t c0 = int64_t(blockIdx.x) * rows_per_chunk;
  const int64_t c1 = (c0 + rows_per_chunk < R) ? c0 + rows_per_chunk : R;
  float s = 0.f;
  if (col < C) {
#pragma unroll 4
    for (int64_t r = c0 + w; r < c1; r += 4) s = s + A[r * C + col];
  }
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && col < C)
    slab[int64_t(blockIdx.x) * C + col] = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
}

inline int grid1d(int total) {
  int g = (total + 255) / 256;
  return g > 65536 ? 65536 : (g < 1 ? 1 : g);
}

}  // namespace

hipError_t launch_lstm_fwd(int gates, int64_t R, int H, const float* gx, const float* gh,
                           const float* bias, const float* c, float* c_out, float* h_out,
                           float* act, hipStream_t s) {
  const int total = int(R * H);
  if (gates == 0)
    hipLaunchKernelGGL(k_lstm_fwd<true>, dim3(grid1d(total)), dim3(256), 0, s, total, H, gx, gh,
                       bias, c, c_out, h_out, act);
  else
    hipLaunchKernelGGL(k_lstm_fwd<false>, dim3(grid1d(total)), dim3(256), 0, s, total, H, gx, gh,
                       bias, c, c_out, h_out, act);
  return hipGetLastError();
}

hipError_t launch_lstm_bwd(int gates, int64_t R, int H, const float* dh, const float* dh_rec,
                           const float* dc,
                           const float* act, const float* c, const float* c_out, float* dpre,
                           float* dc_prev, hipStream_t s, int act_um) {
  const int total = int(R * H);
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (act_um && H % 4 == 0 && al(dh) && al(dh_rec) && al(dc) && al(act) && al(c) && al(c_out) &&
      al(dpre) && al(dc_prev)) {
    const int total4 = total / 4;
    if (gates == 0)
      hipLaunchKernelGGL(k_lstm_bwd_um4<true>, dim3(grid1d(total4)), dim3(256), 0, s, total4, H, dh,
                         dh_rec, dc, act, c, c_out, dpre, dc_prev);
    else
      hipLaunchKernelGGL(k_lstm_bwd_um4<false>, dim3(grid1d(total4)), dim3(256), 0, s, total4, H, dh,
                         dh_rec, dc, act, c, c_out, dpre, dc_prev);
    return hipGetLastError();
  }
  if (gates == 0)
    hipLaunchKernelGGL(k_lstm_bwd<true>, dim3(grid1d(total)), dim3(256), 0, s, total, H, act_um, dh,
                       dh_rec, dc, act, c, c_out, dpre, dc_prev);
  else
    hipLaunchKernelGGL(k_lstm_bwd<false>, dim3(grid1d(total)), dim3(256), 0, s, total, H, act_um, dh,
                       dh_rec, dc, act, c, c_out, dpre, dc_prev);
  return hipGetLastError();
}

int colsum_chunks(int64_t R) {
  int64_t c = (R + 1023) / 1024;  // ~1024 rows per chunk, at most 1024 chunks
  if (c > 1024) c = 1024;
  return int(c < 1 ? 1 : c);
}

hipError_t launch_colsum_slabs(const float* A, int64_t R, int C, float* slab, hipStream_t s) {
  const int chunks = colsum_chunks(R);
  const int64_t rpc = (R + chunks - 1) / chunks;
  hipLaunchKernelGGL(k_colsum_slabs, dim3(chunks, (C + 63) / 64), dim3(256), 0, s, A, R, C, rpc,
                     slab);
  return hipGetLastError();
}

}  // namespace cg
