// Elementwise pieces of the residual GraphConv block and its training step
// (lib/graph_conv.py:234-330, lib/graph_model.py:246-298), for the paths whose
// contraction kernel does not apply them itself:
//   k_act_fwd   y = act(y + res)              (b1relu of x + x_identity, :256-262)
//   k_relu_bwd  dz = y > 0 ? dy : 0           (ReLU gradient from its output)
//   k_bias_act_fwd / k_bias_act_bwd
//               y = act(x + b) with a per-filter (b1*, :189-193) or per-vertex-
//               and-filter (b2relu, :195-199) bias; dz = dy * act'(y)
//   k_mse_*     loss = mean((labels - pred)^2), dpred = 2 (pred - labels) / n
//               (tf.reduce_mean(tf.square(tf.subtract(labels, logits))),
//               lib/graph_model.py:255), fixed-order two-stage reduction, plus
//               the loss moving average of :265-273 (optional)
//   k_slice_channels / k_stack_merge_*
//               the stacked-input ResGNN (_inference with stack_num > 1,
//               lib/graph_conv.py:272-303): channel groups of the input, and
//               X = sum_i relu(net_i(x_i)) * w_i with w_i [M][F] broadcast over N
//   k_dropout   DropoutWrapper(output_keep_prob) of glstm_layer
//               (lib/gconv_lstm.py:616, :623 -> tf.nn.dropout 1.x):
//               y = (x / keep) * floor(keep + u), u ~ U[0,1) from a counter hash of
//               (seed, element), so the backward regenerates the same mask:
//               dx = (dy * floor(keep + u)) / keep (the Mul, then RealDiv gradient)
//   k_clip_norm tf.clip_by_norm + tf.check_numerics of gconvRNN.Model's
//               optimizer (lib/gconvRNN.py:392-402): t' = (t * c) / max(||t||, c),
//               ||t|| from a fixed-order sum of squares, non-finite t' flagged
// The fast resident forward and the streaming row GEMM apply the residual /
// ReLU epilogue in their own y store; these kernels are the fallback.
#include "cg_internal.h"

namespace cg {
namespace {

inline int grid1d(int64_t n, int per_block) {
  int64_t g = (n + per_block - 1) / per_block;
  return int(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

__global__ __launch_bounds__(256) void k_act_fwd(float* __restrict__ y, const float* __restrict__ res,
                                                 int act, int64_t n) {
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    float v = y[i];
    if (res) v = v + res[i];
    if (act) v = v > 0.f ? v : 0.f;
    y[i] = v;
  }
}

// U[0, 1) of element i under `seed` (splitmix64 finaliser of a Weyl sequence;
// 24 random bits, so u + keep rounds like tf.random_uniform's fp32 draw)
__device__ __forceinline__ float drop_u(unsigned long long seed, int64_t i) {
  unsigned long long z = seed + 0x9E3779B97F4A7C15ull * (static_cast<unsigned long long>(i) + 1ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return float(z >> 40) * (1.f / 16777216.f);
}

// bwd = 0: y = (x / keep) * floor(keep + u);  bwd = 1: y = (x * floor(keep + u)) / keep
__device__ __forceinline__ float drop_one(float x, float keep, unsigned long long seed, int64_t i,
                                          int bwd) {
#pragma clang fp contract(off)
  const float b = floorf(keep + drop_u(seed, i));
  return bwd ? (x * b) / keep : (x / keep) * b;
}

__global__ __launch_bounds__(256) void k_dropout(const float* __restrict__ x, float* __restrict__ y,
                                                 int64_t n, float keep, unsigned long long seed,
                                                 int bwd) {
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256)
    y[i] = drop_one(x[i], keep, seed, i, bwd);
}

// 16-byte aligned x / y: four elements per thread (one dwordx4 load and
// store; the same per-element draw and arithmetic, so the same bits), the
// n % 4 tail by the first threads
__global__ __launch_bounds__(256) void k_dropout4(const float4* __restrict__ x, float4* __restrict__ y,
                                                  int64_t n, float keep, unsigned long long seed,
                                                  int bwd) {
  const int64_t n4 = n >> 2;
  for (int64_t q = int64_t(blockIdx.x) * 256 + threadIdx.x; q < n4; q += int64_t(gridDim.x) * 256) {
    const float4 v = x[q];
    float4 o;
    o.x = drop_one(v.x, keep, seed, 4 * q, bwd);
    o.y = drop_one(v.y, keep, seed, 4 * q + 1, bwd);
    o.z = drop_one(v.z, keep, seed, 4 * q + 2, bwd);
    o.w = drop_one(v.w, keep, seed, 4 * q + 3, bwd);
    y[q] = o;
  }
  const int64_t t = 4 * n4 + int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (t < n)
    reinterpret_cast<float*>(y)[t] =
        drop_one(reinterpret_cast<const float*>(x)[t], keep, seed, t, bwd);
}

// one workgroup: t <- (t * c) / max(sqrt(sum t^2), c) in place (the norm's sum
// in a fixed order: lane-strided partials, then a fixed LDS tree), and
// *nonfinite = 1 when any result is NaN / Inf
__global__ __launch_bounds__(1024) void k_clip_norm(float* __restrict__ t, int64_t n, float c,
                                                    int* __restrict__ nonfinite) {
#pragma clang fp contract(off)
  __shared__ float part[1024];
  __shared__ int bad;
  const int tid = threadIdx.x;
  float s2 = 0.f;
  for (int64_t i = tid; i < n; i += 1024) s2 = s2 + t[i] * t[i];
  part[tid] = s2;
  if (tid == 0) bad = 0;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if (tid < w) part[tid] = part[tid] + part[tid + w];
    __syncthreads();
  }
  const float l2sum = part[0];
  // tf.clip_by_norm: l2norm = l2sum > 0 ? sqrt(l2sum) : l2sum
  const float l2norm = l2sum > 0.f ? sqrtf(l2sum) : l2sum;
  const float den = l2norm > c ? l2norm : c;
  int my_bad = 0;
  for (int64_t i = tid; i < n; i += 1024) {
    const float v = (t[i] * c) / den;
    t[i] = v;
    if (!isfinite(v)) my_bad = 1;
  }
  if (my_bad) bad = 1;  // benign race: every writer stores 1
  __syncthreads();
  if (tid == 0 && bad && nonfinite) *nonfinite = 1;
}

__global__ __launch_bounds__(256) void k_relu_bwd(const float* __restrict__ dy,
                                                  const float* __restrict__ y,
                                                  float* __restrict__ dz, int64_t n) {
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256)
    dz[i] = y[i] > 0.f ? dy[i] : 0.f;
}

// the same, four elements per lane (16-byte aligned operands, n % 4 == 0)
__global__ __launch_bounds__(256) void k_relu_bwd4(const float4* __restrict__ dy,
                                                   const float4* __restrict__ y,
                                                   float4* __restrict__ dz, int64_t n4) {
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n4; i += int64_t(gridDim.x) * 256) {
    const float4 g = dy[i], v = y[i];
    dz[i] = make_float4(v.x > 0.f ? g.x : 0.f, v.y > 0.f ? g.y : 0.f, v.z > 0.f ? g.z : 0.f,
                        v.w > 0.f ? g.w : 0.f);
  }
}

// y = act(x + bias[i % blen]) (bias NULL: no add); act 0 none, 1 ReLU, 2 tanh.
// x and y may alias.
__global__ __launch_bounds__(256) void k_bias_act_fwd(const float* __restrict__ x,
                                                      const float* __restrict__ bias, int64_t blen,
                                                      int act, int64_t n, float* __restrict__ y) {
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    float v = x[i];
    if (bias) v = v + bias[i % blen];
    if (act == 1) v = v > 0.f ? v : 0.f;
    else if (act == 2) v = tanhf(v);
    y[i] = v;
  }
}

// dz = dy * act'(y) from the forward OUTPUT y (TF ReluGrad / TanhGrad:
// dy * (1 - y*y)).  dz and dy may alias.
__global__ __launch_bounds__(256) void k_bias_act_bwd(const float* __restrict__ dy,
                                                      const float* __restrict__ y, int act,
                                                      int64_t n, float* __restrict__ dz) {
#pragma clang fp contract(off)
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    const float g = dy[i];
    float d = g;
    if (act == 1) d = y[i] > 0.f ? g : 0.f;
    else if (act == 2) { const float t = y[i]; d = g * (1.f - t * t); }
    dz[i] = d;
  }
}

// Block z sums (labels - pred)^2 over its contiguous chunk (lanes strided,
// then a fixed-order tree in LDS) and writes dpred for the same elements.
__global__ __launch_bounds__(256) void k_mse_part(const float* __restrict__ pred,
                                                  const float* __restrict__ labels, int64_t n,
                                                  int64_t chunk, float inv2n,
                                                  float* __restrict__ slab,
                                                  float* __restrict__ dpred) {
#pragma clang fp contract(off)
  __shared__ float part[256];
  const int64_t c0 = int64_t(blockIdx.x) * chunk;
  const int64_t c1 = (c0 + chunk < n) ? c0 + chunk : n;
  float s = 0.f;
  for (int64_t i = c0 + threadIdx.x; i < c1; i += 256) {
    const float d = labels[i] - pred[i];
    s = s + d * d;
    if (dpred) dpred[i] = (pred[i] - labels[i]) * inv2n;
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (int(threadIdx.x) < w) part[threadIdx.x] = part[threadIdx.x] + part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) slab[blockIdx.x] = part[0];
}

// ema (optional, float[3] = {biased, average, local_step}): TF-1.x
// ExponentialMovingAverage(decay).apply([loss]) of a Tensor, i.e.
// assign_moving_average(zero_debias=True) (moving_averages.py).  TF version assumption: the
// reference pins only "tensorflow-gpu" (requirements.txt:7) and its notebooks ran Python
// 3.4-3.6 (2017, TF 1.0-1.3), where apply() zero-debiases every Tensor average; TF >= 1.4
// added ExponentialMovingAverage(zero_debias=False) and would give 0.1*loss after step 1.
// Parity of this choice is unpinned (no TF in the image):
//   d1 = 1 - decay; biased -= (biased - loss) * d1; step += 1;
//   average -= average - biased / (1 - (1 - d1)^step)
__global__ __launch_bounds__(256) void k_mse_final(const float* __restrict__ slab, int nslab,
                                                   float inv_n, float* __restrict__ loss,
                                                   float* __restrict__ ema, float decay) {
#pragma clang fp contract(off)
  __shared__ float part[256];
  float s = 0.f;
  for (int z = threadIdx.x; z < nslab; z += 256) s = s + slab[z];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (int(threadIdx.x) < w) part[threadIdx.x] = part[threadIdx.x] + part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float l = part[0] * inv_n;
    *loss = l;
    if (ema) {
      const float d1 = 1.f - decay;
      const float biased = ema[0] - (ema[0] - l) * d1;
      const float step = ema[2] + 1.f;
      const float bias_factor = 1.f - powf(1.f - d1, step);
      ema[0] = biased;
      ema[1] = ema[1] - (ema[1] - biased / bias_factor);
      ema[2] = step;
    }
  }
}

// out[r][c] = x[r][c0 + c], c < w: the channel group x[..., c0:c0+w] of an
// [rows][C] tensor (the reshape / unstack / concat of lib/graph_conv.py:281-286)
__global__ __launch_bounds__(256) void k_slice_channels(const float* __restrict__ x, int64_t rows,
                                                        int C, int c0, int w,
                                                        float* __restrict__ out) {
  const int64_t n = rows * w;
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    const int64_t r = i / w;
    out[i] = x[r * C + c0 + (i - r * w)];
  }
}

// y = (accumulate ? y : 0) + relu(o) * w[i mod MF]   (lib/graph_conv.py:297-301:
// X = x1 * w1, then X = X + x1 * w1 with x1 = relu(residual_network(x_i)))
__global__ __launch_bounds__(256) void k_stack_merge_fwd(const float* __restrict__ o,
                                                         const float* __restrict__ w, int64_t n,
                                                         int64_t MF, int accumulate,
                                                         float* __restrict__ y) {
#pragma clang fp contract(off)
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    const float x1 = o[i] > 0.f ? o[i] : 0.f;
    const float v = x1 * w[i % MF];
    y[i] = accumulate ? y[i] + v : v;
  }
}

// TF gradients of X (+)= relu(o) * w: dx1 = dy * w (Mul grad, no reduction on
// x1's side), do = ReluGrad(dx1, relu(o)) = o > 0 ? dx1 : 0
__global__ __launch_bounds__(256) void k_stack_merge_bwd(const float* __restrict__ dy,
                                                         const float* __restrict__ o,
                                                         const float* __restrict__ w, int64_t n,
                                                         int64_t MF, float* __restrict__ d_o) {
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256)
    d_o[i] = o[i] > 0.f ? dy[i] * w[i % MF] : 0.f;
}

// dw[j] = sum_n relu(o[n][j]) * dy[n][j], n ascending (the broadcast reduction of
// the Mul gradient over the batch axis; fixed order, bitwise reproducible)
__global__ __launch_bounds__(256) void k_stack_merge_dw(const float* __restrict__ dy,
                                                        const float* __restrict__ o, int N,
                                                        int64_t MF, float* __restrict__ dw) {
#pragma clang fp contract(off)
  const int64_t j = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (j >= MF) return;
  float s = 0.f;
  for (int n = 0; n < N; ++n) {
    const float x1 = o[n * MF + j] > 0.f ? o[n * MF + j] : 0.f;
    s = s + x1 * dy[n * MF + j];
  }
  dw[j] = s;
}

}  // namespace

hipError_t launch_act_fwd(float* y, const float* res, int act, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_act_fwd, dim3(grid1d(n, 256)), dim3(256), 0, s, y, res, act, n);
  return hipGetLastError();
}

hipError_t launch_relu_bwd(const float* dy, const float* y, float* dz, int64_t n, hipStream_t s) {
  const bool a16 = ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(y) |
                     reinterpret_cast<uintptr_t>(dz)) & 15) == 0;
  if (a16 && n % 4 == 0) {
    hipLaunchKernelGGL(k_relu_bwd4, dim3(grid1d(n / 4, 256)), dim3(256), 0, s,
                       reinterpret_cast<const float4*>(dy), reinterpret_cast<const float4*>(y),
                       reinterpret_cast<float4*>(dz), n / 4);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_relu_bwd, dim3(grid1d(n, 256)), dim3(256), 0, s, dy, y, dz, n);
  return hipGetLastError();
}

hipError_t launch_bias_act_fwd(const float* x, const float* bias, int64_t blen, int act, int64_t n,
                               float* y, hipStream_t s) {
  hipLaunchKernelGGL(k_bias_act_fwd, dim3(grid1d(n, 256)), dim3(256), 0, s, x, bias, blen, act, n, y);
  return hipGetLastError();
}

hipError_t launch_bias_act_bwd(const float* dy, const float* y, int act, int64_t n, float* dz,
                               hipStream_t s) {
  hipLaunchKernelGGL(k_bias_act_bwd, dim3(grid1d(n, 256)), dim3(256), 0, s, dy, y, act, n, dz);
  return hipGetLastError();
}

int mse_chunks(int64_t n) {
  int64_t c = (n + 4095) / 4096;  // ~4096 elements per block, at most 1024 blocks
  if (c > 1024) c = 1024;
  return int(c < 1 ? 1 : c);
}

hipError_t launch_mse(const float* pred, const float* labels, int64_t n, float* slab, float* loss,
                      float* dpred, hipStream_t s, float* ema, float decay) {
  const int chunks = mse_chunks(n);
  const int64_t chunk = (n + chunks - 1) / chunks;
  hipLaunchKernelGGL(k_mse_part, dim3(chunks), dim3(256), 0, s, pred, labels, n, chunk,
                     float(2.0 / double(n)), slab, dpred);
  hipLaunchKernelGGL(k_mse_final, dim3(1), dim3(256), 0, s, slab, chunks, float(1.0 / double(n)),
                     loss, ema, decay);
  return hipGetLastError();
}

hipError_t launch_slice_channels(const float* x, int64_t rows, int C, int c0, int c1, float* out,
                                 hipStream_t s) {
  hipLaunchKernelGGL(k_slice_channels, dim3(grid1d(rows * (c1 - c0), 256)), dim3(256), 0, s, x, rows,
                     C, c0, c1 - c0, out);
  return hipGetLastError();
}

hipError_t launch_stack_merge_fwd(const float* o, const float* w, int N, int64_t MF, int accumulate,
                                  float* y, hipStream_t s) {
  const int64_t n = int64_t(N) * MF;
  hipLaunchKernelGGL(k_stack_merge_fwd, dim3(grid1d(n, 256)), dim3(256), 0, s, o, w, n, MF,
                     accumulate, y);
  return hipGetLastError();
}

hipError_t launch_stack_merge_bwd(const float* dy, const float* o, const float* w, int N, int64_t MF,
                                  float* d_o, float* dw, hipStream_t s) {
  const int64_t n = int64_t(N) * MF;
  if (d_o)
    hipLaunchKernelGGL(k_stack_merge_bwd, dim3(grid1d(n, 256)), dim3(256), 0, s, dy, o, w, n, MF, d_o);
  if (dw)
    hipLaunchKernelGGL(k_stack_merge_dw, dim3(int((MF + 255) / 256)), dim3(256), 0, s, dy, o, N, MF,
                       dw);
  return hipGetLastError();
}

hipError_t launch_dropout(const float* x, float* y, int64_t n, float keep, unsigned long long seed,
                          int bwd, hipStream_t s) {
  if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0 && n >= 4) {
    hipLaunchKernelGGL(k_dropout4, dim3(grid1d((n + 3) / 4, 256)), dim3(256), 0, s,
                       reinterpret_cast<const float4*>(x), reinterpret_cast<float4*>(y), n, keep,
                       seed, bwd);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_dropout, dim3(grid1d(n, 256)), dim3(256), 0, s, x, y, n, keep, seed, bwd);
  return hipGetLastError();
}

hipError_t launch_clip_norm(float* t, int64_t n, float c, int* nonfinite, hipStream_t s) {
  hipLaunchKernelGGL(k_clip_norm, dim3(1), dim3(1024), 0, s, t, n, c, nonfinite);
  return hipGetLastError();
}

}  // namespace cg
