// Ops either side of the Chebyshev filter on gfx950:
//   perm_gather  -- lib/coarsening.py:219-240 perm_data (fake vertices -> 0)
//   maxpool      -- lib/graph_conv.py:201-209 mpool1 (+ first-max argmax, scatter-free grad)
//   avgpool      -- lib/graph_conv.py:211-218 apool1
//   adam         -- lib/graph_model.py:293-298 (TF-1.x AdamOptimizer update rule)
// All are HBM-streaming, one thread per output element, F (the feature axis,
// contiguous in memory) on consecutive lanes so loads and stores coalesce.
#include "cg_internal.h"

namespace cg {
namespace {

inline int grid_for(int64_t total, int block) {
  int64_t g = (total + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return int(g);
}

__global__ __launch_bounds__(256) void k_perm_gather(const float* __restrict__ x,
                                                     const int32_t* __restrict__ perm, int N,
                                                     int M_in, int M_out, int F,
                                                     float* __restrict__ out) {
  const int64_t total = int64_t(N) * M_out * F;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t f = i % F;
    const int64_t t = i / F;
    const int64_t v = t % M_out, n = t / M_out;
    const int src = perm[v];
    out[i] = (src >= 0 && src < M_in) ? x[(n * M_in + src) * F + f] : 0.f;
  }
}

__global__ __launch_bounds__(256) void k_maxpool_fwd(const float* __restrict__ x, int N, int M,
                                                     int F, int p, float* __restrict__ y,
                                                     int32_t* __restrict__ arg) {
  const int Mo = M / p;
  const int64_t total = int64_t(N) * Mo * F;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t f = i % F;
    const int64_t t = i / F;
    const int64_t o = t % Mo, n = t / Mo;
    const float* base = x + (n * M + o * p) * F + f;
    float best = base[0];
    int bi = 0;
    for (int j = 1; j < p; ++j) {
      const float v = base[int64_t(j) * F];
      if (best < v) {  // strict: the first maximum in window order wins
        best = v;
        bi = j;
      }
    }
    y[i] = best;
    if (arg) arg[i] = int32_t(o * p + bi);
  }
}

__global__ __launch_bounds__(256) void k_maxpool_bwd(const float* __restrict__ dy,
                                                     const int32_t* __restrict__ arg, int N, int M,
                                                     int F, int p, float* __restrict__ dx) {
  const int Mo = M / p;
  const int64_t total = int64_t(N) * M * F;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t f = i % F;
    const int64_t t = i / F;
    const int64_t m = t % M, n = t / M;
    const int64_t o = m / p;
    const int64_t oi = (n * Mo + o) * F + f;
    dx[i] = (arg[oi] == m) ? dy[oi] : 0.f;
  }
}

__global__ __launch_bounds__(256) void k_avgpool_fwd(const float* __restrict__ x, int N, int M,
                                                     int F, int p, float* __restrict__ y) {
#pragma clang fp contract(off)
  const int Mo = M / p;
  const int64_t total = int64_t(N) * Mo * F;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t f = i % F;
    const int64_t t = i / F;
    const int64_t o = t % Mo, n = t / Mo;
    const float* base = x + (n * M + o * p) * F + f;
    float s = 0.f;
    for (int j = 0; j < p; ++j) s = s + base[int64_t(j) * F];
    y[i] = s / float(p);
  }
}

__global__ __launch_bounds__(256) void k_avgpool_bwd(const float* __restrict__ dy, int N, int M,
                                                     int F, int p, float* __restrict__ dx) {
  const int Mo = M / p;
  const int64_t total = int64_t(N) * M * F;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t f = i % F;
    const int64_t t = i / F;
    const int64_t m = t % M, n = t / M;
    dx[i] = dy[(n * Mo + m / p) * F + f] / float(p);
  }
}

// m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2 ; p -= lr_t m / (sqrt(v) + eps)
// with lr_t = lr sqrt(1-b2^t)/(1-b1^t) computed on the host (TF's ApplyAdam).
// TF-1.x Adam on one element (lib/graph_model.py:293-298 via tf.train.AdamOptimizer);
// the arithmetic is cg_internal.h::adam_math, shared with cheb_fwd_fast's
// Adam-in-forward prologue, so every Adam path rounds identically.
__device__ __forceinline__ void adam_elem(float* __restrict__ param, float* __restrict__ m,
                                          float* __restrict__ v, int64_t i, float grad,
                                          float grad_scale, float lr_t, float beta1, float beta2,
                                          float eps) {
  const AdamElem r = adam_math(param[i], m[i], v[i], grad, grad_scale, lr_t, beta1, beta2, eps);
  m[i] = r.m;
  v[i] = r.v;
  param[i] = r.p;
}

__global__ __launch_bounds__(256) void k_adam(float* __restrict__ param,
                                              const float* __restrict__ grad, float* __restrict__ m,
                                              float* __restrict__ v, int64_t n, float lr_t,
                                              float beta1, float beta2, float eps,
                                              float grad_scale) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x)
    adam_elem(param, m, v, i, grad[i], grad_scale, lr_t, beta1, beta2, eps);
}

// The other update rules of gconvRNN.Model._build_optim (lib/gconvRNN.py:381-389)
// with TF 1.x's kernels (training_ops.cc), grad * grad_scale first:
//   GradientDescent (ApplyGradientDescent): p -= g lr
//   RMSProp (ApplyRMSProp, not centered):   ms += (g^2 - ms)(1 - rho)
//                                           mom = mom momentum + (g lr) / sqrt(ms + eps)
//                                           p -= mom
__global__ __launch_bounds__(256) void k_sgd(float* __restrict__ param, const float* __restrict__ grad,
                                             int64_t n, float lr, float grad_scale) {
#pragma clang fp contract(off)
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x) {
    const float g = grad[i] * grad_scale;
    param[i] = param[i] - g * lr;
  }
}

__global__ __launch_bounds__(256) void k_rmsprop(float* __restrict__ param,
                                                 const float* __restrict__ grad,
                                                 float* __restrict__ ms, float* __restrict__ mom,
                                                 int64_t n, float lr, float rho, float momentum,
                                                 float eps, float grad_scale) {
#pragma clang fp contract(off)
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x) {
    const float g = grad[i] * grad_scale;
    const float s = ms[i] + (g * g - ms[i]) * (1.f - rho);
    const float u = mom[i] * momentum + (g * lr) / sqrtf(s + eps);
    ms[i] = s;
    mom[i] = u;
    param[i] = param[i] - u;
  }
}

// Slab reduction + Adam for a step with no exchange between them (one GPU):
// the summation is k_reduce_slabs' (wave w sums slabs w, w+16, ..., then the 16
// partials in wave order), so grad is bitwise the unfused dW; wave 0 then
// applies the update.  Saves the separate k_adam launch (~5 us, dispatch-bound).
__global__ __launch_bounds__(1024) void k_reduce_slabs_adam(const float* __restrict__ slab,
                                                            int nslab, int64_t count,
                                                            float* __restrict__ grad,
                                                            AdamStep a) {
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i = int64_t(blockIdx.x) * 64 + lane;
  // wave 0's Adam operands, loaded behind the slab loads instead of after the sum
  float p0 = 0.f, m0 = 0.f, v0 = 0.f;
  if (w == 0 && i < count) {
    p0 = a.param[i];
    m0 = a.m[i];
    v0 = a.v[i];
  }
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
    grad[i] = t;
    const AdamElem r = adam_math(p0, m0, v0, t, a.grad_scale, a.lr_t, a.beta1, a.beta2, a.eps);
    a.m[i] = r.m;
    a.v[i] = r.v;
    a.param[i] = r.p;
  }
}

}  // namespace

hipError_t launch_perm_gather(const float* x, const int32_t* perm, int N, int M_in, int M_out,
                              int F, float* out, hipStream_t s) {
  const int64_t total = int64_t(N) * M_out * F;
  hipLaunchKernelGGL(k_perm_gather, dim3(grid_for(total, 256)), dim3(256), 0, s, x, perm, N, M_in,
                     M_out, F, out);
  return hipGetLastError();
}

hipError_t launch_maxpool_fwd(const float* x, int N, int M, int F, int p, float* y, int32_t* arg,
                              hipStream_t s) {
  const int64_t total = int64_t(N) * (M / p) * F;
  hipLaunchKernelGGL(k_maxpool_fwd, dim3(grid_for(total, 256)), dim3(256), 0, s, x, N, M, F, p, y,
                     arg);
  return hipGetLastError();
}

hipError_t launch_maxpool_bwd(const float* dy, const int32_t* arg, int N, int M, int F, int p,
                              float* dx, hipStream_t s) {
  const int64_t total = int64_t(N) * M * F;
  hipLaunchKernelGGL(k_maxpool_bwd, dim3(grid_for(total, 256)), dim3(256), 0, s, dy, arg, N, M, F,
                     p, dx);
  return hipGetLastError();
}

hipError_t launch_avgpool_fwd(const float* x, int N, int M, int F, int p, float* y,
                              hipStream_t s) {
  const int64_t total = int64_t(N) * (M / p) * F;
  hipLaunchKernelGGL(k_avgpool_fwd, dim3(grid_for(total, 256)), dim3(256), 0, s, x, N, M, F, p, y);
  return hipGetLastError();
}

hipError_t launch_avgpool_bwd(const float* dy, int N, int M, int F, int p, float* dx,
                              hipStream_t s) {
  const int64_t total = int64_t(N) * M * F;
  hipLaunchKernelGGL(k_avgpool_bwd, dim3(grid_for(total, 256)), dim3(256), 0, s, dy, N, M, F, p,
                     dx);
  return hipGetLastError();
}

hipError_t launch_adam(float* param, const float* grad, float* m, float* v, int64_t n, float lr_t,
                       float beta1, float beta2, float eps, float grad_scale, hipStream_t s) {
  hipLaunchKernelGGL(k_adam, dim3(grid_for(n, 256)), dim3(256), 0, s, param, grad, m, v, n, lr_t,
                     beta1, beta2, eps, grad_scale);
  return hipGetLastError();
}

hipError_t launch_sgd(float* param, const float* grad, int64_t n, float lr, float grad_scale,
                      hipStream_t s) {
  hipLaunchKernelGGL(k_sgd, dim3(grid_for(n, 256)), dim3(256), 0, s, param, grad, n, lr, grad_scale);
  return hipGetLastError();
}

hipError_t launch_rmsprop(float* param, const float* grad, float* ms, float* mom, int64_t n, float lr,
                          float rho, float momentum, float eps, float grad_scale, hipStream_t s) {
  hipLaunchKernelGGL(k_rmsprop, dim3(grid_for(n, 256)), dim3(256), 0, s, param, grad, ms, mom, n, lr,
                     rho, momentum, eps, grad_scale);
  return hipGetLastError();
}

hipError_t launch_reduce_slabs_adam(const float* slab, int nslab, int64_t count, float* grad,
                                    const AdamStep& a, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce_slabs_adam, dim3(unsigned((count + 63) / 64)), dim3(1024), 0, s, slab,
                     nslab, count, grad, a);
  return hipGetLastError();
}

}  // namespace cg
