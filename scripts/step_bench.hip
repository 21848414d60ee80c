// Micro-benchmark: cost of one resident Chebyshev step, built up piece by
// piece (barrier-only, +12 register-index LDS gathers, +MFMA pair every other
// step), to locate the per-step overhead of cheb_fwd_resident.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/step_bench.hip -o build/step_bench
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int T = 1024;
constexpr int MP = 993;

template <int VAR>
__global__ __launch_bounds__(T) void step_kernel(int nsteps, int M, const int* __restrict__ colmap,
                                                 float* out) {
#pragma clang fp contract(off)
  extern __shared__ float s[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, li = lane & 31;
  int c[12];
  float v[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    c[j] = colmap[j * T + tid];
    v[j] = 0.01f * (j + 1);
  }
  for (int i = tid; i < 3 * MP; i += T) s[i] = float(i % 7);
  float* sB = s + 3 * MP + 3;
  __syncthreads();
  f32x16 acc0 = {}, acc1 = {};
  const int ntiles = (M + 31) >> 5;
  for (int k = 1; k < nsteps; ++k) {
    if (VAR >= 2 && (k & 1) == 0) {
      const int kk = k - 2 + h, slot = kk % 3;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int tile = wave + t * 16;
        if (tile < ntiles) {
          const int m = tile * 32 + li;
          float a = 0.f;
          if (m < M) {
            a = s[slot * MP + m];
            if (VAR >= 3) sB[m * 25 + kk] = a;
          }
          if (t == 0) acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, 0.5f, acc0, 0, 0, 0);
          else acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, 0.5f, acc1, 0, 0, 0);
        }
      }
    }
    const int cur = k % 3, prv = (k + 2) % 3, prv2 = (k + 1) % 3;
    const float* Tp = s + prv * MP;
    if (tid < M) {
      float a;
      if (VAR >= 1) {
        float g[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) g[j] = Tp[c[j]];
        a = 0.f;
#pragma unroll
        for (int j = 0; j < 12; ++j) a = a + v[j] * g[j];
      } else {
        a = Tp[tid];
      }
      s[cur * MP + tid] = 2.f * a - s[prv2 * MP + tid];
    }
    __syncthreads();
  }
  if (tid == 0) out[blockIdx.x] = s[5] + acc0[0] + acc1[3];
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  const int M = 976;
  float* out;
  int* colmap;
  hipMalloc(&out, 4096 * 4);
  hipMalloc(&colmap, 12 * T * 4);
  int h[12 * T];
  for (int j = 0; j < 12; ++j)
    for (int t = 0; t < T; ++t) {
      // grid-like neighbourhood: +-1, +-28, +-27, +-29 ... clamped; padding -> M
      const int offs[12] = {-29, -28, -27, -1, 1, 27, 28, 29, -56, 56, 2, -2};
      int c = t + offs[j];
      if (j >= 8 && (t % 3)) c = M;  // ragged rows
      if (c < 0 || c > M) c = M;
      h[j * T + t] = c;
    }
  hipMemcpy(colmap, h, sizeof(h), hipMemcpyHostToDevice);
  const int lds = (3 * MP + 3 + M * 25) * 4;
  hipFuncSetAttribute((const void*)step_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipFuncSetAttribute((const void*)step_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipFuncSetAttribute((const void*)step_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipFuncSetAttribute((const void*)step_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int ns : {2, 25}) {
    float t0 = timeit([&] { hipLaunchKernelGGL(step_kernel<0>, dim3(256), dim3(T), lds, 0, ns, M, colmap, out); }, 50);
    float t1 = timeit([&] { hipLaunchKernelGGL(step_kernel<1>, dim3(256), dim3(T), lds, 0, ns, M, colmap, out); }, 50);
    float t2 = timeit([&] { hipLaunchKernelGGL(step_kernel<2>, dim3(256), dim3(T), lds, 0, ns, M, colmap, out); }, 50);
    float t3 = timeit([&] { hipLaunchKernelGGL(step_kernel<3>, dim3(256), dim3(T), lds, 0, ns, M, colmap, out); }, 50);
    printf("nsteps=%d  bare %.2f  +gather %.2f  +mfma_pair %.2f  +lds_basis %.2f us\n", ns, t0, t1, t2, t3);
  }
  return 0;
}
