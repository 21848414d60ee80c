// Micro-benchmark: cost of one "step" (LDS read/read/write + __syncthreads)
// vs workgroup size, to size the per-step overhead of the resident kernels.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/barrier_bench.hip -o build/barrier_bench
#include <hip/hip_runtime.h>
#include <cstdio>

template <int T>
__global__ __launch_bounds__(T) void steps(int nsteps, int M, float* out) {
  extern __shared__ float s[];
  const int tid = threadIdx.x;
  for (int i = tid; i < 3 * 1024; i += T) s[i] = float(i);
  __syncthreads();
  for (int k = 1; k < nsteps; ++k) {
    const int cur = k % 3, prv = (k + 2) % 3, prv2 = (k + 1) % 3;
    for (int r = tid; r < M; r += T) s[cur * 1024 + r] = 2.f * s[prv * 1024 + r] - s[prv2 * 1024 + r];
    __syncthreads();
  }
  if (tid == 0) out[blockIdx.x] = s[5];
}

template <int T>
__global__ __launch_bounds__(T) void steps_nobar(int nsteps, int M, float* out) {
  extern __shared__ float s[];
  const int tid = threadIdx.x;
  for (int i = tid; i < 3 * 1024; i += T) s[i] = float(i);
  __syncthreads();
  for (int k = 1; k < nsteps; ++k) {
    const int cur = k % 3, prv = (k + 2) % 3, prv2 = (k + 1) % 3;
    for (int r = tid; r < M; r += T) s[cur * 1024 + r] = 2.f * s[prv * 1024 + r] - s[prv2 * 1024 + r];
    __builtin_amdgcn_s_waitcnt(0xc07f);
  }
  if (tid == 0) out[blockIdx.x] = s[5];
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
  float* out;
  hipMalloc(&out, 4096 * 4);
  hipFuncSetAttribute((const void*)steps<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipFuncSetAttribute((const void*)steps<512>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipFuncSetAttribute((const void*)steps<256>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipFuncSetAttribute((const void*)steps_nobar<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  const int M = 976, lds = 3 * 1024 * 4 + 100 * 1024;  // ~112 KB like the forward
  for (int nsteps : {2, 25, 49}) {
    float t1024 = timeit([&] { hipLaunchKernelGGL(steps<1024>, dim3(256), dim3(1024), lds, 0, nsteps, M, out); }, 50);
    float t512 = timeit([&] { hipLaunchKernelGGL(steps<512>, dim3(256), dim3(512), lds, 0, nsteps, M, out); }, 50);
    float t256 = timeit([&] { hipLaunchKernelGGL(steps<256>, dim3(256), dim3(256), lds, 0, nsteps, M, out); }, 50);
    float n1024 = timeit([&] { hipLaunchKernelGGL(steps_nobar<1024>, dim3(256), dim3(1024), lds, 0, nsteps, M, out); }, 50);
    float small = timeit([&] { hipLaunchKernelGGL(steps<1024>, dim3(256), dim3(1024), 16384, 0, nsteps, M, out); }, 50);
    printf("nsteps=%d  1024thr %.2f us  512thr %.2f us  256thr %.2f us  1024-nobarrier %.2f us  1024-smallLDS %.2f us\n",
           nsteps, t1024, t512, t256, n1024, small);
  }
  hipFuncSetAttribute((const void*)steps<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  return 0;
}
