// Launch floor of the fast resident kernels' grid shape on MI355X: an empty
// kernel (and one that only touches LDS / does one barrier) with 256 or 512
// workgroups of 1024 threads and up to 160 KB of dynamic LDS, 200 back-to-back
// launches timed with HIP events.   hipcc --offload-arch=gfx950 -O3 launch_floor.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(1024) void k_empty(float* out) {
  if (out && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) out[0] = 1.f;
}
__global__ __launch_bounds__(1024) void k_barrier(float* out) {
  extern __shared__ float lds[];
  lds[threadIdx.x] = float(threadIdx.x);
  __syncthreads();
  if (out && lds[1023 - threadIdx.x] < -1.f) out[0] = 1.f;
}
// 28 coalesced 4-B loads per thread from a 112 KB table shared by all
// workgroups (the fast kernels' per-thread image), then a barrier
__global__ __launch_bounds__(1024) void k_image(const int* img, float* out) {
  extern __shared__ float lds[];
  int acc = 0;
#pragma unroll
  for (int j = 0; j < 28; ++j) acc += img[j * 1024 + threadIdx.x];
  lds[threadIdx.x] = float(acc);
  __syncthreads();
  if (out && lds[1023 - threadIdx.x] < -1.f) out[0] = 1.f;
}

template <typename F>
float time_us(F launch) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) launch();
  hipEventRecord(a);
  for (int i = 0; i < 200; ++i) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / 200.f;
}

int main() {
  float* out;
  int* img;
  hipMalloc(&out, 4);
  hipMalloc(&img, 28 * 1024 * 4);
  hipMemset(img, 0, 28 * 1024 * 4);
  hipFuncSetAttribute(reinterpret_cast<const void*>(k_empty), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipFuncSetAttribute(reinterpret_cast<const void*>(k_barrier), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipFuncSetAttribute(reinterpret_cast<const void*>(k_image), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int grid : {256, 512}) {
    for (int lds : {0, 64 * 1024, 160 * 1024}) {
      const float e = time_us([&] { hipLaunchKernelGGL(k_empty, dim3(grid), dim3(1024), lds, 0, out); });
      const float b = time_us([&] { hipLaunchKernelGGL(k_barrier, dim3(grid), dim3(1024), lds < 4096 ? 4096 : lds, 0, out); });
      const float m = time_us([&] { hipLaunchKernelGGL(k_image, dim3(grid), dim3(1024), lds < 4096 ? 4096 : lds, 0, img, out); });
      printf("{\"grid\": %d, \"lds\": %d, \"empty_us\": %.2f, \"barrier_us\": %.2f, \"image_us\": %.2f}\n", grid, lds, e, b, m);
    }
  }
  return 0;
}
