// Host cost of hipFuncSetAttribute(MaxDynamicSharedMemorySize) per call (the library sets it before
// every launch that needs > 64 KB of dynamic LDS).  Build: hipcc -O2 --offload-arch=gfx950 funcattr.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k(double *p) {
  extern __shared__ double s[];
  s[threadIdx.x] = p[threadIdx.x];
  __syncthreads();
  p[threadIdx.x] = s[(threadIdx.x + 1) % blockDim.x];
}

int main() {
  double *d;
  (void)hipMalloc(&d, 1024 * sizeof(double));
  const int n = 20000;
  for (int bytes : {100000, 150000}) {
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i)
      (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k), hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    auto t1 = std::chrono::steady_clock::now();
    printf("hipFuncSetAttribute(%d): %.2f us per call\n", bytes,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / n);
  }
  for (int lds : {2048, 32768, 65536, 100000, 150000}) {
    for (int nt : {256, 1024}) {
      hipLaunchKernelGGL(k, dim3(1), dim3(nt), lds, 0, d);
      (void)hipDeviceSynchronize();
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k, dim3(1), dim3(nt), lds, 0, d);
      (void)hipDeviceSynchronize();
      auto t1 = std::chrono::steady_clock::now();
      printf("back-to-back launches, %d threads, %6d B dynamic LDS: %.2f us per launch incl. execution\n", nt, lds,
             std::chrono::duration<double, std::micro>(t1 - t0).count() / n);
    }
  }
  return 0;
}
